"""Keys for real-crypto mode (include/bftsim.h bftsim_set_crypto, SPEC.md §11).

A validator set with keys is the reference's: each node's `secret` (examples/c*.toml) derives its
address, and the validator set is the sorted address list (ImplValidatorSet::new). `keyed_config`
builds that config from secrets whose addresses the caller derived (libbftsig's
`Signer.secret_to_address` on the GPU, or any other implementation of ethkey's derivation) and
returns the secrets in the sorted validator order bftsim_set_crypto expects.
"""
from __future__ import annotations

import dataclasses
from typing import List, Sequence, Tuple

from .configs import BftConfig


def synthetic_secrets(n: int, seed: int) -> List[bytes]:
    """n deterministic 32-byte secp256k1 secrets: keccak256("bftsim-key" || seed || i) (a keccak
    output is a valid secret with probability 1 - 2^-127)."""
    from .runtime import keccak256
    return [keccak256(b"bftsim-key" + seed.to_bytes(8, "little") + i.to_bytes(4, "little")) for i in range(n)]


def keyed_config(cfg: BftConfig, secrets: Sequence[bytes], addresses: Sequence[bytes]) -> Tuple[BftConfig, List[bytes]]:
    """(config whose validator set is `addresses` sorted, the secrets in that order)"""
    assert len(secrets) == len(addresses) == cfg.n
    order = sorted(range(cfg.n), key=lambda i: bytes(addresses[i]))
    addrs = [bytes(addresses[i]) for i in order]
    return dataclasses.replace(cfg, addresses=addrs), [bytes(secrets[i]) for i in order]


def gpu_addresses(secrets: Sequence[bytes], device: int = 0) -> List[bytes]:
    """The ethkey addresses of `secrets` through libbftsig (KeyPair::from_secret(..).address())."""
    import numpy as np
    from .sig import Signer
    s = Signer(device)
    try:
        arr = np.frombuffer(b"".join(secrets), np.uint8).reshape(-1, 32)
        _, addr, ok = s.secret_to_address(arr)
        addr, ok = addr.cpu().numpy(), ok.cpu().numpy()
    finally:
        s.close()
    assert ok.all(), "invalid secret"
    return [bytes(a) for a in addr]
