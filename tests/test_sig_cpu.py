"""secp256k1 (real-crypto mode) on the CPU: the oracle pinned by the reference's own
key fixtures and by hashlib/hmac, and the host build of the GPU source (consensus-rs_amd/csrc/secp256k1.h)
checked against the oracle. No GPU needed."""
import ctypes
import hashlib
import json
import os
import random
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import secp256k1_ref as S  # noqa: E402
import oracle_lib as O  # noqa: E402
import sig_lib as H  # noqa: E402

GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "sig_vectors.json")))


def test_curve_constants():
    assert S.on_curve(S.G)
    assert S.point_mul(S.N) is None
    assert S.point_mul(S.N - 1) == (S.GX, S.P - S.GY)


def test_reference_keys_derive_the_genesis_validators():
    """examples/c1..c5.toml `secret` -> examples/c1.toml:14 validator addresses (oracle and host build)."""
    for k in GOLD["reference_keys"]:
        sec = bytes.fromhex(k["secret"])
        assert S.address(S.pubkey(sec), O.keccak256).hex() == k["address"]
        assert H.pub(sec)[1].hex() == k["address"]


def test_oracle_nonce_and_signature_are_self_consistent():
    rng = random.Random(7)
    for _ in range(8):
        sec = rng.randrange(1, S.N).to_bytes(32, "big")
        msg = bytes(rng.randrange(256) for _ in range(32))
        sig = S.sign(sec, msg)
        assert int.from_bytes(sig[32:64], "big") <= S.N // 2          # low s
        assert S.verify(S.pubkey(sec), msg, sig)
        assert S.recover(msg, sig) == S.pubkey(sec)


def test_sha256_matches_hashlib():
    rng = random.Random(3)
    for n in (0, 1, 55, 56, 63, 64, 65, 119, 120, 200):
        d = bytes(rng.randrange(256) for _ in range(n))
        assert H.sha256(d) == hashlib.sha256(d).digest()


@pytest.mark.parametrize("name", list(H.OPS))
def test_field_and_scalar_primitives(name):
    rng = random.Random(hash(name) & 0xffff)
    edge_p = [0, 1, 2, S.P - 1, S.P - 2, 2 ** 255, 2 ** 32 + 977, 2 ** 256 - 2 ** 32 - 978]
    edge_n = [0, 1, S.N - 1, S.N // 2, 2 ** 128, 2 ** 255]
    mod = S.N if name.startswith("sc") else S.P
    vals = (edge_n if mod == S.N else edge_p) + [rng.randrange(mod) for _ in range(60)]
    for a in vals:
        b = vals[(vals.index(a) * 7 + 3) % len(vals)]
        got = H.op(name, a, b)
        exp = {"fe_mul": a * b % S.P, "fe_sqr": a * a % S.P, "fe_add": (a + b) % S.P, "fe_sub": (a - b) % S.P,
               "fe_inv": pow(a, S.P - 2, S.P), "fe_sqrt": pow(a, (S.P + 1) // 4, S.P),
               "sc_mul": a * b % S.N, "sc_inv": pow(a, S.N - 2, S.N), "sc_add": (a + b) % S.N,
               "sc_neg": (-a) % S.N}[name]
        assert got == exp, (name, hex(a), hex(b))


def test_host_build_matches_golden_vectors():
    for v in GOLD["vectors"]:
        sec, msg = bytes.fromhex(v["secret"]), bytes.fromhex(v["digest"])
        p, a = H.pub(sec)
        assert p.hex() == v["pub"] and a.hex() == v["address"]
        assert H.sign(sec, msg).hex() == v["sig"]
        rp, ra = H.recover(msg, bytes.fromhex(v["sig"]))
        assert rp.hex() == v["pub"] and ra.hex() == v["address"]
    for bad in GOLD["invalid"]:
        assert H.recover(bytes.fromhex(bad["digest"]), bytes.fromhex(bad["sig"])) is None, bad["name"]


def test_host_build_matches_oracle_seeded():
    rng = random.Random(11)
    for i in range(12):
        sec = rng.randrange(1, S.N).to_bytes(32, "big")
        msg = bytes(rng.randrange(256) for _ in range(32))
        assert H.nonces(sec, msg, 3) == b"".join(next(g) for g in [S.rfc6979_nonces(sec, msg)] for _ in range(3))
        pub = S.pubkey(sec)
        k = rng.randrange(1, S.N)
        q = S.point_mul(k, (int.from_bytes(pub[:32], "big"), int.from_bytes(pub[32:], "big")))
        assert H.mul_var(k, pub) == q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big")
        sig = H.sign(sec, msg)
        assert sig == S.sign(sec, msg)
        # a flipped recovery id recovers a different key (or none), as in the oracle
        flipped = sig[:64] + bytes([sig[64] ^ 1])
        want = S.recover(msg, flipped)
        got = H.recover(msg, flipped)
        assert (got is None and want is None) or got[0] == want


def test_invalid_secrets_rejected():
    assert H.pub(bytes(32)) is None
    assert H.pub(S.N.to_bytes(32, "big")) is None
    assert H.sign(bytes(32), bytes(32)) is None


def test_libbftsig_exports_every_declared_symbol():
    sys.path.insert(0, os.path.join(ROOT, "consensus-rs_amd"))
    from bftsim import sig
    src = open(os.path.join(ROOT, "include", "bftsig.h")).read()
    syms = sorted(set(re.findall(r"\b(bftsig_[a-z0-9_]+)\s*\(", src)))
    L = sig.lib()
    assert len(syms) == 7
    assert not [s for s in syms if not hasattr(L, s)]
    # handle-free argument checks fail cleanly without a GPU
    assert L.bftsig_sign(None, None, None, None, 1, None, None, None) < 0
    assert L.bftsig_create(0, None) < 0


def test_c_oracle_matches_python_oracle():
    """The two CPU restatements (Python big integers; C with 64-bit limbs) agree, including on the
    recovery ids that do not recover."""
    import numpy as np
    rng = random.Random(21)
    for k in GOLD["reference_keys"]:
        assert S.address(O.secp_pubkey(bytes.fromhex(k["secret"])), O.keccak256).hex() == k["address"]
    msgs, sigs = [], []
    for _ in range(6):
        sec = rng.randrange(1, S.N).to_bytes(32, "big")
        msg = bytes(rng.randrange(256) for _ in range(32))
        sig = S.sign(sec, msg)
        assert O.secp_pubkey(sec) == S.pubkey(sec)
        for rid in range(4):
            s2 = sig[:64] + bytes([rid])
            assert O.secp_recover(msg, s2) == S.recover(msg, s2)
            msgs.append(msg)
            sigs.append(s2)
    for bad in GOLD["invalid"]:
        assert O.secp_recover(bytes.fromhex(bad["digest"]), bytes.fromhex(bad["sig"])) is None, bad["name"]
    pubs, ok = O.secp_recover_batch(np.frombuffer(b"".join(msgs), np.uint8).reshape(-1, 32),
                                    np.frombuffer(b"".join(sigs), np.uint8).reshape(-1, 65), threads=3)
    for i in range(len(msgs)):
        want = S.recover(msgs[i], sigs[i])
        assert bool(ok[i]) == (want is not None) and (want is None or bytes(pubs[i]) == want)


def test_glv_mul_var_edge_scalars():
    """k*P through the GLV split (secp256k1.h mul_var) at scalars where the split or the signed digits
    hit their edges: 1, n-1, n/2, lambda, n-lambda, 2^128 +- 1, all-ones nibbles."""
    lam = 0x5363AD4CC05C30E0A5261C028812645A122E22EA20816678DF02967C1B23BD72
    pub = S.pubkey((12345).to_bytes(32, "big"))
    P = (int.from_bytes(pub[:32], "big"), int.from_bytes(pub[32:], "big"))
    for k in (1, 2, 15, 16, 17, S.N - 1, S.N - 2, S.N // 2, S.N // 2 + 1, lam, S.N - lam, 2 ** 128 - 1, 2 ** 128,
              2 ** 128 + 1, int("7" * 64, 16), int("8" * 63, 16), (lam * 3) % S.N):
        q = S.point_mul(k, P)
        assert H.mul_var(k, pub) == q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big"), hex(k)
