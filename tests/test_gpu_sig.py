"""secp256k1 on the GPU through the C ABI (include/bftsig.h): bit-exact against the CPU oracle
(oracle/secp256k1_ref.py) and the golden vectors, plus size-independent properties at full batch
sizes (sign -> recover round trip, verify_address, corruption rejected)."""
import json
import os
import random
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "consensus-rs_amd"))
import secp256k1_ref as S  # noqa: E402
import oracle_lib as O  # noqa: E402

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "sig_vectors.json")))


@pytest.fixture(scope="module")
def signer():
    from bftsim.sig import Signer
    s = Signer(0)
    yield s
    s.close()


def arr(rows):
    return np.frombuffer(b"".join(rows), dtype=np.uint8).reshape(len(rows), -1).copy()


def test_reference_keys_on_gpu(signer):
    secs = arr([bytes.fromhex(k["secret"]) for k in GOLD["reference_keys"]])
    pub, addr, ok = signer.secret_to_address(secs)
    assert ok.cpu().numpy().tolist() == [1] * 5
    assert [bytes(a).hex() for a in addr.cpu().numpy()] == [k["address"] for k in GOLD["reference_keys"]]


def test_golden_vectors_on_gpu(signer):
    V = GOLD["vectors"]
    secs = arr([bytes.fromhex(v["secret"]) for v in V])
    digs = arr([bytes.fromhex(v["digest"]) for v in V])
    pub, addr, ok = signer.secret_to_address(secs)
    assert (ok.cpu().numpy() == 1).all()
    assert [bytes(p).hex() for p in pub.cpu().numpy()] == [v["pub"] for v in V]
    sig, ok = signer.sign(secs, digs)
    assert (ok.cpu().numpy() == 1).all()
    assert [bytes(s).hex() for s in sig.cpu().numpy()] == [v["sig"] for v in V]
    rpub, raddr, ok = signer.recover(digs, sig)
    assert (ok.cpu().numpy() == 1).all()
    assert [bytes(a).hex() for a in raddr.cpu().numpy()] == [v["address"] for v in V]
    bad = GOLD["invalid"]
    _, baddr, bok = signer.recover(arr([bytes.fromhex(b["digest"]) for b in bad]),
                                   arr([bytes.fromhex(b["sig"]) for b in bad]))
    assert (bok.cpu().numpy() == 0).all() and (baddr.cpu().numpy() == 0).all()


def test_seeded_batch_matches_oracle(signer):
    rng = random.Random(5)
    n = 96
    secs = [rng.randrange(1, S.N).to_bytes(32, "big") for _ in range(n)]
    digs = [bytes(rng.randrange(256) for _ in range(32)) for _ in range(n)]
    sig, ok = signer.sign(arr(secs), arr(digs))
    sig = sig.cpu().numpy()
    assert (ok.cpu().numpy() == 1).all()
    for i in range(n):
        assert bytes(sig[i]) == S.sign(secs[i], digs[i]), i
    # recover with random recovery ids: valid or not, GPU and oracle agree
    mangled = [bytes(sig[i][:64]) + bytes([rng.randrange(4)]) for i in range(n)]
    pub, addr, ok = signer.recover(arr(digs), arr(mangled))
    pub, ok = pub.cpu().numpy(), ok.cpu().numpy()
    for i in range(n):
        want = S.recover(digs[i], mangled[i])
        assert ok[i] == (want is not None), i
        if want is not None:
            assert bytes(pub[i]) == want, i


def test_key_index_and_invalid_secrets(signer):
    secs = arr([bytes(32), bytes.fromhex(GOLD["reference_keys"][0]["secret"]), S.N.to_bytes(32, "big")])
    digs = arr([O.keccak256(b"m%d" % i) for i in range(6)])
    sig, ok = signer.sign(secs, digs, key_index=[1, 0, 2, 1, 1, 0])
    assert ok.cpu().numpy().tolist() == [1, 0, 0, 1, 1, 0]
    sig = sig.cpu().numpy()
    assert bytes(sig[0]) == S.sign(bytes.fromhex(GOLD["reference_keys"][0]["secret"]), bytes(digs[0]))
    assert not sig[1].any()


def test_full_batch_round_trip(signer):
    """65,536 signatures (the per-height message volume of 1,024 N=64 clusters): every one recovers to
    its signer's address and passes verify_address; one flipped digest bit fails it."""
    import torch
    n, keys = 65_536, 64
    g = torch.Generator().manual_seed(9)
    secs = torch.randint(0, 256, (keys, 32), dtype=torch.uint8, generator=g)
    secs[:, 0] &= 0x7f                                  # < n
    digs = torch.randint(0, 256, (n, 32), dtype=torch.uint8, generator=g)
    kidx = torch.arange(n, dtype=torch.int32) % keys
    _, kaddr, kok = signer.secret_to_address(secs)
    assert bool((kok == 1).all())
    sig, ok = signer.sign(secs, digs, key_index=kidx)
    assert bool((ok == 1).all())
    s = sig.cpu().numpy()
    assert (s[:, 64] <= 1).all()                        # R.x >= n never happens in practice
    assert all(int.from_bytes(bytes(s[i, 32:64]), "big") <= S.N // 2 for i in range(0, n, 4099))
    _, addr, ok = signer.recover(digs, sig, want_pub=False)
    assert bool((ok == 1).all())
    want = kaddr[kidx.to(kaddr.device).long()]
    assert bool((addr == want).all())
    assert bool((signer.verify_address(want, digs, sig) == 1).all())
    d2 = digs.clone()
    d2[:, 31] ^= 1
    assert not bool(signer.verify_address(want, d2, sig).any())
    for i in (0, 12345, n - 1):                        # spot checks against the oracle
        assert bytes(s[i]) == S.sign(bytes(secs[i % keys].numpy()), bytes(digs[i].numpy()))


def test_recover_matches_c_oracle_4096(signer):
    """4,096 recoveries with random recovery ids (about half do not recover, or recover another key):
    GPU and the C oracle (oracle/secp_oracle.c, an independent implementation) agree item by item."""
    import torch
    g = torch.Generator().manual_seed(17)
    n, keys = 4096, 32
    secs = torch.randint(0, 256, (keys, 32), dtype=torch.uint8, generator=g)
    secs[:, 0] &= 0x7f
    digs = torch.randint(0, 256, (n, 32), dtype=torch.uint8, generator=g)
    sig, ok = signer.sign(secs, digs, key_index=torch.arange(n, dtype=torch.int32) % keys)
    assert bool((ok == 1).all())
    s = sig.cpu().numpy().copy()
    s[:, 64] = torch.randint(0, 4, (n,), generator=g).numpy()
    pub, _, ok = signer.recover(digs, s)
    want, wok = O.secp_recover_batch(digs.numpy(), s, threads=16)
    assert (ok.cpu().numpy() == wok).all()
    assert (pub.cpu().numpy()[wok == 1] == want[wok == 1]).all()
    assert (pub.cpu().numpy()[wok == 0] == 0).all()
