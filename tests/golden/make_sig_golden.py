#!/usr/bin/env python3
"""Generates tests/golden/sig_vectors.json: secp256k1 vectors from the CPU oracle
(oracle/secp256k1_ref.py) plus the reference's own key fixtures.

`reference_keys`: the `secret` of /root/reference/examples/c1..c5.toml with the genesis validator
addresses of examples/c1.toml:14 they must derive (data copied from the reference's config files;
the oracle reproduces all five). `vectors`: seeded secrets/digests -> public key, address and the
RFC 6979 signature; `invalid`: malformed signatures that must not recover.
Run from the repo root: python tests/golden/make_sig_golden.py"""
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import secp256k1_ref as S  # noqa: E402
import oracle_lib as O  # noqa: E402

REFERENCE_KEYS = [  # examples/c1..c5.toml `secret` -> examples/c1.toml:14 genesis validator
    ("7f3b0a324e13e5358c3fd686737acd7adf2e5556084ec6d9e48b497082b7ef98", "7193d8f91724b39f10cc81e94934c187fa257277"),
    ("ec84caf3d58e6bbcdcd6b243203fbaafee19e91048c61fe34e12fa7a93af27f9", "93908f59c6eff007d228398349214acb6b4ac9a4"),
    ("64115814914b9d1aaa7d485770f50274b673df4634fcdd0ea3347e73e4b800ad", "72d5c75fd6703414aa87f79b3e4797dd09cd9251"),
    ("f9093897ce74d867cdbc5c5a1b6e840ffb4343cbb0ea5b3ad5525edc6bad8c95", "58096d35c7a8ff67eba159f33cea7740fc9a737c"),
    ("6a30cfa9d15d64e4d7b0f15a18d6ea78d242e820e012b9980af5dbdc6403f61a", "c759616c865d349ec2afced268fc6f33ff7414a4"),
]


def main():
    rng = random.Random(20181009)
    vec = []
    secrets = [bytes.fromhex(s) for s, _ in REFERENCE_KEYS] + [
        rng.randrange(1, S.N).to_bytes(32, "big") for _ in range(11)]
    secrets += [(1).to_bytes(32, "big"), (S.N - 1).to_bytes(32, "big")]
    for i, sec in enumerate(secrets):
        msg = O.keccak256(b"consensus-rs gossip %d" % i) if i % 3 else bytes(rng.randrange(256) for _ in range(32))
        if i == len(secrets) - 1:
            msg = b"\xff" * 32                 # digest >= n (reduced mod n)
        pub = S.pubkey(sec)
        sig = S.sign(sec, msg)
        assert S.verify(pub, msg, sig) and S.recover(msg, sig) == pub
        vec.append(dict(secret=sec.hex(), digest=msg.hex(), pub=pub.hex(), address=S.address(pub, O.keccak256).hex(),
                        sig=sig.hex()))
    good = bytes.fromhex(vec[0]["sig"])
    msg0 = bytes.fromhex(vec[0]["digest"])
    n_be = S.N.to_bytes(32, "big")
    invalid = [
        ("r zero", msg0, bytes(32) + good[32:]),
        ("s zero", msg0, good[:32] + bytes(32) + good[64:]),
        ("r = n", msg0, n_be + good[32:]),
        ("s = n", msg0, good[:32] + n_be + good[64:]),
        ("recid 4", msg0, good[:64] + b"\x04"),
        ("recid 2, r + n >= p", msg0, good[:64] + bytes([good[64] | 2])),
    ]
    # an r whose x is not on the curve
    x = 1
    while pow((x ** 3 + 7) % S.P, (S.P - 1) // 2, S.P) == 1:
        x += 1
    invalid.append(("x not on curve", msg0, x.to_bytes(32, "big") + good[32:]))
    for name, m, s in invalid:
        assert S.recover(m, s) is None, name
    out = dict(reference_keys=[dict(secret=s, address=a) for s, a in REFERENCE_KEYS], vectors=vec,
               invalid=[dict(name=n, digest=m.hex(), sig=s.hex()) for n, m, s in invalid])
    with open(os.path.join(ROOT, "tests", "golden", "sig_vectors.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", len(vec), "vectors,", len(invalid), "invalid signatures")


if __name__ == "__main__":
    main()
