#!/usr/bin/env python3
"""Generates tests/golden/*.json from the C oracle (oracle/) and from published known answers.

Committed fixtures = data only (inputs + expected outputs). Re-run after an intentional SPEC
change: python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as O  # noqa: E402
from bftsim.configs import BftConfig, cfg1, cfg2, cfg3, cfg4, cfg5  # noqa: E402

KECCAK_KAT = {   # published Keccak-256 (pre-FIPS padding 0x01) answers
    "": "c5d2460186f7233c927e7db2dcc703c0e500b653ca82273b7bfad8045d85a470",
    "abc": "4e03657aea45a94fc7d47ba826c8d667c0d1e6e33a64a036ec44f58fa12d6c45",
    "The quick brown fox jumps over the lazy dog":
        "4d741b6f1eb29cb2a9b9911c82f56fa8d73b04959d3d9d222895df6c0b28aa15",
}
PHILOX_KAT = [   # Random123 philox4x32-10 known answers: (ctr, key, out)
    ([0, 0, 0, 0], [0, 0], [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
    ([0xffffffff] * 4, [0xffffffff] * 2, [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
    ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
     [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]),
]

RUNS = [   # (name, config factory, first instance, instances)
    ("cfg1_n5", lambda: cfg1(True), 0, 1),
    ("cfg1_n4", lambda: cfg1(False), 0, 1),
    ("cfg2_h20", lambda: cfg2(heights=20), 0, 8),
    ("cfg3_h20", lambda: cfg3(heights=20), 0, 4),
    ("cfg4_n7_h30", lambda: cfg4(7, heights=30), 0, 8),
    ("cfg4_n64_h30", lambda: cfg4(64, heights=30), 0, 2),
    ("cfg5_h60", lambda: cfg5(heights=60), 0, 8),
    ("n4_byz2_unsafe", lambda: BftConfig(n=4, heights=30, seed=9, byz_count=2), 0, 8),
]


def result_json(r, n):
    out = []
    for i in range(n):
        ch = int(r["committed_height"][i])
        out.append(dict(
            committed_height=ch, flags=int(r["flags"][i]), ticks=int(r["ticks"][i]),
            views=int(r["views"][i]),
            round=[int(x) for x in r["round"][i][:ch]],
            proposer=[int(x) for x in r["proposer"][i][:ch]],
            variant=[int(x) for x in r["variant"][i][:ch]],
            time_tick=[int(x) for x in r["time_tick"][i][:ch]],
            block_hash=[bytes(r["block_hash"][i][k]).hex() for k in range(ch)]))
    return out


def main():
    kat = dict(keccak256=KECCAK_KAT,
               philox4x32_10=[dict(ctr=c, key=k, out=o) for c, k, o in PHILOX_KAT],
               sha3_256_crosscheck={m: hashlib.sha3_256(m.encode()).hexdigest() for m in KECCAK_KAT})
    json.dump(kat, open(os.path.join(HERE, "kat.json"), "w"), indent=1)
    runs = {}
    for name, mk, first, n in RUNS:
        cfg = mk()
        r = O.run(cfg, first, n)
        runs[name] = dict(first=first, n=n, results=result_json(r, n))
    json.dump(runs, open(os.path.join(HERE, "oracle_runs.json"), "w"))
    c = cfg1(True)
    import ctypes
    c_, keep = O.to_orc(c)
    g = (ctypes.c_uint8 * 32)()
    O.lib().orc_genesis_hash(ctypes.byref(c_), g)
    json.dump(dict(genesis_hash=bytes(g).hex(), genesis_time=c.genesis_time,
                   genesis_proposer=c.genesis_proposer.hex()),
              open(os.path.join(HERE, "genesis.json"), "w"), indent=1)
    print("wrote", os.listdir(HERE))


if __name__ == "__main__":
    main()
