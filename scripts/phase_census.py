#!/usr/bin/env python3
"""Analysis tool (CPU, not a test): which phase shapes the general kernel body (bft_wave.h Sim) delivers
one message at a time, per workload. Builds the CPU wave emulator with the BFT_PHASE_CENSUS hook into
/tmp and prints, per config, the share of phases by (kinds in flight, uniformity, path)."""
import ctypes, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "consensus-rs_amd"))
import numpy as np
import emu_lib as E
from bftsim.configs import BftConfig, cfg2, cfg3, cfg4
LIB = "/tmp/libwave_emu_census.so"
subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-Wno-unknown-pragmas", "-DBFT_CENSUS_BUILD",
                       "-o", LIB, os.path.join(ROOT, "tests", "emu", "wave_emu.cpp")])
E.LIB = LIB
L = E.lib()
L.emu_census.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
KN = ["PP", "PR", "CM", "OCM", "RC", "SYNC", "BLK"]
PATHS = {0: "GENERAL", 1: "BLK", 2: "PC", 3: "NONE", 4: "PP", 5: "RC"}


def census(cfg, n):
    E.run(cfg, 0, n)
    E.run(cfg, 0, n)
    keys = np.zeros(4096, np.uint32); cnt = np.zeros(4096, np.uint64)
    m = L.emu_census(keys.ctypes.data, cnt.ctypes.data, 4096)
    tot = int(cnt[:m].sum())
    rows = sorted(zip(cnt[:m], keys[:m]), reverse=True)
    r = E.run(cfg, 0, n)
    views = int(r["views"].sum())
    print(f"== {cfg.name}: {tot // 2} segment-phases for {views} instance-rounds ({tot / 2 / max(views, 1):.2f} per "
          f"instance-round)")
    for c, k in rows[:14]:
        kinds = "+".join(n for i, n in enumerate(KN) if k >> i & 1) or "-"
        nu = "".join(x for i, x in ((7, "pr"), (8, "cm"), (9, "blk")) if k >> i & 1)
        print(f"  {100*c/tot:5.1f}%  {PATHS[int(k) >> 12]:8s} {kinds:20s} {'nonuniform:'+nu if nu else ''}")


import dataclasses
W = {"drop64": (BftConfig(n=64, heights=30, seed=15, byz_count=21, drop_ppm=50_000, name="drop64"), 4),
     "cfg2": (cfg2(heights=60), 64), "cfg4-256": (cfg4(256, heights=20), 2), "cfg4-64": (cfg4(64, heights=40), 4),
     "cfg3-le": (dataclasses.replace(cfg3(heights=30), seed_byte_order=1, name="cfg3-le"), 4)}
for name in (sys.argv[1:] or W):
    cfg, n = W[name]
    os.environ["BFT_EMU_FAST"] = "0"
    census(cfg, n)
