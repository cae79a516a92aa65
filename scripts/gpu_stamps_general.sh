#!/bin/bash
# per-section cycle shares of the GENERAL consensus kernel (diagnostic build; through gpurun):
# drop64, cfg2, cfg4 N=256/128 and cfg5 (1,000 heights, windowed), 2,048 instances each (STAMP_CASES picks)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 env BFTSIM_TESTING=1 BFTSIM_LIB=consensus-rs_amd/build/libbftsim_stamps.so python - <<'PY' > gpurun_out/stamps_general.txt 2>&1
import ctypes, dataclasses, sys
sys.path.insert(0, "consensus-rs_amd")
from bftsim import runtime
from bftsim.configs import cfg3, BftConfig
names = ["t_step", "summarize", "publish+classify", "post-sync", "resolve", "mask+offset+miner", "#phases",
         "loop/other", "deliver_blk", "deliver_pc", "deliver_general", "#general", "deliver_pp", "deliver_rc",
         "#rc", "#none", "seg_hash_encode", "seg_hash_keccak"]
import os
from bftsim.configs import cfg2, cfg4, cfg5
cases = {"drop64-full": (BftConfig(n=64, heights=100, seed=15, byz_count=21, drop_ppm=50_000, name="drop64"), 0, 0),
         "cfg2": (cfg2(), 1, 0), "cfg4-256": (cfg4(256), 1, 0), "cfg4-128": (cfg4(128), 1, 0),
         "cfg5-1000": (cfg5(heights=1000), 1, 256)}
want = os.environ.get("STAMP_CASES", "drop64-full cfg2 cfg4-256 cfg4-128").split()
for name in want:
    cfg, fast, window = cases[name]
    sim = runtime.Simulator(cfg)
    if not fast:
        sim.set_fast(False)
    if window:
        sim.set_window(window)
    sim.prepare(2048)
    sim.launch(0); sim.sync()
    L = runtime.lib()
    L.bftsim_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    ns = L.bftsim_debug_stamps(None, 0)           # the build's section count (bft::NSTAMP)
    out = (ctypes.c_uint64 * ns)()
    assert L.bftsim_debug_stamps(out, ns) == ns
    cnt = (6, 11, 14, 15)
    tot = sum(out[k] for k in range(18) if k not in cnt)
    views = int(sim.stats()["views"])
    print(f"== {name}: instance-rounds {views}, phases per instance-round {out[6] / max(views,1):.2f}, general phases {out[11] / max(views,1):.2f}")
    for k in range(18):
        print(f"  {names[k]:18s} {out[k]:16d} {100.0*out[k]/max(tot,1):6.2f}%")
    sim.close()
PY
rc=$?
cat gpurun_out/stamps_general.txt
exit $rc
