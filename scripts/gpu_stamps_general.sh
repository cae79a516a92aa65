#!/bin/bash
# per-section cycle shares of the GENERAL consensus kernel (diagnostic build; through gpurun):
# cfg3 with little-endian seeds (in-kernel hashes) and drop64, 2,048 instances each
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 env BFTSIM_TESTING=1 BFTSIM_LIB=consensus-rs_amd/build/libbftsim_stamps.so python - <<'PY' > gpurun_out/stamps_general.txt 2>&1
import ctypes, dataclasses, sys
sys.path.insert(0, "consensus-rs_amd")
from bftsim import runtime
from bftsim.configs import cfg3, BftConfig
names = ["t_step", "summarize", "publish+classify", "post-sync", "resolve", "mask+offset+miner", "#phases",
         "loop/other", "deliver_blk", "deliver_pc", "deliver_general", "#general", "deliver_pp", "deliver_rc",
         "#rc", "#none"]
for name, cfg, fast in (("drop64-full", BftConfig(n=64, heights=100, seed=15, byz_count=21, drop_ppm=50_000, name="drop64"), 0),
                        ("cfg2", __import__("bftsim.configs", fromlist=["cfg2"]).cfg2(), 1),
                        ("cfg4-256", __import__("bftsim.configs", fromlist=["cfg4"]).cfg4(256), 1),
                        ("cfg4-128", __import__("bftsim.configs", fromlist=["cfg4"]).cfg4(128), 1)):
    sim = runtime.Simulator(cfg)
    if not fast:
        sim.set_fast(False)
    sim.prepare(2048)
    sim.launch(0); sim.sync()
    out = (ctypes.c_uint64 * 16)()
    runtime.lib().bftsim_debug_stamps(out)
    cnt = (6, 11, 14, 15)
    tot = sum(out[k] for k in range(16) if k not in cnt)
    views = int(sim.stats()["views"])
    print(f"== {name}: instance-rounds {views}, phases per instance-round {out[6] / max(views,1):.2f}, general phases {out[11] / max(views,1):.2f}")
    for k in range(16):
        print(f"  {names[k]:18s} {out[k]:16d} {100.0*out[k]/max(tot,1):6.2f}%")
    sim.close()
PY
rc=$?
cat gpurun_out/stamps_general.txt
exit $rc
