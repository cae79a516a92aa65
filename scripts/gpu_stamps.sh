#!/bin/bash
# per-section cycle shares of the consensus kernel (diagnostic build; used through gpurun)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 env BFTSIM_LIB=consensus-rs_amd/build/libbftsim_stamps.so python - <<'PY' > gpurun_out/stamps.txt 2>&1
import ctypes, sys
sys.path.insert(0, "consensus-rs_amd")
from bftsim import runtime
from bftsim.configs import cfg3
sim = runtime.Simulator(cfg3())
sim.prepare(16384)
for _ in range(2):
    sim.launch(0)
    sim.sync()
out = (ctypes.c_uint64 * 12)()
runtime.lib().bftsim_debug_stamps(out)
names = ["t_step", "summarize", "publish+sync", "deliver?", "resolve", "mask+offset", "#phases", "loop/other", "fast_blk", "fast_pc", "general", "#general"]
tot = sum(out[k] for k in range(12) if k not in (6, 11))
print("phases per wave-height", out[6] / (16384 * 100.0), "general", out[11] / (16384 * 100.0))
for k in range(12):
    print(f"{names[k]:14s} {out[k]:16d} {100.0*out[k]/max(tot,1):6.2f}%")
print("kernel ms", sim.kernel_ms())
PY
rc=$?
cat gpurun_out/stamps.txt
exit $rc
