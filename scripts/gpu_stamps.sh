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
names = ["t_step", "summarize", "publish+sync", "deliver?", "resolve", "mask+offset", "-", "loop/other", "fast_blk", "fast_pc", "general", "-"]
tot = sum(out)
for k in range(12):
    print(f"{names[k]:14s} {out[k]:16d} {100.0*out[k]/max(tot,1):6.2f}%")
print("kernel ms", sim.kernel_ms())
PY
rc=$?
cat gpurun_out/stamps.txt
exit $rc
