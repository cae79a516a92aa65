#!/bin/bash
# per-section cycle shares of the consensus kernel (diagnostic build; used through gpurun)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 env BFTSIM_TESTING=1 BFTSIM_LIB=consensus-rs_amd/build/libbftsim_stamps.so python - <<'PY' > gpurun_out/stamps.txt 2>&1
import ctypes, dataclasses, os, sys
sys.path.insert(0, "consensus-rs_amd")
from bftsim import runtime
from bftsim.configs import cfg3
sim = runtime.Simulator(dataclasses.replace(cfg3(), byz_count=int(os.environ.get('BYZ', '21'))))
sim.prepare(16384)
for _ in range(2):
    sim.launch(0)
    sim.sync()
L = runtime.lib()
L.bftsim_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
ns = L.bftsim_debug_stamps(None, 0)           # the build's section count (bft::NSTAMP)
out = (ctypes.c_uint64 * ns)()
assert L.bftsim_debug_stamps(out, ns) == ns
names = ["t_step", "classify", "event_step", "deliver_pp", "deliver_pc", "deliver_blk", "resolve", "loop/other", "#phases", "#pp", "#pc", "#blk"]
cnt = (8, 9, 10, 11)
tot = sum(out[k] for k in range(12) if k not in cnt)
print("per wave-height: phases", out[8] / (16384 * 100.0), "pp", out[9] / 1638400.0, "pc", out[10] / 1638400.0, "blk", out[11] / 1638400.0)
for k in range(12):
    print(f"{names[k]:14s} {out[k]:16d} {100.0*out[k]/max(tot,1):6.2f}%  {out[k]/1638400.0:9.1f} per wave-height")
print("kernel ms", sim.kernel_ms())
PY
rc=$?
cat gpurun_out/stamps.txt
exit $rc
