"""Diagnostic (through gpurun): consensus / hash kernel ms of cfg3 variants, unpipelined.
usage: python scripts/diag_kms.py [byz | byz:le ...]"""
import dataclasses, sys
sys.path.insert(0, "consensus-rs_amd")
from bftsim.runtime import Simulator
from bftsim.configs import cfg3

for arg in sys.argv[1:] or ["21", "0"]:
    byz, _, order = arg.partition(":")
    cfg = dataclasses.replace(cfg3(), byz_count=int(byz), seed_byte_order=1 if order == "le" else 0)
    sim = Simulator(cfg)
    sim.set_pipeline(False)
    sim.prepare(16384)
    for _ in range(2):
        sim.launch(0); sim.sync()
    sim.kernel_ms_sum()
    for _ in range(5):
        sim.launch(0); sim.sync()
    c, h, n = sim.kernel_ms_sum()
    r = sim.fetch()
    print(f"byz={arg}: consensus {c / n:.3f} ms  hash {h / n:.3f} ms  views {int(r['views'].sum())}", flush=True)
    sim.close()
