"""Time windowed cfg5 runs on one GPU (instances x heights), to size tests and the bench leg."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "consensus-rs_amd"))
import torch  # noqa: E402
from bftsim.configs import cfg5  # noqa: E402
from bftsim.runtime import Simulator  # noqa: E402

for n, H in [(int(a), int(b)) for a, b in (x.split("x") for x in sys.argv[1:])]:
    cfg = cfg5(heights=H)
    sim = Simulator(cfg)
    sim.set_window(256)
    sim.prepare(n)
    torch.cuda.synchronize()
    t = time.perf_counter()
    sim.launch(0)
    sim.sync()
    dt = time.perf_counter() - t
    st = sim.stats()
    c, _ = sim.kernel_ms()
    print(json.dumps(dict(instances=n, heights=H, seconds=round(dt, 3), kernel_ms=round(c, 1),
                          ir_per_s=st["views"] / dt, committed=st["committed_heights"], flagged=st["flagged"],
                          round_hist=st["round_hist"][:8], latency_hist=st["latency_hist"][:8])), flush=True)
    sim.close()
