"""GPU: the multi-GPU statistic behind the C ABI (include/bftsim.h bftsim_comm_init /
bftsim_stats_allreduce): one RCCL communicator of world size 1 on the box's GPU; the all-reduced
statistics equal the local ones and the oracle's. (World sizes > 1 run in bench.py under torchrun.)"""
import pytest

import oracle_lib as O
from bftsim.configs import cfg2
from bftsim.distributed import stats_from_result

pytestmark = pytest.mark.gpu


def test_stats_allreduce_world1_matches_local_and_oracle():
    from bftsim.runtime import Simulator
    cfg = cfg2(heights=30)
    sim = Simulator(cfg)
    try:
        uid = Simulator.comm_unique_id()
        assert len(uid) == 128
        sim.comm_init(1, 0, uid)
        sim.prepare(128)
        sim.launch(0)
        sim.sync()
        local = sim.stats()
        red = sim.stats_allreduce()
        red2 = sim.stats_allreduce()               # repeatable: no state kept between calls
    finally:
        sim.close()
    assert red == local == red2
    ref = stats_from_result(O.run(cfg, 0, 128))
    for k in ("instances", "committed_heights", "views", "ticks", "flagged", "round_hist"):
        assert red[k] == ref[k], k


def test_stats_allreduce_needs_comm():
    from bftsim.runtime import Simulator, BftsimError
    sim = Simulator(cfg2(heights=5))
    try:
        sim.prepare(4)
        sim.launch(0)
        sim.sync()
        with pytest.raises(BftsimError):
            sim.stats_allreduce()
    finally:
        sim.close()
