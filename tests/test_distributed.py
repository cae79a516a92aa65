"""Multi-rank path on CPU (gloo, world_size 2): ranks shard instances with no data-path
collective and all-reduce the statistics; the reduced stats equal a single-process run."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from bftsim.distributed import strong_shard, weak_shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.join(os.path.dirname(here), "consensus-rs_amd"))
    import torch.distributed as dist
    import oracle_lib as O
    from bftsim.configs import cfg2
    from bftsim.distributed import all_reduce_stats, stats_from_result, weak_shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, n = weak_shard(rank, 8)
    st = stats_from_result(O.run_stream(cfg2(heights=15), first, n, threads=2))
    tot = all_reduce_stats(st)
    if rank == 0:
        q.put(tot)
    dist.barrier()
    dist.destroy_process_group()


def test_shard_helpers():
    assert weak_shard(3, 100) == (300, 100)
    parts = [strong_shard(r, 3, 10) for r in range(3)]
    assert parts == [(0, 4), (4, 3), (7, 3)]
    assert sum(n for _, n in parts) == 10


def test_gloo_world2_stats_equal_single_process():
    import oracle_lib as O
    from bftsim.configs import cfg2
    from bftsim.distributed import stats_from_result
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    tot = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    single = stats_from_result(O.run_stream(cfg2(heights=15), 0, 16, threads=2))
    assert tot == single
    assert sum(tot["latency_hist"]) == tot["committed_heights"] == sum(tot["round_hist"])
    # the per-height rows give the same rounds-to-commit histogram
    assert stats_from_result(O.run(cfg2(heights=15), 0, 16))["round_hist"] == single["round_hist"]


class _FakeSim:
    """stands in for Simulator in the comm-init decision: fails where told to. comm_init behaves like
    ncclCommInitRank: it returns only once every rank has entered it (a shared barrier), so a rank that
    fails before entering leaves the others blocked there -- the hang the pre-flight must prevent."""
    def __init__(self, fail_avail, fail_id, fail_init, barrier=None):
        self.fail_avail, self.fail_id, self.fail_init, self.barrier = fail_avail, fail_id, fail_init, barrier
        self.entered_init = False

    def comm_available(self):
        if self.fail_avail:
            raise RuntimeError("no librccl")

    def comm_unique_id(self):
        if self.fail_id:
            raise RuntimeError("no librccl")
        return bytes(128)

    def comm_init(self, world, rank, uid):
        assert uid == bytes(128)
        if self.fail_avail:                          # the old path: dlopen fails inside comm_init
            raise RuntimeError("dlopen librccl.so.1 failed")
        self.entered_init = True
        if self.barrier is not None:
            self.barrier.wait(timeout=20)            # threading.BrokenBarrierError = the old hang
        if self.fail_init:
            raise RuntimeError("init failed")


def _comm_worker(rank, world, port, q, fail_avail_rank, fail_id, fail_init_rank, barrier):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "consensus-rs_amd"))
    import torch.distributed as dist
    from bftsim.distributed import capi_comm_init
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sim = _FakeSim(rank == fail_avail_rank, fail_id and rank == 0, rank == fail_init_rank, barrier)
    try:
        ok = capi_comm_init(sim, rank, world)
    except Exception as e:                           # noqa: BLE001
        ok = f"raised {type(e).__name__}"
    q.put((rank, ok, sim.entered_init))
    dist.barrier()                                   # every rank reaches the same next collective
    dist.destroy_process_group()


@pytest.mark.parametrize("fail_avail_rank,fail_id,fail_init_rank,want", [
    (-1, False, -1, True), (-1, True, -1, False), (-1, False, 1, False), (1, False, -1, False), (0, False, -1, False)])
def test_comm_init_decision_is_collective(fail_avail_rank, fail_id, fail_init_rank, want):
    """bench.py's RCCL-or-fallback choice: a failure on any rank sends every rank to the same branch, and a
    rank that cannot open librccl stops everyone before anyone blocks in the (blocking) join"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    barrier = ctx.Barrier(2)
    port = _free_port()
    procs = [ctx.Process(target=_comm_worker, args=(r, 2, port, q, fail_avail_rank, fail_id, fail_init_rank, barrier))
             for r in range(2)]
    for p in procs:
        p.start()
    got = {r: (ok, entered) for r, ok, entered in (q.get(timeout=120) for _ in range(2))}
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert {r: ok for r, (ok, _) in got.items()} == {0: want, 1: want}
    if fail_avail_rank >= 0 or fail_id:              # nobody entered the blocking join
        assert not any(e for _, e in got.values())
