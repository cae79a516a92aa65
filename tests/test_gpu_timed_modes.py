"""GPU: each secondary bench line's timed mode at the size it is timed. The workload, the instances per GPU, the
launches (warmup + timed steps) and the pipeline settings come from bftsim.configs, where bench.py takes them too
(bench_config, bench_instances, bench_steps, timed_pipeline, CFG5_WINDOW), so a change of the bench's settings is a
change of these tests. Every instance is checked against the oracle where the oracle finishes in minutes (cfg2,
drop64, cfg4 N = 256); cfg5's 131,072 x 10,000 heights by whole-slice properties and 256 sampled instances.
The headline (cfg3) and its 8-GPU shard are pinned in test_gpu_pipeline.py."""
import numpy as np
import pytest

import oracle_lib as O
from bftsim.configs import CFG5_WINDOW, bench_config, bench_instances, bench_steps, timed_pipeline
from parity_util import assert_same

pytestmark = pytest.mark.gpu


def _timed(wl, cfg, first=0):
    """bench.py's pipelined launches of `wl`: warmup launches, a sync, the timed launches, the last one fetched."""
    from bftsim.runtime import Simulator
    n = bench_instances(wl)
    steps, warmup = bench_steps(wl)
    depth, batch = timed_pipeline(n)
    sim = Simulator(cfg)
    try:
        sim.set_pipeline(True, depth)
        sim.set_hash_batch(batch)
        sim.prepare(n)
        for _ in range(warmup):
            sim.launch(first)
        sim.sync()
        for _ in range(steps):
            sim.launch(first)
        sim.sync()
        got = sim.fetch()
        st = sim.stats()
    finally:
        sim.close()
    return n, got, st, (steps, warmup, depth, batch)


@pytest.mark.parametrize("wl,nv", [("cfg2", 4), ("drop64", 64), ("cfg4", 256)])
def test_timed_mode_full_size(wl, nv):
    """cfg2 (65,536 x N = 4, 10 % drop; the general kernel, lane chains), drop64 (16,384 x N = 64 with 5 % drop;
    FAST + resume, lane chains) and cfg4 N = 256 (16,384, proposer crashes; workgroup segments), each at bench.py's
    timed settings, every instance of the last launch against the oracle."""
    cfg = bench_config(wl, n=nv)
    n, got, st, mode = _timed(wl, cfg)
    ref = O.run(cfg, 0, n, threads=16)
    assert_same(ref, got, f"{wl} {n} steps/warmup/depth/batch {mode}")
    assert st["views"] == int(ref["views"].sum())


def test_cfg5_timed_mode_full_size():
    """cfg5 as bench.py times it: 131,072 instances x 10,000 heights in one windowed launch (rows kept in a ring
    of CFG5_WINDOW, block hashes in-kernel). Whole-slice properties; 256 instances spread over the slice against the
    streamed oracle bit for bit."""
    from bftsim.runtime import Simulator
    wl = "cfg5"
    cfg = bench_config(wl)
    n = bench_instances(wl)
    sim = Simulator(cfg)
    try:
        got = sim.run_stream(0, n, window=CFG5_WINDOW)
    finally:
        sim.close()
    assert n == 131_072 and cfg.heights == 10_000
    assert (got["committed_height"] == cfg.heights).all()
    assert (got["flags"] == 0).all()
    assert int(got["round_hist"].sum()) == n * cfg.heights == int(got["latency_hist"].sum())
    idx = np.linspace(0, n - 32, 8).astype(np.int64)
    for i in idx:                                  # 8 runs of 32 consecutive instances
        ref = O.run_stream(cfg, int(i), 32, threads=16)
        sl = slice(int(i), int(i) + 32)
        for k in ("committed_height", "flags", "ticks", "views", "tip_hash"):
            assert np.array_equal(ref[k], got[k][sl]), (int(i), k)
