"""GPU: the pipelined launch mode of the benchmark (bftsim_set_pipeline) — a ring of row-table sets,
the block-hash pass of each launch on its set's stream overlapping the following launches —
gives the oracle's results for every launch, and the per-launch HIP-event timings are all read."""
import numpy as np
import pytest

import oracle_lib as O
from bftsim.configs import cfg3, BftConfig
from parity_util import assert_same

pytestmark = pytest.mark.gpu


def _sim(cfg):
    from bftsim.runtime import Simulator
    return Simulator(cfg)


@pytest.mark.parametrize("depth", [2, 3, 4])
@pytest.mark.parametrize("chain,batch,lstreams", [("wave", 4, 2), ("pair", 4, 2), ("pair", 1, 2), ("pair", 2, 1),
                                                  ("pair", 3, 1)])
def test_pipelined_launches_match_oracle(depth, chain, batch, lstreams, monkeypatch):
    """both chain kernels (one wave per instance below BFTSIM_CHAIN_WAVE_MAX, lane pairs above); the consensus
    kernels round-robin over launch streams, the chains of `batch` launches as one kernel on the hash
    streams (a set still waiting in the batch when the ring comes back to it is flushed first: depth < batch)"""
    monkeypatch.setenv("BFTSIM_TESTING", "1")
    monkeypatch.setenv("BFTSIM_CHAIN_WAVE_MAX", "1000000" if chain == "wave" else "0")
    monkeypatch.setenv("BFTSIM_HASH_BATCH", str(batch))
    monkeypatch.setenv("BFTSIM_LAUNCH_STREAMS", str(lstreams))
    cfg = cfg3(heights=30)
    n = 64
    sim = _sim(cfg)
    try:
        sim.set_pipeline(True, depth)
        sim.prepare(n)
        sim.kernel_ms_sum()
        for k in range(5):                       # the ring of sets wraps around
            sim.launch(k * n)
        sim.sync()
        got = sim.fetch()
        c, h, nl = sim.kernel_ms_sum()
        summ = sim.fetch_summary(n)
        st = sim.stats()
    finally:
        sim.close()
    ref = O.run(cfg, 4 * n, n)
    assert_same(ref, got, "pipelined launch 4")
    assert nl == 5 and c > 0 and h > 0
    tips = got["block_hash"][np.arange(n), got["committed_height"] - 1]
    assert np.array_equal(summ["tip_hash"], tips)
    assert st["views"] == int(ref["views"].sum())


@pytest.mark.parametrize("depth,batch,hstreams", [(16, 8, 3), (5, 8, 2), (12, 6, 4), (32, 16, 2), (7, 16, 3)])
def test_deep_ring_and_large_hash_batches(depth, batch, hstreams, monkeypatch):
    """rings up to 32 sets and chain kernels over up to 16 launches (a set still waiting in the batch when the
    ring comes back to it is flushed first: depth 5 < batch 8, 7 < 16), 20 launches of the same instances"""
    monkeypatch.setenv("BFTSIM_TESTING", "1")
    monkeypatch.setenv("BFTSIM_HASH_STREAMS", str(hstreams))
    cfg = cfg3(heights=30)
    n = 96
    sim = _sim(cfg)
    try:
        sim.set_pipeline(True, depth)
        sim.set_hash_batch(batch)
        sim.prepare(n)
        for k in range(20):
            sim.launch(k * n)
        got = sim.fetch()
    finally:
        sim.close()
    assert_same(O.run(cfg, 19 * n, n), got, f"depth {depth} batch {batch}")


def test_pipeline_toggle_and_sizes():
    cfg = BftConfig(n=16, heights=20, seed=21, drop_ppm=100_000)
    sim = _sim(cfg)
    try:
        for on in (True, False, True):
            sim.set_pipeline(on)
            sim.prepare(32)
            sim.launch(0)
            sim.launch(32)
            sim.sync()
            got = sim.fetch()
            assert_same(O.run(cfg, 32, 32), got, f"pipeline={on}")
    finally:
        sim.close()


def _timed_run(cfg, first, n, launches=25):
    """bench.py's timed mode for n instances per GPU: the pipeline depth and hash batch it picks
    (bftsim.configs.timed_pipeline), then `launches` launches of the same instances (its 5 warmup + 20 timed
    steps), the last one's results fetched."""
    from bftsim.configs import timed_pipeline
    depth, batch = timed_pipeline(n)
    sim = _sim(cfg)
    try:
        sim.set_pipeline(True, depth)
        sim.set_hash_batch(batch)
        sim.prepare(n)
        for _ in range(launches):
            sim.launch(first)
        sim.sync()
        got = sim.fetch()
        st = sim.stats()
    finally:
        sim.close()
    return got, st, (depth, batch)


def test_timed_mode_full_size():
    """The exact configuration of the headline number: cfg3 at 16,384 instances on one GPU with bench.py's
    pipeline depth and hash batch (32 x 8, lane-per-instance chains), 25 launches of the same instances; every
    instance against the oracle."""
    from bftsim.configs import INSTANCES
    cfg = cfg3()
    n = INSTANCES["cfg3"]
    got, st, (depth, batch) = _timed_run(cfg, 0, n)
    assert (depth, batch) == (32, 8)
    ref = O.run(cfg, 0, n, threads=16)
    assert_same(ref, got, f"cfg3 {n} depth {depth} batch {batch} x25")
    assert st["views"] == int(ref["views"].sum()) == n * 100


def test_strong_shard_timed_mode():
    """The 8-GPU strong-scaling shard of BASELINE configs[2] (rank 7's 2,048 of 16,384 instances) with the
    settings bench.py picks for it (depth 32 x batch 8, predicted chains), 25 launches; every instance against the
    oracle."""
    from bftsim.distributed import strong_shard
    cfg = cfg3()
    first, n = strong_shard(7, 8, 16_384)
    got, st, (depth, batch) = _timed_run(cfg, first, n)
    assert (n, depth, batch) == (2048, 32, 8)
    ref = O.run(cfg, first, n, threads=16)
    assert_same(ref, got, f"cfg3 shard {first}+{n} depth {depth} batch {batch} x25")
    assert st["views"] == int(ref["views"].sum()) == n * 100


def test_batch_split_on_launch_size_change():
    """A launch of another size while chains are pending in the hash batch starts a batch of its own (the
    chain kernel runs every launch of a batch with one instance count and suffix-row stride)."""
    cfg = cfg3(heights=30)
    sim = _sim(cfg)
    try:
        sim.set_pipeline(True, 8)
        sim.set_hash_batch(4)
        sim.prepare(96)
        sim.launch(0)
        a = sim.fetch()                          # flushes the pending batch
        sim.launch(96)
        sim.prepare(64)                          # fits the tables: no re-allocation, no flush
        sim.launch(300)
        sim.sync()
        b = sim.fetch()
        sim.prepare(96)
        sim.launch(500)
        sim.launch(700)
        sim.prepare(33)
        sim.launch(900)
        c = sim.fetch()
    finally:
        sim.close()
    assert_same(O.run(cfg, 0, 96), a, "96 at 0")
    assert_same(O.run(cfg, 300, 64), b, "64 after 96")
    assert_same(O.run(cfg, 900, 33), c, "33 after 96 x2")


@pytest.mark.gpu
def test_chunked_hash_pass(monkeypatch):
    """Heights hashed in chunks (the suffix rows of every height would exceed the 2 GiB per row-table set
    for large batches): chunks of 7 and 1 heights, each chunk's chains starting from the previous chunk's
    last hash, pipelined and not, against the oracle."""
    from bftsim.configs import cfg2
    monkeypatch.setenv("BFTSIM_TESTING", "1")
    for cfg, rows, depth in ((cfg3(heights=30), "7", 0), (cfg3(heights=30), "7", 3), (cfg3(heights=30), "1", 3),
                             (cfg2(heights=30), "7", 0), (cfg2(heights=30), "1", 3)):
        # cfg3: the FAST kernel (suffix rows by a thread per (instance, height)); cfg2: the general kernel
        # (a thread per instance over the chunk's heights)
        monkeypatch.setenv("BFTSIM_SFX_ROWS", rows)
        if True:
            sim = _sim(cfg)
            try:
                if depth:
                    sim.set_pipeline(True, depth)
                sim.prepare(96)
                for _ in range(2):
                    sim.launch(0)
                got = sim.fetch()
            finally:
                sim.close()
            assert_same(O.run(cfg, 0, 96), got, f"chunk rows {rows} depth {depth}")


@pytest.mark.parametrize("chain", ["wave", "pair"])
def test_small_shard_both_chain_kernels(chain, monkeypatch):
    """The 2,048-instance shard at pipeline depth 3 (concurrent launches, repeated launches of the same
    instances) with both chain kernels: one wave per instance (an A/B arm) and lane pairs (the product)."""
    monkeypatch.setenv("BFTSIM_TESTING", "1")
    monkeypatch.setenv("BFTSIM_CHAIN_WAVE_MAX", "1000000" if chain == "wave" else "0")
    cfg = cfg3()
    n = 2048
    sim = _sim(cfg)
    try:
        sim.set_pipeline(True, 3)
        sim.prepare(n)
        for _ in range(4):
            sim.launch(2048)
        sim.sync()
        got = sim.fetch()
        st = sim.stats()
    finally:
        sim.close()
    ref = O.run(cfg, 2048, n, threads=16)
    assert_same(ref, got, f"cfg3 2048 pipelined x4 ({chain})")
    assert st["views"] == int(ref["views"].sum()) == n * 100


@pytest.mark.parametrize("name,mk,depth,batch", [
    ("cfg3-30", lambda: cfg3(heights=30), 6, 2),
    ("n64-drop", lambda: BftConfig(n=64, heights=30, seed=17, byz_count=21, drop_ppm=50_000, name="n64-drop"), 8, 4),
    ("n64-crash", lambda: BftConfig(n=64, heights=30, seed=18, proposer_crash_ppm=300_000, name="n64-crash"), 4, 3),
    ("n64-silent0", lambda: BftConfig(n=64, heights=25, seed=19, byz_count=10, silent=[0, 5], name="n64-silent0"),
     5, 2),
    ("n64-fork", lambda: BftConfig(n=64, heights=30, seed=20, byz_count=30, drop_ppm=20_000, name="n64-fork"), 3, 5)])
def test_predicted_chains_match_oracle(name, mk, depth, batch, monkeypatch):
    """Big-endian seeds at N = 64, pipelined: the chains of a batch run on the predicted canonical
    blocks from launch time on; the recorded blocks are checked against the predictions and the chains re-run from
    the first one that differs. Lossless cfg3 (every prediction right), drops and forks (the repair from a height
    inside the chain), proposer crashes and a silent validator 0 (wrong from height 1: the whole chain repaired).
    12 launches of the same instances, with predictions on and off, against the oracle."""
    monkeypatch.setenv("BFTSIM_TESTING", "1")
    cfg = mk()
    n = 96
    outs = []
    for spec in ("2", "0"):                          # 2: predicted for lossy schedules too
        monkeypatch.setenv("BFTSIM_HASH_SPEC", spec)
        sim = _sim(cfg)
        try:
            sim.set_pipeline(True, depth)
            sim.set_hash_batch(batch)
            sim.prepare(n)
            for k in range(12):
                sim.launch(7 * n)
            sim.sync()
            outs.append(sim.fetch())
        finally:
            sim.close()
    ref = O.run(cfg, 7 * n, n)
    assert_same(ref, outs[0], name + " predicted chains")
    assert_same(ref, outs[1], name + " recorded chains")


@pytest.mark.parametrize("grid", ["0", "3"])
@pytest.mark.parametrize("inline", ["0", "1"])
@pytest.mark.parametrize("spec", ["2", "0"])
@pytest.mark.parametrize("name,mk", [("cfg3-30", lambda: cfg3(heights=30)),
                                     ("n64-drop", lambda: BftConfig(n=64, heights=30, seed=17, byz_count=21,
                                                                    drop_ppm=50_000, name="n64-drop"))])
def test_lane_chain_kernel(name, mk, spec, inline, grid, monkeypatch):
    """The lane-per-instance chain kernel (BFTSIM_CHAIN_LANE_MIN) in all three chain modes: recorded blocks, and
    predicted blocks with the repair from the first one that differs; the suffix spliced from the suffix rows or
    encoded by each lane from the recorded row or its own prediction (BFTSIM_CHAIN_INLINE); one wave per task or 3
    persistent waves for
    the whole batch (BFTSIM_CHAIN_GRID)."""
    monkeypatch.setenv("BFTSIM_TESTING", "1")
    monkeypatch.setenv("BFTSIM_CHAIN_LANE_MIN", "1")
    monkeypatch.setenv("BFTSIM_HASH_SPEC", spec)
    monkeypatch.setenv("BFTSIM_CHAIN_INLINE", inline)
    monkeypatch.setenv("BFTSIM_CHAIN_GRID", grid)
    cfg = mk()
    n = 160
    sim = _sim(cfg)
    try:
        sim.set_pipeline(True, 6)
        sim.set_hash_batch(3)
        sim.prepare(n)
        for k in range(7):
            sim.launch(3 * n)
        sim.sync()
        got = sim.fetch()
    finally:
        sim.close()
    assert_same(O.run(cfg, 3 * n, n), got, f"{name} lane chains, predicted={spec}")


@pytest.mark.parametrize("seed,byz,drop,crash,heights", [
    (31, 21, 0, 0, 60), (32, 0, 0, 0, 40), (33, 42, 0, 0, 50), (34, 21, 20_000, 0, 40), (35, 10, 0, 200_000, 40),
    (36, 30, 5_000, 0, 70)])
def test_predicted_lane_chains_sweep(seed, byz, drop, crash, heights, monkeypatch):
    """Predicted LANE chains (each lane predicts, masks and encodes its blocks; 56-dword LDS columns;
    the register-resident prefix) over seeds, Byzantine counts (0 .. 42), drops and proposer crashes, forced at a
    small size (BFTSIM_CHAIN_LANE_MIN=1; BFTSIM_HASH_SPEC=2: lossy schedules too), 9 launches in batches of 4,
    every instance against the oracle."""
    monkeypatch.setenv("BFTSIM_TESTING", "1")
    monkeypatch.setenv("BFTSIM_CHAIN_LANE_MIN", "1")
    monkeypatch.setenv("BFTSIM_HASH_SPEC", "2")
    cfg = BftConfig(n=64, heights=heights, seed=seed, byz_count=byz, drop_ppm=drop, proposer_crash_ppm=crash,
                    name=f"sweep{seed}")
    n = 192
    sim = _sim(cfg)
    try:
        sim.set_pipeline(True, 8)
        sim.set_hash_batch(4)
        sim.prepare(n)
        for _ in range(9):
            sim.launch(5 * n)
        sim.sync()
        got = sim.fetch()
    finally:
        sim.close()
    assert_same(O.run(cfg, 5 * n, n), got, f"predicted lane chains {cfg.name}")


@pytest.mark.parametrize("name,mk,depth", [
    ("cfg3-le",lambda: __import__("dataclasses").replace(cfg3(heights=40), seed_byte_order=1, name="cfg3-le"), 6),
    ("n64-le-drop", lambda: BftConfig(n=64, heights=20, seed=15, byz_count=21, drop_ppm=50_000, seed_byte_order=1,
                                      name="n64-le-drop"), 16)])
def test_little_endian_pipelined_predictions(name, mk, depth, monkeypatch):
    """Little-endian seeds at N = 64, pipelined: each launch runs its seed chain, FAST and resume
    kernels on one of the seeded launch streams; the predictions are taken while they match and the wave hashes
    from the first recorded block that differs (drops). 12 launches of the same instances; predictions on and
    off against the oracle."""
    monkeypatch.setenv("BFTSIM_TESTING", "1")
    cfg = mk()
    n = 96
    outs = []
    for spec in ("1", "0"):
        monkeypatch.setenv("BFTSIM_SEED_SPEC", spec)
        sim = _sim(cfg)
        try:
            sim.set_pipeline(True, depth)
            sim.prepare(n)
            for k in range(12):
                sim.launch(5 * n)
            sim.sync()
            outs.append(sim.fetch())
        finally:
            sim.close()
    ref = O.run(cfg, 5 * n, n)
    assert_same(ref, outs[0], name + " predictions")
    assert_same(ref, outs[1], name + " wave hash only")
