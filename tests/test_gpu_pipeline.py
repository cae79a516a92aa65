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


def test_timed_mode_full_size():
    """The exact mode bench.py times: cfg3 at 16,384 instances, pipeline depth 3 (so the hash pass is
    the block-hash pass (bft_hash_suffix_kernel + bft_hash_chain_kernel) on its set's stream under the ring), repeated launches of the same instances;
    the last launch's results against the oracle over every instance."""
    from bftsim.configs import INSTANCES
    cfg = cfg3()
    n = INSTANCES["cfg3"]
    sim = _sim(cfg)
    try:
        sim.set_pipeline(True, 3)
        sim.prepare(n)
        for _ in range(5):                       # wraps the ring of three sets
            sim.launch(0)
        sim.sync()
        got = sim.fetch()
        st = sim.stats()
    finally:
        sim.close()
    ref = O.run(cfg, 0, n, threads=16)
    assert_same(ref, got, "cfg3 16384 pipelined x5")
    assert st["views"] == int(ref["views"].sum()) == n * 100


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
def test_small_shard_timed_mode(chain, monkeypatch):
    """The strong-scaling shard of 8 GPUs (2,048 cfg3 instances per GPU), as bench.py times it (pipeline depth
    3, concurrent launches, repeated launches of the same instances), with both chain kernels."""
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


@pytest.mark.parametrize("name,mk,depth", [
    ("cfg3-le", lambda: __import__("dataclasses").replace(cfg3(heights=40), seed_byte_order=1, name="cfg3-le"), 6),
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
