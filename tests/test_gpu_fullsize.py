"""GPU at BASELINE.json's full sizes: bit-exact parity against the (multithreaded) oracle over
EVERY instance, size-independent properties (the oracle re-hashes every committed header chain in
C; quorum/liveness invariants), determinism, shard independence and the stats reduction."""
import numpy as np
import pytest

import oracle_lib as O
from bftsim.configs import cfg2, cfg3, cfg4, INSTANCES
from bftsim.distributed import stats_from_result
from parity_util import FIELDS, assert_same

pytestmark = pytest.mark.gpu


def _sim(cfg):
    from bftsim.runtime import Simulator
    return Simulator(cfg)


def _take(r, idx):
    return {k: r[k][idx] for k in FIELDS}


def _full_parity(cfg, got, first, n):
    ref = O.run(cfg, first, n, threads=16)
    assert_same(ref, got, f"{cfg.name} [{first}, {first + n})")


def test_cfg3_full_16384():
    cfg = cfg3()
    sim = _sim(cfg)
    n = INSTANCES["cfg3"]
    r = sim.run(0, n)
    sim.close()
    assert (r["committed_height"] == 100).all()
    assert (r["flags"] == 0).all()
    assert (r["round"] == 0).all()              # equivocation never needs a round change
    assert int(r["views"].sum()) == n * 100
    assert O.verify_chains(cfg, 0, r, threads=16) == 0
    assert set(np.unique(r["variant"])) == {0, 1}
    _full_parity(cfg, r, 0, n)


def test_cfg3_full_16384_little_endian_seed():
    # BFTSIM_SEED_LE: the proposer of every height depends on the previous block hash, so N = 64
    # runs with in-kernel hashes; every instance against the oracle
    import dataclasses
    cfg = dataclasses.replace(cfg3(), seed_byte_order=1, name="cfg3-le")
    sim = _sim(cfg)
    n = INSTANCES["cfg3"]
    r = sim.run(0, n)
    sim.close()
    assert (r["committed_height"] == 100).all()
    assert O.verify_chains(cfg, 0, r, threads=16) == 0
    assert len(np.unique(r["proposer"])) == 64        # proposers vary with the hashes (BE: round 0 is 0)
    _full_parity(cfg, r, 0, n)


def test_cfg2_full_65536():
    cfg = cfg2()
    sim = _sim(cfg)
    n = INSTANCES["cfg2"]
    r = sim.run(0, n)
    sim.close()
    done = r["committed_height"] == 100
    # 10% drops: a few instances livelock in round changes until max_ticks (the oracle agrees)
    assert done.mean() > 0.999
    assert (r["flags"][~done] & 16).all()
    assert (r["flags"][done] == 0).all()
    assert O.verify_chains(cfg, 0, r, threads=16) == 0
    assert (r["round"] > 0).mean() > 0.02          # drops cause round changes
    _full_parity(cfg, r, 0, n)


@pytest.mark.parametrize("nv", [4, 7, 16, 31, 64])
def test_cfg4_sweep_4096(nv):
    cfg = cfg4(nv)
    sim = _sim(cfg)
    r = sim.run(0, 4096)
    sim.close()
    assert (r["committed_height"] == 100).all()
    assert O.verify_chains(cfg, 0, r, threads=16) == 0
    _full_parity(cfg, r, 0, 4096)


@pytest.mark.parametrize("nv", [65, 100, 128, 200, 256])
def test_cfg4_large_n(nv):
    # N > 64 (workgroup segments): whole-output oracle parity on 512 instances, 100 heights
    cfg = cfg4(nv)
    sim = _sim(cfg)
    r = sim.run(0, 512)
    sim.close()
    assert (r["committed_height"] == 100).all()
    assert O.verify_chains(cfg, 0, r, threads=16) == 0
    _full_parity(cfg, r, 0, 512)


def test_determinism_shards_and_stats():
    cfg = cfg2(heights=40)
    sim = _sim(cfg)
    a = sim.run(1000, 2048)
    b = sim.run(1000, 2048)
    c1 = sim.run(1000, 777)
    c2 = sim.run(1777, 2048 - 777)
    for k in FIELDS:
        assert np.array_equal(a[k], b[k]), k
        assert np.array_equal(np.concatenate([c1[k], c2[k]]), a[k]), k
    sim.prepare(2048)
    sim.launch(1000)
    st = sim.stats()
    sim.close()
    assert st == stats_from_result(a)
