"""GPU: the in-kernel rounds-to-commit / commit-latency histograms and tip hashes, and windowed runs
(a ring of canonical rows, bftsim_set_window) for cfg5's long horizon — against the streamed oracle
(oracle/bft_oracle.c orc_run_stream), bit for bit."""
import numpy as np
import pytest

import oracle_lib as O
from bftsim.configs import BftConfig, cfg2, cfg3, cfg4, cfg5, INSTANCES

pytestmark = pytest.mark.gpu

KEYS = ("committed_height", "flags", "ticks", "views", "tip_hash", "round_hist", "latency_hist")


def _same(ref, got, what):
    for k in KEYS:
        assert np.array_equal(ref[k], got[k]), (what, k)


FULL = [
    ("cfg2-4096", lambda: cfg2(), 0, 4096),
    ("cfg3-512", lambda: cfg3(), 1000, 512),
    ("cfg4-n7-1024", lambda: cfg4(7), 0, 1024),
    ("cfg4-n200-64", lambda: cfg4(200), 0, 64),
]


@pytest.mark.parametrize("name,mk,first,n", FULL, ids=[c[0] for c in FULL])
def test_full_rows_histograms_and_tips(name, mk, first, n):
    from bftsim.runtime import Simulator
    cfg = mk()
    sim = Simulator(cfg)
    r = sim.run(first, n)
    summ = sim.fetch_summary(n)
    sim.close()
    got = dict(summ, round_hist=r["round_hist"], latency_hist=r["latency_hist"])
    _same(O.run_stream(cfg, first, n, threads=16), got, name)


WINDOWED = [
    ("cfg5-8192x1000-w128", lambda: cfg5(heights=1000), 0, 8192, 128),
    ("cfg2-full-w64", lambda: cfg2(), 5000, 4096, 64),
    ("cfg3-pow2-w64", lambda: cfg3(), 0, 256, 64),
    ("n10-crash-drop-w64", lambda: BftConfig(n=10, heights=400, seed=51, drop_ppm=100_000,
                                             proposer_crash_ppm=200_000), 0, 512, 64),
]


@pytest.mark.parametrize("name,mk,first,n,window", WINDOWED, ids=[c[0] for c in WINDOWED])
def test_windowed_run_matches_streamed_oracle(name, mk, first, n, window):
    from bftsim.runtime import Simulator
    cfg = mk()
    sim = Simulator(cfg)
    got = sim.run_stream(first, n, window=window)
    sim.close()
    _same(O.run_stream(cfg, first, n, threads=16), got, name)
    assert not (got["flags"] & 64).any()          # no lookup fell out of the ring


def test_cfg5_full_horizon_sampled():
    """cfg5's 10,000 heights on a 65,536-instance slice: whole-slice properties, bit-exact summaries
    of 256 sampled instances against the oracle."""
    from bftsim.runtime import Simulator
    cfg = cfg5()
    n = 65_536
    sim = Simulator(cfg)
    got = sim.run_stream(0, n, window=256)
    sim.close()
    assert (got["committed_height"] == cfg.heights).all()
    assert (got["flags"] == 0).all()
    assert int(got["round_hist"].sum()) == n * cfg.heights == int(got["latency_hist"].sum())
    # views = sum of (round + 1); bin 64 of the rounds histogram is an overflow bucket (round >= 64)
    part = sum(int(k + 1) * int(c) for k, c in enumerate(got["round_hist"][:64]))
    over = int(got["round_hist"][64])
    if over == 0:
        assert int(got["views"].sum()) == part
    else:
        assert int(got["views"].sum()) >= part + 65 * over
    idx = np.linspace(0, n - 1, 256).astype(np.int64)
    for i in idx[::32]:
        ref = O.run_stream(cfg, int(i), 32, threads=16)
        sl = slice(int(i), int(i) + 32)
        for k in ("committed_height", "flags", "ticks", "views", "tip_hash"):
            assert np.array_equal(ref[k], got[k][sl]), (int(i), k)
