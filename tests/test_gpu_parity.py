"""GPU parity: the HIP path (libbftsim through the C ABI) against the CPU oracle, bit for bit,
on the same seeded schedules (SPEC.md). Sizes are chosen so the oracle finishes in seconds."""
import numpy as np
import pytest

import oracle_lib as O
from bftsim.configs import BftConfig, cfg1, cfg2, cfg3, cfg4, cfg5
from parity_util import assert_same

pytestmark = pytest.mark.gpu


def _le(cfg):
    import dataclasses
    return dataclasses.replace(cfg, seed_byte_order=1, name=cfg.name + "-le")


def _replay(cfg):
    import dataclasses
    return dataclasses.replace(cfg, backlog_mode=1, name=cfg.name + "-replay")


def gpu_run(cfg, first, n, trace_ticks=0):
    from bftsim.runtime import Simulator
    sim = Simulator(cfg)
    try:
        return sim.run(first, n, trace_ticks)
    finally:
        sim.close()


CASES = [
    ("cfg1-n5", lambda: cfg1(True), 0, 1),
    ("cfg1-n4", lambda: cfg1(False), 0, 1),
    ("cfg2", lambda: cfg2(), 0, 256),
    ("cfg2-tail", lambda: cfg2(), 65_000, 64),
    ("cfg3", lambda: cfg3(), 0, 48),
    ("cfg3-tail", lambda: cfg3(), 16_300, 16),
    ("cfg5", lambda: cfg5(heights=300), 0, 64),
    # the tolerated f of cfg2 / cfg5 run as equivocating validators (SPEC.md §6)
    ("cfg2-byz", lambda: cfg2(byz=1), 0, 256),
    ("cfg5-byz", lambda: cfg5(heights=300, byz=2), 0, 64),
    ("n4-byz2-unsafe", lambda: BftConfig(n=4, heights=40, seed=9, byz_count=2), 0, 64),
    ("n64-byz32-fork", lambda: BftConfig(n=64, heights=20, seed=31, byz_count=32), 0, 32),
    ("n64-byz40-drop5-fork", lambda: BftConfig(n=64, heights=20, seed=31, byz_count=40, drop_ppm=50_000), 0, 16),
    ("n7-byz3-drop", lambda: BftConfig(n=7, heights=40, seed=9, byz_count=3, drop_ppm=100_000), 0, 64),
    ("n10-mix", lambda: BftConfig(n=10, heights=40, seed=11, byz_count=3, drop_ppm=200_000,
                                  proposer_crash_ppm=200_000), 0, 32),
    ("n4-cap3", lambda: BftConfig(n=4, heights=40, seed=12, drop_ppm=300_000, phase_cap=3), 0, 64),
    ("n16-drop40", lambda: BftConfig(n=16, heights=30, seed=13, drop_ppm=400_000), 0, 16),
    ("n5-2silent", lambda: BftConfig(n=5, heights=30, seed=14, silent=[0, 3]), 0, 8),
    ("n64-byz21-drop5", lambda: BftConfig(n=64, heights=20, seed=15, byz_count=21, drop_ppm=50_000), 0, 4),
    # lossless N = 64 with phase caps that end a tick at (3) or just after (4) the commit phase: the FAST
    # kernel's fused block-gossip phase at the cap boundary (bft_fast64.h run, p + 1 < phase_cap)
    ("n64-byz21-cap3", lambda: BftConfig(n=64, heights=20, seed=45, byz_count=21, phase_cap=3), 0, 16),
    ("n64-byz21-cap4", lambda: BftConfig(n=64, heights=20, seed=46, byz_count=21, phase_cap=4), 0, 16),
    ("n1", lambda: BftConfig(n=1, heights=20), 0, 8),
    ("n2", lambda: BftConfig(n=2, heights=20, drop_ppm=100_000), 0, 8),
    # N > 64: one workgroup of 128 / 256 lanes per instance
    ("n100-byz33-drop10", lambda: BftConfig(n=100, heights=30, seed=16, byz_count=33, drop_ppm=100_000), 0, 8),
    ("n256-byz85", lambda: BftConfig(n=256, heights=20, seed=17, byz_count=85), 0, 4),
    ("n129-silent-crash", lambda: BftConfig(n=129, heights=30, seed=18, silent=[0, 64, 128],
                                            proposer_crash_ppm=300_000, drop_ppm=20_000), 0, 8),
    # little-endian U128 seeds (include/bftsim.h BFTSIM_SEED_LE): block hashes in-kernel for every N
    ("cfg1-n5-le", lambda: _le(cfg1(True)), 0, 1),
    ("cfg2-le", lambda: _le(cfg2()), 0, 128),
    ("cfg3-le", lambda: _le(cfg3()), 0, 48),
    ("cfg4-n64-le", lambda: _le(cfg4(64, heights=60)), 0, 24),
    ("cfg4-n7-le", lambda: _le(cfg4(7, heights=60)), 0, 24),
    ("cfg4-n256-le", lambda: _le(cfg4(256, heights=30)), 0, 4),
    # backlog replay mode (BFTSIM_BACKLOG_REPLAY, SPEC.md §10): the general path with the backlog table
    ("cfg2-replay", lambda: _replay(cfg2()), 0, 256),
    ("cfg5-replay", lambda: _replay(cfg5(heights=200)), 0, 64),
    ("n4-drop30-replay", lambda: _replay(BftConfig(n=4, heights=40, seed=7, drop_ppm=300_000)), 0, 64),
    ("n7-byz2-drop-replay", lambda: _replay(BftConfig(n=7, heights=40, seed=8, byz_count=2,
                                                      drop_ppm=200_000)), 0, 32),
    ("cfg4-n16-replay", lambda: _replay(cfg4(16, heights=40)), 0, 16),
    ("n64-drop10-replay", lambda: _replay(BftConfig(n=64, heights=20, seed=5, drop_ppm=100_000)), 0, 8),
    ("cfg3-replay", lambda: _replay(cfg3(heights=30)), 0, 8),
    ("n100-drop-replay", lambda: _replay(BftConfig(n=100, heights=20, seed=6, drop_ppm=200_000)), 0, 4),
    ("n256-drop-replay", lambda: _replay(BftConfig(n=256, heights=10, seed=6, drop_ppm=100_000)), 0, 2),
] + [(f"cfg4-n{n}", (lambda n=n: cfg4(n, heights=60)), 0, 24)
     for n in (4, 7, 10, 16, 31, 32, 33, 63, 64, 65, 100, 128, 200, 256)]


@pytest.mark.parametrize("name,mk,first,n", CASES, ids=[c[0] for c in CASES])
def test_gpu_matches_oracle(name, mk, first, n):
    cfg = mk()
    ref = O.run(cfg, first, n)
    got = gpu_run(cfg, first, n)
    assert_same(ref, got, name)


@pytest.mark.parametrize("name,mk,n", [("cfg3", lambda: cfg3(heights=30), 16),
                                       ("n64-byz21-drop5", lambda: BftConfig(n=64, heights=20, seed=15, byz_count=21,
                                                                             drop_ppm=50_000), 8)])
def test_gpu_full_kernel_alone_n64(name, mk, n, monkeypatch):
    """bftsim_set_fast(h, 0): N = 64 through the full kernel alone (no FAST kernel, no hand-over)."""
    from bftsim.runtime import Simulator
    cfg = mk()
    sim = Simulator(cfg)
    try:
        sim.set_fast(False)
        got = sim.run(0, n)
    finally:
        sim.close()
    assert_same(O.run(cfg, 0, n), got, name + " full kernel")


@pytest.mark.gpu
def test_gpu_roundchangeset_capacity_grows_until_no_overflow():
    """A RoundChangeSet capacity of one round overflows on a lossy N=7 batch and a crash-storm N=16
    batch; bftsim_run re-runs at twice the capacity until no instance overflows (the reference's map is
    unbounded, round_change_set.rs:11-35), and the outputs are the oracle's."""
    from bftsim.runtime import Simulator
    for cfg, n in ((BftConfig(n=7, heights=30, seed=8, drop_ppm=300_000), 64),
                   (BftConfig(n=16, heights=30, seed=4, proposer_crash_ppm=300_000, name="cfg4-n16"), 64)):
        sim = Simulator(cfg)
        try:
            sim.set_rcs_capacity(1)
            got = sim.run(0, n)
        finally:
            sim.close()
        assert not ((got["flags"] & 32) != 0).any()
        assert_same(O.run(cfg, 0, n), got, f"{cfg.name} rcs capacity 1 -> grown")
