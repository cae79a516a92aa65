"""The HIP kernel bodies (bft_wave.h, bft_fast64.h) run by the CPU wave emulator against the oracle,
bit for bit: closed-form fast paths on and off, the N = 64 FAST kernel with its hand-overs, all
segment sizes."""
import pytest

import oracle_lib as O
import emu_lib as E
from bftsim.configs import BftConfig, cfg1, cfg2, cfg3, cfg4, cfg5
from parity_util import assert_same


def _le(cfg):
    import dataclasses
    return dataclasses.replace(cfg, seed_byte_order=1, name=cfg.name + "-le")


def _replay(cfg):
    import dataclasses
    return dataclasses.replace(cfg, backlog_mode=1, name=cfg.name + "-replay")

CASES = [
    ("cfg1-n5", lambda: cfg1(True, heights=40), 0, 1),
    ("cfg2", lambda: cfg2(heights=25), 0, 16),
    ("cfg3", lambda: cfg3(heights=10), 0, 2),
    ("cfg4-n10", lambda: cfg4(10, heights=25), 3, 8),
    ("cfg4-n33", lambda: cfg4(33, heights=15), 3, 2),
    ("cfg5", lambda: cfg5(heights=40), 0, 8),
    ("cfg2-byz", lambda: cfg2(heights=25, byz=1), 0, 16),
    ("cfg5-byz", lambda: cfg5(heights=40, byz=2), 0, 8),
    ("n7-byz3-drop", lambda: BftConfig(n=7, heights=25, seed=9, byz_count=3, drop_ppm=100_000), 0, 8),
    ("n4-cap2-drop30", lambda: BftConfig(n=4, heights=25, seed=12, drop_ppm=300_000, phase_cap=2), 0, 16),
    ("n16-crash-drop", lambda: BftConfig(n=16, heights=15, seed=21, drop_ppm=150_000,
                                         proposer_crash_ppm=300_000), 0, 4),
    # N = 64: the FAST kernel hands instances needing the general path over to the full kernel
    ("n64-fast-handover-drop", lambda: BftConfig(n=64, heights=10, seed=15, byz_count=21, drop_ppm=50_000), 0, 2),
    ("n64-fast-handover-crash", lambda: BftConfig(n=64, heights=10, seed=22, drop_ppm=100_000,
                                                  proposer_crash_ppm=300_000), 0, 2),
    ("cfg4-n64", lambda: cfg4(64, heights=12), 0, 3),
    # lossless N = 64 (the cfg3 shape): the FAST kernel's fused block-gossip phase, also with phase caps
    # that end a tick right at (3) or just after (4) the commit phase
    ("cfg3-40", lambda: cfg3(heights=40), 11, 4),
    ("n64-honest-40", lambda: BftConfig(n=64, heights=40, seed=44), 0, 3),
    ("n64-byz21-cap3", lambda: BftConfig(n=64, heights=20, seed=45, byz_count=21, phase_cap=3), 0, 3),
    ("n64-byz21-cap4", lambda: BftConfig(n=64, heights=20, seed=46, byz_count=21, phase_cap=4), 0, 3),
    # f >= N/3 equivocators at N = 64: forks freeze instances (the S = 64 commit resolution's safety path)
    ("n64-byz32-fork", lambda: BftConfig(n=64, heights=12, seed=31, byz_count=32), 0, 4),
    ("n64-byz40-drop5-fork", lambda: BftConfig(n=64, heights=12, seed=31, byz_count=40, drop_ppm=50_000), 0, 3),
    # workgroup segments (N > 64: 2 or 4 waves per instance, multi-word sender bitmaps)
    ("cfg4-n65", lambda: cfg4(65, heights=10), 5, 2),
    ("cfg4-n100", lambda: cfg4(100, heights=8), 0, 1),
    ("cfg4-n256", lambda: cfg4(256, heights=6), 2, 1),
    ("n130-byz43-drop", lambda: BftConfig(n=130, heights=8, seed=31, byz_count=43, drop_ppm=100_000), 0, 1),
    ("n200-silent-crash", lambda: BftConfig(n=200, heights=6, seed=32, silent=[0, 77, 199],
                                            proposer_crash_ppm=300_000), 0, 1),
    # little-endian U128 seed (bftsim.h BFTSIM_SEED_LE): every N needs in-kernel block hashes
    ("cfg1-n5-le", lambda: _le(cfg1(True, heights=30)), 0, 1),
    ("cfg2-le", lambda: _le(cfg2(heights=20)), 0, 16),
    ("cfg3-le", lambda: _le(cfg3(heights=8)), 0, 2),
    ("cfg4-n64-le", lambda: _le(cfg4(64, heights=10)), 0, 2),
    ("cfg4-n128-le", lambda: _le(cfg4(128, heights=6)), 0, 1),
    # N = 64 with little-endian seeds: the seed chain's predicted blocks, taken while they match (cfg3 shape),
    # left at the first height that differs (drops, forks, phase caps)
    ("cfg3-le-30", lambda: _le(cfg3(heights=30)), 5, 3),
    ("n64-le-drop", lambda: _le(BftConfig(n=64, heights=12, seed=15, byz_count=21, drop_ppm=50_000)), 0, 3),
    ("n64-le-byz32-fork", lambda: _le(BftConfig(n=64, heights=12, seed=31, byz_count=32)), 0, 3),
    ("n64-le-byz21-cap4", lambda: _le(BftConfig(n=64, heights=20, seed=46, byz_count=21, phase_cap=4)), 0, 3),
    # backlog replay mode (bftsim.h BFTSIM_BACKLOG_REPLAY, SPEC.md §10): every phase one message at a time
    ("cfg2-replay", lambda: _replay(cfg2(heights=30)), 0, 16),
    ("n4-drop30-replay", lambda: _replay(BftConfig(n=4, heights=25, seed=7, drop_ppm=300_000)), 0, 8),
    ("n7-byz2-drop-replay", lambda: _replay(BftConfig(n=7, heights=25, seed=8, byz_count=2,
                                                      drop_ppm=200_000)), 0, 8),
    ("n16-crash-drop-replay", lambda: _replay(BftConfig(n=16, heights=15, seed=3, drop_ppm=200_000,
                                                        proposer_crash_ppm=300_000)), 0, 4),
    ("n64-drop10-replay", lambda: _replay(BftConfig(n=64, heights=10, seed=5, drop_ppm=100_000)), 0, 2),
    ("n100-drop-replay", lambda: _replay(BftConfig(n=100, heights=8, seed=6, drop_ppm=200_000)), 0, 1),
    ("cfg2-le-replay", lambda: _replay(_le(cfg2(heights=20))), 0, 8),
]


@pytest.mark.parametrize("name,mk,first,n", CASES, ids=[c[0] for c in CASES])
def test_emulated_kernel_matches_oracle(name, mk, first, n):
    cfg = mk()
    assert_same(O.run(cfg, first, n), E.run(cfg, first, n), name)


def test_fast_paths_off_is_identical(monkeypatch):
    cfg = BftConfig(n=8, heights=20, seed=33, drop_ppm=120_000, byz_count=2)
    fast = E.run(cfg, 0, 8)
    monkeypatch.setenv("BFT_EMU_SLOW", "1")
    slow = E.run(cfg, 0, 8)
    assert_same(fast, slow, "fast vs one-message-at-a-time")
    assert_same(O.run(cfg, 0, 8), slow, "oracle vs slow")


STREAM_CASES = [
    ("cfg5-300", lambda: cfg5(heights=300), 0, 16, 64),
    ("cfg2-60", lambda: cfg2(heights=60), 100, 32, 64),
    ("cfg3-12", lambda: cfg3(heights=12), 7, 2, 64),
    ("cfg4-n100", lambda: cfg4(100, heights=8), 0, 1, 64),
    ("n7-crash-drop-w128", lambda: BftConfig(n=7, heights=200, seed=41, drop_ppm=150_000,
                                             proposer_crash_ppm=300_000), 0, 8, 128),
    ("cfg2-replay-w64", lambda: _replay(cfg2(heights=150)), 0, 8, 64),
]


@pytest.mark.parametrize("name,mk,first,n,window", STREAM_CASES, ids=[c[0] for c in STREAM_CASES])
def test_emulated_windowed_run_matches_streamed_oracle(name, mk, first, n, window):
    import numpy as np
    cfg = mk()
    ref = O.run_stream(cfg, first, n, threads=4)
    got = E.run_stream(cfg, first, n, window=window)
    for k in ("committed_height", "flags", "ticks", "views", "tip_hash", "round_hist", "latency_hist"):
        assert np.array_equal(ref[k], got[k]), (name, k)
    # the full-row kernel accumulates the same histograms in-kernel
    full = E.run(cfg, first, n)
    assert np.array_equal(full["round_hist"], ref["round_hist"])
    assert np.array_equal(full["latency_hist"], ref["latency_hist"])


@pytest.mark.parametrize("name,mk", [("cfg3", lambda: cfg3(heights=8)),
                                     ("cfg4-n64", lambda: cfg4(64, heights=8))])
def test_full_kernel_alone_n64(name, mk, monkeypatch):
    """bftsim_set_fast(h, 0) on the GPU: the full kernel runs N = 64 by itself."""
    monkeypatch.setenv("BFT_EMU_FAST", "0")
    cfg = mk()
    assert_same(O.run(cfg, 0, 2), E.run(cfg, 0, 2), name + " full kernel")


def test_block_hash_splice_matches_one_piece_encoder():
    """The block-hash pass encodes every height's header suffix in one parallel kernel and splices
    prev_hash in front in the chain (kern_fast.hip, bft_common.h header_suffix / splice_word). The
    splice equals the one-piece encoder of the header (SPEC.md §7) for random headers (and the device
    rows, dword-major across instances, hold the same dwords), including parents
    of all-high and all-low bytes (prefix 68 and 36 bytes, so 2- and 3-block messages) and heights /
    times at every MessagePack width boundary."""
    import ctypes
    lib = E.lib()
    lib.emu_splice_check.argtypes = [ctypes.c_uint32, ctypes.c_uint64]
    assert lib.emu_splice_check(20000, 12345) == 0
    assert lib.emu_splice_check(20000, 987654321) == 0


def test_wave_chain_matches_lane_splice():
    """The small-shard block-hash chain (bft_kwave.h kw50_chain, one wave per instance: the 50-lane Keccak,
    the prefix written byte-wise by 36 lanes with ballot prefix counts, lanes < 34 absorbing the spliced
    message dwords) gives the same chain of hashes as the lane splice (spliced_block_hash) over the same
    device-layout suffix rows, run by the emulator's 64 lane fibers: 2- and 3-block headers (parents of
    all-high / all-low bytes), heights and times across MessagePack width boundaries."""
    import ctypes
    lib = E.lib()
    lib.emu_wave_chain_check.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]
    assert lib.emu_wave_chain_check(24, 9, 4242) == 0
    assert lib.emu_wave_chain_check(12, 17, 77) == 0


def test_roundchangeset_capacity_overflow_is_flagged_and_local(monkeypatch):
    """The GPU RoundChangeSet holds a runtime number of rounds per validator (Params::rcs_k,
    bftsim_set_rcs_capacity); the reference's is an unbounded HashMap (round_change_set.rs:11-35). A
    validator that needs more sets BFTSIM_FLAG_RCS_OVERFLOW on its instance; every instance that did not
    overflow is exactly the oracle's (instances are independent), and at a capacity that suffices the
    whole batch is (bftsim_run re-runs an overflowing batch at twice the capacity)."""
    cfg = BftConfig(n=16, heights=30, seed=4, proposer_crash_ppm=300_000, name="cfg4-n16")
    ref = O.run(cfg, 0, 32)
    monkeypatch.setenv("BFT_EMU_RCS_K", "1")
    got = E.run(cfg, 0, 32)
    over = (got["flags"] & 32) != 0
    assert over.any() and not over.all()
    keep = ~over
    for k in ("committed_height", "ticks", "views", "flags"):
        assert (got[k][keep] == ref[k][keep]).all(), k
    for k in ("round", "proposer", "variant", "time_tick", "block_hash"):
        assert (got[k][keep] == ref[k][keep]).all(), k
    cfg7 = BftConfig(n=7, heights=30, seed=8, drop_ppm=300_000)
    monkeypatch.setenv("BFT_EMU_RCS_K", "2")
    assert ((E.run(cfg7, 0, 16)["flags"] & 32) != 0).all()
    monkeypatch.setenv("BFT_EMU_RCS_K", "8")
    assert_same(O.run(cfg7, 0, 16), E.run(cfg7, 0, 16), "n7-drop30 rcs_k=8")

def test_drop_draw_hoisted_products_match_philox():
    """deliver_mask's drop draw (bft_common.h philox_drop: round 1's products from the uniform instance
    word and a 64-bit add per 8-sender block, round 2's product uniform) gives the words of
    philox(seed, inst, tick, phase << 24 | recv << 8 | block, DOM_DROP), SPEC.md §3, on random counters
    and at the largest phase / receiver / block fields."""
    import ctypes
    lib = E.lib()
    lib.emu_philox_drop_check.argtypes = [ctypes.c_uint32, ctypes.c_uint64]
    assert lib.emu_philox_drop_check(200000, 31337) == 0


@pytest.mark.parametrize("name,mk,first,n", [
    ("cfg3-le", lambda: _le(cfg3(heights=30)), 0, 3),
    ("n64-le-drop", lambda: _le(BftConfig(n=64, heights=12, seed=15, byz_count=21, drop_ppm=50_000)), 3, 3),
    ("n64-le-honest", lambda: _le(BftConfig(n=64, heights=25, seed=47)), 0, 2)])
def test_seed_predictions_change_nothing(name, mk, first, n, monkeypatch):
    """Little-endian seeds at N = 64: the run with the seed chain's predicted blocks (Fast64::hash_pending
    takes a prediction while the recorded block equals it) equals the run where the wave hashes every
    height (BFT_EMU_SPEC=0), and both equal the oracle."""
    cfg = mk()
    with_spec = E.run(cfg, first, n)
    monkeypatch.setenv("BFT_EMU_SPEC", "0")
    without = E.run(cfg, first, n)
    assert_same(with_spec, without, name + " predictions on / off")
    assert_same(O.run(cfg, first, n), with_spec, name)


def test_general_body_fusions_are_taken(tmp_path, monkeypatch):
    """The general kernel's two shortcuts (bft_wave.h: the block-gossip phase after a uniform commit fused,
    the canonical view composed in one step) actually run: on cfg4 N = 256 (proposer crashes, no
    drops) the emulator's phase census sees no Blocks phase and about one phase per instance-round (3.1 without
    them), and the results equal the oracle's."""
    import ctypes
    import os
    import subprocess
    import numpy as np
    lib_path = str(tmp_path / "libwave_emu_census.so")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-Wno-unknown-pragmas", "-DBFT_CENSUS_BUILD",
                           "-o", lib_path, os.path.join(E.EMU_DIR, "wave_emu.cpp")])
    saved_lib, saved_path = E._lib, E.LIB
    try:
        E._lib, E.LIB = None, lib_path
        L = E.lib()
        L.emu_census.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        cfg = cfg4(256, heights=8)
        got = E.run(cfg, 0, 1)
        keys = np.zeros(256, np.uint32)
        cnt = np.zeros(256, np.uint64)
        m = L.emu_census(keys.ctypes.data, cnt.ctypes.data, 256)
        phases = int(cnt[:m].sum())
        kinds = [int(k) & 127 for k in keys[:m]]
        assert all(not (k >> 6) & 1 for k in kinds), "a Blocks phase was delivered"
        views = int(got["views"].sum())
        assert views > 0 and phases / views < 1.3, (phases, views)
    finally:
        E._lib, E.LIB = saved_lib, saved_path
    assert_same(O.run(cfg, 0, 1), got, "cfg4-n256 census run")
