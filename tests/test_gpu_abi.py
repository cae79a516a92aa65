"""Lifecycle of a libbftsim handle through the C ABI on the GPU: the requested instance count of a
prepare is what launch / fetch / stats use even when the buffers are larger (a smaller prepare after a
larger one), and a buffer reset (set_window / set_pipeline) invalidates the last launch's results
instead of reading freed memory."""
import ctypes

import numpy as np
import pytest

import oracle_lib as O
from bftsim import _abi, runtime
from bftsim.configs import cfg2, cfg3
from bftsim.runtime import Simulator
from parity_util import assert_same

pytestmark = pytest.mark.gpu


def test_prepare_shrinks_requested_count():
    cfg = cfg2(heights=20)
    sim = Simulator(cfg)
    try:
        sim.prepare(256)
        sim.launch(0)
        sim.sync()
        sim.prepare(64)                                # buffers stay, 64 instances run and come back
        sim.launch(0)
        got = sim.fetch()
        assert len(got["committed_height"]) == 64
        assert_same(O.run(cfg, 0, 64), got, "prepare 256 then 64")
        summ = sim.fetch_summary(64)
        assert np.array_equal(summ["committed_height"], got["committed_height"])
        assert sim.stats()["instances"] == 64
        # the synchronous path re-uses the larger buffers the same way
        got2 = sim.run(5, 10)
        assert_same(O.run(cfg, 5, 10), got2, "run 10 after prepare 256")
    finally:
        sim.close()


def test_buffer_reset_invalidates_last_launch():
    cfg = cfg3(heights=5)
    sim = Simulator(cfg)
    L = runtime.lib()
    try:
        sim.prepare(8)
        sim.launch(0)
        sim.sync()
        sim.set_window(64)                             # frees the row tables of that launch
        st = _abi.CStats()
        assert L.bftsim_stats_get(sim.h, ctypes.byref(st)) == -1
        assert L.bftsim_fetch_summary(sim.h, 8, None, None, None, None, None) == -1
        assert b"nothing launched" in L.bftsim_last_error(sim.h)
        sim.set_window(0)
        sim.prepare(8)
        sim.set_pipeline(True)                         # also re-sizes: again nothing to read
        assert L.bftsim_stats_get(sim.h, ctypes.byref(st)) == -1
        got = sim.run(0, 8)                            # and the handle still works afterwards
        assert_same(O.run(cfg, 0, 8), got, "after resets")
    finally:
        sim.close()


def test_short_result_buffers_are_refused_and_never_written():
    """The fetch family writes one row per launched instance: a buffer declared shorter than the launch
    (bftsim_launched_count) is refused with BFTSIM_EINVAL before anything is written (include/bftsim.h)."""
    cfg = cfg3(heights=5)
    sim = Simulator(cfg)
    L = runtime.lib()
    n, H = 64, cfg.heights
    try:
        sim.prepare(n)
        sim.launch(7)
        sim.sync()
        assert sim.launched() == (7, n)
        sentinel = 0xA5
        # bftsim_fetch: capacity n - 1
        r, arrs = _abi.alloc_result(n, H)
        for a in arrs.values():
            a.view(np.uint8)[:] = sentinel
        r.capacity = n - 1
        assert L.bftsim_fetch(sim.h, ctypes.byref(r)) == -1
        assert b"buffers hold 63 instances" in L.bftsim_last_error(sim.h)
        assert all((a.view(np.uint8) == sentinel).all() for a in arrs.values())
        r.capacity = n
        assert L.bftsim_fetch(sim.h, ctypes.byref(r)) == 0
        assert_same(O.run(cfg, 7, n), _abi.shape_result(arrs, n, H), "fetch at full capacity")
        # bftsim_fetch_summary
        ch = np.full(n, sentinel, np.uint64)
        tips = np.full((n, 32), sentinel, np.uint8)
        assert L.bftsim_fetch_summary(sim.h, n - 1, ch.ctypes.data, None, None, None, tips.ctypes.data) == -1
        assert (ch == sentinel).all() and (tips == sentinel).all()
        assert L.bftsim_fetch_summary(sim.h, n, ch.ctypes.data, None, None, None, tips.ctypes.data) == 0
        assert (ch == 5).all()
        # bftsim_export_headers
        buf = np.full(n * H * runtime.HEADER_SLOT, sentinel, np.uint8)
        lens = np.full(n * H, sentinel, np.uint32)
        assert L.bftsim_export_headers(sim.h, n - 1, buf.ctypes.data, lens.ctypes.data) == -1
        assert (buf == sentinel).all() and (lens == sentinel).all()
        assert L.bftsim_export_headers(sim.h, n, buf.ctypes.data, lens.ctypes.data) == 0
        assert (lens > 0).all()
        # bftsim_run: the requested n against the declared capacity
        r2, arrs2 = _abi.alloc_result(4, H)
        r2.capacity = 3
        assert L.bftsim_run(sim.h, 0, 4, ctypes.byref(r2)) == -1
        assert not any(a.any() for a in arrs2.values())
    finally:
        sim.close()
