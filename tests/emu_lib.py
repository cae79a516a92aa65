"""ctypes wrapper of the CPU wave emulator (tests/emu/libwave_emu.so) — test-only."""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "consensus-rs_amd"))
from bftsim import _abi  # noqa: E402

EMU_DIR = os.path.join(ROOT, "tests", "emu")
LIB = os.path.join(EMU_DIR, "libwave_emu.so")
SRCS = [os.path.join(EMU_DIR, "wave_emu.cpp")] + [
    os.path.join(ROOT, "consensus-rs_amd", "csrc", f) for f in ("bft_wave.h", "bft_fast64.h", "bft_kwave.h", "bft_common.h", "bft_host.h")]

_lib = None


def build():
    if os.path.exists(LIB) and all(os.path.getmtime(LIB) >= os.path.getmtime(s) for s in SRCS):
        return
    # build to a private name and rename: concurrent test workers never load a half-written library
    tmp = f"{LIB}.{os.getpid()}.tmp"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-Wno-unknown-pragmas", "-DBFT_EMU_CHECKS",
                           "-o", tmp, SRCS[0]])
    os.replace(tmp, LIB)


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(LIB)
        _lib.emu_run.argtypes = [ctypes.POINTER(_abi.CConfig), ctypes.c_uint64, ctypes.c_uint64,
                                 ctypes.POINTER(_abi.CResult), ctypes.c_void_p, ctypes.c_uint32,
                                 ctypes.c_void_p]
        _lib.emu_run_stream.argtypes = [ctypes.POINTER(_abi.CConfig), ctypes.c_uint64, ctypes.c_uint64,
                                        ctypes.c_uint32] + [ctypes.c_void_p] * 6
    return _lib


def run(cfg, first, n_inst, trace_ticks=0):
    c, keep = _abi.to_cconfig(cfg)
    r, arrs = _abi.alloc_result(n_inst, cfg.heights)
    tr = None
    if trace_ticks:
        tr = np.zeros(n_inst * trace_ticks * cfg.n, np.uint64)
    hist = np.zeros(130, np.uint64)
    rc = lib().emu_run(ctypes.byref(c), first, n_inst, ctypes.byref(r),
                       tr.ctypes.data if tr is not None else None, trace_ticks, hist.ctypes.data)
    del keep
    if rc != 0:
        raise RuntimeError(f"emu_run failed: {rc}")
    arrs = _abi.shape_result(arrs, n_inst, cfg.heights)
    if tr is not None:
        arrs["trace"] = tr.reshape(n_inst, trace_ticks, cfg.n)
    arrs["round_hist"], arrs["latency_hist"] = hist[:65], hist[65:]
    return arrs


def run_crypto(cfg, first, n_inst, forged=(), cap=4096):
    """The kernel body in real-crypto mode (SPEC.md §11): results + the per-instance broadcast log."""
    fm = np.zeros(4, np.uint64)
    for v in forged:
        fm[v >> 6] |= np.uint64(1) << np.uint64(v & 63)
    mlog = np.zeros((n_inst, cap, 8), np.uint32)
    mlog_n = np.zeros(n_inst, np.uint32)
    L = lib()
    L.emu_set_crypto.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint32]
    L.emu_set_crypto(fm.ctypes.data, mlog.ctypes.data, mlog_n.ctypes.data, cap)
    out = run(cfg, first, n_inst)
    out["mlog"], out["mlog_n"] = mlog, mlog_n
    return out


def run_stream(cfg, first, n_inst, window=128):
    """The windowed kernel body (ring of `window` rows, in-kernel hashes): per-instance outputs,
    tip hashes and the two histograms."""
    c, keep = _abi.to_cconfig(cfg)
    out = dict(committed_height=np.zeros(n_inst, np.uint32), flags=np.zeros(n_inst, np.uint32),
               ticks=np.zeros(n_inst, np.uint32), views=np.zeros(n_inst, np.uint64),
               tip_hash=np.zeros((n_inst, 32), np.uint8))
    hist = np.zeros(130, np.uint64)
    rc = lib().emu_run_stream(ctypes.byref(c), first, n_inst, window, out["committed_height"].ctypes.data,
                              out["flags"].ctypes.data, out["ticks"].ctypes.data, out["views"].ctypes.data,
                              out["tip_hash"].ctypes.data, hist.ctypes.data)
    del keep
    if rc != 0:
        raise RuntimeError(f"emu_run_stream failed: {rc}")
    out["round_hist"], out["latency_hist"] = hist[:65], hist[65:]
    return out
