"""ctypes wrapper of the CPU oracle (oracle/_build/liboracle.so). Test infrastructure only."""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "consensus-rs_amd"))
from bftsim.configs import BftConfig  # noqa: E402

LIB_PATH = os.path.join(ROOT, "oracle", "_build", "liboracle.so")


class OrcConfig(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint32), ("heights", ctypes.c_uint32), ("max_ticks", ctypes.c_uint32),
        ("block_period", ctypes.c_uint32), ("genesis_time", ctypes.c_uint64),
        ("seed", ctypes.c_uint64), ("drop_ppm", ctypes.c_uint32), ("byz_count", ctypes.c_uint32),
        ("proposer_crash_ppm", ctypes.c_uint32), ("phase_cap", ctypes.c_uint32),
        ("silent_mask", ctypes.c_uint64 * 4), ("addresses", ctypes.c_void_p),
        ("genesis_proposer", ctypes.c_uint8 * 20), ("genesis_gas_used", ctypes.c_uint64),
        ("seed_byte_order", ctypes.c_uint32), ("header_encoding", ctypes.c_uint32),
        ("backlog_mode", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
    ]


class OrcResult(ctypes.Structure):
    _fields_ = [(k, ctypes.c_void_p) for k in (
        "committed_height", "flags", "ticks", "views", "round", "proposer", "variant",
        "time_tick", "block_hash")]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        _lib = ctypes.CDLL(LIB_PATH)
        _lib.orc_run.argtypes = [ctypes.POINTER(OrcConfig), ctypes.c_uint64, ctypes.c_uint64,
                                 ctypes.POINTER(OrcResult)]
        _lib.orc_run_threads.argtypes = [ctypes.POINTER(OrcConfig), ctypes.c_uint64,
                                         ctypes.c_uint64, ctypes.POINTER(OrcResult),
                                         ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
        _lib.orc_trace.argtypes = [ctypes.POINTER(OrcConfig), ctypes.c_uint64, ctypes.c_void_p,
                                   ctypes.c_uint32]
        _lib.orc_two_thirds_majority.restype = ctypes.c_uint32
        _lib.orc_seed_from_hash.restype = ctypes.c_uint32
        _lib.orc_encode_header.restype = ctypes.c_size_t
        _lib.orc_encode_header.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                           ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                           ctypes.c_char_p, ctypes.c_size_t]
        _lib.orc_seed_from_hash.argtypes = [ctypes.c_char_p, ctypes.c_uint32]
        _lib.orc_seed_from_hash_order.restype = ctypes.c_uint32
        _lib.orc_seed_from_hash_order.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32]
        _lib.orc_two_thirds_majority.argtypes = [ctypes.c_uint32]
    return _lib


def to_orc(cfg: BftConfig):
    c = OrcConfig()
    c.n, c.heights, c.max_ticks = cfg.n, cfg.heights, cfg.max_ticks
    c.block_period, c.genesis_time, c.seed = cfg.block_period, cfg.genesis_time, cfg.seed
    c.drop_ppm, c.byz_count = cfg.drop_ppm, cfg.byz_count
    c.proposer_crash_ppm, c.phase_cap = cfg.proposer_crash_ppm, cfg.phase_cap
    for i, m in enumerate(cfg.silent_mask()):
        c.silent_mask[i] = m
    addr = ctypes.create_string_buffer(cfg.address_bytes(), 20 * cfg.n)
    c.addresses = ctypes.cast(addr, ctypes.c_void_p)
    for i, b in enumerate(cfg.genesis_proposer):
        c.genesis_proposer[i] = b
    c.genesis_gas_used = cfg.genesis_gas_used
    c.seed_byte_order = cfg.seed_byte_order
    c.header_encoding = 0
    c.backlog_mode = cfg.backlog_mode
    return c, addr


def alloc_result(n_inst: int, heights: int):
    arrs = dict(
        committed_height=np.zeros(n_inst, np.uint32), flags=np.zeros(n_inst, np.uint32),
        ticks=np.zeros(n_inst, np.uint32), views=np.zeros(n_inst, np.uint64),
        round=np.zeros(n_inst * heights, np.uint16), proposer=np.zeros(n_inst * heights, np.uint16),
        variant=np.zeros(n_inst * heights, np.uint8), time_tick=np.zeros(n_inst * heights, np.uint32),
        block_hash=np.zeros(n_inst * heights * 32, np.uint8))
    r = OrcResult()
    for k, a in arrs.items():
        setattr(r, k, a.ctypes.data)
    return r, arrs


def run(cfg: BftConfig, first: int, n_inst: int, threads: int = 1):
    c, keep = to_orc(cfg)
    r, arrs = alloc_result(n_inst, cfg.heights)
    secs = ctypes.c_double(0)
    if threads > 1:
        lib().orc_run_threads(ctypes.byref(c), first, n_inst, ctypes.byref(r), threads,
                              ctypes.byref(secs))
    else:
        lib().orc_run(ctypes.byref(c), first, n_inst, ctypes.byref(r))
    del keep
    H = cfg.heights
    arrs["round"] = arrs["round"].reshape(n_inst, H)
    arrs["proposer"] = arrs["proposer"].reshape(n_inst, H)
    arrs["variant"] = arrs["variant"].reshape(n_inst, H)
    arrs["time_tick"] = arrs["time_tick"].reshape(n_inst, H)
    arrs["block_hash"] = arrs["block_hash"].reshape(n_inst, H, 32)
    arrs["seconds"] = secs.value
    return arrs


def run_crypto(cfg: BftConfig, first: int, n_inst: int, forged=(), cap: int = 4096):
    """orc_run_crypto (SPEC.md §11): results + the per-instance broadcast log [n][cap][8] and counts."""
    c, keep = to_orc(cfg)
    r, arrs = alloc_result(n_inst, cfg.heights)
    fm = (ctypes.c_uint64 * 4)()
    for v in forged:
        fm[v >> 6] |= 1 << (v & 63)
    mlog = np.zeros((n_inst, cap, 8), np.uint32)
    mlog_n = np.zeros(n_inst, np.uint32)
    L = lib()
    L.orc_run_crypto.argtypes = [ctypes.POINTER(OrcConfig), ctypes.c_uint64, ctypes.c_uint64,
                                 ctypes.POINTER(OrcResult), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_uint32]
    L.orc_run_crypto(ctypes.byref(c), first, n_inst, ctypes.byref(r), ctypes.cast(fm, ctypes.c_void_p),
                     mlog.ctypes.data, mlog_n.ctypes.data, cap)
    del keep
    H = cfg.heights
    for k in ("round", "proposer", "variant", "time_tick"):
        arrs[k] = arrs[k].reshape(n_inst, H)
    arrs["block_hash"] = arrs["block_hash"].reshape(n_inst, H, 32)
    arrs["mlog"], arrs["mlog_n"] = mlog, mlog_n
    return arrs


def verify_chains(cfg: BftConfig, first: int, res: dict, threads: int = 8) -> int:
    """Re-hash every committed header chain of a result dict (any producer); returns the number
    of instances that do not verify."""
    n = len(res["committed_height"])
    c, keep = to_orc(cfg)
    dt = dict(committed_height=np.uint32, flags=np.uint32, ticks=np.uint32, views=np.uint64, round=np.uint16,
              proposer=np.uint16, variant=np.uint8, time_tick=np.uint32, block_hash=np.uint8)
    arrs = {k: np.ascontiguousarray(res[k], dtype=t).reshape(-1) for k, t in dt.items()}
    r = OrcResult()
    for k, a in arrs.items():
        setattr(r, k, a.ctypes.data)
    L = lib()
    L.orc_verify_chains.restype = ctypes.c_uint64
    L.orc_verify_chains.argtypes = [ctypes.POINTER(OrcConfig), ctypes.c_uint64, ctypes.c_uint64,
                                    ctypes.POINTER(OrcResult), ctypes.c_int]
    bad = L.orc_verify_chains(ctypes.byref(c), first, n, ctypes.byref(r), threads)
    del keep
    return int(bad)


class OrcStream(ctypes.Structure):
    _fields_ = [("committed_height", ctypes.c_void_p), ("flags", ctypes.c_void_p),
                ("ticks", ctypes.c_void_p), ("views", ctypes.c_void_p), ("tip_hash", ctypes.c_void_p),
                ("hist", ctypes.c_uint64 * 130)]


def run_stream(cfg: BftConfig, first: int, n_inst: int, threads: int = 8):
    """Streamed run: per-instance totals, tip hashes and the summed rounds-to-commit (hist[:65])
    and commit-latency (hist[65:]) histograms."""
    c, keep = to_orc(cfg)
    arrs = dict(committed_height=np.zeros(n_inst, np.uint32), flags=np.zeros(n_inst, np.uint32),
                ticks=np.zeros(n_inst, np.uint32), views=np.zeros(n_inst, np.uint64),
                tip_hash=np.zeros((n_inst, 32), np.uint8))
    st = OrcStream()
    for k, a in arrs.items():
        setattr(st, k, a.ctypes.data)
    L = lib()
    L.orc_run_stream.argtypes = [ctypes.POINTER(OrcConfig), ctypes.c_uint64, ctypes.c_uint64,
                                 ctypes.POINTER(OrcStream), ctypes.c_int]
    L.orc_run_stream(ctypes.byref(c), first, n_inst, ctypes.byref(st), threads)
    del keep
    h = np.array(st.hist[:], dtype=np.uint64)
    arrs["round_hist"] = h[:65]
    arrs["latency_hist"] = h[65:]
    return arrs


def trace(cfg: BftConfig, instance: int, max_rec: int = 512):
    c, keep = to_orc(cfg)
    out = np.zeros(max_rec * cfg.n, np.uint64)
    lib().orc_trace(ctypes.byref(c), instance, out.ctypes.data, max_rec)
    del keep
    return out.reshape(max_rec, cfg.n)


def keccak256(data: bytes) -> bytes:
    o = (ctypes.c_uint8 * 32)()
    lib().orc_keccak256(data, len(data), o)
    return bytes(o)


def secp_pubkey(secret: bytes):
    """C oracle (oracle/secp_oracle.c): 64-byte public key or None."""
    out = (ctypes.c_uint8 * 64)()
    return bytes(out) if lib().orc_secp_pubkey(secret, out) else None


def secp_recover(msg: bytes, sig: bytes):
    out = (ctypes.c_uint8 * 64)()
    return bytes(out) if lib().orc_secp_recover(msg, sig, out) else None


def secp_recover_batch(msgs: np.ndarray, sigs: np.ndarray, threads: int = 1):
    """[n,32] digests, [n,65] signatures -> ([n,64] public keys, [n] ok) on `threads` threads."""
    msgs = np.ascontiguousarray(msgs, dtype=np.uint8)
    sigs = np.ascontiguousarray(sigs, dtype=np.uint8)
    n = msgs.shape[0]
    pubs = np.zeros((n, 64), dtype=np.uint8)
    ok = np.zeros(n, dtype=np.uint8)
    L = lib()
    L.orc_secp_recover_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_int]
    L.orc_secp_recover_batch(msgs.ctypes.data, sigs.ctypes.data, n, pubs.ctypes.data, ok.ctypes.data, threads)
    return pubs, ok
