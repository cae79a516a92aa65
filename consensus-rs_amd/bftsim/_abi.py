"""ctypes mirror of include/bftsim.h (structs + prototypes)."""
from __future__ import annotations

import ctypes

import numpy as np

from .configs import BftConfig


class CConfig(ctypes.Structure):
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


class CResult(ctypes.Structure):
    _fields_ = [(k, ctypes.c_void_p) for k in (
        "committed_height", "flags", "ticks", "views", "round", "proposer", "variant",
        "time_tick", "block_hash")] + [("capacity", ctypes.c_uint64)]


class CStats(ctypes.Structure):
    _fields_ = [("instances", ctypes.c_uint64), ("committed_heights", ctypes.c_uint64),
                ("views", ctypes.c_uint64), ("ticks", ctypes.c_uint64),
                ("flagged", ctypes.c_uint64 * 7), ("round_hist", ctypes.c_uint64 * 65),
                ("latency_hist", ctypes.c_uint64 * 65)]


class CCryptoReport(ctypes.Structure):
    _fields_ = [(k, ctypes.c_uint64) for k in (
        "messages", "seals", "forged", "recovered_as_sender", "mismatches", "seal_errors", "signatures",
        "recoveries", "log_overflows")]


def to_cconfig(cfg: BftConfig):
    """Returns (struct, keepalive) — keep the second object alive while the struct is used."""
    c = CConfig()
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
        committed_height=np.zeros(n_inst, np.uint64), flags=np.zeros(n_inst, np.uint32),
        ticks=np.zeros(n_inst, np.uint32), views=np.zeros(n_inst, np.uint64),
        round=np.zeros(n_inst * heights, np.uint16), proposer=np.zeros(n_inst * heights, np.uint16),
        variant=np.zeros(n_inst * heights, np.uint8), time_tick=np.zeros(n_inst * heights, np.uint32),
        block_hash=np.zeros(n_inst * heights * 32, np.uint8))
    r = CResult()
    for k, a in arrs.items():
        setattr(r, k, a.ctypes.data)
    r.capacity = n_inst
    return r, arrs


def shape_result(arrs, n_inst: int, heights: int):
    for k in ("round", "proposer", "variant", "time_tick"):
        arrs[k] = arrs[k].reshape(n_inst, heights)
    arrs["block_hash"] = arrs["block_hash"].reshape(n_inst, heights, 32)
    return arrs
