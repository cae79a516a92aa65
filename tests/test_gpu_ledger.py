"""Ledger export (core/ledger.rs:193-245 add_block -> the `headers` map of
store/schema.rs:66-68): the Header bytes the GPU exports for every committed height equal the oracle's
header encoder (oracle/bft_oracle.c orc_encode_header, itself pinned to the msgpack package by
tests/test_oracle_kat.py) and hash to the block hashes of the run — for a power-of-two N (hash pass: cfg3, cfg1-n4) and
for N = 5 / 7 and little-endian seeds (hashes computed inside the consensus kernel)."""
import ctypes

import numpy as np
import pytest

from bftsim.configs import BftConfig, cfg1, cfg3, cfg4
from bftsim.runtime import Simulator
import oracle_lib as O

pytestmark = pytest.mark.gpu


def _le(cfg):
    import dataclasses
    return dataclasses.replace(cfg, seed_byte_order=1, name=cfg.name + "-le")


def expected_header(cfg, inst, x, prop, var, tick, prev):
    L = O.lib()
    u32, u64, cp = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_char_p
    L.orc_tx_hash.argtypes = [u64, u32, u32, u32, u32, ctypes.c_void_p]
    L.orc_encode_header.argtypes = [ctypes.c_void_p, cp, cp, cp, u64, u64, u64, u64, cp, ctypes.c_size_t]
    L.orc_encode_header.restype = ctypes.c_size_t
    tx = (ctypes.c_uint8 * 32)()
    L.orc_tx_hash(cfg.seed, inst, x, prop, var, tx)
    extra = b"Coinse base"                       # minner/mod.rs:113; gas_limit = gas_used = 0
    buf = (ctypes.c_uint8 * 512)()
    time = cfg.genesis_time + cfg.block_period * (tick + 1)
    n = L.orc_encode_header(buf, prev, bytes(cfg.addresses[prop]), bytes(tx), x, 0, 0, time, extra, len(extra))
    return bytes(buf[:n])


@pytest.mark.parametrize("name,mk,first,n", [("cfg3", lambda: cfg3(heights=12), 0, 6),
                                             ("cfg1-n4", lambda: cfg1(False, heights=15), 0, 1),
                                             ("cfg1-n5", lambda: cfg1(True, heights=15), 0, 1),
                                             ("cfg3-le", lambda: _le(cfg3(heights=8)), 0, 4),
                                             ("cfg4-n7-crash", lambda: cfg4(7, heights=10), 3, 8)])
def test_exported_headers(name, mk, first, n):
    cfg = mk()
    sim = Simulator(cfg, device=0)
    res = sim.run(first, n)
    hdrs = sim.export_headers(n)
    sim.close()
    g = (ctypes.c_uint8 * 32)()
    c_, keep = O.to_orc(cfg)
    O.lib().orc_genesis_hash(ctypes.byref(c_), g)
    checked = 0
    for i in range(n):
        ch = int(res["committed_height"][i])
        prev = bytes(g)
        for x in range(1, cfg.heights + 1):
            h = hdrs[i][x - 1]
            if x > ch:
                assert h == b""
                continue
            bh = bytes(res["block_hash"][i, x - 1])
            assert O.keccak256(h) == bh, (name, i, x)
            want = expected_header(cfg, first + i, x, int(res["proposer"][i, x - 1]), int(res["variant"][i, x - 1]),
                                   int(res["time_tick"][i, x - 1]), prev)
            assert h == want, (name, i, x)
            prev = bh
            checked += 1
    assert checked > 0
