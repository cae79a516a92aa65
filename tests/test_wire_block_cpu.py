"""Block-carrying frames of the wire codec (SPEC.md §9b) on the CPU: the host build of
consensus-rs_amd/csrc/bft_wire_block.h (what the GPU kernels run) against the msgpack oracle
(oracle/wire_ref.py) — Preprepare (PrePrepare{view, Block}), Block (Blocks) and Sync (Height) frames,
their sign digests, round trips, serde-default short arrays and malformed frames."""
import ctypes
import os
import random
import struct
import subprocess
import sys
import tempfile

import msgpack
import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "consensus-rs_amd"))
import wire_ref as R  # noqa: E402
import wire_lib as W  # noqa: E402
import oracle_lib as O  # noqa: E402
from bftsim import wire  # noqa: E402

EDGE = [0, 1, 127, 128, 255, 256, 65535, 65536, 2 ** 32 - 1, 2 ** 32, 2 ** 64 - 1]


def rand_block(rng, txs=None):
    u = lambda: rng.choice(EDGE) if rng.random() < 0.3 else rng.randrange(1 << rng.choice([8, 20, 40, 64]))  # noqa: E731
    rb = lambda n: bytes(rng.randrange(256) for _ in range(n))  # noqa: E731
    nt = rng.randrange(3) if txs is None else txs
    return dict(prev_hash=rb(32), proposer=rb(20), root=rb(32), tx_hash=rb(32), receipt_hash=rb(32), bloom=u(),
                difficulty=u(), height=u(), gas_limit=u(), gas_used=u(), time=u(),
                extra=rb(rng.randrange(33)) if rng.random() < 0.7 else None,
                votes=[rb(65) for _ in range(rng.randrange(17))] if rng.random() < 0.6 else None,
                txs=[dict(nonce=u(), price=u(), gas_limit=u(), amount=u(),
                          recipient=rb(20) if rng.random() < 0.8 else None, payload=rb(rng.randrange(65)),
                          sig=rb(65) if rng.random() < 0.7 else None) for _ in range(nt)])


def rand_pp(rng):
    return dict(round=rng.choice(EDGE[:6]), height=rng.choice(EDGE), create_time=rng.choice(EDGE),
                ttl=rng.choice([10, 0, 300]), raw_time=rng.randrange(1 << 41),
                signature=bytes(rng.randrange(256) for _ in range(65)) if rng.random() < 0.8 else None,
                block=rand_block(rng))


def host_pp_encode(m):
    L = W.lib()
    a = wire.preprepares_to_array([m])
    out = (ctypes.c_uint8 * 65536)()
    sd, mh = (ctypes.c_uint8 * 32)(), (ctypes.c_uint8 * 32)()
    L.wire_host_pp_encode.restype = ctypes.c_uint32
    n = L.wire_host_pp_encode(ctypes.c_void_p(a.ctypes.data), out, 65536, sd, mh)
    return bytes(out[:n]), bytes(sd), bytes(mh)


def host_pp_decode(f):
    a = np.zeros(1, wire.PP_DTYPE)
    ok = W.lib().wire_host_pp_decode(f, len(f), ctypes.c_void_p(a.ctypes.data))
    return wire.array_to_preprepares(a)[0] if ok else None


def host_blocks_encode(blocks, ttl=10, rt=0):
    a = wire.blocks_to_array(blocks) if blocks else np.zeros(1, wire.BLOCK_DTYPE)
    out = (ctypes.c_uint8 * 262144)()
    L = W.lib()
    L.wire_host_blocks_encode.restype = ctypes.c_uint32
    n = L.wire_host_blocks_encode(ctypes.c_void_p(a.ctypes.data), len(blocks), ctypes.c_uint64(ttl),
                                  ctypes.c_uint64(rt), out, 262144)
    return bytes(out[:n])


def host_blocks_decode(f, mx=8):
    a = np.zeros(mx, wire.BLOCK_DTYPE)
    cnt = ctypes.c_uint32()
    ok = W.lib().wire_host_blocks_decode(f, len(f), ctypes.c_void_p(a.ctypes.data), mx, ctypes.byref(cnt))
    return [wire.rec_to_block(a[j]) for j in range(cnt.value)] if ok else None


def test_struct_layouts_match_header():
    L = W.lib()
    assert [L.wire_host_struct_size(k) for k in range(3)] == [wire.TX_DTYPE.itemsize, wire.BLOCK_DTYPE.itemsize,
                                                              wire.PP_DTYPE.itemsize]
    fields = {"bftwire_tx": wire.TX_DTYPE, "bftwire_block": wire.BLOCK_DTYPE, "bftwire_preprepare": wire.PP_DTYPE}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "bftwire.h"', "int main(void) {"]
    for st, dt in fields.items():
        for f in dt.names:
            lines.append(f'printf("{st} {f} %zu\\n", offsetof({st}, {f}));')
    lines.append("return 0; }")
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "l.c"), os.path.join(d, "l")
        open(src, "w").write("\n".join(lines))
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), "-o", exe, src])
        out = subprocess.check_output([exe]).decode().split("\n")
    got = {tuple(l.split()[:2]): int(l.split()[2]) for l in out if l}
    for st, dt in fields.items():
        for f in dt.names:
            assert got[(st, f)] == dt.fields[f][1], (st, f)


def test_preprepare_frames_match_oracle():
    rng = random.Random(3)
    for _ in range(60):
        m = rand_pp(rng)
        f, sd, mh = host_pp_encode(m)
        rf, sp, g = R.preprepare_frame(m)
        assert f == rf
        assert sd == O.keccak256(sp) and mh == O.keccak256(g)
        back = host_pp_decode(f)
        assert back == R.decode_preprepare(f) == m


def test_block_and_sync_frames_match_oracle():
    rng = random.Random(4)
    for k in range(30):
        blocks = [rand_block(rng) for _ in range(rng.randrange(4))]
        f = host_blocks_encode(blocks, 10, 1000 + k)
        assert f == R.blocks_frame(blocks, 10, 1000 + k)
        assert host_blocks_decode(f) == R.decode_blocks(f) == blocks
    L = W.lib()
    L.wire_host_sync_encode.restype = ctypes.c_uint32
    for h in EDGE:
        out = (ctypes.c_uint8 * 64)()
        n = L.wire_host_sync_encode(ctypes.c_uint64(h), ctypes.c_uint64(10), ctypes.c_uint64(7), out, 64)
        f = bytes(out[:n])
        assert f == R.sync_frame(h, 10, 7)
        v = ctypes.c_uint64()
        assert L.wire_host_sync_decode(f, len(f), ctypes.byref(v)) == 1 and v.value == h == R.decode_sync(f)


def test_serde_default_and_malformed():
    rng = random.Random(5)
    m = rand_pp(rng)
    m["block"]["extra"], m["block"]["votes"] = b"abc", None
    f, _, g = R.preprepare_frame(m)
    # header without votes (12 fields) and without extra + votes (11): #[serde(default)] -> None
    for k in (12, 11):
        msg = msgpack.packb([[m["round"], m["height"]], [R.header_obj(m["block"])[:k],
                                                           [R.tx_obj(t) for t in m["block"]["txs"]]]])
        gg = msgpack.packb([[0, []], m["create_time"], list(msg), None, None])
        ff = R.frame(gg, m["ttl"], m["raw_time"])
        want, got = R.decode_preprepare(ff), host_pp_decode(ff)
        assert want is not None and got == want and got["block"]["votes"] is None
        assert (got["block"]["extra"] is None) == (k == 11)
    # GossipMessage without signature / commit_seal (3 elements)
    gl = msgpack.unpackb(g)[:3]
    ff = R.frame(msgpack.packb(gl), m["ttl"], m["raw_time"])
    assert host_pp_decode(ff) == R.decode_preprepare(ff) is not None
    # truncations, a Subject message's code, a transaction with 6 fields: rejected by both
    for cut in range(5, len(f), max(1, len(f) // 23)):
        t = struct.pack(">I", cut - 4) + f[4:cut]
        assert host_pp_decode(t) is None and R.decode_preprepare(t) is None
    bad = R.frame(R.gossip(2, 0, R.subject(0, 1, bytes(32)), None, None))
    assert host_pp_decode(bad) is None and R.decode_preprepare(bad) is None
    b = rand_block(rng, txs=1)
    blk = R.block_obj(b)
    blk[1][0] = blk[1][0][:6]
    ff = R.frame(msgpack.packb([blk]), code=R.P2P_BLOCK)
    assert host_blocks_decode(ff) is None and R.decode_blocks(ff) is None
    assert host_blocks_decode(R.sync_frame(5)) is None and R.decode_blocks(R.sync_frame(5)) is None
