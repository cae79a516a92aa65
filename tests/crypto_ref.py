"""CPU reference of real-crypto mode's sign pass (SPEC.md §11), test infrastructure only: from the
oracle's broadcast log (oracle_lib.run_crypto) and its run outputs, the bytes every message is signed
over (msgpack oracle of SPEC.md §9, oracle/wire_ref.py), the signatures (RFC 6979, the Python
secp256k1 oracle) and the per-instance checksum libbftsim's bftsim_crypto_verify reports."""
from __future__ import annotations

import ctypes
import os
import sys

import msgpack
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import secp256k1_ref as S  # noqa: E402
import wire_ref as R  # noqa: E402
import oracle_lib as O  # noqa: E402

EXTRA = b"Coinse base"


def _unpack(b):
    return dict(h=b & 0xffffff, prop=(b >> 24) & 0x1ff, var=(b >> 33) & 1, valid=(b >> 34) & 1, T=b >> 35)


def _header(cfg, inst, x, prop, var, T, prev):
    L = O.lib()
    tx = (ctypes.c_uint8 * 32)()
    L.orc_tx_hash(ctypes.c_uint64(cfg.seed), inst, x, prop, var, tx)
    buf = (ctypes.c_uint8 * 512)()
    time = cfg.genesis_time + cfg.block_period * (T + 1)
    L.orc_encode_header.restype = ctypes.c_size_t
    n = L.orc_encode_header(buf, bytes(prev), cfg.addresses[prop], bytes(tx), ctypes.c_uint64(x), ctypes.c_uint64(0),
                            ctypes.c_uint64(0), ctypes.c_uint64(time), EXTRA, len(EXTRA))
    return bytes(buf[:n])


def _parent(cfg, res, i, x, genesis):
    ch = int(res["committed_height"][i])
    if x <= 1:
        return genesis
    if x - 1 <= ch:
        return bytes(res["block_hash"][i, x - 2])
    return bytes(32)


def _digest(cfg, res, i, inst, b, genesis):
    u = _unpack(b)
    x = u["h"]
    if not u["valid"] or x == 0:
        return bytes(32)
    if x <= int(res["committed_height"][i]) and int(res["proposer"][i, x - 1]) == u["prop"] and \
            int(res["variant"][i, x - 1]) == u["var"]:
        return bytes(res["block_hash"][i, x - 1])
    return O.keccak256(_header(cfg, inst, x, u["prop"], u["var"], u["T"], _parent(cfg, res, i, x, genesis)))


def instance_checksums(cfg, first, res, secrets, forged=(), sigs_out=None):
    """[n, 32] XOR over each instance's logged messages of keccak(signature || seal or 0^65);
    sigs_out (a dict) receives {(instance, sender, code, height, round, old): signature}"""
    n = len(res["committed_height"])
    L = O.lib()
    c, keep = O.to_orc(cfg)
    g = (ctypes.c_uint8 * 32)()
    L.orc_genesis_hash(ctypes.byref(c), g)
    genesis = bytes(g)
    keys = list(secrets) + [O.keccak256(k) for k in secrets]
    fs = set(forged)
    out = np.zeros((n, 32), np.uint8)
    for i in range(n):
        inst = first + i
        acc = bytearray(32)
        for e in res["mlog"][i, : int(res["mlog_n"][i])]:
            tick, w1, h, r = int(e[0]), int(e[1]), int(e[2]), int(e[3])
            code, sender = (w1 >> 8) & 0xff, w1 >> 16
            b = int(e[4]) | (int(e[5]) << 32)
            key = keys[sender + (cfg.n if sender in fs else 0)]
            ctime = 1000 * (cfg.genesis_time + cfg.block_period * tick) if code == 4 else 0
            d = bytes(32) if code == 4 else _digest(cfg, res, i, inst, b, genesis)
            seal = S.sign(key, O.keccak256(bytes([3]) + d)) if code == 3 else None
            if code == 1:
                u = _unpack(b)
                hdr = _header(cfg, inst, u["h"], u["prop"], u["var"], u["T"], _parent(cfg, res, i, u["h"], genesis))
                msg = b"\x92" + msgpack.packb([r, h]) + b"\x92" + hdr + b"\x90"
            else:
                msg = R.subject(r, h, d)
            sig = S.sign(key, O.keccak256(R.gossip(code, ctime, msg, None, seal)))
            if sigs_out is not None:
                sigs_out[(i, sender, code, h, r, bool(int(e[6]) & 8))] = sig
            t = O.keccak256(sig + (seal if seal is not None else bytes(65)))
            acc = bytearray(a ^ b_ for a, b_ in zip(acc, t))
        out[i] = np.frombuffer(bytes(acc), np.uint8)
    del keep
    return out
