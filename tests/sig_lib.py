"""ctypes wrapper of tests/emu/libsig_host.so — TEST-ONLY host build of the exact secp256k1 source the
gfx950 kernels run (consensus-rs_amd/csrc/secp256k1.h), checked against oracle/secp256k1_ref.py."""
from __future__ import annotations

import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU_DIR = os.path.join(ROOT, "tests", "emu")
LIB = os.path.join(EMU_DIR, "libsig_host.so")
SRCS = [os.path.join(EMU_DIR, "sig_host.cpp")] + [
    os.path.join(ROOT, "consensus-rs_amd", "csrc", f) for f in ("secp256k1.h", "bft_common.h")]

OPS = {"fe_mul": 0, "fe_sqr": 1, "fe_add": 2, "fe_sub": 3, "fe_inv": 4, "fe_sqrt": 5, "sc_mul": 6, "sc_inv": 7,
       "sc_add": 8, "sc_neg": 9}
_lib = None


def build():
    if os.path.exists(LIB) and all(os.path.getmtime(LIB) >= os.path.getmtime(s) for s in SRCS):
        return
    tmp = f"{LIB}.{os.getpid()}.tmp"      # private name + rename: safe under concurrent test workers
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-Wno-unknown-pragmas", "-o", tmp, SRCS[0]])
    os.replace(tmp, LIB)


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(LIB)
    return _lib


def op(name: str, a: int, b: int = 0) -> int:
    out = (ctypes.c_uint8 * 32)()
    lib().sig_host_op(OPS[name], a.to_bytes(32, "big"), b.to_bytes(32, "big"), out)
    return int.from_bytes(bytes(out), "big")


def sha256(data: bytes) -> bytes:
    out = (ctypes.c_uint8 * 32)()
    lib().sig_host_sha256(data, len(data), out)
    return bytes(out)


def nonces(secret: bytes, msg: bytes, count: int) -> bytes:
    out = (ctypes.c_uint8 * (32 * count))()
    lib().sig_host_nonces(secret, msg, count, out)
    return bytes(out)


def pub(secret: bytes):
    p, a = (ctypes.c_uint8 * 64)(), (ctypes.c_uint8 * 20)()
    ok = lib().sig_host_pub(secret, p, a)
    return (bytes(p), bytes(a)) if ok else None


def mul_var(k: int, pub64: bytes):
    out = (ctypes.c_uint8 * 64)()
    ok = lib().sig_host_mul_var(k.to_bytes(32, "big"), pub64, out)
    return bytes(out) if ok else None


def sign(secret: bytes, msg: bytes):
    out = (ctypes.c_uint8 * 65)()
    return bytes(out) if lib().sig_host_sign(secret, msg, out) else None


def recover(msg: bytes, sig: bytes):
    p, a = (ctypes.c_uint8 * 64)(), (ctypes.c_uint8 * 20)()
    return (bytes(p), bytes(a)) if lib().sig_host_recover(msg, sig, p, a) else None


def counts():
    """(fe_mul, fe_sqr, sc_mul, sc_sqr) executed since the previous call."""
    out = (ctypes.c_uint64 * 4)()
    lib().sig_host_counts(out)
    return tuple(out)
