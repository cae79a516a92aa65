"""ctypes wrapper of tests/emu/libwire_host.so — TEST-ONLY host build of consensus-rs_amd/csrc/bft_wire.h
(the serial encoder / streaming decoder the GPU codec shares), checked against oracle/wire_ref.py."""
from __future__ import annotations

import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU_DIR = os.path.join(ROOT, "tests", "emu")
LIB = os.path.join(EMU_DIR, "libwire_host.so")
SRCS = [os.path.join(EMU_DIR, "wire_host.cpp")] + [
    os.path.join(ROOT, "consensus-rs_amd", "csrc", f) for f in ("bft_wire.h", "bft_common.h", "bft_wire_block.h",
                                                               "bft_crypto.h")] + [
    os.path.join(ROOT, "include", "bftwire.h")]
_lib = None


class Decoded(ctypes.Structure):
    _fields_ = [("code", ctypes.c_uint32), ("create_time", ctypes.c_uint64), ("height", ctypes.c_uint64),
                ("round", ctypes.c_uint64), ("digest", ctypes.c_uint8 * 32), ("has_sig", ctypes.c_uint32),
                ("has_seal", ctypes.c_uint32), ("sig", ctypes.c_uint8 * 65), ("seal", ctypes.c_uint8 * 65),
                ("ttl", ctypes.c_uint64), ("raw_time", ctypes.c_uint64), ("peer_len", ctypes.c_uint32),
                ("peer", ctypes.c_uint8 * 64)]


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
        _lib.wire_host_encode.restype = ctypes.c_uint32
        _lib.wire_host_encode.argtypes = [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_char_p,
                                          ctypes.c_uint64, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint64,
                                          ctypes.c_uint64, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        _lib.wire_host_decode.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.POINTER(Decoded)]
        assert _lib.wire_host_decoded_size() == ctypes.sizeof(Decoded)
    return _lib


def encode(m: dict):
    """-> (frame, GossipMessage bytes, sign-payload bytes) of one message dict (oracle/wire_ref.py keys)."""
    f, g, sp = (ctypes.c_uint8 * 1028)(), (ctypes.c_uint8 * 512)(), (ctypes.c_uint8 * 512)()
    gl, spl = ctypes.c_uint32(), ctypes.c_uint32()
    peer = m.get("peer_id")
    n = lib().wire_host_encode(m["code"], m["round"], m["height"], m["digest"], m["create_time"], m.get("signature"),
                               m.get("commit_seal"), m.get("ttl", 10), m.get("raw_time", 0), peer,
                               len(peer) if peer else 0, f, g, ctypes.byref(gl), sp, ctypes.byref(spl))
    return bytes(f[:n]), bytes(g[:gl.value]), bytes(sp[:spl.value])


def decode(fr: bytes):
    d = Decoded()
    if not lib().wire_host_decode(fr, len(fr), ctypes.byref(d)):
        return None
    return dict(code=d.code, create_time=d.create_time, round=d.round, height=d.height, digest=bytes(d.digest),
                signature=bytes(d.sig) if d.has_sig else None, commit_seal=bytes(d.seal) if d.has_seal else None,
                ttl=d.ttl, raw_time=d.raw_time,
                peer_id=None if d.peer_len == 0xffffffff else bytes(d.peer[:d.peer_len]))
