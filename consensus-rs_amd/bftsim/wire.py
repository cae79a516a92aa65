"""Host binding of libbftwire (include/bftwire.h): the consensus wire codec on the GPU, batched.

Mirrors the reference's codec surface for Subject-carrying consensus messages:
  * `encode(batch)`       Subject::into_bytes -> GossipMessage::into_payload -> RawMessage ->
                          MsgPacketCodec::encode (src/consensus/types.rs:101-104, src/protocol/mod.rs:44-53,
                          src/p2p/protocol.rs:30-70, src/p2p/codec.rs:43-53), plus sign_digest (mod.rs:128-137)
                          and the message hash of the outbound cache (backend.rs:141-148);
  * `split_frames(bytes)` MsgPacketCodec::decode's frame loop (codec.rs:18-40), on the host;
  * `decode(stream, offs)` RawMessage / GossipMessage / Subject from_bytes (core.rs:50-60).
A batch is a dict of torch tensors on the GPU (or numpy arrays): code [n] u8, round / height /
create_time [n] u64 (int64 tensors), digest [n,32] u8, and optional signature / commit_seal [n,65] u8,
ttl / raw_time [n]. No CPU fallback: a missing libbftwire.so raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("BFTWIRE_LIB") or os.path.join(PKG_DIR, "build", "libbftwire.so")
_lib = None


class BftwireError(RuntimeError):
    pass


class CBatch(ctypes.Structure):
    _fields_ = [("code", ctypes.c_void_p), ("round", ctypes.c_void_p), ("height", ctypes.c_void_p),
                ("digest", ctypes.c_void_p), ("create_time", ctypes.c_void_p), ("signature", ctypes.c_void_p),
                ("commit_seal", ctypes.c_void_p), ("ttl", ctypes.c_void_p), ("raw_time", ctypes.c_void_p)]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise BftwireError(f"libbftwire.so not built ({LIB_PATH}); run __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        vp, u64 = ctypes.c_void_p, ctypes.c_uint64
        L.bftwire_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
        L.bftwire_destroy.argtypes = [vp]
        L.bftwire_last_error.argtypes = [vp]
        L.bftwire_last_error.restype = ctypes.c_char_p
        L.bftwire_encode.argtypes = [vp, ctypes.POINTER(CBatch), u64, vp, u64, vp, vp, vp, vp, vp]
        L.bftwire_decode.argtypes = [vp, vp, vp, u64, ctypes.POINTER(CBatch), vp, vp, vp, vp]
        L.bftwire_split_frames.argtypes = [vp, u64, vp, u64]
        L.bftwire_split_frames.restype = u64
        _lib = L
    return _lib


def split_frames(stream, max_frames: int | None = None) -> np.ndarray:
    """Frame offsets [k+1] of the complete frames at the start of a received byte stream."""
    b = np.frombuffer(bytes(stream), dtype=np.uint8) if not isinstance(stream, np.ndarray) else stream
    b = np.ascontiguousarray(b, dtype=np.uint8)
    mx = max_frames if max_frames is not None else max(1, len(b) // 4)
    offs = np.zeros(mx + 1, dtype=np.uint64)
    k = lib().bftwire_split_frames(b.ctypes.data, len(b), offs.ctypes.data, mx)
    return offs[:k + 1]


class Codec:
    def __init__(self, device: int = 0):
        import torch
        self.torch = torch
        self.device = torch.device("cuda", device)
        h = ctypes.c_void_p()
        rc = lib().bftwire_create(device, ctypes.byref(h))
        self.h = h.value
        self._check(rc, "bftwire_create")

    def close(self):
        if self.h:
            lib().bftwire_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            raise BftwireError(f"{what} failed ({rc}): {lib().bftwire_last_error(self.h).decode() if self.h else ''}")

    def _t(self, a, dtype):
        t = self.torch
        if a is None:
            return None
        if isinstance(a, np.ndarray):
            a = np.ascontiguousarray(a)
            a = t.from_numpy(a if a.flags.writeable else a.copy())
        return a.to(self.device).to(dtype).contiguous()

    def _cbatch(self, d, keep):
        t = self.torch
        fields = {"code": t.uint8, "round": t.int64, "height": t.int64, "digest": t.uint8, "create_time": t.int64,
                  "signature": t.uint8, "commit_seal": t.uint8, "ttl": t.int64, "raw_time": t.int64}
        c = CBatch()
        for k, dt in fields.items():
            v = self._t(d.get(k), dt)
            keep.append(v)
            setattr(c, k, v.data_ptr() if v is not None else None)
        return c

    def encode(self, batch: dict, cap: int | None = None, hashes: bool = True, stream=None):
        """-> (stream bytes [cap] u8, frame_off [n+1] int64, sign_digest [n,32], msg_hash [n,32], ok [n])"""
        t = self.torch
        n = int(batch["code"].shape[0])
        cap = cap if cap is not None else max(1, n) * 1028
        keep = []
        c = self._cbatch(batch, keep)
        out = t.empty(cap, dtype=t.uint8, device=self.device)
        offs = t.empty(n + 1, dtype=t.int64, device=self.device)
        ok = t.empty(max(n, 1), dtype=t.uint8, device=self.device)
        sd = t.empty((n, 32), dtype=t.uint8, device=self.device) if hashes else None
        mh = t.empty((n, 32), dtype=t.uint8, device=self.device) if hashes else None
        s = stream if stream is not None else t.cuda.current_stream(self.device).cuda_stream
        self._check(lib().bftwire_encode(self.h, ctypes.byref(c), n, out.data_ptr(), cap, offs.data_ptr(),
                                         sd.data_ptr() if hashes else None, mh.data_ptr() if hashes else None,
                                         ok.data_ptr(), s), "bftwire_encode")
        return out, offs, sd, mh, ok[:n]

    def decode(self, stream_bytes, frame_off, stream=None):
        """-> (dict of field tensors incl. has_sig / has_seal, ok [n])"""
        t = self.torch
        sb = self._t(stream_bytes, t.uint8)
        offs = self._t(frame_off, t.int64)
        n = int(offs.shape[0]) - 1
        shapes = {"code": ((n,), t.uint8), "round": ((n,), t.int64), "height": ((n,), t.int64),
                  "digest": ((n, 32), t.uint8), "create_time": ((n,), t.int64), "signature": ((n, 65), t.uint8),
                  "commit_seal": ((n, 65), t.uint8), "ttl": ((n,), t.int64), "raw_time": ((n,), t.int64)}
        out = {k: t.empty(sh, dtype=dt, device=self.device) for k, (sh, dt) in shapes.items()}
        keep = []
        c = self._cbatch(out, keep)
        hs = t.empty(max(n, 1), dtype=t.uint8, device=self.device)
        hl = t.empty(max(n, 1), dtype=t.uint8, device=self.device)
        ok = t.empty(max(n, 1), dtype=t.uint8, device=self.device)
        s = stream if stream is not None else t.cuda.current_stream(self.device).cuda_stream
        self._check(lib().bftwire_decode(self.h, sb.data_ptr(), offs.data_ptr(), n, ctypes.byref(c), hs.data_ptr(),
                                         hl.data_ptr(), ok.data_ptr(), s), "bftwire_decode")
        out["has_sig"], out["has_seal"] = hs[:n], hl[:n]
        return out, ok[:n]
