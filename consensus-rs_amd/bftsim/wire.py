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

from .runtime import lib_override

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = lib_override("BFTWIRE_LIB") or os.path.join(PKG_DIR, "build", "libbftwire.so")
_lib = None


class BftwireError(RuntimeError):
    pass


class CBatch(ctypes.Structure):
    _fields_ = [("code", ctypes.c_void_p), ("round", ctypes.c_void_p), ("height", ctypes.c_void_p),
                ("digest", ctypes.c_void_p), ("create_time", ctypes.c_void_p), ("signature", ctypes.c_void_p),
                ("commit_seal", ctypes.c_void_p), ("ttl", ctypes.c_void_p), ("raw_time", ctypes.c_void_p)]


# array-of-structures mirrors of include/bftwire.h (bftwire_tx / _block / _preprepare), C layout
NONE = 0xFFFFFFFF
MAX_EXTRA, MAX_VOTES, MAX_TX, MAX_PAYLOAD = 32, 16, 2, 64
TX_DTYPE = np.dtype({"names": ["nonce", "price", "gas_limit", "amount", "payload_len", "has_recipient", "has_sig",
                               "recipient", "payload", "sig"],
                     "formats": ["<u8", "<u8", "<u8", "<u8", "<u4", "u1", "u1", ("u1", 20), ("u1", MAX_PAYLOAD),
                                 ("u1", 65)],
                     "offsets": [0, 8, 16, 24, 32, 36, 37, 40, 60, 124], "itemsize": 200})
BLOCK_DTYPE = np.dtype({"names": ["bloom", "difficulty", "height", "gas_limit", "gas_used", "time", "extra_len",
                                  "n_votes", "n_tx", "prev_hash", "root", "tx_hash", "receipt_hash", "proposer",
                                  "extra", "votes", "tx"],
                        "formats": ["<u8"] * 6 + ["<u4"] * 3 + [("u1", 32)] * 4 + [("u1", 20), ("u1", MAX_EXTRA),
                                                                                 ("u1", (MAX_VOTES, 65)),
                                                                                 (TX_DTYPE, MAX_TX)],
                        "offsets": [0, 8, 16, 24, 32, 40, 48, 52, 56, 64, 96, 128, 160, 192, 212, 244, 1288],
                        "itemsize": 1688})
PP_DTYPE = np.dtype({"names": ["round", "height", "create_time", "ttl", "raw_time", "has_sig", "signature", "block"],
                     "formats": ["<u8"] * 5 + ["u1", ("u1", 65), BLOCK_DTYPE],
                     "offsets": [0, 8, 16, 24, 32, 40, 48, 120], "itemsize": 1808})


def block_to_rec(b: dict, rec):
    """a block dict (oracle/wire_ref.py keys) into one BLOCK_DTYPE record"""
    for k in ("bloom", "difficulty", "height", "gas_limit", "gas_used", "time"):
        rec[k] = b[k]
    for k in ("prev_hash", "root", "tx_hash", "receipt_hash", "proposer"):
        rec[k] = np.frombuffer(bytes(b[k]), np.uint8)
    ex = b.get("extra")
    rec["extra_len"] = NONE if ex is None else len(ex)
    if ex is not None:
        rec["extra"][: len(ex)] = np.frombuffer(bytes(ex), np.uint8)
    vs = b.get("votes")
    rec["n_votes"] = NONE if vs is None else len(vs)
    for j, v in enumerate(vs or []):
        rec["votes"][j] = np.frombuffer(bytes(v), np.uint8)
    rec["n_tx"] = len(b["txs"])
    for j, t in enumerate(b["txs"]):
        r = rec["tx"][j]
        for k in ("nonce", "price", "gas_limit", "amount"):
            r[k] = t[k]
        r["has_recipient"] = t.get("recipient") is not None
        if t.get("recipient") is not None:
            r["recipient"] = np.frombuffer(bytes(t["recipient"]), np.uint8)
        r["payload_len"] = len(t["payload"])
        r["payload"][: len(t["payload"])] = np.frombuffer(bytes(t["payload"]), np.uint8)
        r["has_sig"] = t.get("sig") is not None
        if t.get("sig") is not None:
            r["sig"] = np.frombuffer(bytes(t["sig"]), np.uint8)
        rec["tx"][j] = r


def rec_to_block(rec) -> dict:
    b = {k: int(rec[k]) for k in ("bloom", "difficulty", "height", "gas_limit", "gas_used", "time")}
    for k in ("prev_hash", "root", "tx_hash", "receipt_hash", "proposer"):
        b[k] = bytes(rec[k])
    el, nv = int(rec["extra_len"]), int(rec["n_votes"])
    b["extra"] = None if el == NONE else bytes(rec["extra"][:el])
    b["votes"] = None if nv == NONE else [bytes(rec["votes"][j]) for j in range(nv)]
    b["txs"] = []
    for j in range(int(rec["n_tx"])):
        r = rec["tx"][j]
        b["txs"].append(dict(nonce=int(r["nonce"]), price=int(r["price"]), gas_limit=int(r["gas_limit"]),
                             amount=int(r["amount"]), recipient=bytes(r["recipient"]) if r["has_recipient"] else None,
                             payload=bytes(r["payload"][: int(r["payload_len"])]),
                             sig=bytes(r["sig"]) if r["has_sig"] else None))
    return b


def preprepares_to_array(ms) -> np.ndarray:
    a = np.zeros(len(ms), PP_DTYPE)
    for i, m in enumerate(ms):
        for k in ("round", "height", "create_time"):
            a[i][k] = m[k]
        a[i]["ttl"], a[i]["raw_time"] = m.get("ttl", 10), m.get("raw_time", 0)
        a[i]["has_sig"] = m.get("signature") is not None
        if m.get("signature") is not None:
            a[i]["signature"] = np.frombuffer(bytes(m["signature"]), np.uint8)
        blk = a[i]["block"]
        block_to_rec(m["block"], blk)
        a[i]["block"] = blk
    return a


def array_to_preprepares(a) -> list:
    out = []
    for r in a:
        out.append(dict(round=int(r["round"]), height=int(r["height"]), create_time=int(r["create_time"]),
                        ttl=int(r["ttl"]), raw_time=int(r["raw_time"]),
                        signature=bytes(r["signature"]) if r["has_sig"] else None, block=rec_to_block(r["block"])))
    return out


def blocks_to_array(blocks) -> np.ndarray:
    a = np.zeros(len(blocks), BLOCK_DTYPE)
    for i, b in enumerate(blocks):
        rec = a[i]
        block_to_rec(b, rec)
        a[i] = rec
    return a


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
        L.bftwire_encode_preprepare.argtypes = [vp, vp, u64, vp, u64, vp, vp, vp, vp, vp]
        L.bftwire_decode_preprepare.argtypes = [vp, vp, vp, u64, vp, vp, vp]
        L.bftwire_encode_blocks.argtypes = [vp, vp, vp, u64, vp, vp, vp, u64, vp, vp, vp]
        L.bftwire_decode_blocks.argtypes = [vp, vp, vp, u64, ctypes.c_uint32, vp, vp, vp, vp]
        L.bftwire_encode_sync.argtypes = [vp, vp, u64, vp, vp, vp, u64, vp, vp, vp]
        L.bftwire_decode_sync.argtypes = [vp, vp, vp, u64, vp, vp, vp]
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



    def encode_preprepare(self, ms, cap: int | None = None, hashes: bool = True):
        """Preprepare frames of a list of dicts (oracle/wire_ref.py keys) -> (stream, offsets, sign_digest,
        msg_hash, ok) tensors (bftwire_encode_preprepare)"""
        t = self.torch
        a = preprepares_to_array(ms)
        n = len(a)
        d_in = _dev_bytes(self, a)
        cap = cap or n * 16384
        sd = t.zeros((max(n, 1), 32), dtype=t.uint8, device=self.device) if hashes else None
        mh = t.zeros((max(n, 1), 32), dtype=t.uint8, device=self.device) if hashes else None
        def go(stream, off, ok):
            self._check(lib().bftwire_encode_preprepare(self.h, d_in.data_ptr(), n, stream.data_ptr(), cap, off.data_ptr(),
                                                        sd.data_ptr() if hashes else None,
                                                        mh.data_ptr() if hashes else None, ok.data_ptr(), None),
                        "bftwire_encode_preprepare")
        stream, off, ok = _encode_frames(self, n, go, cap)
        return stream, off, (sd[:n] if hashes else None), (mh[:n] if hashes else None), ok


    def decode_preprepare(self, stream_bytes, frame_off):
        t = self.torch
        s = t.as_tensor(np.frombuffer(bytes(stream_bytes), np.uint8) if not t.is_tensor(stream_bytes) else stream_bytes)
        s = s.to(self.device) if s.numel() else t.zeros(1, dtype=t.uint8, device=self.device)
        offs = t.as_tensor(np.asarray(frame_off, dtype=np.int64)).to(self.device)
        n = offs.numel() - 1
        out = t.zeros(max(n, 1) * PP_DTYPE.itemsize, dtype=t.uint8, device=self.device)
        ok = t.zeros(max(n, 1), dtype=t.uint8, device=self.device)
        self._check(lib().bftwire_decode_preprepare(self.h, s.data_ptr(), offs.data_ptr(), n, out.data_ptr(), ok.data_ptr(),
                                                    None), "bftwire_decode_preprepare")
        t.cuda.synchronize(self.device)
        arr = out.cpu().numpy().view(PP_DTYPE)[:n]
        return arr, ok.cpu().numpy()[:n]


    def encode_blocks(self, frames, ttl=None, raw_time=None, cap: int | None = None):
        """Block frames: `frames` = list of block-dict lists (one RawMessage{Block, Blocks} each)"""
        t = self.torch
        blocks = [b for f in frames for b in f]
        boff = np.cumsum([0] + [len(f) for f in frames]).astype(np.uint64)
        n = len(frames)
        d_b = _dev_bytes(self, blocks_to_array(blocks)) if blocks else t.zeros(8, dtype=t.uint8, device=self.device)
        d_off = t.as_tensor(boff.view(np.int64)).to(self.device)
        d_ttl = t.as_tensor(np.asarray(ttl, np.int64)).to(self.device) if ttl is not None else None
        d_rt = t.as_tensor(np.asarray(raw_time, np.int64)).to(self.device) if raw_time is not None else None
        cap = cap or max(1, len(blocks)) * 16384 + n * 64
        def go(stream, off, ok):
            self._check(lib().bftwire_encode_blocks(self.h, d_b.data_ptr(), d_off.data_ptr(), n,
                                                    d_ttl.data_ptr() if d_ttl is not None else None,
                                                    d_rt.data_ptr() if d_rt is not None else None, stream.data_ptr(), cap,
                                                    off.data_ptr(), ok.data_ptr(), None), "bftwire_encode_blocks")
        return _encode_frames(self, n, go, cap)


    def decode_blocks(self, stream_bytes, frame_off, max_per_frame: int = 4):
        t = self.torch
        s = t.as_tensor(np.frombuffer(bytes(stream_bytes), np.uint8) if not t.is_tensor(stream_bytes) else stream_bytes)
        s = s.to(self.device) if s.numel() else t.zeros(1, dtype=t.uint8, device=self.device)
        offs = t.as_tensor(np.asarray(frame_off, dtype=np.int64)).to(self.device)
        n = offs.numel() - 1
        out = t.zeros(max(n, 1) * max_per_frame * BLOCK_DTYPE.itemsize, dtype=t.uint8, device=self.device)
        cnt = t.zeros(max(n, 1), dtype=t.int32, device=self.device)
        ok = t.zeros(max(n, 1), dtype=t.uint8, device=self.device)
        self._check(lib().bftwire_decode_blocks(self.h, s.data_ptr(), offs.data_ptr(), n, max_per_frame, out.data_ptr(),
                                                cnt.data_ptr(), ok.data_ptr(), None), "bftwire_decode_blocks")
        t.cuda.synchronize(self.device)
        arr = out.cpu().numpy().view(BLOCK_DTYPE)[: n * max_per_frame].reshape(n, max_per_frame)
        return arr, cnt.cpu().numpy()[:n], ok.cpu().numpy()[:n]


    def encode_sync(self, heights, ttl=None, raw_time=None, cap: int | None = None):
        t = self.torch
        h = t.as_tensor(np.asarray(heights, np.uint64).view(np.int64)).to(self.device)
        n = h.numel()
        cap = cap or n * 64
        def go(stream, off, ok):
            self._check(lib().bftwire_encode_sync(self.h, h.data_ptr(), n, None, None, stream.data_ptr(), cap,
                                                  off.data_ptr(), ok.data_ptr(), None), "bftwire_encode_sync")
        return _encode_frames(self, n, go, cap)


    def decode_sync(self, stream_bytes, frame_off):
        t = self.torch
        s = t.as_tensor(np.frombuffer(bytes(stream_bytes), np.uint8) if not t.is_tensor(stream_bytes) else stream_bytes)
        s = s.to(self.device) if s.numel() else t.zeros(1, dtype=t.uint8, device=self.device)
        offs = t.as_tensor(np.asarray(frame_off, dtype=np.int64)).to(self.device)
        n = offs.numel() - 1
        h = t.zeros(max(n, 1), dtype=t.int64, device=self.device)
        ok = t.zeros(max(n, 1), dtype=t.uint8, device=self.device)
        self._check(lib().bftwire_decode_sync(self.h, s.data_ptr(), offs.data_ptr(), n, h.data_ptr(), ok.data_ptr(), None),
                    "bftwire_decode_sync")
        t.cuda.synchronize(self.device)
        return h.cpu().numpy()[:n].view(np.uint64), ok.cpu().numpy()[:n]


def _dev_bytes(codec, arr: np.ndarray):
    t = codec.torch
    return t.from_numpy(np.ascontiguousarray(arr).view(np.uint8).reshape(-1).copy()).to(codec.device)


def _encode_frames(codec, n, launch, cap):
    """shared tail of the block-frame encoders: device offsets / ok, stream of `cap` bytes"""
    t = codec.torch
    stream = t.zeros(max(cap, 1), dtype=t.uint8, device=codec.device)
    off = t.zeros(n + 1, dtype=t.int64, device=codec.device)
    ok = t.zeros(max(n, 1), dtype=t.uint8, device=codec.device)
    launch(stream, off, ok)
    t.cuda.synchronize(codec.device)
    end = int(off[n].item())
    return stream[:end], off, ok[:n]

