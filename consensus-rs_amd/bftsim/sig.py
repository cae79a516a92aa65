"""Host binding of libbftsig (include/bftsig.h): batched secp256k1 recoverable ECDSA on the GPU.

Mirrors the ethkey calls the reference makes per message (names and argument meaning kept):
  * `sign(secrets, digests)`          Hash::sign / ethkey::sign (src/protocol/mod.rs:88-92,
                                      src/types/votes.rs:94-101, src/consensus/backend.rs:245-252);
  * `recover(digests, signatures)`    recover_bytes + public_to_address (src/protocol/mod.rs:103-116);
  * `verify_address(addresses, digests, signatures)`  verify_address (commit.rs:96-100);
  * `secret_to_address(secrets)`      KeyPair::from_secret(..).address().
Batches are torch uint8 tensors on the GPU ([n,32] secrets/digests, [n,65] signatures, [n,20]
addresses) or numpy arrays (copied to the device). Per-item failures come back as ok == 0 (the
reference's `Err`); there is no CPU fallback: a missing libbftsig.so raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .runtime import lib_override

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = lib_override("BFTSIG_LIB") or os.path.join(PKG_DIR, "build", "libbftsig.so")

_lib = None


class BftsigError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise BftsigError(f"libbftsig.so not built ({LIB_PATH}); run __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        vp, u64 = ctypes.c_void_p, ctypes.c_uint64
        L.bftsig_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
        L.bftsig_destroy.argtypes = [vp]
        L.bftsig_last_error.argtypes = [vp]
        L.bftsig_last_error.restype = ctypes.c_char_p
        L.bftsig_secret_to_address.argtypes = [vp, vp, u64, vp, vp, vp, vp]
        L.bftsig_sign.argtypes = [vp, vp, vp, vp, u64, vp, vp, vp]
        L.bftsig_recover.argtypes = [vp, vp, vp, u64, vp, vp, vp, vp]
        L.bftsig_verify_address.argtypes = [vp, vp, vp, vp, u64, vp, vp]
        _lib = L
    return _lib


class Signer:
    """One device's signer (holds the fixed-base table of G)."""

    def __init__(self, device: int = 0):
        import torch
        self.torch = torch
        self.device = torch.device("cuda", device)
        h = ctypes.c_void_p()
        rc = lib().bftsig_create(device, ctypes.byref(h))
        self.h = h.value
        self._check(rc, "bftsig_create")

    def close(self):
        if self.h:
            lib().bftsig_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            msg = lib().bftsig_last_error(self.h).decode() if self.h else ""
            raise BftsigError(f"{what} failed ({rc}): {msg}")

    def _dev(self, a, width, dtype=None):
        t = self.torch
        if isinstance(a, (bytes, bytearray)):
            a = np.frombuffer(bytes(a), dtype=np.uint8)
        if isinstance(a, np.ndarray):
            a = t.from_numpy(np.ascontiguousarray(a))
        a = a.to(self.device).contiguous()
        if width is not None:
            a = a.view(t.uint8).reshape(-1, width)
        return a

    def _stream(self, stream):
        return stream if stream is not None else self.torch.cuda.current_stream(self.device).cuda_stream

    def secret_to_address(self, secrets, stream=None):
        t = self.torch
        s = self._dev(secrets, 32)
        n = s.shape[0]
        pub = t.empty((n, 64), dtype=t.uint8, device=self.device)
        addr = t.empty((n, 20), dtype=t.uint8, device=self.device)
        ok = t.empty((n,), dtype=t.uint8, device=self.device)
        self._check(lib().bftsig_secret_to_address(self.h, s.data_ptr(), n, pub.data_ptr(), addr.data_ptr(),
                                                   ok.data_ptr(), self._stream(stream)), "bftsig_secret_to_address")
        return pub, addr, ok

    def sign(self, secrets, digests, key_index=None, stream=None):
        t = self.torch
        s = self._dev(secrets, 32)
        d = self._dev(digests, 32)
        n = d.shape[0]
        ki = None
        if key_index is not None:
            ki = self._dev(np.asarray(key_index, dtype=np.int32) if not isinstance(key_index, t.Tensor)
                           else key_index.to(t.int32), None)
            if ki.numel() != n or (n and (int(ki.min()) < 0 or int(ki.max()) >= s.shape[0])):
                raise BftsigError("key_index out of range")
        elif s.shape[0] != n:
            raise BftsigError("one secret per digest, or a key_index")
        sig = t.empty((n, 65), dtype=t.uint8, device=self.device)
        ok = t.empty((n,), dtype=t.uint8, device=self.device)
        self._check(lib().bftsig_sign(self.h, s.data_ptr(), ki.data_ptr() if ki is not None else None, d.data_ptr(), n,
                                      sig.data_ptr(), ok.data_ptr(), self._stream(stream)), "bftsig_sign")
        return sig, ok

    def recover(self, digests, signatures, want_pub=True, stream=None):
        t = self.torch
        d = self._dev(digests, 32)
        g = self._dev(signatures, 65)
        n = d.shape[0]
        if g.shape[0] != n:
            raise BftsigError("one signature per digest")
        pub = t.empty((n, 64), dtype=t.uint8, device=self.device) if want_pub else None
        addr = t.empty((n, 20), dtype=t.uint8, device=self.device)
        ok = t.empty((n,), dtype=t.uint8, device=self.device)
        self._check(lib().bftsig_recover(self.h, d.data_ptr(), g.data_ptr(), n, pub.data_ptr() if want_pub else None,
                                         addr.data_ptr(), ok.data_ptr(), self._stream(stream)), "bftsig_recover")
        return pub, addr, ok

    def verify_address(self, addresses, digests, signatures, stream=None):
        t = self.torch
        a = self._dev(addresses, 20)
        d = self._dev(digests, 32)
        g = self._dev(signatures, 65)
        n = d.shape[0]
        if a.shape[0] != n or g.shape[0] != n:
            raise BftsigError("one address and one signature per digest")
        ok = t.empty((n,), dtype=t.uint8, device=self.device)
        self._check(lib().bftsig_verify_address(self.h, a.data_ptr(), d.data_ptr(), g.data_ptr(), n, ok.data_ptr(),
                                                self._stream(stream)), "bftsig_verify_address")
        return ok
