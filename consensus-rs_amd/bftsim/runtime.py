"""Host binding of libbftsim (the HIP path). Mirrors the reference's engine surface:
`Simulator` stands for one `create_bft_engine` per instance (src/consensus/consensus.rs:42-60),
batched. There is no CPU fallback: if the HIP library is missing this raises."""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _abi
from .configs import BftConfig

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def lib_override(var: str):
    """A/B builds (scripts/gpu_ab*.sh) may point a binding at another library, but only when
    BFTSIM_TESTING=1 is set too: a stray BFTSIM_LIB-style variable never swaps the product library silently."""
    v = os.environ.get(var)
    if not v:
        return None
    if os.environ.get("BFTSIM_TESTING") != "1":
        raise RuntimeError(f"{var}={v} is set but BFTSIM_TESTING=1 is not: refusing to load a non-product library")
    import sys
    print(f"bftsim: {var} override -> {v} (BFTSIM_TESTING)", file=sys.stderr)
    return v


LIB_PATH = lib_override("BFTSIM_LIB") or os.path.join(PKG_DIR, "build", "libbftsim.so")

_lib = None
HEADER_SLOT = 288                       # BFTSIM_HEADER_SLOT (include/bftsim.h)


class BftsimError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise BftsimError(f"libbftsim.so not built ({LIB_PATH}); run __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        L.bftsim_create.argtypes = [ctypes.POINTER(_abi.CConfig), ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        L.bftsim_destroy.argtypes = [ctypes.c_void_p]
        L.bftsim_last_error.argtypes = [ctypes.c_void_p]
        L.bftsim_last_error.restype = ctypes.c_char_p
        L.bftsim_run.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(_abi.CResult)]
        L.bftsim_prepare.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        L.bftsim_launch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        L.bftsim_sync.argtypes = [ctypes.c_void_p]
        L.bftsim_fetch.argtypes = [ctypes.c_void_p, ctypes.POINTER(_abi.CResult)]
        L.bftsim_stats_get.argtypes = [ctypes.c_void_p, ctypes.POINTER(_abi.CStats)]
        L.bftsim_stats_allreduce.argtypes = [ctypes.c_void_p, ctypes.POINTER(_abi.CStats)]
        L.bftsim_comm_unique_id.argtypes = [ctypes.c_void_p]
        L.bftsim_set_crypto.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint32]
        L.bftsim_ledger_slot_bytes.argtypes = [ctypes.c_uint32]
        L.bftsim_ledger_slot_bytes.restype = ctypes.c_uint64
        L.bftsim_export_ledger.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                           ctypes.c_void_p]
        L.bftsim_crypto_verify.argtypes = [ctypes.c_void_p, ctypes.POINTER(_abi.CCryptoReport), ctypes.c_uint64,
                                           ctypes.c_void_p, ctypes.c_void_p]
        L.bftsim_launched_count.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                                            ctypes.POINTER(ctypes.c_uint64)]
        L.bftsim_comm_init.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_char_p]
        L.bftsim_last_kernel_ms.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float),
                                            ctypes.POINTER(ctypes.c_float)]
        L.bftsim_kernel_ms_sum.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint32)]
        L.bftsim_set_pipeline.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.bftsim_set_hash_batch.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        L.bftsim_set_fast.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.bftsim_set_trace.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
        L.bftsim_set_window.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        if hasattr(L, "bftsim_set_rcs_capacity"):     # (absent from A/B builds of earlier rounds)
            L.bftsim_set_rcs_capacity.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        L.bftsim_fetch_summary.argtypes = [ctypes.c_void_p, ctypes.c_uint64] + [ctypes.c_void_p] * 5
        L.bftsim_two_thirds_majority.restype = ctypes.c_uint32
        L.bftsim_seed_from_hash.restype = ctypes.c_uint32
        L.bftsim_seed_from_hash.argtypes = [ctypes.c_char_p, ctypes.c_uint32]
        L.bftsim_seed_from_hash_order.restype = ctypes.c_uint32
        L.bftsim_seed_from_hash_order.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32]
        L.bftsim_two_thirds_majority.argtypes = [ctypes.c_uint32]
        L.bftsim_calc_proposer.restype = ctypes.c_uint32
        L.bftsim_calc_proposer.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint64]
        L.bftsim_keccak256.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p]
        L.bftsim_genesis_hash.argtypes = [ctypes.POINTER(_abi.CConfig), ctypes.c_void_p]
        L.bftsim_view_cmp.argtypes = [ctypes.c_uint64] * 4
        L.bftsim_export_headers.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
        _lib = L
    return _lib


def keccak256(data: bytes) -> bytes:
    """Keccak-256 (`hash`, cryptocurrency-kit) through libbftsim (host code, no GPU needed)."""
    out = ctypes.create_string_buffer(32)
    lib().bftsim_keccak256(data, len(data), out)
    return out.raw


def _check(h, rc, what):
    if rc != 0:
        msg = lib().bftsim_last_error(h).decode() if h else ""
        raise BftsimError(f"{what} failed ({rc}): {msg}")


class Simulator:
    """Runs many independent seeded consensus-rs clusters of one configuration on one GPU."""

    def __init__(self, cfg: BftConfig, device: int = 0):
        self.cfg = cfg
        self._c, self._keep = _abi.to_cconfig(cfg)
        h = ctypes.c_void_p()
        rc = lib().bftsim_create(ctypes.byref(self._c), device, ctypes.byref(h))
        self.h = h.value
        _check(self.h, rc, "bftsim_create")
        self.n_prepared = 0
        self.n_launched = 0             # instances of the last launch: what fetch / crypto_verify read

    def close(self):
        if self.h:
            lib().bftsim_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def run(self, first: int, n: int, trace_ticks: int = 0):
        r, arrs = _abi.alloc_result(n, self.cfg.heights)
        tr = None
        if trace_ticks:
            tr = np.zeros(n * trace_ticks * self.cfg.n, np.uint64)
            _check(self.h, lib().bftsim_set_trace(self.h, tr.ctypes.data, trace_ticks), "set_trace")
        try:
            _check(self.h, lib().bftsim_run(self.h, first, n, ctypes.byref(r)), "bftsim_run")
            self.n_prepared = self.n_launched = n
        finally:
            if trace_ticks:
                lib().bftsim_set_trace(self.h, None, 0)
        arrs = _abi.shape_result(arrs, n, self.cfg.heights)
        if tr is not None:
            arrs["trace"] = tr.reshape(n, trace_ticks, self.cfg.n)
        st = self.stats()
        arrs["round_hist"] = np.array(st["round_hist"], np.uint64)
        arrs["latency_hist"] = np.array(st["latency_hist"], np.uint64)
        return arrs

    def set_window(self, window: int):
        """Keep a ring of `window` canonical rows per instance (0: every height); see bftsim.h."""
        _check(self.h, lib().bftsim_set_window(self.h, window), "bftsim_set_window")

    def set_rcs_capacity(self, rounds: int):
        """RoundChangeSet rounds kept per validator (bftsim_set_rcs_capacity); run() re-runs an
        overflowing batch at twice the capacity."""
        _check(self.h, lib().bftsim_set_rcs_capacity(self.h, rounds), "bftsim_set_rcs_capacity")

    def launched(self):
        """(first, n) of the last launch: the rows the fetch family writes (bftsim_launched_count)."""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        _check(self.h, lib().bftsim_launched_count(self.h, ctypes.byref(a), ctypes.byref(b)), "bftsim_launched_count")
        return a.value, b.value

    def fetch_summary(self, n: int = None, tips: bool = True):
        """Per-instance outputs of the last launch into buffers of `n` instances (default: the launched
        count; a smaller n is refused by the library, bftsim.h)."""
        if n is None:
            n = self.launched()[1]
        out = dict(committed_height=np.zeros(n, np.uint64), flags=np.zeros(n, np.uint32),
                   ticks=np.zeros(n, np.uint32), views=np.zeros(n, np.uint64))
        if tips:
            out["tip_hash"] = np.zeros((n, 32), np.uint8)
        _check(self.h, lib().bftsim_fetch_summary(
            self.h, n, out["committed_height"].ctypes.data, out["flags"].ctypes.data, out["ticks"].ctypes.data,
            out["views"].ctypes.data, out["tip_hash"].ctypes.data if tips else None), "bftsim_fetch_summary")
        return out

    def run_stream(self, first: int, n: int, window: int = 256):
        """Windowed run (long horizons): per-instance outputs, tip hashes and histograms."""
        self.set_window(window)
        self.prepare(n)
        self.launch(first)
        out = self.fetch_summary(n)
        st = self.stats()
        out["round_hist"] = np.array(st["round_hist"], np.uint64)
        out["latency_hist"] = np.array(st["latency_hist"], np.uint64)
        return out

    # device-resident path (bench)
    def prepare(self, n: int):
        _check(self.h, lib().bftsim_prepare(self.h, n), "bftsim_prepare")
        self.n_prepared = n

    def launch(self, first: int, stream: int = 0):
        _check(self.h, lib().bftsim_launch(self.h, first, ctypes.c_void_p(stream)), "bftsim_launch")
        self.n_launched = self.n_prepared

    def fetch(self):
        """Per-height results of the last launch (all its instances), as run() returns them. Sized by the
        launch, not by a later prepare: the C side writes the launched count."""
        n = self.n_launched
        r, arrs = _abi.alloc_result(n, self.cfg.heights)
        _check(self.h, lib().bftsim_fetch(self.h, ctypes.byref(r)), "bftsim_fetch")
        return _abi.shape_result(arrs, n, self.cfg.heights)

    def export_headers(self, n: int = None):
        """Ledger export of the last run / launch (core/ledger.rs:193-245): ([n, H] list of the Header
        bytes of every committed height, empty beyond it). Keccak-256 of each is its block hash."""
        if n is None:
            n = self.launched()[1]
        H = self.cfg.heights
        slot = HEADER_SLOT
        buf = np.zeros(n * H * slot, np.uint8)
        lens = np.zeros(n * H, np.uint32)
        _check(self.h, lib().bftsim_export_headers(self.h, n, buf.ctypes.data, lens.ctypes.data),
               "bftsim_export_headers")
        buf = buf.reshape(n, H, slot)
        lens = lens.reshape(n, H)
        return [[bytes(buf[i, x, :lens[i, x]]) for x in range(H)] for i in range(n)]

    def sync(self):
        _check(self.h, lib().bftsim_sync(self.h), "bftsim_sync")

    def kernel_ms(self):
        a, b = ctypes.c_float(), ctypes.c_float()
        _check(self.h, lib().bftsim_last_kernel_ms(self.h, ctypes.byref(a), ctypes.byref(b)), "kernel_ms")
        return a.value, b.value

    def kernel_ms_sum(self):
        """(consensus ms, hash ms, launches) summed over the launches since the previous call."""
        a, b, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_uint32()
        _check(self.h, lib().bftsim_kernel_ms_sum(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(n)),
               "kernel_ms_sum")
        return a.value, b.value, n.value

    def set_fast(self, on: bool):
        """Verification switch: False runs N = 64 through the full kernel alone (identical results)."""
        _check(self.h, lib().bftsim_set_fast(self.h, 1 if on else 0), "bftsim_set_fast")

    def set_pipeline(self, on, depth: int = 2):
        """Batch throughput mode: a ring of `depth` row-table sets; the hash pass of each launch overlaps
        the following launches (include/bftsim.h bftsim_set_pipeline)."""
        _check(self.h, lib().bftsim_set_pipeline(self.h, depth if on else 0), "bftsim_set_pipeline")

    def set_hash_batch(self, launches: int):
        """Pipelined launches: the chains of this many consecutive launches as one kernel (include/bftsim.h)."""
        _check(self.h, lib().bftsim_set_hash_batch(self.h, launches), "bftsim_set_hash_batch")

    @staticmethod
    def _stats_dict(s):
        return dict(instances=s.instances, committed_heights=s.committed_heights, views=s.views,
                    ticks=s.ticks, flagged=list(s.flagged), round_hist=list(s.round_hist),
                    latency_hist=list(s.latency_hist))

    def stats(self):
        s = _abi.CStats()
        _check(self.h, lib().bftsim_stats_get(self.h, ctypes.byref(s)), "bftsim_stats_get")
        return self._stats_dict(s)

    def set_crypto(self, secrets, forged=(), log_cap: int = 0):
        """Real-crypto mode (include/bftsim.h bftsim_set_crypto, SPEC.md §11): `secrets` = one 32-byte
        key per validator in the sorted validator order (None turns the mode off); `forged` = indices
        that sign with a key that is not theirs. Applies at the next prepare."""
        if secrets is None:
            _check(self.h, lib().bftsim_set_crypto(self.h, None, None, 0), "bftsim_set_crypto")
            return
        assert len(secrets) == self.cfg.n and all(len(k) == 32 for k in secrets)
        fb = bytes(1 if v in set(forged) else 0 for v in range(self.cfg.n))
        _check(self.h, lib().bftsim_set_crypto(self.h, b"".join(secrets), fb, log_cap), "bftsim_set_crypto")

    def crypto_verify(self):
        """The batched sign / recover pass over the last launch's messages: report dict, per-instance
        checksum [n, 32] (XOR of keccak(signature || seal)) and message counts [n]."""
        n = self.n_launched
        rep = _abi.CCryptoReport()
        ck = np.zeros((n, 32), np.uint8)
        cnt = np.zeros(n, np.uint32)
        _check(self.h, lib().bftsim_crypto_verify(self.h, ctypes.byref(rep), n, ck.ctypes.data, cnt.ctypes.data),
               "bftsim_crypto_verify")
        out = {k: getattr(rep, k) for k, _ in _abi.CCryptoReport._fields_}
        out["checksum"], out["inst_messages"] = ck, cnt
        return out

    def export_ledger(self):
        """The ledger Headers with votes of the last launch (after crypto_verify): per instance a list of
        header byte strings, height 1..committed (include/bftsim.h bftsim_export_ledger)."""
        n, H = self.n_launched, self.cfg.heights
        slot = lib().bftsim_ledger_slot_bytes(self.cfg.n)
        buf = np.zeros(n * H * slot, np.uint8)
        lens = np.zeros(n * H, np.uint32)
        _check(self.h, lib().bftsim_export_ledger(self.h, n, buf.ctypes.data, slot, lens.ctypes.data),
               "bftsim_export_ledger")
        out = []
        for i in range(n):
            row = []
            for x in range(H):
                k = int(lens[i * H + x])
                if k == 0:
                    break
                o = (i * H + x) * slot
                row.append(bytes(buf[o:o + k]))
            out.append(row)
        return out

    @staticmethod
    def comm_available():
        """raises unless librccl opens with every entry point libbftsim uses (bftsim_comm_available): the
        pre-flight each rank runs, and the ranks agree on, before any of them enters ncclCommInitRank"""
        rc = lib().bftsim_comm_available()
        if rc != 0:
            raise BftsimError(f"bftsim_comm_available failed ({rc}): librccl.so.1 cannot be opened")

    @staticmethod
    def comm_unique_id() -> bytes:
        """rank 0: the 128-byte RCCL id every rank passes to comm_init (include/bftsim.h)"""
        buf = ctypes.create_string_buffer(128)
        rc = lib().bftsim_comm_unique_id(buf)
        if rc != 0:
            raise BftsimError(f"bftsim_comm_unique_id failed ({rc})")
        return buf.raw

    def comm_init(self, world: int, rank: int, unique_id: bytes):
        assert len(unique_id) == 128
        _check(self.h, lib().bftsim_comm_init(self.h, world, rank, unique_id), "bftsim_comm_init")

    def stats_allreduce(self):
        """bftsim_stats of the last launch summed over every rank: one RCCL all-reduce in libbftsim"""
        s = _abi.CStats()
        _check(self.h, lib().bftsim_stats_allreduce(self.h, ctypes.byref(s)), "bftsim_stats_allreduce")
        return self._stats_dict(s)
