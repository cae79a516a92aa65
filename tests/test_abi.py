"""libbftsim loads without a GPU and exports every entry point include/bftsim.h declares."""
import ctypes
import os
import re

import pytest

from bftsim import runtime, _abi
from bftsim.configs import cfg3

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "bftsim.h")).read()
    return sorted(set(re.findall(r"\b(bftsim_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = runtime.lib()
    syms = declared_symbols()
    assert len(syms) >= 15
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing


def test_struct_layouts_match_header():
    # offsets the C side relies on (x86-64 SysV)
    assert ctypes.sizeof(_abi.CConfig) == 4 * 4 + 8 * 2 + 4 * 4 + 8 * 4 + 8 + 20 + 4 + 8
    assert ctypes.sizeof(_abi.CResult) == 9 * 8
    assert ctypes.sizeof(_abi.CStats) == 8 * (4 + 7 + 65 + 65)


def test_create_rejects_bad_configs_without_gpu():
    L = runtime.lib()
    c = cfg3(heights=5)
    cc, keep = _abi.to_cconfig(c)
    h = ctypes.c_void_p()
    cc.n = 0
    assert L.bftsim_create(ctypes.byref(cc), 0, ctypes.byref(h)) < 0
    cc.n = 257
    assert L.bftsim_create(ctypes.byref(cc), 0, ctypes.byref(h)) == -4      # N > 256: unsupported
    cc.n = 64
    cc.phase_cap = 0
    assert L.bftsim_create(ctypes.byref(cc), 0, ctypes.byref(h)) < 0


def test_no_cpu_fallback_when_library_missing(monkeypatch, tmp_path):
    monkeypatch.setattr(runtime, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(runtime, "_lib", None)
    with pytest.raises(runtime.BftsimError):
        runtime.lib()
