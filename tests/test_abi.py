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


def _c_layout():
    """offsetof/sizeof of every field, as the C compiler lays out include/bftsim.h"""
    import subprocess, tempfile
    structs = {"bftsim_config": [f for f, _ in _abi.CConfig._fields_],
               "bftsim_result": [f for f, _ in _abi.CResult._fields_],
               "bftsim_stats": [f for f, _ in _abi.CStats._fields_]}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "bftsim.h"', "int main(void) {"]
    for st, fields in structs.items():
        lines.append(f'printf("{st} sizeof %zu\\n", sizeof({st}));')
        for f in fields:
            lines.append(f'printf("{st} {f} %zu\\n", offsetof({st}, {f}));')
    lines.append("return 0; }")
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "l.c"), os.path.join(d, "l")
        open(src, "w").write("\n".join(lines))
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), "-o", exe, src])
        out = subprocess.check_output([exe]).decode().split("\n")
    return {tuple(l.split()[:2]): int(l.split()[2]) for l in out if l}


def test_struct_layouts_match_header():
    # the ctypes mirror (bftsim/_abi.py) against the C compiler's layout of include/bftsim.h
    lay = _c_layout()
    for name, cls in (("bftsim_config", _abi.CConfig), ("bftsim_result", _abi.CResult),
                      ("bftsim_stats", _abi.CStats)):
        assert lay[(name, "sizeof")] == ctypes.sizeof(cls), name
        for f, _ in cls._fields_:
            assert lay[(name, f)] == getattr(cls, f).offset, (name, f)


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
    # convention switches outside their enums (include/bftsim.h BFTSIM_SEED_* / _ENC_* / _BACKLOG_*)
    for field, bad in (("seed_byte_order", 2), ("header_encoding", 1), ("backlog_mode", 2), ("reserved", 1)):
        cc, keep = _abi.to_cconfig(c)
        setattr(cc, field, bad)
        assert L.bftsim_create(ctypes.byref(cc), 0, ctypes.byref(h)) == -1, field


def test_no_cpu_fallback_when_library_missing(monkeypatch, tmp_path):
    monkeypatch.setattr(runtime, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(runtime, "_lib", None)
    with pytest.raises(runtime.BftsimError):
        runtime.lib()
