"""CPU: the oracle (oracle/bft_oracle.c) and the wave emulator running the kernel bodies (tests/emu/wave_emu.cpp
over consensus-rs_amd/csrc/bft_wave.h, bft_fast64.h, bft_kwave.h) built with -fsanitize=address,undefined into one
executable (tests/emu/san_main.cpp), which compares them on the emulator-parity shapes and a short fuzz pass.

Any out-of-bounds access, use-after-free or undefined operation (shift widths, signed overflow, misaligned
loads) in the restated handlers or in the kernel bodies' index arithmetic aborts the run; the exit status also
counts parity mismatches. Test-only (SURVEY §5 sanitizers)."""
import os
import random
import shutil
import subprocess

import pytest

from bftsim.configs import BftConfig, cfg1, cfg2, cfg3, cfg4, cfg5

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tests", "emu", "_san")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O0"]


def _build():
    exe = os.path.join(OUT, "san_parity")
    srcs = [os.path.join(ROOT, "tests", "emu", "san_main.cpp"), os.path.join(ROOT, "tests", "emu", "wave_emu.cpp"),
            os.path.join(ROOT, "oracle", "bft_oracle.c"), os.path.join(ROOT, "oracle", "secp_oracle.c")]
    srcs += [os.path.join(ROOT, "consensus-rs_amd", "csrc", f) for f in
             ("bft_wave.h", "bft_fast64.h", "bft_kwave.h", "bft_common.h", "bft_host.h")]
    if os.path.exists(exe) and all(os.path.getmtime(exe) >= os.path.getmtime(s) for s in srcs):
        return exe
    os.makedirs(OUT, exist_ok=True)
    objs = []
    for c in ("bft_oracle.c", "secp_oracle.c"):
        o = os.path.join(OUT, c + ".o")
        subprocess.check_call(["gcc", "-std=gnu11", "-mpopcnt", "-c", "-o", o, os.path.join(ROOT, "oracle", c)] + SAN)
        objs.append(o)
    tmp = f"{exe}.{os.getpid()}.tmp"
    subprocess.check_call(["g++", "-std=c++17", "-Wno-unknown-pragmas", "-DBFT_EMU_CHECKS", "-o", tmp, srcs[0]] + objs + SAN +
                          ["-lpthread"])
    os.replace(tmp, exe)
    return exe


def _line(cfg: BftConfig, first: int, n_inst: int, window: int = 0) -> str:
    s = cfg.silent_mask()
    v = [cfg.n, cfg.heights, cfg.max_ticks, cfg.seed, cfg.drop_ppm, cfg.byz_count, cfg.proposer_crash_ppm,
         cfg.phase_cap, *s, cfg.seed_byte_order, cfg.backlog_mode, first, n_inst, window]
    return " ".join(str(int(x)) for x in v) + " " + cfg.address_bytes().hex()


def _cases():
    import dataclasses
    out = [
        (cfg1(True, heights=20), 0, 1, 0), (cfg1(False, heights=20), 0, 1, 0),
        (cfg2(heights=20), 100, 48, 0), (cfg2(heights=20, byz=1), 7, 16, 0),
        (cfg3(heights=12), 0, 2, 0), (dataclasses.replace(cfg3(heights=10), seed_byte_order=1), 3, 1, 0),
        (BftConfig(n=64, heights=10, seed=15, byz_count=21, drop_ppm=50_000), 0, 2, 0),   # FAST → resume hand-over
        (cfg4(7, heights=15), 0, 8, 0), (cfg4(100, heights=6), 0, 1, 0), (cfg4(256, heights=4), 0, 1, 0),
        (BftConfig(n=10, heights=15, seed=9, drop_ppm=100_000, backlog_mode=1), 0, 6, 0),  # replay mode
        (cfg5(heights=150), 0, 8, 64), (BftConfig(n=10, heights=150, seed=51, drop_ppm=100_000,
                                                  proposer_crash_ppm=200_000), 0, 4, 64),
    ]
    sys_path_tests = os.path.join(ROOT, "tests")
    import sys
    sys.path.insert(0, sys_path_tests)
    import fuzz_parity as F
    rng = random.Random(20260518)
    for k in range(24):
        mode = k % 4
        cfg = F.random_config(rng, big=(mode == 1), n64=(mode == 2), replay=False, le=(k % 5 == 0),
                              lossless=(mode == 3))
        if cfg.n > 64:
            cfg = dataclasses.replace(cfg, heights=min(cfg.heights, 6), max_ticks=40)
        out.append((cfg, rng.randrange(1 << 20), 1 if cfg.n > 64 else 2, 0))
    return out


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="needs gcc/g++")
def test_oracle_and_emulator_under_asan_ubsan():
    exe = _build()
    cases = _cases()
    stdin = "\n".join(_line(*c) for c in cases) + "\n"
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:detect_stack_use_after_return=0:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe], input=stdin, capture_output=True, text=True, env=env, timeout=1500)
    oks = [l for l in r.stdout.splitlines() if l.startswith("ok ")]
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-6000:])
    assert len(oks) == len(cases), r.stdout[-2000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-6000:]
