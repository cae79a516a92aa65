"""Randomized parity fuzz: CPU wave emulator (the kernel body) vs the oracle on random configs.
Usage: python tests/fuzz_parity.py [seconds] [rng seed] [big]. `big` draws N in 65..256 (the
workgroup-segment kernels), `n64` N = 64 (the FAST kernel and its hand-overs), `lossless64` N = 64 without drops
or crashes (the canonical step and tick, with phase caps, short max_ticks and silent validators); a fourth argument
`replay` runs every config in backlog replay mode (SPEC.md §10), `le` with little-endian U128 seeds. Test-only tool (not collected by pytest)."""
import random
import sys
import time

import oracle_lib as O
import emu_lib as E
from bftsim.configs import BftConfig
from parity_util import mismatches


def random_config(rng, big=False, n64=False, replay=False, le=False, lossless=False):
    if lossless:                         # N = 64 without drops or crashes: the canonical step and tick
        n = 64
        byz = rng.choice([0, 1, 5, 21, 21, 21, 30, 42, 43])
        cap = rng.choice([16, 16, 3, 4, 5, 6, 8])
        silent = rng.sample(range(n), k=rng.choice([0, 0, 0, 1]))
        heights = rng.choice([5, 20, 70, 130])
        return BftConfig(n=n, heights=heights, seed=rng.randrange(1 << 40), byz_count=byz, phase_cap=cap,
                         silent=silent, max_ticks=heights * rng.choice([1, 2, 4]) + rng.choice([0, 1, 16]),
                         seed_byte_order=1 if le else 0,
                         name=f"lossless-b{byz}-cap{cap}-s{len(silent)}-h{heights}{'-le' if le else ''}")
    if n64:                              # the FAST kernel (bft_fast64.h) and its hand-overs
        n = 64
    elif big:
        n = rng.choice([65, 66, 80, 100, 127, 128, 129, 150, 200, 255, 256])
    else:
        n = rng.choice([1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 13, 16, 17, 21, 31, 32, 33, 40, 63, 64])
    byz = rng.choice([0, 0, 0, 1, n // 3, max(0, (n - 1) // 3), n // 2])
    drop = rng.choice([0, 0, 20_000, 100_000, 250_000, 500_000])
    crash = rng.choice([0, 0, 100_000, 400_000])
    cap = rng.choice([16, 16, 4, 2, 8])
    silent = rng.sample(range(n), k=rng.choice([0, 0, 1, min(2, n)])) if n > 1 else []
    heights = rng.choice([5, 20, 40])
    return BftConfig(n=n, heights=heights, seed=rng.randrange(1 << 40), byz_count=byz,
                     drop_ppm=drop, proposer_crash_ppm=crash, phase_cap=cap, silent=silent,
                     max_ticks=heights * 4 + 16, backlog_mode=1 if replay else 0, seed_byte_order=1 if le else 0,
                     name=f"n{n}-b{byz}-d{drop}-c{crash}-cap{cap}-s{len(silent)}{'-replay' if replay else ''}"
                          f"{'-le' if le else ''}")


def main():
    budget = float(sys.argv[1]) if len(sys.argv) > 1 else 60
    rng = random.Random(int(sys.argv[2]) if len(sys.argv) > 2 else 1234)
    big = len(sys.argv) > 3 and sys.argv[3] == "big"
    n64 = len(sys.argv) > 3 and sys.argv[3] == "n64"
    replay = "replay" in sys.argv[3:]
    le = "le" in sys.argv[3:]                     # little-endian U128 seeds (hash-dependent proposers)
    lossless = len(sys.argv) > 3 and sys.argv[3] == "lossless64"
    t0, runs, fails = time.time(), 0, 0
    while time.time() - t0 < budget:
        cfg = random_config(rng, big, n64, replay, le, lossless)
        first = rng.randrange(1 << 20)
        n_inst = rng.choice([1, 2] if big else [1, 3, 8])
        a = O.run(cfg, first, n_inst)
        b = E.run(cfg, first, n_inst)
        bad = mismatches(a, b)
        runs += 1
        if bad:
            fails += 1
            print("MISMATCH", cfg.name, cfg.seed, first, n_inst, bad, flush=True)
    print(f"fuzz: {runs} configs, {fails} mismatches", flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
