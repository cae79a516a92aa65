#!/usr/bin/env python3
"""Concurrency profile of a rocprofv3 kernel trace (test/analysis tool): for the last `--launches` consensus
launches of a bench run, the wall time, the time each kernel family is running, and the time with none.
usage: trace_overlap.py run_kernel_trace.csv [--window-from-kernel NAME] [--last N]"""
import csv
import sys


def fam(name):
    for k in ("fast_kernel", "resume_kernel", "hash_chain", "hash_suffix", "consensus_kernel", "fill", "copy"):
        if k in name:
            return k
    return "other"


def main():
    path = sys.argv[1]
    last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 20
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), fam(r["Kernel_Name"]), r["Queue_Id"])
            for r in csv.DictReader(open(path))]
    rows.sort()
    fast = [r for r in rows if r[2] == "fast_kernel"]
    t0 = fast[-last][0]
    t1 = max(e for s, e, f, q in rows if s >= t0)
    ev = []
    for s, e, f, q in rows:
        if e <= t0 or s >= t1:
            continue
        ev.append((max(s, t0), 1, f))
        ev.append((min(e, t1), -1, f))
    ev.sort()
    active, busy, cur, prev = {}, {}, 0, t0
    none = 0
    for t, d, f in ev:
        dt = t - prev
        if cur == 0:
            none += dt
        for k, n in active.items():
            if n > 0:
                busy[k] = busy.get(k, 0) + dt
        active[f] = active.get(f, 0) + d
        cur += d
        prev = t
    wall = t1 - t0
    print(f"window: last {last} FAST launches, {wall / 1e6:.3f} ms; idle (no kernel) {none / 1e6:.3f} ms "
          f"({100 * none / wall:.1f} %)")
    for k, v in sorted(busy.items(), key=lambda kv: -kv[1]):
        print(f"  {k:18s} running {v / 1e6:8.3f} ms ({100 * v / wall:5.1f} % of the window)")
    queues = sorted({q for s, e, f, q in rows if s >= t0})
    print("  hardware queues used:", queues)


if __name__ == "__main__":
    main()
