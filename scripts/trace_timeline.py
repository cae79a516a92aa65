#!/usr/bin/env python3
"""Kernel timeline of a rocprofv3 kernel trace (analysis tool): every kernel dispatch of the window that starts
at the `--last` N-th last FAST kernel, one line each (start and duration in ms from the window's start, hardware
queue, kernel family, grid size).
usage: trace_timeline.py run_kernel_trace.csv [--last N]"""
import csv
import sys


def fam(name):
    for k in ("fast_kernel", "resume_kernel", "hash_chain", "hash_suffix", "spec_byz", "spec_suffix",
              "spec_verify", "consensus_kernel", "fill", "copy"):
        if k in name:
            return k
    return name[:30]


def main():
    path = sys.argv[1]
    last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 20
    rows = []
    for r in csv.DictReader(open(path)):
        grid = r.get("Grid_Size_X") or r.get("Grid_Size") or ""
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), fam(r["Kernel_Name"]), r["Queue_Id"], grid))
    rows.sort()
    fast = [r for r in rows if r[2] == "fast_kernel"]
    t0 = fast[-last][0]
    for s, e, f, q, g in rows:
        if s < t0:
            continue
        print(f"{(s - t0) / 1e6:8.3f} {(e - s) / 1e6:8.3f}  q{q:>3s}  {f:16s} {g}")


if __name__ == "__main__":
    main()
