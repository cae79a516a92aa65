#!/usr/bin/env python3
"""Each counter of a rocprofv3 --pmc pass summed per kernel family, with the dispatch count (analysis tool).
usage: pmc_by_kernel.py run_counter_collection.csv"""
import csv
import sys
from collections import defaultdict


def fam(name):
    for k in ("fast_kernel", "resume_kernel", "hash_chain_lane", "hash_chain", "hash_suffix", "spec_byz",
              "spec_suffix", "spec_verify", "clear_kernel", "stats_kernel"):
        if k in name:
            return k
    return name[:40]


def main():
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in csv.DictReader(open(sys.argv[1])):
        f = fam(r["Kernel_Name"])
        tot[f][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[f].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    for f in sorted(tot, key=lambda k: -len(disp[k])):
        print(f"{f:18s} dispatches {len(disp[f]):4d}  " +
              "  ".join(f"{c} {v:.4g}" for c, v in sorted(tot[f].items())))


if __name__ == "__main__":
    main()
