#!/usr/bin/env python3
"""Summarise rocprofv3 outputs of scripts/gpu_profile.sh into one JSON (profiles/<round>/pmc_summary.json):
per kernel, the average duration (kernel trace), and per dispatch the HBM bytes from the PMC passes,
corrected as /opt/skills/guides/MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE and WRITE_SIZE are
KiB; on gfx950 FETCH_SIZE reports half of the bytes of wide streaming reads, so it is doubled
(an upper bound for narrower reads). bench.py reads `traffic` from this file.

usage: pmc_summary.py <prof dir> <out.json>"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SHORT = {"bft_consensus_fast_kernel": "bft_consensus_fast_kernel",
         "bft_consensus_resume_kernel": "bft_consensus_resume_kernel",
         "bft_consensus_kernel": "bft_consensus_kernel", "bft_hash_pair_kernel": "bft_hash_kernel",
         "bft_hash_lane_kernel": "bft_hash_kernel", "bft_hash_suffix_kernel": "bft_hash_suffix_kernel",
         "bft_hash_chain_kernel": "bft_hash_chain_kernel",
         "bft_stats_kernel": "bft_stats_kernel", "bft_tip_kernel": "bft_tip_kernel"}


def short(name):
    for k, v in SHORT.items():
        if k in name:
            return v
    return None


def counters(path):
    acc = defaultdict(lambda: defaultdict(list))
    meta = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if not k:
                continue
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta[k] = dict(kernel_name=r["Kernel_Name"], vgpr=int(r["VGPR_Count"]), sgpr=int(r["SGPR_Count"]),
                           lds_bytes=int(r["LDS_Block_Size"]), scratch=int(r["Scratch_Size"]),
                           grid=int(r["Grid_Size"]), workgroup=int(r["Workgroup_Size"]))
    return acc, meta


def stats(path):
    out = {}
    for f in glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Name"])
            if k:
                out[k] = dict(calls=int(r["Calls"]), avg_ns=float(r["AverageNs"]), name=r["Name"])
    return out


def main():
    root, dst = sys.argv[1], sys.argv[2]
    res = {"source": "rocprofv3 --kernel-trace --stats and separate --pmc passes (scripts/gpu_profile.sh)",
           "kernels": {}}
    st = stats(os.path.join(root, "stats"))
    fetch, meta = counters(os.path.join(root, "fetch"))
    write, meta2 = counters(os.path.join(root, "write"))
    sq, meta3 = counters(os.path.join(root, "sq"))
    meta.update(meta2)
    meta.update(meta3)
    for k in set(st) | set(fetch) | set(write) | set(sq):
        e = dict(meta.get(k, {}))
        if k in st:
            e.update(avg_ms=st[k]["avg_ns"] / 1e6, calls=st[k]["calls"])
        f = fetch.get(k, {}).get("FETCH_SIZE")
        w = write.get(k, {}).get("WRITE_SIZE")
        if f:
            e["fetch_bytes_raw"] = 1024.0 * sum(f) / len(f)
            e["fetch_bytes"] = 2.0 * e["fetch_bytes_raw"]      # gfx950 FETCH_SIZE correction
        if w:
            e["write_bytes"] = 1024.0 * sum(w) / len(w)
        if f and w:
            e["hbm_bytes_per_dispatch"] = e["fetch_bytes"] + e["write_bytes"]
        for c, v in sq.get(k, {}).items():
            e[c] = sum(v) / len(v)
        res["kernels"][k] = e
    # N = 64 launches run the FAST kernel then the resume kernel (one dispatch each per launch):
    # bench.py's HIP events bracket both, so the consensus entry is their per-launch sum
    ks = res["kernels"]
    parts = [ks.get("bft_consensus_fast_kernel"), ks.get("bft_consensus_resume_kernel")]
    if all(parts) and "bft_consensus_kernel" not in ks:
        e = {"composed_of": ["bft_consensus_fast_kernel", "bft_consensus_resume_kernel"]}
        for f in ("avg_ms", "fetch_bytes_raw", "fetch_bytes", "write_bytes", "hbm_bytes_per_dispatch"):
            if all(f in x for x in parts):
                e[f] = parts[0][f] + parts[1][f]
        ks["bft_consensus_kernel"] = e
    # the block-hash pass is a suffix kernel then a chain kernel per launch (kern_fast.hip); bench.py's HIP
    # events bracket both, so the hash entry is their per-launch sum (SQ counters summed too)
    parts = [ks.get("bft_hash_suffix_kernel"), ks.get("bft_hash_chain_kernel")]
    if all(parts) and "bft_hash_kernel" not in ks:
        e = {"composed_of": ["bft_hash_suffix_kernel", "bft_hash_chain_kernel"]}
        for f in ["avg_ms", "fetch_bytes_raw", "fetch_bytes", "write_bytes", "hbm_bytes_per_dispatch"] + \
                 [c for c in parts[1] if c.startswith("SQ_")]:
            if all(f in x for x in parts):
                e[f] = parts[0][f] + parts[1][f]
        ks["bft_hash_kernel"] = e
    json.dump(res, open(dst, "w"), indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
