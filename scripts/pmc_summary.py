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

SHORT = {"bft_hash_chain_lane_kernel": "bft_hash_chain_kernel",     # the chain dispatch, whichever kernel runs it
         "bft_spec_byz_kernel": "bft_spec_byz_kernel", "bft_spec_suffix_kernel": "bft_spec_suffix_kernel",
         "bft_spec_verify_kernel": "bft_spec_verify_kernel", "bft_clear_kernel": "bft_clear_kernel",
         "bft_consensus_fast_kernel": "bft_consensus_fast_kernel",
         "bft_consensus_resume_kernel": "bft_consensus_resume_kernel",
         "bft_consensus_kernel": "bft_consensus_kernel", "bft_hash_pair_kernel": "bft_hash_kernel",
         "bft_hash_lane_kernel": "bft_hash_kernel", "bft_hash_suffix_kernel": "bft_hash_suffix_kernel",
         "bft_hash_chain_kernel": "bft_hash_chain_kernel", "bft_seed_chain_kernel": "bft_seed_chain_kernel",
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


def attributed_writes(path):
    """The attribution pass (BFTSIM_PMC_EVICT=1, unpipelined: one queue): every kernel of a launch is followed
    by bft_l2_evict_kernel, which reads 64 MiB and so writes back what the kernel left dirty in L2. A kernel's
    attributed WRITE_SIZE = its own + that of the eviction right after it (same queue, next dispatch)."""
    rows = []
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == "WRITE_SIZE":
                rows.append((int(r["Queue_Id"]), int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    rows.sort()
    acc = defaultdict(list)
    for i, (q, _, name, v) in enumerate(rows):
        k = short(name)
        if not k or "bft_l2_evict_kernel" in name:
            continue
        ev = 0.0
        if i + 1 < len(rows) and rows[i + 1][0] == q and "bft_l2_evict_kernel" in rows[i + 1][2]:
            ev = rows[i + 1][3]
        acc[k].append((1024.0 * v, 1024.0 * ev))
    # per LAUNCH, not per dispatch: a launch whose heights exceed the suffix rows of one chunk runs a suffix + chain
    # dispatch per chunk, so each kernel's bytes are summed and divided by the launches (consensus dispatches)
    launches = len(acc.get("bft_consensus_fast_kernel") or acc.get("bft_consensus_kernel") or []) or None
    out = {}
    for k, v in acc.items():
        nl = launches or len(v)
        out[k] = {"write_bytes_own": sum(a for a, _ in v) / nl, "write_bytes_evicted_after": sum(b for _, b in v) / nl,
                  "write_bytes_attributed": sum(a + b for a, b in v) / nl, "dispatches": len(v),
                  "dispatches_per_launch": len(v) / nl}
    return out


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
    attr = attributed_writes(os.path.join(root, "write_evict")) if os.path.isdir(os.path.join(root, "write_evict")) else {}
    # launches per chain dispatch in the (pipelined) FETCH pass: the bench line it printed
    batch = 1
    try:
        cfg = json.load(open(os.path.join(root, "fetch.json"))).get("config", {})
        batch = max(1, int(cfg.get("hash_batch") or 1)) if cfg.get("pipelined") else 1
    except (OSError, ValueError):
        pass
    res["fetch_pass_hash_batch"] = batch
    meta.update(meta2)
    meta.update(meta3)

    # launches of each pass = its consensus dispatches (one FAST or general kernel per launch); a chain dispatch
    # carries however many launches its batch held in that pass (a short pass flushes partial batches), so the
    # per-launch figures are each kernel's sum over the pass divided by the pass's launches
    def launches(acc):
        c = acc.get("bft_consensus_fast_kernel") or acc.get("bft_consensus_kernel") or {}
        return max((len(v) for v in c.values()), default=0) or None
    nl_fetch, nl_write, nl_sq = launches(fetch), launches(write), launches(sq)
    res["launches_per_pass"] = {"fetch": nl_fetch, "write": nl_write, "sq": nl_sq}
    st_launches = (st.get("bft_consensus_fast_kernel") or st.get("bft_consensus_kernel") or {}).get("calls")
    for k in set(st) | set(fetch) | set(write) | set(sq) | set(attr):
        e = dict(meta.get(k, {}))
        if k in st:
            e.update(avg_ms=st[k]["avg_ns"] / 1e6, calls=st[k]["calls"])
            if st_launches:                              # device time per launch (the stats pass's own launches)
                e["ms_per_launch"] = st[k]["avg_ns"] * st[k]["calls"] / st_launches / 1e6
        f = fetch.get(k, {}).get("FETCH_SIZE")
        w = write.get(k, {}).get("WRITE_SIZE")
        if f:
            e["fetch_bytes_raw"] = 1024.0 * sum(f) / len(f)
            e["fetch_bytes"] = 2.0 * e["fetch_bytes_raw"]      # gfx950 FETCH_SIZE correction
            if nl_fetch:
                e["fetch_bytes_per_launch"] = 2.0 * 1024.0 * sum(f) / nl_fetch
        if w:
            e["write_bytes"] = 1024.0 * sum(w) / len(w)
            if nl_write:
                e["write_bytes_per_launch"] = 1024.0 * sum(w) / nl_write
        if f and w:
            e["hbm_bytes_per_dispatch"] = e["fetch_bytes"] + e["write_bytes"]
            if nl_fetch and nl_write:
                e["hbm_bytes_per_launch"] = e["fetch_bytes_per_launch"] + e["write_bytes_per_launch"]
        if k in attr:
            # writes measured with an L2 eviction after every kernel of unpipelined launches (one dispatch of each
            # kernel per launch): the kernel's own write-backs, none borrowed from or lent to kernels running
            # beside it; with the FETCH pass's bytes per launch (a chain dispatch of that pass carries `batch`
            # launches) this is the kernel's HBM traffic per launch
            e["write_attribution"] = attr[k]
            if f and nl_fetch:
                e["hbm_bytes_per_launch_attributed"] = e["fetch_bytes_per_launch"] + attr[k]["write_bytes_attributed"]
        for c, v in sq.get(k, {}).items():
            e[c] = sum(v) / len(v)
            if nl_sq:
                e[c + "_per_launch"] = sum(v) / nl_sq
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
