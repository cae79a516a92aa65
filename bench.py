#!/usr/bin/env python3
"""bench.py — BFT instance-rounds/s of the batched PBFT core on MI355X (BASELINE.json metric).

One step = one full run of the metric workload on every rank: cfg3 =
16,384 independent consensus-rs clusters of N=64 validators with f=21 equivocating Byzantine
validators, 100 heights, seeded synthetic schedule — the consensus kernel plus the block-hash
kernel, inputs resident on the GPU, results left in HBM. Ranks shard instances (rank r runs ids
[r*I, (r+1)*I)), no data-path collective; the per-run statistics are all-reduced over RCCL.

Prints ONE JSON line (rank 0). See DESIGN.md §Measurement for the roofline model.

`--workload cfg5` measures SURVEY §8d cfg5 instead (not the headline): N=7, 5 % drops, 10,000 heights,
131,072 instances per GPU (1,048,576 on 8 GPUs), windowed rows (bftsim_set_window) with in-kernel
hashes; the rounds-to-commit and commit-latency histograms are all-reduced over RCCL and printed.
One step takes ~11 s on one MI355X: run it with --steps 1 --warmup 0.

`--workload cfg2` / `cfg4` / `drop64` measure the other consensus configurations (not the headline;
`--byz 1` / `--byz 2` turn cfg2 / cfg5 into their Byzantine variants, SPEC.md §6):
cfg2 = 65,536 instances N=4, 10 % drops (BASELINE configs[1]); cfg4 = 16,384 instances of one N of the
validator sweep with proposer crashes (`--n`, default 256: the workgroup-segment kernel); drop64 = 16,384
instances N=64 f=21 with 5 % drops (most instances hand over from the FAST kernel to the resume kernel).

`--workload sig` measures the real-crypto row (not the headline): one step =
secp256k1 public-key recovery (`GossipMessage::address`, src/protocol/mod.rs:103-116) of a batch of
262,144 signed 32-byte digests per GPU resident in HBM (libbftsig, include/bftsig.h).

`--workload wire` measures the wire-codec row: one step = encode (frames + sign
digest + message hash) and decode of 262,144 Prepare / Commit / RoundChange messages per GPU
(libbftwire, include/bftwire.h).

`--workload crypto` runs cfg3 in real-crypto mode (SPEC.md §11): one step = the
consensus launch with its broadcast log + bftsim_crypto_verify (every message and commit seal signed
with its sender's key and recovered, membership checked) for 1,024 instances x 10 heights per GPU.

`--workload msgpath` composes both rows into the reference's per-message path (sign per
broadcast, decode + recover per received message): one step = 262,144 Prepare / Commit / RoundChange
messages of 64 validators: sign digest, seal and signature (bftsig_sign), frames, then on the receiving
side decode, sign-payload re-encode, recover and address check.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "consensus-rs_amd"))

METRIC = "BFT instance-rounds/sec (whole node), N=64 f=21, 1/2/4/8 GPUs; bit-exact"
METRIC_CFG5 = "cfg5 instance-rounds/sec (whole node), N=7, 5% drop, 10,000 heights; windowed, bit-exact"
VALU_PEAK = 256 * 4 * 32 * 2.4e9        # lane-ops/s (MI355X_MICROARCH.md chip table)
HBM_PEAK = 8.0e12                       # B/s spec


def consensus_ops_per_view(n: int) -> int:
    """Algorithmic 32-bit lane-ops of one instance-round in the consensus kernel:
    4 delivery phases x N receivers x (AND + 2 popcount per 64-bit word + compare/update)."""
    return 4 * n * (3 * ((n + 63) // 64) + 8)


HEADER_HASH_OPS = 14_976                # 2 Keccak-f[1600] x 24 rounds x 156 64-bit ops x 2
# SURVEY §8d algorithmic HBM bytes per instance-round with in-kernel delivery masks: 8 B view descriptor
# + 40 B result per committed height (hash 32 + round/proposer/time 8)
ALGO_BYTES_PER_VIEW = 48


def _pmc_files(workload: str):
    """The committed PMC summaries of a workload, oldest first: profiles/<round>/pmc_summary.json for the
    headline (cfg3), profiles/<round>/<workload>/pmc_summary.json for the others (cfg4 per validator count:
    profiles/<round>/cfg4_n<N>/, so that two sweep points never share one record)."""
    import glob
    sub = "" if workload == "cfg3" else workload
    return sorted(glob.glob(os.path.join(ROOT, "profiles", "*", sub, "pmc_summary.json")))


def pmc_traffic(workload: str = "cfg3"):
    """HBM bytes per dispatch per kernel from the newest committed PMC summary of this workload
    (written by scripts/pmc_summary.py from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this
    same bench command)."""
    files = _pmc_files(workload)
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    return {k: v.get("hbm_bytes_per_dispatch") for k, v in d.get("kernels", {}).items()}, \
        os.path.relpath(files[-1], ROOT)


def step_traffic(workload: str, batch: int):
    """HBM bytes of one step (one launch) from the newest PMC summary of this workload: the launch's own kernels
    (FAST + resume, or the general consensus kernel; the seed chain; the suffix rows) plus its share of a chain
    dispatch. Writes are the attributed ones where the summary has them (an L2 eviction after every kernel of
    unpipelined launches, one chain dispatch per launch: scripts/gpu_profile.sh), else the pipelined pass's
    per-dispatch bytes with the chain dispatch divided by the launches it carries. Same unit as the line's
    `hbm.algorithmic_bytes` (per step on this rank)."""
    files = _pmc_files(workload)
    if not files:
        return None
    ks = json.load(open(files[-1])).get("kernels", {})
    names = ["bft_consensus_fast_kernel", "bft_consensus_resume_kernel"] if "bft_consensus_fast_kernel" in ks \
        else ["bft_consensus_kernel"]
    names += ["bft_clear_kernel", "bft_seed_chain_kernel", "bft_hash_suffix_kernel", "bft_spec_byz_kernel",
              "bft_spec_suffix_kernel", "bft_spec_verify_kernel", "bft_hash_chain_kernel"]
    parts, attributed = {}, True
    for k in names:
        e = ks.get(k)
        if not e:
            continue
        if "hbm_bytes_per_launch_attributed" in e:
            parts[k] = e["hbm_bytes_per_launch_attributed"]            # per launch (attribution pass)
        elif "hbm_bytes_per_launch" in e:                              # per launch (the pass's launches)
            attributed = False
            parts[k] = e["hbm_bytes_per_launch"]
        elif "hbm_bytes_per_dispatch" in e:
            attributed = False
            parts[k] = e["hbm_bytes_per_dispatch"] / (batch if k == "bft_hash_chain_kernel" else 1)
    if not parts:
        return None
    return {"bytes_per_step": sum(parts.values()), "per_kernel_bytes_per_step": parts,
            "writes": "attributed (L2 eviction after every kernel)" if attributed else "as counted (pipelined pass)",
            "source": os.path.relpath(files[-1], ROOT)}


VALU_ISSUE_PEAK = 256 * 4 * 2.4e9 / 2   # wave64 VALU instructions/s: one per 2 cycles per SIMD (SIMD-32)
SALU_ISSUE_PEAK = 256 * 2.4e9           # scalar instructions/s: one scalar unit per CU, one per cycle


def pmc_issue(workload: str = "cfg3", kernel: str = "bft_consensus_kernel"):
    """Per launch VALU / SALU wave-instructions of a kernel (the consensus kernel: its FAST body) from the
    newest PMC summary of this workload (SQ_INSTS_VALU, SQ_INSTS_SALU of scripts/gpu_profile.sh's SQ pass),
    or None."""
    files = _pmc_files(workload)
    if not files:
        return None
    k = json.load(open(files[-1])).get("kernels", {})
    e = ((k.get("bft_consensus_fast_kernel") or k.get("bft_consensus_kernel") or {}) if kernel == "bft_consensus_kernel"
         else k.get(kernel) or {})
    if "SQ_INSTS_VALU" not in e:
        return None
    # per launch where the summary has it (a chain dispatch carries several launches), else per dispatch
    return {"valu": e.get("SQ_INSTS_VALU_per_launch", e["SQ_INSTS_VALU"]),
            "salu": e.get("SQ_INSTS_SALU_per_launch", e.get("SQ_INSTS_SALU"))}


def pmc_issue_step(workload: str = "cfg3"):
    """VALU / SALU wave-instructions per launch of every kernel of the step (the summary's kernels, each counted
    once: the composite consensus entry is left out), or None."""
    files = _pmc_files(workload)
    if not files:
        return None
    k = json.load(open(files[-1])).get("kernels", {})
    es = [e for e in k.values() if "SQ_INSTS_VALU" in e and "composed_of" not in e]
    if not es:
        return None
    return {"valu": sum(e.get("SQ_INSTS_VALU_per_launch", e["SQ_INSTS_VALU"]) for e in es),
            "salu": sum(e.get("SQ_INSTS_SALU_per_launch", e.get("SQ_INSTS_SALU") or 0) for e in es)}


def cfg_desc(cfg) -> str:
    d = [f"N={cfg.n}"]
    if cfg.byz_count:
        d.append(f"f={cfg.byz_count} equivocating")
    if cfg.drop_ppm:
        d.append(f"{cfg.drop_ppm / 1e4:g}% drop")
    if cfg.proposer_crash_ppm:
        d.append(f"proposer crash p={cfg.proposer_crash_ppm / 1e6:g}")
    return ", ".join(d)


def usable_cpus() -> int:
    """CPUs this process may use: the affinity mask, capped by the cgroup CPU quota (a container
    limited to 16 CPUs of a 256-CPU host runs 256 threads slower than 16)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return n


def native_oracle():
    """SURVEY §8d builds the CPU comparator -O3 -march=native for the host it runs on; the shipped
    oracle/_build/liboracle.so comes from the build container (-O3 -mpopcnt, another CPU). Builds
    `make -C oracle native` once into oracle/_build_native (git- and gpurun-ignored; rebuilt when the host CPU
    differs from the one recorded beside it) and points the oracle loader at it, unless a library is loaded
    already. Returns the build flags of the library the oracle actually runs."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    d = os.path.join(ROOT, "oracle", "_build_native")
    lib, stamp = os.path.join(d, "liboracle.so"), os.path.join(d, "host_cpu.txt")
    cpu = host_cpu()
    try:
        built_for = open(stamp).read() if os.path.exists(lib) and os.path.exists(stamp) else None
        if built_for != cpu:
            subprocess.run(["make", "-s", "-B", "-C", os.path.join(ROOT, "oracle"), "native", f"NATIVE={d}"], check=True,
                           stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=120)
            open(stamp, "w").write(cpu)
        if O._lib is None:
            O.LIB_PATH = lib
    except (OSError, subprocess.SubprocessError):
        pass
    O.lib()                                   # loads LIB_PATH now: the flags below are those of the running library
    return "-O3 -march=native (built on this host)" if os.path.abspath(O.LIB_PATH) == os.path.abspath(lib) \
        else "-O3 -mpopcnt (shipped build)"


def cpu_baseline(cfg, sample: int, threads: int, name: str = "cfg3"):
    """The C oracle (oracle/, a scalar restatement of the reference handlers) timed on this
    host's cores over a bounded sample of the same workload: every usable core (`value`),
    beside a 16-thread and a single-thread rate."""
    build = native_oracle()
    import oracle_lib as O

    def timed(n_inst, nthr):
        if name == "cfg5":
            t = time.perf_counter()
            r = O.run_stream(cfg, 0, n_inst, threads=nthr)
            secs = time.perf_counter() - t
        else:
            t = time.perf_counter()
            r = O.run(cfg, 0, n_inst, threads=nthr)
            secs = r["seconds"] if nthr > 1 else time.perf_counter() - t
        return int(r["views"].sum()), secs

    views, secs = timed(sample, threads)
    out = dict(value=views / secs, unit="instance-rounds/s", cores=threads, kind="port",
               sample=f"{sample} {name} instances ({views} instance-rounds) on {threads} threads, "
                      f"{secs:.1f} s", host=host_cpu(), build=build)
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else threads
    if aff > threads:                         # the affinity mask, oversubscribing the quota
        va, sa = timed(sample, aff)
        out["affinity_threads"] = dict(value=va / sa, threads=aff,
                                       sample=f"{sample} instances on {aff} threads, {sa:.1f} s")
    if name != "cfg5":                        # also the single-thread rate
        s1 = max(1, sample // 64)
        v1, t1 = timed(s1, 1)
        out["single_thread"] = dict(value=v1 / t1, sample=f"{s1} instances on 1 thread, {t1:.2f} s")
    return out


def host_cpu() -> str:
    """lscpu model name and the CPU count this process may use (SURVEY §8d asks for both)."""
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return f"{model} ({usable_cpus()} usable CPUs)"


def _free_port() -> int:
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def spawn_ranks(n: int) -> int:
    """`--gpus N` without an external launcher (no WORLD_SIZE in the environment): start N rank processes of
    this same command, one per GPU, the way torch.distributed.run would (RANK, LOCAL_RANK, WORLD_SIZE,
    LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT), and wait for them. This process never imports
    torch or touches HIP: the ranks are fresh children, not an exec of a process that initialised the GPU.
    Rank 0 writes the one JSON line on this process's stdout; the other ranks' stdout goes to stderr. If any
    rank fails, the others are stopped (they may be blocked in a collective with it) and its exit code is
    returned. The reference's counterpart is its multi-process cluster launch (build.sh:7-13)."""
    import signal
    port = _free_port()
    cmd = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), BFTSIM_BENCH_SPAWNED="1")
        procs.append(subprocess.Popen(cmd, env=env, stdout=None if r == 0 else sys.stderr.fileno()))
    if os.environ.get("BFTSIM_TESTING") == "1" and os.environ.get("BFTSIM_BENCH_STUB_DIR"):
        with open(os.path.join(os.environ["BFTSIM_BENCH_STUB_DIR"], "parent.json"), "w") as f:
            json.dump({"pids": [p.pid for p in procs], "gpu_modules": sorted(
                m for m in sys.modules if m == "torch" or m.startswith("torch.") or m.startswith("bftsim"))}, f)
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in live:                       # peers may wait forever in a collective with it
                    q.send_signal(signal.SIGTERM)
        if live:
            time.sleep(0.05)
    return rc


def stub_rank(args) -> None:
    """BFTSIM_TESTING stub of a rank (tests/test_bench_launcher.py): records its environment, prints the
    JSON line shape of rank 0 with n_gpus from WORLD_SIZE; touches no GPU."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
    with open(os.path.join(os.environ["BFTSIM_BENCH_STUB_DIR"], f"rank{rank}.json"), "w") as f:
        json.dump({k: os.environ.get(k) for k in keys} | {"pid": os.getpid(), "ppid": os.getppid()}, f)
    if os.environ.get("BFTSIM_BENCH_STUB_FAIL") == str(rank):
        sys.exit(3)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": 0.0, "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "data": "stub"}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default: 20 for cfg3, the driver's setting; 10 for the other workloads)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps first (default: 5 for cfg3, else 2)")
    ap.add_argument("--workload", choices=("cfg3", "cfg2", "cfg4", "drop64", "cfg5", "sig", "wire", "msgpath",
                                           "crypto"),
                    default="cfg3")
    ap.add_argument("--n", type=int, default=256, help="cfg4: validators per instance")
    ap.add_argument("--instances", type=int, default=None, help="instances per GPU")
    ap.add_argument("--heights", type=int, default=None)
    ap.add_argument("--window", type=int, default=None, help="cfg5: canonical rows kept per instance (default "
                    "bftsim.configs.CFG5_WINDOW)")
    ap.add_argument("--cpu-sample", type=int, default=None)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="run each step's block-hash pass on the launch stream (no overlap across steps)")
    ap.add_argument("--pipeline-depth", type=int, default=None,
                    help="launches in flight (bftsim_set_pipeline: a ring of row-table sets, each launch on its set's "
                         "stream). Default: 6 at >= 12,288 instances per GPU, 16 below (profiles/r04/ab_deep_ring)")
    ap.add_argument("--hash-batch", type=int, default=None,
                    help="launches whose block-hash chains run as one kernel (bftsim_set_hash_batch, 1..32). Default: 2 "
                         "at >= 12,288 instances per GPU, 8 below (profiles/r04/ab_deep_ring)")
    ap.add_argument("--hw-queues", type=int, default=8,
                    help="GPU_MAX_HW_QUEUES for this process (HIP's default is 4): every set's stream needs its own "
                         "hardware queue, or launches serialize behind each other (profiles/r04/ab_depth_queues); "
                         "0 leaves the environment as it is")
    ap.add_argument("--byz", type=int, default=None,
                    help="cfg2 / cfg5: run the tolerated f as this many equivocating validators (SPEC.md §6: "
                         "cfg2-byz = 1, cfg5-byz = 2)")
    ap.add_argument("--seed-order", choices=("be", "le"), default="be",
                    help="U128 byte order of randon_seed (validator.rs:39-48; include/bftsim.h BFTSIM_SEED_*)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default=None,
                    help="weak: --instances per GPU; strong: --instances in total, split over the ranks. Default: "
                         "strong for cfg3 (BASELINE configs[2]: 16,384 sharded over 1/2/4/8 GPUs; at N > 1 the "
                         "weak number, 16,384 per GPU, is measured too and reported in config.weak), weak for the "
                         "other workloads")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))           # before anything touches the GPU (or imports bftsim)
    from bftsim.configs import bench_steps, bench_instances, bench_config
    if args.window is None:
        from bftsim.configs import CFG5_WINDOW
        args.window = CFG5_WINDOW
    if args.steps is None:
        args.steps = bench_steps(args.workload)[0]
    if args.warmup is None:
        args.warmup = bench_steps(args.workload)[1]
    if os.environ.get("BFTSIM_TESTING") == "1" and os.environ.get("BFTSIM_BENCH_STUB_DIR"):
        return stub_rank(args)
    if args.hw_queues > 0:                         # read by the HIP runtime at its initialisation (below)
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']} from the launcher; "
              "using WORLD_SIZE", file=sys.stderr)
    if args.workload == "sig":
        return main_sig(args)
    if args.workload == "wire":
        return main_wire(args)
    if args.workload == "msgpath":
        return main_msgpath(args)
    if args.workload == "crypto":
        return main_crypto(args)

    import torch
    import torch.distributed as dist
    from bftsim.configs import BftConfig, cfg2, cfg3, cfg4, cfg5
    from bftsim.distributed import all_reduce_stats
    from bftsim.runtime import Simulator
    c5 = args.workload == "cfg5"
    wl = args.workload
    if args.instances is None:
        args.instances = bench_instances(wl)
    if args.heights is None:
        args.heights = 10_000 if c5 else 100
    if args.cpu_sample is None:
        args.cpu_sample = {"cfg5": 4096, "cfg2": 16_384, "cfg4": 1024 if args.n > 64 else 8192}.get(wl, 16_384)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    cfg = bench_config(wl, n=args.n, heights=args.heights, byz=args.byz or 0)
    if args.seed_order == "le":
        import dataclasses
        cfg = dataclasses.replace(cfg, seed_byte_order=1, name=cfg.name + "-le")
    sim = Simulator(cfg, device=local)
    pipelined = not c5 and not args.no_pipeline
    if args.scaling is None:
        args.scaling = "strong" if wl == "cfg3" else "weak"
    if args.scaling == "strong":
        from bftsim.distributed import strong_shard
        first, I = strong_shard(rank, world, args.instances)
    else:
        I = args.instances
        first = rank * I
    from bftsim.configs import timed_pipeline
    auto_depth = args.pipeline_depth is None
    if auto_depth:
        args.pipeline_depth = timed_pipeline(I)[0]
    if args.hash_batch is None:
        args.hash_batch = timed_pipeline(I)[1]
    sim.set_pipeline(pipelined, args.pipeline_depth)
    sim.set_hash_batch(args.hash_batch)
    if c5:
        sim.set_window(args.window)
    sim.prepare(I)
    stream = torch.cuda.current_stream(dev).cuda_stream

    enqueue_s = []

    def timed_steps(first_id):
        """K launches between two barriers + device synchronisations; the max over ranks (s)"""
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            sim.launch(first_id, stream)
        enqueue_s.append(time.perf_counter() - t0)   # host time of the K launch calls (diagnostic)
        sim.sync()                        # enqueues the last partial hash batch and waits for every stream
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        tmax = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        return float(tmax.item())

    for _ in range(args.warmup):
        sim.launch(first, stream)
    sim.sync()
    torch.cuda.synchronize(dev)

    # work per step: instance-rounds of this shard (identical every step), summed over ranks
    if args.warmup == 0:                  # the work of a step is read from one run's statistics
        sim.launch(first, stream)
        sim.sync()
        torch.cuda.synchronize(dev)
    st = sim.stats()
    # node-wide statistics: one RCCL all-reduce inside libbftsim (bftsim_stats_allreduce, over xGMI);
    # torch.distributed's all-reduce of the same counts only if librccl cannot be opened
    # (the decision is collective: every rank takes the same branch, capi_comm_init)
    from bftsim.distributed import capi_comm_init
    if capi_comm_init(sim, rank, world):
        tot = sim.stats_allreduce()
        reduce_via = "libbftsim bftsim_stats_allreduce (RCCL)"
    else:
        tot = all_reduce_stats(st, device=dev)
        reduce_via = f"torch.distributed (libbftsim's RCCL communicator unavailable: {getattr(sim, 'comm_error', '')})"
    views_all, heights_all = tot["views"], tot["committed_heights"]
    safety_all, timeout_all = tot["flagged"][0], tot["flagged"][4]

    torch.cuda.synchronize(dev)
    sim.kernel_ms_sum()                   # drop the warmup launches
    dt = timed_steps(first)

    ms_step = 1000.0 * dt / args.steps
    value = views_all * args.steps / dt
    cms_sum, hms_sum, nl = sim.kernel_ms_sum()    # HIP events around every launch of the timed region
    cms = cms_sum / max(nl, 1)
    hms = hms_sum / max(nl, 1)

    # the weak counterpart of a multi-GPU strong headline: --instances per GPU on every rank, same K / W
    weak = None
    if args.scaling == "strong" and world > 1:
        Iw, first_w = args.instances, rank * args.instances
        if auto_depth:
            sim.set_pipeline(pipelined, timed_pipeline(Iw)[0])
            sim.set_hash_batch(timed_pipeline(Iw)[1])
        sim.prepare(Iw)
        for _ in range(max(args.warmup, 1)):
            sim.launch(first_w, stream)
        sim.sync()
        torch.cuda.synchronize(dev)
        vw = torch.tensor([sim.stats()["views"]], dtype=torch.int64, device=dev)
        dist.all_reduce(vw)
        dtw = timed_steps(first_w)
        weak = {"value": int(vw.item()) * args.steps / dtw, "instances_per_gpu": Iw,
                "instances_total": Iw * world, "ms_per_step": 1000.0 * dtw / args.steps,
                "instance_rounds_per_step": int(vw.item()), "scaling": "weak"}
        sim.kernel_ms_sum()

    if rank == 0:
        views_rank = st["views"]
        # dominant kernel by device time
        c_ops = consensus_ops_per_view(cfg.n) * views_rank
        h_ops = HEADER_HASH_OPS * st["committed_heights"]
        if c5 or cfg.seed_byte_order or (cfg.n & (cfg.n - 1)):   # block hashes inside the consensus kernel
            c_ops, h_ops = c_ops + h_ops, 0
        # the dominant kernel is the one with the larger device time per launch: the consensus kernel (FAST +
        # resume, HIP events c0..c1 per launch) or the prev_hash chains (events around each chain dispatch;
        # pipelined, one dispatch hashes `hash_batch` launches and its time is shared among them). Launches
        # overlap when pipelined, so these are stretched durations, as rocprof reports them.
        batch = args.hash_batch if (pipelined and h_ops) else 1
        # Everything is priced per LAUNCH (one step): a chain dispatch's time is shared among the launches it
        # carries (bftsim_kernel_ms_sum), as rocprof's total chain time over the launches of a pass is
        # (pmc_summary.json ms_per_launch)
        if cms >= hms:
            dom, ops, ms = "bft_consensus_kernel", c_ops, cms
        else:
            dom, ops, ms = "bft_hash_chain_kernel", h_ops, hms
        achieved = ops / (ms / 1e3) / 1e12
        peak = VALU_PEAK / 1e12
        # the PMC summary of this exact line: cfg4 per validator count, cfg3 per shard size and seed byte order
        pmc_key = f"cfg4_n{cfg.n}" if wl == "cfg4" else wl
        if wl == "cfg3" and cfg.seed_byte_order:
            pmc_key = "cfg3le"
        elif wl == "cfg3" and I != 16_384:
            pmc_key = f"cfg3_{I}"
        traffic, traffic_src = pmc_traffic(pmc_key)
        algo_bytes = ALGO_BYTES_PER_VIEW * views_rank
        stp = step_traffic(pmc_key, args.hash_batch if pipelined else 1)
        def trim(h):
            h = list(h)
            while h and h[-1] == 0:
                h.pop()
            return h
        out = {
            "metric": METRIC if wl == "cfg3" else METRIC_CFG5 if c5 and not cfg.byz_count else (
                f"{wl} instance-rounds/sec (whole node), {cfg_desc(cfg)}; bit-exact"),
            "value": value,
            "unit": "instance-rounds/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (seeded Philox schedule, SPEC.md)",
            "config": {
                "workload": (f"{cfg.name}: {I} instances per GPU, {cfg_desc(cfg)}, {args.heights} heights, "
                             f"window {args.window}") if c5 else
                            ((f"{wl}: {args.instances} instances sharded over {world} GPU(s) ({I} on rank 0)"
                              if args.scaling == "strong" else f"{wl}: {I} instances per GPU") +
                             f", {cfg_desc(cfg)}, {args.heights} heights" +
                             (", little-endian U128 seeds" if cfg.seed_byte_order else "")),
                "instances_per_gpu": I, "n_validators": cfg.n, "byzantine": cfg.byz_count,
                "instances_total": args.instances if args.scaling == "strong" else args.instances * world,
                "weak": weak,
                "seed_byte_order": "le" if cfg.seed_byte_order else "be",
                "heights": args.heights, "parallelism": f"instance-sharded x{world}",
                "pipelined": pipelined, "pipeline_depth": args.pipeline_depth if pipelined else 0,
                "hash_batch": args.hash_batch if pipelined else 0,
                "host_enqueue_ms": round(1e3 * enqueue_s[0], 3),
                "instance_rounds_per_step": views_all,
                "stats_allreduce": reduce_via,
                "committed_heights_per_step": heights_all,
                "safety_violations": safety_all, "timeouts": timeout_all,
                "rounds_to_commit_hist": trim(tot["round_hist"]),
                "commit_latency_ticks_hist": trim(tot["latency_hist"]),
            },
            "roofline": {
                "bound": "valu", "kernel": dom, "achieved": achieved, "peak": peak,
                "unit": "Tops/s", "frac": achieved / peak,
                # HBM bytes per step (PMC, all kernels of one launch), in the unit of hbm.algorithmic_bytes
                "traffic": stp["bytes_per_step"] if stp else None,
                "traffic_unit": "HBM bytes per step (one launch of this rank)",
                "traffic_step": stp,
                "traffic_dominant_per_dispatch": (traffic or {}).get(dom),
                # what the hardware issues, beside the algorithmic model: VALU wave-instructions of
                # the profiled launch (PMC) per second of this run's kernel time vs the issue peak
                "issue": (lambda q: None if q is None else {
                    "valu_wave_instr_per_launch": q["valu"], "salu_wave_instr_per_launch": q["salu"],
                    "valu_per_s": q["valu"] / (ms / 1e3), "valu_peak_per_s": VALU_ISSUE_PEAK,
                    "valu_frac": q["valu"] / (ms / 1e3) / VALU_ISSUE_PEAK,
                    "salu_per_s": q["salu"] / (ms / 1e3), "salu_peak_per_s": SALU_ISSUE_PEAK,
                    "salu_frac": q["salu"] / (ms / 1e3) / SALU_ISSUE_PEAK,
                    "per_instance_round": {"valu": q["valu"] / max(views_rank, 1),
                                           "salu": q["salu"] / max(views_rank, 1)}})(pmc_issue(pmc_key, dom)),
                # the whole step: every kernel's VALU per launch over the step time (the chain kernels run under the
                # consensus kernels at a lower priority, so their own event time is stretched)
                "issue_step": (lambda q: None if q is None else {
                    "valu_wave_instr_per_launch": q["valu"], "salu_wave_instr_per_launch": q["salu"],
                    "valu_per_s": q["valu"] / (ms_step / 1e3), "valu_frac": q["valu"] / (ms_step / 1e3) / VALU_ISSUE_PEAK,
                    "salu_frac": q["salu"] / (ms_step / 1e3) / SALU_ISSUE_PEAK})(pmc_issue_step(pmc_key)),
                "per": "launch (one step; a chain dispatch's time and counters shared among the launches it carries)",
                "dispatch": {"launches_per_dispatch": batch, "ops_per_dispatch": ops * batch, "ms_per_dispatch": ms * batch},
                "traffic_source": traffic_src,
                "hbm": {"algorithmic_bytes": algo_bytes, "unit": "bytes per step",
                        "achieved_GBps": algo_bytes / (ms_step / 1e3) / 1e9,
                        "peak_GBps": HBM_PEAK / 1e9, "frac": algo_bytes / (ms_step / 1e3) / HBM_PEAK,
                        "traffic_bytes": stp["bytes_per_step"] if stp else None,
                        "traffic_over_algorithmic": stp["bytes_per_step"] / algo_bytes if stp and algo_bytes else None,
                        "traffic_GBps": stp["bytes_per_step"] / (ms_step / 1e3) / 1e9 if stp else None},
                "kernel_ms": {"bft_consensus_kernel": cms, "bft_hash_kernel": hms},   # per launch
                # both kernels' fractions, whichever is dominant, and the whole step against the full
                # per-instance-round model (consensus + one header hash per committed height). The hash
                # pass's own time is exclusive only with --no-pipeline (pipelined, it runs beside the
                # next launches' consensus kernels and its event time is stretched wall time)
                "per_kernel": {
                    "bft_consensus_kernel": {"ops": c_ops, "ms": cms,
                                             "frac": c_ops / (cms / 1e3) / VALU_PEAK if cms > 0 else None},
                    "bft_hash_kernel": {"ops": h_ops, "ms": hms, "exclusive": not pipelined,
                                        "frac": h_ops / (hms / 1e3) / VALU_PEAK if hms > 0 and h_ops else None},
                },
                "step": {"ops": c_ops + h_ops, "ms": ms_step,
                         "frac": (c_ops + h_ops) / (ms_step / 1e3) / VALU_PEAK},
                "ops_model": "consensus 4*N*(3*ceil(N/64)+8) lane-ops per instance-round; "
                             "hash 14976 lane-ops per header (SURVEY.md 8d)",
            },
        }
        if not args.no_cpu and world == 1:    # the CPU leg: rank 0 at N = 1 only
            try:
                out["cpu_baseline"] = cpu_baseline(cfg, args.cpu_sample, usable_cpus(), args.workload)
            except Exception as e:  # the baseline is reported, never the target
                out["cpu_baseline"] = {"error": str(e)}
        print(json.dumps(out), flush=True)
    sim.close()
    if world > 1:
        dist.destroy_process_group()


METRIC_SIG = "secp256k1 public-key recoveries/sec (whole node), GossipMessage::address; bit-exact"
# 32x32->64 multiply-adds of one recovery, counted on the host build of the same source
# (tests/sig_lib.counts(): 1224 fe_mul x 73 + 1584.8 fe_sqr x 45 + 69 sc_mul x 134 + 253 sc_sqr x 106;
# GLV split: 128 doublings)
SIG_RECOVER_MADS = 196_732
MAD_PEAK = 256 * 32 * 2.4e9             # v_mad_u64_u32 per s: quarter rate (build/mad_peak measured 1.963e13)


def sig_cpu_baseline(digs, sigs, sample: int, threads: int):
    """The C oracle (oracle/secp_oracle.c: 64-bit limbs, double-and-add) on this host's cores."""
    build = native_oracle()
    import oracle_lib as O
    t = time.perf_counter()
    _, ok = O.secp_recover_batch(digs[:sample], sigs[:sample], threads)
    secs = time.perf_counter() - t
    assert ok.all()
    return dict(value=sample / secs, unit="recoveries/s", cores=threads, kind="port",
                sample=f"{sample} recoveries of the same batch by the C oracle on {threads} threads, {secs:.1f} s",
                build=build)


METRIC_CRYPTO = "real-crypto cfg3 instance-rounds/sec (whole node), N=64 f=21; every broadcast signed and recovered"


def main_crypto(args):
    """cfg3 with real signatures (SPEC.md §11): launch (consensus + broadcast log) + the batched sign /
    recover pass, per step; the CPU leg times the C secp256k1 oracle's recoveries and prices the
    reference's per-receiver recoveries with them."""
    import torch
    import torch.distributed as dist
    from bftsim.configs import cfg3
    from bftsim.crypto import synthetic_secrets, keyed_config, gpu_addresses
    from bftsim.runtime import Simulator
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    I = args.instances or 1024
    heights = args.heights or 10
    sec = synthetic_secrets(64, 3)
    cfg, secrets = keyed_config(cfg3(heights=heights), sec, gpu_addresses(sec, local))
    sim = Simulator(cfg, device=local)
    sim.set_crypto(secrets, (), 24_576)
    sim.prepare(I)
    first = rank * I
    for _ in range(max(1, args.warmup)):
        sim.launch(first)
        rep = sim.crypto_verify()
    assert rep["mismatches"] == 0 and rep["seal_errors"] == 0, rep
    views = sim.stats()["views"]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    sim.kernel_ms_sum()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sim.launch(first)
        rep = sim.crypto_verify()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    tmax = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    dt = float(tmax.item())
    cms, hms, nl = sim.kernel_ms_sum()
    sim.close()
    if rank == 0:
        msgs, seals = rep["messages"], rep["seals"]
        out = {
            "metric": METRIC_CRYPTO, "value": views * world * args.steps / dt, "unit": "instance-rounds/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1000.0 * dt / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (seeded schedule, keccak-derived secp256k1 keys)",
            "config": {"workload": f"crypto: {I} cfg3 instances per GPU, {heights} heights, real signatures",
                       "instances_per_gpu": I, "heights": heights, "n_validators": 64, "byzantine": 21,
                       "instance_rounds_per_step": views, "messages_per_step": msgs, "seals_per_step": seals,
                       "signatures_per_s": (msgs + seals) * world * args.steps / dt,
                       "recoveries_per_s": (msgs + seals) * world * args.steps / dt,
                       "consensus_kernel_ms_per_step": cms / max(nl, 1), "hash_kernel_ms_per_step": hms / max(nl, 1),
                       "mismatches": rep["mismatches"], "parallelism": f"instance-sharded x{world}"},
            "roofline": None,
        }
        if not args.no_cpu:
            try:
                # the reference recovers each message at each of its N receivers (core.rs:314-322) and each
                # seal at each receiver (commit.rs:94-100); priced at the C oracle's measured recovery rate
                build = native_oracle()
                import oracle_lib as O
                from bftsim.sig import Signer
                sg = Signer(local)
                m = 4096
                g = torch.Generator().manual_seed(7)
                digs = torch.randint(0, 256, (m, 32), dtype=torch.uint8, generator=g).to(dev)
                kk = torch.frombuffer(bytearray(b"".join(secrets)), dtype=torch.uint8).reshape(64, 32).to(dev)
                kidx = (torch.arange(m, dtype=torch.int32) % 64).to(dev)
                sigs, _ = sg.sign(kk, digs, key_index=kidx)
                sg.close()
                thr = min(16, usable_cpus())
                t = time.perf_counter()
                _, ok = O.secp_recover_batch(digs.cpu().numpy(), sigs.cpu().numpy(), thr)
                secs = time.perf_counter() - t
                rate = m / secs
                per_view = (msgs + seals) * 64 / views
                out["cpu_baseline"] = dict(
                    value=rate / per_view, unit="instance-rounds/s", cores=thr, kind="port",
                    sample=f"{m} recoveries by the C oracle on {thr} threads in {secs:.1f} s ({rate:.0f}/s), "
                           f"x {per_view:.0f} recoveries per instance-round (each message and seal at 64 receivers)",
                    build=build)
            except Exception as e:          # noqa: BLE001
                out["cpu_baseline"] = {"error": str(e)}
        print(json.dumps(out), flush=True)


def main_sig(args):
    import torch
    import torch.distributed as dist
    from bftsim.sig import Signer
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    n = args.instances or 262_144
    keys = 64
    g = torch.Generator().manual_seed(1000 + rank)       # each rank its own shard of messages
    secs = torch.randint(0, 256, (keys, 32), dtype=torch.uint8, generator=g)
    secs[:, 0] &= 0x7f
    digs = torch.randint(0, 256, (n, 32), dtype=torch.uint8, generator=g).to(dev)
    kidx = (torch.arange(n, dtype=torch.int32) % keys).to(dev)
    sg = Signer(local)
    sigs, ok = sg.sign(secs.to(dev), digs, key_index=kidx)
    assert bool((ok == 1).all())
    _, kaddr, _ = sg.secret_to_address(secs.to(dev))
    want = kaddr[kidx.long()]
    for _ in range(args.warmup):
        sg.recover(digs, sigs, want_pub=False)
    _, addr, ok = sg.recover(digs, sigs, want_pub=False)
    assert bool((ok == 1).all()) and bool((addr == want).all()), "recovery mismatch"
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for e0, e1 in evs:
        e0.record()
        sg.recover(digs, sigs, want_pub=False)
        e1.record()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    tmax = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    dt = float(tmax.item())
    kms = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
    if rank == 0:
        achieved = SIG_RECOVER_MADS * n / (kms / 1e3) / 1e12
        out = {
            "metric": METRIC_SIG, "value": n * world * args.steps / dt, "unit": "recoveries/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1000.0 * dt / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (seeded secrets and digests; signatures made by bftsig_sign)",
            "config": {"workload": f"sig: {n} recoverable signatures per GPU (64 signers), recover + address",
                       "batch_per_gpu": n, "parallelism": f"batch-sharded x{world}"},
            "roofline": {"bound": "valu", "kernel": "sig_recover_kernel", "achieved": achieved,
                         "peak": MAD_PEAK / 1e12, "unit": "T mad_u64_u32/s", "frac": achieved / (MAD_PEAK / 1e12),
                         "traffic": None, "kernel_ms": kms,
                         "ops_model": f"{SIG_RECOVER_MADS} 32x32->64 multiply-adds per recovery (host-counted)"},
        }
        if not args.no_cpu:
            try:
                d, s_ = digs.cpu().numpy(), sigs.cpu().numpy()
                out["cpu_baseline"] = sig_cpu_baseline(d, s_, args.cpu_sample or 65536, min(16, os.cpu_count() or 1))
            except Exception as e:
                out["cpu_baseline"] = {"error": str(e)}
        print(json.dumps(out), flush=True)
    sg.close()
    if world > 1:
        dist.destroy_process_group()


METRIC_WIRE = "consensus wire messages/sec (whole node): encode + 2 Keccak digests + decode; bit-exact"


def wire_algo_bytes(frame_bytes: int, n: int, n_commit: int) -> int:
    """Algorithmic HBM bytes of one encode + decode step: the input fields read (code 1, round /
    height / create_time / ttl / raw_time 5x8, digest 32, signature 65, seal 65 for Commits), the
    frames written, the two 32-byte digests written, the frames read back and the fields written."""
    fields = n * (1 + 40 + 32 + 65) + n_commit * 65
    return 2 * fields + 2 * frame_bytes + 64 * n + 8 * (n + 1) * 2


def main_wire(args):
    import numpy as np
    import torch
    import torch.distributed as dist
    from bftsim.wire import Codec
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    n = args.instances or 262_144
    rng = np.random.default_rng(2000 + rank)
    code = rng.choice(np.array([2, 3, 4], dtype=np.uint8), n)          # Prepare / Commit / RoundChange
    batch = {"code": code, "round": rng.integers(0, 4, n), "height": rng.integers(1, 1 << 20, n),
             "digest": rng.integers(0, 256, (n, 32), dtype=np.uint8),
             "create_time": 1536517089000 + rng.integers(0, 1 << 30, n),
             "signature": rng.integers(0, 256, (n, 65), dtype=np.uint8),
             "commit_seal": rng.integers(0, 256, (n, 65), dtype=np.uint8)}
    cd = Codec(local)
    b = {k: cd._t(v, torch.uint8 if v.dtype == np.uint8 else torch.int64) for k, v in batch.items()}
    cap = n * 1028
    out, offs, sd, mh, ok = cd.encode(b, cap=cap)
    assert bool((ok == 1).all())
    total = int(offs[-1])
    fields, ok2 = cd.decode(out, offs)
    assert bool((ok2 == 1).all()) and torch.equal(fields["digest"], b["digest"])

    def step():
        o, f, _, _, _ = cd.encode(b, cap=cap)
        cd.decode(o, f)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for e0, e1 in evs:
        e0.record()
        step()
        e1.record()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    tmax = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    dt = float(tmax.item())
    kms = sum(a.elapsed_time(c) for a, c in evs) / len(evs)
    if rank == 0:
        algo = wire_algo_bytes(total, n, int((code == 3).sum()))
        achieved = algo / (kms / 1e3) / 1e9
        out_j = {
            "metric": METRIC_WIRE, "value": n * world * args.steps / dt, "unit": "messages/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1000.0 * dt / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (seeded Prepare/Commit/RoundChange fields, random 65-byte signatures and seals)",
            "config": {"workload": f"wire: {n} messages per GPU, encode (frames + sign digest + message hash) "
                                   f"+ decode", "batch_per_gpu": n, "frame_bytes": total,
                       "parallelism": f"batch-sharded x{world}"},
            "roofline": {"bound": "hbm", "kernel": "bftwire encode+decode (encode, scan, pack, hash, decode)",
                         "achieved": achieved, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                         "frac": achieved / (HBM_PEAK / 1e9), "traffic": None, "kernel_ms": kms,
                         "algorithmic_bytes_per_step": algo},
        }
        if not args.no_cpu:
            try:
                out_j["cpu_baseline"] = wire_cpu_baseline(batch, args.cpu_sample or 20000)
            except Exception as e:
                out_j["cpu_baseline"] = {"error": str(e)}
        print(json.dumps(out_j), flush=True)
    cd.close()
    if world > 1:
        dist.destroy_process_group()


def wire_cpu_baseline(batch, sample: int):
    """The msgpack oracle (oracle/wire_ref.py: encode + both Keccak digests + decode) on one core."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    import wire_ref as R
    msgs = [dict(code=int(batch["code"][i]), round=int(batch["round"][i]), height=int(batch["height"][i]),
                 digest=bytes(batch["digest"][i]), create_time=int(batch["create_time"][i]),
                 signature=bytes(batch["signature"][i]),
                 commit_seal=bytes(batch["commit_seal"][i]) if batch["code"][i] == 3 else None,
                 raw_time=int(batch["create_time"][i])) for i in range(sample)]
    t = time.perf_counter()
    for m in msgs:
        f, g, sp = R.encode(m)
        O.keccak256(g)
        O.keccak256(sp)
        R.decode(f)
    secs = time.perf_counter() - t
    return dict(value=sample / secs, unit="messages/s", cores=1, kind="port",
                sample=f"{sample} messages through the msgpack oracle on 1 core, {secs:.1f} s")


METRIC_MSGPATH = ("consensus messages/sec through the per-message path (whole node): encode + sign digest + "
                  "sign + frame | decode + re-encode + recover + address check; bit-exact")


def main_msgpath(args):
    import numpy as np
    import torch
    import torch.distributed as dist
    from bftsim.sig import Signer
    from bftsim.wire import Codec
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    n, n_val = args.instances or 262_144, 64
    rng = np.random.default_rng(3000 + rank)
    secs = torch.from_numpy(rng.integers(0, 128, (n_val, 32), dtype=np.uint8)).to(dev)
    sender = torch.arange(n, dtype=torch.int32, device=dev) % n_val
    batch = {"code": torch.from_numpy(rng.choice(np.array([2, 3, 4], dtype=np.uint8), n)).to(dev),
             "round": torch.from_numpy(rng.integers(0, 4, n)).to(dev),
             "height": torch.from_numpy(rng.integers(1, 1 << 20, n)).to(dev),
             "digest": torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).to(dev),
             "create_time": torch.from_numpy(1536517089000 + rng.integers(0, 1 << 30, n)).to(dev)}
    sg, cd = Signer(local), Codec(local)
    _, vaddr, _ = sg.secret_to_address(secs)
    want = vaddr[sender.long()]

    def step():
        seal, _ = sg.sign(secs, batch["digest"], key_index=sender)          # commit seals (votes.rs:94-101)
        b = {**batch, "commit_seal": seal}
        _, _, sd, _, _ = cd.encode(b)                                        # sign digest (+ message hash)
        sig, _ = sg.sign(secs, sd, key_index=sender)                         # set_sign
        frames, offs, _, _, _ = cd.encode({**b, "signature": sig}, hashes=False)
        dec, _ = cd.decode(frames, offs)                                     # receiver
        rx = {k: dec[k] for k in ("code", "round", "height", "digest", "create_time", "commit_seal")}
        _, _, sd_rx, _, _ = cd.encode(rx)
        _, addr, ok = sg.recover(sd_rx, dec["signature"], want_pub=False)   # GossipMessage::address
        return addr, ok
    addr, ok = step()
    assert bool((ok == 1).all()) and torch.equal(addr, want), "per-message path mismatch"
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(args.steps):
        step()
    e1.record()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    tmax = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    dt = float(tmax.item())
    gpu_ms = e0.elapsed_time(e1) / args.steps
    if rank == 0:
        mads = 2 * 69_848 + SIG_RECOVER_MADS                # two signatures + one recovery per message
        achieved = mads * n / (gpu_ms / 1e3) / 1e12
        out = {
            "metric": METRIC_MSGPATH, "value": n * world * args.steps / dt, "unit": "messages/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1000.0 * dt / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (seeded validator keys, message fields and digests)",
            "config": {"workload": f"msgpath: {n} messages per GPU from 64 validators, sender + receiver path",
                       "batch_per_gpu": n, "parallelism": f"batch-sharded x{world}"},
            "roofline": {"bound": "valu", "kernel": "sig_sign x2 + sig_recover + wire encode x3 + decode",
                         "achieved": achieved, "peak": MAD_PEAK / 1e12, "unit": "T mad_u64_u32/s",
                         "frac": achieved / (MAD_PEAK / 1e12), "traffic": None, "step_gpu_ms": gpu_ms,
                         "ops_model": f"{mads} multiply-adds per message (2 signatures + 1 recovery)"},
        }
        print(json.dumps(out), flush=True)
    sg.close()
    cd.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
