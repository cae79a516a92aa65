"""Multi-GPU plumbing: instances are independent, so ranks shard them with no data-path
collective; only the per-run statistics are all-reduced (RCCL over xGMI with the `nccl`
backend, gloo on CPU). SURVEY.md §8(e)."""
from __future__ import annotations

from typing import Dict, Tuple

STAT_KEYS = ("instances", "committed_heights", "views", "ticks")


def weak_shard(rank: int, per_rank: int) -> Tuple[int, int]:
    """Weak scaling: rank r simulates instance ids [r*I, (r+1)*I)."""
    return rank * per_rank, per_rank


def strong_shard(rank: int, world: int, total: int) -> Tuple[int, int]:
    """Strong scaling: a fixed total split into contiguous near-equal ranges."""
    base, rem = divmod(total, world)
    first = rank * base + min(rank, rem)
    return first, base + (1 if rank < rem else 0)


N_FLAGS = 7


def stats_vector(st: Dict) -> list:
    return ([st[k] for k in STAT_KEYS] + list(st["flagged"]) + list(st["round_hist"]) +
            list(st.get("latency_hist", [0] * 65)))


def all_reduce_stats(st: Dict, device=None) -> Dict:
    """Sum a bftsim_stats dict (totals + the rounds-to-commit and commit-latency histograms) over
    all ranks of the default process group: one int64 all-reduce of 145 words."""
    import torch
    import torch.distributed as dist
    v = torch.tensor(stats_vector(st), dtype=torch.int64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(v)
    v = [int(x) for x in v.tolist()]
    out = dict(zip(STAT_KEYS, v[:4]))
    f0 = 4 + N_FLAGS
    out["flagged"] = v[4:f0]
    out["round_hist"] = v[f0:f0 + 65]
    out["latency_hist"] = v[f0 + 65:f0 + 130]
    return out


def _agree(ok: bool, multi: bool) -> bool:
    """MIN over the ranks of the default group (every rank calls it, whatever it holds)."""
    if not multi:
        return ok
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else None
    flag = torch.tensor([1 if ok else 0], dtype=torch.int64, device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return bool(flag.item())


def capi_comm_init(sim, rank: int, world: int) -> bool:
    """Join `sim` to the node's RCCL communicator of libbftsim (bftsim_comm_init): rank 0 makes the id,
    the default torch.distributed group carries it to the other ranks (any channel would do).

    Collective and all-or-nothing: every rank returns the same answer, True only if every rank joined.
    ncclCommInitRank blocks until all ranks have joined, so no rank may enter it unless every rank will:
      1. pre-flight: each rank checks that librccl opens (bftsim_comm_available); one MIN all-reduce;
      2. rank 0 makes the id and broadcasts it, or a failure marker that every rank sees;
      3. only then does every rank call comm_init; one more MIN all-reduce agrees on the result.
    A rank that cannot open the library therefore fails in step 1, before anyone blocks in step 3. What
    the pre-flight cannot see (ncclCommInitRank itself failing on one rank after the others entered it)
    is RCCL's own bootstrap error path. On any failure all ranks take the torch.distributed fallback of
    all_reduce_stats."""
    import torch.distributed as dist
    multi = world > 1 and dist.is_available() and dist.is_initialized()
    why = ""
    try:
        sim.comm_available()
        ok = True
    except Exception as e:                         # noqa: BLE001 — reported by the caller
        ok, why = False, str(e)
    if not _agree(ok, multi):
        sim.comm_error = why or "another rank cannot open librccl (bftsim_comm_available)"
        return False
    uid = None
    if rank == 0:
        try:
            uid = sim.comm_unique_id()
        except Exception as e:                     # noqa: BLE001
            why = str(e)
    box = [uid]
    if multi:
        dist.broadcast_object_list(box, src=0)
    if box[0] is None:                             # every rank sees the marker: nobody joins
        sim.comm_error = why or "rank 0 could not make the RCCL id"
        return False
    ok = True
    try:
        sim.comm_init(world, rank, box[0])
    except Exception as e:                         # noqa: BLE001
        ok, why = False, str(e)
    ok = _agree(ok, multi)
    sim.comm_error = why
    return ok


def stats_from_result(r) -> Dict:
    """The bftsim_stats of a result dict (host arrays), as bft_stats_kernel computes it."""
    ch = r["committed_height"]
    if "round" in r:
        hist = [0] * 65
        for i in range(len(ch)):
            for x in r["round"][i][: ch[i]]:
                hist[min(int(x), 64)] += 1
    else:                              # a streamed result carries its histograms
        hist = [int(x) for x in r["round_hist"]]
    out = dict(instances=len(ch), committed_heights=int(ch.sum()), views=int(r["views"].sum()),
               ticks=int(r["ticks"].sum()),
               flagged=[int(((r["flags"] >> b) & 1).sum()) for b in range(N_FLAGS)], round_hist=hist)
    if "latency_hist" in r:            # commit ticks are not per-height rows: taken from the producer
        out["latency_hist"] = [int(x) for x in r["latency_hist"]]
    return out
