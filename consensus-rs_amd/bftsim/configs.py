"""Workload configurations (BASELINE.json `configs`, restated in SURVEY.md §8d).

A config is plain data: the validator set (sorted addresses, `ImplValidatorSet::new`,
src/consensus/validator.rs:58-70), the genesis fields (src/core/genesis.rs:44-55,
examples/c1.toml:13-18) and the seeded schedule knobs of SPEC.md §3-§6.
"""
from __future__ import annotations

import dataclasses
import hashlib
from typing import List, Optional, Sequence

GENESIS_TIME = 1536517089          # 2018-09-09T09:09:09.09-09:09 (examples/c1.toml:15)
GENESIS_PROPOSER = "0x5701fbd05e77cac003a6894e4b2a3c12287ed313"   # examples/c1.toml:16
GENESIS_GAS_USED = 10000           # examples/c1.toml:17

# examples/c1.toml:14 — the 5-validator genesis set, in file order c1..c5
C_ADDRESSES = [
    "0x7193d8f91724b39f10cc81e94934c187fa257277",
    "0x93908f59c6eff007d228398349214acb6b4ac9a4",
    "0x72d5c75fd6703414aa87f79b3e4797dd09cd9251",
    "0x58096d35c7a8ff67eba159f33cea7740fc9a737c",
    "0xc759616c865d349ec2afced268fc6f33ff7414a4",
]


def string_to_address(s: str) -> bytes:
    """common::string_to_address (src/common/mod.rs:96-108)."""
    if len(s) < 40:
        raise ValueError("less than 40 chars")
    if len(s) > 42:
        raise ValueError("more than 42 chars")
    if len(s) == 42:
        s = s[2:]
    return bytes.fromhex(s)


def sorted_addresses(addrs: Sequence[bytes]) -> List[bytes]:
    """Validators sorted ascending by address (validator.rs:68, types/mod.rs:87-91)."""
    return sorted(addrs)


def synthetic_addresses(n: int) -> List[bytes]:
    """Deterministic 20-byte addresses for synthetic validator sets (sha3-256 of a label)."""
    return sorted_addresses(
        [hashlib.sha3_256(b"bftsim-validator-%d" % i).digest()[:20] for i in range(n)])


@dataclasses.dataclass
class BftConfig:
    n: int
    heights: int = 100
    max_ticks: int = 0                   # 0 → 4 * heights + 64
    block_period: int = 3
    genesis_time: int = GENESIS_TIME
    seed: int = 1
    drop_ppm: int = 0
    byz_count: int = 0
    proposer_crash_ppm: int = 0
    phase_cap: int = 16
    silent: Sequence[int] = ()
    addresses: Optional[List[bytes]] = None
    genesis_proposer: bytes = dataclasses.field(
        default_factory=lambda: string_to_address(GENESIS_PROPOSER))
    genesis_gas_used: int = GENESIS_GAS_USED
    name: str = ""
    # conventions the reference leaves to unvendored crates (include/bftsim.h BFTSIM_SEED_*):
    # 0 = U128::from([u8;16]) big-endian (validator.rs:39-48 read as bigint's byte-slice order), 1 = LE
    seed_byte_order: int = 0
    # BackLogActor semantics (back_log.rs:38-91): 0 = reference (dropped), 1 = replay (SPEC.md §10)
    backlog_mode: int = 0

    def __post_init__(self):
        if self.addresses is None:
            self.addresses = synthetic_addresses(self.n)
        if len(self.addresses) != self.n:
            raise ValueError("address table does not match n")
        if list(self.addresses) != sorted(self.addresses):
            raise ValueError("addresses must be sorted ascending (validator index order)")
        if self.max_ticks == 0:
            self.max_ticks = 4 * self.heights + 64
        if self.seed_byte_order not in (0, 1) or self.backlog_mode not in (0, 1):
            raise ValueError("seed_byte_order / backlog_mode must be 0 or 1")

    @property
    def quorum(self) -> int:
        return (2 * self.n) // 3 + 1

    def silent_mask(self) -> List[int]:
        m = [0, 0, 0, 0]
        for i in self.silent:
            m[i >> 6] |= 1 << (i & 63)
        return m

    def address_bytes(self) -> bytes:
        return b"".join(self.addresses)


def cfg1(n5: bool = True, heights: int = 100, seed: int = 1) -> BftConfig:
    """One cluster from examples/c1..c5.toml; only c1-c4 run (build.sh), so c5 is silent."""
    addrs = [string_to_address(a) for a in C_ADDRESSES]
    if not n5:
        addrs = addrs[:4]
    srt = sorted_addresses(addrs)
    silent = [srt.index(addrs[4])] if n5 else []
    return BftConfig(n=len(srt), heights=heights, seed=seed, addresses=srt, silent=silent,
                     name="cfg1-n5" if n5 else "cfg1-n4")


def cfg2(heights: int = 100, byz: int = 0) -> BftConfig:
    """65,536 instances, N=4 f=1, 10% message drop (BASELINE.json configs[1]). f is the tolerance
    ⌊(N−1)/3⌋ here (SPEC.md §6); byz=1 runs that f as an equivocating validator ("cfg2-byz")."""
    return BftConfig(n=4, heights=heights, seed=2, drop_ppm=100_000, byz_count=byz,
                     name="cfg2-byz" if byz else "cfg2")


def cfg3(heights: int = 100) -> BftConfig:
    """16,384 instances, N=64, f=21 Byzantine equivocation (BASELINE.json configs[2], the metric)."""
    return BftConfig(n=64, heights=heights, seed=3, byz_count=21, name="cfg3")


def cfg4(n: int, heights: int = 100) -> BftConfig:
    """Validator-count sweep with proposer crashes (p=0.3 per view) → round-change storms."""
    return BftConfig(n=n, heights=heights, seed=4, proposer_crash_ppm=300_000, name=f"cfg4-n{n}")


def cfg5(heights: int = 10_000, byz: int = 0) -> BftConfig:
    """1M instances, N=7 (tolerates f=2), 5% drop, long horizon; all validators honest. byz=2 runs
    the tolerated f as equivocating validators ("cfg5-byz")."""
    return BftConfig(n=7, heights=heights, seed=5, drop_ppm=50_000, byz_count=byz,
                     name="cfg5-byz" if byz else "cfg5")


INSTANCES = {"cfg1": 1, "cfg2": 65_536, "cfg3": 16_384, "cfg4": 16_384, "cfg5": 1_048_576}


def timed_pipeline(instances_per_gpu: int):
    """(pipeline depth, hash batch) that bench.py times a launch size with (bftsim_set_pipeline /
    bftsim_set_hash_batch): a ring of 32 row-table sets, so that no launch of the 5 warmup + 20 timed ones waits for a
    set to come back from its chain batch, with the chains of 8 launches per kernel -- a lane per instance from 8,192
    instances per launch, lane pairs on the predicted blocks below (§4h). tests/test_gpu_pipeline.py
    runs exactly these settings at full size (`instances_per_gpu` kept for the shape of the call)."""
    return (32, 8)


# ---- the benchmark's workloads (bench.py --workload), shared with the tests that pin each timed mode ----
def drop64(heights: int = 100) -> BftConfig:
    """cfg3 with 5 % link drops (N = 64, f = 21 equivocating): the lossy FAST / resume path."""
    return BftConfig(n=64, heights=heights, seed=15, byz_count=21, drop_ppm=50_000, name="drop64")


BENCH_INSTANCES = {"cfg5": 131_072, "cfg2": 65_536}    # per GPU; every other workload 16,384
CFG5_WINDOW = 256                                      # canonical rows kept per instance (bftsim_set_window)


def bench_instances(workload: str) -> int:
    return BENCH_INSTANCES.get(workload, 16_384)


def bench_steps(workload: str):
    """(timed steps, warmup steps) bench.py defaults to: the driver's 20 / 5 for the headline, 10 / 2 otherwise."""
    return (20, 5) if workload == "cfg3" else (10, 2)


def bench_config(workload: str, n: int = 256, heights: int = None, byz: int = 0) -> BftConfig:
    """The BftConfig bench.py times a workload on (cfg4: `n` validators)."""
    if workload == "cfg5":
        return cfg5(heights=heights or 10_000, byz=byz)
    h = heights or 100
    if workload == "cfg2":
        return cfg2(heights=h, byz=byz)
    if workload == "cfg4":
        return cfg4(n, heights=h)
    if workload == "drop64":
        return drop64(heights=h)
    return cfg3(heights=h)

