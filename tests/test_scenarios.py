"""Behaviour of the reference state machine under the seeded schedule (oracle), checked against
what the reference handlers imply. Each test names the handler lines it exercises."""
import numpy as np

import oracle_lib as O
from bftsim.configs import BftConfig, cfg1, cfg2, cfg3, cfg4
from bftsim.distributed import stats_from_result


def test_silent_proposer_forces_round_change():
    """cfg1: c5 (sorted index 4) never runs (build.sh starts c1-c4). When the round-0 proposer
    (validator.rs:33-48 seed of the parent hash) is c5, the 3 s timer fires (core.rs:207-225),
    round changes are exchanged (round_change.rs:26-98) and the height commits in round >= 1."""
    cfg = cfg1(True)
    r = O.run(cfg, 0, 1)
    assert r["committed_height"][0] == 100 and r["flags"][0] == 0
    import json, os
    gpath = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "genesis.json")
    hashes = [bytes.fromhex(json.load(open(gpath))["genesis_hash"])]
    hashes += [bytes(r["block_hash"][0][k]) for k in range(100)]
    silent_views = 0
    for h in range(1, 101):
        seed = O.lib().orc_seed_from_hash(hashes[h - 1], 5)
        rnd = int(r["round"][0][h - 1])
        prop = int(r["proposer"][0][h - 1])
        assert prop != 4, "the silent validator never proposes a committed block"
        assert prop == (seed + rnd) % 5, "committed block comes from the view's proposer"
        if seed % 5 == 4:
            silent_views += 1
            assert rnd >= 1
    assert silent_views > 5


def test_n4_cluster_never_changes_round():
    """cfg1 with only c1-c4 (N=4, power of two: seed ≡ 0, proposer = round mod 4)."""
    r = O.run(cfg1(False), 0, 1)
    assert r["committed_height"][0] == 100
    assert (r["round"][0] == 0).all() and (r["proposer"][0] == 0).all()


def test_equivocation_commits_exactly_one_variant_per_height():
    """cfg3: N=64, f=21. The round-0 proposer is validator 0; when it is Byzantine it
    equivocates (SPEC §6). Quorum intersection (Q=43 > (64+21)/2) keeps safety, and with no
    drops every height commits in round 0 with variant 0 or 1."""
    r = O.run(cfg3(heights=30), 0, 24)
    assert (r["flags"] == 0).all()
    assert (r["committed_height"] == 30).all()
    assert (r["round"] == 0).all()
    byz0 = []
    import ctypes
    c, keep = O.to_orc(cfg3())
    for i in range(24):
        m = (ctypes.c_uint64 * 4)()
        O.lib().orc_byz_mask(ctypes.byref(c), i, m)
        byz0.append(m[0] & 1)
    for i in range(24):
        if byz0[i]:
            assert set(np.unique(r["variant"][i])) <= {0, 1}
        else:
            assert (r["variant"][i] == 0).all()
    assert any(byz0) and not all(byz0)
    assert (r["variant"] == 1).any(), "some equivocated second blocks win"


def test_too_many_byzantine_breaks_safety():
    """f >= N/3 breaks quorum intersection: N=4, f=2 commits conflicting blocks (flag 1)."""
    r = O.run(BftConfig(n=4, heights=30, seed=9, byz_count=2), 0, 32)
    assert (r["flags"] & 1).any()


def test_equivocation_with_drops_can_deadlock_locked_validators():
    """Locks are never released (round_state.rs:113 unlock_hash has no caller): after an
    equivocation splits the honest validators' locks, neither block can reach Q again."""
    r = O.run(BftConfig(n=7, heights=40, seed=9, byz_count=2, drop_ppm=50_000), 0, 64)
    stalled = (r["flags"] & 16) != 0
    assert stalled.any()
    assert (r["flags"] & 1 == 0).all(), "stalls, but never unsafe (f < N/3)"


def test_proposer_crashes_cause_round_changes():
    """cfg4: the view's proposer stays silent with p=0.3 → timeout → round change."""
    r = O.run(cfg4(10, heights=60), 0, 32)
    assert (r["committed_height"] == 60).all()
    frac = (r["round"] > 0).mean()
    assert 0.2 < frac < 0.4
    st = stats_from_result(r)
    assert st["views"] == int((r["round"].astype(np.int64) + 1).sum())


def test_message_drops_stay_live():
    """cfg2: 10% drops; every instance still reaches H (catch-up by block gossip and Sync,
    core.rs:58-110)."""
    r = O.run(cfg2(heights=60), 0, 64)
    assert (r["committed_height"] == 60).all()
    assert (r["round"] > 0).any()


def test_determinism_and_instance_independence():
    cfg = cfg2(heights=20)
    a = O.run(cfg, 10, 12)
    b = O.run(cfg, 10, 12)
    for k in ("committed_height", "round", "block_hash", "ticks"):
        assert np.array_equal(a[k], b[k])
    c1 = O.run(cfg, 10, 5)
    c2 = O.run(cfg, 15, 7)
    assert np.array_equal(np.concatenate([c1["block_hash"], c2["block_hash"]]), a["block_hash"])
    d = O.run(cfg2(heights=20).__class__(**{**cfg.__dict__, "seed": 99}), 10, 12)
    assert not np.array_equal(d["block_hash"], a["block_hash"])
