"""Backlog replay mode (include/bftsim.h BFTSIM_BACKLOG_REPLAY, SPEC.md §10) on the CPU: the oracle's
replay semantics against the default drop mode, and the kernel body (wave emulator) against the
oracle with replay on. GPU parity of the mode is in test_gpu_parity.py (the *-replay cases)."""
import dataclasses

import numpy as np
import pytest

import oracle_lib as O
import emu_lib as E
from bftsim.configs import BftConfig, cfg1, cfg2, cfg3, cfg4
from parity_util import assert_same, mismatches


def _replay(cfg):
    return dataclasses.replace(cfg, backlog_mode=1, name=cfg.name + "-replay")


@pytest.mark.parametrize("mk,n", [(lambda: cfg1(True, heights=40), 1), (lambda: cfg4(7, heights=40), 32),
                                  (lambda: cfg3(heights=12), 4),
                                  (lambda: BftConfig(n=7, heights=30, seed=9, byz_count=2), 32)])
def test_lossless_runs_never_store(mk, n):
    # without message loss every Prepare / Commit finds its Preprepare first (SPEC.md §2 phase order)
    # and no RoundChange outruns a quorum: nothing is future, replay mode = drop mode
    cfg = mk()
    assert mismatches(O.run(cfg, 0, n), O.run(_replay(cfg), 0, n)) == []


def test_replay_changes_lossy_outcomes_and_stays_safe():
    cfg = cfg2(heights=100)
    drop = O.run(cfg, 0, 128, threads=8)
    rep = O.run(_replay(cfg), 0, 128, threads=8)
    changed = np.nonzero(drop["ticks"] != rep["ticks"])[0]
    assert len(changed) > 0                                  # stored messages were handled
    assert not (rep["flags"] & 1).any()                     # BFTSIM_FLAG_SAFETY: honest, no forks
    # deterministic: the same seeded schedule gives the same replayed run
    assert mismatches(rep, O.run(_replay(cfg), 0, 128, threads=4)) == []


def test_replay_heights_are_valid_chains():
    # every committed block of a replayed run links to its parent (block hash chain from the genesis)
    cfg = _replay(BftConfig(n=7, heights=30, seed=8, drop_ppm=200_000))
    res = O.run(cfg, 0, 16, threads=4)
    assert O.verify_chains(cfg, 0, res, threads=4) == 0


@pytest.mark.parametrize("name,mk,n", [
    ("n4-drop30", lambda: BftConfig(n=4, heights=30, seed=7, drop_ppm=300_000), 8),
    ("n10-mix", lambda: BftConfig(n=10, heights=20, seed=11, byz_count=3, drop_ppm=200_000,
                                  proposer_crash_ppm=200_000), 4),
    ("n33-drop-silent", lambda: BftConfig(n=33, heights=12, seed=12, drop_ppm=150_000, silent=[3, 20]), 2),
    ("n64-byz21-drop", lambda: BftConfig(n=64, heights=10, seed=15, byz_count=21, drop_ppm=100_000), 2),
    ("n129-drop", lambda: BftConfig(n=129, heights=6, seed=16, drop_ppm=200_000), 1),
])
def test_emulated_replay_matches_oracle(name, mk, n):
    cfg = _replay(mk())
    assert_same(O.run(cfg, 0, n), E.run(cfg, 0, n), name)
