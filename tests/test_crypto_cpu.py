"""Real-crypto mode on the CPU (SPEC.md §11): the kernel body's broadcast log (wave emulator) equals the
oracle's entry for entry; logging alone changes no result; a forged sender's consensus messages reach
no receiver (the oracle and the kernel body agree on the resulting run)."""
import numpy as np
import pytest

import emu_lib as E
import oracle_lib as O
from bftsim.configs import BftConfig, cfg1, cfg2, cfg3
from parity_util import mismatches

CASES = [
    ("cfg1-n5", lambda: cfg1(True, heights=15), (), 1),
    ("cfg2", lambda: cfg2(heights=15), (), 4),
    ("cfg2-forged1", lambda: cfg2(heights=15), (1,), 4),
    ("n7-byz2-drop-forged3", lambda: BftConfig(n=7, heights=12, seed=8, byz_count=2, drop_ppm=100_000), (3,), 4),
    ("n10-crash-forged", lambda: BftConfig(n=10, heights=10, seed=9, proposer_crash_ppm=300_000), (0, 9), 2),
    ("cfg3-forged", lambda: cfg3(heights=4), (0, 5), 2),
    ("n100-drop-forged", lambda: BftConfig(n=100, heights=4, seed=3, drop_ppm=50_000), (7,), 1),
]


def _core(r):
    return {k: v for k, v in r.items() if k not in ("mlog", "mlog_n", "seconds")}


@pytest.mark.parametrize("name,mk,forged,n", CASES, ids=[c[0] for c in CASES])
def test_emulated_log_matches_oracle(name, mk, forged, n):
    cfg = mk()
    a, b = O.run_crypto(cfg, 0, n, forged), E.run_crypto(cfg, 0, n, forged)
    assert mismatches(_core(a), _core(b)) == [], name
    assert np.array_equal(a["mlog_n"], b["mlog_n"])
    for i in range(n):
        k = int(a["mlog_n"][i])
        assert np.array_equal(a["mlog"][i, :k], b["mlog"][i, :k]), (name, i)


@pytest.mark.parametrize("mk,n", [(lambda: cfg2(heights=20), 8), (lambda: cfg3(heights=5), 2),
                                  (lambda: BftConfig(n=7, heights=15, seed=4, drop_ppm=100_000, byz_count=2), 8)])
def test_logging_changes_nothing(mk, n):
    cfg = mk()
    assert mismatches(_core(O.run_crypto(cfg, 0, n)), O.run(cfg, 0, n)) == []


def test_log_entries_are_the_broadcasts():
    # cfg1 (c5 silent): entries in (tick, phase, sender, kind) order, senders are the running validators,
    # every committed height was proposed, nothing forged
    cfg = cfg1(True, heights=6)
    r = O.run_crypto(cfg, 0, 1)
    log = r["mlog"][0, : int(r["mlog_n"][0])]
    codes = (log[:, 1] >> 8) & 0xff
    senders = set(int(x) for x in log[:, 1] >> 16)
    assert senders == set(range(5)) - set(cfg.silent)
    assert (codes == 1).sum() >= 6 and (codes == 2).sum() >= 24 and (codes == 3).sum() >= 24
    key = [(int(e[0]), int(e[1]) & 0xff, int(e[1]) >> 16) for e in log]
    assert key == sorted(key)
    assert not (log[:, 6] & 1).any()


def test_forged_proposer_is_heard_by_nobody():
    # validator 0 proposes round 0 of every height (BE seeds, N = 4): with a forged key its Preprepares
    # are dropped everywhere, each height needs a round change and no committed block is its own
    cfg = cfg1(False, heights=5)
    r = O.run_crypto(cfg, 0, 1, forged=(0,))
    ch = int(r["committed_height"][0])
    assert ch == 5
    assert (r["round"][0, :ch] >= 1).all() and (r["proposer"][0, :ch] != 0).all()
    log = r["mlog"][0, : int(r["mlog_n"][0])]
    assert ((log[:, 1] >> 16 == 0) == ((log[:, 6] & 1) == 1)).all()
    plain = O.run(cfg, 0, 1)
    assert (plain["round"][0] == 0).all()
