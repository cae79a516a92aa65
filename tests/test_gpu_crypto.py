"""GPU: real-crypto mode (include/bftsim.h bftsim_set_crypto / bftsim_crypto_verify, SPEC.md §11).
The simulated run equals the oracle's (forged senders' messages dropped at every receiver); the batched
sign / recover pass recovers every honest message to its sender and no forged one to any validator;
the per-instance signature checksums equal the CPU reference's (RFC 6979 signatures of the msgpack
sign payloads, tests/crypto_ref.py), with the reference's own c1..c5 keys."""
import json
import os

import numpy as np
import pytest

import crypto_ref as C
import oracle_lib as O
from bftsim.configs import BftConfig, cfg1, cfg3
from parity_util import assert_same

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "sig_vectors.json")))


def _core(r):
    return {k: v for k, v in r.items() if k not in ("mlog", "mlog_n", "seconds", "round_hist", "latency_hist")}


def _run(cfg, secrets, first, n, forged=(), log_cap=0):
    from bftsim.runtime import Simulator
    sim = Simulator(cfg)
    try:
        sim.set_crypto(secrets, forged, log_cap)
        got = sim.run(first, n)
        rep = sim.crypto_verify()
    finally:
        sim.close()
    return got, rep


def _keyed(cfg, seed):
    from bftsim.crypto import synthetic_secrets, keyed_config, gpu_addresses
    sec = synthetic_secrets(cfg.n, seed)
    return keyed_config(cfg, sec, gpu_addresses(sec))


def test_reference_keys_cfg1():
    keys = {bytes.fromhex(k["address"]): bytes.fromhex(k["secret"]) for k in GOLD["reference_keys"]}
    cfg = cfg1(True, heights=10)
    secrets = [keys[a] for a in cfg.addresses]           # c1..c5 of examples/*.toml, validator order
    got, rep = _run(cfg, secrets, 0, 1)
    ref = O.run_crypto(cfg, 0, 1)
    assert_same(_core(ref), _core(got), "cfg1 crypto")
    assert rep["messages"] == int(ref["mlog_n"][0]) > 0
    assert rep["mismatches"] == 0 and rep["seal_errors"] == 0 and rep["forged"] == 0
    assert rep["recovered_as_sender"] == rep["messages"]
    assert rep["seals"] == int(((ref["mlog"][0, : rep["messages"], 1] >> 8) & 0xff == 3).sum())
    assert np.array_equal(rep["checksum"], C.instance_checksums(cfg, 0, ref, secrets))


def test_ledger_with_votes_cfg1():
    """bftsim_export_ledger: each committed Header carries, in ascending validator order, the Commit
    signatures of more than 2N/3 validators for that height and committed round (backend.rs:163-174);
    without the votes the bytes are the oracle's header, whose hash is the run's block hash."""
    import msgpack
    from bftsim.runtime import Simulator
    keys = {bytes.fromhex(k["address"]): bytes.fromhex(k["secret"]) for k in GOLD["reference_keys"]}
    cfg = cfg1(True, heights=6)
    secrets = [keys[a] for a in cfg.addresses]
    sim = Simulator(cfg)
    try:
        sim.set_crypto(secrets)
        got = sim.run(0, 1)
        sim.crypto_verify()
        ledger = sim.export_ledger()[0]
    finally:
        sim.close()
    ref = O.run_crypto(cfg, 0, 1)
    sigs = {}
    C.instance_checksums(cfg, 0, ref, secrets, sigs_out=sigs)
    ch = int(got["committed_height"][0])
    assert len(ledger) == ch == 6
    q = (2 * cfg.n) // 3
    for x, hdr in enumerate(ledger, start=1):
        fields = msgpack.unpackb(hdr)
        assert len(fields) == 13 and fields[7] == x
        votes = [bytes(v) for v in fields[12]]
        assert len(votes) > q
        rnd = int(got["round"][0, x - 1])
        cands = {s: sigs[(0, s, 3, x, rnd, False)] for s in range(cfg.n) if (0, s, 3, x, rnd, False) in sigs}
        order = [s for s, sg in sorted(cands.items()) if sg in votes]
        assert [cands[s] for s in order] == votes          # every vote is a sender's Commit, ascending
        plain = msgpack.packb(fields[:12] + [None])
        assert O.keccak256(plain) == bytes(got["block_hash"][0, x - 1])


def test_forged_sender_dropped():
    cfg, secrets = _keyed(BftConfig(n=4, heights=6, seed=21), 7)
    got, rep = _run(cfg, secrets, 3, 1, forged=(2,))
    ref = O.run_crypto(cfg, 3, 1, forged=(2,))
    assert_same(_core(ref), _core(got), "forged 2")
    assert rep["messages"] == int(ref["mlog_n"][0])
    assert rep["forged"] > 0 and rep["mismatches"] == 0 and rep["seal_errors"] == 0
    assert rep["recovered_as_sender"] == rep["messages"] - rep["forged"]
    assert np.array_equal(rep["checksum"], C.instance_checksums(cfg, 3, ref, secrets, forged=(2,)))


def test_cfg3_keys_and_forgers():
    cfg, secrets = _keyed(cfg3(heights=4), 3)
    got, rep = _run(cfg, secrets, 0, 4, forged=(0, 5), log_cap=16384)   # round-change storms: 8k+ messages
    ref = O.run_crypto(cfg, 0, 4, forged=(0, 5), cap=16384)
    assert_same(_core(ref), _core(got), "cfg3 crypto")
    assert np.array_equal(rep["inst_messages"], ref["mlog_n"])
    assert rep["mismatches"] == 0 and rep["seal_errors"] == 0 and rep["forged"] > 0
    assert rep["recovered_as_sender"] == rep["messages"] - rep["forged"]


def test_wrong_secret_rejected():
    from bftsim.runtime import Simulator, BftsimError
    cfg, secrets = _keyed(BftConfig(n=4, heights=3), 1)
    sim = Simulator(cfg)
    try:
        with pytest.raises(BftsimError):
            sim.set_crypto(secrets[::-1])                   # keys not in the validator order
    finally:
        sim.close()
