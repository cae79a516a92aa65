"""The oracle reproduces the committed golden runs (determinism / fixture pin), and the CPU
emulation of the HIP kernel body reproduces them too."""
import json
import os

import numpy as np
import pytest

import oracle_lib as O
import emu_lib as E
from tests_golden_cases import CASES

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "oracle_runs.json")))


def check(r, gold):
    for i, g in enumerate(gold["results"]):
        ch = g["committed_height"]
        assert int(r["committed_height"][i]) == ch
        assert int(r["flags"][i]) == g["flags"]
        assert int(r["ticks"][i]) == g["ticks"]
        assert int(r["views"][i]) == g["views"]
        assert [int(x) for x in r["round"][i][:ch]] == g["round"]
        assert [int(x) for x in r["proposer"][i][:ch]] == g["proposer"]
        assert [int(x) for x in r["variant"][i][:ch]] == g["variant"]
        assert [int(x) for x in r["time_tick"][i][:ch]] == g["time_tick"]
        assert [bytes(r["block_hash"][i][k]).hex() for k in range(ch)] == g["block_hash"]


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_matches_golden(name):
    cfg = CASES[name]()
    gold = GOLD[name]
    check(O.run(cfg, gold["first"], gold["n"]), gold)


@pytest.mark.parametrize("name", ["cfg1_n5", "cfg1_n4", "cfg3_h20", "cfg4_n7_h30", "n4_byz2_unsafe"])
def test_kernel_emulation_matches_golden(name):
    cfg = CASES[name]()
    gold = GOLD[name]
    check(E.run(cfg, gold["first"], gold["n"]), gold)
