"""Shared helpers for parity tests: compare two result dicts field by field."""
import numpy as np

FIELDS = ("committed_height", "flags", "ticks", "views", "round", "proposer", "variant",
          "time_tick", "block_hash")


def mismatches(a, b):
    return [k for k in FIELDS if not np.array_equal(a[k], b[k])]


def assert_same(a, b, what=""):
    bad = mismatches(a, b)
    if bad:
        idx = None
        for i in range(len(a["committed_height"])):
            if any(not np.array_equal(a[k][i], b[k][i]) for k in bad):
                idx = i
                break
        raise AssertionError(f"{what}: fields {bad} differ; first instance {idx}: " +
                             ", ".join(f"{k}: {a[k][idx]} vs {b[k][idx]}" for k in bad
                                       if np.ndim(a[k][idx]) == 0))
