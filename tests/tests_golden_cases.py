"""Config factories of the golden runs (must match tests/golden/make_golden.py RUNS)."""
from bftsim.configs import BftConfig, cfg1, cfg2, cfg3, cfg4, cfg5

CASES = {
    "cfg1_n5": lambda: cfg1(True),
    "cfg1_n4": lambda: cfg1(False),
    "cfg2_h20": lambda: cfg2(heights=20),
    "cfg3_h20": lambda: cfg3(heights=20),
    "cfg4_n7_h30": lambda: cfg4(7, heights=30),
    "cfg4_n64_h30": lambda: cfg4(64, heights=30),
    "cfg5_h60": lambda: cfg5(heights=60),
    "n4_byz2_unsafe": lambda: BftConfig(n=4, heights=30, seed=9, byz_count=2),
}
