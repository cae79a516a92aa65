"""bftsim — MI355X-native batched BFT simulator (host side).

The compute path is `libbftsim.so` (HIP kernels for gfx950 behind the C ABI of
include/bftsim.h); this package only configures and calls it.
"""
from .configs import BftConfig, cfg1, cfg2, cfg3, cfg4, cfg5, INSTANCES  # noqa: F401
