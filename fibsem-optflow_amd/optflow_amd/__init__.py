"""Host-side Python mirror of the MI355X TV-L1 engine's C-ABI (include/tvl1.h).

The compute path is libtvl1_hip.so (HIP kernels for gfx950).  Nothing here
falls back to a CPU implementation: if the library is missing, Engine() raises.
"""
from .capi import (DEFAULTS, Engine, TVL1Error, TVL1Params, TVL1Stats, epe, load_engine,
                   make_params)

__all__ = ["DEFAULTS", "Engine", "TVL1Error", "TVL1Params", "TVL1Stats", "epe",
           "load_engine", "make_params"]
