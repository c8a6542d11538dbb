"""mapfx — MI355X-native batched MAPF gridworld step (HIP kernels behind a C ABI).

Importing this package loads libmapfx.so (built by __graft_entry__.build());
there is no CPU fallback.
"""
from . import rng, maps  # noqa: F401  (pure host utilities)
from ._abi import lib, MapfxError  # noqa: F401  (fails loudly if the library is missing)
from .batch import MapfGridBatch  # noqa: F401
from .partial import MarlPartialBatch  # noqa: F401
from .primal import PrimalBatch  # noqa: F401

__all__ = ["MapfGridBatch", "MarlPartialBatch", "MapfxError", "lib", "rng", "maps"]
