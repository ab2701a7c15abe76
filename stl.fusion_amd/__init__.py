"""stl.fusion_amd — MI355X-native engine for Stl.Fusion's cascading-invalidation hot path.

The package holds only what that path needs:
  csrc/   gfx950 HIP kernels + the C-ABI library (include/fgi.h) -> lib/libfgi.so
  host/   C++ mirror of ComputedRegistry / Computed.Invalidate() scopes / Invalidated handlers
  fgi.py  ctypes binding of the C-ABI (tests, bench)

Load it by path (the directory name contains a dot): see ``_pkg.load()`` at the repo root.
"""
from .fgi import (COMPUTING, CONSISTENT, INVALIDATED, F_DELAY_STARTED, F_HAS_DELAY, F_IOSO, NONE,  # noqa: F401
                  USED_ADDED, USED_DROPPED, USED_ESTATE, USED_INVALIDATED, FgiError, Graph, PruneStats,
                  WaveStats, load_library, LIB_PATH)

__all__ = ["Graph", "WaveStats", "PruneStats", "FgiError", "load_library", "LIB_PATH"]
