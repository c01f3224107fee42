"""chiara_amd -- MI355X-native hot path of CHiArA (Configurable Hierarchical Allreduce
Algorithms): fused bucket-reduction HIP kernels + radix/batch schedules over RCCL.

The compute lives in libchiara.so (hand-written gfx950 HIP + host C++ schedule); this
package is the Python mirror of the reference's operator interface over its C ABI.
"""
import os as _os

# Multi-process RCCL on this driver needs dmabuf IPC (HSA_ENABLE_IPC_MODE_LEGACY=0).  Set the default
# before torch (imported by _lib) or the HIP runtime load; a value the caller set is kept.
# C callers: the MPI shim and the harness mains set it themselves (csrc/api.cpp).
_os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

from ._lib import EXPORTED, ChiaraError, lib  # noqa: F401  (fails loudly without libchiara.so)
from .collectives import *  # noqa: F401,F403  (the reference-interface mirror; __all__ in collectives.py)
