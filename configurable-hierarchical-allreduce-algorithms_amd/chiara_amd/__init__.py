"""chiara_amd -- MI355X-native hot path of CHiArA (Configurable Hierarchical Allreduce
Algorithms): fused bucket-reduction HIP kernels + radix/batch schedules over RCCL.

The compute lives in libchiara.so (hand-written gfx950 HIP + host C++ schedule); this
package is the Python mirror of the reference's operator interface over its C ABI.
"""
from ._lib import EXPORTED, ChiaraError, lib  # noqa: F401  (fails loudly without libchiara.so)
from .collectives import *  # noqa: F401,F403  (the reference-interface mirror; __all__ in collectives.py)
