"""chiara_amd -- MI355X-native hot path of CHiArA (Configurable Hierarchical Allreduce
Algorithms): fused bucket-reduction HIP kernels + radix/batch schedules over RCCL.

The compute lives in libchiara.so (hand-written gfx950 HIP + host C++ schedule); this
package is the Python mirror of the reference's operator interface over its C ABI.
"""
from ._lib import EXPORTED, ChiaraError, lib  # noqa: F401  (fails loudly without libchiara.so)
from .collectives import (  # noqa: F401
    BFLOAT16, DOUBLE, DTYPE_SIZE, FLOAT, FLOAT32, FLOAT64, IN_PLACE, INT, INT32, MAX, MIN,
    MODE_ALLGATHER, MODE_ALLREDUCE, MODE_MPICH_KRSAG, MODE_MPICH_RD, MODE_MPICH_RECEXCH, MODE_MPICH_RING,
    MODE_MPICH_RMULT, MODE_MPICH_RSAG, MPICH_Allreduce_k_reduce_scatter_allgather,
    MPICH_Allreduce_recursive_multiplying,
    MODE_REDUCE_SCATTER, PROD, REDUCE_RUNNING_FIRST, SCHEDULE_BALANCED, SCHEDULE_EXACT, SCHEDULE_FLAT, SCHEDULE_FLAT_AG, SCHEDULE_FLAT_SEQ, SCHEDULE_AUTO,
    SCHEDULE_REFERENCE,
    SUCCESS, SUM, Comm, LocalGroup,
    MPICH_Allreduce_recursive_doubling, MPICH_Allreduce_recursive_exchange,
    MPICH_Allreduce_reduce_scatter_allgather, MPICH_Allreduce_ring, all_reduce_radix_batch,
    allgather_radix_batch, check,
    describe_plan, fill, get_unique_id, parse_plan, reduce_local, reduce_multi, reduce_multi_ex, reduce_tree,
    reduce_scatter_radix_batch,
)
