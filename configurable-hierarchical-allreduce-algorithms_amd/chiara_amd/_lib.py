"""Loader for libchiara.so (the in-tree MI355X build of the CHiArA hot path).

There is no CPU fallback: if the library is missing, importing the package fails
loudly with the build command to run.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)
LIB_PATH = os.path.join(HERE, "libchiara.so")


class ChiaraError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = code
        msg = _lib.chr_error_string(code).decode() if _lib is not None else str(code)
        super().__init__(f"{what}: chiara error {code} ({msg})" if what else f"chiara error {code} ({msg})")


class UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


def _load():
    # One HIP runtime per process: torch bundles its own libamdhip64.so.7 / librccl.so.1.
    # Loading torch first makes libchiara's NEEDED entries resolve (by SONAME) to those
    # copies instead of a second runtime from /opt/rocm competing for the device.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libchiara.so not found at {LIB_PATH}; build it with "
            f"`make -C {PKG_ROOT}` (hipcc --offload-arch=gfx950) or __graft_entry__.build()")
    L = ctypes.CDLL(LIB_PATH)
    vp, sz, i, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64
    pp = ctypes.POINTER(ctypes.c_void_p)
    sig = {
        "chr_abi_version": ([], i),
        "chr_error_string": ([i], ctypes.c_char_p),
        "chr_reduce_local": ([vp, vp, sz, i, i, vp], i),
        "chr_reduce_multi": ([vp, vp, pp, i, sz, i, i, vp], i),
        "chr_fill": ([vp, sz, i, i, u64, i, u64, vp], i),
        "chr_get_unique_id": ([ctypes.POINTER(UniqueId)], i),
        "chr_comm_init_rank": ([ctypes.POINTER(vp), i, ctypes.POINTER(UniqueId), i, i], i),
        "chr_comm_destroy": ([vp], i),
        "chr_comm_rank": ([vp, ctypes.POINTER(i)], i),
        "chr_comm_size": ([vp, ctypes.POINTER(i)], i),
        "chr_comm_info": ([vp, ctypes.POINTER(i), ctypes.POINTER(i), ctypes.POINTER(i), ctypes.c_char_p, i], i),
        "chr_comm_stream": ([vp, pp], i),
        "chr_allreduce_radix_batch": ([vp, vp, sz, i, i, vp, i, i], i),
        "chr_reduce_scatter_radix_batch": ([vp, vp, sz, i, i, vp, i, i], i),
        "chr_allreduce_radix_batch_async": ([vp, vp, sz, i, i, vp, i, i], i),
        "chr_reduce_scatter_radix_batch_async": ([vp, vp, sz, i, i, vp, i, i], i),
        "chr_local_group_create": ([ctypes.POINTER(vp), i, i], i),
        "chr_local_group_destroy": ([vp], i),
        "chr_local_group_stream": ([vp, pp], i),
        "chr_local_allreduce_radix_batch": ([vp, pp, pp, sz, i, i, i, i], i),
        "chr_local_reduce_scatter_radix_batch": ([vp, pp, pp, sz, i, i, i, i], i),
        "chr_plan_describe": ([i, i, i, i, i, sz, i, ctypes.c_char_p, sz], ctypes.c_long),
        "chr_comm_set_slices": ([vp, i], i),
        "chr_comm_profile": ([vp, i], i),
        "chr_comm_profile_read": ([vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(ctypes.c_long), i], i),
        "chr_local_group_set_slices": ([vp, i], i),
        "chr_reduce_multi_ex": ([vp, vp, pp, i, sz, i, i, i, vp], i),
        "chr_allreduce_mpich": ([vp, vp, sz, i, i, vp, i, i, i], i),
        "chr_allreduce_mpich_async": ([vp, vp, sz, i, i, vp, i, i, i], i),
        "chr_local_allreduce_mpich": ([vp, pp, pp, sz, i, i, i, i, i], i),
        "chr_allgather_radix_batch": ([vp, sz, i, vp, vp, i, i], i),
        "chr_comm_set_schedule": ([vp, i], i),
        "chr_comm_set_overlap": ([vp, i], i),
        "chr_comm_get_overlap": ([vp, ctypes.POINTER(i)], i),
        "chr_op_create": ([vp, vp, i, ctypes.POINTER(i)], i),
        "chr_op_free": ([i], i),
        "chr_plan_describe_op": ([i, i, i, i, i, sz, i, i, i, ctypes.c_char_p, sz], ctypes.c_long),
        "chr_local_group_set_schedule": ([vp, i], i),
        "chr_plan_describe_ex": ([i, i, i, i, i, sz, i, i, ctypes.c_char_p, sz], ctypes.c_long),
        "chr_allgather_radix_batch_async": ([vp, sz, i, vp, vp, i, i], i),
        "chr_local_allgather_radix_batch": ([vp, pp, pp, sz, i, i, i], i),
        "chr_reduce_tree": ([vp, pp, i, ctypes.c_char_p, ctypes.c_char_p, sz, i, i, vp], i),
        "chr_comm_profile_phases": ([vp, ctypes.c_char_p, sz, i], ctypes.c_long),
        "chr_comm_tuned_schedule": ([vp, i, sz, i, i, i, ctypes.POINTER(i), ctypes.POINTER(i)], i),
        "chr_comm_set_graphs": ([vp, i], i),
        "chr_comm_set_host_pipeline": ([vp, i], i),
        "chr_comm_set_timeout": ([vp, i], i),
        "chr_comm_abort": ([vp], i),
        "chr_comm_synchronize": ([vp], i),
        "chr_comm_is_aborted": ([vp], i),
        "chr_reduce_tree_batch": ([pp, pp, i, i, ctypes.c_char_p, ctypes.c_char_p, sz, i, i, vp], i),
        "chr_reduce_scatter_mpich": ([vp, vp, sz, i, i, vp, i, i], i),
        "chr_reduce_scatter_mpich_async": ([vp, vp, sz, i, i, vp, i, i], i),
        "chr_local_reduce_scatter_mpich": ([vp, pp, pp, sz, i, i, i, i], i),
        "chr_local_group_profile": ([vp, i], i),
        "chr_local_group_set_batching": ([vp, i], i),
        "chr_intra_reduce_scatter_radix_batch": ([vp, vp, sz, i, i, vp, i, i], i),
        "chr_inter_reduce_linear": ([vp, vp, sz, i, i, vp, i], i),
        "chr_intra_scatter_radix_batch": ([vp, sz, i, vp, vp, i, i], i),
        "chr_local_phase_collective": ([vp, i, pp, pp, sz, i, i, i, i], i),
        "chr_local_group_profile_read": ([vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                          ctypes.POINTER(ctypes.c_long), i], i),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    return L


_lib = None
_lib = _load()


def lib():
    return _lib


# Every symbol include/chiara.h declares (checked by tests/test_abi.py).
EXPORTED = [
    "chr_reduce_local", "chr_reduce_multi", "chr_get_unique_id", "chr_comm_init_rank", "chr_comm_destroy",
    "chr_comm_rank", "chr_comm_size", "chr_comm_stream", "chr_comm_set_slices", "chr_local_group_set_slices",
    "chr_comm_profile", "chr_comm_profile_read", "chr_allreduce_radix_batch",
    "chr_reduce_scatter_radix_batch", "chr_allreduce_radix_batch_async", "chr_reduce_scatter_radix_batch_async",
    "chr_local_group_create", "chr_local_group_destroy", "chr_local_group_stream",
    "chr_local_allreduce_radix_batch", "chr_local_reduce_scatter_radix_batch", "chr_plan_describe", "chr_fill",
    "chr_error_string", "chr_abi_version", "chr_reduce_multi_ex", "chr_allreduce_mpich",
    "chr_allreduce_mpich_async", "chr_local_allreduce_mpich", "chr_allgather_radix_batch",
    "chr_allgather_radix_batch_async", "chr_local_allgather_radix_batch", "chr_comm_set_schedule", "chr_comm_set_overlap",
    "chr_local_group_set_schedule", "chr_plan_describe_ex", "chr_reduce_tree", "chr_comm_profile_phases",
    "chr_comm_tuned_schedule", "chr_comm_set_graphs", "chr_comm_set_host_pipeline", "chr_comm_set_timeout", "chr_comm_abort",
    "chr_comm_synchronize", "chr_comm_is_aborted", "chr_reduce_tree_batch", "chr_local_group_profile",
    "chr_local_group_profile_read", "chr_reduce_scatter_mpich", "chr_reduce_scatter_mpich_async",
    "chr_local_reduce_scatter_mpich", "chr_local_group_set_batching",
    "chr_intra_reduce_scatter_radix_batch", "chr_inter_reduce_linear", "chr_intra_scatter_radix_batch",
    "chr_local_phase_collective", "chr_comm_info", "chr_comm_get_overlap", "chr_op_create", "chr_op_free",
    "chr_plan_describe_op",
]
