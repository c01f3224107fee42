"""Host-side mirror of CHiArA's operator interface, over the libchiara C ABI.

Same names, argument meaning and status-code behaviour as the reference:
  all_reduce_radix_batch(sendbuf, recvbuf, count, datatype, op, comm, k, b) -> int
      Fugaku_experiments/Allreduce/all_reduce_radix_batch.cpp:202-204
  reduce_scatter_radix_batch(sendbuf, recvbuf, recvcount, datatype, op, comm, k, b) -> int
      Fugaku_experiments/Reduce-scatter/reduce_scatter_radix_batch.cpp:200-202
  reduce_local(inbuf, inoutbuf, count, datatype, op) -> int      (MPI_Reduce_local)
Return value 0 == MPI_SUCCESS.  Unlike the reference (which always returns MPI_SUCCESS)
the preconditions it leaves unchecked come back as nonzero codes (CHR_ERR_*).

Buffers may be torch tensors (device: device-resident path; CPU: staged through HBM),
numpy arrays (host) or raw integer addresses.  PyTorch is only plumbing here.
"""
import ctypes
import os

from ._lib import ChiaraError, UniqueId, lib

# datatypes (chr_dtype) with MPI-style aliases
FLOAT32 = FLOAT = 0
FLOAT64 = DOUBLE = 1
INT32 = INT = 2
BFLOAT16 = 3
INT8 = SIGNED_CHAR = 4
UINT8 = UNSIGNED_CHAR = BYTE = 5
INT16 = SHORT = 6
UINT16 = UNSIGNED_SHORT = 7
UINT32 = UNSIGNED = 8
INT64 = LONG = LONG_LONG = 9
UINT64 = UNSIGNED_LONG = 10
# MPI's MAXLOC / MINLOC pair types ({value; int index} C structs) and the C99 complex types
FLOAT_INT, DOUBLE_INT, LONG_INT, TWO_INT, SHORT_INT = 11, 12, 13, 14, 15
C_FLOAT_COMPLEX = C_COMPLEX = 16
C_DOUBLE_COMPLEX = 17
# ops (chr_op): MPI's predefined ops with MPICH's (type, op) table: the logical and bitwise ones on
# integer types only (logical also on float / double), MAXLOC / MINLOC on the pair types only, SUM /
# PROD on the complex types only
SUM, PROD, MAX, MIN = 0, 1, 2, 3
LAND, LOR, LXOR, BAND, BOR, BXOR = 4, 5, 6, 7, 8, 9
MAXLOC, MINLOC = 10, 11
SUCCESS = 0
ERR_INVALID_ARG, ERR_COUNT_NOT_DIVISIBLE, ERR_BATCH_NOT_DIVISOR = 1, 2, 3
ERR_RCCL, ERR_UNSUPPORTED, ERR_TIMEOUT, ERR_ABORTED = 5, 8, 9, 10
IN_PLACE = object()  # MPI_IN_PLACE analogue
_IN_PLACE_PTR = 1     # CHR_IN_PLACE

DTYPE_SIZE = {FLOAT32: 4, FLOAT64: 8, INT32: 4, BFLOAT16: 2, INT8: 1, UINT8: 1, INT16: 2, UINT16: 2, UINT32: 4,
              INT64: 8, UINT64: 8, FLOAT_INT: 8, DOUBLE_INT: 16, LONG_INT: 16, TWO_INT: 8, SHORT_INT: 8,
              C_FLOAT_COMPLEX: 8, C_DOUBLE_COMPLEX: 16}
MODE_ALLREDUCE, MODE_REDUCE_SCATTER = 0, 1
# MPICH baselines (testing/mpich_implementations/all_reduce/), chr_mode numbering
MODE_MPICH_RING, MODE_MPICH_RD, MODE_MPICH_RSAG, MODE_MPICH_RECEXCH = 2, 3, 4, 5
MODE_MPICH_KRSAG, MODE_MPICH_RMULT = 6, 7
MODE_ALLGATHER = 8
# MPICH baseline reduce-scatters (testing/mpich_implementations/reduce_scatter/)
MODE_MPICH_RS_RADIX, MODE_MPICH_RS_HALVING, MODE_MPICH_RS_DOUBLING, MODE_MPICH_RS_PAIRWISE = 9, 10, 11, 12
RS_MODES = (1, 9, 10, 11, 12)  # count = recvcount, send = nranks * recvcount
# CHiArA's phases as stand-alone collectives (testing/custom_implementations/work_dir/reduce_scatter/;
# count = recvcount)
MODE_INTRA_REDUCE_SCATTER, MODE_INTER_REDUCE_LINEAR, MODE_INTRA_SCATTER = 13, 14, 15
PHASE_MODES = (13, 14, 15)
SCHEDULE_REFERENCE, SCHEDULE_BALANCED, SCHEDULE_FLAT, SCHEDULE_EXACT, SCHEDULE_FLAT_AG, SCHEDULE_FLAT_SEQ = 0, 1, 2, 3, 4, 5
SCHEDULE_AUTO = 6  # measured choice among FLAT / FLAT_SEQ / FLAT_AG (/ FLAT_1SHOT) and the depth (Comm only)
SCHEDULE_FLAT_1SHOT = 7  # allreduce: one exchange step, every rank evaluates the whole buffer (small messages)
REDUCE_RUNNING_FIRST = 1  # chr_reduce_multi_ex flag (MPICH_do_reduce operand order)


def _addr(buf):
    """Raw address of a buffer (torch tensor, numpy array, ctypes object or int)."""
    if buf is None:
        return None
    if buf is IN_PLACE:
        return _IN_PLACE_PTR
    if isinstance(buf, int):
        return buf
    if hasattr(buf, "data_ptr"):
        return buf.data_ptr()
    if hasattr(buf, "ctypes"):
        return buf.ctypes.data
    if isinstance(buf, ctypes.Array):
        return ctypes.addressof(buf)
    raise TypeError(f"unsupported buffer type {type(buf)!r}")


def _stream(stream):
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    if hasattr(stream, "cuda_stream"):
        return stream.cuda_stream
    raise TypeError(f"unsupported stream {type(stream)!r}")


def check(code, what=""):
    if code != SUCCESS:
        raise ChiaraError(code, what)
    return code


# ---- kernel boundary ------------------------------------------------------------------------

def reduce_local(inbuf, inoutbuf, count, datatype, op, stream=None):
    """MPI_Reduce_local on device buffers: inout = in (op) inout (enqueued on `stream`)."""
    return lib().chr_reduce_local(_addr(inbuf), _addr(inoutbuf), count, datatype, op, _stream(stream))


def reduce_multi(out, acc, ins, count, datatype, op, stream=None):
    """Fused left-to-right reduction of len(ins) incoming buckets into acc (written to out)."""
    arr = (ctypes.c_void_p * max(1, len(ins)))(*[_addr(x) for x in ins])
    return lib().chr_reduce_multi(_addr(out), _addr(acc), arr, len(ins), count, datatype, op, _stream(stream))


def op_create(launcher, commute=False, ctx=None):
    """A user-defined op (chr_op_create, MPI_Op_create's analogue): `launcher` is the address of a chr_user_reduce_fn
    -- the caller's own device code, e.g. built with include/chiara_user_op.hpp -- as an int or a ctypes function.
    Returns the op code for every chr_reduce_* call and CHiArA's collectives."""
    addr = ctypes.cast(launcher, ctypes.c_void_p).value if not isinstance(launcher, int) else launcher
    op = ctypes.c_int(0)
    check(lib().chr_op_create(addr, ctx, int(bool(commute)), ctypes.byref(op)), "chr_op_create")
    return op.value


def op_free(op):
    """Release a user-defined op (chr_op_free); its code may be handed out again."""
    return lib().chr_op_free(op)


def fill(buf, count, datatype, pattern, seed, rank, count_for_seq=None, stream=None):
    """Device-side synthetic inputs (same generator as the oracle)."""
    cfs = count if count_for_seq is None else count_for_seq
    return lib().chr_fill(_addr(buf), count, datatype, pattern, seed, rank, cfs, _stream(stream))


# ---- communicators --------------------------------------------------------------------------

def get_unique_id():
    uid = UniqueId()
    check(lib().chr_get_unique_id(ctypes.byref(uid)), "chr_get_unique_id")
    return ctypes.string_at(ctypes.addressof(uid), ctypes.sizeof(uid))  # all 128 bytes (NULs included)


class Comm:
    """RCCL-backed communicator (one rank per process, one MI355X per rank)."""

    def __init__(self, nranks, unique_id, rank, device):
        if len(unique_id) != ctypes.sizeof(UniqueId):
            raise ValueError("unique_id must be the 128 bytes returned by get_unique_id()")
        uid = UniqueId.from_buffer_copy(unique_id)
        h = ctypes.c_void_p()
        check(lib().chr_comm_init_rank(ctypes.byref(h), nranks, ctypes.byref(uid), rank, device),
              "chr_comm_init_rank")
        self._h = h
        self.rank, self.nranks, self.device = rank, nranks, device

    @classmethod
    def from_torch_distributed(cls, group=None, device=None):
        """Bootstrap over an initialised torch.distributed group (gloo is enough): rank 0
        creates the RCCL unique id and broadcasts its 128 bytes."""
        import torch
        import torch.distributed as dist

        rank, n = dist.get_rank(group), dist.get_world_size(group)
        buf = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            buf.copy_(torch.frombuffer(bytearray(get_unique_id()), dtype=torch.uint8))
        dist.broadcast(buf, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        return cls(n, bytes(buf.numpy().tobytes()), rank, device)

    @property
    def handle(self):
        return self._h

    def info(self):
        """What RCCL's communicator reports (chr_comm_info): {"nranks": ncclCommCount, "rank":
        ncclCommUserRank, "device": ncclCommCuDevice, "pci_bus_id": hipDeviceGetPCIBusId}."""
        n, r, d = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        bus = ctypes.create_string_buffer(64)
        check(lib().chr_comm_info(self._h, ctypes.byref(n), ctypes.byref(r), ctypes.byref(d), bus, len(bus)),
              "chr_comm_info")
        return {"nranks": n.value, "rank": r.value, "device": d.value, "pci_bus_id": bus.value.decode()}

    def set_slices(self, slices):
        """Pipeline depth (0 = automatic); results are bit-identical for every depth."""
        check(lib().chr_comm_set_slices(self._h, slices))

    def set_overlap(self, enable):
        """Reductions on a second stream, overlapped with the RCCL transfers (default on)."""
        check(lib().chr_comm_set_overlap(self._h, int(bool(enable))))

    @property
    def overlap(self):
        """Whether local reductions run on the compute stream beside the transfers: the library's own setting
        (chr_comm_get_overlap), so a record reports what runs."""
        v = ctypes.c_int(0)
        check(lib().chr_comm_get_overlap(self._h, ctypes.byref(v)), "chr_comm_get_overlap")
        return bool(v.value)

    def set_schedule(self, schedule):
        """SCHEDULE_REFERENCE / SCHEDULE_BALANCED / SCHEDULE_FLAT / SCHEDULE_EXACT / SCHEDULE_FLAT_AG /
        SCHEDULE_FLAT_SEQ / SCHEDULE_FLAT_1SHOT / SCHEDULE_AUTO: where reductions are evaluated (never what
        they compute)."""
        check(lib().chr_comm_set_schedule(self._h, int(schedule)))

    def set_graphs(self, enable):
        """Replay device-resident collectives from captured HIP graphs (one per plan and buffers)."""
        check(lib().chr_comm_set_graphs(self._h, int(bool(enable))))

    def set_host_pipeline(self, window_mib):
        """Host-buffer allreduce / reduce-scatter calls larger than one window run as pipelined
        windows (H2D, collective and D2H on three streams); 0 = off.  Every rank must then pass host
        buffers for the same calls.  Same bits (block-window property)."""
        check(lib().chr_comm_set_host_pipeline(self._h, int(window_mib)))

    def set_timeout(self, timeout_ms):
        """Blocking calls give up after timeout_ms (0 = never): the communicator is aborted and
        ERR_TIMEOUT returned, so a lost peer is an error code instead of a hang."""
        check(lib().chr_comm_set_timeout(self._h, int(timeout_ms)))

    def abort(self):
        """Abort the RCCL communicator (ncclCommAbort); later calls return ERR_ABORTED."""
        check(lib().chr_comm_abort(self._h))

    def synchronize(self):
        """Wait for this communicator's enqueued work under the timeout; returns the status code."""
        return lib().chr_comm_synchronize(self._h)

    @property
    def aborted(self):
        return bool(lib().chr_comm_is_aborted(self._h))

    def tuned_schedule(self, mode, count, datatype, k, b):
        """(schedule, slices) SCHEDULE_AUTO kept for a collective already called with these arguments,
        or None; under a fixed schedule, that schedule and the depth such a call runs at."""
        sc, sl = ctypes.c_int(), ctypes.c_int()
        rc = lib().chr_comm_tuned_schedule(self._h, mode, count, datatype, k, b, ctypes.byref(sc), ctypes.byref(sl))
        return (sc.value, sl.value) if rc == SUCCESS else None

    def profile(self, enable=True):
        """Time every fused reduction launch and every step's RCCL group of this communicator (HIP events)."""
        check(lib().chr_comm_profile(self._h, 1 if enable else 0))

    def profile_read(self, reset=True):
        """(kernel_ms, algorithmic_bytes, launches) of the reductions since the last reset."""
        ms, by, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_long()
        check(lib().chr_comm_profile_read(self._h, ctypes.byref(ms), ctypes.byref(by), ctypes.byref(n),
                                          1 if reset else 0))
        return ms.value, by.value, n.value

    def profile_phases(self, reset=True):
        """{phase: transfer milliseconds} of the steps since the last reset (profiling on)."""
        n = lib().chr_comm_profile_phases(self._h, None, 0, 0)
        if n < 0:
            raise ChiaraError(1, "profile_phases")
        buf = ctypes.create_string_buffer(n + 1)
        lib().chr_comm_profile_phases(self._h, buf, n + 1, 1 if reset else 0)
        out = {}
        for ln in buf.value.decode().splitlines():
            name, ms = ln.rsplit(" ", 1)
            out[name] = float(ms)
        return out

    @property
    def stream(self):
        s = ctypes.c_void_p()
        check(lib().chr_comm_stream(self._h, ctypes.byref(s)))
        return s.value

    def destroy(self):
        if self._h:
            lib().chr_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


class LocalGroup:
    """n virtual ranks on ONE device (loopback transport, same plans and kernels)."""

    def __init__(self, nranks, device=0):
        h = ctypes.c_void_p()
        check(lib().chr_local_group_create(ctypes.byref(h), nranks, device), "chr_local_group_create")
        self._h = h
        self.nranks, self.device = nranks, device

    @property
    def stream(self):
        s = ctypes.c_void_p()
        check(lib().chr_local_group_stream(self._h, ctypes.byref(s)))
        return s.value

    def set_slices(self, slices):
        check(lib().chr_local_group_set_slices(self._h, slices))

    def set_schedule(self, schedule):
        check(lib().chr_local_group_set_schedule(self._h, int(schedule)))

    def set_batching(self, enable):
        """Virtual ranks' tree evaluations of one step share launches (default on); same bits."""
        check(lib().chr_local_group_set_batching(self._h, int(bool(enable))))

    def profile(self, enable=True):
        """Time every virtual rank's fused reduction launches (HIP events)."""
        check(lib().chr_local_group_profile(self._h, 1 if enable else 0))

    def profile_read(self, reset=True):
        """(kernel_ms, algorithmic_bytes, launches) of the reductions since the last reset."""
        ms, by, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_long()
        check(lib().chr_local_group_profile_read(self._h, ctypes.byref(ms), ctypes.byref(by), ctypes.byref(n),
                                                 1 if reset else 0))
        return ms.value, by.value, n.value

    def all_reduce_radix_batch(self, sendbufs, recvbufs, count, datatype, op, k, b):
        S = (ctypes.c_void_p * self.nranks)(*[_addr(x) for x in sendbufs])
        R = (ctypes.c_void_p * self.nranks)(*[_addr(x) for x in recvbufs])
        return lib().chr_local_allreduce_radix_batch(self._h, S, R, count, datatype, op, k, b)

    def reduce_scatter_radix_batch(self, sendbufs, recvbufs, recvcount, datatype, op, k, b):
        S = (ctypes.c_void_p * self.nranks)(*[_addr(x) for x in sendbufs])
        R = (ctypes.c_void_p * self.nranks)(*[_addr(x) for x in recvbufs])
        return lib().chr_local_reduce_scatter_radix_batch(self._h, S, R, recvcount, datatype, op, k, b)

    def allgather_radix_batch(self, sendbufs, sendcount, datatype, recvbufs, k, b):
        S = (ctypes.c_void_p * self.nranks)(*[_addr(x) for x in sendbufs])
        R = (ctypes.c_void_p * self.nranks)(*[_addr(x) for x in recvbufs])
        return lib().chr_local_allgather_radix_batch(self._h, S, R, sendcount, datatype, k, b)

    def reduce_scatter_mpich(self, algo, sendbufs, recvbufs, recvcount, datatype, op, k=2):
        """algo: MODE_MPICH_RS_RADIX / _HALVING / _DOUBLING / _PAIRWISE."""
        S = (ctypes.c_void_p * self.nranks)(*[_addr(x) for x in sendbufs])
        R = (ctypes.c_void_p * self.nranks)(*[_addr(x) for x in recvbufs])
        return lib().chr_local_reduce_scatter_mpich(self._h, S, R, recvcount, datatype, op, algo, k)

    def phase_collective(self, mode, sendbufs, recvbufs, recvcount, datatype, op, k, b):
        """mode: MODE_INTRA_REDUCE_SCATTER / MODE_INTER_REDUCE_LINEAR / MODE_INTRA_SCATTER (the stand-alone
        phases; a rank whose plan reads no input may pass None)."""
        S = (ctypes.c_void_p * self.nranks)(*[_addr(x) for x in sendbufs])
        R = (ctypes.c_void_p * self.nranks)(*[_addr(x) for x in recvbufs])
        return lib().chr_local_phase_collective(self._h, mode, S, R, recvcount, datatype, op, k, b)

    def allreduce_mpich(self, algo, sendbufs, recvbufs, count, datatype, op, k=2, single_phase_recv=0):
        """algo: MODE_MPICH_RING / _RD / _RSAG / _RECEXCH."""
        S = (ctypes.c_void_p * self.nranks)(*[_addr(x) for x in sendbufs])
        R = (ctypes.c_void_p * self.nranks)(*[_addr(x) for x in recvbufs])
        return lib().chr_local_allreduce_mpich(self._h, S, R, count, datatype, op, algo, k, single_phase_recv)

    def destroy(self):
        if self._h:
            lib().chr_local_group_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


# ---- schedule boundary (the reference's entry points) ------------------------------------------

def all_reduce_radix_batch(sendbuf, recvbuf, count, datatype, op, comm, k, b, async_op=False):
    fn = lib().chr_allreduce_radix_batch_async if async_op else lib().chr_allreduce_radix_batch
    return fn(_addr(sendbuf), _addr(recvbuf), count, datatype, op, comm.handle, k, b)


def reduce_scatter_radix_batch(sendbuf, recvbuf, recvcount, datatype, op, comm, k, b, async_op=False):
    fn = lib().chr_reduce_scatter_radix_batch_async if async_op else lib().chr_reduce_scatter_radix_batch
    return fn(_addr(sendbuf), _addr(recvbuf), recvcount, datatype, op, comm.handle, k, b)


def allgather_radix_batch(sendbuf, sendcount, datatype, recvbuf, comm, k, b, async_op=False):
    """all_gather_radix_batch_1_0.cpp:37 -- same argument order (sendbuf, sendcount, datatype, recvbuf, comm, k, b)."""
    fn = lib().chr_allgather_radix_batch_async if async_op else lib().chr_allgather_radix_batch
    return fn(_addr(sendbuf), sendcount, datatype, _addr(recvbuf), comm.handle, k, b)


# ---- MPICH baselines driven by testing/main.cpp (same names and argument order) -----------------

def _mpich(algo, sendbuf, recvbuf, count, datatype, op, comm, k=0, single_phase_recv=0, async_op=False):
    fn = lib().chr_allreduce_mpich_async if async_op else lib().chr_allreduce_mpich
    return fn(_addr(sendbuf), _addr(recvbuf), count, datatype, op, comm.handle, algo, k, single_phase_recv)


def MPICH_Allreduce_ring(sendbuf, recvbuf, count, datatype, op, comm, async_op=False):
    """allreduce_ring.cpp:3 -- ring reduce-scatter (reduction :80) + allgatherv."""
    return _mpich(MODE_MPICH_RING, sendbuf, recvbuf, count, datatype, op, comm, async_op=async_op)


def MPICH_Allreduce_recursive_doubling(sendbuf, recvbuf, count, datatype, op, comm, async_op=False):
    """allreduce_recursive_doubling.cpp:4."""
    return _mpich(MODE_MPICH_RD, sendbuf, recvbuf, count, datatype, op, comm, async_op=async_op)


def MPICH_Allreduce_reduce_scatter_allgather(sendbuf, recvbuf, count, datatype, op, comm, async_op=False):
    """allreduce_reduce_scatter_allgather.cpp:3 (Rabenseifner)."""
    return _mpich(MODE_MPICH_RSAG, sendbuf, recvbuf, count, datatype, op, comm, async_op=async_op)


def MPICH_Allreduce_recursive_exchange(sendbuf, recvbuf, count, datatype, op, comm, k, single_phase_recv,
                                       async_op=False):
    """allreduce_recexch.cpp:188 -- k-way MPICH_do_reduce (:147-186) on the fused kernel."""
    return _mpich(MODE_MPICH_RECEXCH, sendbuf, recvbuf, count, datatype, op, comm, k, single_phase_recv,
                  async_op=async_op)


def MPICH_Allreduce_k_reduce_scatter_allgather(sendbuf, recvbuf, count, datatype, op, comm, k, single_phase_recv,
                                               async_op=False):
    """allreduce_k_reduce_scatter_allgather.cpp:257 -- k-ary digit-reversed reduce-scatter + allgather."""
    return _mpich(MODE_MPICH_KRSAG, sendbuf, recvbuf, count, datatype, op, comm, k, single_phase_recv,
                  async_op=async_op)


def MPICH_Allreduce_recursive_multiplying(sendbuf, recvbuf, count, datatype, op, comm, k, async_op=False):
    """allreduce_recursive_multiplying.cpp:3 -- k-ary recursive doubling."""
    return _mpich(MODE_MPICH_RMULT, sendbuf, recvbuf, count, datatype, op, comm, k, async_op=async_op)


# ---- MPICH baseline reduce-scatters driven by testing/mpich_implementations/reduce_scatter/main.cpp ----

def _mpich_rs(algo, sendbuf, recvbuf, recvcount, datatype, op, comm, k=0, async_op=False):
    fn = lib().chr_reduce_scatter_mpich_async if async_op else lib().chr_reduce_scatter_mpich
    return fn(_addr(sendbuf), _addr(recvbuf), recvcount, datatype, op, comm.handle, algo, k)


def MPICH_reduce_scatter_radix(sendbuf, recvbuf, recvcount, datatype, op, comm, k, async_op=False):
    """reduce_scatter_radix.cpp:204 -- recexch reduce-scatter, the single-level ancestor of CHiArA's phase 1."""
    return _mpich_rs(MODE_MPICH_RS_RADIX, sendbuf, recvbuf, recvcount, datatype, op, comm, k, async_op)


def MPICH_reduce_scatter_rec_halving(sendbuf, recvbuf, count, datatype, op, comm, async_op=False):
    """reduce_scatter_recursive_halving.cpp:7."""
    return _mpich_rs(MODE_MPICH_RS_HALVING, sendbuf, recvbuf, count, datatype, op, comm, 0, async_op)


def MPICH_reduce_scatter_rec_doubling(sendbuf, recvbuf, recvcount, datatype, op, comm, async_op=False):
    """reduce_scatter_recursive_doubling.cpp:10."""
    return _mpich_rs(MODE_MPICH_RS_DOUBLING, sendbuf, recvbuf, recvcount, datatype, op, comm, 0, async_op)


def MPICH_reduce_scatter_pairwise(sendbuf, recvbuf, recvcount, datatype, op, comm, async_op=False):
    """reduce_scatter_pairwise.cpp:4."""
    return _mpich_rs(MODE_MPICH_RS_PAIRWISE, sendbuf, recvbuf, recvcount, datatype, op, comm, 0, async_op)


# ---- CHiArA's phases as stand-alone collectives (testing/custom_implementations/work_dir/reduce_scatter/) ----

def intra_reduce_scatter_radix_batch(sendbuf, recvbuf, recvcount, datatype, op, comm, k, b):
    """intra_reduce_scatter_radix.cpp:208 -- phase 1: per stage, the group's radix-k recexch reduce-scatter
    of IRC-element chunks; recvbuf[s * IRC] gets chunk s * b + lane (the leftover stage's for lanes < nu)."""
    return lib().chr_intra_reduce_scatter_radix_batch(_addr(sendbuf), _addr(recvbuf), recvcount, datatype, op,
                                                      comm.handle, k, b)


def inter_reduce_linear(sendbuf, recvbuf, recvcount, datatype, op, comm, b):
    """inter_linear_reduce.cpp:11 -- phase 2: the lane's root node of iteration i (node i * b + lane) folds
    every node's chunk i in ascending node order into recvbuf."""
    return lib().chr_inter_reduce_linear(_addr(sendbuf), _addr(recvbuf), recvcount, datatype, op, comm.handle, b)


def intra_scatter_radix_batch(sendbuf, recvcount, datatype, recvbuf, comm, k, b):
    """intra_scatter_radix_batch.cpp:10 -- the reduce-scatter's phase 3: the node root's b blocks go to the
    node's ranks through a k-nomial tree (same argument order as the reference)."""
    return lib().chr_intra_scatter_radix_batch(_addr(sendbuf), recvcount, datatype, _addr(recvbuf), comm.handle, k, b)


def reduce_multi_ex(out, acc, ins, count, datatype, op, flags, stream=None):
    arr = (ctypes.c_void_p * max(1, len(ins)))(*[_addr(x) for x in ins])
    return lib().chr_reduce_multi_ex(_addr(out), _addr(acc), arr, len(ins), count, datatype, op, flags,
                                     _stream(stream))


def reduce_tree(out, leaves, comb, swaps, count, datatype, op, stream=None):
    """Fused expression tree (chr_reduce_tree): leaves pushed in order, comb[j] combines after
    leaf j, swaps[c] = running value first for combine c."""
    arr = (ctypes.c_void_p * max(1, len(leaves)))(*[_addr(x) for x in leaves])
    cb = bytes(bytearray(comb))
    sb = bytes(bytearray(swaps)) if swaps is not None else None
    return lib().chr_reduce_tree(_addr(out), arr, len(leaves), cb, sb, count, datatype, op, _stream(stream))


def reduce_tree_batch(outs, leaves, comb, swaps, count, datatype, op, stream=None):
    """chr_reduce_tree_batch: len(outs) trees of len(leaves[t]) leaves each (all equal), programs
    comb[t] / swaps[t] (swaps may be None), batched into as few launches as possible."""
    nt = len(outs)
    nl = len(leaves[0]) if nt else 1
    O = (ctypes.c_void_p * max(1, nt))(*[_addr(x) for x in outs])
    L = (ctypes.c_void_p * max(1, nt * nl))(*[_addr(x) for lv in leaves for x in lv])
    cb = bytes(bytearray([c for prog in comb for c in prog]))
    sb = None if swaps is None else bytes(bytearray([x for prog in swaps for x in prog]))
    return lib().chr_reduce_tree_batch(O, L, nt, nl, cb, sb, count, datatype, op, _stream(stream))


# ---- plan introspection (host only) --------------------------------------------------------------

def describe_plan(mode, nranks, rank, k, b, count, slices=1, schedule=None, commutative=True):
    """Rank `rank`'s plan as text (chr_plan_describe_op); commutative=False: the plan a call with a non-commutative
    user op runs (the MPICH baselines branch on it)."""
    bal = SCHEDULE_FLAT if schedule is None else int(schedule)
    c = int(bool(commutative))
    n = lib().chr_plan_describe_op(mode, nranks, rank, k, b, count, slices, bal, c, None, 0)
    if n < 0:
        raise ValueError("bad plan request")
    buf = ctypes.create_string_buffer(n + 1)
    lib().chr_plan_describe_op(mode, nranks, rank, k, b, count, slices, bal, c, buf, n + 1)
    return buf.value.decode()


def parse_plan(text):
    """Parse describe_plan() output into {'header':{...}, 'pre':[...], 'steps':[...]}."""
    lines = text.strip().split("\n")
    head = dict(kv.split("=") for kv in lines[0].split()[1:])
    header = {k: int(v) for k, v in head.items()}
    plan = {"header": header, "pre": [], "steps": []}
    cur = None

    def local(tok):
        if tok[0] == "copy":
            return ("copy", (tok[1], int(tok[2])), (tok[3], int(tok[4])), int(tok[5]), [])
        if tok[0] == "copy2d":  # (width, rows, dpitch, spitch) in the last field
            return ("copy2d", (tok[1], int(tok[2])), (tok[3], int(tok[4])), int(tok[5]),
                    [int(tok[6]), int(tok[7]), int(tok[8])])
        m = int(tok[6])
        ins = [(tok[7 + 2 * j], int(tok[8 + 2 * j])) for j in range(m)]
        if tok[0] == "tree":  # leaves = [acc] + ins; then "c" comb... "s" swaps...
            rest = tok[7 + 2 * m:]
            si = rest.index("s")
            prog = ([int(x) for x in rest[1:si]], [int(x) for x in rest[si + 1:]])
            return ("tree", (tok[1], int(tok[2])), (tok[3], int(tok[4])), int(tok[5]), ins, prog)
        # "reduce_sw": running value first in every step (MPICH_do_reduce order)
        return (tok[0], (tok[1], int(tok[2])), (tok[3], int(tok[4])), int(tok[5]), ins)

    for ln in lines[1:]:
        tok = ln.split()
        if tok[0] == "pre":
            plan["pre"].append(local(tok[1:]))
        elif tok[0] == "step":
            wait = int(tok[3].split("=")[1]) if len(tok) > 3 and tok[3].startswith("wait=") else -1
            kv = dict(t.split("=", 1) for t in tok[4:] if "=" in t)
            deps = lambda v: [] if v in (None, "-") else [int(x) for x in v.split(",")]  # noqa: E731
            cur = {"label": tok[2], "wait": wait, "deps": deps(kv.get("deps")),
                   "sends": [], "recvs": [], "allgathers": [], "post": []}
            plan["steps"].append(cur)
        elif tok[0] in ("send", "recv"):
            cur[tok[0] + "s"].append((int(tok[1]), (tok[2], int(tok[3])), int(tok[4])))
        elif tok[0] == "allgather":  # in-place collective: (region ref, elements per rank)
            cur["allgathers"].append(((tok[1], int(tok[2])), int(tok[3])))
        else:
            cur["post"].append(local(tok))
    return plan


__all__ = [_n for _n in dir() if not _n.startswith("_") and _n not in ("ctypes", "os", "lib", "UniqueId")]
