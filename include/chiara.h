/*
 * chiara.h -- C ABI of the MI355X-native CHiArA hot path (libchiara.so).
 *
 * Drop-in boundary for the per-step local bucket reduction of CHiArA's hierarchical
 * radix/batch collectives (reference snapshot 2025-11-21, paths relative to the
 * reference root).  Every entry point cites the reference interface it replaces.
 * Plain pointers and sizes only; streams are HIP streams (hipStream_t).
 *
 * Status codes: 0 = CHR_SUCCESS (== MPI_SUCCESS), nonzero = chr_result below.  Unlike
 * the reference (which returns MPI_SUCCESS unconditionally, all_reduce_radix_batch.cpp:206,
 * :784), every precondition the reference leaves unchecked is rejected with a code.
 */
#ifndef CHIARA_H
#define CHIARA_H

#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CHR_ABI_VERSION 11 /* 11: user-defined ops (chr_op_create); 10: chr_comm_get_overlap; 9: chr_comm_info; 8: the stand-alone phase collectives (chr_intra_reduce_scatter_radix_batch, ...) */

/* Element types.  The reference is generic over MPI_Datatype (all_reduce_radix_batch.cpp:202-204,
 * sizes from MPI_Type_size at :234-277); these are the MPI predefined types MPICH's
 * MPI_Reduce_local accepts for the ops below.  Integer arithmetic wraps (two's complement), as
 * MPICH's C loops do on every supported platform. */
typedef enum {
    CHR_FLOAT32 = 0,   /* MPI_FLOAT */
    CHR_FLOAT64 = 1,   /* MPI_DOUBLE (testing/main.cpp harness) */
    CHR_INT32 = 2,     /* MPI_INT, MPI_INT32_T (Fugaku_experiments harnesses) */
    CHR_BFLOAT16 = 3,  /* no MPI equivalent: f32 arithmetic, RNE-rounded after every step */
    CHR_INT8 = 4,      /* MPI_SIGNED_CHAR, MPI_INT8_T, MPI_CHAR */
    CHR_UINT8 = 5,     /* MPI_UNSIGNED_CHAR, MPI_UINT8_T, MPI_BYTE (bitwise ops), MPI_C_BOOL (logical ops) */
    CHR_INT16 = 6,     /* MPI_SHORT, MPI_INT16_T */
    CHR_UINT16 = 7,    /* MPI_UNSIGNED_SHORT, MPI_UINT16_T */
    CHR_UINT32 = 8,    /* MPI_UNSIGNED, MPI_UINT32_T */
    CHR_INT64 = 9,     /* MPI_LONG, MPI_LONG_LONG, MPI_INT64_T */
    CHR_UINT64 = 10,   /* MPI_UNSIGNED_LONG, MPI_UNSIGNED_LONG_LONG, MPI_UINT64_T */
    /* The value/index pair types of MPI_MAXLOC / MPI_MINLOC, one element = the C struct MPI defines
     * ({value; int index}, naturally aligned; sizes below are the element stride, i.e. MPI's extent). */
    CHR_FLOAT_INT = 11,   /* MPI_FLOAT_INT   {float; int}    8 B */
    CHR_DOUBLE_INT = 12,  /* MPI_DOUBLE_INT  {double; int}  16 B (MPI_Type_size 12) */
    CHR_LONG_INT = 13,    /* MPI_LONG_INT    {long; int}    16 B (MPI_Type_size 12) */
    CHR_2INT = 14,        /* MPI_2INT        {int; int}      8 B */
    CHR_SHORT_INT = 15,   /* MPI_SHORT_INT   {short; int}    8 B (MPI_Type_size 6) */
    /* C99 complex types: SUM and PROD (C99 Annex G multiplication, as MPICH's C loop does) */
    CHR_C_FLOAT_COMPLEX = 16,   /* MPI_C_FLOAT_COMPLEX (MPI_C_COMPLEX)  8 B */
    CHR_C_DOUBLE_COMPLEX = 17   /* MPI_C_DOUBLE_COMPLEX                16 B */
} chr_dtype;

/* Reduction ops: MPI's predefined ops with MPICH 3.3.2's element semantics
 * (inout[i] = inout[i] OP in[i]), and MPICH's table of which (type, op) pairs it accepts.  SUM/PROD/
 * MAX/MIN on every integer and floating type; the logical ops (result 0 or 1) on the integer types
 * and on float/double (MPICH accepts those; C truth: NaN is true, -0 false); the bitwise ops on the
 * integer types only; MAXLOC/MINLOC on the five pair types only (equal values: the lower index wins,
 * the inout element is kept otherwise; NaN compares keep inout); SUM/PROD on the complex types only.
 * User-defined ops: chr_op_create below (device code; codes 64..127).  MPI_Op_create's host functions stay MPI_ERR_OP
 * through the shim. */
typedef enum {
    CHR_SUM = 0, CHR_PROD = 1, CHR_MAX = 2, CHR_MIN = 3,
    CHR_LAND = 4, CHR_LOR = 5, CHR_LXOR = 6,  /* MPI_LAND, MPI_LOR, MPI_LXOR */
    CHR_BAND = 7, CHR_BOR = 8, CHR_BXOR = 9,  /* MPI_BAND, MPI_BOR, MPI_BXOR */
    CHR_MAXLOC = 10, CHR_MINLOC = 11          /* MPI_MAXLOC, MPI_MINLOC */
} chr_op;

typedef enum {
    CHR_SUCCESS = 0,
    CHR_ERR_INVALID_ARG = 1,
    CHR_ERR_COUNT_NOT_DIVISIBLE = 2, /* count % nranks != 0: reference silently leaves a
                                        wrong tail (all_reduce_radix_batch.cpp:239) */
    CHR_ERR_BATCH_NOT_DIVISOR = 3,   /* nranks % b != 0: reference aborts in MPI_Irecv */
    CHR_ERR_HIP = 4,
    CHR_ERR_RCCL = 5,
    CHR_ERR_NO_DEVICE = 6,
    CHR_ERR_OUT_OF_MEMORY = 7,
    CHR_ERR_UNSUPPORTED = 8,
    CHR_ERR_TIMEOUT = 9,     /* a blocking call exceeded chr_comm_set_timeout; the communicator was
                                aborted (ncclCommAbort) */
    CHR_ERR_ABORTED = 10     /* the communicator was aborted by an earlier failure or chr_comm_abort */
} chr_result;

/* MPI_IN_PLACE analogue (all_reduce_radix_batch.cpp:234, :306-321): pass as `send`. */
#define CHR_IN_PLACE ((const void*)(uintptr_t)1)

/* ---- user-defined ops: MPI_Op_create's analogue ---------------------------------------
 * The reference is generic over MPI_Op (all_reduce_radix_batch.cpp:202-204), user-defined ops included: its
 * MPI_Reduce_local calls the op's function on host buffers.  Here a user op's arithmetic is the caller's own DEVICE
 * code -- the library never runs a reduction on the host: `fn` enqueues it on `stream` and returns 0 (anything else:
 * the op refuses the call, e.g. a type it does not implement; the library returns CHR_ERR_UNSUPPORTED).  For every
 * element i, with MPI's user-function convention x o y = fn(invec = x, inoutvec = y):
 *   running_first == 0:  out[i] = ins[m-1][i] o ( ... (ins[0][i] o acc[i]))    (MPI_Reduce_local(ins[j], acc) chained)
 *   running_first != 0:  out[i] = (((acc[i] o ins[0][i]) o ins[1][i]) ...)     (MPICH_do_reduce's order)
 * `out` may alias `acc`; m >= 0 (m == 0: out = acc).  include/chiara_user_op.hpp builds such a launcher from a device
 * functor.  chr_op_create returns the op (codes 64..127) for every chr_reduce_* entry point and CHiArA's collectives
 * (allreduce_radix_batch, reduce_scatter_radix_batch, the stand-alone phases, on communicators and local groups), each
 * taking the reference's operand order for any op -- commutative or not (tests/test_gpu_user_op.py against the
 * reference run with a user-defined non-commutative MPI_Op).  The MPICH baselines take user ops too and, as the
 * reference's, branch on `commute` (MPI_Op_commutative): rank-ordered operands for a non-commutative op in recursive
 * doubling (allreduce_recursive_doubling.cpp:69-80, reduce_scatter_recursive_doubling.cpp:134-160), and
 * CHR_ERR_UNSUPPORTED where the reference returns MPI_ERR_OP (k-reduce-scatter-allgather,
 * allreduce_k_reduce_scatter_allgather.cpp:278-283; recursive multiplying when nranks is not a power of k,
 * allreduce_recursive_multiplying.cpp:43-49).  Calls with a user op are never captured into HIP graphs.  64 ops may
 * be live at once.  The MPI shim still maps MPI_Op_create's host functions to MPI_ERR_OP. */
typedef int (*chr_user_reduce_fn)(void* out, const void* acc, const void* const* ins, int m, size_t n, chr_dtype dtype,
                                  int running_first, hipStream_t stream, void* ctx);
int chr_op_create(chr_user_reduce_fn fn, void* ctx, int commute, chr_op* op);
int chr_op_free(chr_op op);

/* ---- kernel boundary: replaces MPI_Reduce_local --------------------------------------
 * Reference call sites (MPI_Reduce_local(in, inout, count, datatype, op)):
 *   Fugaku_experiments/Allreduce/all_reduce_radix_batch.cpp:332, :364, :446, :529
 *   Fugaku_experiments/Reduce-scatter/reduce_scatter_radix_batch.cpp:332, :366, :447, :552
 * Semantics (MPICH 3.3.2 predefined ops): inout[i] = in[i] (op) inout[i].
 * Device pointers; the kernel is enqueued on `stream` and the call returns at once. */
int chr_reduce_local(const void* in, void* inout, size_t n, chr_dtype dtype, chr_op op,
                     hipStream_t stream);

/* Fused form of the k-1 (phase 1) or nnodes-1 (phase 2) consecutive Reduce_local calls
 * that target one region: out = (...((acc (op) ins[0]) (op) ins[1]) ...) (op) ins[m-1],
 * left to right, rounding after every step exactly as the sequential calls do
 * (all_reduce_radix_batch.cpp:343-364, :523-530).  `out` may alias `acc`. m >= 0. */
int chr_reduce_multi(void* out, const void* acc, const void* const* ins, int m, size_t n,
                     chr_dtype dtype, chr_op op, hipStream_t stream);
/* chr_reduce_multi with flags.  CHR_REDUCE_RUNNING_FIRST: the running value is the FIRST
 * operand of every step, acc = acc (op) ins[j], i.e. MPI_Reduce_local(acc, ins[j]) chained
 * the way MPICH_do_reduce does it
 * (testing/mpich_implementations/all_reduce/allreduce_recexch.cpp:147-186).  Only the floating
 * types (and the floating-valued pairs and the complex types) can differ bitwise from the default
 * order: MAX/MIN(LOC) on ties of -0/+0 and NaN compares, SUM/PROD on which NaN survives when two
 * meet -- MPICH's rules on x86, pinned by its own outputs (tests/golden/nan_reduce_local.npz):
 * inout's for float / double / bf16, in's in each part of a complex SUM, libgcc __mulsc3's operand
 * order for a complex PROD. */
#define CHR_REDUCE_RUNNING_FIRST 1
int chr_reduce_multi_ex(void* out, const void* acc, const void* const* ins, int m, size_t n,
                        chr_dtype dtype, chr_op op, int flags, hipStream_t stream);

/* Fused expression tree: one HBM pass evaluating the nested MPI_Reduce_local calls that
 * build one chunk's result across the reference's phases -- recexch folds
 * (all_reduce_radix_batch.cpp:364, :446), step-1 folds (:332) and the lane reduction (:529);
 * reduce_scatter_radix_batch.cpp:332, :366, :447, :552 -- with every intermediate kept in
 * registers.  Post-order stack program: leaves[j] is pushed in order j = 0..nleaves-1; after
 * leaf j, comb[j] combines follow.  A combine pops `in` and folds it into the value below
 * (the running value): below = MPI_Reduce_local(in, below), or with swaps[c] != 0 (combine c
 * in program order) MPI_Reduce_local(below, in) (MPICH_do_reduce order).  The program must
 * leave exactly one value: sum(comb) == nleaves-1, comb[0] == 0.  Limits: 1 <= nleaves <= 8,
 * stack depth <= 4 (CHR_ERR_UNSUPPORTED otherwise).  `out` may alias a leaf at the same
 * element offset.  swaps may be NULL (all zero). */
int chr_reduce_tree(void* out, const void* const* leaves, int nleaves, const unsigned char* comb,
                    const unsigned char* swaps, size_t n, chr_dtype dtype, chr_op op,
                    hipStream_t stream);

/* Several such trees in as few launches as possible (the flat schedule evaluates one per chunk of
 * a pipeline slice): tree t writes outs[t] from leaves[t*nleaves .. t*nleaves+nleaves-1] with the
 * program comb[t*nleaves ..] / swaps[t*(nleaves-1) ..] (swaps may be NULL).  Trees must not write
 * what another tree of the batch reads or writes (an in-place root over its own leaf is fine).
 * Bit-identical to ntrees chr_reduce_tree calls. */
int chr_reduce_tree_batch(void* const* outs, const void* const* leaves, int ntrees, int nleaves,
                          const unsigned char* comb, const unsigned char* swaps, size_t n,
                          chr_dtype dtype, chr_op op, hipStream_t stream);

/* ---- communicator (replaces MPI_Comm + MPI p2p: RCCL over xGMI) -------------------- */
typedef struct chr_comm chr_comm;
typedef struct { char internal[128]; } chr_unique_id; /* == ncclUniqueId */

int chr_get_unique_id(chr_unique_id* id);
/* One rank per process (or thread), one MI355X per rank.  Collective across `nranks`. */
int chr_comm_init_rank(chr_comm** comm, int nranks, const chr_unique_id* id, int rank, int device);
/* Releases the communicator.  On an aborted communicator this never blocks. */
int chr_comm_destroy(chr_comm* comm);
/* Failure handling (the reference relies on MPI_ERRORS_ARE_FATAL; a lost peer is a hang there).
 * A call that fails after posting RCCL operations aborts the communicator (ncclCommAbort) instead
 * of leaving its peers posted; every later call returns CHR_ERR_ABORTED.
 * chr_comm_set_timeout: blocking calls (and chr_comm_synchronize) poll the stream and RCCL's
 * asynchronous error state and give up after timeout_ms milliseconds, aborting the communicator
 * and returning CHR_ERR_TIMEOUT (or CHR_ERR_RCCL for a reported error); 0 = wait forever (the
 * default; env CHR_TIMEOUT_MS).  Tuning calls of CHR_SCHEDULE_AUTO use it too.
 * chr_comm_abort: abort on purpose (the MPI_Abort analogue for this communicator); peers then
 * get an error from their pending or next calls if they set a timeout.
 * chr_comm_synchronize: wait for the communicator's enqueued (_async) work under the timeout. */
int chr_comm_set_timeout(chr_comm* comm, int timeout_ms);
int chr_comm_abort(chr_comm* comm);
int chr_comm_synchronize(chr_comm* comm);
int chr_comm_is_aborted(const chr_comm* comm);
int chr_comm_rank(const chr_comm* comm, int* rank);
int chr_comm_size(const chr_comm* comm, int* nranks);
/* What RCCL's communicator itself reports -- ncclCommCount, ncclCommUserRank, ncclCommCuDevice --
 * and that device's PCI bus id (hipDeviceGetPCIBusId, "dddd:bb:dd.f", NUL-terminated in `len` bytes;
 * len 0 skips it).  The record of which GPUs a multi-GPU run's ranks were on (bench.py's N>1 line):
 * the reference's ranks are MPI processes (MPI_Comm_rank / MPI_Comm_size,
 * Fugaku_experiments/Allreduce/main.cpp:116-117).  CHR_ERR_ABORTED on an aborted communicator. */
int chr_comm_info(const chr_comm* comm, int* rccl_nranks, int* rccl_rank, int* rccl_device, char* pci_bus_id,
                  int len);
/* The stream all of this communicator's collective work is enqueued on.  It is a blocking
 * stream: it orders after work on the legacy NULL stream (hipMemset, default-stream kernels),
 * as an MPI caller expects.  Work that produces `send` on another non-blocking stream must be
 * ordered before the call (hipStreamWaitEvent on this stream, or a synchronize). */
int chr_comm_stream(const chr_comm* comm, hipStream_t* stream);
/* Pipeline depth of the schedules: every chunk is cut into `slices` element slices and
 * consecutive phases of different slices share one RCCL group (different xGMI links
 * busy at once).  0 = automatic (~64 MiB per slice message, up to 8; the flat schedules stop
 * where an evaluated piece would drop below 16 MiB, e.g. 4 at C4/C5; env CHR_SLICES).
 * Results are bit-identical for every depth. */
int chr_comm_set_slices(chr_comm* comm, int slices);
/* Where the radix/batch reductions are evaluated.  The result bits never depend on it: every
 * element gets the reference's expression (recexch phases in neighbour order, folds, lane
 * reduction in stage order) whatever the schedule.
 *   CHR_SCHEDULE_REFERENCE  the reference's reductions at its owner lanes / root nodes, its
 *                           recexch exchanges; results spread by a link-balanced distribute
 *   CHR_SCHEDULE_BALANCED   single-phase geometries (k == b, or b == 1): each rank evaluates
 *                           1/n of every chunk, hierarchical exchanges
 *   CHR_SCHEDULE_FLAT       (default) any geometry: each rank gathers the n-1 other inputs of
 *                           its piece directly over the xGMI mesh, evaluates the expression
 *                           tree, then the pieces are allgathered; 2S/n per link in all
 *   CHR_SCHEDULE_EXACT      the reference's communication pattern end to end, unsliced:
 *                           phases 0-2 as REFERENCE, then its inter-node bcast + intra-node
 *                           k-port Bruck allgather with rotation (all_reduce_radix_batch.cpp
 *                           :552-756), or its k-nomial scatter (reduce_scatter_radix_batch.cpp
 *                           :572-627); per GPU pair the same bytes as the reference
 *                           (tests/golden/msg_trace.json).  For multi-node shapes.
 *   CHR_SCHEDULE_FLAT_AG    FLAT with its allgather phase on RCCL's ncclAllGather collective
 *                           (in place, one per chunk) where the pieces are equal; data
 *                           movement only, so identical bits
 *   CHR_SCHEDULE_FLAT_SEQ   FLAT with its gather and allgather in separate RCCL groups (FLAT
 *                           merges the gather of slice t with the allgather of slice t-2)
 * Env CHR_SCHEDULE=reference|balanced|flat|exact|flat_ag|flat_seq|auto|flat_1shot sets the default.  DESIGN.md §5. */
#define CHR_SCHEDULE_REFERENCE 0
#define CHR_SCHEDULE_BALANCED 1
#define CHR_SCHEDULE_FLAT 2
#define CHR_SCHEDULE_EXACT 3
#define CHR_SCHEDULE_FLAT_AG 4
#define CHR_SCHEDULE_FLAT_SEQ 5
/*   CHR_SCHEDULE_AUTO       chooses among FLAT, FLAT_SEQ and FLAT_AG (and FLAT_1SHOT for
 *                           allreduces of <= 8 MiB per rank) and the pipeline depth by
 *                           measurement: on the first device-resident call for a (collective,
 *                           count, dtype, k, b) every candidate runs a few complete collectives,
 *                           the ranks agree on the slowest rank's times (one ncclAllReduce) and
 *                           the fastest is kept.  Same bits as every other schedule.  Host-staged
 *                           calls and the other collectives use FLAT. */
#define CHR_SCHEDULE_AUTO 6
/*   CHR_SCHEDULE_FLAT_1SHOT allreduce: every rank receives the whole buffer from every peer in one
 *                           exchange step and evaluates every chunk's expression tree itself (no
 *                           allgather): one RCCL group per slice instead of two, (n-1)·S bytes per
 *                           rank instead of 2(n-1)/n·S -- the latency-bound small-message variant of
 *                           FLAT.  Reduce-scatter runs FLAT (already one step).  Same bits. */
#define CHR_SCHEDULE_FLAT_1SHOT 7
int chr_comm_set_schedule(chr_comm* comm, int schedule);
/* What CHR_SCHEDULE_AUTO chose for a collective already called with these arguments
 * (mode: 0 allreduce_radix_batch, 1 reduce_scatter_radix_batch; count as passed); CHR_ERR_INVALID_ARG
 * under AUTO before such a call.  Under any other schedule: that schedule and the pipeline depth a
 * device-resident call with these arguments runs at. */
int chr_comm_tuned_schedule(const chr_comm* comm, int mode, size_t count, chr_dtype dtype, int k, int b, int* schedule,
                            int* slices);
/* Compute/xGMI overlap (default on; env CHR_OVERLAP=0): local reductions run on a second HIP
 * stream, ordered against the RCCL transfers by events where the plan's data dependencies
 * require it, so e.g. the flat schedule reduces slice s while slice s+1 is being gathered.
 * The call still completes on chr_comm_stream. */
int chr_comm_set_overlap(chr_comm* comm, int enable);
/* The overlap setting the communicator runs with (set_overlap, else CHR_OVERLAP as the library read it once per
 * process), so that a record of a call reports what ran rather than a re-read of the environment. */
int chr_comm_get_overlap(const chr_comm* comm, int* enable);
/* HIP graph replay (default off; env CHR_GRAPHS=1): a device-resident collective is captured once
 * per (plan, send, recv, dtype, op) -- its RCCL groups, fused reductions and copies on both streams
 * -- and later calls with the same arguments replay it with one hipGraphLaunch.  Cuts the host
 * cost per call to one launch (small messages are bound by it).  Buffers must stay allocated
 * while graphs that name them may be replayed; disabling drops every cached graph.  Same bits. */
int chr_comm_set_graphs(chr_comm* comm, int enable);
/* Pipelined host staging (default off; env CHR_HOST_WINDOW_MIB).  The reference's contract starts
 * and ends in host memory; with window_mib > 0 a host-buffer allreduce_radix_batch or
 * reduce_scatter_radix_batch whose per-rank buffer exceeds one window runs as a sequence of
 * collectives over windows of every recvcount block (about window_mib MiB per rank each): the
 * H2D copy of window j+1, the collective of window j and the D2H copy of window j-1 run on three
 * streams at once.  The bits are those of the whole call (an output window depends only on the
 * same window of every block: tests/test_oracle_golden.py::test_block_window_property).  Every
 * rank of the communicator must then pass host buffers for the same calls (the number of RCCL
 * collectives a call issues depends on it).  0 restores one H2D, one collective, one D2H.  The
 * D2H copies are issued from a second host thread, so copies from and to pageable memory overlap
 * in both directions too.  The MPI-signature shim turns this on (32 MiB) for its communicators. */
int chr_comm_set_host_pipeline(chr_comm* comm, int window_mib);
/* Opt-in timing of the fused bucket-reduction launches of this communicator (HIP events
 * on its stream).  _read synchronises on the recorded launches and returns the summed
 * kernel milliseconds, the algorithmic bytes ((m+2)*n*sizeof(T) per launch) and the
 * launch count since the last reset. */
int chr_comm_profile(chr_comm* comm, int enable);
int chr_comm_profile_read(chr_comm* comm, double* reduce_ms, double* reduce_bytes, long* launches,
                          int reset);
/* Per-phase transfer time while profiling: HIP events around every step's RCCL group on the
 * transfer stream, summed per phase (the plan step's label without slice suffixes, e.g.
 * "gather", "fdist", "phase0+lane", "bruck1").  The analogue of the reference's DEBUG_MODE
 * phase timers (all_reduce_radix_batch.cpp:228-232, :480-489, :542-548, :572-578, :758-764).
 * Writes "name milliseconds" lines into buf (NUL-terminated, truncated to len) and returns the
 * full text length; reset != 0 clears the sums. */
long chr_comm_profile_phases(chr_comm* comm, char* buf, size_t len, int reset);

/* ---- schedule boundary ----------------------------------------------------------------
 * Replaces  int all_reduce_radix_batch(char* sendbuf, char* recvbuf, int count,
 *             MPI_Datatype, MPI_Op, MPI_Comm, int k, int b)
 *           (Fugaku_experiments/Allreduce/all_reduce_radix_batch.cpp:202-204)
 * and       int reduce_scatter_radix_batch(const void* sendbuf, void* recvbuf,
 *             MPI_Aint recvcount, MPI_Datatype, MPI_Op, MPI_Comm, int k, int b)
 *           (Fugaku_experiments/Reduce-scatter/reduce_scatter_radix_batch.cpp:200-202).
 * Same arguments and results (bit-identical for the same (nranks, k, b)).
 * send/recv may be device pointers (device-resident path) or host pointers (staged
 * through HBM: the reference's host-memory-in / host-memory-out contract).  The call
 * returns once the result is in `recv` (stream synchronised).  Scratch is owned by the
 * communicator and reused across calls (the reference mallocs 2x the buffer per call). */
int chr_allreduce_radix_batch(const void* send, void* recv, size_t count, chr_dtype dtype,
                              chr_op op, chr_comm* comm, int k, int b);
int chr_reduce_scatter_radix_batch(const void* send, void* recv, size_t recvcount,
                                   chr_dtype dtype, chr_op op, chr_comm* comm, int k, int b);
/* Replaces  int allgather_radix_batch(char* sendbuf, int sendcount, MPI_Datatype,
 *             char* recvbuf, MPI_Comm, int k, int b)
 *           (Fugaku_experiments/Allgather/all_gather_radix_batch_1_0.cpp:37).
 * recv holds nranks*sendcount elements, rank-major (the reference's output on every
 * geometry).  k = peers per step (k-port), b = group size (nranks % b == 0; group peers
 * first).  send may be CHR_IN_PLACE: the own block is then already at recv + rank*sendcount.
 * Pure data movement: any dtype, bit-exact. */
int chr_allgather_radix_batch(const void* send, size_t sendcount, chr_dtype dtype, void* recv,
                              chr_comm* comm, int k, int b);
/* Asynchronous device-resident variants: enqueue on the comm stream and return. */
int chr_allreduce_radix_batch_async(const void* send, void* recv, size_t count, chr_dtype dtype,
                                    chr_op op, chr_comm* comm, int k, int b);
int chr_reduce_scatter_radix_batch_async(const void* send, void* recv, size_t recvcount,
                                         chr_dtype dtype, chr_op op, chr_comm* comm, int k, int b);
int chr_allgather_radix_batch_async(const void* send, size_t sendcount, chr_dtype dtype,
                                    void* recv, chr_comm* comm, int k, int b);

/* ---- virtual ranks on one device (loopback transport) ---------------------------------
 * `nranks` logical ranks sharing ONE device, messages become device-to-device copies;
 * every reduction runs the same HIP kernels as the RCCL path.  One call performs the
 * collective for all ranks: sends[r] / recvs[r] are rank r's device buffers. */
typedef struct chr_local_group chr_local_group;
int chr_local_group_create(chr_local_group** group, int nranks, int device);
int chr_local_group_destroy(chr_local_group* group);
int chr_local_group_stream(const chr_local_group* group, hipStream_t* stream);
int chr_local_group_set_slices(chr_local_group* group, int slices);
int chr_local_group_set_schedule(chr_local_group* group, int schedule);
/* Whether the virtual ranks' tree evaluations of one step share launches (default 1; env
 * CHR_LG_BATCH=0 sets the default to 0).  The ranks' trees are independent, so the bits are the
 * same either way; batched, a step pays a grid's fixed launch cost once per 8 trees instead of once
 * per rank.  No reference counterpart (the virtual-rank group is this library's own). */
int chr_local_group_set_batching(chr_local_group* group, int enable);
/* Timing of every virtual rank's fused reductions (HIP events on the group's stream), as
 * chr_comm_profile / chr_comm_profile_read: the collective's own kernels at full size with the
 * leaves just written by the loopback copies, one rank at a time. */
int chr_local_group_profile(chr_local_group* group, int enable);
int chr_local_group_profile_read(chr_local_group* group, double* reduce_ms, double* reduce_bytes,
                                 long* launches, int reset);
int chr_local_allreduce_radix_batch(chr_local_group* group, const void* const* sends,
                                    void* const* recvs, size_t count, chr_dtype dtype, chr_op op,
                                    int k, int b);
int chr_local_reduce_scatter_radix_batch(chr_local_group* group, const void* const* sends,
                                         void* const* recvs, size_t recvcount, chr_dtype dtype,
                                         chr_op op, int k, int b);
int chr_local_allgather_radix_batch(chr_local_group* group, const void* const* sends,
                                    void* const* recvs, size_t sendcount, chr_dtype dtype, int k,
                                    int b);

/* ---- schedule introspection (host only, no device needed) -----------------------------
 * The radix/batch schedule is compiled once per (mode, nranks, rank, k, b, count) into a
 * plan of steps; each step is one RCCL group of sends/receives followed by local ops.
 * chr_plan_describe writes rank `rank`'s plan as text (one op per line) into buf
 * (truncated to len, NUL-terminated); returns the length needed (excluding NUL) or < 0. */
typedef enum {
    CHR_MODE_ALLREDUCE = 0,        /* all_reduce_radix_batch */
    CHR_MODE_REDUCE_SCATTER = 1,   /* reduce_scatter_radix_batch */
    CHR_MODE_MPICH_RING = 2,       /* testing/mpich_implementations/all_reduce/allreduce_ring.cpp:3 */
    CHR_MODE_MPICH_RD = 3,         /* .../allreduce_recursive_doubling.cpp:4 */
    CHR_MODE_MPICH_RSAG = 4,       /* .../allreduce_reduce_scatter_allgather.cpp:3 */
    CHR_MODE_MPICH_RECEXCH = 5,    /* .../allreduce_recexch.cpp:188 (k, b = single_phase_recv) */
    CHR_MODE_MPICH_KRSAG = 6,      /* .../allreduce_k_reduce_scatter_allgather.cpp:257 (k, b = spr) */
    CHR_MODE_MPICH_RMULT = 7,      /* .../allreduce_recursive_multiplying.cpp:3 (k) */
    CHR_MODE_ALLGATHER = 8,        /* allgather_radix_batch (count = sendcount) */
    /* MPICH baseline reduce-scatters (block), testing/mpich_implementations/reduce_scatter/
     * (count = recvcount) */
    CHR_MODE_MPICH_RS_RADIX = 9,    /* reduce_scatter_radix.cpp:204 (k) */
    CHR_MODE_MPICH_RS_HALVING = 10, /* reduce_scatter_recursive_halving.cpp:7 */
    CHR_MODE_MPICH_RS_DOUBLING = 11,/* reduce_scatter_recursive_doubling.cpp:10 */
    CHR_MODE_MPICH_RS_PAIRWISE = 12,/* reduce_scatter_pairwise.cpp:4 */
    /* CHiArA's building blocks, stand-alone (testing/custom_implementations/work_dir/reduce_scatter/;
     * count = recvcount) */
    CHR_MODE_INTRA_REDUCE_SCATTER = 13, /* intra_reduce_scatter_radix.cpp:208 (k, b): phase 1 */
    CHR_MODE_INTER_REDUCE_LINEAR = 14,  /* inter_linear_reduce.cpp:11 (b): phase 2 */
    CHR_MODE_INTRA_SCATTER = 15         /* intra_scatter_radix_batch.cpp:10 (k, b): RS phase 3 */
} chr_mode;
long chr_plan_describe(chr_mode mode, int nranks, int rank, int k, int b, size_t count,
                       int slices, char* buf, size_t len);
/* The same for a given CHR_SCHEDULE_* (chr_plan_describe describes CHR_SCHEDULE_FLAT). */
long chr_plan_describe_ex(chr_mode mode, int nranks, int rank, int k, int b, size_t count,
                          int slices, int schedule, char* buf, size_t len);
/* The plan a call with an op of the given commutativity runs (MPI_Op_commutative; commutative = 0: a user op created
 * with commute = 0).  The MPICH baselines branch on it (recursive doubling, reduce-scatter recursive doubling) or
 * refuse a non-commutative op (k-reduce-scatter-allgather; recursive multiplying when nranks is not a power of k),
 * as the reference does; CHiArA's own plans do not depend on it.  (ABI 11) */
long chr_plan_describe_op(chr_mode mode, int nranks, int rank, int k, int b, size_t count, int slices, int schedule,
                          int commutative, char* buf, size_t len);

/* ---- MPICH baseline allreduces (the ones testing/main.cpp benchmarks CHiArA against) --
 * Replace  int MPICH_Allreduce_ring(const char* sendbuf, char* recvbuf, int count,
 *            MPI_Datatype, MPI_Op, MPI_Comm)                       (allreduce_ring.cpp:3)
 *          MPICH_Allreduce_recursive_doubling(...)        (allreduce_recursive_doubling.cpp:4)
 *          MPICH_Allreduce_reduce_scatter_allgather(...)  (allreduce_reduce_scatter_allgather.cpp:3)
 *          MPICH_Allreduce_recursive_exchange(..., int k, int single_phase_recv)
 *                                                             (allreduce_recexch.cpp:188)
 *          MPICH_Allreduce_k_reduce_scatter_allgather(..., int k, int single_phase_recv)
 *                                          (allreduce_k_reduce_scatter_allgather.cpp:257)
 *          MPICH_Allreduce_recursive_multiplying(..., int k)
 *                                              (allreduce_recursive_multiplying.cpp:3)
 * algo is one of CHR_MODE_MPICH_*; k is used by RECEXCH / KRSAG / RMULT, single_phase_recv
 * by RECEXCH / KRSAG (it changes MPICH's receive posting, not the data flow or result).  Same
 * buffer contract as chr_allreduce_radix_batch; results bit-identical to the reference's
 * code on the same inputs, every reduction on the fused HIP kernel. */
int chr_allreduce_mpich(const void* send, void* recv, size_t count, chr_dtype dtype, chr_op op,
                        chr_comm* comm, chr_mode algo, int k, int single_phase_recv);
int chr_allreduce_mpich_async(const void* send, void* recv, size_t count, chr_dtype dtype,
                              chr_op op, chr_comm* comm, chr_mode algo, int k,
                              int single_phase_recv);
int chr_local_allreduce_mpich(chr_local_group* group, const void* const* sends,
                              void* const* recvs, size_t count, chr_dtype dtype, chr_op op,
                              chr_mode algo, int k, int single_phase_recv);

/* ---- MPICH baseline reduce-scatters (the ones testing/mpich_implementations/reduce_scatter/
 * main.cpp benchmarks) ------------------------------------------------------------------------
 * Replace  int MPICH_reduce_scatter_radix(const void* sendbuf, void* recvbuf, MPI_Aint recvcount,
 *            MPI_Datatype, MPI_Op, MPI_Comm, int k)                (reduce_scatter_radix.cpp:204)
 *          MPICH_reduce_scatter_rec_halving(const char*, char*, int count, ...)
 *                                                   (reduce_scatter_recursive_halving.cpp:7)
 *          MPICH_reduce_scatter_rec_doubling(const void*, void*, MPI_Aint recvcount, ...)
 *                                                   (reduce_scatter_recursive_doubling.cpp:10)
 *          MPICH_reduce_scatter_pairwise(const void*, void*, MPI_Aint recvcount, ...)
 *                                                   (reduce_scatter_pairwise.cpp:4)
 * algo is one of CHR_MODE_MPICH_RS_*; k is used by RS_RADIX.  MPI_Reduce_scatter_block semantics:
 * send holds nranks*recvcount elements (recv does, under CHR_IN_PLACE), recv gets block `rank`.
 * Results bit-identical to the reference's code on the same inputs; every reduction on the fused
 * HIP kernel. */
int chr_reduce_scatter_mpich(const void* send, void* recv, size_t recvcount, chr_dtype dtype, chr_op op,
                             chr_comm* comm, chr_mode algo, int k);
int chr_reduce_scatter_mpich_async(const void* send, void* recv, size_t recvcount, chr_dtype dtype,
                                   chr_op op, chr_comm* comm, chr_mode algo, int k);
int chr_local_reduce_scatter_mpich(chr_local_group* group, const void* const* sends,
                                   void* const* recvs, size_t recvcount, chr_dtype dtype, chr_op op,
                                   chr_mode algo, int k);

/* ---- CHiArA's phases as stand-alone collectives ------------------------------------------
 * testing/custom_implementations/work_dir/reduce_scatter/ keeps each phase of the hierarchical
 * reduce-scatter as its own function with a DEBUG_MODE self-test main.  Ranks form nnodes = n / b
 * groups of b (node = rank / b, lane = rank % b); IRC = recvcount * b; nstages = nnodes / b,
 * nu = nnodes % b, niters = nstages + (nu != 0).  Results bit-identical to the reference's code on
 * the same inputs; reductions on the fused HIP kernel, messages RCCL send/recv.
 *
 * Replaces  int intra_reduce_scatter_radix_batch(const void* sendbuf, void* recvbuf,
 *             MPI_Aint recvcount, MPI_Datatype, MPI_Op, MPI_Comm, int k, int b)
 *           (intra_reduce_scatter_radix.cpp:208-541; phase 1 of reduce_scatter_radix_batch.cpp).
 * send: recvcount * n elements (recv under CHR_IN_PLACE); chunk c = send[c * IRC, +IRC).  Per
 * stage s, the group's radix-k recexch reduces chunk s * b + lane over the group into
 * recv[s * IRC, +IRC); the leftover stage's chunk nstages * b + lane only for lanes < nu (recv
 * beyond what a rank writes is left untouched). */
int chr_intra_reduce_scatter_radix_batch(const void* send, void* recv, size_t recvcount, chr_dtype dtype,
                                         chr_op op, chr_comm* comm, int k, int b);
/* Replaces  int inter_reduce_linear(const void* sendbuf, void* recvbuf, MPI_Aint recvcount,
 *             MPI_Datatype, MPI_Op, MPI_Comm, int b)   (inter_linear_reduce.cpp:11-73; phase 2).
 * send: niters chunks of IRC; for iteration i the lane's root node is i * b + lane (if < nnodes):
 * recv[0, IRC) = own chunk i reduced with the other nodes' chunk i in ascending node order.  Ranks
 * that are nobody's root leave recv untouched and may pass NULL (the reference never touches it there).
 * send may not be CHR_IN_PLACE (nor in the reference). */
int chr_inter_reduce_linear(const void* send, void* recv, size_t recvcount, chr_dtype dtype, chr_op op,
                            chr_comm* comm, int b);
/* Replaces  int intra_scatter_radix_batch(char* sendbuf, int recvcount, MPI_Datatype,
 *             char* recvbuf, MPI_Comm, int k, int b)  (intra_scatter_radix_batch.cpp:10-110; RS phase 3).
 * The node root (lane node % b) holds b blocks of recvcount in send; every rank of the node gets
 * block `lane` in recv through a k-nomial tree.  send is read on node roots only (may be NULL
 * elsewhere).  Data movement only: any dtype. */
int chr_intra_scatter_radix_batch(const void* send, size_t recvcount, chr_dtype dtype, void* recv,
                                  chr_comm* comm, int k, int b);
/* All three on virtual ranks (mode = CHR_MODE_INTRA_REDUCE_SCATTER / _INTER_REDUCE_LINEAR /
 * _INTRA_SCATTER; op is unused by the scatter, k by the linear reduce). */
int chr_local_phase_collective(chr_local_group* group, chr_mode mode, const void* const* sends,
                               void* const* recvs, size_t recvcount, chr_dtype dtype, chr_op op, int k,
                               int b);

/* ---- utilities -------------------------------------------------------------------------- */
/* Synthetic inputs on the device with the shared generator (oracle/chiara_oracle.h):
 * pattern 0 = U[-1,1) (random 32-bit ints for INT32), 1 = rank*count_for_seq + i,
 * 2 = ties probe for MAX/MIN ({+0,-0,1,-1,0.5, NaN with per-rank payload}; integers {0,1,-1,2,7}),
 * 3 = sparse (integer types: zero with probability 1/8, else nonzero random bits; floats: as 0).
 * Integer types beyond int32: 0 = random bits of the full width, 1 = rank*count_for_seq + i
 * truncated to the width. */
int chr_fill(void* buf, size_t n, chr_dtype dtype, int pattern, uint64_t seed, int rank,
             uint64_t count_for_seq, hipStream_t stream);
const char* chr_error_string(int code);
int chr_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* CHIARA_H */
