// chiara_mpi_shim.cpp -- the reference-side binding: CHiArA's own entry points, same
// C++ signatures, implemented on libchiara.  Linking this file instead of
// all_reduce_radix_batch.cpp / reduce_scatter_radix_batch.cpp makes the reference's
// harnesses (Fugaku_experiments/{Allreduce,Reduce-scatter}/main.cpp) drive the MI355X path
// unchanged.
//
//   int all_reduce_radix_batch(char*, char*, int, MPI_Datatype, MPI_Op, MPI_Comm, int k, int b)
//       replaces Fugaku_experiments/Allreduce/all_reduce_radix_batch.cpp:202-204
//   int reduce_scatter_radix_batch(const void*, void*, MPI_Aint, MPI_Datatype, MPI_Op, MPI_Comm, int, int)
//       replaces Fugaku_experiments/Reduce-scatter/reduce_scatter_radix_batch.cpp:200-202
//   int allgather_radix_batch(char*, int, MPI_Datatype, char*, MPI_Comm, int k, int b)
//       replaces Fugaku_experiments/Allgather/all_gather_radix_batch_1_0.cpp:37
//   MPICH_Allreduce_{ring, recursive_doubling, reduce_scatter_allgather, recursive_exchange,
//                    k_reduce_scatter_allgather, recursive_multiplying}
//       replace testing/mpich_implementations/all_reduce/allreduce_{ring.cpp:3,
//       recursive_doubling.cpp:4, reduce_scatter_allgather.cpp:3, recexch.cpp:188,
//       k_reduce_scatter_allgather.cpp:257, recursive_multiplying.cpp:3}: all six baselines
//       testing/main.cpp times, so that harness links against libchiara unchanged
//   MPICH_reduce_scatter_{radix, rec_halving, rec_doubling, pairwise}
//       replace testing/mpich_implementations/reduce_scatter/reduce_scatter_{radix.cpp:204,
//       recursive_halving.cpp:7, recursive_doubling.cpp:10, pairwise.cpp:4}: the baselines that
//       directory's main.cpp times
//   intra_reduce_scatter_radix_batch, inter_reduce_linear, intra_scatter_radix_batch
//       replace testing/custom_implementations/work_dir/reduce_scatter/{intra_reduce_scatter_radix.cpp:208,
//       inter_linear_reduce.cpp:11, intra_scatter_radix_batch.cpp:10}: CHiArA's phases as stand-alone
//       functions, so their DEBUG_MODE self-test mains run on libchiara
//
// One chr_comm per MPI communicator, created on first use (RCCL unique id broadcast with
// MPI_Bcast, device = node-local rank mod visible GPUs) and cached as an MPI attribute.
// Buffers are the reference's host buffers: libchiara stages them through HBM.
//
// User-defined ops: MPI_Op_create's function is host code the device cannot call.  A caller that has the same
// arithmetic as device code (a chr_user_reduce_fn, include/chiara_user_op.hpp) binds it to its MPI_Op once,
//   chiara_shim_op_bind(op, launcher, ctx)      (commutativity from MPI_Op_commutative, as the reference reads it)
// and every entry point below then takes that MPI_Op; an unbound user op stays MPI_ERR_OP.  A baseline that refuses
// a non-commutative op returns MPI_ERR_OP, as the reference's do.
//
// CHR_SHIM_TRACE=1: at exit, every process writes one line to stderr,
//   [chiara-shim] rank R calls: <entry point>=<count> ...
// the positive marker that a reference main really ran these definitions (and not its own file's
// function, which the self-test builds only weaken: oracle/selftests.sh).
#include <mpi.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "chiara.h"

namespace {

// Multi-process GPU work on this driver needs dmabuf IPC: without HSA_ENABLE_IPC_MODE_LEGACY=0,
// RCCL's P2P/IPC transport between the ranks of one node fails in hipIpcGetMemHandle.  The
// reference's harnesses reach libchiara through this shim with whatever environment mpiexec gives
// them (Fugaku_experiments/Allreduce/main.cpp:111-113), so the shim -- linked into the harness
// executable -- sets the default at program load, before main and so before any thread or HIP
// call.  A value the caller set is kept.
__attribute__((constructor)) void shim_default_ipc_mode() { setenv("HSA_ENABLE_IPC_MODE_LEGACY", "0", 0); }

int g_keyval = MPI_KEYVAL_INVALID;

// Call counts for CHR_SHIM_TRACE (plain arrays: read by an atexit handler, after which no static
// destructor may have run first).  Not synchronised: the reference's harnesses call the collectives
// from one thread per rank (MPI_Init, not MPI_Init_thread).
constexpr int kMaxTraced = 32;
const char* g_trace_name[kMaxTraced];
long g_trace_count[kMaxTraced];
int g_trace_n = 0, g_trace_rank = -1;

void trace_report() {
    std::fprintf(stderr, "[chiara-shim] rank %d calls:", g_trace_rank);
    for (int i = 0; i < g_trace_n; ++i) std::fprintf(stderr, " %s=%ld", g_trace_name[i], g_trace_count[i]);
    std::fprintf(stderr, "\n");
    std::fflush(stderr);
}

void trace(const char* fn) {
    static const bool on = [] {
        const char* e = std::getenv("CHR_SHIM_TRACE");
        return e && std::atoi(e) != 0;
    }();
    if (!on) return;
    if (g_trace_rank < 0) {
        int init = 0, r = 0;
        MPI_Initialized(&init);
        if (init) MPI_Comm_rank(MPI_COMM_WORLD, &r);
        g_trace_rank = r;
        std::atexit(trace_report);
    }
    for (int i = 0; i < g_trace_n; ++i)
        if (std::strcmp(g_trace_name[i], fn) == 0) {
            ++g_trace_count[i];
            return;
        }
    if (g_trace_n < kMaxTraced) {
        g_trace_name[g_trace_n] = fn;
        g_trace_count[g_trace_n++] = 1;
    }
}

int delete_comm(MPI_Comm, int, void* attr, void*) {
    chr_comm_destroy(static_cast<chr_comm*>(attr));
    return MPI_SUCCESS;
}

chr_comm* comm_for(MPI_Comm mc) {
    if (g_keyval == MPI_KEYVAL_INVALID)
        MPI_Comm_create_keyval(MPI_COMM_NULL_COPY_FN, delete_comm, &g_keyval, nullptr);
    void* attr = nullptr;
    int found = 0;
    MPI_Comm_get_attr(mc, g_keyval, &attr, &found);
    if (found) return static_cast<chr_comm*>(attr);
    int rank, n, lrank, ndev = 0;
    MPI_Comm_rank(mc, &rank);
    MPI_Comm_size(mc, &n);
    MPI_Comm local;
    MPI_Comm_split_type(mc, MPI_COMM_TYPE_SHARED, rank, MPI_INFO_NULL, &local);
    MPI_Comm_rank(local, &lrank);
    MPI_Comm_free(&local);
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return nullptr;
    chr_unique_id id;
    if (rank == 0) chr_get_unique_id(&id);
    MPI_Bcast(&id, sizeof(id), MPI_BYTE, 0, mc);
    chr_comm* c = nullptr;
    if (chr_comm_init_rank(&c, n, &id, rank, lrank % ndev) != CHR_SUCCESS) return nullptr;
    // The MPI signatures' contract is host memory on every rank (the reference harness mallocs
    // its buffers), which is what pipelined host staging needs: on by default here, 32 MiB windows
    // per rank, unless CHR_HOST_WINDOW_MIB says otherwise.
    if (!std::getenv("CHR_HOST_WINDOW_MIB")) chr_comm_set_host_pipeline(c, 32);
    MPI_Comm_set_attr(mc, g_keyval, c);
    return c;
}

// MPI predefined types -> element types.  The reference is generic over MPI_Datatype (sizes from
// MPI_Type_size, all_reduce_radix_batch.cpp:234-277); its arithmetic is MPICH's predefined-op loop
// for the pair.  C integer types map by size and signedness (MPI_LONG is 64-bit on this LP64
// platform); MPI_CHAR reduces as a signed char, as in MPICH.  MPI_BYTE takes the bitwise ops and
// MPI_C_BOOL the logical ones (checked in map_pair).  The MAXLOC / MINLOC pair types and the C
// complex types are supported; everything else -- MPI_LONG_DOUBLE and its pair / complex types,
// derived types -- is MPI_ERR_TYPE.
bool map_type(MPI_Datatype d, chr_dtype* out) {
    if (d == MPI_FLOAT) *out = CHR_FLOAT32;
    else if (d == MPI_DOUBLE) *out = CHR_FLOAT64;
    else if (d == MPI_INT || d == MPI_INT32_T) *out = CHR_INT32;
    else if (d == MPI_UNSIGNED || d == MPI_UINT32_T) *out = CHR_UINT32;
    else if (d == MPI_SIGNED_CHAR || d == MPI_INT8_T || d == MPI_CHAR) *out = CHR_INT8;
    else if (d == MPI_UNSIGNED_CHAR || d == MPI_UINT8_T || d == MPI_BYTE || d == MPI_C_BOOL) *out = CHR_UINT8;
    else if (d == MPI_SHORT || d == MPI_INT16_T) *out = CHR_INT16;
    else if (d == MPI_UNSIGNED_SHORT || d == MPI_UINT16_T) *out = CHR_UINT16;
    else if (d == MPI_LONG || d == MPI_LONG_LONG || d == MPI_LONG_LONG_INT || d == MPI_INT64_T)
        *out = sizeof(long) == 8 || d != MPI_LONG ? CHR_INT64 : CHR_INT32;
    else if (d == MPI_UNSIGNED_LONG || d == MPI_UNSIGNED_LONG_LONG || d == MPI_UINT64_T)
        *out = sizeof(unsigned long) == 8 || d != MPI_UNSIGNED_LONG ? CHR_UINT64 : CHR_UINT32;
    // MAXLOC / MINLOC pair types (the C structs MPI defines; element stride = MPI's extent) and the
    // C complex types
    else if (d == MPI_FLOAT_INT) *out = CHR_FLOAT_INT;
    else if (d == MPI_DOUBLE_INT) *out = CHR_DOUBLE_INT;
    else if (d == MPI_LONG_INT && sizeof(long) == 8) *out = CHR_LONG_INT;
    else if (d == MPI_2INT) *out = CHR_2INT;
    else if (d == MPI_SHORT_INT) *out = CHR_SHORT_INT;
    else if (d == MPI_C_FLOAT_COMPLEX || d == MPI_C_COMPLEX) *out = CHR_C_FLOAT_COMPLEX;
    else if (d == MPI_C_DOUBLE_COMPLEX) *out = CHR_C_DOUBLE_COMPLEX;
    else return false;
    return true;
}

// User ops bound to a device launcher (chiara_shim_op_bind): MPI_Op handle -> chr_op code.
constexpr int kMaxBound = 64;
struct BoundOp {
    MPI_Op mpi;
    chr_op op;
};
BoundOp g_bound[kMaxBound];
int g_nbound = 0;

bool bound_op(MPI_Op o, chr_op* out) {
    for (int i = 0; i < g_nbound; ++i)
        if (g_bound[i].mpi == o) {
            *out = g_bound[i].op;
            return true;
        }
    return false;
}

// MPI predefined ops.  MPI_REPLACE/NO_OP and unbound user ops (MPI_Op_create: a host function pointer
// the device cannot call) are MPI_ERR_OP.
bool map_op(MPI_Op o, chr_op* out) {
    if (o == MPI_SUM) *out = CHR_SUM;
    else if (o == MPI_PROD) *out = CHR_PROD;
    else if (o == MPI_MAX) *out = CHR_MAX;
    else if (o == MPI_MIN) *out = CHR_MIN;
    else if (o == MPI_LAND) *out = CHR_LAND;
    else if (o == MPI_LOR) *out = CHR_LOR;
    else if (o == MPI_LXOR) *out = CHR_LXOR;
    else if (o == MPI_BAND) *out = CHR_BAND;
    else if (o == MPI_BOR) *out = CHR_BOR;
    else if (o == MPI_BXOR) *out = CHR_BXOR;
    else if (o == MPI_MAXLOC) *out = CHR_MAXLOC;
    else if (o == MPI_MINLOC) *out = CHR_MINLOC;
    else return false;
    return true;
}

// MPI's op/type table as MPICH 3.3.2 applies it (probed with MPI_Reduce_local): MPI_BYTE only with
// the bitwise ops, MPI_C_BOOL only with the logical ops, float/double with the logical ops (an MPICH
// extension of MPI-3.1 §5.9.2) but not the bitwise ones; 0 or the MPI error class to return.
int map_pair(MPI_Datatype d, MPI_Op o, chr_dtype* dt, chr_op* op) {
    if (!map_type(d, dt)) return MPI_ERR_TYPE;
    if (bound_op(o, op)) return 0;  // a user op: its launcher decides which types it implements
    if (!map_op(o, op)) return MPI_ERR_OP;
    const bool bitwise = *op == CHR_BAND || *op == CHR_BOR || *op == CHR_BXOR;
    const bool logical = *op == CHR_LAND || *op == CHR_LOR || *op == CHR_LXOR;
    if (d == MPI_BYTE && !bitwise) return MPI_ERR_OP;
    if (d == MPI_C_BOOL && !logical) return MPI_ERR_OP;
    if ((*dt == CHR_FLOAT32 || *dt == CHR_FLOAT64) && bitwise) return MPI_ERR_OP;
    // MAXLOC / MINLOC only on the pair types, which take nothing else; complex takes SUM / PROD only
    const bool loc = *op == CHR_MAXLOC || *op == CHR_MINLOC;
    const bool pair = *dt >= CHR_FLOAT_INT && *dt <= CHR_SHORT_INT;
    const bool cplx = *dt == CHR_C_FLOAT_COMPLEX || *dt == CHR_C_DOUBLE_COMPLEX;
    if (loc != pair) return MPI_ERR_OP;
    if (cplx && *op != CHR_SUM && *op != CHR_PROD) return MPI_ERR_OP;
    return 0;
}

int to_mpi(int rc) {
    if (rc == CHR_SUCCESS) return MPI_SUCCESS;
    if (rc == CHR_ERR_COUNT_NOT_DIVISIBLE) return MPI_ERR_COUNT;
    if (rc == CHR_ERR_BATCH_NOT_DIVISOR || rc == CHR_ERR_INVALID_ARG) return MPI_ERR_ARG;
    if (rc == CHR_ERR_UNSUPPORTED) return MPI_ERR_OP;  // a user op refused (by its launcher, or a baseline)
    return MPI_ERR_OTHER;  // HIP / RCCL errors, timeouts and aborted communicators
}

}  // namespace

// Binds a user-defined MPI_Op to the device launcher with its arithmetic (chr_op_create, with MPI_Op_commutative's
// answer as `commute`).  Binding the same MPI_Op again replaces the launcher.  MPI_SUCCESS, or MPI_ERR_OP.
extern "C" int chiara_shim_op_bind(MPI_Op op, chr_user_reduce_fn fn, void* ctx) {
    chr_op code;
    if (!fn || op == MPI_OP_NULL || map_op(op, &code)) return MPI_ERR_OP;  // predefined ops stay the library's
    int commute = 0;
    if (MPI_Op_commutative(op, &commute) != MPI_SUCCESS) return MPI_ERR_OP;
    if (chr_op_create(fn, ctx, commute, &code) != CHR_SUCCESS) return MPI_ERR_OP;
    for (int i = 0; i < g_nbound; ++i)
        if (g_bound[i].mpi == op) {
            chr_op_free(g_bound[i].op);
            g_bound[i].op = code;
            return MPI_SUCCESS;
        }
    if (g_nbound == kMaxBound) {
        chr_op_free(code);
        return MPI_ERR_OP;
    }
    g_bound[g_nbound++] = {op, code};
    return MPI_SUCCESS;
}

// Drops a binding (before MPI_Op_free); the MPI_Op is MPI_ERR_OP again.
extern "C" int chiara_shim_op_unbind(MPI_Op op) {
    for (int i = 0; i < g_nbound; ++i)
        if (g_bound[i].mpi == op) {
            chr_op_free(g_bound[i].op);
            g_bound[i] = g_bound[--g_nbound];
            return MPI_SUCCESS;
        }
    return MPI_ERR_OP;
}

int all_reduce_radix_batch(char* sendbuf, char* recvbuf, int count, MPI_Datatype datatype, MPI_Op op,
                           MPI_Comm comm, int k, int b) {
    trace(__func__);
    chr_dtype dt;
    chr_op o;
    if (int err = map_pair(datatype, op, &dt, &o)) return err;
    chr_comm* c = comm_for(comm);
    if (!c) return MPI_ERR_OTHER;
    const void* send = sendbuf == (char*)MPI_IN_PLACE ? CHR_IN_PLACE : (const void*)sendbuf;
    return to_mpi(chr_allreduce_radix_batch(send, recvbuf, (size_t)count, dt, o, c, k, b));
}

int reduce_scatter_radix_batch(const void* sendbuf, void* recvbuf, MPI_Aint recvcount, MPI_Datatype datatype,
                               MPI_Op op, MPI_Comm comm, int k, int b) {
    trace(__func__);
    chr_dtype dt;
    chr_op o;
    if (int err = map_pair(datatype, op, &dt, &o)) return err;
    chr_comm* c = comm_for(comm);
    if (!c) return MPI_ERR_OTHER;
    const void* send = sendbuf == MPI_IN_PLACE ? CHR_IN_PLACE : sendbuf;
    return to_mpi(chr_reduce_scatter_radix_batch(send, recvbuf, (size_t)recvcount, dt, o, c, k, b));
}

namespace {

int mpich_call(chr_mode algo, const char* sendbuf, char* recvbuf, int count, MPI_Datatype datatype, MPI_Op op,
               MPI_Comm comm, int k, int single_phase_recv) {
    chr_dtype dt;
    chr_op o;
    if (int err = map_pair(datatype, op, &dt, &o)) return err;
    if (count < 0) return MPI_ERR_COUNT;
    chr_comm* c = comm_for(comm);
    if (!c) return MPI_ERR_OTHER;
    const void* send = sendbuf == (const char*)MPI_IN_PLACE ? CHR_IN_PLACE : (const void*)sendbuf;
    return to_mpi(chr_allreduce_mpich(send, recvbuf, (size_t)count, dt, o, c, algo, k, single_phase_recv));
}

}  // namespace

int MPICH_Allreduce_ring(const char* sendbuf, char* recvbuf, int count, MPI_Datatype datatype, MPI_Op op,
                         MPI_Comm comm) {
    trace(__func__);
    return mpich_call(CHR_MODE_MPICH_RING, sendbuf, recvbuf, count, datatype, op, comm, 0, 0);
}

int MPICH_Allreduce_recursive_doubling(const char* sendbuf, char* recvbuf, int count, MPI_Datatype datatype,
                                       MPI_Op op, MPI_Comm comm) {
    trace(__func__);
    return mpich_call(CHR_MODE_MPICH_RD, sendbuf, recvbuf, count, datatype, op, comm, 0, 0);
}

int MPICH_Allreduce_reduce_scatter_allgather(const char* sendbuf, char* recvbuf, int count, MPI_Datatype datatype,
                                             MPI_Op op, MPI_Comm comm) {
    trace(__func__);
    return mpich_call(CHR_MODE_MPICH_RSAG, sendbuf, recvbuf, count, datatype, op, comm, 0, 0);
}

int MPICH_Allreduce_recursive_exchange(const char* sendbuf, char* recvbuf, int count, MPI_Datatype datatype,
                                       MPI_Op op, MPI_Comm comm, int k, int single_phase_recv) {
    trace(__func__);
    return mpich_call(CHR_MODE_MPICH_RECEXCH, sendbuf, recvbuf, count, datatype, op, comm, k, single_phase_recv);
}

int MPICH_Allreduce_k_reduce_scatter_allgather(const char* sendbuf, char* recvbuf, int count, MPI_Datatype datatype,
                                               MPI_Op op, MPI_Comm comm, int k, int single_phase_recv) {
    trace(__func__);
    return mpich_call(CHR_MODE_MPICH_KRSAG, sendbuf, recvbuf, count, datatype, op, comm, k, single_phase_recv);
}

int MPICH_Allreduce_recursive_multiplying(const char* sendbuf, char* recvbuf, int count, MPI_Datatype datatype,
                                          MPI_Op op, MPI_Comm comm, int k) {
    trace(__func__);
    return mpich_call(CHR_MODE_MPICH_RMULT, sendbuf, recvbuf, count, datatype, op, comm, k, 0);
}

// Pure data movement: any datatype the reference accepts (all_gather_radix_batch_1_0.cpp:37 sizes
// it with MPI_Type_size), moved as bytes; contiguous layouts only (MPI_Type_size == extent).
int allgather_radix_batch(char* sendbuf, int sendcount, MPI_Datatype datatype, char* recvbuf, MPI_Comm comm, int k,
                          int b) {
    trace(__func__);
    if (sendcount < 0) return MPI_ERR_COUNT;
    int tsize = 0;
    MPI_Aint lb = 0, extent = 0;
    if (MPI_Type_size(datatype, &tsize) != MPI_SUCCESS || MPI_Type_get_extent(datatype, &lb, &extent) != MPI_SUCCESS ||
        tsize <= 0 || lb != 0 || extent != tsize)
        return MPI_ERR_TYPE;
    chr_comm* c = comm_for(comm);
    if (!c) return MPI_ERR_OTHER;
    const void* send = sendbuf == (char*)MPI_IN_PLACE ? CHR_IN_PLACE : (const void*)sendbuf;
    return to_mpi(chr_allgather_radix_batch(send, (size_t)sendcount * (size_t)tsize, CHR_UINT8, recvbuf, c, k, b));
}

namespace {

int mpich_rs_call(chr_mode algo, const void* sendbuf, void* recvbuf, long long recvcount, MPI_Datatype datatype,
                  MPI_Op op, MPI_Comm comm, int k) {
    chr_dtype dt;
    chr_op o;
    if (int err = map_pair(datatype, op, &dt, &o)) return err;
    if (recvcount < 0) return MPI_ERR_COUNT;
    chr_comm* c = comm_for(comm);
    if (!c) return MPI_ERR_OTHER;
    const void* send = sendbuf == MPI_IN_PLACE ? CHR_IN_PLACE : sendbuf;
    return to_mpi(chr_reduce_scatter_mpich(send, recvbuf, (size_t)recvcount, dt, o, c, algo, k));
}

}  // namespace

int MPICH_reduce_scatter_radix(const void* sendbuf, void* recvbuf, MPI_Aint recvcount, MPI_Datatype datatype,
                               MPI_Op op, MPI_Comm comm, int k) {
    trace(__func__);
    return mpich_rs_call(CHR_MODE_MPICH_RS_RADIX, sendbuf, recvbuf, recvcount, datatype, op, comm, k);
}

int MPICH_reduce_scatter_rec_halving(const char* sendbuf, char* recvbuf, int count, MPI_Datatype datatype, MPI_Op op,
                                     MPI_Comm comm) {
    trace(__func__);
    return mpich_rs_call(CHR_MODE_MPICH_RS_HALVING, sendbuf, recvbuf, count, datatype, op, comm, 0);
}

int MPICH_reduce_scatter_rec_doubling(const void* sendbuf, void* recvbuf, MPI_Aint recvcount, MPI_Datatype datatype,
                                      MPI_Op op, MPI_Comm comm) {
    trace(__func__);
    return mpich_rs_call(CHR_MODE_MPICH_RS_DOUBLING, sendbuf, recvbuf, recvcount, datatype, op, comm, 0);
}

int MPICH_reduce_scatter_pairwise(const void* sendbuf, void* recvbuf, MPI_Aint recvcount, MPI_Datatype datatype,
                                  MPI_Op op, MPI_Comm comm) {
    trace(__func__);
    return mpich_rs_call(CHR_MODE_MPICH_RS_PAIRWISE, sendbuf, recvbuf, recvcount, datatype, op, comm, 0);
}

// CHiArA's phases as stand-alone functions (testing/custom_implementations/work_dir/reduce_scatter/)
int intra_reduce_scatter_radix_batch(const void* sendbuf, void* recvbuf, MPI_Aint recvcount, MPI_Datatype datatype,
                                     MPI_Op op, MPI_Comm comm, int k, int b) {
    trace(__func__);
    chr_dtype dt;
    chr_op o;
    if (int err = map_pair(datatype, op, &dt, &o)) return err;
    if (recvcount < 0) return MPI_ERR_COUNT;
    chr_comm* c = comm_for(comm);
    if (!c) return MPI_ERR_OTHER;
    const void* send = sendbuf == MPI_IN_PLACE ? CHR_IN_PLACE : sendbuf;
    return to_mpi(chr_intra_reduce_scatter_radix_batch(send, recvbuf, (size_t)recvcount, dt, o, c, k, b));
}

int inter_reduce_linear(const void* sendbuf, void* recvbuf, MPI_Aint recvcount, MPI_Datatype datatype, MPI_Op op,
                        MPI_Comm comm, int b) {
    trace(__func__);
    chr_dtype dt;
    chr_op o;
    if (int err = map_pair(datatype, op, &dt, &o)) return err;
    if (recvcount < 0) return MPI_ERR_COUNT;
    chr_comm* c = comm_for(comm);
    if (!c) return MPI_ERR_OTHER;
    return to_mpi(chr_inter_reduce_linear(sendbuf, recvbuf, (size_t)recvcount, dt, o, c, b));
}

// Data movement only: any contiguous type, moved as bytes (as allgather_radix_batch).  Non-roots may
// pass a NULL sendbuf (the reference's self-test does, intra_scatter_radix_batch.cpp:213).
int intra_scatter_radix_batch(char* sendbuf, int recvcount, MPI_Datatype datatype, char* recvbuf, MPI_Comm comm, int k,
                              int b) {
    trace(__func__);
    if (k < 2 || b <= 0) return MPI_SUCCESS;  // the reference's no-op (intra_scatter_radix_batch.cpp:24)
    if (recvcount < 0) return MPI_ERR_COUNT;
    int tsize = 0;
    MPI_Aint lb = 0, extent = 0;
    if (MPI_Type_size(datatype, &tsize) != MPI_SUCCESS || MPI_Type_get_extent(datatype, &lb, &extent) != MPI_SUCCESS ||
        tsize <= 0 || lb != 0 || extent != tsize)
        return MPI_ERR_TYPE;
    chr_comm* c = comm_for(comm);
    if (!c) return MPI_ERR_OTHER;
    return to_mpi(chr_intra_scatter_radix_batch(sendbuf, (size_t)recvcount * (size_t)tsize, CHR_UINT8, recvbuf, c, k, b));
}
