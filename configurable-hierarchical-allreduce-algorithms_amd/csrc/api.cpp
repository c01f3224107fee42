// api.cpp -- C ABI glue for the kernel boundary, plan introspection and utilities.
#include <hip/hip_runtime_api.h>

#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "chr_internal.hpp"
#include "schedule.hpp"
#include "user_ops.hpp"

// The library leaves the process environment alone.  Multi-process GPU work on this driver needs
// dmabuf IPC (HSA_ENABLE_IPC_MODE_LEGACY=0); the entry paths that start ranks set that default
// before any HIP call -- the MPI shim (csrc/shim/chiara_mpi_shim.cpp, for the reference's
// harnesses), this package's own harness mains, the Python package and bench.py -- and
// chr_comm_init_rank warns when a multi-rank communicator starts without it.

extern "C" {

int chr_abi_version(void) { return CHR_ABI_VERSION; }

const char* chr_error_string(int code) {
    switch (code) {
    case CHR_SUCCESS: return "success";
    case CHR_ERR_INVALID_ARG: return "invalid argument";
    case CHR_ERR_COUNT_NOT_DIVISIBLE: return "count is not a multiple of the number of ranks";
    case CHR_ERR_BATCH_NOT_DIVISOR: return "batch b does not divide the number of ranks";
    case CHR_ERR_HIP: return "HIP runtime error";
    case CHR_ERR_RCCL: return "RCCL error";
    case CHR_ERR_NO_DEVICE: return "no HIP device";
    case CHR_ERR_OUT_OF_MEMORY: return "out of device memory";
    case CHR_ERR_UNSUPPORTED: return "unsupported";
    case CHR_ERR_TIMEOUT: return "call timed out; communicator aborted";
    case CHR_ERR_ABORTED: return "communicator aborted by an earlier failure";
    default: return "unknown error";
    }
}

static int status(hipError_t e) {
    if (e == hipSuccess) return CHR_SUCCESS;
    return e == hipErrorOutOfMemory ? CHR_ERR_OUT_OF_MEMORY : CHR_ERR_HIP;
}

int chr_reduce_local(const void* in, void* inout, size_t n, chr_dtype dtype, chr_op op, hipStream_t stream) {
    if (!chr::valid_any(dtype, op)) return CHR_ERR_INVALID_ARG;
    if (n == 0) return CHR_SUCCESS;
    if (!in || !inout) return CHR_ERR_INVALID_ARG;
    const void* ins[1] = {in};
    return chr::reduce_any(inout, inout, ins, 1, n, dtype, op, stream);
}

int chr_reduce_multi(void* out, const void* acc, const void* const* ins, int m, size_t n, chr_dtype dtype, chr_op op,
                     hipStream_t stream) {
    if (!chr::valid_any(dtype, op) || m < 0) return CHR_ERR_INVALID_ARG;
    if (n == 0) return CHR_SUCCESS;
    if (!out || !acc || (m > 0 && !ins)) return CHR_ERR_INVALID_ARG;
    for (int j = 0; j < m; ++j)
        if (!ins[j]) return CHR_ERR_INVALID_ARG;
    return chr::reduce_any(out, acc, ins, m, n, dtype, op, stream);
}

int chr_reduce_multi_ex(void* out, const void* acc, const void* const* ins, int m, size_t n, chr_dtype dtype,
                        chr_op op, int flags, hipStream_t stream) {
    if (!chr::valid_any(dtype, op) || m < 0 || (flags & ~CHR_REDUCE_RUNNING_FIRST)) return CHR_ERR_INVALID_ARG;
    if (n == 0) return CHR_SUCCESS;
    if (!out || !acc || (m > 0 && !ins)) return CHR_ERR_INVALID_ARG;
    for (int j = 0; j < m; ++j)
        if (!ins[j]) return CHR_ERR_INVALID_ARG;
    return chr::reduce_any(out, acc, ins, m, n, dtype, op, stream, (flags & CHR_REDUCE_RUNNING_FIRST) != 0);
}

int chr_reduce_tree(void* out, const void* const* leaves, int nleaves, const unsigned char* comb,
                    const unsigned char* swaps, size_t n, chr_dtype dtype, chr_op op, hipStream_t stream) {
    if (!chr::valid_any(dtype, op) || nleaves < 1 || !comb || !leaves) return CHR_ERR_INVALID_ARG;
    uint32_t cb = 0, sb = 0;
    if (!chr::tree_program_ok(nleaves, comb, swaps, &cb, &sb)) return CHR_ERR_UNSUPPORTED;
    if (n == 0) return CHR_SUCCESS;
    if (!out) return CHR_ERR_INVALID_ARG;
    for (int j = 0; j < nleaves; ++j)
        if (!leaves[j]) return CHR_ERR_INVALID_ARG;
    return chr::reduce_tree_any(out, leaves, nleaves, comb, swaps, n, dtype, op, stream);
}

int chr_reduce_tree_batch(void* const* outs, const void* const* leaves, int ntrees, int nleaves,
                          const unsigned char* comb, const unsigned char* swaps, size_t n, chr_dtype dtype, chr_op op,
                          hipStream_t stream) {
    if (!chr::valid_any(dtype, op) || ntrees < 0 || nleaves < 1 || nleaves > 8) return CHR_ERR_INVALID_ARG;
    if (ntrees > 0 && (!outs || !leaves || !comb)) return CHR_ERR_INVALID_ARG;
    std::vector<chr::TreeJob> jobs((size_t)ntrees);
    for (int t = 0; t < ntrees; ++t) {
        uint32_t cb = 0, sb = 0;
        const unsigned char* sw = swaps ? swaps + (size_t)t * (nleaves - 1) : nullptr;
        if (!chr::tree_program_ok(nleaves, comb + (size_t)t * nleaves, sw, &cb, &sb)) return CHR_ERR_UNSUPPORTED;
        chr::TreeJob& jb = jobs[t];
        jb.out = outs[t];
        jb.nl = nleaves;
        jb.comb = comb + (size_t)t * nleaves;
        jb.swaps = sw;
        jb.n = n;
        if (n && !jb.out) return CHR_ERR_INVALID_ARG;
        for (int j = 0; j < nleaves; ++j) {
            jb.leaves[j] = leaves[(size_t)t * nleaves + j];
            if (n && !jb.leaves[j]) return CHR_ERR_INVALID_ARG;
        }
    }
    if (n == 0 || ntrees == 0) return CHR_SUCCESS;
    return chr::reduce_tree_multi_any(jobs.data(), ntrees, dtype, op, stream);
}

int chr_fill(void* buf, size_t n, chr_dtype dtype, int pattern, uint64_t seed, int rank, uint64_t count_for_seq,
             hipStream_t stream) {
    if (!chr::dtype_size(dtype) || (pattern < 0 || pattern > 3)) return CHR_ERR_INVALID_ARG;
    if (n == 0) return CHR_SUCCESS;
    if (!buf) return CHR_ERR_INVALID_ARG;
    return status(chr::launch_fill(buf, n, dtype, pattern, seed, rank, count_for_seq, stream));
}

long chr_plan_describe(chr_mode mode, int nranks, int rank, int k, int b, size_t count, int slices, char* buf,
                       size_t len) {
    if (mode < CHR_MODE_ALLREDUCE || mode > CHR_MODE_INTRA_SCATTER) return -1;
    return chr_plan_describe_ex(mode, nranks, rank, k, b, count, slices, CHR_SCHEDULE_FLAT, buf, len);
}

long chr_plan_describe_ex(chr_mode mode, int nranks, int rank, int k, int b, size_t count, int slices, int schedule,
                          char* buf, size_t len) {
    return chr_plan_describe_op(mode, nranks, rank, k, b, count, slices, schedule, 1, buf, len);
}

long chr_plan_describe_op(chr_mode mode, int nranks, int rank, int k, int b, size_t count, int slices, int schedule,
                          int commutative, char* buf, size_t len) {
    if (mode < CHR_MODE_ALLREDUCE || mode > CHR_MODE_INTRA_SCATTER) return -1;
    if (!chr::plan_schedule(schedule)) return -1;
    const std::string s = chr::describe(
        chr::build_plan((chr::Mode)mode, nranks, rank, k, b, count, slices, schedule, commutative != 0));
    if (buf && len) {
        const size_t c = s.size() < len - 1 ? s.size() : len - 1;
        std::memcpy(buf, s.data(), c);
        buf[c] = '\0';
    }
    return (long)s.size();
}

}  // extern "C"
