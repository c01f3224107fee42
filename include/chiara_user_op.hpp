/* chiara_user_op.hpp -- a chr_user_reduce_fn (chiara.h) from a device functor: the user-defined op's
 * arithmetic in the caller's own HIP code object, the way MPI_Op_create takes a function.
 *
 *   struct MyOp { __device__ float operator()(float in, float inout) const { return ...; } };  // in o inout
 *   CHR_DEFINE_USER_OP(my_op_launcher, float, MyOp)
 *   ...
 *   chr_op op;
 *   chr_op_create(my_op_launcher, nullptr, 0, &op);
 *   chr_allreduce_radix_batch(send, recv, count, CHR_FLOAT32, op, comm, k, b);
 *
 * The functor follows MPI's user-function convention: f(in, inout) returns the new inout (x o y = f(x, y)).  Build the
 * code object with the flags your arithmetic needs to be reproducible (e.g. -ffp-contract=off). */
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>

#include "chiara.h"

namespace chr_user {

constexpr int kMaxIns = 16;

struct FoldArgs {
    void* out;
    const void* acc;
    const void* ins[kMaxIns];
    int m;
    size_t n;
    int running_first;
};

// out[i] = ins[m-1][i] o ( ... (ins[0][i] o acc[i])), or with running_first (((acc[i] o ins[0][i]) o ...)
template <typename T, typename F>
__global__ void k_fold(FoldArgs a) {
    const F f{};
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
        T v = static_cast<const T*>(a.acc)[i];
        for (int j = 0; j < a.m; ++j) {
            const T x = static_cast<const T*>(a.ins[j])[i];
            v = a.running_first ? f(v, x) : f(x, v);
        }
        static_cast<T*>(a.out)[i] = v;
    }
}

// Fan-in beyond kMaxIns runs as consecutive launches, each continuing from `out`.
template <typename T, typename F>
int launch_fold(void* out, const void* acc, const void* const* ins, int m, size_t n, int running_first,
                hipStream_t stream) {
    if (m < 0) return 1;
    const unsigned block = 256;
    const size_t blocks = (n + block - 1) / block;
    const unsigned grid = (unsigned)(blocks < 4096 ? (blocks ? blocks : 1) : 4096);
    int done = 0;
    const void* cur = acc;
    do {
        FoldArgs a{};
        a.out = out;
        a.acc = cur;
        a.m = m - done < kMaxIns ? m - done : kMaxIns;
        for (int j = 0; j < a.m; ++j) a.ins[j] = ins[done + j];
        a.n = n;
        a.running_first = running_first;
        hipLaunchKernelGGL((k_fold<T, F>), dim3(grid), dim3(block), 0, stream, a);
        if (hipGetLastError() != hipSuccess) return 1;
        done += a.m;
        cur = out;
    } while (done < m);
    return 0;
}

}  // namespace chr_user

/* Defines `extern "C" int name(...)`, a chr_user_reduce_fn for element type T (the dtype argument is not checked:
 * register it for the type it was built for). */
#define CHR_DEFINE_USER_OP(name, T, F)                                                                               \
    extern "C" int name(void* out, const void* acc, const void* const* ins, int m, size_t n, chr_dtype,             \
                        int running_first, hipStream_t stream, void*) {                                           \
        return chr_user::launch_fold<T, F>(out, acc, ins, m, n, running_first, stream);                           \
    }
