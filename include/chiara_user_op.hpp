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
#include <cstdint>

#include "chiara.h"

namespace chr_user {

constexpr int kMaxIns = 16;
#ifndef CHR_USER_FOLD_U
#define CHR_USER_FOLD_U 4
#endif
constexpr int kU = CHR_USER_FOLD_U;  // 16-B vectors per lane per trip of the fold kernel (1, 2, 8: within 2 %)

struct FoldArgs {
    void* out;
    const void* acc;
    const void* ins[kMaxIns];
    int m;
    size_t n;
    int running_first;
    int vec;  // every pointer 16-B aligned: 16-B vector loads and stores
};

// 16 bytes of T (T of 1, 2, 4, 8 or 16 bytes), or one T otherwise
template <typename T>
struct FoldVec {
    static constexpr int kN = (sizeof(T) <= 16 && 16 % sizeof(T) == 0) ? int(16 / sizeof(T)) : 1;
    T e[kN];
};

// out[i] = ins[m-1][i] o ( ... (ins[0][i] o acc[i])), or with running_first (((acc[i] o ins[0][i]) o ...).  Each
// element is read and written by one thread at one index, so `out` may alias `acc`.  HBM-bound streaming: 16-B
// vectors when every pointer allows it, kU of them per lane per trip in chunks of consecutive vectors (measured:
// 5.48 TB/s for m = 1 and 5.58 for m = 3 at 64 MiB against 5.21 / 5.37 for one vector per lane, grid-stride;
// non-temporal loads and stores made no difference, tools/userop_ab.sh), then the scalar tail.
template <typename T, typename F>
__global__ void k_fold(FoldArgs a) {
    using V = FoldVec<T>;
    constexpr int kN = V::kN;
    const F f{};
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t done = 0;
    if (kN > 1 && a.vec) {
        const size_t nv = a.n / kN;
        const V* accv = static_cast<const V*>(a.acc);
        V* outv = static_cast<V*>(a.out);
        // each workgroup takes chunks of kU x blockDim consecutive vectors (a wave's loads coalesced, a chunk's
        // pages shared), every load of a chunk issued before its combines: bytes in flight
        const size_t chunk = (size_t)kU * blockDim.x;
        const size_t nfull = nv / chunk;
        for (size_t c = blockIdx.x; c < nfull; c += gridDim.x) {
            const size_t base = c * chunk + threadIdx.x;
            V r[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) r[u] = accv[base + (size_t)u * blockDim.x];
            for (int j = 0; j < a.m; ++j) {
                const V* inv = static_cast<const V*>(a.ins[j]);
                V x[kU];
#pragma unroll
                for (int u = 0; u < kU; ++u) x[u] = inv[base + (size_t)u * blockDim.x];
#pragma unroll
                for (int u = 0; u < kU; ++u)
#pragma unroll
                    for (int e = 0; e < kN; ++e)
                        r[u].e[e] = a.running_first ? f(r[u].e[e], x[u].e[e]) : f(x[u].e[e], r[u].e[e]);
            }
#pragma unroll
            for (int u = 0; u < kU; ++u) outv[base + (size_t)u * blockDim.x] = r[u];
        }
        for (size_t v = nfull * chunk + tid; v < nv; v += stride) {
            V r = accv[v];
            for (int j = 0; j < a.m; ++j) {
                const V x = static_cast<const V*>(a.ins[j])[v];
#pragma unroll
                for (int e = 0; e < kN; ++e) r.e[e] = a.running_first ? f(r.e[e], x.e[e]) : f(x.e[e], r.e[e]);
            }
            outv[v] = r;
        }
        done = nv * kN;
    }
    for (size_t i = done + tid; i < a.n; i += stride) {
        T r = static_cast<const T*>(a.acc)[i];
        for (int j = 0; j < a.m; ++j) {
            const T x = static_cast<const T*>(a.ins[j])[i];
            r = a.running_first ? f(r, x) : f(x, r);
        }
        static_cast<T*>(a.out)[i] = r;
    }
}

// Fan-in beyond kMaxIns runs as consecutive launches, each continuing from `out`.
template <typename T, typename F>
int launch_fold(void* out, const void* acc, const void* const* ins, int m, size_t n, int running_first,
                hipStream_t stream) {
    if (m < 0) return 1;
    const unsigned block = 256;
    auto aligned = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    bool vec = aligned(out) && aligned(acc);
    for (int j = 0; j < m; ++j) vec = vec && aligned(ins[j]);
    const size_t lanes = vec ? (n / FoldVec<T>::kN + kU - 1) / kU + n % FoldVec<T>::kN : n;
    const size_t blocks = (lanes + block - 1) / block;
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
        a.vec = vec ? 1 : 0;
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

/* The same for one chr_dtype: a call on any other type is refused (the library returns CHR_ERR_UNSUPPORTED), as an
 * MPI user function may reject a datatype it does not implement. */
#define CHR_DEFINE_USER_OP_FOR(name, T, F, DTYPE)                                                                     \
    extern "C" int name(void* out, const void* acc, const void* const* ins, int m, size_t n, chr_dtype dt,          \
                        int running_first, hipStream_t stream, void*) {                                           \
        if (dt != (DTYPE)) return 1;                                                                                 \
        return chr_user::launch_fold<T, F>(out, acc, ins, m, n, running_first, stream);                           \
    }
