// reduce_tree.hip -- fused expression-tree reduction for gfx950 (one HBM pass per chunk).
#include <hip/hip_runtime.h>

#include "reduce_common.hpp"

namespace chr {

// ---- fused expression tree: one HBM pass for a whole chunk's reduction ---------------------
//
// The flat schedule (schedule.cpp build_plan_flat) evaluates, per chunk, the expression
// tree the reference builds across its phases: recexch folds (all_reduce_radix_batch.cpp
// :364 / :446), step-1 folds (:332) and the lane reduction (:529).  As separate launches every
// inner node is written to HBM and read back; here the whole tree is evaluated in registers,
// so one launch reads each leaf once and writes the root once: (NL + 1) * n * sizeof(T)
// bytes instead of sum over nodes of (m + 2) * n * sizeof(T) (C4's 8-leaf tree: 9 vs 13).
//
// Program: a stack machine in post-order.  Leaves arrive in the order they are pushed;
// after pushing leaf j, comb_j binary combines follow (2 bits per leaf).  A combine pops
// the top (the next operand `in` of a left fold) into the value below it (the fold's running
// value): below = OP(in, below), i.e. MPI_Reduce_local(in, below); with the combine's swap
// bit set the running value is the `in` of MPI_Reduce_local (MPICH_do_reduce order).
// The stack depth is uniform across the grid, so every stack access is a scalar branch over
// static register slots (no scratch).  Depth <= kTreeDepth, leaves <= kMaxLeaves.
constexpr int kMaxLeaves = 8;
constexpr int kTreeDepth = 4;

struct TreeArgs {
    u32x4* out;
    const u32x4* leaves[kMaxLeaves];
    size_t nvec;
    int nl;
    uint32_t comb;   // 2 bits per leaf
    uint32_t swaps;  // 1 bit per combine, in program order
};

template <int OP>
constexpr int swapped_op() {
    return OP == CHR_MAX ? kMaxSw : OP == CHR_MIN ? kMinSw : OP;
}

// Generic over the value carried per lane (W values of type V, combined with F).  The stack
// slots are four named values per w, never an array: an array indexed by the runtime depth
// would be merged into dynamically addressed scratch; named values stay in registers
// (pushes become v_cndmask with a scalar condition, combines scalar branches).
template <typename V, int NL, int W, typename F>
__device__ __forceinline__ void tree_eval(const V (&x)[NL][W], V (&r)[W], uint32_t comb, uint32_t swaps) {
#pragma unroll
    for (int w = 0; w < W; ++w) {
        V s0 = x[0][w], s1 = s0, s2 = s0, s3 = s0;  // leaf 0 is pushed first, comb[0] == 0
        int d = 1, ci = 0;
#pragma unroll
        for (int j = 1; j < NL; ++j) {
            const V v = x[j][w];
            if (d == 1) s1 = v;
            else if (d == 2) s2 = v;
            else s3 = v;
            ++d;
            for (int c = (int)((comb >> (2 * j)) & 3u); c > 0; --c, ++ci) {
                const bool sw = (swaps >> ci) & 1u;
                if (d == 2) s0 = sw ? F::template ap<true>(s1, s0) : F::template ap<false>(s1, s0);
                else if (d == 3) s1 = sw ? F::template ap<true>(s2, s1) : F::template ap<false>(s2, s1);
                else s2 = sw ? F::template ap<true>(s3, s2) : F::template ap<false>(s3, s2);
                --d;
            }
        }
        r[w] = s0;
    }
}

template <int DT, int OP>
struct VecOp {
    template <bool SW>
    __device__ __forceinline__ static u32x4 ap(u32x4 in, u32x4 run) {
        if constexpr (SW && DT != CHR_INT32) return apply_vec<DT, swapped_op<OP>()>(in, run);
        else return apply_vec<DT, OP>(in, run);
    }
};

template <int DT, int OP>
struct ScalarOp {
    using T = typename DTy<DT>::T;
    template <bool SW>
    __device__ __forceinline__ static T ap(T in, T run) {
        if constexpr (SW && DT != CHR_INT32) return apply<DT, swapped_op<OP>()>(in, run);
        else return apply<DT, OP>(in, run);
    }
};

// U vectors per lane per trip for NL leaves: every leaf load of the trip is issued before
// the first combine (NL * U <= 16 loads of 16 B in flight per lane).
template <int DT, int OP, int NL, int U, bool NT, int BL>
__global__ __launch_bounds__(BL) void k_reduce_tree(TreeArgs a) {
    const size_t stride = (size_t)gridDim.x * BL * U;
    for (size_t base = (size_t)blockIdx.x * BL * U + threadIdx.x; base < a.nvec; base += stride) {
        if (base + (size_t)(U - 1) * BL < a.nvec) {
            u32x4 x[NL][U];
#pragma unroll
            for (int j = 0; j < NL; ++j)
#pragma unroll
                for (int u = 0; u < U; ++u) x[j][u] = ld<NT>(&a.leaves[j][base + (size_t)u * BL]);
            __builtin_amdgcn_sched_barrier(0);
            u32x4 r[U];
            tree_eval<u32x4, NL, U, VecOp<DT, OP>>(x, r, a.comb, a.swaps);
#pragma unroll
            for (int u = 0; u < U; ++u) st<NT>(&a.out[base + (size_t)u * BL], r[u]);
        } else {
            for (int u = 0; u < U; ++u) {
                const size_t i = base + (size_t)u * BL;
                if (i >= a.nvec) break;
                u32x4 x[NL][1];
#pragma unroll
                for (int j = 0; j < NL; ++j) x[j][0] = a.leaves[j][i];
                u32x4 r[1];
                tree_eval<u32x4, NL, 1, VecOp<DT, OP>>(x, r, a.comb, a.swaps);
                a.out[i] = r[0];
            }
        }
    }
}

struct TreeScalarArgs {
    void* out;
    const void* leaves[kMaxLeaves];
    size_t n;
    int nl;
    uint32_t comb, swaps;
};

template <int DT, int OP, int NL>
__global__ __launch_bounds__(kBlock) void k_reduce_tree_scalar(TreeScalarArgs a) {
    using T = typename DTy<DT>::T;
    for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < a.n; i += (size_t)gridDim.x * kBlock) {
        T x[NL][1];
#pragma unroll
        for (int j = 0; j < NL; ++j) x[j][0] = ((const T*)a.leaves[j])[i];
        T r[1];
        tree_eval<T, NL, 1, ScalarOp<DT, OP>>(x, r, a.comb, a.swaps);
        ((T*)a.out)[i] = r[0];
    }
}

template <int DT, int OP, int NL, int BL>
static hipError_t launch_tree_vec(const TreeArgs& a, bool nt, hipStream_t s) {
    constexpr int U = NL <= 4 ? 4 : 2;
    const size_t trips = (a.nvec + (size_t)BL * U - 1) / ((size_t)BL * U);
    const size_t cap = reduce_tuning().max_blocks > 0 ? (size_t)reduce_tuning().max_blocks : trips;
    const int grid = (int)(trips < cap ? trips : cap);
    if (nt) hipLaunchKernelGGL((k_reduce_tree<DT, OP, NL, U, true, BL>), dim3(grid), dim3(BL), 0, s, a);
    else hipLaunchKernelGGL((k_reduce_tree<DT, OP, NL, U, false, BL>), dim3(grid), dim3(BL), 0, s, a);
    return hipGetLastError();
}

template <int DT, int OP, int NL>
static hipError_t launch_tree_nl(const TreeArgs& a, const TreeScalarArgs* sa, hipStream_t s) {
    if (sa) {
        const size_t trips = (sa->n + kBlock - 1) / kBlock;
        const int grid = (int)(trips < 2048 ? trips : 2048);
        hipLaunchKernelGGL((k_reduce_tree_scalar<DT, OP, NL>), dim3(grid), dim3(kBlock), 0, s, *sa);
        return hipGetLastError();
    }
    // same policy as launch_vec_m: streaming calls (>= 128 MiB) nt with one-wave workgroups
    const ReduceTuning& t = reduce_tuning();
    const size_t call_bytes = (size_t)(a.nl + 1) * a.nvec * 16;
    const bool nt = t.nt_mode == 1 || (t.nt_mode < 0 && call_bytes >= t.nt_min_bytes);
    const int bl = t.block ? t.block : nt ? 64 : 256;
    return bl == 64 ? launch_tree_vec<DT, OP, NL, 64>(a, nt, s) : launch_tree_vec<DT, OP, NL, 256>(a, nt, s);
}

template <int DT, int OP>
static hipError_t launch_tree_op(const TreeArgs& a, const TreeScalarArgs* sa, hipStream_t s) {
    switch (sa ? sa->nl : a.nl) {
    case 2: return launch_tree_nl<DT, OP, 2>(a, sa, s);
    case 3: return launch_tree_nl<DT, OP, 3>(a, sa, s);
    case 4: return launch_tree_nl<DT, OP, 4>(a, sa, s);
    case 5: return launch_tree_nl<DT, OP, 5>(a, sa, s);
    case 6: return launch_tree_nl<DT, OP, 6>(a, sa, s);
    case 7: return launch_tree_nl<DT, OP, 7>(a, sa, s);
    case 8: return launch_tree_nl<DT, OP, 8>(a, sa, s);
    default: return hipErrorInvalidValue;
    }
}

template <int DT>
static hipError_t launch_tree_dt(const TreeArgs& a, const TreeScalarArgs* sa, int op, hipStream_t s) {
    switch (op) {
    case CHR_SUM: return launch_tree_op<DT, CHR_SUM>(a, sa, s);
    case CHR_PROD: return launch_tree_op<DT, CHR_PROD>(a, sa, s);
    case CHR_MAX: return launch_tree_op<DT, CHR_MAX>(a, sa, s);
    case CHR_MIN: return launch_tree_op<DT, CHR_MIN>(a, sa, s);
    default: return hipErrorInvalidValue;
    }
}

static hipError_t launch_tree_any(const TreeArgs& a, const TreeScalarArgs* sa, int dtype, int op, hipStream_t s) {
    switch (dtype) {
    case CHR_FLOAT32: return launch_tree_dt<CHR_FLOAT32>(a, sa, op, s);
    case CHR_FLOAT64: return launch_tree_dt<CHR_FLOAT64>(a, sa, op, s);
    case CHR_INT32: return launch_tree_dt<CHR_INT32>(a, sa, op, s);
    case CHR_BFLOAT16: return launch_tree_dt<CHR_BFLOAT16>(a, sa, op, s);
    default: return hipErrorInvalidValue;
    }
}

bool tree_program_ok(int nl, const uint8_t* comb, const uint8_t* swaps, uint32_t* comb_bits, uint32_t* swap_bits) {
    if (nl < 1 || nl > kMaxLeaves || !comb) return false;
    int d = 0, nc = 0;
    uint32_t cb = 0, sb = 0;
    for (int j = 0; j < nl; ++j) {
        if (++d > kTreeDepth) return false;
        if ((int)comb[j] > d - 1) return false;  // a combine needs two values on the stack
        cb |= (uint32_t)comb[j] << (2 * j);
        for (int c = 0; c < comb[j]; ++c, ++nc) {
            if (swaps && swaps[nc]) sb |= 1u << nc;
            --d;
        }
    }
    if (d != 1 || nc != nl - 1) return false;
    *comb_bits = cb;
    *swap_bits = sb;
    return true;
}

hipError_t launch_reduce_tree(void* out, const void* const* leaves, int nl, const uint8_t* comb, const uint8_t* swaps,
                              size_t n, int dtype, int op, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (op < CHR_SUM || op > CHR_MIN) return hipErrorInvalidValue;
    uint32_t cb = 0, sb = 0;
    if (!tree_program_ok(nl, comb, swaps, &cb, &sb)) return hipErrorInvalidValue;
    const size_t es = dtype_size(dtype);
    if (!es) return hipErrorInvalidValue;
    if (nl == 1) return out == leaves[0] ? hipSuccess
                                         : hipMemcpyAsync(out, leaves[0], n * es, hipMemcpyDeviceToDevice, stream);
    const uintptr_t mis = (uintptr_t)out & 15u;
    bool congruent = (mis % es) == 0;
    for (int j = 0; j < nl; ++j) congruent = congruent && (((uintptr_t)leaves[j] & 15u) == mis);
    auto scalar = [&](size_t off, size_t cnt) -> hipError_t {
        if (!cnt) return hipSuccess;
        TreeScalarArgs sa{};
        sa.out = (char*)out + off * es;
        for (int j = 0; j < nl; ++j) sa.leaves[j] = (const char*)leaves[j] + off * es;
        sa.n = cnt;
        sa.nl = nl;
        sa.comb = cb;
        sa.swaps = sb;
        TreeArgs dummy{};
        return launch_tree_any(dummy, &sa, dtype, op, stream);
    };
    if (!congruent) return scalar(0, n);
    size_t head = mis ? (16 - mis) / es : 0;
    if (head > n) head = n;
    const size_t E = 16 / es;
    const size_t nvec = (n - head) / E;
    const size_t tail = n - head - nvec * E;
    hipError_t err = scalar(0, head);
    if (err != hipSuccess) return err;
    if (nvec) {
        TreeArgs a{};
        a.out = (u32x4*)((char*)out + head * es);
        for (int j = 0; j < nl; ++j) a.leaves[j] = (const u32x4*)((const char*)leaves[j] + head * es);
        a.nvec = nvec;
        a.nl = nl;
        a.comb = cb;
        a.swaps = sb;
        if ((err = launch_tree_any(a, nullptr, dtype, op, stream)) != hipSuccess) return err;
    }
    return scalar(head + nvec * E, tail);
}

}  // namespace chr
