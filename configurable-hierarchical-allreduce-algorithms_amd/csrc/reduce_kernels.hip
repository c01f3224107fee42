// reduce_kernels.hip -- the hot path: CDNA4 (gfx950) fused bucket-reduction kernels.
//
// Replaces MPI_Reduce_local(in, inout, n, dtype, op) at
//   Fugaku_experiments/Allreduce/all_reduce_radix_batch.cpp:332, :364, :446, :529 and
//   Fugaku_experiments/Reduce-scatter/reduce_scatter_radix_batch.cpp:332, :366, :447, :552,
// and fuses the k-1 (or nnodes-1) consecutive calls that hit one region into one pass:
//   out = (...((acc op in_0) op in_1)...) op in_{m-1}
// rounding after every step exactly like the sequential calls (MPICH's loop is
// inout[i] = OP(in[i], inout[i]), src/mpi/coll/op/*.c in MPICH 3.3.2).
//
// Roofline: pure HBM streaming, (m + 2) * n * sizeof(T) bytes per call (read m inputs
// and the accumulator, write the result), ~0.1-0.5 FLOP/byte: no MFMA.  Design:
//  * one 16-byte global_load_dwordx4 per lane per operand (1 KiB per wave-instruction),
//    U independent vectors per lane in flight (ILP) with every operand's loads issued
//    before the first add, one trip per workgroup (the full grid measured faster than a
//    capped grid-stride grid on large buckets);
//  * non-temporal loads and stores for calls that stream >= 128 MiB (HBM-cold buckets
//    +15-40 % over plain accesses; plain stays faster on small, cache-warm calls);
//  * workgroup size by regime: one wave (64 threads) for the streaming (nt) calls, +3 % on
//    the 64 MiB m=1 bucket and up to +5 % for m >= 3 (profiles/r01/block_ab_*); 256 threads
//    for the small cache-warm calls, where one-wave workgroups lose up to 5 %;
//  * no LDS: a pure stream has no reuse, and staging through LDS (global_load_lds) was
//    measured null-to-negative for this regime (profiles/);
//  * no XCD remap: no inter-workgroup reuse; an XCD-contiguous workgroup map measured 0.88x
//    (HBM wants every XCD spread over all addresses, profiles/r01/microbench_focus5.txt);
//  * IEEE semantics kept bit-exact with the CPU oracle: no fast-math, selects (not
//    v_max) for MAX/MIN, int32 wraps, bf16 = f32 op then RNE per step with NaN kept
//    (v_cvt_pk_bf16_f32, reduce_common.hpp).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "reduce_common.hpp"

namespace chr {

constexpr int kMaxFanIn = 8;

size_t dtype_size(int dtype) {
    switch (dtype) {
    case CHR_FLOAT32: return 4;
    case CHR_FLOAT64: return 8;
    case CHR_INT32: return 4;
    case CHR_BFLOAT16: return 2;
    default: return 0;
    }
}

bool valid_dtype_op(int dtype, int op) { return dtype_size(dtype) != 0 && op >= CHR_SUM && op <= CHR_MIN; }

ReduceTuning& reduce_tuning() {
    static ReduceTuning t = [] {
        ReduceTuning r;
        const char* s = std::getenv("CHR_REDUCE_MAX_BLOCKS");
        r.max_blocks = s ? std::atoi(s) : 0;  // 0: one trip per workgroup (full grid)
        s = std::getenv("CHR_REDUCE_NT");     // 0 / 1 / unset = by size
        r.nt_mode = s ? std::atoi(s) : -1;
        s = std::getenv("CHR_REDUCE_NT_MIN_BYTES");
        r.nt_min_bytes = s ? (size_t)std::atoll(s) : (size_t)128 << 20;
        s = std::getenv("CHR_REDUCE_ACC0");   // 0 / 1 / unset = by fan-in and size
        r.acc0_mode = s ? std::atoi(s) : -1;
        s = std::getenv("CHR_REDUCE_ACC0_MIN_BYTES");
        r.acc0_min_bytes = s ? (size_t)std::atoll(s) : 0;
        s = std::getenv("CHR_REDUCE_BLOCK");  // 64 / 256 / unset = by policy (launch_vec_m)
        r.block = s ? (std::atoi(s) == 64 ? 64 : 256) : 0;
        return r;
    }();
    return t;
}

struct VecArgs {
    u32x4* out;
    const u32x4* acc;
    const u32x4* ins[kMaxFanIn];
    size_t nvec;
};

// U vectors (16 B each) per lane per trip; all M+1 operands of the trip are loaded
// before the first add so (M+1)*U*16 bytes per lane are in flight.  NT: non-temporal
// loads and stores (global_load/store_dwordx4 ... nt) for calls that stream far more than
// the caches hold: +15-40 % on HBM-cold buckets.  ACC0: under NT, the FIRST of the U
// accumulator vectors keeps the default policy (in place, a quarter of the write-backs then
// go through the Infinity Cache): per-slot policy sweep
// (profiles/r01/microbench_focus4_slot_policy.txt) +15 % at 1 GiB m=1, +3-5 % for m>=2 with
// 256-thread workgroups; with one-wave workgroups it also gains on the 64 MiB m=1 bucket
// (6 440-6 464 vs 6 041-6 052 GB/s all-nt, profiles/r01/block_ab_bench.txt), so it is used for
// every nt call; making ALL accumulator slots temporal thrashes the cache (-7 %).  Slot 0 is peeled so that the two policies
// are separate instructions (a select between a plain and an nt load of one address is
// merged by LLVM, dropping the nt bit).
template <int DT, int OP, int M, int U, bool NT, bool ACC0, int BL>
__global__ __launch_bounds__(BL) void k_reduce_vec(VecArgs a) {
    const size_t stride = (size_t)gridDim.x * BL * U;
    for (size_t base = (size_t)blockIdx.x * BL * U + threadIdx.x; base < a.nvec; base += stride) {
        if (base + (size_t)(U - 1) * BL < a.nvec) {
            u32x4 acc[U], x[M][U];
            acc[0] = ld<NT && !ACC0>(&a.acc[base]);
#pragma unroll
            for (int u = 1; u < U; ++u) acc[u] = ld<NT>(&a.acc[base + (size_t)u * BL]);
#pragma unroll
            for (int j = 0; j < M; ++j)
#pragma unroll
                for (int u = 0; u < U; ++u) x[j][u] = ld<NT>(&a.ins[j][base + (size_t)u * BL]);
            // Keep every load of the trip ahead of the first add: without this the
            // scheduler interleaves the first add (and its vmcnt(0)) between the loads.
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < M; ++j)
#pragma unroll
                for (int u = 0; u < U; ++u) acc[u] = apply_vec<DT, OP>(x[j][u], acc[u]);
#pragma unroll
            for (int u = 0; u < U; ++u) st<NT>(&a.out[base + (size_t)u * BL], acc[u]);
        } else {
            for (int u = 0; u < U; ++u) {
                const size_t i = base + (size_t)u * BL;
                if (i >= a.nvec) break;
                u32x4 acc = a.acc[i];
#pragma unroll
                for (int j = 0; j < M; ++j) acc = apply_vec<DT, OP>(a.ins[j][i], acc);
                a.out[i] = acc;
            }
        }
    }
}

struct ScalarArgs {
    void* out;
    const void* acc;
    const void* ins[kMaxFanIn];
    int m;
    size_t n;
};

// Any alignment (odd sizes / offsets): one element per lane per trip.
template <int DT, int OP>
__global__ __launch_bounds__(kBlock) void k_reduce_scalar(ScalarArgs a) {
    using T = typename DTy<DT>::T;
    T* out = (T*)a.out;
    const T* acc = (const T*)a.acc;
    for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < a.n; i += (size_t)gridDim.x * kBlock) {
        T v = acc[i];
        for (int j = 0; j < a.m; ++j) v = apply<DT, OP>(((const T*)a.ins[j])[i], v);
        out[i] = v;
    }
}

// ---- host launchers ----------------------------------------------------------------------

template <int DT, int OP, int M, int BL>
static hipError_t launch_vec_mb(const VecArgs& a, bool nt, bool acc0, hipStream_t s) {
    constexpr int U = M <= 2 ? 4 : 2;
    const size_t trips = (a.nvec + (size_t)BL * U - 1) / ((size_t)BL * U);
    const size_t cap = reduce_tuning().max_blocks > 0 ? (size_t)reduce_tuning().max_blocks : trips;
    const int grid = (int)(trips < cap ? trips : cap);
    if (!nt)
        hipLaunchKernelGGL((k_reduce_vec<DT, OP, M, U, false, false, BL>), dim3(grid), dim3(BL), 0, s, a);
    else if (acc0)
        hipLaunchKernelGGL((k_reduce_vec<DT, OP, M, U, true, true, BL>), dim3(grid), dim3(BL), 0, s, a);
    else
        hipLaunchKernelGGL((k_reduce_vec<DT, OP, M, U, true, false, BL>), dim3(grid), dim3(BL), 0, s, a);
    return hipGetLastError();
}

// Policy (profiles/r01/block_ab_*): calls that stream >= 128 MiB run non-temporal with
// one-wave workgroups and the first accumulator slot temporal (ACC0); smaller, cache-warm
// calls keep plain accesses and 256-thread workgroups.
template <int DT, int OP, int M>
static hipError_t launch_vec_m(const VecArgs& a, hipStream_t s) {
    const ReduceTuning& t = reduce_tuning();
    const size_t call_bytes = (size_t)(M + 2) * a.nvec * 16;
    const bool nt = t.nt_mode == 1 || (t.nt_mode < 0 && call_bytes >= t.nt_min_bytes);
    const bool acc0 = t.acc0_mode == 1 || (t.acc0_mode < 0 && (M >= 2 || a.nvec * 16 >= t.acc0_min_bytes));
    const int bl = t.block ? t.block : nt ? 64 : 256;
    return bl == 64 ? launch_vec_mb<DT, OP, M, 64>(a, nt, acc0, s) : launch_vec_mb<DT, OP, M, 256>(a, nt, acc0, s);
}

template <int DT, int OP>
static hipError_t launch_vec_op(const VecArgs& a, int m, hipStream_t s) {
    switch (m) {
    case 1: return launch_vec_m<DT, OP, 1>(a, s);
    case 2: return launch_vec_m<DT, OP, 2>(a, s);
    case 3: return launch_vec_m<DT, OP, 3>(a, s);
    case 4: return launch_vec_m<DT, OP, 4>(a, s);
    case 5: return launch_vec_m<DT, OP, 5>(a, s);
    case 6: return launch_vec_m<DT, OP, 6>(a, s);
    case 7: return launch_vec_m<DT, OP, 7>(a, s);
    case 8: return launch_vec_m<DT, OP, 8>(a, s);
    default: return hipErrorInvalidValue;
    }
}

template <int DT>
static hipError_t launch_vec_dt(const VecArgs& a, int m, int op, hipStream_t s) {
    switch (op) {
    case CHR_SUM: return launch_vec_op<DT, CHR_SUM>(a, m, s);
    case CHR_PROD: return launch_vec_op<DT, CHR_PROD>(a, m, s);
    case CHR_MAX: return launch_vec_op<DT, CHR_MAX>(a, m, s);
    case CHR_MIN: return launch_vec_op<DT, CHR_MIN>(a, m, s);
    case kMaxSw:
        if constexpr (DT == CHR_INT32) return launch_vec_op<DT, CHR_MAX>(a, m, s);
        else return launch_vec_op<DT, kMaxSw>(a, m, s);
    case kMinSw:
        if constexpr (DT == CHR_INT32) return launch_vec_op<DT, CHR_MIN>(a, m, s);
        else return launch_vec_op<DT, kMinSw>(a, m, s);
    default: return hipErrorInvalidValue;
    }
}

template <int DT>
static hipError_t launch_scalar_dt(const ScalarArgs& a, int op, hipStream_t s) {
    const size_t trips = (a.n + kBlock - 1) / kBlock;
    const int grid = (int)(trips < 2048 ? trips : 2048);
    switch (op) {
    case CHR_SUM: hipLaunchKernelGGL((k_reduce_scalar<DT, CHR_SUM>), dim3(grid), dim3(kBlock), 0, s, a); break;
    case CHR_PROD: hipLaunchKernelGGL((k_reduce_scalar<DT, CHR_PROD>), dim3(grid), dim3(kBlock), 0, s, a); break;
    case CHR_MAX: hipLaunchKernelGGL((k_reduce_scalar<DT, CHR_MAX>), dim3(grid), dim3(kBlock), 0, s, a); break;
    case CHR_MIN: hipLaunchKernelGGL((k_reduce_scalar<DT, CHR_MIN>), dim3(grid), dim3(kBlock), 0, s, a); break;
    case kMaxSw: hipLaunchKernelGGL((k_reduce_scalar<DT, kMaxSw>), dim3(grid), dim3(kBlock), 0, s, a); break;
    case kMinSw: hipLaunchKernelGGL((k_reduce_scalar<DT, kMinSw>), dim3(grid), dim3(kBlock), 0, s, a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

static hipError_t launch_scalar(void* out, const void* acc, const void* const* ins, int m, size_t n, int dtype,
                                int op, hipStream_t s) {
    if (n == 0) return hipSuccess;
    ScalarArgs a{};
    a.out = out;
    a.acc = acc;
    a.m = m;
    a.n = n;
    for (int j = 0; j < m; ++j) a.ins[j] = ins[j];
    switch (dtype) {
    case CHR_FLOAT32: return launch_scalar_dt<CHR_FLOAT32>(a, op, s);
    case CHR_FLOAT64: return launch_scalar_dt<CHR_FLOAT64>(a, op, s);
    case CHR_INT32: return launch_scalar_dt<CHR_INT32>(a, op, s);
    case CHR_BFLOAT16: return launch_scalar_dt<CHR_BFLOAT16>(a, op, s);
    default: return hipErrorInvalidValue;
    }
}

// One pass over at most kMaxFanIn inputs.
static hipError_t launch_group(void* out, const void* acc, const void* const* ins, int m, size_t n, int dtype,
                               int op, hipStream_t s) {
    const size_t es = dtype_size(dtype);
    const uintptr_t mis = (uintptr_t)out & 15u;
    bool congruent = ((uintptr_t)acc & 15u) == mis && (mis % es) == 0;
    for (int j = 0; j < m; ++j) congruent = congruent && (((uintptr_t)ins[j] & 15u) == mis);
    if (!congruent) return launch_scalar(out, acc, ins, m, n, dtype, op, s);
    size_t head = mis ? (16 - mis) / es : 0;
    if (head > n) head = n;
    const size_t E = 16 / es;
    const size_t nvec = (n - head) / E;
    const size_t tail = n - head - nvec * E;
    hipError_t err;
    if (head && (err = launch_scalar(out, acc, ins, m, head, dtype, op, s)) != hipSuccess) return err;
    if (nvec) {
        VecArgs a{};
        a.out = (u32x4*)((char*)out + head * es);
        a.acc = (const u32x4*)((const char*)acc + head * es);
        for (int j = 0; j < m; ++j) a.ins[j] = (const u32x4*)((const char*)ins[j] + head * es);
        a.nvec = nvec;
        switch (dtype) {
        case CHR_FLOAT32: err = launch_vec_dt<CHR_FLOAT32>(a, m, op, s); break;
        case CHR_FLOAT64: err = launch_vec_dt<CHR_FLOAT64>(a, m, op, s); break;
        case CHR_INT32: err = launch_vec_dt<CHR_INT32>(a, m, op, s); break;
        case CHR_BFLOAT16: err = launch_vec_dt<CHR_BFLOAT16>(a, m, op, s); break;
        default: err = hipErrorInvalidValue;
        }
        if (err != hipSuccess) return err;
    }
    if (tail) {
        const size_t o = (head + nvec * E) * es;
        const void* tins[kMaxFanIn];
        for (int j = 0; j < m; ++j) tins[j] = (const char*)ins[j] + o;
        return launch_scalar((char*)out + o, (const char*)acc + o, tins, m, tail, dtype, op, s);
    }
    return hipSuccess;
}

hipError_t launch_reduce(void* out, const void* acc, const void* const* ins, int m, size_t n, int dtype, int op,
                         hipStream_t stream, bool running_first) {
    if (n == 0) return hipSuccess;
    if (op < CHR_SUM || op > CHR_MIN) return hipErrorInvalidValue;
    if (running_first && (op == CHR_MAX || op == CHR_MIN)) op = op == CHR_MAX ? kMaxSw : kMinSw;
    const size_t es = dtype_size(dtype);
    if (m == 0) {
        if (out == acc) return hipSuccess;
        return hipMemcpyAsync(out, acc, n * es, hipMemcpyDeviceToDevice, stream);
    }
    // Left-to-right chaining keeps the reference's association for any fan-in.
    for (int j0 = 0; j0 < m; j0 += kMaxFanIn) {
        const int mg = (m - j0) < kMaxFanIn ? (m - j0) : kMaxFanIn;
        hipError_t err = launch_group(out, j0 == 0 ? acc : out, ins + j0, mg, n, dtype, op, stream);
        if (err != hipSuccess) return err;
    }
    return hipSuccess;
}

// ---- synthetic inputs (same generator as oracle/chiara_oracle.h) -------------------------

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ __launch_bounds__(kBlock) void k_fill(void* buf, size_t n, int dtype, int pattern, uint64_t seed,
                                                 uint64_t rank, uint64_t count_for_seq) {
    for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) {
        if (pattern == 1) {
            const int32_t v = (int32_t)(uint32_t)(rank * count_for_seq + i);
            switch (dtype) {
            case CHR_FLOAT32: ((float*)buf)[i] = (float)v; break;
            case CHR_FLOAT64: ((double*)buf)[i] = (double)v; break;
            case CHR_INT32: ((int32_t*)buf)[i] = v; break;
            default: ((uint16_t*)buf)[i] = f2bf((float)v); break;
            }
        } else if (pattern == 2) {  // ties / signed zeros / per-rank NaN payloads
            const unsigned sel = (unsigned)(splitmix64(seed ^ (rank << 40) ^ (uint64_t)i) >> 61);
            const uint32_t pay = (uint32_t)(rank + 1) & 0x3Fu;
            const float fv = sel == 2 ? 1.0f : sel == 3 ? -1.0f : sel == 6 ? 0.5f : (sel & 1) ? -0.0f : 0.0f;
            switch (dtype) {
            case CHR_FLOAT32:
                ((uint32_t*)buf)[i] = sel == 7 ? (0x7FC00000u | (pay << 16) | pay) : __float_as_uint(fv);
                break;
            case CHR_FLOAT64:
                ((uint64_t*)buf)[i] = sel == 7 ? (0x7FF8000000000000ull | ((uint64_t)pay << 40) | pay)
                                               : (uint64_t)__double_as_longlong((double)fv);
                break;
            case CHR_INT32: ((int32_t*)buf)[i] = sel == 6 ? 2 : sel == 7 ? 7 : sel == 2 ? 1 : sel == 3 ? -1 : 0; break;
            default: ((uint16_t*)buf)[i] = sel == 7 ? (uint16_t)(0x7FC0u | pay) : f2bf(fv); break;
            }
        } else {
            const uint64_t u = splitmix64(seed ^ (rank << 40) ^ (uint64_t)i);
            switch (dtype) {
            case CHR_FLOAT32: ((float*)buf)[i] = (float)(u >> 40) * (1.0f / 8388608.0f) - 1.0f; break;
            case CHR_FLOAT64: ((double*)buf)[i] = (double)(u >> 11) * (1.0 / 4503599627370496.0) - 1.0; break;
            case CHR_INT32: ((int32_t*)buf)[i] = (int32_t)(uint32_t)(u >> 32); break;
            default: ((uint16_t*)buf)[i] = f2bf((float)(u >> 40) * (1.0f / 8388608.0f) - 1.0f); break;
            }
        }
    }
}

hipError_t launch_fill(void* buf, size_t n, int dtype, int pattern, uint64_t seed, int rank, uint64_t count_for_seq,
                       hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const size_t trips = (n + kBlock - 1) / kBlock;
    const int grid = (int)(trips < 8192 ? trips : 8192);
    hipLaunchKernelGGL(k_fill, dim3(grid), dim3(kBlock), 0, stream, buf, n, dtype, pattern, seed, (uint64_t)rank,
                       count_for_seq);
    return hipGetLastError();
}

}  // namespace chr
