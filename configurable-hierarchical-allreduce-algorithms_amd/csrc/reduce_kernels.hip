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
//  * non-temporal loads and stores for calls that stream >= 40 MiB (HBM-cold buckets
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

#include <algorithm>

#include <cstdlib>

#include "reduce_vec.hpp"

namespace chr {

size_t dtype_size(int dtype) {
    switch (dtype) {
    case CHR_FLOAT32: return 4;
    case CHR_FLOAT64: return 8;
    case CHR_INT32: return 4;
    case CHR_BFLOAT16: return 2;
    case CHR_INT8: case CHR_UINT8: return 1;
    case CHR_INT16: case CHR_UINT16: return 2;
    case CHR_UINT32: return 4;
    case CHR_INT64: case CHR_UINT64: return 8;
    // the pair and complex types: the C struct, i.e. MPI's extent (the element stride of a buffer)
    case CHR_FLOAT_INT: case CHR_2INT: case CHR_SHORT_INT: case CHR_C_FLOAT_COMPLEX: return 8;
    case CHR_DOUBLE_INT: case CHR_LONG_INT: case CHR_C_DOUBLE_COMPLEX: return 16;
    default: return 0;
    }
}

static bool is_pair_dtype(int dtype) { return dtype >= CHR_FLOAT_INT && dtype <= CHR_SHORT_INT; }
static bool is_complex_dtype(int dtype) { return dtype == CHR_C_FLOAT_COMPLEX || dtype == CHR_C_DOUBLE_COMPLEX; }

static bool is_float_dtype(int dtype) {
    return dtype == CHR_FLOAT32 || dtype == CHR_FLOAT64 || dtype == CHR_BFLOAT16;
}

// MPI's predefined-op/type table as MPICH 3.3.2's MPI_Reduce_local applies it (probed): SUM/PROD/
// MAX/MIN on every type, the logical ops on the integer types and on float/double (an MPICH
// extension of the standard's table), the bitwise ops on the integer types.  bf16 is this
// library's own type: arithmetic and MAX/MIN only.
bool valid_dtype_op(int dtype, int op) {
    if (!dtype_size(dtype)) return false;
    // MPICH 3.3.2's table for the pair and complex types (oracle/ref_pairs_probe table,
    // tests/golden/pairs_manifest.json): MAXLOC / MINLOC on the pairs only, SUM / PROD on complex only
    if (is_pair_dtype(dtype)) return op == CHR_MAXLOC || op == CHR_MINLOC;
    if (is_complex_dtype(dtype)) return op == CHR_SUM || op == CHR_PROD;
    if (op == CHR_MAXLOC || op == CHR_MINLOC) return false;
    if (op >= CHR_SUM && op <= CHR_MIN) return true;
    if (op >= CHR_LAND && op <= CHR_LXOR) return dtype != CHR_BFLOAT16;
    return op >= CHR_BAND && op <= CHR_BXOR && !is_float_dtype(dtype);
}

// The kernel instantiation that computes (dtype, op).  Signedness only matters to MAX/MIN:
// wrapping SUM/PROD, the logical and the bitwise ops give the same bits on the unsigned type of
// the same width (int32's kernels serve uint32 there).  running_first (MPICH_do_reduce order)
// changes results only for floating types: MAX/MIN on ties of -0/+0 and NaN compares, SUM/PROD on
// which NaN survives when two meet (kSumSw / kProdSw).
void canon_op(int dtype, int op, bool running_first, int* kdt, int* kop) {
    *kop = op;
    if (is_pair_dtype(dtype) || is_complex_dtype(dtype)) {
        *kdt = dtype;
        if (running_first && (dtype == CHR_FLOAT_INT || dtype == CHR_DOUBLE_INT))  // ties of -0/+0, NaN
            *kop = op == CHR_MAXLOC ? kMaxLocSw : op == CHR_MINLOC ? kMinLocSw : op;
        if (running_first && is_complex_dtype(dtype))  // which NaN survives, per part (reduce_common.hpp apply)
            *kop = op == CHR_SUM ? kSumSw : op == CHR_PROD ? kProdSw : op;
        return;
    }
    if (is_float_dtype(dtype)) {
        *kdt = dtype;
        if (running_first && (op == CHR_MAX || op == CHR_MIN)) *kop = op == CHR_MAX ? kMaxSw : kMinSw;
        if (running_first && (op == CHR_SUM || op == CHR_PROD)) *kop = op == CHR_SUM ? kSumSw : kProdSw;  // NaN payloads
        return;
    }
    if (op == CHR_MAX || op == CHR_MIN) {
        *kdt = dtype;
        return;
    }
    switch (dtype_size(dtype)) {
    case 1: *kdt = CHR_UINT8; break;
    case 2: *kdt = CHR_UINT16; break;
    case 4: *kdt = CHR_INT32; break;
    default: *kdt = CHR_UINT64; break;
    }
}

// kernel types compiled in this translation unit; the rest: reduce_int.hip
static bool in_core_tu(int kdt, int kop) {
    return (is_float_dtype(kdt) || kdt == CHR_INT32) && ((kop >= CHR_SUM && kop <= CHR_MIN) || kop == kMaxSw ||
                                                         kop == kMinSw || kop == kSumSw || kop == kProdSw);
}

int& coresident_depth() {
    static thread_local int depth = 0;
    return depth;
}

ReduceTuning& reduce_tuning() {
    static ReduceTuning t = [] {
        ReduceTuning r;
        const char* s = std::getenv("CHR_REDUCE_MAX_LAUNCH_VEC");
        r.max_launch_vec = s ? (size_t)std::atoll(s) : 0;
        s = std::getenv("CHR_XCD_RUN_KIB");
        r.xcd_run_kib = s ? std::atoi(s) : -1;  // -1: policy (vec_xcd_run_kib / tree_xcd_run_kib)
        s = std::getenv("CHR_REDUCE_NT");     // 0 / 1 / unset = by size
        r.nt_mode = s ? std::atoi(s) : -1;
        s = std::getenv("CHR_REDUCE_NT_MIN_BYTES");
        // bucket launches stream from 40 MiB per call (profiles/r05/ab_mid/, 2-3 alternating
        // rounds, gated back-to-back launches): the streaming shape (nt, one wave, U / cap / XCD runs per fan-in)
        // against plain 256-thread workgroups -- m = 1 at 16 MiB (48 MiB per call) 0.624-0.626 vs 0.583-0.585 on
        // a 2 GiB rotation and 0.644-0.647 vs 0.586-0.589 on the sweep's 16 sets, 32 MiB 0.72-0.75 vs 0.65, m = 3
        // at 8 MiB (40 MiB) 0.61-0.64 vs 0.56-0.57; below, plain wins where the rotation stays cache-resident
        // (m = 1 at 8 MiB over 16 sets 0.604 vs 0.535, m = 3 at 4 MiB 0.565 vs 0.508).  One set reused call
        // after call (fully cache-resident) prefers plain up to 48 MiB per call too (m = 1 16 MiB 1.26 vs
        // 0.87 of 8 TB/s): a just-reduced region reduced again; the collectives' trees keep their own threshold.
        r.nt_min_bytes = s ? (size_t)std::atoll(s) : (size_t)40 << 20;
        // trees stream 3-9 operands at once: from 64 MiB per launch the nt shapes win on HBM-cold
        // leaves and tie on cache-warm ones (C4 slice, 4 MiB pieces = 72 MiB: nt 0.591-0.602 vs
        // plain 0.572-0.577 cold, 0.651-0.657 vs 0.599-0.666 warm; 2 MiB pieces tie;
        // profiles/r02/occupancy_cap/microbench_focus19_nt_threshold.txt)
        r.tree_nt_min_bytes = s ? r.nt_min_bytes : (size_t)64 << 20;
        s = std::getenv("CHR_WG_PER_CU_VEC");
        r.wg_per_cu_vec = s ? std::max(0, std::atoi(s)) : -1;
        s = std::getenv("CHR_WG_PER_CU_TREE");
        r.wg_per_cu_tree = s ? std::max(0, std::atoi(s)) : -1;
        s = std::getenv("CHR_XCD_HAND_SHIFT");
        r.xcd_hand_shift = s ? std::min(31, std::max(0, std::atoi(s))) : -1;  // [0, 31]; 31 hands nothing
        int dev = 0, lds = 0, blk = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) != hipSuccess ||
            lds <= 0)
            lds = 0;  // unknown: no cap
        if (hipDeviceGetAttribute(&blk, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess || blk <= 0)
            blk = 0;
        r.lds_per_cu = (unsigned)lds;
        r.lds_per_block = (unsigned)blk;
        return r;
    }();
    return t;
}

// ---- host launchers ----------------------------------------------------------------------

template <int DT>
static hipError_t launch_vec_dt(const VecArgs& a, int m, int op, hipStream_t s) {
    switch (op) {
    case CHR_SUM: return launch_vec_op<DT, CHR_SUM>(a, m, s);
    case CHR_PROD: return launch_vec_op<DT, CHR_PROD>(a, m, s);
    case CHR_MAX: return launch_vec_op<DT, CHR_MAX>(a, m, s);
    case CHR_MIN: return launch_vec_op<DT, CHR_MIN>(a, m, s);
    case kMaxSw:
        if constexpr (DT == CHR_INT32) return hipErrorInvalidValue;
        else return launch_vec_op<DT, kMaxSw>(a, m, s);
    case kMinSw:
        if constexpr (DT == CHR_INT32) return hipErrorInvalidValue;
        else return launch_vec_op<DT, kMinSw>(a, m, s);
    case kSumSw:
        if constexpr (DT == CHR_INT32) return hipErrorInvalidValue;
        else return launch_vec_op<DT, kSumSw>(a, m, s);
    case kProdSw:
        if constexpr (DT == CHR_INT32) return hipErrorInvalidValue;
        else return launch_vec_op<DT, kProdSw>(a, m, s);
    default: return hipErrorInvalidValue;
    }
}

template <int DT>
static hipError_t launch_scalar_dt(const ScalarArgs& a, int op, hipStream_t s) {
    switch (op) {
    case CHR_SUM: return launch_scalar_op<DT, CHR_SUM>(a, s);
    case CHR_PROD: return launch_scalar_op<DT, CHR_PROD>(a, s);
    case CHR_MAX: return launch_scalar_op<DT, CHR_MAX>(a, s);
    case CHR_MIN: return launch_scalar_op<DT, CHR_MIN>(a, s);
    case kMaxSw:
        if constexpr (DT == CHR_INT32) return hipErrorInvalidValue;
        else return launch_scalar_op<DT, kMaxSw>(a, s);
    case kMinSw:
        if constexpr (DT == CHR_INT32) return hipErrorInvalidValue;
        else return launch_scalar_op<DT, kMinSw>(a, s);
    case kSumSw:
        if constexpr (DT == CHR_INT32) return hipErrorInvalidValue;
        else return launch_scalar_op<DT, kSumSw>(a, s);
    case kProdSw:
        if constexpr (DT == CHR_INT32) return hipErrorInvalidValue;
        else return launch_scalar_op<DT, kProdSw>(a, s);
    default: return hipErrorInvalidValue;
    }
}

// kdt/kop: the kernel type and op from canon_op
static hipError_t launch_scalar(void* out, const void* acc, const void* const* ins, int m, size_t n, int kdt,
                                int kop, hipStream_t s) {
    if (n == 0) return hipSuccess;
    ScalarArgs a{};
    a.out = out;
    a.acc = acc;
    a.m = m;
    a.n = n;
    for (int j = 0; j < m; ++j) a.ins[j] = ins[j];
    if (is_pair_dtype(kdt) || is_complex_dtype(kdt)) return launch_scalar_pair(a, kdt, kop, s);
    if (!in_core_tu(kdt, kop)) return launch_scalar_int(a, kdt, kop, s);
    switch (kdt) {
    case CHR_FLOAT32: return launch_scalar_dt<CHR_FLOAT32>(a, kop, s);
    case CHR_FLOAT64: return launch_scalar_dt<CHR_FLOAT64>(a, kop, s);
    case CHR_INT32: return launch_scalar_dt<CHR_INT32>(a, kop, s);
    case CHR_BFLOAT16: return launch_scalar_dt<CHR_BFLOAT16>(a, kop, s);
    default: return hipErrorInvalidValue;
    }
}

// One pass over at most kMaxFanIn inputs.
static hipError_t launch_group(void* out, const void* acc, const void* const* ins, int m, size_t n, int dtype,
                               int op, hipStream_t s) {
    const size_t es = dtype_size(dtype);  // dtype, op: the kernel type and op (canon_op)
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
        if (is_pair_dtype(dtype) || is_complex_dtype(dtype)) {
            err = launch_vec_pair(a, dtype, op, m, s);
        } else if (!in_core_tu(dtype, op)) {
            err = launch_vec_int(a, dtype, op, m, s);
        } else {
            switch (dtype) {
            case CHR_FLOAT32: err = launch_vec_dt<CHR_FLOAT32>(a, m, op, s); break;
            case CHR_FLOAT64: err = launch_vec_dt<CHR_FLOAT64>(a, m, op, s); break;
            case CHR_INT32: err = launch_vec_dt<CHR_INT32>(a, m, op, s); break;
            case CHR_BFLOAT16: err = launch_vec_dt<CHR_BFLOAT16>(a, m, op, s); break;
            default: err = hipErrorInvalidValue;
            }
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
    if (!valid_dtype_op(dtype, op)) return hipErrorInvalidValue;
    const size_t es = dtype_size(dtype);
    canon_op(dtype, op, running_first, &dtype, &op);
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

__device__ __forceinline__ float gen_f32(uint64_t seed, uint64_t rank, uint64_t i) {
    return (float)(splitmix64(seed ^ (rank << 40) ^ i) >> 40) * (1.0f / 8388608.0f) - 1.0f;
}
__device__ __forceinline__ double gen_f64(uint64_t seed, uint64_t rank, uint64_t i) {
    return (double)(splitmix64(seed ^ (rank << 40) ^ i) >> 11) * (1.0 / 4503599627370496.0) - 1.0;
}

// The pair and complex types (oracle/chiara_oracle.c orc_fill_pair, the same formulas): pair value a
// small integer in [-4, 3] (uniform / sparse), rank*count + i with index = rank (seq), or for the
// floating pairs {+0, -0, 1, -1, 0.5, NaN with a per-rank payload} (ties); index from 6 random bits;
// complex: U[-1,1) parts from elements 2g and 2g + 1 of the float generator, rank*count + i and its
// negation (seq), the float ties values.  Padding bytes zero.
__device__ void fill_pair(char* elem, int dtype, int pattern, uint64_t seed, uint64_t rank, uint64_t count_for_seq,
                          uint64_t g) {
    const float ft[8] = {0.0f, -0.0f, 1.0f, -1.0f, 0.0f, -0.0f, 0.5f, 0.0f};
    const uint64_t key = splitmix64(seed ^ (rank << 40) ^ g);
    const unsigned sel = (unsigned)(key >> 61);
    const uint32_t pay = (uint32_t)(rank + 1) & 0x3Fu;
    const int32_t small = (int32_t)(key >> 61) - 4;
    const int32_t idx = pattern == 1 ? (int32_t)rank : (int32_t)((key >> 32) & 0x3F);
    const int32_t seq = (int32_t)(uint32_t)(rank * count_for_seq + g);
    uint32_t w[4] = {0, 0, 0, 0};
    switch (dtype) {
    case CHR_FLOAT_INT: {
        const float v = pattern == 1 ? (float)seq : pattern == 2 ? ft[sel] : (float)small;
        w[0] = pattern == 2 && sel == 7 ? (0x7FC00000u | (pay << 16) | pay) : __float_as_uint(v);
        w[1] = (uint32_t)idx;
        break;
    }
    case CHR_DOUBLE_INT: {
        const double v = pattern == 1 ? (double)seq : pattern == 2 ? (double)ft[sel] : (double)small;
        const uint64_t u = pattern == 2 && sel == 7 ? (0x7FF8000000000000ull | ((uint64_t)pay << 40) | pay)
                                                     : (uint64_t)__double_as_longlong(v);
        w[0] = (uint32_t)u;
        w[1] = (uint32_t)(u >> 32);
        w[2] = (uint32_t)idx;
        break;
    }
    case CHR_LONG_INT: {
        const uint64_t u = (uint64_t)(int64_t)(pattern == 1 ? seq : small);
        w[0] = (uint32_t)u;
        w[1] = (uint32_t)(u >> 32);
        w[2] = (uint32_t)idx;
        break;
    }
    case CHR_2INT:
        w[0] = (uint32_t)(pattern == 1 ? seq : small);
        w[1] = (uint32_t)idx;
        break;
    case CHR_SHORT_INT:
        w[0] = (uint32_t)(uint16_t)(int16_t)(pattern == 1 ? seq : small);
        w[1] = (uint32_t)idx;
        break;
    case CHR_C_FLOAT_COMPLEX: {
        const float re = pattern == 1 ? (float)seq : pattern == 2 ? ft[sel] : gen_f32(seed, rank, 2 * g);
        const float im = pattern == 1 ? -(float)seq : pattern == 2 ? ft[(key >> 58) & 7] : gen_f32(seed, rank, 2 * g + 1);
        w[0] = __float_as_uint(re);
        w[1] = __float_as_uint(im);
        break;
    }
    default: {  // CHR_C_DOUBLE_COMPLEX
        const double re = pattern == 1 ? (double)seq : pattern == 2 ? (double)ft[sel] : gen_f64(seed, rank, 2 * g);
        const double im = pattern == 1 ? -(double)seq : pattern == 2 ? (double)ft[(key >> 58) & 7]
                                                                     : gen_f64(seed, rank, 2 * g + 1);
        const uint64_t ur = (uint64_t)__double_as_longlong(re), ui = (uint64_t)__double_as_longlong(im);
        w[0] = (uint32_t)ur;
        w[1] = (uint32_t)(ur >> 32);
        w[2] = (uint32_t)ui;
        w[3] = (uint32_t)(ui >> 32);
        break;
    }
    }
    const int nw = dtype == CHR_DOUBLE_INT || dtype == CHR_LONG_INT || dtype == CHR_C_DOUBLE_COMPLEX ? 4 : 2;
    for (int k = 0; k < nw; ++k) ((uint32_t*)elem)[k] = w[k];
}

__global__ __launch_bounds__(kBlock) void k_fill(void* buf, size_t n, int dtype, int pattern, uint64_t seed,
                                                 uint64_t rank, uint64_t count_for_seq) {
    if (dtype >= CHR_FLOAT_INT) {
        const size_t es = dtype == CHR_DOUBLE_INT || dtype == CHR_LONG_INT || dtype == CHR_C_DOUBLE_COMPLEX ? 16 : 8;
        for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock)
            fill_pair((char*)buf + i * es, dtype, pattern, seed, rank, count_for_seq, i);
        return;
    }
    const int es = dtype == CHR_INT8 || dtype == CHR_UINT8 ? 1 : dtype == CHR_INT16 || dtype == CHR_UINT16 ? 2
                   : dtype == CHR_UINT32 || (dtype == CHR_INT32 && pattern == 3) ? 4
                   : dtype == CHR_INT64 || dtype == CHR_UINT64 ? 8 : 0;
    for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) {
        if (es) {  // the integer types beyond int32 (and int32's sparse pattern): seq = rank*count + i,
                   // ties = {0, 1, -1, 2, 7}, sparse = 1/8 zeros else nonzero random bits, uniform = the
                   // top 8*es random bits; truncated to the width (orc_fill_at)
            const uint64_t u = splitmix64(seed ^ (rank << 40) ^ (uint64_t)i);
            const unsigned sel = (unsigned)(u >> 61);
            const uint64_t v = pattern == 1   ? rank * count_for_seq + i
                               : pattern == 2 ? (uint64_t)(int64_t)(sel == 6 ? 2 : sel == 7 ? 7 : sel == 2 ? 1
                                                                    : sel == 3 ? -1 : 0)
                               : pattern == 3 ? (sel ? (u >> (64 - 8 * es)) | 1u : 0)
                                              : u >> (64 - 8 * es);
            if (es == 1) ((uint8_t*)buf)[i] = (uint8_t)v;
            else if (es == 2) ((uint16_t*)buf)[i] = (uint16_t)v;
            else if (es == 4) ((uint32_t*)buf)[i] = (uint32_t)v;
            else ((uint64_t*)buf)[i] = v;
            continue;
        }
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
