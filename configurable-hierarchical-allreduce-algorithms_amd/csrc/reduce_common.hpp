// reduce_common.hpp -- element semantics shared by the fused reduction kernels
// (reduce_kernels.hip: fan-in folds; reduce_tree.hip: whole expression trees).
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>

#include "chr_internal.hpp"

namespace chr {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef short i16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

constexpr int kBlock = 256;

// ---- element semantics -----------------------------------------------------------------

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
// f32 -> bf16, round to nearest even, NaN quieted as (u >> 16) | 0x40: the oracle's orc_f2bf.
// gfx950's v_cvt_pk_bf16_f32 (what clang emits for a float -> __bf16 conversion) gives exactly
// these bits for all 2^32 inputs (tools/bf16_cvt_check.hip, profiles/r01/bf16_cvt_check.json),
// so the kernels use it: one instruction per two elements instead of ~7 ALU ops per element.
__device__ __forceinline__ uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t f2bf_pk(float lo, float hi) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){lo, hi}, bf16x2));
}

// a + b and a * b with a's NaN surviving when both are NaN (see kSumSw): the operand order is written into the
// instruction, which the compiler cannot commute.  Rounding and every non-NaN result are those of the plain op.
__device__ __forceinline__ float add_keep(float a, float b) {
    float r;
    asm("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float mul_keep(float a, float b) {
    float r;
    asm("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double add_keep(double a, double b) {
    double r;
    asm("v_add_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double mul_keep(double a, double b) {
    double r;
    asm("v_mul_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ f32x2 pk_add_keep(f32x2 a, f32x2 b) {
    f32x2 r;
    asm("v_pk_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ f32x2 pk_mul_keep(f32x2 a, f32x2 b) {
    f32x2 r;
    asm("v_pk_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// MPI's pair types for MAXLOC / MINLOC and the C99 complex types, as element types of the kernels.
// A pair element is carried as its raw 32-bit words (the C struct {value; int index} MPI defines,
// padding included): MPICH replaces a whole element when the incoming one wins (padding bytes and
// all, tests/golden/pairs_reduce_local.npz), and a word copy does the same, where a struct copy may
// drop padding.  Value and index are read out of the words.
template <int NW>
struct RawPair {
    uint32_t w[NW];
};
struct PairFI : RawPair<2> {};  // {float v; int i;}        8 B
struct PairDI : RawPair<4> {};  // {double v; int i;}      16 B (4 B padding)
struct PairLI : RawPair<4> {};  // {long v; int i;}        16 B (4 B padding)
struct Pair2I : RawPair<2> {};  // {int v; int i;}          8 B
struct PairSI : RawPair<2> {};  // {short v; int i;}        8 B (2 B padding after v)
struct CplxF { float re, im; };
struct CplxD { double re, im; };
static_assert(sizeof(PairFI) == 8 && sizeof(PairDI) == 16 && sizeof(PairLI) == 16 && sizeof(Pair2I) == 8 &&
                  sizeof(PairSI) == 8 && sizeof(CplxF) == 8 && sizeof(CplxD) == 16,
              "pair / complex layouts");
__host__ __device__ __forceinline__ float pair_value(const PairFI& p) { return __builtin_bit_cast(float, p.w[0]); }
__host__ __device__ __forceinline__ double pair_value(const PairDI& p) {
    return __builtin_bit_cast(double, (uint64_t)p.w[0] | ((uint64_t)p.w[1] << 32));
}
__host__ __device__ __forceinline__ int64_t pair_value(const PairLI& p) {
    return (int64_t)((uint64_t)p.w[0] | ((uint64_t)p.w[1] << 32));
}
__host__ __device__ __forceinline__ int32_t pair_value(const Pair2I& p) { return (int32_t)p.w[0]; }
__host__ __device__ __forceinline__ int16_t pair_value(const PairSI& p) { return (int16_t)(p.w[0] & 0xFFFFu); }
template <int NW>
__host__ __device__ __forceinline__ constexpr int pair_index_word() { return NW == 2 ? 1 : 2; }

template <int DT> struct DTy;
template <> struct DTy<CHR_FLOAT32> { using T = float; };
template <> struct DTy<CHR_FLOAT64> { using T = double; };
template <> struct DTy<CHR_INT32> { using T = int32_t; };
template <> struct DTy<CHR_BFLOAT16> { using T = uint16_t; };
template <> struct DTy<CHR_INT8> { using T = int8_t; };
template <> struct DTy<CHR_UINT8> { using T = uint8_t; };
template <> struct DTy<CHR_INT16> { using T = int16_t; };
template <> struct DTy<CHR_UINT16> { using T = uint16_t; };
template <> struct DTy<CHR_UINT32> { using T = uint32_t; };
template <> struct DTy<CHR_INT64> { using T = int64_t; };
template <> struct DTy<CHR_UINT64> { using T = uint64_t; };
template <> struct DTy<CHR_FLOAT_INT> { using T = PairFI; };
template <> struct DTy<CHR_DOUBLE_INT> { using T = PairDI; };
template <> struct DTy<CHR_LONG_INT> { using T = PairLI; };
template <> struct DTy<CHR_2INT> { using T = Pair2I; };
template <> struct DTy<CHR_SHORT_INT> { using T = PairSI; };
template <> struct DTy<CHR_C_FLOAT_COMPLEX> { using T = CplxF; };
template <> struct DTy<CHR_C_DOUBLE_COMPLEX> { using T = CplxD; };

template <int DT>
constexpr bool is_pair_dt() { return DT >= CHR_FLOAT_INT && DT <= CHR_SHORT_INT; }
template <int DT>
constexpr bool is_complex_dt() { return DT == CHR_C_FLOAT_COMPLEX || DT == CHR_C_DOUBLE_COMPLEX; }

template <int DT>
constexpr bool is_float_dt() { return DT == CHR_FLOAT32 || DT == CHR_FLOAT64 || DT == CHR_BFLOAT16; }

// Internal op codes for the running-value-first order of MPICH_do_reduce
// (allreduce_recexch.cpp:147-186): each step is MPI_Reduce_local(running, next).  Integer SUM
// and PROD are bitwise commutative (wrapping); MAX/MIN differ on ties such as -0/+0 and on NaN
// compares, so they have their own codes.
constexpr int kMaxSw = 16, kMinSw = 17;
// SUM / PROD on the floating types are bitwise commutative except for one thing: when both operands are NaN, IEEE
// 754 leaves open whose payload survives.  The reference's loop (inout = inout + in, MPICH on x86) keeps inout's;
// gfx950 keeps the FIRST SOURCE OPERAND's (tools/nan_rule_probe.hip), and the compiler may commute a plain + or *
// (`a + b` and `b + a` both compiled to a-first there).  So the kernels pin the order in the instruction
// (add_keep / mul_keep above: the first argument's NaN survives), and the running-value-first order gets its own
// codes, as MAX / MIN do: kSumSw / kProdSw keep the incoming operand's NaN (tests/test_gpu_nan_payloads.py).
constexpr int kSumSw = 20, kProdSw = 21;
// The same for MAXLOC / MINLOC on the pairs with a floating value: a NaN compare keeps inout, and a
// tie keeps inout's value bits (-0 vs +0), so the operand order shows.
constexpr int kMaxLocSw = 18, kMinLocSw = 19;

// x86 SSE arithmetic with its NaN rules written out, for the complex types (the oracle's orc_x86f / orc_x86d):
// two NaNs -> the FIRST operand's, quieted; one NaN -> that NaN, quieted (sign and payload kept); an invalid
// operation on numbers (inf - inf, 0 * inf) -> x86's default NaN, sign set.  gfx950's v_add / v_mul follow the same
// three rules (tools/nan_invalid_probe.hip, profiles/r06/nan/nan_invalid.txt), but its v_sub_f32 flips the sign of a
// NaN second operand, and the compiler picks add operand orders freely, so the complex kernels spell the rules out as
// selects.  They are not on a BASELINE path; the f32 / f64 / bf16 reductions keep their one-instruction combines
// (add_keep / mul_keep), whose operand order is pinned and which never subtract.
enum { kXAdd, kXSub, kXMul };
__device__ __forceinline__ float quiet_nan(float v) { return __uint_as_float(__float_as_uint(v) | 0x00400000u); }
__device__ __forceinline__ double quiet_nan(double v) {
    return __longlong_as_double(__double_as_longlong(v) | 0x0008000000000000ll);
}
__device__ __forceinline__ float x86_default_nan(float) { return __uint_as_float(0xFFC00000u); }
__device__ __forceinline__ double x86_default_nan(double) { return __longlong_as_double((long long)0xFFF8000000000000ull); }
template <int XOP, typename F>
__device__ __forceinline__ F x86op(F p, F q) {
    const F r = XOP == kXAdd ? p + q : XOP == kXSub ? p - q : p * q;
    return __builtin_isnan(p) ? quiet_nan(p)
           : __builtin_isnan(q) ? quiet_nan(q)
           : __builtin_isnan(r) ? x86_default_nan(r)
                                : r;
}

// C99 Annex G complex multiplication as MPICH's `a = a * b` on `float _Complex` compiles (gcc, x86): the plain
// formula inline and, when both parts come out NaN, libgcc's __mulsc3 / __muldc3, which computes the products
// again (rounded one by one; the library is built with -ffp-contract=off) and, if both parts are still NaN, recovers
// the infinities (C11 G.5.1).  (a + bi) = inout, (c + di) = in.  Every input NaN makes both inline parts NaN, so the
// NaN that survives follows __mulsc3's operand order, which MPICH's own outputs pin (tests/golden/
// gen_nan_payloads.py, all orders searched: a*c, b*d, a*d, c*b, (ac) - (bd), (ad) + (bc), first operand first);
// the inline formula and the recalculation see numbers only, so they can only yield the default NaN.
template <typename F>
__device__ __forceinline__ void cmul(F a, F b, F c, F d, F* re, F* im) {
    F x = x86op<kXSub>(x86op<kXMul>(a, c), x86op<kXMul>(b, d));
    F y = x86op<kXAdd>(x86op<kXMul>(a, d), x86op<kXMul>(b, c));
    if (__builtin_isnan(x) && __builtin_isnan(y)) {  // __mulsc3
        const F ac = x86op<kXMul>(a, c), bd = x86op<kXMul>(b, d), ad = x86op<kXMul>(a, d), bc = x86op<kXMul>(c, b);
        x = x86op<kXSub>(ac, bd);
        y = x86op<kXAdd>(ad, bc);
        bool recalc = false;
        if (__builtin_isinf(a) || __builtin_isinf(b)) {
            a = __builtin_copysign(__builtin_isinf(a) ? (F)1 : (F)0, a);
            b = __builtin_copysign(__builtin_isinf(b) ? (F)1 : (F)0, b);
            if (__builtin_isnan(c)) c = __builtin_copysign((F)0, c);
            if (__builtin_isnan(d)) d = __builtin_copysign((F)0, d);
            recalc = true;
        }
        if (__builtin_isinf(c) || __builtin_isinf(d)) {
            c = __builtin_copysign(__builtin_isinf(c) ? (F)1 : (F)0, c);
            d = __builtin_copysign(__builtin_isinf(d) ? (F)1 : (F)0, d);
            if (__builtin_isnan(a)) a = __builtin_copysign((F)0, a);
            if (__builtin_isnan(b)) b = __builtin_copysign((F)0, b);
            recalc = true;
        }
        if (!recalc && (__builtin_isinf(ac) || __builtin_isinf(bd) || __builtin_isinf(ad) || __builtin_isinf(bc))) {
            if (__builtin_isnan(a)) a = __builtin_copysign((F)0, a);
            if (__builtin_isnan(b)) b = __builtin_copysign((F)0, b);
            if (__builtin_isnan(c)) c = __builtin_copysign((F)0, c);
            if (__builtin_isnan(d)) d = __builtin_copysign((F)0, d);
            recalc = true;
        }
        if (recalc) {
            const F inf = (F)__builtin_inf();
            x = x86op<kXMul>(inf, x86op<kXSub>(x86op<kXMul>(a, c), x86op<kXMul>(b, d)));
            y = x86op<kXMul>(inf, x86op<kXAdd>(x86op<kXMul>(a, d), x86op<kXMul>(b, c)));
        }
    }
    *re = x;
    *im = y;
}

// MPI_Reduce_local(in = x, inout = y): MPICH 3.3.2's loop is inout = OP(inout, in) with
// MAX(p, q) = p > q ? p : q (MPIR_OP_TYPE_REDUCE_CASE, a = inoutvec, b = invec), so MAX/MIN
// take `in` on ties (-0 / +0) and whenever a NaN makes the compare false (MAXLOC / MINLOC, whose loop
// replaces inout only by a strictly better in, keep inout there).  kMaxSw/kMinSw: the running value is the
// `in` operand and the result takes the place of the incoming buffer: OP(x, y).
template <int DT, int OP>
__device__ __forceinline__ typename DTy<DT>::T apply(typename DTy<DT>::T x, typename DTy<DT>::T y) {
    if constexpr (is_pair_dt<DT>()) {
        // MPICH's MAXLOC / MINLOC loop (a = inout, b = in): equal values keep a's words with the
        // lower index, a strictly better b replaces a (the whole element), else a stays
        if constexpr (OP == kMaxLocSw) return apply<DT, CHR_MAXLOC>(y, x);
        else if constexpr (OP == kMinLocSw) return apply<DT, CHR_MINLOC>(y, x);
        else {
            using T = typename DTy<DT>::T;
            constexpr int IW = pair_index_word<sizeof(T) / 4>();
            const auto vx = pair_value(x), vy = pair_value(y);
            T r = y;
            if (vy == vx) {
                const int32_t ix = (int32_t)x.w[IW], iy = (int32_t)y.w[IW];
                r.w[IW] = (uint32_t)(ix < iy ? ix : iy);
            } else if (OP == CHR_MAXLOC ? vy < vx : vy > vx) {
                r = x;
            }
            return r;
        }    } else if constexpr (is_complex_dt<DT>()) {
        // MPICH's complex SUM keeps in's NaN in each part (its compiled loop adds in + inout; tests/golden/
        // nan_reduce_local.npz), where MPI_FLOAT's keeps inout's.  kSumSw / kProdSw (the running value is `in`, the
        // result lands in the incoming buffer) are the plain ops on exchanged operands.
        typename DTy<DT>::T r;
        if constexpr (OP == CHR_SUM) {
            r.re = x86op<kXAdd>(x.re, y.re);
            r.im = x86op<kXAdd>(x.im, y.im);
        } else if constexpr (OP == kSumSw) {
            r.re = x86op<kXAdd>(y.re, x.re);
            r.im = x86op<kXAdd>(y.im, x.im);
        } else if constexpr (OP == CHR_PROD) {
            cmul(y.re, y.im, x.re, x.im, &r.re, &r.im);
        } else {
            static_assert(OP == kProdSw);
            cmul(x.re, x.im, y.re, y.im, &r.re, &r.im);
        }
        return r;
    } else if constexpr (DT == CHR_BFLOAT16) {
        const float fx = bf2f(x), fy = bf2f(y);
        if constexpr (OP == CHR_SUM) return f2bf(add_keep(fy, fx));
        else if constexpr (OP == CHR_PROD) return f2bf(mul_keep(fy, fx));
        else if constexpr (OP == kSumSw) return f2bf(add_keep(fx, fy));
        else if constexpr (OP == kProdSw) return f2bf(mul_keep(fx, fy));
        else if constexpr (OP == CHR_MAX) return fy > fx ? y : x;
        else if constexpr (OP == CHR_MIN) return fy < fx ? y : x;
        else if constexpr (OP == kMaxSw) return fx > fy ? x : y;
        else return fx < fy ? x : y;
    } else if constexpr (!is_float_dt<DT>()) {
        // integers (MPICH's C loops): wrapping SUM/PROD (computed unsigned, at least 32 bits wide,
        // so no signed overflow and no promotion surprises), MAX/MIN (ties are bitwise equal, so
        // the swapped orders coincide), logical ops with a 0/1 result, bitwise ops
        using T = typename DTy<DT>::T;
        using UT = std::make_unsigned_t<T>;
        using W = std::conditional_t<(sizeof(T) < 4), uint32_t, UT>;
        if constexpr (OP == CHR_SUM) return (T)(UT)((W)(UT)y + (W)(UT)x);
        else if constexpr (OP == CHR_PROD) return (T)(UT)((W)(UT)y * (W)(UT)x);
        else if constexpr (OP == CHR_MAX || OP == kMaxSw) return y > x ? y : x;
        else if constexpr (OP == CHR_MIN || OP == kMinSw) return y < x ? y : x;
        else if constexpr (OP == CHR_LAND) return (T)((y != 0) && (x != 0));
        else if constexpr (OP == CHR_LOR) return (T)((y != 0) || (x != 0));
        else if constexpr (OP == CHR_LXOR) return (T)((y != 0) != (x != 0));
        else if constexpr (OP == CHR_BAND) return (T)(y & x);
        else if constexpr (OP == CHR_BOR) return (T)(y | x);
        else return (T)(y ^ x);
    } else {
        using T = typename DTy<DT>::T;
        if constexpr (OP == CHR_SUM) return add_keep(y, x);  // inout's NaN survives (kSumSw)
        else if constexpr (OP == CHR_PROD) return mul_keep(y, x);
        else if constexpr (OP == kSumSw) return add_keep(x, y);
        else if constexpr (OP == kProdSw) return mul_keep(x, y);
        else if constexpr (OP == CHR_MAX) return y > x ? y : x;
        else if constexpr (OP == CHR_MIN) return y < x ? y : x;
        else if constexpr (OP == kMaxSw) return x > y ? x : y;
        else if constexpr (OP == kMinSw) return x < y ? x : y;
        // MPICH also accepts the logical ops on float/double (C truth: NaN true, -0 false)
        else if constexpr (OP == CHR_LAND) return (T)((y != 0) && (x != 0));
        else if constexpr (OP == CHR_LOR) return (T)((y != 0) || (x != 0));
        else return (T)((y != 0) != (x != 0));
    }
}

template <int DT, int OP>
__device__ __forceinline__ u32x4 apply_vec(u32x4 in, u32x4 acc) {
    // bitwise ops do not see element boundaries: whole dwords
    if constexpr (OP == CHR_BAND) return acc & in;
    if constexpr (OP == CHR_BOR) return acc | in;
    if constexpr (OP == CHR_BXOR) return acc ^ in;
    constexpr bool SUMLIKE = OP == CHR_SUM || OP == kSumSw, PRODLIKE = OP == CHR_PROD || OP == kProdSw;
    constexpr bool SW = OP == kSumSw || OP == kProdSw;  // the incoming operand's NaN survives
    if constexpr (DT == CHR_BFLOAT16 && (SUMLIKE || PRODLIKE)) {
        // two bf16 per dword: widen by shift / mask, one packed f32 op (operand order pinned), one packed RNE convert
        u32x4 r;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const f32x2 x2 = {__uint_as_float(in[e] << 16), __uint_as_float(in[e] & 0xFFFF0000u)};
            const f32x2 y2 = {__uint_as_float(acc[e] << 16), __uint_as_float(acc[e] & 0xFFFF0000u)};
            const f32x2 o = SUMLIKE ? (SW ? pk_add_keep(x2, y2) : pk_add_keep(y2, x2))
                                    : (SW ? pk_mul_keep(x2, y2) : pk_mul_keep(y2, x2));
            r[e] = f2bf_pk(o.x, o.y);
        }
        return r;
    }
    if constexpr (DT == CHR_INT8 || DT == CHR_UINT8) {
        // four bytes per dword, worked on in place (SIMD within a register): per-element code on sixteen byte lanes
        // per vector held the streaming kernels at 88-152 VGPRs, above the 72 RCCL's waves leave room for
        // (tests/test_kernel_resources.py).  Every result is MPICH's C loop's, bit for bit (integers: wrapping
        // SUM / PROD, ties bitwise equal, so the swapped MAX / MIN codes are the same op).
        constexpr uint32_t LO7 = 0x7F7F7F7Fu, HI = 0x80808080u, EVEN = 0x00FF00FFu;
        u32x4 r;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const uint32_t x = in[e], y = acc[e];
            if constexpr (OP == CHR_SUM) {
                r[e] = ((x & LO7) + (y & LO7)) ^ ((x ^ y) & HI);  // carries stay inside each byte
            } else if constexpr (OP == CHR_PROD) {
                // the low byte of a 16-bit product depends only on the operands' low bytes
                const uint32_t pe = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, x) * __builtin_bit_cast(u16x2, y));
                const uint32_t po = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, x >> 8) * __builtin_bit_cast(u16x2, y >> 8));
                r[e] = (pe & EVEN) | ((po << 8) & ~EVEN);
            } else if constexpr (OP == CHR_LAND || OP == CHR_LOR || OP == CHR_LXOR) {
                const uint32_t nx = (((x & LO7) + LO7) | x) & HI, ny = (((y & LO7) + LO7) | y) & HI;  // bit 7: byte != 0
                const uint32_t t = OP == CHR_LAND ? (nx & ny) : OP == CHR_LOR ? (nx | ny) : (nx ^ ny);
                r[e] = t >> 7;
            } else {
                // MAX / MIN: even and odd bytes as two 16-bit pairs, sign- or zero-extended in place, one packed
                // 16-bit max / min each, re-packed
                constexpr bool MX = OP == CHR_MAX || OP == kMaxSw;
                static_assert(OP == CHR_MAX || OP == CHR_MIN || OP == kMaxSw || OP == kMinSw);
                if constexpr (DT == CHR_INT8) {
                    const i16x2 xe = __builtin_bit_cast(i16x2, x << 8) >> 8, xo = __builtin_bit_cast(i16x2, x) >> 8;
                    const i16x2 ye = __builtin_bit_cast(i16x2, y << 8) >> 8, yo = __builtin_bit_cast(i16x2, y) >> 8;
                    const i16x2 re = MX ? __builtin_elementwise_max(ye, xe) : __builtin_elementwise_min(ye, xe);
                    const i16x2 ro = MX ? __builtin_elementwise_max(yo, xo) : __builtin_elementwise_min(yo, xo);
                    r[e] = (__builtin_bit_cast(uint32_t, re) & EVEN) | ((__builtin_bit_cast(uint32_t, ro) << 8) & ~EVEN);
                } else {
                    const u16x2 xe = __builtin_bit_cast(u16x2, x & EVEN), xo = __builtin_bit_cast(u16x2, (x >> 8) & EVEN);
                    const u16x2 ye = __builtin_bit_cast(u16x2, y & EVEN), yo = __builtin_bit_cast(u16x2, (y >> 8) & EVEN);
                    const u16x2 re = MX ? __builtin_elementwise_max(ye, xe) : __builtin_elementwise_min(ye, xe);
                    const u16x2 ro = MX ? __builtin_elementwise_max(yo, xo) : __builtin_elementwise_min(yo, xo);
                    r[e] = __builtin_bit_cast(uint32_t, re) | (__builtin_bit_cast(uint32_t, ro) << 8);
                }
            }
        }
        return r;
    }
    if constexpr (DT == CHR_FLOAT32 && (SUMLIKE || PRODLIKE)) {
        u32x4 r;
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
            const f32x2 x2 = {__uint_as_float(in[e]), __uint_as_float(in[e + 1])};
            const f32x2 y2 = {__uint_as_float(acc[e]), __uint_as_float(acc[e + 1])};
            const f32x2 o = SUMLIKE ? (SW ? pk_add_keep(x2, y2) : pk_add_keep(y2, x2))
                                    : (SW ? pk_mul_keep(x2, y2) : pk_mul_keep(y2, x2));
            r[e] = __float_as_uint(o.x);
            r[e + 1] = __float_as_uint(o.y);
        }
        return r;
    }
    using T = typename DTy<DT>::T;
    constexpr int E = 16 / sizeof(T);
    T a[E], b[E];
    __builtin_memcpy(a, &in, 16);
    __builtin_memcpy(b, &acc, 16);
#pragma unroll
    for (int e = 0; e < E; ++e) b[e] = apply<DT, OP>(a[e], b[e]);
    u32x4 r;
    __builtin_memcpy(&r, b, 16);
    return r;
}

// ---- XCD-aware workgroup -> trip map -----------------------------------------------------
// Workgroups are dispatched round-robin over the 8 XCDs (block b runs on XCD b % 8).  Every
// kernel here does one trip (BL x U vectors per operand) per workgroup.  With the identity map
// the 8 XCDs interleave at trip granularity (1-4 KiB); xcd_trip gives each XCD runs of C = 2^cs
// consecutive trips instead: block b's (b / 8)-th trip goes to run (b / 8) / C of XCD b % 8, and
// XCD x owns runs x, x + 8, x + 16, ...  Blocks from `full` on (past the last whole 8·C group of
// the grid, xcd_full) keep the identity, so the map is a bijection on [0, n).  Runs of 256-512 KiB measured +2-4 % on HBM-cold
// streams (tools/reduce_microbench focus8/focus9, profiles/r02/microbench_focus9_xcd_runs.txt):
// each XCD's translation caches and DRAM pages see fewer distinct pages per unit time, while
// the 8 XCDs still stream within a few MiB of each other.
__host__ __device__ __forceinline__ uint32_t xcd_full(uint32_t n, uint32_t cs) {
    return n & ~((8u << cs) - 1u);
}
__host__ __device__ __forceinline__ size_t xcd_trip(uint32_t b, uint32_t full, uint32_t cs) {
    if (b >= full) return b;
    const uint32_t x = b & 7u, i = b >> 3;
    return ((((size_t)(i >> cs)) * 8u + x) << cs) | (i & ((1u << cs) - 1u));
}

// Odd XCDs stream slower.  Stamped C2 launches (tools/reduce_microbench focus25-28,
// profiles/r04/c2_timeline/) have XCDs 1, 3, 5, 7 finishing 2.5-3 % after XCDs 0, 2, 4, 6, on every
// box measured, under every trip map (identity, 256 KiB / 1 MiB runs, runs shifted to the neighbour
// XCD), and in proportion to the launch size (16 MiB: 0.1 us, 64 MiB: 0.9 us, 256 MiB: 2.9 us):
// a rate, which follows the XCD and not the addresses.  Since every XCD gets exactly 1/8 of a
// grid's workgroups, the launch ends when the odd ones do.  xcd_trip_w rebalances statically: each
// odd XCD hands the last `hand` trips of its share to the even XCD below it (the even XCD runs them
// after its own; the odd XCD's last 2 x hand workgroups exit at once).  hand = per-XCD trips >> 6
// (1.6 %) balanced the end times at 64 MiB: span 30.68 -> 29.86 us (focus27, h = 16 / 32 / 48).
// The weighted region is blocks [0, full + 8 x hand), over trips [0, full); later blocks keep the
// identity (trip = block - 8 x hand).  kIdleTrip: a workgroup with nothing to do.
constexpr size_t kIdleTrip = ~(size_t)0;
constexpr int kXcdHandShift = 6;
// `env` < 0: the policy shift; 0: off; shifts past 31 hand nothing (a 32-bit shift by >= 32 is undefined)
inline uint32_t xcd_hand(uint32_t full, int env) {
    const int shift = env >= 0 ? env : kXcdHandShift;
    return shift <= 0 || shift > 31 ? 0u : (full >> 3) >> shift;
}
__host__ __device__ __forceinline__ size_t xcd_own(uint32_t x, uint32_t i, uint32_t cs) {
    return ((((size_t)(i >> cs)) * 8u + x) << cs) | (i & ((1u << cs) - 1u));
}
__host__ __device__ __forceinline__ size_t xcd_trip_w(uint32_t b, uint32_t full, uint32_t cs, uint32_t hand) {
    if (hand == 0) return xcd_trip(b, full, cs);
    if (b >= full + 8u * hand) return (size_t)(b - 8u * hand);
    const uint32_t x = b & 7u, i = b >> 3, q = full >> 3;
    if ((x & 1u) == 0) {
        if (i < q) return xcd_own(x, i, cs);
        return xcd_own(x + 1u, q - hand + (i - q), cs);  // i < q + hand in this region
    }
    return i < q - hand ? xcd_own(x, i, cs) : kIdleTrip;
}

// log2 of the trips in one XCD run for a launch of `trip_bytes` per operand per workgroup:
// CHR_XCD_RUN_KIB if set, else `policy_kib` (0 = identity map).
inline uint32_t xcd_run_shift(size_t policy_kib, size_t trip_bytes) {
    const int env = reduce_tuning().xcd_run_kib;
    const size_t kib = env >= 0 ? (size_t)env : policy_kib;
    uint32_t cs = 0;
    while (((size_t)2 << cs) * trip_bytes <= kib * 1024 && cs < 16) ++cs;
    return cs;
}

// Dynamic LDS per workgroup that caps the workgroups resident per CU (the kernels use no LDS; the
// allocation only caps occupancy).  env >= 0 overrides the policy (and stream_wg_cap below); 0 =
// uncapped.  Clamped to the
// per-workgroup limit (a cap of 1 asks for the whole CU).  Measured residency of one-wave workgroups
// per `cap` (tools/coresidency_probe --census, profiles/r03/coresidency/census.jsonl): 8 -> 8,
// 10 -> 9, 12 -> 11, 13 -> 12, 14 -> 14, 16 -> 16, uncapped -> 32 (the wave-slot limit).
inline int stream_wg_cap(int env, int policy);
inline unsigned nt_lds_bytes(int env, int policy) {
    const unsigned lds = reduce_tuning().lds_per_cu;
    const int cap = stream_wg_cap(env, policy);
    if (cap <= 0 || lds == 0) return 0;
    const unsigned b = (lds / (unsigned)cap) & ~255u;
    const unsigned lim = reduce_tuning().lds_per_block;
    return lim && b > lim ? lim & ~255u : b;
}

// Launches that share the GPU with RCCL's kernels.  Inside an overlapped collective the fused
// reductions of one pipeline slice run on the compute stream while RCCL's send/recv kernel of the
// next slice runs on the transfer stream, and RCCL's kernel needs a CU with room for 256 threads at
// ~288 VGPRs per wave plus 19 744 B of LDS (torch's RCCL) or 37 664 B (ROCm 7.2's).  With a
// streaming reduction resident on every CU, a kernel of that footprint was admitted within 3-31 us
// of its submission when the reduction ran at cap <= 12 (11 resident workgroups per CU), but only
// once the reduction launch drained (median ~170 us into a 200 us launch) at cap 14, 16 or uncapped
// (tools/coresidency_probe, profiles/r03/coresidency/).  Alone, the 8-leaf tree runs as fast at 12
// as at 16 in that probe, but the whole-call in-collective rows measured 2-3 % lower, so the
// tighter cap applies only where RCCL runs beside the launch: the executor opens a CoresidentScope
// around the local ops it puts on the compute stream of a multi-rank overlapped collective, and every
// streaming launch issued on that thread meanwhile takes at most kCoresidentWgPerCu (uncapped
// policies included; CoresidentScope in chr_internal.hpp).  An explicit CHR_WG_PER_CU_VEC / _TREE
// still wins.
inline int stream_wg_cap(int env, int policy) {
    if (env >= 0) return env;
    if (coresident_depth() > 0 && (policy <= 0 || policy > kCoresidentWgPerCu)) return kCoresidentWgPerCu;
    return policy;
}

// Materialise a wave-uniform pointer (a kernel argument) in SGPRs at this point: an empty asm
// with an SGPR operand, so every such pointer is loaded by the scalar loads at the kernel's top
// and waited for once, instead of being fetched lazily between vector loads.
template <typename P>
__device__ __forceinline__ void pin_sgpr(P* p) {
    asm volatile("" ::"s"(p));
}
template <typename P, typename Q>
__device__ __forceinline__ void pin_sgpr(P* p, Q* q, size_t n, uint32_t k, uint32_t f) {
    asm volatile("" ::"s"(p), "s"(q), "s"(n), "s"(k), "s"(f));
}
__device__ __forceinline__ void pin_sgpr_u32(uint32_t x, uint32_t y) {
    asm volatile("" ::"s"(x), "s"(y));
}
template <typename P, typename Q>
__device__ __forceinline__ void pin_sgpr(P* p, Q* q, size_t n, uint32_t k) {
    asm volatile("" ::"s"(p), "s"(q), "s"(n), "s"(k));
}

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

}  // namespace chr
