/*
 * chiara_oracle.c -- TEST INFRASTRUCTURE ONLY (see chiara_oracle.h).
 *
 * A bulk-synchronous, single-process restatement of every rank of CHiArA's
 * all_reduce_radix_batch / reduce_scatter_radix_batch.  Each block of code cites the
 * reference lines it follows (paths relative to /root/reference/Fugaku_experiments/).
 * All arithmetic goes through orc_reduce_local, the MPI_Reduce_local restatement.
 *
 * Why a bulk-synchronous simulation reproduces the MPI program exactly: inside one
 * recexch phase a participant only writes its own region R(phase, me) and only reads
 * its neighbours' copies of that same region, which those neighbours do not write in
 * that phase (neighbours differ in base-k digit `phase`, so their regions are
 * disjoint: all_reduce_radix_batch.cpp:106-131, :348-364).  Phase-2 roots only write
 * their own lane chunk, and read the other nodes' copies of it.  So executing the
 * ranks one after another per phase gives the same operands, in the same order, as
 * the message-passing program.  tests/test_oracle_golden.py pins this against the
 * real reference's outputs.
 */
#include "chiara_oracle.h"

#include <math.h>
#include <stdlib.h>

size_t orc_dtype_size(int dtype) {
    switch (dtype) {
    case ORC_F32: return 4;
    case ORC_F64: return 8;
    case ORC_I32: return 4;
    case ORC_BF16: return 2;
    case ORC_I8: case ORC_U8: return 1;
    case ORC_I16: case ORC_U16: return 2;
    case ORC_U32: return 4;
    case ORC_I64: case ORC_U64: return 8;
    case ORC_FI: case ORC_2I: case ORC_SI: case ORC_CF: return 8;
    case ORC_DI: case ORC_LI: case ORC_CD: return 16;
    default: return 0;
    }
}

int orc_commutative(int op) { return op != ORC_USER_HALFADD; }

int orc_valid(int dtype, int op) {
    if (op == ORC_USER_HALFADD || op == ORC_USER_HALFADD_C) return dtype == ORC_F32 || dtype == ORC_F64 || dtype == ORC_I32;
    if (!orc_dtype_size(dtype) || op < ORC_SUM || op > ORC_MINLOC) return 0;
    if (dtype >= ORC_FI && dtype <= ORC_SI) return op == ORC_MAXLOC || op == ORC_MINLOC;
    if (dtype == ORC_CF || dtype == ORC_CD) return op == ORC_SUM || op == ORC_PROD;
    if (op >= ORC_MAXLOC) return 0;
    if (dtype == ORC_BF16) return op <= ORC_MIN;
    if (dtype == ORC_F32 || dtype == ORC_F64) return op <= ORC_LXOR;
    return 1;
}

/* The pair and complex element structs (C layout, as MPI defines the types). */
typedef struct { float v; int32_t i; } orc_fi;
typedef struct { double v; int32_t i; } orc_di;
typedef struct { int64_t v; int32_t i; } orc_li;
typedef struct { int32_t v; int32_t i; } orc_2i;
typedef struct { int16_t v; int32_t i; } orc_si;
typedef struct { float re, im; } orc_cf;
typedef struct { double re, im; } orc_cd;

/* Pair and complex types: value = a small integer in [-4, 3] (UNIFORM / SPARSE; many ties, so
 * MAXLOC's lower-index rule is exercised), rank*count + i (SEQ, index = rank), or for the floating
 * pairs {+0, -0, 1, -1, 0.5, NaN with a per-rank payload} (TIES); index from 6 random bits.  Complex:
 * U[-1,1) parts from elements 2g and 2g + 1 of the float generator (UNIFORM), rank*count + i and its
 * negation (SEQ), the float TIES values.  Padding bytes are zero. */
static void orc_fill_pair(void* elem, int dtype, int pattern, uint64_t seed, int rank, uint64_t count_for_seq,
                          uint64_t g) {
    static const float ft[8] = {0.0f, -0.0f, 1.0f, -1.0f, 0.0f, -0.0f, 0.5f, 0.0f};
    const uint64_t key = orc_key(seed, (uint64_t)rank, g);
    const unsigned sel = (unsigned)(key >> 61);
    const uint32_t pay = (uint32_t)(rank + 1) & 0x3Fu;
    const int32_t small = (int32_t)(key >> 61) - 4;
    const int32_t idx = pattern == ORC_PAT_SEQ ? rank : (int32_t)((key >> 32) & 0x3F);
    const int32_t seq = (int32_t)(uint32_t)((uint64_t)rank * count_for_seq + g);
    memset(elem, 0, orc_dtype_size(dtype));
    if (dtype == ORC_FI || dtype == ORC_DI) {
        double v = pattern == ORC_PAT_SEQ ? (double)seq : (double)small;
        int nan = 0;
        if (pattern == ORC_PAT_TIES) {
            v = (double)ft[sel];
            nan = sel == 7;
        }
        if (dtype == ORC_FI) {
            orc_fi* e = (orc_fi*)elem;
            e->v = (float)v;
            if (nan) {
                uint32_t u = 0x7FC00000u | (pay << 16) | pay;
                memcpy(&e->v, &u, 4);
            } else if (pattern == ORC_PAT_TIES) {
                memcpy(&e->v, &ft[sel], 4); /* keeps the sign of -0 */
            }
            e->i = idx;
        } else {
            orc_di* e = (orc_di*)elem;
            e->v = v;
            if (nan) {
                uint64_t u = 0x7FF8000000000000ull | ((uint64_t)pay << 40) | pay;
                memcpy(&e->v, &u, 8);
            }
            e->i = idx;
        }
        return;
    }
    {
        const int64_t v = pattern == ORC_PAT_SEQ ? (int64_t)seq : (int64_t)small;
        switch (dtype) {
        case ORC_LI: ((orc_li*)elem)->v = v; ((orc_li*)elem)->i = idx; return;
        case ORC_2I: ((orc_2i*)elem)->v = (int32_t)v; ((orc_2i*)elem)->i = idx; return;
        case ORC_SI: ((orc_si*)elem)->v = (int16_t)v; ((orc_si*)elem)->i = idx; return;
        }
    }
    if (dtype == ORC_CF) {
        orc_cf* e = (orc_cf*)elem;
        if (pattern == ORC_PAT_SEQ) {
            e->re = (float)seq;
            e->im = -(float)seq;
        } else if (pattern == ORC_PAT_TIES) {
            e->re = ft[sel];
            e->im = ft[(key >> 58) & 7];
        } else {
            e->re = orc_gen_f32(seed, (uint64_t)rank, 2 * g);
            e->im = orc_gen_f32(seed, (uint64_t)rank, 2 * g + 1);
        }
    } else if (dtype == ORC_CD) {
        orc_cd* e = (orc_cd*)elem;
        if (pattern == ORC_PAT_SEQ) {
            e->re = (double)seq;
            e->im = -(double)seq;
        } else if (pattern == ORC_PAT_TIES) {
            e->re = (double)ft[sel];
            e->im = (double)ft[(key >> 58) & 7];
        } else {
            e->re = orc_gen_f64(seed, (uint64_t)rank, 2 * g);
            e->im = orc_gen_f64(seed, (uint64_t)rank, 2 * g + 1);
        }
    }
}

/* Elements [start, start + n) of rank `rank`'s input, written to buf[0 .. n): the same values as
 * orc_fill's, so windows of a full-size input can be generated without the whole buffer. */
void orc_fill_at(void* buf, size_t n, int dtype, int pattern, uint64_t seed, int rank,
                 uint64_t count_for_seq, uint64_t start) {
    size_t i;
    const size_t ies = ((dtype >= ORC_I8 && dtype <= ORC_U64) || (dtype == ORC_I32 && pattern == ORC_PAT_SPARSE))
                           ? orc_dtype_size(dtype) : 0;
    if (dtype >= ORC_FI && dtype <= ORC_CD) {
        const size_t es = orc_dtype_size(dtype);
        for (i = 0; i < n; ++i) orc_fill_pair((char*)buf + i * es, dtype, pattern, seed, rank, count_for_seq, start + i);
        return;
    }
    for (i = 0; i < n; ++i) {
        const uint64_t g = start + i;
        if (ies) {
            /* integer types beyond int32: SEQ = rank*count + i, TIES = {0, 1, -1, 2, 7}, UNIFORM = the
             * top 8*es random bits; stored truncated to the width (two's complement) */
            static const int64_t it8[8] = {0, 0, 1, -1, 0, 0, 2, 7};
            const uint64_t key = orc_key(seed, (uint64_t)rank, g);
            const uint64_t v = pattern == ORC_PAT_SEQ      ? (uint64_t)rank * count_for_seq + g
                               : pattern == ORC_PAT_TIES   ? (uint64_t)it8[key >> 61]
                               : pattern == ORC_PAT_SPARSE ? ((key >> 61) ? (key >> (64 - 8 * ies)) | 1u : 0)
                                                           : key >> (64 - 8 * ies);
            switch (ies) {
            case 1: ((uint8_t*)buf)[i] = (uint8_t)v; break;
            case 2: ((uint16_t*)buf)[i] = (uint16_t)v; break;
            case 4: ((uint32_t*)buf)[i] = (uint32_t)v; break;
            default: ((uint64_t*)buf)[i] = v; break;
            }
            continue;
        }
        if (pattern == ORC_PAT_SEQ) {
            /* Fugaku_experiments/Allreduce/main.cpp:48-49 (int wraps as on the reference). */
            uint32_t v = (uint32_t)((uint64_t)rank * count_for_seq + g);
            switch (dtype) {
            case ORC_F32: ((float*)buf)[i] = (float)(int32_t)v; break;
            case ORC_F64: ((double*)buf)[i] = (double)(int32_t)v; break;
            case ORC_I32: ((int32_t*)buf)[i] = (int32_t)v; break;
            case ORC_BF16: ((uint16_t*)buf)[i] = orc_f32_to_bf16((float)(int32_t)v); break;
            }
        } else if (pattern == ORC_PAT_TIES) {
            const unsigned sel = (unsigned)(orc_key(seed, (uint64_t)rank, g) >> 61);
            const uint32_t pay = (uint32_t)(rank + 1) & 0x3Fu;
            static const float ft[7] = {0.0f, -0.0f, 1.0f, -1.0f, 0.0f, -0.0f, 0.5f};
            static const int32_t it[8] = {0, 0, 1, -1, 0, 0, 2, 7};
            switch (dtype) {
            case ORC_F32: {
                uint32_t u;
                if (sel == 7) u = 0x7FC00000u | (pay << 16) | pay;
                else memcpy(&u, &ft[sel], 4);
                memcpy((char*)buf + 4 * i, &u, 4);
                break;
            }
            case ORC_F64: {
                double d;
                if (sel == 7) {
                    uint64_t u = 0x7FF8000000000000ull | ((uint64_t)pay << 40) | pay;
                    memcpy(&d, &u, 8);
                } else {
                    d = (double)ft[sel];
                }
                ((double*)buf)[i] = d;
                break;
            }
            case ORC_I32: ((int32_t*)buf)[i] = it[sel]; break;
            case ORC_BF16:
                ((uint16_t*)buf)[i] = sel == 7 ? (uint16_t)(0x7FC0u | pay) : orc_f32_to_bf16(ft[sel]);
                break;
            }
        } else {
            switch (dtype) {
            case ORC_F32: ((float*)buf)[i] = orc_gen_f32(seed, (uint64_t)rank, g); break;
            case ORC_F64: ((double*)buf)[i] = orc_gen_f64(seed, (uint64_t)rank, g); break;
            case ORC_I32: ((int32_t*)buf)[i] = (int32_t)(uint32_t)(orc_key(seed, (uint64_t)rank, g) >> 32); break;
            case ORC_BF16:
                ((uint16_t*)buf)[i] = orc_f32_to_bf16(orc_gen_f32(seed, (uint64_t)rank, g));
                break;
            }
        }
    }
}

void orc_fill(void* buf, size_t n, int dtype, int pattern, uint64_t seed, int rank,
              uint64_t count_for_seq) {
    orc_fill_at(buf, n, dtype, pattern, seed, rank, count_for_seq, 0);
}

/* MPICH 3.3.2 predefined ops (src/mpi/coll/op/opsum.c, opmax.c, ... via
 * MPIR_OP_TYPE_REDUCE_CASE): with a = inoutvec and b = invec the loop is
 * `a[i] = OP(a[i], b[i])`, OP(p, q) = p + q, p * q, (p > q ? p : q), (p < q ? p : q).  So
 * MAX/MIN take the in value on ties (-0/+0) and whenever a NaN makes the compare false (pinned by the
 * ties goldens; MAXLOC / MINLOC below keep inout there).
 * Below: x = in[i], y = inout[i], result = OP(y, x). */
#define ORC_LOOP(T, EXPR)                                     \
    do {                                                      \
        const T* a = (const T*)in;                            \
        T* b = (T*)inout;                                     \
        size_t i;                                             \
        for (i = 0; i < n; ++i) { T x = a[i], y = b[i]; b[i] = (EXPR); } \
    } while (0)

/* Integer types: MPICH's C loops on the type (two's complement wrap for SUM/PROD, computed here
 * in the unsigned type of at least 32 bits so C's promotions cannot overflow), LAND/LOR/LXOR give
 * 0 or 1 ((a && b), (a || b), (!a != !b)), BAND/BOR/BXOR the bitwise ops. */
#define ORC_INT_CASE(T, UT, WT)                                                          \
    switch (op) {                                                                        \
    case ORC_SUM: ORC_LOOP(T, (T)(UT)((WT)(UT)y + (WT)(UT)x)); break;                    \
    case ORC_PROD: ORC_LOOP(T, (T)(UT)((WT)(UT)y * (WT)(UT)x)); break;                   \
    case ORC_MAX: ORC_LOOP(T, y > x ? y : x); break;                                     \
    case ORC_MIN: ORC_LOOP(T, y < x ? y : x); break;                                     \
    case ORC_LAND: ORC_LOOP(T, (T)(y && x)); break;                                      \
    case ORC_LOR: ORC_LOOP(T, (T)(y || x)); break;                                       \
    case ORC_LXOR: ORC_LOOP(T, (T)(!y != !x)); break;                                    \
    case ORC_BAND: ORC_LOOP(T, (T)(y & x)); break;                                       \
    case ORC_BOR: ORC_LOOP(T, (T)(y | x)); break;                                        \
    case ORC_BXOR: ORC_LOOP(T, (T)(y ^ x)); break;                                       \
    }

/* MPICH 3.3.2's MAXLOC / MINLOC loop (src/mpi/coll/op/opmaxloc.c, opminloc.c; a = inoutvec,
 * b = invec): `if (a.value == b.value) a.loc = MIN(a.loc, b.loc); else if (a.value < b.value) a = b;`
 * (MINLOC: `>`).  Ties keep a's value bits (-0 vs +0), NaN compares keep a, a better b replaces the
 * whole element.  Pinned by tests/golden/pairs_reduce_local.npz (MPICH's own outputs). */
#define ORC_LOC_LOOP(T, BETTER)                                                      \
    do {                                                                             \
        const T* xs = (const T*)in;                                                  \
        T* ys = (T*)inout;                                                           \
        size_t i;                                                                    \
        for (i = 0; i < n; ++i) {                                                    \
            if (ys[i].v == xs[i].v) ys[i].i = xs[i].i < ys[i].i ? xs[i].i : ys[i].i; \
            else if (BETTER) memcpy(&ys[i], &xs[i], sizeof(T)); /* padding too */    \
        }                                                                            \
    } while (0)
#define ORC_LOC_CASE(T)                                        \
    if (op == ORC_MAXLOC) ORC_LOC_LOOP(T, ys[i].v < xs[i].v);  \
    else if (op == ORC_MINLOC) ORC_LOC_LOOP(T, ys[i].v > xs[i].v)

/* x86 SSE arithmetic with its NaN rules written out, so that the oracle does not depend on which operand order the
 * compiler of the oracle picks (the reference's MPICH loops run on x86):
 *   two NaNs      -> the FIRST operand's, quieted (sign and payload kept);
 *   one NaN       -> that NaN, quieted;
 *   invalid operation on numbers (inf - inf, 0 * inf) -> the x86 default NaN, sign set (0xFFC00000 /
 *                    0xFFF8000000000000).
 * Which operand of each add / multiply is first in MPICH's compiled loops is what tests/golden/nan_reduce_local.npz
 * (MPICH 3.3.2's own outputs on two-NaN, one-NaN and invalid operands) pins: inout first for MPI_FLOAT / MPI_DOUBLE
 * SUM and PROD (opsum.c, opprod.c: `a = a op b`, a = inoutvec); in first for the C complex SUM, both parts. */
enum { ORC_XADD, ORC_XSUB, ORC_XMUL };
static float orc_quietf(float v) {
    uint32_t u;
    memcpy(&u, &v, 4);
    u |= 0x00400000u;
    memcpy(&v, &u, 4);
    return v;
}
static double orc_quietd(double v) {
    uint64_t u;
    memcpy(&u, &v, 8);
    u |= 0x0008000000000000ull;
    memcpy(&v, &u, 8);
    return v;
}
static float orc_x86f(float p, float q, int op) {
    float r;
    if (isnan(p)) return orc_quietf(p);
    if (isnan(q)) return orc_quietf(q);
    r = op == ORC_XADD ? p + q : op == ORC_XSUB ? p - q : p * q;
    if (isnan(r)) {
        const uint32_t u = 0xFFC00000u;
        memcpy(&r, &u, 4);
    }
    return r;
}
static double orc_x86d(double p, double q, int op) {
    double r;
    if (isnan(p)) return orc_quietd(p);
    if (isnan(q)) return orc_quietd(q);
    r = op == ORC_XADD ? p + q : op == ORC_XSUB ? p - q : p * q;
    if (isnan(r)) {
        const uint64_t u = 0xFFF8000000000000ull;
        memcpy(&r, &u, 8);
    }
    return r;
}

/* C99 Annex G complex multiplication, as MPICH's `a = a * b` on `float _Complex` compiles (gcc): the plain formula
 * inline, and when both parts come out NaN a call to libgcc's __mulsc3 / __muldc3, which computes the products again
 * (rounded one by one; the library is built with -ffp-contract=off) and, if both parts are still NaN, recovers the
 * infinities (C11 G.5.1).  (a + bi) = inout, (c + di) = in.  Every input NaN makes both inline parts NaN, so the NaN
 * that survives is decided by __mulsc3's operand order, which MPICH's fixture pins (tests/golden/gen_nan_payloads.py,
 * searched over all orders: a*c, b*d, a*d, c*b, (ac) - (bd), (ad) + (bc), first operand first); the inline order and
 * the recalc order only ever see numbers, so only the default NaN of an invalid operation can come out of them. */
#define ORC_CMUL(F, X, INF, a_, b_, c_, d_, re_, im_)                                                               \
    do {                                                                                                           \
        F a = (a_), b = (b_), c = (c_), d = (d_);                                                                  \
        F ac = X(a, c, ORC_XMUL), bd = X(b, d, ORC_XMUL), ad = X(a, d, ORC_XMUL), bc = X(b, c, ORC_XMUL);         \
        F x = X(ac, bd, ORC_XSUB), y = X(ad, bc, ORC_XADD);                                                        \
        if (isnan(x) && isnan(y)) { /* __mulsc3 */                                                                 \
            int recalc = 0;                                                                                       \
            ac = X(a, c, ORC_XMUL), bd = X(b, d, ORC_XMUL), ad = X(a, d, ORC_XMUL), bc = X(c, b, ORC_XMUL);       \
            x = X(ac, bd, ORC_XSUB);                                                                               \
            y = X(ad, bc, ORC_XADD);                                                                               \
            if (isinf(a) || isinf(b)) {                                                                            \
                a = copysign(isinf(a) ? (F)1 : (F)0, a);                                                           \
                b = copysign(isinf(b) ? (F)1 : (F)0, b);                                                           \
                if (isnan(c)) c = copysign((F)0, c);                                                               \
                if (isnan(d)) d = copysign((F)0, d);                                                               \
                recalc = 1;                                                                                        \
            }                                                                                                      \
            if (isinf(c) || isinf(d)) {                                                                            \
                c = copysign(isinf(c) ? (F)1 : (F)0, c);                                                           \
                d = copysign(isinf(d) ? (F)1 : (F)0, d);                                                           \
                if (isnan(a)) a = copysign((F)0, a);                                                               \
                if (isnan(b)) b = copysign((F)0, b);                                                               \
                recalc = 1;                                                                                        \
            }                                                                                                      \
            if (!recalc && (isinf(ac) || isinf(bd) || isinf(ad) || isinf(bc))) {                                   \
                if (isnan(a)) a = copysign((F)0, a);                                                               \
                if (isnan(b)) b = copysign((F)0, b);                                                               \
                if (isnan(c)) c = copysign((F)0, c);                                                               \
                if (isnan(d)) d = copysign((F)0, d);                                                               \
                recalc = 1;                                                                                        \
            }                                                                                                      \
            if (recalc) {                                                                                          \
                x = X((F)(INF), X(X(a, c, ORC_XMUL), X(b, d, ORC_XMUL), ORC_XSUB), ORC_XMUL);                      \
                y = X((F)(INF), X(X(a, d, ORC_XMUL), X(b, c, ORC_XMUL), ORC_XADD), ORC_XMUL);                      \
            }                                                                                                      \
        }                                                                                                          \
        (re_) = x;                                                                                                 \
        (im_) = y;                                                                                                 \
    } while (0)

void orc_reduce_local(const void* in, void* inout, size_t n, int dtype, int op) {
    switch (dtype) {
    case ORC_FI: ORC_LOC_CASE(orc_fi); break;
    case ORC_DI: ORC_LOC_CASE(orc_di); break;
    case ORC_LI: ORC_LOC_CASE(orc_li); break;
    case ORC_2I: ORC_LOC_CASE(orc_2i); break;
    case ORC_SI: ORC_LOC_CASE(orc_si); break;
    case ORC_CF: {
        const orc_cf* xs = (const orc_cf*)in;
        orc_cf* ys = (orc_cf*)inout;
        size_t i;
        for (i = 0; i < n; ++i) {
            if (op == ORC_SUM) { /* in's NaN survives, each part (MPICH's fixture) */
                ys[i].re = orc_x86f(xs[i].re, ys[i].re, ORC_XADD);
                ys[i].im = orc_x86f(xs[i].im, ys[i].im, ORC_XADD);
            } else {
                ORC_CMUL(float, orc_x86f, INFINITY, ys[i].re, ys[i].im, xs[i].re, xs[i].im, ys[i].re, ys[i].im);
            }
        }
        break;
    }
    case ORC_CD: {
        const orc_cd* xs = (const orc_cd*)in;
        orc_cd* ys = (orc_cd*)inout;
        size_t i;
        for (i = 0; i < n; ++i) {
            if (op == ORC_SUM) {
                ys[i].re = orc_x86d(xs[i].re, ys[i].re, ORC_XADD);
                ys[i].im = orc_x86d(xs[i].im, ys[i].im, ORC_XADD);
            } else {
                ORC_CMUL(double, orc_x86d, INFINITY, ys[i].re, ys[i].im, xs[i].re, xs[i].im, ys[i].re, ys[i].im);
            }
        }
        break;
    }
    /* MPICH 3.3.2 also takes LAND/LOR/LXOR on float and double (probed: rc 0), C truth values. */
    case ORC_F32:
        if (op == ORC_USER_HALFADD || op == ORC_USER_HALFADD_C)
            ORC_LOOP(float, x * 0.5f + y); /* the user op: inout = in o inout */
        else if (op == ORC_SUM) ORC_LOOP(float, orc_x86f(y, x, ORC_XADD)); /* inout's NaN survives */
        else if (op == ORC_PROD) ORC_LOOP(float, orc_x86f(y, x, ORC_XMUL));
        else if (op == ORC_MAX) ORC_LOOP(float, y > x ? y : x);
        else if (op == ORC_MIN) ORC_LOOP(float, y < x ? y : x);
        else if (op == ORC_LAND) ORC_LOOP(float, (float)(y && x));
        else if (op == ORC_LOR) ORC_LOOP(float, (float)(y || x));
        else if (op == ORC_LXOR) ORC_LOOP(float, (float)(!y != !x));
        break;
    case ORC_F64:
        if (op == ORC_USER_HALFADD || op == ORC_USER_HALFADD_C) ORC_LOOP(double, x * 0.5 + y);
        else if (op == ORC_SUM) ORC_LOOP(double, orc_x86d(y, x, ORC_XADD));
        else if (op == ORC_PROD) ORC_LOOP(double, orc_x86d(y, x, ORC_XMUL));
        else if (op == ORC_MAX) ORC_LOOP(double, y > x ? y : x);
        else if (op == ORC_MIN) ORC_LOOP(double, y < x ? y : x);
        else if (op == ORC_LAND) ORC_LOOP(double, (double)(y && x));
        else if (op == ORC_LOR) ORC_LOOP(double, (double)(y || x));
        else if (op == ORC_LXOR) ORC_LOOP(double, (double)(!y != !x));
        break;
    case ORC_I32:
        if (op == ORC_USER_HALFADD || op == ORC_USER_HALFADD_C) ORC_LOOP(int32_t, (int32_t)((uint32_t)x * 3u + (uint32_t)y));
        else ORC_INT_CASE(int32_t, uint32_t, uint32_t)
        break;
    case ORC_I8: ORC_INT_CASE(int8_t, uint8_t, uint32_t) break;
    case ORC_U8: ORC_INT_CASE(uint8_t, uint8_t, uint32_t) break;
    case ORC_I16: ORC_INT_CASE(int16_t, uint16_t, uint32_t) break;
    case ORC_U16: ORC_INT_CASE(uint16_t, uint16_t, uint32_t) break;
    case ORC_U32: ORC_INT_CASE(uint32_t, uint32_t, uint32_t) break;
    case ORC_I64: ORC_INT_CASE(int64_t, uint64_t, uint64_t) break;
    case ORC_U64: ORC_INT_CASE(uint64_t, uint64_t, uint64_t) break;
    case ORC_BF16:
        /* The reference has no bf16; the golden driver runs it as a user-defined op on
         * MPI_Type_contiguous(2, MPI_BYTE) computing bf16_rne(f32(inout) op f32(in)) with the
         * same operand order as the predefined float ops: inout first, with x86's NaN rules (orc_x86f). */
        if (op == ORC_SUM)
            ORC_LOOP(uint16_t, orc_f32_to_bf16(orc_x86f(orc_bf16_to_f32(y), orc_bf16_to_f32(x), ORC_XADD)));
        else if (op == ORC_PROD)
            ORC_LOOP(uint16_t, orc_f32_to_bf16(orc_x86f(orc_bf16_to_f32(y), orc_bf16_to_f32(x), ORC_XMUL)));
        else if (op == ORC_MAX)
            ORC_LOOP(uint16_t, orc_bf16_to_f32(y) > orc_bf16_to_f32(x) ? y : x);
        else
            ORC_LOOP(uint16_t, orc_bf16_to_f32(y) < orc_bf16_to_f32(x) ? y : x);
        break;
    }
}

void orc_reduce_multi(void* acc, const void* const* ins, int m, size_t n, int dtype, int op) {
    int j;
    for (j = 0; j < m; ++j) orc_reduce_local(ins[j], acc, n, dtype, op);
}

/* ---- recexch tables: all_reduce_radix_batch.cpp:11-198 ---------------------------- */

int orc_recexch_neighbors(int rank, int nranks, int k, orc_recexch_t* o) {
    int i, j, p_of_k = 1, log_p_of_k = 0, rem, T, newrank;
    memset(o, 0, sizeof(*o));
    if (k < 2) return 1;
    if (nranks < k) k = (nranks > 2) ? nranks : 2;                       /* :19-21 */
    if (k > 64) return 1;
    o->k = k;
    while (p_of_k <= nranks) { p_of_k *= k; log_p_of_k++; }               /* :23-28 */
    p_of_k /= k;
    log_p_of_k--;
    if (log_p_of_k > 32) return 1;
    o->step2_nphases = log_p_of_k;                                         /* :45 */
    rem = nranks - p_of_k;                                                 /* :47 */
    T = (rem * k) / (k - 1);                                               /* :49 */
    o->T = T;
    o->p_of_k = p_of_k;
    o->rem = rem;
    o->step1_nrecvs = 0;
    o->step1_sendto = -1;
    if (rank < T) {                                                        /* :56-70 */
        if (rank % k != (k - 1)) {
            o->step1_sendto = rank + (k - 1 - rank % k);
            if (o->step1_sendto > T - 1) o->step1_sendto = T;
            newrank = -1;
        } else {
            for (i = 0; i < k - 1; i++) o->step1_recvfrom[i] = rank - i - 1;
            o->step1_nrecvs = k - 1;
            newrank = rank / k;
        }
    } else {                                                               /* :71-82 */
        newrank = rank - rem;
        if (rank == T && (T - 1) % k != k - 1 && T >= 1) {
            int nsenders = (T - 1) % k + 1;
            for (j = nsenders - 1; j >= 0; j--) o->step1_recvfrom[nsenders - 1 - j] = T - nsenders + j;
            o->step1_nrecvs = nsenders;
        }
    }
    if (o->step1_sendto == -1) {                                           /* :84-134 */
        int digit[32];
        int temprank = newrank, mask = 1, phase = 0, i_digit = 0;
        for (i = 0; i < log_p_of_k; i++) digit[i] = 0;
        while (temprank != 0) {
            digit[i_digit++] = temprank % k;
            temprank /= k;
        }
        while (mask < p_of_k) {
            int cbit = digit[phase], cnt = 0;
            for (i = 0; i < k; i++) {
                if (i != cbit) {
                    int nbr = 0, power = 1;
                    digit[phase] = i;
                    for (j = 0; j < log_p_of_k; j++) { nbr += digit[j] * power; power *= k; }
                    o->step2_nbrs[phase][cnt++] = (nbr < rem / (k - 1)) ? (nbr * k) + (k - 1) : nbr + rem;
                }
            }
            digit[phase] = cbit;
            phase++;
            mask *= k;
        }
    }
    return 0;
}

static int orc_step2_to_orig(int r, int rem, int k) {                      /* :152-161 */
    return (r < rem / (k - 1)) ? (r * k) + (k - 1) : r + rem;
}

void orc_recexch_count_offset(int nranks, int max_phases, int k, int* count, int* offset) {
    int p_of_k = 1, rem, T, phase, rank, kpp = 1;                          /* :163-198 */
    while (p_of_k <= nranks) p_of_k *= k;
    p_of_k /= k;
    rem = nranks - p_of_k;
    T = (rem * k) / (k - 1);
    for (phase = 0; phase < max_phases; phase++) {
        for (rank = 0; rank < nranks; rank++) {
            int s2 = (rank < T) ? rank / k : rank - rem;                   /* :140-149 */
            int mn = ((s2 / kpp) * kpp) - 1;
            int mx = mn + kpp;
            int omn = (mn >= 0) ? orc_step2_to_orig(mn, rem, k) : mn;
            int omx = orc_step2_to_orig(mx, rem, k);
            count[phase * nranks + rank] = omx - omn;
            offset[phase * nranks + rank] = omn + 1;
        }
        kpp *= k;
    }
}

/* ---- phases 0-2, shared by allreduce and reduce-scatter ---------------------------- */

typedef struct {
    int nranks, b, k, nnodes, nstages, nu_count, nph;
    size_t recvcount, irc, total, es;
    orc_recexch_t* rx; /* per lane */
    int *cnt, *off;
    char **tres, **trecv; /* per-rank tmp_results / tmp_recvbuf */
} orc_state;

static void orc_free_state(orc_state* s) {
    int r;
    if (s->tres)
        for (r = 0; r < s->nranks; r++) free(s->tres[r]);
    if (s->trecv)
        for (r = 0; r < s->nranks; r++) free(s->trecv[r]);
    free(s->tres);
    free(s->trecv);
    free(s->rx);
    free(s->cnt);
    free(s->off);
}

#define ORC_AT(buf, elem) ((buf) + (size_t)(elem) * s->es)

/* Runs phases 0-2 (all_reduce_radix_batch.cpp:234-539 ==
 * reduce_scatter_radix_batch.cpp:228-562).  Afterwards the fully reduced chunk N
 * (IRC elements) lives at trecv[N*b + N%b] + (N/b)*IRC. */
static int orc_phases_0_2(orc_state* s, int nranks, int k_in, int b, size_t recvcount,
                          int dtype, int op, const void* const* send, void* const* recv) {
    int r, l, node, st, ph, i;
    memset(s, 0, sizeof(*s));
    if (b < 1 || nranks < 1 || nranks % b != 0 || k_in < 2) return 1;
    s->es = orc_dtype_size(dtype);
    if (!s->es || !orc_valid(dtype, op)) return 1;
    s->nranks = nranks;
    s->b = b;
    s->recvcount = recvcount;
    s->nnodes = nranks / b;                                                /* :241-244 */
    s->nstages = s->nnodes / b;
    s->nu_count = s->nnodes % b;                                           /* :258 */
    s->irc = recvcount * (size_t)b;                                        /* :249 */
    s->total = recvcount * (size_t)nranks;                                 /* :254 */
    s->rx = (orc_recexch_t*)calloc((size_t)b, sizeof(orc_recexch_t));
    for (l = 0; l < b; l++)
        if (orc_recexch_neighbors(l, b, k_in, &s->rx[l])) return 1;     /* :283 */
    s->k = s->rx[0].k;
    s->nph = s->rx[0].step2_nphases;
    s->cnt = (int*)calloc((size_t)(s->nph * b + 1), sizeof(int));
    s->off = (int*)calloc((size_t)(s->nph * b + 1), sizeof(int));
    orc_recexch_count_offset(b, s->nph, s->k, s->cnt, s->off);            /* :288 */
    s->tres = (char**)calloc((size_t)nranks, sizeof(char*));
    s->trecv = (char**)calloc((size_t)nranks, sizeof(char*));
    for (r = 0; r < nranks; r++) {
        s->tres[r] = (char*)calloc(s->total + 1, s->es);                   /* :296-297 */
        s->trecv[r] = (char*)calloc(s->total + 1, s->es);
        if (!s->tres[r] || !s->trecv[r]) return 3;
    }
#define SB(rr) ((const char*)(send[rr] ? send[rr] : recv[rr]))
    /* Phase 0 (:306-312): participants copy their input into tmp_results. */
    for (r = 0; r < nranks; r++)
        if (s->rx[r % b].step1_sendto == -1) memcpy(s->tres[r], SB(r), s->total * s->es);
    /* Phase 1a step-1 fold (:315-335): reduce the whole buffers of the non-participants,
     * in step1_recvfrom order. */
    for (r = 0; r < nranks; r++) {
        const orc_recexch_t* x = &s->rx[r % b];
        node = r / b;
        if (x->step1_sendto != -1) continue;
        for (i = 0; i < x->step1_nrecvs; i++)
            orc_reduce_local(SB(x->step1_recvfrom[i] + b * node), s->tres[r], s->total, dtype, op);
    }
    /* Phase 1b: full stages (:339-400) and 1c: the truncated leftover stage (:404-478). */
    for (st = 0; st <= s->nstages; st++) {
        size_t base = (size_t)st * b * s->irc;
        int leftover = (st == s->nstages);
        if (leftover && s->nu_count == 0) break;
        for (ph = s->nph - 1; ph >= 0; ph--) {
            for (r = 0; r < nranks; r++) {
                const orc_recexch_t* x = &s->rx[r % b];
                l = r % b;
                node = r / b;
                if (x->step1_sendto != -1) continue;
                for (i = 0; i < s->k - 1; i++) {
                    int dst = x->step2_nbrs[ph][i];
                    int rc = s->cnt[ph * b + l], o = s->off[ph * b + l];
                    if (leftover) {                                        /* :432-446 */
                        int mrc = rc < (s->nu_count - o) ? rc : (s->nu_count - o);
                        if (!(o < s->nu_count && mrc > 0)) continue;
                        rc = mrc;
                    }
                    /* :364 / :446 -- MPI_Reduce_local(tmp_recvbuf, tmp_results + off). */
                    orc_reduce_local(ORC_AT(s->tres[dst + b * node], base + (size_t)o * s->irc),
                                     ORC_AT(s->tres[r], base + (size_t)o * s->irc),
                                     (size_t)rc * s->irc, dtype, op);
                }
            }
        }
        /* phase_buf[st] (:372-385, :459-473): own block for participants, block returned
         * by the step-1 partner for non-participants. */
        for (r = 0; r < nranks; r++) {
            const orc_recexch_t* x = &s->rx[r % b];
            l = r % b;
            node = r / b;
            if (leftover && l >= s->nu_count) continue;
            if (x->step1_sendto == -1)
                memcpy(ORC_AT(s->trecv[r], (size_t)st * s->irc),
                       ORC_AT(s->tres[r], base + (size_t)l * s->irc), s->irc * s->es);
            else
                memcpy(ORC_AT(s->trecv[r], (size_t)st * s->irc),
                       ORC_AT(s->tres[x->step1_sendto + b * node], base + (size_t)l * s->irc),
                       s->irc * s->es);
        }
    }
    /* Phase 2 inter-node linear reduce to rotating lane roots (:498-539). */
    {
        int nIters = (s->nu_count == 0) ? s->nstages : 1 + s->nstages;
        for (l = 0; l < b; l++) {
            for (i = 0; i < nIters; i++) {
                int root_node = i * b + l, X;
                char* acc;
                if (root_node >= s->nnodes) break;
                acc = ORC_AT(s->trecv[root_node * b + l], (size_t)i * s->irc);
                for (X = 0; X < s->nnodes; X++) {
                    if (X == root_node) continue;
                    /* :529 MPI_Reduce_local(incoming stage X chunk, tmp_recvbuf + i*IRC) */
                    orc_reduce_local(ORC_AT(s->trecv[X * b + l], (size_t)i * s->irc), acc, s->irc,
                                     dtype, op);
                }
            }
        }
    }
#undef SB
    return 0;
}

static const char* orc_chunk(const orc_state* s, int N) {
    int b = s->b;
    return s->trecv[N * b + N % b] + (size_t)(N / b) * s->irc * s->es;
}

int orc_allreduce_radix_batch(int nranks, int k, int b, size_t count, int dtype, int op,
                              const void* const* send, void* const* recv) {
    orc_state st;
    int rc, R, N;
    if (nranks < 1 || count % (size_t)nranks != 0) return 2; /* :239 truncates silently */
    rc = orc_phases_0_2(&st, nranks, k, b, count / (size_t)nranks, dtype, op, send, recv);
    if (rc) { orc_free_state(&st); return rc; }
    /* Phases 3-4 (:552-756) are pure data movement: lane roots broadcast their chunk
     * across nodes, then a k-Bruck allgather inside each node; every rank ends with
     * chunk N at recvbuf + N*IRC.  (Golden vectors confirm the reference does exactly
     * that on every geometry in the grid.) */
    for (R = 0; R < nranks; R++)
        for (N = 0; N < st.nnodes; N++)
            memcpy((char*)recv[R] + (size_t)N * st.irc * st.es, orc_chunk(&st, N), st.irc * st.es);
    orc_free_state(&st);
    return 0;
}

int orc_reduce_scatter_radix_batch(int nranks, int k, int b, size_t recvcount, int dtype,
                                   int op, const void* const* send, void* const* recv) {
    orc_state st;
    int rc, N, j;
    rc = orc_phases_0_2(&st, nranks, k, b, recvcount, dtype, op, send, recv);
    if (rc) { orc_free_state(&st); return rc; }
    /* Root re-layout + intra k-nomial scatter + own-block copy (:572-627): rank N*b+j
     * receives sub-block j of reduced chunk N. */
    for (N = 0; N < st.nnodes; N++)
        for (j = 0; j < b; j++)
            memcpy(recv[N * b + j], orc_chunk(&st, N) + (size_t)j * recvcount * st.es, recvcount * st.es);
    orc_free_state(&st);
    return 0;
}

/* ==== MPICH baseline allreduces driven by testing/main.cpp ============
 * Paths relative to /root/reference/testing/mpich_implementations/all_reduce/.  Every rank's
 * buffers live in one process; each step reads the sending rank's buffer region that the
 * sender does not modify in that step (disjoint regions), or a snapshot where both ends
 * update the whole buffer (recursive doubling / exchange). */

static void orc_copy_in(int n, size_t count, size_t es, const void* const* send, void* const* recv) {
    int r;
    for (r = 0; r < n; r++)
        if (send[r]) memcpy(recv[r], send[r], count * es);
}

/* MPICH_Allreduce_ring (allreduce_ring.cpp:3-104) */
int orc_allreduce_ring(int n, size_t count, int dtype, int op, const void* const* send, void* const* recv) {
    size_t es = orc_dtype_size(dtype), total = 0, *cnts, *displs;
    int i, r;
    char** R = (char**)recv;
    if (n < 1 || !es) return 1;
    cnts = (size_t*)calloc((size_t)n, sizeof(size_t));
    displs = (size_t*)calloc((size_t)n, sizeof(size_t));
    for (i = 0; i < n; i++) { /* :31-38 */
        cnts[i] = (count + (size_t)n - 1) / (size_t)n;
        if (total + cnts[i] > count) {
            cnts[i] = count - total;
            break;
        }
        total += cnts[i];
    }
    for (i = 1; i < n; i++) displs[i] = displs[i - 1] + cnts[i - 1];
    orc_copy_in(n, count, es, send, recv); /* :44-47 */
    for (i = 0; i < n - 1; i++) {          /* :56-84 */
        for (r = 0; r < n; r++) {
            int src = (n + r - 1) % n, recv_rank = (2 * n + r - 2 - i) % n;
            /* src sends its block recv_rank (its send_rank), reduced into mine (:80) */
            orc_reduce_local(R[src] + displs[recv_rank] * es, R[r] + displs[recv_rank] * es, cnts[recv_rank],
                             dtype, op);
        }
    }
    for (r = 0; r < n; r++) /* MPI_Allgatherv (:86): block j comes from rank j */
        for (i = 0; i < n; i++)
            if (i != r) memcpy(R[r] + displs[i] * es, R[i] + displs[i] * es, cnts[i] * es);
    free(cnts);
    free(displs);
    return 0;
}

/* MPICH_Allreduce_recursive_doubling (allreduce_recursive_doubling.cpp:4-101).  A non-commutative op keeps rank
 * order (:69-80): the partner's buffer is the left operand when it is the lower rank, else the right one. */
int orc_allreduce_recursive_doubling(int n, size_t count, int dtype, int op, const void* const* send,
                                     void* const* recv) {
    size_t es = orc_dtype_size(dtype);
    int pof2 = 1, rem, r, mask;
    char** R = (char**)recv;
    char* snap;
    if (n < 1 || !es) return 1;
    orc_copy_in(n, count, es, send, recv);
    while (pof2 <= n) pof2 <<= 1;
    pof2 >>= 1;
    rem = n - pof2;
    for (r = 1; r < 2 * rem; r += 2) orc_reduce_local(R[r - 1], R[r], count, dtype, op); /* :35-50 */
    snap = (char*)malloc(count * es * (size_t)n + 1);
    for (mask = 1; mask < pof2; mask <<= 1) { /* :59-85 */
        for (r = 0; r < n; r++) memcpy(snap + (size_t)r * count * es, R[r], count * es);
        for (r = 0; r < n; r++) {
            int newrank = r < 2 * rem ? (r % 2 ? r / 2 : -1) : r - rem, newdst, dst;
            if (newrank < 0) continue;
            newdst = newrank ^ mask;
            dst = newdst < rem ? newdst * 2 + 1 : newdst + rem;
            if (orc_commutative(op) || dst < r) {
                orc_reduce_local(snap + (size_t)dst * count * es, R[r], count, dtype, op); /* :70 */
            } else { /* :75-79: MPI_Reduce_local(recvbuf, tmp_buf), then tmp_buf -> recvbuf */
                char* t = (char*)malloc(count * es + 1);
                memcpy(t, snap + (size_t)dst * count * es, count * es);
                orc_reduce_local(R[r], t, count, dtype, op);
                memcpy(R[r], t, count * es);
                free(t);
            }
        }
    }
    free(snap);
    for (r = 0; r < 2 * rem; r += 2) memcpy(R[r], R[r + 1], count * es); /* :88-97 */
    return 0;
}

/* MPICH_Allreduce_reduce_scatter_allgather (allreduce_reduce_scatter_allgather.cpp:3-173) */
int orc_allreduce_reduce_scatter_allgather(int n, size_t count, int dtype, int op, const void* const* send,
                                           void* const* recv) {
    size_t es = orc_dtype_size(dtype);
    int pof2 = 1, rem, r, i, mask;
    char** R = (char**)recv;
    size_t *cnts, *disps;
    int *send_idx, *recv_idx, *last_idx;
    if (n < 1 || !es) return 1;
    orc_copy_in(n, count, es, send, recv);
    while (pof2 <= n) pof2 *= 2;
    pof2 /= 2;
    rem = n - pof2;
    for (r = 1; r < 2 * rem; r += 2) orc_reduce_local(R[r - 1], R[r], count, dtype, op); /* :28-51 */
    cnts = (size_t*)calloc((size_t)pof2, sizeof(size_t));
    disps = (size_t*)calloc((size_t)pof2, sizeof(size_t));
    for (i = 0; i < pof2; i++) cnts[i] = count / (size_t)pof2 + ((size_t)i < count % (size_t)pof2 ? 1 : 0);
    for (i = 1; i < pof2; i++) disps[i] = disps[i - 1] + cnts[i - 1];
    send_idx = (int*)calloc((size_t)n, sizeof(int));
    recv_idx = (int*)calloc((size_t)n, sizeof(int));
    last_idx = (int*)calloc((size_t)n, sizeof(int));
    for (r = 0; r < n; r++) last_idx[r] = pof2;
#define NEWRANK(rr) ((rr) < 2 * rem ? ((rr) % 2 ? (rr) / 2 : -1) : (rr) - rem)
#define REALRANK(nr) ((nr) < rem ? (nr) * 2 + 1 : (nr) + rem)
    for (mask = 1; mask < pof2; mask <<= 1) { /* reduce-scatter :76-117 */
        /* indices first (every rank), then data: rank r reduces [recv_idx, ...) from dst's buffer */
        int *rs = (int*)calloc((size_t)n, sizeof(int)), *re = (int*)calloc((size_t)n, sizeof(int));
        for (r = 0; r < n; r++) {
            int nr = NEWRANK(r), nd;
            if (nr < 0) continue;
            nd = nr ^ mask;
            if (nr < nd) {
                send_idx[r] = recv_idx[r] + pof2 / (mask * 2);
                rs[r] = recv_idx[r];
                re[r] = send_idx[r];
            } else {
                recv_idx[r] = send_idx[r] + pof2 / (mask * 2);
                rs[r] = recv_idx[r];
                re[r] = last_idx[r];
            }
        }
        for (r = 0; r < n; r++) {
            int nr = NEWRANK(r), dst;
            size_t cnt = 0;
            if (nr < 0) continue;
            dst = REALRANK(nr ^ mask);
            for (i = rs[r]; i < re[r]; i++) cnt += cnts[i];
            orc_reduce_local(R[dst] + disps[rs[r]] * es, R[r] + disps[rs[r]] * es, cnt, dtype, op); /* :104 */
        }
        for (r = 0; r < n; r++) {
            if (NEWRANK(r) < 0) continue;
            send_idx[r] = recv_idx[r];
            if ((mask << 1) < pof2) last_idx[r] = recv_idx[r] + pof2 / (mask << 1);
        }
        free(rs);
        free(re);
    }
    /* allgather (:119-160): pure data movement; after it every participant holds all blocks */
    {
        int nr;
        char* full = (char*)malloc(count * es + 1);
        for (nr = 0; nr < pof2; nr++) {
            /* newrank nr ends the reduce-scatter owning block index (bit-reversal is not used here:
             * the owner of block b is the participant whose final recv_idx == b) */
            (void)nr;
        }
        for (r = 0; r < n; r++) {
            if (NEWRANK(r) < 0) continue;
            memcpy(full + disps[recv_idx[r]] * es, R[r] + disps[recv_idx[r]] * es, cnts[recv_idx[r]] * es);
        }
        for (r = 0; r < n; r++)
            if (NEWRANK(r) >= 0) memcpy(R[r], full, count * es);
        free(full);
    }
#undef NEWRANK
#undef REALRANK
    for (r = 0; r < 2 * rem; r += 2) memcpy(R[r], R[r + 1], count * es); /* :161-171 */
    free(cnts);
    free(disps);
    free(send_idx);
    free(recv_idx);
    free(last_idx);
    return 0;
}

/* MPICH_do_reduce (allreduce_recexch.cpp:147-186): acc_{i+1} = OP(acc_i, next): the running
 * value is the `in` operand. */
static void orc_do_reduce(char** bufs, char* recvbuf, int k, int idx, size_t count, int dtype, int op) {
    int i;
    size_t es = orc_dtype_size(dtype);
    for (i = 0; i < idx - 1; i++) orc_reduce_local(bufs[i], bufs[i + 1], count, dtype, op);
    if (idx > 0) orc_reduce_local(bufs[idx - 1], recvbuf, count, dtype, op);
    if (idx < k - 1) {
        orc_reduce_local(recvbuf, bufs[idx], count, dtype, op);
        for (i = idx; i < k - 2; i++) orc_reduce_local(bufs[i], bufs[i + 1], count, dtype, op);
        memcpy(recvbuf, bufs[k - 2], count * es);
    }
}

/* MPICH_Allreduce_recursive_exchange (allreduce_recexch.cpp:188-440), float path (myidx from
 * MPICH_find_myidx, :137-145); single_phase_recv changes buffering only, not the data flow. */
int orc_allreduce_recexch(int n, int k_in, size_t count, int dtype, int op, const void* const* send,
                          void* const* recv) {
    size_t es = orc_dtype_size(dtype);
    int r, i, ph, k;
    char** R = (char**)recv;
    orc_recexch_t* x;
    char *snap, **bufs;
    if (n < 1 || !es || k_in < 2) return 1;
    orc_copy_in(n, count, es, send, recv);
    if (n == 1) return 0;
    x = (orc_recexch_t*)calloc((size_t)n, sizeof(orc_recexch_t));
    for (r = 0; r < n; r++)
        if (orc_recexch_neighbors(r, n, k_in, &x[r])) {
            free(x);
            return 1;
        }
    k = x[0].k;
    for (r = 0; r < n; r++) /* step 1 (:267-296) */
        if (x[r].step1_sendto == -1)
            for (i = 0; i < x[r].step1_nrecvs; i++) orc_reduce_local(R[x[r].step1_recvfrom[i]], R[r], count, dtype, op);
    snap = (char*)malloc(count * es * (size_t)n + 1);
    bufs = (char**)calloc((size_t)k, sizeof(char*));
    for (i = 0; i < k; i++) bufs[i] = (char*)malloc(count * es + 1);
    for (ph = 0; ph < x[0].step2_nphases; ph++) { /* step 2 (:298-365) */
        for (r = 0; r < n; r++) memcpy(snap + (size_t)r * count * es, R[r], count * es);
        for (r = 0; r < n; r++) {
            int idx = k - 1;
            if (x[r].step1_sendto != -1) continue;
            for (i = 0; i < k - 1; i++) memcpy(bufs[i], snap + (size_t)x[r].step2_nbrs[ph][i] * count * es, count * es);
            for (i = 0; i < k - 1; i++) /* MPICH_find_myidx */
                if (x[r].step2_nbrs[ph][i] > r) {
                    idx = i;
                    break;
                }
            orc_do_reduce(bufs, R[r], k, idx, count, dtype, op);
        }
    }
    for (r = 0; r < n; r++) /* step 3 (:367-386) */
        if (x[r].step1_sendto != -1) memcpy(R[r], R[x[r].step1_sendto], count * es);
    for (i = 0; i < k; i++) free(bufs[i]);
    free(bufs);
    free(snap);
    free(x);
    return 0;
}

/* ---- testing/mpich_implementations/all_reduce/allreduce_recursive_multiplying.cpp ---- */

/* running-value-first chain over seq[0..m-1] (MPI_Reduce_local(running, next) per step),
 * result into out. */
static void orc_chain_running_first(char* const* seq, int m, char* out, size_t count, int dtype, int op) {
    size_t nb = count * orc_dtype_size(dtype);
    char* run = (char*)malloc(nb + 1);
    char* nxt = (char*)malloc(nb + 1);
    int j;
    memcpy(run, seq[0], nb);
    for (j = 1; j < m; j++) {
        char* t;
        memcpy(nxt, seq[j], nb);
        orc_reduce_local(run, nxt, count, dtype, op);
        t = run;
        run = nxt;
        nxt = t;
    }
    memcpy(out, run, nb);
    free(run);
    free(nxt);
}

int orc_allreduce_recursive_multiplying(int n, int k, size_t count, int dtype, int op, const void* const* send,
                                        void* const* recv) {
    size_t es = orc_dtype_size(dtype), nb;
    int r, pofk = 1, distance, next_distance;
    char** R = (char**)recv;
    char *snap, **seq;
    if (n < 1 || !es || k < 2) return 1;
    nb = count * es;
    orc_copy_in(n, count, es, send, recv);
    while (pofk * k <= n) pofk *= k; /* :13-17 */
    if (pofk < n && !orc_commutative(op)) return 8; /* :43-49: MPI_ERR_OP ("non pofk works only for commutative") */
    seq = (char**)calloc((size_t)(n > k ? n : k) + 1, sizeof(char*));
    if (pofk < n) /* :43-86: rank r < pofk folds r+pofk, r+2pofk, ... then its own buffer */
        for (r = 0; r < pofk; r++) {
            int m = 0, src;
            for (src = r + pofk; src < n; src += pofk) seq[m++] = R[src];
            if (!m) continue;
            seq[m++] = R[r];
            orc_chain_running_first(seq, m, R[r], count, dtype, op);
        }
    snap = (char*)malloc(nb * (size_t)n + 1);
    for (distance = 1, next_distance = k; distance < pofk; distance = next_distance, next_distance *= k) {
        for (r = 0; r < pofk; r++) memcpy(snap + (size_t)r * nb, R[r], nb);
        for (r = 0; r < pofk; r++) { /* :88-152: group members ascending, folded left */
            int start = r / next_distance * next_distance, m = 0, dst;
            for (dst = start + r % distance; dst < start + next_distance; dst += distance)
                seq[m++] = snap + (size_t)dst * nb;
            orc_chain_running_first(seq, m, R[r], count, dtype, op);
        }
    }
    for (r = pofk; r < n; r++) memcpy(R[r], R[r % pofk], nb); /* :154-172 */
    free(snap);
    free(seq);
    return 0;
}

/* ---- testing/mpich_implementations/all_reduce/allreduce_k_reduce_scatter_allgather.cpp ---- */

static int orc_reverse_digits_step2(int rank, int n, int k) { /* :66-120 */
    int pofk = 1, log_pofk = 0, rem, T, s2, i, rev = 0, power = 1;
    int digit[32];
    while (pofk <= n) { pofk *= k; log_pofk++; }
    pofk /= k;
    log_pofk--;
    rem = n - pofk;
    T = (rem * k) / (k - 1);
    s2 = (rank < T) ? rank / k : rank - rem;
    for (i = 0; i < log_pofk; i++) digit[i] = 0;
    for (i = 0; s2 != 0; i++) { digit[i] = s2 % k; s2 /= k; }
    for (i = 0; i < log_pofk; i++) { rev += digit[log_pofk - 1 - i] * power; power *= k; }
    return orc_step2_to_orig(rev, rem, k);
}

static void orc_krsag_block(int rank, int level, int n, int k, const size_t* cnts, const size_t* displs,
                            size_t* off, size_t* cnt) { /* :25-63 on the reversed rank */
    int pofk = 1, rem, T, s2, kpp = 1, mn, mx, omn, omx, x;
    int rr = orc_reverse_digits_step2(rank, n, k);
    while (pofk <= n) pofk *= k;
    pofk /= k;
    rem = n - pofk;
    T = (rem * k) / (k - 1);
    while (level-- > 0) kpp *= k;
    s2 = (rr < T) ? rr / k : rr - rem;
    mn = ((s2 / kpp) * kpp) - 1;
    mx = mn + kpp;
    omn = (mn >= 0) ? orc_step2_to_orig(mn, rem, k) : mn;
    omx = orc_step2_to_orig(mx, rem, k);
    *off = displs[omn + 1];
    *cnt = 0;
    for (x = 0; x < omx - omn; x++) *cnt += cnts[omn + 1 + x];
}

int orc_allreduce_k_reduce_scatter_allgather(int n, int k_in, size_t count, int dtype, int op,
                                             const void* const* send, void* const* recv) {
    size_t es = orc_dtype_size(dtype), nb;
    int r, i, p, k, nph, pofk, rem;
    char** R = (char**)recv;
    orc_recexch_t* x;
    size_t *cnts, *displs;
    char* snap;
    if (n < 1 || !es) return 1;
    if (k_in <= 1) k_in = 2; /* :273-275 */
    if (!orc_commutative(op)) return 8; /* :278-283: MPI_ERR_OP for a non-commutative op */
    nb = count * es;
    orc_copy_in(n, count, es, send, recv);
    x = (orc_recexch_t*)calloc((size_t)n, sizeof(orc_recexch_t));
    for (r = 0; r < n; r++)
        if (orc_recexch_neighbors(r, n, k_in, &x[r])) {
            free(x);
            return 1;
        }
    k = x[0].k;
    nph = x[0].step2_nphases;
    pofk = x[0].p_of_k;
    rem = n - pofk;
    for (r = 0; r < n; r++) /* step 1 (:313-333) */
        if (x[r].step1_sendto == -1)
            for (i = 0; i < x[r].step1_nrecvs; i++) orc_reduce_local(R[x[r].step1_recvfrom[i]], R[r], count, dtype, op);
    /* block sizes (:335-351); the last participant (always rank n-1: rem/(k-1) < p_of_k)
     * takes the remainder */
    cnts = (size_t*)calloc((size_t)n + 1, sizeof(size_t));
    displs = (size_t*)calloc((size_t)n + 1, sizeof(size_t));
    for (i = 0; i < pofk - 1; i++) cnts[orc_step2_to_orig(i, rem, k)] = count / (size_t)pofk;
    cnts[n - 1] = count - (count / (size_t)pofk) * (size_t)(pofk - 1);
    for (i = 1; i < n; i++) displs[i] = displs[i - 1] + cnts[i - 1];
    snap = (char*)malloc(nb * (size_t)n + 1);
    for (p = 0; p < nph; p++) { /* reduce-scatter (:353-401): level j = nph-1-p */
        const int j = nph - 1 - p;
        for (r = 0; r < n; r++) memcpy(snap + (size_t)r * nb, R[r], nb);
        for (r = 0; r < n; r++) {
            size_t off, cnt;
            if (x[r].step1_sendto != -1) continue;
            orc_krsag_block(r, j, n, k, cnts, displs, &off, &cnt);
            for (i = 0; i < k - 1; i++)
                orc_reduce_local(snap + (size_t)x[r].step2_nbrs[p][i] * nb + off * es, R[r] + off * es, cnt, dtype, op);
        }
    }
    for (p = 0; p < nph; p++) { /* allgather (:403-493): level p with phase nph-1-p nbrs */
        const int ph = nph - 1 - p;
        for (r = 0; r < n; r++) memcpy(snap + (size_t)r * nb, R[r], nb);
        for (r = 0; r < n; r++) {
            if (x[r].step1_sendto != -1) continue;
            for (i = 0; i < k - 1; i++) {
                size_t off, cnt;
                const int nbr = x[r].step2_nbrs[ph][i];
                orc_krsag_block(nbr, p, n, k, cnts, displs, &off, &cnt);
                memcpy(R[r] + off * es, snap + (size_t)nbr * nb + off * es, cnt * es);
            }
        }
    }
    for (r = 0; r < n; r++) /* step 3 (:496-520) */
        if (x[r].step1_sendto != -1) memcpy(R[r], R[x[r].step1_sendto], nb);
    free(snap);
    free(cnts);
    free(displs);
    free(x);
    return 0;
}

/* ---- Fugaku_experiments/Allgather/all_gather_radix_batch_1_0.cpp:37 ---------------------
 * Pure data movement; the reference's output is the rank-major concatenation of the send
 * blocks on every geometry of tests/golden (its k-nomial gather :55-133, linear inter-root
 * exchange :137-163 and k-Bruck :168-360 only decide the route).  Preconditions as the
 * product: k >= 2, b >= 1, nranks % b == 0.  send[r] NULL = in place (block already at
 * recv[r] + r*count). */
int orc_allgather_radix_batch(int n, int k, int b, size_t count, int dtype, const void* const* send,
                              void* const* recv) {
    size_t es = orc_dtype_size(dtype), nb;
    int r, j;
    char** R = (char**)recv;
    if (n < 1 || !es || k < 2 || b < 1) return 1;
    if (n % b) return 3;
    nb = count * es;
    for (r = 0; r < n; r++) {
        const char* src = send[r] ? (const char*)send[r] : R[r] + (size_t)r * nb;
        for (j = 0; j < n; j++)
            if (j != r || send[j]) memmove(R[j] + (size_t)r * nb, src, nb);
    }
    return 0;
}

/* ---- MPICH baseline reduce-scatters (block): testing/mpich_implementations/reduce_scatter/ ---- */
/* Every rank's input is send[r] (n*rc elements) or, under MPI_IN_PLACE (send[r] == NULL), recv[r];
 * every rank's result (rc elements) goes to recv[r][0 .. rc).  Results are written only after
 * every rank's computation, so in place the inputs stay intact while they are read. */

static const char* orc_rs_input(const void* const* send, void* const* recv, int r) {
    return send && send[r] ? (const char*)send[r] : (const char*)recv[r];
}

static void orc_rs_store(int n, size_t rc, size_t es, char** res, void* const* recv) {
    int r;
    for (r = 0; r < n; r++) {
        memcpy(recv[r], res[r], rc * es);
        free(res[r]);
    }
    free(res);
}

/* reduce_scatter_pairwise.cpp:4-74: own block, then the block from rank (r - i) for i = 1..n-1,
 * each MPI_Reduce_local(tmp, result) (:54 / :56). */
int orc_reduce_scatter_pairwise(int n, size_t rc, int dtype, int op, const void* const* send, void* const* recv) {
    size_t es = orc_dtype_size(dtype);
    char** res;
    int r, i;
    if (n < 1 || !es) return 1;
    res = (char**)calloc((size_t)n, sizeof(char*));
    for (r = 0; r < n; r++) {
        res[r] = (char*)malloc(rc * es + 1);
        memcpy(res[r], orc_rs_input(send, recv, r) + (size_t)r * rc * es, rc * es);
        for (i = 1; i < n; i++) {
            int src = (r - i + n) % n;
            orc_reduce_local(orc_rs_input(send, recv, src) + (size_t)r * rc * es, res[r], rc, dtype, op);
        }
    }
    orc_rs_store(n, rc, es, res, recv);
    return 0;
}

/* reduce_scatter_recursive_halving.cpp:7-153. */
int orc_reduce_scatter_rec_halving(int n, size_t rc, int dtype, int op, const void* const* send,
                                   void* const* recv) {
    size_t es = orc_dtype_size(dtype), total = rc * (size_t)n, *cnts, *disps;
    int pof2 = 1, rem, r, i, mask;
    char **tmp, **snap, **res;
    int *newrank, *send_idx, *recv_idx, *last_idx;
    if (n < 1 || !es) return 1;
    while (pof2 <= n) pof2 *= 2; /* :40-46 */
    pof2 = pof2 == n ? pof2 : pof2 / 2;
    rem = n - pof2;
    tmp = (char**)calloc((size_t)n, sizeof(char*));
    snap = (char**)calloc((size_t)n, sizeof(char*));
    res = (char**)calloc((size_t)n, sizeof(char*));
    newrank = (int*)calloc((size_t)n, sizeof(int));
    send_idx = (int*)calloc((size_t)n, sizeof(int));
    recv_idx = (int*)calloc((size_t)n, sizeof(int));
    last_idx = (int*)calloc((size_t)n, sizeof(int));
    for (r = 0; r < n; r++) {
        tmp[r] = (char*)malloc(total * es + 1);
        snap[r] = (char*)malloc(total * es + 1);
        res[r] = (char*)malloc(rc * es + 1);
        memcpy(tmp[r], orc_rs_input(send, recv, r), total * es); /* :34-38 */
    }
    for (r = 0; r < n; r++) { /* :50-66: odd r < 2*rem folds its even partner's whole buffer */
        if (r < 2 * rem) {
            newrank[r] = r % 2 ? r / 2 : -1;
            if (r % 2) orc_reduce_local(tmp[r - 1], tmp[r], total, dtype, op);
        } else {
            newrank[r] = r - rem;
        }
        send_idx[r] = recv_idx[r] = 0;
        last_idx[r] = pof2;
    }
    cnts = (size_t*)calloc((size_t)pof2, sizeof(size_t));
    disps = (size_t*)calloc((size_t)pof2, sizeof(size_t));
    for (i = 0; i < pof2; i++) { /* :74-86 */
        int old_i = i < rem ? i * 2 + 1 : i + rem;
        cnts[i] = old_i < 2 * rem ? 2 * rc : rc;
        if (i) disps[i] = disps[i - 1] + cnts[i - 1];
    }
    for (mask = pof2 >> 1; mask > 0; mask >>= 1) { /* :91-128, every rank from the pre-step state */
        for (r = 0; r < n; r++) memcpy(snap[r], tmp[r], total * es);
        for (r = 0; r < n; r++) {
            int nr = newrank[r], newdst, dst, j;
            size_t recv_cnt = 0;
            if (nr < 0) continue;
            newdst = nr ^ mask;
            dst = newdst < rem ? newdst * 2 + 1 : newdst + rem;
            if (nr < newdst) {
                send_idx[r] = recv_idx[r] + mask;
                for (j = recv_idx[r]; j < send_idx[r]; j++) recv_cnt += cnts[j];
            } else {
                recv_idx[r] = send_idx[r] + mask;
                for (j = recv_idx[r]; j < last_idx[r]; j++) recv_cnt += cnts[j];
            }
            /* the partner sends exactly this range of its tmp_results (:112-117) */
            if (recv_cnt)
                orc_reduce_local(snap[dst] + disps[recv_idx[r]] * es, tmp[r] + disps[recv_idx[r]] * es, recv_cnt,
                                 dtype, op);
            send_idx[r] = recv_idx[r];
            last_idx[r] = recv_idx[r] + mask;
        }
    }
    for (r = 0; r < n; r++) { /* :130, :137-143 */
        if (newrank[r] >= 0) memcpy(res[r], tmp[r] + (size_t)r * rc * es, rc * es);
        else memcpy(res[r], tmp[r + 1] + (size_t)r * rc * es, rc * es);
    }
    for (r = 0; r < n; r++) {
        free(tmp[r]);
        free(snap[r]);
    }
    free(tmp);
    free(snap);
    free(cnts);
    free(disps);
    free(newrank);
    free(send_idx);
    free(recv_idx);
    free(last_idx);
    orc_rs_store(n, rc, es, res, recv);
    return 0;
}

/* reduce_scatter_recursive_doubling.cpp:10-177.  A non-commutative op (:132-160) reduces the received blocks as the
 * left operand only when the partner's subtree is the lower one; otherwise tmp_results is the left operand, reduced
 * into tmp_recvbuf and copied back (the Sendrecv-to-self at :158). */
int orc_reduce_scatter_rec_doubling(int n, size_t rc, int dtype, int op, const void* const* send,
                                    void* const* recv) {
    const int P = n;
    size_t es = orc_dtype_size(dtype), total = rc * (size_t)n;
    char **tmp, **trecv, **res;
    int *received, r, mask, stage;
    if (n < 1 || !es) return 1;
    tmp = (char**)calloc((size_t)n, sizeof(char*));
    trecv = (char**)calloc((size_t)n, sizeof(char*));
    res = (char**)calloc((size_t)n, sizeof(char*));
    received = (int*)calloc((size_t)n, sizeof(int));
    for (r = 0; r < n; r++) {
        tmp[r] = (char*)malloc(total * es + 1);
        trecv[r] = (char*)calloc(total * es + 1, 1);
        res[r] = (char*)malloc(rc * es + 1);
        memcpy(tmp[r], orc_rs_input(send, recv, r), total * es); /* :31-40 */
    }
    for (mask = 1, stage = 0; mask < P; mask <<= 1, stage++) { /* :52-168 */
        /* receive blocks (:71-81): everything outside the partner's subtree */
        for (r = 0; r < n; r++) {
            int dst = r ^ mask, dtr = (dst >> stage) << stage;
            size_t r0 = rc * (size_t)(dtr < P ? dtr : P);
            size_t r1 = P - (dtr + mask) > 0 ? (size_t)(P - (dtr + mask)) * rc : 0;
            size_t r1off = r0 + rc * (size_t)(((dtr + mask) < P ? (dtr + mask) : P) - dtr);
            received[r] = 0;
            if (dst < P) { /* :98-104: the partner's tmp_results at these blocks (not yet reduced) */
                memcpy(trecv[r], tmp[dst], r0 * es);
                memcpy(trecv[r] + r1off * es, tmp[dst] + r1off * es, r1 * es);
                received[r] = 1;
            }
        }
        if ((P & (P - 1)) != 0) { /* :106-130, level by level (tmp_mask decreasing) */
            int level_mask, kk = 0, j;
            for (j = mask; j >>= 1;) kk++;
            for (level_mask = mask >> 1; level_mask; level_mask >>= 1, kk--) {
                for (r = 0; r < n; r++) {
                    int dst = r ^ mask, dtr = (dst >> stage) << stage, mtr = (r >> stage) << stage;
                    int npc = P - mtr - mask, sd = r ^ level_mask, tree_root = (r >> kk) << kk;
                    if (!(dtr + mask > P)) continue;
                    if (sd < r && sd < tree_root + npc && r >= tree_root + npc) {
                        size_t r0 = rc * (size_t)(dtr < P ? dtr : P);
                        size_t r1 = P - (dtr + mask) > 0 ? (size_t)(P - (dtr + mask)) * rc : 0;
                        size_t r1off = r0 + rc * (size_t)(((dtr + mask) < P ? (dtr + mask) : P) - dtr);
                        memcpy(trecv[r], trecv[sd], r0 * es); /* the relaying rank's recvtype blocks */
                        memcpy(trecv[r] + r1off * es, trecv[sd] + r1off * es, r1 * es);
                        received[r] = 1;
                    }
                }
            }
        }
        for (r = 0; r < n; r++) { /* :132-155: tmp_results op= received blocks */
            int dst = r ^ mask, dtr = (dst >> stage) << stage;
            size_t r0 = rc * (size_t)(dtr < P ? dtr : P);
            size_t r1 = P - (dtr + mask) > 0 ? (size_t)(P - (dtr + mask)) * rc : 0;
            size_t r1off = r0 + rc * (size_t)(((dtr + mask) < P ? (dtr + mask) : P) - dtr);
            const int mtr = (r >> stage) << stage;
            if (!received[r]) continue;
            if (orc_commutative(op) || dtr < mtr) {
                if (r0) orc_reduce_local(trecv[r], tmp[r], r0, dtype, op);
                if (r1) orc_reduce_local(trecv[r] + r1off * es, tmp[r] + r1off * es, r1, dtype, op);
            } else {
                if (r0) {
                    orc_reduce_local(tmp[r], trecv[r], r0, dtype, op);
                    memcpy(tmp[r], trecv[r], r0 * es);
                }
                if (r1) {
                    orc_reduce_local(tmp[r] + r1off * es, trecv[r] + r1off * es, r1, dtype, op);
                    memcpy(tmp[r] + r1off * es, trecv[r] + r1off * es, r1 * es);
                }
            }
        }
    }
    for (r = 0; r < n; r++) memcpy(res[r], tmp[r] + (size_t)r * rc * es, rc * es); /* :171-174 */
    for (r = 0; r < n; r++) {
        free(tmp[r]);
        free(trecv[r]);
    }
    free(tmp);
    free(trecv);
    free(received);
    orc_rs_store(n, rc, es, res, recv);
    return 0;
}

/* reduce_scatter_radix.cpp:204-377. */
int orc_reduce_scatter_radix(int n, int k_in, size_t rc, int dtype, int op, const void* const* send,
                             void* const* recv) {
    size_t es = orc_dtype_size(dtype), total = rc * (size_t)n;
    orc_recexch_t* rx;
    char **tmp, **res;
    int *cnt, *off, r, i, ph, nph, k;
    if (n < 1 || !es || k_in < 2) return 1;
    rx = (orc_recexch_t*)calloc((size_t)n, sizeof(orc_recexch_t));
    for (r = 0; r < n; r++)
        if (orc_recexch_neighbors(r, n, k_in, &rx[r])) { /* :230 */
            free(rx);
            return 1;
        }
    k = rx[0].k;
    nph = rx[0].step2_nphases;
    cnt = (int*)calloc((size_t)(nph > 0 ? nph : 1) * (size_t)n, sizeof(int));
    off = (int*)calloc((size_t)(nph > 0 ? nph : 1) * (size_t)n, sizeof(int));
    orc_recexch_count_offset(n, nph > 0 ? nph : 1, k, cnt, off);
    tmp = (char**)calloc((size_t)n, sizeof(char*));
    res = (char**)calloc((size_t)n, sizeof(char*));
    for (r = 0; r < n; r++) {
        tmp[r] = (char*)malloc(total * es + 1);
        res[r] = (char*)malloc(rc * es + 1);
        memcpy(tmp[r], orc_rs_input(send, recv, r), total * es); /* :238-244 */
    }
    for (r = 0; r < n; r++) /* step 1 (:255-272): the non-participants' whole inputs, recvfrom order */
        if (rx[r].step1_sendto == -1)
            for (i = 0; i < rx[r].step1_nrecvs; i++)
                orc_reduce_local(orc_rs_input(send, recv, rx[r].step1_recvfrom[i]), tmp[r], total, dtype, op);
    for (ph = nph - 1; ph >= 0; ph--) /* step 2 (:279-318): regions of a phase are disjoint */
        for (r = 0; r < n; r++) {
            size_t moff = (size_t)off[ph * n + r] * rc, mlen = (size_t)cnt[ph * n + r] * rc;
            if (rx[r].step1_sendto != -1) continue;
            for (i = 0; i < k - 1; i++) {
                int dst = rx[r].step2_nbrs[ph][i];
                orc_reduce_local(tmp[dst] + moff * es, tmp[r] + moff * es, mlen, dtype, op);
            }
        }
    for (r = 0; r < n; r++) { /* :321-343 */
        const int owner = rx[r].step1_sendto == -1 ? r : rx[r].step1_sendto;
        memcpy(res[r], tmp[owner] + (size_t)r * rc * es, rc * es);
    }
    for (r = 0; r < n; r++) free(tmp[r]);
    free(tmp);
    free(cnt);
    free(off);
    free(rx);
    orc_rs_store(n, rc, es, res, recv);
    return 0;
}

/* ---- CHiArA's phases as stand-alone functions: testing/custom_implementations/work_dir/reduce_scatter/ ---- */

/* intra_reduce_scatter_radix.cpp:208-541, bulk-synchronous per group.  A participant's tmp_results
 * starts as its input (:274-280) and folds its step-1 senders' whole buffers in step1_recvfrom order
 * (:292-311).  Per stage, every step-2 phase (highest digit first) folds, in neighbour order, the
 * neighbours' copies of the participant's own count/offset region (:317-356) -- all taken before any
 * rank of the group reduces in that phase; the leftover stage clips every region to its nu chunks
 * (:400-475).  Step 3: participants copy their chunk out (:360 / :478), non-participants receive it
 * from their step-1 partner (:370 / :488). */
int orc_intra_reduce_scatter(int n, int k, int b, size_t rc, int dtype, int op, const void* const* send,
                             void* const* recv) {
    size_t es = orc_dtype_size(dtype), irc, total, blk;
    int nnodes, nstages, nu, node, l, i, ph, st;
    orc_recexch_t* x;
    int *cnt, *off;
    char **tres, **snap;
    if (n < 1 || !es || k < 2 || b < 1) return 1;
    if (n % b) return 3;
    nnodes = n / b;
    nstages = nnodes / b;
    nu = nnodes % b;
    irc = rc * (size_t)b;
    total = rc * (size_t)n;
    blk = irc * (size_t)b;
    x = (orc_recexch_t*)calloc((size_t)b, sizeof(orc_recexch_t));
    tres = (char**)calloc((size_t)b, sizeof(char*));
    snap = (char**)calloc((size_t)b, sizeof(char*));
    cnt = (int*)calloc(64 * (size_t)b + 1, sizeof(int));
    off = (int*)calloc(64 * (size_t)b + 1, sizeof(int));
    for (l = 0; l < b; l++) orc_recexch_neighbors(l, b, k, &x[l]);
    orc_recexch_count_offset(b, x[0].step2_nphases > 0 ? x[0].step2_nphases : 1, x[0].k, cnt, off);
    for (node = 0; node < nnodes; node++) {
        const int base = node * b;
        for (l = 0; l < b; l++) {
            tres[l] = NULL;
            if (x[l].step1_sendto != -1) continue;
            tres[l] = (char*)malloc(total * es + 1);
            snap[l] = (char*)malloc(total * es + 1);
            memcpy(tres[l], orc_rs_input(send, recv, base + l), total * es);
            for (i = 0; i < x[l].step1_nrecvs; i++)
                orc_reduce_local(orc_rs_input(send, recv, base + x[l].step1_recvfrom[i]), tres[l], total, dtype, op);
        }
        for (st = 0; st <= nstages; st++) {
            const size_t sb = (size_t)st * blk, lim = st < nstages ? blk : (size_t)nu * irc;
            if (st == nstages && nu == 0) break;
            for (ph = x[0].step2_nphases - 1; ph >= 0; ph--) {
                for (l = 0; l < b; l++)
                    if (tres[l]) memcpy(snap[l], tres[l], total * es);
                for (l = 0; l < b; l++) {
                    size_t mo, ml;
                    if (!tres[l]) continue;
                    mo = (size_t)off[ph * b + l] * irc;
                    ml = (size_t)cnt[ph * b + l] * irc;
                    if (mo >= lim) continue;
                    if (ml > lim - mo) ml = lim - mo;
                    for (i = 0; i < x[l].k - 1; i++)
                        orc_reduce_local(snap[x[l].step2_nbrs[ph][i]] + (sb + mo) * es, tres[l] + (sb + mo) * es, ml,
                                         dtype, op);
                }
            }
            for (l = 0; l < b; l++) {
                const int owner = x[l].step1_sendto == -1 ? l : x[l].step1_sendto;
                if ((size_t)l * irc >= lim) continue;
                memcpy((char*)recv[base + l] + (size_t)st * irc * es, tres[owner] + (sb + (size_t)l * irc) * es,
                       irc * es);
            }
        }
        for (l = 0; l < b; l++) {
            free(tres[l]);
            if (tres[l]) free(snap[l]);
        }
    }
    free(x);
    free(tres);
    free(snap);
    free(cnt);
    free(off);
    return 0;
}

/* inter_linear_reduce.cpp:11-73: root of iteration i = node i * b + lane (skipped past the last
 * node, :48); recvbuf = own chunk i (:55), then MPI_Reduce_local(chunk i of node j, recvbuf) for
 * j ascending, j != root (:58-63). */
int orc_inter_reduce_linear(int n, int b, size_t rc, int dtype, int op, const void* const* send, void* const* recv) {
    size_t es = orc_dtype_size(dtype), irc;
    int nnodes, niters, r, i, j;
    if (n < 1 || !es || b < 1) return 1;
    if (n % b) return 3;
    nnodes = n / b;
    niters = nnodes / b + (nnodes % b ? 1 : 0);
    irc = rc * (size_t)b;
    for (r = 0; r < n; r++) {
        const int node = r / b, lane = r % b;
        for (i = 0; i < niters; i++) {
            if (i * b + lane != node) continue;
            memcpy(recv[r], (const char*)send[r] + (size_t)i * irc * es, irc * es);
            for (j = 0; j < nnodes; j++)
                if (j != node)
                    orc_reduce_local((const char*)send[j * b + lane] + (size_t)i * irc * es, recv[r], irc, dtype, op);
        }
    }
    return 0;
}

/* intra_scatter_radix_batch.cpp:10-110: the k-nomial tree only routes the blocks; every rank ends
 * with block `lane` of its node root's (lane node % b) send buffer (the self-test's expectation,
 * :226-233). */
int orc_intra_scatter(int n, int k, int b, size_t rc, int dtype, const void* const* send, void* const* recv) {
    size_t es = orc_dtype_size(dtype);
    int r;
    if (n < 1 || !es || k < 2 || b < 1) return 1;
    if (n % b) return 3;
    for (r = 0; r < n; r++) {
        const int node = r / b, lane = r % b, root = node * b + node % b;
        memcpy(recv[r], (const char*)send[root] + (size_t)lane * rc * es, rc * es);
    }
    return 0;
}
