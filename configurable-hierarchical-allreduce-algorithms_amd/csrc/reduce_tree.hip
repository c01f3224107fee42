// reduce_tree.hip -- fused expression-tree reduction for gfx950 (one HBM pass per chunk).
#include <hip/hip_runtime.h>

#include "reduce_tree.hpp"

namespace chr {

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

// dtype, op: the kernel type and op (canon_op)
static hipError_t launch_tree_any(const TreeArgs& a, const TreeScalarArgs* sa, int dtype, int op, hipStream_t s) {
    if (dtype >= CHR_FLOAT_INT && dtype <= CHR_C_DOUBLE_COMPLEX) return launch_tree_pair(a, sa, dtype, op, s);
    const bool core = (dtype == CHR_FLOAT32 || dtype == CHR_FLOAT64 || dtype == CHR_BFLOAT16 || dtype == CHR_INT32) &&
                      op <= CHR_MIN;
    if (!core) return launch_tree_int(a, sa, dtype, op, s);
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

// Several trees in as few launches as possible: the vector bodies of trees with equal leaf counts
// share a launch (up to kMaxTreeSegs segments); heads and tails that are not 16-B congruent run
// on the scalar kernel per tree.  Every tree keeps its own program, so the bits are unchanged.
hipError_t launch_reduce_tree_multi(const TreeJob* jobs, int njobs, int dtype, int op, hipStream_t stream) {
    if (!valid_dtype_op(dtype, op)) return hipErrorInvalidValue;
    const size_t es = dtype_size(dtype);
    const int dtype0 = dtype, op0 = op;       // the caller's (type, op), for the bucket kernel
    canon_op(dtype, op, false, &dtype, &op);  // the per-combine swap bits carry the operand order
    const size_t E = 16 / es;
    TreeArgs pend[kMaxLeaves + 1] = {};  // pending vector segments, by leaf count
    auto flush = [&](int nl) -> hipError_t {
        TreeArgs& a = pend[nl];
        if (!a.nseg) return hipSuccess;
        a.nl = nl;
        const hipError_t e = launch_tree_any(a, nullptr, dtype, op, stream);
        a.nseg = 0;
        return e;
    };
    for (int t = 0; t < njobs; ++t) {
        const TreeJob& jb = jobs[t];
        if (jb.n == 0) continue;
        uint32_t cb = 0, sb = 0;
        if (!tree_program_ok(jb.nl, jb.comb, jb.swaps, &cb, &sb)) return hipErrorInvalidValue;
        const int nl = jb.nl;
        if (nl == 1) {
            if (jb.out != jb.leaves[0]) {
                const hipError_t e = hipMemcpyAsync(jb.out, jb.leaves[0], jb.n * es, hipMemcpyDeviceToDevice, stream);
                if (e != hipSuccess) return e;
            }
            continue;
        }
        // A streaming 2-leaf tree is one fold: MPI_Reduce_local(l1, l0), or with the swap bit MPI_Reduce_local(l0, l1),
        // into `out` -- the bucket kernel out of place, 1.6 % faster than the tree kernel at identical traffic
        // (rocprof, profiles/r06/leaf2_rocprof/).  Unless `out` is the fold's input (the bucket
        // kernel takes out == acc only).
        if (nl == 2 && 3 * jb.n * es >= reduce_tuning().nt_min_bytes) {
            const bool sw = (sb & 1u) != 0;
            const void* acc = jb.leaves[sw ? 1 : 0];
            const void* in = jb.leaves[sw ? 0 : 1];
            if (jb.out != in) {
                const hipError_t e = launch_reduce(jb.out, acc, &in, 1, jb.n, dtype0, op0, stream);
                if (e != hipSuccess) return e;
                continue;
            }
        }
        const uintptr_t mis = (uintptr_t)jb.out & 15u;
        bool congruent = (mis % es) == 0;
        for (int j = 0; j < nl; ++j) congruent = congruent && (((uintptr_t)jb.leaves[j] & 15u) == mis);
        auto scalar = [&](size_t off, size_t cnt) -> hipError_t {
            if (!cnt) return hipSuccess;
            TreeScalarArgs sa{};
            sa.out = (char*)jb.out + off * es;
            for (int j = 0; j < nl; ++j) sa.leaves[j] = (const char*)jb.leaves[j] + off * es;
            sa.n = cnt;
            sa.nl = nl;
            sa.comb = cb;
            sa.swaps = sb;
            TreeArgs dummy{};
            return launch_tree_any(dummy, &sa, dtype, op, stream);
        };
        hipError_t err;
        if (!congruent) {
            if ((err = scalar(0, jb.n)) != hipSuccess) return err;
            continue;
        }
        size_t head = mis ? (16 - mis) / es : 0;
        if (head > jb.n) head = jb.n;
        const size_t nvec = (jb.n - head) / E;
        const size_t tail = jb.n - head - nvec * E;
        if ((err = scalar(0, head)) != hipSuccess || (err = scalar(head + nvec * E, tail)) != hipSuccess) return err;
        const size_t cap = reduce_tuning().max_launch_vec;
        const size_t seg_cap = cap && cap < kMaxSegVec ? cap : kMaxSegVec;
        for (size_t off = 0; off < nvec; off += seg_cap) {  // pieces of at most 1 GiB per operand
            TreeArgs& a = pend[nl];
            TreeSeg& g = a.seg[a.nseg++];
            g.out = (u32x4*)((char*)jb.out + head * es) + off;
            for (int j = 0; j < nl; ++j) g.leaves[j] = (const u32x4*)((const char*)jb.leaves[j] + head * es) + off;
            g.nvec = nvec - off < seg_cap ? nvec - off : seg_cap;
            g.comb = cb;
            g.swaps = sb;
            if (a.nseg == kMaxTreeSegs && (err = flush(nl)) != hipSuccess) return err;
        }
    }
    for (int nl = 2; nl <= kMaxLeaves; ++nl) {
        const hipError_t e = flush(nl);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_reduce_tree(void* out, const void* const* leaves, int nl, const uint8_t* comb, const uint8_t* swaps,
                              size_t n, int dtype, int op, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (nl < 1 || nl > kMaxLeaves) return hipErrorInvalidValue;
    TreeJob jb{out, {}, nl, comb, swaps, n};
    for (int j = 0; j < nl; ++j) jb.leaves[j] = leaves[j];
    return launch_reduce_tree_multi(&jb, 1, dtype, op, stream);
}

}  // namespace chr
