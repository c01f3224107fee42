// reduce_tree.hip -- fused expression-tree reduction for gfx950 (one HBM pass per chunk).
#include <hip/hip_runtime.h>

#include "reduce_tree.hpp"

namespace chr {

template <int DT>
static hipError_t launch_tree_dt(const TreeArgs& a, const TreeScalarArgs* sa, int op, hipStream_t s) {
    switch (op) {
    case CHR_SUM: return launch_tree_op<DT, CHR_SUM, true>(a, sa, s);
    case CHR_PROD: return launch_tree_op<DT, CHR_PROD, true>(a, sa, s);
    case CHR_MAX: return launch_tree_op<DT, CHR_MAX, true>(a, sa, s);
    case CHR_MIN: return launch_tree_op<DT, CHR_MIN, true>(a, sa, s);
    default: return hipErrorInvalidValue;
    }
}

// dtype, op: the kernel type and op (canon_op)
static hipError_t launch_tree_any(const TreeArgs& a, const TreeScalarArgs* sa, int dtype, int op, hipStream_t s) {
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

hipError_t launch_reduce_tree(void* out, const void* const* leaves, int nl, const uint8_t* comb, const uint8_t* swaps,
                              size_t n, int dtype, int op, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (!valid_dtype_op(dtype, op)) return hipErrorInvalidValue;
    uint32_t cb = 0, sb = 0;
    if (!tree_program_ok(nl, comb, swaps, &cb, &sb)) return hipErrorInvalidValue;
    const size_t es = dtype_size(dtype);
    canon_op(dtype, op, false, &dtype, &op);  // the per-combine swap bits carry the operand order
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
