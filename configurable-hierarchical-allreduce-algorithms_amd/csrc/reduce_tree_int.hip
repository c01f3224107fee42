// reduce_tree_int.hip -- the fused expression-tree kernel for the MPI integer types beyond int32
// arithmetic and for the logical / bitwise ops (see reduce_int.hip for the type mapping and
// reduce_tree.hip for the kernel).  Policy shapes only; its own translation unit so it builds in
// parallel with the floating-point trees.
#include <hip/hip_runtime.h>

#include "reduce_tree.hpp"

namespace chr {

template <int DT>
static hipError_t tree_all_ops(const TreeArgs& a, const TreeScalarArgs* sa, int op, hipStream_t s) {
    switch (op) {
    case CHR_SUM: return launch_tree_op<DT, CHR_SUM, false>(a, sa, s);
    case CHR_PROD: return launch_tree_op<DT, CHR_PROD, false>(a, sa, s);
    case CHR_MAX: return launch_tree_op<DT, CHR_MAX, false>(a, sa, s);
    case CHR_MIN: return launch_tree_op<DT, CHR_MIN, false>(a, sa, s);
    case CHR_LAND: return launch_tree_op<DT, CHR_LAND, false>(a, sa, s);
    case CHR_LOR: return launch_tree_op<DT, CHR_LOR, false>(a, sa, s);
    case CHR_LXOR: return launch_tree_op<DT, CHR_LXOR, false>(a, sa, s);
    case CHR_BAND: return launch_tree_op<DT, CHR_BAND, false>(a, sa, s);
    case CHR_BOR: return launch_tree_op<DT, CHR_BOR, false>(a, sa, s);
    case CHR_BXOR: return launch_tree_op<DT, CHR_BXOR, false>(a, sa, s);
    default: return hipErrorInvalidValue;
    }
}

template <int DT>
static hipError_t tree_minmax(const TreeArgs& a, const TreeScalarArgs* sa, int op, hipStream_t s) {
    if (op == CHR_MAX) return launch_tree_op<DT, CHR_MAX, false>(a, sa, s);
    if (op == CHR_MIN) return launch_tree_op<DT, CHR_MIN, false>(a, sa, s);
    return hipErrorInvalidValue;
}

static hipError_t tree_i32_logic(const TreeArgs& a, const TreeScalarArgs* sa, int op, hipStream_t s) {
    switch (op) {
    case CHR_LAND: return launch_tree_op<CHR_INT32, CHR_LAND, false>(a, sa, s);
    case CHR_LOR: return launch_tree_op<CHR_INT32, CHR_LOR, false>(a, sa, s);
    case CHR_LXOR: return launch_tree_op<CHR_INT32, CHR_LXOR, false>(a, sa, s);
    case CHR_BAND: return launch_tree_op<CHR_INT32, CHR_BAND, false>(a, sa, s);
    case CHR_BOR: return launch_tree_op<CHR_INT32, CHR_BOR, false>(a, sa, s);
    case CHR_BXOR: return launch_tree_op<CHR_INT32, CHR_BXOR, false>(a, sa, s);
    default: return hipErrorInvalidValue;
    }
}

template <int DT>
static hipError_t tree_logic(const TreeArgs& a, const TreeScalarArgs* sa, int op, hipStream_t s) {
    if (op == CHR_LAND) return launch_tree_op<DT, CHR_LAND, false>(a, sa, s);
    if (op == CHR_LOR) return launch_tree_op<DT, CHR_LOR, false>(a, sa, s);
    if (op == CHR_LXOR) return launch_tree_op<DT, CHR_LXOR, false>(a, sa, s);
    return hipErrorInvalidValue;
}

hipError_t launch_tree_int(const TreeArgs& a, const TreeScalarArgs* sa, int kdt, int kop, hipStream_t s) {
    switch (kdt) {
    case CHR_FLOAT32: return tree_logic<CHR_FLOAT32>(a, sa, kop, s);  // MPICH's logical ops on floats
    case CHR_FLOAT64: return tree_logic<CHR_FLOAT64>(a, sa, kop, s);
    case CHR_UINT8: return tree_all_ops<CHR_UINT8>(a, sa, kop, s);
    case CHR_UINT16: return tree_all_ops<CHR_UINT16>(a, sa, kop, s);
    case CHR_UINT64: return tree_all_ops<CHR_UINT64>(a, sa, kop, s);
    case CHR_INT32: return tree_i32_logic(a, sa, kop, s);
    case CHR_INT8: return tree_minmax<CHR_INT8>(a, sa, kop, s);
    case CHR_INT16: return tree_minmax<CHR_INT16>(a, sa, kop, s);
    case CHR_UINT32: return tree_minmax<CHR_UINT32>(a, sa, kop, s);
    case CHR_INT64: return tree_minmax<CHR_INT64>(a, sa, kop, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace chr
