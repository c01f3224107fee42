// reduce_tree_int.hip -- the fused expression-tree kernel for the MPI integer types beyond int32
// arithmetic and for the logical / bitwise ops (see reduce_int.hip for the type mapping and
// reduce_tree.hip for the kernel).  Policy shapes only; its own translation unit so it builds in
// parallel with the floating-point trees, and compiled twice (CHR_TREE_INT_PART 1: the 8- and 16-bit
// kernel types; 2: the rest and the dispatcher) so the two halves build in parallel too.
#include <hip/hip_runtime.h>

#include "reduce_tree.hpp"

#ifndef CHR_TREE_INT_PART
#error "compile with -DCHR_TREE_INT_PART=1 or 2"
#endif

namespace chr {

hipError_t launch_tree_int_narrow(const TreeArgs& a, const TreeScalarArgs* sa, int kdt, int kop, hipStream_t s);

template <int DT>
[[maybe_unused]] static hipError_t tree_all_ops(const TreeArgs& a, const TreeScalarArgs* sa, int op, hipStream_t s) {
    switch (op) {
    case CHR_SUM: return launch_tree_op<DT, CHR_SUM>(a, sa, s);
    case CHR_PROD: return launch_tree_op<DT, CHR_PROD>(a, sa, s);
    case CHR_MAX: return launch_tree_op<DT, CHR_MAX>(a, sa, s);
    case CHR_MIN: return launch_tree_op<DT, CHR_MIN>(a, sa, s);
    case CHR_LAND: return launch_tree_op<DT, CHR_LAND>(a, sa, s);
    case CHR_LOR: return launch_tree_op<DT, CHR_LOR>(a, sa, s);
    case CHR_LXOR: return launch_tree_op<DT, CHR_LXOR>(a, sa, s);
    // bitwise: the vector kernels work on whole dwords, so int32's serve every width; the scalar
    // heads and tails keep the element width
    // (compiled once, in part 2)
    case CHR_BAND: return sa ? launch_tree_scalar_op<DT, CHR_BAND>(*sa, s) : launch_tree_int(a, sa, CHR_INT32, op, s);
    case CHR_BOR: return sa ? launch_tree_scalar_op<DT, CHR_BOR>(*sa, s) : launch_tree_int(a, sa, CHR_INT32, op, s);
    case CHR_BXOR: return sa ? launch_tree_scalar_op<DT, CHR_BXOR>(*sa, s) : launch_tree_int(a, sa, CHR_INT32, op, s);
    default: return hipErrorInvalidValue;
    }
}

template <int DT>
[[maybe_unused]] static hipError_t tree_minmax(const TreeArgs& a, const TreeScalarArgs* sa, int op, hipStream_t s) {
    if (op == CHR_MAX) return launch_tree_op<DT, CHR_MAX>(a, sa, s);
    if (op == CHR_MIN) return launch_tree_op<DT, CHR_MIN>(a, sa, s);
    return hipErrorInvalidValue;
}

#if CHR_TREE_INT_PART == 2  // kernel instantiations happen when a function body is parsed
[[maybe_unused]] static hipError_t tree_i32_logic(const TreeArgs& a, const TreeScalarArgs* sa, int op, hipStream_t s) {
    switch (op) {
    case CHR_LAND: return launch_tree_op<CHR_INT32, CHR_LAND>(a, sa, s);
    case CHR_LOR: return launch_tree_op<CHR_INT32, CHR_LOR>(a, sa, s);
    case CHR_LXOR: return launch_tree_op<CHR_INT32, CHR_LXOR>(a, sa, s);
    case CHR_BAND: return launch_tree_op<CHR_INT32, CHR_BAND>(a, sa, s);
    case CHR_BOR: return launch_tree_op<CHR_INT32, CHR_BOR>(a, sa, s);
    case CHR_BXOR: return launch_tree_op<CHR_INT32, CHR_BXOR>(a, sa, s);
    default: return hipErrorInvalidValue;
    }
}

template <int DT>
[[maybe_unused]] static hipError_t tree_logic(const TreeArgs& a, const TreeScalarArgs* sa, int op, hipStream_t s) {
    if (op == CHR_LAND) return launch_tree_op<DT, CHR_LAND>(a, sa, s);
    if (op == CHR_LOR) return launch_tree_op<DT, CHR_LOR>(a, sa, s);
    if (op == CHR_LXOR) return launch_tree_op<DT, CHR_LXOR>(a, sa, s);
    return hipErrorInvalidValue;
}
#endif

#if CHR_TREE_INT_PART == 1
hipError_t launch_tree_int_narrow(const TreeArgs& a, const TreeScalarArgs* sa, int kdt, int kop, hipStream_t s) {
    switch (kdt) {
    case CHR_UINT8: return tree_all_ops<CHR_UINT8>(a, sa, kop, s);
    case CHR_UINT16: return tree_all_ops<CHR_UINT16>(a, sa, kop, s);
    case CHR_INT8: return tree_minmax<CHR_INT8>(a, sa, kop, s);
    case CHR_INT16: return tree_minmax<CHR_INT16>(a, sa, kop, s);
    default: return hipErrorInvalidValue;
    }
}
#else
hipError_t launch_tree_int(const TreeArgs& a, const TreeScalarArgs* sa, int kdt, int kop, hipStream_t s) {
    switch (kdt) {
    case CHR_FLOAT32: return tree_logic<CHR_FLOAT32>(a, sa, kop, s);  // MPICH's logical ops on floats
    case CHR_FLOAT64: return tree_logic<CHR_FLOAT64>(a, sa, kop, s);
    case CHR_UINT8:
    case CHR_UINT16:
    case CHR_INT8:
    case CHR_INT16: return launch_tree_int_narrow(a, sa, kdt, kop, s);
    case CHR_UINT64: return tree_all_ops<CHR_UINT64>(a, sa, kop, s);
    case CHR_INT32: return tree_i32_logic(a, sa, kop, s);
    case CHR_UINT32: return tree_minmax<CHR_UINT32>(a, sa, kop, s);
    case CHR_INT64: return tree_minmax<CHR_INT64>(a, sa, kop, s);
    default: return hipErrorInvalidValue;
    }
}
#endif

}  // namespace chr
