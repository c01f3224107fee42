// reduce_tree_pair.hip -- the fused expression-tree kernel for MPI's pair types under MAXLOC /
// MINLOC and the C complex types under SUM / PROD (see reduce_pair.hip for the types and
// reduce_tree.hpp for the kernel).  The swap bits of a program pick MPICH_do_reduce's operand order
// per combine, which matters for the floating-valued pairs (order_sensitive in reduce_tree.hpp).
#include <hip/hip_runtime.h>

#include "reduce_tree.hpp"

namespace chr {

template <int DT>
static hipError_t tree_loc(const TreeArgs& a, const TreeScalarArgs* sa, int op, hipStream_t s) {
    if (op == CHR_MAXLOC) return launch_tree_op<DT, CHR_MAXLOC>(a, sa, s);
    if (op == CHR_MINLOC) return launch_tree_op<DT, CHR_MINLOC>(a, sa, s);
    return hipErrorInvalidValue;
}

template <int DT>
static hipError_t tree_cplx(const TreeArgs& a, const TreeScalarArgs* sa, int op, hipStream_t s) {
    if (op == CHR_SUM) return launch_tree_op<DT, CHR_SUM>(a, sa, s);
    if (op == CHR_PROD) return launch_tree_op<DT, CHR_PROD>(a, sa, s);
    return hipErrorInvalidValue;
}

hipError_t launch_tree_pair(const TreeArgs& a, const TreeScalarArgs* sa, int kdt, int kop, hipStream_t s) {
    switch (kdt) {
    case CHR_FLOAT_INT: return tree_loc<CHR_FLOAT_INT>(a, sa, kop, s);
    case CHR_DOUBLE_INT: return tree_loc<CHR_DOUBLE_INT>(a, sa, kop, s);
    case CHR_LONG_INT: return tree_loc<CHR_LONG_INT>(a, sa, kop, s);
    case CHR_2INT: return tree_loc<CHR_2INT>(a, sa, kop, s);
    case CHR_SHORT_INT: return tree_loc<CHR_SHORT_INT>(a, sa, kop, s);
    case CHR_C_FLOAT_COMPLEX: return tree_cplx<CHR_C_FLOAT_COMPLEX>(a, sa, kop, s);
    case CHR_C_DOUBLE_COMPLEX: return tree_cplx<CHR_C_DOUBLE_COMPLEX>(a, sa, kop, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace chr
