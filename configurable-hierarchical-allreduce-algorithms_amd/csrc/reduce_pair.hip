// reduce_pair.hip -- the fused bucket reduction for MPI's pair types under MAXLOC / MINLOC
// (MPI_FLOAT_INT, MPI_DOUBLE_INT, MPI_LONG_INT, MPI_2INT, MPI_SHORT_INT) and the C complex types
// under SUM / PROD (MPI_C_FLOAT_COMPLEX, MPI_C_DOUBLE_COMPLEX).  The reference is generic over
// MPI_Datatype x MPI_Op (all_reduce_radix_batch.cpp:202-204) and reduces with MPICH's
// MPI_Reduce_local (:332, :364, :446, :529), which accepts exactly these pairs for these types
// (tests/golden/pairs_manifest.json).  Element semantics: reduce_common.hpp apply<> (MPICH's loops,
// pinned by tests/golden/pairs_reduce_local.npz and nan_reduce_local.npz).  Same kernels and policy shapes as reduce_int.hip:
// an element is 8 or 16 bytes, so one 16-B vector holds two or one of them.
#include <hip/hip_runtime.h>

#include "reduce_vec.hpp"

namespace chr {

template <int DT>
static hipError_t vec_loc(const VecArgs& a, int op, int m, hipStream_t s) {
    switch (op) {
    case CHR_MAXLOC: return launch_vec_op<DT, CHR_MAXLOC>(a, m, s);
    case CHR_MINLOC: return launch_vec_op<DT, CHR_MINLOC>(a, m, s);
    case kMaxLocSw:
        if constexpr (DT == CHR_FLOAT_INT || DT == CHR_DOUBLE_INT) return launch_vec_op<DT, kMaxLocSw>(a, m, s);
        else return hipErrorInvalidValue;
    case kMinLocSw:
        if constexpr (DT == CHR_FLOAT_INT || DT == CHR_DOUBLE_INT) return launch_vec_op<DT, kMinLocSw>(a, m, s);
        else return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
    }
}

template <int DT>
static hipError_t vec_cplx(const VecArgs& a, int op, int m, hipStream_t s) {
    if (op == CHR_SUM) return launch_vec_op<DT, CHR_SUM>(a, m, s);
    if (op == CHR_PROD) return launch_vec_op<DT, CHR_PROD>(a, m, s);
    if (op == kSumSw) return launch_vec_op<DT, kSumSw>(a, m, s);
    if (op == kProdSw) return launch_vec_op<DT, kProdSw>(a, m, s);
    return hipErrorInvalidValue;
}

hipError_t launch_vec_pair(const VecArgs& a, int kdt, int kop, int m, hipStream_t s) {
    switch (kdt) {
    case CHR_FLOAT_INT: return vec_loc<CHR_FLOAT_INT>(a, kop, m, s);
    case CHR_DOUBLE_INT: return vec_loc<CHR_DOUBLE_INT>(a, kop, m, s);
    case CHR_LONG_INT: return vec_loc<CHR_LONG_INT>(a, kop, m, s);
    case CHR_2INT: return vec_loc<CHR_2INT>(a, kop, m, s);
    case CHR_SHORT_INT: return vec_loc<CHR_SHORT_INT>(a, kop, m, s);
    case CHR_C_FLOAT_COMPLEX: return vec_cplx<CHR_C_FLOAT_COMPLEX>(a, kop, m, s);
    case CHR_C_DOUBLE_COMPLEX: return vec_cplx<CHR_C_DOUBLE_COMPLEX>(a, kop, m, s);
    default: return hipErrorInvalidValue;
    }
}

template <int DT>
static hipError_t scalar_loc(const ScalarArgs& a, int op, hipStream_t s) {
    switch (op) {
    case CHR_MAXLOC: return launch_scalar_op<DT, CHR_MAXLOC>(a, s);
    case CHR_MINLOC: return launch_scalar_op<DT, CHR_MINLOC>(a, s);
    case kMaxLocSw:
        if constexpr (DT == CHR_FLOAT_INT || DT == CHR_DOUBLE_INT) return launch_scalar_op<DT, kMaxLocSw>(a, s);
        else return hipErrorInvalidValue;
    case kMinLocSw:
        if constexpr (DT == CHR_FLOAT_INT || DT == CHR_DOUBLE_INT) return launch_scalar_op<DT, kMinLocSw>(a, s);
        else return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
    }
}

template <int DT>
static hipError_t scalar_cplx(const ScalarArgs& a, int op, hipStream_t s) {
    if (op == CHR_SUM) return launch_scalar_op<DT, CHR_SUM>(a, s);
    if (op == CHR_PROD) return launch_scalar_op<DT, CHR_PROD>(a, s);
    if (op == kSumSw) return launch_scalar_op<DT, kSumSw>(a, s);
    if (op == kProdSw) return launch_scalar_op<DT, kProdSw>(a, s);
    return hipErrorInvalidValue;
}

hipError_t launch_scalar_pair(const ScalarArgs& a, int kdt, int kop, hipStream_t s) {
    switch (kdt) {
    case CHR_FLOAT_INT: return scalar_loc<CHR_FLOAT_INT>(a, kop, s);
    case CHR_DOUBLE_INT: return scalar_loc<CHR_DOUBLE_INT>(a, kop, s);
    case CHR_LONG_INT: return scalar_loc<CHR_LONG_INT>(a, kop, s);
    case CHR_2INT: return scalar_loc<CHR_2INT>(a, kop, s);
    case CHR_SHORT_INT: return scalar_loc<CHR_SHORT_INT>(a, kop, s);
    case CHR_C_FLOAT_COMPLEX: return scalar_cplx<CHR_C_FLOAT_COMPLEX>(a, kop, s);
    case CHR_C_DOUBLE_COMPLEX: return scalar_cplx<CHR_C_DOUBLE_COMPLEX>(a, kop, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace chr
