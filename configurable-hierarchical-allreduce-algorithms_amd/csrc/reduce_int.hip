// reduce_int.hip -- the fused bucket reduction for the MPI integer types beyond int32
// arithmetic: (u)int8/16/64 and uint32, the logical (LAND/LOR/LXOR) and bitwise (BAND/BOR/BXOR)
// ops on every integer type, and the logical ops on float/double (MPICH accepts them).  The
// reference is generic over MPI_Datatype and MPI_Op (all_reduce_radix_batch.cpp:202-204,
// MPI_Type_size at :234-277); its arithmetic is
// MPICH's MPI_Reduce_local loop for the pair.  Same kernels as reduce_kernels.hip (reduce_vec.hpp),
// compiled here in the two policy shapes only, so this translation unit builds in parallel with
// the floating-point one.  Kernel types come from canon_op: signedness only matters to MAX/MIN,
// everything else runs on the unsigned type of the width (int32's kernels for 32-bit).
#include <hip/hip_runtime.h>

#include "reduce_vec.hpp"

namespace chr {

template <int DT>
static hipError_t vec_all_ops(const VecArgs& a, int op, int m, hipStream_t s) {
    switch (op) {
    case CHR_SUM: return launch_vec_op<DT, CHR_SUM>(a, m, s);
    case CHR_PROD: return launch_vec_op<DT, CHR_PROD>(a, m, s);
    case CHR_MAX: return launch_vec_op<DT, CHR_MAX>(a, m, s);
    case CHR_MIN: return launch_vec_op<DT, CHR_MIN>(a, m, s);
    case CHR_LAND: return launch_vec_op<DT, CHR_LAND>(a, m, s);
    case CHR_LOR: return launch_vec_op<DT, CHR_LOR>(a, m, s);
    case CHR_LXOR: return launch_vec_op<DT, CHR_LXOR>(a, m, s);
    // the bitwise ops see no element boundaries (apply_vec works on whole dwords): int32's
    // kernels serve every width
    case CHR_BAND: return launch_vec_op<CHR_INT32, CHR_BAND>(a, m, s);
    case CHR_BOR: return launch_vec_op<CHR_INT32, CHR_BOR>(a, m, s);
    case CHR_BXOR: return launch_vec_op<CHR_INT32, CHR_BXOR>(a, m, s);
    default: return hipErrorInvalidValue;
    }
}

template <int DT>
static hipError_t vec_minmax(const VecArgs& a, int op, int m, hipStream_t s) {
    if (op == CHR_MAX) return launch_vec_op<DT, CHR_MAX>(a, m, s);
    if (op == CHR_MIN) return launch_vec_op<DT, CHR_MIN>(a, m, s);
    return hipErrorInvalidValue;
}

static hipError_t vec_i32_logic(const VecArgs& a, int op, int m, hipStream_t s) {
    switch (op) {
    case CHR_LAND: return launch_vec_op<CHR_INT32, CHR_LAND>(a, m, s);
    case CHR_LOR: return launch_vec_op<CHR_INT32, CHR_LOR>(a, m, s);
    case CHR_LXOR: return launch_vec_op<CHR_INT32, CHR_LXOR>(a, m, s);
    case CHR_BAND: return launch_vec_op<CHR_INT32, CHR_BAND>(a, m, s);
    case CHR_BOR: return launch_vec_op<CHR_INT32, CHR_BOR>(a, m, s);
    case CHR_BXOR: return launch_vec_op<CHR_INT32, CHR_BXOR>(a, m, s);
    default: return hipErrorInvalidValue;
    }
}

template <int DT>
static hipError_t vec_logic(const VecArgs& a, int op, int m, hipStream_t s) {
    if (op == CHR_LAND) return launch_vec_op<DT, CHR_LAND>(a, m, s);
    if (op == CHR_LOR) return launch_vec_op<DT, CHR_LOR>(a, m, s);
    if (op == CHR_LXOR) return launch_vec_op<DT, CHR_LXOR>(a, m, s);
    return hipErrorInvalidValue;
}

hipError_t launch_vec_int(const VecArgs& a, int kdt, int kop, int m, hipStream_t s) {
    switch (kdt) {
    case CHR_FLOAT32: return vec_logic<CHR_FLOAT32>(a, kop, m, s);  // MPICH's logical ops on floats
    case CHR_FLOAT64: return vec_logic<CHR_FLOAT64>(a, kop, m, s);
    case CHR_UINT8: return vec_all_ops<CHR_UINT8>(a, kop, m, s);
    case CHR_UINT16: return vec_all_ops<CHR_UINT16>(a, kop, m, s);
    case CHR_UINT64: return vec_all_ops<CHR_UINT64>(a, kop, m, s);
    case CHR_INT32: return vec_i32_logic(a, kop, m, s);
    case CHR_INT8: return vec_minmax<CHR_INT8>(a, kop, m, s);
    case CHR_INT16: return vec_minmax<CHR_INT16>(a, kop, m, s);
    case CHR_UINT32: return vec_minmax<CHR_UINT32>(a, kop, m, s);
    case CHR_INT64: return vec_minmax<CHR_INT64>(a, kop, m, s);
    default: return hipErrorInvalidValue;
    }
}

template <int DT>
static hipError_t scalar_all_ops(const ScalarArgs& a, int op, hipStream_t s) {
    switch (op) {
    case CHR_SUM: return launch_scalar_op<DT, CHR_SUM>(a, s);
    case CHR_PROD: return launch_scalar_op<DT, CHR_PROD>(a, s);
    case CHR_MAX: return launch_scalar_op<DT, CHR_MAX>(a, s);
    case CHR_MIN: return launch_scalar_op<DT, CHR_MIN>(a, s);
    case CHR_LAND: return launch_scalar_op<DT, CHR_LAND>(a, s);
    case CHR_LOR: return launch_scalar_op<DT, CHR_LOR>(a, s);
    case CHR_LXOR: return launch_scalar_op<DT, CHR_LXOR>(a, s);
    case CHR_BAND: return launch_scalar_op<DT, CHR_BAND>(a, s);
    case CHR_BOR: return launch_scalar_op<DT, CHR_BOR>(a, s);
    case CHR_BXOR: return launch_scalar_op<DT, CHR_BXOR>(a, s);
    default: return hipErrorInvalidValue;
    }
}

template <int DT>
static hipError_t scalar_minmax(const ScalarArgs& a, int op, hipStream_t s) {
    if (op == CHR_MAX) return launch_scalar_op<DT, CHR_MAX>(a, s);
    if (op == CHR_MIN) return launch_scalar_op<DT, CHR_MIN>(a, s);
    return hipErrorInvalidValue;
}

template <int DT>
static hipError_t scalar_logic(const ScalarArgs& a, int op, hipStream_t s) {
    if (op == CHR_LAND) return launch_scalar_op<DT, CHR_LAND>(a, s);
    if (op == CHR_LOR) return launch_scalar_op<DT, CHR_LOR>(a, s);
    if (op == CHR_LXOR) return launch_scalar_op<DT, CHR_LXOR>(a, s);
    return hipErrorInvalidValue;
}

hipError_t launch_scalar_int(const ScalarArgs& a, int kdt, int kop, hipStream_t s) {
    switch (kdt) {
    case CHR_FLOAT32: return scalar_logic<CHR_FLOAT32>(a, kop, s);
    case CHR_FLOAT64: return scalar_logic<CHR_FLOAT64>(a, kop, s);
    case CHR_UINT8: return scalar_all_ops<CHR_UINT8>(a, kop, s);
    case CHR_UINT16: return scalar_all_ops<CHR_UINT16>(a, kop, s);
    case CHR_UINT64: return scalar_all_ops<CHR_UINT64>(a, kop, s);
    case CHR_INT32:
        if (kop < CHR_LAND) return hipErrorInvalidValue;  // int32 arithmetic: reduce_kernels.hip
        return scalar_all_ops<CHR_INT32>(a, kop, s);
    case CHR_INT8: return scalar_minmax<CHR_INT8>(a, kop, s);
    case CHR_INT16: return scalar_minmax<CHR_INT16>(a, kop, s);
    case CHR_UINT32: return scalar_minmax<CHR_UINT32>(a, kop, s);
    case CHR_INT64: return scalar_minmax<CHR_INT64>(a, kop, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace chr
