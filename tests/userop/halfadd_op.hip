// halfadd_op.hip -- TEST INFRASTRUCTURE: the device side of the user-op tests (tests/test_gpu_user_op.py).
// A user-defined, non-commutative op, MPI's user-function convention inout = in o inout with in o inout =
// in * 0.5 + inout on float and double, rounded after the multiply (built with -ffp-contract=off), and
// 3 * in + inout (wrapping) on int32: the same function the reference runs as MPI_Op_create(halfadd, commute = 0) in
// oracle/ref_driver.cpp, restated by the oracle as ORC_USER_HALFADD.  Exported as chr_user_reduce_fns through
// include/chiara_user_op.hpp.
#include "chiara_user_op.hpp"

struct HalfAdd {
    __device__ float operator()(float in, float inout) const {
        const float h = in * 0.5f;
        return h + inout;
    }
};
struct HalfAddD {
    __device__ double operator()(double in, double inout) const {
        const double h = in * 0.5;
        return h + inout;
    }
};
struct Mix3 {  // the same MPI function on MPI_INT: 3 * in + inout, wrapping
    __device__ int32_t operator()(int32_t in, int32_t inout) const {
        return (int32_t)((uint32_t)in * 3u + (uint32_t)inout);
    }
};

CHR_DEFINE_USER_OP(chr_test_halfadd_f32, float, HalfAdd)

// One op over three types, as an MPI user function switches on its datatype argument: the launcher picks the
// instantiation by dtype and refuses the others.
extern "C" int chr_test_halfadd(void* out, const void* acc, const void* const* ins, int m, size_t n, chr_dtype dt,
                                int running_first, hipStream_t stream, void*) {
    switch (dt) {
    case CHR_FLOAT32: return chr_user::launch_fold<float, HalfAdd>(out, acc, ins, m, n, running_first, stream);
    case CHR_FLOAT64: return chr_user::launch_fold<double, HalfAddD>(out, acc, ins, m, n, running_first, stream);
    case CHR_INT32: return chr_user::launch_fold<int32_t, Mix3>(out, acc, ins, m, n, running_first, stream);
    default: return 1;
    }
}

// A commutative, associative user op (int32 wrapping add): any schedule gives MPI's own collective's bits, so the
// MPI-signature shim's binding can be checked against MPI_Allreduce (csrc/harness/shim_types_main.cpp).
struct IAdd {
    __device__ int32_t operator()(int32_t in, int32_t inout) const { return (int32_t)((uint32_t)in + (uint32_t)inout); }
};
CHR_DEFINE_USER_OP_FOR(chr_test_isum, int32_t, IAdd, CHR_INT32)

// A launcher that refuses every call: the library must hand its verdict back (CHR_ERR_UNSUPPORTED).
extern "C" int chr_test_refuse(void*, const void*, const void* const*, int, size_t, chr_dtype, int, hipStream_t,
                               void*) {
    return 1;
}
