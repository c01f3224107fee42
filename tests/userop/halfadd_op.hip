// halfadd_op.hip -- TEST INFRASTRUCTURE: the device side of the user-op tests (tests/test_gpu_user_op.py).
// A user-defined, non-commutative op on float, MPI's user-function convention inout = in o inout with
// in o inout = in * 0.5f + inout, rounded after the multiply (built with -ffp-contract=off): the same function the
// reference runs as MPI_Op_create(halfadd, commute = 0) in oracle/ref_driver.cpp, restated by the oracle as
// ORC_USER_HALFADD.  Exported as a chr_user_reduce_fn through include/chiara_user_op.hpp.
#include "chiara_user_op.hpp"

struct HalfAdd {
    __device__ float operator()(float in, float inout) const {
        const float h = in * 0.5f;
        return h + inout;
    }
};

CHR_DEFINE_USER_OP(chr_test_halfadd, float, HalfAdd)

// A launcher that refuses every call: the library must hand its verdict back (CHR_ERR_UNSUPPORTED).
extern "C" int chr_test_refuse(void*, const void*, const void* const*, int, size_t, chr_dtype, int, hipStream_t,
                               void*) {
    return 1;
}
