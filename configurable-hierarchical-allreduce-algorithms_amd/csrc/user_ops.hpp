// user_ops.hpp -- user-defined reduction ops (chr_op_create) and the dispatchers every reduction of the library goes
// through: a user op runs the caller's own device launcher, a predefined op the library's kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "chr_internal.hpp"

namespace chr {

// User ops take the chr_op codes [kUserOpBase, kUserOpBase + kMaxUserOps): above every predefined op and every
// internal kernel code (kMaxSw ... kProdSw).
constexpr int kUserOpBase = 64;
constexpr int kMaxUserOps = 64;

bool is_user_op(int op);
// MPI_Op_commutative: every predefined op is commutative; a user op as chr_op_create recorded it.
bool op_commutative(int op);
// A live user op on a type with a size, or a (type, op) pair MPICH's table accepts (valid_dtype_op).
bool valid_any(int dtype, int op);

// The reductions: chr_result codes.  reduce_any is MPI_Reduce_local chained over ins (launch_reduce's contract);
// reduce_tree_any evaluates one post-order program (launch_reduce_tree's); reduce_tree_multi_any a batch of them.
int reduce_any(void* out, const void* acc, const void* const* ins, int m, size_t n, int dtype, int op, hipStream_t s,
               bool running_first = false);
int reduce_tree_any(void* out, const void* const* leaves, int nl, const uint8_t* comb, const uint8_t* swaps, size_t n,
                    int dtype, int op, hipStream_t s);
int reduce_tree_multi_any(const TreeJob* jobs, int njobs, int dtype, int op, hipStream_t s);

}  // namespace chr
