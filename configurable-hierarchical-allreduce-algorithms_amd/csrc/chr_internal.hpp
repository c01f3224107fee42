// chr_internal.hpp -- declarations shared by the libchiara translation units.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>

#include "chiara.h"

namespace chr {

size_t dtype_size(int dtype);
bool valid_dtype_op(int dtype, int op);
// The kernel instantiation (type, op) that computes (dtype, op) bit-exactly (reduce_kernels.hip).
void canon_op(int dtype, int op, bool running_first, int* kdt, int* kop);

// Fused bucket reduction: out = (...((acc op ins[0]) op ins[1])...) op ins[m-1], each step
// MPI_Reduce_local(ins[j], acc) = OP(ins[j], acc); with running_first each step is
// OP(acc, ins[j]) instead (MPICH_do_reduce's order).  Device pointers.  m may exceed the
// kernel's fan-in: chained left to right.
hipError_t launch_reduce(void* out, const void* acc, const void* const* ins, int m, size_t n,
                         int dtype, int op, hipStream_t stream, bool running_first = false);

// Fused expression tree (reduce_kernels.hip, k_reduce_tree): leaves in push order; comb[j] =
// binary combines after pushing leaf j; swaps[c] = 1 if combine c takes the running value as
// the `in` operand.  At most 8 leaves, stack depth 4 (tree_program_ok checks).
hipError_t launch_reduce_tree(void* out, const void* const* leaves, int nl, const uint8_t* comb,
                              const uint8_t* swaps, size_t n, int dtype, int op, hipStream_t stream);
bool tree_program_ok(int nl, const uint8_t* comb, const uint8_t* swaps, uint32_t* comb_bits,
                     uint32_t* swap_bits);
// Several trees, batched: the vector bodies of equal-leaf-count trees share launches (at most 8
// per launch).  Each job is one chr_reduce_tree call.
struct TreeJob {
    void* out;
    const void* leaves[8];
    int nl;
    const uint8_t* comb;
    const uint8_t* swaps;
    size_t n;
};
hipError_t launch_reduce_tree_multi(const TreeJob* jobs, int njobs, int dtype, int op, hipStream_t stream);

hipError_t launch_fill(void* buf, size_t n, int dtype, int pattern, uint64_t seed, int rank,
                       uint64_t count_for_seq, hipStream_t stream);

// Tunables (read once from the environment):
//   CHR_REDUCE_MAX_LAUNCH_VEC  cap on the 16-B vectors one bucket launch or one tree segment
//                            covers (default: 2^31 threads / 1 GiB); tests set it small to run the
//                            splitting paths at oracle sizes
//   CHR_XCD_RUN_KIB          streaming (NT) calls: KiB of consecutive trips each XCD takes before
//                            the next XCD's run (0 = plain round-robin); unset = policy
//                            (xcd_run_shift in reduce_common.hpp)
//   CHR_REDUCE_NT            0 / 1 forces plain / non-temporal loads+stores; unset = by size
//   CHR_REDUCE_NT_MIN_BYTES  bytes streamed by one call from which NT is used (40 MiB for
//                            bucket launches, 64 MiB for tree launches; the variable sets both)
//   CHR_WG_PER_CU_VEC        streaming (NT) bucket launches: at most this many workgroups resident
//   CHR_WG_PER_CU_TREE       per CU, capped through dynamic LDS (0 = uncapped); unset = policy
//                            (nt_lds_bytes in reduce_common.hpp); likewise for the tree kernel
struct ReduceTuning {
    int xcd_run_kib;        // -1: policy
    size_t max_launch_vec;  // 0: the grid limit; else cap on 16-B vectors per launch / tree segment
    int nt_mode;
    size_t nt_min_bytes;       // bucket launches
    size_t tree_nt_min_bytes;  // tree launches
    int wg_per_cu_vec;   // -1: policy
    int wg_per_cu_tree;  // -1: policy
    int xcd_hand_shift;  // -1: policy (xcd_hand in reduce_common.hpp); 0: off
    unsigned lds_per_cu; // bytes of LDS per CU (device attribute; 160 KiB on gfx950)
    unsigned lds_per_block;  // bytes of LDS one workgroup may allocate (device attribute)
};
ReduceTuning& reduce_tuning();

// Streaming launches issued on this host thread while a CoresidentScope is open share the GPU with
// RCCL's kernels and leave them room: at most kCoresidentWgPerCu resident workgroups per CU
// (stream_wg_cap in reduce_common.hpp, which gives the measurements).
constexpr int kCoresidentWgPerCu = 12;
int& coresident_depth();  // per host thread (reduce_kernels.hip)
struct CoresidentScope {
    bool on;
    explicit CoresidentScope(bool enable) : on(enable) {
        if (on) ++coresident_depth();
    }
    ~CoresidentScope() {
        if (on) --coresident_depth();
    }
    CoresidentScope(const CoresidentScope&) = delete;
    CoresidentScope& operator=(const CoresidentScope&) = delete;
};

}  // namespace chr
