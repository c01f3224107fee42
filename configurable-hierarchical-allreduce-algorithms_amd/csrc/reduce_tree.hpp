// reduce_tree.hpp -- the fused expression-tree kernel (templates), shared by reduce_tree.hip
// (floating types, int32 arithmetic) and reduce_tree_int.hip (the other integer types, logical
// and bitwise ops).
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>

#include "reduce_common.hpp"

namespace chr {

// ---- fused expression tree: one HBM pass for a whole chunk's reduction ---------------------
//
// The flat schedule (schedule.cpp build_plan_flat) evaluates, per chunk, the expression
// tree the reference builds across its phases: recexch folds (all_reduce_radix_batch.cpp
// :364 / :446), step-1 folds (:332) and the lane reduction (:529).  As separate launches every
// inner node is written to HBM and read back; here the whole tree is evaluated in registers,
// so one launch reads each leaf once and writes the root once: (NL + 1) * n * sizeof(T)
// bytes instead of sum over nodes of (m + 2) * n * sizeof(T) (C4's 8-leaf tree: 9 vs 13).
//
// Program: a stack machine in post-order.  Leaves arrive in the order they are pushed;
// after pushing leaf j, comb_j binary combines follow (2 bits per leaf).  A combine pops
// the top (the next operand `in` of a left fold) into the value below it (the fold's running
// value): below = OP(in, below), i.e. MPI_Reduce_local(in, below); with the combine's swap
// bit set the running value is the `in` of MPI_Reduce_local (MPICH_do_reduce order).
// The stack depth is uniform across the grid, so every stack access is a scalar branch over
// static register slots (no scratch).  Depth <= kTreeDepth, leaves <= kMaxLeaves.
constexpr int kMaxLeaves = 8;
constexpr int kTreeDepth = 4;

// Segments: one launch may evaluate several trees with the same leaf count (the flat schedule's
// chunks of one pipeline slice): each has its own leaves, output, length and program, and owns
// the workgroups [block0, next block0).  At C4 this halves the launches per call and doubles the
// bytes per launch, so the fixed fill/drain cost of a grid (~4 us) is paid half as often.
constexpr int kMaxTreeSegs = 8;

struct TreeSeg {
    u32x4* out;
    const u32x4* leaves[kMaxLeaves];
    size_t nvec;
    uint32_t comb;    // 2 bits per leaf
    uint32_t swaps;   // 1 bit per combine, in program order
};

// The per-segment workgroup table comes first, so a workgroup finds its segment from one scalar
// load of 64 bytes (set by launch_tree_vec): block0 ascending, ~0u past the last segment.
struct TreeArgs {
    uint32_t block0[kMaxTreeSegs];  // first workgroup of each segment
    uint32_t xfull[kMaxTreeSegs];   // each segment's blocks [0, xfull) take the XCD map (xcd_full)
    TreeSeg seg[kMaxTreeSegs];
    int nseg;
    int nl;
    uint32_t hand[kMaxTreeSegs];   // each segment's odd-XCD handover in trips (xcd_trip_w); 0 = none.  Computed
                                   // once, by the launcher, which also sizes the grid from it
    uint32_t xrun;    // log2 of the trips per XCD run within a segment (xcd_trip); set by the launcher
};

// A segment's vector body is at most this many 16-B vectors (1 GiB per operand); longer trees are
// cut into several segments, so a grid stays far below 2^31 threads.
constexpr size_t kMaxSegVec = (size_t)1 << 26;

// Whether MPI_Reduce_local(running, next) can differ bitwise from MPI_Reduce_local(next, running):
// MAX / MIN on floating types and MAXLOC / MINLOC on floating-valued pairs (ties, -0 / +0, NaN), and SUM / PROD on
// the floating and the complex types when two NaNs meet (whose payload survives: kSumSw in reduce_common.hpp).
template <int DT, int OP>
constexpr bool order_sensitive() {
    return (is_float_dt<DT>() && (OP == CHR_MAX || OP == CHR_MIN || OP == CHR_SUM || OP == CHR_PROD)) ||
           ((DT == CHR_FLOAT_INT || DT == CHR_DOUBLE_INT) && (OP == CHR_MAXLOC || OP == CHR_MINLOC)) ||
           (is_complex_dt<DT>() && (OP == CHR_SUM || OP == CHR_PROD));
}

// Generic over the value carried per lane (W values of type V, combined with F).  The stack
// slots are four named values per w, never an array: an array indexed by the runtime depth
// would be merged into dynamically addressed scratch; named values stay in registers
// (pushes become v_cndmask with a scalar condition, combines scalar branches).
template <typename V, int NL, int W, typename F>
__device__ __forceinline__ void tree_eval(const V (&x)[NL][W], V (&r)[W], uint32_t comb, uint32_t swaps) {
#pragma unroll
    for (int w = 0; w < W; ++w) {
        V s0 = x[0][w], s1 = s0, s2 = s0, s3 = s0;  // leaf 0 is pushed first, comb[0] == 0
        int d = 1, ci = 0;
#pragma unroll
        for (int j = 1; j < NL; ++j) {
            const V v = x[j][w];
            if (d == 1) s1 = v;
            else if (d == 2) s2 = v;
            else s3 = v;
            ++d;
            for (int c = (int)((comb >> (2 * j)) & 3u); c > 0; --c, ++ci) {
                const bool sw = (swaps >> ci) & 1u;
                if constexpr (F::kOrderSensitive) {
                    // a swapped combine is the plain one on exchanged operands: select them, combine once.
                    // Written as `sw ? apply<kSumSw>(in, run) : apply<SUM>(in, run)`, both pinned-order
                    // combines were computed and one selected, and the bf16 SUM trees held 80 VGPRs instead of
                    // 61 (RCCL's room beside them)
                    if (d == 2) s0 = F::ap(sw ? s0 : s1, sw ? s1 : s0);
                    else if (d == 3) s1 = F::ap(sw ? s1 : s2, sw ? s2 : s1);
                    else s2 = F::ap(sw ? s2 : s3, sw ? s3 : s2);
                } else {  // bitwise commutative: the swap bit changes nothing
                    if (d == 2) s0 = F::ap(s1, s0);
                    else if (d == 3) s1 = F::ap(s2, s1);
                    else s2 = F::ap(s3, s2);
                }
                --d;
            }
        }
        r[w] = s0;
    }
}

// ---- programs known at compile time ------------------------------------------------------------------------
// tree_eval interprets the program at run time: every push and combine is a scalar branch over the stack depth,
// with u32x4 moves between the named slots.  That VALU tail after a trip's loads land stretches the workgroup's
// life, which costs the most where residency is capped -- beside RCCL, 12 workgroups per CU -- and for bf16, whose
// combines widen, add and RNE-pack (tools/reduce_microbench focus34, profiles/r05/microbench_focus34_static_tree.txt:
// C4's tree at cap 12, 16 MiB pieces, cold f32 0.753-0.762 -> 0.782-0.784, bf16 0.723-0.737 -> 0.778-0.793; 8 MiB
// f32 0.684-0.689 -> 0.721-0.724, bf16 0.646-0.652 -> 0.710-0.715; cap 16 +1-3 %).  The programs the flat
// schedule emits at 2, 4 and 8 ranks (every k and b; enumerated from chr_plan_describe) are unrolled at compile time
// and chosen by one scalar compare per workgroup; anything else (other rank counts, swapped combines) keeps the
// interpreter.  Same combines in the same order: only the instruction stream changes.  Through the product: one
// GPU's own C4 grids at cap 12 0.767 -> 0.798, 0.688 -> 0.752 on just-received leaves, C5 0.705 -> 0.763
// (profiles/r05/static_tree/).
constexpr uint32_t tree_prog(const int (&c)[8], int nl) {
    uint32_t v = 0;
    for (int j = 0; j < nl; ++j) v |= (uint32_t)c[j] << (2 * j);
    return v;
}
template <int NL> struct StaticProgs { static constexpr int n = 0; static constexpr uint32_t v[1] = {0}; };
template <> struct StaticProgs<8> {
    static constexpr int n = 6;
    static constexpr uint32_t v[6] = {
        tree_prog({0, 1, 1, 1, 0, 1, 1, 2}, 8),  // b = 4, k >= 3: C4 / C5
        tree_prog({0, 1, 0, 2, 0, 2, 0, 2}, 8),  // b = 2, any k
        tree_prog({0, 1, 0, 2, 0, 1, 0, 3}, 8),  // b = 4 / 8, k = 2
        tree_prog({0, 1, 1, 0, 1, 2, 0, 2}, 8),  // b = 8, k = 3
        tree_prog({0, 1, 1, 1, 0, 2, 1, 1}, 8),  // b = 8, k = 4
        tree_prog({0, 1, 1, 1, 1, 1, 1, 1}, 8)}; // b = 8, k >= 5: a left fold
};
template <> struct StaticProgs<2> {  // the tree API's 2-leaf program: no flat plan emits one (a 2-operand
                                     // expression is one fold, k_reduce_vec; C3 and the N = 2 line fold)
    static constexpr int n = 1;
    static constexpr uint32_t v[1] = {tree_prog({0, 1, 0, 0, 0, 0, 0, 0}, 2)};
};
template <> struct StaticProgs<4> {
    static constexpr int n = 2;
    static constexpr uint32_t v[2] = {tree_prog({0, 1, 0, 2, 0, 0, 0, 0}, 4), tree_prog({0, 1, 1, 1, 0, 0, 0, 0}, 4)};
};

// One program, unrolled: push leaf j, then its combines, each below = F(in = top, below) (no swapped combines).
template <typename V, int NL, int W, typename F, uint32_t COMB>
__device__ __forceinline__ void tree_eval_static(const V (&x)[NL][W], V (&r)[W]) {
#pragma unroll
    for (int w = 0; w < W; ++w) {
        V st[kTreeDepth];
        int d = 0;
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            st[d++] = x[j][w];
#pragma unroll
            for (int c = (int)((COMB >> (2 * j)) & 3u); c > 0; --c) {
                st[d - 2] = F::ap(st[d - 1], st[d - 2]);
                --d;
            }
        }
        r[w] = st[0];
    }
}

// The unrolled body of `comb` when it is one of StaticProgs<NL> and no combine is swapped (or the op is bitwise
// commutative, so a swap bit changes nothing), else the interpreter.
template <typename V, int NL, int W, typename F, int I = 0>
__device__ __forceinline__ void tree_eval_fast(const V (&x)[NL][W], V (&r)[W], uint32_t comb, uint32_t swaps) {
    if constexpr (I < StaticProgs<NL>::n) {
        constexpr uint32_t P = StaticProgs<NL>::v[I];
        if ((swaps == 0 || !F::kOrderSensitive) && comb == P) {
            tree_eval_static<V, NL, W, F, P>(x, r);
            return;
        }
        tree_eval_fast<V, NL, W, F, I + 1>(x, r, comb, swaps);
    } else {
        tree_eval<V, NL, W, F>(x, r, comb, swaps);
    }
}

// F::ap(in, run) is MPI_Reduce_local(in, inout = run).  A swapped combine -- MPICH_do_reduce's
// MPI_Reduce_local(run, in) -- is F::ap(run, in): the tree evaluators exchange the operands (the swapped codes
// kMaxSw ... kProdSw of reduce_common.hpp serve the bucket kernels, whose result lands in the other buffer).
template <int DT, int OP>
struct VecOp {
    static constexpr bool kOrderSensitive = order_sensitive<DT, OP>();
    __device__ __forceinline__ static u32x4 ap(u32x4 in, u32x4 run) { return apply_vec<DT, OP>(in, run); }
};

// The scalar kernel's stack slots: the element type itself, except for the pair and complex
// structs, which ride the slots as vectors of their 32-bit words and are bit-cast to the struct only
// inside a combine.  With the structs themselves as slot values, the slot selects of tree_eval were
// miscompiled for C_FLOAT_COMPLEX at depth 4 (a leaf's words shifted by one: tests/test_gpu_tree.py
// ::test_tree_scalar_path_pair_and_complex_every_program, round 3).
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
template <int NW> struct WordsOf;
template <> struct WordsOf<2> { using V = u32x2; };
template <> struct WordsOf<4> { using V = u32x4; };
template <int DT, bool WORDS = is_pair_dt<DT>() || is_complex_dt<DT>()>
struct SlotOf {
    using V = typename DTy<DT>::T;
};
template <int DT>
struct SlotOf<DT, true> {
    using V = typename WordsOf<sizeof(typename DTy<DT>::T) / 4>::V;
};
template <int DT>
using slot_t = typename SlotOf<DT>::V;

template <int DT, int OP>
struct ScalarOp {
    using T = typename DTy<DT>::T;
    using V = slot_t<DT>;
    static constexpr bool kOrderSensitive = order_sensitive<DT, OP>();
    __device__ __forceinline__ static V ap(V in, V run) {
        if constexpr (std::is_same_v<V, T>) return apply<DT, OP>(in, run);
        else return __builtin_bit_cast(V, apply<DT, OP>(__builtin_bit_cast(T, in), __builtin_bit_cast(T, run)));
    }
};

// U vectors per lane per trip for NL leaves: every leaf load of the trip is issued before
// the first combine (NL * U <= 16 loads of 16 B in flight per lane).  One trip per workgroup;
// within its segment a workgroup's trip is placed by xcd_trip (the segment's first block may sit
// anywhere in the 8-XCD rotation: blocks of one local residue class still share one XCD).
// ACC0 (streaming trees, round 6): leaf 0's first vector keeps the default policy, as the bucket kernel's ACC0 slot
// (reduce_vec.hpp).  One GPU's own C4 / C5 grids at the in-collective cap, rocprof kernel duration per grid, off -> on
// (bench.py --rank-trees, profiles/r06/acc0_ab/, 2 alternating rounds): C4 4 slices 0.779-0.792 -> 0.828-0.833,
// 8 slices 0.735-0.738 -> 0.790, 8 slices after the receive copies 0.687-0.692 -> 0.732-0.735; C5 4 slices 0.769 ->
// 0.812-0.814, 8 slices 0.737-0.766 -> 0.794-0.797, after copies 0.675-0.679 -> 0.732-0.739; 4 slices after the
// copies tie.  The C4 tree alone over a 4.5 GiB rotation (tools/tree_pmc.py, past the translation cliff) loses 2 %
// (0.779-0.791 -> 0.766-0.773), as the 2-leaf tree does over 3.9 GiB (tools/leaf2_ab.py: -2.5 %; +3.5-4 % at 1.9
// GiB).  A rank's call holds ~3 GiB (send, recv, STAGE), the rows that gain.
template <int DT, int OP, int NL, int U, bool NT, int BL, bool ACC0 = false>
__global__ __launch_bounds__(BL) void k_reduce_tree(TreeArgs a) {
    // this workgroup's segment: one pass over the block0 table (scalar compares, no loop-carried
    // loads), then the segment's pointers pinned into SGPRs before the first vector load
    const uint32_t b = blockIdx.x, xrun = a.xrun;
    uint32_t b0s[kMaxTreeSegs], xfs[kMaxTreeSegs], hds[kMaxTreeSegs];
#pragma unroll
    for (int j = 0; j < kMaxTreeSegs; ++j) {
        b0s[j] = a.block0[j];
        xfs[j] = a.xfull[j];
        hds[j] = a.hand[j];
        pin_sgpr_u32(b0s[j], xfs[j]);
        pin_sgpr_u32(hds[j], xrun);
    }
    int s = 0;
    uint32_t b0 = 0, xfull = xfs[0], hand = hds[0];
#pragma unroll
    for (int j = 1; j < kMaxTreeSegs; ++j)
        if (b >= b0s[j]) {
            s = j;
            b0 = b0s[j];
            xfull = xfs[j];
            hand = hds[j];
        }
    const TreeSeg& g = a.seg[s];
    u32x4* const out = g.out;
    const u32x4* leaves[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) leaves[j] = g.leaves[j];
    const size_t nvec = g.nvec;
    const uint32_t comb = g.comb, swaps = g.swaps;
    pin_sgpr(out, leaves[0], nvec, comb, swaps);
#pragma unroll
    for (int j = 1; j < NL; ++j) pin_sgpr(leaves[j]);
    // segments start on a multiple of 8 blocks when a handover is set, so a local block's XCD parity is
    // its global one
    const size_t trip = xcd_trip_w(b - b0, xfull, xrun, hand);
    if (trip == kIdleTrip) return;
    const size_t base = trip * BL * U + threadIdx.x;
    if ((trip + 1) * BL * U <= nvec) {
        u32x4 x[NL][U];
        x[0][0] = ld<NT && !ACC0>(&leaves[0][base]);  // peeled: one instruction per policy (reduce_vec.hpp)
#pragma unroll
        for (int u = 1; u < U; ++u) x[0][u] = ld<NT>(&leaves[0][base + (size_t)u * BL]);
#pragma unroll
        for (int j = 1; j < NL; ++j)
#pragma unroll
            for (int u = 0; u < U; ++u) x[j][u] = ld<NT>(&leaves[j][base + (size_t)u * BL]);
        __builtin_amdgcn_sched_barrier(0);
        u32x4 r[U];
        tree_eval_fast<u32x4, NL, U, VecOp<DT, OP>>(x, r, comb, swaps);
#pragma unroll
        for (int u = 0; u < U; ++u) st<NT>(&out[base + (size_t)u * BL], r[u]);
    } else {
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * BL;
            if (i >= nvec) break;
            u32x4 x[NL][1];
#pragma unroll
            for (int j = 0; j < NL; ++j) x[j][0] = leaves[j][i];
            u32x4 r[1];
            tree_eval<u32x4, NL, 1, VecOp<DT, OP>>(x, r, comb, swaps);
            out[i] = r[0];
        }
    }
}

struct TreeScalarArgs {
    void* out;
    const void* leaves[kMaxLeaves];
    size_t n;
    int nl;
    uint32_t comb, swaps;
};

template <int DT, int OP, int NL>
__global__ __launch_bounds__(kBlock) void k_reduce_tree_scalar(TreeScalarArgs a) {
    using T = typename DTy<DT>::T;
    using V = slot_t<DT>;
    for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < a.n; i += (size_t)gridDim.x * kBlock) {
        V x[NL][1];
#pragma unroll
        for (int j = 0; j < NL; ++j) x[j][0] = __builtin_bit_cast(V, ((const T*)a.leaves[j])[i]);
        V r[1];
        tree_eval<V, NL, 1, ScalarOp<DT, OP>>(x, r, a.comb, a.swaps);
        ((T*)a.out)[i] = __builtin_bit_cast(T, r[0]);
    }
}

// The odd-XCD handover for streaming tree launches (xcd_trip_w): each odd XCD hands 1/2^shift of its
// share of a segment to the even XCD below.  Same-box A/Bs (profiles/r04/ab_hand/, 2 alternating rounds
// each):
//  * HBM-cold leaves -- whole C4 calls on 8 virtual ranks, one grid per rank and slice
//    (bench.py --collective-kernels): shift 7 0.754, 6 0.756-0.759, 5 0.760, 4 0.759-0.765, 3 0.745-0.749,
//    off 0.749; tree_bench's cold batched slices: 6 and 4 +0.5-1.3 % over off;
//  * leaves just rewritten (tree_bench's warm batched slices, 7 of 8 leaves copied in first, as RCCL's
//    receives leave them on a node): off 0.759 / 0.756 at 16 MiB pieces, 6 0.752 / 0.757, 4 0.715 / 0.721.
// (The bucket kernel's odd XCDs still lag on cache-resident operands, 2.2 % against 3 % cold: reduce_microbench
// focus29; what the warm tree rows respond to is not pinned down.)  On a node 7 of a tree's 8 leaves arrive
// over xGMI just before the launch, so the mild shift 6 is kept: it gains on cold leaves and costs at most
// ~1 % on warm ones, where 4 costs 5 %.  Round 5 re-ran it on one GPU's own grids with the receive copies in
// front (bench.py rank-alone rows, profiles/r05/ab_treebl/, 2 alternating rounds): off 0.671 / 0.673 vs 6 0.657
// / 0.690 at 4 slices, 0.594 / 0.544 vs 0.540 / 0.603 at 8 -- a tie inside the rows' noise -- and 6 ahead on
// cold leaves (whole-call spans 0.763 / 0.774 vs 0.736 / 0.747).
constexpr int kTreeXcdHandShift = 6;

// XCD runs for streaming (nt) tree launches (profiles/r02/xcd_runs/ab_tree_*.json, C4 slice of 2
// batched 8-leaf trees, HBM-cold, identity -> 512 KiB): 8 MiB pieces 0.571 -> 0.634, 16 MiB
// 0.668 -> 0.700, 32 MiB 0.719 -> 0.750; fused reductions of a whole C4 call 0.676 -> 0.719.
// Two leaves move the m = 1 bucket's traffic (2 reads + 1 write) and kept the identity until focus18's
// microbench lead for 256 KiB runs under a cap was product-verified:
// Round 5, the product A/B focus18 asked for (tools/gpu_small_tree_ab.sh, profiles/r05/small_tree_ab/, 2
// alternating rounds, HBM-cold, f32): the 2- and 4-leaf trees (4-rank flat plans with k < b; the tree API) take 256 KiB runs and 12
// per CU (tree_wg_per_cu) -- alone 0.745-0.747 -> 0.765-0.766 (2 leaves, 64 MiB pieces), 0.677-0.690 -> 0.707 (two
// trees of 16 MiB), 0.778-0.784 -> 0.791-0.800 (4 leaves, 64 MiB), 0.744-0.745 -> 0.750-0.757 (2 x 16 MiB); at
// the in-collective cap 12 the runs add 0-1.4 %.
template <int NL>
constexpr size_t tree_xcd_run_kib() {
    return NL <= 4 ? 256 : 512;
}

// Two-wave workgroups at the same 16 waves per CU (fewer dispatches per grid): the
// microbench put them 1-2 % ahead on C4's slice at 8 / 16 MiB pieces (tools/reduce_microbench focus30,
// profiles/r05/microbench_focus30_tree_bl.txt: 0.771-0.780 vs 0.754-0.764 cold at 16 MiB); through the product
// (a CHR_TREE_BL knob, profiles/r05/ab_treebl/, 2 alternating rounds) the rank-alone C4 / C5 rows moved within
// their +-3 % noise, so the one-wave shape stays.  U = 2 and 256-thread shapes lost 1-4 % in the microbench.
// Vectors per lane per trip and resident workgroups per CU (nt_lds_bytes; 0 = uncapped) of
// streaming tree launches.  At U = 2, 8-12 per CU moved the C4/C5 collective rows by -2..+1 %
// (profiles/r02/occupancy_cap/); U = 1 with 16 per CU measured 0.751-0.763 against U = 2
// uncapped's 0.739-0.750 on the C4 slice (2 x 8 leaves x 16 MiB, 4.5 and 1.1 GiB rotations, 2
// rounds: microbench_focus17_tree_u_cap.txt), so trees of 5+ leaves take that shape.  The small
// trees of 2 and 4 leaves (focus18, microbench_focus18_small_trees.txt, 2 rounds,
// 6 HBM-cold sets) showed 2 leaves at 128 MiB U = 4 uncapped 0.774-0.783 -> 0.801-0.804 with 12 per
// CU and 256 KiB runs, and 4 leaves at 64 MiB 0.741-0.750 -> 0.774-0.781 at U = 2 with 12 per CU,
// but the microbench over-predicted the 8-leaf change below, so trees of <= 4 leaves kept the round-1
// shapes (U = 4, uncapped) until round 5's product A/Bs: U = 2 for 3-4 leaves (below), 12 per CU and 256 KiB
// runs for 2-4 (tree_xcd_run_kib).
// For the U = 1 8-leaf tree the microbench preferred 12 per CU with 1-2 MiB
// XCD runs (focus20: 0.760 -> 0.772-0.782 on the C4 slice), but the same-box product A/B over the
// whole C4/C5 calls reversed it (profiles/r02/ab_tree/: 16 per CU / 512 KiB 0.7245-0.7255 (C4),
// 0.703-0.709 (C5) against 0.695-0.697 / 0.688), so 16 / 512 KiB stays -- except beside RCCL
// (stream_wg_cap), where every tree takes kCoresidentWgPerCu: at 16 or uncapped RCCL's kernel waits
// for the tree launch to drain (profiles/r03/coresidency/).
// Beside RCCL (cap 12) U = 2 would keep more bytes in flight -- one GPU's own C4 / C5 grids on just-received leaves
// +4-7 % (profiles/r05/ab_treeu/, 3 rounds) -- but it needs 82-90 VGPRs per wave against U = 1's 50-58, and then
// three tree waves on a SIMD leave less than the ~288 VGPRs rcclGenericKernel's waves need: an RCCL-sized kernel
// was admitted only when the tree launch drained (median 170 us against 4 us) and the real RCCL kernel beside the
// C4 slice took 164-165 us against 114-120 us (tools/gpu_cores_u.sh, profiles/r05/cores_u/).  U = 1 stays.
// The same budget (<= 72 VGPRs, tests/test_kernel_resources.py) moved the streaming 3- and 4-leaf trees of 4-rank
// flat plans with k < b from U = 4 (104 f32 / 112 bf16 VGPRs) to U = 2 (62 / 65): beside 4-leaf f32 trees of 64 MiB
// pieces at cap 12 an RCCL-sized kernel's median workgroup was admitted after 5.5 / 17.6 us instead of ~90 us
// (the launch drained first), the real RCCL kernel took 122-123 us instead of 129-133, and the trees ran faster
// too, 0.770 / 0.780 vs 0.761 / 0.741 at cap 12 and 0.759 vs 0.746 at the stand-alone policy
// (tools/gpu_cores_ab.sh LEAVES=4, profiles/r05/cores_ab_l4/, 2 alternating rounds of 3).
template <int NL, bool NT>
constexpr int tree_u() {
    if constexpr (!NT) return NL <= 4 ? 4 : 2;  // cache-warm (plain) launches: the round-1 shapes
    return NL <= 2 ? 4 : NL <= 4 ? 2 : 1;
}
template <int NL>
constexpr int tree_wg_per_cu() {
    return NL <= 4 ? 12 : 16;
}

template <int DT, int OP, int NL, int BL, bool NT>
inline hipError_t launch_tree_vec(const TreeArgs& a_in, hipStream_t s) {
    constexpr int U = is_complex_dt<DT>() && (OP == CHR_PROD || OP == kProdSw) ? 1 : tree_u<NL, NT>();  // vec_u_dt
    TreeArgs a = a_in;
    a.xrun = NT ? xcd_run_shift(tree_xcd_run_kib<NL>(), (size_t)BL * U * 16) : 0;
    // the odd-XCD handover of streaming launches (xcd_hand / xcd_trip_w in reduce_common.hpp), per segment
    const int henv = reduce_tuning().xcd_hand_shift;
    const int hshift = NT ? (henv >= 0 ? henv : kTreeXcdHandShift) : 0;
    size_t grid = 0;
    for (int j = 0; j < kMaxTreeSegs; ++j) {
        if (j >= a.nseg) {
            a.block0[j] = ~0u;
            a.xfull[j] = 0;
            a.hand[j] = 0;
            continue;
        }
        if (a.seg[j].nvec > kMaxSegVec) return hipErrorInvalidValue;  // launch_reduce_tree_multi cuts them
        const size_t trips = (a.seg[j].nvec + (size_t)BL * U - 1) / ((size_t)BL * U);
        if (hshift) grid = (grid + 7) & ~(size_t)7;  // the segment starts on XCD 0 (its padding blocks idle)
        a.block0[j] = (uint32_t)grid;
        a.xfull[j] = xcd_full((uint32_t)trips, a.xrun);
        a.hand[j] = xcd_hand(a.xfull[j], hshift);  // the kernel maps with exactly the hand the grid is sized for
        grid += trips + 8u * (size_t)a.hand[j];
    }
    if (grid == 0) return hipSuccess;
    const unsigned lds = NT ? nt_lds_bytes(reduce_tuning().wg_per_cu_tree, tree_wg_per_cu<NL>()) : 0;
    constexpr bool ACC0 = NT && !is_pair_dt<DT>() && !is_complex_dt<DT>();  // the ACC0 slot (k_reduce_tree)
    hipLaunchKernelGGL((k_reduce_tree<DT, OP, NL, U, NT, BL, ACC0>), dim3((unsigned)grid), dim3(BL), lds, s, a);
    return hipGetLastError();
}

template <int DT, int OP, int NL>
inline hipError_t launch_tree_scalar_nl(const TreeScalarArgs& sa, hipStream_t s) {
    const size_t trips = (sa.n + kBlock - 1) / kBlock;
    const int grid = (int)(trips < 2048 ? trips : 2048);
    hipLaunchKernelGGL((k_reduce_tree_scalar<DT, OP, NL>), dim3(grid), dim3(kBlock), 0, s, sa);
    return hipGetLastError();
}

// Scalar (any alignment) trees only.
template <int DT, int OP>
inline hipError_t launch_tree_scalar_op(const TreeScalarArgs& sa, hipStream_t s) {
    switch (sa.nl) {
    case 2: return launch_tree_scalar_nl<DT, OP, 2>(sa, s);
    case 3: return launch_tree_scalar_nl<DT, OP, 3>(sa, s);
    case 4: return launch_tree_scalar_nl<DT, OP, 4>(sa, s);
    case 5: return launch_tree_scalar_nl<DT, OP, 5>(sa, s);
    case 6: return launch_tree_scalar_nl<DT, OP, 6>(sa, s);
    case 7: return launch_tree_scalar_nl<DT, OP, 7>(sa, s);
    case 8: return launch_tree_scalar_nl<DT, OP, 8>(sa, s);
    default: return hipErrorInvalidValue;
    }
}

// The policy shapes only (nt: one wave; plain: 256 threads), as in reduce_vec.hpp.
template <int DT, int OP, int NL>
inline hipError_t launch_tree_nl(const TreeArgs& a, const TreeScalarArgs* sa, hipStream_t s) {
    if (sa) return launch_tree_scalar_nl<DT, OP, NL>(*sa, s);
    // as launch_vec_m: streaming calls (>= 64 MiB for trees) nt with one-wave workgroups
    const ReduceTuning& t = reduce_tuning();
    size_t nvec = 0;
    for (int j = 0; j < a.nseg; ++j) nvec += a.seg[j].nvec;
    const size_t call_bytes = (size_t)(a.nl + 1) * nvec * 16;
    const bool nt = t.nt_mode == 1 || (t.nt_mode < 0 && call_bytes >= t.tree_nt_min_bytes);
    if constexpr (is_pair_dt<DT>() || is_complex_dt<DT>()) return launch_tree_vec<DT, OP, NL, 256, false>(a, s);  // as launch_vec_m
    else return nt ? launch_tree_vec<DT, OP, NL, 64, true>(a, s) : launch_tree_vec<DT, OP, NL, 256, false>(a, s);
}

template <int DT, int OP>
inline hipError_t launch_tree_op(const TreeArgs& a, const TreeScalarArgs* sa, hipStream_t s) {
    switch (sa ? sa->nl : a.nl) {
    case 2: return launch_tree_nl<DT, OP, 2>(a, sa, s);
    case 3: return launch_tree_nl<DT, OP, 3>(a, sa, s);
    case 4: return launch_tree_nl<DT, OP, 4>(a, sa, s);
    case 5: return launch_tree_nl<DT, OP, 5>(a, sa, s);
    case 6: return launch_tree_nl<DT, OP, 6>(a, sa, s);
    case 7: return launch_tree_nl<DT, OP, 7>(a, sa, s);
    case 8: return launch_tree_nl<DT, OP, 8>(a, sa, s);
    default: return hipErrorInvalidValue;
    }
}

// The integer kernel types of reduce_tree_int.hip (kdt/kop from canon_op).
hipError_t launch_tree_int(const TreeArgs& a, const TreeScalarArgs* sa, int kdt, int kop, hipStream_t s);
// The pair (MAXLOC / MINLOC) and complex (SUM / PROD) types of reduce_tree_pair.hip.
hipError_t launch_tree_pair(const TreeArgs& a, const TreeScalarArgs* sa, int kdt, int kop, hipStream_t s);


}  // namespace chr
