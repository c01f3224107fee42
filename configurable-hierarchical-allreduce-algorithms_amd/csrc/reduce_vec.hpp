// reduce_vec.hpp -- the fused bucket-reduction kernels (templates), shared by the translation
// units that instantiate them: reduce_kernels.hip (floating types, int32 arithmetic) and
// reduce_int.hip (the other MPI integer types, logical and bitwise ops).  See reduce_kernels.hip
// for the design notes.
#pragma once

#include <hip/hip_runtime.h>

#include "reduce_common.hpp"

namespace chr {

constexpr int kMaxFanIn = 8;

struct VecArgs {
    u32x4* out;
    const u32x4* acc;
    const u32x4* ins[kMaxFanIn];
    size_t nvec;
    uint32_t xrun;   // log2 of the trips per XCD run (xcd_trip); set by the launcher
    uint32_t xfull;  // blocks [0, xfull) are remapped (xcd_full of the grid); set per launch
    uint32_t hand;   // trips each odd XCD hands to the even one below (xcd_trip_w); 0 = none
};

// U vectors (16 B each) per lane per trip; all M+1 operands of the trip are loaded
// before the first add so (M+1)*U*16 bytes per lane are in flight.  NT: non-temporal
// loads and stores (global_load/store_dwordx4 ... nt) for calls that stream far more than
// the caches hold: +15-40 % on HBM-cold buckets.  ACC0: under NT, the FIRST of the U
// accumulator vectors keeps the default policy (in place, a quarter of the write-backs then
// go through the Infinity Cache): per-slot policy sweep
// (profiles/r01/microbench_focus4_slot_policy.txt) +15 % at 1 GiB m=1, +3-5 % for m>=2 with
// 256-thread workgroups; with one-wave workgroups it also gains on the 64 MiB m=1 bucket
// (6 440-6 464 vs 6 041-6 052 GB/s all-nt, profiles/r01/block_ab_bench.txt), so it is used for
// every nt call; making ALL accumulator slots temporal thrashes the cache (-7 %).  Slot 0 is
// peeled so that the two policies are separate instructions (a select between a plain and an nt
// load of one address is merged by LLVM, dropping the nt bit).
//
// One trip per workgroup (grid = trips, no grid-stride loop), trips placed by xcd_trip.  With the
// pinned arguments below this kernel runs within 0.3-1 % of a bare one-trip kernel without any
// bounds check (microbench focus9: C2 shape 0.813-0.821 vs 0.822-0.824); the earlier grid-stride
// form with lazily loaded pointers ran at 0.798-0.802.
//
// Every operand pointer is pinned into SGPRs before the trip's first load (pin_sgpr): left
// to itself the compiler loads the input pointers from the kernel arguments between the
// accumulator and input loads, which puts a second scalar-load round trip (s_waitcnt lgkmcnt)
// in front of half of the trip's loads.  The full/partial decision is per trip (scalar).
template <int DT, int OP, int M, int U, bool NT, bool ACC0, int BL>
__global__ __launch_bounds__(BL) void k_reduce_vec(VecArgs a) {
    u32x4* const out = a.out;
    const u32x4* const accp = a.acc;
    const u32x4* ins[M];
#pragma unroll
    for (int j = 0; j < M; ++j) ins[j] = a.ins[j];
    const size_t nvec = a.nvec;
    const uint32_t xrun = a.xrun, xfull = a.xfull, hand = a.hand;
    pin_sgpr(out, accp, nvec, xrun, xfull);
    pin_sgpr_u32(hand, hand);
#pragma unroll
    for (int j = 0; j < M; ++j) pin_sgpr(ins[j]);
    const size_t trip = xcd_trip_w(blockIdx.x, xfull, xrun, hand);
    if (trip == kIdleTrip) return;
    const size_t base = trip * BL * U + threadIdx.x;
    if ((trip + 1) * BL * U <= nvec) {
        u32x4 acc[U], x[M][U];
        acc[0] = ld<NT && !ACC0>(&accp[base]);
#pragma unroll
        for (int u = 1; u < U; ++u) acc[u] = ld<NT>(&accp[base + (size_t)u * BL]);
#pragma unroll
        for (int j = 0; j < M; ++j)
#pragma unroll
            for (int u = 0; u < U; ++u) x[j][u] = ld<NT>(&ins[j][base + (size_t)u * BL]);
        // Keep every load of the trip ahead of the first add: without this the
        // scheduler interleaves the first add (and its vmcnt(0)) between the loads.
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < M; ++j)
#pragma unroll
            for (int u = 0; u < U; ++u) acc[u] = apply_vec<DT, OP>(x[j][u], acc[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) st<NT>(&out[base + (size_t)u * BL], acc[u]);
    } else {
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * BL;
            if (i >= nvec) break;
            u32x4 acc = accp[i];
#pragma unroll
            for (int j = 0; j < M; ++j) acc = apply_vec<DT, OP>(ins[j][i], acc);
            out[i] = acc;
        }
    }
}

struct ScalarArgs {
    void* out;
    const void* acc;
    const void* ins[kMaxFanIn];
    int m;
    size_t n;
};

// Any alignment (odd sizes / offsets): one element per lane per trip.
template <int DT, int OP>
__global__ __launch_bounds__(kBlock) void k_reduce_scalar(ScalarArgs a) {
    using T = typename DTy<DT>::T;
    T* out = (T*)a.out;
    const T* acc = (const T*)a.acc;
    for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < a.n; i += (size_t)gridDim.x * kBlock) {
        T v = acc[i];
        for (int j = 0; j < a.m; ++j) v = apply<DT, OP>(((const T*)a.ins[j])[i], v);
        out[i] = v;
    }
}

// XCD runs for streaming calls, measured through the product API (profiles/r02/xcd_runs/,
// fraction of 8 TB/s, identity -> 512 KiB runs): m = 3 at 256 MiB 0.854 -> 0.896 (1.25 GiB working
// set) and 0.784 -> 0.795 (10 GiB); m = 7 0.811 -> 0.833 / 0.747 -> 0.751.  m = 1: uncapped, the C2
// bucket measured 0.806 identity, 0.803 at 256 KiB, 0.792 at 512 KiB; under the 12-per-CU cap
// (vec_wg_per_cu) 256 KiB runs win instead, 0.829-0.831 -> 0.833 over three alternating rounds
// (profiles/r02/ab_runs/; microbench focus13: 0.814-0.822 -> 0.828).  m = 2 kept the identity
// until round 5 (below).  Cache-warm (plain) calls keep the identity map too.
//
// Round 5 (profiles/r05/ab_xrun/xrun3.jsonl, 3 alternating rounds, 2 GiB rotation, 16-256 MiB buckets): m = 2
// and m = 3 prefer 256 KiB -- m = 2 against the identity 0.687 vs 0.624 at 16 MiB, 0.735 vs 0.687 at 32, 0.770
// vs 0.746 at 64, 0.914 vs 0.902 at 256; m = 3 against 512 KiB 0.820 vs 0.801 at 32 MiB, 0.865 vs 0.852 at 64,
// ties at 128 / 256 (0.887 / 0.904 vs 0.887 / 0.901).  Wider fan-in keeps 512 KiB (256 not measured there).
template <int M>
constexpr size_t vec_xcd_run_kib() {
    return M <= 3 ? 256 : 512;
}

// Resident workgroups per CU for streaming launches (nt_lds_bytes; 0 = uncapped).  Uncapped, a CU
// holds 32 one-wave workgroups, each with (m+1)*U*1 KiB of loads in flight the moment it starts;
// cap 12 (11 resident, census in nt_lds_bytes) measured best for m <= 3 through the product API
// (profiles/r02/occupancy_cap/, 2 rounds, bench.py C2: 0.815 -> 0.823-0.826; m = 3 at 256 MiB 0.893 ->
// 0.924 with a 1.25 GiB rotation, 0.814 -> 0.830 with 10 GiB; 16 and 10 per CU lose or tie).  Wider
// fan-in takes 12 with U = 1 (vec_u_nt below); m = 2 takes 16 (0.817-0.830 in the microbench), or 12
// beside RCCL (stream_wg_cap).
template <int M>
constexpr int vec_wg_per_cu() {
    return M == 2 ? 16 : 12;
}

// Vectors per lane per trip of streaming launches.  U x cap over m = 1..8 with the product template
// (tools/reduce_microbench focus12/14/15, profiles/r02/occupancy_cap/, 2 rounds each): m = 1 U = 4
// (U = 2 / 8 lose 3-9 %); m = 2 U = 2 with 16 per CU, 0.817-0.830 against U = 4's 0.80-0.817; m = 3
// U = 2 with 12 per CU (U = 1 loses 10 %); m >= 4 U = 1 with 12 per CU.  Within the translation
// reach (rotations <= 2 GiB) U = 1 gains 2-4 % over U = 2 at every measured shape (m = 4 at 128 MiB
// 0.846-0.851 -> 0.859-0.896, m = 5 at 64 MiB 0.812-0.815 -> 0.827-0.852, m = 7 at 256 MiB
// 0.803-0.820 -> 0.843-0.867, m = 8 at 128 MiB 0.807-0.812 -> 0.831-0.840); past it (focus16, 4-16
// GiB rotations) twice the workgroups each touch m + 1 pages for 1 KiB, and U = 1 ties at m = 7 /
// 256 MiB (0.769-0.772 vs 0.762-0.774), wins at m = 4 (0.790-0.798 vs 0.760-0.772) and loses ~4 %
// at m = 7 / 64 MiB (uncapped and at 16 per CU; 12 not measured there).  With U = 1 the ACC0 slot
// is the whole accumulator stream: that is the measured shape.  Cache-warm (plain) launches keep
// U = 4 / 2.
template <int M>
constexpr int vec_u_nt() {
    return M == 1 ? 4 : M <= 3 ? 2 : 1;
}
template <int M, bool NT>
constexpr int vec_u() {
    return NT ? vec_u_nt<M>() : M <= 2 ? 4 : 2;
}
// Complex PROD (C99 Annex G multiplication per element) keeps one vector per lane per trip.
template <int DT, int OP, int M, bool NT>
constexpr int vec_u_dt() {
    return is_complex_dt<DT>() && (OP == CHR_PROD || OP == kProdSw) ? 1 : vec_u<M, NT>();
}

// A grid holds at most 2^31 threads here; larger calls (> 32 GiB per operand at BL = 64, U = 2)
// run as consecutive launches over consecutive pieces.  WEIGHTED: the odd-XCD handover
// (xcd_trip_w) adds 8 x hand workgroups to the grid.
template <int BL, int U, bool WEIGHTED = false, typename L>
inline hipError_t for_each_launch_piece(VecArgs a, L launch) {
    const size_t cap = reduce_tuning().max_launch_vec;
    const size_t max_vec = cap ? cap : ((size_t)1 << 31) / BL * BL * U;
    for (size_t off = 0; off < a.nvec; off += max_vec) {
        VecArgs p = a;
        p.out = a.out + off;
        p.acc = a.acc + off;
        for (int j = 0; j < kMaxFanIn; ++j) p.ins[j] = a.ins[j] ? a.ins[j] + off : nullptr;
        p.nvec = a.nvec - off < max_vec ? a.nvec - off : max_vec;
        const unsigned trips = (unsigned)((p.nvec + (size_t)BL * U - 1) / ((size_t)BL * U));
        p.xfull = xcd_full(trips, p.xrun);
        p.hand = WEIGHTED ? xcd_hand(p.xfull, reduce_tuning().xcd_hand_shift) : 0u;
        launch(p, trips + 8u * p.hand);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// Policy (profiles/r01/block_ab_*, profiles/r05/ab_mid/): calls that stream >= 40 MiB (nt_min_bytes)
// run non-temporal with one-wave workgroups and the first accumulator slot temporal (ACC0); smaller,
// cache-warm calls keep plain accesses and 256-thread workgroups.  Only these two shapes are compiled into
// the library; the design-space variants (other workgroup sizes, all-nt accumulators) live in
// tools/reduce_microbench.hip, which instantiates the kernel templates directly.
template <int DT, int OP, int M, int BL, bool NT, bool ACC0>
inline hipError_t launch_vec_mb_one(VecArgs a, hipStream_t s) {
    constexpr int U = vec_u_dt<DT, OP, M, NT>();
    a.xrun = NT ? xcd_run_shift(vec_xcd_run_kib<M>(), (size_t)BL * U * 16) : 0;
    const unsigned lds = NT ? nt_lds_bytes(reduce_tuning().wg_per_cu_vec, vec_wg_per_cu<M>()) : 0;
    // the odd-XCD handover applies where the kernel streams from HBM (nt launches)
    return for_each_launch_piece<BL, U, NT>(a, [&](const VecArgs& p, unsigned grid) {
        hipLaunchKernelGGL((k_reduce_vec<DT, OP, M, U, NT, ACC0, BL>), dim3(grid), dim3(BL), lds, s, p);
    });
}

template <int DT, int OP, int M>
inline hipError_t launch_vec_m(const VecArgs& a, hipStream_t s) {
    // The pair and complex types (MAXLOC / MINLOC, complex SUM / PROD) are compiled in the plain
    // shape only: a rarely used element type does not buy its own streaming instantiations.
    if constexpr (is_pair_dt<DT>() || is_complex_dt<DT>()) {
        return launch_vec_mb_one<DT, OP, M, 256, false, false>(a, s);
    } else {
        const ReduceTuning& t = reduce_tuning();
        const size_t call_bytes = (size_t)(M + 2) * a.nvec * 16;
        const bool nt = t.nt_mode == 1 || (t.nt_mode < 0 && call_bytes >= t.nt_min_bytes);
        if (nt) return launch_vec_mb_one<DT, OP, M, 64, true, true>(a, s);
        return launch_vec_mb_one<DT, OP, M, 256, false, false>(a, s);
    }
}

template <int DT, int OP>
inline hipError_t launch_vec_op(const VecArgs& a, int m, hipStream_t s) {
    switch (m) {
    case 1: return launch_vec_m<DT, OP, 1>(a, s);
    case 2: return launch_vec_m<DT, OP, 2>(a, s);
    case 3: return launch_vec_m<DT, OP, 3>(a, s);
    case 4: return launch_vec_m<DT, OP, 4>(a, s);
    case 5: return launch_vec_m<DT, OP, 5>(a, s);
    case 6: return launch_vec_m<DT, OP, 6>(a, s);
    case 7: return launch_vec_m<DT, OP, 7>(a, s);
    case 8: return launch_vec_m<DT, OP, 8>(a, s);
    default: return hipErrorInvalidValue;
    }
}

template <int DT, int OP>
inline hipError_t launch_scalar_op(const ScalarArgs& a, hipStream_t s) {
    const size_t trips = (a.n + kBlock - 1) / kBlock;
    const int grid = (int)(trips < 2048 ? trips : 2048);
    hipLaunchKernelGGL((k_reduce_scalar<DT, OP>), dim3(grid), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}


// Launches for the integer kernel types of reduce_int.hip (kdt/kop from canon_op).
hipError_t launch_vec_int(const VecArgs& a, int kdt, int kop, int m, hipStream_t s);
hipError_t launch_scalar_int(const ScalarArgs& a, int kdt, int kop, hipStream_t s);
// The pair (MAXLOC / MINLOC) and complex (SUM / PROD) types of reduce_pair.hip.
hipError_t launch_vec_pair(const VecArgs& a, int kdt, int kop, int m, hipStream_t s);
hipError_t launch_scalar_pair(const ScalarArgs& a, int kdt, int kop, hipStream_t s);

}  // namespace chr
