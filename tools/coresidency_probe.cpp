// coresidency_probe -- does an RCCL transfer kernel get CUs while a streaming reduction is resident?
//
// Inside an overlapped collective (flat schedule) the fused tree evaluation of slice
// t-2 runs on the compute stream while RCCL's send/recv kernel for slice t runs on the transfer
// stream.  RCCL's kernel (rcclGenericKernel on gfx950: 256 threads, 19 744 B of LDS, ~280 VGPRs +
// scratch; read from librccl's code-object metadata, profiles/r03/coresidency/rccl_kernel_resources.txt)
// can start only on a CU with that much room.  This probe reproduces the situation on one GPU:
//   stream A: `launches` batched C4 tree launches (2 trees x 8 leaves x `piece` MiB each, fp32 SUM,
//             the flat schedule's per-slice launch at C4), rotating over distinct leaf sets;
//   stream B: one transfer of `xfer` MiB, either a real RCCL send/recv to self on a 1-rank
//             communicator (--mode rccl: rcclGenericKernel itself) or a copy kernel with RCCL's
//             footprint (--mode mimic: 256 threads, 19 744 B dynamic LDS, ~288 VGPRs).
// Both streams are timed with HIP events; run under `rocprofv3 --kernel-trace` the kernel rows show
// whether the transfer kernel started inside the tree launches' window
// (tools/coresidency_report.py).  Every setting runs alone first (tree only, transfer only), then
// concurrently, `reps` times.  The reduction's occupancy policy is the product's (libchiara), so
// CHR_WG_PER_CU_TREE=0 / unset is the A/B of the LDS cap.
//
//   coresidency_probe [--mode rccl|mimic] [--prio 0|1] [--cumask R] [--piece MiB] [--xfer MiB]
//                     [--launches L] [--reps N] [--nsets S]
//                     [--dtype f32|bf16]  (C4's f32 trees or C5's bf16 ones)  [--leaves 8|4|2]
//   --prio 1:   stream B is created with the highest stream priority
//   --cumask R: stream A runs with R CUs per XCD masked off (hipExtStreamCreateWithCUMask)
//   --delay-us D: in the concurrent runs the transfer is submitted D us after the trees start (both
//             streams wait on one host flag, released once everything is enqueued)
// Built twice: tools/coresidency_probe links ROCm 7.2's RCCL (what the reference's harnesses get
// through the MPI shim); tools/libcoresidency_probe.so is called from Python after `import torch`
// (tools/coresidency_probe.py), so it runs torch's RCCL (what bench.py's N>1 line gets).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "chiara.h"

#define HIPCHECK(x)                                                                                    \
    do {                                                                                               \
        hipError_t e_ = (x);                                                                           \
        if (e_ != hipSuccess) {                                                                        \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
            std::exit(1);                                                                              \
        }                                                                                              \
    } while (0)
#define CHRCHECK(x)                                                                                    \
    do {                                                                                               \
        int r_ = (x);                                                                                  \
        if (r_ != 0) {                                                                                 \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, chr_error_string(r_));      \
            std::exit(1);                                                                              \
        }                                                                                              \
    } while (0)
#define NCCLCHECK(x)                                                                                   \
    do {                                                                                               \
        ncclResult_t r_ = (x);                                                                         \
        if (r_ != ncclSuccess) {                                                                       \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, ncclGetErrorString(r_));    \
            std::exit(1);                                                                              \
        }                                                                                              \
    } while (0)

constexpr unsigned kMimicLds = 19744;  // rcclGenericKernel's group segment on gfx950

// 256 threads, RCCL's LDS, and a register footprint near RCCL's: the asm clobbers force the
// allocation of v0..v255 and a0..a31 (288 per wave), so the kernel needs a wave slot with 288
// VGPRs free on each of the CU's four SIMDs, like rcclGenericKernel (vgpr_count 261-280).
// stamps[blockIdx.x] = the wall clock when this workgroup started (its admission time).
__global__ __launch_bounds__(256) void k_mimic_copy(const float4* __restrict__ src, float4* __restrict__ dst,
                                                    size_t nvec, uint64_t* stamps) {
    extern __shared__ float lds[];
    if (threadIdx.x == 0) {
        lds[0] = 0.f;
        stamps[blockIdx.x] = wall_clock64();
    }
    asm volatile("" ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13",
                 "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27",
                 "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41",
                 "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55",
                 "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69",
                 "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83",
                 "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97",
                 "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109",
                 "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121",
                 "v122", "v123", "v124", "v125", "v126", "v127", "v128", "v129", "v130", "v131", "v132", "v133",
                 "v134", "v135", "v136", "v137", "v138", "v139", "v140", "v141", "v142", "v143", "v144", "v145",
                 "v146", "v147", "v148", "v149", "v150", "v151", "v152", "v153", "v154", "v155", "v156", "v157",
                 "v158", "v159", "v160", "v161", "v162", "v163", "v164", "v165", "v166", "v167", "v168", "v169",
                 "v170", "v171", "v172", "v173", "v174", "v175", "v176", "v177", "v178", "v179", "v180", "v181",
                 "v182", "v183", "v184", "v185", "v186", "v187", "v188", "v189", "v190", "v191", "v192", "v193",
                 "v194", "v195", "v196", "v197", "v198", "v199", "v200", "v201", "v202", "v203", "v204", "v205",
                 "v206", "v207", "v208", "v209", "v210", "v211", "v212", "v213", "v214", "v215", "v216", "v217",
                 "v218", "v219", "v220", "v221", "v222", "v223", "v224", "v225", "v226", "v227", "v228", "v229",
                 "v230", "v231", "v232", "v233", "v234", "v235", "v236", "v237", "v238", "v239", "v240", "v241",
                 "v242", "v243", "v244", "v245", "v246", "v247", "v248", "v249", "v250", "v251", "v252", "v253",
                 "v254", "v255", "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11", "a12",
                 "a13", "a14", "a15", "a16", "a17", "a18", "a19", "a20", "a21", "a22", "a23", "a24", "a25", "a26",
                 "a27", "a28", "a29", "a30", "a31");
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

// Holds stream B for `us` microseconds after the gate opens, so the transfer is submitted while the
// first tree launch is already resident (one 64-thread workgroup; the wall clock runs at `khz`).
__global__ void k_delay(uint64_t us, uint64_t khz, uint64_t* stamp) {
    const uint64_t t0 = wall_clock64(), ticks = us * khz / 1000;
    uint64_t t = t0;
    while ((t = wall_clock64()) - t0 < ticks) __builtin_amdgcn_s_sleep(2);
    if (threadIdx.x == 0) *stamp = t;
}

// Residency census: every workgroup counts itself in on its CU (__smid: XCC, SE, CU), records the
// count it saw, stays `ticks` of the wall clock, and counts itself out; peak[cu] is then the most
// workgroups of this launch resident on that CU at once.
__global__ void k_census(unsigned* cur, unsigned* peak, uint64_t ticks) {
    const unsigned id = __smid() & 4095u;
    if (threadIdx.x == 0) {
        const unsigned old = atomicAdd(&cur[id], 1u);
        atomicMax(&peak[id], old + 1u);
    }
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
    __syncthreads();
    if (threadIdx.x == 0) atomicSub(&cur[id], 1u);
}

// The LDS the product's occupancy cap reserves per workgroup (reduce_common.hpp nt_lds_bytes) for a
// few caps, and the residency each gives to one-wave workgroups.
static void census(int ncu) {
    int lds_cu = 0, lds_blk = 0, khz = 0;
    HIPCHECK(hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, 0));
    HIPCHECK(hipDeviceGetAttribute(&lds_blk, hipDeviceAttributeMaxSharedMemoryPerBlock, 0));
    HIPCHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    unsigned *cur = nullptr, *peak = nullptr;
    HIPCHECK(hipMalloc(&cur, 4096 * sizeof(unsigned)));
    HIPCHECK(hipMalloc(&peak, 4096 * sizeof(unsigned)));
    std::printf("{\"census\": true, \"lds_per_cu_attr\": %d, \"lds_per_block_attr\": %d, \"wall_khz\": %d, \"cus\": %d}\n",
                lds_cu, lds_blk, khz, ncu);
    for (int cap : {0, 8, 10, 11, 12, 13, 14, 16, 20}) {
        const unsigned lds = cap ? ((unsigned)lds_cu / (unsigned)cap) & ~255u : 0u;
        HIPCHECK(hipMemset(cur, 0, 4096 * sizeof(unsigned)));
        HIPCHECK(hipMemset(peak, 0, 4096 * sizeof(unsigned)));
        hipLaunchKernelGGL(k_census, dim3(ncu * 40), dim3(64), lds, 0, cur, peak, (uint64_t)khz * 50 / 1000);
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipDeviceSynchronize());
        std::vector<unsigned> h(4096);
        HIPCHECK(hipMemcpy(h.data(), peak, 4096 * sizeof(unsigned), hipMemcpyDeviceToHost));
        unsigned mx = 0, mn = ~0u, used = 0;
        double sum = 0;
        for (unsigned v : h)
            if (v) {
                ++used;
                mx = v > mx ? v : mx;
                mn = v < mn ? v : mn;
                sum += v;
            }
        std::printf("{\"census\": true, \"cap\": %d, \"dyn_lds\": %u, \"cus_seen\": %u, \"peak_min\": %u, "
                    "\"peak_max\": %u, \"peak_mean\": %.2f}\n",
                    cap, lds, used, mn, mx, used ? sum / used : 0.0);
    }
    HIPCHECK(hipFree(cur));
    HIPCHECK(hipFree(peak));
}

struct Opts {
    std::string mode = "rccl";
    int prio = 0, cumask = 0, launches = 4, reps = 5, nsets = 4, mimic_grid = 64, delay_us = 10, census = 0;
    unsigned mimic_lds = kMimicLds;
    size_t piece_mib = 16, xfer_mib = 56;
    chr_dtype dtype = CHR_FLOAT32;  // --dtype f32|bf16: C4's trees or C5's
    int leaves = 8;                 // --leaves 8|4|2: C4 / C5's trees, or the N = 4 / N = 2 flat schedules
};

extern "C" int probe_main(int argc, char** argv) {
    Opts o;
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string k = argv[i];
        const char* v = argv[i + 1];
        if (k == "--mode") o.mode = v;
        else if (k == "--prio") o.prio = std::atoi(v);
        else if (k == "--cumask") o.cumask = std::atoi(v);
        else if (k == "--piece") o.piece_mib = (size_t)std::atoll(v);
        else if (k == "--xfer") o.xfer_mib = (size_t)std::atoll(v);
        else if (k == "--launches") o.launches = std::atoi(v);
        else if (k == "--reps") o.reps = std::atoi(v);
        else if (k == "--nsets") o.nsets = std::atoi(v);
        else if (k == "--mimic-grid") o.mimic_grid = std::atoi(v);
        else if (k == "--delay-us") o.delay_us = std::atoi(v);
        else if (k == "--census") o.census = std::atoi(v);
        else if (k == "--mimic-lds") o.mimic_lds = (unsigned)std::atoi(v);
        else if (k == "--dtype") o.dtype = std::string(v) == "bf16" ? CHR_BFLOAT16 : CHR_FLOAT32;
        else if (k == "--leaves") o.leaves = std::atoi(v);
        else {
            std::fprintf(stderr, "unknown option %s\n", k.c_str());
            return 2;
        }
    }
    if (o.launches < 1 || o.nsets < 1 || o.reps < 1 || o.piece_mib < 1 || o.xfer_mib < 1 || o.launches > 64) return 2;
    if (o.leaves != 8 && o.leaves != 4 && o.leaves != 2) return 2;
    HIPCHECK(hipSetDevice(0));
    hipDeviceProp_t prop;
    HIPCHECK(hipGetDeviceProperties(&prop, 0));
    const int ncu = prop.multiProcessorCount;
    if (o.census) {
        census(ncu);
        return 0;
    }

    // streams: A = reductions (optionally CU-masked), B = transfers (optionally high priority)
    hipStream_t sA, sB;
    if (o.cumask > 0) {
        // CU mask bits are spread round-robin over the XCDs (bit i -> XCD i % 8): clearing the lowest
        // 8*R bits takes R CUs off every XCD
        std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
        for (int i = 0; i < ncu; ++i)
            if (i >= 8 * o.cumask) mask[i / 32] |= 1u << (i % 32);
        HIPCHECK(hipExtStreamCreateWithCUMask(&sA, (uint32_t)mask.size(), mask.data()));
    } else {
        HIPCHECK(hipStreamCreateWithFlags(&sA, hipStreamNonBlocking));
    }
    if (o.prio) {
        int lo = 0, hi = 0;
        HIPCHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIPCHECK(hipStreamCreateWithPriority(&sB, hipStreamNonBlocking, hi));
    } else {
        HIPCHECK(hipStreamCreateWithFlags(&sB, hipStreamNonBlocking));
    }

    // tree leaf sets: nsets x 2 trees x L leaves + 2 outputs, `piece` MiB each
    const size_t es = o.dtype == CHR_BFLOAT16 ? 2 : 4, n = (o.piece_mib << 20) / es;
    struct Set {
        std::vector<void*> leaves;  // 16 (tree-major)
        void* outs[2];
    };
    std::vector<Set> sets(o.nsets);
    for (int s = 0; s < o.nsets; ++s) {
        sets[s].leaves.resize(2 * o.leaves);
        for (int j = 0; j < 2 * o.leaves; ++j) {
            HIPCHECK(hipMalloc(&sets[s].leaves[j], n * es));
            CHRCHECK(chr_fill(sets[s].leaves[j], n, o.dtype, 0, 7, 16 * s + j, 0, sA));
        }
        for (int t = 0; t < 2; ++t) HIPCHECK(hipMalloc(&sets[s].outs[t], n * es));
    }
    // C4's per-chunk tree ((l0 l1 l2 l3)(l4 l5 l6 l7)), both trees; the 4-rank flat schedule's ((l0 l1)(l2 l3)); 2
    const unsigned char c8[8] = {0, 1, 1, 1, 0, 1, 1, 2}, c4[4] = {0, 1, 0, 2}, c2[2] = {0, 1};
    const unsigned char* comb1 = o.leaves == 8 ? c8 : o.leaves == 4 ? c4 : c2;
    unsigned char comb[16];
    std::memcpy(comb, comb1, o.leaves);
    std::memcpy(comb + o.leaves, comb1, o.leaves);
    auto trees = [&](int launch) {
        Set& st = sets[launch % o.nsets];
        CHRCHECK(chr_reduce_tree_batch(st.outs, (const void* const*)st.leaves.data(), 2, o.leaves, comb, nullptr, n,
                                       o.dtype, CHR_SUM, sA));
    };

    // transfer buffers
    const size_t xb = o.xfer_mib << 20;
    void *xs = nullptr, *xr = nullptr;
    HIPCHECK(hipMalloc(&xs, xb));
    HIPCHECK(hipMalloc(&xr, xb));
    HIPCHECK(hipMemset(xs, 1, xb));
    uint64_t* stamps = nullptr;  // [0]: k_delay's end, [1 + i]: mimic workgroup i's start
    HIPCHECK(hipMalloc(&stamps, (1 + (size_t)o.mimic_grid) * sizeof(uint64_t)));
    ncclComm_t comm = nullptr;
    if (o.mode == "rccl") {
        ncclUniqueId id;
        NCCLCHECK(ncclGetUniqueId(&id));
        NCCLCHECK(ncclCommInitRank(&comm, 1, id, 0));
    } else if (o.mode != "mimic") {
        std::fprintf(stderr, "--mode rccl|mimic\n");
        return 2;
    }
    auto xfer = [&]() {
        if (comm) {
            NCCLCHECK(ncclGroupStart());
            NCCLCHECK(ncclSend(xs, xb, ncclUint8, 0, comm, sB));
            NCCLCHECK(ncclRecv(xr, xb, ncclUint8, 0, comm, sB));
            NCCLCHECK(ncclGroupEnd());
        } else {
            hipLaunchKernelGGL(k_mimic_copy, dim3(o.mimic_grid), dim3(256), o.mimic_lds, sB, (const float4*)xs,
                               (float4*)xr, xb / 16, stamps + 1);
            HIPCHECK(hipGetLastError());
        }
    };

    hipEvent_t a0, a1, b0, b1;
    HIPCHECK(hipEventCreate(&a0));
    HIPCHECK(hipEventCreate(&a1));
    HIPCHECK(hipEventCreate(&b0));
    HIPCHECK(hipEventCreate(&b1));
    auto ms = [](hipEvent_t x, hipEvent_t y) {
        float t = 0;
        HIPCHECK(hipEventElapsedTime(&t, x, y));
        return (double)t;
    };
    int khz = 0;
    HIPCHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    uint32_t* gate = nullptr;  // both streams wait on it, so neither starts before everything is enqueued
    HIPCHECK(hipHostMalloc((void**)&gate, sizeof(uint32_t), hipHostMallocCoherent));
    *gate = 0;
    // warm: every set once, one transfer (RCCL connection setup)
    for (int l = 0; l < o.nsets; ++l) trees(l);
    xfer();
    HIPCHECK(hipDeviceSynchronize());

    const double tree_bytes = 2.0 * (o.leaves + 1.0) * (double)n * (double)es * o.launches;
    std::printf("{\"config\": {\"mode\": \"%s\", \"prio\": %d, \"cumask_per_xcd\": %d, \"piece_mib\": %zu, "
                "\"xfer_mib\": %zu, \"launches\": %d, \"nsets\": %d, \"wg_per_cu_tree_env\": \"%s\", \"cus\": %d, "
                "\"dtype\": \"%s\", \"leaves\": %d}}\n",
                o.mode.c_str(), o.prio, o.cumask, o.piece_mib, o.xfer_mib, o.launches, o.nsets,
                std::getenv("CHR_WG_PER_CU_TREE") ? std::getenv("CHR_WG_PER_CU_TREE") : "policy", ncu,
                o.dtype == CHR_BFLOAT16 ? "bf16" : "f32", o.leaves);
    int launch = 0;
    for (int r = 0; r < o.reps; ++r) {
        // alone: trees, then the transfer
        HIPCHECK(hipEventRecord(a0, sA));
        for (int l = 0; l < o.launches; ++l) trees(launch++);
        HIPCHECK(hipEventRecord(a1, sA));
        HIPCHECK(hipStreamSynchronize(sA));
        const double tree_alone = ms(a0, a1);
        HIPCHECK(hipEventRecord(b0, sB));
        xfer();
        HIPCHECK(hipEventRecord(b1, sB));
        HIPCHECK(hipStreamSynchronize(sB));
        const double xfer_alone = ms(b0, b1);
        // concurrent: both streams wait at the gate; once it opens, stream A runs the trees and
        // stream B submits the transfer `delay_us` later, while the first tree launch is resident
        HIPCHECK(hipDeviceSynchronize());
        __atomic_store_n(gate, 0u, __ATOMIC_SEQ_CST);
        const uint32_t want = 1u + (uint32_t)r;
        HIPCHECK(hipStreamWaitValue32(sA, gate, want, hipStreamWaitValueGte, 0xFFFFFFFFu));
        HIPCHECK(hipStreamWaitValue32(sB, gate, want, hipStreamWaitValueGte, 0xFFFFFFFFu));
        HIPCHECK(hipEventRecord(a0, sA));
        for (int l = 0; l < o.launches; ++l) trees(launch++);
        HIPCHECK(hipEventRecord(a1, sA));
        HIPCHECK(hipEventRecord(b0, sB));
        if (o.delay_us > 0)
            hipLaunchKernelGGL(k_delay, dim3(1), dim3(64), 0, sB, (uint64_t)o.delay_us, (uint64_t)khz, stamps);
        xfer();
        HIPCHECK(hipEventRecord(b1, sB));
        __atomic_store_n(gate, want, __ATOMIC_SEQ_CST);
        HIPCHECK(hipDeviceSynchronize());
        const double tree_conc = ms(a0, a1), xfer_end = ms(a0, b1), xfer_conc = ms(b0, b1);
        // mimic: when its workgroups were admitted, relative to the submission (k_delay's end)
        double adm_first = -1, adm_median = -1, adm_last = -1;
        if (!comm && o.delay_us > 0) {
            std::vector<uint64_t> h(1 + (size_t)o.mimic_grid);
            HIPCHECK(hipMemcpy(h.data(), stamps, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
            std::vector<double> d;
            for (int i = 0; i < o.mimic_grid; ++i) d.push_back(((double)h[1 + i] - (double)h[0]) * 1000.0 / khz);
            std::sort(d.begin(), d.end());
            adm_first = d.front();
            adm_median = d[d.size() / 2];
            adm_last = d.back();
        }
        std::printf("{\"rep\": %d, \"tree_alone_ms\": %.4f, \"xfer_alone_ms\": %.4f, \"tree_concurrent_ms\": %.4f, "
                    "\"xfer_concurrent_ms\": %.4f, \"xfer_end_after_tree_start_ms\": %.4f, "
                    "\"xfer_done_inside_tree_window\": %s, \"tree_alone_frac\": %.4f, \"tree_concurrent_frac\": %.4f, "
                    "\"mimic_admit_us\": [%.2f, %.2f, %.2f]}\n",
                    r, tree_alone, xfer_alone, tree_conc, xfer_conc, xfer_end, xfer_end < tree_conc ? "true" : "false",
                    tree_bytes / (tree_alone * 1e-3) / 8e12, tree_bytes / (tree_conc * 1e-3) / 8e12, adm_first,
                    adm_median, adm_last);
        std::fflush(stdout);
    }
    if (comm) NCCLCHECK(ncclCommDestroy(comm));
    for (auto& st : sets) {
        for (void* p : st.leaves) HIPCHECK(hipFree(p));
        for (void* p : st.outs) HIPCHECK(hipFree(p));
    }
    HIPCHECK(hipFree(xs));
    HIPCHECK(hipFree(xr));
    HIPCHECK(hipHostFree(gate));
    HIPCHECK(hipFree(stamps));
    HIPCHECK(hipStreamDestroy(sA));
    HIPCHECK(hipStreamDestroy(sB));
    return 0;
}

#ifdef PROBE_EXE
int main(int argc, char** argv) { return probe_main(argc, argv); }
#endif
