// reduce_microbench.hip -- design-space sweep for the fused bucket reduction on gfx950.
// Not part of the product: each variant here is a candidate for csrc/reduce_kernels.hip.
//   hipcc -O3 --offload-arch=gfx950 -o reduce_microbench reduce_microbench.hip
//   ./reduce_microbench [bucket_MiB ...]
// Output: one line per (variant, m, bucket): us per launch and algorithmic GB/s
// ((m+2) x bucket bytes per launch), buffers rotated so the working set exceeds the
// 256 MiB Infinity Cache.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdio>

#include "chiara.h"
#include "../configurable-hierarchical-allreduce-algorithms_amd/csrc/reduce_vec.hpp"
#include "../configurable-hierarchical-allreduce-algorithms_amd/csrc/reduce_tree.hpp"
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct Args {
    f32x4* out;
    const f32x4* acc;
    const f32x4* ins[8];
    size_t nvec;
};

template <int M, int U, int BLOCK, bool NTL, bool NTS, bool NTA = NTL>
__global__ __launch_bounds__(BLOCK) void k_reg(Args a) {
    const size_t stride = (size_t)gridDim.x * BLOCK * U;
    for (size_t base = (size_t)blockIdx.x * BLOCK * U + threadIdx.x; base < a.nvec; base += stride) {
        if (base + (size_t)(U - 1) * BLOCK < a.nvec) {
            f32x4 acc[U], x[M][U];
#pragma unroll
            for (int u = 0; u < U; ++u)
                acc[u] = NTA ? __builtin_nontemporal_load(&a.acc[base + (size_t)u * BLOCK]) : a.acc[base + (size_t)u * BLOCK];
#pragma unroll
            for (int j = 0; j < M; ++j)
#pragma unroll
                for (int u = 0; u < U; ++u)
                    x[j][u] = NTL ? __builtin_nontemporal_load(&a.ins[j][base + (size_t)u * BLOCK])
                                  : a.ins[j][base + (size_t)u * BLOCK];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < M; ++j)
#pragma unroll
                for (int u = 0; u < U; ++u) acc[u] = x[j][u] + acc[u];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (NTS)
                    __builtin_nontemporal_store(acc[u], &a.out[base + (size_t)u * BLOCK]);
                else
                    a.out[base + (size_t)u * BLOCK] = acc[u];
            }
        } else {
            for (int u = 0; u < U; ++u) {
                const size_t i = base + (size_t)u * BLOCK;
                if (i >= a.nvec) break;
                f32x4 v = a.acc[i];
                for (int j = 0; j < M; ++j) v = a.ins[j][i] + v;
                a.out[i] = v;
            }
        }
    }
}

// Contiguous-chunk-per-block form: block b owns [b*CH, (b+1)*CH) vectors.
template <int M, int U, int BLOCK, bool NT = false>
__global__ __launch_bounds__(BLOCK) void k_chunk(Args a, size_t chunk) {
    const size_t lo = (size_t)blockIdx.x * chunk;
    size_t hi = lo + chunk;
    if (hi > a.nvec) hi = a.nvec;
    for (size_t base = lo + threadIdx.x; base < hi; base += (size_t)BLOCK * U) {
        if (base + (size_t)(U - 1) * BLOCK < hi) {
            f32x4 acc[U], x[M][U];
#pragma unroll
            for (int u = 0; u < U; ++u)
                acc[u] = NT ? __builtin_nontemporal_load(&a.acc[base + (size_t)u * BLOCK]) : a.acc[base + (size_t)u * BLOCK];
#pragma unroll
            for (int j = 0; j < M; ++j)
#pragma unroll
                for (int u = 0; u < U; ++u)
                    x[j][u] = NT ? __builtin_nontemporal_load(&a.ins[j][base + (size_t)u * BLOCK]) : a.ins[j][base + (size_t)u * BLOCK];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < M; ++j)
#pragma unroll
                for (int u = 0; u < U; ++u) acc[u] = x[j][u] + acc[u];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (NT) __builtin_nontemporal_store(acc[u], &a.out[base + (size_t)u * BLOCK]);
                else a.out[base + (size_t)u * BLOCK] = acc[u];
            }
        } else {
            for (int u = 0; u < U; ++u) {
                const size_t i = base + (size_t)u * BLOCK;
                if (i >= hi) break;
                f32x4 v = a.acc[i];
                for (int j = 0; j < M; ++j) v = a.ins[j][i] + v;
                a.out[i] = v;
            }
        }
    }
}

// LDS-DMA staging: every operand tile goes global -> LDS by global_load_lds_dwordx4
// (1 KiB per wave-instruction), double-buffered, then ds_read_b128 -> add -> store.
// Each lane reads back exactly the 16 B its own DMA wrote, so only the wave's own
// vmcnt orders the read (no workgroup barrier).
template <int M, int U>
__global__ __launch_bounds__(256) void k_lds(Args a) {
    constexpr int OPS = M + 1;
    constexpr int TILE = U * 64;                       // vectors per wave per operand
    __shared__ __attribute__((aligned(16))) f32x4 lds[2][4][OPS][TILE];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const size_t per_block = (size_t)256 * U;
    const size_t ntiles = a.nvec / per_block;           // full tiles only (tail below)
    auto issue = [&](size_t t, int buf) {
        const size_t base = t * per_block + (size_t)wave * TILE;
#pragma unroll
        for (int o = 0; o < OPS; ++o) {
            const f32x4* src = o == 0 ? a.acc : a.ins[o - 1];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)(src + base + u * 64 + lane),
                    (__attribute__((address_space(3))) void*)&lds[buf][wave][o][u * 64], 16, 0, 0);
            }
        }
    };
    size_t t = blockIdx.x;
    int buf = 0;
    if (t < ntiles) issue(t, 0);
    for (; t < ntiles; t += gridDim.x) {
        const size_t tn = t + gridDim.x;
        if (tn < ntiles) {
            issue(tn, buf ^ 1);
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OPS * U) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const size_t base = t * per_block + (size_t)wave * TILE;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            f32x4 v = lds[buf][wave][0][u * 64 + lane];
#pragma unroll
            for (int j = 1; j < OPS; ++j) v = lds[buf][wave][j][u * 64 + lane] + v;
            a.out[base + u * 64 + lane] = v;
        }
        buf ^= 1;
    }
    if (blockIdx.x == 0) {  // tail vectors
        for (size_t i = ntiles * per_block + threadIdx.x; i < a.nvec; i += 256) {
            f32x4 v = a.acc[i];
            for (int j = 0; j < M; ++j) v = a.ins[j][i] + v;
            a.out[i] = v;
        }
    }
}

__global__ __launch_bounds__(256) void k_copy(f32x4* out, const f32x4* in, size_t nvec) {
    for (size_t i = (size_t)blockIdx.x * 1024 + threadIdx.x; i < nvec; i += (size_t)gridDim.x * 1024) {
        f32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i + u * 256 < nvec) v[u] = in[i + u * 256];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i + u * 256 < nvec) out[i + u * 256] = v[u];
    }
}

// Random fp32 in [-1,1): benchmarking on zero-filled buffers reads high (DVFS / bus energy).
__global__ void k_rand(f32x4* p, size_t nvec, unsigned long long seed) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (size_t)gridDim.x * 256) {
        f32x4 v;
        for (int c = 0; c < 4; ++c) {
            unsigned long long x = seed ^ (i * 4 + c) * 0x9E3779B97F4A7C15ull;
            x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
            x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
            x ^= x >> 31;
            v[c] = (float)(x >> 40) * (1.0f / 8388608.0f) - 1.0f;
        }
        p[i] = v;
    }
}

struct Sets {
    std::vector<std::vector<f32x4*>> bufs;  // [set][operand]
};

static Sets make_sets(int m, size_t nvec, int sets) {
    Sets s;
    s.bufs.resize(sets);
    for (int i = 0; i < sets; ++i)
        for (int j = 0; j < m + 1; ++j) {
            f32x4* p;
            CK(hipMalloc(&p, nvec * 16));
            hipLaunchKernelGGL(k_rand, dim3(4096), dim3(256), 0, 0, p, nvec, 0x1234567ull * (i * 16 + j + 1));
            s.bufs[i].push_back(p);
        }
    return s;
}
static void free_sets(Sets& s) {
    for (auto& v : s.bufs)
        for (auto* p : v) CK(hipFree(p));
}

template <typename L>
static double time_launches(L launch, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 5; ++i) launch(i);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) launch(i);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return ms * 1e3 / reps;  // us
}

static void report(const char* name, int m, size_t bytes, double us) {
    const double gbps = (m + 2) * (double)bytes / (us * 1e-6) / 1e9;
    std::printf("%-34s m=%d bucket=%6zu MiB  %9.2f us  %8.1f GB/s  %.3f of 8 TB/s\n", name, m, bytes >> 20, us, gbps,
                gbps / 8000.0);
    std::fflush(stdout);
}

template <int M>
static void run_m(size_t bytes) {
    const size_t nvec = bytes / 16;
    const int sets = std::max(1, std::min(8, (int)((1024ull << 20) / ((M + 2) * bytes))));
    Sets S = make_sets(M, nvec, sets);
    const int reps = std::max(10, std::min(300, (int)((8ull << 30) / ((M + 2) * bytes))));
    auto args_for = [&](int i) {
        Args a{};
        auto& b = S.bufs[i % sets];
        a.out = b[0];
        a.acc = b[0];
        for (int j = 0; j < M; ++j) a.ins[j] = b[j + 1];
        a.nvec = nvec;
        return a;
    };
#define REG(U, BL, GRIDCAP, NTL, NTS, NAME)                                                              \
    {                                                                                                  \
        const size_t trips = (nvec + (size_t)BL * U - 1) / ((size_t)BL * U);                          \
        const int grid = (int)std::min<size_t>(trips, GRIDCAP);                                        \
        double us = time_launches([&](int i) { hipLaunchKernelGGL((k_reg<M, U, BL, NTL, NTS>), dim3(grid), dim3(BL), 0, 0, args_for(i)); }, reps); \
        report(NAME, M, bytes, us);                                                                    \
    }
    REG(4, 256, 2048, false, false, "reg U4 B256 cap2048 (product)");
    REG(4, 256, 1 << 30, false, false, "reg U4 B256 full-grid");
    REG(4, 256, 1024, false, false, "reg U4 B256 cap1024");
    REG(4, 256, 4096, false, false, "reg U4 B256 cap4096");
    REG(2, 256, 1 << 30, false, false, "reg U2 B256 full-grid");
    REG(8, 256, 1 << 30, false, false, "reg U8 B256 full-grid");
    REG(8, 256, 2048, false, false, "reg U8 B256 cap2048");
    REG(1, 256, 1 << 30, false, false, "reg U1 B256 full-grid");
    REG(4, 512, 1 << 30, false, false, "reg U4 B512 full-grid");
    REG(2, 1024, 1 << 30, false, false, "reg U2 B1024 full-grid");
    REG(4, 256, 1 << 30, true, false, "reg U4 full-grid NT-load");
    REG(4, 256, 1 << 30, false, true, "reg U4 full-grid NT-store");
    REG(4, 256, 1 << 30, true, true, "reg U4 full-grid NT-load+store");
    REG(4, 256, 2048, true, true, "reg U4 cap2048 NT-load+store");
#undef REG
    for (size_t blocks : {256ul, 512ul, 1024ul, 2048ul}) {
        const size_t chunk = (nvec + blocks - 1) / blocks;
        double us = time_launches([&](int i) { hipLaunchKernelGGL((k_chunk<M, 4, 256>), dim3(blocks), dim3(256), 0, 0, args_for(i), chunk); }, reps);
        char name[64];
        std::snprintf(name, sizeof name, "chunk U4 B256 blocks=%zu", blocks);
        report(name, M, bytes, us);
    }
    if (M <= 3) {
        for (int cap : {512, 1024, 2048}) {
            const size_t trips = nvec / (256 * 2);
            const int grid = (int)std::min<size_t>(std::max<size_t>(trips, 1), cap);
            double us = time_launches([&](int i) { hipLaunchKernelGGL((k_lds<M, 2>), dim3(grid), dim3(256), 0, 0, args_for(i)); }, reps);
            char name[64];
            std::snprintf(name, sizeof name, "LDS-DMA U2 dbuf cap%d", cap);
            report(name, M, bytes, us);
        }
    }
    if (M == 1) {
        double us = time_launches([&](int i) {
            auto& b = S.bufs[i % sets];
            hipLaunchKernelGGL(k_copy, dim3(2048), dim3(256), 0, 0, b[0], b[1], nvec);
        }, reps);
        const double gbps = 2.0 * bytes / (us * 1e-6) / 1e9;
        std::printf("%-34s      bucket=%6zu MiB  %9.2f us  %8.1f GB/s  (copy: 2 x bytes)\n", "float4 copy (ceiling ref)",
                    bytes >> 20, us, gbps);
    }
    free_sets(S);
}


template <int M>
static void focus_m(size_t bytes, int sets_override, int rounds) {
    const size_t nvec = bytes / 16;
    const int sets = sets_override > 0 ? sets_override : std::max(1, std::min(8, (int)((1024ull << 20) / ((M + 2) * bytes))));
    Sets S = make_sets(M, nvec, sets);
    const int reps = std::max(10, std::min(300, (int)((8ull << 30) / ((M + 2) * bytes))));
    auto args_for = [&](int i) {
        Args a{};
        auto& b = S.bufs[i % sets];
        a.out = b[0];
        a.acc = b[0];
        for (int j = 0; j < M; ++j) a.ins[j] = b[j + 1];
        a.nvec = nvec;
        return a;
    };
    char tag[64];
    std::snprintf(tag, sizeof tag, " sets=%d", sets);
    for (int r = 0; r < rounds; ++r) {
#define F(U, CAP, NTL, NTS, NTA, NAME)                                                              \
    {                                                                                                  \
        const size_t trips = (nvec + (size_t)256 * U - 1) / ((size_t)256 * U);                          \
        const int grid = (int)std::min<size_t>(trips, CAP);                                            \
        double us = time_launches([&](int i) { hipLaunchKernelGGL((k_reg<M, U, 256, NTL, NTS, NTA>), dim3(grid), dim3(256), 0, 0, args_for(i)); }, reps); \
        report((std::string(NAME) + tag).c_str(), M, bytes, us);                                                                    \
    }
        F(4, 2048, false, false, false, "plain U4 cap2048 (product)");
        F(1, 1 << 30, false, false, false, "plain U1 full");
        F(4, 1 << 30, true, false, false, "ntIN U4 full");
        F(4, 1 << 30, true, false, true, "ntIN+ACC U4 full");
        F(4, 1 << 30, true, true, false, "ntIN+ST U4 full");
        F(4, 1 << 30, true, true, true, "ntIN+ACC+ST U4 full");
        F(2, 1 << 30, true, false, true, "ntIN+ACC U2 full");
        F(2, 1 << 30, true, true, true, "ntIN+ACC+ST U2 full");
        F(1, 1 << 30, true, false, true, "ntIN+ACC U1 full");
        F(1, 1 << 30, true, true, true, "ntIN+ACC+ST U1 full");
        F(8, 1 << 30, true, false, true, "ntIN+ACC U8 full");
        F(4, 2048, true, false, true, "ntIN+ACC U4 cap2048");
        F(4, 2048, true, true, true, "ntIN+ACC+ST U4 cap2048");
        F(4, 4096, true, false, true, "ntIN+ACC U4 cap4096");
#undef F
        std::printf("--\n");
    }
    free_sets(S);
}


template <int M>
static void focus2_m(size_t bytes, int sets, int rounds) {
    const size_t nvec = bytes / 16;
    Sets S = make_sets(M, nvec, sets);
    const int reps = std::max(10, std::min(300, (int)((8ull << 30) / ((M + 2) * bytes))));
    auto args_for = [&](int i) {
        Args a{};
        auto& b = S.bufs[i % sets];
        a.out = b[0];
        a.acc = b[0];
        for (int j = 0; j < M; ++j) a.ins[j] = b[j + 1];
        a.nvec = nvec;
        return a;
    };
    char tag[64];
    std::snprintf(tag, sizeof tag, " sets=%d", sets);
    for (int r = 0; r < rounds; ++r) {
#define F(U, BL, CAP, NAME)                                                                             \
    {                                                                                                  \
        const size_t trips = (nvec + (size_t)BL * U - 1) / ((size_t)BL * U);                          \
        const int grid = (int)std::min<size_t>(trips, CAP);                                            \
        double us = time_launches([&](int i) { hipLaunchKernelGGL((k_reg<M, U, BL, true, true, true>), dim3(grid), dim3(BL), 0, 0, args_for(i)); }, reps); \
        report((std::string(NAME) + tag).c_str(), M, bytes, us);                                      \
    }
        F(4, 256, 1 << 30, "NT U4 B256 full (shipped)");
        {
            double us = time_launches([&](int i) {
                Args a = args_for(i);
                const void* ins[8];
                for (int j = 0; j < M; ++j) ins[j] = a.ins[j];
                chr_reduce_multi(a.out, a.acc, ins, M, a.nvec * 4, CHR_FLOAT32, CHR_SUM, 0);
            }, reps);
            report((std::string("libchiara chr_reduce_multi") + tag).c_str(), M, bytes, us);
        }
        F(8, 256, 1 << 30, "NT U8 B256 full");
        F(16, 256, 1 << 30, "NT U16 B256 full");
        F(4, 512, 1 << 30, "NT U4 B512 full");
        F(2, 1024, 1 << 30, "NT U2 B1024 full");
        F(4, 1024, 1 << 30, "NT U4 B1024 full");
        F(8, 256, 2048, "NT U8 B256 cap2048");
        F(4, 256, 8192, "NT U4 B256 cap8192");
#undef F
        for (size_t blocks : {1024ul, 2048ul, 4096ul}) {
            const size_t chunk = (nvec + blocks - 1) / blocks;
            double us = time_launches([&](int i) { hipLaunchKernelGGL((k_chunk<M, 4, 256, true>), dim3(blocks), dim3(256), 0, 0, args_for(i), chunk); }, reps);
            char name[64];
            std::snprintf(name, sizeof name, "NT chunk U4 blocks=%zu%s", blocks, tag);
            report(name, M, bytes, us);
        }
        std::printf("--\n");
    }
    free_sets(S);
}


// Per-slot cache policy: bit u of PA / PI / PS set = the acc load / every input load /
// the store of unroll slot u is PLAIN (temporal); clear = non-temporal.
template <int M, int U, int PA, int PI, int PS>
__global__ __launch_bounds__(256) void k_mask(Args a) {
    const size_t stride = (size_t)gridDim.x * 256 * U;
    for (size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x; base < a.nvec; base += stride) {
        if (base + (size_t)(U - 1) * 256 < a.nvec) {
            f32x4 acc[U], x[M][U];
#pragma unroll
            for (int u = 0; u < U; ++u)
                acc[u] = ((PA >> u) & 1) ? a.acc[base + (size_t)u * 256] : __builtin_nontemporal_load(&a.acc[base + (size_t)u * 256]);
#pragma unroll
            for (int j = 0; j < M; ++j)
#pragma unroll
                for (int u = 0; u < U; ++u)
                    x[j][u] = ((PI >> u) & 1) ? a.ins[j][base + (size_t)u * 256] : __builtin_nontemporal_load(&a.ins[j][base + (size_t)u * 256]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < M; ++j)
#pragma unroll
                for (int u = 0; u < U; ++u) acc[u] = x[j][u] + acc[u];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if ((PS >> u) & 1) a.out[base + (size_t)u * 256] = acc[u];
                else __builtin_nontemporal_store(acc[u], &a.out[base + (size_t)u * 256]);
            }
        } else {
            for (int u = 0; u < U; ++u) {
                const size_t i = base + (size_t)u * 256;
                if (i >= a.nvec) break;
                f32x4 v = __builtin_nontemporal_load(&a.acc[i]);
                for (int j = 0; j < M; ++j) v = __builtin_nontemporal_load(&a.ins[j][i]) + v;
                __builtin_nontemporal_store(v, &a.out[i]);
            }
        }
    }
}

template <int M>
static void focus3_m(size_t bytes, int sets, int rounds) {
    const size_t nvec = bytes / 16;
    Sets S = make_sets(M, nvec, sets);
    const int reps = std::max(10, std::min(300, (int)((8ull << 30) / ((M + 2) * bytes))));
    auto args_for = [&](int i) {
        Args a{};
        auto& b = S.bufs[i % sets];
        a.out = b[0];
        a.acc = b[0];
        for (int j = 0; j < M; ++j) a.ins[j] = b[j + 1];
        a.nvec = nvec;
        return a;
    };
    char tag[64];
    std::snprintf(tag, sizeof tag, " sets=%d", sets);
    for (int r = 0; r < rounds; ++r) {
#define F(U, PA, PI, PS, NAME)                                                                          \
    {                                                                                                  \
        const int grid = (int)((nvec + (size_t)256 * U - 1) / ((size_t)256 * U));                      \
        double us = time_launches([&](int i) { hipLaunchKernelGGL((k_mask<M, U, PA, PI, PS>), dim3(grid), dim3(256), 0, 0, args_for(i)); }, reps); \
        report((std::string(NAME) + tag).c_str(), M, bytes, us);                                      \
    }
        F(4, 0, 0, 0, "mask all-NT (product)");
        F(4, 1, 0, 0, "mask acc0 plain");
        F(4, 3, 0, 0, "mask acc0,1 plain");
        F(4, 5, 0, 0, "mask acc0,2 plain");
        F(4, 15, 0, 0, "mask acc all plain");
        F(4, 0, 1, 0, "mask in0 plain");
        F(4, 1, 1, 0, "mask acc0+in0 plain");
        F(4, 0, 0, 1, "mask st0 plain");
        F(4, 1, 0, 1, "mask acc0+st0 plain");
        F(2, 1, 0, 0, "U2 mask acc0 plain");
        F(8, 1, 0, 0, "U8 mask acc0 plain");
        F(8, 17, 0, 0, "U8 mask acc0,4 plain");
#undef F
        {
            double us = time_launches([&](int i) { hipLaunchKernelGGL((k_reg<M, 4, 256, true, true, true>), dim3((nvec + 1023) / 1024), dim3(256), 0, 0, args_for(i)); }, reps);
            report((std::string("k_reg NT (hoisted acc0)") + tag).c_str(), M, bytes, us);
        }
        std::printf("--\n");
    }
    free_sets(S);
}


typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
template <int AUX>
__device__ __forceinline__ u32x4v bload(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX);
}
template <int AUX>
__device__ __forceinline__ void bstore(u32x4v v, __amdgpu_buffer_rsrc_t r, unsigned off) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, AUX);
}
// Buffer-load form with an explicit cache policy per slot: aux 2 = nt, 0 = default.
// Bit u of PA / PI / PS = slot u's acc load / input loads / store use the DEFAULT policy.
template <int M, int U, int PA, int PI, int PS>
__global__ __launch_bounds__(256) void k_buf(Args a) {
    const __amdgpu_buffer_rsrc_t racc = __builtin_amdgcn_make_buffer_rsrc((void*)a.acc, 0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc((void*)a.out, 0, 0x7FFFFFFF, 0x00020000);
    __amdgpu_buffer_rsrc_t rin[M];
#pragma unroll
    for (int j = 0; j < M; ++j) rin[j] = __builtin_amdgcn_make_buffer_rsrc((void*)a.ins[j], 0, 0x7FFFFFFF, 0x00020000);
    const size_t stride = (size_t)gridDim.x * 256 * U;
    for (size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x; base < a.nvec; base += stride) {
        if (base + (size_t)(U - 1) * 256 < a.nvec) {
            u32x4v acc[U], x[M][U];
#pragma unroll
            for (int u = 0; u < U; ++u)
                acc[u] = ((PA >> u) & 1) ? bload<0>(racc, (unsigned)((base + u * 256) * 16)) : bload<2>(racc, (unsigned)((base + u * 256) * 16));
#pragma unroll
            for (int j = 0; j < M; ++j)
#pragma unroll
                for (int u = 0; u < U; ++u)
                    x[j][u] = ((PI >> u) & 1) ? bload<0>(rin[j], (unsigned)((base + u * 256) * 16)) : bload<2>(rin[j], (unsigned)((base + u * 256) * 16));
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < M; ++j)
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    f32x4 p, q;
                    __builtin_memcpy(&p, &x[j][u], 16);
                    __builtin_memcpy(&q, &acc[u], 16);
                    q = p + q;
                    __builtin_memcpy(&acc[u], &q, 16);
                }
#pragma unroll
            for (int u = 0; u < U; ++u)
                if ((PS >> u) & 1) bstore<0>(acc[u], rout, (unsigned)((base + u * 256) * 16));
                else bstore<2>(acc[u], rout, (unsigned)((base + u * 256) * 16));
        } else {
            for (int u = 0; u < U; ++u) {
                const size_t i = base + (size_t)u * 256;
                if (i >= a.nvec) break;
                f32x4 v = a.acc[i];
                for (int j = 0; j < M; ++j) v = a.ins[j][i] + v;
                a.out[i] = v;
            }
        }
    }
}

template <int M>
static void focus4_m(size_t bytes, int sets, int rounds) {
    const size_t nvec = bytes / 16;
    Sets S = make_sets(M, nvec, sets);
    const int reps = std::max(10, std::min(300, (int)((8ull << 30) / ((M + 2) * bytes))));
    auto args_for = [&](int i) {
        Args a{};
        auto& b = S.bufs[i % sets];
        a.out = b[0];
        a.acc = b[0];
        for (int j = 0; j < M; ++j) a.ins[j] = b[j + 1];
        a.nvec = nvec;
        return a;
    };
    char tag[64];
    std::snprintf(tag, sizeof tag, " sets=%d", sets);
    for (int r = 0; r < rounds; ++r) {
#define F(U, PA, PI, PS, NAME)                                                                          \
    {                                                                                                  \
        const int grid = (int)((nvec + (size_t)256 * U - 1) / ((size_t)256 * U));                      \
        double us = time_launches([&](int i) { hipLaunchKernelGGL((k_buf<M, U, PA, PI, PS>), dim3(grid), dim3(256), 0, 0, args_for(i)); }, reps); \
        report((std::string(NAME) + tag).c_str(), M, bytes, us);                                      \
    }
        F(4, 0, 0, 0, "buf all-nt U4");
        F(4, 1, 0, 0, "buf acc0 dflt U4");
        F(4, 3, 0, 0, "buf acc0,1 dflt U4");
        F(4, 15, 0, 0, "buf acc* dflt U4");
        F(4, 0, 1, 0, "buf in0 dflt U4");
        F(4, 0, 0, 1, "buf st0 dflt U4");
        F(4, 1, 1, 0, "buf acc0+in0 dflt U4");
        F(4, 15, 15, 15, "buf all dflt U4");
        F(2, 0, 0, 0, "buf all-nt U2");
        F(2, 1, 0, 0, "buf acc0 dflt U2");
        F(8, 1, 0, 0, "buf acc0 dflt U8");
        F(8, 0, 0, 0, "buf all-nt U8");
#undef F
        {
            double us = time_launches([&](int i) { hipLaunchKernelGGL((k_reg<M, 4, 256, true, true, true>), dim3((nvec + 1023) / 1024), dim3(256), 0, 0, args_for(i)); }, reps);
            report((std::string("k_reg NT (hoisted acc0 plain)") + tag).c_str(), M, bytes, us);
        }
        {
            double us = time_launches([&](int i) {
                Args a = args_for(i);
                const void* ins[8];
                for (int j = 0; j < M; ++j) ins[j] = a.ins[j];
                chr_reduce_multi(a.out, a.acc, ins, M, a.nvec * 4, CHR_FLOAT32, CHR_SUM, 0);
            }, reps);
            report((std::string("libchiara chr_reduce_multi") + tag).c_str(), M, bytes, us);
        }
        std::printf("--\n");
    }
    free_sets(S);
}

// ---- focus5: m = 1 streaming variants not covered above (all nt loads + nt stores) ----------
// k_pipe: persistent grid, software pipelined: the loads of trip t+1 are issued before trip t's
// add and store, so reads and writes of neighbouring trips overlap inside each wave.
template <int U, int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_pipe(Args a) {
    const size_t stride = (size_t)gridDim.x * BLOCK * U;
    size_t base = (size_t)blockIdx.x * BLOCK * U + threadIdx.x;
    if (base + (size_t)(U - 1) * BLOCK >= a.nvec) return;  // focus5 sizes are whole trips
    f32x4 acc[U], x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        acc[u] = __builtin_nontemporal_load(&a.acc[base + (size_t)u * BLOCK]);
        x[u] = __builtin_nontemporal_load(&a.ins[0][base + (size_t)u * BLOCK]);
    }
    for (;;) {
        const size_t next = base + stride;
        const bool more = next + (size_t)(U - 1) * BLOCK < a.nvec;
        f32x4 acc2[U], x2[U];
        if (more) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                acc2[u] = __builtin_nontemporal_load(&a.acc[next + (size_t)u * BLOCK]);
                x2[u] = __builtin_nontemporal_load(&a.ins[0][next + (size_t)u * BLOCK]);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) __builtin_nontemporal_store(x[u] + acc[u], &a.out[base + (size_t)u * BLOCK]);
        if (!more) break;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            acc[u] = acc2[u];
            x[u] = x2[u];
        }
        base = next;
    }
}

// k_map: one trip per workgroup, nt, with the workgroup -> address mapping varied.
//   MAP 0: identity;  1: XCD-contiguous (workgroups dispatch round-robin over the 8 XCDs, so
//   b -> (b % 8) * (G / 8) + b / 8 gives each XCD one contiguous eighth of the bucket);
//   2: reversed;  3: input loaded before the accumulator.
template <int U, int MAP>
__global__ __launch_bounds__(256) void k_map(Args a) {
    const unsigned G = gridDim.x, b = blockIdx.x;
    const unsigned bb = MAP == 1 ? (b % 8) * (G / 8) + b / 8 : MAP == 2 ? G - 1 - b : b;
    const size_t base = (size_t)bb * 256 * U + threadIdx.x;
    f32x4 acc[U], x[U];
    if (MAP == 3) {
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = __builtin_nontemporal_load(&a.ins[0][base + (size_t)u * 256]);
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] = __builtin_nontemporal_load(&a.acc[base + (size_t)u * 256]);
    } else {
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] = __builtin_nontemporal_load(&a.acc[base + (size_t)u * 256]);
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = __builtin_nontemporal_load(&a.ins[0][base + (size_t)u * 256]);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(x[u] + acc[u], &a.out[base + (size_t)u * 256]);
}

static void focus5(size_t bytes, int sets, int rounds) {
    const size_t nvec = bytes / 16;
    Sets S = make_sets(1, nvec, sets);
    const int reps = 200;
    auto args_for = [&](int i) {
        Args a{};
        auto& b = S.bufs[i % sets];
        a.out = b[0];
        a.acc = b[0];
        a.ins[0] = b[1];
        a.nvec = nvec;
        return a;
    };
    char tag[64];
    std::snprintf(tag, sizeof tag, " sets=%d", sets);
    auto product = [&]() {
        double us = time_launches([&](int i) {
            Args a = args_for(i);
            const void* ins[1] = {a.ins[0]};
            chr_reduce_multi(a.out, a.acc, ins, 1, a.nvec * 4, CHR_FLOAT32, CHR_SUM, 0);
        }, reps);
        report((std::string("libchiara chr_reduce_multi") + tag).c_str(), 1, bytes, us);
    };
    for (int r = 0; r < rounds; ++r) {
        product();
#define P(U, BL, G, NAME)                                                                                     \
    {                                                                                                         \
        double us = time_launches([&](int i) { hipLaunchKernelGGL((k_pipe<U, BL>), dim3(G), dim3(BL), 0, 0, args_for(i)); }, reps); \
        report((std::string(NAME) + tag).c_str(), 1, bytes, us);                                              \
    }
        P(4, 256, 256, "pipe U4 B256 G256");
        P(4, 256, 512, "pipe U4 B256 G512");
        P(4, 256, 1024, "pipe U4 B256 G1024");
        P(2, 256, 1024, "pipe U2 B256 G1024");
        P(2, 256, 2048, "pipe U2 B256 G2048");
        P(4, 512, 512, "pipe U4 B512 G512");
        P(2, 1024, 512, "pipe U2 B1024 G512");
#undef P
#define M_(U, MAP, NAME)                                                                                      \
    {                                                                                                         \
        const int G = (int)(nvec / (256 * U));                                                                \
        double us = time_launches([&](int i) { hipLaunchKernelGGL((k_map<U, MAP>), dim3(G), dim3(256), 0, 0, args_for(i)); }, reps); \
        report((std::string(NAME) + tag).c_str(), 1, bytes, us);                                              \
    }
        M_(4, 0, "map U4 identity");
        M_(4, 1, "map U4 xcd-contiguous");
        M_(4, 2, "map U4 reversed");
        M_(4, 3, "map U4 input-first");
        M_(8, 0, "map U8 identity");
        M_(8, 1, "map U8 xcd-contiguous");
#undef M_
#define R(U, BL, NAME)                                                                                        \
    {                                                                                                         \
        const int G = (int)((nvec + (size_t)BL * U - 1) / ((size_t)BL * U));                                  \
        double us = time_launches([&](int i) { hipLaunchKernelGGL((k_reg<1, U, BL, true, true, true>), dim3(G), dim3(BL), 0, 0, args_for(i)); }, reps); \
        report((std::string(NAME) + tag).c_str(), 1, bytes, us);                                              \
    }
        R(4, 512, "reg NT U4 B512");
        R(2, 1024, "reg NT U2 B1024");
        R(4, 1024, "reg NT U4 B1024");
#undef R
        product();
        std::printf("--\n");
    }
    free_sets(S);
}

// ---- focus6: the achievable ceiling for this traffic mix, and small workgroups ----------------
// k_rd: R read streams (nt), no store unless a sum hits a sentinel no random input produces, so
// the loads cannot be removed.  k_wr: W nt store streams of a constant.  Together they say what
// 2 reads + 1 write per element can reach on this HBM, which bounds the m = 1 kernel better
// than the 8 TB/s spec.
template <int R>
__global__ __launch_bounds__(256) void k_rd(Args a, float sentinel) {
    const size_t base = (size_t)blockIdx.x * 256 * 4 + threadIdx.x;
    f32x4 x[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int u = 0; u < 4; ++u)
            x[r][u] = __builtin_nontemporal_load(r == 0 ? &a.acc[base + (size_t)u * 256] : &a.ins[r - 1][base + (size_t)u * 256]);
    __builtin_amdgcn_sched_barrier(0);
    f32x4 s = x[0][0];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (r || u) s += x[r][u];
    if (s[0] == sentinel && s[1] == sentinel) a.out[base] = s;
}

template <int W>
__global__ __launch_bounds__(256) void k_wr(Args a, float v) {
    const size_t base = (size_t)blockIdx.x * 256 * 4 + threadIdx.x;
    f32x4 c = {v, v + 1.f, v + 2.f, v + 3.f};
#pragma unroll
    for (int w = 0; w < W; ++w)
#pragma unroll
        for (int u = 0; u < 4; ++u)
            __builtin_nontemporal_store(c, (w == 0 ? a.out : (f32x4*)a.ins[w - 1]) + base + (size_t)u * 256);
}

static void report_moved(const char* name, double moved_bytes, double us) {
    const double gbps = moved_bytes / (us * 1e-6) / 1e9;
    std::printf("%-34s moved=%7.1f MiB  %9.2f us  %8.1f GB/s  %.3f of 8 TB/s\n", name, moved_bytes / (1 << 20), us,
                gbps, gbps / 8000.0);
    std::fflush(stdout);
}

static void focus6(size_t bytes, int sets, int rounds) {
    const size_t nvec = bytes / 16;
    Sets S = make_sets(1, nvec, sets);
    const int reps = 200;
    const int G = (int)(nvec / 1024);
    auto args_for = [&](int i) {
        Args a{};
        auto& b = S.bufs[i % sets];
        a.out = b[0];
        a.acc = b[0];
        a.ins[0] = b[1];
        a.nvec = nvec;
        return a;
    };
    char tag[64];
    std::snprintf(tag, sizeof tag, " sets=%d", sets);
    for (int r = 0; r < rounds; ++r) {
        double us = time_launches([&](int i) {
            Args a = args_for(i);
            const void* ins[1] = {a.ins[0]};
            chr_reduce_multi(a.out, a.acc, ins, 1, a.nvec * 4, CHR_FLOAT32, CHR_SUM, 0);
        }, reps);
        report_moved((std::string("product 2R+1W") + tag).c_str(), 3.0 * bytes, us);
        const double t_prod = us;
        us = time_launches([&](int i) { hipLaunchKernelGGL(k_rd<2>, dim3(G), dim3(256), 0, 0, args_for(i), 1e30f); }, reps);
        report_moved((std::string("read-only 2R") + tag).c_str(), 2.0 * bytes, us);
        const double t_rd = us;
        us = time_launches([&](int i) { hipLaunchKernelGGL(k_rd<1>, dim3(G), dim3(256), 0, 0, args_for(i), 1e30f); }, reps);
        report_moved((std::string("read-only 1R") + tag).c_str(), 1.0 * bytes, us);
        us = time_launches([&](int i) { hipLaunchKernelGGL(k_wr<1>, dim3(G), dim3(256), 0, 0, args_for(i), (float)i); }, reps);
        report_moved((std::string("write-only 1W") + tag).c_str(), 1.0 * bytes, us);
        const double t_wr = us;
        us = time_launches([&](int i) { hipLaunchKernelGGL(k_wr<2>, dim3(G), dim3(256), 0, 0, args_for(i), (float)i); }, reps);
        report_moved((std::string("write-only 2W") + tag).c_str(), 2.0 * bytes, us);
        std::printf("serial bound (2R time + 1W time) = %.2f us -> %.1f GB/s; product at %.3f of it\n", t_rd + t_wr,
                    3.0 * bytes / ((t_rd + t_wr) * 1e-6) / 1e9, (t_rd + t_wr) / t_prod);
#define R(U, BL, NAME)                                                                                        \
    {                                                                                                         \
        const int Gr = (int)((nvec + (size_t)BL * U - 1) / ((size_t)BL * U));                                 \
        double u_ = time_launches([&](int i) { hipLaunchKernelGGL((k_reg<1, U, BL, true, true, true>), dim3(Gr), dim3(BL), 0, 0, args_for(i)); }, reps); \
        report((std::string(NAME) + tag).c_str(), 1, bytes, u_);                                              \
    }
        R(4, 256, "reg NT U4 B256");
        R(4, 128, "reg NT U4 B128");
        R(8, 128, "reg NT U8 B128");
        R(4, 64, "reg NT U4 B64");
        R(8, 64, "reg NT U8 B64");
        R(16, 64, "reg NT U16 B64");
#undef R
        std::printf("--\n");
    }
    free_sets(S);
}

// ---- focus7: vectors per lane (U) for fan-in m >= 3 with one-wave workgroups -----------------
// k_reg's slot-0 accumulator load is plain (LLVM merges it with the tail path's), i.e. the
// product's ACC0 policy, which the product uses for every m >= 2 call.
template <int M>
static void focus7_m(size_t bytes, int sets, int rounds) {
    const size_t nvec = bytes / 16;
    Sets S = make_sets(M, nvec, sets);
    const int reps = 100;
    auto args_for = [&](int i) {
        Args a{};
        auto& b = S.bufs[i % sets];
        a.out = b[0];
        a.acc = b[0];
        for (int j = 0; j < M; ++j) a.ins[j] = b[j + 1];
        a.nvec = nvec;
        return a;
    };
    char tag[64];
    std::snprintf(tag, sizeof tag, " sets=%d", sets);
    for (int r = 0; r < rounds; ++r) {
        double us = time_launches([&](int i) {
            Args a = args_for(i);
            const void* ins[8];
            for (int j = 0; j < M; ++j) ins[j] = a.ins[j];
            chr_reduce_multi(a.out, a.acc, ins, M, a.nvec * 4, CHR_FLOAT32, CHR_SUM, 0);
        }, reps);
        report((std::string("libchiara chr_reduce_multi") + tag).c_str(), M, bytes, us);
#define R(U, BL, NAME)                                                                                        \
    {                                                                                                         \
        const int Gr = (int)((nvec + (size_t)BL * U - 1) / ((size_t)BL * U));                                 \
        double u_ = time_launches([&](int i) { hipLaunchKernelGGL((k_reg<M, U, BL, true, true, true>), dim3(Gr), dim3(BL), 0, 0, args_for(i)); }, reps); \
        report((std::string(NAME) + tag).c_str(), M, bytes, u_);                                              \
    }
        R(1, 64, "reg NT U1 B64");
        R(2, 64, "reg NT U2 B64");
        R(4, 64, "reg NT U4 B64");
        R(2, 128, "reg NT U2 B128");
        R(2, 256, "reg NT U2 B256");
#undef R
        std::printf("--\n");
    }
    free_sets(S);
}

// correctness spot check of every variant family against a host sum
static void check() {
    const size_t nvec = (1 << 20) + 37;
    std::vector<f32x4> h0(nvec), h1(nvec);
    for (size_t i = 0; i < nvec; ++i) {
        h0[i] = f32x4{(float)(i % 7), 1.f, 2.f, (float)(i % 3)};
        h1[i] = f32x4{0.5f, (float)(i % 5), 0.25f, 1.f};
    }
    f32x4 *d0, *d1;
    CK(hipMalloc(&d0, nvec * 16));
    CK(hipMalloc(&d1, nvec * 16));
    auto reset = [&] {
        CK(hipMemcpy(d0, h0.data(), nvec * 16, hipMemcpyHostToDevice));
        CK(hipMemcpy(d1, h1.data(), nvec * 16, hipMemcpyHostToDevice));
    };
    auto verify = [&](const char* name) {
        std::vector<f32x4> r(nvec);
        CK(hipMemcpy(r.data(), d0, nvec * 16, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < nvec; ++i)
            for (int c = 0; c < 4; ++c)
                if (r[i][c] != h0[i][c] + h1[i][c]) {
                    std::printf("CHECK FAIL %s at %zu\n", name, i);
                    std::exit(2);
                }
    };
    Args a{};
    a.out = d0;
    a.acc = d0;
    a.ins[0] = d1;
    a.nvec = nvec;
    reset();
    hipLaunchKernelGGL((k_reg<1, 4, 256, true, true>), dim3(777), dim3(256), 0, 0, a);
    verify("reg");
    reset();
    hipLaunchKernelGGL((k_chunk<1, 4, 256>), dim3(300), dim3(256), 0, 0, a, (nvec + 299) / 300);
    verify("chunk");
    reset();
    hipLaunchKernelGGL((k_lds<1, 2>), dim3(555), dim3(256), 0, 0, a);
    verify("lds");
    reset();
    hipLaunchKernelGGL((k_buf<1, 4, 1, 0, 0>), dim3(777), dim3(256), 0, 0, a);
    verify("buf");
    {  // whole-trip variants: a multiple of 1024 vectors
        Args w = a;
        w.nvec = (nvec / 8192) * 8192;
        const size_t keep = nvec;
        auto verify_n = [&](const char* name) {
            std::vector<f32x4> r(keep);
            CK(hipMemcpy(r.data(), d0, keep * 16, hipMemcpyDeviceToHost));
            for (size_t i = 0; i < keep; ++i)
                for (int c = 0; c < 4; ++c) {
                    const float want = i < w.nvec ? h0[i][c] + h1[i][c] : h0[i][c];
                    if (r[i][c] != want) {
                        std::printf("CHECK FAIL %s at %zu\n", name, i);
                        std::exit(2);
                    }
                }
        };
        reset();
        hipLaunchKernelGGL((k_pipe<4, 256>), dim3(3), dim3(256), 0, 0, w);
        verify_n("pipe");
        reset();
        hipLaunchKernelGGL((k_map<4, 1>), dim3((unsigned)(w.nvec / 1024)), dim3(256), 0, 0, w);
        verify_n("map-xcd");
    }
    CK(hipFree(d0));
    CK(hipFree(d1));
    std::printf("variant correctness: ok\n");
}

// Layout sensitivity of the product kernel (m = 1, 64 MiB buckets, 16 sets):
//   paired   acc_s, in_s allocated back to back (per set)
//   split    all acc buffers, then all in buffers (bench.py's order)
//   split+off  split, every buffer inside a larger allocation at +odd*4 KiB
//   slab     one slab, acc_s / in_s at s*2*B and s*2*B+B (exact power-of-two distances)
//   slab+off the slab with in_s shifted by 4 KiB * (2s+1)
static void layout_mode() {
    const size_t B = 64ull << 20, nvec = B / 16;
    const int sets = 16, reps = 200;
    auto run = [&](const char* name, std::vector<f32x4*> acc, std::vector<f32x4*> in) {
        for (int i = 0; i < sets; ++i) {
            hipLaunchKernelGGL(k_rand, dim3(4096), dim3(256), 0, 0, acc[i], nvec, 0x9E37ull * (2 * i + 1));
            hipLaunchKernelGGL(k_rand, dim3(4096), dim3(256), 0, 0, in[i], nvec, 0x9E37ull * (2 * i + 2));
        }
        CK(hipDeviceSynchronize());
        for (int round = 0; round < 2; ++round) {
            double us = time_launches([&](int i) {
                const void* ins[1] = {in[i % sets]};
                chr_reduce_multi(acc[i % sets], acc[i % sets], ins, 1, nvec * 4, CHR_FLOAT32, CHR_SUM, 0);
            }, reps);
            report(name, 1, B, us);
        }
    };
    std::vector<void*> owned;
    auto alloc = [&](size_t bytes) { void* p; CK(hipMalloc(&p, bytes)); owned.push_back(p); return (char*)p; };
    auto release = [&]() { for (void* p : owned) CK(hipFree(p)); owned.clear(); };
    std::vector<f32x4*> a(sets), b(sets);
    for (int i = 0; i < sets; ++i) { a[i] = (f32x4*)alloc(B); b[i] = (f32x4*)alloc(B); }
    run("layout paired", a, b);
    release();
    for (int i = 0; i < sets; ++i) a[i] = (f32x4*)alloc(B);
    for (int i = 0; i < sets; ++i) b[i] = (f32x4*)alloc(B);
    run("layout split", a, b);
    release();
    for (int i = 0; i < sets; ++i) a[i] = (f32x4*)(alloc(B + (1 << 20)) + 4096 * (2 * i + 1));
    for (int i = 0; i < sets; ++i) b[i] = (f32x4*)(alloc(B + (1 << 20)) + 4096 * (2 * i + 1) + 65536);
    run("layout split+off", a, b);
    release();
    char* slab = alloc(2 * B * sets + (4 << 20));
    for (int i = 0; i < sets; ++i) { a[i] = (f32x4*)(slab + 2 * B * i); b[i] = (f32x4*)(slab + 2 * B * i + B); }
    run("layout slab", a, b);
    for (int i = 0; i < sets; ++i) b[i] = (f32x4*)(slab + 2 * B * i + B + 4096 * (2 * i + 1));
    run("layout slab+off", a, b);
    release();
}

// ---- focus8: XCD-chunked workgroup -> address maps under a warm vs a cold translation state ---
// The product (one trip per one-wave workgroup, ACC0 nt policy) with blockIdx remapped so each XCD
// streams runs of C consecutive trips: workgroups dispatch round-robin over the 8 XCDs, so block b
// runs on XCD b % 8; its (b / 8)-th trip goes to chunk (b / 8) / C of that XCD, and XCD x owns
// chunks x, x + 8, x + 16, ...  C = 1 is the identity map.  A large C lets each XCD's translation
// caches see fewer distinct pages per unit time; a small C keeps all XCDs in the same DRAM rows.
template <int M, int U>
__global__ __launch_bounds__(64) void k_xmap(Args a, unsigned C) {
    const unsigned b = blockIdx.x, x = b % 8, i = b / 8;
    const size_t trip = ((size_t)(i / C) * 8 + x) * C + i % C;
    const size_t base = trip * 64 * U + threadIdx.x;
    f32x4 acc[U], v[M][U];
    acc[0] = a.acc[base];
#pragma unroll
    for (int u = 1; u < U; ++u) acc[u] = __builtin_nontemporal_load(&a.acc[base + (size_t)u * 64]);
#pragma unroll
    for (int j = 0; j < M; ++j)
#pragma unroll
        for (int u = 0; u < U; ++u) v[j][u] = __builtin_nontemporal_load(&a.ins[j][base + (size_t)u * 64]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < M; ++j)
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] = v[j][u] + acc[u];
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(acc[u], &a.out[base + (size_t)u * 64]);
}

template <int M, int U>
static void focus8_m(size_t bytes, int sets, int rounds, std::vector<unsigned> Cs = {1u, 4u, 16u, 64u, 256u, 1024u}) {
    const size_t nvec = bytes / 16;
    const unsigned G = (unsigned)(nvec / (64 * U));
    if ((size_t)G * 64 * U != nvec || G % 8) {
        std::fprintf(stderr, "focus8: bucket must be a whole number of 8-trip groups\n");
        std::exit(1);
    }
    Sets S = make_sets(M, nvec, sets);
    const int reps = 64;
    auto args_for = [&](int i) {
        Args a{};
        auto& b = S.bufs[i % sets];
        a.out = b[0];
        a.acc = b[0];
        for (int j = 0; j < M; ++j) a.ins[j] = b[j + 1];
        a.nvec = nvec;
        return a;
    };
    char tag[64];
    std::snprintf(tag, sizeof tag, " sets=%d ws=%zuMiB", sets, (size_t)sets * (M + 1) * (bytes >> 20));
    for (int r = 0; r < rounds; ++r) {
        double us = time_launches([&](int i) {
            Args a = args_for(i);
            const void* ins[8];
            for (int j = 0; j < M; ++j) ins[j] = a.ins[j];
            chr_reduce_multi(a.out, a.acc, ins, M, a.nvec * 4, CHR_FLOAT32, CHR_SUM, 0);
        }, reps);
        report((std::string("libchiara chr_reduce_multi") + tag).c_str(), M, bytes, us);
        {  // the product's kernel template, launched directly (isolates the host path)
            double t = time_launches([&](int i) {
                Args a = args_for(i);
                chr::VecArgs v{};
                v.out = (chr::u32x4*)a.out;
                v.acc = (const chr::u32x4*)a.acc;
                for (int j = 0; j < M; ++j) v.ins[j] = (const chr::u32x4*)a.ins[j];
                v.nvec = a.nvec;
                hipLaunchKernelGGL((chr::k_reduce_vec<CHR_FLOAT32, CHR_SUM, M, U, true, true, 64>), dim3(G), dim3(64), 0, 0, v);
            }, reps);
            report((std::string("product k_reduce_vec direct") + tag).c_str(), M, bytes, t);
        }
        for (unsigned C : Cs) {
            if ((G / 8) % C) continue;
            double t = time_launches([&](int i) { hipLaunchKernelGGL((k_xmap<M, U>), dim3(G), dim3(64), 0, 0, args_for(i), C); },
                                     reps);
            char name[96];
            std::snprintf(name, sizeof name, "xmap C=%u (%zu KiB/XCD run)%s", C, (size_t)C * 64 * U * 16 >> 10, tag);
            report(name, M, bytes, t);
        }
        std::printf("--\n");
    }
    free_sets(S);
}

// ---- focus10: the product tree kernel's U and XCD runs at the C4 slice shape -------------------
// Two 8-leaf trees (C4's ((l0 l1 l2 l3)(l4 l5 l6 l7)) program) of `piece` bytes per leaf in one
// launch, as the flat schedule's batched evaluation issues them; leaves rotated over `sets`.
template <int U>
static double tree_launches(const std::vector<std::vector<f32x4*>>& bufs, size_t nvec, int sets, uint32_t cs, int reps) {
    auto args_for = [&](int i) {
        chr::TreeArgs a{};
        const auto& b = bufs[i % sets];  // 18 buffers: tree t leaves b[9t .. 9t+7], out b[9t+8]
        a.nseg = 2;
        a.nl = 8;
        a.xrun = cs;
        const uint32_t trips = (uint32_t)((nvec + 64 * U - 1) / (64 * U));
        for (int j = 0; j < chr::kMaxTreeSegs; ++j) {
            a.block0[j] = j < 2 ? j * trips : ~0u;
            a.xfull[j] = j < 2 ? chr::xcd_full(trips, cs) : 0;
        }
        for (int t = 0; t < 2; ++t) {
            chr::TreeSeg& g = a.seg[t];
            for (int l = 0; l < 8; ++l) g.leaves[l] = (const chr::u32x4*)b[9 * t + l];
            g.out = (chr::u32x4*)b[9 * t + 8];
            g.nvec = nvec;
            g.comb = 0;
            const int comb[8] = {0, 1, 1, 1, 0, 1, 1, 2};
            for (int l = 0; l < 8; ++l) g.comb |= (uint32_t)comb[l] << (2 * l);
            g.swaps = 0;
        }
        return std::make_pair(a, 2 * trips);
    };
    return time_launches([&](int i) {
        auto [a, grid] = args_for(i);
        hipLaunchKernelGGL((chr::k_reduce_tree<CHR_FLOAT32, CHR_SUM, 8, U, true, 64>), dim3(grid), dim3(64), 0, 0, a);
    }, reps);
}

static void focus10(size_t piece, int sets, int rounds) {
    const size_t nvec = piece / 16;
    Sets S = make_sets(17, nvec, sets);  // 18 operands per set
    const double bytes = 2.0 * 9 * piece;
    char tag[96];
    std::snprintf(tag, sizeof tag, " piece=%zuMiB sets=%d ws=%zuMiB", piece >> 20, sets, (size_t)sets * 18 * (piece >> 20));
    for (int r = 0; r < rounds; ++r) {
        for (int u : {1, 2, 4})
            for (uint32_t run_kib : {0u, 256u, 512u, 1024u}) {
                const size_t trip = (size_t)64 * u * 16;
                uint32_t cs = 0;
                while (((size_t)2 << cs) * trip <= (size_t)run_kib * 1024 && cs < 16) ++cs;
                const double us = u == 1 ? tree_launches<1>(S.bufs, nvec, sets, cs, 40)
                                : u == 2 ? tree_launches<2>(S.bufs, nvec, sets, cs, 40)
                                         : tree_launches<4>(S.bufs, nvec, sets, cs, 40);
                char name[160];
                std::snprintf(name, sizeof name, "tree8x2 U=%d run=%uKiB%s", u, run_kib, tag);
                report_moved(name, bytes, us);
            }
        std::printf("--\n");
    }
    free_sets(S);
}

// ---- focus11: occupancy caps on the product kernels --------------------------------------------
// One-wave workgroups of the nt kernels reach ~20 waves per CU (82 VGPRs for the tree, fewer for
// the bucket kernel), i.e. every CU has 16-20 workgroups' loads queued at once at the start of a
// launch.  Dynamic LDS caps the resident workgroups per CU (160 KiB / shmem) without touching the
// kernel: does fewer, earlier-finishing waves shorten the ramp/drain of a ~30-55 us launch?
static unsigned lds_for_cap(int cap) { return cap <= 0 ? 0u : (unsigned)((160u << 10) / (unsigned)cap) & ~255u; }

static void focus11_vec(size_t bytes, int sets, int rounds) {
    const size_t nvec = bytes / 16;
    constexpr int U = 4;
    const unsigned G = (unsigned)(nvec / (64 * U));
    Sets S = make_sets(1, nvec, sets);
    char tag[64];
    std::snprintf(tag, sizeof tag, " sets=%d ws=%zuMiB", sets, (size_t)sets * 2 * (bytes >> 20));
    for (int r = 0; r < rounds; ++r) {
        for (int cap : {0, 16, 12, 8, 6, 4}) {
            const unsigned lds = lds_for_cap(cap);
            double t = time_launches([&](int i) {
                auto& b = S.bufs[i % sets];
                chr::VecArgs v{};
                v.out = (chr::u32x4*)b[0];
                v.acc = (const chr::u32x4*)b[0];
                v.ins[0] = (const chr::u32x4*)b[1];
                v.nvec = nvec;
                hipLaunchKernelGGL((chr::k_reduce_vec<CHR_FLOAT32, CHR_SUM, 1, U, true, true, 64>), dim3(G), dim3(64), lds, 0,
                                   v);
            }, 200);
            char name[96];
            std::snprintf(name, sizeof name, "vec m=1 cap=%d/CU (lds %u)%s", cap, lds, tag);
            report(name, 1, bytes, t);
        }
        std::printf("--\n");
    }
    free_sets(S);
}

template <int U = 2>
static void focus11_tree(size_t piece, int sets, int rounds, std::initializer_list<int> caps = {0, 16, 12, 8, 6, 4}) {
    const size_t nvec = piece / 16;
    Sets S = make_sets(17, nvec, sets);
    const double bytes = 2.0 * 9 * piece;
    uint32_t cs = 0;
    while (((size_t)2 << cs) * (64 * U * 16) <= (size_t)512 * 1024 && cs < 16) ++cs;  // the shipped 512 KiB runs
    char tag[96];
    std::snprintf(tag, sizeof tag, " piece=%zuMiB sets=%d ws=%zuMiB", piece >> 20, sets, (size_t)sets * 18 * (piece >> 20));
    for (int r = 0; r < rounds; ++r) {
        for (int cap : caps) {
            const unsigned lds = lds_for_cap(cap);
            double t = time_launches([&](int i) {
                chr::TreeArgs a{};
                const auto& b = S.bufs[i % sets];
                a.nseg = 2;
                a.nl = 8;
                a.xrun = cs;
                const uint32_t trips = (uint32_t)((nvec + 64 * U - 1) / (64 * U));
                for (int j = 0; j < chr::kMaxTreeSegs; ++j) {
                    a.block0[j] = j < 2 ? j * trips : ~0u;
                    a.xfull[j] = j < 2 ? chr::xcd_full(trips, cs) : 0;
                }
                const int comb[8] = {0, 1, 1, 1, 0, 1, 1, 2};
                for (int t2 = 0; t2 < 2; ++t2) {
                    chr::TreeSeg& g = a.seg[t2];
                    for (int l = 0; l < 8; ++l) g.leaves[l] = (const chr::u32x4*)b[9 * t2 + l];
                    g.out = (chr::u32x4*)b[9 * t2 + 8];
                    g.nvec = nvec;
                    g.comb = 0;
                    for (int l = 0; l < 8; ++l) g.comb |= (uint32_t)comb[l] << (2 * l);
                    g.swaps = 0;
                }
                hipLaunchKernelGGL((chr::k_reduce_tree<CHR_FLOAT32, CHR_SUM, 8, U, true, 64>), dim3(2 * trips), dim3(64), lds,
                                   0, a);
            }, 40);
            char name[160];
            std::snprintf(name, sizeof name, "tree8x2 U=%d cap=%d/CU (lds %u)%s", U, cap, lds, tag);
            report_moved(name, bytes, t);
        }
        std::printf("--\n");
    }
    free_sets(S);
}

// ---- focus12: U x occupancy cap for the product bucket kernel -----------------------------------
template <int M, int U>
static void focus12_mu(size_t bytes, int sets, std::initializer_list<int> caps) {
    const size_t nvec = bytes / 16;
    const unsigned G = (unsigned)(nvec / (64 * U));
    Sets S = make_sets(M, nvec, sets);
    uint32_t cs = 0;  // the shipped XCD runs: identity for m <= 2, 512 KiB above
    if (M > 2)
        while (((size_t)2 << cs) * (64 * U * 16) <= (size_t)512 * 1024 && cs < 16) ++cs;
    char tag[64];
    std::snprintf(tag, sizeof tag, " sets=%d ws=%zuMiB", sets, (size_t)sets * (M + 1) * (bytes >> 20));
    for (int cap : caps) {
        const unsigned lds = lds_for_cap(cap);
        double t = time_launches([&](int i) {
            auto& b = S.bufs[i % sets];
            chr::VecArgs v{};
            v.out = (chr::u32x4*)b[0];
            v.acc = (const chr::u32x4*)b[0];
            for (int j = 0; j < M; ++j) v.ins[j] = (const chr::u32x4*)b[j + 1];
            v.nvec = nvec;
            v.xrun = cs;
            v.xfull = chr::xcd_full(G, cs);
            hipLaunchKernelGGL((chr::k_reduce_vec<CHR_FLOAT32, CHR_SUM, M, U, true, true, 64>), dim3(G), dim3(64), lds, 0, v);
        }, M == 1 ? 200 : 40);
        char name[96];
        std::snprintf(name, sizeof name, "vec U=%d cap=%d/CU%s", U, cap, tag);
        report(name, M, bytes, t);
    }
    free_sets(S);
}

// ---- focus13: the C2 shape under the occupancy cap: XCD runs, ACC0 and workgroup size ----------
template <bool ACC0, int BL>
static double c2_variant(Sets& S, size_t nvec, int sets, unsigned lds, uint32_t cs) {
    constexpr int U = 4;
    const unsigned G = (unsigned)(nvec / (BL * U));
    return time_launches([&](int i) {
        auto& b = S.bufs[i % sets];
        chr::VecArgs v{};
        v.out = (chr::u32x4*)b[0];
        v.acc = (const chr::u32x4*)b[0];
        v.ins[0] = (const chr::u32x4*)b[1];
        v.nvec = nvec;
        v.xrun = cs;
        v.xfull = chr::xcd_full(G, cs);
        hipLaunchKernelGGL((chr::k_reduce_vec<CHR_FLOAT32, CHR_SUM, 1, U, true, ACC0, BL>), dim3(G), dim3(BL), lds, 0, v);
    }, 200);
}

static void focus13(int rounds) {
    const size_t bytes = 64 << 20, nvec = bytes / 16;
    const int sets = 16;
    Sets S = make_sets(1, nvec, sets);
    for (int r = 0; r < rounds; ++r) {
        for (int cap : {12, 13}) {
            for (unsigned run_kib : {0u, 64u, 256u, 1024u}) {
                uint32_t cs = 0;
                while (((size_t)2 << cs) * (64 * 4 * 16) <= (size_t)run_kib * 1024 && cs < 16) ++cs;
                char name[96];
                std::snprintf(name, sizeof name, "c2 cap=%d run=%uKiB acc0", cap, run_kib);
                report(name, 1, bytes, c2_variant<true, 64>(S, nvec, sets, lds_for_cap(cap), cs));
            }
            char name[96];
            std::snprintf(name, sizeof name, "c2 cap=%d all-nt", cap);
            report(name, 1, bytes, c2_variant<false, 64>(S, nvec, sets, lds_for_cap(cap), 0));
        }
        for (int cap : {0, 5, 6, 7, 8}) {  // two-wave workgroups: cap counts workgroups
            char name[96];
            std::snprintf(name, sizeof name, "c2 BL=128 cap=%d acc0", cap);
            report(name, 1, bytes, c2_variant<true, 128>(S, nvec, sets, lds_for_cap(cap), 0));
        }
        for (int cap : {0, 3, 4}) {
            char name[96];
            std::snprintf(name, sizeof name, "c2 BL=256 cap=%d acc0", cap);
            report(name, 1, bytes, c2_variant<true, 256>(S, nvec, sets, lds_for_cap(cap), 0));
        }
        std::printf("--\n");
    }
    free_sets(S);
}

// ---- focus18: small trees (the N = 2 / N = 4 flat schedules: 2 and 4 leaves) -------------------
// One segment of NL leaves (a left fold, MPI_Reduce_local order) of `piece` bytes per leaf.
template <int NL, int U>
static void focus18_tree(size_t piece, int sets, std::initializer_list<int> caps, uint32_t run_kib) {
    const size_t nvec = piece / 16;
    Sets S = make_sets(NL, nvec, sets);  // NL + 1 operands: leaves b[0..NL-1], out b[NL]
    const double bytes = (NL + 1.0) * piece;
    uint32_t cs = 0;
    while (run_kib && ((size_t)2 << cs) * (64 * U * 16) <= (size_t)run_kib * 1024 && cs < 16) ++cs;
    for (int cap : caps) {
        const unsigned lds = lds_for_cap(cap);
        double t = time_launches([&](int i) {
            chr::TreeArgs a{};
            const auto& b = S.bufs[i % sets];
            a.nseg = 1;
            a.nl = NL;
            a.xrun = cs;
            const uint32_t trips = (uint32_t)((nvec + 64 * U - 1) / (64 * U));
            for (int j = 0; j < chr::kMaxTreeSegs; ++j) {
                a.block0[j] = j == 0 ? 0 : ~0u;
                a.xfull[j] = j == 0 ? chr::xcd_full(trips, cs) : 0;
            }
            chr::TreeSeg& g = a.seg[0];
            for (int l = 0; l < NL; ++l) g.leaves[l] = (const chr::u32x4*)b[l];
            g.out = (chr::u32x4*)b[NL];
            g.nvec = nvec;
            g.comb = 0;
            for (int l = 1; l < NL; ++l) g.comb |= 1u << (2 * l);  // left fold
            g.swaps = 0;
            hipLaunchKernelGGL((chr::k_reduce_tree<CHR_FLOAT32, CHR_SUM, NL, U, true, 64>), dim3(trips), dim3(64), lds, 0, a);
        }, 40);
        char name[160];
        std::snprintf(name, sizeof name, "tree NL=%d U=%d cap=%d run=%uKiB piece=%zuMiB sets=%d", NL, U, cap, run_kib,
                      piece >> 20, sets);
        report_moved(name, bytes, t);
    }
    free_sets(S);
}

// ---- focus19: the NT threshold under the new shapes (mid sizes: plain 256-thread vs nt one-wave) ---
template <int U, bool NT, int BL>
static double tree8x2_time(Sets& S, size_t nvec, int sets, unsigned lds, uint32_t cs) {
    return time_launches([&](int i) {
        chr::TreeArgs a{};
        const auto& b = S.bufs[i % sets];
        a.nseg = 2;
        a.nl = 8;
        a.xrun = cs;
        const uint32_t trips = (uint32_t)((nvec + BL * U - 1) / (BL * U));
        for (int j = 0; j < chr::kMaxTreeSegs; ++j) {
            a.block0[j] = j < 2 ? j * trips : ~0u;
            a.xfull[j] = j < 2 ? chr::xcd_full(trips, cs) : 0;
        }
        const int comb[8] = {0, 1, 1, 1, 0, 1, 1, 2};
        for (int t2 = 0; t2 < 2; ++t2) {
            chr::TreeSeg& g = a.seg[t2];
            for (int l = 0; l < 8; ++l) g.leaves[l] = (const chr::u32x4*)b[9 * t2 + l];
            g.out = (chr::u32x4*)b[9 * t2 + 8];
            g.nvec = nvec;
            g.comb = 0;
            for (int l = 0; l < 8; ++l) g.comb |= (uint32_t)comb[l] << (2 * l);
            g.swaps = 0;
        }
        hipLaunchKernelGGL((chr::k_reduce_tree<CHR_FLOAT32, CHR_SUM, 8, U, NT, BL>), dim3(2 * trips), dim3(BL), lds, 0, a);
    }, 100);
}

static void focus19(size_t piece, int sets) {
    const size_t nvec = piece / 16;
    Sets S = make_sets(17, nvec, sets);
    const double bytes = 2.0 * 9 * piece;
    uint32_t cs = 0;
    while (((size_t)2 << cs) * (64 * 1 * 16) <= (size_t)512 * 1024 && cs < 16) ++cs;
    char name[128];
    std::snprintf(name, sizeof name, "tree8x2 plain U=2 BL=256 piece=%zuMiB sets=%d", piece >> 20, sets);
    report_moved(name, bytes, tree8x2_time<2, false, 256>(S, nvec, sets, 0, 0));
    std::snprintf(name, sizeof name, "tree8x2 nt U=1 cap16 runs piece=%zuMiB sets=%d", piece >> 20, sets);
    report_moved(name, bytes, tree8x2_time<1, true, 64>(S, nvec, sets, lds_for_cap(16), cs));
    std::snprintf(name, sizeof name, "tree8x2 nt U=2 uncapped piece=%zuMiB sets=%d", piece >> 20, sets);
    report_moved(name, bytes, tree8x2_time<2, true, 64>(S, nvec, sets, 0, 0));
    free_sets(S);
}

// ---- focus30: fewer, fatter workgroups for the in-collective 8-leaf trees -------
// C4's slice at 8 and 16 MiB pieces (2 trees x 9 operands), back to back: the product shape (one wave,
// U = 1, 16 per CU) against U = 2 and 128 / 256-thread workgroups with the cap scaled to the same waves
// per CU, all with 512 KiB XCD runs.  A fatter workgroup means fewer dispatches per grid and a shorter
// ramp if the dispatcher, not memory latency, paces the start of a grid.
template <int U, int BL>
static void focus30_shape(Sets& S, size_t nvec, int sets, int waves_per_cu, size_t piece) {
    uint32_t cs = 0;
    while (((size_t)2 << cs) * ((size_t)BL * U * 16) <= (size_t)512 * 1024 && cs < 16) ++cs;
    const int cap = waves_per_cu / (BL / 64);
    char name[160];
    std::snprintf(name, sizeof name, "tree8x2 nt U=%d BL=%d cap=%d (%d waves/CU) piece=%zuMiB sets=%d", U, BL, cap,
                  waves_per_cu, piece >> 20, sets);
    report_moved(name, 2.0 * 9 * piece, tree8x2_time<U, true, BL>(S, nvec, sets, lds_for_cap(cap), cs));
}

static void focus30(size_t piece, int sets) {
    const size_t nvec = piece / 16;
    Sets S = make_sets(17, nvec, sets);
    focus30_shape<1, 64>(S, nvec, sets, 16, piece);
    focus30_shape<2, 64>(S, nvec, sets, 16, piece);
    focus30_shape<1, 128>(S, nvec, sets, 16, piece);
    focus30_shape<1, 256>(S, nvec, sets, 16, piece);
    focus30_shape<2, 256>(S, nvec, sets, 16, piece);
    focus30_shape<1, 256>(S, nvec, sets, 32, piece);
    free_sets(S);
}

// ---- focus31: page-local streaming past the translation reach (second attempt) -------
// The product's one-trip grid hands consecutive trips of a run to every CU of an XCD, so every CU touches every
// 2 MiB page of its XCD's share: (pages x CUs) first-level translations per launch.  Here a resident grid of
// G one-wave workgroups walks chunks of C consecutive trips (chunk c -> workgroup c mod G), so a page is
// touched by 2 MiB / (C x trip bytes) workgroups: C = 1 is the old grid-stride form, C x 2 KiB = 2 MiB gives
// each page to one workgroup (one CU).  Same loads, adds and nt / ACC0 policy as k_reduce_vec's trip.
template <int M, int U>
__global__ __launch_bounds__(64) void k_span(chr::VecArgs a, unsigned chunk, unsigned G) {
    using chr::u32x4;
    u32x4* const out = a.out;
    const u32x4* const accp = a.acc;
    const u32x4* ins[M];
#pragma unroll
    for (int j = 0; j < M; ++j) ins[j] = a.ins[j];
    const size_t nvec = a.nvec;
    const size_t trips = nvec / (64 * U);  // whole trips only (focus31 sizes are multiples)
    for (size_t c = blockIdx.x;; c += G) {
        const size_t t0 = c * chunk;
        if (t0 >= trips) break;
        const size_t t1 = t0 + chunk < trips ? t0 + chunk : trips;
        for (size_t t = t0; t < t1; ++t) {
            const size_t base = t * 64 * U + threadIdx.x;
            u32x4 acc[U], x[M][U];
            acc[0] = chr::ld<false>(&accp[base]);
#pragma unroll
            for (int u = 1; u < U; ++u) acc[u] = chr::ld<true>(&accp[base + (size_t)u * 64]);
#pragma unroll
            for (int j = 0; j < M; ++j)
#pragma unroll
                for (int u = 0; u < U; ++u) x[j][u] = chr::ld<true>(&ins[j][base + (size_t)u * 64]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < M; ++j)
#pragma unroll
                for (int u = 0; u < U; ++u) acc[u] = chr::apply_vec<CHR_FLOAT32, CHR_SUM>(x[j][u], acc[u]);
#pragma unroll
            for (int u = 0; u < U; ++u) chr::st<true>(&out[base + (size_t)u * 64], acc[u]);
        }
    }
}

template <int M, int U>
static void focus31_m(size_t bytes, int sets, int ncu) {
    const size_t nvec = bytes / 16;
    const unsigned trips = (unsigned)(nvec / (64 * U));
    Sets S = make_sets(M, nvec, sets);
    uint32_t cs = 0;  // the product's runs (vec_xcd_run_kib)
    const size_t run_kib = M <= 3 ? 256 : 512;
    while (((size_t)2 << cs) * (64 * U * 16) <= run_kib * 1024 && cs < 16) ++cs;
    const unsigned lds = lds_for_cap(12);
    char tag[64];
    std::snprintf(tag, sizeof tag, " sets=%d ws=%zuMiB", sets, (size_t)sets * (M + 1) * (bytes >> 20));
    auto vargs = [&](int i) {
        auto& b = S.bufs[i % sets];
        chr::VecArgs v{};
        v.out = (chr::u32x4*)b[0];
        v.acc = (const chr::u32x4*)b[0];
        for (int j = 0; j < M; ++j) v.ins[j] = (const chr::u32x4*)b[j + 1];
        v.nvec = nvec;
        return v;
    };
    const int reps = std::max(6, (int)std::min<size_t>(60, (16ull << 30) / ((M + 1) * bytes)));
    double t = time_launches([&](int i) {
        chr::VecArgs v = vargs(i);
        v.xrun = cs;
        v.xfull = chr::xcd_full(trips, cs);
        hipLaunchKernelGGL((chr::k_reduce_vec<CHR_FLOAT32, CHR_SUM, M, U, true, true, 64>), dim3(trips), dim3(64), lds,
                           0, v);
    }, reps);
    char name[128];
    std::snprintf(name, sizeof name, "product one-trip runs%zuK%s", run_kib, tag);
    report(name, M, bytes, t);
    for (unsigned per_cu : {11u, 8u}) {
        const unsigned G = (unsigned)ncu * per_cu;
        for (unsigned chunk : {1u, 16u, 128u, 1024u, (trips + G - 1) / G}) {
            t = time_launches([&](int i) {
                hipLaunchKernelGGL((k_span<M, U>), dim3(G), dim3(64), lds, 0, vargs(i), chunk, G);
            }, reps);
            std::snprintf(name, sizeof name, "span G=%u/CU chunk=%u trips (%u KiB)%s", per_cu, chunk,
                          chunk * 64u * U * 16u >> 10, tag);
            report(name, M, bytes, t);
        }
    }
    free_sets(S);
}

// ---- focus32: the bf16 tree (C5) against the f32 one (C4) at the in-collective shapes ---------------
// C5's per-GPU grids run 3-6 % below C4's at equal bytes (profiles/r05/rank_trees/).  A bf16 combine widens both
// operands, adds in f32 and packs with RNE: ~7 VALU per dword against 1 for f32, which stretches a one-trip
// workgroup's life after its loads land.  More bytes per wave (U = 2) or more waves per CU (cap 16 / 20 /
// uncapped) keep more loads in flight through that tail; cap 12 is what the collective runs beside RCCL.
template <int DT, int U>
static double tree8x2_time_dt(Sets& S, size_t nvec, int sets, unsigned lds, uint32_t cs) {
    return time_launches([&](int i) {
        chr::TreeArgs a{};
        const auto& b = S.bufs[i % sets];
        a.nseg = 2;
        a.nl = 8;
        a.xrun = cs;
        const uint32_t trips = (uint32_t)((nvec + 64 * U - 1) / (64 * U));
        for (int j = 0; j < chr::kMaxTreeSegs; ++j) {
            a.block0[j] = j < 2 ? j * trips : ~0u;
            a.xfull[j] = j < 2 ? chr::xcd_full(trips, cs) : 0;
        }
        const int comb[8] = {0, 1, 1, 1, 0, 1, 1, 2};
        for (int t2 = 0; t2 < 2; ++t2) {
            chr::TreeSeg& g = a.seg[t2];
            for (int l = 0; l < 8; ++l) g.leaves[l] = (const chr::u32x4*)b[9 * t2 + l];
            g.out = (chr::u32x4*)b[9 * t2 + 8];
            g.nvec = nvec;
            g.comb = 0;
            for (int l = 0; l < 8; ++l) g.comb |= (uint32_t)comb[l] << (2 * l);
            g.swaps = 0;
        }
        hipLaunchKernelGGL((chr::k_reduce_tree<DT, CHR_SUM, 8, U, true, 64>), dim3(2 * trips), dim3(64), lds, 0, a);
    }, 60);
}

template <int DT, int U>
static void focus32_row(Sets& S, size_t nvec, int sets, size_t piece, int cap) {
    uint32_t cs = 0;  // the product's 512 KiB runs for 5+ leaves
    while (((size_t)2 << cs) * ((size_t)64 * U * 16) <= (size_t)512 * 1024 && cs < 16) ++cs;
    char name[160];
    std::snprintf(name, sizeof name, "tree8x2 %s U=%d cap=%d piece=%zuMiB sets=%d", DT == CHR_FLOAT32 ? "f32 " : "bf16",
                  U, cap, piece >> 20, sets);
    report_moved(name, 2.0 * 9 * piece, tree8x2_time_dt<DT, U>(S, nvec, sets, lds_for_cap(cap), cs));
}

static void focus32(size_t piece, int sets) {
    const size_t nvec = piece / 16;
    Sets S = make_sets(17, nvec, sets);
    for (int cap : {12, 16, 20, 0}) {
        focus32_row<CHR_FLOAT32, 1>(S, nvec, sets, piece, cap);
        focus32_row<CHR_BFLOAT16, 1>(S, nvec, sets, piece, cap);
        focus32_row<CHR_BFLOAT16, 2>(S, nvec, sets, piece, cap);
    }
    free_sets(S);
}

// ---- focus33: the second vector of each leaf through LDS (in-collective cap 12) -----------------------------
// U = 2 in registers recovers the bytes in flight that cap 12 costs the trees but needs 82-90 VGPRs, which locks
// RCCL's ~288-VGPR waves out (profiles/r05/cores_u/).  The cap already reserves 13.5 KiB of LDS per workgroup
// that nothing uses: here the trip is U = 2 vectors per lane, the first held in registers as in k_reduce_tree, the
// second landed in that LDS by global_load_lds_dwordx4 (1 KiB per leaf per wave; each lane reads back only the
// 16 B its own DMA wrote, so the wave's own vmcnt orders it).  Half 0 is evaluated while half 1 sits in LDS, so
// the register peak stays near U = 1's.
template <int DT, int OP, int NL, bool NT>
__global__ __launch_bounds__(64) void k_tree_lds(chr::TreeArgs a) {
    using chr::u32x4;
    extern __shared__ u32x4 lbuf[];
    const uint32_t b = blockIdx.x, xrun = a.xrun;
    uint32_t b0s[chr::kMaxTreeSegs], xfs[chr::kMaxTreeSegs], hds[chr::kMaxTreeSegs];
#pragma unroll
    for (int j = 0; j < chr::kMaxTreeSegs; ++j) {
        b0s[j] = a.block0[j];
        xfs[j] = a.xfull[j];
        hds[j] = a.hand[j];
        chr::pin_sgpr_u32(b0s[j], xfs[j]);
        chr::pin_sgpr_u32(hds[j], xrun);
    }
    int s = 0;
    uint32_t b0 = 0, xfull = xfs[0], hand = hds[0];
#pragma unroll
    for (int j = 1; j < chr::kMaxTreeSegs; ++j)
        if (b >= b0s[j]) {
            s = j;
            b0 = b0s[j];
            xfull = xfs[j];
            hand = hds[j];
        }
    const chr::TreeSeg& g = a.seg[s];
    u32x4* const out = g.out;
    const u32x4* leaves[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) leaves[j] = g.leaves[j];
    const size_t nvec = g.nvec;
    const uint32_t comb = g.comb, swaps = g.swaps;
    chr::pin_sgpr(out, leaves[0], nvec, comb, swaps);
#pragma unroll
    for (int j = 1; j < NL; ++j) chr::pin_sgpr(leaves[j]);
    const size_t trip = chr::xcd_trip_w(b - b0, xfull, xrun, hand);
    if (trip == chr::kIdleTrip) return;
    const size_t base = trip * 128 + threadIdx.x;
    if ((trip + 1) * 128 <= nvec) {
        u32x4 x[NL][1];
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            x[j][0] = chr::ld<NT>(&leaves[j][base]);
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)&leaves[j][base + 64],
                                             (__attribute__((address_space(3))) void*)&lbuf[j * 64], 16, 0,
                                             NT ? 2 : 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        u32x4 r0[1];
        chr::tree_eval<u32x4, NL, 1, chr::VecOp<DT, OP>>(x, r0, comb, swaps);
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        u32x4 y[NL][1];
#pragma unroll
        for (int j = 0; j < NL; ++j) y[j][0] = lbuf[j * 64 + threadIdx.x];
        u32x4 r1[1];
        chr::tree_eval<u32x4, NL, 1, chr::VecOp<DT, OP>>(y, r1, comb, swaps);
        chr::st<NT>(&out[base], r0[0]);
        chr::st<NT>(&out[base + 64], r1[0]);
    } else {
        for (int u = 0; u < 2; ++u) {
            const size_t i = base + (size_t)u * 64;
            if (i >= nvec) break;
            u32x4 x[NL][1];
#pragma unroll
            for (int j = 0; j < NL; ++j) x[j][0] = leaves[j][i];
            u32x4 r[1];
            chr::tree_eval<u32x4, NL, 1, chr::VecOp<DT, OP>>(x, r, comb, swaps);
            out[i] = r[0];
        }
    }
}

// tree8x2 at the product's 512 KiB runs and the odd-XCD handover (shift 6), kernel chosen by KIND: 0 = product U = 1,
// 1 = product U = 2, 2 = k_tree_lds
template <int DT, int KIND>
static double tree8x2_kind(Sets& S, size_t nvec, int sets, unsigned lds) {
    constexpr int U = KIND == 0 ? 1 : 2;
    uint32_t cs = 0;
    while (((size_t)2 << cs) * ((size_t)64 * U * 16) <= (size_t)512 * 1024 && cs < 16) ++cs;
    return time_launches([&](int i) {
        chr::TreeArgs a{};
        const auto& b = S.bufs[i % sets];
        a.nseg = 2;
        a.nl = 8;
        a.xrun = cs;
        const uint32_t trips = (uint32_t)((nvec + 64 * U - 1) / (64 * U));
        size_t grid = 0;
        for (int j = 0; j < chr::kMaxTreeSegs; ++j) {
            if (j >= 2) {
                a.block0[j] = ~0u;
                continue;
            }
            grid = (grid + 7) & ~(size_t)7;
            a.block0[j] = (uint32_t)grid;
            a.xfull[j] = chr::xcd_full(trips, cs);
            a.hand[j] = chr::xcd_hand(a.xfull[j], 6);
            grid += trips + 8u * (size_t)a.hand[j];
        }
        const int comb[8] = {0, 1, 1, 1, 0, 1, 1, 2};
        for (int t2 = 0; t2 < 2; ++t2) {
            chr::TreeSeg& g = a.seg[t2];
            for (int l = 0; l < 8; ++l) g.leaves[l] = (const chr::u32x4*)b[9 * t2 + l];
            g.out = (chr::u32x4*)b[9 * t2 + 8];
            g.nvec = nvec;
            g.comb = 0;
            for (int l = 0; l < 8; ++l) g.comb |= (uint32_t)comb[l] << (2 * l);
            g.swaps = 0;
        }
        if constexpr (KIND == 2)
            hipLaunchKernelGGL((k_tree_lds<DT, CHR_SUM, 8, true>), dim3((unsigned)grid), dim3(64), lds, 0, a);
        else
            hipLaunchKernelGGL((chr::k_reduce_tree<DT, CHR_SUM, 8, U, true, 64>), dim3((unsigned)grid), dim3(64), lds, 0,
                               a);
    }, 60);
}

static void focus33(size_t piece, int sets) {
    const size_t nvec = piece / 16;
    Sets S = make_sets(17, nvec, sets);
    const char* kinds[3] = {"U=1    ", "U=2    ", "U=1+LDS"};
    for (int cap : {12, 16}) {
        const unsigned lds = lds_for_cap(cap);
        char name[160];
#define F33(DT, K)                                                                                             \
    std::snprintf(name, sizeof name, "tree8x2 %s %s cap=%d piece=%zuMiB sets=%d", DT == CHR_FLOAT32 ? "f32 " : "bf16", \
                  kinds[K], cap, piece >> 20, sets);                                                          \
    report_moved(name, 2.0 * 9 * piece, tree8x2_kind<DT, K>(S, nvec, sets, lds));
        F33(CHR_FLOAT32, 0) F33(CHR_FLOAT32, 1) F33(CHR_FLOAT32, 2)
        F33(CHR_BFLOAT16, 0) F33(CHR_BFLOAT16, 1) F33(CHR_BFLOAT16, 2)
#undef F33
    }
    free_sets(S);
}

// A correctness check of k_tree_lds against the product U = 1 kernel (bit-identical outputs), run once.
static bool focus33_check() {
    const size_t nvec = (size_t)(3 << 20) / 16 + 37;  // a partial trip at the end
    Sets S = make_sets(17, nvec, 1);
    chr::u32x4 *o1, *o2;
    CK(hipMalloc(&o1, nvec * 16));
    CK(hipMalloc(&o2, nvec * 16));
    bool ok = true;
    for (int kind = 0; kind < 2 && ok; ++kind) {
        chr::TreeArgs a{};
        auto& b = S.bufs[0];
        a.nseg = 1;
        a.nl = 8;
        a.xrun = 0;
        const int comb[8] = {0, 1, 0, 1, 1, 0, 2, 2};
        for (int j = 0; j < chr::kMaxTreeSegs; ++j) a.block0[j] = j ? ~0u : 0;
        chr::TreeSeg& g = a.seg[0];
        for (int l = 0; l < 8; ++l) g.leaves[l] = (const chr::u32x4*)b[l];
        g.nvec = nvec;
        g.comb = 0;
        for (int l = 0; l < 8; ++l) g.comb |= (uint32_t)comb[l] << (2 * l);
        g.swaps = 0x15;
        const uint32_t t1 = (uint32_t)((nvec + 63) / 64), t2 = (uint32_t)((nvec + 127) / 128);
        a.xfull[0] = chr::xcd_full(t1, 0);
        g.out = o1;
        hipLaunchKernelGGL((chr::k_reduce_tree<CHR_FLOAT32, CHR_MAX, 8, 1, true, 64>), dim3(t1), dim3(64), 0, 0, a);
        a.xfull[0] = chr::xcd_full(t2, 0);
        g.out = o2;
        if (kind == 0)
            hipLaunchKernelGGL((k_tree_lds<CHR_FLOAT32, CHR_MAX, 8, true>), dim3(t2), dim3(64), lds_for_cap(12), 0, a);
        else
            hipLaunchKernelGGL((k_tree_lds<CHR_BFLOAT16, CHR_SUM, 8, true>), dim3(t2), dim3(64), lds_for_cap(16), 0, a);
        if (kind == 1) {  // compare against the product's bf16 U = 1
            a.xfull[0] = chr::xcd_full(t1, 0);
            g.out = o1;
            hipLaunchKernelGGL((chr::k_reduce_tree<CHR_BFLOAT16, CHR_SUM, 8, 1, true, 64>), dim3(t1), dim3(64), 0, 0, a);
        }
        CK(hipDeviceSynchronize());
        std::vector<uint32_t> h1(nvec * 4), h2(nvec * 4);
        CK(hipMemcpy(h1.data(), o1, nvec * 16, hipMemcpyDeviceToHost));
        CK(hipMemcpy(h2.data(), o2, nvec * 16, hipMemcpyDeviceToHost));
        ok = h1 == h2;
        std::printf("{\"focus33_check\": %d, \"bit_identical\": %s}\n", kind, ok ? "true" : "false");
    }
    CK(hipFree(o1));
    CK(hipFree(o2));
    free_sets(S);
    return ok;
}

// ---- focus34: the tree program known at compile time ---------------------------------------------------------
// k_reduce_tree interprets the post-order program (comb / swap bits) at run time: every push and combine is a scalar
// branch over the stack depth with u32x4 moves between named slots.  For bf16 each combine also widens, adds and
// RNE-packs (~6 VALU per dword), so a trip's VALU tail after its loads land is longest there, and at the
// in-collective cap of 12 workgroups per CU bf16 trees run 3-6 % behind f32 (focus32).  Here the same trip with
// the program as a template argument (C4 / C5's ((l0 l1 l2 l3)(l4 l5 l6 l7)), no swaps): the branches and slot
// moves fold away.  Same arithmetic, same order.
template <int DT, int OP, int NL, uint32_t COMB>
__device__ __forceinline__ chr::u32x4 tree_eval_static(const chr::u32x4 (&x)[NL]) {
    chr::u32x4 st[4];
    int d = 0;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
        st[d++] = x[j];
#pragma unroll
        for (int c = (int)((COMB >> (2 * j)) & 3u); c > 0; --c) {
            st[d - 2] = chr::apply_vec<DT, OP>(st[d - 1], st[d - 2]);
            --d;
        }
    }
    return st[0];
}

template <int DT, int OP, int NL, uint32_t COMB>
__global__ __launch_bounds__(64) void k_tree_static(chr::TreeArgs a) {
    using chr::u32x4;
    const uint32_t b = blockIdx.x, xrun = a.xrun;
    uint32_t b0s[chr::kMaxTreeSegs], xfs[chr::kMaxTreeSegs], hds[chr::kMaxTreeSegs];
#pragma unroll
    for (int j = 0; j < chr::kMaxTreeSegs; ++j) {
        b0s[j] = a.block0[j];
        xfs[j] = a.xfull[j];
        hds[j] = a.hand[j];
        chr::pin_sgpr_u32(b0s[j], xfs[j]);
        chr::pin_sgpr_u32(hds[j], xrun);
    }
    int s = 0;
    uint32_t b0 = 0, xfull = xfs[0], hand = hds[0];
#pragma unroll
    for (int j = 1; j < chr::kMaxTreeSegs; ++j)
        if (b >= b0s[j]) {
            s = j;
            b0 = b0s[j];
            xfull = xfs[j];
            hand = hds[j];
        }
    const chr::TreeSeg& g = a.seg[s];
    u32x4* const out = g.out;
    const u32x4* leaves[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) leaves[j] = g.leaves[j];
    const size_t nvec = g.nvec;
    chr::pin_sgpr(out, leaves[0], nvec, 0u, 0u);
#pragma unroll
    for (int j = 1; j < NL; ++j) chr::pin_sgpr(leaves[j]);
    const size_t trip = chr::xcd_trip_w(b - b0, xfull, xrun, hand);
    if (trip == chr::kIdleTrip) return;
    const size_t base = trip * 64 + threadIdx.x;
    if ((trip + 1) * 64 <= nvec) {
        u32x4 x[NL];
#pragma unroll
        for (int j = 0; j < NL; ++j) x[j] = chr::ld<true>(&leaves[j][base]);
        __builtin_amdgcn_sched_barrier(0);
        chr::st<true>(&out[base], tree_eval_static<DT, OP, NL, COMB>(x));
    } else if (base < nvec) {
        u32x4 x[NL];
#pragma unroll
        for (int j = 0; j < NL; ++j) x[j] = leaves[j][base];
        out[base] = tree_eval_static<DT, OP, NL, COMB>(x);
    }
}

constexpr uint32_t kC4Comb = (0u << 0) | (1u << 2) | (1u << 4) | (1u << 6) | (0u << 8) | (1u << 10) | (1u << 12) | (2u << 14);

// tree8x2 at the product's 512 KiB runs and handover shift 6: KIND 0 = product k_reduce_tree U = 1, 1 = k_tree_static
template <int DT, int KIND>
static double tree8x2_static(Sets& S, size_t nvec, int sets, unsigned lds) {
    uint32_t cs = 0;
    while (((size_t)2 << cs) * ((size_t)64 * 16) <= (size_t)512 * 1024 && cs < 16) ++cs;
    return time_launches([&](int i) {
        chr::TreeArgs a{};
        const auto& b = S.bufs[i % sets];
        a.nseg = 2;
        a.nl = 8;
        a.xrun = cs;
        const uint32_t trips = (uint32_t)((nvec + 63) / 64);
        size_t grid = 0;
        for (int j = 0; j < chr::kMaxTreeSegs; ++j) {
            if (j >= 2) {
                a.block0[j] = ~0u;
                continue;
            }
            grid = (grid + 7) & ~(size_t)7;
            a.block0[j] = (uint32_t)grid;
            a.xfull[j] = chr::xcd_full(trips, cs);
            a.hand[j] = chr::xcd_hand(a.xfull[j], 6);
            grid += trips + 8u * (size_t)a.hand[j];
        }
        for (int t2 = 0; t2 < 2; ++t2) {
            chr::TreeSeg& g = a.seg[t2];
            for (int l = 0; l < 8; ++l) g.leaves[l] = (const chr::u32x4*)b[9 * t2 + l];
            g.out = (chr::u32x4*)b[9 * t2 + 8];
            g.nvec = nvec;
            g.comb = kC4Comb;
            g.swaps = 0;
        }
        if constexpr (KIND == 1)
            hipLaunchKernelGGL((k_tree_static<DT, CHR_SUM, 8, kC4Comb>), dim3((unsigned)grid), dim3(64), lds, 0, a);
        else
            hipLaunchKernelGGL((chr::k_reduce_tree<DT, CHR_SUM, 8, 1, true, 64>), dim3((unsigned)grid), dim3(64), lds, 0,
                               a);
    }, 60);
}

static void focus34(size_t piece, int sets) {
    const size_t nvec = piece / 16;
    Sets S = make_sets(17, nvec, sets);
    for (int cap : {12, 16}) {
        const unsigned lds = lds_for_cap(cap);
        char name[160];
#define F34(DT, K)                                                                                              \
    std::snprintf(name, sizeof name, "tree8x2 %s %s cap=%d piece=%zuMiB sets=%d", DT == CHR_FLOAT32 ? "f32 " : "bf16", \
                  K ? "static " : "runtime", cap, piece >> 20, sets);                                            \
    report_moved(name, 2.0 * 9 * piece, tree8x2_static<DT, K>(S, nvec, sets, lds));
        F34(CHR_FLOAT32, 0) F34(CHR_FLOAT32, 1) F34(CHR_BFLOAT16, 0) F34(CHR_BFLOAT16, 1)
#undef F34
    }
    free_sets(S);
}

// k_tree_static against the product kernel on the same leaves: bit-identical (f32 and bf16 SUM)
static bool focus34_check() {
    const size_t nvec = (size_t)(3 << 20) / 16 + 37;
    Sets S = make_sets(17, nvec, 1);
    chr::u32x4 *o1, *o2;
    CK(hipMalloc(&o1, nvec * 16));
    CK(hipMalloc(&o2, nvec * 16));
    bool ok = true;
    for (int kind = 0; kind < 2 && ok; ++kind) {
        chr::TreeArgs a{};
        auto& b = S.bufs[0];
        a.nseg = 1;
        a.nl = 8;
        for (int j = 0; j < chr::kMaxTreeSegs; ++j) a.block0[j] = j ? ~0u : 0;
        chr::TreeSeg& g = a.seg[0];
        for (int l = 0; l < 8; ++l) g.leaves[l] = (const chr::u32x4*)b[l];
        g.nvec = nvec;
        g.comb = kC4Comb;
        g.swaps = 0;
        const uint32_t t1 = (uint32_t)((nvec + 63) / 64);
        a.xfull[0] = chr::xcd_full(t1, 0);
        g.out = o1;
        if (kind == 0) {
            hipLaunchKernelGGL((chr::k_reduce_tree<CHR_FLOAT32, CHR_SUM, 8, 1, true, 64>), dim3(t1), dim3(64), 0, 0, a);
            g.out = o2;
            hipLaunchKernelGGL((k_tree_static<CHR_FLOAT32, CHR_SUM, 8, kC4Comb>), dim3(t1), dim3(64), 0, 0, a);
        } else {
            hipLaunchKernelGGL((chr::k_reduce_tree<CHR_BFLOAT16, CHR_SUM, 8, 1, true, 64>), dim3(t1), dim3(64), 0, 0, a);
            g.out = o2;
            hipLaunchKernelGGL((k_tree_static<CHR_BFLOAT16, CHR_SUM, 8, kC4Comb>), dim3(t1), dim3(64), 0, 0, a);
        }
        CK(hipDeviceSynchronize());
        std::vector<uint32_t> h1(nvec * 4), h2(nvec * 4);
        CK(hipMemcpy(h1.data(), o1, nvec * 16, hipMemcpyDeviceToHost));
        CK(hipMemcpy(h2.data(), o2, nvec * 16, hipMemcpyDeviceToHost));
        size_t diff = 0, diff_nan = 0;  // differing 16-bit halves (bf16) / words (f32), and those where both are NaN
        for (size_t w = 0; w < h1.size(); ++w) {
            if (h1[w] == h2[w]) continue;
            if (kind == 0) {
                ++diff;
                diff_nan += ((h1[w] & 0x7F800000u) == 0x7F800000u && (h1[w] & 0x7FFFFFu)) &&
                            ((h2[w] & 0x7F800000u) == 0x7F800000u && (h2[w] & 0x7FFFFFu));
                continue;
            }
            for (int hf = 0; hf < 2; ++hf) {
                const uint32_t a1 = (h1[w] >> (16 * hf)) & 0xFFFFu, a2 = (h2[w] >> (16 * hf)) & 0xFFFFu;
                if (a1 == a2) continue;
                ++diff;
                diff_nan += ((a1 & 0x7F80u) == 0x7F80u && (a1 & 0x7Fu)) && ((a2 & 0x7F80u) == 0x7F80u && (a2 & 0x7Fu));
            }
        }
        ok = diff == diff_nan;  // only NaN payloads may differ (operand order of a commuted add)
        std::printf("{\"focus34_check\": %d, \"bit_identical\": %s, \"differing\": %zu, \"differing_both_nan\": %zu}\n",
                    kind, diff ? "false" : "true", diff, diff_nan);
    }
    CK(hipFree(o1));
    CK(hipFree(o2));
    free_sets(S);
    return ok;
}

// ---- focus21: back-to-back tree launches with the AQL barrier bit cleared ----------------------
// hipExtAnyOrderLaunch lets the packet processor start launch i+1 while launch i drains; the flat
// plan's consecutive slice evaluations touch disjoint memory, so only the ramp/drain gap is at stake.
__global__ void k_spin_write(unsigned* p, unsigned v, long long ticks) {
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
    if (threadIdx.x == 0) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void k_read_to(const unsigned* p, unsigned* out) {
    if (threadIdx.x == 0) out[0] = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// What an any-order launch still waits for: (a) the kernel before it on the same stream, (b) an
// event wait (barrier-AND packet) before it.  Prints the value the reader saw (1 = it waited).
static void any_order_semantics() {
    unsigned *flag, *out;
    CK(hipMalloc(&flag, 256));
    CK(hipMalloc(&out, 256));
    hipStream_t sa, sb;
    CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    for (uint32_t fl : {0u, (uint32_t)hipExtAnyOrderLaunch}) {
        for (int r = 0; r < 3; ++r) {
            CK(hipMemset(flag, 0, 256));
            CK(hipMemset(out, 0xff, 256));
            CK(hipDeviceSynchronize());
            hipLaunchKernelGGL(k_spin_write, dim3(1), dim3(64), 0, sa, flag, 1u, 20000ll);  // ~200 us at 100 MHz
            hipExtLaunchKernelGGL(k_read_to, dim3(1), dim3(64), 0, sa, nullptr, nullptr, fl, (const unsigned*)flag, out);
            CK(hipStreamSynchronize(sa));
            unsigned same = 0;
            CK(hipMemcpy(&same, out, 4, hipMemcpyDeviceToHost));
            CK(hipMemset(flag, 0, 256));
            CK(hipMemset(out, 0xff, 256));
            CK(hipDeviceSynchronize());
            hipLaunchKernelGGL(k_spin_write, dim3(1), dim3(64), 0, sa, flag, 1u, 20000ll);
            CK(hipEventRecord(ev, sa));
            CK(hipStreamWaitEvent(sb, ev, 0));
            hipExtLaunchKernelGGL(k_read_to, dim3(1), dim3(64), 0, sb, nullptr, nullptr, fl, (const unsigned*)flag, out);
            CK(hipDeviceSynchronize());
            unsigned cross = 0;
            CK(hipMemcpy(&cross, out, 4, hipMemcpyDeviceToHost));
            std::printf("semantics flags=%u rep=%d same-stream reader saw %u, after event wait saw %u\n", fl, r, same, cross);
        }
    }
    std::fflush(stdout);
    CK(hipEventDestroy(ev));
    CK(hipStreamDestroy(sa));
    CK(hipStreamDestroy(sb));
    CK(hipFree(flag));
    CK(hipFree(out));
}

template <int U>
static double tree8x2_time_flags(Sets& S, size_t nvec, int sets, unsigned lds, uint32_t cs, uint32_t flags) {
    return time_launches([&](int i) {
        chr::TreeArgs a{};
        const auto& b = S.bufs[i % sets];
        a.nseg = 2;
        a.nl = 8;
        a.xrun = cs;
        const uint32_t trips = (uint32_t)((nvec + 64 * U - 1) / (64 * U));
        for (int j = 0; j < chr::kMaxTreeSegs; ++j) {
            a.block0[j] = j < 2 ? j * trips : ~0u;
            a.xfull[j] = j < 2 ? chr::xcd_full(trips, cs) : 0;
        }
        const int comb[8] = {0, 1, 1, 1, 0, 1, 1, 2};
        for (int t2 = 0; t2 < 2; ++t2) {
            chr::TreeSeg& g = a.seg[t2];
            for (int l = 0; l < 8; ++l) g.leaves[l] = (const chr::u32x4*)b[9 * t2 + l];
            g.out = (chr::u32x4*)b[9 * t2 + 8];
            g.nvec = nvec;
            g.comb = 0;
            for (int l = 0; l < 8; ++l) g.comb |= (uint32_t)comb[l] << (2 * l);
            g.swaps = 0;
        }
        hipExtLaunchKernelGGL((chr::k_reduce_tree<CHR_FLOAT32, CHR_SUM, 8, U, true, 64>), dim3(2 * trips), dim3(64), lds,
                              0, nullptr, nullptr, flags, a);
    }, 64);
}

// ---- focus22: where a tree launch loses time against its steady rate -------------------------
// The product's 8-leaf tree body (k_reduce_tree<f32, SUM, 8, U, nt, 64>, C4's program) with each
// workgroup's start and end (after its stores are acknowledged) on the 100 MHz wall clock and its
// XCC.  Launches run back to back on one stream, as the flat plan's slice evaluations do on a
// rank's compute stream; from the stamps: ramp (first start -> steady completion rate), tail
// (95 % done -> last end), per-XCD finish spread and the bubble between consecutive launches.
// SAUX: the root's store. -1 = the product's (global_store ... nt); >= 0 = a buffer store with that
// cache-policy aux (gfx950 CPol: sc0 = 1, nt = 2, sc1 = 16); -2 = no store (diagnostic: what the
// end-of-kernel gap costs without dirty lines to write back; the result is not written).
template <int U, int SAUX = -1>
__global__ __launch_bounds__(64) void k_tree_stamped(chr::TreeArgs a, unsigned long long* st) {
    const unsigned long long t0 = wall_clock64();
    const uint32_t b = blockIdx.x, xrun = a.xrun;
    int s = 0;
    uint32_t b0 = 0, xfull = a.xfull[0];
#pragma unroll
    for (int j = 1; j < chr::kMaxTreeSegs; ++j)
        if (b >= a.block0[j]) {
            s = j;
            b0 = a.block0[j];
            xfull = a.xfull[j];
        }
    const chr::TreeSeg& g = a.seg[s];
    const size_t trip = chr::xcd_trip(b - b0, xfull, xrun);
    const size_t base = trip * 64 * U + threadIdx.x;
    if ((trip + 1) * 64 * U <= g.nvec) {
        chr::u32x4 x[8][U];
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int u = 0; u < U; ++u) x[j][u] = chr::ld<true>(&g.leaves[j][base + (size_t)u * 64]);
        __builtin_amdgcn_sched_barrier(0);
        chr::u32x4 r[U];
        chr::tree_eval<chr::u32x4, 8, U, chr::VecOp<CHR_FLOAT32, CHR_SUM>>(x, r, g.comb, g.swaps);
        if constexpr (SAUX == -1) {
#pragma unroll
            for (int u = 0; u < U; ++u) chr::st<true>(&g.out[base + (size_t)u * 64], r[u]);
        } else if constexpr (SAUX >= 0) {
            const __amdgpu_buffer_rsrc_t ro =
                __builtin_amdgcn_make_buffer_rsrc((void*)(g.out + trip * 64 * U), 0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
            for (int u = 0; u < U; ++u)
                __builtin_amdgcn_raw_buffer_store_b128(r[u], ro, (unsigned)((threadIdx.x + u * 64) * 16), 0, SAUX);
        } else {
            if (r[0][0] == 0x7fc00001u && r[0][1] == 0x7fc00002u) g.out[base] = r[0];
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t1 = wall_clock64();
    if (threadIdx.x == 0) {
        st[3 * (size_t)b] = t0;
        st[3 * (size_t)b + 1] = t1;
        st[3 * (size_t)b + 2] = __smid();
    }
}

template <int SAUX = -1>
static void focus22(size_t piece, int sets, int cap, int nlaunch, uint32_t flags = 0, const char* label = "product",
                    bool synced_too = true) {
    constexpr int U = 1;
    const size_t nvec = piece / 16;
    Sets S = make_sets(17, nvec, sets);
    uint32_t cs = 0;
    while (((size_t)2 << cs) * (64 * U * 16) <= (size_t)512 * 1024 && cs < 16) ++cs;
    const uint32_t trips = (uint32_t)((nvec + 64 * U - 1) / (64 * U));
    const size_t grid = 2 * (size_t)trips;
    unsigned long long* st = nullptr;
    CK(hipMalloc(&st, 3 * grid * nlaunch * sizeof(unsigned long long)));
    int khz = 0;
    CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    const double us_per_tick = 1e3 / khz;
    auto args = [&](int i) {
        chr::TreeArgs a{};
        const auto& bb = S.bufs[i % sets];
        a.nseg = 2;
        a.nl = 8;
        a.xrun = cs;
        for (int j = 0; j < chr::kMaxTreeSegs; ++j) {
            a.block0[j] = j < 2 ? j * trips : ~0u;
            a.xfull[j] = j < 2 ? chr::xcd_full(trips, cs) : 0;
        }
        const int comb[8] = {0, 1, 1, 1, 0, 1, 1, 2};
        for (int t2 = 0; t2 < 2; ++t2) {
            chr::TreeSeg& g = a.seg[t2];
            for (int l = 0; l < 8; ++l) g.leaves[l] = (const chr::u32x4*)bb[9 * t2 + l];
            g.out = (chr::u32x4*)bb[9 * t2 + 8];
            g.nvec = nvec;
            g.comb = 0;
            for (int l = 0; l < 8; ++l) g.comb |= (uint32_t)comb[l] << (2 * l);
            g.swaps = 0;
        }
        return a;
    };
    const unsigned lds = lds_for_cap(cap);
    for (int mode = 0; mode < (synced_too ? 2 : 1); ++mode) {  // 0: back to back on one stream; 1: host sync between
        for (int i = 0; i < 4; ++i)
            hipExtLaunchKernelGGL(k_tree_stamped<U, SAUX>, dim3((unsigned)grid), dim3(64), lds, 0, nullptr, nullptr, flags,
                                  args(i), st);
        CK(hipDeviceSynchronize());
        std::vector<hipEvent_t> ev(nlaunch + 1);
        for (auto& e : ev) CK(hipEventCreate(&e));
        CK(hipEventRecord(ev[0], 0));
        for (int i = 0; i < nlaunch; ++i) {
            hipExtLaunchKernelGGL(k_tree_stamped<U, SAUX>, dim3((unsigned)grid), dim3(64), lds, 0, nullptr, nullptr, flags,
                                  args(i + 4), st + 3 * grid * i);
            CK(hipEventRecord(ev[i + 1], 0));
            if (mode == 1) CK(hipEventSynchronize(ev[i + 1]));
        }
        CK(hipDeviceSynchronize());
        std::vector<unsigned long long> h(3 * grid * nlaunch);
        CK(hipMemcpy(h.data(), st, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        const double bytes = 2.0 * 9 * piece;
        unsigned long long prev_end = 0;
        for (int i = 0; i < nlaunch; ++i) {
            const unsigned long long* p = h.data() + 3 * grid * i;
            unsigned long long tmin = ~0ull, tmax = 0, smin = ~0ull;
            std::vector<unsigned long long> ends(grid);
            unsigned long long xend[16] = {}, xstart[16];
            for (auto& x : xstart) x = ~0ull;
            for (size_t w = 0; w < grid; ++w) {
                const unsigned long long t0 = p[3 * w], t1 = p[3 * w + 1];
                const unsigned xcc = (unsigned)(p[3 * w + 2] >> 6) & 15u;  // __smid: XCC | SE (2 bits) | CU (4 bits)
                tmin = std::min(tmin, t0);
                tmax = std::max(tmax, t1);
                smin = std::min(smin, t1);
                ends[w] = t1;
                xend[xcc] = std::max(xend[xcc], t1);
                xstart[xcc] = std::min(xstart[xcc], t0);
            }
            std::sort(ends.begin(), ends.end());
            auto at = [&](double f) { return (ends[(size_t)std::min<double>(grid - 1, f * grid)] - tmin) * us_per_tick; };
            const double span = (tmax - tmin) * us_per_tick;
            // steady rate: workgroups completed between 20 % and 80 % over that time
            const double t20 = at(0.2), t80 = at(0.8);
            const double ideal = (t80 - t20) / 0.6;
            double xe_min = 1e30, xe_max = 0, xs_max = 0;
            for (int x = 0; x < 16; ++x) {
                if (!xend[x]) continue;
                xe_min = std::min(xe_min, (xend[x] - tmin) * us_per_tick);
                xe_max = std::max(xe_max, (xend[x] - tmin) * us_per_tick);
                xs_max = std::max(xs_max, (xstart[x] - tmin) * us_per_tick);
            }
            float ms = 0;
            CK(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
            std::printf("{\"focus22\": \"%s\", \"mode\": \"%s\", \"piece_mib\": %zu, \"sets\": %d, \"cap\": %d, \"launch\": %d, "
                        "\"event_us\": %.2f, \"span_us\": %.2f, \"gap_from_prev_us\": %.2f, \"ideal_us\": %.2f, "
                        "\"first_end_us\": %.2f, \"t5\": %.2f, \"t20\": %.2f, \"t50\": %.2f, \"t80\": %.2f, \"t95\": %.2f, "
                        "\"t99\": %.2f, \"xcd_first_start_max_us\": %.2f, \"xcd_end_min_us\": %.2f, \"xcd_end_max_us\": %.2f, "
                        "\"frac_event\": %.4f, \"frac_span\": %.4f, \"frac_steady\": %.4f}\n",
                        label, mode ? "synced" : "back_to_back", piece >> 20, sets, cap, i, ms * 1e3, span,
                        prev_end ? (tmin - prev_end) * us_per_tick : -1.0, ideal, (smin - tmin) * us_per_tick, at(0.05),
                        t20, at(0.5), t80, at(0.95), at(0.99), xs_max, xe_min, xe_max, bytes / (ms * 1e-3) / 8e12,
                        bytes / (span * 1e-6) / 8e12, bytes / (ideal * 1e-6) / 8e12);
            prev_end = tmax;
        }
        std::fflush(stdout);
        for (auto& e : ev) CK(hipEventDestroy(e));
    }
    CK(hipFree(st));
    free_sets(S);
}

template <bool NT, int BL, int U>
static double vec1_time(Sets& S, size_t nvec, int sets, unsigned lds, uint32_t cs) {
    const unsigned G = (unsigned)(nvec / (BL * U));
    return time_launches([&](int i) {
        auto& b = S.bufs[i % sets];
        chr::VecArgs v{};
        v.out = (chr::u32x4*)b[0];
        v.acc = (const chr::u32x4*)b[0];
        v.ins[0] = (const chr::u32x4*)b[1];
        v.nvec = nvec;
        v.xrun = cs;
        v.xfull = chr::xcd_full(G, cs);
        hipLaunchKernelGGL((chr::k_reduce_vec<CHR_FLOAT32, CHR_SUM, 1, U, NT, NT, BL>), dim3(G), dim3(BL), lds, 0, v);
    }, 200);
}

static void focus19_vec(size_t bytes, int sets) {
    const size_t nvec = bytes / 16;
    Sets S = make_sets(1, nvec, sets);
    uint32_t cs = 0;
    while (((size_t)2 << cs) * (64 * 4 * 16) <= (size_t)256 * 1024 && cs < 16) ++cs;
    char name[128];
    std::snprintf(name, sizeof name, "vec m=1 plain BL=256 sets=%d", sets);
    report(name, 1, bytes, vec1_time<false, 256, 4>(S, nvec, sets, 0, 0));
    std::snprintf(name, sizeof name, "vec m=1 nt cap12 runs256 sets=%d", sets);
    report(name, 1, bytes, vec1_time<true, 64, 4>(S, nvec, sets, lds_for_cap(12), cs));
    free_sets(S);
}


// ---- focus24: the C2 launch's timeline, and a persistent variant that balances the XCDs -------
// The product's C2 body (k_reduce_vec<f32, SUM, 1, 4, nt, ACC0, 64>, 12 per CU, 256 KiB XCD runs)
// with each workgroup's start and end stamped (as focus22).  The hardware hands every XCD exactly
// 1/8 of a grid's workgroups, so an XCD that streams slower finishes last and the others idle: the
// tail.  PERSIST: a grid of resident workgroups that take runs of R trips from a per-launch counter
// (one vector atomic per run, the next run's index fetched while the current run streams), so the
// XCDs share the work until it runs out.  Counters are one per launch, zeroed once up front.
template <bool PERSIST, int R, int MAPV = 0>
__global__ __launch_bounds__(64) void k_c2_stamped(chr::VecArgs a, unsigned* ctr, unsigned long long* st) {
    constexpr int U = 4, BL = 64;
    const unsigned long long t0 = wall_clock64();
    chr::u32x4* const out = a.out;
    const chr::u32x4* const accp = a.acc;
    const chr::u32x4* const in0 = a.ins[0];
    const size_t nvec = a.nvec;
    const uint32_t ntrips = (uint32_t)(nvec / (BL * U));
    auto body = [&](size_t trip) {
        const size_t base = trip * BL * U + threadIdx.x;
        chr::u32x4 acc[U], x[U];
        acc[0] = chr::ld<false>(&accp[base]);
#pragma unroll
        for (int u = 1; u < U; ++u) acc[u] = chr::ld<true>(&accp[base + (size_t)u * BL]);
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = chr::ld<true>(&in0[base + (size_t)u * BL]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] = chr::apply_vec<CHR_FLOAT32, CHR_SUM>(x[u], acc[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) chr::st<true>(&out[base + (size_t)u * BL], acc[u]);
    };
    if constexpr (!PERSIST) {
        chr::pin_sgpr(out, accp, nvec, a.xrun, a.xfull);
        chr::pin_sgpr(in0);
        if constexpr (MAPV == 3) {
            // weighted runs: in the last round of runs each odd XCD hands the last h trips of its run to
            // the even XCD below it (grid = 8 x (runs_per_xcd x C + h); only whole-run grids)
            const uint32_t h = *ctr, cs = a.xrun, C = 1u << cs, x = blockIdx.x & 7u, i = blockIdx.x >> 3;
            const uint32_t RPX = ntrips >> (cs + 3), L = (RPX - 1) << cs;
            size_t trip;
            if (i < L) {
                trip = ((((size_t)(i >> cs)) * 8u + x) << cs) | (i & (C - 1u));
            } else {
                const uint32_t t = i - L;
                const size_t g0 = (size_t)(RPX - 1) * 8u + x;
                if ((x & 1u) == 0) {
                    if (t < C) trip = (g0 << cs) | t;
                    else if (t < C + h) trip = ((g0 + 1) << cs) | (C - h + (t - C));
                    else trip = ~(size_t)0;
                } else {
                    trip = t < C - h ? (g0 << cs) | t : ~(size_t)0;
                }
            }
            if (trip != ~(size_t)0) body(trip);
        } else {
            // MAPV 2: each XCD takes its neighbour's runs (block b does block b ^ 1's trip)
            const uint32_t bb = MAPV == 2 ? (blockIdx.x ^ 1u) : blockIdx.x;
            const size_t trip = chr::xcd_trip(bb, a.xfull, a.xrun);
            if ((trip + 1) * BL * U <= nvec) body(trip);
        }
    } else {
        const uint32_t nruns = (ntrips + R - 1) / R;
        auto grab = [&]() -> uint32_t {
            uint32_t v = 0;
            if (threadIdx.x == 0) v = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
        };
        uint32_t run = grab();
        while (run < nruns) {
            const uint32_t next = grab();
            for (int r = 0; r < R; ++r) {
                const uint32_t trip = run * R + r;
                if (trip < ntrips) body(trip);
            }
            run = next;
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t1 = wall_clock64();
    if (threadIdx.x == 0) {
        st[3 * (size_t)blockIdx.x] = t0;
        st[3 * (size_t)blockIdx.x + 1] = t1;
        st[3 * (size_t)blockIdx.x + 2] = __smid();
    }
}

template <bool PERSIST, int R, int MAPV = 0>
static void focus24_one(Sets& S, size_t nvec, int sets, int cap, unsigned pgrid, int nlaunch, const char* label,
                        int run_kib = 256) {
    constexpr int U = 4, BL = 64;
    const unsigned trips = (unsigned)(nvec / (BL * U));
    uint32_t cs = 0;
    while (((size_t)2 << cs) * (BL * U * 16) <= (size_t)run_kib * 1024 && cs < 16) ++cs;
    // MAPV 3: pgrid carries h, the trips each odd XCD hands over in the last round
    const unsigned grid = PERSIST ? pgrid : MAPV == 3 ? trips + 8u * pgrid : trips;
    unsigned long long* st = nullptr;
    unsigned* ctr = nullptr;
    const int total = nlaunch + 4;
    CK(hipMalloc(&st, 3 * (size_t)grid * total * sizeof(unsigned long long)));
    CK(hipMalloc(&ctr, total * sizeof(unsigned)));
    CK(hipMemset(ctr, 0, total * sizeof(unsigned)));
    if (MAPV == 3) {
        std::vector<unsigned> hv(total, pgrid);
        CK(hipMemcpy(ctr, hv.data(), total * sizeof(unsigned), hipMemcpyHostToDevice));
    }
    int khz = 0;
    CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    const double us_per_tick = 1e3 / khz;
    const unsigned lds = lds_for_cap(cap);
    auto launch = [&](int i) {
        auto& b = S.bufs[i % sets];
        chr::VecArgs v{};
        v.out = (chr::u32x4*)b[0];
        v.acc = (const chr::u32x4*)b[0];
        v.ins[0] = (const chr::u32x4*)b[1];
        v.nvec = nvec;
        v.xrun = cs;
        v.xfull = chr::xcd_full(trips, cs);
        hipLaunchKernelGGL((k_c2_stamped<PERSIST, R, MAPV>), dim3(grid), dim3(BL), lds, 0, v, ctr + i,
                           st + 3 * (size_t)grid * i);
    };
    for (int i = 0; i < 4; ++i) launch(i);
    CK(hipDeviceSynchronize());
    std::vector<hipEvent_t> ev(nlaunch + 1);
    for (auto& e : ev) CK(hipEventCreate(&e));
    CK(hipEventRecord(ev[0], 0));
    for (int i = 0; i < nlaunch; ++i) {
        launch(4 + i);
        CK(hipEventRecord(ev[i + 1], 0));
    }
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> h(3 * (size_t)grid * total);
    CK(hipMemcpy(h.data(), st, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    const double bytes = 3.0 * nvec * 16;
    double sum_ms = 0;
    unsigned long long prev_end = 0;
    for (int i = 0; i < nlaunch; ++i) {
        const unsigned long long* p = h.data() + 3 * (size_t)grid * (4 + i);
        unsigned long long tmin = ~0ull, tmax = 0, smin = ~0ull, xend[16] = {};
        std::vector<unsigned long long> ends(grid);
        for (size_t w = 0; w < grid; ++w) {
            const unsigned long long t0 = p[3 * w], t1 = p[3 * w + 1];
            const unsigned xcc = (unsigned)(p[3 * w + 2] >> 6) & 15u;
            tmin = std::min(tmin, t0);
            tmax = std::max(tmax, t1);
            smin = std::min(smin, t1);
            ends[w] = t1;
            xend[xcc] = std::max(xend[xcc], t1);
        }
        std::sort(ends.begin(), ends.end());
        auto at = [&](double f) { return (ends[(size_t)std::min<double>(grid - 1, f * grid)] - tmin) * us_per_tick; };
        double xe_min = 1e30, xe_max = 0;
        for (int x = 0; x < 16; ++x) {
            if (!xend[x]) continue;
            xe_min = std::min(xe_min, (xend[x] - tmin) * us_per_tick);
            xe_max = std::max(xe_max, (xend[x] - tmin) * us_per_tick);
        }
        float ms = 0;
        CK(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
        sum_ms += ms;
        const double span = (tmax - tmin) * us_per_tick;
        char xe[256];
        int o = 0;
        for (int x = 0; x < 8; ++x)
            o += std::snprintf(xe + o, sizeof xe - o, "%s%.2f", x ? ", " : "", xend[x] ? (xend[x] - tmin) * us_per_tick : -1.0);
        std::printf("{\"focus24\": \"%s\", \"cap\": %d, \"grid\": %u, \"launch\": %d, \"event_us\": %.2f, \"span_us\": %.2f, "
                    "\"gap_from_prev_us\": %.2f, \"first_end_us\": %.2f, \"t50\": %.2f, \"t95\": %.2f, \"t99\": %.2f, "
                    "\"xcd_end_min_us\": %.2f, \"xcd_end_max_us\": %.2f, \"xcd_end_us\": [%s], \"frac_event\": %.4f, "
                    "\"frac_span\": %.4f}\n",
                    label, cap, grid, i, ms * 1e3, span, prev_end ? (tmin - prev_end) * us_per_tick : -1.0,
                    (smin - tmin) * us_per_tick, at(0.5), at(0.95), at(0.99), xe_min, xe_max, xe,
                    bytes / (ms * 1e-3) / 8e12, bytes / (span * 1e-6) / 8e12);
        prev_end = tmax;
    }
    std::printf("{\"focus24_summary\": \"%s\", \"cap\": %d, \"grid\": %u, \"mean_event_us\": %.2f, \"frac\": %.4f}\n",
                label, cap, grid, sum_ms * 1e3 / nlaunch, bytes / (sum_ms / nlaunch * 1e-3) / 8e12);
    std::fflush(stdout);
    for (auto& e : ev) CK(hipEventDestroy(e));
    CK(hipFree(st));
    CK(hipFree(ctr));
}

static void focus24(int rounds) {
    const size_t nvec = (64u << 20) / 16;
    const int sets = 16;
    Sets S = make_sets(1, nvec, sets);
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    for (int r = 0; r < rounds; ++r) {
        focus24_one<false, 1>(S, nvec, sets, 12, 0, 16, "product_shape");
        // resident grid: 11 per CU at cap 12 (census), runs of R trips (4 KiB per operand per trip)
        focus24_one<true, 4>(S, nvec, sets, 12, (unsigned)ncu * 11, 16, "persist_r4_grid11pcu");
        focus24_one<true, 16>(S, nvec, sets, 12, (unsigned)ncu * 11, 16, "persist_r16_grid11pcu");
        focus24_one<true, 4>(S, nvec, sets, 0, (unsigned)ncu * 16, 16, "persist_r4_uncapped_grid16pcu");
        focus24_one<true, 1>(S, nvec, sets, 12, (unsigned)ncu * 11, 16, "persist_r1_grid11pcu");
    }
    free_sets(S);
}

int main(int argc, char** argv) {
    check();
    if (argc > 1 && std::string(argv[1]) == "layout") {
        layout_mode();
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus24") {  // C2 timeline: the XCD tail; persistent balancing
        focus24(argc > 2 ? std::atoi(argv[2]) : 2);
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus26") {  // does the late XCD set follow the XCD or the addresses?
        const size_t nvec = (64u << 20) / 16;
        Sets S = make_sets(1, nvec, 16);
        for (int r = 0; r < (argc > 2 ? std::atoi(argv[2]) : 2); ++r) {
            focus24_one<false, 1, 0>(S, nvec, 16, 12, 0, 32, "runs256");
            focus24_one<false, 1, 2>(S, nvec, 16, 12, 0, 32, "runs256_neighbour");
            focus24_one<false, 1, 0>(S, nvec, 16, 12, 0, 32, "identity", 0);
            focus24_one<false, 1, 0>(S, nvec, 16, 12, 0, 32, "runs1024", 1024);
        }
        free_sets(S);
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus27") {  // weighted last round: odd XCDs hand h trips to even ones
        const size_t nvec = (64u << 20) / 16;
        Sets S = make_sets(1, nvec, 16);
        for (int r = 0; r < (argc > 2 ? std::atoi(argv[2]) : 2); ++r) {
            focus24_one<false, 1, 0>(S, nvec, 16, 12, 0, 32, "runs256");
            for (unsigned h : {16u, 32u, 48u}) {
                char lab[64];
                std::snprintf(lab, sizeof lab, "runs256_odd_hand_%u", h);
                focus24_one<false, 1, 3>(S, nvec, 16, 12, h, 32, lab);
            }
        }
        free_sets(S);
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus28") {  // is the odd XCDs' lag a fixed delay or a rate?
        for (size_t mib : {16, 64, 256}) {
            const size_t nvec = (mib << 20) / 16;
            const int sets = (int)std::max<size_t>(2, (2048 / (2 * mib)));
            Sets S = make_sets(1, nvec, sets);
            char lab[64];
            std::snprintf(lab, sizeof lab, "runs256_%zuMiB", mib);
            focus24_one<false, 1, 0>(S, nvec, sets, 12, 0, 24, lab);
            free_sets(S);
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus29") {  // the odd-XCD lag with cache-resident (warm) operands
        for (int sets : {16, 1}) {  // 2 GiB rotation (HBM-cold) vs one 128 MiB set (Infinity Cache)
            const size_t nvec = (64u << 20) / 16;
            Sets S = make_sets(1, nvec, sets);
            char lab[64];
            std::snprintf(lab, sizeof lab, "runs256_sets%d", sets);
            for (int r = 0; r < 2; ++r) focus24_one<false, 1, 0>(S, nvec, sets, 12, 0, 24, lab);
            free_sets(S);
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus25") {  // C2 timeline only: which XCD finishes last, launch after launch
        const size_t nvec = (64u << 20) / 16;
        Sets S = make_sets(1, nvec, 16);
        for (int r = 0; r < (argc > 2 ? std::atoi(argv[2]) : 2); ++r) focus24_one<false, 1>(S, nvec, 16, 12, 0, 32, "product_shape");
        free_sets(S);
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus23") {  // what the ~4 us between back-to-back launches is
        for (int r = 0; r < 2; ++r)
            for (size_t mib : {16, 8}) {
                focus22<-1>(mib << 20, 4, 16, 8, 0, "product", false);
                focus22<-1>(mib << 20, 4, 16, 8, hipExtAnyOrderLaunch, "product_any_order", false);
                focus22<-2>(mib << 20, 4, 16, 8, 0, "no_store", false);
                focus22<2>(mib << 20, 4, 16, 8, 0, "buf_nt", false);
                focus22<0>(mib << 20, 4, 16, 8, 0, "buf_plain", false);
                focus22<19>(mib << 20, 4, 16, 8, 0, "buf_nt_sc0_sc1", false);
                focus22<18>(mib << 20, 4, 16, 8, 0, "buf_nt_sc1", false);
                focus22<3>(mib << 20, 4, 16, 8, 0, "buf_nt_sc0", false);
            }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus22") {  // timeline of C4-slice tree launches
        for (size_t mib : {16, 8, 32})
            for (int cap : {16, 12}) focus22(mib << 20, 4, cap, 8);
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus21") {  // barrier bit vs any-order launches, C4 slice shape
        any_order_semantics();
        for (int r = 0; r < 3; ++r)
            for (size_t mib : {8, 16, 32})
                for (int sets : {16, 4}) {
                    const size_t piece = mib << 20, nvec = piece / 16;
                    Sets S = make_sets(17, nvec, sets);
                    uint32_t cs = 0;
                    while (((size_t)2 << cs) * (64 * 1 * 16) <= (size_t)512 * 1024 && cs < 16) ++cs;
                    for (uint32_t fl : {0u, (uint32_t)hipExtAnyOrderLaunch}) {
                        char name[128];
                        std::snprintf(name, sizeof name, "tree8x2 U=1 cap16 %s piece=%zuMiB sets=%d",
                                      fl ? "any-order" : "ordered  ", mib, sets);
                        report_moved(name, 2.0 * 9 * piece,
                                     tree8x2_time_flags<1>(S, nvec, sets, lds_for_cap(16), cs, fl));
                    }
                    free_sets(S);
                }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus34") {  // the tree program at compile time
        if (!focus34_check()) return 1;
        for (int r = 0; r < 3; ++r) {
            for (size_t mib : {16, 8}) {
                focus34(mib << 20, 16);  // cold
                focus34(mib << 20, 2);   // warm
            }
            std::printf("--\n");
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus33") {  // second vector through LDS at the in-collective cap
        if (!focus33_check()) return 1;
        for (int r = 0; r < 3; ++r) {
            for (size_t mib : {16, 8}) {
                focus33(mib << 20, 16);  // cold
                focus33(mib << 20, 2);   // warm
            }
            std::printf("--\n");
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus32") {  // bf16 vs f32 trees: U and waves per CU
        for (int r = 0; r < 2; ++r) {
            for (size_t mib : {16, 8}) {
                focus32(mib << 20, 16);  // cold: 2.25 / 4.5 GiB rotation
                focus32(mib << 20, 2);   // warm
            }
            std::printf("--\n");
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus31") {  // page-local chunks past the translation reach
        int ncu = 0;
        CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
        for (int r = 0; r < 2; ++r) {
            focus31_m<3, 2>(1024ull << 20, 1, ncu);  // 4 GiB per launch: the cliff
            focus31_m<3, 2>(256ull << 20, 4, ncu);   // 4 GiB rotation
            focus31_m<3, 2>(256ull << 20, 1, ncu);   // 1 GiB: inside the reach (control)
            focus31_m<7, 1>(256ull << 20, 2, ncu);   // 4 GiB rotation, 8 streams
            focus31_m<1, 4>(1024ull << 20, 1, ncu);  // 2 GiB per launch
            std::printf("--\n");
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus30") {  // fatter workgroups for the 8-leaf trees
        for (int r = 0; r < 2; ++r) {
            for (size_t mib : {8, 16}) {
                focus30(mib << 20, 16);  // cold: 2.25 / 4.5 GiB rotation
                focus30(mib << 20, 2);   // warm: 288 / 576 MiB
            }
            std::printf("--\n");
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus20") {  // XCD run length for the U = 1 tree shape
        for (int r = 0; r < 2; ++r)
            for (int sets : {16, 4}) {
                const size_t piece = 16 << 20, nvec = piece / 16;
                Sets S = make_sets(17, nvec, sets);
                for (unsigned run_kib : {0u, 128u, 256u, 512u, 1024u, 2048u}) {
                    uint32_t cs = 0;
                    while (run_kib && ((size_t)2 << cs) * (64 * 1 * 16) <= (size_t)run_kib * 1024 && cs < 16) ++cs;
                    for (int cap : {12, 16, 20}) {
                        char name[128];
                        std::snprintf(name, sizeof name, "tree8x2 U=1 cap=%d run=%uKiB sets=%d", cap, run_kib, sets);
                        report_moved(name, 2.0 * 9 * piece, tree8x2_time<1, true, 64>(S, nvec, sets, lds_for_cap(cap), cs));
                    }
                }
                free_sets(S);
                std::printf("--\n");
            }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus19") {
        for (int r = 0; r < 2; ++r) {
            for (size_t mib : {2, 4, 8}) {
                focus19(mib << 20, 32);  // cold
                focus19(mib << 20, 2);   // warm (Infinity Cache)
            }
            for (size_t mib : {8, 16, 32}) {
                focus19_vec(mib << 20, 64);
                focus19_vec(mib << 20, 2);
            }
            std::printf("--\n");
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus18") {
        for (int r = 0; r < 2; ++r) {
            focus18_tree<2, 4>(128 << 20, 6, {0, 12, 16}, 0);
            focus18_tree<2, 4>(128 << 20, 6, {0, 12}, 256);
            focus18_tree<2, 2>(128 << 20, 6, {0, 12, 16}, 0);
            focus18_tree<4, 4>(64 << 20, 6, {0, 12, 16}, 512);
            focus18_tree<4, 2>(64 << 20, 6, {0, 12, 16}, 512);
            focus18_tree<4, 1>(64 << 20, 6, {0, 12, 16}, 512);
            std::printf("--\n");
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus17") {  // tree: U = 1 vs 2 under caps
        for (int r = 0; r < 2; ++r) {
            focus11_tree<2>(16 << 20, 16, 1, {0, 12, 16});
            focus11_tree<1>(16 << 20, 16, 1, {0, 12, 16, 20});
            focus11_tree<2>(16 << 20, 4, 1, {0, 12, 16});
            focus11_tree<1>(16 << 20, 4, 1, {0, 12, 16, 20});
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus16") {  // the cold (large rotation) side of U = 1
        for (int r = 0; r < 2; ++r) {
            focus12_mu<7, 2>(256 << 20, 8, {0, 16});
            focus12_mu<7, 1>(256 << 20, 8, {0, 12, 16});
            focus12_mu<4, 2>(256 << 20, 8, {0, 16});
            focus12_mu<4, 1>(256 << 20, 8, {0, 12, 16});
            focus12_mu<7, 2>(64 << 20, 8, {0, 16});
            focus12_mu<7, 1>(64 << 20, 8, {0, 16});
            std::printf("--\n");
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus15") {  // m = 2 and 3: U x cap
        for (int r = 0; r < 2; ++r) {
            focus12_mu<2, 4>(64 << 20, 8, {0, 12, 16});
            focus12_mu<2, 2>(64 << 20, 8, {0, 12, 16});
            focus12_mu<2, 1>(64 << 20, 8, {0, 12, 16});
            focus12_mu<3, 2>(64 << 20, 8, {0, 12, 16});
            focus12_mu<3, 1>(64 << 20, 8, {0, 12, 16});
            focus12_mu<3, 2>(256 << 20, 2, {0, 12, 16});
            focus12_mu<3, 1>(256 << 20, 2, {0, 12, 16});
            focus12_mu<6, 2>(64 << 20, 4, {0, 12, 16});
            focus12_mu<6, 1>(64 << 20, 4, {0, 12, 16});
            std::printf("--\n");
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus14") {  // U = 1 vs 2 for wide fan-in, with and without the cap
        for (int r = 0; r < 2; ++r) {
            focus12_mu<5, 2>(64 << 20, 4, {0, 12});
            focus12_mu<5, 1>(64 << 20, 4, {0, 12, 16});
            focus12_mu<7, 2>(64 << 20, 4, {0, 12});
            focus12_mu<7, 1>(64 << 20, 4, {0, 12, 16});
            focus12_mu<7, 2>(256 << 20, 1, {0, 12});
            focus12_mu<7, 1>(256 << 20, 1, {0, 12, 16});
            focus12_mu<8, 2>(128 << 20, 2, {0, 12});
            focus12_mu<8, 1>(128 << 20, 2, {0, 12, 16});
            focus12_mu<4, 2>(128 << 20, 2, {0, 12});
            focus12_mu<4, 1>(128 << 20, 2, {0, 12, 16});
            std::printf("--\n");
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus13") {
        focus13(3);
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus12") {
        for (int r = 0; r < 2; ++r) {
            focus12_mu<1, 2>(64 << 20, 16, {0, 12, 16, 20, 24});
            focus12_mu<1, 4>(64 << 20, 16, {0, 10, 11, 12, 13, 14});
            focus12_mu<1, 8>(64 << 20, 16, {0, 6, 8, 10, 12});
            focus12_mu<3, 2>(256 << 20, 1, {0, 10, 12, 14, 16});
            focus12_mu<3, 4>(256 << 20, 1, {0, 6, 8, 10, 12});
            focus12_mu<7, 2>(64 << 20, 4, {0, 8, 10, 12, 16});
            focus12_mu<7, 1>(64 << 20, 4, {0, 12, 16, 20, 24});
            std::printf("--\n");
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus11") {
        focus11_vec(64 << 20, 16, 2);    // C2
        focus11_tree(16 << 20, 16, 2);   // C4 slice, cold rotation
        focus11_tree(16 << 20, 4, 2);    // warm translations
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus10") {
        focus10(16 << 20, 16, 2);  // C4 slice at the automatic depth, 4.5 GiB rotation (cold)
        focus10(16 << 20, 4, 2);   // 1.1 GiB rotation (warm translations)
        focus10(32 << 20, 8, 1);
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus9") {  // finer runs: 128 KiB .. 1 MiB per XCD
        const std::vector<unsigned> c4 = {1u, 32u, 64u, 128u, 256u}, c2 = {1u, 64u, 128u, 256u, 512u};
        focus8_m<1, 4>(64 << 20, 16, 3, c4);
        focus8_m<1, 4>(64 << 20, 64, 3, c4);
        focus8_m<3, 2>(256 << 20, 1, 3, c2);
        focus8_m<3, 2>(256 << 20, 8, 3, c2);
        focus8_m<7, 2>(64 << 20, 4, 3, c2);
        focus8_m<7, 2>(64 << 20, 16, 3, c2);
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus8") {
        focus8_m<1, 4>(64 << 20, 16, 2);   // C2: 2 GiB rotation (warm translations)
        focus8_m<1, 4>(64 << 20, 64, 2);   // C2 shape, 8 GiB rotation (cold)
        focus8_m<3, 2>(256 << 20, 1, 2);   // m = 3, 1.25 GiB (warm)
        focus8_m<3, 2>(256 << 20, 8, 2);   // m = 3, 10 GiB (cold)
        focus8_m<7, 2>(64 << 20, 16, 1);   // the tree-like 9-stream shape, 8 GiB (cold)
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus7") {
        focus7_m<3>(64 << 20, 8, 2);
        focus7_m<3>(256 << 20, 2, 1);
        focus7_m<7>(64 << 20, 4, 2);
        focus7_m<7>(16 << 20, 16, 1);
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus6") {
        focus6(64 << 20, 16, 2);
        focus6(1024ull << 20, 2, 1);
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus5") {
        focus5(64 << 20, 16, 3);
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus4") {
        focus4_m<1>(1024ull << 20, 1, 2);
        focus4_m<1>(64 << 20, 16, 2);
        focus4_m<3>(512ull << 20, 1, 1);
        focus4_m<3>(64 << 20, 8, 1);
        focus4_m<7>(64 << 20, 4, 1);
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus3") {
        focus3_m<1>(1024ull << 20, 1, 2);
        focus3_m<1>(64 << 20, 16, 2);
        focus3_m<3>(512ull << 20, 1, 1);
        focus3_m<3>(64 << 20, 8, 1);
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus2") {
        focus2_m<1>(64 << 20, 16, 2);
        focus2_m<1>(1024ull << 20, 1, 1);
        focus2_m<3>(64 << 20, 8, 1);
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "focus") {
        focus_m<1>(64 << 20, 16, 2);
        focus_m<1>(1024ull << 20, 1, 2);
        focus_m<3>(512ull << 20, 1, 1);
        focus_m<3>(64 << 20, 8, 1);
        focus_m<7>(64 << 20, 4, 1);
        focus_m<1>(16 << 20, 0, 1);
        return 0;
    }
    std::vector<size_t> mib;
    for (int i = 1; i < argc; ++i) mib.push_back(std::strtoul(argv[i], nullptr, 10));
    if (mib.empty()) mib = {64, 1024};
    for (size_t mb : mib) {
        run_m<1>(mb << 20);
        run_m<3>(mb << 20);
        if (mb <= 256) run_m<7>(mb << 20);
    }
    return 0;
}
