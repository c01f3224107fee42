// bf16_cvt_check.hip -- exhaustive check: gfx950's v_cvt_pk_bf16_f32 (what clang emits for a
// float -> __bf16 conversion) against the software RNE the kernels and the oracle use
// (f2bf in csrc/reduce_common.hpp, orc_f2bf in oracle/chiara_oracle.c), over all 2^32 f32
// bit patterns.  Prints mismatch counts per class (NaN / Inf / zero+denormal / normal) and the
// first mismatching inputs.  Build: hipcc -O3 --offload-arch=gfx950 -o tools/bf16_cvt_check
// tools/bf16_cvt_check.hip
#include <hip/hip_runtime.h>

#include <cstdio>

__device__ __forceinline__ unsigned short sw_f2bf(float f) {
    unsigned u = __float_as_uint(f);
    if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x007FFFFFu)) return (unsigned short)((u >> 16) | 0x40u);
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (unsigned short)(u >> 16);
}

__global__ void check(unsigned long long base, unsigned long long* counts, unsigned* first, unsigned* nfirst) {
    const unsigned long long i = base + (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned u = (unsigned)i;
    const float f = __uint_as_float(u);
    const unsigned short hw = __builtin_bit_cast(unsigned short, (__bf16)f);
    const unsigned short sw = sw_f2bf(f);
    if (hw != sw) {
        const unsigned e = u & 0x7F800000u, m = u & 0x007FFFFFu;
        const int cls = e == 0x7F800000u ? (m ? 0 : 1) : e == 0 ? 2 : 3;
        atomicAdd(&counts[cls], 1ull);
        const unsigned slot = atomicAdd(nfirst, 1u);
        if (slot < 16) {
            first[3 * slot] = u;
            first[3 * slot + 1] = hw;
            first[3 * slot + 2] = sw;
        }
    }
}

int main() {
    unsigned long long* counts;
    unsigned *first, *nfirst;
    hipMalloc(&counts, 4 * sizeof(unsigned long long));
    hipMalloc(&first, 48 * sizeof(unsigned));
    hipMalloc(&nfirst, sizeof(unsigned));
    hipMemset(counts, 0, 4 * sizeof(unsigned long long));
    hipMemset(nfirst, 0, sizeof(unsigned));
    const unsigned long long chunk = 1ull << 28;
    for (unsigned long long base = 0; base < (1ull << 32); base += chunk)
        hipLaunchKernelGGL(check, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, base, counts, first, nfirst);
    if (hipDeviceSynchronize() != hipSuccess) {
        std::printf("{\"error\": \"kernel failed\"}\n");
        return 1;
    }
    unsigned long long c[4];
    unsigned f[48], nf;
    hipMemcpy(c, counts, sizeof(c), hipMemcpyDeviceToHost);
    hipMemcpy(f, first, sizeof(f), hipMemcpyDeviceToHost);
    hipMemcpy(&nf, nfirst, sizeof(nf), hipMemcpyDeviceToHost);
    std::printf("{\"mismatch\": {\"nan\": %llu, \"inf\": %llu, \"zero_denormal\": %llu, \"normal\": %llu}, \"first\": [",
                c[0], c[1], c[2], c[3]);
    for (unsigned s = 0; s < (nf < 16 ? nf : 16); ++s)
        std::printf("%s[\"0x%08x\", \"0x%04x\", \"0x%04x\"]", s ? ", " : "", f[3 * s], f[3 * s + 1], f[3 * s + 2]);
    std::printf("]}\n");
    return 0;
}
