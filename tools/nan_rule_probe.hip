// nan_rule_probe -- which NaN survives a gfx950 add / multiply of two NaNs, by source-operand position.
// IEEE 754 leaves the payload open; the reference's x86 loop keeps the running value's (inout's) NaN.  One wave
// computes v_add_f32 / v_mul_f32 / v_pk_add_f32 / v_pk_mul_f32 with explicit operand positions (inline asm) on
// a = NaN payload 0x111, b = NaN payload 0x222 and prints the result's payload.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k(const uint32_t* in, uint32_t* out) {
    if (threadIdx.x) return;
    const float a = __uint_as_float(in[0]), b = __uint_as_float(in[1]);
    float r;
    asm volatile("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    out[0] = __float_as_uint(r);
    asm volatile("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(b), "v"(a));
    out[1] = __float_as_uint(r);
    asm volatile("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    out[2] = __float_as_uint(r);
    asm volatile("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(b), "v"(a));
    out[3] = __float_as_uint(r);
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 pa = {a, a}, pb = {b, b}, pr;
    asm volatile("v_pk_add_f32 %0, %1, %2" : "=v"(pr) : "v"(pa), "v"(pb));
    out[4] = __float_as_uint(pr.x);
    asm volatile("v_pk_add_f32 %0, %1, %2" : "=v"(pr) : "v"(pb), "v"(pa));
    out[5] = __float_as_uint(pr.x);
    asm volatile("v_pk_mul_f32 %0, %1, %2" : "=v"(pr) : "v"(pa), "v"(pb));
    out[6] = __float_as_uint(pr.x);
    // what plain C gives (the compiler picks the operand order)
    out[7] = __float_as_uint(a + b);
    out[8] = __float_as_uint(b + a);
}

int main() {
    uint32_t h[2] = {0x7FC00111u, 0x7F800222u}, *din, *dout, o[9];
    hipMalloc(&din, 8);
    hipMalloc(&dout, 36);
    hipMemcpy(din, h, 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, din, dout);
    hipMemcpy(o, dout, 36, hipMemcpyDeviceToHost);
    const char* names[9] = {"v_add_f32 a,b", "v_add_f32 b,a", "v_mul_f32 a,b", "v_mul_f32 b,a", "v_pk_add_f32 a,b",
                            "v_pk_add_f32 b,a", "v_pk_mul_f32 a,b", "C a+b", "C b+a"};
    std::printf("a = %08x (quiet, payload 0x111), b = %08x (signalling, payload 0x222)\n", h[0], h[1]);
    for (int i = 0; i < 9; ++i) std::printf("%-18s -> %08x  (%s)\n", names[i], o[i],
                                            (o[i] & 0x3FFFFF) == 0x111 ? "a's" : (o[i] & 0x3FFFFF) == 0x222 ? "b's" : "other");
    return 0;
}
