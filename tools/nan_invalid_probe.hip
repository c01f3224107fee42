// nan_invalid_probe -- what gfx950 returns where x86 (the reference's MPICH loops) returns its "default NaN":
// invalid operations (inf - inf, 0 * inf) give 0xFFC00000 / 0xFFF8000000000000 on x86 (sign set).  Also the
// subtract with a NaN second operand (x86: that NaN, sign unchanged; an add of a negated operand would flip it),
// and a lone NaN on either side (quieted, sign and payload kept on x86).  One lane; inline asm pins each
// instruction and its operand order.  Output: one line per case, result bits in hex.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define ADD32(o, a, b) asm volatile("v_add_f32 %0, %1, %2" : "=v"(o) : "v"(a), "v"(b))
#define SUB32(o, a, b) asm volatile("v_sub_f32 %0, %1, %2" : "=v"(o) : "v"(a), "v"(b))
#define MUL32(o, a, b) asm volatile("v_mul_f32 %0, %1, %2" : "=v"(o) : "v"(a), "v"(b))
#define ADD64(o, a, b) asm volatile("v_add_f64 %0, %1, %2" : "=v"(o) : "v"(a), "v"(b))
#define MUL64(o, a, b) asm volatile("v_mul_f64 %0, %1, %2" : "=v"(o) : "v"(a), "v"(b))

__global__ void k(const uint32_t* in32, const uint64_t* in64, uint32_t* o32, uint64_t* o64) {
    if (threadIdx.x) return;
    const float inf = __uint_as_float(in32[0]), ninf = __uint_as_float(in32[1]), zero = __uint_as_float(in32[2]),
                one = __uint_as_float(in32[3]), nq = __uint_as_float(in32[4]), nsn = __uint_as_float(in32[5]);
    float r;
    int i = 0;
    ADD32(r, inf, ninf); o32[i++] = __float_as_uint(r);   // 0 inf + -inf
    SUB32(r, inf, inf); o32[i++] = __float_as_uint(r);    // 1 inf - inf
    MUL32(r, zero, inf); o32[i++] = __float_as_uint(r);   // 2 0 * inf
    MUL32(r, inf, zero); o32[i++] = __float_as_uint(r);   // 3 inf * 0
    SUB32(r, one, nq); o32[i++] = __float_as_uint(r);     // 4 1 - (+NaN q)
    SUB32(r, one, nsn); o32[i++] = __float_as_uint(r);    // 5 1 - (-NaN s)
    SUB32(r, nq, one); o32[i++] = __float_as_uint(r);     // 6 (+NaN q) - 1
    SUB32(r, nsn, one); o32[i++] = __float_as_uint(r);    // 7 (-NaN s) - 1
    ADD32(r, one, nsn); o32[i++] = __float_as_uint(r);    // 8 1 + (-NaN s)
    MUL32(r, nsn, one); o32[i++] = __float_as_uint(r);    // 9 (-NaN s) * 1
    MUL32(r, ninf, nsn); o32[i++] = __float_as_uint(r);   // 10 -inf * (-NaN s)
    o32[i++] = __float_as_uint(one - nsn);                // 11 C: 1 - NaN
    o32[i++] = __float_as_uint(inf + ninf);               // 12 C: inf + -inf
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 pa = {inf, zero}, pb = {ninf, inf}, pr;
    asm volatile("v_pk_add_f32 %0, %1, %2" : "=v"(pr) : "v"(pa), "v"(pb));
    o32[i++] = __float_as_uint(pr.x);                     // 13 pk: inf + -inf
    asm volatile("v_pk_mul_f32 %0, %1, %2" : "=v"(pr) : "v"(pa), "v"(pb));
    o32[i++] = __float_as_uint(pr.y);                     // 14 pk: 0 * inf
    const double dinf = __longlong_as_double(in64[0]), dninf = __longlong_as_double(in64[1]),
                 dzero = __longlong_as_double(in64[2]);
    double d;
    int j = 0;
    ADD64(d, dinf, dninf); o64[j++] = __double_as_longlong(d);  // 0 inf + -inf
    MUL64(d, dzero, dinf); o64[j++] = __double_as_longlong(d);  // 1 0 * inf
    o64[j++] = __double_as_longlong(dinf - dinf);               // 2 C: inf - inf
}

int main() {
    const uint32_t h32[6] = {0x7F800000u, 0xFF800000u, 0u, 0x3F800000u, 0x7FC00123u, 0xFF800456u};
    const uint64_t h64[3] = {0x7FF0000000000000ull, 0xFFF0000000000000ull, 0ull};
    uint32_t *d32, *o32, r32[15];
    uint64_t *d64, *o64, r64[3];
    hipMalloc(&d32, sizeof h32);
    hipMalloc(&d64, sizeof h64);
    hipMalloc(&o32, sizeof r32);
    hipMalloc(&o64, sizeof r64);
    hipMemcpy(d32, h32, sizeof h32, hipMemcpyHostToDevice);
    hipMemcpy(d64, h64, sizeof h64, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d32, d64, o32, o64);
    hipMemcpy(r32, o32, sizeof r32, hipMemcpyDeviceToHost);
    hipMemcpy(r64, o64, sizeof r64, hipMemcpyDeviceToHost);
    const char* n32[15] = {"add inf,-inf", "sub inf,inf", "mul 0,inf", "mul inf,0", "sub 1,+qNaN123",
                           "sub 1,-sNaN456", "sub +qNaN123,1", "sub -sNaN456,1", "add 1,-sNaN456", "mul -sNaN456,1",
                           "mul -inf,-sNaN456", "C 1-(-sNaN456)", "C inf+-inf", "pk_add inf,-inf", "pk_mul 0,inf"};
    for (int i = 0; i < 15; ++i) std::printf("f32 %-20s -> %08x\n", n32[i], r32[i]);
    const char* n64[3] = {"add inf,-inf", "mul 0,inf", "C inf-inf"};
    for (int i = 0; i < 3; ++i) std::printf("f64 %-20s -> %016llx\n", n64[i], (unsigned long long)r64[i]);
    return 0;
}
