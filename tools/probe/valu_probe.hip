// VALU issue-rate probe for the integer instructions the KoalaBear kernels are built from.
// Each thread runs 8 independent dependency chains of one instruction; the rate is reported as
// wave64-instructions per SIMD-cycle-equivalent (full rate on a SIMD-32 = 0.5 wave-inst/cycle).
// Build: hipcc -O3 --offload-arch=gfx950 valu_probe.hip -o valu_probe
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 2048

#define CHAIN8(INS)                                                                         \
    asm volatile(INS : "+v"(a0) : "v"(b)); asm volatile(INS : "+v"(a1) : "v"(b));             \
    asm volatile(INS : "+v"(a2) : "v"(b)); asm volatile(INS : "+v"(a3) : "v"(b));             \
    asm volatile(INS : "+v"(a4) : "v"(b)); asm volatile(INS : "+v"(a5) : "v"(b));             \
    asm volatile(INS : "+v"(a6) : "v"(b)); asm volatile(INS : "+v"(a7) : "v"(b));

#define KERNEL32(NAME, INS)                                                              \
    __global__ void NAME(unsigned *out, unsigned seed) {                                  \
        unsigned a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, \
                 a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, b = seed * 3 + 1;                  \
        for (int i = 0; i < ITERS; i++) { CHAIN8(INS) }                                     \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;  \
    }

KERNEL32(k_add, "v_add_u32 %0, %0, %1")
KERNEL32(k_min, "v_min_u32 %0, %0, %1")
KERNEL32(k_mul_lo, "v_mul_lo_u32 %0, %0, %1")
KERNEL32(k_mul_hi, "v_mul_hi_u32 %0, %0, %1")
KERNEL32(k_mul_u24, "v_mul_u32_u24 %0, %0, %1")
KERNEL32(k_mad_u24, "v_mad_u32_u24 %0, %0, %1, %0")
KERNEL32(k_add3, "v_add3_u32 %0, %0, %1, %0")
KERNEL32(k_lshl_add, "v_lshl_add_u32 %0, %0, 3, %1")
KERNEL32(k_sub, "v_sub_u32 %0, %0, %1")
KERNEL32(k_add_lit, "v_add_u32 %0, 0x80ffffff, %0")
KERNEL32(k_add_e64, "v_add_u32_e64 %0, %0, %1")
KERNEL32(k_and, "v_and_b32 %0, %0, %1")
KERNEL32(k_xor, "v_xor_b32 %0, %0, %1")
KERNEL32(k_lshl, "v_lshlrev_b32 %0, 3, %0")
KERNEL32(k_max, "v_max_u32 %0, %0, %1")
KERNEL32(k_min3, "v_min3_u32 %0, %0, %1, %0")
KERNEL32(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
KERNEL32(k_addmin, "v_add_u32 %0, %0, %1\n v_min_u32 %0, %0, %1")
KERNEL32(k_mov, "v_mov_b32 %0, %1")
KERNEL32(k_pk_add_u16, "v_pk_add_u16 %0, %0, %1")

#define CHAIN8_64(INS)                                                                      \
    asm volatile(INS : "+v"(a0) : "v"(b)); asm volatile(INS : "+v"(a1) : "v"(b));             \
    asm volatile(INS : "+v"(a2) : "v"(b)); asm volatile(INS : "+v"(a3) : "v"(b));             \
    asm volatile(INS : "+v"(a4) : "v"(b)); asm volatile(INS : "+v"(a5) : "v"(b));             \
    asm volatile(INS : "+v"(a6) : "v"(b)); asm volatile(INS : "+v"(a7) : "v"(b));

#define KERNEL64(NAME, INS)                                                                  \
    __global__ void NAME(unsigned *out, unsigned seed) {                                      \
        unsigned long long a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3,     \
                           a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, b = seed * 3 + 1; \
        for (int i = 0; i < ITERS; i++) { CHAIN8_64(INS) }                                      \
        out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7); \
    }
KERNEL64(k_lshl_add_u64, "v_lshl_add_u64 %0, %0, 0, %1")

__global__ void k_mad_u64(unsigned *out, unsigned seed) {
    unsigned long long a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
                       a6 = a0 + 6, a7 = a0 + 7;
    unsigned b = seed * 3 + 1, c = seed ^ 77;
#define M(a) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(a) : "v"(b), "v"(c) : "s40", "s41");
    for (int i = 0; i < ITERS; i++) { M(a0) M(a1) M(a2) M(a3) M(a4) M(a5) M(a6) M(a7) }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}


// 64-bit add as a carry pair: v_add_co_u32 (carry out to an SGPR pair) + v_addc_co_u32
#define ADDC(lo, hi, S) asm volatile("v_add_co_u32_e64 %0, " S ", %0, %2\n v_addc_co_u32_e64 %1, " S ", %1, 0, " S \
                                     : "+v"(lo), "+v"(hi) : "v"(b) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55");
__global__ void k_add64_pair(unsigned *out, unsigned seed) {
    unsigned l0 = threadIdx.x ^ seed, l1 = l0 + 1, l2 = l0 + 2, l3 = l0 + 3, h0 = 0, h1 = 0, h2 = 0, h3 = 0, b = seed * 3 + 1;
    for (int i = 0; i < ITERS; i++) {
        ADDC(l0, h0, "s[40:41]") ADDC(l1, h1, "s[42:43]") ADDC(l2, h2, "s[44:45]") ADDC(l3, h3, "s[46:47]")
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = l0 ^ l1 ^ l2 ^ l3 ^ h0 ^ h1 ^ h2 ^ h3;
}
KERNEL32(k_add_co, "v_add_co_u32 %0, vcc, %0, %1")
KERNEL32(k_sub_co, "v_sub_co_u32 %0, vcc, %0, %1")


typedef void (*kfn)(unsigned *, unsigned);

int main() {
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    const double clk = prop.clockRate * 1e3;  // Hz
    const int threads = 256, blocks = cus * 32;
    unsigned *out;
    hipMalloc(&out, (size_t)threads * blocks * 4);
    struct { const char *name; kfn f; } ks[] = {
        {"v_add_u32", k_add}, {"v_min_u32", k_min}, {"v_mul_lo_u32", k_mul_lo}, {"v_mul_hi_u32", k_mul_hi},
        {"v_mul_u32_u24", k_mul_u24}, {"v_mad_u32_u24", k_mad_u24}, {"v_add3_u32", k_add3},
        {"v_lshl_add_u32", k_lshl_add}, {"v_lshl_add_u64", k_lshl_add_u64}, {"v_mad_u64_u32", k_mad_u64},
        {"v_sub_u32", k_sub}, {"v_add_u32 literal", k_add_lit}, {"v_add_u32_e64", k_add_e64}, {"v_and_b32", k_and},
        {"v_xor_b32", k_xor}, {"v_lshlrev_b32", k_lshl}, {"v_max_u32", k_max}, {"v_min3_u32", k_min3},
        {"v_cndmask_b32", k_cndmask}, {"add+min (x2 ops)", k_addmin}, {"v_mov_b32", k_mov},
        {"v_pk_add_u16", k_pk_add_u16}, {"v_add_co_u32 (vcc)", k_add_co}, {"v_sub_co_u32 (vcc)", k_sub_co},
        {"add_co+addc pair (x2 ops)", k_add64_pair},
    };
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    printf("CUs %d clock %.0f MHz\n", cus, clk / 1e6);
    for (auto &k : ks) {
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 1u);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 1u);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double lane_ops = 5.0 * blocks * threads * ITERS * 8;
        const double rate = lane_ops / (ms * 1e-3);                // lane-ops / s
        const double per_cu_clk = rate / cus / clk;                 // lane-ops / CU / cycle
        printf("%-16s %8.3f ms  %7.2f Tlane-op/s  %6.1f lane-op/CU/clk  (full rate = 128)\n", k.name, ms, rate / 1e12,
               per_cu_clk);
    }
    hipFree(out);
    return 0;
}
