// ubench_issue.hip — issue cost of the instruction mixes the BSGS encode is
// built from, on gfx950, in SHADER CYCLES (not part of the product; informs
// DESIGN.md §3).  Every kernel runs W waves per SIMD (W workgroups of 256
// threads per CU), each lane L iterations of an unrolled block of independent
// instructions; workgroup thread 0 records s_memtime / s_memrealtime so the
// shader clock of the run is measured, and the result is reported as SIMD
// cycles per wave-instruction of each kind.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "../sidekick_amd/csrc/field.h"

#define CHK(x)                                                                              \
    do {                                                                                    \
        hipError_t e = (x);                                                                 \
        if (e != hipSuccess) {                                                              \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);    \
            return 1;                                                                       \
        }                                                                                   \
    } while (0)

constexpr int L = 16384;

#define CLK_BEGIN                                                                          \
    const uint64_t clk_c0 = __builtin_amdgcn_s_memtime(), clk_r0 = __builtin_amdgcn_s_memrealtime();
#define CLK_END                                                                            \
    const uint64_t clk_c1 = __builtin_amdgcn_s_memtime(), clk_r1 = __builtin_amdgcn_s_memrealtime(); \
    if (threadIdx.x == 0) { clk[2 * blockIdx.x] = clk_c1 - clk_c0; clk[2 * blockIdx.x + 1] = clk_r1 - clk_r0; }

// 8 VALU adds
__global__ void k_vadd(uint32_t *out, uint64_t *clk, uint32_t b) {
    CLK_BEGIN
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < L; ++i)
        asm volatile("v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t"
                     "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    CLK_END
}
// 8 v_mad_u64_u32
__global__ void k_vmad(uint32_t *out, uint64_t *clk, uint32_t b) {
    CLK_BEGIN
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < L; ++i)
        asm volatile("v_mad_u64_u32 %0, s[40:41], %8, %8, %0\n\tv_mad_u64_u32 %1, s[42:43], %8, %8, %1\n\t"
                     "v_mad_u64_u32 %2, s[44:45], %8, %8, %2\n\tv_mad_u64_u32 %3, s[46:47], %8, %8, %3\n\t"
                     "v_mad_u64_u32 %4, s[40:41], %8, %8, %4\n\tv_mad_u64_u32 %5, s[42:43], %8, %8, %5\n\t"
                     "v_mad_u64_u32 %6, s[44:45], %8, %8, %6\n\tv_mad_u64_u32 %7, s[46:47], %8, %8, %7"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(b)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47");
    const uint64_t s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(s ^ (s >> 32));
    CLK_END
}
// 8 SALU adds (independent SGPRs)
__global__ void k_sadd(uint32_t *out, uint64_t *clk, uint32_t b) {
    CLK_BEGIN
    uint32_t a0 = b, a1 = b + 1, a2 = b + 2, a3 = b + 3, a4 = b + 4, a5 = b + 5, a6 = b + 6, a7 = b + 7;
    for (int i = 0; i < L; ++i)
        asm volatile("s_add_u32 %0, %0, %8\n\ts_add_u32 %1, %1, %8\n\ts_add_u32 %2, %2, %8\n\ts_add_u32 %3, %3, %8\n\t"
                     "s_add_u32 %4, %4, %8\n\ts_add_u32 %5, %5, %8\n\ts_add_u32 %6, %6, %8\n\ts_add_u32 %7, %7, %8"
                     : "+s"(a0), "+s"(a1), "+s"(a2), "+s"(a3), "+s"(a4), "+s"(a5), "+s"(a6), "+s"(a7)
                     : "s"(b)
                     : "scc");
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + threadIdx.x;
    CLK_END
}
// 8 VALU adds interleaved with 8 SALU adds
__global__ void k_vadd_sadd(uint32_t *out, uint64_t *clk, uint32_t b) {
    CLK_BEGIN
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t s0 = b, s1 = b + 1, s2 = b + 2, s3 = b + 3;
    for (int i = 0; i < L; ++i)
        asm volatile("v_add_u32 %0, %0, %12\n\ts_add_u32 %8, %8, %13\n\tv_add_u32 %1, %1, %12\n\ts_add_u32 %9, %9, %13\n\t"
                     "v_add_u32 %2, %2, %12\n\ts_add_u32 %10, %10, %13\n\tv_add_u32 %3, %3, %12\n\ts_add_u32 %11, %11, %13\n\t"
                     "v_add_u32 %4, %4, %12\n\ts_add_u32 %8, %8, %13\n\tv_add_u32 %5, %5, %12\n\ts_add_u32 %9, %9, %13\n\t"
                     "v_add_u32 %6, %6, %12\n\ts_add_u32 %10, %10, %13\n\tv_add_u32 %7, %7, %12\n\ts_add_u32 %11, %11, %13"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), "+s"(s0),
                       "+s"(s1), "+s"(s2), "+s"(s3)
                     : "v"(b), "s"(b)
                     : "scc");
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + s0 + s1 + s2 + s3;
    CLK_END
}
// 8 v_mad_u64_u32 interleaved with 8 SALU adds
__global__ void k_vmad_sadd(uint32_t *out, uint64_t *clk, uint32_t b) {
    CLK_BEGIN
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t s0 = b, s1 = b + 1, s2 = b + 2, s3 = b + 3;
    for (int i = 0; i < L; ++i)
        asm volatile("v_mad_u64_u32 %0, s[40:41], %12, %12, %0\n\ts_add_u32 %8, %8, %13\n\t"
                     "v_mad_u64_u32 %1, s[42:43], %12, %12, %1\n\ts_add_u32 %9, %9, %13\n\t"
                     "v_mad_u64_u32 %2, s[44:45], %12, %12, %2\n\ts_add_u32 %10, %10, %13\n\t"
                     "v_mad_u64_u32 %3, s[46:47], %12, %12, %3\n\ts_add_u32 %11, %11, %13\n\t"
                     "v_mad_u64_u32 %4, s[40:41], %12, %12, %4\n\ts_add_u32 %8, %8, %13\n\t"
                     "v_mad_u64_u32 %5, s[42:43], %12, %12, %5\n\ts_add_u32 %9, %9, %13\n\t"
                     "v_mad_u64_u32 %6, s[44:45], %12, %12, %6\n\ts_add_u32 %10, %10, %13\n\t"
                     "v_mad_u64_u32 %7, s[46:47], %12, %12, %7\n\ts_add_u32 %11, %11, %13"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), "+s"(s0),
                       "+s"(s1), "+s"(s2), "+s"(s3)
                     : "v"(b), "s"(b)
                     : "scc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47");
    const uint64_t s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(s ^ (s >> 32)) + s0 + s1 + s2 + s3;
    CLK_END
}
// the VALU-counted MAC group: 4 x (v_mad_u64_u32 -> carry) + 4 x v_addc
__global__ void k_mac4v(uint32_t *out, uint64_t *clk, uint32_t b) {
    CLK_BEGIN
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    for (int i = 0; i < L; ++i)
        asm volatile("v_mad_u64_u32 %0, s[40:41], %8, %8, %0\n\tv_mad_u64_u32 %1, s[42:43], %8, %8, %1\n\t"
                     "v_mad_u64_u32 %2, s[44:45], %8, %8, %2\n\tv_mad_u64_u32 %3, s[46:47], %8, %8, %3\n\t"
                     "v_addc_co_u32_e64 %4, s[40:41], %4, 0, s[40:41]\n\tv_addc_co_u32_e64 %5, s[42:43], %5, 0, s[42:43]\n\t"
                     "v_addc_co_u32_e64 %6, s[44:45], %6, 0, s[44:45]\n\tv_addc_co_u32_e64 %7, s[46:47], %7, 0, s[46:47]\n\t"
                     "v_mad_u64_u32 %0, s[48:49], %8, %8, %0\n\tv_mad_u64_u32 %1, s[50:51], %8, %8, %1\n\t"
                     "v_mad_u64_u32 %2, s[52:53], %8, %8, %2\n\tv_mad_u64_u32 %3, s[54:55], %8, %8, %3\n\t"
                     "v_addc_co_u32_e64 %4, s[48:49], %4, 0, s[48:49]\n\tv_addc_co_u32_e64 %5, s[50:51], %5, 0, s[50:51]\n\t"
                     "v_addc_co_u32_e64 %6, s[52:53], %6, 0, s[52:53]\n\tv_addc_co_u32_e64 %7, s[54:55], %7, 0, s[54:55]"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3)
                     : "v"(b)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52",
                       "s53", "s54", "s55");
    const uint64_t s = a0 + a1 + a2 + a3;
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(s ^ (s >> 32)) + c0 + c1 + c2 + c3;
    CLK_END
}
// the SALU-counted MAC group: 4 x (v_mad_u64_u32 -> carry) + 4 x (s_bcnt1 + s_add)
__global__ void k_mac4s(uint32_t *out, uint64_t *clk, uint32_t b) {
    CLK_BEGIN
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0, t0, t1, t2, t3;
    for (int i = 0; i < L; ++i)
        asm volatile("v_mad_u64_u32 %0, s[40:41], %12, %12, %0\n\tv_mad_u64_u32 %1, s[42:43], %12, %12, %1\n\t"
                     "v_mad_u64_u32 %2, s[44:45], %12, %12, %2\n\tv_mad_u64_u32 %3, s[46:47], %12, %12, %3\n\t"
                     "s_bcnt1_i32_b64 %8, s[40:41]\n\ts_add_u32 %4, %4, %8\n\ts_bcnt1_i32_b64 %9, s[42:43]\n\ts_add_u32 %5, %5, %9\n\t"
                     "s_bcnt1_i32_b64 %10, s[44:45]\n\ts_add_u32 %6, %6, %10\n\ts_bcnt1_i32_b64 %11, s[46:47]\n\ts_add_u32 %7, %7, %11\n\t"
                     "v_mad_u64_u32 %0, s[48:49], %12, %12, %0\n\tv_mad_u64_u32 %1, s[50:51], %12, %12, %1\n\t"
                     "v_mad_u64_u32 %2, s[52:53], %12, %12, %2\n\tv_mad_u64_u32 %3, s[54:55], %12, %12, %3\n\t"
                     "s_bcnt1_i32_b64 %8, s[48:49]\n\ts_add_u32 %4, %4, %8\n\ts_bcnt1_i32_b64 %9, s[50:51]\n\ts_add_u32 %5, %5, %9\n\t"
                     "s_bcnt1_i32_b64 %10, s[52:53]\n\ts_add_u32 %6, %6, %10\n\ts_bcnt1_i32_b64 %11, s[54:55]\n\ts_add_u32 %7, %7, %11"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+s"(c0), "+s"(c1), "+s"(c2), "+s"(c3), "=&s"(t0),
                       "=&s"(t1), "=&s"(t2), "=&s"(t3)
                     : "v"(b)
                     : "scc", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51",
                       "s52", "s53", "s54", "s55");
    const uint64_t s = a0 + a1 + a2 + a3;
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(s ^ (s >> 32)) + c0 + c1 + c2 + c3;
    CLK_END
}
// the lazy modmul of the encode (field.h mulfold32_fast as compiled: 2 x
// v_mad_u64_u32 + sub + lshl_add + add_co), 4 independent chains
__global__ void k_modmul(uint32_t *out, uint64_t *clk, uint32_t b) {
    CLK_BEGIN
    uint32_t y0 = threadIdx.x, y1 = y0 + 1, y2 = y0 + 2, y3 = y0 + 3, w = 0;
    const uint32_t x = 0x9E3779B1u ^ b;
    for (int i = 0; i < L; ++i) {
        y0 = qk::mulfold32_fast(y0, x, w);
        y1 = qk::mulfold32_fast(y1, x, w);
        y2 = qk::mulfold32_fast(y2, x, w);
        y3 = qk::mulfold32_fast(y3, x, w);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = y0 + y1 + y2 + y3 + w;
    CLK_END
}

// 8 v_mad_u64_u32 whose (dead) carry-outs all go to ONE SGPR pair
__global__ void k_vmad_same(uint32_t *out, uint64_t *clk, uint32_t b) {
    CLK_BEGIN
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < L; ++i)
        asm volatile("v_mad_u64_u32 %0, s[40:41], %8, %8, %0\n\tv_mad_u64_u32 %1, s[40:41], %8, %8, %1\n\t"
                     "v_mad_u64_u32 %2, s[40:41], %8, %8, %2\n\tv_mad_u64_u32 %3, s[40:41], %8, %8, %3\n\t"
                     "v_mad_u64_u32 %4, s[40:41], %8, %8, %4\n\tv_mad_u64_u32 %5, s[40:41], %8, %8, %5\n\t"
                     "v_mad_u64_u32 %6, s[40:41], %8, %8, %6\n\tv_mad_u64_u32 %7, s[40:41], %8, %8, %7"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(b)
                     : "s40", "s41");
    const uint64_t s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(s ^ (s >> 32));
    CLK_END
}
// 8 v_mad_u64_u32, 8 distinct carry pairs
__global__ void k_vmad_8p(uint32_t *out, uint64_t *clk, uint32_t b) {
    CLK_BEGIN
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < L; ++i)
        asm volatile("v_mad_u64_u32 %0, s[40:41], %8, %8, %0\n\tv_mad_u64_u32 %1, s[42:43], %8, %8, %1\n\t"
                     "v_mad_u64_u32 %2, s[44:45], %8, %8, %2\n\tv_mad_u64_u32 %3, s[46:47], %8, %8, %3\n\t"
                     "v_mad_u64_u32 %4, s[48:49], %8, %8, %4\n\tv_mad_u64_u32 %5, s[50:51], %8, %8, %5\n\t"
                     "v_mad_u64_u32 %6, s[52:53], %8, %8, %6\n\tv_mad_u64_u32 %7, s[54:55], %8, %8, %7"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(b)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52",
                       "s53", "s54", "s55");
    const uint64_t s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(s ^ (s >> 32));
    CLK_END
}
// 8 v_mul_lo_u32 (no SGPR write at all)
__global__ void k_vmullo(uint32_t *out, uint64_t *clk, uint32_t b) {
    CLK_BEGIN
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < L; ++i)
        asm volatile("v_mul_lo_u32 %0, %0, %8\n\tv_mul_lo_u32 %1, %1, %8\n\tv_mul_lo_u32 %2, %2, %8\n\tv_mul_lo_u32 %3, %3, %8\n\t"
                     "v_mul_lo_u32 %4, %4, %8\n\tv_mul_lo_u32 %5, %5, %8\n\tv_mul_lo_u32 %6, %6, %8\n\tv_mul_lo_u32 %7, %7, %8"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    CLK_END
}
// 8 v_add_co_u32 (carry to SGPR), all to one pair / to 8 pairs
__global__ void k_vaddco_same(uint32_t *out, uint64_t *clk, uint32_t b) {
    CLK_BEGIN
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < L; ++i)
        asm volatile("v_add_co_u32_e64 %0, s[40:41], %0, %8\n\tv_add_co_u32_e64 %1, s[40:41], %1, %8\n\t"
                     "v_add_co_u32_e64 %2, s[40:41], %2, %8\n\tv_add_co_u32_e64 %3, s[40:41], %3, %8\n\t"
                     "v_add_co_u32_e64 %4, s[40:41], %4, %8\n\tv_add_co_u32_e64 %5, s[40:41], %5, %8\n\t"
                     "v_add_co_u32_e64 %6, s[40:41], %6, %8\n\tv_add_co_u32_e64 %7, s[40:41], %7, %8"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(b)
                     : "s40", "s41");
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    CLK_END
}
__global__ void k_vaddco_8p(uint32_t *out, uint64_t *clk, uint32_t b) {
    CLK_BEGIN
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < L; ++i)
        asm volatile("v_add_co_u32_e64 %0, s[40:41], %0, %8\n\tv_add_co_u32_e64 %1, s[42:43], %1, %8\n\t"
                     "v_add_co_u32_e64 %2, s[44:45], %2, %8\n\tv_add_co_u32_e64 %3, s[46:47], %3, %8\n\t"
                     "v_add_co_u32_e64 %4, s[48:49], %4, %8\n\tv_add_co_u32_e64 %5, s[50:51], %5, %8\n\t"
                     "v_add_co_u32_e64 %6, s[52:53], %6, %8\n\tv_add_co_u32_e64 %7, s[54:55], %7, %8"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(b)
                     : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52",
                       "s53", "s54", "s55");
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    CLK_END
}

// single-instruction issue costs (8 independent per iteration)
__global__ void k_lshladd(uint32_t *out, uint64_t *clk, uint32_t b) {
    CLK_BEGIN
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < L; ++i)
        asm volatile("v_lshl_add_u32 %0, %0, 2, %8\n\tv_lshl_add_u32 %1, %1, 2, %8\n\tv_lshl_add_u32 %2, %2, 2, %8\n\tv_lshl_add_u32 %3, %3, 2, %8\n\tv_lshl_add_u32 %4, %4, 2, %8\n\tv_lshl_add_u32 %5, %5, 2, %8\n\tv_lshl_add_u32 %6, %6, 2, %8\n\tv_lshl_add_u32 %7, %7, 2, %8"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(b));
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    CLK_END
}
__global__ void k_adde64(uint32_t *out, uint64_t *clk, uint32_t b) {
    CLK_BEGIN
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < L; ++i)
        asm volatile("v_add_u32_e64 %0, %0, %8\n\tv_add_u32_e64 %1, %1, %8\n\tv_add_u32_e64 %2, %2, %8\n\tv_add_u32_e64 %3, %3, %8\n\tv_add_u32_e64 %4, %4, %8\n\tv_add_u32_e64 %5, %5, %8\n\tv_add_u32_e64 %6, %6, %8\n\tv_add_u32_e64 %7, %7, %8"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(b));
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    CLK_END
}
__global__ void k_min3(uint32_t *out, uint64_t *clk, uint32_t b) {
    CLK_BEGIN
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < L; ++i)
        asm volatile("v_min3_u32 %0, %0, %8, %0\n\tv_min3_u32 %1, %1, %8, %1\n\tv_min3_u32 %2, %2, %8, %2\n\tv_min3_u32 %3, %3, %8, %3\n\tv_min3_u32 %4, %4, %8, %4\n\tv_min3_u32 %5, %5, %8, %5\n\tv_min3_u32 %6, %6, %8, %6\n\tv_min3_u32 %7, %7, %8, %7"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(b));
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    CLK_END
}
__global__ void k_addce32(uint32_t *out, uint64_t *clk, uint32_t b) {
    CLK_BEGIN
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < L; ++i)
        asm volatile("v_addc_co_u32_e32 %0, vcc, 0, %0, vcc\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\tv_addc_co_u32_e32 %2, vcc, 0, %2, vcc\n\tv_addc_co_u32_e32 %3, vcc, 0, %3, vcc\n\tv_addc_co_u32_e32 %4, vcc, 0, %4, vcc\n\tv_addc_co_u32_e32 %5, vcc, 0, %5, vcc\n\tv_addc_co_u32_e32 %6, vcc, 0, %6, vcc\n\tv_addc_co_u32_e32 %7, vcc, 0, %7, vcc"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(b) : "vcc");
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    CLK_END
}
__global__ void k_cndmask(uint32_t *out, uint64_t *clk, uint32_t b) {
    CLK_BEGIN
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < L; ++i)
        asm volatile("v_cndmask_b32_e64 %0, %0, %8, s[40:41]\n\tv_cndmask_b32_e64 %1, %1, %8, s[40:41]\n\tv_cndmask_b32_e64 %2, %2, %8, s[40:41]\n\tv_cndmask_b32_e64 %3, %3, %8, s[40:41]\n\tv_cndmask_b32_e64 %4, %4, %8, s[40:41]\n\tv_cndmask_b32_e64 %5, %5, %8, s[40:41]\n\tv_cndmask_b32_e64 %6, %6, %8, s[40:41]\n\tv_cndmask_b32_e64 %7, %7, %8, s[40:41]"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(b) : "s40", "s41");
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    CLK_END
}
__global__ void k_madu24(uint32_t *out, uint64_t *clk, uint32_t b) {
    CLK_BEGIN
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < L; ++i)
        asm volatile("v_mad_u32_u24 %0, %0, %8, %0\n\tv_mad_u32_u24 %1, %1, %8, %1\n\tv_mad_u32_u24 %2, %2, %8, %2\n\tv_mad_u32_u24 %3, %3, %8, %3\n\tv_mad_u32_u24 %4, %4, %8, %4\n\tv_mad_u32_u24 %5, %5, %8, %5\n\tv_mad_u32_u24 %6, %6, %8, %6\n\tv_mad_u32_u24 %7, %7, %8, %7"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(b));
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    CLK_END
}
__global__ void k_mov(uint32_t *out, uint64_t *clk, uint32_t b) {
    CLK_BEGIN
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < L; ++i)
        asm volatile("v_mov_b32 %0, %8\n\tv_mov_b32 %1, %8\n\tv_mov_b32 %2, %8\n\tv_mov_b32 %3, %8\n\tv_mov_b32 %4, %8\n\tv_mov_b32 %5, %8\n\tv_mov_b32 %6, %8\n\tv_mov_b32 %7, %8"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(b));
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    CLK_END
}
__global__ void k_add3(uint32_t *out, uint64_t *clk, uint32_t b) {
    CLK_BEGIN
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < L; ++i)
        asm volatile("v_add3_u32 %0, %0, %8, %0\n\tv_add3_u32 %1, %1, %8, %1\n\tv_add3_u32 %2, %2, %8, %2\n\tv_add3_u32 %3, %3, %8, %3\n\tv_add3_u32 %4, %4, %8, %4\n\tv_add3_u32 %5, %5, %8, %5\n\tv_add3_u32 %6, %6, %8, %6\n\tv_add3_u32 %7, %7, %8, %7"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(b));
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    CLK_END
}

typedef void (*kern_t)(uint32_t *, uint64_t *, uint32_t);

int main(int argc, char **argv) {
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    int wall_khz = 0;
    CHK(hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, 0));
    const int cus = prop.multiProcessorCount, threads = 256;
    const int maxw = 8;
    uint32_t *out;
    uint64_t *clk;
    CHK(hipMalloc(&out, (size_t)cus * maxw * threads * 4));
    CHK(hipMalloc(&clk, (size_t)cus * maxw * 16));
    // insts per loop iteration per lane: {valu_simple, valu_mul, salu}
    struct { const char *name; kern_t k; int vs, vm, s; } ks[] = {
        {"vadd8", k_vadd, 8, 0, 0},         {"vmad8", k_vmad, 0, 8, 0},
        {"sadd8", k_sadd, 0, 0, 8},         {"vadd8+sadd8", k_vadd_sadd, 8, 0, 8},
        {"vmad8+sadd8", k_vmad_sadd, 0, 8, 8}, {"mac4v x2 (8 mad + 8 addc)", k_mac4v, 8, 8, 0},
        {"mac4s x2 (8 mad + 16 salu)", k_mac4s, 0, 8, 16}, {"modmul x4 (8 mad + 14 simple)", k_modmul, 14, 8, 0},
        {"vmad8 one carry pair", k_vmad_same, 0, 8, 0}, {"vmad8 8 carry pairs", k_vmad_8p, 0, 8, 0},
        {"vmullo8", k_vmullo, 0, 8, 0}, {"vaddco8 one carry pair", k_vaddco_same, 8, 0, 0},
        {"vaddco8 8 carry pairs", k_vaddco_8p, 8, 0, 0},
        {"lshladd x8", k_lshladd, 8, 0, 0},
        {"adde64 x8", k_adde64, 8, 0, 0},
        {"min3 x8", k_min3, 8, 0, 0},
        {"addce32 x8", k_addce32, 8, 0, 0},
        {"cndmask x8", k_cndmask, 8, 0, 0},
        {"madu24 x8", k_madu24, 8, 0, 0},
        {"mov x8", k_mov, 8, 0, 0},
        {"add3 x8", k_add3, 8, 0, 0},

    };
    std::vector<uint64_t> h(2 * cus * maxw);
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    printf("{\"cus\": %d, \"L\": %d, \"results\": [\n", cus, L);
    const int wlist[] = {2, 8};
    bool first = true;
    for (size_t i = 0; i < sizeof(ks) / sizeof(ks[0]); ++i) {
        for (int W : wlist) {
            const int blocks = cus * W;
            hipLaunchKernelGGL(ks[i].k, dim3(blocks), dim3(threads), 0, 0, out, clk, 3u);
            CHK(hipDeviceSynchronize());
            CHK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(ks[i].k, dim3(blocks), dim3(threads), 0, 0, out, clk, 3u);
            CHK(hipEventRecord(e1, 0));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            CHK(hipMemcpy(h.data(), clk, 16ull * blocks, hipMemcpyDeviceToHost));
            double cyc = 0, rt = 0;
            for (int b = 0; b < blocks; ++b) { cyc += h[2 * b]; rt += h[2 * b + 1]; }
            const double mhz = cyc / rt * wall_khz / 1e3;
            // kernel wall time in shader cycles over the W*L wave-iterations every SIMD runs
            const double per_iter = ms * 1e-3 * mhz * 1e6 / ((double)W * L);
            const double blk_cyc = cyc / blocks;  // one workgroup's lifetime (residency check)
            printf("%s  {\"mix\": \"%s\", \"waves_per_simd\": %d, \"mhz\": %.0f, \"ms\": %.3f, "
                   "\"simd_cycles_per_iter\": %.2f, \"block_cycles_over_kernel\": %.2f, \"valu_simple\": %d, "
                   "\"valu_mul\": %d, \"salu\": %d}",
                   first ? "" : ",\n", ks[i].name, W, mhz, ms, per_iter, blk_cyc / (ms * 1e-3 * mhz * 1e6),
                   ks[i].vs, ks[i].vm, ks[i].s);
            first = false;
        }
    }
    printf("\n]}\n");
    return 0;
}
