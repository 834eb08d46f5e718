// probe_i8.hip — pins two gfx950 behaviours the i8-MFMA encode relies on
// (not product code): the byte gather of ds_read_b64_tr_b8, and the operand /
// accumulator lane maps of v_mfma_i32_16x16x64_i8, both with exact integer
// data against a CPU model.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v2i __attribute__((ext_vector_type(2)));
typedef int v4i __attribute__((ext_vector_type(4)));

// every lane reads at lds + addr[lane]; LDS byte i holds i (sel 0) or i >> 8 (sel 1)
__global__ void k_tr8(const int *addr, int sel, uint8_t *out) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[2048];
    for (int i = threadIdx.x; i < 2048; i += 64) lds[i] = sel ? (uint8_t)(i >> 8) : (uint8_t)i;
    __syncthreads();
    v2i r = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i *)(lds + addr[threadIdx.x]));
    for (int b = 0; b < 8; ++b) out[threadIdx.x * 8 + b] = (uint8_t)(((b < 4 ? r.x : r.y) >> (8 * (b & 3))) & 0xFF);
}

// A[16][64], B[64][16] int8 row-major; lane fragments built per the hypothesis
//   A: lane l, byte e -> A[l & 15][16 (l >> 4) + e];  B: lane l, byte e -> B[16 (l >> 4) + e][l & 15]
//   C: lane l, reg r -> C[4 (l >> 4) + r][l & 15]
__global__ void k_mfma(const int8_t *A, const int8_t *B, int *C) {
    const int l = threadIdx.x;
    v4i a, b;
    uint8_t *pa = (uint8_t *)&a, *pb = (uint8_t *)&b;
    for (int e = 0; e < 16; ++e) {
        pa[e] = (uint8_t)A[(l & 15) * 64 + 16 * (l >> 4) + e];
        pb[e] = (uint8_t)B[(16 * (l >> 4) + e) * 16 + (l & 15)];
    }
    v4i c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) C[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

int main() {
    int *d_addr;
    uint8_t *d_out;
    hipMalloc(&d_addr, 64 * 4);
    hipMalloc(&d_out, 64 * 8);
    // pattern 1: lane l -> 8 l (contiguous); pattern 2: lane l -> 16 l (rows of 16 bytes, stride 16)
    for (int pat = 0; pat < 3; ++pat) {
        int h_addr[64];
        for (int l = 0; l < 64; ++l) h_addr[l] = pat == 0 ? 8 * l : pat == 1 ? 16 * l : 32 * (l >> 1) + 8 * (l & 1);
        hipMemcpy(d_addr, h_addr, sizeof h_addr, hipMemcpyHostToDevice);
        uint8_t lo[512], hi[512];
        hipLaunchKernelGGL(k_tr8, dim3(1), dim3(64), 0, 0, d_addr, 0, d_out);
        hipMemcpy(lo, d_out, 512, hipMemcpyDeviceToHost);
        hipLaunchKernelGGL(k_tr8, dim3(1), dim3(64), 0, 0, d_addr, 1, d_out);
        hipMemcpy(hi, d_out, 512, hipMemcpyDeviceToHost);
        printf("tr8 pattern %d (lane address: %s)\n", pat, pat == 0 ? "8 l" : pat == 1 ? "16 l" : "32 (l>>1) + 8 (l&1)");
        for (int l = 0; l < 64; ++l) {
            printf("  lane %2d addr %4d <-", l, h_addr[l]);
            for (int b = 0; b < 8; ++b) printf(" %4d", lo[l * 8 + b] | (hi[l * 8 + b] << 8));
            printf("\n");
        }
    }
    int8_t A[16 * 64], B[64 * 16];
    srand(7);
    for (int i = 0; i < 16 * 64; ++i) A[i] = (int8_t)(rand() & 0xFF);
    for (int i = 0; i < 64 * 16; ++i) B[i] = (int8_t)(rand() & 0xFF);
    int8_t *dA, *dB;
    int *dC, C[256];
    hipMalloc(&dA, sizeof A);
    hipMalloc(&dB, sizeof B);
    hipMalloc(&dC, sizeof C);
    hipMemcpy(dA, A, sizeof A, hipMemcpyHostToDevice);
    hipMemcpy(dB, B, sizeof B, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_mfma, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    hipMemcpy(C, dC, sizeof C, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int m = 0; m < 16; ++m)
        for (int n = 0; n < 16; ++n) {
            int s = 0;
            for (int k = 0; k < 64; ++k) s += A[m * 64 + k] * B[k * 16 + n];
            if (s != C[m * 16 + n]) ++bad;
        }
    printf("mfma_i32_16x16x64_i8 layout hypothesis: %d of 256 outputs differ\n", bad);
    return 0;
}
