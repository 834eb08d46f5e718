// mfma64.hip — the u64 matrix-core encode (mfma64.h) in its own translation
// unit: built with -mllvm -amdgpu-mfma-vgpr-form (accumulators in VGPRs; the
// AGPR form keeps a second copy of the 80 accumulator registers at t = 80
// and halves the occupancy), which the u32 kernels do not want.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "ctx.h"
#include "field.h"
#include "mfma64.h"

namespace qk {
namespace {

constexpr int BLOCK = 256;
constexpr int WAVES = BLOCK / 64;

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
    const uint32_t lo = __shfl_xor((int)(uint32_t)v, m, 64);
    const uint32_t hi = __shfl_xor((int)(uint32_t)(v >> 32), m, 64);
    return ((uint64_t)hi << 32) | lo;
}

template <typename KernelT>
uint32_t grid_for(qk_ctx *ctx, KernelT kern, uint64_t units, uint32_t per_block) {
    if (ctx->grid_override) return ctx->grid_override;
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, BLOCK, 0) != hipSuccess || occ < 1) occ = 1;
    const uint64_t full = (uint64_t)ctx->num_cus * (uint64_t)occ;
    uint64_t need = (units + per_block - 1) / per_block;
    if (need < 1) need = 1;
    return (uint32_t)(need < full ? need : full);
}

// ---- u64 form (mfma64.h): NM tiles of 2 giants x NN tiles of 2 babies
template <int NM, int NN, bool OFF>
__global__ __launch_bounds__(mf8::BLOCK) void k_encode_u64_mfma(const uint64_t *__restrict__ ids, uint64_t n,
                                                               uint64_t *__restrict__ partials, uint32_t base) {
    mf64::body<NM, NN, 0, OFF>(ids, n, partials, base);
}

// canonical per-block values [power][block] -> cw[m] = their sum mod p64
__global__ __launch_bounds__(BLOCK) void k_finalize_cw64(const uint64_t *__restrict__ partials, uint32_t nblocks,
                                                         uint64_t *__restrict__ cw) {
    __shared__ uint64_t sm[2][WAVES];
    const uint32_t m = blockIdx.x;
    uint64_t a = 0, b = 0;   // 32-bit limb sums (< nblocks * 2^32)
    for (uint32_t i = threadIdx.x; i < nblocks; i += BLOCK) {
        const uint64_t v = partials[(size_t)m * nblocks + i];
        a += (uint32_t)v;
        b += v >> 32;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        a += shfl_xor_u64(a, off);
        b += shfl_xor_u64(b, off);
    }
    if ((threadIdx.x & 63) == 0) { sm[0][threadIdx.x >> 6] = a; sm[1][threadIdx.x >> 6] = b; }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t sa = 0, sb = 0;
        for (int w = 0; w < WAVES; ++w) { sa += sm[0][w]; sb += sm[1][w]; }
        cw[m] = add64(canon64(sa), mul64(canon64(sb), 1ull << 32));
    }
}

// mfma64.h's signed-byte corrections for the pass's powers base + 1 ..
// base + NB*NA (see k_mfma32_fix); S = the batch's canonical sums; out in the
// u64 partial layout (power m as 32-bit halves out[2m], out[2m+1]; count
// out[2T]; last id out[2T+1], written by pass 0)
__global__ __launch_bounds__(64) void k_mfma64_fix(const uint64_t *__restrict__ cw, uint32_t NB, uint32_t NA,
                                                   uint32_t T, uint32_t base, uint32_t Tp, uint64_t nmod,
                                                   uint64_t inv, const uint64_t *__restrict__ ids, uint64_t n,
                                                   uint64_t *__restrict__ out, int accumulate,
                                                   uint64_t *__restrict__ S) {
    const uint64_t r128 = 0x8080808080808080ull;         // 128 R, R = sum_{j<8} 256^j (< p)
    const uint64_t c1 = mul64(r128, nmod);
    const uint64_t c2 = mul64(mul64(r128, r128), nmod);
    uint32_t a0 = 0;
    if (base == 0) {
        for (uint32_t b = threadIdx.x; b < NB; b += blockDim.x) S[b] = add64(mul64(cw[b], inv), c1);
        __syncthreads();
        a0 = 1;
    }
    for (uint32_t a = a0; a < NA; ++a) {
        const uint64_t ga = S[base + a * NB - 1];
        for (uint32_t b = threadIdx.x; b < NB; b += blockDim.x) {
            const uint32_t m = a * NB + b;
            S[base + m] = sub64(add64(cw[m], mul64(r128, add64(ga, S[b]))), c2);
        }
        __syncthreads();
    }
    for (uint32_t m = threadIdx.x; m < Tp; m += blockDim.x) {
        const uint32_t o = base + m;
        uint64_t v = S[o];
        if (accumulate) v = add64(canon64(out[2 * o] | (out[2 * o + 1] << 32)), v);
        out[2 * o] = (uint32_t)v;
        out[2 * o + 1] = v >> 32;
    }
    if (threadIdx.x == 0 && base == 0) {
        out[2 * T] = accumulate ? out[2 * T] + n : n;
        if (n) out[2 * T + 1] = ids[n - 1];
        else if (!accumulate) out[2 * T + 1] = 0;
    }
}

template <int NM, int NN, bool OFF>
static int enc64_mfma_pass(qk_ctx *ctx, const uint64_t *ids, size_t n, uint32_t T, uint32_t base, uint32_t Tp,
                           uint64_t *out, int acc, uint64_t *partials, uint64_t *cw, uint64_t *S, uint32_t nb,
                           hipStream_t s) {
    using Sh = mf64::Shape<NM, NN>;
    constexpr int NP = Sh::NP;
    static const uint64_t inv = inv64(sub64(1, 0x8080808080808080ull));
    hipEvent_t e0 = prof_begin(ctx, s);
    hipLaunchKernelGGL((k_encode_u64_mfma<NM, NN, OFF>), dim3(nb), dim3(mf8::BLOCK), 0, s, ids, (uint64_t)n, partials,
                       base);
    prof_end(ctx, s, e0);
    QK_HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_finalize_cw64, dim3(NP), dim3(BLOCK), 0, s, partials, nb, cw);
    hipLaunchKernelGGL(k_mfma64_fix, dim3(1), dim3(64), 0, s, cw, (uint32_t)Sh::NB, (uint32_t)Sh::NA, T, base, Tp,
                       (uint64_t)((n + 255) / 256 * 256), inv, ids, (uint64_t)n, out, acc, S);
    QK_HIP_TRY(hipGetLastError());
    return QK_OK;
}

template <int NM, int NN, bool OFF>
uint32_t grid64(qk_ctx *ctx, size_t n) {
    return grid_for(ctx, k_encode_u64_mfma<NM, NN, OFF>, (n + 255) / 256, mf8::WAVES);
}

} // namespace

// T >= 9: 8 babies (NN = 4); T <= 80 in one pass of NM = ceil(T / 16) tiles
// of 2 giants, larger T in passes of <= 80 powers (pass 0 the (8, 10) shape,
// then offset passes with the same babies)
int launch_encode_u64_mfma(qk_ctx *ctx, const uint64_t *ids, size_t n, uint32_t T, uint64_t *out, int acc,
                           hipStream_t s) {
    const uint32_t nb = std::max(grid64<1, 4, false>(ctx, n), grid64<1, 4, true>(ctx, n));
    if (int rc = ensure_scratch(ctx, ((size_t)nb * 80 + 80 + T + 80) * sizeof(uint64_t), s)) return rc;
    uint64_t *partials = (uint64_t *)ctx->d_scratch, *cw = partials + (size_t)nb * 80, *S = cw + 80;
    if (int rc = scratch_acquire(ctx, s)) return rc;
    int rc = QK_OK;
#define QK_MF64(NM_, OFF_, B_, TP_)                                                                     \
    enc64_mfma_pass<NM_, 4, OFF_>(ctx, ids, n, T, B_, TP_, out, acc, partials, cw, S,                  \
                                  std::min(nb, grid64<NM_, 4, OFF_>(ctx, n)), s)
    const uint32_t T0 = std::min<uint32_t>(T, 80);
    switch ((T0 + 15) / 16) {
    case 1: rc = QK_MF64(1, false, 0, T0); break;
    case 2: rc = QK_MF64(2, false, 0, T0); break;
    case 3: rc = QK_MF64(3, false, 0, T0); break;
    case 4: rc = QK_MF64(4, false, 0, T0); break;
    default: rc = QK_MF64(5, false, 0, T0); break;
    }
    for (uint32_t base = 80; base < T && !rc; base += 80) {
        const uint32_t Tp = std::min<uint32_t>(80, T - base);
        switch ((Tp + 15) / 16) {
        case 1: rc = QK_MF64(1, true, base, Tp); break;
        case 2: rc = QK_MF64(2, true, base, Tp); break;
        case 3: rc = QK_MF64(3, true, base, Tp); break;
        case 4: rc = QK_MF64(4, true, base, Tp); break;
        default: rc = QK_MF64(5, true, base, Tp); break;
        }
    }
#undef QK_MF64
    if (int e = scratch_release(ctx, s); e && !rc) rc = e;
    return rc;
}

} // namespace qk
