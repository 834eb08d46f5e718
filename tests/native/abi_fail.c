#define _POSIX_C_SOURCE 199309L
/* abi_fail.c — every error path of the C ABI, many times over (not product
 * code).  Each call must return its documented status and leave nothing
 * behind: under AddressSanitizer's leak checker in host mode, and without
 * device memory growth in device mode.
 *
 *   abi_fail host      host functions: malformed / mismatched bincode,
 *                      capacity and undecodable errors, threshold 0,
 *                      mismatched thresholds, null arguments
 *   abi_fail device    the device entry points' early and late failures
 *                      (host pointers where device memory is required,
 *                      threshold limits, hit-buffer capacity, undecodable
 *                      differences, flow-output capacity) on one context;
 *                      free device memory is compared before and after
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "quack_hip.h"

#define EXPECT(call, want)                                                                         \
    do {                                                                                           \
        int rc_ = (call);                                                                          \
        if (rc_ != (want)) {                                                                       \
            fprintf(stderr, "abi_fail line %d: %s returned %d, want %d\n", __LINE__, #call, rc_, (want)); \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

static uint64_t rng = 0x5EEDull;
static uint64_t next(void) {
    uint64_t z = (rng += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static void host_round(void) {
    const uint32_t t = 8;
    qk_u32 *a = malloc(qk_u32_size(t)), *b = malloc(qk_u32_size(t + 1)), *z = malloc(qk_u32_size(0));
    qk_u64 *w = malloc(qk_u64_size(t));
    uint32_t c32[16], d = 0;
    uint64_t hits[4];
    size_t nh = 0, len = 0;
    uint8_t buf[512];
    EXPECT(qk_u32_init(a, t), QK_OK);
    EXPECT(qk_u32_init(b, t + 1), QK_OK);
    EXPECT(qk_u32_init(z, 0), QK_OK);
    EXPECT(qk_u64_init(w, t), QK_OK);
    EXPECT(qk_u32_insert(z, 1), QK_E_THRESHOLD);
    EXPECT(qk_u32_remove(z, 1), QK_E_THRESHOLD);
    EXPECT(qk_u32_insert(NULL, 1), QK_E_INVAL);
    EXPECT(qk_u32_sub_assign(a, b), QK_E_MISMATCH);
    EXPECT(qk_u32_merge(a, b), QK_E_MISMATCH);
    for (uint32_t i = 0; i < t + 3; ++i) qk_u32_insert(a, (uint32_t)next());
    EXPECT(qk_u32_to_coeffs(a, c32, 16, &d), QK_E_UNDECODABLE);      /* count 11 > threshold 8 */
    qk_u32_init(a, t);
    for (uint32_t i = 0; i < 5; ++i) qk_u32_insert(a, (uint32_t)next());
    EXPECT(qk_u32_to_coeffs(a, c32, 2, &d), QK_E_CAPACITY);
    EXPECT(d == 5 ? QK_OK : -99, QK_OK);
    uint32_t log[64];
    for (int i = 0; i < 64; ++i) log[i] = (uint32_t)next();
    qk_u32_init(a, t);
    for (int i = 0; i < 6; ++i) qk_u32_insert(a, log[i * 9]);
    EXPECT(qk_u32_decode_host(a, log, 64, 0, hits, 4, &nh), QK_E_CAPACITY);   /* 6 hits, room for 4 */
    EXPECT(nh == 6 ? QK_OK : -99, QK_OK);
    /* bincode: truncated, trailing bytes, bad Option tag, non-canonical sums,
     * wrong threshold for the target sketch, random garbage */
    EXPECT(qk_u32_serialize(a, buf, sizeof buf, &len), QK_OK);
    EXPECT(qk_u32_serialize(a, buf, 3, &len), QK_E_CAPACITY);
    EXPECT(qk_u32_deserialize(buf, len - 1, NULL, &d), QK_E_FORMAT);
    EXPECT(qk_u32_deserialize(buf, len + 1, NULL, &d), QK_E_FORMAT);
    EXPECT(qk_u32_deserialize(buf, len, b, NULL), QK_E_MISMATCH);
    uint8_t bad[512];
    memcpy(bad, buf, len);
    bad[8 + 4 * t] = 7;   /* Option tag */
    EXPECT(qk_u32_deserialize(bad, len, a, NULL), QK_E_FORMAT);
    memcpy(bad, buf, len);
    memset(bad + 8, 0xFF, 4);   /* S_1 = 2^32 - 1 >= p */
    EXPECT(qk_u32_deserialize(bad, len, a, NULL), QK_E_FORMAT);
    for (int k = 0; k < 8; ++k) {
        const size_t n = next() % sizeof bad;
        for (size_t i = 0; i < n; ++i) bad[i] = (uint8_t)next();
        (void)qk_u32_deserialize(bad, n, NULL, &d);     /* any status, no crash, no leak */
        (void)qk_u64_deserialize(bad, n, NULL, &d);
    }
    EXPECT(qk_u64_insert(NULL, 1), QK_E_INVAL);
    free(a);
    free(b);
    free(z);
    free(w);
}

static void device_round(qk_ctx *ctx, uint32_t *d_log, size_t n, uint8_t *d_recs) {
    uint32_t host[16];
    qk_u32 *q = malloc(qk_u32_size(32)), *big = malloc(qk_u32_size(QK_MAX_THRESHOLD + 1));
    qk_u32_init(q, 32);
    qk_u32_init(big, QK_MAX_THRESHOLD + 1);
    uint64_t hits[2], part[64];
    size_t nh = 0, nf = 0;
    EXPECT(qk_u32_encode_device(ctx, host, 16, q, NULL), QK_E_INVAL);        /* host pointer */
    EXPECT(qk_u32_encode_device_async(ctx, d_log, n, 32, part, NULL), QK_E_INVAL);   /* host partial */
    EXPECT(qk_u32_encode_device(ctx, d_log, n, big, NULL), QK_E_THRESHOLD);
    EXPECT(qk_u32_encode_host(ctx, host, 16, big), QK_E_THRESHOLD);
    /* a polynomial whose roots are 40 log entries: capacity 2 -> QK_E_CAPACITY, then rerun */
    qk_u32 *r = malloc(qk_u32_size(40));
    qk_u32_init(r, 40);
    uint32_t h40[40];
    hipMemcpy(h40, d_log, sizeof h40, hipMemcpyDeviceToHost);
    for (int i = 0; i < 40; ++i) qk_u32_insert(r, h40[i]);
    EXPECT(qk_u32_decode_device(ctx, r, d_log, n, 0, hits, 2, &nh, NULL), QK_E_CAPACITY);
    EXPECT(nh >= 40 ? QK_OK : -99, QK_OK);
    for (int i = 0; i < 3; ++i) qk_u32_insert(r, (uint32_t)next());
    EXPECT(qk_u32_decode_device(ctx, r, d_log, n, 0, hits, 2, &nh, NULL), QK_E_UNDECODABLE);   /* count 43 > 40 */
    free(r);
    /* flows: 3 flows into room for 1 */
    qk_flow_key keys[1];
    uint8_t sk[4096];
    EXPECT(qk_u32_encode_flows_device(ctx, d_recs, 3, 67, NULL, NULL, 8, keys, sk, 1, &nf, NULL, NULL),
           QK_E_CAPACITY);
    EXPECT(nf == 3 ? QK_OK : -99, QK_OK);
    EXPECT(qk_u32_encode_flows_device(ctx, d_recs, 3, 66, NULL, NULL, 8, keys, sk, 1, &nf, NULL, NULL), QK_E_INVAL);
    free(q);
    free(big);
}

int main(int argc, char **argv) {
    const int device = argc > 1 && strcmp(argv[1], "device") == 0;
    const int rounds = argc > 2 ? atoi(argv[2]) : (device ? 300 : 3000);
    if (!device) {
        for (int i = 0; i < rounds; ++i) host_round();
        printf("abi_fail host ok: %d rounds\n", rounds);
        return 0;
    }
    qk_ctx *ctx = NULL;
    EXPECT(qk_ctx_create(0, &ctx), QK_OK);
    const size_t n = 1 << 20;
    uint32_t *d_log = NULL;
    uint8_t *d_recs = NULL;
    EXPECT(qk_fill_splitmix_u32(ctx, NULL, n, 1, 0, NULL), QK_E_INVAL);
    if (hipMalloc((void **)&d_log, n * 4) != hipSuccess || hipMalloc((void **)&d_recs, 3 * 67) != hipSuccess) return 1;
    EXPECT(qk_fill_splitmix_u32(ctx, d_log, n, 77, 0, NULL), QK_OK);
    /* three UDP records of three flows (byte 23 = 17, distinct src ips) */
    uint8_t recs[3 * 67];
    memset(recs, 0, sizeof recs);
    for (int i = 0; i < 3; ++i) { recs[i * 67 + 23] = 17; recs[i * 67 + 26] = (uint8_t)(i + 1); recs[i * 67 + 66] = (uint8_t)i; }
    hipMemcpy(d_recs, recs, sizeof recs, hipMemcpyHostToDevice);
    device_round(ctx, d_log, n, d_recs);      /* first round: every grow-only buffer reaches its size */
    hipDeviceSynchronize();
    size_t free0 = 0, total = 0, free1 = 0;
    hipMemGetInfo(&free0, &total);
    for (int i = 0; i < rounds; ++i) device_round(ctx, d_log, n, d_recs);
    hipDeviceSynchronize();
    hipMemGetInfo(&free1, &total);
    const long long lost = (long long)free0 - (long long)free1;
    printf("abi_fail device: %d rounds, device memory lost %lld bytes\n", rounds, lost);
    hipFree(d_log);
    hipFree(d_recs);
    qk_ctx_destroy(ctx);
    if (lost > (2ll << 20)) { fprintf(stderr, "abi_fail: device memory grew by %lld bytes\n", lost); return 1; }
    printf("abi_fail device ok\n");
    return 0;
}
