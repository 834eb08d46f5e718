/* abi_c.c — the C ABI used from plain C exactly as the Rust FFI binds it
 * (include/quack_hip.h): the receiver sequence of
 * media_client.rs:223-321, one quACK round, with bincode on the wire.
 *
 *   abi_c host      host functions only (runs in the CPU test suite)
 *   abi_c device    the same round with the log's root test on the GPU
 *                   (qk_u32_decode_device) and the sender's batch encode
 *                   (qk_u32_encode_host), checked against the host round
 *
 * Sender: sends n ids, logs (seqno, id).  Proxy: sees all but a few of them
 * (inserted per packet, sidekick.rs:42) and ships its quACK serialized.
 * Receiver: deserialize (:227); skip if last values match (:233); insert the
 * log prefix up to the quACK's last value (:240-252); reset rules (:258-261);
 * diff = my.clone(); diff.sub_assign(quack) (:295-296); to_coeffs (:304);
 * scan the log, stopping at diff.last_value (:306-313); remove the missing
 * ids from my quACK (:319).  Exit status 0 iff every check passes.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "quack_hip.h"

#define CHECK(c)                                                                                   \
    do {                                                                                           \
        if (!(c)) {                                                                                \
            fprintf(stderr, "abi_c: check failed at line %d: %s\n", __LINE__, #c);                \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)
#define OK(rc) CHECK((rc) == QK_OK)

/* hipMalloc / hipMemcpy / hipFree, resolved only in device mode */
typedef int (*malloc_fn)(void **, size_t);
typedef int (*memcpy_fn)(void *, const void *, size_t, int);
typedef int (*free_fn)(void *);
#include <dlfcn.h>

static uint32_t next_id(uint64_t *s) { /* splitmix64, high half */
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return (uint32_t)((z ^ (z >> 31)) >> 32);
}

int main(int argc, char **argv) {
    const int device = argc > 1 && strcmp(argv[1], "device") == 0;
    const uint32_t t = 16, n = 5000;
    const uint32_t drop_at[] = {17, 1203, 2999, 4321};   /* lost before the proxy */
    uint32_t *ids = malloc(n * 4);
    uint64_t seed = 0xC0FFEE;
    for (uint32_t i = 0; i < n; ++i) ids[i] = next_id(&seed);

    /* proxy: per-packet inserts (sidekick.rs:42), then bincode (sidekick.rs:187) */
    qk_u32 *proxy = malloc(qk_u32_size(t));
    OK(qk_u32_init(proxy, t));
    for (uint32_t i = 0, k = 0; i < n; ++i) {
        if (k < 4 && i == drop_at[k]) { ++k; continue; }
        OK(qk_u32_insert(proxy, ids[i]));
    }
    const size_t wlen = qk_u32_serialized_size(proxy);
    uint8_t *wire = malloc(wlen);
    size_t got = 0;
    OK(qk_u32_serialize(proxy, wire, wlen, &got));
    CHECK(got == wlen && wlen == 8 + 4 * t + 1 + 4 + 4);

    /* receiver: bincode::deserialize (media_client.rs:227) */
    uint32_t tq = 0;
    OK(qk_u32_deserialize(wire, wlen, NULL, &tq));
    CHECK(tq == t);
    qk_u32 *quack = malloc(qk_u32_size(tq));
    OK(qk_u32_init(quack, tq));
    OK(qk_u32_deserialize(wire, wlen, quack, NULL));
    CHECK(memcmp(quack, proxy, qk_u32_size(t)) == 0);
    qk_u32 *small = malloc(qk_u32_size(4));
    OK(qk_u32_init(small, 4));
    CHECK(qk_u32_deserialize(wire, wlen, small, NULL) == QK_E_MISMATCH);   /* wrong-size sketch refused */

    qk_u32 *my = malloc(qk_u32_size(t));
    OK(qk_u32_init(my, t));
    CHECK(!(quack->has_last && my->has_last && quack->last_value == my->last_value));   /* :233 */
    long last_index = -1;                                                                /* :240-246 */
    for (uint32_t i = 0; i < n; ++i)
        if (quack->has_last && ids[i] == quack->last_value) { last_index = i; break; }
    CHECK(last_index == n - 1);
    if (device) {                                                      /* :247-252 as one batch */
        qk_ctx *ctx = NULL;
        OK(qk_ctx_create(0, &ctx));
        OK(qk_u32_encode_host(ctx, ids, (size_t)last_index + 1, my));
        qk_ctx_destroy(ctx);
    } else {
        for (long i = 0; i <= last_index; ++i) OK(qk_u32_insert(my, ids[i]));
    }
    const int reset1 = my->count < quack->count;                       /* :258-261 */
    const int reset2 = my->count > (uint32_t)(quack->count + t);
    CHECK(!reset1 && !reset2);

    qk_u32 *diff = malloc(qk_u32_size(t));                             /* :295-296 */
    memcpy(diff, my, qk_u32_size(t));
    OK(qk_u32_sub_assign(diff, quack));
    CHECK(diff->count == 4 && diff->has_last && diff->last_value == ids[n - 1]);

    uint32_t coeffs[16], d = 0;                                        /* :304 */
    OK(qk_u32_to_coeffs(diff, coeffs, 16, &d));
    CHECK(d == 4);
    uint32_t missing[16];                                              /* :306-313 */
    uint32_t nm = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (diff->has_last && ids[i] == diff->last_value) break;
        if (qk_u32_eval(coeffs, d, ids[i]) == 0) missing[nm++] = i;
    }
    CHECK(nm == 4);
    for (uint32_t k = 0; k < 4; ++k) CHECK(missing[k] == drop_at[k]);

    /* the same scan as one call: host, and (device mode) the GPU root test */
    uint64_t hits[16];
    size_t nh = 0;
    OK(qk_u32_decode_host(diff, ids, n, 1, hits, 16, &nh));
    CHECK(nh == 4);
    for (uint32_t k = 0; k < 4; ++k) CHECK(hits[k] == drop_at[k]);
    if (device) {
        void *h = dlopen("libamdhip64.so", RTLD_NOW | RTLD_GLOBAL);
        CHECK(h != NULL);
        malloc_fn hmalloc = (malloc_fn)dlsym(h, "hipMalloc");
        memcpy_fn hmemcpy = (memcpy_fn)dlsym(h, "hipMemcpy");
        free_fn hfree = (free_fn)dlsym(h, "hipFree");
        CHECK(hmalloc && hmemcpy && hfree);
        void *dlog = NULL;
        CHECK(hmalloc(&dlog, n * 4) == 0);
        CHECK(hmemcpy(dlog, ids, n * 4, 1 /* hipMemcpyHostToDevice */) == 0);
        qk_ctx *ctx = NULL;
        OK(qk_ctx_create(0, &ctx));
        uint64_t dh[16];
        size_t dn = 0;
        OK(qk_u32_decode_device(ctx, diff, dlog, n, 1, dh, 16, &dn, NULL));
        CHECK(dn == 4 && memcmp(dh, hits, 4 * sizeof(uint64_t)) == 0);
        qk_ctx_destroy(ctx);
        CHECK(hfree(dlog) == 0);
    }

    for (uint32_t k = 0; k < nm; ++k) OK(qk_u32_remove(my, ids[missing[k]]));   /* :319 */
    CHECK(my->count == quack->count);
    for (uint32_t k = 0; k < t; ++k) CHECK(my->power_sums[k] == quack->power_sums[k]);

    printf("abi_c %s ok: %u ids, %u missing recovered, wire %zu bytes\n", device ? "device" : "host", n, nm, wlen);
    free(ids); free(proxy); free(wire); free(quack); free(small); free(my); free(diff);
    return 0;
}
