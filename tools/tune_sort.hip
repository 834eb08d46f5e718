// A/B harness for the per-flow batch's grouping sort (flows.hip step 3):
// stable (slot key, id) pair sort over the key's low `bits` bits, hipCUB's
// default onesweep (8-bit digits) against rocPRIM onesweep configs with
// wider digits (fewer passes).  Keys: 1e6 flows on random slots of a 4M-slot
// table (22 bits), each packet of a random flow — the 1e6-flow batch shape.
// Every config's output is compared with the default's (stable sorts:
// identical).  Not product code.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rocprim/rocprim.hpp>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <cstring>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

static uint64_t sm(uint64_t &s) {
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

using rocprim::kernel_config;
using rocprim::block_radix_rank_algorithm;

template <unsigned HB, unsigned HI, unsigned SB, unsigned SI, unsigned R, block_radix_rank_algorithm A>
using OS = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                      rocprim::radix_sort_onesweep_config<kernel_config<HB, HI>, kernel_config<SB, SI>, R, A>,
                                      0>;

struct Bufs { uint32_t *k, *v, *k2, *v2; size_t n; int bits; };

template <class Cfg>
static float run(const char *name, Bufs &b, const std::vector<uint32_t> &want_k, const std::vector<uint32_t> &want_v,
                 hipStream_t s) {
    size_t tb = 0;
    CK(rocprim::radix_sort_pairs<Cfg>(nullptr, tb, b.k, b.k2, b.v, b.v2, b.n, 0, b.bits, s));
    void *tmp; CK(hipMalloc(&tmp, tb));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) CK(rocprim::radix_sort_pairs<Cfg>(tmp, tb, b.k, b.k2, b.v, b.v2, b.n, 0, b.bits, s));
    const int R = 20;
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < R; ++i) CK(rocprim::radix_sort_pairs<Cfg>(tmp, tb, b.k, b.k2, b.v, b.v2, b.n, 0, b.bits, s));
    CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= R;
    bool ok = true;
    if (!want_k.empty()) {
        std::vector<uint32_t> gk(b.n), gv(b.n);
        CK(hipMemcpy(gk.data(), b.k2, b.n * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(gv.data(), b.v2, b.n * 4, hipMemcpyDeviceToHost));
        ok = !memcmp(gk.data(), want_k.data(), b.n * 4) && !memcmp(gv.data(), want_v.data(), b.n * 4);
    }
    printf("{\"config\": \"%s\", \"n\": %zu, \"bits\": %d, \"ms\": %.4f, \"temp_mb\": %.1f, \"identical\": %s}\n", name, b.n,
           b.bits, ms, tb / 1048576.0, ok ? "true" : "false");
    fflush(stdout);
    CK(hipFree(tmp));
    return ms;
}

int main(int argc, char **argv) {
    size_t n = argc > 1 ? strtoull(argv[1], 0, 0) : 100000000;
    int nflows = argc > 2 ? atoi(argv[2]) : 1000000;
    int bits = argc > 3 ? atoi(argv[3]) : 22;
    std::vector<uint32_t> fslot(nflows), hk(n), hv(n);
    uint64_t st = 7;
    for (int f = 0; f < nflows; ++f) fslot[f] = (uint32_t)(sm(st) & ((1u << bits) - 2));
    for (size_t i = 0; i < n; ++i) { hk[i] = fslot[sm(st) % nflows]; hv[i] = (uint32_t)sm(st); }
    Bufs b{nullptr, nullptr, nullptr, nullptr, n, bits};
    CK(hipMalloc(&b.k, n * 4)); CK(hipMalloc(&b.v, n * 4)); CK(hipMalloc(&b.k2, n * 4)); CK(hipMalloc(&b.v2, n * 4));
    CK(hipMemcpy(b.k, hk.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(b.v, hv.data(), n * 4, hipMemcpyHostToDevice));
    hipStream_t s; CK(hipStreamCreate(&s));

    // baseline: hipCUB default
    {
        size_t tb = 0;
        CK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, b.k, b.k2, b.v, b.v2, (uint32_t)n, 0, bits, s));
        void *tmp; CK(hipMalloc(&tmp, tb));
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        for (int i = 0; i < 3; ++i) CK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, b.k, b.k2, b.v, b.v2, (uint32_t)n, 0, bits, s));
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < 20; ++i) CK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, b.k, b.k2, b.v, b.v2, (uint32_t)n, 0, bits, s));
        CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"config\": \"hipcub_default\", \"n\": %zu, \"bits\": %d, \"ms\": %.4f}\n", n, bits, ms / 20);
        CK(hipFree(tmp));
    }
    std::vector<uint32_t> wk(n), wv(n);
    CK(hipMemcpy(wk.data(), b.k2, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(wv.data(), b.v2, n * 4, hipMemcpyDeviceToHost));
    constexpr auto M = block_radix_rank_algorithm::match;
    run<OS<256, 12, 256, 12, 8, M>>("os8_256x12_match", b, wk, wv, s);
    run<OS<256, 12, 512, 12, 8, M>>("os8_512x12_match", b, wk, wv, s);
    run<OS<256, 12, 256, 12, 11, M>>("os11_256x12_match", b, wk, wv, s);
    run<OS<256, 12, 512, 12, 11, M>>("os11_512x12_match", b, wk, wv, s);
    run<OS<256, 12, 512, 16, 11, M>>("os11_512x16_match", b, wk, wv, s);
    run<OS<256, 12, 1024, 8, 11, M>>("os11_1024x8_match", b, wk, wv, s);
    run<OS<256, 12, 256, 16, 11, M>>("os11_256x16_match", b, wk, wv, s);
    return 0;
}
