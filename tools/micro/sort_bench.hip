// Micro-benchmark: rocPRIM radix sort configurations for the finish's key sort
// (2.9 M pairs, 23-bit u32 keys, u32 rank payload).  hipcc --offload-arch=gfx950.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <cstdio>
#include <vector>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <class Config>
void run(const char *name, uint32_t *k0, uint32_t *v0, uint32_t *ka, uint32_t *kb_, uint32_t *va, uint32_t *vb_,
         size_t n, int bits) {
    size_t tb = 0;
    rocprim::double_buffer<uint32_t> kb(ka, kb_);
    rocprim::double_buffer<uint32_t> vb(va, vb_);
    CK(rocprim::radix_sort_pairs<Config>(nullptr, tb, kb, vb, n, 0, bits));
    void *t;
    CK(hipMalloc(&t, tb));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float best = 1e9, tot = 0;
    for (int it = 0; it < 14; ++it) {
        CK(hipMemcpy(ka, k0, n * 4, hipMemcpyDeviceToDevice));
        CK(hipMemcpy(va, v0, n * 4, hipMemcpyDeviceToDevice));
        rocprim::double_buffer<uint32_t> kb2(ka, kb_);
        rocprim::double_buffer<uint32_t> vb2(va, vb_);
        hipEventRecord(a, 0);
        CK(rocprim::radix_sort_pairs<Config>(t, tb, kb2, vb2, n, 0, bits));
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (it >= 4) { tot += ms; if (ms < best) best = ms; }
    }
    printf("%-44s avg %7.1f us  best %7.1f us\n", name, tot / 10 * 1000, best * 1000);
    hipFree(t);
}

int main() {
    const size_t n = 2900000;
    std::vector<uint32_t> hk(n), hv(n);
    std::mt19937_64 rng(1);
    for (size_t i = 0; i < n; ++i) {
        hk[i] = (i % 11 == 0) ? (1u << 22) : (uint32_t)(rng() & ((1u << 22) - 1));
        hv[i] = (uint32_t)i;
    }
    uint32_t *k0, *ka, *kb, *v0, *va, *vb;
    CK(hipMalloc(&k0, n * 4)); CK(hipMalloc(&ka, n * 4)); CK(hipMalloc(&kb, n * 4));
    CK(hipMalloc(&v0, n * 4)); CK(hipMalloc(&va, n * 4)); CK(hipMalloc(&vb, n * 4));
    CK(hipMemcpy(k0, hk.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(v0, hv.data(), n * 4, hipMemcpyHostToDevice));
    using namespace rocprim;
    run<default_config>("default", k0, v0, ka, kb, va, vb, n, 23);
#define CFG(HB, HI, SB, SI, BITS) \
    run<radix_sort_config<default_config, default_config, \
        radix_sort_onesweep_config<kernel_config<HB, HI>, kernel_config<SB, SI>, BITS>>>( \
        "hist " #HB "x" #HI " sort " #SB "x" #SI " bits " #BITS, k0, v0, ka, kb, va, vb, n, 23)
    CFG(256, 12, 256, 12, 8);
    CFG(256, 16, 256, 8, 8);
    CFG(256, 8, 256, 16, 8);
    CFG(256, 12, 256, 12, 6);
    CFG(256, 12, 256, 24, 4);
    return 0;
}
