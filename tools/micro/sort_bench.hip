// Micro-benchmark: rocPRIM radix sort configurations for the finish's key sort
// (2.6 M pairs, 23-bit keys, u32 rank payload).  hipcc --offload-arch=gfx950.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <cstdio>
#include <vector>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <class Config, class K>
float run(const char *name, K *k0, uint32_t *v0, K *kbuf, K *kbuf2, uint32_t *vbuf, uint32_t *vbuf2, size_t n, int bits) {
    size_t tb = 0;
    rocprim::double_buffer<K> kb(kbuf, kbuf2);
    rocprim::double_buffer<uint32_t> vb(vbuf, vbuf2);
    CK(rocprim::radix_sort_pairs<Config>(nullptr, tb, kb, vb, n, 0, bits));
    void *t;
    CK(hipMalloc(&t, tb));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float best = 1e9, tot = 0;
    for (int it = 0; it < 12; ++it) {
        CK(hipMemcpy(kbuf, k0, n * sizeof(K), hipMemcpyDeviceToDevice));
        CK(hipMemcpy(vbuf, v0, n * 4, hipMemcpyDeviceToDevice));
        rocprim::double_buffer<K> kb2(kbuf, kbuf2);
        rocprim::double_buffer<uint32_t> vb2(vbuf, vbuf2);
        hipEventRecord(a, 0);
        CK(rocprim::radix_sort_pairs<Config>(t, tb, kb2, vb2, n, 0, bits));
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (it >= 2) { tot += ms; if (ms < best) best = ms; }
    }
    printf("%-40s n=%zu bits=%d  avg %.1f us  best %.1f us\n", name, n, bits, tot / 10 * 1000, best * 1000);
    hipFree(t);
    return best;
}

int main() {
    const size_t n = 2635074 + 300000;
    std::vector<uint64_t> hk(n);
    std::vector<uint32_t> hv(n);
    std::mt19937_64 rng(1);
    for (size_t i = 0; i < n; ++i) {
        hk[i] = (i % 10 == 0) ? (1ull << 22) : (rng() & ((1ull << 22) - 1));
        hv[i] = (uint32_t)i;
    }
    std::vector<uint32_t> hk32(n);
    for (size_t i = 0; i < n; ++i) hk32[i] = (uint32_t)hk[i];
    uint64_t *k64, *a64, *b64;
    uint32_t *k32, *a32, *b32, *v0, *va, *vb;
    CK(hipMalloc(&k64, n * 8)); CK(hipMalloc(&a64, n * 8)); CK(hipMalloc(&b64, n * 8));
    CK(hipMalloc(&k32, n * 4)); CK(hipMalloc(&a32, n * 4)); CK(hipMalloc(&b32, n * 4));
    CK(hipMalloc(&v0, n * 4)); CK(hipMalloc(&va, n * 4)); CK(hipMalloc(&vb, n * 4));
    CK(hipMemcpy(k64, hk.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(k32, hk32.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(v0, hv.data(), n * 4, hipMemcpyHostToDevice));
    using namespace rocprim;
    run<default_config>("u64 key default", k64, v0, a64, b64, va, vb, n, 23);
    run<default_config>("u32 key default", k32, v0, a32, b32, va, vb, n, 23);
    using C12 = radix_sort_config<default_config, default_config,
                                  radix_sort_onesweep_config<kernel_config<512, 32>, kernel_config<512, 12>, 12>>;
    using C11 = radix_sort_config<default_config, default_config,
                                  radix_sort_onesweep_config<kernel_config<512, 32>, kernel_config<512, 12>, 11>>;
    using C12b = radix_sort_config<default_config, default_config,
                                   radix_sort_onesweep_config<kernel_config<1024, 16>, kernel_config<1024, 8>, 12>>;
    run<C12>("u32 key 12 bits 512x12", k32, v0, a32, b32, va, vb, n, 23);
    run<C11>("u32 key 11 bits 512x12", k32, v0, a32, b32, va, vb, n, 23);
    run<C12b>("u32 key 12 bits 1024x8", k32, v0, a32, b32, va, vb, n, 23);
    run<C12>("u64 key 12 bits 512x12", k64, v0, a64, b64, va, vb, n, 23);
    run<C11>("u64 key 11 bits 512x12", k64, v0, a64, b64, va, vb, n, 23);
    return 0;
}
