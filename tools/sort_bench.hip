// Sort variants for the dedup plan: rocprim radix_sort_keys on u64 keys vs
// radix_sort_pairs on u32 keys + u32 values, at plan sizes.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/sort_bench.hip -o tools/sort_bench
#include <cstring>
#include <algorithm>
#include <hip/hip_runtime.h>
#include <rocprim/rocprim.hpp>

#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <class F>
static float time_it(F f, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  f();
  (void)hipEventRecord(a, 0);
  for (int r = 0; r < reps; ++r) f();
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0; (void)hipEventElapsedTime(&ms, a, b);
  return 1000.f * ms / reps;
}

int main() {
  const size_t sizes[] = {1u << 17, 1u << 19, 1u << 20, 1u << 21, 1u << 22};
  for (size_t n : sizes) {
    std::vector<uint64_t> hk(n);
    std::vector<uint32_t> hk32(n), hv(n);
    std::mt19937_64 rng(1);
    const int ob = 64 - __builtin_clzll(n);
    const uint32_t nb = 8;
    for (size_t x = 0; x < n; ++x) {
      uint64_t t = x * nb / n, row = rng() % 5000001ull;
      hk[x] = ((t * 5000001ull + row) << ob) | x;
      hk32[x] = (uint32_t)(t * 5000001ull + row);
      hv[x] = (uint32_t)x;
    }
    uint64_t *k, *ko; uint32_t *k32, *k32o, *v, *vo;
    CK(hipMalloc(&k, n * 8)); CK(hipMalloc(&ko, n * 8));
    CK(hipMalloc(&k32, n * 4)); CK(hipMalloc(&k32o, n * 4)); CK(hipMalloc(&v, n * 4)); CK(hipMalloc(&vo, n * 4));
    CK(hipMemcpy(k, hk.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(k32, hk32.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(v, hv.data(), n * 4, hipMemcpyHostToDevice));
    const int kbits = 64 - __builtin_clzll((uint64_t)nb * 5000001ull);
    size_t t1 = 0, t2 = 0;
    CK(rocprim::radix_sort_keys(nullptr, t1, k, ko, n, 0, ob + kbits));
    CK(rocprim::radix_sort_pairs(nullptr, t2, k32, k32o, v, vo, n, 0, kbits));
    void* tmp; CK(hipMalloc(&tmp, std::max(t1, t2) + 16));
    float us64 = time_it([&] { size_t tb = t1; (void)rocprim::radix_sort_keys(tmp, tb, k, ko, n, 0, ob + kbits); }, 20);
    float us32 = time_it([&] { size_t tb = t2; (void)rocprim::radix_sort_pairs(tmp, tb, k32, k32o, v, vo, n, 0, kbits); }, 20);
    printf("n=%zu keys64(%d bits): %.1f us   pairs32(%d bits): %.1f us\n", n, ob + kbits, us64, kbits, us32);
    CK(hipFree(k)); CK(hipFree(ko)); CK(hipFree(k32)); CK(hipFree(k32o)); CK(hipFree(v)); CK(hipFree(vo)); CK(hipFree(tmp));
  }
  return 0;
}
