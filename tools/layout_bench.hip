// Random-row read-modify-write bandwidth: weights and Adagrad slots in separate
// tables ([N][d] + [N][d]) vs interleaved ([N][2d] = w | acc), d = 64 / 128.
// One lane-group of d/4 lanes per row (float4 per lane), like the step kernels.
// Build: hipcc --offload-arch=gfx950 -O3 tools/layout_bench.hip -o tools/layout_bench
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int LPR>
__global__ void k_sep(float* __restrict__ w, float* __restrict__ a, const int* __restrict__ rows, int n, int d) {
  const int64_t g = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / LPR;
  const int l = threadIdx.x & (LPR - 1);
  if (g >= n) return;
  const int64_t r = rows[g];
  float4* pw = reinterpret_cast<float4*>(w + r * d) + l;
  float4* pa = reinterpret_cast<float4*>(a + r * d) + l;
  float4 x = *pw, c = *pa;
  c.x += 1e-3f; c.y += 1e-3f; c.z += 1e-3f; c.w += 1e-3f;
  x.x -= 1e-4f * c.x; x.y -= 1e-4f * c.y; x.z -= 1e-4f * c.z; x.w -= 1e-4f * c.w;
  *pw = x; *pa = c;
}

template <int LPR>
__global__ void k_int(float* __restrict__ wa, const int* __restrict__ rows, int n, int d) {
  const int64_t g = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / LPR;
  const int l = threadIdx.x & (LPR - 1);
  if (g >= n) return;
  const int64_t r = rows[g];
  float4* pw = reinterpret_cast<float4*>(wa + r * 2 * d) + l;
  float4* pa = reinterpret_cast<float4*>(wa + r * 2 * d + d) + l;
  float4 x = *pw, c = *pa;
  c.x += 1e-3f; c.y += 1e-3f; c.z += 1e-3f; c.w += 1e-3f;
  x.x -= 1e-4f * c.x; x.y -= 1e-4f * c.y; x.z -= 1e-4f * c.z; x.w -= 1e-4f * c.w;
  *pw = x; *pa = c;
}

template <class F>
static float time_us(F f, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  f();
  (void)hipEventRecord(a, 0);
  for (int i = 0; i < reps; ++i) f();
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0; (void)hipEventElapsedTime(&ms, a, b);
  return 1000.f * ms / reps;
}

template <int LPR>
static int run(int d, int64_t N, int n) {
  std::vector<int> hr(n);
  std::mt19937_64 rng(7);
  for (auto& x : hr) x = (int)(rng() % N);
  int* rows; float *w, *a, *wa;
  CK(hipMalloc(&rows, n * 4));
  CK(hipMalloc(&w, N * d * 4)); CK(hipMalloc(&a, N * d * 4)); CK(hipMalloc(&wa, N * 2 * d * 4));
  CK(hipMemset(w, 0, N * d * 4)); CK(hipMemset(a, 0, N * d * 4)); CK(hipMemset(wa, 0, N * 2 * d * 4));
  CK(hipMemcpy(rows, hr.data(), n * 4, hipMemcpyHostToDevice));
  const int threads = n * LPR, grid = (threads + 255) / 256;
  float ts = time_us([&] { k_sep<LPR><<<grid, 256>>>(w, a, rows, n, d); }, 20);
  float ti = time_us([&] { k_int<LPR><<<grid, 256>>>(wa, rows, n, d); }, 20);
  const double bytes = (double)n * d * 4 * 4;  // w + acc, read + write
  printf("d=%d rows=%lld updates=%d  separate: %.1f us %.0f GB/s   interleaved: %.1f us %.0f GB/s\n", d,
         (long long)N, n, ts, bytes / ts / 1e3, ti, bytes / ti / 1e3);
  CK(hipFree(rows)); CK(hipFree(w)); CK(hipFree(a)); CK(hipFree(wa));
  return 0;
}

int main() {
  const int64_t N = 10000000;
  for (int n : {65536 * 3, 65536 * 12}) {
    if (run<16>(64, N, n)) return 1;
    if (run<32>(128, N, n)) return 1;
  }
  return 0;
}
