// FETCH_SIZE / WRITE_SIZE calibration for the access widths of the step kernels
// (MI355X_MICROARCH §HBM: "other access widths are uncalibrated: calibrate on a
// known byte count in your own access pattern").  Each kernel touches exactly
// `bytes` of a buffer far larger than the 256 MiB Infinity Cache:
//   kind 0: 16-B/lane plain loads (float4), the guide's calibrated case
//   kind 1: 8-B/lane relaxed agent-scope atomic loads, four consecutive granules
//           per lane (try_row's version-granule read in k_stream)
//   kind 2: 8-B/lane relaxed agent-scope atomic stores, same layout (store_ver
//           before the component-major granule order)
//   kind 3: the same stores, each instruction's lanes on consecutive granules
//           (store_ver's component-major order)
// Built by tools/calib_fetch.py; run under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned long long u64;

__global__ void k_read16(const float4* __restrict__ src, int64_t n, float* __restrict__ sink) {
  float acc = 0.f;
  for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < n; x += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = src[x];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 1234.5f) sink[0] = acc;
}

// one lane = 4 consecutive granules (32 B), 16 lanes = one 512-B row group
__global__ void k_read_granules(const u64* __restrict__ src, int64_t n4, float* __restrict__ sink) {
  u64 acc = 0;
  for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < n4; x += (int64_t)gridDim.x * blockDim.x) {
    const u64* g = src + 4 * x;
#pragma unroll
    for (int e = 0; e < 4; ++e) acc += __hip_atomic_load(g + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (acc == 12345ull) sink[0] = 1.f;
}

__global__ void k_write_granules(u64* __restrict__ dst, int64_t n4) {
  for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < n4; x += (int64_t)gridDim.x * blockDim.x) {
    u64* g = dst + 4 * x;
#pragma unroll
    for (int e = 0; e < 4; ++e) __hip_atomic_store(g + e, (u64)x + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void k_write_granules_cm(u64* __restrict__ dst, int64_t n4) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < n4; x += stride) {
    // lane-consecutive granules: wave w's 4 stores cover 4 contiguous 512-B runs
    const int64_t w = x >> 6, l = x & 63;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      __hip_atomic_store(dst + (w * 4 + e) * 64 + l, (u64)x + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

extern "C" int calib_run(int kind, void* buf, int64_t bytes, float* sink) {
  const dim3 grid(4096), block(256);
  if (kind == 0)
    hipLaunchKernelGGL(k_read16, grid, block, 0, 0, (const float4*)buf, bytes / 16, sink);
  else if (kind == 1)
    hipLaunchKernelGGL(k_read_granules, grid, block, 0, 0, (const u64*)buf, bytes / 32, sink);
  else if (kind == 2)
    hipLaunchKernelGGL(k_write_granules, grid, block, 0, 0, (u64*)buf, bytes / 32);
  else
    hipLaunchKernelGGL(k_write_granules_cm, grid, block, 0, 0, (u64*)buf, bytes / 32);
  if (hipGetLastError() != hipSuccess) return 1;
  return hipDeviceSynchronize() == hipSuccess ? 0 : 2;
}
