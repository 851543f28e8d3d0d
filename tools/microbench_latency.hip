// Latency floor probes for the B = 512 APR step (not part of the product).
//  1. empty kernel: hipExt event duration and per-node time in a hipGraph chain
//  2. dependent-load chain of L levels (pointer chase over a 4 MB buffer that
//     another kernel rewrote just before: the state the step kernels see)
// Build: hipcc --offload-arch=gfx950 -O3 microbench_latency.hip -o mb
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("%s: %s\n", #x, hipGetErrorString(e));                            \
      return 1;                                                                \
    }                                                                          \
  } while (0)

__global__ void k_empty(int* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0xFFFFFF) p[0] = 1;
}

__global__ void k_touch(int* buf, int n, int salt) {
  int x = blockIdx.x * blockDim.x + threadIdx.x;
  if (x < n) buf[x] = (buf[x] & 0x3FFFFF) | (salt << 22 & 0);
}

__global__ void k_chase(const int* __restrict__ buf, int levels, int* out) {
  int x = (blockIdx.x * blockDim.x + threadIdx.x) * 977;
  int v = x & 0xFFFFF;
  for (int l = 0; l < levels; ++l) v = buf[v] & 0xFFFFF;
  if (v == -1) out[0] = v;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int n = 1 << 20;
  int* buf;
  int* out;
  CK(hipMalloc(&buf, n * 4));
  CK(hipMalloc(&out, 64));
  std::vector<int> h(n);
  for (int i = 0; i < n; ++i) h[i] = (int)((i * 2654435761u) >> 12) & 0xFFFFF;
  CK(hipMemcpy(buf, h.data(), n * 4, hipMemcpyHostToDevice));
  const int grids[] = {1, 96, 256, 1024};
  for (int g : grids) {
    float tot = 0;
    for (int r = 0; r < 200; ++r) {
      hipExtLaunchKernelGGL(k_empty, dim3(g), dim3(256), 0, s, e0, e1, 0, (int*)nullptr);
      CK(hipStreamSynchronize(s));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 20) tot += ms;
    }
    printf("empty kernel grid=%d: hipExt event duration %.3f us\n", g, 1e3 * tot / 180);
  }
  // graph chain of N empty kernels
  for (int g : {96, 256}) {
    const int N = 2000;
    hipGraph_t gr;
    hipGraphExec_t ex;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < N; ++i) k_empty<<<g, 256, 0, s>>>(nullptr);
    CK(hipStreamEndCapture(s, &gr));
    CK(hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ex, s));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < 5; ++r) CK(hipGraphLaunch(ex, s));
    CK(hipEventRecord(e1, s));
    CK(hipStreamSynchronize(s));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("graph chain of %d empty kernels grid=%d: %.3f us per node\n", N, g, 1e3 * ms / (5 * N));
  }
  // dependent-load chains right after a rewrite of the buffer
  for (int L : {0, 1, 2, 4, 8}) {
    float tot = 0;
    for (int r = 0; r < 100; ++r) {
      k_touch<<<n / 256, 256, 0, s>>>(buf, n, r);
      hipExtLaunchKernelGGL(k_chase, dim3(96), dim3(256), 0, s, e0, e1, 0, (const int*)buf, L, out);
      CK(hipStreamSynchronize(s));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 10) tot += ms;
    }
    printf("dependent chain L=%d (after rewrite, 96 WGs): %.3f us\n", L, 1e3 * tot / 90);
  }
  for (int L : {1, 4, 8}) {
    float tot = 0;
    for (int r = 0; r < 100; ++r) {
      hipExtLaunchKernelGGL(k_chase, dim3(96), dim3(256), 0, s, e0, e1, 0, (const int*)buf, L, out);
      CK(hipStreamSynchronize(s));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 10) tot += ms;
    }
    printf("dependent chain L=%d (warm, 96 WGs): %.3f us\n", L, 1e3 * tot / 90);
  }
  return 0;
}
