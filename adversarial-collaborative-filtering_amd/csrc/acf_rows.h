// acf_rows.h — device row helpers shared by the APR step kernels (acf_apr.hip)
// and the decomposed per-op kernels (acf_ops.hip): row-group loads/stores, the
// TF-order dot product, the BPR term, and the counter-based RNG.
#ifndef ACF_ROWS_H
#define ACF_ROWS_H

#include <hip/hip_runtime.h>
#include <stdint.h>

// ---------------------------------------------------------------------------
// A table row of `d` floats is held by a row-group of LPR lanes, NV float4 per
// lane: lane l owns float4 chunks c = l + LPR*v.  LPR is a power of two <= 64,
// so row-groups never straddle a wavefront and reduce with __shfl_xor.
template <int NV>
struct RowV {
  float4 v[NV];
};

template <int LPR, int NV>
__device__ __forceinline__ RowV<NV> load_row(const float* __restrict__ base, int64_t row,
                                             int d, int l) {
  RowV<NV> r;
  const float* p = base + row * (int64_t)d;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    int c = l + LPR * v;
    if (c * 4 < d)
      r.v[v] = *reinterpret_cast<const float4*>(p + c * 4);
    else
      r.v[v] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  return r;
}

template <int LPR, int NV>
__device__ __forceinline__ void store_row(float* __restrict__ base, int64_t row, int d, int l,
                                          const RowV<NV>& r) {
  float* p = base + row * (int64_t)d;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    int c = l + LPR * v;
    if (c * 4 < d) *reinterpret_cast<float4*>(p + c * 4) = r.v[v];
  }
}

// store_row with device-scope write-through stores (sc1): once the wave's
// vmcnt drains they are visible to every XCD, with no L2 write-back (the
// release fence a flag would otherwise need writes back the whole L2).
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <int LPR, int NV>
__device__ __forceinline__ void store_row_wt(float* __restrict__ base, int64_t row, int d, int l,
                                             const RowV<NV>& r) {
  float* p = base + row * (int64_t)d;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    int c = l + LPR * v;
    if (c * 4 < d) {
      const f32x4 x = {r.v[v].x, r.v[v].y, r.v[v].z, r.v[v].w};
      // s_nop 1 inside the string: without it hipcc's next instruction may
      // overwrite the data registers before the store has read them (MI355X
      // guide, inline-asm stores)
      asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p + c * 4), "v"(x) : "memory");
    }
  }
}

template <int NV>
__device__ __forceinline__ RowV<NV> zero_row() {
  RowV<NV> r;
#pragma unroll
  for (int v = 0; v < NV; ++v) r.v[v] = make_float4(0.f, 0.f, 0.f, 0.f);
  return r;
}

template <int NV>
__device__ __forceinline__ RowV<NV> add_row(const RowV<NV>& a, const RowV<NV>& b) {
  RowV<NV> r;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    r.v[v].x = a.v[v].x + b.v[v].x;
    r.v[v].y = a.v[v].y + b.v[v].y;
    r.v[v].z = a.v[v].z + b.v[v].z;
    r.v[v].w = a.v[v].w + b.v[v].w;
  }
  return r;
}

// acc += s * x with the product rounded first (TF's IndexedSlices sums are of
// rounded products, so contributions that cancel, e.g. item i == j, cancel
// exactly instead of leaving an fma residue that l2_normalize would blow up)
template <int NV>
__device__ __forceinline__ void axpy_row(RowV<NV>& acc, float s, const RowV<NV>& x) {
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    acc.v[v].x = acc.v[v].x + s * x.v[v].x;
    acc.v[v].y = acc.v[v].y + s * x.v[v].y;
    acc.v[v].z = acc.v[v].z + s * x.v[v].z;
    acc.v[v].w = acc.v[v].w + s * x.v[v].w;
  }
}

template <int NV>
__device__ __forceinline__ RowV<NV> scale_row(const RowV<NV>& a, float s) {
  RowV<NV> r;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    r.v[v].x = a.v[v].x * s;
    r.v[v].y = a.v[v].y * s;
    r.v[v].z = a.v[v].z * s;
    r.v[v].w = a.v[v].w * s;
  }
  return r;
}

// DPP lane exchange inside a 16-lane row (v_add_f32_dpp, no LDS round trip)
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// Sum over the LPR lanes of a row-group.  xor1 / xor2 (quad_perm), then the
// half-row and row mirrors (lane i <-> 7-i, 15-i): after each step the lanes of
// the merged block hold identical bits, so pairing by mirror equals pairing by
// xor.  Beyond 16 lanes, __shfl_xor.  Every lane ends with the same bits.
template <int LPR>
__device__ __forceinline__ float group_sum(float s) {
  if (LPR >= 2) s += dpp<0xB1>(s);   // quad_perm [1,0,3,2]
  if (LPR >= 4) s += dpp<0x4E>(s);   // quad_perm [2,3,0,1]
  if (LPR >= 8) s += dpp<0x141>(s);  // row_half_mirror
  if (LPR >= 16) s += dpp<0x140>(s); // row_mirror
  if (LPR >= 32) s += __shfl_xor(s, 16, 64);
  if (LPR >= 64) s += __shfl_xor(s, 32, 64);
  return s;
}

// Row dot product (p*q)·h of APR.py:127: per-lane partial sums of rounded
// products, then the row-group sum.
template <int LPR, int NV>
__device__ __forceinline__ float dot_row(const RowV<NV>& a, const RowV<NV>& b) {
  float s = 0.f;
#pragma unroll
  for (int v = 0; v < NV; ++v) {  // (p*q) rounded, then summed (APR.py:127)
    s = s + a.v[v].x * b.v[v].x;
    s = s + a.v[v].y * b.v[v].y;
    s = s + a.v[v].z * b.v[v].z;
    s = s + a.v[v].w * b.v[v].w;
  }
  return group_sum<LPR>(s);
}

// softplus threshold of TF's SoftplusOp: log(FLT_EPSILON) + 2.
#define ACF_SOFTPLUS_T 13.942385f

// d/dx of softplus(-clip(x)) (APR.py:148-150): TF SoftplusGrad gives
// 1/(exp(r)+1) on features -r, negated by the Neg; clip_by_value passes the
// gradient only where lo <= x <= hi.  Also returns the loss term.
__device__ __forceinline__ void bpr_term(float x, float lo, float hi, float& g, float& loss) {
  float xc = fminf(fmaxf(x, lo), hi);
  bool pass = (x >= lo) && (x <= hi);
  float ex = expf(xc);
  g = pass ? -__builtin_amdgcn_rcpf(ex + 1.0f) : 0.0f;  // v_rcp_f32 (1 ulp)
  float f = -xc;
  loss = f > ACF_SOFTPLUS_T ? f : (f < -ACF_SOFTPLUS_T ? expf(f) : logf(expf(f) + 1.0f));
}

// counter-based RNG (splitmix64 finaliser over a mixed counter)
__device__ __host__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ float u01(uint64_t h) {  // (0,1]
  return ((float)(h >> 40) + 1.0f) * (1.0f / 16777216.0f);
}

// tf.truncated_normal(stddev) element: normal redrawn while |z| > 2 sigma.
__device__ __forceinline__ float trunc_normal(uint64_t key, float stddev) {
  for (uint32_t a = 0;; ++a) {
    uint64_t h1 = mix64(key ^ mix64(2ull * a + 1));
    uint64_t h2 = mix64(key ^ mix64(2ull * a + 2));
    float r = sqrtf(-2.0f * logf(u01(h1)));
    float z = r * cosf(6.283185307179586f * u01(h2));
    if (fabsf(z) <= 2.0f || a > 64) return z * stddev;
  }
}

#endif  // ACF_ROWS_H
