// acf_apr.hip — MI355X (gfx950) kernels + C-ABI for the APR (adversarial BPR-MF)
// training hot path of feay1234/Adversarial-Collaborative-Filtering.
//
// What the reference computes per mini-batch (APR.py:121-195 driven by
// utils.py:106-119) and how it maps here:
//
//   reference (TF1 graph, CPU)                      here (HIP, one batch)
//   ------------------------------------------      ----------------------------------
//   Unique/UnsortedSegmentSum dedup of the          plan: one radix sort per call over
//   IndexedSlices (Optimizer, APR.py:195) and       (batch, row, occurrence) keys for a
//   IndexedSlices->dense (APR.py:183-187)           whole epoch -> per-batch unique rows
//                                                   + ordered occurrence records
//   sess.run([update_P, update_Q]):                 k_clean: one row-group (d/4 lanes,
//     gather, (p*q)h, clip, softplus, grads,        float4 per lane) per UNIQUE row; it
//     dense l2_normalize * eps, full-table assign   sums its occurrences' clean-loss
//                                                   gradient in occurrence order and
//                                                   writes delta = eps*g/|g| for that row
//   sess.run(optimizer):                            k_adv: same row-centric pass over
//     clean + adversarial fwd/bwd, dedup,           p+dP, q+dQ; writes the row's total
//     SparseApplyAdagrad                            gradient.  k_apply: Adagrad on the
//                                                   unique rows, in place.
//
// Row-centric aggregation keeps every sum in a fixed order (bitwise
// reproducible, no float atomics).  Rows untouched by a batch have delta = 0 in
// the reference and are never read, so the dense full-table work of APR.py:183-191
// is skipped exactly.
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -shared -fPIC
// (fp-contract off: every multiply-add below is written out, so the same dot
// product evaluates to the same bits in every kernel that recomputes it).

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "acf_apr.h"

// ---------------------------------------------------------------------------
// error plumbing
// ---------------------------------------------------------------------------
static thread_local std::string g_last_error;

static int set_error(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

#define HIP_TRY(expr)                                                          \
  do {                                                                         \
    hipError_t e_ = (expr);                                                    \
    if (e_ != hipSuccess)                                                      \
      return set_error(ACF_E_HIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

#define ACF_CHECK(cond, code, ...)                                             \
  do {                                                                         \
    if (!(cond)) return set_error((code), __VA_ARGS__);                        \
  } while (0)

// ---------------------------------------------------------------------------
// device helpers
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

// Row dot product (p*q)·h of APR.py:127: per-lane partial sums, then a butterfly
// over the row-group.  Every lane of the group ends with the same bits.
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
#pragma unroll
  for (int m = LPR / 2; m > 0; m >>= 1) s += __shfl_xor(s, m, 64);
  return s;
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
  g = pass ? -1.0f / (ex + 1.0f) : 0.0f;
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

// ---------------------------------------------------------------------------
// plan kernels
// ---------------------------------------------------------------------------
struct PlanBits {
  uint32_t occ_bits;   // bits of the occurrence index
  uint64_t occ_mask;
};

// Stage triplets, validate ranges, build sort keys.
// user key  = ((t*U1 + u)      << ob_u) | x          (x = triplet index)
// item key  = ((t*I1 + item)   << ob_i) | (2x + role) (role 0 = pos, 1 = neg)
__global__ void k_stage(const int32_t* __restrict__ user, const int32_t* __restrict__ ipos,
                        const int32_t* __restrict__ ineg, int64_t E, int32_t B, int64_t U1,
                        int64_t I1, int32_t* __restrict__ tu, int32_t* __restrict__ ti,
                        int32_t* __restrict__ tj, uint64_t* __restrict__ ukey,
                        uint64_t* __restrict__ ikey, uint32_t ob_u, uint32_t ob_i,
                        int32_t* __restrict__ err) {
  int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (x >= E) return;
  int64_t t = x / B;
  int32_t u = user[x], i = ipos[x], j = ineg[x];
  if (u < 0 || u >= U1) { atomicOr(err, 1); u = 0; }
  if (i < 0 || i >= I1) { atomicOr(err, 2); i = 0; }
  if (j < 0 || j >= I1) { atomicOr(err, 2); j = 0; }
  tu[x] = u; ti[x] = i; tj[x] = j;
  ukey[x] = ((uint64_t)(t * U1 + u) << ob_u) | (uint64_t)x;
  ikey[2 * x] = ((uint64_t)(t * I1 + i) << ob_i) | (uint64_t)(2 * x);
  ikey[2 * x + 1] = ((uint64_t)(t * I1 + j) << ob_i) | (uint64_t)(2 * x + 1);
}

__global__ void k_heads(const uint64_t* __restrict__ key, int64_t n, uint32_t ob,
                        int32_t* __restrict__ flag) {
  int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (x >= n) return;
  flag[x] = (x == 0 || (key[x] >> ob) != (key[x - 1] >> ob)) ? 1 : 0;
}

// After an inclusive scan of the head flags: unique rows, occurrence offsets,
// per-batch unique ranges, the slot of every occurrence, occurrence values.
__global__ void k_compact(const uint64_t* __restrict__ key, const int32_t* __restrict__ inc,
                          int64_t n, uint32_t ob, uint64_t omask, int64_t R, int32_t nb,
                          int32_t* __restrict__ uniq, int32_t* __restrict__ off,
                          int32_t* __restrict__ bstart, int32_t* __restrict__ occ,
                          int32_t* __restrict__ slot_a, int32_t* __restrict__ slot_b,
                          int32_t item_side) {
  int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (x >= n) return;
  uint64_t k = key[x];
  uint64_t seg = k >> ob;
  int32_t v = (int32_t)(k & omask);
  int32_t s = inc[x] - 1;
  occ[x] = v;
  if (item_side) {
    if (v & 1) slot_b[v >> 1] = s; else slot_a[v >> 1] = s;
  } else {
    slot_a[v] = s;
  }
  bool head = (x == 0) || ((key[x - 1] >> ob) != seg);
  if (head) {
    uniq[s] = (int32_t)(seg % (uint64_t)R);
    off[s] = (int32_t)x;
    int64_t t = (int64_t)(seg / (uint64_t)R);
    bool bhead = (x == 0) || (((key[x - 1] >> ob) / (uint64_t)R) != (uint64_t)t);
    if (bhead) bstart[t] = s;
  }
  if (x == n - 1) {
    off[s + 1] = (int32_t)n;
    bstart[nb] = s + 1;
  }
}

// Per-occurrence records so that step kernels reach partner rows in one hop.
// user occurrence x (triplet e):  {i, j, slot(i), slot(j)}
// item occurrence x (e, role):    {u, other item, slot(u), slot(other)}
__global__ void k_records(const int32_t* __restrict__ uocc, const int32_t* __restrict__ iocc,
                          int64_t E, const int32_t* __restrict__ tu,
                          const int32_t* __restrict__ ti, const int32_t* __restrict__ tj,
                          const int32_t* __restrict__ uslot, const int32_t* __restrict__ pslot,
                          const int32_t* __restrict__ nslot, int4* __restrict__ urec,
                          int4* __restrict__ irec) {
  int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (x < E) {
    int32_t e = uocc[x];
    urec[x] = make_int4(ti[e], tj[e], pslot[e], nslot[e]);
  }
  if (x < 2 * E) {
    int32_t v = iocc[x];
    int32_t e = v >> 1;
    if (v & 1)
      irec[x] = make_int4(tu[e], ti[e], uslot[e], pslot[e]);
    else
      irec[x] = make_int4(tu[e], tj[e], uslot[e], nslot[e]);
  }
}

// ---------------------------------------------------------------------------
// step kernels
// ---------------------------------------------------------------------------
struct StepArgs {
  float* P;
  float* Q;
  float* accP;
  float* accQ;
  const int32_t* uuniq;
  const int32_t* uoff;
  const int32_t* ubs;
  const int32_t* uocc;
  const int4* urec;
  const int32_t* iuniq;
  const int32_t* ioff;
  const int32_t* ibs;
  const int32_t* iocc;
  const int4* irec;
  float* g0;      // [3B, d] clean-loss gradient per local slot
  float* delta;   // [3B, d] delta per local slot
  float* gsum;    // [3B, d] total gradient per local slot
  float* loss_clean;  // [E]
  float* loss_adv;    // [E]
  int32_t d;
  int32_t B;
  int32_t t;
  float lr, eps, reg, reg_adv, clip_lo, clip_hi;
  int32_t adver, adv_mode, zero_delta;
  uint64_t seed;
};

// Phase 1 (= sess.run([update_P, update_Q]) and the clean half of the
// optimizer): for every unique row of batch t, the clean-loss gradient summed
// over its occurrences, and (adver) its delta.
template <int LPR, int NV>
__global__ void __launch_bounds__(256) k_clean(StepArgs a) {
  const int64_t gtid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int grp = (int)(gtid / LPR);
  const int l = threadIdx.x & (LPR - 1);
  const int ub0 = a.ubs[a.t], nU = a.ubs[a.t + 1] - ub0;
  const int ib0 = a.ibs[a.t], nI = a.ibs[a.t + 1] - ib0;
  if (grp >= nU + nI) return;
  const int d = a.d;
  RowV<NV> G = zero_row<NV>();
  int64_t row;
  bool is_user = grp < nU;
  if (is_user) {
    const int s = ub0 + grp;
    row = a.uuniq[s];
    const RowV<NV> p = load_row<LPR, NV>(a.P, row, d, l);
    const int o1 = a.uoff[s + 1];
    for (int o = a.uoff[s]; o < o1; ++o) {
      const int4 r = a.urec[o];
      const RowV<NV> qi = load_row<LPR, NV>(a.Q, r.x, d, l);
      const RowV<NV> qj = load_row<LPR, NV>(a.Q, r.y, d, l);
      const float x = dot_row<LPR, NV>(p, qi) - dot_row<LPR, NV>(p, qj);
      float g, loss;
      bpr_term(x, a.clip_lo, a.clip_hi, g, loss);
      axpy_row(G, g, qi);   // pos branch: dx+/dp = qi
      axpy_row(G, -g, qj);  // neg branch: dx-/dp = qj
      if (l == 0) a.loss_clean[a.uocc[o]] = loss;
    }
  } else {
    const int s = ib0 + (grp - nU);
    row = a.iuniq[s];
    const RowV<NV> q = load_row<LPR, NV>(a.Q, row, d, l);
    const int o1 = a.ioff[s + 1];
    for (int o = a.ioff[s]; o < o1; ++o) {
      const int4 r = a.irec[o];
      const int role = a.iocc[o] & 1;
      const RowV<NV> p = load_row<LPR, NV>(a.P, r.x, d, l);
      const RowV<NV> qo = load_row<LPR, NV>(a.Q, r.y, d, l);
      const float dq = dot_row<LPR, NV>(p, q), dqo = dot_row<LPR, NV>(p, qo);
      const float x = role ? (dqo - dq) : (dq - dqo);
      float g, loss;
      bpr_term(x, a.clip_lo, a.clip_hi, g, loss);
      axpy_row(G, role ? -g : g, p);
    }
  }
  const int64_t slot = grp;
  store_row<LPR, NV>(a.g0, slot, d, l, G);
  if (!a.adver) return;
  RowV<NV> dl;
  if (a.zero_delta) {
    dl = zero_row<NV>();
  } else if (a.adv_mode == 0) {
    // tf.nn.l2_normalize(g, 1) * eps  (epsilon 1e-12 on the squared norm)
    const float ss = dot_row<LPR, NV>(G, G);
    const float inv = 1.0f / sqrtf(fmaxf(ss, 1e-12f));
    dl = scale_row(scale_row(G, inv), a.eps);
  } else {
    // "random": l2_normalize(truncated_normal(0, 0.01)) * eps, redrawn every run
    RowV<NV> z;
    const uint64_t rk = mix64(a.seed ^ mix64(((uint64_t)a.t << 1) | (is_user ? 0 : 1))) ^
                        mix64((uint64_t)row * 0x100000001B3ull);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int c = l + LPR * v;
      float e4[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        e4[k] = (c * 4 + k < d) ? trunc_normal(rk ^ mix64((uint64_t)(c * 4 + k)), 0.01f) : 0.f;
      z.v[v] = make_float4(e4[0], e4[1], e4[2], e4[3]);
    }
    const float ss = dot_row<LPR, NV>(z, z);
    const float inv = 1.0f / sqrtf(fmaxf(ss, 1e-12f));
    dl = scale_row(scale_row(z, inv), a.eps);
  }
  store_row<LPR, NV>(a.delta, slot, d, l, dl);
}

// Phase 2 (adversarial half of sess.run(optimizer), APR.py:130-141,156-165):
// loss on p+dP[u], q+dQ[i] with the deltas of phase 1; the row's total
// gradient G = G_clean + reg_adv * G_adv.
template <int LPR, int NV>
__global__ void __launch_bounds__(256) k_adv(StepArgs a) {
  const int64_t gtid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int grp = (int)(gtid / LPR);
  const int l = threadIdx.x & (LPR - 1);
  const int ub0 = a.ubs[a.t], nU = a.ubs[a.t + 1] - ub0;
  const int ib0 = a.ibs[a.t], nI = a.ibs[a.t + 1] - ib0;
  if (grp >= nU + nI) return;
  const int d = a.d;
  RowV<NV> G = zero_row<NV>();
  if (grp < nU) {
    const int s = ub0 + grp;
    const int64_t row = a.uuniq[s];
    const RowV<NV> pp = add_row(load_row<LPR, NV>(a.P, row, d, l),
                                load_row<LPR, NV>(a.delta, grp, d, l));
    const int o1 = a.uoff[s + 1];
    for (int o = a.uoff[s]; o < o1; ++o) {
      const int4 r = a.urec[o];
      const RowV<NV> qi = add_row(load_row<LPR, NV>(a.Q, r.x, d, l),
                                  load_row<LPR, NV>(a.delta, nU + (r.z - ib0), d, l));
      const RowV<NV> qj = add_row(load_row<LPR, NV>(a.Q, r.y, d, l),
                                  load_row<LPR, NV>(a.delta, nU + (r.w - ib0), d, l));
      const float x = dot_row<LPR, NV>(pp, qi) - dot_row<LPR, NV>(pp, qj);
      float g, loss;
      bpr_term(x, a.clip_lo, a.clip_hi, g, loss);
      axpy_row(G, g, qi);
      axpy_row(G, -g, qj);
      if (l == 0) a.loss_adv[a.uocc[o]] = loss;
    }
  } else {
    const int k = grp - nU;
    const int s = ib0 + k;
    const int64_t row = a.iuniq[s];
    const RowV<NV> qq = add_row(load_row<LPR, NV>(a.Q, row, d, l),
                                load_row<LPR, NV>(a.delta, grp, d, l));
    const int o1 = a.ioff[s + 1];
    for (int o = a.ioff[s]; o < o1; ++o) {
      const int4 r = a.irec[o];
      const int role = a.iocc[o] & 1;
      const RowV<NV> pp = add_row(load_row<LPR, NV>(a.P, r.x, d, l),
                                  load_row<LPR, NV>(a.delta, r.z - ub0, d, l));
      const RowV<NV> qo = add_row(load_row<LPR, NV>(a.Q, r.y, d, l),
                                  load_row<LPR, NV>(a.delta, nU + (r.w - ib0), d, l));
      const float dq = dot_row<LPR, NV>(pp, qq), dqo = dot_row<LPR, NV>(pp, qo);
      const float x = role ? (dqo - dq) : (dq - dqo);
      float g, loss;
      bpr_term(x, a.clip_lo, a.clip_hi, g, loss);
      axpy_row(G, role ? -g : g, pp);
    }
  }
  RowV<NV> G0 = load_row<LPR, NV>(a.g0, grp, d, l);
  axpy_row(G0, a.reg_adv, G);
  store_row<LPR, NV>(a.gsum, grp, d, l, G0);
}

// Sparse Adagrad on the unique rows (TF SparseApplyAdagrad after the dedup):
//   acc += g*g;  w -= lr * g * rsqrt(acc)
// plus the reg * mean(w^2) terms of APR.py:153-154,164-165 (2*reg*w/(B*d) per
// occurrence, counted twice in the APR graph).
__global__ void __launch_bounds__(256) k_apply(StepArgs a) {
  const int64_t gtid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int d4 = a.d >> 2;
  const int slot = (int)(gtid / d4);
  const int c = (int)(gtid - (int64_t)slot * d4);
  const int ub0 = a.ubs[a.t], nU = a.ubs[a.t + 1] - ub0;
  const int ib0 = a.ibs[a.t], nI = a.ibs[a.t + 1] - ib0;
  if (slot >= nU + nI) return;
  float* W;
  float* A;
  int64_t row;
  int m;
  if (slot < nU) {
    const int s = ub0 + slot;
    row = a.uuniq[s];
    m = a.uoff[s + 1] - a.uoff[s];
    W = a.P;
    A = a.accP;
  } else {
    const int s = ib0 + (slot - nU);
    row = a.iuniq[s];
    m = a.ioff[s + 1] - a.ioff[s];
    W = a.Q;
    A = a.accQ;
  }
  const float* Gsrc = a.adver ? a.gsum : a.g0;
  float4 g = *reinterpret_cast<const float4*>(Gsrc + (int64_t)slot * a.d + c * 4);
  float4* wp = reinterpret_cast<float4*>(W + row * a.d + c * 4);
  float4* ap = reinterpret_cast<float4*>(A + row * a.d + c * 4);
  float4 w = *wp, acc = *ap;
  if (a.reg != 0.f) {
    const float coef = (2.0f * a.reg / ((float)a.B * (float)a.d)) * (float)(a.adver ? 2 * m : m);
    g.x = g.x + coef * w.x;
    g.y = g.y + coef * w.y;
    g.z = g.z + coef * w.z;
    g.w = g.w + coef * w.w;
  }
  acc.x = acc.x + g.x * g.x;
  acc.y = acc.y + g.y * g.y;
  acc.z = acc.z + g.z * g.z;
  acc.w = acc.w + g.w * g.w;
  w.x -= (a.lr * g.x) * (1.0f / sqrtf(acc.x));
  w.y -= (a.lr * g.y) * (1.0f / sqrtf(acc.y));
  w.z -= (a.lr * g.z) * (1.0f / sqrtf(acc.z));
  w.w -= (a.lr * g.w) * (1.0f / sqrtf(acc.w));
  *ap = acc;
  *wp = w;
}

__global__ void k_delta_scatter(StepArgs a, float* __restrict__ dP, float* __restrict__ dQ) {
  const int64_t gtid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int d4 = a.d >> 2;
  const int slot = (int)(gtid / d4);
  const int c = (int)(gtid - (int64_t)slot * d4);
  const int ub0 = a.ubs[a.t], nU = a.ubs[a.t + 1] - ub0;
  const int ib0 = a.ibs[a.t], nI = a.ibs[a.t + 1] - ib0;
  if (slot >= nU + nI) return;
  const float4 v = *reinterpret_cast<const float4*>(a.delta + (int64_t)slot * a.d + c * 4);
  if (slot < nU)
    *reinterpret_cast<float4*>(dP + (int64_t)a.uuniq[ub0 + slot] * a.d + c * 4) = v;
  else
    *reinterpret_cast<float4*>(dQ + (int64_t)a.iuniq[ib0 + slot - nU] * a.d + c * 4) = v;
}

// ---------------------------------------------------------------------------
// forward only (training_loss_acc, utils.py:159-175): one workgroup per batch,
// deterministic per-batch sums.
// ---------------------------------------------------------------------------
template <int LPR, int NV>
__global__ void __launch_bounds__(256) k_forward(const float* __restrict__ P,
                                                 const float* __restrict__ Q, int d,
                                                 const int32_t* __restrict__ user,
                                                 const int32_t* __restrict__ ipos,
                                                 const int32_t* __restrict__ ineg, int B,
                                                 float lo, float hi, float* batch_loss,
                                                 int32_t* batch_correct, float* out_pos,
                                                 float* out_neg) {
  constexpr int GPB = 256 / LPR;
  __shared__ float s_loss[GPB];
  __shared__ int s_cnt[GPB];
  const int t = blockIdx.x;
  const int grp = threadIdx.x / LPR;
  const int l = threadIdx.x & (LPR - 1);
  float lsum = 0.f;
  int cnt = 0;
  for (int b = grp; b < B; b += GPB) {
    const int64_t e = (int64_t)t * B + b;
    const RowV<NV> p = load_row<LPR, NV>(P, user[e], d, l);
    const RowV<NV> qi = load_row<LPR, NV>(Q, ipos[e], d, l);
    const RowV<NV> qj = load_row<LPR, NV>(Q, ineg[e], d, l);
    const float xp = dot_row<LPR, NV>(p, qi), xn = dot_row<LPR, NV>(p, qj);
    float g, loss;
    bpr_term(xp - xn, lo, hi, g, loss);
    lsum += loss;
    cnt += (xp - xn) > 0.f ? 1 : 0;
    if (l == 0) {
      if (out_pos) out_pos[e] = xp;
      if (out_neg) out_neg[e] = xn;
    }
  }
  if (l == 0) {
    s_loss[grp] = lsum;
    s_cnt[grp] = cnt;
  }
  __syncthreads();
  for (int w = GPB / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) {
      s_loss[threadIdx.x] += s_loss[threadIdx.x + w];
      s_cnt[threadIdx.x] += s_cnt[threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (batch_loss) batch_loss[t] = s_loss[0];
    if (batch_correct) batch_correct[t] = s_cnt[0];
  }
}

// ---------------------------------------------------------------------------
// evaluation (_eval_by_user, utils.py:244-254)
// score(u,c) = sequential sum over k of round(P[u][k]*Q[c][k]); the same chain
// is used for the test item, the dense sweep and the exclusion correction so
// that equal pairs give equal bits and ">=" ties are decided exactly.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float seq_dot(const float* __restrict__ p, const float* __restrict__ q,
                                         int d) {
  float s = 0.f;
  for (int k = 0; k < d; k += 4) {
    const float4 qv = *reinterpret_cast<const float4*>(q + k);
    const float4 pv = *reinterpret_cast<const float4*>(p + k);
    s = s + pv.x * qv.x;
    s = s + pv.y * qv.y;
    s = s + pv.z * qv.z;
    s = s + pv.w * qv.w;
  }
  return s;
}

constexpr int EVAL_UB = 8;  // users per workgroup

__global__ void __launch_bounds__(256) k_eval_all(const float* __restrict__ P,
                                                  const float* __restrict__ Q, int d,
                                                  const int32_t* __restrict__ users,
                                                  const int32_t* __restrict__ tests, int n_users,
                                                  int num_cand, const int64_t* __restrict__ excl_off,
                                                  const int32_t* __restrict__ excl,
                                                  int32_t* __restrict__ positions) {
  extern __shared__ float smem[];  // [EVAL_UB][d]
  __shared__ float s_test[EVAL_UB];
  __shared__ int s_cnt[EVAL_UB];
  const int u0 = blockIdx.x * EVAL_UB;
  const int nu = min(EVAL_UB, n_users - u0);
  for (int idx = threadIdx.x; idx < EVAL_UB * d; idx += blockDim.x) {
    const int uu = idx / d, k = idx - uu * d;
    smem[idx] = uu < nu ? P[(int64_t)users[u0 + uu] * d + k] : 0.f;
  }
  __syncthreads();
  if (threadIdx.x < EVAL_UB) {
    s_cnt[threadIdx.x] = 0;
    s_test[threadIdx.x] =
        threadIdx.x < nu ? seq_dot(smem + threadIdx.x * d, Q + (int64_t)tests[u0 + threadIdx.x] * d, d)
                         : 0.f;
  }
  __syncthreads();
  int cnt[EVAL_UB];
#pragma unroll
  for (int uu = 0; uu < EVAL_UB; ++uu) cnt[uu] = 0;
  for (int c = threadIdx.x; c < num_cand; c += blockDim.x) {
    const float* q = Q + (int64_t)c * d;
    float acc[EVAL_UB];
#pragma unroll
    for (int uu = 0; uu < EVAL_UB; ++uu) acc[uu] = 0.f;
    for (int k = 0; k < d; k += 4) {
      const float4 qv = *reinterpret_cast<const float4*>(q + k);
#pragma unroll
      for (int uu = 0; uu < EVAL_UB; ++uu) {
        const float4 pv = *reinterpret_cast<const float4*>(smem + uu * d + k);
        float s = acc[uu];
        s = s + pv.x * qv.x;
        s = s + pv.y * qv.y;
        s = s + pv.z * qv.z;
        s = s + pv.w * qv.w;
        acc[uu] = s;
      }
    }
#pragma unroll
    for (int uu = 0; uu < EVAL_UB; ++uu) cnt[uu] += acc[uu] >= s_test[uu] ? 1 : 0;
  }
  // exclusion correction: candidates in trainList[u] (and the test item)
  for (int uu = 0; uu < nu; ++uu) {
    const int64_t a0 = excl_off[u0 + uu], a1 = excl_off[u0 + uu + 1];
    for (int64_t x = a0 + threadIdx.x; x < a1; x += blockDim.x) {
      const float s = seq_dot(smem + uu * d, Q + (int64_t)excl[x] * d, d);
      cnt[uu] -= s >= s_test[uu] ? 1 : 0;
    }
  }
#pragma unroll
  for (int uu = 0; uu < EVAL_UB; ++uu) atomicAdd(&s_cnt[uu], cnt[uu]);
  __syncthreads();
  if (threadIdx.x < nu) positions[u0 + threadIdx.x] = s_cnt[threadIdx.x];
}

__global__ void __launch_bounds__(256) k_eval_list(const float* __restrict__ P,
                                                   const float* __restrict__ Q, int d,
                                                   const int32_t* __restrict__ users,
                                                   const int32_t* __restrict__ tests,
                                                   const int64_t* __restrict__ cand_off,
                                                   const int32_t* __restrict__ cand,
                                                   int32_t* __restrict__ positions) {
  extern __shared__ float smem[];  // [d]
  __shared__ float s_test;
  __shared__ int s_cnt;
  const int uu = blockIdx.x;
  for (int k = threadIdx.x; k < d; k += blockDim.x) smem[k] = P[(int64_t)users[uu] * d + k];
  __syncthreads();
  if (threadIdx.x == 0) {
    s_cnt = 0;
    s_test = seq_dot(smem, Q + (int64_t)tests[uu] * d, d);
  }
  __syncthreads();
  int cnt = 0;
  for (int64_t x = cand_off[uu] + threadIdx.x; x < cand_off[uu + 1]; x += blockDim.x)
    cnt += seq_dot(smem, Q + (int64_t)cand[x] * d, d) >= s_test ? 1 : 0;
  atomicAdd(&s_cnt, cnt);
  __syncthreads();
  if (threadIdx.x == 0) positions[uu] = s_cnt;
}

// ---------------------------------------------------------------------------
// sampler (shuffle / _get_train_batch, APR.py:39-81)
// ---------------------------------------------------------------------------
__global__ void k_perm_keys(int64_t n, uint64_t seed, uint64_t* __restrict__ keys,
                            int32_t* __restrict__ vals) {
  int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (x >= n) return;
  keys[x] = mix64(seed ^ mix64((uint64_t)x + 0x5bd1e995ull));
  vals[x] = (int32_t)x;
}

__device__ __forceinline__ bool sorted_contains(const int32_t* __restrict__ a, int64_t n,
                                                int32_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    int32_t m = a[mid];
    if (m < v) lo = mid + 1; else hi = mid;
  }
  return lo < n && a[lo] == v;
}

__global__ void k_negatives(const int32_t* __restrict__ perm, const int32_t* __restrict__ pu,
                            const int32_t* __restrict__ pi, int64_t n_out, int32_t num_items,
                            int32_t num_lists, const int64_t* __restrict__ loff,
                            const int32_t* __restrict__ litems, uint64_t seed, int32_t max_tries,
                            int32_t* __restrict__ ou, int32_t* __restrict__ op,
                            int32_t* __restrict__ on, int32_t* __restrict__ err) {
  int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (x >= n_out) return;
  const int32_t src = perm[x];
  const int32_t u = pu[src];
  ou[x] = u;
  op[x] = pi[src];
  if (u < 0 || u >= num_lists) {
    atomicOr(err, 1);
    on[x] = -1;
    return;
  }
  const int32_t* lst = litems + loff[u];
  const int64_t ln = loff[u + 1] - loff[u];
  const uint64_t base = mix64(seed ^ 0xA0761D6478BD642Full) ^ mix64((uint64_t)x);
  for (int32_t a = 0; a < max_tries; ++a) {
    const uint64_t h = mix64(base + (uint64_t)a * 0x9E3779B97F4A7C15ull);
    const int32_t j = (int32_t)(((h >> 32) * (uint64_t)num_items) >> 32);
    if (!sorted_contains(lst, ln, j)) {
      on[x] = j;
      return;
    }
  }
  atomicOr(err, 2);
  on[x] = -1;
}

// dns > 1 (utils.py:121-133): argmax of the clean score over dns candidates.
template <int LPR, int NV>
__global__ void __launch_bounds__(256) k_dns_select(const float* __restrict__ P,
                                                    const float* __restrict__ Q, int d,
                                                    const int32_t* __restrict__ user,
                                                    const int32_t* __restrict__ cand, int64_t n,
                                                    int dns, int32_t* __restrict__ out) {
  const int64_t gtid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t e = gtid / LPR;
  const int l = threadIdx.x & (LPR - 1);
  if (e >= n) return;
  const RowV<NV> p = load_row<LPR, NV>(P, user[e], d, l);
  float best = 0.f;
  int32_t bi = 0;
  for (int k = 0; k < dns; ++k) {
    const int32_t c = cand[e * dns + k];
    const float s = dot_row<LPR, NV>(p, load_row<LPR, NV>(Q, c, d, l));
    if (k == 0 || s > best) {
      best = s;
      bi = c;
    }
  }
  if (l == 0) out[e] = bi;
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
struct GraphKey {
  const void* ptrs[4];
  acf_apr_hparams hp;
  int32_t first, n, B, d;
  bool operator<(const GraphKey& o) const { return memcmp(this, &o, sizeof(GraphKey)) < 0; }
};

struct acf_apr_ctx {
  int64_t U1 = 0, I1 = 0;
  int32_t d = 0, maxB = 0, maxNB = 0;
  int64_t maxE = 0;
  // staged triplets
  int32_t *tu = nullptr, *ti = nullptr, *tj = nullptr;
  // plan
  uint64_t *ukey_in = nullptr, *ukey_out = nullptr, *ikey_in = nullptr, *ikey_out = nullptr;
  int32_t *flag = nullptr, *inc = nullptr;
  int32_t *uuniq = nullptr, *uoff = nullptr, *ubs = nullptr, *uocc = nullptr, *uslot = nullptr;
  int32_t *iuniq = nullptr, *ioff = nullptr, *ibs = nullptr, *iocc = nullptr;
  int32_t *pslot = nullptr, *nslot = nullptr;
  int4 *urec = nullptr, *irec = nullptr;
  int32_t* err = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  // per-batch scratch
  float *g0 = nullptr, *delta = nullptr, *gsum = nullptr;
  float *loss_clean = nullptr, *loss_adv = nullptr;
  // state
  int32_t B = 0, nb = 0;
  int32_t last_delta_batch = -1;
  hipStream_t cap_stream = nullptr;
  std::map<GraphKey, hipGraphExec_t> graphs;
  std::vector<void*> allocs;
};

static uint32_t bits_for(uint64_t v) {  // bits to represent values in [0, v)
  uint32_t b = 0;
  while (b < 64 && (v > (1ull << b))) ++b;
  return b == 0 ? 1 : b;
}

template <typename T>
static int dalloc(acf_apr_ctx* c, T** p, size_t n) {
  void* q = nullptr;
  if (hipMalloc(&q, n * sizeof(T) + 16) != hipSuccess) {
    (void)hipGetLastError();
    return set_error(ACF_E_NOMEM, "hipMalloc of %zu bytes failed", n * sizeof(T));
  }
  c->allocs.push_back(q);
  *p = static_cast<T*>(q);
  return ACF_OK;
}

#define ACF_RET(x)                  \
  do {                              \
    int r_ = (x);                   \
    if (r_ != ACF_OK) return r_;    \
  } while (0)

static inline unsigned grid_for(int64_t n, int bs = 256) {
  return (unsigned)((n + bs - 1) / bs);
}

// Row-group geometry for a given dim: LPR lanes per row, NV float4 per lane.
static void geometry(int d, int* lpr, int* nv) {
  int d4 = d / 4;
  int l = 1;
  while (l < d4 && l < 64) l <<= 1;
  *lpr = l;
  *nv = (d4 + l - 1) / l;
}

#define DISPATCH_GEOM(d, KFN, ...)                                                    \
  [&]() -> int {                                                                    \
    int lpr_, nv_;                                                                  \
    geometry((d), &lpr_, &nv_);                                                     \
    switch (lpr_ * 100 + nv_) {                                                     \
      case 101: KFN<1, 1>(__VA_ARGS__); break;                                      \
      case 201: KFN<2, 1>(__VA_ARGS__); break;                                      \
      case 401: KFN<4, 1>(__VA_ARGS__); break;                                      \
      case 801: KFN<8, 1>(__VA_ARGS__); break;                                      \
      case 1601: KFN<16, 1>(__VA_ARGS__); break;                                    \
      case 3201: KFN<32, 1>(__VA_ARGS__); break;                                    \
      case 6401: KFN<64, 1>(__VA_ARGS__); break;                                    \
      case 6402: KFN<64, 2>(__VA_ARGS__); break;                                    \
      case 6403: KFN<64, 3>(__VA_ARGS__); break;                                    \
      case 6404: KFN<64, 4>(__VA_ARGS__); break;                                    \
      default: return set_error(ACF_E_INVALID, "unsupported dim %d", (int)(d));     \
    }                                                                               \
    return ACF_OK;                                                                  \
  }()

static int check_dim(int d) {
  ACF_CHECK(d >= 4 && d <= 1024 && d % 4 == 0, ACF_E_INVALID,
            "dim must be a multiple of 4 in [4, 1024], got %d", d);
  return ACF_OK;
}

extern "C" int acf_apr_abi_version(void) { return ACF_APR_ABI_VERSION; }

extern "C" const char* acf_apr_last_error(void) { return g_last_error.c_str(); }

extern "C" int acf_apr_destroy(acf_apr_ctx* c) {
  if (!c) return ACF_OK;
  for (auto& kv : c->graphs) (void)hipGraphExecDestroy(kv.second);
  c->graphs.clear();
  for (void* p : c->allocs) (void)hipFree(p);
  if (c->cap_stream) (void)hipStreamDestroy(c->cap_stream);
  delete c;
  return ACF_OK;
}

extern "C" int acf_apr_create(acf_apr_ctx** out, int64_t U1, int64_t I1, int32_t d,
                              int32_t maxB, int32_t maxNB) {
  ACF_CHECK(out != nullptr, ACF_E_INVALID, "out is NULL");
  *out = nullptr;
  ACF_RET(check_dim(d));
  ACF_CHECK(U1 > 0 && I1 > 0 && U1 < (1ll << 31) && I1 < (1ll << 31), ACF_E_INVALID,
            "table rows must be in [1, 2^31): got %lld, %lld", (long long)U1, (long long)I1);
  ACF_CHECK(maxB > 0 && maxNB > 0, ACF_E_INVALID, "max_batch_size and max_batches must be > 0");
  int64_t maxE = (int64_t)maxB * maxNB;
  ACF_CHECK(2 * maxE < (1ll << 31), ACF_E_INVALID, "plan too large: %lld triplets", (long long)maxE);
  uint32_t ob_i = bits_for((uint64_t)(2 * maxE));
  uint32_t sb_i = bits_for((uint64_t)maxNB * (uint64_t)I1);
  uint32_t sb_u = bits_for((uint64_t)maxNB * (uint64_t)U1);
  ACF_CHECK(ob_i + sb_i <= 64 && ob_i + sb_u <= 64, ACF_E_INVALID,
            "plan key does not fit 64 bits (rows x batches x batch too large)");
  acf_apr_ctx* c = new acf_apr_ctx();
  c->U1 = U1; c->I1 = I1; c->d = d; c->maxB = maxB; c->maxNB = maxNB; c->maxE = maxE;
  int r = ACF_OK;
  auto A = [&](auto** p, size_t n) { if (r == ACF_OK) r = dalloc(c, p, n); };
  A(&c->tu, maxE); A(&c->ti, maxE); A(&c->tj, maxE);
  A(&c->ukey_in, maxE); A(&c->ukey_out, maxE);
  A(&c->ikey_in, 2 * maxE); A(&c->ikey_out, 2 * maxE);
  A(&c->flag, 2 * maxE); A(&c->inc, 2 * maxE);
  A(&c->uuniq, maxE); A(&c->uoff, maxE + 1); A(&c->ubs, maxNB + 1); A(&c->uocc, maxE);
  A(&c->uslot, maxE);
  A(&c->iuniq, 2 * maxE); A(&c->ioff, 2 * maxE + 1); A(&c->ibs, maxNB + 1); A(&c->iocc, 2 * maxE);
  A(&c->pslot, maxE); A(&c->nslot, maxE);
  A(&c->urec, maxE); A(&c->irec, 2 * maxE);
  A(&c->err, 4);
  A(&c->g0, (size_t)3 * maxB * d); A(&c->delta, (size_t)3 * maxB * d);
  A(&c->gsum, (size_t)3 * maxB * d);
  A(&c->loss_clean, maxE); A(&c->loss_adv, maxE);
  if (r != ACF_OK) { acf_apr_destroy(c); return r; }
  size_t b1 = 0, b2 = 0, b3 = 0;
  if (rocprim::radix_sort_keys(nullptr, b1, c->ikey_in, c->ikey_out, (size_t)(2 * maxE), 0, 64) !=
          hipSuccess ||
      rocprim::inclusive_scan(nullptr, b2, c->flag, c->inc, (size_t)(2 * maxE),
                              rocprim::plus<int32_t>()) != hipSuccess ||
      rocprim::radix_sort_keys(nullptr, b3, c->ukey_in, c->ukey_out, (size_t)maxE, 0, 64) !=
          hipSuccess) {
    acf_apr_destroy(c);
    return set_error(ACF_E_HIP, "rocprim temporary-storage query failed");
  }
  c->tmp_bytes = std::max(b1, std::max(b2, b3));
  r = dalloc(c, reinterpret_cast<char**>(&c->tmp), c->tmp_bytes);
  if (r != ACF_OK) { acf_apr_destroy(c); return r; }
  if (hipStreamCreateWithFlags(&c->cap_stream, hipStreamNonBlocking) != hipSuccess) {
    acf_apr_destroy(c);
    return set_error(ACF_E_HIP, "hipStreamCreate failed");
  }
  if (hipMemset(c->err, 0, 16) != hipSuccess) {
    acf_apr_destroy(c);
    return set_error(ACF_E_HIP, "hipMemset failed");
  }
  *out = c;
  return ACF_OK;
}

extern "C" int acf_apr_plan(acf_apr_ctx* c, const int32_t* user, const int32_t* ipos,
                            const int32_t* ineg, int32_t B, int32_t nb, int32_t check,
                            void* stream_) {
  ACF_CHECK(c, ACF_E_INVALID, "ctx is NULL");
  ACF_CHECK(user && ipos && ineg, ACF_E_INVALID, "triplet pointers must be non-NULL");
  ACF_CHECK(B > 0 && B <= c->maxB, ACF_E_INVALID, "batch_size %d outside (0, %d]", B, c->maxB);
  ACF_CHECK(nb > 0 && nb <= c->maxNB, ACF_E_INVALID, "n_batches %d outside (0, %d]", nb, c->maxNB);
  hipStream_t s = static_cast<hipStream_t>(stream_);
  const int64_t E = (int64_t)B * nb;
  const uint32_t ob_u = bits_for((uint64_t)E), ob_i = bits_for((uint64_t)(2 * E));
  const uint32_t eb_u = ob_u + bits_for((uint64_t)nb * (uint64_t)c->U1);
  const uint32_t eb_i = ob_i + bits_for((uint64_t)nb * (uint64_t)c->I1);
  ACF_CHECK(eb_u <= 64 && eb_i <= 64, ACF_E_INVALID, "plan key does not fit 64 bits");
  c->B = 0;
  c->nb = 0;
  c->last_delta_batch = -1;
  HIP_TRY(hipMemsetAsync(c->err, 0, sizeof(int32_t), s));
  k_stage<<<grid_for(E), 256, 0, s>>>(user, ipos, ineg, E, B, c->U1, c->I1, c->tu, c->ti, c->tj,
                                      c->ukey_in, c->ikey_in, ob_u, ob_i, c->err);
  HIP_TRY(hipGetLastError());
  size_t tb = c->tmp_bytes;
  HIP_TRY(rocprim::radix_sort_keys(c->tmp, tb, c->ukey_in, c->ukey_out, (size_t)E, 0, eb_u, s));
  tb = c->tmp_bytes;
  HIP_TRY(rocprim::radix_sort_keys(c->tmp, tb, c->ikey_in, c->ikey_out, (size_t)(2 * E), 0, eb_i, s));
  // users
  k_heads<<<grid_for(E), 256, 0, s>>>(c->ukey_out, E, ob_u, c->flag);
  tb = c->tmp_bytes;
  HIP_TRY(rocprim::inclusive_scan(c->tmp, tb, c->flag, c->inc, (size_t)E, rocprim::plus<int32_t>(), s));
  k_compact<<<grid_for(E), 256, 0, s>>>(c->ukey_out, c->inc, E, ob_u, (1ull << ob_u) - 1, c->U1, nb,
                                        c->uuniq, c->uoff, c->ubs, c->uocc, c->uslot, nullptr, 0);
  // items
  k_heads<<<grid_for(2 * E), 256, 0, s>>>(c->ikey_out, 2 * E, ob_i, c->flag);
  tb = c->tmp_bytes;
  HIP_TRY(rocprim::inclusive_scan(c->tmp, tb, c->flag, c->inc, (size_t)(2 * E), rocprim::plus<int32_t>(), s));
  k_compact<<<grid_for(2 * E), 256, 0, s>>>(c->ikey_out, c->inc, 2 * E, ob_i, (1ull << ob_i) - 1, c->I1,
                                            nb, c->iuniq, c->ioff, c->ibs, c->iocc, c->pslot, c->nslot, 1);
  k_records<<<grid_for(2 * E), 256, 0, s>>>(c->uocc, c->iocc, E, c->tu, c->ti, c->tj, c->uslot,
                                            c->pslot, c->nslot, c->urec, c->irec);
  HIP_TRY(hipGetLastError());
  if (check) {
    int32_t herr = 0;
    HIP_TRY(hipMemcpyAsync(&herr, c->err, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    ACF_CHECK(herr == 0, ACF_E_RANGE, "triplet index out of range (%s%s)",
              (herr & 1) ? "user >= num_user_rows " : "",
              (herr & 2) ? "item >= num_item_rows" : "");
  }
  c->B = B;
  c->nb = nb;
  return ACF_OK;
}

static StepArgs make_args(acf_apr_ctx* c, const acf_apr_tables* tb, const acf_apr_hparams* hp,
                          int32_t t) {
  StepArgs a;
  a.P = tb->P; a.Q = tb->Q; a.accP = tb->accP; a.accQ = tb->accQ;
  a.uuniq = c->uuniq; a.uoff = c->uoff; a.ubs = c->ubs; a.uocc = c->uocc; a.urec = c->urec;
  a.iuniq = c->iuniq; a.ioff = c->ioff; a.ibs = c->ibs; a.iocc = c->iocc; a.irec = c->irec;
  a.g0 = c->g0; a.delta = c->delta; a.gsum = c->gsum;
  a.loss_clean = c->loss_clean; a.loss_adv = c->loss_adv;
  a.d = c->d; a.B = c->B; a.t = t;
  a.lr = hp->lr; a.eps = hp->eps; a.reg = hp->reg; a.reg_adv = hp->reg_adv;
  a.clip_lo = hp->clip_lo; a.clip_hi = hp->clip_hi;
  a.adver = hp->adver; a.adv_mode = hp->adv_mode; a.zero_delta = hp->zero_delta; a.seed = hp->seed;
  return a;
}

template <int LPR, int NV>
static void launch_clean(const StepArgs& a, hipStream_t s) {
  const int64_t threads = (int64_t)3 * a.B * LPR;
  k_clean<LPR, NV><<<grid_for(threads), 256, 0, s>>>(a);
}
template <int LPR, int NV>
static void launch_adv(const StepArgs& a, hipStream_t s) {
  const int64_t threads = (int64_t)3 * a.B * LPR;
  k_adv<LPR, NV><<<grid_for(threads), 256, 0, s>>>(a);
}
static void launch_apply(const StepArgs& a, hipStream_t s) {
  const int64_t threads = (int64_t)3 * a.B * (a.d / 4);
  k_apply<<<grid_for(threads), 256, 0, s>>>(a);
}

static int check_step(acf_apr_ctx* c, const acf_apr_tables* tb, const acf_apr_hparams* hp,
                      int32_t t) {
  ACF_CHECK(c && tb && hp, ACF_E_INVALID, "NULL ctx/tables/hparams");
  ACF_CHECK(tb->P && tb->Q && tb->accP && tb->accQ, ACF_E_INVALID, "NULL table pointer");
  ACF_CHECK(c->nb > 0, ACF_E_STATE, "no batches planned (call acf_apr_plan first)");
  ACF_CHECK(t >= 0 && t < c->nb, ACF_E_INVALID, "batch %d outside planned range [0, %d)", t, c->nb);
  return ACF_OK;
}

// one batch: [clean] [adv] apply, eagerly on stream s
static int run_batch(acf_apr_ctx* c, const StepArgs& a, bool need_clean, hipStream_t s) {
  if (need_clean) ACF_RET(DISPATCH_GEOM(c->d, launch_clean, a, s));
  if (a.adver) ACF_RET(DISPATCH_GEOM(c->d, launch_adv, a, s));
  launch_apply(a, s);
  HIP_TRY(hipGetLastError());
  return ACF_OK;
}

extern "C" int acf_apr_delta_update(acf_apr_ctx* c, const acf_apr_tables* tb,
                                    const acf_apr_hparams* hp, int32_t t, void* stream_) {
  ACF_RET(check_step(c, tb, hp, t));
  ACF_CHECK(hp->adver, ACF_E_INVALID, "delta_update needs hparams.adver = 1 (APR graph)");
  hipStream_t s = static_cast<hipStream_t>(stream_);
  StepArgs a = make_args(c, tb, hp, t);
  ACF_RET(DISPATCH_GEOM(c->d, launch_clean, a, s));
  HIP_TRY(hipGetLastError());
  c->last_delta_batch = t;
  return ACF_OK;
}

extern "C" int acf_apr_optimizer_step(acf_apr_ctx* c, const acf_apr_tables* tb,
                                      const acf_apr_hparams* hp, int32_t t, void* stream_) {
  ACF_RET(check_step(c, tb, hp, t));
  hipStream_t s = static_cast<hipStream_t>(stream_);
  StepArgs a = make_args(c, tb, hp, t);
  bool need_clean = true;
  if (hp->adver) {
    ACF_CHECK(c->last_delta_batch == t, ACF_E_STATE,
              "APR optimizer step on batch %d needs acf_apr_delta_update on the same batch first", t);
    need_clean = false;
  }
  ACF_RET(run_batch(c, a, need_clean, s));
  c->last_delta_batch = -1;
  return ACF_OK;
}

extern "C" int acf_apr_train_planned(acf_apr_ctx* c, const acf_apr_tables* tb,
                                     const acf_apr_hparams* hp, int32_t first, int32_t n,
                                     int32_t graph_mode, void* stream_) {
  ACF_CHECK(c && tb && hp, ACF_E_INVALID, "NULL ctx/tables/hparams");
  ACF_CHECK(n > 0 && first >= 0 && first + n <= c->nb, ACF_E_INVALID,
            "batch range [%d, %d) outside planned range [0, %d)", first, first + n, c->nb);
  ACF_RET(check_step(c, tb, hp, first));
  hipStream_t s = static_cast<hipStream_t>(stream_);
  if (!graph_mode) {
    for (int32_t t = first; t < first + n; ++t) ACF_RET(run_batch(c, make_args(c, tb, hp, t), true, s));
    c->last_delta_batch = -1;
    return ACF_OK;
  }
  GraphKey key;
  memset(&key, 0, sizeof(key));
  key.ptrs[0] = tb->P; key.ptrs[1] = tb->Q; key.ptrs[2] = tb->accP; key.ptrs[3] = tb->accQ;
  key.hp = *hp;
  key.first = first; key.n = n; key.B = c->B; key.d = c->d;
  auto it = c->graphs.find(key);
  if (it == c->graphs.end()) {
    hipGraph_t g = nullptr;
    HIP_TRY(hipStreamBeginCapture(c->cap_stream, hipStreamCaptureModeThreadLocal));
    int r = ACF_OK;
    for (int32_t t = first; t < first + n && r == ACF_OK; ++t)
      r = run_batch(c, make_args(c, tb, hp, t), true, c->cap_stream);
    hipError_t ec = hipStreamEndCapture(c->cap_stream, &g);
    if (r != ACF_OK) { if (g) (void)hipGraphDestroy(g); return r; }
    if (ec != hipSuccess) return set_error(ACF_E_HIP, "hipStreamEndCapture: %s", hipGetErrorString(ec));
    hipGraphExec_t ex = nullptr;
    hipError_t ei = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (ei != hipSuccess) return set_error(ACF_E_HIP, "hipGraphInstantiate: %s", hipGetErrorString(ei));
    if (c->graphs.size() >= 16) {  // bounded cache
      (void)hipGraphExecDestroy(c->graphs.begin()->second);
      c->graphs.erase(c->graphs.begin());
    }
    it = c->graphs.emplace(key, ex).first;
  }
  HIP_TRY(hipGraphLaunch(it->second, s));
  c->last_delta_batch = -1;
  return ACF_OK;
}

// kernel pointer per geometry, so hipExtLaunchKernelGGL can bracket it with events
template <int LPR, int NV>
static void pick_kernels(void** clean, void** adv) {
  *clean = reinterpret_cast<void*>(&k_clean<LPR, NV>);
  *adv = reinterpret_cast<void*>(&k_adv<LPR, NV>);
}

extern "C" int acf_apr_time_kernels(acf_apr_ctx* c, const acf_apr_tables* tb,
                                    const acf_apr_hparams* hp, int32_t first, int32_t n,
                                    double* ms_out, int32_t* launches_out, void* stream_) {
  ACF_CHECK(c && tb && hp && ms_out && launches_out, ACF_E_INVALID, "NULL argument");
  ACF_CHECK(n > 0 && first >= 0 && first + n <= c->nb, ACF_E_INVALID,
            "batch range [%d, %d) outside planned range [0, %d)", first, first + n, c->nb);
  ACF_RET(check_step(c, tb, hp, first));
  hipStream_t s = static_cast<hipStream_t>(stream_);
  void *kc = nullptr, *ka = nullptr;
  int lpr = 0, nv = 0;
  geometry(c->d, &lpr, &nv);
  ACF_RET(DISPATCH_GEOM(c->d, pick_kernels, &kc, &ka));
  const int kinds = 3;
  std::vector<hipEvent_t> ev((size_t)2 * kinds * n, nullptr);
  for (auto& e : ev) HIP_TRY(hipEventCreate(&e));
  for (int k = 0; k < kinds; ++k) { ms_out[k] = 0.0; launches_out[k] = 0; }
  for (int32_t t = first; t < first + n; ++t) {
    StepArgs a = make_args(c, tb, hp, t);
    const size_t base = (size_t)2 * kinds * (t - first);
    const dim3 gr((unsigned)grid_for((int64_t)3 * a.B * lpr)), bl(256);
    hipExtLaunchKernelGGL(reinterpret_cast<void (*)(StepArgs)>(kc), gr, bl, 0, s, ev[base + 0],
                          ev[base + 1], 0, a);
    if (a.adver)
      hipExtLaunchKernelGGL(reinterpret_cast<void (*)(StepArgs)>(ka), gr, bl, 0, s, ev[base + 2],
                            ev[base + 3], 0, a);
    hipExtLaunchKernelGGL(k_apply, dim3(grid_for((int64_t)3 * a.B * (a.d / 4))), bl, 0, s,
                          ev[base + 4], ev[base + 5], 0, a);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipStreamSynchronize(s));
  for (int32_t t = 0; t < n; ++t)
    for (int k = 0; k < kinds; ++k) {
      if (k == 1 && !hp->adver) continue;
      float ms = 0.f;
      const size_t base = (size_t)2 * kinds * t + 2 * k;
      HIP_TRY(hipEventElapsedTime(&ms, ev[base], ev[base + 1]));
      ms_out[k] += ms;
      launches_out[k] += 1;
    }
  for (auto& e : ev) (void)hipEventDestroy(e);
  c->last_delta_batch = -1;
  return ACF_OK;
}

extern "C" int acf_apr_copy_losses(acf_apr_ctx* c, float* lc, float* la, void* stream_) {
  ACF_CHECK(c, ACF_E_INVALID, "ctx is NULL");
  ACF_CHECK(c->nb > 0, ACF_E_STATE, "no batches planned");
  hipStream_t s = static_cast<hipStream_t>(stream_);
  const size_t n = (size_t)c->B * c->nb * sizeof(float);
  if (lc) HIP_TRY(hipMemcpyAsync(lc, c->loss_clean, n, hipMemcpyDeviceToDevice, s));
  if (la) HIP_TRY(hipMemcpyAsync(la, c->loss_adv, n, hipMemcpyDeviceToDevice, s));
  return ACF_OK;
}

extern "C" int acf_apr_delta_scatter(acf_apr_ctx* c, float* dP, float* dQ, void* stream_) {
  ACF_CHECK(c && dP && dQ, ACF_E_INVALID, "NULL argument");
  ACF_CHECK(c->last_delta_batch >= 0, ACF_E_STATE, "no delta computed since the last step");
  hipStream_t s = static_cast<hipStream_t>(stream_);
  acf_apr_tables tb{nullptr, nullptr, nullptr, nullptr};
  acf_apr_hparams hp;
  memset(&hp, 0, sizeof(hp));
  StepArgs a = make_args(c, &tb, &hp, c->last_delta_batch);
  k_delta_scatter<<<grid_for((int64_t)3 * c->B * (c->d / 4)), 256, 0, s>>>(a, dP, dQ);
  HIP_TRY(hipGetLastError());
  return ACF_OK;
}

template <int LPR, int NV>
static void launch_forward(const float* P, const float* Q, int d, const int32_t* u,
                           const int32_t* i, const int32_t* j, int B, int nb, float lo, float hi,
                           float* bl, int32_t* bc, float* op, float* on, hipStream_t s) {
  k_forward<LPR, NV><<<nb, 256, 0, s>>>(P, Q, d, u, i, j, B, lo, hi, bl, bc, op, on);
}

extern "C" int acf_bpr_forward(const float* P, const float* Q, int64_t U1, int64_t I1, int32_t d,
                               const int32_t* u, const int32_t* i, const int32_t* j, int32_t B,
                               int32_t nb, float lo, float hi, float* bl, int32_t* bc, float* op,
                               float* on, void* stream_) {
  ACF_RET(check_dim(d));
  ACF_CHECK(P && Q && u && i && j, ACF_E_INVALID, "NULL argument");
  ACF_CHECK(B > 0 && nb > 0 && U1 > 0 && I1 > 0, ACF_E_INVALID, "empty problem");
  hipStream_t s = static_cast<hipStream_t>(stream_);
  ACF_RET(DISPATCH_GEOM(d, launch_forward, P, Q, d, u, i, j, B, nb, lo, hi, bl, bc, op, on, s));
  HIP_TRY(hipGetLastError());
  return ACF_OK;
}

extern "C" int acf_eval_positions_all(const float* P, const float* Q, int64_t U1, int64_t I1,
                                      int32_t d, const int32_t* users, const int32_t* tests,
                                      int32_t n_users, int32_t num_cand, const int64_t* excl_off,
                                      const int32_t* excl, int32_t* positions, void* stream_) {
  ACF_RET(check_dim(d));
  ACF_CHECK(P && Q && users && tests && excl_off && positions, ACF_E_INVALID, "NULL argument");
  ACF_CHECK(num_cand >= 0 && num_cand <= I1, ACF_E_INVALID, "num_candidates %d > item rows", num_cand);
  if (n_users <= 0) return ACF_OK;
  hipStream_t s = static_cast<hipStream_t>(stream_);
  const size_t lds = (size_t)EVAL_UB * d * sizeof(float);
  k_eval_all<<<(n_users + EVAL_UB - 1) / EVAL_UB, 256, lds, s>>>(P, Q, d, users, tests, n_users,
                                                                  num_cand, excl_off, excl, positions);
  HIP_TRY(hipGetLastError());
  return ACF_OK;
}

extern "C" int acf_eval_positions_list(const float* P, const float* Q, int64_t U1, int64_t I1,
                                       int32_t d, const int32_t* users, const int32_t* tests,
                                       int32_t n_users, const int64_t* cand_off,
                                       const int32_t* cand, int32_t* positions, void* stream_) {
  ACF_RET(check_dim(d));
  ACF_CHECK(P && Q && users && tests && cand_off && positions, ACF_E_INVALID, "NULL argument");
  if (n_users <= 0) return ACF_OK;
  hipStream_t s = static_cast<hipStream_t>(stream_);
  k_eval_list<<<n_users, 256, d * sizeof(float), s>>>(P, Q, d, users, tests, cand_off, cand, positions);
  HIP_TRY(hipGetLastError());
  return ACF_OK;
}

extern "C" int acf_sample_epoch(const int32_t* pu, const int32_t* pi, int64_t n_pos, int32_t B,
                                int32_t num_items, int32_t num_lists, const int64_t* loff,
                                const int32_t* litems, uint64_t seed, int32_t max_tries,
                                int32_t check, int32_t* ou, int32_t* op, int32_t* on,
                                void* stream_) {
  ACF_CHECK(pu && pi && loff && ou && op && on, ACF_E_INVALID, "NULL argument");
  ACF_CHECK(B > 0 && num_items > 0 && n_pos >= 0 && n_pos < (1ll << 31), ACF_E_INVALID,
            "bad sizes");
  const int64_t n_out = (n_pos / B) * B;
  if (n_out == 0) return ACF_OK;
  hipStream_t s = static_cast<hipStream_t>(stream_);
  uint64_t *k_in = nullptr, *k_out = nullptr;
  int32_t *v_in = nullptr, *v_out = nullptr, *err = nullptr;
  void* tmp = nullptr;
  size_t tb = 0;
  HIP_TRY(rocprim::radix_sort_pairs(nullptr, tb, k_in, k_out, v_in, v_out, (size_t)n_pos, 0, 64));
  HIP_TRY(hipMallocAsync((void**)&k_in, n_pos * 8, s));
  HIP_TRY(hipMallocAsync((void**)&k_out, n_pos * 8, s));
  HIP_TRY(hipMallocAsync((void**)&v_in, n_pos * 4, s));
  HIP_TRY(hipMallocAsync((void**)&v_out, n_pos * 4, s));
  HIP_TRY(hipMallocAsync((void**)&err, 16, s));
  HIP_TRY(hipMallocAsync(&tmp, tb + 16, s));
  HIP_TRY(hipMemsetAsync(err, 0, 16, s));
  k_perm_keys<<<grid_for(n_pos), 256, 0, s>>>(n_pos, seed, k_in, v_in);
  HIP_TRY(rocprim::radix_sort_pairs(tmp, tb, k_in, k_out, v_in, v_out, (size_t)n_pos, 0, 64, s));
  k_negatives<<<grid_for(n_out), 256, 0, s>>>(v_out, pu, pi, n_out, num_items, num_lists, loff,
                                              litems, seed, max_tries, ou, op, on, err);
  HIP_TRY(hipGetLastError());
  int32_t herr = 0;
  if (check) HIP_TRY(hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipFreeAsync(k_in, s));
  HIP_TRY(hipFreeAsync(k_out, s));
  HIP_TRY(hipFreeAsync(v_in, s));
  HIP_TRY(hipFreeAsync(v_out, s));
  HIP_TRY(hipFreeAsync(tmp, s));
  HIP_TRY(hipFreeAsync(err, s));
  if (check) {
    HIP_TRY(hipStreamSynchronize(s));
    ACF_CHECK(herr == 0, ACF_E_RANGE, "sampler: %s%s", (herr & 1) ? "user outside trainList " : "",
              (herr & 2) ? "no admissible negative within max_tries" : "");
  }
  return ACF_OK;
}

template <int LPR, int NV>
static void launch_dns(const float* P, const float* Q, int d, const int32_t* u, const int32_t* cand,
                       int64_t n, int dns, int32_t* out, hipStream_t s) {
  k_dns_select<LPR, NV><<<grid_for(n * LPR), 256, 0, s>>>(P, Q, d, u, cand, n, dns, out);
}

extern "C" int acf_dns_select(const float* P, const float* Q, int64_t U1, int64_t I1, int32_t d,
                              const int32_t* u, const int32_t* cand, int64_t n, int32_t dns,
                              int32_t* out, void* stream_) {
  ACF_RET(check_dim(d));
  ACF_CHECK(P && Q && u && cand && out && dns > 0, ACF_E_INVALID, "bad argument");
  if (n <= 0) return ACF_OK;
  hipStream_t s = static_cast<hipStream_t>(stream_);
  ACF_RET(DISPATCH_GEOM(d, launch_dns, P, Q, d, u, cand, n, dns, out, s));
  HIP_TRY(hipGetLastError());
  return ACF_OK;
}
