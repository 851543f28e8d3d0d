// acf_neumf.hip — MI355X (gfx950) kernels + C-ABI for NeuMF and adversarial
// NeuMF training (include/acf_neumf.h; SURVEY.md §8(f)3, BASELINE configs[3]).
//
// Reference graph: NeuMF.py:10-52 (Keras), trained by MF.py:30-33 (fit: mean
// binary cross-entropy + Adam) and scored by MF.py:38-40.  One training step
// (Keras train_on_batch) here:
//
//   k_nmf_inst<CLEAN>   workgroups looping over blocks of 16 instances: gather
//                       MF_U[u], MF_I[i], MLP_U[u], MLP_I[i]; MLP [2d -> 2d -> d]
//                       relu on f32 MFMA (16x16x4, exact f32 products); head;
//                       BCE (prediction clipped to [1e-7, 1-1e-7]); backward
//                       through head and MLP; per-instance row contributions;
//                       the weight gradients of the block (outer products over
//                       its 16 instances on MFMA) into the workgroup's slot
//   k_nmf_rows          one wave per (instance, side): the row's first
//                       occurrence owns it and sums every occurrence's
//                       contribution in instance order into the gradient row;
//                       with adver also delta = eps * g / |g| of that row.  The
//                       step's last k_nmf_rows launch also sums the weight-
//                       gradient slots in slot order (deterministic, no atomics)
//   (adver) k_nmf_inst<ADV>, k_nmf_rows on the perturbed rows, scaled by reg_adv
//
// Batches of <= FR_MAXB instances (r05) sum their rows in line instead: one
// k_nmf_step launch per adversarial step (k_nmf_inst<MODE, DC, true> per pass
// otherwise) holds the instance workgroups, which take their weight-gradient
// tiles from LDS and count arrivals at their rows, and the row waves, whose
// owners wait for the arrivals and sum the rows in k_nmf_rows' order.
//   k_nmf_adam          Keras 2.2 Adam over the WHOLE flat parameter buffer
//                       (Keras densifies the embedding IndexedSlices, so every
//                       row's moments decay and every row moves): one HBM
//                       stream of p, g, m, v, zeroing g behind it.
//
// acf_neumf_train runs that Adam lazily, with the same arithmetic per element
// (bit-identical results): a row's zero-gradient iterations are deferred until
// the next batch gathers it (k_nmf_adam_next, with the MLP / head parameters on
// the caller's stream) or a rotating catch-up slice on a side stream reaches it
// (k_nmf_adam_catchup, beside the next step's latency-bound kernels), so a step
// moves the rows it touches instead of the whole tables.
//
// The MLP is tiny per instance (2d x 2d and 2d x d at d = 64); the step is a
// latency-bound chain (gather -> 4 MFMA layers -> weight gradients -> rows).

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <string>
#include <vector>

#include "acf_apr.h"
#include "acf_neumf.h"

static thread_local std::string g_neumf_error;

static int set_error(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_neumf_error = buf;
  return code;
}

#define HIP_TRY(expr)                                                             \
  do {                                                                            \
    hipError_t e_ = (expr);                                                       \
    if (e_ != hipSuccess)                                                         \
      return set_error(ACF_E_HIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

#define ACF_CHECK(cond, code, ...)                      \
  do {                                                  \
    if (!(cond)) return set_error((code), __VA_ARGS__); \
  } while (0)

// parameter segments, in Keras order
enum { S_MF_U = 0, S_MF_I, S_MLP_U, S_MLP_I, S_W1, S_B1, S_W2, S_B2, S_WO, S_BO, S_COUNT };

struct Layout {
  int64_t off[S_COUNT];
  int64_t total;
};

static Layout make_layout(int64_t U1, int64_t I1, int64_t d) {
  Layout L;
  L.off[S_MF_U] = 0;
  L.off[S_MF_I] = U1 * d;
  L.off[S_MLP_U] = (U1 + I1) * d;
  L.off[S_MLP_I] = (2 * U1 + I1) * d;
  L.off[S_W1] = 2 * (U1 + I1) * d;
  L.off[S_B1] = L.off[S_W1] + 4 * d * d;
  L.off[S_W2] = L.off[S_B1] + 2 * d;
  L.off[S_B2] = L.off[S_W2] + 2 * d * d;
  L.off[S_WO] = L.off[S_B2] + d;
  L.off[S_BO] = L.off[S_WO] + 2 * d;
  L.total = L.off[S_BO] + 4;  // bo + pad: every segment starts 16-B aligned
  return L;
}


struct NArgs {
  const float* P;
  float* G;
  int64_t off[S_COUNT];
  const int32_t* u;
  const int32_t* i;
  const float* y;
  int64_t U1, I1;
  int32_t B, d;
  float scale_over_B;    // 1/B (clean) or reg_adv/B (adversarial)
  float* contrib;        // [B][4][d] per-instance row contributions
  // the activations the weight gradients need (k_nmf_inst -> k_nmf_rows' gradient workgroups)
  float *h0, *a1, *dz1, *dz2;  // [B][2d], [B][2d], [B][2d], [B][d]
  float* wpart;          // [gridDim.x][nout] this pass's weight-gradient partials (one slot per workgroup)
  const float* delta;    // [B][4][d], rows written at their owner instance
  const int32_t* owner;  // [B][2] first occurrence of the instance's user / item
  // rows in line (k_nmf_inst<.., .., true>, B <= FR_MAXB): arrivals at each row
  // (users, then items; zero between passes), and the clean pass's delta
  int32_t* rcnt;         // [U1 + I1]
  int32_t with_delta;
  float eps;
  // both passes in one launch (k_nmf_step): per row, (gen << 32 | its first
  // occurrence) once the clean pass's owner has stored the row's delta and gradient
  unsigned long long* rdone;  // [U1 + I1]
  int32_t gen;
  // polls a rows-in-line wait makes before it gives up (err bit 512; 0: give up at
  // once -- acf_neumf_set_spin_limit, the failsafe's forcing test)
  int32_t spin;
  float* pred;
  int32_t* err;
};

__device__ __forceinline__ int32_t clamp_idx(int32_t r, int64_t n) { return (r < 0 || r >= n) ? 0 : r; }

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int MR = 16;        // instances per block = the MFMA tile height
constexpr int NSLOT = 256;    // workgroups (= weight-gradient partial slots) per training pass, at most
constexpr int DFAST = 64;     // the dimension with a compile-time specialisation of k_nmf_inst
constexpr int MAX_Q = 2;      // d <= 128: each lane holds up to 2 of a row's elements
// occurrences whose contributions are loaded together (r05 same-box A/B, yelp
// shape: 1 / 2 / 3 / 4 / 8 / 16 -> 7.40-7.50 / 7.47-7.49 / 7.44-7.48 / 7.43-7.58 /
// 7.18-7.19 / 6.61-6.68M instances/s; most rows have few occurrences, and the
// unrolled predicated loads of a wide batch cost more than the round trips save;
// profiles/r05/neumf_rbatch_ab.txt)
constexpr int RBATCH = 4;
// rows in line (k_nmf_inst<MODE, DC, true>) up to this batch: one block of MR
// instances per workgroup, the batch's indices in LDS
constexpr int FR_MAXB = 1024;

// device-scope write-through store / load of one float (the contributions a row's
// last arrival in another workgroup reads in the same launch; MI355X guide,
// Guideline 16: no L2 write-back or invalidate)
__device__ __forceinline__ void st_wt(float* p, float v) {
  asm volatile("global_store_dword %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ float ld_dev(const float* p) {
  return __uint_as_float(__hip_atomic_load((const __attribute__((address_space(1))) uint32_t*)p, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT));
}

// Weight-gradient partial vector of one workgroup: the parameter buffer's tail from
// S_W1 on, element for element -- W1 [2d][2d] | b1 [2d] | W2 [2d][d] | b2 [d] |
// Wo [2d] | bo | (pad: the loss sum, 2 spare) -- so slot element x is the gradient
// of parameter off[S_W1] + x, and the slot sum can ride on the Adam stream.
struct WOut {
  int64_t w1, b1, w2, b2, wo, bo, loss, n;
};

__host__ __device__ __forceinline__ WOut wout(int64_t d) {
  WOut o;
  o.w1 = 0;
  o.b1 = 4 * d * d;
  o.w2 = o.b1 + 2 * d;
  o.b2 = o.w2 + 2 * d * d;
  o.wo = o.b2 + d;
  o.bo = o.wo + 2 * d;
  o.loss = o.bo + 1;
  o.n = o.bo + 4;  // = Layout total - off[S_W1], a multiple of 4
  return o;
}

// W1 and W2 are staged in LDS (row stride +1 float: the transposed reads of the
// backward products are then conflict-free) when they fit beside the activations
__host__ __device__ __forceinline__ bool weights_in_lds(int d) { return d <= 64; }

// k_nmf_inst's LDS in floats (the rows-in-line batch indices come after it)
__host__ __device__ __forceinline__ int64_t inst_floats(int d) {
  int64_t f = (int64_t)3 * MR * (2 * d + 1) + 3 * MR * (d + 1) + 2 * MR + 5 * d + 4;
  if (weights_in_lds(d)) f += (int64_t)2 * d * (2 * d + 1) + (int64_t)2 * d * (d + 1);
  return f;
}

// C[MR x N] = A[MR x K] . w(k, n) on v_mfma_f32_16x16x4_f32 (exact f32 products,
// k-ordered fma chain).  A: LDS, row-major with leading dimension lda (padded so
// the 16 lanes reading one k hit different banks); w(k, n) = W[k*ldw + n], or
// W[n*ldw + k] with TRANS (the backward products with W^T).  The 4 waves take
// 32-column panels (two 16x16 tiles, two independent accumulators) round-robin;
// epi(row, col, value) consumes every output element.  With a compile-time d
// every bound and offset folds to an immediate.
// Lane maps (cdna_hip_programming.md §3): A[l&15][k0 + (l>>4)], B[k0 + (l>>4)][l&15],
// C/D: col = l&15, row = 4*(l>>4) + reg.
template <bool TRANS>
__device__ __forceinline__ float w_at(const float* __restrict__ W, int ldw, int k, int col) {
  return TRANS ? W[(int64_t)col * ldw + k] : W[(int64_t)k * ldw + col];
}

template <bool TRANS, class Epi>
__device__ __forceinline__ void mfma_panel(const float* sA, int lda, const float* __restrict__ W, int ldw,
                                           int K, int N, Epi epi) {
  constexpr int KB = 8;  // k-steps whose operands are read before their MFMAs issue
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 15, h = lane >> 4;
  if (N > 64) {
    // two 16-column tiles per wave (independent accumulators), 32-column panels
    for (int n0 = wave * 32; n0 < N; n0 += 4 * 32) {
      f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
      const int ca = n0 + r, cb = n0 + 16 + r;
      for (int kb = 0; kb < K; kb += 4 * KB) {
        float av[KB], ba[KB], bb[KB];
#pragma unroll
        for (int j = 0; j < KB; ++j) {
          const int k = kb + 4 * j + h;
          const bool ok = k < K;
          av[j] = ok ? sA[r * lda + k] : 0.f;
          ba[j] = (ok && ca < N) ? w_at<TRANS>(W, ldw, k, ca) : 0.f;
          bb[j] = (ok && cb < N) ? w_at<TRANS>(W, ldw, k, cb) : 0.f;
        }
#pragma unroll
        for (int j = 0; j < KB; ++j) {
          c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j], ba[j], c0, 0, 0, 0);
          c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j], bb[j], c1, 0, 0, 0);
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (ca < N) epi(4 * h + q, ca, c0[q]);
        if (cb < N) epi(4 * h + q, cb, c1[q]);
      }
    }
  } else {
    // N <= 64: one 16-column tile per wave, K split over two accumulators
    const int c = wave * 16 + r;
    if (wave * 16 >= N) return;
    f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
    for (int kb = 0; kb < K; kb += 8 * KB) {
      float a0[KB], a1[KB], w0[KB], w1[KB];
#pragma unroll
      for (int j = 0; j < KB; ++j) {
        const int k = kb + 8 * j + h, k1 = k + 4;
        a0[j] = k < K ? sA[r * lda + k] : 0.f;
        a1[j] = k1 < K ? sA[r * lda + k1] : 0.f;
        w0[j] = (k < K && c < N) ? w_at<TRANS>(W, ldw, k, c) : 0.f;
        w1[j] = (k1 < K && c < N) ? w_at<TRANS>(W, ldw, k1, c) : 0.f;
      }
#pragma unroll
      for (int j = 0; j < KB; ++j) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[j], w0[j], c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[j], w1[j], c1, 0, 0, 0);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (c < N) epi(4 * h + q, c, c0[q] + c1[q]);
  }
}

// Weight gradients of a block over its MR instances, 16x16 output tiles:
// W1 += h0^T dz1 [2d][2d], then W2 += a1^T dz2 [2d][d];
// out[k][n] (+)= sum_t A[t][k] * Bm[t][n] with A / Bm in LDS (row t), a t-ordered
// chain of 4 MFMAs per tile; each wave takes OG tiles at a time (independent
// chains).  The slot is accumulated across the workgroup's blocks (ACC: add to what
// this lane stored for the previous block -- the same lane, the same address).
constexpr int OG = 4;

// one weight gradient [K][N] (A rows with leading dimension lda, Bm rows ldb),
// its tiles [tlo, thi) (row-major over 16x16 tiles); EXACT: K and N multiples of
// 16 (no bounds); tiles tt = tlo + wave + 4 * (OG*i + g)
template <bool ACC, bool EXACT>
__device__ __forceinline__ void outer_mat(const float* A, int lda, const float* Bm, int ldb, int K, int N,
                                          float* __restrict__ out, int tlo, int thi) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 15, h = lane >> 4;
  const int tn = (N + 15) / 16, T = thi;
  const float* Ar = A + h * lda + r;   // lane's element of row t = h, column r
  const float* Br = Bm + h * ldb + r;
  for (int tb = tlo + wave; tb < T; tb += 4 * OG) {
    float av[OG][MR / 4], bv[OG][MR / 4];
    int k0[OG], n0[OG];
#pragma unroll
    for (int g = 0; g < OG; ++g) {
      const int tt = tb + 4 * g;  // wave-uniform
      k0[g] = (tt / tn) * 16;
      n0[g] = (tt % tn) * 16;
#pragma unroll
      for (int j = 0; j < MR / 4; ++j) {
        const bool okA = tt < T && (EXACT || k0[g] + r < K), okB = tt < T && (EXACT || n0[g] + r < N);
        av[g][j] = okA ? Ar[4 * j * lda + k0[g]] : 0.f;
        bv[g][j] = okB ? Br[4 * j * ldb + n0[g]] : 0.f;
      }
    }
    f32x4 c[OG];
#pragma unroll
    for (int g = 0; g < OG; ++g) c[g] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < MR / 4; ++j)
#pragma unroll
      for (int g = 0; g < OG; ++g) c[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[g][j], bv[g][j], c[g], 0, 0, 0);
#pragma unroll
    for (int g = 0; g < OG; ++g) {
      if (tb + 4 * g >= T) break;
      float* o = out + (int64_t)(k0[g] + 4 * h) * N + n0[g] + r;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (EXACT || (k0[g] + 4 * h + q < K && n0[g] + r < N)) {
          float* p = o + (int64_t)q * N;
          *p = ACC ? *p + c[g][q] : c[g][q];  // (ACC a template: no speculative load of the slot)
        }
      }
    }
  }
}

// tiles [lo, hi) of the two gradients' tile space (W1's T1 tiles, then W2's)
__host__ __device__ __forceinline__ int wtiles1(int d) { return ((2 * d + 15) / 16) * ((2 * d + 15) / 16); }
__host__ __device__ __forceinline__ int wtiles(int d) { return wtiles1(d) + ((2 * d + 15) / 16) * ((d + 15) / 16); }

template <bool ACC, bool EXACT>
__device__ __forceinline__ void outer_tiles(const float* s_h0, const float* s_dz1, const float* s_a1,
                                            const float* s_dz2, int d, float* __restrict__ w1,
                                            float* __restrict__ w2, int lo, int hi) {
  const int d2 = 2 * d, T1 = wtiles1(d);
  if (lo < T1) outer_mat<ACC, EXACT>(s_h0, d2 + 1, s_dz1, d2 + 1, d2, d2, w1, lo, min(hi, T1));
  if (hi > T1) outer_mat<ACC, EXACT>(s_a1, d2 + 1, s_dz2, d + 1, d2, d, w2, max(lo, T1) - T1, hi - T1);
}

// k_nmf_rows' weight-gradient workgroups take the tiles in groups of one wave round
constexpr int WG_TILES = 4 * OG;

// Weight-gradient workgroup (slot w, tile group g) -- extra workgroups of the NEXT
// launch after k_nmf_inst (the adversarial k_nmf_inst for the clean pass, the last
// k_nmf_rows for the adversarial pass), which leave most CUs idle: for the blocks
// w, w + nslot, ... of k_nmf_inst's 16 instances, stage h0, dz1, a1, dz2 in LDS
// (padded rows; instances past the batch are zero) and add tiles
// [g WG_TILES, (g+1) WG_TILES) of W1 += h0^T dz1, W2 += a1^T dz2 to slot w (the
// slot k_nmf_inst's workgroup w writes the vector partials of).
#ifdef NMF_DIAG
__device__ uint64_t g_nmf_wstamps[8];  // weight-gradient workgroup (0, 0) of the last launch that ran one
#define WSTAMP(i)                                                                          \
  do {                                                                                     \
    uint64_t t_;                                                                           \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");         \
    if (w == 0 && g == 0 && threadIdx.x == 0) g_nmf_wstamps[i] = t_;                      \
  } while (0)
#else
#define WSTAMP(i) \
  do {            \
  } while (0)
#endif

template <bool EXACT>
__device__ __forceinline__ void wgrad_group(const NArgs& a, int w, int g, int nslot, float* sm) {
  WSTAMP(0);
  const int d = a.d, d2 = 2 * d, L2 = d2 + 1, L1 = d + 1, tid = threadIdx.x;
  float* s_h0 = sm;
  float* s_dz1 = s_h0 + MR * L2;
  float* s_a1 = s_dz1 + MR * L2;
  float* s_dz2 = s_a1 + MR * L2;
  const WOut o = wout(d);
  float* slot = a.wpart + (int64_t)w * o.n;
  const int64_t nblk = ((int64_t)a.B + MR - 1) / MR;
  const int lo = g * WG_TILES, hi = min(lo + WG_TILES, wtiles(d));
  for (int64_t blk = w; blk < nblk; blk += nslot) {
    const int64_t b0 = blk * MR;
    const int nt = (int)min((int64_t)MR, (int64_t)a.B - b0);
    if (blk != w) __syncthreads();  // the previous block's tiles are done with LDS
    // every load first (one round trip), the LDS stores after them
    constexpr int QA = MR * 256 / 256, QB = MR * 128 / 256;  // d <= 128
    float v0[QA], v1[QA], v2[QA], v3[QB];
#pragma unroll
    for (int q = 0; q < QA; ++q) {
      const int x = tid + 256 * q, t = x / d2, k = x - t * d2;
      if (256 * q < MR * d2) {  // uniform (MR d2 is a multiple of 64)
        const int64_t gi = (b0 + (x < MR * d2 && t < nt ? t : 0)) * d2 + (x < MR * d2 ? k : 0);
        v0[q] = a.h0[gi];
        v1[q] = a.dz1[gi];
        v2[q] = a.a1[gi];
      }
    }
#pragma unroll
    for (int q = 0; q < QB; ++q) {
      const int x = tid + 256 * q, t = x / d, k = x - t * d;
      if (256 * q < MR * d) v3[q] = a.dz2[(b0 + (x < MR * d && t < nt ? t : 0)) * d + (x < MR * d ? k : 0)];
    }
    WSTAMP(1);
#pragma unroll
    for (int q = 0; q < QA; ++q) {
      const int x = tid + 256 * q, t = x / d2, k = x - t * d2;
      if (x < MR * d2) {
        const bool ok = t < nt;
        s_h0[t * L2 + k] = ok ? v0[q] : 0.f;
        s_dz1[t * L2 + k] = ok ? v1[q] : 0.f;
        s_a1[t * L2 + k] = ok ? v2[q] : 0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < QB; ++q) {
      const int x = tid + 256 * q, t = x / d, k = x - t * d;
      if (x < MR * d) s_dz2[t * L1 + k] = t < nt ? v3[q] : 0.f;
    }
    __syncthreads();
    WSTAMP(2);
    if (blk == w)
      outer_tiles<false, EXACT>(s_h0, s_dz1, s_a1, s_dz2, d, slot + o.w1, slot + o.w2, lo, hi);
    else
      outer_tiles<true, EXACT>(s_h0, s_dz1, s_a1, s_dz2, d, slot + o.w1, slot + o.w2, lo, hi);
    WSTAMP(3);
  }
}

static size_t wgrad_smem(int d) { return (size_t)MR * (3 * (2 * d + 1) + (d + 1)) * sizeof(float); }

#ifndef ACF_SPIN_LIMIT
#define ACF_SPIN_LIMIT (1 << 22)
#endif

// Rows in line (k_nmf_inst<MODE, DC, true>): the last arrival at a row (side s,
// row r, first occurrence f; L = the side's clamped batch indices in LDS) sums
// every occurrence's contribution in instance order -- k_nmf_rows' sum, bit for
// bit -- adds it to the gradient rows and (with_delta) writes delta at f.  One wave;
// the contributions are loaded RB occurrences at a time.
// MG (both passes in one launch): the clean pass stores the row write-through and
// then publishes it (rdone); the adversarial pass reads the gradient row that way.
template <int MODE, bool MG>
__device__ __forceinline__ void row_finish(const NArgs& a, const int32_t* L, int s, int32_t r, int f) {
  constexpr int RB = RBATCH;
  const int lane = threadIdx.x & 63, B = a.B, d = a.d;
  const int tA = s ? S_MF_I : S_MF_U, tB = s ? S_MLP_I : S_MLP_U;
  float gA[MAX_Q], gB[MAX_Q], oA[MAX_Q], oB[MAX_Q];
#pragma unroll
  for (int q = 0; q < MAX_Q; ++q) {
    const int k = lane + 64 * q;
    gA[q] = gB[q] = 0.f;
    const float* pA = a.G + a.off[tA] + (int64_t)r * d + k;
    const float* pB = a.G + a.off[tB] + (int64_t)r * d + k;
    oA[q] = k < d ? (MG && MODE == 1 ? ld_dev(pA) : *pA) : 0.f;
    oB[q] = k < d ? (MG && MODE == 1 ? ld_dev(pB) : *pB) : 0.f;
  }
  // occurrences in instance order, RB per round trip across 64-instance chunks
  // (a row's occurrences are spread over the batch: one chunk at a time would be
  // one round trip per chunk)
  int base = f & ~63;
  uint64_t mask = __ballot(base + lane < B && base + lane >= f && L[base + lane] == r);
  while (true) {
    int js[RB];
#pragma unroll
    for (int e = 0; e < RB; ++e) {
      while (!mask && base + 64 < B) {
        base += 64;
        mask = __ballot(base + lane < B && L[base + lane] == r);
      }
      js[e] = -1;
      if (mask) {
        js[e] = base + __ffsll((unsigned long long)mask) - 1;
        mask &= mask - 1;
      }
    }
    if (js[0] < 0) break;
    {
      float va[RB][MAX_Q], vb[RB][MAX_Q];
#pragma unroll
      for (int e = 0; e < RB; ++e)
#pragma unroll
        for (int q = 0; q < MAX_Q; ++q) {
          const int k = lane + 64 * q;
          const bool ok = js[e] >= 0 && k < d;
          va[e][q] = ok ? ld_dev(a.contrib + ((int64_t)js[e] * 4 + tA) * d + k) : 0.f;
          vb[e][q] = ok ? ld_dev(a.contrib + ((int64_t)js[e] * 4 + tB) * d + k) : 0.f;
        }
#pragma unroll
      for (int e = 0; e < RB; ++e)
        if (js[e] >= 0)
#pragma unroll
          for (int q = 0; q < MAX_Q; ++q) {
            gA[q] = gA[q] + va[e][q];
            gB[q] = gB[q] + vb[e][q];
          }
    }
  }
  float ssA = 0.f, ssB = 0.f;
#pragma unroll
  for (int q = 0; q < MAX_Q; ++q) {
    const int k = lane + 64 * q;
    if (k < d) {
      float* pA = a.G + a.off[tA] + (int64_t)r * d + k;
      float* pB = a.G + a.off[tB] + (int64_t)r * d + k;
      if (MG && MODE == 0) {
        st_wt(pA, oA[q] + gA[q]);
        st_wt(pB, oB[q] + gB[q]);
      } else {
        *pA = oA[q] + gA[q];
        *pB = oB[q] + gB[q];
      }
      ssA = ssA + gA[q] * gA[q];
      ssB = ssB + gB[q] * gB[q];
    }
  }
  if (!a.with_delta) return;
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    ssA += __shfl_xor(ssA, m, 64);
    ssB += __shfl_xor(ssB, m, 64);
  }
  const float invA = 1.0f / sqrtf(fmaxf(ssA, 1e-12f)), invB = 1.0f / sqrtf(fmaxf(ssB, 1e-12f));
  float* delta = const_cast<float*>(a.delta);
#pragma unroll
  for (int q = 0; q < MAX_Q; ++q) {
    const int k = lane + 64 * q;
    if (k < d) {
      float* dA = delta + ((int64_t)f * 4 + tA) * d + k;
      float* dB = delta + ((int64_t)f * 4 + tB) * d + k;
      if (MG) {
        st_wt(dA, gA[q] * invA * a.eps);
        st_wt(dB, gB[q] * invB * a.eps);
      } else {
        *dA = gA[q] * invA * a.eps;
        *dB = gB[q] * invB * a.eps;
      }
    }
  }
  if (MG && MODE == 0) {  // the row is out: publish it to the adversarial pass
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0)
      __hip_atomic_store(a.rdone + (s ? a.U1 : 0) + r, ((unsigned long long)(uint32_t)a.gen << 32) | (uint32_t)f,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

#ifdef NMF_DIAG  // diagnostic build only: phase stamps (100 MHz) of workgroup 0, clean pass
__device__ uint64_t g_nmf_stamps[16];
__device__ uint64_t g_nmf_rstamps[8];  // k_nmf_rows, workgroup 0 wave 0 (owner of u[0]), clean pass
#define RSTAMP(i)                                                                          \
  do {                                                                                     \
    uint64_t t_;                                                                           \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");         \
    if (with_delta && blockIdx.x == 0 && threadIdx.x == 0) g_nmf_rstamps[i] = t_;          \
  } while (0)
#define NSTAMP(i)                                                                          \
  do {                                                                                     \
    uint64_t t_;                                                                           \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");         \
    if (MODE == 0 && blockIdx.x == 0 && threadIdx.x == 0) g_nmf_stamps[i] = t_;           \
  } while (0)
#else
#define NSTAMP(i) \
  do {            \
  } while (0)
#define RSTAMP(i) \
  do {            \
  } while (0)
#endif

// Row waves of a rows-in-line launch (k_nmf_inst workgroups past the instance
// workgroups): k_nmf_rows' wave per (instance, side) -- find the pair's first
// occurrence (the clean pass records it for the adversarial pass's delta
// gathers) -- then the row's owner counts the row's occurrences, waits until that
// many arrivals are in (no wave of the instance workgroups ever waits for a row
// wave, and they are dispatched first), re-arms the counter and sums the row
// (row_finish).
template <int MODE, bool MG>
__device__ __forceinline__ void row_wait_finish_one(const NArgs& a, const int32_t* s_idx, int b, int s) {
  const int lane = threadIdx.x & 63, B = a.B;
  const int32_t* L = s_idx + s * B;
  const int32_t r = L[b];
  int first = b;
  for (int base = 0; base <= b; base += 64) {
    const int j = base + lane;
    const uint64_t mask = __ballot(j <= b && L[j] == r);
    if (mask) {
      first = base + __ffsll((unsigned long long)mask) - 1;
      break;
    }
  }
  if (MODE == 0 && lane == 0) const_cast<int32_t*>(a.owner)[2 * b + s] = first;
  if (first != b) return;
  int cnt = 0;
  for (int base = b & ~63; base < B; base += 64) {
    const int j = base + lane;
    cnt += __popcll(__ballot(j < B && j >= b && L[j] == r));
  }
  int32_t* ctr = a.rcnt + (s ? a.U1 : 0) + r;
  // a give-up leaves the launch's results undefined (never its addresses: every
  // index is clamped) and its counters stale: the host resets them and, with the
  // failsafe on, replays the call on the row-sum path (acf_neumf_train / _grad)
  if (a.spin == 0 && lane == 0) atomicOr(a.err, 512);  // forced: every owner reports a give-up
  for (int it = 0; __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < cnt;) {
    if (++it > a.spin) {
      if (lane == 0) atomicOr(a.err, 512);
      break;
    }
    __builtin_amdgcn_s_sleep(8);
  }
  if (lane == 0) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // every arrival is in
  // (r05 same-box A/B: hot rows' contributions 8 or 16 at a time measured the same
  // as RBATCH, 8.35-8.61M instances/s, profiles/r05/neumf_rows_in_line_ab.txt)
  row_finish<MODE, MG>(a, L, s, r, b);
}

// a row workgroup: the batch's indices into LDS, then its waves' pairs (strided
// over the row workgroups)
template <int MODE, bool MG>
__device__ __forceinline__ void row_wait_finish(const NArgs& a, unsigned fb, unsigned nrow, int32_t* s_idx) {
  const int tid = threadIdx.x, wave = tid >> 6, B = a.B;
  {
    int32_t su[FR_MAXB / 256], si[FR_MAXB / 256];
#pragma unroll
    for (int q = 0; q < FR_MAXB / 256; ++q) {
      const int x = tid + 256 * q;
      su[q] = x < B ? a.u[x] : 0;
      si[q] = x < B ? a.i[x] : 0;
    }
#pragma unroll
    for (int q = 0; q < FR_MAXB / 256; ++q) {
      const int x = tid + 256 * q;
      if (x < B) {
        s_idx[x] = clamp_idx(su[q], a.U1);
        s_idx[B + x] = clamp_idx(si[q], a.I1);
      }
    }
  }
  __syncthreads();
  for (int64_t item = (int64_t)fb * 4 + wave; item < 2 * (int64_t)B; item += 4 * (int64_t)nrow)
    row_wait_finish_one<MODE, MG>(a, s_idx, (int)(item >> 1), (int)(item & 1));
}

// One workgroup per slot, looping over blocks of MR instances (blk = blockIdx.x,
// + gridDim.x, ...): the MLP forward (and, MODE 0 / 1, the backward) of a block on
// MFMA with every operand in LDS, the row contributions to global scratch, and the
// block's weight gradients accumulated into the workgroup's slot of a.wpart
// (outer products on MFMA; bias / head / loss sums per owning thread).  MODE 2 is
// prediction only.  DC = compile-time d (0: a.d at run time).
// FR (rows in line, B <= FR_MAXB: one block per workgroup): no k_nmf_rows launch
// and no weight-gradient workgroups.  The block's weight-gradient tiles are taken
// from LDS by the workgroup itself; once the block's contributions are out
// (write-through) each (instance, side) counts its arrival at its row.  Workgroups
// past inst_blocks are the row waves (row_wait_finish, a wave per (instance,
// side) as in k_nmf_rows): the owner of a row waits for all its arrivals and sums
// the row.  Same sums in the same order: bit-identical to the k_nmf_rows path
// (test_neumf_rows_in_line_matches_rows_kernel).
// (instance workgroup bx of the pass; MG: the clean and adversarial passes share
// one launch, k_nmf_step)
template <int MODE, int DC, bool FR, bool MG>
__device__ __forceinline__ void inst_block(const NArgs& a, unsigned bx, unsigned inst_blocks, float* sm) {
  __shared__ int32_t s_own[MG && MODE == 1 ? 2 * MR : 1];  // the block's pairs' owners (first occurrences)
  NSTAMP(0);
  const int d = DC ? DC : a.d, d2 = 2 * d, tid = threadIdx.x;
  const int L2 = d2 + 1, L1 = d + 1;  // padded leading dimensions
  const int64_t nblk = ((int64_t)a.B + MR - 1) / MR;
  float* s_x = sm;                 // [MR][L2]  h0 = MLP_U[u] | MLP_I[i]
  float* s_a1 = s_x + MR * L2;     // [MR][L2]
  float* s_f = s_a1 + MR * L2;     // [MR][L2]  MF_U*MF_I | a2; later dz1
  float* s_mu = s_f + MR * L2;     // [MR][L1]
  float* s_mi = s_mu + MR * L1;    // [MR][L1]
  float* s_dz2 = s_mi + MR * L1;   // [MR][L1]
  float* s_dl = s_dz2 + MR * L1;   // [MR] d loss / d logit
  float* s_ls = s_dl + MR;         // [MR] per-instance loss
  float* s_vec = s_ls + MR;        // b1 [2d] | b2 [d] | Wo [2d] | bo (+3)
  float* s_b1 = s_vec, *s_b2 = s_vec + d2, *s_wo = s_b2 + d, *s_bo = s_wo + d2;
  float* s_w1 = s_bo + 4;          // [2d][2d+1] (weights_in_lds)
  float* s_w2 = s_w1 + d2 * L2;    // [2d][d+1]
  const bool wl = weights_in_lds(d);
  // Prologue, in issue order: the first block's indices (and owners), its row
  // gathers, the weights, biases and head (once per workgroup), and only then the
  // LDS stores -- the weights stream in behind the row gathers.
  // Row gathers of a block: one round trip for the indices (and owners), one for
  // every row element; no branch on the data (a bad index is clamped to row 0 and
  // flagged once at the end).
  constexpr int QG = MR * 128 / 256;  // gather elements per thread (d <= 128)
  // element x = tid + 256 q of the block's MR x d; with a compile-time d that is a
  // multiple of 16 the live q are known and the gathers need no branch
  auto live = [&](int q) { return (MR * d) % 256 == 0 ? q < MR * d / 256 : tid + 256 * q < MR * d; };
  float g[QG][4];
  int bad = 0;
  int32_t uu[QG], ii[QG], ou[QG], oi[QG];
  auto gather_idx = [&](int64_t blk) {
    const int64_t b0 = blk * MR;
    const int nt = (int)min((int64_t)MR, (int64_t)a.B - b0);
#pragma unroll
    for (int q = 0; q < QG; ++q) {
      const int x = tid + 256 * q, t = x / d;
      const int64_t b = b0 + ((x < MR * d && t < nt) ? t : 0);
      uu[q] = a.u[b];
      ii[q] = a.i[b];
      if (MODE == 1 && MG) {
        ou[q] = s_own[2 * (b - b0)];
        oi[q] = s_own[2 * (b - b0) + 1];
      } else if (MODE == 1) {
        ou[q] = a.owner[2 * b];
        oi[q] = a.owner[2 * b + 1];
      }
    }
  };
  auto gather_rows = [&](int64_t blk) {
    const int64_t b0 = blk * MR;
    const int nt = (int)min((int64_t)MR, (int64_t)a.B - b0);
#pragma unroll
    for (int q = 0; q < QG; ++q) {
      const int x = tid + 256 * q;
      if (live(q)) {
        const int t = x / d, k = x - t * d;
        const bool ok = t < nt;
        const bool ub = uu[q] < 0 || uu[q] >= a.U1, ib = ii[q] < 0 || ii[q] >= a.I1;
        bad |= (ok && ub ? 1 : 0) | (ok && ib ? 2 : 0);
        const int64_t ru = (int64_t)(ub ? 0 : uu[q]) * d + k, ri = (int64_t)(ib ? 0 : ii[q]) * d + k;
        float v0 = a.P[a.off[S_MF_U] + ru], v1_ = a.P[a.off[S_MF_I] + ri];
        float v2_ = a.P[a.off[S_MLP_U] + ru], v3 = a.P[a.off[S_MLP_I] + ri];
        if (MODE == 1) {
          const float* du = a.delta + (int64_t)ou[q] * 4 * d;
          const float* di = a.delta + (int64_t)oi[q] * 4 * d;
          if (MG) {  // stored in this launch (write-through)
            v0 = v0 + ld_dev(du + 0 * d + k);
            v1_ = v1_ + ld_dev(di + 1 * d + k);
            v2_ = v2_ + ld_dev(du + 2 * d + k);
            v3 = v3 + ld_dev(di + 3 * d + k);
          } else {
            v0 = v0 + du[0 * d + k];
            v1_ = v1_ + di[1 * d + k];
            v2_ = v2_ + du[2 * d + k];
            v3 = v3 + di[3 * d + k];
          }
        }
        g[q][0] = ok ? v0 : 0.f;
        g[q][1] = ok ? v1_ : 0.f;
        g[q][2] = ok ? v2_ : 0.f;
        g[q][3] = ok ? v3 : 0.f;
      }
    }
  };
  int64_t blk = bx;
  // FR: the row of the block's pair tid (instance tid >> 1; user, item), for its arrival
  int32_t prow = 0;
  if constexpr (FR) {
    const int64_t b = blk * MR + (tid >> 1);
    if (tid < 2 * MR && b < a.B) prow = (tid & 1) ? clamp_idx(a.i[b], a.I1) : clamp_idx(a.u[b], a.U1);
  }
  if (!(MG && MODE == 1) && blk < nblk) {
    gather_idx(blk);
    gather_rows(blk);
  }
  constexpr int Q1 = 64 * 64 * 4 / 4 / 256, Q2 = 64 * 64 * 2 / 4 / 256;  // weights_in_lds: d <= 64
  const int n1 = wl ? d2 * d2 / 4 : 0, n2 = wl ? d2 * d / 4 : 0;
  float4 v1[Q1], v2[Q2];
  {
    const float4* g1 = reinterpret_cast<const float4*>(a.P + a.off[S_W1]);
    const float4* g2 = reinterpret_cast<const float4*>(a.P + a.off[S_W2]);
#pragma unroll
    for (int q = 0; q < Q1; ++q) if (tid + 256 * q < n1) v1[q] = g1[tid + 256 * q];
#pragma unroll
    for (int q = 0; q < Q2; ++q) if (tid + 256 * q < n2) v2[q] = g2[tid + 256 * q];
  }
  const int nvec = 5 * d + 1;  // b1, b2, Wo, bo
  constexpr int QV = (5 * 128 + 1 + 255) / 256;  // d <= 128
  float vv[QV];
#pragma unroll
  for (int q = 0; q < QV; ++q) {
    const int x = tid + 256 * q;
    vv[q] = 0.f;
    if (x < nvec) {
      const int64_t src = x < d2 ? a.off[S_B1] + x
                                 : x < 3 * d ? a.off[S_B2] + (x - d2)
                                             : x < 5 * d ? a.off[S_WO] + (x - 3 * d) : a.off[S_BO];
      vv[q] = a.P[src];
    }
  }
#pragma unroll
  for (int q = 0; q < QV; ++q)
    if (tid + 256 * q < nvec) s_vec[tid + 256 * q] = vv[q];
#pragma unroll
  for (int q = 0; q < Q1; ++q) {
    const int x = tid + 256 * q;
    if (x < n1) {
      const int e = 4 * x, rr = e / d2, cc = e - rr * d2;
      float* dst = s_w1 + rr * L2 + cc;
      dst[0] = v1[q].x; dst[1] = v1[q].y; dst[2] = v1[q].z; dst[3] = v1[q].w;
    }
  }
#pragma unroll
  for (int q = 0; q < Q2; ++q) {
    const int x = tid + 256 * q;
    if (x < n2) {
      const int e = 4 * x, rr = e / d, cc = e - rr * d;
      float* dst = s_w2 + rr * L1 + cc;
      dst[0] = v2[q].x; dst[1] = v2[q].y; dst[2] = v2[q].z; dst[3] = v2[q].w;
    }
  }
  if constexpr (MG && MODE == 1) {
    // the adversarial pass beside the clean one: the block's rows wait for their
    // clean owners (delta and gradient stored, owner index in the flag), then gather
    if (tid < 2 * MR) {
      const int64_t b = blk * MR + (tid >> 1);
      int32_t own = 0;
      if (b < a.B) {
        unsigned long long* fl = a.rdone + ((tid & 1) ? a.U1 : 0) + prow;
        unsigned long long v = 0;
        for (int it = 0;; ++it) {
          v = __hip_atomic_load(fl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((int32_t)(v >> 32) == a.gen) break;
          if (it >= a.spin) {
            atomicOr(a.err, 512);
            break;
          }
          __builtin_amdgcn_s_sleep(4);
        }
        own = (int32_t)(v & 0xFFFFFFFFull);
      }
      s_own[tid] = own;
    }
    __syncthreads();
    if (blk < nblk) {
      gather_idx(blk);
      gather_rows(blk);
    }
  }
  NSTAMP(1);
  const float* W1 = wl ? s_w1 : a.P + a.off[S_W1];
  const float* W2 = wl ? s_w2 : a.P + a.off[S_W2];
  const int ld1 = wl ? L2 : d2, ld2 = wl ? L1 : d;
  const float* Wo = s_wo;
  const float* b1 = s_b1;
  const float* b2 = s_b2;
  const WOut wo_ = wout(d);
  float* slot = MODE == 2 ? nullptr : a.wpart + (int64_t)bx * wo_.n;
  // vector partials owned by threads across the workgroup's blocks
  float acc_wo = 0.f, acc_b1 = 0.f, acc_b2 = 0.f, acc_bo = 0.f, acc_ls = 0.f;
  for (; blk < nblk; blk += inst_blocks) {
    const int64_t b0 = blk * MR;
    const int nt = (int)min((int64_t)MR, (int64_t)a.B - b0);
#pragma unroll
    for (int q = 0; q < QG; ++q) {
      const int x = tid + 256 * q;
      if (live(q)) {
        const int t = x / d, k = x - t * d;
        const float mu = g[q][0], mi = g[q][1], lu = g[q][2], li = g[q][3];
        s_mu[t * L1 + k] = mu;
        s_mi[t * L1 + k] = mi;
        s_x[t * L2 + k] = lu;
        s_x[t * L2 + d + k] = li;
        s_f[t * L2 + k] = mu * mi;  // GMF tower
      }
    }
    __syncthreads();
    // the next block's rows fly while this one computes
    if (blk + inst_blocks < nblk) {
      gather_idx(blk + inst_blocks);
      gather_rows(blk + inst_blocks);
    }
    NSTAMP(2);
    // layer 1: a1 = relu(h0 W1 + b1)
    mfma_panel<false>(s_x, L2, W1, ld1, d2, d2, [&](int row, int col, float v) {
      const float z = v + b1[col];
      s_a1[row * L2 + col] = z > 0.f ? z : 0.f;
    });
    __syncthreads();
    NSTAMP(3);
    // layer 2: a2 = relu(a1 W2 + b2) -> f[d:2d]
    mfma_panel<false>(s_a1, L2, W2, ld2, d2, d, [&](int row, int col, float v) {
      const float z = v + b2[col];
      s_f[row * L2 + d + col] = z > 0.f ? z : 0.f;
    });
    __syncthreads();
    NSTAMP(4);
    // head: 16 lanes per instance, p = sigmoid(f Wo + bo); Keras BCE on clip(p)
    {
      const int row = tid >> 4, part = tid & 15;
      float sacc = 0.f;
      for (int k = part; k < d2; k += 16) sacc = sacc + s_f[row * L2 + k] * Wo[k];
#pragma unroll
      for (int m = 1; m < 16; m <<= 1) sacc += __shfl_xor(sacc, m, 64);
      if (part == 0) {
        const float logit = sacc + s_bo[0];
        const float p = 1.0f / (1.0f + expf(-logit));
        if (MODE == 2) {
          if (row < nt) a.pred[b0 + row] = p;
        } else {
          const float y = row < nt ? a.y[b0 + row] : 0.f;
          const bool inside = p >= 1e-7f && p <= 1.0f - 1e-7f;  // clip_by_value's gradient
          const float pc = fminf(fmaxf(p, 1e-7f), 1.0f - 1e-7f);
          s_dl[row] = (row < nt && inside) ? (p - y) * a.scale_over_B : 0.f;
          s_ls[row] = row < nt ? -(y * logf(pc) + (1.0f - y) * logf(1.0f - pc)) : 0.f;
        }
      }
    }
    __syncthreads();
    if (MODE == 2) continue;
    NSTAMP(5);
    // dz2 = (dl * Wo[d:2d]) * (a2 > 0); GMF row contributions dmf * MF_I / dmf * MF_U;
    // the head's weight gradients (f^T dl, sum dl) and the loss sum
    for (int x = tid; x < MR * d; x += 256) {
      const int t = x / d, k = x - t * d;
      const float dl = s_dl[t];
      const float dz = s_f[t * L2 + d + k] > 0.f ? dl * Wo[d + k] : 0.f;
      s_dz2[t * L1 + k] = dz;
      if (t < nt) {
        const float dmf = dl * Wo[k];
        float* cu = a.contrib + ((b0 + t) * 4 + S_MF_U) * d + k;
        float* ci = a.contrib + ((b0 + t) * 4 + S_MF_I) * d + k;
        if constexpr (FR) {
          st_wt(cu, dmf * s_mi[t * L1 + k]);
          st_wt(ci, dmf * s_mu[t * L1 + k]);
        } else {
          *cu = dmf * s_mi[t * L1 + k];
          *ci = dmf * s_mu[t * L1 + k];
        }
      }
    }
    if (tid < d2)
      for (int t = 0; t < nt; ++t) acc_wo = acc_wo + s_f[t * L2 + tid] * s_dl[t];
    if (tid == 0)
      for (int t = 0; t < nt; ++t) {
        acc_bo = acc_bo + s_dl[t];
        acc_ls = acc_ls + s_ls[t];
      }
    __syncthreads();
    NSTAMP(6);
    // dz1 = (dz2 W2^T) * (a1 > 0) -> s_f (f is spent)
    mfma_panel<true>(s_dz2, L1, W2, ld2, d, d2, [&](int row, int col, float v) {
      s_f[row * L2 + col] = s_a1[row * L2 + col] > 0.f ? v : 0.f;
    });
    __syncthreads();
    NSTAMP(7);
    // dh0 = dz1 W1^T -> MLP_U / MLP_I row contributions
    mfma_panel<true>(s_f, L2, W1, ld1, d2, d2, [&](int row, int col, float v) {
      if (row < nt) {
        const int tab = col < d ? S_MLP_U : S_MLP_I, kk = col < d ? col : col - d;
        float* cp = a.contrib + ((b0 + row) * 4 + tab) * d + kk;
        if constexpr (FR) st_wt(cp, v);
        else *cp = v;
      }
    });
    NSTAMP(8);
    if constexpr (FR) {
      if (tid < d2)
        for (int t = 0; t < nt; ++t) acc_b1 = acc_b1 + s_f[t * L2 + tid];
      if (tid < d)
        for (int t = 0; t < nt; ++t) acc_b2 = acc_b2 + s_dz2[t * L1 + tid];
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's contributions are out
      __syncthreads();
      if (tid < 2 * nt)  // arrival at the row (its owner's row wave waits for all of them)
        __hip_atomic_fetch_add(a.rcnt + ((tid & 1) ? a.U1 : 0) + prow, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (nt < MR) {  // a partial block: rows past the batch zero, as wgrad_group stages them
        for (int x = tid; x < (MR - nt) * L2; x += 256) {
          s_a1[nt * L2 + x] = 0.f;
          s_f[nt * L2 + x] = 0.f;
        }
        for (int x = tid; x < (MR - nt) * L1; x += 256) s_dz2[nt * L1 + x] = 0.f;
        __syncthreads();
      }
      // the block's weight gradients into the slot (wgrad_group's tiles, from LDS)
      if (d % 16 == 0) outer_tiles<false, true>(s_x, s_f, s_a1, s_dz2, d, slot + wo_.w1, slot + wo_.w2, 0, wtiles(d));
      else outer_tiles<false, false>(s_x, s_f, s_a1, s_dz2, d, slot + wo_.w1, slot + wo_.w2, 0, wtiles(d));
      continue;
    }
    // the weight gradients' operands -> k_nmf_rows' gradient workgroups (W1 += h0^T dz1,
    // W2 += a1^T dz2 on MFMA there, beside the row sums); b1 += sum dz1, b2 += sum dz2 here
    for (int x = tid; x < MR * d2; x += 256) {
      const int t = x / d2, k = x - t * d2;
      if (t < nt) {
        const int64_t g = (b0 + t) * d2 + k;
        a.h0[g] = s_x[t * L2 + k];
        a.a1[g] = s_a1[t * L2 + k];
        a.dz1[g] = s_f[t * L2 + k];
      }
    }
    for (int x = tid; x < MR * d; x += 256) {
      const int t = x / d, k = x - t * d;
      if (t < nt) a.dz2[(b0 + t) * d + k] = s_dz2[t * L1 + k];
    }
    if (tid < d2)
      for (int t = 0; t < nt; ++t) acc_b1 = acc_b1 + s_f[t * L2 + tid];
    if (tid < d)
      for (int t = 0; t < nt; ++t) acc_b2 = acc_b2 + s_dz2[t * L1 + tid];
    NSTAMP(9);
    __syncthreads();
    NSTAMP(10);
  }
  if (MODE != 2) {
    if (tid < d2) {
      slot[wo_.wo + tid] = acc_wo;
      slot[wo_.b1 + tid] = acc_b1;
    }
    if (tid < d) slot[wo_.b2 + tid] = acc_b2;
    if (tid == 0) {
      slot[wo_.bo] = acc_bo;
      slot[wo_.loss] = acc_ls;
    }
  }
  if (bad) atomicOr(a.err, bad);
}

template <int MODE, int DC, bool FR = false>
__global__ void __launch_bounds__(256) k_nmf_inst(NArgs a, NArgs wg, unsigned inst_blocks) {
  extern __shared__ float sm[];
  if (FR && blockIdx.x >= inst_blocks) {  // the pass's row waves
    row_wait_finish<MODE, false>(a, blockIdx.x - inst_blocks, gridDim.x - inst_blocks, reinterpret_cast<int32_t*>(sm));
    return;
  }
  if (blockIdx.x >= inst_blocks) {  // the previous pass's weight-gradient workgroups
    const int x = (int)(blockIdx.x - inst_blocks), ns = (int)inst_blocks;
    if (wg.d % 16 == 0) wgrad_group<true>(wg, x % ns, x / ns, ns, sm);
    else wgrad_group<false>(wg, x % ns, x / ns, ns, sm);
    return;
  }
  inst_block<MODE, DC, FR, false>(a, blockIdx.x, inst_blocks, sm);
}

// Both passes of an adversarial rows-in-line step in ONE launch, in dispatch
// order: the clean instance workgroups (a), the clean row waves, the adversarial
// instance workgroups (b: each waits for its rows' clean owners, rdone), the
// adversarial row waves.  Every wait is on workgroups earlier in the grid, and
// the first ones never wait.  Bit-identical to the two launches.  (r05: the
// adversarial instance workgroups second, staging their weights at once and
// then waiting, measured 3-5% slower: they hold CUs the clean row waves need.)
template <int DC>
__global__ void __launch_bounds__(256) k_nmf_step(NArgs a, NArgs b, unsigned gi, unsigned gr) {
  extern __shared__ float sm[];
  unsigned x = blockIdx.x;
  if (x < gi) return inst_block<0, DC, true, true>(a, x, gi, sm);
  x -= gi;
  if (x < gr) return row_wait_finish<0, true>(a, x, gr, reinterpret_cast<int32_t*>(sm));
  x -= gr;
  if (x < gi) return inst_block<1, DC, true, true>(b, x, gi, sm);
  x -= gi;
  row_wait_finish<1, true>(b, x, gr, reinterpret_cast<int32_t*>(sm));
}

// Weight gradients of the step: slot element x summed over the passes' slots
// (deterministic, no atomics): groups of SB consecutive slots summed in slot
// order, then the group sums in group order; G += clean sum, then += adversarial
// sum; the loss element gives the passes' mean losses.  acf_neumf_train does the
// same sums with a lane per group (k_nmf_adam_next), so train == grad + adam bit
// for bit.
constexpr int SB = 8;

__device__ __forceinline__ float slot_sum(const float* part, int p, int nslot, int64_t nout, int64_t x) {
  float acc = 0.f;
  const float* q = part + (int64_t)p * nslot * nout + x;
  for (int s0 = 0; s0 < nslot; s0 += SB) {
    float v[SB];
#pragma unroll
    for (int j = 0; j < SB; ++j) v[j] = s0 + j < nslot ? q[(int64_t)(s0 + j) * nout] : 0.f;
    float gs = 0.f;
#pragma unroll
    for (int j = 0; j < SB; ++j)
      if (s0 + j < nslot) gs = gs + v[j];
    acc = acc + gs;
  }
  return acc;
}

// group gi's sum of four consecutive elements (x a multiple of 4, nout a multiple of 4)
__device__ __forceinline__ float4 slot_group4(const float* part, int p, int nslot, int64_t nout, int64_t x, int gi) {
  const float4* q = reinterpret_cast<const float4*>(part + (int64_t)p * nslot * nout + x);
  const int64_t st = nout / 4;
  const int s0 = gi * SB;
  float4 v[SB];
#pragma unroll
  for (int j = 0; j < SB; ++j) v[j] = s0 + j < nslot ? q[(s0 + j) * st] : make_float4(0.f, 0.f, 0.f, 0.f);
  float4 gs = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int j = 0; j < SB; ++j)
    if (s0 + j < nslot) {
      gs.x = gs.x + v[j].x;
      gs.y = gs.y + v[j].y;
      gs.z = gs.z + v[j].z;
      gs.w = gs.w + v[j].w;
    }
  return gs;
}

__device__ __forceinline__ float4 slot_sum4(const float* part, int p, int nslot, int64_t nout, int64_t x) {
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int gi = 0; gi * SB < nslot; ++gi) {
    const float4 gs = slot_group4(part, p, nslot, nout, x, gi);
    acc.x = acc.x + gs.x;
    acc.y = acc.y + gs.y;
    acc.z = acc.z + gs.z;
    acc.w = acc.w + gs.w;
  }
  return acc;
}

__device__ __forceinline__ void wsum_one(const NArgs& a, int64_t x, int nslot, int npass, const float* part,
                                         float* loss_out) {
  const WOut o = wout(a.d);
  if (x > o.loss) return;
  const float acc0 = slot_sum(part, 0, nslot, o.n, x);
  const float acc1 = npass > 1 ? slot_sum(part, 1, nslot, o.n, x) : 0.f;
  if (x == o.loss) {
    if (loss_out) {
      loss_out[0] = acc0 / (float)a.B;
      loss_out[1] = npass > 1 ? acc1 / (float)a.B : 0.f;
    }
    return;
  }
  float* dst = a.G + a.off[S_W1] + x;
  float v = *dst + acc0;
  if (npass > 1) v = v + acc1;
  *dst = v;
}

// acf_neumf_grad: the passes' slots summed into G (acf_neumf_train does it on the Adam stream)
__global__ void __launch_bounds__(256) k_nmf_wsum(NArgs a, int nslot, int npass, const float* __restrict__ part,
                                                  float* loss_out) {
  wsum_one(a, blockIdx.x * (int64_t)blockDim.x + threadIdx.x, nslot, npass, part, loss_out);
}

constexpr int RCH = 2048;  // batch indices staged in LDS per round

// One wave per (instance b, side s): s = 0 the user's MF_U / MLP_U rows, s = 1
// the item's MF_I / MLP_I rows.  The first occurrence of the row in the batch
// owns it: sums all its occurrences' contributions in instance order, adds the
// sum to the gradient rows and (with_delta) writes delta = eps*g/|g| per table.
// The workgroup stages the batch's indices in LDS (rounds of RCH); an owner's
// occurrences are loaded RBATCH at a time and added in order.  Workgroups past
// the rows' (blockIdx.x >= rows_blocks) are the pass's weight-gradient
// workgroups (wgrad_group; nslot slots x tile groups): latency-bound row sums
// leave the CUs free for their MFMA tiles.
__global__ void __launch_bounds__(256) k_nmf_rows(NArgs a, int32_t* __restrict__ owner,
                                                  float* __restrict__ delta, int with_delta, float eps,
                                                  unsigned rows_blocks, int nslot) {
  extern __shared__ float sm_w[];
  if (blockIdx.x >= rows_blocks) {
    const int x = (int)(blockIdx.x - rows_blocks);
    if (a.d % 16 == 0) wgrad_group<true>(a, x % nslot, x / nslot, nslot, sm_w);
    else wgrad_group<false>(a, x % nslot, x / nslot, nslot, sm_w);
    return;
  }
  __shared__ int32_t s_idx[2][RCH];
  RSTAMP(0);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int B = a.B, d = a.d;
  const int64_t item = (int64_t)blockIdx.x * 4 + wave;
  const bool live = item < 2 * (int64_t)B;
  const int b = live ? (int)(item >> 1) : 0, s = (int)(item & 1);
  const int64_t nrows = s ? a.I1 : a.U1;
  const int32_t r = clamp_idx((s ? a.i : a.u)[b], nrows);
  const int tA = s ? S_MF_I : S_MF_U, tB = s ? S_MLP_I : S_MLP_U;
  int first = -1;
  float gA[MAX_Q], gB[MAX_Q], oA[MAX_Q], oB[MAX_Q];
  // the row's gradient, fetched now (used if this wave owns the row)
#pragma unroll
  for (int q = 0; q < MAX_Q; ++q) {
    const int k = lane + 64 * q;
    gA[q] = gB[q] = 0.f;
    oA[q] = live && k < d ? a.G[a.off[tA] + (int64_t)r * d + k] : 0.f;
    oB[q] = live && k < d ? a.G[a.off[tB] + (int64_t)r * d + k] : 0.f;
  }
  for (int c0 = 0; c0 < B; c0 += RCH) {
    const int n = min(RCH, B - c0);
    if (c0 > 0) __syncthreads();
    int32_t su[RCH / 256], si[RCH / 256];
#pragma unroll
    for (int q = 0; q < RCH / 256; ++q) {
      const int x = threadIdx.x + 256 * q;
      su[q] = x < n ? a.u[c0 + x] : 0;
      si[q] = x < n ? a.i[c0 + x] : 0;
    }
#pragma unroll
    for (int q = 0; q < RCH / 256; ++q) {
      const int x = threadIdx.x + 256 * q;
      if (x < n) {
        s_idx[0][x] = clamp_idx(su[q], a.U1);
        s_idx[1][x] = clamp_idx(si[q], a.I1);
      }
    }
    __syncthreads();
    RSTAMP(1);
    if (!live) continue;
    const int32_t* L = s_idx[s];
    if (first < 0) {  // the first occurrence (b itself at the latest)
      for (int base = 0; base < n && c0 + base <= b; base += 64) {
        const int j = base + lane;
        const uint64_t mask = __ballot(j < n && c0 + j <= b && L[j] == r);
        if (mask) {
          first = c0 + base + __ffsll((unsigned long long)mask) - 1;
          break;
        }
      }
    }
    RSTAMP(2);
    if (first != b) continue;
    for (int base = max(b - c0, 0) & ~63; base < n; base += 64) {
      const int j = base + lane;
      uint64_t mask = __ballot(j < n && c0 + j >= b && L[j] == r);
      while (mask) {
        int js[RBATCH];
#pragma unroll
        for (int e = 0; e < RBATCH; ++e) {
          js[e] = -1;
          if (mask) {
            js[e] = c0 + base + __ffsll((unsigned long long)mask) - 1;
            mask &= mask - 1;
          }
        }
        float va[RBATCH][MAX_Q], vb[RBATCH][MAX_Q];
#pragma unroll
        for (int e = 0; e < RBATCH; ++e)
#pragma unroll
          for (int q = 0; q < MAX_Q; ++q) {
            const int k = lane + 64 * q;
            const bool ok = js[e] >= 0 && k < d;
            va[e][q] = ok ? a.contrib[((int64_t)js[e] * 4 + tA) * d + k] : 0.f;
            vb[e][q] = ok ? a.contrib[((int64_t)js[e] * 4 + tB) * d + k] : 0.f;
          }
#pragma unroll
        for (int e = 0; e < RBATCH; ++e)
          if (js[e] >= 0)
#pragma unroll
            for (int q = 0; q < MAX_Q; ++q) {
              gA[q] = gA[q] + va[e][q];
              gB[q] = gB[q] + vb[e][q];
            }
      }
    }
  }
  RSTAMP(3);
  if (!live) return;
  if (lane == 0) owner[2 * b + s] = first;
  if (first != b) return;
  float ssA = 0.f, ssB = 0.f;
#pragma unroll
  for (int q = 0; q < MAX_Q; ++q) {
    const int k = lane + 64 * q;
    if (k < d) {
      a.G[a.off[tA] + (int64_t)r * d + k] = oA[q] + gA[q];
      a.G[a.off[tB] + (int64_t)r * d + k] = oB[q] + gB[q];
      ssA = ssA + gA[q] * gA[q];
      ssB = ssB + gB[q] * gB[q];
    }
  }
  RSTAMP(4);
  if (!with_delta) return;
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    ssA += __shfl_xor(ssA, m, 64);
    ssB += __shfl_xor(ssB, m, 64);
  }
  const float invA = 1.0f / sqrtf(fmaxf(ssA, 1e-12f)), invB = 1.0f / sqrtf(fmaxf(ssB, 1e-12f));
#pragma unroll
  for (int q = 0; q < MAX_Q; ++q) {
    const int k = lane + 64 * q;
    if (k < d) {
      delta[((int64_t)b * 4 + tA) * d + k] = gA[q] * invA * eps;
      delta[((int64_t)b * 4 + tB) * d + k] = gB[q] * invB * eps;
    }
  }
  RSTAMP(5);
}

// NeuMF's weight-gradient slots handed to k_nmf_adam (acf_neumf_train): the
// float4s from base4 on get the slot sums of k_nmf_inst (wsum_one's arithmetic)
// added to their gradient first; the loss element goes to loss_out.
struct AdamSlots {
  const float* part = nullptr;  // nullptr: plain Adam
  int nslot = 0, npass = 0;
  int64_t base4 = 0, nout = 0;  // first float4 of the slot range; slot length (floats)
  float* loss_out = nullptr;
  float B = 1.f;  // the batch, for the mean losses
};

// Keras 2.2 Adam (keras/optimizers.py Adam.get_updates) of float4 x:
// m = b1*m + (1-b1)*g; v = b2*v + (1-b2)*g^2; p -= lr_t*m / (sqrt(v) + eps); g = 0.
// With slots (ws.part) the float4s from base4 on first get the slot sums of
// k_nmf_inst added to their gradient (wsum_one's arithmetic); the loss element
// goes to loss_out.
struct AdamK {
  float b1, b2, lr_t, eps;
};

// the float4's operands, loaded together (a wave issues them before its slot
// sums or its row claim resolve)
struct Adam4V {
  float4 g, m, v, p;
};

__device__ __forceinline__ Adam4V adam4_load(const float4* p, const float4* g, const float4* m, const float4* v,
                                             int64_t x) {
  return Adam4V{g[x], m[x], v[x], p[x]};
}

// the slot sums s4[pass] of float4 x (x >= ws.base4) added to its gradient; the loss element
__device__ __forceinline__ void adam4_fold(float4& gg, int64_t x, const AdamSlots& ws, const float4* s4) {
  const int64_t e0 = 4 * (x - ws.base4);
  const int64_t loss_x = ws.nout - 3;
  const float sum[2][4] = {{s4[0].x, s4[0].y, s4[0].z, s4[0].w}, {s4[1].x, s4[1].y, s4[1].z, s4[1].w}};
  float* gc = &gg.x;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (e0 + c < loss_x) {
      float t = gc[c] + sum[0][c];
      if (ws.npass > 1) t = t + sum[1][c];
      gc[c] = t;
    } else if (e0 + c == loss_x && ws.loss_out) {
      ws.loss_out[0] = sum[0][c] / ws.B;
      ws.loss_out[1] = ws.npass > 1 ? sum[1][c] / ws.B : 0.f;
    }
  }
}

// one Adam iteration of the float4 with learning rate lr_t (every path's arithmetic)
__device__ __forceinline__ void adam_math(Adam4V& a, const AdamK& k, float lr_t) {
  const float c1 = 1.0f - k.b1, c2 = 1.0f - k.b2;
#define ACF_ADAM(c)                                          \
  a.m.c = k.b1 * a.m.c + c1 * a.g.c;                         \
  a.v.c = k.b2 * a.v.c + c2 * (a.g.c * a.g.c);               \
  a.p.c = a.p.c - (lr_t * a.m.c) / (sqrtf(a.v.c) + k.eps);
  ACF_ADAM(x) ACF_ADAM(y) ACF_ADAM(z) ACF_ADAM(w)
#undef ACF_ADAM
}

__device__ __forceinline__ void adam4_store(float4* p, float4* g, float4* m, float4* v, int64_t x, const AdamK& k,
                                            Adam4V a) {
  adam_math(a, k, k.lr_t);
  m[x] = a.m;
  v[x] = a.v;
  p[x] = a.p;
  g[x] = make_float4(0.f, 0.f, 0.f, 0.f);
}

__device__ __forceinline__ void adam4(float4* __restrict__ p, float4* __restrict__ g, float4* __restrict__ m,
                                      float4* __restrict__ v, int64_t x, const AdamK& k, const AdamSlots& ws) {
  Adam4V a = adam4_load(p, g, m, v, x);
  if (ws.part && x >= ws.base4) {
    const int64_t e0 = 4 * (x - ws.base4);
    float4 s4[2];
    s4[0] = slot_sum4(ws.part, 0, ws.nslot, ws.nout, e0);
    s4[1] = ws.npass > 1 ? slot_sum4(ws.part, 1, ws.nslot, ws.nout, e0) : make_float4(0.f, 0.f, 0.f, 0.f);
    adam4_fold(a.g, x, ws, s4);
  }
  adam4_store(p, g, m, v, x, k, a);
}

// dense, float4 stream; with slots the stream runs from the top down: the slot
// range (the buffer's tail) is summed in the first sweep, under the rest of it
__global__ void __launch_bounds__(256) k_nmf_adam(float4* __restrict__ p, float4* __restrict__ g,
                                                  float4* __restrict__ m, float4* __restrict__ v,
                                                  int64_t n4, float b1, float b2, float lr_t,
                                                  float eps, AdamSlots ws = AdamSlots()) {
  const AdamK k{b1, b2, lr_t, eps};
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x)
    adam4(p, g, m, v, ws.part ? n4 - 1 - i : i, k, ws);
}

// acf_neumf_train runs Keras's dense Adam lazily with the same per-element
// arithmetic, so train == grad + adam bit for bit.  Each row holds in G the
// gradient of at most one pending iteration pend[r] (the step that gathered it);
// at every other iteration its gradient is 0, and such an iteration (m = b1 m,
// v = b2 v, p -= lr_t m / (sqrt(v) + eps)) depends on (p, m, v) and lr_t only.
// So a row's iterations can run later, in order, all at once, as long as that
// happens before anything reads the row or adds to its G:
//  k_nmf_adam_next    (caller's stream, after step k's gradients: iteration t)
//                     the rows of batch k+1, which step k+1 gathers and adds
//                     gradients to: a wave per (instance, side) claims its user /
//                     item row (atomicExch of the row's last iteration: the first
//                     claimer runs it) and runs the row's iterations up to t in
//                     both of its tables (MF_x, MLP_x), the pending one with G;
//                     pend = t + 1.  And the parameter tail (MLP / head) with the
//                     slot sums and the losses, every iteration;
//  k_nmf_adam_catchup (side stream, beside step k+1's kernels) slice k % LAZY_S
//                     of the rows brought to iteration t, so no row is more than
//                     LAZY_S iterations behind; after the call's last step, every
//                     row (caller's stream).
// catch-up period (acf_neumf_ctx::lazy_s = LAZY_S):
// a row is at most lazy_s iterations behind; a step's slice is 1/lazy_s of the
// rows, so a longer period is a smaller slice beside each step (r04, yelp shape,
// d 64, B 512, one box: period 8 6.47M instances/s, 16 7.10-7.15M, 24 6.91M, 31 6.74M;
// r05, same-box A/B with the workgroups below: 16 x 192 7.24M, 24 x 128 6.96-7.06M,
// 31 x 192 6.84-6.86M, 31 x 96 6.75-6.88M -- the env knobs of those A/Bs are gone;
// r05 beside the one-launch step with 512 workgroups, same box: 8 9.33-9.40M,
// 16 9.12-9.19M, 24 8.84M; another box: 4 9.08-9.11M, 8 9.35-9.38M, 16 9.13-9.14M,
// profiles/r05/neumf_catchup_wg_ab.txt)
constexpr int LAZY_S = 8;
constexpr int LAZY_W = 32;  // lr_t window (> the catch-up period)
// workgroups of a step's catch-up slice, beside the step's kernels (r03, period
// 8: 32 WGs 3.9M instances/s (the slice outlasts the step), 64 5.6M, 96 7.55M,
// 128 7.3M, 192 7.45M, 256 7.35M; r04, period 16: 48 5.1M, 64 5.8-6.0M, 96 7.10M,
// 128 7.10-7.15M, 192 7.16-7.18M, 256 7.13M; r05 beside the one-launch step
// (k_nmf_step), same box: 96 6.83-6.84M, 128 7.49-7.67M, 192 8.35M, 384 8.82-8.85M;
// another box: 192 8.19-8.32M, 384 8.83-8.85M, 512 9.03-9.05M, 768 9.01-9.06M,
// profiles/r05/neumf_catchup_wg_ab.txt)
constexpr int64_t CATCHUP_WG = 512;
static_assert(LAZY_W > LAZY_S, "lr window");

struct AdamLazy {
  int64_t U1, I1, d4;
  int32_t* last_u;   // [U1] the last Adam iteration the user's rows have taken
  int32_t* last_i;   // [I1]
  int32_t* pend_u;   // [U1] the iteration whose gradient G holds for the user's rows (<= last: none)
  int32_t* pend_i;   // [I1]
  int32_t* err;      // bit 8: a row more than LAZY_W - 1 iterations behind (never, by construction)
  int32_t t;         // this step's Adam iteration
  float lr[LAZY_W];  // lr[x] = lr_t of iteration t - (LAZY_W - 1) + x

  // the row's float4 q (q < d4: MF table, else MLP table)
  __device__ int64_t at(int side, int64_t r, int64_t q) const {
    if (q < d4) return side ? U1 * d4 + r * d4 + q : r * d4 + q;                            // S_MF_U / S_MF_I
    return side ? (2 * U1 + I1) * d4 + r * d4 + (q - d4) : (U1 + I1) * d4 + r * d4 + (q - d4);  // S_MLP_x
  }
};

// iterations (from, t] of a float4 (from >= t - LAZY_W), a.g the gradient of
// iteration gp, 0 at the others; unrolled so that every lr[x] is a kernel-argument load
__device__ __forceinline__ void lazy_iters(Adam4V& a, const AdamK& k, const AdamLazy& z, int32_t from,
                                           int32_t gp) {
  const float4 g = a.g;
#pragma unroll
  for (int x = 0; x < LAZY_W; ++x) {
    const int32_t tau = z.t - (LAZY_W - 1) + x;
    if (tau > from) {
      a.g = tau == gp ? g : make_float4(0.f, 0.f, 0.f, 0.f);
      adam_math(a, k, z.lr[x]);
    }
  }
}

__global__ void __launch_bounds__(256) k_nmf_adam_next(float4* __restrict__ p, float4* __restrict__ g,
                                                       float4* __restrict__ m, float4* __restrict__ v,
                                                       int64_t n4, int64_t emb4, AdamK k, AdamSlots ws,
                                                       AdamLazy z, const int32_t* __restrict__ un,
                                                       const int32_t* __restrict__ in, int32_t Bn,
                                                       unsigned row_blocks) {
  if (blockIdx.x >= row_blocks) {
    // the parameter tail: a lane per (float4, pass, slot group), 64 / (2 gp) float4s
    // per wave (gp = slot groups rounded up to a power of two)
    const int64_t t4 = n4 - emb4;
    const int lane = threadIdx.x & 63;
    const int ng = (ws.nslot + SB - 1) / SB;  // <= 32 (nslot <= NSLOT)
    int gp = 1;
    while (gp < ng) gp <<= 1;
    const int fpw = 32 / gp;  // float4s per wave
    const int f = lane / (2 * gp), pass = (lane / gp) & 1, gi = lane & (gp - 1);
    const int lead = f * 2 * gp;  // the float4's pass-0 leader; pass 1's is lead + gp
    const int64_t w0 = ((blockIdx.x - row_blocks) * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nw = ((int64_t)(gridDim.x - row_blocks) * blockDim.x) >> 6;
    for (int64_t i0 = w0 * fpw; i0 < t4; i0 += nw * fpw) {
      const int64_t i = i0 + f;
      const int64_t x = emb4 + i;
      const bool live = i < t4;
      Adam4V a{};
      if (live && lane == lead) a = adam4_load(p, g, m, v, x);
      float4 gs = make_float4(0.f, 0.f, 0.f, 0.f);
      if (live && gi < ng && pass < ws.npass) gs = slot_group4(ws.part, pass, ws.nslot, ws.nout, 4 * i, gi);
      // the group sums in group order (slot_sum4's arithmetic), by the pass leaders
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int j = 0; j < ng; ++j) {
        const int src = (lane & ~(gp - 1)) + j;
        acc.x = acc.x + __shfl(gs.x, src, 64);
        acc.y = acc.y + __shfl(gs.y, src, 64);
        acc.z = acc.z + __shfl(gs.z, src, 64);
        acc.w = acc.w + __shfl(gs.w, src, 64);
      }
      float4 sums[2];
      sums[0] = acc;
      sums[1] = make_float4(__shfl(acc.x, lead + gp, 64), __shfl(acc.y, lead + gp, 64),
                            __shfl(acc.z, lead + gp, 64), __shfl(acc.w, lead + gp, 64));
      if (ws.npass < 2) sums[1] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (live && lane == lead) {
        adam4_fold(a.g, x, ws, sums);
        adam4_store(p, g, m, v, x, k, a);
      }
    }
    return;
  }
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= 2 * (int64_t)Bn) return;
  const int b = (int)(wave >> 1), side = (int)(wave & 1);
  const int64_t nrows = side ? z.I1 : z.U1;
  int32_t r = side ? in[b] : un[b];
  if (r < 0 || r >= nrows) r = 0;  // the step flags bad indices; row 0 stays a valid address
  int32_t* lst = (side ? z.last_i : z.last_u) + r;
  int32_t* pnd = (side ? z.pend_i : z.pend_u) + r;
  int32_t old = 0;
  if (lane == 0) old = atomicExch(lst, z.t);
  const int32_t gp = *pnd;
  // the row's float4s, loaded beside the claim: nothing else writes the row
  // before the claimer's stores
  const int64_t d4 = z.d4;
  for (int64_t q = lane; q < 2 * d4; q += 64) {
    const int64_t x = z.at(side, r, q);
    Adam4V a = adam4_load(p, g, m, v, x);
    const int32_t from = __shfl(old, 0, 64);
    if (from == z.t) return;  // another occurrence claimed the row
    if (z.t - from > LAZY_W) {
      if (lane == 0) atomicOr(z.err, 256);
      return;
    }
    lazy_iters(a, k, z, from, gp);
    m[x] = a.m;
    v[x] = a.v;
    p[x] = a.p;
    g[x] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (lane == 0) *pnd = z.t + 1;  // step k+1's gradient
}

// rows [lo, hi) of the (users, then items) row space brought to iteration t; a
// lane-group of 32 (2 d4 <= 32) or 64 lanes per row, CR rows per lane-group in
// flight (2: 103 VGPRs and no faster beside the step)
constexpr int CR = 1;

__global__ void __launch_bounds__(256) k_nmf_adam_catchup(float4* __restrict__ p, float4* __restrict__ g,
                                                          float4* __restrict__ m, float4* __restrict__ v,
                                                          AdamK k, AdamLazy z, int64_t lo, int64_t hi) {
  const int64_t d4 = z.d4;
  const int lpr = 2 * d4 <= 32 ? 32 : 64;
  const int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t groups = (int64_t)gridDim.x * blockDim.x / lpr;
  const int l = (int)(threadIdx.x & (lpr - 1));
  for (int64_t r0 = lo + gid / lpr; r0 < hi; r0 += CR * groups) {
    int32_t from[CR], gp[CR];
    int64_t rr[CR];
#pragma unroll
    for (int j = 0; j < CR; ++j) {
      rr[j] = r0 + j * groups;
      from[j] = z.t;
      gp[j] = 0;
      if (rr[j] < hi) {
        const int side = rr[j] >= z.U1 ? 1 : 0;
        const int64_t r = side ? rr[j] - z.U1 : rr[j];
        from[j] = (side ? z.last_i : z.last_u)[r];
        gp[j] = (side ? z.pend_i : z.pend_u)[r];
      }
    }
    for (int64_t q = l; q < 2 * d4; q += lpr) {
      Adam4V a[CR];
      int64_t x[CR];
#pragma unroll
      for (int j = 0; j < CR; ++j) {  // all loads first
        if (from[j] >= z.t || z.t - from[j] > LAZY_W) continue;  // claimed at t / (never) too far behind
        const int side = rr[j] >= z.U1 ? 1 : 0;
        x[j] = z.at(side, side ? rr[j] - z.U1 : rr[j], q);
        const bool wg = gp[j] > from[j] && gp[j] <= z.t;  // G holds a gradient of the range
        a[j] = Adam4V{wg ? g[x[j]] : make_float4(0.f, 0.f, 0.f, 0.f), m[x[j]], v[x[j]], p[x[j]]};
      }
#pragma unroll
      for (int j = 0; j < CR; ++j) {
        if (from[j] >= z.t || z.t - from[j] > LAZY_W) continue;
        lazy_iters(a[j], k, z, from[j], gp[j]);
        m[x[j]] = a[j].m;
        v[x[j]] = a[j].v;
        p[x[j]] = a[j].p;
        if (gp[j] > from[j] && gp[j] <= z.t) g[x[j]] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    if (l == 0) {
#pragma unroll
      for (int j = 0; j < CR; ++j) {
        if (from[j] >= z.t) continue;
        if (z.t - from[j] > LAZY_W) {
          atomicOr(z.err, 256);
          continue;
        }
        const int side = rr[j] >= z.U1 ? 1 : 0;
        (side ? z.last_i : z.last_u)[side ? rr[j] - z.U1 : rr[j]] = z.t;  // read again only after this launch
      }
    }
  }
}

__global__ void k_nmf_fill_i32(int32_t* __restrict__ a, int64_t n, int32_t val) {
  const int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (x < n) a[x] = val;
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
struct acf_neumf_ctx {
  int64_t U1 = 0, I1 = 0;
  int32_t d = 0, maxB = 0;
  Layout L;
  float *contrib = nullptr, *delta = nullptr;
  float *h0 = nullptr, *a1 = nullptr, *dz1 = nullptr, *dz2 = nullptr;  // weight-gradient operands
  float* wpart = nullptr;  // [2 passes][slots][weight-gradient outputs]
  int32_t nslot = 0;       // workgroups (slots) of a training pass at max_batch
  int32_t *owner = nullptr, *err = nullptr;
  int32_t* rcnt = nullptr;  // rows in line: arrivals per row [2][U1 + I1] (clean, adversarial)
  unsigned long long* rdone = nullptr;  // [U1 + I1] k_nmf_step's published rows
  int32_t gen = 0;                      // k_nmf_step launches so far
  int32_t rows_in_line = 1;  // B <= FR_MAXB: rows in line (acf_neumf_set_rows_in_line: 0 = k_nmf_rows)
  // acf_neumf_train's lazy Adam: each row's last iteration, the side stream and its events
  int32_t *last_u = nullptr, *last_i = nullptr, *pend_u = nullptr, *pend_i = nullptr;
  hipStream_t side = nullptr;
  hipEvent_t ev_next = nullptr, ev_rest = nullptr;
  int32_t lazy_s = LAZY_S;           // catch-up period (< LAZY_W)
  int64_t catchup_wg = CATCHUP_WG;   // workgroups of a catch-up slice
  // rows-in-line failure safety (acf_neumf_set_spin_limit / _set_failsafe): a give-up
  // (err bit 512) is replayed from a snapshot of the call's inputs on the row-sum path
  int32_t spin = ACF_SPIN_LIMIT;
  int32_t failsafe = 1;
  int64_t recoveries = 0;     // calls replayed
  bool unchecked_fr = false;  // an unchecked rows-in-line grad has not been verified yet
  float* snap = nullptr;      // [P | G | m | v] of the call being verified (allocated at first use)
  size_t snap_n = 0;          // floats in snap
  std::vector<void*> allocs;
};

extern "C" const char* acf_neumf_last_error(void) { return g_neumf_error.c_str(); }

#ifndef ACF_BUILD_HASH
#define ACF_BUILD_HASH "unhashed"
#endif
extern "C" const char* acf_neumf_build_hash(void) { return "ACF_BUILD_HASH=" ACF_BUILD_HASH; }

static int check_dims(int64_t U1, int64_t I1, int32_t d) {
  ACF_CHECK(U1 > 0 && I1 > 0 && U1 < (1ll << 31) && I1 < (1ll << 31), ACF_E_INVALID,
            "table rows must be in [1, 2^31): got %lld, %lld", (long long)U1, (long long)I1);
  ACF_CHECK(d >= 4 && d <= 64 * MAX_Q && d % 4 == 0, ACF_E_INVALID,
            "dim must be a multiple of 4 in [4, %d], got %d", 64 * MAX_Q, d);
  return ACF_OK;
}

extern "C" int64_t acf_neumf_param_count(int64_t U1, int64_t I1, int32_t d) {
  if (check_dims(U1, I1, d) != ACF_OK) return -1;
  return make_layout(U1, I1, d).total;
}

extern "C" int acf_neumf_param_offsets(int64_t U1, int64_t I1, int32_t d, int64_t* off) {
  int r = check_dims(U1, I1, d);
  if (r != ACF_OK) return r;
  ACF_CHECK(off != nullptr, ACF_E_INVALID, "offsets pointer is NULL");
  const Layout L = make_layout(U1, I1, d);
  for (int k = 0; k < S_COUNT; ++k) off[k] = L.off[k];
  return ACF_OK;
}

extern "C" int acf_neumf_set_rows_in_line(acf_neumf_ctx* c, int32_t on) {
  ACF_CHECK(c != nullptr, ACF_E_INVALID, "ctx is NULL");
  c->rows_in_line = on ? 1 : 0;
  return ACF_OK;
}

extern "C" int acf_neumf_set_spin_limit(acf_neumf_ctx* c, int32_t polls) {
  ACF_CHECK(c != nullptr, ACF_E_INVALID, "ctx is NULL");
  ACF_CHECK(polls >= 0, ACF_E_INVALID, "spin limit must be >= 0, got %d", polls);
  c->spin = polls;
  return ACF_OK;
}

extern "C" int acf_neumf_set_failsafe(acf_neumf_ctx* c, int32_t on) {
  ACF_CHECK(c != nullptr, ACF_E_INVALID, "ctx is NULL");
  c->failsafe = on ? 1 : 0;
  return ACF_OK;
}

extern "C" int acf_neumf_recoveries(acf_neumf_ctx* c, int64_t* out) {
  ACF_CHECK(c != nullptr && out != nullptr, ACF_E_INVALID, "NULL argument");
  *out = c->recoveries;
  return ACF_OK;
}

extern "C" int acf_neumf_destroy(acf_neumf_ctx* c) {
  if (!c) return ACF_OK;
  if (c->side) (void)hipStreamSynchronize(c->side);
  for (void* p : c->allocs) (void)hipFree(p);
  if (c->snap) (void)hipFree(c->snap);
  if (c->ev_next) (void)hipEventDestroy(c->ev_next);
  if (c->ev_rest) (void)hipEventDestroy(c->ev_rest);
  if (c->side) (void)hipStreamDestroy(c->side);
  delete c;
  return ACF_OK;
}

static int set_inst_smem_limit();

extern "C" int acf_neumf_create(acf_neumf_ctx** out, int64_t U1, int64_t I1, int32_t d,
                                int32_t maxB) {
  ACF_CHECK(out != nullptr, ACF_E_INVALID, "out is NULL");
  *out = nullptr;
  int r = check_dims(U1, I1, d);
  if (r != ACF_OK) return r;
  ACF_CHECK(maxB > 0 && maxB <= (1 << 24), ACF_E_INVALID, "max_batch must be in (0, 2^24], got %d", maxB);
  acf_neumf_ctx* c = new acf_neumf_ctx();
  c->U1 = U1; c->I1 = I1; c->d = d; c->maxB = maxB;
  c->L = make_layout(U1, I1, d);
  const size_t B = (size_t)maxB, dd = (size_t)d;
  auto A = [&](auto** p, size_t n) {
    if (r != ACF_OK) return;
    void* q = nullptr;
    if (hipMalloc(&q, n * sizeof(**p) + 16) != hipSuccess) {
      (void)hipGetLastError();
      r = set_error(ACF_E_NOMEM, "hipMalloc of %zu bytes failed", n * sizeof(**p));
      return;
    }
    c->allocs.push_back(q);
    *p = static_cast<std::remove_reference_t<decltype(*p)>>(q);
  };
  A(&c->contrib, B * 4 * dd); A(&c->delta, B * 4 * dd); A(&c->owner, 2 * B); A(&c->err, 4);
  A(&c->rcnt, 2 * (size_t)(U1 + I1)); A(&c->rdone, (size_t)(U1 + I1));
  // two sets (clean / adversarial pass): the clean pass's gradient workgroups read theirs
  // while the adversarial k_nmf_inst writes its own
  A(&c->h0, 2 * B * 2 * dd); A(&c->a1, 2 * B * 2 * dd); A(&c->dz1, 2 * B * 2 * dd); A(&c->dz2, 2 * B * dd);
  A(&c->last_u, (size_t)U1); A(&c->last_i, (size_t)I1); A(&c->pend_u, (size_t)U1); A(&c->pend_i, (size_t)I1);
  // (r05: the catch-up stream at the least stream priority measured the same, 7.17-7.19M
  // instances/s either way, profiles/r05/neumf_side_priority_ab.txt)
  if (r == ACF_OK && (hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess ||
                      hipEventCreateWithFlags(&c->ev_next, hipEventDisableTiming) != hipSuccess ||
                      hipEventCreateWithFlags(&c->ev_rest, hipEventDisableTiming) != hipSuccess))
    r = set_error(ACF_E_HIP, "lazy-Adam setup failed");
  c->nslot = (int32_t)std::min<int64_t>(((int64_t)maxB + MR - 1) / MR, NSLOT);
  A(&c->wpart, 2 * (size_t)c->nslot * (size_t)wout(d).n);
  if (r == ACF_OK && (hipMemset(c->err, 0, 16) != hipSuccess || hipMemset(c->rcnt, 0, 2 * (size_t)(U1 + I1) * sizeof(int32_t)) != hipSuccess ||
                      hipMemset(c->rdone, 0, (size_t)(U1 + I1) * sizeof(unsigned long long)) != hipSuccess ||
                      hipDeviceSynchronize() != hipSuccess))
    r = set_error(ACF_E_HIP, "hipMemset failed");
  if (r == ACF_OK) r = set_inst_smem_limit();
  if (r != ACF_OK) { acf_neumf_destroy(c); return r; }
  *out = c;
  return ACF_OK;
}

static NArgs make_args(acf_neumf_ctx* c, const float* P, float* G, const int32_t* u, const int32_t* i,
                       const float* y, int32_t B, float scale) {
  NArgs a;
  a.P = P; a.G = G;
  for (int k = 0; k < S_COUNT; ++k) a.off[k] = c->L.off[k];
  a.u = u; a.i = i; a.y = y;
  a.U1 = c->U1; a.I1 = c->I1; a.B = B; a.d = c->d;
  a.scale_over_B = (float)((double)scale / (double)B);
  a.contrib = c->contrib; a.wpart = c->wpart;
  a.h0 = c->h0; a.a1 = c->a1; a.dz1 = c->dz1; a.dz2 = c->dz2;
  a.delta = c->delta; a.owner = c->owner; a.pred = nullptr; a.err = c->err;
  a.rcnt = c->rcnt; a.with_delta = 0; a.eps = 0.f; a.rdone = c->rdone; a.gen = 0; a.spin = c->spin;
  return a;
}

// fr_b: the batch of a rows-in-line launch (its row waves stage its indices), 0 otherwise
static size_t inst_smem(int d, int fr_b = 0) {
  return (size_t)std::max<int64_t>(inst_floats(d), 2 * (int64_t)fr_b) * sizeof(float);
}

// allow the large dynamic LDS of k_nmf_inst (gfx950: 160 KB per CU)
static int set_inst_smem_limit() {
  static int done = 0;
  if (done) return ACF_OK;
  const int bytes = 150 * 1024;
  const void* fns[] = {reinterpret_cast<const void*>(&k_nmf_inst<0, 0>),
                       reinterpret_cast<const void*>(&k_nmf_inst<1, 0>),
                       reinterpret_cast<const void*>(&k_nmf_inst<2, 0>),
                       reinterpret_cast<const void*>(&k_nmf_inst<0, DFAST>),
                       reinterpret_cast<const void*>(&k_nmf_inst<1, DFAST>),
                       reinterpret_cast<const void*>(&k_nmf_inst<2, DFAST>),
                       reinterpret_cast<const void*>(&k_nmf_inst<0, 0, true>),
                       reinterpret_cast<const void*>(&k_nmf_inst<1, 0, true>),
                       reinterpret_cast<const void*>(&k_nmf_inst<0, DFAST, true>),
                       reinterpret_cast<const void*>(&k_nmf_inst<1, DFAST, true>),
                       reinterpret_cast<const void*>(&k_nmf_step<0>),
                       reinterpret_cast<const void*>(&k_nmf_step<DFAST>)};
  for (const void* f : fns) HIP_TRY(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  // k_nmf_rows: 16 KB of indices + the gradient workgroups' operands (d = 128: 58 KB)
  HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_nmf_rows),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)wgrad_smem(128)));
  done = 1;
  return ACF_OK;
}

static int fetch_err(acf_neumf_ctx* c, hipStream_t s, int32_t* herr) {
  *herr = 0;
  HIP_TRY(hipMemcpyAsync(herr, c->err, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  return ACF_OK;
}

static int check_err(int32_t herr) {
  ACF_CHECK(!(herr & 256), ACF_E_HIP, "lazy Adam: a row fell behind the learning-rate window (internal)");
  ACF_CHECK(!(herr & 512), ACF_E_HIP, "rows in line: a row wave timed out waiting for its arrivals "
            "(failsafe off: the call's results are undefined)");
  ACF_CHECK(herr == 0, ACF_E_RANGE, "index out of range (%s%s)", (herr & 1) ? "user >= num_user_rows " : "",
            (herr & 2) ? "item >= num_item_rows" : "");
  return ACF_OK;
}

static int read_err(acf_neumf_ctx* c, hipStream_t s) {
  int32_t herr = 0;
  int r = fetch_err(c, s, &herr);
  return r != ACF_OK ? r : check_err(herr);
}

// After a give-up: late arrivals may have landed after their owner re-armed its
// counter, so every arrival counter is zeroed (the stream is idle: fetch_err
// synchronised it) before anything else runs on this context.  rdone needs no
// reset: its entries carry the launch generation.
static int reset_row_counters(acf_neumf_ctx* c, hipStream_t s) {
  HIP_TRY(hipMemsetAsync(c->rcnt, 0, 2 * (size_t)(c->U1 + c->I1) * sizeof(int32_t), s));
  HIP_TRY(hipMemsetAsync(c->err, 0, sizeof(int32_t), s));
  HIP_TRY(hipStreamSynchronize(s));
  return ACF_OK;
}

// An unchecked acf_neumf_grad on the rows-in-line path is verified by the next
// call that reads the error word (grad with check, train, predict) before that
// call clears it: a give-up there cannot be replayed any more (the caller may have
// consumed the gradient), so it is reported, never dropped.
static int settle_unchecked(acf_neumf_ctx* c, hipStream_t s) {
  if (!c->unchecked_fr) return ACF_OK;
  int32_t herr = 0;
  int r = fetch_err(c, s, &herr);
  if (r != ACF_OK) return r;
  c->unchecked_fr = false;
  if (herr & 512) {
    r = reset_row_counters(c, s);
    if (r != ACF_OK) return r;
    return set_error(ACF_E_HIP, "rows in line: an earlier unchecked acf_neumf_grad call timed out waiting for "
                     "its arrivals; the gradient it added is undefined");
  }
  return ACF_OK;
}

// the failsafe's snapshot of the buffers a call writes (nbuf of P, G, m, v: each
// L.total floats), taken on the call's stream before its first launch
static int take_snapshot(acf_neumf_ctx* c, hipStream_t s, float* const* bufs, int nbuf) {
  const size_t n = (size_t)c->L.total;
  if (c->snap_n < 4 * n) {
    if (c->snap) HIP_TRY(hipFree(c->snap));
    c->snap = nullptr;
    c->snap_n = 0;
    if (hipMalloc(&c->snap, 4 * n * sizeof(float)) != hipSuccess) {
      (void)hipGetLastError();
      c->snap = nullptr;
      return set_error(ACF_E_NOMEM, "failsafe snapshot: hipMalloc of %zu bytes failed", 4 * n * sizeof(float));
    }
    c->snap_n = 4 * n;
  }
  for (int k = 0; k < nbuf; ++k)
    HIP_TRY(hipMemcpyAsync(c->snap + k * n, bufs[k], n * sizeof(float), hipMemcpyDeviceToDevice, s));
  return ACF_OK;
}

static int restore_snapshot(acf_neumf_ctx* c, hipStream_t s, float* const* bufs, int nbuf) {
  const size_t n = (size_t)c->L.total;
  for (int k = 0; k < nbuf; ++k)
    HIP_TRY(hipMemcpyAsync(bufs[k], c->snap + k * n, n * sizeof(float), hipMemcpyDeviceToDevice, s));
  return ACF_OK;
}

// grid = inst workgroups + (optional) the previous pass's weight-gradient workgroups (args wg)
template <int MODE, bool FR = false>
static void launch_inst(const NArgs& a, unsigned inst_blocks, hipStream_t s, const NArgs* wg = nullptr,
                        unsigned wg_blocks = 0) {
  const NArgs& w = wg ? *wg : a;
  // extra workgroups: the previous pass's weight-gradient workgroups (wg), or FR's row waves
  const unsigned grid = inst_blocks + ((wg || FR) ? wg_blocks : 0u);
  const size_t sm = inst_smem(a.d, FR ? a.B : 0);
  if (a.d == DFAST)
    k_nmf_inst<MODE, DFAST, FR><<<grid, 256, sm, s>>>(a, w, inst_blocks);
  else
    k_nmf_inst<MODE, 0, FR><<<grid, 256, sm, s>>>(a, w, inst_blocks);
}

// clean pass: k_nmf_inst<0> -> k_nmf_rows (owners, rows, delta; + the pass's
// weight-gradient tiles); adversarial pass: k_nmf_inst<1> -> k_nmf_rows; then
// k_nmf_wsum sums the passes' slots into G, unless the caller leaves that to
// k_nmf_adam (acf_neumf_train).  B <= FR_MAXB: one k_nmf_inst<.., true> per pass
// (rows and weight-gradient tiles in line).
static int launch_grad(acf_neumf_ctx* c, const float* P, float* G, const int32_t* u, const int32_t* i,
                       const float* y, int32_t B, const acf_neumf_hparams* hp, float* loss_out,
                       hipStream_t s, bool wsum = true) {
  const unsigned gi = (unsigned)std::min<int64_t>(((int64_t)B + MR - 1) / MR, NSLOT);
  const unsigned gr = (unsigned)((2 * (int64_t)B + 3) / 4);
  const unsigned gw = gi * (unsigned)((wtiles(c->d) + WG_TILES - 1) / WG_TILES);  // gradient workgroups
  const size_t sw = wgrad_smem(c->d);
  const WOut o = wout(c->d);
  const int npass = hp->adver ? 2 : 1;
  NArgs a = make_args(c, P, G, u, i, y, B, 1.0f);
  // both passes in one launch (r05 same-box A/B against one launch per pass:
  // 8.52-8.96M vs 8.38-8.40M instances/s, profiles/r05/neumf_rows_in_line_ab.txt)
  if (B <= FR_MAXB && c->rows_in_line && hp->adver) {
    a.with_delta = 1;
    a.eps = hp->eps;
    a.gen = ++c->gen;
    NArgs b = make_args(c, P, G, u, i, y, B, hp->reg_adv);
    b.wpart = c->wpart + (int64_t)gi * o.n;
    b.rcnt = c->rcnt + (c->U1 + c->I1);
    b.gen = a.gen;
    const size_t sm = inst_smem(c->d, B);
    if (c->d == DFAST) k_nmf_step<DFAST><<<2 * (gi + gr), 256, sm, s>>>(a, b, gi, gr);
    else k_nmf_step<0><<<2 * (gi + gr), 256, sm, s>>>(a, b, gi, gr);
    HIP_TRY(hipGetLastError());
  } else if (B <= FR_MAXB && c->rows_in_line) {
    a.with_delta = hp->adver ? 1 : 0;
    a.eps = hp->eps;
    // a row wave per (instance, side); half as many (two pairs per wave) or as many as
    // fit beside the instance workgroups measured 1-3% slower (same box,
    // profiles/r05/neumf_rows_in_line_ab.txt)
    launch_inst<0, true>(a, gi, s, nullptr, gr);
    HIP_TRY(hipGetLastError());
    if (hp->adver) {
      NArgs b = make_args(c, P, G, u, i, y, B, hp->reg_adv);
      b.wpart = c->wpart + (int64_t)gi * o.n;
      launch_inst<1, true>(b, gi, s, nullptr, gr);
      HIP_TRY(hipGetLastError());
    }
  } else {
    launch_inst<0>(a, gi, s);
    // APR-style: the clean pass's gradient workgroups ride in the adversarial
    // k_nmf_inst (32 workgroups at B = 512: the other CUs are idle); BPR-style
    // (no adversary) in its k_nmf_rows
    k_nmf_rows<<<gr + (hp->adver ? 0u : gw), 256, sw, s>>>(a, c->owner, c->delta, hp->adver ? 1 : 0, hp->eps, gr,
                                                          (int)gi);
    HIP_TRY(hipGetLastError());
    if (hp->adver) {
      NArgs b = make_args(c, P, G, u, i, y, B, hp->reg_adv);
      b.wpart = c->wpart + (int64_t)gi * o.n;
      const int64_t ab = (int64_t)c->maxB;  // the second activation buffer
      b.h0 += ab * 2 * c->d; b.a1 += ab * 2 * c->d; b.dz1 += ab * 2 * c->d; b.dz2 += ab * c->d;
      launch_inst<1>(b, gi, s, &a, gw);
      k_nmf_rows<<<gr + gw, 256, sw, s>>>(b, c->owner, c->delta, 0, 0.f, gr, (int)gi);
      HIP_TRY(hipGetLastError());
    }
  }
  if (wsum) {
    k_nmf_wsum<<<(unsigned)((o.n + 255) / 256), 256, 0, s>>>(a, (int)gi, npass, c->wpart, loss_out);
    HIP_TRY(hipGetLastError());
  }
  return ACF_OK;
}

extern "C" int acf_neumf_grad(acf_neumf_ctx* c, const float* P, float* G, const int32_t* u,
                              const int32_t* i, const float* y, int32_t B, const acf_neumf_hparams* hp,
                              float* loss_out, int32_t check, void* stream_) {
  ACF_CHECK(c && P && G && u && i && y && hp, ACF_E_INVALID, "NULL argument");
  ACF_CHECK(B > 0 && B <= c->maxB, ACF_E_INVALID, "batch %d outside (0, %d]", B, c->maxB);
  hipStream_t s = static_cast<hipStream_t>(stream_);
  const bool fr = B <= FR_MAXB && c->rows_in_line;
  if (!check) {  // verified by the next checking call (settle_unchecked)
    int r = launch_grad(c, P, G, u, i, y, B, hp, loss_out, s);
    if (r == ACF_OK && fr) c->unchecked_fr = true;
    return r;
  }
  int r = settle_unchecked(c, s);
  if (r != ACF_OK) return r;
  HIP_TRY(hipMemsetAsync(c->err, 0, sizeof(int32_t), s));
  float* bufs[1] = {G};
  const bool snap = fr && c->failsafe;
  if (snap && (r = take_snapshot(c, s, bufs, 1)) != ACF_OK) return r;
  if ((r = launch_grad(c, P, G, u, i, y, B, hp, loss_out, s)) != ACF_OK) return r;
  int32_t herr = 0;
  if ((r = fetch_err(c, s, &herr)) != ACF_OK) return r;
  if ((herr & 512) && fr) {
    if ((r = reset_row_counters(c, s)) != ACF_OK) return r;
    if (!snap) return check_err(herr);
    // the exact replay: G as the call found it, the row-sum path (same bits)
    if ((r = restore_snapshot(c, s, bufs, 1)) != ACF_OK) return r;
    c->rows_in_line = 0;
    r = launch_grad(c, P, G, u, i, y, B, hp, loss_out, s);
    c->rows_in_line = 1;
    if (r != ACF_OK) return r;
    ++c->recoveries;
    if ((r = fetch_err(c, s, &herr)) != ACF_OK) return r;
  }
  return check_err(herr);
}

// lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t), evaluated in float32 as Keras does
static float adam_lr_t(const acf_neumf_hparams* hp, int64_t t) {
  const float tt = (float)t;
  return hp->lr * (sqrtf(1.0f - powf(hp->beta2, tt)) / (1.0f - powf(hp->beta1, tt)));
}

static int launch_adam(acf_neumf_ctx* c, float* P, float* G, float* m, float* v, int64_t t,
                       const acf_neumf_hparams* hp, hipStream_t s, const AdamSlots& ws = AdamSlots()) {
  const float lr_t = adam_lr_t(hp, t);
  const int64_t n4 = c->L.total / 4;
  const unsigned grid = (unsigned)std::min<int64_t>((n4 + 255) / 256, 256 * 32);
  k_nmf_adam<<<grid, 256, 0, s>>>(reinterpret_cast<float4*>(P), reinterpret_cast<float4*>(G),
                                  reinterpret_cast<float4*>(m), reinterpret_cast<float4*>(v), n4,
                                  hp->beta1, hp->beta2, lr_t, hp->adam_eps, ws);
  HIP_TRY(hipGetLastError());
  return ACF_OK;
}

extern "C" int acf_neumf_adam(acf_neumf_ctx* c, float* P, float* G, float* m, float* v, int64_t t,
                              const acf_neumf_hparams* hp, void* stream_) {
  ACF_CHECK(c && P && G && m && v && hp, ACF_E_INVALID, "NULL argument");
  ACF_CHECK(t >= 1, ACF_E_INVALID, "Adam iteration must be >= 1, got %lld", (long long)t);
  return launch_adam(c, P, G, m, v, t, hp, static_cast<hipStream_t>(stream_));
}

static int train_launches(acf_neumf_ctx* c, float* P, float* G, float* m, float* v, const int32_t* u,
                          const int32_t* i, const float* y, int64_t n, int32_t batch, int64_t t_first,
                          const acf_neumf_hparams* hp, float* losses, hipStream_t s) {
  HIP_TRY(hipMemsetAsync(c->err, 0, sizeof(int32_t), s));
  float4 *P4 = reinterpret_cast<float4*>(P), *G4 = reinterpret_cast<float4*>(G);
  float4 *m4 = reinterpret_cast<float4*>(m), *v4 = reinterpret_cast<float4*>(v);
  const int64_t n4 = c->L.total / 4, emb4 = c->L.off[S_W1] / 4;
  const int64_t nsteps = (n + batch - 1) / batch;
  ACF_CHECK(t_first + nsteps < INT32_MAX, ACF_E_INVALID, "Adam iteration overflows int32");
  AdamLazy z;
  z.U1 = c->U1; z.I1 = c->I1; z.d4 = c->d / 4;
  z.last_u = c->last_u; z.last_i = c->last_i; z.pend_u = c->pend_u; z.pend_i = c->pend_i; z.err = c->err;
  // every row has taken iteration t_first - 1, and G holds its gradient of
  // iteration t_first (what the caller accumulated, plus step 0's)
  k_nmf_fill_i32<<<(unsigned)((c->U1 + 255) / 256), 256, 0, s>>>(c->last_u, c->U1, (int32_t)(t_first - 1));
  k_nmf_fill_i32<<<(unsigned)((c->I1 + 255) / 256), 256, 0, s>>>(c->last_i, c->I1, (int32_t)(t_first - 1));
  k_nmf_fill_i32<<<(unsigned)((c->U1 + 255) / 256), 256, 0, s>>>(c->pend_u, c->U1, (int32_t)t_first);
  k_nmf_fill_i32<<<(unsigned)((c->I1 + 255) / 256), 256, 0, s>>>(c->pend_i, c->I1, (int32_t)t_first);
  HIP_TRY(hipGetLastError());
  const int64_t nrows = c->U1 + c->I1;
  // k_nmf_adam_next's tail: 32 / gp float4s per wave, gp = the slot groups of a full
  // batch rounded up to a power of two (a smaller last batch packs more per wave)
  const int ng_max = (int)((std::min<int64_t>((batch + MR - 1) / MR, NSLOT) + SB - 1) / SB);
  int gp2 = 1;
  while (gp2 < ng_max) gp2 <<= 1;
  const int64_t tail_waves = (n4 - emb4 + 32 / gp2 - 1) / (32 / gp2);
  const unsigned tail_blocks = (unsigned)std::min<int64_t>((tail_waves + 3) / 4, 2048);
  const int lpr = 2 * z.d4 <= 32 ? 32 : 64;
  auto rows_grid = [&](int64_t rows, int64_t cap) {
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>((rows * lpr + 255) / 256, cap));
  };
  const int64_t slice = (nrows + c->lazy_s - 1) / c->lazy_s;
  bool side_pending = false;
  AdamK ak{};
  int64_t k = 0;
  for (int64_t o = 0; o < n; o += batch, ++k) {
    const int32_t B = (int32_t)std::min<int64_t>(batch, n - o);
    int r = launch_grad(c, P, G, u + o, i + o, y + o, B, hp, nullptr, s, false);
    if (r != ACF_OK) {
      if (side_pending) (void)hipStreamWaitEvent(s, c->ev_rest, 0);
      return r;
    }
    // Adam iteration t of step k: batch k+1's rows (up to t) and the parameter tail
    // now, with the weight-gradient slot sums (acf_neumf_grad's wsum arithmetic);
    // every other row's iterations later (k_nmf_adam_catchup)
    AdamSlots ws;
    ws.part = c->wpart;
    ws.nslot = (int)std::min<int64_t>(((int64_t)B + MR - 1) / MR, NSLOT);
    ws.npass = hp->adver ? 2 : 1;
    ws.base4 = emb4;
    ws.nout = wout(c->d).n;
    ws.loss_out = losses ? losses + 2 * k : nullptr;
    ws.B = (float)B;
    const int64_t t = t_first + k;
    ak = AdamK{hp->beta1, hp->beta2, adam_lr_t(hp, t), hp->adam_eps};
    z.t = (int32_t)t;
    for (int x = 0; x < LAZY_W; ++x) {
      const int64_t tau = t - (LAZY_W - 1) + x;
      z.lr[x] = tau >= 1 ? adam_lr_t(hp, tau) : 0.f;
    }
    const int64_t on = o + batch;
    const int32_t Bn = on < n ? (int32_t)std::min<int64_t>(batch, n - on) : 0;
    const unsigned row_blocks = (unsigned)((2 * (int64_t)Bn * 64 + 255) / 256);
    if (side_pending) HIP_TRY(hipStreamWaitEvent(s, c->ev_rest, 0));  // the catch-up of step k-1
    k_nmf_adam_next<<<row_blocks + tail_blocks, 256, 0, s>>>(P4, G4, m4, v4, n4, emb4, ak, ws, z, u + on, i + on,
                                                            Bn, row_blocks);
    HIP_TRY(hipGetLastError());
    side_pending = false;
    if (Bn > 0) {  // slice k % LAZY_S of the rows, beside step k+1
      const int64_t lo = (k % c->lazy_s) * slice, hi = std::min<int64_t>(lo + slice, nrows);
      if (lo < hi) {
        HIP_TRY(hipEventRecord(c->ev_next, s));
        HIP_TRY(hipStreamWaitEvent(c->side, c->ev_next, 0));
        k_nmf_adam_catchup<<<rows_grid(hi - lo, c->catchup_wg), 256, 0, c->side>>>(P4, G4, m4, v4, ak, z, lo, hi);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(c->ev_rest, c->side));
        side_pending = true;
      }
    }
  }
  if (side_pending) HIP_TRY(hipStreamWaitEvent(s, c->ev_rest, 0));
  if (k > 0) {  // every row to the last iteration
    k_nmf_adam_catchup<<<rows_grid(nrows, 256 * 16), 256, 0, s>>>(P4, G4, m4, v4, ak, z, 0, nrows);
    HIP_TRY(hipGetLastError());
  }
  return ACF_OK;
}

// The call is verified once, at its end (it synchronises there anyway).  With the
// rows-in-line step and the failsafe on, P, G, m, v are copied first (4 x the
// parameter bytes, D2D: ~40 us for the yelp shape against a ~150 ms epoch); a
// give-up (err bit 512) restores them and replays the whole call on the row-sum
// path, which gives the same bits (test_neumf_give_up_replays_exactly).
extern "C" int acf_neumf_train(acf_neumf_ctx* c, float* P, float* G, float* m, float* v,
                               const int32_t* u, const int32_t* i, const float* y, int64_t n,
                               int32_t batch, int64_t t_first, const acf_neumf_hparams* hp,
                               float* losses, void* stream_) {
  ACF_CHECK(c && P && G && m && v && u && i && y && hp, ACF_E_INVALID, "NULL argument");
  ACF_CHECK(batch > 0 && batch <= c->maxB, ACF_E_INVALID, "batch %d outside (0, %d]", batch, c->maxB);
  ACF_CHECK(n >= 0 && t_first >= 1, ACF_E_INVALID, "bad instance count or Adam iteration");
  hipStream_t s = static_cast<hipStream_t>(stream_);
  int r = settle_unchecked(c, s);
  if (r != ACF_OK) return r;
  const bool fr = n > 0 && std::min<int64_t>(batch, n) <= FR_MAXB && c->rows_in_line;
  float* bufs[4] = {P, G, m, v};
  const bool snap = fr && c->failsafe;
  if (snap && (r = take_snapshot(c, s, bufs, 4)) != ACF_OK) return r;
  r = train_launches(c, P, G, m, v, u, i, y, n, batch, t_first, hp, losses, s);
  if (r != ACF_OK) return r;
  int32_t herr = 0;
  if ((r = fetch_err(c, s, &herr)) != ACF_OK) return r;
  if ((herr & 512) && fr) {
    if ((r = reset_row_counters(c, s)) != ACF_OK) return r;
    if (!snap) return check_err(herr);
    if ((r = restore_snapshot(c, s, bufs, 4)) != ACF_OK) return r;
    c->rows_in_line = 0;
    r = train_launches(c, P, G, m, v, u, i, y, n, batch, t_first, hp, losses, s);
    c->rows_in_line = 1;
    if (r != ACF_OK) return r;
    ++c->recoveries;
    if ((r = fetch_err(c, s, &herr)) != ACF_OK) return r;
  }
  return check_err(herr);
}

#ifdef NMF_DIAG
extern "C" int acf_neumf_diag_stamps(uint64_t* out) {
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_nmf_stamps), 16 * sizeof(uint64_t)));
  HIP_TRY(hipMemcpyFromSymbol(out + 16, HIP_SYMBOL(g_nmf_rstamps), 8 * sizeof(uint64_t)));
  HIP_TRY(hipMemcpyFromSymbol(out + 24, HIP_SYMBOL(g_nmf_wstamps), 8 * sizeof(uint64_t)));
  return ACF_OK;
}
#endif

extern "C" int acf_neumf_predict(acf_neumf_ctx* c, const float* P, const int32_t* u, const int32_t* i,
                                 int64_t n, float* out, void* stream_) {
  ACF_CHECK(c && P && u && i && out, ACF_E_INVALID, "NULL argument");
  ACF_CHECK(n >= 0, ACF_E_INVALID, "negative count");
  hipStream_t s = static_cast<hipStream_t>(stream_);
  int r = settle_unchecked(c, s);
  if (r != ACF_OK) return r;
  HIP_TRY(hipMemsetAsync(c->err, 0, sizeof(int32_t), s));
  const int64_t chunk = 1 << 28;
  for (int64_t o = 0; o < n; o += chunk) {
    const int32_t m = (int32_t)std::min(chunk, n - o);
    NArgs a = make_args(c, P, nullptr, u + o, i + o, nullptr, m, 1.0f);
    a.pred = out + o;
    launch_inst<2>(a, (unsigned)std::min<int64_t>(((int64_t)m + MR - 1) / MR, 512), s);
    HIP_TRY(hipGetLastError());
  }
  return read_err(c, s);
}

// ---------------------------------------------------------------------------
// Keras BPR (BPR.py:23-99; run.py --model bpr, BASELINE configs[0]).
// params = [uEmb (U1 x d) | iEmb (I1 x d)] (BPR.py:35-36), gradient and Adam
// moments in the same layout.  Per batch of B triplets:
//   x = u.p - u.n (Dot layers, BPR.py:42-43); loss = 1 - log(sigmoid(x))
//   (bpr_triplet_loss, BPR.py:11-16); Keras loss = mean over the batch
//   (identity_loss, BPR.py:19-20), so d loss / d x = SigmoidGrad(LogGrad(-1/B)).
//   The gathered rows' gradients are summed per table row in occurrence order
//   (users: batch order; items: the positive gathers, then the negative ones:
//   TF's IndexedSlices densified), then Keras 2.2 Adam over the whole buffer.
// ---------------------------------------------------------------------------
template <int LPR>
__device__ __forceinline__ float kb_sum(float s) {
#pragma unroll
  for (int m = 1; m < LPR; m <<= 1) s += __shfl_xor(s, m, 64);
  return s;
}

// one lane-group of LPR lanes (one float4 each, d <= 4 LPR) per triplet
template <int LPR>
__global__ void __launch_bounds__(256) k_kbpr_inst(const float* __restrict__ P, const int32_t* __restrict__ u,
                                                   const int32_t* __restrict__ ip, const int32_t* __restrict__ in,
                                                   int32_t B, int32_t d, int64_t U1, int64_t I1,
                                                   float* __restrict__ contrib, float* __restrict__ loss,
                                                   int32_t* __restrict__ err) {
  const int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int b = (int)(gid / LPR), l = (int)(threadIdx.x & (LPR - 1));
  if (b >= B) return;
  int32_t ru = u[b], rp = ip[b], rn = in[b];
  if (l == 0 && (ru < 0 || ru >= U1)) atomicOr(err, 1);
  if (l == 0 && (rp < 0 || rp >= I1 || rn < 0 || rn >= I1)) atomicOr(err, 2);
  ru = (ru < 0 || ru >= U1) ? 0 : ru;
  rp = (rp < 0 || rp >= I1) ? 0 : rp;
  rn = (rn < 0 || rn >= I1) ? 0 : rn;
  const float* Q = P + U1 * (int64_t)d;
  const bool on = l * 4 < d;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 pu = on ? *reinterpret_cast<const float4*>(P + (int64_t)ru * d + 4 * l) : z;
  const float4 pp = on ? *reinterpret_cast<const float4*>(Q + (int64_t)rp * d + 4 * l) : z;
  const float4 pn = on ? *reinterpret_cast<const float4*>(Q + (int64_t)rn * d + 4 * l) : z;
  const float dp = kb_sum<LPR>(pu.x * pp.x + pu.y * pp.y + pu.z * pp.z + pu.w * pp.w);
  const float dn = kb_sum<LPR>(pu.x * pn.x + pu.y * pn.y + pu.z * pn.z + pu.w * pn.w);
  const float x = dp - dn;
  const float sg = 1.0f / (1.0f + expf(-x));           // K.sigmoid
  if (l == 0) loss[b] = 1.0f - logf(sg);               // 1 - K.log(.)
  const float up = -1.0f / (float)B;                   // d mean / d loss_b, through "1 - ."
  const float g = (up * (1.0f / sg)) * sg * (1.0f - sg);  // LogGrad, then SigmoidGrad
  if (!on) return;
  float4 gu, gp, gn;
  gu.x = g * pp.x + (-g) * pn.x; gu.y = g * pp.y + (-g) * pn.y;
  gu.z = g * pp.z + (-g) * pn.z; gu.w = g * pp.w + (-g) * pn.w;
  gp = make_float4(g * pu.x, g * pu.y, g * pu.z, g * pu.w);
  gn = make_float4(-g * pu.x, -g * pu.y, -g * pu.z, -g * pu.w);
  float* c = contrib + (int64_t)b * 3 * d + 4 * l;
  *reinterpret_cast<float4*>(c) = gu;
  *reinterpret_cast<float4*>(c + d) = gp;
  *reinterpret_cast<float4*>(c + 2 * d) = gn;
}

// one wave per gathered row occurrence: occurrence o < B is user b = o, o >= B
// is item slot o - B of [positives | negatives].  The first occurrence of a
// table row owns it and adds every occurrence's contribution in order.
__global__ void __launch_bounds__(256) k_kbpr_rows(const int32_t* __restrict__ u, const int32_t* __restrict__ ip,
                                                   const int32_t* __restrict__ in, int32_t B, int32_t d,
                                                   int64_t U1, int64_t I1, const float* __restrict__ contrib,
                                                   float* __restrict__ G) {
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= 3 * (int64_t)B) return;
  const int o = (int)wave;
  const bool item = o >= B;
  const int n = item ? 2 * B : B;  // occurrences of this table
  auto row_of = [&](int k) -> int32_t {  // table row of occurrence k of this table
    int32_t r = item ? (k < B ? ip[k] : in[k - B]) : u[k];
    const int64_t rows = item ? I1 : U1;
    return (r < 0 || r >= rows) ? 0 : r;
  };
  auto contrib_of = [&](int k) -> const float* {  // its gradient row
    return item ? contrib + ((int64_t)(k < B ? k : k - B) * 3 + (k < B ? 1 : 2)) * d
                : contrib + (int64_t)k * 3 * d;
  };
  const int me = item ? o - B : o;
  const int32_t r = row_of(me);
  for (int base = 0; base < me; base += 64) {  // an earlier occurrence owns the row
    const int k = base + lane;
    if (__any(k < me && row_of(k) == r)) return;
  }
  float acc[4] = {0.f, 0.f, 0.f, 0.f};  // d <= 256: lane holds elements lane + 64 q
  for (int base = me; base < n; base += 64) {
    const int k = base + lane;
    uint64_t mask = __ballot(k < n && row_of(k) == r);
    while (mask) {
      const int kk = base + __ffsll((unsigned long long)mask) - 1;
      mask &= mask - 1;
      const float* c = contrib_of(kk);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (lane + 64 * q < d) acc[q] = acc[q] + c[lane + 64 * q];
    }
  }
  float* g = G + (item ? U1 * (int64_t)d : 0) + (int64_t)r * d;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (lane + 64 * q < d) g[lane + 64 * q] = g[lane + 64 * q] + acc[q];
}

struct acf_kbpr_ctx {
  int64_t U1 = 0, I1 = 0;
  int32_t d = 0, maxB = 0;
  float* contrib = nullptr;
  int32_t* err = nullptr;
  std::vector<void*> allocs;
};

extern "C" int acf_kbpr_destroy(acf_kbpr_ctx* c) {
  if (!c) return ACF_OK;
  for (void* p : c->allocs) (void)hipFree(p);
  delete c;
  return ACF_OK;
}

extern "C" int acf_kbpr_create(acf_kbpr_ctx** out, int64_t U1, int64_t I1, int32_t d, int32_t maxB) {
  ACF_CHECK(out != nullptr, ACF_E_INVALID, "out is NULL");
  *out = nullptr;
  ACF_CHECK(U1 > 0 && I1 > 0 && U1 < (1ll << 31) && I1 < (1ll << 31), ACF_E_INVALID, "bad table rows");
  ACF_CHECK(d >= 4 && d <= 256 && d % 4 == 0, ACF_E_INVALID, "dim must be a multiple of 4 in [4, 256], got %d", d);
  ACF_CHECK(maxB > 0 && maxB <= (1 << 24), ACF_E_INVALID, "max_batch must be in (0, 2^24], got %d", maxB);
  acf_kbpr_ctx* c = new acf_kbpr_ctx();
  c->U1 = U1; c->I1 = I1; c->d = d; c->maxB = maxB;
  for (auto pr : {std::make_pair((void**)&c->contrib, (size_t)maxB * 3 * d * 4),
                  std::make_pair((void**)&c->err, (size_t)16)}) {
    if (hipMalloc(pr.first, pr.second) != hipSuccess) {
      (void)hipGetLastError();
      acf_kbpr_destroy(c);
      return set_error(ACF_E_NOMEM, "hipMalloc of %zu bytes failed", pr.second);
    }
    c->allocs.push_back(*pr.first);
  }
  if (hipMemset(c->err, 0, 16) != hipSuccess) {
    acf_kbpr_destroy(c);
    return set_error(ACF_E_HIP, "hipMemset failed");
  }
  *out = c;
  return ACF_OK;
}

template <int LPR>
static void launch_kbpr_inst(const acf_kbpr_ctx* c, const float* P, const int32_t* u, const int32_t* ip,
                             const int32_t* in, int32_t B, float* loss, hipStream_t s) {
  k_kbpr_inst<LPR><<<(unsigned)(((int64_t)B * LPR + 255) / 256), 256, 0, s>>>(P, u, ip, in, B, c->d, c->U1,
                                                                              c->I1, c->contrib, loss, c->err);
}

extern "C" int acf_kbpr_train(acf_kbpr_ctx* c, float* P, float* G, float* m, float* v, const int32_t* u,
                              const int32_t* ip, const int32_t* in, int64_t n, int32_t batch, int64_t t_first,
                              const acf_neumf_hparams* hp, float* losses, void* stream_) {
  ACF_CHECK(c && P && G && m && v && u && ip && in && hp && losses, ACF_E_INVALID, "NULL argument");
  ACF_CHECK(batch > 0 && batch <= c->maxB, ACF_E_INVALID, "batch %d outside (0, %d]", batch, c->maxB);
  ACF_CHECK(n >= 0 && t_first >= 1, ACF_E_INVALID, "bad triplet count or Adam iteration");
  hipStream_t s = static_cast<hipStream_t>(stream_);
  HIP_TRY(hipMemsetAsync(c->err, 0, sizeof(int32_t), s));
  const int64_t total = (c->U1 + c->I1) * (int64_t)c->d;
  const int64_t n4 = total / 4;
  const unsigned ga = (unsigned)std::min<int64_t>((n4 + 255) / 256, 256 * 32);
  int lpr = 1;
  while (lpr * 4 < c->d) lpr <<= 1;
  int64_t k = 0;
  for (int64_t o = 0; o < n; o += batch, ++k) {
    const int32_t B = (int32_t)std::min<int64_t>(batch, n - o);
    switch (lpr) {
      case 1: launch_kbpr_inst<1>(c, P, u + o, ip + o, in + o, B, losses + o, s); break;
      case 2: launch_kbpr_inst<2>(c, P, u + o, ip + o, in + o, B, losses + o, s); break;
      case 4: launch_kbpr_inst<4>(c, P, u + o, ip + o, in + o, B, losses + o, s); break;
      case 8: launch_kbpr_inst<8>(c, P, u + o, ip + o, in + o, B, losses + o, s); break;
      case 16: launch_kbpr_inst<16>(c, P, u + o, ip + o, in + o, B, losses + o, s); break;
      case 32: launch_kbpr_inst<32>(c, P, u + o, ip + o, in + o, B, losses + o, s); break;
      default: launch_kbpr_inst<64>(c, P, u + o, ip + o, in + o, B, losses + o, s); break;
    }
    k_kbpr_rows<<<(unsigned)((3 * (int64_t)B * 64 + 255) / 256), 256, 0, s>>>(u + o, ip + o, in + o, B, c->d,
                                                                             c->U1, c->I1, c->contrib, G);
    const float tt = (float)(t_first + k);
    const float lr_t = hp->lr * (sqrtf(1.0f - powf(hp->beta2, tt)) / (1.0f - powf(hp->beta1, tt)));
    k_nmf_adam<<<ga, 256, 0, s>>>(reinterpret_cast<float4*>(P), reinterpret_cast<float4*>(G),
                                  reinterpret_cast<float4*>(m), reinterpret_cast<float4*>(v), n4, hp->beta1,
                                  hp->beta2, lr_t, hp->adam_eps);
    HIP_TRY(hipGetLastError());
  }
  int32_t herr = 0;
  HIP_TRY(hipMemcpyAsync(&herr, c->err, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  ACF_CHECK(herr == 0, ACF_E_RANGE, "index out of range (%s%s)", (herr & 1) ? "user >= num_user_rows " : "",
            (herr & 2) ? "item >= num_item_rows" : "");
  return ACF_OK;
}

// predictor = Model([user, item], pDot) (BPR.py:57): u . i per pair
template <int LPR>
__global__ void __launch_bounds__(256) k_kbpr_predict(const float* __restrict__ P, const int32_t* __restrict__ u,
                                                      const int32_t* __restrict__ it, int64_t n, int32_t d,
                                                      int64_t U1, int64_t I1, float* __restrict__ out,
                                                      int32_t* __restrict__ err) {
  const int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t b = gid / LPR;
  const int l = (int)(threadIdx.x & (LPR - 1));
  if (b >= n) return;
  int32_t ru = u[b], ri = it[b];
  if (l == 0 && (ru < 0 || ru >= U1 || ri < 0 || ri >= I1)) atomicOr(err, (ru < 0 || ru >= U1) ? 1 : 2);
  ru = (ru < 0 || ru >= U1) ? 0 : ru;
  ri = (ri < 0 || ri >= I1) ? 0 : ri;
  const bool on = l * 4 < d;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 a = on ? *reinterpret_cast<const float4*>(P + (int64_t)ru * d + 4 * l) : z;
  const float4 q = on ? *reinterpret_cast<const float4*>(P + (U1 + ri) * (int64_t)d + 4 * l) : z;
  const float s = kb_sum<LPR>(a.x * q.x + a.y * q.y + a.z * q.z + a.w * q.w);
  if (l == 0) out[b] = s;
}

extern "C" int acf_kbpr_predict(acf_kbpr_ctx* c, const float* P, const int32_t* u, const int32_t* it, int64_t n,
                                float* out, void* stream_) {
  ACF_CHECK(c && P && u && it && out, ACF_E_INVALID, "NULL argument");
  ACF_CHECK(n >= 0, ACF_E_INVALID, "negative count");
  if (n == 0) return ACF_OK;
  hipStream_t s = static_cast<hipStream_t>(stream_);
  HIP_TRY(hipMemsetAsync(c->err, 0, sizeof(int32_t), s));
  int lpr = 1;
  while (lpr * 4 < c->d) lpr <<= 1;
  const unsigned g = (unsigned)((n * lpr + 255) / 256);
  switch (lpr) {
    case 1: k_kbpr_predict<1><<<g, 256, 0, s>>>(P, u, it, n, c->d, c->U1, c->I1, out, c->err); break;
    case 2: k_kbpr_predict<2><<<g, 256, 0, s>>>(P, u, it, n, c->d, c->U1, c->I1, out, c->err); break;
    case 4: k_kbpr_predict<4><<<g, 256, 0, s>>>(P, u, it, n, c->d, c->U1, c->I1, out, c->err); break;
    case 8: k_kbpr_predict<8><<<g, 256, 0, s>>>(P, u, it, n, c->d, c->U1, c->I1, out, c->err); break;
    case 16: k_kbpr_predict<16><<<g, 256, 0, s>>>(P, u, it, n, c->d, c->U1, c->I1, out, c->err); break;
    case 32: k_kbpr_predict<32><<<g, 256, 0, s>>>(P, u, it, n, c->d, c->U1, c->I1, out, c->err); break;
    default: k_kbpr_predict<64><<<g, 256, 0, s>>>(P, u, it, n, c->d, c->U1, c->I1, out, c->err); break;
  }
  HIP_TRY(hipGetLastError());
  int32_t herr = 0;
  HIP_TRY(hipMemcpyAsync(&herr, c->err, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  ACF_CHECK(herr == 0, ACF_E_RANGE, "index out of range (%s%s)", (herr & 1) ? "user >= num_user_rows " : "",
            (herr & 2) ? "item >= num_item_rows" : "");
  return ACF_OK;
}

// ---------------------------------------------------------------------------
// FastAdversarialMF (FastAdversarialMF.py:13-144; run.py --model amf2).
// params = [P (U1 x d) | Q (I1 x d) | D_u | D_i], a discriminator block being
// [W1 (d x d, Keras [in, out]) | b1 (d) | W2 (d) | b2 (1) | 3 pad]; gradient and
// Adam moments in the same layout.  Per batch of B instances (u, i, y) with the
// adversarial indices (ua, ia) and the players' popularity targets:
//   pred = P[u] . Q[i]; MSE vs y                                   (:48, :74)
//   D(e) = sigmoid(relu(e W1 + b1) . W2 + b2) on e = P[ua] / Q[ia]  (:119-127)
//   player mf (P, Q): MSE + BCE(D_u, tu) + BCE(D_i, ti), the discriminators
//   frozen; players disc_u / disc_i: BCE(D, du) / BCE(D, di), the embeddings
//   frozen; all at the same pre-step parameters (AdversarialOptimizerSimultaneous),
//   then one dense Keras Adam over the whole buffer (every player steps each batch).
// Kernels: k_amf_inst (one lane-group per instance: gathers, MSE, both
// discriminators forward and backward, row contributions + the per-instance
// factors of the weight gradients), k_amf_rows (per-row sums in occurrence
// order: P gets the u then the ua gathers, Q the i then the ia gathers),
// k_amf_wgrad (one thread per discriminator parameter, instances in order),
// k_nmf_adam.  Parity with the reference is unpinned (oracle/amf_oracle.py).
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ int64_t amf_disc_block(int64_t d) { return d * d + 2 * d + 4; }

#define ACF_RET_NEUMF(x)         \
  do {                           \
    int r_ = (x);                \
    if (r_ != ACF_OK) return r_; \
  } while (0)

struct AmfArgs {
  const float* params;
  float* grad;
  const int32_t *u, *i, *ua, *ia;
  const float *y, *tu, *ti, *du, *di;
  int32_t B, d;
  int64_t U1, I1;
  float* contrib;  // [B][4][d]: MSE -> P[u], MSE -> Q[i], D_u -> P[ua], D_i -> Q[ia]
  float* dscr;     // [2][B][3d + 4]: e, relu'(h) * dz_d * W2, relu(h), dz_d
  float* loss;     // [B][3]: squared error, BCE(D_u, tu), BCE(D_i, ti)
  int32_t* err;
};

__device__ __forceinline__ float4 f4_or0(const float* p, bool on) {
  return on ? *reinterpret_cast<const float4*>(p) : make_float4(0.f, 0.f, 0.f, 0.f);
}

template <int LPR>
__global__ void __launch_bounds__(256) k_amf_inst(AmfArgs a) {
  const int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int b = (int)(gid / LPR), l = (int)(threadIdx.x & (LPR - 1));
  if (b >= a.B) return;
  const int d = a.d;
  int32_t ru = a.u[b], ri = a.i[b], rua = a.ua[b], ria = a.ia[b];
  if (l == 0 && (ru < 0 || ru >= a.U1 || rua < 0 || rua >= a.U1)) atomicOr(a.err, 1);
  if (l == 0 && (ri < 0 || ri >= a.I1 || ria < 0 || ria >= a.I1)) atomicOr(a.err, 2);
  ru = (ru < 0 || ru >= a.U1) ? 0 : ru;
  rua = (rua < 0 || rua >= a.U1) ? 0 : rua;
  ri = (ri < 0 || ri >= a.I1) ? 0 : ri;
  ria = (ria < 0 || ria >= a.I1) ? 0 : ria;
  const float* P = a.params;
  const float* Q = P + a.U1 * (int64_t)d;
  const bool on = l * 4 < d;
  const float invB = 1.0f / (float)a.B;
  // prediction and MSE (the Dot layer's gradient: dpred * the other row)
  const float4 pu = f4_or0(P + (int64_t)ru * d + 4 * l, on), qi = f4_or0(Q + (int64_t)ri * d + 4 * l, on);
  const float pred = kb_sum<LPR>(pu.x * qi.x + pu.y * qi.y + pu.z * qi.z + pu.w * qi.w);
  const float diff = pred - a.y[b];
  if (l == 0) a.loss[(int64_t)b * 3] = diff * diff;
  const float dpred = (diff * 2.0f) * invB;  // mean's 1/B times SquareGrad's 2x
  float* c = a.contrib + (int64_t)b * 4 * d + 4 * l;
  if (on) {
    *reinterpret_cast<float4*>(c) = make_float4(dpred * qi.x, dpred * qi.y, dpred * qi.z, dpred * qi.w);
    *reinterpret_cast<float4*>(c + d) = make_float4(dpred * pu.x, dpred * pu.y, dpred * pu.z, dpred * pu.w);
  }
  const float* const D0 = P + (a.U1 + a.I1) * (int64_t)d;
#pragma unroll 1
  for (int X = 0; X < 2; ++X) {
    const float* W1 = D0 + X * amf_disc_block(d);
    const float* b1 = W1 + (int64_t)d * d;
    const float* W2 = b1 + d;
    const float b2 = W2[d];
    const float4 e = f4_or0((X ? Q + (int64_t)ria * d : P + (int64_t)rua * d) + 4 * l, on);
    // h = e W1 + b1: lane l holds outputs 4l..4l+3; e_k broadcast inside the lane-group
    float4 h = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int kk = 0; kk < d / 4; ++kk) {
      const float ek[4] = {__shfl(e.x, kk, LPR), __shfl(e.y, kk, LPR), __shfl(e.z, kk, LPR),
                           __shfl(e.w, kk, LPR)};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 w = f4_or0(W1 + (int64_t)(4 * kk + q) * d + 4 * l, on);
        h.x = fmaf(ek[q], w.x, h.x); h.y = fmaf(ek[q], w.y, h.y);
        h.z = fmaf(ek[q], w.z, h.z); h.w = fmaf(ek[q], w.w, h.w);
      }
    }
    const float4 bb = f4_or0(b1 + 4 * l, on), w2 = f4_or0(W2 + 4 * l, on);
    h = make_float4(h.x + bb.x, h.y + bb.y, h.z + bb.z, h.w + bb.w);
    const float4 act = make_float4(fmaxf(h.x, 0.f), fmaxf(h.y, 0.f), fmaxf(h.z, 0.f), fmaxf(h.w, 0.f));
    const float z = kb_sum<LPR>(act.x * w2.x + act.y * w2.y + act.z * w2.z + act.w * w2.w) + b2;
    const float s = 1.0f / (1.0f + expf(-z));
    const bool inside = s >= 1e-7f && s <= 1.0f - 1e-7f;  // clip_by_value's gradient
    const float tm = (X ? a.ti : a.tu)[b], td = (X ? a.di : a.du)[b];
    if (l == 0) {
      const float sc = fminf(fmaxf(s, 1e-7f), 1.0f - 1e-7f);
      a.loss[(int64_t)b * 3 + 1 + X] = -(tm * logf(sc) + (1.0f - tm) * logf(1.0f - sc));
    }
    const float dzm = inside ? (s - tm) * invB : 0.f, dzd = inside ? (s - td) * invB : 0.f;
    const float4 dhm = make_float4(h.x > 0.f ? dzm * w2.x : 0.f, h.y > 0.f ? dzm * w2.y : 0.f,
                                   h.z > 0.f ? dzm * w2.z : 0.f, h.w > 0.f ? dzm * w2.w : 0.f);
    // de = W1 dh_m: lane l holds rows 4l..4l+3 of W1, dh_m broadcast
    float4 de = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int nn = 0; nn < d / 4; ++nn) {
      const float4 g = make_float4(__shfl(dhm.x, nn, LPR), __shfl(dhm.y, nn, LPR), __shfl(dhm.z, nn, LPR),
                                   __shfl(dhm.w, nn, LPR));
      float* dst[4] = {&de.x, &de.y, &de.z, &de.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 w = f4_or0(W1 + (int64_t)(4 * l + q) * d + 4 * nn, on);
        float acc = *dst[q];
        acc = fmaf(w.x, g.x, acc); acc = fmaf(w.y, g.y, acc);
        acc = fmaf(w.z, g.z, acc); acc = fmaf(w.w, g.w, acc);
        *dst[q] = acc;
      }
    }
    if (on) {
      *reinterpret_cast<float4*>(c + (2 + X) * d) = de;
      float* sc = a.dscr + ((int64_t)X * a.B + b) * (3 * d + 4);
      *reinterpret_cast<float4*>(sc + 4 * l) = e;
      *reinterpret_cast<float4*>(sc + d + 4 * l) =
          make_float4(h.x > 0.f ? dzd * w2.x : 0.f, h.y > 0.f ? dzd * w2.y : 0.f, h.z > 0.f ? dzd * w2.z : 0.f,
                      h.w > 0.f ? dzd * w2.w : 0.f);
      *reinterpret_cast<float4*>(sc + 2 * d + 4 * l) = act;
      if (l == 0) sc[3 * d] = dzd;
    }
  }
}

// one wave per gathered row occurrence, 4B of them: P's [u_0..u_{B-1}, ua_0..],
// then Q's [i_0.., ia_0..].  The first occurrence of a row owns it and adds every
// occurrence's contribution in that order.
__global__ void __launch_bounds__(256) k_amf_rows(AmfArgs a) {
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const int B = a.B, d = a.d;
  if (wave >= 4 * (int64_t)B) return;
  const bool item = wave >= 2 * B;
  const int me = (int)(item ? wave - 2 * B : wave), n = 2 * B;
  auto row_of = [&](int k) -> int32_t {
    int32_t r = item ? (k < B ? a.i[k] : a.ia[k - B]) : (k < B ? a.u[k] : a.ua[k - B]);
    const int64_t rows = item ? a.I1 : a.U1;
    return (r < 0 || r >= rows) ? 0 : r;
  };
  auto contrib_of = [&](int k) -> const float* {
    const int b = k < B ? k : k - B, slot = (k < B ? 0 : 2) + (item ? 1 : 0);
    return a.contrib + ((int64_t)b * 4 + slot) * d;
  };
  const int32_t r = row_of(me);
  for (int base = 0; base < me; base += 64) {
    const int k = base + lane;
    if (__any(k < me && row_of(k) == r)) return;
  }
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int base = me; base < n; base += 64) {
    const int k = base + lane;
    uint64_t mask = __ballot(k < n && row_of(k) == r);
    while (mask) {
      const int kk = base + __ffsll((unsigned long long)mask) - 1;
      mask &= mask - 1;
      const float* cc = contrib_of(kk);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (lane + 64 * q < d) acc[q] = acc[q] + cc[lane + 64 * q];
    }
  }
  float* g = a.grad + (item ? a.U1 * (int64_t)d : 0) + (int64_t)r * d;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (lane + 64 * q < d) g[lane + 64 * q] = g[lane + 64 * q] + acc[q];
}

// one thread per discriminator parameter: W1[k][n] = sum_b e_b[k] dh_b[n],
// b1 = sum_b dh_b, W2 = sum_b relu(h_b) dz_b, b2 = sum_b dz_b (instances in order)
__global__ void __launch_bounds__(256) k_amf_wgrad(AmfArgs a) {
  const int64_t d = a.d, DB = amf_disc_block(d);
  const int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (x >= 2 * DB) return;
  const int X = (int)(x / DB);
  const int64_t j = x - X * DB;
  const float* sc = a.dscr + (int64_t)X * a.B * (3 * d + 4);
  const int64_t S = 3 * d + 4;
  float acc = 0.f;
  if (j < d * d) {
    const int64_t k = j / d, n = j - k * d;
    for (int b = 0; b < a.B; ++b) acc = acc + sc[b * S + k] * sc[b * S + d + n];
  } else if (j < d * d + d) {
    const int64_t n = j - d * d;
    for (int b = 0; b < a.B; ++b) acc = acc + sc[b * S + d + n];
  } else if (j < d * d + 2 * d) {
    const int64_t n = j - d * d - d;
    for (int b = 0; b < a.B; ++b) acc = acc + sc[b * S + 2 * d + n] * sc[b * S + 3 * d];
  } else if (j == d * d + 2 * d) {
    for (int b = 0; b < a.B; ++b) acc = acc + sc[b * S + 3 * d];
  } else {
    return;  // padding
  }
  float* g = a.grad + (a.U1 + a.I1) * d + x;
  *g = *g + acc;
}

struct acf_amf_ctx {
  int64_t U1 = 0, I1 = 0;
  int32_t d = 0, maxB = 0;
  float *contrib = nullptr, *dscr = nullptr;
  int32_t* err = nullptr;
  std::vector<void*> allocs;
};

extern "C" int64_t acf_amf_param_count(int64_t U1, int64_t I1, int32_t d) {
  return (U1 + I1) * (int64_t)d + 2 * amf_disc_block(d);
}

extern "C" int acf_amf_destroy(acf_amf_ctx* c) {
  if (!c) return ACF_OK;
  for (void* p : c->allocs) (void)hipFree(p);
  delete c;
  return ACF_OK;
}

extern "C" int acf_amf_create(acf_amf_ctx** out, int64_t U1, int64_t I1, int32_t d, int32_t maxB) {
  ACF_CHECK(out != nullptr, ACF_E_INVALID, "out is NULL");
  *out = nullptr;
  ACF_CHECK(U1 > 0 && I1 > 0 && U1 < (1ll << 31) && I1 < (1ll << 31), ACF_E_INVALID, "bad table rows");
  ACF_CHECK(d >= 4 && d <= 256 && d % 4 == 0, ACF_E_INVALID, "dim must be a multiple of 4 in [4, 256], got %d", d);
  ACF_CHECK(maxB > 0 && maxB <= (1 << 24), ACF_E_INVALID, "max_batch must be in (0, 2^24], got %d", maxB);
  acf_amf_ctx* c = new acf_amf_ctx();
  c->U1 = U1; c->I1 = I1; c->d = d; c->maxB = maxB;
  for (auto pr : {std::make_pair((void**)&c->contrib, (size_t)maxB * 4 * d * 4),
                  std::make_pair((void**)&c->dscr, (size_t)2 * maxB * (3 * d + 4) * 4),
                  std::make_pair((void**)&c->err, (size_t)16)}) {
    if (hipMalloc(pr.first, pr.second) != hipSuccess) {
      (void)hipGetLastError();
      acf_amf_destroy(c);
      return set_error(ACF_E_NOMEM, "hipMalloc of %zu bytes failed", pr.second);
    }
    c->allocs.push_back(*pr.first);
  }
  if (hipMemset(c->err, 0, 16) != hipSuccess) {
    acf_amf_destroy(c);
    return set_error(ACF_E_HIP, "hipMemset failed");
  }
  *out = c;
  return ACF_OK;
}

template <int LPR>
static void launch_amf_inst(const AmfArgs& a, hipStream_t s) {
  k_amf_inst<LPR><<<(unsigned)(((int64_t)a.B * LPR + 255) / 256), 256, 0, s>>>(a);
}

static int amf_batch(acf_amf_ctx* c, const AmfArgs& a, hipStream_t s) {
  int lpr = 1;
  while (lpr * 4 < c->d) lpr <<= 1;
  switch (lpr) {
    case 1: launch_amf_inst<1>(a, s); break;
    case 2: launch_amf_inst<2>(a, s); break;
    case 4: launch_amf_inst<4>(a, s); break;
    case 8: launch_amf_inst<8>(a, s); break;
    case 16: launch_amf_inst<16>(a, s); break;
    case 32: launch_amf_inst<32>(a, s); break;
    default: launch_amf_inst<64>(a, s); break;
  }
  k_amf_rows<<<(unsigned)((4 * (int64_t)a.B * 64 + 255) / 256), 256, 0, s>>>(a);
  k_amf_wgrad<<<(unsigned)((2 * amf_disc_block(c->d) + 255) / 256), 256, 0, s>>>(a);
  HIP_TRY(hipGetLastError());
  return ACF_OK;
}

static int amf_read_err(acf_amf_ctx* c, hipStream_t s) {
  int32_t herr = 0;
  HIP_TRY(hipMemcpyAsync(&herr, c->err, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  ACF_CHECK(herr == 0, ACF_E_RANGE, "index out of range (%s%s)", (herr & 1) ? "user >= num_user_rows " : "",
            (herr & 2) ? "item >= num_item_rows" : "");
  return ACF_OK;
}

extern "C" int acf_amf_grad(acf_amf_ctx* c, const float* params, float* grad, const int32_t* u, const int32_t* i,
                            const float* y, const int32_t* ua, const int32_t* ia, const float* tu, const float* ti,
                            const float* du, const float* di, int32_t B, float* loss, void* stream_) {
  ACF_CHECK(c && params && grad && u && i && y && ua && ia && tu && ti && du && di && loss, ACF_E_INVALID,
            "NULL argument");
  ACF_CHECK(B > 0 && B <= c->maxB, ACF_E_INVALID, "batch %d outside (0, %d]", B, c->maxB);
  hipStream_t s = static_cast<hipStream_t>(stream_);
  HIP_TRY(hipMemsetAsync(c->err, 0, sizeof(int32_t), s));
  const AmfArgs a{params, grad, u, i, ua, ia, y, tu, ti, du, di, B, c->d, c->U1, c->I1, c->contrib, c->dscr,
                  loss, c->err};
  ACF_RET_NEUMF(amf_batch(c, a, s));
  return amf_read_err(c, s);
}

extern "C" int acf_amf_train(acf_amf_ctx* c, float* params, float* grad, float* m, float* v, const int32_t* u,
                             const int32_t* i, const float* y, const int32_t* ua, const int32_t* ia, const float* tu,
                             const float* ti, const float* du, const float* di, int64_t n, int32_t batch,
                             int64_t t_first, const acf_neumf_hparams* hp, float* losses, void* stream_) {
  ACF_CHECK(c && params && grad && m && v && u && i && y && ua && ia && tu && ti && du && di && hp && losses,
            ACF_E_INVALID, "NULL argument");
  ACF_CHECK(batch > 0 && batch <= c->maxB, ACF_E_INVALID, "batch %d outside (0, %d]", batch, c->maxB);
  ACF_CHECK(n >= 0 && t_first >= 1, ACF_E_INVALID, "bad instance count or Adam iteration");
  hipStream_t s = static_cast<hipStream_t>(stream_);
  HIP_TRY(hipMemsetAsync(c->err, 0, sizeof(int32_t), s));
  const int64_t n4 = acf_amf_param_count(c->U1, c->I1, c->d) / 4;
  const unsigned ga = (unsigned)std::min<int64_t>((n4 + 255) / 256, 256 * 32);
  int64_t k = 0;
  for (int64_t o = 0; o < n; o += batch, ++k) {
    const int32_t B = (int32_t)std::min<int64_t>(batch, n - o);
    const AmfArgs a{params, grad, u + o, i + o, ua + o, ia + o, y + o, tu + o, ti + o, du + o, di + o,
                    B, c->d, c->U1, c->I1, c->contrib, c->dscr, losses + 3 * o, c->err};
    ACF_RET_NEUMF(amf_batch(c, a, s));
    const float tt = (float)(t_first + k);
    const float lr_t = hp->lr * (sqrtf(1.0f - powf(hp->beta2, tt)) / (1.0f - powf(hp->beta1, tt)));
    k_nmf_adam<<<ga, 256, 0, s>>>(reinterpret_cast<float4*>(params), reinterpret_cast<float4*>(grad),
                                  reinterpret_cast<float4*>(m), reinterpret_cast<float4*>(v), n4, hp->beta1,
                                  hp->beta2, lr_t, hp->adam_eps);
    HIP_TRY(hipGetLastError());
  }
  return amf_read_err(c, s);
}

// model = Model([user, item], pred) (FastAdversarialMF.py:51; MF.py:38-40): u . i per pair
extern "C" int acf_amf_predict(acf_amf_ctx* c, const float* params, const int32_t* u, const int32_t* it, int64_t n,
                               float* out, void* stream_) {
  ACF_CHECK(c && params && u && it && out, ACF_E_INVALID, "NULL argument");
  ACF_CHECK(n >= 0, ACF_E_INVALID, "negative count");
  if (n == 0) return ACF_OK;
  hipStream_t s = static_cast<hipStream_t>(stream_);
  HIP_TRY(hipMemsetAsync(c->err, 0, sizeof(int32_t), s));
  int lpr = 1;
  while (lpr * 4 < c->d) lpr <<= 1;
  const unsigned g = (unsigned)((n * lpr + 255) / 256);
  switch (lpr) {
    case 1: k_kbpr_predict<1><<<g, 256, 0, s>>>(params, u, it, n, c->d, c->U1, c->I1, out, c->err); break;
    case 2: k_kbpr_predict<2><<<g, 256, 0, s>>>(params, u, it, n, c->d, c->U1, c->I1, out, c->err); break;
    case 4: k_kbpr_predict<4><<<g, 256, 0, s>>>(params, u, it, n, c->d, c->U1, c->I1, out, c->err); break;
    case 8: k_kbpr_predict<8><<<g, 256, 0, s>>>(params, u, it, n, c->d, c->U1, c->I1, out, c->err); break;
    case 16: k_kbpr_predict<16><<<g, 256, 0, s>>>(params, u, it, n, c->d, c->U1, c->I1, out, c->err); break;
    case 32: k_kbpr_predict<32><<<g, 256, 0, s>>>(params, u, it, n, c->d, c->U1, c->I1, out, c->err); break;
    default: k_kbpr_predict<64><<<g, 256, 0, s>>>(params, u, it, n, c->d, c->U1, c->I1, out, c->err); break;
  }
  HIP_TRY(hipGetLastError());
  return amf_read_err(c, s);
}
