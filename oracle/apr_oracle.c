/*
 * apr_oracle.c — CPU restatement of the reference APR / BPR-MF training step.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline.  The product path (adversarial-collaborative-filtering_amd) never
 * calls it.
 *
 * What it restates (reference = feay1234/Adversarial-Collaborative-Filtering):
 *   MF graph           APR.py:121-195  (clean/adv inference, loss, delta, Adagrad)
 *   training_batch     utils.py:106-119 (update_P/update_Q run, then optimizer run)
 *   training_loss_acc  utils.py:159-175
 *   _eval_by_user      utils.py:244-254 (position = #neg >= pos)
 * with these TensorFlow-1 op semantics (TF is not installed here; the reference
 * pins no version — the API surface implies TF ~1.13-1.15):
 *   matmul(p*q, h)        product rounded, then summed                (APR.py:127)
 *   clip_by_value         gradient passes where lo <= x <= hi          (APR.py:148)
 *   softplus(f)           f > 13.9424 -> f; f < -13.9424 -> e^f; else log(e^f + 1)
 *   SoftplusGrad          upstream / (exp(-f) + 1)
 *   tf.gradients of a gathered table -> IndexedSlices; dense conversion and the
 *   optimizer's _deduplicate_indexed_slices both sum duplicate rows
 *   l2_normalize(x, 1)    x * rsqrt(max(sum x^2, 1e-12))               (APR.py:190)
 *   AdagradOptimizer      acc0 = 0.1; sparse apply: acc += g^2; w -= lr*g*rsqrt(acc)
 *
 * Parity status: the training-step arithmetic is PINNED STATISTICALLY only —
 * TensorFlow is absent, so no op-level output of the reference can be produced
 * here ("parity unpinned" at op level).  It is cross-checked against an
 * independent numpy restatement that materialises the TF graph densely
 * (oracle/apr_oracle.py) and against torch-CPU autograd of the same graph
 * (tests/test_oracle.py), and against the published Video/ml-1m run logs at
 * the end-to-end level.  The evaluation and data/sampler restatements are pinned
 * against fixtures produced by the reference's own Python (tests/golden/).
 *
 * `dense` = 1 reproduces the reference's per-batch work literally: the clean
 * gradient is densified to [rows, d] tables, every row is l2-normalised and
 * assigned to full delta tables (APR.py:183-191).  `dense` = 0 touches only the
 * rows in the batch (mathematically identical; rows outside the batch have
 * delta = 0 and are never read).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  float lr, eps, reg, reg_adv, clip_lo, clip_hi;
  int32_t adver;      /* APR graph (1) or BPR graph (0) */
  int32_t zero_delta; /* dns>1 branch: delta tables never assigned (stay 0) */
  int32_t dense;      /* 1: reference's dense delta work (see header) */
  int32_t adv_mode;   /* 0: adv = "grad" (APR.py:180-191); 1: adv = "random" (APR.py:170-177) */
  uint32_t call;      /* random mode: the context's call counter the HIP step read */
  int32_t t;          /* random mode: batch index inside the planned range */
  uint64_t seed;      /* random mode: hparams seed */
} oracle_hparams;

/* adv = "random" (APR.py:170-177): delta = eps * l2_normalize(truncated_normal(stddev
 * 0.01)), redrawn every run.  TF's Philox stream cannot be reproduced (TF is absent,
 * and the reference's own random branch assigns a [U, d] draw to a [U+1, d]
 * variable and does not build), so this restates the HIP path's counter-based
 * draw: splitmix64 keys over (seed, call counter, batch, side, row, element),
 * Box-Muller normals redrawn beyond 2 sigma; parity is with that definition. */
static uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static float u01(uint64_t h) { return ((float)(h >> 40) + 1.0f) * (1.0f / 16777216.0f); }

static float trunc_normal(uint64_t key, float stddev) {
  for (uint32_t a = 0;; ++a) {
    uint64_t h1 = mix64(key ^ mix64(2ull * a + 1));
    uint64_t h2 = mix64(key ^ mix64(2ull * a + 2));
    float r = sqrtf(-2.0f * logf(u01(h1)));
    float z = r * cosf(6.283185307179586f * u01(h2));
    if (fabsf(z) <= 2.0f || a > 64) return z * stddev;
  }
}

static void random_delta(const oracle_hparams* hp, int is_item, int32_t row, int d, float* out) {
  const uint64_t rk = mix64(hp->seed ^ mix64(((uint64_t)hp->call << 33) ^
                                             (((uint64_t)hp->t << 1) | (uint64_t)is_item))) ^
                      mix64((uint64_t)row * 0x100000001B3ull);
  float ss = 0.f;
  for (int k = 0; k < d; ++k) {
    out[k] = trunc_normal(rk ^ mix64((uint64_t)k), 0.01f);
    ss = ss + out[k] * out[k];
  }
  float inv = 1.0f / sqrtf(ss > 1e-12f ? ss : 1e-12f);
  for (int k = 0; k < d; ++k) out[k] = (out[k] * inv) * hp->eps;
}

#define SOFTPLUS_T 13.942385f

static float dotp(const float* a, const float* b, int d) {
  /* matmul(p*q, h): elementwise product rounded to fp32, then summed */
  float s = 0.f;
  for (int k = 0; k < d; ++k) {
    float pr = a[k] * b[k];
    s = s + pr;
  }
  return s;
}

static void bpr_term(float x, float lo, float hi, float* g, float* loss) {
  float xc = x < lo ? lo : (x > hi ? hi : x);
  int pass = (x >= lo) && (x <= hi);
  float f = -xc;
  *g = pass ? -(1.0f / (expf(-f) + 1.0f)) : 0.0f;
  *loss = f > SOFTPLUS_T ? f : (f < -SOFTPLUS_T ? expf(f) : logf(expf(f) + 1.0f));
}

/* row -> slot map for the rows a batch touches */
typedef struct {
  int32_t* slot_of; /* [rows], -1 when untouched */
  int32_t* rows;    /* [cap] unique rows in first-touch order */
  int32_t* count;   /* [cap] occurrences */
  float* acc;       /* [cap, d] gradient accumulator */
  int n, d;
} rowset;

static int rowset_init(rowset* r, int64_t rows, int cap, int d) {
  r->slot_of = (int32_t*)malloc(sizeof(int32_t) * (size_t)rows);
  r->rows = (int32_t*)malloc(sizeof(int32_t) * (size_t)cap);
  r->count = (int32_t*)malloc(sizeof(int32_t) * (size_t)cap);
  r->acc = (float*)malloc(sizeof(float) * (size_t)cap * d);
  if (!r->slot_of || !r->rows || !r->count || !r->acc) return -1;
  for (int64_t x = 0; x < rows; ++x) r->slot_of[x] = -1;
  r->n = 0;
  r->d = d;
  return 0;
}

static void rowset_free(rowset* r) {
  free(r->slot_of); free(r->rows); free(r->count); free(r->acc);
}

static int rowset_touch(rowset* r, int32_t row) {
  int s = r->slot_of[row];
  if (s < 0) {
    s = r->n++;
    r->slot_of[row] = s;
    r->rows[s] = row;
    r->count[s] = 0;
    memset(r->acc + (size_t)s * r->d, 0, sizeof(float) * r->d);
  }
  return s;
}

static void rowset_clear(rowset* r) {
  for (int s = 0; s < r->n; ++s) r->slot_of[r->rows[s]] = -1;
  r->n = 0;
}

static void axpy(float* y, float a, const float* x, int d) {
  for (int k = 0; k < d; ++k) y[k] = y[k] + a * x[k];
}

/* One mini-batch of training_batch (utils.py:114-119).  Tables are updated in
 * place.  loss_clean / loss_adv (length B) receive the per-triplet softplus
 * terms; delta_P / delta_Q (dense, optional) receive the assigned delta tables. */
int oracle_apr_batch(float* P, float* Q, float* accP, float* accQ, int64_t U1, int64_t I1, int d,
                     const int32_t* u, const int32_t* ip, const int32_t* in, int B,
                     const oracle_hparams* hp, float* loss_clean, float* loss_adv,
                     float* delta_P, float* delta_Q) {
  for (int b = 0; b < B; ++b)
    if (u[b] < 0 || u[b] >= U1 || ip[b] < 0 || ip[b] >= I1 || in[b] < 0 || in[b] >= I1) return -2;
  rowset RU, RI;
  if (rowset_init(&RU, U1, B, d) || rowset_init(&RI, I1, 2 * B, d)) return -1;
  float* g = (float*)malloc(sizeof(float) * B);
  float* ga = (float*)malloc(sizeof(float) * B);
  float* pp = (float*)malloc(sizeof(float) * d);
  float* qi = (float*)malloc(sizeof(float) * d);
  float* qj = (float*)malloc(sizeof(float) * d);
  /* slot-indexed delta rows (sparse) */
  float* dU = (float*)calloc((size_t)B * d, sizeof(float));
  float* dI = (float*)calloc((size_t)2 * B * d, sizeof(float));
  float* G0U = (float*)calloc((size_t)B * d, sizeof(float));
  float* G0I = (float*)calloc((size_t)2 * B * d, sizeof(float));
  float *denseU = NULL, *denseI = NULL;
  if (!g || !ga || !pp || !qi || !qj || !dU || !dI || !G0U || !G0I) return -1;

  /* 1. clean forward, per-triplet gradient scale (APR.py:146-150) */
  for (int b = 0; b < B; ++b) {
    const float* p = P + (int64_t)u[b] * d;
    float x = dotp(p, Q + (int64_t)ip[b] * d, d) - dotp(p, Q + (int64_t)in[b] * d, d);
    float l;
    bpr_term(x, hp->clip_lo, hp->clip_hi, &g[b], &l);
    if (loss_clean) loss_clean[b] = l;
  }
  /* touch rows: users, then items (pos then neg) — the concat order of the
   * IndexedSlices of the pos branch then the neg branch */
  for (int b = 0; b < B; ++b) RU.count[rowset_touch(&RU, u[b])]++;
  for (int b = 0; b < B; ++b) RI.count[rowset_touch(&RI, ip[b])]++;
  for (int b = 0; b < B; ++b) RI.count[rowset_touch(&RI, in[b])]++;

  if (hp->adver) {
    /* 2. clean-loss gradient, segment-summed (tf.gradients(loss, [P, Q])) */
    for (int b = 0; b < B; ++b) { /* pos branch */
      axpy(G0U + (size_t)RU.slot_of[u[b]] * d, g[b], Q + (int64_t)ip[b] * d, d);
      axpy(G0I + (size_t)RI.slot_of[ip[b]] * d, g[b], P + (int64_t)u[b] * d, d);
    }
    for (int b = 0; b < B; ++b) { /* neg branch */
      axpy(G0U + (size_t)RU.slot_of[u[b]] * d, -g[b], Q + (int64_t)in[b] * d, d);
      axpy(G0I + (size_t)RI.slot_of[in[b]] * d, -g[b], P + (int64_t)u[b] * d, d);
    }
    /* 3. delta = eps * l2_normalize(grad)   (APR.py:186-191) */
    if (hp->dense) {
      /* the reference's dense work: densify, normalise every row, assign */
      denseU = (float*)calloc((size_t)U1 * d, sizeof(float));
      denseI = (float*)calloc((size_t)I1 * d, sizeof(float));
      if (!denseU || !denseI) return -1;
      for (int s = 0; s < RU.n; ++s)
        memcpy(denseU + (int64_t)RU.rows[s] * d, G0U + (size_t)s * d, sizeof(float) * d);
      for (int s = 0; s < RI.n; ++s)
        memcpy(denseI + (int64_t)RI.rows[s] * d, G0I + (size_t)s * d, sizeof(float) * d);
      float* tabs[2] = {denseU, denseI};
      int64_t nrows[2] = {U1, I1};
      for (int t = 0; t < 2; ++t)
        for (int64_t r = 0; r < nrows[t]; ++r) {
          float* x = tabs[t] + r * d;
          float ss = 0.f;
          for (int k = 0; k < d; ++k) ss = ss + x[k] * x[k];
          float inv = 1.0f / sqrtf(ss > 1e-12f ? ss : 1e-12f);
          for (int k = 0; k < d; ++k) x[k] = hp->zero_delta ? 0.f : (x[k] * inv) * hp->eps;
        }
      for (int s = 0; s < RU.n; ++s)
        memcpy(dU + (size_t)s * d, denseU + (int64_t)RU.rows[s] * d, sizeof(float) * d);
      for (int s = 0; s < RI.n; ++s)
        memcpy(dI + (size_t)s * d, denseI + (int64_t)RI.rows[s] * d, sizeof(float) * d);
    } else {
      float* src[2] = {G0U, G0I};
      float* dst[2] = {dU, dI};
      int ns[2] = {RU.n, RI.n};
      for (int t = 0; t < 2; ++t)
        for (int s = 0; s < ns[t]; ++s) {
          const float* x = src[t] + (size_t)s * d;
          float ss = 0.f;
          for (int k = 0; k < d; ++k) ss = ss + x[k] * x[k];
          float inv = 1.0f / sqrtf(ss > 1e-12f ? ss : 1e-12f);
          for (int k = 0; k < d; ++k)
            dst[t][(size_t)s * d + k] = hp->zero_delta ? 0.f : (x[k] * inv) * hp->eps;
        }
    }
    if (hp->adv_mode == 1 && !hp->zero_delta) {
      for (int s = 0; s < RU.n; ++s) random_delta(hp, 0, RU.rows[s], d, dU + (size_t)s * d);
      for (int s = 0; s < RI.n; ++s) random_delta(hp, 1, RI.rows[s], d, dI + (size_t)s * d);
    }
    if (delta_P)
      for (int s = 0; s < RU.n; ++s)
        memcpy(delta_P + (int64_t)RU.rows[s] * d, dU + (size_t)s * d, sizeof(float) * d);
    if (delta_Q)
      for (int s = 0; s < RI.n; ++s)
        memcpy(delta_Q + (int64_t)RI.rows[s] * d, dI + (size_t)s * d, sizeof(float) * d);
    /* 4. adversarial forward on p + dP[u], q + dQ[i]   (APR.py:130-141,158-162) */
    for (int b = 0; b < B; ++b) {
      const float* du = dU + (size_t)RU.slot_of[u[b]] * d;
      const float* di = dI + (size_t)RI.slot_of[ip[b]] * d;
      const float* dj = dI + (size_t)RI.slot_of[in[b]] * d;
      const float* p = P + (int64_t)u[b] * d;
      for (int k = 0; k < d; ++k) {
        pp[k] = p[k] + du[k];
        qi[k] = Q[(int64_t)ip[b] * d + k] + di[k];
        qj[k] = Q[(int64_t)in[b] * d + k] + dj[k];
      }
      float x = dotp(pp, qi, d) - dotp(pp, qj, d);
      float l;
      bpr_term(x, hp->clip_lo, hp->clip_hi, &ga[b], &l);
      if (loss_adv) loss_adv[b] = l;
    }
  }

  /* 5. optimizer gradient of opt_loss, deduplicated (concat order: clean pos,
   *    clean neg, [adv pos, adv neg]; reg terms add 2*reg*w/(B*d) per
   *    occurrence, twice in the APR graph) */
  for (int b = 0; b < B; ++b) {
    axpy(RU.acc + (size_t)RU.slot_of[u[b]] * d, g[b], Q + (int64_t)ip[b] * d, d);
    axpy(RI.acc + (size_t)RI.slot_of[ip[b]] * d, g[b], P + (int64_t)u[b] * d, d);
  }
  for (int b = 0; b < B; ++b) {
    axpy(RU.acc + (size_t)RU.slot_of[u[b]] * d, -g[b], Q + (int64_t)in[b] * d, d);
    axpy(RI.acc + (size_t)RI.slot_of[in[b]] * d, -g[b], P + (int64_t)u[b] * d, d);
  }
  if (hp->reg != 0.f) {
    float coef = (2.0f * hp->reg / ((float)B * (float)d)) * (hp->adver ? 2.0f : 1.0f);
    for (int s = 0; s < RU.n; ++s)
      axpy(RU.acc + (size_t)s * d, coef * (float)RU.count[s], P + (int64_t)RU.rows[s] * d, d);
    for (int s = 0; s < RI.n; ++s)
      axpy(RI.acc + (size_t)s * d, coef * (float)RI.count[s], Q + (int64_t)RI.rows[s] * d, d);
  }
  if (hp->adver) {
    float lam = hp->reg_adv;
    for (int pass = 0; pass < 2; ++pass)
      for (int b = 0; b < B; ++b) {
        const float* du = dU + (size_t)RU.slot_of[u[b]] * d;
        const float* p = P + (int64_t)u[b] * d;
        int item = pass == 0 ? ip[b] : in[b];
        const float* dq = dI + (size_t)RI.slot_of[item] * d;
        const float* q = Q + (int64_t)item * d;
        float sgn = pass == 0 ? 1.f : -1.f;
        for (int k = 0; k < d; ++k) { pp[k] = p[k] + du[k]; qi[k] = q[k] + dq[k]; }
        axpy(RU.acc + (size_t)RU.slot_of[u[b]] * d, lam * sgn * ga[b], qi, d);
        axpy(RI.acc + (size_t)RI.slot_of[item] * d, lam * sgn * ga[b], pp, d);
      }
  }
  /* 6. SparseApplyAdagrad on the unique rows */
  rowset* sets[2] = {&RU, &RI};
  float* W[2] = {P, Q};
  float* A[2] = {accP, accQ};
  for (int t = 0; t < 2; ++t)
    for (int s = 0; s < sets[t]->n; ++s) {
      float* w = W[t] + (int64_t)sets[t]->rows[s] * d;
      float* a = A[t] + (int64_t)sets[t]->rows[s] * d;
      const float* gr = sets[t]->acc + (size_t)s * d;
      for (int k = 0; k < d; ++k) {
        a[k] = a[k] + gr[k] * gr[k];
        w[k] = w[k] - (hp->lr * gr[k]) * (1.0f / sqrtf(a[k]));
      }
    }
  rowset_clear(&RU);
  rowset_clear(&RI);
  rowset_free(&RU);
  rowset_free(&RI);
  free(g); free(ga); free(pp); free(qi); free(qj);
  free(dU); free(dI); free(G0U); free(G0I); free(denseU); free(denseI);
  return 0;
}

/* training_batch over n_batches consecutive batches (utils.py:113-119). */
int oracle_apr_train(float* P, float* Q, float* accP, float* accQ, int64_t U1, int64_t I1, int d,
                     const int32_t* u, const int32_t* ip, const int32_t* in, int B, int n_batches,
                     const oracle_hparams* hp) {
  oracle_hparams h = *hp;
  for (int t = 0; t < n_batches; ++t) {
    int64_t o = (int64_t)t * B;
    h.t = hp->t + t;
    int r = oracle_apr_batch(P, Q, accP, accQ, U1, I1, d, u + o, ip + o, in + o, B, &h, NULL, NULL,
                             NULL, NULL);
    if (r) return r;
  }
  return 0;
}

/* training_loss_acc (utils.py:159-175) per batch: loss sum and #(x+ > x-). */
int oracle_bpr_forward(const float* P, const float* Q, int64_t U1, int64_t I1, int d,
                       const int32_t* u, const int32_t* ip, const int32_t* in, int B,
                       int n_batches, float lo, float hi, float* batch_loss, int32_t* batch_correct,
                       float* out_pos, float* out_neg) {
  for (int t = 0; t < n_batches; ++t) {
    float ls = 0.f;
    int32_t c = 0;
    for (int b = 0; b < B; ++b) {
      int64_t e = (int64_t)t * B + b;
      if (u[e] < 0 || u[e] >= U1 || ip[e] < 0 || ip[e] >= I1 || in[e] < 0 || in[e] >= I1) return -2;
      const float* p = P + (int64_t)u[e] * d;
      float xp = dotp(p, Q + (int64_t)ip[e] * d, d), xn = dotp(p, Q + (int64_t)in[e] * d, d);
      float g, l;
      bpr_term(xp - xn, lo, hi, &g, &l);
      ls += l;
      c += (xp - xn) > 0.f;
      if (out_pos) out_pos[e] = xp;
      if (out_neg) out_neg[e] = xn;
    }
    if (batch_loss) batch_loss[t] = ls;
    if (batch_correct) batch_correct[t] = c;
  }
  return 0;
}

/* _eval_by_user, "all" candidates (utils.py:211-215, 253-254). */
int oracle_eval_positions_all(const float* P, const float* Q, int d, const int32_t* users,
                              const int32_t* tests, int n_users, int num_cand,
                              const int64_t* excl_off, const int32_t* excl, int32_t* positions) {
  for (int k = 0; k < n_users; ++k) {
    const float* p = P + (int64_t)users[k] * d;
    float st = dotp(p, Q + (int64_t)tests[k] * d, d);
    int64_t e = excl_off[k], e1 = excl_off[k + 1];
    int32_t pos = 0;
    for (int c = 0; c < num_cand; ++c) {
      while (e < e1 && excl[e] < c) ++e;
      if (e < e1 && excl[e] == c) continue;
      pos += dotp(p, Q + (int64_t)c * d, d) >= st;
    }
    positions[k] = pos;
  }
  return 0;
}

/* _eval_by_user with an explicit candidate list ("sample" mode). */
int oracle_eval_positions_list(const float* P, const float* Q, int d, const int32_t* users,
                               const int32_t* tests, int n_users, const int64_t* cand_off,
                               const int32_t* cand, int32_t* positions) {
  for (int k = 0; k < n_users; ++k) {
    const float* p = P + (int64_t)users[k] * d;
    float st = dotp(p, Q + (int64_t)tests[k] * d, d);
    int32_t pos = 0;
    for (int64_t x = cand_off[k]; x < cand_off[k + 1]; ++x)
      pos += dotp(p, Q + (int64_t)cand[x] * d, d) >= st;
    positions[k] = pos;
  }
  return 0;
}

/* ---- the CPU baseline on every host core (bench.py cpu_baseline) ----
 * oracle_apr_train with the batch's work split over `nthreads` OpenMP threads,
 * every sum kept in the single-thread order, so the result is bit-identical to
 * oracle_apr_train (tests/test_oracle.py::test_threaded_oracle_bit_identical):
 *   per-triplet terms (clean / adversarial forward)      split by triplet;
 *   per-row sums (IndexedSlices, reg, adversarial terms)  split by row slot
 *     (slot % T): each thread walks every occurrence in the batch's order and
 *     adds only its own rows' terms, so a row's additions keep their order;
 *   the dense delta work (APR.py:183-191: zero, scatter, l2-normalise every
 *     row of both tables, gather) and the Adagrad apply   split by row.
 * Finding the batch's unique rows (first-touch order) stays on one thread. */
#include <omp.h>

int oracle_apr_train_mt(float* P, float* Q, float* accP, float* accQ, int64_t U1, int64_t I1, int d,
                        const int32_t* u0, const int32_t* ip0, const int32_t* in0, int B, int n_batches,
                        const oracle_hparams* hp, int nthreads) {
  for (int64_t e = 0; e < (int64_t)B * n_batches; ++e)
    if (u0[e] < 0 || u0[e] >= U1 || ip0[e] < 0 || ip0[e] >= I1 || in0[e] < 0 || in0[e] >= I1) return -2;
  rowset RU, RI;
  if (rowset_init(&RU, U1, B, d) || rowset_init(&RI, I1, 2 * B, d)) return -1;
  float* g = (float*)malloc(sizeof(float) * B);
  float* ga = (float*)malloc(sizeof(float) * B);
  int32_t* su = (int32_t*)malloc(sizeof(int32_t) * B);   /* triplet -> user slot */
  int32_t* si = (int32_t*)malloc(sizeof(int32_t) * B);   /* -> positive item slot */
  int32_t* sj = (int32_t*)malloc(sizeof(int32_t) * B);   /* -> negative item slot */
  float* dU = (float*)calloc((size_t)B * d, sizeof(float));
  float* dI = (float*)calloc((size_t)2 * B * d, sizeof(float));
  float* G0U = (float*)calloc((size_t)B * d, sizeof(float));
  float* G0I = (float*)calloc((size_t)2 * B * d, sizeof(float));
  float* denseU = hp->dense ? (float*)malloc(sizeof(float) * (size_t)U1 * d) : NULL;
  float* denseI = hp->dense ? (float*)malloc(sizeof(float) * (size_t)I1 * d) : NULL;
  if (!g || !ga || !su || !si || !sj || !dU || !dI || !G0U || !G0I || (hp->dense && (!denseU || !denseI)))
    return -1;
  const float lam = hp->reg_adv;
  const float coef = (2.0f * hp->reg / ((float)B * (float)d)) * (hp->adver ? 2.0f : 1.0f);
#pragma omp parallel num_threads(nthreads)
  {
    const int tid = omp_get_thread_num(), T = omp_get_num_threads();
    float* pp = (float*)malloc(sizeof(float) * d);
    float* qi = (float*)malloc(sizeof(float) * d);
    float* qj = (float*)malloc(sizeof(float) * d);
    oracle_hparams h = *hp;
    for (int t = 0; t < n_batches; ++t) {
      const int32_t *u = u0 + (int64_t)t * B, *ip = ip0 + (int64_t)t * B, *in = in0 + (int64_t)t * B;
      h.t = hp->t + t;
#pragma omp for schedule(static)
      for (int b = 0; b < B; ++b) { /* 1. clean forward */
        const float* p = P + (int64_t)u[b] * d;
        float x = dotp(p, Q + (int64_t)ip[b] * d, d) - dotp(p, Q + (int64_t)in[b] * d, d);
        float l;
        bpr_term(x, h.clip_lo, h.clip_hi, &g[b], &l);
      }
#pragma omp single
      {
        for (int b = 0; b < B; ++b) RU.count[su[b] = rowset_touch(&RU, u[b])]++;
        for (int b = 0; b < B; ++b) RI.count[si[b] = rowset_touch(&RI, ip[b])]++;
        for (int b = 0; b < B; ++b) RI.count[sj[b] = rowset_touch(&RI, in[b])]++;
      } /* (rowset_touch zeroes each new slot's acc row) */
      if (h.adver) {
        /* 2. clean gradient segment sums, each slot in occurrence order */
#pragma omp for schedule(static)
        for (int s = 0; s < 2 * B; ++s) {
          if (s < B) memset(G0U + (size_t)s * d, 0, sizeof(float) * d);
          memset(G0I + (size_t)s * d, 0, sizeof(float) * d);
        }
        for (int b = 0; b < B; ++b) {
          if (su[b] % T == tid) axpy(G0U + (size_t)su[b] * d, g[b], Q + (int64_t)ip[b] * d, d);
          if (si[b] % T == tid) axpy(G0I + (size_t)si[b] * d, g[b], P + (int64_t)u[b] * d, d);
        }
        for (int b = 0; b < B; ++b) {
          if (su[b] % T == tid) axpy(G0U + (size_t)su[b] * d, -g[b], Q + (int64_t)in[b] * d, d);
          if (sj[b] % T == tid) axpy(G0I + (size_t)sj[b] * d, -g[b], P + (int64_t)u[b] * d, d);
        }
#pragma omp barrier
        /* 3. delta = eps * l2_normalize(grad) */
        if (h.dense) {
#pragma omp for schedule(static)
          for (int64_t r = 0; r < U1 + I1; ++r)
            memset(r < U1 ? denseU + r * d : denseI + (r - U1) * d, 0, sizeof(float) * d);
#pragma omp for schedule(static)
          for (int s = 0; s < RU.n + RI.n; ++s) {
            if (s < RU.n) memcpy(denseU + (int64_t)RU.rows[s] * d, G0U + (size_t)s * d, sizeof(float) * d);
            else memcpy(denseI + (int64_t)RI.rows[s - RU.n] * d, G0I + (size_t)(s - RU.n) * d, sizeof(float) * d);
          }
#pragma omp for schedule(static)
          for (int64_t r = 0; r < U1 + I1; ++r) {
            float* x = r < U1 ? denseU + r * d : denseI + (r - U1) * d;
            float ss = 0.f;
            for (int k = 0; k < d; ++k) ss = ss + x[k] * x[k];
            float inv = 1.0f / sqrtf(ss > 1e-12f ? ss : 1e-12f);
            for (int k = 0; k < d; ++k) x[k] = h.zero_delta ? 0.f : (x[k] * inv) * h.eps;
          }
#pragma omp for schedule(static)
          for (int s = 0; s < RU.n + RI.n; ++s) {
            if (s < RU.n) memcpy(dU + (size_t)s * d, denseU + (int64_t)RU.rows[s] * d, sizeof(float) * d);
            else memcpy(dI + (size_t)(s - RU.n) * d, denseI + (int64_t)RI.rows[s - RU.n] * d, sizeof(float) * d);
          }
        } else {
#pragma omp for schedule(static)
          for (int s = 0; s < RU.n + RI.n; ++s) {
            const float* x = s < RU.n ? G0U + (size_t)s * d : G0I + (size_t)(s - RU.n) * d;
            float* y = s < RU.n ? dU + (size_t)s * d : dI + (size_t)(s - RU.n) * d;
            float ss = 0.f;
            for (int k = 0; k < d; ++k) ss = ss + x[k] * x[k];
            float inv = 1.0f / sqrtf(ss > 1e-12f ? ss : 1e-12f);
            for (int k = 0; k < d; ++k) y[k] = h.zero_delta ? 0.f : (x[k] * inv) * h.eps;
          }
        }
        if (h.adv_mode == 1 && !h.zero_delta) {
#pragma omp for schedule(static)
          for (int s = 0; s < RU.n + RI.n; ++s) {
            if (s < RU.n) random_delta(&h, 0, RU.rows[s], d, dU + (size_t)s * d);
            else random_delta(&h, 1, RI.rows[s - RU.n], d, dI + (size_t)(s - RU.n) * d);
          }
        }
        /* 4. adversarial forward */
#pragma omp for schedule(static)
        for (int b = 0; b < B; ++b) {
          const float *du = dU + (size_t)su[b] * d, *di = dI + (size_t)si[b] * d, *dj = dI + (size_t)sj[b] * d;
          const float* p = P + (int64_t)u[b] * d;
          for (int k = 0; k < d; ++k) {
            pp[k] = p[k] + du[k];
            qi[k] = Q[(int64_t)ip[b] * d + k] + di[k];
            qj[k] = Q[(int64_t)in[b] * d + k] + dj[k];
          }
          float x = dotp(pp, qi, d) - dotp(pp, qj, d);
          float l;
          bpr_term(x, h.clip_lo, h.clip_hi, &ga[b], &l);
        }
      }
      /* 5. the optimizer's deduplicated gradient, each slot in the single-thread order */
      for (int b = 0; b < B; ++b) {
        if (su[b] % T == tid) axpy(RU.acc + (size_t)su[b] * d, g[b], Q + (int64_t)ip[b] * d, d);
        if (si[b] % T == tid) axpy(RI.acc + (size_t)si[b] * d, g[b], P + (int64_t)u[b] * d, d);
      }
      for (int b = 0; b < B; ++b) {
        if (su[b] % T == tid) axpy(RU.acc + (size_t)su[b] * d, -g[b], Q + (int64_t)in[b] * d, d);
        if (sj[b] % T == tid) axpy(RI.acc + (size_t)sj[b] * d, -g[b], P + (int64_t)u[b] * d, d);
      }
      if (h.reg != 0.f) {
        for (int s = tid; s < RU.n; s += T)
          axpy(RU.acc + (size_t)s * d, coef * (float)RU.count[s], P + (int64_t)RU.rows[s] * d, d);
        for (int s = tid; s < RI.n; s += T)
          axpy(RI.acc + (size_t)s * d, coef * (float)RI.count[s], Q + (int64_t)RI.rows[s] * d, d);
      }
      if (h.adver)
        for (int pass = 0; pass < 2; ++pass)
          for (int b = 0; b < B; ++b) {
            const int32_t sq = pass == 0 ? si[b] : sj[b];
            const int mine_u = su[b] % T == tid, mine_i = sq % T == tid;
            if (!mine_u && !mine_i) continue;
            const float* du = dU + (size_t)su[b] * d;
            const float* p = P + (int64_t)u[b] * d;
            const int item = pass == 0 ? ip[b] : in[b];
            const float* dq = dI + (size_t)sq * d;
            const float* q = Q + (int64_t)item * d;
            const float sgn = pass == 0 ? 1.f : -1.f;
            for (int k = 0; k < d; ++k) { pp[k] = p[k] + du[k]; qi[k] = q[k] + dq[k]; }
            if (mine_u) axpy(RU.acc + (size_t)su[b] * d, lam * sgn * ga[b], qi, d);
            if (mine_i) axpy(RI.acc + (size_t)sq * d, lam * sgn * ga[b], pp, d);
          }
#pragma omp barrier
      /* 6. SparseApplyAdagrad on the unique rows */
#pragma omp for schedule(static)
      for (int s = 0; s < RU.n + RI.n; ++s) {
        const int side = s >= RU.n, x = side ? s - RU.n : s;
        const rowset* R = side ? &RI : &RU;
        float* w = (side ? Q : P) + (int64_t)R->rows[x] * d;
        float* a = (side ? accQ : accP) + (int64_t)R->rows[x] * d;
        const float* gr = R->acc + (size_t)x * d;
        for (int k = 0; k < d; ++k) {
          a[k] = a[k] + gr[k] * gr[k];
          w[k] = w[k] - (h.lr * gr[k]) * (1.0f / sqrtf(a[k]));
        }
      }
#pragma omp single
      {
        rowset_clear(&RU);
        rowset_clear(&RI);
      }
    }
    free(pp); free(qi); free(qj);
  }
  rowset_free(&RU);
  rowset_free(&RI);
  free(g); free(ga); free(su); free(si); free(sj);
  free(dU); free(dI); free(G0U); free(G0I); free(denseU); free(denseI);
  return 0;
}
