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
//   sess.run([update_P, update_Q]):                 k_clean: one wavefront per UNIQUE
//     gather, (p*q)h, clip, softplus, grads,        row; its lane-groups (d/4 lanes,
//     dense l2_normalize * eps, full-table assign   float4 each) take the row's
//                                                   occurrences in parallel, sum their
//                                                   clean-loss gradients and write
//                                                   delta = eps*g/|g| for that row
//   sess.run(optimizer):                            k_adv: same pass over p+dP, q+dQ,
//     clean + adversarial fwd/bwd, dedup,           total gradient, Adagrad; the new
//     SparseApplyAdagrad                            row goes to scratch and is flushed
//                                                   by the next batch's k_clean
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
#include <rocprim/block/block_radix_sort.hpp>
#include <rocprim/block/block_scan.hpp>

#include <algorithm>
#include <cmath>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <string>
#include <thread>
#include <mutex>
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

// for the other translation units of the library (acf_ops.hip)
int acf_set_error(int code, const char* fmt, ...) {
  char buf[512];
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
// device helpers (row groups, the TF-order dot product, BPR term, RNG)
// ---------------------------------------------------------------------------
#include "acf_rows.h"

// ---------------------------------------------------------------------------
// plan kernels
// ---------------------------------------------------------------------------
// The plan sorts every occurrence by its segment (t, row) — users and items in
// one sort, items after users — with the occurrence index as tie-break so the
// order inside a segment is the occurrence order.  Two key layouts:
//   Key64: (segment << ob | occurrence) in one 64-bit key;
//   Key32: 32-bit segment key, occurrence as the sort value (fewer radix passes;
//          used when batches x rows fits 31 bits).
struct Key64 {
  const uint64_t* k;
  uint32_t ob;
  uint64_t kmask;  // clears the item bit
  __device__ uint64_t seg(int64_t x) const { return (k[x] & kmask) >> ob; }
  __device__ int32_t occ(int64_t x) const { return (int32_t)(k[x] & ((1ull << ob) - 1)); }
};
struct Key32 {
  const uint32_t* k;
  const int32_t* v;
  uint32_t kmask;
  __device__ uint64_t seg(int64_t x) const { return k[x] & kmask; }
  __device__ int32_t occ(int64_t x) const { return v[x]; }
};

template <bool PAIRS>
__global__ void k_stage(const int32_t* __restrict__ user, const int32_t* __restrict__ ipos,
                        const int32_t* __restrict__ ineg, int64_t E, int32_t B, int64_t U1,
                        int64_t I1, void* __restrict__ keys, int32_t* __restrict__ vals,
                        uint32_t ob_u, uint32_t ob_i, uint64_t item_bit, int32_t* __restrict__ err) {
  int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (x >= E) return;
  int64_t t = x / B;
  int32_t u = user[x], i = ipos[x], j = ineg[x];
  if (u < 0 || u >= U1) { atomicOr(err, 1); u = 0; }
  if (i < 0 || i >= I1) { atomicOr(err, 2); i = 0; }
  if (j < 0 || j >= I1) { atomicOr(err, 2); j = 0; }
  // [E user keys | 2E item keys]; item_bit (above both key ranges) puts every
  // item key after every user key
  if (PAIRS) {
    uint32_t* k = static_cast<uint32_t*>(keys);
    k[x] = (uint32_t)(t * U1 + u);
    k[E + 2 * x] = (uint32_t)item_bit | (uint32_t)(t * I1 + i);
    k[E + 2 * x + 1] = (uint32_t)item_bit | (uint32_t)(t * I1 + j);
    vals[x] = (int32_t)x;
    vals[E + 2 * x] = (int32_t)(2 * x);
    vals[E + 2 * x + 1] = (int32_t)(2 * x + 1);
  } else {
    uint64_t* k = static_cast<uint64_t*>(keys);
    k[x] = ((uint64_t)(t * U1 + u) << ob_u) | (uint64_t)x;
    k[E + 2 * x] = item_bit | ((uint64_t)(t * I1 + i) << ob_i) | (uint64_t)(2 * x);
    k[E + 2 * x + 1] = item_bit | ((uint64_t)(t * I1 + j) << ob_i) | (uint64_t)(2 * x + 1);
  }
}

// head flags over the sorted [E user keys | 2E item keys]
template <class KT>
__global__ void k_heads(KT ku, KT ki, int64_t E, int32_t* __restrict__ flag) {
  int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (x >= 3 * E) return;
  bool h;
  if (x < E) h = x == 0 || ku.seg(x) != ku.seg(x - 1);
  else h = x == E || ki.seg(x - E) != ki.seg(x - E - 1);
  flag[x] = h ? 1 : 0;
}

// After an inclusive scan of the head flags: unique rows, occurrence offsets,
// per-batch unique ranges, and for every triplet the slots and CSR positions of
// its occurrences.  Item side: the scan ran over users and items together,
// *sbase = user uniques.
template <class KT>
__global__ void k_compact(KT key, const int32_t* __restrict__ inc, const int32_t* __restrict__ sbase,
                          int64_t n, int64_t R, int32_t nb, int32_t* __restrict__ uniq,
                          int32_t* __restrict__ off, int32_t* __restrict__ bstart,
                          int32_t* __restrict__ tsl, int32_t* __restrict__ tpos, int32_t item_side) {
  int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (x >= n) return;
  const uint64_t seg = key.seg(x);
  const int32_t v = key.occ(x);
  const int32_t s = inc[x] - 1 - (sbase ? *sbase : 0);
  // tsl[e] = {user slot, positive-item slot, negative-item slot, -}; tpos alike
  const int64_t at = item_side ? (int64_t)(v >> 1) * 4 + 1 + (v & 1) : (int64_t)v * 4;
  tsl[at] = s;
  tpos[at] = (int32_t)x;
  const bool head = (x == 0) || key.seg(x - 1) != seg;
  if (head) {
    uniq[s] = (int32_t)(seg % (uint64_t)R);
    off[s] = (int32_t)x;
    int64_t t = (int64_t)(seg / (uint64_t)R);
    bool bhead = (x == 0) || (key.seg(x - 1) / (uint64_t)R) != (uint64_t)t;
    if (bhead) bstart[t] = s;
  }
  if (x == n - 1) {
    off[s + 1] = (int32_t)n;
    bstart[nb] = s + 1;
  }
}

// For every unique row of batch t: where its current value lives when batch t
// starts ("src").  src = row (>= 0) when no earlier batch of the plan touches
// the row; otherwise src = ~((dt << kb) | k): the row was last updated dt >= 1
// batches earlier, in that batch's local slot k (kb = slot bits of the plan).
//  - the two-kernel step reads dt = 1 rows from W scratch of batch t-1 (the
//    flush to the table happens inside batch t's first kernel) and every other
//    row from the table (pend1);
//  - the streamed step (k_stream) reads any dt from that batch's row version.
// Plans with one lane-group per slot (packed) encode dt = 1 only (binary
// search of batch t-1); one-wave-per-slot plans encode every dt (k_prev_next).
// user local slot = g - ubs[t]; item local slot = nU(t) + g - ibs[t].
// info[g] = {row, src, occurrence count | NEXT (batch t+1 touches the row too),
//            CSR offset of the first occurrence}.
#define ACF_INFO_NEXT (1 << 30)

__device__ __forceinline__ int32_t src_dt(int32_t src, int kb) {
  return src < 0 ? (int32_t)((uint32_t)(~src) >> kb) : 0;
}
__device__ __forceinline__ int32_t src_slot(int32_t src, int kb) { return (~src) & ((1 << kb) - 1); }
__device__ __forceinline__ int32_t make_src(int32_t dt, int32_t k, int kb) { return ~((dt << kb) | k); }

// src names W scratch of batch t-1 (not an older batch, not the table)
__device__ __forceinline__ bool pend1(int32_t src, int kb) { return src_dt(src, kb) == 1; }

// local slot in batch tb of the row (binary search of tb's sorted unique rows), or -1
__device__ __forceinline__ int find_local(const int32_t* __restrict__ uniq, const int32_t* __restrict__ ubs,
                                          const int32_t* __restrict__ bstart, int tb, int32_t row,
                                          int item_side) {
  int a = bstart[tb], b = bstart[tb + 1];
  while (a < b) {
    int mid = (a + b) >> 1;
    if (uniq[mid] < row) a = mid + 1; else b = mid;
  }
  if (a < bstart[tb + 1] && uniq[a] == row) {
    const int nU = ubs[tb + 1] - ubs[tb];
    return item_side ? nU + (a - bstart[tb]) : (a - bstart[tb]);
  }
  return -1;
}

// inplace (triplet-centric plans, every row updated in its table): every row is
// read from its table and nothing depends on the next batch, so no search.
__global__ void k_slot_info(const int32_t* __restrict__ uniq, const int32_t* __restrict__ off,
                            const int32_t* __restrict__ ubs, const int32_t* __restrict__ bstart,
                            int32_t n_uniq, int32_t nb, int32_t item_side, int32_t kb,
                            int4* __restrict__ info, int32_t inplace) {
  int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (g >= n_uniq || g >= bstart[nb]) return;  // bstart[nb] = unique rows of the plan
  if (inplace) {
    const int32_t row = uniq[g], o = off[g];
    info[g] = make_int4(row, row, off[g + 1] - o, o);
    return;
  }
  // batch of g: last t with bstart[t] <= g
  int lo = 0, hi = nb;  // answer in [0, nb)
  while (hi - lo > 1) {
    int mid = (lo + hi) >> 1;
    if (bstart[mid] <= g) lo = mid; else hi = mid;
  }
  const int t = lo;
  const int32_t row = uniq[g];
  int32_t s = row;
  if (t > 0) {
    const int local = find_local(uniq, ubs, bstart, t - 1, row, item_side);
    if (local >= 0) s = make_src(1, local, kb);
  }
  int32_t in_next = 0;
  if (t + 1 < nb) {
    int a = bstart[t + 1], b = bstart[t + 2];
    while (a < b) {
      int mid = (a + b) >> 1;
      if (uniq[mid] < row) a = mid + 1; else b = mid;
    }
    in_next = (a < bstart[t + 2] && uniq[a] == row) ? 1 : 0;
  }
  const int32_t o = off[g];
  info[g] = make_int4(row, s, (off[g + 1] - o) | (in_next ? ACF_INFO_NEXT : 0), o);
}

// One-wave-per-slot plans: the previous and next batch that touch each unique
// row, at any distance, from one sort of the unique (side, row, batch) keys.
// Entry x < E names user unique x, entry E + x item unique x; entries past a
// side's unique count sort last (all-ones key).  The key layout:
//   32-bit (VK32): side << (rb + tb) | row << tb | t, the entry as the value;
//   64-bit: (side << (rb + tb) | row << tb | t) << 30 | entry.
struct VKeys {
  int32_t rb, tb, k32;
  __device__ uint64_t key(int32_t side, int32_t row, int32_t t) const {
    return ((uint64_t)side << (rb + tb)) | ((uint64_t)row << tb) | (uint64_t)t;
  }
};

__device__ __forceinline__ int batch_of(const int32_t* __restrict__ bstart, int nb, int64_t g) {
  int lo = 0, hi = nb;  // last t with bstart[t] <= g
  while (hi - lo > 1) {
    int mid = (lo + hi) >> 1;
    if (bstart[mid] <= g) lo = mid; else hi = mid;
  }
  return lo;
}

__global__ void k_vkeys(const int32_t* __restrict__ uuniq, const int32_t* __restrict__ iuniq,
                        const int32_t* __restrict__ ubs, const int32_t* __restrict__ ibs, int64_t E,
                        int32_t nb, VKeys vk, void* __restrict__ keys, int32_t* __restrict__ vals) {
  const int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (x >= 3 * E) return;
  const int32_t side = x >= E ? 1 : 0;
  const int64_t g = side ? x - E : x;
  const int32_t* bs = side ? ibs : ubs;
  const bool valid = g < bs[nb];
  uint64_t k = ~0ull;
  if (valid) k = vk.key(side, (side ? iuniq : uuniq)[g], batch_of(bs, nb, g));
  if (vk.k32) {
    static_cast<uint32_t*>(keys)[x] = valid ? (uint32_t)k : ~0u;
    vals[x] = (int32_t)x;
  } else {
    static_cast<uint64_t*>(keys)[x] = valid ? (k << 30) | (uint64_t)x : ~0ull;
  }
}

// Over the sorted keys: info[g] of each unique row (src from the previous batch
// that touches it, NEXT when batch t+1 does) and nextt[t][slot] = the next batch
// that touches it (0x7fffffff: none in the plan).
__global__ void k_prev_next(const void* __restrict__ keys, const int32_t* __restrict__ vals, int64_t E,
                            VKeys vk, const int32_t* __restrict__ uoff, const int32_t* __restrict__ ioff,
                            const int32_t* __restrict__ ubs, const int32_t* __restrict__ ibs, int32_t S,
                            int32_t kb, int4* __restrict__ uinfo, int4* __restrict__ iinfo,
                            int32_t* __restrict__ nextt) {
  const int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (p >= 3 * E) return;
  const uint64_t tmask = (1ull << vk.tb) - 1;
  auto rd = [&](int64_t q, uint64_t& k, int64_t& x) {  // (side,row,t) key and entry at sorted q
    if (vk.k32) {
      const uint32_t v = static_cast<const uint32_t*>(keys)[q];
      k = v == ~0u ? ~0ull : (uint64_t)v;
      x = vals[q];
    } else {
      const uint64_t v = static_cast<const uint64_t*>(keys)[q];
      k = v == ~0ull ? ~0ull : (v >> 30);
      x = (int64_t)(v & ((1ull << 30) - 1));
    }
  };
  uint64_t k;
  int64_t x;
  rd(p, k, x);
  if (k == ~0ull) return;
  const int32_t side = x >= E ? 1 : 0;
  const int64_t g = side ? x - E : x;
  const int32_t t = (int32_t)(k & tmask);
  const uint64_t rowkey = k >> vk.tb;  // side | row
  const int32_t row = (int32_t)(rowkey & ((1ull << vk.rb) - 1));
  auto local = [&](int32_t s, int64_t gg, int32_t tt) -> int32_t {
    return s ? (ubs[tt + 1] - ubs[tt]) + (int32_t)(gg - ibs[tt]) : (int32_t)(gg - ubs[tt]);
  };
  int32_t src = row;
  if (p > 0) {
    uint64_t kp;
    int64_t xp;
    rd(p - 1, kp, xp);
    if (kp != ~0ull && (kp >> vk.tb) == rowkey) {
      const int32_t tp = (int32_t)(kp & tmask);
      src = make_src(t - tp, local(side, side ? xp - E : xp, tp), kb);
    }
  }
  int32_t tn = 0x7fffffff;
  if (p + 1 < 3 * E) {
    uint64_t kn;
    int64_t xn;
    rd(p + 1, kn, xn);
    if (kn != ~0ull && (kn >> vk.tb) == rowkey) tn = (int32_t)(kn & tmask);
  }
  const int32_t* off = side ? ioff : uoff;
  const int32_t o = off[g];
  (side ? iinfo : uinfo)[g] = make_int4(row, src, (off[g + 1] - o) | (tn == t + 1 ? ACF_INFO_NEXT : 0), o);
  nextt[(int64_t)t * S + local(side, g, t)] = tn;
}

// Occurrence record: everything one lane-group needs to process one occurrence
// of a unique row, so that a step kernel reaches the partner rows after ONE
// dependent load.  Records are written in CSR order (all occurrences) and the
// first R of each slot are also inlined at [batch][slot][r] so the kernel finds
// them by address arithmetic alone.  `gen` tags the plan that wrote a record:
// inlined records of an older plan read as absent.
struct __align__(16) OccRec {
  int32_t own_row;  // the unique row this slot updates
  int32_t own_src;  // where its value lives at batch start (see k_prev_src)
  int32_t meta;     // occurrence count | ITEM_BIT for item slots
  int32_t ovf;      // CSR index of the slot's first occurrence
  int32_t e_role;   // user slot: triplet e; item slot: 2e + role (0 pos, 1 neg)
  int32_t pa_row;   // user slot: item i;  item slot: user u
  int32_t pb_row;   // user slot: item j;  item slot: the other item of the triplet
  int32_t pa_src;
  int32_t pb_src;
  int32_t pa_slot;  // local slot of pa in batch t (for its delta) | SOLO_BIT if pa occurs once
  int32_t pb_slot;
  int32_t gen;
};
// A partner row that occurs once in the batch ("solo"): its batch-summed clean
// gradient is this occurrence's own term, so a reader can form its delta itself
// (k_stream, solo_delta) instead of waiting for the partner's wave to publish it.
#define ACF_SOLO_BIT (1 << 30)
#define ACF_SLOT_MASK (ACF_SOLO_BIT - 1)
#define ACF_ITEM_BIT (1 << 28)
#define ACF_SINGLE_BIT (1 << 29)   // the slot's only occurrence is a fused triplet
#define ACF_INPLACE_BIT (1 << 30)  // the fused triplet writes this row to the table itself
#define ACF_COUNT_MASK ((1 << 28) - 1)

// A triplet is FUSED when its user, positive and negative item each occur once
// in the batch (so i != j): its rows' batch-aggregated gradients are its own
// contributions, and the whole APR step for it runs in one lane-group with no
// batch-wide reduction (k_single).  A fused row is written straight to its table
// ("in place") unless the next batch touches it or it is pending from the
// previous batch; otherwise it goes through the W scratch like any other row.
struct FuseInfo {
  int fused, in_u, in_i, in_j;
};

__device__ __forceinline__ int info_count(const int4& f) { return f.z & (ACF_INFO_NEXT - 1); }

__device__ __forceinline__ FuseInfo fuse_info(const int4& U, const int4& I, const int4& J, int kb) {
  FuseInfo f;
  f.fused = info_count(U) == 1 && info_count(I) == 1 && info_count(J) == 1;
  f.in_u = f.fused && !pend1(U.y, kb) && !(U.z & ACF_INFO_NEXT);
  f.in_i = f.fused && !pend1(I.y, kb) && !(I.z & ACF_INFO_NEXT);
  f.in_j = f.fused && !pend1(J.y, kb) && !(J.z & ACF_INFO_NEXT);
  return f;
}

// Fused-triplet record (same 48-B shape as OccRec; fields by position):
//  a = {u, i, j, local slot of u}, b = {slot i, slot j, src u, src i},
//  c = {src j, flags (1 fused | 2 in-place u | 4 in-place i | 8 in-place j), e, gen}

// item occurrence record: own = the item's slot info, oth = the triplet's other item
__device__ __forceinline__ OccRec item_rec(const int4& own, const int4& oth, const int4& U, int32_t v,
                                           int32_t ku, int32_t k_oth, int fused, int in_place,
                                           int32_t gen) {
  OccRec r;
  r.own_row = own.x;
  r.own_src = own.y;
  r.meta = info_count(own) | ACF_ITEM_BIT | (fused ? ACF_SINGLE_BIT : 0) |
           (in_place ? ACF_INPLACE_BIT : 0);
  r.ovf = own.w;
  r.e_role = v;
  r.pa_row = U.x;
  r.pb_row = oth.x;
  r.pa_src = U.y;
  r.pb_src = oth.y;
  r.pa_slot = ku | (info_count(U) == 1 ? ACF_SOLO_BIT : 0);
  r.pb_slot = k_oth | (info_count(oth) == 1 ? ACF_SOLO_BIT : 0);
  r.gen = gen;
  return r;
}

// One thread per triplet: its user and two item occurrence records and, when
// fused, its fused-triplet record.  The first R records of a slot go inline
// only (that is the only place they are read from), later ones to the CSR.
// Hot slots of packed (one lane-group per slot) plans.  A large batch of
// Zipf-popular items holds a few rows with thousands of occurrences (10M x 5M,
// B = 65,536: the top item ~4,000), and one lane-group would sum them one pass
// after another.  A non-fused slot with more than ACF_HOT_MIN occurrences is
// therefore split into pieces of consecutive occurrences (at least
// ACF_HOT_PIECE each, at most ACF_HOT_MAXP pieces); one wave sums a piece into
// hot_part, and k_hot_combine adds a slot's pieces in piece order (fixed order:
// deterministic bits).  Each plan appends a batch's hot slots and their pieces
// with atomics; the order of the lists changes nothing but which wave does what.
#ifndef ACF_HOT_MIN
#define ACF_HOT_MIN 8
#endif
#ifndef ACF_HOT_PIECE
#define ACF_HOT_PIECE 16
#endif
#define ACF_HOT_MAXP 256

__host__ __device__ __forceinline__ int32_t hot_pieces(int32_t count) {
  const int32_t np = (count + ACF_HOT_PIECE - 1) / ACF_HOT_PIECE;
  return np < ACF_HOT_MAXP ? np : ACF_HOT_MAXP;
}

// Per-batch capacity of the hot lists: slots with > ACF_HOT_MIN of a batch's
// 3B occurrences, and sum(ceil(count / ACF_HOT_PIECE)) <= 3B / ACF_HOT_PIECE + hot slots.
__host__ __forceinline__ int32_t hot_stride_for(int32_t B) { return 3 * B / (ACF_HOT_MIN + 1) + 1; }
__host__ __forceinline__ int32_t piece_stride_for(int32_t B) { return 3 * B / ACF_HOT_PIECE + hot_stride_for(B); }

struct HotLists {
  int4* list;       // [nb][hot_stride]   {slot, pieces, piece base, count}
  int4* piece;      // [nb][piece_stride] {slot, piece, pieces, piece base}
  int32_t* cnt;     // [nb] hot slots of the batch
  int32_t* pcnt;    // [nb] pieces of the batch
  int32_t* arrive;  // [nb][piece_stride] at a hot slot's piece base: its pieces stored so far
                    // (triplet-centric combine: the slot's combine waits for all of them)
  int2* paux;       // [nb][piece_stride] beside each piece: {slot count, local CSR base | item << 31}
  int32_t hot_stride, piece_stride;
};

// Per-slot flags of packed plans (non-fused and not hot << 32 | row stays in W
// scratch), written by k_records for the slot's first occurrence (the hot
// lists likewise); scanned into the per-batch slot and write-back lists.
// csr: the slot's local CSR base | item << 31 (the triplet-centric combine's piece waves read it beside the piece)
__device__ __forceinline__ void slot_flag(uint64_t* __restrict__ sflags, const HotLists& hl, int64_t t, int32_t S,
                                          int32_t k, int32_t count, bool single, bool inplace, int32_t csr) {
  const bool hot = !single && count > ACF_HOT_MIN;
  sflags[t * S + k] = ((uint64_t)(!single && !hot) << 32) | (uint64_t)(!inplace);
  if (hot) {
    const int32_t np = hot_pieces(count);
    const int32_t h = atomicAdd(hl.cnt + t, 1);
    const int32_t base = atomicAdd(hl.pcnt + t, np);
    hl.list[t * hl.hot_stride + h] = make_int4(k, np, base, count);
    for (int32_t p = 0; p < np; ++p) {
      hl.piece[t * hl.piece_stride + base + p] = make_int4(k, p, np, base);
      hl.paux[t * hl.piece_stride + base + p] = make_int2(count, csr);
    }
  }
}

// tri (triplet-centric list plans, see k_tri_*): every row that occurs once in
// its batch is "single" (its triplet's lane-group steps it: SINGLE bit, and
// INPLACE by fuse_info's rule), and every triplet gets a record in trec with
// the single bits 16 / 32 / 64 (u / i / j) beside the fused / in-place flags.
// the records of triplet e of batch t (its user slots start at ub0, its item slots
// at ib0, nU user slots); shared by k_records and the one-workgroup shard plan
__device__ __forceinline__ void records_one(int64_t e, int32_t t, int32_t ub0, int32_t nU, int32_t ib0, int32_t S,
                                            int32_t R, int32_t gen, int32_t kb, int32_t no_fuse, int32_t tri,
                                            const int4* tsl, const int4* tpos, const int4* uinfo, const int4* iinfo,
                                            OccRec* urec, OccRec* irec, OccRec* inl, OccRec* trec,
                                            uint64_t* sflags, const HotLists& hl) {
  const int4 sl = tsl[e], ps = tpos[e];
  const int4 U = uinfo[sl.x], I = iinfo[sl.y], J = iinfo[sl.z];
  const int32_t k = sl.x - ub0, ki = nU + (sl.y - ib0), kj = nU + (sl.z - ib0);
  FuseInfo f = fuse_info(U, I, J, kb);
  if (no_fuse) f.fused = f.in_u = f.in_i = f.in_j = 0;  // shard mode: item counts are rank-local
  const int su = info_count(U) == 1, si = info_count(I) == 1, sj = info_count(J) == 1;
  if (tri) {  // single rows step in their triplet; in place by the fused rule
    f.in_u = su && !pend1(U.y, kb) && !(U.z & ACF_INFO_NEXT);
    f.in_i = si && !pend1(I.y, kb) && !(I.z & ACF_INFO_NEXT);
    f.in_j = sj && !pend1(J.y, kb) && !(J.z & ACF_INFO_NEXT);
  }
  const int xu = tri ? su : f.fused, xi = tri ? si : f.fused, xj = tri ? sj : f.fused;
  OccRec r;
  r.own_row = U.x;
  r.own_src = U.y;
  r.meta = info_count(U) | (xu ? ACF_SINGLE_BIT : 0) | (f.in_u ? ACF_INPLACE_BIT : 0);
  r.ovf = U.w;
  r.e_role = (int32_t)e;
  r.pa_row = I.x;
  r.pb_row = J.x;
  r.pa_src = I.y;
  r.pb_src = J.y;
  r.pa_slot = ki | (info_count(I) == 1 ? ACF_SOLO_BIT : 0);
  r.pb_slot = kj | (info_count(J) == 1 ? ACF_SOLO_BIT : 0);
  r.gen = gen;
  // the CSR records (occurrences past the first R) are read by the slot kernels
  // only: the triplet-centric step reads a shared slot's first record (its
  // combine) and trec -- a single row's slot is read by nothing (its triplet
  // steps it from trec), so tri plans write neither its record nor its slot
  // flags (0, the cleared value: not listed, written in place), ~60% of
  // k_records' scattered 48-B stores at configs[4]
  const int64_t base = (int64_t)t * S;
  int32_t rr = ps.x - U.w;
  if (rr < R) { if (!(tri && su)) inl[(base + k) * R + rr] = r; }
  else if (!tri) urec[ps.x] = r;
  const OccRec ri = item_rec(I, J, U, (int32_t)(2 * e), k, kj, xi, f.in_i, gen);
  rr = ps.y - I.w;
  if (rr < R) { if (!(tri && si)) inl[(base + ki) * R + rr] = ri; }
  else if (!tri) irec[ps.y] = ri;
  const OccRec rj = item_rec(J, I, U, (int32_t)(2 * e + 1), k, ki, xj, f.in_j, gen);
  rr = ps.z - J.w;
  if (rr < R) { if (!(tri && sj)) inl[(base + kj) * R + rr] = rj; }
  else if (!tri) irec[ps.z] = rj;
  if (sflags) {  // packed plans: the slot flags and hot lists, from each slot's first occurrence
    // local CSR bases (users: t * B + x, items: t * 2B + x; t is 0 in the shard plan's batch)
    const int32_t Bt = S / 3;
    if (ps.x == U.w && !(tri && su)) slot_flag(sflags, hl, t, S, k, info_count(U), xu, f.in_u, U.w - (int32_t)t * Bt);
    if (ps.y == I.w && !(tri && si))
      slot_flag(sflags, hl, t, S, ki, info_count(I), xi, f.in_i, (I.w - (int32_t)t * 2 * Bt) | (int32_t)0x80000000);
    if (ps.z == J.w && !(tri && sj))
      slot_flag(sflags, hl, t, S, kj, info_count(J), xj, f.in_j, (J.w - (int32_t)t * 2 * Bt) | (int32_t)0x80000000);
  }
  if (f.fused || tri) {  // other triplets' records read as absent (older generation)
    OccRec q;
    q.own_row = U.x; q.own_src = I.x; q.meta = J.x; q.ovf = k;
    q.e_role = ki; q.pa_row = kj; q.pb_row = U.y; q.pa_src = I.y;
    q.pb_src = J.y;
    q.pa_slot = (f.fused ? 1 : 0) | (f.in_u ? 2 : 0) | (f.in_i ? 4 : 0) | (f.in_j ? 8 : 0) |
                (su ? 16 : 0) | (si ? 32 : 0) | (sj ? 64 : 0);
    q.pb_slot = (int32_t)e; q.gen = gen;
    trec[e] = q;
  }
}

__global__ void k_records(int64_t E, int32_t B, int32_t S, int32_t R, int32_t gen, int32_t kb, int32_t no_fuse,
                          int32_t tri,
                          const int4* __restrict__ tsl, const int4* __restrict__ tpos,
                          const int4* __restrict__ uinfo, const int4* __restrict__ iinfo,
                          const int32_t* __restrict__ ubs, const int32_t* __restrict__ ibs,
                          OccRec* __restrict__ urec, OccRec* __restrict__ irec,
                          OccRec* __restrict__ inl, OccRec* __restrict__ trec,
                          int32_t* __restrict__ gen_ptr, uint64_t* __restrict__ sflags, HotLists hl) {
  const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (e == 0) *gen_ptr = gen;
  if (e >= E) return;
  const int32_t t = (int32_t)(e / B);
  records_one(e, t, ubs[t], ubs[t + 1] - ubs[t], ibs[t], S, R, gen, kb, no_fuse, tri, tsl, tpos, uinfo, iinfo,
              urec, irec, inl, trec, sflags, hl);
}

__global__ void k_slot_lists(const uint64_t* __restrict__ flags, const uint64_t* __restrict__ incl,
                             int64_t n, int32_t S, int32_t* __restrict__ slot_list,
                             int32_t* __restrict__ flush_list, int32_t* __restrict__ slot_cnt,
                             int32_t* __restrict__ flush_cnt) {
  const int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (x >= n) return;
  const int64_t t = x / S;
  const int32_t k = (int32_t)(x - t * S);
  const uint64_t base = t > 0 ? incl[t * S - 1] : 0;
  const uint64_t f = flags[x], v = incl[x] - base;  // inclusive counts inside batch t
  if (f >> 32) slot_list[t * S + (int64_t)(v >> 32) - 1] = k;
  if (f & 0xFFFFFFFFull) flush_list[t * S + (int64_t)(v & 0xFFFFFFFFull) - 1] = k;
  if (k == S - 1) {
    slot_cnt[t] = (int32_t)(v >> 32);
    flush_cnt[t] = (int32_t)(v & 0xFFFFFFFFull);
  }
}

// Streamed-step task lists (one-wave-per-slot plans): per batch its non-fused
// slots (slot order), then the groups of `opw` consecutive triplets that hold a
// fused one (as S + group).  Flags over [nb][S + G], scanned into the lists.
__global__ void k_task_flags(const OccRec* __restrict__ inl, const OccRec* __restrict__ trec, int64_t n,
                             int32_t S, int32_t G, int32_t B, int32_t R, int32_t opw, int32_t gen,
                             int32_t* __restrict__ flags) {
  const int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (x >= n) return;
  const int64_t t = x / (S + G);
  const int32_t y = (int32_t)(x - t * (S + G));
  int32_t f = 0;
  if (y < S) {
    const OccRec* r = inl + (t * S + y) * R;
    f = r->gen == gen && (r->meta & ACF_COUNT_MASK) != 0 && !(r->meta & ACF_SINGLE_BIT);
  } else {
    const int32_t b0 = (y - S) * opw, b1 = min(b0 + opw, B);
    for (int32_t b = b0; b < b1; ++b) {
      const OccRec* q = trec + t * B + b;
      f |= (q->gen == gen && (q->pa_slot & 1)) ? 1 : 0;
    }
  }
  flags[x] = f;
}

__global__ void k_task_list(const int32_t* __restrict__ flags, const int32_t* __restrict__ incl, int64_t n,
                            int32_t stride, int32_t* __restrict__ list, int32_t* __restrict__ cnt) {
  const int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (x >= n) return;
  const int64_t t = x / stride;
  const int32_t y = (int32_t)(x - t * stride);
  const int32_t base = t > 0 ? incl[t * stride - 1] : 0;
  if (flags[x]) list[t * stride + incl[x] - base - 1] = y;
  if (y == stride - 1) cnt[t] = incl[x] - base;
}

#include "acf_hplan.h"  // the hash plan (k_hplan_*): DESIGN.md §3

// diagnostic build (-DACF_DIAG): s_memrealtime stamps of the plan and step kernels
#ifdef ACF_DIAG
__device__ uint64_t* g_stamps = nullptr;
__device__ int g_stamp_launch = 0;
__device__ int g_stamp_cap = 0;
#define STAMP(launch, wave, i)                                                       \
  do {                                                                               \
    uint64_t t_;                                                                     \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
    if (g_stamps && (threadIdx.x & 63) == 0 && (wave) < g_stamp_cap)                 \
      g_stamps[((int64_t)(launch) * g_stamp_cap + (wave)) * 8 + (i)] = t_;          \
  } while (0)
#define CLOCKSTAMP(launch, wave, i)                                                  \
  do {                                                                               \
    uint64_t t_;                                                                     \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");     \
    if (g_stamps && (threadIdx.x & 63) == 0 && (wave) < g_stamp_cap)                 \
      g_stamps[((int64_t)(launch) * g_stamp_cap + (wave)) * 8 + (i)] = t_;          \
  } while (0)
#else
#define CLOCKSTAMP(launch, wave, i) \
  do {                              \
  } while (0)
#define STAMP(launch, wave, i) \
  do {                         \
  } while (0)
#endif

// ---------------------------------------------------------------------------
// Batch-local plan (one-wave-per-slot plans, B <= 1024): the same records,
// task lists and next-batch table as the sort plan above, in TWO launches with
// one workgroup per batch instead of ~30 launches of device-wide sorts/scans.
//  - k_bplan_sort: the batch's 3B occurrences sorted by (side, row) in LDS
//    (rocPRIM block radix sort, stable: occurrence order inside a row), its
//    unique rows, their CSR starts, each occurrence's (slot, rank); each unique
//    row marks batch t in its row's batch bitmap and records its local slot.
//  - k_bplan_build: per unique row, the previous / next batch that touches the
//    row from the bitmap (any distance: the streamed step's version source) and
//    the previous batch's local slot; then k_records' occurrence / fused-triplet
//    records and k_task_flags/k_task_list's task list, from LDS.
// The occurrence order, slot order (users by row, then items by row) and CSR
// positions (t*B + position in the sorted user part, t*2B + position in the
// item part) are the sort plan's, so the records are bit-identical
// (test_batch_plan_matches_sort_plan).  The bitmaps come in two buffers by
// plan generation parity: a plan sets bits in one and clears the other, which
// the previous plan used.
// ---------------------------------------------------------------------------
struct BPlanArgs {
  const int32_t* user;
  const int32_t* ipos;
  const int32_t* ineg;
  int64_t U1, I1;
  int32_t B, S, nb, rb, kb, W, nbs;  // nbs: batch stride of slot_of (max batches)
  int32_t R, opw, stride, gen;
  unsigned long long* mask;        // [U1 + I1][W] batches touching each row (this plan)
  unsigned long long* mask_clear;  // the other bitmap buffer: cleared here
  int64_t clear_words;
  uint16_t* slot_of;  // [U1 + I1][nbs] local slot of the row in batch t (valid where mask has t)
  uint32_t* bkey;     // [nb][S] sorted unique keys (side << rb | row)
  int32_t* bstart;    // [nb][S + 1] CSR start of each unique row in the sorted batch
  int32_t* bocc;      // [nb][S] occurrence o -> slot | rank << 16
  int2* bn;           // [nb] {unique rows, unique user rows}
  int32_t* berr;      // [nb] range-check bits of the batch
  int32_t* err;       // err[0] = OR of berr
  int32_t* gen_ptr;
  OccRec *urec, *irec, *inl, *trec;
  int32_t* nextt;
  int32_t* task_list;
  int32_t* task_cnt;
  int2* final_list;   // slots no later batch of the plan touches (k_stream's tail write-back)
  int32_t* final_cnt;
};

// Workgroup barrier for LDS data only.  __syncthreads() also waits for every
// outstanding global store and atomic of the wave (vmcnt(0)): after a phase of
// scattered global writes that is a full memory round trip (≈2-4 us per barrier
// in the plan kernels, tools/diag_plan.py) for data no other thread of the
// workgroup reads back.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int BS, int IPT>
__global__ void __launch_bounds__(BS) k_bplan_sort(BPlanArgs p) {
  constexpr int N = BS * IPT;
  using Sort = rocprim::block_radix_sort<uint32_t, BS, IPT, int32_t>;
  using Scan = rocprim::block_scan<int32_t, BS>;
  __shared__ union {
    typename Sort::storage_type sort;
    struct {
      uint32_t key[N];
      int32_t val[N];
      int32_t start[N + 1];
    } a;
  } sm;
  __shared__ typename Scan::storage_type scan_st;
  __shared__ int32_t s_err, s_nu;
  const int t = blockIdx.x, tid = threadIdx.x, B = p.B, S3 = 3 * B;
  STAMP(t, tid >> 6, 0);
  if (tid == 0) { s_err = 0; s_nu = -1; }
  if (t == 0 && tid == 0) *p.final_cnt = 0;  // k_bplan_build appends to it
  const uint32_t side_bit = 1u << p.rb;
  uint32_t keys[IPT];
  int32_t vals[IPT];
  int err = 0;
  // all loads first, the range checks after them: a check right behind its load
  // made the compiler wait for each load in turn (IPT serial round trips)
  int32_t raw[IPT];
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const int o = tid * IPT + k;  // occurrence: users [0, B), items B + 2e + role
    raw[k] = 0;
    if (o < B) {
      raw[k] = p.user[(int64_t)t * B + o];
    } else if (o < S3) {
      const int v = o - B;
      raw[k] = ((v & 1) ? p.ineg : p.ipos)[(int64_t)t * B + (v >> 1)];
    }
  }
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const int o = tid * IPT + k;
    uint32_t key = ~0u;  // padding sorts after every key (stable: after equal ones too)
    int32_t x = raw[k];
    if (o < B) {
      if (x < 0 || x >= p.U1) { err |= 1; x = 0; }
      key = (uint32_t)x;
    } else if (o < S3) {
      if (x < 0 || x >= p.I1) { err |= 2; x = 0; }
      key = side_bit | (uint32_t)x;
    }
    keys[k] = key;
    vals[k] = o;
  }
  __syncthreads();
  STAMP(t, tid >> 6, 1);
  if (err) atomicOr(&s_err, err);
  Sort().sort(keys, vals, sm.sort, 0, p.rb + 1);
  __syncthreads();
  STAMP(t, tid >> 6, 2);
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    sm.a.key[tid * IPT + k] = keys[k];
    sm.a.val[tid * IPT + k] = vals[k];
  }
  __syncthreads();
  int cnt = 0;
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const int q = tid * IPT + k;
    cnt += (q < S3 && (q == 0 || keys[k] != sm.a.key[q - 1])) ? 1 : 0;
  }
  int32_t excl = 0, total = 0;
  Scan().exclusive_scan(cnt, excl, 0, total, scan_st);
  STAMP(t, tid >> 6, 3);
  int32_t sl[IPT];
  int32_t s = excl - 1;
  const int64_t rbase = (int64_t)t * p.S;
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const int q = tid * IPT + k;
    sl[k] = -1;
    if (q >= S3) continue;
    const uint32_t key = keys[k];
    if (q == 0 || key != sm.a.key[q - 1]) {
      ++s;
      sm.a.start[s] = q;
      const int side = (key & side_bit) ? 1 : 0;
      const int64_t row = (int64_t)(key & (side_bit - 1));
      const int64_t rid = side ? p.U1 + row : row;
      p.bkey[rbase + s] = key;
      p.bstart[(int64_t)t * (p.S + 1) + s] = q;
      p.slot_of[rid * p.nbs + t] = (uint16_t)s;
      atomicOr(p.mask + rid * p.W + (t >> 6), 1ull << (t & 63));
      if (side && (q == 0 || !(sm.a.key[q - 1] & side_bit))) s_nu = s;
    }
    sl[k] = s;
  }
  lds_barrier();  // run starts and s_nu (LDS); the row writes above stay in flight
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const int q = tid * IPT + k;
    if (q < S3) p.bocc[rbase + vals[k]] = sl[k] | ((q - sm.a.start[sl[k]]) << 16);
  }
  if (tid == 0) {
    p.bstart[(int64_t)t * (p.S + 1) + total] = S3;
    p.bn[t] = make_int2(total, s_nu < 0 ? total : s_nu);
    p.berr[t] = s_err;
  }
  STAMP(t, tid >> 6, 4);
}

// ---------------------------------------------------------------------------
// One-workgroup shard plan (shard mode, one batch of B <= 1,024 triplets:
// distributed.ShardedAPR's per-step plan).  It writes what the device-wide sort
// plan writes for nb = 1 -- unique rows and CSR offsets, slot info, the triplets'
// slots and CSR positions, occurrence records, slot flags, hot lists and the
// slot / write-back lists -- in ONE launch instead of ~17 (stage, radix sort,
// head flags, two scans, compaction, slot info, four clears, records, list
// scan), which a captured split step replays every step.  Same keys and the
// same stable order (users by row, then items by row, occurrence order inside a
// row), so the records are the sort plan's bit for bit
// (test_shard_plan_small_matches_sort_plan).
// ---------------------------------------------------------------------------
struct SPlanArgs {
  const int32_t* user;
  const int32_t* ipos;
  const int32_t* ineg;
  int64_t U1, I1;
  int32_t B, rb, kb, gen;
  int32_t *uuniq, *uoff, *ubs, *iuniq, *ioff, *ibs;
  int32_t *tsl, *tpos;  // [E][4]
  int4 *uinfo, *iinfo;
  OccRec *urec, *irec, *inl, *trec;
  int32_t *gen_ptr, *err;
  uint64_t* sflags;
  HotLists hl;
  int32_t *slot_list, *flush_list, *slot_cnt, *flush_cnt;
};

template <int BS, int IPT>
__global__ void __launch_bounds__(BS) k_shard_plan(SPlanArgs p) {
  constexpr int N = BS * IPT;
  using Sort = rocprim::block_radix_sort<uint32_t, BS, IPT, int32_t>;
  using Scan = rocprim::block_scan<int32_t, BS>;
  using Scan64 = rocprim::block_scan<uint64_t, BS>;
  __shared__ union {
    typename Sort::storage_type sort;
    struct {
      uint32_t key[N];
      int32_t start[N + 1];
    } a;
    typename Scan64::storage_type scan64;
  } sm;
  __shared__ typename Scan::storage_type scan_st;
  __shared__ int32_t s_err, s_nu;
  const int tid = threadIdx.x, B = p.B, S3 = 3 * B;
  // what the sort plan clears: slot flags, inline records (shard plans), hot counters
  for (int x = tid; x < S3; x += BS) {
    p.sflags[x] = 0;
    p.inl[x] = OccRec{};
  }
  for (int x = tid; x < p.hl.piece_stride; x += BS) p.hl.arrive[x] = 0;
  if (tid == 0) {
    p.hl.cnt[0] = 0;
    p.hl.pcnt[0] = 0;
    *p.gen_ptr = p.gen;
    s_err = 0;
    s_nu = 0;
  }
  // keys: users [0, B) by row, items B + 2e + role after them (side bit)
  const uint32_t side_bit = 1u << p.rb;
  uint32_t keys[IPT];
  int32_t vals[IPT], raw[IPT];
  int err = 0;
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const int o = tid * IPT + k;
    raw[k] = 0;
    if (o < B) {
      raw[k] = p.user[o];
    } else if (o < S3) {
      const int v = o - B;
      raw[k] = ((v & 1) ? p.ineg : p.ipos)[v >> 1];
    }
  }
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const int o = tid * IPT + k;
    uint32_t key = ~0u;  // padding sorts after every key (stable: after equal ones too)
    int32_t x = raw[k];
    if (o < B) {
      if (x < 0 || x >= p.U1) { err |= 1; x = 0; }
      key = (uint32_t)x;
    } else if (o < S3) {
      if (x < 0 || x >= p.I1) { err |= 2; x = 0; }
      key = side_bit | (uint32_t)x;
    }
    keys[k] = key;
    vals[k] = o;
  }
  __syncthreads();
  if (err) atomicOr(&s_err, err);
  Sort().sort(keys, vals, sm.sort, 0, p.rb + 1);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < IPT; ++k) sm.a.key[tid * IPT + k] = keys[k];
  __syncthreads();
  int cnt = 0;
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const int q = tid * IPT + k;
    cnt += (q < S3 && (q == 0 || keys[k] != sm.a.key[q - 1])) ? 1 : 0;
  }
  int32_t excl = 0, total = 0;
  Scan().exclusive_scan(cnt, excl, 0, total, scan_st);
  int32_t sl[IPT];
  int32_t s = excl - 1;
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const int q = tid * IPT + k;
    sl[k] = -1;
    if (q >= S3) continue;
    if (q == 0 || keys[k] != sm.a.key[q - 1]) {
      ++s;
      sm.a.start[s] = q;
      if (q == B) s_nu = s;  // position B holds the first item occurrence: a head
    }
    sl[k] = s;
  }
  if (tid == 0) sm.a.start[total] = S3;
  __syncthreads();
  const int nU = s_nu, nI = total - nU;
  // unique rows, CSR offsets and slot info (user part [0, B), item part [0, 2B));
  // every triplet's slots and CSR positions
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const int q = tid * IPT + k;
    if (q >= S3) continue;
    const int32_t sk = sl[k];
    const int32_t row = (int32_t)(keys[k] & (side_bit - 1));
    if (sm.a.start[sk] == q) {
      const int32_t c = sm.a.start[sk + 1] - q;
      if (q < B) {
        p.uuniq[sk] = row;
        p.uoff[sk] = q;
        p.uinfo[sk] = make_int4(row, row, c, q);
      } else {
        p.iuniq[sk - nU] = row;
        p.ioff[sk - nU] = q - B;
        p.iinfo[sk - nU] = make_int4(row, row, c, q - B);
      }
    }
    const int o = vals[k];
    if (o < B) {
      p.tsl[o * 4] = sk;
      p.tpos[o * 4] = q;
    } else {
      const int v = o - B;
      const int at = (v >> 1) * 4 + 1 + (v & 1);
      p.tsl[at] = sk - nU;
      p.tpos[at] = q - B;
    }
  }
  if (tid == 0) {
    p.uoff[nU] = B;
    p.ioff[nI] = 2 * B;
    p.ubs[0] = 0;
    p.ubs[1] = nU;
    p.ibs[0] = 0;
    p.ibs[1] = nI;
    *p.err = s_err;
  }
  __syncthreads();  // the slot info and triplet slots above, for the records
  for (int e = tid; e < B; e += BS)
    records_one(e, 0, 0, nU, 0, S3, 1, p.gen, p.kb, 1, 0, reinterpret_cast<const int4*>(p.tsl),
                reinterpret_cast<const int4*>(p.tpos), p.uinfo, p.iinfo, p.urec, p.irec, p.inl, p.trec,
                p.sflags, p.hl);
  __syncthreads();  // the slot flags, for the lists
  uint64_t f[IPT], inc[IPT];
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const int x = tid * IPT + k;
    f[k] = x < S3 ? p.sflags[x] : 0ull;
  }
  Scan64().inclusive_scan(f, inc, sm.scan64, rocprim::plus<uint64_t>());
#pragma unroll
  for (int k = 0; k < IPT; ++k) {
    const int x = tid * IPT + k;
    if (x >= S3) continue;
    if (f[k] >> 32) p.slot_list[(inc[k] >> 32) - 1] = x;
    if (f[k] & 0xFFFFFFFFull) p.flush_list[(inc[k] & 0xFFFFFFFFull) - 1] = x;
    if (x == S3 - 1) {
      *p.slot_cnt = (int32_t)(inc[k] >> 32);
      *p.flush_cnt = (int32_t)(inc[k] & 0xFFFFFFFFull);
    }
  }
}

template <int BS, int MAXB>
__global__ void __launch_bounds__(BS) k_bplan_build(BPlanArgs p) {
  using Scan = rocprim::block_scan<int32_t, BS>;
  __shared__ int4 info[3 * MAXB];
  __shared__ uint8_t single[3 * MAXB];
  __shared__ uint8_t gflag[MAXB];
  __shared__ typename Scan::storage_type scan_st;
  __shared__ int32_t s_fin, s_fbase;
  const int t = blockIdx.x, tid = threadIdx.x, B = p.B, S = p.S;
  const int G = (B + p.opw - 1) / p.opw;
  STAMP(t, 16 + (tid >> 6), 0);
  if (tid == 0) s_fin = 0;
  const int2 n = p.bn[t];
  const int64_t rbase = (int64_t)t * S;
  // the triplet's occurrence slots, loaded now (k_bplan_sort wrote them): off
  // the dependent chain of the slot pass below (B <= MAXB <= BS: one triplet per thread)
  int32_t ou = 0, oi = 0, oj = 0;
  if (tid < B) {
    ou = p.bocc[rbase + tid];
    oi = p.bocc[rbase + B + 2 * tid];
    oj = p.bocc[rbase + B + 2 * tid + 1];
  }
  // per unique row: key and CSR bounds, then the row's batch bitmap word, then
  // the previous batch's local slot.  The SPT slots of a thread go through each
  // stage together, so their dependent loads overlap (three round trips, not 3 SPT).
  constexpr int SPT = (3 * MAXB + BS - 1) / BS;
  const uint32_t side_bit = 1u << p.rb;
  uint32_t key[SPT];
  int32_t st[SPT], en[SPT];
  unsigned long long mw[SPT];
#pragma unroll
  for (int q = 0; q < SPT; ++q) {
    const int s = tid + q * BS;
    if (s < S) single[s] = 0;
    if (s < n.x) {
      key[q] = p.bkey[rbase + s];
      st[q] = p.bstart[(int64_t)t * (S + 1) + s];
      en[q] = p.bstart[(int64_t)t * (S + 1) + s + 1];
    }
  }
  auto rid_of = [&](uint32_t k) -> int64_t {
    const int32_t row = (int32_t)(k & (side_bit - 1));
    return (k & side_bit) ? p.U1 + row : (int64_t)row;
  };
  STAMP(t, 16 + (tid >> 6), 1);
#pragma unroll
  for (int q = 0; q < SPT; ++q)
    if (tid + q * BS < n.x) mw[q] = p.mask[rid_of(key[q]) * p.W + (t >> 6)];
  int32_t tp[SPT], prev_slot[SPT], tn[SPT];
#pragma unroll
  for (int q = 0; q < SPT; ++q) {
    tp[q] = -1;
    tn[q] = 0x7fffffff;
    if (tid + q * BS >= n.x) continue;
    const unsigned long long* m = p.mask + rid_of(key[q]) * p.W;
    // previous batch touching the row: highest bit below t
    int w = t >> 6;
    unsigned long long bits = mw[q] & ((1ull << (t & 63)) - 1);
    while (!bits && w > 0) bits = m[--w];
    if (bits) tp[q] = w * 64 + 63 - __clzll((long long)bits);
    // next batch touching the row: lowest bit above t
    w = t >> 6;
    bits = (t & 63) == 63 ? 0ull : (mw[q] & ~((2ull << (t & 63)) - 1));
    const int wl = (p.nb - 1) >> 6;
    while (!bits && w < wl) bits = m[++w];
    if (bits) tn[q] = w * 64 + __ffsll((long long)bits) - 1;
  }
  STAMP(t, 16 + (tid >> 6), 2);
#pragma unroll
  for (int q = 0; q < SPT; ++q)
    if (tp[q] >= 0) prev_slot[q] = p.slot_of[rid_of(key[q]) * p.nbs + tp[q]];
#pragma unroll
  for (int q = 0; q < SPT; ++q) {
    const int s = tid + q * BS;
    if (s >= n.x) continue;
    const int side = (key[q] & side_bit) ? 1 : 0;
    const int32_t row = (int32_t)(key[q] & (side_bit - 1));
    const int32_t cnt = en[q] - st[q];
    const int32_t ovf = side ? t * 2 * B + st[q] - B : t * B + st[q];
    const int32_t src = tp[q] >= 0 ? make_src(t - tp[q], prev_slot[q], p.kb) : row;
    info[s] = make_int4(row, src, cnt | (tn[q] == t + 1 ? ACF_INFO_NEXT : 0), ovf);
  }
  for (int g = tid; g < G; g += BS) gflag[g] = 0;
  lds_barrier();  // info (LDS); the nextt stores stay in flight
  // final slots (no later batch of the plan touches the row): their place in
  // this batch's share of the final-slot list
  int32_t fidx[SPT];
#pragma unroll
  for (int q = 0; q < SPT; ++q) {
    fidx[q] = -1;
    if (tid + q * BS < n.x && tn[q] == 0x7fffffff) fidx[q] = atomicAdd(&s_fin, 1);
  }
  const int gen = p.gen;
  STAMP(t, 16 + (tid >> 6), 3);
  static_assert(MAXB <= BS, "k_bplan_build: one triplet per thread");
  // records: formed now (the fused flags feed the task list), stored after it,
  // so no barrier waits for them
  OccRec r, ri, rj, q;
  int64_t ar = 0, ai = 0, aj = 0;  // destinations: >= 0 inline index, < 0 CSR index - 1
  bool fused = false;
  int64_t e = 0;
  if (tid < B) {
    const int b = tid;
    e = (int64_t)t * B + b;
    const int32_t k = ou & 0xFFFF, ki = oi & 0xFFFF, kj = oj & 0xFFFF;
    const int4 U = info[k], I = info[ki], J = info[kj];
    const FuseInfo f = fuse_info(U, I, J, p.kb);
    r.own_row = U.x;
    r.own_src = U.y;
    r.meta = info_count(U) | (f.fused ? ACF_SINGLE_BIT : 0) | (f.in_u ? ACF_INPLACE_BIT : 0);
    r.ovf = U.w;
    r.e_role = (int32_t)e;
    r.pa_row = I.x;
    r.pb_row = J.x;
    r.pa_src = I.y;
    r.pb_src = J.y;
    r.pa_slot = ki | (info_count(I) == 1 ? ACF_SOLO_BIT : 0);
    r.pb_slot = kj | (info_count(J) == 1 ? ACF_SOLO_BIT : 0);
    r.gen = gen;
    int32_t rr = ou >> 16;
    ar = rr < p.R ? (rbase + k) * p.R + rr : -1 - ((int64_t)U.w + rr);
    ri = item_rec(I, J, U, (int32_t)(2 * e), k, kj, f.fused, f.in_i, gen);
    rr = oi >> 16;
    ai = rr < p.R ? (rbase + ki) * p.R + rr : -1 - ((int64_t)I.w + rr);
    rj = item_rec(J, I, U, (int32_t)(2 * e + 1), k, ki, f.fused, f.in_j, gen);
    rr = oj >> 16;
    aj = rr < p.R ? (rbase + kj) * p.R + rr : -1 - ((int64_t)J.w + rr);
    fused = f.fused;
    if (f.fused) {
      q.own_row = U.x; q.own_src = I.x; q.meta = J.x; q.ovf = k;
      q.e_role = ki; q.pa_row = kj; q.pb_row = U.y; q.pa_src = I.y;
      q.pb_src = J.y;
      q.pa_slot = 1 | (f.in_u ? 2 : 0) | (f.in_i ? 4 : 0) | (f.in_j ? 8 : 0);
      q.pb_slot = (int32_t)e; q.gen = gen;
      single[k] = single[ki] = single[kj] = 1;  // the fused triplet's slots are its own
      gflag[b / p.opw] = 1;
    }
  }
  lds_barrier();
  STAMP(t, 16 + (tid >> 6), 4);
  // the batch's share of the final-slot list: the atomic stays in flight over
  // the task-list scans below (they wait on LDS only)
  int32_t fret = 0;
  if (tid == 0 && s_fin > 0) fret = atomicAdd(p.final_cnt, s_fin);
  // task list: the non-fused slots in slot order, then the groups holding a fused triplet
  int32_t base = 0;
  for (int y0 = 0; y0 < S + G; y0 += BS) {
    const int y = y0 + tid;
    int32_t f = 0;
    if (y < S) f = (y < n.x && !single[y]) ? 1 : 0;
    else if (y < S + G) f = gflag[y - S];
    int32_t excl = 0, tot = 0;
    Scan().exclusive_scan(f, excl, 0, tot, scan_st);
    if (f) p.task_list[(int64_t)t * p.stride + base + excl] = y;
    base += tot;
    lds_barrier();  // scan storage reuse
  }
  STAMP(t, 16 + (tid >> 6), 5);
  if (tid == 0) s_fbase = fret;
  lds_barrier();
  // every global store of the kernel from here on: on gfx950 vmcnt counts stores
  // too, so an earlier store would have held up the loads the phases above wait for
#pragma unroll
  for (int q = 0; q < SPT; ++q) {
    const int s = tid + q * BS;
    if (s < S) p.nextt[rbase + s] = s < n.x ? tn[q] : 0;  // 0: no row, never written back
    if (fidx[q] >= 0)
      p.final_list[s_fbase + fidx[q]] =
          make_int2((int32_t)(rbase + s), (int32_t)(key[q] & (side_bit - 1)) | ((key[q] & side_bit) ? (int32_t)0x80000000 : 0));
  }
  if (tid < B) {
    (ar >= 0 ? p.inl[ar] : p.urec[-1 - ar]) = r;
    (ai >= 0 ? p.inl[ai] : p.irec[-1 - ai]) = ri;
    (aj >= 0 ? p.inl[aj] : p.irec[-1 - aj]) = rj;
    if (fused) p.trec[e] = q;
  }
  if (tid == 0) {
    p.task_cnt[t] = base;
    if (t == 0) {
      int32_t e = 0;
      for (int x = 0; x < p.nb; ++x) e |= p.berr[x];
      p.err[0] = e;
      *p.gen_ptr = gen;
    }
  }
  // clear the other bitmap buffer (used by the previous plan), a stripe per batch
  const int64_t w0 = p.clear_words * t / p.nb, w1 = p.clear_words * (t + 1) / p.nb;
  for (int64_t x = w0 + tid; x < w1; x += BS) p.mask_clear[x] = 0ull;
  STAMP(t, 16 + (tid >> 6), 6);
}

// ---------------------------------------------------------------------------
// Diagnostic build only (-DACF_DIAG, libacf_apr_diag.so): per-wave
// s_memrealtime stamps (100 MHz) to locate latency inside the step kernels.
// The product library compiles every STAMP() to nothing.
// ---------------------------------------------------------------------------

// ---------------------------------------------------------------------------
// step kernels: one wavefront per unique row ("slot") of the batch.  The 64
// lanes form OPW = 64/LPR lane-groups; group g takes occurrences g, g+OPW, ...
// of the slot, so the gathers of a popular row's occurrences are in flight
// together; the groups' partial sums are then added by a fixed butterfly.
//
// Table updates never go to the tables inside the batch that computes them:
// the Adagrad result of batch t goes to W scratch wnew[t%2][slot], and batch
// t+1's first kernel (a) reads rows that batch t touched from there (the plan's
// src encoding) and (b) flushes them to the tables.  So every kernel reads a
// consistent snapshot without a grid barrier, and a batch costs 2 kernels (APR)
// or 1 kernel (BPR).
// ---------------------------------------------------------------------------
struct StepArgs {
  float* P;
  float* Q;
  float* accP;
  float* accQ;
  const OccRec* inl;   // [nb][S][R]
  const OccRec* urec;  // CSR, user occurrences
  const OccRec* irec;  // CSR, item occurrences
  const OccRec* trec;  // [E] fused-triplet records (see fuse_info)
  float* g0;           // [S, d] clean-loss gradient per slot
  float* delta;        // [S, d] delta per slot
  float* wnew_cur;     // [S, d] updated rows of batch t
  float* wnew_prev;    // [S, d] updated rows of batch t-1 (read + flushed)
  float* loss_clean;   // [E]
  float* loss_adv;     // [E]
  const int32_t* gen_ptr;  // plan generation (device: graphs stay valid across plans)
  int32_t d, B, S, R, t;
  int32_t kb;          // slot bits of the plan's src encoding
  int32_t prev_valid;  // 1: rows of batch t-1 are still pending in wnew_prev
  int32_t diag_launch; // diagnostic build: stamp slot of this launch
  int32_t use_single;  // fused triplets run in k_single waves; their slots are skipped
  int32_t touch_next;  // phase 2 reads batch t+1's inline records (brings them on-die)
  const int32_t* slot_list;   // [nb][S] non-fused slots of each batch (list kernels)
  const int32_t* flush_list;  // [nb][S] slots whose row stays in W scratch
  const int32_t* slot_cnt;    // [nb]
  const int32_t* flush_cnt;   // [nb]
  int32_t slot_waves;  // waves [0, slot_waves) are slot waves, the rest fused-triplet waves
  int32_t* step_err;    // bit 0: a wait gave up (acf_apr_set_spin_limit), sticky until read
  // streamed step (k_stream): one launch runs batches [first, t_end); every row a
  // batch updates becomes a VERSION at [batch][slot] (weights ver_w, Adagrad slot
  // ver_a) and every delta too (ver_d), as tagged granules (tag = *epoch)
  int32_t first, t_end;
  unsigned long long* ver_w;
  unsigned long long* ver_a;
  unsigned long long* ver_d;
  const uint32_t* epoch;
  const int32_t* nextt;  // [nb][S] next batch touching the slot's row (flush)
  const int32_t* task_list;  // [nb][task_stride] a batch's tasks (slot, or S + fused group); null: positions
  const int32_t* task_cnt;   // [nb]
  int32_t task_stride, max_depth;
  int32_t poll_sleep;  // k_stream: s_sleep between polls of a version (0-3; 4/5/6 = 8/16/32)
  // k_stream's give-ups: a version wait that gave up after spin_limit polls
  // stores the launch's seq into the failure word `fail` (so the word needs no
  // reset between calls: a launch failed iff *fail == its seq).  The write-back
  // of a failed launch writes nothing, so the tables are as before the call.
  int32_t* fail;
  int32_t spin_limit;
  // (r04) the end of a streamed call, decided once per launch (stream_end):
  //  - seq: the host's number of this launch (status ring slot seq % 8);
  //  - verify: a failed call is replayed by the host later (acf_apr_resolve):
  //    the decider sets the group's gate, so every later streamed launch of the
  //    group runs nothing until the replays, and leaves the epoch alone; an
  //    unverified failure sets step_err bit 0 and bumps the epoch;
  //  - tail: the launch ends in a barrier over an arrival counter (workgroups
  //    arrive once each; arrive_target = the host's running total), the first
  //    workgroup to reach the decide word records COMMIT / FAIL for seq, and on
  //    COMMIT every workgroup writes back its share of the plan's final-slot
  //    list (the rows' last versions) -- no k_stream_flush launch;
  //  - status: host-mapped ring where the decider reports (seq << 2) | failed.
  uint32_t seq;
  int32_t verify;
  int32_t* gate;
  unsigned long long* decide;
  unsigned long long decide_prev;  // the decide word as the host expects it (the last tail launch committed)
  unsigned long long* arrive;  // two sets (by tail_par) of a top counter + 8 shard counters, 128 B apart
  int32_t tail_par;
  int32_t tail;
  int32_t flushers;  // tail: workgroups [0, flushers) wait for the outcome and write back
  unsigned long long* tail_diag;  // ACF_TAIL_DIAG: s_memrealtime stamps of the tail (tools/tail_diag.py)
  const int2* final_list;   // [n] {t * S + slot, row | item << 31}: slots no later batch of the plan touches
  const int32_t* final_cnt;
  unsigned long long* status;
  // hot slots of list plans (k_records): piece waves [slot_waves, slot_waves +
  // hot_waves) of a list kernel stride over the batch's pieces; partial sums in hot_part
  HotLists hot;
  float* hot_part;     // [piece_stride, d]
  int32_t hot_waves;
  int32_t hot_blocks;  // k_tri_combine: hot-slot combining workgroups after the piece waves (0: k_hot_combine)
  // shard mode (distributed.ShardedAPR): item rows of the batch are this rank's
  // partial sums; an item slot's clean / adversarial sum goes to g0[k] for the
  // exchange instead of Adagrad, and item rows are never written back
  int32_t shard;
  int32_t reg_B;       // batch size of reg * mean(w^2) (the global batch in shard mode)
  // shard mode with export (acf_apr_shard_pass_export): an item slot's partial sum
  // also goes to xbuf row xmap[slot - nU] (the split step's exchange rows): the hot
  // combine stores its hot slots there, and its last xblocks workgroups copy the
  // other item slots' sums from g0 (no separate copy launch)
  float* xbuf;
  const int64_t* xmap;
  // triplet-centric shard passes (r05): the owners' item deltas, row w's at
  // xdelta[xdmap[w]] (the exchange rows acf_apr_shard_items_mapped dir 1 names),
  // read by k_tri_adv in place of a copy into the delta slots
  const float* xdelta;
  const int64_t* xdmap;
  const int32_t* xubs;  // the plan's user / item slot bounds (one batch)
  const int32_t* xibs;
  int32_t xn, xblocks;
  // ... and, for the pass that updates the users, the user rows' write-back (the
  // k_flush of the pass): hot user slots go to their table in the combine, the
  // last xflush of the xblocks workgroups copy the others from W scratch
  int32_t xflush;
  // triplet-centric list step (k_tri_*): per-occurrence contributions of shared rows
  const int4* tpos;    // [E] CSR positions of a triplet's three occurrences
  // hash plans (r06): [nb] fused triplets of each batch, placed first in trec /
  // tpos (the clean pass starts past them); null: plans in triplet order
  const int32_t* tri_nf;
  // k_tri_cadv (r06): per shared slot of the batch, (call counter << 32 | t) once
  // its clean sum and delta are stored (the adversarial triplets of the same
  // launch wait for it)
  unsigned long long* ready;
  float* contrib;      // users [B][2][d] (positive, negative branch), then items [2B][d]
  int32_t inplace;     // triplet-centric plans: every row is updated in its table (no W scratch)
  float lr, eps, reg, reg_adv, clip_lo, clip_hi;
  int32_t adver, adv_mode, zero_delta;
  uint64_t seed;
};

// An OccRec as three int4 registers (kept in VGPRs; a struct of scalars passed
// by reference got demoted to scratch).  Field order as in OccRec.
struct RecV {
  int4 a, b, c;
  __device__ int own_row() const { return a.x; }
  __device__ int own_src() const { return a.y; }
  __device__ int meta() const { return a.z; }
  __device__ int ovf() const { return a.w; }
  __device__ int e_role() const { return b.x; }
  __device__ int pa_row() const { return b.y; }
  __device__ int pb_row() const { return b.z; }
  __device__ int pa_src() const { return b.w; }
  __device__ int pb_src() const { return c.x; }
  __device__ int pa_slot() const { return c.y & ACF_SLOT_MASK; }
  __device__ int pb_slot() const { return c.z & ACF_SLOT_MASK; }
  __device__ bool pa_solo() const { return (c.y & ACF_SOLO_BIT) != 0; }
  __device__ bool pb_solo() const { return (c.z & ACF_SOLO_BIT) != 0; }
  __device__ int gen() const { return c.w; }
};

__device__ __forceinline__ RecV load_rec(const OccRec* __restrict__ p) {
  const int4* q = reinterpret_cast<const int4*>(p);
  RecV r;
  r.a = q[0];
  r.b = q[1];
  r.c = q[2];
  return r;
}

// current value of a row at batch start: pending scratch or the table
__device__ __forceinline__ const float* row_src(const StepArgs& a, const float* table, int32_t row,
                                                int32_t src) {
  return (pend1(src, a.kb) && a.prev_valid) ? a.wnew_prev + (int64_t)src_slot(src, a.kb) * a.d
                                            : table + (int64_t)row * a.d;
}

#define ACF_SPIN_LIMIT (1 << 16)  // default version polls before a k_stream wait gives up

template <int LPR, int NV>
__device__ __forceinline__ RowV<NV> load_at(const float* __restrict__ p, int d, int l) {
  return load_row<LPR, NV>(p, 0, d, l);
}

// butterfly over the lane-groups of a wave (fixed order -> deterministic)
template <int LPR, int NV>
__device__ __forceinline__ void group_allreduce(RowV<NV>& G) {
#pragma unroll
  for (int m = LPR; m < 64; m <<= 1) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      G.v[v].x += __shfl_xor(G.v[v].x, m, 64);
      G.v[v].y += __shfl_xor(G.v[v].y, m, 64);
      G.v[v].z += __shfl_xor(G.v[v].z, m, 64);
      G.v[v].w += __shfl_xor(G.v[v].w, m, 64);
    }
  }
}

// Slot header from the group-0 inline record, broadcast to the wave.
struct SlotHdr {
  int32_t count, is_item, own_row, own_src, ovf;
};

// Lane-groups are organised in teams of TEAM groups; a team owns one slot and
// member m of the team takes occurrences m, m+TEAM, ...  TEAM = 64/LPR is one
// wave per slot (hot rows of small batches); TEAM = 1 packs 64/LPR slots per
// wave (large batches, where almost every slot has one occurrence).
struct SlotRec {
  SlotHdr h;
  RecV r0, r1;  // inline records of occurrences m and m + TEAM
  bool r0_valid, r1_valid;
};

// Records m and m + TEAM of slot k (those < R; both addresses are known up
// front, so a slot of up to 2 TEAM occurrences needs no CSR hop) and the slot
// header broadcast from the team leader's lane.
template <int LPR, int TEAM>
__device__ __forceinline__ SlotRec slot_header(const StepArgs& a, int k, int m, int leader_lane) {
  const int32_t gen = *a.gen_ptr;
  SlotRec s;
  s.r0.a = s.r0.b = s.r0.c = make_int4(0, 0, 0, -1);
  s.r1 = s.r0;
  const OccRec* base = a.inl + ((int64_t)a.t * a.S + k) * a.R;
  if (m < a.R && k < a.S) s.r0 = load_rec(base + m);
  if (m + TEAM < a.R && k < a.S) s.r1 = load_rec(base + m + TEAM);
  s.r0_valid = s.r0.gen() == gen;
  s.r1_valid = s.r1.gen() == gen;
  // one team per wave: the leader is lane 0, read with v_readlane (no LDS trip)
  auto from_leader = [&](int32_t v) -> int32_t {
    if constexpr (LPR * TEAM == 64) return __builtin_amdgcn_readlane(v, 0);
    else return __shfl(v, leader_lane, 64);
  };
  const int32_t meta = from_leader(s.r0_valid ? s.r0.meta() : 0);
  // a fused triplet's slots are handled by its k_single lane-group
  s.h.count = (a.use_single && (meta & ACF_SINGLE_BIT)) ? 0 : (meta & ACF_COUNT_MASK);
  s.h.is_item = (meta & ACF_ITEM_BIT) != 0;
  s.h.own_row = from_leader(s.r0.own_row());
  s.h.own_src = from_leader(s.r0.own_src());
  s.h.ovf = from_leader(s.r0.ovf());
  return s;
}

// record of occurrence idx of the slot (idx < count): the member's inline
// records for occurrences m and m + TEAM, the CSR records otherwise
template <int TEAM>
__device__ __forceinline__ RecV occ_rec(const StepArgs& a, const SlotRec& s, int idx, int m) {
  if (idx == m && m < a.R && s.r0_valid) return s.r0;
  if (idx == m + TEAM && m + TEAM < a.R && s.r1_valid) return s.r1;
  return load_rec((s.h.is_item ? a.irec : a.urec) + s.h.ovf + idx);
}

// record of occurrence idx of slot k re-read from memory (inline or CSR): the
// streamed step's hot-row passes, which keep no records in registers
__device__ __forceinline__ RecV occ_rec_mem(const StepArgs& a, const SlotHdr& h, int k, int idx) {
  if (idx < a.R) return load_rec(a.inl + ((int64_t)a.t * a.S + k) * a.R + idx);
  return load_rec((h.is_item ? a.irec : a.urec) + h.ovf + idx);
}

// One occurrence's BPR term (APR.py:127-150) against the slot's own row (clean,
// or own + delta for the adversarial loss) and the partner rows ra / rb; the
// gradient w.r.t. the own row goes into G, the loss to loss[e] (or to *keep,
// for the caller to store later).
template <int LPR, int NV>
__device__ __forceinline__ void occ_term(const StepArgs& a, int is_item, const RowV<NV>& own, const RecV& r,
                                         const RowV<NV>& ra, const RowV<NV>& rb, bool active, int l,
                                         float* __restrict__ loss_out, RowV<NV>& G, float* keep = nullptr,
                                         float* gkeep = nullptr) {
  float gb, loss;
  if (!is_item) {
    const float x = dot_row<LPR, NV>(own, ra) - dot_row<LPR, NV>(own, rb);
    bpr_term(x, a.clip_lo, a.clip_hi, gb, loss);
    if (gkeep) *gkeep = gb;
    if (active) {
      axpy_row(G, gb, ra);   // pos branch: dx+/dp = q_i
      axpy_row(G, -gb, rb);  // neg branch: dx-/dp = q_j
      if (keep) *keep = loss;
      else if (l == 0) loss_out[r.e_role()] = loss;
    }
  } else {
    const float dq = dot_row<LPR, NV>(ra, own), dqo = dot_row<LPR, NV>(ra, rb);
    const int role = active ? (r.e_role() & 1) : 0;
    const float x = role ? (dqo - dq) : (dq - dqo);
    bpr_term(x, a.clip_lo, a.clip_hi, gb, loss);
    if (gkeep) *gkeep = gb;
    if (active) axpy_row(G, role ? -gb : gb, ra);
  }
}

// copy the pending row of slot k of batch tb (in wsrc) to its table; the
// team's tl-th lane of tn copies float4 chunks tl, tl+tn, ...
__device__ __forceinline__ void flush_slot(const StepArgs& a, int tb, const float* __restrict__ wsrc,
                                           int k, int tl, int tn) {
  if (k >= a.S) return;
  const RecV r = load_rec(a.inl + ((int64_t)tb * a.S + k) * a.R);
  if (r.gen() != *a.gen_ptr || (r.meta() & ACF_COUNT_MASK) == 0) return;
  if (a.use_single && (r.meta() & ACF_INPLACE_BIT)) return;  // written by its fused triplet
  if (a.shard && (r.meta() & ACF_ITEM_BIT)) return;            // owned by another rank's update
  float* dst = ((r.meta() & ACF_ITEM_BIT) ? a.Q : a.P) + (int64_t)r.own_row() * a.d;
  const float* src = wsrc + (int64_t)k * a.d;
  for (int c = tl; c * 4 < a.d; c += tn)
    *reinterpret_cast<float4*>(dst + c * 4) = *reinterpret_cast<const float4*>(src + c * 4);
}

// The write-back of slot k of batch t-1 split in two so that it never sits in
// front of the wave's own loads: begin() loads the record, then (once the
// record is there) the pending row chunk this lane copies; end() stores it.
struct FlushOp {
  float4 v;
  float* dst;
};

__device__ __forceinline__ RecV flush_rec(const StepArgs& a, int tb, int k) {
  RecV r;
  r.a = r.b = r.c = make_int4(0, 0, 0, -1);
  if (k < a.S) r = load_rec(a.inl + ((int64_t)tb * a.S + k) * a.R);
  return r;
}

// lane tl of a team of tn lanes copies float4 chunk tl (d/4 <= tn) of the row
__device__ __forceinline__ FlushOp flush_load(const StepArgs& a, const RecV& r, const float* __restrict__ wsrc,
                                              int k, int tl, int tn) {
  FlushOp f;
  f.dst = nullptr;
  if (r.gen() != *a.gen_ptr || (r.meta() & ACF_COUNT_MASK) == 0) return f;
  if (a.use_single && (r.meta() & ACF_INPLACE_BIT)) return f;
  if (tl * 4 >= a.d) return f;
  f.dst = ((r.meta() & ACF_ITEM_BIT) ? a.Q : a.P) + (int64_t)r.own_row() * a.d + tl * 4;
  f.v = *reinterpret_cast<const float4*>(wsrc + (int64_t)k * a.d + tl * 4);
  return f;
}

__device__ __forceinline__ void flush_store(const FlushOp& f) {
  if (f.dst) *reinterpret_cast<float4*>(f.dst) = f.v;
}

// Adagrad (TF SparseApplyAdagrad after the dedup) for one row held by a
// lane-group, plus the reg*mean(w^2) terms of APR.py:153-154,164-165.
template <int NV>
__device__ __forceinline__ void adagrad_row(const StepArgs& a, RowV<NV>& G, const RowV<NV>& w,
                                            RowV<NV>& acc, int m, RowV<NV>& wout) {
  if (a.reg != 0.f) {
    const float coef = (2.0f * a.reg / ((float)a.reg_B * (float)a.d)) * (float)(a.adver ? 2 * m : m);
    axpy_row(G, coef, w);
  }
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    float4& c = acc.v[v];
    const float4 g = G.v[v];
    const float4 x = w.v[v];
    c.x = c.x + g.x * g.x;
    c.y = c.y + g.y * g.y;
    c.z = c.z + g.z * g.z;
    c.w = c.w + g.w * g.w;
    // Eigen's a.rsqrt(); v_rsq_f32 (1 ulp)
    wout.v[v].x = x.x - (a.lr * g.x) * __builtin_amdgcn_rsqf(c.x);
    wout.v[v].y = x.y - (a.lr * g.y) * __builtin_amdgcn_rsqf(c.y);
    wout.v[v].z = x.z - (a.lr * g.z) * __builtin_amdgcn_rsqf(c.z);
    wout.v[v].w = x.w - (a.lr * g.w) * __builtin_amdgcn_rsqf(c.w);
  }
}

// butterfly over the TEAM lane-groups of a team (fixed order -> deterministic)
template <int LPR, int TEAM, int NV>
__device__ __forceinline__ void team_allreduce(RowV<NV>& G) {
#pragma unroll
  for (int m = LPR; m < LPR * TEAM; m <<= 1) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      G.v[v].x += __shfl_xor(G.v[v].x, m, 64);
      G.v[v].y += __shfl_xor(G.v[v].y, m, 64);
      G.v[v].z += __shfl_xor(G.v[v].z, m, 64);
      G.v[v].w += __shfl_xor(G.v[v].w, m, 64);
    }
  }
}

// The same butterfly for a team that spans a whole, fully active wave
// (k_stream): the lane^16 and lane^32 exchanges use gfx950's
// v_permlane16_swap / v_permlane32_swap (VALU) instead of ds_bpermute (an LDS
// round trip each).  Pure data movement: the sums, and so the bits, are
// team_allreduce's.  With vdst = src0 = x, a lane's partner value is the
// swapped vdst in the upper half of each pair of rows, the swapped src0 below.
template <int M>
__device__ __forceinline__ float xor_lane_wave(float x) {
  const uint32_t u = __float_as_uint(x);
  if constexpr (M == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    return __uint_as_float((threadIdx.x & 16) ? r[0] : r[1]);
  } else if constexpr (M == 32) {
    const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    return __uint_as_float((threadIdx.x & 32) ? r[0] : r[1]);
  } else {
    return __shfl_xor(x, M, 64);
  }
}

template <int M, int END, int NV>
__device__ __forceinline__ void wave_butterfly(RowV<NV>& G) {
  if constexpr (M < END) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      G.v[v].x += xor_lane_wave<M>(G.v[v].x);
      G.v[v].y += xor_lane_wave<M>(G.v[v].y);
      G.v[v].z += xor_lane_wave<M>(G.v[v].z);
      G.v[v].w += xor_lane_wave<M>(G.v[v].w);
    }
    wave_butterfly<2 * M, END, NV>(G);
  }
}

template <int LPR, int TEAM, int NV>
__device__ __forceinline__ void team_allreduce_wave(RowV<NV>& G) {
  static_assert(LPR * TEAM == 64, "team_allreduce_wave: one team per wave");
  wave_butterfly<LPR, 64, NV>(G);
}

// Lane geometry of a step kernel: slot k of this team, member m, lane l in the
// row-group, the team leader's lane, the lane index inside the team.
template <int LPR, int TEAM>
struct Geo {
  int wave, k, m, l, leader, tl;
  __device__ Geo() {
    constexpr int OPW = 64 / LPR;
    const int lane = threadIdx.x & 63;
    const int g = lane / LPR;
    wave = (int)((blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6);
    k = wave * (OPW / TEAM) + g / TEAM;
    m = g % TEAM;
    l = lane & (LPR - 1);
    leader = (g / TEAM) * TEAM * LPR;
    tl = lane - leader;
  }
};

// "random" delta: l2_normalize(truncated_normal(0, 0.01)) * eps, redrawn every
// run (APR.py:180-191, adv == "random").  Out of line: the gradient mode never
// runs it and it would otherwise bloat every step kernel's instruction stream.
template <int LPR, int NV>
__device__ __noinline__ RowV<NV> random_delta(uint64_t seed, uint32_t call, int32_t t, int32_t d, float eps,
                                              int is_item, int32_t row, int l) {
  RowV<NV> z;
  const uint64_t rk = mix64(seed ^ mix64(((uint64_t)call << 33) ^ (((uint64_t)t << 1) | (is_item ? 1 : 0)))) ^
                      mix64((uint64_t)row * 0x100000001B3ull);
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c = l + LPR * v;
    float e4[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      e4[e] = (c * 4 + e < d) ? trunc_normal(rk ^ mix64((uint64_t)(c * 4 + e)), 0.01f) : 0.f;
    z.v[v] = make_float4(e4[0], e4[1], e4[2], e4[3]);
  }
  const float ss = dot_row<LPR, NV>(z, z);
  const float inv = __builtin_amdgcn_rsqf(fmaxf(ss, 1e-12f));
  return scale_row(scale_row(z, inv), eps);
}

// delta of one row from its batch-summed clean gradient G (APR.py:180-191)
template <int LPR, int NV>
__device__ __forceinline__ RowV<NV> make_delta(const StepArgs& a, const RowV<NV>& G, int is_item,
                                               int32_t row, int l) {
  if (a.zero_delta) return zero_row<NV>();
  if (a.adv_mode == 0) {
    // tf.nn.l2_normalize(g, 1) * eps  (epsilon 1e-12 on the squared norm)
    const float ss = dot_row<LPR, NV>(G, G);
    const float inv = __builtin_amdgcn_rsqf(fmaxf(ss, 1e-12f));
    return scale_row(scale_row(G, inv), a.eps);
  }
  // keyed on the context's call counter too (advanced by every call's write-back
  // kernel), so every run draws fresh noise, as truncated_normal does per sess.run
  return random_delta<LPR, NV>(a.seed, *a.epoch, a.t, a.d, a.eps, is_item, row, l);
}

// A fused triplet (fuse_info): its whole step in one lane-group.  The operation
// sequence per row is the one the slot kernels execute for a row with a single
// occurrence (same products, same rounding order), so fused and slot paths give
// identical bits.  ADV (APR graph, inside k_adv): the tables are current and
// the row goes clean -> delta -> adversarial -> Adagrad; otherwise (BPR graph,
// inside k_clean<FUSE_APPLY>) rows are read through their batch-start source and
// the clean gradient is applied.
template <int LPR, int NV, bool ADV>
__device__ __forceinline__ void k_single(const StepArgs& a, int b, int l) {
  if (b >= a.B) return;
  const int64_t e = (int64_t)a.t * a.B + b;
  const RecV r = load_rec(a.trec + e);
  if (r.c.w != *a.gen_ptr || !(r.c.y & 1)) return;
  const int d = a.d;
  const int32_t u = r.a.x, i = r.a.y, j = r.a.z, flags = r.c.y;
  RowV<NV> p, qi, qj;
  if (ADV) {
    p = load_row<LPR, NV>(a.P, u, d, l);
    qi = load_row<LPR, NV>(a.Q, i, d, l);
    qj = load_row<LPR, NV>(a.Q, j, d, l);
  } else {
    p = load_at<LPR, NV>(row_src(a, a.P, u, r.b.z), d, l);
    qi = load_at<LPR, NV>(row_src(a, a.Q, i, r.b.w), d, l);
    qj = load_at<LPR, NV>(row_src(a, a.Q, j, r.c.x), d, l);
  }
  RowV<NV> cu = load_row<LPR, NV>(a.accP, u, d, l);
  RowV<NV> ci = load_row<LPR, NV>(a.accQ, i, d, l);
  RowV<NV> cj = load_row<LPR, NV>(a.accQ, j, d, l);
  float g, loss;
  bpr_term(dot_row<LPR, NV>(p, qi) - dot_row<LPR, NV>(p, qj), a.clip_lo, a.clip_hi, g, loss);
  if (l == 0) a.loss_clean[e] = loss;
  RowV<NV> Gu = zero_row<NV>(), Gi = zero_row<NV>(), Gj = zero_row<NV>();
  axpy_row(Gu, g, qi);
  axpy_row(Gu, -g, qj);
  axpy_row(Gi, g, p);
  axpy_row(Gj, -g, p);
  if (ADV) {
    const RowV<NV> pp = add_row(p, make_delta<LPR, NV>(a, Gu, 0, u, l));
    const RowV<NV> qip = add_row(qi, make_delta<LPR, NV>(a, Gi, 1, i, l));
    const RowV<NV> qjp = add_row(qj, make_delta<LPR, NV>(a, Gj, 1, j, l));
    float ga, la;
    bpr_term(dot_row<LPR, NV>(pp, qip) - dot_row<LPR, NV>(pp, qjp), a.clip_lo, a.clip_hi, ga, la);
    if (l == 0) a.loss_adv[e] = la;
    RowV<NV> Au = zero_row<NV>(), Ai = zero_row<NV>(), Aj = zero_row<NV>();
    axpy_row(Au, ga, qip);
    axpy_row(Au, -ga, qjp);
    axpy_row(Ai, ga, pp);
    axpy_row(Aj, -ga, pp);
    axpy_row(Gu, a.reg_adv, Au);
    axpy_row(Gi, a.reg_adv, Ai);
    axpy_row(Gj, a.reg_adv, Aj);
  }
  RowV<NV> wu, wi, wj;
  adagrad_row(a, Gu, p, cu, 1, wu);
  adagrad_row(a, Gi, qi, ci, 1, wi);
  adagrad_row(a, Gj, qj, cj, 1, wj);
  store_row<LPR, NV>(a.accP, u, d, l, cu);
  store_row<LPR, NV>(a.accQ, i, d, l, ci);
  store_row<LPR, NV>(a.accQ, j, d, l, cj);
  // in place unless the row is pending from batch t-1 or read by batch t+1
  store_row<LPR, NV>((flags & 2) ? a.P : a.wnew_cur, (flags & 2) ? u : r.a.w, d, l, wu);
  store_row<LPR, NV>((flags & 4) ? a.Q : a.wnew_cur, (flags & 4) ? i : r.b.x, d, l, wi);
  store_row<LPR, NV>((flags & 8) ? a.Q : a.wnew_cur, (flags & 8) ? j : r.b.y, d, l, wj);
}

// Phase 1 = sess.run([update_P, update_Q]) (APR.py:180-191) and the clean half
// of the optimizer: clean-loss gradient of every unique row of batch t summed
// over its occurrences, its delta (APR graph), or — BPR graph, FUSE_APPLY — the
// Adagrad update straight away.  Slot k, team member m, lane l of the row-group,
// the team leader's lane.
template <int LPR, int NV, bool FUSE_APPLY, int TEAM, bool FLUSH = false>
__device__ __forceinline__ void clean_slot(const StepArgs& a, int k, int m, int l, int leader, int wave,
                                           int tl = 0) {
  // write-back of slot k of batch t-1: its record is loaded next to our header
  RecV frec;
  if (FLUSH) frec = flush_rec(a, a.t - 1, k);
  const SlotRec sr = slot_header<LPR, TEAM>(a, k, m, leader);
  const SlotHdr& h = sr.h;
  FlushOp fo;
  if (FLUSH) fo = flush_load(a, frec, a.wnew_prev, k, tl, TEAM * LPR);
  STAMP(a.diag_launch, wave, 1);
  if (h.count == 0) {
    if (FLUSH) flush_store(fo);
    return;
  }
  const int d = a.d;
  const float* own_tab = h.is_item ? a.Q : a.P;
  const RowV<NV> own = load_at<LPR, NV>(row_src(a, own_tab, h.own_row, h.own_src), d, l);
  RowV<NV> acc;
  if (FUSE_APPLY && m == 0)
    acc = load_row<LPR, NV>(h.is_item ? a.accQ : a.accP, h.own_row, d, l);
  RowV<NV> G = zero_row<NV>();
  // member m takes occurrences m, m + TEAM, m + 2 TEAM, ... (in that order into
  // G); two per pass, all their loads in flight before either is used
  for (int base = 0; base < h.count; base += 2 * TEAM) {
    const int i0 = base + m, i1 = base + TEAM + m;
    const bool a0 = i0 < h.count, a1 = i1 < h.count;
    RowV<NV> ra0 = zero_row<NV>(), rb0 = zero_row<NV>(), ra1 = zero_row<NV>(), rb1 = zero_row<NV>();
    RecV r0, r1;
    if (a0) r0 = occ_rec<TEAM>(a, sr, i0, m);
    if (a1) r1 = occ_rec<TEAM>(a, sr, i1, m);
    // user slot: ra = Q[i], rb = Q[j];  item slot: ra = P[u], rb = Q[other]
    if (a0) {
      ra0 = load_at<LPR, NV>(row_src(a, h.is_item ? a.P : a.Q, r0.pa_row(), r0.pa_src()), d, l);
      rb0 = load_at<LPR, NV>(row_src(a, a.Q, r0.pb_row(), r0.pb_src()), d, l);
    }
    if (a1) {
      ra1 = load_at<LPR, NV>(row_src(a, h.is_item ? a.P : a.Q, r1.pa_row(), r1.pa_src()), d, l);
      rb1 = load_at<LPR, NV>(row_src(a, a.Q, r1.pb_row(), r1.pb_src()), d, l);
    }
    occ_term<LPR, NV>(a, h.is_item, own, r0, ra0, rb0, a0, l, a.loss_clean, G);
    if (__any(a1)) occ_term<LPR, NV>(a, h.is_item, own, r1, ra1, rb1, a1, l, a.loss_clean, G);
  }
  STAMP(a.diag_launch, wave, 2);
  team_allreduce<LPR, TEAM, NV>(G);
  if (FLUSH) flush_store(fo);
  if (FUSE_APPLY) {
    if (m == 0 && a.shard && h.is_item) {  // partial item sum for the owner
      store_row<LPR, NV>(a.g0, k, d, l, G);
    } else if (m == 0) {
      RowV<NV> wout;
      adagrad_row(a, G, own, acc, h.count, wout);
      store_row<LPR, NV>(h.is_item ? a.accQ : a.accP, h.own_row, d, l, acc);
      store_row<LPR, NV>(a.wnew_cur, k, d, l, wout);
    }
    return;
  }
  const RowV<NV> dl = make_delta<LPR, NV>(a, G, h.is_item, h.own_row, l);
  STAMP(a.diag_launch, wave, 3);
  if (m == 0) {
    store_row<LPR, NV>(a.g0, k, d, l, G);
    store_row<LPR, NV>(a.delta, k, d, l, dl);
  }
}

// Phase 2 = adversarial half of sess.run(optimizer) (APR.py:130-141,156-165)
// and SparseApplyAdagrad: loss on p+dP[u], q+dQ[i]; G = G_clean + reg_adv*G_adv;
// Adagrad into wnew_cur.  The tables are current (flushed by phase 1).
template <int LPR, int NV, int TEAM>
__device__ __forceinline__ void adv_slot(const StepArgs& a, int k, int m, int l, int leader, int wave) {
  // read (not copy) batch t+1's record of this slot: phase 1 of the next batch
  // then finds it in the Infinity Cache instead of HBM
  int4 nxt = make_int4(0, 0, 0, 0), nxt1 = nxt;
  if (a.touch_next && k < a.S) {
    const OccRec* nb = a.inl + ((int64_t)(a.t + 1) * a.S + k) * a.R;
    if (m < a.R) nxt = *reinterpret_cast<const int4*>(nb + m);
    if (m + TEAM < a.R) nxt1 = *reinterpret_cast<const int4*>(nb + m + TEAM);
  }
  const SlotRec sr = slot_header<LPR, TEAM>(a, k, m, leader);
  const SlotHdr& h = sr.h;
  STAMP(a.diag_launch, wave, 1);
  if (h.count == 0) {
    if (nxt.x == -0x7fffffff && nxt1.y == 0x7fffffff) a.loss_adv[0] = 0.f;
    return;
  }
  const int d = a.d;
  const float* own_tab = h.is_item ? a.Q : a.P;
  const RowV<NV> own = load_row<LPR, NV>(own_tab, h.own_row, d, l);
  const RowV<NV> ownp = add_row(own, load_row<LPR, NV>(a.delta, k, d, l));
  RowV<NV> acc, G0;
  if (m == 0) {
    acc = load_row<LPR, NV>(h.is_item ? a.accQ : a.accP, h.own_row, d, l);
    G0 = load_row<LPR, NV>(a.g0, k, d, l);
  }
  RowV<NV> G = zero_row<NV>();
  for (int base = 0; base < h.count; base += 2 * TEAM) {  // as in clean_slot
    const int i0 = base + m, i1 = base + TEAM + m;
    const bool a0 = i0 < h.count, a1 = i1 < h.count;
    RowV<NV> ra0 = zero_row<NV>(), rb0 = zero_row<NV>(), ra1 = zero_row<NV>(), rb1 = zero_row<NV>();
    RecV r0, r1;
    if (a0) r0 = occ_rec<TEAM>(a, sr, i0, m);
    if (a1) r1 = occ_rec<TEAM>(a, sr, i1, m);
    const float* ptab = h.is_item ? a.P : a.Q;
    if (a0) {
      ra0 = add_row(load_row<LPR, NV>(ptab, r0.pa_row(), d, l), load_row<LPR, NV>(a.delta, r0.pa_slot(), d, l));
      rb0 = add_row(load_row<LPR, NV>(a.Q, r0.pb_row(), d, l), load_row<LPR, NV>(a.delta, r0.pb_slot(), d, l));
    }
    if (a1) {
      ra1 = add_row(load_row<LPR, NV>(ptab, r1.pa_row(), d, l), load_row<LPR, NV>(a.delta, r1.pa_slot(), d, l));
      rb1 = add_row(load_row<LPR, NV>(a.Q, r1.pb_row(), d, l), load_row<LPR, NV>(a.delta, r1.pb_slot(), d, l));
    }
    occ_term<LPR, NV>(a, h.is_item, ownp, r0, ra0, rb0, a0, l, a.loss_adv, G);
    if (__any(a1)) occ_term<LPR, NV>(a, h.is_item, ownp, r1, ra1, rb1, a1, l, a.loss_adv, G);
  }
  STAMP(a.diag_launch, wave, 2);
  team_allreduce<LPR, TEAM, NV>(G);
  if (m == 0 && a.shard && h.is_item) {  // partial adversarial item sum for the owner
    store_row<LPR, NV>(a.g0, k, d, l, G);
  } else if (m == 0) {
    axpy_row(G0, a.reg_adv, G);
    RowV<NV> wout;
    adagrad_row(a, G0, own, acc, h.count, wout);
    store_row<LPR, NV>(h.is_item ? a.accQ : a.accP, h.own_row, d, l, acc);
    store_row<LPR, NV>(a.wnew_cur, k, d, l, wout);
  }
  if (nxt.x == -0x7fffffff && nxt1.y == 0x7fffffff) a.loss_adv[0] = 0.f;  // keeps the reads alive; never true
}

// One team per slot; the team also writes back slot k of batch t-1.  Waves past
// slot_waves (SINGLE) run fused triplets.
template <int LPR, int NV, bool FUSE_APPLY, int TEAM, bool SINGLE = false>
__global__ void __launch_bounds__(256) k_clean(StepArgs a) {
  const Geo<LPR, TEAM> q;
  if (SINGLE && FUSE_APPLY && q.wave >= a.slot_waves) {
    k_single<LPR, NV, false>(a, (q.wave - a.slot_waves) * (64 / LPR) + (int)(threadIdx.x & 63) / LPR,
                             q.l);
    return;
  }
  STAMP(a.diag_launch, q.wave, 0);
  CLOCKSTAMP(a.diag_launch, q.wave, 6);
  // one wave per slot and a row of <= 64 float4: the write-back overlaps the slot's loads
  if (TEAM * LPR >= 64 && a.d <= 4 * TEAM * LPR && a.prev_valid) {
    clean_slot<LPR, NV, FUSE_APPLY, TEAM, true>(a, q.k, q.m, q.l, q.leader, q.wave, q.tl);
  } else {
    if (a.prev_valid) flush_slot(a, a.t - 1, a.wnew_prev, q.k, q.tl, TEAM * LPR);
    clean_slot<LPR, NV, FUSE_APPLY, TEAM>(a, q.k, q.m, q.l, q.leader, q.wave);
  }
  STAMP(a.diag_launch, q.wave, 4);
  CLOCKSTAMP(a.diag_launch, q.wave, 7);
}

template <int LPR, int NV, int TEAM, bool SINGLE = false>
__global__ void __launch_bounds__(256) k_adv(StepArgs a) {
  const Geo<LPR, TEAM> q;
  if (SINGLE && q.wave >= a.slot_waves) {
    k_single<LPR, NV, true>(a, (q.wave - a.slot_waves) * (64 / LPR) + (int)(threadIdx.x & 63) / LPR,
                            q.l);
    return;
  }
  STAMP(a.diag_launch, q.wave, 0);
  adv_slot<LPR, NV, TEAM>(a, q.k, q.m, q.l, q.leader, q.wave);
  STAMP(a.diag_launch, q.wave, 4);
}

// ---------------------------------------------------------------------------
// Streamed APR step (small batches, one wave per slot): ONE launch runs a whole
// range of batches.  Nothing is written to the tables inside it: the Adagrad
// result of row r in batch t becomes the version [t][slot] of r (weights in
// ver_w, accumulator in ver_a), and a reader at batch t' > t finds it through
// the plan's src (dt = t' - t at any distance, k_prev_next).  Versions are never
// overwritten inside a launch, so there is no write-after-read hazard; a reader
// only has to wait until the version exists.
//
// Hand-off (MI355X guide, Guideline 16 R2): a version row is a run of 8-B
// granules {value, tag = epoch of this launch}, each written by a device-scope
// write-through (sc1) store and read by sc1 loads; the reader re-reads the
// granules whose tag is not yet this launch's until every one matches.  No flag,
// no fence, no drain: the data is the flag.  The epoch is bumped by the flush
// kernel after every launch, so a granule left by an earlier launch never
// matches.
//
// Granule order inside a version row is component-major: element 4c + e sits at
// granule e*(d/4) + c, so each of a lane's four 8-B accesses is one contiguous
// run across the row-group's lanes (the element-major order put the lanes 32 B
// apart: every store instruction wrote each 128-B line of the row partially,
// and WRITE_SIZE read 4x the version bytes; tools/calib_fetch.hip).
//
// Schedule: wave w takes position p = w % P of batches t = first + w / P,
// + D, + 2D, ... (P = slot waves + fused-triplet waves of a batch, D = waves / P).
// A position is one unique row (clean half -> delta -> adversarial half ->
// Adagrad, all in the same wave, so G_clean and the own row stay in registers)
// or a group of fused triplets.  No deadlock while every wave is resident (the
// launcher checks occupancy): a clean half waits only for versions of earlier
// batches; an adversarial half waits only for deltas of the same batch, which
// clean halves produce before they wait for anything of that batch, and a wave
// holds at most one position of any batch.  Every wait is bounded; a give-up
// sets step_err bit 0 and makes every other waiting wave give up too.
// ---------------------------------------------------------------------------
typedef unsigned long long u64;

__device__ __forceinline__ const u64* vrow(const u64* base, const StepArgs& a, int32_t t, int32_t k) {
  return base + ((int64_t)t * a.S + k) * a.d;
}

// where the value of a row at the start of batch a.t lives, as ONE 64-bit word:
// the table row's address, or a version row's address | 1 (a version of an
// earlier batch of this launch)
typedef uint64_t VSrc;

__device__ __forceinline__ VSrc ver_src(const StepArgs& a, const float* table, const u64* vbase, int32_t row,
                                        int32_t src) {
  if (src < 0) {
    const int32_t tp = a.t - src_dt(src, a.kb);
    if (tp >= a.first) return (VSrc)(uintptr_t)vrow(vbase, a, tp, src_slot(src, a.kb)) | 1ull;
  }
  return (VSrc)(uintptr_t)(table + (int64_t)row * a.d);
}

__device__ __forceinline__ VSrc ver_at(const u64* p) { return (VSrc)(uintptr_t)p | 1ull; }

// a row as version granules: one aligned 8-B device-scope store per granule
// (write-through, sc1), the guide's R2 form.  (A first version stored two
// granules per inline-asm 16-B store without the trailing s_nop the guide
// requires; readers then saw tags with stale values.)
template <int LPR, int NV>
__device__ __forceinline__ void store_ver(u64* dst, int d, int l, const RowV<NV>& r, uint32_t tag) {
  const u64 hi = (u64)tag << 32;
  const int d4 = d >> 2;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c = l + LPR * v;
    if (c * 4 < d) {
      u64* g = dst + c;  // component-major granules
      __hip_atomic_store(g, hi | __float_as_uint(r.v[v].x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(g + d4, hi | __float_as_uint(r.v[v].y), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(g + 2 * d4, hi | __float_as_uint(r.v[v].z), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(g + 3 * d4, hi | __float_as_uint(r.v[v].w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// wave-uniform end of a wait round: true = stop (all there, or give up)
__device__ __forceinline__ bool wait_round(const StepArgs& a, bool ok, int it) {
  if (__all(ok)) return true;
  if (it >= a.spin_limit) {
    if ((threadIdx.x & 63) == 0)
      __hip_atomic_store(a.fail, (int32_t)a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
  }
  if ((it & 31) == 31 &&
      __any(__hip_atomic_load(a.fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int32_t)a.seq))
    return true;  // another wave gave up: the launch is failing, drain it
  switch (a.poll_sleep) {  // s_sleep takes an immediate
    case 0: break;
    case 1: __builtin_amdgcn_s_sleep(1); break;
    case 3: __builtin_amdgcn_s_sleep(3); break;
    case 4: __builtin_amdgcn_s_sleep(8); break;
    case 5: __builtin_amdgcn_s_sleep(16); break;
    case 6: __builtin_amdgcn_s_sleep(32); break;
    default: __builtin_amdgcn_s_sleep(2); break;
  }
  return false;
}

// Batched attempt over K rows: every row's loads are issued first and the tags
// checked after, so one attempt costs one round trip however many rows wait
// (a per-row load-then-compare made the compiler drain vmcnt between rows:
// six serial round trips in the first wait of a slot).  Version granules are
// read through global-address-space pointers (global_load, not flat_load,
// which would also count in lgkmcnt).
typedef const __attribute__((address_space(1))) u64* gu64_ptr;
typedef const __attribute__((address_space(1))) f32x4* gf4_ptr;

template <int NV>
struct RawRow {
  u64 x[NV][4];
};

template <int LPR, int NV>
__device__ __forceinline__ void issue_row(VSrc s, int d, int l, bool ok, RawRow<NV>& w, RowV<NV>& r) {
  if (ok) return;
  if (!(s & 1ull)) {  // table row: nothing writes it in this launch
    const float* p = reinterpret_cast<const float*>((uintptr_t)s);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int c = l + LPR * v;
      if (c * 4 < d) {
        const f32x4 x = *(gf4_ptr)(p + c * 4);
        r.v[v] = make_float4(x[0], x[1], x[2], x[3]);
      } else {
        r.v[v] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    return;
  }
  const u64* base = reinterpret_cast<const u64*>((uintptr_t)(s & ~1ull));
  const int d4 = d >> 2;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c = l + LPR * v;
    if (c * 4 < d) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        w.x[v][e] = __hip_atomic_load((gu64_ptr)(base + c + e * d4), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <int LPR, int NV>
__device__ __forceinline__ void check_row(VSrc s, int d, int l, uint32_t tag, const RawRow<NV>& w, RowV<NV>& r,
                                          bool& ok) {
  if (ok) return;
  if (!(s & 1ull)) {
    ok = true;
    return;
  }
  bool all = true;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c = l + LPR * v;
    if (c * 4 < d) {
      r.v[v] = make_float4(__uint_as_float((uint32_t)w.x[v][0]), __uint_as_float((uint32_t)w.x[v][1]),
                           __uint_as_float((uint32_t)w.x[v][2]), __uint_as_float((uint32_t)w.x[v][3]));
#pragma unroll
      for (int e = 0; e < 4; ++e) all = all && (uint32_t)(w.x[v][e] >> 32) == tag;
    } else {
      r.v[v] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  ok = all;
}

// Wait until every listed row is there (ok[k] true on entry: not needed).
template <int LPR, int NV, int K>
__device__ __forceinline__ void poll_rows(const StepArgs& a, const VSrc (&s)[K], RowV<NV>* const (&r)[K],
                                          bool (&ok)[K], uint32_t tag, int l) {
  for (int it = 0;; ++it) {
    RawRow<NV> w[K];
#pragma unroll
    for (int k = 0; k < K; ++k) issue_row<LPR, NV>(s[k], a.d, l, ok[k], w[k], *r[k]);
    bool all = true;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      check_row<LPR, NV>(s[k], a.d, l, tag, w[k], *r[k], ok[k]);
      all = all && ok[k];
    }
    if (wait_round(a, all, it)) break;
  }
}

// Partner rows of the member's two occurrences of a pass (batch-start values)
template <int LPR, int NV>
__device__ __forceinline__ void stream_partners(const StepArgs& a, int is_item, const RecV& r0, const RecV& r1,
                                                bool a0, bool a1, uint32_t tag, int l, RowV<NV>& ra0,
                                                RowV<NV>& rb0, RowV<NV>& ra1, RowV<NV>& rb1) {
  const float* ptab = is_item ? a.P : a.Q;
  const VSrc sa0 = a0 ? ver_src(a, ptab, a.ver_w, r0.pa_row(), r0.pa_src()) : 0;
  const VSrc sb0 = a0 ? ver_src(a, a.Q, a.ver_w, r0.pb_row(), r0.pb_src()) : 0;
  const VSrc sa1 = a1 ? ver_src(a, ptab, a.ver_w, r1.pa_row(), r1.pa_src()) : 0;
  const VSrc sb1 = a1 ? ver_src(a, a.Q, a.ver_w, r1.pb_row(), r1.pb_src()) : 0;
  const VSrc src[4] = {sa0, sb0, sa1, sb1};
  RowV<NV>* const dst[4] = {&ra0, &rb0, &ra1, &rb1};
  bool ok[4] = {!a0, !a0, !a1, !a1};
  poll_rows<LPR, NV, 4>(a, src, dst, ok, tag, l);
}

// Delta of a SOLO partner (pb = 0: pa, 1: pb) of one occurrence, formed here
// with the operation sequence the partner's own wave runs for a one-occurrence
// row: its clean term from zero (occ_term), the team reduction's additions of
// +0 (team_allreduce: member 0 holds the only term), then make_delta.  Same bits
// as the published delta.  own / ra / rb are batch-start rows; gk (if given) is
// the occurrence's clean dloss/dx from this wave's clean term: the partner's
// occ_term evaluates the same dot products of the same rows, so it is the
// same bits and the dots and the loss chain need not run again.  (Forming both
// partners' deltas in one straight-line block, with the published-delta loads
// issued before it, measured slower: 4.56 vs 4.37 us per batch.)
template <int LPR, int NV, int TEAM>
__device__ __forceinline__ RowV<NV> solo_delta(const StepArgs& a, int is_item, const RowV<NV>& own,
                                               const RecV& r, const RowV<NV>& ra, const RowV<NV>& rb, int pb,
                                               int l, const float* gk = nullptr) {
  float gb, loss;
  RowV<NV> G = zero_row<NV>();
  int p_item;
  if (!is_item) {  // own = p_u, ra = q_i, rb = q_j: partner item i (pos) or j (neg)
    if (gk) gb = *gk;
    else bpr_term(dot_row<LPR, NV>(own, ra) - dot_row<LPR, NV>(own, rb), a.clip_lo, a.clip_hi, gb, loss);
    axpy_row(G, pb ? -gb : gb, own);
    p_item = 1;
  } else {  // own = this item, ra = p_u, rb = the other item
    const int role = r.e_role() & 1;
    if (gk) {
      gb = *gk;
    } else {
      const float dq = dot_row<LPR, NV>(ra, own), dqo = dot_row<LPR, NV>(ra, rb);
      bpr_term(role ? (dqo - dq) : (dq - dqo), a.clip_lo, a.clip_hi, gb, loss);
    }
    if (!pb) {  // the user: q_pos, q_neg terms in the user slot's order
      axpy_row(G, gb, role ? rb : own);
      axpy_row(G, -gb, role ? own : rb);
      p_item = 0;
    } else {  // the other item, in the opposite role
      axpy_row(G, role ? gb : -gb, ra);
      p_item = 1;
    }
  }
#pragma unroll
  for (int s = 1; s < TEAM; s <<= 1) G = add_row(G, zero_row<NV>());
  return make_delta<LPR, NV>(a, G, p_item, pb ? r.pb_row() : r.pa_row(), l);
}

// Adversarial terms of one pass: partner rows (batch-start values) plus their
// deltas: formed here for a solo partner, otherwise the one its clean half
// publishes in this batch (wait for it).
template <int LPR, int NV, int TEAM>
__device__ __forceinline__ void stream_adv_pass(const StepArgs& a, int is_item, const RowV<NV>& own,
                                                const RowV<NV>& ownp, const RecV& r0, const RecV& r1, bool a0,
                                                bool a1, RowV<NV> ra0, RowV<NV> rb0, RowV<NV> ra1,
                                                RowV<NV> rb1, uint32_t tag, int l, RowV<NV>& GA,
                                                int k = 0,  // k: diagnostic stamps only
                                                const float* g0 = nullptr, const float* g1 = nullptr) {
  RowV<NV> da0 = zero_row<NV>(), db0 = da0, da1 = da0, db1 = da0;
  const bool sa0 = a0 && r0.pa_solo(), sb0 = a0 && r0.pb_solo();
  const bool sa1 = a1 && r1.pa_solo(), sb1 = a1 && r1.pb_solo();
  const VSrc ta0 = a0 && !sa0 ? ver_at(vrow(a.ver_d, a, a.t, r0.pa_slot())) : 0;
  const VSrc tb0 = a0 && !sb0 ? ver_at(vrow(a.ver_d, a, a.t, r0.pb_slot())) : 0;
  const VSrc ta1 = a1 && !sa1 ? ver_at(vrow(a.ver_d, a, a.t, r1.pa_slot())) : 0;
  const VSrc tb1 = a1 && !sb1 ? ver_at(vrow(a.ver_d, a, a.t, r1.pb_slot())) : 0;
  bool pa0 = !ta0, pb0 = !tb0, pa1 = !ta1, pb1 = !tb1;
  if (__any(sa0)) {
    const RowV<NV> x = solo_delta<LPR, NV, TEAM>(a, is_item, own, r0, ra0, rb0, 0, l, g0);
    if (sa0) da0 = x;
  }
  if (__any(sb0)) {
    const RowV<NV> x = solo_delta<LPR, NV, TEAM>(a, is_item, own, r0, ra0, rb0, 1, l, g0);
    if (sb0) db0 = x;
  }
  if (__any(sa1)) {
    const RowV<NV> x = solo_delta<LPR, NV, TEAM>(a, is_item, own, r1, ra1, rb1, 0, l, g1);
    if (sa1) da1 = x;
  }
  if (__any(sb1)) {
    const RowV<NV> x = solo_delta<LPR, NV, TEAM>(a, is_item, own, r1, ra1, rb1, 1, l, g1);
    if (sb1) db1 = x;
  }
  STAMP(a.t, k, 6);
  {
    const VSrc src[4] = {ta0, tb0, ta1, tb1};
    RowV<NV>* const dst[4] = {&da0, &db0, &da1, &db1};
    bool ok[4] = {pa0, pb0, pa1, pb1};
    poll_rows<LPR, NV, 4>(a, src, dst, ok, tag, l);
  }
  STAMP(a.t, k, 7);
  ra0 = add_row(ra0, da0);
  rb0 = add_row(rb0, db0);
  ra1 = add_row(ra1, da1);
  rb1 = add_row(rb1, db1);
  occ_term<LPR, NV>(a, is_item, ownp, r0, ra0, rb0, a0, l, a.loss_adv, GA);
  if (__any(a1)) occ_term<LPR, NV>(a, is_item, ownp, r1, ra1, rb1, a1, l, a.loss_adv, GA);
}

// One unique row of batch a.t: clean half (utils.py:117, APR.py:180-191), its
// delta published as a version, then the adversarial half and Adagrad
// (APR.py:130-165,193-195).  The operation sequence is clean_slot's followed by
// adv_slot's, so the bits equal the two-kernel step's.  A slot of at most
// 2 TEAM occurrences (one pass) keeps its partner rows for the adversarial half;
// the Adagrad slot is fetched with the first gathers.
template <int LPR, int NV, int TEAM>
__device__ __forceinline__ void stream_slot(const StepArgs& a, int k, int m, int l, int leader, uint32_t tag) {
  STAMP(a.t, k, 0);
  const SlotRec sr = slot_header<LPR, TEAM>(a, k, m, leader);
  const SlotHdr& h = sr.h;
  if (h.count == 0) return;
  STAMP(a.t, k, 1);
  const int d = a.d;
  const VSrc own_s = ver_src(a, h.is_item ? a.Q : a.P, a.ver_w, h.own_row, h.own_src);
  const VSrc acc_s = m == 0 ? ver_src(a, h.is_item ? a.accQ : a.accP, a.ver_a, h.own_row, h.own_src) : 0;
  RowV<NV> own = zero_row<NV>(), acc = own, G = own;
  RowV<NV> ra0 = own, rb0 = own, ra1 = own, rb1 = own;
  RecV r0, r1;
  bool a0 = false, a1 = false;
  float lc0 = 0.f, lc1 = 0.f, gc0 = 0.f, gc1 = 0.f;
  {  // first pass: own row, Adagrad slot, partners in one wait
    a0 = m < h.count;
    a1 = TEAM + m < h.count;
    if (a0) r0 = occ_rec<TEAM>(a, sr, m, m);
    if (a1) r1 = occ_rec<TEAM>(a, sr, TEAM + m, m);
    const float* ptab = h.is_item ? a.P : a.Q;
    const VSrc sa0 = a0 ? ver_src(a, ptab, a.ver_w, r0.pa_row(), r0.pa_src()) : 0;
    const VSrc sb0 = a0 ? ver_src(a, a.Q, a.ver_w, r0.pb_row(), r0.pb_src()) : 0;
    const VSrc sa1 = a1 ? ver_src(a, ptab, a.ver_w, r1.pa_row(), r1.pa_src()) : 0;
    const VSrc sb1 = a1 ? ver_src(a, a.Q, a.ver_w, r1.pb_row(), r1.pb_src()) : 0;
    {
      const VSrc src[6] = {own_s, acc_s, sa0, sb0, sa1, sb1};
      RowV<NV>* const dst[6] = {&own, &acc, &ra0, &rb0, &ra1, &rb1};
      bool ok[6] = {false, m != 0, !a0, !a0, !a1, !a1};
      poll_rows<LPR, NV, 6>(a, src, dst, ok, tag, l);
    }
    STAMP(a.t, k, 2);
    // clean losses are stored at the end of the task: on gfx950 vmcnt counts
    // stores too, so a store here would hold up every later wait on a load
    occ_term<LPR, NV>(a, h.is_item, own, r0, ra0, rb0, a0, l, a.loss_clean, G, &lc0, &gc0);
    if (__any(a1)) occ_term<LPR, NV>(a, h.is_item, own, r1, ra1, rb1, a1, l, a.loss_clean, G, &lc1, &gc1);
  }
  // the clean half's end: batch-summed gradient, delta, delta published
  auto finish_clean = [&](RowV<NV>& Gc) -> RowV<NV> {
    team_allreduce_wave<LPR, TEAM, NV>(Gc);
    const RowV<NV> dl = make_delta<LPR, NV>(a, Gc, h.is_item, h.own_row, l);
    // a one-occurrence row's delta is never read: its readers form it (solo_delta)
    if (m == 0 && h.count > 1) store_ver<LPR, NV>(const_cast<u64*>(vrow(a.ver_d, a, a.t, k)), d, l, dl, tag);
    STAMP(a.t, k, 3);
    return add_row(own, dl);
  };
  RowV<NV> GA = zero_row<NV>();
  if (h.count <= 2 * TEAM) {  // one pass (wave-uniform): partner rows kept for the adversarial half
    const RowV<NV> ownp = finish_clean(G);
    stream_adv_pass<LPR, NV, TEAM>(a, h.is_item, own, ownp, r0, r1, a0, a1, ra0, rb0, ra1, rb1, tag, l, GA, k, &gc0,
                                   &gc1);
  } else {  // hot rows: more passes, partner rows re-read (versions never change)
    for (int base = 2 * TEAM; base < h.count; base += 2 * TEAM) {
      const int i0 = base + m, i1 = base + TEAM + m;
      const bool b0 = i0 < h.count, b1 = i1 < h.count;
      RecV q0, q1;
      if (b0) q0 = occ_rec_mem(a, h, k, i0);
      if (b1) q1 = occ_rec_mem(a, h, k, i1);
      RowV<NV> xa0 = zero_row<NV>(), xb0 = xa0, xa1 = xa0, xb1 = xa0;
      stream_partners<LPR, NV>(a, h.is_item, q0, q1, b0, b1, tag, l, xa0, xb0, xa1, xb1);
      occ_term<LPR, NV>(a, h.is_item, own, q0, xa0, xb0, b0, l, a.loss_clean, G);
      if (__any(b1)) occ_term<LPR, NV>(a, h.is_item, own, q1, xa1, xb1, b1, l, a.loss_clean, G);
    }
    const RowV<NV> ownp = finish_clean(G);
    for (int base = 0; base < h.count; base += 2 * TEAM) {
      const int i0 = base + m, i1 = base + TEAM + m;
      const bool b0 = i0 < h.count, b1 = i1 < h.count;
      RecV q0, q1;
      if (b0) q0 = occ_rec_mem(a, h, k, i0);
      if (b1) q1 = occ_rec_mem(a, h, k, i1);
      RowV<NV> xa0 = zero_row<NV>(), xb0 = xa0, xa1 = xa0, xb1 = xa0;
      stream_partners<LPR, NV>(a, h.is_item, q0, q1, b0, b1, tag, l, xa0, xb0, xa1, xb1);
      stream_adv_pass<LPR, NV, TEAM>(a, h.is_item, own, ownp, q0, q1, b0, b1, xa0, xb0, xa1, xb1, tag, l, GA);
    }
  }
  STAMP(a.t, k, 4);
  team_allreduce_wave<LPR, TEAM, NV>(GA);
  if (m == 0) {
    axpy_row(G, a.reg_adv, GA);
    RowV<NV> wout;
    adagrad_row(a, G, own, acc, h.count, wout);
    store_ver<LPR, NV>(const_cast<u64*>(vrow(a.ver_w, a, a.t, k)), d, l, wout, tag);
    store_ver<LPR, NV>(const_cast<u64*>(vrow(a.ver_a, a, a.t, k)), d, l, acc, tag);
  }
  if (!h.is_item && l == 0) {
    if (a0) a.loss_clean[r0.e_role()] = lc0;
    if (a1) a.loss_clean[r1.e_role()] = lc1;
  }
  STAMP(a.t, k, 5);
}

// A fused triplet of batch a.t (k_single's APR sequence): rows and Adagrad
// slots from their versions or the tables, results as versions of its 3 slots.
template <int LPR, int NV>
__device__ __forceinline__ void stream_single(const StepArgs& a, int b, int l, uint32_t tag) {
  const int64_t e = (int64_t)a.t * a.B + b;
  RecV r;
  r.a = r.b = r.c = make_int4(0, 0, 0, -1);
  if (b < a.B) r = load_rec(a.trec + e);
  const bool act = r.c.w == *a.gen_ptr && (r.c.y & 1);
  const int d = a.d;
  const int32_t u = r.a.x, i = r.a.y, j = r.a.z;
  const VSrc su = act ? ver_src(a, a.P, a.ver_w, u, r.b.z) : 0;
  const VSrc si = act ? ver_src(a, a.Q, a.ver_w, i, r.b.w) : 0;
  const VSrc sj = act ? ver_src(a, a.Q, a.ver_w, j, r.c.x) : 0;
  const VSrc cu_s = act ? ver_src(a, a.accP, a.ver_a, u, r.b.z) : 0;
  const VSrc ci_s = act ? ver_src(a, a.accQ, a.ver_a, i, r.b.w) : 0;
  const VSrc cj_s = act ? ver_src(a, a.accQ, a.ver_a, j, r.c.x) : 0;
  RowV<NV> p = zero_row<NV>(), qi = p, qj = p, cu = p, ci = p, cj = p;
  {
    const VSrc src[6] = {su, si, sj, cu_s, ci_s, cj_s};
    RowV<NV>* const dst[6] = {&p, &qi, &qj, &cu, &ci, &cj};
    bool ok[6] = {!act, !act, !act, !act, !act, !act};
    poll_rows<LPR, NV, 6>(a, src, dst, ok, tag, l);
  }
  if (!act) return;
  float g, loss;
  bpr_term(dot_row<LPR, NV>(p, qi) - dot_row<LPR, NV>(p, qj), a.clip_lo, a.clip_hi, g, loss);
  if (l == 0) a.loss_clean[e] = loss;
  RowV<NV> Gu = zero_row<NV>(), Gi = zero_row<NV>(), Gj = zero_row<NV>();
  axpy_row(Gu, g, qi);
  axpy_row(Gu, -g, qj);
  axpy_row(Gi, g, p);
  axpy_row(Gj, -g, p);
  const RowV<NV> pp = add_row(p, make_delta<LPR, NV>(a, Gu, 0, u, l));
  const RowV<NV> qip = add_row(qi, make_delta<LPR, NV>(a, Gi, 1, i, l));
  const RowV<NV> qjp = add_row(qj, make_delta<LPR, NV>(a, Gj, 1, j, l));
  float ga, la;
  bpr_term(dot_row<LPR, NV>(pp, qip) - dot_row<LPR, NV>(pp, qjp), a.clip_lo, a.clip_hi, ga, la);
  if (l == 0) a.loss_adv[e] = la;
  RowV<NV> Au = zero_row<NV>(), Ai = zero_row<NV>(), Aj = zero_row<NV>();
  axpy_row(Au, ga, qip);
  axpy_row(Au, -ga, qjp);
  axpy_row(Ai, ga, pp);
  axpy_row(Aj, -ga, pp);
  axpy_row(Gu, a.reg_adv, Au);
  axpy_row(Gi, a.reg_adv, Ai);
  axpy_row(Gj, a.reg_adv, Aj);
  RowV<NV> wu, wi, wj;
  adagrad_row(a, Gu, p, cu, 1, wu);
  adagrad_row(a, Gi, qi, ci, 1, wi);
  adagrad_row(a, Gj, qj, cj, 1, wj);
  store_ver<LPR, NV>(const_cast<u64*>(vrow(a.ver_w, a, a.t, r.a.w)), d, l, wu, tag);
  store_ver<LPR, NV>(const_cast<u64*>(vrow(a.ver_w, a, a.t, r.b.x)), d, l, wi, tag);
  store_ver<LPR, NV>(const_cast<u64*>(vrow(a.ver_w, a, a.t, r.b.y)), d, l, wj, tag);
  store_ver<LPR, NV>(const_cast<u64*>(vrow(a.ver_a, a, a.t, r.a.w)), d, l, cu, tag);
  store_ver<LPR, NV>(const_cast<u64*>(vrow(a.ver_a, a, a.t, r.b.x)), d, l, ci, tag);
  store_ver<LPR, NV>(const_cast<u64*>(vrow(a.ver_a, a, a.t, r.b.y)), d, l, cj, tag);
}

// The end of a streamed call, decided once: thread 0 of the deciding workgroup
// (the first to record an outcome for a.seq) moves the epoch on after a COMMIT,
// sets the group's gate after a verified failure (the host replays the call
// later) or step_err bit 0 after an unverified one (the call is dropped), and
// reports the outcome in the host-mapped status ring.  A verified failure leaves
// the epoch alone: the replay reads the same call counter (random delta) and
// bumps it as this call would have; the failed launch's granules keep their
// tag, and the next streamed launch of the context has a later one.
__device__ __forceinline__ void stream_decided(const StepArgs& a, bool failed) {
  uint32_t* ep = const_cast<uint32_t*>(a.epoch);
  if (!failed) {
    atomicAdd(ep, 1u);
  } else if (a.verify) {
    __hip_atomic_store(a.gate, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    atomicOr(a.step_err, 1);
    atomicAdd(ep, 1u);
  }
  if (a.verify && a.status)
    __hip_atomic_store(a.status + (a.seq & 7), ((unsigned long long)a.seq << 2) | (failed ? 1ull : 0ull),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Record the outcome of launch a.seq in the decide word unless one is recorded
// already; returns the recorded outcome (bit 0: failed) and, through *me,
// whether this call recorded it (the decider runs stream_decided).
__device__ __forceinline__ int stream_decide(const StepArgs& a, bool failed, bool* me) {
  const unsigned long long want = ((unsigned long long)a.seq << 1) | (failed ? 1ull : 0ull);
  // first attempt against the host's guess of the current word (one round trip)
  unsigned long long cur = a.decide_prev;
  *me = false;
  while ((cur >> 1) != (unsigned long long)a.seq) {
    unsigned long long exp = cur;
    if (__hip_atomic_compare_exchange_strong(a.decide, &exp, want, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT)) {
      cur = want;
      *me = true;
      break;
    }
    cur = exp;
  }
  return (int)(cur & 1);
}

// k_stream's tail (a.tail): every workgroup, once its four waves have no
// version store in flight, arrives: an agent-scope add to its shard counter
// (blockIdx % 8; the Guideline 16 counter form: every handed-off byte stored
// and loaded sc1), and the shard's last arrival adds to the top counter (one
// counter for 512 arrivals serialised ~6 us at the end of a call).  The last
// arrival at the top decides the launch's outcome (COMMIT unless a wait gave up
// or the launch was gated).  Workgroups [0, a.flushers) then poll the decide
// word (bounded: a launch that cannot become fully resident times out and
// fails) and, on COMMIT, write back the plan's final-slot list, lane-group gw
// taking entries gw, gw + G, ... two at a time: the row's last version in the
// launch -> weights and Adagrad slot (the granules k_stream_flush copies).
// Every other workgroup leaves after it has arrived.  The counters come in two
// sets used by alternate tail launches; each launch's block 0 zeroes the set
// the previous tail launch used (that launch has ended: kernel boundary).
template <int LPR>
__device__ __forceinline__ void stream_tail(const StepArgs& a, uint32_t tag, bool gated, int32_t fcnt) {
  __shared__ int s_out;
  const int flushers = max(1, min((int)gridDim.x, a.flushers));
  const bool flusher = (int)blockIdx.x < flushers;
  unsigned long long* set = a.arrive + a.tail_par * 144;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (a.tail_diag) atomicMax(a.tail_diag + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
    const int G = (int)gridDim.x, k = (int)(blockIdx.x & 7);
    const unsigned long long nk = (unsigned long long)(G / 8 + (k < G % 8 ? 1 : 0));
    const unsigned long long nsh = (unsigned long long)min(G, 8);
    bool last = false;
    if (__hip_atomic_fetch_add(set + 16 * (k + 1), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1 == nk)
      last = __hip_atomic_fetch_add(set, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1 == nsh;
    int out = -1;
    bool me = false;
    if (last) {
      if (a.tail_diag) a.tail_diag[2] = __builtin_amdgcn_s_memrealtime();
      const bool failed =
          gated || __hip_atomic_load(a.fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int32_t)a.seq;
      out = stream_decide(a, failed, &me);
      if (a.tail_diag) a.tail_diag[3] = __builtin_amdgcn_s_memrealtime();
      if (me) stream_decided(a, out != 0);
      if (a.tail_diag) a.tail_diag[4] = __builtin_amdgcn_s_memrealtime();
    }
    if (flusher && out < 0) {
      const int64_t lim = (int64_t)a.spin_limit * 8;
      for (int64_t it = 0;; ++it) {
        const unsigned long long v = __hip_atomic_load(a.decide, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((v >> 1) == (unsigned long long)a.seq) { out = (int)(v & 1); break; }
        if (it >= lim) {  // never all resident: fail the launch (and drain its late waves)
          __hip_atomic_store(a.fail, (int32_t)a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          out = stream_decide(a, true, &me);
          if (me) stream_decided(a, out != 0);
          break;
        }
        __builtin_amdgcn_s_sleep(8);
      }
    }
    s_out = out;
    if (a.tail_diag && flusher && blockIdx.x == 0) a.tail_diag[5] = __builtin_amdgcn_s_memrealtime();
  }
  __syncthreads();
  if (!flusher || s_out != 0) return;
  const int64_t groups = (int64_t)flushers * (blockDim.x / LPR);
  const int l = (int)(threadIdx.x & (LPR - 1));
  const int d4 = a.d >> 2;
  for (int64_t e = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / LPR; e < fcnt; e += 2 * groups) {
    const bool two = e + groups < fcnt;
    const int2 f0 = a.final_list[e];
    const int2 f1 = two ? a.final_list[e + groups] : f0;
    if (l >= d4) continue;
    u64 w[2][4], c[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int2 f = h ? f1 : f0;
      const u64* vw = a.ver_w + (int64_t)f.x * a.d;
      const u64* va = a.ver_a + (int64_t)f.x * a.d;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        w[h][k] = __hip_atomic_load((gu64_ptr)(vw + l + k * d4), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        c[h][k] = __hip_atomic_load((gu64_ptr)(va + l + k * d4), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h && !two) break;
      const int2 f = h ? f1 : f0;
      bool ok = true;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        ok = ok && (uint32_t)(w[h][k] >> 32) == tag && (uint32_t)(c[h][k] >> 32) == tag;
      if (!ok) atomicOr(a.step_err, 4);  // a final version missing after the barrier: never expected
      const int item = f.y < 0;
      const int64_t off = (int64_t)(f.y & 0x7fffffff) * a.d + 4 * l;
      *reinterpret_cast<float4*>((item ? a.Q : a.P) + off) =
          make_float4(__uint_as_float((uint32_t)w[h][0]), __uint_as_float((uint32_t)w[h][1]),
                      __uint_as_float((uint32_t)w[h][2]), __uint_as_float((uint32_t)w[h][3]));
      *reinterpret_cast<float4*>((item ? a.accQ : a.accP) + off) =
          make_float4(__uint_as_float((uint32_t)c[h][0]), __uint_as_float((uint32_t)c[h][1]),
                      __uint_as_float((uint32_t)c[h][2]), __uint_as_float((uint32_t)c[h][3]));
    }
  }
  if (a.tail_diag && blockIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (threadIdx.x == 0) a.tail_diag[6] = __builtin_amdgcn_s_memrealtime();
  }
}

// The work of a batch is a list of tasks: task k < S is slot k, task S + g the
// group of 64/LPR consecutive triplets g*64/LPR, ... (its fused ones).  With the
// plan's task lists (fusion on) a batch's tasks are its non-fused slots, then
// the groups that hold a fused triplet, and a launch has P = the largest task
// count of its batches positions; without them (fusion off) position p is task
// p of every batch, P = `positions`.  depth = min(max_depth, waves / P) waves
// share a position, taking every depth-th batch; a wave loads its next task
// while it runs the current one.  A gated launch (a failed verified call of the
// group awaits its replay) runs no task.
template <int LPR, int NV, int TEAM>
__global__ void __launch_bounds__(256, 2) k_stream(StepArgs a, int32_t positions) {
  static_assert(TEAM * LPR == 64, "k_stream: one wave per slot");
  const Geo<LPR, TEAM> q;
  const int lane = (int)(threadIdx.x & 63);
  int P = positions;
  if (a.task_list) {
    int mx = 1;
    for (int32_t t = a.first + lane; t < a.t_end; t += 64) mx = max(mx, a.task_cnt[t]);
#pragma unroll
    for (int o = 32; o; o >>= 1) mx = max(mx, __shfl_xor(mx, o, 64));
    P = mx;
  }
  const int waves = (int)((gridDim.x * (int64_t)blockDim.x) >> 6);
  const int depth = min(a.max_depth, waves / P);
  const int pos = q.wave % P, phase = q.wave / P;
  // version tag: the launch's seq, never reused by the context, so a granule a
  // late wave of a failed launch stores can never match a later launch
  const uint32_t tag = a.seq;
  const bool gated = *a.gate != 0;  // set by an earlier launch (kernel boundary)
  int32_t fcnt = 0;
  if (a.tail) {
    if ((int)blockIdx.x < a.flushers) fcnt = *a.final_cnt;  // the plan's (an earlier launch)
    if (blockIdx.x == 0 && threadIdx.x < 9)  // the counter set the previous tail launch used
      __hip_atomic_store(a.arrive + (a.tail_par ^ 1) * 144 + 16 * threadIdx.x, 0ull, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  if (a.tail_diag && blockIdx.x == 0 && threadIdx.x == 0) a.tail_diag[0] = __builtin_amdgcn_s_memrealtime();
  if (phase < depth && !gated) {
    int32_t t = a.first + phase;
    int32_t nxt = pos, ncnt = positions;
    if (a.task_list && t < a.t_end) {
      nxt = a.task_list[(int64_t)t * a.task_stride + pos];
      ncnt = a.task_cnt[t];
    }
    for (; t < a.t_end; t += depth) {
      const int32_t task = nxt, cnt = ncnt;
      if (a.task_list && t + depth < a.t_end) {
        nxt = a.task_list[(int64_t)(t + depth) * a.task_stride + pos];
        ncnt = a.task_cnt[t + depth];
      }
      if (pos >= cnt) continue;
      StepArgs b = a;
      b.t = t;
      if (task < a.S) {
        stream_slot<LPR, NV, TEAM>(b, task, q.m, q.l, q.leader, tag);
      } else {
        STAMP(t, task, 0);
        stream_single<LPR, NV>(b, (task - a.S) * (64 / LPR) + lane / LPR, q.l, tag);
        STAMP(t, task, 5);
      }
    }
  }
  if (a.tail) {
    stream_tail<LPR>(a, tag, gated, fcnt);
  } else if (a.tail_diag && (threadIdx.x & 63) == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    atomicMax(a.tail_diag + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
  }
}

// After a k_stream launch without a tail (a partial range of the plan, a plan
// without a final-slot list, a captured or timed call): the last version of
// every row the launch updated goes to the tables (weights and Adagrad slot).
// One lane-group per slot of the range: lane c gathers granules c, c + d/4,
// c + d/2, c + 3d/4 (elements 4c .. 4c+3 in the component-major order) of both
// versions and stores them as one float4 each, so every slot's loads are in
// flight at once.  A failed launch (a wait gave up: *fail == seq) or a gated one
// writes nothing; thread 0 decides the call's end as stream_tail's decider does.
template <int LPR>
__global__ void __launch_bounds__(256) k_stream_flush(StepArgs a, uint32_t* __restrict__ epoch) {
  constexpr int OPW = 64 / LPR;
  const int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t x = (gid >> 6) * OPW + (int64_t)((threadIdx.x & 63) / LPR);
  const int l = (int)(threadIdx.x & (LPR - 1));
  const int64_t n = (int64_t)(a.t_end - a.first) * a.S;
  // k_stream has ended (kernel boundary); the gate is only set below, by
  // thread 0, for this same failed call
  const bool failed = *a.fail == (int32_t)a.seq || *a.gate != 0;
  (void)epoch;
  if (gid == 0) stream_decided(a, failed);
  if (failed || x >= n) return;
  const int32_t t = a.first + (int32_t)(x / a.S);
  const int32_t k = (int32_t)(x - (int64_t)(t - a.first) * a.S);
  if (a.nextt[(int64_t)t * a.S + k] < a.t_end) return;  // a later batch of the launch has it
  const RecV r = load_rec(a.inl + ((int64_t)t * a.S + k) * a.R);
  if (r.gen() != *a.gen_ptr || (r.meta() & ACF_COUNT_MASK) == 0) return;
  const int d4 = a.d >> 2;
  if (l >= d4) return;
  const int item = (r.meta() & ACF_ITEM_BIT) != 0;
  const u64* vw = vrow(a.ver_w, a, t, k);
  const u64* va = vrow(a.ver_a, a, t, k);
  const float4 w = make_float4(__uint_as_float((uint32_t)vw[l]), __uint_as_float((uint32_t)vw[l + d4]),
                               __uint_as_float((uint32_t)vw[l + 2 * d4]), __uint_as_float((uint32_t)vw[l + 3 * d4]));
  const float4 c = make_float4(__uint_as_float((uint32_t)va[l]), __uint_as_float((uint32_t)va[l + d4]),
                               __uint_as_float((uint32_t)va[l + 2 * d4]), __uint_as_float((uint32_t)va[l + 3 * d4]));
  const int64_t off = (int64_t)r.own_row() * a.d + 4 * l;
  *reinterpret_cast<float4*>((item ? a.Q : a.P) + off) = w;
  *reinterpret_cast<float4*>((item ? a.accQ : a.accP) + off) = c;
}

// Large batches with fusion (one lane-group per slot): the slot work of batch t
// is the plan's list of its NON-fused slots and the write-back the list of the
// rows batch t-1 left in W scratch; a fixed set of slot waves strides over both
// (most slots belong to fused triplets and would only read their record).
// Piece p of hot slot k (pc = {k, p, pieces, piece base}): occurrences
// [p*count/pieces, (p+1)*count/pieces), one wave whose 64/LPR lane-groups take
// them as clean_slot's team members do (two per pass); the wave's sum goes to
// hot_part[base + p].  ADV: adv_slot's term (own + delta, partners + their
// deltas; the tables are current).  Losses of user occurrences as in the slot kernels.
template <int LPR, int NV, bool ADV>
__device__ __forceinline__ void hot_piece(const StepArgs& a, const int4 pc, int m, int l) {
  constexpr int TEAM = 64 / LPR;
  const int k = pc.x, d = a.d;
  const RecV r00 = load_rec(a.inl + ((int64_t)a.t * a.S + k) * a.R);
  SlotHdr h;
  h.count = r00.meta() & ACF_COUNT_MASK;
  h.is_item = (r00.meta() & ACF_ITEM_BIT) != 0;
  h.own_row = r00.own_row();
  h.own_src = r00.own_src();
  h.ovf = r00.ovf();
  const int o0 = (int)((int64_t)pc.y * h.count / pc.z), o1 = (int)((int64_t)(pc.y + 1) * h.count / pc.z);
  const float* own_tab = h.is_item ? a.Q : a.P;
  const float* ptab = h.is_item ? a.P : a.Q;
  const RowV<NV> own = ADV ? add_row(load_row<LPR, NV>(own_tab, h.own_row, d, l), load_row<LPR, NV>(a.delta, k, d, l))
                           : load_at<LPR, NV>(row_src(a, own_tab, h.own_row, h.own_src), d, l);
  RowV<NV> G = zero_row<NV>();
  for (int base = o0; base < o1; base += 2 * TEAM) {
    const int i0 = base + m, i1 = base + TEAM + m;
    const bool a0 = i0 < o1, a1 = i1 < o1;
    RowV<NV> ra0 = zero_row<NV>(), rb0 = zero_row<NV>(), ra1 = zero_row<NV>(), rb1 = zero_row<NV>();
    RecV r0, r1;
    if (a0) r0 = occ_rec_mem(a, h, k, i0);
    if (a1) r1 = occ_rec_mem(a, h, k, i1);
    if (ADV) {
      if (a0) {
        ra0 = add_row(load_row<LPR, NV>(ptab, r0.pa_row(), d, l), load_row<LPR, NV>(a.delta, r0.pa_slot(), d, l));
        rb0 = add_row(load_row<LPR, NV>(a.Q, r0.pb_row(), d, l), load_row<LPR, NV>(a.delta, r0.pb_slot(), d, l));
      }
      if (a1) {
        ra1 = add_row(load_row<LPR, NV>(ptab, r1.pa_row(), d, l), load_row<LPR, NV>(a.delta, r1.pa_slot(), d, l));
        rb1 = add_row(load_row<LPR, NV>(a.Q, r1.pb_row(), d, l), load_row<LPR, NV>(a.delta, r1.pb_slot(), d, l));
      }
    } else {
      if (a0) {
        ra0 = load_at<LPR, NV>(row_src(a, ptab, r0.pa_row(), r0.pa_src()), d, l);
        rb0 = load_at<LPR, NV>(row_src(a, a.Q, r0.pb_row(), r0.pb_src()), d, l);
      }
      if (a1) {
        ra1 = load_at<LPR, NV>(row_src(a, ptab, r1.pa_row(), r1.pa_src()), d, l);
        rb1 = load_at<LPR, NV>(row_src(a, a.Q, r1.pb_row(), r1.pb_src()), d, l);
      }
    }
    occ_term<LPR, NV>(a, h.is_item, own, r0, ra0, rb0, a0, l, ADV ? a.loss_adv : a.loss_clean, G);
    if (__any(a1)) occ_term<LPR, NV>(a, h.is_item, own, r1, ra1, rb1, a1, l, ADV ? a.loss_adv : a.loss_clean, G);
  }
  team_allreduce<LPR, TEAM, NV>(G);
  if (m == 0) store_row<LPR, NV>(a.hot_part, (int64_t)pc.w + pc.y, d, l, G);
}

// piece waves of a list kernel (wave index hw in [0, hot_waves)): stride over the batch's pieces
template <int LPR, int NV, bool ADV>
__device__ __forceinline__ void hot_piece_waves(const StepArgs& a, int hw) {
  const int lane = threadIdx.x & 63, m = lane / LPR, l = lane & (LPR - 1);
  const int n = a.hot.pcnt[a.t];
  const int4* pl = a.hot.piece + (int64_t)a.t * a.hot.piece_stride;
  for (int x = hw; x < n; x += a.hot_waves) hot_piece<LPR, NV, ADV>(a, pl[x], m, l);
}

// Hot-slot combine: one workgroup per hot slot (strided).  Lane-group g of the
// 256/LPR sums pieces g, g + 256/LPR, ... in turn; group 0 then adds the groups'
// sums in group order and finishes the slot as the slot kernels' team leader does:
// MODE 0 (APR clean): G -> g0, delta; MODE 1 (BPR): Adagrad on G;
// MODE 2 (APR adversarial): g0 + reg_adv * G -> Adagrad.  Rows go to W scratch.
// a piece sum read back: plain loads, or (SC1) device-scope loads of the 8-B
// halves of each float4 (the pieces were stored write-through in this launch by
// other workgroups: MI355X guide, Guideline 16)
template <int LPR, int NV, bool SC1>
__device__ __forceinline__ RowV<NV> load_piece(const float* __restrict__ base, int64_t row, int d, int l) {
  if constexpr (!SC1) {
    return load_row<LPR, NV>(base, row, d, l);
  } else {
    RowV<NV> r;
    const float* p = base + row * (int64_t)d;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int c = l + LPR * v;
      if (c * 4 < d) {
        const u64 lo = __hip_atomic_load((const __attribute__((address_space(1))) u64*)(p + c * 4),
                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const u64 hi = __hip_atomic_load((const __attribute__((address_space(1))) u64*)(p + c * 4 + 2),
                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        r.v[v] = make_float4(__uint_as_float((uint32_t)lo), __uint_as_float((uint32_t)(lo >> 32)),
                             __uint_as_float((uint32_t)hi), __uint_as_float((uint32_t)(hi >> 32)));
      } else {
        r.v[v] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    return r;
  }
}

// One hot slot e = {slot, pieces, piece base, count} by a 256-thread workgroup:
// lane-group g of the 256/LPR sums pieces g, g + 256/LPR, ... in turn; group 0
// then adds the groups' sums in group order and finishes the slot as the slot
// kernels' team leader does: MODE 0 (APR clean): G -> g0, delta; MODE 1 (BPR):
// Adagrad on G; MODE 2 (APR adversarial): g0 + reg_adv * G -> Adagrad.  Rows go
// to W scratch, or to their table in place (a.inplace).  Ends with a barrier.
template <int LPR, int NV, int MODE, bool SC1>
__device__ __forceinline__ void hot_combine_slot(const StepArgs& a, const int4 e, float4* __restrict__ red) {
  constexpr int NG = 256 / LPR;
  const int g = threadIdx.x / LPR, l = threadIdx.x & (LPR - 1), d = a.d;
  RowV<NV> G = zero_row<NV>();
  for (int p0 = g; p0 < e.y; p0 += 8 * NG) {  // 8 pieces' loads in flight per lane-group; the adds in order
    RowV<NV> x[8];
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (p0 + q * NG < e.y) x[q] = load_piece<LPR, NV, SC1>(a.hot_part, (int64_t)e.z + p0 + q * NG, d, l);
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (p0 + q * NG < e.y) G = add_row(G, x[q]);
  }
#pragma unroll
  for (int v = 0; v < NV; ++v) red[v * 256 + threadIdx.x] = G.v[v];
  __syncthreads();
  if (g == 0) {
    for (int gg = 1; gg < NG; ++gg) {
      RowV<NV> o;
#pragma unroll
      for (int v = 0; v < NV; ++v) o.v[v] = red[v * 256 + gg * LPR + l];
      G = add_row(G, o);
    }
    const int k = e.x;
    const RecV r = load_rec(a.inl + ((int64_t)a.t * a.S + k) * a.R);
    const int is_item = (r.meta() & ACF_ITEM_BIT) != 0;
    const int32_t row = r.own_row();
    const float* own_tab = is_item ? a.Q : a.P;
    float* acc_tab = is_item ? a.accQ : a.accP;
    if (a.shard && is_item && a.xbuf)  // the owner's partial sum, straight to its exchange row
      store_row_wt<LPR, NV>(a.xbuf, a.xmap[k - (a.xubs[1] - a.xubs[0])], d, l, G);
    if (MODE != 0 && a.shard && is_item) {  // partial item sum for the owner
      store_row<LPR, NV>(a.g0, k, d, l, G);
    } else if (MODE == 0) {
      const RowV<NV> dl = make_delta<LPR, NV>(a, G, is_item, row, l);
      store_row<LPR, NV>(a.g0, k, d, l, G);
      store_row<LPR, NV>(a.delta, k, d, l, dl);
    } else {
      RowV<NV> acc = load_row<LPR, NV>(acc_tab, row, d, l);
      RowV<NV> wout;
      if (MODE == 1) {
        const RowV<NV> own = load_at<LPR, NV>(row_src(a, own_tab, row, r.own_src()), d, l);
        adagrad_row(a, G, own, acc, e.w, wout);
      } else {
        RowV<NV> G0 = load_row<LPR, NV>(a.g0, k, d, l);
        axpy_row(G0, a.reg_adv, G);
        const RowV<NV> own = load_row<LPR, NV>(own_tab, row, d, l);
        adagrad_row(a, G0, own, acc, e.w, wout);
      }
      store_row<LPR, NV>(acc_tab, row, d, l, acc);
      // (a shard pass with the write-back in this launch: nothing reads the user
      // rows any more, so a hot user slot goes straight to its table)
      if (a.inplace || (a.xflush && !is_item)) store_row<LPR, NV>(is_item ? a.Q : a.P, row, d, l, wout);
      else store_row<LPR, NV>(a.wnew_cur, k, d, l, wout);
    }
  }
  __syncthreads();
}

// Export workgroups of the shard-mode combine: one lane-group per item slot of
// the batch (strided), the non-hot slots' partial sums g0 -> their exchange rows
// (hot slots are exported by the workgroup that combines them).
template <int LPR, int NV>
__device__ __forceinline__ void shard_export_rest(const StepArgs& a, int bx) {
  const int l = threadIdx.x & (LPR - 1), d = a.d;
  const int nU = a.xubs[1] - a.xubs[0], nI = a.xibs[1] - a.xibs[0];
  const int xb = a.xblocks - a.xflush;  // item-export workgroups, then user write-back ones
  if (bx >= xb) {
    const int ustride = a.xflush * (256 / LPR);
    for (int k = (bx - xb) * (256 / LPR) + (int)threadIdx.x / LPR; k < nU; k += ustride) {
      const RecV r = load_rec(a.inl + ((int64_t)a.t * a.S + k) * a.R);
      const int cnt = r.meta() & ACF_COUNT_MASK;
      if (!(r.meta() & ACF_SINGLE_BIT) && cnt > ACF_HOT_MIN) continue;  // hot: written by its combine
      store_row<LPR, NV>(a.P, r.own_row(), d, l, load_row<LPR, NV>(a.wnew_cur, k, d, l));
    }
    return;
  }
  const int n = nI < a.xn ? nI : a.xn;
  const int stride = xb * (256 / LPR);
  for (int w = bx * (256 / LPR) + (int)threadIdx.x / LPR; w < n; w += stride) {
    const int k = nU + w;
    const RecV r = load_rec(a.inl + ((int64_t)a.t * a.S + k) * a.R);
    const int cnt = r.meta() & ACF_COUNT_MASK;
    if (!(r.meta() & ACF_SINGLE_BIT) && cnt > ACF_HOT_MIN) continue;  // a hot slot: its combine exports it
    store_row_wt<LPR, NV>(a.xbuf, a.xmap[w], d, l, load_row<LPR, NV>(a.g0, k, d, l));
  }
}

// Hot-slot combine: one workgroup per hot slot (strided); see hot_combine_slot.
// With export (shard mode), the last a.xblocks workgroups run shard_export_rest.
template <int LPR, int NV, int MODE>
__global__ void __launch_bounds__(256) k_hot_combine(StepArgs a) {
  __shared__ float4 red[NV * 256];
  const int cb = (int)gridDim.x - a.xblocks;  // combining workgroups
  if ((int)blockIdx.x >= cb) {
    shard_export_rest<LPR, NV>(a, (int)blockIdx.x - cb);
    return;
  }
  const int n = a.hot.cnt[a.t];
  const int4* hl = a.hot.list + (int64_t)a.t * a.hot.hot_stride;
  for (int hx = blockIdx.x; hx < n; hx += cb) hot_combine_slot<LPR, NV, MODE, false>(a, hl[hx], red);
}

template <int LPR, int NV, bool FUSE_APPLY>
__global__ void __launch_bounds__(256) k_clean_list(StepArgs a) {
  const int wave = (int)((blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63, g = lane / LPR, l = lane & (LPR - 1);
  if (wave >= a.slot_waves) {  // piece waves, then (BPR) fused-triplet waves
    const int hw = wave - a.slot_waves;
    if (hw < a.hot_waves) hot_piece_waves<LPR, NV, false>(a, hw);
    else if (FUSE_APPLY) k_single<LPR, NV, false>(a, (hw - a.hot_waves) * (64 / LPR) + g, l);
    return;
  }
  const int ngroups = a.slot_waves * (64 / LPR), gid = wave * (64 / LPR) + g;
  if (a.prev_valid) {
    const int n = a.flush_cnt[a.t - 1];
    const int32_t* lst = a.flush_list + (int64_t)(a.t - 1) * a.S;
    for (int x = gid; x < n; x += ngroups) flush_slot(a, a.t - 1, a.wnew_prev, lst[x], l, LPR);
  }
  const int n = a.slot_cnt[a.t];
  const int32_t* lst = a.slot_list + (int64_t)a.t * a.S;
  for (int x = gid; x < n; x += ngroups) clean_slot<LPR, NV, FUSE_APPLY, 1>(a, lst[x], 0, l, g * LPR, wave);
}

template <int LPR, int NV>
__global__ void __launch_bounds__(256) k_adv_list(StepArgs a) {
  const int wave = (int)((blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63, g = lane / LPR, l = lane & (LPR - 1);
  if (wave >= a.slot_waves) {  // piece waves, then fused-triplet waves
    const int hw = wave - a.slot_waves;
    if (hw < a.hot_waves) hot_piece_waves<LPR, NV, true>(a, hw);
    else k_single<LPR, NV, true>(a, (hw - a.hot_waves) * (64 / LPR) + g, l);
    return;
  }
  const int ngroups = a.slot_waves * (64 / LPR), gid = wave * (64 / LPR) + g;
  const int n = a.slot_cnt[a.t];
  const int32_t* lst = a.slot_list + (int64_t)a.t * a.S;
  for (int x = gid; x < n; x += ngroups) adv_slot<LPR, NV, 1>(a, lst[x], 0, l, g * LPR, wave);
}

// ---------------------------------------------------------------------------
// Triplet-centric list step (packed plans with fusion, not shard mode: large
// batches).  The slot kernels above compute a triplet's BPR term once per row
// it touches (its user slot and both item slots each re-read the partner rows
// and deltas).  Here every triplet's lane-group computes its term ONCE:
//  - a row that occurs once in the batch ("single") is stepped by its triplet
//    in registers (k_single's operation sequence: delta, adversarial term,
//    Adagrad), written in place or to W scratch by the fused rule;
//  - a row with more occurrences ("shared") gets the triplet's rounded
//    products as CONTRIBUTIONS (users: the positive and the negative branch,
//    items: one vector), stored at the occurrence's CSR position; a combine
//    sums a slot's contributions in occurrence order -- exactly the additions
//    the one-lane-group slot path makes, so the bits are the slot path's --
//    and finishes the row (delta, or Adagrad into W scratch).  Slots with more
//    than ACF_HOT_MIN occurrences sum their contributions in pieces, then
//    k_hot_combine.
// Per batch (APR): k_tri_clean (write-back of t-1, clean contributions) ->
// k_tri_combine<0> + k_hot_combine<0> (shared deltas) -> k_tri_adv (every
// triplet: fused ones as k_single, the others as above) -> k_tri_combine<2> +
// k_hot_combine<2> (shared Adagrad).  BPR: k_tri_clean<BPR> -> combine<1>.
// ---------------------------------------------------------------------------
// The triplet-centric kernels' contributions and the combine's finished
// small-slot rows are stored write-through (sc1): a launch then ends with fewer
// dirty L2 lines to write back at its boundary (MI355X guide, "boundary": + B /
// 6 TB/s for B dirty bytes).  r05 same-box A/B at configs[4] d = 64: 726-727M ->
// 737-740M triplets/s; the in-place table writes of k_tri_adv stay write-back
// (write-through there was 0.5% slower); d = 128 flat
// (profiles/r05/store_writethrough_ab.json).
#define TRI_SU 16
#define TRI_SI 32
#define TRI_SJ 64

// the tag k_tri_cadv's finishers publish per slot and its triplets wait for:
// unique per call (the call counter, bumped by the flush at the end of every
// call) and batch
__device__ __forceinline__ unsigned long long ready_tag(const StepArgs& a) {
  return ((unsigned long long)*a.epoch << 32) | (uint32_t)a.t;
}


__device__ __forceinline__ float* tri_cu(const StepArgs& a) { return a.contrib; }
__device__ __forceinline__ float* tri_ci(const StepArgs& a) { return a.contrib + (int64_t)2 * a.B * a.d; }

// PASS 0: APR clean (shared rows: clean contributions; single rows: nothing,
// k_tri_adv recomputes their term); 1: BPR (single rows: Adagrad; shared:
// contributions); 2: APR adversarial.
// Shard mode (r05, distributed.ShardedAPR's local passes): an item's sum here is
// a partial one for its owner, so a single item row is neither perturbed nor
// stepped locally: its one product is its partial sum, stored straight to its
// exchange row (the slot path's 0 + product), and pass 2 reads the owners'
// item deltas from theirs; users are complete locally and step as above.
template <int LPR, int NV, int PASS, bool MERGED = false>
__device__ __forceinline__ void tri_triplet_r(const StepArgs& a, int b, int l, const RecV& r, const int4 ps) {
  if (b >= a.B) return;
  if (r.c.w != *a.gen_ptr) return;
  const int64_t e = r.c.z;  // the triplet (its losses); b is its place in the plan (hash plans: fused first)
  const int flags = r.c.y;
  // a fused triplet (all three rows single) takes the same code as the others
  // (k_single's operation sequence), so a wave's lane-groups do not diverge
  // into two paths; its clean pass is empty (PASS 2 recomputes the term)
  if (PASS == 0 && (flags & 1)) return;
  const int d = a.d;
  const int32_t u = r.a.x, i = r.a.y, j = r.a.z;
  const int32_t ku = r.a.w, ki = r.b.x, kj = r.b.y;
  const bool su = (flags & TRI_SU) != 0, si = (flags & TRI_SI) != 0, sj = (flags & TRI_SJ) != 0;
  const bool ai = si && !a.shard, aj = sj && !a.shard;  // single item rows stepped here
  RowV<NV> p, qi, qj;
  if (PASS == 2) {  // the tables are current (k_tri_clean wrote back batch t-1)
    p = load_row<LPR, NV>(a.P, u, d, l);
    qi = load_row<LPR, NV>(a.Q, i, d, l);
    qj = load_row<LPR, NV>(a.Q, j, d, l);
  } else {
    p = load_at<LPR, NV>(row_src(a, a.P, u, r.b.z), d, l);
    qi = load_at<LPR, NV>(row_src(a, a.Q, i, r.b.w), d, l);
    qj = load_at<LPR, NV>(row_src(a, a.Q, j, r.c.x), d, l);
  }
  RowV<NV> cu, ci, cj, du, di, dj;  // Adagrad slots of the single rows, deltas of the shared ones
  if (PASS != 0) {
    if (su) cu = load_row<LPR, NV>(a.accP, u, d, l);
    if (ai) ci = load_row<LPR, NV>(a.accQ, i, d, l);
    if (aj) cj = load_row<LPR, NV>(a.accQ, j, d, l);
  }
  if (PASS == 2) {  // issued with the row loads, not after the clean term
    // (MERGED, k_tri_cadv: the deltas were stored in this launch by other
    // workgroups -- device-scope loads, after their tags, tri_wait_ready)
    if (!su) du = load_piece<LPR, NV, MERGED>(a.delta, ku, d, l);
    if (a.shard) {  // items: the owners' deltas, straight from the exchange rows
      di = load_row<LPR, NV>(a.xdelta, a.xdmap[i], d, l);
      dj = load_row<LPR, NV>(a.xdelta, a.xdmap[j], d, l);
    } else {
      if (!si) di = load_piece<LPR, NV, MERGED>(a.delta, ki, d, l);
      if (!sj) dj = load_piece<LPR, NV, MERGED>(a.delta, kj, d, l);
    }
  }
  const int64_t lu = ps.x - (int64_t)a.t * a.B, li = ps.y - (int64_t)a.t * 2 * a.B,
                lj = ps.z - (int64_t)a.t * 2 * a.B;
  float* cuB = tri_cu(a);
  float* ciB = tri_ci(a);
  float g, loss;
  bpr_term(dot_row<LPR, NV>(p, qi) - dot_row<LPR, NV>(p, qj), a.clip_lo, a.clip_hi, g, loss);
  if ((PASS != 2 || (flags & 1)) && l == 0) a.loss_clean[e] = loss;
  if (PASS != 2) {  // clean contributions of the shared rows
    if (!su) {
      store_row_wt<LPR, NV>(cuB, 2 * lu, d, l, scale_row(qi, g));
      store_row_wt<LPR, NV>(cuB, 2 * lu + 1, d, l, scale_row(qj, -g));
    }
    if (!si) store_row_wt<LPR, NV>(ciB, li, d, l, scale_row(p, g));
    else if (a.shard) store_row_wt<LPR, NV>(a.xbuf, a.xmap[i], d, l, scale_row(p, g));
    if (!sj) store_row_wt<LPR, NV>(ciB, lj, d, l, scale_row(p, -g));
    else if (a.shard) store_row_wt<LPR, NV>(a.xbuf, a.xmap[j], d, l, scale_row(p, -g));
    if (PASS == 0) return;
  }
  // the single rows' clean gradients (k_single's order)
  RowV<NV> Gu = zero_row<NV>(), Gi = zero_row<NV>(), Gj = zero_row<NV>();
  axpy_row(Gu, g, qi);
  axpy_row(Gu, -g, qj);
  axpy_row(Gi, g, p);
  axpy_row(Gj, -g, p);
  if (PASS == 2) {
    if (su) du = make_delta<LPR, NV>(a, Gu, 0, u, l);
    if (ai) di = make_delta<LPR, NV>(a, Gi, 1, i, l);
    if (aj) dj = make_delta<LPR, NV>(a, Gj, 1, j, l);
    const RowV<NV> pp = add_row(p, du), qip = add_row(qi, di), qjp = add_row(qj, dj);
    float ga, la;
    bpr_term(dot_row<LPR, NV>(pp, qip) - dot_row<LPR, NV>(pp, qjp), a.clip_lo, a.clip_hi, ga, la);
    if (l == 0) a.loss_adv[e] = la;
    if (!su) {
      store_row_wt<LPR, NV>(cuB, 2 * lu, d, l, scale_row(qip, ga));
      store_row_wt<LPR, NV>(cuB, 2 * lu + 1, d, l, scale_row(qjp, -ga));
    }
    if (!si) store_row_wt<LPR, NV>(ciB, li, d, l, scale_row(pp, ga));
    else if (a.shard) store_row_wt<LPR, NV>(a.xbuf, a.xmap[i], d, l, scale_row(pp, ga));
    if (!sj) store_row_wt<LPR, NV>(ciB, lj, d, l, scale_row(pp, -ga));
    else if (a.shard) store_row_wt<LPR, NV>(a.xbuf, a.xmap[j], d, l, scale_row(pp, -ga));
    if (su) {
      RowV<NV> Au = zero_row<NV>();
      axpy_row(Au, ga, qip);
      axpy_row(Au, -ga, qjp);
      axpy_row(Gu, a.reg_adv, Au);
    }
    if (ai) {
      RowV<NV> Ai = zero_row<NV>();
      axpy_row(Ai, ga, pp);
      axpy_row(Gi, a.reg_adv, Ai);
    }
    if (aj) {
      RowV<NV> Aj = zero_row<NV>();
      axpy_row(Aj, -ga, pp);
      axpy_row(Gj, a.reg_adv, Aj);
    }
  }
  // Adagrad of the single rows: in place unless pending from t-1 or read by t+1
  if (su) {
    RowV<NV> w;
    adagrad_row(a, Gu, p, cu, 1, w);
    store_row<LPR, NV>(a.accP, u, d, l, cu);
    store_row<LPR, NV>((flags & 2) ? a.P : a.wnew_cur, (flags & 2) ? u : ku, d, l, w);
  }
  if (ai) {
    RowV<NV> w;
    adagrad_row(a, Gi, qi, ci, 1, w);
    store_row<LPR, NV>(a.accQ, i, d, l, ci);
    store_row<LPR, NV>((flags & 4) ? a.Q : a.wnew_cur, (flags & 4) ? i : ki, d, l, w);
  }
  if (aj) {
    RowV<NV> w;
    adagrad_row(a, Gj, qj, cj, 1, w);
    store_row<LPR, NV>(a.accQ, j, d, l, cj);
    store_row<LPR, NV>((flags & 8) ? a.Q : a.wnew_cur, (flags & 8) ? j : kj, d, l, w);
  }
}

// triplet b's record and CSR positions (loaded together, before the rows)
__device__ __forceinline__ void tri_rec(const StepArgs& a, int b, RecV& r, int4& ps) {
  r.a = r.b = r.c = make_int4(0, 0, 0, -1);
  ps = make_int4(0, 0, 0, 0);
  if (b < a.B) {
    const int64_t e = (int64_t)a.t * a.B + b;
    r = load_rec(a.trec + e);
    ps = a.tpos[e];
  }
}

// tri_gpw(NV) groups of 64/LPR consecutive triplets per wave (d <= 256: two):
// both groups' records are loaded up front, so the second group's rows are
// addressed without another dependent round trip, and the grid runs half as
// many wave rounds
__host__ __device__ constexpr int tri_gpw(int nv) { return nv == 1 ? 2 : 1; }

// k_tri_cadv: the wave's triplets wait until the shared slots whose deltas they
// read carry this batch's tag (finished by the combine part of the launch,
// dispatched before every triplet wave, so the wait always ends); a lane-group's
// lanes poll its triplets' (up to) 3 x GPW slots.  All-single (fused) triplets
// wait for nothing.  Bounded: a give-up sets step_err bit 0.
template <int LPR, int GPW>
__device__ __forceinline__ void tri_wait_ready(const StepArgs& a, const int* bs, const RecV* r, int l) {
  const unsigned long long tag = ready_tag(a);
  const int32_t gen = *a.gen_ptr;
  constexpr int NQ = (3 * GPW + LPR - 1) / LPR;
  int32_t slot[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) slot[q] = -1;
  // candidate c = 3x + which (x: the wave's group, which: u / i / j) goes to lane
  // c % LPR, entry c / LPR -- every index a compile-time constant (no scratch)
#pragma unroll
  for (int x = 0; x < GPW; ++x) {
    const bool live = bs[x] < a.B && r[x].c.w == gen;
    const int flags = r[x].c.y;
#pragma unroll
    for (int which = 0; which < 3; ++which) {
      const int c = 3 * x + which;
      if (l != c % LPR || !live) continue;
      const int mask = which == 0 ? TRI_SU : which == 1 ? TRI_SI : TRI_SJ;
      const int32_t k = which == 0 ? r[x].a.w : which == 1 ? r[x].b.x : r[x].b.y;
      if (!(flags & mask)) slot[c / LPR] = k;
    }
  }
  bool need = false;
#pragma unroll
  for (int q = 0; q < NQ; ++q) need |= slot[q] >= 0;
  if (!__any(need)) return;
  for (int it = 0;; ++it) {
    bool ok = true;
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      if (slot[q] >= 0 && __hip_atomic_load(a.ready + slot[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != tag)
        ok = false;
    if (__all(ok)) return;
    if (it >= a.spin_limit) {
      if ((threadIdx.x & 63) == 0) atomicOr(a.step_err, 1);
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// triplets at places [boff + tw * GPW * OPW, ...) below bend (default: the batch)
template <int LPR, int NV, int PASS, bool MERGED = false>
__device__ __forceinline__ void tri_triplets(const StepArgs& a, int tw, int lane, int boff = 0, int bend = -1) {
  constexpr int OPW = 64 / LPR, GPW = tri_gpw(NV);
  const int b0 = boff + tw * GPW * OPW + lane / LPR;
  RecV r[GPW];
  int4 ps[GPW];
  int bs[GPW];
#pragma unroll
  for (int x = 0; x < GPW; ++x) {
    bs[x] = b0 + x * OPW;
    if (bend >= 0 && bs[x] >= bend) bs[x] = a.B;  // past the range: no triplet
    tri_rec(a, bs[x], r[x], ps[x]);
  }
  if (MERGED) tri_wait_ready<LPR, GPW>(a, bs, r, lane & (LPR - 1));
#pragma unroll
  for (int x = 0; x < GPW; ++x) tri_triplet_r<LPR, NV, PASS, MERGED>(a, bs[x], lane & (LPR - 1), r[x], ps[x]);
}

// header of shared slot k: count, side, own row, source, local CSR base
struct TriSlot {
  int32_t count, is_item, row, src;
  int64_t base;
};

__device__ __forceinline__ TriSlot tri_slot(const StepArgs& a, int k) {
  const RecV r = load_rec(a.inl + ((int64_t)a.t * a.S + k) * a.R);
  TriSlot h;
  h.count = (r.gen() == *a.gen_ptr) ? (r.meta() & ACF_COUNT_MASK) : 0;
  h.is_item = (r.meta() & ACF_ITEM_BIT) != 0;
  h.row = r.own_row();
  h.src = r.own_src();
  h.base = (int64_t)r.ovf() - (int64_t)a.t * (h.is_item ? 2 : 1) * a.B;
  return h;
}

// contributions of occurrences [o0, o1) of a slot, added in order (a user
// occurrence: its positive, then its negative branch, as the slot path's axpys)
template <int LPR, int NV>
__device__ __forceinline__ void tri_add(const StepArgs& a, const TriSlot& h, int o0, int o1, int step, int l,
                                        RowV<NV>& G) {
  const int d = a.d;
  if (h.is_item) {
    const float* c = tri_ci(a);
    for (int o = o0; o < o1; o += step) G = add_row(G, load_row<LPR, NV>(c, h.base + o, d, l));
  } else {
    const float* c = tri_cu(a);
    for (int o = o0; o < o1; o += step) {
      G = add_row(G, load_row<LPR, NV>(c, 2 * (h.base + o), d, l));
      G = add_row(G, load_row<LPR, NV>(c, 2 * (h.base + o) + 1, d, l));
    }
  }
}

// tri_add with a lane-group's loads issued together, Q occurrences at a time;
// the additions keep tri_add's order (same bits)
template <int LPR, int NV>
__device__ __forceinline__ void tri_add_q(const StepArgs& a, const TriSlot& h, int o0, int o1, int step, int l,
                                          RowV<NV>& G) {
  constexpr int Q = 4;
  const int d = a.d;
  for (int ob = o0; ob < o1; ob += Q * step) {
    if (h.is_item) {
      const float* c = tri_ci(a);
      RowV<NV> x[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if (ob + q * step < o1) x[q] = load_row<LPR, NV>(c, h.base + ob + q * step, d, l);
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if (ob + q * step < o1) G = add_row(G, x[q]);
    } else {
      const float* c = tri_cu(a);
      RowV<NV> x[2 * Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        if (ob + q * step < o1) {
          x[2 * q] = load_row<LPR, NV>(c, 2 * (h.base + ob + q * step), d, l);
          x[2 * q + 1] = load_row<LPR, NV>(c, 2 * (h.base + ob + q * step) + 1, d, l);
        }
      }
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        if (ob + q * step < o1) {
          G = add_row(G, x[2 * q]);
          G = add_row(G, x[2 * q + 1]);
        }
      }
    }
  }
}

// finish a shared row from its summed G (as the slot kernels' team leader and
// k_hot_combine do): MODE 0 g0 + delta, 1 BPR Adagrad, 2 APR Adagrad
template <int LPR, int NV, int MODE>
__device__ __forceinline__ void tri_finish(const StepArgs& a, int k, const TriSlot& h, RowV<NV>& G, int l) {
  const int d = a.d;
  // (the exchange rows are stored write-through: r05 same-box A/B, configs[4]
  // split step 0.403-0.409 -> 0.398-0.401 ms; the owner kernels' outputs
  // write-through were slower, 0.47 ms: profiles/r05/shard_writethrough_ab.json)
  if (a.shard && h.is_item) {  // shard mode: the partial item sum, straight to its exchange row
    store_row_wt<LPR, NV>(a.xbuf, a.xmap[h.row], d, l, G);
    return;
  }
  if (MODE == 0) {
    const RowV<NV> dl = make_delta<LPR, NV>(a, G, h.is_item, h.row, l);
    store_row_wt<LPR, NV>(a.g0, k, d, l, G);
    store_row_wt<LPR, NV>(a.delta, k, d, l, dl);
    return;
  }
  float* acc_tab = h.is_item ? a.accQ : a.accP;
  RowV<NV> acc = load_row<LPR, NV>(acc_tab, h.row, d, l);
  RowV<NV> wout;
  if (MODE == 1) {
    const RowV<NV> own = load_at<LPR, NV>(row_src(a, h.is_item ? a.Q : a.P, h.row, h.src), d, l);
    adagrad_row(a, G, own, acc, h.count, wout);
  } else {
    RowV<NV> G0 = load_row<LPR, NV>(a.g0, k, d, l);
    axpy_row(G0, a.reg_adv, G);
    const RowV<NV> own = load_row<LPR, NV>(h.is_item ? a.Q : a.P, h.row, d, l);
    adagrad_row(a, G0, own, acc, h.count, wout);
  }
  store_row_wt<LPR, NV>(acc_tab, h.row, d, l, acc);
  if (a.inplace) store_row_wt<LPR, NV>(h.is_item ? a.Q : a.P, h.row, d, l, wout);
  else store_row<LPR, NV>(a.wnew_cur, k, d, l, wout);
}

template <int LPR, int NV, bool BPR>
__global__ void __launch_bounds__(256) k_tri_clean(StepArgs a) {
  const int wave = (int)((blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63, g = lane / LPR, l = lane & (LPR - 1);
  if (wave >= a.slot_waves) {
    STAMP(a.diag_launch, wave, 0);
    // APR clean pass: fused triplets have no clean work; a hash plan places them first
    const int boff = (!BPR && a.tri_nf) ? a.tri_nf[a.t] : 0;
    tri_triplets<LPR, NV, BPR ? 1 : 0>(a, wave - a.slot_waves, lane, boff);
    STAMP(a.diag_launch, wave, 5);
    return;
  }
  if (!a.prev_valid) return;  // write-back of the rows batch t-1 left in W scratch
  const int ngroups = a.slot_waves * (64 / LPR), gid = wave * (64 / LPR) + g;
  const int n = a.flush_cnt[a.t - 1];
  const int32_t* lst = a.flush_list + (int64_t)(a.t - 1) * a.S;
  for (int x = gid; x < n; x += ngroups) flush_slot(a, a.t - 1, a.wnew_prev, lst[x], l, LPR);
}

// The triplet-centric combine's hot slot, as hot_combine_slot<LPR, NV, MODE,
// true> computes it (the same additions in the same order), except that the
// finish runs on lane-group FG = the first of wave 1, which loads what the
// finish reads besides the pieces -- the slot record, then the Adagrad slot, g0
// and the row (MODE 2), or the Adagrad slot and the row (MODE 1) -- BEFORE the
// workgroup waits for the pieces: none of it depends on them (in place: the
// tables are current; g0 came from the previous launch).  It has to be another
// wave than the polling thread's: a wave's load counter is shared, and the poll
// would wait for the prefetch (tried on lane-group 0: slower).
template <int LPR, int NV>
struct TriHotPre {
  int32_t row, src, is_item;
  RowV<NV> acc, own, g0;
};

template <int LPR, int NV, int MODE>
__device__ __forceinline__ TriHotPre<LPR, NV> tri_hot_prefetch(const StepArgs& a, const int4 e) {
  TriHotPre<LPR, NV> f;
  const int l = threadIdx.x & (LPR - 1), d = a.d;
  const RecV r = load_rec(a.inl + ((int64_t)a.t * a.S + e.x) * a.R);
  f.is_item = (r.meta() & ACF_ITEM_BIT) != 0;
  f.row = r.own_row();
  f.src = r.own_src();
  if (MODE != 0 && !(a.shard && f.is_item)) {
    f.acc = load_row<LPR, NV>(f.is_item ? a.accQ : a.accP, f.row, d, l);
    if (MODE == 1) f.own = load_at<LPR, NV>(row_src(a, f.is_item ? a.Q : a.P, f.row, f.src), d, l);
    else f.own = load_row<LPR, NV>(f.is_item ? a.Q : a.P, f.row, d, l);
  }
  if (MODE == 2 && !(a.shard && f.is_item)) f.g0 = load_row<LPR, NV>(a.g0, e.x, d, l);
  return f;
}

template <int LPR, int NV, int MODE, bool READY = false>
__device__ __forceinline__ void tri_hot_finish(const StepArgs& a, const int4 e, float4* __restrict__ red,
                                               TriHotPre<LPR, NV>& f) {
  constexpr int NG = 256 / LPR, FG = 64 / LPR;
  const int g = threadIdx.x / LPR, l = threadIdx.x & (LPR - 1), d = a.d;
  RowV<NV> G = zero_row<NV>();
  for (int p0 = g; p0 < e.y; p0 += 8 * NG) {
    RowV<NV> x[8];
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (p0 + q * NG < e.y) x[q] = load_piece<LPR, NV, true>(a.hot_part, (int64_t)e.z + p0 + q * NG, d, l);
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (p0 + q * NG < e.y) G = add_row(G, x[q]);
  }
#pragma unroll
  for (int v = 0; v < NV; ++v) red[v * 256 + threadIdx.x] = G.v[v];
  __syncthreads();
  if (g == FG) {
    // group 0's sum, then groups 1, 2, ... in order: hot_combine_slot's additions
    RowV<NV> T;
#pragma unroll
    for (int v = 0; v < NV; ++v) T.v[v] = red[v * 256 + l];
    for (int gg = 1; gg < NG; ++gg) {
      RowV<NV> o;
#pragma unroll
      for (int v = 0; v < NV; ++v) o.v[v] = red[v * 256 + gg * LPR + l];
      T = add_row(T, o);
    }
    const int k = e.x;
    if (a.shard && f.is_item) {  // shard mode: the partial item sum, straight to its exchange row
      store_row_wt<LPR, NV>(a.xbuf, a.xmap[f.row], d, l, T);
    } else if (MODE == 0) {
      const RowV<NV> dl = make_delta<LPR, NV>(a, T, f.is_item, f.row, l);
      if (READY) {  // read in this launch: write-through, drained, then the tag
        store_row_wt<LPR, NV>(a.g0, k, d, l, T);
        store_row_wt<LPR, NV>(a.delta, k, d, l, dl);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (l == 0) __hip_atomic_store(a.ready + k, ready_tag(a), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        store_row<LPR, NV>(a.g0, k, d, l, T);
        store_row<LPR, NV>(a.delta, k, d, l, dl);
      }
    } else {
      RowV<NV> wout;
      if (MODE == 1) {
        adagrad_row(a, T, f.own, f.acc, e.w, wout);
      } else {
        RowV<NV> G0 = f.g0;
        axpy_row(G0, a.reg_adv, T);
        adagrad_row(a, G0, f.own, f.acc, e.w, wout);
      }
      store_row<LPR, NV>(f.is_item ? a.accQ : a.accP, f.row, d, l, f.acc);
      store_row<LPR, NV>(f.is_item ? a.Q : a.P, f.row, d, l, wout);  // in place (tri plans)
    }
  }
  __syncthreads();
}

// Hot pieces first in dispatch order, so their chain (pieces -> arrival count ->
// combining workgroup) starts at once: piece waves [0, hot_waves) into hot_part,
// then slot waves [.., + slot_waves): shared slots with <= ACF_HOT_MIN
// occurrences, one lane-group each, in order, then hot_blocks workgroups that
// each combine hot slots as k_hot_combine does once all their pieces are stored
// (r05: before the slot waves they held the CUs while they waited, and the slot
// waves, the launch's tail in the diag-build stamps, started up to 9 us late).  A piece
// is stored write-through, the wave drains its stores, and one lane adds 1 to
// the slot's arrival count; a combining workgroup polls that count (device
// scope), and every load of the pieces is a device-scope load (Guideline 16,
// row 1).  The combining workgroups come after every piece wave in dispatch
// order, so the pieces they wait for are already running: the launch always
// drains.  (hot_waves is a multiple of 4: whole workgroups.)
// (READY: k_tri_cadv's combine part -- the finished slots publish their tags)
template <int LPR, int NV, int MODE, bool READY>
__device__ __forceinline__ void tri_combine_wave(const StepArgs& a, const int wave, float4* __restrict__ red) {
  const int lane = threadIdx.x & 63, g = lane / LPR, l = lane & (LPR - 1);
  int32_t* arrive = a.hot.arrive + (int64_t)a.t * a.hot.piece_stride;
  STAMP(a.diag_launch, wave, 0);  // diagnostic builds: 1 piece, 2 / 3 combiner waited / done, 4 slot wave done
  if (wave < a.hot_waves) {
    const int hw = wave;
    constexpr int TEAM = 64 / LPR;
    const int n = a.hot.pcnt[a.t];
    const int4* pl = a.hot.piece + (int64_t)a.t * a.hot.piece_stride;
    const int2* pxa = a.hot.paux + (int64_t)a.t * a.hot.piece_stride;
    for (int x = hw; x < n; x += a.hot_waves) {
      const int4 pc = pl[x];  // {slot, piece, pieces, piece base}
      const int2 px = pxa[x];  // {count, CSR base | item << 31}: no dependent slot-record load
      TriSlot h;
      h.count = px.x;
      h.is_item = px.y < 0;
      h.base = px.y & 0x7FFFFFFF;
      h.row = h.src = 0;  // not read here
      const int o0 = (int)((int64_t)pc.y * h.count / pc.z), o1 = (int)((int64_t)(pc.y + 1) * h.count / pc.z);
      RowV<NV> G = zero_row<NV>();
      tri_add_q<LPR, NV>(a, h, o0 + g, o1, TEAM, l, G);
      team_allreduce<LPR, TEAM, NV>(G);
      if (a.hot_blocks == 0) {  // combined by k_hot_combine (the next launch)
        if (g == 0) store_row<LPR, NV>(a.hot_part, (int64_t)pc.w + pc.y, a.d, l, G);
        continue;
      }
      if (g == 0) store_row_wt<LPR, NV>(a.hot_part, (int64_t)pc.w + pc.y, a.d, l, G);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_fetch_add(arrive + pc.w, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    STAMP(a.diag_launch, wave, 1);
    return;
  }
  // then the small-slot waves [hot_waves, + slot_waves), then the combining
  // workgroups (r05: the small slots first, so they do not queue behind
  // workgroups that are waiting for pieces; 727M -> 747-763M triplets/s at
  // configs[4] d = 64, same box)
  const int w2 = wave - a.hot_waves;
  if (w2 >= a.slot_waves) {  // hot-slot combining workgroups (whole workgroups)
    const int hb = (w2 - a.slot_waves) >> 2;
    if (hb >= a.hot_blocks) return;
    const int n = a.hot.cnt[a.t];
    const int4* hl = a.hot.list + (int64_t)a.t * a.hot.hot_stride;
    for (int hx = hb; hx < n; hx += a.hot_blocks) {
      const int4 e = hl[hx];  // {slot, pieces, piece base, count}
      TriHotPre<LPR, NV> pre;
      if (threadIdx.x / LPR == 64 / LPR) pre = tri_hot_prefetch<LPR, NV, MODE>(a, e);  // the finishing group
      if (threadIdx.x == 0) {
        int it = 0;
        while (__hip_atomic_load(arrive + e.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < e.y) {
          if (++it > ACF_SPIN_LIMIT) {
            atomicOr(a.step_err, 1);
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
        // every piece of this pass is in: ready for the next pass over the batch
        __hip_atomic_store(arrive + e.z, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      if (hx == hb) STAMP(a.diag_launch, wave, 2);
      tri_hot_finish<LPR, NV, MODE, READY>(a, e, red, pre);
    }
    STAMP(a.diag_launch, wave, 3);
    return;
  }
  const int sw = w2;
  const int ngroups = a.slot_waves * (64 / LPR), gid = sw * (64 / LPR) + g;
  const int n = a.slot_cnt[a.t];
  const int32_t* lst = a.slot_list + (int64_t)a.t * a.S;
  for (int x = gid; x < n; x += ngroups) {
    const int k = lst[x];
    const TriSlot h = tri_slot(a, k);
    RowV<NV> G = zero_row<NV>();
    tri_add_q<LPR, NV>(a, h, 0, h.count, 1, l, G);
    tri_finish<LPR, NV, MODE>(a, k, h, G, l);
    if (READY) {  // g0 and delta went out write-through: drained, then the tag
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (l == 0) __hip_atomic_store(a.ready + k, ready_tag(a), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  STAMP(a.diag_launch, wave, 4);
}

template <int LPR, int NV, int MODE>
__global__ void __launch_bounds__(256) k_tri_combine(StepArgs a) {
  __shared__ float4 red[NV * 256];
  const int wave = (int)((blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6);
  tri_combine_wave<LPR, NV, MODE, false>(a, wave, red);
}

// k_tri_adv: 4 blocks (16 waves) per CU asked of the register allocator (d <= 256)
template <int LPR, int NV>
__global__ void __launch_bounds__(256, NV == 1 ? 4 : 1) k_tri_adv(StepArgs a) {
  const int wave = (int)((blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6);
  STAMP(a.diag_launch, wave, 0);
  tri_triplets<LPR, NV, 2>(a, wave, threadIdx.x & 63);
  STAMP(a.diag_launch, wave, 5);
}

// (r06) The clean combine and the adversarial pass of a batch in ONE launch:
// the combine's piece waves, small-slot waves and combining workgroups first
// (k_tri_combine<0>'s, each finished slot publishing its tag after write-through
// stores of g0 / delta), then the triplet waves of k_tri_adv.  The hash plan
// places each batch's fused triplets first (k_hplan_trip): they read no delta
// and run while the combine's chains finish; the other triplets wait for their
// shared slots' tags (tri_wait_ready).  Every wait is on work dispatched earlier
// in the grid, so the launch always drains.  No launch boundary between the two
// passes, and the combine's idle tail is filled: configs[4] d = 64 727-736M ->
// 752-760M triplets/s, d = 128 +1.5% (same box, profiles/r06/tri_cadv_v1_ab.json).
// (Dispatching the fused triplets before the small-slot waves instead was slower,
// 715M: the small slots queued behind them, profiles/r06/tri_cadv_v2_layout_ab.json.)
template <int LPR, int NV>
__global__ void __launch_bounds__(256, NV == 1 ? 4 : 1) k_tri_cadv(StepArgs a) {
  __shared__ float4 red[NV * 256];
  const int wave = (int)((blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6);
  const int cw = a.hot_waves + a.slot_waves + 4 * a.hot_blocks;  // whole workgroups
  if (wave < cw) {
    tri_combine_wave<LPR, NV, 0, true>(a, wave, red);
    return;
  }
  STAMP(a.diag_launch, wave, 0);
  tri_triplets<LPR, NV, 2, true>(a, wave - cw, threadIdx.x & 63);
  STAMP(a.diag_launch, wave, 5);
}

// Flush the pending rows of batch t (wnew_cur) to the tables (end of a call):
// one wave per slot.
__global__ void __launch_bounds__(256) k_flush(StepArgs a) {
  const int wave = (int)((blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6);
  // the call counter (random delta); every kernel of this call has read it
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(const_cast<uint32_t*>(a.epoch), 1u);
  if (a.inplace) return;  // nothing left in W scratch
  flush_slot(a, a.t, a.wnew_cur, wave, threadIdx.x & 63, 64);
}

__global__ void k_delta_scatter(StepArgs a, float* __restrict__ dP, float* __restrict__ dQ) {
  const int wave = (int)((blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  if (wave >= a.S) return;
  const RecV r = load_rec(a.inl + ((int64_t)a.t * a.S + wave) * a.R);
  if (r.gen() != *a.gen_ptr || (r.meta() & ACF_COUNT_MASK) == 0) return;
  float* dst = ((r.meta() & ACF_ITEM_BIT) ? dQ : dP) + (int64_t)r.own_row() * a.d;
  const float* src = a.delta + (int64_t)wave * a.d;
  for (int c = lane; c * 4 < a.d; c += 64)
    *reinterpret_cast<float4*>(dst + c * 4) = *reinterpret_cast<const float4*>(src + c * 4);
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

#include "acf_eval.h"  // all-items evaluation (k_eval_*): DESIGN.md §4

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

// One negative per triplet: a proposal from [0, num_items) — uniform
// (APR.py:76), or from an alias table (Walker / Vose: column k kept with
// probability prob[k], else alias[k]) — redrawn while it is in the user's
// trainList (APR.py:77-78).
__global__ void k_negatives(const int32_t* __restrict__ perm, const int32_t* __restrict__ pu,
                            const int32_t* __restrict__ pi, int64_t n_out, int32_t num_items,
                            int32_t num_lists, const int64_t* __restrict__ loff,
                            const int32_t* __restrict__ litems, uint64_t seed, int32_t max_tries,
                            const float* __restrict__ prob, const int32_t* __restrict__ alias,
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
    int32_t j = (int32_t)(((h >> 32) * (uint64_t)num_items) >> 32);
    if (prob && (float)(h & 0xFFFFFFull) * (1.0f / 16777216.0f) >= prob[j]) j = alias[j];
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
#define ACF_PACKED_MIN_BATCH 4096  // auto slot mapping: packed from this batch size

struct GraphKey {
  const void* ptrs[4];
  acf_apr_hparams hp;
  int32_t first, n, B, d, mapping, fusion, ovl;
  bool operator<(const GraphKey& o) const { return memcmp(this, &o, sizeof(GraphKey)) < 0; }
};

// (r04) Verified streamed calls are checked lazily, without a host sync per
// call.  Each one is queued on its group's FIFO (the contexts that train the same
// tables on one stream: a PlanPipeline's two contexts share one group); its
// launch reports COMMIT / FAIL in the context's host-mapped status ring.  A
// failed call applied nothing and set the group's gate, so every later streamed
// launch of the group ran nothing either (and applied nothing).  acf_apr_resolve
// (and every entry point that needs settled tables or re-plans a context with a
// queued call) walks the FIFO: committed calls leave it; at the first failed one
// the gate is cleared and that call and every later queued call are replayed,
// in order, on the two-kernel schedule, which waits on nothing -- exact, as
// k_stream is bit-identical to it.  A context keeps its plan while it has a
// queued call (acf_apr_plan resolves the context's calls first).
struct acf_apr_ctx;
struct Pending {
  acf_apr_ctx* c;
  uint32_t seq;
  int32_t first, n;
  acf_apr_tables tb;
  acf_apr_hparams hp;
  hipStream_t s;
};
struct FailGroup {
  int32_t* gate = nullptr;  // device word, see StepArgs.gate
  std::deque<Pending> q;
  int refs = 0;
};
// every live group, for acf_apr_resolve_all (readers outside a group: evaluation,
// forward, checkpoints)
// (ctypes releases the GIL around native calls, so contexts may be created,
// destroyed and resolved from several threads: the list is guarded; recursive,
// because acf_apr_resolve_all holds it across resolve())
static std::vector<FailGroup*> g_groups;
static std::recursive_mutex g_groups_mu;
static FailGroup* new_group() {
  FailGroup* g = new FailGroup();
  g->refs = 1;
  std::lock_guard<std::recursive_mutex> lk(g_groups_mu);
  g_groups.push_back(g);
  return g;
}
static void drop_group(FailGroup* g) {
  if (g->gate) (void)hipFree(g->gate);
  {
    std::lock_guard<std::recursive_mutex> lk(g_groups_mu);
    g_groups.erase(std::find(g_groups.begin(), g_groups.end(), g));
  }
  delete g;
}

struct acf_apr_ctx {
  int64_t U1 = 0, I1 = 0;
  int32_t d = 0, maxB = 0, maxNB = 0, lpr = 0, nv = 0, R = 0;
  int64_t maxE = 0;
  // plan
  uint64_t *key_in = nullptr, *key_out = nullptr;  // [E user keys | 2E item keys]
  int32_t *flag = nullptr, *inc = nullptr;
  int32_t *uuniq = nullptr, *uoff = nullptr, *ubs = nullptr;
  int32_t* tsl = nullptr;                    // [E][4] slots of each triplet's rows
  int32_t* tpos = nullptr;                   // [E][4] CSR positions of its occurrences
  int4 *uinfo = nullptr, *iinfo = nullptr;   // per unique row, see k_slot_info
  int32_t *iuniq = nullptr, *ioff = nullptr, *ibs = nullptr;
  OccRec* trec = nullptr;
  OccRec *urec = nullptr, *irec = nullptr, *inl = nullptr;
  int32_t *err = nullptr, *gen_dev = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  // per-batch scratch
  float *g0 = nullptr, *delta = nullptr, *wnew[2] = {nullptr, nullptr};
  float *loss_clean = nullptr, *loss_adv = nullptr;
  // state
  int32_t B = 0, nb = 0, gen = 0;
  int32_t last_delta_batch = -1;
  int32_t mapping = 0;  // slot mapping, see get_kernels
  int32_t plan_R = 1;   // inline records per slot in the current plan (<= R)
  int32_t lists = 0;    // the plan built slot / write-back lists (packed mode)
  int32_t touch_next = 1;  // phase 2 reads the next batch's records (ACF_TOUCH_NEXT=0 disables)
  int32_t *slot_list = nullptr, *flush_list = nullptr, *slot_cnt = nullptr, *flush_cnt = nullptr;
  HotLists hot = {};            // hot slots of list plans (k_records)
  int32_t shard = 0;            // shard mode (acf_apr_set_shard_mode): item rows are partial sums
  int32_t tri = 0;              // the plan is triplet-centric (packed, not shard: k_tri_*)
  float* contrib = nullptr;     // [4 maxB, d] per-occurrence contributions of shared rows (k_tri_*)
  unsigned long long* ready = nullptr;  // [3 maxB] k_tri_cadv's per-slot tags (zeroed: never a tag)
  int32_t reg_batch = 0;        // batch size of the reg mean (0: the planned batch size)
  int32_t shard_t = 0;          // the batch shard passes use (acf_apr_set_shard_batch)
  float* hot_part = nullptr;    // their piece sums
  int32_t fusion = 1;   // fused triplets in train_planned / time_kernels
  const float* xdelta = nullptr;    // triplet-centric shard passes: the owners' item deltas (acf_apr_shard_items_mapped)
  const int64_t* xdmap = nullptr;
  int32_t plan_kind2 = 0;  // the plan encodes sources at every distance (k_prev_next)
  int32_t plan_kb = 1;     // slot bits of the plan's src encoding
  int32_t* nextt = nullptr;  // [maxNB][S] next batch touching each slot's row (k_prev_next)
  // streamed step (k_stream): row versions of every batch of a launch
  int32_t stream = 1;        // ACF_STREAM=0 disables
  int32_t stream_depth = 2;  // ACF_STREAM_DEPTH: max waves per position (batches in flight)
  int32_t poll_sleep = 2;    // ACF_POLL_SLEEP: s_sleep between version polls (0-3; 4/5/6 = 8/16/32)
  int32_t spin_limit = ACF_SPIN_LIMIT;  // k_stream version polls before a give-up (acf_apr_set_spin_limit)
  int32_t failsafe = 1;      // verify every streamed call, replay a failed one (acf_apr_set_failsafe)
  unsigned long long* status = nullptr;      // host-mapped ring of 8: (seq << 2) | failed, per streamed launch
  unsigned long long* status_dev = nullptr;  // its device address
  int64_t recoveries = 0;    // streamed calls replayed on the two-kernel schedule
  uint32_t seq = 0;          // streamed launches so far (StepArgs.seq)
  uint32_t last_tail_seq = 0;  // seq of the last launch with a tail (StepArgs.decide_prev)
  unsigned long long* tail_diag = nullptr;  // diagnostic builds, ACF_TAIL_DIAG=1: tail stamps (acf_apr_diag_tail)
  unsigned long long* decide = nullptr;  // [0] decide word, [16, 16 + 288) the tail's arrival counters
  uint32_t tail_launches = 0;            // launches with a tail so far (StepArgs.tail_par)
  FailGroup* grp = nullptr;  // contexts whose streamed calls are verified together (PlanPipeline)
  int2* final_list = nullptr;  // the batch plan's final slots (k_stream's tail write-back)
  int32_t* final_cnt = nullptr;
  int32_t final_ok = 0;        // the current plan wrote final_list
  int32_t stream_ok = -1;    // -1 unknown, 0 unavailable (allocation / occupancy), 1 ready
  int64_t stream_max_waves = 0;
  unsigned long long *ver_w = nullptr, *ver_a = nullptr, *ver_d = nullptr;
  uint32_t* epoch = nullptr;
  int32_t *task_list = nullptr, *task_cnt = nullptr;  // streamed-step task lists of the plan
  int32_t task_lists = 0, task_stride = 0;
  // batch-local plan (k_bplan_sort / k_bplan_build)
  int32_t plan_mode = 0;     // 0 auto (batch-local plan where it applies), 1 always the sort plan
  // hash plan of triplet-centric steps (k_hplan_*); acf_apr_set_plan_mode(ctx, 1) keeps the sort plan (A/B)
  int32_t plan_kind = -1;    // acf_apr_plan_kind
  int32_t hplan_ok = -1;     // -1 unknown, 0 unavailable, 1 buffers allocated
  int2* hplan_occ = nullptr;   // [3 maxE] occurrence -> {slot or -1, CSR position}
  int32_t* hplan_pcnt = nullptr;  // [2][maxNB << pb][tiles] partition counts, their scan
  int4* hplan_claims = nullptr;   // [3 maxE / 2] shared keys, partition-local numbering
  int32_t* hplan_ptot = nullptr;  // [2][maxNB << pb][6] partition totals, their scan
  void* hplan_tmp = nullptr;   // rocPRIM temporary storage when c->tmp is too small
  size_t hplan_tmp_bytes = 0;
  int32_t* hplan_cnt = nullptr;  // [3][maxNB] shared slots, user / item CSR positions
  int32_t* hplan_haux = nullptr;  // [maxNB][hot_stride] CSR base | item of each hot-list entry
  int32_t* hplan_perm = nullptr;  // [maxE] triplet -> its place (fused first, r06)
  int32_t* hplan_tcnt = nullptr;  // [maxNB] fused triplets per batch
  unsigned long long* hplan_ttc = nullptr;  // [maxNB * tiles + 1] triplet classes per tile of 256, then its scan
  int32_t bplan_ok = -1;     // -1 unknown, 0 unavailable, 1 buffers allocated
  unsigned long long* bmask[2] = {nullptr, nullptr};
  size_t bmask_words = 0;
  int32_t bmask_dirty[2] = {0, 0};
  uint16_t* slot_of = nullptr;
  uint32_t* bkey = nullptr;
  int32_t *bstart = nullptr, *bocc = nullptr, *berr = nullptr;
  int2* bn = nullptr;
  hipStream_t cap_stream = nullptr;
  std::map<GraphKey, hipGraphExec_t> graphs;
  std::vector<void*> allocs;
};

// one lane-group per slot: large batches (auto), mapping 2, and always in shard mode
static int is_packed(const acf_apr_ctx* c, int32_t B) {
  return c->shard || c->mapping == 2 || (c->mapping == 0 && B >= ACF_PACKED_MIN_BATCH);
}

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

#ifndef ACF_BUILD_HASH
#define ACF_BUILD_HASH "unhashed"
#endif
extern "C" const char* acf_apr_build_hash(void) { return "ACF_BUILD_HASH=" ACF_BUILD_HASH; }

extern "C" const char* acf_apr_last_error(void) { return g_last_error.c_str(); }

static int resolve(acf_apr_ctx* c, int mode);
static void leave_group(acf_apr_ctx* c);

extern "C" int acf_apr_destroy(acf_apr_ctx* c) {
  if (!c) return ACF_OK;
  int r = ACF_OK;
  if (c->grp) {
    r = resolve(c, 2);  // the group's queued calls still need this context's plan
    leave_group(c);
  }
  for (auto& kv : c->graphs) (void)hipGraphExecDestroy(kv.second);
  c->graphs.clear();
  for (void* p : c->allocs) (void)hipFree(p);
  if (c->cap_stream) (void)hipStreamDestroy(c->cap_stream);
  if (c->status) (void)hipHostFree(c->status);
  delete c;
  return r;
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
  ACF_CHECK(2 * maxE < (1ll << 30), ACF_E_INVALID, "plan too large: %lld triplets", (long long)maxE);
  uint32_t ob_i = bits_for((uint64_t)(2 * maxE));
  uint32_t sb_i = bits_for((uint64_t)maxNB * (uint64_t)I1);
  uint32_t sb_u = bits_for((uint64_t)maxNB * (uint64_t)U1);
  ACF_CHECK(ob_i + sb_i < 64 && ob_i + sb_u < 64, ACF_E_INVALID,
            "plan key does not fit 64 bits (rows x batches x batch too large)");
  acf_apr_ctx* c = new acf_apr_ctx();
  c->U1 = U1; c->I1 = I1; c->d = d; c->maxB = maxB; c->maxNB = maxNB; c->maxE = maxE;
  geometry(d, &c->lpr, &c->nv);
  c->R = std::min(128 / c->lpr, 8);  // 2 records per team member (see slot_header)
  const size_t S = (size_t)3 * maxB;
  int r = ACF_OK;
  auto A = [&](auto** p, size_t n) { if (r == ACF_OK) r = dalloc(c, p, n); };
  A(&c->key_in, 3 * maxE); A(&c->key_out, 3 * maxE);
  A(&c->flag, 3 * maxE); A(&c->inc, 3 * maxE);
  A(&c->uuniq, maxE); A(&c->uoff, maxE + 1); A(&c->ubs, maxNB + 1);
  A(&c->tsl, 4 * maxE); A(&c->tpos, 4 * maxE); A(&c->uinfo, maxE);
  A(&c->slot_list, 3 * maxE); A(&c->flush_list, 3 * maxE);
  A(&c->slot_cnt, maxNB); A(&c->flush_cnt, maxNB);
  c->hot.hot_stride = hot_stride_for(maxB);
  c->hot.piece_stride = piece_stride_for(maxB);
  A(&c->hot.list, (size_t)maxNB * c->hot.hot_stride); A(&c->hot.piece, (size_t)maxNB * c->hot.piece_stride);
  A(&c->hot.cnt, 2 * (size_t)maxNB);
  A(&c->hot.arrive, (size_t)maxNB * c->hot.piece_stride);
  A(&c->hot.paux, (size_t)maxNB * c->hot.piece_stride);
  A(&c->hot_part, (size_t)c->hot.piece_stride * d);
  A(&c->contrib, (size_t)4 * maxB * d);
  A(&c->ready, (size_t)3 * maxB);
  A(&c->iuniq, 2 * maxE); A(&c->ioff, 2 * maxE + 1); A(&c->ibs, maxNB + 1);
  A(&c->iinfo, 2 * maxE);
  A(&c->urec, maxE); A(&c->irec, 2 * maxE); A(&c->trec, maxE);
  A(&c->inl, (size_t)maxNB * S * c->R);
  A(&c->err, 4); A(&c->gen_dev, 4); A(&c->epoch, 4); A(&c->decide, 16 + 2 * 144);
  A(&c->g0, 2 * S * d); A(&c->delta, 2 * S * d);  // by batch parity

  A(&c->nextt, 3 * maxE);
  A(&c->task_list, 4 * maxE); A(&c->task_cnt, maxNB);
  A(&c->wnew[0], S * d); A(&c->wnew[1], S * d);
  A(&c->loss_clean, maxE); A(&c->loss_adv, maxE);
  if (r != ACF_OK) { acf_apr_destroy(c); return r; }
  c->hot.pcnt = c->hot.cnt + maxNB;
  size_t b1 = 0, b2 = 0, b3 = 0, b4 = 0;
  uint32_t* k32 = reinterpret_cast<uint32_t*>(c->key_in);
  int32_t* v32 = reinterpret_cast<int32_t*>(k32 + 3 * maxE);
  if (rocprim::radix_sort_keys(nullptr, b1, c->key_in, c->key_out, (size_t)(3 * maxE), 0, 64) !=
          hipSuccess ||
      rocprim::radix_sort_pairs(nullptr, b3, k32, k32, v32, v32, (size_t)(3 * maxE), 0, 32) !=
          hipSuccess ||
      rocprim::inclusive_scan(nullptr, b2, c->flag, c->inc, (size_t)(4 * maxE),
                              rocprim::plus<int32_t>()) != hipSuccess ||
      rocprim::inclusive_scan(nullptr, b4, c->key_in, c->key_out, (size_t)(3 * maxE),
                              rocprim::plus<uint64_t>()) != hipSuccess) {
    acf_apr_destroy(c);
    return set_error(ACF_E_HIP, "rocprim temporary-storage query failed");
  }
  c->tmp_bytes = std::max(std::max(b1, b4), std::max(b2, b3));
  r = dalloc(c, reinterpret_cast<char**>(&c->tmp), c->tmp_bytes);
  if (r != ACF_OK) { acf_apr_destroy(c); return r; }
  if (hipStreamCreateWithFlags(&c->cap_stream, hipStreamNonBlocking) != hipSuccess) {
    acf_apr_destroy(c);
    return set_error(ACF_E_HIP, "hipStreamCreate failed");
  }
  // generation 0 never matches a plan: zeroed inline / fused-triplet records read as absent;
  // the epoch (version tag and call counter) starts at 1: zeroed version granules never match
  const uint32_t kOne = 1;
  if (hipMemset(c->inl, 0, (size_t)maxNB * S * c->R * sizeof(OccRec)) != hipSuccess ||
      hipMemset(c->trec, 0, (size_t)maxE * sizeof(OccRec)) != hipSuccess ||
      hipMemset(c->err, 0, 16) != hipSuccess || hipMemset(c->gen_dev, 0, 16) != hipSuccess ||
      hipMemset(c->ready, 0, (size_t)3 * maxB * sizeof(unsigned long long)) != hipSuccess ||
      hipMemset(c->decide, 0, (16 + 2 * 144) * 8) != hipSuccess ||
      hipMemcpy(c->epoch, &kOne, sizeof(kOne), hipMemcpyHostToDevice) != hipSuccess || hipMemset(c->nextt, 0, 3 * maxE * sizeof(int32_t)) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess) {
    acf_apr_destroy(c);
    return set_error(ACF_E_HIP, "hipMemset failed");
  }
#ifdef ACF_DIAG  // the tail's stamps (tools/tail_diag.py): diagnostic builds only
  if (const char* e = getenv("ACF_TAIL_DIAG"))
    if (atoi(e) && dalloc(c, &c->tail_diag, 8) == ACF_OK) (void)hipMemset(c->tail_diag, 0, 64);
#endif
  c->grp = new_group();
  if (hipMalloc(&c->grp->gate, 16) != hipSuccess || hipMemset(c->grp->gate, 0, 16) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess) {
    (void)hipGetLastError();
    acf_apr_destroy(c);
    return set_error(ACF_E_NOMEM, "failure-gate allocation failed");
  }
  *out = c;
  return ACF_OK;
}

static void leave_group(acf_apr_ctx* c) {
  FailGroup* g = c->grp;
  c->grp = nullptr;
  if (!g) return;
  for (auto it = g->q.begin(); it != g->q.end();)
    it = it->c == c ? g->q.erase(it) : it + 1;
  if (--g->refs == 0) drop_group(g);
}

static bool decided(const Pending& p, bool* failed) {
  const unsigned long long v = *(volatile unsigned long long*)(p.c->status + (p.seq & 7));
  *failed = (v & 1) != 0;
  return (v >> 2) == (unsigned long long)p.seq;
}

static int run_loop(acf_apr_ctx* c, const acf_apr_tables* tb, const acf_apr_hparams* hp,
                    int32_t first, int32_t n, hipStream_t s, hipEvent_t* events, int* kinds,
                    int allow_stream, int tri_phases);

// Block until queued call p has reported its outcome: poll its word of the
// host-mapped status ring, not the stream (a stream sync also waited
// for every call enqueued after p, e.g. the other context's chunk of a
// PlanPipeline).  A stream that has gone idle without an outcome is an error.
static int wait_decided(const Pending& p, bool* failed) {
  for (;;) {
    if (decided(p, failed)) return ACF_OK;
    const hipError_t q = hipStreamQuery(p.s);
    if (q == hipSuccess) {
      if (decided(p, failed)) return ACF_OK;
      return set_error(ACF_E_STATE, "streamed call %u reported no outcome", p.seq);
    }
    if (q != hipErrorNotReady) return set_error(ACF_E_HIP, "hipStreamQuery: %s", hipGetErrorString(q));
    std::this_thread::yield();
  }
}

// Settle the queued verified streamed calls of c's group (see FailGroup), front
// to back.  mode 0: only calls that have already reported; 1: block until every
// call of c itself has been settled; 2: block until the queue is empty.
static int resolve(acf_apr_ctx* c, int mode) {
  FailGroup* g = c->grp;
  if (!g) return ACF_OK;
  while (!g->q.empty()) {
    const Pending p = g->q.front();
    bool failed = false;
    if (!decided(p, &failed)) {
      bool need = mode == 2;
      for (const auto& x : g->q) need = need || (mode == 1 && x.c == c);
      if (!need) return ACF_OK;
      ACF_RET(wait_decided(p, &failed));
    }
    if (!failed) {
      g->q.pop_front();
      continue;
    }
    // every later queued call ran gated: wait until each has reported, then
    // clear the gate and replay them all, in order
    for (const auto& x : g->q) {
      bool f2 = false;
      ACF_RET(wait_decided(x, &f2));
    }
    std::deque<Pending> todo;
    todo.swap(g->q);
    HIP_TRY(hipMemsetAsync(g->gate, 0, sizeof(int32_t), todo.front().s));
    hipStream_t prev = todo.front().s;
    for (auto& x : todo) {
      if (x.s != prev) HIP_TRY(hipStreamSynchronize(prev));  // one stream per group in practice
      prev = x.s;
      ACF_RET(run_loop(x.c, &x.tb, &x.hp, x.first, x.n, x.s, nullptr, nullptr, 0, 3));
      ++x.c->recoveries;
    }
  }
  return ACF_OK;
}

// diagnostic (ACF_TAIL_DIAG=1, tools/tail_diag.py): the last tail's stamps
// (s_memrealtime, 100 MHz): [0] kernel start (block 0), [1] last workgroup done,
// [2] last arrival's add returned, [3] decided, [4] decider's actions issued,
// [5] last flusher saw the outcome, [6] last flusher wave done; zeroed after reading
extern "C" int acf_apr_diag_tail(acf_apr_ctx* c, uint64_t* out, void* stream_) {
  ACF_CHECK(c && out, ACF_E_INVALID, "NULL argument");
  ACF_CHECK(c->tail_diag, ACF_E_STATE, "ACF_TAIL_DIAG was not set when the context was created");
  hipStream_t s = static_cast<hipStream_t>(stream_);
  HIP_TRY(hipMemcpyAsync(out, c->tail_diag, 64, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemsetAsync(c->tail_diag, 0, 64, s));
  HIP_TRY(hipStreamSynchronize(s));
  return ACF_OK;
}

extern "C" int acf_apr_resolve(acf_apr_ctx* c) {
  ACF_CHECK(c, ACF_E_INVALID, "ctx is NULL");
  return resolve(c, 2);
}

extern "C" int acf_apr_share_failsafe(acf_apr_ctx* c, acf_apr_ctx* peer) {
  ACF_CHECK(c && peer, ACF_E_INVALID, "ctx is NULL");
  if (c->grp == peer->grp) return ACF_OK;
  ACF_RET(resolve(c, 2));
  ACF_RET(resolve(peer, 2));
  FailGroup* g = c->grp;
  c->grp = peer->grp;
  ++c->grp->refs;
  if (--g->refs == 0) drop_group(g);
  return ACF_OK;
}

extern "C" int acf_apr_resolve_all(void) {
  std::lock_guard<std::recursive_mutex> lk(g_groups_mu);
  for (size_t k = 0; k < g_groups.size(); ++k)
    if (!g_groups[k]->q.empty()) ACF_RET(resolve(g_groups[k]->q.front().c, 2));
  return ACF_OK;
}

// Batch-local plan buffers, allocated at first use: the two batch bitmaps, the
// per-row local slots and the per-batch sort outputs.  Off (sort plan) when
// the bitmaps or slot table would be large (big tables: packed plans anyway).
static bool bplan_ready(acf_apr_ctx* c) {
  if (c->bplan_ok >= 0) return c->bplan_ok == 1;
  c->bplan_ok = 0;
  const int64_t rows = c->U1 + c->I1;
  const int32_t W = (c->maxNB + 63) / 64;
  const size_t mask_words = (size_t)rows * W;
  const size_t S = (size_t)3 * c->maxB;
  if (c->maxB > 1024 || mask_words * 8 > ((size_t)64 << 20) ||
      (size_t)rows * c->maxNB * 2 > ((size_t)256 << 20))
    return false;
  std::vector<void*> got;
  auto A = [&](auto** p, size_t n) -> bool {
    if (dalloc(c, p, n) != ACF_OK) return false;
    got.push_back(*p);
    return true;
  };
  bool ok = A(&c->bmask[0], mask_words) && A(&c->bmask[1], mask_words) &&
            A(&c->slot_of, (size_t)rows * c->maxNB) && A(&c->bkey, (size_t)c->maxNB * S) &&
            A(&c->bstart, (size_t)c->maxNB * (S + 1)) && A(&c->bocc, (size_t)c->maxNB * S) &&
            A(&c->bn, (size_t)c->maxNB) && A(&c->berr, (size_t)c->maxNB) &&
            A(&c->final_list, (size_t)std::min<int64_t>(rows, (int64_t)c->maxNB * S)) && A(&c->final_cnt, 4);
  ok = ok && hipMemset(c->bmask[0], 0, mask_words * 8) == hipSuccess &&
       hipMemset(c->bmask[1], 0, mask_words * 8) == hipSuccess && hipDeviceSynchronize() == hipSuccess;
  if (!ok) {  // give back what was allocated; the sort plan stays in use
    (void)hipGetLastError();
    for (void* p : got) {
      (void)hipFree(p);
      c->allocs.erase(std::find(c->allocs.begin(), c->allocs.end(), p));
    }
    c->bmask[0] = c->bmask[1] = nullptr;
    c->final_list = nullptr;
    c->final_cnt = nullptr;
    return false;
  }
  c->bmask_words = mask_words;
  c->bmask_dirty[0] = c->bmask_dirty[1] = 0;
  c->bplan_ok = 1;
  return true;
}

// partition bits of a batch of B triplets: 2^pb partitions of <= ACF_HPLAN_PART occurrences on average
static int32_t hplan_pbits(int32_t B, int32_t part) {
  const uint64_t parts = ((uint64_t)3 * B + part - 1) / part;
  return parts <= 1 ? 0 : (int32_t)bits_for(parts - 1);
}

static bool hplan_ready(acf_apr_ctx* c) {
  if (c->hplan_ok >= 0) return c->hplan_ok == 1;
  c->hplan_ok = 0;
  if (c->maxB > ACF_HPLAN_MAXB) return false;
  const int32_t pb = hplan_pbits(c->maxB, ACF_HPLAN_PART);
  if (pb + (int32_t)bits_for((uint64_t)c->maxNB) > 32) return false;
  const size_t n3 = (size_t)3 * c->maxE;
  const size_t ncnt = ((size_t)c->maxNB << pb) * (((size_t)3 * c->maxB + ACF_HPLAN_PTILE - 1) / ACF_HPLAN_PTILE);
  const size_t ntt = (size_t)c->maxNB * ((c->maxB + 255) / 256) + 1;  // triplet tiles (+ a zero)
  size_t tb = 0;
  size_t tb2 = 0;
  if (rocprim::exclusive_scan(nullptr, tb, c->flag, c->inc, 0, ncnt, rocprim::plus<int32_t>()) != hipSuccess ||
      rocprim::exclusive_scan(nullptr, tb2, (unsigned long long*)nullptr, (unsigned long long*)nullptr, 0ull, ntt,
                              rocprim::plus<unsigned long long>()) != hipSuccess)
    return false;
  tb = std::max(tb, tb2);
  std::vector<void*> got;
  auto A = [&](auto** p, size_t m) -> bool {
    if (dalloc(c, p, m) != ACF_OK) return false;
    got.push_back(*p);
    return true;
  };
  bool ok = A(&c->hplan_occ, n3) && A(&c->hplan_pcnt, 2 * ncnt) && A(&c->hplan_claims, n3 / 2 + 1) &&
            A(&c->hplan_ptot, ((size_t)c->maxNB << pb) * 2 * ACF_HPLAN_TOT) &&
            A(&c->hplan_cnt, (size_t)3 * c->maxNB) && A(&c->hplan_haux, (size_t)c->maxNB * c->hot.hot_stride) &&
            A(&c->hplan_perm, (size_t)c->maxE) && A(&c->hplan_tcnt, (size_t)c->maxNB) &&
            A(&c->hplan_ttc, 2 * ntt);
  c->hplan_tmp_bytes = tb;
  if (ok && tb > c->tmp_bytes) ok = A(reinterpret_cast<char**>(&c->hplan_tmp), tb);
  if (!ok) {
    (void)hipGetLastError();
    for (void* p : got) {
      (void)hipFree(p);
      c->allocs.erase(std::find(c->allocs.begin(), c->allocs.end(), p));
    }
    c->hplan_occ = nullptr;
    c->hplan_pcnt = nullptr;
    c->hplan_claims = nullptr;
    c->hplan_ptot = nullptr;
    c->hplan_cnt = nullptr;
    c->hplan_haux = nullptr;
    c->hplan_perm = nullptr;
    c->hplan_tcnt = nullptr;
    c->hplan_ttc = nullptr;
    c->hplan_tmp = nullptr;
    return false;
  }
  c->hplan_ok = 1;
  return true;
}

// triplet-centric plans (see k_hplan_*): the same step inputs as the sort plan's
// tri branch, slot ids and CSR ranges numbered in allocation order
static int hash_plan(acf_apr_ctx* c, const int32_t* user, const int32_t* ipos, const int32_t* ineg, int32_t B,
                     int32_t nb, int32_t gen, int32_t kb, int32_t check, hipStream_t s) {
  const int32_t pb = hplan_pbits(B, ACF_HPLAN_PART);
  HIP_TRY(hipMemsetAsync(c->err, 0, sizeof(int32_t), s));  // the other counters: k_hplan_keys
  HPlanArgs p;
  p.user = user; p.ipos = ipos; p.ineg = ineg;
  p.U1 = c->U1; p.I1 = c->I1;
  p.B = B; p.S = 3 * B; p.nb = nb; p.gen = gen; p.pb = pb;
  p.tpb = (3 * B + ACF_HPLAN_PTILE - 1) / ACF_HPLAN_PTILE;
  p.ppr = reinterpret_cast<uint32_t*>(c->flag);
  p.pstage = reinterpret_cast<unsigned long long*>(c->key_in);
  p.pval = reinterpret_cast<unsigned long long*>(c->key_out);
  const int64_t ncnt = ((int64_t)nb << pb) * p.tpb;
  p.pcnt = c->hplan_pcnt;
  p.poff = c->hplan_pcnt + ((size_t)c->maxNB << hplan_pbits(c->maxB, ACF_HPLAN_PART)) *
                               (((size_t)3 * c->maxB + ACF_HPLAN_PTILE - 1) / ACF_HPLAN_PTILE);
  p.occ = c->hplan_occ; p.csr = c->tsl;
  p.claims = c->hplan_claims;
  p.ptot = c->hplan_ptot;
  p.pbase = c->hplan_ptot + ((size_t)c->maxNB << hplan_pbits(c->maxB, ACF_HPLAN_PART)) * ACF_HPLAN_TOT;
  p.scnt = c->hplan_cnt; p.ucsr = c->hplan_cnt + c->maxNB; p.icsr = c->hplan_cnt + 2 * c->maxNB;
  p.inl = c->inl; p.trec = c->trec; p.tpos = c->tpos;
  p.perm = c->hplan_perm; p.tcnt = c->hplan_tcnt;
  p.ttiles = (B + 255) / 256;
  p.ttc = c->hplan_ttc;
  p.tto = c->hplan_ttc + (size_t)c->maxNB * ((c->maxB + 255) / 256) + 1;
  p.slot_list = c->slot_list; p.slot_cnt = c->slot_cnt; p.flush_cnt = c->flush_cnt;
  p.saux = c->flush_list;  // unused by in-place plans
  p.haux = c->hplan_haux;
  p.hl = c->hot;
  p.err = c->err; p.gen_ptr = c->gen_dev;
  p.shard = c->shard;
  const unsigned tiles = (unsigned)(nb * p.tpb);
  k_hplan_keys<<<tiles, 256, 0, s>>>(p);
  HIP_TRY(hipGetLastError());
  {
    void* tmp = c->hplan_tmp ? c->hplan_tmp : c->tmp;
    size_t tb = c->hplan_tmp ? c->hplan_tmp_bytes : c->tmp_bytes;
    HIP_TRY(rocprim::exclusive_scan(tmp, tb, p.pcnt, p.poff, 0, (size_t)ncnt, rocprim::plus<int32_t>(), s));
  }
  k_hplan_scatter<<<tiles, 256, 0, s>>>(p);
  k_hplan_dedup<ACF_HPLAN_BUCKETS><<<(unsigned)(nb << pb), 256, 0, s>>>(p);
  k_hplan_bases<<<(unsigned)nb, 1024, 0, s>>>(p);
  k_hplan_emit<<<(unsigned)(nb << pb), 256, 0, s>>>(p);
  {  // the triplets' places (fused first): per-tile counts, their scan, the records
    const unsigned ttl = (unsigned)(nb * p.ttiles);
    k_hplan_tcount<<<ttl, 256, 0, s>>>(p);
    void* tmp = c->hplan_tmp ? c->hplan_tmp : c->tmp;
    size_t tb = c->hplan_tmp ? c->hplan_tmp_bytes : c->tmp_bytes;
    HIP_TRY(rocprim::exclusive_scan(tmp, tb, p.ttc, p.tto, 0ull, (size_t)ttl + 1, rocprim::plus<unsigned long long>(),
                                    s));
    k_hplan_trip<<<ttl, 256, 0, s>>>(p);
  }
  // (a one-batch plan, the split step's, gets more workgroups per batch)
  const unsigned rx = (unsigned)std::max(64, 1024 / nb);
  k_hplan_rank_small<<<dim3(rx, nb), 256, 0, s>>>(p);
  k_hplan_rank_hot<<<dim3(rx, nb), 256, (size_t)2 * ((2 * B + 31) / 32) * sizeof(uint32_t), s>>>(p);
  HIP_TRY(hipGetLastError());
  c->plan_R = 1;
  c->plan_kind2 = 0;
  c->plan_kb = kb;
  c->tri = 1;
  c->plan_kind = 3;
  c->task_lists = 0;
  c->lists = 1;
  if (check) {
    int32_t herr = 0;
    HIP_TRY(hipMemcpyAsync(&herr, c->err, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    ACF_CHECK(herr == 0, ACF_E_RANGE, "triplet index out of range (%s%s)",
              (herr & 1) ? "user >= num_user_rows " : "", (herr & 2) ? "item >= num_item_rows" : "");
  }
  c->B = B;
  c->nb = nb;
  return ACF_OK;
}

static int batch_plan(acf_apr_ctx* c, const int32_t* user, const int32_t* ipos, const int32_t* ineg,
                      int32_t B, int32_t nb, int32_t gen, int32_t kb, int32_t check, hipStream_t s) {
  const int cur = gen & 1, oth = cur ^ 1;
  if (c->bmask_dirty[cur])  // a plan used it and no later batch plan cleared it
    HIP_TRY(hipMemsetAsync(c->bmask[cur], 0, c->bmask_words * 8, s));
  BPlanArgs p;
  p.user = user; p.ipos = ipos; p.ineg = ineg;
  p.U1 = c->U1; p.I1 = c->I1;
  p.B = B; p.S = 3 * B; p.nb = nb;
  p.rb = (int32_t)bits_for((uint64_t)std::max(c->U1, c->I1));
  p.kb = kb;
  p.W = (c->maxNB + 63) / 64;
  p.nbs = c->maxNB;
  p.R = c->R;
  p.opw = 64 / c->lpr;
  p.stride = 3 * B + (B + p.opw - 1) / p.opw;
  p.gen = gen;
  p.mask = c->bmask[cur];
  p.mask_clear = c->bmask[oth];
  p.clear_words = c->bmask_dirty[oth] ? (int64_t)c->bmask_words : 0;
  p.slot_of = c->slot_of;
  p.bkey = c->bkey; p.bstart = c->bstart; p.bocc = c->bocc; p.bn = c->bn; p.berr = c->berr;
  p.err = c->err; p.gen_ptr = c->gen_dev;
  p.urec = c->urec; p.irec = c->irec; p.inl = c->inl; p.trec = c->trec;
  p.nextt = c->nextt;
  p.task_list = c->task_list; p.task_cnt = c->task_cnt;
  p.final_list = c->final_list; p.final_cnt = c->final_cnt;
  // 3 occurrences per thread in the sort, one thread per slot / triplet in the
  // build: ~24 us for a 20-batch plan against ~32 us for 6 per thread / 256-thread
  // builds (per-thread loops serialise the build's dependent loads)
  if (B <= 512) {
    k_bplan_sort<512, 3><<<nb, 512, 0, s>>>(p);
    k_bplan_build<1024, 512><<<nb, 1024, 0, s>>>(p);
  } else {
    k_bplan_sort<1024, 3><<<nb, 1024, 0, s>>>(p);
    k_bplan_build<1024, 1024><<<nb, 1024, 0, s>>>(p);
  }
  HIP_TRY(hipGetLastError());
  c->bmask_dirty[cur] = 1;
  c->bmask_dirty[oth] = 0;
  c->plan_R = c->R;
  c->tri = 0;
  c->plan_kind = 1;
  c->plan_kind2 = 1;
  c->plan_kb = kb;
  c->task_lists = 1;
  c->task_stride = p.stride;
  c->lists = 0;
  c->final_ok = (int64_t)c->maxNB * 3 * c->maxB < (1ll << 31) ? 1 : 0;
  if (check) {
    int32_t herr = 0;
    HIP_TRY(hipMemcpyAsync(&herr, c->err, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    ACF_CHECK(herr == 0, ACF_E_RANGE, "triplet index out of range (%s%s)",
              (herr & 1) ? "user >= num_user_rows " : "", (herr & 2) ? "item >= num_item_rows" : "");
  }
  c->B = B;
  c->nb = nb;
  return ACF_OK;
}

// shard mode, one batch of B <= 1,024: the one-workgroup plan (k_shard_plan)
static int shard_plan_small(acf_apr_ctx* c, const int32_t* user, const int32_t* ipos, const int32_t* ineg,
                            int32_t B, int32_t gen, int32_t check, hipStream_t s) {
  const int32_t kb = (int32_t)bits_for((uint64_t)3 * B + 1);
  SPlanArgs p;
  p.user = user; p.ipos = ipos; p.ineg = ineg;
  p.U1 = c->U1; p.I1 = c->I1;
  p.B = B;
  p.rb = (int32_t)bits_for((uint64_t)std::max(c->U1, c->I1));
  p.kb = kb;
  p.gen = gen;
  p.uuniq = c->uuniq; p.uoff = c->uoff; p.ubs = c->ubs;
  p.iuniq = c->iuniq; p.ioff = c->ioff; p.ibs = c->ibs;
  p.tsl = c->tsl; p.tpos = c->tpos;
  p.uinfo = c->uinfo; p.iinfo = c->iinfo;
  p.urec = c->urec; p.irec = c->irec; p.inl = c->inl; p.trec = c->trec;
  p.gen_ptr = c->gen_dev; p.err = c->err;
  p.sflags = c->key_in;
  p.hl = c->hot;
  p.slot_list = c->slot_list; p.flush_list = c->flush_list;
  p.slot_cnt = c->slot_cnt; p.flush_cnt = c->flush_cnt;
  k_shard_plan<1024, 3><<<1, 1024, 0, s>>>(p);
  HIP_TRY(hipGetLastError());
  c->plan_R = 1;
  c->plan_kind2 = 0;
  c->plan_kb = kb;
  c->tri = 0;
  c->plan_kind = 2;
  c->task_lists = 0;
  c->lists = 1;
  if (check) {
    int32_t herr = 0;
    HIP_TRY(hipMemcpyAsync(&herr, c->err, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    ACF_CHECK(herr == 0, ACF_E_RANGE, "triplet index out of range (%s%s)",
              (herr & 1) ? "user >= num_user_rows " : "", (herr & 2) ? "item >= num_item_rows" : "");
  }
  c->B = B;
  c->nb = 1;
  return ACF_OK;
}

// sorted keys -> head flags -> one scan -> per-side compaction
template <class KT>
static int plan_groups(acf_apr_ctx* c, const KT& ku, const KT& ki, int64_t E, int32_t nb,
                       hipStream_t s) {
  k_heads<KT><<<grid_for(3 * E), 256, 0, s>>>(ku, ki, E, c->flag);
  size_t tb = c->tmp_bytes;
  HIP_TRY(rocprim::inclusive_scan(c->tmp, tb, c->flag, c->inc, (size_t)(3 * E), rocprim::plus<int32_t>(), s));
  k_compact<KT><<<grid_for(E), 256, 0, s>>>(ku, c->inc, nullptr, E, c->U1, nb, c->uuniq, c->uoff, c->ubs,
                                            c->tsl, c->tpos, 0);
  k_compact<KT><<<grid_for(2 * E), 256, 0, s>>>(ki, c->inc + E, c->inc + E - 1, 2 * E, c->I1, nb, c->iuniq,
                                                c->ioff, c->ibs, c->tsl, c->tpos, 1);
  HIP_TRY(hipGetLastError());
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
  const uint32_t eb = std::max(eb_u, eb_i);  // item keys carry bit eb
  ACF_CHECK(eb < 64, ACF_E_INVALID, "plan key does not fit 64 bits");
  ACF_RET(resolve(c, 1));  // a queued streamed call of this context still needs its plan
  c->B = 0;
  c->nb = 0;
  c->last_delta_batch = -1;
  c->final_ok = 0;  // set by the batch plan
  const int32_t gen = ++c->gen;
  {
    const int packed = is_packed(c, B);
    const int32_t kb = (int32_t)bits_for((uint64_t)3 * B + 1);
    if (!packed && c->plan_mode == 0 && B <= 1024 && kb + bits_for((uint64_t)nb + 1) <= 31 && bplan_ready(c))
      return batch_plan(c, user, ipos, ineg, B, nb, gen, kb, check, s);
  }
  if (c->shard && nb == 1 && B <= 1024 && c->plan_mode == 0 &&
      bits_for((uint64_t)std::max(c->U1, c->I1)) <= 30)
    return shard_plan_small(c, user, ipos, ineg, B, gen, check, s);
  // triplet-centric plans (r05: in shard mode too, from B = 1,025)
  if (is_packed(c, B) && c->fusion && c->plan_mode == 0 && B <= ACF_HPLAN_MAXB && hplan_ready(c))
    return hash_plan(c, user, ipos, ineg, B, nb, gen, (int32_t)bits_for((uint64_t)3 * B + 1), check, s);
  HIP_TRY(hipMemsetAsync(c->err, 0, sizeof(int32_t), s));
  // 32-bit keys (segment only, occurrence as the sort value) when they fit
  const uint32_t sb = std::max(bits_for((uint64_t)nb * (uint64_t)c->U1),
                               bits_for((uint64_t)nb * (uint64_t)c->I1));
  const bool pairs = sb < 32;
  const uint64_t item_bit = 1ull << (pairs ? sb : eb);
  const int64_t n3 = 3 * E;
  size_t tb = c->tmp_bytes;
  if (pairs) {
    uint32_t* kin = reinterpret_cast<uint32_t*>(c->key_in);
    int32_t* vin = reinterpret_cast<int32_t*>(kin + n3);
    uint32_t* kout = reinterpret_cast<uint32_t*>(c->key_out);
    int32_t* vout = reinterpret_cast<int32_t*>(kout + n3);
    k_stage<true><<<grid_for(E), 256, 0, s>>>(user, ipos, ineg, E, B, c->U1, c->I1, kin, vin, 0, 0,
                                              item_bit, c->err);
    HIP_TRY(hipGetLastError());
    HIP_TRY(rocprim::radix_sort_pairs(c->tmp, tb, kin, kout, vin, vout, (size_t)n3, 0, sb + 1, s));
    const Key32 ku{kout, vout, ~0u}, ki{kout + E, vout + E, ~(uint32_t)item_bit};
    ACF_RET(plan_groups(c, ku, ki, E, nb, s));
  } else {
    k_stage<false><<<grid_for(E), 256, 0, s>>>(user, ipos, ineg, E, B, c->U1, c->I1, c->key_in,
                                               nullptr, ob_u, ob_i, item_bit, c->err);
    HIP_TRY(hipGetLastError());
    HIP_TRY(rocprim::radix_sort_keys(c->tmp, tb, c->key_in, c->key_out, (size_t)n3, 0, eb + 1, s));
    const Key64 ku{c->key_out, ob_u, ~0ull}, ki{c->key_out + E, ob_i, ~item_bit};
    ACF_RET(plan_groups(c, ku, ki, E, nb, s));
  }
  // where each unique row's value lives at batch start, then the records; one
  // lane-group per slot (large batches) reads only a slot's first record inline
  // (one-wave-per-slot plans encode every earlier batch, below)
  const int packed = is_packed(c, B);
  const int32_t kb = (int32_t)bits_for((uint64_t)3 * B + 1);
  // one-wave-per-slot plans encode every earlier batch (dt < nb must fit the src)
  const VKeys vk{(int32_t)bits_for((uint64_t)std::max(c->U1, c->I1)), (int32_t)bits_for((uint64_t)nb), 0};
  const int all_dt = !packed && kb + bits_for((uint64_t)nb + 1) <= 31 && vk.rb + vk.tb <= 32;
  if (all_dt) {
    // slots k_prev_next does not name (no row) read as "next batch 0": never flushed
    HIP_TRY(hipMemsetAsync(c->nextt, 0, (size_t)n3 * sizeof(int32_t), s));
    VKeys v = vk;
    v.k32 = 1 + vk.rb + vk.tb <= 31;
    uint32_t* k32 = reinterpret_cast<uint32_t*>(c->key_in);
    int32_t* v32 = reinterpret_cast<int32_t*>(k32 + n3);
    uint32_t* o32 = reinterpret_cast<uint32_t*>(c->key_out);
    int32_t* w32 = reinterpret_cast<int32_t*>(o32 + n3);
    k_vkeys<<<grid_for(n3), 256, 0, s>>>(c->uuniq, c->iuniq, c->ubs, c->ibs, E, nb, v,
                                         v.k32 ? (void*)k32 : (void*)c->key_in, v32);
    HIP_TRY(hipGetLastError());
    size_t tb3 = c->tmp_bytes;
    const int bits = 1 + vk.rb + vk.tb;
    if (v.k32) {
      // padding keys are all ones: past every valid key in the sorted bits (ties keep input order)
      HIP_TRY(rocprim::radix_sort_pairs(c->tmp, tb3, k32, o32, v32, w32, (size_t)n3, 0, bits, s));
    } else {
      HIP_TRY(rocprim::radix_sort_keys(c->tmp, tb3, c->key_in, c->key_out, (size_t)n3, 0, bits + 30, s));
    }
    k_prev_next<<<grid_for(n3), 256, 0, s>>>(v.k32 ? (const void*)o32 : (const void*)c->key_out, w32, E, v,
                                             c->uoff, c->ioff, c->ubs, c->ibs, 3 * B, kb, c->uinfo, c->iinfo,
                                             c->nextt);
  } else {
    // triplet-centric plans (packed, fusion on, not shard mode) update every row in
    // its table: no source / next-batch search (k_slot_info inplace)
    const int32_t tri_plan = packed && !c->shard && c->fusion;
    k_slot_info<<<grid_for(E), 256, 0, s>>>(c->uuniq, c->uoff, c->ubs, c->ubs, (int32_t)E, nb, 0, kb,
                                            c->uinfo, tri_plan);
    k_slot_info<<<grid_for(2 * E), 256, 0, s>>>(c->iuniq, c->ioff, c->ubs, c->ibs, (int32_t)(2 * E), nb, 1,
                                                kb, c->iinfo, tri_plan);
  }
  HIP_TRY(hipGetLastError());
  c->plan_R = packed ? 1 : c->R;
  c->plan_kind = 0;
  c->plan_kind2 = all_dt;
  c->plan_kb = kb;
  c->tri = packed && !c->shard && c->fusion;
  if (c->shard) {
    // Shard plans are replayed inside captured step graphs (distributed.ShardedAPR),
    // where a step's generation repeats from one replay to the next: clear the
    // inline records so that a slot this plan does not write never reads as
    // current (k_flush scans every slot of the batch).
    HIP_TRY(hipMemsetAsync(c->inl, 0, (size_t)nb * 3 * B * sizeof(OccRec), s));
  }
  if (packed) {  // k_records writes the slot flags of the slots it finds; the rest read 0
    HIP_TRY(hipMemsetAsync(c->key_in, 0, (size_t)3 * E * sizeof(uint64_t), s));
    HIP_TRY(hipMemsetAsync(c->hot.cnt, 0, 2 * (size_t)c->maxNB * sizeof(int32_t), s));
    HIP_TRY(hipMemsetAsync(c->hot.arrive, 0, (size_t)nb * c->hot.piece_stride * sizeof(int32_t), s));
  }
  k_records<<<grid_for(E), 256, 0, s>>>(E, B, 3 * B, c->plan_R, gen, kb, c->shard, c->tri,
                                        reinterpret_cast<const int4*>(c->tsl),
                                        reinterpret_cast<const int4*>(c->tpos), c->uinfo, c->iinfo,
                                        c->ubs, c->ibs, c->urec, c->irec, c->inl, c->trec, c->gen_dev,
                                        packed ? c->key_in : nullptr, c->hot);
  HIP_TRY(hipGetLastError());
  c->task_lists = 0;
  if (all_dt) {  // streamed-step task lists
    const int32_t opw = 64 / c->lpr, G = (B + opw - 1) / opw, stride = 3 * B + G;
    const int64_t n = (int64_t)nb * stride;
    int32_t* fl = reinterpret_cast<int32_t*>(c->key_in);
    int32_t* inc = reinterpret_cast<int32_t*>(c->key_out);
    k_task_flags<<<grid_for(n), 256, 0, s>>>(c->inl, c->trec, n, 3 * B, G, B, c->plan_R, opw, gen, fl);
    size_t tb4 = c->tmp_bytes;
    HIP_TRY(rocprim::inclusive_scan(c->tmp, tb4, fl, inc, (size_t)n, rocprim::plus<int32_t>(), s));
    k_task_list<<<grid_for(n), 256, 0, s>>>(fl, inc, n, stride, c->task_list, c->task_cnt);
    HIP_TRY(hipGetLastError());
    c->task_lists = 1;
    c->task_stride = stride;
  }
  c->lists = 0;
  if (packed) {  // per-batch lists of non-fused slots and of rows left in W scratch
    const int64_t n = (int64_t)nb * 3 * B;
    size_t tb2 = c->tmp_bytes;
    HIP_TRY(rocprim::inclusive_scan(c->tmp, tb2, c->key_in, c->key_out, (size_t)n, rocprim::plus<uint64_t>(), s));
    k_slot_lists<<<grid_for(n), 256, 0, s>>>(c->key_in, c->key_out, n, 3 * B, c->slot_list, c->flush_list,
                                             c->slot_cnt, c->flush_cnt);
    HIP_TRY(hipGetLastError());
    c->lists = 1;
  }
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
                          int32_t t, int32_t prev_valid) {
  StepArgs a;
  a.P = tb->P; a.Q = tb->Q; a.accP = tb->accP; a.accQ = tb->accQ;
  a.inl = c->inl; a.urec = c->urec; a.irec = c->irec; a.trec = c->trec;
  a.use_single = 0;
  a.touch_next = 0;
  a.slot_waves = 1 << 30;  // set by the launcher
  a.slot_list = c->slot_list; a.flush_list = c->flush_list;
  a.slot_cnt = c->slot_cnt; a.flush_cnt = c->flush_cnt;
  const size_t par = (size_t)(t & 1) * 3 * c->B * c->d;
  a.g0 = c->g0 + par; a.delta = c->delta + par;
  a.wnew_cur = c->wnew[t & 1];
  a.wnew_prev = c->wnew[(t + 1) & 1];
  a.step_err = c->err + 1;
  a.loss_clean = c->loss_clean; a.loss_adv = c->loss_adv;
  a.gen_ptr = c->gen_dev;
  a.d = c->d; a.B = c->B; a.S = 3 * c->B; a.R = c->plan_R; a.t = t; a.kb = c->plan_kb;
  a.prev_valid = prev_valid;
  a.diag_launch = 0;
  a.first = 0; a.t_end = 0;
  a.ver_w = c->ver_w; a.ver_a = c->ver_a; a.ver_d = c->ver_d;
  a.epoch = c->epoch; a.nextt = c->nextt;
  a.task_list = nullptr; a.task_cnt = c->task_cnt; a.task_stride = 0; a.max_depth = 1;
  a.poll_sleep = c->poll_sleep;
  a.fail = c->err + 2;  // seq of a streamed launch that gave up
  a.spin_limit = c->spin_limit;
  a.seq = 0; a.verify = 0; a.tail = 0; a.flushers = 1; a.decide_prev = 0; a.tail_diag = c->tail_diag;
  a.gate = c->grp ? c->grp->gate : nullptr;
  a.decide = c->decide; a.arrive = c->decide + 16; a.tail_par = 0;
  a.final_list = c->final_list; a.final_cnt = c->final_cnt;
  a.status = c->status_dev;
  a.hot = c->hot;
  a.hot_part = c->hot_part;
  a.hot_waves = 0;
  a.hot_blocks = 0;
  a.shard = c->shard;
  a.xbuf = nullptr;  // shard export: set by acf_apr_shard_pass_export
  a.xmap = nullptr;
  a.xubs = a.xibs = nullptr;
  a.xn = a.xblocks = a.xflush = 0;
  a.xdelta = c->xdelta;
  a.xdmap = c->xdmap;
  a.reg_B = c->reg_batch > 0 ? c->reg_batch : c->B;
  a.tpos = reinterpret_cast<const int4*>(c->tpos);
  a.tri_nf = c->plan_kind == 3 ? c->hplan_tcnt : nullptr;
  a.ready = c->ready;
  a.contrib = c->contrib;
  a.inplace = c->tri;
  a.lr = hp->lr; a.eps = hp->eps; a.reg = hp->reg; a.reg_adv = hp->reg_adv;
  a.clip_lo = hp->clip_lo; a.clip_hi = hp->clip_hi;
  a.adver = hp->adver; a.adv_mode = hp->adv_mode; a.zero_delta = hp->zero_delta; a.seed = hp->seed;
  return a;
}

// kernel kinds for timing: 0 = phase-1 (clean, or fused BPR), 1 = adversarial, 2 = flush
struct Kernels {
  void *clean_apr = nullptr, *clean_bpr = nullptr, *adv = nullptr, *flush = nullptr;
  void* stream = nullptr;  // k_stream (one wave per slot, d <= 256)
  void* stream_flush = nullptr;  // its write-back, k_stream_flush<LPR>
  void *hot_clean = nullptr, *hot_bpr = nullptr, *hot_adv = nullptr;  // k_hot_combine (list kernels)
  // triplet-centric list step (tri plans with fusion): clean (APR / BPR), combine (MODE 0/1/2), adversarial
  void *tri_clean = nullptr, *tri_clean_bpr = nullptr, *tri_adv = nullptr;
  void* tri_cadv = nullptr;  // the clean combine + adversarial pass in one launch (hash plans, r06)
  void* tri_comb[3] = {nullptr, nullptr, nullptr};
  int tri = 0;
  int slots_per_wave = 1;
  int lists = 0;  // list kernels: slot waves stride over the plan's per-batch lists
};

#define ACF_LIST_WAVES 4096  // slot waves of a list kernel
#define ACF_TRI_COMB_WAVES 4096  // small-slot waves of k_tri_combine (512 / 1,024 slower: r04 A/B)
#define ACF_TAIL_FLUSHERS 128    // workgroups of k_stream's tail write-back
#define ACF_HOT_WAVES 2048   // piece waves of a list kernel (hot slots)
#define ACF_HOT_BLOCKS 1024  // workgroups of k_hot_combine
#define ACF_TRI_HOT_BLOCKS 512  // hot-slot combining workgroups of k_tri_combine
// the same two inside k_tri_cadv (the clean combine at the head of the adversarial launch)
#ifndef ACF_CADV_SLOT_WAVES
#define ACF_CADV_SLOT_WAVES 4096
#endif
#ifndef ACF_CADV_HOT_BLOCKS
#define ACF_CADV_HOT_BLOCKS 512
#endif
// (r05 same-box A/B: 2,048 / 8,192 small-slot waves, 256 / 1,024 combining
// workgroups, 1,024 / 4,096 piece waves -- none faster; profiles/r05/combine_params_ab.json)

template <int LPR, int NV, int TEAM>
static void kernel_ptrs_team(Kernels* k, int fused) {
  k->clean_apr = reinterpret_cast<void*>(&k_clean<LPR, NV, false, TEAM>);
  if (fused) {
    k->clean_bpr = reinterpret_cast<void*>(&k_clean<LPR, NV, true, TEAM, true>);
    k->adv = reinterpret_cast<void*>(&k_adv<LPR, NV, TEAM, true>);
  } else {
    k->clean_bpr = reinterpret_cast<void*>(&k_clean<LPR, NV, true, TEAM>);
    k->adv = reinterpret_cast<void*>(&k_adv<LPR, NV, TEAM>);
  }
}

// fused: the phase-2 (APR) / fused-BPR kernels also run the fused-triplet waves;
// lists: one lane-group per slot over the plan's slot lists (packed + fused)
template <int LPR, int NV>
static void kernel_ptrs(Kernels* k, int packed, int fused, int lists, int tri) {
  constexpr int OPW = 64 / LPR;
  k->flush = reinterpret_cast<void*>(&k_flush);
  if (packed && fused && lists && tri) {
    k->tri_clean = reinterpret_cast<void*>(&k_tri_clean<LPR, NV, false>);
    k->tri_clean_bpr = reinterpret_cast<void*>(&k_tri_clean<LPR, NV, true>);
    k->tri_adv = reinterpret_cast<void*>(&k_tri_adv<LPR, NV>);
    k->tri_cadv = reinterpret_cast<void*>(&k_tri_cadv<LPR, NV>);
    k->tri_comb[0] = reinterpret_cast<void*>(&k_tri_combine<LPR, NV, 0>);
    k->tri_comb[1] = reinterpret_cast<void*>(&k_tri_combine<LPR, NV, 1>);
    k->tri_comb[2] = reinterpret_cast<void*>(&k_tri_combine<LPR, NV, 2>);
    k->hot_clean = reinterpret_cast<void*>(&k_hot_combine<LPR, NV, 0>);
    k->hot_bpr = reinterpret_cast<void*>(&k_hot_combine<LPR, NV, 1>);
    k->hot_adv = reinterpret_cast<void*>(&k_hot_combine<LPR, NV, 2>);
    k->slots_per_wave = OPW;
    k->lists = 1;
    k->tri = 1;
    return;
  }
  if (packed && fused && lists) {
    k->clean_apr = reinterpret_cast<void*>(&k_clean_list<LPR, NV, false>);
    k->clean_bpr = reinterpret_cast<void*>(&k_clean_list<LPR, NV, true>);
    k->adv = reinterpret_cast<void*>(&k_adv_list<LPR, NV>);
    k->hot_clean = reinterpret_cast<void*>(&k_hot_combine<LPR, NV, 0>);
    k->hot_bpr = reinterpret_cast<void*>(&k_hot_combine<LPR, NV, 1>);
    k->hot_adv = reinterpret_cast<void*>(&k_hot_combine<LPR, NV, 2>);
    k->slots_per_wave = OPW;
    k->lists = 1;
    return;
  }
  if (packed && OPW > 1) {
    kernel_ptrs_team<LPR, NV, 1>(k, fused);
    k->slots_per_wave = OPW;
  } else {
    kernel_ptrs_team<LPR, NV, OPW>(k, fused);
    if constexpr (NV == 1) {
      k->stream = reinterpret_cast<void*>(&k_stream<LPR, NV, OPW>);
      k->stream_flush = reinterpret_cast<void*>(&k_stream_flush<LPR>);
    }
    k->slots_per_wave = 1;
  }
  k->flush = reinterpret_cast<void*>(&k_flush);
}

// slot mapping: 0 auto (packed for batches >= ACF_PACKED_MIN_BATCH), 1 one wave
// per slot, 2 one lane-group per slot

static int get_kernels(const acf_apr_ctx* c, Kernels* k, int fused = 0) {
  return DISPATCH_GEOM(c->d, kernel_ptrs, k, is_packed(c, c->B), fused || c->shard, c->lists,
                       c->tri && (fused || c->shard));
}

typedef void (*StepKernel)(StepArgs);

// Launch one step kernel; with events (timing mode) via hipExtLaunchKernelGGL.
static int launch(void* fn, const StepArgs& a, int waves, hipStream_t s, hipEvent_t e0 = nullptr,
                  hipEvent_t e1 = nullptr) {
  const dim3 grid((unsigned)((waves + 3) / 4)), block(256);
  // waves past slot_waves run fused triplets: only when fusion is on
  if (!a.use_single && a.slot_waves + a.hot_waves < waves) return set_error(ACF_E_STATE, "bad step geometry");
  if (e0)
    hipExtLaunchKernelGGL(reinterpret_cast<StepKernel>(fn), grid, block, 0, s, e0, e1, 0, a);
  else
    hipLaunchKernelGGL(reinterpret_cast<StepKernel>(fn), grid, block, 0, s, a);
  HIP_TRY(hipGetLastError());
  return ACF_OK;
}

static int check_step(acf_apr_ctx* c, const acf_apr_tables* tb, const acf_apr_hparams* hp,
                      int32_t t) {
  ACF_CHECK(c && tb && hp, ACF_E_INVALID, "NULL ctx/tables/hparams");
  ACF_CHECK(tb->P && tb->Q && tb->accP && tb->accQ, ACF_E_INVALID, "NULL table pointer");
  ACF_CHECK(c->nb > 0, ACF_E_STATE, "no batches planned (call acf_apr_plan first)");
  ACF_CHECK(t >= 0 && t < c->nb, ACF_E_INVALID, "batch %d outside planned range [0, %d)", t, c->nb);
  return ACF_OK;
}

// training_batch over planned batches [first, first+n): per batch phase 1
// (+ flush of the previous batch) and, for APR, phase 2; a final flush.
// events != nullptr: timing mode, 2 events per launch, kinds[] per launch.
// (r05: the overlapped schedule k_ovl -- adv(t) + clean(t+1) per launch -- is
// gone; k_stream replaced it for d <= 256, the two-kernel schedule serves the
// rest and the failsafe replay.)

// Streamed step: version buffers (allocated at first use: 3 x maxNB x S x d
// granules) and the resident-wave budget of k_stream.
static int stream_positions(const acf_apr_ctx* c, const Kernels& K, int fuse);

static void free_alloc(acf_apr_ctx* c, void* p) {
  auto it = std::find(c->allocs.begin(), c->allocs.end(), p);
  if (it != c->allocs.end()) {
    (void)hipFree(p);
    c->allocs.erase(it);
  }
}

static int stream_ready(acf_apr_ctx* c, const Kernels& K) {
  if (c->stream_ok >= 0) return c->stream_ok;
  if (!K.stream) return 0;
  if (c->stream_max_waves == 0) {
    int dev = 0, cus = 0, blocks = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, reinterpret_cast<const void*>(K.stream), 256, 0) !=
            hipSuccess) {
      (void)hipGetLastError();
      c->stream_ok = 0;
      return 0;
    }
    // MI355X guide (residency): 256-thread blocks admitted per CU = min(API, 8,
    // 800 / (ceil(sgpr/16)*16 + 16)); k_stream's SGPR count (< 144) caps it at 5
    c->stream_max_waves = (int64_t)std::max(0, std::min(blocks, 5)) * cus * 4;
  }
  // the version buffers only for a plan the launch can keep resident (otherwise
  // not now: a later plan with a smaller batch may fit)
  if (stream_positions(c, K, c->fusion) > c->stream_max_waves) return 0;
  c->stream_ok = 0;
  const size_t n = (size_t)c->maxNB * 3 * c->maxB * c->d;
  if (dalloc(c, &c->ver_w, n) != ACF_OK || dalloc(c, &c->ver_a, n) != ACF_OK ||
      dalloc(c, &c->ver_d, n) != ACF_OK) {
    for (void* p : {(void*)c->ver_w, (void*)c->ver_a, (void*)c->ver_d})
      if (p) free_alloc(c, p);
    c->ver_w = c->ver_a = c->ver_d = nullptr;
    return 0;
  }
  // tag 0 never matches: the epoch starts at 1 (acf_apr_create)
  if (hipMemset(c->ver_w, 0, n * 8) != hipSuccess || hipMemset(c->ver_a, 0, n * 8) != hipSuccess ||
      hipMemset(c->ver_d, 0, n * 8) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  // the host-mapped status ring the end of a verified call reports to
  if (!c->status) {
    void* h = nullptr;
    void* dptr = nullptr;
    if (hipHostMalloc(&h, 64, hipHostMallocMapped) != hipSuccess || hipHostGetDevicePointer(&dptr, h, 0) != hipSuccess) {
      (void)hipGetLastError();
      if (h) (void)hipHostFree(h);
      return 0;
    }
    c->status = static_cast<unsigned long long*>(h);
    c->status_dev = static_cast<unsigned long long*>(dptr);
    memset(h, 0, 64);
  }
  c->stream_ok = 1;
  return 1;
}

static int stream_positions(const acf_apr_ctx* c, const Kernels& K, int fuse) {
  const int TW = fuse ? (c->B + 64 / c->lpr - 1) / (64 / c->lpr) : 0;
  return 3 * c->B + TW;
}

static int capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return st != hipStreamCaptureStatusNone;
}

// (stream_ready allocates: call prepare_stream before any capture)
static bool use_stream(acf_apr_ctx* c, const Kernels& K, const acf_apr_hparams* hp) {
  if (!(c->stream && hp->adver && K.stream && !K.lists && K.slots_per_wave == 1 && c->plan_kind2)) return false;
  if (c->stream_ok != 1) return false;
  return stream_positions(c, K, c->fusion) <= c->stream_max_waves;
}

static void prepare_stream(acf_apr_ctx* c, const acf_apr_hparams* hp) {
  Kernels K;
  if (c->stream && hp->adver && c->stream_ok < 0 && get_kernels(c, &K, c->fusion) == ACF_OK) (void)stream_ready(c, K);
}

// kinds: 0 phase 1 / fused BPR, 1 phase 2, 2 flush, 3 (unused since r05: k_ovl), 4 k_stream,
// 5 hot-slot combine (list kernels)
// tri_phases (triplet-centric plans, one batch through the two-phase API): bit 0
// the clean phase (delta_update), bit 1 the adversarial / BPR phase + the
// call-counter bump (optimizer_step); train_planned runs both.
static int run_loop(acf_apr_ctx* c, const acf_apr_tables* tb, const acf_apr_hparams* hp,
                    int32_t first, int32_t n, hipStream_t s, hipEvent_t* events, int* kinds,
                    int allow_stream = 2, int tri_phases = 3) {
  ACF_CHECK(!(c->tri && !c->fusion), ACF_E_STATE,
            "fusion was switched off after a triplet-centric plan (rows are updated in place): plan again");
  Kernels K;
  ACF_RET(get_kernels(c, &K, c->fusion));
  const int S = 3 * c->B;
  int SW = (S + K.slots_per_wave - 1) / K.slots_per_wave;  // slot waves of a step kernel
  if (K.lists) SW = std::min(SW, ACF_LIST_WAVES);
  const int fuse = c->fusion;
  const int TW = fuse ? (c->B + 64 / c->lpr - 1) / (64 / c->lpr) : 0;  // fused-triplet waves
  int li = 0;
  auto L = [&](void* fn, const StepArgs& a, int waves, int kind) -> int {
    hipEvent_t e0 = events ? events[2 * li] : nullptr, e1 = events ? events[2 * li + 1] : nullptr;
    if (kinds) kinds[li] = kind;
    StepArgs b = a;
    b.diag_launch = li;
    ++li;
    return launch(fn, b, waves, s, e0, e1);
  };
  if (allow_stream >= 2 && use_stream(c, K, hp)) {
    const int P = stream_positions(c, K, fuse);  // upper bound of the tasks of a batch
    const int lists = fuse && c->task_lists;
    // with task lists the kernel sizes its positions from the plan: give it the
    // resident maximum; otherwise P x depth waves
    const int64_t waves = lists ? c->stream_max_waves
                                : std::min<int64_t>(c->stream_max_waves, (int64_t)P * c->stream_depth);
    const int cap = capturing(s);
    // verified: queued for acf_apr_resolve (no host sync here); a timed or
    // captured call is unverified (a give-up sets step_err bit 0, the call is dropped)
    const bool verify = c->failsafe && !events && cap == 0;
    // the write-back in k_stream's tail: the whole plan in one launch (the final-
    // slot list is the plan's), and a launch the host counts (not captured)
    const bool tail = c->final_ok && first == 0 && n == c->nb && cap == 0;
    // an unverified launch behind queued verified calls would run gated if one of
    // them failed (dropped for good): settle the group first (not
    // possible while capturing: a captured call is documented as unverified)
    if (!verify && cap == 0 && !c->grp->q.empty()) ACF_RET(resolve(c, 2));
    if (verify) {  // at most 8 queued calls per context (its status ring)
      int mine = 0;
      for (const auto& x : c->grp->q) mine += x.c == c;
      if (mine >= 8) ACF_RET(resolve(c, 1));
    }
    const dim3 grid((unsigned)((waves + 3) / 4)), block(256);
    StepArgs a = make_args(c, tb, hp, first, 0);
    a.use_single = fuse;
    a.slot_waves = S;
    a.first = first;
    a.t_end = first + n;
    a.task_list = lists ? c->task_list : nullptr;
    a.task_stride = c->task_stride;
    a.max_depth = c->stream_depth;
    a.poll_sleep = c->poll_sleep;
    if (++c->seq == 0) ++c->seq;  // seq 0 is never a launch's (zeroed words)
    a.seq = c->seq;
    a.verify = verify ? 1 : 0;
    if (tail) {
      a.tail_par = (int32_t)(c->tail_launches++ & 1);
      a.tail = 1;
      a.flushers = ACF_TAIL_FLUSHERS;
      a.decide_prev = (unsigned long long)c->last_tail_seq << 1;
      c->last_tail_seq = a.seq;
    }
    hipEvent_t e0 = events ? events[2 * li] : nullptr, e1 = events ? events[2 * li + 1] : nullptr;
    if (kinds) kinds[li] = 4;
    ++li;
    typedef void (*SK)(StepArgs, int32_t);
    if (e0)
      hipExtLaunchKernelGGL(reinterpret_cast<SK>(K.stream), grid, block, 0, s, e0, e1, 0, a, (int32_t)P);
    else
      hipLaunchKernelGGL(reinterpret_cast<SK>(K.stream), grid, block, 0, s, a, (int32_t)P);
    HIP_TRY(hipGetLastError());
    if (!tail) {
      e0 = events ? events[2 * li] : nullptr;
      e1 = events ? events[2 * li + 1] : nullptr;
      if (kinds) kinds[li] = 2;
      ++li;
      typedef void (*FK)(StepArgs, uint32_t*);
      const dim3 fgrid(grid_for((int64_t)n * S * c->lpr));  // one lane-group per slot
      if (e0)
        hipExtLaunchKernelGGL(reinterpret_cast<FK>(K.stream_flush), fgrid, block, 0, s, e0, e1, 0, a, c->epoch);
      else
        hipLaunchKernelGGL(reinterpret_cast<FK>(K.stream_flush), fgrid, block, 0, s, a, c->epoch);
      HIP_TRY(hipGetLastError());
    }
    if (verify) {
      Pending p;
      p.c = c; p.seq = a.seq; p.first = first; p.n = n; p.tb = *tb; p.hp = *hp; p.s = s;
      c->grp->q.push_back(p);
    }
    return ACF_OK;
  }
  {
  // list kernels: piece waves of the hot slots after the slot waves, and a
  // combine launch (kind 5) after each pass
  const int HW = K.lists ? std::min(c->hot.piece_stride, ACF_HOT_WAVES) : 0;
  const int HB = std::min(c->hot.hot_stride, ACF_HOT_BLOCKS);
  if (K.tri) {  // triplet-centric list step (see k_tri_*)
    // k_tri_combine with its hot-slot combining workgroups after the piece waves
    // (whole workgroups: the two wave ranges rounded up to multiples of 4)
    const int SWT = std::min(SW, ACF_TRI_COMB_WAVES);
    const int SW4 = (SWT + 3) & ~3, HW4 = (HW + 3) & ~3, HBT = std::min(HB, ACF_TRI_HOT_BLOCKS);
    const int TWT = (c->B + 64 / c->lpr - 1) / (64 / c->lpr);  // one lane-group per triplet
    for (int32_t t = first; t < first + n; ++t) {
      // every row is updated in its table (StepArgs.inplace): nothing pending from t-1
      StepArgs a = make_args(c, tb, hp, t, 0);
      a.use_single = 1;
      a.slot_waves = SW;
      a.hot_waves = HW;
      StepArgs ah = a;
      ah.slot_waves = 4 * HB;
      StepArgs at = a;
      at.slot_waves = 0;  // k_tri_clean: triplet waves only (no write-back of t-1)
      StepArgs ac = a;
      ac.slot_waves = SW4;
      ac.hot_waves = HW4;
      ac.hot_blocks = HBT;
      const int CW = SW4 + HW4 + 4 * HBT;
      (void)ah;
      // hash plans (fused triplets placed first), a whole step, not shard mode: the
      // clean combine rides at the head of the adversarial launch (k_tri_cadv)
      const bool merged = tri_phases == 3 && !c->shard && c->plan_kind == 3 && K.tri_cadv;
      if (hp->adver) {
        if (tri_phases & 1) {
          ACF_RET(L(K.tri_clean, at, (TWT + tri_gpw(c->nv) - 1) / tri_gpw(c->nv), 0));
          if (!merged) ACF_RET(L(K.tri_comb[0], ac, CW, 5));
        }
        if (tri_phases & 2) {
          if (merged) {
            StepArgs am = ac;
            am.slot_waves = (std::min(SW, ACF_CADV_SLOT_WAVES) + 3) & ~3;
            am.hot_blocks = std::min(HB, ACF_CADV_HOT_BLOCKS);
            const int CWm = am.slot_waves + HW4 + 4 * am.hot_blocks;
            ACF_RET(L(K.tri_cadv, am, CWm + (TWT + tri_gpw(c->nv) - 1) / tri_gpw(c->nv), 1));
          }
          else ACF_RET(L(K.tri_adv, a, (TWT + tri_gpw(c->nv) - 1) / tri_gpw(c->nv), 1));
          ACF_RET(L(K.tri_comb[2], ac, CW, 5));
        }
      } else if (tri_phases & 2) {
        ACF_RET(L(K.tri_clean_bpr, at, (TWT + tri_gpw(c->nv) - 1) / tri_gpw(c->nv), 0));
        ACF_RET(L(K.tri_comb[1], ac, CW, 5));
      }
    }
    if (!(tri_phases & 2)) return ACF_OK;  // delta_update: no call-counter bump
  } else {
  for (int32_t t = first; t < first + n; ++t) {
    const int pv = t > first ? 1 : 0;
    StepArgs a = make_args(c, tb, hp, t, pv);
    a.use_single = fuse;
    a.slot_waves = SW;
    a.hot_waves = HW;
    a.touch_next = (c->touch_next && !K.lists && t + 1 < first + n) ? 1 : 0;
    if (hp->adver) {
      ACF_RET(L(K.clean_apr, a, SW + HW, 0));
      StepArgs ah = a;
      ah.slot_waves = 4 * HB;  // k_hot_combine: workgroups stride over the hot slots
      if (K.lists) ACF_RET(L(K.hot_clean, ah, 4 * HB, 5));
      ACF_RET(L(K.adv, a, SW + HW + TW, 1));
      if (K.lists) ACF_RET(L(K.hot_adv, ah, 4 * HB, 5));
    } else {
      ACF_RET(L(K.clean_bpr, a, SW + HW + TW, 0));
      StepArgs ah = a;
      ah.slot_waves = 4 * HB;
      if (K.lists) ACF_RET(L(K.hot_bpr, ah, 4 * HB, 5));
    }
  }
  }
  }
  StepArgs af = make_args(c, tb, hp, first + n - 1, 0);
  af.use_single = fuse;
  af.slot_waves = S;
  ACF_RET(L(K.flush, af, K.tri ? 4 : S, 2));  // in place (tri): the call-counter bump only
  return ACF_OK;
}

extern "C" int acf_apr_delta_update(acf_apr_ctx* c, const acf_apr_tables* tb,
                                    const acf_apr_hparams* hp, int32_t t, void* stream_) {
  ACF_RET(check_step(c, tb, hp, t));
  ACF_RET(resolve(c, 2));  // settle queued streamed calls first (FailGroup)
  ACF_CHECK(hp->adver, ACF_E_INVALID, "delta_update needs hparams.adver = 1 (APR graph)");
  hipStream_t s = static_cast<hipStream_t>(stream_);
  if (c->tri) {  // triplet-centric plan: its clean phase
    ACF_RET(run_loop(c, tb, hp, t, 1, s, nullptr, nullptr, 0, 1));
    c->last_delta_batch = t;
    return ACF_OK;
  }
  Kernels K;
  ACF_RET(get_kernels(c, &K));
  const int SW = (3 * c->B + K.slots_per_wave - 1) / K.slots_per_wave;
  StepArgs a = make_args(c, tb, hp, t, 0);
  a.slot_waves = SW;
  ACF_RET(launch(K.clean_apr, a, SW, s));
  c->last_delta_batch = t;
  return ACF_OK;
}

extern "C" int acf_apr_optimizer_step(acf_apr_ctx* c, const acf_apr_tables* tb,
                                      const acf_apr_hparams* hp, int32_t t, void* stream_) {
  ACF_RET(check_step(c, tb, hp, t));
  ACF_RET(resolve(c, 2));  // settle queued streamed calls first (FailGroup)
  hipStream_t s = static_cast<hipStream_t>(stream_);
  if (c->tri) {  // triplet-centric plan: its adversarial (or BPR) phase, rows in place
    ACF_CHECK(!hp->adver || c->last_delta_batch == t, ACF_E_STATE,
              "APR optimizer step on batch %d needs acf_apr_delta_update on the same batch first", t);
    return run_loop(c, tb, hp, t, 1, s, nullptr, nullptr, 0, 2);
  }
  Kernels K;
  ACF_RET(get_kernels(c, &K));
  const int SW = (3 * c->B + K.slots_per_wave - 1) / K.slots_per_wave;
  StepArgs a = make_args(c, tb, hp, t, 0);
  a.slot_waves = SW;
  if (hp->adver) {
    ACF_CHECK(c->last_delta_batch == t, ACF_E_STATE,
              "APR optimizer step on batch %d needs acf_apr_delta_update on the same batch first", t);
    ACF_RET(launch(K.adv, a, SW, s));
  } else {
    ACF_RET(launch(K.clean_bpr, a, SW, s));
  }
  a.slot_waves = 3 * c->B;
  ACF_RET(launch(K.flush, a, 3 * c->B, s));
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
  c->last_delta_batch = -1;
  prepare_stream(c, hp);
  Kernels K;
  const bool streamed = get_kernels(c, &K, c->fusion) == ACF_OK && use_stream(c, K, hp);
  // a streamed call runs gated behind a queued call of the group that may have
  // failed; any other schedule needs the tables settled first
  ACF_RET(resolve(c, streamed ? 0 : 2));
  // the streamed step is one or two launches: a graph buys nothing
  if (!graph_mode || streamed) return run_loop(c, tb, hp, first, n, s, nullptr, nullptr);
  GraphKey key;
  memset(&key, 0, sizeof(key));
  key.ptrs[0] = tb->P; key.ptrs[1] = tb->Q; key.ptrs[2] = tb->accP; key.ptrs[3] = tb->accQ;
  key.hp = *hp;
  key.first = first; key.n = n; key.B = c->B; key.d = c->d; key.mapping = c->mapping;
  key.fusion = c->fusion;
  key.ovl = c->stream;
  auto it = c->graphs.find(key);
  if (it == c->graphs.end()) {
    hipGraph_t g = nullptr;
    HIP_TRY(hipStreamBeginCapture(c->cap_stream, hipStreamCaptureModeThreadLocal));
    int r = run_loop(c, tb, hp, first, n, c->cap_stream, nullptr, nullptr);
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
  return ACF_OK;
}

extern "C" int acf_apr_train(acf_apr_ctx* c, const acf_apr_tables* tb, const acf_apr_hparams* hp,
                             const int32_t* user, const int32_t* ipos, const int32_t* ineg, int32_t B,
                             int32_t nb, int32_t check, int32_t graph_mode, void* stream_) {
  ACF_RET(acf_apr_plan(c, user, ipos, ineg, B, nb, check, stream_));
  return acf_apr_train_planned(c, tb, hp, 0, nb, graph_mode, stream_);
}

static int time_kernels(acf_apr_ctx* c, const acf_apr_tables* tb, const acf_apr_hparams* hp, int32_t first,
                        int32_t n, double* ms_out, int32_t* launches_out, void* stream_, int nkinds) {
  ACF_CHECK(c && tb && hp && ms_out && launches_out, ACF_E_INVALID, "NULL argument");
  ACF_RET(resolve(c, 2));
  ACF_CHECK(n > 0 && first >= 0 && first + n <= c->nb, ACF_E_INVALID,
            "batch range [%d, %d) outside planned range [0, %d)", first, first + n, c->nb);
  ACF_RET(check_step(c, tb, hp, first));
  hipStream_t s = static_cast<hipStream_t>(stream_);
  prepare_stream(c, hp);
  const int nl = 6 * n + 2;
  std::vector<hipEvent_t> ev((size_t)2 * nl, nullptr);
  std::vector<int> kinds(nl, -1);
  for (auto& e : ev) HIP_TRY(hipEventCreate(&e));
  int r = run_loop(c, tb, hp, first, n, s, ev.data(), kinds.data(), nkinds > 4 ? 2 : (nkinds > 3 ? 1 : 0));
  if (r == ACF_OK && hipStreamSynchronize(s) != hipSuccess) r = set_error(ACF_E_HIP, "sync failed");
  for (int k = 0; k < nkinds; ++k) { ms_out[k] = 0.0; launches_out[k] = 0; }
  for (int x = 0; r == ACF_OK && x < nl; ++x) {
    if (kinds[x] < 0 || kinds[x] >= nkinds) continue;
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, ev[2 * x], ev[2 * x + 1]) != hipSuccess) {
      r = set_error(ACF_E_HIP, "hipEventElapsedTime failed");
      break;
    }
    ms_out[kinds[x]] += ms;
    launches_out[kinds[x]] += 1;
  }
  for (auto& e : ev) (void)hipEventDestroy(e);
  c->last_delta_batch = -1;
  return r;
}

// per-kind launch times of the launch sequence acf_apr_train_planned runs
// (kinds: see run_loop; include/acf_apr.h)
extern "C" int acf_apr_time_kernels(acf_apr_ctx* c, const acf_apr_tables* tb,
                                    const acf_apr_hparams* hp, int32_t first, int32_t n,
                                    double* ms_out, int32_t* launches_out, void* stream_) {
  return time_kernels(c, tb, hp, first, n, ms_out, launches_out, stream_, 6);
}

extern "C" int acf_apr_set_slot_mapping(acf_apr_ctx* c, int32_t mode) {
  ACF_CHECK(c, ACF_E_INVALID, "ctx is NULL");
  ACF_RET(resolve(c, 2));  // settle queued streamed calls first (FailGroup)
  ACF_CHECK(mode >= 0 && mode <= 2, ACF_E_INVALID, "slot mapping must be 0 (auto), 1 or 2, got %d", mode);
  c->mapping = mode;
  return ACF_OK;
}

extern "C" int acf_apr_set_plan_mode(acf_apr_ctx* c, int32_t mode) {
  ACF_CHECK(c, ACF_E_INVALID, "ctx is NULL");
  ACF_RET(resolve(c, 2));  // settle queued streamed calls first (FailGroup)
  ACF_CHECK(mode == 0 || mode == 1, ACF_E_INVALID, "plan mode must be 0 (auto) or 1 (sort plan)");
  c->plan_mode = mode;
  return ACF_OK;
}

extern "C" int acf_apr_plan_kind(const acf_apr_ctx* c) { return c ? c->plan_kind : -1; }

extern "C" int acf_apr_set_fusion(acf_apr_ctx* c, int32_t on) {
  ACF_CHECK(c, ACF_E_INVALID, "ctx is NULL");
  ACF_RET(resolve(c, 2));  // settle queued streamed calls first (FailGroup)
  ACF_CHECK(on == 0 || on == 1, ACF_E_INVALID, "fusion must be 0 or 1, got %d", on);
  c->fusion = on;
  return ACF_OK;
}

extern "C" int acf_apr_set_stream(acf_apr_ctx* c, int32_t on) {
  ACF_CHECK(c, ACF_E_INVALID, "ctx is NULL");
  ACF_RET(resolve(c, 2));  // settle queued streamed calls first (FailGroup)
  c->stream = on != 0;
  return ACF_OK;
}

// ---------------------------------------------------------------------------
// Shard mode (distributed.ShardedAPR).  Users live on rank u % G
// and every triplet runs on its user's rank, so user rows are complete here;
// an item's occurrences are spread over the ranks, so its clean / adversarial
// sums are partial and are summed by the item's owner (rank i % G) between
// the two passes.  One step = one plan of this rank's triplets of the batch
// (tables: the local user shard and the fetched item working set, slots in
// working-set order) and two passes:
//   pass 0: clean sums.  Users: g0, delta.  Items: partial sums in g0
//           (acf_apr_shard_items dir 0 copies them out; the owners' deltas come
//           back through dir 1 into the delta rows).  BPR: users are updated here.
//   pass 1: adversarial sums.  Users: Adagrad + write-back.  Items: partial
//           sums in g0 for the owners' Adagrad (acf_shard_reduce_apply).
// ---------------------------------------------------------------------------
extern "C" int acf_apr_set_shard_mode(acf_apr_ctx* c, int32_t on, int32_t reg_batch) {
  ACF_CHECK(c, ACF_E_INVALID, "ctx is NULL");
  ACF_RET(resolve(c, 2));  // settle queued streamed calls first (FailGroup)
  ACF_CHECK(reg_batch >= 0, ACF_E_INVALID, "reg_batch must be >= 0");
  c->shard = on != 0;
  c->reg_batch = reg_batch;
  c->nb = 0;  // re-plan: the records depend on the mode
  c->shard_t = 0;
  return ACF_OK;
}

// (r06) the batch of a multi-batch triplet-centric shard plan that the next
// shard pass / item map calls use (distributed.ShardedAPR plans a chunk of
// steps at once)
extern "C" int acf_apr_set_shard_batch(acf_apr_ctx* c, int32_t t) {
  ACF_CHECK(c != nullptr, ACF_E_INVALID, "ctx is NULL");
  ACF_CHECK(t >= 0 && t < c->maxNB, ACF_E_INVALID, "batch %d outside [0, %d)", t, c->maxNB);
  c->shard_t = t;
  return ACF_OK;
}

extern "C" int acf_apr_shard_pass_export(acf_apr_ctx* c, const acf_apr_tables* tb, const acf_apr_hparams* hp,
                                         int32_t pass, float* xbuf, const int64_t* xmap, int64_t n_items,
                                         void* stream_) {
  ACF_RET(check_step(c, tb, hp, 0));
  ACF_RET(resolve(c, 2));  // settle queued streamed calls first (FailGroup)
  ACF_CHECK(c->shard && c->lists && (c->nb == 1 || (c->tri && c->nb > 1)), ACF_E_STATE,
            "shard pass needs shard mode and a one-batch plan (or a triplet-centric plan of several)");
  ACF_CHECK(c->shard_t < c->nb, ACF_E_STATE, "shard batch %d outside the plan's %d", c->shard_t, c->nb);
  ACF_CHECK(pass == 0 || (pass == 1 && hp->adver), ACF_E_INVALID, "pass must be 0, or 1 for APR");
  ACF_CHECK(hp->adv_mode == 0, ACF_E_INVALID, "shard mode supports adv = grad only");
  ACF_CHECK((xbuf == nullptr) == (xmap == nullptr), ACF_E_INVALID, "xbuf and xmap go together");
  ACF_CHECK(n_items >= 0 && n_items <= 2 * (int64_t)c->B, ACF_E_INVALID, "n_items %lld outside [0, 2B]",
            (long long)n_items);
  hipStream_t s = static_cast<hipStream_t>(stream_);
  Kernels K;
  ACF_RET(get_kernels(c, &K, 0));
  ACF_CHECK(K.lists, ACF_E_STATE, "shard mode needs the list kernels");
  const int S = 3 * c->B;
  const int SW = std::min((S + K.slots_per_wave - 1) / K.slots_per_wave, ACF_LIST_WAVES);
  const int HW = std::min(c->hot.piece_stride, ACF_HOT_WAVES);
  const int HB = std::min(c->hot.hot_stride, ACF_HOT_BLOCKS);
  if (K.tri) {
    // (r05) triplet-centric shard passes (hash plan): the triplet pass (a single
    // item's product goes straight to its exchange row), then k_tri_combine,
    // whose item slots store their partial sums there too and whose user slots
    // finish as in the unsharded step (delta; Adagrad in place).  Pass 1 reads
    // the owners' item deltas from the exchange rows (acf_apr_shard_items_mapped
    // dir 1 names them).
    ACF_CHECK(xbuf, ACF_E_INVALID, "triplet-centric shard passes export their item sums: xbuf is required");
    ACF_CHECK(pass == 0 || c->xdelta, ACF_E_STATE, "pass 1 needs the owners' deltas (acf_apr_shard_items_mapped)");
    const int SW4 = (std::min(SW, ACF_TRI_COMB_WAVES) + 3) & ~3, HW4 = (HW + 3) & ~3;
    const int HBT = std::min(HB, ACF_TRI_HOT_BLOCKS);
    const int TWT = (c->B + 64 / c->lpr - 1) / (64 / c->lpr);
    const int TW = (TWT + tri_gpw(c->nv) - 1) / tri_gpw(c->nv);
    StepArgs a = make_args(c, tb, hp, c->shard_t, 0);  // batch shard_t of the plan
    a.use_single = 1;
    a.xbuf = xbuf;
    a.xmap = xmap;
    a.xn = (int32_t)n_items;
    StepArgs at = a, ac = a;
    at.slot_waves = 0;
    ac.slot_waves = SW4;
    ac.hot_waves = HW4;
    ac.hot_blocks = HBT;
    if (pass == 0) {
      ACF_RET(launch(hp->adver ? K.tri_clean : K.tri_clean_bpr, at, TW, s));
      ACF_RET(launch(K.tri_comb[hp->adver ? 0 : 1], ac, SW4 + HW4 + 4 * HBT, s));
    } else {
      ACF_RET(launch(K.tri_adv, a, TW, s));
      ACF_RET(launch(K.tri_comb[2], ac, SW4 + HW4 + 4 * HBT, s));
    }
    return ACF_OK;
  }
  ACF_CHECK(c->nb == 1 && c->shard_t == 0, ACF_E_STATE, "slot-kernel shard passes take one-batch plans");
  StepArgs a = make_args(c, tb, hp, 0, 0);
  a.use_single = 0;
  a.slot_waves = SW;
  a.hot_waves = HW;
  if (pass == 0) {
    ACF_RET(launch(hp->adver ? K.clean_apr : K.clean_bpr, a, SW + HW, s));
  } else {
    ACF_RET(launch(K.adv, a, SW + HW, s));
  }
  StepArgs ah = a;
  int XB = 0;
  const bool users_done = pass == 1 || !hp->adver;  // this pass updates the user rows
  if (xbuf) {  // export (and write-back) workgroups after the combining ones
    const int XF = users_done ? (c->B * c->lpr + 255) / 256 : 0;  // one lane-group per user slot
    XB = (int)((n_items * c->lpr + 255) / 256) + XF;                 // one lane-group per item slot
    ah.xbuf = xbuf;
    ah.xmap = xmap;
    ah.xubs = c->ubs;
    ah.xibs = c->ibs;
    ah.xn = (int32_t)n_items;
    ah.xblocks = XB;
    ah.xflush = XF;
  }
  ah.slot_waves = 4 * (HB + XB);  // k_hot_combine: workgroups stride over the hot slots
  ACF_RET(launch(pass == 1 ? K.hot_adv : (hp->adver ? K.hot_clean : K.hot_bpr), ah, 4 * (HB + XB), s));
  if (users_done && !xbuf) {  // user rows W scratch -> the user shard
    a.slot_waves = S;
    a.hot_waves = 0;
    ACF_RET(launch(K.flush, a, S, s));
  }
  return ACF_OK;
}

extern "C" int acf_apr_shard_pass(acf_apr_ctx* c, const acf_apr_tables* tb, const acf_apr_hparams* hp,
                                  int32_t pass, void* stream_) {
  return acf_apr_shard_pass_export(c, tb, hp, pass, nullptr, nullptr, 0, stream_);
}

// item slot rows of the current one-batch plan (slots nU .. nU + n, nU read
// on device): dir 0 copies g0 -> buf, dir 1 copies buf -> delta; with a map,
// working-set entry w sits in buf row map[w] (the split step's exchange rows)
__global__ void k_shard_items(float* __restrict__ g0, float* __restrict__ delta, const int32_t* __restrict__ ubs,
                              float* __restrict__ buf, const int64_t* __restrict__ map, int64_t n4, int32_t d4,
                              int32_t dir) {
  const int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (x >= n4) return;
  const int64_t off = (int64_t)(ubs[1] - ubs[0]) * d4;
  int64_t bx = x;
  if (map) {
    const int64_t w = x / d4;
    bx = map[w] * d4 + (x - w * d4);
  }
  float4* b = reinterpret_cast<float4*>(buf) + bx;
  if (dir == 0) *b = reinterpret_cast<const float4*>(g0)[off + x];
  else reinterpret_cast<float4*>(delta)[off + x] = *b;
}

extern "C" int acf_apr_shard_items_mapped(acf_apr_ctx* c, int32_t dir, float* buf, const int64_t* map,
                                          int64_t n_items, void* stream_) {
  ACF_CHECK(c && (buf || n_items == 0), ACF_E_INVALID, "NULL argument");
  ACF_RET(resolve(c, 2));  // settle queued streamed calls first (FailGroup)
  ACF_CHECK(c->shard && (c->nb == 1 || (c->tri && c->nb > 1)), ACF_E_STATE,
            "shard items need shard mode and a one-batch plan (or a triplet-centric plan of several)");
  ACF_CHECK(dir == 0 || dir == 1, ACF_E_INVALID, "dir must be 0 or 1");
  ACF_CHECK(n_items >= 0 && n_items <= 2 * (int64_t)c->B, ACF_E_INVALID, "n_items %lld outside [0, 2B]",
            (long long)n_items);
  if (c->tri) {  // triplet-centric shard passes read the deltas where they are (dir 1)
    ACF_CHECK(dir == 1 && map, ACF_E_STATE, "triplet-centric shard plans take the owners' deltas by map (dir 1)");
    c->xdelta = buf;
    c->xdmap = map;
    return ACF_OK;
  }
  if (n_items == 0) return ACF_OK;
  ACF_CHECK(c->nb == 1, ACF_E_STATE, "slot-plan shard items take one-batch plans");
  hipStream_t s = static_cast<hipStream_t>(stream_);
  const int64_t n4 = n_items * (c->d / 4);
  k_shard_items<<<grid_for(n4), 256, 0, s>>>(c->g0, c->delta, c->ubs, buf, map, n4, c->d / 4, dir);
  HIP_TRY(hipGetLastError());
  return ACF_OK;
}

extern "C" int acf_apr_shard_items(acf_apr_ctx* c, int32_t dir, float* buf, int64_t n_items, void* stream_) {
  return acf_apr_shard_items_mapped(c, dir, buf, nullptr, n_items, stream_);
}

// Owner side: the partial rows the requesters sent, grouped per owned row by
// `seg` (seg[s] .. seg[s+1] index `pos`, positions into `recv` in requester
// order: a fixed summation order).  One lane-group per owned row.
// k_shard_delta: G = sum -> G0[s]; delta = eps * l2_normalize(G) (APR.py:186-191)
// to every position of the row (the reply, in `recv` order).
template <int LPR, int NV>
__global__ void __launch_bounds__(256) k_shard_delta(StepArgs a, const float* __restrict__ recv,
                                                     const int32_t* __restrict__ seg,
                                                     const int32_t* __restrict__ pos, int32_t nseg,
                                                     float* __restrict__ G0, float* __restrict__ reply) {
  const int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int sx = (int)(gid / LPR), l = (int)(threadIdx.x & (LPR - 1));
  if (sx >= nseg) return;
  const int d = a.d;
  RowV<NV> G = zero_row<NV>();
  for (int p = seg[sx]; p < seg[sx + 1]; ++p) G = add_row(G, load_row<LPR, NV>(recv, pos[p], d, l));
  store_row<LPR, NV>(G0, sx, d, l, G);
  const RowV<NV> dl = a.zero_delta ? zero_row<NV>() : make_delta<LPR, NV>(a, G, 1, 0, l);
  for (int p = seg[sx]; p < seg[sx + 1]; ++p) store_row<LPR, NV>(reply, pos[p], d, l, dl);
}

// k_shard_apply: G = G0[s] + reg_adv * sum (APR) or sum (BPR), then TF's sparse
// Adagrad on the owned row (Q[rows[s]], accQ[rows[s]]), the reg term counting
// the row's occurrences in the global batch (count[s]).
template <int LPR, int NV>
__global__ void __launch_bounds__(256) k_shard_apply(StepArgs a, const float* __restrict__ recv,
                                                     const int32_t* __restrict__ seg,
                                                     const int32_t* __restrict__ pos, int32_t nseg,
                                                     const float* __restrict__ G0,
                                                     const int32_t* __restrict__ rows,
                                                     const int32_t* __restrict__ count) {
  const int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int sx = (int)(gid / LPR), l = (int)(threadIdx.x & (LPR - 1));
  if (sx >= nseg) return;
  const int d = a.d;
  RowV<NV> G = zero_row<NV>();
  for (int p = seg[sx]; p < seg[sx + 1]; ++p) G = add_row(G, load_row<LPR, NV>(recv, pos[p], d, l));
  RowV<NV> Gt = G;
  if (a.adver) {
    Gt = load_row<LPR, NV>(G0, sx, d, l);
    axpy_row(Gt, a.reg_adv, G);
  }
  const int32_t row = rows[sx];
  const RowV<NV> w = load_row<LPR, NV>(a.Q, row, d, l);
  RowV<NV> acc = load_row<LPR, NV>(a.accQ, row, d, l);
  RowV<NV> wout;
  adagrad_row(a, Gt, w, acc, count ? count[sx] : 0, wout);
  store_row<LPR, NV>(a.accQ, row, d, l, acc);
  store_row<LPR, NV>(a.Q, row, d, l, wout);
}

static StepArgs owner_args(const acf_apr_hparams* hp, float* Q, float* accQ, int32_t d, int32_t reg_batch) {
  StepArgs a;
  memset(&a, 0, sizeof(a));
  a.Q = Q; a.accQ = accQ; a.d = d; a.B = reg_batch; a.reg_B = reg_batch;
  a.lr = hp->lr; a.eps = hp->eps; a.reg = hp->reg; a.reg_adv = hp->reg_adv;
  a.clip_lo = hp->clip_lo; a.clip_hi = hp->clip_hi;
  a.adver = hp->adver; a.adv_mode = hp->adv_mode; a.zero_delta = hp->zero_delta; a.seed = hp->seed;
  return a;
}

template <int LPR, int NV>
static void launch_shard_delta(const StepArgs& a, const float* recv, const int32_t* seg, const int32_t* pos,
                               int32_t nseg, float* G0, float* reply, hipStream_t s) {
  k_shard_delta<LPR, NV><<<grid_for((int64_t)nseg * LPR), 256, 0, s>>>(a, recv, seg, pos, nseg, G0, reply);
}

template <int LPR, int NV>
static void launch_shard_apply(const StepArgs& a, const float* recv, const int32_t* seg, const int32_t* pos,
                               int32_t nseg, const float* G0, const int32_t* rows, const int32_t* count,
                               hipStream_t s) {
  k_shard_apply<LPR, NV><<<grid_for((int64_t)nseg * LPR), 256, 0, s>>>(a, recv, seg, pos, nseg, G0, rows, count);
}

extern "C" int acf_shard_reduce_delta(const float* recv, const int32_t* seg, const int32_t* pos, int32_t n_rows,
                                      int32_t d, const acf_apr_hparams* hp, float* G0, float* reply,
                                      void* stream_) {
  ACF_RET(check_dim(d));
  ACF_CHECK(hp && n_rows >= 0, ACF_E_INVALID, "bad argument");
  ACF_CHECK(hp->adv_mode == 0, ACF_E_INVALID, "shard mode supports adv = grad only");
  if (n_rows == 0) return ACF_OK;
  ACF_CHECK(recv && seg && pos && G0 && reply, ACF_E_INVALID, "NULL pointer");
  const StepArgs a = owner_args(hp, nullptr, nullptr, d, 1);
  ACF_RET(DISPATCH_GEOM(d, launch_shard_delta, a, recv, seg, pos, n_rows, G0, reply,
                        static_cast<hipStream_t>(stream_)));
  HIP_TRY(hipGetLastError());
  return ACF_OK;
}

extern "C" int acf_shard_reduce_apply(float* Q, float* accQ, const float* recv, const int32_t* seg,
                                      const int32_t* pos, int32_t n_rows, int32_t d, const acf_apr_hparams* hp,
                                      const float* G0, const int32_t* rows, const int32_t* count,
                                      int32_t reg_batch, void* stream_) {
  ACF_RET(check_dim(d));
  ACF_CHECK(hp && n_rows >= 0, ACF_E_INVALID, "bad argument");
  if (n_rows == 0) return ACF_OK;
  ACF_CHECK(Q && accQ && recv && seg && pos && rows && (G0 || !hp->adver), ACF_E_INVALID, "NULL pointer");
  ACF_CHECK(hp->reg == 0.f || (count && reg_batch > 0), ACF_E_INVALID, "reg != 0 needs counts and reg_batch");
  const StepArgs a = owner_args(hp, Q, accQ, d, reg_batch > 0 ? reg_batch : 1);
  ACF_RET(DISPATCH_GEOM(d, launch_shard_apply, a, recv, seg, pos, n_rows, G0, rows, count,
                        static_cast<hipStream_t>(stream_)));
  HIP_TRY(hipGetLastError());
  return ACF_OK;
}

extern "C" int acf_apr_step_errors(acf_apr_ctx* c, int32_t* out, void* stream_) {
  ACF_CHECK(c && out, ACF_E_INVALID, "NULL argument");
  ACF_RET(resolve(c, 2));  // settle queued streamed calls first (FailGroup)
  hipStream_t s = static_cast<hipStream_t>(stream_);
  int32_t w = 0;
  HIP_TRY(hipMemcpyAsync(&w, c->err + 1, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemsetAsync(c->err + 1, 0, sizeof(int32_t), s));
  HIP_TRY(hipStreamSynchronize(s));
  *out = w;  // sticky: step waits that gave up, and unverified streamed calls that did (dropped)
  return ACF_OK;
}

extern "C" int acf_apr_set_failsafe(acf_apr_ctx* c, int32_t on) {
  ACF_CHECK(c, ACF_E_INVALID, "ctx is NULL");
  ACF_RET(resolve(c, 2));  // settle queued streamed calls first (FailGroup)
  ACF_CHECK(on == 0 || on == 1, ACF_E_INVALID, "failsafe must be 0 or 1, got %d", on);
  c->failsafe = on;
  return ACF_OK;
}

extern "C" int acf_apr_set_spin_limit(acf_apr_ctx* c, int32_t polls) {
  ACF_CHECK(c, ACF_E_INVALID, "ctx is NULL");
  ACF_RET(resolve(c, 2));  // settle queued streamed calls first (FailGroup)
  ACF_CHECK(polls >= 0, ACF_E_INVALID, "spin limit must be >= 0, got %d", polls);
  c->spin_limit = polls;
  return ACF_OK;
}

extern "C" int acf_apr_stream_recoveries(acf_apr_ctx* c, int64_t* out) {
  ACF_CHECK(c && out, ACF_E_INVALID, "NULL argument");
  ACF_RET(resolve(c, 2));  // settle queued streamed calls first (FailGroup)
  *out = c->recoveries;
  return ACF_OK;
}

extern "C" int acf_apr_copy_losses(acf_apr_ctx* c, float* lc, float* la, void* stream_) {
  ACF_CHECK(c, ACF_E_INVALID, "ctx is NULL");
  ACF_RET(resolve(c, 2));  // settle queued streamed calls first (FailGroup)
  ACF_CHECK(c->nb > 0, ACF_E_STATE, "no batches planned");
  hipStream_t s = static_cast<hipStream_t>(stream_);
  const size_t n = (size_t)c->B * c->nb * sizeof(float);
  if (lc) HIP_TRY(hipMemcpyAsync(lc, c->loss_clean, n, hipMemcpyDeviceToDevice, s));
  if (la) HIP_TRY(hipMemcpyAsync(la, c->loss_adv, n, hipMemcpyDeviceToDevice, s));
  return ACF_OK;
}

extern "C" int acf_apr_delta_scatter(acf_apr_ctx* c, float* dP, float* dQ, void* stream_) {
  ACF_CHECK(c && dP && dQ, ACF_E_INVALID, "NULL argument");
  ACF_RET(resolve(c, 2));  // settle queued streamed calls first (FailGroup)
  ACF_CHECK(c->last_delta_batch >= 0, ACF_E_STATE, "no delta computed since the last step");
  hipStream_t s = static_cast<hipStream_t>(stream_);
  acf_apr_tables tb{nullptr, nullptr, nullptr, nullptr};
  acf_apr_hparams hp;
  memset(&hp, 0, sizeof(hp));
  StepArgs a = make_args(c, &tb, &hp, c->last_delta_batch, 0);
  k_delta_scatter<<<(3 * c->B + 3) / 4, 256, 0, s>>>(a, dP, dQ);
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

// kernel: 0 auto (ACF_EVAL_AUTO_VALU_PAIRS), 1 the fused MFMA sweep, 2 the VALU
// sweep k_eval_all (A/B and tests); positions are identical.
#define ACF_EVAL_VALU_PAIRS 0  // auto: the VALU sweep below this many user x candidate pairs

static int eval_positions_all(const float* P, const float* Q, int64_t U1, int64_t I1, int32_t d,
                              const int32_t* users, const int32_t* tests, int32_t n_users, int32_t num_cand,
                              const int64_t* excl_off, const int32_t* excl, int32_t* positions, int32_t kernel,
                              void* stream_) {
  ACF_RET(check_dim(d));
  ACF_CHECK(P && Q && users && tests && excl_off && positions, ACF_E_INVALID, "NULL argument");
  ACF_CHECK(num_cand >= 0 && num_cand <= I1, ACF_E_INVALID, "num_candidates %d > item rows", num_cand);
  ACF_CHECK(kernel >= 0 && kernel <= 2, ACF_E_INVALID, "kernel must be 0 (auto), 1 (MFMA) or 2 (VALU), got %d",
            kernel);
  if (n_users <= 0) return ACF_OK;
  hipStream_t s = static_cast<hipStream_t>(stream_);
  if (kernel == 0) kernel = (int64_t)n_users * num_cand < ACF_EVAL_VALU_PAIRS ? 2 : 1;
  if (kernel == 2) {
    const size_t lds = (size_t)EVAL_UB * d * sizeof(float);
    k_eval_all<<<(n_users + EVAL_UB - 1) / EVAL_UB, 256, lds, s>>>(P, Q, d, users, tests, n_users,
                                                                    num_cand, excl_off, excl, positions);
    HIP_TRY(hipGetLastError());
    return ACF_OK;
  }
  float* tscore = nullptr;
  HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&tscore), (size_t)n_users * sizeof(float), s));
  k_eval_tscore<<<grid_for(n_users), 256, 0, s>>>(P, Q, d, users, tests, n_users, tscore, positions);
  if (num_cand > 0) {
    const float eb = 4.0f * (float)(d + 2) * 5.9604645e-8f;  // 4 (d + 2) 2^-24
    const float floor_e = (float)d * 1.1754944e-38f * 4.0f;   // denormal products flushed by MFMA
    const dim3 grid((unsigned)((num_cand + EVM_C - 1) / EVM_C), (unsigned)((n_users + EVM_U - 1) / EVM_U));
    k_eval_fused<<<grid, 256, 0, s>>>(P, Q, d, users, tscore, n_users, num_cand, excl_off, excl, eb, floor_e,
                                      positions);
  }
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipFreeAsync(tscore, s));
  return ACF_OK;
}

extern "C" int acf_eval_positions_all(const float* P, const float* Q, int64_t U1, int64_t I1,
                                      int32_t d, const int32_t* users, const int32_t* tests,
                                      int32_t n_users, int32_t num_cand, const int64_t* excl_off,
                                      const int32_t* excl, int32_t* positions, void* stream_) {
  return eval_positions_all(P, Q, U1, I1, d, users, tests, n_users, num_cand, excl_off, excl, positions, 0,
                            stream_);
}

extern "C" int acf_eval_positions_all_kernel(const float* P, const float* Q, int64_t U1, int64_t I1, int32_t d,
                                             const int32_t* users, const int32_t* tests, int32_t n_users,
                                             int32_t num_cand, const int64_t* excl_off, const int32_t* excl,
                                             int32_t* positions, int32_t kernel, void* stream_) {
  return eval_positions_all(P, Q, U1, I1, d, users, tests, n_users, num_cand, excl_off, excl, positions, kernel,
                            stream_);
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

static int sample_epoch(const int32_t* pu, const int32_t* pi, int64_t n_pos, int32_t B, int32_t num_items,
                        int32_t num_lists, const int64_t* loff, const int32_t* litems, uint64_t seed,
                        int32_t max_tries, int32_t check, const float* prob, const int32_t* alias, int32_t* ou,
                        int32_t* op, int32_t* on, void* stream_);

extern "C" int acf_sample_epoch(const int32_t* pu, const int32_t* pi, int64_t n_pos, int32_t B,
                                int32_t num_items, int32_t num_lists, const int64_t* loff,
                                const int32_t* litems, uint64_t seed, int32_t max_tries,
                                int32_t check, int32_t* ou, int32_t* op, int32_t* on,
                                void* stream_) {
  return sample_epoch(pu, pi, n_pos, B, num_items, num_lists, loff, litems, seed, max_tries, check, nullptr,
                      nullptr, ou, op, on, stream_);
}

extern "C" int acf_sample_epoch_alias(const int32_t* pu, const int32_t* pi, int64_t n_pos, int32_t B,
                                      int32_t num_items, int32_t num_lists, const int64_t* loff,
                                      const int32_t* litems, const float* prob, const int32_t* alias,
                                      uint64_t seed, int32_t max_tries, int32_t check, int32_t* ou,
                                      int32_t* op, int32_t* on, void* stream_) {
  ACF_CHECK(prob && alias, ACF_E_INVALID, "NULL alias table");
  return sample_epoch(pu, pi, n_pos, B, num_items, num_lists, loff, litems, seed, max_tries, check, prob, alias,
                      ou, op, on, stream_);
}

// Vose's alias method, on the host in double precision (one pass, O(n)):
// prob[k] = the chance that column k keeps k; otherwise it yields alias[k].
extern "C" int acf_alias_build(const float* w, int64_t n, float* prob, int32_t* alias) {
  ACF_CHECK(w && prob && alias && n > 0 && n < (1ll << 31), ACF_E_INVALID, "bad alias-table arguments");
  double total = 0.0;
  for (int64_t k = 0; k < n; ++k) {
    ACF_CHECK(w[k] >= 0.f && std::isfinite(w[k]), ACF_E_INVALID, "weight %lld is negative or not finite",
              (long long)k);
    total += w[k];
  }
  ACF_CHECK(total > 0.0, ACF_E_INVALID, "weights sum to zero");
  std::vector<double> q((size_t)n);
  std::vector<int32_t> small, large;
  for (int64_t k = 0; k < n; ++k) {
    q[(size_t)k] = (double)w[k] * (double)n / total;
    (q[(size_t)k] < 1.0 ? small : large).push_back((int32_t)k);
  }
  while (!small.empty() && !large.empty()) {
    const int32_t s = small.back(), l = large.back();
    small.pop_back();
    prob[s] = (float)q[(size_t)s];
    alias[s] = l;
    q[(size_t)l] = (q[(size_t)l] + q[(size_t)s]) - 1.0;
    if (q[(size_t)l] < 1.0) {
      large.pop_back();
      small.push_back(l);
    }
  }
  for (int32_t k : large) { prob[k] = 1.0f; alias[k] = k; }
  for (int32_t k : small) { prob[k] = 1.0f; alias[k] = k; }  // rounding leftovers
  return ACF_OK;
}

static int sample_epoch(const int32_t* pu, const int32_t* pi, int64_t n_pos, int32_t B, int32_t num_items,
                        int32_t num_lists, const int64_t* loff, const int32_t* litems, uint64_t seed,
                        int32_t max_tries, int32_t check, const float* prob, const int32_t* alias, int32_t* ou,
                        int32_t* op, int32_t* on, void* stream_) {
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
                                              litems, seed, max_tries, prob, alias, ou, op, on, err);
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

#ifdef ACF_DIAG
// diagnostic build only: stamp buffer [launches][cap waves][8] of uint64
extern "C" int acf_diag_set_stamps(void* buf, int32_t cap) {
  uint64_t* p = static_cast<uint64_t*>(buf);
  HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &p, sizeof(p)));
  HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_cap), &cap, sizeof(cap)));
  return ACF_OK;
}
#endif
