// Hash plan kernels (r04) of libacf_apr.so: included by acf_apr.hip after the
// plan records (OccRec, HotLists, hot_pieces) they fill; one translation unit.
#pragma once

// ---------------------------------------------------------------------------
// Hash plan (r04): the plan of triplet-centric steps (one lane-group per slot,
// fusion on, not shard mode; B >= 4,096) without the full-key radix sort.  What
// such a step reads of its plan: per triplet its rows, which of them occur once
// in the batch ("single": stepped by the triplet itself) and, for the others
// ("shared"), a slot id and the CSR position of the occurrence; per shared slot
// its row, count and CSR range (the inline record), in which the combine adds
// the occurrences' contributions IN OCCURRENCE ORDER (the slot path's bits);
// the per-batch lists of shared slots and of hot slots with their pieces.  Slot
// ids and CSR ranges may be numbered in any order; only the order inside a range
// is fixed.  So (APR.py:183-195's Unique + UnsortedSegmentSum, restated):
//  1. k_hplan_keys / k_hplan_scatter: a one-pass partition of each batch's
//     occurrences by the top pb bits of a Fibonacci hash of the (side, row) key
//     (2^pb partitions of ~384 occurrences, disjoint in keys): per-tile counts,
//     their exclusive scan, a scatter -- in place of the sort plan's radix sort;
//  2. k_hplan_dedup, one workgroup per partition: its keys counted in an LDS hash
//     table (LDS atomics only); the shared keys claim slot ids, CSR ranges and
//     list places (one global atomic per counter and workgroup) and write their
//     inline records; every occurrence gets {slot or -1, CSR position} and the
//     shared ones enter their CSR range (in LDS-atomic order).  A partition with
//     more distinct keys than the table holds is split by further hash bits and
//     done in rounds (terminates: the hash is a bijection of 32-bit keys);
//  3. k_hplan_trip: per triplet its record (coalesced reads of step 2's output),
//     at its place: the batch's fused triplets first (r06);
//  4. k_hplan_rank_small / k_hplan_rank_hot: each CSR range put in occurrence
//     order -- <= 8 entries by one thread, <= 64 by a wave (all-pairs ranks), more
//     by a workgroup (an LDS bitmap of the side's occurrence ids and its prefix
//     popcounts) -- and every shared occurrence's CSR position written.
// The bits of a step are the sort plan's (test_hash_plan_matches_sort_plan).
// (A first form inserted every occurrence into a device-wide open-addressing
// table with 64-bit CAS / add: 1.3 ms per 32-batch chunk at configs[4], the
// returning atomics serialising at the memory side on the Zipf-popular items;
// tile-aggregated, still 0.48 ms: slower than the sort plan.)
// ---------------------------------------------------------------------------
#define ACF_HPLAN_MAXB 65536
#define ACF_OCC_HOT 0x40000000  // occ[].x: the slot is hot (more than ACF_HOT_MIN occurrences)  // the hot-rank bitmap: 2B bits of LDS per workgroup
// partitions of ~384 occurrences, 1,024 LDS buckets (~768 / 2,048 was 0.5% slower at
// configs[4], r04 A/B); a round takes at most 3/4 of the buckets
#define ACF_HPLAN_PART 384
#define ACF_HPLAN_BUCKETS 1024

struct HPlanArgs {
  const int32_t* user;
  const int32_t* ipos;
  const int32_t* ineg;
  int64_t U1, I1;
  int32_t B, S, nb, gen, pb;  // pb: partition bits (2^pb partitions per batch)
  int32_t tpb;                // tiles of ACF_HPLAN_PTILE occurrences per batch
  uint32_t* ppr;              // [nb][3B] partition << 16 | place in the tile's share of it
  unsigned long long* pstage; // [nb][3B] key << 32 | occurrence, occurrence order
  unsigned long long* pval;   // [nb][3B] the same, partition order
  int32_t* pcnt;              // [nb][2^pb][tpb] occurrences per (partition, tile)
  int32_t* poff;              // its exclusive scan: where each (partition, tile) share starts
  int2* occ;                  // [nb][3B] occurrence -> {slot or -1 (single), CSR position}
  int4* claims;               // [nb][3B / 2] HClaim: a partition's shared keys from x0 / 2
  int32_t shard;              // shard mode: no fused triplets (an item's single occurrence is a partial sum)
  int32_t* ptot;              // [nb << pb][6] partition totals
  int32_t* pbase;             // [nb << pb][6] their exclusive scans over the batch
  int32_t* csr;               // [nb][3B] occurrence ids by CSR position: users [0, B), items B + [0, 2B)
  int32_t* scnt;              // [nb] shared slots
  int32_t* ucsr;              // [nb] user CSR positions taken
  int32_t* icsr;              // [nb] item CSR positions taken
  OccRec* inl;
  OccRec* trec;
  int32_t* tpos;              // [E][4] CSR positions of the triplet's occurrences (at its place, perm)
  // (r06) triplet places: each batch's fused triplets first, the others after them
  // (k_hplan_trip), so the step's waves are all-fused or all-shared and the clean
  // pass starts past the fused ones
  int32_t* perm;              // [E] triplet e -> its place t * B + x (trec / tpos index)
  int32_t* tcnt;              // [nb] fused triplets of each batch (placed first)
  int32_t ttiles;             // tiles of 256 triplets per batch (k_hplan_tcount / k_hplan_trip)
  unsigned long long* ttc;    // [nb * ttiles + 1] per tile: fused | plain << 32 (+ a zero)
  unsigned long long* tto;    // its exclusive scan: both counts before each tile (the last: all)
  int32_t* slot_list;
  int32_t* slot_cnt;
  int32_t* flush_cnt;
  int32_t* saux;              // [nb][S] beside slot_list: CSR base | count << 24 | item << 31
  int32_t* haux;              // [nb][hot_stride] beside the hot list: CSR base | item << 31
  HotLists hl;
  int32_t* err;
  int32_t* gen_ptr;
};

__device__ __forceinline__ uint32_t hplan_hash(uint32_t key) { return key * 2654435761u; }  // Fibonacci

// the (side, row) of occurrence o of batch t (users [0, B), items B + 2e + role)
__device__ __forceinline__ uint32_t hplan_key(const HPlanArgs& p, int32_t t, int32_t o, int& err) {
  const int B = p.B;
  if (o < B) {
    int32_t row = p.user[(int64_t)t * B + o];
    if (row < 0 || row >= p.U1) { err |= 1; row = 0; }
    return (uint32_t)row;
  }
  const int v = o - B;
  int32_t row = ((v & 1) ? p.ineg : p.ipos)[(int64_t)t * B + (v >> 1)];
  if (row < 0 || row >= p.I1) { err |= 2; row = 0; }
  return 0x80000000u | (uint32_t)row;
}

// One workgroup per tile of ACF_HPLAN_PTILE occurrences of a batch: keys,
// partitions, each occurrence's place among the tile's occurrences of its
// partition (LDS atomics) and the tile's per-partition counts; after their
// exclusive scan (partition-major inside each batch) k_hplan_scatter moves
// every occurrence to its partition's range -- a one-pass partition, instead of
// a radix sort.  The plan's counters start at zero here too (instead of six
// fills: a fill launch costs ~9 us).
#define ACF_HPLAN_PIPT 8
#define ACF_HPLAN_PTILE (256 * ACF_HPLAN_PIPT)

__global__ void __launch_bounds__(256) k_hplan_keys(HPlanArgs p) {
  __shared__ int32_t hist[512];
  const int S3 = 3 * p.B, P = 1 << p.pb, tid = threadIdx.x;
  const int32_t t = blockIdx.x / p.tpb, tile = blockIdx.x - t * p.tpb;
  const int64_t gx = blockIdx.x * 256ll + tid, G = (int64_t)gridDim.x * 256;
  for (int64_t x = gx; x < (int64_t)p.nb * p.hl.piece_stride; x += G) p.hl.arrive[x] = 0;
  if (gx < p.nb) {
    p.scnt[gx] = p.ucsr[gx] = p.icsr[gx] = 0;
    p.slot_cnt[gx] = p.flush_cnt[gx] = 0;
    p.hl.cnt[gx] = p.hl.pcnt[gx] = 0;
  }
  for (int q = tid; q < P; q += 256) hist[q] = 0;
  __syncthreads();
  // every key's loads first, then the LDS counts, then the stores
  int err = 0;
  uint32_t key[ACF_HPLAN_PIPT];
#pragma unroll
  for (int q = 0; q < ACF_HPLAN_PIPT; ++q) {
    const int32_t o = tile * ACF_HPLAN_PTILE + q * 256 + tid;
    key[q] = o < S3 ? hplan_key(p, t, o, err) : 0u;
  }
  if (err) atomicOr(p.err, err);
  uint32_t pr[ACF_HPLAN_PIPT];
#pragma unroll
  for (int q = 0; q < ACF_HPLAN_PIPT; ++q) {
    const int32_t o = tile * ACF_HPLAN_PTILE + q * 256 + tid;
    const uint32_t part = p.pb ? hplan_hash(key[q]) >> (32 - p.pb) : 0u;
    pr[q] = o < S3 ? (part << 16) | (uint32_t)atomicAdd(&hist[part], 1) : 0u;
  }
#pragma unroll
  for (int q = 0; q < ACF_HPLAN_PIPT; ++q) {
    const int32_t o = tile * ACF_HPLAN_PTILE + q * 256 + tid;
    if (o >= S3) continue;
    p.ppr[(int64_t)t * S3 + o] = pr[q];
    p.pstage[(int64_t)t * S3 + o] = ((unsigned long long)key[q] << 32) | (uint32_t)o;
    p.occ[(int64_t)t * S3 + o] = make_int2(-1, 0);  // single until k_hplan_emit says otherwise
  }
  __syncthreads();
  for (int q = tid; q < P; q += 256) p.pcnt[((int64_t)t * P + q) * p.tpb + tile] = hist[q];
}

__global__ void __launch_bounds__(256) k_hplan_scatter(HPlanArgs p) {
  const int S3 = 3 * p.B, P = 1 << p.pb, tid = threadIdx.x;
  const int32_t t = blockIdx.x / p.tpb, tile = blockIdx.x - t * p.tpb;
  // loads in three rounds, each with all of the thread's occurrences in flight
  uint32_t pr[ACF_HPLAN_PIPT];
  unsigned long long pv[ACF_HPLAN_PIPT];
  int32_t pos[ACF_HPLAN_PIPT];
#pragma unroll
  for (int q = 0; q < ACF_HPLAN_PIPT; ++q) {
    const int32_t o = tile * ACF_HPLAN_PTILE + q * 256 + tid;
    pr[q] = o < S3 ? p.ppr[(int64_t)t * S3 + o] : 0u;
    pv[q] = o < S3 ? p.pstage[(int64_t)t * S3 + o] : 0ull;
  }
#pragma unroll
  for (int q = 0; q < ACF_HPLAN_PIPT; ++q)
    pos[q] = p.poff[((int64_t)t * P + (pr[q] >> 16)) * p.tpb + tile] + (int32_t)(pr[q] & 0xFFFFu);
#pragma unroll
  for (int q = 0; q < ACF_HPLAN_PIPT; ++q) {
    const int32_t o = tile * ACF_HPLAN_PTILE + q * 256 + tid;
    if (o < S3) p.pval[pos[q]] = pv[q];
  }
}

// exclusive prefix sum over the wave; total = the wave's sum
__device__ __forceinline__ int32_t wave_excl_sum(int32_t v, int32_t& total) {
  const int lane = threadIdx.x & 63;
  int32_t incl = v;
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) {
    const int32_t y = __shfl_up(incl, s);
    if (lane >= s) incl += y;
  }
  total = __shfl(incl, 63);
  return incl - v;
}


// Partition dedup, in three launches so that no global counter is contended
// (one workgroup per partition claiming from per-batch counters queued ~256
// same-address atomics per counter):
//  k_hplan_dedup (one workgroup per partition): the keys counted in an LDS hash
//    table, the shared ones numbered partition-locally (slot j, user / item CSR
//    offset, list / hot-list / piece places) into claims[x0 / 2 + j] (a
//    partition of n occurrences has <= n / 2 shared keys), the shared
//    occurrences as {occurrence, local CSR position, j} from x0, seven totals;
//  k_hplan_bases (one workgroup per batch): exclusive scans of the totals over
//    the batch's partitions, and the batch's list lengths;
//  k_hplan_emit (one workgroup per partition): local -> batch numbering, the
//    inline records, lists and pieces, the shared occurrences' {slot, CSR
//    position} and CSR entries (k_hplan_keys preset every occurrence to single).
// Equal LDS buckets inside a wave are counted with one atomic (the wave's first
// active lane's bucket: a Zipf-popular item fills most of its partition).
struct HClaim {
  uint32_t key;
  int32_t count;
  int32_t csr;    // CSR offset inside the partition's user or item share
  int32_t place;  // place in the partition's shared-slot list, or hot-list place | first piece << 16
};
#define ACF_HPLAN_DQ 4   // occurrences per thread loaded together in k_hplan_dedup
#define ACF_HPLAN_TOT 8  // partition totals: slots, user CSR, item CSR, list, hot, pieces, shared occurrences

// lanes with act add 1 to cnt[lh]; returns each lane's count before its add.
// The first active lane's bucket is added once for all lanes that share it.
__device__ __forceinline__ int32_t wave_lds_count(int32_t* cnt, uint32_t lh, bool act) {
  const unsigned long long m = __ballot(act);
  int32_t before = 0;
  if (!m) return 0;
  const int lane = threadIdx.x & 63, lead = __ffsll((long long)m) - 1;
  const uint32_t L = __shfl(lh, lead);
  const bool mine = act && lh == L;
  const unsigned long long same = __ballot(mine);
  int32_t b = 0;
  if (lane == lead) b = atomicAdd(&cnt[L], __popcll(same));
  b = __shfl(b, lead);
  if (mine) before = b + __popcll(same & ((1ull << lane) - 1ull));
  else if (act) before = atomicAdd(&cnt[lh], 1);
  return before;
}

template <int TS>
__global__ void __launch_bounds__(256) k_hplan_dedup(HPlanArgs p) {
  constexpr int EPT = TS / 256;  // LDS buckets per thread in the claims
  __shared__ uint32_t lkey[TS];
  __shared__ int32_t lcnt[TS];  // count, then the CSR cursor
  __shared__ int32_t lk[TS];    // local slot (-1: the row occurs once)
  __shared__ int32_t lb[TS];    // local CSR offset
  __shared__ int32_t s_at[4][6];
  __shared__ int32_t s_run[ACF_HPLAN_TOT];
  __shared__ int32_t s_distinct, s_over;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int B = p.B, S3 = 3 * B;
  const int64_t nparts = (int64_t)p.nb << p.pb;
  const int2 seg = make_int2(p.poff[(int64_t)blockIdx.x * p.tpb],
                             blockIdx.x + 1 < nparts ? p.poff[(int64_t)(blockIdx.x + 1) * p.tpb] : p.nb * S3);
  if (tid < ACF_HPLAN_TOT) s_run[tid] = 0;
  unsigned long long* shl = p.pstage + seg.x;  // shared occurrences (k_hplan_scatter consumed pstage)
  int rbits = 0;  // rounds: 2^rbits sub-partitions by the next hash bits
  for (int r = 0; r < (1 << rbits) && seg.y > seg.x;) {
    for (int e = tid; e < TS; e += 256) {
      lkey[e] = 0xFFFFFFFFu;
      lcnt[e] = 0;
    }
    if (tid == 0) { s_distinct = 0; s_over = 0; }
    __syncthreads();
    auto in_round = [&](uint32_t key) -> bool {
      if (!rbits) return true;
      return (int)((hplan_hash(key) << p.pb) >> (32 - rbits)) == r;
    };
    for (int32_t i00 = seg.x; i00 < seg.y; i00 += 256 * ACF_HPLAN_DQ) {  // wave-uniform trip counts
      unsigned long long pvq[ACF_HPLAN_DQ];  // loads issued together: one round trip per 256 x DQ
#pragma unroll
      for (int q = 0; q < ACF_HPLAN_DQ; ++q) {
        const int32_t i = i00 + q * 256 + tid;
        pvq[q] = i < seg.y ? p.pval[i] : 0ull;
      }
#pragma unroll
    for (int q = 0; q < ACF_HPLAN_DQ; ++q) {
      const int32_t i = i00 + q * 256 + tid;
      const uint32_t key = (uint32_t)(pvq[q] >> 32);
      bool act = i < seg.y && in_round(key);
      uint32_t lh = (hplan_hash(key) >> 7) & (TS - 1);
      if (act) {
        for (;;) {
          uint32_t cur = lkey[lh];
          if (cur == 0xFFFFFFFFu) {
            if (__hip_atomic_load(&s_over, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
              act = false;
              break;
            }
            cur = atomicCAS(&lkey[lh], 0xFFFFFFFFu, key);
            if (cur == 0xFFFFFFFFu) {
              cur = key;
              if (atomicAdd(&s_distinct, 1) >= TS * 3 / 4) atomicOr(&s_over, 1);
            }
          }
          if (cur == key) break;
          lh = (lh + 1u) & (TS - 1);
        }
      }
      (void)wave_lds_count(lcnt, lh, act);
    }
    }
    __syncthreads();
    if (s_over) {  // too many distinct keys: this round again as two halves
      r <<= 1;
      ++rbits;
      __syncthreads();
      continue;
    }
    // local numbering of the round's shared keys (count > 1), after the earlier rounds'
    int32_t v[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
      const int e = tid * EPT + q;
      const int32_t c = lkey[e] == 0xFFFFFFFFu ? 0 : lcnt[e];
      if (c < 2) continue;
      const bool item = (lkey[e] & 0x80000000u) != 0, hot = c > ACF_HOT_MIN;
      v[0] += 1;
      v[item ? 2 : 1] += c;
      v[hot ? 4 : 3] += 1;
      if (hot) v[5] += hot_pieces(c);
    }
    int32_t ex[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      int32_t tot = 0;
      ex[c] = wave_excl_sum(v[c], tot);
      if (lane == 0) s_at[wave][c] = tot;
    }
    __syncthreads();
    if (tid < 6) {
      int32_t sum = s_run[tid];
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const int32_t x = s_at[w][tid];
        s_at[w][tid] = sum;
        sum += x;
      }
      s_run[tid] = sum;
    }
    __syncthreads();
    int32_t nx[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) nx[c] = s_at[wave][c] + ex[c];
    HClaim* claims = reinterpret_cast<HClaim*>(p.claims) + seg.x / 2;
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
      const int e = tid * EPT + q;
      const uint32_t key = lkey[e];
      const int32_t c = key == 0xFFFFFFFFu ? 0 : lcnt[e];
      lk[e] = -1;
      lcnt[e] = 0;  // the CSR cursor from here on
      if (c < 2) continue;
      const bool item = (key & 0x80000000u) != 0, hot = c > ACF_HOT_MIN;
      const int32_t j = nx[0]++;
      const int32_t off = nx[item ? 2 : 1];
      nx[item ? 2 : 1] += c;
      lk[e] = j;
      lb[e] = off;
      HClaim h;
      h.key = key;
      h.count = c;
      h.csr = off;
      if (hot) {
        h.place = nx[4]++ | (nx[5] << 16);
        nx[5] += hot_pieces(c);
      } else {
        h.place = nx[3]++;
      }
      claims[j] = h;
    }
    __syncthreads();
    // the round's shared occurrences: {occurrence, local CSR position, local slot}
    for (int32_t i00 = seg.x; i00 < seg.y; i00 += 256 * ACF_HPLAN_DQ) {
      unsigned long long pvq[ACF_HPLAN_DQ];
#pragma unroll
      for (int q = 0; q < ACF_HPLAN_DQ; ++q) {
        const int32_t i = i00 + q * 256 + tid;
        pvq[q] = i < seg.y ? p.pval[i] : 0ull;
      }
#pragma unroll
    for (int q = 0; q < ACF_HPLAN_DQ; ++q) {
      const int32_t i = i00 + q * 256 + tid;
      const unsigned long long pv = pvq[q];
      const uint32_t key = (uint32_t)(pv >> 32);
      bool act = i < seg.y && in_round(key);
      uint32_t lh = (hplan_hash(key) >> 7) & (TS - 1);
      if (act) {
        while (lkey[lh] != key) lh = (lh + 1u) & (TS - 1);
        act = lk[lh] >= 0;
      }
      const int32_t rank = wave_lds_count(lcnt, lh, act);
      // append (one LDS atomic per wave)
      const unsigned long long m = __ballot(act);
      int32_t at = 0;
      if (m) {
        const int lead = __ffsll((long long)m) - 1;
        if (lane == lead) at = atomicAdd(&s_run[6], __popcll(m));
        at = __shfl(at, lead) + __popcll(m & ((1ull << lane) - 1ull));
      }
      if (act)
        shl[at] = (unsigned long long)(uint32_t)pv | ((unsigned long long)(lb[lh] + rank) << 18) |
                  ((unsigned long long)lk[lh] << 36);
    }
    }
    __syncthreads();
    ++r;
  }
  if (tid < ACF_HPLAN_TOT) p.ptot[(int64_t)blockIdx.x * ACF_HPLAN_TOT + tid] = s_run[tid];
}

// one workgroup per batch: partition bases (exclusive scans of the totals over
// the batch's partitions, <= 1,024 of them) and the batch's list lengths
__global__ void __launch_bounds__(1024) k_hplan_bases(HPlanArgs p) {
  using Scan = rocprim::block_scan<int32_t, 1024>;
  __shared__ typename Scan::storage_type st;
  const int32_t t = blockIdx.x, P = 1 << p.pb, tid = threadIdx.x;
  const int64_t at = ((int64_t)t * P + tid) * ACF_HPLAN_TOT;
  for (int c = 0; c < 6; ++c) {
    const int32_t v = tid < P ? p.ptot[at + c] : 0;
    int32_t ex = 0, tot = 0;
    Scan().exclusive_scan(v, ex, 0, tot, st);
    if (tid < P) p.pbase[at + c] = ex;
    if (tid == 0) {
      if (c == 3) p.slot_cnt[t] = tot;
      if (c == 4) p.hl.cnt[t] = tot;
      if (c == 5) p.hl.pcnt[t] = tot;
    }
    __syncthreads();  // the scan storage is reused
  }
}

__global__ void __launch_bounds__(256) k_hplan_emit(HPlanArgs p) {
  __shared__ int32_t base[6];
  const int tid = threadIdx.x;
  const int B = p.B, S3 = 3 * B;
  const int32_t t = blockIdx.x >> p.pb;
  const int64_t x0 = p.poff[(int64_t)blockIdx.x * p.tpb];
  if (tid < 6) base[tid] = p.pbase[(int64_t)blockIdx.x * ACF_HPLAN_TOT + tid];
  const int32_t nclaims = p.ptot[(int64_t)blockIdx.x * ACF_HPLAN_TOT];
  const int32_t nsh = p.ptot[(int64_t)blockIdx.x * ACF_HPLAN_TOT + 6];
  if (nclaims == 0) return;  // uniform
  __syncthreads();
  const HClaim* claims = reinterpret_cast<const HClaim*>(p.claims) + x0 / 2;
  for (int32_t j = tid; j < nclaims; j += 256) {
    const HClaim h = claims[j];
    const bool item = (h.key & 0x80000000u) != 0, hot = h.count > ACF_HOT_MIN;
    const int32_t k = base[0] + j, csr = (item ? base[2] : base[1]) + h.csr;
    OccRec rec = {};
    rec.own_row = (int32_t)(h.key & 0x7FFFFFFFu);
    rec.own_src = rec.own_row;
    rec.meta = h.count | (item ? ACF_ITEM_BIT : 0);
    rec.ovf = (item ? t * 2 * B : t * B) + csr;
    rec.e_role = -1;
    rec.gen = p.gen;
    p.inl[(int64_t)t * p.S + k] = rec;
    const int32_t aux = csr | (item ? (int32_t)0x80000000 : 0);  // the rank kernels' view
    if (!hot) {
      const int32_t ls = base[3] + h.place;
      p.slot_list[(int64_t)t * p.S + ls] = k;
      p.saux[(int64_t)t * p.S + ls] = aux | (h.count << 24);
    } else {
      const int32_t hx = base[4] + (h.place & 0xFFFF), pb0 = base[5] + (h.place >> 16), np = hot_pieces(h.count);
      p.hl.list[(int64_t)t * p.hl.hot_stride + hx] = make_int4(k, np, pb0, h.count);
      p.haux[(int64_t)t * p.hl.hot_stride + hx] = aux;
      int4* pc = p.hl.piece + (int64_t)t * p.hl.piece_stride + pb0;
      int2* pa = p.hl.paux + (int64_t)t * p.hl.piece_stride + pb0;
      for (int32_t w = 0; w < np; ++w) {
        pc[w] = make_int4(k, w, np, pb0);
        pa[w] = make_int2(h.count, aux);
      }
    }
  }
  const unsigned long long* shl = p.pstage + x0;
  for (int32_t x = tid; x < nsh; x += 256) {
    const unsigned long long v = shl[x];
    const int32_t o = (int32_t)(v & 0x3FFFFull), lpos = (int32_t)((v >> 18) & 0x3FFFFull), j = (int32_t)(v >> 36);
    const bool item = o >= B;
    const int32_t pos = (item ? base[2] : base[1]) + lpos;
    // a hot slot's occurrences carry ACF_OCC_HOT (k_hplan_trip places their triplets last)
    const bool hot = claims[j].count > ACF_HOT_MIN;
    p.occ[(int64_t)t * S3 + o] = make_int2((base[0] + j) | (hot ? ACF_OCC_HOT : 0), pos);
    p.csr[(int64_t)t * S3 + (item ? B : 0) + pos] = item ? o - B : o;
  }
}

// (r06) triplet places, in three classes: the batch's fused triplets (all rows
// single), then the "plain" ones (shared rows, none of them hot), then those
// with a hot row -- each class in triplet order.  k_tri_cadv runs them in that
// order: the fused ones need no delta, and the hot slots' deltas (the longest
// chains of the combine at the head of the launch) are needed last.  Per tile of
// 256 triplets the two counts (k_hplan_tcount), their exclusive scan over the
// tiles (rocPRIM, packed fused | plain << 32), then k_hplan_trip writes every
// triplet at its place.  Deterministic; any place gives the same bits (a
// triplet's arithmetic and the CSR order of its contributions do not depend on
// it).  (A first form took places from two per-batch counters with one atomic
// per wave: ~1,000 same-address returning atomics per counter and batch
// serialised at the memory side and slowed the plan beside the step, configs[4]
// d = 64 737M -> 662M.)
// class of triplet b of batch t: 0 fused, 1 plain, 2 hot (occ rows as k_hplan_emit left them)
__device__ __forceinline__ int hplan_class(const HPlanArgs& p, int2 su, int2 si, int2 sj) {
  if (su.x < 0 && si.x < 0 && sj.x < 0 && !p.shard) return 0;
  const bool hot = (su.x >= 0 && (su.x & ACF_OCC_HOT)) || (si.x >= 0 && (si.x & ACF_OCC_HOT)) ||
                   (sj.x >= 0 && (sj.x & ACF_OCC_HOT));
  return hot ? 2 : 1;
}

// ranks of the workgroup's lanes among those with f0 / with f1 (lanes in order),
// and the workgroup totals
__device__ __forceinline__ int2 block_rank2(bool f0, bool f1, int32_t* s_w, int2& total) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const unsigned long long m0 = __ballot(f0), m1 = __ballot(f1);
  if (lane == 0) {
    s_w[wave] = __popcll(m0);
    s_w[4 + wave] = __popcll(m1);
  }
  __syncthreads();
  int2 before = make_int2(0, 0);
  total = make_int2(0, 0);
  for (int w = 0; w < 4; ++w) {
    if (w < wave) {
      before.x += s_w[w];
      before.y += s_w[4 + w];
    }
    total.x += s_w[w];
    total.y += s_w[4 + w];
  }
  const unsigned long long below = (1ull << lane) - 1ull;
  return make_int2(before.x + __popcll(m0 & below), before.y + __popcll(m1 & below));
}

__device__ __forceinline__ void hplan_occ3(const HPlanArgs& p, int32_t t, int32_t b, int2& su, int2& si, int2& sj) {
  const int64_t ob = (int64_t)t * 3 * p.B;
  su = p.occ[ob + b];
  si = p.occ[ob + p.B + 2 * b];
  sj = p.occ[ob + p.B + 2 * b + 1];
}

__global__ void __launch_bounds__(256) k_hplan_tcount(HPlanArgs p) {
  __shared__ int32_t s_w[8];
  const int32_t t = blockIdx.x / p.ttiles, tile = blockIdx.x - t * p.ttiles, b = tile * 256 + threadIdx.x;
  int cls = 3;
  if (b < p.B) {
    int2 su, si, sj;
    hplan_occ3(p, t, b, su, si, sj);
    cls = hplan_class(p, su, si, sj);
  }
  int2 tot;
  (void)block_rank2(cls == 0, cls == 1, s_w, tot);
  if (threadIdx.x == 0) p.ttc[blockIdx.x] = (unsigned long long)(uint32_t)tot.x | ((unsigned long long)tot.y << 32);
  if (blockIdx.x == 0 && threadIdx.x == 0) p.ttc[p.nb * p.ttiles] = 0ull;
}

__global__ void __launch_bounds__(256) k_hplan_trip(HPlanArgs p) {
  __shared__ int32_t s_w[8];
  const int B = p.B;
  const int32_t t = blockIdx.x / p.ttiles, tile = blockIdx.x - t * p.ttiles, b = tile * 256 + threadIdx.x;
  const int64_t e = (int64_t)t * B + b;
  if (e == 0) *p.gen_ptr = p.gen;
  const bool valid = b < B;
  int2 su_ = make_int2(-1, 0), si_ = su_, sj_ = su_;
  if (valid) hplan_occ3(p, t, b, su_, si_, sj_);
  const unsigned long long o0 = p.tto[(int64_t)t * p.ttiles], ob_ = p.tto[blockIdx.x],
                           o1 = p.tto[(int64_t)(t + 1) * p.ttiles];
  const int32_t fb = (int32_t)((uint32_t)ob_ - (uint32_t)o0), pbf = (int32_t)((ob_ >> 32) - (o0 >> 32));
  const int32_t nf = (int32_t)((uint32_t)o1 - (uint32_t)o0), np = (int32_t)((o1 >> 32) - (o0 >> 32));
  const int cls = valid ? hplan_class(p, su_, si_, sj_) : 3;
  int2 tot;
  const int2 rk = block_rank2(cls == 0, cls == 1, s_w, tot);
  if (tile == 0 && threadIdx.x == 0) p.tcnt[t] = nf;
  if (!valid) return;
  // fused: after the batch's fused triplets of earlier tiles; plain: after every
  // fused one and the earlier tiles' plain ones; hot: after both classes and the
  // earlier tiles' hot ones (earlier tiles are full: 256 triplets each)
  const int32_t x = cls == 0   ? fb + rk.x
                    : cls == 1 ? nf + pbf + rk.y
                               : nf + np + (tile * 256 - fb - pbf) + ((int32_t)threadIdx.x - rk.x - rk.y);
  const int64_t at = (int64_t)t * B + x;
  su_.x = su_.x < 0 ? su_.x : (su_.x & ~ACF_OCC_HOT);
  si_.x = si_.x < 0 ? si_.x : (si_.x & ~ACF_OCC_HOT);
  sj_.x = sj_.x < 0 ? sj_.x : (sj_.x & ~ACF_OCC_HOT);
  const bool su = su_.x < 0, si = si_.x < 0, sj = sj_.x < 0;
  int err = 0;
  const int32_t u = (int32_t)hplan_key(p, t, b, err), i = (int32_t)(hplan_key(p, t, B + 2 * b, err) & 0x7FFFFFFFu),
                j = (int32_t)(hplan_key(p, t, B + 2 * b + 1, err) & 0x7FFFFFFFu);
  // fused-triplet record layout (see records_one): a = {u, i, j, slot u}, b = {slot i,
  // slot j, src u, src i}, c = {src j, flags, e, gen}; in place: sources are the rows
  OccRec q;
  q.own_row = u; q.own_src = i; q.meta = j; q.ovf = su ? 0 : su_.x;
  q.e_role = si ? 0 : si_.x; q.pa_row = sj ? 0 : sj_.x; q.pb_row = u; q.pa_src = i;
  q.pb_src = j;
  q.pa_slot = ((su && si && sj && !p.shard) ? 1 : 0) | (su ? 2 + 16 : 0) | (si ? 4 + 32 : 0) | (sj ? 8 + 64 : 0);
  q.pb_slot = (int32_t)e;  // the triplet itself (its losses' index)
  q.gen = p.gen;
  p.trec[at] = q;
  p.perm[e] = (int32_t)at;
}

// CSR position of occurrence id v (users: b; items: 2b + role) of batch t at sorted place x
__device__ __forceinline__ void hplan_put(const HPlanArgs& p, int32_t t, bool item, int32_t base, int32_t v,
                                          int32_t x) {
  const int B = p.B;
  if (!item) p.tpos[(int64_t)p.perm[(int64_t)t * B + v] * 4] = t * B + base + x;
  else p.tpos[(int64_t)p.perm[(int64_t)t * B + (v >> 1)] * 4 + 1 + (v & 1)] = t * 2 * B + base + x;
}

// shared slots of <= ACF_HOT_MIN occurrences: one thread each, a fixed
// compare-exchange network; blockIdx.y = the batch
__global__ void __launch_bounds__(256) k_hplan_rank_small(HPlanArgs p) {
  const int32_t t = blockIdx.y, n = p.slot_cnt[t];
  for (int32_t x = blockIdx.x * 256 + threadIdx.x; x < n; x += gridDim.x * 256) {
    const int32_t aux = p.saux[(int64_t)t * p.S + x];
    const bool item = aux < 0;
    const int32_t base = aux & 0xFFFFFF, cnt = (aux >> 24) & 0x7F;
    const int32_t* seg = p.csr + (int64_t)t * 3 * p.B + (item ? p.B : 0) + base;
    int32_t v[ACF_HOT_MIN];
#pragma unroll
    for (int q = 0; q < ACF_HOT_MIN; ++q) v[q] = q < cnt ? seg[q] : 0x7fffffff;
#pragma unroll
    for (int q = 1; q < ACF_HOT_MIN; ++q) {
#pragma unroll
      for (int w = q; w > 0; --w) {
        const int32_t lo = min(v[w - 1], v[w]), hi = max(v[w - 1], v[w]);
        v[w - 1] = lo;
        v[w] = hi;
      }
    }
#pragma unroll
    for (int q = 0; q < ACF_HOT_MIN; ++q)
      if (q < cnt) hplan_put(p, t, item, base, v[q], q);
  }
}

// hot slots of batch blockIdx.y: <= 64 occurrences by one wave (all-pairs
// ranks), more by the workgroup through an LDS bitmap of the side's occurrence
// ids (2B bits) and its prefix popcounts.  Dynamic LDS: 2 x ceil(2B / 32) words.
__global__ void __launch_bounds__(256) k_hplan_rank_hot(HPlanArgs p) {
  using Scan = rocprim::block_scan<int32_t, 256>;
  __shared__ typename Scan::storage_type scan_st;
  extern __shared__ uint32_t hbits[];
  const int nw = (2 * p.B + 31) >> 5;
  uint32_t* pre = hbits + nw;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int32_t t = blockIdx.y, n = p.hl.cnt[t];
  const int4* hl = p.hl.list + (int64_t)t * p.hl.hot_stride;
  const int32_t* ha = p.haux + (int64_t)t * p.hl.hot_stride;
  for (int32_t x = blockIdx.x * 4 + wave; x < n; x += gridDim.x * 4) {
    const int32_t cnt = hl[x].w;
    if (cnt > 64) continue;  // wave-uniform
    const int32_t aux = ha[x];
    const bool item = aux < 0;
    const int32_t base = aux & 0x7FFFFFFF;
    const int32_t* seg = p.csr + (int64_t)t * 3 * p.B + (item ? p.B : 0) + base;
    const int32_t v = lane < cnt ? seg[lane] : 0x7fffffff;
    int32_t rank = 0;
    for (int j = 0; j < 64; ++j) rank += __shfl(v, j) < v ? 1 : 0;
    if (lane < cnt) hplan_put(p, t, item, base, v, rank);
  }
  for (int32_t x = blockIdx.x; x < n; x += gridDim.x) {
    const int32_t cnt = hl[x].w;
    if (cnt <= 64) continue;  // uniform over the workgroup
    const int32_t aux = ha[x];
    const bool item = aux < 0;
    const int32_t base = aux & 0x7FFFFFFF;
    const int32_t* seg = p.csr + (int64_t)t * 3 * p.B + (item ? p.B : 0) + base;
    for (int w = tid; w < nw; w += 256) hbits[w] = 0u;
    __syncthreads();
    for (int32_t i = tid; i < cnt; i += 256) {
      const int32_t v = seg[i];
      atomicOr(&hbits[v >> 5], 1u << (v & 31));
    }
    __syncthreads();
    const int wpt = (nw + 255) / 256, w0 = tid * wpt;
    int32_t sum = 0;
    for (int w = w0; w < min(w0 + wpt, nw); ++w) sum += __popc(hbits[w]);
    int32_t excl = 0, tot = 0;
    Scan().exclusive_scan(sum, excl, 0, tot, scan_st);
    for (int w = w0; w < min(w0 + wpt, nw); ++w) {
      pre[w] = (uint32_t)excl;
      excl += __popc(hbits[w]);
    }
    __syncthreads();
    for (int32_t i = tid; i < cnt; i += 256) {
      const int32_t v = seg[i];
      const int32_t rank = (int32_t)pre[v >> 5] + __popc(hbits[v >> 5] & ((1u << (v & 31)) - 1u));
      hplan_put(p, t, item, base, v, rank);
    }
    __syncthreads();  // the bitmap is reused
  }
}

