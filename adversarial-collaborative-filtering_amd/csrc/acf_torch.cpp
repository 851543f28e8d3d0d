// acf_torch.cpp — PyTorch custom ops (TORCH_LIBRARY(acf, m)) over the C-ABI of
// libacf_apr.so: the APR hot path as torch.ops.acf.* on HIP tensors, the
// interface SURVEY.md §8(b) proposes.  Each op validates device / dtype /
// contiguity / shape with TORCH_CHECK, runs on the current HIP stream, and
// mutates its (a!) arguments in place.  No computation happens here: every op
// is one or two calls of the C-ABI (include/acf_apr.h).
//
//   acf::bpr_apr_step          one training_batch iteration (utils.py:114-119;
//                              APR.py:143-195): the fused streamed step
//   acf::apr_train             training_batch over n_batches (utils.py:113-119)
//   acf::gather_bpr_fwd_bwd    gathers + BPR loss + IndexedSlices grads (APR.py:121-150,183)
//   acf::row_segment_sum       IndexedSlices dedup (APR.py:183-187,195)
//   acf::l2norm_perturb        delta = eps * l2_normalize(g) (APR.py:186-191)
//   acf::sparse_adagrad_apply  SparseApplyAdagrad (APR.py:193-195)
//   acf::score_rank            _eval_by_user positions over candidate lists (utils.py:244-254)
//   acf::score_rank_all        the same over all items minus exclusions (utils.py:211-254)
#include <torch/library.h>
#include <ATen/ATen.h>
// ROCm builds of PyTorch keep the "cuda" device type: the guard and stream
// wrappers that accept it are the *MasqueradingAsCUDA ones
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include <map>
#include <memory>
#include <mutex>
#include <tuple>

#include "acf_apr.h"

namespace {

void ok(int rc, const char* what) {
  TORCH_CHECK(rc == ACF_OK, what, " failed (code ", rc, "): ", acf_apr_last_error());
}

void* stream_of(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

void need(const at::Tensor& t, const char* name, at::ScalarType dt, int64_t dim) {
  TORCH_CHECK(t.is_cuda(), name, " must be a HIP tensor (there is no CPU path)");
  TORCH_CHECK(t.scalar_type() == dt, name, " must be ", dt, ", got ", t.scalar_type());
  TORCH_CHECK(t.dim() == dim, name, " must be ", dim, "-D, got ", t.dim(), "-D");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

void need_table(const at::Tensor& t, const char* name, const at::Tensor& like) {
  need(t, name, at::kFloat, 2);
  TORCH_CHECK(t.device() == like.device(), name, " is on ", t.device(), ", expected ", like.device());
  const int64_t d = t.size(1);
  TORCH_CHECK(d >= 4 && d <= 1024 && d % 4 == 0, name, ": dim must be a multiple of 4 in [4, 1024], got ", d);
}

at::Tensor idx32(const at::Tensor& t, const char* name, const at::Tensor& like) {
  TORCH_CHECK(t.is_cuda() && t.device() == like.device(), name, " must live on ", like.device());
  TORCH_CHECK(t.scalar_type() == at::kInt || t.scalar_type() == at::kLong, name, " must be int32 or int64");
  return t.reshape({-1}).to(at::kInt).contiguous();
}

acf_apr_hparams hparams(double lr, double eps, double reg, double reg_adv, bool adver, double clip_lo,
                        double clip_hi) {
  acf_apr_hparams h;
  h.lr = (float)lr; h.eps = (float)eps; h.reg = (float)reg; h.reg_adv = (float)reg_adv;
  h.clip_lo = (float)clip_lo; h.clip_hi = (float)clip_hi;
  h.adver = adver ? 1 : 0; h.adv_mode = 0; h.seed = 0; h.zero_delta = 0; h.reserved = 0;
  return h;
}

// contexts (plan workspace + version buffers) by (device, tables, batch shape);
// one MF graph owns one in the reference (APR.py:197-202).  A context is shared
// (reference-counted) and carries its own lock, held for a whole
// train / copy_losses / step_errors sequence, so a concurrent call that evicts
// it from the cache cannot destroy it under a running op.
struct CtxKey {
  int dev;
  int64_t U1, I1;
  int32_t d, B, nb;
  bool operator<(const CtxKey& o) const {
    return std::tie(dev, U1, I1, d, B, nb) < std::tie(o.dev, o.U1, o.I1, o.d, o.B, o.nb);
  }
};
struct Ctx {
  acf_apr_ctx* c = nullptr;
  std::mutex mu;
  ~Ctx() {
    if (c) acf_apr_destroy(c);
  }
};
struct Entry {
  std::shared_ptr<Ctx> ctx;
  uint64_t last_use;
};
std::mutex g_mu;
std::map<CtxKey, Entry> g_ctx;
uint64_t g_clock = 0;
constexpr size_t kMaxContexts = 8;

std::shared_ptr<Ctx> context(const at::Tensor& P, const at::Tensor& Q, int32_t B, int32_t nb) {
  const CtxKey k{P.device().index(), P.size(0), Q.size(0), (int32_t)P.size(1), B, nb};
  std::lock_guard<std::mutex> lock(g_mu);
  auto it = g_ctx.find(k);
  if (it != g_ctx.end()) {
    it->second.last_use = ++g_clock;
    return it->second.ctx;
  }
  if (g_ctx.size() >= kMaxContexts) {  // bounded: drop the least recently used context
    auto lru = g_ctx.begin();
    for (auto e = g_ctx.begin(); e != g_ctx.end(); ++e)
      if (e->second.last_use < lru->second.last_use) lru = e;
    g_ctx.erase(lru);  // destroyed when the last running op lets go of it
  }
  auto h = std::make_shared<Ctx>();
  ok(acf_apr_create(&h->c, k.U1, k.I1, k.d, B, nb), "acf_apr_create");
  g_ctx.emplace(k, Entry{h, ++g_clock});
  return h;
}

// releases every cached context (plan workspace and k_stream version buffers,
// linear in d and batches per call); contexts still in use by a running op are
// destroyed when it returns.  Returns how many were dropped from the cache.
int64_t release_contexts() {
  std::lock_guard<std::mutex> lock(g_mu);
  const int64_t n = (int64_t)g_ctx.size();
  g_ctx.clear();
  return n;
}

// an index tensor must lie in [0, rows): TF Gather's InvalidArgument, checked
// before any kernel reads a row through it (one aminmax + one host sync)
void check_range(const at::Tensor& idx, int64_t rows, const char* name) {
  if (idx.numel() == 0) return;
  auto mm = idx.aminmax();
  const int64_t lo = std::get<0>(mm).item<int64_t>(), hi = std::get<1>(mm).item<int64_t>();
  TORCH_CHECK_INDEX(lo >= 0 && hi < rows, name, ": index ", lo < 0 ? lo : hi, " is outside [0, ", rows, ")");
}

void check_tables(const at::Tensor& P, const at::Tensor& Q, const at::Tensor& aP, const at::Tensor& aQ) {
  need_table(P, "embedding_P", P);
  need_table(Q, "embedding_Q", P);
  need_table(aP, "accumulator_P", P);
  need_table(aQ, "accumulator_Q", P);
  TORCH_CHECK(Q.size(1) == P.size(1), "embedding_P and embedding_Q dims differ");
  TORCH_CHECK(aP.sizes() == P.sizes() && aQ.sizes() == Q.sizes(), "accumulators must match their tables");
}

// training_batch over nb batches of B triplets; per-triplet losses
std::tuple<at::Tensor, at::Tensor> train(at::Tensor& P, at::Tensor& Q, at::Tensor& aP, at::Tensor& aQ,
                                         const at::Tensor& u_, const at::Tensor& i_, const at::Tensor& j_,
                                         int64_t B, double lr, double eps, double reg, double reg_adv, bool adver,
                                         double clip_lo, double clip_hi) {
  check_tables(P, Q, aP, aQ);
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(P.device());
  at::Tensor u = idx32(u_, "user", P), i = idx32(i_, "item_pos", P), j = idx32(j_, "item_neg", P);
  const int64_t n = u.numel();
  TORCH_CHECK(i.numel() == n && j.numel() == n, "triplet lengths differ");
  TORCH_CHECK(B > 0 && n > 0 && n % B == 0, n, " triplets is not a positive multiple of batch_size ", B);
  const int32_t nb = (int32_t)(n / B);
  std::shared_ptr<Ctx> held = context(P, Q, (int32_t)B, nb);
  std::lock_guard<std::mutex> ctx_lock(held->mu);
  acf_apr_ctx* c = held->c;
  acf_apr_tables tb{P.data_ptr<float>(), Q.data_ptr<float>(), aP.data_ptr<float>(), aQ.data_ptr<float>()};
  const acf_apr_hparams h = hparams(lr, eps, reg, reg_adv, adver, clip_lo, clip_hi);
  void* s = stream_of(P);
  // check = 1: an index outside its table raises (TF Gather's InvalidArgument)
  ok(acf_apr_train(c, &tb, &h, u.data_ptr<int32_t>(), i.data_ptr<int32_t>(), j.data_ptr<int32_t>(), (int32_t)B,
                   nb, 1, 1, s),
     "acf_apr_train");
  at::Tensor lc = at::empty({n}, P.options()), la = at::empty({n}, P.options());
  ok(acf_apr_copy_losses(c, lc.data_ptr<float>(), la.data_ptr<float>(), s), "acf_apr_copy_losses");
  int32_t err = 0;
  ok(acf_apr_step_errors(c, &err, s), "acf_apr_step_errors");
  TORCH_CHECK(err == 0, "the streamed step gave up waiting for a row version (step error ", err,
              "): the tables of this call are not trustworthy");
  if (!adver) la.zero_();
  return {lc, la};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> bpr_apr_step(at::Tensor& P, at::Tensor& Q, at::Tensor& aP,
                                                            at::Tensor& aQ, const at::Tensor& u, const at::Tensor& i,
                                                            const at::Tensor& j, double lr, double eps, double reg,
                                                            double reg_adv, bool adver, double clip_lo,
                                                            double clip_hi) {
  check_tables(P, Q, aP, aQ);
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(P.device());
  at::Tensor uu = idx32(u, "user", P), ii = idx32(i, "item_pos", P), jj = idx32(j, "item_neg", P);
  const int64_t B = uu.numel();
  TORCH_CHECK(B > 0 && ii.numel() == B && jj.numel() == B, "user / item_pos / item_neg must be equal, non-empty");
  // the forward below gathers rows before train()'s device-side check runs
  check_range(uu, P.size(0), "user");
  check_range(ii, Q.size(0), "item_pos");
  check_range(jj, Q.size(0), "item_neg");
  // pairwise accuracy of the batch (training_loss_acc's ACC, utils.py:159-175) before the step
  at::Tensor corr = at::empty({1}, P.options().dtype(at::kInt));
  ok(acf_bpr_forward(P.data_ptr<float>(), Q.data_ptr<float>(), P.size(0), Q.size(0), (int32_t)P.size(1),
                     uu.data_ptr<int32_t>(), ii.data_ptr<int32_t>(), jj.data_ptr<int32_t>(), (int32_t)B, 1,
                     (float)clip_lo, (float)clip_hi, nullptr, corr.data_ptr<int32_t>(), nullptr, nullptr,
                     stream_of(P)),
     "acf_bpr_forward");
  auto [lc, la] = train(P, Q, aP, aQ, uu, ii, jj, B, lr, eps, reg, reg_adv, adver, clip_lo, clip_hi);
  return {lc.sum(), la.sum(), corr.reshape({})};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> gather_bpr_fwd_bwd(
    const at::Tensor& P, const at::Tensor& Q, const at::Tensor& u_, const at::Tensor& i_, const at::Tensor& j_,
    double clip_lo, double clip_hi) {
  need_table(P, "embedding_P", P);
  need_table(Q, "embedding_Q", P);
  TORCH_CHECK(Q.size(1) == P.size(1), "embedding_P and embedding_Q dims differ");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(P.device());
  at::Tensor u = idx32(u_, "user", P), i = idx32(i_, "item_pos", P), j = idx32(j_, "item_neg", P);
  const int64_t n = u.numel(), d = P.size(1);
  TORCH_CHECK(i.numel() == n && j.numel() == n, "triplet lengths differ");
  check_range(u, P.size(0), "user");
  check_range(i, Q.size(0), "item_pos");
  check_range(j, Q.size(0), "item_neg");
  at::Tensor loss = at::empty({n}, P.options()), x = at::empty({n}, P.options());
  at::Tensor pi = at::empty({2 * n}, u.options()), qi = at::empty({2 * n}, u.options());
  at::Tensor pv = at::empty({2 * n, d}, P.options()), qv = at::empty({2 * n, d}, P.options());
  ok(acf_gather_bpr_fwd_bwd(P.data_ptr<float>(), Q.data_ptr<float>(), P.size(0), Q.size(0), (int32_t)d,
                            u.data_ptr<int32_t>(), i.data_ptr<int32_t>(), j.data_ptr<int32_t>(), n, (float)clip_lo,
                            (float)clip_hi, loss.data_ptr<float>(), x.data_ptr<float>(), pi.data_ptr<int32_t>(),
                            pv.data_ptr<float>(), qi.data_ptr<int32_t>(), qv.data_ptr<float>(), stream_of(P)),
     "acf_gather_bpr_fwd_bwd");
  return {loss, x, pi, pv, qi, qv};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> row_segment_sum(const at::Tensor& idx_, const at::Tensor& vals,
                                                               int64_t num_rows) {
  need(vals, "values", at::kFloat, 2);
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(vals.device());
  at::Tensor idx = idx32(idx_, "indices", vals);
  const int64_t m = idx.numel(), d = vals.size(1);
  TORCH_CHECK(vals.size(0) == m, "indices and values disagree: ", m, " vs ", vals.size(0), " rows");
  TORCH_CHECK(d >= 4 && d <= 1024 && d % 4 == 0, "values: dim must be a multiple of 4 in [4, 1024]");
  if (m > 0) {
    auto mm = idx.aminmax();
    TORCH_CHECK(std::get<0>(mm).item<int32_t>() >= 0 && std::get<1>(mm).item<int32_t>() < num_rows,
                "row_segment_sum: an index is outside [0, ", num_rows, ")");
  }
  size_t ws = 0;
  ok(acf_row_segment_sum_workspace(m, &ws), "acf_row_segment_sum_workspace");
  at::Tensor work = at::empty({(int64_t)ws}, vals.options().dtype(at::kByte));
  at::Tensor uniq = at::empty({m}, idx.options()), cnt = at::empty({m}, idx.options());
  at::Tensor sum = at::empty({m, d}, vals.options());
  at::Tensor k = at::empty({1}, idx.options().dtype(at::kLong));
  ok(acf_row_segment_sum(idx.data_ptr<int32_t>(), vals.data_ptr<float>(), m, (int32_t)d, num_rows,
                         work.data_ptr(), ws, uniq.data_ptr<int32_t>(), sum.data_ptr<float>(),
                         cnt.data_ptr<int32_t>(), k.data_ptr<int64_t>(), stream_of(vals)),
     "acf_row_segment_sum");
  const int64_t kk = k.item<int64_t>();  // the unique count sizes the outputs (one sync)
  return {uniq.narrow(0, 0, kk), sum.narrow(0, 0, kk), cnt.narrow(0, 0, kk)};
}

at::Tensor l2norm_perturb(const at::Tensor& g, double eps) {
  need(g, "g_rows", at::kFloat, 2);
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(g.device());
  at::Tensor out = at::empty_like(g);
  ok(acf_l2norm_perturb(g.data_ptr<float>(), g.size(0), (int32_t)g.size(1), (float)eps, out.data_ptr<float>(),
                        stream_of(g)),
     "acf_l2norm_perturb");
  return out;
}

void sparse_adagrad_apply(at::Tensor& W, at::Tensor& acc, const at::Tensor& idx_, const at::Tensor& g, double lr) {
  need_table(W, "W", W);
  need_table(acc, "accumulator", W);
  need(g, "g_rows", at::kFloat, 2);
  TORCH_CHECK(acc.sizes() == W.sizes(), "accumulator must match W");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(W.device());
  at::Tensor idx = idx32(idx_, "unique indices", W);
  TORCH_CHECK(g.size(0) == idx.numel() && g.size(1) == W.size(1), "g_rows must be [len(indices), dim]");
  check_range(idx, W.size(0), "unique indices");
  ok(acf_sparse_adagrad_apply(W.data_ptr<float>(), acc.data_ptr<float>(), W.size(0), (int32_t)W.size(1),
                              idx.data_ptr<int32_t>(), g.data_ptr<float>(), idx.numel(), (float)lr, stream_of(W)),
     "acf_sparse_adagrad_apply");
}

at::Tensor score_rank(const at::Tensor& P, const at::Tensor& Q, const at::Tensor& users_, const at::Tensor& tests_,
                      const at::Tensor& cand_off, const at::Tensor& cand_items_) {
  need_table(P, "embedding_P", P);
  need_table(Q, "embedding_Q", P);
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(P.device());
  at::Tensor users = idx32(users_, "users", P), tests = idx32(tests_, "test_items", P);
  at::Tensor cands = idx32(cand_items_, "cand_items", P);
  need(cand_off, "cand_off", at::kLong, 1);
  TORCH_CHECK(cand_off.numel() == users.numel() + 1 && tests.numel() == users.numel(),
              "cand_off must have len(users) + 1 entries and test_items len(users)");
  check_range(users, P.size(0), "users");
  check_range(tests, Q.size(0), "test_items");
  check_range(cands, Q.size(0), "cand_items");
  if (cands.numel() == 0) cands = at::zeros({1}, users.options());
  at::Tensor pos = at::empty({users.numel()}, users.options());
  ok(acf_eval_positions_list(P.data_ptr<float>(), Q.data_ptr<float>(), P.size(0), Q.size(0), (int32_t)P.size(1),
                             users.data_ptr<int32_t>(), tests.data_ptr<int32_t>(), (int32_t)users.numel(),
                             cand_off.data_ptr<int64_t>(), cands.data_ptr<int32_t>(), pos.data_ptr<int32_t>(),
                             stream_of(P)),
     "acf_eval_positions_list");
  return pos;
}

at::Tensor score_rank_all(const at::Tensor& P, const at::Tensor& Q, const at::Tensor& users_,
                          const at::Tensor& tests_, int64_t num_candidates, const at::Tensor& excl_off,
                          const at::Tensor& excl_items_) {
  need_table(P, "embedding_P", P);
  need_table(Q, "embedding_Q", P);
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(P.device());
  at::Tensor users = idx32(users_, "users", P), tests = idx32(tests_, "test_items", P);
  at::Tensor excl = idx32(excl_items_, "excl_items", P);
  need(excl_off, "excl_off", at::kLong, 1);
  TORCH_CHECK(excl_off.numel() == users.numel() + 1 && tests.numel() == users.numel(),
              "excl_off must have len(users) + 1 entries and test_items len(users)");
  TORCH_CHECK(num_candidates >= 0 && num_candidates <= Q.size(0), "num_candidates exceeds item rows");
  check_range(users, P.size(0), "users");
  check_range(tests, Q.size(0), "test_items");
  check_range(excl, Q.size(0), "excl_items");
  if (excl.numel() == 0) excl = at::zeros({1}, users.options());
  at::Tensor pos = at::empty({users.numel()}, users.options());
  ok(acf_eval_positions_all(P.data_ptr<float>(), Q.data_ptr<float>(), P.size(0), Q.size(0), (int32_t)P.size(1),
                            users.data_ptr<int32_t>(), tests.data_ptr<int32_t>(), (int32_t)users.numel(),
                            (int32_t)num_candidates, excl_off.data_ptr<int64_t>(), excl.data_ptr<int32_t>(),
                            pos.data_ptr<int32_t>(), stream_of(P)),
     "acf_eval_positions_all");
  return pos;
}

}  // namespace

#ifndef ACF_BUILD_HASH
#define ACF_BUILD_HASH "unhashed"
#endif
// "ACF_BUILD_HASH=<32 hex>" of this library's sources (build_native.source_hash)
extern "C" const char* acf_torch_build_hash(void) { return "ACF_BUILD_HASH=" ACF_BUILD_HASH; }

TORCH_LIBRARY(acf, m) {
  m.def("bpr_apr_step(Tensor(a!) P, Tensor(b!) Q, Tensor(c!) accP, Tensor(d!) accQ, Tensor u, Tensor i, "
        "Tensor j, float lr=0.05, float eps=0.5, float reg=0., float reg_adv=1., bool adver=True, "
        "float clip_lo=-80., float clip_hi=100000000.) -> (Tensor loss_clean, Tensor loss_adv, Tensor n_correct)");
  m.def("apr_train(Tensor(a!) P, Tensor(b!) Q, Tensor(c!) accP, Tensor(d!) accQ, Tensor u, Tensor i, Tensor j, "
        "int batch_size, float lr=0.05, float eps=0.5, float reg=0., float reg_adv=1., bool adver=True, "
        "float clip_lo=-80., float clip_hi=100000000.) -> (Tensor loss_clean, Tensor loss_adv)");
  m.def("gather_bpr_fwd_bwd(Tensor P, Tensor Q, Tensor u, Tensor i, Tensor j, float clip_lo=-80., "
        "float clip_hi=100000000.) -> (Tensor loss, Tensor x, Tensor p_idx, Tensor p_val, Tensor q_idx, "
        "Tensor q_val)");
  m.def("row_segment_sum(Tensor idx, Tensor vals, int num_rows) -> (Tensor uniq_idx, Tensor summed, Tensor count)");
  m.def("l2norm_perturb(Tensor g_rows, float eps) -> Tensor");
  m.def("sparse_adagrad_apply(Tensor(a!) W, Tensor(b!) acc, Tensor uniq_idx, Tensor g_rows, float lr) -> ()");
  m.def("score_rank(Tensor P, Tensor Q, Tensor users, Tensor test_items, Tensor cand_off, Tensor cand_items) "
        "-> Tensor");
  m.def("release_contexts() -> int", &release_contexts);
  m.def("score_rank_all(Tensor P, Tensor Q, Tensor users, Tensor test_items, int num_candidates, "
        "Tensor excl_off, Tensor excl_items) -> Tensor");
}

TORCH_LIBRARY_IMPL(acf, CUDA, m) {
  m.impl("bpr_apr_step", &bpr_apr_step);
  m.impl("apr_train", &train);
  m.impl("gather_bpr_fwd_bwd", &gather_bpr_fwd_bwd);
  m.impl("row_segment_sum", &row_segment_sum);
  m.impl("l2norm_perturb", &l2norm_perturb);
  m.impl("sparse_adagrad_apply", &sparse_adagrad_apply);
  m.impl("score_rank", &score_rank);
  m.impl("score_rank_all", &score_rank_all);
}
