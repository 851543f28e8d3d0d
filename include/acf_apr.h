/*
 * acf_apr.h — C-ABI of the MI355X-native adversarial BPR-MF (APR) hot path.
 *
 * The reference (feay1234/Adversarial-Collaborative-Filtering) has no FFI: its hot
 * path is a TensorFlow-1 graph driven from Python through `sess.run`.  Every entry
 * point below replaces one such `sess.run` call site (or the op group behind it);
 * the citation on each names the reference line it stands in for.  Python binds
 * these with ctypes (adversarial-collaborative-filtering_amd/_native.py); the
 * binding a maintainer would add to the reference is shown in INTEGRATION.md.
 *
 * Conventions
 *   - All array arguments are DEVICE pointers (HIP, gfx950) unless noted.
 *   - Tables are fp32, row-major, contiguous, [rows, dim]; indices are int32.
 *   - `stream` is a hipStream_t passed as void* (NULL = the legacy null stream).
 *   - Every call is asynchronous on `stream` unless documented otherwise.
 *   - Return value: ACF_OK (0) or an ACF_E_* code; acf_last_error() gives a
 *     thread-local message for the last failing call.
 *   - dim must be a multiple of 4 and <= 1024 (all configurations the reference
 *     runs use dim in {8,16,32,64,128}).
 */
#ifndef ACF_APR_H
#define ACF_APR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ACF_APR_ABI_VERSION 2

enum {
  ACF_OK = 0,
  ACF_E_INVALID = 1,     /* bad argument (shape, null pointer, unsupported dim) */
  ACF_E_RANGE = 2,       /* index out of range (TF Gather's InvalidArgument)     */
  ACF_E_HIP = 3,         /* HIP runtime error                                    */
  ACF_E_NOMEM = 4,       /* device allocation failed                             */
  ACF_E_STATE = 5        /* call out of order (e.g. step before plan)            */
};

/* Opaque per-model context: owns the device workspace, the batch plans and the
 * cached hipGraph executables.  One context per (process, device, model). */
typedef struct acf_apr_ctx acf_apr_ctx;

/* Trainable state of MF (APR.py:105-119) plus its Adagrad slots
 * (APR.py:193-195, TF initial_accumulator_value = 0.1). */
typedef struct acf_apr_tables {
  float* P;    /* embedding_P  [num_user_rows, dim] */
  float* Q;    /* embedding_Q  [num_item_rows, dim] */
  float* accP; /* Adagrad accumulator of P, same shape */
  float* accQ; /* Adagrad accumulator of Q, same shape */
} acf_apr_tables;

/* Hyper-parameters read by MF.__init__ (APR.py:86-97) and the graph constants. */
typedef struct acf_apr_hparams {
  float lr;        /* args.lr       (run_adv_ori.py:42, default 0.05)  */
  float eps;       /* args.eps      (run_adv_ori.py:54, default 0.5)   */
  float reg;       /* args.reg      (run_adv_ori.py:40, default 0)     */
  float reg_adv;   /* args.reg_adv  (run_adv_ori.py:44, default 1)     */
  float clip_lo;   /* clip_by_value lower bound, -80  (APR.py:148)     */
  float clip_hi;   /* clip_by_value upper bound, 1e8  (APR.py:148)     */
  int32_t adver;   /* 0: BPR graph, 1: APR graph (APR.py:156)          */
  int32_t adv_mode;/* 0: "grad" (APR.py:180-191); 1: "random" (APR.py:170-177) */
  uint64_t seed;   /* counter-based RNG seed for adv_mode = 1          */
  int32_t zero_delta; /* 1: adversarial terms use delta = 0 (the dns>1 branch of
                         utils.py:121-139 never runs update_P/update_Q)  */
  int32_t reserved;
} acf_apr_hparams;

/* ---- library ------------------------------------------------------------ */
int acf_apr_abi_version(void);
const char* acf_apr_last_error(void);
/* "ACF_BUILD_HASH=<32 hex>": hash of the sources, headers and flags the library
 * was built from (build_native.source_hash); the loaders refuse a mismatch. */
const char* acf_apr_build_hash(void);

/* ---- context ------------------------------------------------------------ */
/* Allocates the workspace for plans of up to max_batches_per_plan batches of up
 * to max_batch_size triplets.  Synchronous.  Replaces MF(...).build_graph()
 * (APR.py:197-202) as the point where per-model device state is created. */
int acf_apr_create(acf_apr_ctx** out, int64_t num_user_rows, int64_t num_item_rows,
                   int32_t dim, int32_t max_batch_size, int32_t max_batches_per_plan);
int acf_apr_destroy(acf_apr_ctx* ctx);

/* ---- batch planning: TF's sparse-gradient de-duplication ------------------
 * Stages n_batches consecutive mini-batches (batch b = triplets
 * [b*batch_size, (b+1)*batch_size)) and builds, per batch, the unique user and
 * item rows with the ordered list of their occurrences — the structure TF builds
 * with Unique + UnsortedSegmentSum in Optimizer._apply_sparse_duplicate_indices
 * (behind APR.py:195) and that IndexedSlices->dense conversion sums
 * (APR.py:183-187).  If `check` != 0 the call synchronises the stream and
 * returns ACF_E_RANGE when any index is outside its table (TF CPU Gather raises
 * InvalidArgument there); with check == 0 bad indices are clamped to row 0. */
int acf_apr_plan(acf_apr_ctx* ctx, const int32_t* user, const int32_t* item_pos,
                 const int32_t* item_neg, int32_t batch_size, int32_t n_batches,
                 int32_t check, void* stream);

/* sess.run([model.update_P, model.update_Q], feed_dict)  (utils.py:117-118,
 * APR.py:167-191): delta rows for every row touched by planned batch `batch`.
 * Rows not touched have delta = 0 in the reference and are never read, so only
 * touched rows are materialised (in the context). */
int acf_apr_delta_update(acf_apr_ctx* ctx, const acf_apr_tables* tables,
                         const acf_apr_hparams* hp, int32_t batch, void* stream);

/* sess.run(model.optimizer, feed_dict)  (utils.py:119, APR.py:143-165,193-195):
 * clean + (if hp->adver) adversarial forward/backward, per-row gradient
 * aggregation, sparse Adagrad on the unique rows — in place on `tables`.
 * With hp->adver the delta of the last acf_apr_delta_update on the same batch
 * is used. */
int acf_apr_optimizer_step(acf_apr_ctx* ctx, const acf_apr_tables* tables,
                           const acf_apr_hparams* hp, int32_t batch, void* stream);

/* The hot loop of training_batch (utils.py:106-119, dns == 1): for planned
 * batches [first_batch, first_batch + n_batches): delta_update (if adver) then
 * optimizer_step.  graph_mode 1 replays a cached hipGraph of the whole loop
 * (captured on first use for this (tables, hparams, range)); 0 launches
 * eagerly. */
int acf_apr_train_planned(acf_apr_ctx* ctx, const acf_apr_tables* tables,
                          const acf_apr_hparams* hp, int32_t first_batch,
                          int32_t n_batches, int32_t graph_mode, void* stream);

/* training_batch over a triplet range in ONE call (utils.py:106-119 for
 * n_batches consecutive batches): acf_apr_plan(user, item_pos, item_neg,
 * batch_size, n_batches, check) followed by acf_apr_train_planned over all the
 * planned batches.  The triplet arrays are device pointers that must stay valid
 * until the stream has run the call. */
int acf_apr_train(acf_apr_ctx* ctx, const acf_apr_tables* tables, const acf_apr_hparams* hp,
                  const int32_t* user, const int32_t* item_pos, const int32_t* item_neg,
                  int32_t batch_size, int32_t n_batches, int32_t check, int32_t graph_mode,
                  void* stream);

/* Kernel timing for roofline accounting: runs planned batches
 * [first_batch, first_batch + n_batches) exactly like acf_apr_train_planned
 * (eager, same stream, same kernels, tables updated) but brackets every kernel
 * with hipExtLaunchKernelGGL start/stop events.  Writes, per kernel kind
 * k = 0 (clean pass, or the fused BPR step), 1 (adversarial pass + Adagrad),
 * 2 (write-back: k_flush / k_stream_flush), 3 (unused since r05: the
 * overlapped step k_ovl is gone), 4 (streamed step k_stream), 5 (hot-slot combine of large-batch plans), the
 * summed kernel time in ms to ms_out[k] and the launch count to
 * launches_out[k] (arrays of 6).  Synchronous.  Not part of the reference
 * surface. */
int acf_apr_time_kernels(acf_apr_ctx* ctx, const acf_apr_tables* tables,
                         const acf_apr_hparams* hp, int32_t first_batch,
                         int32_t n_batches, double* ms_out, int32_t* launches_out,
                         void* stream);

/* How step kernels map unique rows ("slots") to lanes: 0 = auto (default: one
 * wavefront per slot below 4,096 triplets per batch, where hot rows have many
 * occurrences; one lane-group of dim/4 lanes per slot at and above it, where
 * almost every row occurs once), 1 = one wavefront per slot, 2 = one lane-group
 * per slot.  Results are deterministic for a given mapping and agree across
 * mappings to fp32 summation order.  Not part of the reference surface. */
int acf_apr_set_slot_mapping(acf_apr_ctx* ctx, int32_t mode);

/* Triplet fusion in acf_apr_train_planned / acf_apr_time_kernels (1 = on, the
 * default; 0 = off).  A triplet whose user, positive and negative item each
 * occur once in its batch is stepped start to finish by one lane-group (no
 * batch-wide aggregation is needed for it); the arithmetic per row is the slot
 * kernels' own, so on and off give identical bits.  For one-lane-group-per-slot
 * plans (batches >= 4,096) the setting at acf_apr_plan time decides the plan: on
 * gives a triplet-centric plan whose steps (train_planned and the split per-batch
 * calls alike) update every row in its table; training such a plan with fusion
 * switched off returns ACF_E_STATE (plan again).  Otherwise the split per-batch
 * calls (delta_update / optimizer_step) never fuse.  Not part of the reference
 * surface. */
int acf_apr_set_fusion(acf_apr_ctx* ctx, int32_t on);

/* Which planner acf_apr_plan uses: 0 = auto (the default: the batch-local plan,
 * one workgroup per batch in two launches, for one-wavefront-per-slot plans of
 * batches up to 1,024 triplets on tables whose batch bitmaps fit 64 MB; the hash
 * plan for triplet-centric plans -- one lane-group per slot, fusion on, not
 * shard mode, batches up to 65,536; the device-wide sort plan otherwise), 1 = always the
 * device-wide sort plan.  Every planner gives the step identical bits (the hash
 * plan numbers slots and CSR ranges in another order, and keeps the occurrence
 * order inside each range).  Not part of the reference surface (A/B and the
 * planner-equivalence tests). */
int acf_apr_set_plan_mode(acf_apr_ctx* ctx, int32_t mode);

/* The planner the last acf_apr_plan used: 0 device-wide sort plan, 1 batch-local
 * plan, 2 one-workgroup shard plan, 3 hash plan; -1 before any plan.  Not part
 * of the reference surface (tests and bench). */
int acf_apr_plan_kind(const acf_apr_ctx* ctx);

/* Streamed APR steps in acf_apr_train_planned (1 = on, the default; 0 = off;
 * the setting is per context).  For plans with one wavefront
 * per slot and dim <= 256, ONE launch runs the whole batch range: every row a
 * batch updates becomes a tagged version that later batches read (bounded spin
 * until it exists), and one write-back kernel moves the last versions to the
 * tables.  Arithmetic and order of every sum are unchanged, so on and off give
 * identical bits.  Uses 3 x max_batches x 3 x max_batch_size x dim x 8 bytes of
 * device memory, allocated at first use (off when that fails, or when the
 * device cannot keep the launch resident).  Not part of the reference surface. */
int acf_apr_set_stream(acf_apr_ctx* ctx, int32_t on);

/* Failure safety of the streamed step (k_stream).  k_stream needs every one of
 * its waves resident; when a hand-off wait gives up (another process or a
 * concurrent persistent kernel on the device), its flush writes nothing, so the
 * tables are as before the call.  failsafe = 1 (default): every streamed call
 * stays asynchronous and is queued for verification; its launch reports its
 * outcome to host-mapped memory.  A failed call sets the group's gate, so every
 * later streamed call of the group applies nothing either; the queue is settled
 * by acf_apr_resolve and, implicitly, by every entry point that needs settled
 * tables (the setters, acf_apr_step_errors, acf_apr_stream_recoveries,
 * acf_apr_copy_losses, the two-phase and shard calls, a non-streamed
 * train_planned) or that re-plans a context with a queued call (acf_apr_plan):
 * the failed call and every later queued one are replayed, in order, on the
 * two-kernel schedule (exact: same result as acf_apr_set_stream 0).
 * failsafe = 0 (and timed or graph-captured calls): a give-up is reported by
 * acf_apr_step_errors (bit 0, sticky until read) and that call's rows are not
 * applied; later calls are applied normally.  Such an unverified call settles
 * the group's queue before it launches (except inside a capture), so it never
 * runs behind the gate of an earlier failed verified call.
 * acf_apr_set_spin_limit: version polls before a give-up (default 65,536; 0
 * gives up at the first unready poll -- tests force the replay with it).
 * acf_apr_stream_recoveries: streamed calls replayed so far. */
int acf_apr_set_failsafe(acf_apr_ctx* ctx, int32_t on);
int acf_apr_set_spin_limit(acf_apr_ctx* ctx, int32_t polls);
int acf_apr_stream_recoveries(acf_apr_ctx* ctx, int64_t* out);
/* Settle every queued verified streamed call of the context's group (blocks
 * until they have all reported; replays failed ones, see above). */
int acf_apr_resolve(acf_apr_ctx* ctx);
/* acf_apr_resolve for every group of the process with a queued call: what a
 * reader of the tables outside the group calls first (evaluation, forward,
 * checkpoints; the Python layer does so in ops.settle_tables). */
int acf_apr_resolve_all(void);
/* ctx joins peer's verification group: contexts that train the same tables on
 * one stream (a PlanPipeline's contexts) must share one, so that a failed call
 * of either gates the later calls of both.  Settles both groups first. */
int acf_apr_share_failsafe(acf_apr_ctx* ctx, acf_apr_ctx* peer);

/* ---- shard mode: users and items row-sharded over the ranks of one node ----
 * SURVEY §8(e) (no reference counterpart: the reference trains on one CPU
 * process; this splits one training_batch, utils.py:113-119, across ranks so
 * the result is the single-process one up to fp32 summation order).  Row r of
 * P lives on rank r % G, row r of Q on rank r % G; each rank plans the
 * triplets of ITS users for one global batch on (its user shard, the item rows
 * it fetched, in working-set order), and the batch-global item sums of
 * APR.py:183-195 are completed by the item owners between the passes. */

/* Shard mode on/off for the context (forces one lane-group per slot, no triplet
 * fusion; a one-batch plan per step).  reg_batch: the global batch size the
 * reg * mean(w^2) terms divide by (0 = the planned batch size). */
int acf_apr_set_shard_mode(acf_apr_ctx* ctx, int32_t on, int32_t reg_batch);

/* (r06) Which batch of the plan the next shard pass / item map calls step: a
 * triplet-centric shard plan (batches over 1,024 triplets) may hold a chunk of
 * steps planned at once (distributed.ShardedAPR); slot-kernel shard plans are
 * one batch (0).  Reset to 0 by acf_apr_set_shard_mode. */
int acf_apr_set_shard_batch(acf_apr_ctx* ctx, int32_t batch);

/* pass 0: clean sums (users complete: delta; items: partial sums in the item
 * slots' rows; BPR also updates the users); pass 1 (APR): adversarial sums
 * (users: Adagrad + write-back to the user shard; items: partial sums).  The
 * item rows of `tables` are the fetched working set (never written). */
int acf_apr_shard_pass(acf_apr_ctx* ctx, const acf_apr_tables* tables, const acf_apr_hparams* hp,
                       int32_t pass, void* stream);

/* The item slots of the current one-batch plan, in working-set order:
 * dir 0 copies their partial sums to buf [n_items, dim]; dir 1 copies buf into
 * their delta rows (the owners' deltas, before pass 1). */
int acf_apr_shard_items(acf_apr_ctx* ctx, int32_t dir, float* buf, int64_t n_items, void* stream);

/* acf_apr_shard_pass, and the item slots' partial sums of the pass also written to
 * row map[w] of buf for working-set entry w < n_items (what acf_apr_shard_items_mapped
 * dir 0 does after the pass), by the pass's own combine launch (export workgroups):
 * the split step hands its exchange rows to the pass and needs no copy launch. */
int acf_apr_shard_pass_export(acf_apr_ctx* ctx, const acf_apr_tables* tables, const acf_apr_hparams* hp,
                              int32_t pass, float* buf, const int64_t* map, int64_t n_items, void* stream);

/* As acf_apr_shard_items, with working-set entry w at row map[w] of buf (int64
 * row indices): the split step moves the item partial sums and deltas straight
 * between the slots and its fixed-layout exchange rows (distributed.py "Static
 * step layout"), with no gather or scatter pass of its own. */
int acf_apr_shard_items_mapped(acf_apr_ctx* ctx, int32_t dir, float* buf, const int64_t* map, int64_t n_items,
                               void* stream);

/* Owner side, per owned row s of the step: the partial rows recv[pos[p]] for p
 * in [seg[s], seg[s+1]) (requester order) are summed in that order.
 * reduce_delta (APR.py:183-191): G0[s] = the sum; reply[pos[p]] = eps *
 * l2_normalize(sum) for every p of the row (hp->zero_delta: 0).
 * reduce_apply (APR.py:193-195): G = G0[s] + reg_adv * sum (APR; BPR: the sum),
 * then Adagrad on Q[rows[s]] / accQ[rows[s]]; count[s] = the row's occurrences
 * in the global batch (needed only when hp->reg != 0, with reg_batch). */
int acf_shard_reduce_delta(const float* recv, const int32_t* seg, const int32_t* pos, int32_t n_rows,
                           int32_t dim, const acf_apr_hparams* hp, float* G0, float* reply, void* stream);
int acf_shard_reduce_apply(float* Q, float* accQ, const float* recv, const int32_t* seg, const int32_t* pos,
                           int32_t n_rows, int32_t dim, const acf_apr_hparams* hp, const float* G0,
                           const int32_t* rows, const int32_t* count, int32_t reg_batch, void* stream);

/* Reads into *out and clears the step error word: bit 0 = an overlapped step
 * gave up waiting for a row (results of that call are not trustworthy).
 * Synchronous on `stream`.  Not part of the reference surface. */
int acf_apr_step_errors(acf_apr_ctx* ctx, int32_t* out, void* stream);

/* Per-triplet clean / adversarial losses computed by the last step of each
 * planned batch (softplus(-clip(x)) terms of APR.py:150,162), for the staged
 * triplets [0, n_batches*batch_size).  Either pointer may be NULL. */
int acf_apr_copy_losses(acf_apr_ctx* ctx, float* loss_clean, float* loss_adv,
                        void* stream);

/* Writes the delta rows of the last acf_apr_delta_update into dense tables
 * delta_P [num_user_rows, dim] / delta_Q [num_item_rows, dim]; untouched rows
 * are left as the caller initialised them (zero in the reference). */
int acf_apr_delta_scatter(acf_apr_ctx* ctx, float* delta_P, float* delta_Q,
                          void* stream);

/* ---- forward only: training_loss_acc (utils.py:159-175) ------------------
 * Per batch b of n_batches: batch_loss[b] = sum softplus(-clip(x+ - x-)) and
 * batch_correct[b] = #(x+ - x- > 0); optional per-triplet scores out_pos /
 * out_neg (model.output / model.output_neg).  Any output may be NULL. */
int acf_bpr_forward(const float* P, const float* Q, int64_t num_user_rows,
                    int64_t num_item_rows, int32_t dim, const int32_t* user,
                    const int32_t* item_pos, const int32_t* item_neg,
                    int32_t batch_size, int32_t n_batches, float clip_lo,
                    float clip_hi, float* batch_loss, int32_t* batch_correct,
                    float* out_pos, float* out_neg, void* stream);

/* ---- evaluation: _eval_by_user (utils.py:244-254) ------------------------
 * position[u] = #{candidate c : score(u,c) >= score(u,test_item[u])} with
 * score = P[u] . Q[c].
 * _all:  candidates = [0, num_candidates) minus the sorted, unique exclusion
 *        list excl_items[excl_off[k] .. excl_off[k+1]) of user k (the caller
 *        passes trainList[u] union {test item}, restricted to the range:
 *        utils.py:211-215).
 * _list: candidates = cand_items[cand_off[k] .. cand_off[k+1]) verbatim, with
 *        repeats ("sample" mode, utils.py:201-209). */
int acf_eval_positions_all(const float* P, const float* Q, int64_t num_user_rows,
                           int64_t num_item_rows, int32_t dim, const int32_t* users,
                           const int32_t* test_items, int32_t n_users,
                           int32_t num_candidates, const int64_t* excl_off,
                           const int32_t* excl_items, int32_t* positions,
                           void* stream);
int acf_eval_positions_list(const float* P, const float* Q, int64_t num_user_rows,
                            int64_t num_item_rows, int32_t dim, const int32_t* users,
                            const int32_t* test_items, int32_t n_users,
                            const int64_t* cand_off, const int32_t* cand_items,
                            int32_t* positions, void* stream);

/* acf_eval_positions_all with the sweep chosen per call: kernel 0 = auto (what
 * acf_eval_positions_all runs), 1 = the MFMA sweep (one kernel:
 * v_mfma_f32_16x16x4_f32 tiles, exact rescoring of candidates within the f32
 * error band of the test score, exclusions as a per-tile bitmap), 2 = the VALU
 * sweep.  Positions are identical for every kernel; no process-wide state. */
int acf_eval_positions_all_kernel(const float* P, const float* Q, int64_t num_user_rows,
                                  int64_t num_item_rows, int32_t dim, const int32_t* users,
                                  const int32_t* test_items, int32_t n_users,
                                  int32_t num_candidates, const int64_t* excl_off,
                                  const int32_t* excl_items, int32_t* positions, int32_t kernel,
                                  void* stream);

/* ---- sampler: shuffle/_get_train_batch (APR.py:39-81) --------------------
 * Shuffles the n_pos positive pairs with a counter-based permutation of
 * `seed`, keeps floor(n_pos / batch_size) * batch_size of them (drop-last,
 * APR.py:52), and draws one negative per triplet uniformly from
 * [0, num_items), redrawn while it is in the user's list
 * list_items[list_off[u] .. list_off[u+1]) (sorted ascending; the
 * OriginalDataset.trainList of APR.py:77).  Writes out_user/out_pos/out_neg of
 * length n_out = floor(n_pos/batch_size)*batch_size.  Users with a full list
 * (no admissible negative) get -1 after max_tries draws; with check != 0 the
 * call synchronises and returns ACF_E_RANGE in that case. */
int acf_sample_epoch(const int32_t* pos_user, const int32_t* pos_item, int64_t n_pos,
                     int32_t batch_size, int32_t num_items, int32_t num_lists,
                     const int64_t* list_off, const int32_t* list_items,
                     uint64_t seed, int32_t max_tries, int32_t check,
                     int32_t* out_user, int32_t* out_pos, int32_t* out_neg,
                     void* stream);

/* acf_sample_epoch with the negatives proposed from an alias table instead of
 * uniformly (SURVEY §8(f)1, config 5's on-GPU alias sampler): column k of the
 * table (prob, alias: DEVICE arrays of num_items) keeps k with probability
 * prob[k], else yields alias[k]; the proposal is then accepted or redrawn by
 * the same trainList rule (APR.py:76-78).  A table of equal weights is the
 * reference's uniform sampler. */
int acf_sample_epoch_alias(const int32_t* pos_user, const int32_t* pos_item, int64_t n_pos,
                           int32_t batch_size, int32_t num_items, int32_t num_lists,
                           const int64_t* list_off, const int32_t* list_items,
                           const float* prob, const int32_t* alias, uint64_t seed,
                           int32_t max_tries, int32_t check, int32_t* out_user,
                           int32_t* out_pos, int32_t* out_neg, void* stream);

/* Builds an alias table (Vose) for sampling k with probability w[k] / sum(w).
 * HOST arrays: w [n] (>= 0, finite, not all 0) in; prob [n], alias [n] out.
 * Synchronous, deterministic. */
int acf_alias_build(const float* w, int64_t n, float* prob, int32_t* alias);

/* dns > 1 negative selection (utils.py:121-133): per triplet, the candidate of
 * cand[e*dns .. e*dns+dns) with the largest clean score P[user[e]].Q[c] (first
 * maximum wins, np.argmax). */
int acf_dns_select(const float* P, const float* Q, int64_t num_user_rows,
                   int64_t num_item_rows, int32_t dim, const int32_t* user,
                   const int32_t* cand, int64_t n, int32_t dns, int32_t* out_neg,
                   void* stream);

/* ---- the step decomposed into TF's ops (csrc/acf_ops.hip) ----------------
 * The fused step above is the training path; these expose its pieces one
 * kernel each, with TF's data flow, for callers that compose the step (the
 * PyTorch custom ops acf::gather_bpr_fwd_bwd, row_segment_sum, l2norm_perturb,
 * sparse_adagrad_apply) and for op-level tests.  All asynchronous on `stream`. */

/* The inference gathers + BPR loss of APR.py:121-150 and the gradient of the
 * loss w.r.t. the gathered rows, as TF's IndexedSlices (APR.py:183): for each of
 * n triplets, loss[b] = softplus(-clip(x_b)), x[b] = p.q_i - p.q_j, and
 *   P slices: p_idx = [u ; u],  p_val = [g*q_i ; -g*q_j]   ([2n], [2n, dim])
 *   Q slices: q_idx = [i ; j],  q_val = [g*p ; -g*p]
 * with g = d loss / d x (zero outside the clip range): pos-branch lookups
 * first, then neg-branch, each product rounded as TF's Mul. */
int acf_gather_bpr_fwd_bwd(const float* P, const float* Q, int64_t num_user_rows,
                           int64_t num_item_rows, int32_t dim, const int32_t* user,
                           const int32_t* item_pos, const int32_t* item_neg, int64_t n,
                           float clip_lo, float clip_hi, float* loss, float* x,
                           int32_t* p_idx, float* p_val, int32_t* q_idx, float* q_val,
                           void* stream);

/* IndexedSlices -> unique rows (unsorted_segment_sum behind APR.py:183-187 and
 * the optimizer's dedup, APR.py:195): the m (index, value-row) pairs become
 * *out_k <= m unique indices in ascending order (out_uniq), each with the
 * sequential sum of its value rows in input order (out_sum [m, dim], first
 * *out_k rows used) and their count.  Indices must lie in [0, num_rows).
 * out_k is a DEVICE int64.  workspace: acf_row_segment_sum_workspace(m). */
int acf_row_segment_sum_workspace(int64_t m, size_t* bytes);
int acf_row_segment_sum(const int32_t* idx, const float* vals, int64_t m, int32_t dim,
                        int64_t num_rows, void* workspace, size_t workspace_bytes,
                        int32_t* out_uniq, float* out_sum, int32_t* out_count,
                        int64_t* out_k, void* stream);

/* delta = eps * l2_normalize(g, 1) = eps * g * rsqrt(max(sum g^2, 1e-12)) for k
 * rows (APR.py:186-191). */
int acf_l2norm_perturb(const float* g, int64_t k, int32_t dim, float eps, float* out,
                       void* stream);

/* TF SparseApplyAdagrad on k UNIQUE rows idx of W / acc ([rows, dim]) with
 * gradient rows g [k, dim]: acc += g^2; W -= lr * g * rsqrt(acc) (APR.py:195). */
int acf_sparse_adagrad_apply(float* W, float* acc, int64_t rows, int32_t dim,
                             const int32_t* idx, const float* g, int64_t k, float lr,
                             void* stream);

#ifdef __cplusplus
}
#endif

#endif /* ACF_APR_H */
