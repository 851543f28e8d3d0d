/* acf_neumf.h — C-ABI of the MI355X NeuMF / adversarial-NeuMF training path
 * (libacf_neumf.so).  §8(f)3 of SURVEY.md, BASELINE.json configs[3].
 *
 * The reference model is the Keras `NeuMF` (NeuMF.py:10-52) trained by run.py
 * (`ranker.train(x_train, y_train, batch_size)`, MF.py:30-33 = Keras fit with
 * binary cross-entropy and Adam) on MF.py:42-56 `get_train_instances`, and scored
 * by `ranker.rank(users, items)` (MF.py:38-40) in evaluation.py:54-80.  The
 * reference's `AdversarialNeuMF` (NeuMF.py:58-185) does not run (NeuMF.py:131);
 * the adversarial step here is APR's FGSM applied to the four embedding tables
 * (oracle/neumf_oracle.py states it).
 *
 * Parameters live in ONE flat fp32 buffer in Keras order (offsets from
 * acf_neumf_param_offsets): MF_U [U1,d], MF_I [I1,d], MLP_U [U1,d], MLP_I [I1,d],
 * W1 [2d,2d], b1 [2d], W2 [2d,d], b2 [d], Wo [2d,1], bo [1] (+3 pad).  Gradient
 * and Adam moments use the same layout, so the dense Keras Adam is one stream.
 * All pointers are device pointers; `stream` is a hipStream_t.  Return 0 or an
 * ACF_E_* code (acf_apr.h); acf_neumf_last_error() holds the message.
 */
#ifndef ACF_NEUMF_H
#define ACF_NEUMF_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct acf_neumf_ctx acf_neumf_ctx;

typedef struct {
  float lr;       /* Adam learning rate (Keras default 0.001) */
  float beta1;    /* 0.9 */
  float beta2;    /* 0.999 */
  float adam_eps; /* 1e-7 (Keras 2.2 K.epsilon()) */
  float eps;      /* adversarial perturbation norm */
  float reg_adv;  /* weight of the adversarial loss */
  int32_t adver;  /* 0: NeuMF (NeuMF.py:10-52); 1: + FGSM adversarial loss */
  int32_t reserved;
} acf_neumf_hparams;

const char* acf_neumf_last_error(void);
/* "ACF_BUILD_HASH=<32 hex>" of this library's sources (see acf_apr_build_hash). */
const char* acf_neumf_build_hash(void);

/* Number of floats of the flat parameter buffer, and the 10 segment offsets. */
int64_t acf_neumf_param_count(int64_t num_user_rows, int64_t num_item_rows, int32_t dim);
int acf_neumf_param_offsets(int64_t num_user_rows, int64_t num_item_rows, int32_t dim,
                            int64_t* offsets10);

/* Workspace for batches of up to max_batch instances; dim % 4 == 0, dim <= 256. */
int acf_neumf_create(acf_neumf_ctx** ctx, int64_t num_user_rows, int64_t num_item_rows,
                     int32_t dim, int32_t max_batch);
int acf_neumf_destroy(acf_neumf_ctx* ctx);

/* Gradient of the batch's mean binary cross-entropy (Keras train_on_batch loss,
 * MF.py:30-33) w.r.t. every parameter, ADDED to `grad` (zero it before the first
 * call; acf_neumf_adam re-zeroes it).  adver = 1 adds reg_adv x the loss on the
 * embedding rows perturbed by eps * g/|g| (g: the clean gradient of the row).
 * loss_out (device, 2 floats, may be NULL): clean and adversarial mean loss.
 * check = 1: indices are validated (synchronises; ACF_E_RANGE when outside). */
int acf_neumf_grad(acf_neumf_ctx* ctx, const float* params, float* grad, const int32_t* user,
                   const int32_t* item, const float* label, int32_t batch,
                   const acf_neumf_hparams* hp, float* loss_out, int32_t check, void* stream);

/* Batches of at most 1,024 instances take the rows-in-line kernels (one launch
 * per pass); on = 0 sends them through the row-sum kernel instead, as larger
 * batches go (the same sums in the same order: bit-identical; for tests and
 * same-box A/B).  Default 1. */
int acf_neumf_set_rows_in_line(acf_neumf_ctx* ctx, int32_t on);

/* Failure safety of the rows-in-line kernels (no reference counterpart: Keras has
 * no cross-workgroup waits).  Their row owners wait, bounded, for the other
 * workgroups' contributions; a wait that gives up after `polls` polls (default
 * 2^22; 0 = give up at once, for tests) leaves the launch's results undefined.
 * With the failsafe on (default) acf_neumf_train and a checked acf_neumf_grad
 * snapshot the buffers they write first (train: params, grad, m, v; grad: grad)
 * and, on a give-up, restore them and replay the call on the row-sum kernels:
 * the same bits as a call that never gave up.  Failsafe off: ACF_E_HIP.  An
 * unchecked grad that gave up is reported (ACF_E_HIP) by the next grad with
 * check, train or predict on the context.  acf_neumf_recoveries: calls replayed. */
int acf_neumf_set_spin_limit(acf_neumf_ctx* ctx, int32_t polls);
int acf_neumf_set_failsafe(acf_neumf_ctx* ctx, int32_t on);
int acf_neumf_recoveries(acf_neumf_ctx* ctx, int64_t* count);

/* Keras 2.2 Adam over the whole buffer, iteration t (1-based); zeroes grad. */
int acf_neumf_adam(acf_neumf_ctx* ctx, float* params, float* grad, float* m, float* v,
                   int64_t t, const acf_neumf_hparams* hp, void* stream);

/* One Keras fit epoch over n already-shuffled instances (MF.py:30-33): batches
 * of `batch` (the last one partial), each acf_neumf_grad + acf_neumf_adam with
 * Adam iterations t_first, t_first+1, ...  losses (device, [ceil(n/batch)][2],
 * may be NULL): per-batch clean / adversarial mean loss.  Indices are validated
 * once at the end (ACF_E_RANGE; out-of-range rows were read as row 0).  The
 * result is bit-identical to that grad + adam sequence; inside the call each
 * embedding row's zero-gradient Adam iterations run late (when a batch gathers
 * the row, or in a rotating catch-up), and every row is current on return. */
int acf_neumf_train(acf_neumf_ctx* ctx, float* params, float* grad, float* m, float* v,
                    const int32_t* user, const int32_t* item, const float* label, int64_t n,
                    int32_t batch, int64_t t_first, const acf_neumf_hparams* hp, float* losses,
                    void* stream);

/* ranker.rank(users, items) (MF.py:38-40): sigmoid scores of n (user, item) pairs. */
int acf_neumf_predict(acf_neumf_ctx* ctx, const float* params, const int32_t* user,
                      const int32_t* item, int64_t n, float* scores, void* stream);

/* ---- Keras BPR (BPR.py:23-99): run.py --model bpr, BASELINE configs[0] ----
 * Parameters in one flat fp32 buffer [uEmb (num_user_rows x dim) | iEmb
 * (num_item_rows x dim)] (BPR.py:35-36); gradient and Adam moments share the
 * layout.  dim % 4 == 0, dim <= 256. */
typedef struct acf_kbpr_ctx acf_kbpr_ctx;
int acf_kbpr_create(acf_kbpr_ctx** ctx, int64_t num_user_rows, int64_t num_item_rows, int32_t dim,
                    int32_t max_batch);
int acf_kbpr_destroy(acf_kbpr_ctx* ctx);

/* One Keras fit epoch over n already-shuffled triplets (BPR.py:70-81): per
 * batch of `batch` (the last one partial) the gradient of
 * mean(1 - log(sigmoid(u.p - u.n))) (BPR.py:11-20), summed per table row in
 * occurrence order into grad, then Keras 2.2 Adam iteration t_first + k over the
 * whole buffer (grad re-zeroed; hp: lr, beta1, beta2, adam_eps).  losses
 * (device, [n]): each triplet's loss term.  Indices are validated at the end
 * (ACF_E_RANGE; out-of-range rows were read as row 0).  Synchronous. */
int acf_kbpr_train(acf_kbpr_ctx* ctx, float* params, float* grad, float* m, float* v, const int32_t* user,
                   const int32_t* item_pos, const int32_t* item_neg, int64_t n, int32_t batch, int64_t t_first,
                   const acf_neumf_hparams* hp, float* losses, void* stream);

/* ranker.rank(users, items) (BPR.py:67-68, predictor pDot): u . i of n pairs. */
int acf_kbpr_predict(acf_kbpr_ctx* ctx, const float* params, const int32_t* user, const int32_t* item,
                     int64_t n, float* out, void* stream);

/* ---- FastAdversarialMF (FastAdversarialMF.py:13-144): run.py --model amf2 ----
 * Parameters in one flat fp32 buffer [P (num_user_rows x dim) | Q (num_item_rows x
 * dim) | D_u | D_i] (acf_amf_param_count floats); a discriminator block (Dense(d,
 * relu) -> Dense(1, sigmoid), FastAdversarialMF.py:119-127) is [W1 (dim x dim,
 * Keras [in, out]) | b1 (dim) | W2 (dim) | b2 (1) | 3 pad].  Gradient and Adam
 * moments share the layout.  A batch holds B instances: (user, item, label) of
 * MF.py:42-56 and the adversarial indices (user_adv, item_adv) with the players'
 * popularity targets: t_user / t_item for the mf player, d_user / d_item for the
 * two discriminator players (FastAdversarialMF.py:89-117).  The three players'
 * gradients are taken at the same parameters (keras_adversarial's
 * AdversarialOptimizerSimultaneous): mf = MSE + BCE(D_u(P[ua]), t_user) +
 * BCE(D_i(Q[ia]), t_item) w.r.t. P, Q; each discriminator its BCE w.r.t. its own
 * weights.  dim % 4 == 0, dim <= 256.  Replaces the advModel.fit of
 * FastAdversarialMF.py:115 (parity with the reference unpinned: it does not run). */
typedef struct acf_amf_ctx acf_amf_ctx;
int64_t acf_amf_param_count(int64_t num_user_rows, int64_t num_item_rows, int32_t dim);
int acf_amf_create(acf_amf_ctx** ctx, int64_t num_user_rows, int64_t num_item_rows, int32_t dim,
                   int32_t max_batch);
int acf_amf_destroy(acf_amf_ctx* ctx);

/* The three players' gradient of one batch ADDED to grad; loss (device, [B][3]):
 * squared error, BCE(D_u, t_user), BCE(D_i, t_item) per instance.  Validates the
 * indices (synchronises; ACF_E_RANGE). */
int acf_amf_grad(acf_amf_ctx* ctx, const float* params, float* grad, const int32_t* user, const int32_t* item,
                 const float* label, const int32_t* user_adv, const int32_t* item_adv, const float* t_user,
                 const float* t_item, const float* d_user, const float* d_item, int32_t batch, float* loss,
                 void* stream);

/* One Keras fit epoch over n already-shuffled instances: batches of `batch` (the
 * last one partial), each acf_amf_grad + Keras 2.2 Adam iteration t_first + k over
 * the whole buffer (grad re-zeroed).  losses (device, [n][3]) as above.  Indices
 * are validated at the end (ACF_E_RANGE; out-of-range rows were read as row 0). */
int acf_amf_train(acf_amf_ctx* ctx, float* params, float* grad, float* m, float* v, const int32_t* user,
                  const int32_t* item, const float* label, const int32_t* user_adv, const int32_t* item_adv,
                  const float* t_user, const float* t_item, const float* d_user, const float* d_item, int64_t n,
                  int32_t batch, int64_t t_first, const acf_neumf_hparams* hp, float* losses, void* stream);

/* ranker.rank(users, items) (MF.py:38-40 on FastAdversarialMF.py:51's model): u . i. */
int acf_amf_predict(acf_amf_ctx* ctx, const float* params, const int32_t* user, const int32_t* item, int64_t n,
                    float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif
