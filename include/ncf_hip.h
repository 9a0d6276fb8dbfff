/*
 * ncf_hip.h -- C ABI of libncf_hip.so, the MI355X (gfx950) NeuMF training hot path.
 *
 * Plain C: raw device pointers, sizes, and a `void *stream` (a hipStream_t, e.g.
 * torch.cuda.current_stream().cuda_stream).  No torch or HIP types in any
 * signature.  Every entry point is asynchronous on `stream`, allocates nothing
 * (workspaces are passed in) and is therefore capturable into a hipGraph.
 * Return value: NCF_OK (0) or a negative NCF_E* code; the Python host layer
 * (ncf_amd/_lib.py) turns a non-zero code into RuntimeError.
 *
 * The reference (YonkaMayonkaZ/NCF) has no FFI: its hot path is a set of ATen ops
 * reached from Python.  Each entry point below replaces the reference code cited
 * next to it (paths relative to the reference root).
 */
#ifndef NCF_HIP_H
#define NCF_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 19: NCF_LAYOUT_FACT_IN_ADAM (0x20) removed -- measured slower than the two launches it
 * replaced; the bit is retired (NCF_LAYOUT_RETIRED_0X20: rejected by
 * ncf_reduce_adam_step).
 * 18: in-step Adam for small batches: ncf_ais_bufs, ncf_ais_supported, ncf_ais_begin,
 * ncf_train_step_ais, ncf_ais_bump, ncf_ais_flush.
 * 17: the owner-sharded sparse exchange (dp_mode "owner"): ncf_owner_plan,
 * ncf_owner_plan_init, ncf_owner_lists, ncf_owner_pack, ncf_owner_adam, ncf_owner_unpack;
 * NCF_LAYOUT_FACT_IN_ADAM (the factored expansion inside ncf_reduce_adam_step).
 * 16: NCF_LAYOUT_USER_STORE (ncf_layout_tune; ncf_uses_user_order covers it),
 * ncf_debug_set_user_store; ncf_adam_step_fact: one launch, clears the local bucket
 * (grads_local, grads_n arguments), gshard may be written.
 * 15: ncf_layout.flags gains the fused step's workgroup geometry (NCF_LAYOUT_GEO_*) and
 * NCF_LAYOUT_FACT_DEFER_DX; new ncf_adam_step_fact, ncf_prepare_epoch2
 * (NCF_PREP_CANONICAL), ncf_probe_gather_scatter, ncf_debug_set_geometry. */
#define NCF_ABI_VERSION 19

#define NCF_OK 0
#define NCF_E_UNSUPPORTED (-1) /* (model_type, factor_num, num_layers) has no compiled kernel */
#define NCF_E_ARG (-2)         /* bad pointer / size */
#define NCF_E_LAUNCH (-3)      /* hipGetLastError() after launch */

/*
 * Packed interaction row: one uint64 per (user, item, label) sample of the
 * training stream (datasets.py:57-60 features_fill / labels_fill):
 *   bits  0..31  user id (int32; -1 marks a padding row, which is skipped)
 *   bits 32..62  item id
 *   bit  63      label (1 = positive; the reference labels are 1.0 / 0.0)
 * 8 bytes per row instead of three 4-byte streams: one load per row in the fused
 * step and one random gather per row in the epoch shuffle.
 */
#define NCF_ROW_PACK(u, i, y) \
    ((uint64_t)(uint32_t)(u) | ((uint64_t)((uint32_t)(i) & 0x7fffffffu) << 32) | ((uint64_t)((y) != 0) << 63))

/* model_type: src/ncf/models.py:30-33,98-107 */
#define NCF_MODEL_GMF 0
#define NCF_MODEL_MLP 1
#define NCF_MODEL_NEUMF 2 /* "NeuMF-end" and "NeuMF-pre" share the forward */

/* dz_mode of ncf_train_step */
#define NCF_DZ_BCE 0    /* fused nn.BCEWithLogitsLoss() (mean) from labels (train_neumf.py:86,113) */
#define NCF_DZ_DLOGIT 1 /* upstream dL/dlogit given per row (autograd backward of NCF.forward) */
#define NCF_DZ_KD 2     /* distillation: w_task * BCE + w_resp * response term (ncf_train_step_kd) */

/* Flat parameter buffer layout, offsets in floats.  Order and shapes follow the
 * reference state_dict (models.py:11-34): embed_user_GMF [U,f], embed_item_GMF [I,f],
 * embed_user_MLP [U,dm], embed_item_MLP [I,dm], MLP_layers.{3k+1}.weight [s_{k+1}, s_k]
 * and .bias, predict_layer.weight [1,P], .bias [1]; every segment starts 64-float aligned.
 * [tower_begin, tower_begin + tower_len) covers tower + predict parameters (the part
 * whose gradient is produced through per-workgroup partial slabs); the float at
 * tower_begin + tower_len is the loss slot (sum of per-row BCE / global batch). */
typedef struct ncf_layout {
    int64_t ug, ig, um, im;
    int64_t w[4], b[4];
    int64_t wp, bp;
    int64_t tower_begin, tower_len;
    int64_t total; /* floats in the flat buffer, loss slot included */
    int32_t user_num, item_num, factor_num, num_layers, model_type;
    int32_t flags; /* 0 from ncf_layout_init; ncf_layout_tune sets the launch shape */
    float dropout;         /* training steps: nn.Dropout(p) before every tower Linear (0: none) */
    uint32_t dropout_seed; /* keep mask of (seed, adam_t, layer, epoch-stream row, column):
                              ncf_dropout_keep; since ABI 11 */
} ncf_layout;

/* ncf_layout.flags (set by ncf_layout_tune; every entry point reads them from the
 * layout it is given, so one tuned layout must be used for a whole step) */
#define NCF_LAYOUT_PER_ROW_L0 0x1   /* per-row layer-0 gradients even where the factored path applies */
#define NCF_LAYOUT_LAYERED 0x2      /* training steps on the layered path even where a fused kernel exists */
#define NCF_LAYOUT_WG_SHIFT 8       /* bits 8..19: workgroups of the fused step (0 = ncf_slab_rows()) */
#define NCF_LAYOUT_WG_MASK 0xfff
#define NCF_LAYOUT_GEO_SHIFT 20     /* bits 20..21: workgroup geometry of the fused step -- 0: 8 waves on */
#define NCF_LAYOUT_GEO_MASK 0x3     /* 128-row tiles; 1, 2, 3: 4, 2, 1 waves on 64, 32, 16-row tiles */
#define NCF_LAYOUT_FACT_DEFER_DX 0x8 /* factored layer 0: the step forms only the dW0 partials and leaves the
                                        per-entity sums G in grads' Um / Im rows (ncf_adam_step_fact expands them
                                        per shard after the reduce-scatter); set by the caller, kept by tune */
#define NCF_LAYOUT_RETIRED_0X20 0x20 /* was NCF_LAYOUT_FACT_IN_ADAM (ABI 17-18); rejected since ABI 19 */
#define NCF_LAYOUT_USER_STORE 0x10  /* fused step (set by ncf_layout_tune when ncf_debug_set_user_store
                                       enables it; since ABI 16): the user-side embedding gradients of each
                                       row are stored plainly into the workspace and summed per user by a
                                       second launch over ncf_user_order's runs instead of float atomics
                                       (needs the user_order argument of ncf_train_step, else the atomics
                                       stay) */

/* Device-resident step control block (16-byte aligned, 6 x int64).  Lets a
 * captured hipGraph replay consecutive batches with no host involvement. */
typedef struct ncf_step_ctl {
    int64_t batch;      /* global batch index inside the epoch stream             */
    int64_t adam_t;     /* optimizer steps completed (torch Adam state['step'])   */
    int64_t n_total;    /* rows in the epoch stream (positives + negatives)       */
    int64_t reserved;   /* keep 0                                                */
    int64_t snap_batch; /* written by ncf_train_step: the batch this step trains  */
    int64_t snap_t;     /* written by ncf_train_step: adam_t + 1 (this step's t)  */
} ncf_step_ctl;

int ncf_abi_version(void);

/* Which path runs this shape: NCF_PATH_FUSED (one fused launch per step, tower
 * weights in LDS), NCF_PATH_LAYERED (per-layer MFMA GEMM kernels with activations in
 * the workspace: any factor_num, tower weights of any size), 0 = invalid shape. */
#define NCF_PATH_FUSED 1
#define NCF_PATH_LAYERED 2
int ncf_supported(int model_type, int factor_num, int num_layers);

/* Bytes of the `workspace` that ncf_train_step needs for up to `rows` rows per launch
 * (rows = ceil(batch_global / world)): the fused path's partial slab
 * [ncf_slab_rows()][ncf_slab_stride()], or the layered path's slab row + activations. */
int64_t ncf_workspace_bytes(const ncf_layout *lay, int64_t rows);

/* Bytes of the workspace ncf_forward needs for n rows (0 on the fused path). */
int64_t ncf_forward_workspace_bytes(const ncf_layout *lay, int64_t n);

/* Host-only: fill *out for NCF(user_num, item_num, factor_num, num_layers, model_type). */
int ncf_layout_init(int user_num, int item_num, int factor_num, int num_layers, int model_type,
                    ncf_layout *out);

/* Workgroups the fused step launches at most (rows of its partial slab). */
int ncf_slab_rows(void);

/*
 * Host-only: shape the fused step for launches of up to `rows_per_launch` rows
 * (ceil(batch_global / world)) by setting lay->flags:
 *   - workgroups = min(ncf_slab_rows(), ceil(rows / 128)) -- a 1,024-row batch
 *     (config C2) runs 8 workgroups and the reductions read 8 slab rows, not 256;
 *   - per-row layer-0 gradients when rows < (user_num + item_num) / 2: the factored
 *     path's expansion costs per table row, the per-row form per batch row.
 * Call before sizing the workspace (ncf_workspace_bytes depends on the flags).
 */
int ncf_layout_tune(ncf_layout *lay, int64_t rows_per_launch);

/* Floats per slab row: tower_len + 64 (16-byte aligned rows; loss at index tower_len). */
int64_t ncf_slab_stride(const ncf_layout *lay);

/*
 * Fused forward + loss + backward for one global batch (replaces, per step,
 * NCF.forward models.py:97-118, BCEWithLogitsLoss train_neumf.py:113 and
 * loss.backward() train_neumf.py:114: embedding gathers, GMF product, MLP tower
 * GEMM+bias+ReLU, predict layer, BCE, tower dgrad/wgrad and embedding_dense_backward).
 *
 * Rows: global batch `ctl->batch % ceil(n_total / batch_global)` of the packed epoch
 * stream rows[0 .. ctl->n_total) (ncf_prepare_epoch output), last batch partial
 * (DataLoader drop_last=False); this rank takes rows [rank*ceil(gb/world), ...) of it.
 * grads: dense flat gradient buffer; embedding rows are scatter-added (f32
 * atomics), the tower/predict part is written to the slab at the start of
 * `workspace` (ncf_workspace_bytes(lay, ceil(batch_global/world)) bytes) and moved into
 * grads by ncf_reduce_slab.
 * dz_mode NCF_DZ_BCE: the label is bit 63 of the row, `dlogit` is ignored (may be NULL).
 * dz_mode NCF_DZ_DLOGIT: dlogit[row] holds dL/dlogit per row (same indexing as rows).
 * logits_out (optional, may be NULL): per-row logits of this rank's rows.
 * user_order (optional, may be NULL; since ABI 12): ncf_user_order of the same rows,
 * batch_global and world.  Where ncf_uses_user_order(lay), the step then sums the
 * user-side layer-0 gradients over runs of equal users before its atomics instead
 * of adding per row (same gradient up to fp32 summation order); on the fused path
 * with NCF_LAYOUT_USER_STORE every user-side gradient row (Um and Ug) is stored into
 * the workspace and a second launch sums each 32-position piece of the user order
 * (one float atomic per user and piece instead of one per row).
 */
int ncf_train_step(const ncf_layout *lay, const float *params, float *grads, const uint64_t *rows,
                   const int64_t *user_order,
                   const float *dlogit, ncf_step_ctl *ctl, int64_t batch_global, int world,
                   int rank, int dz_mode, void *workspace, int64_t workspace_bytes,
                   float *logits_out, void *stream);

/*
 * Distillation step of the student (src/distillation/base.py:36-50,
 * response.py:15-32, feature.py:125-147, attention.py:81-102): ncf_train_step with
 * dz_mode NCF_DZ_KD, i.e. per row of the global batch B
 *   loss_i = w_task * bce(z_i, y_i) + w_resp * r_i,   loss = sum_i loss_i / B
 *   temperature <= 0:  r_i = (z_i - t_i)^2                    (response.py:28-32)
 *   temperature T > 0: r_i = T^2 (sigmoid(z_i/T) - sigmoid(t_i/T))^2   (base.py:27-34)
 *   dL/dz_i = (w_task * (sigmoid(z_i) - y_i) + w_resp * dr_i/dz_i) / B
 * teacher_logits[row]: the teacher's logit per row of the epoch stream (same indexing
 * as rows; ncf_forward of the teacher over the stream).  Feature terms are added by
 * ncf_kd_feature_step.
 */
int ncf_train_step_kd(const ncf_layout *lay, const float *params, float *grads, const uint64_t *rows,
                      const int64_t *user_order, const float *teacher_logits, ncf_step_ctl *ctl, int64_t batch_global, int world,
                      int rank, float w_task, float w_resp, float temperature, void *workspace,
                      int64_t workspace_bytes,
                      float *logits_out, void *stream);

/* ---- In-step Adam for small batches (ABI 18) ----------------------------------
 * The previous step's dense Adam (torch.optim.Adam, train_neumf.py:90,115) runs inside
 * the next training launch: the launch's training workgroups apply it on the fly to
 * every tower float and embedding row they read, its extra workgroups write it for
 * every active float, so a small-batch step is ONE launch (fused path, per-row layer 0,
 * the 4-wave geometry; single process).  Two state buffers (params / exp_avg /
 * exp_avg_sq: the caller's and `*_b`) and three gradient buffers (the caller's grads,
 * grads_1, grads_2) rotate: state S_n (after update n) lives in buffer (n + par) & 1,
 * update n's gradient (tower partials and loss slot included) in buffer n % 3.
 * Sequence: ncf_ais_begin; per chunk of k launches ncf_train_step_ais with step_i =
 * 0 .. k-1 (capturable), then ncf_ais_bump(k); ncf_ais_flush writes the last update
 * into the caller's buffers and advances ctl->adam_t -- the parameters, moments and
 * ctl are then exactly the two-launch form's.  All buffers hold ncf_layout.total
 * floats; `state` is 4 device int64. */
typedef struct ncf_ais_bufs {
    float *params_b, *exp_avg_b, *exp_avg_sq_b;
    float *grads_1, *grads_2;
    int64_t *state;
} ncf_ais_bufs;
int ncf_ais_supported(const ncf_layout *lay);
int ncf_ais_begin(const ncf_layout *lay, float *params, float *grads, float *exp_avg, float *exp_avg_sq,
                  const ncf_ais_bufs *b, const int64_t *ranges, int nranges, ncf_step_ctl *ctl, void *stream);
int ncf_train_step_ais(const ncf_layout *lay, float *params, float *grads, float *exp_avg, float *exp_avg_sq,
                       const ncf_ais_bufs *b, const int64_t *ranges, int nranges, const uint64_t *rows,
                       const float *dlogit, ncf_step_ctl *ctl, int64_t batch_global, int dz_mode, float kd_wt,
                       float kd_wr, float kd_temp, double lr, double beta1, double beta2, double eps,
                       float *loss_hist, int64_t hist_len, int64_t step_i, void *stream);
int ncf_ais_bump(ncf_step_ctl *ctl, const ncf_ais_bufs *b, int64_t k, void *stream);
int ncf_ais_flush(const ncf_layout *lay, float *params, float *grads, float *exp_avg, float *exp_avg_sq,
                  const ncf_ais_bufs *b, const int64_t *ranges, int nranges, ncf_step_ctl *ctl, double lr,
                  double beta1, double beta2, double eps, float *loss_hist, int64_t hist_len, void *stream);

/*
 * Feature distillation terms (src/distillation/feature.py:51-123) of the same batch
 * as the preceding ncf_train_step[_kd] launch (reads ctl->batch; run it before
 * ncf_reduce_slab / ncf_reduce_adam_step).  Two feature keys:
 *   key 0 "gmf_features": x = Ug_s[u] * Ig_s[i] (f_s),   teacher Ug_t[u] * Ig_t[i] (f_t)
 *   key 1 "mlp_input":    x = [Um_s[u] | Im_s[i]] (2dm_s), teacher [Um_t[u] | Im_t[i]] (2dm_t)
 * a = A x + c (adapter nn.Linear [T, S] + bias [T]; A == NULL: identity, S == T);
 * loss += coef_k / (B * T_k) * sum_o (a_o - x_t,o)^2 with coef_k = beta / count (0 skips
 * the key); dL/dx = A^T (2 coef_k / (B T_k) (a - x_t)) is scatter-added into the student
 * embedding gradients (GMF through the product rule).  The loss term is added to the
 * loss column of slab row 0 of `workspace` (the student's train workspace).
 * Limits: f_s, f_t <= 64; 2dm_s <= 1024; 2dm_t <= 2048.
 */
int ncf_kd_feature_step(const ncf_layout *student, const float *s_params, float *s_grads,
                        const ncf_layout *teacher, const float *t_params, const uint64_t *rows,
                        const ncf_step_ctl *ctl, int64_t batch_global, int world, int rank,
                        const float *gmf_w, const float *gmf_b, float gmf_coef,
                        const float *mlp_w, const float *mlp_b, float mlp_coef,
                        void *workspace, void *stream);

/* Forward only (NCF.forward under no_grad, metrics.py:11-12): logits[n] of rows[n].
 * workspace: ncf_forward_workspace_bytes(lay, n) bytes (may be NULL when that is 0). */
int ncf_forward(const ncf_layout *lay, const float *params, const uint64_t *rows, int64_t n,
                float *logits, void *workspace, int64_t workspace_bytes, void *stream);

/* rows_out[k] = NCF_ROW_PACK(users[k], items[k], labels ? labels[k] : 0) (the feature /
 * label tensors the reference DataLoader yields, datasets.py:72-78). */
int ncf_pack_rows(const int32_t *users, const int32_t *items, const float *labels, int64_t n,
                  uint64_t *rows_out, void *stream);

/*
 * Factored layer 0 (MLP shapes with user_num + item_num <= 32768 and dm in
 * {8, 16, 32, 64, 128}, on the layered path also 256 and 512, unless
 * NCF_LAYOUT_PER_ROW_L0; ncf_fact_mode says whether it runs): the step scatter-adds,
 * per row, the layer-0 pre-activation gradient D0
 * (width dm) into the user and item rows of grads[um] / grads[im] instead of
 * forming the layer-0 weight and data gradients per row, and a second launch turns
 * those row sums into the true gradients (from the same params the step used):
 *   dUm = G W0[:, :dm],  dIm = H W0[:, dm:]   (in place),
 *   dW0 = [G^T Um | H^T Im]                   (per-block partials in the tail of the
 *                                              train workspace; ncf_reduce_slab /
 *                                              ncf_reduce_adam_step sum them in a fixed
 *                                              order with the other tower columns;
 *                                              dm > 128: added into the slab's W0
 *                                              columns by GEMM blocks, no partials).
 * Since ABI 8 ncf_train_step / ncf_train_step_kd issue that second launch
 * themselves, so a step is always: ncf_train_step[_kd] -> [ncf_kd_feature_step] ->
 * ncf_reduce_slab or ncf_reduce_adam_step.  ncf_expand_grads is kept as a no-op
 * (NCF_OK) so an ABI-7 sequence that still calls it trains correctly.
 */
int ncf_expand_grads(const ncf_layout *lay, const float *params, float *grads, void *workspace, void *stream);

/* 1 if ncf_train_step runs the factored layer 0 for this layout (fused path, or
 * since ABI 10 the layered path too: there the layer-0 forward is a per-step
 * projection of both tables through W0, P = [Um W0[:, :dm]^T ; Im W0[:, dm:]^T],
 * gathered per row), else 0.  The train workspace then holds the dW0 partials after
 * the slab (ncf_workspace_bytes includes them). */
int ncf_fact_mode(const ncf_layout *lay);

/* Rows of the partial slab ncf_reduce_slab / ncf_reduce_adam_step sum for this
 * layout (fused: the step's workgroups, ncf_layout_tune; layered: up to 16 rows the
 * weight-gradient and predict blocks spread their atomics over), and the bytes of
 * dW0 partials after it (0 unless ncf_fact_mode).  Since ABI 10. */
int ncf_reduce_rows(const ncf_layout *lay);

/*
 * Dropout (models.py:23, nn.Dropout(p) before each of the L tower Linears; p > 0 in
 * lay->dropout): training steps (ncf_train_step[_kd]) with p > 0 run the layered
 * path with per-row layer 0; element (row r of the epoch stream, column c) of the
 * input of tower layer k is kept, at optimizer step t = ctl->adam_t, when
 * ncf_dropout_hash(seed, t, k, r, c) >= p * 2^32, and scaled by 1.0f / (1.0f - p)
 * (torch's inverted dropout).  The mask depends on the global row, so every rank
 * and every batch split sees the same one.  torch's own dropout draws from its
 * Philox stream, which is not reproduced: masks are not the reference's bits (parity
 * of the arithmetic given a mask is tested; the mask's statistics too).
 *   h = seed << 32 ^ t * 0x9E3779B97F4A7C15 ^ r * 0xBF58476D1CE4E5B9
 *       ^ (k << 16 | c) * 0x94D049BB133111EB  (64-bit wrap), then the splitmix64
 *   finalizer; the hash is its upper 32 bits.  Host-side: the same function.
 */
uint32_t ncf_dropout_hash(uint32_t seed, uint32_t t, uint32_t layer, int64_t row, uint32_t col);
int64_t ncf_fact_partials_bytes(const ncf_layout *lay);

/* p[0 .. n) = 0 with a kernel (no memset node in a captured graph); p 16-byte aligned,
 * n a multiple of 4.  Zeroes the local gradient bucket after the data-parallel
 * reduce-scatter (the replacement of optimizer.zero_grad, train_neumf.py:111, on
 * the sharded optimizer path). */
int ncf_zero_f32(float *p, int64_t n, void *stream);

/* grads[tower_begin + j] = sum_w slab[w][j] over the slab rows at the start of the
 * train workspace (loss slot included), in a fixed order (bitwise reproducible).  If
 * ctl != NULL, also advances ctl->batch and ctl->adam_t by one: the step's optimizer
 * then runs as step t = ctl->adam_t. */
int ncf_reduce_slab(const ncf_layout *lay, const void *workspace, float *grads, ncf_step_ctl *ctl,
                    void *stream);

/*
 * Dense Adam over the active ranges of the flat buffers (torch.optim.Adam,
 * _single_tensor_adam arithmetic; train_neumf.py:90,115), grads zeroed after
 * use (optimizer.zero_grad, train_neumf.py:111).  ranges: host array of
 * 2*nranges int64 [begin, end) pairs (16-byte aligned).  t = ctl->adam_t (already
 * advanced by ncf_reduce_slab).  If loss_hist != NULL, one thread stores
 * grads[loss_slot] into loss_hist[(ctl->batch - 1) % hist_len].
 */
int ncf_adam_step(float *params, float *grads, float *exp_avg, float *exp_avg_sq,
                  const int64_t *ranges, int nranges, ncf_step_ctl *ctl, double lr,
                  double beta1, double beta2, double eps, int64_t loss_slot, float *loss_hist,
                  int64_t hist_len, void *stream);

/*
 * Sharded Adam of the factored path (data-parallel dp_mode "zero1" with
 * NCF_LAYOUT_FACT_DEFER_DX; replaces optimizer.step(), train_neumf.py:90,115, on
 * this rank's shard).  gshard holds the reduce-scattered flat gradient shard
 * [shard_begin, shard_begin + n): in its Um / Im rows the summed per-entity D0 sums
 * G (the step deferred their expansion), elsewhere the gradient itself.  One launch
 * (since ABI 16): blocks over the shard's Um / Im rows form dX = G W0[:, half] on
 * MFMA tiles (W0 being the weights the step ran with, saved in the step's workspace)
 * and apply Adam to those elements from LDS; other blocks run Adam on the remaining
 * active ranges (shard-relative) of params (the flat parameters + shard_begin); the
 * rest clear grads_local[0, grads_n) (the local gradient bucket; may be NULL with
 * grads_n 0) for the next step.  gshard itself is not cleared (the next
 * reduce-scatter overwrites it).  Where a table window is not inside one active range
 * or more than 8 ranges remain, the expansion runs in place in gshard and
 * ncf_adam_step follows (same result).  Fused path, factored layer 0 with dm <= 64,
 * shard_begin a multiple of 64: NCF_E_UNSUPPORTED otherwise.  Loss bookkeeping as
 * ncf_adam_step (loss_slot shard-relative, or loss_hist NULL on the other ranks).
 */
int ncf_adam_step_fact(const ncf_layout *lay, const void *workspace, float *params, float *gshard,
                       float *exp_avg, float *exp_avg_sq, const int64_t *ranges, int nranges, int64_t shard_begin,
                       float *grads_local, int64_t grads_n, ncf_step_ctl *ctl, double lr, double beta1,
                       double beta2, double eps, int64_t loss_slot, float *loss_hist, int64_t hist_len,
                       void *stream);

/*
 * ncf_reduce_slab + ncf_adam_step in one launch (single-process training: no
 * gradient exchange between the two).  The tower/predict gradient is summed from
 * the slab in the same fixed order and applied by Adam in the same block, without
 * being stored; embedding ranges take the plain Adam path.  Reads the step from the
 * snapshot ncf_train_step wrote (ctl->snap_t, ctl->snap_batch), then sets
 * ctl->adam_t = snap_t and ctl->batch = snap_batch + 1, and records the loss into
 * loss_hist[snap_batch % hist_len].
 */
int ncf_reduce_adam_step(const ncf_layout *lay, const void *workspace, float *params, float *grads,
                         float *exp_avg, float *exp_avg_sq, const int64_t *ranges, int nranges,
                         ncf_step_ctl *ctl, double lr, double beta1, double beta2, double eps,
                         float *loss_hist, int64_t hist_len, void *stream);

/*
 * Deferred ("catch-up") Adam -- since ABI 13.  Exactly the dense Adam of
 * ncf_reduce_adam_step (torch.optim.Adam, train_neumf.py:90,115: every row moves
 * every step through its moments), moving only the embedding rows that need it:
 * for a row whose gradient is exactly zero, Adam step s is a fixed per-element fp32
 * sequence with step-s scalars, so the steps a row sat out are replayed, in order,
 * with the same arithmetic, when the row is next needed -- bitwise the dense result.
 *
 * ncf_batch_touched (layout since ABI 14): for every global batch b of the epoch stream
 * (rows[0..n), batches of batch_global rows, padding rows skipped) and each side
 * (users, items), three disjoint sorted id lists:
 *   A_b = the ids batch b holds (their gradient is this step's),
 *   B_b = the ids batch b + 1 holds that A_b does not (the next forward reads them);
 *         on the epoch's last batch, every id not in A_b,
 *   C_b = the ids of slice (b % span) that are in neither (rolling catch-up: no row
 *         falls more than span steps behind; span = NCF_LAZY_SPAN, default 32).
 * touched (ncf_touched_bytes bytes, 8-byte aligned): int64 seg[6 nb + 1] -- list
 * k = 2 * list + side of batch b is ids[seg[6b + k] .. seg[6b + k + 1]) -- then the
 * int32 ids.  nb = ceil(n / batch_global).  U, I <= 2^19 (two LDS bitmaps per block).
 *
 * ncf_lazy_adam_step: ncf_reduce_adam_step's tower part (slab reduction + Adam, loss,
 * ctl commit) and, over the embedding tables, the rows of batch b = snap_batch % nb's
 * three lists, each brought from last_step[row] + 1 to t = snap_t: replays with g = 0,
 * then step t (A rows: with their gradient, which is cleared).  The lists are
 * disjoint: no atomics.  last_step: int32 [U + I] (users, then items; 0 = none since
 * Adam state zero, or the step the optimizer state was loaded at).  step_scalars:
 * float [ring][2], written for step t by this launch; ring >= 514.  n_total /
 * batch_global: the epoch stream's.  factor_num % 4 == 0 (NCF_E_UNSUPPORTED otherwise).
 *
 * ncf_lazy_adam_flush: every embedding row through t = ctl->adam_t (after that step's
 * ncf_lazy_adam_step): parameters and moments equal the dense optimizer's again --
 * before a metrics() pass, state_dict() or a checkpoint.
 */
int64_t ncf_touched_bytes(int64_t n, int64_t batch_global, int user_num, int item_num);
int ncf_batch_touched(const uint64_t *rows, int64_t n, int64_t batch_global, int user_num, int item_num,
                      int32_t *touched, void *stream);
int ncf_lazy_adam_step(const ncf_layout *lay, const void *workspace, float *params, float *grads,
                       float *exp_avg, float *exp_avg_sq, const int64_t *ranges, int nranges,
                       ncf_step_ctl *ctl, double lr, double beta1, double beta2, double eps,
                       float *loss_hist, int64_t hist_len, const int32_t *touched, int64_t n_total,
                       int64_t batch_global, int32_t *last_step, float *step_scalars, int64_t ring,
                       void *stream);
int ncf_lazy_adam_flush(const ncf_layout *lay, float *params, float *grads, float *exp_avg,
                        float *exp_avg_sq, const int64_t *ranges, int nranges, const ncf_step_ctl *ctl,
                        double beta1, double beta2, double eps, int32_t *last_step,
                        const float *step_scalars, int64_t ring, void *stream);

/*
 * Data-parallel deferred Adam (dp_mode "touched"; since ABI 13).  Every rank knows
 * the global batch, so every rank holds the same lists A_b of the rows batch b
 * touches (ncf_batch_touched) and packs its partial gradient of exactly those rows,
 * in list order, into one buffer of ncf_touched_packed_floats(lay, ranges, nranges,
 * batch_global) floats:
 *   [min(U, B)] user rows ((Ug active ? f : 0) + (Um active ? dm : 0) floats each),
 *   [min(I, B)] item rows, then ncf_slab_stride floats of tower gradient (+ loss).
 * ncf_touched_pack (after ncf_train_step): the slab / W0 partial reduction into the
 * tail, batch b's A rows into the list slots (slots past the list's count zeroed),
 * those rows of grads cleared.  Then one
 * all-reduce (sum) of the whole buffer, and ncf_lazy_adam_step_packed -- the
 * deferred Adam of ncf_lazy_adam_step with batch b's gradients (and the tower's)
 * read from the summed buffer, the same on every rank: no parameter all-gather.
 */
int64_t ncf_touched_packed_floats(const ncf_layout *lay, const int64_t *ranges, int nranges, int64_t batch_global);
int ncf_touched_pack(const ncf_layout *lay, const void *workspace, float *grads, const int64_t *ranges,
                     int nranges, const int32_t *touched, int64_t n_total, int64_t batch_global,
                     const ncf_step_ctl *ctl, float *packed, void *stream);
int ncf_lazy_adam_step_packed(const ncf_layout *lay, float *params, float *exp_avg, float *exp_avg_sq,
                              const int64_t *ranges, int nranges, ncf_step_ctl *ctl, double lr, double beta1,
                              double beta2, double eps, float *loss_hist, int64_t hist_len,
                              const int32_t *touched, int64_t n_total, int64_t batch_global,
                              int32_t *last_step, float *step_scalars, int64_t ring, const float *packed,
                              void *stream);

/*
 * Owner-sharded sparse gradient exchange (data-parallel dp_mode "owner"; since ABI 17).
 * Replaces, across `world` ranks, the reference's single-device loss.backward() +
 * optimizer.step() over dense nn.Embedding tables (scripts/train_neumf.py:90,114-115;
 * src/ncf/models.py:11-16): the embedding row `id` of either side (user, item) is owned
 * by rank id % world; every rank holds the same epoch stream, so every rank knows the
 * rows each rank slice of each global batch touches.  Per step, after ncf_train_step:
 *   ncf_owner_pack    this rank's gradient rows of batch b into send[o] (o = 0..world-1,
 *                     plan.send_floats each): slot k of side s holds the row of the k-th
 *                     id (ascending) of S_b(o, s) = the ids of this rank's slice owned by o;
 *                     the tower gradient (slab + W0 partials + loss, ncf_slab_stride
 *                     floats) at plan.tail_offset of every chunk; those grads rows cleared
 *   all_to_all        recv[r] = rank r's send[this rank]   (equal chunks; caller's RCCL)
 *   ncf_owner_adam    for every row this rank owns: the world ranks' rows summed in rank
 *                     order (R_b(r, s) = the ids of rank r's slice owned here), dense Adam
 *                     over every owned row (torch.optim.Adam, _single_tensor_adam
 *                     arithmetic, as ncf_adam_step); the tower: the world tails summed in
 *                     rank order, Adam on the active ranges (replicated: bitwise the same
 *                     on every rank); loss_hist and ctl as ncf_reduce_adam_step (snapshot);
 *                     the updated rows of R_{b+1}(q, s) into send2[q] (plan.param_floats
 *                     each, same slot order), q != this rank
 *   all_to_all        recv2[o] = rank o's send2[this rank]
 *   ncf_owner_unpack  rows of S_{b+1}(o, s), o != this rank, from recv2[o] into params.
 * b + 1 wraps to batch 0 of the same stream.  A rank's replica holds current values of
 * the rows it reads; every other row may be stale until the caller gathers the owners'
 * rows (e.g. at the end of a run).  exp_avg / exp_avg_sq: full flat layout; the owned rows
 * and the tower are used.
 *
 * ncf_owner_plan_init (host): geometry for the stream (n_total rows, batch_global) and
 * max_u / max_i list slots per (rank, owner) -- the all_to_all chunk sizes.
 * ncf_owner_lists: the per-batch records (plan.lists_bytes) for this rank, and in
 * max_counts[2] (device int32, overwritten) the longest S list over every (batch, rank,
 * owner) per side.  If max_counts exceeds max_u / max_i, the lists were truncated: build
 * a plan with larger slots and call again before any step uses them.
 * Limits: world <= 16, factor_num % 4 == 0, user_num, item_num <= 2^19, rows of at most 1,024 floats.
 */
typedef struct ncf_owner_plan {
    int32_t world, rank, max_u, max_i;
    int64_t n_total, batch_global, nb;  /* the epoch stream and its batches */
    int32_t row_u, row_i;               /* floats per user / item row (its active tables) */
    int32_t chunk_u, chunk_i;           /* owned rows per optimizer block */
    int64_t nchunk_u, nchunk_i;
    int64_t record_ints, lists_bytes;   /* int32 per batch record; bytes of the lists */
    int64_t send_floats, param_floats;  /* floats per destination: gradient / parameter exchange */
    int64_t tail_offset;                /* tower gradient inside a gradient chunk */
    int64_t off[4];                     /* Ug, Ig, Um, Im flat offsets (-1: inactive) */
} ncf_owner_plan;
int ncf_owner_plan_init(const ncf_layout *lay, const int64_t *ranges, int nranges, int64_t n_total,
                        int64_t batch_global, int world, int rank, int max_u, int max_i, ncf_owner_plan *out);
int ncf_owner_lists(const ncf_owner_plan *plan, const ncf_layout *lay, const uint64_t *rows, int32_t *lists,
                    int32_t *max_counts, void *stream);
int ncf_owner_pack(const ncf_owner_plan *plan, const ncf_layout *lay, const void *workspace, float *grads,
                   const int32_t *lists, const ncf_step_ctl *ctl, float *send, void *stream);
int ncf_owner_adam(const ncf_owner_plan *plan, const ncf_layout *lay, float *params, float *exp_avg,
                   float *exp_avg_sq, const int64_t *ranges, int nranges, const int32_t *lists, ncf_step_ctl *ctl,
                   double lr, double beta1, double beta2, double eps, float *loss_hist, int64_t hist_len,
                   const float *recv, float *send2, void *stream);
int ncf_owner_unpack(const ncf_owner_plan *plan, const ncf_layout *lay, float *params, const int32_t *lists,
                     const ncf_step_ctl *ctl, const float *recv2, void *stream);

/* Plain SGD p -= lr * g (optim.SGD(lr*10) on the --pretraining path, train_neumf.py:87-88). */
int ncf_sgd_step(float *params, float *grads, const int64_t *ranges, int nranges,
                 ncf_step_ctl *ctl, double lr, int64_t loss_slot, float *loss_hist, int64_t hist_len,
                 void *stream);

/* rows_out[k] = rows[perm[k]] (DataLoader shuffle=True order, no grouping). */
int ncf_gather_epoch(const uint64_t *rows, const int64_t *perm, int64_t n, uint64_t *rows_out,
                     void *stream);

/*
 * Epoch stream for the fused step: global batch b holds rows perm[b*B .. b*B+cnt)
 * of the unshuffled packed stream (the DataLoader(shuffle=True) batch membership,
 * train_neumf.py:55,106), written back grouped by item id (sort per batch; order
 * inside an item group is unspecified).  Order inside a batch does not change the
 * batch gradient; grouping lets the fused step reduce item-side gradients per item
 * before its atomics.  Three kernels: shuffle + per-batch item histogram, per-batch
 * scan into item offsets and part boundaries, per-part LDS sort with coalesced writes.
 * Global batches under 4096 rows are only shuffled (item runs would be ~1 row long).
 * workspace: device buffer of at least ncf_prepare_epoch_workspace() bytes.
 */
int64_t ncf_prepare_epoch_workspace(int64_t n, int64_t batch_global, int item_num);
int ncf_prepare_epoch(const uint64_t *rows, const int64_t *perm, int64_t n, int64_t batch_global,
                      int item_num, uint64_t *rows_out, void *workspace, int64_t workspace_bytes,
                      void *stream);

/*
 * ncf_prepare_epoch with flags.  NCF_PREP_CANONICAL: the rows of each item inside a
 * batch come out sorted by (user, label) -- a canonical order that does not depend
 * on the placement order of the grouping, so every rank of a data-parallel group
 * that builds the same epoch stream gets the same rows in the same positions (rank r
 * takes positions [r per, (r + 1) per) of each global batch).  Batches below 4,096
 * rows are not grouped (the shuffle alone is deterministic).  Same workspace.
 */
#define NCF_PREP_CANONICAL 0x1
int ncf_prepare_epoch2(const uint64_t *rows, const int64_t *perm, int64_t n, int64_t batch_global, int item_num,
                       int flags, uint64_t *rows_out, void *workspace, int64_t workspace_bytes, void *stream);

/*
 * User order of an epoch stream (since ABI 12): each global batch b of rows[0 .. n)
 * is cut into the `world` rank slices ncf_train_step takes (cnt = its rows, slice r =
 * [r*ceil(cnt/world), ...)), and order[slice start + k], k over the slice, lists the
 * slice's rows by ascending user id, padding rows (user -1) last, as entries
 * (int64_t)user << 32 | offset (offset 0-based within the slice, user -1 for
 * padding): the step reads the user with the offset.  The order among rows of one
 * user is unspecified.  The buffer holds n such entries followed by n int32 inverse
 * positions: ((int32_t *)(order + n))[slice start + k] = the position of the slice's
 * row k in its order (12 bytes per row in all).  One counting sort per slice in LDS:
 * user_num <= 32767.
 * Computed once per epoch; the step reads it where ncf_uses_user_order(lay) (the
 * layered factored layer 0).
 */
int ncf_user_order(const uint64_t *rows, int64_t n, int64_t batch_global, int world, int user_num,
                   int64_t *order, void *stream);
int ncf_uses_user_order(const ncf_layout *lay);

/*
 * Device epoch pipeline: the DataLoader(shuffle=True) permutation and the epoch's
 * rows built on the device (the negatives come from the host sampler,
 * ncf_sampler.h; the generator words from ncf_mt_words).
 *
 * ncf_randperm: torch.randperm(n, generator=g) after g.manual_seed(seed) (the
 * RandomSampler of DataLoader(shuffle=True), train_neumf.py:55): Fisher-Yates
 * swapping r[i] with r[i + words[i] % (n - i)], words = the first n - 1 words of
 * ncf_mt_seed(seed & 0xffffffff).  Computed in closed form (three passes, no
 * rounds; see ncf_epoch.hip), always complete.  Since ABI 9 (was: a `rounds`
 * count and a device `remaining` report of the round-based version).
 *
 * ncf_build_rows: rows_out = NCF_ROW_PACK of features_fill / labels_fill
 * (datasets.py:65-69): positives in file order, then positive p's num_ng
 * negatives neg[p*num_ng .. (p+1)*num_ng).
 */
int64_t ncf_randperm_workspace(int64_t n);
int ncf_randperm(const uint32_t *words, int64_t n, int64_t *perm, void *workspace, int64_t workspace_bytes,
                 void *stream);
int ncf_build_rows(const int32_t *pos_users, const int32_t *pos_items, int64_t n_pos, const int32_t *neg, int num_ng,
                   uint64_t *rows_out, void *stream);

/*
 * HR@K / NDCG@K per DataLoader batch (metrics.py:4-25): batches of `batch`
 * consecutive rows (last one partial), ground truth = the batch's first item,
 * recommends = items of the top_k logits.  hr[b] in {0,1}; ndcg[b] = 1/log2(pos+2).
 * Returns NCF_E_ARG if a batch is shorter than top_k (torch.topk raises there).
 */
int ncf_hr_ndcg(const float *logits, const int32_t *items, int64_t n, int batch, int top_k,
                int32_t *hr, float *ndcg, void *stream);

/* Diagnostics only: ablation switches for the next ncf_train_step launches
 * (1 = skip embedding scatter-add, 2 = skip weight-gradient MFMAs).  Results are
 * wrong while any switch is set; 0 restores the production kernel. */
int ncf_debug_set_diag(int flags);

/*
 * Ceiling probe of the embedding access pattern (bench.py `roofline_cache`): for the
 * n packed rows, the 16-byte pieces of their four embedding rows (Ug[u], Ig[i],
 * Um[u], Im[i]; models.py:108-112) gathered (mode 1), float-atomically added into
 * the same rows of grads (mode 2), or both (mode 3) -- the fused step's gather and
 * scatter with no arithmetic, on tables that sit in L2 / the MALL at ml-1m.  NeuMF
 * layouts with factor_num % 4 == 0.  sink: NCF_PROBE_BLOCKS * 256 floats (modes 1, 3).
 */
#define NCF_PROBE_BLOCKS 2048
int ncf_probe_gather_scatter(const ncf_layout *lay, const float *params, float *grads, float *sink,
                             const uint64_t *rows, int64_t n, int mode, void *stream);
/* Workgroup geometry of the fused step for later ncf_layout_tune calls: 0 = chosen by
 * the per-rank batch (narrower workgroups for small batches), 8, 4, 2 or 1 waves =
 * forced where that kernel exists (A/B measurements, tests).  NCF_E_ARG otherwise. */
int ncf_debug_set_geometry(int waves);
/* Per-row layer 0 (NCF_LAYOUT_PER_ROW_L0) for later ncf_layout_tune calls: -1 = the
 * tune rule (the default), 0 = never, 1 = always (A/B measurements). */
int ncf_debug_set_per_row(int mode);
/* User-side store-and-sum (NCF_LAYOUT_USER_STORE) for later ncf_layout_tune calls:
 * 0 = never (the default), -1 = from 16,384 rows per launch, 1 = wherever it applies. */
int ncf_debug_set_user_store(int mode);

/* Diagnostics only: device buffer of ncf_slab_rows() x 64 uint64 that the next
 * ncf_train_step launches fill with per-workgroup s_memtime phase stamps
 * (NULL = off, the production setting). */
int ncf_debug_set_stamps(unsigned long long *dev_buf);

#ifdef __cplusplus
}
#endif
#endif /* NCF_HIP_H */
