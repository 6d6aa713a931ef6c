/*
 * hvae.h -- C ABI of libhvae.so, the MI355X (gfx950) HybridVAE train/eval path.
 *
 * Conventions (every entry point):
 *   - all pointers are DEVICE pointers owned by the caller (PyTorch tensors in
 *     the Python host code), except the small config structs, which live on
 *     the host and are read during the call;
 *   - sizes are int64_t; matrices are row-major with an explicit leading
 *     dimension where it matters;
 *   - `stream` is a hipStream_t passed as void*; work is enqueued on it and
 *     the call returns without synchronising;
 *   - nothing allocates, frees or synchronises, so any sequence of calls can
 *     be captured into a hipGraph;
 *   - the return value is HVAE_OK (0) or a negative HVAE_ERR_*; the text of
 *     the last error of the calling thread is available via hvae_last_error.
 *
 * Each entry point names the reference interface it replaces
 * (/root/reference = Aymane-Nouhail/Recommendation-System).
 */
#ifndef HVAE_H_
#define HVAE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HVAE_ABI_VERSION 5

enum {
  HVAE_OK = 0,
  HVAE_ERR_ARG = -1,         /* bad shape / null pointer / inconsistent sizes */
  HVAE_ERR_HIP = -2,         /* HIP runtime error (launch or API)              */
  HVAE_ERR_UNSUPPORTED = -3, /* shape or dtype this build has no kernel for    */
  HVAE_ERR_WORKSPACE = -4    /* workspace smaller than the *_workspace() query */
};

enum { HVAE_F32 = 0, HVAE_BF16 = 1, HVAE_FP8 = 2 };

/* ----------------------------------------------------------------- misc -- */
int hvae_version(void);
/* Copies the calling thread's last error text (NUL-terminated) into buf. */
int hvae_last_error(char* buf, size_t len);
/* Live kernel timing for benchmarks: arm one kernel by name ("decoder_sweep",
 * "decoder_finalize", "adam_rows", "adam_dense", "encoder_fwd", "gemm",
 * "ln_bwd", "rowgrad_apply", "clip"); its next max_launches launches
 * (outside stream capture) are bracketed by a hipEvent pair recorded on the
 * launch stream. hvae_probe_collect synchronizes those events and returns the
 * mean launch duration. hvae_probe_arm(NULL, 0) disarms. */
int hvae_probe_arm(const char* kernel, int max_launches);
int hvae_probe_collect(double* avg_us, int* launches);

/* ------------------------------------------------------------ data view -- */
/* A batch of user rows of a CSR interaction matrix (users x items).
 * Replaces the dense row materialisation of UserInteractionDataset.__getitem__
 * + DataLoader collate (src/ml/train.py:35-47, 248-259): rows are read
 * in place from the device-resident CSR, never densified. Values are floats
 * because _build_matrix sums duplicate (user, item) pairs
 * (src/ml/train.py:175-182), so an entry can be 2.0 or more. */
typedef struct hvae_csr_batch {
  const int64_t* row_ptr; /* [n_rows + 1]                                     */
  const int32_t* col_idx; /* [nnz] item ids                                   */
  const float* vals;      /* [nnz] interaction values                         */
  const int32_t* rows;    /* matrix rows of this batch; NULL => 0..nb-1       */
  const int64_t* rows_offset; /* device index of the batch's first entry in  */
                          /* `rows` (NULL => 0): a hipGraph replayed once   */
                          /* per batch advances it with hvae_counter_add    */
  int64_t nb;             /* users in the batch                               */
  int64_t n_items;        /* N                                                */
} hvae_csr_batch;

/* Dense [B, N] input (the reference's collated batch, also what its unit tests
 * feed: tests/test_unit.py:167, including negative values) -> CSR of its
 * nonzeros, row order preserved. row_ptr[B] receives the nnz; entries beyond
 * `cap` are not written (caller sizes cap >= B*N or checks row_ptr[B]). */
int hvae_dense_to_csr(const float* x, int64_t B, int64_t N, int64_t* row_ptr, int32_t* col_idx,
                      float* vals, int64_t cap, void* ws, size_t ws_bytes, void* stream);
size_t hvae_dense_to_csr_workspace(int64_t B, int64_t N);

/* ------------------------------------------------------------- encoder -- */
/* First encoder layer over sparse rows, fused with its epilogue:
 *   a = x W1^T + b1 ; h = Dropout(GELU(LayerNorm(a)))
 * Replaces nn.Linear(N,H) -> LayerNorm(H) -> GELU() -> Dropout(p) of
 * HybridVAE._build_encoder / encode (src/ml/model.py:111-119, 149).
 * w1t is the item-major [N, H] image of encoder.0.weight ([H, N]).
 * drop_mult: optional [nb, H] explicit dropout multipliers (parity mode);
 * otherwise Philox(seed, *step_dev, layer) masks. train=0 => no dropout.
 * xhat_out [nb,H] and rstd_out [nb] are saved for the backward (nullable). */
int hvae_encoder_fwd(const hvae_csr_batch* x, const float* w1t, const float* b1, const float* ln_w,
                     const float* ln_b, int64_t H, float p_drop, const float* drop_mult,
                     uint64_t seed, const int64_t* step_dev, int train, float* h_out,
                     float* xhat_out, float* rstd_out, void* stream);

/* Same epilogue on a dense pre-activation a [nb, H] (hidden layers >= 2,
 * src/ml/model.py:111-119). `layer` selects the dropout stream. */
int hvae_ln_gelu_drop_fwd(const float* a, const float* ln_w, const float* ln_b, int64_t nb,
                          int64_t H, float p_drop, const float* drop_mult, uint64_t seed,
                          const int64_t* step_dev, uint32_t layer, int train, float* h_out,
                          float* xhat_out, float* rstd_out, void* stream);

/* Backward of Dropout(GELU(LayerNorm(a))): dh -> da, and d(ln_w), d(ln_b)
 * (written, not accumulated) and, if d_bias != NULL, d_bias = sum_b da[b, :]
 * (the bias gradient of the Linear that produced `a`, fused here instead of a
 * separate column-sum pass). Deterministic column sums through ws. */
int hvae_ln_gelu_drop_bwd(const float* dh, const float* xhat, const float* rstd,
                          const float* ln_w, const float* ln_b, int64_t nb, int64_t H,
                          float p_drop, const float* drop_mult, uint64_t seed,
                          const int64_t* step_dev, uint32_t layer, int train, float* da,
                          float* d_ln_w, float* d_ln_b, float* d_bias, void* ws, size_t ws_bytes,
                          void* stream);
size_t hvae_ln_gelu_drop_bwd_workspace(int64_t nb, int64_t H);

/* Row-sparse gradient of the item-major first-layer weight W1t [N, H]:
 *   dW1t[j, :] = sum_{b : j in row b} x_bj * da[b, :]
 * (autograd of nn.Linear(N,H) at src/ml/model.py:114 under loss.backward(),
 * src/ml/train.py:90). Only the items present in the batch get a row; rows
 * are summed in ascending batch-row order, so the result is bitwise
 * reproducible. Slots are assigned in ascending item order. */
#define HVAE_ROWSQ_PARTS 16
typedef struct hvae_rowgrad {
  int32_t* cnt;         /* [N]   scratch; must be zero on entry, left zero      */
  int32_t* slot_of;     /* [N]   item -> slot, valid iff slot < *n_unique and   */
                        /*       item_of[slot] == item                          */
  int32_t* item_of;     /* [cap] slot -> item (ascending)                       */
  int32_t* seg_off;     /* [cap + 1]                                            */
  int32_t* fill;        /* [cap] scratch; must be zero on entry, left zero      */
  int32_t* contrib_row; /* [cap]                                                */
  float* contrib_val;   /* [cap]                                                */
  float* rows;          /* [cap, H] gradient rows                               */
  int32_t* n_unique;    /* [1] device                                           */
  int64_t cap;          /* >= nnz of any batch                                  */
  int64_t n_items;      /* N                                                    */
  int32_t* contrib_slot;/* [cap] slot of each (sorted) contribution             */
  float* part;          /* [part_floats] scratch of the chunked row gather      */
  int64_t part_floats;  /* >= hvae_rowgrad_part_floats(cap, H)                  */
  double* rowsq;        /* [cap, HVAE_ROWSQ_PARTS] or NULL: partial sums over h */
                        /*       of rows[s, h]^2 (fp64), written by the apply   */
                        /*       with each row, so the clip reads 128 B per row */
                        /*       instead of the row. Non-NULL ONLY when         */
                        /*       hvae_w1_rowgrad_apply produced `rows`: a      */
                        /*       caller that writes rows itself passes NULL,   */
                        /*       or the clip adds stale sums                   */
                        /*       instead of 4 H                                 */
} hvae_rowgrad;
/* Scratch the row gather needs for hidden width H (chunk partials, and the
 * staging copy of the long-segment sort). */
int64_t hvae_rowgrad_part_floats(int64_t cap, int64_t H);
int hvae_w1_rowgrad(const hvae_csr_batch* x, const float* da, int64_t H, const hvae_rowgrad* rg,
                    void* ws, size_t ws_bytes, void* stream);
size_t hvae_w1_rowgrad_workspace(int64_t n_items);
/* hvae_w1_rowgrad in two halves. _plan depends on the batch only (per-item
 * counts, slots, segments, and each segment's contributions sorted by batch
 * row), so a train step can run it on a side stream while the forward runs;
 * _apply then gathers x * da into the rows. plan + apply == hvae_w1_rowgrad. */
int hvae_w1_rowgrad_plan(const hvae_csr_batch* x, const hvae_rowgrad* rg, void* ws, size_t ws_bytes,
                         void* stream);
int hvae_w1_rowgrad_apply(const float* da, int64_t H, const hvae_rowgrad* rg, void* stream);

/* Trainable item embeddings (HybridVAE(freeze_embeddings=False), reference src/ml/model.py:72-75): the pieces the
 * fused step adds for E's gradient dE_i = (1/B) sum_b (n_b softmax(u_b E^T)_i - x_bi) u_b (ABI 4).
 *   hvae_csr_row_sums:        out[b] = n_b = sum of batch row b's stored values.
 *   hvae_softmax_weights:     S[b][c] = alpha * w[b] * exp(S[b][c] - lse[b]), in place (S: nb rows of ld floats).
 *   hvae_rowgrad_scatter_rows: dst[item_of[s]][0:width] += alpha * rows[s][0:width] for the plan's slots
 *                             s < n_unique (rows as hvae_w1_rowgrad_apply wrote them with H = width). */
int hvae_csr_row_sums(const hvae_csr_batch* x, float* out, void* stream);
int hvae_softmax_weights(float* S, int64_t ld, int64_t nb, int64_t ncol, const float* lse, const float* w,
                         float alpha, void* stream);
int hvae_rowgrad_scatter_rows(const hvae_rowgrad* rg, int64_t width, float alpha, float* dst, int64_t ldd,
                              void* stream);
/* Scatter the row-sparse gradient into a dense, caller-zeroed buffer laid out
 * [N, ld] (item-major; ld >= H). */
int hvae_rowgrad_to_dense(const hvae_rowgrad* rg, int64_t H, float* dense, int64_t ld, void* stream);

/* ---------------------------------------------------------- dense GEMM -- */
/* C[M,N] = alpha * op(A)[M,K] * op(B)[K,N] + beta * C, then the epilogue.
 * op(A) = A ([M,K], lda) or A^T (A stored [K,M]); op(B) = B ([K,N]) or B^T
 * (B stored [N,K], i.e. an nn.Linear weight). fp32 in, fp32 out, on the
 * exact-f32 MFMA (v_mfma_f32_16x16x4_f32). Replaces the addmm / mm of every
 * small nn.Linear on the path and its autograd: fc_mu/fc_logvar
 * (src/ml/model.py:126-127,152-153), the projection MLP (:90-95,195), the
 * deeper encoder layers (:114), and the materialised scores u E^T (:198). */
enum {
  HVAE_EPI_NONE = 0,
  HVAE_EPI_BIAS = 1,           /* + bias[n]                                        */
  HVAE_EPI_BIAS_GELU_DROP = 2, /* pre = acc + bias -> pre_out; C = Drop(GELU(pre)) */
  HVAE_EPI_GELU_DROP_BWD = 3,  /* C = acc * dropmult * GELU'(pre_in)               */
  HVAE_EPI_DROP_BWD = 4,       /* C = acc * dropmult                               */
  HVAE_EPI_REPARAM_BWD = 5     /* acc = dz; pre_in = heads [M, ldc] (mu | logvar at */
                               /* col n | N + n); writes C[:, n] = dmu and          */
                               /* C[:, N + n] = dlogvar (hvae_reparam_kl_bwd's math) */
};
typedef struct hvae_epilogue {
  int kind;
  const float* bias;      /* [N]                                                   */
  float* pre_out;         /* [M, ldc] (BIAS_GELU_DROP)                             */
  const float* pre_in;    /* [M, ldc] (GELU_DROP_BWD)                              */
  float p_drop;           /* dropout probability                                   */
  const float* drop_mult; /* [M, N] explicit multipliers (parity mode) or NULL     */
  uint64_t seed;
  const int64_t* step_dev;
  uint32_t tag;           /* Philox stream tag (see hvae_common.h)                 */
  int train;              /* 0 => dropout is identity                              */
  float* opa_rowsum;      /* [M] or NULL: sum_k op(A)[m, k] (x alpha), computed from */
                          /* the A tiles the GEMM already stages: the bias gradient */
                          /* of a Linear alongside its weight gradient dY^T X       */
  const float* aux;       /* REPARAM_BWD: eps [M, N]                                */
  float aux_scale;        /* REPARAM_BWD: KL gradient scale beta / B               */
  const float* aux_scale_dev; /* REPARAM_BWD: if non-NULL, the device scalar that   */
                          /* replaces aux_scale (an annealed beta / B written by    */
                          /* hvae_anneal_beta earlier on the stream)                */
} hvae_epilogue;
int hvae_gemm_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, float alpha,
                  const float* A, int64_t lda, const float* B, int64_t ldb, float beta, float* C,
                  int64_t ldc, const hvae_epilogue* epi, void* ws, size_t ws_bytes, void* stream);
size_t hvae_gemm_f32_workspace(int64_t M, int64_t N, int64_t K);
/* One problem of hvae_gemm_f32_pair: hvae_gemm_f32's arguments, with its own workspace. */
typedef struct hvae_gemm_desc {
  int trans_a, trans_b;
  int64_t M, N, K;
  float alpha;
  const float* A; int64_t lda;
  const float* B; int64_t ldb;
  float beta;
  float* C; int64_t ldc;
  const hvae_epilogue* epi;
  void* ws; size_t ws_bytes;
} hvae_gemm_desc;
/* Two independent GEMMs of one layer's backward -- the weight gradient (w: trans_a = 1,
 * trans_b = 0) and the data gradient (x: both 0) -- in one launch (the two matmuls autograd
 * runs for each nn.Linear of model.py:100-155 in backward). Other pairings run as two
 * hvae_gemm_f32 launches. Split-K problems need distinct workspaces. */
int hvae_gemm_f32_pair(const hvae_gemm_desc* w, const hvae_gemm_desc* x, void* stream);

/* out[n] = beta * out[n] + sum_m X[m, n]  (bias gradients; deterministic) */
int hvae_colsum(const float* X, int64_t M, int64_t N, int64_t ldx, float beta, float* out,
                void* ws, size_t ws_bytes, void* stream);
size_t hvae_colsum_workspace(int64_t M, int64_t N);

/* ------------------------------------------------------ latent (K5, K9) -- */
/* z = mu + eps * exp(0.5 logvar) (train) or z = mu (eval), and the per-row KL
 * term kl_rows[b] = -0.5 * sum_l (1 + lv - mu^2 - exp(lv)).
 * Replaces HybridVAE.reparameterize (src/ml/model.py:157-179) and the KL line
 * of vae_loss_function (src/ml/model.py:287). eps_in: explicit noise [nb,L]
 * (parity mode) or NULL for Philox normals; eps_out saves it (nullable). */
int hvae_reparam_kl_fwd(const float* mu, const float* logvar, int64_t ld, int64_t nb, int64_t L,
                        int train, const float* eps_in, uint64_t seed, const int64_t* step_dev,
                        float* z, float* eps_out, float* kl_rows, void* stream);
/* dmu = dz + kl_scale * mu ; dlv = dz * eps * 0.5 exp(0.5 lv) + kl_scale * 0.5 (exp(lv) - 1)
 * with kl_scale = beta / nb (dz may be NULL: KL-only gradient); kl_scale_dev (nullable) is a
 * device scalar that replaces kl_scale (hvae_anneal_beta's out2[1]). */
int hvae_reparam_kl_bwd(const float* dz, const float* mu, const float* logvar, int64_t ld,
                        const float* eps, int64_t nb, int64_t L, float kl_scale, const float* kl_scale_dev,
                        int train, float* dmu, float* dlogvar, int64_t ld_out, void* stream);
/* AnnealedVAE's KL-weight schedule (src/ml/model.py:312-334) on the device, so that an
 * annealed epoch replays one captured step: with s = *anneal_step,
 *   beta = s >= anneal_steps ? beta_max : beta_min + (s / anneal_steps) (beta_max - beta_min)
 * in double, as the reference's Python floats (get_current_beta); out2[0] = (float) beta,
 * out2[1] = (float)(beta / nb) (the KL gradient scale); then *anneal_step = s + 1
 * (step_annealing, src/ml/train.py:74-76). One launch per train step, before the kernels
 * that read out2 (hvae_decoder_train's beta_dev, the REPARAM_BWD epilogue's aux_scale_dev,
 * hvae_reparam_kl_bwd's kl_scale_dev). */
int hvae_anneal_beta(int64_t* anneal_step, double beta_min, double beta_max, int64_t anneal_steps, int64_t nb,
                     float* out2, void* stream);

/* ------------------------------------------- latent + projection MLP, row-parallel -- */
/* The chain between the encoder's last hidden layer and the decoder, for batches of at most
 * HVAE_MLP_ROWS_MAX_NB rows, in one launch per direction (each block owns a few batch rows and
 * streams the three weight matrices once; replaces four launches forward and three data-gradient
 * GEMMs backward). Forward (src/ml/model.py:126-127,152-153 fc_mu / fc_logvar, :157-179
 * reparameterize, :90-95,195 the projection Linear -> GELU -> Dropout -> Linear):
 *   heads = h W_heads^T + b_heads           [nb, 2L]  (mu | logvar)
 *   z, eps, kl_rows                          as hvae_reparam_kl_fwd (same Philox stream)
 *   p1 = z W_a^T + b_a ; q = Drop(GELU(p1))  [nb, D]   (dropout as HVAE_EPI_BIAS_GELU_DROP, tag 0x200)
 *   u = q W_b^T + b_b                        [nb, D]
 * Backward (their autograd, data gradients only; the weight gradients follow with
 * hvae_gemm_f32_multi):
 *   dp1 = (dU W_b) * dropmult * GELU'(p1) ; dz = dp1 W_a ;
 *   dheads = [dz + ks mu | dz eps 0.5 exp(0.5 lv) + ks 0.5 (exp(lv) - 1)] (hvae_reparam_kl_bwd's math,
 *   ks = beta / B or *ks_dev) ; dh = dheads W_heads.
 * Every matrix is row-major and dense (ld = its width); H, L, D multiples of 32, at most 1024. */
#define HVAE_MLP_ROWS_MAX_NB 1024
struct hvae_adam;  /* below: the Adam hyperparameters (hvae_adam) */
typedef struct hvae_mlp_rows {
  int64_t nb, H, L, D;
  const float* W_heads; const float* b_heads; /* [2L, H], [2L] */
  const float* W_a; const float* b_a;         /* [D, L], [D]   */
  const float* W_b; const float* b_b;         /* [D, D], [D]   */
  int train;
  float p_drop;
  const float* drop_mult;                     /* [nb, D] explicit dropout multipliers or NULL  */
  const float* eps_in;                        /* [nb, L] explicit noise or NULL (Philox)       */
  uint64_t seed;
  const int64_t* step_dev;
  /* forward: in h; out heads, z, eps (nullable), kl_rows, p1, q, u */
  const float* h;
  float* heads; float* z; float* eps; float* kl_rows; float* p1; float* q; float* u;
  /* backward: in dU (and heads, eps, p1 above); out dp1, dheads, dh */
  const float* dU;
  float ks; const float* ks_dev;
  float* dp1; float* dheads; float* dh;
  /* forward, optional: the batch's W1 row-gradient plan (hvae_w1_rowgrad_plan) run by one more block of the
   * same launch, beside the rows -- for batches whose plan fits one block (rg->cap <= 4096, nb <= 4096);
   * both NULL: no plan */
  const hvae_csr_batch* plan_x;
  const hvae_rowgrad* plan_rg;
  /* backward, optional: the last hidden layer's LayerNorm -> GELU -> Dropout backward on dh, fused
   * (hvae_ln_gelu_drop_bwd's outputs: da, d_ln_w, d_ln_b and, if non-NULL, d_bias; its dropout stream
   * `enc_layer`, multipliers enc_drop_mult [nb, H] or NULL); ln_w == NULL: dh only. ws >=
   * hvae_mlp_bwd_rows_workspace(nb, H) bytes for the column sums. With d_ln_w == d_ln_b == d_bias == NULL the
   * launch stops at the per-block column sums: ws then holds [hvae_mlp_rows_blocks(nb)][3][H] partials
   * (d(ln_w) | d(ln_b) | d(bias) terms, each block's rows added in order) for the caller to add in block order,
   * e.g. as three more products of the hvae_gemm_f32_multi launch that follows (partials^T x ones) -- one
   * launch boundary instead of an in-kernel cross-block hand-off */
  const float* ln_w; const float* ln_b; const float* xhat; const float* rstd;
  const float* enc_drop_mult; uint32_t enc_layer;
  float* da; float* d_ln_w; float* d_ln_b; float* d_bias;
  void* ws; size_t ws_bytes;
  /* forward, optional (one hidden layer, H <= 512): the first encoder layer (hvae_encoder_fwd) in the same launch --
   * reads enc_x, w1t, b1, ln_w, ln_b, enc_drop_mult; writes h (as h_out), xhat and rstd; NULL: h is an input */
  const hvae_csr_batch* enc_x;
  const float* w1t; const float* b1;
  /* forward with enc_x, optional: w1t read through exact lazy Adam -- each entry's row is brought from its
   * last_step stamp to *adam->step_dev steps in registers (hvae_adam_lazy_catchup_csr's replay, nothing stored:
   * the step's hvae_adam_lazy replays p, m and v itself), so no catch-up launch has to precede the forward;
   * adam == NULL: w1t is read as it is */
  const struct hvae_adam* adam;
  const float* adam_m; const float* adam_v; const int32_t* last_step; const float* adam_tab;
} hvae_mlp_rows;
int hvae_mlp_fwd_rows(const hvae_mlp_rows* a, void* stream);
int hvae_mlp_bwd_rows(const hvae_mlp_rows* a, void* stream);
size_t hvae_mlp_bwd_rows_workspace(int64_t nb, int64_t H);
/* blocks of the row-parallel MLP launches for nb rows (the partial count of the deferred column sums) */
int64_t hvae_mlp_rows_blocks(int64_t nb);
/* 1 if hvae_mlp_fwd_rows and hvae_mlp_bwd_rows accept a batch of nb rows at these widths (fused_enc: with the
 * first encoder layer in the forward launch), else 0 -- the caller then runs the GEMM chain */
int hvae_mlp_rows_supported(int64_t nb, int64_t H, int64_t L, int64_t D, int fused_enc);
/* Up to 8 independent weight gradients dW = A^T B (each desc trans_a = 1, trans_b = 0, no split-K,
 * its own epilogue, e.g. opa_rowsum for the bias gradient) in one launch: the three Linear weight
 * gradients of the latent / projection MLP's backward (model.py:126-127,90-95) after hvae_mlp_bwd_rows. */
int hvae_gemm_f32_multi(const hvae_gemm_desc* d, int n, void* stream);

/* -------------------------------------------------- decoder (K7, K8, K10) -- */
/* Streaming decoder over all N items, scores never stored:
 *   lse[b] = log sum_i exp(u_b . E_i)         (multinomial normaliser)
 *   O[b,:] = sum_i softmax(u_b E^T)_i E_i     (what d(u) needs; O may be NULL)
 * i.e. one flash-attention style pass with Q = U, K = V = E (E frozen, so no dE).
 * Replaces torch.matmul(u, E.t()) (src/ml/model.py:198), F.log_softmax
 * (src/ml/model.py:281) and their autograd. dtype HVAE_BF16: E is a bf16 copy,
 * U is rounded to bf16, MFMA 32x32x16 bf16 with f32 accumulation, and
 * e_maxnorm (device scalar, hvae_row_norm_max) bounds the scores; HVAE_FP8:
 * block-scaled e4m3 MFMA 32x32x64 (E with one power-of-two scale, U with one
 * per user, P block floating point per user and 64-item tile), e_maxnorm as
 * for bf16 (take it from the image's bf16 part); HVAE_F32: exact-f32 MFMA
 * (e_maxnorm unused). ws >= hvae_decoder_workspace() bytes. */
/* The decoder's image of the frozen embeddings, built once per model:
 *   HVAE_BF16: E rounded to bf16 [N, D], then (at a 256-B aligned offset) the
 *              same values tile-transposed, [ceil(N/32)][D][32] with items in the
 *              MFMA k order, so that both products of the sweep read LDS tiles
 *              with plain 16-B reads;
 *   HVAE_FP8:  the bf16 E [N, D] as above (score bound, exact fixups), then at a
 *              256-B aligned offset ceil(N/64) tiles of [64][D] e4m3 (16-B chunks
 *              XOR-swizzled by item row; tail items 0), then the int exponent ke
 *              of E's scale (E8 = E 2^ke); D in {128, 256, 384, 768};
 *   HVAE_F32:  E itself [N, D].
 * Every `E` argument of the decoder functions below is this image. */
size_t hvae_decoder_image_bytes(int dtype, int64_t N, int64_t D);
int hvae_decoder_image(int dtype, const float* E32, int64_t N, int64_t D, void* out, void* stream);
int hvae_decoder_fwd(int dtype, const float* U, int64_t ldu, const void* E, const float* e_maxnorm,
                     int64_t nb, int64_t N, int64_t D, float* lse, float* O, void* ws,
                     size_t ws_bytes, void* stream);
size_t hvae_decoder_workspace(int dtype, int64_t nb, int64_t N, int64_t D);
/* Users that share one E tile in LDS in the sweep hvae_decoder_fwd / _train plan for (dtype, nb, N, D): every
 * user block streams all of E from L2 into LDS once, so a sweep moves ceil(nb / this) x the image bytes
 * (the L2 -> LDS bound the bench reports beside the MFMA one). Informational; 0 for bad arguments. */
int64_t hvae_decoder_users_per_tile(int dtype, int64_t nb, int64_t N, int64_t D);
/* 1 if this build has a streaming decoder kernel for (dtype, D). */
int hvae_decoder_supported(int dtype, int64_t D);
/* *out = max_i ||E_i||_2 of an fp32 / bf16 [N, D] matrix (computed once: E is frozen). */
int hvae_row_norm_max(int dtype, const void* E, int64_t N, int64_t D, float* out, void* stream);
/* The train-step form: the streaming sweep above plus, in the same finalize
 * launch (one block per user, after the split merge), the sparse half of the
 * loss and of d(u) against the fp32 E32 (see hvae_decoder_bwd). nb = x->nb,
 * N = x->n_items. O may be NULL (kept internal); dU NULL => loss only.
 * If loss3 != NULL the last finalize block also does hvae_loss_finalize
 * (recon_rows, kl_rows, beta -> loss3, accum3) with the same arithmetic; beta_dev
 * (nullable) is a device scalar that replaces beta (hvae_anneal_beta's out2[0]). */
int hvae_decoder_train(int dtype, const float* U, int64_t ldu, const void* E, const float* e_maxnorm,
                       const float* E32, const hvae_csr_batch* x, int64_t D, float grad_scale, float* lse,
                       float* O, float* recon_rows, float* dU, const float* kl_rows, float beta,
                       const float* beta_dev, float* loss3, double* accum3, void* ws, size_t ws_bytes,
                       void* stream);
/* Sparse half of the loss and of d(u), in fp32 against the fp32 E:
 *   recon_rows[b] = n_b * lse[b] - sum_{j in row b} x_bj (u_b . E_j),  n_b = sum_j x_bj
 *   dU[b,:]       = grad_scale * (n_b * O[b,:] - sum_{j in row b} x_bj E_j)
 * (dU / O may be NULL for a loss-only pass, e.g. VAETrainer.validate). */
int hvae_decoder_bwd(const hvae_csr_batch* x, const float* U, int64_t ldu, const float* E32,
                     int64_t D, const float* lse, const float* O, float grad_scale,
                     float* recon_rows, float* dU, void* stream);

/* Materialised-score form of the multinomial loss (the module API path where
 * forward() returns the [nb, N] scores, src/ml/model.py:202-221, 281):
 *   lse[b] = logsumexp(S[b,:]); recon_rows[b] = sum_i X[b,i] * (lse[b] - S[b,i])
 *   dS[b,i] = scale * (n_b * softmax(S[b,:])_i - X[b,i]),  n_b = sum_i X[b,i]  */
int hvae_nll_rows_fwd(const float* S, int64_t lds, const float* X, int64_t ldx, int64_t nb,
                      int64_t N, float* lse, float* recon_rows, void* stream);
int hvae_nll_rows_bwd(const float* S, int64_t lds, const float* X, int64_t ldx, const float* lse,
                      int64_t nb, int64_t N, float scale, float* dS, int64_t ldd, void* stream);

/* total = mean(recon_rows) + beta * mean(kl_rows) -> out3 = {total, recon, kl};
 * accum3 (nullable, fp64) += out3: the epoch sums of VAETrainer.train_epoch
 * (src/ml/train.py:94-96) without a host sync per batch. */
int hvae_loss_finalize(const float* recon_rows, const float* kl_rows, int64_t nb, float beta,
                       float* out3, double* accum3, void* stream);

/* ------------------------------------------------- optimiser (K13, K14) -- */
/* Global L2 norm over a dense flat gradient and an optional row-sparse one,
 * then coef = min(1, max_norm / (norm + 1e-6)):
 * torch.nn.utils.clip_grad_norm_(params, 5.0) at src/ml/train.py:91. The
 * multiplier is applied inside the Adam launches (no extra pass). */
int hvae_clip_grad_norm(const float* g_dense, int64_t n_dense, const hvae_rowgrad* rg, int64_t H,
                        float max_norm, float* norm_out, float* coef_out, void* ws,
                        size_t ws_bytes, void* stream);
size_t hvae_clip_grad_norm_workspace(int64_t n_dense, int64_t cap, int64_t H);
/* The same launch, also advancing the step counters once the norm is known:
 * *step_snap = *step_dev; *step_dev += 1; *boff += advance (boff may be NULL
 * when advance == 0). Give the Adam launches that follow step_dev = step_snap.
 * Saves the separate counter launch at the end of every train step. */
int hvae_clip_grad_norm_step(const float* g_dense, int64_t n_dense, const hvae_rowgrad* rg, int64_t H,
                             float max_norm, float* norm_out, float* coef_out, int64_t* step_dev,
                             int64_t* step_snap, int64_t* boff, int64_t advance, void* ws, size_t ws_bytes,
                             void* stream);

/* torch.optim.Adam (src/ml/train.py:63, 92; single-tensor semantics):
 *   g = coef * grad (+ wd * p); m = lerp(m, g, 1-b1); v = b2 v + (1-b2) g^2
 *   p -= lr / (1 - b1^t) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
 * with t = *step_dev + 1 (the caller advances step_dev afterwards). */
typedef struct hvae_adam {
  double lr, beta1, beta2, eps, weight_decay; /* Python-float values, as torch */
  const int64_t* step_dev; /* completed optimizer steps                        */
  const float* coef_dev;   /* clip multiplier or NULL (=> 1)                    */
} hvae_adam;
/* hvae_clip_grad_norm_step that also records the coming Adam step's scalars
 * (lr / (1 - b1^t), sqrt(1 - b2^t)) for t = *step_dev + 1 in tab[t] (float2 entries, the
 * lazy-Adam step table), computed once in double, so hvae_adam_lazy reads them instead of
 * evaluating pow() in every thread. Pass hvae_adam_lazy step_dev = step_snap as usual. */
int hvae_clip_grad_norm_step_adam(const float* g_dense, int64_t n_dense, const hvae_rowgrad* rg, int64_t H,
                                  float max_norm, float* norm_out, float* coef_out, int64_t* step_dev,
                                  int64_t* step_snap, int64_t* boff, int64_t advance, const hvae_adam* cfg,
                                  float* tab, void* ws, size_t ws_bytes, void* stream);
int hvae_adam_dense(const hvae_adam* cfg, float* p, float* m, float* v, const float* g, int64_t n,
                    void* stream);
/* Dense Adam over the item-major W1t [N, H] whose gradient is row-sparse:
 * untouched rows get g = 0 (their moments still decay, as in torch). */
int hvae_adam_rows(const hvae_adam* cfg, float* p, float* m, float* v, const hvae_rowgrad* rg,
                   int64_t N, int64_t H, void* stream);
/* Both Adam updates of one train step in one launch over the flat parameter
 * buffer: p[0 : N*H] (item-major W1t, row-sparse gradient rg) and
 * p[dense_off : dense_off + n_dense] (dense gradient g_dense). */
int hvae_adam_flat(const hvae_adam* cfg, float* p, float* m, float* v, const hvae_rowgrad* rg, int64_t N,
                   int64_t H, const float* g_dense, int64_t dense_off, int64_t n_dense, void* stream);

/* Exact lazy Adam for the item-major W1t. torch's Adam moves every row every
 * step, with g = 0 for rows outside the batch; those steps are a fixed map per
 * step, so they are deferred and replayed -- the same float operations in the
 * same order, bitwise equal to updating eagerly -- when the row is next needed.
 *   last_step [N] int32: steps already applied to each row (start at 0): bits 0-23 to m and v, bits 24-29 how
 *                        many steps further p is (hvae_adam_lazy_catchup_csr moves p alone when weight_decay
 *                        is 0: the forward reads only p, and the step's hvae_adam_lazy replays m and v itself);
 *                        steps stay below 2^24 (tab_len <= 2^24)
 *   tab [tab_len][2] float: per-step (lr / bc1_t, 1 / sqrt(bc2_t)), entry t written
 *                           by step t's hvae_adam_lazy; tab_len > total steps
 * hvae_adam_lazy: step t = *cfg->step_dev + 1 for the dense segment and for the
 *   gradient rows of rg (their missed steps replayed first).
 * hvae_adam_lazy_catchup: bring rows to *cfg->step_dev completed steps: the
 *   rows listed by `rows` (item_of[0 : *n_unique]; before a batch's forward),
 *   or all N rows when rows == NULL (before anything else reads W1t, m or v).
 * hvae_adam_lazy_catchup_csr: the same for the rows the CSR batch x lists (duplicates
 *   replayed once), without the W1-gradient plan: the plan can then run beside
 *   the forward. Its p is bitwise that of hvae_adam_lazy_catchup on the plan's rows (m and v may stay behind,
 *   as last_step records, until the step's hvae_adam_lazy or a catch-up over all rows). */
/* The hvae_adam_lazy sweep period for N items: ceil(N / period) W1t rows are brought up to date per step, and
 * no replay is longer than period steps (32 from 65,536 items, else 8). */
int hvae_adam_lazy_sweep_period(int64_t N);
int hvae_adam_lazy(const hvae_adam* cfg, float* tab, int64_t tab_len, float* p, float* m, float* v,
                   int32_t* last_step, const hvae_rowgrad* rg, int64_t H, const float* g_dense, int64_t dense_off,
                   int64_t n_dense, void* stream);
int hvae_adam_lazy_catchup(const hvae_adam* cfg, const float* tab, float* p, float* m, float* v,
                           int32_t* last_step, const hvae_rowgrad* rows, int64_t N, int64_t H, void* stream);
int hvae_adam_lazy_catchup_csr(const hvae_adam* cfg, const float* tab, float* p, float* m, float* v,
                               int32_t* last_step, const hvae_csr_batch* x, int64_t H, void* stream);
/* Deferred W1t update (ABI 5; no reference counterpart -- a schedule of the same torch.optim.Adam step,
 * src/ml/train.py:92). hvae_adam_lazy_defer is hvae_adam_lazy except that the gradient rows do not move: the
 * dense segment steps, and each gradient row j is recorded as pending (last_step[j] bit 30, pend->slot_of[j] =
 * its slot in rg, pend->item_of[slot] = j, the step, rg->rows, H, the clip multiplier and the row count in
 * pend->hdr). The rows then take that step later, with hvae_adam_lazy's float operations (bitwise the same
 * parameters and moments):
 *   hvae_adam_lazy_catchup_csr_pending -- hvae_adam_lazy_catchup_csr that also applies the recorded step to the
 *     listed rows that carry it (the next batch's rows, before its forward reads them; *cfg->step_dev must equal
 *     the recorded step, i.e. no clip in between);
 *   hvae_adam_lazy_pending -- every pending row no catch-up has claimed, and the recorded step's sweep range
 *     (hvae_adam_lazy_sweep_period), on any stream, beside the next step's forward; max_rows bounds the rows
 *     recorded (grid size). A second run is a no-op.
 * The recorded gradient rows (rg->rows) must stay as they are until hvae_adam_lazy_pending has run, and it must
 * run before the next hvae_adam_lazy / _defer, a catch-up over all rows, or any other read of W1t, m or v.
 *   pend->slot_of [N] int32, pend->item_of [N] int32, pend->hdr 32 bytes of device memory, zeroed once. */
typedef struct hvae_adam_pend {
  int32_t* slot_of;
  int32_t* item_of;
  void* hdr;
} hvae_adam_pend;
int hvae_adam_lazy_defer(const hvae_adam* cfg, float* tab, int64_t tab_len, float* p, float* m, float* v,
                         int32_t* last_step, const hvae_rowgrad* rg, int64_t H, const float* g_dense,
                         int64_t dense_off, int64_t n_dense, const hvae_adam_pend* pend, void* stream);
int hvae_adam_lazy_catchup_csr_pending(const hvae_adam* cfg, const float* tab, float* p, float* m, float* v,
                                       int32_t* last_step, const hvae_csr_batch* x, int64_t H,
                                       const hvae_adam_pend* pend, void* stream);
int hvae_adam_lazy_pending(const hvae_adam* cfg, const float* tab, float* p, float* m, float* v, int32_t* last_step,
                           int64_t N, int64_t H, int64_t max_rows, const hvae_adam_pend* pend, void* stream);
/* *counter += delta (device-side step/batch counters for graph replay). */
int hvae_counter_add(int64_t* counter, int64_t delta, void* stream);
/* *a += da and, if b != NULL, *b += db, in one launch (end of a train step). */
int hvae_counters_add(int64_t* a, int64_t da, int64_t* b, int64_t db, void* stream);

/* ------------------------------------------------------- data parallel -- */
/* No reference counterpart (the reference trainer is single-device). One rank's share of a
 * data-parallel step: its batch x compacted into row_ptr_out[0..nb] (int32 offsets from 0; [nb] = nnz),
 * col_out[0..cap) and vals_out[0..cap) = scale * vals. Ranks all-gather these packets with their da [nb, H]
 * and rebuild the union batch's first-layer row gradient with hvae_w1_rowgrad (hvae/dist.py). cap is sized
 * from the host CSR (the batch's largest possible nnz); a batch with more entries keeps its first cap (row
 * pointers clamped, so the packet stays a valid CSR) and sets *overflow = 1 (nullable), on which the host
 * raises. */
int hvae_csr_batch_pack(const hvae_csr_batch* x, float scale, int32_t* row_ptr_out, int32_t* col_out,
                        float* vals_out, int64_t cap, int32_t* overflow, void* stream);

/* ------------------------------------------------------------ eval (K16) -- */
/* scores[r, c] = U[user_row[r], :] . E32[cand[r, c], :]   (fp32)
 * The 99-negative protocol of RecommendationEvaluator.evaluate_user_with_negatives
 * (src/ml/evaluate.py:149-185), batched over test rows. */
int hvae_score_candidates(const float* U, int64_t ldu, const int32_t* user_row, const float* E32,
                          int64_t D, const int32_t* cand, int64_t R, int64_t C, float* scores,
                          void* stream);
/* rank[r] = #{c : scores[r,c] > scores[r,0]} + #{c > 0 : scores[r,c] == scores[r,0]}
 * i.e. the position of candidate 0 in a stable descending-then-reversed order
 * (candidates[np.argsort(s)[::-1]] with argsort stable). */
int hvae_rank_first(const float* scores, int64_t R, int64_t C, int32_t* rank, void* stream);
/* Exact top-K per row of a score matrix [R, N] (ld), seen items of row r
 * (exclude, nullable) masked to -inf first, in place in `scores` (get_user_recommendations,
 * src/ml/evaluate.py:137-147; HybridVAE.recommend, src/ml/model.py:236-256).
 * Order: score descending, ties by larger item index first. K <= 64. */
int hvae_topk(const float* scores, int64_t R, int64_t N, int64_t ld, const hvae_csr_batch* exclude,
              int64_t K, int32_t* idx, float* val, void* stream);

/* Fused exact top-K over all N items without the [R, N] score matrix (full-ranking
 * eval and the /recommend core: RecommendationEvaluator.get_user_recommendations,
 * src/ml/evaluate.py:137-147; HybridVAE.recommend, src/ml/model.py:236-256; the
 * /recommend handler, src/api/server.py:115-183, scores -> seen masked to -inf ->
 * np.argsort(scores)[::-1][:top_k]). U [R, ldu] fp32 user vectors, E_bf16 the bf16
 * [N, D] image (hvae_decoder_image's first part), E32 the fp32 [N, D] embeddings,
 * e32_maxnorm = max_i ||E32_i|| (device scalar). A bf16 MFMA sweep keeps every item
 * that can still be in a user's top-(K + |seen|) by a provable bound, then the
 * candidates are rescored in fp32 and ordered (score desc, item desc), as hvae_topk.
 * idx / val [R, K]; flag[r] = 1 marks rows the fused path could not certify (candidate
 * overflow, fewer than K unseen items, K + |seen| > 256): the caller ranks those
 * exactly (hvae_gemm_f32 + hvae_topk). D in {64, 128, 256, 384, 512, 768}, K <= 256. */
size_t hvae_topk_fused_workspace(int64_t R, int64_t N, int64_t D, int64_t K);
int hvae_topk_fused(const float* U, int64_t ldu, const void* E_bf16, const float* E32,
                    const float* e32_maxnorm, int64_t N, int64_t D, const hvae_csr_batch* exclude,
                    int64_t R, int64_t K, int32_t* idx, float* val, int32_t* flag, void* ws,
                    size_t ws_bytes, void* stream);

/* The 99-negative protocol's negatives, host only, draw for draw numpy's: per test row r, the items
 * neither in row users[r] of the training CSR (row_ptr / col_idx) nor tests[r], ascending ("available",
 * src/ml/evaluate.py:159-165); all of them when fewer than n_neg (counts[r] = that number, no draw), else
 * np.random.choice(available, n_neg, replace=False) (:166-170) = available[permutation(len)[:n_neg]] of the
 * legacy RandomState, counts[r] = n_neg. n_users = the CSR's row count (row_ptr has n_users + 1 entries): every
 * users[r] must lie in [0, n_users). mt_key [624] / mt_pos: numpy's MT19937 state
 * (np.random.get_state()[1:3]), advanced in place as the per-row choices in row order would leave it.
 * out [n_rows, n_neg], n_neg <= 32767. Threads: the caller's plus up to 8 workers (HVAE_NEG_WORKERS overrides the count);
 * AVX-512 where the host has it (HVAE_NEG_SCALAR=1 forces the scalar form; the results are identical). */
int hvae_negatives_legacy(uint32_t* mt_key, int32_t* mt_pos, const int64_t* row_ptr, int64_t n_users,
                          const int32_t* col_idx, int64_t n_items, const int32_t* users, const int32_t* tests, int64_t n_rows,
                          int32_t n_neg, int32_t* out, int32_t* counts);

/* ---------------------------------------------------- data artifacts (host) -- */
/* A host CSR plus the file's users, allocated by hvae_read_interactions and
 * released by hvae_host_csr_free. */
typedef struct hvae_host_csr {
  int64_t* row_ptr;     /* [n_rows + 1]                                        */
  int32_t* col_idx;     /* [nnz], ascending within a row                       */
  float* vals;          /* [nnz], duplicate (user, item) rows summed            */
  int64_t n_rows, n_cols, nnz;
  int64_t* users;       /* [n_users_seen] users of the file, first appearance   */
  int64_t n_users_seen;
  int64_t n_records;    /* data rows read                                       */
} hvae_host_csr;
/* train.csv / val.csv -> CSR (load_training_data + _build_matrix +
 * get_user_indices_from_df, src/ml/train.py:153-193): rows with
 * binary_rating == 1 when positives_only and the column exists, user_id /
 * asin looked up in the mappings' keys (user_keys: n_users NUL-separated keys,
 * key i <-> index i; likewise items), shape (n_users, n_items). One pass over
 * the memory-mapped file, RFC 4180 quoting. A positive row whose user or item
 * the mappings do not know is an error (HVAE_ERR_ARG), as in the reference.
 * Host only: no device work. */
int hvae_read_interactions(const char* csv_path, const char* user_keys, int64_t user_keys_len, int64_t n_users,
                           const char* item_keys, int64_t item_keys_len, int64_t n_items, int positives_only,
                           hvae_host_csr* out);
void hvae_host_csr_free(hvae_host_csr* c);

/* fp32 -> bf16 (round to nearest even) copy of the frozen embeddings. */
int hvae_cast_bf16(const float* x, void* y, int64_t n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* HVAE_H_ */
