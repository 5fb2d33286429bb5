/*
 * smmd_hip.h -- C ABI of libsmmd_hip.so, the MI355X (gfx950) hot path of the
 * Scaled-MMD-GAN training step.
 *
 * Plain pointers and sizes only.  Every device buffer (inputs, outputs and
 * workspace) is owned by the caller; the library never allocates or frees
 * device memory and never synchronises the stream.  Every entry point is
 * stream-ordered on the caller's stream (a hipStream_t passed as void*; NULL
 * = the legacy default stream) and is safe to capture in a hipGraph.
 * Reductions use a fixed order, so results are bit-identical run to run for
 * the same shapes.  No entry point throws or aborts: errors come back as an
 * smmd_status code.
 *
 * Which reference interface each entry point replaces is cited next to it
 * (paths relative to the playHing/Scaled-MMD-GAN tree).
 */
#ifndef SMMD_HIP_H
#define SMMD_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    SMMD_OK = 0,
    SMMD_EINVAL = 1,        /* bad argument (shape, range, NULL pointer)      */
    SMMD_EHIP = 2,          /* a HIP launch / runtime error                   */
    SMMD_EWORKSPACE = 3,    /* workspace NULL or smaller than *_workspace_bytes */
    SMMD_EUNSUPPORTED = 4   /* valid request this build does not implement    */
} smmd_status;

typedef void *smmd_stream_t;   /* hipStream_t */

/* Kernel family of gan/core/mmd.py:18-188, selected in the reference by
 * getattr(mmd, '_%s_kernel' % config.kernel) (gan/core/smmd.py:11).       */
typedef enum {
    SMMD_KIND_RBF = 0,       /* sum_k wt_k exp(-D2 / (2 sigma_k^2))   mmd.py:55-116  */
    SMMD_KIND_RQ = 1,        /* sum_k wt_k (1 + D2/(2 a_k))^-a_k + add_dot <x,y>   mmd.py:143-188 */
    SMMD_KIND_DISTANCE = 2,  /* ms(|x|^2)+ms(|y|^2)-ms(raw D2)       mmd.py:18-37   */
    SMMD_KIND_DOT = 3        /* <x,y>                                mmd.py:44-52   */
} smmd_kernel_kind;

#define SMMD_MAX_TERMS 8

typedef struct {
    int32_t kind;                   /* smmd_kernel_kind                          */
    int32_t n_terms;                /* RBF/RQ mixture size, 1..SMMD_MAX_TERMS    */
    double param[SMMD_MAX_TERMS];   /* RBF: sigma_k ; RQ: alpha_k                */
    double wt[SMMD_MAX_TERMS];      /* mixture weights                           */
    double add_dot;                 /* RQ only (mix_rq_*dot variants)            */
    int32_t tanh_inputs;            /* tanh_mix_rq / tanh_distance (mmd.py:40,139) */
    int32_t has_const_diag;         /* 1: subtract m*const_diag; 0: the trace   */
    double const_diag;              /* mmd.py:82, :116, :188 ("False" -> 0 flag) */
} smmd_kernel_desc;

const char *smmd_status_string(smmd_status s);
int smmd_abi_version(void);         /* bumped on any ABI change (2: Gram/poly,
                                       3: smmd_sn_layer.fold, 4: smmd_adam_flat_ex,
                                       5: smmd_conv3x3_thin*,
                                       6: smmd_mask_pool2*, smmd_up_add,
                                       smmd_bn_relu_fwd, 7: smmd_smmd_loss_fwd/bwd,
                                       smmd_source_hash, smmd_sn_grad_stats,
                                       smmd_adam_flat_sn2, smmd_bn_relu_fwd_save / _bwd,
                                       8: smmd_wino3x3_*, smmd_wino4x4s2*,
                                       smmd_wino3x3_wgrad*, 9: smmd_wino4x4s2_wgrad*,
                                       smmd_wino3x3_filter_sn, smmd_wino4x4s2(t)_filter_sn,
                                       smmd_sn_clip_g, 10: smmd_wino3x3_conv2*,
                                       smmd_wino4x4s2_conv2*, 11: smmd_fold_up_weight,
                                       smmd_conv1x1*, 12: smmd_wino4x4s2t_conv_mask,
                                       smmd_row_lrelu_sum, smmd_row_lrelu_bcast,
                                       13: the weight gradients' *_acc forms,
                                       14: smmd_wino3x3_conv_mask,
                                       15: smmd_wino4x4s2_conv_acc,
                                       16: smmd_conv1x1_t,
                                       17: smmd_smmd_loss_fwd_gathered,
                                       smmd_smmd_loss_bwd_ex) */
const char *smmd_source_hash(void); /* first 16 hex digits of the SHA-256 of the
                                       sources this binary was built from
                                       (csrc .hip and .hpp files in byte order,
                                       then this header): gan.core._lib refuses
                                       a binary older than its sources */

/* ---------------------------------------------------------------------------
 * Fused pairwise MMD^2 (forward + unit gradient).
 * Replaces mmd.mmd2(mmd._<kind>_kernel(X, Y))  (gan/core/mmd.py:55-82 and
 * :194-220, called from gan/core/smmd.py:11-15) together with TF's autodiff of
 * it: the N x N kernel matrices are never materialised.
 *
 * X [m, d], Y [n, d]: row-major fp32 feature matrices (critic outputs d_G and
 * d_images, gan/core/model.py:307-311).  m, n are the GLOBAL batch sizes that
 * define the estimator's weights.  This call evaluates the rows
 * [x_begin, x_end) of X and [y_begin, y_end) of Y against all m + n columns
 * (the whole range for one GPU; a rank's shard in the all-gather mode).
 *
 * out_sums[8] (device, fp32), partial over the evaluated rows:
 *   [0] sum K_XX  [1] sum K_XY  [2] sum K_YY  [3] trace K_XX  [4] trace K_YY
 *   [5] sum K_YX (only with a gradient request)   [6], [7] zero
 * out_mmd2 (device, 1 float, may be NULL): the estimator from out_sums; equal
 *   to the reference's value only when the rows cover everything.
 * grad_x [x_end-x_begin, d], grad_y [y_end-y_begin, d] (device, may both be
 *   NULL): d mmd2 / d X[row], d mmd2 / d Y[row] for the evaluated rows, taken
 *   against ALL columns (TF tie rule of tf.maximum: gradient passes at 0).
 * ws: zero-filled at allocation, at least smmd_mmd2_workspace_bytes(); the
 *   library leaves it zero-filled again after every call.
 * ------------------------------------------------------------------------- */
size_t smmd_mmd2_workspace_bytes(int m, int n, int d);

smmd_status smmd_mmd2_fwd(const smmd_kernel_desc *desc,
                          const float *X, int m, const float *Y, int n, int d,
                          int biased,
                          int x_begin, int x_end, int y_begin, int y_end,
                          float *out_sums, float *out_mmd2,
                          float *grad_x, float *grad_y,
                          void *ws, size_t ws_bytes, smmd_stream_t stream);

/* The estimator of gan/core/mmd.py:199-220 from (all-reduced) sums:
 * sums[8] as above -> out_mmd2[1].  Used by the all-gather mode after the
 * RCCL all_reduce of the per-rank partial sums. */
smmd_status smmd_mmd2_combine(const smmd_kernel_desc *desc, const float *sums,
                              int m, int n, int biased, float *out_mmd2,
                              smmd_stream_t stream);

/* ---------------------------------------------------------------------------
 * Witness function of the gradient penalty (gan/core/model.py:336-339):
 *   w_i = mean_j K(H_i, R_j) - mean_j K(H_i, F_j)   (K_XY_only=True kernels)
 * out_w [b] (may be NULL), out_dH [b, d] = d(sum_i w_i)/dH (may be NULL).
 * H [b, d], R [nr, d], F [nf, d].
 * smmd_witness_bwd: the vector-Jacobian product of out_dH, i.e. given
 * gdH [b, d] (= dL/d out_dH) it returns dL/dH [b, d], dL/dR [nr, d],
 * dL/dF [nf, d] -- the second-order term the penalty's parameter gradient
 * needs (gan/core/model.py:339-345).
 * ------------------------------------------------------------------------- */
smmd_status smmd_witness_fwd(const smmd_kernel_desc *desc,
                             const float *H, int b, const float *R, int nr,
                             const float *F, int nf, int d,
                             float *out_w, float *out_dH, smmd_stream_t stream);

smmd_status smmd_witness_bwd(const smmd_kernel_desc *desc,
                             const float *H, int b, const float *R, int nr,
                             const float *F, int nf, int d, const float *gdH,
                             float *gH, float *gR, float *gF,
                             smmd_stream_t stream);

/* ---------------------------------------------------------------------------
 * Scaling regulariser (SMMD / SWGAN).
 * Replaces ops.squared_norm_jacobian (gan/core/ops.py:228-233),
 * MMD_GAN.add_scaling (gan/core/model.py:366-403) and the apply_scaling
 * hooks (gan/core/smmd.py:21-23, :40-42).
 *
 * smmd_scaled_loss_fwd: jac [n_cols * b, per_sample]: for each critic output
 *   column c the gradient d(sum_b D(x_b)_c)/dx of this caller's b samples
 *   (ops.py:230-232 stacks them column-major over c).  feat [b, dof] (critic
 *   output; read only when variant == 1 'value_and_grad').
 *   b_total: the normaliser of the means (global batch in the all-gather
 *   mode, else b; <= 0 means b).  base_loss [1]: mmd2 (SMMD) or
 *   mean(images) - mean(G) (SWGAN).
 *   out (device, 8 floats): [0] g_loss [1] d_loss [2] scale
 *   [3] J = sum_b ||grad||^2 / b_total  [4] norm_discriminator
 *   [5] base_loss  [6],[7] zero.
 *   per_sample [b] (may be NULL): sum_c ||d D_c / d x_b||^2.
 *   variant: 0 'grad', 1 'value_and_grad' (model.py:387-390).
 *   sqrt_scale: 0 SMMD (g_loss = base*scale), 1 SWGAN (base*sqrt(scale)).
 * smmd_scaled_loss_finalize: recompute out[0..2] from out[3..5] (after the
 *   caller all-reduced out[3], out[4] and replaced out[5]).
 * smmd_scaled_loss_bwd: given dL/dg_loss (device scalar, NULL = 1) writes
 *   d_base [1] (may be NULL), gjac [n_cols*b, per_sample] and gfeat [b, dof]
 *   (only when variant == 1).
 * ------------------------------------------------------------------------- */
size_t smmd_scaled_loss_workspace_bytes(int rows, int64_t per_sample);

smmd_status smmd_scaled_loss_fwd(const float *jac, int n_cols, int b, int b_total,
                                 int64_t per_sample, const float *feat, int dof,
                                 const float *base_loss, float sc, int variant,
                                 int sqrt_scale, float *out, float *per_sample_out,
                                 void *ws, size_t ws_bytes, smmd_stream_t stream);

smmd_status smmd_scaled_loss_finalize(float *out, float sc, int variant, int sqrt_scale,
                                      smmd_stream_t stream);

smmd_status smmd_scaled_loss_bwd(const float *jac, int n_cols, int b, int b_total,
                                 int64_t per_sample, const float *feat, int dof,
                                 const float *fwd_out, float sc, int variant,
                                 int sqrt_scale, const float *g_loss_grad,
                                 float *d_base, float *gjac, float *gfeat,
                                 smmd_stream_t stream);

/* ---------------------------------------------------------------------------
 * The SMMD critic loss in ONE launch: g_loss = mmd2(kernel(X, Y)) * scale
 * (gan/core/smmd.py:10-23 set_loss + apply_scaling, model.py:366-403
 * add_scaling) -- smmd_mmd2_fwd's tile sweep over all rows (one process, or
 * a tower: b_total = b) and smmd_scaled_loss_fwd's squared-norm pass of
 * the Jacobian in one grid; the last block to finish forms the estimator's
 * scaled loss with base = out_mmd2.  Outputs as those two calls
 * (out_sums, out_mmd2, grad_x / grad_y = d mmd2 / dX, dY; out[8] of
 * smmd_scaled_loss_fwd).  ws: smmd_mmd2_workspace_bytes(m, n, d); loss_ws:
 * smmd_scaled_loss_workspace_bytes(n_cols * b, per_sample).  Returns
 * SMMD_EUNSUPPORTED where smmd_mmd2_fwd would not take its 2-D tiled path
 * (d > 8, or the MFMA Gram path): the caller then makes the two calls.
 *
 * smmd_smmd_loss_bwd: the backward of both outputs in one launch:
 *   dX, dY = (g_mmd2 + g_loss f) * grad_x, grad_y  (f = scale, or sqrt(scale)
 *   with sqrt_scale), gjac and gfeat as smmd_scaled_loss_bwd with dL/dg_loss
 *   = g_loss_grad (device scalar, required); g_mmd2_grad may be NULL (0);
 *   gjac / gfeat may be NULL (not written: the Jacobian is a constant).
 * ------------------------------------------------------------------------- */
smmd_status smmd_smmd_loss_fwd(const smmd_kernel_desc *desc, const float *X, int m,
                               const float *Y, int n, int d, int biased, const float *jac,
                               int n_cols, int b, int64_t per_sample, const float *feat, int dof,
                               float sc, int variant, int sqrt_scale, float *out_sums,
                               float *out_mmd2, float *grad_x, float *grad_y, float *out,
                               float *per_sample_out, void *ws, size_t ws_bytes, void *loss_ws,
                               size_t loss_ws_bytes, smmd_stream_t stream);

smmd_status smmd_smmd_loss_bwd(const float *jac, int n_cols, int b, int64_t per_sample,
                               const float *feat, int dof, const float *fwd_out, float sc,
                               int variant, int sqrt_scale, const float *g_loss_grad,
                               const float *g_mmd2_grad, const float *gx_unit, int m,
                               const float *gy_unit, int n, int d, float *gjac, float *gfeat,
                               float *dX, float *dY, smmd_stream_t stream);

/* The all-gather ('global') data-parallel mode's fused loss (ABI 17).
 * Replaces, for the data-parallel SMMD step, the same reference code as
 * smmd_smmd_loss_fwd (smmd.py:10-23, model.py:366-403 over the global batch
 * of model.py:187-216) when every rank sweeps the gathered rows whole:
 * X [m, d], Y [n, d] are the GLOBAL gathered feature rows, and J / nD are
 * not reduced from a Jacobian here but summed in rank order from the
 * gathered per-rank partials stats[r * stats_stride + 0] (J share) and
 * [r * stats_stride + 1] (nD share), r < world -- each rank's
 * smmd_scaled_loss_fwd out[3..4] over its own rows with b_total = the global
 * batch (gan.core.ops.scaling_partials), carried by the feature all-gather.
 * Outputs as smmd_smmd_loss_fwd (grad_x / grad_y for ALL m + n rows; out[8]
 * with J, nD the summed values; per-sample norms are not formed).  loss_ws:
 * at least smmd_scaled_loss_workspace_bytes(1, 1) (its arrival ticket).
 * Returns SMMD_EUNSUPPORTED where smmd_smmd_loss_fwd would.
 *
 * smmd_smmd_loss_bwd_ex: smmd_smmd_loss_bwd with the Jacobian's normaliser
 *   b_total (the global batch; b = this rank's samples in jac): gjac =
 *   dL/dQ * 2 jac / b_total.  smmd_smmd_loss_bwd is this with b_total = b.
 *   gx_unit / gy_unit: this rank's rows of the forward's unit gradients. */
smmd_status smmd_smmd_loss_fwd_gathered(const smmd_kernel_desc *desc, const float *X, int m,
                                        const float *Y, int n, int d, int biased,
                                        const float *stats, int world, int stats_stride,
                                        float sc, int variant, int sqrt_scale, float *out_sums,
                                        float *out_mmd2, float *grad_x, float *grad_y, float *out,
                                        void *ws, size_t ws_bytes, void *loss_ws,
                                        size_t loss_ws_bytes, smmd_stream_t stream);

smmd_status smmd_smmd_loss_bwd_ex(const float *jac, int n_cols, int b, int b_total,
                                  int64_t per_sample, const float *feat, int dof,
                                  const float *fwd_out, float sc, int variant, int sqrt_scale,
                                  const float *g_loss_grad, const float *g_mmd2_grad,
                                  const float *gx_unit, int m, const float *gy_unit, int n, int d,
                                  float *gjac, float *gfeat, float *dX, float *dY,
                                  smmd_stream_t stream);

/* ---------------------------------------------------------------------------
 * Spectral normalisation, all layers of a network in one set of launches.
 * Replaces sn.spectral_normed_weight (gan/core/sn.py:16-59) and the s * W_bar
 * product of the SN layer wrappers (gan/core/snops.py:82-84, :118-120,
 * :180-183; gan/core/resnet/ops/conv2d.py:29-33).
 *
 * Layout: W is the layer weight flattened to [N = out channels, K] row-major
 * (a torch conv/linear weight as stored); the reference reshapes to
 * [K', N] (sn.py:19) with K' a permutation of K, which leaves sigma and u
 * unchanged and permutes v.
 * Power iteration (num_iters times, sn.py:24-35):
 *   v = l2n(W^T u), u' = l2n(W v), l2n(x) = x / (||x|| + eps);
 *   sigma = (W v) . u'  (sn.py:42);   W_eff = s * (W / sigma)  (snops.py:84).
 * ------------------------------------------------------------------------- */
#define SMMD_SN_MAX_LAYERS 32

typedef struct {
    const float *W;      /* [N, K]                                            */
    float *W_eff;        /* [N, K] out: s * W / sigma (NULL: not written);    */
                         /* fold = 1: [N, K/9, 4, 4], see below               */
    float *u;            /* [N] in: current u ; out: u' when update_u         */
    float *v;            /* [K] out: v (normalised)                           */
    float *sigma;        /* [1] out                                           */
    const float *s;      /* [1] SN scale (NULL -> 1.0), snops.py:82           */
    const float *G;      /* bwd: dL/dW_eff, W_eff's shape                     */
    float *gW;           /* bwd: [N, K] out dL/dW                             */
    float *gs;           /* bwd: [1] out dL/ds (NULL: not written)            */
    int32_t N;
    int32_t K;
    /* fold = 1: the layer is the 3x3 stride-1 conv of a ConvMeanPool
     * (gan/core/resnet/block.py:63-66), W [N, C, 3, 3] (K = 9 C, 16-byte
     * aligned).  W_eff is then written directly as the pool-folded filter
     * W'[n, c] (4 x 4) = 1/4 sum_{a,b in {0,1}} W_bar[n, c][. - a, . - b],
     * W_bar = s W / sigma, so conv(x, W', stride 2) = meanpool2(conv(x, W_bar));
     * the backward's G is dL/dW' and its adjoint is applied on the fly.
     * fold = 0: W_eff = s W / sigma as is. */
    int32_t fold;
} smmd_sn_layer;

size_t smmd_sn_workspace_bytes(const smmd_sn_layer *layers, int n_layers);

/* update_u = 1 mirrors update_collection=None (u.assign(u'), sn.py:39-46);
 * 0 mirrors "NO_OPS" (u left untouched). layers[] is a HOST array read during
 * the call; the pointers in it are device pointers. n_layers <= SMMD_SN_MAX_LAYERS.
 * ws: zero-filled at allocation and then reused as is (its first 256 bytes
 * are reserved). */
smmd_status smmd_sn_power_iter(const smmd_sn_layer *layers, int n_layers,
                               int num_iters, float eps, int update_u,
                               void *ws, size_t ws_bytes, smmd_stream_t stream);

/* flags = SMMD_SN_P1_READY: the column partials of the first iteration (u^T W
 * per 32-row tile) are already in ws, written by smmd_adam_flat_sn from the
 * current W and u; the call skips that pass (one read of every W).  The
 * caller guarantees neither W nor u changed since.  flags = 0 is
 * smmd_sn_power_iter. */
#define SMMD_SN_P1_READY 1
smmd_status smmd_sn_power_iter_ex(const smmd_sn_layer *layers, int n_layers,
                                  int num_iters, float eps, int update_u, int flags,
                                  void *ws, size_t ws_bytes, smmd_stream_t stream);

/* dL/dW = (s/sigma) (G - (<G,W>/sigma) u' v^T),  dL/ds = <G,W>/sigma,
 * u', v, sigma from the last smmd_sn_power_iter (stop_gradient, sn.py:32-34);
 * ws must be the workspace that call used (it holds u'), and layers[] the
 * same array of layers (the workspace is carved by it): a layer whose G is
 * NULL is skipped, so a subset (one gradient bucket's layers) is the same
 * array with the other layers' G NULL. */
smmd_status smmd_sn_weight_bwd(const smmd_sn_layer *layers, int n_layers,
                               void *ws, size_t ws_bytes, smmd_stream_t stream);

/* The backward WITHOUT forming dL/dW (the G-direct update, one process):
 * from G (layers[].G, dL/dW_eff or dL/dW' of a fold layer) and W it reduces
 * d = <G, W> (the sums and order of smmd_sn_weight_bwd), ||G||^2 and
 * u'^T G v, writes gs = d / sigma (layers[].gs, may be NULL) and keeps per
 * layer in ws the record {coef = s d / sigma^2, ||dL/dW||^2 (analytic:
 * (s/sigma)^2 ||G||^2 - 2 (s/sigma) coef u'^T G v + coef^2 ||u'||^2 ||v||^2),
 * sigma, s} that smmd_adam_flat_sn2 with SMMD_ADAM_SN_GDIRECT reads.  G must
 * stay alive (unchanged) until that update has run.  A layer whose G is NULL
 * is skipped (its record untouched): one gradient bucket's layers. */
smmd_status smmd_sn_grad_stats(const smmd_sn_layer *layers, int n_layers,
                               void *ws, size_t ws_bytes, smmd_stream_t stream);

/* The per-rank clip of the data-parallel G-direct tower mode: for each layer
 * with G (non-fold: G has W's shape) G *= clip / max(||dL/dW||, clip), the
 * norm from its smmd_sn_grad_stats record (dL/dW is linear in G: this is
 * tf.clip_by_norm of the rank's dL/dW, gan/core/model.py:449-455), and
 * gs *= clip / max(|gs|, clip) (the scale's own clip).  Layers with G NULL
 * are skipped (smmd_sn_grad_stats skips them too). */
smmd_status smmd_sn_clip_g(const smmd_sn_layer *layers, int n_layers, float clip, void *ws,
                           size_t ws_bytes, smmd_stream_t stream);

/* ---------------------------------------------------------------------------
 * Materialised kernel matrix K(A, B) [na, nb] (row-major) and its backward
 * (gA = dL/dA, gB = dL/dB from G = dL/dK; either output may be NULL).
 * Serves the tuple-returning API of mmd._<kind>_kernel (gan/core/mmd.py:18-188)
 * and its K_XY_only form; the training loss never calls it.
 * ------------------------------------------------------------------------- */
smmd_status smmd_kernel_matrix_fwd(const smmd_kernel_desc *desc, const float *A, int na,
                                   const float *B, int nb, int d, float *out,
                                   smmd_stream_t stream);

smmd_status smmd_kernel_matrix_bwd(const smmd_kernel_desc *desc, const float *A, int na,
                                   const float *B, int nb, int d, const float *G,
                                   float *gA, float *gB, smmd_stream_t stream);

/* ---------------------------------------------------------------------------
 * TF-semantics gradient clip and Adam over the tensors of one flat buffer:
 * tensor i occupies elements [offsets[i], offsets[i+1]) (offsets: HOST array
 * of n_tensors + 1 entries).
 * Replaces clip_by_norm in MMD_GAN.compute_grads (gan/core/model.py:444-456)
 * and tf.train.AdamOptimizer.apply_gradients (model.py:405-412, :458-468).
 *  smmd_clip_by_norm_flat: g <- g * clip * min(rsqrt(sum g^2), 1/clip), per
 *    tensor, in place (the per-tower clip before the tower mean).
 *  smmd_adam_flat: g' = grad_scale * g, then (clip_norm > 0) the same clip,
 *    then Eigen's ApplyAdam: m += (g'-m)(1-b1); v += (g'^2-v)(1-b2);
 *    p -= lr_t m / (sqrt(v) + eps), lr_t = lr sqrt(1-b2^step)/(1-b1^step).
 * ------------------------------------------------------------------------- */
size_t smmd_opt_workspace_bytes(const int64_t *offsets, int n_tensors);

smmd_status smmd_clip_by_norm_flat(float *grad, const int64_t *offsets, int n_tensors,
                                   float clip_norm, void *ws, size_t ws_bytes,
                                   smmd_stream_t stream);

smmd_status smmd_adam_flat(float *param, const float *grad, float *m, float *v,
                           const int64_t *offsets, int n_tensors, float grad_scale,
                           float clip_norm, float lr, float beta1, float beta2, float eps,
                           int64_t step, void *ws, size_t ws_bytes, smmd_stream_t stream);

/* smmd_adam_flat whose SN weight tensors are updated tile by tile together
 * with the first pass of the next power iteration (layers[i].W must be tensor
 * sn_tensor[i] of param, layers[i].u the u the next smmd_sn_power_iter_ex
 * reads; sn_ws that call's workspace).  Same bits as smmd_adam_flat followed
 * by that pass, in one launch after the norm pass.  n_tensors <= 96 and
 * n_layers <= 16 (else SMMD_EUNSUPPORTED: use smmd_adam_flat). */
smmd_status smmd_adam_flat_sn(float *param, const float *grad, float *m, float *v,
                              const int64_t *offsets, int n_tensors, float grad_scale,
                              float clip_norm, float lr, float beta1, float beta2, float eps,
                              int64_t step, void *ws, size_t ws_bytes,
                              const smmd_sn_layer *layers, const int32_t *sn_tensor,
                              int n_layers, void *sn_ws, size_t sn_ws_bytes,
                              smmd_stream_t stream);

/* smmd_adam_flat / smmd_adam_flat_sn (n_layers = 0: the plain update) with the
 * bias-corrected step size lr_t = lr sqrt(1 - b2^t) / (1 - b1^t) read from
 * DEVICE memory (lr_t [1] fp32) when the kernels execute, instead of lr and
 * step passed by value: a HIP graph capturing the update then replays every
 * step with the value the host writes before the replay (model.py:405-412,
 * :458-468 semantics unchanged). */
smmd_status smmd_adam_flat_ex(float *param, const float *grad, float *m, float *v,
                              const int64_t *offsets, int n_tensors, float grad_scale,
                              float clip_norm, const float *lr_t, float beta1, float beta2,
                              float eps, void *ws, size_t ws_bytes,
                              const smmd_sn_layer *layers, const int32_t *sn_tensor,
                              int n_layers, void *sn_ws, size_t sn_ws_bytes,
                              smmd_stream_t stream);

/* smmd_adam_flat_sn and smmd_adam_flat_ex in one entry, with flags:
 * lr_t != NULL reads the step size from that device scalar (graph replay;
 * lr and step unused), else lr_t = lr sqrt(1 - b2^step) / (1 - b1^step).
 * flags = SMMD_ADAM_SN_GDIRECT: the SN weights' gradients are NOT in grad:
 * each is formed in the update from layers[].G / .fold / .v and the record
 * smmd_sn_grad_stats left in sn_ws, dL/dW = (s G)/sigma - coef u' v^T, and
 * clipped by the record's norm; the norm pass skips those tensors.  One read
 * of G replaces dL/dW's write, its accumulation into grad and its two reads. */
#define SMMD_ADAM_SN_GDIRECT 1
smmd_status smmd_adam_flat_sn2(float *param, const float *grad, float *m, float *v,
                               const int64_t *offsets, int n_tensors, float grad_scale,
                               float clip_norm, float lr, float beta1, float beta2, float eps,
                               int64_t step, const float *lr_t, void *ws, size_t ws_bytes,
                               const smmd_sn_layer *layers, const int32_t *sn_tensor,
                               int n_layers, void *sn_ws, size_t sn_ws_bytes, int flags,
                               smmd_stream_t stream);

/* ---------------------------------------------------------------------------
 * Polynomial-kernel MMD statistics of the KID scorer and the 3-sample LR
 * scheduler, on the f32 matrix cores.
 * Replaces polynomial_kernel + _mmd2_and_variance (gan/compute_scores.py:
 * 232-335, via polynomial_mmd_averages :211-229 from gan/utils/scorer.py:103)
 * and _np_get_sums / _np_diff_mmd2_and_ratio_from_sums (gan/core/mmd.py:
 * 429-539, from gan/utils/scorer.py:124-162).
 *
 * smmd_poly_kernel_sums: K = (gamma A B^T + coef0)^degree for A [na, dim],
 *   B [nb, dim] (row-major fp32; K is never materialised).  Outputs (device,
 *   double, each may be NULL): row_sums [na] = K 1, col_sums [nb] = K^T 1,
 *   diag [min(na, nb)] = K_ii, stats [4] = { sum K, sum K^2, sum_i K_ii,
 *   sum_i K_ii^2 }.  degree 1..8.  ws: zero-filled at allocation.
 * A "sums record" below is (rows, cols, diag, stats) of one such call.
 * smmd_poly_mmd2_var: mmd2 and its variance estimate (_mmd2_and_variance)
 *   from the XX, YY and XY records (m = na = nb): estimator 0 'unbiased',
 *   1 'biased', 2 'u-statistic'; var_at_m <= 0 means m.
 *   out [2] (device, double) = { mmd2, var_est }.
 * smmd_poly_diff_ratio: mmd2(X,Y) - mmd2(X,Z) and its ratio to the estimated
 *   std (the 3-sample test statistic, _np_diff_mmd2_and_ratio_from_sums) from
 *   the YY, XY, ZZ, XZ records.  out [2] = { mmd2_diff, ratio }.
 * ------------------------------------------------------------------------- */
size_t smmd_poly_sums_workspace_bytes(int na, int nb, int dim);

smmd_status smmd_poly_kernel_sums(const float *A, int na, const float *B, int nb, int dim,
                                  double gamma, double coef0, int degree,
                                  double *row_sums, double *col_sums, double *diag,
                                  double *stats, void *ws, size_t ws_bytes,
                                  smmd_stream_t stream);

typedef struct {
    const double *rows;   /* [m] */
    const double *cols;   /* [m] */
    const double *diag;   /* [m] */
    const double *stats;  /* [4] */
} smmd_poly_sums;

smmd_status smmd_poly_mmd2_var(const smmd_poly_sums *xx, const smmd_poly_sums *yy,
                               const smmd_poly_sums *xy, int m, double var_at_m,
                               int estimator, double *out, smmd_stream_t stream);

smmd_status smmd_poly_diff_ratio(const smmd_poly_sums *yy, const smmd_poly_sums *xy,
                                 const smmd_poly_sums *zz, const smmd_poly_sums *xz, int m,
                                 double *out, smmd_stream_t stream);

/* ---------------------------------------------------------------------------
 * ConvMeanPool filter fold (gan/core/resnet/block.py:63-66: conv3x3 SAME, then
 * the mean of the four strided slices), run by the product as ONE 4x4
 * stride-2 conv.  A filter is one (cout, cin) pair, row-major.  One launch
 * covers n_layers <= 16 layers (host arrays of device pointers / counts; a
 * zero count skips the layer).
 *  adjoint = 0: src [n_filters, 3, 3] -> dst [n_filters, 4, 4],
 *               dst[s,t] = 1/4 sum_{a,b in {0,1}} src[s-a, t-b]
 *  adjoint = 1: src [n_filters, 4, 4] -> dst [n_filters, 3, 3],
 *               dst[u,v] = 1/4 sum_{a,b in {0,1}} src[u+a, v+b]  (the gradient)
 * Every src / dst must be 16-byte aligned.
 * ------------------------------------------------------------------------- */
smmd_status smmd_fold_pool_weights(const float *const *src, float *const *dst,
                                   const int64_t *n_filters, int n_layers, int adjoint,
                                   smmd_stream_t stream);

/* UpsampleConv filter fold (gan/core/resnet/block.py:53-60: concat x4 +
 * depth_to_space, i.e. a nearest x2 upsample, then conv3x3 SAME), run by the
 * product as ONE 4x4 stride-2 transposed conv (ABI 11; replaces
 * convops.fold_up_weight's pad / avg_pool / scale / flip / transpose ops).
 *  adjoint = 0: src W [cout, cin, 3, 3] -> dst K [cin, cout, 4, 4],
 *               K[ci][co][s][t] = sum_{a,b in {0,1}} W[co][ci][3-s-a][3-t-b]
 *               (4 x the ConvMeanPool fold, flipped in both axes, transposed)
 *  adjoint = 1: src gK [cin, cout, 4, 4] -> dst gW [cout, cin, 3, 3],
 *               gW[co][ci][u][v] = sum_{a,b in {0,1}} gK[ci][co][3-u-a][3-v-b]
 * src and dst 16-byte aligned. */
smmd_status smmd_fold_up_weight(const float *src, float *dst, int cout, int cin, int adjoint,
                                smmd_stream_t stream);

/* ---------------------------------------------------------------------------
 * Convolution bias gradient: out[c] = sum_{n, hw} gy[n, c, hw] over an NCHW
 * tensor [N, C, HW] (TF's BiasAddGrad of the bias_add in snops.conv2d,
 * gan/core/snops.py:89-90, and resnet Conv2D, gan/core/resnet/ops/conv2d.py:37-39).
 * Fixed-order two-stage sum; workspace from smmd_channel_sum_workspace_bytes.
 * float4 loads when HW % 4 == 0 and gy is 16-byte aligned, scalar otherwise.
 * ------------------------------------------------------------------------- */
size_t smmd_channel_sum_workspace_bytes(int N, int C);

smmd_status smmd_channel_sum(const float *gy, int N, int C, int HW, float *out, void *ws,
                             size_t ws_bytes, smmd_stream_t stream);

/* ---------------------------------------------------------------------------
 * The input of a critic down block feeds two ops: the main path's ReLU
 * (gan/core/resnet/block.py:44, norm off in the critic) and the shortcut's 2x2
 * mean pool (MeanPoolConv, block.py:69-71); the block output is their paths'
 * sum (block.py:50).  These two entry points read it once forward (from the
 * previous block's two paths, or the first conv's pre-activation) and write
 * its gradient in one pass backward.  Planes [planes, H, W] NCHW fp32, H even,
 * W % 4 == 0, 16-byte aligned full-size tensors, 8-byte aligned pooled ones.
 * With s(m) = 1 where m > 0, else the slope, and u = (x + bx) (+ (y + by) if y
 * != NULL), bx / by per-channel biases [C] of planes = N * C (NULL: none):
 * smmd_mask_pool2:     out_masked = u * s_m(m)   (slope_m 0: the ReLU; NULL: skip),
 *                      out_pool[i][j] = (((v[2i][2j] + v[2i][2j+1]) + v[2i+1][2j])
 *                                        + v[2i+1][2j+1]) / 4,  v = u * s_p(m)
 *                      (NULL: skip); m NULL: the mask source is u itself.
 *                      slope_p 1 pools u; 0.2 pools lrelu(u) (the first block's
 *                      input, architecture.py:393, never written); y is the
 *                      previous block's second path (block.py:50's add, fused).
 * smmd_mask_pool2_adj: out = a * s_m(m) + s_p(m) * nearest_up(b / 4)  (a or b
 *                      NULL: that term absent) -- the adjoint of smmd_mask_pool2 in
 *                      u, so each is the other's backward (linear, m constant).
 * The selects, the pooling order and the one add are those of torch's relu /
 * leaky_relu / avg_pool2d / their backward / nearest upsample and autograd's
 * gradient sum, so results are bit-identical to that composition.
 * ------------------------------------------------------------------------- */
smmd_status smmd_mask_pool2(const float *x, const float *y, const float *bx, const float *by,
                            int C, const float *m, float slope_m, float slope_p, int64_t planes,
                            int H, int W, float *out_masked, float *out_pool,
                            smmd_stream_t stream);

smmd_status smmd_mask_pool2_adj(const float *a, const float *b, const float *m, float slope_m,
                                float slope_p, int64_t planes, int H, int W, float *out,
                                smmd_stream_t stream);

/* A generator up block's output (block.py:50; its UpsampleConv shortcut,
 * block.py:53-60, runs the 1x1 conv before the nearest upsample):
 *   out[n][c][i][j] = (s[n][c][i/2][j/2] + bs[c]) + (h[n][c][i][j] + bh[c])
 * s [planes, H/2, W/2] (8-byte aligned), h and out [planes, H, W] (16-byte
 * aligned), planes = N * C, bs / bh NULL: no bias; H even, W % 4 == 0.  The
 * order of the unfused bias adds, upsample and add, so bit-identical to them. */
smmd_status smmd_up_add(const float *s, const float *bs, const float *h, const float *bh, int C,
                        int64_t planes, int H, int W, float *out, smmd_stream_t stream);

/* The critic's tail, lrelu(h).sum(dim=(2, 3)) with h = a + b the last block's
 * two paths (architecture.py:430-433; the reference's final lrelu and
 * tf.reduce_sum): rows = N * C of hw pixels (hw % 4 == 0, 16-byte aligned).
 * smmd_row_lrelu_sum: y[r] = sum_i lrelu(a + b) (b NULL: a alone); with mu
 *   set, y[r] = sum_i (a + b) * s(mu + mv), s(h) = 1 for h > 0 else slope --
 *   the adjoint of smmd_row_lrelu_bcast (the tail's double backward).
 * smmd_row_lrelu_bcast: out[r][i] = h > 0 ? g[r] : g[r] * slope, h = mu + mv
 *   (mv NULL: mu) -- the tail's backward, bit-identical to torch's expand +
 *   leaky_relu_backward.  The row sums run in pixel order (not torch's). */
smmd_status smmd_row_lrelu_sum(const float *a, const float *b, const float *mu, const float *mv,
                               float *y, int64_t rows, int hw, float slope, smmd_stream_t stream);

smmd_status smmd_row_lrelu_bcast(const float *g, const float *mu, const float *mv, float *out,
                                 int64_t rows, int hw, float slope, smmd_stream_t stream);

/* ---------------------------------------------------------------------------
 * Training-mode batch norm + ReLU when no gradient is taken (the generator's
 * forward in a critic step): tf.layers.batch_normalization(training=True,
 * momentum 0.9, eps) + tf.nn.relu (gan/core/snops.py:31-40,
 * resnet/ops/batchnorm.py:10-18, resnet/block.py:42-47, architecture.py:178-208).
 *   y = relu(x * scale + shift), scale = gamma / sqrt(var + eps),
 *   shift = beta - mean * scale, mean / biased var of x[:, c] over (N, HW),
 *   running_mean / running_var (NULL: not kept) <- (1 - momentum) * old +
 *   momentum * (mean / unbiased var).  x, y [N, C, HW] NCHW fp32, 16-byte
 *   aligned, HW % 4 == 0; gamma / beta NULL: 1 / 0.  Statistics in double in
 *   a fixed order; workspace from smmd_bn_relu_workspace_bytes.
 * ------------------------------------------------------------------------- */
size_t smmd_bn_relu_workspace_bytes(int N, int C);

smmd_status smmd_bn_relu_fwd(const float *x, int N, int C, int HW, const float *gamma,
                             const float *beta, float *running_mean, float *running_var,
                             float momentum, float eps, float *y, void *ws, size_t ws_bytes,
                             smmd_stream_t stream);

/* The same forward, also writing save[4 C] = per channel {k, mean - k,
 * 1 / sqrt(var + eps), gamma / sqrt(var + eps)} (k: the channel's first
 * element, the statistics' shift) for the backward; save may be NULL. */
smmd_status smmd_bn_relu_fwd_save(const float *x, int N, int C, int HW, const float *gamma,
                                  const float *beta, float *running_mean, float *running_var,
                                  float momentum, float eps, float *y, float *save, void *ws,
                                  size_t ws_bytes, smmd_stream_t stream);

/* Backward of y = relu(batch_norm(x)) in training mode (the generator step,
 * resnet/block.py:42-47, snops.py:31-40 / resnet/ops/batchnorm.py:8-18 with
 * TF's autodiff): with z recomputed from x and save exactly as the forward
 * formed it (the ReLU mask bit for bit), gz = gy [z > 0], M = N HW:
 * gbeta = sum gz, ggamma = sum gz xhat (per channel; either may be NULL),
 * gx = gamma inv (gz - gbeta / M - xhat ggamma / M).  Workspace as the
 * forward's.  x, gy, gx NCHW fp32, 16-byte aligned, HW % 4 == 0. */
smmd_status smmd_bn_relu_bwd(const float *x, const float *gy, int N, int C, int HW,
                             const float *beta, const float *save, float *gx, float *ggamma,
                             float *gbeta, void *ws, size_t ws_bytes, smmd_stream_t stream);

/* ---------------------------------------------------------------------------
 * Thin 3x3 convolutions: stride 1, zero padding 1 (TF SAME at stride 1), NCHW
 * fp32, one side with <= 4 channels.  They serve the critics' first layer
 * (3 -> dim: snops.conv2d / resnet Conv2D, gan/core/snops.py:69-90,
 * gan/core/resnet/ops/conv2d.py:16-39, as used at architecture.py:395-407 and
 * :410-434) and the generators' last (dim -> 3: snops.deconv2d at stride 1,
 * gan/core/snops.py:104-126, architecture.py:178-208, :211-230), with their
 * input and weight gradients (the TF autodiff of those ops, to second order
 * through the scaling regulariser's Jacobian).
 *
 * Tap t = 3 kh + kw reads the input at (h + kh - 1, w + kw - 1), zero outside.
 * smmd_conv3x3_thin: y[n][o][p] = bias[o] + sum_{i, t} A[o][i][t] x[n][i][p + d(t)]
 *   x [n, ci, h, w_img], y [n, co, h, w_img], bias [co] or NULL;
 *   mode 0: A[o][i][t] = w[o][i][t],     w [co, ci, 3, 3] (the convolution);
 *   mode 1: A[o][i][t] = w[i][o][8 - t], w [ci, co, 3, 3] (the input gradient
 *           of a convolution with weight w; also a stride-1 SAME conv2d_transpose).
 *   Needs ci <= 4, or co <= 4 and w_img <= 64; otherwise SMMD_EUNSUPPORTED.
 * smmd_conv3x3_thin_wgrad: gw[o][i][t] = sum_{n, p} gy[n][o][p] x[n][i][p + d(t)]
 *   gy [n, co, h, w_img], x [n, ci, h, w_img], gw [co, ci, 3, 3]; needs
 *   min(ci, co) <= 4 and w_img <= 64.  Workspace from
 *   smmd_conv3x3_thin_wgrad_workspace_bytes (per-image partials, added over
 *   the images in order).
 * ------------------------------------------------------------------------- */
smmd_status smmd_conv3x3_thin(const float *x, const float *w, const float *bias, float *y,
                              int n, int ci, int co, int h, int w_img, int mode,
                              smmd_stream_t stream);

size_t smmd_conv3x3_thin_wgrad_workspace_bytes(int n, int ci, int co, int h, int w_img);

smmd_status smmd_conv3x3_thin_wgrad(const float *gy, const float *x, float *gw, int n, int ci,
                                    int co, int h, int w_img, void *ws, size_t ws_bytes,
                                    smmd_stream_t stream);

/* *_acc: the same weight gradient ADDED into gw (gw += dW, one rounding: the
 * add autograd would run for a weight used by several convolutions; the
 * caller's gw holds the earlier contributions), gan.core.convops._late_gw. */
smmd_status smmd_conv3x3_thin_wgrad_acc(const float *gy, const float *x, float *gw, int n,
                                        int ci, int co, int h, int w_img, void *ws,
                                        size_t ws_bytes, smmd_stream_t stream);

/* ---------------------------------------------------------------------------
 * 3x3 stride-1 SAME convolutions as fused Winograd F(2x2, 3x3) on the f32
 * MFMA: the critics' and generators' wide 3x3 layers (snops.conv2d /
 * resnet Conv2D with padding SAME, gan/core/snops.py:69-90,
 * gan/core/resnet/ops/conv2d.py:16-39, in the residual blocks of
 * gan/core/resnet/block.py:38-50 and architecture.py:395-434), forward and
 * input gradient (TF's Conv2DBackpropInput), to every order of the critic's
 * double backward.  NCHW fp32, tap t = 3 kh + kw reads (h + kh - 1, w + kw - 1),
 * zero outside.
 *
 * smmd_wino3x3_filter: u = the 16 transform-point images of the filters,
 *   U = G g G^T per (ko, ci), in the conv kernel's staging order;
 *   mode 0: g = w[ko][ci], w [ko, ci, 3, 3] (the convolution);
 *   mode 1: g[a][b] = w[ci][ko][2 - a][2 - b], w [ci, ko, 3, 3] (the input
 *           gradient of a convolution with weight w).
 *   u holds smmd_wino3x3_filter_bytes(ko, ci) bytes; needs ko % 64 == 0 and
 *   ci % 8 == 0.
 * smmd_wino3x3_conv: y[n][ko][p] = bias[ko] + sum_{ci, t} g[ko][ci][t] x[n][ci][p + d(t)]
 *   x [n, ci, h, w_img], y [n, ko, h, w_img] (16-byte aligned), bias [ko] or
 *   NULL, u from smmd_wino3x3_filter; h and w_img even (smmd_wino3x3_supported).
 *   Small grids split the input channels over several workgroups and add the
 *   partial outputs in slice order from the workspace
 *   (smmd_wino3x3_workspace_bytes; 0 = none needed).  Deterministic.
 * ------------------------------------------------------------------------- */
int smmd_wino3x3_supported(int n, int ci, int ko, int h, int w_img);

size_t smmd_wino3x3_filter_bytes(int ko, int ci);

smmd_status smmd_wino3x3_filter(const float *w, int ko, int ci, int mode, float *u,
                                size_t u_bytes, smmd_stream_t stream);

size_t smmd_wino3x3_workspace_bytes(int n, int ci, int ko, int h, int w_img);

smmd_status smmd_wino3x3_conv(const float *x, const float *u, const float *bias, float *y, int n,
                              int ci, int ko, int h, int w_img, void *ws, size_t ws_bytes,
                              smmd_stream_t stream);

/* the same with tf.nn.relu applied to the output (the critic's first conv of
 * each down block, gan/core/resnet/block.py:44-46 with norm off): y = relu(conv + bias) */
smmd_status smmd_wino3x3_conv_relu(const float *x, const float *u, const float *bias, float *y,
                                   int n, int ci, int ko, int h, int w_img, void *ws,
                                   size_t ws_bytes, smmd_stream_t stream);

/* the same with the next layer's ReLU mask applied to the output: y = (mask <= 0 ?
 * 0 : conv + bias), mask [n, ko, h, w_img] (TF's relu gradient, threshold_backward's
 * select).  The double backward's upstream gradient of a conv-ReLU whose consumer
 * masks (gan/core/resnet/block.py:44-46 -> :63-66; convops _ConvBackward gy_mask). */
smmd_status smmd_wino3x3_conv_mask(const float *x, const float *u, const float *bias,
                                   const float *mask, float *y, int n, int ci, int ko, int h,
                                   int w_img, void *ws, size_t ws_bytes, smmd_stream_t stream);

/* the pair form: y = conv(x, u) + conv(x2, u2) + bias, both inputs [n, ci, h,
 * w_img] and both filters from smmd_wino3x3_filter at the same (ko, ci), in
 * ONE launch whose input-channel loop runs over both (the double backward's
 * gradient of a conv's upstream, conv(ggx, w) + conv(x, ggw),
 * gan/core/convops._ConvBackward: one output instead of two and their sum).
 * Workspace: smmd_wino3x3_conv2_workspace_bytes. */
size_t smmd_wino3x3_conv2_workspace_bytes(int n, int ci, int ko, int h, int w_img);

smmd_status smmd_wino3x3_conv2(const float *x, const float *u, const float *x2, const float *u2,
                               const float *bias, float *y, int n, int ci, int ko, int h,
                               int w_img, void *ws, size_t ws_bytes, smmd_stream_t stream);

/* ---------------------------------------------------------------------------
 * 4x4 stride-2 padding-1 convolutions as polyphase Winograd F(2x2, 2x2) on the
 * f32 MFMA: the critics' ConvMeanPool layers (gan/core/resnet/block.py:63-66;
 * mean_pool2(conv3x3(x, W)) is conv4x4_s2(x, W'), W' the pool-folded filter,
 * smmd_fold_pool_weights) and their input gradient, which is also the
 * generators' UpsampleConv folded into one transposed conv
 * (block.py:53-60).  NCHW fp32; x split into its four 2 x 2 phases makes each
 * an F(2x2, 2x2) problem: 9 point products per 2 x 2 output tile against 16
 * multiplies of the direct conv.
 *
 * smmd_wino4x4s2_filter / smmd_wino4x4s2t_filter: the transformed filters of
 *   W' [ko, ci, 4, 4] for the conv, or of W' [k, c, 4, 4] for the transposed
 *   conv; u holds smmd_wino4x4s2_filter_bytes(ko, ci) bytes (16-byte aligned).
 * smmd_wino4x4s2_conv: y [n, ko, h/2, w/2] = conv2d(x [n, ci, h, w], W',
 *   stride 2, padding 1) + bias; needs h, w % 4 == 0, ci % 2 == 0, ko % 64 == 0.
 * smmd_wino4x4s2t_conv: dx [n, c, 2 hg, 2 wg] = conv_transpose2d(gy [n, k, hg,
 *   wg], W', stride 2, padding 1) + bias; needs hg, wg even, k % 8 == 0,
 *   c % 64 == 0.
 * Small grids split the reduction over several workgroups and add the partial
 * outputs in slice order from the workspace (*_workspace_bytes; 0 = none).
 * ------------------------------------------------------------------------- */
int smmd_wino4x4s2_supported(int n, int ci, int ko, int h, int w_img);

int smmd_wino4x4s2t_supported(int n, int k, int c, int hg, int wg);

size_t smmd_wino4x4s2_filter_bytes(int ko, int ci);

smmd_status smmd_wino4x4s2_filter(const float *w, int ko, int ci, float *u, size_t u_bytes,
                                  smmd_stream_t stream);

smmd_status smmd_wino4x4s2t_filter(const float *w, int k, int c, float *u, size_t u_bytes,
                                   smmd_stream_t stream);

size_t smmd_wino4x4s2_workspace_bytes(int n, int ci, int ko, int h, int w_img);

size_t smmd_wino4x4s2t_workspace_bytes(int n, int k, int c, int hg, int wg);

smmd_status smmd_wino4x4s2_conv(const float *x, const float *u, const float *bias, float *y,
                                int n, int ci, int ko, int h, int w_img, void *ws,
                                size_t ws_bytes, smmd_stream_t stream);

/* the same added into y: y += conv(x, W') + bias (the earlier value first, so
 * y_old + result, autograd's sum of two gradient contributions; convops
 * _ConvBackward: a critic block's main-path and shortcut gradients of the
 * gradient both read, in the scaling regulariser's double backward) */
smmd_status smmd_wino4x4s2_conv_acc(const float *x, const float *u, const float *bias, float *y,
                                    int n, int ci, int ko, int h, int w_img, void *ws,
                                    size_t ws_bytes, smmd_stream_t stream);

smmd_status smmd_wino4x4s2t_conv(const float *gy, const float *u, const float *bias, float *dx,
                                 int n, int k, int c, int hg, int wg, void *ws, size_t ws_bytes,
                                 smmd_stream_t stream);

/* smmd_wino4x4s2t_conv followed by TF's ReLU gradient in the same launch:
 * dx = (mask <= 0 ? 0 : conv_transpose2d(gy, W') + bias), mask [n, c, 2 hg,
 * 2 wg] (16-byte aligned) the conv's input, a ReLU output whose producer then
 * skips its own mask (convops._Conv2dReLU with consumer_masks; replaces
 * threshold_backward(dx, mask, 0) after the input gradient of the critic's
 * ConvMeanPool conv, gan/core/resnet/block.py:44-50, :63-66). */
smmd_status smmd_wino4x4s2t_conv_mask(const float *gy, const float *u, const float *bias,
                                      const float *mask, float *dx, int n, int k, int c, int hg,
                                      int wg, void *ws, size_t ws_bytes, smmd_stream_t stream);

/* the pair form of smmd_wino4x4s2_conv: y = conv(x, u) + conv(x2, u2) + bias
 * in one launch (as smmd_wino3x3_conv2). */
size_t smmd_wino4x4s2_conv2_workspace_bytes(int n, int ci, int ko, int h, int w_img);

smmd_status smmd_wino4x4s2_conv2(const float *x, const float *u, const float *x2,
                                 const float *u2, const float *bias, float *y, int n, int ci,
                                 int ko, int h, int w_img, void *ws, size_t ws_bytes,
                                 smmd_stream_t stream);

/* ---------------------------------------------------------------------------
 * Filter transforms straight from a spectrally normalised layer's raw weight
 * W and its device scalars sigma (smmd_sn_power_iter's output) and s (NULL:
 * 1): the filter is W_eff = (W / sigma) * s (sn.py:43, snops.py:84), and with
 * fold = 1 the ConvMeanPool fold of it from the raw 3 x 3 W [ko, ci, 3, 3]
 * (block.py:63-66), computed with the refresh's own arithmetic (no
 * contraction), so u is bit-identical to smmd_wino3x3_filter /
 * smmd_wino4x4s2(t)_filter of the W_eff the refresh would have written --
 * which it then need not write (smmd_sn_layer.W_eff = NULL).  Layouts, modes
 * and requirements as the plain transforms; fold = 0 takes W [.., .., 4, 4].
 * ------------------------------------------------------------------------- */
smmd_status smmd_wino3x3_filter_sn(const float *w, const float *sigma, const float *s, int ko,
                                   int ci, int mode, float *u, size_t u_bytes,
                                   smmd_stream_t stream);

smmd_status smmd_wino4x4s2_filter_sn(const float *w, const float *sigma, const float *s, int fold,
                                     int ko, int ci, float *u, size_t u_bytes,
                                     smmd_stream_t stream);

smmd_status smmd_wino4x4s2t_filter_sn(const float *w, const float *sigma, const float *s,
                                      int fold, int k, int c, float *u, size_t u_bytes,
                                      smmd_stream_t stream);

/* ---------------------------------------------------------------------------
 * The weight gradient of the 3x3 stride-1 SAME conv (TF's
 * Conv2DBackpropFilter of snops.conv2d / resnet Conv2D, gan/core/snops.py:69-90,
 * the wide layers of gan/core/resnet/block.py:38-50) as Winograd F(2x2, 3x3):
 * dU_p = sum over 2 x 2 tiles of (A dY A^T)_p (B^T d B)_p on the f32 MFMA,
 * then gw = G^T dU G.  gw [co, ci, 3, 3], x [n, ci, h, w_img], gy [n, co, h,
 * w_img]; needs ci, co % 64 == 0, h even, w_img % 4 == 0
 * (smmd_wino3x3_wgrad_supported).  The tiles are split over workgroups whose
 * partial dU (smmd_wino3x3_wgrad_workspace_bytes) are added in slice order.
 * Deterministic.
 * ------------------------------------------------------------------------- */
int smmd_wino3x3_wgrad_supported(int n, int ci, int co, int h, int w_img);


size_t smmd_wino3x3_wgrad_workspace_bytes(int n, int ci, int co, int h, int w_img);

smmd_status smmd_wino3x3_wgrad(const float *x, const float *gy, float *gw, int n, int ci, int co,
                               int h, int w_img, void *ws, size_t ws_bytes,
                               smmd_stream_t stream);

/* (gw += dW, as smmd_conv3x3_thin_wgrad_acc) */
smmd_status smmd_wino3x3_wgrad_acc(const float *x, const float *gy, float *gw, int n, int ci,
                                   int co, int h, int w_img, void *ws, size_t ws_bytes,
                                   smmd_stream_t stream);

/* ---------------------------------------------------------------------------
 * The weight gradient of the 4x4 stride-2 pad-1 conv (TF's
 * Conv2DBackpropFilter of the folded ConvMeanPool layers, gan/core/resnet/
 * block.py:63-66, snops.py:69-90; with x and gy swapped, of the generator's
 * folded UpsampleConv, block.py:53-60) as polyphase Winograd F(2x2, 2x2):
 * dU_p = sum over 2 x 2 output tiles of (A dY A^T)_p (B^T d B)_p for every
 * (input channel, x phase) column on the f32 MFMA, then each phase's 2 x 2 tap
 * block of gw = G^T dU G.  gw [co, ci, 4, 4], x [n, ci, h, w_img], gy [n, co,
 * h/2, w_img/2]; needs ci % 16 == 0, co % 64 == 0 and an output tile grid
 * (h/4) x (w_img/4) of 16 columns, 8 columns and an even row count, 4 columns
 * and a row count divisible by 4, or 2 x 2, and n times the tiles per image
 * divisible by 16 (smmd_wino4x4s2_wgrad_supported).
 * The tiles are split over workgroups whose partial gw
 * (smmd_wino4x4s2_wgrad_workspace_bytes) are added in slice order.
 * Deterministic.
 * ------------------------------------------------------------------------- */
int smmd_wino4x4s2_wgrad_supported(int n, int ci, int co, int h, int w_img);

size_t smmd_wino4x4s2_wgrad_workspace_bytes(int n, int ci, int co, int h, int w_img);

smmd_status smmd_wino4x4s2_wgrad(const float *x, const float *gy, float *gw, int n, int ci,
                                 int co, int h, int w_img, void *ws, size_t ws_bytes,
                                 smmd_stream_t stream);

/* (gw += dW, as smmd_conv3x3_thin_wgrad_acc) */
smmd_status smmd_wino4x4s2_wgrad_acc(const float *x, const float *gy, float *gw, int n, int ci,
                                     int co, int h, int w_img, void *ws, size_t ws_bytes,
                                     smmd_stream_t stream);

/* ---------------------------------------------------------------------------
 * The 1x1 stride-1 convolutions of the residual shortcuts (ABI 11;
 * gan/core/resnet/block.py:28-40: MeanPoolConv in the critic's down blocks,
 * the 1x1 conv of the generator's up-block shortcut, snops.conv2d's
 * tf.nn.conv2d / Conv2DBackpropInput / Conv2DBackpropFilter, snops.py:69-90)
 * on the f32 MFMA, NCHW without layout transposes.  p = pixels per image.
 *
 * smmd_conv1x1: y [n, m, p] = a [m, r] . x [n, r, p] (+ bias [m], may be NULL).
 *   The forward is a = W [k, c] (m = k, r = c); the input gradient is
 *   a = W^T as a [c, k] row-major copy (m = c, r = k) with x = gy.  Needs
 *   m % 64 == 0, r % 32 == 0, p % 4 == 0, n p % 64 == 0
 *   (smmd_conv1x1_supported(n, r, m, p)); a, x, y 16-byte aligned.  Shapes
 *   with few output tiles split the reduction over workgroups whose partial
 *   outputs (smmd_conv1x1_workspace_bytes; 0 = none) are added in slice order.
 * smmd_conv1x1_wgrad: gw [k, c] = sum over n, p of gy [n, k, p] x [n, c, p];
 *   needs c, k % 64 == 0, p % 4 == 0, n p % 32 == 0; the columns are split
 *   over workgroups whose partials (smmd_conv1x1_wgrad_workspace_bytes; 0 =
 *   none) are added in slice order.  Deterministic.
 * ------------------------------------------------------------------------- */
int smmd_conv1x1_supported(int n, int r, int m, int p);

size_t smmd_conv1x1_workspace_bytes(int n, int r, int m, int p);

smmd_status smmd_conv1x1(const float *a, const float *x, const float *bias, float *y, int n,
                         int r, int m, int p, void *ws, size_t ws_bytes, smmd_stream_t stream);

/* the same with a given transposed, a [r][m]: y = a^T x (+ bias).  The input
 * gradient of a 1x1 conv straight from its weight W [K][C] (dx = W^T gy,
 * r = K, m = C) without a per-step W^T copy; same workspace as smmd_conv1x1. */
smmd_status smmd_conv1x1_t(const float *a, const float *x, const float *bias, float *y, int n,
                           int r, int m, int p, void *ws, size_t ws_bytes, smmd_stream_t stream);

int smmd_conv1x1_wgrad_supported(int n, int c, int k, int p);

size_t smmd_conv1x1_wgrad_workspace_bytes(int n, int c, int k, int p);

smmd_status smmd_conv1x1_wgrad(const float *gy, const float *x, float *gw, int n, int c, int k,
                               int p, void *ws, size_t ws_bytes, smmd_stream_t stream);

/* (gw += dW, as smmd_conv3x3_thin_wgrad_acc) */
smmd_status smmd_conv1x1_wgrad_acc(const float *gy, const float *x, float *gw, int n, int c,
                                   int k, int p, void *ws, size_t ws_bytes,
                                   smmd_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* SMMD_HIP_H */
