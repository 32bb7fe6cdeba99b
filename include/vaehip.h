/*
 * vaehip.h — C ABI of libvaehip.so, the MI355X (gfx950) kernels of the VAE training step.
 *
 * The reference (bplaut/PyTorch-VAE) has no native code and no FFI: its hot path is the
 * models.base.BaseVAE interface (models/base.py:5-28) implemented with torch.nn modules
 * (models/vanilla_vae.py:8-173, beta_vae.py, iwae.py, vq_vae.py) and driven by
 * experiment.VAEXperiment.training_step (experiment.py:45-86).  Each entry point below
 * replaces the forward or backward of one of those nn ops; the comment on each names the
 * reference line whose op it replaces.  The Python host (pytorch-vae_amd/vae_amd) binds
 * them with ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions
 *   - Return 0 on success, a negative VAE_E_* code on a bad argument, or a positive
 *     hipError_t.  vae_last_error() gives a thread-local message.  Nothing aborts.
 *   - The caller owns all memory (PyTorch caching allocator); the library never allocates,
 *     frees or synchronises.  Every launch goes on `stream` (a hipStream_t), so a caller may
 *     capture any sequence of calls into a HIP graph.
 *   - Activations are NHWC.  The only NCHW tensors are the user-facing image x and the
 *     reconstruction (the reference's [B,3,H,W] fp32 tensors).
 *   - `dtype` selects the storage/MFMA type of activations and weight copies:
 *     VAE_F32 (v_mfma_f32_16x16x4_f32, exact fp32 — parity mode) or VAE_BF16
 *     (v_mfma_f32_16x16x32_bf16, fp32 accumulate — throughput mode).  Per-channel
 *     statistics, gradients of weights, losses and optimizer state are always fp32.
 *   - Native weight layouts (state-dict conversion in vae_amd/layout.py):
 *       Conv2d          torch [Co][Ci][R][S]  -> native [Co][R][S][Ci]
 *       ConvTranspose2d torch [Ci][Co][R][S]  -> native [Ci][R][S][Co]
 *       Linear          torch [Out][In]       -> native [Out][In'] (In' = NHWC order of a
 *                                                flattened [C,2,2] map where applicable)
 */
#ifndef VAEHIP_H
#define VAEHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VAE_ABI_VERSION 25

enum vae_dtype { VAE_F32 = 0, VAE_BF16 = 1 };

enum vae_status {
  VAE_OK = 0,
  VAE_E_BADARG = -1,     /* null pointer / inconsistent sizes              */
  VAE_E_BADSHAPE = -2,   /* shape not supported by the kernels             */
  VAE_E_BADDTYPE = -3,
  VAE_E_UNSUPPORTED = -4
};

/* Per-channel transform applied to a tensor element when a kernel loads it (it is how
 * BatchNorm + LeakyReLU of the reference, vanilla_vae.py:30-31, are fused into the
 * consumer instead of being separate passes).  `t` is the stored element, c its channel. */
enum vae_xform_kind {
  VAE_X_NONE = 0,    /* v = t                                                            */
  VAE_X_ACT = 1,     /* v = lrelu(t, slope)           (slope 0 = ReLU)                   */
  VAE_X_BN_ACT = 2,  /* v = lrelu(gamma_c*(t-mean_c)*invstd_c + beta_c, slope)  — BN train */
  VAE_X_BN_DY = 3    /* v = gamma_c*invstd_c*(t - dbeta_c/M - xhat*dgamma_c/M),           */
                     /*     xhat = (aux - mean_c)*invstd_c          — BN backward to dy    */
};

typedef struct vae_xform {
  int32_t kind;            /* vae_xform_kind */
  int32_t channels;        /* channel count C (channel of an element = index % C) */
  float slope;             /* LeakyReLU negative slope (reference default 0.01) */
  float count;             /* M = elements per channel in the BN reduction (N*H*W) */
  float eps;               /* BN eps (1e-5) */
  float momentum;          /* BN momentum (0.1), used only when running_* are set */
  const float* sum;        /* [C] Σ(y - shift)   written by the producing kernel */
  const float* sumsq;      /* [C] Σ(y - shift)^2 */
  const float* shift;      /* [C] shift the sums are taken against (the conv bias) or NULL */
  const float* gamma;      /* [C] BN weight */
  const float* beta;       /* [C] BN bias */
  const float* dgamma;     /* [C] BN_DY: Σ g*xhat (== dL/dgamma) */
  const float* dbeta;      /* [C] BN_DY: Σ g      (== dL/dbeta)  */
  const void* aux;         /* BN_DY: pre-BN tensor y, indexed like the operand (dtype) */
  float* running_mean;     /* optional: updated once per call (unbiased var, as torch) */
  float* running_var;
  /* Replicated statistics: sum/sumsq (and dgamma/dbeta) hold `reps` partial copies, replica r
   * at offset r*rstride floats; the value of channel c is the sum over replicas.  Producers
   * spread their per-block atomics over the replicas so that thousands of workgroups do not
   * serialise on the same 2*C addresses.  reps <= 1: a single copy. */
  int32_t reps;
  int32_t rstride;
  /* BN_DY only: when set, the operation writes the reduced dL/dgamma, dL/dbeta here
   * (accumulating) — the BatchNorm affine gradients the optimizer reads. */
  float* dgamma_out;
  float* dbeta_out;
  /* Precomputed coefficient table (vae_bn_finalize), planar fp32:
   *   BN_ACT [4][C] = {gamma*invstd, beta - mean*gamma*invstd, invstd, -mean*invstd}
   *   BN_DY  [3][C] = {A, B, C} with dy = A*g + B*y + C.
   * When set, consumers load it instead of reducing the statistics themselves, and running
   * statistics / dgamma_out / dbeta_out are left to vae_bn_finalize. */
  const float* table;
} vae_xform;

/* One BatchNorm's per-step finalisation, run once between the kernel that produces its
 * statistics and the kernels that consume them (vanilla_vae.py:30,56,71 BatchNorm2d in
 * train mode; torch semantics for the running-statistic update).
 *   mode 0 (forward):  xf.sum/sumsq replicas -> table [4][C]; running_mean/var updated
 *                      (momentum, unbiased variance) when set.
 *   mode 1 (backward): xf.dgamma/dbeta replicas -> table [3][C]; dL/dgamma, dL/dbeta added to
 *                      xf.dgamma_out / dbeta_out; when db is set, the gradient of the bias of
 *                      the conv feeding the BatchNorm is added in closed form,
 *                      db_c = A*Σg + B*Σy + C*M.
 *   mode 2 (eval):     table [4][C] from xf.running_mean / running_var (BatchNorm2d in eval
 *                      mode — validation_step, sample, generate: experiment.py:122-132,
 *                      vanilla_vae.py:148-173); nothing is updated. */
typedef struct vae_bn_args {
  int32_t mode;
  vae_xform xf;
  float* table;
  float* db;
} vae_bn_args;

/* One convolution-family operation.  Geometry is that of the reference layer:
 *   Conv2d:          x [n,h,w,c] -> y [n,p,q,k]
 *   ConvTranspose2d: x [n,h,w,c] -> y [n,p,q,k]   (p = 2h for k3 s2 p1 op1 and k4 s2 p1)
 * Fields unused by an entry point are ignored. */
typedef struct vae_conv_args {
  int32_t dtype;           /* vae_dtype of activations / weight copies */
  int32_t n, h, w, c;      /* input of the layer (as in the reference) */
  int32_t k, p, q;         /* output channels / spatial */
  int32_t r, stride, pad;  /* square kernel, stride, padding (output_padding implied) */
  int32_t x_nchw_f32;      /* 1: x is the fp32 NCHW image (first layer), 0: NHWC dtype */
  /* tensors */
  const void* x;           /* layer input (stored pre-activation; see x_xf) */
  vae_xform x_xf;          /* transform applied to x elements on load */
  const void* wt;          /* weights in native layout (dtype) */
  const float* bias;       /* [k] or NULL */
  void* y;                 /* fwd: output pre-activation (NHWC, dtype) */
  float* y_sum;            /* fwd: optional per-channel Σ(acc), Σ(acc^2) for the next BN */
  float* y_sumsq;
  int32_t sum_reps;        /* replicas of y_sum/y_sumsq (fwd) or dx_dgamma/dx_dbeta (bwd_data), */
  int32_t sum_rstride;     /* see vae_xform.reps; <= 1: one copy */
  const void* residual;    /* fwd: optional y += xf(residual) (VQ-VAE ResidualLayer,
                              models/vq_vae.py:69); conv2d bwd_data: optional dx += residual (the
                              gradient reaching x through the skip connection) before dx_epi */
  vae_xform residual_xf;
  /* backward */
  const void* dy;          /* gradient w.r.t. the layer output (stored, dtype) */
  vae_xform dy_xf;         /* e.g. BN_DY: dy = BN-backward(g, y) computed on load */
  void* dx;                /* bwd_data: gradient w.r.t. the layer input (dtype) */
  vae_xform dx_epi;        /* bwd_data epilogue: how x was activated (BN_ACT/ACT/NONE);
                              BN_ACT/ACT need aux = stored pre-activation x; the kernel
                              writes g = dL/dz of that activation and, for BN_ACT,
                              accumulates Σg -> dx_dbeta, Σg*xhat -> dx_dgamma */
  float* dx_dgamma;
  float* dx_dbeta;
  float* dw;               /* bwd_filter: fp32 weight gradient, native layout (accumulated) */
  float* db;               /* bwd_filter: fp32 bias gradient (accumulated) or NULL */
  int32_t split_k;         /* 0 = choose automatically, 1 = no split-K */
  void* workspace;         /* fp32 scratch for split-K partial slabs (may be NULL: no split
                              of fwd / bwd_data); reused by every call on the stream */
  int64_t workspace_bytes;
  /* Optional BatchNorm finalisation of the statistics this call produces (forward: the
   * y_sum/y_sumsq of the next BatchNorm; bwd_data: its dx_dgamma/dx_dbeta): the call then also
   * does what vae_bn_finalize(bn_finalize) would (launched right after its own kernels).
   * bn_counter: reserved (a zeroed uint32 slot; may be NULL). */
  const struct vae_bn_args* bn_finalize;
  uint32_t* bn_counter;
  /* Optional bf16 copy of wt with its first and last axes swapped ([k][r][s][c] of a
   * ConvTranspose2d's [c][r][s][k], [c][r][s][k] of a Conv2d's [k][r][s][c]): the k-contiguous
   * weight rows the bf16 convT2d_fwd / conv2d_bwd_data GEMMs read (vae_swap_axes).  NULL: the
   * call builds it at the end of the workspace first (one extra launch). */
  const void* wt_t;
  /* bwd_filter: the stored innermost dimension of dw (c of a Conv2d's [k][r][s][c], k of a
   * ConvTranspose2d's [c][r][s][k]); 0 = all of it.  Smaller: dw is the parameter's own gradient
   * of an operand zero-padded on that axis (the 8-channel RGB image), indices >= dw_inner are
   * dropped (bf16 weight-gradient GEMM path only; elsewhere VAE_E_UNSUPPORTED). */
  int32_t dw_inner;
  /* 1: every cross-workgroup reduction of this call runs in a fixed order (partials to the
   * workspace, summed by an ordered pass) instead of float atomics, so repeated calls give
   * bit-identical results (the parity mode of experiment.py:308-311's gradients).  Needs the
   * workspace *_workspace_size reports for it; dtype VAE_F32 only (VAE_E_UNSUPPORTED otherwise). */
  int32_t deterministic;
  /* bwd_filter (bf16 grouped weight gradients of vae_conv_bwd_filter_batch, and the full-resolution
   * vae_convT2d_bwd): 1 = leave this weight gradient as fp32 partial rows in the workspace instead
   * of summing them into dw — no reduction launch; the call records a vae_grad_slab descriptor
   * (vae_deferred_take) for the caller to reduce later (vae_adam_step_ex).  dw is then WRITTEN, not
   * accumulated: by that reduction, or by the call itself where one workgroup covers the whole pixel
   * range (no partial rows, no descriptor).  The workspace must stay untouched until then. */
  int32_t defer_reduce;
} vae_conv_args;

/* Linear y[m][n] = x[m][:]·W[n][:] + b[n] (fc_mu|fc_var fused as one N=2D layer,
 * decoder_input).  Same transform / epilogue conventions as vae_conv_args. */
typedef struct vae_linear_args {
  int32_t dtype;
  int32_t m, n, k;         /* rows (batch), out features, in features */
  const void* x; vae_xform x_xf;
  const void* wt; const float* bias;
  void* y;
  int32_t y_f32;           /* fwd: write y as fp32 (fc_mu|fc_var output) instead of dtype */
  const void* dy;          /* [m][n] */
  int32_t dy_f32;          /* bwd: dy is fp32 (d[mu|logvar]) instead of dtype */
  void* dx; vae_xform dx_epi; float* dx_dgamma; float* dx_dbeta;
  int32_t sum_reps, sum_rstride;   /* replicas of dx_dgamma / dx_dbeta (vae_xform.reps) */
  float* dw; float* db;
  /* reparameterization backward epilogue (decoder_input bwd_data): when mulv != NULL the
   * kernel turns dz into d[mu|logvar] (vanilla_vae.py:107-117 + the analytic KL of :143) */
  const float* mulv;       /* [rows_mu][2*k] fc output (mu | log_var) */
  const float* eps;        /* [m][k] */
  const float* kl_coef;    /* [m] per-row coefficient of dKL (see vae_elbo_fwd) or NULL */
  float* dmulv;            /* [rows_mu][2*k], accumulated */
  int32_t samples;         /* rows per mu row (IWAE S; 1 otherwise) */
  void* workspace;         /* as vae_conv_args.workspace */
  int64_t workspace_bytes;
  /* Optional BatchNorm finalisation of the statistics this call produces (forward: the
   * y_sum/y_sumsq of the next BatchNorm; bwd_data: its dx_dgamma/dx_dbeta): the call then also
   * does what vae_bn_finalize(bn_finalize) would (launched right after its own kernels).
   * bn_counter: reserved (a zeroed uint32 slot; may be NULL). */
  const struct vae_bn_args* bn_finalize;
  uint32_t* bn_counter;
  int32_t deterministic;    /* as vae_conv_args.deterministic */
} vae_linear_args;

/* Final layer of the decoder: Conv2d(C->3, k3, s1, p1) + Tanh (vanilla_vae.py:73-75,
 * autoencoder.py:84-86) and the reconstruction term of the ELBO (F.mse_loss, vanilla_vae.py:140).
 * bf16 with w = 64 and C = 32, 64 or 128: MFMA kernels (vae_head.hip); otherwise VALU kernels. */
typedef struct vae_head_args {
  int32_t dtype;
  int32_t n, h, w, c;      /* input of the conv (NHWC, pre-activation, see x_xf) */
  const void* x; vae_xform x_xf;
  const float* wt;         /* fp32 native [3][3][3][c] */
  const float* bias;       /* [3] */
  const float* target;     /* fp32 NCHW [n,3,h,w] image the reconstruction is scored against;
                              for IWAE row i is scored against image i / samples */
  int32_t samples;         /* IWAE S (1 otherwise) */
  float* recon;            /* fp32 NCHW [n,3,h,w] */
  float* sse;              /* [n] Σ(recon-target)^2 per image, accumulated */
  const float* coef;       /* bwd: [n] dL/d(sse_i); g = coef*(recon-target)*(1-recon^2) */
  void* dx; vae_xform dx_epi; float* dx_dgamma; float* dx_dbeta;
  int32_t sum_reps, sum_rstride;   /* replicas of dx_dgamma / dx_dbeta (vae_xform.reps) */
  float* dw; float* db;
  const float* grad_recon; /* bwd alternative to coef: dL/drecon (NCHW fp32), g = grad*(1-recon^2) */
  void* workspace;         /* bwd (bf16): fp32 scratch for per-workgroup dW/db partials (summed in a
                              fixed order); NULL: atomics straight into dw/db */
  int64_t workspace_bytes;
  const struct vae_bn_args* bn_finalize;   /* as vae_conv_args.bn_finalize (bwd: final BatchNorm) */
  uint32_t* bn_counter;
  /* bwd, optional (bf16 MFMA path, kind VAE_LOSS_VANILLA or VAE_LOSS_BETA_H, samples 1): the loss
   * this backward seeds from.  Its seed coefficient is the constant 2/(n*3*h*w) (coef is not read)
   * and the call also evaluates the loss — vae_elbo_fwd's outputs: out, per_img, head_coef, kl_coef
   * — in one extra workgroup of its filter-partial reduction, so the step needs no vae_elbo_fwd
   * launch.  NULL: coef as above. */
  const struct vae_elbo_args* elbo;
  int32_t deterministic;    /* as vae_conv_args.deterministic (VALU kernels, fp32) */
  /* bwd (bf16 MFMA path, 32-channel head): as vae_conv_args.defer_reduce for the filter partials;
   * with elbo set the loss is deferred too (vae_deferred_take returns its arguments). */
  int32_t defer_reduce;
} vae_head_args;



/* Loss kinds (vanilla_vae.py:124-146, beta_vae.py:129-152, iwae.py:129-160, vq_vae.py:194-211) */
enum vae_loss_kind { VAE_LOSS_VANILLA = 0, VAE_LOSS_BETA_H = 1, VAE_LOSS_BETA_B = 2, VAE_LOSS_IWAE = 3,
                     VAE_LOSS_VQ = 4 };

typedef struct vae_elbo_args {
  int32_t kind;            /* vae_loss_kind */
  int32_t batch, samples, latent;
  int32_t img_elems;       /* C*H*W of one image */
  float kld_weight;        /* M_N */
  float beta, gamma, c_max, c_stop_iter;
  const float* iter;       /* BetaVAE-B: device num_iter (after the reference's +=1) */
  const float* mulv;       /* [batch][2*latent] */
  const float* sse;        /* [batch*samples] */
  float* out;              /* [4]: loss, Reconstruction_Loss, KLD (as the reference reports it), kld_raw */
  float* per_img;          /* [batch*samples] per-image MSE (experiment.py:60-62) */
  float* head_coef;        /* [batch*samples] dL/d(sse_i) for vae_head_bwd_* */
  float* kl_coef;          /* [batch*samples] per-row KL gradient coefficient */
  /* VAE_LOSS_VQ (mulv / head_coef / kl_coef unused): loss = recon + VQ_Loss with
   * VQ_Loss = (1 + vq_beta) * vq_sse / vq_elems (commitment*beta + embedding, vq_vae.py:47-50);
   * out = {loss, Reconstruction_Loss, VQ_Loss, 0} */
  const float* vq_sse;     /* [1] Σ(q - latents)^2 written by vae_vq_fwd */
  float vq_beta;
  float vq_elems;          /* number of latent elements (N*H*W*D) */
} vae_elbo_args;

/* VectorQuantizer (models/vq_vae.py:24-55) on NHWC latents [rows][dim] (rows = N*H*W, the
 * reference's flat_latents after its permute, :25-27) against the fp32 codebook [codes][dim].
 *   fwd: dist_k = (Σz² + Σ_e E_ke²) - 2 z·E_k in fp32 (the reference's formula, :30-32),
 *        indices = argmin with the first-minimum tie-break of torch.argmin (:35), q = E[index]
 *        written in `dtype` (the straight-through decoder input, :43,53), sse += Σ(q - z)².
 *   bwd: g = dq + s*beta*2(z - q)/n  ->  dlat = g*act'(lat)  (commitment loss + straight-through,
 *        :47,53; act' of lat_xf), dcodebook[index] += s*2(q - z)/n (embedding loss, :48), with
 *        n = rows*dim and s = *loss_grad (dL/dVQ_Loss; 1 when NULL). */
typedef struct vae_vq_args {
  int32_t dtype;
  int32_t rows, dim, codes;
  const void* lat;         /* [rows][dim] stored encoder output (pre-activation, see lat_xf) */
  vae_xform lat_xf;        /* NONE or ACT (the encoder's final LeakyReLU, vq_vae.py:117-121) */
  const float* codebook;   /* fp32 [codes][dim] (vq_layer.embedding.weight) */
  int64_t* indices;        /* fwd out [rows] */
  void* q;                 /* fwd out [rows][dim] (dtype) */
  float* sse;              /* fwd: [1] accumulated */
  float beta;              /* commitment weight (0.25) */
  const void* dq;          /* bwd: [rows][dim] dL/dq from the decoder (dtype) */
  const float* loss_grad;  /* bwd: device scalar dL/dVQ_Loss, or NULL for 1 */
  void* dlat;              /* bwd out [rows][dim] (dtype) */
  float* dcodebook;        /* bwd: fp32 [codes][dim], accumulated */
} vae_vq_args;

/* Tanh output layer + reconstruction error on an NHWC pre-activation y [n,h,w,c] (the
 * VQ-VAE decoder's last ConvTranspose2d + Tanh, vq_vae.py:156-160, and F.mse_loss at :203).
 *   fwd: recon (fp32 NCHW) = tanh(y); sse[i] += Σ(recon - target)² per image; when dy is set
 *        and grad_recon is NULL also dy = grad_scale*2(recon - target)*(1 - recon²)
 *        (the fused-loss backward seed, grad_scale = dL/dΣ = 1/(n*c*h*w) for a mean).
 *   bwd: dy = grad_recon*(1 - recon²) from a caller-supplied fp32 NCHW dL/drecon. */
typedef struct vae_recon_args {
  int32_t dtype;
  int32_t n, h, w, c;
  const void* y;
  const float* target;     /* fp32 NCHW */
  float* recon;            /* fp32 NCHW */
  float* sse;              /* [n] accumulated */
  void* dy;                /* NHWC (dtype) or NULL */
  float grad_scale;
  const float* grad_recon;
  int32_t ld;              /* channel stride of y and dy (>= c; 0: c) — an 8-channel padded layout keeps
                              the output convolution on the packed path; dy's pad channels are written 0 */
} vae_recon_args;

int vae_abi_version(void);
const char* vae_last_error(void);
/* Build identity and launch introspection (measurement tooling; no GPU work).
 * vae_build_digest: a digest of the sources this library was compiled from (csrc + this header),
 *   written into profiles so a counter summary is only ever matched with the code it measured.
 * vae_launch_log(1) starts recording (per host thread) the device kernels every later entry point
 *   launches, vae_launch_log(0) stops; vae_launch_log_names writes the recorded kernels as lines
 *   "<mangled>\t<demangled>\t<launches>\n" (first-launch order; <launches>: how many times the
 *   kernel was launched while recording) into buf (NUL-terminated, truncated to cap) and returns the
 *   bytes the full text needs. */
const char* vae_build_digest(void);
int vae_launch_log(int32_t on);
int64_t vae_launch_log_names(char* buf, int64_t cap);

/* --- Conv2d (encoder block, vanilla_vae.py:28-29 run at :84) ----------------------- */
int vae_conv2d_fwd(const vae_conv_args* a, void* stream);
int vae_conv2d_bwd_data(const vae_conv_args* a, void* stream);
int vae_conv2d_bwd_filter(const vae_conv_args* a, void* stream);
/* --- ConvTranspose2d (decoder block, vanilla_vae.py:50-55, :65-70) ------------------ */
int vae_convT2d_fwd(const vae_conv_args* a, void* stream);
int vae_convT2d_bwd_data(const vae_conv_args* a, void* stream);
int vae_convT2d_bwd_filter(const vae_conv_args* a, void* stream);
/* both gradients of the layer in one call (the bwd_data and bwd_filter fields together): the
 * decoder's full-resolution last ConvTranspose2d (final_layer.0, vanilla_vae.py:64-70; bf16,
 * 32 -> 32 channels, 32x32 -> 64x64) in ONE pass over dy on a fused kernel whose filter partials
 * take vae_convT2d_workspace_size(a, VAE_OP_BWD) bytes of workspace; any other layer runs
 * vae_convT2d_bwd_data then vae_convT2d_bwd_filter. */
int vae_convT2d_bwd(const vae_conv_args* a, void* stream);
/* The output ConvTranspose2d of the VQ-VAE fused with its Tanh + reconstruction + SSE (+ backward
 * seed) (vq_vae.py:160-164, :203; what vae_convT2d_fwd followed by vae_recon_fwd(rc) computes,
 * without storing the pre-tanh output): bf16, wide side [n][32][32][128] (LeakyReLU or none on
 * load), RGB side packed to 8 channels (k = 8, 3 real; rc->ld = 8).  Other shapes run the two calls
 * (a->y must then be set).  vae_convT2d_bwd of that layer with dw_inner = 3 runs its data, weight
 * and bias gradients in one pass (workspace: vae_convT2d_workspace_size(a, VAE_OP_BWD)); the input
 * Conv2d(3 -> 128, k4 s2) weight gradient of the same network (vae_conv2d_bwd_filter, c = 8 packed,
 * dw_inner = 3) likewise has its own kernel. */
int vae_convT2d_fwd_recon(const vae_conv_args* a, const vae_recon_args* rc, void* stream);
/* --- Linear (fc_mu/fc_var vanilla_vae.py:36-37,89-90; decoder_input :43,101) -------- */
int vae_linear_fwd(const vae_linear_args* a, void* stream);
int vae_linear_bwd_data(const vae_linear_args* a, void* stream);
int vae_linear_bwd_filter(const vae_linear_args* a, void* stream);
/* --- final Conv2d + Tanh + reconstruction SSE (vanilla_vae.py:73-75, :140) ---------- */
int vae_head_fwd(const vae_head_args* a, void* stream);
int vae_head_bwd_data(const vae_head_args* a, void* stream);
int vae_head_bwd_filter(const vae_head_args* a, void* stream);
/* both halves of the head backward in one pass over the input tile (bf16 MFMA path; the fp32
 * path runs bwd_data then bwd_filter) */
int vae_head_bwd(const vae_head_args* a, void* stream);
/* --- BatchNorm finalisation (see vae_bn_args) ------------------------------------------ */
int vae_bn_finalize(const vae_bn_args* a, void* stream);
/* --- reparameterization (vanilla_vae.py:107-117): z = eps*exp(.5*logvar) + mu,
 *     row r uses mu row r/samples.  z is written in `dtype`. */
int vae_reparam_fwd(int32_t dtype, int32_t rows, int32_t samples, int32_t latent,
                    const float* mulv, const float* eps, void* z, void* stream);
/* --- VectorQuantizer (vq_vae.py:24-55), see vae_vq_args ------------------------------ */
int vae_vq_fwd(const vae_vq_args* a, void* stream);
int vae_vq_bwd(const vae_vq_args* a, void* stream);
/* --- Tanh output + reconstruction SSE (vq_vae.py:156-160, :203), see vae_recon_args --- */
int vae_recon_fwd(const vae_recon_args* a, void* stream);
int vae_recon_bwd(const vae_recon_args* a, void* stream);
/* --- channel padding for 3-channel layers (the RGB image and the RGB output conv) -----------
 * The packed GEMM paths need channel counts that are multiples of 8, so the 3-channel tensors
 * at both ends of the network are carried padded to 8 channels (zeros):
 *   vae_nchw_to_nhwc_pad: x fp32 NCHW [n][c][h][w] (c <= cp) -> y NHWC [n][h][w][cp] in dtype;
 *   vae_pad_channels:     dst[r][j] = j < c ? src[r][j] : 0, rows x cp (dtype: both sides;
 *                         weights in the bf16 copy, biases fp32);
 *   vae_unpad_accumulate: dst[r][j] += src[r][j] for j < c (fp32; padded weight gradient ->
 *                         the parameter's gradient). */
int vae_nchw_to_nhwc_pad(int32_t dtype, int32_t n, int32_t c, int32_t h, int32_t w, int32_t cp, const float* x,
                         void* y, void* stream);
int vae_pad_channels(int32_t dtype, int64_t rows, int32_t c, int32_t cp, const void* src, void* dst, void* stream);
int vae_unpad_accumulate(int64_t rows, int32_t cp, int32_t c, const float* src, float* dst, void* stream);
/* --- ELBO terms + backward seeds (vanilla_vae.py:124-146 and variants) -------------- */
int vae_elbo_fwd(const vae_elbo_args* a, void* stream);
/* --- Adam (experiment.py:308-311; torch.optim.Adam semantics), flat fp32 buffers.
 *     step/lr are device scalars so the call can be replayed from a graph.  When
 *     p_lowp != NULL the updated parameters are also written as bf16 (weight copies). --- */
int vae_adam_step(int64_t n, float* p, const float* g, float* m, float* v,
                  const int32_t* step, const float* lr, double beta1, double beta2, float eps,
                  float weight_decay, void* p_lowp, void* stream);
/* --- Deferred weight-gradient reductions + Adam in one launch ---------------------------
 * A bf16 call with defer_reduce set leaves a weight gradient as fp32 partial rows and records
 *   dst[j] = sum_{r < rows} slab[r * ld + j]   (j < count, rows summed in ascending order)
 * in a per-host-thread list instead of launching its reduction (the fused ELBO of vae_head_args
 * likewise).  vae_deferred_take copies the list out (up to max descriptors; returns how many there
 * are; *has_elbo / *elbo: the deferred loss, if any) and clears it; vae_deferred_reset clears it.
 * A gradient deferred again before it was taken (the same dst) replaces its earlier descriptor.
 * Workspace queries record nothing.
 * A descriptor with rows == 0 (slab NULL) records a gradient the call wrote whole itself (one K
 * slice: no reduction left); vae_adam_step_ex treats it as a plain gradient, and a step head may
 * leave it out of its zeroing (vae_step_begin_args.keep).
 * vae_adam_step_ex: vae_adam_step over the flat buffers, with the slab descriptors reduced in the
 * same launch (each dst inside g: the reduced gradient is written there, then that element's Adam
 * update runs), and the deferred loss evaluated by one extra workgroup — the step's three slab
 * reductions (head, full-resolution ConvT, grouped weight gradients) and the loss without launches
 * of their own (models/vanilla_vae.py:124-146, experiment.py:308-311). */
#define VAE_SLAB_MAX 32
typedef struct vae_grad_slab {
  float* dst;              /* inside vae_adam_args.g */
  int64_t count;
  const float* slab;
  int32_t rows;
  int64_t ld;              /* floats between rows */
} vae_grad_slab;
int vae_deferred_reset(void);
int32_t vae_deferred_take(vae_grad_slab* out, int32_t max, vae_elbo_args* elbo, int32_t* has_elbo);
typedef struct vae_adam_args {
  int64_t n;
  float* p; float* g; float* m; float* v;
  const int32_t* step; const float* lr;
  double beta1, beta2;
  float eps, weight_decay;
  void* p_lowp;
  int32_t nslab;
  vae_grad_slab slab[VAE_SLAB_MAX];
  int32_t has_elbo;
  vae_elbo_args elbo;
} vae_adam_args;
int vae_adam_step_ex(const vae_adam_args* a, void* stream);
/* --- fp32 -> bf16 copy (weight copies when the optimizer is not vae_adam_step) -------- */
int vae_cast_bf16(int64_t n, const float* src, void* dst, void* stream);
/* --- swapped-axes bf16 weight copies (vae_conv_args.wt_t), several tensors per launch:
 *     dst[b][t][a] = bf16(src[a][t][b]), src fp32 [a][rs][b] (the master weights), dst bf16
 *     [b][rs][a].  A ConvTranspose2d weight [c][r][s][k] gives the [k][r][s][c] rows its bf16
 *     forward GEMM reads; a Conv2d weight [k][r][s][c] the [c][r][s][k] rows of its data
 *     gradient.  Replaces the per-call rebuild at the end of the workspace. ------------ */
#define VAE_SWAP_MAX 16
typedef struct vae_swap_desc {
  const void* src;
  void* dst;
  int32_t a, rs, b;
  int32_t src_dtype;                 /* VAE_F32 (the master weights) or VAE_BF16 (their bf16 copy:
                                        half the bytes, the same rounded values) */
} vae_swap_desc;
int vae_swap_axes(int32_t count, const vae_swap_desc* descs, void* stream);
/* --- workspace queries ----------------------------------------------------
 * Bytes of workspace the call `op` would use with these arguments — pass exactly the arguments
 * the call will get (pointers included: alignment selects the kernel path; the workspace fields
 * are ignored).  The query runs the call's own planning without launching anything (no device,
 * no stream needed).  A call given a non-NULL workspace smaller than this fails with
 * VAE_E_BADARG; a NULL workspace selects the plan that uses none (no split-K slabs, no staged
 * weight copy, atomics for the head's filter partials).  Replaces the fixed host-side constant
 * of round 1 and the silent split-K downgrade on a short workspace. */
enum vae_op { VAE_OP_FWD = 0, VAE_OP_BWD_DATA = 1, VAE_OP_BWD_FILTER = 2, VAE_OP_BWD = 3 /* head: both halves */ };
int vae_conv2d_workspace_size(const vae_conv_args* a, int32_t op, size_t* bytes);
int vae_convT2d_workspace_size(const vae_conv_args* a, int32_t op, size_t* bytes);
int vae_linear_workspace_size(const vae_linear_args* a, int32_t op, size_t* bytes);
int vae_head_workspace_size(const vae_head_args* a, int32_t op, size_t* bytes);
/* --- weight gradients of several layers in one call ------------------------------------
 * The vae_conv2d_bwd_filter / vae_convT2d_bwd_filter calls of one gradient bucket of the
 * backward (the reference's loss.backward() over models/vanilla_vae.py:25-75, experiment.py:45-86):
 * items[i] holds the arguments that call would get, kinds[i] says which entry point.  The results
 * equal the calls made one after another; the bf16 GEMMs of layers sharing a tile class run as one
 * grouped launch (a layer's weight gradient is read only by the optimizer, so the layers of a
 * bucket can run concurrently).  The items' own workspace fields are ignored: `workspace` holds
 * every item's workspace back to back (vae_conv_bwd_filter_batch_workspace_size). */
enum vae_layer_kind { VAE_LAYER_CONV2D = 0, VAE_LAYER_CONVT2D = 1 };
int vae_conv_bwd_filter_batch(int32_t n, const int32_t* kinds, const vae_conv_args* const* items,
                              void* workspace, int64_t workspace_bytes, void* stream);
int vae_conv_bwd_filter_batch_workspace_size(int32_t n, const int32_t* kinds, const vae_conv_args* const* items,
                                             size_t* bytes);
/* --- the bookkeeping of one training step (experiment.py:45-86 training_step after the loss):
 * one launch instead of a dozen small tensor ops.
 *   terms[0..nterms) = src_terms[0..nterms)                 (the logged loss terms)
 *   per[b] = mean_s per_img[b*samples + s]                  (per-image MSE, experiment.py:58-62)
 *   the running extremes (experiment.py:65-84): if max_b per[b] > best[0] (strictly; the first
 *   index wins ties) then best[0] = that loss, at[0..1] = {step, b}, hi_img = img[b],
 *   hi_recon = recon[b*samples] (first sample); the same with min / best[1] / at[2..3] / lo_*.
 * img: [batch][img_elems] fp32, recon: [batch*samples][img_elems] fp32; one workgroup. */
typedef struct vae_record_args {
  int32_t batch, samples, img_elems, nterms, step;
  const float* src_terms; float* terms;
  const float* per_img; float* per;
  const float* img; const float* recon;
  float* best; int32_t* at;            /* best[2] = {highest, lowest}, at[4] */
  float* hi_img; float* hi_recon; float* lo_img; float* lo_recon;
} vae_record_args;
int vae_step_record(const vae_record_args* a, void* stream);
/* --- start of a training step: zero `bytes` at `zero` and ++*step ------------------ */
int vae_step_begin(void* zero, int64_t bytes, int32_t* step, void* stream);

/* --- start of a training step in ONE launch: what vae_step_begin, vae_nchw_to_nhwc_pad and up to
 *     VAE_PAD_MAX vae_pad_channels calls do (the zero region and ++*step, the RGB image as 8
 *     zero-padded NHWC channels, the padded first-layer weight copies), as block ranges of one grid.
 *     Replaces the three dependent launches at the head of every step (experiment.py:45-49 → the
 *     inputs of models/vanilla_vae.py:84; 16.5 us of launches in profiles/r3a). ---------------- */
#define VAE_PAD_MAX 4
typedef struct vae_pad_desc {
  int64_t rows;
  int32_t c, cp;                     /* dst[r][j] = j < c ? src[r][j] : 0, j < cp */
  const void* src;                   /* dtype (the step's weight copies) */
  void* dst;
} vae_pad_desc;
typedef struct vae_step_begin_args {
  void* zero;                        /* 16-B aligned; bytes may be 0 */
  int64_t bytes;
  int32_t* step;                     /* ++ once, or NULL */
  int32_t dtype;                     /* of the padded image and the pad descriptors */
  int32_t n, c, h, w, cp;            /* image: fp32 NCHW x -> NHWC y with cp channels (x NULL: none) */
  const float* x;
  void* y;
  int32_t npad;
  vae_pad_desc pad[VAE_PAD_MAX];
  /* up to VAE_SWAP_MAX swapped-axes weight copies (what vae_swap_axes does with these descriptors),
   * refreshed from the fp32 weights as the step starts — after the previous step's optimizer,
   * before the first GEMM that reads them — instead of a launch of their own behind the optimizer */
  int32_t nswap;
  vae_swap_desc swap[VAE_SWAP_MAX];
  /* byte ranges [off, off + bytes) of the zero region left as they are: gradients the step writes
   * whole instead of accumulating (defer_reduce: the deferred reductions' destinations and the
   * weight gradients a call writes itself — vae_deferred_take lists both); 16-byte multiples */
  int32_t nkeep;
  struct { int64_t off, bytes; } keep[VAE_SLAB_MAX];
} vae_step_begin_args;
int vae_step_begin_ex(const vae_step_begin_args* a, void* stream);

/* --- the VAE bottleneck, bf16, as two launches each way (VanillaVAE / BetaVAE / IWAE training):
 *   vae_latent_fc_fwd   mulv += act(x)·W1^T (+ b1)      fc_mu|fc_var (vanilla_vae.py:36-37, :89-90).
 *                       x: the last encoder map, stored pre-BatchNorm, NHWC [batch][in_features];
 *                       x_xf its BatchNorm+LeakyReLU (running statistics updated when set).  K is
 *                       split over workgroups that add with fp32 atomics: mulv must be ZERO on entry
 *                       (the step's zero region).  Replaces vae_linear_fwd + its split-K finalize.
 *   vae_latent_dec_fwd  z = mu + eps*exp(logvar/2)       reparameterize (vanilla_vae.py:107-117; row
 *                       r of z uses mu row r/samples), z written bf16 [batch*samples][latent], and
 *                       h = z·W2^T + b2                  decoder_input (vanilla_vae.py:43, :101), bf16
 *                       [batch*samples][out_features] — one launch for vae_reparam_fwd +
 *                       vae_linear_fwd.  eps NULL: z is an input (decode of a given z).
 *   vae_latent_dec_bwd  d[mu|logvar] += the reparameterization backward of dz = dh·W2 plus the KL
 *                       seed kl_coef (as vae_linear_bwd_data with mulv set; dmulv accumulated, zero on
 *                       entry), dW2 += dh^T·z, db2 += sum_r dh — one launch for the decoder_input
 *                       bwd_data (+ finalize) and bwd_filter.
 *   vae_latent_fc_bwd   dx = dx_epi-backward(dmulv·W1) of x (BatchNorm+LeakyReLU backward; sums
 *                       Sg -> dx_dbeta, Sg*xhat -> dx_dgamma replicas, as vae_linear_bwd_data),
 *                       dW1 += dmulv^T·act(x), db1 += sum_r dmulv — one launch for fc bwd_data and
 *                       bwd_filter.
 * Shapes: latent % 32 == 0, latent <= 256; x_xf.channels % 128 == 0 and in_features a multiple of
 * it; out_features % 64 == 0; weights native ([2*latent][in_features], [out_features][latent]). */
typedef struct vae_latent_args {
  int32_t dtype;                     /* VAE_BF16 */
  int32_t batch, samples, latent;
  int32_t in_features, out_features;
  const void* x;                     /* [batch][in_features] bf16, stored pre-activation */
  vae_xform x_xf;                    /* BN_ACT (the encoder's last BatchNorm+LeakyReLU) */
  const void* w1;                    /* fc_mu|fc_var [2*latent][in_features] bf16 */
  const float* b1;
  float* mulv;                       /* [batch][2*latent] fp32, accumulated */
  const float* eps;                  /* [batch*samples][latent] or NULL */
  void* z;                           /* [batch*samples][latent] bf16 (out, or in when eps NULL) */
  const void* w2;                    /* decoder_input [out_features][latent] bf16 */
  const float* b2;
  void* h;                           /* [batch*samples][out_features] bf16 */
  const void* dh;                    /* backward: dL/dh [batch*samples][out_features] bf16 */
  const float* kl_coef;              /* [batch*samples] or NULL */
  float* dmulv;                      /* [batch][2*latent], accumulated */
  float* dw2; float* db2;            /* fp32, accumulated */
  void* dx;                          /* [batch][in_features] bf16: gradient w.r.t. x's BN output */
  vae_xform dx_epi;                  /* BN_ACT of x, aux = x */
  float* dx_dgamma; float* dx_dbeta;
  int32_t sum_reps, sum_rstride;
  float* dw1; float* db1;            /* fp32, accumulated */
  /* eps_gen = 1: vae_latent_dec_fwd DRAWS eps ~ N(0,1) itself (torch.randn_like(std) of
   * reparameterize, vanilla_vae.py:116, every step) and writes it to `eps` (an output then) for the
   * backward: Philox4x32-10 keyed by eps_seed, counter (element/4, *eps_step, 0x5EED, 0), then
   * Box-Muller on each pair of words.  *eps_step is the device step counter vae_step_begin_ex
   * advances, so every replay of a captured step draws fresh noise.  eps_gen = 0: eps is read. */
  const int32_t* eps_step;
  uint64_t eps_seed;
  int32_t eps_gen;
} vae_latent_args;
int vae_latent_fc_fwd(const vae_latent_args* a, void* stream);
int vae_latent_dec_fwd(const vae_latent_args* a, void* stream);
int vae_latent_dec_bwd(const vae_latent_args* a, void* stream);
int vae_latent_fc_bwd(const vae_latent_args* a, void* stream);

/* --- Materialised per-channel transform (the operand of the large transform-free GEMMs) ---------
 * out[r][c] = xf(x[r][c]) in bf16, same [rows][channels] layout: lrelu(BN(y)) of a forward
 * activation (xf BN_ACT; running statistics updated when set — this call is then the BatchNorm's
 * first consumer), lrelu(y) (ACT), or the BatchNorm-backward gradient A g + B y + C of the stored
 * gradient g (xf BN_DY, aux = y; dgamma_out / dbeta_out and the closed-form conv-bias gradient db
 * published when set, as a weight-gradient call applying BN_DY itself would).  The Autoencoder's
 * wide layers (models/autoencoder.py:16-86) and the VQ-VAE's strided 4x4 layers take it so their
 * GEMMs run on the LDS-DMA pipeline (vae_bgemm.hip) with plain operands. */
typedef struct vae_bn_apply_args {
  int32_t dtype;             /* VAE_BF16 */
  int64_t rows;
  int32_t channels;          /* % 8 */
  const void* x;
  vae_xform xf;
  float* db;
  void* out;
} vae_bn_apply_args;
int vae_bn_apply(const vae_bn_apply_args* a, void* stream);

/* --- The Autoencoder's other reconstruction losses (forward + backward seed) ----------------------
 * VAE_RLOSS_CENTER: mean(mask * (recon - target)^2) over n*c*h*w (models/autoencoder.py:95-146,
 *   :259-265; mask = create_center_weight_mask, [h][w]).
 * VAE_RLOSS_MSSIM: 1 - prod_{l < L-1} cs_l^w_l * ssim_{L-1}^w_{L-1} over `levels` avg-pooled levels,
 *   depthwise window = outer(window, window) with zero padding window_size/2, C1 = 1e-4, C2 = 9e-4,
 *   size_average, (s + 1) / 2 when normalize (models/mssim_vae.py:182-282, autoencoder.py:266-267).
 *   window[] is the reference's normalised 1-D window (its Gaussian with a POSITIVE exponent).
 * Writes out[0] = loss, out[1] = Reconstruction_Loss (= loss), out[2] = 0; grad (if set) =
 * grad_scale * dL/drecon (NCHW fp32), the seed of the fused backward (vae_head_args.grad_recon /
 * vae_recon_args.grad_recon); per_img (if set with sse) = sse / (c*h*w), the per-image MSE of
 * experiment.py:60-62.  Planes of up to 64 x 64; workspace: vae_recon_loss_workspace_size. */
enum vae_recon_loss_kind { VAE_RLOSS_CENTER = 0, VAE_RLOSS_MSSIM = 1 };
typedef struct vae_recon_loss_args {
  int32_t kind;
  int32_t n, c, h, w;
  const float* recon;        /* NCHW fp32 (img1) */
  const float* target;       /* NCHW fp32 (img2) */
  const float* mask;         /* CENTER: [h][w] */
  float window[16];          /* MSSIM: 1-D window (window_size <= 15, odd) */
  int32_t window_size;
  int32_t levels;            /* MSSIM: 5 */
  float level_weights[8];    /* MSSIM: 0.0448, 0.2856, 0.3001, 0.2363, 0.1333 */
  int32_t normalize;
  int32_t size_average;      /* must be 1 (the reference's default) */
  float* grad;
  float grad_scale;
  float* out;                /* [3] */
  const float* sse;          /* optional [n] */
  float* per_img;            /* optional [n] */
  float* workspace;
  int64_t workspace_bytes;
} vae_recon_loss_args;
int vae_recon_loss(const vae_recon_loss_args* a, void* stream);
int vae_recon_loss_workspace_size(const vae_recon_loss_args* a, size_t* bytes);

#ifdef __cplusplus
}
#endif
#endif /* VAEHIP_H */
