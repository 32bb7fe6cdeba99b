// C-ABI entry points of Conv2d (encoder blocks, models/vanilla_vae.py:28-29 run at :84).
#include "vae_launch.hpp"
#include "vae_wgrad.hpp"

using namespace vae;

// y[n,p,q,k] = Σ_{r,s,c} xf(x)[n, p*S-P+r, q*S-P+s, c] · W[k][r][s][c] + b[k]
extern "C" int vae_conv2d_fwd(const vae_conv_args* a, void* stream) {
  if (!geom_ok(a, "conv2d_fwd") || !a->x || !a->wt || !a->y) return fail(VAE_E_BADARG, "conv2d_fwd: null tensor");
  if (!xf_ok(a->x_xf, "conv2d_fwd.x")) return VAE_E_BADARG;
  GemmParams p = base_params();
  p.M = a->n * a->p * a->q; p.N = a->k; p.K = a->r * a->r * a->c;
  p.a_ptr = a->x; p.a_xf = sanitize(a->x_xf); p.g_nchw = a->x_nchw_f32;
  p.b_ptr = a->wt; p.b_ld = p.K;
  p.gn = a->n; p.gh = a->h; p.gw = a->w; p.gc = a->c; p.gp = a->p; p.gq = a->q;
  p.gr = a->r; p.gs = a->stride; p.gpad = a->pad;
  p.out = a->y; p.out_ld = a->k; p.bias = a->bias; p.sum = a->y_sum; p.sumsq = a->y_sumsq;
  p.sum_reps = a->sum_reps; p.sum_rstride = a->sum_rstride;
  p.residual = a->residual; p.res_xf = sanitize(a->residual_xf);
  if (int rc = check_finalize(a->bn_finalize, a->bn_counter, "conv2d_fwd")) return rc;
  return then_finalize(launch<A_CONV, B_NK, E_STORE, false, false, true>(a->dtype, a->x_nchw_f32 != 0, false, p, a->split_k, a->workspace,
                                             a->workspace_bytes, (hipStream_t)stream), a->bn_finalize, (hipStream_t)stream);
}

// dx[n,h,w,c] = Σ_{r,s,k: h = p*S-P+r} dy'[n,p,q,k] · W[k][r][s][c]  (transposed conv of dy);
// epilogue: [+ residual gradient], g = dx·act'(z) of x's BatchNorm/LeakyReLU, Σg -> dβ, Σg·x̂ -> dγ
extern "C" int vae_conv2d_bwd_data(const vae_conv_args* a, void* stream) {
  if (!geom_ok(a, "conv2d_bwd_data") || !a->dy || !a->wt || !a->dx) return fail(VAE_E_BADARG, "conv2d_bwd_data: null tensor");
  if (!xf_ok(a->dy_xf, "conv2d_bwd_data.dy") || !epi_ok(a->dx_epi, "conv2d_bwd_data.epi")) return VAE_E_BADARG;
  if (a->x_nchw_f32) return fail(VAE_E_UNSUPPORTED, "conv2d_bwd_data: no gradient for the NCHW image input");
  const int S = a->stride;
  if (a->h % S || a->w % S || a->h / S != a->p || a->w / S != a->q)
    return fail(VAE_E_BADSHAPE, "conv2d_bwd_data: needs h == p*stride (got h=%d p=%d S=%d)", a->h, a->p, S);
  const long wbytes = (long)a->k * a->r * a->r * a->c * 2;
  if (S == 1 && a->dtype == VAE_BF16 && a->c % 8 == 0 && a->k % 8 == 0 && a->workspace &&
      a->workspace_bytes >= 2 * wbytes && !getenv("VAE_NO_DGRAD_FLIP")) {
    // stride 1: dx = conv(dy, W') with W'[c][r][s][k] = W[k][R-1-r][R-1-s][c] and pad R-1-P — the
    // forward conv path (k-contiguous weight rows, packed im2col gather of dy) instead of the
    // phase-gather with k-strided weights.  W' lives at the end of the workspace.
    char* ws = static_cast<char*>(a->workspace);
    const long wsoff = ((a->workspace_bytes - wbytes) / 256) * 256;
    __bf16* wf = reinterpret_cast<__bf16*>(ws + wsoff);
    int rc = flip_weights_launch(static_cast<const __bf16*>(a->wt), wf, a->k, a->r, a->c, (hipStream_t)stream);
    if (rc) return rc;
    GemmParams p = base_params();
    p.M = a->n * a->h * a->w; p.N = a->c; p.K = a->r * a->r * a->k;
    p.a_ptr = a->dy; p.a_xf = sanitize(a->dy_xf);
    p.b_ptr = wf; p.b_ld = p.K;
    p.gn = a->n; p.gh = a->p; p.gw = a->q; p.gc = a->k; p.gp = a->h; p.gq = a->w;
    p.gr = a->r; p.gs = 1; p.gpad = a->r - 1 - a->pad;
    p.out = a->dx; p.out_ld = a->c;
    p.epi_xf = sanitize(a->dx_epi); p.dgamma = a->dx_dgamma; p.dbeta = a->dx_dbeta;
    p.sum_reps = a->sum_reps; p.sum_rstride = a->sum_rstride;
    p.residual = a->residual;
    if (p.epi_xf.kind == VAE_X_BN_ACT && (!p.dgamma || !p.dbeta)) return fail(VAE_E_BADARG, "conv2d_bwd_data: dgamma/dbeta");
    if (int rc2 = check_finalize(a->bn_finalize, a->bn_counter, "conv2d_bwd_data")) return rc2;
    return then_finalize(launch<A_CONV, B_NK, E_BNBWD, true, false>(a->dtype, false, false, p, a->split_k, ws, wsoff, (hipStream_t)stream), a->bn_finalize, (hipStream_t)stream);
  }
  GemmParams p = base_params();
  if (!make_taps(p, S, a->r, a->pad)) return fail(VAE_E_UNSUPPORTED, "conv2d_bwd_data: stride/kernel");
  p.nphase = S * S;
  p.M = a->n * (a->h / S) * (a->w / S); p.N = a->c; p.K = 0;
  p.a_ptr = a->dy; p.a_xf = sanitize(a->dy_xf);
  p.b_ptr = a->wt; p.b_ld = a->c; p.b_taps = 1;
  p.gn = a->n; p.gh = a->p; p.gw = a->q; p.gc = a->k;          // gathered tensor = dy
  p.gp = a->h / S; p.gq = a->w / S; p.gr = a->r; p.gs = S; p.gpad = a->pad; p.gho = a->h; p.gwo = a->w;
  p.out = a->dx; p.out_ld = a->c; p.out_phase = 1;
  p.epi_xf = sanitize(a->dx_epi); p.dgamma = a->dx_dgamma; p.dbeta = a->dx_dbeta;
  p.sum_reps = a->sum_reps; p.sum_rstride = a->sum_rstride;
  p.residual = a->residual;                                    // + gradient through a skip connection
  if (p.epi_xf.kind == VAE_X_BN_ACT && (!p.dgamma || !p.dbeta)) return fail(VAE_E_BADARG, "conv2d_bwd_data: dgamma/dbeta");
  if (int rc = check_finalize(a->bn_finalize, a->bn_counter, "conv2d_bwd_data")) return rc;
  return then_finalize(launch<A_CONVT, B_KN, E_BNBWD, true, false>(a->dtype, false, false, p, a->split_k, a->workspace, a->workspace_bytes,
                                        (hipStream_t)stream), a->bn_finalize, (hipStream_t)stream);
}

// dW[k][r][s][c] += Σ_{n,p,q} dy'[n,p,q,k] · xf(x)[n, p*S-P+r, q*S-P+s, c];  db[k] += Σ dy'
extern "C" int vae_conv2d_bwd_filter(const vae_conv_args* a, void* stream) {
  if (!geom_ok(a, "conv2d_bwd_filter") || !a->dy || !a->x || !a->dw) return fail(VAE_E_BADARG, "conv2d_bwd_filter: null tensor");
  if (!xf_ok(a->dy_xf, "conv2d_bwd_filter.dy") || !xf_ok(a->x_xf, "conv2d_bwd_filter.x")) return VAE_E_BADARG;
  const bool closed = a->db && a->dy_xf.kind == VAE_X_BN_DY;   // Σdy from the BN sums
  if (!a->x_nchw_f32 && !closed &&
      wgrad_ok(a->dtype, a->dy_xf, a->x_xf, (long)a->n * a->p * a->q * a->k, (long)a->n * a->h * a->w * a->c, a->k, a->c)) {
    // bf16 fast path: U = dy (output grid, m = k), V = x (input grid, j = c)
    WgradParams w;
    memset(&w, 0, sizeof(w));
    w.u = a->dy; w.u_xf = sanitize(a->dy_xf); w.v = a->x; w.v_xf = sanitize(a->x_xf);
    w.n = a->n; w.hu = a->p; w.wu = a->q; w.M = a->k; w.hv = a->h; w.wv = a->w; w.J = a->c;
    w.R = a->r; w.S = a->stride; w.P = a->pad; w.dw = a->dw;
    int rc = wgrad_launch(w, (hipStream_t)stream);
    if (rc || !a->db) return rc;
    return column_sum_launch(a->dtype, a->dy, (long)a->n * a->p * a->q, a->k, a->db, (hipStream_t)stream);
  }
  GemmParams p = base_params();
  const int Nw = a->r * a->r * a->c;
  const bool ones = a->db && !closed;                           // Σdy as an extra GEMM column
  p.M = a->k; p.N = Nw + (ones ? 1 : 0); p.K = a->n * a->p * a->q;
  p.ones_col = ones ? Nw : -1; p.bias_grad = ones ? a->db : nullptr;
  p.dbc = closed ? a->db : nullptr; p.dbc_from_b = 0;
  p.a_ptr = a->dy; p.a_ld = a->k; p.a_xf = sanitize(a->dy_xf);
  p.b_ptr = a->x; p.b_xf = sanitize(a->x_xf); p.g_nchw = a->x_nchw_f32;
  p.gn = a->n; p.gh = a->h; p.gw = a->w; p.gc = a->c; p.gp = a->p; p.gq = a->q;
  p.gr = a->r; p.gs = a->stride; p.gpad = a->pad;
  p.out = a->dw; p.out_ld = Nw;
  return launch<A_KM, B_GATHER, E_ACC, true, false, false, true>(a->dtype, false, a->x_nchw_f32 != 0, p, a->split_k, nullptr, 0,
                                                    (hipStream_t)stream);
}
