// C-ABI entry points of Conv2d (encoder blocks, models/vanilla_vae.py:28-29 run at :84).
#include "vae_launch.hpp"
#include "vae_wgrad.hpp"
#include "vae_wgemm.hpp"
#include "vae_c3.hpp"
#include "vae_rgb.hpp"

using namespace vae;

// dW[k][r][s][c] += Σ_{n,p,q} dy'[n,p,q,k] · xf(x)[n, p*S-P+r, q*S-P+s, c];  db[k] += Σ dy'
extern "C" int vae_conv2d_bwd_filter(const vae_conv_args* a, void* stream) {
  if (!geom_ok(a, "conv2d_bwd_filter") || !a->dy || !a->x || !a->dw) return fail(VAE_E_BADARG, "conv2d_bwd_filter: null tensor");
  if (!xf_ok(a->dy_xf, "conv2d_bwd_filter.dy") || !xf_ok(a->x_xf, "conv2d_bwd_filter.x")) return VAE_E_BADARG;
  const bool closed = a->db && a->dy_xf.kind == VAE_X_BN_DY;   // Σdy from the BN sums
  if (a->dtype == VAE_BF16) {                                   // the VQ-VAE's input Conv2d(3 -> C, k4 s2)
    const int rc = rgb_in_wgrad_launch(a, (hipStream_t)stream);
    if (rc != kHeadFallback) return rc;
  }
  // 3x3 stride-1 on a 16 x 16 grid (the VQ-VAE's residual stacks): image-group tiles with the
  // halo patch staged once per image (vae_c3.hip); needs a workspace for the partial slabs
  if (a->dtype == VAE_BF16 && !a->x_nchw_f32 && c3_enabled() && (a->workspace || querying()) &&
      c3w_shape_ok(a->n, a->h, a->w, a->p, a->q, a->r, a->stride, a->pad, a->k, a->c) &&
      a->dy_xf.kind == VAE_X_NONE && (a->x_xf.kind == VAE_X_NONE || a->x_xf.kind == VAE_X_ACT) &&
      (a->dw_inner <= 0 || a->dw_inner == a->c)) {
    C3WArgs c;
    c.u = a->dy; c.v = a->x; c.v_act = a->x_xf.kind == VAE_X_ACT; c.v_slope = a->x_xf.slope;
    c.dw = static_cast<float*>(a->dw); c.n = a->n; c.M = a->k; c.J = a->c;
    int rc = c3w_launch(c, a->workspace, a->workspace_bytes, (hipStream_t)stream);
    if (rc || !a->db) return rc;
    return column_sum_launch(a->dtype, a->dy, (long)a->n * a->p * a->q, a->k, a->db, (hipStream_t)stream);
  }
  if (a->dtype == VAE_BF16 && !a->x_nchw_f32 && c3_enabled() && (a->workspace || querying()) &&
      c1w_shape_ok(a->n, a->h, a->w, a->p, a->q, a->r, a->stride, a->pad, a->k, a->c) &&
      a->dy_xf.kind == VAE_X_NONE && (a->x_xf.kind == VAE_X_NONE || a->x_xf.kind == VAE_X_ACT) &&
      (a->dw_inner <= 0 || a->dw_inner == a->c)) {
    C3WArgs c;
    c.u = a->dy; c.v = a->x; c.v_act = a->x_xf.kind == VAE_X_ACT; c.v_slope = a->x_xf.slope;
    c.dw = static_cast<float*>(a->dw); c.n = a->n; c.M = a->k; c.J = a->c;
    int rc = c1w_launch(c, a->workspace, a->workspace_bytes, (hipStream_t)stream);
    if (rc || !a->db) return rc;
    return column_sum_launch(a->dtype, a->dy, (long)a->n * a->p * a->q, a->k, a->db, (hipStream_t)stream);
  }
  {
    // bf16 weight-gradient GEMM (vae_wgemm.hpp)
    WgParams w;
    bool closed_wg;
    if (conv_wg_params(a, false, &w, &closed_wg)) {
      int rc = wg2_launch(w, a->workspace, a->workspace_bytes, (hipStream_t)stream);
      if (rc || !a->db || closed_wg) return rc;
      return column_sum_launch(a->dtype, a->dy, (long)a->n * a->p * a->q, a->k, a->db, (hipStream_t)stream);
    }
  }
  if (a->dw_inner > 0 && a->dw_inner < a->c)
    return fail(VAE_E_UNSUPPORTED, "conv2d_bwd_filter: dw_inner %d < c %d needs the bf16 weight-gradient GEMM path",
                a->dw_inner, a->c);
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
  p.det = a->deterministic;
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
  return launch<A_KM, B_GATHER, E_ACC, true, false, false, true>(a->dtype, false, a->x_nchw_f32 != 0, p, a->split_k,
                                                    p.det ? a->workspace : nullptr, p.det ? a->workspace_bytes : 0,
                                                    (hipStream_t)stream);
}
