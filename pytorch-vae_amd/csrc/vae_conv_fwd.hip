// C-ABI entry points of Conv2d (encoder blocks, models/vanilla_vae.py:28-29 run at :84).
#include "vae_launch.hpp"
#include "vae_wgrad.hpp"
#include "vae_c3.hpp"

using namespace vae;

// y[n,p,q,k] = Σ_{r,s,c} xf(x)[n, p*S-P+r, q*S-P+s, c] · W[k][r][s][c] + b[k]
extern "C" int vae_conv2d_fwd(const vae_conv_args* a, void* stream) {
  if (!geom_ok(a, "conv2d_fwd") || !a->x || !a->wt || !a->y) return fail(VAE_E_BADARG, "conv2d_fwd: null tensor");
  if (!xf_ok(a->x_xf, "conv2d_fwd.x")) return VAE_E_BADARG;
  // 1x1 stride-1 convs (the VQ-VAE ResidualLayer's Conv1x1 + skip add): pixel-tile kernel
  if (a->dtype == VAE_BF16 && !a->x_nchw_f32 && c3_enabled() && a->r == 1 && a->stride == 1 && a->pad == 0 &&
      a->h == a->p && a->w == a->q && p1_shape_ok((long)a->n * a->p * a->q, a->c, a->k) &&
      (a->x_xf.kind == VAE_X_NONE || a->x_xf.kind == VAE_X_ACT) &&
      (a->residual_xf.kind == VAE_X_NONE || a->residual_xf.kind == VAE_X_ACT) && !a->y_sum && !a->y_sumsq &&
      !a->bn_finalize && a->split_k <= 0) {
    P1Args c;
    memset(&c, 0, sizeof(c));
    c.a = a->x; c.a_act = a->x_xf.kind == VAE_X_ACT; c.a_slope = a->x_xf.slope;
    c.b = a->wt; c.out = a->y; c.bias = a->bias;
    c.residual = a->residual; c.res_act = a->residual && a->residual_xf.kind == VAE_X_ACT; c.res_slope = a->residual_xf.slope;
    c.M = (long)a->n * a->p * a->q; c.C = a->c; c.N = a->k;
    return p1_launch(c, (hipStream_t)stream);
  }
  // 3x3 stride-1 convs on a 16 x 16 grid (the VQ-VAE's residual stacks): image-tile kernel
  if (a->dtype == VAE_BF16 && !a->x_nchw_f32 && c3_enabled() &&
      c3_shape_ok(a->n, a->h, a->w, a->p, a->q, a->r, a->stride, a->pad, a->c, a->k) &&
      (a->x_xf.kind == VAE_X_NONE || a->x_xf.kind == VAE_X_ACT) && !a->y_sum && !a->y_sumsq && !a->residual &&
      !a->bn_finalize && a->split_k <= 0) {
    C3Args c;
    memset(&c, 0, sizeof(c));
    c.a = a->x; c.a_act = a->x_xf.kind == VAE_X_ACT; c.a_slope = a->x_xf.slope;
    c.b = a->wt; c.flip = 0; c.out = a->y; c.bias = a->bias;
    c.n = a->n; c.C = a->c; c.N = a->k;
    return c3_launch(c, (hipStream_t)stream);
  }
  GemmParams p = base_params();
  p.det = a->deterministic;
  p.M = a->n * a->p * a->q; p.N = a->k; p.K = a->r * a->r * a->c;
  p.a_ptr = a->x; p.a_xf = sanitize(a->x_xf); p.g_nchw = a->x_nchw_f32;
  p.b_ptr = a->wt; p.b_ld = p.K;
  p.gn = a->n; p.gh = a->h; p.gw = a->w; p.gc = a->c; p.gp = a->p; p.gq = a->q;
  p.gr = a->r; p.gs = a->stride; p.gpad = a->pad;
  p.out = a->y; p.out_ld = a->k; p.bias = a->bias; p.sum = a->y_sum; p.sumsq = a->y_sumsq;
  p.sum_reps = a->sum_reps; p.sum_rstride = a->sum_rstride;
  p.residual = a->residual; p.res_xf = sanitize(a->residual_xf);
  if (int rc = check_finalize(a->bn_finalize, a->bn_counter, "conv2d_fwd")) return rc;
  if (a->dtype == VAE_BF16 && cg_ok(p, E_STORE))
    return then_finalize(cg_launch<A_CONV, E_STORE>(p, a->split_k, a->workspace, a->workspace_bytes, (hipStream_t)stream),
                         a->bn_finalize, (hipStream_t)stream);
  return then_finalize(launch<A_CONV, B_NK, E_STORE, false, false, true>(a->dtype, a->x_nchw_f32 != 0, false, p, a->split_k, a->workspace,
                                             a->workspace_bytes, (hipStream_t)stream), a->bn_finalize, (hipStream_t)stream);
}
