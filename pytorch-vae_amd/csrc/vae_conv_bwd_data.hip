// C-ABI entry points of Conv2d (encoder blocks, models/vanilla_vae.py:28-29 run at :84).
#include "vae_launch.hpp"
#include "vae_wgrad.hpp"
#include "vae_c3.hpp"

using namespace vae;

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
  // 1x1 stride 1 (the VQ-VAE ResidualLayer's Conv1x1): pixel-tile GEMM over WT[c][k]
  if (a->dtype == VAE_BF16 && a->wt_t && c3_enabled() && a->r == 1 && a->stride == 1 && a->pad == 0 &&
      a->h == a->p && a->w == a->q && p1_shape_ok((long)a->n * a->h * a->w, a->k, a->c) &&
      a->dy_xf.kind == VAE_X_NONE && (a->dx_epi.kind == VAE_X_NONE || a->dx_epi.kind == VAE_X_ACT) &&
      !a->dx_dgamma && !a->bn_finalize && a->split_k <= 0) {
    P1Args c;
    memset(&c, 0, sizeof(c));
    c.a = a->dy; c.b = a->wt_t; c.out = a->dx; c.residual = a->residual;
    if (a->dx_epi.kind == VAE_X_ACT) { c.aux = a->dx_epi.aux; c.aux_slope = a->dx_epi.slope; }
    c.M = (long)a->n * a->h * a->w; c.C = a->k; c.N = a->c;
    return p1_launch(c, (hipStream_t)stream);
  }
  // 3x3 stride-1 on a 16 x 16 grid (the VQ-VAE's residual stacks): the image-tile kernel, taps
  // flipped, over the caller's swapped-axes weights WT[c][r][s][k]
  if (a->dtype == VAE_BF16 && a->wt_t && c3_enabled() &&
      c3_shape_ok(a->n, a->p, a->q, a->h, a->w, a->r, a->stride, a->pad, a->k, a->c) &&
      a->dy_xf.kind == VAE_X_NONE && (a->dx_epi.kind == VAE_X_NONE || a->dx_epi.kind == VAE_X_ACT) &&
      !a->dx_dgamma && !a->bn_finalize && a->split_k <= 0) {
    C3Args c;
    memset(&c, 0, sizeof(c));
    c.a = a->dy; c.b = a->wt_t; c.flip = 1; c.out = a->dx; c.residual = a->residual;
    if (a->dx_epi.kind == VAE_X_ACT) { c.aux = a->dx_epi.aux; c.aux_slope = a->dx_epi.slope; }
    c.n = a->n; c.C = a->k; c.N = a->c;
    return c3_launch(c, (hipStream_t)stream);
  }
  if (a->dtype == VAE_BF16) {
    // bf16 conv-GEMM: phase gather of dy (any stride; stride 1 is one phase of R*R taps) against
    // the swapped-axes weights WT[c][r][s][k] (caller's wt_t, or built at the workspace's end)
    GemmParams q = base_params();
    q.det = a->deterministic;
    if (make_taps(q, S, a->r, a->pad)) {
      q.nphase = S * S;
      q.M = a->n * (a->h / S) * (a->w / S); q.N = a->c; q.K = 0;
      q.a_ptr = a->dy; q.a_xf = sanitize(a->dy_xf);
      q.b_ld = a->r * a->r * a->k;
      q.gn = a->n; q.gh = a->p; q.gw = a->q; q.gc = a->k;
      q.gp = a->h / S; q.gq = a->w / S; q.gr = a->r; q.gs = S; q.gpad = a->pad; q.gho = a->h; q.gwo = a->w;
      q.out = a->dx; q.out_ld = a->c; q.out_phase = 1;
      q.epi_xf = sanitize(a->dx_epi); q.dgamma = a->dx_dgamma; q.dbeta = a->dx_dbeta;
      q.sum_reps = a->sum_reps; q.sum_rstride = a->sum_rstride;
      q.residual = a->residual;
      long ws_slab = a->workspace_bytes;
      q.b_ptr = a->wt_t;
      const bool tail = !q.b_ptr && a->workspace;
      if (tail) {
        ws_slab = ((a->workspace_bytes - wbytes) / 256) * 256;
        q.b_ptr = static_cast<char*>(a->workspace) + (ws_slab > 0 ? ws_slab : 0);
      }
      if (q.epi_xf.kind == VAE_X_BN_ACT && (!q.dgamma || !q.dbeta)) return fail(VAE_E_BADARG, "conv2d_bwd_data: dgamma/dbeta");
      if (q.b_ptr && cg_ok(q, E_BNBWD)) {
        if (int rc = check_finalize(a->bn_finalize, a->bn_counter, "conv2d_bwd_data")) return rc;
        return with_ws_tail(tail ? wbytes : 0, [&]() -> int {
          if (tail && !ws_fits(wbytes, a->workspace_bytes, "conv2d_bwd_data weight copy")) return VAE_E_BADARG;
          if (!a->wt_t) {
            if (int rc = flip_weights_launch(static_cast<const __bf16*>(a->wt), static_cast<__bf16*>(const_cast<void*>(q.b_ptr)),
                                             a->k, a->r, a->c, (hipStream_t)stream, 0)) return rc;
          }
          return then_finalize(cg_launch<A_CONVT, E_BNBWD>(q, a->split_k, a->workspace, ws_slab, (hipStream_t)stream),
                               a->bn_finalize, (hipStream_t)stream);
        });
      }
    }
  }
  if (S == 1 && a->dtype == VAE_BF16 && a->c % 8 == 0 && a->k % 8 == 0 && a->workspace) {
    // stride 1: dx = conv(dy, W') with W'[c][r][s][k] = W[k][R-1-r][R-1-s][c] and pad R-1-P — the
    // forward conv path (k-contiguous weight rows, packed im2col gather of dy) instead of the
    // phase-gather with k-strided weights.  W' lives at the end of the workspace.
    return with_ws_tail(wbytes, [&]() -> int {
    if (!ws_fits(wbytes, a->workspace_bytes, "conv2d_bwd_data weight copy")) return VAE_E_BADARG;
    char* ws = static_cast<char*>(a->workspace);
    long wsoff = ((a->workspace_bytes - wbytes) / 256) * 256;
    if (wsoff < 0) wsoff = 0;
    __bf16* wf = reinterpret_cast<__bf16*>(ws + wsoff);
    int rc = flip_weights_launch(static_cast<const __bf16*>(a->wt), wf, a->k, a->r, a->c, (hipStream_t)stream);
    if (rc) return rc;
    GemmParams p = base_params();
    p.det = a->deterministic;
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
    });
  }
  GemmParams p = base_params();
  p.det = a->deterministic;
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
