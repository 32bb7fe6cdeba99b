// C-ABI entry points of ConvTranspose2d (decoder blocks, models/vanilla_vae.py:50-55, :65-70).
#include "vae_launch.hpp"
#include "vae_wgrad.hpp"

using namespace vae;

// y[n,ho,wo,k] = Σ_{r,s,c: ho = h*S-P+r} xf(x)[n,h,w,c] · W[c][r][s][k] + b[k]   (phase GEMMs)
extern "C" int vae_convT2d_fwd(const vae_conv_args* a, void* stream) {
  if (!geom_ok(a, "convT2d_fwd") || !a->x || !a->wt || !a->y) return fail(VAE_E_BADARG, "convT2d_fwd: null tensor");
  if (!xf_ok(a->x_xf, "convT2d_fwd.x")) return VAE_E_BADARG;
  const int S = a->stride;
  if (a->p % S || a->q % S) return fail(VAE_E_BADSHAPE, "convT2d_fwd: output not a multiple of stride");
  GemmParams p = base_params();
  if (!make_taps(p, S, a->r, a->pad)) return fail(VAE_E_UNSUPPORTED, "convT2d_fwd: stride/kernel");
  p.nphase = S * S;
  p.M = a->n * (a->p / S) * (a->q / S); p.N = a->k; p.K = 0;
  p.a_ptr = a->x; p.a_xf = sanitize(a->x_xf);
  p.b_ptr = a->wt; p.b_ld = a->k; p.b_taps = 1;
  p.gn = a->n; p.gh = a->h; p.gw = a->w; p.gc = a->c;
  p.gp = a->p / S; p.gq = a->q / S; p.gr = a->r; p.gs = S; p.gpad = a->pad; p.gho = a->p; p.gwo = a->q;
  p.out = a->y; p.out_ld = a->k; p.out_phase = 1; p.bias = a->bias; p.sum = a->y_sum; p.sumsq = a->y_sumsq;
  p.sum_reps = a->sum_reps; p.sum_rstride = a->sum_rstride;
  p.residual = a->residual; p.res_xf = sanitize(a->residual_xf);
  if (int rc = check_finalize(a->bn_finalize, a->bn_counter, "convT2d_fwd")) return rc;
  return then_finalize(launch<A_CONVT, B_KN, E_STORE, false, false>(a->dtype, false, false, p, a->split_k, a->workspace, a->workspace_bytes,
                                        (hipStream_t)stream), a->bn_finalize, (hipStream_t)stream);
}

// dx[n,h,w,c] = Σ_{r,s,k} dy'[n, h*S-P+r, w*S-P+s, k] · W[c][r][s][k]   (strided conv of dy)
extern "C" int vae_convT2d_bwd_data(const vae_conv_args* a, void* stream) {
  if (!geom_ok(a, "convT2d_bwd_data") || !a->dy || !a->wt || !a->dx) return fail(VAE_E_BADARG, "convT2d_bwd_data: null tensor");
  if (!xf_ok(a->dy_xf, "convT2d_bwd_data.dy") || !epi_ok(a->dx_epi, "convT2d_bwd_data.epi")) return VAE_E_BADARG;
  GemmParams p = base_params();
  p.M = a->n * a->h * a->w; p.N = a->c; p.K = a->r * a->r * a->k;
  p.a_ptr = a->dy; p.a_xf = sanitize(a->dy_xf);
  p.b_ptr = a->wt; p.b_ld = p.K;
  p.gn = a->n; p.gh = a->p; p.gw = a->q; p.gc = a->k; p.gp = a->h; p.gq = a->w;
  p.gr = a->r; p.gs = a->stride; p.gpad = a->pad;
  p.out = a->dx; p.out_ld = a->c;
  p.epi_xf = sanitize(a->dx_epi); p.dgamma = a->dx_dgamma; p.dbeta = a->dx_dbeta;
  p.sum_reps = a->sum_reps; p.sum_rstride = a->sum_rstride;
  if (p.epi_xf.kind == VAE_X_BN_ACT && (!p.dgamma || !p.dbeta)) return fail(VAE_E_BADARG, "convT2d_bwd_data: dgamma/dbeta");
  if (int rc = check_finalize(a->bn_finalize, a->bn_counter, "convT2d_bwd_data")) return rc;
  return then_finalize(launch<A_CONV, B_NK, E_BNBWD, true, false>(a->dtype, false, false, p, a->split_k, a->workspace, a->workspace_bytes,
                                       (hipStream_t)stream), a->bn_finalize, (hipStream_t)stream);
}

// dW[c][r][s][k] += Σ_{n,h,w} xf(x)[n,h,w,c] · dy'[n, h*S-P+r, w*S-P+s, k];  db[k] += Σ dy'
extern "C" int vae_convT2d_bwd_filter(const vae_conv_args* a, void* stream) {
  if (!geom_ok(a, "convT2d_bwd_filter") || !a->dy || !a->x || !a->dw) return fail(VAE_E_BADARG, "convT2d_bwd_filter: null tensor");
  if (!xf_ok(a->dy_xf, "convT2d_bwd_filter.dy") || !xf_ok(a->x_xf, "convT2d_bwd_filter.x")) return VAE_E_BADARG;
  const bool closed = a->db && a->dy_xf.kind == VAE_X_BN_DY;
  if (!closed &&
      wgrad_ok(a->dtype, a->x_xf, a->dy_xf, (long)a->n * a->h * a->w * a->c, (long)a->n * a->p * a->q * a->k, a->c, a->k)) {
    // bf16 fast path: U = x (input grid, m = c), V = dy (output grid, j = k)
    WgradParams w;
    memset(&w, 0, sizeof(w));
    w.u = a->x; w.u_xf = sanitize(a->x_xf); w.v = a->dy; w.v_xf = sanitize(a->dy_xf);
    w.n = a->n; w.hu = a->h; w.wu = a->w; w.M = a->c; w.hv = a->p; w.wv = a->q; w.J = a->k;
    w.R = a->r; w.S = a->stride; w.P = a->pad; w.dw = a->dw;
    int rc = wgrad_launch(w, (hipStream_t)stream);
    if (rc || !a->db) return rc;
    return column_sum_launch(a->dtype, a->dy, (long)a->n * a->p * a->q, a->k, a->db, (hipStream_t)stream);
  }
  GemmParams p = base_params();
  const int Nw = a->r * a->r * a->k;
  p.M = a->c; p.N = Nw; p.K = a->n * a->h * a->w;
  p.dbc = closed ? a->db : nullptr; p.dbc_from_b = 1;
  p.a_ptr = a->x; p.a_ld = a->c; p.a_xf = sanitize(a->x_xf);
  p.b_ptr = a->dy; p.b_xf = sanitize(a->dy_xf);
  p.gn = a->n; p.gh = a->p; p.gw = a->q; p.gc = a->k; p.gp = a->h; p.gq = a->w;
  p.gr = a->r; p.gs = a->stride; p.gpad = a->pad;
  p.out = a->dw; p.out_ld = Nw;
  int rc = launch<A_KM, B_GATHER, E_ACC, false, true>(a->dtype, false, false, p, a->split_k, nullptr, 0, (hipStream_t)stream);
  if (rc) return rc;
  if (a->db && !closed) return column_sum_launch(a->dtype, a->dy, (long)a->n * a->p * a->q, a->k, a->db, (hipStream_t)stream);
  return VAE_OK;
}
