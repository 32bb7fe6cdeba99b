// C-ABI entry points of ConvTranspose2d (decoder blocks, models/vanilla_vae.py:50-55, :65-70).
#include "vae_launch.hpp"
#include "vae_wgrad.hpp"
#include "vae_wgemm.hpp"

using namespace vae;

// dW[c][r][s][k] += Σ_{n,h,w} xf(x)[n,h,w,c] · dy'[n, h*S-P+r, w*S-P+s, k];  db[k] += Σ dy'
extern "C" int vae_convT2d_bwd_filter(const vae_conv_args* a, void* stream) {
  if (!geom_ok(a, "convT2d_bwd_filter") || !a->dy || !a->x || !a->dw) return fail(VAE_E_BADARG, "convT2d_bwd_filter: null tensor");
  if (!xf_ok(a->dy_xf, "convT2d_bwd_filter.dy") || !xf_ok(a->x_xf, "convT2d_bwd_filter.x")) return VAE_E_BADARG;
  const bool closed = a->db && a->dy_xf.kind == VAE_X_BN_DY;
  {
    // bf16 weight-gradient GEMM (vae_wgemm.hpp)
    WgParams w;
    bool closed_wg;
    if (conv_wg_params(a, true, &w, &closed_wg)) {
      int rc = wg2_launch(w, a->workspace, a->workspace_bytes, (hipStream_t)stream);
      if (rc || !a->db || closed_wg) return rc;
      return column_sum_launch(a->dtype, a->dy, (long)a->n * a->p * a->q, a->k, a->db, (hipStream_t)stream);
    }
  }
  if (a->dw_inner > 0 && a->dw_inner < a->k)
    return fail(VAE_E_UNSUPPORTED, "convT2d_bwd_filter: dw_inner %d < k %d needs the bf16 weight-gradient GEMM path",
                a->dw_inner, a->k);
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
  p.det = a->deterministic;
  const int Nw = a->r * a->r * a->k;
  p.M = a->c; p.N = Nw; p.K = a->n * a->h * a->w;
  p.dbc = closed ? a->db : nullptr; p.dbc_from_b = 1;
  p.a_ptr = a->x; p.a_ld = a->c; p.a_xf = sanitize(a->x_xf);
  p.b_ptr = a->dy; p.b_xf = sanitize(a->dy_xf);
  p.gn = a->n; p.gh = a->p; p.gw = a->q; p.gc = a->k; p.gp = a->h; p.gq = a->w;
  p.gr = a->r; p.gs = a->stride; p.gpad = a->pad;
  p.out = a->dw; p.out_ld = Nw;
  int rc = launch<A_KM, B_GATHER, E_ACC, false, true>(a->dtype, false, false, p, a->split_k, p.det ? a->workspace : nullptr, p.det ? a->workspace_bytes : 0, (hipStream_t)stream);
  if (rc) return rc;
  if (a->db && !closed) return column_sum_launch(a->dtype, a->dy, (long)a->n * a->p * a->q, a->k, a->db, (hipStream_t)stream);
  return VAE_OK;
}
