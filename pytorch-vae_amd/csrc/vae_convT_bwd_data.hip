// C-ABI entry points of ConvTranspose2d (decoder blocks, models/vanilla_vae.py:50-55, :65-70).
#include "vae_launch.hpp"
#include "vae_wgrad.hpp"

using namespace vae;

// dx[n,h,w,c] = Σ_{r,s,k} dy'[n, h*S-P+r, w*S-P+s, k] · W[c][r][s][k]   (strided conv of dy)
extern "C" int vae_convT2d_bwd_data(const vae_conv_args* a, void* stream) {
  if (!geom_ok(a, "convT2d_bwd_data") || !a->dy || !a->wt || !a->dx) return fail(VAE_E_BADARG, "convT2d_bwd_data: null tensor");
  if (!xf_ok(a->dy_xf, "convT2d_bwd_data.dy") || !epi_ok(a->dx_epi, "convT2d_bwd_data.epi")) return VAE_E_BADARG;
  GemmParams p = base_params();
  p.det = a->deterministic;
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
  if (a->dtype == VAE_BF16 && cg_ok(p, E_BNBWD))
    return then_finalize(cg_launch<A_CONV, E_BNBWD>(p, a->split_k, a->workspace, a->workspace_bytes, (hipStream_t)stream),
                         a->bn_finalize, (hipStream_t)stream);
  return then_finalize(launch<A_CONV, B_NK, E_BNBWD, true, false>(a->dtype, false, false, p, a->split_k, a->workspace, a->workspace_bytes,
                                       (hipStream_t)stream), a->bn_finalize, (hipStream_t)stream);
}
