// C-ABI entry points of the Linear layers: fc_mu|fc_var fused as one N=2D layer
// (models/vanilla_vae.py:36-37, :89-90) and decoder_input (:43, :101).  One entry point per
// translation unit: each instantiates its own family of generic GEMM kernels, and one file with all
// three was the build's longest compile (~10 min); apart they build in parallel.
#include "vae_launch.hpp"

using namespace vae;

// dx[m][k] = Σ_n dy[m][n] · W[n][k];  epilogue: activation backward (dx_epi) or, when
// mulv is set, the reparameterization + KL backward into dmulv
extern "C" int vae_linear_bwd_data(const vae_linear_args* a, void* stream) {
  if (!a || !a->dy || !a->wt || a->m <= 0 || a->n <= 0 || a->k <= 0) return fail(VAE_E_BADARG, "linear_bwd_data: args");
  if (!a->mulv && !epi_ok(a->dx_epi, "linear_bwd_data.epi")) return VAE_E_BADARG;
  GemmParams p = base_params();
  p.det = a->deterministic;
  p.M = a->m; p.N = a->k; p.K = a->n;
  p.a_ptr = a->dy; p.a_ld = a->n;
  p.b_ptr = a->wt; p.b_ld = a->k;
  p.out = a->dx; p.out_ld = a->k;
  if (a->mulv) {
    if (!a->eps || !a->dmulv || a->samples <= 0) return fail(VAE_E_BADARG, "linear_bwd_data: reparam args");
    p.mulv = a->mulv; p.eps = a->eps; p.kl_coef = a->kl_coef; p.dmulv = a->dmulv;
    p.samples = a->samples; p.latent = a->k;
    return launch<A_DENSE, B_KN, E_REPARAM, false, false, true>(a->dtype, a->dy_f32 != 0, false, p, 0, a->workspace,
                                                  a->workspace_bytes, (hipStream_t)stream);
  }
  if (!a->dx) return fail(VAE_E_BADARG, "linear_bwd_data: dx");
  p.epi_xf = sanitize(a->dx_epi); p.dgamma = a->dx_dgamma; p.dbeta = a->dx_dbeta;
  p.sum_reps = a->sum_reps; p.sum_rstride = a->sum_rstride;
  if (p.epi_xf.kind == VAE_X_BN_ACT && (!p.dgamma || !p.dbeta)) return fail(VAE_E_BADARG, "linear_bwd_data: dgamma/dbeta");
  if (int rc = check_finalize(a->bn_finalize, a->bn_counter, "linear_bwd_data")) return rc;
  return then_finalize(launch<A_DENSE, B_KN, E_BNBWD, false, false, true>(a->dtype, a->dy_f32 != 0, false, p, 0, a->workspace, a->workspace_bytes,
                                              (hipStream_t)stream), a->bn_finalize, (hipStream_t)stream);
}
