// C-ABI entry points of the Linear layers: fc_mu|fc_var fused as one N=2D layer
// (models/vanilla_vae.py:36-37, :89-90) and decoder_input (:43, :101).  One entry point per
// translation unit: each instantiates its own family of generic GEMM kernels, and one file with all
// three was the build's longest compile (~10 min); apart they build in parallel.
#include "vae_launch.hpp"

using namespace vae;

// dW[n][k] += Σ_m dy[m][n] · xf(x)[m][k];  db[n] += Σ_m dy[m][n]  (ones column)
extern "C" int vae_linear_bwd_filter(const vae_linear_args* a, void* stream) {
  if (!a || !a->dy || !a->x || !a->dw || a->m <= 0 || a->n <= 0 || a->k <= 0) return fail(VAE_E_BADARG, "linear_bwd_filter: args");
  if (!xf_ok(a->x_xf, "linear_bwd_filter.x")) return VAE_E_BADARG;
  GemmParams p = base_params();
  p.det = a->deterministic;
  p.M = a->n; p.N = a->k + (a->db ? 1 : 0); p.K = a->m;
  p.ones_col = a->db ? a->k : -1; p.bias_grad = a->db;
  p.a_ptr = a->dy; p.a_ld = a->n;
  p.b_ptr = a->x; p.b_ld = a->k; p.b_xf = sanitize(a->x_xf);
  p.out = a->dw; p.out_ld = a->k;
  return launch<A_KM, B_KN, E_ACC, false, false, true>(a->dtype, a->dy_f32 != 0, false, p, 0, p.det ? a->workspace : nullptr,
                                                          p.det ? a->workspace_bytes : 0, (hipStream_t)stream);
}
