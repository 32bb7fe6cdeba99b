// C-ABI entry points of the Linear layers: fc_mu|fc_var fused as one N=2D layer
// (models/vanilla_vae.py:36-37, :89-90) and decoder_input (:43, :101).  One entry point per
// translation unit: each instantiates its own family of generic GEMM kernels, and one file with all
// three was the build's longest compile (~10 min); apart they build in parallel.
#include "vae_launch.hpp"

using namespace vae;

extern "C" int vae_linear_fwd(const vae_linear_args* a, void* stream) {
  if (!a || !a->x || !a->wt || !a->y || a->m <= 0 || a->n <= 0 || a->k <= 0) return fail(VAE_E_BADARG, "linear_fwd: args");
  if (!xf_ok(a->x_xf, "linear_fwd.x")) return VAE_E_BADARG;
  GemmParams p = base_params();
  p.det = a->deterministic;
  p.M = a->m; p.N = a->n; p.K = a->k;
  p.a_ptr = a->x; p.a_ld = a->k; p.a_xf = sanitize(a->x_xf);
  p.b_ptr = a->wt; p.b_ld = a->k;
  p.out = a->y; p.out_ld = a->n; p.bias = a->bias; p.out_f32 = a->y_f32;
  return launch<A_DENSE, B_NK, E_STORE, false, false>(a->dtype, false, false, p, 0, a->workspace, a->workspace_bytes,
                                        (hipStream_t)stream);
}
