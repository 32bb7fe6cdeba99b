// C-ABI entry points of ConvTranspose2d (decoder blocks, models/vanilla_vae.py:50-55, :65-70).
#include "vae_launch.hpp"
#include "vae_wgrad.hpp"

using namespace vae;

namespace vae {
int hires_convT_fwd_launch(const vae_conv_args* a, hipStream_t st);   // vae_hires.hip
}

// y[n,ho,wo,k] = Σ_{r,s,c: ho = h*S-P+r} xf(x)[n,h,w,c] · W[c][r][s][k] + b[k]   (phase GEMMs)
extern "C" int vae_convT2d_fwd(const vae_conv_args* a, void* stream) {
  if (!geom_ok(a, "convT2d_fwd") || !a->x || !a->wt || !a->y) return fail(VAE_E_BADARG, "convT2d_fwd: null tensor");
  if (!xf_ok(a->x_xf, "convT2d_fwd.x")) return VAE_E_BADARG;
  const int S = a->stride;
  if (a->p % S || a->q % S) return fail(VAE_E_BADSHAPE, "convT2d_fwd: output not a multiple of stride");
  GemmParams p = base_params();
  p.det = a->deterministic;
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
  if (a->dtype == VAE_BF16) {
    // the decoder's full-resolution last ConvTranspose2d (32 -> 32, 32x32 -> 64x64)
    const int rc = hires_convT_fwd_launch(a, (hipStream_t)stream);
    if (rc != kHeadFallback) return rc;
  }
  if (a->dtype == VAE_BF16) {
    // bf16 conv-GEMM: B = the swapped-axes weight copy WT[k][r][s][c] (k-contiguous rows), taken
    // from the caller (wt_t, refreshed with the weights) or built at the end of the workspace
    GemmParams q = p;
    q.b_taps = 0; q.b_ld = a->r * a->r * a->c;
    const long wbytes = (long)a->k * a->r * a->r * a->c * 2;
    long ws_slab = a->workspace_bytes;
    q.b_ptr = a->wt_t;
    const bool tail = !q.b_ptr && a->workspace;
    if (tail) {
      ws_slab = ((a->workspace_bytes - wbytes) / 256) * 256;
      q.b_ptr = static_cast<char*>(a->workspace) + (ws_slab > 0 ? ws_slab : 0);
    }
    if (q.b_ptr && cg_ok(q, E_STORE)) {
      return with_ws_tail(tail ? wbytes : 0, [&]() -> int {
        if (tail && !ws_fits(wbytes, a->workspace_bytes, "convT2d_fwd weight copy")) return VAE_E_BADARG;
        if (!a->wt_t) {
          if (int rc = flip_weights_launch(static_cast<const __bf16*>(a->wt), static_cast<__bf16*>(const_cast<void*>(q.b_ptr)),
                                           a->c, a->r, a->k, (hipStream_t)stream, 0)) return rc;
        }
        return then_finalize(cg_launch<A_CONVT, E_STORE>(q, a->split_k, a->workspace, ws_slab, (hipStream_t)stream),
                             a->bn_finalize, (hipStream_t)stream);
      });
    }
  }
  return then_finalize(launch<A_CONVT, B_KN, E_STORE, false, false>(a->dtype, false, false, p, a->split_k, a->workspace, a->workspace_bytes,
                                        (hipStream_t)stream), a->bn_finalize, (hipStream_t)stream);
}
