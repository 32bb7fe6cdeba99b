// ELBO of the VAE family on one workgroup (vaehip.h vae_elbo_fwd; vanilla_vae.py:124-146,
// beta_vae.py:129-152, iwae.py:129-160, vq_vae.py:194-211).
#pragma once
#include "vae_common.hpp"

namespace vae {

// The loss of vaehip.h vae_elbo_fwd by one 256-thread workgroup (kld_row: 1024 floats of LDS, red:
// 16) — run by elbo_kernel, and by the head backward's slab-reduction launch when the step fuses it
// (vae_head_args.elbo).
__device__ __forceinline__ void elbo_block(const vae_elbo_args& a, float* kld_row, float (*red)[4]) {
  const int B = a.batch, S = a.samples > 0 ? a.samples : 1, D = a.latent;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // kld_b = -0.5 Σ_d (1 + lv - mu^2 - exp(lv)): 4 threads per row, each a quarter of the latent
  // dims with all its loads in flight at once (64 rows per pass)
  if (a.kind != VAE_LOSS_VQ) {
    const int part = threadIdx.x & 3, per = (D + 3) / 4;
    for (int b0 = 0; b0 < B; b0 += 64) {
      const int b = b0 + (threadIdx.x >> 2);
      float s = 0.f;
      if (b < B) {
        const float* mu = a.mulv + (long)b * 2 * D;
        const float* lv = mu + D;
        const int d0 = part * per, d1 = min(D, d0 + per);
#pragma unroll 32
        for (int d = d0; d < d1; ++d) s += 1.f + lv[d] - mu[d] * mu[d] - expf(lv[d]);
      }
      s += __shfl_xor(s, 1);
      s += __shfl_xor(s, 2);
      if (part == 0 && b < B) kld_row[b] = -0.5f * s;
    }
  }
  __syncthreads();
  const float inv_img = 1.f / (float)a.img_elems;
  // totals: Σ sse, Σ kld_b
  float ts = 0.f, tk = 0.f;
  for (int i = threadIdx.x; i < B * S; i += 256) ts += a.sse[i];
  for (int b = threadIdx.x; b < B && a.kind != VAE_LOSS_VQ; b += 256) tk += kld_row[b];
  for (int off = 32; off > 0; off >>= 1) { ts += __shfl_xor(ts, off); tk += __shfl_xor(tk, off); }
  if (lane == 0) { red[0][wv] = ts; red[1][wv] = tk; }
  __syncthreads();
  const float sse_tot = red[0][0] + red[0][1] + red[0][2] + red[0][3];
  const float kld_mean = (red[1][0] + red[1][1] + red[1][2] + red[1][3]) / (float)B;
  for (int i = threadIdx.x; i < B * S; i += 256) a.per_img[i] = a.sse[i] * inv_img;

  if (a.kind == VAE_LOSS_VQ) {                  // vq_vae.py:203-211
    const float recon = sse_tot / ((float)B * (float)a.img_elems);
    const float vq = (1.f + a.vq_beta) * (*a.vq_sse) / a.vq_elems;
    if (threadIdx.x == 0) { a.out[0] = recon + vq; a.out[1] = recon; a.out[2] = vq; a.out[3] = 0.f; }
    return;
  }
  if (a.kind != VAE_LOSS_IWAE) {
    const float recon = sse_tot / ((float)B * (float)a.img_elems);
    float loss, klc, kld_report;
    if (a.kind == VAE_LOSS_VANILLA) {
      loss = recon + a.kld_weight * kld_mean; klc = a.kld_weight; kld_report = -kld_mean;
    } else if (a.kind == VAE_LOSS_BETA_H) {
      loss = recon + a.beta * a.kld_weight * kld_mean; klc = a.beta * a.kld_weight; kld_report = kld_mean;
    } else {
      const float it = a.iter ? *a.iter : 1.f;
      const float C = fminf(fmaxf(a.c_max / a.c_stop_iter * it, 0.f), a.c_max);
      const float dlt = kld_mean - C;
      loss = recon + a.gamma * a.kld_weight * fabsf(dlt);
      klc = a.gamma * a.kld_weight * (dlt > 0.f ? 1.f : (dlt < 0.f ? -1.f : 0.f));
      kld_report = kld_mean;
    }
    const float hc = 2.f / ((float)B * (float)a.img_elems);
    for (int i = threadIdx.x; i < B; i += 256) { a.head_coef[i] = hc; a.kl_coef[i] = klc / (float)B; }
    if (threadIdx.x == 0) { a.out[0] = loss; a.out[1] = recon; a.out[2] = kld_report; a.out[3] = kld_mean; }
    return;
  }
  // IWAE: lw[b,s] = sse/img + M_N*kld_b ; w = softmax_s(lw) ; loss = mean_b Σ_s w lw
  float lsum = 0.f;
  for (int b = threadIdx.x; b < B; b += 256) {
    float mx = -INFINITY;
    for (int s = 0; s < S; ++s) mx = fmaxf(mx, a.sse[b * S + s] * inv_img + a.kld_weight * kld_row[b]);
    float den = 0.f;
    for (int s = 0; s < S; ++s) den += expf(a.sse[b * S + s] * inv_img + a.kld_weight * kld_row[b] - mx);
    float wl = 0.f;
    for (int s = 0; s < S; ++s) {
      const float lw = a.sse[b * S + s] * inv_img + a.kld_weight * kld_row[b];
      wl += expf(lw - mx) / den * lw;
    }
    for (int s = 0; s < S; ++s) {
      const float lw = a.sse[b * S + s] * inv_img + a.kld_weight * kld_row[b];
      const float w = expf(lw - mx) / den;
      const float g = w * (1.f + lw - wl) / (float)B;          // dL/dlw
      a.head_coef[b * S + s] = g * 2.f * inv_img;
      a.kl_coef[b * S + s] = g * a.kld_weight;
    }
    lsum += wl;
  }
  for (int off = 32; off > 0; off >>= 1) lsum += __shfl_xor(lsum, off);
  __syncthreads();
  if (lane == 0) red[2][wv] = lsum;
  __syncthreads();
  if (threadIdx.x == 0) {
    a.out[0] = (red[2][0] + red[2][1] + red[2][2] + red[2][3]) / (float)B;
    a.out[1] = sse_tot * inv_img / (float)(B * S);
    a.out[2] = -kld_mean;
    a.out[3] = kld_mean;
  }
}

}  // namespace vae
