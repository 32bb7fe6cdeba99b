// The Autoencoder's reconstruction losses other than the plain MSE, forward and backward seed on
// the GPU (vaehip.h vae_recon_loss):
//   * centre-weighted MSE   mean(mask * (recon - x)^2)        models/autoencoder.py:95-146, :259-265
//   * MS-SSIM               1 - prod_l cs_l^w_l * ssim_L^w_L   models/mssim_vae.py:182-282, autoencoder.py:266-267
// Both write dL/drecon (NCHW fp32) for the fused backward (the head kernels' grad_recon seed) and the
// loss terms into the step's `out`, so the Autoencoder configs with these losses run inside the
// graph-replayed training step instead of as torch ops between a HIP forward and a HIP backward.
//
// Layout: one workgroup per image plane (n, c) — the whole five-level pyramid of a 64x64 plane and
// the per-level Gaussian-moment maps live in LDS (<= 145 KB), so each level's 11x11 windows
// (separable: a row pass and a column pass, zero padding 5 as F.conv2d(padding=5)) are LDS reads.
// MS-SSIM couples the levels through global means, so it runs as three launches:
//   1. per plane: sum of ssim_map and of cs_map (v1/v2) at every level -> workspace partials;
//   2. one workgroup: the means in fixed plane order, the loss, and dloss/d(mean) per level;
//   3. per plane: the moment maps again, their pointwise backward, the transposed window pass (the
//      window is symmetric: G^T = G), and avg_pool2d's backward from the coarsest level up.
// The centre-weighted MSE is linear in its seed: launch 1 writes dL/drecon and per-plane sums,
// launch 2 the loss.  Partials are reduced in a fixed order (deterministic).
#include "vae_common.hpp"

namespace vae {
namespace {

constexpr int RL_T = 256;            // threads per workgroup
constexpr int RL_MAXHW = 4096;       // plane of up to 64 x 64 at level 0
constexpr int RL_MAXLV = 8;
constexpr int RL_MAXWIN = 15;

struct RlGeom {
  int H[RL_MAXLV], W[RL_MAXLV], off[RL_MAXLV + 1];   // level sizes, pyramid offsets
};

__device__ __forceinline__ void rl_geom(int h, int w, int levels, RlGeom& g) {
  g.off[0] = 0;
  for (int l = 0; l < levels; ++l) {
    g.H[l] = h >> l;
    g.W[l] = w >> l;
    g.off[l + 1] = g.off[l] + g.H[l] * g.W[l];
  }
}

// F.avg_pool2d((2, 2)) on the CPU: ((x00 + x01) + x10) + x11, then / 4
__device__ void rl_pyramid(float* p, const RlGeom& g, int levels) {
  for (int l = 1; l < levels; ++l) {
    const float* s = p + g.off[l - 1];
    float* d = p + g.off[l];
    const int W = g.W[l], Ws = g.W[l - 1], n = g.H[l] * W;
    for (int i = threadIdx.x; i < n; i += RL_T) {
      const int y = i / W, x = i - y * W;
      const float* q = s + (2 * y) * Ws + 2 * x;
      float t = q[0];
      t += q[1];
      t += q[Ws];
      t += q[Ws + 1];
      d[i] = t / 4.f;
    }
    __syncthreads();
  }
}

// dst = G(src) at one level: row pass into tmp, column pass into dst (zero padding R/2).
// src(i) is a functor of the flat pixel index (a product of pyramid planes), evaluated per tap.
template <class F>
__device__ void rl_window(F src, float* tmp, float* dst, const float* win, int R, int H, int W) {
  const int P = R / 2, n = H * W;
  for (int i = threadIdx.x; i < n; i += RL_T) {
    const int y = i / W, x = i - y * W;
    float a = 0.f;
    for (int t = 0; t < R; ++t) {
      const int xx = x + t - P;
      if ((unsigned)xx < (unsigned)W) a = fmaf(win[t], src(y * W + xx), a);
    }
    tmp[i] = a;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += RL_T) {
    const int y = i / W, x = i - y * W;
    float a = 0.f;
    for (int t = 0; t < R; ++t) {
      const int yy = y + t - P;
      if ((unsigned)yy < (unsigned)H) a = fmaf(win[t], tmp[yy * W + x], a);
    }
    dst[i] = a;
  }
  __syncthreads();
}

__device__ float rl_block_sum(float v, float* red) {
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  const int wave = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[wave] = v;
  __syncthreads();
  float s = 0.f;
  for (int k = 0; k < RL_T / 64; ++k) s += red[k];
  return s;
}

constexpr float kC1 = 0.01f * 0.01f, kC2 = 0.03f * 0.03f;   // (0.01 * range)^2, (0.03 * range)^2, range 1

// LDS of the MS-SSIM plane kernels (static, sized for a 64 x 64 plane): x, y pyramids (<= 4/3 of
// the plane each), the dx pyramid of levels >= 1, 5 moment maps and the row-pass scratch = 144 KB
constexpr int RL_PYR = RL_MAXHW + RL_MAXHW / 3 + 8;
constexpr int RL_LDS = 2 * RL_PYR + (RL_PYR - RL_MAXHW) + 6 * RL_MAXHW;

template <bool BWD>
__global__ void __launch_bounds__(RL_T) mssim_plane_kernel(const vae_recon_loss_args a) {
  kernarg_prefetch<(sizeof(vae_recon_loss_args) < 1024 ? sizeof(vae_recon_loss_args) : 1024)>();
  __shared__ float sm[RL_LDS];
  const vae_recon_loss_args& r = a;
  const int plane = blockIdx.x, HW = a.h * a.w, L = a.levels, R = a.window_size;
  RlGeom g;
  rl_geom(a.h, a.w, L, g);
  const int NP = g.off[L];
  float* xp = sm;                      // [NP]
  float* yp = xp + NP;                 // [NP]
  float* dxp = yp + NP;                // [NP - HW]: levels >= 1 (level 0 goes to global)
  float* m = dxp + (NP - HW);          // [5][HW]
  float* tmp = m + 5 * HW;             // [HW]
  __shared__ float red[RL_T / 64];
  const float* x0 = a.recon + (long)plane * HW;
  const float* y0 = a.target + (long)plane * HW;
  for (int i = threadIdx.x; i < HW; i += RL_T) { xp[i] = x0[i]; yp[i] = y0[i]; }
  __syncthreads();
  rl_pyramid(xp, g, L);
  rl_pyramid(yp, g, L);
  const float* coef = a.workspace + (long)gridDim.x * 2 * L;   // BWD: [L][2] = dloss/dS_l, dloss/dcs_l
  for (int li = 0; li < L; ++li) {
    const int l = BWD ? L - 1 - li : li;                      // backward: coarsest level first
    const int H = g.H[l], W = g.W[l], n = H * W;
    const float* x = xp + g.off[l];
    const float* y = yp + g.off[l];
    float dS = 0.f, dcs = 0.f;
    if (BWD) {
      dS = coef[2 * l];
      dcs = coef[2 * l + 1];
    }
    float* dX = (l == 0) ? nullptr : dxp + (g.off[l] - HW);
    if (BWD && dS == 0.f && dcs == 0.f) {
      // no direct term at this level: only the coarser levels' gradient, unpooled below
      for (int i = threadIdx.x; i < n; i += RL_T) {
        float v = 0.f;
        if (l + 1 < L) {
          const int yy = i / W, xx = i - yy * W;
          v = dxp[(g.off[l + 1] - HW) + (yy >> 1) * g.W[l + 1] + (xx >> 1)] / 4.f;
        }
        if (l == 0) a.grad[(long)plane * HW + i] = v * a.grad_scale;
        else dX[i] = v;
      }
      __syncthreads();
      continue;
    }
    rl_window([&](int i) { return x[i]; }, tmp, m + 0 * HW, r.window, R, H, W);
    rl_window([&](int i) { return y[i]; }, tmp, m + 1 * HW, r.window, R, H, W);
    rl_window([&](int i) { return x[i] * x[i]; }, tmp, m + 2 * HW, r.window, R, H, W);
    rl_window([&](int i) { return y[i] * y[i]; }, tmp, m + 3 * HW, r.window, R, H, W);
    rl_window([&](int i) { return x[i] * y[i]; }, tmp, m + 4 * HW, r.window, R, H, W);
    const float Nl = (float)a.n * (float)a.c * (float)n;
    float s_ssim = 0.f, s_cs = 0.f;
    for (int i = threadIdx.x; i < n; i += RL_T) {
      const float mu1 = m[i], mu2 = m[HW + i];
      const float mu1_sq = mu1 * mu1, mu2_sq = mu2 * mu2, mu12 = mu1 * mu2;
      const float s11 = m[2 * HW + i] - mu1_sq, s22 = m[3 * HW + i] - mu2_sq, s12 = m[4 * HW + i] - mu12;
      const float v1 = 2.0f * s12 + kC2, v2 = s11 + s22 + kC2;
      const float A = 2.f * mu12 + kC1, Bm = mu1_sq + mu2_sq + kC1;
      if (!BWD) {
        s_cs += v1 / v2;
        s_ssim += (A * v1) / (Bm * v2);
      } else {
        const float inv = 1.f / (Nl * v2);
        const float dv1 = dcs * inv + dS * A / (Bm * v2 * Nl);
        const float dv2 = -dcs * v1 * inv / v2 - dS * A * v1 / (Bm * v2 * v2 * Nl);
        const float dA = dS * v1 / (Bm * v2 * Nl);
        const float dB = -dS * A * v1 / (Bm * Bm * v2 * Nl);
        // P = dL/dmu1, Q = dL/dG(x^2), R = dL/dG(xy)   (mu2 terms belong to the target: no gradient)
        m[2 * HW + i] = 2.f * mu2 * dA + 2.f * mu1 * dB - 2.f * mu2 * dv1 - 2.f * mu1 * dv2;
        m[3 * HW + i] = dv2;
        m[4 * HW + i] = 2.f * dv1;
      }
    }
    if (!BWD) {
      const float t1 = rl_block_sum(s_ssim, red);
      const float t2 = rl_block_sum(s_cs, red);
      if (threadIdx.x == 0) {
        a.workspace[((long)plane * L + l) * 2 + 0] = t1;
        a.workspace[((long)plane * L + l) * 2 + 1] = t2;
      }
      __syncthreads();
      continue;
    }
    __syncthreads();
    // dx_l = G(P) + 2 x G(Q) + y G(R)  (+ the unpooled gradient of level l + 1)
    rl_window([&](int i) { return m[2 * HW + i]; }, tmp, m + 0 * HW, r.window, R, H, W);
    rl_window([&](int i) { return m[3 * HW + i]; }, tmp, m + 1 * HW, r.window, R, H, W);
    rl_window([&](int i) { return m[4 * HW + i]; }, tmp, m + 2 * HW, r.window, R, H, W);
    for (int i = threadIdx.x; i < n; i += RL_T) {
      float v = m[i] + 2.f * x[i] * m[HW + i] + y[i] * m[2 * HW + i];
      if (l + 1 < L) {
        const int yy = i / W, xx = i - yy * W;
        v += dxp[(g.off[l + 1] - HW) + (yy >> 1) * g.W[l + 1] + (xx >> 1)] / 4.f;
      }
      if (l == 0) a.grad[(long)plane * HW + i] = v * a.grad_scale;
      else dX[i] = v;
    }
    __syncthreads();
  }
}

// one workgroup: plane partials -> means (fixed order) -> loss and the per-level seeds
__global__ void __launch_bounds__(RL_T) mssim_finalize_kernel(const vae_recon_loss_args a, int planes) {
  const int L = a.levels;
  __shared__ float red[RL_T / 64];
  __shared__ float S[RL_MAXLV], CS[RL_MAXLV];
  for (int l = 0; l < L; ++l) {
    for (int q = 0; q < 2; ++q) {
      float s = 0.f;
      for (int p = threadIdx.x; p < planes; p += RL_T) s += a.workspace[((long)p * L + l) * 2 + q];
      s = rl_block_sum(s, red);
      if (threadIdx.x == 0) {
        const float N = (float)a.n * (float)a.c * (float)((a.h >> l) * (a.w >> l));
        (q == 0 ? S : CS)[l] = s / N;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float ms[RL_MAXLV], mcs[RL_MAXLV];
    for (int l = 0; l < L; ++l) {
      ms[l] = a.normalize ? (S[l] + 1.f) / 2.f : S[l];
      mcs[l] = a.normalize ? (CS[l] + 1.f) / 2.f : CS[l];
    }
    // output = prod_{l < L-1} mcs_l^w_l * ms_{L-1}^w_{L-1}   (mssim_vae.py:277-280)
    const float p2 = powf(ms[L - 1], a.level_weights[L - 1]);
    float out = 1.f;
    for (int l = 0; l + 1 < L; ++l) out *= powf(mcs[l], a.level_weights[l]) * p2;
    const float loss = 1.f - out;
    a.out[0] = loss;
    a.out[1] = loss;
    a.out[2] = 0.f;
    float* coef = a.workspace + (long)planes * 2 * L;
    const float nf = a.normalize ? 0.5f : 1.f;
    for (int l = 0; l < L; ++l) {
      coef[2 * l] = 0.f;
      coef[2 * l + 1] = (l + 1 < L) ? -out * a.level_weights[l] / mcs[l] * nf : 0.f;
    }
    coef[2 * (L - 1)] = -out * (float)(L - 1) * a.level_weights[L - 1] / ms[L - 1] * nf;
  }
  if (a.sse && a.per_img) {
    const float inv = 1.f / ((float)a.c * a.h * a.w);
    for (int i = threadIdx.x; i < a.n; i += RL_T) a.per_img[i] = a.sse[i] * inv;
  }
}

// centre-weighted MSE: per plane sum of mask * d^2 and the seed 2 * mask * d / N
__global__ void __launch_bounds__(RL_T) center_plane_kernel(const vae_recon_loss_args a) {
  kernarg_prefetch<(sizeof(vae_recon_loss_args) < 1024 ? sizeof(vae_recon_loss_args) : 1024)>();
  __shared__ float red[RL_T / 64];
  const int plane = blockIdx.x, HW = a.h * a.w;
  const float* x = a.recon + (long)plane * HW;
  const float* y = a.target + (long)plane * HW;
  const float g = 2.f * a.grad_scale / ((float)a.n * a.c * HW);
  float s = 0.f;
  for (int i = threadIdx.x; i < HW; i += RL_T) {
    const float d = x[i] - y[i], mk = a.mask[i];
    s = fmaf(d * d, mk, s);
    if (a.grad) a.grad[(long)plane * HW + i] = g * mk * d;
  }
  s = rl_block_sum(s, red);
  if (threadIdx.x == 0) a.workspace[plane] = s;
}

__global__ void __launch_bounds__(RL_T) center_finalize_kernel(const vae_recon_loss_args a, int planes) {
  __shared__ float red[RL_T / 64];
  float s = 0.f;
  for (int p = threadIdx.x; p < planes; p += RL_T) s += a.workspace[p];
  s = rl_block_sum(s, red);
  if (threadIdx.x == 0) {
    const float loss = s / ((float)a.n * a.c * a.h * a.w);
    a.out[0] = loss;
    a.out[1] = loss;
    a.out[2] = 0.f;
  }
  if (a.sse && a.per_img) {
    const float inv = 1.f / ((float)a.c * a.h * a.w);
    for (int i = threadIdx.x; i < a.n; i += RL_T) a.per_img[i] = a.sse[i] * inv;
  }
}

long rl_workspace_floats(const vae_recon_loss_args* a) {
  const long planes = (long)a->n * a->c;
  return a->kind == VAE_RLOSS_MSSIM ? planes * 2 * a->levels + 2 * a->levels : planes;
}

int rl_check(const vae_recon_loss_args* a, bool tensors = true) {
  if (!a) return fail(VAE_E_BADARG, "recon_loss: null args");
  if (a->n <= 0 || a->c <= 0 || a->h <= 0 || a->w <= 0) return fail(VAE_E_BADSHAPE, "recon_loss: bad shape");
  if (a->kind != VAE_RLOSS_CENTER && a->kind != VAE_RLOSS_MSSIM) return fail(VAE_E_BADARG, "recon_loss: kind %d", a->kind);
  if (a->kind == VAE_RLOSS_MSSIM) {
    if (a->levels < 1 || a->levels > RL_MAXLV) return fail(VAE_E_BADARG, "recon_loss: %d levels", a->levels);
    if ((a->h % (1 << (a->levels - 1))) || (a->w % (1 << (a->levels - 1))))
      return fail(VAE_E_BADSHAPE, "recon_loss: %dx%d not divisible by 2^%d", a->h, a->w, a->levels - 1);
    if (a->window_size < 1 || a->window_size > RL_MAXWIN || !(a->window_size & 1))
      return fail(VAE_E_BADARG, "recon_loss: window %d (odd, <= %d)", a->window_size, RL_MAXWIN);
    if (!a->size_average) return fail(VAE_E_UNSUPPORTED, "recon_loss: size_average=False (the reference's MS-SSIM "
                                                        "combines per-level scalars)");
  } else if (tensors && !a->mask) {
    return fail(VAE_E_BADARG, "recon_loss: centre-weighted MSE needs the mask");
  }
  if ((long)a->h * a->w > RL_MAXHW) return fail(VAE_E_UNSUPPORTED, "recon_loss: plane %dx%d > 64x64", a->h, a->w);
  if (tensors && (!a->recon || !a->target || !a->out)) return fail(VAE_E_BADARG, "recon_loss: recon / target / out");
  return VAE_OK;
}

}  // namespace
}  // namespace vae

using namespace vae;

extern "C" int vae_recon_loss_workspace_size(const vae_recon_loss_args* a, size_t* bytes) {
  if (int rc = rl_check(a, false)) return rc;              // (sizes only: tensors may be unset)
  if (!bytes) return fail(VAE_E_BADARG, "recon_loss_workspace_size: bytes");
  *bytes = (size_t)rl_workspace_floats(a) * 4;
  return VAE_OK;
}

extern "C" int vae_recon_loss(const vae_recon_loss_args* a, void* stream) {
  if (int rc = rl_check(a)) return rc;
  if (!ws_fits(rl_workspace_floats(a) * 4, a->workspace ? a->workspace_bytes : 0, "recon_loss")) return VAE_E_BADARG;
  hipStream_t st = (hipStream_t)stream;
  const int planes = a->n * a->c;
  if (a->kind == VAE_RLOSS_CENTER) {
    VAE_LAUNCH(center_plane_kernel, dim3(planes), dim3(RL_T), 0, st, *a);
    if (int rc = check_launch("recon_loss center")) return rc;
    VAE_LAUNCH(center_finalize_kernel, dim3(1), dim3(RL_T), 0, st, *a, planes);
    return check_launch("recon_loss center finalize");
  }
  const size_t lds = 0;                     // (static LDS, RL_LDS floats)
  VAE_LAUNCH(mssim_plane_kernel<false>, dim3(planes), dim3(RL_T), lds, st, *a);
  if (int rc = check_launch("recon_loss mssim")) return rc;
  VAE_LAUNCH(mssim_finalize_kernel, dim3(1), dim3(RL_T), 0, st, *a, planes);
  if (int rc = check_launch("recon_loss mssim finalize")) return rc;
  if (a->grad) {
    VAE_LAUNCH(mssim_plane_kernel<true>, dim3(planes), dim3(RL_T), lds, st, *a);
    return check_launch("recon_loss mssim backward");
  }
  return VAE_OK;
}
