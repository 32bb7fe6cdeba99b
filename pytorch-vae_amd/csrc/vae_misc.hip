// Non-GEMM kernels of the VAE step: the decoder head (final Conv2d(C->3)+Tanh+SSE, a thin-N
// layer that would waste 13/16 of an MFMA tile, so it runs on the VALU with its input tile
// staged once in LDS), the reparameterization, the ELBO reductions, Adam, and utilities.
#include <cxxabi.h>
#include <algorithm>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>

#include <math.h>

#include "vae_common.hpp"
#include "vae_elbo.hpp"

namespace vae {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int check_launch(const char* what) {
  if (querying()) return VAE_OK;            // nothing was launched (workspace query)
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail((int)e, "%s: %s", what, hipGetErrorString(e));
  return VAE_OK;
}

namespace {

constexpr int HEAD_MAXC = 512;     // channels entering the head (the Autoencoder's widest final layer:
                                   // configs/patient_vvbig_ae.yaml, hidden_dims[0] = 512)
constexpr int HEAD_CW = 32;        // channels staged per pass when the input has more than 64
constexpr int HEAD_T = 256;        // threads = pixels per tile
constexpr int CO = 3;              // RGB
constexpr int HEAD_GS = 774;       // max (rows+2)*(w+2) with rows*w == 256

struct HeadP {
  int n, h, w, c, rows, samples, tiles;
  const void* x; vae_xform xf;
  const float* wt; const float* bias; const float* target;
  float* recon; float* sse; const float* coef;
  void* dx; vae_xform epi; float* dgamma; float* dbeta;
  int sum_reps, sum_rstride;
  float* dw; float* db;
  const float* grad_recon;
  float* det_slab;           // deterministic calls: per-workgroup partial rows (OrdSum)
};

__device__ __forceinline__ float act_of(const vae_xform& xf, const float* ta, const float* tb, float v, int ch) {
  if (xf.kind == VAE_X_BN_ACT) return lrelu(fmaf(v, ta[ch], tb[ch]), xf.slope);
  if (xf.kind == VAE_X_ACT) return lrelu(v, xf.slope);
  return v;
}

// BN forward coefficients of the head input (and x̂ = y*p + q for the backward epilogue);
// `update_running`: this block also applies the BatchNorm running-stat update (once per call)
__device__ void head_coefs(const vae_xform& xf, float* ta, float* tb, float* tp, float* tq,
                           bool update_running = false) {
  if (xf.kind != VAE_X_BN_ACT) return;
  if (xf.table) {
    const int C = xf.channels;
    for (int ch = threadIdx.x; ch < C; ch += blockDim.x) {
      ta[ch] = xf.table[ch]; tb[ch] = xf.table[C + ch];
      if (tp) { tp[ch] = xf.table[2 * C + ch]; tq[ch] = xf.table[3 * C + ch]; }
    }
    return;
  }
  for (int ch = threadIdx.x; ch < xf.channels; ch += blockDim.x) {
    float mean, invstd, var;
    bn_moments(xf, ch, mean, invstd, var);
    ta[ch] = xf.gamma[ch] * invstd;
    tb[ch] = xf.beta[ch] - mean * ta[ch];
    if (tp) { tp[ch] = invstd; tq[ch] = -mean * invstd; }
    if (update_running && xf.running_mean) {
      const float m = xf.momentum;
      const float unb = xf.count > 1.f ? var * xf.count / (xf.count - 1.f) : var;
      xf.running_mean[ch] = (1.f - m) * xf.running_mean[ch] + m * mean;
      xf.running_var[ch] = (1.f - m) * xf.running_var[ch] + m * unb;
    }
  }
}

// Channels staged per pass: all of them up to 32 (one tile of (rows+2) x (w+2) x (c+4) floats),
// HEAD_CW at a time above (a 64-channel tile of a 64-wide image is already 105 KB)
__host__ __device__ inline int head_cw(int c) { return c > 32 ? HEAD_CW : c; }

// Stage act(x) rows [h0-1, h0+rows] x cols [-1, w], channels [c0, c0+cw) into LDS as
// [(rows+2)][(w+2)][cw+4] floats
template <class T>
__device__ void stage_input(const HeadP& p, int n, int h0, float* xs, const float* ta, const float* tb, int c0,
                            int cw) {
  const int CP = cw + 4, WP = p.w + 2;
  const int oct_per_pix = cw / 8;
  const int total = (p.rows + 2) * WP * oct_per_pix;
  const T* X = static_cast<const T*>(p.x);
  for (int e = threadIdx.x; e < total; e += blockDim.x) {
    const int o = e % oct_per_pix;
    const int pix = e / oct_per_pix;
    const int cc = pix % WP, rr = pix / WP;
    const int hi = h0 + rr - 1, wi = cc - 1;
    float v[8];
    if (hi >= 0 && hi < p.h && wi >= 0 && wi < p.w) {
      ld8(X + (((long)n * p.h + hi) * p.w + wi) * p.c + c0 + o * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = act_of(p.xf, ta, tb, v[j], c0 + o * 8 + j);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = 0.f;
    }
    float* d = xs + (rr * WP + cc) * CP + o * 8;
    *reinterpret_cast<f32x4*>(d) = f32x4{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<f32x4*>(d + 4) = f32x4{v[4], v[5], v[6], v[7]};
  }
}

// recon = tanh(conv3x3(act(x)) + b) -> NCHW; sse[n] += Σ (recon - target)^2
template <class T>
__global__ void __launch_bounds__(HEAD_T) head_fwd_kernel(HeadP p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ float ta[HEAD_MAXC], tb[HEAD_MAXC], ws[CO * 9 * 64], red[HEAD_T / 64];
  const int tiles_per_img = p.h / p.rows;
  const int n = blockIdx.x / tiles_per_img, h0 = (blockIdx.x % tiles_per_img) * p.rows;
  head_coefs(p.xf, ta, tb, nullptr, nullptr, blockIdx.x == 0);
  const int cw = head_cw(p.c);
  const int CP = cw + 4, WP = p.w + 2;
  const int tr = threadIdx.x / p.w, tc = threadIdx.x % p.w;
  float o[CO] = {p.bias[0], p.bias[1], p.bias[2]};
  for (int c0 = 0; c0 < p.c; c0 += cw) {
    __syncthreads();                                 // tables / the previous pass's reads
    for (int i = threadIdx.x; i < CO * 9 * cw; i += blockDim.x) {   // weights [co][tap][c0 .. c0+cw)
      const int ct = i / cw, c = i - ct * cw;
      ws[i] = p.wt[ct * p.c + c0 + c];
    }
    stage_input<T>(p, n, h0, smem, ta, tb, c0, cw);
    __syncthreads();
    for (int r = 0; r < 3; ++r)
      for (int s = 0; s < 3; ++s) {
        const float* xp = smem + ((tr + r) * WP + tc + s) * CP;
        const float* wp = ws + (r * 3 + s) * cw;
        for (int c = 0; c < cw; c += 4) {
          const f32x4 xv = *reinterpret_cast<const f32x4*>(xp + c);
#pragma unroll
          for (int co = 0; co < CO; ++co) {
            const float* wq = wp + co * 9 * cw + c;
            o[co] = fmaf(xv[0], wq[0], fmaf(xv[1], wq[1], fmaf(xv[2], wq[2], fmaf(xv[3], wq[3], o[co]))));
          }
        }
      }
  }
  const int hh = h0 + tr;
  const int img_t = n / p.samples;
  float sq = 0.f;
#pragma unroll
  for (int co = 0; co < CO; ++co) {
    const float y = tanhf(o[co]);
    const long oi = (((long)n * CO + co) * p.h + hh) * p.w + tc;
    p.recon[oi] = y;
    const float d = y - p.target[(((long)img_t * CO + co) * p.h + hh) * p.w + tc];
    sq = fmaf(d, d, sq);
  }
  for (int off = 32; off > 0; off >>= 1) sq += __shfl_xor(sq, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sq;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < HEAD_T / 64; ++i) t += red[i];
    if (p.det_slab) p.det_slab[blockIdx.x] = t;
    else atomicAdd(p.sse + n, t);
  }
}

// gseed = coef[img] * (recon - target) * (1 - recon^2)   (d loss / d pre-tanh)
__device__ __forceinline__ float gseed_at(const HeadP& p, int n, int co, int h, int w) {
  const long oi = (((long)n * CO + co) * p.h + h) * p.w + w;
  const float y = p.recon[oi];
  if (p.grad_recon) return p.grad_recon[oi] * (1.f - y * y);
  const float t = p.target[(((long)(n / p.samples) * CO + co) * p.h + h) * p.w + w];
  return p.coef[n] * (y - t) * (1.f - y * y);
}

// dx[h,w,c] = Σ_{r,s,co} gseed[h+1-r, w+1-s, co] · W[co][r][s][c], then the BN/LReLU backward
template <class T, int C>
__global__ void __launch_bounds__(HEAD_T) head_bwd_data_kernel(HeadP p) {
  __shared__ float ta[C], tb[C], tp[C], tq[C];
  __shared__ float ws[CO * 9 * C];
  __shared__ float gs[HEAD_GS * CO];                         // (rows+2) x (w+2) x 3
  __shared__ float r1[4][C], r2[4][C];
  const int tiles_per_img = p.h / p.rows;
  const int n = blockIdx.x / tiles_per_img, h0 = (blockIdx.x % tiles_per_img) * p.rows;
  head_coefs(p.epi, ta, tb, tp, tq);
  for (int i = threadIdx.x; i < CO * 9 * C; i += blockDim.x) ws[i] = p.wt[i];
  const int WP = p.w + 2;
  for (int e = threadIdx.x; e < (p.rows + 2) * WP; e += blockDim.x) {
    const int cc = e % WP, rr = e / WP;
    const int hi = h0 + rr - 1, wi = cc - 1;
    const bool in = hi >= 0 && hi < p.h && wi >= 0 && wi < p.w;
#pragma unroll
    for (int co = 0; co < CO; ++co) gs[e * CO + co] = in ? gseed_at(p, n, co, hi, wi) : 0.f;
  }
  __syncthreads();
  const int tr = threadIdx.x / p.w, tc = threadIdx.x % p.w;
  float da[C];
#pragma unroll
  for (int c = 0; c < C; ++c) da[c] = 0.f;
#pragma unroll 1
  for (int r = 0; r < 3; ++r)
#pragma unroll 1
    for (int s = 0; s < 3; ++s) {
      const float* g = gs + ((tr + 2 - r) * WP + (tc + 2 - s)) * CO;
#pragma unroll
      for (int co = 0; co < CO; ++co) {
        const float gv = g[co];
        const float* wq = ws + co * 9 * C + (r * 3 + s) * C;
#pragma unroll
        for (int c = 0; c < C; ++c) da[c] = fmaf(gv, wq[c], da[c]);
      }
    }
  // BN + LeakyReLU backward of the head input
  const long base = (((long)n * p.h + h0 + tr) * p.w + tc) * C;
  const T* Y = static_cast<const T*>(p.epi.aux);
  T* DX = static_cast<T*>(p.dx);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int c0 = 0; c0 < C; c0 += 8) {
    float y[8];
    if (p.epi.kind != VAE_X_NONE) ld8(Y + base + c0, y);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j;
      float gv = da[c], s1 = 0.f, s2 = 0.f;
      if (p.epi.kind == VAE_X_BN_ACT) {
        const float z = fmaf(y[j], ta[c], tb[c]);
        gv = z > 0.f ? gv : gv * p.epi.slope;
        s1 = gv;
        s2 = gv * fmaf(y[j], tp[c], tq[c]);
      } else if (p.epi.kind == VAE_X_ACT) {
        gv = y[j] > 0.f ? gv : gv * p.epi.slope;
      }
      DX[base + c] = cvt<T>(gv);
      if (p.epi.kind == VAE_X_BN_ACT) {
        for (int off = 32; off > 0; off >>= 1) { s1 += __shfl_xor(s1, off); s2 += __shfl_xor(s2, off); }
        if (lane == 0) { r1[wv][c] = s1; r2[wv][c] = s2; }
      }
    }
  }
  if (p.epi.kind == VAE_X_BN_ACT) {
    __syncthreads();
    const long roff = p.sum_reps > 1 ? (long)(blockIdx.x % p.sum_reps) * p.sum_rstride : 0;
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      const float b = r1[0][c] + r1[1][c] + r1[2][c] + r1[3][c], g = r2[0][c] + r2[1][c] + r2[2][c] + r2[3][c];
      if (p.det_slab) {
        p.det_slab[(long)blockIdx.x * 2 * C + c] = b;
        p.det_slab[(long)blockIdx.x * 2 * C + C + c] = g;
      } else {
        atomicAdd(p.dbeta + roff + c, b);
        atomicAdd(p.dgamma + roff + c, g);
      }
    }
  }
}

// head_bwd_data_kernel for inputs wider than 64 channels (the Autoencoder's 128-512-channel final
// layers): the same sums, HEAD_CW channels at a time (a register accumulator per channel of the
// pass, the pass's weights in LDS)
template <class T>
__global__ void __launch_bounds__(HEAD_T) head_bwd_data_wide_kernel(HeadP p) {
  constexpr int CW = HEAD_CW;
  __shared__ float ta[HEAD_MAXC], tb[HEAD_MAXC], tp[HEAD_MAXC], tq[HEAD_MAXC];
  __shared__ float ws[CO * 9 * CW];
  __shared__ float gs[HEAD_GS * CO];
  __shared__ float r1[4][CW], r2[4][CW];
  const int C = p.c;
  const int tiles_per_img = p.h / p.rows;
  const int n = blockIdx.x / tiles_per_img, h0 = (blockIdx.x % tiles_per_img) * p.rows;
  head_coefs(p.epi, ta, tb, tp, tq);
  const int WP = p.w + 2;
  for (int e = threadIdx.x; e < (p.rows + 2) * WP; e += blockDim.x) {
    const int cc = e % WP, rr = e / WP;
    const int hi = h0 + rr - 1, wi = cc - 1;
    const bool in = hi >= 0 && hi < p.h && wi >= 0 && wi < p.w;
#pragma unroll
    for (int co = 0; co < CO; ++co) gs[e * CO + co] = in ? gseed_at(p, n, co, hi, wi) : 0.f;
  }
  const int tr = threadIdx.x / p.w, tc = threadIdx.x % p.w;
  const long base = (((long)n * p.h + h0 + tr) * p.w + tc) * C;
  const T* Y = static_cast<const T*>(p.epi.aux);
  T* DX = static_cast<T*>(p.dx);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long roff = p.sum_reps > 1 ? (long)(blockIdx.x % p.sum_reps) * p.sum_rstride : 0;
  for (int c0 = 0; c0 < C; c0 += CW) {
    __syncthreads();                                 // gs / tables, and the previous pass's ws, r1, r2
    for (int i = threadIdx.x; i < CO * 9 * CW; i += blockDim.x) {
      const int ct = i / CW, c = i - ct * CW;
      ws[i] = p.wt[ct * C + c0 + c];
    }
    __syncthreads();
    float da[CW];
#pragma unroll
    for (int c = 0; c < CW; ++c) da[c] = 0.f;
#pragma unroll 1
    for (int r = 0; r < 3; ++r)
#pragma unroll 1
      for (int s = 0; s < 3; ++s) {
        const float* g = gs + ((tr + 2 - r) * WP + (tc + 2 - s)) * CO;
#pragma unroll
        for (int co = 0; co < CO; ++co) {
          const float gv = g[co];
          const float* wq = ws + co * 9 * CW + (r * 3 + s) * CW;
#pragma unroll
          for (int c = 0; c < CW; ++c) da[c] = fmaf(gv, wq[c], da[c]);
        }
      }
#pragma unroll
    for (int k0 = 0; k0 < CW; k0 += 8) {
      float y[8];
      if (p.epi.kind != VAE_X_NONE) ld8(Y + base + c0 + k0, y);
      else {
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = c0 + k0 + j;
        float gv = da[k0 + j], s1 = 0.f, s2 = 0.f;
        if (p.epi.kind == VAE_X_BN_ACT) {
          const float z = fmaf(y[j], ta[c], tb[c]);
          gv = z > 0.f ? gv : gv * p.epi.slope;
          s1 = gv;
          s2 = gv * fmaf(y[j], tp[c], tq[c]);
        } else if (p.epi.kind == VAE_X_ACT) {
          gv = y[j] > 0.f ? gv : gv * p.epi.slope;
        }
        DX[base + c] = cvt<T>(gv);
        if (p.epi.kind == VAE_X_BN_ACT) {
          for (int off = 32; off > 0; off >>= 1) { s1 += __shfl_xor(s1, off); s2 += __shfl_xor(s2, off); }
          if (lane == 0) { r1[wv][k0 + j] = s1; r2[wv][k0 + j] = s2; }
        }
      }
    }
    if (p.epi.kind == VAE_X_BN_ACT) {
      __syncthreads();
      if (threadIdx.x < CW) {
        const int c = threadIdx.x;
        const float b = r1[0][c] + r1[1][c] + r1[2][c] + r1[3][c], g = r2[0][c] + r2[1][c] + r2[2][c] + r2[3][c];
        if (p.det_slab) {
          p.det_slab[(long)blockIdx.x * 2 * C + c0 + c] = b;
          p.det_slab[(long)blockIdx.x * 2 * C + C + c0 + c] = g;
        } else {
          atomicAdd(p.dbeta + roff + c0 + c, b);
          atomicAdd(p.dgamma + roff + c0 + c, g);
        }
      }
    }
  }
}

// dW[co][r][s][c] += Σ_pix gseed[pix][co] · act(x)[pix + (r-1, s-1)][c];  db[co] += Σ gseed
template <class T>
__global__ void __launch_bounds__(HEAD_T) head_bwd_filter_kernel(HeadP p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ float ta[HEAD_MAXC], tb[HEAD_MAXC], gs[HEAD_T * CO], red[CO][HEAD_T / 64];
  constexpr int NI = (9 * HEAD_MAXC + HEAD_T - 1) / HEAD_T;    // dW elements per thread
  const int nidx = 9 * p.c;
  const int cw = head_cw(p.c);
  float acc[NI][CO];
  float dbacc[CO] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int co = 0; co < CO; ++co) acc[i][co] = 0.f;
  head_coefs(p.xf, ta, tb, nullptr, nullptr);
  const int tiles_per_img = p.h / p.rows;
  const int CP = cw + 4, WP = p.w + 2;
  for (int tile = blockIdx.x; tile < p.tiles; tile += gridDim.x) {
    const int n = tile / tiles_per_img, h0 = (tile % tiles_per_img) * p.rows;
    __syncthreads();
    {
      const int tr = threadIdx.x / p.w, tc = threadIdx.x % p.w;
#pragma unroll
      for (int co = 0; co < CO; ++co) {
        const float g = gseed_at(p, n, co, h0 + tr, tc);
        gs[threadIdx.x * CO + co] = g;
        dbacc[co] += g;
      }
    }
    for (int c0 = 0; c0 < p.c; c0 += cw) {
      if (c0) __syncthreads();                       // the previous pass's reads of the tile
      stage_input<T>(p, n, h0, smem, ta, tb, c0, cw);
      __syncthreads();
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int idx = threadIdx.x + i * HEAD_T;
        if (idx >= nidx) break;
        const int tap = idx / p.c, c = idx - tap * p.c;
        if (c < c0 || c >= c0 + cw) continue;        // (this pass stages channels [c0, c0+cw))
        const int r = tap / 3, s = tap - r * 3;
        for (int pix = 0; pix < HEAD_T; ++pix) {
          const int tr = pix / p.w, tc = pix - tr * p.w;
          const float xv = smem[((tr + r) * WP + tc + s) * CP + c - c0];
#pragma unroll
          for (int co = 0; co < CO; ++co) acc[i][co] = fmaf(gs[pix * CO + co], xv, acc[i][co]);
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int idx = threadIdx.x + i * HEAD_T;
    if (idx >= nidx) break;
#pragma unroll
    for (int co = 0; co < CO; ++co) {
      if (p.det_slab) p.det_slab[(long)blockIdx.x * (CO * nidx + CO) + co * nidx + idx] = acc[i][co];
      else atomicAdd(p.dw + co * nidx + idx, acc[i][co]);
    }
  }
  if (p.db) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int co = 0; co < CO; ++co) {
      float s = dbacc[co];
      for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
      if (lane == 0) red[co][wv] = s;
    }
    __syncthreads();
    if (threadIdx.x < CO) {
      float t = 0.f;
      for (int i = 0; i < HEAD_T / 64; ++i) t += red[threadIdx.x][i];
      if (p.det_slab) p.det_slab[(long)blockIdx.x * (CO * nidx + CO) + CO * nidx + threadIdx.x] = t;
      else atomicAdd(p.db + threadIdx.x, t);
    }
  }
}

int head_setup(const vae_head_args* a, HeadP& p, const char* what) {
  if (!a || !a->x || !a->wt || !a->bias || !a->target || !a->recon) return fail(VAE_E_BADARG, "%s: null tensor", what);
  if (a->c % 8 || a->c > HEAD_MAXC || a->c <= 0 || (a->c > 32 && a->c % HEAD_CW))
    return fail(VAE_E_UNSUPPORTED, "%s: channels %d", what, a->c);
  if (a->w <= 0 || a->w > 256 || HEAD_T % a->w || a->h % (HEAD_T / a->w))
    return fail(VAE_E_UNSUPPORTED, "%s: spatial %dx%d (need w | 256 and (256/w) | h)", what, a->h, a->w);
  if (a->dtype != VAE_F32 && a->dtype != VAE_BF16) return fail(VAE_E_BADDTYPE, "%s: dtype", what);
  if (a->deterministic && a->dtype != VAE_F32)
    return fail(VAE_E_UNSUPPORTED, "%s: deterministic reductions need dtype VAE_F32", what);
  memset(&p, 0, sizeof(p));
  p.n = a->n; p.h = a->h; p.w = a->w; p.c = a->c; p.rows = HEAD_T / a->w;
  p.samples = a->samples > 0 ? a->samples : 1;
  p.tiles = a->n * (a->h / p.rows);
  p.x = a->x; p.xf = a->x_xf; p.wt = a->wt; p.bias = a->bias; p.target = a->target;
  p.recon = a->recon; p.sse = a->sse; p.coef = a->coef;
  p.dx = a->dx; p.epi = a->dx_epi; p.dgamma = a->dx_dgamma; p.dbeta = a->dx_dbeta;
  p.sum_reps = a->sum_reps; p.sum_rstride = a->sum_rstride;
  p.dw = a->dw; p.db = a->db; p.grad_recon = a->grad_recon;
  if (p.xf.channels <= 0) p.xf.channels = a->c;
  if (p.epi.channels <= 0) p.epi.channels = a->c;
  return VAE_OK;
}

// A deterministic head call keeps its per-workgroup partials (`floats` of them) at the start of
// the workspace; the entry point adds them with ordered_sum_launch after its kernel.
int head_det(const vae_head_args* a, HeadP& p, long floats, const char* what) {
  if (!a->deterministic || floats <= 0) return VAE_OK;
  if (!a->workspace && !querying()) return fail(VAE_E_BADARG, "%s: a deterministic call needs a workspace", what);
  if (!ws_fits(floats * 4, a->workspace_bytes, what)) return VAE_E_BADARG;
  p.det_slab = static_cast<float*>(a->workspace);
  return VAE_OK;
}

// ------------------------------------------------------------------ BatchNorm finalisation
__global__ void __launch_bounds__(256) bn_finalize_kernel(vae_bn_args a) {
  kernarg_prefetch<(sizeof(vae_bn_args) < 1024 ? sizeof(vae_bn_args) : 1024)>(); bn_finalize_block(a, blockIdx.x, gridDim.x); }

// Eval-mode BatchNorm: the forward table from the running statistics (torch eval semantics:
// (y - running_mean) / sqrt(running_var + eps) * gamma + beta).
__global__ void __launch_bounds__(256) bn_eval_table_kernel(vae_bn_args a) {
  const vae_xform& x = a.xf;
  const int C = x.channels;
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const float mean = x.running_mean[c];
  const float invstd = 1.0f / sqrtf(x.running_var[c] + x.eps);
  const float sc = x.gamma[c] * invstd;
  a.table[c] = sc;
  a.table[C + c] = x.beta[c] - mean * sc;
  a.table[2 * C + c] = invstd;
  a.table[3 * C + c] = -mean * invstd;
}

// ------------------------------------------------------------------ reparameterization
template <class T>
__global__ void reparam_kernel(int rows, int samples, int D, const float* mulv, const float* eps, T* z) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)rows * D) return;
  const int r = (int)(i / D), d = (int)(i - (long)r * D);
  const int b = r / samples;
  const float mu = mulv[(long)b * 2 * D + d], lv = mulv[(long)b * 2 * D + D + d];
  z[i] = cvt<T>(fmaf(eps[i], expf(0.5f * lv), mu));
}

// ---------------------------------------------------------------------------- ELBO
__global__ void __launch_bounds__(256) elbo_kernel(vae_elbo_args a) {
  kernarg_prefetch<(sizeof(vae_elbo_args) < 1024 ? sizeof(vae_elbo_args) : 1024)>();
  __shared__ float kld_row[1024];
  __shared__ float red[4][4];
  elbo_block(a, kld_row, red);
}

// ---------------------------------------------------------------------------- Adam
struct AdamK {
  float omb1, omb2, b2f, step_size, bc2s, eps, wd;
};
__device__ __forceinline__ float adam_elem(const AdamK& k, float& pi, float gi, float& mi, float& vi) {
  if (k.wd != 0.f) gi = fmaf(k.wd, pi, gi);
  mi = mi + k.omb1 * (gi - mi);                                      // lerp (torch Adam)
  vi = vi * k.b2f + k.omb2 * gi * gi;                                // mul_(beta2).addcmul_(g, g, 1-beta2)
  const float den = sqrtf(vi) / k.bc2s + k.eps;
  pi = pi - k.step_size * (mi / den);
  return pi;
}
// V = 4: 16-byte accesses (the four fp32 arrays 16-byte aligned, the bf16 copy 8-byte aligned),
// the n % 4 tail by block 0; V = 1: one element per access
template <bool LOWP, int V>
__global__ void __launch_bounds__(256) adam_kernel(long n, float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, const int* step,
                                                   const float* lr, double b1, double b2, float eps, float wd,
                                                   __bf16* __restrict__ lowp) {
  // torch.optim.Adam (single-tensor path): the scalars it derives from the Python-float
  // hyper-parameters (1 - beta, bias corrections, step size) are formed in double and rounded
  // once, as torch does — 1 - 0.999f in fp32 would be 1.3e-5 off 1 - 0.999
  const double t = (double)(*step);
  const double bc1 = 1.0 - pow(b1, t), bc2 = 1.0 - pow(b2, t);
  const AdamK k{(float)(1.0 - b1), (float)(1.0 - b2), (float)b2, (float)((double)*lr / bc1), (float)sqrt(bc2), eps, wd};
  const long stride = (long)gridDim.x * blockDim.x;
  const long nv = n / V;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
    if constexpr (V == 4) {
      f32x4 p4 = reinterpret_cast<const f32x4*>(p)[i];
      const f32x4 g4 = reinterpret_cast<const f32x4*>(g)[i];
      f32x4 m4 = reinterpret_cast<const f32x4*>(m)[i];
      f32x4 v4 = reinterpret_cast<const f32x4*>(v)[i];
      float pe[4], me[4], ve[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        pe[e] = p4[e]; me[e] = m4[e]; ve[e] = v4[e];
        adam_elem(k, pe[e], g4[e], me[e], ve[e]);
      }
      reinterpret_cast<f32x4*>(p)[i] = f32x4{pe[0], pe[1], pe[2], pe[3]};
      reinterpret_cast<f32x4*>(m)[i] = f32x4{me[0], me[1], me[2], me[3]};
      reinterpret_cast<f32x4*>(v)[i] = f32x4{ve[0], ve[1], ve[2], ve[3]};
      if (LOWP) reinterpret_cast<bf16x4*>(lowp)[i] = bf16x4{(__bf16)pe[0], (__bf16)pe[1], (__bf16)pe[2], (__bf16)pe[3]};
    } else {
      float pi = p[i], mi = m[i], vi = v[i];
      adam_elem(k, pi, g[i], mi, vi);
      m[i] = mi; v[i] = vi; p[i] = pi;
      if (LOWP) lowp[i] = (__bf16)pi;
    }
  }
  if (V > 1 && blockIdx.x == 0 && threadIdx.x < n - nv * V) {
    const long i = nv * V + threadIdx.x;
    float pi = p[i], mi = m[i], vi = v[i];
    adam_elem(k, pi, g[i], mi, vi);
    m[i] = mi; v[i] = vi; p[i] = pi;
    if (LOWP) lowp[i] = (__bf16)pi;
  }
}

__global__ void cast_bf16_kernel(long n, const float* src, __bf16* dst) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    dst[i] = (__bf16)src[i];
}

__global__ void step_begin_kernel(f32x4* z, long n16, unsigned char* tail, int ntail, int* step) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (long)gridDim.x * blockDim.x)
    z[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (blockIdx.x == 0 && threadIdx.x < ntail) tail[threadIdx.x] = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0 && step) *step += 1;
}

int grid_for(long n, int per_block = 256, int max_blocks = 2048) {
  long b = (n + per_block - 1) / per_block;
  if (b < 1) b = 1;
  return (int)(b > max_blocks ? max_blocks : b);
}

// The ordered pass of a deterministic call (OrdSum, vae_common.hpp): 32 outputs per workgroup,
// 8 row lanes each taking the rows r = lane (mod 8) in ascending order, the 8 lane totals added
// in lane order — a fixed summation tree whatever the timing.
__global__ void __launch_bounds__(256) ordered_sum_kernel(const OrdSum o) {
  __shared__ float part[8][33];
  const int cl = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const long e = (long)blockIdx.x * 32 + cl;
  const bool ok = e < (long)o.groups * o.cols;
  const int g = ok ? (int)(e / o.cols) : 0;
  const int c = ok ? (int)(e - (long)g * o.cols) : 0;
  const int half = c / o.cw, cc = c - half * o.cw;
  const float* base = o.slab + (long)g * o.rpg * o.rstride + (long)half * o.hstride + cc;
  float s = 0.f;
  if (ok) {
    int r = rl;
    for (; r + 24 < o.rpg; r += 32) {                      // 4 rows' loads in flight
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float t = 0.f;
        for (int f = 0; f < o.folds; ++f) t += base[(long)(r + 8 * u) * o.rstride + (long)f * o.fstride];
        v[u] = t;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) s += v[u];
    }
    for (; r < o.rpg; r += 8) {
      float t = 0.f;
      for (int f = 0; f < o.folds; ++f) t += base[(long)r * o.rstride + (long)f * o.fstride];
      s += t;
    }
  }
  part[rl][cl] = s;
  __syncthreads();
  if (rl == 0 && ok) {
    float t = 0.f;
#pragma unroll
    for (int l = 0; l < 8; ++l) t += part[l][cl];
    float* d = o.dst[half] + (long)g * o.gstride + cc;
    *d += t;
  }
}

}  // namespace

int ordered_sum_launch(const OrdSum& o, hipStream_t st) {
  const long outs = (long)o.groups * o.cols;
  if (outs <= 0 || o.rpg <= 0) return VAE_OK;
  if (!o.slab || !o.dst[0] || (o.cols > o.cw && !o.dst[1]))
    return fail(VAE_E_BADARG, "ordered_sum: null slab or destination");
  VAE_LAUNCH(ordered_sum_kernel, dim3((unsigned)((outs + 31) / 32)), dim3(256), 0, st, o);
  return check_launch("ordered_sum");
}
}  // namespace vae

using namespace vae;

extern "C" int vae_abi_version(void) { return VAE_ABI_VERSION; }

extern "C" int vae_launch_log(int32_t on) {
  LaunchLog& l = launch_log();
  if (on) l.n = 0;
  l.on = on ? 1 : 0;
  return VAE_OK;
}

extern "C" int64_t vae_launch_log_names(char* buf, int64_t cap) {
  const LaunchLog& l = launch_log();
  int64_t need = 0;
  for (int i = 0; i < l.n; ++i) {
    const char* m = hipKernelNameRefByPtr(l.k[i], nullptr);
    if (!m) m = "?";
    int st = 0;
    char* d = abi::__cxa_demangle(m, nullptr, nullptr, &st);
    const int w = snprintf(buf && need < cap ? buf + need : nullptr, buf && need < cap ? (size_t)(cap - need) : 0,
                           "%s\t%s\t%d\n", m, (st == 0 && d) ? d : m, l.count[i]);
    free(d);
    need += w > 0 ? w : 0;
  }
  if (buf && cap > 0 && need >= cap) buf[cap - 1] = '\0';
  return need + 1;
}
extern "C" const char* vae_last_error(void) { return g_err; }

#ifdef VAE_PROBE
// Diagnostics build only: device buffer the GEMM kernels append per-block phase records to.
static unsigned long long* g_probe = nullptr;
extern "C" void vae_probe_set(void* buf) { g_probe = static_cast<unsigned long long*>(buf); }
extern "C" unsigned long long* vae_probe_buffer(void) { return g_probe; }
#endif

namespace vae {
int head_fwd_mfma_launch(const vae_head_args* a, hipStream_t st);
int head_bwd_mfma_launch(const vae_head_args* a, bool data, bool filter, hipStream_t st);
}

extern "C" int vae_head_fwd(const vae_head_args* a, void* stream) {
  HeadP p;
  int rc = head_setup(a, p, "head_fwd");
  if (rc) return rc;
  if (!a->sse) return fail(VAE_E_BADARG, "head_fwd: sse");
  rc = head_fwd_mfma_launch(a, (hipStream_t)stream);   // bf16, 64-wide, 32 channels
  if (rc != kHeadFallback) return rc;
  const size_t lds = (size_t)(p.rows + 2) * (p.w + 2) * (head_cw(p.c) + 4) * sizeof(float);
  if (lds > 64 * 1024) return fail(VAE_E_UNSUPPORTED, "head_fwd: tile too large");
  if ((rc = head_det(a, p, p.tiles, "head_fwd"))) return rc;
  if (a->dtype == VAE_F32) VAE_LAUNCH(head_fwd_kernel<float>, dim3(p.tiles), dim3(HEAD_T), lds, (hipStream_t)stream, p);
  else VAE_LAUNCH(head_fwd_kernel<__bf16>, dim3(p.tiles), dim3(HEAD_T), lds, (hipStream_t)stream, p);
  if ((rc = check_launch("head_fwd")) || !p.det_slab) return rc;
  OrdSum o;                                          // sse[n] += the image's tiles, in tile order
  memset(&o, 0, sizeof(o));
  o.slab = p.det_slab; o.rstride = 1; o.groups = p.n; o.rpg = p.h / p.rows; o.cols = 1; o.cw = 1; o.folds = 1;
  o.dst[0] = p.sse; o.gstride = 1;
  return ordered_sum_launch(o, (hipStream_t)stream);
}

extern "C" int vae_head_bwd_data(const vae_head_args* a, void* stream) {
  HeadP p;
  int rc = head_setup(a, p, "head_bwd_data");
  if (rc) return rc;
  if ((!a->coef && !a->grad_recon) || !a->dx) return fail(VAE_E_BADARG, "head_bwd_data: coef/grad_recon/dx");
  if (p.epi.kind == VAE_X_BN_ACT && (!p.dgamma || !p.dbeta || !p.epi.aux)) return fail(VAE_E_BADARG, "head_bwd_data: BN epilogue");
  if (p.epi.kind != VAE_X_NONE && !p.epi.aux) return fail(VAE_E_BADARG, "head_bwd_data: epilogue aux");
  const hipStream_t st = (hipStream_t)stream;
  rc = head_bwd_mfma_launch(a, true, false, st);
  if (rc != kHeadFallback) return rc;
  const bool f = a->dtype == VAE_F32;
  const bool sums = p.epi.kind == VAE_X_BN_ACT;
  if (sums && (rc = head_det(a, p, (long)p.tiles * 2 * p.c, "head_bwd_data"))) return rc;
  switch (a->c) {
    case 32:
      if (f) VAE_LAUNCH((head_bwd_data_kernel<float, 32>), dim3(p.tiles), dim3(HEAD_T), 0, st, p);
      else VAE_LAUNCH((head_bwd_data_kernel<__bf16, 32>), dim3(p.tiles), dim3(HEAD_T), 0, st, p);
      break;
    case 64:
      if (f) VAE_LAUNCH((head_bwd_data_kernel<float, 64>), dim3(p.tiles), dim3(HEAD_T), 0, st, p);
      else VAE_LAUNCH((head_bwd_data_kernel<__bf16, 64>), dim3(p.tiles), dim3(HEAD_T), 0, st, p);
      break;
    default:      // (head_setup: 64 < c <= HEAD_MAXC, c % HEAD_CW == 0)
      if (a->c <= 64) return fail(VAE_E_UNSUPPORTED, "head_bwd_data: channels %d (32, 64 or a multiple of %d)", a->c, HEAD_CW);
      if (f) VAE_LAUNCH((head_bwd_data_wide_kernel<float>), dim3(p.tiles), dim3(HEAD_T), 0, st, p);
      else VAE_LAUNCH((head_bwd_data_wide_kernel<__bf16>), dim3(p.tiles), dim3(HEAD_T), 0, st, p);
      break;
  }
  if ((rc = check_launch("head_bwd_data")) || !p.det_slab) return rc;
  OrdSum o;                                          // Σg, Σg·x̂ over the tiles, in tile order
  memset(&o, 0, sizeof(o));
  o.slab = p.det_slab; o.rstride = 2L * p.c; o.groups = 1; o.rpg = p.tiles; o.cols = 2 * p.c; o.cw = p.c;
  o.hstride = p.c; o.folds = 1; o.dst[0] = p.dbeta; o.dst[1] = p.dgamma;
  return ordered_sum_launch(o, st);
}

extern "C" int vae_head_bwd_filter(const vae_head_args* a, void* stream) {
  HeadP p;
  int rc = head_setup(a, p, "head_bwd_filter");
  if (rc) return rc;
  if ((!a->coef && !a->grad_recon) || !a->dw) return fail(VAE_E_BADARG, "head_bwd_filter: coef/grad_recon/dw");
  if (9 * a->c > 9 * HEAD_MAXC) return fail(VAE_E_UNSUPPORTED, "head_bwd_filter: channels");
  rc = head_bwd_mfma_launch(a, false, true, (hipStream_t)stream);
  if (rc != kHeadFallback) return rc;
  const size_t lds = (size_t)(p.rows + 2) * (p.w + 2) * (head_cw(p.c) + 4) * sizeof(float);
  const int grid = p.tiles < 256 ? p.tiles : 256;
  const int nw = CO * 9 * p.c;                       // dW elements; db follows in a partial row
  if ((rc = head_det(a, p, (long)grid * (nw + CO), "head_bwd_filter"))) return rc;
  if (a->dtype == VAE_F32) VAE_LAUNCH(head_bwd_filter_kernel<float>, dim3(grid), dim3(HEAD_T), lds, (hipStream_t)stream, p);
  else VAE_LAUNCH(head_bwd_filter_kernel<__bf16>, dim3(grid), dim3(HEAD_T), lds, (hipStream_t)stream, p);
  if ((rc = check_launch("head_bwd_filter")) || !p.det_slab) return rc;
  OrdSum o;                                          // dW, db over the workgroups, in order
  memset(&o, 0, sizeof(o));
  o.slab = p.det_slab; o.rstride = nw + CO; o.groups = 1; o.rpg = grid; o.cols = p.db ? nw + CO : nw; o.cw = nw;
  o.hstride = nw; o.folds = 1; o.dst[0] = p.dw; o.dst[1] = p.db;
  return ordered_sum_launch(o, (hipStream_t)stream);
}

extern "C" int vae_bn_finalize(const vae_bn_args* a, void* stream) { return vae::bn_finalize_launch(a, (hipStream_t)stream); }

int vae::bn_finalize_launch(const vae_bn_args* a, hipStream_t stream) {
  if (!a || !a->table || a->xf.channels <= 0 || !a->xf.sum || !a->xf.sumsq || !a->xf.gamma || !a->xf.beta ||
      a->xf.count <= 0.f)
    return fail(VAE_E_BADARG, "bn_finalize: args");
  if (a->mode < 0 || a->mode > 2) return fail(VAE_E_BADARG, "bn_finalize: mode %d", a->mode);
  if (a->mode == 2) {
    if (!a->xf.running_mean || !a->xf.running_var) return fail(VAE_E_BADARG, "bn_finalize: eval mode needs running statistics");
    VAE_LAUNCH(bn_eval_table_kernel, dim3((a->xf.channels + 255) / 256), dim3(256), 0, (hipStream_t)stream, *a);
    return check_launch("bn_finalize(eval)");
  }
  if (a->mode == 1 && (!a->xf.dgamma || !a->xf.dbeta)) return fail(VAE_E_BADARG, "bn_finalize: backward sums");
  if (a->xf.reps > BNF_LANES * BNF_PER) return fail(VAE_E_UNSUPPORTED, "bn_finalize: %d replicas > %d", a->xf.reps, BNF_LANES * BNF_PER);
  const int grid = (a->xf.channels + 63) / 64;
  VAE_LAUNCH(bn_finalize_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, *a);
  return check_launch("bn_finalize");
}

extern "C" int vae_head_bwd(const vae_head_args* a, void* stream) {
  HeadP p;
  int rc = head_setup(a, p, "head_bwd");
  if (rc) return rc;
  if ((!a->coef && !a->grad_recon && !a->elbo) || !a->dx || !a->dw) return fail(VAE_E_BADARG, "head_bwd: coef/grad_recon/dx/dw");
  if (p.epi.kind == VAE_X_BN_ACT && (!p.dgamma || !p.dbeta || !p.epi.aux)) return fail(VAE_E_BADARG, "head_bwd: BN epilogue");
  rc = head_bwd_mfma_launch(a, true, true, (hipStream_t)stream);
  if (rc == kHeadFallback && a->elbo) return fail(VAE_E_UNSUPPORTED, "head_bwd: a fused ELBO needs the bf16 MFMA path");
  if (rc == kHeadFallback) {
    if ((rc = vae_head_bwd_data(a, stream))) return rc;
    rc = vae_head_bwd_filter(a, stream);
  }
  if (rc || !a->bn_finalize) return rc;
  return bn_finalize_launch(a->bn_finalize, (hipStream_t)stream);     // the final BatchNorm's backward table
}

extern "C" int vae_reparam_fwd(int32_t dtype, int32_t rows, int32_t samples, int32_t latent, const float* mulv,
                               const float* eps, void* z, void* stream) {
  if (!mulv || !eps || !z || rows <= 0 || latent <= 0 || samples <= 0) return fail(VAE_E_BADARG, "reparam_fwd: args");
  const long n = (long)rows * latent;
  const int grid = (int)((n + 255) / 256);
  if (dtype == VAE_F32) VAE_LAUNCH(reparam_kernel<float>, dim3(grid), dim3(256), 0, (hipStream_t)stream, rows, samples, latent, mulv, eps, (float*)z);
  else if (dtype == VAE_BF16) VAE_LAUNCH(reparam_kernel<__bf16>, dim3(grid), dim3(256), 0, (hipStream_t)stream, rows, samples, latent, mulv, eps, (__bf16*)z);
  else return fail(VAE_E_BADDTYPE, "reparam_fwd: dtype");
  return check_launch("reparam_fwd");
}

extern "C" int vae_elbo_fwd(const vae_elbo_args* a, void* stream) {
  if (!a || !a->sse || !a->out || !a->per_img) return fail(VAE_E_BADARG, "elbo_fwd: args");
  if (a->kind < VAE_LOSS_VANILLA || a->kind > VAE_LOSS_VQ) return fail(VAE_E_BADARG, "elbo_fwd: kind");
  if (a->kind == VAE_LOSS_VQ) {
    if (!a->vq_sse || !(a->vq_elems > 0.f)) return fail(VAE_E_BADARG, "elbo_fwd: vq_sse / vq_elems");
    if (a->batch <= 0 || a->img_elems <= 0 || (a->samples > 1)) return fail(VAE_E_BADSHAPE, "elbo_fwd: sizes");
  } else {
    if (!a->mulv || !a->head_coef || !a->kl_coef) return fail(VAE_E_BADARG, "elbo_fwd: args");
    if (a->batch <= 0 || a->batch > 1024 || a->latent <= 0 || a->img_elems <= 0) return fail(VAE_E_BADSHAPE, "elbo_fwd: sizes");
  }
  VAE_LAUNCH(elbo_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, *a);
  return check_launch("elbo_fwd");
}

extern "C" int vae_adam_step(int64_t n, float* p, const float* g, float* m, float* v, const int32_t* step,
                             const float* lr, double beta1, double beta2, float eps, float weight_decay, void* p_lowp,
                             void* stream) {
  if (n <= 0) return VAE_OK;
  if (!p || !g || !m || !v || !step || !lr) return fail(VAE_E_BADARG, "adam_step: null");
  auto al = [](const void* q, uintptr_t a) { return ((uintptr_t)q % a) == 0; };
  const bool vec = al(p, 16) && al(g, 16) && al(m, 16) && al(v, 16) && (!p_lowp || al(p_lowp, 8));
  const hipStream_t st = (hipStream_t)stream;
  __bf16* lp = (__bf16*)p_lowp;
  if (vec) {
    const int grid = grid_for((n + 3) / 4);
    if (p_lowp) VAE_LAUNCH((adam_kernel<true, 4>), dim3(grid), dim3(256), 0, st, (long)n, p, g, m, v, step, lr, beta1, beta2, eps, weight_decay, lp);
    else VAE_LAUNCH((adam_kernel<false, 4>), dim3(grid), dim3(256), 0, st, (long)n, p, g, m, v, step, lr, beta1, beta2, eps, weight_decay, lp);
  } else {
    const int grid = grid_for(n);
    if (p_lowp) VAE_LAUNCH((adam_kernel<true, 1>), dim3(grid), dim3(256), 0, st, (long)n, p, g, m, v, step, lr, beta1, beta2, eps, weight_decay, lp);
    else VAE_LAUNCH((adam_kernel<false, 1>), dim3(grid), dim3(256), 0, st, (long)n, p, g, m, v, step, lr, beta1, beta2, eps, weight_decay, lp);
  }
  return check_launch("adam_step");
}

// ---------------------------------------------------------------------------- deferred reductions
extern "C" int vae_deferred_reset(void) {
  deferred().n = 0;
  deferred().has_elbo = 0;
  return VAE_OK;
}

extern "C" int32_t vae_deferred_take(vae_grad_slab* out, int32_t max, vae_elbo_args* elbo, int32_t* has_elbo) {
  Deferred& d = deferred();
  const int n = d.n;
  for (int i = 0; i < n && i < max && out; ++i) out[i] = d.s[i];
  if (has_elbo) *has_elbo = d.has_elbo;
  if (elbo && d.has_elbo) *elbo = d.elbo;
  d.n = 0;
  d.has_elbo = 0;
  return n;
}

namespace {

// vae_adam_step_ex in one grid (the slab workgroups first: dispatched first, their longer
// reductions overlap the streaming of the plain elements instead of trailing it):
//   [0, nslabblk)             per descriptor: "tall" slabs (rows >= kTallRows: the head's and the
//                             full-resolution ConvT's per-workgroup partials) as 16 columns x 16 row
//                             parts per workgroup, parts combined in LDS in ascending order; "short"
//                             slabs (K slices of the grouped weight gradients) as 256 quads per
//                             workgroup, each thread summing its quad's rows in ascending order —
//                             then g = that sum is written and the element's Adam update runs
//   [nslabblk]                the deferred loss (elbo_block), when present
//   [.., + nreg)              vae_adam_step over the elements no descriptor covers (grid-stride,
//                             16-byte accesses; quads inside a descriptor's range are skipped)
constexpr int kTallRows = 64;
struct AdamEx {
  long n;
  float* p; float* g; float* m; float* v;
  const int* step; const float* lr;
  double b1, b2;
  float eps, wd;
  __bf16* lowp;
  int nreg, nslab;
  int tall[VAE_SLAB_MAX];
  int blk0[VAE_SLAB_MAX + 1];        // first workgroup of each descriptor, relative to nreg
  long q0[VAE_SLAB_MAX], q1[VAE_SLAB_MAX];   // quads [q0, q1) of g a descriptor covers (ascending q0)
  long off[VAE_SLAB_MAX];            // element offset of dst in g
  vae_grad_slab s[VAE_SLAB_MAX];
  int has_elbo;
  vae_elbo_args e;
};

__device__ __forceinline__ AdamK adam_k(const AdamEx& a) {
  const double t = (double)(*a.step);
  const double bc1 = 1.0 - pow(a.b1, t), bc2 = 1.0 - pow(a.b2, t);
  return AdamK{(float)(1.0 - a.b1), (float)(1.0 - a.b2), (float)a.b2, (float)((double)*a.lr / bc1), (float)sqrt(bc2),
               a.eps, a.wd};
}

template <bool LOWP>
__device__ __forceinline__ void adam_one(const AdamEx& a, const AdamK& k, long i, float gi) {
  float pi = a.p[i], mi = a.m[i], vi = a.v[i];
  adam_elem(k, pi, gi, mi, vi);
  a.m[i] = mi; a.v[i] = vi; a.p[i] = pi;
  if (LOWP) a.lowp[i] = (__bf16)pi;
}

template <bool LOWP>
__device__ __forceinline__ void adam_quad(const AdamEx& a, const AdamK& k, long i, const f32x4 g4) {
  f32x4 p4 = reinterpret_cast<const f32x4*>(a.p)[i];
  f32x4 m4 = reinterpret_cast<const f32x4*>(a.m)[i];
  f32x4 v4 = reinterpret_cast<const f32x4*>(a.v)[i];
  float pe[4], me[4], ve[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    pe[e] = p4[e]; me[e] = m4[e]; ve[e] = v4[e];
    adam_elem(k, pe[e], g4[e], me[e], ve[e]);
  }
  reinterpret_cast<f32x4*>(a.p)[i] = f32x4{pe[0], pe[1], pe[2], pe[3]};
  reinterpret_cast<f32x4*>(a.m)[i] = f32x4{me[0], me[1], me[2], me[3]};
  reinterpret_cast<f32x4*>(a.v)[i] = f32x4{ve[0], ve[1], ve[2], ve[3]};
  if (LOWP) reinterpret_cast<bf16x4*>(a.lowp)[i] = bf16x4{(__bf16)pe[0], (__bf16)pe[1], (__bf16)pe[2], (__bf16)pe[3]};
}

// (a streaming kernel: <= 64 VGPRs keeps 8 waves per SIMD; at 104 it ran 4 and took 33 us for the
// 19.6 us of bytes of vae_adam_step plus the slabs)
template <bool LOWP>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) adam_ex_kernel(const AdamEx ka) {
  kernarg_prefetch<1024>();
  // fields read in place (a runtime descriptor index would copy the by-value block to scratch)
  (void)ka;
  const AdamEx& a = *(const AdamEx*)(const void*)__builtin_amdgcn_kernarg_segment_ptr();
  const int tid = threadIdx.x;
  const int nslabblk = a.blk0[a.nslab];
  if (a.has_elbo && (int)blockIdx.x == nslabblk) {
    __shared__ float kld_row[1024];
    __shared__ float ered[4][4];
    elbo_block(a.e, kld_row, ered);
    return;
  }
  const AdamK k = adam_k(a);
  if ((int)blockIdx.x >= nslabblk) {
    const int b = (int)blockIdx.x - nslabblk - (a.has_elbo ? 1 : 0);
    const long nq = a.n / 4;
    const long stride = (long)a.nreg * 256;
    // the workgroup's 256 quads of an iteration start at ib (uniform): the descriptor ranges they
    // can meet are found with scalar loads, each lane then tests only those (ascending q0)
    int j = 0;
    for (long ib = (long)b * 256; ib < nq; ib += stride) {
      while (j < a.nslab && a.q1[j] <= ib) ++j;
      j = __builtin_amdgcn_readfirstlane(j);
      const long i = ib + tid;
      if (i >= nq) break;
      bool own = true;
      for (int t = j; t < a.nslab && a.q0[t] < ib + 256; ++t) own = own && !(i >= a.q0[t] && i < a.q1[t]);
      if (own) adam_quad<LOWP>(a, k, i, reinterpret_cast<const f32x4*>(a.g)[i]);
    }
    if (b == 0 && tid < a.n - nq * 4) {
      const long i = nq * 4 + tid;
      adam_one<LOWP>(a, k, i, a.g[i]);
    }
    return;
  }
  // the descriptor of this workgroup
  const int sb = (int)blockIdx.x;
  int d = 0;
  while (d + 1 < a.nslab && sb >= a.blk0[d + 1]) ++d;
  d = __builtin_amdgcn_readfirstlane(d);
  const vae_grad_slab& s = a.s[d];
  const int lb = sb - a.blk0[d];
  const long count = s.count, ld = s.ld;
  const int rows = s.rows;
  const long base = a.off[d];
  if (a.tall[d]) {
    __shared__ float red[16][17];
    const int c = tid & 15, part = tid >> 4;
    const long col = (long)lb * 16 + c;
    // the element's optimizer state goes out first: its round trip overlaps the column sums
    const long e = (long)lb * 16 + tid;
    const bool upd = tid < 16 && e < ((count + 15) & ~15L);
    float pi = 0.f, mi = 0.f, vi = 0.f;
    if (upd) { pi = a.p[base + e]; mi = a.m[base + e]; vi = a.v[base + e]; }
    float acc = 0.f;
    if (col < count) {
      int r = part;
      for (; r + 16 * 7 < rows; r += 16 * 8) {
        float t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = s.slab[(long)(r + 16 * u) * ld + col];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += t[u];
      }
      for (; r < rows; r += 16) acc += s.slab[(long)r * ld + col];
    }
    red[part][c] = acc;
    __syncthreads();
    if (upd) {
      float t = 0.f;
#pragma unroll
      for (int q = 0; q < 16; ++q) t += red[q][tid];
      // (elements past count up to the 16-column boundary are not the descriptor's: their own
      // gradient)
      const float gv = e < count ? t : a.g[base + e];
      a.g[base + e] = gv;
      adam_elem(k, pi, gv, mi, vi);
      a.m[base + e] = mi; a.v[base + e] = vi; a.p[base + e] = pi;
      if (LOWP) a.lowp[base + e] = (__bf16)pi;
    }
    return;
  }
  // short: one quad per thread, rows in ascending order (the K slices of a grouped weight gradient:
  // 1-32 rows), the quad's optimizer state loaded first so both round trips overlap
  const long q = (long)lb * 256 + tid;
  const long e0 = q * 4;
  if (e0 >= count) return;
  const long gi = (base + e0) / 4;
  f32x4 p4 = reinterpret_cast<const f32x4*>(a.p)[gi];
  f32x4 m4 = reinterpret_cast<const f32x4*>(a.m)[gi];
  f32x4 v4 = reinterpret_cast<const f32x4*>(a.v)[gi];
  const bool vec = (((uintptr_t)s.slab) & 15) == 0 && (ld & 3) == 0;
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  if (vec && e0 + 4 <= count) {
    int r = 0;
    for (; r + 6 <= rows; r += 6) {
      f32x4 t[6];
#pragma unroll
      for (int u = 0; u < 6; ++u) t[u] = *reinterpret_cast<const f32x4*>(s.slab + (long)(r + u) * ld + e0);
#pragma unroll
      for (int u = 0; u < 6; ++u) acc += t[u];
    }
    for (; r < rows; ++r) acc += *reinterpret_cast<const f32x4*>(s.slab + (long)r * ld + e0);
  } else {
    for (int r = 0; r < rows; ++r)
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (e0 + u < count) acc[u] += s.slab[(long)r * ld + e0 + u];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (e0 + u >= count) acc[u] = a.g[base + e0 + u];     // (past the descriptor: its own gradient)
  }
  reinterpret_cast<f32x4*>(a.g)[gi] = acc;
  float pe[4], me[4], ve[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    pe[u] = p4[u]; me[u] = m4[u]; ve[u] = v4[u];
    adam_elem(k, pe[u], acc[u], me[u], ve[u]);
  }
  reinterpret_cast<f32x4*>(a.p)[gi] = f32x4{pe[0], pe[1], pe[2], pe[3]};
  reinterpret_cast<f32x4*>(a.m)[gi] = f32x4{me[0], me[1], me[2], me[3]};
  reinterpret_cast<f32x4*>(a.v)[gi] = f32x4{ve[0], ve[1], ve[2], ve[3]};
  if (LOWP) reinterpret_cast<bf16x4*>(a.lowp)[gi] = bf16x4{(__bf16)pe[0], (__bf16)pe[1], (__bf16)pe[2], (__bf16)pe[3]};
}

}  // namespace

extern "C" int vae_adam_step_ex(const vae_adam_args* a, void* stream) {
  if (!a) return fail(VAE_E_BADARG, "adam_step_ex: args");
  if (a->n <= 0) return VAE_OK;
  if (!a->p || !a->g || !a->m || !a->v || !a->step || !a->lr) return fail(VAE_E_BADARG, "adam_step_ex: null");
  auto al = [](const void* q, uintptr_t n) { return ((uintptr_t)q % n) == 0; };
  if (!al(a->p, 16) || !al(a->g, 16) || !al(a->m, 16) || !al(a->v, 16) || (a->p_lowp && !al(a->p_lowp, 8)))
    return fail(VAE_E_BADARG, "adam_step_ex: buffers must be 16-byte aligned (bf16 copy 8)");
  if (a->nslab < 0 || a->nslab > VAE_SLAB_MAX) return fail(VAE_E_BADARG, "adam_step_ex: %d slabs", a->nslab);
  if (a->has_elbo && (a->elbo.batch <= 0 || a->elbo.batch > 1024 || !a->elbo.out || !a->elbo.sse))
    return fail(VAE_E_BADSHAPE, "adam_step_ex: deferred loss");
  AdamEx k;
  memset(&k, 0, sizeof(k));
  k.n = a->n; k.p = a->p; k.g = a->g; k.m = a->m; k.v = a->v; k.step = a->step; k.lr = a->lr;
  k.b1 = a->beta1; k.b2 = a->beta2; k.eps = a->eps; k.wd = a->weight_decay;
  k.lowp = static_cast<__bf16*>(a->p_lowp);
  // descriptors sorted by their position in g; each must start on a quad and not overlap the next
  // (rows == 0: a gradient its call wrote whole — a plain gradient here)
  int order[VAE_SLAB_MAX], ns = 0;
  for (int i = 0; i < a->nslab; ++i)
    if (a->slab[i].rows != 0) order[ns++] = i;
  std::sort(order, order + ns, [&](int x, int y) { return a->slab[x].dst < a->slab[y].dst; });
  int blk = 0;
  for (int j = 0; j < ns; ++j) {
    const vae_grad_slab& s = a->slab[order[j]];
    const long off = (long)(s.dst - a->g);
    if (!s.dst || !s.slab || s.count <= 0 || s.rows <= 0 || s.ld < s.count || off < 0 || off + s.count > a->n || off % 4)
      return fail(VAE_E_BADARG, "adam_step_ex: slab %d (offset %ld, count %ld)", order[j], off, (long)s.count);
    k.s[j] = s;
    k.off[j] = off;
    k.tall[j] = s.rows >= kTallRows;
    const long span = k.tall[j] ? ((s.count + 15) & ~15L) : ((s.count + 3) & ~3L);
    if (off + span > a->n) return fail(VAE_E_BADARG, "adam_step_ex: slab %d runs past the buffer", order[j]);
    k.q0[j] = off / 4;
    k.q1[j] = (off + span + 3) / 4;
    if (j > 0 && k.q0[j] < k.q1[j - 1]) return fail(VAE_E_BADARG, "adam_step_ex: slabs %d and %d overlap", order[j - 1], order[j]);
    k.blk0[j] = blk;
    blk += (int)(k.tall[j] ? (s.count + 15) / 16 : (s.count + 1023) / 1024);
  }
  k.nslab = ns;
  k.blk0[ns] = blk;
  k.nreg = grid_for((a->n + 3) / 4);
  k.has_elbo = a->has_elbo;
  if (a->has_elbo) k.e = a->elbo;
  const dim3 grid((unsigned)(k.nreg + blk + (a->has_elbo ? 1 : 0)));
  const hipStream_t st = (hipStream_t)stream;
  if (a->p_lowp) VAE_LAUNCH(adam_ex_kernel<true>, grid, dim3(256), 0, st, k);
  else VAE_LAUNCH(adam_ex_kernel<false>, grid, dim3(256), 0, st, k);
  return check_launch("adam_step_ex");
}

extern "C" int vae_cast_bf16(int64_t n, const float* src, void* dst, void* stream) {
  if (n <= 0) return VAE_OK;
  if (!src || !dst) return fail(VAE_E_BADARG, "cast_bf16: null");
  VAE_LAUNCH(cast_bf16_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, (long)n, src, (__bf16*)dst);
  return check_launch("cast_bf16");
}

// ------------------------------------------------------------------ training-step record
namespace {
__global__ void __launch_bounds__(256) step_record_kernel(const vae_record_args a) {
  kernarg_prefetch<(sizeof(vae_record_args) < 1024 ? sizeof(vae_record_args) : 1024)>();
  __shared__ float pv[1024];
  __shared__ float rv[2][256];
  __shared__ int ri[2][256];
  __shared__ int win[2];
  const int tid = threadIdx.x;
  if (tid < a.nterms) a.terms[tid] = a.src_terms[tid];
  const float inv_s = 1.0f / (float)a.samples;
  for (int b = tid; b < a.batch; b += 256) {
    float v = 0.f;
    for (int s = 0; s < a.samples; ++s) v += a.per_img[b * a.samples + s];
    v *= inv_s;
    pv[b] = v;
    a.per[b] = v;
  }
  __syncthreads();
  // first index of the maximum / minimum (ties -> lowest index, as the reference's strict '>'/'<')
  float mx = -INFINITY, mn = INFINITY;
  int imx = 0x7fffffff, imn = 0x7fffffff;
  for (int b = tid; b < a.batch; b += 256) {
    const float v = pv[b];
    if (v > mx) { mx = v; imx = b; }
    if (v < mn) { mn = v; imn = b; }
  }
  rv[0][tid] = mx; ri[0][tid] = imx; rv[1][tid] = mn; ri[1][tid] = imn;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (tid < off) {
      const float v1 = rv[0][tid + off], v0 = rv[0][tid];
      const int i1 = ri[0][tid + off], i0 = ri[0][tid];
      if (v1 > v0 || (v1 == v0 && i1 < i0)) { rv[0][tid] = v1; ri[0][tid] = i1; }
      const float w1 = rv[1][tid + off], w0 = rv[1][tid];
      const int j1 = ri[1][tid + off], j0 = ri[1][tid];
      if (w1 < w0 || (w1 == w0 && j1 < j0)) { rv[1][tid] = w1; ri[1][tid] = j1; }
    }
    __syncthreads();
  }
  if (tid == 0) {
    win[0] = rv[0][0] > a.best[0] ? ri[0][0] : -1;
    win[1] = rv[1][0] < a.best[1] ? ri[1][0] : -1;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int b = win[k];
    if (b < 0) continue;
    float* di = k == 0 ? a.hi_img : a.lo_img;
    float* dr = k == 0 ? a.hi_recon : a.lo_recon;
    for (int e = tid; e < a.img_elems; e += 256) {
      di[e] = a.img[(long)b * a.img_elems + e];
      dr[e] = a.recon[(long)b * a.samples * a.img_elems + e];
    }
    if (tid == 0) { a.best[k] = rv[k][0]; a.at[2 * k] = a.step; a.at[2 * k + 1] = b; }
  }
}
}  // namespace

extern "C" int vae_step_record(const vae_record_args* a, void* stream) {
  if (!a || a->batch <= 0 || a->batch > 1024 || a->samples <= 0 || a->img_elems <= 0 || a->nterms < 0 || a->nterms > 8 ||
      (a->nterms && (!a->src_terms || !a->terms)) || !a->per_img || !a->per || !a->img || !a->recon || !a->best || !a->at ||
      !a->hi_img || !a->hi_recon || !a->lo_img || !a->lo_recon)
    return fail(VAE_E_BADARG, "step_record: args");
  VAE_LAUNCH(step_record_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, *a);
  return check_launch("step_record");
}

extern "C" int vae_step_begin(void* zero, int64_t bytes, int32_t* step, void* stream) {
  if (bytes < 0 || (bytes > 0 && !zero)) return fail(VAE_E_BADARG, "step_begin: args");
  if (((uintptr_t)zero & 15) != 0) return fail(VAE_E_BADARG, "step_begin: zero region must be 16-B aligned");
  const long n16 = bytes / 16;
  const int ntail = (int)(bytes - n16 * 16);
  VAE_LAUNCH(step_begin_kernel, dim3(grid_for(n16 > 0 ? n16 : 1)), dim3(256), 0, (hipStream_t)stream,
                     (f32x4*)zero, n16, (unsigned char*)zero + n16 * 16, ntail, (int*)step);
  return check_launch("step_begin");
}

// ------------------------------------------------------------------ swapped-axes weight copies
// dst[b][t][a] = bf16(src[a][t][b]) for up to VAE_SWAP_MAX tensors in one launch: the k-contiguous
// B operands of the bf16 ConvTranspose2d forward / Conv2d data-gradient GEMMs (vaehip.h wt_t),
// refreshed from the fp32 master right after the optimizer step.  One workgroup = one 32x32
// (a, b) tile of one tap through a padded LDS tile (both sides 64-byte segments).
namespace {
struct SwapBatch {
  vae_swap_desc d[VAE_SWAP_MAX];
  int tiles0[VAE_SWAP_MAX + 1];      // first workgroup of each descriptor
  int count;
};

__global__ void __launch_bounds__(256) swap_axes_kernel(const SwapBatch sb) {
  kernarg_prefetch<(sizeof(SwapBatch) < 1024 ? sizeof(SwapBatch) : 1024)>();
  __shared__ float t[kSwapT][kSwapT + 1];
  int i = 0;
  while (i + 1 < sb.count && (int)blockIdx.x >= sb.tiles0[i + 1]) ++i;
  swap_tile(sb.d[i], blockIdx.x - sb.tiles0[i], t);
}
}  // namespace

extern "C" int vae_swap_axes(int32_t count, const vae_swap_desc* descs, void* stream) {
  if (count <= 0) return VAE_OK;
  if (count > VAE_SWAP_MAX || !descs) return fail(VAE_E_BADARG, "swap_axes: count %d (max %d)", count, VAE_SWAP_MAX);
  SwapBatch sb;
  memset(&sb, 0, sizeof(sb));
  int tiles = 0;
  for (int i = 0; i < count; ++i) {
    const vae_swap_desc& d = descs[i];
    if (!d.src || !d.dst || d.a <= 0 || d.b <= 0 || d.rs <= 0 || (d.src_dtype != VAE_F32 && d.src_dtype != VAE_BF16))
      return fail(VAE_E_BADARG, "swap_axes: descriptor %d", i);
    sb.d[i] = d;
    sb.tiles0[i] = tiles;
    tiles += swap_tiles(d);
  }
  sb.tiles0[count] = tiles;
  sb.count = count;
  VAE_LAUNCH(swap_axes_kernel, dim3(tiles), dim3(256), 0, (hipStream_t)stream, sb);
  return check_launch("swap_axes");
}

// ---------------------------------------------------------------- workspace queries
// The entry point runs on a copy of the arguments with an unbounded (never dereferenced)
// workspace while the thread's query flag is set: its planning is the real one, every workspace
// site records its bytes (vae_common.hpp ws_fits) and nothing is launched, so the query needs no
// device and no stream.
namespace {
template <class A, class F>
int ws_size(const A* a, size_t* bytes, F&& call) {
  if (!a || !bytes) return fail(VAE_E_BADARG, "workspace_size: null argument");
  A c = *a;
  c.workspace = reinterpret_cast<void*>(uintptr_t(1) << 40);
  c.workspace_bytes = int64_t(1) << 50;
  WsQuery& q = ws_query();
  q.on = 1;
  q.need = 0;
  const int rc = call(&c);
  *bytes = rc ? 0 : (size_t)q.need;
  q.on = 0;
  q.need = 0;
  return rc;
}
}  // namespace

extern "C" int vae_conv2d_workspace_size(const vae_conv_args* a, int32_t op, size_t* bytes) {
  switch (op) {
    case VAE_OP_FWD: return ws_size(a, bytes, [](const vae_conv_args* c) { return vae_conv2d_fwd(c, nullptr); });
    case VAE_OP_BWD_DATA: return ws_size(a, bytes, [](const vae_conv_args* c) { return vae_conv2d_bwd_data(c, nullptr); });
    case VAE_OP_BWD_FILTER: return ws_size(a, bytes, [](const vae_conv_args* c) { return vae_conv2d_bwd_filter(c, nullptr); });
  }
  return fail(VAE_E_BADARG, "conv2d_workspace_size: op %d", op);
}

extern "C" int vae_convT2d_workspace_size(const vae_conv_args* a, int32_t op, size_t* bytes) {
  switch (op) {
    case VAE_OP_FWD: return ws_size(a, bytes, [](const vae_conv_args* c) { return vae_convT2d_fwd(c, nullptr); });
    case VAE_OP_BWD_DATA: return ws_size(a, bytes, [](const vae_conv_args* c) { return vae_convT2d_bwd_data(c, nullptr); });
    case VAE_OP_BWD_FILTER: return ws_size(a, bytes, [](const vae_conv_args* c) { return vae_convT2d_bwd_filter(c, nullptr); });
    case VAE_OP_BWD: return ws_size(a, bytes, [](const vae_conv_args* c) { return vae_convT2d_bwd(c, nullptr); });
  }
  return fail(VAE_E_BADARG, "convT2d_workspace_size: op %d", op);
}

extern "C" int vae_linear_workspace_size(const vae_linear_args* a, int32_t op, size_t* bytes) {
  switch (op) {
    case VAE_OP_FWD: return ws_size(a, bytes, [](const vae_linear_args* c) { return vae_linear_fwd(c, nullptr); });
    case VAE_OP_BWD_DATA: return ws_size(a, bytes, [](const vae_linear_args* c) { return vae_linear_bwd_data(c, nullptr); });
    case VAE_OP_BWD_FILTER: return ws_size(a, bytes, [](const vae_linear_args* c) { return vae_linear_bwd_filter(c, nullptr); });
  }
  return fail(VAE_E_BADARG, "linear_workspace_size: op %d", op);
}

extern "C" int vae_head_workspace_size(const vae_head_args* a, int32_t op, size_t* bytes) {
  switch (op) {
    case VAE_OP_FWD: return ws_size(a, bytes, [](const vae_head_args* c) { return vae_head_fwd(c, nullptr); });
    case VAE_OP_BWD_DATA: return ws_size(a, bytes, [](const vae_head_args* c) { return vae_head_bwd_data(c, nullptr); });
    case VAE_OP_BWD_FILTER: return ws_size(a, bytes, [](const vae_head_args* c) { return vae_head_bwd_filter(c, nullptr); });
    case VAE_OP_BWD: return ws_size(a, bytes, [](const vae_head_args* c) { return vae_head_bwd(c, nullptr); });
  }
  return fail(VAE_E_BADARG, "head_workspace_size: op %d", op);
}
