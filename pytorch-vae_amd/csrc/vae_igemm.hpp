// Generic implicit-GEMM kernel on MFMA for every convolution-family op of the VAE step.
//
//   C[m][n] = Σ_k A(m,k) · B(n,k)
//
// A and B are "operands": views of NHWC tensors / weight matrices with a per-channel
// transform (BatchNorm+LeakyReLU forward, or BatchNorm backward) applied on load.  Tiles are
// staged global -> registers -> LDS as [rows][BK] (k contiguous, padded), and read as MFMA
// fragments: lane l owns row (l&15) and the 8 consecutive k of group (l>>4).  fp32 runs
// v_mfma_f32_16x16x4_f32 eight times over those 8 k (k permuted inside the tile — the sum is
// order-free); bf16 runs one v_mfma_f32_16x16x32_bf16.  The next tile's global loads are
// issued before the MFMAs of the current one (register prefetch).
//
// Operand modes (vector direction V_K = 8 contiguous k per load, V_M = 4 contiguous rows):
//   A_CONV   im2col gather of a strided conv (NHWC dtype, or the NCHW fp32 image)    V_K
//   A_CONVT  sub-pixel phase gather of a transposed conv / conv dgrad (blockIdx.z)  V_K
//   A_DENSE  row-major [M][K]                                                      V_K
//   A_KM     k-major [K][M] (weight-gradient GEMMs reduce over pixels/batch)      V_M
//   B_NK     weights [N][K]                                                        V_K
//   B_KN     weights [K'][N] addressed through the phase tap tables (or dense)     V_M
//   B_GATHER conv gather with n = (r,s,c), k = pixel (weight gradient)             V_M
// Epilogues: E_STORE (bias, residual, per-channel Σ/Σ² for the next BatchNorm),
//            E_BNBWD (g = da·act'(z) of the producing layer, Σg -> dβ, Σg·x̂ -> dγ),
//            E_ACC   (split-K fp32 atomic accumulation of weight gradients),
//            E_REPARAM (dz -> d[mu|logvar] incl. the analytic KL gradient).
#pragma once
#include "vae_common.hpp"

namespace vae {

enum AMode { A_CONV = 0, A_CONVT = 1, A_DENSE = 2, A_KM = 3 };
enum BMode { B_NK = 0, B_KN = 1, B_GATHER = 2 };
enum EMode { E_STORE = 0, E_BNBWD = 1, E_ACC = 2, E_REPARAM = 3 };

constexpr int MAXC = 512;   // max channels of a per-channel transform table
constexpr int BK = 32;
constexpr int NTHREADS = 256;

struct GemmParams {
  int M, N, K;               // K of phase 0 for A_CONVT (per-phase K from the tap tables)
  int ksplit, nphase;
  // ---- A operand
  const void* a_ptr; int a_ld; vae_xform a_xf;
  // ---- B operand
  const void* b_ptr; int b_ld; vae_xform b_xf;
  int ones_col;              // B_KN/B_GATHER: column index that reads 1.0 (bias grad) or -1
  int b_taps;                // B_KN: rows addressed through the phase tap tables (else dense)
  int g_nchw;                // A_CONV / B_GATHER: gathered tensor is the fp32 NCHW image
  // ---- conv geometry of the gathered tensor
  //   A_CONV/B_GATHER: tensor [gn][gh][gw][gc], output grid gp x gq, kernel gr, stride gs, pad gpad
  //   A_CONVT: input tensor [gn][gh][gw][gc] -> output gho x gwo, phase grid gp x gq
  int gn, gh, gw, gc, gp, gq, gr, gs, gpad, gho, gwo;
  int ntap_h[2], ntap_w[2], tap_h[2][4], tap_w[2][4];
  // ---- epilogue
  void* out; int out_ld; int out_phase;      // out_phase: rows are phase-grid pixels
  int out_f32;               // E_STORE: write fp32 instead of T
  const float* bias; float* sum; float* sumsq;
  const void* residual; vae_xform res_xf;
  vae_xform epi_xf; float* dgamma; float* dbeta;
  float* bias_grad;
  const float* mulv; const float* eps; const float* kl_coef; float* dmulv; int samples, latent;
};

// ------------------------------------------------------------------ per-element transform
template <class TIn, int MAXCT>
__device__ __forceinline__ float xf_apply(const vae_xform& x, const XfTable<MAXCT, false>& t, float v,
                                          int ch, const TIn* aux, long idx) {
  switch (x.kind) {
    case VAE_X_ACT: return lrelu(v, x.slope);
    case VAE_X_BN_ACT: return lrelu(fmaf(v, t.a[ch], t.b[ch]), x.slope);
    case VAE_X_BN_DY: return fmaf(t.a[ch], v, fmaf(t.b[ch], ld_f(aux + idx), t.c[ch]));
    default: return v;
  }
}

// --------------------------------------------------------------------- operand loading
// Each thread loads "octets" of 8 elements: V_K = one row × 8 k, V_M = 4 rows × 2 k.
template <class T, class TIn, int AM, int MAXCT>
struct AOperand {
  // V_K: rows [row], k0..k0+7
  __device__ __forceinline__ static void load_vk(const GemmParams& p, const XfTable<MAXCT, false>& xt, int phase,
                                 int row, int k0, int Kp, float (&v)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.f;
    if (row >= p.M || k0 >= Kp) return;
    const TIn* X = static_cast<const TIn*>(p.a_ptr);
    const TIn* aux = static_cast<const TIn*>(p.a_xf.aux);
    if constexpr (AM == A_DENSE) {
      const long base = (long)row * p.a_ld + k0;
      if (k0 + 8 <= Kp && (p.a_ld & 7) == 0) {
        ld8(X + base, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = xf_apply<TIn, MAXCT>(p.a_xf, xt, v[j], (k0 + j) % p.a_xf.channels, aux, base + j);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (k0 + j < Kp) v[j] = xf_apply<TIn, MAXCT>(p.a_xf, xt, ld_f(X + base + j), (k0 + j) % p.a_xf.channels, aux, base + j);
      }
    } else if constexpr (AM == A_CONV) {
      // row -> (n, op, oq) of the output grid
      const int oq = row % p.gq;
      const int t = row / p.gq;
      const int op = t % p.gp;
      const int n = t / p.gp;
      const int hb = op * p.gs - p.gpad, wb = oq * p.gs - p.gpad;
      const int C = p.gc;
      if (!p.g_nchw && (C & 7) == 0) {
        const int tap = k0 / C, c = k0 - tap * C;
        const int r = tap / p.gr, s = tap - r * p.gr;
        const int hi = hb + r, wi = wb + s;
        if (hi < 0 || hi >= p.gh || wi < 0 || wi >= p.gw) return;
        const long base = (((long)n * p.gh + hi) * p.gw + wi) * C + c;
        ld8(X + base, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = xf_apply<TIn, MAXCT>(p.a_xf, xt, v[j], c + j, aux, base + j);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = k0 + j;
          const int tap = k / C, c = k - tap * C;
          const int r = tap / p.gr, s = tap - r * p.gr;
          const int hi = hb + r, wi = wb + s;
          if (k >= Kp || hi < 0 || hi >= p.gh || wi < 0 || wi >= p.gw) continue;
          const long idx = p.g_nchw ? (((long)n * C + c) * p.gh + hi) * p.gw + wi
                                    : (((long)n * p.gh + hi) * p.gw + wi) * C + c;
          v[j] = xf_apply<TIn, MAXCT>(p.a_xf, xt, ld_f(X + idx), c, aux, idx);
        }
      }
    } else if constexpr (AM == A_CONVT) {
      const int ph = phase / p.gs, pw = phase - (phase / p.gs) * p.gs;
      const int ww = row % p.gq;
      const int t = row / p.gq;
      const int hh = t % p.gp;
      const int n = t / p.gp;
      const int ho = hh * p.gs + ph, wo = ww * p.gs + pw;
      const int C = p.gc;
      const int ntw = p.ntap_w[pw];
      if ((C & 7) == 0) {
        const int c = k0 % C, tt = k0 / C;
        const int tw = tt % ntw, th = tt / ntw;
        const int r = p.tap_h[ph][th], s = p.tap_w[pw][tw];
        const int hi = (ho + p.gpad - r) / p.gs, wi = (wo + p.gpad - s) / p.gs;
        if (hi < 0 || hi >= p.gh || wi < 0 || wi >= p.gw) return;
        const long base = (((long)n * p.gh + hi) * p.gw + wi) * C + c;
        ld8(X + base, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = xf_apply<TIn, MAXCT>(p.a_xf, xt, v[j], c + j, aux, base + j);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = k0 + j;
          if (k >= Kp) continue;
          const int c = k % C, tt = k / C;
          const int tw = tt % ntw, th = tt / ntw;
          const int r = p.tap_h[ph][th], s = p.tap_w[pw][tw];
          const int hi = (ho + p.gpad - r) / p.gs, wi = (wo + p.gpad - s) / p.gs;
          if (hi < 0 || hi >= p.gh || wi < 0 || wi >= p.gw) continue;
          const long idx = (((long)n * p.gh + hi) * p.gw + wi) * C + c;
          v[j] = xf_apply<TIn, MAXCT>(p.a_xf, xt, ld_f(X + idx), c, aux, idx);
        }
      }
    }
  }
  // V_M: rows row0..row0+3 at k (A_KM: element (m,k) at k*lda + m)
  __device__ __forceinline__ static void load_vm(const GemmParams& p, const XfTable<MAXCT, false>& xt, int row0, int k, float (&v)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = 0.f;
    if constexpr (AM == A_KM) {
      if (k >= p.K || row0 >= p.M) return;
      const TIn* X = static_cast<const TIn*>(p.a_ptr);
      const TIn* aux = static_cast<const TIn*>(p.a_xf.aux);
      const long base = (long)k * p.a_ld + row0;
      if (row0 + 4 <= p.M && (p.a_ld & 3) == 0) {
        ld4(X + base, v);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = xf_apply<TIn, MAXCT>(p.a_xf, xt, v[j], (row0 + j) % p.a_xf.channels, aux, base + j);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (row0 + j < p.M) v[j] = xf_apply<TIn, MAXCT>(p.a_xf, xt, ld_f(X + base + j), (row0 + j) % p.a_xf.channels, aux, base + j);
      }
    }
  }
};

template <class T, class TIn, int BMD, int MAXCT>
struct BOperand {
  __device__ __forceinline__ static void load_vk(const GemmParams& p, int phase, int row, int k0, int Kp, float (&v)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.f;
    if constexpr (BMD == B_NK) {
      if (row >= p.N || k0 >= Kp) return;
      const TIn* W = static_cast<const TIn*>(p.b_ptr);
      const long base = (long)row * p.b_ld + k0;
      if (k0 + 8 <= Kp && (p.b_ld & 7) == 0) {
        ld8(W + base, v);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (k0 + j < Kp) v[j] = ld_f(W + base + j);
      }
    }
  }
  // V_M: 4 consecutive n at one k
  __device__ __forceinline__ static void load_vm(const GemmParams& p, const XfTable<MAXCT, false>& xt, int phase, int n0, int k,
                                 int Kp, float (&v)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = 0.f;
    if (k >= Kp || n0 >= p.N) return;
    if constexpr (BMD == B_KN) {
      // row of the [K'][N] matrix: dense (nphase==0 tables unused) or via phase taps
      long kr;
      if (p.b_taps) {
        const int ph = phase / p.gs, pw = phase - (phase / p.gs) * p.gs;
        const int C = p.gc, ntw = p.ntap_w[pw];
        const int c = k % C, tt = k / C;
        const int tw = tt % ntw, th = tt / ntw;
        const int r = p.tap_h[ph][th], s = p.tap_w[pw][tw];
        kr = ((long)c * p.gr + r) * p.gr + s;
      } else {
        kr = k;
      }
      const TIn* W = static_cast<const TIn*>(p.b_ptr);
      const TIn* aux = static_cast<const TIn*>(p.b_xf.aux);
      const long base = kr * p.b_ld + n0;
      if (n0 + 4 <= p.N && (p.b_ld & 3) == 0 && (p.ones_col < 0 || n0 + 4 <= p.ones_col)) {
        ld4(W + base, v);
        if (p.b_xf.kind != VAE_X_NONE) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = xf_apply<TIn, MAXCT>(p.b_xf, xt, v[j], (n0 + j) % p.b_xf.channels, aux, base + j);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = n0 + j;
          if (n >= p.N) continue;
          if (n == p.ones_col) { v[j] = 1.f; continue; }
          v[j] = xf_apply<TIn, MAXCT>(p.b_xf, xt, ld_f(W + base + j), n % p.b_xf.channels, aux, base + j);
        }
      }
    } else if constexpr (BMD == B_GATHER) {
      // k = pixel (n_img, op, oq) of the gp x gq grid; n = (r, s, c) of the gathered tensor
      const int oq = k % p.gq;
      const int t = k / p.gq;
      const int op = t % p.gp;
      const int nimg = t / p.gp;
      const TIn* X = static_cast<const TIn*>(p.b_ptr);
      const TIn* aux = static_cast<const TIn*>(p.b_xf.aux);
      const int C = p.gc;
      if (!p.g_nchw && (C & 3) == 0 && (p.ones_col < 0 || n0 + 4 <= p.ones_col) && n0 + 4 <= p.N) {
        const int tap = n0 / C, c = n0 - tap * C;
        const int r = tap / p.gr, s = tap - r * p.gr;
        const int hi = op * p.gs - p.gpad + r, wi = oq * p.gs - p.gpad + s;
        if (hi < 0 || hi >= p.gh || wi < 0 || wi >= p.gw) return;
        const long base = (((long)nimg * p.gh + hi) * p.gw + wi) * C + c;
        ld4(X + base, v);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = xf_apply<TIn, MAXCT>(p.b_xf, xt, v[j], c + j, aux, base + j);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = n0 + j;
          if (n >= p.N) continue;
          if (n == p.ones_col) { v[j] = 1.f; continue; }
          const int tap = n / C, c = n - tap * C;
          const int r = tap / p.gr, s = tap - r * p.gr;
          const int hi = op * p.gs - p.gpad + r, wi = oq * p.gs - p.gpad + s;
          if (hi < 0 || hi >= p.gh || wi < 0 || wi >= p.gw) continue;
          // B_GATHER's tensor may be the fp32 NCHW image (first-layer weight gradient)
          const long idx = p.g_nchw ? (((long)nimg * C + c) * p.gh + hi) * p.gw + wi
                                    : (((long)nimg * p.gh + hi) * p.gw + wi) * C + c;
          v[j] = xf_apply<TIn, MAXCT>(p.b_xf, xt, ld_f(X + idx), c, aux, idx);
        }
      }
    }
  }
};

template <int AM> constexpr bool a_is_vm() { return AM == A_KM; }
template <int BMD> constexpr bool b_is_vm() { return BMD != B_NK; }

// ------------------------------------------------------------------------------ kernel
// T: LDS/MFMA type; TA: storage type of the A tensor (fp32 for the NCHW image);
// TB: storage type of B (the gathered activation for B_GATHER, weights otherwise).
template <class T, class TA, class TB, int BM, int BN, int AM, int BMD, int EM>
__global__ void __launch_bounds__(NTHREADS) igemm_kernel(const GemmParams p) {
  constexpr int LDK = BK + (sizeof(T) == 4 ? 4 : 8);        // padded LDS row (elements)
  constexpr int WTM = BM / 2, WTN = BN / 2;                 // 2x2 waves
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr bool A_VM = a_is_vm<AM>();
  constexpr bool B_VM = b_is_vm<BMD>();
  constexpr int A_OCT = BM * BK / 8, B_OCT = BN * BK / 8;   // octets per tile
  constexpr int A_PER = (A_OCT + NTHREADS - 1) / NTHREADS, B_PER = (B_OCT + NTHREADS - 1) / NTHREADS;
  constexpr bool B_XF = (BMD != B_NK);
  constexpr bool EPI_TBL = (EM == E_BNBWD);

  __shared__ __attribute__((aligned(16))) T As[BM * LDK];
  __shared__ __attribute__((aligned(16))) T Bs[BN * LDK];
  __shared__ XfTable<MAXC, false> xa;
  __shared__ XfTable<B_XF ? MAXC : 1, false> xb;
  __shared__ XfTable<EPI_TBL ? MAXC : 1, true> xe;
  __shared__ float red1[BN], red2[BN];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int phase = (p.nphase > 1) ? (int)(blockIdx.z / p.ksplit) : 0;
  const int ks = blockIdx.z - phase * p.ksplit;
  const bool first_block = blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0;

  // per-phase K
  int Kp = p.K;
  if constexpr (AM == A_CONVT) {
    const int ph = phase / p.gs, pw = phase - ph * p.gs;
    Kp = p.ntap_h[ph] * p.ntap_w[pw] * p.gc;
  }
  const int ktiles = (Kp + BK - 1) / BK;
  const int kper = (ktiles + p.ksplit - 1) / p.ksplit;
  const int kt0 = ks * kper;
  const int kt1 = min(ktiles, kt0 + kper);

  // per-channel tables (BN coefficients) and the reduction scratch
  xa.fill(p.a_xf, first_block);
  if constexpr (B_XF) xb.fill(p.b_xf, false);
  if constexpr (EPI_TBL) xe.fill(p.epi_xf, false);
  for (int i = tid; i < BN; i += NTHREADS) { red1[i] = 0.f; red2[i] = 0.f; }

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  float ra[A_PER][8], rb[B_PER][8];

  auto load_tiles = [&](int kt) {
    const int kb = kt * BK;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int o = tid + i * NTHREADS;
      if (o < A_OCT) {
        if constexpr (!A_VM) {
          AOperand<T, TA, AM, MAXC>::load_vk(p, xa, phase, m0 + o / (BK / 8), kb + (o % (BK / 8)) * 8, Kp, ra[i]);
        } else {
          const int rq = o % (BM / 4), kp = o / (BM / 4);
          float v0[4], v1[4];
          AOperand<T, TA, AM, MAXC>::load_vm(p, xa, m0 + rq * 4, kb + 2 * kp, v0);
          AOperand<T, TA, AM, MAXC>::load_vm(p, xa, m0 + rq * 4, kb + 2 * kp + 1, v1);
#pragma unroll
          for (int j = 0; j < 4; ++j) { ra[i][2 * j] = v0[j]; ra[i][2 * j + 1] = v1[j]; }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int o = tid + i * NTHREADS;
      if (o < B_OCT) {
        if constexpr (!B_VM) {
          BOperand<T, TB, BMD, MAXC>::load_vk(p, phase, n0 + o / (BK / 8), kb + (o % (BK / 8)) * 8, Kp, rb[i]);
        } else {
          const int rq = o % (BN / 4), kp = o / (BN / 4);
          float v0[4], v1[4];
          BOperand<T, TB, BMD, (B_XF ? MAXC : 1)>::load_vm(p, xb, phase, n0 + rq * 4, kb + 2 * kp, Kp, v0);
          BOperand<T, TB, BMD, (B_XF ? MAXC : 1)>::load_vm(p, xb, phase, n0 + rq * 4, kb + 2 * kp + 1, Kp, v1);
#pragma unroll
          for (int j = 0; j < 4; ++j) { rb[i][2 * j] = v0[j]; rb[i][2 * j + 1] = v1[j]; }
        }
      }
    }
  };
  auto store_tiles = [&]() {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int o = tid + i * NTHREADS;
      if (o < A_OCT) {
        if constexpr (!A_VM) {
          st8(As + (o / (BK / 8)) * LDK + (o % (BK / 8)) * 8, ra[i]);
        } else {
          const int rq = o % (BM / 4), kp = o / (BM / 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            st2(As + (rq * 4 + j) * LDK + 2 * kp, ra[i][2 * j], ra[i][2 * j + 1]);
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int o = tid + i * NTHREADS;
      if (o < B_OCT) {
        if constexpr (!B_VM) {
          st8(Bs + (o / (BK / 8)) * LDK + (o % (BK / 8)) * 8, rb[i]);
        } else {
          const int rq = o % (BN / 4), kp = o / (BN / 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            st2(Bs + (rq * 4 + j) * LDK + 2 * kp, rb[i][2 * j], rb[i][2 * j + 1]);
          }
        }
      }
    }
  };

  __syncthreads();   // tables ready
  if (kt0 < kt1) load_tiles(kt0);
  for (int kt = kt0; kt < kt1; ++kt) {
    __syncthreads();
    store_tiles();
    __syncthreads();
    if (kt + 1 < kt1) load_tiles(kt + 1);
    const int koff = 8 * (lane >> 4);
    if constexpr (sizeof(T) == 4) {
      float af[TM][8], bfr[TN][8];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const float* src = reinterpret_cast<const float*>(As) + (wm * WTM + i * 16 + (lane & 15)) * LDK + koff;
        f32x4 x0 = *reinterpret_cast<const f32x4*>(src), x1 = *reinterpret_cast<const f32x4*>(src + 4);
        af[i][0] = x0[0]; af[i][1] = x0[1]; af[i][2] = x0[2]; af[i][3] = x0[3];
        af[i][4] = x1[0]; af[i][5] = x1[1]; af[i][6] = x1[2]; af[i][7] = x1[3];
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const float* src = reinterpret_cast<const float*>(Bs) + (wn * WTN + j * 16 + (lane & 15)) * LDK + koff;
        f32x4 x0 = *reinterpret_cast<const f32x4*>(src), x1 = *reinterpret_cast<const f32x4*>(src + 4);
        bfr[j][0] = x0[0]; bfr[j][1] = x0[1]; bfr[j][2] = x0[2]; bfr[j][3] = x0[3];
        bfr[j][4] = x1[0]; bfr[j][5] = x1[1]; bfr[j][6] = x1[2]; bfr[j][7] = x1[3];
      }
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][s], bfr[j][s], acc[i][j], 0, 0, 0);
    } else {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(As + (wm * WTM + i * 16 + (lane & 15)) * LDK + koff);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + (wn * WTN + j * 16 + (lane & 15)) * LDK + koff);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }

  // ------------------------------------------------------------------------ epilogue
  // lane holds rows 4*(lane>>4)+e, column lane&15 of each 16x16 tile
  const int ph = phase / (p.gs > 0 ? p.gs : 1), pw = phase - ph * (p.gs > 0 ? p.gs : 1);
  auto out_index = [&](int row, int col) -> long {
    if (p.out_phase) {
      const int ww = row % p.gq;
      const int t = row / p.gq;
      const int hh = t % p.gp;
      const int n = t / p.gp;
      const int ho = hh * p.gs + ph, wo = ww * p.gs + pw;
      return (((long)n * p.gho + ho) * p.gwo + wo) * p.out_ld + col;
    }
    return (long)row * p.out_ld + col;
  };

  if constexpr (EM == E_ACC) {
    float* out = static_cast<float*>(p.out);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + wn * WTN + j * 16 + (lane & 15);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = m0 + wm * WTM + i * 16 + 4 * (lane >> 4) + e;
          if (row >= p.M || col >= p.N) continue;
          if (col == p.ones_col) {
            if (p.bias_grad) atomicAdd(p.bias_grad + row, acc[i][j][e]);
          } else {
            atomicAdd(out + (long)row * p.out_ld + col, acc[i][j][e]);
          }
        }
      }
    return;
  } else if constexpr (EM == E_REPARAM) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int d = n0 + wn * WTN + j * 16 + (lane & 15);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = m0 + wm * WTM + i * 16 + 4 * (lane >> 4) + e;
          if (row >= p.M || d >= p.N) continue;
          const int b = row / p.samples;
          const float mu = p.mulv[(long)b * 2 * p.latent + d];
          const float lv = p.mulv[(long)b * 2 * p.latent + p.latent + d];
          const float ep = p.eps[(long)row * p.latent + d];
          const float c = p.kl_coef ? p.kl_coef[row] : 0.f;
          const float dz = acc[i][j][e];
          const float sd = expf(0.5f * lv);
          atomicAdd(p.dmulv + (long)b * 2 * p.latent + d, dz + c * mu);
          atomicAdd(p.dmulv + (long)b * 2 * p.latent + p.latent + d, dz * ep * 0.5f * sd + c * 0.5f * (expf(lv) - 1.f));
        }
      }
    return;
  } else {
    T* out = static_cast<T*>(p.out);
    const bool want_sums = (EM == E_STORE) ? (p.sum != nullptr) : (p.epi_xf.kind == VAE_X_BN_ACT);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wn * WTN + j * 16 + (lane & 15);
      const bool col_ok = col < p.N;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = m0 + wm * WTM + i * 16 + 4 * (lane >> 4) + e;
          if (row >= p.M || !col_ok) continue;
          const float v = acc[i][j][e];
          const long idx = out_index(row, col);
          if constexpr (EM == E_STORE) {
            float y = v + (p.bias ? p.bias[col] : 0.f);
            if (p.residual) {
              const T* res = static_cast<const T*>(p.residual);
              float rv = ld_f(res + idx);
              if (p.res_xf.kind == VAE_X_ACT) rv = lrelu(rv, p.res_xf.slope);
              y += rv;
            }
            if (p.out_f32) static_cast<float*>(p.out)[idx] = y;
            else out[idx] = cvt<T>(y);
            s1 += v;
            s2 += v * v;
          } else {  // E_BNBWD
            float g = v;
            if (p.epi_xf.kind == VAE_X_BN_ACT) {
              const int ch = col % p.epi_xf.channels;
              const float yv = ld_f(static_cast<const T*>(p.epi_xf.aux) + idx);
              const float z = fmaf(yv, xe.a[ch], xe.b[ch]);
              g = z > 0.f ? v : v * p.epi_xf.slope;
              const float xh = fmaf(yv, xe.p[ch], xe.q[ch]);
              s1 += g;
              s2 += g * xh;
            } else if (p.epi_xf.kind == VAE_X_ACT) {
              const float yv = ld_f(static_cast<const T*>(p.epi_xf.aux) + idx);
              g = yv > 0.f ? v : v * p.epi_xf.slope;
            }
            out[idx] = cvt<T>(g);
          }
        }
      if (want_sums) {
        s1 += __shfl_xor(s1, 16);
        s1 += __shfl_xor(s1, 32);
        s2 += __shfl_xor(s2, 16);
        s2 += __shfl_xor(s2, 32);
        if (lane < 16 && col_ok) {
          atomicAdd(&red1[wn * WTN + j * 16 + lane], s1);
          atomicAdd(&red2[wn * WTN + j * 16 + lane], s2);
        }
      }
    }
    if (want_sums) {
      __syncthreads();
      float* g1 = (EM == E_STORE) ? p.sum : p.dbeta;
      float* g2 = (EM == E_STORE) ? p.sumsq : p.dgamma;
      const int nch = (EM == E_STORE) ? p.N : p.epi_xf.channels;
      for (int c = tid; c < BN; c += NTHREADS)
        if (n0 + c < p.N) {
          atomicAdd(g1 + (n0 + c) % nch, red1[c]);
          atomicAdd(g2 + (n0 + c) % nch, red2[c]);
        }
    }
  }
}

}  // namespace vae
