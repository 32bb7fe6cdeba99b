// Weight-gradient GEMM of the conv / transposed-conv layers in bf16, staged without transposes.
//
//   dW[m][r][s][j] += Σ_{n,hu,wu} U'[n,hu,wu,m] · V'[n, hu*S-P+r, wu*S-P+s, j]
//
//   Conv2d bwd_filter:          U = dy (output grid), V = x  (input grid);  m = k,  j = c
//   ConvTranspose2d bwd_filter: U = x  (input grid),  V = dy (output grid); m = c,  j = k
//   (U', V' = the stored tensors with their per-channel transforms: BatchNorm+LeakyReLU of the
//   activation, BatchNorm-backward of the gradient — vaehip.h vae_xform.)
//
// Both operands are NHWC with the reduction index (pixels) outermost, so the GEMM's K dimension
// is strided in memory and each operand row (one pixel) is channel-contiguous.  The implicit-GEMM
// kernel of vae_igemm.hpp transposes these tiles on their way into LDS (4-row x 2-k groups, 4-byte
// LDS stores); here every pixel row goes global -> registers -> LDS as whole 16-byte chunks in its
// natural [pixel][channel] order, and the MFMA operand fragments are read back column-major with
// ds_read_b64_tr_b16 (CDNA4's transposing LDS read: a 16-lane group reads a 4-row x 16-column
// block and lane i receives column i).  The LDS image uses 256-byte rows (128 channels) with the
// XOR chunk swizzle off(row, ch) = 256*row + 16*(ch ^ (((row&3)<<2) | ((row>>2)&3))), for which
// the transposed reads of v_mfma_f32_16x16x32_bf16 operands are bank-conflict-free
// (cdna_hip_programming.md T10).
//
// Block tile: 128 (m) x 128 (j) for one tap (r,s), K-step 32 pixels, 4 waves as 2x2, each wave
// 64x64 = 4x4 MFMA fragments.  The grid covers (m tiles, j tiles, taps, K slices); every K slice
// adds its partial tile into dW with fp32 atomics (the E_ACC convention of the igemm path).
// Global loads of K-step t+1 are in flight while the MFMAs of step t run (register staging,
// double-buffered LDS, one barrier per step).
#pragma once
#include "vae_igemm.hpp"

namespace vae {
namespace {

constexpr int WG_BM = 128, WG_BJ = 128, WG_BK = 32;

struct WgradParams {
  const void* u; vae_xform u_xf;     // [n][hu][wu][M]
  const void* v; vae_xform v_xf;     // [n][hv][wv][J]
  int n, hu, wu, M;
  int hv, wv, J;
  int R, S, P;
  int kper;                          // pixels per K slice (multiple of WG_BK)
  float* dw;                         // [M][R][R][J] fp32, accumulated
  FastDiv fd_wu, fd_hu, fd_r;
  uint32_t u_bytes, v_bytes;
};

__device__ __forceinline__ int wg_off(int row, int ch) {
  return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

typedef __bf16 __attribute__((ext_vector_type(4))) __attribute__((address_space(3))) wg_lds_bf16x4;
typedef __bf16 wg_bf16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ wg_bf16x4 wg_tr_read(const char* generic_lds_addr) {
  const uint32_t off = (uint32_t)(uintptr_t)generic_lds_addr;
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((wg_lds_bf16x4*)(uintptr_t)off);
}

// 8 bf16 of one chunk (+ aux chunk for BN_DY) -> transformed, repacked bf16; `ok` false -> zeros
__device__ __forceinline__ uint4 wg_xform(const uint32_t (&w)[4], const uint32_t (&y)[4], int kind, float slope,
                                          const Tab& t, int ch0, bool ok) {
  uint4 out;
  uint32_t* o = reinterpret_cast<uint32_t*>(&out);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float v0 = __uint_as_float(w[e] << 16), v1 = __uint_as_float(w[e] & 0xffff0000u);
    const int c = ch0 + 2 * e;
    if (kind == VAE_X_BN_ACT) {
      v0 = fmaf(v0, t.a[c], t.b[c]);
      v1 = fmaf(v1, t.a[c + 1], t.b[c + 1]);
      v0 = fmaxf(v0, v0 * slope);
      v1 = fmaxf(v1, v1 * slope);
    } else if (kind == VAE_X_ACT) {
      v0 = fmaxf(v0, v0 * slope);
      v1 = fmaxf(v1, v1 * slope);
    } else if (kind == VAE_X_BN_DY) {
      const float y0 = __uint_as_float(y[e] << 16), y1 = __uint_as_float(y[e] & 0xffff0000u);
      v0 = fmaf(t.a[c], v0, fmaf(t.b[c], y0, t.c[c]));
      v1 = fmaf(t.a[c + 1], v1, fmaf(t.b[c + 1], y1, t.c[c + 1]));
    }
    bf16x2 pk;
    pk[0] = (__bf16)(ok ? v0 : 0.f);
    pk[1] = (__bf16)(ok ? v1 : 0.f);
    o[e] = *reinterpret_cast<uint32_t*>(&pk);
  }
  return out;
}

__global__ void __launch_bounds__(256) wgrad_bf16_kernel(const WgradParams p) {
  kernarg_prefetch<(sizeof(WgradParams) < 1024 ? sizeof(WgradParams) : 1024)>();
  __shared__ __attribute__((aligned(16))) char Us[2][WG_BK * 256];
  __shared__ __attribute__((aligned(16))) char Vs[2][WG_BK * 256];
  __shared__ float tabs[6 * WG_BM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.x * WG_BM, j0 = blockIdx.y * WG_BJ;
  const int tap = (int)(blockIdx.z % (uint32_t)(p.R * p.R));
  const int slice = (int)(blockIdx.z / (uint32_t)(p.R * p.R));
  const int r = (int)p.fd_r.div(tap), s = tap - r * p.R;
  const long npix = (long)p.n * p.hu * p.wu;
  const long k0 = (long)slice * p.kper;
  const long k1 = min(npix, k0 + p.kper);

  // per-channel transform tables of this tile's 128 m / 128 j channels
  Tab tu{tabs, tabs + WG_BM, tabs + 2 * WG_BM, nullptr, nullptr};
  Tab tv{tabs + 3 * WG_BM, tabs + 4 * WG_BM, tabs + 5 * WG_BM, nullptr, nullptr};
  for (int i = tid; i < WG_BM; i += 256) {
    const int cu = m0 + i, cv = j0 + i;
    const bool bu = p.u_xf.kind == VAE_X_BN_ACT || p.u_xf.kind == VAE_X_BN_DY;
    const bool bv = p.v_xf.kind == VAE_X_BN_ACT || p.v_xf.kind == VAE_X_BN_DY;
    const int Cu = p.u_xf.channels, Cv = p.v_xf.channels;
    tu.a[i] = bu && cu < Cu ? p.u_xf.table[cu] : 0.f;
    tu.b[i] = bu && cu < Cu ? p.u_xf.table[Cu + cu] : 0.f;
    tu.c[i] = p.u_xf.kind == VAE_X_BN_DY && cu < Cu ? p.u_xf.table[2 * Cu + cu] : 0.f;
    tv.a[i] = bv && cv < Cv ? p.v_xf.table[cv] : 0.f;
    tv.b[i] = bv && cv < Cv ? p.v_xf.table[Cv + cv] : 0.f;
    tv.c[i] = p.v_xf.kind == VAE_X_BN_DY && cv < Cv ? p.v_xf.table[2 * Cv + cv] : 0.f;
  }

  const rsrc_t ru = make_rsrc(p.u, p.u_bytes), rv = make_rsrc(p.v, p.v_bytes);
  const bool udy = p.u_xf.kind == VAE_X_BN_DY, vdy = p.v_xf.kind == VAE_X_BN_DY;
  const rsrc_t ruy = make_rsrc(udy ? p.u_xf.aux : p.u, udy ? p.u_bytes : 0u);
  const rsrc_t rvy = make_rsrc(vdy ? p.v_xf.aux : p.v, vdy ? p.v_bytes : 0u);

  // this thread's two chunks per K-step: rows tid/16 and tid/16 + 16, chunk tid%16 (8 channels)
  const int ch = tid & 15, row0 = tid >> 4;
  const int cu = m0 + ch * 8, cv = j0 + ch * 8;
  const bool cu_ok = cu < p.M, cv_ok = cv < p.J;
  uint32_t wu[2][4], yu[2][4], wv_[2][4], yv[2][4];
  bool oku[2], okv[2];
  auto load = [&](long kb) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const long pix = kb + row0 + 16 * i;
      const bool in = pix < k1;
      const uint32_t pp = in ? (uint32_t)pix : 0u;
      const uint32_t q = p.fd_wu.div(pp);                 // n*hu + hu_i
      const int wu_i = (int)(pp - q * (uint32_t)p.wu);
      const uint32_t nn = p.fd_hu.div(q);
      const int hu_i = (int)(q - nn * (uint32_t)p.hu);
      const int hv_i = hu_i * p.S - p.P + r, wv_i = wu_i * p.S - p.P + s;
      const bool vin = in && (uint32_t)hv_i < (uint32_t)p.hv && (uint32_t)wv_i < (uint32_t)p.wv;
      oku[i] = in && cu_ok;
      okv[i] = vin && cv_ok;
      const uint32_t ou = oku[i] ? (uint32_t)((pix * p.M + cu) * 2) : kOOB;
      const uint32_t ov = okv[i] ? (uint32_t)(((((long)nn * p.hv + hv_i) * p.wv + wv_i) * p.J + cv) * 2) : kOOB;
      bload<16>(ru, ou, wu[i]);
      bload<16>(rv, ov, wv_[i]);
      if (udy) bload<16>(ruy, ou, yu[i]);
      if (vdy) bload<16>(rvy, ov, yv[i]);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = row0 + 16 * i;
      *reinterpret_cast<uint4*>(Us[buf] + wg_off(row, ch)) = wg_xform(wu[i], yu[i], p.u_xf.kind, p.u_xf.slope, tu, ch * 8, oku[i]);
      *reinterpret_cast<uint4*>(Vs[buf] + wg_off(row, ch)) = wg_xform(wv_[i], yv[i], p.v_xf.kind, p.v_xf.slope, tv, ch * 8, okv[i]);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed-read addresses: lane 4q+p of its 16-lane group g reads rows 8g+q (+4), chunk
  // c0 + (p>>1), byte 8*(p&1); c0 = first chunk of the fragment's 16 columns
  const int g = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  int aoff[4][2], boff[4][2];
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = 8 * g + 4 * h + q4;
      aoff[f][h] = wg_off(row, (wm * 64 + f * 16) / 8 + (p4 >> 1)) + 8 * (p4 & 1);
      boff[f][h] = wg_off(row, (wn * 64 + f * 16) / 8 + (p4 >> 1)) + 8 * (p4 & 1);
    }

  __syncthreads();                                  // tables ready
  if (k0 < k1) load(k0);
  int buf = 0;
  for (long kb = k0; kb < k1; kb += WG_BK) {
    store(buf);
    __syncthreads();
    if (kb + WG_BK < k1) load(kb + WG_BK);
    bf16x8 af[4], bfr[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const wg_bf16x4 a0 = wg_tr_read(Us[buf] + aoff[f][0]), a1 = wg_tr_read(Us[buf] + aoff[f][1]);
      const wg_bf16x4 b0 = wg_tr_read(Vs[buf] + boff[f][0]), b1 = wg_tr_read(Vs[buf] + boff[f][1]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        af[f][e] = a0[e]; af[f][4 + e] = a1[e];
        bfr[f][e] = b0[e]; bfr[f][4 + e] = b1[e];
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    buf ^= 1;
  }
  // D[m][j]: lane holds rows 4g + e of fragment i, column li of fragment j
  const long rowstride = (long)p.R * p.R * p.J;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int jj = j0 + wn * 64 + j * 16 + li;
      if (jj >= p.J) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int mm = m0 + wm * 64 + i * 16 + 4 * g + e;
        if (mm < p.M) atomicAdd(p.dw + mm * rowstride + (long)tap * p.J + jj, acc[i][j][e]);
      }
    }
}

// Host: can the fast path take this problem?  (bf16, channel counts multiple of 8, NHWC operands,
// BatchNorm transforms with precomputed tables, 32-bit buffer offsets.)
// Measured (profiles/r1_v3_*): the 128x128 tile pays off on the VQ-VAE shapes (3x3 residual wgrad
// 405 -> 142 us, M = J = 256, 32768 pixels) but loses on the VanillaVAE ones (32-64 channels, or
// 256-1024 pixels: one block's fixed costs over few K-steps), which stay on the igemm path.
inline bool wgrad_ok(int dtype, const vae_xform& ux, const vae_xform& vx, long u_elems, long v_elems, int M, int J) {
  if (dtype != VAE_BF16) return false;
  if (M % 8 || J % 8) return false;
  // (J == 8, the padded RGB ends, measured slower too: 536 -> 692 us on the VQ output ConvT)
  if (M < 64 || J < 64 || u_elems / M < 8192) return false;
  auto xf_ok2 = [](const vae_xform& x) {
    if (x.kind == VAE_X_BN_ACT || x.kind == VAE_X_BN_DY) return x.table != nullptr;
    return x.kind == VAE_X_NONE || x.kind == VAE_X_ACT;
  };
  if (!xf_ok2(ux) || !xf_ok2(vx)) return false;
  if (u_elems * 2 >= (1l << 31) || v_elems * 2 >= (1l << 31)) return false;
  return true;
}

inline int wgrad_launch(WgradParams p, hipStream_t st) {
  p.fd_wu = make_fastdiv(p.wu);
  p.fd_hu = make_fastdiv(p.hu);
  p.fd_r = make_fastdiv(p.R);
  const long npix = (long)p.n * p.hu * p.wu;
  p.u_bytes = (uint32_t)(npix * p.M * 2);
  p.v_bytes = (uint32_t)((long)p.n * p.hv * p.wv * p.J * 2);
  const long tiles = (long)((p.M + WG_BM - 1) / WG_BM) * ((p.J + WG_BJ - 1) / WG_BJ) * p.R * p.R;
  const long ksteps = (npix + WG_BK - 1) / WG_BK;
  // K slices: ~4 workgroups per CU, at least 8 K-steps per slice
  long split = (4 * kCUs + tiles - 1) / tiles;
  if (split > ksteps / 8) split = ksteps / 8;
  if (split < 1) split = 1;
  p.kper = (int)(((ksteps + split - 1) / split) * WG_BK);
  split = (npix + p.kper - 1) / p.kper;
  const dim3 grid((p.M + WG_BM - 1) / WG_BM, (p.J + WG_BJ - 1) / WG_BJ, (unsigned)(p.R * p.R * split));
  VAE_LAUNCH(wgrad_bf16_kernel, grid, dim3(256), 0, st, p);
  return check_launch("wgrad_bf16");
}

}  // namespace
}  // namespace vae
