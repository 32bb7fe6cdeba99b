// Direct-fragment implicit GEMM for the forward / data-gradient shapes of the VAE step.
//
//   C[m][n] = sum_k A(m,k) * B[n][k]         (B = weights with k contiguous: Conv2d [Co][R][S][Ci],
//                                            ConvTranspose2d [Ci][R][S][Co] read as [n][k], Linear)
//
// Why a second GEMM family: at these sizes (M <= 64K rows, N <= 512, K <= 2304) the LDS-staged
// kernel of vae_igemm.hpp pays one register->LDS->barrier round per 64-deep K-tile for a few
// MFMAs per wave (measured ~0.6 us per K-tile).  Here every wave loads its MFMA operand
// fragments straight from global memory — lane l of a 16x16x32 fragment needs 8 consecutive k
// of one row, i.e. 16 contiguous bytes of an NHWC pixel (a 32-deep k-step never crosses a tap
// because the gathered tensor has C % 32 == 0) — applies the per-channel transform
// (BatchNorm+LeakyReLU, or BatchNorm-backward) in registers, and accumulates.  The 4 waves of
// a workgroup split the workgroup's K range among themselves (no barrier in the K loop) and
// reduce their partial tiles once through LDS.  Each wave keeps a ring of FG_PD k-steps of
// loads in flight.
//
// Epilogues are those of vae_igemm.hpp (bias + per-channel sums / activation backward +
// BN-backward sums / split-K slab for igemm_finalize).
#pragma once
#include "vae_igemm.hpp"

namespace vae {

constexpr int FG_PD = 4;          // k-steps of loads in flight per wave

template <class T> struct FragIO;
template <> struct FragIO<__bf16> {
  static constexpr int W = 4;     // uint32 per 8-element fragment row
};
template <> struct FragIO<float> {
  static constexpr int W = 8;
};

// 8 elements (16 B bf16 / 32 B fp32) through a buffer resource; out-of-range offset -> 0
template <class TIn>
__device__ __forceinline__ void fload8(rsrc_t r, uint32_t off, uint32_t* w) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  w[0] = v[0]; w[1] = v[1]; w[2] = v[2]; w[3] = v[3];
  if constexpr (sizeof(TIn) == 4) {
    const auto u = __builtin_amdgcn_raw_buffer_load_b128(r, off == kOOB ? kOOB : off + 16, 0, 0);
    w[4] = u[0]; w[5] = u[1]; w[6] = u[2]; w[7] = u[3];
  }
}

template <class TIn>
__device__ __forceinline__ float felem(const uint32_t* w, int e) {
  if constexpr (sizeof(TIn) == 4) return __uint_as_float(w[e]);
  else return __uint_as_float((e & 1) ? (w[e >> 1] & 0xffff0000u) : (w[e >> 1] << 16));
}

// Transform of one A fragment row (8 consecutive k = 8 consecutive channels starting at ch);
// `ok` false -> all zero (padding / out of range: zero AFTER the transform)
template <class TIn, bool DY>
__device__ __forceinline__ void ftransform(const Src<TIn>& s, const Tab& t, const uint32_t* w, const uint32_t* y,
                                           int ch, bool ok, float (&v)[8]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = felem<TIn>(w, e);
  if (s.kind == VAE_X_BN_ACT) {
    const f32x4 a0 = tab4(t.a, ch), a1 = tab4(t.a, ch + 4), b0 = tab4(t.b, ch), b1 = tab4(t.b, ch + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = lrelu(fmaf(v[e], a0[e], b0[e]), s.slope);
      v[e + 4] = lrelu(fmaf(v[e + 4], a1[e], b1[e]), s.slope);
    }
  } else if (s.kind == VAE_X_ACT) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = lrelu(v[e], s.slope);
  } else if (DY && s.kind == VAE_X_BN_DY) {
    const f32x4 a0 = tab4(t.a, ch), a1 = tab4(t.a, ch + 4), b0 = tab4(t.b, ch), b1 = tab4(t.b, ch + 4);
    const f32x4 c0 = tab4(t.c, ch), c1 = tab4(t.c, ch + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = fmaf(a0[e], v[e], fmaf(b0[e], felem<TIn>(y, e), c0[e]));
      v[e + 4] = fmaf(a1[e], v[e + 4], fmaf(b1[e], felem<TIn>(y, e + 4), c1[e]));
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = ok ? v[e] : 0.f;
}

// A/B fragments of one k-step held by one lane
template <class TA, class TB, int TM, int TN, bool DY>
struct FSlot {
  uint32_t a[TM][FragIO<TA>::W];
  uint32_t y[DY ? TM : 1][DY ? FragIO<TA>::W : 1];
  uint32_t b[TN][FragIO<TB>::W];
  int ch;           // transform channel of the lane's first k
  uint32_t okm;     // bit i: A row i's gathered position is valid
};

template <int BM, int BN> struct FgEpi {
  static constexpr int EPR = BM * BN / 256;          // output elements per lane in the epilogue
  static_assert(EPR >= 1 && EPR <= BN && BN % EPR == 0, "epilogue mapping");
};

// ------------------------------------------------------------------------------ kernel
// grid: (ceil(M / BM), ceil(N / BN), nphase * ksplit); 256 threads = 4 waves, each wave the whole
// BM x BN tile over a quarter of the workgroup's k-steps.  Requirements (host): B_NK weights,
// k-steps of 32 inside one tap (gathered C % 32 == 0; dense K % 32 == 0), 16-B aligned rows.
template <class T, class TA, int BM, int BN, int AM, int EM, bool DYA>
__global__ void __launch_bounds__(256) fgemm_kernel(const GemmParams p) {
  kernarg_prefetch<(sizeof(GemmParams) < 1024 ? sizeof(GemmParams) : 1024)>();
  constexpr int TM = BM / 16, TN = BN / 16;
  constexpr bool EPI_TBL = (EM == E_BNBWD);
  constexpr int EPR = FgEpi<BM, BN>::EPR;
  __shared__ __attribute__((aligned(16))) float red[4][BM][BN + 1];
  __shared__ float cs1[BN], cs2[BN];
  extern __shared__ float tabs[];

#ifdef VAE_PROBE
  unsigned long long clk[4] = {0, 0, 0, 0};
  const unsigned long long wall0 = threadIdx.x == 0 ? wall_clock64() : 0;
#endif
  PROBE_MARK(0);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int phase = (p.nphase > 1) ? (int)(blockIdx.z / p.ksplit) : 0;
  const int ks = blockIdx.z - phase * p.ksplit;

  int Kp = p.K;
  const PhaseInfo pq = make_phase(p, phase);
  if constexpr (AM == A_CONVT) Kp = pq.nth * pq.ntw * p.gc;
  const int nsteps = (Kp + 31) / 32;
  const int per_blk = (nsteps + p.ksplit - 1) / p.ksplit;
  const int sb0 = ks * per_blk, sb1 = min(nsteps, sb0 + per_blk);
  const int per_w = (sb1 - sb0 + 3) / 4;
  const int s0 = min(sb1, sb0 + wave * per_w), s1 = min(sb1, s0 + per_w);
  const int kend = min(Kp, sb1 * 32);

  // tables: A transform, epilogue transform
  Tab ta, te;
  {
    const int ca = tab_stride(p.a_xf.channels), ce = tab_stride(p.epi_xf.channels);
    ta = Tab{tabs, tabs + ca, tabs + 2 * ca, nullptr, nullptr};
    float* q = tabs + (tab_floats(p.a_xf, false) > 0 ? 3 * ca : 0);
    te = Tab{q, q + ce, nullptr, q + 2 * ce, q + 3 * ce};
  }
  const Src<TA> sa = make_src<TA>(p.a_ptr, p.a_bytes, p.a_xf);
  const rsrc_t rb = make_rsrc(p.b_ptr, p.b_bytes);

  // per-lane A rows (fragment i: row m0 + 16i + li) and B rows (fragment j: n0 + 16j + li)
  RowOperand<TA, AM, true> ar[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) ar[i].init(p, m0 + 16 * i + li, p.M, phase, p.a_ld);
  int bbase[TN];
  bool bok[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + 16 * j + li;
    bok[j] = n < p.N;
    bbase[j] = n * p.b_ld;
  }

  using Slot = FSlot<TA, T, TM, TN, DYA>;
  const bool a_bn = p.a_xf.kind >= VAE_X_BN_ACT;
  auto load_step = [&](int s, Slot& sl) {
    const int k0 = s * 32;
    const int kl = k0 + 8 * g;                       // this lane's first k
    const KTap t = RowOperand<TA, AM, true>::tap(p, pq, p.fd_ach, p.a_xf.channels, a_bn, kl, min(kend, s1 * 32));
    sl.ch = t.ch;
    uint32_t okm = 0u;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      bool ok = ar[i].valid && t.kin;
      if constexpr (AM == A_CONV || AM == A_CONVT)
        ok = ok && (uint32_t)(ar[i].hi0 + t.r) < (uint32_t)p.gh && (uint32_t)(ar[i].wi0 + t.s) < (uint32_t)p.gw;
      okm |= (uint32_t)ok << i;
      const uint32_t off = ok ? (uint32_t)(ar[i].base + t.toff) * (uint32_t)sizeof(TA) : kOOB;
      fload8<TA>(sa.x, off, sl.a[i]);
      if constexpr (DYA) fload8<TA>(sa.y, off, sl.y[i]);
    }
    sl.okm = okm;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const uint32_t off = (bok[j] && t.kin) ? (uint32_t)(bbase[j] + kl) * (uint32_t)sizeof(T) : kOOB;
      fload8<T>(rb, off, sl.b[j]);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute_step = [&](const Slot& sl) {
    if constexpr (sizeof(T) == 2) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if (sa.kind == VAE_X_NONE && sizeof(TA) == 2) {
          uint32_t z[4];
          const bool ok = (sl.okm >> i) & 1u;
#pragma unroll
          for (int e = 0; e < 4; ++e) z[e] = ok ? sl.a[i][e] : 0u;
          af[i] = *reinterpret_cast<const bf16x8*>(z);
        } else {
          float v[8];
          ftransform<TA, DYA>(sa, ta, sl.a[i], sl.y[DYA ? i : 0], sl.ch, (sl.okm >> i) & 1u, v);
#pragma unroll
          for (int e = 0; e < 8; ++e) af[i][e] = (__bf16)v[e];
        }
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(sl.b[j]);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    } else {
      float af[TM][8];
#pragma unroll
      for (int i = 0; i < TM; ++i) ftransform<TA, DYA>(sa, ta, sl.a[i], sl.y[DYA ? i : 0], sl.ch, (sl.okm >> i) & 1u, af[i]);
      // 8 k per lane = 8 MFMA k-slots (k permuted; the sum is order-free)
#pragma unroll
      for (int e = 0; e < 8; ++e)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][e], __uint_as_float(sl.b[j][e]), acc[i][j], 0, 0, 0);
    }
  };

  // ---- prologue: the ring's loads go out before the tables are filled
  Slot ring[FG_PD];
#pragma unroll
  for (int u = 0; u < FG_PD; ++u) load_step(s0 + u, ring[u]);
  tab_fill(p.a_xf, ta, false, blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0);
  if constexpr (EPI_TBL) tab_fill(p.epi_xf, te, true, false);
  for (int i = tid; i < BN; i += 256) { cs1[i] = 0.f; cs2[i] = 0.f; }
  __syncthreads();
  PROBE_MARK(1);

  // ---- K loop of this wave (no barriers)
  for (int sb = s0; sb < s1; sb += FG_PD) {
#pragma unroll
    for (int u = 0; u < FG_PD; ++u) {
      if (sb + u < s1) {
        compute_step(ring[u]);
        load_step(sb + u + FG_PD, ring[u]);
      }
    }
  }

  PROBE_MARK(2);
#ifdef VAE_PROBE
  struct ProbeEnd {
    unsigned long long* pr; unsigned long long* clk; unsigned long long w0;
    __device__ ~ProbeEnd() { PROBE_MARK(3); probe_write(pr, clk, w0); }
  } probe_end{p.probe, clk, wall0};
#endif
  // ---- reduce the 4 waves' partial tiles through LDS
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) red[wave][16 * i + 4 * g + e][16 * j + li] = acc[i][j][e];
  __syncthreads();
  // this lane's EPR consecutive outputs
  const int idx0 = wave * (BM * BN / 4) + lane * EPR;
  const int row_l = idx0 / BN, col_l = idx0 - row_l * BN;
  const int row = m0 + row_l;
  float v[EPR];
#pragma unroll
  for (int e = 0; e < EPR; ++e)
    v[e] = (red[0][row_l][col_l + e] + red[1][row_l][col_l + e]) + (red[2][row_l][col_l + e] + red[3][row_l][col_l + e]);

  if (p.slab) {
    float* sl = p.slab + ((long)(phase * p.ksplit + ks) * p.M) * p.N;
#pragma unroll
    for (int e = 0; e < EPR; ++e)
      if (row < p.M && n0 + col_l + e < p.N) sl[(long)row * p.N + n0 + col_l + e] = v[e];
    return;
  }
  if constexpr (EM == E_REPARAM) {
    ReparamIn rin[EPR];
#pragma unroll
    for (int e = 0; e < EPR; ++e) rin[e] = reparam_load(p, row, n0 + col_l + e, row < p.M && n0 + col_l + e < p.N);
#pragma unroll
    for (int e = 0; e < EPR; ++e)
      if (row < p.M && n0 + col_l + e < p.N) reparam_apply(p, row, n0 + col_l + e, v[e], rin[e]);
    return;
  } else {
    const rsrc_t raux = epi_aux_rsrc<EM>(p);
    const rsrc_t rres = epi_res_rsrc<EM>(p);
    const bool has_res = EM == E_BNBWD && p.residual != nullptr;
    const int ob = out_row_base(p, phase, row < p.M ? row : 0);
    float aux[EPR], res[EPR], bias[EPR];
#pragma unroll
    for (int e = 0; e < EPR; ++e) {
      const int col = n0 + col_l + e;
      const bool ok = row < p.M && col < p.N;
      aux[e] = ld_elem<T>(raux, ok ? (uint32_t)(ob + col) * (uint32_t)sizeof(T) : kOOB);
      res[e] = has_res ? ld_elem<T>(rres, ok ? (uint32_t)(ob + col) * (uint32_t)sizeof(T) : kOOB) : 0.f;
      bias[e] = (EM == E_STORE && p.bias && col < p.N) ? p.bias[col] : 0.f;
    }
    float s1[EPR], s2[EPR];
#pragma unroll
    for (int e = 0; e < EPR; ++e) {
      s1[e] = 0.f; s2[e] = 0.f;
      const int col = n0 + col_l + e;
      if (row < p.M && col < p.N) epi_apply<T, EM>(p, te, col, ob + col, v[e], aux[e], bias[e], s1[e], s2[e], res[e]);
    }
    if (epi_wants_sums<EM>(p)) {
      // lanes holding the same columns differ in the bits above log2(BN / EPR)
#pragma unroll
      for (int e = 0; e < EPR; ++e) {
#pragma unroll
        for (int off = BN / EPR; off < 64; off <<= 1) {
          s1[e] += __shfl_xor(s1[e], off);
          s2[e] += __shfl_xor(s2[e], off);
        }
      }
      if (lane < BN / EPR) {
#pragma unroll
        for (int e = 0; e < EPR; ++e) {
          atomicAdd(&cs1[col_l + e], s1[e]);
          atomicAdd(&cs2[col_l + e], s2[e]);
        }
      }
      __syncthreads();
      for (int c = tid; c < BN; c += 256)
        if (n0 + c < p.N) epi_flush_sums<EM>(p, blockIdx.x + blockIdx.z * gridDim.x, n0 + c, cs1[c], cs2[c]);
    }
  }
}

}  // namespace vae
