// 3x3 / stride-1 / pad-1 convolution on a 16 x 16 grid as an image-tile implicit GEMM: the
// VQ-VAE's residual-stack convolutions (models/vq_vae.py:57-70, the Conv3x3 layers at :94-166),
// forward and data gradient (the data gradient of a stride-1 conv is the same correlation with the
// taps flipped, over the swapped-axes weights).
//
//   out[n, h, w, j] = Σ_{r,s,c} A[n, h+dr(r)-1, w+ds(s)-1, c] · B[j][r][s][c]   (+ epilogue)
//
// Why not the conv-GEMM (vae_cgemm.hpp): there, a 128 x 128 tile gathers its A rows per tap from
// L2 — every input element is fetched 9 times and every K-step streams 32 KB for 2.1 MFLOP, at the
// per-CU L2 bandwidth edge (23-31 % of bf16 peak, 50-55 us per call at B=128).  Here one
// workgroup owns one whole image (256 output pixels) x 128 output channels: per 32-channel chunk
// it stages the image's 18 x 18 halo patch once (21 KB) and the chunk's 9 taps x 128 weight rows
// (74 KB) in LDS, then every tap reads its A fragments from the patch at a shifted row — 18.9
// MFLOP per 94 KB staged, 3x the reuse of the 128 x 128 tile.
//
// Block: 512 threads = 8 waves, wave (wm, wn) = output rows 4wm..4wm+3 (one 16-pixel MFMA row
// block each) x output channels 64wn..64wn+63; v_mfma_f32_16x16x32_bf16 (lane l: A row l&15 =
// output column, k 8*(l>>4)..+7; B column l&15; accumulator rows 4*(l>>4)..+3).  LDS rows are
// 32 bf16 (64 B) with the 16-byte chunk c of row P stored at slot c ^ ((P >> 1) & 2): the lane
// groups of ds_read_b128 ({0-3,12-15,20-27}, ... — MI355X_MICROARCH.md LDS table) then hit 16
// distinct 4-bank groups for ANY first row (the A reads start at a tap-shifted patch row); an
// 80-B padded row measured 48 % of the LDS cycles as bank conflicts (SQ_LDS_BANK_CONFLICT).
// The next chunk's global loads are issued before the current chunk's MFMAs (register prefetch,
// 12 x 16 B per thread), so their latency hides behind 144 MFMAs per wave.
#include "vae_c3.hpp"
#include "vae_igemm.hpp"
#include <stdlib.h>

namespace vae {
namespace {

constexpr int C3_LD = 32;                         // bf16 per LDS operand row (32 channels, swizzled)
constexpr int C3_PW = 18;                         // halo patch width (16 + 2)
constexpr int C3_PATCH = C3_PW * C3_PW;           // 324 pixels
constexpr int C3_A_ITEMS = C3_PATCH * 4;          // 16-byte chunks of the patch (1296)
// BN output channels per workgroup, 64 threads per 16 channels (waves of 64 pixel rows x 64
// channels): BN = 128 — 512 threads, 135 KB of LDS (one workgroup per CU); BN = 64 — 256 threads,
// 70 KB, two workgroups per CU whose load / store / epilogue phases overlap each other's MFMAs
template <int BN> struct C3T {
  static constexpr int NT = BN * 4;
  static constexpr int WN = BN / 64;                                // waves across the channels
  static constexpr int B_ITEMS = 9 * BN * 4;                        // 16-byte chunks of the weights
  static constexpr int AP = (C3_A_ITEMS + NT - 1) / NT;
  static constexpr int BP = B_ITEMS / NT;                           // 9
  static constexpr int LDC = BN + 4;                                // fp32 epilogue tile row
  static constexpr int OPER = (C3_PATCH + 9 * BN) * C3_LD * 2;
  static constexpr int EPI = 256 * LDC * 4;
  static constexpr int LDS = OPER > EPI ? OPER : EPI;
  static_assert(B_ITEMS % NT == 0, "weight tile loads");
};

struct C3Params {
  const void* a;
  const void* b;
  void* out;
  const float* bias;
  const void* residual;
  const void* aux;
  uint32_t a_bytes, b_bytes, o_bytes;
  float a_slope, aux_slope;
  int a_act, flip, C, N;
  int dbg;                  // diagnostics (VAE_C3_DBG): 1 no loads in the loop, 2 no MFMAs, 4 no LDS stores
};

// element offset of 16-byte chunk c of LDS row P (the bank-conflict swizzle above)
__device__ __forceinline__ int c3_sw(int P, int c) { return P * C3_LD + ((c ^ ((P >> 1) & 2)) << 3); }

__device__ __forceinline__ uint32_t lrelu_pk(uint32_t w, float slope) {
  f32x2 v = f32x2{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)};
  v = __builtin_elementwise_max(v, v * f32x2{slope, slope});
  bf16x2 pk;
  pk[0] = (__bf16)v[0];
  pk[1] = (__bf16)v[1];
  return *reinterpret_cast<uint32_t*>(&pk);
}

template <int BN>
__global__ void __launch_bounds__(BN * 4) c3_kernel(const C3Params p) {
  kernarg_prefetch<(sizeof(C3Params) < 1024 ? sizeof(C3Params) : 1024)>();
  using T = C3T<BN>;
  constexpr int C3_NT = T::NT, C3_AP = T::AP, C3_BP = T::BP, C3_LDC = T::LDC, C3_BN = BN;
  __shared__ __attribute__((aligned(16))) char smem[T::LDS];
  __bf16* As = reinterpret_cast<__bf16*>(smem);                  // [324][40]
  __bf16* Bs = As + C3_PATCH * C3_LD;                             // [9][128][40]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / T::WN, wn = wave % T::WN;
  // XCD-aware order: workgroup b runs on XCD b % 8; each XCD takes a contiguous tile range, so
  // the two channel tiles of an image share that XCD's L2 copy of the patch
  const int nt = p.N / C3_BN;
  int tile;
  {
    const int nb = (int)gridDim.x, b = (int)blockIdx.x;
    const int q = nb >> 3, r = nb & 7, x = b & 7, loc = b >> 3;
    tile = x * q + min(x, r) + loc;
  }
  const int img = tile / nt, n0 = (tile - img * nt) * C3_BN;
  const rsrc_t ra = make_rsrc(p.a, p.a_bytes);
  const rsrc_t rb = make_rsrc(p.b, p.b_bytes);
  const int C = p.C;

  // per-thread load slots: A patch chunk (pixel, 16-B column) and weight row chunk
  uint32_t abase[C3_AP];
  bool aok[C3_AP];
#pragma unroll
  for (int k = 0; k < C3_AP; ++k) {
    const int it = tid + C3_NT * k;
    const int pix = it >> 2, ch = it & 3;
    const int ph = pix / C3_PW, pw = pix - ph * C3_PW;
    const int h = ph - 1, w = pw - 1;
    aok[k] = it < C3_A_ITEMS && (unsigned)h < 16u && (unsigned)w < 16u;
    abase[k] = (uint32_t)((((img * 16 + (aok[k] ? h : 0)) * 16 + (aok[k] ? w : 0)) * C + ch * 8) * 2);
  }
  uint32_t bbase[C3_BP];
#pragma unroll
  for (int k = 0; k < C3_BP; ++k) {
    const int it = tid + C3_NT * k;
    const int row = it >> 2, ch = it & 3;
    const int t = row / C3_BN, nl = row % C3_BN;
    bbase[k] = (uint32_t)((((n0 + nl) * 9 + t) * C + ch * 8) * 2);
  }
  uint32_t ar[C3_AP][4], br[C3_BP][4];
  auto load = [&](int c0) {
    const uint32_t cb = (uint32_t)c0 * 2u;
#pragma unroll
    for (int k = 0; k < C3_AP; ++k) bload<16>(ra, aok[k] ? abase[k] + cb : kOOB, ar[k]);
#pragma unroll
    for (int k = 0; k < C3_BP; ++k) bload<16>(rb, bbase[k] + cb, br[k]);
  };
  auto store = [&]() {
#pragma unroll
    for (int k = 0; k < C3_AP; ++k) {
      const int it = tid + C3_NT * k;
      if (it < C3_A_ITEMS) {
        uint4 v = uint4{ar[k][0], ar[k][1], ar[k][2], ar[k][3]};
        if (p.a_act) {
          v.x = lrelu_pk(v.x, p.a_slope); v.y = lrelu_pk(v.y, p.a_slope);
          v.z = lrelu_pk(v.z, p.a_slope); v.w = lrelu_pk(v.w, p.a_slope);
        }
        *reinterpret_cast<uint4*>(As + c3_sw(it >> 2, it & 3)) = v;
      }
    }
#pragma unroll
    for (int k = 0; k < C3_BP; ++k) {
      const int it = tid + C3_NT * k;
      *reinterpret_cast<uint4*>(Bs + c3_sw(it >> 2, it & 3)) = uint4{br[k][0], br[k][1], br[k][2], br[k][3]};
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int kq = lane >> 4, lr = lane & 15;
  // the fragments of tap t+1 are read from LDS while tap t's 16 MFMAs run (their latency was
  // exposed at the head of every tap)
  auto frags = [&](int t, bf16x8 (&af)[4], bf16x8 (&bfr)[4]) {
    const int r = t / 3, s = t - 3 * (t / 3);
    const int dr = p.flip ? 2 - r : r, ds = p.flip ? 2 - s : s;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      af[i] = *reinterpret_cast<const bf16x8*>(As + c3_sw((wm * 4 + i + dr) * C3_PW + lr + ds, kq));
#pragma unroll
    for (int j = 0; j < 4; ++j)
      bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + c3_sw(t * C3_BN + wn * 64 + j * 16 + lr, kq));
  };
  auto compute = [&]() {
    bf16x8 af[2][4], bfr[2][4];
    frags(0, af[0], bfr[0]);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      // this tap's fragments (read during the previous tap) have landed: one wait here, fenced
      // by scheduling barriers on both sides (the scheduler otherwise floats it above the
      // previous tap's last MFMAs, or waits after every read), so the next tap's reads issued
      // between the MFMAs below need none (lgkmcnt counts in order)
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt(0xc07f);                  // lgkmcnt(0)
      __builtin_amdgcn_sched_barrier(0);
      if (t + 1 < 9) frags(t + 1, af[(t + 1) & 1], bfr[(t + 1) & 1]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[t & 1][i], bfr[t & 1][j], acc[i][j], 0, 0, 0);
      if (t + 1 < 9) {
        // interleave: the next tap's 8 LDS reads one per MFMA over the first half of this tap's
        // 16, so they have landed by the next tap's head (the scheduler otherwise sinks them to
        // their first use)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
      }
    }
  };

  const int nchunks = C / 32;
  load(0);
  store();
  __syncthreads();
  for (int kc = 0; kc < nchunks; ++kc) {
    const bool more = kc + 1 < nchunks;
    // unconditional (the last chunk reloads itself, unused): a load under a branch makes the
    // compiler merge the prefetch registers with copies that wait for the loads right here,
    // before the MFMAs they were meant to hide behind
    if (!(p.dbg & 1)) load((more ? kc + 1 : kc) * 32);
    __builtin_amdgcn_sched_barrier(0);      // (keep the loads ahead of the MFMAs)
    if (!(p.dbg & 2)) compute();
    __syncthreads();
    if (more && !(p.dbg & 4)) {
      store();
      __syncthreads();
    }
  }

  // ---- epilogue through LDS: fp32 tile [256 pixels][128 (+4)], then 16-byte rows
  float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        Cs[((wm * 4 + i) * 16 + 4 * (lane >> 4) + e) * C3_LDC + wn * 64 + j * 16 + lr] = acc[i][j][e];
  __syncthreads();
  const rsrc_t rres = make_rsrc(p.residual ? p.residual : p.out, p.residual ? p.o_bytes : 0u);
  const rsrc_t raux = make_rsrc(p.aux ? p.aux : p.out, p.aux ? p.o_bytes : 0u);
  __bf16* out = static_cast<__bf16*>(p.out);
#pragma unroll 2
  for (int k = 0; k < 8; ++k) {
    const int it = tid + C3_NT * k;
    const int pix = it / (C3_BN / 8), cg = (it % (C3_BN / 8)) * 8;
    const uint32_t o = (uint32_t)((img * 256 + pix) * p.N + n0 + cg);
    uint32_t rs[4], ax[4];
    bload<16>(rres, p.residual ? o * 2u : kOOB, rs);
    bload<16>(raux, p.aux ? o * 2u : kOOB, ax);
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(Cs + pix * C3_LDC + cg);
    const f32x4 v1 = *reinterpret_cast<const f32x4*>(Cs + pix * C3_LDC + cg + 4);
    float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    uint32_t pk[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float g0 = v[2 * e] + __uint_as_float(rs[e] << 16);
      float g1 = v[2 * e + 1] + __uint_as_float(rs[e] & 0xffff0000u);
      if (p.bias) { g0 += p.bias[n0 + cg + 2 * e]; g1 += p.bias[n0 + cg + 2 * e + 1]; }
      if (p.aux) {
        if (!(__uint_as_float(ax[e] << 16) > 0.f)) g0 *= p.aux_slope;
        if (!(__uint_as_float(ax[e] & 0xffff0000u) > 0.f)) g1 *= p.aux_slope;
      }
      bf16x2 h;
      h[0] = (__bf16)g0;
      h[1] = (__bf16)g1;
      pk[e] = *reinterpret_cast<uint32_t*>(&h);
    }
    *reinterpret_cast<uint4*>(out + o) = uint4{pk[0], pk[1], pk[2], pk[3]};
  }
}

// ------------------------------------------------------------------ forward / data gradient, LDS-DMA
// The same correlation on an LDS-DMA pipeline (buffer_load ... lds: no VGPR staging, no store
// phase between the chunks).  A stage is one 32-channel chunk x one tap row r: the 16 patch rows
// that row reads (18 x 16 = 288 pixels, 64-B LDS rows) and its 3 taps x 128 weight rows — 43 KB,
// three stages in a ring (two in flight while one computes), where the whole-chunk stage of
// c3_kernel (95 KB) left room for one and exposed the chunk loads and LDS stores (~10 us per call,
// DESIGN §4 ablation).  Re-reading the patch per tap row costs 36 % more L2 -> LDS bytes.
// The LDS image is lane-linear (lane l of a wave-instruction writes base + 16 l): row P holds its
// chunk c at slot c ^ ((P >> 1) & 2), set through the per-lane source address; out-of-image patch
// pixels read zeros through the buffer resource's range check.  The LeakyReLU of an activated A
// (ACT) is applied to the fragments after their LDS reads.
constexpr int D3_PROWS = 384;                      // patch image rows per stage (288 used, DMA-uniform)
constexpr int D3_WROWS = 384;                      // 3 taps x 128 weight rows
constexpr int D3_STAGE = (D3_PROWS + D3_WROWS) * 64;        // 49152
constexpr int D3_OPS = 3 * D3_STAGE;                        // 147456
constexpr int D3_EPI = 256 * C3T<128>::LDC * 4;             // 135168
constexpr int D3_LDS = D3_OPS > D3_EPI ? D3_OPS : D3_EPI;

typedef __attribute__((address_space(3))) void c3_lds_void;
__device__ __forceinline__ void c3_glds16(rsrc_t r, const char* lds_wave_base, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (c3_lds_void*)(uintptr_t)(uint32_t)(uintptr_t)lds_wave_base, 16, voff, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 lrelu8(bf16x8 v, float slope) {
  uint32_t* w = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
  for (int e = 0; e < 4; ++e) w[e] = lrelu_pk(w[e], slope);
  return v;
}

template <int ACT>
__global__ void __launch_bounds__(512) c3d_kernel(const C3Params p) {
  kernarg_prefetch<(sizeof(C3Params) < 1024 ? sizeof(C3Params) : 1024)>();
  __shared__ __attribute__((aligned(16))) char smem[D3_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nt = p.N / 128;
  int tile;
  {
    const int nb = (int)gridDim.x, b = (int)blockIdx.x;
    const int q = nb >> 3, r = nb & 7, x = b & 7, loc = b >> 3;
    tile = x * q + min(x, r) + loc;
  }
  const int img = tile / nt, n0 = (tile - img * nt) * 128;
  const rsrc_t ra = make_rsrc(p.a, p.a_bytes);
  const rsrc_t rb = make_rsrc(p.b, p.b_bytes);
  const int C = p.C;
  const int rowb = 16 * C * 2;                                // bytes of one image row of A

  // this wave's 6 DMA instructions per stage: I = wave + 8u; I < 24 patch rows 16I.., else weights
  int poff[3], prow[3], pwok[3];
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int L = 16 * (wave + 8 * u) + (lane >> 2);
    const int c = (lane & 3) ^ ((L >> 1) & 2);
    const int ph = L / C3_PW, pw = L - ph * C3_PW;
    prow[u] = L < 288 ? ph : 99;                              // patch row within the tap row's 16
    pwok[u] = (unsigned)(pw - 1) < 16u;
    poff[u] = (((img * 16 + ph - 1) * 16 + (pw - 1)) * C + c * 8) * 2;   // at dr = 0 (may be < 0: masked)
  }
  int woff[3];
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int L = 16 * (wave + 8 * u) + (lane >> 2);         // weight row s * 128 + nl
    const int c = (lane & 3) ^ ((L >> 1) & 2);
    const int sc = L >> 7, nl = L & 127;
    woff[u] = (((n0 + nl) * 9 + sc) * C + c * 8) * 2;         // at tap row 0
  }
  // stage (chunk kc, tap row r) -> buffer b
  auto issue = [&](int kc, int r, int b) {
    const int dr = p.flip ? 2 - r : r;
    char* base = smem + b * D3_STAGE;
    const uint32_t cb = (uint32_t)kc * 64u;
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const bool ok = pwok[u] && (unsigned)(prow[u] + dr - 1) < 16u;
      c3_glds16(ra, base + (wave + 8 * u) * 1024, ok ? (uint32_t)(poff[u] + dr * rowb) + cb : kOOB);
    }
#pragma unroll
    for (int u = 0; u < 3; ++u)
      c3_glds16(rb, base + D3_PROWS * 64 + (wave + 8 * u) * 1024, (uint32_t)(woff[u] + r * 3 * C * 2) + cb);
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int kq = lane >> 4, lr = lane & 15;
  // fragment byte offsets within a stage: A at tap column shift ds (0..2), B at tap column s
  auto aoff = [&](int i, int ds) {
    const int P = (wm * 4 + i) * C3_PW + lr + ds;
    return P * 64 + ((kq ^ ((P >> 1) & 2)) << 4);
  };
  auto boff = [&](int s, int j) {
    const int P = s * 128 + wn * 64 + j * 16 + lr;
    return D3_PROWS * 64 + P * 64 + ((kq ^ ((P >> 1) & 2)) << 4);
  };
  auto frags = [&](const char* st, int s, bf16x8 (&af)[4], bf16x8 (&bfr)[4]) {
    const int ds = p.flip ? 2 - s : s;
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const bf16x8*>(st + aoff(i, ds));
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(st + boff(s, j));
  };
  auto compute = [&](const char* st) {
    bf16x8 af[2][4], bfr[2][4];
    frags(st, 0, af[0], bfr[0]);
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt(0xc07f);                  // lgkmcnt(0): this tap's fragments
      __builtin_amdgcn_sched_barrier(0);
      if (s + 1 < 3) frags(st, s + 1, af[(s + 1) & 1], bfr[(s + 1) & 1]);
      if constexpr (ACT) {
#pragma unroll
        for (int i = 0; i < 4; ++i) af[s & 1][i] = lrelu8(af[s & 1][i], p.a_slope);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[s & 1][i], bfr[s & 1][j], acc[i][j], 0, 0, 0);
      if (s + 1 < 3) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
      }
    }
  };

  const int nchunks = C / 32;
  const int nst = 3 * nchunks;
  issue(0, 0, 0);
  if (nst > 1) issue(0, 1, 1);
  for (int kc = 0; kc < nchunks; ++kc) {
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int k = 3 * kc + r;
      if (k + 2 < nst) {
        issue(kc + (r + 2) / 3, (r + 2) % 3, (r + 2) % 3);
        asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      } else if (k + 1 < nst) {
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      compute(smem + r * D3_STAGE);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }

  // ---- epilogue through LDS (as c3_kernel): fp32 tile [256 pixels][128 (+4)], 16-byte rows
  constexpr int LDC = C3T<128>::LDC;
  float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        Cs[((wm * 4 + i) * 16 + 4 * (lane >> 4) + e) * LDC + wn * 64 + j * 16 + lr] = acc[i][j][e];
  __syncthreads();
  const rsrc_t rres = make_rsrc(p.residual ? p.residual : p.out, p.residual ? p.o_bytes : 0u);
  const rsrc_t raux = make_rsrc(p.aux ? p.aux : p.out, p.aux ? p.o_bytes : 0u);
  __bf16* out = static_cast<__bf16*>(p.out);
#pragma unroll 2
  for (int k = 0; k < 8; ++k) {
    const int it = tid + 512 * k;
    const int pix = it / 16, cg = (it % 16) * 8;
    const uint32_t o = (uint32_t)((img * 256 + pix) * p.N + n0 + cg);
    uint32_t rs[4], ax[4];
    bload<16>(rres, p.residual ? o * 2u : kOOB, rs);
    bload<16>(raux, p.aux ? o * 2u : kOOB, ax);
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(Cs + pix * LDC + cg);
    const f32x4 v1 = *reinterpret_cast<const f32x4*>(Cs + pix * LDC + cg + 4);
    float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    uint32_t pk[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float g0 = v[2 * e] + __uint_as_float(rs[e] << 16);
      float g1 = v[2 * e + 1] + __uint_as_float(rs[e] & 0xffff0000u);
      if (p.bias) { g0 += p.bias[n0 + cg + 2 * e]; g1 += p.bias[n0 + cg + 2 * e + 1]; }
      if (p.aux) {
        if (!(__uint_as_float(ax[e] << 16) > 0.f)) g0 *= p.aux_slope;
        if (!(__uint_as_float(ax[e] & 0xffff0000u) > 0.f)) g1 *= p.aux_slope;
      }
      bf16x2 h;
      h[0] = (__bf16)g0;
      h[1] = (__bf16)g1;
      pk[e] = *reinterpret_cast<uint32_t*>(&h);
    }
    *reinterpret_cast<uint4*>(out + o) = uint4{pk[0], pk[1], pk[2], pk[3]};
  }
}

// ------------------------------------------------------------------ weight gradient
//   dW[m][r][s][c] += Σ_{n,h,w} U[n,h,w,m] · V'[n, h+r-1, w+s-1, c]     (U = dy, V' = xf(x))
// One workgroup: 128 m x 32 c x all 9 taps over a group of G images.  Per image it stages U
// ([256 pixels][128 m], 288-B rows) and V's 18 x 18 halo patch ([324][32 c], 64-B rows) once, and
// every tap reads its B fragments from the patch at a shifted pixel — the per-tap weight-gradient
// GEMM (vae_wgemm.hpp) gathered V from L2 once per tap.  12 waves (3 per SIMD: 6 left two SIMDs
// with twice the MFMAs of the other two): wave (mq, r) = m rows 32mq..+31 (2 A fragments, reused
// by the 3 taps of its tap row) x the 32 c x taps (r, 0..2): 12 MFMAs per 16 transposed LDS reads
// per 32-pixel K-step.  Operands are [pixel][channel] in LDS; the
// K = pixel direction is read with ds_read_b64_tr_b16 (vae_wgemm.hpp).  Each workgroup writes its
// partial dW tile to slab slice `group` (plain stores); c3w_reduce adds the slices into dW.
typedef __bf16 __attribute__((ext_vector_type(4))) __attribute__((address_space(3))) w3_lds_bf16x4;
typedef __bf16 w3_bf16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ w3_bf16x4 w3_tr_read(const char* generic_lds_addr) {
  const uint32_t off = (uint32_t)(uintptr_t)generic_lds_addr;
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((w3_lds_bf16x4*)(uintptr_t)off);
}

constexpr int W3_NT = 768;
constexpr int W3_BM = 128, W3_BC = 32;
// LDS rows: U 256 B with its 32-byte slots XOR-swizzled by (P & 3) | ((P >> 1) & 4), V 64 B with
// slots swizzled by (P >> 3) & 1: the 32-lane groups of ds_read_b64_tr_b16 read pixel rows
// {0-3, 8-11} (+4) of a block, which then fall in 8 distinct 8-bank windows (a 288-B padded U row
// left rows r and r+8 on the same banks: 42 % of the LDS cycles were conflicts)
constexpr int W3_URS = 256, W3_VRS = 64;                  // LDS row bytes
constexpr int W3_U_BYTES = 256 * W3_URS;                  // 65536
constexpr int W3_V_BYTES = C3_PATCH * W3_VRS;             // 20736
constexpr int W3_UI = 256 * (W3_BM / 8);                  // 16-B chunks of a U tile (4096)
constexpr int W3_VI = C3_PATCH * (W3_BC / 8);             // of a V patch (1296)
constexpr int W3_UP = (W3_UI + W3_NT - 1) / W3_NT;        // 6
constexpr int W3_VP = (W3_VI + W3_NT - 1) / W3_NT;        // 2

// byte offset of 32-byte slot c of LDS row P (U tile / V patch), with the swizzles above
__device__ __forceinline__ int w3_usw(int P, int c) { return P * W3_URS + ((c ^ ((P & 3) | ((P >> 1) & 4))) << 5); }
__device__ __forceinline__ int w3_vsw(int P, int c) { return P * W3_VRS + ((c ^ ((P >> 3) & 1)) << 5); }

struct W3Params {
  const void* u;
  const void* v;
  float* slab;
  long slab_ld;
  uint32_t u_bytes, v_bytes;
  float v_slope;
  int v_act, n, M, J, G;
};

__global__ void __launch_bounds__(W3_NT) c3w_kernel(const W3Params p) {
  kernarg_prefetch<(sizeof(W3Params) < 1024 ? sizeof(W3Params) : 1024)>();
  __shared__ __attribute__((aligned(16))) char smem[W3_U_BYTES + W3_V_BYTES];
  char* const Us = smem;
  char* const Vs = smem + W3_U_BYTES;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int mq = wave / 3, tr = wave - 3 * (wave / 3);   // m rows 32mq..+31, tap row tr
  const int ntc = p.J / W3_BC, per = (p.M / W3_BM) * ntc;
  int tile;
  {
    // XCD-aware order (workgroup b on XCD b % 8): contiguous ranges are image-group major, so
    // the tiles reading the same images share an XCD's L2
    const int nb = (int)gridDim.x, b = (int)blockIdx.x;
    const int q = nb >> 3, r = nb & 7, x = b & 7, loc = b >> 3;
    tile = x * q + min(x, r) + loc;
  }
  const int grp = tile / per, rem = tile - grp * per;
  const int tj = rem / ntc, tc = rem - tj * ntc;
  const int j0 = tj * W3_BM, c0 = tc * W3_BC;
  const int img0 = grp * p.G, img1 = min(p.n, img0 + p.G);
  const rsrc_t ru = make_rsrc(p.u, p.u_bytes);
  const rsrc_t rv = make_rsrc(p.v, p.v_bytes);

  uint32_t ubase[W3_UP], vbase[W3_VP];
  bool vok[W3_VP];
#pragma unroll
  for (int k = 0; k < W3_UP; ++k) {
    const int it = min(tid + W3_NT * k, W3_UI - 1);
    ubase[k] = (uint32_t)(((it >> 4) * p.M + j0 + (it & 15) * 8) * 2);
  }
#pragma unroll
  for (int k = 0; k < W3_VP; ++k) {
    const int it = tid + W3_NT * k;
    const int pix = it >> 2, ph = pix / C3_PW, pw = pix - ph * C3_PW;
    const int h = ph - 1, w = pw - 1;
    vok[k] = it < W3_VI && (unsigned)h < 16u && (unsigned)w < 16u;
    vbase[k] = vok[k] ? (uint32_t)(((h * 16 + w) * p.J + c0 + (it & 3) * 8) * 2) : 0u;
  }
  uint32_t ur[W3_UP][4], vr[W3_VP][4];
  auto load = [&](int img) {
    const uint32_t uo = (uint32_t)img * 256u * (uint32_t)p.M * 2u, vo = (uint32_t)img * 256u * (uint32_t)p.J * 2u;
#pragma unroll
    for (int k = 0; k < W3_UP; ++k) bload<16>(ru, ubase[k] + uo, ur[k]);
#pragma unroll
    for (int k = 0; k < W3_VP; ++k) bload<16>(rv, vok[k] ? vbase[k] + vo : kOOB, vr[k]);
  };
  auto store = [&]() {
#pragma unroll
    for (int k = 0; k < W3_UP; ++k) {
      const int it = tid + W3_NT * k;
      if (it < W3_UI)
        *reinterpret_cast<uint4*>(Us + w3_usw(it >> 4, (it & 15) >> 1) + (it & 1) * 16) = uint4{ur[k][0], ur[k][1], ur[k][2], ur[k][3]};
    }
#pragma unroll
    for (int k = 0; k < W3_VP; ++k) {
      const int it = tid + W3_NT * k;
      if (it < W3_VI) {
        uint4 v = uint4{vr[k][0], vr[k][1], vr[k][2], vr[k][3]};
        if (p.v_act) {
          v.x = lrelu_pk(v.x, p.v_slope); v.y = lrelu_pk(v.y, p.v_slope);
          v.z = lrelu_pk(v.z, p.v_slope); v.w = lrelu_pk(v.w, p.v_slope);
        }
        *reinterpret_cast<uint4*>(Vs + w3_vsw(it >> 2, (it & 3) >> 1) + (it & 1) * 16) = v;
      }
    }
  };

  f32x4 acc[2][2][3];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int s = 0; s < 3; ++s) acc[i][cb][s] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed-read addresses: lane 4q+p of 16-lane group g reads K rows 8g+4h+q, columns 4p..4p+3
  const int g = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  int aoff[2][2], prow[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = 8 * g + 4 * h + q4;                      // pixel within a 32-pixel K block
#pragma unroll
    for (int i = 0; i < 2; ++i) aoff[i][h] = w3_usw(row, mq * 2 + i) + 8 * p4;       // (row & 15 fixed over kb)
    // K block kb = output rows 2kb, 2kb+1; this lane's pixel: output (2kb + (g >> 1), 8(g & 1) + 4h + q)
    // -> patch pixel (2kb + (g >> 1) + r, 8(g & 1) + 4h + q + s)
    prow[h] = ((g >> 1) + tr) * C3_PW + 8 * (g & 1) + 4 * h + q4;
  }
  auto afrag = [&](int kb, bf16x8 (&af)[2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const w3_bf16x4 a0 = w3_tr_read(Us + kb * 32 * W3_URS + aoff[i][0]);
      const w3_bf16x4 a1 = w3_tr_read(Us + kb * 32 * W3_URS + aoff[i][1]);
#pragma unroll
      for (int e = 0; e < 4; ++e) { af[i][e] = a0[e]; af[i][4 + e] = a1[e]; }
    }
  };
  auto bfrag = [&](int kb, int s, bf16x8 (&bfr)[2]) {
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const int P0 = prow[0] + kb * 2 * C3_PW + s, P1 = prow[1] + kb * 2 * C3_PW + s;
      const w3_bf16x4 b0 = w3_tr_read(Vs + w3_vsw(P0, cb) + 8 * p4);
      const w3_bf16x4 b1 = w3_tr_read(Vs + w3_vsw(P1, cb) + 8 * p4);
#pragma unroll
      for (int e = 0; e < 4; ++e) { bfr[cb][e] = b0[e]; bfr[cb][4 + e] = b1[e]; }
    }
  };
  // 24 steps (K block kb, tap column s); the next step's B fragments are read between this step's
  // 8 MFMAs after one wait at the step's head (as c3_kernel); A once per K block
  auto compute = [&]() {
    bf16x8 af[2], bfr[2][2];
    bfrag(0, 0, bfr[0]);
#pragma unroll 1
    for (int kb = 0; kb < 8; ++kb) {
      afrag(kb, af);                                       // (one exposed read per K block)
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        __builtin_amdgcn_sched_barrier(0);                 // (the wait stays between the steps)
        __builtin_amdgcn_s_waitcnt(0xc07f);                // lgkmcnt(0)
        __builtin_amdgcn_sched_barrier(0);
        // next step's B: (kb, s+1), or (kb+1, 0) — past the end a harmless re-read of block 7
        bfrag(s < 2 ? kb : min(kb + 1, 7), s < 2 ? s + 1 : 0, bfr[(s + 1) & 1]);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int cb = 0; cb < 2; ++cb)
            acc[i][cb][s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[s & 1][cb], acc[i][cb][s], 0, 0, 0);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
      }
      // (3 steps per K block: step s = 2 filled bfr[1] for the next block's s = 0 — swap roles)
      bfr[0][0] = bfr[1][0]; bfr[0][1] = bfr[1][1];
    }
  };

  load(img0);
  store();
  __syncthreads();
  for (int img = img0; img < img1; ++img) {
    const bool more = img + 1 < img1;
    load(more ? img + 1 : img);                // (unconditional: see c3_kernel)
    __builtin_amdgcn_sched_barrier(0);
    compute();
    __syncthreads();
    if (more) {
      store();
      __syncthreads();
    }
  }
  // partial tile -> slab slice grp: lane holds rows 4g+e of fragment i (m), column li of fragment cb (c)
  float* part = p.slab + (long)grp * p.slab_ld;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = j0 + mq * 32 + i * 16 + 4 * g + e;
#pragma unroll
      for (int s = 0; s < 3; ++s)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
          part[((long)m * 9 + tr * 3 + s) * p.J + c0 + cb * 16 + li] = acc[i][cb][s][e];
    }
}

// LDS-DMA form of the same weight gradient (c3wd_kernel): a stage is one half image (8 output
// rows = 4 K blocks of 32 pixels) — its U rows [128 pixels][128 m] (32 KB, w3_usw image) and the
// 10 x 18 patch rows of V it reads ([180 (256) pixels][32 c], w3_vsw image) — brought in by
// buffer_load ... lds (the 32-byte-slot swizzles set through the per-lane source address), three
// stages in a ring with two in flight; c3w_kernel staged one whole image through registers and
// LDS stores between the compute phases.  The LeakyReLU of an activated V is applied to the B
// fragments.  Same wave mapping, compute order and slab partials as c3w_kernel.
constexpr int W3D_UROWS = 128, W3D_VROWS = 256;
constexpr int W3D_STAGE = W3D_UROWS * W3_URS + W3D_VROWS * W3_VRS;    // 49152
constexpr int W3D_LDS = 3 * W3D_STAGE;                                 // 147456

// transposed reads as inline asm, waited for explicitly (vae_bgemm.hip bw_tr: the ds_read_tr
// intrinsic makes the wait-count pass drain every LDS-DMA in flight before it)
__device__ __forceinline__ w3_bf16x4 w3d_tr(uint32_t lds_addr) {
  w3_bf16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(lds_addr) : "memory");
  return r;
}

template <int VACT>
__global__ void __launch_bounds__(W3_NT) c3wd_kernel(const W3Params p) {
  kernarg_prefetch<(sizeof(W3Params) < 1024 ? sizeof(W3Params) : 1024)>();
  __shared__ __attribute__((aligned(16))) char smem[W3D_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int mq = wave / 3, tr = wave - 3 * (wave / 3);   // m rows 32mq..+31, tap row tr
  const int ntc = p.J / W3_BC, per = (p.M / W3_BM) * ntc;
  int tile;
  {
    const int nb = (int)gridDim.x, b = (int)blockIdx.x;
    const int q = nb >> 3, r = nb & 7, x = b & 7, loc = b >> 3;
    tile = x * q + min(x, r) + loc;
  }
  const int grp = tile / per, rem = tile - grp * per;
  const int tj = rem / ntc, tc = rem - tj * ntc;
  const int j0 = tj * W3_BM, c0 = tc * W3_BC;
  const int img0 = grp * p.G, img1 = min(p.n, img0 + p.G);
  const rsrc_t ru = make_rsrc(p.u, p.u_bytes);
  const rsrc_t rv = make_rsrc(p.v, p.v_bytes);

  // this wave's 4 DMA instructions per stage: I = wave + 12 u (0..47); I < 32: U rows 4I..4I+3
  // (16 chunks of 16 B per row), else V patch rows 16 (I - 32) .. +15 (4 chunks per row)
  uint32_t goff[4];
  int vph[4];
  bool vok0[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int I = wave + 12 * u;
    if (I < 32) {                                       // (wave-uniform)
      const int P = 4 * I + (lane >> 4), sl = lane & 15;
      const int c16 = ((((sl >> 1) ^ ((P & 3) | ((P >> 1) & 4)))) << 1) | (sl & 1);
      goff[u] = (uint32_t)((P * p.M + j0 + c16 * 8) * 2);          // + image / half offset per stage
      vph[u] = 0;
      vok0[u] = true;
    } else {
      const int P = 16 * (I - 32) + (lane >> 2), sl = lane & 3;
      const int c16 = ((((sl >> 1) ^ ((P >> 3) & 1))) << 1) | (sl & 1);
      const int ph = P / C3_PW, pw = P - ph * C3_PW;
      vph[u] = P < 180 ? ph : 99;                                  // patch row (image row 8hh + ph - 1)
      vok0[u] = (unsigned)(pw - 1) < 16u;
      goff[u] = (uint32_t)((((ph - 1) * 16 + (pw - 1)) * p.J + c0 + c16 * 8) * 2);   // at hh = 0 (wraps: masked)
    }
  }
  // stage (image img, half hh) -> buffer b
  auto issue = [&](int img, int hh, int b) {
    char* base = smem + b * W3D_STAGE;
    const uint32_t uo = (uint32_t)(img * 256 + hh * 128) * (uint32_t)p.M * 2u;
    const uint32_t vo = (uint32_t)(img * 256 + hh * 128) * (uint32_t)p.J * 2u;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int I = wave + 12 * u;
      if (I < 32) {
        c3_glds16(ru, base + I * 1024, goff[u] + uo);
      } else {
        const bool ok = vok0[u] && (unsigned)(8 * hh + vph[u] - 1) < 16u;
        c3_glds16(rv, base + W3D_UROWS * W3_URS + (I - 32) * 1024, ok ? goff[u] + vo : kOOB);
      }
    }
  };

  f32x4 acc[2][2][3];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int s = 0; s < 3; ++s) acc[i][cb][s] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  int aoff[2][2], prow[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = 8 * g + 4 * h + q4;
#pragma unroll
    for (int i = 0; i < 2; ++i) aoff[i][h] = w3_usw(row, mq * 2 + i) + 8 * p4;
    prow[h] = ((g >> 1) + tr) * C3_PW + 8 * (g & 1) + 4 * h + q4;
  }
  auto compute = [&](uint32_t Us) {
    const uint32_t Vs = Us + W3D_UROWS * W3_URS;
    // raw read results, consumed only after a wait that takes these very registers (vae_bgemm.hip
    // bw_tr: waiting on packed copies let the packing moves race the LDS returns)
    w3_bf16x4 ra[2][2], rb[3][2][2];                      // A [i][half]; B [step buffer][cb][half]
    auto afrag = [&](int kb) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        ra[i][0] = w3d_tr(Us + kb * 32 * W3_URS + aoff[i][0]);
        ra[i][1] = w3d_tr(Us + kb * 32 * W3_URS + aoff[i][1]);
      }
    };
    auto bfrag = [&](int kb, int s, w3_bf16x4 (&r)[2][2]) {
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int P0 = prow[0] + kb * 2 * C3_PW + s, P1 = prow[1] + kb * 2 * C3_PW + s;
        r[cb][0] = w3d_tr(Vs + w3_vsw(P0, cb) + 8 * p4);
        r[cb][1] = w3d_tr(Vs + w3_vsw(P1, cb) + 8 * p4);
      }
    };
    bfrag(0, 0, rb[0]);
#pragma unroll 1
    for (int kb = 0; kb < 4; ++kb) {
      afrag(kb);
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        // this step's fragments have landed (the wait takes the raw registers: no consumer above it)
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(ra[0][0]), "+v"(ra[0][1]), "+v"(ra[1][0]), "+v"(ra[1][1]), "+v"(rb[s][0][0]),
                       "+v"(rb[s][0][1]), "+v"(rb[s][1][0]), "+v"(rb[s][1][1])::"memory");
        // the next step's B fragments: steps 0, 1, 2 of a kb use buffers 0, 1, 2 (the next kb's
        // step 0 goes to buffer 0, whose step is done)
        bfrag(s < 2 ? kb : min(kb + 1, 3), s < 2 ? s + 1 : 0, rb[(s + 1) % 3]);
        bf16x8 af[2], bfr[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = __builtin_shufflevector(ra[i][0], ra[i][1], 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          bfr[cb] = __builtin_shufflevector(rb[s][cb][0], rb[s][cb][1], 0, 1, 2, 3, 4, 5, 6, 7);
          if constexpr (VACT) bfr[cb] = lrelu8(bfr[cb], p.v_slope);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int cb = 0; cb < 2; ++cb)
            acc[i][cb][s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[cb], acc[i][cb][s], 0, 0, 0);
      }
    }
  };

  const int nst = 2 * (img1 - img0);
  issue(img0, 0, 0);
  if (nst > 1) issue(img0, 1, 1);
  for (int k = 0; k < nst; ++k) {
    const int b = k % 3;
    if (k + 2 < nst) {
      issue(img0 + ((k + 2) >> 1), (k + 2) & 1, (k + 2) % 3);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else if (k + 1 < nst) {
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    compute((uint32_t)(uintptr_t)smem + b * W3D_STAGE);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  float* part = p.slab + (long)grp * p.slab_ld;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = j0 + mq * 32 + i * 16 + 4 * g + e;
#pragma unroll
      for (int s = 0; s < 3; ++s)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
          part[((long)m * 9 + tr * 3 + s) * p.J + c0 + cb * 16 + li] = acc[i][cb][s][e];
    }
}

// dw[i] += Σ_s slab[s * ld + i] (each element one writer), 4 consecutive floats per thread
__global__ void __launch_bounds__(256) c3w_reduce(const float* slab, long ld, int slices, long cols, float* dw) {
  const long i = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= cols) return;
  // 8 slice loads in flight per thread (a plain loop waited for each one: 16-64 dependent HBM
  // round trips per thread, 18.7 us average per call in the VQ-VAE step)
  f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
  int k = 0;
  for (; k + 8 <= slices; k += 8) {
    f32x4 t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(slab + (long)(k + u) * ld + i));
#pragma unroll
    for (int u = 0; u < 8; ++u) s += t[u];
  }
  for (; k < slices; ++k) s += *reinterpret_cast<const f32x4*>(slab + (long)k * ld + i);
  f32x4 d;
  d[0] = dw[i]; d[1] = dw[i + 1]; d[2] = dw[i + 2]; d[3] = dw[i + 3];     // (parameter slices: 4-B aligned)
  d += s;
  dw[i] = d[0]; dw[i + 1] = d[1]; dw[i + 2] = d[2]; dw[i + 3] = d[3];
}

// 1x1 (pointwise) weight gradient on the same grid (the ResidualLayer's Conv1x1, vq_vae.py:64-68):
//   dW[m][c] += Σ_pix U[pix][m] · V'[pix][c]
// One workgroup: 128 m x 128 c over G images (both operands staged per image as [pixel][channel]
// 256-B rows, swizzled as c3w's U); 8 waves of 64 m x 32 c; partials to slab slice `group`.
constexpr int W1_NT = 512;
constexpr int W1_T = 128;
constexpr int W1_LP = 256 * (W1_T / 8) / W1_NT;            // 16-B loads per thread per operand (8)

struct W1Params {
  const void* u;
  const void* v;
  float* slab;
  long slab_ld;
  uint32_t u_bytes, v_bytes;
  float v_slope;
  int v_act, n, M, J, G;
};

__global__ void __launch_bounds__(W1_NT) c1w_kernel(const W1Params p) {
  kernarg_prefetch<(sizeof(W1Params) < 1024 ? sizeof(W1Params) : 1024)>();
  __shared__ __attribute__((aligned(16))) char smem[2 * 256 * W3_URS];
  char* const Us = smem;
  char* const Vs = smem + 256 * W3_URS;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wc = wave >> 1;
  const int ntc = p.J / W1_T, per = (p.M / W1_T) * ntc;
  int tile;
  {
    const int nb = (int)gridDim.x, b = (int)blockIdx.x;
    const int q = nb >> 3, r = nb & 7, x = b & 7, loc = b >> 3;
    tile = x * q + min(x, r) + loc;
  }
  const int grp = tile / per, rem = tile - grp * per;
  const int tm = rem / ntc, tc = rem - tm * ntc;
  const int m0 = tm * W1_T, c0 = tc * W1_T;
  const int img0 = grp * p.G, img1 = min(p.n, img0 + p.G);
  const rsrc_t ru = make_rsrc(p.u, p.u_bytes);
  const rsrc_t rv = make_rsrc(p.v, p.v_bytes);
  uint32_t ur[W1_LP][4], vr[W1_LP][4];
  auto load = [&](int img) {
#pragma unroll
    for (int k = 0; k < W1_LP; ++k) {
      const int it = tid + W1_NT * k;
      const uint32_t pix = (uint32_t)img * 256u + (uint32_t)(it >> 4);
      bload<16>(ru, (pix * (uint32_t)p.M + (uint32_t)(m0 + (it & 15) * 8)) * 2u, ur[k]);
      bload<16>(rv, (pix * (uint32_t)p.J + (uint32_t)(c0 + (it & 15) * 8)) * 2u, vr[k]);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int k = 0; k < W1_LP; ++k) {
      const int it = tid + W1_NT * k;
      const int off = w3_usw(it >> 4, (it & 15) >> 1) + (it & 1) * 16;
      *reinterpret_cast<uint4*>(Us + off) = uint4{ur[k][0], ur[k][1], ur[k][2], ur[k][3]};
      uint4 v = uint4{vr[k][0], vr[k][1], vr[k][2], vr[k][3]};
      if (p.v_act) {
        v.x = lrelu_pk(v.x, p.v_slope); v.y = lrelu_pk(v.y, p.v_slope);
        v.z = lrelu_pk(v.z, p.v_slope); v.w = lrelu_pk(v.w, p.v_slope);
      }
      *reinterpret_cast<uint4*>(Vs + off) = v;
    }
  };
  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) acc[i][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  int aoff[4][2], boff[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = 8 * g + 4 * h + q4;
#pragma unroll
    for (int i = 0; i < 4; ++i) aoff[i][h] = w3_usw(row, wm * 4 + i) + 8 * p4;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) boff[cb][h] = w3_usw(row, wc * 2 + cb) + 8 * p4;
  }
  auto compute = [&]() {
#pragma unroll 2
    for (int kb = 0; kb < 8; ++kb) {
      bf16x8 af[4], bfr[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const w3_bf16x4 a0 = w3_tr_read(Us + kb * 32 * W3_URS + aoff[i][0]);
        const w3_bf16x4 a1 = w3_tr_read(Us + kb * 32 * W3_URS + aoff[i][1]);
#pragma unroll
        for (int e = 0; e < 4; ++e) { af[i][e] = a0[e]; af[i][4 + e] = a1[e]; }
      }
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const w3_bf16x4 b0 = w3_tr_read(Vs + kb * 32 * W3_URS + boff[cb][0]);
        const w3_bf16x4 b1 = w3_tr_read(Vs + kb * 32 * W3_URS + boff[cb][1]);
#pragma unroll
        for (int e = 0; e < 4; ++e) { bfr[cb][e] = b0[e]; bfr[cb][4 + e] = b1[e]; }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) acc[i][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[cb], acc[i][cb], 0, 0, 0);
    }
  };
  load(img0);
  store();
  __syncthreads();
  for (int img = img0; img < img1; ++img) {
    const bool more = img + 1 < img1;
    load(more ? img + 1 : img);
    __builtin_amdgcn_sched_barrier(0);
    compute();
    __syncthreads();
    if (more) {
      store();
      __syncthreads();
    }
  }
  float* part = p.slab + (long)grp * p.slab_ld;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = m0 + wm * 64 + i * 16 + 4 * g + e;
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) part[(long)m * p.J + c0 + wc * 32 + cb * 16 + li] = acc[i][cb][e];
    }
}

inline void c1w_plan(int n, int M, int J, int* G, int* groups) {
  const int tiles = (M / W1_T) * (J / W1_T);
  int ng = 256 / tiles;
  if (ng < 1) ng = 1;
  if (ng > n) ng = n;
  *G = (n + ng - 1) / ng;
  *groups = (n + *G - 1) / *G;
}

inline void c3w_plan(int n, int M, int J, int* G, int* groups) {
  const int tiles = (M / W3_BM) * (J / W3_BC);
  int ng = 256 / tiles;
  if (ng < 1) ng = 1;
  if (ng > n) ng = n;
  *G = (n + ng - 1) / ng;
  *groups = (n + *G - 1) / *G;
}

inline bool al16(const void* ptr) { return ((uintptr_t)ptr & 15u) == 0; }

}  // namespace

bool c3_enabled() { return true; }

bool c3_shape_ok(int n, int h, int w, int p, int q, int r, int stride, int pad, int C, int N) {
  return n > 0 && h == 16 && w == 16 && p == 16 && q == 16 && r == 3 && stride == 1 && pad == 1 && C % 32 == 0 &&
         C >= 32 && N % 128 == 0 && N > 0 && (long)n * 256 * (C > N ? C : N) * 2 < (1l << 31);
}

int c3_launch(const C3Args& a, hipStream_t st) {
  if (!c3_shape_ok(a.n, 16, 16, 16, 16, 3, 1, 1, a.C, a.N)) return fail(VAE_E_BADSHAPE, "c3: shape");
  if (!al16(a.a) || !al16(a.b) || !al16(a.out) || (a.residual && !al16(a.residual)) || (a.aux && !al16(a.aux)))
    return fail(VAE_E_BADARG, "c3: tensors must be 16-byte aligned");
  C3Params p;
  p.a = a.a; p.b = a.b; p.out = a.out; p.bias = a.bias; p.residual = a.residual; p.aux = a.aux;
  p.a_bytes = (uint32_t)((long)a.n * 256 * a.C * 2);
  p.b_bytes = (uint32_t)((long)a.N * 9 * a.C * 2);
  p.o_bytes = (uint32_t)((long)a.n * 256 * a.N * 2);
  p.a_slope = a.a_slope; p.aux_slope = a.aux_slope;
  p.a_act = a.a_act; p.flip = a.flip; p.C = a.C; p.N = a.N;
  p.dbg = 0;
  const unsigned grid = (unsigned)(a.n * (a.N / 128));
  // An activated input (LeakyReLU of the stored tensor) stays on the register-staged kernel, which
  // applies it once per element as it stages the patch (the LDS-DMA kernel would apply it to the A
  // fragments once per element and tap: 66-71 vs 35 us per call at B=128,
  // profiles/r4_v3_vq_breakdown.txt); untransformed inputs take the LDS-DMA kernel
  if (!a.a_act) VAE_LAUNCH(c3d_kernel<0>, dim3(grid), dim3(512), 0, st, p);
  else VAE_LAUNCH(c3_kernel<128>, dim3(grid), dim3(512), 0, st, p);
  return check_launch("c3");
}

}  // namespace vae

namespace vae {

bool c3w_shape_ok(int n, int h, int w, int p, int q, int r, int stride, int pad, int M, int J) {
  return n > 0 && h == 16 && w == 16 && p == 16 && q == 16 && r == 3 && stride == 1 && pad == 1 && M % W3_BM == 0 &&
         J % W3_BC == 0 && (long)n * 256 * (M > J ? M : J) * 2 < (1l << 31);
}

long c3w_workspace(int n, int M, int J) {
  int G, groups;
  c3w_plan(n, M, J, &G, &groups);
  return (long)groups * M * 9 * J * 4;
}

int c3w_launch(const C3WArgs& a, void* ws, long ws_bytes, hipStream_t st) {
  if (!c3w_shape_ok(a.n, 16, 16, 16, 16, 3, 1, 1, a.M, a.J)) return fail(VAE_E_BADSHAPE, "c3w: shape");
  if (!al16(a.u) || !al16(a.v) || ((uintptr_t)a.dw & 3u)) return fail(VAE_E_BADARG, "c3w: alignment");
  W3Params p;
  int groups;
  c3w_plan(a.n, a.M, a.J, &p.G, &groups);
  const long cols = (long)a.M * 9 * a.J;
  if (!ws_fits((long)groups * cols * 4, ws ? ws_bytes : 0, "c3w slab")) return VAE_E_BADARG;
  p.u = a.u; p.v = a.v; p.slab = static_cast<float*>(ws); p.slab_ld = cols;
  p.u_bytes = (uint32_t)((long)a.n * 256 * a.M * 2);
  p.v_bytes = (uint32_t)((long)a.n * 256 * a.J * 2);
  p.v_act = a.v_act; p.v_slope = a.v_slope;
  p.n = a.n; p.M = a.M; p.J = a.J;
  const unsigned grid = (unsigned)(groups * (a.M / W3_BM) * (a.J / W3_BC));
  // (an activated V operand: the register-staged kernel, as c3_launch — the LDS-DMA kernel took
  // 114-131 vs 50 us per call)
  if (a.v_act) VAE_LAUNCH(c3w_kernel, dim3(grid), dim3(W3_NT), 0, st, p);
  else VAE_LAUNCH(c3wd_kernel<0>, dim3(grid), dim3(W3_NT), 0, st, p);
  if (int rc = check_launch("c3w")) return rc;
  VAE_LAUNCH(c3w_reduce, dim3((unsigned)((cols / 4 + 255) / 256)), dim3(256), 0, st, (const float*)p.slab, cols, groups,
             cols, a.dw);
  return check_launch("c3w_reduce");
}

}  // namespace vae

namespace vae {

bool c1w_shape_ok(int n, int h, int w, int p, int q, int r, int stride, int pad, int M, int J) {
  return n > 0 && h == 16 && w == 16 && p == 16 && q == 16 && r == 1 && stride == 1 && pad == 0 && M % W1_T == 0 &&
         J % W1_T == 0 && (long)n * 256 * (M > J ? M : J) * 2 < (1l << 31);
}

int c1w_launch(const C3WArgs& a, void* ws, long ws_bytes, hipStream_t st) {
  if (!c1w_shape_ok(a.n, 16, 16, 16, 16, 1, 1, 0, a.M, a.J)) return fail(VAE_E_BADSHAPE, "c1w: shape");
  if (!al16(a.u) || !al16(a.v) || ((uintptr_t)a.dw & 3u)) return fail(VAE_E_BADARG, "c1w: alignment");
  W1Params p;
  int groups;
  c1w_plan(a.n, a.M, a.J, &p.G, &groups);
  const long cols = (long)a.M * a.J;
  if (!ws_fits((long)groups * cols * 4, ws ? ws_bytes : 0, "c1w slab")) return VAE_E_BADARG;
  p.u = a.u; p.v = a.v; p.slab = static_cast<float*>(ws); p.slab_ld = cols;
  p.u_bytes = (uint32_t)((long)a.n * 256 * a.M * 2);
  p.v_bytes = (uint32_t)((long)a.n * 256 * a.J * 2);
  p.v_act = a.v_act; p.v_slope = a.v_slope;
  p.n = a.n; p.M = a.M; p.J = a.J;
  const unsigned grid = (unsigned)(groups * (a.M / W1_T) * (a.J / W1_T));
  VAE_LAUNCH(c1w_kernel, dim3(grid), dim3(W1_NT), 0, st, p);
  if (int rc = check_launch("c1w")) return rc;
  VAE_LAUNCH(c3w_reduce, dim3((unsigned)((cols / 4 + 255) / 256)), dim3(256), 0, st, (const float*)p.slab, cols, groups,
             cols, a.dw);
  return check_launch("c3w_reduce");
}

}  // namespace vae
