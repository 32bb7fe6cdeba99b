// Decoder head on MFMA (bf16 throughput mode): final_layer Conv2d(C->3, k3, s1, p1) + Tanh
// (models/vanilla_vae.py:73-75, models/autoencoder.py:84-86), the reconstruction SSE of the ELBO
// (vanilla_vae.py:140) and their backward, for C = 32 (the VAEs), 64 and 128 (the Autoencoder's
// big_ae final layer, configs/big_ae.yaml).
//
// The layer has 3 output channels: as a GEMM over pixels its N is 3, so the forward pads N to
// the 16 of one v_mfma_f32_16x16x32_bf16 (13/16 of the MFMA is wasted, and the MFMA is still far
// from being the limit).  Everything is organised around one LDS tile per workgroup: ROWS image
// rows x 64 columns (+1 halo on every side) x C channels of act = lrelu(BN(y)), bf16, staged once
// per element (the conv-GEMM route gathered every input element 9 times through L2: big_ae's
// head at C = 128 took 112 us forward and 89 us data gradient that way), with the 16-byte channel
// chunks of a pixel XOR-swizzled by the column so that 16 lanes reading 16 consecutive pixels
// hit different bank slots.  ROWS = 4 (C <= 64) or 2 (C = 128: the backward's tile, raw-y copy
// and output staging then fit one CU's LDS).
//
//   forward : 16 pixels x 16 (3 real) outputs, K = 9 taps x C channels (9 C/32 MFMAs);
//             epilogue tanh -> recon (NCHW fp32, float4 stores), (recon - x)^2 -> SSE.
//   backward: one persistent kernel, per tile
//     data   dact[p][c] = sum_{tap,co} gseed[p + 1 - tap][co] W[co][tap][c]: K = 9 taps x 4 (3 co
//            + pad) = 36 -> 2 k-steps, N = C channels; epilogue g = dact * lrelu'(z) (z = BN(y)),
//            BatchNorm-backward sums (sum g, sum g*xhat) and g stored through LDS as whole rows;
//     filter dW[co][tap][c] = sum_p gseed[p][co] act[p + tap - 1][c]: M = co (pad 16), N = 9 C,
//            K = the tile's own pixels; the act operand is read transposed (ds_read_b64_tr_b16)
//            from the same LDS tile; per-block partials go to a slab summed by vae_reduce_rows
//            (fixed order: deterministic, and no same-address atomics).
// Tiles are dealt XCD-aware (workgroup b runs on XCD b % 8): the workgroups one XCD runs at once
// take consecutive tiles, so a tile's halo rows are its neighbours' own rows in the same L2.
#include <stdlib.h>

#include "vae_common.hpp"
#include "vae_elbo.hpp"

namespace vae {
namespace {

constexpr int HW = 64;                 // image width (one tile row)
constexpr int NCO = 3;

// HC: channels one workgroup stages (its LDS tile, fragments); ROWS: image rows per tile
template <int HC, int ROWS_>
struct HT {
  static constexpr int ROWS = ROWS_;
  static constexpr int TR = ROWS + 2, TCOLS = HW + 2, TPIX = TR * TCOLS;   // tile with halo
  static constexpr int CH = HC / 8;                    // 16-byte channel chunks per pixel
  static constexpr int SW = CH >= 8 ? 7 : CH - 1;      // chunk XOR-swizzle mask
  static constexpr int OCT = TPIX * CH;                // 16-byte octets in the act tile
  static constexpr int OCT_PER_T = (OCT + 255) / 256;
  static constexpr int OWN = ROWS * HW;                // pixels a tile produces
  static constexpr int GPW = OWN / 64;                 // 16-pixel groups per wave
  static constexpr int CC = HC / 32;                   // forward K-steps per tap
  static constexpr int NF = HC / 16;                   // data-gradient n-frags (16 channels)
  static constexpr int NFR = 9 * NF;                   // weight-gradient n-frags over (tap, c)
  static constexpr int NFW = (NFR + 3) / 4;            // ... per wave
  static constexpr int NW = NCO * 9 * HC;              // weight-gradient entries
  static constexpr int SLAB_COLS = NW + NCO;           // + 3 bias-gradient entries
};

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr uint32_t kOOB = 0x80000000u;

struct HeadQ {
  int n, h, samples, tiles, xcd;
  const __bf16* x; vae_xform xf;       // fin (pre-BN), its BatchNorm+LeakyReLU
  const float* wt; const float* bias;  // [3][3][3][C] fp32 native, [3]
  const float* target; float* recon; float* sse;
  const float* coef; const float* grad_recon;
  float hc;                            // coef == NULL: the constant dL/d(sse_i) of a fused ELBO
  __bf16* dx; float* dgamma; float* dbeta; int sum_reps, sum_rstride;
  float* slab;                         // [grid][27 C + 3] filter partials, or NULL: atomics into dw/db
  float* dw; float* db;
  int data, filter;
};

__device__ __forceinline__ rsrc_t rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

// byte offset of (tile pixel, 16-byte channel chunk) in the act tile
template <int HC>
__device__ __forceinline__ int act_off(int trow, int tcol, int chunk) {
  constexpr int SW = HC / 8 >= 8 ? 7 : HC / 8 - 1;
  return (trow * (HW + 2) + tcol) * (HC * 2) + ((chunk ^ (tcol & SW)) << 4);
}

// XCD-aware order (a permutation of [0, nb)): the nb / 8 workgroups of XCD x = b % 8 take one
// contiguous range of positions
__device__ __forceinline__ int head_xcd_order(int b, int nb) {
  const int q = nb >> 3, r = nb & 7, x = b & 7, loc = b >> 3;
  return x * q + min(x, r) + loc;
}

__device__ __forceinline__ float bf2f(uint32_t bits16) { return __uint_as_float(bits16 << 16); }

// Per-channel BN coefficients in LDS (from vae_bn_finalize's table when present).
// Without a precomputed table the workgroup reduces the producer's replicated statistics itself
// (tab_build; `update_running`: this workgroup also applies the running-statistic update).
// Channels [cb0, cb0 + HC) of a CT-channel input (CT > HC: a channel slice of the backward).
template <int HC, int CT>
__device__ void head_tables(const vae_xform& xf, float* ta, float* tb, float* tp, float* tq, int cb0,
                            bool update_running = false) {
  if constexpr (CT == HC) {
    if (xf.kind == VAE_X_BN_ACT && !xf.table && xf.channels == HC && bn_fast_ok(xf)) {
      tab_build(xf, Tab{ta, tb, nullptr, tp, tq}, true, update_running);
      return;
    }
  }
  for (int c = threadIdx.x; c < HC; c += blockDim.x) {
    const int cg = cb0 + c;
    if (xf.kind != VAE_X_BN_ACT) { ta[c] = 1.f; tb[c] = 0.f; tp[c] = 0.f; tq[c] = 0.f; continue; }
    if (xf.table) {
      ta[c] = xf.table[cg]; tb[c] = xf.table[CT + cg]; tp[c] = xf.table[2 * CT + cg]; tq[c] = xf.table[3 * CT + cg];
    } else {
      float mean, invstd, var;
      bn_moments(xf, cg, mean, invstd, var);
      ta[c] = xf.gamma[cg] * invstd; tb[c] = xf.beta[cg] - mean * ta[c];
      tp[c] = invstd; tq[c] = -mean * invstd;
      if (update_running && xf.running_mean) {     // (C = 128: 32 statistic replicas, no tab_build)
        const float m = xf.momentum;
        const float unb = xf.count > 1.f ? var * xf.count / (xf.count - 1.f) : var;
        xf.running_mean[cg] = (1.f - m) * xf.running_mean[cg] + m * mean;
        xf.running_var[cg] = (1.f - m) * xf.running_var[cg] + m * unb;
      }
    }
  }
}

// Raw y octets of the tile (halo included) -> registers; issued together (out of image: 0).
template <int HC, int ROWS, int CT>
__device__ __forceinline__ void tile_load(const HeadQ& q, rsrc_t ry, int n, int h0, int cb0,
                                          u32x4 (&raw)[HT<HC, ROWS>::OCT_PER_T]) {
  using T = HT<HC, ROWS>;
#pragma unroll
  for (int j = 0; j < T::OCT_PER_T; ++j) {
    const int o = threadIdx.x + 256 * j;
    const int pix = o / T::CH, ch = o % T::CH;
    const int trow = pix / T::TCOLS, tcol = pix - trow * T::TCOLS;
    const int hi = h0 + trow - 1, wi = tcol - 1;
    const bool ok = o < T::OCT && hi >= 0 && hi < q.h && wi >= 0 && wi < HW;
    const uint32_t off = ok ? (uint32_t)((((n * q.h + hi) * HW + wi) * CT + cb0 + ch * 8) * 2) : kOOB;
    raw[j] = __builtin_amdgcn_raw_buffer_load_b128(ry, off, 0, 0);
  }
}

// act = lrelu(a*y + b) (0 outside the image) -> bf16 tile in LDS
template <int HC, int ROWS>
__device__ __forceinline__ void tile_store(const HeadQ& q, int h0, const u32x4 (&raw)[HT<HC, ROWS>::OCT_PER_T], char* tile,
                                           const float* ta, const float* tb) {
  using T = HT<HC, ROWS>;
#pragma unroll
  for (int j = 0; j < T::OCT_PER_T; ++j) {
    const int o = threadIdx.x + 256 * j;
    if (o >= T::OCT) continue;
    const int pix = o / T::CH, ch = o % T::CH;
    const int trow = pix / T::TCOLS, tcol = pix - trow * T::TCOLS;
    const int hi = h0 + trow - 1, wi = tcol - 1;
    const bool ok = hi >= 0 && hi < q.h && wi >= 0 && wi < HW;
    u32x4 out;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c0 = ch * 8 + 2 * e;
      float lo = bf2f(raw[j][e] & 0xffffu), hi2 = bf2f(raw[j][e] >> 16);
      lo = fmaf(lo, ta[c0], tb[c0]);
      hi2 = fmaf(hi2, ta[c0 + 1], tb[c0 + 1]);
      if (q.xf.kind != VAE_X_NONE) { lo = fmaxf(lo, lo * q.xf.slope); hi2 = fmaxf(hi2, hi2 * q.xf.slope); }
      lo = ok ? lo : 0.f;
      hi2 = ok ? hi2 : 0.f;
      bf16x2 pk; pk[0] = (__bf16)lo; pk[1] = (__bf16)hi2;
      out[e] = *reinterpret_cast<uint32_t*>(&pk);
    }
    *reinterpret_cast<u32x4*>(tile + act_off<HC>(trow, tcol, ch)) = out;
  }
}

// ======================================================================= forward
// One tile per workgroup (C <= 64: 1024 tiles at B = 64, all resident at once).
template <int HC, int ROWS>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) head_fwd_mfma(HeadQ q) {
  kernarg_prefetch<(sizeof(HeadQ) < 1024 ? sizeof(HeadQ) : 1024)>();
  using T = HT<HC, ROWS>;
  __shared__ __attribute__((aligned(16))) char tile[T::TPIX * HC * 2];
  __shared__ float ta[HC], tb[HC], tp[HC], tq[HC];
  __shared__ float red[4];
  __shared__ __attribute__((aligned(16))) __bf16 wsb[T::NW];         // W[co][tap][c] as bf16
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tiles_per_img = q.h / T::ROWS;
  const int ti = q.xcd ? head_xcd_order((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
  const int n = ti / tiles_per_img, h0 = (ti - n * tiles_per_img) * T::ROWS;
  const rsrc_t ry = rsrc(q.x, (uint32_t)((long)q.n * q.h * HW * HC * 2));
  u32x4 raw[T::OCT_PER_T];
  tile_load<HC, ROWS, HC>(q, ry, n, h0, 0, raw);
  const int co = lane & 15, g = lane >> 4;
  // the epilogue's target pixels, in flight with the tile (no global load after the MFMAs)
  f32x4v tgv[T::GPW];
#pragma unroll
  for (int gi = 0; gi < T::GPW; ++gi) {
    const int grp = wave * T::GPW + gi, row = grp >> 2, c0 = (grp & 3) * 16;
    tgv[gi] = co < NCO ? *reinterpret_cast<const f32x4v*>(q.target + (((long)(n / q.samples) * NCO + co) * q.h + h0 + row) * HW +
                                                         c0 + 4 * g)
                       : f32x4v{0.f, 0.f, 0.f, 0.f};
  }
  // the weights: one coalesced pass into LDS (per-lane scattered scalar loads of the fragments
  // cost ~72 vector-memory instructions per wave at C = 32)
  for (int i = threadIdx.x; i < T::NW; i += 256) wsb[i] = (__bf16)q.wt[i];
  const float bco = co < NCO ? q.bias[co] : 0.f;
  head_tables<HC, HC>(q.xf, ta, tb, tp, tq, 0, blockIdx.x == 0);
  __syncthreads();
  tile_store<HC, ROWS>(q, h0, raw, tile, ta, tb);
  // B fragment of (tap t, K-step cc): W[co = lane&15][t][32 cc + 8 (lane>>4) .. +7] (zero for co >= 3);
  // held in registers while they fit (C <= 64), read from LDS per K-step otherwise
  constexpr int KS = 9 * T::CC;
  constexpr bool BREG = KS <= 18;
  const bf16x8 bz = {};
  bf16x8 bw[BREG ? KS : 1];
  if constexpr (BREG) {
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const int t = k / T::CC, cc = k - t * T::CC;
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(&wsb[((co < NCO ? co : 0) * 9 + t) * HC + 32 * cc + 8 * g]);
      bw[k] = co < NCO ? v : bz;
    }
  }
  __syncthreads();
  float sq = 0.f;
#pragma unroll
  for (int gi = 0; gi < T::GPW; ++gi) {
    const int grp = wave * T::GPW + gi;             // groups of 16 pixels, 4 per image row
    const int row = grp >> 2, c0 = (grp & 3) * 16;
    f32x4v acc = {0.f, 0.f, 0.f, 0.f};
    const f32x4v tg = tgv[gi];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int r = t / 3, s = t - 3 * (t / 3);
#pragma unroll
      for (int cc = 0; cc < T::CC; ++cc) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(tile + act_off<HC>(row + r, c0 + (lane & 15) + s, g + 4 * cc));
        bf16x8 b;
        if constexpr (BREG) {
          b = bw[t * T::CC + cc];
        } else {
          const bf16x8 v = *reinterpret_cast<const bf16x8*>(&wsb[((co < NCO ? co : 0) * 9 + t) * HC + 32 * cc + 8 * g]);
          b = co < NCO ? v : bz;
        }
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
      }
    }
    // lane: output channel co, pixels c0 + 4g + i
    if (co < NCO) {
      const int hh = h0 + row, w0 = c0 + 4 * g;
      f32x4v y;
#pragma unroll
      for (int i = 0; i < 4; ++i) y[i] = tanhf(acc[i] + bco);
      *reinterpret_cast<f32x4v*>(q.recon + (((long)n * NCO + co) * q.h + hh) * HW + w0) = y;
#pragma unroll
      for (int i = 0; i < 4; ++i) { const float d = y[i] - tg[i]; sq = fmaf(d, d, sq); }
    }
  }
  for (int off = 32; off > 0; off >>= 1) sq += __shfl_xor(sq, off);
  if (lane == 0) red[wave] = sq;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(q.sse + n, (red[0] + red[1]) + (red[2] + red[3]));
}

// C = 128: the taps move into N.  With the 3 outputs as N (the C <= 64 kernel) every MFMA used 3
// of its 16 columns and every act element was read from LDS once per tap: 9 x 1 KB of A operand
// per 16 pixels and 32 channels, LDS-bandwidth-bound at C = 128 (52 us at B = 64).  Here
// out[p][co*9 + t] = sum_c act[p][c] W[co][t][c] runs over every tile pixel p (halo included):
// N = 27 of 32 columns, K = C, each act element read once; then y[o][co] = sum_t out[o + d_t][co*9+t]
// gathers the 9 shifted partial sums from LDS (fp32) before tanh / recon / SSE.
// Grid-stride over tiles (tile_i = k * gridDim.x + XCD-ordered position), two workgroups per CU,
// the next tile's raw y loaded while the current one computes.
template <int HC, int ROWS>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) head_fwd_stream(HeadQ q) {
  kernarg_prefetch<(sizeof(HeadQ) < 1024 ? sizeof(HeadQ) : 1024)>();
  using T = HT<HC, ROWS>;
  constexpr int NPG = (T::TPIX + 15) / 16;          // 16-pixel groups over the whole tile
  constexpr int OLD = 33;                           // out row stride (floats): conflict-free
  static_assert(NPG * 16 * OLD * 4 <= T::TPIX * HC * 2, "out rows fit the tile area");
  static_assert(T::NW * 2 <= T::TPIX * HC * 2, "bf16 weights fit the tile area");
  __shared__ __attribute__((aligned(16))) char tile[T::TPIX * HC * 2];   // act; then out[p][33] fp32
  __shared__ float ta[HC], tb[HC], tp[HC], tq[HC];
  __shared__ float red[4];
  __bf16* wsb = reinterpret_cast<__bf16*>(tile);    // W[co][tap][c] bf16, before the first tile
  float* outl = reinterpret_cast<float*>(tile);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int tiles_per_img = q.h / T::ROWS;
  const int bpos = q.xcd ? head_xcd_order((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
  const rsrc_t ry = rsrc(q.x, (uint32_t)((long)q.n * q.h * HW * HC * 2));
  u32x4 raw[T::OCT_PER_T];
  if (bpos < q.tiles) {
    const int n0 = bpos / tiles_per_img;
    tile_load<HC, ROWS, HC>(q, ry, n0, (bpos - n0 * tiles_per_img) * T::ROWS, 0, raw);
  }
  for (int i = threadIdx.x; i < T::NW; i += 256) wsb[i] = (__bf16)q.wt[i];
  head_tables<HC, HC>(q.xf, ta, tb, tp, tq, 0, blockIdx.x == 0);
  __syncthreads();
  // B fragments (n-frag nf, K-step cc): column n = nf*16 + lane&15 = co*9 + t (n < 27), rows
  // c = 32 cc + 8 (lane>>4) .. +7
  bf16x8 bw[2][T::CC];
#pragma unroll
  for (int nf = 0; nf < 2; ++nf) {
    const int nn = nf * 16 + li, ok = nn < 27 ? 1 : 0, nc = ok ? nn : 0;
#pragma unroll
    for (int cc = 0; cc < T::CC; ++cc) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(&wsb[nc * HC + 32 * cc + 8 * g]);
      bw[nf][cc] = ok ? v : bf16x8{};
    }
  }
  // the gather's (pixel, co) items: idx = threadIdx.x + 256 k over ROWS*64 pixels x 3 channels;
  // their biases loaded here — a global load inside the tile loop, issued after the next tile's
  // prefetch, would make its wait drain the prefetch too (vmcnt counts in issue order)
  constexpr int GI = (T::OWN * NCO + 255) / 256;
  float bco[GI];
#pragma unroll
  for (int k = 0; k < GI; ++k) {
    const int idx = threadIdx.x + 256 * k;
    bco[k] = idx < T::OWN * NCO ? q.bias[idx / T::OWN] : 0.f;
  }
  for (int tile_i = bpos; tile_i < q.tiles; tile_i += gridDim.x) {
    const int n = tile_i / tiles_per_img, h0 = (tile_i - n * tiles_per_img) * T::ROWS;
    float tgt[GI];
#pragma unroll
    for (int k = 0; k < GI; ++k) {
      const int idx = threadIdx.x + 256 * k, co = idx / T::OWN, pix = idx - co * T::OWN;
      tgt[k] = idx < T::OWN * NCO
                   ? q.target[(((long)(n / q.samples) * NCO + co) * q.h + h0 + pix / HW) * HW + (pix % HW)]
                   : 0.f;
    }
    __syncthreads();                      // the weights / previous tile's out rows are consumed
    tile_store<HC, ROWS>(q, h0, raw, tile, ta, tb);
    __syncthreads();
    {
      const int nx = tile_i + gridDim.x;
      if (nx < q.tiles) {
        const int n1 = nx / tiles_per_img;
        tile_load<HC, ROWS, HC>(q, ry, n1, (nx - n1 * tiles_per_img) * T::ROWS, 0, raw);
      }
    }
    // out = act x W over the tile's pixel groups grp = wave + 4 k
    constexpr int GW = (NPG + 3) / 4;
    f32x4v acc[GW][2];
#pragma unroll
    for (int k = 0; k < GW; ++k) {
      acc[k][0] = f32x4v{0.f, 0.f, 0.f, 0.f};
      acc[k][1] = f32x4v{0.f, 0.f, 0.f, 0.f};
      const int grp = wave + 4 * k;
      if (grp < NPG) {
        int p = grp * 16 + li;
        p = p < T::TPIX ? p : T::TPIX - 1;          // (rows past the tile: never gathered)
        const int trow = p / T::TCOLS, tcol = p - trow * T::TCOLS;
#pragma unroll
        for (int cc = 0; cc < T::CC; ++cc) {
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(tile + act_off<HC>(trow, tcol, g + 4 * cc));
          acc[k][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[0][cc], acc[k][0], 0, 0, 0);
          acc[k][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[1][cc], acc[k][1], 0, 0, 0);
        }
      }
    }
    __syncthreads();                      // every wave is done with the act tile
#pragma unroll
    for (int k = 0; k < GW; ++k) {
      const int grp = wave + 4 * k;
      if (grp < NPG) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int p = grp * 16 + 4 * g + i;
          outl[p * OLD + li] = acc[k][0][i];
          outl[p * OLD + 16 + li] = acc[k][1][i];
        }
      }
    }
    __syncthreads();
    float sq = 0.f;
#pragma unroll
    for (int k = 0; k < GI; ++k) {
      const int idx = threadIdx.x + 256 * k;
      if (idx < T::OWN * NCO) {
        const int co = idx / T::OWN, pix = idx - co * T::OWN, row = pix / HW, col = pix - row * HW;
        float v = bco[k];
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const int r = t / 3, s2 = t - 3 * r;
          v += outl[((row + r) * T::TCOLS + col + s2) * OLD + co * 9 + t];
        }
        const float y = tanhf(v);
        q.recon[(((long)n * NCO + co) * q.h + h0 + row) * HW + col] = y;
        const float d = y - tgt[k];
        sq = fmaf(d, d, sq);
      }
    }
    for (int off = 32; off > 0; off >>= 1) sq += __shfl_xor(sq, off);
    if (lane == 0) red[wave] = sq;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(q.sse + n, (red[0] + red[1]) + (red[2] + red[3]));
  }
}

// ds_read_b64_tr_b16: lane 4q+p of each 16-lane group gives the address of row q, columns
// 4p..4p+3; lane i receives column i of the 4 rows (row q in element q).
typedef __bf16 __attribute__((ext_vector_type(4))) __attribute__((address_space(3))) lds_bf16x4;
__device__ __forceinline__ bf16x4v tr16_read(const char* generic_lds_addr) {
  const uint32_t off = (uint32_t)(uintptr_t)generic_lds_addr;   // LDS addresses are 32-bit
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(uintptr_t)off);
}

// ======================================================================= backward
// gseed = dL/d(pre-tanh) at one pixel/channel, split into its loads (issued one tile ahead)
// and the arithmetic: ld = (recon y, grad_recon or target)
struct SeedLd { float y[2][NCO], t[2][NCO]; };

template <int ROWS>
__device__ __forceinline__ void seed_load(const HeadQ& q, int tile_i, SeedLd& ld) {
  using T = HT<32, ROWS>;
  const int tiles_per_img = q.h / T::ROWS;
  const int n = tile_i / tiles_per_img, h0 = (tile_i - n * tiles_per_img) * T::ROWS;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int pix = threadIdx.x + 256 * j;
    const int trow = pix / T::TCOLS, tcol = pix - trow * T::TCOLS;
    const int hi = h0 + trow - 1, wi = tcol - 1;
    const bool ok = pix < T::TPIX && hi >= 0 && hi < q.h && wi >= 0 && wi < HW;
#pragma unroll
    for (int co = 0; co < NCO; ++co) {
      const long oi = (((long)n * NCO + co) * q.h + hi) * HW + wi;
      ld.y[j][co] = ok ? q.recon[oi] : 0.f;
      ld.t[j][co] = !ok ? 0.f
                        : q.grad_recon ? q.grad_recon[oi]
                                       : q.target[(((long)(n / q.samples) * NCO + co) * q.h + hi) * HW + wi];
    }
  }
}

__device__ __forceinline__ float gseed(const HeadQ& q, int n, const SeedLd& ld, int j, int co) {
  const float y = ld.y[j][co];
  if (q.grad_recon) return ld.t[j][co] * (1.f - y * y);
  return (q.coef ? q.coef[n] : q.hc) * (y - ld.t[j][co]) * (1.f - y * y);   // 0 outside the image (y = t = 0)
}

// One workgroup = one tile x HC of the CT input channels (CT / HC channel slices: the C = 128
// head runs as two 64-channel slices, so that a workgroup's LDS — tile, raw-y copy, output
// staging: 68 KB — leaves room for two per CU; as one 128-channel workgroup per CU it took 119 us
// at B = 64).  Each slice computes the (cheap, 3-channel) seed itself; the data gradient, its
// BatchNorm-backward sums and the weight gradient are per channel, so the slices never meet.
// Registers capped for 2 workgroups per CU; ROWS = 4 at C = 64 keeps one (104 KB of LDS) and all
// 512 VGPRs of a SIMD for its wave.
template <int HC, int ROWS, int CT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(HC >= 64 && ROWS >= 4 ? 1 : 2)))
head_bwd_mfma(HeadQ q) {
  kernarg_prefetch<(sizeof(HeadQ) < 1024 ? sizeof(HeadQ) : 1024)>();
  using T = HT<HC, ROWS>;
  constexpr int NSL = CT / HC;                                              // channel slices
  __shared__ __attribute__((aligned(16))) char tile[T::TPIX * HC * 2];
  __shared__ __attribute__((aligned(16))) uint2 gsA[T::TPIX];              // [pixel][co0..2, 0] bf16
  __shared__ __attribute__((aligned(16))) __bf16 gsT[4][T::OWN];           // [co][own pixel]
  __shared__ __attribute__((aligned(16))) __bf16 gst[4][16 * HC];          // per-wave output staging
  __shared__ __attribute__((aligned(16))) char ytile[T::OWN * HC * 2];     // raw y of the own pixels
  __shared__ float ta[HC], tb[HC], tp[HC], tq[HC];
  __shared__ float r1[4][HC], r2[4][HC], rdb[4][NCO];
  __shared__ bf16x8 bdl[T::NF > 2 ? 2 * T::NF * 64 : 1];                   // [ks][nf][lane] (HC >= 64)
  // the fp32 weights of the slice pass through the output staging area before the first tile
  // (27 HC floats in 128 HC bytes)
  float* wsh = reinterpret_cast<float*>(&gst[0][0]);
  static_assert(T::NW * 4 <= 4 * 16 * HC * 2, "weights fit the staging area");
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int tiles_per_img = q.h / T::ROWS;
  const rsrc_t ry = rsrc(q.x, (uint32_t)((long)q.n * q.h * HW * CT * 2));
  // position bpos = slice * gsl + local, tile_i = local + k * gsl: at every step the workgroups of
  // one XCD hold consecutive tiles of one slice (the host makes gridDim.x a multiple of 8 NSL)
  const int bpos = q.xcd ? head_xcd_order((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
  const int gsl = (int)gridDim.x / NSL;
  const int slice = bpos / gsl, local = bpos - slice * gsl, cb0 = slice * HC;

  for (int i = threadIdx.x; i < T::NW; i += 256) {
    const int ct = i / HC, c = i - ct * HC;                                 // ct = co * 9 + tap
    wsh[i] = q.wt[ct * CT + cb0 + c];
  }
  // filter accumulators: this wave's n-frags f = wave + 4*i (9 HC / 16 n-frags of 16 over (tap, c))
  f32x4v accw[T::NFW];
#pragma unroll
  for (int i = 0; i < T::NFW; ++i) accw[i] = f32x4v{0.f, 0.f, 0.f, 0.f};
  float s1[T::NF], s2[T::NF], dbp[NCO] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int nf = 0; nf < T::NF; ++nf) { s1[nf] = 0.f; s2[nf] = 0.f; }

  head_tables<HC, CT>(q.xf, ta, tb, tp, tq, cb0);
  // software pipeline: the raw y tile and the seed inputs of the next tile are loaded while
  // this tile's MFMAs run (one or two workgroups per CU leave few other waves to hide the latency)
  u32x4 raw[T::OCT_PER_T];
  SeedLd sld;
  if (local < q.tiles) {
    const int n0 = local / tiles_per_img;
    tile_load<HC, ROWS, CT>(q, ry, n0, (local - n0 * tiles_per_img) * T::ROWS, cb0, raw);
    seed_load<ROWS>(q, local, sld);
  }
  __syncthreads();
  // dgrad B fragments: B[k = tap*4 + co][n = c] = W[co][tap][c], k-step ks, n-frag nf — in
  // registers at HC = 32; wider slices (in registers: 28 VGPRs spilled at HC = 64 under the
  // two-workgroup cap) build them once into LDS and read them per use
  constexpr bool BDREG = T::NF <= 2;
  bf16x8 bd[2][BDREG ? T::NF : 1];
  if constexpr (BDREG) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int nf = 0; nf < T::NF; ++nf)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int tap = ks * 8 + 2 * g + (j >> 2), c2 = j & 3, c = nf * 16 + li;
          bd[ks][nf][j] = (__bf16)(tap < 9 && c2 < NCO ? wsh[(c2 * 9 + tap) * HC + c] : 0.f);
        }
  } else {
    for (int idx = threadIdx.x; idx < 2 * T::NF * 64; idx += 256) {
      const int ln = idx & 63, ks = idx / (64 * T::NF), nf = (idx >> 6) - ks * T::NF;
      const int lg = ln >> 4, ll = ln & 15;
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int tap = ks * 8 + 2 * lg + (j >> 2), c2 = j & 3, c = nf * 16 + ll;
        v[j] = (__bf16)(tap < 9 && c2 < NCO ? wsh[(c2 * 9 + tap) * HC + c] : 0.f);
      }
      bdl[idx] = v;
    }
  }
  for (int tile_i = local; tile_i < q.tiles; tile_i += gsl) {
    const int n = tile_i / tiles_per_img, h0 = (tile_i - n * tiles_per_img) * T::ROWS;
    // gseed over the halo tile: threads walk pixels (2 per thread)
    float gv[2][NCO];
    int gpix[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      gpix[j] = threadIdx.x + 256 * j;
#pragma unroll
      for (int c2 = 0; c2 < NCO; ++c2) gv[j][c2] = gseed(q, n, sld, j, c2);
    }
    __syncthreads();                    // previous tile's LDS reads done (and tables / weights read)
    tile_store<HC, ROWS>(q, h0, raw, tile, ta, tb);
    // raw y (pre-BN) of the own pixels for the data epilogue, from the same registers:
    // [own pixel][C] bf16, 16-byte chunks XOR-swizzled by the pixel
    if (q.data) {
#pragma unroll
      for (int j = 0; j < T::OCT_PER_T; ++j) {
        const int o = threadIdx.x + 256 * j;
        if (o >= T::OCT) continue;
        const int pix = o / T::CH, chk = o % T::CH;
        const int trow = pix / T::TCOLS, tcol = pix - trow * T::TCOLS;
        if (trow < 1 || trow > T::ROWS || tcol < 1 || tcol > HW) continue;
        const int own = (trow - 1) * HW + (tcol - 1);
        *reinterpret_cast<u32x4*>(ytile + own * (HC * 2) + ((chk ^ (own & T::SW)) << 4)) = raw[j];
      }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int pix = gpix[j];
      if (pix >= T::TPIX) continue;
      bf16x4v v; v[0] = (__bf16)gv[j][0]; v[1] = (__bf16)gv[j][1]; v[2] = (__bf16)gv[j][2]; v[3] = (__bf16)0.f;
      gsA[pix] = *reinterpret_cast<uint2*>(&v);
      const int trow = pix / T::TCOLS, tcol = pix - trow * T::TCOLS;
      if (trow >= 1 && trow <= T::ROWS && tcol >= 1 && tcol <= HW) {
        const int own = (trow - 1) * HW + (tcol - 1);
#pragma unroll
        for (int c2 = 0; c2 < NCO; ++c2) gsT[c2][own] = v[c2];
        gsT[3][own] = (__bf16)0.f;
#pragma unroll
        for (int c2 = 0; c2 < NCO; ++c2) dbp[c2] += gv[j][c2];
      }
    }
    __syncthreads();
    {
      const int nx = tile_i + gsl;
      if (nx < q.tiles) {
        const int n1 = nx / tiles_per_img;
        tile_load<HC, ROWS, CT>(q, ry, n1, (nx - n1 * tiles_per_img) * T::ROWS, cb0, raw);
        seed_load<ROWS>(q, nx, sld);
      }
    }

    if (q.data) {
      // ---- dact for this wave's groups of 16 pixels, N = C channels (C / 16 n-frags)
#pragma unroll 1
      for (int gi = 0; gi < T::GPW; ++gi) {
        const int grp = wave * T::GPW + gi;
        const int row = grp >> 2, c0 = (grp & 3) * 16;
        const int hh = h0 + row;
        f32x4v acc[T::NF];
#pragma unroll
        for (int nf = 0; nf < T::NF; ++nf) acc[nf] = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          bf16x8 a;
#pragma unroll
          for (int half = 0; half < 2; ++half) {
            const int tap = ks * 8 + 2 * g + half;
            uint2 v = {0u, 0u};
            if (tap < 9) {
              const int r = tap / 3, s = tap - 3 * r;
              v = gsA[(row + 2 - r) * T::TCOLS + (c0 + li + 2 - s)];
            }
            const bf16x4v b4 = *reinterpret_cast<bf16x4v*>(&v);
#pragma unroll
            for (int j = 0; j < 4; ++j) a[4 * half + j] = b4[j];
          }
#pragma unroll
          for (int nf = 0; nf < T::NF; ++nf) {
            bf16x8 b;
            if constexpr (BDREG) b = bd[ks][nf];
            else b = bdl[(ks * T::NF + nf) * 64 + lane];
            acc[nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[nf], 0, 0, 0);
          }
        }
        // g = dact * lrelu'(z); BN-backward sums; stage [16 px][C] for whole-row stores
#pragma unroll
        for (int nf = 0; nf < T::NF; ++nf) {
          const int c = nf * 16 + li;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int own = row * HW + c0 + 4 * g + i;
            const float y = (float)*reinterpret_cast<const __bf16*>(ytile + own * (HC * 2) +
                                                                    (((c >> 3) ^ (own & T::SW)) << 4) + (c & 7) * 2);
            const float z = fmaf(y, ta[c], tb[c]);
            const float gg = z > 0.f ? acc[nf][i] : acc[nf][i] * q.xf.slope;
            s1[nf] += gg;
            s2[nf] += gg * fmaf(y, tp[c], tq[c]);
            gst[wave][(4 * g + i) * HC + c] = (__bf16)gg;
          }
        }
        __builtin_amdgcn_wave_barrier();
        // 16 pixels x HC channels (NHWC, pixel stride CT): 16 B per lane per 1 KB
#pragma unroll
        for (int j = 0; j < HC / 32; ++j) {
          const int e = lane * 8 + 512 * j, px = e / HC, c = e - px * HC;
          const u32x4 v = *reinterpret_cast<const u32x4*>(&gst[wave][e]);
          *reinterpret_cast<u32x4*>(q.dx + (((long)n * q.h + hh) * HW + c0 + px) * CT + cb0 + c) = v;
        }
        __builtin_amdgcn_wave_barrier();
      }
    }

    if (q.filter) {
      // ---- dW partials: M = co (rows 0..2 of 16), N = (tap, c), K = the own pixels
      // (HC >= 64: one K-step at a time — unrolled, the scheduler hoisted every transposed read
      // of the tile: 146 VGPRs spilled at HC = 128)
      constexpr int KU = T::NF >= 4 ? 1 : T::OWN / 32;
#pragma unroll KU
      for (int ks = 0; ks < T::OWN / 32; ++ks) {
        const int k0 = ks * 32 + 8 * g;                 // this lane group's 8 pixels
        const int row = k0 / HW, col = k0 - row * HW;
        // rows co >= 3 of the M = 16 fragment read the all-zero row 3
        const bf16x8 az = *reinterpret_cast<const bf16x8*>(&gsT[li < 4 ? li : 3][k0]);
#pragma unroll
        for (int i = 0; i < T::NFW; ++i) {
          const int f = wave + 4 * i;
          if (f < T::NFR) {
            const int tap = f / T::NF, cb = (f - tap * T::NF) * 16;
            const int r = tap / 3, s = tap - 3 * r;
            // lane 4qq+pp of the 16-lane group: pixel qq (+4), channels cb + 4pp .. +3
            const int qq = li >> 2, pp = li & 3;
            const int ch = cb + 4 * pp;
            bf16x8 b;
#pragma unroll
            for (int half = 0; half < 2; ++half) {
              const int tcol = col + 4 * half + qq + s, trow = row + r;
              const char* addr = tile + act_off<HC>(trow, tcol, ch >> 3) + ((ch & 4) << 1);
              const bf16x4v t4 = tr16_read(addr);
#pragma unroll
              for (int j = 0; j < 4; ++j) b[4 * half + j] = t4[j];
            }
            accw[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(az, b, accw[i], 0, 0, 0);
          }
        }
      }
    }
  }

  // ---- block reductions
  if (q.data) {
#pragma unroll
    for (int nf = 0; nf < T::NF; ++nf) {
      float a = s1[nf], b = s2[nf];
      a += __shfl_xor(a, 16); a += __shfl_xor(a, 32);
      b += __shfl_xor(b, 16); b += __shfl_xor(b, 32);
      if (g == 0) { r1[wave][nf * 16 + li] = a; r2[wave][nf * 16 + li] = b; }
    }
  }
  __syncthreads();
  if (q.data && threadIdx.x < HC) {
    const int c = threadIdx.x;
    const long roff = q.sum_reps > 1 ? (long)(blockIdx.x % q.sum_reps) * q.sum_rstride : 0;
    atomicAdd(q.dbeta + roff + cb0 + c, (r1[0][c] + r1[1][c]) + (r1[2][c] + r1[3][c]));
    atomicAdd(q.dgamma + roff + cb0 + c, (r2[0][c] + r2[1][c]) + (r2[2][c] + r2[3][c]));
  }
#pragma unroll
  for (int c2 = 0; c2 < NCO; ++c2) {
    float v = dbp[c2];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0) rdb[wave][c2] = v;
  }
  __syncthreads();
  // the bias gradient from slice 0 only (every slice summed the same seeds)
  if (q.filter && threadIdx.x < NCO && q.db && slice == 0) {
    const float v = (rdb[0][threadIdx.x] + rdb[1][threadIdx.x]) + (rdb[2][threadIdx.x] + rdb[3][threadIdx.x]);
    if (q.slab) q.slab[(long)bpos * T::SLAB_COLS + T::NW + threadIdx.x] = v;
    else atomicAdd(q.db + threadIdx.x, v);
  }
  if (q.filter) {
    // dW[co][tap][c]: lane li = column within the n-frag, rows 4g+i = co (g == 0, i < 3 real);
    // slab rows are positions (a slice's rows contiguous), columns the slice's own (co, tap, c)
#pragma unroll
    for (int i = 0; i < T::NFW; ++i) {
      const int f = wave + 4 * i;
      if (f >= T::NFR || g != 0) continue;
      const int nn = f * 16 + li;                       // = tap*HC + c
      const int tap = nn / HC, c = nn - tap * HC;
#pragma unroll
      for (int e = 0; e < NCO; ++e) {
        if (q.slab) q.slab[(long)bpos * T::SLAB_COLS + e * 9 * HC + nn] = accw[i][e];
        else atomicAdd(q.dw + (e * 9 + tap) * CT + cb0 + c, accw[i][e]);
      }
    }
  }
}

// Column sums of the [rows][SLAB_COLS] fp32 slab of per-block filter partials, added into dw
// (columns < NW) and db (the NCO columns after): 16 columns x 16 row-parts per workgroup, each
// part's loads issued together, parts combined in a fixed order (deterministic).
constexpr int RR_COLS = 16, RR_PARTS = 16, RR_UNROLL = 8;
// (elbo.kind >= 0: one extra workgroup, the last, evaluates the step's ELBO — vae_head_args.elbo)
template <int HC, int CT>
__global__ void __launch_bounds__(256) reduce_rows_kernel(const float* src, int rows, float* dw, float* db, int cb0,
                                                          const vae_elbo_args elbo) {
  using T = HT<HC, 4>;
  __shared__ float red[RR_PARTS][RR_COLS];
  if (elbo.kind >= 0 && blockIdx.x == gridDim.x - 1) {
    __shared__ float kld_row[1024];
    __shared__ float ered[4][4];
    elbo_block(elbo, kld_row, ered);
    return;
  }
  const int cl = threadIdx.x % RR_COLS, part = threadIdx.x / RR_COLS;
  const int c = blockIdx.x * RR_COLS + cl;
  float s = 0.f;
  if (c < T::SLAB_COLS && (c < T::NW || db)) {
    for (int r0 = part; r0 < rows; r0 += RR_PARTS * RR_UNROLL) {
      float v[RR_UNROLL];
#pragma unroll
      for (int u = 0; u < RR_UNROLL; ++u) {
        const int r = r0 + u * RR_PARTS;
        v[u] = r < rows ? src[(long)r * T::SLAB_COLS + c] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < RR_UNROLL; ++u) s += v[u];
    }
  }
  red[part][cl] = s;
  __syncthreads();
  if (part != 0 || c >= T::SLAB_COLS) return;
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < RR_PARTS; ++i) t += red[i][cl];
  if (c < T::NW) {
    const int ct = c / HC, cl = c - ct * HC;          // ct = co * 9 + tap
    dw[ct * CT + cb0 + cl] += t;
  } else if (db) {
    db[c - T::NW] += t;
  }
}

bool head_mfma_ok(const vae_head_args* a) {
  return a->dtype == VAE_BF16 && (a->c == 32 || a->c == 64 || a->c == 128) && a->w == HW && a->h > 0 &&
         a->h % 4 == 0 && a->n > 0 &&
         ((uintptr_t)a->x & 15) == 0 && ((uintptr_t)a->recon & 15) == 0 && ((uintptr_t)a->target & 15) == 0 &&
         (a->x_xf.kind == VAE_X_BN_ACT || a->x_xf.kind == VAE_X_ACT || a->x_xf.kind == VAE_X_NONE);
}

// XCD-aware tile order
int head_xcd() { return 1; }

HeadQ head_q(const vae_head_args* a) {
  HeadQ q;
  memset(&q, 0, sizeof(q));
  q.n = a->n; q.h = a->h; q.samples = a->samples > 0 ? a->samples : 1;   // (q.tiles: per kernel)
  q.xcd = head_xcd();
  q.x = static_cast<const __bf16*>(a->x); q.xf = a->x_xf;
  if (q.xf.channels <= 0) q.xf.channels = a->c;
  q.wt = a->wt; q.bias = a->bias; q.target = a->target; q.recon = a->recon; q.sse = a->sse;
  q.coef = a->coef; q.grad_recon = a->grad_recon;
  q.dx = static_cast<__bf16*>(a->dx); q.dgamma = a->dx_dgamma; q.dbeta = a->dx_dbeta;
  q.sum_reps = a->sum_reps; q.sum_rstride = a->sum_rstride;
  q.dw = a->dw; q.db = a->db;
  return q;
}

template <int HC, int ROWS, int CT>
int head_bwd_go(const vae_head_args* a, HeadQ q, int gsl_max, hipStream_t st) {
  using T = HT<HC, ROWS>;
  constexpr int NSL = CT / HC;
  q.tiles = q.n * (q.h / ROWS);
  const int gsl = q.tiles < gsl_max ? q.tiles : gsl_max;     // workgroups per channel slice
  const int grid = gsl * NSL;
  const long need = (long)grid * T::SLAB_COLS * 4;
  float* ws = static_cast<float*>(a->workspace);
  if (q.filter && ws && !ws_fits(need, a->workspace_bytes, "head_bwd filter partials")) return VAE_E_BADARG;
  const bool slab = q.filter && ws;
  q.slab = slab ? ws : nullptr;
  vae_elbo_args el;
  memset(&el, 0, sizeof(el));
  el.kind = -1;
  if (a->elbo) {
    el = *a->elbo;
    if ((el.kind != VAE_LOSS_VANILLA && el.kind != VAE_LOSS_BETA_H) || (el.samples > 1) || !slab || !q.filter)
      return fail(VAE_E_UNSUPPORTED, "head_bwd: fused ELBO needs the vanilla / BetaVAE-H loss, samples 1 and a workspace");
    // vae_elbo_fwd's checks (elbo_block keeps per-row KL terms in a 1024-entry LDS array), and the
    // loss must describe the batch this call's seed scales
    if (!el.sse || !el.out || !el.per_img || !el.mulv)
      return fail(VAE_E_BADARG, "head_bwd: fused ELBO args");
    if (el.batch <= 0 || el.batch > 1024 || el.latent <= 0 || el.img_elems <= 0)
      return fail(VAE_E_BADSHAPE, "head_bwd: fused ELBO sizes (batch %d, latent %d)", el.batch, el.latent);
    if (el.batch != q.n || el.img_elems != 3 * q.h * a->w)
      return fail(VAE_E_BADSHAPE, "head_bwd: fused ELBO batch %d / image %d vs the head's %d x %d", el.batch,
                  el.img_elems, q.n, 3 * q.h * a->w);
    q.coef = nullptr;
    q.hc = 2.f / ((float)el.batch * (float)el.img_elems);
  }
  VAE_LAUNCH((head_bwd_mfma<HC, ROWS, CT>), dim3(grid), dim3(256), 0, st, q);
  int rc = check_launch("head_bwd_mfma");
  if (rc || !q.filter || !slab) return rc;
  if (a->defer_reduce && NSL == 1) {
    // the filter partials (slab rows [grid][27 HC + 3], dW index = column for one channel slice) and
    // the loss stay for vae_adam_step_ex
    if (!defer_slab(a->dw, T::NW, ws, gsl, T::SLAB_COLS)) return VAE_E_UNSUPPORTED;
    if (a->db && !defer_slab(a->db, NCO, ws + T::NW, gsl, T::SLAB_COLS)) return VAE_E_UNSUPPORTED;
    if (el.kind >= 0) defer_elbo(el);
    return VAE_OK;
  }
  vae_elbo_args none;
  memset(&none, 0, sizeof(none));
  none.kind = -1;
  for (int sl = 0; sl < NSL && !rc; ++sl) {      // a slice's slab rows are contiguous positions
    const bool e = sl == 0 && el.kind >= 0;
    VAE_LAUNCH((reduce_rows_kernel<HC, CT>), dim3((T::SLAB_COLS + RR_COLS - 1) / RR_COLS + (e ? 1 : 0)), dim3(256), 0,
               st, (const float*)ws + (long)sl * gsl * T::SLAB_COLS, gsl, a->dw, sl == 0 ? a->db : nullptr, sl * HC,
               e ? el : none);
    rc = check_launch("reduce_rows");
  }
  return rc;
}

}  // namespace

// Persistent grid of the backward.  C = 32, swept on MI355X (B=64 step): 128 -> 78.7 us,
// 192 -> 61.7, 256 -> 45.6, 512 -> 50.5, 1024 -> 61.4 (more blocks means more filter partials to
// reduce and more halo re-reads; fewer leaves CUs idle).  Re-swept with the tile-ahead loads:
// 192 -> 50.4 us, 256 -> 38.5, 320 -> 55.6, 384 -> 49.8, 512 -> 43.9 (scripts/gpu_headgrid.sh).
// r2: with the registers capped for 2 workgroups per CU (amdgpu_waves_per_eu(2)), 512 -> 37.2 us
// (two tiles in flight per CU), 256 -> 45.1 (the cap's spills without the second workgroup).
// C = 64 / 128: 64-channel slices of 2 image rows, two workgroups per CU — 512 workgroups, i.e.
// 512 per slice (C = 64) or 256 per slice (C = 128).
constexpr int kHeadGrid = 512;
int head_grid() { return kHeadGrid; }

// Entry points used by vae_misc.hip's C ABI for the bf16 MFMA path.
int head_fwd_mfma_launch(const vae_head_args* a, hipStream_t st) {
  if (!head_mfma_ok(a)) return kHeadFallback;       // caller falls back to the VALU kernels
  HeadQ q = head_q(a);
  switch (a->c) {
    case 32: q.tiles = q.n * (q.h / 4); VAE_LAUNCH((head_fwd_mfma<32, 4>), dim3(q.tiles), dim3(256), 0, st, q); break;
    case 64: q.tiles = q.n * (q.h / 4); VAE_LAUNCH((head_fwd_mfma<64, 4>), dim3(q.tiles), dim3(256), 0, st, q); break;
    default: {
      q.tiles = q.n * (q.h / 2);
      const int grid = q.tiles < head_grid() ? q.tiles : head_grid();   // two workgroups per CU
      VAE_LAUNCH((head_fwd_stream<128, 2>), dim3(grid), dim3(256), 0, st, q);
      break;
    }
  }
  return check_launch("head_fwd_mfma");
}

// data / filter: which halves of the backward to run.  The filter half writes per-block partials
// into the caller's workspace (when large enough) and reduces them into dw/db in fixed order.
int head_bwd_mfma_launch(const vae_head_args* a, bool data, bool filter, hipStream_t st) {
  if (!head_mfma_ok(a)) return kHeadFallback;
  if (data && a->dx_epi.kind != VAE_X_BN_ACT) return kHeadFallback;   // the fused epilogue is BatchNorm+LReLU
  HeadQ q = head_q(a);
  q.data = data; q.filter = filter;
  switch (a->c) {
    case 32: return head_bwd_go<32, 4, 32>(a, q, head_grid(), st);
    case 64: return head_bwd_go<64, 2, 64>(a, q, head_grid(), st);
    default: return head_bwd_go<64, 2, 128>(a, q, head_grid() / 2, st);
  }
}

}  // namespace vae
