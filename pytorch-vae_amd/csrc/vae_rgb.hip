// The VQ-VAE's RGB ends on dedicated kernels (bf16; models/vq_vae.py:98-105, :156-164, :203):
//   * rgb_out_fwd: the output ConvTranspose2d(C -> 3, k4 s2 p1) with LeakyReLU applied to its input
//     on load, fused with Tanh + reconstruction + per-image SSE + the MSE backward seed
//     (vae_recon_fwd's work) — the reconstruction never goes through HBM as a pre-tanh tensor;
//   * rgb_out_bwd: that layer's data gradient (LeakyReLU-backward epilogue), weight gradient and
//     bias gradient in ONE pass over dy and x;
//   * rgb_in_wgrad: the input Conv2d(3 -> C, k4 s2 p1)'s weight and bias gradient.
//
// Why: with 3 output channels the layer is a thin GEMM — the conv-GEMM path padded N = 3 to a
// 16/32-wide MFMA tile and gathered every 128-channel input pixel for each of the 4 phases x 4
// taps of an output-centric GEMM (73.8 us fwd, 71.6 wgrad, 46.5 dgrad at B = 128, r3_v7), while
// the layer's bytes are ~25 MB (~4 us of HBM).  Here the GEMMs are INPUT-centric: one input pixel
// (C channels) against all 16 taps x 4 (3 real) output channels is one 64-wide row, so
// N = 64 instead of 3 -> 16..32, and each input element is read once per workgroup tile (plus a
// one-row halo).  The tap scatter of the forward is a fixed-order gather of the four contributions
// per output pixel from an LDS result tile (deterministic), the weight gradients reduce per-tile
// partials through a workspace slab in a fixed order.
//
// Geometry (checked on the host): wide side [n][H][W][C] with H = W = 32, W * C multiple of 8,
// C == 128; RGB side [n][2H][2W][CP], CP = 8 (3 real channels, zero padded: the VQ plan's packed
// layout) — the forward's weights wt[c][4][4][CP] (ConvTranspose2d native, padded).
#include "vae_common.hpp"
#include "vae_rgb.hpp"

namespace vae {
namespace {

constexpr int RG_C = 128;            // wide-side channels
constexpr int RG_H = 32;             // wide-side spatial size (square)
constexpr int RG_TI = 8;             // wide-side rows per tile
constexpr int RG_CP = 8;             // packed RGB channels (3 real)
constexpr int RG_KK = 64;            // 16 taps x 4 (3 real) GEMM columns
constexpr int RG_LDA = RG_C + 8;     // LDS row pitch (bf16) of C-wide rows: conflict-free b128 reads
constexpr int RG_LDK = RG_KK + 8;    // of 64-wide rows
constexpr int RG_SLAB = RG_C * RG_KK + RG_C;   // per-tile partial: dW [C][64] + bias column [<= C]

typedef __bf16 rg_lds_bf16x4 __attribute__((ext_vector_type(4))) __attribute__((address_space(3)));
typedef __bf16 rg_bf16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ rg_bf16x4 rg_tr_read(const void* generic_lds_addr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((rg_lds_bf16x4*)(uintptr_t)(uint32_t)(uintptr_t)generic_lds_addr);
}

__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  bf16x2 h;
  h[0] = (__bf16)a;
  h[1] = (__bf16)b;
  return *reinterpret_cast<uint32_t*>(&h);
}

// 16 bytes (8 channels) of the wide tensor with LeakyReLU applied (slope >= 1: identity)
__device__ __forceinline__ uint4 act8(uint4 v, float slope) {
  if (slope >= 1.f) return v;
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t o[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) o[e] = pack2(lrelu(bf_lo(w[e]), slope), lrelu(bf_hi(w[e]), slope));
  return uint4{o[0], o[1], o[2], o[3]};
}

// ------------------------------------------------------------------------------------------------
// Forward: workgroup = (image, RG_TI wide rows) -> output rows [2 i0, 2 i0 + 2 TI) x all columns.
// Input rows i0 - 1 .. i0 + TI (a one-row halo each side; rows outside the image are zeros).
constexpr int RF_T = 256;
constexpr int RF_ROWS = (RG_TI + 2) * RG_H;           // 320 input pixels
struct RgbFwd {
  int n;
  const __bf16* x; float slope;                       // [n][32][32][128], LeakyReLU on load
  const __bf16* wt; const float* bias;                // [128][16][CP] bf16, [CP] (first 3 read)
  const float* target; float* recon; float* sse;      // NCHW fp32, [n]
  __bf16* dy; float grad_scale;                       // [n][64][64][CP] seed (or null)
  const float* grad_recon;                            // drop-in: seed from dL/drecon instead
};

constexpr int RF_LDS_A = RF_ROWS * RG_LDA * 2;        // 87,040 B; reused as the fp32 result tile
constexpr int RF_LDG = RG_KK + 4;                     // result row pitch (fp32)
static_assert(RF_ROWS * RF_LDG * 4 <= RF_LDS_A, "result tile fits the operand tile");

__global__ void __launch_bounds__(RF_T) rgb_out_fwd_kernel(const RgbFwd q) {
  kernarg_prefetch<(sizeof(RgbFwd) < 1024 ? sizeof(RgbFwd) : 1024)>();
  __shared__ __attribute__((aligned(16))) char lds_a[RF_LDS_A];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[RG_KK * RG_LDA];
  __shared__ float red[RF_T / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int img = blockIdx.x / (RG_H / RG_TI), i0 = (blockIdx.x % (RG_H / RG_TI)) * RG_TI;
  __bf16* As = reinterpret_cast<__bf16*>(lds_a);
  // ---- A: 320 pixel rows x 128 channels (16 chunks of 16 B), LeakyReLU applied
  const __bf16* xi = q.x + (long)img * RG_H * RG_H * RG_C;
  for (int t = tid; t < RF_ROWS * (RG_C / 8); t += RF_T) {
    const int row = t >> 4, ch = t & 15;
    const int ih = i0 - 1 + row / RG_H, iw = row % RG_H;
    uint4 v = uint4{0u, 0u, 0u, 0u};
    if ((unsigned)ih < (unsigned)RG_H) v = act8(*reinterpret_cast<const uint4*>(xi + ((long)ih * RG_H + iw) * RG_C + 8 * ch), q.slope);
    *reinterpret_cast<uint4*>(As + row * RG_LDA + 8 * ch) = v;
  }
  // ---- B: row kk = tap * 4 + k of the GEMM = wt[c][tap][k] (k < 3), k = 3 zero
  for (int t = tid; t < RG_C * 16; t += RF_T) {
    const int c = t >> 4, tap = t & 15;
    const __bf16* w = q.wt + ((long)c * 16 + tap) * RG_CP;
#pragma unroll
    for (int k = 0; k < 4; ++k) Bs[(tap * 4 + k) * RG_LDA + c] = k < 3 ? w[k] : (__bf16)0.f;
  }
  __syncthreads();
  // ---- G[pix][kk] = sum_c A[pix][c] B[kk][c]: 20 x 4 fragments of 16 x 16, wave w: rows 80w..
  constexpr int FM = RF_ROWS / 16 / 4;                // 5 row fragments per wave
  f32x4 acc[FM][4];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < RG_C / 32; ++ks) {
    bf16x8 bfr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + (j * 16 + (lane & 15)) * RG_LDA + ks * 32 + 8 * (lane >> 4));
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const bf16x8 af = *reinterpret_cast<const bf16x8*>(As + ((wave * FM + i) * 16 + (lane & 15)) * RG_LDA + ks * 32 +
                                                         8 * (lane >> 4));
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();                                     // every wave is done with As
  float* G = reinterpret_cast<float*>(lds_a);         // [320][RF_LDG]
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        G[((wave * FM + i) * 16 + 4 * (lane >> 4) + e) * RF_LDG + j * 16 + (lane & 15)] = acc[i][j][e];
  __syncthreads();
  // ---- outputs: rows 2 i0 .. 2 i0 + 15, columns 0..63; thread -> 4 pixels of one row (coalesced NCHW)
  const float b0 = q.bias[0], b1 = q.bias[1], b2 = q.bias[2];
  const long hw = 4l * RG_H * RG_H;
  float sse = 0.f;
  for (int t = tid; t < 2 * RG_TI * 2 * RG_H; t += RF_T) {
    const int orow = t / (2 * RG_H), ow = t % (2 * RG_H), oh = 2 * i0 + orow;
    float y[3] = {b0, b1, b2};
    const int qh = (oh + 1) >> 1, rh = (oh + 1) & 1, qw = (ow + 1) >> 1, rw = (ow + 1) & 1;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int ih = qh - a, r = rh + 2 * a;
      if ((unsigned)ih >= (unsigned)RG_H) continue;
      const int lr = ih - (i0 - 1);
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int iw = qw - b, s = rw + 2 * b;
        if ((unsigned)iw >= (unsigned)RG_H) continue;
        const float* g = G + (lr * RG_H + iw) * RF_LDG + (r * 4 + s) * 4;
        y[0] += g[0];
        y[1] += g[1];
        y[2] += g[2];
      }
    }
    float gv[3];
    const long pix = (long)oh * 2 * RG_H + ow;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const long o = ((long)img * 3 + c) * hw + pix;
      const float r = tanhf(y[c]);
      q.recon[o] = r;
      const float d = r - q.target[o];
      sse = fmaf(d, d, sse);
      gv[c] = (q.grad_recon ? q.grad_recon[o] : q.grad_scale * 2.f * d) * (1.f - r * r);
    }
    if (q.dy)
      *reinterpret_cast<uint4*>(q.dy + ((long)img * hw + pix) * RG_CP) = uint4{pack2(gv[0], gv[1]), pack2(gv[2], 0.f), 0u, 0u};
  }
  if (!q.sse) return;
  for (int off = 32; off > 0; off >>= 1) sse += __shfl_xor(sse, off);
  if (lane == 0) red[wave] = sse;
  __syncthreads();
  if (tid == 0) atomicAdd(q.sse + img, (red[0] + red[1]) + (red[2] + red[3]));
}

// ------------------------------------------------------------------------------------------------
// Weight-gradient tile shared by both backward kernels: dW[m][kk] += sum_pix U[pix][m] V[pix][kk]
// over the tile's 256 pixels, m < 128, kk < 64.  U and V are [pix][...] row-major in LDS; the MFMA
// operands (k = pixels) come from transposed reads (ds_read_b64_tr_b16).  8 waves: wave w takes
// m rows 16w.. and all 4 kk fragments (4 accumulators).
constexpr int RB_T = 512;
constexpr int RB_PIX = RG_TI * RG_H;                 // 256 pixels per tile
__device__ __forceinline__ void rg_wgrad_tile(const __bf16* U, int ldu, const __bf16* V, int ldv, f32x4 (&acc)[4],
                                              int wave, int lane) {
  const int g = lane >> 4, l16 = lane & 15, qq = l16 >> 2, p = l16 & 3;
#pragma unroll
  for (int ks = 0; ks < RB_PIX / 32; ++ks) {
    const int r0 = ks * 32 + 8 * g;                  // this lane group's 8 pixels
    bf16x8 af;
    {
      const rg_bf16x4 lo = rg_tr_read(U + (r0 + qq) * ldu + wave * 16 + 4 * p);
      const rg_bf16x4 hi = rg_tr_read(U + (r0 + 4 + qq) * ldu + wave * 16 + 4 * p);
      af = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const rg_bf16x4 lo = rg_tr_read(V + (r0 + qq) * ldv + j * 16 + 4 * p);
      const rg_bf16x4 hi = rg_tr_read(V + (r0 + 4 + qq) * ldv + j * 16 + 4 * p);
      const bf16x8 bf = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, acc[j], 0, 0, 0);
    }
  }
}

// per-workgroup partial -> slab row [m][64] (+ the bias column written by the caller)
__device__ __forceinline__ void rg_store_partial(float* slab, const f32x4 (&acc)[4], int wave, int lane) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) slab[(wave * 16 + 4 * (lane >> 4) + e) * RG_KK + j * 16 + (lane & 15)] = acc[j][e];
}

// Backward of the output ConvT.  Workgroup = (image, RG_TI wide rows); tiles_per_wg tiles in turn.
struct RgbBwd {
  int n, tiles, per;
  const __bf16* dy;                                   // [n][64][64][CP]
  const __bf16* x; float slope;                       // [n][32][32][128] pre-activation
  const __bf16* wt;                                   // [128][16][CP]
  __bf16* dx;                                         // [n][32][32][128]: lrelu'(x) * (dy conv W)
  float* slab;                                        // [gridDim][RG_SLAB]
};

constexpr int RB_DYR = 2 * RG_TI + 2;                 // dy rows a tile reads (one halo row each side)
__global__ void __launch_bounds__(RB_T) rgb_out_bwd_kernel(const RgbBwd q) {
  kernarg_prefetch<(sizeof(RgbBwd) < 1024 ? sizeof(RgbBwd) : 1024)>();
  __shared__ __attribute__((aligned(16))) __bf16 Xs[RB_PIX * RG_LDA];   // lrelu(x), then the dx tile
  __shared__ __attribute__((aligned(16))) __bf16 Gs[RB_PIX * RG_LDK];   // gathered dy rows per pixel
  __shared__ __attribute__((aligned(16))) __bf16 Ws[RG_C * RG_LDK];     // W[c][tap*4+k]
  __shared__ __attribute__((aligned(16))) __bf16 Dy[RB_DYR * 2 * RG_H * 4];
  __shared__ float bsum[RB_T / 64][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int t = tid; t < RG_C * 16; t += RB_T) {
    const int c = t >> 4, tap = t & 15;
    const __bf16* w = q.wt + ((long)c * 16 + tap) * RG_CP;
#pragma unroll
    for (int k = 0; k < 4; ++k) Ws[c * RG_LDK + tap * 4 + k] = k < 3 ? w[k] : (__bf16)0.f;
  }
  f32x4 wacc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) wacc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bacc = 0.f;                                   // thread: bias column (tid & 3) partial
  for (int it = 0; it < q.per; ++it) {
    const int tile = blockIdx.x * q.per + it;
    if (tile >= q.tiles) break;                       // (uniform across the workgroup)
    const int img = tile / (RG_H / RG_TI), i0 = (tile % (RG_H / RG_TI)) * RG_TI;
    __syncthreads();                                  // previous tile's readers of Xs / Gs / Dy
    // x tile: 256 pixels x 128 channels, LeakyReLU applied (its sign is the activation's derivative)
    const __bf16* xi = q.x + ((long)img * RG_H + i0) * RG_H * RG_C;
    for (int t = tid; t < RB_PIX * (RG_C / 8); t += RB_T) {
      const int row = t >> 4, ch = t & 15;
      *reinterpret_cast<uint4*>(Xs + row * RG_LDA + 8 * ch) =
          act8(*reinterpret_cast<const uint4*>(xi + (long)row * RG_C + 8 * ch), q.slope);
    }
    // dy rows 2 i0 - 1 .. 2 i0 + 2 TI, 4 channels (3 real) per pixel; the bias sum over the owned rows
    const __bf16* dyi = q.dy + (long)img * 4 * RG_H * RG_H * RG_CP;
    for (int t = tid; t < RB_DYR * 2 * RG_H; t += RB_T) {
      const int lr = t / (2 * RG_H), ow = t % (2 * RG_H), oh = 2 * i0 - 1 + lr;
      uint2 v = uint2{0u, 0u};
      if ((unsigned)oh < (unsigned)(2 * RG_H)) v = *reinterpret_cast<const uint2*>(dyi + ((long)oh * 2 * RG_H + ow) * RG_CP);
      v.y &= 0xffffu;                                  // channel 3: zero
      *reinterpret_cast<uint2*>(Dy + t * 4) = v;
    }
    __syncthreads();
    // owned dy rows (1 .. 2 TI of Dy) -> bias partial: thread t sums channel t & 3 over pixels t >> 2, + 128, ...
    for (int t = tid; t < 2 * RG_TI * 2 * RG_H * 4; t += RB_T) {
      const int pix = t >> 2, c = t & 3;
      bacc += (float)Dy[(2 * RG_H + pix) * 4 + c];   // (rows 1.. of the Dy tile)
    }
    // gather: Gs[pix][tap * 4 + k] = dy[2 ih - 1 + r][2 iw - 1 + s][k]
    for (int t = tid; t < RB_PIX * 16; t += RB_T) {
      const int pix = t >> 4, tap = t & 15, r = tap >> 2, s = tap & 3;
      const int lih = pix / RG_H, iw = pix % RG_H;
      const int lr = 2 * lih + r, ow = 2 * iw - 1 + s;  // Dy row 2 lih - 1 + r + 1 (halo offset)
      uint2 v = uint2{0u, 0u};
      if ((unsigned)ow < (unsigned)(2 * RG_H)) v = *reinterpret_cast<const uint2*>(Dy + (lr * 2 * RG_H + ow) * 4);
      *reinterpret_cast<uint2*>(Gs + pix * RG_LDK + tap * 4) = v;
    }
    __syncthreads();
    // weight gradient: dW[c][kk] += sum_pix lrelu(x)[pix][c] Gs[pix][kk]
    rg_wgrad_tile(Xs, RG_LDA, Gs, RG_LDK, wacc, wave, lane);
    // data gradient: dxp[pix][c] = sum_kk Gs[pix][kk] W[c][kk]; wave w: pixels 32w.. (2 fragments) x 8
    f32x4 dacc[2][8];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) dacc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < RG_KK / 32; ++ks) {
      bf16x8 af[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(Gs + (wave * 32 + i * 16 + (lane & 15)) * RG_LDK + ks * 32 + 8 * (lane >> 4));
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bf16x8 bf = *reinterpret_cast<const bf16x8*>(Ws + (j * 16 + (lane & 15)) * RG_LDK + ks * 32 + 8 * (lane >> 4));
#pragma unroll
        for (int i = 0; i < 2; ++i) dacc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf, dacc[i][j], 0, 0, 0);
      }
    }
    // LeakyReLU backward from the sign of lrelu(x) (the lane's own elements), into registers
    uint32_t dpk[2][8][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int pix = wave * 32 + i * 16 + 4 * (lane >> 4) + e, c = j * 16 + (lane & 15);
          const float xv = (float)Xs[pix * RG_LDA + c];
          v[e] = xv > 0.f ? dacc[i][j][e] : dacc[i][j][e] * q.slope;
        }
        dpk[i][j][0] = pack2(v[0], v[1]);
        dpk[i][j][1] = pack2(v[2], v[3]);
      }
    __syncthreads();                                  // every wave is done reading Xs
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int pix = wave * 32 + i * 16 + 4 * (lane >> 4) + e, c = j * 16 + (lane & 15);
          const uint32_t w = dpk[i][j][e >> 1];
          *reinterpret_cast<unsigned short*>(Xs + pix * RG_LDA + c) = (unsigned short)((e & 1) ? (w >> 16) : (w & 0xffffu));
        }
    __syncthreads();
    __bf16* dxo = q.dx + ((long)img * RG_H + i0) * RG_H * RG_C;
    for (int t = tid; t < RB_PIX * (RG_C / 8); t += RB_T) {
      const int row = t >> 4, ch = t & 15;
      *reinterpret_cast<uint4*>(dxo + (long)row * RG_C + 8 * ch) = *reinterpret_cast<const uint4*>(Xs + row * RG_LDA + 8 * ch);
    }
  }
  // this workgroup's partials: dW [128][64] and the bias column (3 used)
  float* slab = q.slab + (long)blockIdx.x * RG_SLAB;
  rg_store_partial(slab, wacc, wave, lane);
  for (int off = 4; off < 64; off <<= 1) bacc += __shfl_xor(bacc, off);   // lanes of equal (tid & 3)
  if (lane < 4) bsum[wave][lane] = bacc;
  __syncthreads();
  if (tid < RG_C) {
    float s = 0.f;
    if (tid < 4)
      for (int w = 0; w < RB_T / 64; ++w) s += bsum[w][tid];
    slab[RG_C * RG_KK + tid] = s;
  }
}

// Input conv weight gradient: workgroup = (image, RG_TI output rows of the 32 x 32 grid).
// U = dy [pix][128] (as stored), V = the 8-channel image gathered per tap ([pix][tap*4 + c], c < 3).
struct RgbIn {
  int n, tiles, per;
  const __bf16* dy;                                   // [n][32][32][128]
  const __bf16* x;                                    // [n][64][64][CP] (3 real)
  float* slab;
};

constexpr int RI_XR = 2 * RG_TI + 2;                  // image rows a tile reads
__global__ void __launch_bounds__(RB_T) rgb_in_wgrad_kernel(const RgbIn q) {
  kernarg_prefetch<(sizeof(RgbIn) < 1024 ? sizeof(RgbIn) : 1024)>();
  __shared__ __attribute__((aligned(16))) __bf16 Us[RB_PIX * RG_LDA];
  __shared__ __attribute__((aligned(16))) __bf16 Gs[RB_PIX * RG_LDK];
  __shared__ __attribute__((aligned(16))) __bf16 Xi[RI_XR * 2 * RG_H * 4];
  __shared__ float csum[RB_T / 64][RG_C];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  f32x4 wacc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) wacc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float cacc[2] = {0.f, 0.f};                         // bias columns: thread sums channel pair
  for (int it = 0; it < q.per; ++it) {
    const int tile = blockIdx.x * q.per + it;
    if (tile >= q.tiles) break;
    const int img = tile / (RG_H / RG_TI), o0 = (tile % (RG_H / RG_TI)) * RG_TI;
    __syncthreads();
    const __bf16* dyi = q.dy + ((long)img * RG_H + o0) * RG_H * RG_C;
    for (int t = tid; t < RB_PIX * (RG_C / 8); t += RB_T) {
      const int row = t >> 4, ch = t & 15;
      const uint4 v = *reinterpret_cast<const uint4*>(dyi + (long)row * RG_C + 8 * ch);
      *reinterpret_cast<uint4*>(Us + row * RG_LDA + 8 * ch) = v;
    }
    const __bf16* xi = q.x + (long)img * 4 * RG_H * RG_H * RG_CP;
    for (int t = tid; t < RI_XR * 2 * RG_H; t += RB_T) {
      const int lr = t / (2 * RG_H), xw = t % (2 * RG_H), xh = 2 * o0 - 1 + lr;
      uint2 v = uint2{0u, 0u};
      if ((unsigned)xh < (unsigned)(2 * RG_H)) v = *reinterpret_cast<const uint2*>(xi + ((long)xh * 2 * RG_H + xw) * RG_CP);
      v.y &= 0xffffu;
      *reinterpret_cast<uint2*>(Xi + t * 4) = v;
    }
    __syncthreads();
    // bias: column sums of the dy tile, thread t -> channels 2 (t & 63) .. + 1 over rows t >> 6, + 8, ...
    for (int row = tid >> 6; row < RB_PIX; row += RB_T / 64) {
      const uint32_t w = *reinterpret_cast<const uint32_t*>(Us + row * RG_LDA + 2 * lane);
      cacc[0] += bf_lo(w);
      cacc[1] += bf_hi(w);
    }
    // gather: Gs[pix][tap * 4 + c] = x[2 oh - 1 + r][2 ow - 1 + s][c]
    for (int t = tid; t < RB_PIX * 16; t += RB_T) {
      const int pix = t >> 4, tap = t & 15, r = tap >> 2, s = tap & 3;
      const int loh = pix / RG_H, ow = pix % RG_H;
      const int lr = 2 * loh + r, xw = 2 * ow - 1 + s;
      uint2 v = uint2{0u, 0u};
      if ((unsigned)xw < (unsigned)(2 * RG_H)) v = *reinterpret_cast<const uint2*>(Xi + (lr * 2 * RG_H + xw) * 4);
      *reinterpret_cast<uint2*>(Gs + pix * RG_LDK + tap * 4) = v;
    }
    __syncthreads();
    rg_wgrad_tile(Us, RG_LDA, Gs, RG_LDK, wacc, wave, lane);
  }
  float* slab = q.slab + (long)blockIdx.x * RG_SLAB;
  rg_store_partial(slab, wacc, wave, lane);
  csum[wave][2 * lane] = cacc[0];
  csum[wave][2 * lane + 1] = cacc[1];
  __syncthreads();
  if (tid < RG_C) {
    float s = 0.f;
    for (int w = 0; w < RB_T / 64; ++w) s += csum[w][tid];
    slab[RG_C * RG_KK + tid] = s;
  }
}

// dW[m][tap][j] += sum_wg slab[wg][m][tap * 4 + j] (j < 3, fixed order); db[j or m] likewise from the
// bias column (nbias = 3 for the output ConvT, 128 for the input conv).  A workgroup takes RS_COLS
// columns x RS_PARTS row-parts, each part's RS_UNROLL loads in flight, the parts combined in LDS in
// a fixed order: one thread per column walking all 256 rows (25 workgroups over the chip) took
// 21.9 us per call at B = 128 (r4_v6_vq_pmc.json).
constexpr int RS_COLS = 32, RS_PARTS = 8, RS_UNROLL = 8;
__global__ void __launch_bounds__(256) rgb_slab_reduce(const float* slab, int rows, float* dw, float* db, int nbias) {
  __shared__ float red[RS_PARTS][RS_COLS];
  const int cl = threadIdx.x % RS_COLS, part = threadIdx.x / RS_COLS;
  const int col = blockIdx.x * RS_COLS + cl;          // over RG_C * 16 * 3 + nbias
  const int nw = RG_C * 16 * 3;
  const bool ok = col < nw + nbias;
  int src = 0;
  if (col < nw) {
    const int m = col / 48, r = col % 48, tap = r / 3, j = r % 3;
    src = m * RG_KK + tap * 4 + j;
  } else {
    src = RG_C * RG_KK + (col - nw);
  }
  float s = 0.f;
  if (ok) {
    for (int r0 = part; r0 < rows; r0 += RS_PARTS * RS_UNROLL) {
      float v[RS_UNROLL];
#pragma unroll
      for (int u = 0; u < RS_UNROLL; ++u) {
        const int r = r0 + u * RS_PARTS;
        v[u] = r < rows ? slab[(long)r * RG_SLAB + src] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < RS_UNROLL; ++u) s += v[u];
    }
  }
  red[part][cl] = s;
  __syncthreads();
  if (part != 0 || !ok) return;
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < RS_PARTS; ++i) t += red[i][cl];
  if (col < nw) dw[col] += t;
  else if (db) db[col - nw] += t;
}

bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

bool geom_ok_rgb(const vae_conv_args* a) {
  return a && a->n > 0 && a->h > 0 && a->w > 0 && a->c > 0 && a->k > 0 && a->p > 0 && a->q > 0 && a->r > 0 &&
         a->stride > 0 && a->pad >= 0;
}

// the wide side: [n][32][32][128] bf16, the RGB side [n][64][64][8] bf16
bool rgb_geom(const vae_conv_args* a, bool transposed) {
  if (a->dtype != VAE_BF16 || a->r != 4 || a->stride != 2 || a->pad != 1 || a->n <= 0 || a->x_nchw_f32) return false;
  if (transposed) return a->c == RG_C && a->h == RG_H && a->w == RG_H && a->k == RG_CP && a->p == 2 * RG_H && a->q == 2 * RG_H;
  return a->k == RG_C && a->c == RG_CP && a->h == 2 * RG_H && a->w == 2 * RG_H && a->p == RG_H && a->q == RG_H;
}

// act of the wide side: none or LeakyReLU (slope returned; 1 = none)
bool rgb_act(const vae_xform& x, float* slope) {
  if (x.kind == VAE_X_NONE) { *slope = 1.f; return true; }
  if (x.kind == VAE_X_ACT) { *slope = x.slope; return true; }
  return false;
}

constexpr int kRgbGrid = 256;                         // backward workgroups (one round), tiles in turn

}  // namespace

int rgb_out_fwd_launch(const vae_conv_args* a, const vae_recon_args* rc, hipStream_t st) {
  float slope;
  if (!rgb_geom(a, true) || !rgb_act(a->x_xf, &slope) || !a->x || !a->wt || !a->bias || a->residual ||
      a->bn_finalize || a->y_sum || !al16(a->x))
    return kHeadFallback;
  if (!rc || rc->n != a->n || rc->c != 3 || rc->h != 2 * RG_H || rc->w != 2 * RG_H || (rc->ld != 0 && rc->ld != RG_CP) ||
      !rc->target || !rc->recon || (rc->dy && !al16(rc->dy)))
    return kHeadFallback;
  RgbFwd q;
  q.n = a->n;
  q.x = static_cast<const __bf16*>(a->x); q.slope = slope;
  q.wt = static_cast<const __bf16*>(a->wt); q.bias = a->bias;
  q.target = rc->target; q.recon = rc->recon; q.sse = rc->sse;
  q.dy = static_cast<__bf16*>(rc->dy); q.grad_scale = rc->grad_scale; q.grad_recon = rc->grad_recon;
  VAE_LAUNCH(rgb_out_fwd_kernel, dim3((unsigned)(a->n * (RG_H / RG_TI))), dim3(RF_T), 0, st, q);
  return check_launch("rgb_out_fwd");
}

int rgb_out_bwd_launch(const vae_conv_args* a, hipStream_t st) {
  float slope, es = 1.f;
  if (!rgb_geom(a, true) || !rgb_act(a->x_xf, &slope) || !a->dy || !a->x || !a->wt || !a->dx || !a->dw ||
      a->dy_xf.kind != VAE_X_NONE || a->residual || a->bn_finalize || !al16(a->x) || !al16(a->dx) || !al16(a->dy))
    return kHeadFallback;
  // the data gradient's epilogue is the input's LeakyReLU backward (aux = x) or none, matching x_xf
  if (a->dx_epi.kind == VAE_X_ACT) {
    if (a->dx_epi.aux != a->x || a->dx_epi.slope != slope) return kHeadFallback;
    es = slope;
  } else if (a->dx_epi.kind != VAE_X_NONE || slope != 1.f) {
    return kHeadFallback;
  }
  (void)es;
  if (a->dw_inner != 3) return kHeadFallback;         // dW straight into the parameter's [c][4][4][3]
  const int tiles = a->n * (RG_H / RG_TI);
  const int per = (tiles + kRgbGrid - 1) / kRgbGrid;
  const int grid = (tiles + per - 1) / per;
  if (!a->workspace && !querying()) return kHeadFallback;
  if (!ws_fits((long)grid * RG_SLAB * 4, a->workspace_bytes, "rgb_out_bwd partials")) return VAE_E_BADARG;
  RgbBwd q;
  q.n = a->n; q.tiles = tiles; q.per = per;
  q.dy = static_cast<const __bf16*>(a->dy);
  q.x = static_cast<const __bf16*>(a->x); q.slope = slope;
  q.wt = static_cast<const __bf16*>(a->wt);
  q.dx = static_cast<__bf16*>(a->dx);
  q.slab = static_cast<float*>(a->workspace);
  VAE_LAUNCH(rgb_out_bwd_kernel, dim3((unsigned)grid), dim3(RB_T), 0, st, q);
  if (int rc = check_launch("rgb_out_bwd")) return rc;
  VAE_LAUNCH(rgb_slab_reduce, dim3((RG_C * 48 + 3 + RS_COLS - 1) / RS_COLS), dim3(256), 0, st, (const float*)q.slab, grid,
             a->dw, a->db, 3);
  return check_launch("rgb_slab_reduce");
}

int rgb_in_wgrad_launch(const vae_conv_args* a, hipStream_t st) {
  if (!rgb_geom(a, false) || !a->dy || !a->x || !a->dw || a->dy_xf.kind != VAE_X_NONE || a->x_xf.kind != VAE_X_NONE ||
      !al16(a->dy) || ((uintptr_t)a->x & 7) || a->dw_inner != 3)
    return kHeadFallback;
  const int tiles = a->n * (RG_H / RG_TI);
  const int per = (tiles + kRgbGrid - 1) / kRgbGrid;
  const int grid = (tiles + per - 1) / per;
  if (!a->workspace && !querying()) return kHeadFallback;
  if (!ws_fits((long)grid * RG_SLAB * 4, a->workspace_bytes, "rgb_in_wgrad partials")) return VAE_E_BADARG;
  RgbIn q;
  q.n = a->n; q.tiles = tiles; q.per = per;
  q.dy = static_cast<const __bf16*>(a->dy);
  q.x = static_cast<const __bf16*>(a->x);
  q.slab = static_cast<float*>(a->workspace);
  VAE_LAUNCH(rgb_in_wgrad_kernel, dim3((unsigned)grid), dim3(RB_T), 0, st, q);
  if (int rc = check_launch("rgb_in_wgrad")) return rc;
  VAE_LAUNCH(rgb_slab_reduce, dim3((RG_C * 48 + RG_C + RS_COLS - 1) / RS_COLS), dim3(256), 0, st, (const float*)q.slab,
             grid, a->dw, a->db, a->db ? RG_C : 0);
  return check_launch("rgb_slab_reduce");
}

}  // namespace vae

// The output ConvTranspose2d fused with Tanh + reconstruction (vaehip.h): the dedicated kernel for
// the VQ-VAE's packed RGB end, else vae_convT2d_fwd then vae_recon_fwd.
extern "C" int vae_convT2d_fwd_recon(const vae_conv_args* a, const vae_recon_args* rc, void* stream) {
  if (!vae::geom_ok_rgb(a)) return vae::fail(VAE_E_BADARG, "convT2d_fwd_recon: bad geometry");
  const int r = vae::rgb_out_fwd_launch(a, rc, (hipStream_t)stream);
  if (r != vae::kHeadFallback) return r;
  if (!a->y) return vae::fail(VAE_E_UNSUPPORTED, "convT2d_fwd_recon: shape not on the fused kernel and no y to stage");
  if (int e = vae_convT2d_fwd(a, stream)) return e;
  return vae_recon_fwd(rc, stream);
}
