// The decoder's last ConvTranspose2d at full resolution — final_layer.0 of models/vanilla_vae.py:64-70
// (ConvTranspose2d(32, 32, k3, s2, p1, op1): [B,32,32,32] -> [B,32,64,64]) — as kernels of its own.
//
// Why: it is the step's largest tensor (the 64x64x32 output, 16.8 MB bf16 at B=64) and the
// generic conv-GEMM (vae_cgemm.hpp) ran it as 2048 small phase tiles in two rounds of workgroups
// with a per-tile prologue (26.5 us, profiles/r2_v3_kernel_breakdown.txt) against ~3 us of HBM
// traffic.  Here one workgroup owns a band of 4 input rows of one image = 8 full output rows:
//   * the input band (+1 halo row and column) is loaded once, BatchNorm+LeakyReLU applied once,
//     and kept in LDS as bf16 with the 16-byte channel chunks XOR-swizzled by column;
//   * the 9 taps x 32 x 32 weights live in registers as MFMA B fragments (wt_t, [co][r][s][ci]);
//   * each wave computes its input row's two output rows phase by phase: output pixel
//     (2i+ph, 2j+pw) gathers taps r in {1} (ph 0) or {0 -> row i+1, 2 -> row i} (ph 1), same for
//     columns: 16 consecutive j of one phase are one v_mfma_f32_16x16x32_bf16 per tap and
//     16-channel half (K = the 32 input channels of the tap);
//   * the epilogue adds the bias, accumulates the next BatchNorm's Σ / Σ² from the fp32
//     accumulators (the producer contract of vaehip.h y_sum), and stores the rows through LDS as
//     whole 4 KB rows (16 B per lane).
#include "vae_launch.hpp"
#include "vae_rgb.hpp"

namespace vae {
namespace {

constexpr int HC = 32;                     // channels in and out
constexpr int HIN = 32;                    // input height / width (output 64 x 64)
constexpr int HOUT = 2 * HIN;
constexpr int IR = 4;                      // input rows per workgroup (one per wave)
constexpr int TROWS = IR + 1, TCOLS = HIN + 1;
constexpr int TOCT = TROWS * TCOLS * (HC / 8);      // 16-byte octets of the input band
constexpr int TOCT_PT = (TOCT + 255) / 256;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct HiresF {
  int n;
  const __bf16* x; vae_xform xf;           // layer input (pre-BN) and its transform
  const __bf16* wt_t;                      // [co][r][s][ci] bf16 (vaehip.h wt_t)
  const float* bias;                       // [co] or NULL
  __bf16* y;                               // [n][64][64][co]
  float* sum; float* sumsq; int reps, rstride;
};

__device__ __forceinline__ int band_off(int trow, int tcol, int chunk) {
  return (trow * TCOLS + tcol) * (HC * 2) + ((chunk ^ (tcol & 3)) << 4);
}

__global__ void __launch_bounds__(256) hires_convT_fwd_kernel(const HiresF q) {
  kernarg_prefetch<(sizeof(HiresF) < 1024 ? sizeof(HiresF) : 1024)>();
  __shared__ __attribute__((aligned(16))) char band[TROWS * TCOLS * HC * 2];
  __shared__ __attribute__((aligned(16))) __bf16 stage[4][2 * HOUT * HC];    // per wave: its 2 output rows
  __shared__ float tabs[3 * (HC + 8)];
  __shared__ float scr[4 * 256];
  __shared__ float part[4][2][HC];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bands = HIN / IR;
  const int n = blockIdx.x / bands, i0 = (blockIdx.x - n * bands) * IR;

  // ---- the input band's raw octets (row i0 + IR and column HIN are the zero halo)
  const rsrc_t rx = make_rsrc(q.x, (uint32_t)((long)q.n * HIN * HIN * HC * 2));
  u32x4 raw[TOCT_PT];
#pragma unroll
  for (int j = 0; j < TOCT_PT; ++j) {
    const int o = tid + 256 * j;
    const int pix = o >> 2, ch = o & 3;
    const int trow = pix / TCOLS, tcol = pix - trow * TCOLS;
    const int hi = i0 + trow;
    const bool ok = o < TOCT && hi < HIN && tcol < HIN;
    const uint32_t off = ok ? (uint32_t)((((n * HIN + hi) * HIN + tcol) * HC + ch * 8) * 2) : kOOB;
    raw[j] = __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0);
  }
  // ---- B fragments: W'[co][r][s][ci], lane: co = 16 nf + (lane & 15), ci = 8 (lane >> 4) .. +7
  const rsrc_t rw = make_rsrc(q.wt_t, (uint32_t)(HC * 9 * HC * 2));
  bf16x8 bw[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int nf = 0; nf < 2; ++nf) {
      const int co = nf * 16 + (lane & 15);
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rw, (uint32_t)(((co * 9 + t) * HC + 8 * (lane >> 4)) * 2), 0, 0);
      bw[t][nf] = *reinterpret_cast<const bf16x8*>(&v);
    }
  const float bco[2] = {q.bias ? q.bias[lane & 15] : 0.f, q.bias ? q.bias[16 + (lane & 15)] : 0.f};
  // ---- transform table (BatchNorm: built from the producer's statistics; the first workgroup
  //      applies the running-statistic update, as every forward consumer of a BatchNorm does)
  const int ts = HC + 8;
  const Tab ta{tabs, tabs + ts, tabs + 2 * ts, nullptr, nullptr};
  const bool bn = q.xf.kind == VAE_X_BN_ACT;
  if (bn) tab_fill(q.xf, ta, false, blockIdx.x == 0, scr);
  __syncthreads();
  // ---- act = lrelu(a*y + b) (0 in the halo) -> bf16 band
#pragma unroll
  for (int j = 0; j < TOCT_PT; ++j) {
    const int o = tid + 256 * j;
    if (o >= TOCT) continue;
    const int pix = o >> 2, ch = o & 3;
    const int trow = pix / TCOLS, tcol = pix - trow * TCOLS;
    const bool ok = i0 + trow < HIN && tcol < HIN;
    u32x4 out;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c0 = ch * 8 + 2 * e;
      float lo = __uint_as_float(raw[j][e] << 16), hi = __uint_as_float(raw[j][e] & 0xffff0000u);
      if (bn) { lo = fmaf(lo, ta.a[c0], ta.b[c0]); hi = fmaf(hi, ta.a[c0 + 1], ta.b[c0 + 1]); }
      if (q.xf.kind != VAE_X_NONE) { lo = fmaxf(lo, lo * q.xf.slope); hi = fmaxf(hi, hi * q.xf.slope); }
      bf16x2 pk; pk[0] = (__bf16)(ok ? lo : 0.f); pk[1] = (__bf16)(ok ? hi : 0.f);
      out[e] = *reinterpret_cast<uint32_t*>(&pk);
    }
    *reinterpret_cast<u32x4*>(band + band_off(trow, tcol, ch)) = out;
  }
  __syncthreads();

  // ---- wave `wave`: input row i = i0 + wave -> output rows 2i (ph 0) and 2i + 1 (ph 1)
  const int li = lane & 15, g = lane >> 4;
  float s1[2] = {0.f, 0.f}, s2[2] = {0.f, 0.f};
  __bf16* st = stage[wave];
#pragma unroll
  for (int ph = 0; ph < 2; ++ph)
#pragma unroll
    for (int pw = 0; pw < 2; ++pw)
#pragma unroll
      for (int j0 = 0; j0 < HIN; j0 += 16) {
        f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
        // taps of a phase: ph 0 -> r = 1 (row i); ph 1 -> r = 0 (row i + 1), r = 2 (row i)
#pragma unroll
        for (int a = 0; a < (ph ? 2 : 1); ++a) {
          const int r = ph ? 2 * a : 1, dh = (ph && a == 0) ? 1 : 0;
#pragma unroll
          for (int b = 0; b < (pw ? 2 : 1); ++b) {
            const int s = pw ? 2 * b : 1, dw = (pw && b == 0) ? 1 : 0;
            const bf16x8 av = *reinterpret_cast<const bf16x8*>(band + band_off(wave + dh, j0 + li + dw, g));
#pragma unroll
            for (int nf = 0; nf < 2; ++nf)
              acc[nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bw[r * 3 + s][nf], acc[nf], 0, 0, 0);
          }
        }
        // lane: channel co = 16 nf + li, pixels j = j0 + 4g + e of output row 2i + ph, col 2j + pw
#pragma unroll
        for (int nf = 0; nf < 2; ++nf) {
          const int co = nf * 16 + li;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float v = acc[nf][e];
            s1[nf] += v;
            s2[nf] = fmaf(v, v, s2[nf]);
            const int ow = 2 * (j0 + 4 * g + e) + pw;
            st[(ph * HOUT + ow) * HC + co] = (__bf16)(v + bco[nf]);
          }
        }
      }
  __builtin_amdgcn_wave_barrier();
  // ---- the wave's two output rows: 2 x 4 KB contiguous, 16 B per lane
  const long row0 = ((long)n * HOUT + 2 * (i0 + wave)) * HOUT * HC;
#pragma unroll
  for (int it = 0; it < 2 * HOUT * HC / 8 / 64; ++it) {
    const int e8 = (it * 64 + lane) * 8;
    *reinterpret_cast<u32x4*>(q.y + row0 + e8) = *reinterpret_cast<const u32x4*>(st + e8);
  }
  // ---- BatchNorm statistics of the output (pre-bias accumulators), one replica per workgroup
  if (q.sum) {
#pragma unroll
    for (int nf = 0; nf < 2; ++nf) {
      float a = s1[nf], b = s2[nf];
      a += __shfl_xor(a, 16); a += __shfl_xor(a, 32);
      b += __shfl_xor(b, 16); b += __shfl_xor(b, 32);
      if (g == 0) { part[wave][0][nf * 16 + li] = a; part[wave][1][nf * 16 + li] = b; }
    }
    __syncthreads();
    if (tid < HC) {
      const long roff = q.reps > 1 ? (long)(blockIdx.x % q.reps) * q.rstride : 0;
      atomicAdd(q.sum + roff + tid, (part[0][0][tid] + part[1][0][tid]) + (part[2][0][tid] + part[3][0][tid]));
      atomicAdd(q.sumsq + roff + tid, (part[0][1][tid] + part[1][1][tid]) + (part[2][1][tid] + part[3][1][tid]));
    }
  }
}


// ======================================================================= backward
// One pass over dY for both gradients of the layer (the layer's data and weight gradients read
// the same 2 x 16.8 MB of dy and its pre-BN output — before, two launches read them twice):
//   dY' = BN-backward(dy, y) (vaehip.h BN_DY: A*g + B*y + C), loaded once per tile into LDS,
//         the output columns de-interleaved by parity so the stride-2 gathers are contiguous;
//   data:   dx[i, j, ci] = Σ_{r,s,co} dY'[2i-1+r, 2j-1+s, co] W[ci][r][s][co]  (M = 16 pixels of
//           one input row, N = 32 ci, K = 9 taps x 32 co), epilogue: the input BatchNorm+LeakyReLU
//           backward (dx_epi, as the conv-GEMM's E_BNBWD) with its Σg, Σg·x̂, rows stored whole;
//   filter: dW[ci][r][s][co] += Σ_{i,j} act[i, j, ci] dY'[2i-1+r, 2j-1+s, co] (M = 32 ci, N = 32
//           co per tap, K = the tile's pixels), both operands read transposed from LDS
//           (ds_read_b64_tr_b16); accumulated in registers over the workgroup's tiles and written
//           as one row of a slab that wg_slab_reduce sums in fixed order (deterministic).
// Tile: 4 input rows of one image (one per wave) = output rows 2*i0-1 .. 2*i0+7 (9 rows x 65
// columns of dY' with the -1 halo).
constexpr int DROWS = 2 * IR + 1;                  // dY' rows of a tile
constexpr int DIDX = HIN + 1;                      // columns per parity (index j + (s == 2))
constexpr int DOCT = DROWS * 2 * DIDX * (HC / 8);  // 16-byte octets of the dY' tile
constexpr int DOCT_PT = (DOCT + 255) / 256;        // 10
constexpr int DROUND = 5;                          // octets per thread per load round
constexpr int NW = HC * 9 * HC;                    // dW entries

struct HiresB {
  int n, tiles;
  const __bf16* dy; vae_xform dxf;          // dy (g of the next BatchNorm) and its BN_DY (aux = y)
  const __bf16* x; vae_xform xxf;           // layer input (pre-BN) and its BatchNorm+LeakyReLU
  const __bf16* wt;                         // native [ci][r][s][co] bf16
  __bf16* dx; vae_xform exf;                // data gradient and its epilogue (BN_ACT, aux = x)
  float* dgamma; float* dbeta; int reps, rstride;
  float* slab;                              // [gridDim.x][NW] filter partials
  float* db;                                // closed-form bias gradient (workgroup 0)
};

__device__ __forceinline__ int dy_off(int tr, int par, int idx, int chunk) {
  return ((tr * 2 + par) * DIDX + idx) * (HC * 2) + ((chunk ^ ((idx >> 2) & 3)) << 4);
}
__device__ __forceinline__ int px_off(int pix, int chunk) {            // [pixel][32 ch] tiles
  return pix * (HC * 2) + ((chunk ^ ((pix >> 1) & 3)) << 4);
}
typedef __bf16 __attribute__((ext_vector_type(4))) __attribute__((address_space(3))) hr_lds_bf16x4;
typedef __bf16 hr_bf16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ hr_bf16x4 hr_tr_read(const char* generic_lds_addr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((hr_lds_bf16x4*)(uintptr_t)(uint32_t)(uintptr_t)generic_lds_addr);
}

__global__ void __launch_bounds__(256) hires_convT_bwd_kernel(const HiresB q) {
  kernarg_prefetch<(sizeof(HiresB) < 1024 ? sizeof(HiresB) : 1024)>();
  __shared__ __attribute__((aligned(16))) char dyt[DROWS * 2 * DIDX * HC * 2];     // dY' (bf16)
  __shared__ __attribute__((aligned(16))) char actt[IR * HIN * HC * 2];            // act of the tile
  __shared__ __attribute__((aligned(16))) char yt[IR * HIN * HC * 2];              // raw x of the tile
  __shared__ __attribute__((aligned(16))) __bf16 dstage[4][HIN * HC];              // per wave: its dx row
  __shared__ float tdy[3 * (HC + 8)], tx[3 * (HC + 8)], te[5 * (HC + 8)];
  __shared__ float scr[4 * 256];
  __shared__ float part[4][2][HC];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int ts = HC + 8;
  const Tab Tdy{tdy, tdy + ts, tdy + 2 * ts, nullptr, nullptr};
  const Tab Tx{tx, tx + ts, tx + 2 * ts, nullptr, nullptr};
  const Tab Te{te, te + ts, nullptr, te + 3 * ts, te + 4 * ts};
  const uint32_t ybytes = (uint32_t)((long)q.n * HOUT * HOUT * HC * 2);
  const rsrc_t rdy = make_rsrc(q.dy, ybytes), ry = make_rsrc(q.dxf.aux, ybytes);
  const rsrc_t rx = make_rsrc(q.x, (uint32_t)((long)q.n * HIN * HIN * HC * 2));

  // B fragments of the data gradient: W[ci = 16 nf + li][tap][co = 8 g .. +7]
  bf16x8 bw[9][2];
  {
    const rsrc_t rw = make_rsrc(q.wt, (uint32_t)(NW * 2));
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int nf = 0; nf < 2; ++nf) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rw, (uint32_t)((((nf * 16 + li) * 9 + t) * HC + 8 * g) * 2), 0, 0);
        bw[t][nf] = *reinterpret_cast<const bf16x8*>(&v);
      }
  }
  tab_fill(q.dxf, Tdy, false, false, scr);
  tab_fill(q.xxf, Tx, false, false, scr);
  tab_fill(q.exf, Te, true, false, scr);
  if (blockIdx.x == 0 && (q.db || q.dxf.dgamma_out || q.dxf.dbeta_out)) closed_form_db(q.dxf, q.db);
  const bool xbn = q.xxf.kind == VAE_X_BN_ACT, ebn = q.exf.kind == VAE_X_BN_ACT;

  // filter accumulators: this wave's taps t = wave + 4 u (9 taps over 4 waves), [u][mf][nf]
  f32x4 accw[3][2][2];
#pragma unroll
  for (int u = 0; u < 3; ++u)
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) accw[u][a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  float es1[2] = {0.f, 0.f}, es2[2] = {0.f, 0.f};

  for (int tile = blockIdx.x; tile < q.tiles; tile += gridDim.x) {
    const int n = tile / (HIN / IR), i0 = (tile - n * (HIN / IR)) * IR;
    __syncthreads();                      // the previous tile's LDS reads are done (and tables built)
    // ---- x band: act and raw y of the tile's 4 x 32 input pixels (2 octets per thread)
    {
      u32x4 xr[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int o = tid + 256 * k, pix = o >> 2, ch = o & 3;
        const int ii = pix / HIN, jj = pix - ii * HIN;
        xr[k] = __builtin_amdgcn_raw_buffer_load_b128(rx, (uint32_t)((((n * HIN + i0 + ii) * HIN + jj) * HC + ch * 8) * 2), 0, 0);
      }
      // ---- dY' in load rounds of DROUND octets per thread (g and y issued together)
#pragma unroll
      for (int r0 = 0; r0 < DOCT_PT; r0 += DROUND) {
        u32x4 gv[DROUND], yv[DROUND];
#pragma unroll
        for (int k = 0; k < DROUND; ++k) {
          const int o = tid + 256 * (r0 + k);
          const int pos = o >> 2, ch = o & 3;                   // pos = (tr * 2 + par) * DIDX + idx
          const int tr = pos / (2 * DIDX), rem = pos - tr * 2 * DIDX, par = rem / DIDX, idx = rem - par * DIDX;
          const int oh = 2 * i0 - 1 + tr, ow = 2 * idx + par - 1;
          const bool ok = o < DOCT && oh >= 0 && oh < HOUT && ow >= 0 && ow < HOUT;
          const uint32_t off = ok ? (uint32_t)((((n * HOUT + oh) * HOUT + ow) * HC + ch * 8) * 2) : kOOB;
          gv[k] = __builtin_amdgcn_raw_buffer_load_b128(rdy, off, 0, 0);
          yv[k] = __builtin_amdgcn_raw_buffer_load_b128(ry, off, 0, 0);
        }
#pragma unroll
        for (int k = 0; k < DROUND; ++k) {
          const int o = tid + 256 * (r0 + k);
          if (o >= DOCT) continue;
          const int pos = o >> 2, ch = o & 3;
          const int tr = pos / (2 * DIDX), rem = pos - tr * 2 * DIDX, par = rem / DIDX, idx = rem - par * DIDX;
          const int oh = 2 * i0 - 1 + tr, ow = 2 * idx + par - 1;
          const bool ok = oh >= 0 && oh < HOUT && ow >= 0 && ow < HOUT;
          u32x4 out;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int c0 = ch * 8 + 2 * e;
            const float g0 = __uint_as_float(gv[k][e] << 16), g1 = __uint_as_float(gv[k][e] & 0xffff0000u);
            const float y0 = __uint_as_float(yv[k][e] << 16), y1 = __uint_as_float(yv[k][e] & 0xffff0000u);
            const float v0 = fmaf(Tdy.a[c0], g0, fmaf(Tdy.b[c0], y0, Tdy.c[c0]));
            const float v1 = fmaf(Tdy.a[c0 + 1], g1, fmaf(Tdy.b[c0 + 1], y1, Tdy.c[c0 + 1]));
            bf16x2 pk; pk[0] = (__bf16)(ok ? v0 : 0.f); pk[1] = (__bf16)(ok ? v1 : 0.f);
            out[e] = *reinterpret_cast<uint32_t*>(&pk);
          }
          *reinterpret_cast<u32x4*>(dyt + dy_off(tr, par, idx, ch)) = out;
        }
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int o = tid + 256 * k, pix = o >> 2, ch = o & 3;
        *reinterpret_cast<u32x4*>(yt + px_off(pix, ch)) = xr[k];
        u32x4 out;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c0 = ch * 8 + 2 * e;
          float lo = __uint_as_float(xr[k][e] << 16), hi = __uint_as_float(xr[k][e] & 0xffff0000u);
          if (xbn) { lo = fmaf(lo, Tx.a[c0], Tx.b[c0]); hi = fmaf(hi, Tx.a[c0 + 1], Tx.b[c0 + 1]); }
          if (q.xxf.kind != VAE_X_NONE) { lo = fmaxf(lo, lo * q.xxf.slope); hi = fmaxf(hi, hi * q.xxf.slope); }
          bf16x2 pk; pk[0] = (__bf16)lo; pk[1] = (__bf16)hi;
          out[e] = *reinterpret_cast<uint32_t*>(&pk);
        }
        *reinterpret_cast<u32x4*>(actt + px_off(pix, ch)) = out;
      }
    }
    __syncthreads();

    // ---- data gradient: wave -> input row i0 + wave, two groups of 16 pixels
    __bf16* st = dstage[wave];
#pragma unroll
    for (int j0 = 0; j0 < HIN; j0 += 16) {
      f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          // dY'[2i - 1 + r][2j - 1 + s]: tile row 2 wave + r, parity (s & 1), index j + (s == 2)
          const bf16x8 av = *reinterpret_cast<const bf16x8*>(dyt + dy_off(2 * wave + r, s & 1, j0 + li + (s == 2 ? 1 : 0), g));
#pragma unroll
          for (int nf = 0; nf < 2; ++nf)
            acc[nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bw[r * 3 + s][nf], acc[nf], 0, 0, 0);
        }
      // lane: ci = 16 nf + li, pixels j = j0 + 4 g + e of row i0 + wave
#pragma unroll
      for (int nf = 0; nf < 2; ++nf) {
        const int ci = nf * 16 + li;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int j = j0 + 4 * g + e, pix = wave * HIN + j;
          const float y = (float)*reinterpret_cast<const __bf16*>(yt + px_off(pix, ci >> 3) + (ci & 7) * 2);
          float gg = acc[nf][e];
          if (ebn) {
            const float z = fmaf(y, Te.a[ci], Te.b[ci]);
            gg = z > 0.f ? gg : gg * q.exf.slope;
            es1[nf] += gg;
            es2[nf] = fmaf(gg, fmaf(y, Te.p[ci], Te.q[ci]), es2[nf]);
          } else if (q.exf.kind == VAE_X_ACT) {
            gg = y > 0.f ? gg : gg * q.exf.slope;
          }
          st[j * HC + ci] = (__bf16)gg;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    {
      // the wave's dx row: 32 pixels x 64 B = 2 KB contiguous, 16 B per lane
      const long row = ((long)n * HIN + i0 + wave) * HIN * HC;
#pragma unroll
      for (int it = 0; it < HIN * HC / 8 / 64; ++it) {
        const int e8 = (it * 64 + lane) * 8;
        *reinterpret_cast<u32x4*>(q.dx + row + e8) = *reinterpret_cast<const u32x4*>(st + e8);
      }
    }

    // ---- filter gradient: K-step ks = input row i0 + ks (32 pixels); this wave's taps
#pragma unroll
    for (int ks = 0; ks < IR; ++ks) {
      bf16x8 af[2];
#pragma unroll
      for (int mf = 0; mf < 2; ++mf)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          // lane 4qq + pp of its 16-group: pixel 8 g + 4 h + qq, channels 16 mf + 4 pp .. +3
          const int pix = ks * HIN + 8 * g + 4 * h + (li >> 2), ch = 16 * mf + 4 * (li & 3);
          const hr_bf16x4 v = hr_tr_read(actt + px_off(pix, ch >> 3) + (ch & 7) * 2);
#pragma unroll
          for (int e = 0; e < 4; ++e) af[mf][4 * h + e] = v[e];
        }
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const int t = wave + 4 * u;
        if (t >= 9) continue;
        const int r = t / 3, s = t - 3 * r;
#pragma unroll
        for (int nf = 0; nf < 2; ++nf) {
          bf16x8 bf;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int j = 8 * g + 4 * h + (li >> 2), co = 16 * nf + 4 * (li & 3);
            const hr_bf16x4 v = hr_tr_read(dyt + dy_off(2 * ks + r, s & 1, j + (s == 2 ? 1 : 0), co >> 3) + (co & 7) * 2);
#pragma unroll
            for (int e = 0; e < 4; ++e) bf[4 * h + e] = v[e];
          }
#pragma unroll
          for (int mf = 0; mf < 2; ++mf)
            accw[u][mf][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mf], bf, accw[u][mf][nf], 0, 0, 0);
        }
      }
    }
  }

  // ---- this workgroup's filter partial: slab row blockIdx.x, dW layout [ci][tap][co]
  float* srow = q.slab + (long)blockIdx.x * NW;
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int t = wave + 4 * u;
    if (t >= 9) continue;
#pragma unroll
    for (int mf = 0; mf < 2; ++mf)
#pragma unroll
      for (int nf = 0; nf < 2; ++nf)
#pragma unroll
        for (int e = 0; e < 4; ++e) srow[(16 * mf + 4 * g + e) * (9 * HC) + t * HC + 16 * nf + li] = accw[u][mf][nf][e];
  }
  // ---- the input BatchNorm's backward sums (Σg, Σg·x̂), one replica per workgroup
  if (ebn) {
#pragma unroll
    for (int nf = 0; nf < 2; ++nf) {
      float a = es1[nf], b = es2[nf];
      a += __shfl_xor(a, 16); a += __shfl_xor(a, 32);
      b += __shfl_xor(b, 16); b += __shfl_xor(b, 32);
      if (g == 0) { part[wave][0][nf * 16 + li] = a; part[wave][1][nf * 16 + li] = b; }
    }
    __syncthreads();
    if (tid < HC) {
      const long roff = q.reps > 1 ? (long)(blockIdx.x % q.reps) * q.rstride : 0;
      atomicAdd(q.dbeta + roff + tid, (part[0][0][tid] + part[1][0][tid]) + (part[2][0][tid] + part[3][0][tid]));
      atomicAdd(q.dgamma + roff + tid, (part[0][1][tid] + part[1][1][tid]) + (part[2][1][tid] + part[3][1][tid]));
    }
  }
}

// dw += Σ_rows slab[row][c]: 16 columns x 16 row groups per workgroup (64-byte row segments,
// each thread's loads all in flight), the row groups combined in a fixed order (deterministic).
constexpr int SR_COLS = 16, SR_GROUPS = 16;
__global__ void __launch_bounds__(256) hires_slab_reduce(const float* slab, int rows, float* dw) {
  __shared__ float red[SR_GROUPS][SR_COLS];
  const int cl = threadIdx.x % SR_COLS, rg = threadIdx.x / SR_COLS;
  const int c = blockIdx.x * SR_COLS + cl;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int r0 = rg; r0 < rows; r0 += 4 * SR_GROUPS) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int r = r0 + u * SR_GROUPS;
      v[u] = (r < rows && c < NW) ? slab[(long)r * NW + c] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] += v[u];
  }
  red[rg][cl] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  __syncthreads();
  if (rg == 0 && c < NW) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < SR_GROUPS; ++i) t += red[i][cl];
    dw[c] += t;
  }
}

constexpr int kHiresBwdGrid = 256;

}  // namespace

// The shapes these kernels take (checked on the host; the caller falls back otherwise):
// bf16, 32 -> 32 channels, 32x32 -> 64x64, k3 s2 p1 (op1), 16-byte aligned NHWC tensors.
bool hires_convT_ok(const vae_conv_args* a) {
  return a->dtype == VAE_BF16 && a->c == HC && a->k == HC && a->h == HIN && a->w == HIN && a->p == HOUT &&
         a->q == HOUT && a->r == 3 && a->stride == 2 && a->pad == 1 && a->n > 0 && !a->x_nchw_f32 &&
         ((uintptr_t)a->x & 15) == 0 && (a->x_xf.kind == VAE_X_NONE || a->x_xf.kind == VAE_X_ACT ||
                                          (a->x_xf.kind == VAE_X_BN_ACT && a->x_xf.channels == HC));
}

int hires_convT_fwd_launch(const vae_conv_args* a, hipStream_t st) {
  if (!hires_convT_ok(a) || !a->wt_t || ((uintptr_t)a->wt_t & 15) || ((uintptr_t)a->y & 15) || a->residual ||
      a->bn_finalize)
    return kHeadFallback;
  if (a->x_xf.kind == VAE_X_BN_ACT && !a->x_xf.table && !bn_fast_ok(a->x_xf)) return kHeadFallback;
  HiresF q;
  memset(&q, 0, sizeof(q));
  q.n = a->n;
  q.x = static_cast<const __bf16*>(a->x); q.xf = a->x_xf;
  q.wt_t = static_cast<const __bf16*>(a->wt_t); q.bias = a->bias;
  q.y = static_cast<__bf16*>(a->y);
  q.sum = a->y_sum; q.sumsq = a->y_sumsq;
  q.reps = a->sum_reps; q.rstride = a->sum_rstride;
  VAE_LAUNCH(hires_convT_fwd_kernel, dim3((unsigned)(a->n * (HIN / IR))), dim3(256), 0, st, q);
  return check_launch("hires_convT_fwd");
}


// The fused backward of the layer (dgrad + wgrad); kHeadFallback when the shapes / transforms are
// not these kernels' (the caller then runs vae_convT2d_bwd_data and vae_convT2d_bwd_filter).
int hires_convT_bwd_launch(const vae_conv_args* a, hipStream_t st) {
  if (!hires_convT_ok(a) || !a->dy || !a->dx || !a->dw || !a->wt || a->residual || a->bn_finalize) return kHeadFallback;
  if (a->dy_xf.kind != VAE_X_BN_DY || a->dy_xf.channels != HC || a->dy_xf.table || !bn_fast_ok(a->dy_xf) ||
      !a->dy_xf.aux || ((uintptr_t)a->dy_xf.aux & 15) || ((uintptr_t)a->dy & 15) || ((uintptr_t)a->dx & 15) ||
      ((uintptr_t)a->wt & 15))
    return kHeadFallback;
  if (a->db && a->dy_xf.kind != VAE_X_BN_DY) return kHeadFallback;
  const vae_xform& e = a->dx_epi;
  if (!(e.kind == VAE_X_NONE || (e.kind == VAE_X_ACT && e.aux == a->x) ||
        (e.kind == VAE_X_BN_ACT && e.aux == a->x && e.channels == HC && !e.table && bn_fast_ok(e) && a->dx_dgamma && a->dx_dbeta)))
    return kHeadFallback;
  if (a->x_xf.kind == VAE_X_BN_ACT && (a->x_xf.table || !bn_fast_ok(a->x_xf))) return kHeadFallback;
  const int tiles = a->n * (HIN / IR);
  const int gmax = kHiresBwdGrid;
  const int grid = tiles < gmax ? tiles : gmax;
  const long need = (long)grid * NW * 4;
  if (!a->workspace && !querying()) return kHeadFallback;
  if (!ws_fits(need, a->workspace_bytes, "convT2d_bwd filter partials")) return VAE_E_BADARG;
  HiresB q;
  memset(&q, 0, sizeof(q));
  q.n = a->n; q.tiles = tiles;
  q.dy = static_cast<const __bf16*>(a->dy); q.dxf = a->dy_xf;
  q.x = static_cast<const __bf16*>(a->x); q.xxf = a->x_xf;
  q.wt = static_cast<const __bf16*>(a->wt);
  q.dx = static_cast<__bf16*>(a->dx); q.exf = e;
  q.dgamma = a->dx_dgamma; q.dbeta = a->dx_dbeta; q.reps = a->sum_reps; q.rstride = a->sum_rstride;
  q.slab = static_cast<float*>(a->workspace);
  q.db = a->db;
  VAE_LAUNCH(hires_convT_bwd_kernel, dim3((unsigned)grid), dim3(256), 0, st, q);
  if (int rc = check_launch("hires_convT_bwd")) return rc;
  if (a->defer_reduce)                      // the filter partials stay for vae_adam_step_ex
    return defer_slab(a->dw, NW, q.slab, grid, NW) ? VAE_OK : VAE_E_UNSUPPORTED;
  VAE_LAUNCH(hires_slab_reduce, dim3((NW + SR_COLS - 1) / SR_COLS), dim3(256), 0, st, (const float*)q.slab, grid, a->dw);
  return check_launch("hires_slab_reduce");
}

}  // namespace vae

// Both gradients of a ConvTranspose2d in one call (vaehip.h): the fused full-resolution kernel when
// the layer is the decoder's last one, else vae_convT2d_bwd_data then vae_convT2d_bwd_filter.
extern "C" int vae_convT2d_bwd(const vae_conv_args* a, void* stream) {
  if (!vae::geom_ok(a, "convT2d_bwd")) return VAE_E_BADARG;
  if (!a->dy || !a->x || !a->dw || !a->dx || !a->wt) return vae::fail(VAE_E_BADARG, "convT2d_bwd: null tensor");
  if (a->dtype == VAE_BF16) {
    int rc = vae::rgb_out_bwd_launch(a, (hipStream_t)stream);     // the VQ-VAE's output ConvT(C -> 3)
    if (rc != vae::kHeadFallback) return rc;
    rc = vae::hires_convT_bwd_launch(a, (hipStream_t)stream);
    if (rc != vae::kHeadFallback) return rc;
  }
  if (int rc = vae_convT2d_bwd_data(a, stream)) return rc;
  return vae_convT2d_bwd_filter(a, stream);
}
