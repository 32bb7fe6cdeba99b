// The VAE bottleneck in bf16 (vaehip.h vae_latent_*): fc_mu|fc_var, reparameterize and
// decoder_input (models/vanilla_vae.py:36-37, :43, :85-92, :101-102, :107-117) and their backward,
// in two launches each way instead of nine (profiles/r3a: fc split-K GEMM + finalize + reparam +
// decoder_input forward 23 us; decoder_input bwd_data + finalize + bwd_filter, fc bwd_data +
// bwd_filter 39 us).
//
// Every GEMM here is tiny (M = batch rows <= a few hundred, N <= 2048, K <= 2048: 17-67 MFLOP), so a
// workgroup's time is its chain of dependent memory round trips (~1-2 us each from a cold L2), not
// its arithmetic.  The kernels are built to pay ONE round trip before the MFMAs:
//   - every global load of a workgroup (operands, BatchNorm statistics of all replicas, and the
//     epilogue's inputs: mu / log-var / eps rows, the old weight-gradient values) is issued up front
//     into registers, with compile-time trip counts so that nothing waits on a previous load;
//   - operands land in LDS as k-contiguous bf16 rows (the v_mfma_f32_16x16x32_bf16 fragment layout),
//     transposed on the way in where the source is stored the other way round (lanes take
//     consecutive source rows, so the 2-byte transposed LDS stores of a wave fill whole rows);
//   - the long K of fc_mu|fc_var (4*C = 2048) and of the decoder_input data gradient (2048) is split
//     over workgroups whose partial sums meet with fp32 atomics in outputs that are zero on entry
//     (mulv, d[mu|logvar]); the reparameterization backward is linear in dz, so each slice applies it
//     to its own partial and slice 0 adds the KL seed.  Tiles are sized so that a workgroup issues
//     at most 32 atomic wave-instructions (an atomic wave-instruction costs ~50 ns of a CU's time,
//     MI355X_MICROARCH.md atomics), spread over 64-128 workgroups;
//   - independent GEMMs of one direction share a launch as block ranges (decoder_input's data and
//     weight gradients; fc's data and weight gradients).
#include "vae_common.hpp"

namespace vae {
namespace {

constexpr int LT_RPR = 8;             // replicas of a BatchNorm statistic read per round

__device__ __forceinline__ bf16x8 to_bf16x8(const float (&v)[8]) {
  bf16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = (__bf16)v[e];
  return o;
}
__device__ __forceinline__ void unpack8(const uint4& u, float (&v)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[2 * e] = __uint_as_float(w[e] << 16);
    v[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
  }
}
__device__ __forceinline__ uint4 ld16(const void* p) { return *reinterpret_cast<const uint4*>(p); }
__device__ __forceinline__ f32x4 ld4f(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
constexpr uint4 kZero4 = {0u, 0u, 0u, 0u};

// Philox4x32-10 (Salmon et al., SC'11): 4 x 32 random bits per (counter, key)
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = uint4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}
// four N(0,1) draws for eps elements 4q..4q+3 of step `step` (Box-Muller on word pairs; u in (0, 1])
__device__ __forceinline__ f32x4 normal4(uint32_t q, uint32_t step, uint64_t seed) {
  const uint4 w = philox4x32_10(uint4{q, step, 0x5EEDu, 0u}, (uint32_t)seed, (uint32_t)(seed >> 32));
  constexpr float kInv = 2.3283064365386963e-10f;               // 2^-32
  const float u0 = ((float)w.x + 0.5f) * kInv, v0 = (float)w.y * kInv;
  const float u1 = ((float)w.z + 0.5f) * kInv, v1 = (float)w.w * kInv;
  const float r0 = sqrtf(-2.f * logf(u0)), r1 = sqrtf(-2.f * logf(u1));
  float s0, c0, s1, c1;
  sincosf(6.283185307179586f * v0, &s0, &c0);
  sincosf(6.283185307179586f * v1, &s1, &c1);
  return f32x4{r0 * c0, r0 * s0, r1 * c1, r1 * s1};
}

// One wave's 16-row x (16*TN)-column block of a tile, ksteps of 32, from k-contiguous LDS rows:
// A rows ar0.., B rows bc0.. (lda / ldb elements apart).
template <int TN>
__device__ __forceinline__ void mma_block(const __bf16* As, int lda, int ar0, const __bf16* Bs, int ldb, int bc0,
                                          int ksteps, f32x4 (&acc)[TN], int lane) {
  const __bf16* a = As + (ar0 + (lane & 15)) * lda + 8 * (lane >> 4);
  const __bf16* b = Bs + (bc0 + (lane & 15)) * ldb + 8 * (lane >> 4);
  for (int ks = 0; ks < ksteps; ++ks) {
    const bf16x8 af = *reinterpret_cast<const bf16x8*>(a + 32 * ks);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const bf16x8 bf = *reinterpret_cast<const bf16x8*>(b + j * 16 * ldb + 32 * ks);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, acc[j], 0, 0, 0);
    }
  }
}

// BatchNorm coefficients of channel c (training: batch statistics from the producer's replicated
// sums, every replica and gamma / beta / shift loaded in one round; or a precomputed table):
// act = lrelu(t*a + b), xhat = t*p + q.  Optionally updates the running statistics.
struct BnCoef { float a, b, p, q; };
__device__ __forceinline__ BnCoef bn_coef(const vae_xform& x, int c, bool update_running) {
  BnCoef k;
  if (x.table) {
    const int C = x.channels;
    k.a = x.table[c]; k.b = x.table[C + c]; k.p = x.table[2 * C + c]; k.q = x.table[3 * C + c];
    return k;
  }
  const int R = x.reps > 1 ? x.reps : 1;
  const long rs = x.reps > 1 ? x.rstride : 0;
  float ts = 0.f, tq = 0.f;
  const float g = x.gamma[c], be = x.beta[c], sh = x.shift ? x.shift[c] : 0.f;
  for (int r0 = 0; r0 < R; r0 += LT_RPR) {           // (R <= 8 replicas: one round)
    float s[LT_RPR], q[LT_RPR];
#pragma unroll
    for (int u = 0; u < LT_RPR; ++u) {
      const int rr = min(r0 + u, R - 1);
      s[u] = x.sum[rr * rs + c];
      q[u] = x.sumsq[rr * rs + c];
    }
#pragma unroll
    for (int u = 0; u < LT_RPR; ++u) {
      ts += r0 + u < R ? s[u] : 0.f;
      tq += r0 + u < R ? q[u] : 0.f;
    }
  }
  const float inv_m = 1.0f / x.count;
  const float s1 = ts * inv_m;
  const float var = fmaxf(tq * inv_m - s1 * s1, 0.0f);
  const float mean = s1 + sh;
  const float invstd = 1.0f / sqrtf(var + x.eps);
  k.a = g * invstd;
  k.b = be - mean * k.a;
  k.p = invstd;
  k.q = -mean * invstd;
  if (update_running && x.running_mean) {
    const float m = x.momentum;
    const float unb = x.count > 1.f ? var * x.count / (x.count - 1.f) : var;
    x.running_mean[c] = (1.f - m) * x.running_mean[c] + m * mean;
    x.running_var[c] = (1.f - m) * x.running_var[c] + m * unb;
  }
  return k;
}

// ------------------------------------------------------------------------------ fc forward
// grid (2D/32, in_features/128, ceil(batch/64)); tile 64 rows x 32 columns x one 128-deep K slice
// (one pixel's channels c0..c0+127 of the NHWC map: x_xf.channels % 128 == 0)
constexpr int FC_BK = 128, FC_LD = FC_BK + 8;
__global__ void __launch_bounds__(256) latent_fc_fwd_kernel(const vae_latent_args a) {
  kernarg_prefetch<(sizeof(vae_latent_args) < 1024 ? sizeof(vae_latent_args) : 1024)>();
  __shared__ __attribute__((aligned(16))) __bf16 As[64 * FC_LD];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[32 * FC_LD];
  __shared__ float ta[FC_BK], tb[FC_BK];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int K1 = a.in_features, D2 = 2 * a.latent, B = a.batch, C = a.x_xf.channels;
  const int n0 = blockIdx.x * 32, k0 = blockIdx.y * FC_BK, m0 = blockIdx.z * 64;
  const __bf16* x = static_cast<const __bf16*>(a.x);
  const __bf16* w1 = static_cast<const __bf16*>(a.w1);
  uint4 av[4], bv[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ch = tid + 256 * i, r = ch >> 4, kc = ch & 15, row = m0 + r;
    av[i] = row < B ? ld16(x + (long)row * K1 + k0 + 8 * kc) : kZero4;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ch = tid + 256 * i, r = ch >> 4, kc = ch & 15;
    bv[i] = ld16(w1 + (long)(n0 + r) * K1 + k0 + 8 * kc);
  }
  float bias[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) bias[j] = (blockIdx.y == 0 && a.b1) ? a.b1[n0 + 16 * j + (lane & 15)] : 0.f;
  const int c0 = k0 % C;
  if (tid < FC_BK) {
    // running statistics: once per channel, by the column-0 / row-0 workgroup of pixel 0's slices
    const bool run = blockIdx.x == 0 && blockIdx.z == 0 && k0 < C;
    const BnCoef k = bn_coef(a.x_xf, c0 + tid, run);
    ta[tid] = k.a; tb[tid] = k.b;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ch = tid + 256 * i, r = ch >> 4, kc = ch & 15;
    *reinterpret_cast<uint4*>(Bs + r * FC_LD + 8 * kc) = bv[i];
  }
  __syncthreads();
  const float sl = a.x_xf.slope;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ch = tid + 256 * i, r = ch >> 4, kc = ch & 15;
    float v[8];
    unpack8(av[i], v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = lrelu(fmaf(v[e], ta[8 * kc + e], tb[8 * kc + e]), sl);
    *reinterpret_cast<bf16x8*>(As + r * FC_LD + 8 * kc) = to_bf16x8(v);
  }
  __syncthreads();
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  mma_block<2>(As, FC_LD, 16 * wave, Bs, FC_LD, 0, FC_BK / 32, acc, lane);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n0 + 16 * j + (lane & 15);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = m0 + 16 * wave + 4 * (lane >> 4) + e;
      if (row < B) atomicAdd(a.mulv + (long)row * D2 + col, acc[j][e] + bias[j]);
    }
  }
}

// ------------------------------------------------------------------------------ decoder_input fwd
// grid (out_features/64, ceil(batch*samples/32)); tile 32 rows x 64 columns, K = latent (D);
// wave w: rows 16*(w&1).., columns 32*(w>>1)..
template <int D>
__global__ void __launch_bounds__(256) latent_dec_fwd_kernel(const vae_latent_args a) {
  kernarg_prefetch<(sizeof(vae_latent_args) < 1024 ? sizeof(vae_latent_args) : 1024)>();
  constexpr int LD = D + 8, KC = D / 8;                       // 16-byte chunks per row
  constexpr int NA = 32 * KC / 256, NB = 64 * KC / 256;       // chunks per thread: z rows, W2 rows
  __shared__ __attribute__((aligned(16))) __bf16 As[32 * LD];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[64 * LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int D2 = 2 * D, S = a.samples, BS = a.batch * a.samples, N2 = a.out_features;
  const int n0 = blockIdx.x * 64, r0 = blockIdx.y * 32;
  const __bf16* w2 = static_cast<const __bf16*>(a.w2);
  __bf16* z = static_cast<__bf16*>(a.z);
  uint4 bv[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int ch = tid + 256 * i, r = ch / KC, kc = ch % KC;
    bv[i] = ld16(w2 + (long)(n0 + r) * D + 8 * kc);
  }
  const bool rep = a.eps != nullptr;
  const bool gen = a.eps_gen != 0;                 // draw eps here (host-checked: eps, eps_step set)
  const uint32_t step = gen ? (uint32_t)*a.eps_step : 0u;
  f32x4 mu[NA][2], lv[NA][2], ep[NA][2];
  uint4 zv[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int ch = tid + 256 * i, r = ch / KC, d0 = 8 * (ch % KC), row = r0 + r;
    const bool ok = row < BS;
    const long mb = (long)(ok ? row / S : 0) * D2;
    const long eb = (long)(ok ? row : 0) * D;
    if (rep) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        mu[i][h] = ld4f(a.mulv + mb + d0 + 4 * h);
        lv[i][h] = ld4f(a.mulv + mb + D + d0 + 4 * h);
        ep[i][h] = gen ? normal4((uint32_t)((eb + d0) / 4 + h), step, a.eps_seed) : ld4f(a.eps + eb + d0 + 4 * h);
      }
    } else {
      zv[i] = ok ? ld16(z + eb + d0) : kZero4;
    }
  }
  float bias[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) bias[j] = a.b2 ? a.b2[n0 + 32 * (wave >> 1) + 16 * j + (lane & 15)] : 0.f;
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int ch = tid + 256 * i, r = ch / KC, kc = ch % KC;
    *reinterpret_cast<uint4*>(Bs + r * LD + 8 * kc) = bv[i];
  }
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int ch = tid + 256 * i, r = ch / KC, d0 = 8 * (ch % KC), row = r0 + r;
    bf16x8 o;
    if (rep) {
      float zz[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int h = e >> 2, q = e & 3;
        zz[e] = row < BS ? fmaf(ep[i][h][q], expf(0.5f * lv[i][h][q]), mu[i][h][q]) : 0.f;   // = vae_reparam_fwd
      }
      o = to_bf16x8(zz);
      if (blockIdx.x == 0 && row < BS) {
        *reinterpret_cast<bf16x8*>(z + (long)row * D + d0) = o;
        if (gen) {                                 // the drawn noise, for the backward (dlogvar)
          float* e = const_cast<float*>(a.eps) + (long)row * D + d0;
          *reinterpret_cast<f32x4*>(e) = ep[i][0];
          *reinterpret_cast<f32x4*>(e + 4) = ep[i][1];
        }
      }
    } else {
      o = *reinterpret_cast<const bf16x8*>(&zv[i]);
    }
    *reinterpret_cast<bf16x8*>(As + r * LD + d0) = o;
  }
  __syncthreads();
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  mma_block<2>(As, LD, 16 * (wave & 1), Bs, LD, 32 * (wave >> 1), D / 32, acc, lane);
  __bf16* h = static_cast<__bf16*>(a.h);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n0 + 32 * (wave >> 1) + 16 * j + (lane & 15);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = r0 + 16 * (wave & 1) + 4 * (lane >> 4) + e;
      if (row < BS) h[(long)row * N2 + col] = (__bf16)(acc[j][e] + bias[j]);
    }
  }
}

// ------------------------------------------------------------------------------ decoder_input bwd
// 1-D grid: [0, nA) dz tiles: 64 rows x 16 latent columns x a 256-deep K slice of out_features
//           -> d[mu|logvar] (atomics);  [nA, ...) dW2 / db2 tiles: 64 outputs x 64 latent columns
constexpr int DB_BK = 256, DB_LD = DB_BK + 8;
constexpr int WR_BK = 64, WR_LD = WR_BK + 8;                  // K chunk over batch rows
template <int D>
__global__ void __launch_bounds__(256) latent_dec_bwd_kernel(const vae_latent_args a, int nA) {
  kernarg_prefetch<(sizeof(vae_latent_args) < 1024 ? sizeof(vae_latent_args) : 1024)>();
  constexpr int SMEM_A = (64 + 16) * DB_LD * 2, SMEM_B = (64 + 64) * WR_LD * 2;
  __shared__ __attribute__((aligned(16))) char smem[SMEM_A > SMEM_B ? SMEM_A : SMEM_B];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int D2 = 2 * D;
  const int S = a.samples, BS = a.batch * a.samples, N2 = a.out_features;
  const __bf16* dh = static_cast<const __bf16*>(a.dh);
  const __bf16* w2 = static_cast<const __bf16*>(a.w2);
  __bf16* As = reinterpret_cast<__bf16*>(smem);
  if ((int)blockIdx.x < nA) {
    // ---- dz[r][d] = sum_k dh[r][k] W2[k][d] over this K slice, then its reparameterization backward
    __bf16* Bs = As + 64 * DB_LD;                    // [16 d][k]
    constexpr int DT = D / 16;
    const int KS = N2 / DB_BK;
    const int dt = blockIdx.x % DT, ks = (blockIdx.x / DT) % KS, r0 = (blockIdx.x / (DT * KS)) * 64;
    const int d0 = 16 * dt, k0 = ks * DB_BK;
    uint4 av[8], bv[2];
#pragma unroll
    for (int i = 0; i < 8; ++i) {                    // dh[r0..+64][k0..+256]: 64 rows x 32 chunks
      const int ch = tid + 256 * i, r = ch >> 5, kc = ch & 31, row = r0 + r;
      av[i] = row < BS ? ld16(dh + (long)row * N2 + k0 + 8 * kc) : kZero4;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {                    // W2[k0+k][d0..d0+16]: 256 rows x 2 chunks
      const int ch = tid + 256 * i, k = ch & 255, hh = ch >> 8;
      bv[i] = ld16(w2 + (long)(k0 + k) * D + d0 + 8 * hh);
    }
    // epilogue inputs of this lane: rows 16*wave + 4*(lane>>4) + e, latent column d0 + (lane&15)
    const int d = d0 + (lane & 15);
    float lv[4], ep[4], mu[4], kc4[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = r0 + 16 * wave + 4 * (lane >> 4) + e;
      const bool ok = row < BS;
      const long mb = (long)(ok ? row / S : 0) * D2;
      lv[e] = a.mulv[mb + D + d];
      ep[e] = ok ? a.eps[(long)row * D + d] : 0.f;
      mu[e] = a.mulv[mb + d];
      kc4[e] = (ok && ks == 0 && a.kl_coef) ? a.kl_coef[row] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int ch = tid + 256 * i, r = ch >> 5, kc = ch & 31;
      *reinterpret_cast<uint4*>(As + r * DB_LD + 8 * kc) = av[i];
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {                    // transposed: lanes take consecutive k
      const int ch = tid + 256 * i, k = ch & 255, hh = ch >> 8;
      float v[8];
      unpack8(bv[i], v);
#pragma unroll
      for (int e = 0; e < 8; ++e) Bs[(8 * hh + e) * DB_LD + k] = (__bf16)v[e];
    }
    __syncthreads();
    f32x4 acc[1] = {f32x4{0.f, 0.f, 0.f, 0.f}};
    mma_block<1>(As, DB_LD, 16 * wave, Bs, DB_LD, 0, DB_BK / 32, acc, lane);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = r0 + 16 * wave + 4 * (lane >> 4) + e;
      if (row >= BS) continue;
      const long mb = (long)(row / S) * D2;
      const float v = acc[0][e];
      const float sd = expf(0.5f * lv[e]);
      // vae_linear_bwd_data E_REPARAM: dmu += dz + c*mu, dlogvar += dz*eps*std/2 + c*(exp(lv)-1)/2
      const float dmu = v + kc4[e] * mu[e];
      const float dlv = v * ep[e] * 0.5f * sd + kc4[e] * 0.5f * (expf(lv[e]) - 1.f);
      atomicAdd(a.dmulv + mb + d, dmu);
      atomicAdd(a.dmulv + mb + D + d, dlv);
    }
    return;
  }
  // ---- dW2[n][d] += sum_r dh[r][n] z[r][d];  db2[n] += sum_r dh[r][n]   (n0..+64, d0..+64)
  __bf16* Bs = As + 64 * WR_LD;                      // [64 d][r]
  constexpr int DT = D / 64;
  const int nb = blockIdx.x - nA;
  const int n0 = (nb / DT) * 64, d0 = (nb % DT) * 64;
  const __bf16* z = static_cast<const __bf16*>(a.z);
  // old gradient values of this lane's outputs (accumulate semantics), loaded up front;
  // wave w: outputs n0 + 16w.., all 64 latent columns
  float old[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      old[j][e] = a.dw2[(long)(n0 + 16 * wave + 4 * (lane >> 4) + e) * D + d0 + 16 * j + (lane & 15)];
  f32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float dbs = 0.f;
  for (int r0 = 0; r0 < BS; r0 += WR_BK) {
    uint4 av[2], zv[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {                    // dh[r0+r][n0..+64]: lanes take consecutive rows
      const int ch = tid + 256 * i, r = ch & 63, c = ch >> 6, row = r0 + r;
      av[i] = row < BS ? ld16(dh + (long)row * N2 + n0 + 8 * c) : kZero4;
      zv[i] = row < BS ? ld16(z + (long)row * D + d0 + 8 * c) : kZero4;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ch = tid + 256 * i, r = ch & 63, c = ch >> 6;
      float v[8], u[8];
      unpack8(av[i], v);
      unpack8(zv[i], u);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        As[(8 * c + e) * WR_LD + r] = (__bf16)v[e];
        Bs[(8 * c + e) * WR_LD + r] = (__bf16)u[e];
      }
    }
    __syncthreads();
    if (d0 == 0 && tid < 64) {
      float s = 0.f;
#pragma unroll 8
      for (int r = 0; r < WR_BK; ++r) s += (float)As[tid * WR_LD + r];
      dbs += s;
    }
    mma_block<4>(As, WR_LD, 16 * wave, Bs, WR_LD, 0, WR_BK / 32, acc, lane);
    __syncthreads();
  }
  if (d0 == 0 && tid < 64 && a.db2) a.db2[n0 + tid] += dbs;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      a.dw2[(long)(n0 + 16 * wave + 4 * (lane >> 4) + e) * D + d0 + 16 * j + (lane & 15)] = old[j][e] + acc[j][e];
}

// ------------------------------------------------------------------------------ fc backward
// 1-D grid: [0, nA) dx tiles: 32 rows x 64 in_features, K = 2*latent (BatchNorm+LeakyReLU backward
//           epilogue with its sums; wave w: rows 16*(w&1).., columns 32*(w>>1)..);
//           [nA, ...) dW1 / db1 tiles: 64 fc outputs x 128 in_features, K = batch rows
template <int D>
__global__ void __launch_bounds__(256) latent_fc_bwd_kernel(const vae_latent_args a, int nA) {
  kernarg_prefetch<(sizeof(vae_latent_args) < 1024 ? sizeof(vae_latent_args) : 1024)>();
  constexpr int D2 = 2 * D, LDA = D2 + 8;
  constexpr int SMEM_A = (32 + 64) * LDA * 2, SMEM_B = (64 + 128) * WR_LD * 2;
  __shared__ __attribute__((aligned(16))) char smem[SMEM_A > SMEM_B ? SMEM_A : SMEM_B];
  __shared__ float ta[128], tb[128], tp[64], tq[64];
  __shared__ float red[2][2][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int K1 = a.in_features, B = a.batch, C = a.x_xf.channels;
  const __bf16* x = static_cast<const __bf16*>(a.x);
  const __bf16* w1 = static_cast<const __bf16*>(a.w1);
  __bf16* As = reinterpret_cast<__bf16*>(smem);
  const float sl = a.x_xf.slope;
  if ((int)blockIdx.x < nA) {
    // ---- dH[r][k] = sum_j dmulv[r][j] W1[j][k]; g = dH * lrelu'(BN(x)); Sg, Sg*xhat per channel
    __bf16* Bs = As + 32 * LDA;                      // [64 k][j]
    constexpr int AC = 32 * D2 / 8 / 256;            // dmulv chunks of 8 per thread (32 rows)
    constexpr int BC = D2 * 8 / 256;                 // W1 chunks per thread (D2 rows x 8 chunks)
    const int KT = K1 / 64;
    const int n0 = (blockIdx.x % KT) * 64, r0 = (blockIdx.x / KT) * 32;
    const int c0 = n0 % C;
    f32x4 av[AC][2];
#pragma unroll
    for (int i = 0; i < AC; ++i) {
      const int ch = tid + 256 * i, r = ch / (D2 / 8), jc = ch % (D2 / 8), row = r0 + r;
#pragma unroll
      for (int h = 0; h < 2; ++h)
        av[i][h] = row < B ? ld4f(a.dmulv + (long)row * D2 + 8 * jc + 4 * h) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    uint4 bv[BC];
#pragma unroll
    for (int i = 0; i < BC; ++i) {                   // lanes take consecutive rows j
      const int ch = tid + 256 * i, j = ch % D2, c = ch / D2;
      bv[i] = ld16(w1 + (long)j * K1 + n0 + 8 * c);
    }
    // epilogue inputs: rows 16*(wave&1) + 4*(lane>>4) + e, columns 32*(wave>>1) + 16*jj + (lane&15)
    const __bf16* aux = static_cast<const __bf16*>(a.dx_epi.aux);
    float yv[2][4];
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = r0 + 16 * (wave & 1) + 4 * (lane >> 4) + e;
        const int col = n0 + 32 * (wave >> 1) + 16 * jj + (lane & 15);
        yv[jj][e] = row < B ? (float)aux[(long)row * K1 + col] : 0.f;
      }
    if (tid < 64) {
      const BnCoef k = bn_coef(a.dx_epi, c0 + tid, false);
      ta[tid] = k.a; tb[tid] = k.b; tp[tid] = k.p; tq[tid] = k.q;
    }
#pragma unroll
    for (int i = 0; i < AC; ++i) {
      const int ch = tid + 256 * i, r = ch / (D2 / 8), jc = ch % (D2 / 8);
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = av[i][e >> 2][e & 3];
      *reinterpret_cast<bf16x8*>(As + r * LDA + 8 * jc) = to_bf16x8(v);
    }
#pragma unroll
    for (int i = 0; i < BC; ++i) {
      const int ch = tid + 256 * i, j = ch % D2, c = ch / D2;
      float v[8];
      unpack8(bv[i], v);
#pragma unroll
      for (int e = 0; e < 8; ++e) Bs[(8 * c + e) * LDA + j] = (__bf16)v[e];
    }
    __syncthreads();
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    mma_block<2>(As, LDA, 16 * (wave & 1), Bs, LDA, 32 * (wave >> 1), D2 / 32, acc, lane);
    __bf16* dx = static_cast<__bf16*>(a.dx);
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int cl = 32 * (wave >> 1) + 16 * jj + (lane & 15), col = n0 + cl;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = r0 + 16 * (wave & 1) + 4 * (lane >> 4) + e;
        if (row >= B) continue;
        const float y = yv[jj][e], v = acc[jj][e];
        const float g = fmaf(y, ta[cl], tb[cl]) > 0.f ? v : v * sl;
        s1 += g;
        s2 = fmaf(g, fmaf(y, tp[cl], tq[cl]), s2);
        dx[(long)row * K1 + col] = (__bf16)g;
      }
      s1 += __shfl_xor(s1, 16); s2 += __shfl_xor(s2, 16);
      s1 += __shfl_xor(s1, 32); s2 += __shfl_xor(s2, 32);
      if (lane < 16) { red[0][wave & 1][cl] = s1; red[1][wave & 1][cl] = s2; }
    }
    __syncthreads();
    if (tid < 64) {
      const float t1 = red[0][0][tid] + red[0][1][tid];
      const float t2 = red[1][0][tid] + red[1][1][tid];
      const long roff = a.sum_reps > 1 ? (long)(blockIdx.x % a.sum_reps) * a.sum_rstride : 0;
      atomicAdd(a.dx_dbeta + roff + c0 + tid, t1);
      atomicAdd(a.dx_dgamma + roff + c0 + tid, t2);
    }
    return;
  }
  // ---- dW1[j][k] += sum_r dmulv[r][j] act(x)[r][k];  db1[j] += sum_r dmulv[r][j]
  __bf16* Bs = As + 64 * WR_LD;                      // [128 k][r]
  constexpr int JT = D2 / 64;
  const int nb = blockIdx.x - nA;
  const int j0 = (nb % JT) * 64, n0 = (nb / JT) * 128;
  const int c0 = n0 % C;
  float old[8][4];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      old[j][e] = a.dw1[(long)(j0 + 16 * wave + 4 * (lane >> 4) + e) * K1 + n0 + 16 * j + (lane & 15)];
  float bsum = 0.f;
  if (n0 == 0 && tid < 64 && a.db1) bsum = a.db1[j0 + tid];
  if (tid < 128) {
    const BnCoef k = bn_coef(a.x_xf, c0 + tid, false);
    ta[tid] = k.a; tb[tid] = k.b;
  }
  f32x4 acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int r0 = 0; r0 < B; r0 += WR_BK) {
    f32x4 av[2][2];
    uint4 bv[4];
#pragma unroll
    for (int i = 0; i < 2; ++i) {                    // dmulv[r0+r][j0..+64]: lanes take consecutive rows
      const int ch = tid + 256 * i, r = ch & 63, c = ch >> 6, row = r0 + r;
#pragma unroll
      for (int h = 0; h < 2; ++h)
        av[i][h] = row < B ? ld4f(a.dmulv + (long)row * D2 + j0 + 8 * c + 4 * h) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {                    // x[r0+r][n0..+128]
      const int ch = tid + 256 * i, r = ch & 63, c = ch >> 6, row = r0 + r;
      bv[i] = row < B ? ld16(x + (long)row * K1 + n0 + 8 * c) : kZero4;
    }
    __syncthreads();                                 // tables (first pass) / previous chunk's MFMAs
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ch = tid + 256 * i, r = ch & 63, c = ch >> 6;
#pragma unroll
      for (int e = 0; e < 8; ++e) As[(8 * c + e) * WR_LD + r] = (__bf16)av[i][e >> 2][e & 3];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ch = tid + 256 * i, r = ch & 63, c = ch >> 6, row = r0 + r;
      float v[8];
      unpack8(bv[i], v);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float h = lrelu(fmaf(v[e], ta[8 * c + e], tb[8 * c + e]), sl);
        Bs[(8 * c + e) * WR_LD + r] = (__bf16)(row < B ? h : 0.f);
      }
    }
    __syncthreads();
    if (n0 == 0 && tid < 64) {                       // 16 loads in flight per round
      for (int rr = 0; rr < WR_BK; rr += 16) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int row = min(r0 + rr + u, B - 1);
          v[u] = a.dmulv[(long)row * D2 + j0 + tid];
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) bsum += r0 + rr + u < B ? v[u] : 0.f;
      }
    }
    mma_block<8>(As, WR_LD, 16 * wave, Bs, WR_LD, 0, WR_BK / 32, acc, lane);
  }
  if (n0 == 0 && tid < 64 && a.db1) a.db1[j0 + tid] = bsum;
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      a.dw1[(long)(j0 + 16 * wave + 4 * (lane >> 4) + e) * K1 + n0 + 16 * j + (lane & 15)] = old[j][e] + acc[j][e];
}

bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

int latent_check(const vae_latent_args* a, const char* what) {
  if (!a) return fail(VAE_E_BADARG, "%s: null args", what);
  if (a->dtype != VAE_BF16) return fail(VAE_E_BADDTYPE, "%s: bf16 only", what);
  if (a->batch <= 0 || a->samples <= 0 || a->latent <= 0 || a->in_features <= 0 || a->out_features <= 0)
    return fail(VAE_E_BADSHAPE, "%s: sizes", what);
  if (!(a->latent == 64 || a->latent == 128))
    return fail(VAE_E_UNSUPPORTED, "%s: latent %d (64 or 128)", what, a->latent);
  if (a->out_features % 256) return fail(VAE_E_UNSUPPORTED, "%s: out_features %d %% 256", what, a->out_features);
  return VAE_OK;
}

int latent_check_x(const vae_latent_args* a, const vae_xform& xf, const char* what) {
  const int C = xf.channels;
  if (xf.kind != VAE_X_BN_ACT) return fail(VAE_E_UNSUPPORTED, "%s: x transform must be BN_ACT", what);
  if (C <= 0 || C % 128 || a->in_features % C) return fail(VAE_E_UNSUPPORTED, "%s: channels %d / in_features %d", what, C, a->in_features);
  if (!xf.table && (!xf.sum || !xf.sumsq || !xf.gamma || !xf.beta || !(xf.count > 0.f)))
    return fail(VAE_E_BADARG, "%s: BatchNorm statistics", what);
  if (!a->x || !al16(a->x) || !a->w1 || !al16(a->w1)) return fail(VAE_E_BADARG, "%s: x / w1", what);
  return VAE_OK;
}

}  // namespace
}  // namespace vae

using namespace vae;

extern "C" int vae_latent_fc_fwd(const vae_latent_args* a, void* stream) {
  if (int rc = latent_check(a, "latent_fc_fwd")) return rc;
  if (int rc = latent_check_x(a, a->x_xf, "latent_fc_fwd")) return rc;
  if (!a->mulv) return fail(VAE_E_BADARG, "latent_fc_fwd: mulv");
  const dim3 grid((unsigned)(2 * a->latent / 32), (unsigned)(a->in_features / FC_BK), (unsigned)((a->batch + 63) / 64));
  VAE_LAUNCH(latent_fc_fwd_kernel, grid, dim3(256), 0, (hipStream_t)stream, *a);
  return check_launch("latent_fc_fwd");
}

extern "C" int vae_latent_dec_fwd(const vae_latent_args* a, void* stream) {
  if (int rc = latent_check(a, "latent_dec_fwd")) return rc;
  if (!a->w2 || !al16(a->w2) || !a->h || !a->z || !al16(a->z)) return fail(VAE_E_BADARG, "latent_dec_fwd: w2 / h / z");
  if (a->eps && (!a->mulv || !al16(a->mulv) || !al16(a->eps))) return fail(VAE_E_BADARG, "latent_dec_fwd: mulv / eps");
  if (a->eps_gen && (!a->eps || !a->eps_step)) return fail(VAE_E_BADARG, "latent_dec_fwd: eps_gen needs eps and eps_step");
  const int BS = a->batch * a->samples;
  const dim3 grid((unsigned)(a->out_features / 64), (unsigned)((BS + 31) / 32));
  if (a->latent == 128) VAE_LAUNCH(latent_dec_fwd_kernel<128>, grid, dim3(256), 0, (hipStream_t)stream, *a);
  else VAE_LAUNCH(latent_dec_fwd_kernel<64>, grid, dim3(256), 0, (hipStream_t)stream, *a);
  return check_launch("latent_dec_fwd");
}

extern "C" int vae_latent_dec_bwd(const vae_latent_args* a, void* stream) {
  if (int rc = latent_check(a, "latent_dec_bwd")) return rc;
  if (!a->dh || !al16(a->dh) || !a->w2 || !al16(a->w2) || !a->z || !al16(a->z) || !a->mulv || !a->eps || !a->dmulv ||
      !a->dw2)
    return fail(VAE_E_BADARG, "latent_dec_bwd: dh / w2 / z / mulv / eps / dmulv / dw2");
  const int BS = a->batch * a->samples;
  const int nA = (a->latent / 16) * (a->out_features / DB_BK) * ((BS + 63) / 64);
  const int nB = (a->out_features / 64) * (a->latent / 64);
  if (a->latent == 128) VAE_LAUNCH(latent_dec_bwd_kernel<128>, dim3((unsigned)(nA + nB)), dim3(256), 0, (hipStream_t)stream, *a, nA);
  else VAE_LAUNCH(latent_dec_bwd_kernel<64>, dim3((unsigned)(nA + nB)), dim3(256), 0, (hipStream_t)stream, *a, nA);
  return check_launch("latent_dec_bwd");
}

extern "C" int vae_latent_fc_bwd(const vae_latent_args* a, void* stream) {
  if (int rc = latent_check(a, "latent_fc_bwd")) return rc;
  if (int rc = latent_check_x(a, a->x_xf, "latent_fc_bwd")) return rc;
  if (a->dx_epi.kind != VAE_X_BN_ACT || a->dx_epi.channels != a->x_xf.channels || !a->dx_epi.aux)
    return fail(VAE_E_BADARG, "latent_fc_bwd: dx_epi must be x's BN_ACT with aux = x");
  if (!a->dx || !a->dmulv || !al16(a->dmulv) || !a->dw1 || !a->dx_dgamma || !a->dx_dbeta)
    return fail(VAE_E_BADARG, "latent_fc_bwd: dx / dmulv / dw1 / dx sums");
  if (a->sum_reps > 1 && a->sum_rstride < a->x_xf.channels) return fail(VAE_E_BADARG, "latent_fc_bwd: replica stride");
  const int nA = (a->in_features / 64) * ((a->batch + 31) / 32);
  const int nB = (2 * a->latent / 64) * (a->in_features / 128);
  if (a->latent == 128) VAE_LAUNCH(latent_fc_bwd_kernel<128>, dim3((unsigned)(nA + nB)), dim3(256), 0, (hipStream_t)stream, *a, nA);
  else VAE_LAUNCH(latent_fc_bwd_kernel<64>, dim3((unsigned)(nA + nB)), dim3(256), 0, (hipStream_t)stream, *a, nA);
  return check_launch("latent_fc_bwd");
}
