// Pointwise (1x1, stride 1) convolution forward and data gradient as a pixel-tile GEMM: the
// VQ-VAE ResidualLayer's Conv1x1 (models/vq_vae.py:64-68; its skip add and the ReLU backward in
// the epilogue).
//
//   out[pix][n] = epi( Σ_c A'[pix][c] · B[n][c] )
//     forward:        A = x (LeakyReLU / ReLU on load), B = W[k][c];   epi: + bias, + xf(residual)
//     data gradient:  A = dy,                          B = WT[c][k];  epi: (+ residual) * act'(aux)
//
// Why not the conv-GEMM: at K = 256 its 128 x 128 tile runs 4 K-steps of 64 behind a 2-stage
// register ring with the per-element phase/tap addressing of a general conv (19.5 us forward,
// 30.2 us data gradient at B=128, profiles/r3_v5_vq_bench_kernel_stats.csv) for 50 MB of traffic.
// Here one workgroup (4 waves of 64 x 64) owns 128 pixels x 128 channels and stages K in 64-channel
// chunks (A + B 32 KB), the next chunk's loads issued before the current chunk's MFMAs; 66 KB of
// LDS, two workgroups per CU.  (A 256-pixel tile with 128-channel chunks, one workgroup per CU,
// measured the same: 15.7 us forward / 14.9 us data gradient per call at B=128 — the kernel moves
// ~50 MB, so it runs at ~3.3 TB/s either way.)
//
// LDS rows are 128 B (64 channels) with 16-byte chunk c of row P at slot c ^ ((P >> 1) & 7): the
// lane groups of ds_read_b128 ({0-3,12-15,20-27}, ... — MI355X_MICROARCH.md LDS table) read rows
// P0..P0+15 (P0 % 16 == 0) at chunks c0 / c0+1 and land on 16 distinct 4-bank groups, and 8
// consecutive lanes of ds_write_b128 store the 8 slots of one row.
#include "vae_c3.hpp"
#include "vae_igemm.hpp"
#include <stdlib.h>

namespace vae {
namespace {

constexpr int P1_NT = 256;
constexpr int P1_BM = 128, P1_BN = 128, P1_KC = 64;       // pixels, channels, K chunk
constexpr int P1_ROW = P1_KC * 2;                          // LDS row bytes
constexpr int P1_AI = P1_BM * (P1_KC / 8) / P1_NT;         // 16-B A loads per thread per chunk (4)
constexpr int P1_BI = P1_BN * (P1_KC / 8) / P1_NT;         // B (4)
constexpr int P1_CPR = P1_KC / 8;                          // 16-B chunks per LDS row (8)
constexpr int P1_LDC = P1_BN + 4;
constexpr int P1_OPER = (P1_BM + P1_BN) * P1_ROW;          // 32768
constexpr int P1_EPI = P1_BM * P1_LDC * 4;                 // 67584
constexpr int P1_LDS = P1_OPER > P1_EPI ? P1_OPER : P1_EPI;

struct P1Params {
  const void* a;
  const void* b;
  void* out;
  const float* bias;
  const void* residual;
  const void* aux;
  uint32_t a_bytes, b_bytes, o_bytes;
  float a_slope, res_slope, aux_slope;
  int a_act, res_act, M, C, N;
};

__device__ __forceinline__ int p1_sw(int P, int c) { return P * P1_ROW + ((c ^ ((P >> 1) & 7)) << 4); }

__device__ __forceinline__ uint32_t p1_lrelu(uint32_t w, float slope) {
  f32x2 v = f32x2{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)};
  v = __builtin_elementwise_max(v, v * f32x2{slope, slope});
  bf16x2 pk;
  pk[0] = (__bf16)v[0];
  pk[1] = (__bf16)v[1];
  return *reinterpret_cast<uint32_t*>(&pk);
}

// out[m0 + row][n0 + cg..+7] = epi(Cs[row][cg..+7]): + bias, + xf(residual), * act'(aux); bf16
__device__ __forceinline__ void p1_epilogue(const P1Params& p, const float* Cs, int m0, int n0, int tid) {
  const rsrc_t rres = make_rsrc(p.residual ? p.residual : p.out, p.residual ? p.o_bytes : 0u);
  const rsrc_t raux = make_rsrc(p.aux ? p.aux : p.out, p.aux ? p.o_bytes : 0u);
  __bf16* out = static_cast<__bf16*>(p.out);
#pragma unroll 2
  for (int k = 0; k < P1_BM * (P1_BN / 8) / P1_NT; ++k) {
    const int it = tid + P1_NT * k;
    const int row = it >> 4, cg = (it & 15) * 8;
    const uint32_t o = (uint32_t)((m0 + row) * p.N + n0 + cg);
    uint32_t rs[4], ax[4];
    bload<16>(rres, p.residual ? o * 2u : kOOB, rs);
    bload<16>(raux, p.aux ? o * 2u : kOOB, ax);
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(Cs + row * P1_LDC + cg);
    const f32x4 v1 = *reinterpret_cast<const f32x4*>(Cs + row * P1_LDC + cg + 4);
    const float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    uint32_t pk[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float r0 = __uint_as_float(rs[e] << 16), r1 = __uint_as_float(rs[e] & 0xffff0000u);
      if (p.res_act) { r0 = fmaxf(r0, r0 * p.res_slope); r1 = fmaxf(r1, r1 * p.res_slope); }
      float g0 = v[2 * e] + r0, g1 = v[2 * e + 1] + r1;
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

__global__ void __launch_bounds__(P1_NT) p1_kernel(const P1Params p) {
  __shared__ __attribute__((aligned(16))) char smem[P1_LDS];
  char* const As = smem;
  char* const Bs = smem + P1_BM * P1_ROW;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;                  // 64 pixels x 64 channels per wave
  const int nt = p.N / P1_BN;
  int tile;
  {
    // XCD-aware order (workgroup b on XCD b % 8): both channel tiles of a pixel tile on one XCD
    const int nb = (int)gridDim.x, b = (int)blockIdx.x;
    const int q = nb >> 3, r = nb & 7, x = b & 7, loc = b >> 3;
    tile = x * q + min(x, r) + loc;
  }
  const int mt = tile / nt, n0 = (tile - mt * nt) * P1_BN, m0 = mt * P1_BM;
  const rsrc_t ra = make_rsrc(p.a, p.a_bytes);
  const rsrc_t rb = make_rsrc(p.b, p.b_bytes);
  uint32_t ar[P1_AI][4], br[P1_BI][4];
  auto load = [&](int c0) {
#pragma unroll
    for (int k = 0; k < P1_AI; ++k) {
      const int it = tid + P1_NT * k;
      bload<16>(ra, (uint32_t)(((m0 + it / P1_CPR) * p.C + c0 + (it % P1_CPR) * 8) * 2), ar[k]);
    }
#pragma unroll
    for (int k = 0; k < P1_BI; ++k) {
      const int it = tid + P1_NT * k;
      bload<16>(rb, (uint32_t)(((n0 + it / P1_CPR) * p.C + c0 + (it % P1_CPR) * 8) * 2), br[k]);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int k = 0; k < P1_AI; ++k) {
      const int it = tid + P1_NT * k;
      uint4 v = uint4{ar[k][0], ar[k][1], ar[k][2], ar[k][3]};
      if (p.a_act) {
        v.x = p1_lrelu(v.x, p.a_slope); v.y = p1_lrelu(v.y, p.a_slope);
        v.z = p1_lrelu(v.z, p.a_slope); v.w = p1_lrelu(v.w, p.a_slope);
      }
      *reinterpret_cast<uint4*>(As + p1_sw(it / P1_CPR, it % P1_CPR)) = v;
    }
#pragma unroll
    for (int k = 0; k < P1_BI; ++k) {
      const int it = tid + P1_NT * k;
      *reinterpret_cast<uint4*>(Bs + p1_sw(it / P1_CPR, it % P1_CPR)) = uint4{br[k][0], br[k][1], br[k][2], br[k][3]};
    }
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int kq = lane >> 4, lr = lane & 15;
  auto compute = [&]() {
#pragma unroll
    for (int kk = 0; kk < P1_KC / 32; ++kk) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const bf16x8*>(As + p1_sw(wm * 64 + i * 16 + lr, kk * 4 + kq));
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + p1_sw(wn * 64 + j * 16 + lr, kk * 4 + kq));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  const int nchunks = p.C / P1_KC;
  load(0);
  store();
  __syncthreads();
  for (int kc = 0; kc < nchunks; ++kc) {
    const bool more = kc + 1 < nchunks;
    load((more ? kc + 1 : kc) * P1_KC);        // (unconditional: see vae_c3.hip c3_kernel)
    __builtin_amdgcn_sched_barrier(0);
    compute();
    __syncthreads();
    if (more) {
      store();
      __syncthreads();
    }
  }
  // epilogue through LDS (fp32 [128][128 + 4]), then 16-byte rows of 8 channels
  float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) Cs[(wm * 64 + i * 16 + 4 * kq + e) * P1_LDC + wn * 64 + j * 16 + lr] = acc[i][j][e];
  __syncthreads();
  p1_epilogue(p, Cs, m0, n0, tid);
}

// LDS-DMA form (p1d_kernel): the operands go global -> LDS by buffer_load ... lds (lane l of a
// wave-instruction writes base + 16 l; row P holds chunk c at slot c ^ ((P >> 1) & 7), set through
// the source address), two 32 KB stages with one K-step in flight behind the MFMAs (counted vmcnt +
// raw barriers, vae_bgemm.hip), the ReLU / LeakyReLU of an activated A applied to the fragments.
// Same tile, epilogue and XCD order as p1_kernel; 67.6 KB of LDS, two workgroups per CU.
typedef __attribute__((address_space(3))) void p1_lds_void;
__device__ __forceinline__ void p1_glds16(rsrc_t r, const char* lds_wave_base, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (p1_lds_void*)(uintptr_t)(uint32_t)(uintptr_t)lds_wave_base, 16, voff, 0, 0, 0);
}

constexpr int P1D_STAGE = (P1_BM + P1_BN) * P1_ROW;       // 32768
constexpr int P1D_LDS = 2 * P1D_STAGE > P1_EPI ? 2 * P1D_STAGE : P1_EPI;

template <int ACT>
__global__ void __launch_bounds__(P1_NT, 2) p1d_kernel(const P1Params p) {
  kernarg_prefetch<(sizeof(P1Params) < 1024 ? sizeof(P1Params) : 1024)>();
  __shared__ __attribute__((aligned(16))) char smem[P1D_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nt = p.N / P1_BN;
  int tile;
  {
    const int nb = (int)gridDim.x, b = (int)blockIdx.x;
    const int q = nb >> 3, r = nb & 7, x = b & 7, loc = b >> 3;
    tile = x * q + min(x, r) + loc;
  }
  const int mt = tile / nt, n0 = (tile - mt * nt) * P1_BN, m0 = mt * P1_BM;
  const rsrc_t ra = make_rsrc(p.a, p.a_bytes);
  const rsrc_t rb = make_rsrc(p.b, p.b_bytes);
  // wave-instruction j (0..3) of this wave: tile rows 8 (4 wave + j) .. + 7, lane -> row + (lane >> 3)
  uint32_t aoffg[4], boffg[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = 8 * (4 * wave + j) + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    aoffg[j] = (uint32_t)(((m0 + row) * p.C + c * 8) * 2);
    boffg[j] = (uint32_t)(((n0 + row) * p.C + c * 8) * 2);
  }
  auto issue = [&](int kc, int buf) {
    char* la = smem + buf * P1D_STAGE + wave * 4096;
    char* lb = la + P1_BM * P1_ROW;
    const uint32_t cb = (uint32_t)kc * (P1_KC * 2);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      p1_glds16(ra, la + j * 1024, aoffg[j] + cb);
      p1_glds16(rb, lb + j * 1024, boffg[j] + cb);
    }
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int kq = lane >> 4, lr = lane & 15;
  const int nchunks = p.C / P1_KC;
  issue(0, 0);
  for (int kc = 0; kc < nchunks; ++kc) {
    const int buf = kc & 1;
    if (kc + 1 < nchunks) {
      issue(kc + 1, buf ^ 1);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    const char* As = smem + buf * P1D_STAGE;
    const char* Bs = As + P1_BM * P1_ROW;
#pragma unroll
    for (int kk = 0; kk < P1_KC / 32; ++kk) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const bf16x8*>(As + p1_sw(wm * 64 + i * 16 + lr, kk * 4 + kq));
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + p1_sw(wn * 64 + j * 16 + lr, kk * 4 + kq));
      if constexpr (ACT) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          uint32_t* w = reinterpret_cast<uint32_t*>(&af[i]);
#pragma unroll
          for (int e = 0; e < 4; ++e) w[e] = p1_lrelu(w[e], p.a_slope);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) Cs[(wm * 64 + i * 16 + 4 * kq + e) * P1_LDC + wn * 64 + j * 16 + lr] = acc[i][j][e];
  __syncthreads();
  p1_epilogue(p, Cs, m0, n0, tid);
}

inline bool p1_al16(const void* ptr) { return ((uintptr_t)ptr & 15u) == 0; }

}  // namespace

bool p1_shape_ok(long M, int C, int N) {
  return M > 0 && M % P1_BM == 0 && C % P1_KC == 0 && C > 0 && N % P1_BN == 0 && N > 0 &&
         M * (C > N ? C : N) * 2 < (1l << 31);
}

int p1_launch(const P1Args& a, hipStream_t st) {
  if (!p1_shape_ok(a.M, a.C, a.N)) return fail(VAE_E_BADSHAPE, "p1: shape");
  if (!p1_al16(a.a) || !p1_al16(a.b) || !p1_al16(a.out) || (a.residual && !p1_al16(a.residual)) ||
      (a.aux && !p1_al16(a.aux)))
    return fail(VAE_E_BADARG, "p1: tensors must be 16-byte aligned");
  P1Params p;
  p.a = a.a; p.b = a.b; p.out = a.out; p.bias = a.bias; p.residual = a.residual; p.aux = a.aux;
  p.a_bytes = (uint32_t)(a.M * a.C * 2);
  p.b_bytes = (uint32_t)((long)a.N * a.C * 2);
  p.o_bytes = (uint32_t)(a.M * a.N * 2);
  p.a_slope = a.a_slope; p.res_slope = a.res_slope; p.aux_slope = a.aux_slope;
  p.a_act = a.a_act; p.res_act = a.res_act; p.M = (int)a.M; p.C = a.C; p.N = a.N;
  const unsigned grid = (unsigned)((a.M / P1_BM) * (a.N / P1_BN));
  if (a.a_act) VAE_LAUNCH(p1d_kernel<1>, dim3(grid), dim3(P1_NT), 0, st, p);
  else VAE_LAUNCH(p1d_kernel<0>, dim3(grid), dim3(P1_NT), 0, st, p);
  return check_launch("p1");
}

}  // namespace vae
