// The large bf16 implicit-GEMM convolutions (Conv2d / ConvTranspose2d forward and data gradient)
// on an LDS-DMA pipeline: the Autoencoder's wide layers (configs/big_ae.yaml ..
// patient_vvbig_ae.yaml: 9.7 GFLOP per layer and pass at B = 64, models/autoencoder.py:16-86) and
// the VQ-VAE's strided 4x4 layers (models/vq_vae.py:98-105, :140-154), whose arithmetic intensity
// is above the MFMA ridge.
//
// Why a fourth GEMM kernel: the conv-GEMM (vae_cgemm.hpp) stages operands through registers so it
// can apply the BatchNorm / LeakyReLU transform on the way into LDS; at 128 x 128 tiles its
// register budget leaves two K-steps in flight, against a ~1-2 us load latency and ~0.2 us of MFMA
// work per K-step — it ran these layers at 3-10 % of the bf16 peak (profiles/r3_v4_*).  Here the
// operands come transform-free (the caller materialises lrelu(BN(y)) / the BatchNorm-backward
// gradient once per layer, vae_bn_apply) and go global -> LDS by buffer_load ... lds (no VGPR
// staging, no VALU work between load and MFMA):
//   * 128 x 128 x 64 tiles, 4 waves (2 x 2, 64 x 64 each: 4 x 4 v_mfma_f32_16x16x32_bf16 frags),
//     two LDS buffers of 32 KB: K-step k+1 is in flight while k computes (counted vmcnt + raw
//     s_barrier: an LDS-DMA counts on vmcnt, and __syncthreads' fence would drain it);
//   * the LDS image is lane-linear (LDS-DMA writes base + lane * 16): row r of a tile holds its
//     eight 16-byte k-chunks at slot c ^ ((r >> 1) & 7), set through the per-lane SOURCE address,
//     which makes the ds_read_b128 fragment reads of 16 rows x one chunk conflict-free;
//   * one K-step = 64 channels of one tap (host: C % 64 == 0), so a lane's gather address is its
//     row base + one per-step tap offset (out-of-image taps read zeros through the buffer
//     resource's range check);
//   * XCD-aware tile order (n fastest within an XCD's contiguous tile range), split-K through fp32
//     slabs + the shared finalize (vae_launch.hpp launch_finalize) when the tiles do not cover the
//     CUs; the epilogue stages the fp32 tile through LDS in two 64-row halves and applies the bias
//     + BatchNorm statistics (E_STORE) or the activation backward + BatchNorm-backward sums
//     (E_BNBWD) of the cgemm contract, 16-byte stores.
#include "vae_launch.hpp"
#include "vae_bgemm.hpp"
#include "vae_wgemm.hpp"

namespace vae {
namespace {

constexpr int BG_M = 128, BG_N = 128, BG_K = 64, BG_T = 256;
// work (FLOP) from which a transform-free layer takes the LDS-DMA GEMMs instead of the conv GEMM
constexpr double kBgMinFlops = 4e9;
constexpr int BG_TILE = BG_M * BG_K * 2;              // bytes of one operand tile (16 KB)
constexpr int BG_STAGE = 2 * BG_TILE;                 // A + B
// A ring of NSTG stages with NSTG - 1 K-steps in flight: NSTG = 2 at two workgroups per CU (64 KB
// each) when the tiles fill two rounds of CUs, NSTG = 4 at one per CU (128 KB) when they do not —
// there one workgroup with three steps in flight replaces a split-K pair and its slab + finalize
// (big_ae encoder.1: 49.6 -> 23.3 us), while grids of thousands of tiles keep the two-workgroup
// form (its final ConvT: 59 vs 84 us at NSTG = 4; profiles/r4_v4_notes.txt).
template <int NSTG> constexpr int bg_ops() { return NSTG * BG_STAGE; }
constexpr int BG_LDC = BG_N + 4;                      // fp32 epilogue rows (one 64-row half at a time)
constexpr int BG_EPI = (64 * BG_LDC * 4 + 255) / 256 * 256;   // the epilogue's half-tile; its tables follow
static_assert(BG_EPI <= bg_ops<2>(), "epilogue half-tile fits the operand buffers");

// this wave's loads of the current step landed, `newer` later steps (8 LDS-DMA each) left in flight
__device__ __forceinline__ void bg_wait_newer(int newer) {
  if (newer >= 3) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else if (newer == 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if (newer == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// One 16-byte-per-lane LDS-DMA (buffer_load_dwordx4 ... lds: lane l's 16 bytes land at M0 + 16 l).
// (The compiler's wait-count pass leaves the K-step in flight across the loop's ds_reads here —
// one LDS array, explicit vmcnt(N) waits; checked in the ISA.)
typedef __attribute__((address_space(3))) void lds_void;
__device__ __forceinline__ void glds16(rsrc_t r, const char* lds_wave_base, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)(uintptr_t)(uint32_t)(uintptr_t)lds_wave_base, 16, voff, 0, 0, 0);
}

__device__ __forceinline__ int bg_slot(int row, int c) { return c ^ ((row >> 1) & 7); }

template <int AM, int EM, int NSTG>
__global__ void __launch_bounds__(BG_T, NSTG >= 4 ? 1 : 2) bgemm_kernel(const GemmParams p) {
  kernarg_prefetch<(sizeof(GemmParams) < 1024 ? sizeof(GemmParams) : 1024)>();
  static_assert(NSTG >= 2 && NSTG <= 4, "bg_wait_newer counts up to three steps in flight");
  extern __shared__ __attribute__((aligned(16))) char smem[];      // the ONLY LDS object (see header)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  // ---- tile: XCD-aware order (1-D grid), as vae_cgemm.hpp
  const int gm = (p.M + BG_M - 1) / BG_M, gn = p.N / BG_N, gz = p.nphase * p.ksplit;
  int tile;
  {
    const int nb = gm * gn * gz, b = blockIdx.x;
    const int q = nb >> 3, r = nb & 7, x = b & 7, loc = b >> 3;
    tile = x * q + min(x, r) + loc;
  }
  const int tn = tile % gn, tz = (tile / gn) % gz, tmi = tile / (gn * gz);
  const int m0 = tmi * BG_M, n0 = tn * BG_N;
  const int phase = (p.nphase > 1) ? (int)(tz / p.ksplit) : 0;
  const int ks = tz - phase * p.ksplit;
  const PhaseInfo pq = make_phase(p, phase);
  const int Kp = AM == A_CONVT ? pq.nth * pq.ntw * p.gc : p.K;
  const int ktiles = Kp / BG_K;                       // host: Kp % 64 == 0
  const int kper = (ktiles + p.ksplit - 1) / p.ksplit;
  const int kt0 = ks * kper, kt1 = min(ktiles, kt0 + kper);

  // ---- this lane's 4 A rows and 4 B rows (wave-instruction j: tile rows 8 (4 wave + j) .. + 7)
  const rsrc_t ra = make_rsrc(p.a_ptr, p.a_bytes), rb = make_rsrc(p.b_ptr, p.b_bytes);
  RowOperand<__bf16, AM, true> ar[4];
  int bbase[4], slot_c[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = 8 * (4 * wave + j) + (lane >> 3);
    slot_c[j] = bg_slot(row, lane & 7);               // the logical chunk this lane's slot holds
    ar[j].init(p, m0 + row, p.M, phase, p.a_ld);
    bbase[j] = (n0 + row) * p.b_ld;
  }
  auto issue = [&](int kt, int buf) {
    const int k0 = kt * BG_K;
    const KTap t = RowOperand<__bf16, AM, true>::tap(p, pq, p.fd_ach, p.a_xf.channels, false, k0, Kp);
    int boff = k0;
    if constexpr (AM == A_CONVT) {
      const int rr = pq.t0h - p.gs * t.r, ss = pq.t0w - p.gs * t.s;
      boff = (rr * p.gr + ss) * p.gc + t.ch;
    }
    char* la = smem + buf * BG_STAGE + wave * 4 * 1024;
    char* lb = la + BG_TILE;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool ok = ar[j].valid && (uint32_t)(ar[j].hi0 + t.r) < (uint32_t)p.gh &&
                      (uint32_t)(ar[j].wi0 + t.s) < (uint32_t)p.gw;
      const uint32_t offa = ok ? (uint32_t)(ar[j].base + t.toff + 8 * slot_c[j]) * 2u : kOOB;
      glds16(ra, la + j * 1024, offa);
      glds16(rb, lb + j * 1024, (uint32_t)(bbase[j] + boff + 8 * slot_c[j]) * 2u);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets (bytes within a tile): row, chunk (ks2 * 4 + lane >> 4) at its slot
  int aoff[4][2], boffs[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      const int ra_ = wm * 64 + i * 16 + (lane & 15), rb_ = wn * 64 + i * 16 + (lane & 15);
      const int c = k2 * 4 + (lane >> 4);
      aoff[i][k2] = ra_ * 128 + bg_slot(ra_, c) * 16;
      boffs[i][k2] = rb_ * 128 + bg_slot(rb_, c) * 16;
    }

  // ring: steps kt0 .. kt0 + NSTG - 2 requested up front; step i's refill goes into the slot step
  // i - 1 used (released by that step's closing barrier); 8 LDS-DMA per wave per step
  const int nk = kt1 - kt0;
#pragma unroll
  for (int u = 0; u < NSTG - 1; ++u)
    if (u < nk) issue(kt0 + u, u);
  for (int i = 0; i < nk; ++i) {
    const int buf = i % NSTG;
    if (i + NSTG - 1 < nk) issue(kt0 + i + NSTG - 1, (i + NSTG - 1) % NSTG);
    bg_wait_newer(min(NSTG - 1, nk - 1 - i));              // this wave's loads of step i landed
    __builtin_amdgcn_s_barrier();                           // ... and every wave's
    const char* la = smem + buf * BG_STAGE;
    const char* lb = la + BG_TILE;
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const bf16x8*>(la + aoff[i][k2]);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(lb + boffs[j][k2]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                           // every wave is done reading `buf`
  }

  // ================================================================ epilogue (two 64-row halves)
  float* Cs = reinterpret_cast<float*>(smem);              // [64][BG_LDC]
  // per-channel tables of the epilogue transform (E_BNBWD with a BatchNorm+LeakyReLU), after the
  // operand area; scratch for their in-kernel build on the operand area (free by now)
  float* tq = reinterpret_cast<float*>(smem + BG_EPI);
  const int ce = tab_stride(p.epi_xf.channels);
  const Tab te{tq, tq + ce, nullptr, tq + 2 * ce, tq + 3 * ce};
  if constexpr (EM == E_BNBWD) {
    if (!p.slab && p.epi_xf.kind == VAE_X_BN_ACT) tab_fill(p.epi_xf, te, true, false, Cs);
  }
  __syncthreads();
  if (p.slab) {
    // split-K partial -> slab [phase][ks][M][N] (plain fp32, the finalize adds the slices)
    float* sl = p.slab + ((long)(phase * p.ksplit + ks) * p.M) * p.N;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = m0 + wm * 64 + i * 16 + 4 * (lane >> 4) + e, col = n0 + wn * 64 + j * 16 + (lane & 15);
          if (row < p.M) sl[(long)row * p.N + col] = acc[i][j][e];
        }
    return;
  }
  // thread -> 8 consecutive columns (ec) of rows er, er + 16, er + 32, er + 48 of a half
  const int ec = tid & 15, er = tid >> 4;
  const int col = n0 + ec * 8;
  float bias[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bias[e] = (EM == E_STORE && p.bias) ? p.bias[col + e] : 0.f;
  const rsrc_t raux = epi_aux_rsrc<EM>(p);
  int ech = 0;
  if constexpr (EM == E_BNBWD) ech = (int)(col - p.fd_ech.div(col) * p.epi_xf.channels);
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
  __bf16* out = static_cast<__bf16*>(p.out);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (wm == h) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) Cs[(i * 16 + 4 * (lane >> 4) + e) * BG_LDC + wn * 64 + j * 16 + (lane & 15)] = acc[i][j][e];
    }
    __syncthreads();
    int obase[4];
    uint32_t aux[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int row = m0 + h * 64 + er + 16 * u;
      obase[u] = out_row_base(p, phase, row < p.M ? row : 0) + col;
      const bool ld = EM == E_BNBWD && p.epi_xf.kind != VAE_X_NONE && row < p.M;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(raux, ld ? (uint32_t)obase[u] * 2u : kOOB, 0, 0);
      aux[u][0] = v[0]; aux[u][1] = v[1]; aux[u][2] = v[2]; aux[u][3] = v[3];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int rl = er + 16 * u, row = m0 + h * 64 + rl;
      if (row >= p.M) continue;
      const f32x4 v0 = *reinterpret_cast<const f32x4*>(Cs + rl * BG_LDC + ec * 8);
      const f32x4 v1 = *reinterpret_cast<const f32x4*>(Cs + rl * BG_LDC + ec * 8 + 4);
      const float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if constexpr (EM == E_STORE) {
          s1[e] += v[e];
          s2[e] = fmaf(v[e], v[e], s2[e]);
          o[e] = v[e] + bias[e];
        } else {
          const float ax = __uint_as_float((e & 1) ? (aux[u][e >> 1] & 0xffff0000u) : (aux[u][e >> 1] << 16));
          float g = v[e];
          if (p.epi_xf.kind == VAE_X_BN_ACT) {
            const float z = fmaf(ax, te.a[ech + e], te.b[ech + e]);
            g = z > 0.f ? g : g * p.epi_xf.slope;
            s1[e] += g;
            s2[e] = fmaf(g, fmaf(ax, te.p[ech + e], te.q[ech + e]), s2[e]);
          } else if (p.epi_xf.kind == VAE_X_ACT) {
            g = ax > 0.f ? g : g * p.epi_xf.slope;
          }
          o[e] = g;
        }
      }
      uint4 pk;
      uint32_t* pp = reinterpret_cast<uint32_t*>(&pk);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        bf16x2 hh;
        hh[0] = (__bf16)o[2 * e];
        hh[1] = (__bf16)o[2 * e + 1];
        pp[e] = *reinterpret_cast<uint32_t*>(&hh);
      }
      *reinterpret_cast<uint4*>(out + obase[u]) = pk;
    }
    __syncthreads();                                        // Cs is rewritten by the next half
  }
  if (!epi_wants_sums<EM>(p)) return;
  // per-column sums: lanes l and l ^ 16, l ^ 32 hold the same columns (ec = tid & 15) -> butterfly,
  // then one partial per wave and column in LDS, added in wave order
#pragma unroll
  for (int m = 16; m < 64; m <<= 1)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s1[e] += __shfl_xor(s1[e], m);
      s2[e] += __shfl_xor(s2[e], m);
    }
  float* part = Cs;                                         // [4 waves][2][BG_N]
  if (lane < 16) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      part[(wave * 2) * BG_N + lane * 8 + e] = s1[e];
      part[(wave * 2 + 1) * BG_N + lane * 8 + e] = s2[e];
    }
  }
  __syncthreads();
  if (tid < BG_N) {
    const float t1 = (part[0 * BG_N + tid] + part[2 * BG_N + tid]) + (part[4 * BG_N + tid] + part[6 * BG_N + tid]);
    const float t2 = (part[1 * BG_N + tid] + part[3 * BG_N + tid]) + (part[5 * BG_N + tid] + part[7 * BG_N + tid]);
    epi_flush_sums<EM>(p, (int)blockIdx.x, n0 + tid, t1, t2);
  }
}

// ------------------------------------------------------------------ weight gradient
//   dW[m][r][s][j] += Σ_pix U[pix][m] · V[pix -> (hu*S-P+r, wu*S-P+s)][j]     (vae_wgemm.hpp)
// on the same pipeline, for transform-free operands (the materialised activation and gradient of
// the large layers): 128 (m) x 128 (j) tiles of one tap, K-step 64 pixels.  A K-step stages the
// U rows [64 pixels][128 m] and the tap-shifted V rows [64][128 j] as 256-byte LDS rows by
// LDS-DMA, 16-byte chunk c of row P at slot c ^ (((P & 3) << 2) | ((P >> 2) & 3)) (set through
// the source address; cdna_hip_programming.md T10 image (b)), and the MFMA operands are read
// column-major with ds_read_b64_tr_b16 (K = pixels).  Out-of-image taps and pixels past the
// slice read zeros (buffer range check).  Partials: one K slice adds with plain load + store,
// several with fp32 atomics (wg_epilogue).
constexpr int BW_KP = 64;
constexpr int BW_TILE = BW_KP * 256;                  // 16 KB: 64 pixel rows x 128 channels
constexpr int BW_STAGE = 2 * BW_TILE;
template <int NSTG> constexpr int bw_ops() { return NSTG * BW_STAGE; }   // (bgemm's ring choice)

__device__ __forceinline__ int bw_sw(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

// Transposed reads as inline asm: the wait-count pass gives the ds_read_tr intrinsic no LDS address
// and makes it wait for every LDS-DMA in flight (vmcnt(0) at each K-step head, seen in the ISA);
// asm reads are invisible to it, so their results are waited for explicitly.  The wait must take
// the asm's OWN output registers ("+v"): the compiler treats an asm output as ready when the asm
// ends, so any instruction touching those registers — even the register moves that pack two
// 4-element halves into an MFMA operand (v_bfi_b32 vN, s, vN, vN) — may otherwise be scheduled
// before the wait and read or rewrite them while the LDS return is in flight.  Waiting on the packed
// operands instead (this file's first version) let the packing moves race the returns: weight
// gradients off by up to 40 % of their max (tests/test_gpu_bgemm.py test_bwg_weight_gradient).
__device__ __forceinline__ wgm_bf16x4 bw_tr(uint32_t lds_addr) {
  wgm_bf16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(lds_addr) : "memory");
  return r;
}
__device__ __forceinline__ void bw_wait(wgm_bf16x4 (&a)[4][2], wgm_bf16x4 (&b)[4][2]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(a[0][0]), "+v"(a[0][1]), "+v"(a[1][0]), "+v"(a[1][1]), "+v"(a[2][0]), "+v"(a[2][1]),
                 "+v"(a[3][0]), "+v"(a[3][1]), "+v"(b[0][0]), "+v"(b[0][1]), "+v"(b[1][0]), "+v"(b[1][1]),
                 "+v"(b[2][0]), "+v"(b[2][1]), "+v"(b[3][0]), "+v"(b[3][1])::"memory");
}
__device__ __forceinline__ bf16x8 bw_cat(wgm_bf16x4 lo, wgm_bf16x4 hi) {
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

template <int NSTG>
__global__ void __launch_bounds__(BG_T, NSTG >= 4 ? 1 : 2) bwg_kernel(const WgParams p) {
  kernarg_prefetch<(sizeof(WgParams) < 1024 ? sizeof(WgParams) : 1024)>();
  static_assert(NSTG >= 2 && NSTG <= 4, "bg_wait_newer counts up to three steps in flight");
  extern __shared__ __attribute__((aligned(16))) char smem[];      // the ONLY LDS object
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int gm = p.M / 128, gj = p.J / 128, taps = p.R * p.R;
  const int per_slice = gm * gj * taps;
  int b;
  {
    // XCD-aware order: each XCD takes a contiguous range (j fastest, then tap, m tile, slice), so
    // the workgroups re-reading one U slice sit on one L2
    const int nb = (int)gridDim.x, x = (int)blockIdx.x & 7, loc = (int)blockIdx.x >> 3;
    const int q = nb >> 3, rr = nb & 7;
    b = x * q + min(x, rr) + loc;
  }
  const int slice = b / per_slice;
  int t = b - slice * per_slice;
  const int tj = t % gj;
  t /= gj;
  const int tap = t % taps, tmi = t / taps;
  const int r = tap / p.R, s = tap - r * p.R;
  const int m0 = tmi * 128, j0 = tj * 128;
  const long npix = (long)p.n * p.hu * p.wu;
  const long k0 = (long)slice * p.kper;
  const long k1 = min(npix, k0 + p.kper);
  const int nsteps = (int)((k1 - k0 + BW_KP - 1) / BW_KP);
  const rsrc_t ru = make_rsrc(p.u, p.u_bytes), rv = make_rsrc(p.v, p.v_bytes);

  // wave-instruction j writes LDS rows 4 (4 wave + j) .. + 3: lane -> row + (lane >> 4), slot lane & 15
  int rowj[4], cj[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    rowj[j] = 4 * (4 * wave + j) + (lane >> 4);
    cj[j] = (lane & 15) ^ bw_sw(rowj[j]);                       // the logical chunk this slot holds
  }
  auto issue = [&](int step, int buf) {
    const long kb = k0 + (long)step * BW_KP;
    char* lu = smem + buf * BW_STAGE + wave * 4096;
    char* lv = lu + BW_TILE;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long pix = kb + rowj[j];
      const bool in = pix < k1;
      const uint32_t pp = in ? (uint32_t)pix : 0u;
      const uint32_t qd = p.fd_wu.div(pp);                      // n * hu + hu_i
      const int wu_i = (int)(pp - qd * (uint32_t)p.wu);
      const uint32_t nn = p.fd_hu.div(qd);
      const int hu_i = (int)(qd - nn * (uint32_t)p.hu);
      const int hv_i = hu_i * p.S - p.P + r, wv_i = wu_i * p.S - p.P + s;
      const bool vin = in && (uint32_t)hv_i < (uint32_t)p.hv && (uint32_t)wv_i < (uint32_t)p.wv;
      const uint32_t ou = in ? (uint32_t)((pp * (uint32_t)p.M + (uint32_t)(m0 + 8 * cj[j])) * 2u) : kOOB;
      const uint32_t ov = vin ? (uint32_t)(((((uint32_t)nn * p.hv + hv_i) * p.wv + wv_i) * (uint32_t)p.J +
                                            (uint32_t)(j0 + 8 * cj[j])) * 2u) : kOOB;
      glds16(ru, lu + j * 1024, ou);
      glds16(rv, lv + j * 1024, ov);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed reads: lane 4q+p of 16-lane group g reads pixel row 8g + 4h + q, channels
  // c0 + 4p .. +3 of the fragment's 16 (T10: off(row, c0 + (p >> 1)) + 8 (p & 1)); rows + 32 for
  // the second MFMA K-step keep the same swizzle
  const int g = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  int aoff[4][2], boff[4][2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = 8 * g + 4 * h + q4;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int ca = (wm * 64 + f * 16) / 8 + (p4 >> 1), cb = (wn * 64 + f * 16) / 8 + (p4 >> 1);
      aoff[f][h] = row * 256 + 16 * (ca ^ bw_sw(row)) + 8 * (p4 & 1);
      boff[f][h] = row * 256 + 16 * (cb ^ bw_sw(row)) + 8 * (p4 & 1);
    }
  }

#pragma unroll
  for (int u = 0; u < NSTG - 1; ++u)
    if (u < nsteps) issue(u, u);
  for (int st = 0; st < nsteps; ++st) {
    const int buf = st % NSTG;
    if (st + NSTG - 1 < nsteps) issue(st + NSTG - 1, (st + NSTG - 1) % NSTG);
    bg_wait_newer(min(NSTG - 1, nsteps - 1 - st));         // this wave's loads of step st landed
    __builtin_amdgcn_s_barrier();                           // ... and every wave's
    const uint32_t lu = (uint32_t)(uintptr_t)smem + buf * BW_STAGE;
    const uint32_t lv = lu + BW_TILE;
    wgm_bf16x4 ra[2][4][2], rb[2][4][2];                  // raw read results [kk][fragment][half]
    auto rd = [&](int kk) {
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        ra[kk][f][0] = bw_tr(lu + kk * 32 * 256 + aoff[f][0]);
        ra[kk][f][1] = bw_tr(lu + kk * 32 * 256 + aoff[f][1]);
        rb[kk][f][0] = bw_tr(lv + kk * 32 * 256 + boff[f][0]);
        rb[kk][f][1] = bw_tr(lv + kk * 32 * 256 + boff[f][1]);
      }
    };
    auto mma = [&](int kk) {                               // (after bw_wait(ra[kk], rb[kk]))
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) { af[f] = bw_cat(ra[kk][f][0], ra[kk][f][1]); bfr[f] = bw_cat(rb[kk][f][0], rb[kk][f][1]); }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    };
    rd(0);
    bw_wait(ra[0], rb[0]);
    rd(1);                                                  // in flight behind the first 16 MFMAs
    mma(0);
    bw_wait(ra[1], rb[1]);
    mma(1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                           // every wave is done reading `buf`
  }
  const long rowstride = (long)taps * p.J;
  wg_epilogue<4, 4>(p, nullptr, acc, m0 + wm * 64 + 4 * g, j0 + wn * 64 + li, rowstride, (long)tap * p.J);
}

template <int AM, int EM>
int bgemm_go(GemmParams p, void* ws, long ws_bytes, hipStream_t st) {
  int kmax = p.K;
  if (AM == A_CONVT) {
    kmax = 0;
    for (int ph = 0; ph < p.nphase; ++ph) {
      const int k = p.ntap_h[ph / p.gs] * p.ntap_w[ph % p.gs] * p.gc;
      kmax = k > kmax ? k : kmax;
    }
  }
  const int ktiles = kmax / BG_K;
  const long tiles = (long)((p.M + BG_M - 1) / BG_M) * (p.N / BG_N) * p.nphase;
  // ring depth (bg_ops): two stages at two workgroups per CU for grids of >= two rounds of CUs,
  // else four stages at one per CU, K split until the tiles cover the CUs (>= 4 K-steps a slice)
  const int nstg = tiles >= 2l * kCUs ? 2 : 4;
  const int wgpercu = nstg == 2 ? 2 : 1;
  int split = 1;
  if (tiles < (long)wgpercu * kCUs) {
    split = (int)(((long)wgpercu * kCUs) / tiles);
    if (split > ktiles / 4) split = ktiles / 4;
    if (split < 1) split = 1;
  }
  if (split > 1) {
    if (!ws && !querying()) split = 1;
    else if (!ws_fits((long)split * p.M * p.N * p.nphase * 4, ws_bytes, "bgemm split-K")) return VAE_E_BADARG;
  }
  p.ksplit = split;
  p.slab = split > 1 ? static_cast<float*>(ws) : nullptr;
  const size_t lt = (size_t)BG_EPI + (EM == E_BNBWD ? (size_t)tab_floats(p.epi_xf, true) * 4 : 0);
  const size_t ops = (size_t)(nstg == 2 ? bg_ops<2>() : bg_ops<4>());
  const size_t lds = lt > ops ? lt : ops;
  if (lds > (size_t)kLdsBytes) return kHeadFallback;
  const unsigned nb = (unsigned)(tiles * split);
  if (nstg == 2) VAE_LAUNCH((bgemm_kernel<AM, EM, 2>), dim3(nb), dim3(BG_T), lds, st, p);
  else VAE_LAUNCH((bgemm_kernel<AM, EM, 4>), dim3(nb), dim3(BG_T), lds, st, p);
  if (int rc = check_launch("bgemm")) return rc;
  if (p.slab) return launch_finalize<__bf16, EM>(p, st);
  return VAE_OK;
}

}  // namespace

// Eligible: transform-free bf16 operands (the caller materialised the activation), 64-channel
// K-steps that stay inside one tap, 128-column tiles, no residual, work large enough to pay for a
// 128 x 128 tile (>= 1 GFLOP), packed NHWC alignment.
bool bgemm_ok(const GemmParams& p, int am, int em) {
  if ((am != A_CONV && am != A_CONVT) || (em != E_STORE && em != E_BNBWD)) return false;
  if (p.a_xf.kind != VAE_X_NONE || p.g_nchw || p.ones_col >= 0 || p.residual || p.out_f32) return false;
  if (p.gc % BG_K || p.N % BG_N || p.out_ld % 8 || p.b_ld % 8) return false;
  if (((uintptr_t)p.a_ptr | (uintptr_t)p.b_ptr | (uintptr_t)p.out) & 15) return false;
  if (em == E_BNBWD && p.epi_xf.kind != VAE_X_NONE && (((uintptr_t)p.epi_xf.aux & 15) || p.epi_xf.channels % 8)) return false;
  int kmax = p.K;
  if (am == A_CONVT) {
    kmax = 0;
    for (int ph = 0; ph < p.nphase; ++ph) {
      const int k = p.ntap_h[ph / p.gs] * p.ntap_w[ph % p.gs] * p.gc;
      kmax = k > kmax ? k : kmax;
    }
  }
  const double flops = 2.0 * p.M * p.N * (double)kmax * p.nphase;      // (upper bound over phases)
  return flops >= kBgMinFlops;
}

int bgemm_launch(const GemmParams& p, int am, int em, void* ws, long ws_bytes, hipStream_t st) {
  if (am == A_CONV) return em == E_STORE ? bgemm_go<A_CONV, E_STORE>(p, ws, ws_bytes, st) : bgemm_go<A_CONV, E_BNBWD>(p, ws, ws_bytes, st);
  return em == E_STORE ? bgemm_go<A_CONVT, E_STORE>(p, ws, ws_bytes, st) : bgemm_go<A_CONVT, E_BNBWD>(p, ws, ws_bytes, st);
}

// Weight gradients on the LDS-DMA pipeline: transform-free operands (the materialised activation
// and BatchNorm-backward gradient), 128-multiple channel counts, work >= 4 GFLOP (kBgMinFlops).
bool bwg_ok(const WgParams& p) {
  if (p.u_xf.kind != VAE_X_NONE || p.v_xf.kind != VAE_X_NONE || p.jst || p.db) return false;
  if (p.M % 128 || p.J % 128 || p.M <= 0 || p.J <= 0) return false;
  if (((uintptr_t)p.u | (uintptr_t)p.v) & 15) return false;
  const long npix = (long)p.n * p.hu * p.wu;
  if (npix * p.M * 2 >= (1l << 31) || (long)p.n * p.hv * p.wv * p.J * 2 >= (1l << 31)) return false;
  const double flops = 2.0 * p.M * p.J * p.R * p.R * (double)npix;
  return flops >= kBgMinFlops;
}

int bwg_launch(WgParams p, hipStream_t st) {
  p.fd_wu = make_fastdiv(p.wu);
  p.fd_hu = make_fastdiv(p.hu);
  p.fd_r = make_fastdiv(p.R);
  const long npix = (long)p.n * p.hu * p.wu;
  p.u_bytes = (uint32_t)(npix * p.M * 2);
  p.v_bytes = (uint32_t)((long)p.n * p.hv * p.wv * p.J * 2);
  const long tiles = (long)(p.M / 128) * (p.J / 128) * p.R * p.R;
  const long ksteps = (npix + BW_KP - 1) / BW_KP;
  // two stages at two workgroups per CU, K slices: one round of workgroups (floor: no overflow
  // round), >= 8 K-steps each.  (Four stages at one per CU halves the slices the small-tile
  // layers split into and measured slower: VQ-VAE encoder.1 72.6 -> 88.7 us, big_ae's
  // weight-gradient batch 486 -> 512 us.)
  const int nstg = 2;
  const int wgpercu = 2;
  constexpr int mink = 8;
  const long slots = (long)wgpercu * kCUs;
  long split = slots / tiles;
  if (split > ksteps / mink) split = ksteps / mink;
  if (split < 1) split = 1;
  p.kper = (int)(((ksteps + split - 1) / split) * BW_KP);
  split = (npix + p.kper - 1) / p.kper;
  p.slab = nullptr;
  p.slab_ld = 0;
  p.own = split == 1 ? 1 : 0;
  p.jst = 0;
  if (nstg == 2) VAE_LAUNCH(bwg_kernel<2>, dim3((unsigned)(tiles * split)), dim3(BG_T), bw_ops<2>(), st, p);
  else VAE_LAUNCH(bwg_kernel<4>, dim3((unsigned)(tiles * split)), dim3(BG_T), bw_ops<4>(), st, p);
  return check_launch("bwg");
}

}  // namespace vae
