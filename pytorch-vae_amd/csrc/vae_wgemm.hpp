// bf16 weight-gradient GEMM of the conv / transposed-conv layers for every tile size.
//
//   dW[m][r][s][j] += Σ_{n,hu,wu} U'[n,hu,wu,m] · V'[n, hu*S-P+r, wu*S-P+s, j]
//
//   Conv2d bwd_filter:          U = dy (output grid), V = x  (input grid);  m = k,  j = c
//   ConvTranspose2d bwd_filter: U = x  (input grid),  V = dy (output grid); m = c,  j = k
//   (U', V' = the stored tensors with their per-channel transforms, template parameters XU / XV.)
//
// Both operands are NHWC with the reduction index (pixels) outermost: every pixel row goes
// global -> registers -> (transform) -> LDS as whole 16-byte chunks in its natural
// [pixel][channel] order, and the MFMA operand fragments are read back column-major with
// ds_read_b64_tr_b16 (lane 4q+p of a 16-lane group addresses row q, columns 4p..4p+3 of a 4x16
// block; lane i receives column i) — the K = pixel direction needs no transposing store.
//
// Why beside vae_wgrad.hpp's 128x128 kernel: the VanillaVAE layers have 32-512 channels and
// 256-65536 pixels, so one tile size cannot fill the chip; here BM x BJ is 32x32 .. 128x128,
// the pixel range is split over workgroups until ~2 per CU, the register ring keeps ~20 loads
// in flight (one memory round trip per workgroup for most layers, tools/kprobe.py), the
// BatchNorm tables are built in-kernel from the producers' replicated statistics, and the
// first workgroup publishes dL/dgamma, dL/dbeta and the closed-form conv-bias gradient of the
// BatchNorm whose backward it applies (vae_bn_finalize mode 1's work).
//
// LDS rows: 64 B (BM 32), 160 B (64), 288 B (128): the four 32-byte row segments a 16-lane
// transposed read touches fall in distinct bank groups.
#pragma once
#include "vae_cgemm.hpp"

namespace vae {

struct WgParams {
  const void* u; vae_xform u_xf; uint32_t u_bytes;   // [n][hu][wu][M]
  const void* v; vae_xform v_xf; uint32_t v_bytes;   // [n][hv][wv][J]
  int n, hu, wu, M;
  int hv, wv, J;
  int R, S, P;
  int kper;                          // pixels per K slice (multiple of 32)
  float* dw;                         // [M][R][R][J] fp32, accumulated
  float* db;                         // closed-form bias gradient (first workgroup; with u/v BN_DY extras)
  int dy_is_v;                       // which operand carries the BN_DY transform (bias gradient of its conv)
  FastDiv fd_wu, fd_hu, fd_r;
  float* slab;                       // non-NULL: K slice s stores its partial dW at slab + s*slab_ld
  long slab_ld;                      //   (plain stores; wg_slab_reduce adds the slices into dw)
  int own;                           // one K slice: each dW element has one writer, so it is
                                     // accumulated with a plain load + store instead of an atomic;
                                     // 2: written with a plain store (dW is this call's alone:
                                     // vae_conv_args.defer_reduce), no load of the old value
  int jst;                           // stored j extent of dw (0: J): dW is [M][R][R][jst], j >= jst
                                     // dropped (vae_conv_args.dw_inner: a zero-padded operand)
};

template <int BM> constexpr int wg_rs() { return BM == 32 ? 64 : (BM == 64 ? 160 : 288); }

typedef __bf16 __attribute__((ext_vector_type(4))) __attribute__((address_space(3))) wgm_lds_bf16x4;
typedef __bf16 wgm_bf16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ wgm_bf16x4 wgm_tr_read(const char* generic_lds_addr) {
  const uint32_t off = (uint32_t)(uintptr_t)generic_lds_addr;
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((wgm_lds_bf16x4*)(uintptr_t)off);
}

// pixels per K-step: 64 for the 128 x 128 tiles (VQ-VAE's residual convs: half the barriers per
// MFMA; two workgroups still fit a CU's LDS), 32 below
template <int BM> constexpr int wg_kp() { return BM >= 128 ? 64 : 32; }
// operand tiles of one workgroup (bytes of LDS): 2 buffers x (U + V) rows of KP pixels
template <int BM, int BJ, int KPX = 0> constexpr int wgemm_lds_bytes() {
  return 2 * (KPX > 0 ? KPX : wg_kp<BM>()) * (wg_rs<BM>() + wg_rs<BJ>());
}

// Accumulator tile -> dW (or this K slice's partial slab): lane element (i, j, e) is row
// mrow + 16i + e, column jcol + 16j, at offset row * rowstride + coff + column.  A single K slice
// (p.own) adds into dW with plain loads and stores: every old value is loaded first, then every
// sum is stored — interleaved, each load would wait behind the previous store (the compiler cannot
// prove the addresses distinct), one memory round trip per element.
template <int TM, int TJ>
__device__ __forceinline__ void wg_epilogue(const WgParams& p, float* part, const f32x4 (&acc)[TM][TJ], int mrow,
                                            int jcol, long rowstride, long coff) {
  const int jst = p.jst > 0 ? p.jst : p.J;
  if (!part && p.own == 2) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int mm = mrow + i * 16 + e, jj = jcol + j * 16;
          if (mm < p.M && jj < jst) p.dw[mm * rowstride + coff + jj] = acc[i][j][e];
        }
    return;
  }
  if (!part && p.own) {
    // in groups of fragment rows holding <= 32 values (registers: the 128 x 128 tiles run at 256)
    constexpr int GI = TJ * 4 * TM <= 32 ? TM : (32 / (TJ * 4) > 0 ? 32 / (TJ * 4) : 1);
#pragma unroll
    for (int i0 = 0; i0 < TM; i0 += GI) {
      float old[GI][TJ][4];
#pragma unroll
      for (int i = 0; i < GI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int mm = mrow + (i0 + i) * 16 + e, jj = jcol + j * 16;
            old[i][j][e] = (mm < p.M && jj < jst) ? p.dw[mm * rowstride + coff + jj] : 0.f;
          }
#pragma unroll
      for (int i = 0; i < GI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int mm = mrow + (i0 + i) * 16 + e, jj = jcol + j * 16;
            if (mm < p.M && jj < jst) p.dw[mm * rowstride + coff + jj] = old[i][j][e] + acc[i0 + i][j][e];
          }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int jj = jcol + j * 16;
      if (jj >= jst) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int mm = mrow + i * 16 + e;
        if (mm >= p.M) continue;
        const long o = mm * rowstride + coff + jj;
        if (part) part[o] = acc[i][j][e];
        else atomicAdd(p.dw + o, acc[i][j][e]);
      }
    }
}

// The per-tap weight-gradient GEMM of workgroup `bid` of its problem, operand tiles at `lds`
// (wgemm_lds_bytes) — called by wgemm_kernel (one problem per launch) and by wg_group_kernel
// (several layers' weight gradients in one launch, vae_wgrad_batch.hip).
// (clk: VAE_PROBE diagnostics — thread 0 records cycle counts after the prologue and the K loop)
#ifdef VAE_PROBE
#define WG_MARK(i) do { if (clk && threadIdx.x == 0) clk[i] = __builtin_readcyclecounter(); } while (0)
#else
#define WG_MARK(i) do { } while (0)
#endif
// nunits > 1 (the grouped launch, vae_wgrad_batch.hip): the workgroup runs work units bid0 ..
// bid0 + nunits - 1 of its layer one after another, building the BatchNorm tables once.
// KPX: pixels per K-step (0: wg_kp<BM>; the grouped launch runs its 64-wide tiles at 64)
template <int BM, int BJ, int XU, int XV, int KPX = 0>
__device__ __forceinline__ void wgemm_body(const WgParams& p, const int bid0, char* lds,
                                           unsigned long long* clk = nullptr, const int nunits = 1) {
  constexpr int KP = KPX > 0 ? KPX : wg_kp<BM>();
  constexpr int RSU = wg_rs<BM>(), RSV = wg_rs<BJ>();
  constexpr int CU = BM / 8, CV = BJ / 8;              // 16-byte chunks per pixel row
  constexpr int RPU = 256 / CU, RPV = 256 / CV;        // pixel rows per pass
  constexpr int UPT = RPU >= KP ? 1 : KP / RPU, VPT = RPV >= KP ? 1 : KP / RPV;
  constexpr bool DU = XU == VAE_X_BN_DY, DV = XV == VAE_X_BN_DY;
  constexpr bool BU = XU == VAE_X_BN_ACT || DU, BV = XV == VAE_X_BN_ACT || DV;
  constexpr int LOADS = UPT * (DU ? 2 : 1) + VPT * (DV ? 2 : 1);
  constexpr int NS = wg_stages<LOADS>();
  constexpr int WTM = BM / 2, WTJ = BJ / 2;            // 2 x 2 waves
  constexpr int TM = WTM / 16, TJ = WTJ / 16;

  char (*Us)[KP * RSU] = reinterpret_cast<char (*)[KP * RSU]>(lds);
  char (*Vs)[KP * RSV] = reinterpret_cast<char (*)[KP * RSV]>(lds + 2 * KP * RSU);
  extern __shared__ float tabs[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int gm = (p.M + BM - 1) / BM, gj = (p.J + BJ - 1) / BJ;
  const int per_slice = gm * gj * p.R * p.R;
  const long npix = (long)p.n * p.hu * p.wu;
  // per-thread chunk coordinates (all of a thread's rows share the chunk column)
  const int cu = tid % CU, ru0 = tid / CU, cv = tid % CV, rv0 = tid / CV;

  // the work unit: K slice, tap, output tile (re-decoded per unit)
  int slice, tap, r, s, m0, j0, chu, chv, nsteps;
  long k0, k1;
  bool cu_ok, cv_ok;
  auto decode = [&](int bid) {
    slice = bid / per_slice;
    int t = bid - slice * per_slice;
    const int tj = t % gj; t /= gj;
    const int tmi = t % gm;
    tap = t / gm;
    r = (int)p.fd_r.div(tap); s = tap - r * p.R;
    m0 = tmi * BM; j0 = tj * BJ;
    k0 = (long)slice * p.kper;
    k1 = min(npix, k0 + p.kper);
    nsteps = (int)((k1 - k0 + KP - 1) / KP);
    chu = m0 + cu * 8; chv = j0 + cv * 8;
    cu_ok = chu < p.M && ru0 < KP; cv_ok = chv < p.J && rv0 < KP;
  };
  decode(bid0);
  const Src<__bf16> su = make_src<__bf16>(p.u, p.u_bytes, p.u_xf);
  const Src<__bf16> sv = make_src<__bf16>(p.v, p.v_bytes, p.v_xf);

  struct Stage {
    uint32_t u[UPT][4], uy[DU ? UPT : 1][4];
    uint32_t v[VPT][4], vy[DV ? VPT : 1][4];
    uint32_t oku, okv;
  };
  auto issue = [&](int step, Stage& st) {
    const long kb = k0 + (long)step * KP;
    uint32_t oku = 0u, okv = 0u;
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
      const long pix = kb + ru0 + i * RPU;
      const bool in = cu_ok && pix < k1;
      oku |= (uint32_t)in << i;
      const uint32_t off = in ? (uint32_t)((pix * p.M + chu) * 2) : kOOB;
      bload<16>(su.x, off, st.u[i]);
      if constexpr (DU) bload<16>(su.y, off, st.uy[i]);
    }
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const long pix = kb + rv0 + i * RPV;
      const bool in = cv_ok && pix < k1;
      const uint32_t pp = in ? (uint32_t)pix : 0u;
      const uint32_t q = p.fd_wu.div(pp);
      const int wu_i = (int)(pp - q * (uint32_t)p.wu);
      const uint32_t nn = p.fd_hu.div(q);
      const int hu_i = (int)(q - nn * (uint32_t)p.hu);
      const int hv_i = hu_i * p.S - p.P + r, wv_i = wu_i * p.S - p.P + s;
      const bool vin = in && (uint32_t)hv_i < (uint32_t)p.hv && (uint32_t)wv_i < (uint32_t)p.wv;
      okv |= (uint32_t)vin << i;
      const uint32_t off = vin ? (uint32_t)(((((long)nn * p.hv + hv_i) * p.wv + wv_i) * p.J + chv) * 2) : kOOB;
      bload<16>(sv.x, off, st.v[i]);
      if constexpr (DV) bload<16>(sv.y, off, st.vy[i]);
    }
    st.oku = oku; st.okv = okv;
  };

  // tables: U transform [3][stride_u], V transform [3][stride_v]
  const int cau = tab_stride(p.u_xf.channels), cav = tab_stride(p.v_xf.channels);
  const Tab tu{tabs, tabs + cau, tabs + 2 * cau, nullptr, nullptr};
  float* q0 = tabs + (BU ? 3 * cau : 0);
  const Tab tv{q0, q0 + cav, q0 + 2 * cav, nullptr, nullptr};

  // table loads ahead of the ring's; the reductions' LDS scratch is the V tile area (>= 4 KB,
  // unused until the main loop)
  TabPre<DU ? 4 : 2> pu;
  TabPre<DV ? 4 : 2> pv;
  const bool u_pre = BU && tab_pre_ok<XU>(p.u_xf), v_pre = BV && tab_pre_ok<XV>(p.v_xf);
  if (u_pre) tab_pre_load(p.u_xf, pu);
  if (v_pre) tab_pre_load(p.v_xf, pv);
  Stage ring[NS];
#pragma unroll
  for (int u = 0; u < NS; ++u) issue(u, ring[u]);
  float* const scr = reinterpret_cast<float*>(Vs[0]);
  if constexpr (BU) tab_fill_pre(p.u_xf, pu, u_pre, tu, false, false, scr);
  if constexpr (BV) tab_fill_pre(p.v_xf, pv, v_pre, tv, false, false, scr);
  if (bid0 == 0) {
    // the BatchNorm whose backward this call applies: dL/dgamma, dL/dbeta (+ conv bias) once
    const vae_xform& dyx = p.dy_is_v ? p.v_xf : p.u_xf;
    if (dyx.kind == VAE_X_BN_DY && (p.db || dyx.dgamma_out || dyx.dbeta_out)) closed_form_db(dyx, p.db);
  }
  __syncthreads();
  WG_MARK(1);

  f32x4 acc[TM][TJ];

  auto store = [&](int buf, const Stage& st) {
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
      const int row = ru0 + i * RPU;
      if (row < KP) {
        uint4 w;
        if constexpr (XU == VAE_X_NONE) {
          w = uint4{st.u[i][0], st.u[i][1], st.u[i][2], st.u[i][3]};
        } else {
          const int ch = ((st.oku >> i) & 1u) ? chu : su.zs;   // out of range -> 0 after the transform
          w = cg_xform<XU>(st.u[i], st.uy[DU ? i : 0], tu, ch, su.slope);
        }
        *reinterpret_cast<uint4*>(Us[buf] + row * RSU + cu * 16) = w;
      }
    }
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int row = rv0 + i * RPV;
      if (row < KP) {
        uint4 w;
        if constexpr (XV == VAE_X_NONE) {
          w = uint4{st.v[i][0], st.v[i][1], st.v[i][2], st.v[i][3]};
        } else {
          const int ch = ((st.okv >> i) & 1u) ? chv : sv.zs;
          w = cg_xform<XV>(st.v[i], st.vy[DV ? i : 0], tv, ch, sv.slope);
        }
        *reinterpret_cast<uint4*>(Vs[buf] + row * RSV + cv * 16) = w;
      }
    }
  };
  // transposed-read addresses: lane 4q+p of 16-lane group g reads pixel rows 8g+4h+q, channels
  // c0 + 4p .. +3 of the fragment's 16 (byte offsets within a buffer)
  const int g = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  int aoff[TM][2], boff[TJ][2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = 8 * g + 4 * h + q4;
#pragma unroll
    for (int i = 0; i < TM; ++i) aoff[i][h] = row * RSU + (wm * WTM + i * 16 + 4 * p4) * 2;
#pragma unroll
    for (int j = 0; j < TJ; ++j) boff[j][h] = row * RSV + (wn * WTJ + j * 16 + 4 * p4) * 2;
  }
  auto compute = [&](int buf) {
#pragma unroll
    for (int kk = 0; kk < KP / 32; ++kk) {             // MFMA K = 32 pixels
      bf16x8 af[TM], bfr[TJ];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const wgm_bf16x4 a0 = wgm_tr_read(Us[buf] + kk * 32 * RSU + aoff[i][0]);
        const wgm_bf16x4 a1 = wgm_tr_read(Us[buf] + kk * 32 * RSU + aoff[i][1]);
#pragma unroll
        for (int e = 0; e < 4; ++e) { af[i][e] = a0[e]; af[i][4 + e] = a1[e]; }
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const wgm_bf16x4 b0 = wgm_tr_read(Vs[buf] + kk * 32 * RSV + boff[j][0]);
        const wgm_bf16x4 b1 = wgm_tr_read(Vs[buf] + kk * 32 * RSV + boff[j][1]);
#pragma unroll
        for (int e = 0; e < 4; ++e) { bfr[j][e] = b0[e]; bfr[j][4 + e] = b1[e]; }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  const int jst = p.jst > 0 ? p.jst : p.J;
  const long rowstride = (long)p.R * p.R * jst;
  for (int ut = 0; ut < nunits; ++ut) {
    if (ut > 0) {
      decode(bid0 + ut);
      __syncthreads();                                 // every wave is done with the LDS tiles
#pragma unroll
      for (int u = 0; u < NS; ++u) issue(u, ring[u]);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // main loop (vae_cgemm.hpp: loads issued on every path, LDS work skipped past the slice)
    int buf = 0;
    for (int kb = 0; kb < nsteps; kb += NS) {
#pragma unroll
      for (int u = 0; u < NS; ++u) {
        const bool live = kb + u < nsteps;
        if (live) store(buf, ring[u]);
        __syncthreads();
        issue(kb + u + NS, ring[u]);
        if (live) compute(buf);
        buf ^= 1;
      }
    }
    WG_MARK(2);
    // D[m][j]: lane holds rows 4g + e of fragment i, column li of fragment j
    float* const part = p.slab ? p.slab + (long)slice * p.slab_ld : nullptr;
    wg_epilogue<TM, TJ>(p, part, acc, m0 + wm * WTM + 4 * g, j0 + wn * WTJ + li, rowstride, (long)tap * jst);
  }
}

template <int BM, int BJ, int XU, int XV>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BM >= 128 ? 2 : 1)))
wgemm_kernel(const WgParams p) {
  kernarg_prefetch<(sizeof(WgParams) < 1024 ? sizeof(WgParams) : 1024)>();
  __shared__ __attribute__((aligned(16))) char lds[wgemm_lds_bytes<BM, BJ>()];
  wgemm_body<BM, BJ, XU, XV>(p, (int)blockIdx.x, lds);
}

// All R x R taps in one workgroup (small tiles): the U tile of a K-step is loaded and
// transformed once and reused by every tap (per-tap workgroups did it R*R times), V is gathered
// per tap from the pixel decomposition computed once per row.  Accumulators: R*R x the
// (BM/2 x BJ/2) wave tile.
// Stages in flight: one for the all-taps kernels above 10 loads a stage.  Two (the VAE_WGT_NS2
// build: 256 VGPRs + 68 AGPRs, one workgroup per CU, which the grouped launch holds anyway) measured
// no faster: VanillaVAE B=64 0.5395 vs 0.5337 ms/step (profiles/r4_v4_notes.txt); the 4x4
// kernels spilled 33-39 VGPRs at two.
template <int LOADS, int RR> constexpr int wgt_stages() {
#ifdef VAE_WGT_NS2
  return LOADS > 20 || (RR > 3 && LOADS > 10) ? 1 : (LOADS > 10 ? 2 : wg_stages<LOADS>());
#else
  return LOADS > 10 ? 1 : wg_stages<LOADS>();
#endif
}

// K-step: every thread loads one 16-byte chunk of U and of each tap's V row — 64 pixels for the
// 32-channel tiles (128 of the 256 threads idled at 32) — and the LDS holds one step (single
// buffer, two barriers per step) so two workgroups still fit a CU: each memory round trip (the
// loop is latency-bound, one step in flight per ring slot) now carries twice the MFMA work.
template <int BM, int BJ> constexpr int wgt_kp() {
  constexpr int RPU = 256 / (BM / 8), RPV = 256 / (BJ / 8);
  return RPU < RPV ? (RPU < 32 ? 32 : (RPU > 64 ? 64 : RPU)) : (RPV < 32 ? 32 : (RPV > 64 ? 64 : RPV));
}
template <int BM, int BJ> constexpr int wgt_nb() { return wgt_kp<BM, BJ>() > 32 ? 1 : 2; }   // LDS buffers
template <int BM, int BJ, int RR> constexpr int wgemm_taps_lds_bytes() {
  return wgt_nb<BM, BJ>() * wgt_kp<BM, BJ>() * (wg_rs<BM>() + RR * RR * wg_rs<BJ>());
}

template <int BM, int BJ, int XU, int XV, int RR>
__device__ __forceinline__ void wgemm_taps_body(const WgParams& p, const int bid, char* lds,
                                                unsigned long long* clk = nullptr) {
  constexpr int TAPS = RR * RR;
  constexpr int CU = BM / 8, CV = BJ / 8;
  constexpr int RPU = 256 / CU, RPV = 256 / CV;
  constexpr int KP = wgt_kp<BM, BJ>();
  constexpr int NB = wgt_nb<BM, BJ>();
  constexpr int RSU = wg_rs<BM>(), RSV = wg_rs<BJ>();
  constexpr int UPT = RPU >= KP ? 1 : KP / RPU, VPT = RPV >= KP ? 1 : KP / RPV;
  constexpr bool DU = XU == VAE_X_BN_DY, DV = XV == VAE_X_BN_DY;
  constexpr bool BU = XU == VAE_X_BN_ACT || DU, BV = XV == VAE_X_BN_ACT || DV;
  constexpr int LOADS = UPT * (DU ? 2 : 1) + TAPS * VPT * (DV ? 2 : 1);
  constexpr int NS = wgt_stages<LOADS, RR>();
  constexpr int WTM = BM / 2, WTJ = BJ / 2;
  constexpr int TM = WTM / 16, TJ = WTJ / 16;

  char (*Us)[KP * RSU] = reinterpret_cast<char (*)[KP * RSU]>(lds);
  char (*Vs)[TAPS][KP * RSV] = reinterpret_cast<char (*)[TAPS][KP * RSV]>(lds + NB * KP * RSU);
  extern __shared__ float tabs[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int gm = (p.M + BM - 1) / BM, gj = (p.J + BJ - 1) / BJ;
  const int per_slice = gm * gj;
  const int slice = bid / per_slice;
  const int t0 = bid - slice * per_slice;
  const int tj = t0 % gj, tmi = t0 / gj;
  const int m0 = tmi * BM, j0 = tj * BJ;
  const long npix = (long)p.n * p.hu * p.wu;
  const long k0 = (long)slice * p.kper;
  const long k1 = min(npix, k0 + p.kper);
  const int nsteps = (int)((k1 - k0 + KP - 1) / KP);

  const int cu = tid % CU, ru0 = tid / CU, cv = tid % CV, rv0 = tid / CV;
  const int chu = m0 + cu * 8, chv = j0 + cv * 8;
  const bool cu_ok = chu < p.M && ru0 < KP, cv_ok = chv < p.J && rv0 < KP;
  const Src<__bf16> su = make_src<__bf16>(p.u, p.u_bytes, p.u_xf);
  const Src<__bf16> sv = make_src<__bf16>(p.v, p.v_bytes, p.v_xf);

  struct Stage {
    uint32_t u[UPT][4], uy[DU ? UPT : 1][4];
    uint32_t v[TAPS][VPT][4], vy[DV ? TAPS : 1][DV ? VPT : 1][4];
    uint32_t oku, okv[TAPS];
  };
  auto issue = [&](int step, Stage& st) {
    const long kb = k0 + (long)step * KP;
    uint32_t oku = 0u;
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
      const long pix = kb + ru0 + i * RPU;
      const bool in = cu_ok && pix < k1;
      oku |= (uint32_t)in << i;
      const uint32_t off = in ? (uint32_t)((pix * p.M + chu) * 2) : kOOB;
      bload<16>(su.x, off, st.u[i]);
      if constexpr (DU) bload<16>(su.y, off, st.uy[i]);
    }
    st.oku = oku;
#pragma unroll
    for (int t = 0; t < TAPS; ++t) st.okv[t] = 0u;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const long pix = kb + rv0 + i * RPV;
      const bool in = cv_ok && pix < k1;
      const uint32_t pp = in ? (uint32_t)pix : 0u;
      const uint32_t q = p.fd_wu.div(pp);
      const int wu_i = (int)(pp - q * (uint32_t)p.wu);
      const uint32_t nn = p.fd_hu.div(q);
      const int hu_i = (int)(q - nn * (uint32_t)p.hu);
      const int hb = hu_i * p.S - p.P, wb = wu_i * p.S - p.P;
      const long nbase = (long)nn * p.hv;
#pragma unroll
      for (int t = 0; t < TAPS; ++t) {
        const int hv_i = hb + t / RR, wv_i = wb + t % RR;
        const bool vin = in && (uint32_t)hv_i < (uint32_t)p.hv && (uint32_t)wv_i < (uint32_t)p.wv;
        st.okv[t] |= (uint32_t)vin << i;
        const uint32_t off = vin ? (uint32_t)((((nbase + hv_i) * p.wv + wv_i) * p.J + chv) * 2) : kOOB;
        bload<16>(sv.x, off, st.v[t][i]);
        if constexpr (DV) bload<16>(sv.y, off, st.vy[t][i]);
      }
    }
  };

  const int cau = tab_stride(p.u_xf.channels), cav = tab_stride(p.v_xf.channels);
  const Tab tu{tabs, tabs + cau, tabs + 2 * cau, nullptr, nullptr};
  float* q0 = tabs + (BU ? 3 * cau : 0);
  const Tab tv{q0, q0 + cav, q0 + 2 * cav, nullptr, nullptr};

  // table loads ahead of the ring's; the reductions' LDS scratch is the V tile area (>= 4 KB,
  // unused until the main loop)
  TabPre<DU ? 4 : 2> pu;
  TabPre<DV ? 4 : 2> pv;
  const bool u_pre = BU && tab_pre_ok<XU>(p.u_xf), v_pre = BV && tab_pre_ok<XV>(p.v_xf);
  if (u_pre) tab_pre_load(p.u_xf, pu);
  if (v_pre) tab_pre_load(p.v_xf, pv);
  Stage ring[NS];
#pragma unroll
  for (int u = 0; u < NS; ++u) issue(u, ring[u]);
  float* const scr = reinterpret_cast<float*>(Vs[0][0]);
  if constexpr (BU) tab_fill_pre(p.u_xf, pu, u_pre, tu, false, false, scr);
  if constexpr (BV) tab_fill_pre(p.v_xf, pv, v_pre, tv, false, false, scr);
  if (bid == 0) {
    const vae_xform& dyx = p.dy_is_v ? p.v_xf : p.u_xf;
    if (dyx.kind == VAE_X_BN_DY && (p.db || dyx.dgamma_out || dyx.dbeta_out)) closed_form_db(dyx, p.db);
  }
  __syncthreads();
  WG_MARK(1);

  f32x4 acc[TAPS][TM][TJ];
#pragma unroll
  for (int t = 0; t < TAPS; ++t)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) acc[t][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto store = [&](int buf, const Stage& st) {
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
      const int row = ru0 + i * RPU;
      if (row < KP) {
        uint4 w;
        if constexpr (XU == VAE_X_NONE) {
          w = uint4{st.u[i][0], st.u[i][1], st.u[i][2], st.u[i][3]};
        } else {
          const int ch = ((st.oku >> i) & 1u) ? chu : su.zs;
          w = cg_xform<XU>(st.u[i], st.uy[DU ? i : 0], tu, ch, su.slope);
        }
        *reinterpret_cast<uint4*>(Us[buf] + row * RSU + cu * 16) = w;
      }
    }
#pragma unroll
    for (int t = 0; t < TAPS; ++t)
#pragma unroll
      for (int i = 0; i < VPT; ++i) {
        const int row = rv0 + i * RPV;
        if (row < KP) {
          uint4 w;
          if constexpr (XV == VAE_X_NONE) {
            w = uint4{st.v[t][i][0], st.v[t][i][1], st.v[t][i][2], st.v[t][i][3]};
          } else {
            const int ch = ((st.okv[t] >> i) & 1u) ? chv : sv.zs;
            w = cg_xform<XV>(st.v[t][i], st.vy[DV ? t : 0][DV ? i : 0], tv, ch, sv.slope);
          }
          *reinterpret_cast<uint4*>(Vs[buf][t] + row * RSV + cv * 16) = w;
        }
      }
  };
  const int g = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  int aoff[TM][2], boff[TJ][2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = 8 * g + 4 * h + q4;
#pragma unroll
    for (int i = 0; i < TM; ++i) aoff[i][h] = row * RSU + (wm * WTM + i * 16 + 4 * p4) * 2;
#pragma unroll
    for (int j = 0; j < TJ; ++j) boff[j][h] = row * RSV + (wn * WTJ + j * 16 + 4 * p4) * 2;
  }
  auto compute = [&](int buf) {
#pragma unroll
    for (int kk = 0; kk < KP / 32; ++kk) {             // MFMA K = 32 pixels
      bf16x8 af[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const wgm_bf16x4 a0 = wgm_tr_read(Us[buf] + kk * 32 * RSU + aoff[i][0]);
        const wgm_bf16x4 a1 = wgm_tr_read(Us[buf] + kk * 32 * RSU + aoff[i][1]);
#pragma unroll
        for (int e = 0; e < 4; ++e) { af[i][e] = a0[e]; af[i][4 + e] = a1[e]; }
      }
#pragma unroll
      for (int t = 0; t < TAPS; ++t) {
        bf16x8 bfr[TJ];
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const wgm_bf16x4 b0 = wgm_tr_read(Vs[buf][t] + kk * 32 * RSV + boff[j][0]);
          const wgm_bf16x4 b1 = wgm_tr_read(Vs[buf][t] + kk * 32 * RSV + boff[j][1]);
#pragma unroll
          for (int e = 0; e < 4; ++e) { bfr[j][e] = b0[e]; bfr[j][4 + e] = b1[e]; }
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[t][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[t][i][j], 0, 0, 0);
      }
    }
  };

  int buf = 0;
  for (int kb = 0; kb < nsteps; kb += NS) {
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      const bool live = kb + u < nsteps;
      if constexpr (NB == 1) __syncthreads();         // the previous step's reads of the buffer
      if (live) store(buf, ring[u]);
      __syncthreads();
      issue(kb + u + NS, ring[u]);
      if (live) compute(buf);
      if constexpr (NB == 2) buf ^= 1;
    }
  }
  WG_MARK(2);
  const int jst = p.jst > 0 ? p.jst : p.J;
  const long rowstride = (long)TAPS * jst;
  float* const part = p.slab ? p.slab + (long)slice * p.slab_ld : nullptr;
#pragma unroll
  for (int t = 0; t < TAPS; ++t)
    wg_epilogue<TM, TJ>(p, part, acc[t], m0 + wm * WTM + 4 * g, j0 + wn * WTJ + li, rowstride, (long)t * jst);
}

template <int BM, int BJ, int XU, int XV, int RR>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RR >= 4 ? 2 : 1)))
wgemm_taps_kernel(const WgParams p) {
  kernarg_prefetch<(sizeof(WgParams) < 1024 ? sizeof(WgParams) : 1024)>();
  __shared__ __attribute__((aligned(16))) char lds[wgemm_taps_lds_bytes<BM, BJ, RR>()];
  wgemm_taps_body<BM, BJ, XU, XV, RR>(p, (int)blockIdx.x, lds);
}

// dw[c] += sum over the K slices of slab[s][c]: blockIdx.y takes a contiguous run of slices, one
// float4 of columns per thread, one atomic per column per run (cols % 4 == 0, 16-byte aligned).
static __global__ void __launch_bounds__(256) wg_slab_reduce(const float* slab, long cols, int slices, int per_part,
                                                       float* dw) {
  const long c = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (c >= cols) return;
  const int s0 = blockIdx.y * per_part;
  const int s1 = min(slices, s0 + per_part);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  int s = s0;
  for (; s + 4 <= s1; s += 4) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(slab + (long)s * cols + c);
    const f32x4 b = *reinterpret_cast<const f32x4*>(slab + (long)(s + 1) * cols + c);
    const f32x4 d = *reinterpret_cast<const f32x4*>(slab + (long)(s + 2) * cols + c);
    const f32x4 e = *reinterpret_cast<const f32x4*>(slab + (long)(s + 3) * cols + c);
    acc += (a + b) + (d + e);
  }
  for (; s < s1; ++s) acc += *reinterpret_cast<const f32x4*>(slab + (long)s * cols + c);
#pragma unroll
  for (int i = 0; i < 4; ++i) atomicAdd(dw + c + i, acc[i]);
}

// ------------------------------------------------------------------ host
inline bool wg2_ok(int dtype, const vae_xform& ux, const vae_xform& vx, long u_elems, long v_elems, int M, int J,
                   const void* u, const void* v) {
  if (dtype != VAE_BF16) return false;
  if (M % 8 || J % 8) return false;
  if (u_elems * 2 >= (1l << 31) || v_elems * 2 >= (1l << 31)) return false;
  if (((uintptr_t)u & 15) || ((uintptr_t)v & 15)) return false;
  auto ok = [](const vae_xform& x) {
    if (x.kind == VAE_X_BN_DY && ((uintptr_t)x.aux & 15)) return false;
    if (x.kind == VAE_X_BN_ACT || x.kind == VAE_X_BN_DY) return x.channels <= MAXC;
    return true;
  };
  return ok(ux) && ok(vx);
}

template <int BM, int BJ, int XU, int XV>
inline void wg2_launch_k(const WgParams& p, unsigned blocks, hipStream_t st) {
  const bool bu = XU == VAE_X_BN_ACT || XU == VAE_X_BN_DY, bv = XV == VAE_X_BN_ACT || XV == VAE_X_BN_DY;
  const size_t lds = (size_t)((bu ? 3 * tab_stride(p.u_xf.channels) : 0) + (bv ? 3 * tab_stride(p.v_xf.channels) : 0)) * 4;
  if constexpr (BM == 32) {
    // 32 x 32 tiles of 3x3 kernels: every tap in one workgroup (the grid was sized without the
    // tap factor); larger tiles / kernels would exceed the LDS and register budget
    if (p.R == 3) { VAE_LAUNCH((wgemm_taps_kernel<BM, BJ, XU, XV, 3>), dim3(blocks), dim3(256), lds, st, p); return; }
    // 4x4 kernels without BatchNorm transforms (VQ-VAE's RGB ends, 8-channel padded side): the
    // wide operand is read once per K-step for all 16 taps instead of once per tap (wg_taps)
    if constexpr (XU <= VAE_X_ACT && XV <= VAE_X_ACT) {
      if (p.R == 4) { VAE_LAUNCH((wgemm_taps_kernel<BM, BJ, XU, XV, 4>), dim3(blocks), dim3(256), lds, st, p); return; }
    }
  }
  VAE_LAUNCH((wgemm_kernel<BM, BJ, XU, XV>), dim3(blocks), dim3(256), lds, st, p);
}

template <int BM, int BJ, int XU>
inline void wg2_launch_v(const WgParams& p, unsigned blocks, hipStream_t st) {
  switch (p.v_xf.kind) {
    case VAE_X_NONE: wg2_launch_k<BM, BJ, XU, VAE_X_NONE>(p, blocks, st); break;
    case VAE_X_ACT: wg2_launch_k<BM, BJ, XU, VAE_X_ACT>(p, blocks, st); break;
    case VAE_X_BN_ACT: wg2_launch_k<BM, BJ, XU, VAE_X_BN_ACT>(p, blocks, st); break;
    default: wg2_launch_k<BM, BJ, XU, VAE_X_BN_DY>(p, blocks, st); break;
  }
}

template <int BM, int BJ>
inline void wg2_launch_u(const WgParams& p, unsigned blocks, hipStream_t st) {
  switch (p.u_xf.kind) {
    case VAE_X_NONE: wg2_launch_v<BM, BJ, VAE_X_NONE>(p, blocks, st); break;
    case VAE_X_ACT: wg2_launch_v<BM, BJ, VAE_X_ACT>(p, blocks, st); break;
    case VAE_X_BN_ACT: wg2_launch_v<BM, BJ, VAE_X_BN_ACT>(p, blocks, st); break;
    default: wg2_launch_v<BM, BJ, VAE_X_BN_DY>(p, blocks, st); break;
  }
}

// K slices at or above which the partials go through a workspace slab and wg_slab_reduce
// instead of fp32 atomics straight into dw: hundreds of workgroups adding into the same few
// thousand words serialise at the L2.  Measured (B=64): the decoder's final ConvT wgrad (512
// slices x 9216 words) 45.3 -> 33.5 us and the first conv's (512 x 2304) 36.3 -> 20.7 us with the
// slab; at 256 slices x 18432 words or 28 slices x 295k words the slab traffic costs more than the
// atomics save (26 -> 32 us, 19 -> 55 us), hence the slice floor and the byte cap.
constexpr int kWgSlabMin = 384;
constexpr long kWgSlabMaxBytes = 32l << 20;

// A planned weight-gradient GEMM: tile, kernel kind, grid and K slices of one layer.
struct WgPlan {
  WgParams p;
  int T;            // square tile BM = BJ
  int taps;         // RR of the all-taps kernel (wgemm_taps_kernel), 0: one tap per workgroup
  unsigned blocks;
  long split;       // K slices
  long cols;        // dW elements (M * R * R * J)
};

// Plan one layer (tile, K slices, partial slab in `ws` when it pays); launches nothing.
// slots_req > 0: the workgroups this layer should take (a share of a grouped launch) instead of
// ~2 per CU of its own.
inline int wg2_plan(WgParams p, void* ws, long ws_bytes, WgPlan* out, long slots_req = 0, int slab_min = kWgSlabMin) {
  p.fd_wu = make_fastdiv(p.wu);
  p.fd_hu = make_fastdiv(p.hu);
  p.fd_r = make_fastdiv(p.R);
  const long npix = (long)p.n * p.hu * p.wu;
  p.u_bytes = (uint32_t)(npix * p.M * 2);
  p.v_bytes = (uint32_t)((long)p.n * p.hv * p.wv * p.J * 2);
  // tile: square, the largest whose both sides fit the channel counts
  const int mn = p.M < p.J ? p.M : p.J;
  int T = mn >= 128 ? 128 : (mn >= 64 ? 64 : 32);
  // wide BatchNorm tables (the Autoencoder's 2048-4096 channels) and the operand tiles share the LDS
  {
    const bool bu = p.u_xf.kind == VAE_X_BN_ACT || p.u_xf.kind == VAE_X_BN_DY;
    const bool bv = p.v_xf.kind == VAE_X_BN_ACT || p.v_xf.kind == VAE_X_BN_DY;
    const long tab = 4l * ((bu ? 3 * tab_stride(p.u_xf.channels) : 0) + (bv ? 3 * tab_stride(p.v_xf.channels) : 0));
    auto tile_lds = [](int t) -> long { return 2l * (t >= 128 ? 64 : 32) * 2 * (t == 32 ? 64 : (t == 64 ? 160 : 288)); };
    while (T > 32 && tab + tile_lds(T) > kLdsBytes) T /= 2;
    if (tab + tile_lds(T) + 8192 > kLdsBytes) return fail(VAE_E_UNSUPPORTED, "wgemm: per-channel tables exceed the LDS");
  }
  const bool taps_in_block = T == 32 && (p.R == 3 || (p.R == 4 && p.u_xf.kind <= VAE_X_ACT && p.v_xf.kind <= VAE_X_ACT));
  const long tiles = (long)((p.M + T - 1) / T) * ((p.J + T - 1) / T) * (taps_in_block ? 1 : p.R * p.R);
  const long ksteps = (npix + 31) / 32;
  // K slices: ~2 workgroups per CU, >= 4 K-steps per slice (16 for 1x1 kernels: their few output
  // tiles would otherwise be split hundreds of ways and every slice adds its whole tile into dw
  // with fp32 atomics — measured on the VQ-VAE residual 1x1 (M = J = 256, 32768 pixels): 128
  // slices 44.4 us, 64 slices 32.7 us, 32 slices 32.5 us, 16 slices 48.7 us; the 3x3 layers and
  // VanillaVAE's are slower with the higher floor)
  const int mink = p.R == 1 ? 16 : 4;
  const long slots = slots_req > 0 ? slots_req : 2l * kCUs;
  long split = (slots + tiles - 1) / tiles;
  if (split > ksteps / mink) split = ksteps / mink;
  // one round of workgroups: ceil(slots / tiles) slices overfill the slots by up to tiles - 1
  // workgroups, which then run as a second round on a few CUs (VQ-VAE 3x3: 36 tiles x 15 slices
  // = 540 workgroups for 512 slots) — take floor(slots / tiles) slices instead
  if (tiles * split > slots && tiles <= slots) split = slots / tiles;
  if (split < 1) split = 1;
  p.kper = (int)(((ksteps + split - 1) / split) * 32);
  split = (npix + p.kper - 1) / p.kper;
  const long cols = (long)p.M * p.R * p.R * p.J;
  p.slab = nullptr;
  p.slab_ld = cols;
  if (split >= slab_min && split * cols * 4 <= kWgSlabMaxBytes && (ws || querying()) && cols % 4 == 0 && !p.jst) {
    if (!ws_fits(split * cols * 4, ws_bytes, "wgemm K-slice partials")) return VAE_E_BADARG;
    p.slab = static_cast<float*>(ws);
  }
  p.own = (split == 1 && !p.slab) ? 1 : 0;
  out->p = p;
  out->T = T;
  out->taps = taps_in_block ? p.R : 0;
  out->blocks = (unsigned)(tiles * split);
  out->split = split;
  out->cols = cols;
  return VAE_OK;
}

inline void wg2_launch_main(const WgPlan& w, hipStream_t st) {
  if (w.T == 128) wg2_launch_u<128, 128>(w.p, w.blocks, st);
  else if (w.T == 64) wg2_launch_u<64, 64>(w.p, w.blocks, st);
  else wg2_launch_u<32, 32>(w.p, w.blocks, st);
}

// dw += the K slices' partials (a layer whose plan took a slab)
inline int wg2_reduce(const WgPlan& w, hipStream_t st) {
  if (!w.p.slab) return VAE_OK;
  const long split = w.split, cols = w.cols;
  const int parts = split < 32 ? (int)split : 32;
  const int per = (int)((split + parts - 1) / parts);
  const dim3 grid((unsigned)((cols / 4 + 255) / 256), (unsigned)((split + per - 1) / per));
  VAE_LAUNCH(wg_slab_reduce, grid, dim3(256), 0, st, (const float*)w.p.slab, cols, (int)split, per, w.p.dw);
  return check_launch("wg_slab_reduce");
}

// the LDS-DMA weight-gradient GEMM for the large transform-free layers (vae_bgemm.hip)
bool bwg_ok(const WgParams& p);
int bwg_launch(WgParams p, hipStream_t st);

inline int wg2_launch(WgParams p, void* ws, long ws_bytes, hipStream_t st) {
  if (bwg_ok(p)) return bwg_launch(p, st);
  WgPlan w;
  if (int rc = wg2_plan(p, ws, ws_bytes, &w)) return rc;
  wg2_launch_main(w, st);
  if (int rc = check_launch("wgemm")) return rc;
  return wg2_reduce(w, st);
}

// The bf16 weight-gradient GEMM parameters of a Conv2d / ConvTranspose2d bwd_filter call, when
// the call takes that path (bf16 NHWC operands, channels % 8, 16-byte aligned tensors):
//   Conv2d:          U = dy (output grid, m = k), V = x  (input grid, j = c)
//   ConvTranspose2d: U = x  (input grid,  m = c), V = dy (output grid, j = k)
// The bias gradient goes through the GEMM only in closed form (dy_xf BN_DY); *closed says so.
inline bool conv_wg_params(const vae_conv_args* a, bool transposed, WgParams* w, bool* closed) {
  *closed = a->db && a->dy_xf.kind == VAE_X_BN_DY;
  const long xe = (long)a->n * a->h * a->w * a->c, ye = (long)a->n * a->p * a->q * a->k;
  if (a->x_nchw_f32) return false;
  if (!transposed ? !wg2_ok(a->dtype, a->dy_xf, a->x_xf, ye, xe, a->k, a->c, a->dy, a->x)
                  : !wg2_ok(a->dtype, a->x_xf, a->dy_xf, xe, ye, a->c, a->k, a->x, a->dy)) return false;
  memset(w, 0, sizeof(*w));
  if (!transposed) {
    w->u = a->dy; w->u_xf = sanitize(a->dy_xf); w->v = a->x; w->v_xf = sanitize(a->x_xf);
    w->n = a->n; w->hu = a->p; w->wu = a->q; w->M = a->k; w->hv = a->h; w->wv = a->w; w->J = a->c;
  } else {
    w->u = a->x; w->u_xf = sanitize(a->x_xf); w->v = a->dy; w->v_xf = sanitize(a->dy_xf);
    w->n = a->n; w->hu = a->h; w->wu = a->w; w->M = a->c; w->hv = a->p; w->wv = a->q; w->J = a->k;
  }
  w->R = a->r; w->S = a->stride; w->P = a->pad; w->dw = a->dw;
  w->jst = (a->dw_inner > 0 && a->dw_inner < w->J) ? a->dw_inner : 0;
  w->db = *closed ? a->db : nullptr;
  w->dy_is_v = transposed ? 1 : 0;
  return true;
}

}  // namespace vae
