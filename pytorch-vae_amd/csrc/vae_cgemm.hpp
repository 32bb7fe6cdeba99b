// bf16 NHWC implicit GEMM for the forward and data-gradient convolutions of the VAE step
// (Conv2d / ConvTranspose2d forward, and their data gradients) — the hot path of bf16 mode.
//
//   C[m][n] = Σ_k xf(A)(m, k) · B[n][k]
//
//   A: the gathered activation / gradient (im2col of a strided conv, A_CONV; or the sub-pixel
//      phase gather of a transposed conv / conv data gradient, A_CONVT), with its per-channel
//      transform (XA: none, LeakyReLU, BatchNorm+LeakyReLU, BatchNorm-backward) applied once
//      per element on its way into LDS.
//   B: weights, always k-contiguous rows: [N][R][S][C] (Conv2d forward, ConvTranspose2d data
//      gradient: the stored layout), or the swapped-axes copy [N][R][S][C] of a
//      ConvTranspose2d forward / Conv2d data gradient (vae_swap_axes; the phase gather then
//      addresses the taps it uses through (r, s)).
//
// Why a third GEMM kernel (vae_igemm.hpp stays for fp32 parity mode and odd shapes): the
// VanillaVAE layers are latency-bound (0.3-1.2 GFLOP, 1-20 MB each, profiles/r1_v6_*), and the
// generic kernel spent ~0.6 us per 64-deep K-tile on a register ring that the compiler drained
// (vmcnt(0)) at every ring turn behind runtime transform branches.  Here the transform kind is
// a template parameter (no branch between a load and its use), K-steps are up to 128 deep (one
// barrier per step), the prefetch ring is sized from the loads one step needs, and the epilogue
// goes through LDS so aux loads and output stores are 16-byte vectors.
//
// Block: 256 threads = 4 waves, BM x BN tile, wave tile (BM/WM) x (BN/WN) of 16x16 MFMA
// fragments (v_mfma_f32_16x16x32_bf16: lane l holds row l&15, k 8*(l>>4)..+7 of A; col l&15 of
// B; output rows 4*(l>>4)..+3 of col l&15).  LDS rows are BK+8 elements (16-B pad: the
// 16-lane groups of ds_read_b128 hit distinct 4-dword bank groups).
#pragma once
#include "vae_igemm.hpp"

namespace vae {

template <int BM, int BN> struct CgWaves {
  static constexpr int WN = BN >= 2 * BM ? 4 : (BM >= 2 * BN ? 1 : 2);
  static constexpr int WM = 4 / WN;
  static constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  static_assert(TM >= 1 && TN >= 1, "wave tile below 16x16");
};

// transform of one 16-byte chunk (8 consecutive channels from ch) -> 4 packed bf16 pairs
template <int XA>
__device__ __forceinline__ uint4 cg_xform(const uint32_t (&w)[4], const uint32_t (&y)[4], const Tab& t, int ch,
                                          float slope) {
  if constexpr (XA == VAE_X_NONE) {
    return uint4{w[0], w[1], w[2], w[3]};
  } else {
    // channel pairs (2e, 2e+1) in packed fp32 (v_pk_fma_f32 / v_pk_mul_f32: half the VALU issue of
    // the scalar form — this transform runs once per gathered element, measured +1.5-2 us per
    // launch in the K loop, tools/kprobe.py) and one v_cvt_pk_bf16_f32 per pair
    uint4 o;
    uint32_t* op = reinterpret_cast<uint32_t*>(&o);
    f32x2 ab[4], bb[4], cb[4];
    if constexpr (XA != VAE_X_ACT) {                  // (LeakyReLU alone has no table)
      const f32x4 a0 = tab4(t.a, ch), a1 = tab4(t.a, ch + 4);
      ab[0] = f32x2{a0[0], a0[1]}; ab[1] = f32x2{a0[2], a0[3]}; ab[2] = f32x2{a1[0], a1[1]}; ab[3] = f32x2{a1[2], a1[3]};
      {
        const f32x4 b0 = tab4(t.b, ch), b1 = tab4(t.b, ch + 4);
        bb[0] = f32x2{b0[0], b0[1]}; bb[1] = f32x2{b0[2], b0[3]}; bb[2] = f32x2{b1[0], b1[1]}; bb[3] = f32x2{b1[2], b1[3]};
      }
      if constexpr (XA == VAE_X_BN_DY) {
        const f32x4 c0 = tab4(t.c, ch), c1 = tab4(t.c, ch + 4);
        cb[0] = f32x2{c0[0], c0[1]}; cb[1] = f32x2{c0[2], c0[3]}; cb[2] = f32x2{c1[0], c1[1]}; cb[3] = f32x2{c1[2], c1[3]};
      }
    }
    const f32x2 sl = f32x2{slope, slope};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const f32x2 v = f32x2{__uint_as_float(w[e] << 16), __uint_as_float(w[e] & 0xffff0000u)};
      f32x2 r;
      if constexpr (XA == VAE_X_ACT) {
        r = __builtin_elementwise_max(v, v * sl);
      } else if constexpr (XA == VAE_X_BN_ACT) {
        const f32x2 z = __builtin_elementwise_fma(v, ab[e], bb[e]);
        r = __builtin_elementwise_max(z, z * sl);
      } else {  // BN_DY: a*g + b*y + c
        const f32x2 u = f32x2{__uint_as_float(y[e] << 16), __uint_as_float(y[e] & 0xffff0000u)};
        r = __builtin_elementwise_fma(ab[e], v, __builtin_elementwise_fma(bb[e], u, cb[e]));
      }
      bf16x2 pk;
      pk[0] = (__bf16)r[0];
      pk[1] = (__bf16)r[1];
      op[e] = *reinterpret_cast<uint32_t*>(&pk);
    }
    return o;
  }
}

// Register ring depth from the loads one K-step needs per thread: ~20 16-byte loads in flight
// (80 VGPRs).  The VanillaVAE layers have 1-9 K-steps, so for most of them the whole K range is
// requested in the prologue and a block pays one memory round trip, not one per step (the
// round trip under load is 1.5-2 us, tools/kprobe.py).
// ~20 16-byte loads in flight per thread (80 VGPRs).  Measured at 40 (kRingMax 12): the 5-9
// K-step layers gain 1-3 us from one fewer round trip, the big-M maps lose as much or more to the
// halved occupancy (VanillaVAE step 0.760 -> 0.767 ms), so the ring stays at 20.
constexpr int kRingLoads = 20, kRingMax = 8;
constexpr int cg_ring(int loads) {
  return kRingLoads / loads < 2 ? 2 : (kRingLoads / loads > kRingMax ? kRingMax : kRingLoads / loads);
}
template <int LOADS> constexpr int cg_stages() { return cg_ring(LOADS); }
// OR == 3: a one-round kernel with twice the ring, for forward grids of at most two workgroups per
// CU (the deep layers: 256-512 tiles of 5-10 K-steps), whose occupancy the extra registers do not
// lower — their whole K slice is requested in the prologue instead of one ring refill per step
// (VanillaVAE forward convs 1-2 us each faster)
constexpr int kRingLoadsDeep = 40, kRingMaxDeep = 16;
constexpr int cg_ring_deep(int loads) {
  return kRingLoadsDeep / loads < 2 ? 2 : (kRingLoadsDeep / loads > kRingMaxDeep ? kRingMaxDeep : kRingLoadsDeep / loads);
}
// the weight-gradient kernels keep ~20 loads in flight (their K slices are sized for it)
template <int LOADS> constexpr int wg_stages() {
  return 20 / LOADS < 2 ? 2 : (20 / LOADS > 8 ? 8 : 20 / LOADS);
}

template <int BM, int BN, int BK, int NBUF = 2> struct CgSmem {
  static constexpr int LDK = BK + 8;
  static constexpr int LOOP = NBUF * (BM + BN) * LDK * 2;       // bytes: (double-)buffered A and B tiles
  static constexpr int EPI = BM * (BN + 4) * 4;                 // fp32 accumulator tile
  static constexpr int BYTES = LOOP > EPI ? LOOP : EPI;
};

// OR ("one round"): every workgroup's K slice fits the register ring (host-checked), so the
// prologue requests all of it and the loop never refills.  OR == 2: at most two K-steps per slice
// (the big-M maps: K = 72-288), so the ring is cut to two stages — the registers of the unused
// stages would otherwise halve the workgroups a CU holds while these launches are latency-bound.
// Waves per SIMD the register allocation must leave room for: the 128 x 128 tiles (VQ-VAE's
// MFMA-bound convolutions) otherwise take ~300 VGPRs + AGPRs = one workgroup per CU, 4 waves to
// hide every load; the 64 x 32 BatchNorm-backward dgrad tiles fit 3 workgroups in LDS.
template <int BM, int BN, int XA> constexpr int cg_waves_per_eu() {
  return (BM >= 128 && BN >= 128) ? 2 : ((BM == 64 && BN == 32 && XA == VAE_X_BN_DY) ? 3 : 1);
}

// The tile work of workgroup `bid` (operand tiles / epilogue tile at `smem`, CgSmem<...NBUF>::BYTES).
template <int BM, int BN, int BK, int AM, int XA, int EM, int OR>
__device__ __forceinline__ void cgemm_body(const GemmParams& p, const int bid, char* smem) {
  using WG = CgWaves<BM, BN>;
  constexpr int TM = WG::TM, TN = WG::TN, WTM = TM * 16, WTN = TN * 16;
  constexpr int LDK = CgSmem<BM, BN, BK>::LDK;
  constexpr int KC = BK / 8;                         // 16-byte chunks per tile row
  constexpr int RPP = 256 / KC;                      // rows covered per pass of the block
  constexpr int APT = (BM + RPP - 1) / RPP, BPT = (BN + RPP - 1) / RPP;
  constexpr bool DY = XA == VAE_X_BN_DY;
  constexpr int NSF = OR == 3 ? cg_ring_deep(APT * (DY ? 2 : 1) + BPT) : cg_stages<APT * (DY ? 2 : 1) + BPT>();
  constexpr int NS = OR == 2 ? (NSF < 2 ? NSF : 2) : NSF;
  // OR == 2 keeps one LDS buffer (a barrier between its two steps): with half the LDS, 4-6
  // workgroups fit a CU instead of 2-3 — these big-M launches have thousands of short workgroups
  constexpr int NBUF = OR == 2 ? 1 : 2;
  constexpr bool ABN = XA == VAE_X_BN_ACT || XA == VAE_X_BN_DY;
  static_assert(BM % RPP == 0 || BM < RPP, "A tile rows");
  static_assert(BN % RPP == 0 || BN < RPP, "B tile rows");

  extern __shared__ float tabs[];
  __bf16* As = reinterpret_cast<__bf16*>(smem);                 // [2][BM][LDK]
  __bf16* Bs = As + NBUF * BM * LDK;                             // [NBUF][BN][LDK]

#ifdef VAE_PROBE
  unsigned long long clk[4] = {0, 0, 0, 0};
  const unsigned long long wall0 = threadIdx.x == 0 ? wall_clock64() : 0;
#endif
  PROBE_MARK(0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WG::WN, wn = wave % WG::WN;
  // XCD-aware tile order (1-D grid): workgroups are dealt round-robin over the 8 XCDs, so
  // workgroup b runs on XCD b % 8 (speed only, never correctness).  Each XCD takes a contiguous
  // range of tiles ordered n (column tile) fastest, then phase / K slice, then m: the output
  // rows of one XCD gather overlapping input rows (3x3 taps, the phases of a transposed conv,
  // every column tile) that its own L2 then serves, instead of the Infinity Cache.  Layers whose
  // weights outweigh the gathered input (the deep 256-512-channel layers: 2.4 MB of weights
  // against 0.3-1 MB of activations) order m fastest instead (p.m_fast), so an XCD fetches only its
  // own weight columns (the n-fastest order fetched every column on all 8: 19.9 MB of traffic for
  // a 3.2 MB layer, r4_v5_pmc.json).
  const int gm = (p.M + BM - 1) / BM, gn = (p.N + BN - 1) / BN, gz = p.nphase * p.ksplit;
  int tile;
  {
    const int nb = gm * gn * gz, b = bid;
    const int q = nb >> 3, r = nb & 7, x = b & 7, loc = b >> 3;
    tile = x * q + min(x, r) + loc;
  }
  int tn, tz, tmi;
  if (p.m_fast) { tmi = tile % gm; tz = (tile / gm) % gz; tn = tile / (gm * gz); }
  else { tn = tile % gn; tz = (tile / gn) % gz; tmi = tile / (gn * gz); }
  const int m0 = tmi * BM, n0 = tn * BN;
  const int phase = (p.nphase > 1) ? (int)(tz / p.ksplit) : 0;
  const int ks = tz - phase * p.ksplit;
  const bool first_block = tile == 0;

  const PhaseInfo pq = make_phase(p, phase);
  const int Kp = AM == A_CONVT ? pq.nth * pq.ntw * p.gc : p.K;
  const int ktiles = (Kp + BK - 1) / BK;
  const int kper = (ktiles + p.ksplit - 1) / p.ksplit;
  const int kt0 = ks * kper;
  const int kt1 = min(ktiles, kt0 + kper);
  const int kend = min(Kp, kt1 * BK);

  // ---- per-thread operand rows: chunk column kc (same for every row of the thread)
  const int kc = tid % KC, r0 = tid / KC;
  const Src<__bf16> sa = make_src<__bf16>(p.a_ptr, p.a_bytes, p.a_xf);
  const rsrc_t rb = make_rsrc(p.b_ptr, p.b_bytes);
  RowOperand<__bf16, AM, true> ar[APT];
  int bbase[BPT];
  bool bok[BPT];
#pragma unroll
  for (int i = 0; i < APT; ++i) ar[i].init(p, m0 + r0 + i * RPP, p.M, phase, p.a_ld);
#pragma unroll
  for (int i = 0; i < BPT; ++i) {
    const int n = n0 + r0 + i * RPP;
    bok[i] = n < p.N && r0 + i * RPP < BN;
    bbase[i] = n * p.b_ld;
  }
  const bool a_row_in_tile = r0 < BM;        // (BM < RPP: the upper threads load no A)

  struct Stage {
    uint32_t a[APT][4];
    uint32_t y[DY ? APT : 1][4];
    uint32_t b[BPT][4];
    int ch;                                  // transform channel of the chunk (zero slot if out)
    uint32_t okm;                            // A rows whose chunk is in range
  };
  auto issue = [&](int kt, Stage& st) {
    const int kk = kt * BK + 8 * kc;
    const KTap t = RowOperand<__bf16, AM, true>::tap(p, pq, p.fd_ach, p.a_xf.channels, ABN, kk, kend);
    st.ch = t.ch;
    uint32_t okm = 0u;
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      bool ok = ar[i].valid && t.kin && a_row_in_tile;
      ok = ok && (uint32_t)(ar[i].hi0 + t.r) < (uint32_t)p.gh && (uint32_t)(ar[i].wi0 + t.s) < (uint32_t)p.gw;
      okm |= (uint32_t)ok << i;
      const uint32_t off = ok ? (uint32_t)(ar[i].base + t.toff) * 2u : kOOB;
      bload<16>(sa.x, off, st.a[i]);
      if constexpr (DY) bload<16>(sa.y, off, st.y[i]);
    }
    st.okm = okm;
    // B: k-contiguous weight row; the phase gather's taps map to (r, s) of the stored kernel
    int boff = kk;
    if constexpr (AM == A_CONVT) {
      const int rr = pq.t0h - p.gs * t.r, ss = pq.t0w - p.gs * t.s;   // t.r = -th, t.s = -tw
      boff = t.kin ? (rr * p.gr + ss) * p.gc + t.ch : 0;
    }
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const uint32_t off = (bok[i] && t.kin) ? (uint32_t)(bbase[i] + boff) * 2u : kOOB;
      bload<16>(rb, off, st.b[i]);
    }
  };

  // tables: A transform [3][stride], epilogue transform [4][stride] (E_BNBWD)
  const int ca = tab_stride(p.a_xf.channels), ce = tab_stride(p.epi_xf.channels);
  const Tab ta{tabs, tabs + ca, tabs + 2 * ca, nullptr, nullptr};
  float* tq = tabs + (ABN ? 3 * ca : 0);
  const Tab te{tq, tq + ce, nullptr, tq + 2 * ce, tq + 3 * ce};

  // Prologue.  Table loads go out first and the ring's loads after them: vmcnt counts in issue
  // order, so writing the tables to LDS then waits for the table loads only, not the ring.
  // precomputed tables of up to 512 channels are copied with their loads hoisted (2 channels per
  // thread); wider ones (the Autoencoder's 1024-4096-channel layers) take tab_fill's loop below
  constexpr int TCH = 2;
  float tva[3][TCH], tve[4][TCH];
  const bool a_tab = ABN && p.a_xf.table != nullptr && p.a_xf.channels <= 256 * TCH;
  const bool e_tab = EM == E_BNBWD && p.epi_xf.kind == VAE_X_BN_ACT && p.epi_xf.table != nullptr &&
                     p.epi_xf.channels <= 256 * TCH;
  if (a_tab) {
    const int C = p.a_xf.channels;
#pragma unroll
    for (int j = 0; j < TCH; ++j) {
      const int ch = min(tid + 256 * j, C - 1);
#pragma unroll
      for (int q = 0; q < (DY ? 3 : 2); ++q) tva[q][j] = p.a_xf.table[q * C + ch];
    }
  }
  if (e_tab) {
    const int C = p.epi_xf.channels;
#pragma unroll
    for (int j = 0; j < TCH; ++j) {
      const int ch = min(tid + 256 * j, C - 1);
#pragma unroll
      for (int q = 0; q < 4; ++q) tve[q][j] = p.epi_xf.table[q * C + ch];
    }
  }
  // in-kernel BatchNorm tables: their loads go out before the ring's (vae_common.hpp TabPre)
  // (the reductions' LDS scratch is the operand-tile area, unused until the main loop)
  TabPre<DY ? 4 : 2> pa;
  TabPre<2> pe;
  const bool a_pre = ABN && !a_tab && tab_pre_ok<XA>(p.a_xf);
  const bool e_pre = EM == E_BNBWD && !e_tab && tab_pre_ok<VAE_X_BN_ACT>(p.epi_xf);
  if (a_pre) tab_pre_load(p.a_xf, pa);
  if (e_pre) tab_pre_load(p.epi_xf, pe);
  Stage ring[NS];
#pragma unroll
  for (int u = 0; u < NS; ++u) {
    // one round: only the slice's own steps (the first store then waits for all of them — they
    // were requested together); ring mode: every slot, so vmcnt stays exact across the loop
    if (!OR || kt0 + u < kt1) issue(kt0 + u, ring[u]);
  }
  // The epilogue's own loads (the stored pre-activation / residual of the output rows, the bias)
  // go out now, behind the ring: the output tile is known from the start, and issued after the
  // K loop they were one more memory round trip on every workgroup's critical path.
  constexpr int EC = BN / 8, ERS = 256 / EC;
  constexpr int EPT = (BM + ERS - 1) / ERS;
  const int ec = tid % EC, er0 = tid / EC;
  const int col = n0 + ec * 8;
  const bool col_ok = col < p.N;                     // host: N % 8 == 0
  uint32_t aux[EPT][4], res[EPT][4];
  int obase[EPT];
  bool rok[EPT];
  float bias[8];
  const bool has_res = p.residual != nullptr;
  // (the 128-row tiles keep them after the loop: 8 rows x 2 operands per thread would stay live
  // across it, 64 VGPRs under their two-workgroups-per-CU cap; so do the tiles capped at three
  // workgroups per CU, which would spill)
  constexpr bool EARLY = EPT <= 2 && cg_waves_per_eu<BM, BN, XA>() < 3;
  auto epi_loads = [&]() {
    const rsrc_t raux = epi_aux_rsrc<EM>(p);
    const rsrc_t rres = epi_res_rsrc<EM>(p);
    const bool loads = p.slab == nullptr;
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int rl = er0 + i * ERS, row = m0 + rl;
      rok[i] = rl < BM && row < p.M && col_ok;
      obase[i] = out_row_base(p, phase, rok[i] ? row : 0) + col;
      const uint32_t off = (rok[i] && loads) ? (uint32_t)obase[i] * 2u : kOOB;
      bload<16>(raux, off, aux[i]);
      if (EM == E_BNBWD && has_res) bload<16>(rres, off, res[i]);
      else res[i][0] = res[i][1] = res[i][2] = res[i][3] = 0u;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) bias[e] = 0.f;
    if (EM == E_STORE && p.bias && col_ok && loads) {
#pragma unroll
      for (int e = 0; e < 8; ++e) bias[e] = p.bias[col + e];     // (parameter slices are 4-B aligned only)
    }
  };
  if constexpr (EARLY) epi_loads();
  if (a_tab) {
    const int C = p.a_xf.channels;
#pragma unroll
    for (int j = 0; j < TCH; ++j) {
      const int ch = tid + 256 * j;
      if (ch < C) {
        ta.a[ch] = tva[0][j]; ta.b[ch] = tva[1][j];
        if (DY) ta.c[ch] = tva[2][j];
      }
    }
  } else if constexpr (ABN) {
    tab_fill_pre(p.a_xf, pa, a_pre, ta, false, first_block, reinterpret_cast<float*>(smem));
  }
  if constexpr (ABN) {
    if (tid < 8) { const int z = tab_pad(p.a_xf.channels) + tid; ta.a[z] = 0.f; ta.b[z] = 0.f; ta.c[z] = 0.f; }
  }
  if (e_tab) {
    const int C = p.epi_xf.channels;
#pragma unroll
    for (int j = 0; j < TCH; ++j) {
      const int ch = tid + 256 * j;
      if (ch < C) { te.a[ch] = tve[0][j]; te.b[ch] = tve[1][j]; te.p[ch] = tve[2][j]; te.q[ch] = tve[3][j]; }
    }
  } else if constexpr (EM == E_BNBWD) {
    tab_fill_pre(p.epi_xf, pe, e_pre, te, true, false, reinterpret_cast<float*>(smem));
  }
  __syncthreads();
  PROBE_MARK(1);                                     // probe: operands of the first steps + tables in

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto store = [&](int buf, const Stage& st) {
    __bf16* ad = As + buf * BM * LDK + r0 * LDK + kc * 8;
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      if (r0 + i * RPP < BM) {
        uint4 v;
        if constexpr (XA == VAE_X_NONE) {
          v = uint4{st.a[i][0], st.a[i][1], st.a[i][2], st.a[i][3]};
        } else {
          // an out-of-range chunk (padding, tile edge, k >= K) must be 0 AFTER the transform:
          // its channel is the zero slot (all coefficients 0) or, for LeakyReLU, lrelu(0) = 0
          const int ch = ((st.okm >> i) & 1u) ? st.ch : sa.zs;
          v = cg_xform<XA>(st.a[i], st.y[DY ? i : 0], ta, ch, sa.slope);
        }
        *reinterpret_cast<uint4*>(ad + i * RPP * LDK) = v;
      }
    }
    __bf16* bd = Bs + buf * BN * LDK + r0 * LDK + kc * 8;
#pragma unroll
    for (int i = 0; i < BPT; ++i)
      if (r0 + i * RPP < BN) *reinterpret_cast<uint4*>(bd + i * RPP * LDK) = uint4{st.b[i][0], st.b[i][1], st.b[i][2], st.b[i][3]};
  };
  auto compute = [&](int buf) {
    const __bf16* a = As + buf * BM * LDK + (wm * WTM + (lane & 15)) * LDK + 8 * (lane >> 4);
    const __bf16* b = Bs + buf * BN * LDK + (wn * WTN + (lane & 15)) * LDK + 8 * (lane >> 4);
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(a + i * 16 * LDK + 32 * kk);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(b + j * 16 * LDK + 32 * kk);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  // main loop: step kt goes ring slot -> LDS buffer (kt-kt0)&1, then the slot is refilled with
  // step kt+NS (loads past the K range read zeros through the buffer resource)
  // (loads are issued on every path, so the compiler's vmcnt bookkeeping stays exact across
  // the loop back-edge; only the LDS work of steps past the slice's end is skipped)
  if constexpr (OR != 0) {
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      if (kt0 + u < kt1) {
        if (NBUF == 1 && u > 0) __syncthreads();        // the previous step's reads of the buffer
        store(u & (NBUF - 1), ring[u]);
        __syncthreads();
        compute(u & (NBUF - 1));
      }
    }
  } else {
    int buf = 0;
    for (int kb = kt0; kb < kt1; kb += NS) {
#pragma unroll
      for (int u = 0; u < NS; ++u) {
        const bool live = kb + u < kt1;
        if (live) store(buf, ring[u]);
        __syncthreads();
        issue(kb + u + NS, ring[u]);
        if (live) compute(buf);
        buf ^= 1;
      }
    }
  }
  // probe marks: 1 = prologue done (tables built, first loads landed), 2 = K loop done, 3 = end
  PROBE_MARK(2);
#ifdef VAE_PROBE
  struct ProbeEnd {
    unsigned long long* pr; unsigned long long* clk; unsigned long long w0;
    __device__ ~ProbeEnd() { PROBE_MARK(3); probe_write(pr, clk, w0); }
  } probe_end{p.probe, clk, wall0};
#endif

  // ------------------------------------------------------------------ epilogue through LDS
  // E_STORE statistics straight from the accumulators (rows outside M accumulated zeros): lane
  // holds rows 4g..4g+3 of column l&15 of each fragment -> 2 butterfly steps per column fragment
  __shared__ float fpart[CgWaves<BM, BN>::WM][2][BN];
  const bool frag_sums = EM == E_STORE && p.sum != nullptr && p.slab == nullptr;
  if (frag_sums) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float a1 = 0.f, a2 = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) { a1 += acc[i][j][e]; a2 = fmaf(acc[i][j][e], acc[i][j][e], a2); }
      a1 += __shfl_xor(a1, 16); a2 += __shfl_xor(a2, 16);
      a1 += __shfl_xor(a1, 32); a2 += __shfl_xor(a2, 32);
      if (lane < 16) { fpart[wm][0][wn * WTN + j * 16 + lane] = a1; fpart[wm][1][wn * WTN + j * 16 + lane] = a2; }
    }
  }
  __syncthreads();                                   // every wave is done with the K tiles
  float* Cs = reinterpret_cast<float*>(smem);        // [BM][BN+4]
  constexpr int LDC = BN + 4;
  {
    const int rq = wm * WTM + 4 * (lane >> 4), cq = wn * WTN + (lane & 15);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) Cs[(rq + i * 16 + e) * LDC + cq + j * 16] = acc[i][j][e];
  }
  __syncthreads();
  // thread -> 8 consecutive columns of rows er0, er0 + ERS, ... (loads issued in the prologue)
  if (p.slab) {
    float* sl = p.slab + ((long)(phase * p.ksplit + ks) * p.M) * p.N;
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int rl = er0 + i * ERS, row = m0 + rl;
      if (rl < BM && row < p.M && col_ok) {
        const f32x4 v0 = *reinterpret_cast<const f32x4*>(Cs + rl * LDC + ec * 8);
        const f32x4 v1 = *reinterpret_cast<const f32x4*>(Cs + rl * LDC + ec * 8 + 4);
        *reinterpret_cast<f32x4*>(sl + (long)row * p.N + col) = v0;
        *reinterpret_cast<f32x4*>(sl + (long)row * p.N + col + 4) = v1;
      }
    }
    return;
  }
  if constexpr (!EARLY) epi_loads();
  // apply (outputs stay in registers), per-column sums -> this block's flush, then the
  // stores: nothing waits on the stores (a barrier behind them would drain them: vmcnt(0))
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
  int ech = 0;
  if constexpr (EM == E_BNBWD) ech = (int)(col - p.fd_ech.div(col) * p.epi_xf.channels);
  uint4 pk[EPT];
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    const int rl = min(er0 + i * ERS, BM - 1);
    float v[8], ax[8], rs[8];
    {
      const f32x4 v0 = *reinterpret_cast<const f32x4*>(Cs + rl * LDC + ec * 8);
      const f32x4 v1 = *reinterpret_cast<const f32x4*>(Cs + rl * LDC + ec * 8 + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[e] = v0[e]; v[e + 4] = v1[e]; }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      ax[2 * e] = __uint_as_float(aux[i][e] << 16);
      ax[2 * e + 1] = __uint_as_float(aux[i][e] & 0xffff0000u);
      rs[2 * e] = __uint_as_float(res[i][e] << 16);
      rs[2 * e + 1] = __uint_as_float(res[i][e] & 0xffff0000u);
    }
    const float w = rok[i] ? 1.f : 0.f;           // rows / columns outside the output add nothing
    float o[8];
    if constexpr (EM == E_STORE) {
      const bool ract = p.res_xf.kind == VAE_X_ACT;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float y = v[e] + bias[e];
        if (has_res) y += ract ? lrelu(ax[e], p.res_xf.slope) : ax[e];
        o[e] = y;                                  // (statistics: fpart, from the accumulators)
      }
    } else {
      const int ek = p.epi_xf.kind;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float g0 = v[e] + rs[e];
        float g = g0;
        if (ek == VAE_X_BN_ACT) {
          const float z = fmaf(ax[e], te.a[ech + e], te.b[ech + e]);
          g = z > 0.f ? g0 : g0 * p.epi_xf.slope;
          s1[e] = fmaf(w, g, s1[e]);
          s2[e] = fmaf(w * g, fmaf(ax[e], te.p[ech + e], te.q[ech + e]), s2[e]);
        } else if (ek == VAE_X_ACT) {
          g = ax[e] > 0.f ? g0 : g0 * p.epi_xf.slope;
        }
        o[e] = g;
      }
    }
    uint32_t* pp = reinterpret_cast<uint32_t*>(&pk[i]);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      bf16x2 h;
      h[0] = (__bf16)o[2 * e];
      h[1] = (__bf16)o[2 * e + 1];
      pp[e] = *reinterpret_cast<uint32_t*>(&h);
    }
  }
  if (frag_sums) {
    for (int c = tid; c < BN; c += 256) {
      if (n0 + c < p.N) {
        float t1 = 0.f, t2 = 0.f;
#pragma unroll
        for (int w = 0; w < CgWaves<BM, BN>::WM; ++w) { t1 += fpart[w][0][c]; t2 += fpart[w][1][c]; }
        epi_flush_sums<EM>(p, bid, n0 + c, t1, t2);
      }
    }
  } else if (EM == E_BNBWD && epi_wants_sums<EM>(p)) {
    // lanes l, l+EC, l+2EC, ... of a wave hold the same 8 columns: butterfly over the lane
    // bits above EC, then one partial per wave and column in LDS (no atomics), summed in wave order
    float* part = Cs;                                // [4 waves][2][BN] (Cs was read above)
#pragma unroll
    for (int m = EC; m < 64; m <<= 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s1[e] += __shfl_xor(s1[e], m);
        s2[e] += __shfl_xor(s2[e], m);
      }
    }
    __syncthreads();                                 // every wave is done reading Cs
    if (lane < EC) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        part[(wave * 2) * BN + ec * 8 + e] = s1[e];
        part[(wave * 2 + 1) * BN + ec * 8 + e] = s2[e];
      }
    }
    __syncthreads();
    for (int c = tid; c < BN; c += 256) {
      if (n0 + c < p.N) {
        const float t1 = (part[0 * BN + c] + part[2 * BN + c]) + (part[4 * BN + c] + part[6 * BN + c]);
        const float t2 = (part[1 * BN + c] + part[3 * BN + c]) + (part[5 * BN + c] + part[7 * BN + c]);
        epi_flush_sums<EM>(p, bid, n0 + c, t1, t2);
      }
    }
  }
  __bf16* out = static_cast<__bf16*>(p.out);
#pragma unroll
  for (int i = 0; i < EPT; ++i)
    if (rok[i]) *reinterpret_cast<uint4*>(out + obase[i]) = pk[i];
}

template <int BM, int BN, int BK, int OR> constexpr int cg_nbuf() { return OR == 2 ? 1 : 2; }

template <int BM, int BN, int BK, int AM, int XA, int EM, int OR>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(cg_waves_per_eu<BM, BN, XA>())))
cgemm_kernel(const GemmParams p) {
  kernarg_prefetch<sizeof(GemmParams)>();
  __shared__ __attribute__((aligned(16))) char smem[CgSmem<BM, BN, BK, cg_nbuf<BM, BN, BK, OR>()>::BYTES];
  cgemm_body<BM, BN, BK, AM, XA, EM, OR>(p, (int)blockIdx.x, smem);
}

}  // namespace vae
