// Generic implicit-GEMM kernel on MFMA for every convolution-family op of the VAE step.
//
//   C[m][n] = Σ_k A(m,k) · B(n,k)
//
// A and B are "operands": views of NHWC tensors / weight matrices with a per-channel
// transform (BatchNorm+LeakyReLU forward, or BatchNorm backward) applied on load.  Tiles are
// staged global -> registers -> LDS (double-buffered, one barrier per K-tile; the next tile's
// global loads are in flight during the current tile's MFMAs) as [rows][BK] (k contiguous,
// padded), and read as MFMA fragments: lane l owns row (l&15) and 8 consecutive k of group
// (l>>4).  fp32 (BK=32) runs v_mfma_f32_16x16x4_f32 eight times over those 8 k (k permuted
// inside the tile — the sum is order-free); bf16 (BK=64) runs v_mfma_f32_16x16x32_bf16 twice.
//
// Operand modes (vector direction V_K = 8 contiguous k per load, V_M = 4 contiguous rows):
//   A_CONV   im2col gather of a strided conv (NHWC dtype, or the NCHW fp32 image)    V_K
//   A_CONVT  sub-pixel phase gather of a transposed conv / conv dgrad (blockIdx.z)  V_K
//   A_DENSE  row-major [M][K]                                                      V_K
//   A_KM     k-major [K][M] (weight-gradient GEMMs reduce over pixels/batch)      V_M
//   B_NK     weights [N][K]                                                        V_K
//   B_KN     weights [K'][N] addressed through the phase tap tables (or dense)     V_M
//   B_GATHER conv gather with n = (r,s,c), k = pixel (weight gradient)             V_M
// Per-thread row state (pixel coordinates, base offsets) is computed once before the K loop;
// index decompositions inside it use magic-number division (FastDiv).
//
// Epilogues: E_STORE (bias, residual, per-channel Σ/Σ² for the next BatchNorm),
//            E_BNBWD (g = da·act'(z) of the producing layer, Σg -> dβ, Σg·x̂ -> dγ),
//            E_ACC   (split-K fp32 atomic accumulation of weight gradients),
//            E_REPARAM (dz -> d[mu|logvar] incl. the analytic KL gradient).
// Split-K for the non-accumulating epilogues: each K-slice writes an fp32 slab and
// igemm_finalize sums the slabs in a fixed order (deterministic) and runs the epilogue.
#pragma once
#include "vae_common.hpp"

namespace vae {

enum AMode { A_CONV = 0, A_CONVT = 1, A_DENSE = 2, A_KM = 3 };
enum BMode { B_NK = 0, B_KN = 1, B_GATHER = 2 };
enum EMode { E_STORE = 0, E_BNBWD = 1, E_ACC = 2, E_REPARAM = 3 };

// max channels of a per-channel transform table (the Autoencoder's widest BatchNorm: 4096,
// configs/patient_vvbig_ae.yaml); the tables live in dynamic LDS sized by the real channel count,
// and a launch whose tables would not fit the LDS budget falls back or fails (lds_fits)
constexpr int MAXC = 4096;
constexpr int NTHREADS = 256;

template <class T> constexpr int bk_of() { return sizeof(T) == 2 ? 64 : 32; }

// Magic-number division for 0 <= n < 2^31, branch-free ("add" method):
//   q = (umulhi(n, mul) + n) >> shr,  shr = ceil(log2 d),  mul = floor(2^32 (2^shr - d) / d) + 1
// (d = 1: mul = 0, shr = 0).  umulhi(n, mul) < n, so the sum stays below 2^32.
struct FastDiv {
  uint32_t d, mul, shr;
  __device__ __forceinline__ uint32_t div(uint32_t n) const { return (__umulhi(n, mul) + n) >> shr; }
};

inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d < 1 ? 1 : d;
  uint32_t l = 0;
  while ((1ull << l) < f.d) ++l;
  f.shr = l;
  f.mul = (uint32_t)(((1ull << 32) * ((1ull << l) - f.d)) / f.d + 1);
  if (f.d == 1) f.mul = 0;
  return f;
}

struct GemmParams {
  int M, N, K;               // K unused for A_CONVT (per-phase K from the tap tables)
  int ksplit, nphase;
  // ---- A operand
  const void* a_ptr; int a_ld; vae_xform a_xf;
  // ---- B operand
  const void* b_ptr; int b_ld; vae_xform b_xf;
  int ones_col;              // B_KN/B_GATHER: column index that reads 1.0 (bias grad) or -1
  int b_taps;                // B_KN: rows addressed through the phase tap tables (else dense)
  int g_nchw;                // A_CONV / B_GATHER: gathered tensor is the fp32 NCHW image
  // ---- conv geometry of the gathered tensor
  //   A_CONV/B_GATHER: tensor [gn][gh][gw][gc], output grid gp x gq, kernel gr, stride gs, pad gpad
  //   A_CONVT: input tensor [gn][gh][gw][gc] -> output gho x gwo, phase grid gp x gq
  int gn, gh, gw, gc, gp, gq, gr, gs, gpad, gho, gwo;
  int ntap_h[2], ntap_w[2], tap0[2];   // phase ph: taps r = tap0[ph] + gs*t, t < ntap
  int tap_d[2];                        // phase ph: input offset of tap 0, (ph + gpad - tap0[ph]) / gs
  FastDiv fd_gq, fd_gp, fd_gc, fd_gr, fd_ntw[2];
  // ---- epilogue
  void* out; int out_ld; int out_phase;      // out_phase: rows are phase-grid pixels
  int out_f32;               // E_STORE: write fp32 instead of T
  const float* bias; float* sum; float* sumsq;
  const void* residual; vae_xform res_xf;
  vae_xform epi_xf; float* dgamma; float* dbeta;
  float* bias_grad;
  float* dbc; int dbc_from_b;  // closed-form BN-followed bias gradient (wgrad, first block)
  int sum_reps, sum_rstride; // replicas of the per-channel sums the epilogue accumulates
  const float* mulv; const float* eps; const float* kl_coef; float* dmulv; int samples, latent;
  float* slab;               // split-K partials [nphase][ksplit][M][N] (non-ACC epilogues)
  // ---- operand access (host-derived, see vae_launch.hpp)
  uint32_t a_bytes, b_bytes; // buffer-resource extents of the A / B tensors (and their aux)
  FastDiv fd_ach, fd_bch;    // transform channel counts of A / B
  FastDiv fd_ech;            // epilogue transform channel count
  uint32_t out_aux_bytes;    // extent of the out-shaped aux tensor (residual / stored pre-activation)
  unsigned long long* probe; // VAE_PROBE builds: per-block phase timestamps (diagnostics only)
  int m_fast;                // cgemm tile order: m fastest (an XCD's range spans few n columns:
                             // weight-heavy layers) instead of n fastest (host: vae_launch.hpp)
  // deterministic calls (vaehip.h vae_conv_args.deterministic): E_ACC runs on the slab path, and
  // the per-channel sums / reparameterization terms go to det_slab rows (one per contributing
  // block or row) that ordered_sum_launch adds in a fixed order
  int det;
  float* det_slab;
  int det_rows;              // rows of per-channel sums in det_slab
};

// Phase timestamps of one block (VAE_PROBE builds): record = {block id, wall0, wall3, clk0..clk3,
// hw id}; probe[0] is the record counter, probe[1] the capacity.
#ifdef VAE_PROBE
#define PROBE_MARK(i) do { if (threadIdx.x == 0) clk[i] = __builtin_readcyclecounter(); } while (0)
__device__ __forceinline__ void probe_write(unsigned long long* pr, const unsigned long long* clk,
                                           unsigned long long w0) {
  if (!pr || threadIdx.x != 0) return;
  // one fixed slot per block (no shared counter: its atomics would serialise the blocks)
  const unsigned long long slot = blockIdx.x + (unsigned long long)gridDim.x * (blockIdx.y + (unsigned long long)gridDim.y * blockIdx.z);
  if (slot >= pr[1]) return;                 // pr[1]: capacity in records
  unsigned long long* r = pr + 8 + slot * 8;
  r[0] = blockIdx.x | ((unsigned long long)blockIdx.y << 21) | ((unsigned long long)blockIdx.z << 42);
  r[1] = w0;
  r[2] = wall_clock64();
  r[3] = clk[0]; r[4] = clk[1]; r[5] = clk[2]; r[6] = clk[3];
  r[7] = __builtin_amdgcn_s_getreg((23 << 0) | (0 << 6) | (31 << 11));   // HW_ID
}
#else
#define PROBE_MARK(i) do { } while (0)
#endif

// Phase-specific constants of a transposed-conv problem, resolved once per block with selects
// (runtime indexing of kernarg arrays makes the compiler copy the whole struct to scratch).
struct PhaseInfo {
  int ph, pw, t0h, t0w, nth, ntw;
  int dh, dw;      // input offset of tap 0: (ph + pad - t0h) / S, (pw + pad - t0w) / S
  FastDiv fdw;
};

__device__ __forceinline__ PhaseInfo make_phase(const GemmParams& p, int phase) {
  PhaseInfo q;
  q.ph = phase >= p.gs ? 1 : 0;
  q.pw = phase - q.ph * p.gs;
  q.t0h = q.ph ? p.tap0[1] : p.tap0[0];
  q.t0w = q.pw ? p.tap0[1] : p.tap0[0];
  q.nth = q.ph ? p.ntap_h[1] : p.ntap_h[0];
  q.ntw = q.pw ? p.ntap_w[1] : p.ntap_w[0];
  q.fdw = q.pw ? p.fd_ntw[1] : p.fd_ntw[0];
  q.dh = q.ph ? p.tap_d[1] : p.tap_d[0];
  q.dw = q.pw ? p.tap_d[1] : p.tap_d[0];
  return q;
}

// ------------------------------------------------------------------ per-channel tables
// Fill a transform table (vae_common.hpp Tab): a copy of vae_bn_finalize's precomputed table, or
// built by this workgroup from the producer's replicated statistics (tab_build).
// scr: 1024 floats of LDS scratch for the replica reduction, free for the duration of the call.
__device__ __forceinline__ void tab_fill(const vae_xform& x, Tab t, bool epi, bool update_running, float* scr) {
  if (x.kind != VAE_X_BN_ACT && x.kind != VAE_X_BN_DY) return;
  if (threadIdx.x < 8) {
    const int z = tab_pad(x.channels) + threadIdx.x;
    t.a[z] = 0.f; t.b[z] = 0.f;
    if (x.kind == VAE_X_BN_DY) t.c[z] = 0.f;
  }
  if (x.table) {
    // precomputed by vae_bn_finalize: one coalesced copy, four channels of a thread per round of
    // loads (the Autoencoder's 4096-channel tables: 4 rounds, not 16 dependent ones)
    const int C = x.channels;
    const bool dy = x.kind == VAE_X_BN_DY;
    const int nt = blockDim.x;
    for (int c0 = threadIdx.x; c0 < C; c0 += 4 * nt) {
      float v[4][4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int ch = c0 + u * nt, cc = ch < C ? ch : C - 1;
        v[u][0] = x.table[cc];
        v[u][1] = x.table[C + cc];
        v[u][2] = (dy || epi) ? x.table[2 * C + cc] : 0.f;
        v[u][3] = (!dy && epi) ? x.table[3 * C + cc] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int ch = c0 + u * nt;
        if (ch >= C) break;
        t.a[ch] = v[u][0]; t.b[ch] = v[u][1];
        if (dy) t.c[ch] = v[u][2];
        else if (epi) { t.p[ch] = v[u][2]; t.q[ch] = v[u][3]; }
      }
    }
    return;
  }
  if (blockDim.x == 256 && bn_fast_ok(x)) {
    tab_build(x, t, epi, update_running, scr);
    return;
  }
  for (int ch = threadIdx.x; ch < x.channels; ch += blockDim.x) {
    float mean, invstd, var;
    bn_moments(x, ch, mean, invstd, var);
    const float g = x.gamma[ch];
    if (x.kind == VAE_X_BN_ACT) {
      const float sc = g * invstd;
      t.a[ch] = sc;
      t.b[ch] = x.beta[ch] - mean * sc;
      if (epi) { t.p[ch] = invstd; t.q[ch] = -mean * invstd; }
      if (update_running && x.running_mean) {
        const float m = x.momentum;
        const float unb = x.count > 1.f ? var * x.count / (x.count - 1.f) : var;
        x.running_mean[ch] = (1.f - m) * x.running_mean[ch] + m * mean;
        x.running_var[ch] = (1.f - m) * x.running_var[ch] + m * unb;
      }
    } else {
      const float inv_m = 1.0f / x.count;
      const float A = g * invstd;
      const float mg = rsum(x.dbeta, x, ch) * inv_m;         // mean of g
      const float mgx = rsum(x.dgamma, x, ch) * inv_m;       // mean of g*xhat
      t.a[ch] = A;
      t.b[ch] = -A * invstd * mgx;
      t.c[ch] = -A * (mg - mean * invstd * mgx);
    }
  }
}

// tab_fill for kernels without a free operand area at that point: a scratch array of its own
__device__ __forceinline__ void tab_fill(const vae_xform& x, Tab t, bool epi, bool update_running) {
  __shared__ float scr[4 * 256];
  tab_fill(x, t, epi, update_running, scr);
}

// Hoisted table build (TabPre): eligible when the table is built in-kernel on the fast path.
template <int KIND>
__device__ __forceinline__ bool tab_pre_ok(const vae_xform& x) {
  return x.kind == KIND && !x.table && blockDim.x == 256 && bn_fast_ok(x);
}
// tab_fill with the loads already issued (pre: tab_pre_load ran for x), else the plain fill
template <int NS>
__device__ __forceinline__ void tab_fill_pre(const vae_xform& x, const TabPre<NS>& q, bool pre, Tab t, bool epi,
                                             bool update_running, float* scr) {
  if (!pre) { tab_fill(x, t, epi, update_running, scr); return; }
  if (threadIdx.x < 8) {
    const int z = tab_pad(x.channels) + threadIdx.x;
    t.a[z] = 0.f; t.b[z] = 0.f;
    if (x.kind == VAE_X_BN_DY) t.c[z] = 0.f;
  }
  tab_pre_finish(x, q, t, epi, update_running, scr);
}

__host__ __device__ inline int tab_floats(const vae_xform& x, bool epi) {
  if (x.kind != VAE_X_BN_ACT && x.kind != VAE_X_BN_DY) return 0;
  return (epi ? 4 : 3) * tab_stride(x.channels);
}

// ------------------------------------------------------------------ buffer loads
// Operands are read through buffer resources: an offset at or past the resource size returns 0
// without touching memory.  Every load of a K-tile is therefore issued unconditionally (no
// branch, so no wait next to it); out-of-range elements are dropped by a validity mask when
// the tile is written to LDS.  Offsets are 32-bit bytes (host checks tensors < 2 GiB).
constexpr uint32_t kOOB = 0x80000000u;
typedef __amdgpu_buffer_rsrc_t rsrc_t;

__device__ __forceinline__ rsrc_t make_rsrc(const void* ptr, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(ptr), (short)0, (int)bytes, 0x00020000);
}

template <int NB>
__device__ __forceinline__ void bload(rsrc_t r, uint32_t off, uint32_t* d) {
  if constexpr (NB == 16) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    d[0] = v[0]; d[1] = v[1]; d[2] = v[2]; d[3] = v[3];
  } else if constexpr (NB == 8) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
    d[0] = v[0]; d[1] = v[1];
  } else if constexpr (NB == 4) {
    d[0] = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
  } else {
    d[0] = __builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0);
  }
}

// One operand as the kernel sees it: tensor (+ BN_DY aux) resources and its transform.
// The packed-vs-per-element layout is the kernel template parameter VEC (host-decided, see
// operand_vec in vae_launch.hpp): a runtime choice would put a branch between a load and the
// point its value is consumed.
template <class TIn>
struct Src {
  rsrc_t x, y;
  int kind, C;
  int zs;          // zero-slot channel index (tab_pad(C))
  float slope;
  int dy;
};

template <class TIn>
__device__ __forceinline__ Src<TIn> make_src(const void* ptr, uint32_t bytes, const vae_xform& xf) {
  Src<TIn> s;
  s.dy = xf.kind == VAE_X_BN_DY;
  s.x = make_rsrc(ptr, bytes);
  s.y = make_rsrc(s.dy ? xf.aux : ptr, s.dy ? bytes : 0u);
  s.kind = xf.kind;
  s.C = xf.channels;
  s.zs = tab_pad(xf.channels);
  s.slope = xf.slope;
  return s;
}

// ------------------------------------------------------------------ raw staging
// A group of 8 elements in flight between its global load and its LDS store.
//   V_K (row x 8 k):    element e = k offset e
//   V_M (4 rows x 2 k): element e = 4*t + j  (k offset t, row j)
// Packed layout (vec): the raw vector(s) as loaded — bf16 pairs per dword, fp32 one per
// dword.  Generic layout: element e in w[e] (bf16 in the low half).
struct Pend {
  uint32_t w[8], y[8];
  uint32_t m;       // bit e: element e is in range (else it becomes 0)
  uint32_t ones;    // bit e: element e is the bias-gradient ones column (becomes 1)
  int chb;          // transform channel of element 0 (V_K) / row 0 (V_M); generic B_GATHER: row 0
  int chb1;         // packed V_M: channel of row 0 for the second k (zero slot when out of range)
};

template <class TIn, bool VEC>
__device__ __forceinline__ float raw_elem(const uint32_t* w, int e) {
  if constexpr (sizeof(TIn) == 4) return __uint_as_float(w[e]);
  else if constexpr (VEC) return __uint_as_float((e & 1) ? (w[e >> 1] & 0xffff0000u) : (w[e >> 1] << 16));
  else return __uint_as_float(w[e] << 16);
}

template <class TIn, int NB, bool DY>
__device__ __forceinline__ void bload_pair(const Src<TIn>& s, uint32_t off, uint32_t* w, uint32_t* y) {
  bload<NB>(s.x, off, w);
  if constexpr (DY) bload<NB>(s.y, off, y);
}

// ------------------------------------------------------------------ V_K operand (row x 8 k)
// The k-decomposition of a K-tile is shared by all octets of a thread (they sit at the same k
// offset of different rows): KTap is computed once per tile, then each octet needs only its
// row's bounds check and base offset.
struct KTap {
  int r, s;        // conv modes: tap offset added to the row's (hi0, wi0)
  int toff;        // element offset of (k) relative to the row base
  int ch;          // transform channel of the octet's first element
  int kin;         // k < kend
};

template <class TIn, int MODE, bool VEC>
struct RowOperand {
  int valid;       // row in range
  int hi0, wi0;    // conv modes: input coordinate of tap (0,0) for this output row
  int base;        // element offset of (hi0, wi0, c = 0) (NHWC) / dense row offset
  int n, hb, wb;   // non-packed A_CONV (NCHW image): image, top-left input coordinate

  __device__ __forceinline__ void init(const GemmParams& p, int row, int rows, int phase, int ld) {
    valid = row < rows;
    if constexpr (MODE == A_DENSE || MODE == 100 + B_NK) {
      base = row * ld;
    } else if constexpr (MODE == A_CONV) {
      const uint32_t t = p.fd_gq.div(row), oq = row - t * p.gq;
      const uint32_t nn = p.fd_gp.div(t), op = t - nn * p.gp;
      n = nn; hb = op * p.gs - p.gpad; wb = oq * p.gs - p.gpad;
      hi0 = hb; wi0 = wb;
      base = ((n * p.gh + hi0) * p.gw + wi0) * p.gc;
    } else if constexpr (MODE == A_CONVT) {
      // phase (ph, pw) output pixel (hh*S+ph, ww*S+pw) takes input (hh + dh - th, ww + dw - tw)
      // for its taps t = 0..ntap-1, dh = (ph + pad - t0h) / S (exact by construction)
      const PhaseInfo q = make_phase(p, phase);
      const uint32_t t = p.fd_gq.div(row), ww = row - t * p.gq;
      const uint32_t nn = p.fd_gp.div(t), hh = t - nn * p.gp;
      n = nn;
      hi0 = (int)hh + q.dh; wi0 = (int)ww + q.dw;
      base = ((n * p.gh + hi0) * p.gw + wi0) * p.gc;
    }
  }

  // decomposition of the octet's first k (shared by the thread's octets)
  __device__ __forceinline__ static KTap tap(const GemmParams& p, const PhaseInfo& q, const FastDiv& fdc, int chans,
                                            bool xf_bn, int k, int kend) {
    KTap t;
    t.kin = k < kend;
    t.r = 0; t.s = 0; t.ch = 0;
    if constexpr (MODE == A_DENSE || MODE == 100 + B_NK) {
      t.toff = k;
      if (xf_bn) t.ch = (int)(k - fdc.div(k) * chans);
    } else if constexpr (MODE == A_CONV) {
      const uint32_t tp = p.fd_gc.div(k);
      const int c = k - tp * p.gc;
      const uint32_t r = p.fd_gr.div(tp);
      t.r = r; t.s = tp - r * p.gr;
      t.toff = (t.r * p.gw + t.s) * p.gc + c;
      t.ch = c;
    } else {  // A_CONVT: k = (th, tw, c)
      const uint32_t tt = p.fd_gc.div(k);
      const int c = k - tt * p.gc;
      const uint32_t th = q.fdw.div(tt);
      const int tw = tt - th * q.ntw;
      t.r = -(int)th; t.s = -tw;
      t.toff = (t.r * p.gw + t.s) * p.gc + c;
      t.ch = c;
    }
    return t;
  }

  // element offset + in-range flag of k (per-element path: NCHW image, unaligned channels)
  __device__ __forceinline__ int offset(const GemmParams& p, const PhaseInfo& q, int k, bool& ok) const {
    if constexpr (MODE == A_DENSE || MODE == 100 + B_NK) {
      ok = true;
      return base + k;
    } else if constexpr (MODE == A_CONV) {
      const int C = p.gc;
      const uint32_t tap = p.fd_gc.div(k);
      const int c = k - tap * C;
      const uint32_t r = p.fd_gr.div(tap);
      const int s = tap - r * p.gr;
      const int hi = hb + r, wi = wb + s;
      ok = hi >= 0 && hi < p.gh && wi >= 0 && wi < p.gw;
      return p.g_nchw ? ((n * C + c) * p.gh + hi) * p.gw + wi : ((n * p.gh + hi) * p.gw + wi) * C + c;
    } else {  // A_CONVT
      const int C = p.gc;
      const uint32_t tt = p.fd_gc.div(k);
      const int c = k - tt * C;
      const uint32_t th = q.fdw.div(tt);
      const int tw = tt - th * q.ntw;
      const int hi = hi0 - (int)th, wi = wi0 - tw;
      ok = hi >= 0 && hi < p.gh && wi >= 0 && wi < p.gw;
      return ((n * p.gh + hi) * p.gw + wi) * C + c;
    }
  }

  template <bool DY>
  __device__ __forceinline__ void load(const GemmParams& p, const Src<TIn>& s, const PhaseInfo& q, const FastDiv& fdc,
                                       const KTap& t, int k0, int Kp, Pend& g) const {
    constexpr int E = sizeof(TIn);
    g.ones = 0u;
    if constexpr (VEC) {
      // whole group in or out (host: K % 8 == 0); out -> zeros and the zero-slot channel
      bool ok = true;
      if constexpr (MODE == A_CONV || MODE == A_CONVT)
        ok = (uint32_t)(hi0 + t.r) < (uint32_t)p.gh && (uint32_t)(wi0 + t.s) < (uint32_t)p.gw;
      const bool gv = valid && ok && t.kin;
      g.chb = gv ? t.ch : s.zs;
      const uint32_t off = gv ? (uint32_t)(base + t.toff) * E : kOOB;
      bload_pair<TIn, 16, DY>(s, off, g.w, g.y);
      if constexpr (E == 4) bload_pair<TIn, 16, DY>(s, off + 16, g.w + 4, g.y + 4);
    } else {
      g.chb = s.kind >= VAE_X_BN_ACT ? (int)(k0 - fdc.div(k0) * s.C) : 0;
      uint32_t m = 0u;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        bool ok;
        const int idx = offset(p, q, k0 + e, ok);
        ok = ok && valid && k0 + e < Kp;
        m |= (uint32_t)ok << e;
        bload_pair<TIn, E, DY>(s, ok ? (uint32_t)idx * E : kOOB, g.w + e, g.y + e);
      }
      g.m = m;
    }
  }
};

// ------------------------------------------------------------------ V_M operand (4 rows x 2 k)
template <class TIn, int MODE, bool VEC>
struct ColOperand {
  int r0;          // first of the 4 rows (m for A_KM, n for B_KN/B_GATHER)
  uint32_t rmask;  // rows in range, ones column excluded (4 bits)
  uint32_t omask;  // the ones column (4 bits)
  int r, s, c;     // B_GATHER: tap and channel of row r0
  int ch0;         // transform channel of r0 (generic B_GATHER: r0 itself)

  __device__ __forceinline__ void init(const GemmParams& p, int row0, int rows, const vae_xform& xf) {
    r0 = row0;
    rmask = 0u; omask = 0u;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool in = row0 + j < rows;
      const bool one = MODE >= 100 && row0 + j == p.ones_col;
      rmask |= (uint32_t)(in && !one) << j;
      omask |= (uint32_t)(in && one) << j;
    }
    ch0 = xf.kind >= VAE_X_BN_ACT ? row0 % xf.channels : 0;
    if constexpr (MODE == 100 + B_GATHER) {
      const uint32_t tap = p.fd_gc.div(row0);
      c = row0 - tap * p.gc;
      const uint32_t rr = p.fd_gr.div(tap);
      r = rr; s = tap - rr * p.gr;
      ch0 = VEC ? c : row0;
    }
  }

  // element offset of (row r0 + j, k) and whether the gathered position is in range
  __device__ __forceinline__ int offset(const GemmParams& p, const PhaseInfo& q, int k, int j, bool& ok) const {
    ok = true;
    if constexpr (MODE == A_KM) {
      return k * p.a_ld + r0 + j;
    } else if constexpr (MODE == 100 + B_KN) {
      int kr = k;
      if (p.b_taps) {
        const uint32_t tt = p.fd_gc.div(k);
        const int cc = k - tt * p.gc;
        const uint32_t th = q.fdw.div(tt);
        const int tw = tt - th * q.ntw;
        kr = (cc * p.gr + (q.t0h + p.gs * (int)th)) * p.gr + (q.t0w + p.gs * (int)tw);
      }
      return kr * p.b_ld + r0 + j;
    } else {  // B_GATHER: k = pixel (n_img, op, oq) of the gp x gq grid, row = (r, s, c)
      const uint32_t tq = p.fd_gq.div(k), oq = k - tq * p.gq;
      const uint32_t nimg = p.fd_gp.div(tq), op = tq - nimg * p.gp;
      int rr = r, ss = s, cc = c;
      if constexpr (!VEC) {
        const int nn = r0 + j;
        const uint32_t tap = p.fd_gc.div(nn);
        cc = nn - tap * p.gc;
        const uint32_t ru = p.fd_gr.div(tap);
        rr = ru; ss = tap - ru * p.gr;
      }
      const int hi = op * p.gs - p.gpad + rr, wi = oq * p.gs - p.gpad + ss;
      ok = hi >= 0 && hi < p.gh && wi >= 0 && wi < p.gw;
      return p.g_nchw ? ((nimg * p.gc + cc) * p.gh + hi) * p.gw + wi : ((nimg * p.gh + hi) * p.gw + wi) * p.gc + cc;
    }
  }

  template <bool DY>
  __device__ __forceinline__ void load(const GemmParams& p, const Src<TIn>& s, const PhaseInfo& q, int k, int Kp,
                                       Pend& g) const {
    constexpr int E = sizeof(TIn);
    g.chb = ch0;
    g.ones = omask | (omask << 4);
    uint32_t m = 0u;
    if constexpr (VEC) {
      // rows beyond the operand feed output rows/columns that are never stored (host: row
      // count % 4 == 0); a k out of range or a padding position reads zeros + zero slot
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        bool ok;
        const int idx = offset(p, q, k + t, 0, ok);
        ok = ok && k + t < Kp;
        if (t == 0) g.chb = ok ? ch0 : s.zs;
        else g.chb1 = ok ? ch0 : s.zs;
        const uint32_t off = ok ? (uint32_t)idx * E : kOOB;
        if constexpr (E == 2) bload_pair<TIn, 8, DY>(s, off, g.w + 2 * t, g.y + 2 * t);
        else bload_pair<TIn, 16, DY>(s, off, g.w + 4 * t, g.y + 4 * t);
      }
    } else {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          bool ok;
          const int idx = offset(p, q, k + t, j, ok);
          ok = ok && k + t < Kp && ((rmask >> j) & 1u);
          m |= (uint32_t)ok << (4 * t + j);
          bload_pair<TIn, E, DY>(s, ok ? (uint32_t)idx * E : kOOB, g.w + 4 * t + j, g.y + 4 * t + j);
        }
    }
    g.m = m;
  }
};

// Transform of a staged group (after its loads have landed) -> 8 floats in element order.
// Masked elements become 0 after the transform (the transform of a zero pad is not zero).
template <class TIn, int MODE, bool VM, bool VEC, bool DY>
__device__ __forceinline__ void finish(const GemmParams& p, const Src<TIn>& s, const Tab& t, const Pend& g,
                                       float (&v)[8]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = raw_elem<TIn, VEC>(g.w, e);
  if (s.kind == VAE_X_BN_ACT || (DY && s.kind == VAE_X_BN_DY)) {
    const bool dy = DY && s.kind == VAE_X_BN_DY;
    float a[8], b[8], c[8];
    if constexpr (VEC) {
      // channels are consecutive: V_K chb..chb+7, V_M chb..chb+3 (16-byte aligned table reads)
      if constexpr (VM) {
        const f32x4 A = *reinterpret_cast<const f32x4*>(t.a + g.chb);
        const f32x4 B = *reinterpret_cast<const f32x4*>(t.b + g.chb);
        f32x4 Cc = f32x4{0.f, 0.f, 0.f, 0.f};
        if (dy) Cc = *reinterpret_cast<const f32x4*>(t.c + g.chb);
#pragma unroll
        for (int e = 0; e < 8; ++e) { a[e] = A[e & 3]; b[e] = B[e & 3]; c[e] = Cc[e & 3]; }
      } else {
        const f32x4 A0 = *reinterpret_cast<const f32x4*>(t.a + g.chb), A1 = *reinterpret_cast<const f32x4*>(t.a + g.chb + 4);
        const f32x4 B0 = *reinterpret_cast<const f32x4*>(t.b + g.chb), B1 = *reinterpret_cast<const f32x4*>(t.b + g.chb + 4);
        f32x4 C0 = f32x4{0.f, 0.f, 0.f, 0.f}, C1 = C0;
        if (dy) { C0 = *reinterpret_cast<const f32x4*>(t.c + g.chb); C1 = *reinterpret_cast<const f32x4*>(t.c + g.chb + 4); }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[e] = A0[e]; a[e + 4] = A1[e]; b[e] = B0[e]; b[e + 4] = B1[e]; c[e] = C0[e]; c[e + 4] = C1[e];
        }
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        int ch;
        if constexpr (VM && MODE == 100 + B_GATHER) {
          const int nn = g.chb + (e & 3);
          ch = nn - (int)p.fd_gc.div(nn) * p.gc;
        } else {
          ch = (g.chb + (VM ? (e & 3) : e)) % s.C;
        }
        a[e] = t.a[ch]; b[e] = t.b[ch]; c[e] = dy ? t.c[ch] : 0.f;
      }
    }
    if (dy) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaf(a[e], v[e], fmaf(b[e], raw_elem<TIn, VEC>(g.y, e), c[e]));
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = lrelu(fmaf(v[e], a[e], b[e]), s.slope);
    }
  } else if (s.kind == VAE_X_ACT) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = lrelu(v[e], s.slope);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    v[e] = ((g.m >> e) & 1u) ? v[e] : 0.f;
    if constexpr (VM && MODE >= 100) v[e] = ((g.ones >> e) & 1u) ? 1.f : v[e];
  }
}

// ------------------------------------------------------------------ packed (VEC) groups -> LDS
// No masks: out-of-range data is already 0 and its channel is the zero slot.  Untransformed
// groups of the LDS type are copied as raw bits.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 tab4(const float* t, int ch) { return *reinterpret_cast<const f32x4*>(t + ch); }

template <class T, class TIn, bool DY>
__device__ __forceinline__ void store_vk(const Src<TIn>& s, const Tab& t, const Pend& g, T* dst) {
  if constexpr (sizeof(T) == sizeof(TIn)) {
    if (s.kind == VAE_X_NONE) {
      reinterpret_cast<u32x4*>(dst)[0] = u32x4{g.w[0], g.w[1], g.w[2], g.w[3]};
      if constexpr (sizeof(T) == 4) reinterpret_cast<u32x4*>(dst)[1] = u32x4{g.w[4], g.w[5], g.w[6], g.w[7]};
      return;
    }
  }
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = raw_elem<TIn, true>(g.w, e);
  if (s.kind == VAE_X_ACT) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = lrelu(v[e], s.slope);
  } else if (s.kind == VAE_X_BN_ACT) {
    const f32x4 a0 = tab4(t.a, g.chb), a1 = tab4(t.a, g.chb + 4), b0 = tab4(t.b, g.chb), b1 = tab4(t.b, g.chb + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = lrelu(fmaf(v[e], a0[e], b0[e]), s.slope);
      v[e + 4] = lrelu(fmaf(v[e + 4], a1[e], b1[e]), s.slope);
    }
  } else if (DY && s.kind == VAE_X_BN_DY) {
    const f32x4 a0 = tab4(t.a, g.chb), a1 = tab4(t.a, g.chb + 4), b0 = tab4(t.b, g.chb), b1 = tab4(t.b, g.chb + 4);
    const f32x4 c0 = tab4(t.c, g.chb), c1 = tab4(t.c, g.chb + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = fmaf(a0[e], v[e], fmaf(b0[e], raw_elem<TIn, true>(g.y, e), c0[e]));
      v[e + 4] = fmaf(a1[e], v[e + 4], fmaf(b1[e], raw_elem<TIn, true>(g.y, e + 4), c1[e]));
    }
  }
  st8(dst, v);
}

// rows j = 0..3 of the group go to dst + j*ldk as the pair (k, k+1)
template <class T, class TIn, int MODE, bool DY>
__device__ __forceinline__ void store_vm(const Src<TIn>& s, const Tab& t, const Pend& g, T* dst, int ldk) {
  if constexpr (sizeof(T) == 2 && sizeof(TIn) == 2) {
    if (s.kind == VAE_X_NONE && (MODE < 100 || g.ones == 0u)) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t lo = g.w[j >> 1], hi = g.w[2 + (j >> 1)];
        *reinterpret_cast<uint32_t*>(dst + j * ldk) =
            (j & 1) ? ((lo >> 16) | (hi & 0xffff0000u)) : ((lo & 0xffffu) | (hi << 16));
      }
      return;
    }
  }
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = raw_elem<TIn, true>(g.w, e);
  if (s.kind == VAE_X_ACT) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = lrelu(v[e], s.slope);
  } else if (s.kind == VAE_X_BN_ACT) {
    const f32x4 a0 = tab4(t.a, g.chb), a1 = tab4(t.a, g.chb1), b0 = tab4(t.b, g.chb), b1 = tab4(t.b, g.chb1);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = lrelu(fmaf(v[j], a0[j], b0[j]), s.slope);
      v[4 + j] = lrelu(fmaf(v[4 + j], a1[j], b1[j]), s.slope);
    }
  } else if (DY && s.kind == VAE_X_BN_DY) {
    const f32x4 a0 = tab4(t.a, g.chb), a1 = tab4(t.a, g.chb1), b0 = tab4(t.b, g.chb), b1 = tab4(t.b, g.chb1);
    const f32x4 c0 = tab4(t.c, g.chb), c1 = tab4(t.c, g.chb1);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = fmaf(a0[j], v[j], fmaf(b0[j], raw_elem<TIn, true>(g.y, j), c0[j]));
      v[4 + j] = fmaf(a1[j], v[4 + j], fmaf(b1[j], raw_elem<TIn, true>(g.y, 4 + j), c1[j]));
    }
  }
  if constexpr (MODE >= 100) {
    if (g.ones) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = ((g.ones >> e) & 1u) ? 1.f : v[e];
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) st2(dst + j * ldk, v[j], v[4 + j]);
}

// ------------------------------------------------------------------ epilogue helpers
// Row part of the output offset of GEMM row `row` of phase `phase` (elements; the caller adds
// the column).  Output tensors are < 2^31 elements (host-checked).
__device__ __forceinline__ int out_row_base(const GemmParams& p, int phase, int row) {
  if (p.out_phase) {
    const int ph = phase >= p.gs ? 1 : 0, pw = phase - ph * p.gs;
    const uint32_t t = p.fd_gq.div(row), ww = row - t * p.gq;
    const uint32_t n = p.fd_gp.div(t), hh = t - n * p.gp;
    const int ho = hh * p.gs + ph, wo = ww * p.gs + pw;
    return ((n * p.gho + ho) * p.gwo + wo) * p.out_ld;
  }
  return row * p.out_ld;
}

// One element of an out-shaped tensor through a buffer resource (out-of-range offset -> 0).
template <class T>
__device__ __forceinline__ float ld_elem(rsrc_t r, uint32_t off_bytes) {
  if constexpr (sizeof(T) == 4) return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off_bytes, 0, 0));
  else return __uint_as_float((uint32_t)__builtin_amdgcn_raw_buffer_load_b16(r, off_bytes, 0, 0) << 16);
}

// The out-shaped tensor an epilogue reads (E_STORE: residual, E_BNBWD: the stored pre-activation);
// an empty resource when there is none.
template <int EM>
__device__ __forceinline__ rsrc_t epi_aux_rsrc(const GemmParams& p) {
  const void* ptr = nullptr;
  if constexpr (EM == E_STORE) ptr = p.residual;
  if constexpr (EM == E_BNBWD) ptr = p.epi_xf.kind != VAE_X_NONE ? p.epi_xf.aux : nullptr;
  return make_rsrc(ptr ? ptr : p.out, ptr ? p.out_aux_bytes : 0u);
}

// E_BNBWD: the gradient arriving through a residual connection, added before the activation
// backward (an empty resource when there is none).
template <int EM>
__device__ __forceinline__ rsrc_t epi_res_rsrc(const GemmParams& p) {
  const void* ptr = EM == E_BNBWD ? p.residual : nullptr;
  return make_rsrc(ptr ? ptr : p.out, ptr ? p.out_aux_bytes : 0u);
}

// Epilogue of one element whose inputs (accumulator v, aux value, bias) are already in registers.
// s1/s2 collect the per-column sums (BN statistics forward / BN-backward sums).
template <class T, int EM>
__device__ __forceinline__ void epi_apply(const GemmParams& p, const Tab& xe, int col, int idx, float v, float aux,
                                          float bias, float& s1, float& s2, float res = 0.f) {
  if constexpr (EM == E_STORE) {
    float y = v + bias;
    if (p.residual) y += p.res_xf.kind == VAE_X_ACT ? lrelu(aux, p.res_xf.slope) : aux;
    if (p.out_f32) static_cast<float*>(p.out)[idx] = y;
    else static_cast<T*>(p.out)[idx] = cvt<T>(y);
    s1 += v;
    s2 += v * v;
  } else if constexpr (EM == E_BNBWD) {
    v += res;                       // residual branch gradient (VQ-VAE ResidualLayer), 0 otherwise
    float g = v;
    if (p.epi_xf.kind == VAE_X_BN_ACT) {
      const int ch = (int)(col - p.fd_ech.div(col) * p.epi_xf.channels);
      const float z = fmaf(aux, xe.a[ch], xe.b[ch]);
      g = z > 0.f ? v : v * p.epi_xf.slope;
      s1 += g;
      s2 += g * fmaf(aux, xe.p[ch], xe.q[ch]);
    } else if (p.epi_xf.kind == VAE_X_ACT) {
      g = aux > 0.f ? v : v * p.epi_xf.slope;
    }
    static_cast<T*>(p.out)[idx] = cvt<T>(g);
  }
}

// Reparameterization backward of one element (row = z row, col = latent index):
//   dmu += dz + c*mu,  dlogvar += dz*eps*0.5*exp(0.5 lv) + c*0.5*(exp(lv) - 1)
struct ReparamIn { float mu, lv, ep, c; };
__device__ __forceinline__ ReparamIn reparam_load(const GemmParams& p, int row, int col, bool ok) {
  ReparamIn r{0.f, 0.f, 0.f, 0.f};
  if (!ok) return r;
  const int b = row / p.samples;
  r.mu = p.mulv[(long)b * 2 * p.latent + col];
  r.lv = p.mulv[(long)b * 2 * p.latent + p.latent + col];
  r.ep = p.eps[(long)row * p.latent + col];
  r.c = p.kl_coef ? p.kl_coef[row] : 0.f;
  return r;
}
__device__ __forceinline__ void reparam_apply(const GemmParams& p, int row, int col, float v, const ReparamIn& r) {
  const int b = row / p.samples;
  const float sd = expf(0.5f * r.lv);
  const float t1 = v + r.c * r.mu, t2 = v * r.ep * 0.5f * sd + r.c * 0.5f * (expf(r.lv) - 1.f);
  if (p.det_slab) {                       // row's own terms; the ordered pass sums a mu row's samples
    p.det_slab[(long)row * 2 * p.latent + col] = t1;
    p.det_slab[(long)row * 2 * p.latent + p.latent + col] = t2;
    return;
  }
  atomicAdd(p.dmulv + (long)b * 2 * p.latent + col, t1);
  atomicAdd(p.dmulv + (long)b * 2 * p.latent + p.latent + col, t2);
}

template <int EM>
__device__ __forceinline__ bool epi_wants_sums(const GemmParams& p) {
  if constexpr (EM == E_STORE) return p.sum != nullptr;
  if constexpr (EM == E_BNBWD) return p.epi_xf.kind == VAE_X_BN_ACT;
  return false;
}

template <int EM>
__device__ __forceinline__ void epi_flush_sums(const GemmParams& p, int rep, int col, float s1, float s2) {
  const long roff = p.sum_reps > 1 ? (long)(rep % p.sum_reps) * p.sum_rstride : 0;
  float* g1 = ((EM == E_STORE) ? p.sum : p.dbeta) + roff;
  float* g2 = ((EM == E_STORE) ? p.sumsq : p.dgamma) + roff;
  if (p.det_slab) {                       // contributor rep's own row [2][N]; ordered pass folds columns
    p.det_slab[(long)rep * 2 * p.N + col] = s1;
    p.det_slab[(long)rep * 2 * p.N + p.N + col] = s2;
    return;
  }
  const int ch = (EM == E_STORE) ? col : (int)(col - p.fd_ech.div(col) * p.epi_xf.channels);
  atomicAdd(g1 + ch, s1);
  atomicAdd(g2 + ch, s2);
}

// Closed-form bias gradient of a conv followed by train-mode BatchNorm:
//   db = Σ dy = A·Σg + B·Σy + C·M per channel (A,B,C the BN-backward coefficients);
// also publishes the reduced BatchNorm affine gradients (dgamma_out / dbeta_out) when asked.
__device__ __forceinline__ void closed_form_db(const vae_xform& x, float* db) {
  for (int ch = threadIdx.x; ch < x.channels; ch += blockDim.x) {
    float mean, invstd, var;
    bn_moments(x, ch, mean, invstd, var);
    const float inv_m = 1.0f / x.count;
    const float dgam = rsum(x.dgamma, x, ch), dbet = rsum(x.dbeta, x, ch);
    if (x.dgamma_out) x.dgamma_out[ch] += dgam;
    if (x.dbeta_out) x.dbeta_out[ch] += dbet;
    if (!db) continue;
    const float A = x.gamma[ch] * invstd;
    const float mgx = dgam * inv_m;
    const float mg = dbet * inv_m;
    const float B = -A * invstd * mgx;
    const float C = -A * (mg - mean * invstd * mgx);
    const float sum_y = rsum(x.sum, x, ch) + x.count * (x.shift ? x.shift[ch] : 0.f);
    db[ch] += A * dbet + B * sum_y + C * x.count;
  }
}

template <int AM> constexpr bool a_is_vm() { return AM == A_KM; }
template <int BMD> constexpr bool b_is_vm() { return BMD != B_NK; }

// dynamic LDS: per-channel tables of the A, B and epilogue transforms (floats)
__host__ __device__ inline int table_floats(const GemmParams& p, bool epi_tbl) {
  return tab_floats(p.a_xf, false) + tab_floats(p.b_xf, false) + (epi_tbl ? tab_floats(p.epi_xf, true) : 0);
}

// Wave grid of a BM x BN block of 4 waves: thin N -> 4x1, thin M -> 1x4, else 2x2.
template <int BM, int BN> struct WaveGrid {
  static constexpr int WN = (BM <= 32 && BN <= 32) ? 2 : (BN <= 32 ? 1 : (BM <= 32 ? 4 : 2));
  static constexpr int WM = 4 / WN;
  static constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  static_assert(TM >= 1 && TN >= 1, "wave tile below 16x16");
};

// Register stages of the K-loop prefetch ring: enough K-tiles in flight to cover the memory
// latency, bounded by the staging registers one stage costs.
template <int PER> constexpr int ring_stages() { return PER <= 2 ? 4 : (PER <= 4 ? 3 : 2); }

// ------------------------------------------------------------------------------ kernel
// T: LDS/MFMA type; TA: storage type of the A tensor (fp32 for the NCHW image / d[mu|logvar]);
// TB: storage type of B (the gathered activation for B_GATHER, weights otherwise).
// DYA / DYB: the A / B operand may carry a BN_DY transform (its aux tensor is loaded).
template <class T, class TA, class TB, int BM, int BN, int AM, int BMD, int EM, bool VA, bool VB, bool DYA, bool DYB>
__global__ void __launch_bounds__(NTHREADS) igemm_kernel(const GemmParams p) {
  kernarg_prefetch<(sizeof(GemmParams) < 1024 ? sizeof(GemmParams) : 1024)>();
  constexpr int BK = bk_of<T>();
  constexpr int LDK = BK + (sizeof(T) == 4 ? 4 : 8);        // padded LDS row (elements)
  using WG = WaveGrid<BM, BN>;
  constexpr int TM = WG::TM, TN = WG::TN;
  constexpr int WTM = TM * 16, WTN = TN * 16;
  constexpr bool A_VM = a_is_vm<AM>();
  constexpr bool B_VM = b_is_vm<BMD>();
  constexpr int KO = BK / 8;                                // V_K octets per row
  constexpr int A_OCT = BM * BK / 8, B_OCT = BN * BK / 8;   // octets per tile
  constexpr int A_PER = (A_OCT + NTHREADS - 1) / NTHREADS, B_PER = (B_OCT + NTHREADS - 1) / NTHREADS;
  constexpr int NS = ring_stages<A_PER + B_PER>();
  constexpr bool EPI_TBL = (EM == E_BNBWD);
  constexpr int A_MODE = AM;
  constexpr int B_MODE = 100 + BMD;

  __shared__ __attribute__((aligned(16))) T As[2][BM * LDK];
  __shared__ __attribute__((aligned(16))) T Bs[2][BN * LDK];
  __shared__ float red1[WG::WM][BN], red2[WG::WM][BN];   // per-column sums, one row per wave row
  extern __shared__ float tabs[];

#ifdef VAE_PROBE
  unsigned long long clk[4] = {0, 0, 0, 0};
  const unsigned long long wall0 = threadIdx.x == 0 ? wall_clock64() : 0;
#endif
  PROBE_MARK(0);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WG::WN, wn = wave % WG::WN;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int phase = (p.nphase > 1) ? (int)(blockIdx.z / p.ksplit) : 0;
  const int ks = blockIdx.z - phase * p.ksplit;
  const bool first_block = blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0;

  int Kp = p.K;
  if constexpr (AM == A_CONVT) {
    const PhaseInfo q = make_phase(p, phase);
    Kp = q.nth * q.ntw * p.gc;
  }
  const int ktiles = (Kp + BK - 1) / BK;
  const int kper = (ktiles + p.ksplit - 1) / p.ksplit;
  const int kt0 = ks * kper;
  const int kt1 = min(ktiles, kt0 + kper);
  const int kend = min(Kp, kt1 * BK);     // loads past this K (ring overrun, other slices) read 0

  // table views (carved in the order A, B, epilogue)
  Tab ta, tb, te;
  {
    float* q = tabs;
    const int ca = tab_stride(p.a_xf.channels), cb = tab_stride(p.b_xf.channels), ce = tab_stride(p.epi_xf.channels);
    const bool ha = tab_floats(p.a_xf, false) > 0, hb = tab_floats(p.b_xf, false) > 0;
    ta = Tab{q, q + ca, q + 2 * ca, nullptr, nullptr};
    if (ha) q += 3 * ca;
    tb = Tab{q, q + cb, q + 2 * cb, nullptr, nullptr};
    if (hb) q += 3 * cb;
    te = Tab{q, q + ce, nullptr, q + 2 * ce, q + 3 * ce};
  }

  // ---- operand sources and per-thread row state (computed once)
  const Src<TA> sa = make_src<TA>(p.a_ptr, p.a_bytes, p.a_xf);
  const Src<TB> sb = make_src<TB>(p.b_ptr, p.b_bytes, p.b_xf);
  const PhaseInfo pq = make_phase(p, phase);
  RowOperand<TA, A_MODE, VA> ars[A_VM ? 1 : A_PER];
  ColOperand<TA, A_MODE, VA> acs[A_VM ? A_PER : 1];
  RowOperand<TB, B_MODE, VB> brs[B_VM ? 1 : B_PER];
  ColOperand<TB, B_MODE, VB> bcs[B_VM ? B_PER : 1];
#pragma unroll
  for (int i = 0; i < A_PER; ++i) {
    const int o = tid + i * NTHREADS;
    if constexpr (!A_VM) ars[i].init(p, m0 + o / KO, p.M, phase, p.a_ld);
    else acs[i].init(p, m0 + (o % (BM / 4)) * 4, p.M, p.a_xf);
  }
#pragma unroll
  for (int i = 0; i < B_PER; ++i) {
    const int o = tid + i * NTHREADS;
    if constexpr (!B_VM) brs[i].init(p, n0 + o / KO, p.N, phase, p.b_ld);
    else bcs[i].init(p, n0 + (o % (BN / 4)) * 4, p.N, p.b_xf);
  }

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // K-tile loads of one ring slot: issued unconditionally (past kend they read zeros)
  const bool a_bn = p.a_xf.kind >= VAE_X_BN_ACT, b_bn = p.b_xf.kind >= VAE_X_BN_ACT;
  auto load_tiles = [&](int kt, Pend (&qa)[A_PER], Pend (&qb)[B_PER]) {
    const int kb = kt * BK;
    const int kv = kb + (tid % KO) * 8;      // V_K operands: this thread's k (same for all its octets)
    KTap tpa, tpb;
    if constexpr (!A_VM && VA) tpa = RowOperand<TA, A_MODE, VA>::tap(p, pq, p.fd_ach, p.a_xf.channels, a_bn, kv, kend);
    if constexpr (!B_VM && VB) tpb = RowOperand<TB, B_MODE, VB>::tap(p, pq, p.fd_bch, p.b_xf.channels, b_bn, kv, kend);
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int o = tid + i * NTHREADS;
      if (A_OCT % NTHREADS == 0 || o < A_OCT) {
        if constexpr (!A_VM) ars[i].template load<DYA>(p, sa, pq, p.fd_ach, tpa, kv, kend, qa[i]);
        else acs[i].template load<DYA>(p, sa, pq, kb + 2 * (o / (BM / 4)), kend, qa[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int o = tid + i * NTHREADS;
      if (B_OCT % NTHREADS == 0 || o < B_OCT) {
        if constexpr (!B_VM) brs[i].template load<DYB>(p, sb, pq, p.fd_bch, tpb, kv, kend, qb[i]);
        else bcs[i].template load<DYB>(p, sb, pq, kb + 2 * (o / (BN / 4)), kend, qb[i]);
      }
    }
  };
  auto store_tiles = [&](int buf, const Pend (&qa)[A_PER], const Pend (&qb)[B_PER]) {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int o = tid + i * NTHREADS;
      if (A_OCT % NTHREADS == 0 || o < A_OCT) {
        if constexpr (VA) {
          if constexpr (!A_VM) store_vk<T, TA, DYA>(sa, ta, qa[i], As[buf] + (o / KO) * LDK + (o % KO) * 8);
          else store_vm<T, TA, A_MODE, DYA>(sa, ta, qa[i], As[buf] + (o % (BM / 4)) * 4 * LDK + 2 * (o / (BM / 4)), LDK);
          continue;
        }
        float v[8];
        finish<TA, A_MODE, A_VM, VA, DYA>(p, sa, ta, qa[i], v);
        if constexpr (!A_VM) {
          st8(As[buf] + (o / KO) * LDK + (o % KO) * 8, v);
        } else {
          const int rq = o % (BM / 4), kp = o / (BM / 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) st2(As[buf] + (rq * 4 + j) * LDK + 2 * kp, v[j], v[4 + j]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int o = tid + i * NTHREADS;
      if (B_OCT % NTHREADS == 0 || o < B_OCT) {
        if constexpr (VB) {
          if constexpr (!B_VM) store_vk<T, TB, DYB>(sb, tb, qb[i], Bs[buf] + (o / KO) * LDK + (o % KO) * 8);
          else store_vm<T, TB, B_MODE, DYB>(sb, tb, qb[i], Bs[buf] + (o % (BN / 4)) * 4 * LDK + 2 * (o / (BN / 4)), LDK);
          continue;
        }
        float v[8];
        finish<TB, B_MODE, B_VM, VB, DYB>(p, sb, tb, qb[i], v);
        if constexpr (!B_VM) {
          st8(Bs[buf] + (o / KO) * LDK + (o % KO) * 8, v);
        } else {
          const int rq = o % (BN / 4), kp = o / (BN / 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) st2(Bs[buf] + (rq * 4 + j) * LDK + 2 * kp, v[j], v[4 + j]);
        }
      }
    }
  };
  auto compute = [&](int buf) {
    const int koff = 8 * (lane >> 4);
    if constexpr (sizeof(T) == 4) {
      float af[TM][8], bfr[TN][8];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const float* src = reinterpret_cast<const float*>(As[buf]) + (wm * WTM + i * 16 + (lane & 15)) * LDK + koff;
        f32x4 x0 = *reinterpret_cast<const f32x4*>(src), x1 = *reinterpret_cast<const f32x4*>(src + 4);
        af[i][0] = x0[0]; af[i][1] = x0[1]; af[i][2] = x0[2]; af[i][3] = x0[3];
        af[i][4] = x1[0]; af[i][5] = x1[1]; af[i][6] = x1[2]; af[i][7] = x1[3];
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const float* src = reinterpret_cast<const float*>(Bs[buf]) + (wn * WTN + j * 16 + (lane & 15)) * LDK + koff;
        f32x4 x0 = *reinterpret_cast<const f32x4*>(src), x1 = *reinterpret_cast<const f32x4*>(src + 4);
        bfr[j][0] = x0[0]; bfr[j][1] = x0[1]; bfr[j][2] = x0[2]; bfr[j][3] = x0[3];
        bfr[j][4] = x1[0]; bfr[j][5] = x1[1]; bfr[j][6] = x1[2]; bfr[j][7] = x1[3];
      }
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][s], bfr[j][s], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
        bf16x8 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[i] = *reinterpret_cast<const bf16x8*>(As[buf] + (wm * WTM + i * 16 + (lane & 15)) * LDK + koff + 32 * kk);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bfr[j] = *reinterpret_cast<const bf16x8*>(Bs[buf] + (wn * WTN + j * 16 + (lane & 15)) * LDK + koff + 32 * kk);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  };

  // prologue: the ring's first NS K-tiles go out before the table fill (they overlap it)
  Pend pa[NS][A_PER], pb[NS][B_PER];
#pragma unroll
  for (int u = 0; u < NS; ++u) load_tiles(kt0 + u, pa[u], pb[u]);
  tab_fill(p.a_xf, ta, false, first_block);
  tab_fill(p.b_xf, tb, false, false);
  if constexpr (EPI_TBL) tab_fill(p.epi_xf, te, true, false);
  for (int i = tid; i < WG::WM * BN; i += NTHREADS) { red1[i / BN][i % BN] = 0.f; red2[i / BN][i % BN] = 0.f; }
  if constexpr (EM == E_ACC) {
    const vae_xform& dyx = p.dbc_from_b ? p.b_xf : p.a_xf;
    if (first_block && dyx.kind == VAE_X_BN_DY && (p.dbc || dyx.dgamma_out || dyx.dbeta_out)) closed_form_db(dyx, p.dbc);
  }
  __syncthreads();   // tables ready
  PROBE_MARK(1);

  // main loop: K-tile kt is transformed into LDS buffer (kt - kt0) & 1 from ring slot
  // (kt - kt0) % NS, whose registers are then refilled with tile kt + NS.  One barrier per
  // K-tile: a buffer is rewritten two tiles after the compute that read it.
  for (int kb = kt0; kb < kt1; kb += NS) {
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      const int kt = kb + u;
      if (kt < kt1) {
        const int buf = (kt - kt0) & 1;
        store_tiles(buf, pa[u], pb[u]);
        __syncthreads();
        load_tiles(kt + NS, pa[u], pb[u]);
        compute(buf);
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

  // ------------------------------------------------------------------------ epilogue
  // lane holds rows 4*(lane>>4)+e, column lane&15 of each 16x16 tile
  const int rowq = m0 + wm * WTM + 4 * (lane >> 4);
  const int colq = n0 + wn * WTN + (lane & 15);
  if (EM == E_ACC && !p.slab) {
    float* out = static_cast<float*>(p.out);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = colq + j * 16;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = rowq + i * 16 + e;
          if (row >= p.M || col >= p.N) continue;
          if (col == p.ones_col) {
            if (p.bias_grad) atomicAdd(p.bias_grad + row, acc[i][j][e]);
          } else {
            atomicAdd(out + (long)row * p.out_ld + col, acc[i][j][e]);
          }
        }
      }
    return;
  } else {
    if (p.slab) {
      // split-K: raw partial sums to this slice's slab; igemm_finalize runs the epilogue
      float* sl = p.slab + ((long)(phase * p.ksplit + ks) * p.M) * p.N;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = colq + j * 16;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int row = rowq + i * 16 + e;
            if (row < p.M && col < p.N) sl[(long)row * p.N + col] = acc[i][j][e];
          }
        }
      return;
    }
    if constexpr (EM == E_ACC) {
      return;
    } else if constexpr (EM == E_REPARAM) {
      ReparamIn rin[TM][TN][4];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            rin[i][j][e] = reparam_load(p, rowq + i * 16 + e, colq + j * 16, rowq + i * 16 + e < p.M && colq + j * 16 < p.N);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (rowq + i * 16 + e < p.M && colq + j * 16 < p.N)
              reparam_apply(p, rowq + i * 16 + e, colq + j * 16, acc[i][j][e], rin[i][j][e]);
      return;
    } else {
      // pass 1: every load the epilogue needs (aux tensor, bias), before any store
      const rsrc_t raux = epi_aux_rsrc<EM>(p);
      const rsrc_t rres = epi_res_rsrc<EM>(p);
      const bool has_res = EM == E_BNBWD && p.residual != nullptr;
      int obase[TM][4];
      float aux[TM][TN][4], res[TM][TN][4], bias[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) bias[j] = (EM == E_STORE && p.bias && colq + j * 16 < p.N) ? p.bias[colq + j * 16] : 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = rowq + i * 16 + e;
          obase[i][e] = out_row_base(p, phase, row < p.M ? row : 0);
        }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const bool ok = rowq + i * 16 + e < p.M && colq + j * 16 < p.N;
            aux[i][j][e] = ld_elem<T>(raux, ok ? (uint32_t)(obase[i][e] + colq + j * 16) * (uint32_t)sizeof(T) : kOOB);
            res[i][j][e] = has_res ? ld_elem<T>(rres, ok ? (uint32_t)(obase[i][e] + colq + j * 16) * (uint32_t)sizeof(T) : kOOB) : 0.f;
          }
      // pass 2: apply, store, per-column sums
      const bool want_sums = epi_wants_sums<EM>(p);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = colq + j * 16;
        const bool col_ok = col < p.N;
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int row = rowq + i * 16 + e;
            if (row >= p.M || !col_ok) continue;
            epi_apply<T, EM>(p, te, col, obase[i][e] + col, acc[i][j][e], aux[i][j][e], bias[j], s1, s2, res[i][j][e]);
          }
        if (want_sums) {
          s1 += __shfl_xor(s1, 16);
          s1 += __shfl_xor(s1, 32);
          s2 += __shfl_xor(s2, 16);
          s2 += __shfl_xor(s2, 32);
          if (lane < 16 && col_ok) {          // each (wave row, column) has one writer
            red1[wm][wn * WTN + j * 16 + lane] = s1;
            red2[wm][wn * WTN + j * 16 + lane] = s2;
          }
        }
      }
      if (want_sums) {
        __syncthreads();
        for (int c = tid; c < BN; c += NTHREADS) {
          if (n0 + c >= p.N) continue;
          float a = 0.f, b = 0.f;
#pragma unroll
          for (int w = 0; w < WG::WM; ++w) { a += red1[w][c]; b += red2[w][c]; }
          epi_flush_sums<EM>(p, blockIdx.x + blockIdx.z * gridDim.x, n0 + c, a, b);
        }
      }
    }
  }
}

// Split-K finalize: sums the K-slices' slabs in slice order (deterministic) and runs the
// epilogue.  Block = 16 column quads x 16 row lanes, FIN_RPT rows per thread; every slab and
// aux load of a thread is issued before the first one is consumed.
constexpr int FIN_RPT = 2;
constexpr int FIN_ROWS = 16 * FIN_RPT;
template <class T, int EM, bool V4>
__global__ void __launch_bounds__(NTHREADS) igemm_finalize(const GemmParams p) {
  kernarg_prefetch<(sizeof(GemmParams) < 1024 ? sizeof(GemmParams) : 1024)>();
  constexpr bool EPI_TBL = (EM == E_BNBWD);
  __shared__ float r1[16][64], r2[16][64];
  extern __shared__ float tabs[];
  const int ce = tab_stride(p.epi_xf.channels);
  const Tab te{tabs, tabs + ce, nullptr, tabs + 2 * ce, tabs + 3 * ce};
  if constexpr (EPI_TBL) tab_fill(p.epi_xf, te, true, false);
  const int cq = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int col0 = blockIdx.y * 64 + cq * 4;
  const long rows_total = (long)p.M * p.nphase;
  const long slab_elems = rows_total * p.ksplit * p.N;
  const rsrc_t rs = make_rsrc(p.slab, (uint32_t)(slab_elems * 4));
  int phase[FIN_RPT], row[FIN_RPT];
  bool rok[FIN_RPT];
  float v[FIN_RPT][4];
#pragma unroll
  for (int r = 0; r < FIN_RPT; ++r) {
    const long grow = (long)blockIdx.x * FIN_ROWS + rl + 16 * r;
    rok[r] = grow < rows_total;
    phase[r] = rok[r] ? (int)(grow / p.M) : 0;
    row[r] = rok[r] ? (int)(grow - (long)phase[r] * p.M) : 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) v[r][c] = 0.f;
  }
  // slab sums, 4 slices per round (all loads of a round in flight together)
  for (int s0 = 0; s0 < p.ksplit; s0 += 4) {
    float t[4][FIN_RPT][4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int r = 0; r < FIN_RPT; ++r) {
        const bool ok = rok[r] && s0 + u < p.ksplit;
        const uint32_t base = (uint32_t)((((long)phase[r] * p.ksplit + s0 + u) * p.M + row[r]) * p.N + col0);
        if constexpr (V4) {
          const auto q = __builtin_amdgcn_raw_buffer_load_b128(rs, ok && col0 < p.N ? base * 4u : kOOB, 0, 0);
#pragma unroll
          for (int c = 0; c < 4; ++c) t[u][r][c] = __uint_as_float(q[c]);
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c)
            t[u][r][c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, ok && col0 + c < p.N ? (base + c) * 4u : kOOB, 0, 0));
        }
      }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int r = 0; r < FIN_RPT; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) v[r][c] += t[u][r][c];
  }
  __syncthreads();   // epilogue table ready
  if constexpr (EM == E_ACC) {
    // deterministic weight gradient: the slices' sum added once per element (one owner thread)
    float* out = static_cast<float*>(p.out);
#pragma unroll
    for (int r = 0; r < FIN_RPT; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int col = col0 + c;
        if (!rok[r] || col >= p.N) continue;
        if (col == p.ones_col) {
          if (p.bias_grad) p.bias_grad[row[r]] += v[r][c];
        } else {
          out[(long)row[r] * p.out_ld + col] += v[r][c];
        }
      }
    return;
  } else if constexpr (EM == E_REPARAM) {
    ReparamIn rin[FIN_RPT][4];
#pragma unroll
    for (int r = 0; r < FIN_RPT; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) rin[r][c] = reparam_load(p, row[r], col0 + c, rok[r] && col0 + c < p.N);
#pragma unroll
    for (int r = 0; r < FIN_RPT; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (rok[r] && col0 + c < p.N) reparam_apply(p, row[r], col0 + c, v[r][c], rin[r][c]);
    return;
  } else {
    const rsrc_t raux = epi_aux_rsrc<EM>(p);
    const rsrc_t rres = epi_res_rsrc<EM>(p);
    const bool has_res = EM == E_BNBWD && p.residual != nullptr;
    int obase[FIN_RPT];
    float aux[FIN_RPT][4], res[FIN_RPT][4], bias[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) bias[c] = (EM == E_STORE && p.bias && col0 + c < p.N) ? p.bias[col0 + c] : 0.f;
#pragma unroll
    for (int r = 0; r < FIN_RPT; ++r) {
      obase[r] = out_row_base(p, phase[r], row[r]);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint32_t off = rok[r] && col0 + c < p.N ? (uint32_t)(obase[r] + col0 + c) * (uint32_t)sizeof(T) : kOOB;
        aux[r][c] = ld_elem<T>(raux, off);
        res[r][c] = has_res ? ld_elem<T>(rres, off) : 0.f;
      }
    }
    float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < FIN_RPT; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (rok[r] && col0 + c < p.N) epi_apply<T, EM>(p, te, col0 + c, obase[r] + col0 + c, v[r][c], aux[r][c], bias[c], s1[c], s2[c], res[r][c]);
    if (epi_wants_sums<EM>(p)) {
#pragma unroll
      for (int c = 0; c < 4; ++c) { r1[rl][cq * 4 + c] = s1[c]; r2[rl][cq * 4 + c] = s2[c]; }
      __syncthreads();
      if (threadIdx.x < 64) {
        const int col = blockIdx.y * 64 + threadIdx.x;
        float a = 0.f, b = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) { a += r1[i][threadIdx.x]; b += r2[i][threadIdx.x]; }
        if (col < p.N) epi_flush_sums<EM>(p, blockIdx.x, col, a, b);
      }
    }
  }
}

}  // namespace vae
