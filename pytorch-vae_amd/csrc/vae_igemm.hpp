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

constexpr int MAXC = 512;   // max channels of a per-channel transform table
constexpr int NTHREADS = 256;

template <class T> constexpr int bk_of() { return sizeof(T) == 2 ? 64 : 32; }

// Magic-number division for 0 <= n < 2^31 (round-up method; exact for every n in range).
struct FastDiv {
  uint32_t d, mul, shr;
  __device__ __forceinline__ uint32_t div(uint32_t n) const { return d == 1 ? n : (__umulhi(n, mul) >> shr); }
};

inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d < 1 ? 1 : d;
  if (f.d == 1) { f.mul = 0; f.shr = 0; return f; }
  uint32_t l = 0;
  while ((1u << l) < f.d) ++l;
  const uint32_t p = 31 + l;
  f.mul = (uint32_t)(((1ull << p) + f.d - 1) / f.d);
  f.shr = p - 32;
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
  FastDiv fd_gq, fd_gp, fd_gc, fd_gr, fd_ntw[2];
  // ---- epilogue
  void* out; int out_ld; int out_phase;      // out_phase: rows are phase-grid pixels
  int out_f32;               // E_STORE: write fp32 instead of T
  const float* bias; float* sum; float* sumsq;
  const void* residual; vae_xform res_xf;
  vae_xform epi_xf; float* dgamma; float* dbeta;
  float* bias_grad;
  float* dbc; int dbc_from_b;  // closed-form BN-followed bias gradient (wgrad, first block)
  const float* mulv; const float* eps; const float* kl_coef; float* dmulv; int samples, latent;
  float* slab;               // split-K partials [nphase][ksplit][M][N] (non-ACC epilogues)
  // ---- operand access (host-derived, see vae_launch.hpp)
  uint32_t a_bytes, b_bytes; // buffer-resource extents of the A / B tensors (and their aux)
  FastDiv fd_ach, fd_bch;    // transform channel counts of A / B
  unsigned long long* probe; // VAE_PROBE builds: per-block phase timestamps (diagnostics only)
};

// Phase timestamps of one block (VAE_PROBE builds): record = {block id, wall0, wall3, clk0..clk3,
// hw id}; probe[0] is the record counter, probe[1] the capacity.
#ifdef VAE_PROBE
#define PROBE_MARK(i) do { if (threadIdx.x == 0) clk[i] = __builtin_readcyclecounter(); } while (0)
__device__ __forceinline__ void probe_write(unsigned long long* pr, const unsigned long long* clk,
                                           unsigned long long w0) {
  if (!pr || threadIdx.x != 0) return;
  const unsigned long long slot = atomicAdd(pr, 1ull);
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
  return q;
}

// ------------------------------------------------------------------ per-channel tables
// Views into dynamic LDS, sized by the real channel count of each transform (rounded up to 4
// so vector reads of 4 consecutive channels stay 16-byte aligned):
//   BN_ACT: v = lrelu(t*a + b)   BN_DY: v = a*t + b*aux + c   epilogue BN_ACT: x̂ = y*p + q
struct Tab {
  float *a, *b, *c, *p, *q;
};

__host__ __device__ inline int tab_pad(int c) { return (c + 3) & ~3; }
// Each table row is followed by 8 zero entries (the "zero slot" at index tab_pad(C)): a packed
// group that is out of range points its channel there, so any transform maps it to exactly 0.
__host__ __device__ inline int tab_stride(int c) { return tab_pad(c) + 8; }

__device__ __forceinline__ void tab_fill(const vae_xform& x, Tab t, bool epi, bool update_running) {
  if (x.kind != VAE_X_BN_ACT && x.kind != VAE_X_BN_DY) return;
  if (threadIdx.x < 8) {
    const int z = tab_pad(x.channels) + threadIdx.x;
    t.a[z] = 0.f; t.b[z] = 0.f;
    if (x.kind == VAE_X_BN_DY) t.c[z] = 0.f;
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
      const float mg = x.dbeta[ch] * inv_m;         // mean of g
      const float mgx = x.dgamma[ch] * inv_m;       // mean of g*xhat
      t.a[ch] = A;
      t.b[ch] = -A * invstd * mgx;
      t.c[ch] = -A * (mg - mean * invstd * mgx);
    }
  }
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
  s.y = make_rsrc(s.dy ? xf.aux : ptr, bytes);
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

template <class TIn, int NB>
__device__ __forceinline__ void bload_pair(const Src<TIn>& s, uint32_t off, uint32_t* w, uint32_t* y) {
  bload<NB>(s.x, off, w);
  if (s.dy) bload<NB>(s.y, off, y);
}

// ------------------------------------------------------------------ V_K operand (row x 8 k)
// Row state is computed once per thread slot; load() is called once per K-tile.
template <class TIn, int MODE, bool VEC>
struct RowOperand {
  int valid;       // row in range
  int n, hb, wb;   // A_CONV: image, top-left input coordinate; A_CONVT: image, ho, wo
  int base;        // A_DENSE / B_NK: row offset (elements)

  __device__ __forceinline__ void init(const GemmParams& p, int row, int rows, int phase, int ld) {
    valid = row < rows;
    if constexpr (MODE == A_DENSE || MODE == 100 + B_NK) {
      base = row * ld;
    } else if constexpr (MODE == A_CONV) {
      const uint32_t t = p.fd_gq.div(row), oq = row - t * p.gq;
      const uint32_t nn = p.fd_gp.div(t), op = t - nn * p.gp;
      n = nn; hb = op * p.gs - p.gpad; wb = oq * p.gs - p.gpad;
    } else if constexpr (MODE == A_CONVT) {
      const PhaseInfo q = make_phase(p, phase);
      const uint32_t t = p.fd_gq.div(row), ww = row - t * p.gq;
      const uint32_t nn = p.fd_gp.div(t), hh = t - nn * p.gp;
      n = nn; hb = hh * p.gs + q.ph; wb = ww * p.gs + q.pw;
    }
  }

  // element offset + in-range flag of k (per-element path, and the group's k0 in the packed one)
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
      const int r = q.t0h + p.gs * (int)th, s = q.t0w + p.gs * (int)tw;
      const int hi = (hb + p.gpad - r) / p.gs, wi = (wb + p.gpad - s) / p.gs;
      ok = hi >= 0 && hi < p.gh && wi >= 0 && wi < p.gw;
      return ((n * p.gh + hi) * p.gw + wi) * C + c;
    }
  }

  __device__ __forceinline__ void load(const GemmParams& p, const Src<TIn>& s, const PhaseInfo& q, const FastDiv& fdc,
                                       int k0, int Kp, Pend& g) const {
    constexpr int E = sizeof(TIn);
    g.ones = 0u;
    g.chb = s.kind >= VAE_X_BN_ACT ? (int)(k0 - fdc.div(k0) * s.C) : 0;
    if constexpr (VEC) {
      // whole group in or out (host: K % 8 == 0); out -> zeros and the zero-slot channel
      bool ok;
      const int idx = offset(p, q, k0, ok);
      const bool gv = valid && ok && k0 < Kp;
      g.chb = gv ? g.chb : s.zs;
      const uint32_t off = gv ? (uint32_t)idx * E : kOOB;
      bload_pair<TIn, 16>(s, off, g.w, g.y);
      if constexpr (E == 4) bload_pair<TIn, 16>(s, off + 16, g.w + 4, g.y + 4);
    } else {
      uint32_t m = 0u;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        bool ok;
        const int idx = offset(p, q, k0 + e, ok);
        ok = ok && valid && k0 + e < Kp;
        m |= (uint32_t)ok << e;
        bload_pair<TIn, E>(s, ok ? (uint32_t)idx * E : kOOB, g.w + e, g.y + e);
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
        if constexpr (E == 2) bload_pair<TIn, 8>(s, off, g.w + 2 * t, g.y + 2 * t);
        else bload_pair<TIn, 16>(s, off, g.w + 4 * t, g.y + 4 * t);
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
          bload_pair<TIn, E>(s, ok ? (uint32_t)idx * E : kOOB, g.w + 4 * t + j, g.y + 4 * t + j);
        }
    }
    g.m = m;
  }
};

// Transform of a staged group (after its loads have landed) -> 8 floats in element order.
// Masked elements become 0 after the transform (the transform of a zero pad is not zero).
template <class TIn, int MODE, bool VM, bool VEC>
__device__ __forceinline__ void finish(const GemmParams& p, const Src<TIn>& s, const Tab& t, const Pend& g,
                                       float (&v)[8]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = raw_elem<TIn, VEC>(g.w, e);
  if (s.kind == VAE_X_BN_ACT || s.kind == VAE_X_BN_DY) {
    const bool dy = s.kind == VAE_X_BN_DY;
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

template <class T, class TIn>
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
  } else if (s.kind == VAE_X_BN_DY) {
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
template <class T, class TIn, int MODE>
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
  } else if (s.kind == VAE_X_BN_DY) {
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
__device__ __forceinline__ long out_index(const GemmParams& p, int phase, int row, int col) {
  if (p.out_phase) {
    const int ph = phase >= p.gs ? 1 : 0, pw = phase - ph * p.gs;
    const uint32_t t = p.fd_gq.div(row), ww = row - t * p.gq;
    const uint32_t n = p.fd_gp.div(t), hh = t - n * p.gp;
    const int ho = hh * p.gs + ph, wo = ww * p.gs + pw;
    return (((long)n * p.gho + ho) * p.gwo + wo) * p.out_ld + col;
  }
  return (long)row * p.out_ld + col;
}

// One output element of a non-accumulating epilogue.  s1/s2 collect the per-column sums.
template <class T, int EM>
__device__ __forceinline__ void epi_elem(const GemmParams& p, const Tab& xe, int phase, int row,
                                         int col, float v, float& s1, float& s2) {
  if constexpr (EM == E_REPARAM) {
    const int b = row / p.samples;
    const float mu = p.mulv[(long)b * 2 * p.latent + col];
    const float lv = p.mulv[(long)b * 2 * p.latent + p.latent + col];
    const float ep = p.eps[(long)row * p.latent + col];
    const float c = p.kl_coef ? p.kl_coef[row] : 0.f;
    const float sd = expf(0.5f * lv);
    atomicAdd(p.dmulv + (long)b * 2 * p.latent + col, v + c * mu);
    atomicAdd(p.dmulv + (long)b * 2 * p.latent + p.latent + col, v * ep * 0.5f * sd + c * 0.5f * (expf(lv) - 1.f));
  } else {
    const long idx = out_index(p, phase, row, col);
    if constexpr (EM == E_STORE) {
      float y = v + (p.bias ? p.bias[col] : 0.f);
      if (p.residual) {
        float rv = ld_f(static_cast<const T*>(p.residual) + idx);
        if (p.res_xf.kind == VAE_X_ACT) rv = lrelu(rv, p.res_xf.slope);
        y += rv;
      }
      if (p.out_f32) static_cast<float*>(p.out)[idx] = y;
      else static_cast<T*>(p.out)[idx] = cvt<T>(y);
      s1 += v;
      s2 += v * v;
    } else {  // E_BNBWD
      float g = v;
      if (p.epi_xf.kind == VAE_X_BN_ACT) {
        const int ch = col % p.epi_xf.channels;
        const float yv = ld_f(static_cast<const T*>(p.epi_xf.aux) + idx);
        const float z = fmaf(yv, xe.a[ch], xe.b[ch]);
        g = z > 0.f ? v : v * p.epi_xf.slope;
        s1 += g;
        s2 += g * fmaf(yv, xe.p[ch], xe.q[ch]);
      } else if (p.epi_xf.kind == VAE_X_ACT) {
        const float yv = ld_f(static_cast<const T*>(p.epi_xf.aux) + idx);
        g = yv > 0.f ? v : v * p.epi_xf.slope;
      }
      static_cast<T*>(p.out)[idx] = cvt<T>(g);
    }
  }
}

template <int EM>
__device__ __forceinline__ bool epi_wants_sums(const GemmParams& p) {
  if constexpr (EM == E_STORE) return p.sum != nullptr;
  if constexpr (EM == E_BNBWD) return p.epi_xf.kind == VAE_X_BN_ACT;
  return false;
}

template <int EM>
__device__ __forceinline__ void epi_flush_sums(const GemmParams& p, int col, float s1, float s2) {
  float* g1 = (EM == E_STORE) ? p.sum : p.dbeta;
  float* g2 = (EM == E_STORE) ? p.sumsq : p.dgamma;
  const int ch = (EM == E_STORE) ? col : col % p.epi_xf.channels;
  atomicAdd(g1 + ch, s1);
  atomicAdd(g2 + ch, s2);
}

// Closed-form bias gradient of a conv followed by train-mode BatchNorm:
//   db = Σ dy = A·Σg + B·Σy + C·M per channel (A,B,C the BN-backward coefficients)
__device__ __forceinline__ void closed_form_db(const vae_xform& x, float* db) {
  for (int ch = threadIdx.x; ch < x.channels; ch += blockDim.x) {
    float mean, invstd, var;
    bn_moments(x, ch, mean, invstd, var);
    const float inv_m = 1.0f / x.count;
    const float A = x.gamma[ch] * invstd;
    const float mgx = x.dgamma[ch] * inv_m;
    const float mg = x.dbeta[ch] * inv_m;
    const float B = -A * invstd * mgx;
    const float C = -A * (mg - mean * invstd * mgx);
    const float sum_y = x.sum[ch] + x.count * (x.shift ? x.shift[ch] : 0.f);
    db[ch] += A * x.dbeta[ch] + B * sum_y + C * x.count;
  }
}

template <int AM> constexpr bool a_is_vm() { return AM == A_KM; }
template <int BMD> constexpr bool b_is_vm() { return BMD != B_NK; }

// dynamic LDS: per-channel tables of the A, B and epilogue transforms (floats)
__host__ __device__ inline int table_floats(const GemmParams& p, bool epi_tbl) {
  return tab_floats(p.a_xf, false) + tab_floats(p.b_xf, false) + (epi_tbl ? tab_floats(p.epi_xf, true) : 0);
}

// ------------------------------------------------------------------------------ kernel
// T: LDS/MFMA type; TA: storage type of the A tensor (fp32 for the NCHW image / d[mu|logvar]);
// TB: storage type of B (the gathered activation for B_GATHER, weights otherwise).
template <class T, class TA, class TB, int BM, int BN, int AM, int BMD, int EM, bool VEC>
__global__ void __launch_bounds__(NTHREADS) igemm_kernel(const GemmParams p) {
  constexpr int BK = bk_of<T>();
  constexpr int LDK = BK + (sizeof(T) == 4 ? 4 : 8);        // padded LDS row (elements)
  constexpr int WTM = BM / 2, WTN = BN / 2;                 // 2x2 waves
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr bool A_VM = a_is_vm<AM>();
  constexpr bool B_VM = b_is_vm<BMD>();
  constexpr int KO = BK / 8;                                // V_K octets per row
  constexpr int A_OCT = BM * BK / 8, B_OCT = BN * BK / 8;   // octets per tile
  constexpr int A_PER = (A_OCT + NTHREADS - 1) / NTHREADS, B_PER = (B_OCT + NTHREADS - 1) / NTHREADS;
  constexpr bool EPI_TBL = (EM == E_BNBWD);
  constexpr int A_MODE = AM;
  constexpr int B_MODE = 100 + BMD;

  __shared__ __attribute__((aligned(16))) T As[2][BM * LDK];
  __shared__ __attribute__((aligned(16))) T Bs[2][BN * LDK];
  __shared__ float red1[BN], red2[BN];
  extern __shared__ float tabs[];

#ifdef VAE_PROBE
  unsigned long long clk[4] = {0, 0, 0, 0};
  const unsigned long long wall0 = threadIdx.x == 0 ? wall_clock64() : 0;
#endif
  PROBE_MARK(0);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
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
  RowOperand<TA, A_MODE, VEC> ars[A_VM ? 1 : A_PER];
  ColOperand<TA, A_MODE, VEC> acs[A_VM ? A_PER : 1];
  RowOperand<TB, B_MODE, VEC> brs[B_VM ? 1 : B_PER];
  ColOperand<TB, B_MODE, VEC> bcs[B_VM ? B_PER : 1];
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

  Pend pa[A_PER], pb[B_PER];

  auto load_tiles = [&](int kt) {
    const int kb = kt * BK;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int o = tid + i * NTHREADS;
      if (A_OCT % NTHREADS == 0 || o < A_OCT) {
        if constexpr (!A_VM) ars[i].load(p, sa, pq, p.fd_ach, kb + (o % KO) * 8, Kp, pa[i]);
        else acs[i].load(p, sa, pq, kb + 2 * (o / (BM / 4)), Kp, pa[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int o = tid + i * NTHREADS;
      if (B_OCT % NTHREADS == 0 || o < B_OCT) {
        if constexpr (!B_VM) brs[i].load(p, sb, pq, p.fd_bch, kb + (o % KO) * 8, Kp, pb[i]);
        else bcs[i].load(p, sb, pq, kb + 2 * (o / (BN / 4)), Kp, pb[i]);
      }
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int o = tid + i * NTHREADS;
      if (A_OCT % NTHREADS == 0 || o < A_OCT) {
        if constexpr (VEC) {
          if constexpr (!A_VM) store_vk<T, TA>(sa, ta, pa[i], As[buf] + (o / KO) * LDK + (o % KO) * 8);
          else store_vm<T, TA, A_MODE>(sa, ta, pa[i], As[buf] + (o % (BM / 4)) * 4 * LDK + 2 * (o / (BM / 4)), LDK);
          continue;
        }
        float v[8];
        finish<TA, A_MODE, A_VM, VEC>(p, sa, ta, pa[i], v);
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
        if constexpr (VEC) {
          if constexpr (!B_VM) store_vk<T, TB>(sb, tb, pb[i], Bs[buf] + (o / KO) * LDK + (o % KO) * 8);
          else store_vm<T, TB, B_MODE>(sb, tb, pb[i], Bs[buf] + (o % (BN / 4)) * 4 * LDK + 2 * (o / (BN / 4)), LDK);
          continue;
        }
        float v[8];
        finish<TB, B_MODE, B_VM, VEC>(p, sb, tb, pb[i], v);
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

  // prologue: first tile's global loads go out before the table fill (they overlap it)
  if (kt0 < kt1) load_tiles(kt0);
  tab_fill(p.a_xf, ta, false, first_block);
  tab_fill(p.b_xf, tb, false, false);
  if constexpr (EPI_TBL) tab_fill(p.epi_xf, te, true, false);
  for (int i = tid; i < BN; i += NTHREADS) { red1[i] = 0.f; red2[i] = 0.f; }
  if constexpr (EM == E_ACC) {
    if (first_block && p.dbc) closed_form_db(p.dbc_from_b ? p.b_xf : p.a_xf, p.dbc);
  }
  __syncthreads();   // tables ready
  PROBE_MARK(1);
  if (kt0 < kt1) {
    store_tiles(0);
    __syncthreads();
    int buf = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      const bool more = kt + 1 < kt1;
      if (more) load_tiles(kt + 1);       // raw loads in flight during the MFMAs below
      compute(buf);
      if (more) store_tiles(buf ^ 1);     // transform + LDS write; other buffer, read 1 iter ago
      __syncthreads();
      buf ^= 1;
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
  if constexpr (EM == E_ACC) {
    float* out = static_cast<float*>(p.out);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + wn * WTN + j * 16 + (lane & 15);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = m0 + wm * WTM + i * 16 + 4 * (lane >> 4) + e;
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
          const int col = n0 + wn * WTN + j * 16 + (lane & 15);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int row = m0 + wm * WTM + i * 16 + 4 * (lane >> 4) + e;
            if (row < p.M && col < p.N) sl[(long)row * p.N + col] = acc[i][j][e];
          }
        }
      return;
    }
    const bool want_sums = epi_wants_sums<EM>(p);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wn * WTN + j * 16 + (lane & 15);
      const bool col_ok = col < p.N;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = m0 + wm * WTM + i * 16 + 4 * (lane >> 4) + e;
          if (row >= p.M || !col_ok) continue;
          epi_elem<T, EM>(p, te, phase, row, col, acc[i][j][e], s1, s2);
        }
      if (want_sums) {
        s1 += __shfl_xor(s1, 16);
        s1 += __shfl_xor(s1, 32);
        s2 += __shfl_xor(s2, 16);
        s2 += __shfl_xor(s2, 32);
        if (lane < 16 && col_ok) {
          atomicAdd(&red1[wn * WTN + j * 16 + lane], s1);
          atomicAdd(&red2[wn * WTN + j * 16 + lane], s2);
        }
      }
    }
    if (want_sums) {
      __syncthreads();
      for (int c = tid; c < BN; c += NTHREADS)
        if (n0 + c < p.N) epi_flush_sums<EM>(p, n0 + c, red1[c], red2[c]);
    }
  }
}

// Split-K finalize: sums the K-slices' slabs in slice order and runs the epilogue.
// grid: (ceil(M*nphase / 64), ceil(N / 64)); block 256 = 4 row groups x 64 columns.
template <class T, int EM>
__global__ void __launch_bounds__(NTHREADS) igemm_finalize(const GemmParams p) {
  constexpr bool EPI_TBL = (EM == E_BNBWD);
  __shared__ float r1[4][64], r2[4][64];
  extern __shared__ float tabs[];
  const int ce = tab_stride(p.epi_xf.channels);
  const Tab te{tabs, tabs + ce, nullptr, tabs + 2 * ce, tabs + 3 * ce};
  if constexpr (EPI_TBL) tab_fill(p.epi_xf, te, true, false);
  __syncthreads();
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int col = blockIdx.y * 64 + cl;
  const long rows_total = (long)p.M * p.nphase;
  float s1 = 0.f, s2 = 0.f;
  if (col < p.N) {
    for (int rr = rg; rr < 64; rr += 4) {
      const long grow = (long)blockIdx.x * 64 + rr;
      if (grow >= rows_total) break;
      const int phase = (int)(grow / p.M);
      const int row = (int)(grow - (long)phase * p.M);
      const float* sl = p.slab + ((long)phase * p.ksplit * p.M + row) * p.N + col;
      float v = 0.f;
      for (int s = 0; s < p.ksplit; ++s) v += sl[(long)s * p.M * p.N];
      epi_elem<T, EM>(p, te, phase, row, col, v, s1, s2);
    }
  }
  if (epi_wants_sums<EM>(p)) {
    r1[rg][cl] = s1;
    r2[rg][cl] = s2;
    __syncthreads();
    if (rg == 0 && col < p.N)
      epi_flush_sums<EM>(p, col, r1[0][cl] + r1[1][cl] + r1[2][cl] + r1[3][cl],
                         r2[0][cl] + r2[1][cl] + r2[2][cl] + r2[3][cl]);
  }
}

}  // namespace vae
