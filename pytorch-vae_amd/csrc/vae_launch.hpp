// Host-side planning and launching of the implicit-GEMM kernels: tile shape, split-K, FastDiv
// setup, slab workspace and the finalize pass.  Included by the entry-point translation units.
#pragma once
#include "vae_fgemm.hpp"
#include "vae_cgemm.hpp"
#include "vae_bgemm.hpp"
#include <stdlib.h>

#ifdef VAE_PROBE
extern "C" unsigned long long* vae_probe_buffer(void);
#endif

namespace vae {
namespace {

constexpr int kCUs = 256;
constexpr int kTargetBlocks = 512;   // 2 resident workgroups per CU
constexpr long kLdsBytes = 160 * 1024;   // LDS one workgroup may use (MI355X_MICROARCH.md)

// dynamic LDS of the per-channel tables a cgemm launch carries (cg_launch_tile)
inline long cg_table_bytes(const GemmParams& p, int em) {
  const int k = p.a_xf.kind;
  return 4l * (((k == VAE_X_BN_ACT || k == VAE_X_BN_DY) ? 3 * tab_stride(p.a_xf.channels) : 0) +
               (em == E_BNBWD ? 4 * tab_stride(p.epi_xf.channels) : 0));
}
// static LDS of a cgemm tile (operand ring buffers or the epilogue tile, plus the statistic
// partials), with both ring buffers counted
inline long cg_static_bytes(int bm, int bn) {
  const int bk = bm >= 128 ? 64 : 128;
  const long loop = 2l * (bm + bn) * (bk + 8) * 2, epi = (long)bm * (bn + 4) * 4;
  const int wn = bn >= 2 * bm ? 4 : (bm >= 2 * bn ? 1 : 2);
  return (loop > epi ? loop : epi) + (4 / wn) * 2l * bn * 4 + 256;
}

inline vae_xform sanitize(vae_xform x) {
  if (x.channels <= 0) x.channels = 1;
  return x;
}

inline bool xf_ok(const vae_xform& x, const char* what) {
  if (x.kind < VAE_X_NONE || x.kind > VAE_X_BN_DY) { fail(VAE_E_BADARG, "%s: bad xform kind %d", what, x.kind); return false; }
  if (x.kind == VAE_X_BN_ACT || x.kind == VAE_X_BN_DY) {
    if (x.channels > MAXC) { fail(VAE_E_UNSUPPORTED, "%s: %d channels > %d", what, x.channels, MAXC); return false; }
    if (!x.sum || !x.sumsq || !x.gamma || !x.beta || x.count <= 0.f) {
      fail(VAE_E_BADARG, "%s: BatchNorm transform needs sum/sumsq/gamma/beta/count", what); return false;
    }
    if (x.kind == VAE_X_BN_DY && (!x.dgamma || !x.dbeta || !x.aux)) {
      fail(VAE_E_BADARG, "%s: BN_DY transform needs dgamma/dbeta/aux", what); return false;
    }
  }
  if ((x.kind == VAE_X_ACT || x.kind == VAE_X_BN_ACT) && !(x.slope >= 0.f && x.slope <= 1.f)) {
    fail(VAE_E_BADARG, "%s: LeakyReLU slope %g outside [0, 1]", what, x.slope); return false;
  }
  return true;
}

// A backward epilogue that differentiates an activation must be given the stored
// pre-activation tensor (aux); a NULL there would be a device fault, so reject it here.
inline bool epi_ok(const vae_xform& x, const char* what) {
  if (!xf_ok(x, what)) return false;
  if ((x.kind == VAE_X_BN_ACT || x.kind == VAE_X_ACT) && !x.aux) {
    fail(VAE_E_BADARG, "%s: activation-backward epilogue needs aux (the stored pre-activation)", what);
    return false;
  }
  if (x.kind == VAE_X_BN_DY) { fail(VAE_E_BADARG, "%s: BN_DY is not an epilogue transform", what); return false; }
  return true;
}

// Phase tap tables of a transposed conv (or conv dgrad) with stride S, kernel R, padding P:
// output coordinate o of phase ph = o % S receives taps r with (ph + P - r) % S == 0.
inline bool make_taps(GemmParams& p, int S, int R, int P) {
  if (S < 1 || S > 2) return false;
  for (int ph = 0; ph < S; ++ph) {
    const int first = ((ph + P) % S + S) % S;       // smallest r with (ph + P - r) % S == 0
    const int n = first < R ? (R - 1 - first) / S + 1 : 0;
    if (n < 1 || n > 4) return false;
    p.tap0[ph] = first;
    p.ntap_h[ph] = n; p.ntap_w[ph] = n;
    p.tap_d[ph] = (ph + P - first) / S;
  }
  return true;
}

// The optional BatchNorm finalisation a producing call carries (vae_conv_args.bn_finalize):
// validated up front, launched right after the GEMM (see vaehip.h; an in-kernel last-workgroup
// variant measured slower: every workgroup then needs an agent-scope release, and the extra
// epilogue code and LDS lowered the GEMMs' occupancy).
inline int check_finalize(const vae_bn_args* f, const uint32_t* counter, const char* what) {
  if (!f) return VAE_OK;
  (void)counter;
  if (f->mode != 0 && f->mode != 1) return fail(VAE_E_BADARG, "%s: fused finalisation mode %d", what, f->mode);
  if (!f->table || f->xf.channels <= 0 || !f->xf.sum || !f->xf.sumsq || !f->xf.gamma || !f->xf.beta || f->xf.count <= 0.f ||
      (f->mode == 1 && (!f->xf.dgamma || !f->xf.dbeta)) || f->xf.reps > BNF_LANES * BNF_PER)
    return fail(VAE_E_BADARG, "%s: bn_finalize args", what);
  return VAE_OK;
}

inline int then_finalize(int rc, const vae_bn_args* f, hipStream_t st) {
  if (rc || !f) return rc;
  return bn_finalize_launch(f, st);
}

inline GemmParams base_params() {
  GemmParams p;
  memset(&p, 0, sizeof(p));
  p.ksplit = 1; p.nphase = 1; p.ones_col = -1; p.gs = 1; p.samples = 1; p.gr = 1;
  p.a_xf.channels = 1; p.b_xf.channels = 1; p.epi_xf.channels = 1; p.res_xf.channels = 1;
  p.ntap_h[0] = p.ntap_h[1] = p.ntap_w[0] = p.ntap_w[1] = 1;
  return p;
}

// Elements a tensor operand spans (the buffer-resource extent; aux tensors are shaped alike).
template <int AM>
inline long a_elems(const GemmParams& p) {
  if (AM == A_CONV || AM == A_CONVT) return (long)p.gn * p.gh * p.gw * p.gc;
  if (AM == A_DENSE) return (long)(p.M - 1) * p.a_ld + p.K;
  return (long)(p.K - 1) * p.a_ld + p.M;   // A_KM
}

template <int BMD>
inline long b_elems(const GemmParams& p) {
  if (BMD == B_GATHER) return (long)p.gn * p.gh * p.gw * p.gc;
  if (BMD == B_NK) return (long)(p.N - 1) * p.b_ld + p.K;
  const long rows = p.b_taps ? (long)p.gc * p.gr * p.gr : p.K;   // B_KN
  return (rows - 1) * p.b_ld + (p.ones_col >= 0 ? p.N - 1 : p.N);
}

inline bool aligned(const void* ptr, int bytes) { return ((uintptr_t)ptr & (uintptr_t)(bytes - 1)) == 0; }

// Packed (vector) operand layout: V_K groups read 8 consecutive k of one row, V_M groups 4
// consecutive rows of one k.  Needs aligned rows, and for a BatchNorm transform channels that
// run consecutively inside a group.
inline bool bn_kind(const vae_xform& x) { return x.kind == VAE_X_BN_ACT || x.kind == VAE_X_BN_DY; }

template <int MODE>   // AMode, or 100 + BMode
inline int operand_vec(const GemmParams& p, const void* ptr, const vae_xform& xf, int esize) {
  const bool vk = MODE == A_CONV || MODE == A_CONVT || MODE == A_DENSE || MODE == 100 + B_NK;
  const int grp = vk ? 8 : 4;
  const int vbytes = (grp * esize) < 16 ? grp * esize : 16;
  if (!aligned(ptr, vbytes) || (xf.kind == VAE_X_BN_DY && !aligned(xf.aux, vbytes))) return 0;
  if (bn_kind(xf) && xf.channels % grp) return 0;
  // V_K groups must not straddle the end of K, V_M groups the end of the rows: the packed path
  // has no per-element masks (out-of-range groups read as 0 through the buffer resource)
  const int nrows = p.N - (p.ones_col >= 0 ? 1 : 0);
  switch (MODE) {
    case A_CONV: return !p.g_nchw && p.gc % grp == 0;
    case 100 + B_GATHER: return !p.g_nchw && p.gc % grp == 0 && nrows % grp == 0;
    case A_CONVT: return p.gc % grp == 0;
    case A_DENSE: return p.a_ld % grp == 0 && p.K % grp == 0;
    case A_KM: return p.a_ld % grp == 0 && p.M % grp == 0;
    case 100 + B_NK: return p.b_ld % grp == 0 && p.K % grp == 0;
    case 100 + B_KN: return p.b_ld % grp == 0 && nrows % grp == 0;
  }
  return 0;
}

inline void finish_divs(GemmParams& p) {
  p.fd_gq = make_fastdiv(p.gq > 0 ? p.gq : 1);
  p.fd_gp = make_fastdiv(p.gp > 0 ? p.gp : 1);
  p.fd_gc = make_fastdiv(p.gc > 0 ? p.gc : 1);
  p.fd_gr = make_fastdiv(p.gr > 0 ? p.gr : 1);
  p.fd_ntw[0] = make_fastdiv(p.ntap_w[0] > 0 ? p.ntap_w[0] : 1);
  p.fd_ntw[1] = make_fastdiv(p.ntap_w[1] > 0 ? p.ntap_w[1] : 1);
  p.fd_ach = make_fastdiv(p.a_xf.channels > 0 ? p.a_xf.channels : 1);
  p.fd_bch = make_fastdiv(p.b_xf.channels > 0 ? p.b_xf.channels : 1);
  p.fd_ech = make_fastdiv(p.epi_xf.channels > 0 ? p.epi_xf.channels : 1);
}

struct Tile { int bm, bn; };

inline long tile_blocks(long M, long N, int nphase, Tile t) {
  return ((M + t.bm - 1) / t.bm) * ((N + t.bn - 1) / t.bn) * nphase;
}

// Tile (4 waves) for the grid: the largest one that still puts ~4 blocks on every CU, so that
// several waves per SIMD overlap each other's load/transform/barrier stalls; the split-K planner
// below raises the block count further when K is long.
constexpr int kTileBlocks = 4 * kCUs;
inline Tile pick_tile(long M, long N, int nphase) {
  const Tile wide[] = {{64, 64}, {64, 32}, {32, 64}, {32, 32}};
  const Tile thin_n[] = {{128, 32}, {64, 32}, {32, 32}};
  const Tile thin_m[] = {{32, 128}, {32, 64}, {32, 32}};
  const Tile* c = N <= 32 ? thin_n : (M <= 32 ? thin_m : wide);
  const int nc = N <= 32 ? 3 : (M <= 32 ? 3 : 4);
  for (int i = 0; i < nc; ++i)
    if (tile_blocks(M, N, nphase, c[i]) >= kTileBlocks) return c[i];
  return c[nc - 1];
}

// K-slices: enough blocks to cover the CUs twice, >= 4 K-tiles per slice.  The partial slabs of
// a split need workspace (split * rows * N fp32); the caller checks it with split_fits.
inline int pick_split(long blocks, int ktiles) {
  if (blocks >= kTargetBlocks || ktiles < 8) return 1;
  int s = (int)((kTargetBlocks + blocks - 1) / blocks);
  const int maxs = ktiles / 4;
  if (s > maxs) s = maxs;
  return s < 2 ? 1 : s;
}

// Settle a split-K choice against the caller's workspace: no workspace (NULL) -> no split,
// unless the caller asked for one (VAE_E_BADARG); a workspace too small for the slabs ->
// VAE_E_BADARG.  Returns VAE_OK with *split updated, or the error code.
inline int split_fits(int* split, int split_req, const GemmParams& p, const void* ws, long ws_bytes, const char* what) {
  if (*split <= 1) return VAE_OK;
  if (!ws && !querying()) {
    if (split_req > 1) return fail(VAE_E_BADARG, "%s: split_k %d needs a workspace", what, split_req);
    *split = 1;
    return VAE_OK;
  }
  return ws_fits((long)*split * p.M * p.N * p.nphase * 4, ws_bytes, what) ? VAE_OK : VAE_E_BADARG;
}

template <class T, int EM>
inline int launch_finalize(const GemmParams& p, hipStream_t st) {
  const long rows = (long)p.M * p.nphase;
  const dim3 grid((unsigned)((rows + FIN_ROWS - 1) / FIN_ROWS), (unsigned)((p.N + 63) / 64));
  const size_t lds = EM == E_BNBWD ? (size_t)tab_floats(p.epi_xf, true) * 4 : 0;
  if (p.N % 4 == 0) VAE_LAUNCH((igemm_finalize<T, EM, true>), grid, dim3(NTHREADS), lds, st, p);
  else VAE_LAUNCH((igemm_finalize<T, EM, false>), grid, dim3(NTHREADS), lds, st, p);
  return check_launch("igemm_finalize");
}

// ------------------------------------------------------------------ deterministic mode
// Rows of per-channel sums a deterministic launch writes (one per contributing block): the
// finalize's row blocks after a split-K, else the main grid's M blocks x phases.
template <int EM>
inline bool det_wants_sums(const GemmParams& p) {
  return (EM == E_STORE && p.sum) || (EM == E_BNBWD && p.epi_xf.kind == VAE_X_BN_ACT);
}
inline long det_sum_rows(const GemmParams& p, int bm) {
  if (p.ksplit > 1) return ((long)p.M * p.nphase + FIN_ROWS - 1) / FIN_ROWS;
  return (long)((p.M + bm - 1) / bm) * p.nphase;
}
// Bytes of det_slab: the sums' rows [2][N] or the reparameterization terms [rows][2*latent].
template <int EM>
inline long det_slab_bytes(const GemmParams& p, int bm) {
  if (!p.det) return 0;
  if (det_wants_sums<EM>(p)) return det_sum_rows(p, bm) * 2 * p.N * 4;
  if (EM == E_REPARAM) return (long)p.M * 2 * p.latent * 4;
  return 0;
}
// The ordered pass over det_slab (after the main kernel and its finalize).
template <int EM>
inline int det_reduce(const GemmParams& p, hipStream_t st) {
  if (!p.det_slab) return VAE_OK;
  OrdSum o;
  memset(&o, 0, sizeof(o));
  o.slab = p.det_slab;
  if (EM == E_REPARAM) {
    o.rstride = 2L * p.latent; o.groups = p.M / p.samples; o.rpg = p.samples;
    o.cols = 2 * p.latent; o.cw = p.latent; o.hstride = p.latent; o.folds = 1;
    o.dst[0] = p.dmulv; o.dst[1] = p.dmulv + p.latent; o.gstride = 2L * p.latent;
  } else {
    const int ch = EM == E_STORE ? p.N : p.epi_xf.channels;
    o.rstride = 2L * p.N; o.groups = 1; o.rpg = (int)(p.det_rows);
    o.cols = 2 * ch; o.cw = ch; o.hstride = p.N; o.folds = p.N / ch; o.fstride = ch;
    o.dst[0] = EM == E_STORE ? p.sum : p.dbeta;
    o.dst[1] = EM == E_STORE ? p.sumsq : p.dgamma;
  }
  return ordered_sum_launch(o, st);
}

// A launch whose dynamic tables are large (> 64 KB: BatchNorm widths of 2048-4096 channels) is
// checked against the LDS budget with the kernel's own static LDS; the launch is skipped and
// check_launch's caller sees VAE_E_UNSUPPORTED through lds_error.
inline thread_local bool lds_error = false;
template <class K>
inline bool lds_fits(K kernel, size_t dyn) {
  if (dyn <= 64 * 1024 || querying()) return true;
  hipFuncAttributes at;
  if (hipFuncGetAttributes(&at, reinterpret_cast<const void*>(kernel)) != hipSuccess) return true;
  if ((long)(at.sharedSizeBytes + dyn) <= kLdsBytes) return true;
  lds_error = true;
  return false;
}

#define VAE_TILE_CASE(BM_, BN_) \
  if (t.bm == BM_ && t.bn == BN_) { \
    if (lds_fits(igemm_kernel<T, TA, TB, BM_, BN_, AM, BMD, EM, VA, VB, DYA, DYB>, lds)) \
      VAE_LAUNCH((igemm_kernel<T, TA, TB, BM_, BN_, AM, BMD, EM, VA, VB, DYA, DYB>), grid, block, lds, st, p); \
    return; \
  }

template <class T, class TA, class TB, int AM, int BMD, int EM, bool VA, bool VB, bool DYA, bool DYB>
inline void launch_shape(const GemmParams& p, Tile t, hipStream_t st) {
  const dim3 block(NTHREADS);
  const dim3 grid((p.M + t.bm - 1) / t.bm, (p.N + t.bn - 1) / t.bn, p.nphase * p.ksplit);
  const size_t lds = (size_t)table_floats(p, EM == E_BNBWD) * 4;
  VAE_TILE_CASE(64, 64)
  VAE_TILE_CASE(128, 32)
  VAE_TILE_CASE(32, 128)
  VAE_TILE_CASE(64, 32)
  VAE_TILE_CASE(32, 64)
  VAE_TILE_CASE(32, 32)
}
#undef VAE_TILE_CASE

// Output-tensor extent (elements) the epilogue's aux operand spans: rows of the phase grid or
// plain rows, times the row pitch.
inline long out_elems(const GemmParams& p) {
  if (p.out_phase) return (long)p.gn * p.gho * p.gwo * p.out_ld;
  return (long)p.M * p.out_ld;
}

template <class T, class TA, class TB, int AM, int BMD, int EM, bool DYA, bool DYB>
inline int launch_tiled(GemmParams p, Tile t, hipStream_t st) {
  const long ab = a_elems<AM>(p) * (long)sizeof(TA), bb = b_elems<BMD>(p) * (long)sizeof(TB);
  if (ab <= 0 || bb <= 0 || ab >= (1l << 31) || bb >= (1l << 31))
    return fail(VAE_E_UNSUPPORTED, "igemm: operand of %ld / %ld bytes (buffer addressing needs < 2 GiB)", ab, bb);
  p.a_bytes = (uint32_t)ab;
  p.b_bytes = (uint32_t)bb;
  if (EM != E_ACC && EM != E_REPARAM) {
    const long ob = out_elems(p) * (long)(p.out_f32 ? 4 : sizeof(T));
    if (ob >= (1l << 31)) return fail(VAE_E_UNSUPPORTED, "igemm: output of %ld bytes (needs < 2 GiB)", ob);
    p.out_aux_bytes = (uint32_t)(out_elems(p) * (long)sizeof(T));
  }
  if ((!DYA && p.a_xf.kind == VAE_X_BN_DY) || (!DYB && p.b_xf.kind == VAE_X_BN_DY))
    return fail(VAE_E_UNSUPPORTED, "igemm: BN_DY transform on an operand this op does not support");
#ifdef VAE_PROBE
  p.probe = vae_probe_buffer();
#endif
  // packed (vector) staging per operand: an operand that cannot be packed (the NCHW image, a
  // 3-channel tensor or weight matrix) no longer drags the other one onto the per-element path
  const bool va = operand_vec<AM>(p, p.a_ptr, p.a_xf, (int)sizeof(TA));
  const bool vb = operand_vec<100 + BMD>(p, p.b_ptr, p.b_xf, (int)sizeof(TB));
  if (va && vb) launch_shape<T, TA, TB, AM, BMD, EM, true, true, DYA, DYB>(p, t, st);
  else if (va) launch_shape<T, TA, TB, AM, BMD, EM, true, false, DYA, DYB>(p, t, st);
  else if (vb) launch_shape<T, TA, TB, AM, BMD, EM, false, true, DYA, DYB>(p, t, st);
  else launch_shape<T, TA, TB, AM, BMD, EM, false, false, DYA, DYB>(p, t, st);
  if (lds_error) {
    lds_error = false;
    return fail(VAE_E_UNSUPPORTED, "igemm: per-channel tables of %d / %d channels exceed the LDS", p.a_xf.channels,
                p.epi_xf.channels);
  }
  int rc = check_launch("igemm");
  if (rc) return rc;
  if (p.slab && (rc = launch_finalize<T, EM>(p, st))) return rc;
  return det_reduce<EM>(p, st);
}

// ------------------------------------------------------------------ direct-fragment GEMM path
// Shapes fgemm_kernel takes: k-contiguous weights (B_NK), gathered tensors with C % 32 == 0 (a
// 32-deep k-step stays inside one tap), 16-byte aligned rows, packed BatchNorm channels.
template <int AM, int BMD, int EM>
inline bool fgemm_ok(const GemmParams& p, int esize_a, int esize_b) {
  if constexpr (BMD != B_NK || AM == A_KM || EM == E_ACC) return false;
  if (p.g_nchw || p.ones_col >= 0) return false;
  // Measured (profiles/r1_v2_kernel_breakdown.txt): direct fragments win on the deep-K Linear
  // shapes (fc_mu||fc_var 9.7 -> 4.0 us) but lose on the conv / convT ones, whose blocks run two
  // residency rounds of latency-bound phases; those stay on the LDS-staged kernel.
  if (AM == A_CONV || AM == A_CONVT) {
    return false;
  } else {
    if (p.K % 32 || p.a_ld % 8) return false;
  }
  if (p.b_ld % 8 || (p.K % 32 && AM != A_CONVT)) return false;
  if (!aligned(p.a_ptr, 16) || !aligned(p.b_ptr, 16)) return false;
  if (p.a_xf.kind == VAE_X_BN_DY && !aligned(p.a_xf.aux, 16)) return false;
  if (bn_kind(p.a_xf) && p.a_xf.channels % 8) return false;
  (void)esize_a; (void)esize_b;
  return true;
}

template <class T, class TA, int AM, int EM, bool DYA>
inline int launch_fgemm(GemmParams p, void* ws, long ws_bytes, hipStream_t st) {
  constexpr int BM = 32, BN = 32;
  const long ab = a_elems<AM>(p) * (long)sizeof(TA), bb = b_elems<B_NK>(p) * (long)sizeof(T);
  if (ab <= 0 || bb <= 0 || ab >= (1l << 31) || bb >= (1l << 31))
    return fail(VAE_E_UNSUPPORTED, "fgemm: operand of %ld / %ld bytes (buffer addressing needs < 2 GiB)", ab, bb);
  p.a_bytes = (uint32_t)ab;
  p.b_bytes = (uint32_t)bb;
  if (EM != E_REPARAM) p.out_aux_bytes = (uint32_t)(out_elems(p) * (long)sizeof(T));
  int kmax = p.K;
  if (AM == A_CONVT) {
    kmax = 0;
    for (int ph = 0; ph < p.nphase; ++ph) {
      const int k = p.ntap_h[ph / p.gs] * p.ntap_w[ph % p.gs] * p.gc;
      kmax = k > kmax ? k : kmax;
    }
  }
  const int steps = (kmax + 31) / 32;
  const long tiles = (long)((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN) * p.nphase;
  // split-K over workgroups (slabs + igemm_finalize) until ~2 workgroups per CU, >= 4 k-steps
  // per workgroup (one per wave)
  int split = 1;
  if (tiles < 2 * kCUs) {
    split = (int)((2 * kCUs + tiles - 1) / tiles);
    if (split > steps / 4) split = steps / 4;
    if (split < 2) split = 1;
  }
  if (int rc = split_fits(&split, 0, p, ws, ws_bytes, "fgemm split-K")) return rc;
  p.ksplit = split;
  p.slab = split > 1 ? static_cast<float*>(ws) : nullptr;
#ifdef VAE_PROBE
  p.probe = vae_probe_buffer();
#endif
  const dim3 grid((p.M + BM - 1) / BM, (p.N + BN - 1) / BN, p.nphase * p.ksplit);
  const size_t lds = (size_t)(tab_floats(p.a_xf, false) + (EM == E_BNBWD ? tab_floats(p.epi_xf, true) : 0)) * 4;
  VAE_LAUNCH((fgemm_kernel<T, TA, BM, BN, AM, EM, DYA>), grid, dim3(256), lds, st, p);
  int rc = check_launch("fgemm");
  if (rc) return rc;
  if (p.slab) return launch_finalize<T, EM>(p, st);
  return VAE_OK;
}

// Plan tile + split-K, then launch.  A_F32 / B_F32: instantiate the bf16 variant whose A / B
// tensor is fp32 (the NCHW image, d[mu|logvar]).
template <int AM, int BMD, int EM, bool DYA, bool DYB, bool A_F32 = false, bool B_F32 = false>
inline int launch(int dtype, bool a_f32, bool b_f32, GemmParams p, int split_req, void* ws, long ws_bytes,
                  hipStream_t st) {
  if (p.M <= 0 || p.N <= 0) return VAE_OK;
  finish_divs(p);
  if constexpr (BMD == B_NK && AM != A_KM && EM != E_ACC) {
    if (!a_f32 && !b_f32 && split_req <= 0 && !p.det && fgemm_ok<AM, BMD, EM>(p, 0, 0)) {
      if (dtype == VAE_F32) return launch_fgemm<float, float, AM, EM, DYA>(p, ws, ws_bytes, st);
      if (dtype == VAE_BF16) return launch_fgemm<__bf16, __bf16, AM, EM, DYA>(p, ws, ws_bytes, st);
    }
  }
  const Tile t = pick_tile(p.M, p.N, p.nphase);
  const int bk = dtype == VAE_F32 ? 32 : 64;
  int kmax = p.K;
  if (AM == A_CONVT) {
    kmax = 0;
    for (int ph = 0; ph < p.nphase; ++ph) {
      const int k = p.ntap_h[ph / p.gs] * p.ntap_w[ph % p.gs] * p.gc;
      kmax = k > kmax ? k : kmax;
    }
  }
  const int ktiles = (kmax + bk - 1) / bk;
  const long blocks = (long)((p.M + t.bm - 1) / t.bm) * ((p.N + t.bn - 1) / t.bn) * p.nphase;
  if (p.det && dtype != VAE_F32) return fail(VAE_E_UNSUPPORTED, "deterministic reductions need dtype VAE_F32");
  // deterministic weight gradients: K slices to a slab (<= 64 MB) summed by the finalize instead
  // of fp32 atomics into dW
  const bool slab = EM != E_ACC || p.det;
  int split = split_req > 0 ? split_req : pick_split(blocks, ktiles);
  if (EM == E_ACC && p.det && split_req <= 0) {
    const long cap = (64l << 20) / ((long)p.M * p.N * p.nphase * 4);
    if (split > cap) split = cap < 1 ? 1 : (int)cap;
  }
  if (slab && split > 1) {
    if (int rc = split_fits(&split, split_req, p, ws, ws_bytes, "igemm split-K")) return rc;
    if (split > 1) p.slab = static_cast<float*>(ws);
  }
  p.ksplit = split < 1 ? 1 : split;
  if (p.det) {
    const long off = p.slab ? (((long)p.ksplit * p.M * p.N * p.nphase * 4 + 255) & ~255l) : 0;
    const long need = det_slab_bytes<EM>(p, t.bm);
    if (need > 0) {
      if (!ws && !querying()) return fail(VAE_E_BADARG, "igemm: a deterministic call needs a workspace");
      if (!ws_fits(off + need, ws_bytes, "igemm deterministic sums")) return VAE_E_BADARG;
      p.det_slab = reinterpret_cast<float*>(static_cast<char*>(ws) + off);
      p.det_rows = det_wants_sums<EM>(p) ? det_sum_rows(p, t.bm) : 0;
      if (EM == E_REPARAM && p.M % p.samples) return fail(VAE_E_BADARG, "igemm: rows %d not a multiple of samples %d", p.M, p.samples);
      if (EM == E_BNBWD && p.N % p.epi_xf.channels) return fail(VAE_E_UNSUPPORTED, "igemm: %d columns over %d channels", p.N, p.epi_xf.channels);
    }
  }
  if (dtype == VAE_F32) return launch_tiled<float, float, float, AM, BMD, EM, DYA, DYB>(p, t, st);
  if (dtype != VAE_BF16) return fail(VAE_E_BADDTYPE, "dtype %d", dtype);
  if constexpr (A_F32) {
    if (a_f32) return launch_tiled<__bf16, float, __bf16, AM, BMD, EM, DYA, DYB>(p, t, st);
  }
  if constexpr (B_F32) {
    if (b_f32) return launch_tiled<__bf16, __bf16, float, AM, BMD, EM, DYA, DYB>(p, t, st);
  }
  if (a_f32 || b_f32) return fail(VAE_E_UNSUPPORTED, "fp32 operand not instantiated for this op");
  return launch_tiled<__bf16, __bf16, __bf16, AM, BMD, EM, DYA, DYB>(p, t, st);
}

// Column sums of a plain [rows][C] tensor (bias gradient of a layer whose dy is stored as is).
// The tensor is streamed as flat 8-element vectors (C % 8 == 0) or single elements (any C). The
// block size is a multiple of the number of vector groups per row, and so is the grid stride, so
// every thread keeps the same channels for its whole loop; partials meet in LDS and each
// workgroup issues one global atomic per channel (grid capped at one workgroup per CU).
template <class T, int V>
__global__ void __launch_bounds__(256) column_sum_flat(const T* x, long nvec, int C, float* out) {
  extern __shared__ float red[];
  const int groups = C / V;
  for (int c = threadIdx.x; c < C; c += blockDim.x) red[c] = 0.f;
  __syncthreads();
  const int c0 = (int)(threadIdx.x % groups) * V;
  float acc[V];
#pragma unroll
  for (int j = 0; j < V; ++j) acc[j] = 0.f;
  const long stride = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  // 8 independent 16-byte loads in flight (4: 11.9 us per VQ-VAE call at B=128, r4_v6_vq_pmc.json —
  // one workgroup per CU leaves the loads in flight per thread as the only latency cover)
  for (; i + 7 * stride < nvec; i += 8 * stride) {
    if constexpr (V == 8) {
      float v[8][8];
#pragma unroll
      for (int u = 0; u < 8; ++u) ld8(x + (i + u * stride) * 8, v[u]);
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += v[u][j];
    } else {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = ld_f(x + i + u * stride);
      acc[0] += ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
    }
  }
  for (; i < nvec; i += stride) {
    if constexpr (V == 8) {
      float v[8];
      ld8(x + i * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    } else {
      acc[0] += ld_f(x + i);
    }
  }
#pragma unroll
  for (int j = 0; j < V; ++j) atomicAdd(red + c0 + j, acc[j]);
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) atomicAdd(out + c, red[c]);
}

// Fallback for widths the flat kernel does not cover (more than 256 vector groups per row)
template <class T>
__global__ void column_sum(const T* x, long rows, int C, float* out) {
  const int c = blockIdx.y * 64 + (threadIdx.x & 63);
  if (c >= C) return;
  float s = 0.f;
  for (long r = blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += (long)gridDim.x * 4) s += ld_f(x + r * C + c);
  atomicAdd(out + c, s);
}

// W'[c][t'][k] = W[k][t][c] (bf16) with t' = t (swap) or RR-1-t (flip: the data gradient of a
// stride-1 conv as a conv).  Per tap a [K][C] -> [C][K] transpose through a 32x33 LDS tile, so
// reads and writes are both 64-byte row segments (an element-wise gather reads with a stride of
// R*R*C elements).
__global__ void __launch_bounds__(256) flip_weights_kernel(const __bf16* w, __bf16* wf, int K, int RR, int C, int flip) {
  __shared__ float t[32][33];
  const int tap = blockIdx.z, k0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int j = ty; j < 32; j += 8) {
    const int k = k0 + j, c = c0 + tx;
    t[j][tx] = (k < K && c < C) ? (float)w[((long)k * RR + tap) * C + c] : 0.f;
  }
  __syncthreads();
  const int tap2 = flip ? RR - 1 - tap : tap;
  for (int j = ty; j < 32; j += 8) {
    const int c = c0 + j, k = k0 + tx;
    if (c < C && k < K) wf[((long)c * RR + tap2) * K + k] = (__bf16)t[tx][j];
  }
}

inline int flip_weights_launch(const __bf16* w, __bf16* wf, int K, int R, int C, hipStream_t st, int flip = 1) {
  const dim3 grid((C + 31) / 32, (K + 31) / 32, R * R);
  VAE_LAUNCH(flip_weights_kernel, grid, dim3(256), 0, st, w, wf, K, R * R, C, flip);
  return check_launch("flip_weights");
}

// ------------------------------------------------------------------ bf16 conv-GEMM (vae_cgemm.hpp)
// Eligible: bf16 NHWC operands with channel counts % 8 (16-byte chunks never straddle a tap),
// 16-byte aligned tensors, k-contiguous weight rows, and a transform / epilogue pair the kernel
// is instantiated for.  VAE_NO_CGEMM=1 keeps everything on the generic kernel (A/B timing).
inline bool cg_ok(const GemmParams& p, int em) {
  if (p.g_nchw || p.ones_col >= 0 || p.gc % 8 || p.N % 8 || p.out_ld % 8 || p.b_ld % 8) return false;
  if (!aligned(p.a_ptr, 16) || !aligned(p.b_ptr, 16) || !aligned(p.out, 16)) return false;
  const int k = p.a_xf.kind;
  if (em == E_STORE && k == VAE_X_BN_DY) return false;
  if (em == E_BNBWD && k == VAE_X_BN_ACT) return false;
  if ((k == VAE_X_BN_ACT || k == VAE_X_BN_DY) && (p.a_xf.channels != p.gc || p.a_xf.channels > MAXC)) return false;
  if (k == VAE_X_BN_DY && !aligned(p.a_xf.aux, 16)) return false;
  if (p.residual && !aligned(p.residual, 16)) return false;
  // the widest BatchNorm tables (4096 channels on both sides) leave no room for an operand tile
  if (cg_table_bytes(p, em) + cg_static_bytes(32, 32) > kLdsBytes) return false;
  if (em == E_BNBWD && p.epi_xf.kind != VAE_X_NONE) {
    // (a plain LeakyReLU epilogue has no per-channel table: its channel count is not read)
    if (!aligned(p.epi_xf.aux, 16) || (p.epi_xf.kind == VAE_X_BN_ACT && p.epi_xf.channels % 8)) return false;
  }
  return true;
}

struct CgTile { int bm, bn; };

// Launch shape: a tile must give every CU this many workgroups before a smaller one is tried, and
// K is split while a launch has fewer than kCgSplitWg workgroups per CU (swept in round 5,
// profiles/r5_notes.md: 1 / 3 / 4 and 2 / 3 measured slower on the VanillaVAE step)
constexpr int kCgMinWg = 2, kCgSplitWg = 1;
inline int cg_minwg() { return kCgMinWg; }
inline int cg_splitwg() { return kCgSplitWg; }

// Largest tile that still gives every CU ~2 workgroups; split-K (slabs + igemm_finalize) when
// even the smallest leaves the chip half empty and K is deep.  xform: the gathered operand is
// transformed on load (BatchNorm tables, a second raw tensor for BN_DY): those instantiations hold
// two 64 x 32 workgroups per CU, so a 64 x 32 grid of 4 per CU ran as two rounds (tools/kprobe.py:
// the encoder.1 data gradient's second round started 11.9 us in, 21.9 us in all) — 128 x 32 from 4
// per CU makes it one round; transform-free layers keep it for the long thin maps only.
inline CgTile cg_pick(long M, long N, int nphase, long table_bytes = 0, bool xform = false) {
  const CgTile c[] = {{128, 128}, {128, 32}, {64, 64}, {64, 32}, {32, 64}, {32, 32}};
  for (const CgTile& t : c) {
    if (table_bytes + cg_static_bytes(t.bm, t.bn) > kLdsBytes) continue;   // (wide BatchNorm tables)
    if (t.bm > 32 && M < t.bm) continue;
    if (t.bn > 32 && N < t.bn) continue;
    if (t.bm == 128 && t.bn == 32 && tile_blocks(M, N, nphase, Tile{64, 32}) < (xform ? 4 : 8) * kCUs) continue;
    if (tile_blocks(M, N, nphase, Tile{t.bm, t.bn}) >= (long)cg_minwg() * kCUs) return t;
  }
  return CgTile{32, 32};
}

template <int BM, int BN> constexpr int cg_bk() { return BM >= 128 ? 64 : 128; }

template <int AM, int XA, int EM, int OR>
inline void cg_launch_tile(const GemmParams& p, CgTile t, hipStream_t st) {
  const size_t lds = (size_t)((XA == VAE_X_BN_ACT || XA == VAE_X_BN_DY ? 3 * tab_stride(p.a_xf.channels) : 0) +
                              (EM == E_BNBWD ? 4 * tab_stride(p.epi_xf.channels) : 0)) * 4;
#define VAE_CG_CASE(BM_, BN_) \
  if (t.bm == BM_ && t.bn == BN_) { \
    const unsigned nb = (unsigned)(((p.M + BM_ - 1) / BM_) * ((p.N + BN_ - 1) / BN_) * p.nphase * p.ksplit); \
    VAE_LAUNCH((cgemm_kernel<BM_, BN_, cg_bk<BM_, BN_>(), AM, XA, EM, OR>), dim3(nb), dim3(256), lds, st, p); \
    return; \
  }
  VAE_CG_CASE(128, 128)
  VAE_CG_CASE(128, 32)
  VAE_CG_CASE(64, 64)
  VAE_CG_CASE(64, 32)
  VAE_CG_CASE(32, 64)
  VAE_CG_CASE(32, 32)
#undef VAE_CG_CASE
}

// Plan tile + split-K and launch (GemmParams as for launch_tiled; B must be k-contiguous rows)
template <int AM, int EM>
inline int cg_launch(GemmParams p, int split_req, void* ws, long ws_bytes, hipStream_t st) {
  if (p.M <= 0 || p.N <= 0) return VAE_OK;
  finish_divs(p);
  const long ab = a_elems<AM>(p) * 2, bb = (long)(p.N - 1) * p.b_ld * 2 + (long)p.b_ld * 2;
  if (ab <= 0 || bb <= 0 || ab >= (1l << 31) || bb >= (1l << 31))
    return fail(VAE_E_UNSUPPORTED, "cgemm: operand of %ld / %ld bytes (buffer addressing needs < 2 GiB)", ab, bb);
  p.a_bytes = (uint32_t)ab;
  p.b_bytes = (uint32_t)bb;
  const long ob = out_elems(p) * 2;
  if (ob >= (1l << 31)) return fail(VAE_E_UNSUPPORTED, "cgemm: output of %ld bytes", ob);
  p.out_aux_bytes = (uint32_t)ob;
#ifdef VAE_PROBE
  p.probe = vae_probe_buffer();
#endif
  // transform-free large layers (an operand the caller materialised): the LDS-DMA pipeline
  if (split_req <= 0 && bgemm_ok(p, AM, EM)) {
    const int rc = bgemm_launch(p, AM, EM, ws, ws_bytes, st);
    if (rc != kHeadFallback) return rc;
  }
  const CgTile t = cg_pick(p.M, p.N, p.nphase, cg_table_bytes(p, EM),
                           p.a_xf.kind == VAE_X_BN_ACT || p.a_xf.kind == VAE_X_BN_DY);
  const int bk = t.bm >= 128 ? 64 : 128;
  // tile order (vae_cgemm.hpp): m fastest when the weights outweigh the gathered input tensor
  p.m_fast = (long)p.b_bytes > (long)p.a_bytes ? 1 : 0;
  int kmax = p.K;
  if (AM == A_CONVT) {
    kmax = 0;
    for (int ph = 0; ph < p.nphase; ++ph) {
      const int k = p.ntap_h[ph / p.gs] * p.ntap_w[ph % p.gs] * p.gc;
      kmax = k > kmax ? k : kmax;
    }
  }
  const int ktiles = (kmax + bk - 1) / bk;
  const long blocks = tile_blocks(p.M, p.N, p.nphase, Tile{t.bm, t.bn});
  int split = split_req > 0 ? split_req : 1;
  if (split_req <= 0 && blocks < (long)cg_splitwg() * kCUs && ktiles >= 4) {
    split = (int)((2 * (long)cg_splitwg() * kCUs + blocks - 1) / blocks);
    if (split > ktiles / 2) split = ktiles / 2;
  }
  if (int rc = split_fits(&split, split_req, p, ws, ws_bytes, "cgemm split-K")) return rc;
  p.ksplit = split < 1 ? 1 : split;
  p.slab = p.ksplit > 1 ? static_cast<float*>(ws) : nullptr;
  // one-round kernels when every slice's K-steps fit the ring of the chosen instantiation
  const int kps = (ktiles + p.ksplit - 1) / p.ksplit;
  const bool dy = p.a_xf.kind == VAE_X_BN_DY;
  const int KCt = bk / 8, RPPt = 256 / KCt;
  const int loads = ((t.bm + RPPt - 1) / RPPt) * (dy ? 2 : 1) + (t.bn + RPPt - 1) / RPPt;
  const int ns = cg_ring(loads);                                           // == cg_stages<loads>()
  const bool one = kps <= ns;
  // (OR == 3, forward only: the BatchNorm-backward data gradients measured 6-14 us slower with it)
  const bool deep = EM == E_STORE && !one && kps <= cg_ring_deep(loads) && blocks * p.ksplit <= 2l * kCUs;
#define VAE_CG_XA(XA_) (deep ? cg_launch_tile<AM, XA_, EM, (EM == E_STORE ? 3 : 0)>(p, t, st) \
                        : !one ? cg_launch_tile<AM, XA_, EM, 0>(p, t, st) \
                              : kps <= 2 ? cg_launch_tile<AM, XA_, EM, 2>(p, t, st) : cg_launch_tile<AM, XA_, EM, 1>(p, t, st))
  switch (p.a_xf.kind) {
    case VAE_X_NONE: VAE_CG_XA(VAE_X_NONE); break;
    case VAE_X_ACT: VAE_CG_XA(VAE_X_ACT); break;
    case VAE_X_BN_ACT:
      if constexpr (EM == E_STORE) VAE_CG_XA(VAE_X_BN_ACT);
      break;
    case VAE_X_BN_DY:
      if constexpr (EM == E_BNBWD) VAE_CG_XA(VAE_X_BN_DY);
      break;
  }
#undef VAE_CG_XA
  int rc = check_launch("cgemm");
  if (rc) return rc;
  if (p.slab) return launch_finalize<__bf16, EM>(p, st);
  return VAE_OK;
}

inline int column_sum_launch(int dtype, const void* dy, long rows, int C, float* db, hipStream_t st) {
  const int V = (C % 8 == 0 && ((uintptr_t)dy % 16) == 0) ? 8 : 1;   // 16-B aligned vectors
  const int groups = C / V;
  if (groups <= 256 && rows > 0) {
    const int bd = (256 / groups) * groups;
    const long nvec = rows * (long)(C / V);
    long blocks = (nvec + (long)bd * 8 - 1) / ((long)bd * 8);      // >= 8 vectors per thread
    if (blocks > 256) blocks = 256;
    if (blocks < 1) blocks = 1;
    const size_t lds = (size_t)C * sizeof(float);
    if (dtype == VAE_F32) {
      if (V == 8) VAE_LAUNCH((column_sum_flat<float, 8>), dim3((unsigned)blocks), dim3(bd), lds, st, (const float*)dy, nvec, C, db);
      else VAE_LAUNCH((column_sum_flat<float, 1>), dim3((unsigned)blocks), dim3(bd), lds, st, (const float*)dy, nvec, C, db);
    } else {
      if (V == 8) VAE_LAUNCH((column_sum_flat<__bf16, 8>), dim3((unsigned)blocks), dim3(bd), lds, st, (const __bf16*)dy, nvec, C, db);
      else VAE_LAUNCH((column_sum_flat<__bf16, 1>), dim3((unsigned)blocks), dim3(bd), lds, st, (const __bf16*)dy, nvec, C, db);
    }
    return check_launch("column_sum");
  }
  const dim3 grid(64, (C + 63) / 64);
  if (dtype == VAE_F32) VAE_LAUNCH(column_sum<float>, grid, dim3(256), 0, st, (const float*)dy, rows, C, db);
  else VAE_LAUNCH(column_sum<__bf16>, grid, dim3(256), 0, st, (const __bf16*)dy, rows, C, db);
  return check_launch("column_sum");
}

}  // namespace
}  // namespace vae

namespace vae {
namespace {
inline bool geom_ok(const vae_conv_args* a, const char* what) {
  if (!a) { fail(VAE_E_BADARG, "%s: null args", what); return false; }
  if (a->n <= 0 || a->h <= 0 || a->w <= 0 || a->c <= 0 || a->k <= 0 || a->p <= 0 || a->q <= 0 || a->r <= 0 ||
      a->stride <= 0 || a->pad < 0) {
    fail(VAE_E_BADSHAPE, "%s: bad geometry", what); return false;
  }
  if (a->deterministic && a->dtype != VAE_F32) {
    fail(VAE_E_UNSUPPORTED, "%s: deterministic reductions need dtype VAE_F32", what); return false;
  }
  return true;
}
}  // namespace
}  // namespace vae
