// C-ABI entry point: one Conv2d / ConvTranspose2d block's data AND weight gradient as one grid
// (the two bwd calls of one layer of models/vanilla_vae.py:25-75 under experiment.py:45-86's
// loss.backward()).
//
// Why: the VanillaVAE's layers are latency-bound at B=64 — a data-gradient launch of 256-1024
// small conv-GEMM tiles leaves most of the chip's issue slots idle for its 15-25 us, and the
// weight gradients then ran after the whole data-gradient chain as three grouped launches
// (95 us, profiles/r4_v1_kstats.json).  Both gradients of a layer read the same BatchNorm-backward
// gradient dy' (and its table, built from the same statistics), so they can run side by side:
// workgroups [0, nd) run the data-gradient tile body (vae_cgemm.hpp cgemm_body), workgroups
// [nd, nd + nw) the weight-gradient body (vae_wgemm.hpp) in the same LDS allocation.  The
// weight gradient's K slices add into dW with fp32 atomics (one slice: plain accumulation) — no
// slab, no reduction launch.
//
// The pair kernels are instantiated for the transforms a BatchNorm'd block has (dy' = BN-backward
// of the block's output, x = the previous block's lrelu(BN(y)) or the untransformed decoder input)
// and the data-gradient tiles the planner gives the VanillaVAE family (32x32 / 64x32, one- or
// two-step slices); any other combination runs the two calls one after the other.
#include "vae_launch.hpp"
#include "vae_wgrad.hpp"
#include "vae_wgemm.hpp"

namespace vae {

struct PairRider {
  WgParams w;          // the weight-gradient problem (unplanned: its K slices are sized at launch)
  bool used;           // set once a pair grid carried it
};

PairRider*& pair_rider() {
  static thread_local PairRider* r = nullptr;
  return r;
}

namespace {

struct PairArgs {
  GemmParams g;        // data gradient (cgemm_body)
  WgParams w;          // weight gradient (wgemm_body / wgemm_taps_body)
  int nd;              // workgroups of the data gradient
};
static_assert(sizeof(PairArgs) <= 3584, "kernel argument block");

// weight-gradient tile classes: 0 = 32 x 32 with all 3x3 taps per workgroup, 1 = 64 x 64, 2 = 128 x 128
// variants (the weight gradient's operand transforms): 1 = conv (U = dy' BN_DY, V = x BN_ACT);
// 2 / 3 = transposed conv (U = x none / BN_ACT, V = dy' BN_DY)
template <int CLS> constexpr int pair_t() { return CLS == 0 ? 32 : (CLS == 1 ? 64 : 128); }
template <int CLS> constexpr int pair_rr() { return CLS == 0 ? 3 : 0; }
template <int VAR> constexpr int pair_xu() { return VAR == 1 ? VAE_X_BN_DY : (VAR == 3 ? VAE_X_BN_ACT : VAE_X_NONE); }
template <int VAR> constexpr int pair_xv() { return VAR == 1 ? VAE_X_BN_ACT : VAE_X_BN_DY; }

template <int BM, int BN, int OR, int CLS> constexpr int pair_lds() {
  constexpr int cg = CgSmem<BM, BN, cg_bk<BM, BN>(), cg_nbuf<BM, BN, cg_bk<BM, BN>(), OR>()>::BYTES;
  constexpr int T = pair_t<CLS>();
  constexpr int wg = CLS == 0 ? wgemm_taps_lds_bytes<T, T, 3>() : wgemm_lds_bytes<T, T>();
  return cg > wg ? cg : wg;
}
// register budget: two workgroups per CU — unconstrained, the 128 x 128 weight-gradient body
// beside a 32 x 32 data tile took 352 registers (one per CU); at three per CU (the 64 x 32 data
// tile's own budget) the all-taps 32 x 32 weight-gradient body spilled 65 registers
template <int BM, int BN, int CLS> constexpr int pair_waves() { return 2; }

template <int BM, int BN, int AM, int OR, int CLS, int VAR>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(pair_waves<BM, BN, CLS>())))
pair_kernel(const PairArgs a) {
  __shared__ __attribute__((aligned(16))) char lds[pair_lds<BM, BN, OR, CLS>()];
  const int b = (int)blockIdx.x;
  if (b < a.nd) {
    cgemm_body<BM, BN, cg_bk<BM, BN>(), AM, VAE_X_BN_DY, E_BNBWD, OR>(a.g, b, lds);
  } else {
    constexpr int T = pair_t<CLS>();
    if constexpr (CLS == 0) wgemm_taps_body<T, T, pair_xu<VAR>(), pair_xv<VAR>(), 3>(a.w, b - a.nd, lds);
    else wgemm_body<T, T, pair_xu<VAR>(), pair_xv<VAR>()>(a.w, b - a.nd, lds);
  }
}

inline int pair_class(const WgPlan& w) {
  if (w.T == 32) return w.taps == 3 ? 0 : -1;
  return w.taps ? -1 : (w.T == 64 ? 1 : 2);
}
inline int pair_variant(const WgParams& p) {
  if (!p.dy_is_v) return (p.u_xf.kind == VAE_X_BN_DY && p.v_xf.kind == VAE_X_BN_ACT) ? 1 : -1;
  if (p.v_xf.kind != VAE_X_BN_DY) return -1;
  return p.u_xf.kind == VAE_X_NONE ? 2 : (p.u_xf.kind == VAE_X_BN_ACT ? 3 : -1);
}

// Weight-gradient workgroups of a pair grid: VAE_PAIR_SLOTS (default one per CU) — sized with the
// data gradient's own grid in view it would be the same for the deep layers (256-512 tiles) and
// the slice count bounds the atomics every slice adds into dW.
inline long pair_slots() {
  static const int v = tune_env("VAE_PAIR_SLOTS", kCUs);
  return v;
}

template <int BM, int BN, int AM, int OR, int CLS, int VAR>
inline void pair_go(const PairArgs& a, unsigned blocks, size_t lds, hipStream_t st) {
  VAE_LAUNCH((pair_kernel<BM, BN, AM, OR, CLS, VAR>), dim3(blocks), dim3(256), lds, st, a);
}

template <int BM, int BN, int AM, int OR>
inline bool pair_cls(const PairArgs& a, int cls, int var, unsigned blocks, size_t lds, hipStream_t st) {
#define VAE_PAIR_CV(C_, V_) \
  if (cls == C_ && var == V_) { pair_go<BM, BN, AM, OR, C_, V_>(a, blocks, lds, st); return true; }
  if constexpr (AM == A_CONVT) {              // Conv2d data gradient (phase gather of dy')
    VAE_PAIR_CV(0, 1) VAE_PAIR_CV(1, 1) VAE_PAIR_CV(2, 1)
  } else {                                     // ConvTranspose2d data gradient (strided conv of dy')
    VAE_PAIR_CV(0, 2) VAE_PAIR_CV(1, 2) VAE_PAIR_CV(2, 2)
    VAE_PAIR_CV(0, 3) VAE_PAIR_CV(1, 3) VAE_PAIR_CV(2, 3)
  }
#undef VAE_PAIR_CV
  return false;
}

}  // namespace

bool pair_cg_launch(const GemmParams& p, unsigned nb, int bm, int bn, int am, int xa, int em, int orr, size_t lds,
                    hipStream_t st) {
  PairRider* r = pair_rider();
  if (!r || r->used || xa != VAE_X_BN_DY || em != E_BNBWD) return false;
  if (!((bm == 32 && bn == 32 && orr == 0) || (bm == 64 && bn == 32 && (orr == 0 || (orr == 2 && am == A_CONVT)))))
    return false;
  WgPlan w;
  if (wg2_plan(r->w, nullptr, 0, &w, pair_slots()) != VAE_OK) return false;
  const int cls = pair_class(w), var = pair_variant(w.p);
  if (cls < 0 || var < 0 || w.p.slab) return false;
  PairArgs a;
  memset(&a, 0, sizeof(a));
  a.g = p;
  a.w = w.p;
  a.nd = (int)nb;
  const bool bu = w.p.u_xf.kind == VAE_X_BN_ACT || w.p.u_xf.kind == VAE_X_BN_DY;
  const bool bv = w.p.v_xf.kind == VAE_X_BN_ACT || w.p.v_xf.kind == VAE_X_BN_DY;
  const size_t wl = (size_t)((bu ? 3 * tab_stride(w.p.u_xf.channels) : 0) + (bv ? 3 * tab_stride(w.p.v_xf.channels) : 0)) * 4;
  const size_t dl = lds > wl ? lds : wl;
  const unsigned blocks = nb + w.blocks;
  bool ok = false;
  if (am == A_CONVT) {
    if (bm == 64 && orr == 2) ok = pair_cls<64, 32, A_CONVT, 2>(a, cls, var, blocks, dl, st);
    else if (bm == 64) ok = pair_cls<64, 32, A_CONVT, 0>(a, cls, var, blocks, dl, st);
    else ok = pair_cls<32, 32, A_CONVT, 0>(a, cls, var, blocks, dl, st);
  } else if (am == A_CONV) {
    if (bm == 64) ok = pair_cls<64, 32, A_CONV, 0>(a, cls, var, blocks, dl, st);
    else ok = pair_cls<32, 32, A_CONV, 0>(a, cls, var, blocks, dl, st);
  }
  if (ok) r->used = true;
  return ok;
}

}  // namespace vae

using namespace vae;

extern "C" int vae_conv_bwd_pair(int32_t kind, const vae_conv_args* data, const vae_conv_args* filter, void* workspace,
                                 int64_t workspace_bytes, void* stream) {
  if (kind != VAE_LAYER_CONV2D && kind != VAE_LAYER_CONVT2D) return fail(VAE_E_BADARG, "conv_bwd_pair: kind %d", kind);
  if (!data || !filter) return fail(VAE_E_BADARG, "conv_bwd_pair: null args");
  const bool tr = kind == VAE_LAYER_CONVT2D;
  if (data->dy != filter->dy) return fail(VAE_E_BADARG, "conv_bwd_pair: data and filter calls of different dy");
  vae_conv_args d = *data, f = *filter;
  d.workspace = f.workspace = workspace;
  d.workspace_bytes = f.workspace_bytes = workspace ? workspace_bytes : 0;
  // the weight gradient rides on the data gradient's conv-GEMM grid when both take the bf16 paths
  PairRider rider;
  memset(&rider, 0, sizeof(rider));
  bool closed = false;
  const bool ride = !querying() && !getenv("VAE_NO_PAIR") && geom_ok(filter, "conv_bwd_pair") && f.dy && f.x && f.dw &&
                    !f.split_k && xf_ok(f.dy_xf, "conv_bwd_pair.dy") && xf_ok(f.x_xf, "conv_bwd_pair.x") &&
                    conv_wg_params(&f, tr, &rider.w, &closed) && (!f.db || closed) && !bwg_ok(rider.w) &&
                    pair_variant(rider.w) >= 0;
  if (ride) pair_rider() = &rider;
  const int rc = tr ? vae_convT2d_bwd_data(&d, stream) : vae_conv2d_bwd_data(&d, stream);
  pair_rider() = nullptr;
  if (rc) return rc;
  if (rider.used) return check_launch("conv_bwd_pair");
  return tr ? vae_convT2d_bwd_filter(&f, stream) : vae_conv2d_bwd_filter(&f, stream);
}

extern "C" int vae_conv_bwd_pair_workspace_size(int32_t kind, const vae_conv_args* data, const vae_conv_args* filter,
                                                size_t* bytes) {
  if (!bytes) return fail(VAE_E_BADARG, "conv_bwd_pair_workspace_size: null bytes");
  if (kind != VAE_LAYER_CONV2D && kind != VAE_LAYER_CONVT2D) return fail(VAE_E_BADARG, "conv_bwd_pair: kind %d", kind);
  size_t a = 0, b = 0;
  const bool tr = kind == VAE_LAYER_CONVT2D;
  int rc = tr ? vae_convT2d_workspace_size(data, VAE_OP_BWD_DATA, &a) : vae_conv2d_workspace_size(data, VAE_OP_BWD_DATA, &a);
  if (rc) return rc;
  rc = tr ? vae_convT2d_workspace_size(filter, VAE_OP_BWD_FILTER, &b) : vae_conv2d_workspace_size(filter, VAE_OP_BWD_FILTER, &b);
  if (rc) return rc;
  *bytes = a > b ? a : b;
  return VAE_OK;
}
