// C-ABI entry point: the weight gradients of several Conv2d / ConvTranspose2d layers in one call
// (the bwd_filter calls of one gradient bucket of the backward, models/vanilla_vae.py:25-75 via
// experiment.py:45-86's loss.backward()).
//
// Why: a layer's weight gradient is off the backward's critical path (only the optimizer reads
// it), and each one alone is a latency-bound launch of 15-30 us at B=64 (profiles/r2_v3_*).
// Launched one per layer they serialise behind the data-gradient chain; here the layers that
// share a tile class run as ONE grouped launch (wg_group_kernel): workgroup b finds its layer by
// the prefix of block counts and runs that layer's body (vae_wgemm.hpp wgemm_body /
// wgemm_taps_body) — every layer's planning (tile, K slices, slab) is exactly that of its own
// call, so the results are those of the calls made one after another.
#include <string.h>

#include <algorithm>
#include <cmath>

#include "vae_launch.hpp"
#include "vae_wgrad.hpp"
#include "vae_wgemm.hpp"

using namespace vae;

namespace {

constexpr int kWg3Max = 10;     // layers of one grouped launch (kernel arguments: 8 KB measured to
                                // launch fine, tools/ubench/kernarg.hip; the group is ~6.5 KB)

// VAE_PROBE builds (tools/wgprobe.py): one record per workgroup {layer << 32 | local item, wall
// start, wall end, XCD, prologue / K-loop / total cycles, HW_ID} in the probe buffer (vae_probe_set)
#ifdef VAE_PROBE
#define WG_PROBE_BEGIN() const unsigned long long wg_w0 = threadIdx.x == 0 ? wall_clock64() : 0; \
  unsigned long long wclk[4] = {__builtin_readcyclecounter(), 0, 0, 0}; unsigned long long* clkp = wclk
#define WG_PROBE_END(layer, lbid, tag) do { \
    unsigned long long* pr_ = gk->probe; \
    const unsigned long long slot_ = blockIdx.x; \
    if (pr_ && threadIdx.x == 0 && slot_ < pr_[1]) { \
      unsigned long long* r_ = pr_ + 8 + slot_ * 8; \
      r_[0] = ((unsigned long long)(layer) << 32) | (unsigned)(lbid); \
      r_[1] = wg_w0; r_[2] = wall_clock64(); r_[3] = (tag); r_[4] = wclk[1] - wclk[0]; r_[5] = wclk[2] - wclk[0]; \
      r_[6] = __builtin_readcyclecounter() - wclk[0]; \
      r_[7] = __builtin_amdgcn_s_getreg((23 << 0) | (0 << 6) | (31 << 11)); \
    } } while (0)
#else
#define WG_PROBE_BEGIN() unsigned long long* clkp = nullptr
#define WG_PROBE_END(layer, lbid, tag) do { } while (0)
#endif

// One launch for every weight gradient of a backward segment.  The work items (layer, K slice,
// output tile) are listed layer by layer, slice-major, and cut into 8 contiguous ranges of equal
// estimated cost, one per XCD: workgroups are dealt round-robin over the XCDs (block b runs on
// XCD b % 8 — speed only, never correctness), so workgroup b runs item xs[b % 8] + b / 8.  An
// XCD then streams a contiguous pixel range of its layers (the shallow layers' slices) or a
// contiguous range of output tiles (the deep layers'), and the tiles and taps that re-read the
// same pixels hit its own L2 instead of the fabric.  No atomics: a layer split into K slices
// writes each slice's partial tile to its slab (plain stores) and wg3_reduce adds the slices in
// slice order; a single-slice layer adds its tile into dW itself — the result does not depend on
// scheduling (deterministic, bit-identical run to run).
constexpr int kWg3Items = 1024;  // work items of one launch (kernel-argument list, 2 bytes each)

struct Wg3Group {
  int n;
  int xs[9];                       // XCD x runs list entries [xs[x], xs[x+1])
  int var[kWg3Max];                // body: 0-3 32 x 32 all-taps, 4-7 64 x 64 per tap, 8-11 64 x 128 per tap
  int tpi[kWg3Max];                // work units (slice, tap, tile) per item, run one after another
  int units[kWg3Max];              // work units of the layer
  WgParams p[kWg3Max];
  unsigned short item[kWg3Items];  // layer << 12 | the layer's work item (slice * tiles + tile)
  unsigned long long* probe;       // VAE_PROBE builds: per-workgroup records (else NULL)
};
static_assert(sizeof(Wg3Group) <= 7680, "kernel argument block");

// pixels per K-step of the 64-wide per-tap bodies (the standalone kernel's 32 halve the MFMA work
// per barrier)
constexpr int kWg3KP = 64;
constexpr int wg3_max(int a, int b) { return a > b ? a : b; }
constexpr int wg3_lds() {
  return wg3_max(wgemm_taps_lds_bytes<32, 32, 3>(),
                 wg3_max(wgemm_lds_bytes<64, 64, kWg3KP>(), wgemm_lds_bytes<64, 128, kWg3KP>()));
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) wg3_kernel(const Wg3Group g) {
  kernarg_prefetch<(sizeof(Wg3Group) < 1024 ? sizeof(Wg3Group) : 1024)>();
  __shared__ __attribute__((aligned(16))) char lds[wg3_lds()];
  // read in place from the kernel-argument segment (scalar loads at a uniform dynamic offset):
  // indexing the by-value parameter with a runtime layer index copies all of it to scratch
  (void)g;
  const Wg3Group* gk = (const Wg3Group*)(const void*)__builtin_amdgcn_kernarg_segment_ptr();
  const int x = (int)(blockIdx.x & 7u), loc = (int)(blockIdx.x >> 3);
  const int e = gk->xs[x] + loc;
  if (e >= gk->xs[x + 1]) return;
  const int it = gk->item[e];
  const int i = __builtin_amdgcn_readfirstlane(it >> 12);
  const int bid = __builtin_amdgcn_readfirstlane((it & 4095) * gk->tpi[i]);
  const int nu = min(gk->tpi[i], gk->units[i] - bid);
  const WgParams& p = gk->p[i];
  WG_PROBE_BEGIN();
  switch (gk->var[i]) {
    case 0: wgemm_taps_body<32, 32, VAE_X_BN_DY, VAE_X_NONE, 3>(p, bid, lds, clkp); break;
    case 1: wgemm_taps_body<32, 32, VAE_X_BN_DY, VAE_X_BN_ACT, 3>(p, bid, lds, clkp); break;
    case 2: wgemm_taps_body<32, 32, VAE_X_NONE, VAE_X_BN_DY, 3>(p, bid, lds, clkp); break;
    case 3: wgemm_taps_body<32, 32, VAE_X_BN_ACT, VAE_X_BN_DY, 3>(p, bid, lds, clkp); break;
    case 4: wgemm_body<64, 64, VAE_X_BN_DY, VAE_X_NONE, kWg3KP>(p, bid, lds, clkp, nu); break;
    case 5: wgemm_body<64, 64, VAE_X_BN_DY, VAE_X_BN_ACT, kWg3KP>(p, bid, lds, clkp, nu); break;
    case 6: wgemm_body<64, 64, VAE_X_NONE, VAE_X_BN_DY, kWg3KP>(p, bid, lds, clkp, nu); break;
    case 7: wgemm_body<64, 64, VAE_X_BN_ACT, VAE_X_BN_DY, kWg3KP>(p, bid, lds, clkp, nu); break;
    case 8: wgemm_body<64, 128, VAE_X_BN_DY, VAE_X_NONE, kWg3KP>(p, bid, lds, clkp, nu); break;
    case 9: wgemm_body<64, 128, VAE_X_BN_DY, VAE_X_BN_ACT, kWg3KP>(p, bid, lds, clkp, nu); break;
    case 10: wgemm_body<64, 128, VAE_X_NONE, VAE_X_BN_DY, kWg3KP>(p, bid, lds, clkp, nu); break;
    default: wgemm_body<64, 128, VAE_X_BN_ACT, VAE_X_BN_DY, kWg3KP>(p, bid, lds, clkp, nu); break;
  }
  WG_PROBE_END(i, bid, x);
}

// dw[e] += Σ_s slab[s][e] for the sliced layers of a launch, slices summed in order (one thread
// per element; consecutive threads read consecutive words of every slice).
struct Wg3Reduce {
  int n;
  long start[kWg3Max + 1];         // element prefix over the sliced layers
  const float* slab[kWg3Max];
  float* dw[kWg3Max];
  int slices[kWg3Max];
};

__global__ void __launch_bounds__(256) wg3_reduce(const Wg3Reduce r) {
  const Wg3Reduce* rk = (const Wg3Reduce*)(const void*)__builtin_amdgcn_kernarg_segment_ptr();
  (void)r;
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= rk->start[rk->n]) return;
  int i = 0;
#pragma unroll
  for (int j = 1; j < kWg3Max; ++j) i = (j < rk->n && e >= rk->start[j]) ? j : i;
  const long o = e - rk->start[i];
  const long cols = rk->start[i + 1] - rk->start[i];
  const float* sl = rk->slab[i] + o;
  const int S = rk->slices[i];
  float acc = 0.f;
  int s = 0;
  for (; s + 8 <= S; s += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = sl[(long)(s + u) * cols];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; s < S; ++s) acc += sl[(long)s * cols];
  rk->dw[i][o] += acc;
}

inline int wg_variant(const WgParams& p) {
  const vae_xform& dy = p.dy_is_v ? p.v_xf : p.u_xf;
  const vae_xform& x = p.dy_is_v ? p.u_xf : p.v_xf;
  if (dy.kind != VAE_X_BN_DY) return -1;
  if (x.kind != VAE_X_NONE && x.kind != VAE_X_BN_ACT) return -1;
  return 2 * p.dy_is_v + (x.kind == VAE_X_BN_ACT ? 1 : 0);
}

// workspace a single call of item i needs (the thread's query state is saved around it)
inline long item_need(int kind, const vae_conv_args* a) {
  WsQuery& q = ws_query();
  const WsQuery saved = q;
  size_t b = 0;
  const int rc = kind == VAE_LAYER_CONVT2D ? vae_convT2d_workspace_size(a, VAE_OP_BWD_FILTER, &b)
                                           : vae_conv2d_workspace_size(a, VAE_OP_BWD_FILTER, &b);
  q = saved;
  return rc ? -1 : (long)((b + 255) / 256 * 256);
}

// A grouped layer before its slices are chosen: body, tiles, K-steps and the estimated time of one
// K-step (us, one workgroup, measured with tools/wgprobe.py on the VanillaVAE B=64 batch: the
// 64-wide per-tap bodies are latency-bound at ~0.6 us per 32-pixel step; the all-taps body holds
// one step in flight and pays about a round trip plus its bytes per 64-pixel step).
struct Wg3Layer {
  int idx;                 // batch item
  WgParams p;
  int var;                 // Wg3Group.var
  int KP;                  // pixels per K-step of the body
  long tiles, steps;       // output tiles per slice; K-steps over all pixels
  double step_us;
  long cols;               // dW elements (M * R * R * jst)
  long slices, tpi;
};

// fixed parts of a work item (us, tools/wgprobe.py): its first round trip (tables + first K-steps,
// queued behind every other workgroup's), a unit's refill when an item runs several, the epilogue
constexpr double kWg3PrologueUs = 6.0, kWg3RefillUs = 2.0, kWg3EpilogueUs = 3.0;
// the epilogue of a unit that writes its tile into dW without reading it back (a deferred layer's
// single slice, WgParams.own == 2): the store only (tools/wgprobe.py: the deep layers' items ran
// 27-30 us against the 37-40 us of the rest with the read-modify-write cost in the plan)
constexpr double kWg3StoreEpilogueUs = 1.5;

inline bool wg3_layer(const WgParams& w0, int idx, Wg3Layer* L) {
  const int var = wg_variant(w0);
  if (var < 0 || w0.R != 3) return false;
  const int mn = w0.M < w0.J ? w0.M : w0.J;
  WgParams p = w0;
  p.fd_wu = make_fastdiv(p.wu);
  p.fd_hu = make_fastdiv(p.hu);
  p.fd_r = make_fastdiv(p.R);
  const long npix = (long)p.n * p.hu * p.wu;
  p.u_bytes = (uint32_t)(npix * p.M * 2);
  p.v_bytes = (uint32_t)((long)p.n * p.hv * p.wv * p.J * 2);
  const bool du = p.u_xf.kind == VAE_X_BN_DY, dv = p.v_xf.kind == VAE_X_BN_DY;
  L->idx = idx;
  const int jst = p.jst > 0 ? p.jst : p.J;
  L->cols = (long)p.M * p.R * p.R * jst;
  if (mn < 64) {                                       // 32 x 32 tiles, all 9 taps per workgroup
    L->var = var;
    L->KP = wgt_kp<32, 32>();
    L->tiles = (long)((p.M + 31) / 32) * ((p.J + 31) / 32);
    const int cu = p.M < 32 ? p.M : 32, cv = p.J < 32 ? p.J : 32;
    const double bytes = (double)L->KP * 2.0 * (cu * (du ? 2 : 1) + 9.0 * cv * (dv ? 2 : 1));
    L->step_us = 1.2 + bytes / 51200.0;
  } else if (p.J >= 128) {                             // 64 x 128 tiles, one tap per workgroup
    L->var = 8 + var;
    L->KP = kWg3KP;
    L->tiles = (long)((p.M + 63) / 64) * ((p.J + 127) / 128) * p.R * p.R;
    L->step_us = 0.95 * kWg3KP / 32 * 0.75;
  } else {                                             // 64 x 64 tiles, one tap per workgroup
    L->var = 4 + var;
    L->KP = kWg3KP;
    L->tiles = (long)((p.M + 63) / 64) * ((p.J + 63) / 64) * p.R * p.R;
    L->step_us = 0.65 * kWg3KP / 32 * 0.75;
  }
  L->steps = (npix + L->KP - 1) / L->KP;
  L->p = p;
  return true;
}

}  // namespace

extern "C" int vae_conv_bwd_filter_batch(int32_t n, const int32_t* kinds, const vae_conv_args* const* items,
                                         void* workspace, int64_t workspace_bytes, void* stream) {
  if (n < 0 || (n > 0 && (!kinds || !items))) return fail(VAE_E_BADARG, "conv_bwd_filter_batch: null arrays");
  if (n > 64) return fail(VAE_E_BADARG, "conv_bwd_filter_batch: %d items > 64", n);
  hipStream_t st = (hipStream_t)stream;
  // which items group: bf16 3x3 weight gradients with a BN-backward dy (the VanillaVAE family and
  // the Autoencoder); the rest run as their own calls, each with a workspace region of its own
  Wg3Layer lay[kWg3Max];
  int nl = 0;
  bool grouped[64];
  for (int i = 0; i < n; ++i) {
    const vae_conv_args* a = items[i];
    if (!a || (kinds[i] != VAE_LAYER_CONV2D && kinds[i] != VAE_LAYER_CONVT2D))
      return fail(VAE_E_BADARG, "conv_bwd_filter_batch: item %d", i);
    grouped[i] = false;
    WgParams w;
    bool closed = false;
    const bool valid = geom_ok(a, "conv_bwd_filter_batch") && a->dy && a->x && a->dw &&
                       xf_ok(a->dy_xf, "conv_bwd_filter_batch.dy") && xf_ok(a->x_xf, "conv_bwd_filter_batch.x");
    if (nl < kWg3Max && valid && conv_wg_params(a, kinds[i] == VAE_LAYER_CONVT2D, &w, &closed) && (!a->db || closed)) {
      const bool bu = w.u_xf.kind == VAE_X_BN_ACT || w.u_xf.kind == VAE_X_BN_DY;
      const bool bv = w.v_xf.kind == VAE_X_BN_ACT || w.v_xf.kind == VAE_X_BN_DY;
      const long tab = 4l * ((bu ? 3 * tab_stride(w.u_xf.channels) : 0) + (bv ? 3 * tab_stride(w.v_xf.channels) : 0));
      if (tab + wg3_lds() <= 80 * 1024 && wg3_layer(w, i, &lay[nl])) {
        grouped[i] = true;
        ++nl;
      }
    }
  }
  // workspace: the standalone items' regions, then the grouped layers' slabs
  long off[64], total = 0;
  for (int i = 0; i < n; ++i) {
    off[i] = total;
    if (grouped[i]) continue;
    const long need = item_need(kinds[i], items[i]);
    if (need < 0) return VAE_E_BADARG;                        // (the item's own error message)
    total += need;
  }
  // K slices and units per item: the kernel holds two workgroups per CU (512 slots), so the plan
  // aims at one round of at most 512 items of about equal time T: a layer whose unit (one K slice
  // of one tile) takes longer than T is cut into more K slices; a layer of many short units (the
  // deep layers: hundreds of output tiles over few pixels) runs several units per item.  T is the
  // smallest time for which the items fit the round.
  long slab_off[kWg3Max];
  bool defer_of[kWg3Max];
  for (int l = 0; l < nl; ++l) defer_of[l] = items[lay[l].idx]->defer_reduce != 0;
  const long total0 = total;
  auto plan_at = [&](double T) -> long {
    total = total0;
    long items = 0;
    for (int l = 0; l < nl; ++l) {
      Wg3Layer& L = lay[l];
      const double body = T - kWg3PrologueUs - kWg3EpilogueUs;
      long sl = (long)ceil(L.steps * L.step_us / (body > 0.5 ? body : 0.5));
      if (sl < 1) sl = 1;
      if (sl > L.steps) sl = L.steps;
      const long ksteps = (L.steps + sl - 1) / sl;
      L.p.kper = (int)(ksteps * L.KP);
      const long npix = (long)L.p.n * L.p.hu * L.p.wu;
      L.slices = (npix + L.p.kper - 1) / L.p.kper;
      L.tpi = 1;
      if (L.slices == 1) {
        const double unit = ksteps * L.step_us + (defer_of[l] ? kWg3StoreEpilogueUs : kWg3EpilogueUs);
        long t = (long)((T - kWg3PrologueUs + kWg3RefillUs) / (unit + kWg3RefillUs));
        L.tpi = t < 1 ? 1 : (t > L.tiles ? L.tiles : t);
      }
      L.p.slab = nullptr;
      L.p.slab_ld = L.cols;
      // a deferred layer (vae_conv_args.defer_reduce): its K slices stay in the slab for the
      // caller's reduction, which writes dW; with one slice the epilogue writes dW itself, no
      // read-modify-write (the reduction would read back exactly that slice)
      const bool slab = L.slices > 1;
      L.p.own = slab ? 0 : (defer_of[l] ? 2 : 1);
      slab_off[l] = total;
      if (slab) total += (L.slices * L.cols * 4 + 255) / 256 * 256;
      const long li = (L.slices * L.tiles + L.tpi - 1) / L.tpi;
      items += li > 4096 ? (long)kWg3Items + 1 : li;
    }
    return items;
  };
  {
    double lo = 1.0, hi = 1.0;
    while (plan_at(hi) > 2 * kCUs && hi < 1e6) hi *= 2.0;
    for (int it = 0; it < 24; ++it) {
      const double mid = 0.5 * (lo + hi);
      if (plan_at(mid) > 2 * kCUs) lo = mid; else hi = mid;
    }
    if (nl && plan_at(hi) > kWg3Items) return fail(VAE_E_UNSUPPORTED, "conv_bwd_filter_batch: work items");
  }
  if (!ws_fits(total, workspace ? workspace_bytes : 0, "conv_bwd_filter_batch")) return VAE_E_BADARG;
  auto region = [&](long o) -> void* { return querying() ? workspace : static_cast<char*>(workspace) + o; };
  for (int i = 0; i < n; ++i) {
    if (grouped[i]) continue;
    vae_conv_args c = *items[i];
    const long need = item_need(kinds[i], items[i]);
    c.workspace = need > 0 ? region(off[i]) : nullptr;
    c.workspace_bytes = need;
    const int rc = kinds[i] == VAE_LAYER_CONVT2D ? vae_convT2d_bwd_filter(&c, stream) : vae_conv2d_bwd_filter(&c, stream);
    if (rc) return rc;
  }
  if (nl == 0) return VAE_OK;
  // the item list: layers in order, each layer's items slice-major, cut into 8 runs of equal
  // estimated time (XCD x takes run x: contiguous pixel ranges / tile ranges of its layers); within
  // a run the longer items go first (the XCD dispatches its workgroups in list order, so the short
  // items fill the slots the long ones leave)
  Wg3Group g;
  memset(&g, 0, sizeof(g));
#ifdef VAE_PROBE
  g.probe = vae_probe_buffer();
#endif
  g.n = nl;
  struct It { unsigned short code; float us; };
  static thread_local It list[kWg3Items];
  double total_us = 0.0;
  int ni = 0;
  for (int l = 0; l < nl; ++l) {
    Wg3Layer& L = lay[l];
    if (L.slices > 1) L.p.slab = static_cast<float*>(region(slab_off[l]));
    g.p[l] = L.p;
    g.var[l] = L.var;
    g.tpi[l] = (int)L.tpi;
    g.units[l] = (int)(L.slices * L.tiles);
    const long npix = (long)L.p.n * L.p.hu * L.p.wu;
    const long nitems = (L.slices * L.tiles + L.tpi - 1) / L.tpi;
    for (long it = 0; it < nitems; ++it) {
      double us = kWg3PrologueUs;
      for (long u = it * L.tpi; u < (it + 1) * L.tpi && u < L.slices * L.tiles; ++u) {
        const long sl = u / L.tiles;
        const long px = (sl + 1) * L.p.kper < npix ? L.p.kper : npix - sl * L.p.kper;
        const double epi = (L.slices == 1 && defer_of[l]) ? kWg3StoreEpilogueUs : kWg3EpilogueUs;
        us += (double)(px + L.KP - 1) / L.KP * L.step_us + epi + (u > it * L.tpi ? kWg3RefillUs : 0.0);
      }
      list[ni++] = It{(unsigned short)((l << 12) | (int)it), (float)us};
      total_us += us;
    }
  }
  {
    // (an XCD holds 64 workgroups at once: a run of more items would start a second round there)
    constexpr int kPerXcd = 2 * kCUs / 8;
    int e = 0;
    for (int x = 0; x < 8; ++x) {
      g.xs[x] = e;
      double cum = 0.0;
      int cnt = 0;
      while (e < ni && cnt < kPerXcd && (x == 7 || cum < total_us / 8.0 || ni - e > (7 - x) * kPerXcd)) {
        cum += list[e++].us;
        ++cnt;
      }
    }
    g.xs[8] = ni;
    if (e < ni) return fail(VAE_E_UNSUPPORTED, "conv_bwd_filter_batch: %d items over 8 XCD runs", ni);
    for (int r = 0; r < 8; ++r)
      std::stable_sort(list + g.xs[r], list + g.xs[r + 1], [](const It& a, const It& b) { return a.us > b.us; });
    for (int e = 0; e < ni; ++e) g.item[e] = list[e].code;
  }
  int per = 0;
  for (int x = 0; x < 8; ++x) per = g.xs[x + 1] - g.xs[x] > per ? g.xs[x + 1] - g.xs[x] : per;
  size_t lds = 0;
  for (int l = 0; l < nl; ++l) {
    const WgParams& w = g.p[l];
    const bool bu = w.u_xf.kind == VAE_X_BN_ACT || w.u_xf.kind == VAE_X_BN_DY;
    const bool bv = w.v_xf.kind == VAE_X_BN_ACT || w.v_xf.kind == VAE_X_BN_DY;
    const size_t t = (size_t)((bu ? 3 * tab_stride(w.u_xf.channels) : 0) + (bv ? 3 * tab_stride(w.v_xf.channels) : 0)) * 4;
    lds = t > lds ? t : lds;
  }
  VAE_LAUNCH(wg3_kernel, dim3((unsigned)(8 * per)), dim3(256), lds, st, g);
  if (int rc = check_launch("wg3")) return rc;
  Wg3Reduce r;
  memset(&r, 0, sizeof(r));
  for (int l = 0; l < nl; ++l) {
    if (defer_of[l]) {
      // the slices stay for vae_adam_step_ex; one slice: written whole by this call (rows 0)
      const bool sl = lay[l].slices > 1;
      if (!defer_slab(g.p[l].dw, lay[l].cols, sl ? g.p[l].slab : nullptr, sl ? (int)lay[l].slices : 0, lay[l].cols))
        return VAE_E_UNSUPPORTED;
      continue;
    }
    if (lay[l].slices <= 1) continue;
    r.slab[r.n] = g.p[l].slab;
    r.dw[r.n] = g.p[l].dw;
    r.slices[r.n] = (int)lay[l].slices;
    r.start[r.n + 1] = r.start[r.n] + lay[l].cols;
    r.n++;
  }
  if (r.n > 0) {
    VAE_LAUNCH(wg3_reduce, dim3((unsigned)((r.start[r.n] + 255) / 256)), dim3(256), 0, st, r);
    if (int rc = check_launch("wg3_reduce")) return rc;
  }
  return VAE_OK;
}

extern "C" int vae_conv_bwd_filter_batch_workspace_size(int32_t n, const int32_t* kinds, const vae_conv_args* const* items,
                                                        size_t* bytes) {
  if (!bytes) return fail(VAE_E_BADARG, "conv_bwd_filter_batch_workspace_size: null bytes");
  WsQuery& q = ws_query();
  q.on = 1;
  q.need = 0;
  const int rc = vae_conv_bwd_filter_batch(n, kinds, items, reinterpret_cast<void*>(uintptr_t(1) << 40),
                                           int64_t(1) << 50, nullptr);
  *bytes = rc ? 0 : (size_t)q.need;
  q.on = 0;
  q.need = 0;
  return rc;
}
