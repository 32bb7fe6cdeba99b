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

#include "vae_launch.hpp"
#include "vae_wgrad.hpp"
#include "vae_wgemm.hpp"

using namespace vae;

namespace {

constexpr int kWgGroupMax = 6;

// XCD-aware order within each layer of a grouped launch: workgroups are dealt round-robin over the
// 8 XCDs (block b runs on XCD b % 8; speed only, never correctness), so a layer's local index is
// remapped to give each XCD a contiguous range of that layer — its K slices (pixel ranges,
// slice-outermost) then share an L2 instead of every XCD fetching every layer's operands from the
// fabric (VanillaVAE mixed launch: 86 -> 69 MB of FETCH/WRITE traffic at the same 49.5-50 us,
// r4_v5 / r4n PMC).  Per layer, not over the whole grid: a grid-wide remap gave whole
// (unequal-cost) layers to single XCDs and measured 4.7 us slower despite 35 MB less traffic (r4m).
// Mixed launch only: the all-taps 32x32 group measured slower with it (39.6 -> 45.2 us).
__device__ __forceinline__ int wg_xcd_order(int b, int nb) {
  const int q = nb >> 3, r = nb & 7, x = b & 7, loc = b >> 3;
  return x * q + min(x, r) + loc;
}

struct WgGroup {
  int n;
  int start[kWgGroupMax + 1];      // first workgroup of each layer; start[n] = total
  int var[kWgGroupMax];            // body variant: 2 * dy_is_v + (x operand BatchNorm+LeakyReLU)
  WgParams p[kWgGroupMax];
};
static_assert(sizeof(WgGroup) <= 3584, "kernel argument block");

template <int T, int RR, int XU, int XV>
__device__ __forceinline__ void wg_group_body(const WgParams& p, int bid, char* lds) {
  if constexpr (RR > 0) wgemm_taps_body<T, T, XU, XV, RR>(p, bid, lds);
  else wgemm_body<T, T, XU, XV>(p, bid, lds);
}

template <int T, int RR> constexpr int wg_group_lds() {
  if constexpr (RR > 0) return wgemm_taps_lds_bytes<T, T, RR>();
  else return wgemm_lds_bytes<T, T>();
}

// The dy operand carries the BatchNorm backward (BN_DY), the other one is the layer input with
// no transform or its BatchNorm+LeakyReLU (the VanillaVAE family and the Autoencoder).
template <int T, int RR>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(T >= 128 ? 2 : 1)))
wg_group_kernel(const WgGroup g) {
  __shared__ __attribute__((aligned(16))) char lds[wg_group_lds<T, RR>()];
  // The group is read in place from the kernel-argument segment (scalar loads at a uniform
  // dynamic offset): indexing the by-value parameter with a runtime layer index makes the
  // compiler copy all of it to scratch first (2.5 KB per workgroup, measured 10x slower).
  (void)g;
  const WgGroup* gk = (const WgGroup*)(const void*)__builtin_amdgcn_kernarg_segment_ptr();
  const int b = (int)blockIdx.x;
  const int n = gk->n;
  int i = 0;
#pragma unroll
  for (int j = 1; j < kWgGroupMax; ++j) i = (j < n && b >= gk->start[j]) ? j : i;
  i = __builtin_amdgcn_readfirstlane(i);
  const int bid = b - gk->start[i];   // (the per-layer XCD order measured 39.6 -> 45.2 us here, r4n)
  const WgParams& p = gk->p[i];
  switch (gk->var[i]) {
    case 0: wg_group_body<T, RR, VAE_X_BN_DY, VAE_X_NONE>(p, bid, lds); break;
    case 1: wg_group_body<T, RR, VAE_X_BN_DY, VAE_X_BN_ACT>(p, bid, lds); break;
    case 2: wg_group_body<T, RR, VAE_X_NONE, VAE_X_BN_DY>(p, bid, lds); break;
    default: wg_group_body<T, RR, VAE_X_BN_ACT, VAE_X_BN_DY>(p, bid, lds); break;
  }
}

// The 64 x 64 and 128 x 128 classes in ONE grid (per layer: var[i] = 4 * (tile == 128) + variant):
// launched one after the other, each class ran a round of one workgroup per CU on its own (the
// VanillaVAE's 25 + 30 us, profiles/r4_v1_kstats.json); in one grid they share the round.
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) wg_group_mixed_kernel(const WgGroup g) {
  __shared__ __attribute__((aligned(16))) char lds[wgemm_lds_bytes<128, 128>()];
  (void)g;
  const WgGroup* gk = (const WgGroup*)(const void*)__builtin_amdgcn_kernarg_segment_ptr();
  const int b = (int)blockIdx.x;
  const int n = gk->n;
  int i = 0;
#pragma unroll
  for (int j = 1; j < kWgGroupMax; ++j) i = (j < n && b >= gk->start[j]) ? j : i;
  i = __builtin_amdgcn_readfirstlane(i);
  const int bid = wg_xcd_order(b - gk->start[i], gk->start[i + 1] - gk->start[i]);
  const WgParams& p = gk->p[i];
  switch (gk->var[i]) {
    case 0: wgemm_body<64, 64, VAE_X_BN_DY, VAE_X_NONE>(p, bid, lds); break;
    case 1: wgemm_body<64, 64, VAE_X_BN_DY, VAE_X_BN_ACT>(p, bid, lds); break;
    case 2: wgemm_body<64, 64, VAE_X_NONE, VAE_X_BN_DY>(p, bid, lds); break;
    case 3: wgemm_body<64, 64, VAE_X_BN_ACT, VAE_X_BN_DY>(p, bid, lds); break;
    case 4: wgemm_body<128, 128, VAE_X_BN_DY, VAE_X_NONE>(p, bid, lds); break;
    case 5: wgemm_body<128, 128, VAE_X_BN_DY, VAE_X_BN_ACT>(p, bid, lds); break;
    case 6: wgemm_body<128, 128, VAE_X_NONE, VAE_X_BN_DY>(p, bid, lds); break;
    default: wgemm_body<128, 128, VAE_X_BN_ACT, VAE_X_BN_DY>(p, bid, lds); break;
  }
}

// group classes: 0 = 32 x 32 tiles with all 3x3 taps per workgroup, 1 = 64 x 64, 2 = 128 x 128
constexpr int kClasses = 3;
inline int wg_class(const WgPlan& w) {
  if (w.T == 32) return w.taps == 3 ? 0 : -1;
  return w.taps ? -1 : (w.T == 64 ? 1 : 2);
}

inline int wg_variant(const WgParams& p) {
  const vae_xform& dy = p.dy_is_v ? p.v_xf : p.u_xf;
  const vae_xform& x = p.dy_is_v ? p.u_xf : p.v_xf;
  if (dy.kind != VAE_X_BN_DY) return -1;
  if (x.kind != VAE_X_NONE && x.kind != VAE_X_BN_ACT) return -1;
  return 2 * p.dy_is_v + (x.kind == VAE_X_BN_ACT ? 1 : 0);
}

inline int group_launch(int cls, const WgGroup& g, size_t lds, hipStream_t st) {
  const dim3 grid((unsigned)g.start[g.n]);
  switch (cls) {
    case 0: VAE_LAUNCH((wg_group_kernel<32, 3>), grid, dim3(256), lds, st, g); break;
    case 1: VAE_LAUNCH((wg_group_kernel<64, 0>), grid, dim3(256), lds, st, g); break;
    default: VAE_LAUNCH((wg_group_kernel<128, 0>), grid, dim3(256), lds, st, g); break;
  }
  return check_launch("wg_group");
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

}  // namespace

extern "C" int vae_conv_bwd_filter_batch(int32_t n, const int32_t* kinds, const vae_conv_args* const* items,
                                         void* workspace, int64_t workspace_bytes, void* stream) {
  if (n < 0 || (n > 0 && (!kinds || !items))) return fail(VAE_E_BADARG, "conv_bwd_filter_batch: null arrays");
  hipStream_t st = (hipStream_t)stream;
  // every item's own workspace, back to back (the grouped layers run concurrently)
  long total = 0;
  long off[64];
  if (n > 64) return fail(VAE_E_BADARG, "conv_bwd_filter_batch: %d items > 64", n);
  for (int i = 0; i < n; ++i) {
    const vae_conv_args* a = items[i];
    if (!a || (kinds[i] != VAE_LAYER_CONV2D && kinds[i] != VAE_LAYER_CONVT2D))
      return fail(VAE_E_BADARG, "conv_bwd_filter_batch: item %d", i);
    const long need = item_need(kinds[i], a);
    if (need < 0) return VAE_E_BADARG;                        // (the item's own error message)
    off[i] = total;
    total += need;
  }
  if (!ws_fits(total, workspace ? workspace_bytes : 0, "conv_bwd_filter_batch")) return VAE_E_BADARG;
  auto region = [&](int i) -> void* {
    const long need = (i + 1 < n ? off[i + 1] : total) - off[i];
    return need > 0 ? static_cast<char*>(workspace) + off[i] : nullptr;
  };
  auto region_bytes = [&](int i) -> long { return (i + 1 < n ? off[i + 1] : total) - off[i]; };

  WgPlan plans[64];
  int cls[64];
  for (int i = 0; i < n; ++i) {
    const vae_conv_args* a = items[i];
    const bool tr = kinds[i] == VAE_LAYER_CONVT2D;
    cls[i] = -1;
    WgParams w;
    bool closed = false;
    const bool valid = geom_ok(a, "conv_bwd_filter_batch") && a->dy && a->x && a->dw &&
                       xf_ok(a->dy_xf, "conv_bwd_filter_batch.dy") && xf_ok(a->x_xf, "conv_bwd_filter_batch.x");
    if (valid && conv_wg_params(a, tr, &w, &closed) && (!a->db || closed) && wg_variant(w) >= 0) {
      if (int rc = wg2_plan(w, querying() ? workspace : region(i), region_bytes(i), &plans[i])) return rc;
      cls[i] = wg_class(plans[i]);
    }
    if (cls[i] < 0) {
      // not groupable: the call on its own (validation and error messages included)
      vae_conv_args c = *a;
      c.workspace = querying() ? workspace : region(i);
      c.workspace_bytes = region_bytes(i);
      const int rc = tr ? vae_convT2d_bwd_filter(&c, stream) : vae_conv2d_bwd_filter(&c, stream);
      if (rc) return rc;
    }
  }
  // Grouped 64 x 64 / 128 x 128 layers (deep, few pixels, large dW): their K slices were sized
  // for ~2 workgroups per CU each, and every slice adds its whole dW tile with fp32 atomics (the
  // 3x3 128-channel layers: 8 slices x 1.2 MB).  In a group the layers fill the chip together, so
  // each takes its share of one round of workgroups (one per CU), in proportion to its MACs:
  // fewer slices, and a single slice accumulates with plain stores (WgParams.own).
  static const int group_slots = tune_env("VAE_WG_GROUP_SLOTS", kCUs);
  // the 32 x 32 all-taps class (wide, few-channel layers: thousands of pixels per dW element)
  // gets its own round (measured, VanillaVAE B=64: 0 = each layer's standalone split 127 us for
  // the batch, 256 -> 103 us, 512 -> 107, 768 -> 126); VAE_WG_GROUP_SLOTS0=0 keeps the
  // standalone plans
  static const int group_slots0 = tune_env("VAE_WG_GROUP_SLOTS0", kCUs);
  // When a class's output tiles alone exceed that round (the Autoencoder's 1024-2048-channel
  // layers: thousands of 128 x 128 tiles), the round-share would leave the long-K layers (its
  // 64 x 64-pixel ConvT: 65536 pixels, 9 tiles) a handful of workgroups each running hundreds of
  // K-steps behind everything else; there the K slices are sized instead so that every workgroup
  // of the class runs about the same number of K-steps (the class's work over its tile count,
  // >= 16 steps of 32 pixels).
  // VAE_WG_SHARE=steps: shares in proportion to tile-steps (output tiles x 32-pixel K-steps)
  // instead of MACs.  Measured slower (VanillaVAE B=64: 0.5498 vs 0.5416 ms/step, the batch 102.8
  // vs 94 us): the first conv's K-steps (8 of its 32 tile columns real) cost a quarter of its
  // class-mates', so the MAC shares were the balanced ones.
  static const bool share_macs = !(getenv("VAE_WG_SHARE") && !strcmp(getenv("VAE_WG_SHARE"), "steps"));
  for (int c = group_slots0 > 0 ? 0 : 1; c < kClasses; ++c) {
    const int gs = c == 0 ? group_slots0 : group_slots;
    double macs = 0.0;
    long tiles_sum = 0, work = 0;
    for (int i = 0; i < n; ++i)
      if (cls[i] == c) {
        macs += (double)plans[i].cols * ((double)plans[i].p.n * plans[i].p.hu * plans[i].p.wu);
        const long tiles = (long)plans[i].blocks / (plans[i].split > 0 ? plans[i].split : 1);
        const long ks = ((long)plans[i].p.n * plans[i].p.hu * plans[i].p.wu + 31) / 32;
        tiles_sum += tiles;
        work += tiles * ks;
      }
    if (macs <= 0.0) continue;
    const bool balance = c > 0 && tiles_sum > gs;
    long kt = balance ? (work + tiles_sum - 1) / tiles_sum : 0;
    if (kt < 16) kt = 16;
    for (int i = 0; i < n; ++i) {
      if (cls[i] != c) continue;
      const double m = (double)plans[i].cols * ((double)plans[i].p.n * plans[i].p.hu * plans[i].p.wu);
      long slots = (long)(gs * m / macs + 0.5);
      if (!share_macs && work > 0) {
        const long tiles = (long)plans[i].blocks / (plans[i].split > 0 ? plans[i].split : 1);
        const long ks = ((long)plans[i].p.n * plans[i].p.hu * plans[i].p.wu + 31) / 32;
        slots = (long)((double)gs * (double)(tiles * ks) / (double)work + 0.5);
      }
      if (balance) {
        const long tiles = (long)plans[i].blocks / (plans[i].split > 0 ? plans[i].split : 1);
        const long ks = ((long)plans[i].p.n * plans[i].p.hu * plans[i].p.wu + 31) / 32;
        slots = tiles * ((ks + kt - 1) / kt);
      }
      if (slots < 1) slots = 1;
      WgParams w = plans[i].p;
      w.slab = nullptr;
      // (balanced slices add into dw with atomics: their counts were not in the item's workspace)
      void* wsi = balance ? nullptr : (querying() ? workspace : region(i));
      if (int rc = wg2_plan(w, wsi, balance ? 0 : region_bytes(i), &plans[i], slots)) return rc;
      if (wg_class(plans[i]) != c) return fail(VAE_E_UNSUPPORTED, "conv_bwd_filter_batch: replanned class");
    }
  }
  // one launch per tile class (chunks of kWgGroupMax layers); classes 1 and 2 in one grid when
  // their layers fit one group (VAE_WG_MIXED=0: a launch each)
  static const bool mixed_ok = !(getenv("VAE_WG_MIXED") && !strcmp(getenv("VAE_WG_MIXED"), "0"));
  int n12 = 0;
  for (int i = 0; i < n; ++i) n12 += (cls[i] == 1 || cls[i] == 2) ? 1 : 0;
  const bool mixed = mixed_ok && n12 <= kWgGroupMax && n12 > 0;
  for (int c = 0; c < kClasses; ++c) {
    if (mixed && c == 2) continue;                       // (launched with class 1)
    WgGroup g;
    memset(&g, 0, sizeof(g));
    size_t lds = 0;
    for (int i = 0; i <= n; ++i) {
      const bool take = i < n && (cls[i] == c || (mixed && c == 1 && cls[i] == 2));
      if (take) {
        const WgPlan& w = plans[i];
        g.p[g.n] = w.p;
        g.var[g.n] = wg_variant(w.p) + (mixed && cls[i] == 2 ? 4 : 0);
        g.start[g.n + 1] = g.start[g.n] + (int)w.blocks;
        g.n++;
        const bool bu = w.p.u_xf.kind == VAE_X_BN_ACT || w.p.u_xf.kind == VAE_X_BN_DY;
        const bool bv = w.p.v_xf.kind == VAE_X_BN_ACT || w.p.v_xf.kind == VAE_X_BN_DY;
        const size_t l = (size_t)((bu ? 3 * tab_stride(w.p.u_xf.channels) : 0) +
                                  (bv ? 3 * tab_stride(w.p.v_xf.channels) : 0)) * 4;
        lds = l > lds ? l : lds;
      }
      if (g.n > 0 && (g.n == kWgGroupMax || i == n)) {
        if (mixed && c == 1) {
          VAE_LAUNCH(wg_group_mixed_kernel, dim3((unsigned)g.start[g.n]), dim3(256), lds, st, g);
          if (int rc = check_launch("wg_group_mixed")) return rc;
        } else if (int rc = group_launch(c, g, lds, st)) {
          return rc;
        }
        memset(&g, 0, sizeof(g));
        lds = 0;
      }
    }
  }
  for (int i = 0; i < n; ++i)
    if (cls[i] >= 0)
      if (int rc = wg2_reduce(plans[i], st)) return rc;
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
