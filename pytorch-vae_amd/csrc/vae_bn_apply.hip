// Materialised per-channel transforms (vaehip.h vae_bn_apply): out = xf(x) as a bf16 tensor of the
// same [rows][channels] shape — lrelu(BN(y)) of a forward activation, or the BatchNorm-backward
// gradient dy = A g + B y + C — written once per layer so the large transform-free GEMMs
// (vae_bgemm.hip) and weight gradients read plain operands (models/autoencoder.py:16-86 widths;
// the BatchNorm2d + LeakyReLU of vanilla_vae.py:30-31 / :56-57).
//
// The other duties of the first consumer of a BatchNorm go with it: the forward form updates the
// running statistics (first workgroup), the backward form publishes dL/dgamma, dL/dbeta and the
// closed-form bias gradient of the conv feeding the BatchNorm (first workgroup), as the
// weight-gradient kernels do when they apply the transform themselves.
//
// Streaming layout: 16-byte chunks (8 channels), a grid-stride loop with four chunks in flight per
// thread; the per-channel table is built once per workgroup in LDS (tab_fill: a copy of a
// vae_bn_finalize table, or the reduction of the producer's replicated statistics).
#include "vae_igemm.hpp"

namespace vae {
namespace {

constexpr int BA_T = 256, BA_UNROLL = 4;

struct BnApply {
  long chunks;           // rows * channels / 8
  int C;
  const __bf16* x;
  vae_xform xf;
  float* db;
  __bf16* out;
};

__device__ __forceinline__ float lo16(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi16(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

__global__ void __launch_bounds__(BA_T) bn_apply_kernel(const BnApply q) {
  kernarg_prefetch<(sizeof(BnApply) < 1024 ? sizeof(BnApply) : 1024)>();
  extern __shared__ float tab[];                    // [3][tab_stride(C)] + scratch [1024]
  const int ts = tab_stride(q.C);
  const int kind = q.xf.kind;
  const bool bn = kind == VAE_X_BN_ACT || kind == VAE_X_BN_DY;
  const Tab t{tab, tab + ts, tab + 2 * ts, nullptr, nullptr};
  if (bn) tab_fill(q.xf, t, false, blockIdx.x == 0 && kind == VAE_X_BN_ACT, tab + 3 * ts);
  if (kind == VAE_X_BN_DY && blockIdx.x == 0 && (q.db || q.xf.dgamma_out || q.xf.dbeta_out)) closed_form_db(q.xf, q.db);
  __syncthreads();
  const uint4* x = reinterpret_cast<const uint4*>(q.x);
  const uint4* y = reinterpret_cast<const uint4*>(q.xf.aux);
  uint4* o = reinterpret_cast<uint4*>(q.out);
  const int cg = q.C / 8;                            // chunks per row
  const long stride = (long)gridDim.x * BA_T;
  for (long i0 = (long)blockIdx.x * BA_T + threadIdx.x; i0 < q.chunks; i0 += stride * BA_UNROLL) {
    uint4 v[BA_UNROLL], w[BA_UNROLL];
#pragma unroll
    for (int u = 0; u < BA_UNROLL; ++u) {
      const long i = i0 + u * stride;
      v[u] = i < q.chunks ? x[i] : uint4{0u, 0u, 0u, 0u};
      w[u] = (kind == VAE_X_BN_DY && i < q.chunks) ? y[i] : uint4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < BA_UNROLL; ++u) {
      const long i = i0 + u * stride;
      if (i >= q.chunks) break;
      const int c0 = (int)(i % cg) * 8;
      const uint32_t a[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
      const uint32_t b[4] = {w[u].x, w[u].y, w[u].z, w[u].w};
      uint32_t r[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float f0 = lo16(a[e]), f1 = hi16(a[e]);
        const int c = c0 + 2 * e;
        if (kind == VAE_X_BN_ACT) {
          f0 = fmaf(f0, t.a[c], t.b[c]);
          f1 = fmaf(f1, t.a[c + 1], t.b[c + 1]);
        } else if (kind == VAE_X_BN_DY) {
          f0 = fmaf(t.a[c], f0, fmaf(t.b[c], lo16(b[e]), t.c[c]));
          f1 = fmaf(t.a[c + 1], f1, fmaf(t.b[c + 1], hi16(b[e]), t.c[c + 1]));
        }
        if (kind == VAE_X_ACT || kind == VAE_X_BN_ACT) {
          f0 = lrelu(f0, q.xf.slope);
          f1 = lrelu(f1, q.xf.slope);
        }
        bf16x2 h;
        h[0] = (__bf16)f0;
        h[1] = (__bf16)f1;
        r[e] = *reinterpret_cast<uint32_t*>(&h);
      }
      o[i] = uint4{r[0], r[1], r[2], r[3]};
    }
  }
}

}  // namespace
}  // namespace vae

using namespace vae;

extern "C" int vae_bn_apply(const vae_bn_apply_args* a, void* stream) {
  if (!a || !a->x || !a->out || a->rows <= 0 || a->channels <= 0) return fail(VAE_E_BADARG, "bn_apply: args");
  if (a->dtype != VAE_BF16) return fail(VAE_E_BADDTYPE, "bn_apply: bf16 only");
  if (a->channels % 8 || ((uintptr_t)a->x & 15) || ((uintptr_t)a->out & 15))
    return fail(VAE_E_UNSUPPORTED, "bn_apply: channels %% 8 and 16-byte aligned tensors", a->channels);
  const vae_xform& x = a->xf;
  if (x.kind < VAE_X_ACT || x.kind > VAE_X_BN_DY) return fail(VAE_E_BADARG, "bn_apply: transform kind %d", x.kind);
  if (x.kind == VAE_X_BN_ACT || x.kind == VAE_X_BN_DY) {
    if (x.channels != a->channels) return fail(VAE_E_BADARG, "bn_apply: transform of %d channels on %d", x.channels, a->channels);
    if (!x.gamma || !x.beta || !x.sum || !x.sumsq || x.count <= 0.f) return fail(VAE_E_BADARG, "bn_apply: BatchNorm statistics");
    if (x.channels > MAXC) return fail(VAE_E_UNSUPPORTED, "bn_apply: %d channels > %d", x.channels, MAXC);
  }
  if (x.kind == VAE_X_BN_DY && (!x.aux || ((uintptr_t)x.aux & 15) || !x.dgamma || !x.dbeta))
    return fail(VAE_E_BADARG, "bn_apply: BN_DY needs aux (y), dgamma, dbeta");
  if (!(x.slope >= 0.f && x.slope <= 1.f) && x.kind != VAE_X_BN_DY) return fail(VAE_E_BADARG, "bn_apply: slope");
  BnApply q;
  q.chunks = a->rows * (long)a->channels / 8;
  q.C = a->channels;
  q.x = static_cast<const __bf16*>(a->x);
  q.xf = x;
  q.db = a->db;
  q.out = static_cast<__bf16*>(a->out);
  long grid = (q.chunks + (long)BA_T * BA_UNROLL - 1) / ((long)BA_T * BA_UNROLL);
  if (grid > 1024) grid = 1024;
  if (grid < 1) grid = 1;
  const bool bn = x.kind == VAE_X_BN_ACT || x.kind == VAE_X_BN_DY;
  const size_t lds = bn ? (size_t)(3 * tab_stride(a->channels) + 1024) * 4 : 0;
  VAE_LAUNCH(bn_apply_kernel, dim3((unsigned)grid), dim3(BA_T), lds, (hipStream_t)stream, q);
  return check_launch("bn_apply");
}
