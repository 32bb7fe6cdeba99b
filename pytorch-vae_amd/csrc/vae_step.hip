// vae_step_begin_ex: the head of a training step as ONE launch (vaehip.h).  Three kinds of work that
// do not depend on each other share the grid as block ranges:
//   [0, nz)            zero the step's zero region (gradients, BatchNorm sums, SSE, d[mu|logvar]) and
//                      ++*step — vae_step_begin
//   [nz, nz + nx)      the fp32 NCHW image -> NHWC with cp channels (zeros above c), one pixel per
//                      thread, one 16-byte store per pixel for bf16 / cp = 8 — vae_nchw_to_nhwc_pad
//   [nz + nx, ...)     up to VAE_PAD_MAX padded weight copies — vae_pad_channels
//   [..., end)         up to VAE_SWAP_MAX swapped-axes weight copies — vae_swap_axes (they read the fp32
//                      weights the previous step's optimizer wrote; measured as a launch of their own
//                      behind the optimizer: 8.5 us per VanillaVAE step, profiles/r5p)
// The reference's step (experiment.py:45-49) feeds the image straight into the first Conv2d
// (models/vanilla_vae.py:84); the padding exists only so that the first layer runs on the packed
// 16-byte GEMM operand path.  profiles/r3a: the three separate launches took 6.5 + 5.2 + 4.8 us.
#include <algorithm>

#include "vae_common.hpp"

namespace vae {
namespace {

constexpr int kZeroRanges = VAE_SLAB_MAX + 1;
struct StepBegin {
  vae_step_begin_args a;
  long n16;              // 16-byte words of the zero region
  int ntail;             // bytes after them
  int nz, nx;            // blocks of the zeroing and of the image ranges
  int nzr;                          // zeroed ranges (the region minus its keep ranges)
  int zb0[kZeroRanges + 1];         // first block of each range
  long zoff[kZeroRanges], zlen[kZeroRanges];   // in 16-byte words
  int pad0[VAE_PAD_MAX + 1];   // first block of each pad descriptor (relative to nz + nx)
  int np;                      // blocks of the pad range
  int swap0[VAE_SWAP_MAX + 1]; // first block of each swap descriptor (relative to nz + nx + np)
};

template <class T>
__device__ __forceinline__ void image_pixel(const vae_step_begin_args& a, long pix) {
  const long hw = (long)a.h * a.w;
  const long img = pix / hw, sp = pix - img * hw;
  const float* src = a.x + img * a.c * hw + sp;
  T* dst = static_cast<T*>(a.y) + pix * a.cp;
  if constexpr (sizeof(T) == 2) {
    if (a.cp == 8) {                       // the packed RGB case: one 16-byte store
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (__bf16)(j < a.c ? src[j * hw] : 0.f);
      *reinterpret_cast<bf16x8*>(dst) = o;
      return;
    }
  }
  for (int j = 0; j < a.cp; ++j) dst[j] = cvt<T>(j < a.c ? src[j * hw] : 0.f);
}

template <class T>
__global__ void __launch_bounds__(256) step_begin_ex_kernel(const StepBegin s) {
  kernarg_prefetch<(sizeof(StepBegin) < 1024 ? sizeof(StepBegin) : 1024)>();
  const int b = blockIdx.x, tid = threadIdx.x;
  if (b < s.nz) {
    f32x4* z = static_cast<f32x4*>(s.a.zero);
    int k = 0;
    while (k + 1 < s.nzr && b >= s.zb0[k + 1]) ++k;
    const int lb = b - s.zb0[k], nb = s.zb0[k + 1] - s.zb0[k];
    f32x4* zr = z + s.zoff[k];
    for (long i = (long)lb * 256 + tid; i < s.zlen[k]; i += (long)nb * 256) zr[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (b == 0 && tid < s.ntail) reinterpret_cast<unsigned char*>(z + s.n16)[tid] = 0;
    if (b == 0 && tid == 0 && s.a.step) *s.a.step += 1;
    return;
  }
  if (b < s.nz + s.nx) {
    const long pix = (long)(b - s.nz) * 256 + tid;
    if (pix < (long)s.a.n * s.a.h * s.a.w) image_pixel<T>(s.a, pix);
    return;
  }
  const int pb = b - s.nz - s.nx;
  if (pb >= s.np) {
    __shared__ float t[kSwapT][kSwapT + 1];
    const int sb = pb - s.np;
    int k = 0;
    while (k + 1 < s.a.nswap && sb >= s.swap0[k + 1]) ++k;
    swap_tile(s.a.swap[k], sb - s.swap0[k], t);
    return;
  }
  int k = 0;
  while (k + 1 < s.a.npad && pb >= s.pad0[k + 1]) ++k;
  const vae_pad_desc& d = s.a.pad[k];
  const long i = (long)(pb - s.pad0[k]) * 256 + tid;
  if (i >= d.rows * d.cp) return;
  const long r = i / d.cp;
  const int j = (int)(i - r * d.cp);
  static_cast<T*>(d.dst)[i] = j < d.c ? static_cast<const T*>(d.src)[r * d.c + j] : cvt<T>(0.f);
}

}  // namespace
}  // namespace vae

using namespace vae;

extern "C" int vae_step_begin_ex(const vae_step_begin_args* a, void* stream) {
  if (!a || a->bytes < 0 || (a->bytes > 0 && !a->zero)) return fail(VAE_E_BADARG, "step_begin_ex: zero region");
  if (((uintptr_t)a->zero & 15) != 0) return fail(VAE_E_BADARG, "step_begin_ex: zero region must be 16-B aligned");
  if (a->dtype != VAE_F32 && a->dtype != VAE_BF16) return fail(VAE_E_BADDTYPE, "step_begin_ex: dtype");
  if (a->npad < 0 || a->npad > VAE_PAD_MAX) return fail(VAE_E_BADARG, "step_begin_ex: %d pads", a->npad);
  StepBegin s;
  s.a = *a;
  s.n16 = a->bytes / 16;
  s.ntail = (int)(a->bytes - s.n16 * 16);
  // the zeroed ranges: the region minus its keep ranges (sorted, clipped, 16-byte words inward)
  if (a->nkeep < 0 || a->nkeep > VAE_SLAB_MAX) return fail(VAE_E_BADARG, "step_begin_ex: %d keep ranges", a->nkeep);
  long ko[VAE_SLAB_MAX], ke[VAE_SLAB_MAX];
  int nk = 0;
  for (int k = 0; k < a->nkeep; ++k) {
    const long o = (a->keep[k].off + 15) / 16, e = (a->keep[k].off + a->keep[k].bytes) / 16;
    if (a->keep[k].off < 0 || a->keep[k].bytes < 0) return fail(VAE_E_BADARG, "step_begin_ex: keep %d", k);
    const long oo = o < s.n16 ? o : s.n16, ee = e < s.n16 ? e : s.n16;
    if (ee > oo) { ko[nk] = oo; ke[nk] = ee; ++nk; }
  }
  std::sort(ko, ko + nk);
  std::sort(ke, ke + nk);              // (keep ranges do not overlap: the gradients of distinct tensors)
  s.nzr = 0;
  long pos = 0;
  for (int k = 0; k <= nk; ++k) {
    const long end = k < nk ? ko[k] : s.n16;
    if (end > pos) { s.zoff[s.nzr] = pos; s.zlen[s.nzr] = end - pos; ++s.nzr; }
    if (k < nk && ke[k] > pos) pos = ke[k];
  }
  if (s.nzr == 0) { s.zoff[0] = 0; s.zlen[0] = 0; s.nzr = 1; }
  int zb = 0;
  for (int k = 0; k < s.nzr; ++k) {
    s.zb0[k] = zb;
    const long nb = (s.zlen[k] + 255) / 256;
    zb += (int)(nb < 1 ? 1 : (nb > 2048 ? 2048 : nb));
  }
  s.zb0[s.nzr] = zb;
  s.nz = zb;
  s.nx = 0;
  if (a->x) {
    if (!a->y || a->n <= 0 || a->c <= 0 || a->h <= 0 || a->w <= 0 || a->cp < a->c)
      return fail(VAE_E_BADARG, "step_begin_ex: image args");
    if (a->dtype == VAE_BF16 && a->cp == 8 && ((uintptr_t)a->y & 15) != 0)
      return fail(VAE_E_BADARG, "step_begin_ex: padded image must be 16-B aligned");
    s.nx = (int)(((long)a->n * a->h * a->w + 255) / 256);
  }
  int nb = 0;
  for (int k = 0; k < a->npad; ++k) {
    const vae_pad_desc& d = a->pad[k];
    if (!d.src || !d.dst || d.rows <= 0 || d.c <= 0 || d.cp < d.c) return fail(VAE_E_BADARG, "step_begin_ex: pad %d", k);
    s.pad0[k] = nb;
    nb += (int)((d.rows * d.cp + 255) / 256);
  }
  s.pad0[a->npad] = nb;
  s.np = nb;
  if (a->nswap < 0 || a->nswap > VAE_SWAP_MAX) return fail(VAE_E_BADARG, "step_begin_ex: %d swaps", a->nswap);
  int ns = 0;
  for (int k = 0; k < a->nswap; ++k) {
    const vae_swap_desc& d = a->swap[k];
    if (!d.src || !d.dst || d.a <= 0 || d.b <= 0 || d.rs <= 0 || (d.src_dtype != VAE_F32 && d.src_dtype != VAE_BF16))
      return fail(VAE_E_BADARG, "step_begin_ex: swap %d", k);
    s.swap0[k] = ns;
    ns += swap_tiles(d);
  }
  s.swap0[a->nswap] = ns;
  const dim3 grid((unsigned)(s.nz + s.nx + nb + ns));
  if (a->dtype == VAE_BF16) VAE_LAUNCH(step_begin_ex_kernel<__bf16>, grid, dim3(256), 0, (hipStream_t)stream, s);
  else VAE_LAUNCH(step_begin_ex_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, s);
  return check_launch("step_begin_ex");
}
