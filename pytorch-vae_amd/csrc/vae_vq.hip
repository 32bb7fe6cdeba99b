// VQ-VAE pieces that are not convolutions: the VectorQuantizer (models/vq_vae.py:24-55) and the
// Tanh output layer + reconstruction error (vq_vae.py:156-160, :203).
//
// vq_fwd_kernel: nearest codebook row per latent vector.  One workgroup = 64 latent rows x 4
// threads per row; the codebook is streamed through LDS in chunks of 64 codes (16 KB fp32), each
// thread scores 16 codes of a chunk against its row held in registers (LDS reads are wave-
// broadcasts: the 16 rows of a wave read the same 4 codes).  Distances use the reference's fp32
// formula (Σz² + ΣE²) - 2 z·E (:30-32); ties resolve to the smaller index (torch.argmin).
// 2.1 GFLOP at B=128 (rows 32768, codes 512, dim 64) — VALU, ~1 % of the step's MFMA work.
//
// vq_bwd_kernel: elementwise straight-through / commitment gradient to the encoder output and the
// embedding-loss gradient of the codebook.  Each thread owns one latent component e of a run of
// consecutive rows and accumulates dE[index][e] in a register while the index repeats (spatial
// neighbours usually share a code), so the codebook atomics drop by the run length.
#include "vae_common.hpp"

namespace vae {
namespace {

constexpr int VQB_RUN = 32;        // rows per thread (bwd)

template <class T>
__device__ __forceinline__ float lat_val(const T* lat, long i, const vae_xform& xf) {
  const float v = ld_f(lat + i);
  return xf.kind == VAE_X_ACT ? lrelu(v, xf.slope) : v;
}

// Distance GEMM on the f32-input MFMA (v_mfma_f32_16x16x4_f32: an exact k-ordered fmaf chain,
// 64 FLOP/clk/SIMD — 10x what the LDS-fed VALU loop of r1 reached, 15 TF/s).  A workgroup owns
// 64 x RB latent rows (4 waves x RB blocks of 16; RB = 1 by default); lane l supplies, for k-step s, dimension
// (l>>4)*S + s of its row (A) and of its code (B) — any k permutation gives the same dot
// product's terms, and this one makes both fragments contiguous 16-float runs.  The codebook is
// staged through LDS in chunks of VQF_CH codes (rows padded to D+4 floats: conflict-free
// 16-byte reads), the next chunk prefetched into registers while the current one is scored.
// Output tile: lane l holds code (l&15) of the block for rows 4*(l>>4)+i, so each lane scans its
// codes in ascending order (strict <: first minimum) and the 16 lanes of a row combine
// (distance, index) lexicographically: torch.argmin's first-minimum tie-break.
constexpr int VQF_CH = 128;        // codes per LDS chunk
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));

// RB: 16-row blocks per wave (workgroup = 4 waves x RB x 16 rows)
template <class T, int D, int RB>
__global__ void __launch_bounds__(256) vq_fwd_kernel(vae_vq_args a) {
  kernarg_prefetch<(sizeof(vae_vq_args) < 1024 ? sizeof(vae_vq_args) : 1024)>();
  constexpr int VQF_ROWS = 64 * RB;
  constexpr int S = D / 4;                         // k-steps (dims per lane)
  constexpr int LDC = D + 4;                       // padded codebook row (floats)
  constexpr int PF = VQF_CH * D / 4 / 256;         // 16-byte codebook vectors per thread per chunk
  __shared__ __attribute__((aligned(16))) float cb[VQF_CH * LDC];
  __shared__ float cn[VQF_CH];
  __shared__ float zzs[VQF_ROWS];
  __shared__ int bix[VQF_ROWS];
  __shared__ float red[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kg = lane >> 4, lc = lane & 15;
  const long row0 = (long)blockIdx.x * VQF_ROWS;
  const T* lat = static_cast<const T*>(a.lat);
  const f32x4* cbg = reinterpret_cast<const f32x4*>(a.codebook);
  const long cb_vecs = (long)a.codes * D / 4;

  // A fragments: rows row0 + wave*32 + rb*16 + lc, dims kg*S + s
  float af[RB][S];
  float zp[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const long r = row0 + wave * 16 * RB + rb * 16 + lc;
    const bool ok = r < a.rows;
    float s2 = 0.f;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      af[rb][s] = ok ? lat_val(lat, r * D + kg * S + s, a.lat_xf) : 0.f;
      s2 = fmaf(af[rb][s], af[rb][s], s2);
    }
    zp[rb] = s2;
  }
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    float s2 = zp[rb];
    s2 += __shfl_xor(s2, 16);
    s2 += __shfl_xor(s2, 32);
    if (kg == 0) zzs[wave * 16 * RB + rb * 16 + lc] = s2;
  }

  f32x4 pf[PF];
  auto fetch = [&](int c0) {
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      const long v = (long)c0 * D / 4 + tid + 256 * j;
      pf[j] = v < cb_vecs ? cbg[v] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  fetch(0);
  __syncthreads();                                  // zzs
  float zz[RB][4];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int i = 0; i < 4; ++i) zz[rb][i] = zzs[wave * 16 * RB + rb * 16 + kg * 4 + i];

  float best[RB][4];
  int bidx[RB][4];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int i = 0; i < 4; ++i) { best[rb][i] = INFINITY; bidx[rb][i] = 0x7fffffff; }

  for (int c0 = 0; c0 < a.codes; c0 += VQF_CH) {
    const int nc = min(VQF_CH, a.codes - c0);
    __syncthreads();                                // previous chunk fully consumed
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      const int v = tid + 256 * j;                  // vector within the chunk
      const int code = v / (D / 4), e4 = v - code * (D / 4);
      *reinterpret_cast<f32x4*>(cb + code * LDC + 4 * e4) = pf[j];
    }
    if (c0 + VQF_CH < a.codes) fetch(c0 + VQF_CH);
    __syncthreads();
    if (tid < VQF_CH) {
      float s2 = 0.f;
#pragma unroll
      for (int e = 0; e < D; ++e) s2 = fmaf(cb[tid * LDC + e], cb[tid * LDC + e], s2);
      cn[tid] = s2;
    }
    __syncthreads();
    for (int cbk = 0; cbk < nc; cbk += 16) {
      float bf[S];
      const float* src = cb + (cbk + lc) * LDC + kg * S;
#pragma unroll
      for (int s4 = 0; s4 < S / 4; ++s4) {
        const f32x4 w = *reinterpret_cast<const f32x4*>(src + 4 * s4);
        bf[4 * s4 + 0] = w[0]; bf[4 * s4 + 1] = w[1]; bf[4 * s4 + 2] = w[2]; bf[4 * s4 + 3] = w[3];
      }
      f32x4 acc[RB];
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) acc[rb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < S; ++s)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[rb][s], bf[s], acc[rb], 0, 0, 0);
      const int code = cbk + lc;
      if (code < nc) {
        const float c2 = cn[code];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float d = (zz[rb][i] + c2) - 2.f * acc[rb][i];
            if (d < best[rb][i]) { best[rb][i] = d; bidx[rb][i] = c0 + code; }
          }
      }
    }
  }
  // combine the 16 lanes of each row: smaller distance, ties -> smaller index
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float b = best[rb][i];
      int bi = bidx[rb][i];
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) {
        const float ob = __shfl_xor(b, off);
        const int oi = __shfl_xor(bi, off);
        if (ob < b || (ob == b && oi < bi)) { b = ob; bi = oi; }
      }
      if (bi == 0x7fffffff) bi = 0;                 // all-NaN row: keep the index in range
      if (lc == 0) bix[wave * 16 * RB + rb * 16 + kg * 4 + i] = bi;
    }
  __syncthreads();
  // indices, q = E[idx] (coalesced over the tile's rows x D), sum (q - z)^2
  float sse = 0.f;
  if (tid < VQF_ROWS && row0 + tid < a.rows) a.indices[row0 + tid] = bix[tid];
  T* q = static_cast<T*>(a.q);
#pragma unroll 4
  for (int j = tid; j < VQF_ROWS * D; j += 256) {
    const int lr = j / D, e = j - lr * D;
    const long r = row0 + lr;
    if (r >= a.rows) break;
    const float v = a.codebook[(long)bix[lr] * D + e];
    q[r * D + e] = cvt<T>(v);
    const float d = v - lat_val(lat, r * D + e, a.lat_xf);
    sse = fmaf(d, d, sse);
  }
  for (int off = 32; off > 0; off >>= 1) sse += __shfl_xor(sse, off);
  if (lane == 0) red[wave] = sse;
  __syncthreads();
  if (tid == 0) atomicAdd(a.sse, (red[0] + red[1]) + (red[2] + red[3]));
}

// LM: the workgroup merges its rows' codebook-gradient runs in LDS first (a slot per distinct code
// of its rows), then issues one global atomic per (distinct code, dimension): the runs of the 32-row
// thread segments were one atomic each, and rows that share a code across threads and row groups
// (a codebook in use by few codes) all hit the same addresses.  dim <= 64 dividing 256, codes <= 1024.
constexpr int kVqLdsCodes = 1024;
constexpr int kVqLdsRows = 512;                            // rows per workgroup at dim 16
template <class T, bool LM>
__global__ void __launch_bounds__(256) vq_bwd_kernel(vae_vq_args a) {
  kernarg_prefetch<(sizeof(vae_vq_args) < 1024 ? sizeof(vae_vq_args) : 1024)>();
  const int D = a.dim;
  const int e = threadIdx.x % D;
  const int lanes_rows = 256 / D;                            // row groups per workgroup
  const long r0 = ((long)blockIdx.x * lanes_rows + threadIdx.x / D) * VQB_RUN;
  const bool active = threadIdx.x < lanes_rows * D;
  if (!LM && !active) return;
  const float n = (float)a.rows * (float)D;
  const float s = a.loss_grad ? *a.loss_grad : 1.f;
  const float cz = s * a.beta * 2.f / n, ce = s * 2.f / n;
  const T* lat = static_cast<const T*>(a.lat);
  const T* dq = static_cast<const T*>(a.dq);
  T* dlat = static_cast<T*>(a.dlat);
  // every row's loads are issued before any is used (the loop of r2 walked its 32 rows with an
  // index load -> codebook load dependency per row: 61 us at B=128, all of it memory round trips)
  long kk[VQB_RUN];
  float pre[VQB_RUN], dqv[VQB_RUN], qv[VQB_RUN];
#pragma unroll
  for (int i = 0; i < VQB_RUN; ++i) {
    const long r = min(r0 + i, (long)a.rows - 1);
    kk[i] = active ? a.indices[r] : 0;
    pre[i] = active ? ld_f(lat + r * D + e) : 0.f;
    dqv[i] = active ? ld_f(dq + r * D + e) : 0.f;
  }
  __shared__ int slot_of[LM ? kVqLdsCodes : 1];
  __shared__ int code_of[LM ? kVqLdsRows : 1];
  __shared__ float lacc[LM ? 8192 : 1];
  __shared__ int nslot;
  if constexpr (LM) {
    for (int c = threadIdx.x; c < a.codes; c += 256) slot_of[c] = -1;
    if (threadIdx.x == 0) nslot = 0;
    __syncthreads();
    if (active && e == 0)                                    // mark the codes of this thread's rows
      for (int i = 0; i < VQB_RUN; ++i)
        if (r0 + i < a.rows && (unsigned long)kk[i] < (unsigned long)a.codes) slot_of[kk[i]] = -2;
    __syncthreads();
    for (int c = threadIdx.x; c < a.codes; c += 256)
      if (slot_of[c] == -2) {
        const int sl = atomicAdd(&nslot, 1);
        slot_of[c] = sl;
        code_of[sl] = c;
      }
    __syncthreads();
    for (int i = threadIdx.x; i < nslot * D; i += 256) lacc[i] = 0.f;
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < VQB_RUN; ++i) qv[i] = active ? a.codebook[kk[i] * D + e] : 0.f;
  long cur = -1;
  float acc = 0.f;
  auto flush = [&](long code, float v) {
    if constexpr (LM) {
      if ((unsigned long)code < (unsigned long)a.codes) atomicAdd(&lacc[slot_of[code] * D + e], v);
    } else {
      atomicAdd(a.dcodebook + code * D + e, v);
    }
  };
  if (active) {
#pragma unroll
    for (int i = 0; i < VQB_RUN; ++i) {
      const long r = r0 + i;
      if (r >= a.rows) break;
      const long k = kk[i];
      const float z = a.lat_xf.kind == VAE_X_ACT ? lrelu(pre[i], a.lat_xf.slope) : pre[i];
      float g = dqv[i] + cz * (z - qv[i]);
      if (a.lat_xf.kind == VAE_X_ACT) g = pre[i] > 0.f ? g : g * a.lat_xf.slope;
      dlat[r * D + e] = cvt<T>(g);
      if (k != cur) {
        if (cur >= 0) flush(cur, acc);
        cur = k;
        acc = 0.f;
      }
      acc += ce * (qv[i] - z);
    }
    if (cur >= 0) flush(cur, acc);
  }
  if constexpr (LM) {
    __syncthreads();
    for (int i = threadIdx.x; i < nslot * D; i += 256) {
      const int sl = i / D, d = i - sl * D;
      atomicAdd(a.dcodebook + (long)code_of[sl] * D + d, lacc[i]);
    }
  }
}

// Tanh + reconstruction SSE (+ backward seed).  One thread per pixel, 256 pixels of one image per
// workgroup (h*w % 256 == 0, checked on the host).
template <class T, int C>
__global__ void __launch_bounds__(256) recon_kernel(vae_recon_args a, int bwd) {
  kernarg_prefetch<(sizeof(vae_recon_args) < 1024 ? sizeof(vae_recon_args) : 1024)>();
  __shared__ float red[4];
  const long hw = (long)a.h * a.w;
  const long pix = (long)blockIdx.x * 256 + threadIdx.x;     // over n*h*w
  const long img = pix / hw, sp = pix - img * hw;
  const T* y = static_cast<const T*>(a.y);
  const int ld = a.ld > 0 ? a.ld : C;
  // bf16 rows of 8 (the packed RGB ends): one 16-byte load of y and one 16-byte store of dy per pixel
  const bool pk = sizeof(T) == 2 && ld == 8 && ((uintptr_t)a.y & 15) == 0 && ((uintptr_t)a.dy & 15) == 0;
  float yv[C];
  if (!bwd) {
    if (pk) {
      const u32x4v w = *reinterpret_cast<const u32x4v*>(y + pix * 8);
#pragma unroll
      for (int c = 0; c < C; ++c) yv[c] = __uint_as_float(((c & 1) ? (w[c >> 1] >> 16) : (w[c >> 1] & 0xffffu)) << 16);
    } else {
#pragma unroll
      for (int c = 0; c < C; ++c) yv[c] = ld_f(y + pix * ld + c);
    }
  }
  float sse = 0.f;
  float gv[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const long o = (img * C + c) * hw + sp;                  // NCHW
    float r;
    if (bwd) {
      r = a.recon[o];
    } else {
      r = tanhf(yv[c]);
      a.recon[o] = r;
    }
    const float d = r - a.target[o];
    sse = fmaf(d, d, sse);
    gv[c] = 0.f;
    if (a.dy) gv[c] = (a.grad_recon ? a.grad_recon[o] : a.grad_scale * 2.f * d) * (1.f - r * r);
  }
  if (a.dy) {
    if (pk) {
      u32x4v w = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const uint32_t b = (uint32_t)__builtin_bit_cast(unsigned short, (__bf16)gv[c]);
        w[c >> 1] |= (c & 1) ? (b << 16) : b;
      }
      *reinterpret_cast<u32x4v*>(static_cast<T*>(a.dy) + pix * 8) = w;
    } else {
      for (int c = C; c < ld; ++c) static_cast<T*>(a.dy)[pix * ld + c] = cvt<T>(0.f);
#pragma unroll
      for (int c = 0; c < C; ++c) static_cast<T*>(a.dy)[pix * ld + c] = cvt<T>(gv[c]);
    }
  }
  if (bwd || !a.sse) return;
  for (int off = 32; off > 0; off >>= 1) sse += __shfl_xor(sse, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sse;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(a.sse + img, (red[0] + red[1]) + (red[2] + red[3]));
}

int vq_check(const vae_vq_args* a, const char* what) {
  if (!a || !a->lat || !a->codebook) return fail(VAE_E_BADARG, "%s: null tensor", what);
  if (a->rows <= 0 || a->codes <= 0) return fail(VAE_E_BADSHAPE, "%s: rows %d codes %d", what, a->rows, a->codes);
  if (a->dim != 64 && a->dim != 32 && a->dim != 16)
    return fail(VAE_E_UNSUPPORTED, "%s: code dim %d (kernels take 16, 32 or 64)", what, a->dim);
  if (a->lat_xf.kind != VAE_X_NONE && a->lat_xf.kind != VAE_X_ACT)
    return fail(VAE_E_UNSUPPORTED, "%s: latent transform must be NONE or ACT", what);
  if (a->lat_xf.kind == VAE_X_ACT && !(a->lat_xf.slope >= 0.f && a->lat_xf.slope <= 1.f))
    return fail(VAE_E_BADARG, "%s: slope", what);
  if (a->dtype != VAE_F32 && a->dtype != VAE_BF16) return fail(VAE_E_BADDTYPE, "%s: dtype", what);
  return VAE_OK;
}

template <int D, int RB>
void vq_fwd_launch_rb(const vae_vq_args* a, hipStream_t st) {
  const dim3 grid((a->rows + 64 * RB - 1) / (64 * RB));
  if (a->dtype == VAE_F32) VAE_LAUNCH((vq_fwd_kernel<float, D, RB>), grid, dim3(256), 0, st, *a);
  else VAE_LAUNCH((vq_fwd_kernel<__bf16, D, RB>), grid, dim3(256), 0, st, *a);
}

// rows per workgroup 64 * RB (VAE_VQF_RB = 1 | 2 for sweeps)
template <int D>
int vq_fwd_launch(const vae_vq_args* a, hipStream_t st) {
  // measured at B=128 (32768 rows, 512 codes, dim 64): 64 rows 39.0 us, 128 rows 42.6 us — twice
  // the workgroups (two per CU) hide the chunk barriers and the epilogue better than the second
  // row block's reuse of each codebook fragment saves
  vq_fwd_launch_rb<D, 1>(a, st);
  return check_launch("vq_fwd");
}

int recon_launch(const vae_recon_args* a, int bwd, hipStream_t st) {
  if (!a || !a->target || !a->recon) return fail(VAE_E_BADARG, "recon: null tensor");
  if (a->n <= 0 || a->h <= 0 || a->w <= 0) return fail(VAE_E_BADSHAPE, "recon: shape");
  if (a->c != 3) return fail(VAE_E_UNSUPPORTED, "recon: %d channels (the output layer is RGB)", a->c);
  if (a->ld != 0 && a->ld < a->c) return fail(VAE_E_BADARG, "recon: ld %d < c", a->ld);
  if (((long)a->h * a->w) % 256) return fail(VAE_E_UNSUPPORTED, "recon: h*w must be a multiple of 256");
  if (!bwd && !a->y) return fail(VAE_E_BADARG, "recon_fwd: y");
  if (bwd && (!a->grad_recon || !a->dy)) return fail(VAE_E_BADARG, "recon_bwd: grad_recon / dy");
  const dim3 grid((unsigned)((long)a->n * a->h * a->w / 256));
  if (a->dtype == VAE_F32) VAE_LAUNCH((recon_kernel<float, 3>), grid, dim3(256), 0, st, *a, bwd);
  else if (a->dtype == VAE_BF16) VAE_LAUNCH((recon_kernel<__bf16, 3>), grid, dim3(256), 0, st, *a, bwd);
  else return fail(VAE_E_BADDTYPE, "recon: dtype");
  return check_launch("recon");
}

template <class T>
__global__ void nchw_to_nhwc_pad_kernel(int n, int c, int h, int w, int cp, const float* x, T* y) {
  const long pix = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long hw = (long)h * w;
  if (pix >= (long)n * hw) return;
  const long img = pix / hw, sp = pix - img * hw;
  for (int j = 0; j < cp; ++j) y[pix * cp + j] = cvt<T>(j < c ? x[(img * c + j) * hw + sp] : 0.f);
}

template <class T>
__global__ void pad_channels_kernel(long rows, int c, int cp, const T* src, T* dst) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * cp) return;
  const long r = i / cp;
  const int j = (int)(i - r * cp);
  dst[i] = j < c ? src[r * c + j] : cvt<T>(0.f);
}

__global__ void unpad_accumulate_kernel(long rows, int cp, int c, const float* src, float* dst) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * c) return;
  const long r = i / c;
  const int j = (int)(i - r * c);
  dst[i] += src[r * cp + j];
}

}  // namespace
}  // namespace vae

using namespace vae;

extern "C" int vae_nchw_to_nhwc_pad(int32_t dtype, int32_t n, int32_t c, int32_t h, int32_t w, int32_t cp, const float* x,
                                    void* y, void* stream) {
  if (!x || !y || n <= 0 || c <= 0 || h <= 0 || w <= 0 || cp < c) return fail(VAE_E_BADARG, "nchw_to_nhwc_pad: args");
  const long pix = (long)n * h * w;
  const dim3 grid((unsigned)((pix + 255) / 256));
  if (dtype == VAE_F32) VAE_LAUNCH(nchw_to_nhwc_pad_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, n, c, h, w, cp, x, (float*)y);
  else if (dtype == VAE_BF16) VAE_LAUNCH(nchw_to_nhwc_pad_kernel<__bf16>, grid, dim3(256), 0, (hipStream_t)stream, n, c, h, w, cp, x, (__bf16*)y);
  else return fail(VAE_E_BADDTYPE, "nchw_to_nhwc_pad: dtype");
  return check_launch("nchw_to_nhwc_pad");
}

extern "C" int vae_pad_channels(int32_t dtype, int64_t rows, int32_t c, int32_t cp, const void* src, void* dst, void* stream) {
  if (!src || !dst || rows <= 0 || c <= 0 || cp < c) return fail(VAE_E_BADARG, "pad_channels: args");
  const dim3 grid((unsigned)((rows * cp + 255) / 256));
  if (dtype == VAE_F32) VAE_LAUNCH(pad_channels_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, (long)rows, c, cp, (const float*)src, (float*)dst);
  else if (dtype == VAE_BF16) VAE_LAUNCH(pad_channels_kernel<__bf16>, grid, dim3(256), 0, (hipStream_t)stream, (long)rows, c, cp, (const __bf16*)src, (__bf16*)dst);
  else return fail(VAE_E_BADDTYPE, "pad_channels: dtype");
  return check_launch("pad_channels");
}

extern "C" int vae_unpad_accumulate(int64_t rows, int32_t cp, int32_t c, const float* src, float* dst, void* stream) {
  if (!src || !dst || rows <= 0 || c <= 0 || cp < c) return fail(VAE_E_BADARG, "unpad_accumulate: args");
  const dim3 grid((unsigned)((rows * c + 255) / 256));
  VAE_LAUNCH(unpad_accumulate_kernel, grid, dim3(256), 0, (hipStream_t)stream, (long)rows, cp, c, src, dst);
  return check_launch("unpad_accumulate");
}

extern "C" int vae_vq_fwd(const vae_vq_args* a, void* stream) {
  int rc = vq_check(a, "vq_fwd");
  if (rc) return rc;
  if (!a->indices || !a->q || !a->sse) return fail(VAE_E_BADARG, "vq_fwd: indices / q / sse");
  if (reinterpret_cast<uintptr_t>(a->codebook) % 16) return fail(VAE_E_BADARG, "vq_fwd: codebook not 16-byte aligned");
  const hipStream_t st = (hipStream_t)stream;
  if (a->dim == 64) return vq_fwd_launch<64>(a, st);
  if (a->dim == 32) return vq_fwd_launch<32>(a, st);
  return vq_fwd_launch<16>(a, st);
}

extern "C" int vae_vq_bwd(const vae_vq_args* a, void* stream) {
  int rc = vq_check(a, "vq_bwd");
  if (rc) return rc;
  if (!a->indices || !a->dq || !a->dlat || !a->dcodebook) return fail(VAE_E_BADARG, "vq_bwd: indices / dq / dlat / dcodebook");
  const int groups = 256 / a->dim;
  const long runs = ((long)a->rows + VQB_RUN - 1) / VQB_RUN;
  const dim3 grid((unsigned)((runs + groups - 1) / groups));
  const bool lm = a->dim <= 64 && 256 % a->dim == 0 && a->dim >= 16 && a->codes <= kVqLdsCodes;
  const hipStream_t st = (hipStream_t)stream;
  if (a->dtype == VAE_F32) {
    if (lm) VAE_LAUNCH((vq_bwd_kernel<float, true>), grid, dim3(256), 0, st, *a);
    else VAE_LAUNCH((vq_bwd_kernel<float, false>), grid, dim3(256), 0, st, *a);
  } else {
    if (lm) VAE_LAUNCH((vq_bwd_kernel<__bf16, true>), grid, dim3(256), 0, st, *a);
    else VAE_LAUNCH((vq_bwd_kernel<__bf16, false>), grid, dim3(256), 0, st, *a);
  }
  return check_launch("vq_bwd");
}

extern "C" int vae_recon_fwd(const vae_recon_args* a, void* stream) { return recon_launch(a, 0, (hipStream_t)stream); }
extern "C" int vae_recon_bwd(const vae_recon_args* a, void* stream) { return recon_launch(a, 1, (hipStream_t)stream); }
