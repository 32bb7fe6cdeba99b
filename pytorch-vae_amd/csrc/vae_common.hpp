// Shared device/host helpers for libvaehip.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "vaehip.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

namespace vae {

// ---------------------------------------------------------------- error state (host)
void set_error(const char* fmt, ...);
int fail(int code, const char* fmt, ...);
int check_launch(const char* what);
// vae_bn_finalize as a host call (validation + launch); used by fused-finalisation fallbacks
int bn_finalize_launch(const vae_bn_args* a, hipStream_t stream);
// returned by a fast-path launcher whose preconditions do not hold (the caller falls back)
constexpr int kHeadFallback = 0x7fff0001;

// ---------------------------------------------------------------- deterministic reductions
// A call made with `deterministic` set writes every cross-workgroup partial sum it would have
// added with a float atomic to its own row of a workspace slab instead, and one ordered pass
// (ordered_sum_launch, vae_misc.hip) adds the rows in a fixed order:
//   output (g, c), g < groups, c < cols, sums slab rows [g*rpg, (g+1)*rpg) in ascending order,
//   each row at column (c / cw) * hstride + c % cw + f * fstride for f = 0 .. folds-1, and adds the
//   total into dst[c / cw][g * gstride + c % cw] (one thread owns each output: no atomics).
// The result no longer depends on workgroup timing, so repeated calls are bit-identical.
struct OrdSum {
  const float* slab;
  long rstride;
  int groups, rpg, cols, cw;
  long hstride;
  int folds;
  long fstride;
  float* dst[2];
  long gstride;
};
int ordered_sum_launch(const OrdSum& o, hipStream_t st);

// ---------------------------------------------------------------- workspace queries (host)
// vae_*_workspace_size runs an entry point's whole planning with an unbounded workspace and the
// query flag set: every site that would use workspace records its bytes (ws_fits) and VAE_LAUNCH
// launches nothing.  Outside a query, a plan that needs more workspace than the caller passed
// fails with VAE_E_BADARG; a NULL workspace selects the plan that uses none.  One flag per host
// thread, shared by all translation units (inline function with external linkage).
struct WsQuery {
  int on;
  long need;
};
inline WsQuery& ws_query() {
  static thread_local WsQuery q = {0, 0};
  return q;
}
inline bool querying() { return ws_query().on != 0; }
// Deferred weight-gradient reductions (vaehip.h vae_deferred_take): a call with defer_reduce set
// leaves its fp32 partial rows in its workspace and records them here (host thread; not while
// querying) for vae_adam_step_ex to reduce.  Returns false (and fails) when the list is full.
struct Deferred {
  int n;
  vae_grad_slab s[VAE_SLAB_MAX];
  int has_elbo;
  vae_elbo_args elbo;
};
inline Deferred& deferred() {
  static thread_local Deferred d = {};
  return d;
}
inline bool defer_slab(float* dst, long count, const float* slab, int rows, long ld) {
  if (querying()) return true;
  Deferred& d = deferred();
  for (int i = 0; i < d.n; ++i)                 // the same gradient deferred again (a call re-run
    if (d.s[i].dst == dst) {                    // before the reduction): its latest partials count
      d.s[i] = vae_grad_slab{dst, count, slab, rows, ld};
      return true;
    }
  if (d.n >= VAE_SLAB_MAX) {
    fail(VAE_E_UNSUPPORTED, "deferred reductions: more than %d outstanding", VAE_SLAB_MAX);
    return false;
  }
  d.s[d.n++] = vae_grad_slab{dst, count, slab, rows, ld};
  return true;
}
inline void defer_elbo(const vae_elbo_args& e) {
  if (querying()) return;
  Deferred& d = deferred();
  d.has_elbo = 1;
  d.elbo = e;
}
inline bool ws_fits(long need, long have, const char* what) {
  WsQuery& q = ws_query();
  if (q.on) {
    if (need > q.need) q.need = need;
    return true;
  }
  if (need <= have) return true;
  fail(VAE_E_BADARG, "%s: workspace of %ld bytes < %ld required (see vae_*_workspace_size)", what, have, need);
  return false;
}
// Query accounting for a call that stages `tail` bytes at the END of the workspace and gives the
// front to f's own sites: the requirement is f's, rounded to 256, plus the tail.
template <class F>
inline int with_ws_tail(long tail, F&& f) {
  WsQuery& q = ws_query();
  if (!q.on) return f();
  const long outer = q.need;
  q.need = 0;
  const int rc = f();
  const long inner = ((q.need + 255) / 256) * 256 + tail;
  q.need = outer > inner ? outer : inner;
  return rc;
}
// Launch log (host, per thread): while on, every VAE_LAUNCH records its kernel's host stub, so a
// measurement tool can ask which device kernels one ABI call launched (vae_launch_log /
// vae_launch_log_names) and match them against rocprofv3 rows instead of a hand-kept table.
struct LaunchLog {
  int on;
  int n;
  const void* k[64];
  int count[64];       // launches of each kernel while on (a call may launch one kernel several times)
};
inline LaunchLog& launch_log() {
  static thread_local LaunchLog l = {0, 0, {}, {}};
  return l;
}
inline void log_launch(const void* k) {
  LaunchLog& l = launch_log();
  if (!l.on) return;
  for (int i = 0; i < l.n; ++i)
    if (l.k[i] == k) { ++l.count[i]; return; }
  if (l.n < 64) { l.count[l.n] = 1; l.k[l.n++] = k; }
}
}  // namespace vae
#define VAE_LAUNCH(K, ...)                                      \
  do {                                                          \
    if (!::vae::querying()) {                                   \
      ::vae::log_launch((const void*)(K));                      \
      hipLaunchKernelGGL(K, __VA_ARGS__);                       \
    }                                                           \
  } while (0)
namespace vae {

// ---------------------------------------------------------------- kernel-argument prefetch
// A kernel reads its (up to 1 KB) argument block with scalar loads where each field is first
// used, and every branch on a field waits for it: the prologue becomes a chain of dependent
// scalar-cache misses before the first operand load goes out (host-resident kernel arguments made
// the conv GEMMs 5-11 us slower per launch, profiles/r5_notes.md).  Touching every 64-byte line
// of the block first puts all of them in flight at once; the later loads then hit the scalar cache.
// (Reads only; nothing is written through the scalar cache.)
// Lines 1..N-1 of the block (line 0 is read at entry anyway), one asm statement with its own
// wait: no prefetch load is still in flight when the compiler reuses its registers.
template <int BYTES>
__device__ __forceinline__ void kernarg_prefetch() {
  const void* k = (const void*)__builtin_amdgcn_kernarg_segment_ptr();
  unsigned d1, d2, d3, d4, d5, d6, d7;
  // (only lines inside the block: 15, 7, 3 or 1 of them by its size.  Early-clobber outputs: a
  // destination must not share the base-address registers, which later loads of the block still read)
  if constexpr (BYTES > 960) {
    unsigned e1, e2, e3, e4, e5, e6, e7, e8;
    asm volatile(
        "s_load_dword %0, %15, 64\n s_load_dword %1, %15, 128\n s_load_dword %2, %15, 192\n"
        " s_load_dword %3, %15, 256\n s_load_dword %4, %15, 320\n s_load_dword %5, %15, 384\n"
        " s_load_dword %6, %15, 448\n s_load_dword %7, %15, 512\n s_load_dword %8, %15, 576\n"
        " s_load_dword %9, %15, 640\n s_load_dword %10, %15, 704\n s_load_dword %11, %15, 768\n"
        " s_load_dword %12, %15, 832\n s_load_dword %13, %15, 896\n s_load_dword %14, %15, 960\n"
        " s_waitcnt lgkmcnt(0)"
        : "=&s"(d1), "=&s"(d2), "=&s"(d3), "=&s"(d4), "=&s"(d5), "=&s"(d6), "=&s"(d7), "=&s"(e1), "=&s"(e2), "=&s"(e3),
          "=&s"(e4), "=&s"(e5), "=&s"(e6), "=&s"(e7), "=&s"(e8)
        : "s"(k));
  } else if constexpr (BYTES > 448) {
    asm volatile(
        "s_load_dword %0, %7, 64\n s_load_dword %1, %7, 128\n s_load_dword %2, %7, 192\n"
        " s_load_dword %3, %7, 256\n s_load_dword %4, %7, 320\n s_load_dword %5, %7, 384\n"
        " s_load_dword %6, %7, 448\n s_waitcnt lgkmcnt(0)"
        : "=&s"(d1), "=&s"(d2), "=&s"(d3), "=&s"(d4), "=&s"(d5), "=&s"(d6), "=&s"(d7)
        : "s"(k));
  } else if constexpr (BYTES > 192) {
    asm volatile("s_load_dword %0, %3, 64\n s_load_dword %1, %3, 128\n s_load_dword %2, %3, 192\n"
                 " s_waitcnt lgkmcnt(0)"
                 : "=&s"(d1), "=&s"(d2), "=&s"(d3)
                 : "s"(k));
  } else if constexpr (BYTES > 64) {
    asm volatile("s_load_dword %0, %1, 64\n s_waitcnt lgkmcnt(0)" : "=&s"(d1) : "s"(k));
  }
}

// ---------------------------------------------------------------- scalar conversion
__device__ __forceinline__ float ld_f(const float* p) { return *p; }
__device__ __forceinline__ float ld_f(const __bf16* p) { return (float)(*p); }
template <class T> __device__ __forceinline__ T cvt(float v);
template <> __device__ __forceinline__ float cvt<float>(float v) { return v; }
template <> __device__ __forceinline__ __bf16 cvt<__bf16>(float v) { return (__bf16)v; }

// 8 consecutive elements -> floats (16-B aligned for bf16, 32-B for fp32)
__device__ __forceinline__ void ld8(const float* p, float (&v)[8]) {
  f32x4 a = *reinterpret_cast<const f32x4*>(p);
  f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
  v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
}
__device__ __forceinline__ void ld8(const __bf16* p, float (&v)[8]) {
  bf16x8 a = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (float)a[j];
}
__device__ __forceinline__ void ld4(const float* p, float (&v)[4]) {
  f32x4 a = *reinterpret_cast<const f32x4*>(p);
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
}
__device__ __forceinline__ void ld4(const __bf16* p, float (&v)[4]) {
  bf16x4 a = *reinterpret_cast<const bf16x4*>(p);
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = (float)a[j];
}

// LDS stores: 8 contiguous (16-B / 32-B aligned) and 2 contiguous elements
__device__ __forceinline__ void st8(float* d, const float (&v)[8]) {
  *reinterpret_cast<f32x4*>(d) = f32x4{v[0], v[1], v[2], v[3]};
  *reinterpret_cast<f32x4*>(d + 4) = f32x4{v[4], v[5], v[6], v[7]};
}
__device__ __forceinline__ void st8(__bf16* d, const float (&v)[8]) {
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (__bf16)v[j];
  *reinterpret_cast<bf16x8*>(d) = o;
}
__device__ __forceinline__ void st2(float* d, float a, float b) { *reinterpret_cast<f32x2*>(d) = f32x2{a, b}; }
__device__ __forceinline__ void st2(__bf16* d, float a, float b) {
  bf16x2 o; o[0] = (__bf16)a; o[1] = (__bf16)b;
  *reinterpret_cast<bf16x2*>(d) = o;
}

// LeakyReLU for 0 <= slope <= 1 (checked on the host): max(v, slope*v) — two VALU ops, no compare
__device__ __forceinline__ float lrelu(float v, float slope) { return fmaxf(v, v * slope); }

// ---------------------------------------------------------------- BN statistics
// Channel c of a replicated statistic (vae_xform.reps copies, rstride floats apart).  Loads go
// out 16 at a time with clamped (never skipped) addresses, so a 32-replica sum costs two
// dependent round trips, not 32.
__device__ __forceinline__ float rsum(const float* a, const vae_xform& x, int c) {
  if (x.reps <= 1) return a[c];
  float acc = 0.f;
  for (int r0 = 0; r0 < x.reps; r0 += 16) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int r = min(r0 + u, x.reps - 1);
      v[u] = a[(long)r * x.rstride + c];
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) acc += (r0 + u < x.reps) ? v[u] : 0.f;
  }
  return acc;
}

// mean/invstd/var of channel c from the producer's Σ(y-shift), Σ(y-shift)^2.
__device__ __forceinline__ void bn_moments(const vae_xform& x, int c, float& mean, float& invstd, float& var) {
  const float inv_m = 1.0f / x.count;
  const float s = rsum(x.sum, x, c) * inv_m;
  var = fmaxf(rsum(x.sumsq, x, c) * inv_m - s * s, 0.0f);
  mean = s + (x.shift ? x.shift[c] : 0.0f);
  invstd = 1.0f / sqrtf(var + x.eps);
}

// Per-channel coefficient table in LDS for one transform.
//   BN_ACT: v = lrelu(t*a + b)         ACT: v = lrelu(t)        NONE: v = t
//   BN_DY : v = a*t + b*aux + c
//   epilogue use (BN_ACT): also p,q with xhat = y*p + q
template <int MAXC, bool EPI>
struct XfTable {
  float a[MAXC], b[MAXC], c[MAXC];
  float p[EPI ? MAXC : 1], q[EPI ? MAXC : 1];

  // Fill for channels [0, C); optionally update BN running stats (one block only).
  __device__ __forceinline__ void fill(const vae_xform& x, bool update_running) {
    if (x.kind != VAE_X_BN_ACT && x.kind != VAE_X_BN_DY) return;
    for (int ch = threadIdx.x; ch < x.channels; ch += blockDim.x) {
      float mean, invstd, var;
      bn_moments(x, ch, mean, invstd, var);
      const float g = x.gamma[ch];
      if (x.kind == VAE_X_BN_ACT) {
        const float sc = g * invstd;
        a[ch] = sc;
        b[ch] = x.beta[ch] - mean * sc;
        if (EPI) { p[EPI ? ch : 0] = invstd; q[EPI ? ch : 0] = -mean * invstd; }
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
        a[ch] = A;
        b[ch] = -A * invstd * mgx;
        c[ch] = -A * (mg - mean * invstd * mgx);
      }
    }
  }
};

// ---------------------------------------------------------------- BatchNorm finalisation
// The per-step BatchNorm table (vae_bn_args, vaehip.h) for channel groups cg0, cg0+cgs, ... of
// 64 channels, by one 256-thread workgroup: every replica of every statistic a channel needs is
// loaded up front (64 channels x 4 replica lanes, <= 8 replicas per lane), the 4 lanes combine
// through LDS in a fixed order (deterministic) and lane 0 writes the table.  Used by the
// vae_bn_finalize kernel and by the last workgroup of a producing GEMM (fused finalisation).
constexpr int BNF_LANES = 4, BNF_PER = 8;      // replicas <= BNF_LANES * BNF_PER (checked on the host)

__device__ __forceinline__ void bn_finalize_block(const vae_bn_args& a, int cg0, int cgs) {
  __shared__ float red[4][BNF_LANES][64];
  const vae_xform& x = a.xf;
  const int C = x.channels;
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int reps = x.reps > 1 ? x.reps : 1;
  const long rstr = x.reps > 1 ? x.rstride : 0;
  const bool bwd = a.mode != 0;
  const float* arr[4] = {x.sum, x.sumsq, bwd ? x.dgamma : nullptr, bwd ? x.dbeta : nullptr};
  for (int cg = cg0; cg * 64 < C; cg += cgs) {
    const int c = cg * 64 + cl;
    const int cc = c < C ? c : 0;
    float v[4][BNF_PER];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int u = 0; u < BNF_PER; ++u) {
        const int r = rl + BNF_LANES * u;
        v[k][u] = (arr[k] && r < reps) ? arr[k][r * rstr + cc] : 0.f;
      }
    const float g = x.gamma[cc], be = x.beta[cc], sh = x.shift ? x.shift[cc] : 0.f;
    const bool run = !bwd && x.running_mean;
    const float rmean = run ? x.running_mean[cc] : 0.f, rvar = run ? x.running_var[cc] : 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float t = 0.f;
#pragma unroll
      for (int u = 0; u < BNF_PER; ++u) t += v[k][u];
      red[k][rl][cl] = t;
    }
    __syncthreads();
    if (rl == 0 && c < C) {
      float tot[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) tot[k] = (red[k][0][cl] + red[k][1][cl]) + (red[k][2][cl] + red[k][3][cl]);
      const float inv_m = 1.0f / x.count;
      const float s1 = tot[0] * inv_m;
      const float var = fmaxf(tot[1] * inv_m - s1 * s1, 0.0f);
      const float mean = s1 + sh;
      const float invstd = 1.0f / sqrtf(var + x.eps);
      if (!bwd) {
        const float sc = g * invstd;
        a.table[c] = sc;
        a.table[C + c] = be - mean * sc;
        a.table[2 * C + c] = invstd;
        a.table[3 * C + c] = -mean * invstd;
        if (run) {
          const float m = x.momentum;
          const float unb = x.count > 1.f ? var * x.count / (x.count - 1.f) : var;
          x.running_mean[c] = (1.f - m) * rmean + m * mean;
          x.running_var[c] = (1.f - m) * rvar + m * unb;
        }
      } else {
        const float dgam = tot[2], dbet = tot[3];
        const float A = g * invstd;
        const float mgx = dgam * inv_m, mg = dbet * inv_m;
        const float B = -A * invstd * mgx;
        const float Cc = -A * (mg - mean * invstd * mgx);
        a.table[c] = A;
        a.table[C + c] = B;
        a.table[2 * C + c] = Cc;
        if (x.dgamma_out) x.dgamma_out[c] += dgam;
        if (x.dbeta_out) x.dbeta_out[c] += dbet;
        if (a.db) {
          const float sum_y = tot[0] + x.count * sh;
          a.db[c] += A * dbet + B * sum_y + Cc * x.count;
        }
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- per-channel transform tables
// Views into LDS, sized by the real channel count of each transform (rounded up to 4 so vector
// reads of 4 consecutive channels stay 16-byte aligned):
//   BN_ACT: v = lrelu(t*a + b)   BN_DY: v = a*t + b*aux + c   epilogue BN_ACT: x̂ = y*p + q
struct Tab {
  float *a, *b, *c, *p, *q;
};

__host__ __device__ inline int tab_pad(int c) { return (c + 3) & ~3; }
// Each table row is followed by 8 zero entries (the "zero slot" at index tab_pad(C)): a packed
// group that is out of range points its channel there, so any transform maps it to exactly 0.
__host__ __device__ inline int tab_stride(int c) { return tab_pad(c) + 8; }

// A BatchNorm table built by the consuming workgroup from the producer's replicated statistics
// (no vae_bn_finalize launch): all 256 threads call it in uniform control flow.  Every replica
// element is loaded in one round (reps * C <= 1024 per statistic, C dividing 256 or a multiple
// of it: host-checked, bn_fast_ok), partials meet in LDS and are summed in a fixed order, so
// every workgroup of every consumer derives bit-identical coefficients.
__host__ __device__ inline bool bn_fast_ok(const vae_xform& x) {
  const int C = x.channels, R = x.reps > 1 ? x.reps : 1;
  if (C <= 0 || C > 512 || R * C > 1024 || (x.reps > 1 && x.rstride < C)) return false;   // (finish: <= 2 channels a thread)
  return C <= 256 ? (256 % C == 0) : (C % 256 == 0);
}

// The build split in two so a kernel can issue the table's loads BEFORE its operand loads and
// reduce them after: vmcnt counts in issue order, so table loads issued behind the operand ring
// wait for every operand load in flight.  TabPre<NS> holds the loaded replicas of the NS
// statistics the transform needs (2: Σ, Σ² for BN_ACT; 4: + Σg·x̂, Σg for BN_DY) and gamma /
// beta / shift of the thread's first channel — few registers, since they stay live across the
// operand loads (C = 512's second channel and the running statistics are loaded in the finish).
// The LDS scratch of the reduction (1024 floats) is passed in: a kernel hands it a region of its
// operand tiles that is not in use yet, so the table costs no LDS of its own.
template <int NS>
struct TabPre {
  float v[NS][4];
  float g, be, sh;
};

template <int NS>
__device__ __forceinline__ void tab_pre_load(const vae_xform& x, TabPre<NS>& q) {
  const int C = x.channels, R = x.reps > 1 ? x.reps : 1, tid = threadIdx.x;
  const long rs = x.reps > 1 ? x.rstride : 0;
  const int total = R * C;
  const float* arr[4] = {x.sum, x.sumsq, x.dgamma, x.dbeta};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int f = tid + 256 * k;
    const bool ok = f < total;
    const int r = ok ? f / C : 0, c = ok ? f - r * C : 0;
    const long o = (long)r * rs + c;
#pragma unroll
    for (int a = 0; a < NS; ++a) q.v[a][k] = ok ? arr[a][o] : 0.f;
  }
  const int ch = tid < C ? tid : C - 1;
  q.g = x.gamma[ch];
  q.be = x.beta[ch];
  q.sh = x.shift ? x.shift[ch] : 0.0f;
}

template <int NS>
__device__ __forceinline__ void tab_pre_finish(const vae_xform& x, const TabPre<NS>& q, Tab t, bool epi,
                                               bool update_running, float* scr) {
  const int C = x.channels, R = x.reps > 1 ? x.reps : 1, tid = threadIdx.x;
  // channel totals: C <= 256 -> every element of a thread is channel tid % C; C = 256k -> the
  // thread's elements are channels tid + 256j, each complete after summing its replicas
  float tot[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int a = 0; a < 4; ++a) tot[j][a] = 0.f;
  int nch = 1;
  if (C <= 256) {
#pragma unroll
    for (int a = 0; a < NS; ++a) scr[a * 256 + tid] = (q.v[a][0] + q.v[a][1]) + (q.v[a][2] + q.v[a][3]);
    __syncthreads();
    if (tid < C) {
#pragma unroll
      for (int a = 0; a < NS; ++a) {
        float acc = 0.f;
        for (int j = tid; j < 256; j += C) acc += scr[a * 256 + j];
        tot[0][a] = acc;
      }
    }
    __syncthreads();                            // scr is free for the next table of this workgroup
    nch = tid < C ? 1 : 0;
  } else {
    const int per = C / 256;                    // channels per thread (2 for C = 512)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int a = 0; a < NS; ++a) {
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) acc += ((k % per) == j && k / per < R) ? q.v[a][k] : 0.f;
        tot[j][a] = acc;
      }
    nch = per;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (j >= nch) break;
    const int ch = C <= 256 ? tid : tid + 256 * j;
    const float g = j == 0 ? q.g : x.gamma[ch];
    const float be = j == 0 ? q.be : x.beta[ch];
    const float sh = j == 0 ? q.sh : (x.shift ? x.shift[ch] : 0.0f);
    const float inv_m = 1.0f / x.count;
    const float s1 = tot[j][0] * inv_m;
    const float var = fmaxf(tot[j][1] * inv_m - s1 * s1, 0.0f);
    const float mean = s1 + sh;
    const float invstd = 1.0f / sqrtf(var + x.eps);
    if (x.kind == VAE_X_BN_ACT) {
      const float sc = g * invstd;
      t.a[ch] = sc;
      t.b[ch] = be - mean * sc;
      if (epi) { t.p[ch] = invstd; t.q[ch] = -mean * invstd; }
      if (update_running && x.running_mean) {
        const float m = x.momentum;
        const float unb = x.count > 1.f ? var * x.count / (x.count - 1.f) : var;
        x.running_mean[ch] = (1.f - m) * x.running_mean[ch] + m * mean;
        x.running_var[ch] = (1.f - m) * x.running_var[ch] + m * unb;
      }
    } else {
      const float A = g * invstd;
      const float mg = tot[j][3] * inv_m, mgx = tot[j][2] * inv_m;
      t.a[ch] = A;
      t.b[ch] = -A * invstd * mgx;
      t.c[ch] = -A * (mg - mean * invstd * mgx);
    }
  }
}

// Both halves at once, with the caller's LDS scratch (1024 floats).
__device__ __forceinline__ void tab_build(const vae_xform& x, Tab t, bool epi, bool update_running, float* scr) {
  if (x.kind == VAE_X_BN_DY) {
    TabPre<4> q;
    tab_pre_load(x, q);
    tab_pre_finish(x, q, t, epi, update_running, scr);
  } else {
    TabPre<2> q;
    tab_pre_load(x, q);
    tab_pre_finish(x, q, t, epi, update_running, scr);
  }
}

// ... with a scratch array of its own (kernels without a free LDS region at that point)
__device__ __forceinline__ void tab_build(const vae_xform& x, Tab t, bool epi, bool update_running) {
  __shared__ float scr[4 * 256];
  tab_build(x, t, epi, update_running, scr);
}

// One 64x64 (a, b) tile of one tap of a swapped-axes weight copy (vae_swap_axes): dst[b][tap][a] =
// bf16(src[a][tap][b]) (src fp32, or already bf16) through a padded LDS tile.  Each lane moves an
// element PAIR, so a wave's 32 lanes of a row read or write one 128-byte
// segment (32x32 tiles of single elements made 64-byte segments and four times the workgroups:
// 8.7 us for the VanillaVAE step's copies, tools/beginbench.py).  blk < swap_tiles(d).
constexpr int kSwapT = 64;
__host__ __device__ inline int swap_tiles(const vae_swap_desc& d) {
  return ((d.a + kSwapT - 1) / kSwapT) * ((d.b + kSwapT - 1) / kSwapT) * d.rs;
}
__device__ __forceinline__ void swap_tile(const vae_swap_desc& d, int blk, float (*t)[kSwapT + 1]) {
  const int nb = (d.b + kSwapT - 1) / kSwapT, na = (d.a + kSwapT - 1) / kSwapT;
  const int bt = blk % nb; blk /= nb;
  const int at = blk % na;
  const int tap = blk / na;
  const int a0 = at * kSwapT, b0 = bt * kSwapT;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  // rows a of the source tile: lane tx takes columns b0 + 2 tx, +1 — one 4-byte (bf16) / 8-byte
  // (fp32) access when b is even (every channel count but the 3-channel RGB ends), else two
  const bool vb = (d.b & 1) == 0, va = (d.a & 1) == 0;
#pragma unroll
  for (int j = ty; j < kSwapT; j += 8) {
    const int a = a0 + j, b = b0 + 2 * tx;
    const long i = ((long)a * d.rs + tap) * d.b + b;
    float v0 = 0.f, v1 = 0.f;
    if (a < d.a && b < d.b) {
      if (d.src_dtype == VAE_BF16) {
        const __bf16* sp = static_cast<const __bf16*>(d.src) + i;
        if (vb) { const bf16x2 q = *reinterpret_cast<const bf16x2*>(sp); v0 = (float)q[0]; v1 = (float)q[1]; }
        else { v0 = (float)sp[0]; v1 = b + 1 < d.b ? (float)sp[1] : 0.f; }
      } else {
        const float* sp = static_cast<const float*>(d.src) + i;
        if (vb) { const f32x2 q = *reinterpret_cast<const f32x2*>(sp); v0 = q[0]; v1 = q[1]; }
        else { v0 = sp[0]; v1 = b + 1 < d.b ? sp[1] : 0.f; }
      }
    }
    t[j][2 * tx] = v0;
    t[j][2 * tx + 1] = v1;
  }
  __syncthreads();
  __bf16* dst = static_cast<__bf16*>(d.dst);
#pragma unroll
  for (int j = ty; j < kSwapT; j += 8) {
    const int b = b0 + j, a = a0 + 2 * tx;
    if (a < d.a && b < d.b) {
      __bf16* dp = dst + ((long)b * d.rs + tap) * d.a + a;
      if (va) {
        bf16x2 o;
        o[0] = (__bf16)t[2 * tx][j];
        o[1] = (__bf16)t[2 * tx + 1][j];
        *reinterpret_cast<bf16x2*>(dp) = o;
      } else {
        dp[0] = (__bf16)t[2 * tx][j];
        if (a + 1 < d.a) dp[1] = (__bf16)t[2 * tx + 1][j];
      }
    }
  }
}

}  // namespace vae

