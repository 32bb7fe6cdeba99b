// C-ABI entry points of the convolution family and the linear layers.  Each one translates
// the reference-shaped descriptor (vaehip.h) into one implicit-GEMM problem (vae_igemm.hpp),
// picks a tile shape / split-K for the MI355X's 256 CUs, and launches on the caller's stream.
#include "vae_igemm.hpp"

namespace vae {

namespace {

constexpr int kCUs = 256;

vae_xform sanitize(vae_xform x) {
  if (x.channels <= 0) x.channels = 1;
  return x;
}

bool xf_ok(const vae_xform& x, const char* what) {
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
  if (x.kind == VAE_X_ACT && !(x.slope >= 0.f)) { fail(VAE_E_BADARG, "%s: bad slope", what); return false; }
  return true;
}

// Phase tap tables of a transposed conv (or conv dgrad) with stride S, kernel R, padding P:
// output coordinate o of phase ph = o % S receives taps r with (ph + P - r) % S == 0.
bool make_taps(GemmParams& p, int S, int R, int P) {
  if (S < 1 || S > 2) return false;
  for (int ph = 0; ph < S; ++ph) {
    int n = 0;
    for (int r = 0; r < R; ++r)
      if (((ph + P - r) % S + S) % S == 0) {
        if (n >= 4) return false;
        p.tap_h[ph][n] = r; p.tap_w[ph][n] = r; ++n;
      }
    p.ntap_h[ph] = n; p.ntap_w[ph] = n;
  }
  return true;
}

struct Tile { int bm, bn; };

// Largest tile that still gives >= kCUs blocks; fall back to the smallest.
Tile pick_tile(long M, long N, int nphase, bool allow_big) {
  const Tile cands[] = {{64, 64}, {64, 32}, {32, 64}, {32, 32}};
  for (const Tile& t : cands) {
    if (!allow_big && t.bm * t.bn > 64 * 32) continue;
    const long blocks = ((M + t.bm - 1) / t.bm) * ((N + t.bn - 1) / t.bn) * nphase;
    if (blocks >= kCUs) return t;
  }
  return {32, 32};
}

template <class T, class TA, class TB, int AM, int BMD, int EM>
int launch_tiled(const GemmParams& p, Tile t, int gz, hipStream_t st) {
  const dim3 block(NTHREADS);
  const dim3 grid((p.M + t.bm - 1) / t.bm, (p.N + t.bn - 1) / t.bn, gz);
  if (t.bm == 64 && t.bn == 64)
    hipLaunchKernelGGL((igemm_kernel<T, TA, TB, 64, 64, AM, BMD, EM>), grid, block, 0, st, p);
  else if (t.bm == 64 && t.bn == 32)
    hipLaunchKernelGGL((igemm_kernel<T, TA, TB, 64, 32, AM, BMD, EM>), grid, block, 0, st, p);
  else if (t.bm == 32 && t.bn == 64)
    hipLaunchKernelGGL((igemm_kernel<T, TA, TB, 32, 64, AM, BMD, EM>), grid, block, 0, st, p);
  else
    hipLaunchKernelGGL((igemm_kernel<T, TA, TB, 32, 32, AM, BMD, EM>), grid, block, 0, st, p);
  return check_launch("igemm");
}

template <int AM, int BMD, int EM>
int launch(int dtype, bool a_f32, bool b_f32, const GemmParams& p, Tile t, int gz, hipStream_t st) {
  if (p.M <= 0 || p.N <= 0) return VAE_OK;
  if (dtype == VAE_F32) return launch_tiled<float, float, float, AM, BMD, EM>(p, t, gz, st);
  if (dtype != VAE_BF16) return fail(VAE_E_BADDTYPE, "dtype %d", dtype);
  if (a_f32) return launch_tiled<__bf16, float, __bf16, AM, BMD, EM>(p, t, gz, st);
  if (b_f32) return launch_tiled<__bf16, __bf16, float, AM, BMD, EM>(p, t, gz, st);
  return launch_tiled<__bf16, __bf16, __bf16, AM, BMD, EM>(p, t, gz, st);
}

GemmParams base_params() {
  GemmParams p;
  memset(&p, 0, sizeof(p));
  p.ksplit = 1; p.nphase = 1; p.ones_col = -1; p.gs = 1; p.samples = 1;
  p.a_xf.channels = 1; p.b_xf.channels = 1; p.epi_xf.channels = 1; p.res_xf.channels = 1;
  return p;
}

int split_for(long blocks, int ktiles) {
  // enough blocks to cover the CUs twice, but keep >= 4 K-tiles per split
  int s = (int)((2 * kCUs + blocks - 1) / blocks);
  s = s < 1 ? 1 : s;
  const int maxs = ktiles / 4 > 0 ? ktiles / 4 : 1;
  return s > maxs ? maxs : s;
}

// A backward epilogue that differentiates an activation must be given the stored
// pre-activation tensor (aux); a NULL there would be a device fault, so reject it here.
bool epi_ok(const vae_xform& x, const char* what) {
  if (!xf_ok(x, what)) return false;
  if ((x.kind == VAE_X_BN_ACT || x.kind == VAE_X_ACT) && !x.aux) {
    fail(VAE_E_BADARG, "%s: activation-backward epilogue needs aux (the stored pre-activation)", what);
    return false;
  }
  if (x.kind == VAE_X_BN_DY) { fail(VAE_E_BADARG, "%s: BN_DY is not an epilogue transform", what); return false; }
  return true;
}

bool geom_ok(const vae_conv_args* a, const char* what) {
  if (!a) { fail(VAE_E_BADARG, "%s: null args", what); return false; }
  if (a->n <= 0 || a->h <= 0 || a->w <= 0 || a->c <= 0 || a->k <= 0 || a->p <= 0 || a->q <= 0 || a->r <= 0 ||
      a->stride <= 0 || a->pad < 0) {
    fail(VAE_E_BADSHAPE, "%s: bad geometry", what); return false;
  }
  return true;
}

// BN_DY on dy means the bias gradient has the closed form Σdy = A·Σg + B·Σy + C·M per channel
__global__ void bias_grad_closed_form(vae_xform x, float* db) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= x.channels) return;
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

// Column sums of a plain [rows][C] tensor (bias gradient of a layer whose dy is stored as is)
template <class T>
__global__ void column_sum(const T* x, long rows, int C, float* out) {
  const int c = blockIdx.y * 64 + (threadIdx.x & 63);
  if (c >= C) return;
  float s = 0.f;
  for (long r = blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += (long)gridDim.x * 4) s += ld_f(x + r * C + c);
  atomicAdd(out + c, s);
}

int bias_grad(int dtype, const vae_xform& dyxf, const void* dy, long rows, int C, float* db, hipStream_t st) {
  if (!db) return VAE_OK;
  if (dyxf.kind == VAE_X_BN_DY) {
    hipLaunchKernelGGL(bias_grad_closed_form, dim3((C + 255) / 256), dim3(256), 0, st, dyxf, db);
  } else {
    const dim3 grid(64, (C + 63) / 64);
    if (dtype == VAE_F32) hipLaunchKernelGGL(column_sum<float>, grid, dim3(256), 0, st, (const float*)dy, rows, C, db);
    else hipLaunchKernelGGL(column_sum<__bf16>, grid, dim3(256), 0, st, (const __bf16*)dy, rows, C, db);
  }
  return check_launch("bias_grad");
}

}  // namespace

}  // namespace vae

using namespace vae;

// ============================================================================ Conv2d
// y[n,p,q,k] = Σ_{r,s,c} xf(x)[n, p*S-P+r, q*S-P+s, c] · W[k][r][s][c] + b[k]
extern "C" int vae_conv2d_fwd(const vae_conv_args* a, void* stream) {
  if (!geom_ok(a, "conv2d_fwd") || !a->x || !a->wt || !a->y) return fail(VAE_E_BADARG, "conv2d_fwd: null tensor");
  if (!xf_ok(a->x_xf, "conv2d_fwd.x")) return VAE_E_BADARG;
  GemmParams p = base_params();
  p.M = a->n * a->p * a->q; p.N = a->k; p.K = a->r * a->r * a->c;
  p.a_ptr = a->x; p.a_xf = sanitize(a->x_xf); p.g_nchw = a->x_nchw_f32;
  p.b_ptr = a->wt; p.b_ld = p.K;
  p.gn = a->n; p.gh = a->h; p.gw = a->w; p.gc = a->c; p.gp = a->p; p.gq = a->q;
  p.gr = a->r; p.gs = a->stride; p.gpad = a->pad;
  p.out = a->y; p.out_ld = a->k; p.bias = a->bias; p.sum = a->y_sum; p.sumsq = a->y_sumsq;
  p.residual = a->residual; p.res_xf = sanitize(a->residual_xf);
  const Tile t = pick_tile(p.M, p.N, 1, true);
  return launch<A_CONV, B_NK, E_STORE>(a->dtype, a->x_nchw_f32 != 0, false, p, t, 1, (hipStream_t)stream);
}

// dx[n,h,w,c] = Σ_{r,s,k: h = p*S-P+r} dy'[n,p,q,k] · W[k][r][s][c]  (transposed conv of dy);
// epilogue: g = dx·act'(z) of x's BatchNorm/LeakyReLU, Σg -> dβ, Σg·x̂ -> dγ
extern "C" int vae_conv2d_bwd_data(const vae_conv_args* a, void* stream) {
  if (!geom_ok(a, "conv2d_bwd_data") || !a->dy || !a->wt || !a->dx) return fail(VAE_E_BADARG, "conv2d_bwd_data: null tensor");
  if (!xf_ok(a->dy_xf, "conv2d_bwd_data.dy") || !epi_ok(a->dx_epi, "conv2d_bwd_data.epi")) return VAE_E_BADARG;
  if (a->x_nchw_f32) return fail(VAE_E_UNSUPPORTED, "conv2d_bwd_data: no gradient for the NCHW image input");
  const int S = a->stride;
  if (a->h % S || a->w % S || a->h / S != a->p || a->w / S != a->q)
    return fail(VAE_E_BADSHAPE, "conv2d_bwd_data: needs h == p*stride (got h=%d p=%d S=%d)", a->h, a->p, S);
  GemmParams p = base_params();
  if (!make_taps(p, S, a->r, a->pad)) return fail(VAE_E_UNSUPPORTED, "conv2d_bwd_data: stride/kernel");
  p.nphase = S * S;
  p.M = a->n * (a->h / S) * (a->w / S); p.N = a->c; p.K = 0;
  p.a_ptr = a->dy; p.a_xf = sanitize(a->dy_xf);
  p.b_ptr = a->wt; p.b_ld = a->c; p.b_taps = 1;
  p.gn = a->n; p.gh = a->p; p.gw = a->q; p.gc = a->k;          // gathered tensor = dy
  p.gp = a->h / S; p.gq = a->w / S; p.gr = a->r; p.gs = S; p.gpad = a->pad; p.gho = a->h; p.gwo = a->w;
  p.out = a->dx; p.out_ld = a->c; p.out_phase = 1;
  p.epi_xf = sanitize(a->dx_epi); p.dgamma = a->dx_dgamma; p.dbeta = a->dx_dbeta;
  if (p.epi_xf.kind == VAE_X_BN_ACT && (!p.dgamma || !p.dbeta)) return fail(VAE_E_BADARG, "conv2d_bwd_data: dgamma/dbeta");
  const Tile t = pick_tile(p.M, p.N, p.nphase, true);
  return launch<A_CONVT, B_KN, E_BNBWD>(a->dtype, false, false, p, t, p.nphase, (hipStream_t)stream);
}

// dW[k][r][s][c] += Σ_{n,p,q} dy'[n,p,q,k] · xf(x)[n, p*S-P+r, q*S-P+s, c];  db[k] += Σ dy'
extern "C" int vae_conv2d_bwd_filter(const vae_conv_args* a, void* stream) {
  if (!geom_ok(a, "conv2d_bwd_filter") || !a->dy || !a->x || !a->dw) return fail(VAE_E_BADARG, "conv2d_bwd_filter: null tensor");
  if (!xf_ok(a->dy_xf, "conv2d_bwd_filter.dy") || !xf_ok(a->x_xf, "conv2d_bwd_filter.x")) return VAE_E_BADARG;
  GemmParams p = base_params();
  const int Nw = a->r * a->r * a->c;
  const bool ones = a->db && a->dy_xf.kind != VAE_X_BN_DY;
  p.M = a->k; p.N = Nw + (ones ? 1 : 0); p.K = a->n * a->p * a->q;
  p.ones_col = ones ? Nw : -1; p.bias_grad = ones ? a->db : nullptr;
  p.a_ptr = a->dy; p.a_ld = a->k; p.a_xf = sanitize(a->dy_xf);
  p.b_ptr = a->x; p.b_xf = sanitize(a->x_xf); p.g_nchw = a->x_nchw_f32;
  p.gn = a->n; p.gh = a->h; p.gw = a->w; p.gc = a->c; p.gp = a->p; p.gq = a->q;
  p.gr = a->r; p.gs = a->stride; p.gpad = a->pad;
  p.out = a->dw; p.out_ld = Nw;
  const Tile t = pick_tile(p.M, p.N, 1, true);
  const long blocks = (long)((p.M + t.bm - 1) / t.bm) * ((p.N + t.bn - 1) / t.bn);
  p.ksplit = a->split_k > 0 ? a->split_k : split_for(blocks, (p.K + BK - 1) / BK);
  int rc = launch<A_KM, B_GATHER, E_ACC>(a->dtype, false, a->x_nchw_f32 != 0, p, t, p.ksplit, (hipStream_t)stream);
  if (rc) return rc;
  if (a->db && !ones) return bias_grad(a->dtype, a->dy_xf, a->dy, (long)a->n * a->p * a->q, a->k, a->db, (hipStream_t)stream);
  return VAE_OK;
}

// ==================================================================== ConvTranspose2d
// y[n,ho,wo,k] = Σ_{r,s,c: ho = h*S-P+r} xf(x)[n,h,w,c] · W[c][r][s][k] + b[k]   (phase GEMMs)
extern "C" int vae_convT2d_fwd(const vae_conv_args* a, void* stream) {
  if (!geom_ok(a, "convT2d_fwd") || !a->x || !a->wt || !a->y) return fail(VAE_E_BADARG, "convT2d_fwd: null tensor");
  if (!xf_ok(a->x_xf, "convT2d_fwd.x")) return VAE_E_BADARG;
  const int S = a->stride;
  if (a->p % S || a->q % S) return fail(VAE_E_BADSHAPE, "convT2d_fwd: output not a multiple of stride");
  GemmParams p = base_params();
  if (!make_taps(p, S, a->r, a->pad)) return fail(VAE_E_UNSUPPORTED, "convT2d_fwd: stride/kernel");
  p.nphase = S * S;
  p.M = a->n * (a->p / S) * (a->q / S); p.N = a->k; p.K = 0;
  p.a_ptr = a->x; p.a_xf = sanitize(a->x_xf);
  p.b_ptr = a->wt; p.b_ld = a->k; p.b_taps = 1;
  p.gn = a->n; p.gh = a->h; p.gw = a->w; p.gc = a->c;
  p.gp = a->p / S; p.gq = a->q / S; p.gr = a->r; p.gs = S; p.gpad = a->pad; p.gho = a->p; p.gwo = a->q;
  p.out = a->y; p.out_ld = a->k; p.out_phase = 1; p.bias = a->bias; p.sum = a->y_sum; p.sumsq = a->y_sumsq;
  p.residual = a->residual; p.res_xf = sanitize(a->residual_xf);
  const Tile t = pick_tile(p.M, p.N, p.nphase, true);
  return launch<A_CONVT, B_KN, E_STORE>(a->dtype, false, false, p, t, p.nphase, (hipStream_t)stream);
}

// dx[n,h,w,c] = Σ_{r,s,k} dy'[n, h*S-P+r, w*S-P+s, k] · W[c][r][s][k]   (strided conv of dy)
extern "C" int vae_convT2d_bwd_data(const vae_conv_args* a, void* stream) {
  if (!geom_ok(a, "convT2d_bwd_data") || !a->dy || !a->wt || !a->dx) return fail(VAE_E_BADARG, "convT2d_bwd_data: null tensor");
  if (!xf_ok(a->dy_xf, "convT2d_bwd_data.dy") || !epi_ok(a->dx_epi, "convT2d_bwd_data.epi")) return VAE_E_BADARG;
  GemmParams p = base_params();
  p.M = a->n * a->h * a->w; p.N = a->c; p.K = a->r * a->r * a->k;
  p.a_ptr = a->dy; p.a_xf = sanitize(a->dy_xf);
  p.b_ptr = a->wt; p.b_ld = p.K;
  p.gn = a->n; p.gh = a->p; p.gw = a->q; p.gc = a->k; p.gp = a->h; p.gq = a->w;
  p.gr = a->r; p.gs = a->stride; p.gpad = a->pad;
  p.out = a->dx; p.out_ld = a->c;
  p.epi_xf = sanitize(a->dx_epi); p.dgamma = a->dx_dgamma; p.dbeta = a->dx_dbeta;
  if (p.epi_xf.kind == VAE_X_BN_ACT && (!p.dgamma || !p.dbeta)) return fail(VAE_E_BADARG, "convT2d_bwd_data: dgamma/dbeta");
  const Tile t = pick_tile(p.M, p.N, 1, true);
  return launch<A_CONV, B_NK, E_BNBWD>(a->dtype, false, false, p, t, 1, (hipStream_t)stream);
}

// dW[c][r][s][k] += Σ_{n,h,w} xf(x)[n,h,w,c] · dy'[n, h*S-P+r, w*S-P+s, k];  db[k] += Σ dy'
extern "C" int vae_convT2d_bwd_filter(const vae_conv_args* a, void* stream) {
  if (!geom_ok(a, "convT2d_bwd_filter") || !a->dy || !a->x || !a->dw) return fail(VAE_E_BADARG, "convT2d_bwd_filter: null tensor");
  if (!xf_ok(a->dy_xf, "convT2d_bwd_filter.dy") || !xf_ok(a->x_xf, "convT2d_bwd_filter.x")) return VAE_E_BADARG;
  GemmParams p = base_params();
  const int Nw = a->r * a->r * a->k;
  p.M = a->c; p.N = Nw; p.K = a->n * a->h * a->w;
  p.a_ptr = a->x; p.a_ld = a->c; p.a_xf = sanitize(a->x_xf);
  p.b_ptr = a->dy; p.b_xf = sanitize(a->dy_xf);
  p.gn = a->n; p.gh = a->p; p.gw = a->q; p.gc = a->k; p.gp = a->h; p.gq = a->w;
  p.gr = a->r; p.gs = a->stride; p.gpad = a->pad;
  p.out = a->dw; p.out_ld = Nw;
  const Tile t = pick_tile(p.M, p.N, 1, true);
  const long blocks = (long)((p.M + t.bm - 1) / t.bm) * ((p.N + t.bn - 1) / t.bn);
  p.ksplit = a->split_k > 0 ? a->split_k : split_for(blocks, (p.K + BK - 1) / BK);
  int rc = launch<A_KM, B_GATHER, E_ACC>(a->dtype, false, false, p, t, p.ksplit, (hipStream_t)stream);
  if (rc) return rc;
  return bias_grad(a->dtype, a->dy_xf, a->dy, (long)a->n * a->p * a->q, a->k, a->db, (hipStream_t)stream);
}

// ============================================================================= Linear
extern "C" int vae_linear_fwd(const vae_linear_args* a, void* stream) {
  if (!a || !a->x || !a->wt || !a->y || a->m <= 0 || a->n <= 0 || a->k <= 0) return fail(VAE_E_BADARG, "linear_fwd: args");
  if (!xf_ok(a->x_xf, "linear_fwd.x")) return VAE_E_BADARG;
  GemmParams p = base_params();
  p.M = a->m; p.N = a->n; p.K = a->k;
  p.a_ptr = a->x; p.a_ld = a->k; p.a_xf = sanitize(a->x_xf);
  p.b_ptr = a->wt; p.b_ld = a->k;
  p.out = a->y; p.out_ld = a->n; p.bias = a->bias; p.out_f32 = a->y_f32;
  const Tile t = pick_tile(p.M, p.N, 1, false);
  return launch<A_DENSE, B_NK, E_STORE>(a->dtype, false, false, p, t, 1, (hipStream_t)stream);
}

// dx[m][k] = Σ_n dy[m][n] · W[n][k];  epilogue: activation backward (dx_epi) or, when
// mulv is set, the reparameterization + KL backward into dmulv
extern "C" int vae_linear_bwd_data(const vae_linear_args* a, void* stream) {
  if (!a || !a->dy || !a->wt || a->m <= 0 || a->n <= 0 || a->k <= 0) return fail(VAE_E_BADARG, "linear_bwd_data: args");
  if (!a->mulv && !epi_ok(a->dx_epi, "linear_bwd_data.epi")) return VAE_E_BADARG;
  GemmParams p = base_params();
  p.M = a->m; p.N = a->k; p.K = a->n;
  p.a_ptr = a->dy; p.a_ld = a->n;
  p.b_ptr = a->wt; p.b_ld = a->k;
  p.out = a->dx; p.out_ld = a->k;
  const Tile t = pick_tile(p.M, p.N, 1, false);
  if (a->mulv) {
    if (!a->eps || !a->dmulv || a->samples <= 0) return fail(VAE_E_BADARG, "linear_bwd_data: reparam args");
    p.mulv = a->mulv; p.eps = a->eps; p.kl_coef = a->kl_coef; p.dmulv = a->dmulv;
    p.samples = a->samples; p.latent = a->k;
    return launch<A_DENSE, B_KN, E_REPARAM>(a->dtype, a->dy_f32 != 0, false, p, t, 1, (hipStream_t)stream);
  }
  if (!a->dx) return fail(VAE_E_BADARG, "linear_bwd_data: dx");
  p.epi_xf = sanitize(a->dx_epi); p.dgamma = a->dx_dgamma; p.dbeta = a->dx_dbeta;
  if (p.epi_xf.kind == VAE_X_BN_ACT && (!p.dgamma || !p.dbeta)) return fail(VAE_E_BADARG, "linear_bwd_data: dgamma/dbeta");
  return launch<A_DENSE, B_KN, E_BNBWD>(a->dtype, a->dy_f32 != 0, false, p, t, 1, (hipStream_t)stream);
}

// dW[n][k] += Σ_m dy[m][n] · xf(x)[m][k];  db[n] += Σ_m dy[m][n]  (ones column)
extern "C" int vae_linear_bwd_filter(const vae_linear_args* a, void* stream) {
  if (!a || !a->dy || !a->x || !a->dw || a->m <= 0 || a->n <= 0 || a->k <= 0) return fail(VAE_E_BADARG, "linear_bwd_filter: args");
  if (!xf_ok(a->x_xf, "linear_bwd_filter.x")) return VAE_E_BADARG;
  GemmParams p = base_params();
  p.M = a->n; p.N = a->k + (a->db ? 1 : 0); p.K = a->m;
  p.ones_col = a->db ? a->k : -1; p.bias_grad = a->db;
  p.a_ptr = a->dy; p.a_ld = a->n;
  p.b_ptr = a->x; p.b_ld = a->k; p.b_xf = sanitize(a->x_xf);
  p.out = a->dw; p.out_ld = a->k;
  const Tile t = pick_tile(p.M, p.N, 1, true);
  const long blocks = (long)((p.M + t.bm - 1) / t.bm) * ((p.N + t.bn - 1) / t.bn);
  p.ksplit = split_for(blocks, (p.K + BK - 1) / BK);
  return launch<A_KM, B_KN, E_ACC>(a->dtype, a->dy_f32 != 0, false, p, t, p.ksplit, (hipStream_t)stream);
}
