// 3x3 / stride-1 / pad-1 convolutions on a 16 x 16 grid (the VQ-VAE's residual stacks,
// models/vq_vae.py:57-70 ResidualLayer and the Conv3x3 around them, :94-166) — host interface of
// the image-tile kernel in vae_c3.hip.
#pragma once
#include "vae_common.hpp"

namespace vae {

struct C3Args {
  const void* a;            // [n][16][16][C] bf16 (x of a forward, dy of a data gradient)
  int a_act;                // LeakyReLU applied to A on load (forward of an activated input)
  float a_slope;
  const void* b;            // [N][3][3][C] bf16: W[k][r][s][c] (forward) or WT[c][r][s][k] (data gradient)
  int flip;                 // 0: out[h,w] = Σ A[h+r-1, w+s-1]·B[.][r][s];  1: Σ A[h+1-r, w+1-s]·B[.][r][s]
  void* out;                // [n][16][16][N] bf16
  const float* bias;        // [N] fp32 or NULL
  const void* residual;     // [n][16][16][N] bf16 or NULL: added before the activation backward
  const void* aux;          // [n][16][16][N] bf16 or NULL: g *= (aux > 0 ? 1 : aux_slope)
  float aux_slope;
  int n, C, N;
};

// The shapes the kernel takes: 16 x 16 grid, C % 32 == 0, N % 128 == 0, 16-byte aligned tensors.
bool c3_shape_ok(int n, int h, int w, int p, int q, int r, int stride, int pad, int C, int N);
// Launch (VAE_OK or an error code); the caller has checked c3_shape_ok and the transforms.
int c3_launch(const C3Args& a, hipStream_t st);
// Weight gradient of the same convolutions: dW[m][r][s][c] += Σ U[n,h,w,m] · xf(V)[n,h+r-1,w+s-1,c]
// (U = dy [n][16][16][M], V = x [n][16][16][J]); per-image-group partials in `ws` (c3w_workspace
// bytes), then reduced into dW.  M % 128 == 0, J % 32 == 0.
struct C3WArgs {
  const void* u;
  const void* v;
  int v_act;
  float v_slope;
  float* dw;
  int n, M, J;
};
bool c3w_shape_ok(int n, int h, int w, int p, int q, int r, int stride, int pad, int M, int J);
long c3w_workspace(int n, int M, int J);
int c3w_launch(const C3WArgs& a, void* ws, long ws_bytes, hipStream_t st);
// 1x1 stride-1 (pointwise) weight gradient on the same grid: dW[m][c] += Σ U[pix][m] · xf(V)[pix][c]
// (the ResidualLayer's Conv1x1); M % 128 == 0, J % 128 == 0; slab partials as c3w.
bool c1w_shape_ok(int n, int h, int w, int p, int q, int r, int stride, int pad, int M, int J);
int c1w_launch(const C3WArgs& a, void* ws, long ws_bytes, hipStream_t st);
// Pointwise (1x1 stride-1) conv forward / data gradient as a pixel-tile GEMM (vae_p1.hip):
//   out[pix][n] = Σ_c xf(A)[pix][c] · B[n][c] (+ bias, + xf(residual)) (* act'(aux))
// M (pixels) % 256 == 0, C % 128 == 0, N % 128 == 0, 16-byte aligned tensors.
struct P1Args {
  const void* a;
  int a_act;
  float a_slope;
  const void* b;            // [N][C] bf16
  void* out;                // [M][N] bf16
  const float* bias;
  const void* residual;
  int res_act;
  float res_slope;
  const void* aux;
  float aux_slope;
  long M;
  int C, N;
};
bool p1_shape_ok(long M, int C, int N);
int p1_launch(const P1Args& a, hipStream_t st);
// VAE_NO_C3=1 keeps these convolutions on the conv-GEMM (A/B timing)
bool c3_enabled();

}  // namespace vae
