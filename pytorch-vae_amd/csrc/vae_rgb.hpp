// Launchers of the VQ-VAE RGB-end kernels (vae_rgb.hip).  Each returns kHeadFallback when the call
// is not the shape / transform its kernel takes (the caller then runs the general path).
#pragma once
#include "vae_common.hpp"

namespace vae {
int rgb_out_fwd_launch(const vae_conv_args* a, const vae_recon_args* rc, hipStream_t st);
int rgb_out_bwd_launch(const vae_conv_args* a, hipStream_t st);
int rgb_in_wgrad_launch(const vae_conv_args* a, hipStream_t st);
}  // namespace vae
