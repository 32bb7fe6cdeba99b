// The large transform-free bf16 conv GEMMs on the LDS-DMA pipeline (vae_bgemm.hip), reached from
// the conv-GEMM planner (vae_launch.hpp cg_launch) when bgemm_ok holds.
#pragma once
#include "vae_igemm.hpp"

namespace vae {
bool bgemm_ok(const GemmParams& p, int am, int em);
// kHeadFallback when the launch cannot take the shape after all (LDS budget); else a status
int bgemm_launch(const GemmParams& p, int am, int em, void* ws, long ws_bytes, hipStream_t st);
}  // namespace vae
