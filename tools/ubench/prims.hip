// Microbenchmarks of the primitives the VAE step's kernels are built from (diagnostic tool):
// empty-kernel floor, same-address float atomics vs. number of adding workgroups, replicated
// atomics, and a chain of dependent global loads.  hipcc --offload-arch=gfx950 -O3 prims.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void empty_k() {}
// every workgroup: wave 0 adds one float per lane into ADDR[rep * 64 + lane]
__global__ void atomics_k(float* a, int reps, int per_block) {
  if (threadIdx.x >= 64) return;
  const int rep = blockIdx.x % reps;
  for (int i = 0; i < per_block; ++i) atomicAdd(a + rep * 64 * per_block + i * 64 + threadIdx.x, 1.0f);
}
// dependent chain of `n` global loads per lane
__global__ void chain_k(const int* nxt, int n, int* out) {
  int i = (blockIdx.x * blockDim.x + threadIdx.x) & 4095;
  for (int k = 0; k < n; ++k) i = nxt[i];
  if (i == -1) out[0] = i;
}

template <class F>
float timeit(F f, int iters = 200) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int i = 0; i < 20; ++i) f();
  hipEventRecord(a);
  for (int i = 0; i < iters; ++i) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / iters;
}

int main() {
  float* a; int* nxt; int* out;
  CK(hipMalloc(&a, 64 << 20)); CK(hipMalloc(&nxt, 4096 * 4)); CK(hipMalloc(&out, 4));
  CK(hipMemset(a, 0, 64 << 20));
  int h[4096];
  for (int i = 0; i < 4096; ++i) h[i] = (i * 1031 + 17) & 4095;
  CK(hipMemcpy(nxt, h, sizeof(h), hipMemcpyHostToDevice));
  for (int g : {1, 256, 1024, 4096})
    printf("empty kernel, %5d blocks: %.2f us/launch (back-to-back)\n", g, timeit([&] { hipLaunchKernelGGL(empty_k, dim3(g), dim3(256), 0, 0); }));
  for (int g : {64, 256, 1024, 4096})
    for (int r : {1, 8, 32})
      printf("atomics: %5d blocks x 64 lanes -> %2d replica(s) of 64 floats: %.2f us\n", g, r,
             timeit([&] { hipLaunchKernelGGL(atomics_k, dim3(g), dim3(256), 0, 0, a, r, 1); }));
  for (int g : {1024})
    for (int pb : {8, 32})
      printf("atomics: %5d blocks x %2d rows each (distinct rows per replica set, 1 replica): %.2f us\n", g, pb,
             timeit([&] { hipLaunchKernelGGL(atomics_k, dim3(g), dim3(256), 0, 0, a, 1, pb); }));
  for (int n : {1, 2, 4, 8, 16})
    printf("dependent global loads, chain %2d, 1024 blocks: %.2f us\n", n,
           timeit([&] { hipLaunchKernelGGL(chain_k, dim3(1024), dim3(256), 0, 0, nxt, n, out); }));
  return 0;
}
