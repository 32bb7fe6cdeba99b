// Does a kernel take an explicit argument block larger than 4 KB on this ROCm / gfx950?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
template <int N> struct Big { int v[N]; };
template <int N>
__global__ void copy_arg(Big<N> b, int* out) {
  const Big<N>* k = (const Big<N>*)__builtin_amdgcn_kernarg_segment_ptr();
  for (int i = threadIdx.x; i < N; i += blockDim.x) out[i] = k->v[i] + b.v[0] * 0;
}
template <int N> int run() {
  Big<N> b; for (int i = 0; i < N; ++i) b.v[i] = i * 7 + 3;
  int* d; if (hipMalloc(&d, N * 4) != hipSuccess) return 2;
  hipMemset(d, 0, N * 4);
  copy_arg<N><<<1, 256>>>(b, d);
  hipError_t e = hipDeviceSynchronize();
  int* h = new int[N]; hipMemcpy(h, d, N * 4, hipMemcpyDeviceToHost);
  int bad = 0; for (int i = 0; i < N; ++i) bad += h[i] != i * 7 + 3;
  printf("arg bytes %d: launch %s, mismatches %d\n", N * 4, hipGetErrorString(e), bad);
  hipFree(d); delete[] h; return bad || e != hipSuccess;
}
int main() { run<896>(); run<1024>(); run<1500>(); run<2000>(); return 0; }
