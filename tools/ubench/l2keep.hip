// Does a kernel's output stay in its XCD's L2 for the next kernel on the same XCD? (diagnostic)
//
//   hipcc -O3 --offload-arch=gfx950 tools/ubench/l2keep.hip -o tools/ubench/l2keep && tools/ubench/l2keep
//
// 8 regions of R bytes; workgroup b works on region (b % 8) (the XCD it runs on under round-robin
// placement), local part b / 8.  Times a reading kernel after: (a) a write of the same regions by the
// same XCDs, (b) a write with every region written by the NEXT XCD, (c) a read of the same regions,
// (d) a write of other buffers (cold).
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void __launch_bounds__(256) touch(float4* buf, size_t region_f4, int shift, int write, float* sink) {
  const int x = (blockIdx.x + shift) & 7, loc = blockIdx.x >> 3, nloc = gridDim.x >> 3;
  float4* r = buf + (size_t)x * region_f4;
  const size_t per = region_f4 / nloc;
  float acc = 0.f;
  for (size_t i = (size_t)loc * per + threadIdx.x; i < (size_t)(loc + 1) * per; i += 256 * 4) {
    if (write) {
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (i + u * 256 < (size_t)(loc + 1) * per) r[i + u * 256] = make_float4(1.f, 2.f, 3.f, (float)u);
    } else {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = i + u * 256 < (size_t)(loc + 1) * per ? r[i + u * 256] : make_float4(0, 0, 0, 0);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc += v[u].x + v[u].w;
    }
  }
  if (acc == 1234.5f) sink[0] = acc;
}

int main() {
  const size_t region = 1u << 20;              // bytes per XCD (8 MB total)
  const size_t f4 = region / 16;
  float4 *a, *cold;
  float* sink;
  hipMalloc(&a, 8 * region);
  hipMalloc(&cold, 512u << 20);
  hipMalloc(&sink, 64);
  const int blocks = 512;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto timed_read = [&](const char* what, auto&& before) {
    float tot = 0.f;
    const int reps = 20;
    for (int i = 0; i < reps; ++i) {
      before();
      hipEventRecord(e0);
      touch<<<blocks, 256>>>(a, f4, 0, 0, sink);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      tot += ms;
    }
    printf("%-48s read of 8 x %zu KB: %7.2f us\n", what, region >> 10, tot * 1000.f / reps);
  };
  auto flush = [&]() { touch<<<blocks, 256>>>(cold, (512u << 20) / 16 / 8, 0, 1, sink); };
  timed_read("after flush (cold)", [&]() { flush(); });
  timed_read("after write, same XCD mapping", [&]() { flush(); touch<<<blocks, 256>>>(a, f4, 0, 1, sink); });
  timed_read("after write, regions written by the next XCD", [&]() { flush(); touch<<<blocks, 256>>>(a, f4, 1, 1, sink); });
  timed_read("after read, same XCD mapping", [&]() { flush(); touch<<<blocks, 256>>>(a, f4, 0, 0, sink); });
  timed_read("after read, other XCD mapping", [&]() { flush(); touch<<<blocks, 256>>>(a, f4, 3, 0, sink); });
  timed_read("back to back (same kernel twice)", [&]() {});
  return 0;
}
