// Per-CU load throughput of the access shapes the VAE GEMMs use (diagnostic microbenchmark).
//
//   hipcc -O3 --offload-arch=gfx950 tools/ubench/loads.hip -o tools/ubench/loads && tools/ubench/loads
//
// Every workgroup (256 threads) issues LOADS 16-byte buffer loads per thread in flight, then sums
// them (so nothing is dead), ROUNDS times.  Shapes (one wave-instruction = 64 lanes x 16 B):
//   seg=1024: the wave reads 1 KB contiguous
//   seg=256 : 4 segments of 256 B in different rows (the conv-GEMM's 16 chunks of a K-step row)
//   seg=64  : 16 segments of 64 B (a 32-channel tap row)
// The working set is either L2-sized (2 MB, re-read by every workgroup) or streamed (256 MB).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef __amdgpu_buffer_rsrc_t rsrc_t;

__device__ __forceinline__ rsrc_t make_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

template <int LOADS>
__global__ void __launch_bounds__(256) load_kernel(const char* buf, unsigned bytes, int seg, int rounds,
                                                   unsigned wrap, float* out) {
  const rsrc_t r = make_rsrc(buf, bytes);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int per_seg = seg / 16;                       // lanes per contiguous segment
  const int s = lane / per_seg, l = lane % per_seg;
  // segment s of wave instruction i: a pseudo-random row (stride 4 KB + hashed) of the working set
  float acc = 0.f;
  for (int rd = 0; rd < rounds; ++rd) {
    uint32_t v[LOADS][4];
#pragma unroll
    for (int i = 0; i < LOADS; ++i) {
      const unsigned row = (unsigned)(blockIdx.x * 131 + wave * 977 + i * 61 + s * 7919 + rd * 104729);
      const unsigned off = ((row * 4096u) % wrap) + l * 16;
      uint32_t x[4];
      *(uint4*)x = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
      v[i][0] = x[0]; v[i][1] = x[1]; v[i][2] = x[2]; v[i][3] = x[3];
    }
#pragma unroll
    for (int i = 0; i < LOADS; ++i) acc += __uint_as_float(v[i][0] ^ v[i][1] ^ v[i][2] ^ v[i][3]) * 1e-30f;
  }
  if (acc == 123.f) out[blockIdx.x] = acc;
}

template <int LOADS>
float run(const char* buf, unsigned bytes, int seg, int blocks, int rounds, unsigned wrap, float* out) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  load_kernel<LOADS><<<blocks, 256>>>(buf, bytes, seg, rounds, wrap, out);
  hipEventRecord(a);
  const int reps = 20;
  for (int i = 0; i < reps; ++i) load_kernel<LOADS><<<blocks, 256>>>(buf, bytes, seg, rounds, wrap, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

int main() {
  const unsigned big = 256u << 20;
  char* buf;
  float* out;
  if (hipMalloc(&buf, big) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess) return 1;
  hipMemset(buf, 1, big);
  const int rounds = 8;
  for (unsigned wrap : {2u << 20, big}) {
    for (int blocks : {256, 512, 1024}) {
      for (int seg : {1024, 256, 64}) {
        float us4 = run<4>(buf, big, seg, blocks, rounds, wrap - 4096, out);
        float us8 = run<8>(buf, big, seg, blocks, rounds, wrap - 4096, out);
        float us20 = run<20>(buf, big, seg, blocks, rounds, wrap - 4096, out);
        auto gbs = [&](int loads, float us) {
          const double b = (double)blocks * 256 * 16 * loads * rounds;
          return b / (us * 1e-6) / 1e9;
        };
        printf("ws %4u MB blocks %4d seg %4d | 4 in flight %7.2f us %7.0f GB/s (%5.1f/CU) | 8: %7.2f us %7.0f GB/s (%5.1f/CU) | "
               "20: %7.2f us %7.0f GB/s (%5.1f/CU)\n",
               wrap >> 20, blocks, seg, us4, gbs(4, us4), gbs(4, us4) / 256, us8, gbs(8, us8), gbs(8, us8) / 256, us20,
               gbs(20, us20), gbs(20, us20) / 256);
      }
    }
  }
  return 0;
}
