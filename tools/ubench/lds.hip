// Microbenchmark: LDS atomic (ds_add_u32 / ds_or_b32) vs plain store/read
// throughput on lane-private, bank-conflict-free addresses (word w of lane l
// at lds[64 w + l]), 5 waves per CU, as the MI lane kernel uses them.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_lds.hip -o tools/ubench_lds
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kWords = 124;
constexpr int kIters = 4096;

template <int MODE>
__global__ __launch_bounds__(64) void k(unsigned seed, unsigned* out) {
  __shared__ unsigned lds[kWords * 64];
  unsigned* h = lds + threadIdx.x;
  for (int w = 0; w < kWords; ++w) h[64 * w] = 0;
  unsigned x = seed ^ (threadIdx.x * 2654435761u) ^ blockIdx.x;
  unsigned acc = 0;
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int w = (it * 7 + u * 13 + (x & 7)) & 63;  // independent per op
      if (MODE == 0) atomicAdd(&h[64 * w], 1u << (w & 24));
      if (MODE == 1) atomicOr(&h[64 * w], 1u << w);
      if (MODE == 2) h[64 * w] = w;
      if (MODE == 3) acc += h[64 * w];
      if (MODE == 4) acc ^= w;  // VALU only (address math)
    }
  }
  acc += h[64 * (x % 100)];
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  unsigned* d;
  hipMalloc(&d, 4);
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = 5 * ncu;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char* names[] = {"ds_add_u32", "ds_or_b32", "ds_write_b32", "ds_read_b32", "valu only"};
  for (int m = 0; m < 5; ++m) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a);
      if (m == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(64), 0, 0, 1u, d);
      if (m == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(64), 0, 0, 1u, d);
      if (m == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(64), 0, 0, 1u, d);
      if (m == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(64), 0, 0, 1u, d);
      if (m == 4) hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(64), 0, 0, 1u, d);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (rep == 1) {
        const double ops_per_cu = 5.0 * kIters * 8;  // wave-instructions per CU
        printf("%-14s %.3f ms  %.2f CU-cycles per wave-instruction (2.4 GHz)\n", names[m], ms,
               ms * 1e-3 * 2.4e9 / ops_per_cu);
      }
    }
  }
  return 0;
}
