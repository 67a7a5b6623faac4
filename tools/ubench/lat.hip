// Latency micro-benchmarks (dev tool): dependent FP64 ops, rsq, readlane, DPP, LDS round trips.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_fma(double* out, double a, long long* t) {
  double x = a + threadIdx.x;
  long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < 1024; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) x = fma(x, 0.999999, 1e-9);
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) t[0] = t1 - t0;
}
__global__ void k_fma32(float* out, float a, long long* t) {
  float x = a + threadIdx.x;
  long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < 1024; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) x = fmaf(x, 0.999999f, 1e-9f);
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) t[0] = t1 - t0;
}
__global__ void k_rsq(double* out, double a, long long* t) {
  double x = a + threadIdx.x;
  long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < 1024; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) x = __builtin_amdgcn_rsq(x) + 1.0;
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) t[0] = t1 - t0;
}
__global__ void k_readlane(double* out, double a, long long* t) {
  double x = a + threadIdx.x;
  long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < 1024; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      int lo = __builtin_amdgcn_readlane(__double2loint(x), 5);
      int hi = __builtin_amdgcn_readlane(__double2hiint(x), 5);
      x = __hiloint2double(hi, lo) * 0.999 + 1e-9;
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) t[0] = t1 - t0;
}
__global__ void k_bperm(double* out, double a, long long* t) {
  double x = a + threadIdx.x;
  long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < 1024; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) x = __shfl(x, (threadIdx.x + 7) & 63, 64) * 0.999 + 1e-9;
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) t[0] = t1 - t0;
}
__global__ void k_lds(double* out, double a, long long* t) {
  __shared__ double s[64];
  double x = a + threadIdx.x;
  long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < 1024; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s[threadIdx.x] = x;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      x = s[(threadIdx.x + 7) & 63] * 0.999 + 1e-9;
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) t[0] = t1 - t0;
}
__global__ void k_barrier(double* out, double a, long long* t) {
  __shared__ double s[512];
  double x = a + threadIdx.x;
  long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < 1024; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s[threadIdx.x] = x;
      __syncthreads();
      x = s[(threadIdx.x + 77) & 511] * 0.999 + 1e-9;
      __syncthreads();
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) t[0] = t1 - t0;
}

int main() {
  double* d;
  long long* t;
  hipMalloc(&d, 4096 * 8);
  hipMalloc(&t, 64);
  long long h;
  auto run = [&](const char* name, void (*k)(double*, double, long long*), int threads) {
    hipLaunchKernelGGL(k, dim3(1), dim3(threads), 0, 0, d, 1.5, t);
    hipLaunchKernelGGL(k, dim3(1), dim3(threads), 0, 0, d, 1.5, t);
    hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
    printf("%-10s %7.2f ticks/op\n", name, h / 8192.0);
  };
  run("fma64", k_fma, 64);
  {
    hipLaunchKernelGGL(k_fma32, dim3(1), dim3(64), 0, 0, (float*)d, 1.5f, t);
    hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
    printf("%-10s %7.2f ticks/op\n", "fma32", h / 8192.0);
  }
  run("rsq64+add", k_rsq, 64);
  run("readlane", k_readlane, 64);
  run("bpermute", k_bperm, 64);
  run("lds_rt", k_lds, 64);
  run("barrier512", k_barrier, 512);
  return 0;
}
