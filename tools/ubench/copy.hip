// Copy-bandwidth variants for the measured HBM denominator (me_hbm_copy_gbs):
// grid size, loads in flight per lane, nontemporal hints.  hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4v __attribute__((ext_vector_type(4)));
template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_k(const f4v* __restrict__ a, f4v* __restrict__ b, size_t n) {
  const size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    f4v v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(&a[i + u * stride]) : a[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT)
        __builtin_nontemporal_store(v[u], &b[i + u * stride]);
      else
        b[i + u * stride] = v[u];
    }
  }
  for (; i < n; i += stride) b[i] = a[i];
}

// contiguous chunk per workgroup
template <int U>
__global__ __launch_bounds__(256) void copy_chunk(const float4* __restrict__ a, float4* __restrict__ b, size_t n,
                                                  size_t per) {
  const size_t beg = (size_t)blockIdx.x * per, end = beg + per < n ? beg + per : n;
  for (size_t i = beg + threadIdx.x; i < end; i += 256 * U) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = i + 256 * u < end ? a[i + 256 * u] : float4{};
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + 256 * u < end) b[i + 256 * u] = v[u];
  }
}

int main() {
  const size_t bytes = 1ull << 30, n = bytes / 16;
  float4 *a, *b;
  hipMalloc(&a, bytes);
  hipMalloc(&b, bytes);
  hipMemset(a, 1, bytes);
  hipMemset(b, 0, bytes);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto time = [&](const char* name, auto launch) {
    launch();
    hipEventRecord(e0);
    for (int r = 0; r < 20; ++r) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-28s %8.1f GB/s\n", name, 2.0 * bytes * 20 / (ms * 1e-3) / 1e9);
  };
  for (int g : {256, 512, 768, 1024, 1280, 1536}) {
    char nm[64];
    snprintf(nm, sizeof nm, "stride U1 g%d", g);
    time(nm, [&] { copy_k<1, false><<<g, 256>>>((const f4v*)a, (f4v*)b, n); });
    snprintf(nm, sizeof nm, "stride U1 NT g%d", g);
    time(nm, [&] { copy_k<1, true><<<g, 256>>>((const f4v*)a, (f4v*)b, n); });
    snprintf(nm, sizeof nm, "stride U2 g%d", g);
    time(nm, [&] { copy_k<2, false><<<g, 256>>>((const f4v*)a, (f4v*)b, n); });
    snprintf(nm, sizeof nm, "stride U2 NT g%d", g);
    time(nm, [&] { copy_k<2, true><<<g, 256>>>((const f4v*)a, (f4v*)b, n); });
  }
  for (int rep = 0; rep < 2; ++rep)
    time("stride U1 g1024 again", [&] { copy_k<1, false><<<1024, 256>>>((const f4v*)a, (f4v*)b, n); });
  time("hipMemcpyDtoD", [&] { hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0); });
  return 0;
}
