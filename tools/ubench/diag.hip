// Dev microbenchmark: the camera solve's one-wave diagonal-block factorisation
// (csrc/solve_diag.hpp) on a synthetic SPD 16x16 block, s_memtime per block,
// with parts removed to locate the round's critical path.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I../uasl_motion_estimation_amd/csrc ubench_diag.hip
#include "solve_diag.hpp"
#include <cmath>
#include <cstdio>
#include <vector>

template <int V>
__global__ void k_diag(const double* A0, double* out, long long* t, int reps, double* Lout, double* Xout) {
  __shared__ double L[16 * 16], X[256], gx[384];
  const int lane = threadIdx.x, q = lane >> 4, c = lane & 15;
  double acc = 0;
  long long tot = 0;
  for (int r = 0; r < reps; ++r) {
    double4_t A4, Y4;
    for (int i = 0; i < 4; ++i) {
      A4[i] = A0[(q + 4 * i) * 16 + c] + (r + 1 < reps ? 1e-3 * r : 0.0);
      Y4[i] = (q + 4 * i == c) ? 1.0 : 0.0;
    }
    bool ok = true;
    __builtin_amdgcn_s_waitcnt(0);
    long long t0 = __builtin_amdgcn_s_memtime();
    diag_round_mfma<0>(A4, Y4, q, c, 16, ok, L, 16, X, gx);
    diag_round_mfma<1>(A4, Y4, q, c, 16, ok, L, 16, X, gx);
    diag_round_mfma<2>(A4, Y4, q, c, 16, ok, L, 16, X, gx);
    diag_round_mfma<3>(A4, Y4, q, c, 16, ok, L, 16, X, gx);
    solve_wave_sync();
    acc += L[lane] + X[lane] + (ok ? 0 : 1);
    long long t1 = __builtin_amdgcn_s_memtime();
    tot += t1 - t0;
  }
  out[lane] = acc;
  if (lane == 0) t[0] = tot;
  for (int k = lane; k < 256; k += 64) {
    Lout[k] = L[k];
    Xout[k] = X[k];
  }
}

int main() {
  std::vector<double> A(256);
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) A[i * 16 + j] = (i == j ? 20.0 : 0.0) + 1.0 / (1 + i + j);
  double *dA, *dout, *dL, *dX;
  hipMalloc(&dL, 256 * 8);
  hipMalloc(&dX, 256 * 8);
  long long* dt;
  hipMalloc(&dA, 256 * 8);
  hipMalloc(&dout, 64 * 8);
  hipMalloc(&dt, 8);
  hipMemcpy(dA, A.data(), 256 * 8, hipMemcpyHostToDevice);
  const int reps = 1000;
  for (int w = 0; w < 2; ++w) {
    hipLaunchKernelGGL(k_diag<0>, dim3(1), dim3(64), 0, 0, dA, dout, dt, reps, dL, dX);
    hipDeviceSynchronize();
  }
  long long t;
  hipMemcpy(&t, dt, 8, hipMemcpyDeviceToHost);
  printf("one-wave diagonal block (4 rounds, ME_DIAG_GATHER=%d): %.0f ticks per block\n", ME_DIAG_GATHER, (double)t / reps);
  // check against a host Cholesky / inverse of the same block
  std::vector<double> L(256, 0.0), Lg(256), Xg(256), Xh(256, 0.0);
  hipMemcpy(Lg.data(), dL, 256 * 8, hipMemcpyDeviceToHost);
  hipMemcpy(Xg.data(), dX, 256 * 8, hipMemcpyDeviceToHost);
  for (int j = 0; j < 16; ++j) {
    double d = A[j * 16 + j];
    for (int k = 0; k < j; ++k) d -= L[j * 16 + k] * L[j * 16 + k];
    L[j * 16 + j] = sqrt(d);
    for (int i = j + 1; i < 16; ++i) {
      double x = A[i * 16 + j];
      for (int k = 0; k < j; ++k) x -= L[i * 16 + k] * L[j * 16 + k];
      L[i * 16 + j] = x / L[j * 16 + j];
    }
  }
  for (int c = 0; c < 16; ++c)
    for (int i = 0; i < 16; ++i) {
      double x = i == c ? 1.0 : 0.0;
      for (int k = 0; k < i; ++k) x -= L[i * 16 + k] * Xh[k * 16 + c];
      Xh[i * 16 + c] = x / L[i * 16 + i];
    }
  double eL = 0, eX = 0;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j <= i; ++j) eL = fmax(eL, fabs(Lg[i * 16 + j] - L[i * 16 + j]));
  for (int k = 0; k < 256; ++k) eX = fmax(eX, fabs(Xg[k] - Xh[k]));
  printf("max |L - L_host| %.3g  max |X - X_host| %.3g\n", eL, eX);
  return 0;
}
