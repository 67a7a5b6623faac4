// ba.hip — windowed stereo bundle adjustment on MI355X.
// Kernel map in ba_kernels.hpp.  Host side: problem upload + CSR build, the
// per-iteration launch sequence (LM control lives on the device: every kernel
// reads the State flags, so a whole solve can be enqueued — or captured in a
// hipGraph — without host round trips), and the landmark-sharded variant with
// a caller-provided all-reduce.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <numeric>
#include <vector>
#include <hip/hip_ext.h>
#include "me_internal.hpp"
#include "ba_kernels.hpp"
#include "roster.hpp"
#include "solve_diag.hpp"
#include "me_device.hpp"

using me_dev::wave_sync;

using namespace ba;

namespace {

constexpr double kDblMin = 2.2250738585072014e-308;
constexpr double kDblEps = 2.220446049250313e-16;

// ---------------------------------------------------------------- helpers
template <int Ctrl>
__device__ __forceinline__ double dpp_f64(double x);
__device__ __forceinline__ double wave_total(double x);
template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double* out, double* lds /* nw*NV */, int nw_active = 0) {
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = wave_total(v[i]);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < NV; ++i) lds[wave * NV + i] = v[i];
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = nw_active ? nw_active : (blockDim.x + 63) >> 6;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      double s = 0;
      for (int w = 0; w < nw; ++w) s += lds[w * NV + i];
      out[i] = s;
    }
  }
  __syncthreads();
}

// Reductions over aligned groups of W lanes, every lane ending with the same
// bits: each level combines a lane's value with one from the sibling block
// (the blocks are uniform after the previous level, and a + b == b + a
// exactly).  Within a 16-lane row the partners come from DPP (quad permutes,
// row half-mirror, row mirror: a VALU move each); only the 16- and 32-lane
// levels go through the LDS crossbar (ds_bpermute).  (Round 3 used an xor
// butterfly of lane shuffles for every level.)
#ifndef ME_GROUP_DPP
#define ME_GROUP_DPP 1
#endif
template <int Ctrl>
__device__ __forceinline__ int dpp_i32(int x) {
  return __builtin_amdgcn_mov_dpp(x, Ctrl, 0xf, 0xf, false);
}
template <int Ctrl>
__device__ __forceinline__ double dpp_f64(double x) {
  return __hiloint2double(dpp_i32<Ctrl>(__double2hiint(x)), dpp_i32<Ctrl>(__double2loint(x)));
}
constexpr int kDppQuadSwap1 = 0xB1, kDppQuadSwap2 = 0x4E, kDppRowHalfMirror = 0x141, kDppRowMirror = 0x140;
template <int W>
__device__ __forceinline__ double group_sum(double x) {
  if (!ME_GROUP_DPP) {
#pragma unroll
    for (int off = W / 2; off > 0; off >>= 1) x += __shfl_xor(x, off, W);
    return x;
  }
  if (W >= 2) x += dpp_f64<kDppQuadSwap1>(x);
  if (W >= 4) x += dpp_f64<kDppQuadSwap2>(x);
  if (W >= 8) x += dpp_f64<kDppRowHalfMirror>(x);
  if (W >= 16) x += dpp_f64<kDppRowMirror>(x);
  if (W >= 32) x += __shfl_xor(x, 16, W);
  if (W >= 64) x += __shfl_xor(x, 32, W);
  return x;
}

// The wave's sum in every lane, VALU only: the 16-lane row sums by DPP
// (quad swaps, half mirror, mirror), then the four row sums by readlane,
// added in row order (round 6: six dependent ds_bpermute rounds per value
// before -- 3.2k of the step finalize's 7.8k ticks, ME_STEP_TS).
__device__ __forceinline__ double wave_total(double x) {
  x += dpp_f64<kDppQuadSwap1>(x);
  x += dpp_f64<kDppQuadSwap2>(x);
  x += dpp_f64<kDppRowHalfMirror>(x);
  x += dpp_f64<kDppRowMirror>(x);
  auto row = [&](int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), l),
                            __builtin_amdgcn_readlane(__double2loint(x), l));
  };
  return ((row(0) + row(16)) + row(32)) + row(48);
}

__device__ __forceinline__ double block_max(double v, double* lds) {
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_down(v, off, 64));
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) lds[wave] = v;
  __syncthreads();
  double r = 0;
  if (threadIdx.x == 0) {
    const int nw = (blockDim.x + 63) >> 6;
    r = lds[0];
    for (int w = 1; w < nw; ++w) r = fmax(r, lds[w]);
  }
  __syncthreads();
  return r;
}

// p = R(aa) X + t with dp/daa and dp/dX (ceres::AngleAxisRotatePoint values;
// derivative: Gallego & Yezzi, d(Ru)/dw = -R[u]x (w w^T + (R^T - I)[w]x)/theta^2)
__device__ __forceinline__ void rotate(const double* aa, const double* X, double* P, double* dPdw, double* dPdX) {
  const double t2 = aa[0] * aa[0] + aa[1] * aa[1] + aa[2] * aa[2];
  if (t2 > kDblEps) {
    const double th = sqrt(t2), c = cos(th), s = sin(th), ti = 1.0 / th;
    const double w0 = aa[0] * ti, w1 = aa[1] * ti, w2 = aa[2] * ti;
    const double wx0 = w1 * X[2] - w2 * X[1], wx1 = w2 * X[0] - w0 * X[2], wx2 = w0 * X[1] - w1 * X[0];
    const double tmp = (w0 * X[0] + w1 * X[1] + w2 * X[2]) * (1.0 - c);
    P[0] = X[0] * c + wx0 * s + w0 * tmp;
    P[1] = X[1] * c + wx1 * s + w1 * tmp;
    P[2] = X[2] * c + wx2 * s + w2 * tmp;
    if (dPdX) {
      const double oc = 1.0 - c;
      double R[9] = {c + oc * w0 * w0,      oc * w0 * w1 - s * w2, oc * w0 * w2 + s * w1,
                     oc * w1 * w0 + s * w2, c + oc * w1 * w1,      oc * w1 * w2 - s * w0,
                     oc * w2 * w0 - s * w1, oc * w2 * w1 + s * w0, c + oc * w2 * w2};
      for (int i = 0; i < 9; ++i) dPdX[i] = R[i];
      // M = (w w^T + (R^T - I)[w]x) / theta^2 with w = aa (unnormalised)
      const double a0 = aa[0], a1 = aa[1], a2 = aa[2];
      double Wx[9] = {0, -a2, a1, a2, 0, -a0, -a1, a0, 0};
      double M[9];
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
          double acc = aa[i] * aa[j];
          for (int k = 0; k < 3; ++k) acc += (R[k * 3 + i] - (i == k ? 1.0 : 0.0)) * Wx[k * 3 + j];
          M[i * 3 + j] = acc / t2;
        }
      // -R [X]x M
      double Xx[9] = {0, -X[2], X[1], X[2], 0, -X[0], -X[1], X[0], 0};
      double RX[9];
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) RX[i * 3 + j] = R[i * 3 + 0] * Xx[0 * 3 + j] + R[i * 3 + 1] * Xx[1 * 3 + j] + R[i * 3 + 2] * Xx[2 * 3 + j];
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
          dPdw[i * 3 + j] = -(RX[i * 3 + 0] * M[0 * 3 + j] + RX[i * 3 + 1] * M[1 * 3 + j] + RX[i * 3 + 2] * M[2 * 3 + j]);
    }
  } else {
    const double wx0 = aa[1] * X[2] - aa[2] * X[1], wx1 = aa[2] * X[0] - aa[0] * X[2], wx2 = aa[0] * X[1] - aa[1] * X[0];
    P[0] = X[0] + wx0;
    P[1] = X[1] + wx1;
    P[2] = X[2] + wx2;
    if (dPdX) {
      double D[9] = {1, -aa[2], aa[1], aa[2], 1, -aa[0], -aa[1], aa[0], 1};
      for (int i = 0; i < 9; ++i) dPdX[i] = D[i];
      double N[9] = {0, X[2], -X[1], -X[2], 0, X[0], X[1], -X[0], 0};  // -[X]x
      for (int i = 0; i < 9; ++i) dPdw[i] = N[i];
    }
  }
}

// StereoReprojectionError (BundleAdjuster.h:153-171): residual, optional J
__device__ __forceinline__ void stereo_residual(const Geo& g, const double* cam, const double* X, const double* f,
                                                double* r, double* Jc, double* Jp) {
  double P[3], dPdw[9], dPdX[9];
  rotate(cam + 3, X, P, Jc ? dPdw : nullptr, Jc ? dPdX : nullptr);
  P[0] = P[0] + cam[0];
  P[1] = P[1] + cam[1];
  P[2] = P[2] + cam[2];
  const double x1 = g.K0[0] * (P[0] / P[2]) + g.K0[2];
  const double x2 = g.K1[0] * ((P[0] - g.baseline) / P[2]) + g.K1[2];
  const double y = g.K0[4] * (P[1] / P[2]) + g.K0[5];
  r[0] = g.sinv * (x1 - f[0]);
  r[1] = g.sinv * (y - f[1]);
  r[2] = g.sinv * (x2 - f[2]);
  r[3] = g.sinv * (y - f[3]);
  if (!Jc) return;
  const double iz = 1.0 / P[2], iz2 = iz * iz;
  double dr[4][3] = {{g.sinv * g.K0[0] * iz, 0.0, -g.sinv * g.K0[0] * P[0] * iz2},
                     {0.0, g.sinv * g.K0[4] * iz, -g.sinv * g.K0[4] * P[1] * iz2},
                     {g.sinv * g.K1[0] * iz, 0.0, -g.sinv * g.K1[0] * (P[0] - g.baseline) * iz2},
                     {0.0, g.sinv * g.K0[4] * iz, -g.sinv * g.K0[4] * P[1] * iz2}};
  for (int k = 0; k < 4; ++k) {
    for (int j = 0; j < 3; ++j) Jc[k * 6 + j] = dr[k][j];
    for (int j = 0; j < 3; ++j) {
      Jc[k * 6 + 3 + j] = dr[k][0] * dPdw[0 * 3 + j] + dr[k][1] * dPdw[1 * 3 + j] + dr[k][2] * dPdw[2 * 3 + j];
      Jp[k * 3 + j] = dr[k][0] * dPdX[0 * 3 + j] + dr[k][1] * dPdX[1 * 3 + j] + dr[k][2] * dPdX[2 * 3 + j];
    }
  }
}

// BundleAdjuster<2> residuals: StandardReprojectionError (BundleAdjuster.h:71-103)
// for camID 0, StereoRightError (:106-139, p.x += cam[0] - baseline) otherwise;
// both project with K[0].  Rows 2, 3 are zero so the 4-row pipeline is shared
// (zero rows add nothing to J^T J, J^T r or the Huber argument).
__device__ __forceinline__ void mono_residual(const Geo& g, const double* cam, const double* X, const double* f,
                                              bool right, double* r, double* Jc, double* Jp) {
  double P[3], dPdw[9], dPdX[9];
  rotate(cam + 3, X, P, Jc ? dPdw : nullptr, Jc ? dPdX : nullptr);
  P[0] = P[0] + (right ? cam[0] - g.baseline : cam[0]);
  P[1] = P[1] + cam[1];
  P[2] = P[2] + cam[2];
  const double x = g.K0[0] * (P[0] / P[2]) + g.K0[2];
  const double y = g.K0[4] * (P[1] / P[2]) + g.K0[5];
  r[0] = g.sinv * (x - f[0]);
  r[1] = g.sinv * (y - f[1]);
  r[2] = 0.0;
  r[3] = 0.0;
  if (!Jc) return;
  const double iz = 1.0 / P[2], iz2 = iz * iz;
  double dr[2][3] = {{g.sinv * g.K0[0] * iz, 0.0, -g.sinv * g.K0[0] * P[0] * iz2},
                     {0.0, g.sinv * g.K0[4] * iz, -g.sinv * g.K0[4] * P[1] * iz2}};
  for (int k = 0; k < 2; ++k) {
    for (int j = 0; j < 3; ++j) Jc[k * 6 + j] = dr[k][j];
    for (int j = 0; j < 3; ++j) {
      Jc[k * 6 + 3 + j] = dr[k][0] * dPdw[0 * 3 + j] + dr[k][1] * dPdw[1 * 3 + j] + dr[k][2] * dPdw[2 * 3 + j];
      Jp[k * 3 + j] = dr[k][0] * dPdX[0 * 3 + j] + dr[k][1] * dPdX[1 * 3 + j] + dr[k][2] * dPdX[2 * 3 + j];
    }
  }
  for (int k = 12; k < 24; ++k) Jc[k] = 0.0;
  for (int k = 6; k < 12; ++k) Jp[k] = 0.0;
}

// residual (+ optional Jacobian) of observation o; OD = rows of the model
// (a template parameter: one branch-free kernel instance per model)
template <int OD>
__device__ __forceinline__ void obs_residual(const Geo& g, const Bufs& b, long o, const double* cam, const double* X,
                                             double* r, double* Jc, double* Jp) {
  if (OD == 4)
    stereo_residual(g, cam, X, b.obs + 4 * o, r, Jc, Jp);
  else
    mono_residual(g, cam, X, b.obs + 2 * o, b.cam_id[o] != 0, r, Jc, Jp);
}

// ceres::HuberLoss(1.0): rho0 and sqrt(rho1) (Corrector with rho'' <= 0)
__device__ __forceinline__ void huber(double s, double* rho0, double* sqrt_rho1) {
  if (s > 1.0) {
    const double rr = sqrt(s);
    *rho0 = 2.0 * rr - 1.0;
    *sqrt_rho1 = sqrt(fmax(kDblMin, 1.0 / rr));
  } else {
    *rho0 = s;
    *sqrt_rho1 = 1.0;
  }
}

// Written-through hand-off helpers (see "Hand-off form" at the camera solve).
template <bool SC1>
__device__ __forceinline__ double a_ld(const double* p) {
  if (!SC1) return *p;
  return __builtin_bit_cast(double, __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), ME_HO_LD,
                                                      __HIP_MEMORY_SCOPE_AGENT));
}
template <bool SC1>
__device__ __forceinline__ void a_st(double* p, double v) {
  if (!SC1) {
    *p = v;
    return;
  }
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), __builtin_bit_cast(unsigned long long, v),
                     ME_HO_ST, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain_and_barrier() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave, before the barrier
  __syncthreads();
}


// ---------------------------------------------------------------- kernels
constexpr int kPtBlock = 64;   // per-point kernels: spread ~N/64 workgroups over the CUs

// Per observation: corrected residual / Jacobian, cost, and the unscaled
// per-observation normal-equation pieces W_o = Jc^T Jp (6x3), V_o = Jp^T Jp
// (6 unique), g_o = Jp^T r, so the per-point stage only sums.
// Workgroup size by window: one-wave workgroups spread a small window's
// observations over every CU (config 3: 22k observations = 344 workgroups,
// 13.6 -> 11.0 us), 256 threads for large ones (config 4: 100k observations,
// 34.4 us vs 38.6 with one-wave workgroups)
#ifndef ME_LIN_SMALL
#define ME_LIN_SMALL 64  // linearize workgroup for small windows (A/B builds)
#endif
constexpr int kLinSmall = ME_LIN_SMALL, kLinSmallMaxObs = 64 * 512;
__host__ __device__ inline int lin_block(int no) { return no <= kLinSmallMaxObs ? kLinSmall : kBlock; }
template <int OD, int BLK>
__global__ __launch_bounds__(BLK) void linearize_kernel(Geo g, Bufs b) {
  __shared__ double lds[BLK / 64];
  const State* st = b.st;
  if (st->done || !st->need_lin) return;
  const int o = blockIdx.x * BLK + threadIdx.x;
  double cost = 0;
  if (o < g.no) {
    const int cur = st->cur;
    const int ci = b.cam_idx[o], pi = b.pt_idx[o];
    double r[4], Jc[24], Jp[12];
    obs_residual<OD>(g, b, o, b.cams[cur] + 6 * ci, b.pts[cur] + 3 * pi, r, Jc, Jp);
    const double s = r[0] * r[0] + r[1] * r[1] + r[2] * r[2] + r[3] * r[3];
    double rho0, sc;
    huber(s, &rho0, &sc);
    cost = 0.5 * rho0;
    for (int k = 0; k < 4; ++k) r[k] *= sc;
    for (int k = 0; k < 24; ++k) Jc[k] *= sc;
    for (int k = 0; k < 12; ++k) Jp[k] *= sc;
    const long slot = b.pos[o];  // CSR-by-point slot: per-point stages read contiguously
    double* X = b.obsx + slot * kObsxStride;
    X[0] = Jp[0] * Jp[0] + Jp[3] * Jp[3] + Jp[6] * Jp[6] + Jp[9] * Jp[9];
    X[1] = Jp[0] * Jp[1] + Jp[3] * Jp[4] + Jp[6] * Jp[7] + Jp[9] * Jp[10];
    X[2] = Jp[0] * Jp[2] + Jp[3] * Jp[5] + Jp[6] * Jp[8] + Jp[9] * Jp[11];
    X[3] = Jp[1] * Jp[1] + Jp[4] * Jp[4] + Jp[7] * Jp[7] + Jp[10] * Jp[10];
    X[4] = Jp[1] * Jp[2] + Jp[4] * Jp[5] + Jp[7] * Jp[8] + Jp[10] * Jp[11];
    X[5] = Jp[2] * Jp[2] + Jp[5] * Jp[5] + Jp[8] * Jp[8] + Jp[11] * Jp[11];
    for (int a = 0; a < 3; ++a) X[6 + a] = Jp[a] * r[0] + Jp[3 + a] * r[1] + Jp[6 + a] * r[2] + Jp[9 + a] * r[3];
    // (the camera normal-equation pieces are formed by cam_assemble from the
    // same residual and Jacobian: no 216 B per observation through HBM)
    if (ci - g.nf >= 0) {
      double* W = b.Wo + 18 * slot;
      for (int a = 0; a < 6; ++a)
        for (int c = 0; c < 3; ++c)
          W[a * 3 + c] = Jc[a] * Jp[c] + Jc[6 + a] * Jp[3 + c] + Jc[12 + a] * Jp[6 + c] + Jc[18 + a] * Jp[9 + c];
    }
  }
  double v[1] = {cost};
  double out[1];
  block_sum<1>(v, out, lds);
  if (threadIdx.x == 0) b.part[R_COST * g.pstride + blockIdx.x] = out[0];
}

// Unscaled U = Jc^T Jc (21 unique) and g = Jc^T r per variable camera, in
// two deterministic stages (cam_assemble_body): workgroup (c, k) sums chunks
// k, k + ck, ... of 256 slots of camera c into a partial; cam_reduce adds
// the ck partials in order.
// The last workgroup to arrive on a counter, with a written-through hand-off
// (the form of the camera solve's workers): thread 0 stored the workgroup's
// partials with sc1 stores, drains them before a relaxed arrival, and the last
// reads them with sc1 loads -- no L2 write-back (release) per arrival and no
// invalidate (acquire).  The last one re-arms the counter for the next launch.
__device__ __forceinline__ bool last_arrival_wt(unsigned* cnt, unsigned expected) {
  __shared__ int slast;
  __syncthreads();
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned k = __hip_atomic_fetch_add(cnt, 1u, ME_HO_RMW, __HIP_MEMORY_SCOPE_AGENT);
    slast = k == expected - 1;
    if (slast) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return slast != 0;
}

// Camera ci: lane u < 27 sums component u of the ck partials (fixed order)
// -> raw U, column norms, raw gradient; unless sharded, the Jacobi scaling
// (iteration 0) and the scaled blocks.  Called by every thread of a block.
__device__ void cam_reduce_body(const Geo& g, const Bufs& b, int sharded, const double* cpart, double* colnorm,
                                double* gc_raw, double* Uraw, int ci) {
  __shared__ double tot[27];
  __shared__ double csl[6];
  const State* st = b.st;
  const int u = threadIdx.x;
  if (u < 27) {
    double sum = 0.0;
    for (int k = 0; k < g.ck; ++k) sum += a_ld<true>(&cpart[27 * ((long)ci * g.ck + k) + u]);  // (written through)
    tot[u] = sum;
    if (u < 21) Uraw[21 * (long)ci + u] = sum;
    else gc_raw[6 * ci + u - 21] = sum;
  }
  __syncthreads();
  if (u < 6) {
    const int d = u * 6 - u * (u - 1) / 2;  // index of (u, u) in the packed upper triangle
    colnorm[6 * ci + u] = tot[d];
    if (!sharded) {
      double* cs = b.csc + 6 * ci;
      if (!st->scaled) cs[u] = g.jacobi ? 1.0 / (1.0 + sqrt(tot[d])) : 1.0;
      csl[u] = cs[u];
    }
  }
  if (sharded) return;
  __syncthreads();
  if (u < 21) {
    int a = 0, r = u;
    while (r >= 6 - a) {
      r -= 6 - a;
      ++a;
    }
    const int c = a + r;
    const double x = tot[u] * csl[a] * csl[c];
    double* U = b.U + 36 * (long)ci;
    U[a * 6 + c] = x;
    U[c * 6 + a] = x;
  } else if (u < 27) {
    b.gcs[6 * ci + u - 21] = tot[u] * csl[u - 21];
  }
}

// Unscaled U = Jc^T Jc (21 unique) and g = Jc^T r per variable camera, in
// two deterministic stages over the camera's observations in c_obs slot
// order (each piece formed here from the observation's residual and
// Jacobian): workgroup (c, k) sums chunks k, k + ck, ... of 256 slots of
// camera c into a partial; the last of the ck
// workgroups of camera c to finish adds the ck partials in order.
// Threads 0 .. kBlock-1 of the block take part (in a wider block the other
// waves have exited: barriers count only live waves).
#ifdef ME_CAM_TS  // timing experiment only: phase split of camera (0, 0)'s assembly workgroup, s_memtime ticks
__device__ unsigned long long g_cam_ts[8];
#define CAM_T(i)                                                                           \
  do {                                                                                     \
    if (ci == 0 && k == 0 && threadIdx.x == 0) {                                           \
      const long long t_ = (long long)__builtin_amdgcn_s_memtime();                        \
      if ((i) > 0) atomicAdd(&g_cam_ts[(i)], (unsigned long long)(t_ - cam_prev_));        \
      else atomicAdd(&g_cam_ts[0], 1ull);                                                  \
      cam_prev_ = t_;                                                                      \
    }                                                                                      \
  } while (0)
#else
#define CAM_T(i) \
  do {           \
  } while (0)
#endif
template <int OD>
__device__ __forceinline__ void cam_assemble_body(const Geo& g, const Bufs& b, double* cpart, int sharded,
                                                  double* colnorm, double* gc_raw, double* Uraw, int ci, int k) {
  __shared__ double rows[kBlock / 16 * 27];
  const State* st = b.st;
  if (st->done || !st->need_lin) return;
#ifdef ME_CAM_TS
  long long cam_prev_ = 0;
#endif
  CAM_T(0);
  const int beg = b.c_off[ci], end = b.c_off[ci + 1];
  double v[27];
  for (int i = 0; i < 27; ++i) v[i] = 0;
  const int cur = st->cur;
  for (int q = beg + k * kBlock + threadIdx.x; q < end; q += g.ck * kBlock) {
    // the observation's residual and Jacobian at the linearisation point, as
    // linearize_kernel forms them (same function, same Huber scaling: the same
    // pieces bit for bit), then Jc^T Jc (21) and Jc^T r (6)
    const int o = b.c_obs[q];
    const int cam = b.cam_idx[o], pi = b.pt_idx[o];
    double r[4], Jc[24], Jp[12];
    obs_residual<OD>(g, b, o, b.cams[cur] + 6 * cam, b.pts[cur] + 3 * pi, r, Jc, Jp);
    const double s2 = r[0] * r[0] + r[1] * r[1] + r[2] * r[2] + r[3] * r[3];
    double rho0, sc;
    huber(s2, &rho0, &sc);
    for (int kk = 0; kk < 4; ++kk) r[kk] *= sc;
    for (int kk = 0; kk < 24; ++kk) Jc[kk] *= sc;
    int u = 0;
    for (int a = 0; a < 6; ++a)
      for (int c = a; c < 6; ++c, ++u)
        v[u] += Jc[a] * Jc[c] + Jc[6 + a] * Jc[6 + c] + Jc[12 + a] * Jc[12 + c] + Jc[18 + a] * Jc[18 + c];
    for (int a = 0; a < 6; ++a) v[21 + a] += Jc[a] * r[0] + Jc[6 + a] * r[1] + Jc[12 + a] * r[2] + Jc[18 + a] * r[3];
  }
  CAM_T(1);
  // the 27 sums: 16-lane row sums by DPP (VALU only), the 16 row sums of the
  // block through LDS, thread u < 27 adds component u's in row order (round 6:
  // 4.2 -> see DESIGN §5.4 us; six dependent lane-shuffle rounds per value before)
#pragma unroll
  for (int u = 0; u < 27; ++u) {
    double x = v[u];
    x += dpp_f64<kDppQuadSwap1>(x);
    x += dpp_f64<kDppQuadSwap2>(x);
    x += dpp_f64<kDppRowHalfMirror>(x);
    x += dpp_f64<kDppRowMirror>(x);
    v[u] = x;
  }
  if ((threadIdx.x & 15) == 0)
#pragma unroll
    for (int u = 0; u < 27; ++u) rows[(threadIdx.x >> 4) * 27 + u] = v[u];
  __syncthreads();
  CAM_T(2);
  if (threadIdx.x < 27) {  // written through for the last of the camera's workgroups (no release per arrival)
    double sum = 0.0;
#pragma unroll
    for (int r = 0; r < kBlock / 16; ++r) sum += rows[r * 27 + threadIdx.x];
    a_st<true>(&cpart[27 * ((long)ci * g.ck + k) + threadIdx.x], sum);  // (lanes of wave 0: its vmcnt drain covers them)
  }
  const bool last = last_arrival_wt(b.cnt + ci, g.ck);
  CAM_T(3);
  if (!last) return;
  cam_reduce_body(g, b, sharded, cpart, colnorm, gc_raw, Uraw, ci);
  CAM_T(4);
#ifdef ME_CAM_TS
  if (ci == 0 && k == 0 && threadIdx.x == 0) atomicAdd(&g_cam_ts[5], 1ull);
#endif
}

__global__ __launch_bounds__(kBlock) void cam_assemble_kernel(Geo g, Bufs b, double* cpart, int sharded,
                                                              double* colnorm, double* gc_raw, double* Uraw) {
  // (one instance per model: the mono model's row selection would otherwise
  // keep the stereo path's Jacobian arrays out of registers)
  if (g.od == 4)
    cam_assemble_body<4>(g, b, cpart, sharded, colnorm, gc_raw, Uraw, blockIdx.x, blockIdx.y);
  else
    cam_assemble_body<2>(g, b, cpart, sharded, colnorm, gc_raw, Uraw, blockIdx.x, blockIdx.y);
}

// Camera assembly riding in the Schur launch (iterations after the first,
// when the Jacobi scaling is fixed and the two passes are independent).
struct CamArgs {
  double *cpart, *colnorm, *gc_raw, *Uraw;
  int on;
  int ncam;  // leading workgroups of the launch that assemble cameras (m ck, padded to whole rounds of 8 XCDs)
};

// Sharded mode, first linearisation: the rank's input flags (bad index,
// infeasible start) ride behind the column norms in the first exchange, so
// every rank ends the solve alike (each rank only checks its own landmarks).
__global__ void xch_flags_kernel(Geo g, Bufs b, double* colnorm) {
  colnorm[g.n6] = b.st->bad_input ? 1.0 : 0.0;
  colnorm[g.n6 + 1] = b.st->infeasible ? 1.0 : 0.0;
}

// Sharded mode: scaling from the all-reduced column norms, then scale the
// (local) U / g blocks.
__global__ void cam_finish_kernel(Geo g, Bufs b, const double* colnorm, const double* gc_raw, const double* Uraw,
                                  int first) {
  State* st = b.st;
  if (first) {  // (colnorm[n6 ..] = the all-reduced input flags; read before any thread returns)
    const bool bad = colnorm[g.n6] != 0.0, infeasible = colnorm[g.n6 + 1] != 0.0;
    __syncthreads();
    if (bad || infeasible) {
      if (blockIdx.x == 0 && threadIdx.x == 0) {
        st->bad_input = bad;
        st->infeasible = infeasible;
        st->done = 1;
        st->termination = 2;
      }
      return;
    }
  }
  if (st->done || !st->need_lin) return;
  const int ci = blockIdx.x * blockDim.x + threadIdx.x;
  if (ci >= g.m) return;
  double* cs = b.csc + 6 * ci;
  if (!st->scaled)
    for (int a = 0; a < 6; ++a) cs[a] = g.jacobi ? 1.0 / (1.0 + sqrt(colnorm[6 * ci + a])) : 1.0;
  const double* Ur = Uraw + 21 * (long)ci;
  double* U = b.U + 36 * (long)ci;
  int u = 0;
  for (int a = 0; a < 6; ++a)
    for (int c = a; c < 6; ++c, ++u) {
      const double x = Ur[u] * cs[a] * cs[c];
      U[a * 6 + c] = x;
      U[c * 6 + a] = x;
    }
  for (int a = 0; a < 6; ++a) b.gcs[6 * ci + a] = gc_raw[6 * ci + a] * cs[a];
}

__device__ __forceinline__ bool chol3(const double* A, double* L) {
  double d0 = A[0];
  if (!(d0 > 0)) return false;
  d0 = sqrt(d0);
  const double l10 = A[3] / d0, l20 = A[6] / d0;
  double d1 = A[4] - l10 * l10;
  if (!(d1 > 0)) return false;
  d1 = sqrt(d1);
  const double l21 = (A[7] - l20 * l10) / d1;
  double d2 = A[8] - l20 * l20 - l21 * l21;
  if (!(d2 > 0)) return false;
  d2 = sqrt(d2);
  L[0] = d0; L[1] = 0; L[2] = 0;
  L[3] = l10; L[4] = d1; L[5] = 0;
  L[6] = l20; L[7] = l21; L[8] = d2;
  return true;
}
__device__ __forceinline__ void fwd3(const double* L, const double* b, double* y) {
  y[0] = b[0] / L[0];
  y[1] = (b[1] - L[3] * y[0]) / L[4];
  y[2] = (b[2] - L[6] * y[0] - L[7] * y[1]) / L[8];
}
__device__ __forceinline__ void bwd3(const double* L, const double* y, double* x) {
  x[2] = y[2] / L[8];
  x[1] = (y[1] - L[7] * x[2]) / L[4];
  x[0] = (y[0] - L[3] * x[1] - L[6] * x[2]) / L[0];
}

// Point blocks and Schur complement in one pass over the landmarks.  A
// workgroup (8 waves) takes sub-chunks of P landmarks; per sub-chunk:
//  (A) a group of 32 lanes per landmark, one CSR slot per lane, every load
//      issued in one round: V = sum V_o, g = sum g_o (after a linearisation;
//      Jacobi scaling at iteration 0; projected-gradient max-norm), then
//      V + D/radius -> Cholesky L_p, z_p = L_p^-1 g_p on every lane of the
//      group (butterfly sums leave the totals on all of them: no staging);
//  (B) each lane writes its slot's entries of the landmark's 3 rows of
//      Y = (Dc W Dp) L_p^-T into LDS (duplicate residual blocks of one camera
//      add in CSR order, no atomics), z_p as the extra column n6 (so Y^T Y
//      also yields Y^T z);
//  (C) S partial tiles D(16x16) += A(16x4) B(4x16) on v_mfma_f64_16x16x4f64
//      (A[i][k] = Y[k][16I+i], B[k][j] = Y[k][16J+j]), one wave per tile,
//      accumulated over all the workgroup's sub-chunks in registers.  A K-step
//      of 4 rows is skipped for a tile when the rows' camera band (a track's
//      cameras are contiguous in CSR order) misses the tile's columns.
// Band-sorted runs (plan_order_kernel): a workgroup takes one run of rlen
// landmarks in (first tile, last tile) order -- landmarks with similar camera
// bands together -- and one group of stpw tiles of the run's tile set (the
// pairs of tiles in its band plus the z tile), so a wave holds at most 5
// accumulator tiles and a run stores only its band's tiles (config 5: ~16 MB
// of partials per iteration instead of 97, config 4: 12 instead of 33).
// Partials (run x tile) are summed in fixed run order by s_assemble through
// the per-tile slot lists: deterministic, no atomics.  Operand map of the MFMA: lane l holds
// A[l&15][l>>4] and B[l>>4][l&15]; result register i holds D[(l>>4)+4i][l&15].
// Landmarks per sub-chunk: 32 (96 rows of Y, 16 lanes per landmark) while the
// Y block fits the LDS budget, else 16 (48 rows, 32 lanes per landmark).  Each
// Schur workgroup leaves one set of partial tiles that s_assemble sums, so
// twice the landmarks per workgroup halve that traffic.
constexpr int kSchurPts = 16, kSchurPtsWide = 32, kSchurPtsSmall = 8;
#ifndef ME_SCHUR_NT
#define ME_SCHUR_NT 5
#endif
constexpr int kSchurNtMax = ME_SCHUR_NT;  // accumulator tiles per wave (3..5)
constexpr size_t kSchurLdsCap = 150 * 1024;
__host__ __device__ inline size_t schur_lds_bytes(int P, int Rz) { return 8 * (size_t)3 * P * Rz + 4 * 3 * (size_t)P; }

template <int W>
__device__ __forceinline__ int group_min(int x) {
  if (W >= 2) x = min(x, dpp_i32<kDppQuadSwap1>(x));
  if (W >= 4) x = min(x, dpp_i32<kDppQuadSwap2>(x));
  if (W >= 8) x = min(x, dpp_i32<kDppRowHalfMirror>(x));
  if (W >= 16) x = min(x, dpp_i32<kDppRowMirror>(x));
  if (W >= 32) x = min(x, __shfl_xor(x, 16, W));
  if (W >= 64) x = min(x, __shfl_xor(x, 32, W));
  return x;
}
template <int W>
__device__ __forceinline__ int group_max(int x) {
  if (W >= 2) x = max(x, dpp_i32<kDppQuadSwap1>(x));
  if (W >= 4) x = max(x, dpp_i32<kDppQuadSwap2>(x));
  if (W >= 8) x = max(x, dpp_i32<kDppRowHalfMirror>(x));
  if (W >= 16) x = max(x, dpp_i32<kDppRowMirror>(x));
  if (W >= 32) x = max(x, __shfl_xor(x, 16, W));
  if (W >= 64) x = max(x, __shfl_xor(x, 32, W));
  return x;
}

#ifdef ME_SCHUR_STAMPS  // timing experiment only (tools/drivers.py schur_stamps): workgroup 0's phase times in st->stamps[6..11]
#define SCHUR_T(i)                                                                     \
  do {                                                                                 \
    if (sblk == 0 && threadIdx.x == 0) {                                               \
      const long long tt_ = (long long)__builtin_amdgcn_s_memtime();                   \
      if ((i) > 0) st->stamps[5 + (i)] += tt_ - sch_prev_;                             \
      sch_prev_ = tt_;                                                                 \
    }                                                                                  \
  } while (0)
#else
#define SCHUR_T(i) \
  do {             \
  } while (0)
#endif
template <int NT, int BLK, int PTS>
__global__ __launch_bounds__(BLK) void pt_schur_kernel(Geo g, Bufs b, Opts o, CamArgs ca) {
  constexpr int SL = BLK / PTS, NW = BLK / 64;  // lanes per landmark, waves
  extern __shared__ double smem[];
  __shared__ double red[8];
  // camera-assembly blocks of a fused launch come first: dispatched before the
  // Schur runs, their longer chain (slot loop, 27-value reduce, camera reduce)
  // no longer trails the runs (round 6: the launch 14.8 -> see DESIGN §5.4)
  if (ca.on && (int)blockIdx.x < ca.ncam) {
    if (threadIdx.x >= kBlock) return;
    const int q = blockIdx.x;
    if (q >= g.m * g.ck) return;  // (padding to a multiple of 8)
    if (g.od == 4)
      cam_assemble_body<4>(g, b, ca.cpart, 0, ca.colnorm, ca.gc_raw, ca.Uraw, q / g.ck, q % g.ck);
    else
      cam_assemble_body<2>(g, b, ca.cpart, 0, ca.colnorm, ca.gc_raw, ca.Uraw, q / g.ck, q % g.ck);
    return;
  }
  const int sblk = (int)blockIdx.x - (ca.on ? ca.ncam : 0);  // this workgroup's index among the Schur runs
  State* st = b.st;
  if (st->done) return;
#ifdef ME_SCHUR_STAMPS
  long long sch_prev_ = 0;
  if (sblk == 0 && threadIdx.x == 0) st->stamps[12] += 1;
#endif
  SCHUR_T(0);
  const int need_lin = st->need_lin, scaled = st->scaled, cur = st->cur;
  const double* obsx = b.obsx;
  const double* Wo = b.Wo;
  const double radius = st->radius;
  // all allowed steps taken: this pass only evaluates the gradient for the
  // closing test (Ceres HandleSuccessfulStep); no Schur complement is needed
  const bool final_pass = st->iterations >= o.max_num_iterations;
  if (sblk == 0 && threadIdx.x == 0) st->final_pass = final_pass;
  const int P = g.spts, Rz = g.Rpad, rows = 3 * P, nks = rows / 4;
  // this workgroup's run and tile group; the run's tile set is [bA, bB] plus the z tile T - 1
  // Workgroups are dealt round-robin over the 8 XCDs: a run's tile groups sit
  // at blocks b, b + 8, ... so they share an XCD's L2 -- the second group's
  // reads of the run's slots (W, obsx) hit the lines the first one fetched.
  const int sup = sblk / (8 * g.sgrp), r8 = sblk - sup * 8 * g.sgrp;
  const int run = 8 * sup + (r8 & 7), tgrp = r8 >> 3;
  if (run >= g.nruns) {  // (uniform) padding of the last block of 8 runs
    if (need_lin && threadIdx.x == 0) b.part[R_GMAX_PT * g.pstride + sblk] = 0.0;
    return;
  }
  const int bA = g.sorted ? b.rband[2 * run] : 0, bB = g.sorted ? b.rband[2 * run + 1] : g.T - 1;
  const int nb = bB - bA + 1, ns = nb + (bB < g.T - 1 ? 1 : 0), ntile = ns * (ns + 1) / 2;
  if (tgrp * g.stpw >= ntile) {  // (uniform) the run's tiles are all taken by lower groups
    if (need_lin && threadIdx.x == 0) b.part[R_GMAX_PT * g.pstride + sblk] = 0.0;
    return;
  }
  const bool lead = tgrp == 0;  // the run's first group writes the per-landmark results (the others recompute them)
  double* Y = smem;
  int* band = reinterpret_cast<int*>(Y + (size_t)rows * Rz);  // per landmark: first / last camera column, live
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int gi = tid / SL, gl = tid & (SL - 1);
  // this wave's tiles (wave-uniform: scalar registers): canonical index c of
  // the run's tile set (row ka of the set's upper triangle holds ns - ka pairs)
  int tI[NT], tJ[NT];
#pragma unroll
  for (int u = 0; u < NT; ++u) {
    int p = tgrp * g.stpw + wave + NW * u, ka = 0;
    if (p >= ntile) p = -1;
    int rem = p < 0 ? 0 : p;
    while (rem >= ns - ka) {
      rem -= ns - ka;
      ++ka;
    }
    const int kb = ka + rem;
    tI[u] = p < 0 ? -1 : (ka < nb ? bA + ka : g.T - 1);
    tJ[u] = p < 0 ? -1 : (kb < nb ? bA + kb : g.T - 1);
  }
  double4_t acc[NT];
#pragma unroll
  for (int u = 0; u < NT; ++u) acc[u] = double4_t{0.0, 0.0, 0.0, 0.0};
  double gm = 0;
  for (int sc = 0; sc < g.rsub; ++sc) {
    const int pos = run * g.rlen + sc * P + gi;
    const int j = pos < g.np ? (g.sorted ? b.order[pos] : pos) : g.np;
    double* Yp = Y + (size_t)(3 * gi) * Rz;  // this landmark's 3 rows, written by its own lane group only
    for (int i = gl; i < 3 * Rz / 2; i += SL) reinterpret_cast<double2*>(Yp)[i] = double2{0.0, 0.0};
    if (j < g.np) {
      // (A) every load of the landmark and of this lane's first CSR slot in one round
      const int beg = b.p_off[j], end = b.p_off[j + 1];
      const int q0 = beg + gl;
      int ci0 = -1, cprev0 = -1, cnext0 = -2;
      double w0[18], cs0[6], X0[9];
      for (int i = 0; i < 9; ++i) X0[i] = 0.0;
      if (q0 < end) {
        ci0 = b.p_cam[q0];
        if (q0 > beg) cprev0 = b.p_cam[q0 - 1];
        if (q0 + 1 < end) cnext0 = b.p_cam[q0 + 1];  // duplicate test of phase B, requested with the rest
        if (need_lin)
          for (int i = 0; i < 9; ++i) X0[i] = obsx[(long)q0 * kObsxStride + i];
        if (ci0 >= 0) {
          for (int i = 0; i < 18; ++i) w0[i] = Wo[18 * (long)q0 + i];
          for (int a = 0; a < 6; ++a) cs0[a] = b.csc[6 * ci0 + a];
        }
      }
      double Vs[9], gs[3], pv[3], xv[3];
      if (need_lin) {
        for (int a = 0; a < 3; ++a) xv[a] = b.pts[cur][3 * (long)j + a];
        if (scaled)
          for (int a = 0; a < 3; ++a) pv[a] = b.psc[3 * (long)j + a];
        double V[9];  // V_o (6 unique) | g_o (3)
        for (int i = 0; i < 9; ++i) V[i] = X0[i];
        for (int q = q0 + SL; q < end; q += SL)
          for (int i = 0; i < 9; ++i) V[i] += obsx[(long)q * kObsxStride + i];
        SCHUR_T(1);  // loads of phase A issued and returned (first use)
      for (int i = 0; i < 9; ++i) V[i] = group_sum<SL>(V[i]);
        if (!scaled) {
          pv[0] = g.jacobi ? 1.0 / (1.0 + sqrt(V[0])) : 1.0;
          pv[1] = g.jacobi ? 1.0 / (1.0 + sqrt(V[3])) : 1.0;
          pv[2] = g.jacobi ? 1.0 / (1.0 + sqrt(V[5])) : 1.0;
        }
        const double p0 = pv[0], p1 = pv[1], p2 = pv[2];
        Vs[0] = V[0] * p0 * p0; Vs[1] = V[1] * p0 * p1; Vs[2] = V[2] * p0 * p2;
        Vs[3] = Vs[1];          Vs[4] = V[3] * p1 * p1; Vs[5] = V[4] * p1 * p2;
        Vs[6] = Vs[2];          Vs[7] = Vs[5];          Vs[8] = V[5] * p2 * p2;
        gs[0] = V[6] * p0;
        gs[1] = V[7] * p1;
        gs[2] = V[8] * p2;
        if (gl == 0 && lead) {
          if (!scaled)
            for (int a = 0; a < 3; ++a) b.psc[3 * (long)j + a] = pv[a];
          for (int i = 0; i < 9; ++i) b.V[9 * (long)j + i] = Vs[i];
          for (int a = 0; a < 3; ++a) b.gps[3 * (long)j + a] = gs[a];
          for (int a = 0; a < 3; ++a) {
            const double xp = fmin(fmax(xv[a] - V[6 + a], g.lo[a]), g.hi[a]);
            gm = fmax(gm, fabs(xv[a] - xp));
          }
        }
      } else {
        for (int i = 0; i < 9; ++i) Vs[i] = b.V[9 * (long)j + i];
        for (int a = 0; a < 3; ++a) {
          gs[a] = b.gps[3 * (long)j + a];
          pv[a] = b.psc[3 * (long)j + a];
        }
      }
      if (!final_pass) {  // (uniform)
      // point block, redundantly on every lane of the group (the sums are group-uniform)
      double A[9], L[9], z[3];
      for (int i = 0; i < 9; ++i) A[i] = Vs[i];
      for (int a = 0; a < 3; ++a) A[4 * a] += fmin(fmax(Vs[4 * a], o.min_diag), o.max_diag) / radius;
      const bool ok = chol3(A, L);
      fwd3(L, gs, z);
      const double rL0 = 1.0 / L[0], rL4 = 1.0 / L[4], rL8 = 1.0 / L[8];
      if (gl == 0) {
        if (!ok) st->fail = 1;
        if (lead) {
          for (int i = 0; i < 9; ++i) b.Lp[9 * (long)j + i] = L[i];
          for (int a = 0; a < 3; ++a) b.zp[3 * (long)j + a] = z[a];
        }
      }
      SCHUR_T(2);  // group sums, point block
      // (B) this lane's slots -> the landmark's rows of Y (first slot of each camera run only;
      // duplicate residual blocks of one camera are summed in CSR order)
      int lo = 1 << 29, hi = -1;
      for (int q = q0; q < end; q += SL) {
        int ci, cp;
        double w[18], cs[6];
        if (q == q0) {
          ci = ci0;
          cp = cprev0;
          if (ci >= 0) {
            for (int i = 0; i < 18; ++i) w[i] = w0[i];
            for (int a = 0; a < 6; ++a) cs[a] = cs0[a];
          }
        } else {
          ci = b.p_cam[q];
          cp = b.p_cam[q - 1];
          if (ci >= 0) {
            for (int i = 0; i < 18; ++i) w[i] = Wo[18 * (long)q + i];
            for (int a = 0; a < 6; ++a) cs[a] = b.csc[6 * ci + a];
          }
        }
        if (ci < 0) continue;
        lo = min(lo, 6 * ci);
        hi = max(hi, 6 * ci + 5);
        if (cp == ci) continue;  // not the first slot of its camera run
        if (q != q0 || cnext0 == ci)  // (the first slot's next camera came with phase A's loads)
          for (int r = q + 1; r < end && b.p_cam[r] == ci; ++r)
            for (int i = 0; i < 18; ++i) w[i] += Wo[18 * (long)r + i];
        for (int a = 0; a < 6; ++a) {
          const int col = 6 * ci + a;
          const double wa[3] = {w[3 * a] * cs[a] * pv[0], w[3 * a + 1] * cs[a] * pv[1], w[3 * a + 2] * cs[a] * pv[2]};
          double y[3];  // L y = wa with the diagonal reciprocals hoisted out of the slot loop
          y[0] = wa[0] * rL0;
          y[1] = (wa[1] - L[3] * y[0]) * rL4;
          y[2] = (wa[2] - L[6] * y[0] - L[7] * y[1]) * rL8;
          for (int k = 0; k < 3; ++k) Yp[(size_t)k * Rz + col] = y[k];
        }
      }
      lo = group_min<SL>(lo);
      hi = group_max<SL>(hi);
      if (gl == 0) {
        for (int k = 0; k < 3; ++k) Yp[(size_t)k * Rz + g.n6] = z[k];
        band[3 * gi] = lo;
        band[3 * gi + 1] = hi;
        band[3 * gi + 2] = 1;  // z_p (column n6, tile T-1) is live for every landmark
      }
      }  // !final_pass
    } else if (gl == 0) {
      band[3 * gi] = 1 << 29;
      band[3 * gi + 1] = -1;
      band[3 * gi + 2] = 0;
    }
    __syncthreads();
    SCHUR_T(3);  // Y rows in LDS (barrier)
    // (C) partial tiles on the matrix cores.  First the band test of every
    // K-step at once (lane ks of each wave tests step ks, one ballot per tile:
    // wave-uniform hit masks in scalar registers), then the steps run with the
    // next step's operands requested before this step's MFMAs -- no LDS round
    // trip between a step's band test and its operands.
    if (!final_pass) {
      unsigned long long hm[NT];
      {
        int lo = 1 << 29, hi = -1, live = 0;
        if (lane < nks) {
          const int pa = (4 * lane) / 3, pb = min((4 * lane + 3) / 3, P - 1);
          lo = min(band[3 * pa], band[3 * pb]);
          hi = max(band[3 * pa + 1], band[3 * pb + 1]);
          live = band[3 * pa + 2] | band[3 * pb + 2];
        }
#pragma unroll
        for (int u = 0; u < NT; ++u) {
          const int I = tI[u], J = tJ[u];
          // a tile is touched by these rows iff both its column blocks meet the camera band or the z column
          const bool hitI = (hi >= 16 * I && lo <= 16 * I + 15) || (live && I == g.T - 1);
          const bool hitJ = (hi >= 16 * J && lo <= 16 * J + 15) || (live && J == g.T - 1);
          hm[u] = __ballot(lane < nks && I >= 0 && hitI && hitJ);
        }
      }
      auto operands = [&](int ks, double* a, double* bb) {
        const double* Yr = Y + (size_t)(4 * ks + (lane >> 4)) * Rz + (lane & 15);
#pragma unroll
        for (int u = 0; u < NT; ++u) {
          const bool h = (hm[u] >> ks) & 1ull;
          a[u] = h ? Yr[16 * tI[u]] : 0.0;
          bb[u] = h ? Yr[16 * tJ[u]] : 0.0;
        }
      };
      auto contract = [&](int ks, const double* a, const double* bb) {
#pragma unroll
        for (int u = 0; u < NT; ++u)
          if ((hm[u] >> ks) & 1ull) acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u], bb[u], acc[u], 0, 0, 0);
      };
      double av[NT], bv[NT];
      if constexpr (NT <= 6) {
        // A few tiles per wave: the K-steps unrolled with ping-pong operand
        // registers, every operand read issued unconditionally (clamped tile
        // index) and only the MFMAs skipped by the band masks.  Straight-line
        // LDS reads let each MFMA wait for its own operands only (lgkmcnt(N));
        // conditional reads made the compiler wait for all of them (lgkmcnt(0)
        // before every step's first MFMA: the next step's reads were never
        // overlapped).  Scheduling barriers keep one step of reads in flight.
        constexpr int NKS = 3 * PTS / 4;
        static_assert(NKS % 2 == 0, "K-steps are taken in pairs");
        int cI[NT], cJ[NT];
#pragma unroll
        for (int u = 0; u < NT; ++u) {
          cI[u] = 16 * max(tI[u], 0);
          cJ[u] = 16 * max(tJ[u], 0);
        }
        const double* Y0 = Y + (size_t)(lane >> 4) * Rz + (lane & 15);
        const size_t kstride = 4 * (size_t)Rz;
        auto reads = [&](const double* Yr, double* a, double* bb) {
#pragma unroll
          for (int u = 0; u < NT; ++u) {
            a[u] = Yr[cI[u]];
            bb[u] = Yr[cJ[u]];
          }
        };
        double an[NT], bn[NT];
        reads(Y0, av, bv);
#pragma unroll 1
        for (int ks = 0; ks < NKS; ks += 2) {
          reads(Y0 + (ks + 1) * kstride, an, bn);
          __builtin_amdgcn_sched_barrier(0);
          contract(ks, av, bv);
          __builtin_amdgcn_sched_barrier(0);
          reads(Y0 + min(ks + 2, NKS - 1) * kstride, av, bv);  // (the last pair re-reads a valid row, unused)
          __builtin_amdgcn_sched_barrier(0);
          contract(ks + 1, an, bn);
          __builtin_amdgcn_sched_barrier(0);
        }
      } else {
        for (int ks = 0; ks < nks; ++ks) {
          operands(ks, av, bv);
          contract(ks, av, bv);
        }
      }
    }
    __syncthreads();
  }
  SCHUR_T(4);  // MFMA contraction (barrier)
  if (need_lin) {
    const double r = block_max(gm, red);
    if (tid == 0) b.part[R_GMAX_PT * g.pstride + sblk] = r;
  }
  if (final_pass) return;
#pragma unroll
  for (int u = 0; u < NT; ++u) {
    const int p = tgrp * g.stpw + wave + NW * u;
    if (p >= ntile) continue;
    double* dst = b.Spart + ((long)run * g.npairs + p) * 256;
#pragma unroll
    for (int i = 0; i < 4; ++i) dst[((lane >> 4) + 4 * i) * 16 + (lane & 15)] = acc[u][i];
  }
#ifdef ME_SCHUR_STAMPS
  __builtin_amdgcn_s_waitcnt(0);
#endif
  SCHUR_T(5);  // gradient max + partial stores
}

// Linearisation bookkeeping + iteration start: reduce the cost / gradient
// partials (fixed order), Ceres gradient-tolerance test (IterationZero /
// HandleSuccessfulStep), max-iteration and min-radius tests.
// The cost partials are summed by the first kFinBlock threads in the same
// order whatever the block size (256 in s_assemble_kernel, 512 inside the
// camera-solve launch): the same x_cost bits either way.  Sharded (b.xch):
// cost, camera gradient and the per-rank gradient max-norms come from the
// all-reduced exchange.
constexpr int kFinBlock = 256;
__device__ void lin_finalize_body(const Geo& g, const Bufs& b, const Opts& o, const double* gc_raw,
                                  double* lds /* 16 */) {
  State* st = b.st;
  if (st->done) return;
  if (st->need_lin) {
    const bool x = b.xch != nullptr;
    const int t = threadIdx.x;
    const bool in = t < kFinBlock;
    double c = 0, m = 0;
    if (!x && in) {
      for (int i = t; i < g.nblk_lin; i += kFinBlock) c += b.part[R_COST * g.pstride + i];
      for (int i = t; i < g.ksplit; i += kFinBlock) m = fmax(m, b.part[R_GMAX_PT * g.pstride + i]);
    }
    const double* gcv = x ? b.xch + xo_gc(g) : gc_raw;
    if (in)
      for (int i = t; i < g.n6; i += kFinBlock) m = fmax(m, fabs(gcv[i]));
    if (x && in)
      for (int i = t; i < g.xslots; i += kFinBlock) m = fmax(m, b.xch[xo_gmax(g) + i]);
    double v[1] = {c}, out[1];
    block_sum<1>(v, out, lds, kFinBlock / 64);
    const double mm = block_max(m, lds + 8);
    if (threadIdx.x == 0) {
      st->x_cost = x ? b.xch[xo_cost(g)] : out[0];
      const double gm = mm;
      if (!st->scaled) {
        st->initial_cost = st->x_cost;
        st->scaled = 1;
      }
      st->need_lin = 0;
      if (gm <= o.gradient_tolerance) {
        st->done = 1;
        st->termination = 0;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x != 0 || st->done) return;
  if (st->iterations >= o.max_num_iterations) {
    st->done = 1;
    st->termination = 1;
    return;
  }
  if (st->radius <= o.min_radius) {
    st->done = 1;
    st->termination = 0;
    return;
  }
  st->iterations += 1;
}

__global__ __launch_bounds__(kFinBlock) void lin_finalize_kernel(Geo g, Bufs b, Opts o, const double* gc_raw) {
  __shared__ double lds[16];
  lin_finalize_body(g, b, o, gc_raw, lds);
}

// Sharded mode: this rank's linearisation scalars into the exchange tail --
// cost (fixed-order sum of the linearize partials), failure flag, gradient
// max-norm in this rank's slot (0 in the others), raw camera gradient.
__device__ void xch_tail_body(const Geo& g, const Bufs& b, const double* gc_raw, double* lds /* 16 */) {
  const State* st = b.st;
  double c = 0, m = 0;
  if (st->need_lin) {
    for (int i = threadIdx.x; i < g.nblk_lin; i += kFinBlock) c += b.part[R_COST * g.pstride + i];
    for (int i = threadIdx.x; i < g.ksplit; i += kFinBlock) m = fmax(m, b.part[R_GMAX_PT * g.pstride + i]);
  }
  double* x = b.xch;
  for (int i = threadIdx.x; i < g.n6; i += kFinBlock) x[xo_gc(g) + i] = gc_raw[i];
  for (int i = threadIdx.x; i < g.xslots; i += kFinBlock)
    if (i != g.xrank) x[xo_gmax(g) + i] = 0.0;
  double v[1] = {c}, out[1];
  block_sum<1>(v, out, lds);
  const double mm = block_max(m, lds + 8);
  if (threadIdx.x == 0) {
    x[xo_cost(g)] = out[0];
    x[xo_fail(g)] = st->fail ? 1.0 : 0.0;
    x[xo_gmax(g) + g.xrank] = mm;
  }
}

// S = U - sum over the Schur runs' partial tiles, b = g - Y^T z, diag(U)
// (sharded mode: the local pieces, no LM diagonal).  256 threads = 32
// elements x 8 partial groups: group k sums entries k, k + 8, ... of the
// tile's slot list (the runs covering the tile, in run order), then the 8
// group sums are added in order (deterministic).  The threads walk
// the partial tiles in their own layout (the upper block triangle, tile pair
// p = (I <= J), row-major 16 x 16), so consecutive threads read consecutive
// doubles of every partial; the sums land in the lower block triangle of S
// (transposed for I < J; the diagonal tiles as they are), the column n6 of
// the tiles in b.  `full` also writes the upper block triangle (reduced-system
// / covariance read-back); the camera solve reads only the lower one.
constexpr int kSaElems = 32, kSaGroups = kBlock / kSaElems;
// The grid's last workgroup runs the linearisation bookkeeping of
// lin_finalize_kernel instead (one launch less per iteration): the assembly
// blocks do not read what it writes, and the camera solve that follows
// reads both.
// Assembly of elements blk * EL .. blk * EL + EL - 1 by NTH = 8 EL threads
// (8 partial groups of EL elements).  No early return: the fused form's
// workgroup signals after every thread's stores have drained.  SC1: stores
// written through for a consumer workgroup of the same launch.
// mode (sharded runs): SA_PACK sums this rank's partials and U
// into the exchange buffer in the tile layout (element idx of [S | b] at
// xch[idx], diag(U) in the tail) instead of S; SA_UNPACK reads the all-reduced
// exchange (no partials, no U) and stores S / b / diag(U) exactly as SA_SUM.
__host__ __device__ inline int solve_ld(int Ts) { return ((16 * Ts + 31) / 32) * 32 + 2; }  // == 2 mod 32
enum { SA_SUM = 0, SA_PACK = 1, SA_UNPACK = 2 };
// img (fused camera solve, LDS form): instead of S | b | diag(U), the
// assembly writes the solver's image of [S + D; -b^T] itself -- the lower
// block triangle of the N x ld padded matrix the factorisation runs on (the
// LM diagonal clamp(diag U) / radius added, row n = -b^T, the last diagonal
// block symmetric, identity padding), written through -- so the solve copies
// it into LDS with a few LDS-DMA instructions instead of an element-wise load
// (whose one-time code dominated the launch, tools/drivers.py solve_ts).
//
// claim (fused assembly): the unit is first claimed for launch generation
// `gen` (atomic max on its claim word, issued before the loads, its result
// read only before the stores); a unit another workgroup claimed first is
// left to it -- no stores, and the function returns false.
template <int NTH, bool SC1>
__device__ bool s_assemble_body(const Geo& g, const Bufs& b, int blk, int full, int mode = SA_SUM,
                                double* img = nullptr, const Opts* o = nullptr, unsigned* claim = nullptr,
                                unsigned gen = 0) {
  constexpr int EL = NTH / kSaGroups;
  __shared__ double part[kSaGroups][EL];
  __shared__ int s_claimed;
  unsigned claim_old = 0;
  if (claim && threadIdx.x == 0) claim_old = me_roster_dev::fetch_max(claim, gen);  // (roster.hpp CLAIM, split)
  const State* st = b.st;
  const bool live = !(st->done || st->final_pass);  // final pass: no step follows, S is not needed
  const int n = g.n6;
  const int e = threadIdx.x % EL, grp = threadIdx.x / EL;
  const int idx = blk * EL + e;
  int gr = -1, gc = -1;  // position in the (padded) system [S | b]
  bool diag = false;
  if (idx < g.npairs * 256) {
    int p = idx >> 8, I = 0;
    while (p >= g.T - I) {  // tile pair p -> (I, J): row I holds T - I pairs
      p -= g.T - I;
      ++I;
    }
    const int J = I + p;
    diag = I == J;
    gr = 16 * I + ((idx >> 4) & 15);
    gc = 16 * J + (idx & 15);
  }
  // S entries (gr, gc < n) and the right-hand side (gc == n); the padding is skipped
  const bool use = live && gr >= 0 && gr < n && gc <= n;
  const bool fail = st->fail || (mode == SA_UNPACK && b.xch[xo_fail(g)] != 0.0);  // (unpack: any rank's failure)
  double acc = 0.0;
  if (use && !fail && mode != SA_UNPACK) {
    // the partials of the runs covering this tile (run order): entries grp,
    // grp + 8, ... added in order; their loads issued 8 at a time
    // (independent addresses: one memory latency per batch, not per add)
#ifndef ME_SA_BATCH
#define ME_SA_BATCH 16
#endif
    if (g.sorted) {
      // whole lists (padded with -1 at plan time): no wait for the tile's count
      // before the list loads -- two rounds of latency (list, partials) per batch
      const int cnt = g.nruns;
      const int* tl = b.tl + (long)(idx >> 8) * g.nruns;
      const double* src = b.Spart + (idx & 255);
      for (int q0 = grp; q0 < cnt; q0 += ME_SA_BATCH * kSaGroups) {
        int sl[ME_SA_BATCH];
#pragma unroll
        for (int k = 0; k < ME_SA_BATCH; ++k) {
          const int q = q0 + k * kSaGroups;
          sl[k] = q < cnt ? tl[q] : -1;
        }
        double v[ME_SA_BATCH];
#pragma unroll
        for (int k = 0; k < ME_SA_BATCH; ++k) v[k] = sl[k] >= 0 ? src[(long)sl[k] * 256] : 0.0;
#pragma unroll
        for (int k = 0; k < ME_SA_BATCH; ++k)
          if (sl[k] >= 0) acc += v[k];
      }
    } else {  // every run holds every tile, at slot run * npairs + tile
      const double* src = b.Spart + idx;
      const long stride = (long)g.npairs * 256;
      for (int q0 = grp; q0 < g.nruns; q0 += ME_SA_BATCH * kSaGroups) {
        double v[ME_SA_BATCH];
#pragma unroll
        for (int k = 0; k < ME_SA_BATCH; ++k) {
          const int q = q0 + k * kSaGroups;
          v[k] = q < g.nruns ? src[q * stride] : 0.0;
        }
#pragma unroll
        for (int k = 0; k < ME_SA_BATCH; ++k)
          if (q0 + k * kSaGroups < g.nruns) acc += v[k];
      }
    }
  }
  part[grp][e] = acc;
  if (claim && threadIdx.x == 0) s_claimed = claim_old < gen;
  __syncthreads();
  if (claim && !s_claimed) return false;
  if (img != nullptr) {
    // every element of the tile pair when live (padding included): the image
    // is complete without any other writer
    if (grp == 0 && live && gr >= 0) {
      const int ld = solve_ld(g.Ts);
      double sum = 0.0;
      if (mode == SA_UNPACK) {
        sum = b.xch[idx];
      } else {
#pragma unroll
        for (int k = 0; k < kSaGroups; ++k) sum += part[k][e];
      }
      double v;
      if (gr < n && gc < n) {
        if (mode == SA_UNPACK) {
          v = fail ? 0.0 : sum;
        } else {
          v = 0;
          if (gr / 6 == gc / 6) v = b.U[36 * (gr / 6) + (gr % 6) * 6 + (gc % 6)];
          v = fail ? 0.0 : v - sum;
        }
        if (gr == gc) {
          const double du = mode == SA_UNPACK ? b.xch[xo_diag(g) + gr] : b.U[36 * (gr / 6) + (gr % 6) * 7];
          v += fmin(fmax(du, o->min_diag), o->max_diag) / b.st->radius;
        }
      } else if ((gr < n && gc == n) || (gr == n && gc < n)) {
        const int r = gr < n ? gr : gc;  // (the (n, c) partial equals the (c, n) one bit for bit: Y^T Y)
        v = -(fail ? 0.0 : mode == SA_UNPACK ? sum : b.gcs[r] - sum);
      } else {
        v = gr == gc ? 1.0 : 0.0;  // (n, n) and the padding: identity
      }
      a_st<SC1>(&img[diag ? (long)gr * ld + gc : (long)gc * ld + gr], v);
    }
    return true;
  }
  if (grp == 0 && use) {
    double sum = 0.0;
    if (mode == SA_UNPACK) {
      sum = b.xch[idx];
    } else {
#pragma unroll
      for (int k = 0; k < kSaGroups; ++k) sum += part[k][e];
    }
    if (gc < n) {
      double v = 0;
      if (mode == SA_UNPACK) {
        v = fail ? 0.0 : sum;
      } else {
        if (gr / 6 == gc / 6) v = b.U[36 * (gr / 6) + (gr % 6) * 6 + (gc % 6)];  // U blocks are symmetric
        v = fail ? 0.0 : v - sum;
      }
      if (mode == SA_PACK) {
        b.xch[idx] = v;
      } else if (diag) {
        a_st<SC1>(&b.S[(long)gr * n + gc], v);
      } else {
        a_st<SC1>(&b.S[(long)gc * n + gr], v);
        if (full) b.S[(long)gr * n + gc] = v;
      }
    } else {
      const double bv = fail ? 0.0 : mode == SA_UNPACK ? sum : b.gcs[gr] - sum;
      const double du = mode == SA_UNPACK ? b.xch[xo_diag(g) + gr] : b.U[36 * (gr / 6) + (gr % 6) * 7];
      if (mode == SA_PACK) {
        b.xch[idx] = bv;
        b.xch[xo_diag(g) + gr] = du;
      } else {
        a_st<SC1>(&b.bvec[gr], bv);
        a_st<SC1>(&b.diagU[gr], du);
      }
    }
  } else if (mode == SA_PACK && grp == 0 && idx < g.npairs * 256) {
    b.xch[idx] = 0.0;  // padding (and a finished solve): defined values in the exchange
  }
  return true;
}

// mode SA_PACK (sharded, before the exchange): the last workgroup writes the
// exchange tail instead of finalizing; SA_UNPACK (sharded, after it, when
// the camera solve does not unpack itself): as SA_SUM from the exchange.
__global__ __launch_bounds__(kBlock) void s_assemble_kernel(Geo g, Bufs b, Opts o, const double* gc_raw, int full,
                                                            int mode, double* img = nullptr) {
  static_assert(kBlock == kFinBlock, "the finalize block runs with the assembly block size");
  if (blockIdx.x == gridDim.x - 1) {
    __shared__ double lds[16];
    if (mode == SA_PACK) {
      xch_tail_body(g, b, gc_raw, lds);
      return;
    }
    if (threadIdx.x < 2) b.ssync[threadIdx.x] = 0u;  // the camera solve that follows starts its steps at 0
    lin_finalize_body(g, b, o, gc_raw, lds);
    return;
  }
  if (mode != SA_PACK && blockIdx.x == 0 && threadIdx.x == 0 && !(b.st->done || b.st->final_pass))
    b.scal[R_COUNT] = (b.st->fail || (mode == SA_UNPACK && b.xch[xo_fail(g)] != 0.0)) ? 1.0 : 0.0;
  s_assemble_body<kBlock, false>(g, b, blockIdx.x, full, mode, img, &o);
}

// One workgroup: S (assembled by s_assemble_kernel, all-reduced in sharded
// mode) + LM diagonal, blocked right-looking Cholesky with 16x16 blocks.
// The right-hand side rides along as an extra row [-b^T | 1] below S, so the
// factorisation also yields z = L^-1 (-b) (no separate forward solve).
// Per block column J:
//  * diagonal block (wave 0): L_JJ and X_J = L_JJ^-1 together, lane = (row,
//    4-column group), pivots by readlane, row broadcast by quad DPP;
//  * panel L_IJ = A_IJ X_J^T on v_mfma_f64_16x16x4f64, one wave per block row;
//  * trailing update A_IK -= L_IJ L_KJ^T on the matrix cores.
// Then the backward solve L^T y = z in wave 0 with the block inverses.
// The matrix is padded to N = 16 Ts >= n + 1 with an identity block.
#ifndef ME_SOLVE_BLOCK
#define ME_SOLVE_BLOCK 512
#endif
constexpr int kSolveBlock = ME_SOLVE_BLOCK;
constexpr int kLoadBatch = 32;
#define SOLVE_STAMP(i)                                                                      \
  do {                                                                                      \
    if ((skip & 256) && tid == 0) st->stamps[(i)] += (long long)__builtin_amdgcn_s_memtime(); \
  } while (0)
#define SOLVE_START(i)                                                                      \
  do {                                                                                      \
    if ((skip & 256) && tid == 0) st->stamps[(i)] -= (long long)__builtin_amdgcn_s_memtime(); \
  } while (0)

#ifdef ME_SOLVE_TS  // timing experiment only (tools/drivers.py solve_ts): wall-clock phases of cam_solve, 100 MHz ticks
// [1] lin_finalize, [2] assembly wait, [3] load, [4] factorisation, [5] backward
// solve, [6] candidate / cost tail, [8] last assembler exit - wg 0 entry,
// [9] first assembler entry - wg 0 entry, [10] s_memtime ticks of [1..6], [15] calls
__device__ long long g_solve_ts[24];
__device__ unsigned long long g_asm_first = ~0ull, g_asm_last = 0ull;
#define STS_DECL long long sts_prev_ = 0, sts_t0_ = 0, sts_c0_ = 0
#define STS_BEGIN()                                                        \
  do {                                                                     \
    if (threadIdx.x == 0) {                                                \
      sts_t0_ = sts_prev_ = (long long)__builtin_amdgcn_s_memrealtime();   \
      sts_c0_ = (long long)__builtin_amdgcn_s_memtime();                   \
    }                                                                      \
  } while (0)
#define STS(k)                                                             \
  do {                                                                     \
    if (threadIdx.x == 0) {                                                \
      const long long t_ = (long long)__builtin_amdgcn_s_memrealtime();    \
      atomicAdd((unsigned long long*)&g_solve_ts[(k)], (unsigned long long)(t_ - sts_prev_)); \
      sts_prev_ = t_;                                                      \
    }                                                                      \
  } while (0)
#define STS_END()                                                          \
  do {                                                                     \
    if (threadIdx.x == 0) {                                                \
      atomicAdd((unsigned long long*)&g_solve_ts[10],                      \
                (unsigned long long)((long long)__builtin_amdgcn_s_memtime() - sts_c0_)); \
      atomicAdd((unsigned long long*)&g_solve_ts[15], 1ull);               \
    }                                                                      \
  } while (0)
#define STS_ASM()                                                          \
  do {                                                                     \
    if (threadIdx.x == 0) {                                                \
      const unsigned long long a_ = atomicExch(&g_asm_last, 0ull);         \
      const unsigned long long f_ = atomicExch(&g_asm_first, ~0ull);       \
      if (a_) {                                                            \
        atomicAdd((unsigned long long*)&g_solve_ts[8], (unsigned long long)((long long)a_ - sts_t0_)); \
        atomicAdd((unsigned long long*)&g_solve_ts[9], (unsigned long long)((long long)f_ - sts_t0_)); \
      }                                                                    \
    }                                                                      \
  } while (0)
#else
#define STS_DECL
#define STS_BEGIN() do {} while (0)
#define STS(k) do {} while (0)
#define STS_END() do {} while (0)
#define STS_ASM() do {} while (0)
#endif

// dynamic LDS: X (Ts x 256) | z/y (N) | row exchange (256) | A (N x ld, when it fits)
constexpr int kXchDoubles = 192;  // per buffer: the one-wave diagonal factor's LDS scratch (ME_DIAG_GATHER 0)
constexpr int kDiagLd = 17;  // staged diagonal block (global-memory form): 16 x 17 doubles
__host__ __device__ inline size_t solve_small_doubles(int Ts) {
  return 256 * (size_t)Ts + 16 * (size_t)Ts + 2 * (size_t)kXchDoubles + 16 * kDiagLd;
}
__host__ __device__ inline size_t solve_a_doubles(int Ts) { return (size_t)(16 * Ts) * solve_ld(Ts); }

// Global-memory form (windows whose [S; -b^T] does not fit the LDS, config 4
// and 5): block 0 factors the diagonal blocks and panels as below, and the
// trailing update of each block step is spread over the further workgroups
// of the same launch that joined its roster (roster.hpp: block 0 never waits
// for a workgroup that was not dispatched; with none, it updates the tiles
// itself).  Hand-offs through b.ssync (zeroed by
// s_assemble before every solve): block 0 publishes step J (epoch J + 1)
// once the panel of J is stored (every thread: agent-scope release fence,
// barrier, release store); a worker waits for the epoch (acquire, barrier),
// updates its tiles of step J and counts itself done (fence, barrier,
// release add); block 0 waits for all workers before the next diagonal
// block.  Every spin is also bounded (a safety net: every partner waited on
// is resident): a missing partner ends the solve as a failed step, never a
// hang.
constexpr unsigned kSolveTerm = 0x40000000u;  // epoch: stop (block 0 failed)
// Hand-off form (MI355X_MICROARCH.md, inter-workgroup visibility, Valid forms
// row 1): every store of A is write-through (sc1), every storing wave drains
// (vmcnt 0) before the workgroup barrier, ONE lane then stores the epoch / adds
// to the counter (agent-scope atomic), the consumer polls with an sc1 load and
// reads A only with sc1 loads after its barrier -- no release fence (an L2
// write-back) and no acquire (an L1 invalidate) per hand-off.
constexpr long kSolveSpin = 1L << 21;         // bounded waits (~0.5 s with s_sleep)
constexpr int kSkipImg = 4096;                // cam_solve `skip` bit: [S + D; -b^T] already in Abuf (solver layout)
constexpr int kSkipRosterNow = 8192;          // cam_solve `skip` bit (test hook): the roster closes at once
#ifndef ME_SOLVE_IMG
#define ME_SOLVE_IMG 1  // non-fused assembly writes the solver's image (0: S | b | diag U, loaded by the solve)
#endif
constexpr int kSolveMwMinTs = 16;             // block steps from which the trailing workers are used

template <bool SC1>
__device__ void trailing_tiles(double* A, int ld, int Ts, int J, int first, int stride, int lane) {
  const int j0 = 16 * J;
  const int rem = Ts - J - 1;
  const int npairs = rem * (rem + 1) / 2;
  for (int p = first; p < npairs; p += stride) {
    int I = 0, q = p;
    while (q > I) {
      q -= I + 1;
      ++I;
    }
    const int i0 = 16 * (J + 1 + I), k0 = 16 * (J + 1 + q);
    double av[4], bv[4];
    double4_t acc;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int cc = j0 + 4 * s + (lane >> 4);
      av[s] = -a_ld<SC1>(&A[(long)(i0 + (lane & 15)) * ld + cc]);
      bv[s] = a_ld<SC1>(&A[(long)(k0 + (lane & 15)) * ld + cc]);
      acc[s] = a_ld<SC1>(&A[(long)(i0 + (lane >> 4) + 4 * s) * ld + k0 + (lane & 15)]);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s], bv[s], acc, 0, 0, 0);
#pragma unroll
    for (int s = 0; s < 4; ++s) a_st<SC1>(&A[(long)(i0 + (lane >> 4) + 4 * s) * ld + k0 + (lane & 15)], acc[s]);
  }
}

// Trailing tiles of block step J split for the lookahead of the one-workgroup
// solve: `col` = the tiles of column J + 1 only (they feed the next diagonal
// block), else every other tile (the deferred part, overlapped with the next
// diagonal block).  Tiles are dealt round-robin over (first, stride).
template <bool SC1>
__device__ void trailing_split(double* A, int ld, int Ts, int J, bool col, int first, int stride, int lane) {
  const int rem = Ts - J - 1;
  const int cnt = col ? rem : rem * (rem - 1) / 2;
  const int j0 = 16 * J;
  for (int p = first; p < cnt; p += stride) {
    int I, q;
    if (col) {
      I = p;
      q = 0;
    } else {  // p = I (I - 1) / 2 + q - 1, 1 <= q <= I
      I = 1;
      q = p;
      while (q >= I) {
        q -= I;
        ++I;
      }
      ++q;
    }
    const int i0 = 16 * (J + 1 + I), k0 = 16 * (J + 1 + q);
    double av[4], bv[4];
    double4_t acc;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int cc = j0 + 4 * s + (lane >> 4);
      av[s] = -a_ld<SC1>(&A[(long)(i0 + (lane & 15)) * ld + cc]);
      bv[s] = a_ld<SC1>(&A[(long)(k0 + (lane & 15)) * ld + cc]);
      acc[s] = a_ld<SC1>(&A[(long)(i0 + (lane >> 4) + 4 * s) * ld + k0 + (lane & 15)]);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s], bv[s], acc, 0, 0, 0);
#pragma unroll
    for (int s = 0; s < 4; ++s) a_st<SC1>(&A[(long)(i0 + (lane >> 4) + 4 * s) * ld + k0 + (lane & 15)], acc[s]);
  }
}

// One trailing tile of block step J: A_IK -= L_IJ L_KJ^T (16 x 16, v_mfma_f64_16x16x4f64).
template <bool SC1>
__device__ __forceinline__ void trailing_tile(double* A, int ld, int J, int I, int K, int lane) {
  const int j0 = 16 * J, i0 = 16 * I, k0 = 16 * K;
  double av[4], bv[4];
  double4_t acc;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int cc = j0 + 4 * s + (lane >> 4);
    av[s] = -a_ld<SC1>(&A[(long)(i0 + (lane & 15)) * ld + cc]);
    bv[s] = a_ld<SC1>(&A[(long)(k0 + (lane & 15)) * ld + cc]);
    acc[s] = a_ld<SC1>(&A[(long)(i0 + (lane >> 4) + 4 * s) * ld + k0 + (lane & 15)]);
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s], bv[s], acc, 0, 0, 0);
#pragma unroll
  for (int s = 0; s < 4; ++s) a_st<SC1>(&A[(long)(i0 + (lane >> 4) + 4 * s) * ld + k0 + (lane & 15)], acc[s]);
}

// The same update of one tile, the result left in the MFMA accumulator (lane
// l holds A_IK[(l >> 4) + 4 s][l & 15] in element s: the layout the one-wave
// diagonal factorisation takes its block in) instead of stored.
// (Diagonal tile, K = I: both MFMA operands come from the same panel tile.)
template <bool SC1 = false>
__device__ __forceinline__ double4_t trailing_diag_acc(const double* A, int ld, int J, int I, int lane) {
  const int j0 = 16 * J, i0 = 16 * I;
  double av[4], bv[4];
  double4_t acc;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int cc = j0 + 4 * s + (lane >> 4);
    bv[s] = a_ld<SC1>(&A[(long)(i0 + (lane & 15)) * ld + cc]);
    av[s] = -bv[s];
    acc[s] = a_ld<SC1>(&A[(long)(i0 + (lane >> 4) + 4 * s) * ld + i0 + (lane & 15)]);
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s], bv[s], acc, 0, 0, 0);
  return acc;
}

// A bounded cross-workgroup wait of the camera solve timed out (a partner
// not co-resident): me_ba_* returns ME_ERR_STATE.  One GPU: the solve ends
// here.  Sharded: the rank must keep issuing the same collectives
// as its peers, so it only fails its steps -- st->fail reaches every rank
// through the step exchange (R_COUNT), the camera solve keeps failing while
// spin_err is set, and every rank ends alike after max_invalid rejected steps
// (decide, on exchanged values).
__device__ __forceinline__ void spin_timeout(const Bufs& b) {
  State* st = b.st;
  st->spin_err = 1;
  st->fail = 1;
  if (!b.xch) {
    st->done = 1;
    st->termination = 2;
  }
}

// Workers of the multi-workgroup solve.  Tile (I, K), 1 <= K <= I < Ts, is
// owned by one wave of one worker for the whole solve (linear index
// (I-1) I / 2 + K - 1, dealt round-robin over the workers' waves), so its
// successive updates are ordered by that wave's program order.  Per block step
// J (after block 0 publishes the panel of J): the tiles of column J + 1 below
// the diagonal and the diagonal tile (J + 2, J + 2) first -- block 0 needs
// them for the panel of J + 1 and the diagonal block J + 2 -- then the worker
// signals, then its other tiles.  The diagonal tile (J + 1, J + 1) is left to
// block 0, which applies step J to it in registers and factors it while the
// workers update column J + 1.
//
// The workers join the solve's roster (roster.hpp) first; block 0 closes it
// and the tiles are dealt over the P workers that joined (worker p, wave w:
// slot p nw + w), so block 0 never waits for a worker that was not
// dispatched.  Which wave updates a tile does not change its operations:
// the results are the same for any P.
__device__ void cam_solve_worker(const Geo& g, const Bufs& b, int nworkers) {
  __shared__ unsigned sep;
  __shared__ int s_pid, s_np;
  const State* st = b.st;
  if (st->done) return;  // block 0 returns for the same reason (before its close)
  if (threadIdx.x == 0) {
    // (no last-joiner close: the workers depend on block 0, which may not be
    // dispatched yet; without its count within kAbandonTicks they close the
    // roster empty and leave, and block 0 works alone)
    int pid = me_roster::join<me_roster_dev>(b.roster, 0u), np = 0;
    if (pid >= 0) {
      np = me_roster::count_or_abandon<me_roster_dev>(b.roster);
      if (np < 0) {  // a first closer that never published (not reachable: it is running)
        b.st->spin_err = 1;
        atomicOr(&b.st->pad[0], 1);  // spin site: worker roster count
        pid = -1;
      } else if (pid >= np) {
        pid = -1;  // the roster was abandoned (np = 0): block 0 updates every tile
      }
    }
    s_pid = pid;
    s_np = np;
  }
  __syncthreads();
  if (s_pid < 0) return;  // dispatched after the close: the joined workers own every tile
  if (st->fail || b.scal[R_COUNT] != 0.0) return;  // block 0 skips the factorisation for the same reasons
  const int Ts = g.Ts, ld = solve_ld(Ts);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  const int slot0 = s_pid * nw + wave, nslots = s_np * nw;
  const int ntiles = (Ts - 1) * Ts / 2;
  for (int J = 0; J + 1 < Ts; ++J) {
    if (tid == 0) {
      unsigned e = 0;
      long k = 0;
      for (; k < kSolveSpin; ++k) {
        e = __hip_atomic_load(b.ssync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (e >= (unsigned)(J + 1)) break;
        __builtin_amdgcn_s_sleep(2);
      }
      sep = k == kSolveSpin ? kSolveTerm : e;
      if (k == kSolveSpin) {  // block 0 never published the step: the solve ends in error
        b.st->spin_err = 1;
        atomicOr(&b.st->pad[0], 2);  // spin site: worker step poll
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads behind the poll
    __syncthreads();
    if (sep >= kSolveTerm) return;
    for (int pass = 0; pass < 2; ++pass) {
      for (int t = slot0; t < ntiles; t += nslots) {
        int I = 1, r = t;
        while (r >= I) {  // t = (I-1) I / 2 + (K-1)
          r -= I;
          ++I;
        }
        const int K = r + 1;
        // pass 0: column J + 1 below the diagonal tile, and the diagonal tile
        // (J + 2, J + 2); pass 1: the rest.  Tile (J + 1, J + 1) is block 0's
        // (it applies step J to it in registers before factoring it).
        const bool col = K == J + 1 && I > J + 1, nd = I == J + 2 && K == J + 2;
        if (pass == 0 ? (col || nd) : (K > J + 1 && !nd)) trailing_tile<true>(b.Abuf, ld, J, I, K, lane);
      }
      if (pass == 0) {
        drain_and_barrier();
        if (tid == 0) __hip_atomic_fetch_add(b.ssync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// Diagonal block Jd of the LDS-resident system on one wave, from its updated
// values in the accumulator layout (lane l, register r: row (l >> 4) + 4 r,
// column l & 15); false on a non-positive pivot.
__device__ __forceinline__ bool diag_factor_wave(double* A, int ld, double* X, double* xch, int n, int Jd,
                                                 double4_t A4, int lane) {
  const int jd0 = 16 * Jd;
  double* Ablk = A + (long)jd0 * ld + jd0;
  double* XJw = X + 256 * Jd;
  const int q = lane >> 4, c = lane & 15;
  bool ok = true;
  double4_t Y4;
#pragma unroll
  for (int r = 0; r < 4; ++r) Y4[r] = (q + 4 * r == c) ? 1.0 : 0.0;
  diag_round_mfma<0>(A4, Y4, q, c, n - jd0, ok, Ablk, ld, XJw, xch);
  diag_round_mfma<1>(A4, Y4, q, c, n - jd0, ok, Ablk, ld, XJw, xch);
  diag_round_mfma<2>(A4, Y4, q, c, n - jd0, ok, Ablk, ld, XJw, xch);
  diag_round_mfma<3>(A4, Y4, q, c, n - jd0, ok, Ablk, ld, XJw, xch);
  return ok;
}
__device__ __forceinline__ double4_t diag_load_wave(const double* A, int ld, int Jd, int lane) {
  const double* Ablk = A + (long)(16 * Jd) * ld + 16 * Jd;
  double4_t A4;
#pragma unroll
  for (int r = 0; r < 4; ++r) A4[r] = Ablk[((lane >> 4) + 4 * r) * ld + (lane & 15)];
  return A4;
}

// y = sum_m X[m][t] u_m over the 16 lanes of this lane's 16-lane row (lane m
// of the row holds u_m; lane t reads column t of X): DPP row broadcasts, in m
// order.
// (four partial sums over m mod 4, then (y0 + y1) + (y2 + y3): a 4-deep chain)
template <int M>
__device__ __forceinline__ void row_dot16_acc(double u, const double* X, int t, double (&y)[4]) {
  if constexpr (M < 16) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(u), 0x150 + M, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(u), 0x150 + M, 0xf, 0xf, false);
    y[M & 3] = fma(X[M * 16 + t], __hiloint2double(hi, lo), y[M & 3]);
    row_dot16_acc<M + 1>(u, X, t, y);
  }
}
__device__ __forceinline__ double row_dot16(double u, const double* X, int t) {
  double y[4] = {0.0, 0.0, 0.0, 0.0};
  row_dot16_acc<0>(u, X, t, y);
  return (y[0] + y[1]) + (y[2] + y[3]);
}

// kMode: 0 = [S; -b^T] in LDS, one workgroup; 1 = in global memory, one workgroup;
// 2 = in global memory, trailing updates on `nworkers` more workgroups (sc1 hand-offs)
template <int kMode>
// Fused assembly (nasm > 0; single GPU, modes 0 and 1): workgroups 1..nasm
// assemble S | b | diag(U) from the Schur partials (s_assemble_body, written
// through) and count themselves done on b.cnt[g.m + 3]; workgroup 0 runs the
// linearisation bookkeeping (lin_finalize) and, unless the solve has ended,
// waits for the count (bounded), re-arms it and reads S with sc1 loads.  One
// launch per LM iteration fewer than s_assemble_kernel + cam_solve_kernel.
__global__ __launch_bounds__(kSolveBlock) void cam_solve_kernel(Geo g, Bufs b, Opts o, int skip, int nworkers, int nasm,
                                                                const double* gc_raw, unsigned asm_gen) {
  extern __shared__ double smem[];
  __shared__ double red[64];
  __shared__ int sfail;
  constexpr bool kLds = kMode == 0, kSc1 = kMode == 2;
  // lookahead: the trailing update of step J outside column J + 1 overlaps the
  // next diagonal block (config 3: 44.2 -> 42.0 us).  Measured and dropped:
  // the panel fused with the column-(J+1) update in one phase (transposed
  // panel tiles as MFMA operands, no barrier between; 43.8 us) and a one-wave
  // backward solve without workgroup barriers (unchanged).
  // Also measured and dropped (git history keeps the code):
  // the panel tile kept in registers for the diagonal update, E = L^-T
  // accumulated by the workers, a one-wave backward solve, block 0 factored
  // beside the LDS copy, a four-wave diagonal factor.
  constexpr bool kLook = kMode != 2;
  // LDS-resident system: wave 0 alone on the critical path (see below)
  constexpr bool kPipe = kLds;
  __shared__ unsigned pflag, pdone;
  if (kMode == 2 && blockIdx.x > 0) {
    cam_solve_worker(g, b, nworkers);
    return;
  }
  unsigned* asm_cnt = b.cnt + g.m + 3;
  if (kMode != 2 && nasm > 0 && blockIdx.x > 0) {
#ifdef ME_SOLVE_TS
    if (threadIdx.x == 0) atomicMin(&g_asm_first, (unsigned long long)__builtin_amdgcn_s_memrealtime());
#endif
    // Unit u = blockIdx.x - 1, claimed first (s_assemble_body `claim`): block
    // 0 takes the units nobody claimed once it has waited kCloseTicks for them
    // (an assembler held back behind other work, another process's kernels or
    // a CU mask), so it never waits for a workgroup that was not dispatched;
    // a late assembler finds its unit claimed and stores nothing.
    const int u = blockIdx.x - 1;
    // (sharded: the assemblers unpack the all-reduced exchange instead of summing partials)
    const bool mine = s_assemble_body<kSolveBlock, true>(g, b, u, 0, b.xch ? SA_UNPACK : SA_SUM,
                                                         kLds || ME_SOLVE_IMG ? b.Abuf : nullptr, &o,
                                                         b.asm_claim + u, asm_gen);
    drain_and_barrier();  // every wave's written-through stores have left
#ifdef ME_SOLVE_TS
    if (threadIdx.x == 0) atomicMax(&g_asm_last, (unsigned long long)__builtin_amdgcn_s_memrealtime());
#endif
    if (mine && threadIdx.x == 0) __hip_atomic_fetch_add(asm_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  State* st = b.st;
  const bool fused = kMode != 2 && nasm > 0;
  STS_DECL;
  STS_BEGIN();
  __shared__ int s_steal;
  if (fused) {
    lin_finalize_body(g, b, o, gc_raw, red);
    STS(1);
    if (threadIdx.x == 0) {
      const int live = !st->done;
      // (what s_assemble's first block writes in the unfused form; read by decide)
      b.scal[R_COUNT] = (st->fail || (b.xch && b.xch[xo_fail(g)] != 0.0)) ? 1.0 : 0.0;
      // the assemblers' units: wait kCloseTicks for them, then claim and do
      // every unit still unclaimed here (normally none)
      s_steal = 0;
      if (live) {
        const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
        const long long lim = (skip & kSkipRosterNow) ? 0 : me_roster::kCloseTicks;
        while (__hip_atomic_load(asm_cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)nasm) {
          if ((long long)__builtin_amdgcn_s_memrealtime() - t0 >= lim) {
            s_steal = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
    }
    __syncthreads();
    if (s_steal) {
      __shared__ int s_taken;
      for (int u = 0; u < nasm; ++u) {
        // one decision for the whole workgroup (thread 0's load, through LDS):
        // per-wave loads could see an assembler's claim land between them, and
        // waves that skipped the unit would then meet the others' barriers
        // inside s_assemble_body at the wrong place (round 6: the count never
        // completed -- an intermittent hand-off timeout with another process on
        // the GPU)
        if (threadIdx.x == 0)
          s_taken = __hip_atomic_load(b.asm_claim + u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= asm_gen;
        __syncthreads();
        const bool taken = s_taken != 0;
        __syncthreads();  // s_taken is rewritten for the next unit
        if (taken) continue;
        const bool mine = s_assemble_body<kSolveBlock, true>(g, b, u, 0, b.xch ? SA_UNPACK : SA_SUM,
                                                             kLds || ME_SOLVE_IMG ? b.Abuf : nullptr, &o,
                                                             b.asm_claim + u, asm_gen);
        drain_and_barrier();
        if (mine && threadIdx.x == 0) __hip_atomic_fetch_add(asm_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (threadIdx.x == 0) {
      const int live = !st->done;
      long k = (skip & 512) ? kSolveSpin : 0;  // (512: test hook, a forced timeout on this ctx)
      if (live && (s_steal || k)) {  // (all counted in the first wait: nothing left to wait for)
        for (; k < kSolveSpin; ++k) {
          if (__hip_atomic_load(asm_cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)nasm) break;
          __builtin_amdgcn_s_sleep(1);
        }
      }
      if (live) {
        if (k == kSolveSpin) {
          // a unit never counted (not reachable: every claimed unit's owner is
          // running; kept as a safety net and for the test hook): the solve ends
          // in error (a late count may still come, so the counter is not
          // re-armed: the next plan clears it)
          spin_timeout(b);
          atomicOr(&b.st->pad[0], 4);  // spin site: fused assemblers' count
        } else {
          __hip_atomic_store(asm_cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed for the next iteration
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads behind the poll
    __syncthreads();
    STS(2);
    STS_ASM();
    STS(11);
  }
  const int n = g.n6, Ts = g.Ts, N = 16 * Ts;
  const int ld = solve_ld(Ts);
  const int tid = threadIdx.x, nt = blockDim.x;
  const int lane = tid & 63, wave = tid >> 6, nw = nt >> 6;
  double* X = smem;
  double* u = X + 256 * (size_t)Ts;
  double* xch = u + N;  // diagonal-block exchange (2 x kXchDoubles)
  double* A = kLds ? xch + 2 * kXchDoubles : b.Abuf;
  // flags, radius and the whole lower block triangle of [S; -b^T] are
  // requested together: one round of global latency instead of a chain
  const int done = st->done;
  const int fail_in = st->fail || st->spin_err || (fused ? (b.xch && b.xch[xo_fail(g)] != 0.0) : b.scal[R_COUNT] != 0.0) ||
                      (skip & 1024);  // (1024: test hook, a forced solve failure)
  const double radius = st->radius;
  // [S + D; -b^T]: every load of a batch is issued from a computed index
  // before the first use, so a batch costs one round of global latency.
  // (Per-element branches with the use inside them made the compiler wait on
  // every load: the load phase took 15.2 of the 45 us launch at config 3 and
  // 100 of 265 us at config 5, tools/drivers.py solve_ts.)  S | b | diag(U) are one
  // allocation (plan), so every element is an index off b.S.  The LM diagonal
  // (Ceres: clamp(diag(U)) / radius) goes through LDS (u, free until the
  // backward solve), loaded beside the first batch.  Loads are coherent (sc1):
  // the system is written through by this launch's assemblers, or by the
  // previous launch.
  const int CC = (N + 63) >> 6, RT = (N + nw - 1) / nw, NQ = RT * CC;
  const double* S0 = b.S;
  const int nn = n * n;
  // the image of [S + D; -b^T] in Abuf: written by s_assemble_kernel (non-fused), or by this launch's
  // assemblers (fused; written through)
  const bool img_ready = (skip & kSkipImg) != 0 || (fused && (kLds || ME_SOLVE_IMG));
  // LDS-DMA chunks of the image: all, or (pipelined form) the ones holding block row 0 first
  const int dma_bytes = N * ld * 8, dma_chunks = (dma_bytes + 1023) >> 10;
  const int dma_first = kPipe ? min(dma_chunks, (16 * ld * 8 + 1023) >> 10) : dma_chunks;
  auto dma_chunk = [&](int k) {
    const int off = (k << 10) + 16 * lane;
    if (off < dma_bytes)
      __builtin_amdgcn_global_load_lds((const void*)((const char*)b.Abuf + off),
                                       (__attribute__((address_space(3))) void*)((char*)A + (k << 10)), 16, 0,
                                       16 /* sc1 */);
  };
  if (!kLds && img_ready) {
    // the working matrix is Abuf itself: nothing to load.  (Fused: the
    // assemblers' written-through stores bypassed this XCD's L2, which may
    // still hold lines of Abuf from the previous launch's factorisation: an
    // agent-scope acquire invalidates them before the first plain load.)
    if (fused) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  } else if (kLds && img_ready) {
    // the assemblers wrote the solver's image (s_assemble_body img): N x ld
    // doubles, copied by LDS-DMA, 1 KiB per wave-instruction (lane-linear),
    // coherent reads (sc1); the barrier below retires them (vmcnt).  Only the
    // chunks of block row 0 here: the pipelined factorisation (kPipe) has
    // waves 1.. copy the rest while wave 0 factors diagonal block 0.
    if (!done)
      for (int k = wave; k < dma_first; k += nw) dma_chunk(k);
  } else
  for (int q0 = 0; q0 < NQ; q0 += kLoadBatch) {
    double xv[kLoadBatch];
    const int tb = q0 / CC, ub = q0 - tb * CC;  // (t, uu) of the batch's first element, stepped below
    int t = tb, uu = ub;
#pragma unroll
    for (int k = 0; k < kLoadBatch; ++k) {
      const int q = q0 + k;
      const int r = wave + nw * t, c = lane + 64 * uu;
      if (++uu == CC) {
        uu = 0;
        ++t;
      }
      // element class, branch-free: S (r, c < n), b as row n, b as column n
      // of the last diagonal block (it must stay symmetric); others load S[0]
      const bool in = q < NQ && r < N && c < n && (c >> 4) <= (r >> 4);
      const bool colb = q < NQ && c == n && r < n && (r >> 4) == (n >> 4);
      const int ix = in ? (r < n ? r * n + c : (r == n ? nn + c : 0)) : (colb ? nn + r : 0);
      xv[k] = a_ld<true>(S0 + ix);
    }
    if (q0 == 0) {
      STS(12);
      for (int r = tid; r < n; r += nt) u[r] = fmin(fmax(a_ld<true>(S0 + nn + n + r), o.min_diag), o.max_diag) / radius;
      __syncthreads();
      STS(13);
    }
    if (done) return;
    t = tb;
    uu = ub;
#pragma unroll
    for (int k = 0; k < kLoadBatch; ++k) {
      const int q = q0 + k;
      const int r = wave + nw * t, c = lane + 64 * uu;
      if (++uu == CC) {
        uu = 0;
        ++t;
      }
      const bool in = q < NQ && r < N && c < n && (c >> 4) <= (r >> 4);
      const bool colb = q < NQ && c == n && r < n && (r >> 4) == (n >> 4);
      double v = (in && r < n) ? xv[k] : ((in && r == n) || colb) ? -xv[k] : 0.0;
      if (in && r < n && r == c) v += u[r];
      if (q < NQ && r < N && c < N && (c >> 4) <= (r >> 4)) a_st<kSc1>(&A[r * ld + c], (r == c && r >= n) ? 1.0 : v);
    }
  }
  if (done) return;
  // trailing-update workers: close their roster (roster.hpp; at once when the
  // solve fails here anyway) -- the tiles are dealt over those that joined,
  // none of them: block 0 updates them itself (the phased loop)
  __shared__ int s_nwk;
  if (tid == 0) {
    sfail = fail_in;
    pflag = 0u;
    pdone = 0u;
    if (kMode == 2 && nworkers > 0)
      s_nwk = (int)me_roster::close<me_roster_dev>(b.roster, (unsigned)nworkers,
                                                   fail_in || (skip & kSkipRosterNow) ? 0 : me_roster::kCloseTicks);
  }
  if ((skip & 256) && tid == 0) st->stamps[15] += 1;
  SOLVE_START(0);
  __syncthreads();
  STS(3);
  if (sfail) {
    if (tid == 0) st->fail = 1;
    return;
  }
  SOLVE_STAMP(0);
  if constexpr (kPipe) {
    // Wave 0 walks the critical path alone: per block step J it forms the
    // panel tile L_{J+1,J} = A_{J+1,J} X_J^T, publishes it (LDS flag), applies
    // step J to the diagonal tile (J+1, J+1) and factors diagonal block J+1 --
    // no workgroup barrier between.  Meanwhile the workers (waves other than
    // 0 and its SIMD sibling 4) form the other panel tiles of J, update
    // column J + 1 below the diagonal tile (after the flag), and, once every
    // worker's panel tiles are stored (LDS counter), the rest of step J's
    // trailing tiles.  One barrier per step joins both.  Same operations on
    // the same operands as the phased loop below: identical results.
    const bool worker = wave != 0 && !(nw > 4 && wave == 4);
    const int nwk = nw - 1 - (nw > 4 ? 1 : 0);
    const int widx = wave - 1 - (nw > 4 && wave > 4 ? 1 : 0);
    // diagonal block Jd from its (updated) values in the accumulator layout
    auto diag_factor = [&](int Jd, double4_t A4) {
      if (!diag_factor_wave(A, ld, X, xch, n, Jd, A4, lane)) sfail = 1;  // benign race: every writer stores 1
    };
    auto panel_tile = [&](int J, int I) {  // L_IJ = A_IJ X_J^T on the matrix cores
      const int j0 = 16 * J, i0 = 16 * I;
      const double* XJ = X + 256 * J;
      double av[4], bv[4];
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        av[s4] = A[(long)(i0 + (lane & 15)) * ld + j0 + 4 * s4 + (lane >> 4)];
        bv[s4] = XJ[(lane & 15) * 16 + 4 * s4 + (lane >> 4)];
      }
      double4_t acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s4], bv[s4], acc, 0, 0, 0);
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) A[(long)(i0 + (lane >> 4) + 4 * q4) * ld + j0 + (lane & 15)] = acc[q4];
    };
    auto lds_wait = [&](volatile unsigned* f, unsigned want) {
      long k = 0;
      for (; k < kSolveSpin && *f < want; ++k) __builtin_amdgcn_s_sleep(1);
      if (k == kSolveSpin) {
        sfail = 1;
        st->spin_err = 1;
        atomicOr(&st->pad[0], 8);  // spin site: LDS-form step flags (pflag / pdone)
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    };
    if (wave == 0) {
      diag_factor(0, diag_load_wave(A, ld, 0, lane));
    } else if (img_ready && nw > 1) {
      // the rest of the image, beside wave 0's block 0 (its rows are in LDS:
      // the barrier above retired their chunks); retired before the barrier
      for (int k = dma_first + wave - 1; k < dma_chunks; k += nw - 1) dma_chunk(k);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    STS(19);
    __syncthreads();
    for (int J = 0; J + 1 < Ts; ++J) {
      if (sfail) break;
      STS(18);
      if (wave == 0) {
        // step J on the diagonal tile, handed to the factorisation in registers
        // (its updated values are read by no one else: the factorisation
        // overwrites the lower triangle with L, the upper one is never read)
        panel_tile(J, J + 1);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) pflag = (unsigned)(J + 1);
        solve_wave_sync();  // the panel tile just stored is an operand
        STS(16);
        diag_factor(J + 1, trailing_diag_acc(A, ld, J, J + 1, lane));
        STS(17);
      } else if (worker) {
        for (int I = J + 2 + widx; I < Ts; I += nwk) panel_tile(J, I);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) atomicAdd(&pdone, 1u);
        lds_wait(&pflag, (unsigned)(J + 1));
        for (int I = J + 2 + widx; I < Ts; I += nwk) trailing_tile<false>(A, ld, J, I, J + 1, lane);
        lds_wait(&pdone, (unsigned)(nwk * (J + 1)));
        trailing_split<false>(A, ld, Ts, J, false, widx, nwk, lane);  // tiles (I, K), J + 2 <= K <= I
      }
      __syncthreads();
    }
  } else if (kMode == 2 && nworkers > 0 && s_nwk > 0) {
    // Global-memory form with trailing workers (config 5), pipelined like the
    // LDS form: per block step J, wave 0 applies step J - 1 to the diagonal
    // tile (J, J) in registers (the workers left it out) and factors it, while
    // thread 64 waits for the workers' column-J count (their first pass of step
    // J - 1: column J below the diagonal and the diagonal tile (J + 1, J + 1)).
    // Then every wave forms the panel of J, and block 0 publishes step J and
    // goes on to the next diagonal tile without waiting for the workers: their
    // round trip overlaps the next diagonal block.  Same operations on the same
    // operands as the phased loop below: identical results.  (Measured and
    // dropped: wave 0 forming its panel tile transposed in registers and going
    // on without the panel barrier, the other waves publishing through an LDS
    // counter, and LDS-only barriers -- 144 vs 134 us per config-5 solve: the
    // workers' round trip, not wave 0, sets the step.)
    const int c = lane & 15, q = lane >> 4;
    double* Lblk = xch + 2 * kXchDoubles;
    for (int J = 0; J < Ts; ++J) {
      const int j0 = 16 * J;
      double* Ablk = A + (long)j0 * ld + j0;
      if (wave == 0) {
        double4_t A4, Y4;
        if (J > 0) {
          A4 = trailing_diag_acc<true>(A, ld, J - 1, J, lane);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) A4[r] = a_ld<true>(&Ablk[(q + 4 * r) * ld + c]);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) Y4[r] = (q + 4 * r == c) ? 1.0 : 0.0;
        bool ok = true;
        double* XJw = X + 256 * J;
        diag_round_mfma<0>(A4, Y4, q, c, n - j0, ok, Lblk, kDiagLd, XJw, xch);
        diag_round_mfma<1>(A4, Y4, q, c, n - j0, ok, Lblk, kDiagLd, XJw, xch);
        diag_round_mfma<2>(A4, Y4, q, c, n - j0, ok, Lblk, kDiagLd, XJw, xch);
        diag_round_mfma<3>(A4, Y4, q, c, n - j0, ok, Lblk, kDiagLd, XJw, xch);
        solve_wave_sync();
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (c <= q + 4 * r) a_st<true>(&Ablk[(q + 4 * r) * ld + c], Lblk[(q + 4 * r) * kDiagLd + c]);
        if (!ok) sfail = 1;  // benign race: every writer stores 1
        STS(16);
      } else if (tid == 64 && J > 0 && J + 1 < Ts) {
        const unsigned want = (unsigned)s_nwk * (unsigned)J;
        long k = 0;
        for (; k < kSolveSpin; ++k) {
          if (__hip_atomic_load(b.ssync + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want) break;
          __builtin_amdgcn_s_sleep(1);
        }
        if (k == kSolveSpin) {  // a worker not co-resident (narrow CU mask, busy CUs): the solve ends in error
          sfail = 1;
          st->spin_err = 1;
          atomicOr(&st->pad[0], 16);  // spin site: workers' step count
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads behind the poll
      __syncthreads();
      STS(17);
      if (sfail || J + 1 == Ts) break;
      // panel of J on the matrix cores: L_IJ = A_IJ X_J^T
      const double* XJ = X + 256 * J;
      for (int I = J + 1 + wave; I < Ts; I += nw) {
        const int i0 = 16 * I;
        double av[4], bv[4];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          av[s4] = a_ld<true>(&A[(long)(i0 + (lane & 15)) * ld + j0 + 4 * s4 + (lane >> 4)]);
          bv[s4] = XJ[(lane & 15) * 16 + 4 * s4 + (lane >> 4)];
        }
        double4_t acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s4], bv[s4], acc, 0, 0, 0);
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) a_st<true>(&A[(long)(i0 + (lane >> 4) + 4 * q4) * ld + j0 + (lane & 15)], acc[q4]);
      }
      STS(18);
      drain_and_barrier();  // the panel's (and diagonal copy-back's) sc1 stores have left
      if (tid == 0) __hip_atomic_store(b.ssync, (unsigned)(J + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      STS(19);
    }
  } else
  for (int J = 0; J < Ts; ++J) {
    const int j0 = 16 * J;
    SOLVE_START(1);
    // (a) diagonal block + its inverse (wave 0; every wave joins the barrier)
    {
      const int c = lane & 15;
      double* Ablk = A + (long)j0 * ld + j0;
      // global-memory form: the rounds write the block's L into LDS (a round's
      // barrier would otherwise wait for its global stores), copied back after
      double* Lblk = kLds ? Ablk : xch + 2 * kXchDoubles;
      const int lld = kLds ? ld : kDiagLd;
      bool ok = true;
      double* XJw = X + 256 * J;
      {
        // lookahead: the trailing tiles of step J - 1 outside column J run on
        // waves 1-3 and 5-7 while wave 0 factors this block (wave 4 shares
        // wave 0's SIMD and stays out of its way)
        const bool sib = nw > 4 && wave == 4;  // wave 0's SIMD sibling
        if (kLook && J > 0 && wave != 0 && !sib && !(skip & 4))
          trailing_split<kSc1>(A, ld, Ts, J - 1, false, wave - 1 - (nw > 4 && wave > 4), nw - 1 - (nw > 4), lane);
        if (wave == 0 && !(skip & 1)) {
          const int q = lane >> 4;
          double4_t A4, Y4;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            A4[r] = a_ld<kSc1>(&Ablk[(q + 4 * r) * ld + c]);
            Y4[r] = (q + 4 * r == c) ? 1.0 : 0.0;
          }
          diag_round_mfma<0>(A4, Y4, q, c, n - j0, ok, Lblk, lld, XJw, xch);
          diag_round_mfma<1>(A4, Y4, q, c, n - j0, ok, Lblk, lld, XJw, xch);
          diag_round_mfma<2>(A4, Y4, q, c, n - j0, ok, Lblk, lld, XJw, xch);
          diag_round_mfma<3>(A4, Y4, q, c, n - j0, ok, Lblk, lld, XJw, xch);
          if (!kLds) {
            solve_wave_sync();
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (c <= q + 4 * r) a_st<kSc1>(&Ablk[(q + 4 * r) * ld + c], Lblk[(q + 4 * r) * kDiagLd + c]);
          }
          if (!ok) sfail = 1;  // benign race: every writer stores 1
        }
      }
    }
    __syncthreads();
    SOLVE_STAMP(1);
    if (sfail) break;
    SOLVE_START(2);
    // (b) panel on the matrix cores: L_IJ = A_IJ X_J^T
    {
      const double* XJ = X + 256 * J;
      for (int I = J + 1 + wave; I < ((skip & 2) ? 0 : Ts); I += nw) {
        const int i0 = 16 * I;
        double av[4], bv[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          av[s] = a_ld<kSc1>(&A[(long)(i0 + (lane & 15)) * ld + j0 + 4 * s + (lane >> 4)]);
          bv[s] = XJ[(lane & 15) * 16 + 4 * s + (lane >> 4)];
        }
        double4_t acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s], bv[s], acc, 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q) a_st<kSc1>(&A[(long)(i0 + (lane >> 4) + 4 * q) * ld + j0 + (lane & 15)], acc[q]);
      }
      __syncthreads();
    }
    SOLVE_STAMP(2);
    SOLVE_START(3);
    // (c) trailing update on the matrix cores: A_IK -= L_IJ L_KJ^T, J < K <= I
    {
      if (!(skip & 4)) {
        if (kLook)
          trailing_split<kSc1>(A, ld, Ts, J, true, wave, nw, lane);  // column J + 1 now, the rest with the next block
        else
          trailing_tiles<kSc1>(A, ld, Ts, J, wave, nw, lane);
      }
      __syncthreads();
    }
    SOLVE_STAMP(3);
  }
  STS(4);
  if (sfail) {
    if (tid == 0) {
      st->fail = 1;
      if (st->spin_err) spin_timeout(b);  // not a numerical failure: me_ba_* returns an error
      if (kMode == 2 && nworkers > 0) __hip_atomic_store(b.ssync, kSolveTerm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  SOLVE_START(5);
  // backward solve L^T y = z (z = row n of L), block by block.
  // One column per thread (N <= 512): lane cc keeps u[cc] in a register and
  // walks the blocks K from the last down to its own; wave w owns blocks
  // 4w .. 4w + 3 (its 16-lane rows).  Per block K the owning row finalises
  // y_K = X_K^T u_K (its lanes' u by DPP row broadcasts), publishes y_K in
  // LDS and bumps an LDS flag; every lane of a lower block then subtracts
  // L_K^T y_K from its u (the previous form's sums in the same order).  No
  // workgroup barrier on the chain: a wave waits only for the blocks of other
  // waves, and the lanes' L entries of the next block are requested one block
  // ahead (global forms: a memory round trip per block otherwise).
  const int Jlast = (skip & 8) ? -1 : (n - 1) >> 4;
  // Global forms only: in the LDS form the two-barrier loop below is faster
  // (config 3: 3.7 vs 5.3 us); at W = 50 this one is (17.4 vs 19.9 us).
  if (!kLds && N <= nt) {
    if (tid == 0) pflag = 0u;
    __syncthreads();
    const int cc = tid, myJ = cc >> 4, t = cc & 15;
    double acc = (cc < n && myJ <= Jlast) ? a_ld<kSc1>(&A[(long)n * ld + cc]) : 0.0;
    // the L entries of the next block in flight
    constexpr int kPf = 1;  // (3 blocks ahead measured slower: 20.3 vs 17.4 us at W = 50)
    double lpf[kPf][16];
    auto fetchL = [&](int K, double* dst) {
      if (K >= 0 && myJ < K) {
#pragma unroll
        for (int m = 0; m < 16; ++m) dst[m] = a_ld<kSc1>(&A[(long)(16 * K + m) * ld + cc]);
      }
    };
#pragma unroll
    for (int d = 0; d < kPf; ++d) fetchL(Jlast - d, lpf[d]);
    for (int K = Jlast; K >= 4 * wave; --K) {  // (wave-uniform)
      double lk[16];
#pragma unroll
      for (int m = 0; m < 16; ++m) lk[m] = lpf[0][m];
#pragma unroll
      for (int d = 0; d + 1 < kPf; ++d)
#pragma unroll
        for (int m = 0; m < 16; ++m) lpf[d][m] = lpf[d + 1][m];
      fetchL(K - kPf, lpf[kPf - 1]);
      const unsigned want = (unsigned)(Jlast - K + 1);
      if ((K >> 2) == wave) {
        if (myJ == K) {
          double y = row_dot16(acc, X + 256 * K, t);
          y = 16 * K + t < n ? y : 0.0;
          u[16 * K + t] = y;
          acc = y;
        }
        solve_wave_sync();  // y_K in LDS for this wave's lanes
        if (lane == 0) *(volatile unsigned*)&pflag = want;
      } else {
        long k = 0;
        for (; k < kSolveSpin && *(volatile unsigned*)&pflag < want; ++k) __builtin_amdgcn_s_sleep(1);
        if (k == kSolveSpin) {
          sfail = 1;
          st->spin_err = 1;
          atomicOr(&st->pad[0], 32);  // spin site: backward-solve block flags
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      }
      if (myJ < K) {
        double yk[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) yk[m] = u[16 * K + m];
        double a0 = 0.0, a1 = 0.0;
#pragma unroll
        for (int m = 0; m < 16; m += 2) {
          a0 = fma(lk[m], yk[m], a0);
          a1 = fma(lk[m + 1], yk[m + 1], a1);
        }
        acc -= a0 + a1;
      }
    }
    __syncthreads();
  } else {
  // (LDS form, and N > 512: wave 0 forms y_J = X_J^T z_J and every wave
  // updates the entries above the block, two barriers per block)
  for (int c = tid; c < N; c += nt) u[c] = c < n ? a_ld<kSc1>(&A[(long)n * ld + c]) : 0.0;
  __syncthreads();
  for (int J = Jlast; J >= 0; --J) {
    const int j0 = 16 * J;
    if (wave == 0) {
      const double* XJ = X + 256 * J;
      const int t = lane >> 2, gq = lane & 3;
      double s = 0.0;
#pragma unroll
      for (int m = 0; m < 4; ++m) s += XJ[(4 * gq + m) * 16 + t] * u[j0 + 4 * gq + m];
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      solve_wave_sync();
      if (gq == 0) u[j0 + t] = j0 + t < n ? s : 0.0;
    }
    __syncthreads();
    if (j0 > 0) {
      double yj[16];
#pragma unroll
      for (int m = 0; m < 16; ++m) yj[m] = u[j0 + m];
      for (int cc = tid; cc < j0; cc += nt) {
        double a0 = 0.0, a1 = 0.0;
#pragma unroll
        for (int m = 0; m < 16; m += 2) {
          a0 = fma(a_ld<kSc1>(&A[(long)(j0 + m) * ld + cc]), yj[m], a0);
          a1 = fma(a_ld<kSc1>(&A[(long)(j0 + m + 1) * ld + cc]), yj[m + 1], a1);
        }
        u[cc] -= a0 + a1;
      }
    }
    __syncthreads();
  }
  }
  SOLVE_STAMP(5);
  STS(5);
  // the scaled camera step; the candidate cameras and the camera part of the
  // model cost change are pt_step's camera workgroup (cam_step_body), beside
  // the points -- off this launch's serial tail
  for (int r = tid; r < n; r += nt) b.yc[r] = u[r];
  STS(6);
  STS_END();
}

// Point back-substitution and step evaluation, 16 lanes per point (one
// launch for what were three: per-slot W^T Dc y_c, per-point solve, per-
// observation model change / candidate cost).  The lanes of a point take its
// CSR slots round-robin; the slot sums are reduced across the 16 lanes, every
// lane then solves the point's 3x3 system redundantly (no broadcast), and
// each lane evaluates the model cost change and the candidate cost of its own
// observations.  Partials per workgroup, reduced in fixed order by
// step_finalize (deterministic).
// Step partials -> scal (fixed order).  In single-GPU mode the same workgroup
// then runs the Ceres step handling (decide); in sharded mode the host
// all-reduces scal between step_partials and a decide-only launch.
// R_COUNT of a step whose camera solve hit a hand-off timeout: summed over
// the ranks it stays >= kSpinFlag, so every rank of a sharded solve ends at
// the same iteration with spin_err (ME_ERR_STATE) -- no rank is left waiting
// in a collective the others no longer issue.
constexpr double kSpinFlag = 65536.0;

// The Ceres step handling on a State-like object (the device State itself,
// or the finalizing thread's register copy) and the reduced step scalars.
template <class S>
__device__ __forceinline__ void decide_t(S& st, const double* scal, const Opts& o) {
  st.accepted = 0;
  if (scal[R_COUNT] >= kSpinFlag) {
    st.spin_err = 1;
    st.done = 1;
    st.termination = 2;
    return;
  }
  const double model_change = scal[R_MODEL];
  const bool fail = st.fail || scal[R_COUNT] != 0.0;
  st.fail = 0;  // consumed: the next iteration starts clean
  if (fail || !(model_change > 0.0)) {
    st.invalid_count += 1;
    if (st.invalid_count >= o.max_invalid) {
      st.done = 1;
      st.termination = 2;
      return;
    }
    st.radius = st.radius / st.decrease;
    st.decrease *= 2.0;
    return;
  }
  st.invalid_count = 0;
  const double cand_cost = scal[R_CAND];
  const double step_norm = sqrt(scal[R_STEP2] + st.cam_step2);
  const double x_norm = sqrt(scal[R_XN2] + st.cam_xn2);
  st.cand_cost = cand_cost;
  st.model_change = model_change;
  if (step_norm <= o.parameter_tolerance * (x_norm + o.parameter_tolerance)) {
    st.done = 1;
    st.termination = 0;
    return;
  }
  if (fabs(st.x_cost - cand_cost) <= o.function_tolerance * st.x_cost) {
    st.done = 1;
    st.termination = 0;
    return;
  }
  const double q = (st.x_cost - cand_cost) / model_change;
  st.last_q = q;
  if (q > o.min_rel_decrease) {
    st.cur = 1 - st.cur;
    st.x_cost = cand_cost;
    st.successful += 1;
    st.accepted = 1;
    const double t = 2.0 * q - 1.0;
    st.radius = st.radius / fmax(1.0 / 3.0, 1.0 - pow(t, 3.0));
    st.radius = fmin(o.max_radius, st.radius);
    st.decrease = 2.0;
    st.need_lin = 1;
  } else {
    st.radius = st.radius / st.decrease;
    st.decrease *= 2.0;
  }
}

__device__ void decide(Bufs& b, const Opts& o) { decide_t(*b.st, b.scal, o); }

// The fields decide_t reads or writes, loaded by the finalizing thread in one
// round before the partial reduce (round 6: the decision's dependent State
// loads were half of the step's finalize tail, ME_STEP_TS)
struct DecideState {
  int cur, need_lin, done, termination, successful, invalid_count, fail, accepted, spin_err;
  double radius, decrease, x_cost, cand_cost, model_change, cam_step2, cam_xn2, cam_model, last_q;
  __device__ __forceinline__ void load(const State* st) {
    cur = st->cur; need_lin = st->need_lin; done = st->done; termination = st->termination;
    successful = st->successful; invalid_count = st->invalid_count; fail = st->fail; accepted = st->accepted;
    spin_err = st->spin_err; radius = st->radius; decrease = st->decrease; x_cost = st->x_cost;
    cand_cost = st->cand_cost; model_change = st->model_change; last_q = st->last_q;
    // (written through by this launch's camera workgroup, cam_step_body)
    cam_step2 = a_ld<true>(&st->cam_step2);
    cam_xn2 = a_ld<true>(&st->cam_xn2);
    cam_model = a_ld<true>(&st->cam_model);
  }
  __device__ __forceinline__ void store(State* st) const {
    st->cur = cur; st->need_lin = need_lin; st->done = done; st->termination = termination;
    st->successful = successful; st->invalid_count = invalid_count; st->fail = fail; st->accepted = accepted;
    st->spin_err = spin_err; st->radius = radius; st->decrease = decrease; st->x_cost = x_cost;
    st->cand_cost = cand_cost; st->model_change = model_change; st->last_q = last_q;
  }
};

#ifdef ME_STEP_TS  // timing experiment only: phase split of pt_step workgroup 0 (and of the finalizing workgroup)
__device__ unsigned long long g_step_ts[12];
#define STEP_T(i)                                                                          \
  do {                                                                                     \
    if (blockIdx.x == 0 && threadIdx.x == 0) {                                             \
      const long long t_ = (long long)__builtin_amdgcn_s_memtime();                        \
      if ((i) > 0) atomicAdd(&g_step_ts[(i)], (unsigned long long)(t_ - step_prev_));      \
      else atomicAdd(&g_step_ts[0], 1ull);                                                 \
      step_prev_ = t_;                                                                     \
    }                                                                                      \
  } while (0)
#define STEP_FIN_T(i)                                                                      \
  do {                                                                                     \
    if (threadIdx.x == 0) {                                                                \
      const long long t_ = (long long)__builtin_amdgcn_s_memtime();                        \
      atomicAdd(&g_step_ts[(i)], (unsigned long long)(t_ - fin_prev_));                    \
      fin_prev_ = t_;                                                                      \
    }                                                                                      \
  } while (0)
#else
#define STEP_T(i) \
  do {            \
  } while (0)
#define STEP_FIN_T(i) \
  do {                \
  } while (0)
#endif
__device__ void step_finalize_body(const Geo& g, Bufs b, const Opts& o, int do_decide) {
  __shared__ double rows[1024 / 16 * 4];
  State* st = b.st;
#ifdef ME_STEP_TS
  long long f0 = (long long)__builtin_amdgcn_s_memtime();
#endif
  // the decision's State fields, requested with the partials (one round)
  DecideState ds;
  if (threadIdx.x == 0) ds.load(st);
  double v[4] = {0, 0, 0, 0};
  for (int i = threadIdx.x; i < g.nblk_step; i += blockDim.x) {  // (written through by pt_step's workgroups)
    v[0] += a_ld<true>(&b.part[R_MODEL * g.pstride + i]);
    v[1] += a_ld<true>(&b.part[R_CAND * g.pstride + i]);
    v[2] += a_ld<true>(&b.part[R_STEP2 * g.pstride + i]);
    v[3] += a_ld<true>(&b.part[R_XN2 * g.pstride + i]);
  }
#ifdef ME_STEP_TS
  if (threadIdx.x == 0) {
    const long long t_ = (long long)__builtin_amdgcn_s_memtime();
    atomicAdd(&g_step_ts[8], (unsigned long long)(t_ - f0));
    f0 = t_;
  }
#endif
  // the block's sums: 16-lane row sums by DPP, then the rows in order (VALU and
  // one LDS round; round 6: six lane-shuffle rounds per value before)
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    double x = v[u];
    x += dpp_f64<kDppQuadSwap1>(x);
    x += dpp_f64<kDppQuadSwap2>(x);
    x += dpp_f64<kDppRowHalfMirror>(x);
    x += dpp_f64<kDppRowMirror>(x);
    v[u] = x;
  }
  if ((threadIdx.x & 15) == 0)
#pragma unroll
    for (int u = 0; u < 4; ++u) rows[(threadIdx.x >> 4) * 4 + u] = v[u];
  __syncthreads();
#ifdef ME_STEP_TS
  if (threadIdx.x == 0) {
    const long long t_ = (long long)__builtin_amdgcn_s_memtime();
    atomicAdd(&g_step_ts[9], (unsigned long long)(t_ - f0));
    f0 = t_;
  }
#endif
  if (threadIdx.x == 0) {
    double out[4] = {0.0, 0.0, 0.0, 0.0};
    for (int r = 0; r < (int)(blockDim.x >> 4); ++r)
#pragma unroll
      for (int u = 0; u < 4; ++u) out[u] += rows[r * 4 + u];
    double scal[R_COUNT + 1];
    scal[R_MODEL] = out[0] + ds.cam_model;  // (+ this rank's camera part, cam_solve)
    scal[R_CAND] = out[1];
    scal[R_STEP2] = out[2];
    scal[R_XN2] = out[3];
    scal[R_COUNT] = ds.fail ? (ds.spin_err ? kSpinFlag : 1.0) : 0.0;
    for (int k = R_MODEL; k <= R_COUNT; ++k) b.scal[k] = scal[k];
    if (do_decide) {
      decide_t(ds, scal, o);
      ds.store(st);
    }
#ifdef ME_STEP_TS
    atomicAdd(&g_step_ts[10], (unsigned long long)((long long)__builtin_amdgcn_s_memtime() - f0));
#endif
  }
}

// (64-thread workgroups measured slower: 17.2 -> 21.6 us at config 3, the
// last arrival then reduces 4x the partials)
// (Measured and dropped, round 4 as in rounds 2-3: the step linearising
// speculatively at its candidate into a second obsx / Wo set, removing the
// linearize launch of every accepted step -- the step went 15.1 -> 28.7 us
// for 9.3 us saved; config 3 BA 0.821 -> 0.894 ms per 10 iterations.)
constexpr int kStepG = 16, kStepBlock = 256, kStepPts = kStepBlock / kStepG;

// Model cost change in the normal-equation form (Ceres computes
// -(J dx).(r + J dx / 2) per residual block; summed over the blocks that is
// -(g.dx + dx^T J^T J dx / 2) with g = J^T r): per point, in the scaled space,
// -(g_p.y_p + y_p^T V_p y_p / 2 + (D_p y_p).sum_q W_q^T (D_c y_c)) -- the last
// sum is the one the point's back-substitution forms anyway -- and per camera
// -(g_c.y_c + y_c^T U_c y_c / 2) (cam_solve).  The same quantity as the
// per-observation form (rounding aside), without the per-observation Jacobian
// traffic (320 B / observation written by linearize and read here before).

// Candidate camera parameter: x + D_c y_c (ys = csc * yc), never contracted
// into an FMA, so the camera workgroup's stored candidate and the point
// workgroups' own copies agree bit for bit.
__device__ __forceinline__ double cam_cand(double x, double ys) {
#pragma clang fp contract(off)
  return x + ys;
}

// The camera workgroup of pt_step (the last one): the candidate cameras and the
// camera part of the step's scalars, |dx_c|^2, |x_c|^2 and the model change
// -(g_c.y_c + y_c^T U_c y_c / 2) in the scaled space.  Round 6: this was the
// camera solve's tail, on its one workgroup's serial path (1.7 us per
// iteration at config 3, tools/drivers.py solve_ts); here it runs beside the
// points.  The scalars are written through: this launch's finalizing workgroup
// reads them (DecideState::load).
__device__ void cam_step_body(const Geo& g, const Bufs& b, int cur, double* lds) {
  const int tid = threadIdx.x, nt = blockDim.x;
  const int n = g.n6, ncp = 6 * g.nc, f6 = 6 * g.nf;
  const double* x = b.cams[cur];
  double* xc = b.cams[1 - cur];
  double s2 = 0.0, xn2 = 0.0, cm = 0.0;
  for (int i = tid; i < ncp; i += nt) {
    const double xi = x[i];
    if (i < f6) {  // fixed camera
      xc[i] = xi;
      continue;
    }
    const double v = cam_cand(xi, b.csc[i - f6] * b.yc[i - f6]);
    xc[i] = v;
    const double dd = v - xi;
    s2 += dd * dd;
    xn2 += xi * xi;
  }
  for (int r = tid; r < n; r += nt) {
    const double* U = b.U + 36 * (long)(r / 6) + 6 * (r % 6);
    const double* y = b.yc + (r - r % 6);
    const double yr = b.yc[r];
    double uy = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) uy += U[k] * y[k];
    cm += b.gcs[r] * yr + 0.5 * yr * uy;
  }
  double v3[3] = {s2, xn2, -cm}, out[3];
  block_sum<3>(v3, out, lds);
  if (tid == 0) {
    a_st<true>(&b.st->cam_step2, out[0]);
    a_st<true>(&b.st->cam_xn2, out[1]);
    a_st<true>(&b.st->cam_model, out[2]);
  }
}

// Grid: g.nblk_step point workgroups + the camera workgroup (cam_step_body).
template <int OD>
__global__ __launch_bounds__(kStepBlock) void pt_step_kernel(Geo g, Bufs b, Opts o, int do_decide) {
  __shared__ double lds[16];
  const State* st = b.st;
  // the camera solve's roster, re-armed for the next iteration's solve (every
  // workgroup of the solve launch, late joiners included, has finished)
  if (blockIdx.x == 0 && threadIdx.x < 2) b.roster[threadIdx.x] = 0u;
  if (st->done) return;
#ifdef ME_STEP_TS
  long long step_prev_ = 0, fin_prev_ = 0;
#endif
  if ((int)blockIdx.x == g.nblk_step) {
    // (a failed solve wrote no step; thread 0's scalar stores drain before its
    // arrival, last_arrival_wt)
    if (!st->fail) cam_step_body(g, b, st->cur, lds);
  } else {
  STEP_T(0);
  const int gl = threadIdx.x & (kStepG - 1);
  const int j = blockIdx.x * kStepPts + (threadIdx.x / kStepG);
  double mc = 0, cc = 0, s2 = 0, xn2 = 0;
  if (j < g.np && !st->fail) {  // uniform within a 16-lane group
    // Every load of the point and of this lane's first CSR slot is requested
    // in three dependent rounds (point data + offsets | slot: camera, obs
    // index, W | camera step / scales, observation, candidate camera) before
    // any arithmetic; further slots (points with more than 16 observations)
    // load in the loops.  The slot's camera is p_cam + nf (plan_segsort_kernel
    // writes p_cam[q] = cam_idx[p_obs[q]] - nf), so the candidate camera does
    // not wait for a cam_idx read.
    const int cur = st->cur;
    const double* Wo = b.Wo;
    double psv[3], gpv[3], Lv[9], xv[3], Vv[9];
    for (int a = 0; a < 3; ++a) {
      psv[a] = b.psc[3 * (long)j + a];
      gpv[a] = b.gps[3 * (long)j + a];
      xv[a] = b.pts[cur][3 * (long)j + a];
    }
    for (int i = 0; i < 9; ++i) {
      Lv[i] = b.Lp[9 * (long)j + i];
      Vv[i] = b.V[9 * (long)j + i];
    }
    const int beg = b.p_off[j], end = b.p_off[j + 1];
    const int q0 = beg + gl;
    const bool has0 = q0 < end;
    int ci0 = -1, o0 = 0;
    double W0[18];
    if (has0) {
      ci0 = b.p_cam[q0];
      o0 = b.p_obs[q0];
      for (int i = 0; i < 18; ++i) W0[i] = Wo[18 * (long)q0 + i];  // (unused for a fixed camera)
    }
    // candidate cameras x + D_c y_c formed here from the current ones (the
    // camera workgroup stores the same values, cam_cand; not read back)
    const double* cams_x = b.cams[cur];
    double ys0[6], f0[4];
    int cam0 = 0, right0 = 0;
    if (has0) {
      if (ci0 >= 0)
        for (int a = 0; a < 6; ++a) ys0[a] = b.csc[6 * ci0 + a] * b.yc[6 * ci0 + a];
      cam0 = ci0 + g.nf;
      for (int k = 0; k < OD; ++k) f0[k] = b.obs[(long)OD * o0 + k];
      if (OD == 2) right0 = b.cam_id[o0] != 0;
    }
    double cv0[6];
    if (has0)
      for (int a = 0; a < 6; ++a) {
        const double xa = cams_x[6 * cam0 + a];
        cv0[a] = ci0 >= 0 ? cam_cand(xa, ys0[a]) : xa;
      }
    STEP_T(1);  // (the first round of loads issued; returns at first use below)
    // (1) sum over the point's slots of W_q^T (Dc y_c)
    double t[3] = {0.0, 0.0, 0.0};
    for (int q = q0; q < end; q += kStepG) {
      const bool first = q == q0;
      const int ci = first ? ci0 : b.p_cam[q];
      if (ci < 0) continue;
      double ys[6], W[18];
      if (first) {
        for (int a = 0; a < 6; ++a) ys[a] = ys0[a];
        for (int i = 0; i < 18; ++i) W[i] = W0[i];
      } else {
        for (int a = 0; a < 6; ++a) ys[a] = b.csc[6 * ci + a] * b.yc[6 * ci + a];
        for (int i = 0; i < 18; ++i) W[i] = Wo[18 * (long)q + i];
      }
      for (int c = 0; c < 3; ++c) {
        double s = 0;
        for (int a = 0; a < 6; ++a) s += W[a * 3 + c] * ys[a];
        t[c] += s;
      }
    }
    for (int c = 0; c < 3; ++c) t[c] = group_sum<kStepG>(t[c]);
    STEP_T(2);  // slot sums (loads of the first slot returned)
    // (2) point step y_p = -(V + D/r)^-1 (g_p + sum) in the scaled space, candidate point
    double rhs[3];
    for (int c = 0; c < 3; ++c) rhs[c] = -gpv[c] - t[c] * psv[c];
    double u[3], yp[3];
    fwd3(Lv, rhs, u);
    bwd3(Lv, u, yp);
    double d[3], xc[3];
    for (int a = 0; a < 3; ++a) {
      d[a] = yp[a] * psv[a];
      xc[a] = fmin(fmax(xv[a] + d[a], g.lo[a]), g.hi[a]);
    }
    if (gl == 0) {
      double gy = 0.0, yvy = 0.0, cross = 0.0;
      for (int a = 0; a < 3; ++a) {
        b.dp[3 * (long)j + a] = d[a];
        b.pts[1 - cur][3 * (long)j + a] = xc[a];
        const double dd = xc[a] - xv[a];
        s2 += dd * dd;
        xn2 += xv[a] * xv[a];
        gy += gpv[a] * yp[a];
        cross += d[a] * t[a];
        double vy = 0.0;
        for (int c = 0; c < 3; ++c) vy += Vv[3 * a + c] * yp[c];
        yvy += yp[a] * vy;
      }
      mc = -(gy + 0.5 * yvy + cross);
    }
    STEP_T(3);  // point solve, candidate point
    // (3) candidate cost of the point's observations
    for (int q = q0; q < end; q += kStepG) {
      const bool first = q == q0;
      double cv[6], f[4];
      int right = 0;
      if (first) {
        for (int a = 0; a < 6; ++a) cv[a] = cv0[a];
        for (int k = 0; k < OD; ++k) f[k] = f0[k];
        right = right0;
      } else {
        const int o = b.p_obs[q];
        const int ci = b.p_cam[q], cam = ci + g.nf;
        for (int a = 0; a < 6; ++a) {
          const double xa = cams_x[6 * cam + a];
          cv[a] = ci >= 0 ? cam_cand(xa, b.csc[6 * ci + a] * b.yc[6 * ci + a]) : xa;
        }
        for (int k = 0; k < OD; ++k) f[k] = b.obs[(long)OD * o + k];
        if (OD == 2) right = b.cam_id[o] != 0;
      }
      double r[4];
      if (OD == 4)
        stereo_residual(g, cv, xc, f, r, nullptr, nullptr);
      else
        mono_residual(g, cv, xc, f, right, r, nullptr, nullptr);
      const double s = r[0] * r[0] + r[1] * r[1] + r[2] * r[2] + r[3] * r[3];
      double rho0, sc;
      huber(s, &rho0, &sc);
      cc += 0.5 * rho0;
    }
  }
  STEP_T(4);  // candidate costs
  double v4[4] = {mc, cc, s2, xn2}, out[4];
  block_sum<4>(v4, out, lds);
  if (threadIdx.x == 0) {
    a_st<true>(&b.part[R_MODEL * g.pstride + blockIdx.x], out[0]);
    a_st<true>(&b.part[R_CAND * g.pstride + blockIdx.x], out[1]);
    a_st<true>(&b.part[R_STEP2 * g.pstride + blockIdx.x], out[2]);
    a_st<true>(&b.part[R_XN2 * g.pstride + blockIdx.x], out[3]);
  }
  STEP_T(5);  // block sum + partial stores
  }  // (point workgroups)
  // the last workgroup to finish (of either kind) reduces the partials
  // (step_finalize) and, single-GPU, runs the Ceres step handling
  if (!last_arrival_wt(b.cnt + g.m, gridDim.x)) return;
#ifdef ME_STEP_TS
  if (threadIdx.x == 0) fin_prev_ = (long long)__builtin_amdgcn_s_memtime();
#endif
  step_finalize_body(g, b, o, do_decide);
  STEP_FIN_T(6);  // the finalizing workgroup: partial reduce + decide
#ifdef ME_STEP_TS
  if (threadIdx.x == 0) atomicAdd(&g_step_ts[7], 1ull);
#endif
}

__global__ void decide_kernel(Geo g, Bufs b, Opts o) {
  if (threadIdx.x != 0) return;
  if (b.st->done) return;
  decide(b, o);
}

template <int OD>
__global__ __launch_bounds__(kBlock) void cost_kernel(Geo g, Bufs b, int which, double* part) {
  __shared__ double lds[4];
  const int o = blockIdx.x * kBlock + threadIdx.x;
  double c = 0;
  if (o < g.no) {
    double r[4];
    obs_residual<OD>(g, b, o, b.cams[which] + 6 * b.cam_idx[o], b.pts[which] + 3 * b.pt_idx[o], r, nullptr, nullptr);
    const double s = r[0] * r[0] + r[1] * r[1] + r[2] * r[2] + r[3] * r[3];
    double rho0, sc;
    huber(s, &rho0, &sc);
    c = 0.5 * rho0;
  }
  double v[1] = {c}, out[1];
  block_sum<1>(v, out, lds);
  if (threadIdx.x == 0) part[blockIdx.x] = out[0];
}

template <int OD>
__global__ __launch_bounds__(kBlock) void eval_kernel(Geo g, Bufs b, double* res, double* Jc, double* Jp) {
  const int o = blockIdx.x * kBlock + threadIdx.x;
  if (o >= g.no) return;
  double r[4], jc[24], jp[12];
  obs_residual<OD>(g, b, o, b.cams[0] + 6 * b.cam_idx[o], b.pts[0] + 3 * b.pt_idx[o], r, jc, jp);
  constexpr int od = OD;  // output rows per observation: Observation<M>::data size
  for (int k = 0; k < od; ++k) res[od * (long)o + k] = r[k];
  if (Jc)
    for (int k = 0; k < 6 * od; ++k) Jc[6 * od * (long)o + k] = jc[k];
  if (Jp)
    for (int k = 0; k < 3 * od; ++k) Jp[3 * od * (long)o + k] = jp[k];
}

// Pose covariance (BundleAdjuster<M>::extract_covariance, BundleAdjuster.h:478-528):
// the camera blocks of (J^T J)^-1 are the blocks of S^-1, S the undamped,
// unscaled point-eliminated camera system.  One workgroup: in-place dense
// Cholesky of S (global memory, the matrix is at most 300 x 300), X = L^-1 one
// column per thread, then cov_i = (X^T X) over camera i's six columns.  Not on
// the frame path (compute_cov is off by default, BundleAdjuster.h:41-42).
constexpr int kCovBlock = 1024;
__global__ __launch_bounds__(kCovBlock) void cov_kernel(Geo g, Bufs b, double* X, double* cov, int* ok_out) {
  __shared__ int sfail;
  const int n = g.n6, tid = threadIdx.x;
  double* A = b.S;  // row-major n x n, symmetric
  if (tid == 0) sfail = b.st->fail || b.st->bad_input;
  __syncthreads();
  for (int j = 0; j < n && !sfail; ++j) {
    if (tid == 0) {
      const double d = A[(long)j * n + j];
      if (!(d > 0.0)) sfail = 1;
      else A[(long)j * n + j] = sqrt(d);
    }
    __syncthreads();
    if (sfail) break;
    const double djj = A[(long)j * n + j];
    for (int i = j + 1 + tid; i < n; i += kCovBlock) A[(long)i * n + j] /= djj;
    __syncthreads();
    const int m = n - j - 1;  // trailing lower triangle, m(m+1)/2 entries
    for (long e = tid; e < (long)m * (m + 1) / 2; e += kCovBlock) {
      int i = (int)((sqrt(8.0 * e + 1.0) - 1.0) / 2.0);
      while ((long)i * (i + 1) / 2 > e) --i;
      while ((long)(i + 1) * (i + 2) / 2 <= e) ++i;
      const int k = (int)(e - (long)i * (i + 1) / 2);
      const int ii = j + 1 + i, kk = j + 1 + k;
      A[(long)ii * n + kk] -= A[(long)ii * n + j] * A[(long)kk * n + j];
    }
    __syncthreads();
  }
  if (sfail) {
    if (tid == 0) *ok_out = 0;
    return;
  }
  // X = L^-1, column c by forward substitution (X column-major: X[c * n + k] = (L^-1)[k][c])
  for (int c = tid; c < n; c += kCovBlock) {
    double* x = X + (long)c * n;
    for (int k = 0; k < c; ++k) x[k] = 0.0;
    for (int k = c; k < n; ++k) {
      double acc = k == c ? 1.0 : 0.0;
      for (int l = c; l < k; ++l) acc -= A[(long)k * n + l] * x[l];
      x[k] = acc / A[(long)k * n + k];
    }
  }
  __syncthreads();
  for (int e = tid; e < 36 * g.nc; e += kCovBlock) {
    const int ci = e / 36, a = (e % 36) / 6, c = e % 6;
    double v = 0.0;
    if (ci >= g.nf) {  // constant cameras: zero block (ceres::Covariance)
      const int p = 6 * (ci - g.nf) + a, q = 6 * (ci - g.nf) + c;
      const double *xp = X + (long)p * n, *xq = X + (long)q * n;
      for (int k = max(p, q); k < n; ++k) v += xp[k] * xq[k];
    }
    cov[e] = v;
  }
  if (tid == 0) *ok_out = 1;
}

// Ceres covariance ignores the point bounds: an infeasible point does not stop it.
__global__ void cov_prep_kernel(Bufs b) {
  if (!b.st->bad_input) b.st->done = 0;
}

// ---------------------------------------------------------------- device plan
// The observation layout is built on the device from the raw inputs, so a
// problem already resident in HBM (me_ba_problem.mem == ME_DEVICE) never
// crosses PCIe and no host sort sits on the frame's critical path.
//   plan_count   per obs: point histogram (atomics), per-(block, camera)
//                counts (LDS), index validation; per point: box feasibility;
//                copies the starting parameters into the solver buffers.
//   plan_scan    one workgroup: CSR offsets by point, per-camera block offsets,
//                State initialisation.
//   plan_scatter per obs: point slot (atomic), camera slot = block offset +
//                stable rank inside the block (original order kept).
//   plan_segsort per point: its slots sorted by (camera, obs index), exactly
//                the host stable_sort by camera; pos / p_cam / dup.
enum { F_BAD = 0, F_INFEASIBLE = 1 };
struct PlanWork {
  int* cnt_p;
  int* fill_p;
  int* blk_cam;
  int* flags;
};
__device__ __forceinline__ PlanWork plan_work(const Geo& g, int* w) {
  PlanWork pw;
  pw.cnt_p = w;
  pw.fill_p = w + g.np;
  pw.blk_cam = w + 2 * (long)g.np;
  pw.flags = pw.blk_cam + (long)g.nblk_obs * g.nc;
  return pw;
}

__global__ __launch_bounds__(kBlock) void plan_count_kernel(Geo g, Bufs b, const double* cams_in,
                                                            const double* pts_in) {
  extern __shared__ int lcnt[];  // nc
  const PlanWork w = plan_work(g, b.work);
  const int t = threadIdx.x, blk = blockIdx.x;
  const long gid = (long)blk * kBlock + t;
  for (int c = t; c < g.nc; c += kBlock) lcnt[c] = 0;
  __syncthreads();
  if (blk < g.nblk_obs && gid < g.no) {
    const int ci = b.cam_idx[gid], pi = b.pt_idx[gid];
    if (ci < 0 || ci >= g.nc || pi < 0 || pi >= g.np) {
      atomicOr(&w.flags[F_BAD], 1);
    } else {
      atomicAdd(&w.cnt_p[pi], 1);
      atomicAdd(&lcnt[ci], 1);
    }
  }
  if (gid < g.np) {
    for (int a = 0; a < 3; ++a) {
      const double x = pts_in[3 * gid + a];
      if (!(x >= g.lo[a] && x <= g.hi[a])) atomicOr(&w.flags[F_INFEASIBLE], 1);
    }
  }
  if (cams_in != b.cams[0] && gid < 6 * (long)g.nc) b.cams[0][gid] = cams_in[gid];
  if (pts_in != b.pts[0] && gid < 3 * (long)g.np) b.pts[0][gid] = pts_in[gid];
  __syncthreads();
  if (blk < g.nblk_obs)
    for (int c = t; c < g.nc; c += kBlock) w.blk_cam[(long)blk * g.nc + c] = lcnt[c];
}

constexpr int kScanBlock = 1024;
constexpr int kMaxScanCams = 4096;
__global__ __launch_bounds__(kScanBlock) void plan_scan_kernel(Geo g, Bufs b, Opts o) {
  __shared__ int wsum[kScanBlock / 64];
  __shared__ int total;
  const PlanWork w = plan_work(g, b.work);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  // exclusive scan of the point counts: contiguous chunk per thread
  const int chunk = (g.np + kScanBlock - 1) / kScanBlock;
  const int beg = min(g.np, t * chunk), end = min(g.np, beg + chunk);
  int s = 0;
  for (int j = beg; j < end; ++j) s += w.cnt_p[j];
  int x = s;  // inclusive wave scan
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  if (t == 0) {
    int acc = 0;
    for (int k = 0; k < kScanBlock / 64; ++k) {
      const int v = wsum[k];
      wsum[k] = acc;
      acc += v;
    }
    total = acc;
  }
  __syncthreads();
  int run = wsum[wv] + x - s;
  for (int j = beg; j < end; ++j) {
    b.p_off[j] = run;
    run += w.cnt_p[j];
  }
  if (t == 0) b.p_off[g.np] = total;
  // per-camera offsets of every observation block (variable cameras only):
  // one wave per camera scans its column of block counts, then the camera
  // totals are scanned and added
  __shared__ int ctot[kMaxScanCams];
  const int bchunk = (g.nblk_obs + 63) / 64;
  for (int c = wv; c < g.m; c += kScanBlock / 64) {
    const int k0 = min(g.nblk_obs, lane * bchunk), k1 = min(g.nblk_obs, k0 + bchunk);
    int cs = 0;
    for (int k = k0; k < k1; ++k) cs += w.blk_cam[(long)k * g.nc + g.nf + c];
    int cx = cs;
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(cx, off, 64);
      if (lane >= off) cx += y;
    }
    int r = cx - cs;
    for (int k = k0; k < k1; ++k) {
      int* e = &w.blk_cam[(long)k * g.nc + g.nf + c];
      const int v = *e;
      *e = r;
      r += v;
    }
    if (lane == 63) ctot[c] = cx;
  }
  __syncthreads();
  if (t == 0) {
    int acc = 0;
    for (int c = 0; c < g.m; ++c) {
      b.c_off[c] = acc;
      const int v = ctot[c];
      ctot[c] = acc;
      acc += v;
    }
    b.c_off[g.m] = acc;
  }
  __syncthreads();
  for (int c = wv; c < g.m; c += kScanBlock / 64) {
    const int k0 = min(g.nblk_obs, lane * bchunk), k1 = min(g.nblk_obs, k0 + bchunk);
    for (int k = k0; k < k1; ++k) w.blk_cam[(long)k * g.nc + g.nf + c] += ctot[c];
  }
  for (int i = t; i < g.n6; i += kScanBlock) b.csc[i] = 0.0;
  if (t == 0) {
    State* st = b.st;
    st->cur = 0;
    st->need_lin = 1;
    st->done = 0;
    st->termination = 1;
    st->iterations = st->successful = st->invalid_count = 0;
    st->fail = st->scaled = st->accepted = st->final_pass = st->spin_err = 0;
    st->bad_input = w.flags[F_BAD];
    st->infeasible = w.flags[F_INFEASIBLE];
    st->radius = o.initial_radius;
    st->decrease = 2.0;
    st->x_cost = st->cand_cost = st->model_change = st->initial_cost = 0.0;
    st->cam_step2 = st->cam_xn2 = st->cam_model = st->last_q = 0.0;
    for (int k = 0; k < 16; ++k) st->stamps[k] = 0;
    if (st->bad_input || st->infeasible) {
      st->done = 1;
      st->termination = 2;
    }
  }
}

__global__ __launch_bounds__(kBlock) void plan_scatter_kernel(Geo g, Bufs b) {
  __shared__ int scam[kBlock];
  const PlanWork w = plan_work(g, b.work);
  if (w.flags[F_BAD]) return;
  const int t = threadIdx.x, blk = blockIdx.x;
  const int o = blk * kBlock + t;
  const int ci = o < g.no ? b.cam_idx[o] : -1;
  scam[t] = ci;
  if (o < g.no) {
    const int pi = b.pt_idx[o];
    b.tmp_obs[b.p_off[pi] + atomicAdd(&w.fill_p[pi], 1)] = o;
  }
  __syncthreads();
  if (o < g.no) {
    int slot = -1;
    if (ci >= g.nf) {
      int rank = 0;
      for (int k = 0; k < t; ++k) rank += scam[k] == ci;
      slot = w.blk_cam[(long)blk * g.nc + ci] + rank;
      b.c_obs[slot] = o;
    }
    b.cpos[o] = slot;
  }
}

// One wave per point: rank of each slot by (camera, observation index) --
// the order of the host stable_sort by camera -- then p_obs / pos / p_cam /
// dup.  Segments of <= 64 observations rank with shuffles; longer ones with a
// loop over the (cached) segment.
constexpr int kSortBlock = 256;
__global__ __launch_bounds__(kSortBlock) void plan_segsort_kernel(Geo g, Bufs b) {
  const PlanWork w = plan_work(g, b.work);
  if (w.flags[F_BAD]) return;
  const int lane = threadIdx.x & 63;
  const int j = blockIdx.x * (kSortBlock / 64) + (threadIdx.x >> 6);
  if (j >= g.np) return;
  const int beg = b.p_off[j], k = b.p_off[j + 1] - beg;
  auto key_of = [&](int o) { return ((unsigned long long)(unsigned)b.cam_idx[o] << 32) | (unsigned)o; };
  if (k <= 64) {
    const int o = lane < k ? b.tmp_obs[beg + lane] : 0;
    const unsigned long long key = lane < k ? key_of(o) : ~0ull;
    int rank = 0, same = 0;
    for (int l = 0; l < k; ++l) {
      const unsigned long long kl = __shfl(key, l, 64);
      rank += kl < key;
      same += (kl >> 32) == (key >> 32);
    }
    if (lane < k) {
      const int q = beg + rank;
      b.p_obs[q] = o;
      b.pos[o] = q;
      b.p_cam[q] = (int)(key >> 32) - g.nf;
      b.dup[o] = same > 1 ? 1 : 0;
    }
    return;
  }
  for (int e = lane; e < k; e += 64) {
    const int o = b.tmp_obs[beg + e];
    const unsigned long long key = key_of(o);
    int rank = 0, same = 0;
    for (int l = 0; l < k; ++l) {
      const unsigned long long kl = key_of(b.tmp_obs[beg + l]);
      rank += kl < key;
      same += (kl >> 32) == (key >> 32);
    }
    const int q = beg + rank;
    b.p_obs[q] = o;
    b.pos[o] = q;
    b.p_cam[q] = (int)(key >> 32) - g.nf;
    b.dup[o] = same > 1 ? 1 : 0;
  }
}

// Band order of the landmarks for the Schur runs (pt_schur_kernel): key =
// first tile * T + last tile of the landmark's variable-camera columns
// (slots are sorted by camera: the first variable slot and the last slot), a
// landmark without variable cameras in the last bucket.  Stable counting
// sort: per 256-landmark block, the rank of each key among the block's
// earlier landmarks (within a wave by ballots over its distinct keys, plus the
// counts of the earlier waves) and the block's key counts (bucket-major),
// then plan_order_kernel scans the counts and scatters.  Only for windows
// with many tile pairs (g.sorted); otherwise the runs keep the landmark order
// and every run takes the whole tile set.
constexpr int kMaxBandKeys = 19 * 19;  // T <= 19 (npairs <= 192)
__global__ __launch_bounds__(kBlock) void plan_band_kernel(Geo g, Bufs b) {
  __shared__ int wcnt[kBlock / 64][kMaxBandKeys];
  const PlanWork w = plan_work(g, b.work);
  const int t = threadIdx.x, blk = blockIdx.x, j = blk * kBlock + t, lane = t & 63, wv = t >> 6;
  const int K = g.T * g.T;
  for (int k = t; k < (kBlock / 64) * K; k += kBlock) wcnt[k / K][k % K] = 0;
  int key = -1;
  if (j < g.np) {
    key = K - 1;
    const int beg = b.p_off[j], end = b.p_off[j + 1];
    const int hi = (!w.flags[F_BAD] && end > beg) ? b.p_cam[end - 1] : -1;
    if (hi >= 0) {
      int q = beg;
      while (b.p_cam[q] < 0) ++q;  // fixed cameras (negative) sort first
      key = (6 * b.p_cam[q] / 16) * g.T + (6 * hi + 5) / 16;
    }
  }
  __syncthreads();
  // rank among the wave's lower lanes with the same key: one ballot per distinct key
  int rank = 0;
  unsigned long long todo = __ballot(key >= 0);
  while (todo) {
    const int lead = __builtin_ctzll(todo);
    const int kl = __shfl(key, lead, 64);
    const unsigned long long m = __ballot(key == kl);
    if (key == kl) rank = __builtin_popcountll(m & ((1ull << lane) - 1ull));
    if (lane == lead) wcnt[wv][kl] = __builtin_popcountll(m);
    todo &= ~m;
  }
  __syncthreads();
  if (j < g.np) {
    for (int v = 0; v < wv; ++v) rank += wcnt[v][key];
    b.pkey[j] = key;
    b.prank[j] = rank;
  }
  for (int k = t; k < K; k += kBlock) {
    int c = 0;
#pragma unroll
    for (int v = 0; v < kBlock / 64; ++v) c += wcnt[v][k];
    b.phist[(long)k * g.nblkp + blk] = c;
  }
}

// One workgroup: exclusive scan of the block key counts -> band order, and
// with the scatter each run's band (first tile of its first landmark, largest
// last tile: LDS max); then per tile pair the partial slots of the runs whose
// tile set holds it, in run order.
constexpr int kMaxRuns = 1024;
__global__ __launch_bounds__(kScanBlock) void plan_order_kernel(Geo g, Bufs b) {
  __shared__ int wsum[kScanBlock / 64];
  __shared__ int rA[kMaxRuns], rB[kMaxRuns];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  for (int r = t; r < g.nruns; r += kScanBlock) {
    rA[r] = g.T - 1;  // (a run past the last landmark: the z tile alone)
    rB[r] = 0;
  }
  const long nh = (long)g.T * g.T * g.nblkp;
  const long chunk = (nh + kScanBlock - 1) / kScanBlock;
  const long beg = min(nh, t * chunk), end = min(nh, beg + chunk);
  int s = 0;
  for (long i = beg; i < end; ++i) s += b.phist[i];
  int x = s;  // inclusive wave scan
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  if (t == 0) {
    int acc = 0;
    for (int k = 0; k < kScanBlock / 64; ++k) {
      const int v = wsum[k];
      wsum[k] = acc;
      acc += v;
    }
  }
  __syncthreads();
  int run = wsum[wv] + x - s;
  for (long i = beg; i < end; ++i) {
    const int v = b.phist[i];
    b.phist[i] = run;
    run += v;
  }
  __syncthreads();
  for (int j = t; j < g.np; j += kScanBlock) {
    const int key = b.pkey[j];
    const int pos = b.phist[(long)key * g.nblkp + j / kBlock] + b.prank[j];
    b.order[pos] = j;
    const int r = pos / g.rlen;
    if (pos == r * g.rlen) rA[r] = key / g.T;  // keys ascend: the run's first landmark has its smallest first tile
    atomicMax(&rB[r], key % g.T);
  }
  __syncthreads();
  for (int r = t; r < g.nruns; r += kScanBlock) {
    const int B = max(rA[r], rB[r]);
    rB[r] = B;
    b.rband[2 * r] = rA[r];
    b.rband[2 * r + 1] = B;
  }
  __syncthreads();
  for (int p = t; p < g.npairs; p += kScanBlock) {
    int I = 0, rem = p;
    while (rem >= g.T - I) {
      rem -= g.T - I;
      ++I;
    }
    const int J = I + rem;
    int cnt = 0;
    for (int r = 0; r < g.nruns; ++r) {
      const int A = rA[r], B = rB[r];
      const int nb = B - A + 1, ns = nb + (B < g.T - 1 ? 1 : 0);
      const int ka = (I >= A && I <= B) ? I - A : (I == g.T - 1 ? nb : -1);
      const int kb = (J >= A && J <= B) ? J - A : (J == g.T - 1 ? nb : -1);
      if (ka < 0 || kb < 0) continue;
      b.tl[(long)p * g.nruns + cnt++] = r * g.npairs + ka * ns - ka * (ka - 1) / 2 + (kb - ka);
    }
    b.tcnt[p] = cnt;
    for (int q = cnt; q < g.nruns; ++q) b.tl[(long)p * g.nruns + q] = -1;  // (the assembly reads whole lists)
  }
}

// State | cams[cur] | pts[cur] -> one contiguous read-back (or straight into
// the caller's device arrays for a device-resident problem)
__global__ __launch_bounds__(kBlock) void output_kernel(Geo g, Bufs b, double* cams_dst, double* pts_dst) {
  const int cur = b.st->cur;
  const long gid = (long)blockIdx.x * kBlock + threadIdx.x;
  constexpr int kStateWords = (int)(sizeof(State) / 8);
  if (gid < kStateWords) b.out[gid] = ((const double*)b.st)[gid];
  if (gid < 6 * (long)g.nc) cams_dst[gid] = b.cams[cur][gid];
  if (gid < 3 * (long)g.np) pts_dst[gid] = b.pts[cur][gid];
}

// ---------------------------------------------------------------- host plan
struct Plan {
  me_ctx* c = nullptr;
  Geo g;
  unsigned asm_gen = 0;  // fused-assembly launches since the plan cleared the claim words
  Bufs b;
  Opts o;
  double* colnorm = nullptr;
  double* gc_raw = nullptr;
  double* Uraw = nullptr;
  double* cpart = nullptr;  // camera assembly partials (m x ck x 27)
  double* host = nullptr;  // pinned staging (inputs in, State / results out)
  State* hstate[2] = {nullptr, nullptr};  // pinned slots of the pipelined State polls
  bool dev = false;        // problem arrays are device-resident
  bool copy_out = false;   // device-resident problem: the solved cams / pts also staged to the host (me_ba_wait_out)
  bool reserve_only = false;  // me_ba_reserve: size the scratch and staging, queue nothing
  size_t solve_lds = 0;
  size_t schur_lds = 0;
  int use_lds = 0;
  int diag_skip = 0;  // ME_SOLVE_SKIP: timing diagnostics only (results invalid)
  int n_enq = 0;      // linearisations queued so far (the first runs the camera assembly on its own)
  bool sequential = false;  // ME_BA_SEQUENTIAL=1: never fuse (A/B timing)
  bool no_fused_asm = false;  // ME_BA_NOFUSEASM=1: S assembly in its own launch (A/B timing)
  bool full_S = false;      // assemble both block triangles of S (reduced-system / covariance read-back)
  int solve_workers = -1;   // global-memory camera solve: trailing-update workgroups (-1: by size; ME_SOLVE_WORKERS)
  int solve_cap = 0;        // co-resident cam_solve_kernel<2> workgroups on the ctx's CUs (0: not queried)
  int warned_workers = 0;   // an explicit worker count was clamped (reported once per plan)
  me_comm* comm = nullptr;  // sharded solve: the exchange (null: one GPU)
  bool xmax_separate = false;  // ABI-v2 callback (no rank): the gradient max-norm travels in its own max all-reduce
};

inline long rup(long x, long m) { return (x + m - 1) / m * m; }
int blocks(long n, int bs) { return (int)std::max(1L, (n + bs - 1) / bs); }

int ba_drain(me_ctx* c);

// async >= 0: the plan of a queued asynchronous solve, built in scratch and
// staging set `async` (0 or 1) while the other set may still be in flight;
// every other plan first completes the queued solves (they own the scratch)
int plan_build(me_ctx* c, const me_ba_problem* p, const me_ba_options* opt, Plan& P, int slot_base,
               int async = -1, me_comm* comm = nullptr) {
  if (async < 0) ME_TRY(ba_drain(c));
  ME_CHECK(c, p->n_cams > 0 && p->n_pts >= 0 && p->n_obs >= 0, "BA: bad sizes");
  ME_CHECK(c, p->n_cams <= kMaxScanCams, "BA: at most %d cameras per window", kMaxScanCams);
  ME_CHECK(c, p->obs_dim == 0 || p->obs_dim == 2 || p->obs_dim == 4, "BA: obs_dim must be 2 or 4 (Observation<M>)");
  const bool mono = p->obs_dim == 2;
  ME_CHECK(c, p->feat_var > 0 && (mono || p->baseline != 0.0), "BA: wrong calibration parameters (BundleAdjuster.h:147)");
  ME_CHECK(c, !mono || p->cam_id || p->n_obs == 0, "BA: obs_dim 2 needs cam_id (Observation::camID)");
  // BundleAdjuster<2>::optimise: a zero baseline is replaced by 0.5 (BundleAdjuster.h:389-390)
  const double baseline = mono && p->baseline == 0 ? 0.5 : p->baseline;
  ME_CHECK(c, p->mem == ME_HOST || p->mem == ME_DEVICE, "BA: bad memory kind");
  if (p->mem == ME_HOST) {  // device-resident input is validated on the device (State::bad_input)
    for (int i = 0; i < p->n_obs; ++i) {
      ME_CHECK(c, p->cam_idx[i] >= 0 && p->cam_idx[i] < p->n_cams && p->pt_idx[i] >= 0 && p->pt_idx[i] < p->n_pts,
               "BA: observation %d indexes outside the window", i);
    }
  }
  P.c = c;
  if (const char* sk = getenv("ME_SOLVE_SKIP")) P.diag_skip = atoi(sk);
  int dbg = c->dbg_solve_flags;
  if (dbg & 2048) {  // (test hook: every second solve on this ctx has every camera solve fail)
    if (c->dbg_solve_count++ & 1) dbg |= 1024;
    dbg &= ~2048;
  }
  P.diag_skip |= dbg;
  if (const char* sw = getenv("ME_SOLVE_WORKERS")) P.solve_workers = atoi(sw);  // A/B timing (0: one workgroup)
  if (const char* sq = getenv("ME_BA_SEQUENTIAL")) P.sequential = atoi(sq) != 0;
  if (const char* fa = getenv("ME_BA_NOFUSEASM")) P.no_fused_asm = atoi(fa) != 0;
  Geo& g = P.g;
  g.nc = p->n_cams;
  g.np = p->n_pts;
  g.no = p->n_obs;
  g.nf = std::min(std::max(p->fixed_frames, 0), p->n_cams);
  g.od = mono ? 2 : 4;
  // sharded: one gradient max-norm slot per rank (ABI-v2 callback without rank: one slot, max-reduced apart)
  P.comm = comm;
  P.xmax_separate = comm && comm->world == 0;
  g.xslots = comm && comm->world > 0 ? comm->world : 1;
  g.xrank = comm && comm->world > 0 ? comm->rank : 0;
  g.m = g.nc - g.nf;
  g.n6 = 6 * g.m;
  g.Rpad = (int)rup(g.n6 + 1, 16);  // camera columns | z_p column n6 | zero padding
  g.T = g.Rpad / 16;
  g.Ts = (g.n6 + 1 + 15) / 16;
  g.npairs = g.T * (g.T + 1) / 2;
  // wide sub-chunks pay off once the tile count is large (config 4: 66 pairs,
  // -2% BA time); at config 3 (28 pairs) the longer per-workgroup chain costs
  // more than the halved partial traffic saves (1.23 vs 1.19 ms per 10 iterations)
  // landmarks per Schur sub-chunk: 32 while the Y block fits the LDS (half the
  // partial tiles for s_assemble); else 16, or 8 for many tiles (the
  // contraction is MFMA-bound per workgroup: twice the workgroups spread it
  // over more CUs; config 5: BA 5.2 -> 4.96 ms per 10 iterations, config 3
  // slower with 8)
  // (and once 16-landmark sub-chunks outnumber 256 workgroups: the config-3
  // VO window, ~4 400 landmarks, BA_SCHUR 430 -> 340 us per keyframe)
  // Few tiles and landmarks (config 3: 28 pairs, 2 000 landmarks): 32-landmark
  // sub-chunks whose run is split into two tile groups of 2 tiles per wave --
  // the same 48 MFMAs per wave as 16 landmarks x 4 tiles, half the runs, so
  // half the partial tiles written here and summed by the assembly
  // (pt_schur 15.8 -> 14.9 us, cam_solve 31.8 -> 31.4 us per iteration,
  // rocprofv3 A/B); a run's Y block is formed twice (once per group).
  const bool split_wide = g.npairs <= 40 && g.np <= 256 * kSchurPts &&
                          schur_lds_bytes(kSchurPtsWide, g.Rpad) <= kSchurLdsCap;
  if ((g.npairs > 40 || g.np > 256 * kSchurPts || split_wide) && schur_lds_bytes(kSchurPtsWide, g.Rpad) <= kSchurLdsCap)
    g.spts = kSchurPtsWide;
  else
    g.spts = g.npairs > 100 ? kSchurPtsSmall : kSchurPts;
  if (const char* e = getenv("ME_SCHUR_PTS")) {  // A/B timing only
    const int v = atoi(e);
    if (v == kSchurPts || v == kSchurPtsSmall || (v == kSchurPtsWide && schur_lds_bytes(kSchurPtsWide, g.Rpad) <= kSchurLdsCap))
      g.spts = v;
  }
  g.nsub = (int)std::max(1L, ((long)g.np + g.spts - 1) / g.spts);
  // Schur runs: rsub sub-chunks of spts landmarks each (at most ~256 runs), in
  // band order; each run split into tile groups of 8 waves x NT <= 5 tiles
  g.rsub = (int)std::max(1L, ((long)g.nsub + 255) / 256);
  g.rlen = g.spts * g.rsub;
  g.nruns = (int)std::max(1L, ((long)g.np + g.rlen - 1) / g.rlen);
  // (measured, tools/drivers.py ba_wall: 4 tiles per wave at config 4 -- 5 spill -- but 5 for
  // the 50-keyframe window, where fewer tile groups per run recompute fewer Y blocks)
  g.stpw = 8 * std::min((g.npairs + 7) / 8, g.npairs > 100 ? kSchurNtMax : std::min(kSchurNtMax, 4));
  if (split_wide && g.spts == kSchurPtsWide) g.stpw = std::min(g.stpw, 16);
  if (const char* e = getenv("ME_SCHUR_STPW")) {  // A/B timing only: tiles per group (8 x tiles per wave)
    const int v = atoi(e);
    if (v >= 16 && v <= 8 * kSchurNtMax && v % 8 == 0) g.stpw = v;
  }
  g.sgrp = (g.npairs + g.stpw - 1) / g.stpw;
  // Schur workgroups: runs in blocks of 8 (one per XCD) x sgrp tile groups (a
  // run's surplus tile groups and the padding runs exit at once)
  g.ksplit = (g.sgrp > 1 ? (int)rup((long)g.nruns, 8) : g.nruns) * g.sgrp;
  // band order pays once the tile set is large (config 4: 66 pairs, config 5: 190); for
  // config 3 (28 pairs) the two plan launches cost more than the partial traffic saves
  g.sorted = g.npairs > 40 ? 1 : 0;
  if (const char* e = getenv("ME_SCHUR_SORT")) g.sorted = atoi(e) != 0;  // A/B timing only
  ME_CHECK(c, g.nruns <= kMaxRuns, "BA: %d Schur runs exceed %d", g.nruns, kMaxRuns);
  g.nblkp = blocks(std::max(g.np, 1), kBlock);
  ME_CHECK(c, g.npairs <= 8 * 24, "BA: %d variable cameras exceed the Schur tile budget", g.m);
  g.nblk_obs = (int)std::max(1L, rup(std::max(g.no, 1), kBlock) / kBlock);
  g.nblk_lin = (int)std::max(1L, rup(std::max(g.no, 1), lin_block(g.no)) / lin_block(g.no));
  g.nblk_pts = (int)std::max(1L, rup(std::max(g.np, 1), kPtBlock) / kPtBlock);
  g.jacobi = opt->jacobi_scaling ? 1 : 0;
  g.ck = (int)std::min(64L, std::max(1L, rup(std::max(g.no, 1), (long)std::max(g.m, 1) * kBlock) /
                                             ((long)std::max(g.m, 1) * kBlock)));
  g.nblk_step = (int)std::max(1L, rup(std::max(g.np, 1), kStepPts) / kStepPts);
  g.pstride = std::max({g.nblk_obs, g.nblk_lin, g.nblk_pts, g.nblk_step, g.ksplit});
  std::memcpy(g.K0, p->K0, sizeof(g.K0));
  std::memcpy(g.K1, p->K1, sizeof(g.K1));
  g.baseline = baseline;
  g.sinv = 1.0 / std::sqrt(p->feat_var);
  const double Zmax = p->K0[0] * baseline / 0.1;
  const double Zmin = p->K0[0] * baseline / (2 * p->K0[2]);
  g.hi[0] = Zmax / p->K0[0] * p->K0[2];
  g.hi[1] = Zmax / p->K0[4] * p->K0[5];
  g.hi[2] = Zmax;
  g.lo[0] = -Zmax / p->K0[0] * p->K0[2];
  g.lo[1] = -Zmax / p->K0[4] * p->K0[5];
  g.lo[2] = Zmin;
  Opts& o = P.o;
  o.max_num_iterations = opt->max_num_iterations;
  o.function_tolerance = opt->function_tolerance;
  o.gradient_tolerance = opt->gradient_tolerance;
  o.parameter_tolerance = opt->parameter_tolerance;
  o.initial_radius = opt->initial_trust_region_radius;
  o.max_radius = opt->max_trust_region_radius;
  o.min_radius = opt->min_trust_region_radius;
  o.min_diag = opt->min_lm_diagonal;
  o.max_diag = opt->max_lm_diagonal;
  o.min_rel_decrease = opt->min_relative_decrease;
  o.max_invalid = opt->max_num_consecutive_invalid_steps;
  const bool dev = p->mem == ME_DEVICE;
  // one arena; the five inputs first and contiguous (one H2D for host input)
  const long nb = g.pstride;
  Bufs& b = P.b;
  std::vector<std::pair<size_t, void**>> items;
  auto add = [&](size_t bytes, void* dst) { items.push_back({rup((long)std::max<size_t>(bytes, 8), 256), (void**)dst}); };
  add(8 * 6 * (size_t)g.nc, &b.cams[0]);
  add(8 * 3 * (size_t)g.np, &b.pts[0]);
  add(8 * g.od * (size_t)g.no, &b.obs);
  add(4 * (size_t)g.no, &b.cam_idx);
  add(4 * (size_t)g.no, &b.pt_idx);
  add(mono ? 4 * (size_t)g.no : 0, &b.cam_id);
  const size_t n_inputs = items.size();
  add(8 * 6 * (size_t)g.nc, &b.cams[1]);
  add(8 * 3 * (size_t)g.np, &b.pts[1]);
  add(4 * (size_t)(g.np + 1), &b.p_off);
  add(4 * (size_t)g.no, &b.p_obs);
  add(4 * (size_t)g.no, &b.pos);
  add(4 * (size_t)g.no, &b.p_cam);
  add(4 * (size_t)(g.m + 1), &b.c_off);
  add(4 * (size_t)g.no, &b.c_obs);
  add(4 * (size_t)g.no, &b.tmp_obs);
  add(4 * (size_t)g.no, &b.cpos);
  add(8 * kObsxStride * (size_t)g.no, &b.obsx);
  add((size_t)g.no, &b.dup);
  add(8 * solve_a_doubles(g.Ts), &b.Abuf);
  add(8 * 18 * (size_t)g.no, &b.Wo);
  add(8 * (size_t)g.n6, &b.csc);
  add(8 * 3 * (size_t)g.np, &b.psc);
  add(8 * 36 * (size_t)g.m, &b.U);
  add(8 * (size_t)g.n6, &b.gcs);
  add(8 * 9 * (size_t)g.np, &b.V);
  add(8 * 3 * (size_t)g.np, &b.gps);
  add(8 * 9 * (size_t)g.np, &b.Lp);
  add(8 * 3 * (size_t)g.np, &b.zp);
  add(8 * 256 * (size_t)g.nruns * g.npairs, &b.Spart);
  add(4 * (size_t)std::max(g.np, 1), &b.order);
  add(4 * (size_t)std::max(g.np, 1), &b.pkey);
  add(4 * (size_t)std::max(g.np, 1), &b.prank);
  add(4 * (size_t)g.T * g.T * g.nblkp, &b.phist);
  add(8 * (size_t)g.nruns, &b.rband);
  add(4 * (size_t)g.npairs * g.nruns, &b.tl);
  add(4 * (size_t)g.npairs, &b.tcnt);
  add(8 * (size_t)g.n6 * g.n6 + 8 * (size_t)(2 * g.n6 + 2), &b.S);  // S | b | diagU | fail (contiguous for all-reduce)
  add(8 * (size_t)g.n6, &b.yc);
  add(8 * 3 * (size_t)g.np, &b.dp);
  add(8 * R_COUNT * (size_t)nb, &b.part);
  add(8 * (R_COUNT + 2), &b.scal);
  add(sizeof(State), &b.st);
  add(8 * (size_t)(g.n6 + 2), &P.colnorm);  // (+ the sharded first exchange's input flags)
  add(8 * (size_t)g.n6, &P.gc_raw);
  add(8 * 21 * (size_t)std::max(g.m, 1), &P.Uraw);
  add(8 * 27 * (size_t)std::max(g.m, 1) * g.ck, &P.cpart);
  add(4 * (size_t)(g.m + 1 + 3 + 2), &b.cnt);  // counters: per camera (cam_assemble) | pt_step | solve sync (2) | fused assembly | roster (2)
  add(4 * (size_t)blocks((long)g.npairs * 256, kSolveBlock / kSaGroups), &b.asm_claim);  // (cleared with cnt)
  const size_t work_bytes = 4 * (2 * (size_t)g.np + (size_t)g.nblk_obs * g.nc + 4);
  add(work_bytes, &b.work);
  const size_t out_doubles = sizeof(State) / 8 + 6 * (size_t)g.nc + 3 * (size_t)g.np;
  add(8 * out_doubles, &b.out);
  b.xch = nullptr;
  if (comm) add(8 * (size_t)xo_total(g), &b.xch);
  size_t total = 0, input_span = 0;
  for (size_t k = 0; k < items.size(); ++k) {
    total += items[k].first;
    if (k < n_inputs) input_span += items[k].first;
  }
  void* arena;
  ME_TRY(me_scratch(c, SLOT_COUNT + slot_base, total, &arena));
  char* ptr = (char*)arena;
  for (auto& it : items) {
    *it.second = ptr;
    ptr += it.first;
  }
  b.ssync = b.cnt + g.m + 1;
  b.roster = b.cnt + g.m + 4;
  b.bvec = b.S + (size_t)g.n6 * g.n6;
  b.diagU = b.bvec + g.n6;
  void* hp;
  const size_t stage = rup((long)std::max(8 * out_doubles, dev ? (size_t)0 : input_span), 64);
  const size_t hbytes = stage + 2 * rup(sizeof(State), 64);
  if (async >= 0) {  // staging owned by the asynchronous solve (set `async` is free: its last solve was waited)
    if (c->ba_pinned_size[async] < hbytes) {
      if (c->ba_pinned[async]) ME_HIP(c, hipHostFree(c->ba_pinned[async]));
      c->ba_pinned[async] = nullptr;
      c->ba_pinned_size[async] = 0;
      ME_HIP(c, hipHostMalloc(&c->ba_pinned[async], std::max(hbytes, (size_t)4096), hipHostMallocDefault));
      c->ba_pinned_size[async] = std::max(hbytes, (size_t)4096);
    }
    hp = c->ba_pinned[async];
  } else {
    ME_TRY(me_pinned(c, hbytes, &hp));
  }
  P.host = (double*)hp;
  if (P.reserve_only) return ME_OK;
  P.hstate[0] = (State*)((char*)hp + stage);
  P.hstate[1] = (State*)((char*)hp + stage + rup(sizeof(State), 64));
  P.dev = dev;
  hipStream_t s = c->stream;
  if (!dev) {
    // pack the inputs at their arena offsets in pinned memory: one H2D copy
    char* h = (char*)hp;
    const void* src[6] = {p->cams, p->pts, p->obs, p->cam_idx, p->pt_idx, p->cam_id};
    const size_t len[6] = {8 * 6 * (size_t)g.nc, 8 * 3 * (size_t)g.np, 8 * g.od * (size_t)g.no, 4 * (size_t)g.no,
                           4 * (size_t)g.no, mono ? 4 * (size_t)g.no : 0};
    size_t off = 0;
    for (int k = 0; k < 6; ++k) {
      if (len[k]) std::memcpy(h + off, src[k], len[k]);
      off += items[k].first;
    }
    ME_HIP(c, hipMemcpyAsync(b.cams[0], hp, input_span, hipMemcpyHostToDevice, s));
  } else {
    b.obs = p->obs;
    b.cam_idx = p->cam_idx;
    b.pt_idx = p->pt_idx;
    if (mono) b.cam_id = p->cam_id;
  }
  // cnt | work are adjacent in the arena: one fill clears both
  ME_HIP(c, hipMemsetAsync(b.cnt, 0, (size_t)((char*)b.work - (char*)b.cnt) + work_bytes, s));
  P.asm_gen = 0;  // (the claim words were just cleared)
  const double* cams_in = dev ? p->cams : b.cams[0];
  const double* pts_in = dev ? p->pts : b.pts[0];
  const long nthr = std::max({(long)g.nblk_obs * kBlock, (long)g.np, 6L * g.nc, 3L * g.np});
  hipLaunchKernelGGL(plan_count_kernel, dim3(blocks(nthr, kBlock)), dim3(kBlock), 4 * (size_t)g.nc, s, g, b, cams_in,
                     pts_in);
  hipLaunchKernelGGL(plan_scan_kernel, dim3(1), dim3(kScanBlock), 0, s, g, b, o);
  hipLaunchKernelGGL(plan_scatter_kernel, dim3(g.nblk_obs), dim3(kBlock), 0, s, g, b);
  hipLaunchKernelGGL(plan_segsort_kernel, dim3(blocks(std::max(g.np, 1), kSortBlock / 64)), dim3(kSortBlock), 0, s, g,
                     b);
  if (g.sorted) {
    hipLaunchKernelGGL(plan_band_kernel, dim3(g.nblkp), dim3(kBlock), 0, s, g, b);
    hipLaunchKernelGGL(plan_order_kernel, dim3(1), dim3(kScanBlock), 0, s, g, b);
  }
  ME_TRY(me_check_launch(c, "BA plan"));
  // LDS for the camera solve
  P.solve_lds = 8 * (solve_small_doubles(g.Ts) + solve_a_doubles(g.Ts));
  P.use_lds = P.solve_lds <= 150 * 1024 ? 1 : 0;
  if (!P.use_lds) P.solve_lds = 8 * solve_small_doubles(g.Ts);
  ME_CHECK(c, P.solve_lds <= 150 * 1024, "BA: %d variable cameras exceed the camera-solve workspace", g.m);
  P.schur_lds = schur_lds_bytes(g.spts, g.Rpad);
  ME_CHECK(c, P.schur_lds <= kSchurLdsCap, "BA: %d variable cameras exceed the Schur workspace", g.m);
  // dynamic-LDS ceilings of the solve and Schur kernels: set once per context
  // at the cap every plan stays under (not per solve: ~36 runtime calls of
  // host time in front of every queued solve)
  if (!c->ba_lds_attr) {
    for (const void* k : {(const void*)cam_solve_kernel<0>, (const void*)cam_solve_kernel<1>, (const void*)cam_solve_kernel<2>})
      ME_HIP(c, hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
#define ME_SCHUR_K(N)                                                                                   \
  (const void*)pt_schur_kernel<N, 512, kSchurPts>, (const void*)pt_schur_kernel<N, 512, kSchurPtsWide>, \
      (const void*)pt_schur_kernel<N, 512, kSchurPtsSmall>
    for (const void* k : {ME_SCHUR_K(2), ME_SCHUR_K(3), ME_SCHUR_K(4), ME_SCHUR_K(5)})
#undef ME_SCHUR_K
      ME_HIP(c, hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSchurLdsCap));
    c->ba_lds_attr = 1;
  }
  // the multi-workgroup camera solve deals its tiles over the workers that
  // joined its roster (roster.hpp), so residency is never assumed; the
  // workers launched are still capped by what fits on the ctx's CUs (more
  // could only join late and leave), and an explicit worker count is clamped
  // by it too
  if (!P.use_lds) {
    int per_cu = 0;
    ME_HIP(c, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, cam_solve_kernel<2>, kSolveBlock, P.solve_lds));
    P.solve_cap = std::max(0, per_cu) * (c->cu_active > 0 ? c->cu_active : c->num_cu);
    if (P.comm && (g.Ts >= kSolveMwMinTs || P.solve_workers > 0)) {
      // Sharded: every rank solves the camera system redundantly and must run
      // the same solve form (worker count) on the same operands, whatever its
      // own CU mask: the smallest capacity over the ranks (one max exchange of
      // -cap at plan time; the result is read back before any iteration).
      double* d = P.b.scal;  // (free until the first linearisation)
      const double v = -(double)P.solve_cap;
      ME_HIP(c, hipMemcpyAsync(d, &v, 8, hipMemcpyHostToDevice, c->stream));
      ME_TRY(me_comm_allreduce_impl(P.comm, d, 1, ME_COMM_MAX));
      double r = 0.0;
      ME_HIP(c, hipMemcpyAsync(&r, d, 8, hipMemcpyDeviceToHost, c->stream));
      ME_HIP(c, hipStreamSynchronize(c->stream));
      P.solve_cap = (int)-r;
    }
  }
  return ME_OK;
}



// all-reduce of n doubles on the ctx stream through the plan's communicator
#define ME_XCH(ptr, n, op) ME_TRY(me_comm_allreduce_impl(P.comm, (ptr), (long)(n), (op)))

// Linearisation stage (device-skipped when need_lin == 0)
int enqueue_linearize(Plan& P) {
  me_ctx* c = P.c;
  const Geo& g = P.g;
  hipStream_t s = c->stream;
  const bool sh = P.comm != nullptr;
  {
    me_ktimer t(c, ME_KT_BA_LINEARIZE);
    const bool small = lin_block(g.no) == kLinSmall;
    if (g.od == 4 && small)
      hipLaunchKernelGGL((linearize_kernel<4, kLinSmall>), dim3(g.nblk_lin), dim3(kLinSmall), 0, s, g, P.b);
    else if (g.od == 4)
      hipLaunchKernelGGL((linearize_kernel<4, kBlock>), dim3(g.nblk_lin), dim3(kBlock), 0, s, g, P.b);
    else if (small)
      hipLaunchKernelGGL((linearize_kernel<2, kLinSmall>), dim3(g.nblk_lin), dim3(kLinSmall), 0, s, g, P.b);
    else
      hipLaunchKernelGGL((linearize_kernel<2, kBlock>), dim3(g.nblk_lin), dim3(kBlock), 0, s, g, P.b);
  }
  // After the first linearisation the Jacobi scaling is fixed and the Schur
  // pass no longer needs the camera assembly: its m x ck workgroups then ride
  // in the Schur launch (one launch fewer per iteration; a second stream with
  // event fork/join measured slower).  Sharded runs too: a rank's U and g
  // blocks are then scaled by the fixed global scaling, and the exchange sums
  // them.
  const bool first = P.n_enq == 0;
  const bool fused = !first && g.m > 0 && !P.sequential;
  ++P.n_enq;
  CamArgs ca{P.cpart, P.colnorm, P.gc_raw, P.Uraw, fused ? 1 : 0, fused ? (g.m * g.ck + 7) / 8 * 8 : 0};
  if (g.m > 0 && !fused)
    hipLaunchKernelGGL(cam_assemble_kernel, dim3(g.m, g.ck), dim3(kBlock), 0, s, g, P.b, P.cpart, sh ? 1 : 0,
                       P.colnorm, P.gc_raw, P.Uraw);
  if (sh && !fused) {
    // the Jacobi scaling needs the global column norms: the first exchange
    // (with every rank's input flags behind them), then the local blocks scaled
    if (first) {
      hipLaunchKernelGGL(xch_flags_kernel, dim3(1), dim3(1), 0, s, g, P.b, P.colnorm);
      ME_XCH(P.colnorm, g.n6 + 2, ME_COMM_SUM);
    }
    hipLaunchKernelGGL(cam_finish_kernel, dim3(blocks(std::max(g.m, 1), 64)), dim3(64), 0, s, g, P.b,
                       (const double*)P.colnorm, (const double*)P.gc_raw, (const double*)P.Uraw, first ? 1 : 0);
  }
  {
    // point blocks + Schur partial tiles (BA_SCHUR family)
    me_ktimer t(c, ME_KT_BA_SCHUR, true);  // (sampled launches take the timer's events)
    // NT = this wave's tile count, instantiated tight: an unused tile's
    // accumulator costs 8 VGPRs, and at 512 threads (2 waves per SIMD) the
    // budget is 256 registers -- up to 5 tiles nothing spills (9 tiles spilled
    // 120 B); wider windows take more tile groups per run instead.
    const int pw8 = g.stpw / 8;
    const dim3 grd(g.ksplit + ca.ncam);
#define ME_SCHUR(N)                                                                                          \
  do {                                                                                                       \
    if (g.spts == kSchurPtsWide)                                                                             \
      hipExtLaunchKernelGGL((pt_schur_kernel<N, 512, kSchurPtsWide>), grd, dim3(512), P.schur_lds, s, t.a, t.b, 0, g, \
                            P.b, P.o, ca);                                                                   \
    else if (g.spts == kSchurPtsSmall)                                                                       \
      hipExtLaunchKernelGGL((pt_schur_kernel<N, 512, kSchurPtsSmall>), grd, dim3(512), P.schur_lds, s, t.a, t.b, 0, g, \
                            P.b, P.o, ca);                                                                   \
    else                                                                                                     \
      hipExtLaunchKernelGGL((pt_schur_kernel<N, 512, kSchurPts>), grd, dim3(512), P.schur_lds, s, t.a, t.b, 0, g, P.b, \
                            P.o, ca);                                                                        \
  } while (0)
    static_assert(kSchurNtMax >= 3 && kSchurNtMax <= 5, "instantiated tile counts");
    if (pw8 <= 2) ME_SCHUR(2);
    else if (pw8 <= 3) ME_SCHUR(3);
    else if (pw8 <= 4) ME_SCHUR(4);
    else ME_SCHUR(5);
#undef ME_SCHUR
  }
  if (sh) {
    // this rank's reduced camera system, gradient and linearisation scalars
    // packed, then ONE sum over the ranks
    hipLaunchKernelGGL(s_assemble_kernel, dim3(blocks((long)g.npairs * 256, kSaElems) + 1), dim3(kBlock), 0, s, g,
                       P.b, P.o, (const double*)P.gc_raw, 0, (int)SA_PACK);
    if (P.xmax_separate) {
      ME_XCH(P.b.xch, xo_gmax(g), ME_COMM_SUM);
      ME_XCH(P.b.xch + xo_gmax(g), 1, ME_COMM_MAX);
    } else {
      ME_XCH(P.b.xch, xo_total(g), ME_COMM_SUM);
    }
  }
  return me_check_launch(c, "BA linearize");
}

// S / b assembly; its last workgroup closes the linearisation (lin_finalize).
// Sharded: S / b unpacked from the all-reduced exchange.
// img: the assembly writes the camera solve's image of [S + D; -b^T] (the
// solver's padded layout, s_assemble_body) into Abuf, so the solve that
// follows loads nothing: its element-wise load of S cost wg0 ~70 us at config
// 5 (tools/drivers.py solve_ts).  Not with full_S (S itself is read back).
int enqueue_assemble(Plan& P, bool img = false) {
  me_ctx* c = P.c;
  const Geo& g = P.g;
  const int mode = P.comm ? SA_UNPACK : SA_SUM;
  if (g.m > 0)
    hipLaunchKernelGGL(s_assemble_kernel, dim3(blocks((long)g.npairs * 256, kSaElems) + 1), dim3(kBlock), 0,
                       c->stream, g, P.b, P.o, (const double*)P.gc_raw, P.full_S ? 1 : 0, mode,
                       img && !P.full_S ? P.b.Abuf : nullptr);
  else
    hipLaunchKernelGGL(lin_finalize_kernel, dim3(1), dim3(kFinBlock), 0, c->stream, g, P.b, P.o,
                       (const double*)P.gc_raw);
  return me_check_launch(c, "BA assemble");
}

// `last`: the enqueue after max_num_iterations steps.  Its linearisation feeds
// only the closing gradient test and final cost, and its lin_finalize always
// ends the solve (iterations == max_num_iterations), so the camera solve and
// the point step that would follow are never run: they are not queued (two
// no-op launches fewer per solve; every rank of a sharded solve skips alike).
int enqueue_iteration(Plan& P, bool last = false) {
  me_ctx* c = P.c;
  const Geo& g = P.g;
  hipStream_t s = c->stream;
  const bool sh = P.comm != nullptr;
  ME_TRY(enqueue_linearize(P));
  // camera-solve form: 0 = [S; -b^T] in LDS, 1 = global memory, 2 = global
  // memory with trailing-update workers.  Trailing-update workers pay once the
  // block steps are many and wide: config 5 (19 steps) 372 -> 274 us per
  // solve; config 4 (11 steps) is faster on one workgroup (118 vs 131 us: the
  // per-step hand-offs).  The workers are capped by what can be co-resident.
  const int np0 = (g.Ts - 1) * g.Ts / 2;
  int nwk = P.use_lds ? 0
            : P.solve_workers >= 0 ? P.solve_workers
            : g.Ts >= kSolveMwMinTs ? std::min(64, std::max(1, (np0 + kSolveBlock / 64 - 1) / (kSolveBlock / 64)))
                                    : 0;
  if (nwk > 0) {
    const int cap = std::max(0, std::min(nwk, P.solve_cap - 1));
    if (P.solve_workers > 0 && cap != nwk && !P.warned_workers) {  // an explicit count the CUs cannot host
      std::fprintf(stderr, "me_ba: ME_SOLVE_WORKERS=%d exceeds the co-resident capacity, using %d\n", nwk, cap);
      P.warned_workers = 1;
    }
    nwk = cap;
  }
  // S = U - sum of the Schur partials is assembled by wide workgroups
  // (coalesced, all CUs) rather than by the one-workgroup solve, whose
  // dependent cross-XCD loads would otherwise dominate the iteration.  Modes
  // 0 and 1 they ride in the camera-solve launch (fused assembly; sharded:
  // they unpack the exchanged system).
  const bool fuse = g.m > 0 && !P.full_S && !last && !P.sequential && nwk == 0 && !P.no_fused_asm;
  const int nasm = fuse ? blocks((long)g.npairs * 256, kSolveBlock / kSaGroups) : 0;
  const bool img = !fuse && !last && g.m > 0 && !P.full_S && ME_SOLVE_IMG;
  if (!fuse) ME_TRY(enqueue_assemble(P, img));
  if (last) return me_check_launch(c, "BA iteration");
  if (g.m == 0) ME_HIP(c, hipMemsetAsync(P.b.scal + R_COUNT, 0, 8, s));
  {
    me_ktimer t(c, ME_KT_BA_SOLVE);
    const double* gc = P.gc_raw;
    const int sk = P.diag_skip | (img ? kSkipImg : 0);
    const unsigned gen = nasm > 0 ? ++P.asm_gen : 0u;  // fused assembly: this launch's claim generation
    if (P.use_lds)
      hipLaunchKernelGGL(cam_solve_kernel<0>, dim3(1 + nasm), dim3(kSolveBlock), P.solve_lds, s, g, P.b, P.o, sk, 0,
                         nasm, gc, gen);
    else if (nwk > 0)
#ifdef ME_COOP_LAUNCH  // measurement build only (tools/gpu.sh coop): the worker grid as a cooperative launch
    {
      int skv = sk, nwv = nwk, z = 0;
      unsigned gv = gen;
      void* args[] = {(void*)&g, (void*)&P.b, (void*)&P.o, &skv, &nwv, &z, (void*)&gc, &gv};
      ME_HIP(c, hipLaunchCooperativeKernel((const void*)cam_solve_kernel<2>, dim3(1 + nwk), dim3(kSolveBlock), args,
                                           (unsigned)P.solve_lds, s));
    }
#else
      hipLaunchKernelGGL(cam_solve_kernel<2>, dim3(1 + nwk), dim3(kSolveBlock), P.solve_lds, s, g, P.b, P.o, sk, nwk,
                         0, gc, gen);
#endif
    else
      hipLaunchKernelGGL(cam_solve_kernel<1>, dim3(1 + nasm), dim3(kSolveBlock), P.solve_lds, s, g, P.b, P.o, sk, 0,
                         nasm, gc, gen);
  }
  {
    me_ktimer t(c, ME_KT_BA_STEP);
    // (step partials reduced and, single-GPU, the step decided in its last workgroup)
    if (g.od == 4)
      hipLaunchKernelGGL(pt_step_kernel<4>, dim3(g.nblk_step + 1), dim3(kStepBlock), 0, s, g, P.b, P.o, sh ? 0 : 1);
    else
      hipLaunchKernelGGL(pt_step_kernel<2>, dim3(g.nblk_step + 1), dim3(kStepBlock), 0, s, g, P.b, P.o, sh ? 0 : 1);
  }
  if (sh) {
    ME_XCH(P.b.scal + R_MODEL, 5, ME_COMM_SUM);  // model change, candidate cost, step^2, |x|^2, failure count
    hipLaunchKernelGGL(decide_kernel, dim3(1), dim3(64), 0, s, g, P.b, P.o);
  }
  return me_check_launch(c, "BA iteration");
}

// Final state (and host parameters) -> pinned staging; enqueued behind the
// last chunk so the read-back does not wait for a host round trip.
int enqueue_output(Plan& P, me_ba_problem* p) {
  me_ctx* c = P.c;
  const Geo& g = P.g;
  constexpr size_t nst = sizeof(State) / 8;
  double* cams_dst = P.dev ? p->cams : P.b.out + nst;
  double* pts_dst = P.dev ? p->pts : P.b.out + nst + 6 * (size_t)g.nc;
  const long n = std::max({(long)nst, 6L * g.nc, 3L * g.np});
  hipLaunchKernelGGL(output_kernel, dim3(blocks(n, kBlock)), dim3(kBlock), 0, c->stream, g, P.b, cams_dst, pts_dst);
  ME_TRY(me_check_launch(c, "BA output"));
  const size_t bytes = 8 * (P.dev ? nst : nst + 6 * (size_t)g.nc + 3 * (size_t)g.np);
  ME_HIP(c, hipMemcpyAsync(P.host, P.b.out, bytes, hipMemcpyDeviceToHost, c->stream));
  if (P.dev && P.copy_out) {  // (staging holds State | cams | pts: out_doubles)
    ME_HIP(c, hipMemcpyAsync(P.host + nst, p->cams, 8 * 6 * (size_t)g.nc, hipMemcpyDeviceToHost, c->stream));
    if (g.np)
      ME_HIP(c, hipMemcpyAsync(P.host + nst + 6 * (size_t)g.nc, p->pts, 8 * 3 * (size_t)g.np, hipMemcpyDeviceToHost,
                               c->stream));
  }
  return ME_OK;
}

int finish(Plan& P, me_ba_problem* p, me_ba_summary* sum, bool output_queued = false, hipEvent_t done = nullptr) {
  me_ctx* c = P.c;
  const Geo& g = P.g;
  constexpr size_t nst = sizeof(State) / 8;
  static_assert(sizeof(State) % 8 == 0, "State is read back as doubles");
  if (!output_queued) ME_TRY(enqueue_output(P, p));
  if (done) ME_HIP(c, hipEventSynchronize(done));  // asynchronous solve: not the work queued after it
  else ME_HIP(c, hipStreamSynchronize(c->stream));
  State st;
  std::memcpy(&st, P.host, sizeof(State));
  std::memcpy(P.c->dbg, st.stamps, sizeof(st.stamps));
  if (!P.dev) {
    std::memcpy(p->cams, P.host + nst, 8 * 6 * (size_t)g.nc);
    if (g.np) std::memcpy(p->pts, P.host + nst + 6 * (size_t)g.nc, 8 * 3 * (size_t)g.np);
  }
  if (st.bad_input) return me_set_error(c, ME_ERR_INVALID, "BA: an observation indexes outside the window");
  if (st.spin_err)
    return me_set_error(c, ME_ERR_STATE,
                        "BA: a cross-workgroup hand-off of the camera solve timed out (workgroups not co-resident: "
                        "CU mask or concurrent persistent kernels; wait sites 0x%x: 1 worker roster, 2 worker step "
                        "poll, 4 fused assemblers, 8 LDS step flags, 16 workers' count, 32 backward flags, 0 the "
                        "step exchange)",
                        (unsigned)st.pad[0]);
  if (sum) {
    sum->termination = st.termination;
    sum->iterations = st.iterations;
    sum->successful_steps = st.successful;
    sum->initial_cost = st.initial_cost;
    sum->final_cost = st.x_cost;
    sum->status = st.termination == 2 ? 3 : 2;
    if (st.infeasible) {  // Ceres: infeasible start -> FAILURE, parameters untouched
      sum->iterations = 0;
      sum->successful_steps = 0;
      sum->initial_cost = sum->final_cost = NAN;
    }
  }
  return ME_OK;
}

int solve_impl(me_ctx* c, me_ba_problem* p, const me_ba_options* opt, me_comm* comm, me_ba_summary* sum) {
  me_range range_("me_ba_solve");
  if (!c || !p || !opt) return ME_ERR_INVALID;
  ME_HIP(c, hipSetDevice(c->device));
  Plan P;
  ME_TRY(plan_build(c, p, opt, P, 0, -1, comm));
  // Enqueue the solve in chunks of iterations.  The device State after each
  // chunk is copied to a pinned slot behind an event, and the host inspects
  // chunk k only after chunk k + 1 is queued, so the GPU never drains while
  // the host polls; after convergence at most one chunk of no-op launches
  // (every kernel tests State::done first) is left in the queue.
  const int chunk = 4;
  int it = 0;
  auto enqueue_chunk = [&](int slot) -> int {
    for (int k = 0; k < chunk && it <= opt->max_num_iterations; ++k, ++it)
      ME_TRY(enqueue_iteration(P, it == opt->max_num_iterations));
    ME_HIP(c, hipMemcpyAsync(P.hstate[slot], P.b.st, sizeof(State), hipMemcpyDeviceToHost, c->stream));
    ME_HIP(c, hipEventRecord(c->poll_ev[slot], c->stream));
    return ME_OK;
  };
  // once the last possible chunk is queued, the output follows it at once
  bool out_q = false;
  ME_TRY(enqueue_chunk(0));
  if (it > opt->max_num_iterations) {
    ME_TRY(enqueue_output(P, p));
    out_q = true;
  }
  for (int cur = 0;; cur ^= 1) {
    const bool more = it <= opt->max_num_iterations;
    if (more) {
      ME_TRY(enqueue_chunk(cur ^ 1));
      if (it > opt->max_num_iterations) {
        ME_TRY(enqueue_output(P, p));
        out_q = true;
      }
    }
    ME_HIP(c, hipEventSynchronize(c->poll_ev[cur]));
    if (P.hstate[cur]->done || !more) break;
  }
  return finish(P, p, sum, out_q);
}

// Asynchronous solve: every possible iteration is queued at once (launches
// after convergence test State::done and return), then the output kernel and
// read-back behind an event.  The host is free as soon as it is queued.  Up
// to two solves may be queued on a ctx (each in its own scratch / staging
// set), so a caller can queue window t+1 behind window t without waiting:
// the device never idles while the host builds the next plan.
struct AsyncSolve {
  Plan P;
  me_ba_problem prob;  // copy: cams / pts are written back at completion
  hipEvent_t ev = nullptr;
  int set = 0;  // scratch / staging set
  bool completed = false;
  int rc = ME_OK;
  me_ba_summary sum{};
};
constexpr int kBaQueue = 2;
// The queue may be used from two host threads at once: one queueing window
// t (me_ba_solve_async / me_vo_window_submit) while another waits for window
// t-1 (me_ba_wait_out).  The lock guards the FIFO only; the solve's own
// queueing and waiting run outside it.  The newest waited solve is retained
// (`last`) until a newer one is queued: window t may be chained from window
// t-1 (me_vo_ba_chain) after t-1 was waited.
struct AsyncQueue {
  AsyncSolve* q[kBaQueue] = {nullptr, nullptr};  // FIFO: q[0] oldest
  int n = 0;
  AsyncSolve* last = nullptr;  // newest waited solve (chain source)
  int last_set = 1;            // scratch / staging set of the newest queued solve
  std::mutex mu;
};

int ba_complete_one(me_ctx* c, AsyncSolve* A) {
  if (A->completed) return ME_OK;
  A->rc = finish(A->P, &A->prob, &A->sum, true, A->ev);
  A->completed = true;
  return ME_OK;
}

void ba_async_free(me_ctx* c) {
  auto* Q = (AsyncQueue*)c->ba_async;
  if (!Q) return;
  for (int i = 0; i < Q->n; ++i) {
    AsyncSolve* A = Q->q[i];
    if (!A->completed) hipEventSynchronize(A->ev);
    hipEventDestroy(A->ev);
    delete A;
  }
  delete Q->last;  // (its event was destroyed when it was waited)
  delete Q;
  c->ba_async = nullptr;
  c->ba_async_free = nullptr;
}

AsyncQueue* ba_queue(me_ctx* c) {
  if (!c->ba_async) {
    c->ba_async = new AsyncQueue;
    c->ba_async_free = ba_async_free;
  }
  return (AsyncQueue*)c->ba_async;
}

// Any other BA call on the ctx first completes the queued solves (their
// summaries stay readable by me_ba_wait, oldest first).
int ba_drain(me_ctx* c) {
  auto* Q = (AsyncQueue*)c->ba_async;
  if (!Q) return ME_OK;
  for (int i = 0; i < Q->n; ++i) ME_TRY(ba_complete_one(c, Q->q[i]));
  return ME_OK;
}

// the solve a new one is chained from: the newest queued, else the newest waited
AsyncSolve* ba_chain_source(AsyncQueue* Q) {
  std::lock_guard<std::mutex> lk(Q->mu);
  return Q->n ? Q->q[Q->n - 1] : Q->last;
}

}  // namespace

// copy_out: a device-resident problem's solved cams / pts also read back
// into the staging behind the solve (me_vo_window_submit; me_ba_wait_out
// then returns them without touching the stream)
static int solve_async_impl(me_ctx* c, me_ba_problem* p, const me_ba_options* opt, bool copy_out) {
  if (!c || !p || !opt) return ME_ERR_INVALID;
  ME_HIP(c, hipSetDevice(c->device));
  AsyncQueue* Q = ba_queue(c);
  auto* A = new AsyncSolve;
  {
    std::lock_guard<std::mutex> lk(Q->mu);
    if (Q->n >= kBaQueue) {
      delete A;
      return me_set_error(c, ME_ERR_STATE,
                          "me_ba_solve_async: %d solves already queued on this context (me_ba_wait first)", kBaQueue);
    }
    A->set = 1 - Q->last_set;  // never the set of the solve queued before (queued, or being read back)
    Q->last_set = A->set;
  }
  A->prob = *p;
  int rc = plan_build(c, p, opt, A->P, A->set, A->set);
  A->P.copy_out = copy_out && A->P.dev;
  if (rc == ME_OK) {
    for (int it = 0; it <= opt->max_num_iterations && rc == ME_OK; ++it)
      rc = enqueue_iteration(A->P, it == opt->max_num_iterations);
  }
  if (rc == ME_OK) rc = enqueue_output(A->P, &A->prob);
  if (rc == ME_OK && hipEventCreateWithFlags(&A->ev, hipEventDisableTiming) != hipSuccess)
    rc = me_set_error(c, ME_ERR_HIP, "me_ba_solve_async: event creation failed");
  if (rc == ME_OK && hipEventRecord(A->ev, c->stream) != hipSuccess) {
    hipEventDestroy(A->ev);
    rc = me_set_error(c, ME_ERR_HIP, "me_ba_solve_async: event record failed");
  }
  if (rc != ME_OK) {
    hipStreamSynchronize(c->stream);  // nothing queued may outlive the plan
    delete A;
    return rc;
  }
  AsyncSolve* old = nullptr;
  {
    std::lock_guard<std::mutex> lk(Q->mu);
    Q->q[Q->n++] = A;
    std::swap(old, Q->last);  // a newer solve is queued: the retained chain source goes
  }
  delete old;
  return ME_OK;
}

extern "C" int me_ba_solve_async(me_ctx* c, me_ba_problem* p, const me_ba_options* opt) {
  me_range range_("me_ba_solve_async");
  return solve_async_impl(c, p, opt, false);
}

extern "C" int me_ba_wait_out(me_ctx* c, me_ba_summary* s, double* cams, double* pts) {
  me_range range_("me_ba_wait");
  if (!c) return ME_ERR_INVALID;
  auto* Q = (AsyncQueue*)c->ba_async;
  AsyncSolve* A = nullptr;
  if (Q) {
    std::lock_guard<std::mutex> lk(Q->mu);
    if (Q->n) A = Q->q[0];
  }
  if (!A) return me_set_error(c, ME_ERR_STATE, "me_ba_wait: no asynchronous BA solve on this context");
  ME_HIP(c, hipSetDevice(c->device));
  ME_TRY(ba_complete_one(c, A));
  const int rc = A->rc;
  if (s && rc == ME_OK) *s = A->sum;
  if (rc == ME_OK && A->P.dev && (cams || pts)) {
    constexpr size_t nst = sizeof(State) / 8;
    const Geo& g = A->P.g;
    if (A->P.copy_out) {  // from the staging (read back behind the solve's event)
      if (cams) std::memcpy(cams, A->P.host + nst, 8 * 6 * (size_t)g.nc);
      if (pts && g.np) std::memcpy(pts, A->P.host + nst + 6 * (size_t)g.nc, 8 * 3 * (size_t)g.np);
    } else {  // (blocking copies on the null stream: the solve has completed; the ctx stream is not waited)
      if (cams) ME_HIP(c, hipMemcpy(cams, A->prob.cams, 8 * 6 * (size_t)g.nc, hipMemcpyDeviceToHost));
      if (pts && g.np) ME_HIP(c, hipMemcpy(pts, A->prob.pts, 8 * 3 * (size_t)g.np, hipMemcpyDeviceToHost));
    }
  }
  hipEventDestroy(A->ev);
  A->ev = nullptr;
  AsyncSolve* gone = A;
  {
    std::lock_guard<std::mutex> lk(Q->mu);
    for (int i = 1; i < Q->n; ++i) Q->q[i - 1] = Q->q[i];
    Q->q[--Q->n] = nullptr;
    if (Q->n == 0) {  // the newest: retained as the chain source until a newer one is queued
      std::swap(gone, Q->last);
    }
  }
  delete gone;
  return rc;
}

extern "C" int me_ba_wait(me_ctx* c, me_ba_summary* s) { return me_ba_wait_out(c, s, nullptr, nullptr); }

extern "C" int me_ba_reserve(me_ctx* c, int n_cams, int n_pts, int n_obs, int obs_dim, int fixed_frames) {
  me_range range_("me_ba_reserve");
  if (!c || n_cams < 1 || n_pts < 0 || n_obs < 0) return ME_ERR_INVALID;
  ME_HIP(c, hipSetDevice(c->device));
  auto* Q = (AsyncQueue*)c->ba_async;
  if (Q && Q->n > 0) return me_set_error(c, ME_ERR_STATE, "me_ba_reserve: asynchronous solves are queued");
  ME_TRY(ba_drain(c));
  // a problem of these sizes (no arrays: the plan stops once its memory is sized)
  static const int32_t zero = 0;
  me_ba_problem p{};
  p.n_cams = n_cams;
  p.n_pts = n_pts;
  p.n_obs = n_obs;
  p.obs_dim = obs_dim == 2 ? 2 : 4;
  p.fixed_frames = fixed_frames;
  p.mem = ME_DEVICE;
  p.cam_id = &zero;
  p.feat_var = 1.0;
  p.baseline = 1.0;
  const double K[9] = {1, 0, 1, 0, 1, 1, 0, 0, 1};
  std::memcpy(p.K0, K, sizeof(K));
  std::memcpy(p.K1, K, sizeof(K));
  me_ba_options o;
  me_ba_default_options(&o);
  for (int set = 0; set < kBaQueue; ++set) {  // the asynchronous solves' two sets
    Plan P;
    P.reserve_only = true;
    ME_TRY(plan_build(c, &p, &o, P, set, set));
  }
  Plan P;  // and the synchronous one
  P.reserve_only = true;
  return plan_build(c, &p, &o, P, 0);
}

// ---------------------------------------------------------------- VO chain
// The windowed VO loop (pipeline.py, WindowedStereoVO.process step 7) forms
// window t's BA start from window t-1's BA result: the poses and landmarks it
// solved (when it succeeded, BundleAdjuster status 2), pose(t) predicted again
// from the refined poses, and the landmarks new in t moved with it (their
// camera-frame coordinates kept).  On the device the same arithmetic, in the
// same order (fp-contract off; the rotation of the new pose by a fixed Taylor
// series in theta^2: no libm), runs behind window t-1's solve, so window t is
// queued before t-1 completes; the host repeats it on the downloaded result
// (pipeline.rot_series, bit for bit).
namespace {
__device__ __constant__ double kRotA[24] = {
    1.0, -0.16666666666666666, 0.008333333333333333, -0.0001984126984126984, 2.7557319223985893e-06,
    -2.505210838544172e-08, 1.6059043836821613e-10, -7.647163731819816e-13, 2.8114572543455206e-15,
    -8.22063524662433e-18, 1.9572941063391263e-20, -3.868170170630684e-23, 6.446950284384474e-26,
    -9.183689863795546e-29, 1.1309962886447716e-31, -1.216125041553518e-34, 1.151633562077195e-37,
    -9.67759295863189e-41, 7.265460179153071e-44, -4.902469756513544e-47, 2.9893108271424046e-50,
    -1.6552108677421951e-53, 8.359650847182804e-57, -3.866628513960594e-60};  // (-1)^k / (2k+1)!
__device__ __constant__ double kRotB[24] = {
    0.5, -0.041666666666666664, 0.001388888888888889, -2.48015873015873e-05, 2.755731922398589e-07,
    -2.08767569878681e-09, 1.1470745597729725e-11, -4.779477332387385e-14, 1.5619206968586225e-16,
    -4.110317623312165e-19, 8.896791392450574e-22, -1.6117375710961184e-24, 2.4795962632247976e-27,
    -3.279889237069838e-30, 3.7699876288159054e-33, -3.8003907548547434e-36, 3.387157535521162e-39,
    -2.6882202662866363e-42, 1.911963205040282e-45, -1.2256174391283858e-48, 7.117406731291439e-52,
    -3.7618428812322616e-55, 1.817315401561479e-58, -8.055476070751236e-62};  // (-1)^k / (2k+2)!

// R = I + A [a]x + B [a]x^2, A = sin(th) / th, B = (1 - cos th) / th^2, th = |a|
__device__ void rot_series(const double* a, double* R) {
  const double t2 = (a[0] * a[0] + a[1] * a[1]) + a[2] * a[2];
  double A = kRotA[23], B = kRotB[23];
  for (int k = 22; k >= 0; --k) {
    A = A * t2 + kRotA[k];
    B = B * t2 + kRotB[k];
  }
  const double K[9] = {0.0, -a[2], a[1], a[2], 0.0, -a[0], -a[1], a[0], 0.0};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      const double k2 = a[i] * a[j] - (i == j ? t2 : 0.0);
      R[3 * i + j] = ((i == j ? 1.0 : 0.0) + A * K[3 * i + j]) + B * k2;
    }
}

// One launch over the window's landmarks; every workgroup forms pose(t)
// itself, workgroup 0 also writes the cameras.  A camera with a source index
// / a landmark whose track ID the previous window holds takes the previous
// solve's value when that solve succeeded, else keeps the host's (the loop's
// state before the solve); a landmark with ID >= new_from is new in t (moved
// when pose(t) changed).
__global__ __launch_bounds__(256) void vo_chain_kernel(const double* pc, const double* pp, const State* pst, double* cams,
                                                       int nc, double* pts, int np, const int* cam_src,
                                                       const int* win_ids, const int* prev_ids, int n_prev,
                                                       int new_from, me_vo_chain_args a) {
  __shared__ double sh[6 + 9];  // pose(t) | its rotation
  const bool ok = pst->termination != 2;
  auto cam = [&](int k, int j) {
    const int s = cam_src[k];
    return ok && s >= 0 ? pc[6 * s + j] : cams[6 * k + j];
  };
  if (threadIdx.x == 0) {
    double p2[6];
    for (int j = 0; j < 6; ++j) {
      const double c1 = cam(a.k1, j);
      p2[j] = a.mode == 1 ? c1 + (c1 - cam(a.k0, j)) : a.mode == 0 ? c1 + a.vel[j] : cams[6 * (nc - 1) + j];
    }
    for (int j = 0; j < 6; ++j) sh[j] = p2[j];
    rot_series(p2 + 3, sh + 6);
  }
  __syncthreads();
  if (blockIdx.x == 0) {  // (formed in LDS first: cam() reads the fallbacks in place)
    extern __shared__ double scam[];
    for (int e = threadIdx.x; e < 6 * nc; e += blockDim.x) scam[e] = e >= 6 * (nc - 1) ? sh[e % 6] : cam(e / 6, e % 6);
    __syncthreads();
    for (int e = threadIdx.x; e < 6 * nc; e += blockDim.x) cams[e] = scam[e];
  }
  bool moved = false;
  for (int j = 0; j < 6; ++j) moved = moved || sh[j] != a.pose[j];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= np) return;
  // landmark i's source: its track ID in the previous window's ascending IDs
  const int id = win_ids[i];
  int s = -2;
  if (id < new_from) {
    int lo = 0, hi = n_prev;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (prev_ids[mid] < id)
        lo = mid + 1;
      else
        hi = mid;
    }
    s = lo < n_prev && prev_ids[lo] == id ? lo : -1;
  }
  double* X = pts + 3 * (long)i;
  if (s >= 0) {
    if (ok)
      for (int k = 0; k < 3; ++k) X[k] = pp[3 * (long)s + k];
  } else if (s == -2 && moved) {
    const double* R = a.R;
    const double* R2 = sh + 6;
    double d[3];
    for (int k = 0; k < 3; ++k) d[k] = (((X[0] * R[3 * k] + X[1] * R[3 * k + 1]) + X[2] * R[3 * k + 2]) + a.pose[k]) - sh[k];
    double y[3];
    for (int k = 0; k < 3; ++k) y[k] = (d[0] * R2[k] + d[1] * R2[3 + k]) + d[2] * R2[6 + k];
    for (int k = 0; k < 3; ++k) X[k] = y[k];
  }
}
}  // namespace

extern "C" int me_vo_ba_chain(me_ctx* c, double* cams, int n_cams, double* pts, int n_pts, const int32_t* cam_src,
                              const int32_t* win_ids, const int32_t* prev_ids, int n_prev, int32_t new_from,
                              const me_vo_chain_args* a) {
  me_range range_("me_vo_ba_chain");
  if (!c || !a || n_cams < 1 || n_pts < 0 || n_prev < 0 || !cams || !cam_src ||
      (n_pts && (!pts || !win_ids)) || (n_prev && !prev_ids))
    return ME_ERR_INVALID;
  if (a->mode >= 0 && (a->k1 < 0 || a->k1 >= n_cams - 1 || (a->mode == 1 && (a->k0 < 0 || a->k0 >= n_cams - 1))))
    return me_set_error(c, ME_ERR_INVALID, "me_vo_ba_chain: prediction cameras %d, %d outside the window's first %d",
                        a->k1, a->k0, n_cams - 1);
  auto* Q = (AsyncQueue*)c->ba_async;
  AsyncSolve* A = Q ? ba_chain_source(Q) : nullptr;
  if (!A) return me_set_error(c, ME_ERR_STATE, "me_vo_ba_chain: no BA solve to chain from");
  if (!A->P.dev) return me_set_error(c, ME_ERR_STATE, "me_vo_ba_chain: the previous solve is not device-resident");
  ME_HIP(c, hipSetDevice(c->device));
  hipLaunchKernelGGL(vo_chain_kernel, dim3(blocks(std::max(n_pts, 1), 256)), dim3(256), 48 * (size_t)n_cams, c->stream,
                     A->prob.cams, A->prob.pts, A->P.b.st, cams, n_cams, pts, n_pts, (const int*)cam_src,
                     (const int*)win_ids, (const int*)prev_ids, n_prev, (int)new_from, *a);
  return me_check_launch(c, "me_vo_ba_chain");
}

extern "C" int me_vo_window_submit(me_ctx* c, const me_vo_window* w, me_ba_problem* p, const me_ba_options* o) {
  me_range range_("me_vo_window_submit");
  if (!c || !w || !p || !o) return ME_ERR_INVALID;
  ME_HIP(c, hipSetDevice(c->device));
  if (w->stage_bytes) ME_HIP(c, hipMemcpyAsync(w->dev, w->stage, w->stage_bytes, hipMemcpyHostToDevice, c->stream));
  if (w->chain)
    ME_TRY(me_vo_ba_chain(c, p->cams, p->n_cams, p->pts, p->n_pts, w->cam_src, w->win_ids, w->prev_ids, w->n_prev,
                          w->new_from, &w->args));
  // (the problem's index arrays are the caller's device buffers, filled here)
  ME_TRY(me_ba_window_indices(c, w->frame, w->ids, p->n_obs, w->first_frame, w->win_ids, p->n_pts,
                              const_cast<int32_t*>(p->cam_idx), const_cast<int32_t*>(p->pt_idx)));
  return solve_async_impl(c, p, o, true);
}

extern "C" void me_ba_default_options(me_ba_options* o) {
  o->max_num_iterations = 50;
  o->function_tolerance = 1e-3;
  o->gradient_tolerance = 1e-10;
  o->parameter_tolerance = 1e-8;
  o->initial_trust_region_radius = 1e4;
  o->max_trust_region_radius = 1e16;
  o->min_trust_region_radius = 1e-32;
  o->min_lm_diagonal = 1e-6;
  o->max_lm_diagonal = 1e32;
  o->min_relative_decrease = 1e-3;
  o->max_num_consecutive_invalid_steps = 5;
  o->jacobi_scaling = 1;
}

extern "C" int me_ba_solve(me_ctx* c, me_ba_problem* p, const me_ba_options* o, me_ba_summary* s) {
  return solve_impl(c, p, o, nullptr, s);
}


#ifdef ME_SOLVE_TS
extern "C" int me_solve_ts(long long* out, int reset) {
  hipDeviceSynchronize();
  hipMemcpyFromSymbol(out, HIP_SYMBOL(g_solve_ts), sizeof(g_solve_ts));
  if (reset) {
    long long z[24] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(g_solve_ts), z, sizeof(z));
  }
  return 0;
}
#endif

extern "C" int me_ba_solve_comm(me_ctx* c, me_ba_problem* p, const me_ba_options* o, me_comm* comm,
                                me_ba_summary* s) {
  if (!c) return ME_ERR_INVALID;
  if (!comm) return me_set_error(c, ME_ERR_INVALID, "me_ba_solve_comm: null communicator");
  if (comm->ctx != c) return me_set_error(c, ME_ERR_INVALID, "me_ba_solve_comm: the communicator belongs to another ctx");
  return solve_impl(c, p, o, comm, s);
}

// ABI-v2 form: a callback without rank information (world 0: one gradient
// max-norm slot, reduced by its own max all-reduce)
// Per-exchange estimate (µs) of the packed all-reduce at `world` ranks: the
// one-rank RCCL exchange measured on MI355X (~14 µs each, bench
// sharded_ba.rccl_1rank, r03) is the floor; every doubling of the ring adds a
// latency step over xGMI (an estimate until the driver's 8-GPU line measures it).
extern "C" double me_ba_shard_exchange_us(int world) {
  if (world <= 1) return 0.0;
  double us = 14.0;
  for (int w = 2; w <= world; w *= 2) us += 4.0;
  return us;
}

extern "C" int me_ba_shard_worthwhile(long n_obs, int world, double xch_us) {
  if (world <= 1 || n_obs <= 0) return 0;
  if (!(xch_us > 0.0)) xch_us = me_ba_shard_exchange_us(world);
  auto t = [](double n) { return std::max(ME_SHARD_FLOOR_US, n * ME_SHARD_OBS_NS * 1e-3); };
  const double saved = t((double)n_obs) - t(std::ceil((double)n_obs / world));
  return saved > 2.0 * xch_us ? 1 : 0;
}

extern "C" int me_ba_solve_sharded(me_ctx* c, me_ba_problem* p, const me_ba_options* o, me_allreduce_fn ar,
                                   void* user, me_ba_summary* s) {
  if (!c) return ME_ERR_INVALID;
  if (!ar) return me_set_error(c, ME_ERR_INVALID, "me_ba_solve_sharded: null allreduce");
  me_comm m;
  m.ctx = c;
  m.world = 0;
  m.rank = 0;
  m.ar = ar;
  m.user = user;
  return solve_impl(c, p, o, &m, s);
}

extern "C" int me_ba_cost(me_ctx* c, const me_ba_problem* p, double* cost) {
  if (!c || !p) return ME_ERR_INVALID;
  ME_HIP(c, hipSetDevice(c->device));
  me_ba_options o;
  me_ba_default_options(&o);
  Plan P;
  ME_CHECK(c, p->mem == ME_HOST, "BA: evaluation helpers take host arrays");
  int rc = plan_build(c, p, &o, P, 0);
  if (rc < 0) return rc;
  std::vector<double> part(P.g.nblk_obs);
  if (P.g.od == 4)
    hipLaunchKernelGGL(cost_kernel<4>, dim3(P.g.nblk_obs), dim3(kBlock), 0, c->stream, P.g, P.b, 0, P.b.part);
  else
    hipLaunchKernelGGL(cost_kernel<2>, dim3(P.g.nblk_obs), dim3(kBlock), 0, c->stream, P.g, P.b, 0, P.b.part);
  ME_TRY(me_check_launch(c, "cost_kernel"));
  ME_HIP(c, hipMemcpyAsync(part.data(), P.b.part, 8 * part.size(), hipMemcpyDeviceToHost, c->stream));
  ME_HIP(c, hipStreamSynchronize(c->stream));
  double s = 0;
  for (double v : part) s += v;
  *cost = s;
  return ME_OK;
}

extern "C" int me_ba_evaluate(me_ctx* c, const me_ba_problem* p, double* res, double* Jc, double* Jp) {
  if (!c || !p) return ME_ERR_INVALID;
  ME_HIP(c, hipSetDevice(c->device));
  me_ba_options o;
  me_ba_default_options(&o);
  Plan P;
  ME_CHECK(c, p->mem == ME_HOST, "BA: evaluation helpers take host arrays");
  int rc = plan_build(c, p, &o, P, 0);
  if (rc < 0) return rc;
  const int no = P.g.no;
  void* d;
  const size_t od = P.g.od;
  ME_TRY(me_scratch(c, SLOT_GENERIC, 8 * 10 * od * (size_t)std::max(no, 1), &d));
  double* dres = (double*)d;
  double* djc = dres + od * (size_t)no;
  double* djp = djc + 6 * od * (size_t)no;
  if (od == 4)
    hipLaunchKernelGGL(eval_kernel<4>, dim3(blocks(no, kBlock)), dim3(kBlock), 0, c->stream, P.g, P.b, dres, djc, djp);
  else
    hipLaunchKernelGGL(eval_kernel<2>, dim3(blocks(no, kBlock)), dim3(kBlock), 0, c->stream, P.g, P.b, dres, djc, djp);
  ME_TRY(me_check_launch(c, "eval_kernel"));
  ME_HIP(c, hipMemcpyAsync(res, dres, 8 * od * (size_t)no, hipMemcpyDeviceToHost, c->stream));
  if (Jc) ME_HIP(c, hipMemcpyAsync(Jc, djc, 8 * 6 * od * (size_t)no, hipMemcpyDeviceToHost, c->stream));
  if (Jp) ME_HIP(c, hipMemcpyAsync(Jp, djp, 8 * 3 * od * (size_t)no, hipMemcpyDeviceToHost, c->stream));
  ME_HIP(c, hipStreamSynchronize(c->stream));
  return ME_OK;
}

extern "C" int me_ba_reduced_system(me_ctx* c, const me_ba_problem* p, double radius, double* S, double* bout) {
  if (!c || !p) return ME_ERR_INVALID;
  ME_HIP(c, hipSetDevice(c->device));
  me_ba_options o;
  me_ba_default_options(&o);
  o.initial_trust_region_radius = radius;
  Plan P;
  ME_CHECK(c, p->mem == ME_HOST, "BA: evaluation helpers take host arrays");
  int rc = plan_build(c, p, &o, P, 0);
  if (rc < 0) return rc;
  P.full_S = true;
  const Geo& g = P.g;
  ME_TRY(enqueue_linearize(P));
  ME_TRY(enqueue_assemble(P));
  std::vector<double> Sh((size_t)g.n6 * g.n6 + 2 * g.n6);
  if (g.m > 0)
    ME_HIP(c, hipMemcpyAsync(Sh.data(), P.b.S, 8 * Sh.size(), hipMemcpyDeviceToHost, c->stream));
  ME_HIP(c, hipStreamSynchronize(c->stream));
  const int n = g.n6;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double v = Sh[(size_t)i * n + j];
      if (i == j) v += std::min(std::max(Sh[(size_t)n * n + n + i], o.min_lm_diagonal), o.max_lm_diagonal) / radius;
      S[(size_t)i * n + j] = v;
    }
  for (int i = 0; i < n; ++i) bout[i] = Sh[(size_t)n * n + i];
  return ME_OK;
}

extern "C" int me_ba_covariance(me_ctx* c, const me_ba_problem* p, double* cov, int* ok) {
  if (!c || !p || !cov || !ok) return ME_ERR_INVALID;
  ME_HIP(c, hipSetDevice(c->device));
  me_ba_options o;
  me_ba_default_options(&o);
  o.jacobi_scaling = 0;                  // S unscaled: its inverse is the covariance directly
  o.initial_trust_region_radius = INFINITY;  // D / radius = 0: no LM damping
  Plan P;
  ME_CHECK(c, p->mem == ME_HOST, "BA: evaluation helpers take host arrays");
  int rc = plan_build(c, p, &o, P, 0);
  if (rc < 0) return rc;
  P.full_S = true;
  const Geo& g = P.g;
  hipLaunchKernelGGL(cov_prep_kernel, dim3(1), dim3(1), 0, c->stream, P.b);
  ME_TRY(enqueue_linearize(P));
  ME_TRY(enqueue_assemble(P));
  void* d;
  const size_t nx = (size_t)g.n6 * g.n6;
  ME_TRY(me_scratch(c, SLOT_GENERIC, 8 * (nx + 36 * (size_t)g.nc) + 64, &d));
  double* X = (double*)d;
  double* dcov = X + nx;
  int* dok = (int*)(dcov + 36 * (size_t)g.nc);
  hipLaunchKernelGGL(cov_kernel, dim3(1), dim3(kCovBlock), 0, c->stream, g, P.b, X, dcov, dok);
  ME_TRY(me_check_launch(c, "cov_kernel"));
  std::vector<double> h(36 * (size_t)g.nc);
  int hok = 0;
  ME_HIP(c, hipMemcpyAsync(h.data(), dcov, 8 * h.size(), hipMemcpyDeviceToHost, c->stream));
  ME_HIP(c, hipMemcpyAsync(&hok, dok, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  ME_HIP(c, hipStreamSynchronize(c->stream));
  *ok = hok;
  if (hok) std::memcpy(cov, h.data(), 8 * h.size());
  return ME_OK;
}

// BundleAdjuster<M>::initialiseObservations on the device
// (BundleAdjuster.h:354-376): for a window whose observations are stored by
// frame and track ID, camIdx = frame - first_frame and ptIdx = the track's
// index among the window's tracks (win_ids ascending: the order of the
// reference's observations vector).  One thread per observation, binary
// search over win_ids; an ID absent from the window gets -1 (the BA plan then
// reports bad input).
__global__ void window_indices_kernel(const int32_t* __restrict__ frame, const int32_t* __restrict__ ids, int n_obs,
                                      int f0, const int32_t* __restrict__ win_ids, int n_pts,
                                      int32_t* __restrict__ cam_idx, int32_t* __restrict__ pt_idx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_obs) return;
  const int32_t id = ids[i];
  int lo = 0, hi = n_pts;  // first win_ids[k] >= id
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (win_ids[mid] < id) lo = mid + 1;
    else hi = mid;
  }
  cam_idx[i] = frame[i] - f0;
  pt_idx[i] = (lo < n_pts && win_ids[lo] == id) ? lo : -1;
}

extern "C" int me_ba_window_indices(me_ctx* c, const int32_t* frame, const int32_t* ids, int n_obs, int first_frame,
                                    const int32_t* win_ids, int n_pts, int32_t* cam_idx, int32_t* pt_idx) {
  if (!c) return ME_ERR_INVALID;
  ME_CHECK(c, n_obs >= 0 && n_pts >= 0, "me_ba_window_indices: bad sizes");
  if (n_obs == 0) return ME_OK;
  ME_HIP(c, hipSetDevice(c->device));
  hipLaunchKernelGGL(window_indices_kernel, dim3(blocks(n_obs, kBlock)), dim3(kBlock), 0, c->stream, frame, ids, n_obs,
                     first_frame, win_ids, n_pts, cam_idx, pt_idx);
  return me_check_launch(c, "window_indices_kernel");
}

// Test hook (not part of the drop-in ABI): flags OR-ed into this ctx's camera
// solve diagnostics; 512 forces the fused-assembly wait to time out
// (tests/test_distributed.py: a hand-off timeout on one rank of a sharded solve),
// 1024 fails every camera solve (each LM step invalid: the solve ends with
// termination 2 after max_num_consecutive_invalid_steps), 2048 does that to
// every second solve queued on the ctx (tests/test_pipeline.py: the chained
// window start after a failed BA).
extern "C" int me_debug_solve_flags(me_ctx* c, int flags) {
  if (!c) return ME_ERR_INVALID;
  c->dbg_solve_flags = flags;
  c->dbg_solve_count = 0;
  return ME_OK;
}

extern "C" int me_debug_read(me_ctx* c, long long* out, int n) {
  if (!c || n < 0 || n > 16) return ME_ERR_INVALID;
  std::memcpy(out, c->dbg, 8 * (size_t)n);
  return ME_OK;
}

#ifdef ME_CAM_TS
extern "C" int me_cam_ts(long long* out, int reset) {
  unsigned long long h[8];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_cam_ts), sizeof h) != hipSuccess) return -1;
  for (int i = 0; i < 8; ++i) out[i] = (long long)h[i];
  if (reset) {
    const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_cam_ts), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
#endif

#ifdef ME_STEP_TS
extern "C" int me_step_ts(long long* out, int reset) {
  unsigned long long h[12];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_step_ts), sizeof h) != hipSuccess) return -1;
  for (int i = 0; i < 12; ++i) out[i] = (long long)h[i];
  if (reset) {
    const unsigned long long z[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_step_ts), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
#endif
