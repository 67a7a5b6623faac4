// vo.hip — frame-to-frame stereo visual odometry on MI355X.
//
// Replaces me::StereoVisualOdometry::process (src/vo/StereoVisualOdometry.cpp:34-92):
// project3D (:22-32), the RANSAC hypotheses (:58-71: random triples, signed-
// area gate, optimize on 3 matches, computeInliers), and the final optimize
// on the inliers (:78-91), with the reference's GN / LM loop (:165-283),
// Jacobian (:291-329) and reprojection (:116-141).  Design:
//  * the sampling stays on the host: it consumes a glibc-compatible rand()
//    stream owned by the context (the reference calls the unseeded process-
//    global rand(), :150), so the triples are exactly the reference's;
//  * every hypothesis that passes the area gate is optimised by one lane
//    (3 matches: 12 residuals, a 6x6 QR per step), all hypotheses at once;
//  * inlier counting: one workgroup per hypothesis over all matches;
//  * best = first hypothesis with the largest count (the reference keeps a
//    hypothesis only when it has strictly more inliers), its inlier list is
//    compacted in index order on the device;
//  * the final optimize runs in one workgroup: per step the 21 + 6 normal-
//    equation sums and the squared residual are block reductions in fixed
//    order, the 6x6 QR solve and the GN / LM control on lane 0.
// The reference's loop exit `while(!(k++ < stop))` (:277, SURVEY Appendix
// A-1) is kept as written: a loop the reference would never leave is cut at
// max_outer passes and reported (ME_ERR_STATE), never silently truncated.
#include "me_internal.hpp"

#include <cmath>
#include <vector>

namespace {

enum { VO_NO_STOP = 0, VO_SMALL_GRADIENT, VO_SMALL_INCREMENT, VO_MAX_ITERATIONS, VO_SMALL_DECREASE_FUNCTION,
       VO_SMALL_REPROJ_ERROR, VO_NO_CONVERGENCE };

struct VoCfg {
  int method, max_iter, max_outer, n;
  double e1, e2, e3, e4, thr2;
  double b, fu1, fv1, fu2, fv2, cu1, cu2, cv1, cv2;
  double init[6];
};

// Euler<double>::getR3 and the three angle derivatives (rotation_utils.cpp:25-91)
struct Trig {
  double cr, sr, cp, sp, cy, sy;
};
__device__ inline Trig trig(const double* s) {
  return {cos(s[0]), sin(s[0]), cos(s[1]), sin(s[1]), cos(s[2]), sin(s[2])};
}
// Tr = R4(state)^T with the translation column (:120-127); 12 entries (row 3 = 0 0 0 1)
__device__ inline void make_Tr(const double* s, double Tr[12]) {
  const Trig t = trig(s);
  const double R[9] = {t.cp * t.cy,                      t.cp * t.sy,                      -t.sp,
                       t.sp * t.sr * t.cy - t.cr * t.sy, t.sr * t.sp * t.sy + t.cr * t.cy, t.cp * t.sr,
                       t.cr * t.sp * t.cy + t.sr * t.sy, t.cr * t.sp * t.sy - t.sr * t.cy, t.cp * t.cr};
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) Tr[4 * i + j] = R[3 * j + i];
    Tr[4 * i + 3] = s[3 + i];
  }
}
// dR^T of the Euler derivatives (updateJacobian :295-297), dR[k][3i+j]
__device__ inline void make_dRt(const double* s, double dR[3][9]) {
  const Trig t = trig(s);
  const double a[9] = {0, 0, 0, t.cr * t.sp * t.cy + t.sr * t.sy, t.cr * t.sp * t.sy - t.sr * t.cy, t.cr * t.cp,
                       -t.sr * t.sp * t.cy + t.cr * t.sy, -t.sr * t.sp * t.sy - t.cr * t.cy, -t.sr * t.cp};
  const double b[9] = {-t.cy * t.sp,      -t.sy * t.sp,      -t.cp,
                       t.sr * t.cp * t.cy, t.sr * t.cp * t.sy, -t.sr * t.sp,
                       t.cr * t.cp * t.cy, t.cr * t.cp * t.sy, -t.cr * t.sp};
  const double c[9] = {-t.cp * t.sy, t.cp * t.cy, 0, -t.sr * t.sp * t.sy - t.cr * t.cy,
                       t.sr * t.sp * t.cy - t.cr * t.sy, 0, -t.cr * t.sp * t.sy + t.sr * t.cy,
                       t.cr * t.sp * t.cy + t.sr * t.sy, 0};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      dR[0][3 * i + j] = a[3 * j + i];
      dR[1][3 * i + j] = b[3 * j + i];
      dR[2][3 * i + j] = c[3 * j + i];
    }
}
__device__ inline void transform(const double Tr[12], const double* X, double p[4]) {
  for (int i = 0; i < 3; ++i) {
    double s = 0;
    for (int k = 0; k < 4; ++k) s += Tr[4 * i + k] * X[k];
    p[i] = s;
  }
  p[3] = X[3];
}
// residual block obs - reproject (:116-141, :180-185)
__device__ inline void residual1(const VoCfg& c, const double Tr[12], const double* X, const double* obs,
                                 double r[4]) {
  double p[4];
  transform(Tr, X, p);
  const double l0 = c.fu1 * p[0] + 0.0 * p[1] + c.cu1 * p[2] + 0.0 * p[3];
  const double l1 = 0.0 * p[0] + c.fv1 * p[1] + c.cv1 * p[2] + 0.0 * p[3];
  const double l2 = 0.0 * p[0] + 0.0 * p[1] + 1.0 * p[2] + 0.0 * p[3];
  const double r0 = c.fu2 * p[0] + 0.0 * p[1] + c.cu2 * p[2] + (-c.b * c.fu2) * p[3];
  const double r1 = 0.0 * p[0] + c.fv2 * p[1] + c.cv2 * p[2] + 0.0 * p[3];
  r[0] = obs[0] - l0 / l2;
  r[1] = obs[1] - l1 / l2;
  r[2] = obs[2] - r0 / l2;
  r[3] = obs[3] - r1 / l2;
}
// 6 x 4 Jacobian block (:305-327)
__device__ inline void jacobian1(const VoCfg& c, const double Tr[12], const double dR[3][9], const double* X,
                                 double J[6][4]) {
  double pn[4];
  transform(Tr, X, pn);
  pn[0] /= pn[3];
  pn[1] /= pn[3];
  pn[2] /= pn[3];
  const double z2 = pn[2] * pn[2];
  for (int j = 0; j < 6; ++j) {
    double d[3];
    if (j < 3) {
      for (int i = 0; i < 3; ++i) d[i] = dR[j][3 * i] * X[0] + dR[j][3 * i + 1] * X[1] + dR[j][3 * i + 2] * X[2];
    } else {
      d[0] = j == 3 ? 1.0 : 0.0;
      d[1] = j == 4 ? 1.0 : 0.0;
      d[2] = j == 5 ? 1.0 : 0.0;
    }
    J[j][0] = c.fu1 * (d[0] * pn[2] - pn[0] * d[2]) / z2;
    J[j][1] = c.fv1 * (d[1] * pn[2] - pn[1] * d[2]) / z2;
    J[j][2] = c.fu2 * (d[0] * pn[2] - (pn[0] - c.b) * d[2]) / z2;
    J[j][3] = c.fv2 * (d[1] * pn[2] - pn[1] * d[2]) / z2;
  }
}
// cv::solve(A, B, X, DECOMP_QR) on the 6x6 normal equations (Householder QR)
__device__ inline bool qr_solve6(const double* Ain, const double* B, double X[6]) {
  double A[36], b[6], amax = 0;
  for (int i = 0; i < 36; ++i) {
    A[i] = Ain[i];
    amax = fmax(amax, fabs(A[i]));
  }
  for (int i = 0; i < 6; ++i) b[i] = B[i];
  for (int k = 0; k < 6; ++k) {
    double nrm = 0;
    for (int i = k; i < 6; ++i) nrm += A[6 * i + k] * A[6 * i + k];
    nrm = sqrt(nrm);
    if (!(nrm > 1e-300)) return false;
    const double alpha = A[6 * k + k] > 0 ? -nrm : nrm;
    double v[6] = {0, 0, 0, 0, 0, 0};
    for (int i = k; i < 6; ++i) v[i] = A[6 * i + k];
    v[k] -= alpha;
    double vn = 0;
    for (int i = k; i < 6; ++i) vn += v[i] * v[i];
    if (vn > 0) {
      for (int j = k; j < 6; ++j) {
        double d = 0;
        for (int i = k; i < 6; ++i) d += v[i] * A[6 * i + j];
        const double f = 2.0 * d / vn;
        for (int i = k; i < 6; ++i) A[6 * i + j] -= f * v[i];
      }
      double d = 0;
      for (int i = k; i < 6; ++i) d += v[i] * b[i];
      const double f = 2.0 * d / vn;
      for (int i = k; i < 6; ++i) b[i] -= f * v[i];
    }
  }
  for (int i = 5; i >= 0; --i) {
    if (!(fabs(A[6 * i + i]) > 1e-14 * amax)) return false;
    double s = b[i];
    for (int j = i + 1; j < 6; ++j) s -= A[6 * i + j] * X[j];
    X[i] = s / A[6 * i + i];
  }
  return true;
}

// The inner GN / LM loop of optimize (:215-276) on one lane, given the normal
// equations; trial(xt) returns the squared residual at a trial state.  (The
// workgroup optimiser below runs the same steps with block-evaluated trials.)
struct StepCtl {
  double mu = 1e-20, vv = 2.0;
  int k = 0, stop = VO_NO_STOP;
};
template <class Trial>
__device__ inline void lm_inner(const VoCfg& c, StepCtl& s, double A[36], const double B[6], double rr, double* state,
                                Trial trial) {
  for (;;) {
    if (c.method == 1)
      for (int a = 0; a < 6; ++a) A[7 * a] += s.mu;
    double X[6];
    if (!qr_solve6(A, B, X)) {
      s.stop = VO_NO_CONVERGENCE;
      return;
    }
    double xn = 0, sn = 0;
    for (int a = 0; a < 6; ++a) {
      xn += X[a] * X[a];
      sn += state[a] * state[a];
    }
    if (sqrt(xn) <= c.e3 * sqrt(sn)) {
      s.stop = VO_SMALL_INCREMENT;
      return;
    }
    if (c.method == 0) {
      for (int a = 0; a < 6; ++a) state[a] += X[a];
      return;
    }
    double xt[6];
    for (int a = 0; a < 6; ++a) xt[a] = state[a] + X[a];
    const double rtt = trial(xt);
    double den = 0;
    for (int a = 0; a < 6; ++a) den += X[a] * (s.mu * X[a] + B[a]);
    const double rho = (rr - rtt) / den;
    if (rho > 0) {
      s.mu *= fmax(0.333, 1 - pow(2 * rho - 1, 3.0));
      s.vv = 2;
      if (pow(rr - rtt, 2.0) < c.e4 * rr) s.stop = VO_SMALL_DECREASE_FUNCTION;
      for (int a = 0; a < 6; ++a) state[a] = xt[a];
      return;
    }
    s.mu *= s.vv;
    const double v2 = 2 * s.vv;
    if (v2 <= s.vv) {
      s.stop = VO_NO_CONVERGENCE;
      return;
    }
    s.vv = v2;
  }
}
// pre-step tests and the LM mu initialisation (:187-213)
__device__ inline void pre_step(const VoCfg& c, StepCtl& s, const double A[36], const double B[6], double rr,
                                int rows) {
  if (rr / (double)rows < c.e1) s.stop = VO_SMALL_REPROJ_ERROR;
  double binf = 0;
  for (int a = 0; a < 6; ++a) binf = fmax(binf, fabs(B[a]));
  if (binf < c.e2) s.stop = VO_SMALL_GRADIENT;
  if (c.method == 1 && s.k == 0) {
    double mx = A[0];
    for (int a = 1; a < 6; ++a) mx = fmax(mx, A[7 * a]);
    s.mu = fmax(s.mu, mx);
    s.mu = 1e-5 * s.mu;
  }
}
// the loop exit as written: while(!(k++ < (max_iter ? stop : stop = MAX_ITERATIONS))) (:277)
__device__ inline bool loop_again(const VoCfg& c, StepCtl& s) {
  const int x = c.max_iter ? s.stop : (s.stop = VO_MAX_ITERATIONS);
  return !(s.k++ < x);
}

// project3D (:22-32) and updateObservations (:285-289) per match
__global__ void vo_prepare_kernel(const float* __restrict__ m, VoCfg c, double* __restrict__ X,
                                  double* __restrict__ obs) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= c.n) return;
  const float* f = m + 8 * i;
  const double d = (f[0] - c.cu1) - (f[2] - c.cu2);
  double x[4] = {(f[0] - c.cu1) * c.b, (f[1] - c.cv1) * c.b, c.fu1 * c.b, d > 0 ? d : 0.00001};
  x[0] /= x[3];
  x[1] /= x[3];
  x[2] /= x[3];
  x[3] /= x[3];
  for (int k = 0; k < 4; ++k) X[4 * i + k] = x[k];
  obs[4 * i + 0] = f[4];
  obs[4 * i + 1] = f[5];
  obs[4 * i + 2] = f[6];
  obs[4 * i + 3] = f[7];
}

// optimize (:165-283) on one hypothesis' 3 matches, one lane per hypothesis.
// ok[h]: 1 success, 0 failure, -2 the reference would not leave the loop.
__global__ void vo_hypo_kernel(const double* __restrict__ X, const double* __restrict__ obs,
                               const int* __restrict__ sel, int nh, VoCfg c, double* __restrict__ states,
                               int* __restrict__ ok) {
  const int h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= nh) return;
  const int s3[3] = {sel[3 * h], sel[3 * h + 1], sel[3 * h + 2]};
  double state[6];
  for (int a = 0; a < 6; ++a) state[a] = c.init[a];
  StepCtl s;
  int passes = 0, res = 0;
  for (;;) {
    if (++passes > c.max_outer) {
      res = -2;
      break;
    }
    double Tr[12], dR[3][9], r[12], A[36], B[6];
    make_Tr(state, Tr);
    make_dRt(state, dR);
    double rr = 0;
    for (int i = 0; i < 3; ++i) residual1(c, Tr, X + 4 * s3[i], obs + 4 * s3[i], r + 4 * i);
    for (int i = 0; i < 12; ++i) rr += r[i] * r[i];
    for (int i = 0; i < 36; ++i) A[i] = 0;
    for (int i = 0; i < 6; ++i) B[i] = 0;
    for (int i = 0; i < 3; ++i) {
      double J[6][4];
      jacobian1(c, Tr, dR, X + 4 * s3[i], J);
      for (int a = 0; a < 6; ++a) {
        for (int b = 0; b < 6; ++b)
          for (int q = 0; q < 4; ++q) A[6 * a + b] += J[a][q] * J[b][q];
        for (int q = 0; q < 4; ++q) B[a] += J[a][q] * r[4 * i + q];
      }
    }
    pre_step(c, s, A, B, rr, 12);
    lm_inner(c, s, A, B, rr, state, [&](const double* xt) {
      double Tt[12], rt[4], acc = 0;
      make_Tr(xt, Tt);
      for (int i = 0; i < 3; ++i) {
        residual1(c, Tt, X + 4 * s3[i], obs + 4 * s3[i], rt);
        for (int q = 0; q < 4; ++q) acc += rt[q] * rt[q];
      }
      return acc;
    });
    if (!loop_again(c, s)) {
      res = (s.stop == VO_NO_CONVERGENCE || s.stop == VO_MAX_ITERATIONS) ? 0 : 1;
      break;
    }
  }
  for (int a = 0; a < 6; ++a) states[6 * h + a] = state[a];
  ok[h] = res;
}

// computeInliers (:94-114) count per successful hypothesis, one workgroup each
constexpr int kVoBlock = 256;
__global__ __launch_bounds__(kVoBlock) void vo_count_kernel(const double* __restrict__ X,
                                                            const double* __restrict__ obs, VoCfg c,
                                                            const double* __restrict__ states,
                                                            const int* __restrict__ ok, int* __restrict__ counts) {
  __shared__ int red[kVoBlock / 64];
  const int h = blockIdx.x;
  if (ok[h] != 1) {
    if (threadIdx.x == 0) counts[h] = -1;
    return;
  }
  double Tr[12];
  make_Tr(states + 6 * h, Tr);
  int cnt = 0;
  for (int m = threadIdx.x; m < c.n; m += kVoBlock) {
    double r[4];
    residual1(c, Tr, X + 4 * m, obs + 4 * m, r);
    cnt += (r[0] * r[0] + r[1] * r[1] + r[2] * r[2] + r[3] * r[3] < c.thr2) ? 1 : 0;
  }
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_down(cnt, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < kVoBlock / 64; ++w) t += red[w];
    counts[h] = t;
  }
}

// best hypothesis (first strict maximum, as the sequential loop keeps it) and
// its inlier list in index order; without RANSAC every match is an inlier.
constexpr int kVoFinBlock = 1024;
__global__ __launch_bounds__(kVoFinBlock) void vo_select_kernel(const double* __restrict__ X,
                                                                const double* __restrict__ obs, VoCfg c,
                                                                const double* __restrict__ states,
                                                                const int* __restrict__ counts, int nh, int ransac,
                                                                int* __restrict__ list, int* __restrict__ nlist) {
  __shared__ int sbest;
  __shared__ int scan[kVoFinBlock];
  __shared__ int sbase;
  const int tid = threadIdx.x;
  if (tid == 0) {
    int best = -1, bc = 0;
    for (int h = 0; h < nh; ++h)
      if (counts[h] > bc) {
        bc = counts[h];
        best = h;
      }
    sbest = best;
    sbase = 0;
  }
  __syncthreads();
  const int best = sbest;
  if (ransac && best < 0) {
    if (tid == 0) *nlist = 0;
    return;
  }
  double Tr[12];
  if (ransac) make_Tr(states + 6 * best, Tr);
  for (int m0 = 0; m0 < c.n; m0 += kVoFinBlock) {
    const int m = m0 + tid;
    int f = 0;
    if (m < c.n) {
      if (!ransac) {
        f = 1;
      } else {
        double r[4];
        residual1(c, Tr, X + 4 * m, obs + 4 * m, r);
        f = (r[0] * r[0] + r[1] * r[1] + r[2] * r[2] + r[3] * r[3] < c.thr2) ? 1 : 0;
      }
    }
    scan[tid] = f;
    __syncthreads();
    for (int off = 1; off < kVoFinBlock; off <<= 1) {  // inclusive Hillis-Steele scan
      const int v = tid >= off ? scan[tid - off] : 0;
      __syncthreads();
      scan[tid] += v;
      __syncthreads();
    }
    if (f) list[sbase + scan[tid] - 1] = m;
    __syncthreads();
    if (tid == kVoFinBlock - 1) sbase += scan[tid];
    __syncthreads();
  }
  if (tid == 0) *nlist = sbase;
}

// final optimize (:78-91) on the inlier list, one workgroup
template <int NV>
__device__ inline void block_sum_fixed(double (&v)[NV], double* lds /* NV * 16 */) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    double x = v[i];
    for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
    if (lane == 0) lds[i * 16 + wave] = x;
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    double s = 0;
    for (int w = 0; w < kVoFinBlock / 64; ++w) s += lds[threadIdx.x * 16 + w];
    lds[NV * 16 + threadIdx.x] = s;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = lds[NV * 16 + i];
  __syncthreads();
}

__global__ __launch_bounds__(kVoFinBlock) void vo_refine_kernel(const double* __restrict__ X,
                                                                const double* __restrict__ obs, VoCfg c,
                                                                const int* __restrict__ list,
                                                                const int* __restrict__ nlist,
                                                                double* __restrict__ out /* state 6 | result */) {
  __shared__ double lds[28 * 16 + 28];
  __shared__ double sstate[6], strial[6];
  __shared__ int sflag;
  const int tid = threadIdx.x;
  const int n = *nlist;
  if (n < 6) {  // too few inliers: state stays at init, process() returns false (:84-91)
    if (tid < 6) out[tid] = c.init[tid];
    if (tid == 0) out[6] = 0.0;
    return;
  }
  if (tid < 6) sstate[tid] = c.init[tid];
  __syncthreads();
  StepCtl s;                   // lane 0
  double A[36], B[6], Xs[6];  // lane 0
  double rr = 0.0;
  for (int passes = 1;; ++passes) {
    double st[6];
    for (int a = 0; a < 6; ++a) st[a] = sstate[a];
    double Tr[12], dR[3][9];
    make_Tr(st, Tr);
    make_dRt(st, dR);
    double v[28];  // A upper triangle (21) | B (6) | r^T r
    for (int i = 0; i < 28; ++i) v[i] = 0;
    for (int q = tid; q < n; q += kVoFinBlock) {
      const int m = list[q];
      double r[4], J[6][4];
      residual1(c, Tr, X + 4 * m, obs + 4 * m, r);
      jacobian1(c, Tr, dR, X + 4 * m, J);
      int u = 0;
      for (int a = 0; a < 6; ++a)
        for (int b = a; b < 6; ++b, ++u)
          for (int k = 0; k < 4; ++k) v[u] += J[a][k] * J[b][k];
      for (int a = 0; a < 6; ++a)
        for (int k = 0; k < 4; ++k) v[21 + a] += J[a][k] * r[k];
      for (int k = 0; k < 4; ++k) v[27] += r[k] * r[k];
    }
    block_sum_fixed<28>(v, lds);
    if (tid == 0) {
      int u = 0;
      for (int a = 0; a < 6; ++a)
        for (int b = a; b < 6; ++b, ++u) A[6 * a + b] = A[6 * b + a] = v[u];
      for (int a = 0; a < 6; ++a) B[a] = v[21 + a];
      rr = v[27];
      pre_step(c, s, A, B, rr, 4 * n);
    }
    // inner loop (:215-276), block-synchronous: lane 0 decides, the block
    // evaluates the trial costs of the LM branch
    for (;;) {
      if (tid == 0) {
        sflag = 1;  // leave the inner loop unless a trial is requested
        if (c.method == 1)
          for (int a = 0; a < 6; ++a) A[7 * a] += s.mu;
        if (!qr_solve6(A, B, Xs)) {
          s.stop = VO_NO_CONVERGENCE;
        } else {
          double xn = 0, sn = 0;
          for (int a = 0; a < 6; ++a) {
            xn += Xs[a] * Xs[a];
            sn += st[a] * st[a];
          }
          if (sqrt(xn) <= c.e3 * sqrt(sn)) {
            s.stop = VO_SMALL_INCREMENT;
          } else if (c.method == 0) {
            for (int a = 0; a < 6; ++a) sstate[a] = st[a] + Xs[a];
          } else {
            for (int a = 0; a < 6; ++a) strial[a] = st[a] + Xs[a];
            sflag = 0;
          }
        }
      }
      __syncthreads();
      if (sflag) break;
      double xt[6], Tt[12], acc[1] = {0.0};
      for (int a = 0; a < 6; ++a) xt[a] = strial[a];
      make_Tr(xt, Tt);
      for (int q = tid; q < n; q += kVoFinBlock) {
        const int m = list[q];
        double r[4];
        residual1(c, Tt, X + 4 * m, obs + 4 * m, r);
        for (int k = 0; k < 4; ++k) acc[0] += r[k] * r[k];
      }
      block_sum_fixed<1>(acc, lds);
      if (tid == 0) {
        const double rtt = acc[0];
        double den = 0;
        for (int a = 0; a < 6; ++a) den += Xs[a] * (s.mu * Xs[a] + B[a]);
        const double rho = (rr - rtt) / den;
        sflag = 1;
        if (rho > 0) {
          s.mu *= fmax(0.333, 1 - pow(2 * rho - 1, 3.0));
          s.vv = 2;
          if (pow(rr - rtt, 2.0) < c.e4 * rr) s.stop = VO_SMALL_DECREASE_FUNCTION;
          for (int a = 0; a < 6; ++a) sstate[a] = xt[a];
        } else {
          s.mu *= s.vv;
          const double v2 = 2 * s.vv;
          if (v2 <= s.vv) s.stop = VO_NO_CONVERGENCE;
          else {
            s.vv = v2;
            sflag = 0;  // retry with the larger mu; A keeps what was added (:218)
          }
        }
      }
      __syncthreads();
      if (sflag) break;
    }
    if (tid == 0) {
      const bool again = loop_again(c, s);
      sflag = again && passes < c.max_outer ? 1 : 0;
      if (!sflag)
        out[6] = again ? -2.0 : ((s.stop == VO_NO_CONVERGENCE || s.stop == VO_MAX_ITERATIONS) ? 0.0 : 1.0);
    }
    __syncthreads();
    if (!sflag) break;
  }
  if (tid < 6) out[tid] = sstate[tid];
}

// glibc random_r (TYPE_3: degree 31, separation 3) seeded like srandom_r, so
// an unseeded context draws exactly what the reference's unseeded rand() does.
void GlibcRand_seed(int32_t st[31], int& f, int& r, unsigned seed) {
  if (seed == 0) seed = 1;
  int32_t word = (int32_t)seed;
  st[0] = word;
  for (int i = 1; i < 31; ++i) {
    const long hi = word / 127773, lo = word % 127773;
    word = (int32_t)(16807 * lo - 2836 * hi);
    if (word < 0) word += 2147483647;
    st[i] = word;
  }
  f = 3;
  r = 0;
}
int GlibcRand_next(int32_t st[31], int& f, int& r) {
  const uint32_t v = (uint32_t)st[f] + (uint32_t)st[r];
  st[f] = (int32_t)v;
  const int res = (int)(v >> 1);
  if (++f >= 31) {
    f = 0;
    ++r;
  } else if (++r >= 31) {
    r = 0;
  }
  return res;
}


// New-feature cells of the windowed VO loop (pipeline.new_cells, restated on
// the device so the tracked and the new-feature matching share one round
// trip): a tracked feature k is good iff status_k == 1, it lies inside the
// feature margin and its stereo match held (ok_k); a good feature occupies
// grid cell (trunc((u - margin) / cw), trunc((v - margin) / ch)), clamped,
// in FP64; the first max(0, n_feats - #good) empty cells in ascending order
// get a new feature at margin + (cell + 0.5 + jitter(t, cell)) * (cw, ch),
// rounded to float; lo = d_min.  One workgroup.
constexpr int kCellBlock = 1024, kMaxCells = 65536;
__global__ __launch_bounds__(kCellBlock) void vo_cells_kernel(const float* __restrict__ uv,
                                                              const uint8_t* __restrict__ status,
                                                              const uint8_t* __restrict__ ok, int n, int width,
                                                              int height, float margin, int nx, int ny, double cw,
                                                              double ch, int n_feats, unsigned t, int d_min,
                                                              float* __restrict__ out_uv, int32_t* __restrict__ out_lo,
                                                              int32_t* __restrict__ out_count) {
  __shared__ uint32_t occ[kMaxCells / 32];
  __shared__ int wsum[kCellBlock / 64];
  __shared__ int ngood;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int ncell = nx * ny;
  for (int i = tid; i < (ncell + 31) / 32; i += kCellBlock) occ[i] = 0u;
  if (tid == 0) ngood = 0;
  __syncthreads();
  int cnt = 0;
  for (int k = tid; k < n; k += kCellBlock) {
    const float u = uv[2 * k], v = uv[2 * k + 1];
    const bool good = status[k] == 1 && ok[k] != 0 && u >= margin && u < (float)width - margin && v >= margin &&
                      v < (float)height - margin;
    if (!good) continue;
    ++cnt;
    const int cx = min(max((int)(((double)u - (double)margin) / cw), 0), nx - 1);
    const int cy = min(max((int)(((double)v - (double)margin) / ch), 0), ny - 1);
    const int cell = cy * nx + cx;
    atomicOr(&occ[cell >> 5], 1u << (cell & 31));
  }
  atomicAdd(&ngood, cnt);
  __syncthreads();
  const int want = max(0, n_feats - ngood);
  // empty cells in ascending order: contiguous chunk per thread, block scan of the counts
  const int chunk = (ncell + kCellBlock - 1) / kCellBlock;
  const int c0 = min(ncell, tid * chunk), c1 = min(ncell, c0 + chunk);
  int e = 0;
  for (int c = c0; c < c1; ++c) e += ((occ[c >> 5] >> (c & 31)) & 1u) ? 0 : 1;
  int x = e;
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int k = 0; k < kCellBlock / 64; ++k) {
      const int v = wsum[k];
      wsum[k] = acc;
      acc += v;
    }
    *out_count = min(want, acc);
  }
  __syncthreads();
  int r = wsum[wv] + x - e;
  for (int c = c0; c < c1 && r < want; ++c) {
    if ((occ[c >> 5] >> (c & 31)) & 1u) continue;
    // pipeline._cell_jitter: 32-bit hash of (cell, t), two 16-bit fractions * 0.6 - 0.3
    uint32_t h = (uint32_t)c * 2654435761u + t * 40503u;
    h ^= h >> 15;
    h *= 2246822519u;
    const double ja = (double)(h & 0xFFFFu) / 65536.0 * 0.6 - 0.3;
    const double jb = (double)((h >> 16) & 0xFFFFu) / 65536.0 * 0.6 - 0.3;
    const double px = (double)margin + (((double)(c % nx) + 0.5) + ja) * cw;
    const double py = (double)margin + (((double)(c / nx) + 0.5) + jb) * ch;
    out_uv[2 * r] = (float)px;
    out_uv[2 * r + 1] = (float)py;
    out_lo[r] = d_min;
    ++r;
  }
}

}  // namespace

void me_rand_seed(me_ctx* c, unsigned seed) {
  GlibcRand_seed(c->rand_st, c->rand_f, c->rand_r, seed);
  for (int i = 0; i < 310; ++i) GlibcRand_next(c->rand_st, c->rand_f, c->rand_r);
  c->rand_init = true;
}

extern "C" void me_vo_default_params(me_vo_params* p) {
  // VisualOdometry::parameters() (VisualOdometry.h:32) and StereoVisualOdometry::parameters() (StereoVisualOdometry.h:32)
  p->method = 0;
  p->step_size = 1.0;
  p->eps = 1e-9;
  p->e1 = 1e-3;
  p->e2 = 1e-12;
  p->e3 = 1e-12;
  p->e4 = 1e-15;
  p->max_iter = 100;
  p->nb_fixed_frames = 2;
  p->ransac = 1;
  p->n_ransac = 200;
  p->inlier_threshold = 2.0;
  p->baseline = 1.0;
  p->weighting = 0;
  p->fu1 = p->fv1 = p->fu2 = p->fv2 = 1.0;
  p->cu1 = p->cu2 = p->cv1 = p->cv2 = 0.0;
}

extern "C" int me_vo_srand(me_ctx* c, unsigned seed) {
  if (!c) return ME_ERR_INVALID;
  me_rand_seed(c, seed);
  return ME_OK;
}

extern "C" int me_vo_rand(me_ctx* c, int* out) {
  if (!c || !out) return ME_ERR_INVALID;
  if (!c->rand_init) me_rand_seed(c, 1);
  *out = GlibcRand_next(c->rand_st, c->rand_f, c->rand_r);
  return ME_OK;
}

extern "C" int me_vo_process(me_ctx* c, const float* matches, int n, const double* init6, const me_vo_params* p,
                             int max_outer, double* motion, double* state, double* pts3d, int* inliers,
                             int* n_inliers, int* ok) {
  me_range range_("me_vo_process");
  if (!c || !p || !motion || !n_inliers || !ok) return ME_ERR_INVALID;
  ME_CHECK(c, n >= 0 && (n == 0 || matches), "me_vo_process: bad matches");
  ME_CHECK(c, p->method == 0 || p->method == 1, "me_vo_process: method must be GN (0) or LM (1)");
  ME_CHECK(c, max_outer > 0, "me_vo_process: max_outer must be positive");
  ME_HIP(c, hipSetDevice(c->device));
  if (!c->rand_init) me_rand_seed(c, 1);
  VoCfg cfg;
  cfg.method = p->method;
  cfg.max_iter = p->max_iter;
  cfg.max_outer = max_outer;
  cfg.n = n;
  cfg.e1 = p->e1;
  cfg.e2 = p->e2;
  cfg.e3 = p->e3;
  cfg.e4 = p->e4;
  cfg.thr2 = p->inlier_threshold * p->inlier_threshold;
  cfg.b = p->baseline;
  cfg.fu1 = p->fu1;
  cfg.fv1 = p->fv1;
  cfg.fu2 = p->fu2;
  cfg.fv2 = p->fv2;
  cfg.cu1 = p->cu1;
  cfg.cu2 = p->cu2;
  cfg.cv1 = p->cv1;
  cfg.cv2 = p->cv2;
  for (int a = 0; a < 6; ++a) cfg.init[a] = init6 ? init6[a] : 0.0;
  *n_inliers = 0;
  *ok = 0;
  auto motion_of = [&](const double* s) {  // getMotion (:331-342)
    const double cr = std::cos(s[0]), sr = std::sin(s[0]), cp = std::cos(s[1]), sp = std::sin(s[1]);
    const double cy = std::cos(s[2]), sy = std::sin(s[2]);
    const double R[9] = {cp * cy, cp * sy, -sp, sp * sr * cy - cr * sy, sr * sp * sy + cr * cy, cp * sr,
                         cr * sp * cy + sr * sy, cr * sp * sy - sr * cy, cp * cr};
    for (int i = 0; i < 3; ++i) {
      for (int j = 0; j < 3; ++j) motion[4 * i + j] = R[3 * j + i];
      motion[4 * i + 3] = s[3 + i];
    }
    motion[12] = motion[13] = motion[14] = 0.0;
    motion[15] = 1.0;
    if (state)
      for (int a = 0; a < 6; ++a) state[a] = s[a];
  };
  if (n < 6) {  // (:41-42): nothing is computed
    motion_of(cfg.init);
    return ME_OK;
  }
  // RANSAC triples on the host: selectRandomIndices (:143-163) and the
  // float signed-area gate (:63)
  std::vector<int> sel;
  if (p->ransac) {
    for (int it = 0; it < p->n_ransac; ++it) {
      int s3[3], k = 0;
      while (k < 3) {
        const int idx = GlibcRand_next(c->rand_st, c->rand_f, c->rand_r) % n;
        bool exists = false;
        for (int j = 0; j < k; ++j) exists = exists || s3[j] == idx;
        if (!exists) s3[k++] = idx;
      }
      const float* f0 = matches + 8 * s3[0];
      const float* f1 = matches + 8 * s3[1];
      const float* f2 = matches + 8 * s3[2];
      const float area = (f0[4] * (f1[5] - f2[5]) + f1[4] * (f2[5] - f0[5]) + f2[4] * (f0[5] - f1[5])) / 2;
      if (area > 1000)
        for (int j = 0; j < 3; ++j) sel.push_back(s3[j]);
    }
  }
  const int nh = (int)sel.size() / 3;
  // device scratch: matches | X | obs | sel | states | ok | counts | list | nlist | out
  auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t bM = up(32 * (size_t)n), bX = up(32 * (size_t)n), bO = up(32 * (size_t)n);
  const size_t bS = up(12 * (size_t)std::max(nh, 1)), bSt = up(48 * (size_t)std::max(nh, 1));
  const size_t bOk = up(4 * (size_t)std::max(nh, 1)), bC = bOk, bL = up(4 * (size_t)n), bN = 256, bOut = 256;
  void* d;
  ME_TRY(me_scratch(c, SLOT_VO, bM + bX + bO + bS + bSt + bOk + bC + bL + bN + bOut, &d));
  char* base = (char*)d;
  float* dm = (float*)base;
  double* dX = (double*)(base + bM);
  double* dobs = (double*)(base + bM + bX);
  int* dsel = (int*)(base + bM + bX + bO);
  double* dst = (double*)(base + bM + bX + bO + bS);
  int* dok = (int*)(base + bM + bX + bO + bS + bSt);
  int* dcnt = (int*)(base + bM + bX + bO + bS + bSt + bOk);
  int* dlist = (int*)(base + bM + bX + bO + bS + bSt + bOk + bC);
  int* dnl = (int*)(base + bM + bX + bO + bS + bSt + bOk + bC + bL);
  double* dout = (double*)(base + bM + bX + bO + bS + bSt + bOk + bC + bL + bN);
  hipStream_t s = c->stream;
  ME_HIP(c, hipMemcpyAsync(dm, matches, 32 * (size_t)n, hipMemcpyHostToDevice, s));
  if (nh) ME_HIP(c, hipMemcpyAsync(dsel, sel.data(), 12 * (size_t)nh, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(vo_prepare_kernel, dim3((n + 255) / 256), dim3(256), 0, s, dm, cfg, dX, dobs);
  if (nh) {
    hipLaunchKernelGGL(vo_hypo_kernel, dim3((nh + 63) / 64), dim3(64), 0, s, dX, dobs, dsel, nh, cfg, dst, dok);
    hipLaunchKernelGGL(vo_count_kernel, dim3(nh), dim3(kVoBlock), 0, s, dX, dobs, cfg, dst, dok, dcnt);
  }
  hipLaunchKernelGGL(vo_select_kernel, dim3(1), dim3(kVoFinBlock), 0, s, dX, dobs, cfg, dst, dcnt, nh,
                     p->ransac ? 1 : 0, dlist, dnl);
  hipLaunchKernelGGL(vo_refine_kernel, dim3(1), dim3(kVoFinBlock), 0, s, dX, dobs, cfg, dlist, dnl, dout);
  ME_TRY(me_check_launch(c, "stereo VO"));
  std::vector<int> hok(std::max(nh, 1));
  double hout[7];
  int hnl = 0;
  if (nh) ME_HIP(c, hipMemcpyAsync(hok.data(), dok, 4 * (size_t)nh, hipMemcpyDeviceToHost, s));
  ME_HIP(c, hipMemcpyAsync(&hnl, dnl, 4, hipMemcpyDeviceToHost, s));
  ME_HIP(c, hipMemcpyAsync(hout, dout, sizeof(hout), hipMemcpyDeviceToHost, s));
  ME_HIP(c, hipStreamSynchronize(s));
  for (int h = 0; h < nh; ++h)
    if (hok[h] == -2)
      return me_set_error(c, ME_ERR_STATE, "me_vo_process: hypothesis %d never leaves the optimisation loop "
                                          "(StereoVisualOdometry.cpp:277; cut after %d passes)", h, max_outer);
  if (hout[6] == -2.0)
    return me_set_error(c, ME_ERR_STATE, "me_vo_process: the final optimisation never leaves its loop "
                                         "(StereoVisualOdometry.cpp:277; cut after %d passes)", max_outer);
  if (inliers && hnl > 0) ME_HIP(c, hipMemcpy(inliers, dlist, 4 * (size_t)hnl, hipMemcpyDeviceToHost));
  if (pts3d) ME_HIP(c, hipMemcpy(pts3d, dX, 32 * (size_t)n, hipMemcpyDeviceToHost));
  *n_inliers = hnl;
  *ok = hout[6] == 1.0 ? 1 : 0;
  motion_of(hout);
  return ME_OK;
}

extern "C" int me_vo_new_cells(me_ctx* c, const float* uv, const uint8_t* status, const uint8_t* ok, int n, int width,
                               int height, float margin, int nx, int ny, double cw, double ch, int n_feats, int t,
                               int d_min, float* out_uv, int32_t* out_lo, int32_t* out_count) {
  me_range range_("me_vo_new_cells");
  if (!c) return ME_ERR_INVALID;
  ME_CHECK(c, n >= 0 && nx > 0 && ny > 0 && (long)nx * ny <= kMaxCells && n_feats >= 0 && cw > 0 && ch > 0 &&
                  width > 0 && height > 0,
           "me_vo_new_cells: bad sizes (at most %d cells)", kMaxCells);
  ME_HIP(c, hipSetDevice(c->device));
  hipLaunchKernelGGL(vo_cells_kernel, dim3(1), dim3(kCellBlock), 0, c->stream, uv, status, ok, n, width, height, margin,
                     nx, ny, cw, ch, n_feats, (unsigned)t, d_min, out_uv, out_lo, out_count);
  return me_check_launch(c, "vo_cells_kernel");
}
