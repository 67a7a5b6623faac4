// oracle/vo.cpp — TEST INFRASTRUCTURE: CPU restatement of the frame-to-frame
// stereo visual odometry me::StereoVisualOdometry (src/vo/StereoVisualOdometry.cpp:10-342,
// include/MotionEstimation/vo/StereoVisualOdometry.h:24-33, VisualOdometry.h:19-33)
// with Euler<double> R and dR/d(angle) from src/core/rotation_utils.cpp:24-91
// and the StopCondition enum of include/MotionEstimation/core/rotation_utils.h:20.
//
// OpenCV pieces restated, not linked: Matx products (left-to-right sums),
// cv::norm (L2, NORM_INF), cv::solve(..., DECOMP_QR) as a Householder QR
// (OpenCV's own QR: agreement to rounding, not bit for bit).  glibc rand()
// (unseeded in the reference, :150) is the caller's pre-drawn sequence so the
// kernels and this restatement consume identical values.  The reference's
// loop-exit quirk (`while(!(k++ < stop))`, :277) is kept
// as written; max_outer bounds it and the call returns -2 where the reference
// would spin forever.  Parity unpinned (see oracle.h).
#include <cmath>
#include <cstring>
#include <vector>

#include "oracle.h"

namespace {

enum Stop { NO_STOP = 0, SMALL_GRADIENT, SMALL_INCREMENT, MAX_ITERATIONS, SMALL_DECREASE_FUNCTION, SMALL_REPROJ_ERROR,
            NO_CONVERGENCE };

struct Trig {
  double cr, sr, cp, sp, cy, sy;
};
Trig trig(const double s[3]) {
  return {std::cos(s[0]), std::sin(s[0]), std::cos(s[1]), std::sin(s[1]), std::cos(s[2]), std::sin(s[2])};
}
// Euler::getR3 / getR4 (rotation_utils.cpp:25-45), row-major
void euler_R(const Trig& t, double R[9]) {
  R[0] = t.cp * t.cy;                      R[1] = t.cp * t.sy;                      R[2] = -t.sp;
  R[3] = t.sp * t.sr * t.cy - t.cr * t.sy; R[4] = t.sr * t.sp * t.sy + t.cr * t.cy; R[5] = t.cp * t.sr;
  R[6] = t.cr * t.sp * t.cy + t.sr * t.sy; R[7] = t.cr * t.sp * t.sy - t.sr * t.cy; R[8] = t.cp * t.cr;
}
// Euler::getdRdr / getdRdp / getdRdy (rotation_utils.cpp:58-91)
void euler_dR(const Trig& t, double dr[9], double dp[9], double dy[9]) {
  dr[0] = 0;                                dr[1] = 0;                                dr[2] = 0;
  dr[3] = t.cr * t.sp * t.cy + t.sr * t.sy; dr[4] = t.cr * t.sp * t.sy - t.sr * t.cy; dr[5] = t.cr * t.cp;
  dr[6] = -t.sr * t.sp * t.cy + t.cr * t.sy; dr[7] = -t.sr * t.sp * t.sy - t.cr * t.cy; dr[8] = -t.sr * t.cp;
  dp[0] = -t.cy * t.sp;      dp[1] = -t.sy * t.sp;      dp[2] = -t.cp;
  dp[3] = t.sr * t.cp * t.cy; dp[4] = t.sr * t.cp * t.sy; dp[5] = -t.sr * t.sp;
  dp[6] = t.cr * t.cp * t.cy; dp[7] = t.cr * t.cp * t.sy; dp[8] = -t.cr * t.sp;
  dy[0] = -t.cp * t.sy;                      dy[1] = t.cp * t.cy;                      dy[2] = 0;
  dy[3] = -t.sr * t.sp * t.sy - t.cr * t.cy; dy[4] = t.sr * t.sp * t.cy - t.cr * t.sy; dy[5] = 0;
  dy[6] = -t.cr * t.sp * t.sy + t.sr * t.cy; dy[7] = t.cr * t.sp * t.cy + t.sr * t.sy; dy[8] = 0;
}

struct VO {
  const oracle_vo_params* p;
  int n;
  std::vector<double> X;    // project3D: 4 per match, normalised homogeneous (:22-32)
  std::vector<double> obs;  // updateObservations: f3, f4 per match (:285-289)
  double state[6];
};

// Tr = R4(state)^T with the translation column (:120-127)
void make_Tr(const double s[6], double Tr[16]) {
  double R[9];
  euler_R(trig(s), R);
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) Tr[4 * i + j] = R[3 * j + i];
    Tr[4 * i + 3] = s[3 + i];
  }
  Tr[12] = Tr[13] = Tr[14] = 0.0;
  Tr[15] = 1.0;
}

// reproject (:116-141) of one 3D point: left and right image points
void reproject1(const oracle_vo_params* p, const double Tr[16], const double* X, double out[4]) {
  double pt[4];
  for (int i = 0; i < 4; ++i) {
    double s = 0;
    for (int k = 0; k < 4; ++k) s += Tr[4 * i + k] * X[k];
    pt[i] = s;
  }
  const double P1[12] = {p->fu1, 0, p->cu1, 0, 0, p->fv1, p->cv1, 0, 0, 0, 1, 0};
  const double P2[12] = {p->fu2, 0, p->cu2, -p->baseline * p->fu2, 0, p->fv2, p->cv2, 0, 0, 0, 1, 0};
  double l[3], r[3];
  for (int i = 0; i < 3; ++i) {
    double a = 0, b = 0;
    for (int k = 0; k < 4; ++k) {
      a += P1[4 * i + k] * pt[k];
      b += P2[4 * i + k] * pt[k];
    }
    l[i] = a;
    r[i] = b;
  }
  out[0] = l[0] / l[2];
  out[1] = l[1] / l[2];
  out[2] = r[0] / r[2];
  out[3] = r[1] / r[2];
}

// residual block of match m: obs - pred (:180-185)
void residual1(const VO& v, const double Tr[16], int m, double r[4]) {
  double pr[4];
  reproject1(v.p, Tr, &v.X[4 * m], pr);
  for (int k = 0; k < 4; ++k) r[k] = v.obs[4 * m + k] - pr[k];
}

// updateJacobian (:291-329): 6 x 4 block of match m (row j = state element)
void jacobian1(const VO& v, const double Tr[16], const double dR[3][9], int m, double J[6][4]) {
  const oracle_vo_params* p = v.p;
  const double* X = &v.X[4 * m];
  double pn[4];
  for (int i = 0; i < 4; ++i) {
    double s = 0;
    for (int k = 0; k < 4; ++k) s += Tr[4 * i + k] * X[k];
    pn[i] = s;
  }
  pn[0] /= pn[3];
  pn[1] /= pn[3];
  pn[2] /= pn[3];
  pn[3] /= pn[3];
  for (int j = 0; j < 6; ++j) {
    double d[3];
    if (j < 3) {
      for (int i = 0; i < 3; ++i) d[i] = dR[j][3 * i] * X[0] + dR[j][3 * i + 1] * X[1] + dR[j][3 * i + 2] * X[2];
    } else {
      d[0] = j == 3;
      d[1] = j == 4;
      d[2] = j == 5;
    }
    const double z2 = pn[2] * pn[2];
    J[j][0] = p->fu1 * (d[0] * pn[2] - pn[0] * d[2]) / z2;
    J[j][1] = p->fv1 * (d[1] * pn[2] - pn[1] * d[2]) / z2;
    J[j][2] = p->fu2 * (d[0] * pn[2] - (pn[0] - p->baseline) * d[2]) / z2;
    J[j][3] = p->fv2 * (d[1] * pn[2] - pn[1] * d[2]) / z2;
  }
}

// dR^T of the three Euler derivatives (updateJacobian :295-297)
void dRt(const double s[6], double dR[3][9]) {
  double a[9], b[9], c[9];
  euler_dR(trig(s), a, b, c);
  const double* src[3] = {a, b, c};
  for (int k = 0; k < 3; ++k)
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) dR[k][3 * i + j] = src[k][3 * j + i];
}

// cv::solve(A, B, X, DECOMP_QR) for the 6x6 normal equations (Householder QR)
bool qr_solve6(const double Ain[36], const double B[6], double X[6]) {
  double A[36], b[6];
  std::memcpy(A, Ain, sizeof(A));
  std::memcpy(b, B, sizeof(b));
  double amax = 0;
  for (double a : A) amax = std::fmax(amax, std::fabs(a));
  for (int k = 0; k < 6; ++k) {
    double nrm = 0;
    for (int i = k; i < 6; ++i) nrm += A[6 * i + k] * A[6 * i + k];
    nrm = std::sqrt(nrm);
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
    if (!(std::fabs(A[6 * i + i]) > 1e-14 * amax)) return false;
    double s = b[i];
    for (int j = i + 1; j < 6; ++j) s -= A[6 * i + j] * X[j];
    X[i] = s / A[6 * i + i];
  }
  return true;
}

double sumsq(const std::vector<double>& r) {
  double s = 0;
  for (double x : r) s += x * x;
  return s;
}

// optimize (:165-283).  Returns true/false as the reference; *hang when the
// reference's loop would not terminate within max_outer passes.
bool optimize(VO& v, const std::vector<int>& sel, int max_outer, bool* hang) {
  const oracle_vo_params* p = v.p;
  if (sel.size() < 3) return false;
  const int n = (int)sel.size();
  int k = 0;
  double vv = 2, tau = 1e-5, mu = 1e-20;
  const double abs_tol = p->e1, grad_tol = p->e2, incr_tol = p->e3, rel_tol = p->e4;
  int stop = NO_STOP;
  std::vector<double> r(4 * n), rt(4 * n);
  int passes = 0;
  do {
    if (++passes > max_outer) {
      *hang = true;
      return false;
    }
    double Tr[16], dR[3][9];
    make_Tr(v.state, Tr);
    dRt(v.state, dR);
    for (int i = 0; i < n; ++i) residual1(v, Tr, sel[i], &r[4 * i]);
    const double rr = sumsq(r);
    if (rr / (4.0 * n) < abs_tol) stop = SMALL_REPROJ_ERROR;
    double A[36] = {0}, B[6] = {0};
    for (int i = 0; i < n; ++i) {
      double J[6][4];
      jacobian1(v, Tr, dR, sel[i], J);
      for (int a = 0; a < 6; ++a) {
        for (int b = 0; b < 6; ++b)
          for (int c = 0; c < 4; ++c) A[6 * a + b] += J[a][c] * J[b][c];
        for (int c = 0; c < 4; ++c) B[a] += J[a][c] * r[4 * i + c];
      }
    }
    double binf = 0;
    for (double x : B) binf = std::fmax(binf, std::fabs(x));
    if (binf < grad_tol) stop = SMALL_GRADIENT;
    if (p->method == 1 && k == 0) {
      double mx = A[0];
      for (int a = 1; a < 6; ++a) mx = std::fmax(mx, A[7 * a]);
      mu = std::fmax(mu, mx);
      mu = tau * mu;
    }
    for (;;) {
      if (p->method == 1)
        for (int a = 0; a < 6; ++a) A[7 * a] += mu;
      double X[6];
      if (qr_solve6(A, B, X)) {
        double xn = 0, sn = 0;
        for (int a = 0; a < 6; ++a) {
          xn += X[a] * X[a];
          sn += v.state[a] * v.state[a];
        }
        if (std::sqrt(xn) <= incr_tol * std::sqrt(sn)) {
          stop = SMALL_INCREMENT;
          break;
        }
        if (p->method == 0) {
          for (int a = 0; a < 6; ++a) v.state[a] += X[a];
          break;
        }
        double xt[6];
        for (int a = 0; a < 6; ++a) xt[a] = v.state[a] + X[a];
        double Trt[16];
        make_Tr(xt, Trt);
        for (int i = 0; i < n; ++i) residual1(v, Trt, sel[i], &rt[4 * i]);
        const double rtt = sumsq(rt);
        double den = 0;
        for (int a = 0; a < 6; ++a) den += X[a] * (mu * X[a] + B[a]);
        const double rho = (rr - rtt) / den;
        if (rho > 0) {
          mu *= std::fmax(0.333, 1 - std::pow(2 * rho - 1, 3));
          vv = 2;
          if (std::pow(rr - rtt, 2) < rel_tol * rr) stop = SMALL_DECREASE_FUNCTION;
          std::memcpy(v.state, xt, sizeof(xt));
          break;
        }
        mu *= vv;
        const double v2 = 2 * vv;
        if (v2 <= vv) {
          stop = NO_CONVERGENCE;
          break;
        }
        vv = v2;
      } else {
        stop = NO_CONVERGENCE;
        break;
      }
    }
  } while (!(k++ < (p->max_iter ? stop : (stop = MAX_ITERATIONS))));
  return !(stop == NO_CONVERGENCE || stop == MAX_ITERATIONS);
}

// computeInliers (:94-114)
std::vector<int> compute_inliers(const VO& v) {
  double Tr[16];
  make_Tr(v.state, Tr);
  std::vector<int> out;
  const double thr2 = v.p->inlier_threshold * v.p->inlier_threshold;
  for (int m = 0; m < v.n; ++m) {
    double r[4];
    residual1(v, Tr, m, r);
    const double score = r[0] * r[0] + r[1] * r[1] + r[2] * r[2] + r[3] * r[3];
    if (score < thr2) out.push_back(m);
  }
  return out;
}

}  // namespace

extern "C" int oracle_vo_process(const float* m, int n, const double* init6, const oracle_vo_params* p,
                                 const int* rand_seq, int rand_len, double* motion, int* inliers, int* n_inliers,
                                 int max_outer) {
  VO v;
  v.p = p;
  v.n = n;
  double init[6] = {0, 0, 0, 0, 0, 0};
  if (init6) std::memcpy(init, init6, sizeof(init));
  std::memcpy(v.state, init, sizeof(init));
  *n_inliers = 0;
  int ok = 0;
  bool hang = false;
  std::vector<int> best;
  if (n >= 6) {
    v.X.resize(4 * (size_t)n);
    v.obs.resize(4 * (size_t)n);
    for (int i = 0; i < n; ++i) {
      const float* f = m + 8 * i;
      const double d = (f[0] - p->cu1) - (f[2] - p->cu2);
      double* X = &v.X[4 * i];
      X[0] = (f[0] - p->cu1) * p->baseline;
      X[1] = (f[1] - p->cv1) * p->baseline;
      X[2] = p->fu1 * p->baseline;
      X[3] = d > 0 ? d : 0.00001;
      X[0] /= X[3];
      X[1] /= X[3];
      X[2] /= X[3];
      X[3] /= X[3];
      v.obs[4 * i + 0] = f[4];
      v.obs[4 * i + 1] = f[5];
      v.obs[4 * i + 2] = f[6];
      v.obs[4 * i + 3] = f[7];
    }
    if (p->ransac) {
      int rp = 0;
      for (int it = 0; it < p->n_ransac; ++it) {
        std::vector<int> sel;  // selectRandomIndices(3, n) (:143-163)
        while ((int)sel.size() < 3) {
          if (rp >= rand_len) return -3;
          const int idx = rand_seq[rp++] % n;
          bool exists = false;
          for (int s : sel) exists = exists || s == idx;
          if (!exists) sel.push_back(idx);
        }
        const float x0 = m[8 * sel[0] + 4], y0 = m[8 * sel[0] + 5], x1 = m[8 * sel[1] + 4], y1 = m[8 * sel[1] + 5];
        const float x2 = m[8 * sel[2] + 4], y2 = m[8 * sel[2] + 5];
        if ((x0 * (y1 - y2) + x1 * (y2 - y0) + x2 * (y0 - y1)) / 2 > 1000) {  // float arithmetic (:63)
          std::memcpy(v.state, init, sizeof(init));
          if (optimize(v, sel, max_outer, &hang)) {
            std::vector<int> tmp = compute_inliers(v);
            if (tmp.size() > best.size()) best = tmp;
          }
          if (hang) return -2;
        }
      }
    } else {
      for (int i = 0; i < n; ++i) best.push_back(i);
    }
    std::memcpy(v.state, init, sizeof(init));
    if (best.size() >= 6) {
      ok = optimize(v, best, max_outer, &hang) ? 1 : 0;
      if (hang) return -2;
    }
  }
  // getMotion (:331-342)
  double Tr[16];
  make_Tr(v.state, Tr);
  std::memcpy(motion, Tr, sizeof(Tr));
  for (size_t i = 0; i < best.size(); ++i) inliers[i] = best[i];
  *n_inliers = (int)best.size();
  return ok;
}
