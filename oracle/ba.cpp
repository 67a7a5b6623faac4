// oracle/ba.cpp — TEST INFRASTRUCTURE: CPU restatement of the windowed stereo
// bundle adjuster BundleAdjuster<4>::optimise
// (include/MotionEstimation/optimisation/BundleAdjuster.h:142-180, 431-476)
// and of the Ceres Solver semantics it delegates to (Ceres is not vendored;
// version unpinned, >= 1.12 per README.md:8):
//  * AutoDiffCostFunction<StereoReprojectionError,4,6,3>: forward-mode dual
//    numbers (Jets) through ceres::AngleAxisRotatePoint and the pinhole model.
//  * HuberLoss(1.0) + Corrector (rho'' <= 0 -> scale r and J by sqrt(rho')).
//  * TrustRegionMinimizer + LevenbergMarquardtStrategy defaults: radius 1e4,
//    Jacobi scaling 1/(1+||col||) fixed at iteration 0, LM diagonal
//    clamp(diag(JtJ), 1e-6, 1e32)/radius, step quality > 1e-3, radius update
//    r /= max(1/3, 1-(2q-1)^3) on success, r /= f, f *= 2 on failure.
//  * Bounds projection in ParameterBlock::Plus, infeasible start -> FAILURE.
//  * Termination: function/parameter/gradient tolerance, max iterations (the
//    1 s wall-clock cap of BundleAdjuster.h:464 is replaced by the iteration
//    cap so the solve is deterministic — SURVEY Appendix A-9).
// The linear system is solved by point-first Schur elimination and a dense
// Cholesky of the reduced camera matrix (equal, in exact arithmetic, to
// Ceres' SPARSE_SCHUR).  Parity unpinned (see oracle.h).
#include <cmath>
#include <cstring>
#include <vector>
#include <algorithm>
#include "oracle.h"

namespace {

template <int N>
struct Jet {
  double a;
  double v[N];
  Jet() : a(0) { for (int i = 0; i < N; ++i) v[i] = 0; }
  explicit Jet(double x) : a(x) { for (int i = 0; i < N; ++i) v[i] = 0; }
  Jet(double x, int k) : a(x) { for (int i = 0; i < N; ++i) v[i] = 0; v[k] = 1; }
};
template <int N> Jet<N> operator+(const Jet<N>& f, const Jet<N>& g) { Jet<N> r(f.a + g.a); for (int i = 0; i < N; ++i) r.v[i] = f.v[i] + g.v[i]; return r; }
template <int N> Jet<N> operator-(const Jet<N>& f, const Jet<N>& g) { Jet<N> r(f.a - g.a); for (int i = 0; i < N; ++i) r.v[i] = f.v[i] - g.v[i]; return r; }
template <int N> Jet<N> operator-(const Jet<N>& f) { Jet<N> r(-f.a); for (int i = 0; i < N; ++i) r.v[i] = -f.v[i]; return r; }
template <int N> Jet<N> operator*(const Jet<N>& f, const Jet<N>& g) { Jet<N> r(f.a * g.a); for (int i = 0; i < N; ++i) r.v[i] = f.a * g.v[i] + f.v[i] * g.a; return r; }
template <int N> Jet<N> operator/(const Jet<N>& f, const Jet<N>& g) {
  const double ginv = 1.0 / g.a, fg = f.a * ginv;
  Jet<N> r(fg); for (int i = 0; i < N; ++i) r.v[i] = (f.v[i] - fg * g.v[i]) * ginv; return r;
}
template <int N> Jet<N> operator+(const Jet<N>& f, double s) { Jet<N> r = f; r.a += s; return r; }
template <int N> Jet<N> operator-(const Jet<N>& f, double s) { Jet<N> r = f; r.a -= s; return r; }
template <int N> Jet<N> operator*(double s, const Jet<N>& f) { Jet<N> r(s * f.a); for (int i = 0; i < N; ++i) r.v[i] = s * f.v[i]; return r; }
template <int N> Jet<N> operator*(const Jet<N>& f, double s) { Jet<N> r(f.a * s); for (int i = 0; i < N; ++i) r.v[i] = f.v[i] * s; return r; }
template <int N> Jet<N> jsqrt(const Jet<N>& f) { double s = std::sqrt(f.a); Jet<N> r(s); double t = 1.0 / (2.0 * s); for (int i = 0; i < N; ++i) r.v[i] = f.v[i] * t; return r; }
template <int N> Jet<N> jcos(const Jet<N>& f) { Jet<N> r(std::cos(f.a)); double d = -std::sin(f.a); for (int i = 0; i < N; ++i) r.v[i] = d * f.v[i]; return r; }
template <int N> Jet<N> jsin(const Jet<N>& f) { Jet<N> r(std::sin(f.a)); double d = std::cos(f.a); for (int i = 0; i < N; ++i) r.v[i] = d * f.v[i]; return r; }

// ceres::AngleAxisRotatePoint (ceres/rotation.h)
template <int N>
void aa_rotate(const Jet<N> aa[3], const Jet<N> pt[3], Jet<N> out[3]) {
  Jet<N> theta2 = aa[0] * aa[0] + aa[1] * aa[1] + aa[2] * aa[2];
  if (theta2.a > 2.220446049250313e-16) {
    Jet<N> theta = jsqrt(theta2), c = jcos(theta), s = jsin(theta), ti = Jet<N>(1.0) / theta;
    Jet<N> w[3] = {aa[0] * ti, aa[1] * ti, aa[2] * ti};
    Jet<N> wx[3] = {w[1] * pt[2] - w[2] * pt[1], w[2] * pt[0] - w[0] * pt[2], w[0] * pt[1] - w[1] * pt[0]};
    Jet<N> tmp = (w[0] * pt[0] + w[1] * pt[1] + w[2] * pt[2]) * (Jet<N>(1.0) - c);
    for (int i = 0; i < 3; ++i) out[i] = pt[i] * c + wx[i] * s + w[i] * tmp;
  } else {
    Jet<N> wx[3] = {aa[1] * pt[2] - aa[2] * pt[1], aa[2] * pt[0] - aa[0] * pt[2], aa[0] * pt[1] - aa[1] * pt[0]};
    for (int i = 0; i < 3; ++i) out[i] = pt[i] + wx[i];
  }
}

// BundleAdjuster<2>::optimise replaces a zero baseline by 0.5 (BundleAdjuster.h:389-390)
double eff_baseline(const oracle_ba_problem* p) {
  return p->obs_dim == 2 && p->baseline == 0 ? 0.5 : p->baseline;
}

// StandardReprojectionError (BundleAdjuster.h:71-103, camID 0) / StereoRightError
// (:106-139, otherwise) -- the residuals of BundleAdjuster<2> (:395-398); rows 2, 3 zero
void eval_obs_mono(const oracle_ba_problem* p, int o, const double* cam, const double* pt, double r[4],
                   double Jc[24], double Jp[12]) {
  typedef Jet<9> J9;
  J9 c[6], X[3];
  for (int i = 0; i < 6; ++i) c[i] = J9(cam[i], i);
  for (int i = 0; i < 3; ++i) X[i] = J9(pt[i], 6 + i);
  J9 P[3];
  aa_rotate<9>(c + 3, X, P);
  if (p->cam_id[o] == 0) P[0] = P[0] + c[0];
  else P[0] = P[0] + (c[0] - eff_baseline(p));  // p[0] += camera[0] - calib->baseline
  P[1] = P[1] + c[1];
  P[2] = P[2] + c[2];
  const double sinv = 1.0 / std::sqrt(p->feat_var);
  J9 x = p->K0[0] * (P[0] / P[2]) + p->K0[2];
  J9 y = p->K0[4] * (P[1] / P[2]) + p->K0[5];
  const double* f = p->obs + 2 * o;
  J9 res[2] = {sinv * (x - f[0]), sinv * (y - f[1])};
  for (int k = 0; k < 4; ++k) {
    r[k] = k < 2 ? res[k].a : 0.0;
    if (Jc) for (int j = 0; j < 6; ++j) Jc[k * 6 + j] = k < 2 ? res[k].v[j] : 0.0;
    if (Jp) for (int j = 0; j < 3; ++j) Jp[k * 3 + j] = k < 2 ? res[k].v[6 + j] : 0.0;
  }
}

// StereoReprojectionError::operator() (BundleAdjuster.h:153-171)
void eval_obs(const oracle_ba_problem* p, int o, const double* cam, const double* pt, double r[4], double Jc[24],
              double Jp[12]) {
  if (p->obs_dim == 2) {
    eval_obs_mono(p, o, cam, pt, r, Jc, Jp);
    return;
  }
  typedef Jet<9> J9;
  J9 c[6], X[3];
  for (int i = 0; i < 6; ++i) c[i] = J9(cam[i], i);
  for (int i = 0; i < 3; ++i) X[i] = J9(pt[i], 6 + i);
  J9 P[3];
  aa_rotate<9>(c + 3, X, P);
  P[0] = P[0] + c[0];
  P[1] = P[1] + c[1];
  P[2] = P[2] + c[2];
  const double sinv = 1.0 / std::sqrt(p->feat_var);
  J9 x1 = p->K0[0] * (P[0] / P[2]) + p->K0[2];
  J9 x2 = p->K1[0] * ((P[0] - p->baseline) / P[2]) + p->K1[2];
  J9 y = p->K0[4] * (P[1] / P[2]) + p->K0[5];
  const double* f = p->obs + 4 * o;
  J9 res[4] = {sinv * (x1 - f[0]), sinv * (y - f[1]), sinv * (x2 - f[2]), sinv * (y - f[3])};
  for (int k = 0; k < 4; ++k) {
    r[k] = res[k].a;
    if (Jc) for (int j = 0; j < 6; ++j) Jc[k * 6 + j] = res[k].v[j];
    if (Jp) for (int j = 0; j < 3; ++j) Jp[k * 3 + j] = res[k].v[6 + j];
  }
}

// ceres::HuberLoss(1.0)::Evaluate
void huber(double s, double rho[3]) {
  if (s > 1.0) {
    const double r = std::sqrt(s);
    rho[0] = 2.0 * r - 1.0;
    rho[1] = std::max(2.2250738585072014e-308, 1.0 / r);
    rho[2] = -rho[1] / (2.0 * s);
  } else {
    rho[0] = s; rho[1] = 1.0; rho[2] = 0.0;
  }
}

struct Bounds { double lo[3], hi[3]; };
Bounds point_bounds(const oracle_ba_problem* p) {
  // BundleAdjuster.h:442-443, 455-460
  const double Zmax = p->K0[0] * eff_baseline(p) / 0.1;
  const double Zmin = p->K0[0] * eff_baseline(p) / (2 * p->K0[2]);
  Bounds b;
  b.hi[0] = Zmax / p->K0[0] * p->K0[2]; b.hi[1] = Zmax / p->K0[4] * p->K0[5]; b.hi[2] = Zmax;
  b.lo[0] = -Zmax / p->K0[0] * p->K0[2]; b.lo[1] = -Zmax / p->K0[4] * p->K0[5]; b.lo[2] = Zmin;
  return b;
}

double total_cost(const oracle_ba_problem* p, const double* cams, const double* pts) {
  double cost = 0;
  for (int o = 0; o < p->n_obs; ++o) {
    double r[4];
    eval_obs(p, o, cams + 6 * p->cam_idx[o], pts + 3 * p->pt_idx[o], r, nullptr, nullptr);
    double s = r[0] * r[0] + r[1] * r[1] + r[2] * r[2] + r[3] * r[3], rho[3];
    huber(s, rho);
    cost += 0.5 * rho[0];
  }
  return cost;
}

// dense Cholesky in place (lower), returns false if not PD
bool cholesky(std::vector<double>& A, int n) {
  for (int j = 0; j < n; ++j) {
    double d = A[j * n + j];
    for (int k = 0; k < j; ++k) d -= A[j * n + k] * A[j * n + k];
    if (!(d > 0)) return false;
    d = std::sqrt(d);
    A[j * n + j] = d;
    for (int i = j + 1; i < n; ++i) {
      double s = A[i * n + j];
      for (int k = 0; k < j; ++k) s -= A[i * n + k] * A[j * n + k];
      A[i * n + j] = s / d;
    }
  }
  return true;
}
void chol_solve(const std::vector<double>& L, int n, double* x) {
  for (int i = 0; i < n; ++i) { double s = x[i]; for (int k = 0; k < i; ++k) s -= L[i * n + k] * x[k]; x[i] = s / L[i * n + i]; }
  for (int i = n - 1; i >= 0; --i) { double s = x[i]; for (int k = i + 1; k < n; ++k) s -= L[k * n + i] * x[k]; x[i] = s / L[i * n + i]; }
}
void inv3_spd(const double V[9], double Vi[9], bool* ok) {
  std::vector<double> L(V, V + 9);
  *ok = cholesky(L, 3);
  if (!*ok) return;
  for (int c = 0; c < 3; ++c) {
    double e[3] = {0, 0, 0}; e[c] = 1;
    chol_solve(L, 3, e);
    for (int r = 0; r < 3; ++r) Vi[r * 3 + c] = e[r];
  }
}

struct Linearisation {
  std::vector<double> r, Jc, Jp;  // corrected residuals / jacobians (unscaled)
  double cost;
};

void linearise(const oracle_ba_problem* p, const double* cams, const double* pts, Linearisation& L) {
  L.r.assign(4 * p->n_obs, 0); L.Jc.assign(24 * p->n_obs, 0); L.Jp.assign(12 * p->n_obs, 0);
  L.cost = 0;
  for (int o = 0; o < p->n_obs; ++o) {
    double* r = &L.r[4 * o]; double* Jc = &L.Jc[24 * o]; double* Jp = &L.Jp[12 * o];
    eval_obs(p, o, cams + 6 * p->cam_idx[o], pts + 3 * p->pt_idx[o], r, Jc, Jp);
    double s = r[0] * r[0] + r[1] * r[1] + r[2] * r[2] + r[3] * r[3], rho[3];
    huber(s, rho);
    L.cost += 0.5 * rho[0];
    // Corrector (ceres/corrector.cc): rho'' <= 0 for Huber -> plain sqrt(rho') scaling
    double sc = std::sqrt(rho[1]);
    for (int k = 0; k < 4; ++k) r[k] *= sc;
    for (int k = 0; k < 24; ++k) Jc[k] *= sc;
    for (int k = 0; k < 12; ++k) Jp[k] *= sc;
  }
}

struct Solver {
  const oracle_ba_problem* p;
  int nc, np, no, nf, m;  // m = variable cameras
  std::vector<double> csc, psc;  // jacobi scaling per variable camera param / point param
  std::vector<std::vector<int>> pobs;
};

// Builds and solves the LM system in scaled coordinates; returns false on
// linear-solver failure.  y_c (6m), y_p (3np) are the scaled steps.
bool solve_lm(const Solver& S, const Linearisation& L, double radius, std::vector<double>& yc, std::vector<double>& yp,
              std::vector<double>* Sout, std::vector<double>* bout) {
  const oracle_ba_problem* p = S.p;
  const int m = S.m, n6 = 6 * m;
  std::vector<double> U(n6 * n6, 0.0), gc(n6, 0.0);
  std::vector<double> V(9 * S.np, 0.0), gp(3 * S.np, 0.0);
  std::vector<double> Wo(18 * S.no, 0.0);
  // scaled jacobian blocks
  for (int o = 0; o < S.no; ++o) {
    int ci = p->cam_idx[o] - S.nf, pi = p->pt_idx[o];
    const double* r = &L.r[4 * o];
    double Jp[12];
    for (int k = 0; k < 4; ++k) for (int j = 0; j < 3; ++j) Jp[k * 3 + j] = L.Jp[24 * 0 + 12 * o + k * 3 + j] * S.psc[3 * pi + j];
    for (int a = 0; a < 3; ++a) {
      for (int b = 0; b < 3; ++b) { double s = 0; for (int k = 0; k < 4; ++k) s += Jp[k * 3 + a] * Jp[k * 3 + b]; V[9 * pi + a * 3 + b] += s; }
      double g = 0; for (int k = 0; k < 4; ++k) g += Jp[k * 3 + a] * r[k]; gp[3 * pi + a] += g;
    }
    if (ci >= 0) {
      double Jc[24];
      for (int k = 0; k < 4; ++k) for (int j = 0; j < 6; ++j) Jc[k * 6 + j] = L.Jc[24 * o + k * 6 + j] * S.csc[6 * ci + j];
      for (int a = 0; a < 6; ++a) {
        for (int b = 0; b < 6; ++b) { double s = 0; for (int k = 0; k < 4; ++k) s += Jc[k * 6 + a] * Jc[k * 6 + b]; U[(6 * ci + a) * n6 + 6 * ci + b] += s; }
        double g = 0; for (int k = 0; k < 4; ++k) g += Jc[k * 6 + a] * r[k]; gc[6 * ci + a] += g;
        for (int b = 0; b < 3; ++b) { double s = 0; for (int k = 0; k < 4; ++k) s += Jc[k * 6 + a] * Jp[k * 3 + b]; Wo[18 * o + a * 3 + b] = s; }
      }
    }
  }
  // LM diagonal: D = clamp(diag(JtJ)) / radius, added to both cameras and points
  for (int i = 0; i < n6; ++i) { double d = std::min(std::max(U[i * n6 + i], 1e-6), 1e32); U[i * n6 + i] += d / radius; }
  for (int j = 0; j < S.np; ++j) for (int a = 0; a < 3; ++a) { double d = std::min(std::max(V[9 * j + 4 * a], 1e-6), 1e32); V[9 * j + 4 * a] += d / radius; }
  // Schur: S = U - sum_j W_j V_j^-1 W_j^T ; b = gc - sum_j W_j V_j^-1 gp_j
  std::vector<double> Sm = U, bm = gc;
  std::vector<double> Vinv(9 * S.np);
  for (int j = 0; j < S.np; ++j) {
    bool ok;
    inv3_spd(&V[9 * j], &Vinv[9 * j], &ok);
    if (!ok) return false;
    const std::vector<int>& ob = S.pobs[j];
    for (size_t u = 0; u < ob.size(); ++u) {
      int ou = ob[u], cu = p->cam_idx[ou] - S.nf;
      if (cu < 0) continue;
      double WV[18];
      for (int a = 0; a < 6; ++a) for (int b = 0; b < 3; ++b) { double s = 0; for (int c = 0; c < 3; ++c) s += Wo[18 * ou + a * 3 + c] * Vinv[9 * j + c * 3 + b]; WV[a * 3 + b] = s; }
      for (int a = 0; a < 6; ++a) { double s = 0; for (int c = 0; c < 3; ++c) s += WV[a * 3 + c] * gp[3 * j + c]; bm[6 * cu + a] -= s; }
      for (size_t v = 0; v < ob.size(); ++v) {
        int ov = ob[v], cv = p->cam_idx[ov] - S.nf;
        if (cv < 0) continue;
        for (int a = 0; a < 6; ++a) for (int b = 0; b < 6; ++b) {
          double s = 0; for (int c = 0; c < 3; ++c) s += WV[a * 3 + c] * Wo[18 * ov + b * 3 + c];
          Sm[(6 * cu + a) * n6 + 6 * cv + b] -= s;
        }
      }
    }
  }
  if (Sout) *Sout = Sm;
  if (bout) *bout = bm;
  yc.assign(n6, 0.0);
  if (n6 > 0) {
    std::vector<double> Lc = Sm;
    if (!cholesky(Lc, n6)) return false;
    for (int i = 0; i < n6; ++i) yc[i] = -bm[i];
    chol_solve(Lc, n6, yc.data());
  }
  yp.assign(3 * S.np, 0.0);
  for (int j = 0; j < S.np; ++j) {
    double rhs[3] = {-gp[3 * j], -gp[3 * j + 1], -gp[3 * j + 2]};
    for (int ou : S.pobs[j]) {
      int cu = p->cam_idx[ou] - S.nf;
      if (cu < 0) continue;
      for (int b = 0; b < 3; ++b) { double s = 0; for (int a = 0; a < 6; ++a) s += Wo[18 * ou + a * 3 + b] * yc[6 * cu + a]; rhs[b] -= s; }
    }
    for (int a = 0; a < 3; ++a) { double s = 0; for (int b = 0; b < 3; ++b) s += Vinv[9 * j + a * 3 + b] * rhs[b]; yp[3 * j + a] = s; }
  }
  return true;
}

Solver make_solver(const oracle_ba_problem* p) {
  Solver S;
  S.p = p; S.nc = p->n_cams; S.np = p->n_pts; S.no = p->n_obs;
  S.nf = std::min(std::max(p->fixed_frames, 0), p->n_cams);
  S.m = S.nc - S.nf;
  S.pobs.assign(S.np, {});
  for (int o = 0; o < S.no; ++o) S.pobs[p->pt_idx[o]].push_back(o);
  return S;
}

}  // namespace

extern "C" void oracle_ba_default_options(oracle_ba_options* o) {
  o->max_num_iterations = 50;
  o->function_tolerance = 1e-3;  // BundleAdjuster.h:465
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

extern "C" void oracle_ba_evaluate(const oracle_ba_problem* p, double* res, double* Jc, double* Jp) {
  const int D = p->obs_dim == 2 ? 2 : 4;
  for (int o = 0; o < p->n_obs; ++o) {
    double r[4], jc[24], jp[12];
    eval_obs(p, o, p->cams + 6 * p->cam_idx[o], p->pts + 3 * p->pt_idx[o], r, jc, jp);
    for (int k = 0; k < D; ++k) res[D * o + k] = r[k];
    if (Jc) for (int k = 0; k < 6 * D; ++k) Jc[6 * D * o + k] = jc[k];
    if (Jp) for (int k = 0; k < 3 * D; ++k) Jp[3 * D * o + k] = jp[k];
  }
}

// ceres::Covariance over the camera blocks (BundleAdjuster.h:478-528): Jacobian with the
// loss function applied (Covariance::Options::apply_loss_function = true), constant
// cameras excluded, (J^T J)^-1 formed densely here (Ceres: sparse QR; the same matrix).
extern "C" int oracle_ba_covariance(const oracle_ba_problem* p, double* cov) {
  const int nc = p->n_cams, np = p->n_pts;
  const int nf = std::min(std::max(p->fixed_frames, 0), nc), m = nc - nf;
  const int n = 6 * m + 3 * np;
  Linearisation L;
  linearise(p, p->cams, p->pts, L);
  std::vector<double> H((size_t)n * n, 0.0);
  for (int o = 0; o < p->n_obs; ++o) {
    const int ci = p->cam_idx[o] - nf, pi = p->pt_idx[o];
    int col[9], nv = 0;
    double J[4][9];
    for (int k = 0; k < 4; ++k) {
      int q = 0;
      if (ci >= 0) for (int j = 0; j < 6; ++j) J[k][q++] = L.Jc[24 * o + 6 * k + j];
      for (int j = 0; j < 3; ++j) J[k][q++] = L.Jp[12 * o + 3 * k + j];
    }
    if (ci >= 0) for (int j = 0; j < 6; ++j) col[nv++] = 6 * ci + j;
    for (int j = 0; j < 3; ++j) col[nv++] = 6 * m + 3 * pi + j;
    for (int a = 0; a < nv; ++a)
      for (int b = 0; b < nv; ++b) {
        double s = 0;
        for (int k = 0; k < 4; ++k) s += J[k][a] * J[k][b];
        H[(size_t)col[a] * n + col[b]] += s;
      }
  }
  if (!cholesky(H, n)) return 0;
  // X = L^-1 columns of the camera parameters only, cov = X^T X restricted to them
  std::vector<double> X((size_t)6 * m * n, 0.0);
  for (int c = 0; c < 6 * m; ++c) {
    double* x = &X[(size_t)c * n];
    for (int k = c; k < n; ++k) {
      double acc = k == c ? 1.0 : 0.0;
      for (int l = c; l < k; ++l) acc -= H[(size_t)k * n + l] * x[l];
      x[k] = acc / H[(size_t)k * n + k];
    }
  }
  for (int i = 0; i < nc; ++i)
    for (int a = 0; a < 6; ++a)
      for (int b = 0; b < 6; ++b) {
        double v = 0;
        if (i >= nf) {
          const int pp = 6 * (i - nf) + a, qq = 6 * (i - nf) + b;
          for (int k = std::max(pp, qq); k < n; ++k) v += X[(size_t)pp * n + k] * X[(size_t)qq * n + k];
        }
        cov[36 * i + 6 * a + b] = v;
      }
  return 1;
}

extern "C" double oracle_ba_cost(const oracle_ba_problem* p) { return total_cost(p, p->cams, p->pts); }

static void compute_scaling(Solver& S, const Linearisation& L, bool jacobi) {
  const oracle_ba_problem* p = S.p;
  S.csc.assign(6 * S.m, 0.0); S.psc.assign(3 * S.np, 0.0);
  for (int o = 0; o < S.no; ++o) {
    int ci = p->cam_idx[o] - S.nf, pi = p->pt_idx[o];
    for (int k = 0; k < 4; ++k) {
      if (ci >= 0) for (int j = 0; j < 6; ++j) { double v = L.Jc[24 * o + k * 6 + j]; S.csc[6 * ci + j] += v * v; }
      for (int j = 0; j < 3; ++j) { double v = L.Jp[12 * o + k * 3 + j]; S.psc[3 * pi + j] += v * v; }
    }
  }
  for (double& c : S.csc) c = jacobi ? 1.0 / (1.0 + std::sqrt(c)) : 1.0;
  for (double& c : S.psc) c = jacobi ? 1.0 / (1.0 + std::sqrt(c)) : 1.0;
}

// Reduced camera system S = U - W V^-1 W^T, b of the first LM step
// (Ceres SPARSE_SCHUR, BundleAdjuster.h:463).  `jacobi` = 0 leaves the
// columns unscaled, which makes S and b additive over landmark shards (the
// exchange of the multi-GPU solve).
extern "C" int oracle_ba_reduced_system_ex(const oracle_ba_problem* p, double radius, int jacobi, double* Sout,
                                           double* bout) {
  Solver S = make_solver(p);
  Linearisation L;
  linearise(p, p->cams, p->pts, L);
  compute_scaling(S, L, jacobi != 0);
  std::vector<double> yc, yp, Sm, bm;
  bool ok = solve_lm(S, L, radius, yc, yp, &Sm, &bm);
  std::memcpy(Sout, Sm.data(), Sm.size() * 8);
  std::memcpy(bout, bm.data(), bm.size() * 8);
  return ok ? 0 : -1;
}

extern "C" int oracle_ba_reduced_system(const oracle_ba_problem* p, double radius, double* Sout, double* bout) {
  Solver S = make_solver(p);
  Linearisation L;
  linearise(p, p->cams, p->pts, L);
  compute_scaling(S, L, true);
  std::vector<double> yc, yp, Sm, bm;
  bool ok = solve_lm(S, L, radius, yc, yp, &Sm, &bm);
  std::memcpy(Sout, Sm.data(), Sm.size() * 8);
  std::memcpy(bout, bm.data(), bm.size() * 8);
  return ok ? 0 : -1;
}

extern "C" int oracle_ba_solve(oracle_ba_problem* p, const oracle_ba_options* opt, oracle_ba_summary* sum,
                               double* cost_trace, int trace_cap) {
  Solver S = make_solver(p);
  const Bounds bd = point_bounds(p);
  sum->iterations = 0; sum->successful_steps = 0;
  // Problem::IsFeasible check (Ceres preprocessor)
  for (int j = 0; j < S.np; ++j)
    for (int a = 0; a < 3; ++a) {
      double x = p->pts[3 * j + a];
      if (x < bd.lo[a] || x > bd.hi[a]) {
        sum->status = 3; sum->termination = 2; sum->initial_cost = sum->final_cost = NAN;
        return 3;
      }
    }
  const int nvar = 6 * S.m + 3 * S.np;
  auto xnorm = [&](const double* cams, const double* pts) {
    double s = 0;
    for (int i = 6 * S.nf; i < 6 * S.nc; ++i) s += cams[i] * cams[i];
    for (int i = 0; i < 3 * S.np; ++i) s += pts[i] * pts[i];
    return std::sqrt(s);
  };
  (void)nvar;
  Linearisation L;
  linearise(p, p->cams, p->pts, L);
  compute_scaling(S, L, opt->jacobi_scaling != 0);
  double x_cost = L.cost;
  sum->initial_cost = x_cost;
  double radius = opt->initial_trust_region_radius, decrease = 2.0;
  int invalid = 0;
  int termination = 1;
  std::vector<double> cand_c(p->cams, p->cams + 6 * S.nc), cand_p(p->pts, p->pts + 3 * S.np);
  auto grad_max_norm = [&]() {
    // ||x - Plus(x, -g)||_inf with g the (corrected, unscaled) gradient
    std::vector<double> g(6 * S.m + 3 * S.np, 0.0);
    for (int o = 0; o < S.no; ++o) {
      int ci = p->cam_idx[o] - S.nf, pi = p->pt_idx[o];
      for (int k = 0; k < 4; ++k) {
        if (ci >= 0) for (int j = 0; j < 6; ++j) g[6 * ci + j] += L.Jc[24 * o + k * 6 + j] * L.r[4 * o + k];
        for (int j = 0; j < 3; ++j) g[6 * S.m + 3 * pi + j] += L.Jp[12 * o + k * 3 + j] * L.r[4 * o + k];
      }
    }
    double m = 0;
    for (int i = 0; i < 6 * S.m; ++i) m = std::max(m, std::fabs(g[i]));
    for (int j = 0; j < S.np; ++j) for (int a = 0; a < 3; ++a) {
      double x = p->pts[3 * j + a], xp = std::min(std::max(x - g[6 * S.m + 3 * j + a], bd.lo[a]), bd.hi[a]);
      m = std::max(m, std::fabs(x - xp));
    }
    return m;
  };
  int ntr = 0;
  if (grad_max_norm() <= opt->gradient_tolerance) { termination = 0; goto done; }
  for (;;) {
    if (sum->iterations >= opt->max_num_iterations) { termination = 1; break; }
    if (radius <= opt->min_trust_region_radius) { termination = 0; break; }
    sum->iterations++;
    std::vector<double> yc, yp;
    bool ok = solve_lm(S, L, radius, yc, yp, nullptr, nullptr);
    double model_change = 0;
    if (ok) {
      for (int o = 0; o < S.no; ++o) {
        int ci = p->cam_idx[o] - S.nf, pi = p->pt_idx[o];
        double Jd[4];
        for (int k = 0; k < 4; ++k) {
          double s = 0;
          if (ci >= 0) for (int j = 0; j < 6; ++j) s += L.Jc[24 * o + k * 6 + j] * S.csc[6 * ci + j] * yc[6 * ci + j];
          for (int j = 0; j < 3; ++j) s += L.Jp[12 * o + k * 3 + j] * S.psc[3 * pi + j] * yp[3 * pi + j];
          Jd[k] = s;
        }
        for (int k = 0; k < 4; ++k) model_change -= Jd[k] * (L.r[4 * o + k] + Jd[k] / 2.0);
      }
    }
    if (!ok || !(model_change > 0.0)) {
      // invalid step
      if (++invalid >= opt->max_num_consecutive_invalid_steps) { termination = 2; break; }
      radius = radius / decrease; decrease *= 2.0;
      continue;
    }
    invalid = 0;
    // candidate = Plus(x, delta) with bound projection
    double step2 = 0;
    for (int i = 0; i < 6 * S.nc; ++i) cand_c[i] = p->cams[i];
    for (int c = 0; c < S.m; ++c) for (int j = 0; j < 6; ++j) {
      int i = 6 * (S.nf + c) + j;
      cand_c[i] = p->cams[i] + yc[6 * c + j] * S.csc[6 * c + j];
      double d = cand_c[i] - p->cams[i]; step2 += d * d;
    }
    for (int q = 0; q < S.np; ++q) for (int a = 0; a < 3; ++a) {
      int i = 3 * q + a;
      double v = p->pts[i] + yp[i] * S.psc[i];
      v = std::min(std::max(v, bd.lo[a]), bd.hi[a]);
      cand_p[i] = v;
      double d = v - p->pts[i]; step2 += d * d;
    }
    double cand_cost = total_cost(p, cand_c.data(), cand_p.data());
    double step_norm = std::sqrt(step2);
    double xn = xnorm(p->cams, p->pts);
    if (cost_trace && ntr < trace_cap) cost_trace[ntr++] = cand_cost;
    if (step_norm <= opt->parameter_tolerance * (xn + opt->parameter_tolerance)) { termination = 0; break; }
    if (std::fabs(x_cost - cand_cost) <= opt->function_tolerance * x_cost) { termination = 0; break; }
    double q = (x_cost - cand_cost) / model_change;
    if (q > opt->min_relative_decrease) {
      std::memcpy(p->cams, cand_c.data(), 8 * 6 * S.nc);
      std::memcpy(p->pts, cand_p.data(), 8 * 3 * S.np);
      sum->successful_steps++;
      linearise(p, p->cams, p->pts, L);
      x_cost = L.cost;
      radius = radius / std::max(1.0 / 3.0, 1.0 - std::pow(2.0 * q - 1.0, 3));
      radius = std::min(opt->max_trust_region_radius, radius);
      decrease = 2.0;
      if (grad_max_norm() <= opt->gradient_tolerance) { termination = 0; break; }
    } else {
      radius = radius / decrease; decrease *= 2.0;
    }
  }
done:
  sum->termination = termination;
  sum->final_cost = x_cost;
  sum->status = (termination == 2) ? 3 : 2;
  return sum->status;
}
