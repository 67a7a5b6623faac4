// oracle/scale.cpp — TEST INFRASTRUCTURE: CPU restatement of the ScaleState
// optimiser, Optimiser<ScaleState, vector<pair<Mat,Mat>>> in
// src/optimisation/optimisation.cpp:29-147,149-228,435-634,674-747 and
// include/MotionEstimation/optimisation/optimisation.h:22-125.
// Parity unpinned (see oracle.h).  Matx products are restated with OpenCV's
// evaluation order (s = 0; s += a(i,k)*b(k,j), k ascending) so that float
// feature positions, and hence integer ROIs, match bit for bit.
#include <cmath>
#include <cstring>
#include <vector>
#include <algorithm>
#include "oracle.h"

namespace {

enum { NO_STOP = 0, SMALL_GRADIENT, SMALL_INCREMENT, MAX_ITERATIONS, SMALL_DECREASE_FUNCTION,
       SMALL_REPROJ_ERROR, NO_CONVERGENCE };

// Quat<T>::getR4 (rotation_utils.h:222-229) with position in column 3
void pose_T(const double q[4], const double t[3], double T[16]) {
  const double w = q[0], x = q[1], y = q[2], z = q[3];
  T[0] = w * w + x * x - y * y - z * z; T[1] = 2 * (x * y - w * z); T[2] = 2 * (x * z + w * y); T[3] = t[0];
  T[4] = 2 * (x * y + w * z); T[5] = w * w - x * x + y * y - z * z; T[6] = 2 * (y * z - w * x); T[7] = t[1];
  T[8] = 2 * (x * z - w * y); T[9] = 2 * (y * z + w * x); T[10] = w * w - x * x - y * y + z * z; T[11] = t[2];
  T[12] = 0; T[13] = 0; T[14] = 0; T[15] = 1;
}
void R3_of(const double q[4], double R[9]) {
  double T[16]; double z[3] = {0, 0, 0};
  pose_T(q, z, T);
  for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) R[i * 3 + j] = T[i * 4 + j];
}
void mul44x41(const double T[16], const double X[4], double Y[4]) {
  for (int i = 0; i < 4; ++i) { double s = 0; for (int k = 0; k < 4; ++k) s += T[i * 4 + k] * X[k]; Y[i] = s; }
}
// ((K*I34)*s)*Y  (optimisation.cpp:178)
void proj_scaled_K(const double K[9], double s, const double Y[4], double f[3]) {
  double KI[12];
  for (int i = 0; i < 3; ++i) for (int j = 0; j < 4; ++j) {
    double a = 0; for (int k = 0; k < 3; ++k) a += K[i * 3 + k] * (k == j ? 1.0 : 0.0); KI[i * 4 + j] = a * s;
  }
  for (int i = 0; i < 3; ++i) { double a = 0; for (int k = 0; k < 4; ++k) a += KI[i * 4 + k] * Y[k]; f[i] = a; }
}
// (K*I34) * Z  (optimisation.cpp:180)
void proj_K(const double K[9], const double Z[4], double f[3]) {
  double KI[12];
  for (int i = 0; i < 3; ++i) for (int j = 0; j < 4; ++j) {
    double a = 0; for (int k = 0; k < 3; ++k) a += K[i * 3 + k] * (k == j ? 1.0 : 0.0); KI[i * 4 + j] = a;
  }
  for (int i = 0; i < 3; ++i) { double a = 0; for (int k = 0; k < 4; ++k) a += KI[i * 4 + k] * Z[k]; f[i] = a; }
}
struct P2f { float x, y; };
P2f to_euclid_f(const double f[3]) {
  double u = f[0] / f[2], v = f[1] / f[2];
  return {(float)u, (float)v};
}
// cv::Rect::contains(Point2f) -> Point2i via cvRound (round-half-even)
struct RectI { int x, y, w, h; };
bool contains(const RectI& r, P2f p) {
  int px = (int)std::nearbyintf(p.x), py = (int)std::nearbyintf(p.y);
  return r.x <= px && px < r.x + r.w && r.y <= py && py < r.y + r.h;
}
// Rect(feat.x - w, feat.y - w, ...) : float -> int truncation
inline int roi0(float c, int w) { return (int)(c - (float)w); }

int reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) { if (i < 0) i = -i; if (i >= n) i = 2 * n - 2 - i; }
  return i;
}
// cv::Sobel(ROI (view into parent), grad, CV_8U, 1, 0) -> mean -> |.|+1e-20
double sobel_weight_view(const uint8_t* img, int stride, int cols, int rows, int x0, int y0, int pw, int ph) {
  long sum = 0;
  for (int y = 0; y < ph; ++y)
    for (int x = 0; x < pw; ++x) {
      int gx = 0;
      for (int dy = -1; dy <= 1; ++dy) {
        int yy = reflect101(y0 + y + dy, rows);
        int xm = reflect101(x0 + x - 1, cols), xp = reflect101(x0 + x + 1, cols);
        int wgt = dy == 0 ? 2 : 1;
        gx += wgt * ((int)img[(long)yy * stride + xp] - (int)img[(long)yy * stride + xm]);
      }
      sum += std::min(255, std::max(0, gx));
    }
  double m = (double)sum * (1.0 / (double)(pw * ph));
  return std::fabs(m) + 1e-20;
}
// Sobel on an isolated float patch (compute_jacobian right branch, values 0/255)
double sobel_weight_isolated(const uint8_t* p, int pw, int ph) {
  long sum = 0;
  for (int y = 0; y < ph; ++y)
    for (int x = 0; x < pw; ++x) {
      float gx = 0;
      for (int dy = -1; dy <= 1; ++dy) {
        int yy = reflect101(y + dy, ph), xm = reflect101(x - 1, pw), xp = reflect101(x + 1, pw);
        float wgt = dy == 0 ? 2.f : 1.f;
        gx += wgt * ((float)p[yy * pw + xp] - (float)p[yy * pw + xm]);
      }
      int v = (int)std::nearbyintf(gx);
      sum += std::min(255, std::max(0, v));
    }
  double m = (double)sum * (1.0 / (double)(pw * ph));
  return std::fabs(m) + 1e-20;
}

bool roi_ok(int x0, int y0, int pw, int ph, int cols, int rows) {
  return x0 >= 0 && y0 >= 0 && x0 + pw <= cols && y0 + ph <= rows;
}

float mi_at(const uint8_t* A, const uint8_t* B, int stride, int ax, int ay, int bx, int by, int pw, int ph) {
  return oracle_mutual_information(A + (long)ay * stride + ax, stride, B + (long)by * stride + bx, stride, pw, ph);
}
float mi_binarized(const uint8_t* A, const uint8_t* B, int stride, int ax, int ay, int bx, int by, int pw, int ph,
                   std::vector<uint8_t>& ta, std::vector<uint8_t>& tb) {
  ta.resize(pw * ph); tb.resize(pw * ph);
  for (int y = 0; y < ph; ++y) for (int x = 0; x < pw; ++x) {
    ta[y * pw + x] = A[(long)(ay + y) * stride + ax + x] ? 255 : 0;
    tb[y * pw + x] = B[(long)(by + y) * stride + bx + x] ? 255 : 0;
  }
  return oracle_mutual_information(ta.data(), pw, tb.data(), pw, pw, ph);
}

bool masked_out(const oracle_scale_state* s, int idx) {
  return s->mask && s->mask_len > 0 && (idx >= s->mask_len || !s->mask[idx]);
}

long g_mi_evals = 0;
// logical call counts of the last oracle_scale_optimise (optimisation.cpp:51,75,101,702; rejections :719-727)
long g_res_calls = 0, g_neq_calls = 0, g_rejections = 0;

}  // namespace

extern "C" void oracle_optim_default_params(oracle_optim_params* p) {
  // OptimisationParams defaults (optimisation.h:31)
  p->type = 1; p->minim = 1; p->max_nb_iter = 20; p->v = 2; p->tau = 1e-3; p->mu = 1e-20;
  p->abs_tol = 1e-4; p->grad_tol = 1e-4; p->incr_tol = 1e-3; p->rel_tol = 1e-4; p->alpha = 1.0; p->weighting = 0;
}

// optimisation.cpp:149-228
extern "C" int oracle_scale_residuals(const oracle_scale_state* s, int weighting, double* res) {
  const int w = s->window_size;
  RectI bb{w, w, s->bb_cols - 2 * w - 1, s->bb_rows - 2 * w - 1};
  const int P = 2 * w + 1;
  int tot = 0;
  if (s->mask && s->mask_len > 0) { for (int i = 0; i < s->mask_len; ++i) tot += s->mask[i] ? 1 : 0; }
  else tot = s->n_left + s->n_right;
  for (int i = 0; i < tot; ++i) res[i] = 0;
  int k = 0;
  for (int i = 0; i < s->n_left; ++i) {
    if (masked_out(s, i)) continue;
    if (!s->tri_left[i]) continue;
    if (s->last_left[i] == s->lframe) {
      double T[16], Y[4], f[3], Z[4], f2[3];
      pose_T(s->q1, s->t1, T);
      mul44x41(T, s->X_left + 4 * i, Y);
      proj_scaled_K(s->K1, s->scale, Y, f);
      P2f fl = to_euclid_f(f);
      for (int c = 0; c < 4; ++c) Z[c] = s->scale * Y[c];
      Z[0] = Z[0] - s->baseline;
      proj_K(s->K2, Z, f2);
      P2f fr = to_euclid_f(f2);
      if (contains(bb, fl) && contains(bb, fr)) {
        int lx = roi0(fl.x, w), ly = roi0(fl.y, w), rx = roi0(fr.x, w), ry = roi0(fr.y, w);
        if (!roi_ok(lx, ly, P, P, s->cols, s->rows) || !roi_ok(rx, ry, P, P, s->cols, s->rows)) return -2;
        if (k >= tot) return -3;
        double wv = weighting ? sobel_weight_view(s->imgL, s->stride, s->cols, s->rows, lx, ly, P, P) : 1.0;
        float mi = mi_at(s->imgL, s->imgR, s->stride, lx, ly, rx, ry, P, P);
        ++g_mi_evals;
        res[k] = (double)mi * wv;
      }
    }
    k++;
  }
  for (int i = 0; i < s->n_right; ++i) {
    if (masked_out(s, s->n_right + i)) continue;  // reference indexes pts.second.size()+i (A-6)
    if (!s->tri_right[i]) continue;
    if (s->last_right[i] == s->lframe) {
      double X[4]; std::memcpy(X, s->X_right + 4 * i, 32);
      X[0] = X[0] - s->baseline; X[1] = X[1] - 0.0; X[2] = X[2] - 0.0; X[3] = X[3] - 0.0;
      double T[16], Y[4], f[3], Z[4], f2[3], R3[9];
      pose_T(s->q2, s->t2, T);
      R3_of(s->q2, R3);
      for (int r = 0; r < 3; ++r) {  // Tr.col(3) += R4*(b,0,0,0)
        double a = 0; a += R3[r * 3 + 0] * s->baseline; a += R3[r * 3 + 1] * 0.0; a += R3[r * 3 + 2] * 0.0; a += 0.0 * 0.0;
        T[r * 4 + 3] = T[r * 4 + 3] + a;
      }
      mul44x41(T, X, Y);
      proj_scaled_K(s->K2, s->scale, Y, f);
      P2f fr = to_euclid_f(f);
      for (int c = 0; c < 4; ++c) Z[c] = s->scale * Y[c];
      Z[0] = Z[0] + s->baseline;
      proj_K(s->K1, Z, f2);
      P2f fl = to_euclid_f(f2);
      if (contains(bb, fr) && contains(bb, fl)) {
        int lx = roi0(fl.x, w), ly = roi0(fl.y, w), rx = roi0(fr.x, w), ry = roi0(fr.y, w);
        if (!roi_ok(lx, ly, P, P, s->cols, s->rows) || !roi_ok(rx, ry, P, P, s->cols, s->rows)) return -2;
        if (k >= tot) return -3;
        double wv = weighting ? sobel_weight_view(s->imgR, s->stride, s->cols, s->rows, rx, ry, P, P) : 1.0;
        float mi = mi_at(s->imgR, s->imgL, s->stride, rx, ry, lx, ly, P, P);
        ++g_mi_evals;
        res[k] = (double)mi * wv;
      }
    }
    k++;
  }
  return tot;
}

// optimisation.cpp:435-537
extern "C" int oracle_scale_normal_equations(const oracle_scale_state* s, int weighting, const double* res,
                                             double* JJout, double* eout) {
  const int w = s->window_size;
  const double dp = 1;
  RectI bb{w, w, s->bb_cols - 2 * w - 1, s->bb_rows - 2 * w - 1};
  const int P = 2 * w;
  double JJ = 0, e = 0;
  int k = 0;
  for (int i = 0; i < s->n_left; ++i) {
    if (masked_out(s, i)) continue;
    if (!s->tri_left[i]) continue;
    if (s->last_left[i] == s->lframe) {
      const double* X = s->X_left + 4 * i;
      double T[16], Y[4], f[3], Z[4], f2[3], R[9];
      pose_T(s->q1, s->t1, T);
      R3_of(s->q1, R);
      double Xe[3] = {X[0] / X[3], X[1] / X[3], X[2] / X[3]};
      double Zc = 0; Zc += R[6] * Xe[0]; Zc += R[7] * Xe[1]; Zc += R[8] * Xe[2];
      Zc = Zc + s->t1[2];
      double duds = s->K2[0] * s->baseline / (s->scale * Zc);
      mul44x41(T, X, Y);
      proj_scaled_K(s->K1, s->scale, Y, f);
      P2f fl = to_euclid_f(f);
      for (int c = 0; c < 4; ++c) Z[c] = s->scale * Y[c];
      Z[0] = Z[0] - s->baseline;
      proj_K(s->K2, Z, f2);
      P2f fr = to_euclid_f(f2);
      P2f frp{(float)(f2[0] / f2[2] + dp), (float)(f2[1] / f2[2])};
      if (contains(bb, fl) && contains(bb, fr)) {
        int x0x = roi0(fl.x, w), x0y = roi0(fl.y, w);
        int x1x = roi0(fr.x, w), x1y = roi0(fr.y, w);
        int x2x = roi0(frp.x, w), x2y = roi0(frp.y, w);
        if (!roi_ok(x0x, x0y, P, P, s->cols, s->rows) || !roi_ok(x1x, x1y, P, P, s->cols, s->rows) ||
            !roi_ok(x2x, x2y, P, P, s->cols, s->rows)) return -2;
        double wv = weighting ? sobel_weight_view(s->imgL, s->stride, s->cols, s->rows, x0x, x0y, P, P) : 1.0;
        double MIp = mi_at(s->imgR, s->imgL, s->stride, x2x, x2y, x0x, x0y, P, P);
        double MIm = mi_at(s->imgR, s->imgL, s->stride, x1x, x1y, x0x, x0y, P, P);
        g_mi_evals += 2;
        double J = (MIp - MIm) / dp * duds;
        JJ += J * J * wv;
        e += J * res[k];
      }
    }
    k++;
  }
  for (int i = 0; i < s->n_right; ++i) {
    if (masked_out(s, s->n_right + i)) continue;
    if (!s->tri_right[i]) continue;
    if (s->last_right[i] == s->lframe) {
      double X[4]; std::memcpy(X, s->X_right + 4 * i, 32);
      X[0] = X[0] - s->baseline;
      double T[16], Y[4], f[3], Z[4], f2[3], R[9];
      pose_T(s->q2, s->t2, T);
      R3_of(s->q2, R);
      double t[3];
      for (int r = 0; r < 3; ++r) {
        double a = 0; a += R[r * 3 + 0] * s->baseline; a += R[r * 3 + 1] * 0.0; a += R[r * 3 + 2] * 0.0;
        t[r] = s->t2[r] + a;
      }
      for (int r = 0; r < 3; ++r) {
        double a = 0; a += R[r * 3 + 0] * s->baseline; a += R[r * 3 + 1] * 0.0; a += R[r * 3 + 2] * 0.0; a += 0.0 * 0.0;
        T[r * 4 + 3] = T[r * 4 + 3] + a;
      }
      double Xe[3] = {X[0] / X[3], X[1] / X[3], X[2] / X[3]};
      double Zc = 0; Zc += R[6] * Xe[0]; Zc += R[7] * Xe[1]; Zc += R[8] * Xe[2];
      Zc = Zc + t[2];
      double duds = -s->K2[0] * s->baseline / (s->scale * Zc);
      mul44x41(T, X, Y);
      proj_scaled_K(s->K2, s->scale, Y, f);
      P2f fr = to_euclid_f(f);
      for (int c = 0; c < 4; ++c) Z[c] = s->scale * Y[c];
      Z[0] = Z[0] + s->baseline;
      proj_K(s->K2, Z, f2);  // quirk: K.second for the left reprojection (optimisation.cpp:516)
      P2f fl = to_euclid_f(f2);
      P2f flp{(float)(f2[0] / f2[2] + dp), (float)(f2[1] / f2[2])};
      if (contains(bb, fr) && contains(bb, fl)) {
        int x0x = roi0(fr.x, w), x0y = roi0(fr.y, w);
        int x1x = roi0(fl.x, w), x1y = roi0(fl.y, w);
        int x2x = roi0(flp.x, w), x2y = roi0(flp.y, w);
        if (!roi_ok(x0x, x0y, P, P, s->cols, s->rows) || !roi_ok(x1x, x1y, P, P, s->cols, s->rows) ||
            !roi_ok(x2x, x2y, P, P, s->cols, s->rows)) return -2;
        double wv = weighting ? sobel_weight_view(s->imgR, s->stride, s->cols, s->rows, x0x, x0y, P, P) : 1.0;
        double MIp = mi_at(s->imgL, s->imgR, s->stride, x2x, x2y, x0x, x0y, P, P);
        double MIm = mi_at(s->imgL, s->imgR, s->stride, x1x, x1y, x0x, x0y, P, P);
        g_mi_evals += 2;
        double J = (MIp - MIm) / dp * duds;
        JJ += J * J * wv;
        e += J * res[k];
      }
    }
    k++;
  }
  *JJout = JJ;
  *eout = e;
  return 0;
}

// optimisation.cpp:539-634
extern "C" int oracle_scale_jacobian(const oracle_scale_state* s, int weighting, double* JJout) {
  const int w = s->window_size;
  const double dp = 1;
  RectI bb{2 * w, 2 * w, s->bb_cols - 4 * w - 2, s->bb_rows - 4 * w - 2};
  const int P = 2 * w;
  double JJ = 0;
  std::vector<uint8_t> ta, tb, t0;
  for (int i = 0; i < s->n_left; ++i) {
    if (masked_out(s, i)) continue;
    if (!s->tri_left[i]) continue;
    if (s->last_left[i] == s->lframe) {
      const double* X = s->X_left + 4 * i;
      double T[16], Y[4], f[3], Z[4], f2[3], R[9];
      pose_T(s->q1, s->t1, T);
      R3_of(s->q1, R);
      double Xe[3] = {X[0] / X[3], X[1] / X[3], X[2] / X[3]};
      double Zc = 0; Zc += R[6] * Xe[0]; Zc += R[7] * Xe[1]; Zc += R[8] * Xe[2];
      Zc = Zc + s->t1[2];
      double duds = s->K2[0] * s->baseline / (s->scale * Zc);
      mul44x41(T, X, Y);
      proj_scaled_K(s->K1, s->scale, Y, f);
      P2f fl = to_euclid_f(f);
      for (int c = 0; c < 4; ++c) Z[c] = s->scale * Y[c];
      Z[0] = Z[0] - s->baseline;
      proj_K(s->K2, Z, f2);
      P2f frm = to_euclid_f(f2);
      P2f frp{(float)(f2[0] / f2[2] + dp), (float)(f2[1] / f2[2])};
      if (contains(bb, fl) && contains(bb, frm) && contains(bb, frp)) {
        int x0x = roi0(fl.x, w), x0y = roi0(fl.y, w);
        int x1x = roi0(frm.x, w), x1y = roi0(frm.y, w);
        int x2x = roi0(frp.x, w), x2y = roi0(frp.y, w);
        if (!roi_ok(x0x, x0y, P, P, s->cols, s->rows) || !roi_ok(x1x, x1y, P, P, s->cols, s->rows) ||
            !roi_ok(x2x, x2y, P, P, s->cols, s->rows)) return -2;
        double wv = weighting ? sobel_weight_view(s->imgL, s->stride, s->cols, s->rows, x0x, x0y, P, P) : 1.0;
        double MIp = mi_at(s->imgR, s->imgL, s->stride, x2x, x2y, x0x, x0y, P, P);
        double MIm = mi_at(s->imgR, s->imgL, s->stride, x1x, x1y, x0x, x0y, P, P);
        g_mi_evals += 2;
        double J = (MIp - MIm) / dp * duds;
        JJ += J * J * wv;
      }
    }
  }
  for (int i = 0; i < s->n_right; ++i) {
    if (masked_out(s, s->n_left + i)) continue;  // this loop indexes pts.first.size()+i (:593)
    if (!s->tri_right[i]) continue;
    if (s->last_right[i] == s->lframe) {
      double X[4]; std::memcpy(X, s->X_right + 4 * i, 32);
      X[0] = X[0] - s->baseline;
      double T[16], Y[4], f[3], Z[4], f2[3], R[9];
      pose_T(s->q1, s->t1, T);  // quirk: poses.first in the right-track loop (:598-602)
      R3_of(s->q1, R);
      double Xe[3] = {X[0] / X[3], X[1] / X[3], X[2] / X[3]};
      double Zc = 0; Zc += R[6] * Xe[0]; Zc += R[7] * Xe[1]; Zc += R[8] * Xe[2];
      Zc = Zc + s->t1[2];
      double duds = -s->K1[0] * s->baseline / (s->scale * Zc);
      mul44x41(T, X, Y);
      proj_scaled_K(s->K2, s->scale, Y, f);
      P2f fr = to_euclid_f(f);
      for (int c = 0; c < 4; ++c) Z[c] = s->scale * Y[c];
      Z[0] = Z[0] + s->baseline;
      proj_K(s->K1, Z, f2);
      P2f flm = to_euclid_f(f2);
      P2f flp{(float)(f2[0] / f2[2] + dp), (float)(f2[1] / f2[2])};
      if (contains(bb, fr) && contains(bb, flm) && contains(bb, flp)) {
        int x0x = roi0(fr.x, w), x0y = roi0(fr.y, w);
        int x1x = roi0(flm.x, w), x1y = roi0(flm.y, w);
        int x2x = roi0(flp.x, w), x2y = roi0(flp.y, w);
        if (!roi_ok(x0x, x0y, P, P, s->cols, s->rows) || !roi_ok(x1x, x1y, P, P, s->cols, s->rows) ||
            !roi_ok(x2x, x2y, P, P, s->cols, s->rows)) return -2;
        double wv = 1.0;
        if (weighting) {
          t0.resize(P * P);
          for (int y = 0; y < P; ++y) for (int x = 0; x < P; ++x)
            t0[y * P + x] = s->imgR[(long)(x0y + y) * s->stride + x0x + x] ? 255 : 0;
          wv = sobel_weight_isolated(t0.data(), P, P);
        }
        // ROIs * 255 (saturating 8U) then convertTo(CV_32F) -> binary {0,255} patches (:614-619)
        double MIp = mi_binarized(s->imgL, s->imgR, s->stride, x2x, x2y, x0x, x0y, P, P, ta, tb);
        double MIm = mi_binarized(s->imgL, s->imgR, s->stride, x1x, x1y, x0x, x0y, P, P, ta, tb);
        g_mi_evals += 2;
        double J = (MIp - MIm) / dp * duds;
        JJ += J * J * wv;
      }
    }
  }
  *JJout = JJ;
  return 0;
}

namespace {
double sumsq(const std::vector<double>& r, int n) {
  double s = 0;
  for (int i = 0; i < n; ++i) s += r[i] * r[i];
  return s;
}
// Eigen LDLT::solve on a 1x1 system (pseudo-inverse of D below DBL_MIN)
double ldlt1(double JJ, double e) {
  return std::fabs(JJ) > 2.2250738585072014e-308 ? e / JJ : 0.0;
}
}  // namespace

// optimisation.cpp:29-147 (+ run_GN_step :674-683, run_LM_step :685-730)
extern "C" int oracle_scale_optimise(oracle_scale_state* s_in, const oracle_optim_params* p_in, int test,
                                     int* iterations, double* trace, int trace_cap, long* mi_evals) {
  oracle_optim_params p = *p_in;
  oracle_scale_state st = *s_in;
  g_mi_evals = 0;
  g_res_calls = g_neq_calls = g_rejections = 0;
  int stop = NO_STOP;
  if (test) { p.type = 0; p.max_nb_iter = 300; p.abs_tol = 0; p.incr_tol = 0; p.grad_tol = 0; p.rel_tol = 0; }
  const int ntot = s_in->n_left + s_in->n_right;
  std::vector<double> r(ntot > 0 ? ntot : 1), rt(ntot > 0 ? ntot : 1);
  int k = 0;
  int ntrace = 0;
  do {
    int rows = oracle_scale_residuals(&st, p.weighting, r.data());
    ++g_res_calls;
    if (rows < 0) return -100 + rows;
    double e1 = sumsq(r, rows);
    double mre = e1 / (double)(rows * 1);
    if (mre < p.abs_tol) stop = SMALL_REPROJ_ERROR;
    double JJ, e;
    if (test) { JJ = 75; e = 1; }
    else { int rc = oracle_scale_normal_equations(&st, p.weighting, r.data(), &JJ, &e); ++g_neq_calls; if (rc < 0) return -100 + rc; }
    if (k == 0) p.mu = JJ;
    if (std::sqrt(e * e) < p.grad_tol) stop = SMALL_GRADIENT;
    double dX = 0;
    if (p.type == 0) {
      JJ += p.mu;
      dX = ldlt1(JJ, e);
      st.scale += p.alpha * dX;
    } else {
      for (;;) {
        JJ += p.mu;
        dX = ldlt1(JJ, e);
        if (std::sqrt(dX * dX) <= p.incr_tol) { stop = SMALL_INCREMENT; break; }
        oracle_scale_state tmp = st;
        tmp.scale += p.alpha * dX;
        int rows2 = oracle_scale_residuals(&tmp, p.weighting, rt.data());
        ++g_res_calls;
        if (rows2 < 0) return -100 + rows2;
        double e2 = sumsq(rt, rows2);
        double rho = (p.minim ? -1.0 : 1.0) * (e2 - e1);
        if (rho > 0) {
          p.mu *= std::max(1.0 / 3.0, 1 - std::pow(2 * rho - 1, 3));
          p.v = 2;
          double dd = std::sqrt(e1) - std::sqrt(e2);
          if (dd * dd < p.rel_tol * std::sqrt(e1)) stop = SMALL_DECREASE_FUNCTION;
          st = tmp;
          break;
        } else {
          ++g_rejections;
          p.mu *= p.v;
          double v2 = 2 * p.v;
          if (v2 <= p.v) { stop = NO_CONVERGENCE; break; }
          p.v = v2;
        }
      }
    }
    if (!stop && std::sqrt(dX * dX) <= p.incr_tol) stop = SMALL_INCREMENT;
    int rows3 = oracle_scale_residuals(&st, p.weighting, rt.data());
    ++g_res_calls;
    if (rows3 < 0) return -100 + rows3;
    double e2 = sumsq(rt, rows3);
    if (p.type == 0 && (e2 - e1) * (e2 - e1) < p.rel_tol) stop = SMALL_DECREASE_FUNCTION;
    if (trace && ntrace < trace_cap) { trace[2 * ntrace] = e1; trace[2 * ntrace + 1] = st.scale; ntrace++; }
  } while (!stop && k++ < p.max_nb_iter);
  if (k == p.max_nb_iter) stop = MAX_ITERATIONS;
  s_in->scale = st.scale;
  if (iterations) *iterations = ntrace;
  if (mi_evals) *mi_evals = g_mi_evals;
  return stop;
}

// ScaleState::compute_residuals (optimisation.cpp:230-278), evident intent:
// the 2w x 2w patch pairs of the left tracks stacked into one tall image pair
// (rows = pairs * 2w), then computeMutualInformation on it.  The reference's
// `left_img(Range..) = imgs[i].first` (:273-274) copies nothing (it rebinds a
// temporary header), so the literal reference reads uninitialised memory:
// parity unpinned.  Returns 0, -1 (no pair: computeMutualInformation asserts,
// mutual_information.cpp:57) or -2 (ROI outside the image: cv::Exception).
extern "C" int oracle_scale_state_mi(const oracle_scale_state* s, double* out, int* npairs) {
  const int w = s->window_size, P = 2 * w;
  RectI bb{w, w, s->bb_cols - 2 * w, s->bb_rows - 2 * w};  // :232 (no -1)
  std::vector<uint8_t> L, R;
  int n = 0;
  for (int i = 0; i < s->n_left; ++i) {
    if (!s->tri_left[i] || s->last_left[i] != s->lframe) continue;  // :246-248
    double T[16], Y[4], f[3], Z[4], f2[3];
    pose_T(s->q1, s->t1, T);
    mul44x41(T, s->X_left + 4 * i, Y);
    proj_scaled_K(s->K1, s->scale, Y, f);
    P2f fl = to_euclid_f(f);
    for (int c = 0; c < 4; ++c) Z[c] = s->scale * Y[c];
    Z[0] = Z[0] - s->baseline;
    proj_K(s->K2, Z, f2);
    P2f fr = to_euclid_f(f2);
    if (!(contains(bb, fl) && contains(bb, fr))) continue;  // :257
    int lx = roi0(fl.x, w), ly = roi0(fl.y, w), rx = roi0(fr.x, w), ry = roi0(fr.y, w);
    if (!roi_ok(lx, ly, P, P, s->cols, s->rows) || !roi_ok(rx, ry, P, P, s->cols, s->rows)) return -2;
    for (int y = 0; y < P; ++y)
      for (int x = 0; x < P; ++x) {
        L.push_back(s->imgL[(long)(ly + y) * s->stride + lx + x]);
        R.push_back(s->imgR[(long)(ry + y) * s->stride + rx + x]);
      }
    ++n;
  }
  if (npairs) *npairs = n;
  if (n == 0) return -1;
  *out = (double)oracle_mutual_information(L.data(), P, R.data(), P, P, n * P);  // :277
  return 0;
}

extern "C" void oracle_scale_counters(long* out3) {
  out3[0] = g_res_calls;
  out3[1] = g_neq_calls;
  out3[2] = g_rejections;
}

// optimisation.cpp:732-747
extern "C" int oracle_scale_inliers(const oracle_scale_state* s, double threshold, int* idx, int cap) {
  oracle_scale_state t = *s;
  t.mask = nullptr; t.mask_len = 0;
  std::vector<double> r(s->n_left + s->n_right + 1);
  int rows = oracle_scale_residuals(&t, 0, r.data());
  if (rows < 0) return rows;
  int n = 0;
  for (int i = 0; i < rows; ++i)
    if (std::sqrt(r[i] * r[i]) < threshold) { if (n < cap) idx[n] = i; n++; }
  return n;
}
