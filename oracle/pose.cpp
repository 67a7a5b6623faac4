// Oracle (test infrastructure only): pose-covariance propagation of
// src/core/feature_types.cpp:171-251 and the quaternion helpers it uses
// (include/MotionEstimation/core/rotation_utils.h:190-267,
// src/core/rotation_utils.cpp:218-226, 253-311, 357-368), restated with
// plain arrays in the reference's evaluation order.
//
// OpenCV trap reproduced: `((cv::Mat) cv::Mat::eye(3,3,CV_32F)).copyTo(J(...))`
// on a CV_64F J reallocates the temporary ROI header instead of writing into
// J (Mat::copyTo -> create() with a different type), so those blocks of J
// stay ZERO: J(0:3, 6:9) in poseMultiplicationWithCovarianceReverse (:205)
// and J(3:6, 3:6) in invertPoseWithCovariance (:231).
#include <cmath>
#include <cstring>
#include "oracle.h"

namespace {

struct Q { double w, x, y, z; };

Q qnorm(Q q) {  // Quat::normalize (rotation_utils.cpp:218-226); every constructor normalises
  const double n = std::sqrt(q.w * q.w + q.x * q.x + q.y * q.y + q.z * q.z);
  if (n != 0.0) { q.w /= n; q.x /= n; q.y /= n; q.z /= n; }
  return q;
}
Q qmul(const Q& a, const Q& q) {  // Quat::operator* (:261-266)
  return qnorm(Q{a.w * q.w - (a.x * q.x + a.y * q.y + a.z * q.z), a.w * q.x + a.x * q.w + a.y * q.z - a.z * q.y,
                 a.w * q.y - a.x * q.z + a.y * q.w + a.z * q.x, a.w * q.z + a.x * q.y - a.y * q.x + a.z * q.w});
}
Q qconj(const Q& q) { return qnorm(Q{q.w, -q.x, -q.y, -q.z}); }
void R3(const Q& q, double R[9]) {  // getR3 (rotation_utils.h:232-237)
  const double w = q.w, x = q.x, y = q.y, z = q.z;
  const double r[9] = {w * w + x * x - y * y - z * z, 2 * (x * y - w * z), 2 * (x * z + w * y),
                       2 * (x * y + w * z), w * w - x * x + y * y - z * z, 2 * (y * z - w * x),
                       2 * (x * z - w * y), 2 * (y * z + w * x), w * w - x * x - y * y + z * z};
  std::memcpy(R, r, sizeof(r));
}
void rot(const Q& q, const double v[3], double out[3]) {  // Quat * Vec3 = getR3() * v
  double R[9];
  R3(q, R);
  for (int i = 0; i < 3; ++i) out[i] = R[3 * i] * v[0] + R[3 * i + 1] * v[1] + R[3 * i + 2] * v[2];
}
void logq(const Q& q, double v[3]) {  // log_map_Quat (rotation_utils.h:198-204)
  const double norm = std::sqrt(std::pow(q.x, 2) + std::pow(q.y, 2) + std::pow(q.z, 2));
  const double theta = norm < 1e-10 ? 1e-10 : norm;
  const double a = std::acos(q.w) * 2.0;
  v[0] = a * (q.x / theta);
  v[1] = a * (q.y / theta);
  v[2] = a * (q.z / theta);
}
void Gqv(const double v[3], double G[12]) {  // Gq_v (rotation_utils.cpp:357-368), 4x3
  const double snorm = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
  const double norm = std::sqrt(snorm) + 1e-20;
  const double a = std::cos(0.5 * norm) * norm - 2 * std::sin(0.5 * norm);
  const double s = snorm * std::sin(0.5 * norm);
  const double m[12] = {-v[0] * s, -v[1] * s, -v[2] * s,
                        2 * s + v[0] * v[0] * a, v[0] * v[1] * a, v[0] * v[2] * a,
                        v[0] * v[1] * a, 2 * s + v[1] * v[1] * a, v[1] * v[2] * a,
                        v[0] * v[2] * a, v[1] * v[2] * a, 2 * s + v[2] * v[2] * a};
  const double f = 1 / (2 * std::pow(norm, 3));
  for (int i = 0; i < 12; ++i) G[i] = f * m[i];
}
void getG(const Q& q, double G[12]) { double v[3]; logq(q, v); Gqv(v, G); }
void getQl(const Q& q, double M[16]) {  // rotation_utils.h:240-243
  const double m[16] = {q.w, -q.x, -q.y, -q.z, q.x, q.w, -q.z, q.y, q.y, q.z, q.w, -q.x, q.z, -q.y, q.x, q.w};
  std::memcpy(M, m, sizeof(m));
}
void getQr(const Q& q, double M[16]) {  // :245-248
  const double m[16] = {q.w, -q.x, -q.y, -q.z, q.x, q.w, q.z, -q.y, q.y, -q.z, q.w, q.x, q.z, q.y, -q.x, q.w};
  std::memcpy(M, m, sizeof(m));
}
void getH(const Q& q, double H[12]) {  // :255-260, 3x4
  const double c = 1.0 / (1 - q.w * q.w + 1e-20);
  const double d = std::acos(q.w) / std::sqrt(1 - q.w * q.w + 1e-20);
  const double m[12] = {2 * c * q.x * (d * q.w - 1), 2 * d, 0, 0, 2 * c * q.y * (d * q.w - 1), 0, 2 * d, 0,
                        2 * c * q.z * (d * q.w - 1), 0, 0, 2 * d};
  std::memcpy(H, m, sizeof(m));
}
void matmul(const double* A, const double* B, double* C, int n, int k, int m) {
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < m; ++j) {
      double s = 0;
      for (int t = 0; t < k; ++t) s += A[i * k + t] * B[t * m + j];
      C[i * m + j] = s;
    }
}
void getH_qvec(const Q& q, const double x[3], double out[9]) {  // :262-268
  const double qv[3] = {q.x, q.y, q.z};
  double D[12];  // 3x4 dqxdq
  // column 0: 2 w x + 2 [q]x x
  const double sk[3] = {-qv[2] * x[1] + qv[1] * x[2], qv[2] * x[0] - qv[0] * x[2], -qv[1] * x[0] + qv[0] * x[1]};
  for (int i = 0; i < 3; ++i) D[4 * i] = 2 * q.w * x[i] + 2 * sk[i];
  // columns 1..3: 2 ((q.x) I + q x^T - x q^T - w [x]x)
  const double dot = qv[0] * x[0] + qv[1] * x[1] + qv[2] * x[2];
  const double skx[9] = {0, -x[2], x[1], x[2], 0, -x[0], -x[1], x[0], 0};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      D[4 * i + 1 + j] = 2 * ((i == j ? dot : 0.0) + qv[i] * x[j] - x[i] * qv[j] - q.w * skx[3 * i + j]);
  double G[12];
  getG(q, G);
  matmul(D, G, out, 3, 4, 3);
}
void HQG(const Q& h, const double* Qm, const Q& g, double out[9]) {  // H(h) * Qm * G(g)
  double H[12], G[12], T[16];
  getH(h, H);
  getG(g, G);
  matmul(H, Qm, T, 3, 4, 4);
  matmul(T, G, out, 3, 4, 3);
}
void put(double* J, int ld, int r0, int c0, const double* B, int rows, int cols, double sign = 1.0) {
  for (int i = 0; i < rows; ++i)
    for (int j = 0; j < cols; ++j) J[(r0 + i) * ld + c0 + j] = sign * B[i * cols + j];
}
// new_cov = J * aug * J^T (cv::Mat products, double)
void sandwich(const double* J, const double* aug, int n, int m, double* out) {
  double T[6 * 12];
  matmul(J, aug, T, n, m, m);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double s = 0;
      for (int t = 0; t < m; ++t) s += T[i * m + t] * J[j * m + t];
      out[i * n + j] = s;
    }
}
Q load(const double* q) { return qnorm(Q{q[0], q[1], q[2], q[3]}); }
void store(const Q& q, double* o) { o[0] = q.w; o[1] = q.x; o[2] = q.y; o[3] = q.z; }

}  // namespace

// pose = {q (w,x,y,z) 4, t 3}, cov 36 (row-major)
extern "C" void oracle_pose_mul_cov(const double* q1d, const double* t1, const double* c1, const double* q2d,
                                    const double* t2, const double* c2, int reverse, double* q3o, double* t3o,
                                    double* c3o) {
  const Q q1 = load(q1d), q2 = load(q2d);
  double aug[144] = {0};
  put(aug, 12, 0, 0, c1, 6, 6);
  put(aug, 12, 6, 6, c2, 6, 6);
  double J[72] = {0};
  Q q3;
  double t3[3], R[9], M[16], B[9];
  if (!reverse) {  // P3 = P1 * P2 (feature_types.cpp:171-194)
    q3 = qmul(q1, q2);
    rot(q1, t2, t3);
    for (int i = 0; i < 3; ++i) t3[i] = t3[i] + t1[i];
    const double I3[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    put(J, 12, 0, 0, I3, 3, 3);
    getH_qvec(q1, t2, B);
    put(J, 12, 0, 3, B, 3, 3);
    R3(q1, R);
    put(J, 12, 0, 6, R, 3, 3);
    getQr(q2, M);
    HQG(q3, M, q1, B);
    put(J, 12, 3, 3, B, 3, 3);
    getQl(q1, M);
    HQG(q3, M, q2, B);
    put(J, 12, 3, 9, B, 3, 3);
  } else {  // P3 = P2 * P1 (:196-219)
    q3 = qmul(q2, q1);
    rot(q2, t1, t3);
    for (int i = 0; i < 3; ++i) t3[i] = t3[i] + t2[i];
    R3(q2, R);
    put(J, 12, 0, 0, R, 3, 3);
    // J(0:3, 6:9) = eye(CV_32F): not written (the trap above)
    getH_qvec(q2, t1, B);
    put(J, 12, 0, 9, B, 3, 3);
    getQl(q2, M);
    HQG(q3, M, q1, B);
    put(J, 12, 3, 3, B, 3, 3);
    getQr(q1, M);
    HQG(q3, M, q2, B);
    put(J, 12, 3, 9, B, 3, 3);
  }
  sandwich(J, aug, 6, 12, c3o);
  store(q3, q3o);
  std::memcpy(t3o, t3, sizeof(t3));
}

extern "C" void oracle_pose_invert_cov(double* qd, double* t, double* cov) {  // :221-236
  const Q q = load(qd), qc = qconj(q);
  double J[36] = {0}, R[9], B[9];
  R3(qc, R);
  put(J, 6, 0, 0, R, 3, 3, -1.0);
  getH_qvec(qc, t, B);
  put(J, 6, 0, 3, B, 3, 3);
  // J(3:6, 3:6) = -eye(CV_32F): not written (the trap above)
  double tn[3];
  rot(qc, t, tn);
  for (int i = 0; i < 3; ++i) t[i] = -tn[i];
  store(qc, qd);
  double out[36];
  sandwich(J, cov, 6, 6, out);
  std::memcpy(cov, out, sizeof(out));
}

extern "C" void oracle_pose_scale_cov(double* t, double* cov, double s, double var) {  // :238-251
  double aug[49] = {0}, J[42] = {0};
  put(aug, 7, 0, 0, cov, 6, 6);
  aug[48] = var;
  for (int i = 0; i < 3; ++i) J[i * 7 + i] = 1.0 * s;
  for (int i = 3; i < 6; ++i) J[i * 7 + i] = 1.0;
  for (int i = 0; i < 3; ++i) J[i * 7 + 6] = t[i];
  double out[36];
  sandwich(J, aug, 6, 7, out);
  std::memcpy(cov, out, sizeof(out));
  for (int i = 0; i < 3; ++i) t[i] *= s;
}
