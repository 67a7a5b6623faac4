// oracle/mono.cpp -- CPU restatement of MonoVisualOdometry::process
// (src/vo/MonoVisualOdometry.cpp:7-73; include/MotionEstimation/vo/
// MonoVisualOdometry.h:21-28 parameters).  TEST INFRASTRUCTURE ONLY (see
// oracle.h): the checker of csrc/mono.hip.
//
// The reference calls OpenCV's findEssentialMat (five-point solver inside a
// RANSAC or LMedS registrator) and recoverPose.  OpenCV is absent here, so both
// are restated from their published algorithms -- PARITY UNPINNED:
//  * matches with f1.x > 0 and f2.x > 0 (MonoVisualOdometry.cpp:13-17),
//    normalised by K: ((x - cu) / fu, (y - cv) / fv); the pixel threshold
//    divided by (fu + fv) / 2 (findEssentialMat);
//  * five-point relative pose (Nister 2004): null space of the 5 x 9 epipolar
//    system (the four smallest eigenvectors of Q^T Q, cyclic Jacobi: OpenCV's
//    last right singular vectors), the ten cubic constraints det(E) = 0 and
//    2 E E^T E - tr(E E^T) E = 0 over the 20 monomials in Nister's order,
//    Gauss-Jordan of the first ten columns, the 3 x 3 polynomial matrix in z
//    whose determinant is the degree-10 polynomial, its real roots (isolated
//    between the real roots of its derivatives, then bisected), (x, y) from the
//    null vector of B(z), E = x X + y Y + z Z + W normalised to unit norm;
//  * RANSAC as OpenCV's RANSACPointSetRegistrator: cv::RNG seeded with
//    (uint64)-1, subsets of 5 distinct indices by rng.uniform(0, count),
//    Sampson error stored as float against (float)(t * t), a model replaces the
//    best one only with more inliers than max(best, 4), the iteration bound
//    updated by RANSACUpdateNumIters(prob, outlier ratio, 5, bound);
//    maxIters 1000.  LMedS (param ransac = false): fixed iterations
//    round(log(1 - prob) / log(1 - 0.55^5)) (>= 3, <= 1000), the model of least
//    median error (k = count / 2), inliers at
//    sigma = max(2.5 * 1.4826 * (1 + 5 / (count - 5)) * sqrt(median), 0.001)
//    (the 0.001 floor restated from OpenCV's ptsetreg.cpp; unpinned here);
//  * recoverPose (distance threshold 500, as the reference passes): E = U D V^T
//    (det-corrected), R1 = U W V^T, R2 = U W^T V^T, t = U[:, 2]; per pose each
//    inlier triangulated by the DLT (right singular vector of the 4 x 4 system
//    = eigenvector of A^T A, cyclic Jacobi) and kept if in front of both
//    cameras within the distance; the pose with the most points (R1 t, R2 t,
//    R1 -t, R2 -t in that order on ties); the mask becomes mask & that pose's
//    points;
//  * fewer than 10 inliers -> identity motion, false (:46-49); fewer than 8
//    matches -> identity, false (:67-71).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "oracle.h"

namespace {

// OpenCV cv::RNG (multiply-with-carry), state (uint64)-1 as RANSAC seeds it
struct CvRng {
  uint64_t s;
  unsigned next() {
    s = (uint64_t)(unsigned)s * 4164903690u + (unsigned)(s >> 32);
    return (unsigned)s;
  }
  int uniform(int a, int b) { return a == b ? a : (int)(next() % (unsigned)(b - a)) + a; }
};

// ---- polynomials in (x, y, z): linear (4 terms: x y z 1), quadratic (10:
// x^2 y^2 z^2 xy xz yz x y z 1), cubic (20, Nister's order: x^3 y^3 x^2y xy^2
// x^2z x^2 y^2z y^2 xyz xy | xz^2 xz x yz^2 yz y z^3 z^2 z 1)
const int kLin[4][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, 0}};
const int kQuad[10][3] = {{2, 0, 0}, {0, 2, 0}, {0, 0, 2}, {1, 1, 0}, {1, 0, 1},
                          {0, 1, 1}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, 0}};
const int kMono[20][3] = {{3, 0, 0}, {0, 3, 0}, {2, 1, 0}, {1, 2, 0}, {2, 0, 1}, {2, 0, 0}, {0, 2, 1},
                          {0, 2, 0}, {1, 1, 1}, {1, 1, 0}, {1, 0, 2}, {1, 0, 1}, {1, 0, 0}, {0, 1, 2},
                          {0, 1, 1}, {0, 1, 0}, {0, 0, 3}, {0, 0, 2}, {0, 0, 1}, {0, 0, 0}};
int quad_index(int a, int b, int c) {
  for (int k = 0; k < 10; ++k)
    if (kQuad[k][0] == a && kQuad[k][1] == b && kQuad[k][2] == c) return k;
  return -1;
}
int mono_index(int a, int b, int c) {
  for (int k = 0; k < 20; ++k)
    if (kMono[k][0] == a && kMono[k][1] == b && kMono[k][2] == c) return k;
  return -1;
}
// r (quadratic) = p * q (linear x linear), terms accumulated i (p) outer, j (q) inner
void mul_ll(const double* p, const double* q, double* r) {
  for (int k = 0; k < 10; ++k) r[k] = 0.0;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      r[quad_index(kLin[i][0] + kLin[j][0], kLin[i][1] + kLin[j][1], kLin[i][2] + kLin[j][2])] += p[i] * q[j];
}
// r (cubic) = p * q (quadratic x linear)
void mul_ql(const double* p, const double* q, double* r) {
  for (int k = 0; k < 20; ++k) r[k] = 0.0;
  for (int i = 0; i < 10; ++i)
    for (int j = 0; j < 4; ++j)
      r[mono_index(kQuad[i][0] + kLin[j][0], kQuad[i][1] + kLin[j][1], kQuad[i][2] + kLin[j][2])] += p[i] * q[j];
}

// ---- univariate polynomials (c[k] multiplies z^k)
double horner(const double* c, int deg, double z) {
  double v = c[deg];
  for (int k = deg - 1; k >= 0; --k) v = v * z + c[k];
  return v;
}
// one level of the isolation: the real roots of c[0..deg] (ascending), given
// the real roots crit[0..nc) of its derivative; each interval between two
// consecutive critical points (and the Cauchy bounds) holds at most one root,
// bisected to the last representable step
int roots_between(const double* c, int deg, const double* crit, int nc, double* out) {
  if (deg == 1) {
    out[0] = -c[0] / c[1];
    return 1;
  }
  double bound = 0.0;
  for (int k = 0; k < deg; ++k) bound = std::max(bound, std::fabs(c[k] / c[deg]));
  bound += 1.0;
  int n = 0;
  for (int i = 0; i <= nc; ++i) {
    double lo = i == 0 ? -bound : crit[i - 1], hi = i == nc ? bound : crit[i];
    if (!(lo < hi)) continue;
    double flo = horner(c, deg, lo);
    const double fhi = horner(c, deg, hi);
    if (flo == 0.0) {
      if (n == 0 || out[n - 1] != lo) out[n++] = lo;
      continue;
    }
    if (fhi == 0.0 || (flo < 0) == (fhi < 0)) continue;  // (a root at hi is found as the next lo)
    for (int it = 0; it < 2100; ++it) {
      const double mid = 0.5 * (lo + hi);
      if (mid <= lo || mid >= hi) break;
      const double fm = horner(c, deg, mid);
      if (fm == 0.0) {
        lo = mid;
        break;
      }
      if ((fm < 0) == (flo < 0)) {
        lo = mid;
        flo = fm;
      } else {
        hi = mid;
      }
    }
    out[n++] = lo;
  }
  return n;
}
// real roots of c[0..deg] (deg <= 10), ascending: the derivative chain
// (leading zeros stripped at every level), roots from the linear end up
int real_roots(const double* c, int deg, double* out) {
  double chain[11][11];
  int dg[11];
  int L = 0;
  for (int k = 0; k <= deg; ++k) chain[0][k] = c[k];
  dg[0] = deg;
  while (dg[L] > 0 && chain[L][dg[L]] == 0.0) --dg[L];
  while (dg[L] > 1) {
    for (int k = 1; k <= dg[L]; ++k) chain[L + 1][k - 1] = k * chain[L][k];
    dg[L + 1] = dg[L] - 1;
    ++L;
    while (dg[L] > 0 && chain[L][dg[L]] == 0.0) --dg[L];
  }
  if (dg[L] <= 0) {  // (a constant at the end of the chain: no roots below it)
    if (L == 0) return 0;
  }
  double rts[11], tmp[11];
  int nr = 0;
  for (int l = L; l >= 0; --l) {
    if (dg[l] <= 0) {
      nr = 0;
      continue;
    }
    nr = roots_between(chain[l], dg[l], rts, nr, tmp);
    for (int k = 0; k < nr; ++k) rts[k] = tmp[k];
  }
  for (int k = 0; k < nr; ++k) out[k] = rts[k];
  return nr;
}

// symmetric eigen decomposition (cyclic Jacobi), eigenvalues ascending,
// eigenvectors as columns of V (row-major n x n)
void jacobi_eig(double* a, int n, double* w, double* V) {
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) V[i * n + j] = i == j ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0.0;
    for (int p = 0; p < n; ++p)
      for (int q = p + 1; q < n; ++q) off += a[p * n + q] * a[p * n + q];
    if (off == 0.0) break;
    for (int p = 0; p < n; ++p)
      for (int q = p + 1; q < n; ++q) {
        const double apq = a[p * n + q];
        if (apq == 0.0) continue;
        const double theta = (a[q * n + q] - a[p * n + p]) / (2.0 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
        const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < n; ++k) {  // columns p, q
          const double akp = a[k * n + p], akq = a[k * n + q];
          a[k * n + p] = c * akp - s * akq;
          a[k * n + q] = s * akp + c * akq;
        }
        for (int k = 0; k < n; ++k) {  // rows p, q
          const double apk = a[p * n + k], aqk = a[q * n + k];
          a[p * n + k] = c * apk - s * aqk;
          a[q * n + k] = s * apk + c * aqk;
        }
        for (int k = 0; k < n; ++k) {
          const double vkp = V[k * n + p], vkq = V[k * n + q];
          V[k * n + p] = c * vkp - s * vkq;
          V[k * n + q] = s * vkp + c * vkq;
        }
      }
  }
  // sort ascending (selection, stable on ties)
  for (int i = 0; i < n; ++i) w[i] = a[i * n + i];
  for (int i = 0; i < n; ++i) {
    int m = i;
    for (int j = i + 1; j < n; ++j)
      if (w[j] < w[m]) m = j;
    if (m != i) {
      std::swap(w[i], w[m]);
      for (int k = 0; k < n; ++k) std::swap(V[k * n + i], V[k * n + m]);
    }
  }
}

// null space of the 5 x 9 epipolar system: the eigenvectors of Q^T Q with
// the four smallest eigenvalues (OpenCV: the last four right singular vectors
// of Q), an orthonormal basis X, Y, Z, W (W: the smallest)
bool null4(const double q[5][9], double ns[4][9]) {
  double QtQ[81], w[9], V[81];
  for (int i = 0; i < 9; ++i)
    for (int j = 0; j < 9; ++j) {
      double s = 0.0;
      for (int k = 0; k < 5; ++k) s += q[k][i] * q[k][j];
      QtQ[9 * i + j] = s;
    }
  jacobi_eig(QtQ, 9, w, V);
  for (int v = 0; v < 4; ++v)
    for (int k = 0; k < 9; ++k) ns[v][k] = V[9 * k + (3 - v)];  // X, Y, Z by descending eigenvalue, W the smallest
  return w[4] > 0.0;
}

// five-point solver: up to 10 essential matrices (row-major 3 x 3, unit norm)
int five_point(const double* x1, const double* x2, double* E_out) {
  double q[5][9];
  for (int i = 0; i < 5; ++i) {
    const double u1 = x1[2 * i], v1 = x1[2 * i + 1], u2 = x2[2 * i], v2 = x2[2 * i + 1];
    // x2^T E x1 = 0 with E row-major: e00 u2 u1 + e01 u2 v1 + e02 u2 + e10 v2 u1 + ...
    q[i][0] = u2 * u1;
    q[i][1] = u2 * v1;
    q[i][2] = u2;
    q[i][3] = v2 * u1;
    q[i][4] = v2 * v1;
    q[i][5] = v2;
    q[i][6] = u1;
    q[i][7] = v1;
    q[i][8] = 1.0;
  }
  double ns[4][9];
  if (!null4(q, ns)) return 0;
  // E(x, y, z) = x X + y Y + z Z + W: entry (i, j) as a linear polynomial
  double E[9][4];
  for (int e = 0; e < 9; ++e)
    for (int v = 0; v < 4; ++v) E[e][v] = ns[v][e];
  double A[10][20];
  double t1[10], t2[10], m[10], cub[20];
  // row 0: det(E) = e00 (e11 e22 - e12 e21) - e01 (e10 e22 - e12 e20) + e02 (e10 e21 - e11 e20)
  const int cof[3][4] = {{1, 2, 2, 1}, {0, 2, 2, 0}, {0, 1, 1, 0}};
  for (int k = 0; k < 20; ++k) A[0][k] = 0.0;
  for (int j = 0; j < 3; ++j) {
    mul_ll(E[3 + cof[j][0]], E[6 + cof[j][1]], t1);
    mul_ll(E[3 + cof[j][2]], E[6 + cof[j][3]], t2);
    for (int k = 0; k < 10; ++k) m[k] = t1[k] - t2[k];
    mul_ql(m, E[j], cub);
    for (int k = 0; k < 20; ++k) A[0][k] += j == 1 ? -cub[k] : cub[k];
  }
  // rows 1..9: 2 (E E^T) E - tr(E E^T) E, entry (i, j) row-major
  double EEt[9][10], tr[10];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      for (int k = 0; k < 10; ++k) EEt[3 * i + j][k] = 0.0;
      for (int k = 0; k < 3; ++k) {
        mul_ll(E[3 * i + k], E[3 * j + k], t1);
        for (int u = 0; u < 10; ++u) EEt[3 * i + j][u] += t1[u];
      }
    }
  for (int k = 0; k < 10; ++k) tr[k] = EEt[0][k] + EEt[4][k] + EEt[8][k];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double* row = A[1 + 3 * i + j];
      for (int k = 0; k < 20; ++k) row[k] = 0.0;
      for (int k = 0; k < 3; ++k) {
        mul_ql(EEt[3 * i + k], E[3 * k + j], cub);
        for (int u = 0; u < 20; ++u) row[u] += 2.0 * cub[u];
      }
      mul_ql(tr, E[3 * i + j], cub);
      for (int u = 0; u < 20; ++u) row[u] -= cub[u];
    }
  // Gauss-Jordan: [A1 | A2] -> [I | G]
  for (int col = 0; col < 10; ++col) {
    int best = col;
    for (int i = col + 1; i < 10; ++i)
      if (std::fabs(A[i][col]) > std::fabs(A[best][col])) best = i;
    if (!(std::fabs(A[best][col]) > 0.0)) return 0;
    if (best != col)
      for (int k = 0; k < 20; ++k) std::swap(A[col][k], A[best][k]);
    const double inv = 1.0 / A[col][col];
    for (int k = col; k < 20; ++k) A[col][k] *= inv;
    for (int i = 0; i < 10; ++i) {
      if (i == col) continue;
      const double f = A[i][col];
      if (f != 0.0)
        for (int k = col; k < 20; ++k) A[i][k] -= f * A[col][k];
    }
  }
  // rows (4,5), (6,7), (8,9): x^2 z = z x^2, y^2 z = z y^2, xyz = z xy ->
  // B(z) [x y 1]^T = 0 with coefficient polynomials in z (deg 3, 3, 4)
  double B[3][3][5];
  for (int r = 0; r < 3; ++r) {
    const double* p = A[4 + 2 * r] + 10;
    const double* q2 = A[5 + 2 * r] + 10;
    for (int s = 0; s < 2; ++s) {  // x (rest 0..2), y (rest 3..5)
      const int o = 3 * s;
      B[r][s][0] = p[o + 2];
      B[r][s][1] = p[o + 1] - q2[o + 2];
      B[r][s][2] = p[o + 0] - q2[o + 1];
      B[r][s][3] = -q2[o + 0];
      B[r][s][4] = 0.0;
    }
    B[r][2][0] = p[9];
    B[r][2][1] = p[8] - q2[9];
    B[r][2][2] = p[7] - q2[8];
    B[r][2][3] = p[6] - q2[7];
    B[r][2][4] = -q2[6];
  }
  // det B(z): degree-10 polynomial (products of coefficient arrays)
  auto pmul = [](const double* a, int da, const double* b, int db, double* r) {
    for (int k = 0; k <= da + db; ++k) r[k] = 0.0;
    for (int i = 0; i <= da; ++i)
      for (int j = 0; j <= db; ++j) r[i + j] += a[i] * b[j];
  };
  double poly[11] = {0}, m1[9], m2[9], mdiff[9], term[14];
  const int cj[3][4] = {{1, 2, 2, 1}, {0, 2, 2, 0}, {0, 1, 1, 0}};
  for (int j = 0; j < 3; ++j) {
    const int a0 = cj[j][0], a1 = cj[j][1], b0 = cj[j][2], b1 = cj[j][3];
    const int da0 = a0 == 2 ? 4 : 3, da1 = a1 == 2 ? 4 : 3, db0 = b0 == 2 ? 4 : 3, db1 = b1 == 2 ? 4 : 3;
    pmul(B[1][a0], da0, B[2][a1], da1, m1);
    pmul(B[1][b0], db0, B[2][b1], db1, m2);
    const int dm = std::max(da0 + da1, db0 + db1);
    for (int k = 0; k <= dm; ++k) mdiff[k] = (k <= da0 + da1 ? m1[k] : 0.0) - (k <= db0 + db1 ? m2[k] : 0.0);
    const int d0 = j == 2 ? 4 : 3;
    pmul(B[0][j], d0, mdiff, dm, term);
    for (int k = 0; k <= d0 + dm && k <= 10; ++k) poly[k] += (j == 1 ? -term[k] : term[k]);
  }
  double roots[10];
  const int nr = real_roots(poly, 10, roots);
  int count = 0;
  for (int k = 0; k < nr; ++k) {
    const double z = roots[k];
    double Bz[3][3];
    for (int r = 0; r < 3; ++r)
      for (int s = 0; s < 3; ++s) Bz[r][s] = horner(B[r][s], s == 2 ? 4 : 3, z);
    // null vector of the rank-2 B(z): the largest cross product of two rows
    double best[3] = {0, 0, 0}, bn = -1.0;
    const int pr[3][2] = {{0, 1}, {0, 2}, {1, 2}};
    for (int p = 0; p < 3; ++p) {
      const double* a = Bz[pr[p][0]];
      const double* b = Bz[pr[p][1]];
      const double c[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
      const double nn = c[0] * c[0] + c[1] * c[1] + c[2] * c[2];
      if (nn > bn) {
        bn = nn;
        best[0] = c[0];
        best[1] = c[1];
        best[2] = c[2];
      }
    }
    if (!(bn > 0.0)) continue;
    const double inv = 1.0 / std::sqrt(bn);
    const double v0 = best[0] * inv, v1 = best[1] * inv, v2 = best[2] * inv;
    if (std::fabs(v2) < 1e-10) continue;
    const double x = v0 / v2, y = v1 / v2;
    double e[9], nrm = 0.0;
    for (int i = 0; i < 9; ++i) {
      e[i] = x * ns[0][i] + y * ns[1][i] + z * ns[2][i] + ns[3][i];
      nrm += e[i] * e[i];
    }
    nrm = std::sqrt(nrm);
    for (int i = 0; i < 9; ++i) E_out[9 * count + i] = e[i] / nrm;
    ++count;
  }
  return count;
}

// OpenCV EMEstimatorCallback::computeError (Sampson distance, stored as float)
float sampson(const double* E, const double* a, const double* b) {
  const double x1[3] = {a[0], a[1], 1.0}, x2[3] = {b[0], b[1], 1.0};
  double Ex1[3], Etx2[3];
  for (int i = 0; i < 3; ++i) {
    Ex1[i] = E[3 * i] * x1[0] + E[3 * i + 1] * x1[1] + E[3 * i + 2] * x1[2];
    Etx2[i] = E[i] * x2[0] + E[3 + i] * x2[1] + E[6 + i] * x2[2];
  }
  const double x2tEx1 = x2[0] * Ex1[0] + x2[1] * Ex1[1] + x2[2] * Ex1[2];
  const double aa = Ex1[0] * Ex1[0], bb = Ex1[1] * Ex1[1], cc = Etx2[0] * Etx2[0], dd = Etx2[1] * Etx2[1];
  return (float)(x2tEx1 * x2tEx1 / (aa + bb + cc + dd));
}

int update_num_iters(double p, double ep, int model_points, int max_iters) {
  p = std::min(std::max(p, 0.0), 1.0);
  ep = std::min(std::max(ep, 0.0), 1.0);
  double num = std::max(1.0 - p, 2.2250738585072014e-308);
  double denom = 1.0 - std::pow(1.0 - ep, model_points);
  if (denom < 2.2250738585072014e-308) return 0;
  num = std::log(num);
  denom = std::log(denom);
  return denom >= 0 || -num >= max_iters * (-denom) ? max_iters : (int)std::lround(num / denom);
}

// 5 distinct indices (OpenCV getSubset); false when count < 5
bool subset(CvRng& rng, int count, int* idx) {
  if (count < 5) return false;
  for (int i = 0; i < 5;) {
    const int v = rng.uniform(0, count);
    int j = 0;
    for (; j < i; ++j)
      if (idx[j] == v) break;
    if (j == i) idx[i++] = v;
  }
  return true;
}

double det3(const double* m) {
  return m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) + m[2] * (m[3] * m[7] - m[4] * m[6]);
}

// decomposeEssentialMat: R1 = U W V^T, R2 = U W^T V^T, t = U[:, 2]
void decompose(const double* E, double* R1, double* R2, double* t) {
  double EtE[9], w[3], V[9], Vd[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double s = 0.0;
      for (int k = 0; k < 3; ++k) s += E[3 * k + i] * E[3 * k + j];
      EtE[3 * i + j] = s;
    }
  jacobi_eig(EtE, 3, w, V);
  // descending singular order: columns 2, 1, 0 of V
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Vd[3 * i + j] = V[3 * i + (2 - j)];
  double U[9];
  for (int c = 0; c < 2; ++c) {
    double u[3], nn = 0.0;
    for (int i = 0; i < 3; ++i) {
      u[i] = E[3 * i] * Vd[c] + E[3 * i + 1] * Vd[3 + c] + E[3 * i + 2] * Vd[6 + c];
      nn += u[i] * u[i];
    }
    nn = std::sqrt(nn);
    for (int i = 0; i < 3; ++i) U[3 * i + c] = u[i] / nn;
  }
  U[2] = U[3] * U[7] - U[6] * U[4];
  U[5] = U[6] * U[1] - U[0] * U[7];
  U[8] = U[0] * U[4] - U[3] * U[1];
  if (det3(U) < 0)
    for (double& x : U) x = -x;
  if (det3(Vd) < 0)
    for (double& x : Vd) x = -x;
  const double W[9] = {0, 1, 0, -1, 0, 0, 0, 0, 1};
  double UW[9], UWt[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double s1 = 0.0, s2 = 0.0;
      for (int k = 0; k < 3; ++k) {
        s1 += U[3 * i + k] * W[3 * k + j];
        s2 += U[3 * i + k] * W[3 * j + k];
      }
      UW[3 * i + j] = s1;
      UWt[3 * i + j] = s2;
    }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double s1 = 0.0, s2 = 0.0;
      for (int k = 0; k < 3; ++k) {
        s1 += UW[3 * i + k] * Vd[3 * j + k];  // (V^T)[k][j] = V[j][k]
        s2 += UWt[3 * i + k] * Vd[3 * j + k];
      }
      R1[3 * i + j] = s1;
      R2[3 * i + j] = s2;
    }
  for (int i = 0; i < 3; ++i) t[i] = U[3 * i + 2];
}

// triangulation + cheirality of one correspondence under P1 = [R | t] (P0 = [I | 0])
bool cheiral(const double* a, const double* b, const double* R, const double* t, double dist) {
  double P1[12];
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) P1[4 * i + j] = R[3 * i + j];
    P1[4 * i + 3] = t[i];
  }
  const double P0[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
  double A[16];
  for (int k = 0; k < 4; ++k) {
    A[k] = a[0] * P0[8 + k] - P0[k];
    A[4 + k] = a[1] * P0[8 + k] - P0[4 + k];
    A[8 + k] = b[0] * P1[8 + k] - P1[k];
    A[12 + k] = b[1] * P1[8 + k] - P1[4 + k];
  }
  double AtA[16], w[4], V[16];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      double s = 0.0;
      for (int k = 0; k < 4; ++k) s += A[4 * k + i] * A[4 * k + j];
      AtA[4 * i + j] = s;
    }
  jacobi_eig(AtA, 4, w, V);
  double Q[4] = {V[0], V[4], V[8], V[12]};  // smallest eigenvalue's vector
  bool ok = Q[2] * Q[3] > 0;
  for (int i = 0; i < 3; ++i) Q[i] /= Q[3];
  Q[3] = 1.0;
  ok = ok && Q[2] < dist;
  double z2 = 0.0;
  for (int k = 0; k < 4; ++k) z2 += P1[8 + k] * Q[k];
  return ok && z2 > 0 && z2 < dist;
}

}  // namespace

extern "C" {

int oracle_five_point(const double* x1, const double* x2, double* E_out) { return five_point(x1, x2, E_out); }

float oracle_sampson(const double* E, const double* x1, const double* x2) { return sampson(E, x1, x2); }

int oracle_cv_rng_subsets(int count, int n_sets, int32_t* idx) {
  CvRng rng{~0ull};
  for (int s = 0; s < n_sets; ++s)
    if (!subset(rng, count, idx + 5 * s)) return s;
  return n_sets;
}

int oracle_mono_vo_process(const float* f1, const float* f2, int n, const oracle_mono_params* prm, double* Rt,
                           double* E_out, int32_t* inliers, int* n_inliers, int* stats) {
  for (int i = 0; i < 16; ++i) Rt[i] = (i % 5 == 0) ? 1.0 : 0.0;
  *n_inliers = 0;
  for (int i = 0; i < 9; ++i) E_out[i] = 0.0;
  if (stats) stats[0] = stats[1] = stats[2] = 0;
  if (n < 8) return 0;  // "not enough matches!" (:67-71)
  std::vector<int> keep;
  std::vector<double> p1, p2;
  for (int i = 0; i < n; ++i)
    if (f1[2 * i] > 0 && f2[2 * i] > 0) {
      keep.push_back(i);
      p1.push_back(((double)f1[2 * i] - prm->cu) / prm->fu);
      p1.push_back(((double)f1[2 * i + 1] - prm->cv) / prm->fv);
      p2.push_back(((double)f2[2 * i] - prm->cu) / prm->fu);
      p2.push_back(((double)f2[2 * i + 1] - prm->cv) / prm->fv);
    }
  const int count = (int)keep.size();
  const double thr_px = prm->inlier_threshold <= 0 ? 1.0 : prm->inlier_threshold;  // (:19-20)
  const double thr = thr_px / ((prm->fu + prm->fv) * 0.5);
  const int max_iters = 1000;
  std::vector<unsigned char> mask(count, 0), best_mask(count, 0);
  std::vector<float> err(count);
  double bestE[9], models[90];
  int good = 0;
  if (count < 5) return 0;  // empty E
  CvRng rng{~0ull};
  int idx[5];
  double s1[10], s2[10];
  bool found = false;
  if (prm->ransac) {
    const float t = (float)(thr * thr);
    int niters = max_iters, best = 0, iters_run = 0;
    for (int it = 0; it < niters; ++it) {
      if (count > 5) {
        subset(rng, count, idx);
      } else {
        for (int k = 0; k < 5; ++k) idx[k] = k;
      }
      ++iters_run;
      for (int k = 0; k < 5; ++k) {
        s1[2 * k] = p1[2 * idx[k]];
        s1[2 * k + 1] = p1[2 * idx[k] + 1];
        s2[2 * k] = p2[2 * idx[k]];
        s2[2 * k + 1] = p2[2 * idx[k] + 1];
      }
      const int nm = five_point(s1, s2, models);
      for (int m = 0; m < nm; ++m) {
        int gc = 0;
        for (int i = 0; i < count; ++i) {
          err[i] = sampson(models + 9 * m, &p1[2 * i], &p2[2 * i]);
          mask[i] = err[i] <= t;
          gc += mask[i];
        }
        if (gc > std::max(best, 4)) {
          std::swap(mask, best_mask);
          std::memcpy(bestE, models + 9 * m, sizeof(bestE));
          best = gc;
          niters = update_num_iters(prm->prob, (double)(count - gc) / count, 5, niters);
          found = true;
        }
      }
      if (count == 5) break;
    }
    good = best;
    if (stats) {
      stats[0] = iters_run;
      stats[1] = best;
    }
  } else {
    // LMedS (OpenCV LMeDSPointSetRegistrator)
    const double outlier_ratio = 0.45;
    int niters = (int)std::lround(std::log(1 - prm->prob) / std::log(1 - std::pow(1 - outlier_ratio, 5)));
    niters = std::min(std::max(niters, 3), max_iters);
    double min_median = 3.4e38;  // FLT_MAX
    std::vector<float> sorted(count);
    for (int it = 0; it < niters; ++it) {
      if (count > 5) {
        subset(rng, count, idx);
      } else {
        for (int k = 0; k < 5; ++k) idx[k] = k;
      }
      for (int k = 0; k < 5; ++k) {
        s1[2 * k] = p1[2 * idx[k]];
        s1[2 * k + 1] = p1[2 * idx[k] + 1];
        s2[2 * k] = p2[2 * idx[k]];
        s2[2 * k + 1] = p2[2 * idx[k] + 1];
      }
      const int nm = five_point(s1, s2, models);
      for (int m = 0; m < nm; ++m) {
        for (int i = 0; i < count; ++i) sorted[i] = sampson(models + 9 * m, &p1[2 * i], &p2[2 * i]);
        std::nth_element(sorted.begin(), sorted.begin() + count / 2, sorted.end());
        const double med = sorted[count / 2];
        if (med < min_median) {
          min_median = med;
          std::memcpy(bestE, models + 9 * m, sizeof(bestE));
          found = true;
        }
      }
      if (count == 5) break;
    }
    if (found) {
      double th = 2.5 * 1.4826 * (1 + 5.0 / (count - 5 > 0 ? count - 5 : 1)) * std::sqrt(min_median);
      // sigma = MAX(sigma, 0.001): OpenCV LMeDSPointSetRegistrator (calib3d ptsetreg.cpp), restated
      // (no OpenCV here to check it against: the LMedS mask is parity unpinned, like the RANSAC path)
      th = std::max(th, 0.001);
      const float t = (float)(th * th);
      good = 0;
      for (int i = 0; i < count; ++i) {
        best_mask[i] = sampson(bestE, &p1[2 * i], &p2[2 * i]) <= t;
        good += best_mask[i];
      }
    }
    if (stats) {
      stats[0] = niters;
      stats[1] = good;
    }
  }
  if (!found || good <= 0) return 0;  // "empty E matrix!" (:22-26)
  std::memcpy(E_out, bestE, sizeof(bestE));
  // recoverPose (distance threshold 500)
  double R1[9], R2[9], tt[3], nt[3];
  decompose(bestE, R1, R2, tt);
  for (int i = 0; i < 3; ++i) nt[i] = -tt[i];
  const double* Rs[4] = {R1, R2, R1, R2};
  const double* ts[4] = {tt, tt, nt, nt};
  std::vector<unsigned char> pm[4];
  int gcount[4];
  for (int c = 0; c < 4; ++c) {
    pm[c].assign(count, 0);
    gcount[c] = 0;
    for (int i = 0; i < count; ++i) {
      pm[c][i] = best_mask[i] && cheiral(&p1[2 * i], &p2[2 * i], Rs[c], ts[c], 500.0);
      gcount[c] += pm[c][i];
    }
  }
  int bc = 0;
  if (gcount[0] >= gcount[1] && gcount[0] >= gcount[2] && gcount[0] >= gcount[3]) bc = 0;
  else if (gcount[1] >= gcount[0] && gcount[1] >= gcount[2] && gcount[1] >= gcount[3]) bc = 1;
  else if (gcount[2] >= gcount[0] && gcount[2] >= gcount[1] && gcount[2] >= gcount[3]) bc = 2;
  else bc = 3;
  int ni = 0;
  for (int i = 0; i < count; ++i)
    if (pm[bc][i]) inliers[ni++] = keep[i];
  *n_inliers = ni;
  if (stats) stats[2] = bc;
  if (ni < 10) return 0;  // "not enough inliers!" (:46-49)
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) Rt[4 * i + j] = Rs[bc][3 * i + j];
    Rt[4 * i + 3] = ts[bc][i];
  }
  return 1;
}

}  // extern "C"
