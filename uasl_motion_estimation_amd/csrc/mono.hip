// mono.hip -- Mono VO: MonoVisualOdometry::process
// (src/vo/MonoVisualOdometry.cpp:7-73), i.e. OpenCV findEssentialMat (the
// five-point solver inside a RANSAC or LMedS registrator) + recoverPose,
// restated from their published algorithms (oracle/mono.cpp is the checker;
// parity unpinned: OpenCV is absent here).
//
// Device work:
//  * mono_hyp_kernel: one thread per RANSAC / LMedS sample: the five-point
//    solve (null space by a 9 x 9 Jacobi eigen decomposition, the ten cubic
//    constraints, Gauss-Jordan, the degree-10 polynomial, real roots by
//    derivative-chain isolation and bisection) -> up to 10 essential matrices;
//  * mono_score_kernel: one wave per model: Sampson errors (float, OpenCV's
//    computeError) of every match, inlier count at the threshold (RANSAC) or
//    the exact median by a 4 x 8-bit radix select in LDS (LMedS);
//  * mono_mask_kernel: the best model's inlier mask;
//  * mono_pose_kernel (one thread): decomposeEssentialMat (3 x 3 Jacobi SVD);
//  * mono_cheiral_kernel: per match x 4 poses, DLT triangulation (4 x 4
//    Jacobi) and the cheirality / distance test, counts per pose.
// Host: the filter of valid matches and OpenCV's RNG subsets (sequential
// state), the replay of the RANSAC loop over the device counts (the adaptive
// iteration bound needs glibc log / pow in sample order), the pose choice and
// the inlier list.  Every FP64 step is written in the oracle's operation order
// so the inlier indices agree bit for bit.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "me_internal.hpp"

namespace {

constexpr int kMonoMaxIters = 1000;  // OpenCV findEssentialMat maxIters
constexpr int kMonoMaxModels = 10;

__constant__ int cLin[4][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, 0}};
__constant__ int cQuad[10][3] = {{2, 0, 0}, {0, 2, 0}, {0, 0, 2}, {1, 1, 0}, {1, 0, 1},
                                 {0, 1, 1}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, 0}};
__constant__ int cMono[20][3] = {{3, 0, 0}, {0, 3, 0}, {2, 1, 0}, {1, 2, 0}, {2, 0, 1}, {2, 0, 0}, {0, 2, 1},
                                 {0, 2, 0}, {1, 1, 1}, {1, 1, 0}, {1, 0, 2}, {1, 0, 1}, {1, 0, 0}, {0, 1, 2},
                                 {0, 1, 1}, {0, 1, 0}, {0, 0, 3}, {0, 0, 2}, {0, 0, 1}, {0, 0, 0}};

__device__ int quad_index(int a, int b, int c) {
  for (int k = 0; k < 10; ++k)
    if (cQuad[k][0] == a && cQuad[k][1] == b && cQuad[k][2] == c) return k;
  return -1;
}
__device__ int mono_index(int a, int b, int c) {
  for (int k = 0; k < 20; ++k)
    if (cMono[k][0] == a && cMono[k][1] == b && cMono[k][2] == c) return k;
  return -1;
}
__device__ void mul_ll(const double* p, const double* q, double* r) {
  for (int k = 0; k < 10; ++k) r[k] = 0.0;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      r[quad_index(cLin[i][0] + cLin[j][0], cLin[i][1] + cLin[j][1], cLin[i][2] + cLin[j][2])] += p[i] * q[j];
}
__device__ void mul_ql(const double* p, const double* q, double* r) {
  for (int k = 0; k < 20; ++k) r[k] = 0.0;
  for (int i = 0; i < 10; ++i)
    for (int j = 0; j < 4; ++j)
      r[mono_index(cQuad[i][0] + cLin[j][0], cQuad[i][1] + cLin[j][1], cQuad[i][2] + cLin[j][2])] += p[i] * q[j];
}

__device__ double horner(const double* c, int deg, double z) {
  double v = c[deg];
  for (int k = deg - 1; k >= 0; --k) v = v * z + c[k];
  return v;
}
__device__ int roots_between(const double* c, int deg, const double* crit, int nc, double* out) {
  if (deg == 1) {
    out[0] = -c[0] / c[1];
    return 1;
  }
  double bound = 0.0;
  for (int k = 0; k < deg; ++k) bound = fmax(bound, fabs(c[k] / c[deg]));
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
    if (fhi == 0.0 || (flo < 0) == (fhi < 0)) continue;
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
__device__ int real_roots(const double* c, int deg, double* out) {
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
  if (dg[L] <= 0 && L == 0) return 0;
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

// cyclic Jacobi, eigenvalues ascending, eigenvectors as the columns of V (n <= 9)
__device__ void jacobi_eig(double* a, int n, double* w, double* V) {
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
        const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < n; ++k) {
          const double akp = a[k * n + p], akq = a[k * n + q];
          a[k * n + p] = c * akp - s * akq;
          a[k * n + q] = s * akp + c * akq;
        }
        for (int k = 0; k < n; ++k) {
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
  for (int i = 0; i < n; ++i) w[i] = a[i * n + i];
  for (int i = 0; i < n; ++i) {
    int m = i;
    for (int j = i + 1; j < n; ++j)
      if (w[j] < w[m]) m = j;
    if (m != i) {
      const double tw = w[i];
      w[i] = w[m];
      w[m] = tw;
      for (int k = 0; k < n; ++k) {
        const double tv = V[k * n + i];
        V[k * n + i] = V[k * n + m];
        V[k * n + m] = tv;
      }
    }
  }
}

__device__ int five_point(const double* x1, const double* x2, double* E_out) {
  double q[5][9];
  for (int i = 0; i < 5; ++i) {
    const double u1 = x1[2 * i], v1 = x1[2 * i + 1], u2 = x2[2 * i], v2 = x2[2 * i + 1];
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
  {
    double QtQ[81], w[9], V[81];
    for (int i = 0; i < 9; ++i)
      for (int j = 0; j < 9; ++j) {
        double s = 0.0;
        for (int k = 0; k < 5; ++k) s += q[k][i] * q[k][j];
        QtQ[9 * i + j] = s;
      }
    jacobi_eig(QtQ, 9, w, V);
    if (!(w[4] > 0.0)) return 0;
    for (int v = 0; v < 4; ++v)
      for (int k = 0; k < 9; ++k) ns[v][k] = V[9 * k + (3 - v)];
  }
  double E[9][4];
  for (int e = 0; e < 9; ++e)
    for (int v = 0; v < 4; ++v) E[e][v] = ns[v][e];
  double A[10][20];
  double t1[10], t2[10], m[10], cub[20];
  const int cof[3][4] = {{1, 2, 2, 1}, {0, 2, 2, 0}, {0, 1, 1, 0}};
  for (int k = 0; k < 20; ++k) A[0][k] = 0.0;
  for (int j = 0; j < 3; ++j) {
    mul_ll(E[3 + cof[j][0]], E[6 + cof[j][1]], t1);
    mul_ll(E[3 + cof[j][2]], E[6 + cof[j][3]], t2);
    for (int k = 0; k < 10; ++k) m[k] = t1[k] - t2[k];
    mul_ql(m, E[j], cub);
    for (int k = 0; k < 20; ++k) A[0][k] += j == 1 ? -cub[k] : cub[k];
  }
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
  for (int col = 0; col < 10; ++col) {
    int best = col;
    for (int i = col + 1; i < 10; ++i)
      if (fabs(A[i][col]) > fabs(A[best][col])) best = i;
    if (!(fabs(A[best][col]) > 0.0)) return 0;
    if (best != col)
      for (int k = 0; k < 20; ++k) {
        const double tv = A[col][k];
        A[col][k] = A[best][k];
        A[best][k] = tv;
      }
    const double inv = 1.0 / A[col][col];
    for (int k = col; k < 20; ++k) A[col][k] *= inv;
    for (int i = 0; i < 10; ++i) {
      if (i == col) continue;
      const double f = A[i][col];
      if (f != 0.0)
        for (int k = col; k < 20; ++k) A[i][k] -= f * A[col][k];
    }
  }
  double B[3][3][5];
  for (int r = 0; r < 3; ++r) {
    const double* p = A[4 + 2 * r] + 10;
    const double* q2 = A[5 + 2 * r] + 10;
    for (int s = 0; s < 2; ++s) {
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
  auto pmul = [](const double* a, int da, const double* b, int db, double* r) {
    for (int k = 0; k <= da + db; ++k) r[k] = 0.0;
    for (int i = 0; i <= da; ++i)
      for (int j = 0; j <= db; ++j) r[i + j] += a[i] * b[j];
  };
  double poly[11] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, m1[9], m2[9], mdiff[9], term[14];
  const int cj[3][4] = {{1, 2, 2, 1}, {0, 2, 2, 0}, {0, 1, 1, 0}};
  for (int j = 0; j < 3; ++j) {
    const int a0 = cj[j][0], a1 = cj[j][1], b0 = cj[j][2], b1 = cj[j][3];
    const int da0 = a0 == 2 ? 4 : 3, da1 = a1 == 2 ? 4 : 3, db0 = b0 == 2 ? 4 : 3, db1 = b1 == 2 ? 4 : 3;
    pmul(B[1][a0], da0, B[2][a1], da1, m1);
    pmul(B[1][b0], db0, B[2][b1], db1, m2);
    const int dm = max(da0 + da1, db0 + db1);
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
    const double inv = 1.0 / sqrt(bn);
    const double v0 = best[0] * inv, v1 = best[1] * inv, v2 = best[2] * inv;
    if (fabs(v2) < 1e-10) continue;
    const double x = v0 / v2, y = v1 / v2;
    double e[9], nrm = 0.0;
    for (int i = 0; i < 9; ++i) {
      e[i] = x * ns[0][i] + y * ns[1][i] + z * ns[2][i] + ns[3][i];
      nrm += e[i] * e[i];
    }
    nrm = sqrt(nrm);
    for (int i = 0; i < 9; ++i) E_out[9 * count + i] = e[i] / nrm;
    ++count;
  }
  return count;
}

__device__ float sampson(const double* E, const double* a, const double* b) {
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

__device__ double det3(const double* m) {
  return m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) + m[2] * (m[3] * m[7] - m[4] * m[6]);
}

__device__ bool cheiral(const double* a, const double* b, const double* R, const double* t, double dist) {
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
  double Q[4] = {V[0], V[4], V[8], V[12]};
  bool ok = Q[2] * Q[3] > 0;
  for (int i = 0; i < 3; ++i) Q[i] /= Q[3];
  Q[3] = 1.0;
  ok = ok && Q[2] < dist;
  double z2 = 0.0;
  for (int k = 0; k < 4; ++k) z2 += P1[8 + k] * Q[k];
  return ok && z2 > 0 && z2 < dist;
}

// ---- kernels
__global__ void mono_norm_kernel(const float* __restrict__ f, int n, double fu, double fv, double cu, double cv,
                                 double* __restrict__ x) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  x[2 * i] = ((double)f[2 * i] - cu) / fu;
  x[2 * i + 1] = ((double)f[2 * i + 1] - cv) / fv;
}

__global__ __launch_bounds__(64) void mono_hyp_kernel(const double* __restrict__ x1, const double* __restrict__ x2,
                                                       const int* __restrict__ sets, int ns, double* __restrict__ models,
                                                       int* __restrict__ nmod) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= ns) return;
  double a[10], b[10];
  for (int k = 0; k < 5; ++k) {
    const int i = sets[5 * s + k];
    a[2 * k] = x1[2 * i];
    a[2 * k + 1] = x1[2 * i + 1];
    b[2 * k] = x2[2 * i];
    b[2 * k + 1] = x2[2 * i + 1];
  }
  nmod[s] = five_point(a, b, models + 90 * (long)s);
}

// radix select of the k-th smallest of n non-negative floats (their bit
// patterns order as the values), 4 passes of 8 bits over the wave's LDS copy
constexpr int kMonoWaves = 4, kMonoScoreBlock = 64 * kMonoWaves;

__global__ __launch_bounds__(kMonoScoreBlock) void mono_score_kernel(const double* __restrict__ x1,
                                                                     const double* __restrict__ x2, int count,
                                                                     const double* __restrict__ models,
                                                                     const int* __restrict__ nmod, int ns, float t,
                                                                     int lmeds, int* __restrict__ cnt,
                                                                     float* __restrict__ med, float* __restrict__ errbuf) {
  __shared__ unsigned hist[kMonoWaves][256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long mdl = (long)blockIdx.x * kMonoWaves + wave;  // model slot: sample mdl / 10, model mdl % 10
  const int s = (int)(mdl / kMonoMaxModels), m = (int)(mdl % kMonoMaxModels);
  const bool live = s < ns && m < nmod[s];  // (wave-uniform)
  if (!live) return;  // (no workgroup barrier below: per-wave LDS)
  const double* E = models + 90 * (long)s + 9 * m;
  double Ev[9];
  for (int k = 0; k < 9; ++k) Ev[k] = E[k];
  if (!lmeds) {
    int c = 0;
    for (int i = lane; i < count; i += 64) c += sampson(Ev, x1 + 2 * i, x2 + 2 * i) <= t ? 1 : 0;
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
    if (lane == 0) cnt[mdl] = c;
    return;
  }
  float* err = errbuf + mdl * (long)count;
  for (int i = lane; i < count; i += 64) err[i] = sampson(Ev, x1 + 2 * i, x2 + 2 * i);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  unsigned prefix = 0, pmask = 0;
  int k = count / 2;  // nth_element(begin, begin + count / 2, end)
  for (int pass = 3; pass >= 0; --pass) {
    for (int b = lane; b < 256; b += 64) hist[wave][b] = 0u;
    __builtin_amdgcn_wave_barrier();
    const int sh = 8 * pass;
    for (int i = lane; i < count; i += 64) {
      const unsigned v = __float_as_uint(err[i]);
      if ((v & pmask) == prefix) atomicAdd(&hist[wave][(v >> sh) & 255u], 1u);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane == 0) {
      int b = 0;
      for (; b < 256; ++b) {
        const int h = (int)hist[wave][b];
        if (k < h) break;
        k -= h;
      }
      hist[wave][0] = (unsigned)b | ((unsigned)k << 8);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const unsigned r = hist[wave][0];
    k = (int)(r >> 8);
    prefix |= (r & 255u) << sh;
    pmask |= 255u << sh;
    __builtin_amdgcn_wave_barrier();
  }
  if (lane == 0) med[mdl] = __uint_as_float(prefix);
}

__global__ void mono_mask_kernel(const double* __restrict__ x1, const double* __restrict__ x2, int count,
                                 const double* __restrict__ E, float t, unsigned char* __restrict__ mask) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  double Ev[9];
  for (int k = 0; k < 9; ++k) Ev[k] = E[k];
  mask[i] = sampson(Ev, x1 + 2 * i, x2 + 2 * i) <= t ? 1 : 0;
}

// decomposeEssentialMat: out = R1 (9) | R2 (9) | t (3)
__global__ void mono_pose_kernel(const double* __restrict__ Ein, double* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double E[9];
  for (int k = 0; k < 9; ++k) E[k] = Ein[k];
  double EtE[9], w[3], V[9], Vd[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double s = 0.0;
      for (int k = 0; k < 3; ++k) s += E[3 * k + i] * E[3 * k + j];
      EtE[3 * i + j] = s;
    }
  jacobi_eig(EtE, 3, w, V);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Vd[3 * i + j] = V[3 * i + (2 - j)];
  double U[9];
  for (int c = 0; c < 2; ++c) {
    double u[3], nn = 0.0;
    for (int i = 0; i < 3; ++i) {
      u[i] = E[3 * i] * Vd[c] + E[3 * i + 1] * Vd[3 + c] + E[3 * i + 2] * Vd[6 + c];
      nn += u[i] * u[i];
    }
    nn = sqrt(nn);
    for (int i = 0; i < 3; ++i) U[3 * i + c] = u[i] / nn;
  }
  U[2] = U[3] * U[7] - U[6] * U[4];
  U[5] = U[6] * U[1] - U[0] * U[7];
  U[8] = U[0] * U[4] - U[3] * U[1];
  if (det3(U) < 0)
    for (int k = 0; k < 9; ++k) U[k] = -U[k];
  if (det3(Vd) < 0)
    for (int k = 0; k < 9; ++k) Vd[k] = -Vd[k];
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
        s1 += UW[3 * i + k] * Vd[3 * j + k];
        s2 += UWt[3 * i + k] * Vd[3 * j + k];
      }
      out[3 * i + j] = s1;
      out[9 + 3 * i + j] = s2;
    }
  for (int i = 0; i < 3; ++i) out[18 + i] = U[3 * i + 2];
}

// per (match, pose): cheirality flag (pose c: R1 t, R2 t, R1 -t, R2 -t) and per-pose counts
__global__ void mono_cheiral_kernel(const double* __restrict__ x1, const double* __restrict__ x2, int count,
                                    const unsigned char* __restrict__ mask, const double* __restrict__ pose,
                                    double dist, unsigned char* __restrict__ flags, int* __restrict__ counts) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int c = blockIdx.y;
  if (i >= count) return;
  double R[9], t[3];
  for (int k = 0; k < 9; ++k) R[k] = pose[(c & 1) ? 9 + k : k];
  for (int k = 0; k < 3; ++k) t[k] = (c & 2) ? -pose[18 + k] : pose[18 + k];
  const bool ok = mask[i] && cheiral(x1 + 2 * i, x2 + 2 * i, R, t, dist);
  flags[(long)c * count + i] = ok ? 1 : 0;
  if (ok) atomicAdd(&counts[c], 1);
}

// OpenCV cv::RNG (multiply-with-carry), (uint64)-1 as the registrators seed it
struct CvRng {
  uint64_t s;
  unsigned next() {
    s = (uint64_t)(unsigned)s * 4164903690u + (unsigned)(s >> 32);
    return (unsigned)s;
  }
  int uniform(int a, int b) { return a == b ? a : (int)(next() % (unsigned)(b - a)) + a; }
};

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

}  // namespace

extern "C" void me_mono_default_params(me_mono_params* p) {
  if (!p) return;
  p->fu = 1.0;
  p->fv = 1.0;
  p->cu = 0.0;
  p->cv = 0.0;
  p->prob = 0.99;
  p->inlier_threshold = 2.0;
  p->ransac = 1;
}

extern "C" int me_mono_vo_process(me_ctx* c, const float* f1, const float* f2, int n, const me_mono_params* p,
                                  double* Rt, double* E_out, int32_t* inliers, int* n_inliers, int* ok) {
  me_range range_("me_mono_vo_process");
  if (!c || !p || !Rt || !n_inliers || !ok) return ME_ERR_INVALID;
  ME_CHECK(c, n >= 0 && (n == 0 || (f1 && f2)), "me_mono_vo_process: bad matches");
  ME_CHECK(c, p->fu > 0 && p->fv > 0 && p->prob > 0 && p->prob < 1, "me_mono_vo_process: bad parameters");
  for (int i = 0; i < 16; ++i) Rt[i] = (i % 5 == 0) ? 1.0 : 0.0;
  if (E_out)
    for (int i = 0; i < 9; ++i) E_out[i] = 0.0;
  *n_inliers = 0;
  *ok = 0;
  if (n < 8) return ME_OK;  // "not enough matches!" (MonoVisualOdometry.cpp:67-71)
  ME_HIP(c, hipSetDevice(c->device));
  // valid matches (:13-17), packed in order
  std::vector<int> keep;
  std::vector<float> h1, h2;
  for (int i = 0; i < n; ++i)
    if (f1[2 * i] > 0 && f2[2 * i] > 0) {
      keep.push_back(i);
      h1.push_back(f1[2 * i]);
      h1.push_back(f1[2 * i + 1]);
      h2.push_back(f2[2 * i]);
      h2.push_back(f2[2 * i + 1]);
    }
  const int count = (int)keep.size();
  if (count < 5) return ME_OK;  // findEssentialMat: empty E ("empty E matrix!", :22-26)
  const double thr_px = p->inlier_threshold <= 0 ? 1.0 : p->inlier_threshold;  // (:19-20)
  const double thr = thr_px / ((p->fu + p->fv) * 0.5);
  // the samples of OpenCV's registrator loop, in order (the RNG state is
  // sequential; the loop's adaptive bound only truncates the list)
  int nsets = kMonoMaxIters;
  if (!p->ransac) {
    int it = (int)std::lround(std::log(1 - p->prob) / std::log(1 - std::pow(1 - 0.45, 5)));
    nsets = std::min(std::max(it, 3), kMonoMaxIters);
  }
  if (count == 5) nsets = 1;
  std::vector<int> sets(5 * (size_t)nsets);
  {
    CvRng rng{~0ull};
    for (int s = 0; s < nsets; ++s) {
      int* idx = &sets[5 * (size_t)s];
      if (count == 5) {
        for (int k = 0; k < 5; ++k) idx[k] = k;
        continue;
      }
      for (int i = 0; i < 5;) {
        const int v = rng.uniform(0, count);
        int j = 0;
        for (; j < i; ++j)
          if (idx[j] == v) break;
        if (j == i) idx[i++] = v;
      }
    }
  }
  const long nslot = (long)nsets * kMonoMaxModels;
  auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t bF = up(8 * (size_t)count), bX = up(16 * (size_t)count), bS = up(20 * (size_t)nsets);
  const size_t bM = up(720 * (size_t)nsets), bN = up(4 * (size_t)nsets), bC = up(4 * (size_t)nslot);
  const size_t bMed = up(4 * (size_t)nslot), bErr = p->ransac ? 256 : up(4 * (size_t)nslot * count);
  const size_t bMask = up((size_t)count), bPose = 256, bE = 256, bFl = up(4 * (size_t)count), bPc = 256;
  void* d;
  ME_TRY(me_scratch(c, SLOT_MONO, 2 * bF + 2 * bX + bS + bM + bN + bC + bMed + bErr + bMask + bPose + bE + bFl + bPc,
                    &d));
  char* q = (char*)d;
  auto take = [&](size_t b) {
    char* r = q;
    q += b;
    return r;
  };
  float* df1 = (float*)take(bF);
  float* df2 = (float*)take(bF);
  double* dx1 = (double*)take(bX);
  double* dx2 = (double*)take(bX);
  int* dsets = (int*)take(bS);
  double* dmod = (double*)take(bM);
  int* dnm = (int*)take(bN);
  int* dcnt = (int*)take(bC);
  float* dmed = (float*)take(bMed);
  float* derr = (float*)take(bErr);
  unsigned char* dmask = (unsigned char*)take(bMask);
  double* dpose = (double*)take(bPose);
  double* dE = (double*)take(bE);
  unsigned char* dfl = (unsigned char*)take(bFl);
  int* dpc = (int*)take(bPc);
  hipStream_t s = c->stream;
  ME_HIP(c, hipMemcpyAsync(df1, h1.data(), 8 * (size_t)count, hipMemcpyHostToDevice, s));
  ME_HIP(c, hipMemcpyAsync(df2, h2.data(), 8 * (size_t)count, hipMemcpyHostToDevice, s));
  ME_HIP(c, hipMemcpyAsync(dsets, sets.data(), 20 * (size_t)nsets, hipMemcpyHostToDevice, s));
  const int nb = (count + 255) / 256;
  hipLaunchKernelGGL(mono_norm_kernel, dim3(nb), dim3(256), 0, s, df1, count, p->fu, p->fv, p->cu, p->cv, dx1);
  hipLaunchKernelGGL(mono_norm_kernel, dim3(nb), dim3(256), 0, s, df2, count, p->fu, p->fv, p->cu, p->cv, dx2);
  hipLaunchKernelGGL(mono_hyp_kernel, dim3((nsets + 63) / 64), dim3(64), 0, s, dx1, dx2, dsets, nsets, dmod, dnm);
  const float t2 = (float)(thr * thr);
  hipLaunchKernelGGL(mono_score_kernel, dim3((unsigned)((nslot + kMonoWaves - 1) / kMonoWaves)), dim3(kMonoScoreBlock),
                     0, s, dx1, dx2, count, dmod, dnm, nsets, t2, p->ransac ? 0 : 1, dcnt, dmed, derr);
  ME_TRY(me_check_launch(c, "mono VO hypotheses"));
  std::vector<int> hnm(nsets), hcnt(p->ransac ? nslot : 0);
  std::vector<float> hmed(p->ransac ? 0 : nslot);
  ME_HIP(c, hipMemcpyAsync(hnm.data(), dnm, 4 * (size_t)nsets, hipMemcpyDeviceToHost, s));
  if (p->ransac) ME_HIP(c, hipMemcpyAsync(hcnt.data(), dcnt, 4 * (size_t)nslot, hipMemcpyDeviceToHost, s));
  else ME_HIP(c, hipMemcpyAsync(hmed.data(), dmed, 4 * (size_t)nslot, hipMemcpyDeviceToHost, s));
  ME_HIP(c, hipStreamSynchronize(s));
  // the registrator's loop replayed over the device scores, in sample order
  long best_slot = -1;
  float mask_t = t2;
  if (p->ransac) {
    int niters = kMonoMaxIters, best = 0;
    for (int it = 0; it < niters && it < nsets; ++it)
      for (int m = 0; m < hnm[it]; ++m) {
        const int gc = hcnt[(long)it * kMonoMaxModels + m];
        if (gc > std::max(best, 4)) {
          best = gc;
          best_slot = (long)it * kMonoMaxModels + m;
          niters = update_num_iters(p->prob, (double)(count - gc) / count, 5, niters);
        }
      }
  } else {
    double min_median = 3.4e38;
    for (int it = 0; it < nsets; ++it)
      for (int m = 0; m < hnm[it]; ++m) {
        const double med = hmed[(long)it * kMonoMaxModels + m];
        if (med < min_median) {
          min_median = med;
          best_slot = (long)it * kMonoMaxModels + m;
        }
      }
    if (best_slot >= 0) {
      double th = 2.5 * 1.4826 * (1 + 5.0 / (count - 5 > 0 ? count - 5 : 1)) * std::sqrt(min_median);
      // sigma = MAX(sigma, 0.001): OpenCV LMeDSPointSetRegistrator (calib3d ptsetreg.cpp), restated
      // (no OpenCV here to check it against: the LMedS mask is parity unpinned, like the RANSAC path)
      th = std::max(th, 0.001);
      mask_t = (float)(th * th);
    }
  }
  if (best_slot < 0) return ME_OK;  // no model: "empty E matrix!"
  const double* Ebest = dmod + 90 * (best_slot / kMonoMaxModels) + 9 * (best_slot % kMonoMaxModels);
  ME_HIP(c, hipMemcpyAsync(dE, Ebest, 72, hipMemcpyDeviceToDevice, s));
  hipLaunchKernelGGL(mono_mask_kernel, dim3(nb), dim3(256), 0, s, dx1, dx2, count, (const double*)dE, mask_t, dmask);
  hipLaunchKernelGGL(mono_pose_kernel, dim3(1), dim3(64), 0, s, (const double*)dE, dpose);
  ME_HIP(c, hipMemsetAsync(dpc, 0, 16, s));
  hipLaunchKernelGGL(mono_cheiral_kernel, dim3(nb, 4), dim3(256), 0, s, dx1, dx2, count, (const unsigned char*)dmask,
                     (const double*)dpose, 500.0, dfl, dpc);
  ME_TRY(me_check_launch(c, "mono VO pose"));
  double hE[9], hpose[21];
  int hpc[4];
  std::vector<unsigned char> hfl(4 * (size_t)count);
  ME_HIP(c, hipMemcpyAsync(hE, dE, 72, hipMemcpyDeviceToHost, s));
  ME_HIP(c, hipMemcpyAsync(hpose, dpose, sizeof(hpose), hipMemcpyDeviceToHost, s));
  ME_HIP(c, hipMemcpyAsync(hpc, dpc, 16, hipMemcpyDeviceToHost, s));
  ME_HIP(c, hipMemcpyAsync(hfl.data(), dfl, 4 * (size_t)count, hipMemcpyDeviceToHost, s));
  ME_HIP(c, hipStreamSynchronize(s));
  if (E_out) std::memcpy(E_out, hE, sizeof(hE));
  // recoverPose's choice (ties in the order R1 t, R2 t, R1 -t, R2 -t)
  int bc;
  if (hpc[0] >= hpc[1] && hpc[0] >= hpc[2] && hpc[0] >= hpc[3]) bc = 0;
  else if (hpc[1] >= hpc[0] && hpc[1] >= hpc[2] && hpc[1] >= hpc[3]) bc = 1;
  else if (hpc[2] >= hpc[0] && hpc[2] >= hpc[1] && hpc[2] >= hpc[3]) bc = 2;
  else bc = 3;
  int ni = 0;
  for (int i = 0; i < count; ++i)
    if (hfl[(size_t)bc * count + i]) {
      if (inliers) inliers[ni] = keep[i];
      ++ni;
    }
  *n_inliers = ni;
  if (ni < 10) return ME_OK;  // "not enough inliers!" (:46-49)
  const double* R = hpose + ((bc & 1) ? 9 : 0);
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) Rt[4 * i + j] = R[3 * i + j];
    Rt[4 * i + 3] = (bc & 2) ? -hpose[18 + i] : hpose[18 + i];
  }
  *ok = 1;
  return ME_OK;
}
