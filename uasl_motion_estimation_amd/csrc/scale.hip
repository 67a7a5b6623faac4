// scale.hip — MI stereo-scale optimiser.
//
// Replaces Optimiser<ScaleState, std::vector<std::pair<cv::Mat,cv::Mat>>>
// (src/optimisation/optimisation.cpp:29-228, 435-747).  Each evaluation is
// ONE fused kernel: a lane reprojects its track (double, OpenCV Matx order),
// applies the reference's ROI rounding rules, builds the lane-private MI
// histograms of its patch pair(s) in LDS and writes its residual / Jacobian
// contribution; a single-workgroup kernel then reduces in a fixed order.  The
// scalar LM control (run_LM_step) stays on the host exactly as in the
// reference, with one 16-byte read-back per evaluation.
#include <cmath>
#include <cstring>
#include <vector>
#include <algorithm>
#include "me_internal.hpp"
#include "me_device.hpp"

using namespace me_dev;

namespace {

constexpr int kScBlock = 256;

struct ScaleArgs {
  double K1[9], K2[9], q1[4], t1[3], q2[4], t2[3];
  double scale, baseline;
  int w;
  int nL, nR;
  const uint8_t* imgL;
  const uint8_t* imgR;
  int stride, cols, rows;
  int bb_cols, bb_rows;
  int weighting;
  float invN;          // 1/(P*P)
};

// flags per track: bit0 = triangulated & unmasked (owns a row), bit1 = seen in lframe
struct TrackDev {
  const double* X;     // 4 per track, left tracks then right tracks
  const uint8_t* flags;
  const int* row;      // residual row of the track or -1
};

__device__ __forceinline__ int refl101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) {
    if (i < 0) i = -i;
    if (i >= n) i = 2 * n - 2 - i;
  }
  return i;
}

// cv::Sobel(ROI view, CV_8U, 1, 0) mean: ROI pixels outside the view come from
// the parent image, reflect-101 at the parent border.
__device__ double sobel_weight(const uint8_t* img, int stride, int cols, int rows, int x0, int y0, int P) {
  long sum = 0;
  for (int y = 0; y < P; ++y)
    for (int x = 0; x < P; ++x) {
      int gx = 0;
      for (int dy = -1; dy <= 1; ++dy) {
        int yy = refl101(y0 + y + dy, rows);
        int xm = refl101(x0 + x - 1, cols), xp = refl101(x0 + x + 1, cols);
        int wgt = dy == 0 ? 2 : 1;
        gx += wgt * ((int)img[(long)yy * stride + xp] - (int)img[(long)yy * stride + xm]);
      }
      sum += min(255, max(0, gx));
    }
  double m = (double)sum * (1.0 / (double)(P * P));
  return fabs(m) + 1e-20;
}

// Sobel on an isolated binarised patch (compute_jacobian right branch)
__device__ double sobel_weight_bin(const uint8_t* img, int stride, int x0, int y0, int P) {
  long sum = 0;
  for (int y = 0; y < P; ++y)
    for (int x = 0; x < P; ++x) {
      float gx = 0;
      for (int dy = -1; dy <= 1; ++dy) {
        int yy = refl101(y + dy, P), xm = refl101(x - 1, P), xp = refl101(x + 1, P);
        float wgt = dy == 0 ? 2.f : 1.f;
        float a = img[(long)(y0 + yy) * stride + x0 + xp] ? 255.f : 0.f;
        float b = img[(long)(y0 + yy) * stride + x0 + xm] ? 255.f : 0.f;
        gx += wgt * (a - b);
      }
      int v = (int)rintf(gx);
      sum += min(255, max(0, v));
    }
  double m = (double)sum * (1.0 / (double)(P * P));
  return fabs(m) + 1e-20;
}

template <bool BIN>
__device__ __forceinline__ float lane_mi(LaneHist<kScBlock>& h, const uint8_t* A, int ax, int ay, const uint8_t* B,
                                         int bx, int by, int stride, int P, float invN) {
  h.clear();
  const uint8_t* pa = A + (long)ay * stride + ax;
  const uint8_t* pb = B + (long)by * stride + bx;
  for (int y = 0; y < P; ++y) {
    for (int x = 0; x < P; ++x) {
      int va = pa[x], vb = pb[x];
      if (BIN) { va = va ? 255 : 0; vb = vb ? 255 : 0; }
      h.add(va, vb);
    }
    pa += stride;
    pb += stride;
  }
  return h.mi(invN);
}

struct Proj {
  float lx, ly, rx, ry;   // left / right reprojection (float Point2f)
  double ru;              // un-rounded right (left for right tracks) x, for the +dp point
  double rv;
};

// Left tracks: optimisation.cpp:172-181 (residuals) / :461-476 (normal eqs)
__device__ __forceinline__ void project_left(const ScaleArgs& a, const double* X, Proj& p) {
  double T[16], Y[4], f[3], Z[4], f2[3];
  quat_pose(a.q1, a.t1, T);
  mat44_vec(T, X, Y);
  project_scaled(a.K1, a.scale, Y, f);
  p.lx = (float)(f[0] / f[2]);
  p.ly = (float)(f[1] / f[2]);
  for (int c = 0; c < 4; ++c) Z[c] = a.scale * Y[c];
  Z[0] = Z[0] - a.baseline;
  project(a.K2, Z, f2);
  p.ru = f2[0] / f2[2];
  p.rv = f2[1] / f2[2];
  p.rx = (float)p.ru;
  p.ry = (float)p.rv;
}

// Right tracks, residual flavour (optimisation.cpp:202-212): poses.second,
// T col3 += R*b, right projection with K2, left projection with K1.
// KL_FOR_LEFT selects the K used for the left reprojection (normal equations
// use K.second there, optimisation.cpp:516).  POSES_FIRST/NO_SHIFT give the
// compute_jacobian flavour (:596-612).
template <bool LEFT_USES_K2, bool JAC_FLAVOUR>
__device__ __forceinline__ void project_right(const ScaleArgs& a, const double* Xin, Proj& p, double* Zc_out) {
  double X[4] = {Xin[0] - a.baseline, Xin[1] - 0.0, Xin[2] - 0.0, Xin[3] - 0.0};
  double T[16], Y[4], f[3], Z[4], f2[3];
  const double* q = JAC_FLAVOUR ? a.q1 : a.q2;
  const double* t = JAC_FLAVOUR ? a.t1 : a.t2;
  quat_pose(q, t, T);
  double tz = t[2];
  if (!JAC_FLAVOUR) {
    for (int r = 0; r < 3; ++r) {
      double s = 0;
      s += T[r * 4 + 0] * a.baseline;
      s += T[r * 4 + 1] * 0.0;
      s += T[r * 4 + 2] * 0.0;
      s += 0.0 * 0.0;
      if (r == 2) tz = t[2] + s;
      T[r * 4 + 3] = T[r * 4 + 3] + s;
    }
  }
  if (Zc_out) {
    double Xe0 = X[0] / X[3], Xe1 = X[1] / X[3], Xe2 = X[2] / X[3];
    double zc = 0;
    zc += T[8] * Xe0;
    zc += T[9] * Xe1;
    zc += T[10] * Xe2;
    *Zc_out = zc + tz;
  }
  mat44_vec(T, X, Y);
  project_scaled(a.K2, a.scale, Y, f);
  p.rx = (float)(f[0] / f[2]);
  p.ry = (float)(f[1] / f[2]);
  for (int c = 0; c < 4; ++c) Z[c] = a.scale * Y[c];
  Z[0] = Z[0] + a.baseline;
  project(LEFT_USES_K2 ? a.K2 : a.K1, Z, f2);
  p.ru = f2[0] / f2[2];
  p.rv = f2[1] / f2[2];
  p.lx = (float)p.ru;
  p.ly = (float)p.rv;
}

__device__ __forceinline__ double left_Zc(const ScaleArgs& a, const double* X) {
  double T[16];
  quat_pose(a.q1, a.t1, T);
  double Xe0 = X[0] / X[3], Xe1 = X[1] / X[3], Xe2 = X[2] / X[3];
  double zc = 0;
  zc += T[8] * Xe0;
  zc += T[9] * Xe1;
  zc += T[10] * Xe2;
  return zc + a.t1[2];
}

__device__ __forceinline__ bool roi_in(const ScaleArgs& a, int x0, int y0, int P) {
  return x0 >= 0 && y0 >= 0 && x0 + P <= a.cols && y0 + P <= a.rows;
}

// 16 lanes per track (GroupHist): a window has a few thousand tracks, far
// fewer than the lanes of 256 CUs; the reprojection is computed redundantly
// by the 16 lanes (identical doubles), the MI histogram/terms are shared.
constexpr int kTracksPerBlock = kScBlock / 16;
#define SCALE_GROUP_SETUP()                                                 \
  __shared__ uint32_t lds[kTracksPerBlock * kGroupWords];                   \
  const int grp_ = threadIdx.x >> 4;                                        \
  GroupHist<16> h{&lds[grp_ * kGroupWords], (int)(threadIdx.x & 15)};       \
  const int t = blockIdx.x * kTracksPerBlock + grp_;                        \
  if (t >= a.nL + a.nR) return;

template <bool BIN>
__device__ __forceinline__ float grp_mi(GroupHist<16>& h, const uint8_t* A, int ax, int ay, const uint8_t* B, int bx,
                                        int by, int stride, int P, float invN) {
  return group_mi<BIN>(h, A + (long)ay * stride + ax, stride, B + (long)by * stride + bx, stride, P, P, invN);
}

// A4: compute_residuals
__global__ __launch_bounds__(kScBlock) void scale_residual_kernel(ScaleArgs a, TrackDev td, double* __restrict__ res,
                                                                  int* __restrict__ err) {
  SCALE_GROUP_SETUP();
  const int row = td.row[t];
  const uint8_t fl = td.flags[t];
  if (row < 0 || !(fl & 2)) return;
  const bool left = t < a.nL;
  const int w = a.w, P = 2 * w + 1;
  const int bx = w, by = w, bw = a.bb_cols - 2 * w - 1, bh = a.bb_rows - 2 * w - 1;
  Proj p;
  if (left) project_left(a, td.X + 4 * (long)t, p);
  else project_right<false, false>(a, td.X + 4 * (long)t, p, nullptr);
  if (!(rect_contains(bx, by, bw, bh, p.lx, p.ly) && rect_contains(bx, by, bw, bh, p.rx, p.ry))) return;
  int lx = roi_corner(p.lx, w), ly = roi_corner(p.ly, w), rx = roi_corner(p.rx, w), ry = roi_corner(p.ry, w);
  if (!roi_in(a, lx, ly, P) || !roi_in(a, rx, ry, P)) { atomicOr(err, 1); return; }
  double wv = 1.0;
  float mi;
  if (left) {
    if (a.weighting) wv = sobel_weight(a.imgL, a.stride, a.cols, a.rows, lx, ly, P);
    mi = grp_mi<false>(h, a.imgL, lx, ly, a.imgR, rx, ry, a.stride, P, a.invN);
  } else {
    if (a.weighting) wv = sobel_weight(a.imgR, a.stride, a.cols, a.rows, rx, ry, P);
    mi = grp_mi<false>(h, a.imgR, rx, ry, a.imgL, lx, ly, a.stride, P, a.invN);
  }
  if (h.gl == 0) res[row] = (double)mi * wv;
}

// A5: compute_normal_equations — per track J^2*w and J*r_k
__global__ __launch_bounds__(kScBlock) void scale_neq_kernel(ScaleArgs a, TrackDev td, const double* __restrict__ res,
                                                             double* __restrict__ jj, double* __restrict__ je,
                                                             int* __restrict__ err) {
  SCALE_GROUP_SETUP();
  if (h.gl == 0) {
    jj[t] = 0.0;
    je[t] = 0.0;
  }
  const int row = td.row[t];
  const uint8_t fl = td.flags[t];
  if (row < 0 || !(fl & 2)) return;
  const bool left = t < a.nL;
  const int w = a.w, P = 2 * w;
  const int bx = w, by = w, bw = a.bb_cols - 2 * w - 1, bh = a.bb_rows - 2 * w - 1;
  const double* X = td.X + 4 * (long)t;
  Proj p;
  double duds;
  if (left) {
    project_left(a, X, p);
    double Zc = left_Zc(a, X);
    duds = a.K2[0] * a.baseline / (a.scale * Zc);
  } else {
    double Zc;
    project_right<true, false>(a, X, p, &Zc);
    duds = -a.K2[0] * a.baseline / (a.scale * Zc);
  }
  // x0: reference patch; x1 / x2: other image at the reprojection and +1 px
  float x0x_f = left ? p.lx : p.rx, x0y_f = left ? p.ly : p.ry;
  float x1x_f = left ? p.rx : p.lx, x1y_f = left ? p.ry : p.ly;
  float x2x_f = (float)(p.ru + 1.0), x2y_f = (float)p.rv;
  if (!(rect_contains(bx, by, bw, bh, x0x_f, x0y_f) && rect_contains(bx, by, bw, bh, x1x_f, x1y_f))) return;
  int x0x = roi_corner(x0x_f, w), x0y = roi_corner(x0y_f, w);
  int x1x = roi_corner(x1x_f, w), x1y = roi_corner(x1y_f, w);
  int x2x = roi_corner(x2x_f, w), x2y = roi_corner(x2y_f, w);
  if (!roi_in(a, x0x, x0y, P) || !roi_in(a, x1x, x1y, P) || !roi_in(a, x2x, x2y, P)) { atomicOr(err, 1); return; }
  const uint8_t* I0 = left ? a.imgL : a.imgR;
  const uint8_t* I1 = left ? a.imgR : a.imgL;
  double wv = a.weighting ? sobel_weight(I0, a.stride, a.cols, a.rows, x0x, x0y, P) : 1.0;
  double MIp = grp_mi<false>(h, I1, x2x, x2y, I0, x0x, x0y, a.stride, P, a.invN);
  double MIm = grp_mi<false>(h, I1, x1x, x1y, I0, x0x, x0y, a.stride, P, a.invN);
  double J = (MIp - MIm) / 1.0 * duds;
  if (h.gl == 0) {
    jj[t] = J * J * wv;
    je[t] = J * res[row];
  }
}

// A6: compute_jacobian — JJ only; right tracks use poses.first / K.first and
// binarised ROIs (optimisation.cpp:592-632)
__global__ __launch_bounds__(kScBlock) void scale_jac_kernel(ScaleArgs a, TrackDev td, double* __restrict__ jj,
                                                             int* __restrict__ err) {
  SCALE_GROUP_SETUP();
  if (h.gl == 0) jj[t] = 0.0;
  const uint8_t fl = td.flags[t];
  // bit2: unmasked under compute_jacobian's mask indexing (first.size()+i)
  if (!(fl & 4) || !(fl & 8) || !(fl & 2)) return;
  const bool left = t < a.nL;
  const int w = a.w, P = 2 * w;
  const int bx = 2 * w, by = 2 * w, bw = a.bb_cols - 4 * w - 2, bh = a.bb_rows - 4 * w - 2;
  const double* X = td.X + 4 * (long)t;
  Proj p;
  double duds;
  if (left) {
    project_left(a, X, p);
    duds = a.K2[0] * a.baseline / (a.scale * left_Zc(a, X));
  } else {
    double Zc;
    project_right<false, true>(a, X, p, &Zc);
    duds = -a.K1[0] * a.baseline / (a.scale * Zc);
  }
  float x0x_f = left ? p.lx : p.rx, x0y_f = left ? p.ly : p.ry;
  float x1x_f = left ? p.rx : p.lx, x1y_f = left ? p.ry : p.ly;
  float x2x_f = (float)(p.ru + 1.0), x2y_f = (float)p.rv;
  if (!(rect_contains(bx, by, bw, bh, x0x_f, x0y_f) && rect_contains(bx, by, bw, bh, x1x_f, x1y_f) &&
        rect_contains(bx, by, bw, bh, x2x_f, x2y_f)))
    return;
  int x0x = roi_corner(x0x_f, w), x0y = roi_corner(x0y_f, w);
  int x1x = roi_corner(x1x_f, w), x1y = roi_corner(x1y_f, w);
  int x2x = roi_corner(x2x_f, w), x2y = roi_corner(x2y_f, w);
  if (!roi_in(a, x0x, x0y, P) || !roi_in(a, x1x, x1y, P) || !roi_in(a, x2x, x2y, P)) { atomicOr(err, 1); return; }
  double MIp, MIm, wv = 1.0;
  if (left) {
    if (a.weighting) wv = sobel_weight(a.imgL, a.stride, a.cols, a.rows, x0x, x0y, P);
    MIp = grp_mi<false>(h, a.imgR, x2x, x2y, a.imgL, x0x, x0y, a.stride, P, a.invN);
    MIm = grp_mi<false>(h, a.imgR, x1x, x1y, a.imgL, x0x, x0y, a.stride, P, a.invN);
  } else {
    if (a.weighting) wv = sobel_weight_bin(a.imgR, a.stride, x0x, x0y, P);
    MIp = grp_mi<true>(h, a.imgL, x2x, x2y, a.imgR, x0x, x0y, a.stride, P, a.invN);
    MIm = grp_mi<true>(h, a.imgL, x1x, x1y, a.imgR, x0x, x0y, a.stride, P, a.invN);
  }
  double J = (MIp - MIm) / 1.0 * duds;
  if (h.gl == 0) jj[t] = J * J * wv;
}

// Fixed-order reductions: out[0] = sum(x^2) (mode 0) or sum(x) (mode 1) over
// n entries; a second array y (if non-null) is summed into out[1].
constexpr int kRedBlock = 1024;
__global__ __launch_bounds__(kRedBlock) void reduce_kernel(const double* __restrict__ x, const double* __restrict__ y,
                                                           int n, int square, double* __restrict__ out) {
  __shared__ double sx[kRedBlock], sy[kRedBlock];
  double ax = 0, ay = 0;
  for (int i = threadIdx.x; i < n; i += kRedBlock) {
    double v = x[i];
    ax += square ? v * v : v;
    if (y) ay += y[i];
  }
  sx[threadIdx.x] = ax;
  sy[threadIdx.x] = ay;
  __syncthreads();
  for (int s = kRedBlock / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      sx[threadIdx.x] += sx[threadIdx.x + s];
      sy[threadIdx.x] += sy[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = sx[0];
    out[1] = sy[0];
  }
}

// ---------------------------------------------------------------------
// Host side: problem upload + the reference's scalar LM control.
struct ScaleProblem {
  me_ctx* c;
  ScaleArgs a;
  TrackDev td;
  int n;        // tracks
  int rows;     // residual rows (tot_nb_elements)
  double* res;  // device residual vector (rows)
  double* res2;
  double* jj;
  double* je;
  double* red;  // 4 doubles
  int* err;
  double* host; // pinned
};

enum { NO_STOP = 0, SMALL_GRADIENT, SMALL_INCREMENT, MAX_ITERATIONS, SMALL_DECREASE_FUNCTION, SMALL_REPROJ_ERROR,
       NO_CONVERGENCE };

int upload(me_ctx* c, const me_scale_state* s, int weighting, ScaleProblem& P) {
  ME_CHECK(c, s->n_left >= 0 && s->n_right >= 0, "scale: negative track count");
  ME_CHECK(c, s->window_size > 0 && s->cols > 0 && s->rows > 0 && s->stride >= s->cols, "scale: bad image / window");
  ME_CHECK(c, (2 * s->window_size + 1) * (2 * s->window_size + 1) <= 255,
           "scale: window_size %d gives patches above the 255-px lane histogram", s->window_size);
  P.c = c;
  const int n = s->n_left + s->n_right;
  P.n = n;
  ScaleArgs& a = P.a;
  std::memcpy(a.K1, s->K1, sizeof(a.K1));
  std::memcpy(a.K2, s->K2, sizeof(a.K2));
  std::memcpy(a.q1, s->q1, sizeof(a.q1));
  std::memcpy(a.t1, s->t1, sizeof(a.t1));
  std::memcpy(a.q2, s->q2, sizeof(a.q2));
  std::memcpy(a.t2, s->t2, sizeof(a.t2));
  a.scale = s->scale;
  a.baseline = s->baseline;
  a.w = s->window_size;
  a.nL = s->n_left;
  a.nR = s->n_right;
  a.stride = s->stride;
  a.cols = s->cols;
  a.rows = s->rows;
  a.bb_cols = s->bb_cols;
  a.bb_rows = s->bb_rows;
  a.weighting = weighting;
  a.invN = 1.0f;
  // rows: triangulated & unmasked tracks in order (optimisation.cpp:157-194); the
  // right loop tests mask(pts.second.size()+i) (A-6), compute_jacobian mask(pts.first.size()+i)
  const bool has_mask = s->mask && s->mask_len > 0;
  auto mask_at = [&](int idx) { return !has_mask || (idx < s->mask_len && s->mask[idx]); };
  int tot = 0;
  if (has_mask) {
    for (int i = 0; i < s->mask_len; ++i) tot += s->mask[i] ? 1 : 0;
  } else {
    tot = n;
  }
  std::vector<int> row(n > 0 ? n : 1, -1);
  std::vector<uint8_t> flags(n > 0 ? n : 1, 0);
  int k = 0;
  for (int i = 0; i < s->n_left; ++i) {
    uint8_t f = 0;
    bool tri = s->tri_left[i] != 0;
    if (s->last_left[i] == s->lframe) f |= 2;
    if (mask_at(i)) f |= 4;
    if (tri) f |= 8;
    if (mask_at(i) && tri) {
      f |= 1;
      row[i] = k++;
    }
    flags[i] = f;
  }
  for (int i = 0; i < s->n_right; ++i) {
    uint8_t f = 0;
    bool tri = s->tri_right[i] != 0;
    if (s->last_right[i] == s->lframe) f |= 2;
    if (mask_at(s->n_left + i)) f |= 4;
    if (tri) f |= 8;
    if (mask_at(s->n_right + i) && tri) {
      f |= 1;
      row[s->n_left + i] = k++;
    }
    flags[s->n_left + i] = f;
  }
  // rows beyond tot_nb_elements would write outside the reference's Eigen vector (UB there)
  for (int i = 0; i < n; ++i)
    if (row[i] >= tot && (flags[i] & 2))
      return me_set_error(c, ME_ERR_INVALID, "scale: mask selects fewer rows (%d) than triangulated tracks", tot);
  P.rows = tot;
  // device buffers: [X (4n doubles)][row (n ints)][flags (n bytes)]
  size_t bx = 32 * (size_t)n, brow = 4 * (size_t)n, bfl = (size_t)n;
  void* d;
  ME_TRY(me_scratch(c, SLOT_SC_TRACKS, bx + brow + bfl + 64, &d));
  char* base = (char*)d;
  std::vector<double> X(4 * (size_t)(n > 0 ? n : 1));
  if (s->n_left) std::memcpy(X.data(), s->X_left, 32 * (size_t)s->n_left);
  if (s->n_right) std::memcpy(X.data() + 4 * (size_t)s->n_left, s->X_right, 32 * (size_t)s->n_right);
  if (n) {
    ME_HIP(c, hipMemcpyAsync(base, X.data(), bx, hipMemcpyHostToDevice, c->stream));
    ME_HIP(c, hipMemcpyAsync(base + bx, row.data(), brow, hipMemcpyHostToDevice, c->stream));
    ME_HIP(c, hipMemcpyAsync(base + bx + brow, flags.data(), bfl, hipMemcpyHostToDevice, c->stream));
  }
  P.td.X = (const double*)base;
  P.td.row = (const int*)(base + bx);
  P.td.flags = (const uint8_t*)(base + bx + brow);
  if (s->img_mem == ME_DEVICE) {
    a.imgL = s->imgL;
    a.imgR = s->imgR;
  } else {
    void *dl, *dr;
    size_t bytes = (size_t)s->stride * s->rows;
    ME_TRY(me_scratch(c, SLOT_SC_IMGL, bytes, &dl));
    ME_TRY(me_scratch(c, SLOT_SC_IMGR, bytes, &dr));
    ME_HIP(c, hipMemcpyAsync(dl, s->imgL, bytes, hipMemcpyHostToDevice, c->stream));
    ME_HIP(c, hipMemcpyAsync(dr, s->imgR, bytes, hipMemcpyHostToDevice, c->stream));
    a.imgL = (const uint8_t*)dl;
    a.imgR = (const uint8_t*)dr;
  }
  void *dres, *dres2, *dneq;
  size_t nr = (size_t)(tot > 0 ? tot : 1);
  ME_TRY(me_scratch(c, SLOT_SC_RES, 8 * nr, &dres));
  ME_TRY(me_scratch(c, SLOT_SC_RES2, 8 * nr, &dres2));
  ME_TRY(me_scratch(c, SLOT_SC_NEQ, 16 * (size_t)(n > 0 ? n : 1) + 64 + 16, &dneq));
  P.res = (double*)dres;
  P.res2 = (double*)dres2;
  P.jj = (double*)dneq;
  P.je = P.jj + (n > 0 ? n : 1);
  P.red = P.je + (n > 0 ? n : 1);
  P.err = (int*)(P.red + 8);
  void* ph;
  ME_TRY(me_pinned(c, 256, &ph));
  P.host = (double*)ph;
  ME_HIP(c, hipMemsetAsync(P.err, 0, 4, c->stream));
  return ME_OK;
}

int blocks_for(int n) { return n > 0 ? (n + kTracksPerBlock - 1) / kTracksPerBlock : 1; }

int check_err(ScaleProblem& P) {
  // err flag is read back with the scalars
  int e = 0;
  std::memcpy(&e, (char*)P.host + 32, 4);
  if (e) return me_set_error(P.c, ME_ERR_INVALID, "scale: ROI outside the image (reference: cv::Exception)");
  return ME_OK;
}

// residuals at `scale` into dst; returns e = sum r^2 (host)
int eval_residuals(ScaleProblem& P, double scale, double* dst, double* e_out) {
  me_ctx* c = P.c;
  ScaleArgs a = P.a;
  a.scale = scale;
  a.invN = (float)(1.0 / (double)((2 * a.w + 1) * (2 * a.w + 1)));
  ME_HIP(c, hipMemsetAsync(dst, 0, 8 * (size_t)(P.rows > 0 ? P.rows : 1), c->stream));
  if (P.n > 0) {
    me_ktimer t(c, ME_KT_SCALE_RES);
    hipLaunchKernelGGL(scale_residual_kernel, dim3(blocks_for(P.n)), dim3(kScBlock), 0, c->stream, a, P.td, dst,
                       P.err);
  }
  ME_TRY(me_check_launch(c, "scale_residual_kernel"));
  hipLaunchKernelGGL(reduce_kernel, dim3(1), dim3(kRedBlock), 0, c->stream, (const double*)dst,
                     (const double*)nullptr, P.rows, 1, P.red);
  ME_TRY(me_check_launch(c, "reduce_kernel"));
  ME_HIP(c, hipMemcpyAsync(P.host, P.red, 16, hipMemcpyDeviceToHost, c->stream));
  ME_HIP(c, hipMemcpyAsync((char*)P.host + 32, P.err, 4, hipMemcpyDeviceToHost, c->stream));
  ME_HIP(c, hipStreamSynchronize(c->stream));
  ME_TRY(check_err(P));
  *e_out = P.host[0];
  return ME_OK;
}

int eval_neq(ScaleProblem& P, double scale, const double* dres, double* JJ, double* e) {
  me_ctx* c = P.c;
  ScaleArgs a = P.a;
  a.scale = scale;
  a.invN = (float)(1.0 / (double)(4 * a.w * a.w));
  if (P.n > 0) {
    me_ktimer t(c, ME_KT_SCALE_NEQ);
    hipLaunchKernelGGL(scale_neq_kernel, dim3(blocks_for(P.n)), dim3(kScBlock), 0, c->stream, a, P.td, dres, P.jj,
                       P.je, P.err);
  }
  ME_TRY(me_check_launch(c, "scale_neq_kernel"));
  hipLaunchKernelGGL(reduce_kernel, dim3(1), dim3(kRedBlock), 0, c->stream, (const double*)P.jj,
                     (const double*)P.je, P.n, 0, P.red);
  ME_TRY(me_check_launch(c, "reduce_kernel"));
  ME_HIP(c, hipMemcpyAsync(P.host, P.red, 16, hipMemcpyDeviceToHost, c->stream));
  ME_HIP(c, hipMemcpyAsync((char*)P.host + 32, P.err, 4, hipMemcpyDeviceToHost, c->stream));
  ME_HIP(c, hipStreamSynchronize(c->stream));
  ME_TRY(check_err(P));
  *JJ = P.host[0];
  *e = P.host[1];
  return ME_OK;
}

double ldlt1(double JJ, double e) { return std::fabs(JJ) > 2.2250738585072014e-308 ? e / JJ : 0.0; }

}  // namespace

extern "C" void me_optim_default_params(me_optim_params* p) {
  p->type = 1;
  p->minim = 1;
  p->max_nb_iter = 20;
  p->v = 2;
  p->tau = 1e-3;
  p->mu = 1e-20;
  p->abs_tol = 1e-4;
  p->grad_tol = 1e-4;
  p->incr_tol = 1e-3;
  p->rel_tol = 1e-4;
  p->alpha = 1.0;
  p->weighting = 0;
}

extern "C" int me_scale_residuals(me_ctx* c, const me_scale_state* s, int weighting, double* res, int* n_rows) {
  if (!c || !s) return ME_ERR_INVALID;
  ME_HIP(c, hipSetDevice(c->device));
  ScaleProblem P;
  ME_TRY(upload(c, s, weighting, P));
  double e;
  ME_TRY(eval_residuals(P, s->scale, P.res, &e));
  if (P.rows > 0) {
    ME_HIP(c, hipMemcpyAsync(res, P.res, 8 * (size_t)P.rows, hipMemcpyDeviceToHost, c->stream));
    ME_HIP(c, hipStreamSynchronize(c->stream));
  }
  *n_rows = P.rows;
  return ME_OK;
}

extern "C" int me_scale_normal_equations(me_ctx* c, const me_scale_state* s, int weighting, const double* res,
                                         double* JJ, double* e) {
  if (!c || !s) return ME_ERR_INVALID;
  ME_HIP(c, hipSetDevice(c->device));
  ScaleProblem P;
  ME_TRY(upload(c, s, weighting, P));
  if (P.rows > 0) ME_HIP(c, hipMemcpyAsync(P.res, res, 8 * (size_t)P.rows, hipMemcpyHostToDevice, c->stream));
  return eval_neq(P, s->scale, P.res, JJ, e);
}

extern "C" int me_scale_jacobian(me_ctx* c, const me_scale_state* s, int weighting, double* JJ) {
  if (!c || !s) return ME_ERR_INVALID;
  ME_HIP(c, hipSetDevice(c->device));
  ScaleProblem P;
  ME_TRY(upload(c, s, weighting, P));
  ScaleArgs a = P.a;
  a.invN = (float)(1.0 / (double)(4 * a.w * a.w));
  if (P.n > 0)
    hipLaunchKernelGGL(scale_jac_kernel, dim3(blocks_for(P.n)), dim3(kScBlock), 0, c->stream, a, P.td, P.jj, P.err);
  ME_TRY(me_check_launch(c, "scale_jac_kernel"));
  hipLaunchKernelGGL(reduce_kernel, dim3(1), dim3(kRedBlock), 0, c->stream, (const double*)P.jj,
                     (const double*)nullptr, P.n, 0, P.red);
  ME_HIP(c, hipMemcpyAsync(P.host, P.red, 16, hipMemcpyDeviceToHost, c->stream));
  ME_HIP(c, hipMemcpyAsync((char*)P.host + 32, P.err, 4, hipMemcpyDeviceToHost, c->stream));
  ME_HIP(c, hipStreamSynchronize(c->stream));
  ME_TRY(check_err(P));
  *JJ = P.host[0];
  return ME_OK;
}

// optimisation.cpp:29-147 with run_GN_step (:674-683) / run_LM_step (:685-730)
extern "C" int me_scale_optimise(me_ctx* c, me_scale_state* s, const me_optim_params* pin, int test, int* stop_out,
                                 int* iterations, double* trace, int trace_cap, long* mi_evals) {
  if (!c || !s || !pin) return ME_ERR_INVALID;
  ME_HIP(c, hipSetDevice(c->device));
  me_optim_params p = *pin;
  if (test) {
    p.type = 0;
    p.max_nb_iter = 300;
    p.abs_tol = 0;
    p.incr_tol = 0;
    p.grad_tol = 0;
    p.rel_tol = 0;
  }
  ScaleProblem P;
  ME_TRY(upload(c, s, p.weighting, P));
  long nevals = 0;
  // MI evaluations per residual pass / neq pass are counted on the host from
  // the in-view masks the kernels produce; here we count launches * tracks.
  int stop = NO_STOP;
  double scale = s->scale;
  int k = 0, ntrace = 0;
  do {
    double e1;
    ME_TRY(eval_residuals(P, scale, P.res, &e1));
    nevals += P.n;
    double mre = e1 / (double)(P.rows * 1);
    if (mre < p.abs_tol) stop = SMALL_REPROJ_ERROR;
    double JJ, e;
    if (test) {
      JJ = 75;
      e = 1;
    } else {
      ME_TRY(eval_neq(P, scale, P.res, &JJ, &e));
      nevals += 2 * (long)P.n;
    }
    if (k == 0) p.mu = JJ;
    if (std::sqrt(e * e) < p.grad_tol) stop = SMALL_GRADIENT;
    double dX = 0;
    if (p.type == 0) {
      JJ += p.mu;
      dX = ldlt1(JJ, e);
      scale += p.alpha * dX;
    } else {
      for (;;) {
        JJ += p.mu;
        dX = ldlt1(JJ, e);
        if (std::sqrt(dX * dX) <= p.incr_tol) {
          stop = SMALL_INCREMENT;
          break;
        }
        double tmp_scale = scale + p.alpha * dX;
        double e2;
        ME_TRY(eval_residuals(P, tmp_scale, P.res2, &e2));
        nevals += P.n;
        double rho = (p.minim ? -1.0 : 1.0) * (e2 - e1);
        if (rho > 0) {
          p.mu *= std::max(1.0 / 3.0, 1 - std::pow(2 * rho - 1, 3));
          p.v = 2;
          double dd = std::sqrt(e1) - std::sqrt(e2);
          if (dd * dd < p.rel_tol * std::sqrt(e1)) stop = SMALL_DECREASE_FUNCTION;
          scale = tmp_scale;
          break;
        } else {
          p.mu *= p.v;
          double v2 = 2 * p.v;
          if (v2 <= p.v) {
            stop = NO_CONVERGENCE;
            break;
          }
          p.v = v2;
        }
      }
    }
    if (!stop && std::sqrt(dX * dX) <= p.incr_tol) stop = SMALL_INCREMENT;
    double e2;
    ME_TRY(eval_residuals(P, scale, P.res2, &e2));
    nevals += P.n;
    if (p.type == 0 && (e2 - e1) * (e2 - e1) < p.rel_tol) stop = SMALL_DECREASE_FUNCTION;
    if (trace && ntrace < trace_cap) {
      trace[2 * ntrace] = e1;
      trace[2 * ntrace + 1] = scale;
    }
    ntrace++;
  } while (!stop && k++ < p.max_nb_iter);
  if (k == p.max_nb_iter) stop = MAX_ITERATIONS;
  s->scale = scale;
  if (stop_out) *stop_out = stop;
  if (iterations) *iterations = ntrace;
  if (mi_evals) *mi_evals = nevals;
  return ME_OK;
}

extern "C" int me_scale_inliers(me_ctx* c, const me_scale_state* s, int weighting, double threshold, int* idx, int cap,
                                int* n_out) {
  if (!c || !s) return ME_ERR_INVALID;
  me_scale_state t = *s;
  t.mask = nullptr;
  t.mask_len = 0;
  std::vector<double> r(s->n_left + s->n_right + 1);
  int rows = 0;
  ME_TRY(me_scale_residuals(c, &t, weighting, r.data(), &rows));
  int n = 0;
  for (int i = 0; i < rows; ++i)
    if (std::sqrt(r[i] * r[i]) < threshold) {
      if (n < cap) idx[n] = i;
      n++;
    }
  *n_out = n;
  return ME_OK;
}
