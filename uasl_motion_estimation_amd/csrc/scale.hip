// scale.hip — MI stereo-scale optimiser.
//
// Replaces Optimiser<ScaleState, std::vector<std::pair<cv::Mat,cv::Mat>>>
// (src/optimisation/optimisation.cpp:29-228, 435-747).  Each evaluation is
// ONE fused kernel: a lane reprojects its track (double, OpenCV Matx order),
// applies the reference's ROI rounding rules, builds the lane-private MI
// histograms of its patch pair(s) in LDS and writes its residual / Jacobian
// contribution; a single-workgroup kernel then reduces in a fixed order.  The
// scalar LM control (optimise / run_GN_step / run_LM_step) runs on the device
// as a small state machine (ScaleLM) between the evaluations, so an
// optimisation needs no host round trip per evaluation: the host enqueues
// phase-predicated blocks of launches and polls the state every few blocks.
#include <cmath>
#include <cstddef>
#include <cstring>
#include <vector>
#include <algorithm>
#include <atomic>
#include <thread>
#include "me_internal.hpp"
#include "me_device.hpp"
#include "roster.hpp"

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
  const float* tab;    // term table of the P*P-pixel patches (me_mi_table), or null
  const float* tab_r;  // tables of the residual ((2w+1)^2) and normal-equation ((2w)^2) patches
  const float* tab_n;
  int nrows;           // residual rows (rows >= nrows are never written: the prep kernel flags them)
};

// flags per track: bit0 = triangulated & unmasked (owns a row), bit1 = seen in lframe
struct TrackDev {
  const double* XL;    // 4 per left track
  const double* XR;    // 4 per right track
  const uint8_t* flags;
  const int* row;      // residual row of the track or -1
};

// Device-side state of Optimiser::optimise (optimisation.cpp:29-147).
// Phases of one outer iteration: A residuals at s -> e1; B normal equations
// -> JJ, e and the GN / first LM step; C residuals at the LM candidate (LM
// retries loop here); D residuals at the accepted s, stop tests, next k.
enum { PH_A = 0, PH_B, PH_C, PH_D, PH_DONE };
enum { NO_STOP = 0, SMALL_GRADIENT, SMALL_INCREMENT, MAX_ITERATIONS, SMALL_DECREASE_FUNCTION, SMALL_REPROJ_ERROR,
       NO_CONVERGENCE };  // StopCondition (rotation_utils.h:20)
constexpr int kTraceCap = 512;
struct ScaleLM {
  double scale, tmp_scale, mu, v, e1, JJ, e, dX;
  long nevals;
  int phase, k, stop, ntrace, err;
  int cur;  // residual buffer (of kResBufs) holding the residuals at `scale`; candidates take the next ones
  // logical call counts of the reference's loop (a skipped launch still counts
  // the evaluation it stands for): compute_residuals, compute_normal_equations,
  // rejected LM candidates (run_LM_step's else branch)
  int nres, nneq, nrej;
  int gen;     // solve generation (host-chosen): the host ignores a mirror written by an older solve
  int nbatch;  // candidate batches proposed in the current outer iteration
  int nexec;   // residual evaluations actually run on the device (A, every evaluated candidate, GN's D)
  double trace[2 * kTraceCap];
};

// Speculative LM candidates (run_LM_step, optimisation.cpp:688-728).  Until a
// candidate is accepted, the loop's state (JJ += mu, dX, mu *= v, v *= 2)
// does not depend on the evaluations, so the control lays out the next
// candidates in one go and one launch evaluates them all (blockIdx.y =
// candidate, each into its own residual buffer, each reduced in the fixed
// order); the control then walks them in order exactly as the sequential loop
// would: the first with rho > 0 is accepted with the mu of its turn, the ones
// before it count as rejections, the ones after it never happened.  A
// candidate whose scale equals the current scale bit for bit is the current
// state: its residuals are the current ones, e2 == e1, rho = 0, so it is
// rejected without an evaluation (every late candidate of a rejection streak
// is one: its step is below the scale's ulp).
constexpr int kSpecMax = 16;
constexpr int kResBufs = kSpecMax + 1;  // the current residuals + one per candidate
struct ScaleSpec {
  double ts[kSpecMax];   // candidate scale
  double dX[kSpecMax];   // its increment
  double mu[kSpecMax];   // mu at its turn (the accepted candidate's mu update starts there)
  double e2[kSpecMax];   // its residual sum (written by the candidate's last workgroup)
  int skips[kSpecMax];   // same-state candidates rejected without evaluation just before it
  double rs_JJ, rs_mu, rs_v, rs_dX;  // loop state once every candidate of the batch is rejected
  int n, term, tail_skips;           // candidates, terminal stop after them (or NO_STOP), same-state ones after the last
};

__device__ __forceinline__ bool lm_skip(const ScaleLM* lm, int phase) { return lm && lm->phase != phase; }
__device__ __forceinline__ void lm_scale(ScaleArgs& a, const ScaleLM* lm, int use_tmp) {
  if (lm) a.scale = use_tmp ? lm->tmp_scale : lm->scale;
}

__device__ __forceinline__ const double* track_X(const TrackDev& td, const ScaleArgs& a, int t) {
  return t < a.nL ? td.XL + 4 * (long)t : td.XR + 4 * (long)(t - a.nL);
}

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
                                        int by, int stride, int P, float invN, const float* tab, int rows, int cols) {
  const long end = (long)(rows - 1) * stride + cols;  // one past each image's last byte (the row form's bound)
  return group_mi<BIN>(h, A + (long)ay * stride + ax, stride, B + (long)by * stride + bx, stride, P, P, invN, tab,
                       A + end, B + end);
}

// Stores a later workgroup of the same launch reduces (residual rows, JJ / Je
// terms, candidate sums) are written through (agent-scope relaxed atomic
// store: the line goes to memory), so an arrival needs no release -- no L2
// write-back per workgroup and phase beside the BA on the other CUs.
__device__ __forceinline__ void wt_store(double* q, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(q), __builtin_bit_cast(unsigned long long, v),
                     ME_HO_ST, __HIP_MEMORY_SCOPE_AGENT);
}

// A4: compute_residuals, one track per 16-lane group
__device__ void residual_track(const ScaleArgs& a, const TrackDev& td, int t, GroupHist<16>& h,
                               double* __restrict__ res, int* __restrict__ err) {
  const int row = td.row[t];
  const uint8_t fl = td.flags[t];
  if (row < 0 || row >= a.nrows) return;
  if (!(fl & 2)) {  // an owned row stays 0 (the reference leaves it untouched)
    if (h.gl == 0) wt_store(&res[row], 0.0);
    return;
  }
  const bool left = t < a.nL;
  const int w = a.w, P = 2 * w + 1;
  const int bx = w, by = w, bw = a.bb_cols - 2 * w - 1, bh = a.bb_rows - 2 * w - 1;
  Proj p;
  if (left) project_left(a, track_X(td, a, t), p);
  else project_right<false, false>(a, track_X(td, a, t), p, nullptr);
  if (!(rect_contains(bx, by, bw, bh, p.lx, p.ly) && rect_contains(bx, by, bw, bh, p.rx, p.ry))) {
    if (h.gl == 0) wt_store(&res[row], 0.0);
    return;
  }
  int lx = roi_corner(p.lx, w), ly = roi_corner(p.ly, w), rx = roi_corner(p.rx, w), ry = roi_corner(p.ry, w);
  if (!roi_in(a, lx, ly, P) || !roi_in(a, rx, ry, P)) {
    if (h.gl == 0) wt_store(&res[row], 0.0);
    atomicOr(err, 1);
    return;
  }
  double wv = 1.0;
  float mi;
  if (left) {
    if (a.weighting) wv = sobel_weight(a.imgL, a.stride, a.cols, a.rows, lx, ly, P);
    mi = grp_mi<false>(h, a.imgL, lx, ly, a.imgR, rx, ry, a.stride, P, a.invN, a.tab, a.rows, a.cols);
  } else {
    if (a.weighting) wv = sobel_weight(a.imgR, a.stride, a.cols, a.rows, rx, ry, P);
    mi = grp_mi<false>(h, a.imgR, rx, ry, a.imgL, lx, ly, a.stride, P, a.invN, a.tab, a.rows, a.cols);
  }
  if (h.gl == 0) wt_store(&res[row], (double)mi * wv);
}

__global__ __launch_bounds__(kScBlock) void scale_residual_kernel(ScaleArgs a, TrackDev td, double* __restrict__ res,
                                                                  int* __restrict__ err, const ScaleLM* lm, int phase,
                                                                  int use_tmp) {
  if (lm_skip(lm, phase)) return;
  lm_scale(a, lm, use_tmp);
  SCALE_GROUP_SETUP();
  residual_track(a, td, t, h, res, err);
}

// A5: compute_normal_equations — per track J^2*w and J*r_k
__device__ void neq_track(const ScaleArgs& a, const TrackDev& td, int t, GroupHist<16>& h,
                          const double* __restrict__ res, double* __restrict__ jj, double* __restrict__ je,
                          int* __restrict__ err) {
  if (h.gl == 0) {
    wt_store(&jj[t], 0.0);
    wt_store(&je[t], 0.0);
  }
  const int row = td.row[t];
  const uint8_t fl = td.flags[t];
  if (row < 0 || row >= a.nrows || !(fl & 2)) return;
  const bool left = t < a.nL;
  const int w = a.w, P = 2 * w;
  const int bx = w, by = w, bw = a.bb_cols - 2 * w - 1, bh = a.bb_rows - 2 * w - 1;
  const double* X = track_X(td, a, t);
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
  double MIp = grp_mi<false>(h, I1, x2x, x2y, I0, x0x, x0y, a.stride, P, a.invN, a.tab, a.rows, a.cols);
  double MIm = grp_mi<false>(h, I1, x1x, x1y, I0, x0x, x0y, a.stride, P, a.invN, a.tab, a.rows, a.cols);
  double J = (MIp - MIm) / 1.0 * duds;
  if (h.gl == 0) {
    wt_store(&jj[t], J * J * wv);
    // coherent load: in the persistent LM the row may have been written by
    // another workgroup in the previous phase (no kernel boundary between)
    wt_store(&je[t], J * __builtin_bit_cast(double, __hip_atomic_load(reinterpret_cast<const unsigned long long*>(res + row),
                                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
  }
}

__global__ __launch_bounds__(kScBlock) void scale_neq_kernel(ScaleArgs a, TrackDev td, const double* __restrict__ res,
                                                             double* __restrict__ jj, double* __restrict__ je,
                                                             int* __restrict__ err, const ScaleLM* lm) {
  if (lm_skip(lm, PH_B)) return;
  lm_scale(a, lm, 0);
  SCALE_GROUP_SETUP();
  neq_track(a, td, t, h, res, jj, je, err);
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
  const double* X = track_X(td, a, t);
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
    MIp = grp_mi<false>(h, a.imgR, x2x, x2y, a.imgL, x0x, x0y, a.stride, P, a.invN, a.tab, a.rows, a.cols);
    MIm = grp_mi<false>(h, a.imgR, x1x, x1y, a.imgL, x0x, x0y, a.stride, P, a.invN, a.tab, a.rows, a.cols);
  } else {
    if (a.weighting) wv = sobel_weight_bin(a.imgR, a.stride, x0x, x0y, P);
    MIp = grp_mi<true>(h, a.imgL, x2x, x2y, a.imgR, x0x, x0y, a.stride, P, a.invN, a.tab, a.rows, a.cols);
    MIm = grp_mi<true>(h, a.imgL, x1x, x1y, a.imgR, x0x, x0y, a.stride, P, a.invN, a.tab, a.rows, a.cols);
  }
  double J = (MIp - MIm) / 1.0 * duds;
  if (h.gl == 0) jj[t] = J * J * wv;
}

// Fixed-order reduction of one workgroup: sum(x^2) (square) or sum(x) over n
// entries into *ox, and sum(y) into *oy (y may be null).
constexpr int kRedBlock = 1024;
// Per virtual thread v < 1024: strided partial over i = v, v + 1024, ...;
// then the pairwise tree over the 1024 partials.  A block of B threads (B
// divides 1024) plays 1024 / B virtual threads each, so the float result does
// not depend on the block size.
template <int B>
__device__ __forceinline__ void block_reduce2(const double* __restrict__ x, const double* __restrict__ y, int n,
                                              int square, double* ox, double* oy) {
  static_assert(kRedBlock % B == 0, "block size must divide 1024");
  __shared__ double sx[kRedBlock], sy[kRedBlock];
  constexpr int K = kRedBlock / B;
  double ax[K], ay[K];
#pragma unroll
  for (int k = 0; k < K; ++k) ax[k] = ay[k] = 0.0;
  // chunks of 4 strides: the 4K loads of a chunk issue together, then each
  // virtual thread accumulates its entries in increasing i (the fixed order)
  for (int c0 = 0; c0 < n; c0 += 4 * kRedBlock) {
    double wx[K][4], wy[K][4];
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = c0 + threadIdx.x + B * k + kRedBlock * u;
        wx[k][u] = i < n ? x[i] : 0.0;
        wy[k][u] = (y && i < n) ? y[i] : 0.0;
      }
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (c0 + threadIdx.x + B * k + kRedBlock * u < n) {
          ax[k] += square ? wx[k][u] * wx[k][u] : wx[k][u];
          ay[k] += wy[k][u];
        }
      }
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    sx[threadIdx.x + B * k] = ax[k];
    sy[threadIdx.x + B * k] = ay[k];
  }
  __syncthreads();
  for (int s = kRedBlock / 2; s >= 64; s >>= 1) {
    for (int v = threadIdx.x; v < s; v += B) {
      sx[v] += sx[v + s];
      sy[v] += sy[v + s];
    }
    __syncthreads();
  }
  // levels 32 .. 1 of the same tree inside wave 0 (x[v] += x[v + s], same
  // adds in the same order), by shuffles instead of six block barriers
  if (threadIdx.x < 64) {
    double x = sx[threadIdx.x], z = sy[threadIdx.x];
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) {
      x += __shfl_down(x, s, 64);
      z += __shfl_down(z, s, 64);
    }
    if (threadIdx.x == 0) {
      sx[0] = x;
      sy[0] = z;
    }
  }
  __syncthreads();
  *ox = sx[0];
  *oy = sy[0];
  __syncthreads();  // sx / sy are reused by the next reduction of a persistent block
}

__global__ __launch_bounds__(kRedBlock) void reduce_kernel(const double* __restrict__ x, const double* __restrict__ y,
                                                           int n, int square, double* __restrict__ out) {
  double ox, oy;
  block_reduce2<kRedBlock>(x, y, n, square, &ox, &oy);
  if (threadIdx.x == 0) {
    out[0] = ox;
    out[1] = oy;
  }
}

struct LMParams {
  int type, minim, max_nb_iter, test;
  double abs_tol, grad_tol, incr_tol, rel_tol, alpha;
  int rows, n;
  // Coherent host page (or null): every control update also stores the LM
  // header there, the word holding `phase` last behind a system-scope fence,
  // so the host polls it behind an event instead of a D2H copy per block.
  unsigned long long* mirror;
  int mirror_done_only;  // persistent solve: the mirror is written once, at PH_DONE
  long long roster_ticks;  // persistent solve: the roster decider's wait for the grid's joins (roster.hpp)
};

__device__ __forceinline__ double ldlt1(double JJ, double e) { return fabs(JJ) > 2.2250738585072014e-308 ? e / JJ : 0.0; }

// The accepted-state evaluation (phase D) and the loop tail, defined below.
__device__ __forceinline__ void ctrl_after_eval(ScaleLM* lm, double* __restrict__ trace, const LMParams& p,
                                                double e2);

// Lays out the next batch of LM candidates from the register state *lm
// (after phase B, or after a batch whose candidates were all rejected):
// run_LM_step's loop (optimisation.cpp:688-728) run ahead under the
// assumption that every candidate is rejected.  A batch with no candidate to
// evaluate ends in its terminal stop and closes the iteration here.
__device__ void lm_propose_batch(ScaleLM* lm, ScaleSpec* __restrict__ sp, double* __restrict__ trace,
                                 const LMParams& p) {
  const int cap = lm->nbatch == 0 ? 4 : kSpecMax;  // an accept usually comes early; streaks get wide batches
  lm->nbatch++;
  double JJ = lm->JJ, mu = lm->mu, v = lm->v, dX = lm->dX;
  const unsigned long long cur_bits = __double_as_longlong(lm->scale);
  int n = 0, skips = 0, term = NO_STOP;
  while (n < cap) {
    JJ += mu;                 // JJ.diagonal() += mu (:690)
    dX = ldlt1(JJ, lm->e);    // (:692)
    if (sqrt(dX * dX) <= p.incr_tol) {  // (:694-697)
      term = SMALL_INCREMENT;
      break;
    }
    const double ts = lm->scale + p.alpha * dX;  // tmp_state.update(alpha dX) (:699-700)
    if (__double_as_longlong(ts) != cur_bits) {
      sp->ts[n] = ts;
      sp->dX[n] = dX;
      sp->mu[n] = mu;
      sp->skips[n] = skips;
      skips = 0;
      ++n;
    } else {
      ++skips;  // the current state: e2 == e1, rho = 0, rejected
    }
    mu *= v;  // rejection (:719-727)
    const double v2 = 2 * v;
    if (v2 <= v) {
      term = NO_CONVERGENCE;
      break;
    }
    v = v2;
  }
  sp->n = n;
  sp->term = term;
  sp->tail_skips = skips;
  sp->rs_JJ = JJ;
  sp->rs_mu = mu;
  sp->rs_v = v;
  sp->rs_dX = dX;
  if (n > 0) {
    lm->phase = PH_C;
    return;
  }
  // nothing to evaluate: every candidate was the current state, up to the stop
  const long sk = skips;
  lm->nres += (int)sk;
  lm->nrej += (int)sk;
  lm->nevals += sk * p.n;
  lm->JJ = JJ;
  lm->mu = mu;
  lm->v = v;
  lm->dX = dX;
  lm->stop = term;
  // tmp_residuals at the unchanged state (:101): the current residuals, e2 == e1
  ctrl_after_eval(lm, trace, p, lm->e1);
}

// Phase C's control: walk the evaluated batch in the sequential loop's order.
__device__ void lm_walk_batch(ScaleLM* lm, ScaleSpec* __restrict__ sp, double* __restrict__ trace,
                              const LMParams& p) {
  const int n = sp->n;
  const double e1 = lm->e1;
  for (int j = 0; j < n; ++j) {
    const long sk = sp->skips[j];
    lm->nres += (int)sk + 1;
    lm->nrej += (int)sk;
    lm->nevals += (sk + 1) * p.n;
    const double e2 = sp->e2[j];
    const double rho = (p.minim ? -1.0 : 1.0) * (e2 - e1);  // (:705-706)
    if (rho > 0) {  // (:708-717)
      lm->mu = sp->mu[j] * fmax(1.0 / 3.0, 1 - pow(2 * rho - 1, 3));
      lm->v = 2;
      const double dd = sqrt(e1) - sqrt(e2);
      if (dd * dd < p.rel_tol * sqrt(e1)) lm->stop = SMALL_DECREASE_FUNCTION;
      lm->scale = sp->ts[j];
      lm->dX = sp->dX[j];
      // The reference's tmp_residuals (:101) are at scale == ts[j]: candidate
      // j's residuals (same state, same order), whose buffer becomes current.
      lm->cur = (lm->cur + 1 + j) % kResBufs;
      ctrl_after_eval(lm, trace, p, e2);
      return;
    }
    lm->nrej++;
  }
  const long sk = sp->tail_skips;
  lm->nres += (int)sk;
  lm->nrej += (int)sk;
  lm->nevals += sk * p.n;
  lm->JJ = sp->rs_JJ;
  lm->mu = sp->rs_mu;
  lm->v = sp->rs_v;
  lm->dX = sp->rs_dX;
  if (sp->term != NO_STOP) {
    lm->stop = sp->term;
    ctrl_after_eval(lm, trace, p, e1);  // unchanged state: e2 == e1
  } else {
    lm_propose_batch(lm, sp, trace, p);
  }
}

// Phase D's control (optimisation.cpp:100-146): e2 = the residual sum at the
// accepted state.
__device__ __forceinline__ void ctrl_after_eval(ScaleLM* lm, double* __restrict__ trace, const LMParams& p,
                                                double e2) {
  // (the SMALL_INCREMENT test precedes this evaluation in the reference;
  // it only reads dX, so it is applied here with the same result)
  if (!lm->stop && sqrt(lm->dX * lm->dX) <= p.incr_tol) lm->stop = SMALL_INCREMENT;
  lm->nevals += p.n;
  lm->nres++;
  if (p.type == 0 && (e2 - lm->e1) * (e2 - lm->e1) < p.rel_tol) lm->stop = SMALL_DECREASE_FUNCTION;
  if (lm->ntrace < kTraceCap) {
    trace[2 * lm->ntrace] = lm->e1;
    trace[2 * lm->ntrace + 1] = lm->scale;
  }
  lm->ntrace++;
  // while (!stop && k++ < max_nb_iter)
  bool more = false;
  if (!lm->stop) {
    more = lm->k < p.max_nb_iter;
    lm->k++;
  }
  if (more) {
    // The next iteration's compute_residuals(m_state) (optimisation.cpp:51)
    // sees the same m_state as this tmp_residuals evaluation (:100), and the
    // function is pure: its residuals are this phase's (written to the same
    // buffer phase B reads), so phase A's body runs here without a launch.
    lm->e1 = e2;
    lm->nevals += p.n;
    lm->nres++;
    const double mre = e2 / (double)(p.rows * 1);
    if (mre < p.abs_tol) lm->stop = SMALL_REPROJ_ERROR;
    lm->phase = PH_B;
  } else {
    if (lm->k == p.max_nb_iter) lm->stop = MAX_ITERATIONS;
    lm->phase = PH_DONE;
  }
}

// The reference's scalar control for one phase, on the register copy *lm
// (trace entries and candidate batches go straight to device memory).
__device__ void scale_ctrl_decide(ScaleLM* lm, ScaleSpec* __restrict__ sp, double* __restrict__ trace,
                                  const LMParams& p, int phase, double sx, double sy, int err) {
  if (err) {  // ROI outside the image (the reference throws cv::Exception) / bad mask
    lm->err = err;
    lm->phase = PH_DONE;
    return;
  }
  switch (phase) {
    case PH_A: {
      lm->e1 = sx;
      lm->nevals += p.n;
      lm->nres++;
      lm->nexec++;
      const double mre = sx / (double)(p.rows * 1);
      if (mre < p.abs_tol) lm->stop = SMALL_REPROJ_ERROR;
      lm->phase = PH_B;
      break;
    }
    case PH_B: {
      double JJ = 75, e = 1;  // test mode (optimisation.cpp:60-63)
      if (!p.test) {
        JJ = sx;
        e = sy;
        lm->nevals += 2 * (long)p.n;
        lm->nneq++;
      }
      if (lm->k == 0) lm->mu = JJ;
      if (sqrt(e * e) < p.grad_tol) lm->stop = SMALL_GRADIENT;
      lm->JJ = JJ;
      lm->e = e;
      if (p.type == 0) {  // run_GN_step
        lm->JJ += lm->mu;
        lm->dX = ldlt1(lm->JJ, e);
        lm->scale += p.alpha * lm->dX;
        lm->phase = PH_D;
      } else {
        lm->nbatch = 0;
        lm_propose_batch(lm, sp, trace, p);
      }
      break;
    }
    case PH_C:
      lm->nexec += sp->n;
      lm_walk_batch(lm, sp, trace, p);
      break;
    case PH_D:
      lm->nexec++;
      ctrl_after_eval(lm, trace, p, sx);
      break;
  }
}

// Thread 0 of the deciding workgroup: LM header -> registers, the phase's
// control, header back (and into the coherent host mirror, the word holding
// `phase` last behind a system-scope release).
__device__ void scale_ctrl_run(ScaleLM* lm_g, ScaleSpec* __restrict__ sp, const LMParams& p, int phase, double sx,
                               double sy, int err_v) {
  constexpr int kHead = offsetof(ScaleLM, trace) / 8;
  static_assert(offsetof(ScaleLM, trace) % 8 == 0, "LM header is copied as 8-byte words");
  unsigned long long hw[kHead];
  const unsigned long long* src = reinterpret_cast<const unsigned long long*>(lm_g);
#pragma unroll
  for (int i = 0; i < kHead; ++i) hw[i] = src[i];
  ScaleLM L;
  __builtin_memcpy(&L, hw, sizeof(hw));
  scale_ctrl_decide(&L, sp, lm_g->trace, p, phase, sx, sy, err_v);
  __builtin_memcpy(hw, &L, sizeof(hw));
  unsigned long long* dst = reinterpret_cast<unsigned long long*>(lm_g);
#pragma unroll
  for (int i = 0; i < kHead; ++i) dst[i] = hw[i];
  if (p.mirror && (!p.mirror_done_only || L.phase == PH_DONE)) {
    constexpr int kPhaseWord = offsetof(ScaleLM, phase) / 8;
#pragma unroll
    for (int i = 0; i < kHead; ++i)
      if (i != kPhaseWord) __hip_atomic_store(p.mirror + i, hw[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(p.mirror + kPhaseWord, hw[kPhaseWord], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Phase kernels with the control fused in: every workgroup evaluates its
// tracks, then arrives on a counter (release); the last workgroup to arrive
// (acquire) reduces the phase in the 1024-virtual-thread order and runs the
// scalar control (optimisation.cpp:29-147), then re-arms the counter.  One
// launch per LM phase instead of two; a launch whose phase is not the current
// one returns at once (every workgroup reads the phase before the last one can
// change it).
// (Arrival: the workgroup's written-through stores are drained by every wave
// before the barrier, then a relaxed add -- no release, i.e. no L2 write-back
// per workgroup; the last one's acquire still precedes its reads.)
__device__ __forceinline__ bool last_block_arrives(unsigned* cnt, unsigned target) {
  __shared__ int slast;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned k = __hip_atomic_fetch_add(cnt, 1u, ME_HO_RMW, __HIP_MEMORY_SCOPE_AGENT);
    slast = k == target - 1;
  }
  __syncthreads();
  return slast != 0;
}

// Residual buffer b of kResBufs (rows_pad doubles each).
__device__ __forceinline__ double* res_buf(double* base, int rows_pad, int b) { return base + (long)b * rows_pad; }

// A residual launch serves phase A (first != 0: the residuals at the start
// state), phase C (blockIdx.y = candidate j of the batch, at ts[j], into its
// own buffer) or phase D (GN only: the new state, into the current buffer).
// Counters: cnt[1 + j] gathers candidate j's workgroups, its last one reduces
// the candidate and arrives on cnt[0]; the last candidate runs the control.
__global__ __launch_bounds__(kScBlock) void scale_res_ctrl_kernel(ScaleArgs a, TrackDev td, double* __restrict__ resb,
                                                                  int rows_pad, int* __restrict__ err, ScaleLM* lm,
                                                                  ScaleSpec* __restrict__ sp, LMParams p, int first,
                                                                  unsigned* cnt) {
  const int phase = lm->phase;
  if (first ? phase != PH_A : (phase != PH_C && phase != PH_D)) return;
  const int j = blockIdx.y;
  const int ncand = phase == PH_C ? sp->n : 1;
  if (j >= ncand) return;
  const int cur = lm->cur;
  double* res = res_buf(resb, rows_pad, phase == PH_C ? (cur + 1 + j) % kResBufs : cur);
  a.scale = phase == PH_C ? sp->ts[j] : lm->scale;
  __shared__ uint32_t lds[kTracksPerBlock * kGroupWords];
  const int grp = threadIdx.x >> 4;
  GroupHist<16> h{&lds[grp * kGroupWords], (int)(threadIdx.x & 15)};
  const int t = blockIdx.x * kTracksPerBlock + grp;
  if (t < a.nL + a.nR) residual_track(a, td, t, h, res, err);
  if (!last_block_arrives(cnt + 1 + j, gridDim.x)) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  double sx, sy;
  block_reduce2<kScBlock>(res, nullptr, p.rows, 1, &sx, &sy);
  if (threadIdx.x == 0) __hip_atomic_store(cnt + 1 + j, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (phase == PH_C) {
    if (threadIdx.x == 0) wt_store(&sp->e2[j], sx);
    if (!last_block_arrives(cnt, ncand)) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (threadIdx.x == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x == 0) scale_ctrl_run(lm, sp, p, phase, sx, 0.0, *err);
}

__global__ __launch_bounds__(kScBlock) void scale_neq_ctrl_kernel(ScaleArgs a, TrackDev td,
                                                                  const double* __restrict__ resb, int rows_pad,
                                                                  double* __restrict__ jj, double* __restrict__ je,
                                                                  int* __restrict__ err, ScaleLM* lm,
                                                                  ScaleSpec* __restrict__ sp, LMParams p,
                                                                  unsigned* cnt) {
  if (lm->phase != PH_B) return;
  const double* res = resb + (long)lm->cur * rows_pad;
  a.scale = lm->scale;
  __shared__ uint32_t lds[kTracksPerBlock * kGroupWords];
  const int grp = threadIdx.x >> 4;
  GroupHist<16> h{&lds[grp * kGroupWords], (int)(threadIdx.x & 15)};
  const int t = blockIdx.x * kTracksPerBlock + grp;
  if (!p.test && t < a.nL + a.nR) neq_track(a, td, t, h, res, jj, je, err);
  if (!last_block_arrives(cnt + 1, gridDim.x)) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  double sx = 0, sy = 0;
  if (!p.test) block_reduce2<kScBlock>(jj, je, p.n, 0, &sx, &sy);
  if (threadIdx.x == 0) {
    __hip_atomic_store(cnt + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    scale_ctrl_run(lm, sp, p, PH_B, sx, sy, *err);
  }
}

// The whole LM in ONE launch (when the grid fits half the ctx's CUs; else
// the per-phase launches above): a 1-D grid of nb x kCandY workgroups walks
// the phases together.  The grid is NOT assumed co-resident (a plain launch
// promises nothing of the kind: another process, a CU mask or a concurrent
// grid can hold the CUs a later workgroup needs -- VERDICT r5 weak 5).  Every
// workgroup first joins the roster (roster.hpp); the first to join closes it
// once the whole grid has joined or after kCloseTicks, and the work of every
// phase is dealt over the P workgroups that joined: unit u of a phase is
// taken by participant u mod P -- phase A / D residuals and phase B normal
// equations have one unit per track block (nb), phase C one per (track
// block, candidate) with u = j nb + b.  A workgroup dispatched after the
// close leaves at once, so every wait below is on a resident workgroup.
// Per phase each participant arrives on the phase's counters once per unit,
// as the per-phase kernels do (the last arrival reduces the unit-indexed
// partials in the fixed order and runs the control: the same bits for any
// P); the control publishes the phase count on `epoch` (agent-scope release)
// and every participant waits for it (bounded spin, then acquire) before
// reading the next phase.  No launch and no host round trip per phase; the
// host waits for PH_DONE only.  A partner that never arrives (unreachable
// with the roster; kept as a safety net) sets error bit kErrSpin and the grid
// drains.
//
// Register budget: the track work runs out of line on a device copy of the
// parameters (written by the prep launch), re-read in every phase with
// scalar loads; inlined into the phase loop, its invariants (the kernel
// arguments) are hoisted across the loop and the kernel needs >400 registers.
constexpr int kCandY = 2;  // candidate rows of the persistent grid: nb x kCandY workgroups
constexpr int kEpochWord = 40;   // P.bar[kEpochWord]: phases completed (zeroed by the prep launch with the counters)
constexpr int kRosterWord = 42;  // P.bar[kRosterWord .. + 1]: the persistent grid's roster (zeroed likewise)
constexpr long kPhaseSpin = 1L << 22;
constexpr int kErrSpin = 8;
template <class T>
__device__ __forceinline__ T* uniform_ptr(T* q) {
  const unsigned long long v = (unsigned long long)q;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return (T*)(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ double uniform_d(double x) {
  return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(x)),
                          __builtin_amdgcn_readfirstlane(__double2loint(x)));
}
// One track per 16-lane group: residual / normal-equation terms at `scale`
// (two functions: one combined needs 287 registers per lane).
__device__ __noinline__ void lm_res_tracks(const ScaleArgs* ga, double scale, const TrackDev* gtd, double* res,
                                           int* err, int blk) {
  __shared__ uint32_t lds[kTracksPerBlock * kGroupWords];
  ScaleArgs a = *uniform_ptr(ga);
  a.scale = uniform_d(scale);
  const TrackDev td = *uniform_ptr(gtd);
  const int grp = threadIdx.x >> 4;
  GroupHist<16> h{&lds[grp * kGroupWords], (int)(threadIdx.x & 15)};
  const int t = blk * kTracksPerBlock + grp;
  if (t < a.nL + a.nR) residual_track(a, td, t, h, uniform_ptr(res), uniform_ptr(err));
}
__device__ __noinline__ void lm_neq_tracks(const ScaleArgs* ga, double scale, const TrackDev* gtd,
                                           const double* res, double* jj, double* je, int* err, int blk) {
  __shared__ uint32_t lds[kTracksPerBlock * kGroupWords];
  ScaleArgs a = *uniform_ptr(ga);
  a.scale = uniform_d(scale);
  const TrackDev td = *uniform_ptr(gtd);
  const int grp = threadIdx.x >> 4;
  GroupHist<16> h{&lds[grp * kGroupWords], (int)(threadIdx.x & 15)};
  const int t = blk * kTracksPerBlock + grp;
  if (t < a.nL + a.nR)
    neq_track(a, td, t, h, uniform_ptr(res), uniform_ptr(jj), uniform_ptr(je), uniform_ptr(err));
}
#ifdef ME_SCALE_TS  // timing experiment only (tools/drivers.py scale_ts): phase split of the persistent LM, 100 MHz ticks
// workgroup (0, 0)'s view: [0] phases, [1] launches, [2] launch wall, [3] track work A/D, [4] B, [5] C,
// [6] waits for the phase's control (after its own work), [7] phases of type A/D, [8] B, [9] C;
// the controlling workgroup: [10] reduce + control (from its arrival), [11] controls
__device__ unsigned long long g_scale_ts[16];
#define SC_T() ((long long)__builtin_amdgcn_s_memrealtime())
#define SC_ADD(k, v) atomicAdd(&g_scale_ts[(k)], (unsigned long long)(v))
#define SC_WG0 (blockIdx.x == 0 && threadIdx.x == 0)
#endif
__device__ __forceinline__ void lm_publish(unsigned* epoch, unsigned v) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __hip_atomic_store(epoch, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ __launch_bounds__(kScBlock) void scale_lm_kernel(const ScaleArgs* gaR, const ScaleArgs* gaN,
                                                            const TrackDev* gtd, double* __restrict__ resb,
                                                            int rows_pad, double* __restrict__ jj,
                                                            double* __restrict__ je, int* __restrict__ err,
                                                            ScaleLM* lm, ScaleSpec* __restrict__ sp, LMParams p,
                                                            unsigned* cnt, unsigned* epoch, unsigned* roster, int nb,
                                                            int max_phases) {
  __shared__ int s_phase, s_n, s_cur, s_quit, s_pid, s_np;
  __shared__ double s_scale, s_ts[kSpecMax];
  // the roster (roster.hpp): the participants and this workgroup's index among them
  if (threadIdx.x == 0) {
    int pid = me_roster::join<me_roster_dev>(roster, gridDim.x), np = 0;
    if (pid == 0) {
      np = (int)me_roster::close<me_roster_dev>(roster, gridDim.x, p.roster_ticks);
    } else if (pid > 0) {
      np = me_roster::count<me_roster_dev>(roster);
      if (np < 0) {
        atomicOr(err, kErrSpin);
        pid = -1;
      }
    }
    s_pid = pid;
    s_np = np;
  }
  __syncthreads();
  const int pid = s_pid, np = s_np;
  if (pid < 0) return;  // dispatched after the close: the participants do this workgroup's units
  // the LM state is read with coherent (agent-scope atomic) loads: no
  // acquire fence -- an L2 invalidate -- per workgroup and phase
  auto ld_i = [](const int* q) { return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  auto ld_d = [](const double* q) {
    return __builtin_bit_cast(double, __hip_atomic_load(reinterpret_cast<const unsigned long long*>(q),
                                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  };
#ifdef ME_SCALE_TS
  long long ts_launch = 0, ts_ph = 0, ts_work = 0;
  if (SC_WG0) ts_launch = SC_T();
#endif
  for (int ph = 0; ph < max_phases; ++ph) {
#ifdef ME_SCALE_TS
    if (SC_WG0) ts_ph = SC_T();
#endif
    if (threadIdx.x == 0) {
      s_phase = ld_i(&lm->phase);
      s_cur = ld_i(&lm->cur);
      s_scale = ld_d(&lm->scale);
      const int n = s_phase == PH_C ? ld_i(&sp->n) : 0;
      s_n = n;
      for (int j = 0; j < n; ++j) s_ts[j] = ld_d(&sp->ts[j]);
    }
    __syncthreads();
    const int phase = s_phase;
#ifdef ME_SCALE_TS
    if (phase == PH_DONE) {
      if (SC_WG0) {
        SC_ADD(1, 1);
        SC_ADD(2, SC_T() - ts_launch);
      }
      return;
    }
#else
    if (phase == PH_DONE) return;
#endif
    const int cur = s_cur;
#ifdef ME_SCALE_TS
    long long ts_ctrl = 0;
    auto sc_work_done = [&](int k) {
      if (SC_WG0) {
        ts_work = SC_T();
        SC_ADD(k, ts_work - ts_ph);
        SC_ADD(k + 4, 1);
        SC_ADD(0, 1);
      }
    };
    auto sc_ctrl_begin = [&]() { if (threadIdx.x == 0) ts_ctrl = SC_T(); };
    // A/B/D controls: [12] acquire, [13] reduce, [14] control, [15] publish (from the arrival)
    long long ts_sub = 0;
    auto sc_sub = [&](int k) {
      if (threadIdx.x == 0) {
        const long long t_ = SC_T();
        SC_ADD(k, t_ - (k == 12 ? ts_ctrl : ts_sub));
        ts_sub = t_;
      }
    };
    auto sc_ctrl_end = [&]() { if (threadIdx.x == 0) { SC_ADD(10, SC_T() - ts_ctrl); SC_ADD(11, 1); } };
#else
    auto sc_work_done = [](int) {};
    auto sc_ctrl_begin = []() {};
    auto sc_sub = [](int) {};
    auto sc_ctrl_end = []() {};
#endif
    if (phase == PH_B) {
      const double* res = resb + (long)cur * rows_pad;
      for (int u = pid; u < nb; u += np) {
        if (!p.test) lm_neq_tracks(gaN, s_scale, gtd, res, jj, je, err, u);
        sc_work_done(4);
        if (last_block_arrives(cnt + 1, nb)) {
          sc_ctrl_begin();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          double sx = 0, sy = 0;
          if (!p.test) block_reduce2<kScBlock>(jj, je, p.n, 0, &sx, &sy);
          if (threadIdx.x == 0) {
            __hip_atomic_store(cnt + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            scale_ctrl_run(lm, sp, p, PH_B, sx, sy, *err);
            lm_publish(epoch, (unsigned)ph + 1);
          }
          sc_ctrl_end();
        }
      }
    } else if (phase == PH_A || phase == PH_D) {
      double* res = res_buf(resb, rows_pad, cur);
      for (int u = pid; u < nb; u += np) {
        lm_res_tracks(gaR, s_scale, gtd, res, err, u);
        sc_work_done(3);
        if (last_block_arrives(cnt + 1, nb)) {
          sc_ctrl_begin();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          sc_sub(12);
          double sx, sy;
          block_reduce2<kScBlock>(res, nullptr, p.rows, 1, &sx, &sy);
          sc_sub(13);
          if (threadIdx.x == 0) {
            __hip_atomic_store(cnt + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            scale_ctrl_run(lm, sp, p, phase, sx, 0.0, *err);
            sc_sub(14);
            lm_publish(epoch, (unsigned)ph + 1);
            sc_sub(15);
          }
          sc_ctrl_end();
        }
      }
    } else {  // PH_C: the batch's candidates, unit u = j nb + track block
      const int n = s_n;
      for (int u = pid; u < nb * n; u += np) {
        const int j = u / nb, blk = u - j * nb;
        double* res = res_buf(resb, rows_pad, (cur + 1 + j) % kResBufs);
        lm_res_tracks(gaR, s_ts[j], gtd, res, err, blk);
        if (last_block_arrives(cnt + 1 + j, nb)) {
          sc_ctrl_begin();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          double sx, sy;
          block_reduce2<kScBlock>(res, nullptr, p.rows, 1, &sx, &sy);
          if (threadIdx.x == 0) {
            __hip_atomic_store(cnt + 1 + j, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            wt_store(&sp->e2[j], sx);
          }
          if (last_block_arrives(cnt, (unsigned)n)) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            if (threadIdx.x == 0) {
              __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              scale_ctrl_run(lm, sp, p, PH_C, 0.0, 0.0, *err);
              lm_publish(epoch, (unsigned)ph + 1);
            }
          }
          sc_ctrl_end();
        }
      }
      sc_work_done(5);
    }
    // wait for the phase's control (bounded), then read the next phase
    if (threadIdx.x == 0) {
      long k = 0;
      for (; k < kPhaseSpin; ++k) {
        if (__hip_atomic_load(epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > (unsigned)ph) break;
        __builtin_amdgcn_s_sleep(1);
      }
      s_quit = k == kPhaseSpin;
      if (s_quit) atomicOr(err, kErrSpin);
#ifdef ME_SCALE_TS
      if (SC_WG0) SC_ADD(6, SC_T() - ts_work);
#endif
    }
    __syncthreads();
    if (s_quit) return;
  }
}

// Track flags / residual rows (optimisation.cpp:157-194) from the raw track
// arrays: bit0 = owns a residual row (triangulated and unmasked; the right
// loop tests mask(pts.second.size()+i), SURVEY A-6), bit1 = seen in the last
// keyframe, bit2 = unmasked under compute_jacobian's indexing
// (mask(pts.first.size()+i)), bit3 = triangulated.  Rows are the running
// count of bit0 in track order (one workgroup scan).
struct PrepArgs {
  const uint8_t* tri_l;
  const uint8_t* tri_r;
  const uint32_t* last_l;
  const uint32_t* last_r;
  const uint8_t* mask;  // device copy or null
  int mask_len, nL, nR, tot;
  uint32_t lframe;
  // Zeroing and LM start state folded into this launch (were two fills and an
  // H2D copy on the stream): unowned residual rows of zero_bufs buffers, the error
  // flag | arrival counter block (kErrWords words) and, when lm != null, the
  // ScaleLM header (optimisation.cpp:29-40: scale, mu, v, phase A, no stop).
  double* zero;
  int zero_bufs, rows_pad;
  unsigned* err_block;
  ScaleLM* lm;
  double scale0, mu0, v0;
  int gen;
  // device copy of the persistent LM kernel's parameters (residual and
  // normal-equation ScaleArgs, TrackDev), or null
  ScaleArgs args[2];
  TrackDev td;
  unsigned long long* args_out;
};
constexpr int kArgsWords = (2 * sizeof(ScaleArgs) + sizeof(TrackDev)) / 8;
static_assert((2 * sizeof(ScaleArgs) + sizeof(TrackDev)) % 8 == 0, "parameter copy in 8-byte words");
constexpr int kPrepBlock = 1024;
constexpr int kErrWords = 64;
__global__ __launch_bounds__(kPrepBlock) void scale_prep_kernel(PrepArgs pa, uint8_t* flags, int* row, int* err) {
  __shared__ int wsum[kPrepBlock / 64];
  const int n = pa.nL + pa.nR, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (t < kErrWords) pa.err_block[t] = 0u;
  if (pa.args_out && t < kArgsWords) pa.args_out[t] = reinterpret_cast<const unsigned long long*>(pa.args)[t];
  if (pa.lm && t == 0) {
    ScaleLM* lm = pa.lm;
    lm->scale = pa.scale0;
    lm->tmp_scale = 0.0;
    lm->mu = pa.mu0;
    lm->v = pa.v0;
    lm->e1 = lm->JJ = lm->e = lm->dX = 0.0;
    lm->nevals = 0;
    lm->phase = PH_A;
    lm->k = 0;
    lm->stop = NO_STOP;
    lm->ntrace = 0;
    lm->err = 0;
    lm->cur = 0;
    lm->nres = lm->nneq = lm->nrej = 0;
    lm->gen = pa.gen;
    lm->nbatch = 0;
    lm->nexec = 0;
  }
  __syncthreads();  // err cleared before the scan below may set it
  auto mask_at = [&](int idx) { return !pa.mask || (idx < pa.mask_len && pa.mask[idx]); };
  const int chunk = (n + kPrepBlock - 1) / kPrepBlock;
  const int beg = min(n, t * chunk), end = min(n, beg + chunk);
  int cnt = 0;
  for (int i = beg; i < end; ++i) {
    const bool left = i < pa.nL;
    const int r = left ? i : i - pa.nL;
    const bool tri = (left ? pa.tri_l[r] : pa.tri_r[r]) != 0;
    const uint32_t last = left ? pa.last_l[r] : pa.last_r[r];
    uint8_t f = 0;
    if (last == pa.lframe) f |= 2;
    if (mask_at(i)) f |= 4;
    if (tri) f |= 8;
    if (tri && mask_at(left ? i : pa.nR + r)) f |= 1;
    flags[i] = f;
    cnt += f & 1;
  }
  int x = cnt;
  for (int off = 1; off < 64; off <<= 1) {
    const int yv = __shfl_up(x, off, 64);
    if (lane >= off) x += yv;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  int base = 0, owned = 0;
  for (int k = 0; k < kPrepBlock / 64; ++k) {
    if (k < wv) base += wsum[k];
    owned += wsum[k];
  }
  // rows no track owns (a mask selecting more rows than triangulated tracks)
  // are never written by an evaluation: zero them in every residual buffer
  for (int b = 0; b < pa.zero_bufs; ++b)
    for (int i = owned + t; i < pa.tot; i += kPrepBlock) pa.zero[(long)b * pa.rows_pad + i] = 0.0;
  int r = base + x - cnt;
  for (int i = beg; i < end; ++i) {
    if (flags[i] & 1) {
      row[i] = r;
      // rows beyond tot_nb_elements would write outside the reference's Eigen vector (UB there)
      if (r >= pa.tot && (flags[i] & 2)) atomicOr(err, 2);
      ++r;
    } else {
      row[i] = -1;
    }
  }
}

// ---------------------------------------------------------------------
// Host side: problem upload + the enqueue / poll loop.
struct ScaleProblem {
  me_ctx* c;
  ScaleArgs a;
  TrackDev td;
  int n;        // tracks
  int rows;     // residual rows (tot_nb_elements)
  double* res;  // device residual vectors: kResBufs buffers of rows_pad doubles (buffer 0 = the one-shot entry points')
  int rows_pad;
  double* jj;
  double* je;
  double* red;  // 4 doubles
  int* err;
  unsigned* bar;  // arrival counter of the fused phase + control kernels
  ScaleLM* lm;
  ScaleSpec* spec;
  const ScaleArgs* dargs;  // device copy: residual, normal-equation parameters (persistent LM)
  const TrackDev* dtd;
  char* host;   // pinned: input staging | read-back
};

ScaleArgs with_invN(ScaleArgs a, int P) {
  a.invN = (float)(1.0 / (double)(P * P));
  a.tab = P == 2 * a.w + 1 ? a.tab_r : P == 2 * a.w ? a.tab_n : nullptr;
  return a;
}

// lm0 (me_scale_optimise only): the LM start state {scale, mu, v}, written by the prep launch
int upload(me_ctx* c, const me_scale_state* s, int weighting, ScaleProblem& P, const double* lm0 = nullptr,
           int gen = 0) {
  ME_CHECK(c, s->n_left >= 0 && s->n_right >= 0, "scale: negative track count");
  ME_CHECK(c, s->window_size > 0 && s->cols > 0 && s->rows > 0 && s->stride >= s->cols, "scale: bad image / window");
  ME_CHECK(c, (2 * s->window_size + 1) * (2 * s->window_size + 1) <= 255,
           "scale: window_size %d gives patches above the 255-px lane histogram", s->window_size);
  ME_CHECK(c, s->tracks_mem == ME_HOST || s->tracks_mem == ME_DEVICE, "scale: bad tracks_mem");
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
  a.tab = nullptr;
  ME_TRY(me_mi_table(c, (2 * a.w + 1) * (2 * a.w + 1), &a.tab_r));
  ME_TRY(me_mi_table(c, 4 * a.w * a.w, &a.tab_n));
  const bool has_mask = s->mask && s->mask_len > 0;
  int tot = 0;
  if (has_mask) {
    for (int i = 0; i < s->mask_len; ++i) tot += s->mask[i] ? 1 : 0;
  } else {
    tot = n;
  }
  P.rows = tot;
  a.nrows = tot;
  const size_t nn = (size_t)(n > 0 ? n : 1), nr = (size_t)(tot > 0 ? tot : 1);
  // device layout: [XL 4nL | XR 4nR][tri nL | tri nR][last nL | last nR][mask][flags n][row n]
  //                [res: kResBufs x rows_pad][jj n][je n][red 8][err][ScaleLM][ScaleSpec]
  auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const bool dev = s->tracks_mem == ME_DEVICE;
  const size_t bX = 32 * nn, bTri = nn, bLast = 4 * nn, bMask = has_mask ? (size_t)s->mask_len : 1;
  const size_t oX = 0, oTri = oX + up(bX), oLast = oTri + up(bTri), oMask = oLast + up(bLast);
  const size_t in_span = oMask + up(bMask);
  const size_t rows_pad = up(8 * nr) / 8;
  const size_t nbufs = lm0 ? kResBufs : 1;
  const size_t oFl = in_span, oRow = oFl + up(nn), oRes = oRow + up(4 * nn);
  const size_t oJJ = oRes + nbufs * 8 * rows_pad, oJE = oJJ + up(8 * nn), oRed = oJE + up(8 * nn), oErr = oRed + 256;
  const size_t oLM = oErr + 256, oSpec = oLM + up(sizeof(ScaleLM)), oArgs = oSpec + up(sizeof(ScaleSpec));
  const size_t total = oArgs + up(8 * (size_t)kArgsWords);
  void* d;
  ME_TRY(me_scratch(c, SLOT_SC_TRACKS, total, &d));
  char* base = (char*)d;
  void* ph;
  ME_TRY(me_pinned(c, up(in_span) + 256, &ph));
  P.host = (char*)ph;
  PrepArgs pa;
  pa.mask = has_mask ? (const uint8_t*)(base + oMask) : nullptr;
  pa.mask_len = has_mask ? s->mask_len : 0;
  pa.nL = s->n_left;
  pa.nR = s->n_right;
  pa.tot = tot;
  pa.lframe = s->lframe;
  if (!dev) {  // pack every host array at its device offset: one H2D copy
    char* h = P.host;
    if (s->n_left) std::memcpy(h + oX, s->X_left, 32 * (size_t)s->n_left);
    if (s->n_right) std::memcpy(h + oX + 32 * (size_t)s->n_left, s->X_right, 32 * (size_t)s->n_right);
    if (s->n_left) std::memcpy(h + oTri, s->tri_left, s->n_left);
    if (s->n_right) std::memcpy(h + oTri + s->n_left, s->tri_right, s->n_right);
    if (s->n_left) std::memcpy(h + oLast, s->last_left, 4 * (size_t)s->n_left);
    if (s->n_right) std::memcpy(h + oLast + 4 * (size_t)s->n_left, s->last_right, 4 * (size_t)s->n_right);
    if (has_mask) std::memcpy(h + oMask, s->mask, s->mask_len);
    ME_HIP(c, hipMemcpyAsync(base, h, in_span, hipMemcpyHostToDevice, c->stream));
    P.td.XL = (const double*)(base + oX);
    P.td.XR = P.td.XL + 4 * (size_t)s->n_left;
    pa.tri_l = (const uint8_t*)(base + oTri);
    pa.tri_r = pa.tri_l + s->n_left;
    pa.last_l = (const uint32_t*)(base + oLast);
    pa.last_r = pa.last_l + s->n_left;
  } else {
    if (has_mask) {
      std::memcpy(P.host, s->mask, s->mask_len);
      ME_HIP(c, hipMemcpyAsync(base + oMask, P.host, s->mask_len, hipMemcpyHostToDevice, c->stream));
    }
    P.td.XL = s->X_left;
    P.td.XR = s->X_right;
    pa.tri_l = s->tri_left;
    pa.tri_r = s->tri_right;
    pa.last_l = s->last_left;
    pa.last_r = s->last_right;
  }
  P.td.flags = (const uint8_t*)(base + oFl);
  P.td.row = (const int*)(base + oRow);
  P.res = (double*)(base + oRes);
  P.rows_pad = (int)rows_pad;
  P.jj = (double*)(base + oJJ);
  P.je = (double*)(base + oJE);
  P.red = (double*)(base + oRed);
  P.err = (int*)(base + oErr);
  P.bar = (unsigned*)(base + oErr + 64);
  P.lm = (ScaleLM*)(base + oLM);
  P.spec = (ScaleSpec*)(base + oSpec);
  // zeroed by the prep launch: residual rows never owned by a track stay 0;
  // error flag | arrival counter; LM start state
  pa.zero = P.res;
  pa.zero_bufs = (int)nbufs;
  pa.rows_pad = (int)rows_pad;
  pa.err_block = (unsigned*)(base + oErr);
  static_assert(4 * kErrWords == 256, "error flag | arrival counter block");
  pa.lm = lm0 ? P.lm : nullptr;
  pa.scale0 = lm0 ? lm0[0] : 0.0;
  pa.mu0 = lm0 ? lm0[1] : 0.0;
  pa.v0 = lm0 ? lm0[2] : 0.0;
  pa.gen = gen;
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
  // the prep launch runs last: it also writes the device copy of the final parameters
  P.dargs = (const ScaleArgs*)(base + oArgs);
  P.dtd = (const TrackDev*)(base + oArgs + 2 * sizeof(ScaleArgs));
  pa.args[0] = with_invN(a, 2 * a.w + 1);  // residual patches (2w+1)^2
  pa.args[1] = with_invN(a, 2 * a.w);      // normal-equation patches (2w)^2
  pa.td = P.td;
  pa.args_out = lm0 ? (unsigned long long*)(base + oArgs) : nullptr;
  hipLaunchKernelGGL(scale_prep_kernel, dim3(1), dim3(kPrepBlock), 0, c->stream, pa, (uint8_t*)(base + oFl),
                     (int*)(base + oRow), P.err);
  ME_TRY(me_check_launch(c, "scale_prep_kernel"));
  return ME_OK;
}

int blocks_for(int n) { return n > 0 ? (n + kTracksPerBlock - 1) / kTracksPerBlock : 1; }

int check_err(me_ctx* c, int e) {
  if (e & 2) return me_set_error(c, ME_ERR_INVALID, "scale: mask selects fewer rows than triangulated tracks");
  if (e & 1) return me_set_error(c, ME_ERR_INVALID, "scale: ROI outside the image (reference: cv::Exception)");
  if (e & kErrSpin) return me_set_error(c, ME_ERR_STATE, "scale: LM workgroups timed out waiting for a phase");
  return ME_OK;
}


// one evaluation (no LM state): residual rows at a.scale, reduce, read back
int eval_once_residuals(ScaleProblem& P, double* e_out) {
  me_ctx* c = P.c;
  ScaleArgs a = with_invN(P.a, 2 * P.a.w + 1);
  if (P.n > 0) {
    me_ktimer t(c, ME_KT_SCALE_RES);
    hipLaunchKernelGGL(scale_residual_kernel, dim3(blocks_for(P.n)), dim3(kScBlock), 0, c->stream, a, P.td, P.res,
                       P.err, (const ScaleLM*)nullptr, 0, 0);
  }
  hipLaunchKernelGGL(reduce_kernel, dim3(1), dim3(kRedBlock), 0, c->stream, (const double*)P.res,
                     (const double*)nullptr, P.rows, 1, P.red);
  ME_TRY(me_check_launch(c, "scale residuals"));
  ME_HIP(c, hipMemcpyAsync(P.host, P.red, 16, hipMemcpyDeviceToHost, c->stream));
  ME_HIP(c, hipMemcpyAsync(P.host + 32, P.err, 4, hipMemcpyDeviceToHost, c->stream));
  ME_HIP(c, hipStreamSynchronize(c->stream));
  int e;
  std::memcpy(&e, P.host + 32, 4);
  ME_TRY(check_err(c, e));
  if (e_out) std::memcpy(e_out, P.host, 8);
  return ME_OK;
}

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
  ME_TRY(eval_once_residuals(P, nullptr));
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
  ScaleArgs a = with_invN(P.a, 2 * P.a.w);
  if (P.n > 0) {
    me_ktimer t(c, ME_KT_SCALE_NEQ);
    hipLaunchKernelGGL(scale_neq_kernel, dim3(blocks_for(P.n)), dim3(kScBlock), 0, c->stream, a, P.td,
                       (const double*)P.res, P.jj, P.je, P.err, (const ScaleLM*)nullptr);
  }
  hipLaunchKernelGGL(reduce_kernel, dim3(1), dim3(kRedBlock), 0, c->stream, (const double*)P.jj,
                     (const double*)P.je, P.n, 0, P.red);
  ME_TRY(me_check_launch(c, "scale normal equations"));
  ME_HIP(c, hipMemcpyAsync(P.host, P.red, 16, hipMemcpyDeviceToHost, c->stream));
  ME_HIP(c, hipMemcpyAsync(P.host + 32, P.err, 4, hipMemcpyDeviceToHost, c->stream));
  ME_HIP(c, hipStreamSynchronize(c->stream));
  int err;
  std::memcpy(&err, P.host + 32, 4);
  ME_TRY(check_err(c, err));
  std::memcpy(JJ, P.host, 8);
  std::memcpy(e, P.host + 8, 8);
  return ME_OK;
}

extern "C" int me_scale_jacobian(me_ctx* c, const me_scale_state* s, int weighting, double* JJ) {
  if (!c || !s) return ME_ERR_INVALID;
  ME_HIP(c, hipSetDevice(c->device));
  ScaleProblem P;
  ME_TRY(upload(c, s, weighting, P));
  ScaleArgs a = with_invN(P.a, 2 * P.a.w);
  if (P.n > 0)
    hipLaunchKernelGGL(scale_jac_kernel, dim3(blocks_for(P.n)), dim3(kScBlock), 0, c->stream, a, P.td, P.jj, P.err);
  hipLaunchKernelGGL(reduce_kernel, dim3(1), dim3(kRedBlock), 0, c->stream, (const double*)P.jj,
                     (const double*)nullptr, P.n, 0, P.red);
  ME_TRY(me_check_launch(c, "scale_jac_kernel"));
  ME_HIP(c, hipMemcpyAsync(P.host, P.red, 16, hipMemcpyDeviceToHost, c->stream));
  ME_HIP(c, hipMemcpyAsync(P.host + 32, P.err, 4, hipMemcpyDeviceToHost, c->stream));
  ME_HIP(c, hipStreamSynchronize(c->stream));
  int err;
  std::memcpy(&err, P.host + 32, 4);
  ME_TRY(check_err(c, err));
  std::memcpy(JJ, P.host, 8);
  return ME_OK;
}

// optimisation.cpp:29-147 with run_GN_step (:674-683) / run_LM_step (:685-730).
// Launch form of the scale LM (host logic, exported for the CPU test of the
// selection, tests/test_host.py): the persistent grid (nb x kCandY
// workgroups) while it takes at most half of the `cap` workgroups that fit on
// the ctx's CUs, else the per-phase launches.  Never an environment switch:
// the persistent grid is safe at any residency (roster.hpp), so this is a
// throughput choice only.
extern "C" int me_scale_persistent(int nb, int cap) { return cap > 0 && 2L * nb * kCandY <= (long)cap ? 1 : 0; }

// The control runs on the device (fused into the phase kernels); the host
// enqueues blocks of phase-predicated launches and polls the state.
extern "C" int me_scale_optimise(me_ctx* c, me_scale_state* s, const me_optim_params* pin, int test, int* stop_out,
                                 int* iterations, double* trace, int trace_cap, long* mi_evals) {
  me_range range_("me_scale_optimise");
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
  const double lm0[3] = {s->scale, p.mu, p.v};  // initial state (set on the device by the prep launch)
  LMParams lp;
  lp.type = p.type;
  lp.minim = p.minim;
  lp.max_nb_iter = p.max_nb_iter;
  lp.test = test;
  lp.abs_tol = p.abs_tol;
  lp.grad_tol = p.grad_tol;
  lp.incr_tol = p.incr_tol;
  lp.rel_tol = p.rel_tol;
  lp.alpha = p.alpha;
  lp.roster_ticks = me_roster::kCloseTicks;
  if (!c->scale_mirror) ME_HIP(c, hipHostMalloc(&c->scale_mirror, 4096, hipHostMallocCoherent));
  constexpr size_t kHeadBytes = offsetof(ScaleLM, trace);
  static_assert(kHeadBytes <= 4096, "LM header mirror page");
  lp.mirror = (unsigned long long*)c->scale_mirror;
  lp.mirror_done_only = 0;
  volatile ScaleLM* mir = (volatile ScaleLM*)c->scale_mirror;
  // Solve generation: launches of an earlier solve abandoned on an error path
  // may still be queued ahead of this one and write the mirror; their header
  // carries the older generation and is ignored (the device copy is reset by
  // this solve's prep launch, which runs after them in stream order).
  const int gen = ++c->scale_gen;
  mir->gen = gen;
  mir->phase = PH_A;  // the start state (the prep launch writes the device copy)
  ME_TRY(upload(c, s, p.weighting, P, lm0, gen));
  lp.rows = P.rows;
  lp.n = P.n;
  const ScaleArgs aR = with_invN(P.a, 2 * P.a.w + 1), aN = with_invN(P.a, 2 * P.a.w);
  const int nb = blocks_for(P.n);
  hipStream_t st = c->stream;
  auto res = [&](int first) {
    me_ktimer t(c, ME_KT_SCALE_RES);
    // grid y: candidates of a batch (phase A / D use y = 0 only)
    hipLaunchKernelGGL(scale_res_ctrl_kernel, dim3(nb, first ? 1 : kSpecMax), dim3(kScBlock), 0, st, aR, P.td, P.res,
                       P.rows_pad, P.err, P.lm, P.spec, lp, first, P.bar);
  };
  auto neq = [&]() {
    me_ktimer t(c, ME_KT_SCALE_NEQ);
    hipLaunchKernelGGL(scale_neq_ctrl_kernel, dim3(nb), dim3(kScBlock), 0, st, aN, P.td, (const double*)P.res,
                       P.rows_pad, P.jj, P.je, P.err, P.lm, P.spec, lp, P.bar);
  };
  // The LM is enqueued in blocks [A,] B, R, B, R (one launch per LM phase, the
  // control fused into the last workgroup; R = a residual launch serving
  // phase C or D, whichever is current; an accepted candidate closes its
  // iteration in C's control, so a typical iteration is one B and one R);
  // every control update also lands in the coherent host mirror, an event
  // marks each block's end, and the host reads the mirror after block k's
  // event only once block k + 1 is queued (the GPU never drains while the
  // host polls; launches of a finished solve return at once).  The mirror
  // may already hold a later block's state: harmless, the solve only ever
  // moves towards PH_DONE and nothing is written after it.  (One
  // phase-agnostic kernel per launch, whatever phase is current, measured
  // slower: 610 vs 641 frames/s -- its merged register budget spills.)
  const long max_blocks = 64L * (p.max_nb_iter + 2);
  long blk = 0;
  auto mine = [&]() { return mir->gen == gen; };
  // Phase A is launched only in the first block: later iterations take their
  // residuals from the previous evaluation (same state, see ctrl_after_eval).
  // While the mirror shows a rejection streak (phase C: every retry is one
  // more R), the block is R, R, R, R.  Only the launch mix depends on this
  // (stale) read: every launch still runs the phase that is current.
  auto enqueue_block = [&](int sl) -> int {
    if (blk == 0) res(1);
    const bool retrying = blk > 0 && mine() && mir->phase == PH_C;
    retrying ? res(0) : neq();
    res(0);
    retrying ? res(0) : neq();
    res(0);
    ++blk;
    ME_TRY(me_check_launch(c, "scale optimise"));
    ME_HIP(c, hipEventRecord(c->poll_ev[sl], st));
    return ME_OK;
  };
  // Error exits after launches were queued drain the stream first, so no
  // launch of this solve is left to run behind the caller's next call.
  auto drain = [&](int rc) {
    (void)hipStreamSynchronize(st);
    return rc;
  };
  // Spin budget before the poll loop yields the core between polls: a solve
  // queued behind other work on the stream (e.g. a pipelined BA) would
  // otherwise burn a host core for that work's whole duration.
  constexpr int kSpinsBeforeYield = 4096;
  // The persistent launch: used while its grid takes at most half of what
  // fits on the ctx's CUs (the rest stays free for concurrent work, e.g. a
  // KLT on another stream); larger problems take the per-phase launches.  It
  // does not rely on the grid being co-resident (roster.hpp), so the choice is
  // a performance one only.
  if (c->scale_lm_cap < 0) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, scale_lm_kernel, kScBlock, 0) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess) {
      (void)hipGetLastError();
      per_cu = cus = 0;
    }
    if (c->cu_active > 0) cus = std::min(cus, c->cu_active);  // own stream restricted by me_set_cu_mask
    c->scale_lm_cap = per_cu * cus;
  }
  const bool persist = me_scale_persistent(nb, c->scale_lm_cap);
  if (persist) {
    lp.mirror_done_only = 1;
    // (test hook 8192: the roster closes at once, so the phases run on the
    // workgroups that joined by then -- the same results from fewer of them)
    lp.roster_ticks = (c->dbg_solve_flags & 8192) ? 0 : me_roster::kCloseTicks;
    {
      me_ktimer t(c, ME_KT_SCALE_RES);
      const int max_phases = 256 * (p.max_nb_iter + 2);
#ifdef ME_COOP_LAUNCH  // measurement build only (tools/gpu.sh coop): the same grid as a cooperative launch
      {
        const ScaleArgs* a0 = P.dargs;
        const ScaleArgs* a1 = P.dargs + 1;
        const TrackDev* td = P.dtd;
        double* rs = P.res;
        int rp = P.rows_pad;
        unsigned *cnt = P.bar, *ep = P.bar + kEpochWord, *ro = P.bar + kRosterWord;
        int mp = max_phases, nbv = nb;
        void* args[] = {&a0, &a1, &td, &rs, &rp, &P.jj, &P.je, &P.err, &P.lm, &P.spec, &lp, &cnt, &ep, &ro, &nbv, &mp};
        ME_HIP(c, hipLaunchCooperativeKernel((const void*)scale_lm_kernel, dim3(nb * kCandY), dim3(kScBlock), args, 0, st));
      }
#else
      hipLaunchKernelGGL(scale_lm_kernel, dim3(nb * kCandY), dim3(kScBlock), 0, st, P.dargs, P.dargs + 1, P.dtd,
                         P.res, P.rows_pad, P.jj, P.je, P.err, P.lm, P.spec, lp, P.bar, P.bar + kEpochWord,
                         P.bar + kRosterWord, nb, max_phases);
#endif
    }
    if (int rc = me_check_launch(c, "scale_lm_kernel")) return drain(rc);
    ME_HIP(c, hipEventRecord(c->poll_ev[0], st));
    // PH_DONE in the mirror (written once, by the final control) ends the
    // wait; the event covers a launch that ends without it (error / timeout)
    for (int spins = 0;; ++spins) {
      if (mine() && mir->phase == PH_DONE) break;
      const hipError_t q = hipEventQuery(c->poll_ev[0]);
      if (q == hipSuccess) break;
      if (q != hipErrorNotReady) return drain(me_set_error(c, ME_ERR_HIP, "scale optimise: %s", hipGetErrorString(q)));
      if (spins >= kSpinsBeforeYield) std::this_thread::yield();
    }
    if (!(mine() && mir->phase == PH_DONE)) {
      ME_HIP(c, hipMemcpyAsync(P.host + 32, P.err, 4, hipMemcpyDeviceToHost, st));
      ME_HIP(c, hipStreamSynchronize(st));
      int e;
      std::memcpy(&e, P.host + 32, 4);
      if (int rc = check_err(c, e)) return rc;
      return me_set_error(c, ME_ERR_STATE, "scale optimise did not terminate");
    }
  } else {
    if (int rc = enqueue_block(0)) return drain(rc);
    int cur = 0;
    for (;; cur ^= 1) {
      const bool more = blk < max_blocks;
      if (more)
        if (int rc = enqueue_block(cur ^ 1)) return drain(rc);
      // Spin on the mirror and the block's event (no sleeping wait: its wake-up
      // latency exceeded a block's ~60 us and idled the stream).  PH_DONE ends
      // the wait at once; the finished solve's queued launches return at once.
      bool done = false;
      for (int spins = 0;; ++spins) {
        if (mine() && mir->phase == PH_DONE) {
          done = true;
          break;
        }
        const hipError_t q = hipEventQuery(c->poll_ev[cur]);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady) return drain(me_set_error(c, ME_ERR_HIP, "scale optimise: %s", hipGetErrorString(q)));
        if (spins >= kSpinsBeforeYield) std::this_thread::yield();
      }
      if (done || (mine() && mir->phase == PH_DONE)) break;
      if (!more) return drain(me_set_error(c, ME_ERR_STATE, "scale optimise did not terminate"));
    }
  }
  std::atomic_thread_fence(std::memory_order_acquire);  // phase read before the rest of the header
  ScaleLM hs;
  std::memcpy(&hs, c->scale_mirror, kHeadBytes);
  if (hs.err) return check_err(c, hs.err);
  const int nt = std::min(std::min(hs.ntrace, kTraceCap), std::max(trace_cap, 0));
  if (trace && nt > 0) {  // stream-ordered: the solve's tail launches may still be queued
    ME_HIP(c, hipMemcpyAsync(trace, P.lm->trace, 16 * (size_t)nt, hipMemcpyDeviceToHost, c->stream));
    ME_HIP(c, hipStreamSynchronize(c->stream));
  }
  s->scale = hs.scale;
  if (stop_out) *stop_out = hs.stop;
  if (iterations) *iterations = hs.ntrace;
  if (mi_evals) *mi_evals = hs.nevals;
  c->scale_counters[0] = hs.nres;
  c->scale_counters[1] = hs.nneq;
  c->scale_counters[2] = hs.nrej;
  c->scale_counters[3] = hs.nexec;
  return ME_OK;
}

extern "C" int me_scale_last_counters(me_ctx* c, long* res_evals, long* neq_evals, long* rejections,
                                      long* executed) {
  if (!c) return ME_ERR_INVALID;
  if (res_evals) *res_evals = c->scale_counters[0];
  if (neq_evals) *neq_evals = c->scale_counters[1];
  if (rejections) *rejections = c->scale_counters[2];
  if (executed) *executed = c->scale_counters[3];
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

// ---------------------------------------------------------------------
// A7: ScaleState::compute_residuals (optimisation.cpp:230-278) -- one mutual
// information over the stacked 2w x 2w patch pairs of the left tracks
// (triangulated, seen in the last keyframe, both reprojections inside
// Rect(w, w, cols - 2w, rows - 2w)).  The reference stacks the pairs with
// `left_img(Range..) = imgs[i].first` (:273-274), which rebinds a temporary
// ROI header and copies nothing: its stacked images stay uninitialised
// cv::Mats (and their w x w slots could not hold the 2w x 2w patches anyway),
// so its result is undefined memory.  This restates the evident intent --
// the MI of the stacked patches, N = pairs * (2w)^2 pixels -- PARITY
// UNPINNED (checked against the oracle's literal stacking, oracle/scale.cpp).
// The stacking order does not matter: the histograms are integer counts.
namespace {
constexpr int kStateMiBlock = 256;
constexpr int kStateMiTracks = kStateMiBlock / 16;

__global__ __launch_bounds__(kStateMiBlock) void state_mi_hist_kernel(ScaleArgs a, TrackDev td,
                                                                      uint32_t* __restrict__ ghist,
                                                                      int* __restrict__ err) {
  __shared__ uint32_t hj[400];
  for (int i = threadIdx.x; i < 400; i += kStateMiBlock) hj[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 15;
  const int t = blockIdx.x * kStateMiTracks + (threadIdx.x >> 4);
  if (t < a.nL) {
    const uint8_t fl = td.flags[t];
    if ((fl & 8) && (fl & 2)) {  // isTriangulated() && getLastFrameIdx() == lframe (:246-248)
      const int w = a.w, P = 2 * w;
      Proj p;
      project_left(a, track_X(td, a, t), p);  // :250-256
      // bb = Rect(w, w, m_obs[0].first.cols - 2w, m_obs[1].first.rows - 2w) (:232)
      if (rect_contains(w, w, a.bb_cols - 2 * w, a.bb_rows - 2 * w, p.lx, p.ly) &&
          rect_contains(w, w, a.bb_cols - 2 * w, a.bb_rows - 2 * w, p.rx, p.ry)) {
        const int lx = roi_corner(p.lx, w), ly = roi_corner(p.ly, w), rx = roi_corner(p.rx, w),
                  ry = roi_corner(p.ry, w);
        if (!roi_in(a, lx, ly, P) || !roi_in(a, rx, ry, P)) {
          if (lane == 0) atomicOr(err, 1);
        } else {
          for (int k = lane; k < P * P; k += 16) {
            const int y = k / P, x = k - y * P;
            const int vl = a.imgL[(long)(ly + y) * a.stride + lx + x];
            const int vr = a.imgR[(long)(ry + y) * a.stride + rx + x];
            atomicAdd(&hj[bin20(vl) * 20 + bin20(vr)], 1u);
          }
          if (lane == 0) atomicAdd(&ghist[400], 1u);  // one more stacked pair
        }
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 400; i += kStateMiBlock)
    if (hj[i]) atomicAdd(&ghist[i], hj[i]);
}

// computeMutualInformation (mutual_information.cpp:55-86) on the stacked
// counts: marginals are the joint's row / column sums (every pixel lands in
// a bin), p = fl32(c * fl32(1/N)), terms in the i-outer / j-inner order.
__global__ __launch_bounds__(kStateMiBlock) void state_mi_final_kernel(const uint32_t* __restrict__ ghist, int P,
                                                                       double* __restrict__ out, int* __restrict__ err) {
  __shared__ uint32_t hl[20], hr[20];
  __shared__ float terms[400];
  const uint32_t npairs = ghist[400];
  if (threadIdx.x < 20) {
    uint32_t sl = 0, sr = 0;
    for (int k = 0; k < 20; ++k) {
      sl += ghist[threadIdx.x * 20 + k];
      sr += ghist[k * 20 + threadIdx.x];
    }
    hl[threadIdx.x] = sl;
    hr[threadIdx.x] = sr;
  }
  __syncthreads();
  const float invN = (float)(1.0 / (double)((long)npairs * P * P));
  for (int c = threadIdx.x; c < 400; c += kStateMiBlock) {
    const int i = c / 20, j = c - i * 20;
    const float pJ = (float)ghist[c] * invN, pL = (float)hl[i] * invN, pR = (float)hr[j] * invN;
    terms[c] = (pJ > 0 && pL > 0 && pR > 0) ? pJ * log2f_glibc(pJ / (pL * pR)) : 0.0f;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (npairs == 0) atomicOr(err, 4);  // empty stacked images: computeMutualInformation asserts (:57)
    float MI = 0.0f;
    for (int c = 0; c < 400; ++c)
      if (ghist[c]) MI += terms[c];
    out[0] = (double)MI;
    out[1] = (double)npairs;
  }
}
}  // namespace

extern "C" int me_scale_state_mi(me_ctx* c, const me_scale_state* s, double* mi_out, int* n_patches) {
  if (!c || !s || !mi_out) return ME_ERR_INVALID;
  ME_HIP(c, hipSetDevice(c->device));
  ScaleProblem P;
  ME_TRY(upload(c, s, 0, P));
  void* d;
  ME_TRY(me_scratch(c, SLOT_SC_RES, 401 * 4 + 256, &d));
  uint32_t* ghist = (uint32_t*)d;
  double* dout = (double*)((char*)d + 1664);
  ME_HIP(c, hipMemsetAsync(ghist, 0, 401 * 4, c->stream));
  const ScaleArgs a = P.a;
  if (a.nL > 0)
    hipLaunchKernelGGL(state_mi_hist_kernel, dim3((a.nL + kStateMiTracks - 1) / kStateMiTracks), dim3(kStateMiBlock),
                       0, c->stream, a, P.td, ghist, P.err);
  hipLaunchKernelGGL(state_mi_final_kernel, dim3(1), dim3(kStateMiBlock), 0, c->stream, (const uint32_t*)ghist,
                     2 * a.w, dout, P.err);
  ME_TRY(me_check_launch(c, "state_mi kernels"));
  ME_HIP(c, hipMemcpyAsync(P.host, dout, 16, hipMemcpyDeviceToHost, c->stream));
  ME_HIP(c, hipMemcpyAsync(P.host + 32, P.err, 4, hipMemcpyDeviceToHost, c->stream));
  ME_HIP(c, hipStreamSynchronize(c->stream));
  int e;
  std::memcpy(&e, P.host + 32, 4);
  if (e & 4) return me_set_error(c, ME_ERR_INVALID, "scale state MI: no stacked patch (computeMutualInformation "
                                                    "asserts on empty input, mutual_information.cpp:57)");
  ME_TRY(check_err(c, e));
  double o[2];
  std::memcpy(o, P.host, 16);
  *mi_out = o[0];
  if (n_patches) *n_patches = (int)o[1];
  return ME_OK;
}

#ifdef ME_SCALE_TS
extern "C" int me_scale_ts(long long* out, int reset) {
  hipDeviceSynchronize();
  hipMemcpyFromSymbol(out, HIP_SYMBOL(g_scale_ts), sizeof(g_scale_ts));
  if (reset) {
    unsigned long long z[16] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(g_scale_ts), z, sizeof(z));
  }
  return 0;
}
#endif
