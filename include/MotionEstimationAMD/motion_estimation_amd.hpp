// motion_estimation_amd.hpp — C++ host mirror of the reference's hot-path API
// over the C ABI of libme_hip.so (include/me_hip.h).
//
// The reference's signatures take cv::Mat / Eigen / Ceres types; those
// libraries are absent from this build, so the mirror keeps the reference's
// names, argument meaning and status semantics with plain views:
//   me::computeMutualInformation  <- include/MotionEstimation/core/mutual_information.h:20
//   me::computeEntropy            <- src/core/mutual_information.cpp:28-45
//   me::nonMaxSupScanline3x3      <- include/MotionEstimation/core/feature_types.h:270
//   me::optimisation::BundleAdjuster<M> (StereoBundleAdjuster = <4>, MonoBundleAdjuster = <2>)
//                                 <- BundleAdjuster<M> (include/MotionEstimation/optimisation/BundleAdjuster.h:182-528)
//   me::optimisation::Optimiser<ScaleState, std::vector<std::pair<ImageView, ImageView>>>, ScaleState
//                                 <- include/MotionEstimation/optimisation/optimisation.h:20-125
//   me::StereoVisualOdometry      <- include/MotionEstimation/vo/StereoVisualOdometry.h:18-60
//   me::amd::flatten_scale_state  the reference-side glue of INTEGRATION.md §3 (templated on the
//                                 reference's own ScaleState / m_obs / mask types)
// Errors: the reference asserts on empty input (mutual_information.cpp:57);
// here invalid input throws std::invalid_argument, device/runtime failures
// throw std::runtime_error.  BundleAdjuster misuse reports through std::cerr
// and the returned Status, exactly like the reference (no exceptions).
#pragma once

#include <array>
#include <cstdint>
#include <iostream>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../me_hip.h"

namespace me {
namespace amd {

// One HIP device + stream + scratch (the ABI's me_ctx), one per host thread.
class Context {
 public:
  explicit Context(int device = 0) {
    me_ctx* c = nullptr;
    int rc = me_create(&c, device);
    if (rc != ME_OK) throw std::runtime_error("me_create failed (" + std::to_string(rc) + ")");
    c_.reset(c);
  }
  me_ctx* get() const { return c_.get(); }
  void check(int rc, const char* what) const {
    if (rc == ME_OK) return;
    std::string msg = std::string(what) + ": " + me_last_error(c_.get());
    if (rc == ME_ERR_INVALID) throw std::invalid_argument(msg);
    throw std::runtime_error(msg);
  }
  // CUs of the device, and a restriction of this ctx's stream to a CU set
  // (me_set_cu_mask; an empty set restores every CU)
  int cuCount() const {
    int n = 0;
    check(me_cu_count(c_.get(), &n), "me_cu_count");
    return n;
  }
  void setCuMask(const std::vector<int>& cus) {
    std::vector<uint32_t> w;
    for (int i : cus) {
      if ((int)w.size() <= i / 32) w.resize(i / 32 + 1, 0u);
      w[i / 32] |= 1u << (i % 32);
    }
    check(me_set_cu_mask(c_.get(), w.empty() ? nullptr : w.data(), (int)w.size()), "me_set_cu_mask");
  }
  static Context& thread_default() {
    thread_local Context ctx(0);
    return ctx;
  }

 private:
  struct Del {
    void operator()(me_ctx* c) const { me_destroy(c); }
  };
  std::unique_ptr<me_ctx, Del> c_;
};

// The landmark-sharded BA's communicator (me_comm): native RCCL
// over xGMI, one process per GPU.  Rank 0 draws unique_id() and hands the
// bytes to the other ranks; every rank constructs its Comm (collective).
class Comm {
 public:
  using Id = std::array<uint8_t, ME_COMM_ID_BYTES>;
  static Id unique_id() {
    Id id{};
    if (me_comm_unique_id(id.data(), (int)id.size()) != ME_OK) throw std::runtime_error("me_comm_unique_id failed");
    return id;
  }
  Comm(Context& ctx, int world, int rank, const Id& id) {
    me_comm* m = nullptr;
    ctx.check(me_comm_create_rccl(ctx.get(), world, rank, id.data(), &m), "me_comm_create_rccl");
    m_.reset(m);
  }
  me_comm* get() const { return m_.get(); }

 private:
  struct Del {
    void operator()(me_comm* m) const { me_comm_destroy(m); }
  };
  std::unique_ptr<me_comm, Del> m_;
};

// Row-major 8-bit grayscale view (cv::Mat CV_8U: data, rows, cols, step).
struct ImageView {
  const uint8_t* data = nullptr;
  int rows = 0, cols = 0;
  int step = 0;  // bytes per row
  bool empty() const { return !data || rows <= 0 || cols <= 0; }
  const uint8_t* ptr() const { return data; }  // cv::Mat::ptr()
};

}  // namespace amd

// float me::computeMutualInformation(const cv::Mat& L, const cv::Mat& R)
inline float computeMutualInformation(const amd::ImageView& L, const amd::ImageView& R,
                                      amd::Context& ctx = amd::Context::thread_default()) {
  if (L.empty() || R.empty()) throw std::invalid_argument("computeMutualInformation: empty patch");
  if (L.rows != R.rows || L.cols != R.cols) throw std::invalid_argument("computeMutualInformation: size mismatch");
  float out = 0.f;
  ctx.check(me_mutual_information(ctx.get(), ME_HOST, L.data, L.step, R.data, R.step, L.cols, L.rows, &out),
            "computeMutualInformation");
  return out;
}

// float computeEntropy(const cv::Mat& img)
inline float computeEntropy(const amd::ImageView& I, amd::Context& ctx = amd::Context::thread_default()) {
  if (I.empty()) throw std::invalid_argument("computeEntropy: empty patch");
  float out = 0.f;
  ctx.check(me_entropy(ctx.get(), ME_HOST, I.data, I.step, I.cols, I.rows, &out), "computeEntropy");
  return out;
}

// Batched form of computeMutualInformation over patch corners (the residual
// loop of Optimiser<ScaleState,...>::compute_residuals, optimisation.cpp:149-228).
inline std::vector<float> computeMutualInformation(const amd::ImageView& imgL, const amd::ImageView& imgR,
                                                   const std::vector<std::array<int32_t, 2>>& cornersL,
                                                   const std::vector<std::array<int32_t, 2>>& cornersR, int patch_w,
                                                   int patch_h, amd::Context& ctx = amd::Context::thread_default()) {
  if (cornersL.size() != cornersR.size()) throw std::invalid_argument("computeMutualInformation: corner lists differ");
  std::vector<float> out(cornersL.size());
  if (out.empty()) return out;
  ctx.check(me_mi_scores(ctx.get(), ME_HOST, imgL.data, imgL.step, imgR.data, imgR.step, imgL.cols, imgL.rows,
                         cornersL[0].data(), cornersR[0].data(), (int)out.size(), patch_w, patch_h, out.data()),
            "me_mi_scores");
  return out;
}

using pt2D = std::pair<double, double>;  // (row + 0.5 + dr, col + 0.5 + dc), feature_types.cpp:340-345

// std::vector<pt2D> nonMaxSupScanline3x3(const cv::Mat& input, cv::Mat& output)
inline std::vector<pt2D> nonMaxSupScanline3x3(const double* input, int rows, int cols, std::vector<uint8_t>& output,
                                              amd::Context& ctx = amd::Context::thread_default()) {
  output.assign((size_t)rows * cols, 0);
  const int cap = rows * cols / 2 + 1;
  std::vector<double> mx(2 * (size_t)cap);
  int n = 0;
  ctx.check(me_nms_scanline3x3(ctx.get(), ME_HOST, input, cols, rows, output.data(), mx.data(), cap, &n),
            "nonMaxSupScanline3x3");
  std::vector<pt2D> pts((size_t)std::min(n, cap));
  for (size_t k = 0; k < pts.size(); ++k) pts[k] = {mx[2 * k], mx[2 * k + 1]};
  return pts;
}

namespace optimisation {

// CalibrationParameters (BundleAdjuster.h:35-45); K row-major 3x3, K[0] left, K[1] right.
struct CalibrationParameters {
  std::vector<std::array<double, 9>> K;
  double feat_var = 0.0;
  double baseline = 0.0;
  bool compute_cov = false;
};

// Observation<M> (BundleAdjuster.h:22-32): M = 4 left (x, y), right (x, y);
// M = 2 one image (x, y) whose camID picks the residual of BundleAdjuster<2>.
template <int M>
struct Observation {
  std::array<double, M> xy;
  int camIdx;
  int ptIdx;
  int camID = 0;
};
using StereoObservation = Observation<4>;
using MonoObservation = Observation<2>;

// BundleAdjuster<M> over libme_hip.so.  Parameters: cameras {t, angle-axis}
// (Matx61d, :286-300), points {X, Y, Z}.  optimise() runs the device LM with
// the reference's Ceres options (function_tolerance 1e-3, Huber(1), point
// bounds, fixed leading frames), the 1 s time cap replaced by
// max_num_iterations (SURVEY A-9).  M = 4: StereoReprojectionError
// (:142-180, :431-476); M = 2: StandardReprojectionError / StereoRightError by
// camID, K[0] only, zero baseline -> 0.5 (:71-139, :378-429).  With
// compute_cov the pose covariances follow the solve (extract_covariance,
// :478-528; fixed cameras get zero blocks).
template <int M>
class BundleAdjuster {
  static_assert(M == 2 || M == 4, "BundleAdjuster<M>: M is 2 or 4");

 public:
  enum class Status { UNINITIALISED, INITIALISED, SUCCESSFUL, FAILED };

  BundleAdjuster(const CalibrationParameters& params, std::vector<std::array<double, 6>> cams,
                 std::vector<std::array<double, 3>> pts, std::vector<Observation<M>> obs,
                 amd::Context& ctx = amd::Context::thread_default())
      : calib_(params), cams_(std::move(cams)), pts_(std::move(pts)), obs_(std::move(obs)), ctx_(&ctx) {
    if (calib_.K.size() < (M == 4 ? 2u : 1u)) {  // StereoReprojectionError needs K[1] (BundleAdjuster.h:163)
      std::cerr << "[Bundle Adjuster] " << (M == 4 ? "stereo BA needs two calibration matrices"
                                                   : "BA needs a calibration matrix") << std::endl;
      return;
    }
    if (!cams_.empty() && !pts_.empty() && !obs_.empty()) status_ = Status::INITIALISED;
  }

  me_ba_options& options() { return opts_; }

  // comm: this rank holds all cameras and its landmark shard (ptIdx local to
  // the shard); the cameras come out identical on every rank.
  Status optimise(int fixedFrames, amd::Comm* comm = nullptr) {
    if (status_ == Status::UNINITIALISED) {
      std::cerr << "[Bundle Adjuster] parameters and observations must be initialised first" << std::endl;
      return status_;
    }
    if (M == 2 && calib_.baseline == 0) calib_.baseline = 0.5;  // BundleAdjuster.h:389-390
    std::vector<double> o(M * obs_.size());
    std::vector<int32_t> ci(obs_.size()), pi(obs_.size()), cid(obs_.size());
    for (size_t k = 0; k < obs_.size(); ++k) {
      for (int a = 0; a < M; ++a) o[M * k + a] = obs_[k].xy[a];
      ci[k] = obs_[k].camIdx;
      pi[k] = obs_[k].ptIdx;
      cid[k] = obs_[k].camID;
    }
    me_ba_problem p{};
    p.n_cams = (int)cams_.size();
    p.n_pts = (int)pts_.size();
    p.n_obs = (int)obs_.size();
    p.cams = cams_[0].data();
    p.pts = pts_[0].data();
    p.obs = o.data();
    p.cam_idx = ci.data();
    p.pt_idx = pi.data();
    p.obs_dim = M;
    p.cam_id = cid.data();
    for (int a = 0; a < 9; ++a) {
      p.K0[a] = calib_.K[0][a];
      p.K1[a] = calib_.K[calib_.K.size() > 1 ? 1 : 0][a];
    }
    p.baseline = calib_.baseline;
    p.feat_var = calib_.feat_var;
    p.fixed_frames = fixedFrames;
    int rc = comm ? me_ba_solve_comm(ctx_->get(), &p, &opts_, comm->get(), &summary_)
                  : me_ba_solve(ctx_->get(), &p, &opts_, &summary_);
    if (rc != ME_OK) {
      std::cerr << "[Bundle Adjuster] " << me_last_error(ctx_->get()) << std::endl;
      return status_ = Status::FAILED;
    }
    if (calib_.compute_cov) {
      std::vector<double> cov(36 * cams_.size());
      int ok = 0;
      rc = me_ba_covariance(ctx_->get(), &p, cov.data(), &ok);
      if (rc != ME_OK || !ok) {
        std::cerr << "[Bundle Adjuster] error computing the covariance matrix" << std::endl;
      } else {
        covs_.assign(cams_.size(), {});
        for (size_t i = 0; i < cams_.size(); ++i) std::copy(&cov[36 * i], &cov[36 * i] + 36, covs_[i].begin());
      }
    }
    return status_ = (summary_.status == 2 ? Status::SUCCESSFUL : Status::FAILED);
  }

  const std::vector<std::array<double, 3>>& getPoints() const { return pts_; }
  const std::vector<std::array<double, 6>>& getCameraParams() const { return cams_; }
  // 6x6 row-major per camera (empty unless compute_cov and the covariance succeeded)
  const std::vector<std::array<double, 36>>& getPosesCovariance() const { return covs_; }
  int getNbPoints() const { return (int)pts_.size(); }
  int getNbCameras() const { return (int)cams_.size(); }
  int getNbObservations() const { return (int)obs_.size(); }
  Status getStatus() const { return status_; }
  const me_ba_summary& summary() const { return summary_; }

 private:
  static me_ba_options defaults() {
    me_ba_options o;
    me_ba_default_options(&o);
    return o;
  }
  CalibrationParameters calib_;
  std::vector<std::array<double, 6>> cams_;
  std::vector<std::array<double, 3>> pts_;
  std::vector<Observation<M>> obs_;
  std::vector<std::array<double, 36>> covs_;
  amd::Context* ctx_;
  Status status_ = Status::UNINITIALISED;
  me_ba_options opts_ = defaults();
  me_ba_summary summary_{};
};
using StereoBundleAdjuster = BundleAdjuster<4>;
using MonoBundleAdjuster = BundleAdjuster<2>;

}  // namespace optimisation
}  // namespace me

// ===========================================================================
// ScaleState optimiser (A4-A9), the stacked state MI (A7), StereoVO (A19),
// KLT (A12).
// ===========================================================================
namespace me {
namespace amd {

// Host arrays behind a flattened me_scale_state (kept alive by the caller
// for as long as the struct is used).
struct ScaleStateBuffers {
  std::vector<double> XL, XR;
  std::vector<uint8_t> triL, triR, mask;
  std::vector<uint32_t> lastL, lastR;
};

namespace detail {
template <class M>
inline int row_stride(const M& m) {
  return static_cast<int>(static_cast<size_t>(m.step));  // cv::Mat::step (MStep -> size_t) or ImageView::step
}
template <class Track>
inline void flatten_tracks(const std::vector<Track>& v, std::vector<double>& X, std::vector<uint8_t>& tri,
                           std::vector<uint32_t>& last) {
  X.resize(4 * v.size());
  tri.resize(v.size());
  last.resize(v.size());
  for (size_t i = 0; i < v.size(); ++i) {
    const auto pt = v[i].get3DLocation();  // ptH3D (cv::Matx41d)
    for (int k = 0; k < 4; ++k) X[4 * i + k] = pt(k);
    tri[i] = v[i].isTriangulated() ? 1 : 0;
    last[i] = v[i].getLastFrameIdx();
  }
}
template <class Pose>
inline void flatten_pose(const Pose& p, double q[4], double t[3]) {
  q[0] = p.orientation.w();
  q[1] = p.orientation.x();
  q[2] = p.orientation.y();
  q[3] = p.orientation.z();
  for (int k = 0; k < 3; ++k) t[k] = p.position[k];
}
}  // namespace detail

// The flattening step of the reference-side binding: a
// ScaleState (optimisation.h:76-98) + its observations m_obs
// (vector<pair<cv::Mat, cv::Mat>>) + the optional mask (Eigen::VectorXi) ->
// me_scale_state.  Templated on the reference's own types; it uses only the
// members they have:
//   state.pts.{first,second}[i].get3DLocation()(k) / .isTriangulated() / .getLastFrameIdx()
//     (WBA_Ptf, feature_types.h:121-197)
//   state.poses.{first,second}: [0].ID, .size(), .back().orientation.w()..z(), .back().position[k]
//     (CamPose_qd, feature_types.h:202-230; Quat::w() etc., rotation_utils.h:183-186)
//   state.K.{first,second}(r, c) (cv::Matx33d), state.scale, state.baseline, state.window_size
//   obs[f].first / .second: .ptr(), .step, .cols, .rows (cv::Mat, CV_8U)
//   mask.size(), mask(i) (Eigen::VectorXi)
// The frame is m_obs[poses.first.size() - 1] (optimisation.cpp:174), the
// residual bounds use m_obs[0].first.cols and m_obs[1].first.rows (:155), and
// lframe = poses.first[0].ID + poses.first.size() - 1 (:165).
template <class State, class Obs, class Mask>
inline void flatten_scale_state(const State& st, const Obs& obs, const Mask& mask, me_scale_state* s,
                                ScaleStateBuffers& buf) {
  if (st.poses.first.empty() || st.poses.second.empty())
    throw std::invalid_argument("flatten_scale_state: empty pose window");
  const size_t f = st.poses.first.size() - 1;
  if (obs.size() < 2 || obs.size() <= f)
    throw std::invalid_argument("flatten_scale_state: m_obs must hold the window's image pairs (>= 2)");
  *s = me_scale_state{};
  detail::flatten_tracks(st.pts.first, buf.XL, buf.triL, buf.lastL);
  detail::flatten_tracks(st.pts.second, buf.XR, buf.triR, buf.lastR);
  s->n_left = (int)st.pts.first.size();
  s->n_right = (int)st.pts.second.size();
  s->X_left = buf.XL.data();
  s->X_right = buf.XR.data();
  s->tri_left = buf.triL.data();
  s->tri_right = buf.triR.data();
  s->last_left = buf.lastL.data();
  s->last_right = buf.lastR.data();
  s->lframe = (uint32_t)(st.poses.first[0].ID + st.poses.first.size() - 1);
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      s->K1[3 * r + c] = st.K.first(r, c);
      s->K2[3 * r + c] = st.K.second(r, c);
    }
  detail::flatten_pose(st.poses.first.back(), s->q1, s->t1);
  detail::flatten_pose(st.poses.second.back(), s->q2, s->t2);
  s->scale = st.scale;
  s->baseline = st.baseline;
  s->window_size = st.window_size;
  const auto& L = obs[f].first;
  const auto& R = obs[f].second;
  if (L.rows != R.rows || L.cols != R.cols || detail::row_stride(L) != detail::row_stride(R))
    throw std::invalid_argument("flatten_scale_state: left / right images differ in shape or stride");
  s->imgL = static_cast<const uint8_t*>(L.ptr());
  s->imgR = static_cast<const uint8_t*>(R.ptr());
  s->stride = detail::row_stride(L);
  s->cols = L.cols;
  s->rows = L.rows;
  s->bb_cols = obs[0].first.cols;
  s->bb_rows = obs[1].first.rows;
  buf.mask.resize((size_t)mask.size());
  for (int i = 0; i < (int)mask.size(); ++i) buf.mask[i] = mask(i) ? 1 : 0;
  s->mask = buf.mask.empty() ? nullptr : buf.mask.data();
  s->mask_len = (int)buf.mask.size();
  s->img_mem = ME_HOST;
  s->tracks_mem = ME_HOST;
}

}  // namespace amd

// ---- reference-shaped value types (plain, no OpenCV / Eigen) -------------
using ptH3D = std::array<double, 4>;  // cv::Matx41d: pt(k) is pt[k] here
struct Point2f {
  float x = 0.f, y = 0.f;
};
template <class T>
struct StereoOdoMatches {  // feature_types.h:101-109 (f1, f2 previous L/R, f3, f4 current L/R)
  T f1, f2, f3, f4;
  float m_score = -1.f;
};
using StereoOdoMatchesf = StereoOdoMatches<Point2f>;
enum StopCondition { NO_STOP, SMALL_GRADIENT, SMALL_INCREMENT, MAX_ITERATIONS, SMALL_DECREASE_FUNCTION,
                     SMALL_REPROJ_ERROR, NO_CONVERGENCE };  // rotation_utils.h:20

// Quat / CamPose_qd / WBA_Ptf reduced to the members the scale optimiser reads.
struct Quat {
  double m_w = 1, m_x = 0, m_y = 0, m_z = 0;
  double w() const { return m_w; }
  double x() const { return m_x; }
  double y() const { return m_y; }
  double z() const { return m_z; }
};
struct CamPose_qd {
  int ID = 0;
  Quat orientation;
  std::array<double, 3> position{{0, 0, 0}};
};
struct Matx33d {
  std::array<double, 9> val{{1, 0, 0, 0, 1, 0, 0, 0, 1}};
  double operator()(int r, int c) const { return val[3 * r + c]; }
};
struct WBA_Ptf {  // the 3-D location and the frame bookkeeping of WBA_Point<Point2f>
  struct Loc {
    ptH3D v{{0, 0, 0, 1}};
    double operator()(int k) const { return v[k]; }
  } pt;
  unsigned last_frame = (unsigned)-1;
  bool isTriangulated() const { return !(pt.v[0] == 0 && pt.v[1] == 0 && pt.v[2] == 0 && pt.v[3] == 1); }
  unsigned getLastFrameIdx() const { return last_frame; }
  Loc get3DLocation() const { return pt; }
};
struct VectorXi {  // Eigen::VectorXi
  std::vector<int> v;
  int size() const { return (int)v.size(); }
  int operator()(int i) const { return v[i]; }
};

namespace optimisation {

enum class OptimType { GN, LM };

// OptimisationParams (optimisation.h:22-32), same defaults
struct OptimisationParams {
  int MAX_NB_ITER;
  double v, tau, mu;
  double abs_tol, grad_tol, incr_tol, rel_tol;
  double alpha;
  OptimType type;
  bool minim;
  bool weighting;
  OptimisationParams(OptimType type_ = OptimType::LM, bool min = true, int it = 20, double v_ = 2, double t = 1e-3,
                     double m = 1e-20, double e1 = 1e-4, double e2 = 1e-4, double e3 = 1e-3, double e4 = 1e-4,
                     double a = 1.0)
      : MAX_NB_ITER(it), v(v_), tau(t), mu(m), abs_tol(e1), grad_tol(e2), incr_tol(e3), rel_tol(e4), alpha(a),
        type(type_), minim(min), weighting(false) {}
  me_optim_params to_c() const {
    me_optim_params p;
    me_optim_default_params(&p);
    p.type = (int)type;
    p.minim = minim;
    p.max_nb_iter = MAX_NB_ITER;
    p.v = v;
    p.tau = tau;
    p.mu = mu;
    p.abs_tol = abs_tol;
    p.grad_tol = grad_tol;
    p.incr_tol = incr_tol;
    p.rel_tol = rel_tol;
    p.alpha = alpha;
    p.weighting = weighting;
    return p;
  }
};

using ImagePairs = std::vector<std::pair<amd::ImageView, amd::ImageView>>;

// ScaleState (optimisation.h:76-98)
struct ScaleState {
  std::pair<std::vector<WBA_Ptf>, std::vector<WBA_Ptf>> pts;
  std::pair<Matx33d, Matx33d> K;
  std::pair<std::vector<CamPose_qd>, std::vector<CamPose_qd>> poses;
  double scale = 1.0;
  double baseline = 0.0;
  int window_size = 0;
  int nb_params = 1;
  // double ScaleState::compute_residuals(std::vector<std::pair<cv::Mat,cv::Mat>>&) (optimisation.cpp:230-278):
  // the MI of the stacked 2w x 2w pairs (evident intent; see me_scale_state_mi in me_hip.h)
  double compute_residuals(const ImagePairs& m_obs,
                           amd::Context& ctx = amd::Context::thread_default()) const {
    amd::ScaleStateBuffers buf;
    me_scale_state s;
    amd::flatten_scale_state(*this, m_obs, VectorXi{}, &s, buf);
    double mi = 0;
    ctx.check(me_scale_state_mi(ctx.get(), &s, &mi, nullptr), "ScaleState::compute_residuals");
    return mi;
  }
  void update(double dX) { scale += dX; }  // optimisation.h:90-93
};

template <class S, class T>
class Optimiser;

// Optimiser<ScaleState, vector<pair<Mat,Mat>>> (optimisation.h:100-125,
// optimisation.cpp:29-228,435-747) over me_scale_*: the same public
// members; MatrixXd results are std::vector<double> (residual column) and a
// double (the 1x1 Jacobian product).  Device errors throw (the reference
// would throw cv::Exception on an out-of-image ROI).
template <>
class Optimiser<ScaleState, ImagePairs> {
 public:
  Optimiser(const ImagePairs& observations, const OptimisationParams& params = OptimisationParams(),
            amd::Context& ctx = amd::Context::thread_default())
      : m_obs(observations), m_params(params), m_ctx(&ctx) {}

  StopCondition optimise(ScaleState& state, const bool test = false, const VectorXi& mask = VectorXi()) {
    m_state = state;
    m_mask = mask;
    amd::ScaleStateBuffers buf;
    me_scale_state s;
    amd::flatten_scale_state(m_state, m_obs, m_mask, &s, buf);
    const me_optim_params p = m_params.to_c();
    int stop = 0, iters = 0;
    long evals = 0;
    m_ctx->check(me_scale_optimise(m_ctx->get(), &s, &p, test ? 1 : 0, &stop, &iters, nullptr, 0, &evals),
                 "Optimiser::optimise");
    m_state.scale = s.scale;
    m_iterations = iters;
    m_stop = static_cast<StopCondition>(stop);
    state = m_state;
    return m_stop;
  }
  std::vector<double> compute_residuals(const ScaleState& state) {
    amd::ScaleStateBuffers buf;
    me_scale_state s;
    amd::flatten_scale_state(state, m_obs, m_mask, &s, buf);
    std::vector<double> res((size_t)(s.n_left + s.n_right) + 1);
    int rows = 0;
    m_ctx->check(me_scale_residuals(m_ctx->get(), &s, m_params.weighting, res.data(), &rows),
                 "Optimiser::compute_residuals");
    res.resize((size_t)rows);
    return res;
  }
  std::vector<int> compute_inliers(const double threshold) {
    amd::ScaleStateBuffers buf;
    me_scale_state s;
    amd::flatten_scale_state(m_state, m_obs, VectorXi{}, &s, buf);  // the mask is cleared (:735-736)
    std::vector<int> idx((size_t)(s.n_left + s.n_right) + 1);
    int n = 0;
    m_ctx->check(me_scale_inliers(m_ctx->get(), &s, m_params.weighting, threshold, idx.data(), (int)idx.size(), &n),
                 "Optimiser::compute_inliers");
    idx.resize((size_t)std::min<int>(n, (int)idx.size()));
    return idx;
  }
  double getJacobian() {
    amd::ScaleStateBuffers buf;
    me_scale_state s;
    amd::flatten_scale_state(m_state, m_obs, m_mask, &s, buf);
    double JJ = 0;
    m_ctx->check(me_scale_jacobian(m_ctx->get(), &s, m_params.weighting, &JJ), "Optimiser::getJacobian");
    return JJ;
  }
  int iterations() const { return m_iterations; }

 private:
  ScaleState m_state;
  ImagePairs m_obs;
  VectorXi m_mask;
  OptimisationParams m_params;
  StopCondition m_stop = NO_STOP;
  amd::Context* m_ctx;
  int m_iterations = 0;
};

}  // namespace optimisation

// StereoVisualOdometry (StereoVisualOdometry.h:18-60, StereoVisualOdometry.cpp:34-342)
// over me_vo_process.  cv::Mat results are row-major arrays: getMotion() 4x4,
// getPts3D() homogeneous points, the state six values (Euler angles,
// translation).  The RANSAC triples come from the context's glibc rand()
// stream (srand() reseeds it, as the reference's unseeded rand()).
class StereoVisualOdometry {
 public:
  enum class Method { GN, LM };
  struct parameters {  // VisualOdometry::parameters (VisualOdometry.h:19-33) + Stereo (:24-33), same defaults
    Method method;
    double step_size, eps, e1, e2, e3, e4;
    int max_iter, nb_fixed_frames;
    bool ransac;
    int n_ransac;
    double inlier_threshold;
    double baseline;
    bool weighting;
    double fu1, fv1, fu2, fv2, cu1, cu2, cv1, cv2;
    parameters()
        : method(Method::GN), step_size(1.0), eps(1e-9), e1(1e-3), e2(1e-12), e3(1e-12), e4(1e-15), max_iter(100),
          nb_fixed_frames(2), ransac(true), n_ransac(200), inlier_threshold(2.0), baseline(1.0), weighting(false),
          fu1(1.0), fv1(1.0), fu2(1.0), fv2(1.0), cu1(0.0), cu2(0.0), cv1(0.0), cv2(0.0) {}
  };
  explicit StereoVisualOdometry(parameters param = parameters(), amd::Context& ctx = amd::Context::thread_default(),
                                int max_outer = 10000)
      : m_param(param), m_ctx(&ctx), m_max_outer(max_outer) {}

  void srand(unsigned seed) { m_ctx->check(me_vo_srand(m_ctx->get(), seed), "srand"); }

  // bool process(const std::vector<StereoOdoMatchesf>&, cv::Mat init = zeros(6,1))
  bool process(const std::vector<StereoOdoMatchesf>& matches, const std::array<double, 6>& init = {}) {
    if (matches.size() < 6) return false;  // StereoVisualOdometry.cpp:40-42
    const int n = (int)matches.size();
    std::vector<float> m(8 * (size_t)n);
    for (int i = 0; i < n; ++i) {
      const StereoOdoMatchesf& q = matches[i];
      const float v[8] = {q.f1.x, q.f1.y, q.f2.x, q.f2.y, q.f3.x, q.f3.y, q.f4.x, q.f4.y};
      std::copy(v, v + 8, &m[8 * (size_t)i]);
    }
    me_vo_params p;
    me_vo_default_params(&p);
    p.method = (int)m_param.method;
    p.step_size = m_param.step_size;
    p.eps = m_param.eps;
    p.e1 = m_param.e1;
    p.e2 = m_param.e2;
    p.e3 = m_param.e3;
    p.e4 = m_param.e4;
    p.max_iter = m_param.max_iter;
    p.nb_fixed_frames = m_param.nb_fixed_frames;
    p.ransac = m_param.ransac;
    p.n_ransac = m_param.n_ransac;
    p.inlier_threshold = m_param.inlier_threshold;
    p.baseline = m_param.baseline;
    p.weighting = m_param.weighting;
    p.fu1 = m_param.fu1;
    p.fv1 = m_param.fv1;
    p.fu2 = m_param.fu2;
    p.fv2 = m_param.fv2;
    p.cu1 = m_param.cu1;
    p.cu2 = m_param.cu2;
    p.cv1 = m_param.cv1;
    p.cv2 = m_param.cv2;
    m_pts3D.assign((size_t)n, ptH3D{{0, 0, 0, 0}});
    m_inliers.assign((size_t)n, 0);
    int nin = 0, ok = 0;
    m_ctx->check(me_vo_process(m_ctx->get(), m.data(), n, init.data(), &p, m_max_outer, m_motion.data(),
                               m_state.data(), m_pts3D[0].data(), m_inliers.data(), &nin, &ok),
                 "StereoVisualOdometry::process");
    m_inliers.resize((size_t)nin);
    return ok != 0;
  }
  const std::array<double, 16>& getMotion() const { return m_motion; }
  const std::array<double, 6>& getState() const { return m_state; }
  const std::vector<ptH3D>& getPts3D() const { return m_pts3D; }
  const std::vector<int>& getInliers_idx() const { return m_inliers; }
  parameters getParams() const { return m_param; }

 private:
  parameters m_param;
  amd::Context* m_ctx;
  int m_max_outer;
  std::array<double, 16> m_motion{};
  std::array<double, 6> m_state{};
  std::vector<ptH3D> m_pts3D;
  std::vector<int> m_inliers;
};

// me::MonoVisualOdometry (include/MotionEstimation/vo/MonoVisualOdometry.h:18-57,
// src/vo/MonoVisualOdometry.cpp:7-73): findEssentialMat + recoverPose on the
// device (me_mono_vo_process).  Matches are StereoMatch<Point2f> {f1, f2}.
template <class T>
struct StereoMatch {
  T f1, f2;
  float m_score = -1.0f;
};
class MonoVisualOdometry {
 public:
  struct parameters {  // MonoVisualOdometry::parameters (MonoVisualOdometry.h:21-28) + the fields of the base it reads
    bool ransac;
    double inlier_threshold;
    double prob;
    double fu, fv, cu, cv;
    parameters() : ransac(true), inlier_threshold(2.0), prob(0.99), fu(1.0), fv(1.0), cu(0.0), cv(0.0) {}
  };
  explicit MonoVisualOdometry(const parameters& param = parameters(),
                              amd::Context& ctx = amd::Context::thread_default())
      : m_param(param), m_ctx(&ctx) {
    for (int i = 0; i < 16; ++i) m_Rt[i] = (i % 5 == 0) ? 1.0 : 0.0;
  }
  bool process(const std::vector<StereoMatch<Point2f>>& matches) {
    const int n = (int)matches.size();
    std::vector<float> f1(2 * (size_t)n), f2(2 * (size_t)n);
    for (int i = 0; i < n; ++i) {
      f1[2 * i] = matches[i].f1.x;
      f1[2 * i + 1] = matches[i].f1.y;
      f2[2 * i] = matches[i].f2.x;
      f2[2 * i + 1] = matches[i].f2.y;
    }
    me_mono_params p;
    me_mono_default_params(&p);
    p.fu = m_param.fu;
    p.fv = m_param.fv;
    p.cu = m_param.cu;
    p.cv = m_param.cv;
    p.prob = m_param.prob;
    p.inlier_threshold = m_param.inlier_threshold;
    p.ransac = m_param.ransac ? 1 : 0;
    std::vector<int32_t> inl((size_t)std::max(n, 1));
    std::array<double, 9> E{};
    int ni = 0, ok = 0;
    m_ctx->check(me_mono_vo_process(m_ctx->get(), f1.data(), f2.data(), n, &p, m_Rt.data(), E.data(), inl.data(),
                                    &ni, &ok),
                 "MonoVisualOdometry::process");
    // MonoVisualOdometry.cpp:9-52: fewer than 8 matches leaves m_E and the
    // inlier / outlier lists as they were; an empty E is assigned (empty) and
    // the lists are kept; otherwise all three are replaced
    if (n < 8) return ok != 0;
    bool any = false;
    for (double v : E) any = any || v != 0.0;
    m_E = E;
    m_E_empty = !any;
    if (!any) return ok != 0;
    m_inliers.assign(inl.begin(), inl.begin() + ni);
    m_outliers.clear();
    for (int i = 0, k = 0; i < n; ++i) {
      if (k < ni && inl[k] == i) ++k;
      else m_outliers.push_back(i);
    }
    return ok != 0;
  }
  const std::array<double, 16>& getMotion() const { return m_Rt; }
  // the reference's m_E as a 3 x 3 array; essentialMatEmpty() is its m_E.empty()
  const std::array<double, 9>& getEssentialMat() const { return m_E; }
  bool essentialMatEmpty() const { return m_E_empty; }
  const std::vector<int>& getInliersIdx() const { return m_inliers; }
  const std::vector<int>& getOutliersIdx() const { return m_outliers; }

 private:
  parameters m_param;
  amd::Context* m_ctx;
  std::array<double, 16> m_Rt{};
  std::array<double, 9> m_E{};
  bool m_E_empty = false;  // (the reference ctor sets m_E = eye(4, 4): not empty)
  std::vector<int> m_inliers, m_outliers;
};

// Pyramidal LK tracking of n points from prev to next (A12, no reference
// counterpart: the application's feature tracker).  status[i] = 1 tracked.
inline void calcOpticalFlowPyrLK(const amd::ImageView& prev, const amd::ImageView& next,
                                 const std::vector<Point2f>& pts_in, std::vector<Point2f>& pts_out,
                                 std::vector<uint8_t>& status, amd::Context& ctx = amd::Context::thread_default()) {
  if (prev.rows != next.rows || prev.cols != next.cols || prev.step != next.step)
    throw std::invalid_argument("calcOpticalFlowPyrLK: images differ in shape");
  pts_out.resize(pts_in.size());
  status.assign(pts_in.size(), 0);
  if (pts_in.empty()) return;
  me_klt_params kp;
  me_klt_default_params(&kp);
  ctx.check(me_klt_track(ctx.get(), ME_HOST, prev.data, next.data, prev.cols, prev.rows, prev.step,
                         &pts_in[0].x, &pts_out[0].x, status.data(), (int)pts_in.size(), &kp),
            "calcOpticalFlowPyrLK");
}

// The windowed stereo VO loop (me_vo_loop_*, csrc/vo_loop.hip): the
// application loop the reference leaves to its caller -- per keyframe KLT,
// epipolar MI matching, WBA_Point bookkeeping (feature_types.h:121-197),
// scale LM (Optimiser<ScaleState,...>) and the sliding-window
// BundleAdjuster<4> -- in native code, the same decisions as
// uasl_motion_estimation_amd.pipeline.WindowedStereoVO.  Two contexts of one
// GPU: `ba` runs the window solves, `front` the front end; with
// frontCus in (0, 16) the two streams get whole XCDs (frontCus / 2 of the 8
// XCDs to the front end: CU i sits on XCD i mod 8).  `ba` and `front` may be
// the same context (one stream, no worker threads).
class WindowedStereoVO {
 public:
  struct Config : me_vo_loop_config {
    Config() { me_vo_loop_default_config(this); }
  };
  WindowedStereoVO(amd::Context& ba, amd::Context& front, const Config& cfg, int frontCus = 4)
      : ba_(ba), front_(front), width_(cfg.width), height_(cfg.height) {
    if (&ba != &front && frontCus > 0 && frontCus < 16) {
      const int ncu = ba.cuCount();
      std::vector<int> f, b;
      for (int i = 0; i < ncu; ++i) (i % 8 < frontCus / 2 ? f : b).push_back(i);
      front.setCuMask(f);
      ba.setCuMask(b);
      masked_ = true;
    }
    me_vo_loop* v = nullptr;
    try {
      ba.check(me_vo_loop_create(ba.get(), front.get(), &cfg, &v), "me_vo_loop_create");
    } catch (...) {  // no destructor runs: give the caller's contexts their CUs back
      if (masked_) {
        front.setCuMask({});
        ba.setCuMask({});
      }
      throw;
    }
    v_.reset(v);
  }
  ~WindowedStereoVO() {
    v_.reset();
    if (masked_) {
      front_.setCuMask({});
      ba_.setCuMask({});
    }
  }
  WindowedStereoVO(const WindowedStereoVO&) = delete;
  WindowedStereoVO& operator=(const WindowedStereoVO&) = delete;
  // keyframe t (0, 1, 2, ...): host images of the configured size, copied in
  void process(int t, const amd::ImageView& left, const amd::ImageView& right) {
    if (left.empty() || right.empty() || left.step != left.cols || right.step != right.cols)
      throw std::invalid_argument("WindowedStereoVO::process: dense 8-bit images expected");
    if (left.rows != height_ || left.cols != width_ || right.rows != height_ || right.cols != width_)
      throw std::invalid_argument("WindowedStereoVO::process: images of the configured width x height expected");
    check(me_vo_loop_process(v_.get(), t, left.data, right.data, ME_HOST), "WindowedStereoVO::process");
  }
  // keyframe t from device memory: dense width x height bytes each, written
  // before the call in stream order with the loop (or synchronised by the
  // caller), alive until process(t + 1) returns
  void processDevice(int t, const uint8_t* left, const uint8_t* right) {
    if (!left || !right) throw std::invalid_argument("WindowedStereoVO::processDevice: null image");
    check(me_vo_loop_process(v_.get(), t, left, right, ME_DEVICE), "WindowedStereoVO::processDevice");
  }
  void finish() { check(me_vo_loop_finish(v_.get()), "WindowedStereoVO::finish"); }
  std::vector<me_vo_frame_result> results() const {
    int n = 0;
    check(me_vo_loop_results(v_.get(), nullptr, 0, &n), "results");
    std::vector<me_vo_frame_result> r((size_t)n);
    check(me_vo_loop_results(v_.get(), r.data(), n, &n), "results");
    return r;
  }
  std::vector<me_vo_event> events() const {
    long n = 0;
    check(me_vo_loop_events(v_.get(), nullptr, 0, &n), "events");
    std::vector<me_vo_event> e((size_t)n);
    check(me_vo_loop_events(v_.get(), e.data(), n, &n), "events");
    return e;
  }
  std::vector<std::pair<int, std::array<double, 6>>> poses() const {
    int n = 0;
    check(me_vo_loop_poses(v_.get(), nullptr, nullptr, 0, &n), "poses");
    std::vector<int32_t> ts((size_t)n);
    std::vector<std::array<double, 6>> p((size_t)n);
    check(me_vo_loop_poses(v_.get(), ts.data(), n ? p[0].data() : nullptr, n, &n), "poses");
    std::vector<std::pair<int, std::array<double, 6>>> out;
    for (int i = 0; i < n; ++i) out.emplace_back(ts[i], p[i]);
    return out;
  }
  // live tracks: IDs (WBA_Point::getID) and landmarks (get3DLocation)
  void tracks(std::vector<int64_t>& ids, std::vector<std::array<double, 3>>& X) const {
    int n = 0;
    check(me_vo_loop_tracks(v_.get(), nullptr, nullptr, nullptr, nullptr, nullptr, 0, &n), "tracks");
    ids.resize((size_t)n);
    X.resize((size_t)n);
    check(me_vo_loop_tracks(v_.get(), ids.data(), n ? X[0].data() : nullptr, nullptr, nullptr, nullptr, n, &n),
          "tracks");
  }

 private:
  void check(int rc, const char* what) const {
    if (rc == ME_OK) return;
    std::string msg = std::string(what) + ": " + me_vo_loop_last_error(v_.get());
    if (rc == ME_ERR_INVALID) throw std::invalid_argument(msg);
    throw std::runtime_error(msg);
  }
  struct Del {
    void operator()(me_vo_loop* v) const { me_vo_loop_destroy(v); }
  };
  amd::Context& ba_;
  amd::Context& front_;
  int width_, height_;
  bool masked_ = false;
  std::unique_ptr<me_vo_loop, Del> v_;
};

}  // namespace me
