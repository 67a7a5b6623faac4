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

// Row-major 8-bit grayscale view (cv::Mat CV_8U: data, rows, cols, step).
struct ImageView {
  const uint8_t* data = nullptr;
  int rows = 0, cols = 0;
  int step = 0;  // bytes per row
  bool empty() const { return !data || rows <= 0 || cols <= 0; }
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

  Status optimise(int fixedFrames) {
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
    int rc = me_ba_solve(ctx_->get(), &p, &opts_, &summary_);
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
