/* oracle.h — CPU restatement of the uasl_motion_estimation hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load liboracle.so, and only as the checker
 * (or the timed CPU baseline).  The product (libme_hip.so) never links it.
 *
 * PARITY UNPINNED: the reference (abeauvisage/uasl_motion_estimation) needs
 * OpenCV 4 + Eigen3 + Ceres, none of which exist in this image, and it ships no
 * tests, fixtures or golden vectors.  This file restates the reference's
 * algorithms from its sources (file:line cited per function) and restates the
 * third-party semantics it depends on (OpenCV calcHist / Mat scaling / Rect,
 * glibc log2f, Ceres LM + Huber + Jacobi scaling) from their documented
 * behaviour.  Golden vectors in tests/golden/ are produced by this oracle
 * (tests/golden/make_golden.py) and by hand-derivable known-answer tests.
 *
 * Every function is plain C ABI so Python tests can bind it with ctypes.
 */
#ifndef ME_ORACLE_H
#define ME_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* ---- A1/A2: mutual information (src/core/mutual_information.cpp:28-86) ---- */
float oracle_mutual_information(const uint8_t* L, int strideL, const uint8_t* R, int strideR, int w, int h);
float oracle_entropy(const uint8_t* img, int stride, int w, int h);
/* A3 (mutual_information.cpp:14-25, 136-140, 48-53): batched over n pairs of
   rows x cols float patches, pair k at A + k*rows*cols */
void oracle_compare_pc(const float* A, const float* B, int n, int rows, int cols, float* out);
void oracle_ccoeff_normed(const float* A, const float* B, int n, int rows, int cols, float* out);
void oracle_quantise(uint8_t* img, int stride, int w, int h, int lo, int hi);
/* histogram dump: hl[20], hr[20], hj[400] integer counts */
void oracle_mi_histograms(const uint8_t* L, int strideL, const uint8_t* R, int strideR, int w, int h,
                          int32_t* hl, int32_t* hr, int32_t* hj);
/* batched form: n patch pairs of size pw x ph at integer top-left corners */
void oracle_mi_scores(const uint8_t* imgL, int strideL, const uint8_t* imgR, int strideR,
                      const int32_t* xyL, const int32_t* xyR, int n, int pw, int ph, float* out);
/* glibc-2.35 log2f restated (published ARM optimized-routines algorithm) */
float oracle_log2f(float x);

/* ---- A4-A8: ScaleState optimiser (src/optimisation/optimisation.cpp) ---- */
typedef struct {
  int n_left, n_right;
  const double* X_left;     /* 4*n_left homogeneous */
  const double* X_right;    /* 4*n_right */
  const uint8_t* tri_left;  /* WBA_Point::isTriangulated() */
  const uint8_t* tri_right;
  const uint32_t* last_left;  /* WBA_Point::getLastFrameIdx() */
  const uint32_t* last_right;
  uint32_t lframe;          /* poses.first[0].ID + poses.first.size()-1 */
  double K1[9], K2[9];      /* state.K.first / state.K.second, row-major */
  double q1[4], t1[3];      /* poses.first.back(): quaternion (w,x,y,z) + position */
  double q2[4], t2[3];      /* poses.second.back() */
  double scale, baseline;
  int window_size;
  const uint8_t* imgL; const uint8_t* imgR; int stride, cols, rows; /* m_obs[f_idx] */
  int bb_cols, bb_rows;     /* m_obs[0].first.cols, m_obs[1].first.rows */
  const uint8_t* mask; int mask_len;  /* optional Eigen::VectorXi mask (0/1) */
} oracle_scale_state;

typedef struct {
  int type;          /* 0 = GN, 1 = LM (OptimType) */
  int minim;
  int max_nb_iter;
  double v, tau, mu, abs_tol, grad_tol, incr_tol, rel_tol, alpha;
  int weighting;
} oracle_optim_params;

void oracle_optim_default_params(oracle_optim_params* p);
/* returns number of rows (or -1 on error); res must hold n_left+n_right */
int oracle_scale_residuals(const oracle_scale_state* s, int weighting, double* res);
int oracle_scale_normal_equations(const oracle_scale_state* s, int weighting, const double* res, double* JJ, double* e);
int oracle_scale_jacobian(const oracle_scale_state* s, int weighting, double* JJ);
/* runs Optimiser::optimise; writes final scale into s->scale; returns StopCondition.
   trace (optional): per outer iteration {e1, scale_after}; counts MI evaluations. */
int oracle_scale_optimise(oracle_scale_state* s, const oracle_optim_params* p, int test,
                          int* iterations, double* trace, int trace_cap, long* mi_evals);
int oracle_scale_inliers(const oracle_scale_state* s, double threshold, int* idx, int cap);
/* ScaleState::compute_residuals (optimisation.cpp:230-278), evident intent (parity unpinned) */
int oracle_scale_state_mi(const oracle_scale_state* s, double* out, int* npairs);
void oracle_scale_counters(long* out3);

/* ---- A13-A17: windowed stereo BA (BundleAdjuster.h + Ceres LM semantics) ---- */
typedef struct {
  int n_cams, n_pts, n_obs;
  double* cams;          /* n_cams*6 {tx,ty,tz,rx,ry,rz}  in/out */
  double* pts;           /* n_pts*3 in/out */
  const double* obs;     /* n_obs*4 {xL,yL,xR,yR} */
  const int32_t* cam_idx;
  const int32_t* pt_idx;
  double K0[9], K1[9];
  double baseline, feat_var;
  int fixed_frames;
  int obs_dim;            /* 4 (or 0): Observation<4>; 2: BundleAdjuster<2> Observation<2> {x,y} */
  const int32_t* cam_id;  /* obs_dim 2: Observation::camID (0 Standard-, else StereoRightError) */
} oracle_ba_problem;

typedef struct {
  int max_num_iterations;
  double function_tolerance, gradient_tolerance, parameter_tolerance;
  double initial_trust_region_radius, max_trust_region_radius, min_trust_region_radius;
  double min_lm_diagonal, max_lm_diagonal, min_relative_decrease;
  int max_num_consecutive_invalid_steps;
  int jacobi_scaling;
} oracle_ba_options;

typedef struct {
  int status;           /* BundleAdjuster::Status: 2 SUCCESSFUL, 3 FAILED */
  int termination;      /* 0 CONVERGENCE, 1 NO_CONVERGENCE, 2 FAILURE */
  int iterations;       /* Ceres iterations (steps attempted) */
  int successful_steps;
  double initial_cost, final_cost;
} oracle_ba_summary;

void oracle_ba_default_options(oracle_ba_options* o);
/* residuals (D/obs, D = obs_dim, sigma-scaled, uncorrected) + jacobians by Jets (Dx6, Dx3) */
void oracle_ba_evaluate(const oracle_ba_problem* p, double* res, double* Jc, double* Jp);
double oracle_ba_cost(const oracle_ba_problem* p);
int oracle_ba_solve(oracle_ba_problem* p, const oracle_ba_options* o, oracle_ba_summary* s,
                    double* cost_trace, int trace_cap);
/* one linearisation at the given params: reduced camera system of the first
   LM step (scaled coordinates, radius r).  S is (6m)x(6m), b 6m, m = non-fixed cams. */
int oracle_ba_reduced_system(const oracle_ba_problem* p, double radius, double* S, double* b);
/* pose covariance (BundleAdjuster.h:478-528 / ceres::Covariance): dense (J^T J)^-1 over all
   variable parameters by Cholesky, camera blocks out (zero for constant cameras); 0 if not PD */
int oracle_ba_covariance(const oracle_ba_problem* p, double* cov /* n_cams*36 */);
int oracle_ba_reduced_system_ex(const oracle_ba_problem* p, double radius, int jacobi, double* S, double* b);

/* ---- A11: nonMaxSupScanline3x3 (src/core/feature_types.cpp:253-351) ---- */
int oracle_nms_scanline3x3(const double* resp, int w, int h, uint8_t* mask, double* maxima, int cap);

/* ---- A12: KLT (build-defined; no reference) ---- */
typedef struct { int win; int max_level; int max_iters; double eps; double min_eig; } oracle_klt_params;
void oracle_klt_track(const uint8_t* prev, const uint8_t* next, int w, int h, int stride,
                      const float* pts_in, float* pts_out, uint8_t* status, int n, const oracle_klt_params* kp);
/* pyramid + scharr helpers (exposed for unit tests) */
void oracle_pyr_down(const uint8_t* src, int w, int h, int sstride, uint8_t* dst, int dw, int dh, int dstride);
void oracle_scharr(const uint8_t* src, int w, int h, int stride, int16_t* dx, int16_t* dy);

/* ---- A19: StereoVisualOdometry glue (src/vo/StereoVisualOdometry.cpp) ---- */
typedef struct {
  int method;  /* 0 GN, 1 LM */
  double e1, e2, e3, e4; int max_iter; int ransac; int n_ransac; double inlier_threshold;
  double baseline, fu1, fv1, fu2, fv2, cu1, cu2, cv1, cv2;
} oracle_vo_params;
/* matches: n * 8 floats {f1x,f1y,f2x,f2y,f3x,f3y,f4x,f4y}.  rand_seq: pre-drawn rand()
   values (as glibc would return) consumed by selectRandomIndices.  Returns process() result;
   motion 16 doubles row-major; inliers (ascending).  max_outer bounds the LM/GN loop
   (the reference's loop-exit quirk can spin forever). */
int oracle_vo_process(const float* matches, int n, const double* init6, const oracle_vo_params* p,
                      const int* rand_seq, int rand_len, double* motion, int* inliers, int* n_inliers,
                      int max_outer);

/* ---- Mono VO (src/vo/MonoVisualOdometry.cpp:7-73): OpenCV findEssentialMat
   (five-point + RANSAC / LMedS) + recoverPose restated (oracle/mono.cpp) ---- */
typedef struct {
  double fu, fv, cu, cv;     /* MonoVisualOdometry::parameters (MonoVisualOdometry.h:21-28) */
  double prob;               /* 0.99 */
  double inlier_threshold;   /* VisualOdometry::parameters, 2.0 (<= 0 -> 1.0) */
  int ransac;                /* 1 RANSAC, 0 LMedS */
} oracle_mono_params;
/* f1, f2: n matches (x, y) float; Rt 16 (row-major 4x4), E 9; inliers: indices
   into the matches; stats (optional): iterations run, best inlier count,
   recoverPose branch.  Returns process(): 1 / 0. */
int oracle_mono_vo_process(const float* f1, const float* f2, int n, const oracle_mono_params* p, double* Rt,
                           double* E, int32_t* inliers, int* n_inliers, int* stats);
int oracle_five_point(const double* x1, const double* x2, double* E_out /* 90 */);
float oracle_sampson(const double* E, const double* x1, const double* x2);
/* the first n_sets RANSAC subsets (5 indices each) of cv::RNG((uint64)-1) */
int oracle_cv_rng_subsets(int count, int n_sets, int32_t* idx);

/* ---- pose-covariance propagation (src/core/feature_types.cpp:171-251) ---- */
void oracle_pose_mul_cov(const double* q1, const double* t1, const double* c1, const double* q2, const double* t2,
                         const double* c2, int reverse, double* q3, double* t3, double* c3);
void oracle_pose_invert_cov(double* q, double* t, double* cov);
void oracle_pose_scale_cov(double* t, double* cov, double s, double var);

#ifdef __cplusplus
}
#endif
#endif
