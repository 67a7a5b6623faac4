/* me_hip.h — C ABI of the MI355X-native stereo-VO hot path (libme_hip.so).
 *
 * Drop-in boundary for abeauvisage/uasl_motion_estimation.  Every entry point
 * names the reference interface it replaces (paths relative to the reference
 * root).  Plain pointers and sizes only: no OpenCV / Eigen / Ceres / torch
 * types cross this boundary.  The C++ adapters that keep the reference's
 * include/MotionEstimation signatures live in include/MotionEstimationAMD/.
 *
 * Conventions
 *  - Every function returns ME_OK (0) or a negative ME_ERR_* code; the
 *    message of the last error on a context is returned by me_last_error().
 *  - One me_ctx per host thread (the reference is single-threaded).  A ctx
 *    owns a HIP device, a stream and scratch memory.
 *  - `mem` = ME_HOST: pointers are host memory, the call copies in/out and
 *    returns when results are on the host.  ME_DEVICE: pointers are device
 *    memory on the ctx device; the call is asynchronous on the ctx stream
 *    (call me_synchronize() before reading results on the host).
 *  - Images are 8-bit grayscale, row-major with a stride in bytes (the
 *    reference reads CV_8U images, src/core/file_IO.cpp:300,304).
 */
#ifndef ME_HIP_H
#define ME_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ME_ABI_VERSION 4

enum {
  ME_OK = 0,
  ME_ERR_INVALID = -1,     /* bad argument / shape (reference: assert / cv::Exception) */
  ME_ERR_HIP = -2,         /* HIP runtime error */
  ME_ERR_NOMEM = -3,
  ME_ERR_UNSUPPORTED = -4,
  ME_ERR_STATE = -5,       /* misuse of a stateful object (reference: std::cerr + status) */
  ME_ERR_NO_DEVICE = -6    /* no HIP device: the product path never falls back to the CPU */
};

typedef enum { ME_HOST = 0, ME_DEVICE = 1 } me_mem;

typedef struct me_ctx me_ctx;

/* ---- context ---------------------------------------------------------- */
int me_abi_version(void);
/* roctx ranges (rocprofv3 --marker-trace): every compute entry point opens
   one named after itself; callers can bracket their own stages (the VO
   loop's KLT / matching / BA / scale stages). */
int me_range_push(const char* name);
int me_range_pop(void);
int me_device_count(int* n);
int me_create(me_ctx** out, int hip_device);
void me_destroy(me_ctx* ctx);
const char* me_last_error(const me_ctx* ctx);
/* Use an external HIP stream (e.g. torch.cuda.current_stream().cuda_stream);
   NULL restores the ctx-owned stream. */
int me_set_stream(me_ctx* ctx, void* hip_stream);
void* me_get_stream(me_ctx* ctx);
/* Restrict the ctx-owned stream to a set of compute units (bit i of mask[i/32]
   = CU i; nwords = 0 restores all CUs): the stream is re-created with
   hipExtStreamCreateWithCUMask after the old one drains.  Lets two contexts
   of one GPU (e.g. a tracking front end and a BA back end) run side by side
   on disjoint CUs instead of sharing every CU's issue slots.  No reference
   counterpart (the reference runs one CPU thread).  hipExtStreamCreateWithCUMask
   takes no flags: the masked stream is a blocking stream (it orders with
   work on the legacy null stream, e.g. torch's default stream), unlike the
   hipStreamNonBlocking stream a ctx owns otherwise; me_stream_flags reports
   the flags of the ctx's current stream.  On MI355X logical CU i sits on XCD
   i mod 8: give each context whole XCDs (CU i to the front end iff
   i mod 8 < k) so the two keep separate L2s -- measured +2 % on the bench
   frame and +7 / +15 % on the config-3 / config-5 VO loop against a split
   that shares every XCD. */
int me_set_cu_mask(me_ctx* ctx, const uint32_t* mask, int nwords);
int me_stream_flags(me_ctx* ctx, unsigned* flags);
/* Compute units of the ctx device (the CU count a me_set_cu_mask split divides). */
int me_cu_count(me_ctx* ctx, int* n);
int me_synchronize(me_ctx* ctx);
int me_malloc(me_ctx* ctx, void** dptr, size_t bytes);
int me_free(me_ctx* ctx, void* dptr);
int me_memcpy_h2d(me_ctx* ctx, void* dst, const void* src, size_t bytes);
int me_memcpy_d2h(me_ctx* ctx, void* dst, const void* src, size_t bytes);
int me_memcpy_d2d(me_ctx* ctx, void* dst, const void* src, size_t bytes);
/* Asynchronous copy in any direction on the ctx stream (page-locked host
   memory from me_host_alloc for a truly asynchronous host side). */
int me_memcpy_async(me_ctx* ctx, void* dst, const void* src, size_t bytes);
int me_host_alloc(me_ctx* ctx, void** hptr, size_t bytes);
int me_host_free(me_ctx* ctx, void* hptr);

/* Per-kernel timing with HIP events on the ctx stream (for bench.py's
   roofline): enable a bitmask of families (bit k = ME_KT k; ME_KT_ALL = every
   family, 0 = off), then read the number of launches and the summed
   milliseconds of a family.  Each timed launch adds two event records to the
   stream, so time only the families a measurement needs. */
enum { ME_KT_MI = 0, ME_KT_SCALE_RES = 1, ME_KT_SCALE_NEQ = 2, ME_KT_BA_LINEARIZE = 3, ME_KT_BA_POINTS = 4,
       ME_KT_BA_SCHUR = 5, ME_KT_BA_SOLVE = 6, ME_KT_BA_STEP = 7, ME_KT_KLT = 8, ME_KT_PYR = 9, ME_KT_NMS = 10,
       ME_KT_COUNT = 16, ME_KT_ALL = 0xffff };
int me_timing_enable(me_ctx* ctx, int family_mask);
int me_timing_read(me_ctx* ctx, int kernel, long* launches, double* total_ms);
int me_timing_reset(me_ctx* ctx);
/* Time only every k-th launch of each timed family (k >= 1; 1 = every launch,
   the default): a live measurement of the average launch duration whose
   event records perturb the stream k times less. */
int me_timing_sample(me_ctx* ctx, int every);
/* Measured HBM bandwidth of this device (GB/s, read + write bytes / time):
   a 16-byte-per-lane streaming copy of `bytes` bytes, `reps` timed launches
   on the ctx stream (after one untimed) -- the measured denominator beside
   the 8 TB/s datasheet peak in bench.py's roofline objects.  Allocates and
   frees 2 x bytes of device memory; synchronises the ctx stream. */
int me_hbm_copy_gbs(me_ctx* ctx, size_t bytes, int reps, double* gbs);

/* ---- A1/A2: mutual information ---------------------------------------
 * Replaces float me::computeMutualInformation(const cv::Mat&, const cv::Mat&)
 * (include/MotionEstimation/core/mutual_information.h:20,
 *  src/core/mutual_information.cpp:55-86), batched: n patch pairs of
 * patch_w x patch_h pixels whose top-left corners are xyL[2k],xyL[2k+1] in imgL
 * and xyR[2k],xyR[2k+1] in imgR (the reference truncates ROI corners to int,
 * SURVEY A-4).  Bit-exact with the reference's float result (20-bin calcHist,
 * fl32(c*fl32(1/N)) normalisation, row-major float sum, glibc log2f). */
int me_mi_scores(me_ctx* ctx, me_mem mem, const uint8_t* imgL, int strideL, const uint8_t* imgR, int strideR,
                 int width, int height, const int32_t* xyL, const int32_t* xyR, int n, int patch_w, int patch_h,
                 float* mi_out);
/* Whole-patch form (any size, the literal computeMutualInformation(L, R)). */
int me_mutual_information(me_ctx* ctx, me_mem mem, const uint8_t* L, int strideL, const uint8_t* R, int strideR,
                          int w, int h, float* mi_out);
/* Epipolar stereo matcher of the VO loop (the application's MI stereo
   matching around me::computeMutualInformation; build-defined like KLT, no
   reference symbol): feature k at (u_k, v_k) of imgL (rectified pair, one
   stride), candidate disparities d = lo_k .. lo_k + nd - 1, left patch at
   (floor(u - patch/2), floor(v - patch/2)), right patch d pixels to its
   left; a candidate is scored (MI, the bits of me_mi_scores) iff its right
   patch starts at x >= 0, d <= d_max and the feature is valid (valid_k != 0
   when valid is given; status_k == 1 and margin <= u < width - margin,
   margin <= v < height - margin when status is given -- the KLT gate).
   Pick: first maximum, interior, FP64 parabola vertex, optional uniqueness
   (best >= ratio * best outside +-2 candidates); xr_k = u_k - disparity
   (float), ok_k = 1 iff the pick holds and xr_k >= margin.  Every array is
   device memory; asynchronous on the ctx stream. */
int me_mi_epipolar_match(me_ctx* ctx, const uint8_t* imgL, const uint8_t* imgR, int width, int height, int stride,
                         const float* uv, const int32_t* lo, const uint8_t* valid, const uint8_t* status, int n,
                         int nd, int patch, int d_max, int unique, double ratio, float margin, float* xr_out,
                         uint8_t* ok_out);
/* me_mi_epipolar_match over the first *n_dev features (a device count left
   by a preceding kernel, at most n_max), no valid / status gate. */
int me_mi_epipolar_match_count(me_ctx* ctx, const uint8_t* imgL, const uint8_t* imgR, int width, int height,
                               int stride, const float* uv, const int32_t* lo, const int32_t* n_dev, int n_max,
                               int nd, int patch, int d_max, int unique, double ratio, float margin, float* xr_out,
                               uint8_t* ok_out);
/* New-feature cells of the VO loop (pipeline.new_cells on the device; no
   reference symbol -- the application's grid detector around WBA_Point
   creation): tracked feature k is good iff status_k == 1, ok_k != 0 and it
   lies inside the margin; good features occupy their grid cell
   (trunc((u - margin) / cw), trunc((v - margin) / ch)) clamped, FP64; the
   first max(0, n_feats - #good) empty cells in ascending order get a feature
   at margin + (cell + 0.5 + jitter(t, cell)) * (cw, ch) (float), lo = d_min;
   *out_count = their number.  Device memory, asynchronous on the ctx stream:
   with me_mi_epipolar_match_count the new features are matched in the same
   submission as the tracked ones. */
int me_vo_new_cells(me_ctx* ctx, const float* uv, const uint8_t* status, const uint8_t* ok, int n, int width,
                    int height, float margin, int nx, int ny, double cw, double ch, int n_feats, int t, int d_min,
                    float* out_uv, int32_t* out_lo, int32_t* out_count);
/* me::computeEntropy (src/core/mutual_information.cpp:28-45). */
int me_entropy(me_ctx* ctx, me_mem mem, const uint8_t* img, int stride, int w, int h, float* out);

/* ---- A3: the other patch utilities of src/core/mutual_information.cpp -
 * Batched over n pairs of rows x cols float patches stored contiguously
 * (pair k at A + k * rows * cols, row-major).  me_compare_pc replaces
 * me::comparePC (mutual_information.cpp:14-25, bit-exact); me_ccoeff_normed
 * replaces me::applyCCOEFFNormed (:136-140; OpenCV MatExpr rounding restated,
 * parity unpinned); me_quantise replaces me::quantise(img, {lo, hi}) (:48-53),
 * in place, lo != hi. */
int me_compare_pc(me_ctx* ctx, me_mem mem, const float* A, const float* B, int n, int rows, int cols, float* out);
int me_ccoeff_normed(me_ctx* ctx, me_mem mem, const float* A, const float* B, int n, int rows, int cols, float* out);
int me_quantise(me_ctx* ctx, me_mem mem, uint8_t* img, int stride, int w, int h, int lo, int hi);

/* ---- A4-A9: ScaleState optimiser --------------------------------------
 * Replaces me::optimisation::Optimiser<ScaleState, std::vector<std::pair<cv::Mat,cv::Mat>>>
 * (include/MotionEstimation/optimisation/optimisation.h:76-125,
 *  src/optimisation/optimisation.cpp:29-228,435-747).  The state is the
 * flattened ScaleState: tracks (WBA_Ptf) as homogeneous points + flags, the
 * last poses of the window, intrinsics, scale, baseline, window size and the
 * last keyframe image pair (m_obs[poses.first.size()-1]). */
typedef struct {
  int n_left, n_right;
  const double* X_left;      /* 4*n_left, WBA_Point::get3DLocation() */
  const double* X_right;     /* 4*n_right */
  const uint8_t* tri_left;   /* WBA_Point::isTriangulated() */
  const uint8_t* tri_right;
  const uint32_t* last_left; /* WBA_Point::getLastFrameIdx() */
  const uint32_t* last_right;
  uint32_t lframe;           /* poses.first[0].ID + poses.first.size()-1 */
  double K1[9], K2[9];       /* state.K.first / .second, row-major */
  double q1[4], t1[3];       /* poses.first.back(): Quat (w,x,y,z), position */
  double q2[4], t2[3];       /* poses.second.back() */
  double scale, baseline;
  int window_size;
  const uint8_t* imgL;       /* m_obs[f_idx].first  (mem = img_mem) */
  const uint8_t* imgR;       /* m_obs[f_idx].second */
  int stride, cols, rows;
  int bb_cols, bb_rows;      /* m_obs[0].first.cols, m_obs[1].first.rows */
  const uint8_t* mask;       /* optional Eigen::VectorXi mask as 0/1 bytes (host) */
  int mask_len;
  me_mem img_mem;
  me_mem tracks_mem;         /* X_*, tri_*, last_* in host (ME_HOST) or device memory; mask is always host */
} me_scale_state;

typedef struct {
  int type;                  /* 0 = OptimType::GN, 1 = OptimType::LM */
  int minim;
  int max_nb_iter;
  double v, tau, mu, abs_tol, grad_tol, incr_tol, rel_tol, alpha;
  int weighting;
} me_optim_params;

/* OptimisationParams() defaults (optimisation.h:31) */
void me_optim_default_params(me_optim_params* p);
/* Optimiser::compute_residuals (optimisation.cpp:149-228): res has
   n_left+n_right slots; *n_rows receives the row count. */
int me_scale_residuals(me_ctx* ctx, const me_scale_state* s, int weighting, double* res, int* n_rows);
/* Optimiser::compute_normal_equations (optimisation.cpp:435-537). */
int me_scale_normal_equations(me_ctx* ctx, const me_scale_state* s, int weighting, const double* res, double* JJ,
                              double* e);
/* Optimiser::compute_jacobian / getJacobian (optimisation.cpp:539-634). */
int me_scale_jacobian(me_ctx* ctx, const me_scale_state* s, int weighting, double* JJ);
/* Optimiser::optimise (optimisation.cpp:29-147): updates s->scale, returns the
   StopCondition (rotation_utils.h:20) in *stop. trace: {e1, scale} per outer
   iteration (optional). */
int me_scale_optimise(me_ctx* ctx, me_scale_state* s, const me_optim_params* p, int test, int* stop,
                      int* iterations, double* trace, int trace_cap, long* mi_evals);
/* Counters of the last me_scale_optimise on this ctx, in the reference loop's
   terms (optimisation.cpp:29-147, :685-730): compute_residuals calls,
   compute_normal_equations calls and rejected LM candidates (the else branch
   of run_LM_step, :719-727).  An evaluation the device skips because its
   result is already known (same state) still counts.  executed = residual
   evaluations the device actually ran (speculative candidates included). */
int me_scale_last_counters(me_ctx* ctx, long* res_evals, long* neq_evals, long* rejections, long* executed);
/* Launch form me_scale_optimise picks for nb track blocks (16 tracks each)
   when `cap` workgroups of the persistent LM kernel fit on the ctx's CUs:
   1 = the one persistent launch (nb x 2 workgroups, at most half of cap),
   0 = one launch per LM phase.  The persistent grid does not need to be
   co-resident (a workgroup roster deals the work over the workgroups that
   run), so this is a throughput choice; no environment
   variable changes it.  Host only: no device, no ctx. */
int me_scale_persistent(int nb, int cap);
/* double ScaleState::compute_residuals(std::vector<std::pair<cv::Mat,cv::Mat>>&)
   (include/MotionEstimation/optimisation/optimisation.h:86, src/optimisation/optimisation.cpp:230-278):
   one mutual information over the stacked 2w x 2w patch pairs of the left
   tracks (triangulated, seen in the last keyframe, both reprojections inside
   Rect(w, w, cols - 2w, rows - 2w)).  The reference's stacking
   (`left_img(Range..) = imgs[i].first`, :273-274) rebinds a temporary ROI
   header and copies no pixels, so its stacked images are uninitialised and
   its result undefined; this computes the evident intent (the MI of the
   stacked patches), parity unpinned.  n_patches (optional) receives the
   number of stacked pairs; none -> ME_ERR_INVALID (the reference's
   computeMutualInformation asserts on empty input). */
int me_scale_state_mi(me_ctx* ctx, const me_scale_state* s, double* mi_out, int* n_patches);
/* Optimiser::compute_inliers (optimisation.cpp:732-747): row indices. */
int me_scale_inliers(me_ctx* ctx, const me_scale_state* s, int weighting, double threshold, int* idx, int cap,
                     int* n_out);

/* ---- A13-A17: windowed stereo bundle adjustment ----------------------
 * Replaces me::optimisation::BundleAdjuster<4>::optimise(int fixedFrames)
 * (include/MotionEstimation/optimisation/BundleAdjuster.h:142-180,431-476)
 * and the Ceres solve it wraps: StereoReprojectionError residual/Jacobian,
 * HuberLoss(1.0), LM trust region with Jacobi scaling, point-first Schur
 * elimination, box bounds on points.  cams are Matx61d {t, angle-axis}
 * (BundleAdjuster.h:297-310), observations Observation<4>.
 * obs_dim = 2 selects BundleAdjuster<2>::optimise (BundleAdjuster.h:378-429):
 * Observation<2> {x, y} with cam_id = Observation::camID, residual
 * StandardReprojectionError (:71-103) for camID 0 and StereoRightError
 * (:106-139) otherwise, K[0] only, a zero baseline replaced by 0.5 (:389-390). */
typedef struct {
  int n_cams, n_pts, n_obs;
  double* cams;              /* n_cams*6, updated in place */
  double* pts;               /* n_pts*3, updated in place */
  const double* obs;         /* n_obs*4 {xL, yL, xR, yR} */
  const int32_t* cam_idx;    /* Observation::camIdx */
  const int32_t* pt_idx;     /* Observation::ptIdx */
  double K0[9], K1[9];       /* CalibrationParameters::K[0], K[1] */
  double baseline, feat_var;
  int fixed_frames;          /* optimise(fixedFrames) */
  me_mem mem;                /* ME_HOST: the arrays above are host memory (copied in/out);
                                ME_DEVICE: device memory on the ctx device, cams/pts updated in
                                place on the device (me_ba_solve / me_ba_solve_sharded only) */
  int obs_dim;               /* 4 (or 0): Observation<4>; 2: Observation<2> (BundleAdjuster<2>) */
  const int32_t* cam_id;     /* obs_dim 2: Observation::camID per observation; ignored otherwise */
} me_ba_problem;

typedef struct {
  int max_num_iterations;          /* Ceres default 50 */
  double function_tolerance;       /* 1e-3 (BundleAdjuster.h:465) */
  double gradient_tolerance;       /* 1e-10 */
  double parameter_tolerance;      /* 1e-8 */
  double initial_trust_region_radius, max_trust_region_radius, min_trust_region_radius;
  double min_lm_diagonal, max_lm_diagonal, min_relative_decrease;
  int max_num_consecutive_invalid_steps;
  int jacobi_scaling;
} me_ba_options;

typedef struct {
  int status;                /* BundleAdjuster::Status: 2 SUCCESSFUL, 3 FAILED */
  int termination;           /* 0 CONVERGENCE, 1 NO_CONVERGENCE, 2 FAILURE */
  int iterations;
  int successful_steps;
  double initial_cost, final_cost;
} me_ba_summary;

void me_ba_default_options(me_ba_options* o);
int me_ba_solve(me_ctx* ctx, me_ba_problem* p, const me_ba_options* o, me_ba_summary* s);
/* Asynchronous form of me_ba_solve (same BundleAdjuster<M>::optimise,
   BundleAdjuster.h:378-476, same results bit for bit): queues every
   possible iteration (max_num_iterations + 1 linearisations; launches after
   convergence return at once, so it suits fixed-iteration windows) and the
   read-back on the ctx stream, and returns without waiting.  The caller keeps
   *p's arrays alive until me_ba_wait, which blocks on this solve only (not on
   work queued after it), writes host-problem results back and fills *s.  Up
   to two solves may be queued per ctx (each in its own scratch and staging):
   window t+1 can be queued behind window t before t is waited, so the device
   never idles while the host builds the next plan; me_ba_wait completes the
   oldest.  A third me_ba_solve_async before a wait is ME_ERR_STATE.  Any other
   BA call on the ctx completes the queued solves first (their summaries stay
   readable by me_ba_wait). */
int me_ba_solve_async(me_ctx* ctx, me_ba_problem* p, const me_ba_options* o);
int me_ba_wait(me_ctx* ctx, me_ba_summary* s);
/* me_ba_wait, and for a device-resident problem (ME_DEVICE) its solved cams
   (6 per camera) / pts (3 per point) copied to host arrays (either may be
   NULL): read back behind the solve, so the wait does not block on work
   queued after it. */
int me_ba_wait_out(me_ctx* ctx, me_ba_summary* s, double* cams, double* pts);
/* Sizes the ctx's BA scratch and page-locked staging (synchronous and both
   asynchronous sets) for windows up to these sizes, so a growing window does
   not reallocate (a reallocation waits for the ctx stream).  No solve may be
   queued. */
int me_ba_reserve(me_ctx* ctx, int n_cams, int n_pts, int n_obs, int obs_dim, int fixed_frames);
/* Windowed VO loop (pipeline.py WindowedStereoVO.process, step 7), no
   counterpart in the reference (whose loop solves each window before the
   next keyframe, WBA_Point / BundleAdjuster.h): window t's BA start formed on
   the device from the last queued device-resident solve (window t-1) before
   that solve completes.  cams (n_cams x 6) / pts (n_pts x 3), device memory,
   hold the host's values (the loop state before window t-1's result); camera
   k with cam_src >= 0 takes that solve's camera cam_src, landmark i (track ID
   win_ids[i]) that solve's point of the same ID in prev_ids (window t-1's
   ascending IDs, n_prev), when it succeeded (termination != FAILURE); a
   landmark with ID >= new_from is new in keyframe t, moved from pose
   (rotation R, row-major) to the new pose(t) when they differ; camera
   n_cams - 1 is pose(t):
   mode 1: c[k1] + (c[k1] - c[k0]), mode 0: c[k1] + vel, mode -1: kept.  The
   new pose's rotation is a fixed Taylor series in theta^2 (the loop's host
   code repeats the arithmetic bit for bit).  Asynchronous on the ctx stream. */
typedef struct me_vo_chain_args {
  double pose[6];
  double R[9];
  double vel[6];
  int k1, k0, mode;
} me_vo_chain_args;
int me_vo_ba_chain(me_ctx* ctx, double* cams, int n_cams, double* pts, int n_pts, const int32_t* cam_src,
                   const int32_t* win_ids, const int32_t* prev_ids, int n_prev, int32_t new_from,
                   const me_vo_chain_args* a);
/* One keyframe's window solve in one call (for a thread that queues window t
   while another waits for window t-1 with me_ba_wait_out -- the two may run
   concurrently on one ctx; no other call on the ctx meanwhile): the staged
   H2D (stage -> dev, stage_bytes, may be 0), me_vo_ba_chain when `chain`
   (on p->cams / p->pts), me_ba_window_indices (frame / ids of the window's
   p->n_obs observations, first_frame, win_ids -> p->cam_idx / p->pt_idx),
   me_ba_solve_async(p, o). */
typedef struct me_vo_window {
  const void* stage;
  void* dev;
  size_t stage_bytes;
  int chain;
  const int32_t* cam_src;
  const int32_t* win_ids;
  const int32_t* prev_ids;
  int n_prev;
  int32_t new_from;
  me_vo_chain_args args;
  const int32_t* frame;
  const int32_t* ids;
  int first_frame;
} me_vo_window;
int me_vo_window_submit(me_ctx* ctx, const me_vo_window* w, me_ba_problem* p, const me_ba_options* o);
/* ---- the windowed stereo VO loop, native (round 5) ----------------------
 * The application loop around the hot path (pipeline.py WindowedStereoVO
 * with its GPU backend, every step in C++ behind this ABI): per keyframe t
 * the KLT of the active tracks, the epipolar MI matching of the tracked and
 * of the new features (one front-end round trip), the WBA_Point bookkeeping
 * (include/MotionEstimation/core/feature_types.h:121-197: IDs from the value
 * constructor, addMatch, pop of features leaving the window, deletion of
 * empty tracks) over a structure-of-arrays track table, the scale LM
 * (Optimiser<ScaleState,...>::optimise, optimisation.cpp:29-147) of keyframe
 * t-1 and the sliding-window BA (BundleAdjuster<4>::optimise over the last
 * `window` keyframes, initialiseObservations order, BundleAdjuster.h:354-376,
 * 431-476) queued behind the previous window's solve (me_vo_window_submit).
 * The loop is lagged exactly as pipeline.py's: BA(t-1) enters the state after
 * keyframe t is matched and booked.  Two contexts of one device: `ba` runs the
 * window solves, `front` the KLT, the matchers and the scale LM (they may be
 * the same ctx: then nothing runs on a worker thread).  Results are the
 * Python loop's bit for bit (tests/test_pipeline.py (test_native_loop_*, test_cpp_host_drives_the_loop)).  One loop per pair of
 * contexts; no other call on either ctx while a loop call runs. */
typedef struct {
  int width, height, n_feats, window;
  int ba_iters, scale_iters, fixed_frames, d_min, d_max;
  double baseline, feat_var;
  double K[9];                /* row-major intrinsics (both cameras) */
  double first_pose[6];       /* {t, angle-axis} world -> camera of keyframe 0 */
  double velocity[6];         /* motion prior of keyframe 1 (has_velocity) */
  int has_velocity;
  int log_events;             /* keep the WBA_Point event log (me_vo_loop_events) */
  int async_enqueue;          /* window solves queued from a worker thread (ignored when ba == front) */
} me_vo_loop_config;
typedef struct {              /* pipeline.FrameResult */
  int t, n_tracked, n_new, n_active, n_window_pts, n_window_obs;
  double scale;
  int scale_stop, scale_iters, ba_iters;
  double ba_cost;
  double pose[6];
} me_vo_frame_result;
typedef struct {              /* one WBA_Point call: kind 0 new (value ctor), 1 addMatch, 2 pop, 3 deleted */
  int kind, t;
  int64_t id;
  float feat[4];              /* {xl, yl, xr, yr} (new / add) */
} me_vo_event;
typedef struct me_vo_loop me_vo_loop;
void me_vo_loop_default_config(me_vo_loop_config* c);
int me_vo_loop_create(me_ctx* ba, me_ctx* front, const me_vo_loop_config* cfg, me_vo_loop** out);
void me_vo_loop_destroy(me_vo_loop* v);
const char* me_vo_loop_last_error(const me_vo_loop* v);
/* Keyframe t (t = 0, 1, 2, ... in order): left / right 8-bit images of
   width x height (stride = width).  mem = ME_DEVICE: device memory on the
   ctx device, read during this call and the next one (keep it alive until
   me_vo_loop_process(t + 1) returns); ME_HOST: copied in. */
int me_vo_loop_process(me_vo_loop* v, int t, const uint8_t* left, const uint8_t* right, me_mem mem);
/* Completes the last keyframe (its pops, scale LM and BA). */
int me_vo_loop_finish(me_vo_loop* v);
/* Results of the completed keyframes (*n = their number; min(cap, *n) copied). */
int me_vo_loop_results(me_vo_loop* v, me_vo_frame_result* out, int cap, int* n);
int me_vo_loop_events(me_vo_loop* v, me_vo_event* out, long cap, long* n);
/* Live track table (creation = ID order): IDs, landmarks (3 per track), active flag, first held / last frame. */
int me_vo_loop_tracks(me_vo_loop* v, int64_t* ids, double* X, uint8_t* active, int64_t* first, int64_t* last, int cap,
                      int* n);
int me_vo_loop_poses(me_vo_loop* v, int32_t* ts, double* poses, int cap, int* n);
/* Observations of keyframe t still held (ascending track IDs, {xl, yl, xr, yr}); *n = -1 when none. */
int me_vo_loop_frame_obs(me_vo_loop* v, int t, int64_t* ids, float* feats, int cap, int* n);
int me_vo_loop_frames(me_vo_loop* v, int32_t* ts, int cap, int* n);
/* [0] host seconds outside waits, [1] seconds blocked on device results, [2] tracks created (latestID),
   [3..8] seconds blocked in: KLT + matching, first-keyframe matching, scale LM submit, window submit,
   BA result, scale LM result. */
int me_vo_loop_stats(me_vo_loop* v, double* out, int n);

/* BundleAdjuster<M>::initialiseObservations (BundleAdjuster.h:354-376) for a
   device-resident window: observation i was seen in frame[i] by the track
   ids[i]; cam_idx[i] = frame[i] - first_frame and pt_idx[i] = the position of
   ids[i] in win_ids (the window's track IDs, ascending), -1 if absent.  All
   arrays device memory; asynchronous on the ctx stream.  With the
   observations stored frame by frame, a sliding window appends one keyframe's
   observations per step and re-indexes on the device. */
int me_ba_window_indices(me_ctx* ctx, const int32_t* frame, const int32_t* ids, int n_obs, int first_frame,
                         const int32_t* win_ids, int n_pts, int32_t* cam_idx, int32_t* pt_idx);
/* Cost (Ceres ½Σρ) at the problem's current parameters. */
int me_ba_cost(me_ctx* ctx, const me_ba_problem* p, double* cost);
/* Residuals (sigma-scaled, uncorrected) and Jacobian blocks per observation:
   res D/obs, Jc 6D/obs (row-major Dx6), Jp 3D/obs (Dx3), D = obs_dim (4 or 2). */
int me_ba_evaluate(me_ctx* ctx, const me_ba_problem* p, double* res, double* Jc, double* Jp);
/* Reduced camera system of the first LM step at trust radius `radius`
   (scaled coordinates), S (6m x 6m row-major) and b (6m), m = non-fixed cams. */
int me_ba_reduced_system(me_ctx* ctx, const me_ba_problem* p, double radius, double* S, double* b);
/* Pose covariance at the problem's current parameters: replaces
   BundleAdjuster<M>::extract_covariance (BundleAdjuster.h:478-528), i.e.
   ceres::Covariance over the camera blocks with the loss function applied:
   cov[36 i .. 36 i + 35] = 6x6 row-major block i of (J^T J)^-1, obtained as
   the inverse of the point-eliminated camera system; constant (fixed) cameras
   get zero blocks as in Ceres.  *ok = 0 (and cov untouched) when J^T J is not
   positive definite (Ceres reports a rank-deficient Jacobian). */
int me_ba_covariance(me_ctx* ctx, const me_ba_problem* p, double* cov /* n_cams*36 */, int* ok);

/* ---- §8e: landmark-sharded BA over several GPUs ----------------------
 * No reference counterpart (the reference solves on one CPU thread); the
 * sharded solve replaces BundleAdjuster<4>::optimise (BundleAdjuster.h:431-476)
 * when the window's landmarks are split over ranks: every rank holds all
 * cameras and a contiguous landmark range with its observations.
 *
 * A communicator joins the ranks, one process (one me_ctx) per GPU:
 *  - me_comm_create_rccl: native RCCL over xGMI.  Rank 0 draws an id with
 *    me_comm_unique_id and hands the ME_COMM_ID_BYTES bytes to the other
 *    ranks (any side channel: a torch.distributed store, a file, MPI); every
 *    rank then creates its communicator on its ctx device (collective call).
 *    All-reduces are enqueued on the ctx stream: no host round trip.
 *  - me_comm_create_callback: a caller all-reduce (allreduce(dev_ptr, n, user)
 *    sums n doubles in place over the ranks, n < 0: max over |n|; it must be
 *    ordered on the ctx stream, e.g. host-staged gloo, or threads driving
 *    several contexts of one GPU).  Collective like the RCCL form: every
 *    rank creates its communicator concurrently.
 * Both creators calibrate the communicator (me_comm_calibrate): a few
 * all-reduces at the two exchange sizes of a sharded LM iteration, timed on
 * this rank, then the max over the ranks (one more exchange), so every rank
 * holds the same per-exchange costs and the landmark-count gate takes the
 * same decision everywhere (me_ba_shard_worthwhile_comm).
 * Per LM iteration the sharded solve exchanges twice: one sum of the packed
 * reduced camera system [S upper block triangle | b | diag(U) | camera
 * gradient | cost | failure count | per-rank gradient max-norm slots] after
 * the Schur pass, and one sum of the five step scalars after the point step;
 * the first linearisation also sums the Jacobi column norms.  Every rank
 * solves the camera system redundantly and steps its own landmarks. */
typedef int (*me_allreduce_fn)(double* dev_buf, int n, void* user);
typedef struct me_comm me_comm;
#define ME_COMM_ID_BYTES 128
enum { ME_COMM_SUM = 0, ME_COMM_MAX = 1 };
int me_comm_unique_id(void* id_out, int id_bytes);
int me_comm_create_rccl(me_ctx* ctx, int world, int rank, const void* id, me_comm** out);
int me_comm_create_callback(me_ctx* ctx, int world, int rank, me_allreduce_fn allreduce, void* user,
                            me_comm** out);
void me_comm_destroy(me_comm* comm);
int me_comm_info(const me_comm* comm, int* world, int* rank, int* native);
/* In-place all-reduce of n doubles of device memory on the ctx stream. */
int me_comm_allreduce(me_comm* comm, double* dev_buf, long n, int op);
/* Re-measures the communicator's exchange costs (collective: every rank
   calls it): `reps` timed all-reduces (after 3 untimed) of ME_COMM_CAL_SYSTEM
   doubles -- the packed reduced camera system of a 30-keyframe window -- and
   of 5 doubles (the step scalars), wall time per call including the stream
   synchronisation, max over the ranks.  The creators run it with reps = 10. */
#define ME_COMM_CAL_SYSTEM 17000
int me_comm_calibrate(me_comm* comm, int reps);
/* The calibrated costs (microseconds per exchange) of the system and the
   scalar exchange; 0 before any calibration. */
int me_comm_exchange_us(const me_comm* comm, double* system_us, double* scalars_us);
/* The gate below with this communicator's world and calibrated costs
   (xch_us = the mean of the two, so 2 * xch_us is one LM iteration's
   exchanges); uncalibrated: the built-in estimate.  Host only. */
int me_ba_shard_worthwhile_comm(const me_comm* comm, long n_obs);
int me_ba_solve_comm(me_ctx* ctx, me_ba_problem* p, const me_ba_options* o, me_comm* comm, me_ba_summary* s);
/* The same with a bare callback and no rank information (ABI v2 form): the
   gradient max-norm then travels in a separate max all-reduce. */
int me_ba_solve_sharded(me_ctx* ctx, me_ba_problem* p, const me_ba_options* o, me_allreduce_fn allreduce,
                        void* user, me_ba_summary* s);
/* Landmark-count gate of the sharded solve (shard "only when the
   landmark count warrants it").  Every rank solves the camera system
   redundantly, so sharding saves only landmark-kernel time (linearisation,
   Schur pass, point step) and costs two all-reduces per LM iteration.  Model
   per LM iteration: t(n) = max(ME_SHARD_FLOOR_US, n * ME_SHARD_OBS_NS / 1000)
   microseconds for n observations (fitted to the one-GPU shard timings of
   bench.py's sharded_ba.crossover_model); returns 1 when
   t(n_obs) - t(ceil(n_obs / world)) > 2 * xch_us, else 0 (world <= 1: 0).
   xch_us <= 0 takes the built-in per-exchange estimate for `world`
   (me_ba_shard_exchange_us, a fallback only: a communicator measures its
   own, me_comm_exchange_us).  Host only: no device, no ctx. */
#define ME_SHARD_OBS_NS 1.0
#define ME_SHARD_FLOOR_US 40.0
int me_ba_shard_worthwhile(long n_obs, int world, double xch_us);
double me_ba_shard_exchange_us(int world);

/* ---- A12: KLT feature tracking (build-defined; no reference) ---------- */
typedef struct { int win; int max_level; int max_iters; double eps; double min_eig; } me_klt_params;
void me_klt_default_params(me_klt_params* p);
int me_klt_track(me_ctx* ctx, me_mem mem, const uint8_t* prev, const uint8_t* next, int width, int height,
                 int stride, const float* pts_in, float* pts_out, uint8_t* status, int n, const me_klt_params* p);

/* ---- A11: non-maximum suppression ------------------------------------
 * Replaces std::vector<pt2D> me::nonMaxSupScanline3x3(const cv::Mat& input,
 * cv::Mat& output) (include/MotionEstimation/core/feature_types.h:270,
 * src/core/feature_types.cpp:253-351): response is CV_64F (h x w doubles),
 * mask_out h*w bytes (255 = maximum), maxima 2*cap doubles (row-major scan
 * order, (row+0.5+dr, col+0.5+dc)). */
int me_nms_scanline3x3(me_ctx* ctx, me_mem mem, const double* response, int width, int height, uint8_t* mask_out,
                       double* maxima, int cap, int* n_out);

/* ---- A19 / §8f-1: frame-to-frame stereo VO ---------------------------
 * Replaces bool me::StereoVisualOdometry::process(const std::vector<StereoOdoMatchesf>&,
 * cv::Mat init) (include/MotionEstimation/vo/StereoVisualOdometry.h:41,
 * src/vo/StereoVisualOdometry.cpp:34-92) with getMotion() (:331-342) and
 * getInliers_idx() (.h:47).  Parameters are StereoVisualOdometry::parameters
 * (StereoVisualOdometry.h:24-33 + VisualOdometry.h:19-33).  matches: n x 8
 * floats {f1.x, f1.y, f2.x, f2.y, f3.x, f3.y, f4.x, f4.y} (StereoOdoMatchesf:
 * previous left/right, current left/right).  The RANSAC triples come from
 * the context's glibc-compatible rand() stream (unseeded: as the
 * reference's rand(), reseed with me_vo_srand).  The reference's GN/LM loop
 * can run forever (StereoVisualOdometry.cpp:277); such a run is cut at
 * max_outer passes and reported as ME_ERR_STATE.  ok = process()'s result;
 * motion = getMotion() (4x4 row-major); state = the 6 state values
 * (Euler angles, translation); pts3d = getPts3D() (n x 4 homogeneous,
 * filled when n >= 6); inliers = getInliers_idx() (capacity n).  Any of
 * state, pts3d and inliers may be NULL. */
typedef struct {
  int method;                /* VisualOdometry::Method: 0 GN, 1 LM */
  double step_size, eps, e1, e2, e3, e4;
  int max_iter, nb_fixed_frames, ransac, n_ransac;
  double inlier_threshold;
  double baseline;
  int weighting;
  double fu1, fv1, fu2, fv2, cu1, cu2, cv1, cv2;
} me_vo_params;
void me_vo_default_params(me_vo_params* p);
int me_vo_srand(me_ctx* ctx, unsigned seed);
int me_vo_rand(me_ctx* ctx, int* out);  /* one draw of the context's rand() stream (tests) */
int me_vo_process(me_ctx* ctx, const float* matches, int n, const double* init6, const me_vo_params* p,
                  int max_outer, double* motion, double* state, double* pts3d, int* inliers, int* n_inliers,
                  int* ok);

/* ---- §8f-4: monocular VO -----------------------------------------------
 * Replaces bool me::MonoVisualOdometry::process(const std::vector<StereoMatch<
 * cv::Point2f>>&) (src/vo/MonoVisualOdometry.cpp:7-73) with getMotion(),
 * getEssentialMat(), getInliersIdx() (MonoVisualOdometry.h:35-41).  The
 * reference's OpenCV findEssentialMat (five-point + RANSAC at prob, or LMedS
 * when ransac = 0; threshold <= 0 -> 1 px) and recoverPose (distance 500) are
 * restated on the device (csrc/mono.hip; parity unpinned: OpenCV absent).
 * f1, f2: n (x, y) floats (StereoMatch f1 / f2; a match with f1.x <= 0 or
 * f2.x <= 0 is skipped as in the reference).  ok = process()'s result; Rt =
 * getMotion() (4x4 row-major, identity when ok = 0); E = getEssentialMat()
 * (3x3, zero when none; may be NULL); inliers = getInliersIdx() (indices into
 * the matches, capacity n; may be NULL). */
typedef struct {
  double fu, fv, cu, cv;     /* MonoVisualOdometry::parameters (MonoVisualOdometry.h:21-28) */
  double prob;               /* 0.99 */
  double inlier_threshold;   /* VisualOdometry::parameters: 2.0 */
  int ransac;                /* 1: RANSAC, 0: LMedS */
} me_mono_params;
void me_mono_default_params(me_mono_params* p);
int me_mono_vo_process(me_ctx* ctx, const float* f1, const float* f2, int n, const me_mono_params* p, double* Rt,
                       double* E, int32_t* inliers, int* n_inliers, int* ok);

#ifdef __cplusplus
}
#endif
#endif /* ME_HIP_H */
