// vo_loop.hip -- the windowed stereo VO loop in native code (me_vo_loop_*).
//
// The application loop around the hot path that pipeline.py's
// WindowedStereoVO + GPUBackend run in Python, step for step in C++ over the
// library's own entry points: KLT (me_klt_track), the epipolar MI matchers
// (me_mi_epipolar_match / me_vo_new_cells / me_mi_epipolar_match_count), the
// scale LM (me_scale_optimise) and the sliding-window BA queued behind the
// previous window (me_vo_window_submit / me_ba_wait_out).  The WBA_Point
// bookkeeping (include/MotionEstimation/core/feature_types.h:121-197) is a
// structure-of-arrays track table: IDs from the value constructor's counter
// (latestID++, :137-139), addMatch of contiguous frames (:140), pop() of the
// oldest feature (:142), empty tracks deleted; the BA window in
// initialiseObservations order (BundleAdjuster.h:354-376).  Host only: no
// kernels here.  The arithmetic of every host step is pipeline.py's, in the
// same order (rot_series / move_landmarks bit for bit with vo_chain_kernel).
#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "me_internal.hpp"

namespace {

constexpr int kPatch = 11;                // MI patch (11 x 11)
constexpr int kWScale = 5;                // ScaleState::window_size
constexpr int kMargin = 4 * kWScale + 4;  // feature margin (pipeline.MARGIN)
constexpr int kHalf = 6;                  // tracked features search +-6 px around the predicted disparity
constexpr double kRatio = 1.2;            // uniqueness ratio of new features

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// A one-job-at-a-time worker thread: submit() hands it a job, wait(seq)
// blocks until the job numbered seq (or a later one) has finished.
class Worker {
 public:
  ~Worker() {
    {
      std::lock_guard<std::mutex> lk(m_);
      quit_ = true;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
  }
  long submit(std::function<int()> f) {
    if (!th_.joinable()) th_ = std::thread([this] { run(); });
    std::unique_lock<std::mutex> lk(m_);
    // one job at a time: a job still pending or running is finished first
    // (its result code stays for the next wait), so queued_ never runs ahead
    // of a job that would be overwritten
    cv_.wait(lk, [&] { return done_ >= queued_; });
    job_ = std::move(f);
    has_ = true;
    ++queued_;
    cv_.notify_all();
    return queued_;
  }
  int wait(long seq) {
    std::unique_lock<std::mutex> lk(m_);
    cv_.wait(lk, [&] { return done_ >= seq; });
    const int r = rc_;
    rc_ = ME_OK;
    return r;
  }
  int wait_all() { return wait(queued_); }

 private:
  void run() {
    std::unique_lock<std::mutex> lk(m_);
    for (;;) {
      cv_.wait(lk, [&] { return has_ || quit_; });
      if (!has_) return;
      auto f = std::move(job_);
      has_ = false;
      lk.unlock();
      const int r = f();
      lk.lock();
      if (r != ME_OK && rc_ == ME_OK) rc_ = r;
      ++done_;
      cv_.notify_all();
    }
  }
  std::thread th_;
  std::mutex m_;
  std::condition_variable cv_;
  std::function<int()> job_;
  bool has_ = false, quit_ = false;
  long queued_ = 0, done_ = 0;
  int rc_ = ME_OK;
};

using Pose = std::array<double, 6>;
using Mat3 = std::array<double, 9>;

// synthetic.aa_to_R: Rodrigues, I + sin(th) [w]x + (1 - cos th) [w]x^2
Mat3 aa_to_R(const double* aa) {
  const double th = std::sqrt(aa[0] * aa[0] + aa[1] * aa[1] + aa[2] * aa[2]);
  Mat3 R{1, 0, 0, 0, 1, 0, 0, 0, 1};
  if (th < 1e-12) return R;
  const double w[3] = {aa[0] / th, aa[1] / th, aa[2] / th};
  const double W[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
  const double s = std::sin(th), c1 = 1 - std::cos(th);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double w2 = 0.0;
      for (int k = 0; k < 3; ++k) w2 += W[3 * i + k] * W[3 * k + j];
      R[3 * i + j] = (R[3 * i + j] + s * W[3 * i + j]) + c1 * w2;
    }
  return R;
}

// synthetic.R_to_quat: (w, x, y, z), w >= 0, through the trace angle-axis
std::array<double, 4> R_to_quat(const Mat3& R) {
  const double c = std::max(-1.0, std::min(1.0, ((R[0] + R[4] + R[8]) - 1) / 2));
  const double th = std::acos(c);
  if (th < 1e-12) return {1.0, 0.0, 0.0, 0.0};
  const double v[3] = {R[7] - R[5], R[2] - R[6], R[3] - R[1]};
  const double k = th / (2 * std::sin(th));
  const double aa[3] = {v[0] * k, v[1] * k, v[2] * k};
  const double n = std::sqrt(aa[0] * aa[0] + aa[1] * aa[1] + aa[2] * aa[2]);
  if (n < 1e-12) return {1.0, 0.0, 0.0, 0.0};
  const double s = std::sin(n / 2);
  return {std::cos(n / 2), aa[0] / n * s, aa[1] / n * s, aa[2] / n * s};
}

// pipeline.rot_series / vo_chain_kernel's rot_series: the same literals and order
const double kRotA[24] = {1.0, -0.16666666666666666, 0.008333333333333333, -0.0001984126984126984,
                          2.7557319223985893e-06, -2.505210838544172e-08, 1.6059043836821613e-10,
                          -7.647163731819816e-13, 2.8114572543455206e-15, -8.22063524662433e-18,
                          1.9572941063391263e-20, -3.868170170630684e-23, 6.446950284384474e-26,
                          -9.183689863795546e-29, 1.1309962886447716e-31, -1.216125041553518e-34,
                          1.151633562077195e-37, -9.67759295863189e-41, 7.265460179153071e-44,
                          -4.902469756513544e-47, 2.9893108271424046e-50, -1.6552108677421951e-53,
                          8.359650847182804e-57, -3.866628513960594e-60};
const double kRotB[24] = {0.5, -0.041666666666666664, 0.001388888888888889, -2.48015873015873e-05,
                          2.755731922398589e-07, -2.08767569878681e-09, 1.1470745597729725e-11,
                          -4.779477332387385e-14, 1.5619206968586225e-16, -4.110317623312165e-19,
                          8.896791392450574e-22, -1.6117375710961184e-24, 2.4795962632247976e-27,
                          -3.279889237069838e-30, 3.7699876288159054e-33, -3.8003907548547434e-36,
                          3.387157535521162e-39, -2.6882202662866363e-42, 1.911963205040282e-45,
                          -1.2256174391283858e-48, 7.117406731291439e-52, -3.7618428812322616e-55,
                          1.817315401561479e-58, -8.055476070751236e-62};
Mat3 rot_series(const double* a) {
  const double a0 = a[0], a1 = a[1], a2 = a[2];
  const double t2 = (a0 * a0 + a1 * a1) + a2 * a2;
  double A = kRotA[23], B = kRotB[23];
  for (int k = 22; k >= 0; --k) {
    A = A * t2 + kRotA[k];
    B = B * t2 + kRotB[k];
  }
  const double av[3] = {a0, a1, a2};
  const double K[9] = {0.0, -a2, a1, a2, 0.0, -a0, -a1, a0, 0.0};
  Mat3 R;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      const double k2 = av[i] * av[j] - (i == j ? t2 : 0.0);
      R[3 * i + j] = ((i == j ? 1.0 : 0.0) + A * K[3 * i + j]) + B * k2;
    }
  return R;
}

// pipeline.move_landmarks: x_c = R X + t, then R2^T (x_c - t2), elementwise in that order
void move_landmark(double* X, const Mat3& R, const Pose& pose, const Pose& pose2, const Mat3& R2) {
  double d[3];
  for (int k = 0; k < 3; ++k)
    d[k] = (((X[0] * R[3 * k] + X[1] * R[3 * k + 1]) + X[2] * R[3 * k + 2]) + pose[k]) - pose2[k];
  for (int k = 0; k < 3; ++k) X[k] = (d[0] * R2[k] + d[1] * R2[3 + k]) + d[2] * R2[6 + k];
}

// pipeline._cell_jitter: deterministic jitter in [-0.3, 0.3) per (frame, cell)
void cell_jitter(int t, int64_t cell, double* j) {
  uint64_t h = ((uint64_t)cell * 2654435761ull + (uint64_t)t * 40503ull) & 0xFFFFFFFFull;
  h ^= h >> 15;
  h = (h * 2246822519ull) & 0xFFFFFFFFull;
  const double a = (double)(h & 0xFFFF) / 65536.0, b = (double)((h >> 16) & 0xFFFF) / 65536.0;
  j[0] = a * 0.6 - 0.3;
  j[1] = b * 0.6 - 0.3;
}

struct Buf {
  void* p = nullptr;
  size_t n = 0;
};

}  // namespace

struct me_vo_loop {
  me_ctx* ctx = nullptr;   // BA
  me_ctx* tctx = nullptr;  // front end (KLT, matchers, scale LM)
  bool shared = false;
  me_vo_loop_config cfg{};
  std::string err;
  double f = 0, cx = 0, cy = 0;
  int nx = 1, ny = 1;
  double cw = 1, ch = 1;
  // ---- track table (index = creation order = ID order)
  std::vector<int64_t> ids, first, last;
  std::vector<double> X;  // 3 per track
  std::vector<uint8_t> active;
  int64_t latest_id = 0;
  int gen = 0;
  std::vector<int64_t> remap;  // the last compaction's index map (-1: deleted)
  struct FrameObs {
    std::vector<int64_t> ids;
    std::vector<float> feats;  // 4 per feature
  };
  std::map<int, FrameObs> obs;
  std::map<int, Pose> poses;
  Pose first_pose{};
  // ---- images (device pointers of the keyframes in use)
  struct Imgs {
    const uint8_t* L = nullptr;
    const uint8_t* R = nullptr;
  };
  std::map<int, Imgs> imgs;
  Buf img_slot[3];
  bool has_prev = false;
  int prev_t = -1;
  // ---- lagged state
  struct BaRec {
    int t = -1, f0 = 0;
    std::vector<int64_t> wids, upts;
    int nobs = 0, gen = 0;
  };
  struct Pending {
    int t, n_tracked, n_new, n_active;
    bool has_ba;
    BaRec ba;
  };
  bool has_pending = false;
  Pending pending{};
  bool has_scale_args = false;
  int scale_t = -1;
  std::vector<int64_t> scale_tids;
  // ---- scale LM call (kept alive while the worker runs it)
  std::vector<double> sc_X;
  std::vector<uint8_t> sc_tri;
  std::vector<uint32_t> sc_last;
  me_scale_state sc_s{};
  me_optim_params sc_p{};
  int sc_stop = 0, sc_it = 0;
  long sc_nmi = 0, sc_cnt[4] = {0, 0, 0, 0};
  std::vector<double> sc_trace = std::vector<double>(800);
  bool scale_queued = false;
  long scale_seq = 0;
  bool failed = false;  // a process() call returned an error: later calls are refused
  Worker scale_worker, ba_worker;
  // ---- results / events / stats
  std::vector<me_vo_frame_result> results;
  std::vector<me_vo_event> events;
  double host_s = 0, wait_s = 0, wait_stage[6] = {0, 0, 0, 0, 0, 0};
  // ---- persistent device / page-locked buffers (grow-only)
  std::map<std::string, Buf> dev, pin;
  // ---- device-resident BA window: obs (4 doubles) | frame | track ID per observation, frame by frame
  long wcap = 0, wend = 0;
  void* wstore[2] = {nullptr, nullptr};
  long wcaps[2] = {0, 0};
  int wcur = 0;
  std::map<int, std::pair<long, long>> wfrm;  // frame -> (offset, count)
  struct QSolve {
    me_ba_problem p{};
    me_ba_options o{};
    me_vo_window w{};
    int nc = 0, npts = 0;
    const int32_t* dev_ids = nullptr;
    int n_ids = 0;
    long seq = 0;  // worker job (0: queued inline)
  };
  std::deque<std::unique_ptr<QSolve>> baq;
  int bw_k = 0;
  long enq_seq = 0;  // newest queued worker job not yet joined (0: none)

  // ------------------------------------------------------------ helpers
  int fail(int rc, const char* what) {
    if (rc == ME_OK) return rc;
    const me_ctx* c = ctx;
    err = std::string(what) + ": " + (c ? me_last_error(c) : "");
    if (tctx && tctx != ctx) {
      const char* m2 = me_last_error(tctx);
      if (m2 && *m2) err += std::string(" | front: ") + m2;
    }
    return rc;
  }
#define VL_TRY(expr, what)                      \
  do {                                          \
    int rc_ = (expr);                           \
    if (rc_ != ME_OK) return fail(rc_, (what)); \
  } while (0)

  // Joins the worker threads before a buffer grows: the growth path
  // synchronises, frees and allocates on both contexts, which a worker may be
  // using (a ctx takes one call at a time).  reserve() sizes every
  // buffer for the configuration, so this is not expected after it.
  int quiesce() {
    if (scale_queued) {
      scale_queued = false;
      VL_TRY(scale_worker.wait(scale_seq), "me_scale_optimise");
    }
    if (enq_seq) {
      const long q = enq_seq;
      enq_seq = 0;
      VL_TRY(ba_worker.wait(q), "window submit");
    }
    return ME_OK;
  }
  int dbuf(const char* name, size_t nbytes, void** out) {
    Buf& b = dev[name];
    if (b.p == nullptr || b.n < nbytes) {
      VL_TRY(quiesce(), "grow");
      if (b.p) {
        VL_TRY(me_synchronize(tctx), "sync");
        VL_TRY(me_synchronize(ctx), "sync");
        VL_TRY(me_free(tctx, b.p), "free");
        b.p = nullptr;
      }
      const size_t nb = std::max<size_t>(4096, (size_t)(nbytes * 1.5));
      VL_TRY(me_malloc(tctx, &b.p, nb), "malloc");
      b.n = nb;
    }
    *out = b.p;
    return ME_OK;
  }
  int hbuf(const char* name, size_t nbytes, void** out) {
    Buf& b = pin[name];
    if (b.p == nullptr || b.n < nbytes) {
      VL_TRY(quiesce(), "grow");
      if (b.p) {
        VL_TRY(me_synchronize(tctx), "sync");
        VL_TRY(me_synchronize(ctx), "sync");
        VL_TRY(me_host_free(tctx, b.p), "host_free");
        b.p = nullptr;
      }
      const size_t nb = std::max<size_t>(4096, (size_t)(nbytes * 1.5));
      VL_TRY(me_host_alloc(tctx, &b.p, nb), "host_alloc");
      b.n = nb;
    }
    *out = b.p;
    return ME_OK;
  }
  template <class F>
  int timed_wait(int stage, F&& fn) {
    const double t0 = now_s();
    const int rc = fn();
    const double dt = now_s() - t0;
    wait_s += dt;
    wait_stage[stage] += dt;
    return rc;
  }
  size_t ntab() const { return ids.size(); }
  int64_t find_id(int64_t id) const {  // searchsorted in the ascending ID column
    return std::lower_bound(ids.begin(), ids.end(), id) - ids.begin();
  }

  // ------------------------------------------------------------ setup
  int init(const me_vo_loop_config& c) {
    cfg = c;
    f = cfg.K[0];
    cx = cfg.K[2];
    cy = cfg.K[5];
    const double aw = cfg.width - 2 * kMargin, ah = cfg.height - 2 * kMargin;
    nx = std::max(1, (int)std::nearbyint(std::sqrt(cfg.n_feats * aw / ah)));
    ny = std::max(1, (int)std::ceil((double)cfg.n_feats / nx));
    cw = aw / nx;
    ch = ah / ny;
    for (int k = 0; k < 6; ++k) first_pose[k] = cfg.first_pose[k];
    shared = ctx == tctx;
    if (shared) cfg.async_enqueue = 0;
    return reserve();
  }
  // GPUBackend.reserve: the BA side sized for the configuration's fullest window up front
  int reserve() {
    const long n_obs = (long)cfg.window * cfg.n_feats + cfg.n_feats;
    const long n_pts = n_obs;
    const int nc = cfg.window;
    const long cap = 2 * n_obs;
    if (wend == 0 && wcap < cap) {
      for (int k = 0; k < 2; ++k) {
        if (wstore[k]) VL_TRY(me_free(ctx, wstore[k]), "free");
        wstore[k] = nullptr;
        VL_TRY(me_malloc(ctx, &wstore[k], 40 * cap), "malloc");
        wcaps[k] = cap;
      }
      wcap = cap;
    }
    const size_t nb = 48 * nc + 24 * n_pts + 4 * n_pts + 4 * nc;
    void* q;
    for (int k = 0; k < 2; ++k) {
      const std::string s = "bw" + std::to_string(k);
      VL_TRY(hbuf(s.c_str(), nb, &q), "reserve");
      VL_TRY(dbuf(s.c_str(), nb, &q), "reserve");
      VL_TRY(dbuf(("bw_idx" + std::to_string(k)).c_str(), 8 * n_obs, &q), "reserve");
    }
    for (int k = 0; k < 2; ++k) VL_TRY(hbuf(("w_add" + std::to_string(k)).c_str(), 40 * cfg.n_feats, &q), "reserve");
    VL_TRY(me_ba_reserve(ctx, nc, (int)n_pts, (int)n_obs, 4, cfg.fixed_frames), "me_ba_reserve");
    return ME_OK;
  }
  int close() {
    int rc = ME_OK;
    if (scale_queued) {
      scale_worker.wait(scale_seq);
      scale_queued = false;
    }
    if (enq_seq) ba_worker.wait(enq_seq);
    enq_seq = 0;
    while (!baq.empty()) {
      std::vector<double> c, p;
      me_ba_summary s;
      const int r = ba_result(c, p, s);
      if (rc == ME_OK) rc = r;
    }
    me_synchronize(tctx);
    me_synchronize(ctx);
    for (auto& w : wstore)
      if (w) me_free(ctx, w);
    for (auto& b : img_slot)
      if (b.p) me_free(tctx, b.p);
    for (auto& kv : dev) me_free(tctx, kv.second.p);
    for (auto& kv : pin) me_host_free(tctx, kv.second.p);
    dev.clear();
    pin.clear();
    return rc;
  }

  // ------------------------------------------------------------ loop steps (pipeline.py)
  Pose predict_pose(int t) {
    if (t == 0) return first_pose;
    const Pose& p1 = poses[t - 1];
    Pose v{};
    if (t == 1 || !poses.count(t - 2)) {
      if (cfg.has_velocity)
        for (int k = 0; k < 6; ++k) v[k] = cfg.velocity[k];
    } else {
      const Pose& p2 = poses[t - 2];
      for (int k = 0; k < 6; ++k) v[k] = p1[k] - p2[k];
    }
    Pose out;
    for (int k = 0; k < 6; ++k) out[k] = p1[k] + v[k];
    return out;
  }
  bool in_margin(float u, float v) const {
    return u >= kMargin && u < cfg.width - kMargin && v >= kMargin && v < cfg.height - kMargin;
  }
  // new_cells on the host (first keyframe: no tracked features)
  void new_cells_host(int t, int n_good, const float* uv_good, std::vector<float>& out) {
    std::vector<uint8_t> occ((size_t)nx * ny, 0);
    for (int i = 0; i < n_good; ++i) {
      long ccx = (long)(((double)uv_good[2 * i] - kMargin) / cw), ccy = (long)(((double)uv_good[2 * i + 1] - kMargin) / ch);
      ccx = std::min<long>(std::max<long>(ccx, 0), nx - 1);
      ccy = std::min<long>(std::max<long>(ccy, 0), ny - 1);
      occ[ccy * nx + ccx] = 1;
    }
    const long want = std::max(0, cfg.n_feats - n_good);
    out.clear();
    for (long cell = 0; cell < (long)occ.size() && (long)out.size() / 2 < want; ++cell) {
      if (occ[cell]) continue;
      double j[2];
      cell_jitter(t, cell, j);
      out.push_back((float)(kMargin + (((double)(cell % nx) + 0.5) + j[0]) * cw));
      out.push_back((float)(kMargin + (((double)(cell / nx) + 0.5) + j[1]) * ch));
    }
  }
  void triangulate(float u, float v, float xr, const Pose& pose, const Mat3& R, double* Xo) const {
    const double disp = (double)u - (double)xr;
    const double Z = f * cfg.baseline / disp;
    const double pc[3] = {((double)u - cx) * Z / f, ((double)v - cy) * Z / f, Z};
    for (int j = 0; j < 3; ++j) {
      double s = 0.0;
      for (int i = 0; i < 3; ++i) s += (pc[i] - pose[i]) * R[3 * i + j];
      Xo[j] = s;
    }
  }

  int frame_images(int t, const uint8_t* L, const uint8_t* R, me_mem mem) {
    if (imgs.count(t)) return ME_OK;
    Imgs im;
    if (mem == ME_DEVICE) {
      im.L = L;
      im.R = R;
    } else {
      const size_t nb = (size_t)cfg.width * cfg.height;
      Buf& b = img_slot[t % 3];
      if (b.p == nullptr) {
        VL_TRY(me_malloc(tctx, &b.p, 2 * nb), "malloc");
        b.n = 2 * nb;
      }
      VL_TRY(me_memcpy_async(tctx, b.p, L, nb), "image upload");
      VL_TRY(me_memcpy_async(tctx, (uint8_t*)b.p + nb, R, nb), "image upload");
      im.L = (const uint8_t*)b.p;
      im.R = (const uint8_t*)b.p + nb;
    }
    imgs[t] = im;
    return ME_OK;
  }

  // ---- front end
  int klt_submit(const Imgs& prev, const Imgs& cur, const std::vector<float>& pts) {
    const int n = (int)pts.size() / 2;
    void *hp, *d_in, *dres;
    VL_TRY(hbuf("klt_in", 8 * (size_t)n, &hp), "klt");
    std::memcpy(hp, pts.data(), 8 * (size_t)n);
    VL_TRY(dbuf("klt_in", 8 * (size_t)n, &d_in), "klt");
    VL_TRY(dbuf("res", 14 * (size_t)n, &dres), "klt");
    VL_TRY(me_memcpy_async(tctx, d_in, hp, 8 * (size_t)n), "klt H2D");
    me_klt_params kp;
    me_klt_default_params(&kp);
    VL_TRY(me_klt_track(tctx, ME_DEVICE, prev.L, cur.L, cfg.width, cfg.height, cfg.width, (const float*)d_in,
                        (float*)dres, (uint8_t*)dres + 12 * (size_t)n, n, &kp),
           "me_klt_track");
    return ME_OK;
  }
  // GPUBackend.klt_match_new: tracked features' matcher, the cells they leave
  // empty, the new features' matcher -- one submission, one round trip
  int klt_match_new(int n, const Imgs& im, const std::vector<int32_t>& lo, const std::vector<uint8_t>& dvalid, int t,
                    int nd, int nd_new, std::vector<float>& uv, std::vector<uint8_t>& st, std::vector<float>& xr,
                    std::vector<uint8_t>& ok, std::vector<float>& nuv, std::vector<float>& nxr,
                    std::vector<uint8_t>& nok) {
    void *hp, *dl, *dres, *dn, *ho;
    VL_TRY(hbuf("lo", 5 * (size_t)n, &hp), "match");
    std::memcpy(hp, lo.data(), 4 * (size_t)n);
    std::memcpy((uint8_t*)hp + 4 * (size_t)n, dvalid.data(), n);
    VL_TRY(dbuf("lo", 5 * (size_t)n, &dl), "match");
    VL_TRY(me_memcpy_async(tctx, dl, hp, 5 * (size_t)n), "match H2D");
    VL_TRY(dbuf("res", 14 * (size_t)n, &dres), "match");
    uint8_t* r8 = (uint8_t*)dres;
    VL_TRY(me_mi_epipolar_match(tctx, im.L, im.R, cfg.width, cfg.height, cfg.width, (const float*)dres,
                                (const int32_t*)dl, (const uint8_t*)dl + 4 * (size_t)n, r8 + 12 * (size_t)n, n, nd,
                                kPatch, cfg.d_max, 0, kRatio, (float)kMargin, (float*)(r8 + 8 * (size_t)n),
                                r8 + 13 * (size_t)n),
           "me_mi_epipolar_match");
    const int m = std::max(cfg.n_feats, 1);
    VL_TRY(dbuf("new", 16 + 17 * (size_t)m, &dn), "match");
    uint8_t* n8 = (uint8_t*)dn;
    VL_TRY(me_vo_new_cells(tctx, (const float*)dres, r8 + 12 * (size_t)n, r8 + 13 * (size_t)n, n, cfg.width,
                           cfg.height, (float)kMargin, nx, ny, cw, ch, cfg.n_feats, t, cfg.d_min,
                           (float*)(n8 + 16), (int32_t*)(n8 + 16 + 12 * (size_t)m), (int32_t*)n8),
           "me_vo_new_cells");
    VL_TRY(me_mi_epipolar_match_count(tctx, im.L, im.R, cfg.width, cfg.height, cfg.width, (const float*)(n8 + 16),
                                      (const int32_t*)(n8 + 16 + 12 * (size_t)m), (const int32_t*)n8, m, nd_new,
                                      kPatch, cfg.d_max, 1, kRatio, (float)kMargin,
                                      (float*)(n8 + 16 + 8 * (size_t)m), n8 + 16 + 16 * (size_t)m),
           "me_mi_epipolar_match_count");
    const size_t o = 16 * ((14 * (size_t)n + 15) / 16);
    VL_TRY(hbuf("out", o + 16 + 17 * (size_t)m, &ho), "match");
    VL_TRY(me_memcpy_async(tctx, ho, dres, 14 * (size_t)n), "match D2H");
    VL_TRY(me_memcpy_async(tctx, (uint8_t*)ho + o, dn, 16 + 17 * (size_t)m), "match D2H");
    VL_TRY(timed_wait(0, [&] { return me_synchronize(tctx); }), "klt_match_new");
    const uint8_t* h8 = (const uint8_t*)ho;
    uv.assign((const float*)h8, (const float*)h8 + 2 * (size_t)n);
    xr.assign((const float*)(h8 + 8 * (size_t)n), (const float*)(h8 + 8 * (size_t)n) + n);
    st.assign(h8 + 12 * (size_t)n, h8 + 13 * (size_t)n);
    ok.assign(h8 + 13 * (size_t)n, h8 + 14 * (size_t)n);
    int k = *(const int32_t*)(h8 + o);
    k = std::max(0, std::min(k, m));
    const uint8_t* nb = h8 + o + 16;
    nuv.assign((const float*)nb, (const float*)nb + 2 * (size_t)k);
    nxr.assign((const float*)(nb + 8 * (size_t)m), (const float*)(nb + 8 * (size_t)m) + k);
    nok.assign(nb + 16 * (size_t)m, nb + 16 * (size_t)m + k);
    return ME_OK;
  }
  // GPUBackend.match: the first keyframe's new features (uniqueness test)
  int match(const Imgs& im, const std::vector<float>& uv, int nd, std::vector<float>& xr, std::vector<uint8_t>& ok) {
    const int n = (int)uv.size() / 2;
    xr.assign(n, 0.0f);
    ok.assign(n, 0);
    if (n == 0) return ME_OK;
    void *hp, *d, *ho;
    VL_TRY(hbuf("m_in", 12 * (size_t)n, &hp), "match");
    std::memcpy(hp, uv.data(), 8 * (size_t)n);
    int32_t* lo = (int32_t*)((uint8_t*)hp + 8 * (size_t)n);
    for (int i = 0; i < n; ++i) lo[i] = cfg.d_min;
    VL_TRY(dbuf("m", 17 * (size_t)n, &d), "match");
    VL_TRY(me_memcpy_async(tctx, d, hp, 12 * (size_t)n), "match H2D");
    uint8_t* d8 = (uint8_t*)d;
    VL_TRY(me_mi_epipolar_match(tctx, im.L, im.R, cfg.width, cfg.height, cfg.width, (const float*)d,
                                (const int32_t*)(d8 + 8 * (size_t)n), nullptr, nullptr, n, nd, kPatch, cfg.d_max, 1,
                                kRatio, (float)kMargin, (float*)(d8 + 12 * (size_t)n), d8 + 16 * (size_t)n),
           "me_mi_epipolar_match");
    VL_TRY(hbuf("m_out", 5 * (size_t)n, &ho), "match");
    VL_TRY(me_memcpy_async(tctx, ho, d8 + 12 * (size_t)n, 5 * (size_t)n), "match D2H");
    VL_TRY(timed_wait(1, [&] { return me_synchronize(tctx); }), "match");
    std::memcpy(xr.data(), ho, 4 * (size_t)n);
    std::memcpy(ok.data(), (uint8_t*)ho + 4 * (size_t)n, n);
    return ME_OK;
  }

  // ---- scale LM (Optimiser<ScaleState,...>::optimise over the tracks seen in t, images of t)
  int scale_submit(int t, const std::vector<int64_t>& tids) {
    if (scale_queued) {  // a scale job left queued by an earlier error return: it reads sc_s / sc_X
      scale_queued = false;
      VL_TRY(scale_worker.wait(scale_seq), "me_scale_optimise");
    }
    const size_t n = tids.size();
    const Pose& pose = poses[t];
    const Mat3 R = aa_to_R(&pose[3]);
    const auto q = R_to_quat(R);
    sc_X.resize(4 * n);
    sc_tri.assign(n, 1);
    sc_last.assign(n, (uint32_t)t);
    for (size_t i = 0; i < n; ++i) {
      const int64_t j = find_id(tids[i]);
      for (int k = 0; k < 3; ++k) sc_X[4 * i + k] = X[3 * j + k];
      sc_X[4 * i + 3] = 1.0;
    }
    me_scale_state& s = sc_s;
    s = me_scale_state{};
    s.n_left = (int)n;
    s.n_right = 0;
    s.X_left = sc_X.data();
    s.X_right = sc_X.data();
    s.tri_left = sc_tri.data();
    s.tri_right = sc_tri.data();
    s.last_left = sc_last.data();
    s.last_right = sc_last.data();
    s.lframe = (uint32_t)t;
    for (int k = 0; k < 9; ++k) s.K1[k] = s.K2[k] = cfg.K[k];
    for (int k = 0; k < 4; ++k) s.q1[k] = s.q2[k] = q[k];
    for (int k = 0; k < 3; ++k) s.t1[k] = s.t2[k] = pose[k];
    s.scale = 1.0;
    s.baseline = cfg.baseline;
    s.window_size = kWScale;
    const Imgs& im = imgs[t];
    s.imgL = im.L;
    s.imgR = im.R;
    s.stride = s.cols = cfg.width;
    s.rows = cfg.height;
    s.bb_cols = cfg.width;
    s.bb_rows = cfg.height;
    s.mask = nullptr;
    s.mask_len = 0;
    s.img_mem = ME_DEVICE;
    s.tracks_mem = ME_HOST;
    me_optim_params& p = sc_p;
    p.type = 1;
    p.minim = 1;
    p.max_nb_iter = cfg.scale_iters;
    p.v = 2.0;
    p.tau = 1e-3;
    p.mu = 1e-20;
    p.abs_tol = p.grad_tol = p.incr_tol = p.rel_tol = 0.0;
    p.alpha = 1.0;
    p.weighting = 0;
    auto run = [this]() -> int {
      int rc = me_scale_optimise(tctx, &sc_s, &sc_p, 0, &sc_stop, &sc_it, sc_trace.data(), 400, &sc_nmi);
      if (rc == ME_OK) rc = me_scale_last_counters(tctx, &sc_cnt[0], &sc_cnt[1], &sc_cnt[2], &sc_cnt[3]);
      return rc;
    };
    if (shared) {  // (one context: no second caller -- run it now, in loop order)
      if (enq_seq) {
        VL_TRY(ba_worker.wait(enq_seq), "window submit");
        enq_seq = 0;
      }
      VL_TRY(timed_wait(2, run), "me_scale_optimise");
      scale_queued = false;
      return ME_OK;
    }
    scale_seq = scale_worker.submit(run);
    scale_queued = true;
    return ME_OK;
  }
  int scale_result(double* scale, int* stop, int* iters) {
    if (scale_queued) {
      VL_TRY(timed_wait(5, [&] { return scale_worker.wait(scale_seq); }), "me_scale_optimise");
      scale_queued = false;
    }
    *scale = sc_s.scale;
    *stop = sc_stop;
    *iters = sc_it;
    return ME_OK;
  }

  // ---- device-resident BA window (GPUBackend.window_add / ba_submit_window / ba_result)
  void wview(int k, uint8_t** o, uint8_t** fr, uint8_t** id) {
    uint8_t* base = (uint8_t*)wstore[k];
    *o = base;
    *fr = base + 32 * wcap;
    *id = base + 36 * wcap;
  }
  int join_enqueue() {
    if (enq_seq) {
      const long s = enq_seq;
      enq_seq = 0;
      VL_TRY(ba_worker.wait(s), "me_vo_window_submit");
    }
    return ME_OK;
  }
  int window_add(int t, const std::vector<int64_t>& fid, const std::vector<float>& feats) {
    VL_TRY(join_enqueue(), "window");
    const long n = (long)fid.size();
    long live0 = wend;
    for (auto& kv : wfrm) live0 = std::min(live0, kv.second.first);
    const long live = wend - live0;
    if (wend + n > wcap) {
      long cap = std::max<long>(std::max<long>(1L << 16, 2 * (live + n)), wcap);
      const int k = 1 - wcur;
      if (wcaps[k] < cap) {
        if (wstore[k]) VL_TRY(me_free(ctx, wstore[k]), "free");
        wstore[k] = nullptr;
        VL_TRY(me_malloc(ctx, &wstore[k], 40 * cap), "malloc");
        wcaps[k] = cap;
      }
      cap = wcaps[k];
      const long old = wcap;
      if (live) {
        uint8_t* src = (uint8_t*)wstore[wcur];
        wcap = cap;
        uint8_t *no, *nf, *ni;
        wview(k, &no, &nf, &ni);
        VL_TRY(me_memcpy_d2d(ctx, no, src + 32 * live0, 32 * live), "window compaction");
        VL_TRY(me_memcpy_d2d(ctx, nf, src + 32 * old + 4 * live0, 4 * live), "window compaction");
        VL_TRY(me_memcpy_d2d(ctx, ni, src + 36 * old + 4 * live0, 4 * live), "window compaction");
      }
      wcap = cap;
      wcur = k;
      for (auto& kv : wfrm) kv.second.first -= live0;
      wend = live;
    }
    if (n) {
      void* hp;
      VL_TRY(hbuf((std::string("w_add") + std::to_string(t & 1)).c_str(), 40 * (size_t)n, &hp), "window");
      double* ho = (double*)hp;
      for (long i = 0; i < 4 * n; ++i) ho[i] = (double)feats[i];
      int32_t* hf = (int32_t*)((uint8_t*)hp + 32 * n);
      int32_t* hi = (int32_t*)((uint8_t*)hp + 36 * n);
      for (long i = 0; i < n; ++i) {
        hf[i] = t;
        hi[i] = (int32_t)fid[i];
      }
      uint8_t *o, *fr, *id;
      wview(wcur, &o, &fr, &id);
      const long e = wend;
      VL_TRY(me_memcpy_async(ctx, o + 32 * e, hp, 32 * n), "window H2D");
      VL_TRY(me_memcpy_async(ctx, fr + 4 * e, (uint8_t*)hp + 32 * n, 4 * n), "window H2D");
      VL_TRY(me_memcpy_async(ctx, id + 4 * e, (uint8_t*)hp + 36 * n, 4 * n), "window H2D");
    }
    wfrm[t] = {wend, n};
    wend += n;
    return ME_OK;
  }
  struct Chain {
    std::vector<int32_t> cam_src;
    int32_t new_from;
    me_vo_chain_args a;
    int nc;
  };
  int ba_submit_window(int t, int f0, const std::vector<int32_t>& win_ids, const std::vector<double>& Xw,
                       const std::vector<Pose>& cams, const Chain* chain, int* n_obs_out) {
    VL_TRY(join_enqueue(), "window");
    const long off0 = wfrm[f0].first;
    const long n_obs = wend - off0;
    const int npts = (int)win_ids.size(), nc = (int)cams.size();
    const int k = bw_k;
    bw_k ^= 1;
    const size_t o_ids = 48 * (size_t)nc + 24 * (size_t)npts, o_cs = o_ids + 4 * (size_t)npts,
                 nb = o_cs + 4 * (size_t)nc;
    void *hp, *d, *di;
    VL_TRY(hbuf(("bw" + std::to_string(k)).c_str(), nb, &hp), "window");
    uint8_t* h8 = (uint8_t*)hp;
    for (int c = 0; c < nc; ++c) std::memcpy(h8 + 48 * (size_t)c, cams[c].data(), 48);
    std::memcpy(h8 + 48 * (size_t)nc, Xw.data(), 24 * (size_t)npts);
    std::memcpy(h8 + o_ids, win_ids.data(), 4 * (size_t)npts);
    VL_TRY(dbuf(("bw" + std::to_string(k)).c_str(), nb, &d), "window");
    VL_TRY(dbuf(("bw_idx" + std::to_string(k)).c_str(), 8 * (size_t)std::max<long>(n_obs, 1), &di), "window");
    auto q = std::make_unique<QSolve>();
    me_vo_window& w = q->w;
    w = me_vo_window{};
    w.stage = hp;
    w.dev = d;
    w.stage_bytes = chain ? nb : o_cs;
    uint8_t* d8 = (uint8_t*)d;
    if (chain) {
      if (chain->nc != nc || baq.empty()) return fail(ME_ERR_STATE, "chain without a queued window");
      std::memcpy(h8 + o_cs, chain->cam_src.data(), 4 * (size_t)nc);
      const QSolve& prev = *baq.back();
      w.chain = 1;
      w.cam_src = (const int32_t*)(d8 + o_cs);
      w.prev_ids = prev.dev_ids;
      w.n_prev = prev.n_ids;
      w.new_from = chain->new_from;
      w.args = chain->a;
    }
    uint8_t *o, *fr, *id;
    wview(wcur, &o, &fr, &id);
    w.win_ids = (const int32_t*)(d8 + o_ids);
    w.frame = (const int32_t*)(fr + 4 * off0);
    w.ids = (const int32_t*)(id + 4 * off0);
    w.first_frame = f0;
    me_ba_problem& p = q->p;
    p = me_ba_problem{};
    p.n_cams = nc;
    p.n_pts = npts;
    p.n_obs = (int)n_obs;
    p.cams = (double*)d8;
    p.pts = (double*)(d8 + 48 * (size_t)nc);
    p.obs = (const double*)(o + 32 * off0);
    p.cam_idx = (const int32_t*)di;
    p.pt_idx = (const int32_t*)((uint8_t*)di + 4 * (size_t)n_obs);
    for (int i = 0; i < 9; ++i) p.K0[i] = p.K1[i] = cfg.K[i];
    p.baseline = cfg.baseline;
    p.feat_var = cfg.feat_var;
    p.fixed_frames = cfg.fixed_frames;
    p.mem = ME_DEVICE;
    p.obs_dim = 4;
    me_ba_default_options(&q->o);
    q->o.max_num_iterations = cfg.ba_iters;
    q->o.function_tolerance = q->o.gradient_tolerance = q->o.parameter_tolerance = 0.0;
    q->nc = nc;
    q->npts = npts;
    q->dev_ids = (const int32_t*)(d8 + o_ids);
    q->n_ids = npts;
    QSolve* qp = q.get();
    auto enqueue = [this, qp]() -> int { return me_vo_window_submit(ctx, &qp->w, &qp->p, &qp->o); };
    if (cfg.async_enqueue) {
      // queued by the worker (the loop thread goes on to wait for the
      // previous window: me_ba_wait_out may run beside the queueing)
      q->seq = enq_seq = ba_worker.submit(enqueue);
    } else {
      VL_TRY(timed_wait(3, enqueue), "me_vo_window_submit");
    }
    baq.push_back(std::move(q));
    *n_obs_out = (int)n_obs;
    return ME_OK;
  }
  int ba_result(std::vector<double>& cams, std::vector<double>& pts, me_ba_summary& s) {
    if (baq.empty()) return fail(ME_ERR_STATE, "no window solve queued");
    std::unique_ptr<QSolve> q = std::move(baq.front());
    baq.pop_front();
    if (q->seq) {  // this window's own queueing (a newer one's may run on beside the wait)
      VL_TRY(ba_worker.wait(q->seq), "me_vo_window_submit");
      if (enq_seq == q->seq) enq_seq = 0;
    }
    cams.assign(6 * (size_t)q->nc, 0.0);
    pts.assign(3 * (size_t)q->npts, 0.0);
    VL_TRY(timed_wait(4, [&] { return me_ba_wait_out(ctx, &s, cams.data(), pts.data()); }), "me_ba_wait_out");
    return ME_OK;
  }

  // ---- WindowedStereoVO steps
  bool chain_args(int t, const Pose& pose, const Mat3& R_pose, const std::vector<int64_t>& new_ids, Chain& ch) {
    if (!has_pending || !pending.has_ba) return false;
    const int f0 = std::max(0, t - cfg.window + 1);
    if (t - f0 + 1 <= cfg.fixed_frames) return false;
    const int pt = pending.ba.t, pf0 = pending.ba.f0;
    const int nc = t - f0 + 1, k1 = t - 1 - f0;
    int mode, k0;
    double vel[6] = {0, 0, 0, 0, 0, 0};
    if (t == 1 || !poses.count(t - 2)) {
      mode = 0;
      k0 = -1;
      if (cfg.has_velocity)
        for (int k = 0; k < 6; ++k) vel[k] = cfg.velocity[k];
    } else if (t - 2 >= f0) {
      mode = 1;
      k0 = t - 2 - f0;
    } else {
      return false;
    }
    if (k1 < 0 || pt != t - 1) return false;
    ch.cam_src.clear();
    for (int fr = f0; fr < t; ++fr) ch.cam_src.push_back(pf0 <= fr && fr <= pt ? fr - pf0 : -1);
    ch.cam_src.push_back(-1);
    ch.new_from = new_ids.empty() ? (int32_t)2147483647 : (int32_t)new_ids[0];
    for (int k = 0; k < 6; ++k) ch.a.pose[k] = pose[k];
    for (int k = 0; k < 9; ++k) ch.a.R[k] = R_pose[k];
    for (int k = 0; k < 6; ++k) ch.a.vel[k] = vel[k];
    ch.a.k1 = k1;
    ch.a.k0 = k0;
    ch.a.mode = mode;
    ch.nc = nc;
    return true;
  }
  int ba_submit(int t, const Chain* chain, bool* has, BaRec* rec) {
    *has = false;
    const int f0 = std::max(0, t - cfg.window + 1);
    if (t - f0 + 1 <= cfg.fixed_frames) return ME_OK;
    rec->t = t;
    rec->f0 = f0;
    rec->upts.clear();
    rec->wids.clear();
    std::vector<int32_t> wid32;
    std::vector<double> Xw;
    for (size_t i = 0; i < ntab(); ++i)
      if (last[i] >= f0) {
        rec->upts.push_back((int64_t)i);
        rec->wids.push_back(ids[i]);
        if (ids[i] >= 2147483647LL) return fail(ME_ERR_STATE, "track IDs exceed the device window's int32");
        wid32.push_back((int32_t)ids[i]);
        Xw.insert(Xw.end(), &X[3 * i], &X[3 * i] + 3);
      }
    std::vector<Pose> cams;
    for (int fr = f0; fr <= t; ++fr) cams.push_back(poses[fr]);
    VL_TRY(ba_submit_window(t, f0, wid32, Xw, cams, chain, &rec->nobs), "window");
    rec->gen = gen;
    *has = true;
    return ME_OK;
  }
  int ba_finish(bool has, const BaRec& ba, int* nwp, int* nwo, int* iters, double* cost) {
    if (!has) {
      *nwp = *nwo = *iters = 0;
      *cost = std::numeric_limits<double>::quiet_NaN();
      return ME_OK;
    }
    std::vector<double> c, p;
    me_ba_summary s;
    VL_TRY(ba_result(c, p, s), "BA result");
    const size_t m = ba.upts.size();
    std::vector<int64_t> j(m);
    std::vector<uint8_t> live(m, 1);
    if (ba.gen == gen) {
      for (size_t i = 0; i < m; ++i) j[i] = ba.upts[i];
    } else if (ba.gen + 1 == gen) {
      for (size_t i = 0; i < m; ++i) {
        const int64_t r = remap[ba.upts[i]];
        live[i] = r >= 0;
        j[i] = std::max<int64_t>(r, 0);
      }
    } else {  // (not reached by the loop: one pop at most between a window's submit and its result)
      for (size_t i = 0; i < m; ++i) {
        const int64_t r = std::min<int64_t>(find_id(ba.wids[i]), std::max<int64_t>((int64_t)ntab() - 1, 0));
        live[i] = ntab() > 0 && ids[r] == ba.wids[i];
        j[i] = r;
      }
    }
    if (s.status == 2) {
      for (int k = 0, fr = ba.f0; fr <= ba.t; ++fr, ++k)
        for (int q = 0; q < 6; ++q) poses[fr][q] = c[6 * (size_t)k + q];
      for (size_t i = 0; i < m; ++i)
        if (live[i])
          for (int q = 0; q < 3; ++q) X[3 * j[i] + q] = p[3 * i + q];
    }
    *nwp = (int)ba.wids.size();
    *nwo = ba.nobs;
    *iters = s.iterations;
    *cost = s.final_cost;
    return ME_OK;
  }
  void pop(int new_first) {
    while (!obs.empty() && obs.begin()->first < new_first) {
      auto it = obs.begin();
      const int fr = it->first;
      if (cfg.log_events)
        for (int64_t id : it->second.ids) events.push_back(me_vo_event{2, fr, id, {0, 0, 0, 0}});
      obs.erase(it);
      wfrm.erase(fr);  // window_pop
      for (auto& x : first)
        if (x == fr) x = fr + 1;
    }
    std::vector<uint8_t> keep(ntab());
    size_t n2 = 0;
    for (size_t i = 0; i < ntab(); ++i) {
      keep[i] = !(last[i] < new_first);
      n2 += keep[i];
    }
    if (n2 == ntab()) return;
    if (cfg.log_events)
      for (size_t i = 0; i < ntab(); ++i)
        if (!keep[i]) events.push_back(me_vo_event{3, -1, ids[i], {0, 0, 0, 0}});
    remap.assign(ntab(), -1);
    size_t w = 0;
    for (size_t i = 0; i < ntab(); ++i) {
      if (!keep[i]) continue;
      remap[i] = (int64_t)w;
      ids[w] = ids[i];
      first[w] = first[i];
      last[w] = last[i];
      active[w] = active[i];
      for (int q = 0; q < 3; ++q) X[3 * w + q] = X[3 * i + q];
      ++w;
    }
    ids.resize(n2);
    first.resize(n2);
    last.resize(n2);
    active.resize(n2);
    X.resize(3 * n2);
    ++gen;
  }
  int complete_result(bool have, int t, int n_tracked, int n_new, int n_active, int nwp, int nwo, int ba_iters,
                      double cost) {
    if (!have) return ME_OK;
    me_vo_frame_result r{};
    VL_TRY(scale_result(&r.scale, &r.scale_stop, &r.scale_iters), "scale");
    r.t = t;
    r.n_tracked = n_tracked;
    r.n_new = n_new;
    r.n_active = n_active;
    r.n_window_pts = nwp;
    r.n_window_obs = nwo;
    r.ba_iters = ba_iters;
    r.ba_cost = cost;
    for (int k = 0; k < 6; ++k) r.pose[k] = poses[t][k];
    results.push_back(r);
    return ME_OK;
  }

  // pipeline.WindowedStereoVO.process (the steps are numbered as there)
  int process(int t, const uint8_t* left, const uint8_t* right, me_mem mem) {
    const double t_in = now_s();
    const double w0 = wait_s;
    VL_TRY(frame_images(t, left, right, mem), "images");
    const Imgs im = imgs[t];
    // 1. KLT of the active tracks, queued first (it needs only frame t-1's features)
    std::vector<int64_t> act;
    for (size_t i = 0; i < ntab(); ++i)
      if (active[i]) act.push_back((int64_t)i);
    const bool klt = has_prev && !act.empty();
    if (klt) {
      const FrameObs& po = obs[prev_t];
      std::vector<float> pts(2 * act.size());
      const bool same = po.ids.size() == act.size() &&
                        std::equal(act.begin(), act.end(), po.ids.begin(), [&](int64_t a, int64_t pid) { return ids[a] == pid; });
      for (size_t k = 0; k < act.size(); ++k) {
        const size_t pos =
            same ? k : (size_t)(std::lower_bound(po.ids.begin(), po.ids.end(), ids[act[k]]) - po.ids.begin());
        pts[2 * k] = po.feats[4 * pos];
        pts[2 * k + 1] = po.feats[4 * pos + 1];
      }
      VL_TRY(klt_submit(imgs[prev_t], im, pts), "klt");
    }
    // 2. pops of frame t-1's completion
    if (has_pending) pop(pending.t + 1 - cfg.window);
    // 3. prediction from the lagged state
    const Pose pose = predict_pose(t);
    poses[t] = pose;
    const int nd_new = cfg.d_max - cfg.d_min + 1;
    std::vector<int64_t> trk_idx;
    std::vector<float> trk_uv, xr_trk, nuv, nxr;
    std::vector<uint8_t> nok;
    if (klt) {
      // 4. KLT gate + matching of the tracked features around their predicted disparity, the new
      // features of the cells they leave empty -- one round trip
      act.clear();
      for (size_t i = 0; i < ntab(); ++i)
        if (active[i]) act.push_back((int64_t)i);
      const int n = (int)act.size();
      const Mat3 R = aa_to_R(&pose[3]);
      std::vector<int32_t> lo(n);
      std::vector<uint8_t> dvalid(n);
      for (int k = 0; k < n; ++k) {
        const double* Xk = &X[3 * act[k]];
        const double Z = (Xk[0] * R[6] + Xk[1] * R[7] + Xk[2] * R[8]) + pose[2];
        const double dp = Z > 0 ? f * cfg.baseline / Z : std::numeric_limits<double>::quiet_NaN();
        const bool fin = std::isfinite(dp);
        const double dpc = fin ? std::min(dp, 1e9) : -1e9;  // (numpy's float -> int64 of a huge rint is undefined too)
        long l = (long)std::nearbyint(dpc) - kHalf;
        l = std::min<long>(std::max<long>(l, cfg.d_min), cfg.d_max);
        lo[k] = (int32_t)l;
        dvalid[k] = fin && dp > 0;
      }
      std::vector<float> uv, xr_all;
      std::vector<uint8_t> st, ok;
      VL_TRY(klt_match_new(n, im, lo, dvalid, t, 2 * kHalf + 1, nd_new, uv, st, xr_all, ok, nuv, nxr, nok),
             "klt_match_new");
      for (int k = 0; k < n; ++k) {
        const bool good = st[k] == 1 && in_margin(uv[2 * k], uv[2 * k + 1]) && ok[k];
        if (!good) {
          active[act[k]] = 0;
          continue;
        }
        trk_idx.push_back(act[k]);
        trk_uv.push_back(uv[2 * k]);
        trk_uv.push_back(uv[2 * k + 1]);
        xr_trk.push_back(xr_all[k]);
      }
    } else {
      new_cells_host(t, 0, nullptr, nuv);
      VL_TRY(match(im, nuv, nd_new, nxr, nok), "match");
    }
    // 6. frame t-1's scale LM queued now (front end, beside BA(t-1))
    if (has_scale_args) {
      VL_TRY(scale_submit(scale_t, scale_tids), "scale");
      has_scale_args = false;
    }
    const int n_tracked = (int)trk_idx.size();
    // 5. bookkeeping: new tracks (triangulated at the predicted pose), this frame's features
    const Mat3 R_pose = aa_to_R(&pose[3]);
    std::vector<int64_t> new_idx;
    std::vector<float> new_feats;
    {
      const size_t n0 = ntab();
      for (size_t k = 0; k < nok.size(); ++k) {
        if (!nok[k]) continue;
        double Xn[3];
        triangulate(nuv[2 * k], nuv[2 * k + 1], nxr[k], pose, R_pose, Xn);
        ids.push_back(latest_id++);
        X.insert(X.end(), Xn, Xn + 3);
        active.push_back(1);
        first.push_back(t);
        last.push_back(t);
        new_idx.push_back((int64_t)(n0 + new_feats.size() / 4));
        new_feats.insert(new_feats.end(), {nuv[2 * k], nuv[2 * k + 1], nxr[k], nuv[2 * k + 1]});
      }
    }
    // tracked first, then new; sorted by table index (= ID order; stable)
    const size_t nf = trk_idx.size() + new_idx.size();
    std::vector<int64_t> idx(nf);
    std::vector<float> feats(4 * nf);
    std::vector<uint8_t> is_new(nf, 0);
    {
      std::vector<std::pair<int64_t, size_t>> ord(nf);
      for (size_t k = 0; k < trk_idx.size(); ++k) ord[k] = {trk_idx[k], k};
      for (size_t k = 0; k < new_idx.size(); ++k) ord[trk_idx.size() + k] = {new_idx[k], trk_idx.size() + k};
      std::stable_sort(ord.begin(), ord.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
      for (size_t q = 0; q < nf; ++q) {
        const size_t k = ord[q].second;
        idx[q] = ord[q].first;
        if (k < trk_idx.size()) {
          const float fe[4] = {trk_uv[2 * k], trk_uv[2 * k + 1], xr_trk[k], trk_uv[2 * k + 1]};
          std::memcpy(&feats[4 * q], fe, 16);
        } else {
          std::memcpy(&feats[4 * q], &new_feats[4 * (k - trk_idx.size())], 16);
          is_new[q] = 1;
        }
      }
    }
    FrameObs fo;
    fo.ids.resize(nf);
    for (size_t q = 0; q < nf; ++q) {
      fo.ids[q] = ids[idx[q]];
      last[idx[q]] = t;
    }
    fo.feats = feats;
    if (cfg.log_events)
      for (size_t q = 0; q < nf; ++q) {
        me_vo_event e{is_new[q] ? 0 : 1, t, fo.ids[q], {0, 0, 0, 0}};
        std::memcpy(e.feat, &feats[4 * q], 16);
        events.push_back(e);
      }
    std::vector<int64_t> new_ids(new_idx.size());
    for (size_t k = 0; k < new_idx.size(); ++k) new_ids[k] = ids[new_idx[k]];
    const std::vector<int64_t> fid = fo.ids;
    obs[t] = std::move(fo);
    // 8 (chained). BA(t) queued now, behind BA(t-1), its start formed on the device
    Chain ch;
    const bool chained = chain_args(t, pose, R_pose, new_ids, ch);
    bool has_ba = false;
    BaRec rec;
    if (chained) {
      VL_TRY(window_add(t, fid, obs[t].feats), "window");
      VL_TRY(ba_submit(t, &ch, &has_ba, &rec), "BA");
    }
    // 7. frame t-1's BA applied
    bool done = false;
    int d_t = 0, d_tr = 0, d_new = 0, d_act = 0, nwp = 0, nwo = 0, bit = 0;
    double bcost = 0;
    if (has_pending) {
      done = true;
      d_t = pending.t;
      d_tr = pending.n_tracked;
      d_new = pending.n_new;
      d_act = pending.n_active;
      const Pending pd = pending;
      has_pending = false;
      VL_TRY(ba_finish(pd.has_ba, pd.ba, &nwp, &nwo, &bit, &bcost), "BA");
    }
    // pose(t) again from the refined poses; the new landmarks of t keep their camera-frame coordinates
    const Pose pose2 = predict_pose(t);
    if (pose2 != pose && !new_ids.empty()) {
      const Mat3 R2 = rot_series(&pose2[3]);
      for (int64_t id : new_ids) move_landmark(&X[3 * find_id(id)], R_pose, pose, pose2, R2);
    }
    poses[t] = pose2;
    // 8. the window's observations, BA(t) queued (unchained)
    if (!chained) {
      VL_TRY(window_add(t, fid, obs[t].feats), "window");
      VL_TRY(ba_submit(t, nullptr, &has_ba, &rec), "BA");
    }
    has_scale_args = true;
    scale_t = t;
    scale_tids = fid;
    int n_act = 0;
    for (uint8_t a : active) n_act += a;
    pending = Pending{t, n_tracked, (int)new_idx.size(), n_act, has_ba, std::move(rec)};
    has_pending = true;
    has_prev = true;
    prev_t = t;
    // (images older than t - 1 are no longer read: KLT(t+1) reads t, the scale LM of t runs in process(t + 1))
    for (auto it = imgs.begin(); it != imgs.end();)
      it = it->first < t - 1 ? imgs.erase(it) : std::next(it);
    // 9. frame t-1's FrameResult (its scale LM result), while BA(t) runs
    VL_TRY(complete_result(done, d_t, d_tr, d_new, d_act, nwp, nwo, bit, bcost), "result");
    host_s += (now_s() - t_in) - (wait_s - w0);
    return ME_OK;
  }
  int finish() {
    const double t_in = now_s();
    const double w0 = wait_s;
    if (has_pending) pop(pending.t + 1 - cfg.window);
    if (has_scale_args) {
      VL_TRY(scale_submit(scale_t, scale_tids), "scale");
      has_scale_args = false;
    }
    if (has_pending) {
      int nwp, nwo, bit;
      double bcost;
      const Pending pd = pending;
      has_pending = false;
      VL_TRY(ba_finish(pd.has_ba, pd.ba, &nwp, &nwo, &bit, &bcost), "BA");
      VL_TRY(complete_result(true, pd.t, pd.n_tracked, pd.n_new, pd.n_active, nwp, nwo, bit, bcost), "result");
    }
    host_s += (now_s() - t_in) - (wait_s - w0);
    return ME_OK;
  }
#undef VL_TRY
};

extern "C" {

void me_vo_loop_default_config(me_vo_loop_config* c) {
  *c = me_vo_loop_config{};
  c->width = 1280;
  c->height = 720;
  c->n_feats = 2000;
  c->window = 20;
  c->ba_iters = 10;
  c->scale_iters = 10;
  c->fixed_frames = 2;
  c->d_min = 2;
  c->d_max = 128;
  c->baseline = 0.5;
  c->feat_var = 0.25;
  const double f = 0.9 * c->width;
  const double K[9] = {f, 0, c->width / 2.0, 0, f, c->height / 2.0, 0, 0, 1};
  for (int k = 0; k < 9; ++k) c->K[k] = K[k];
  c->async_enqueue = 1;
}

int me_vo_loop_create(me_ctx* ba, me_ctx* front, const me_vo_loop_config* cfg, me_vo_loop** out) {
  if (!out) return ME_ERR_INVALID;
  *out = nullptr;
  if (!ba || !front || !cfg) return ME_ERR_INVALID;
  if (cfg->width < 2 * kMargin + 1 || cfg->height < 2 * kMargin + 1 || cfg->n_feats <= 0 || cfg->window < 1 ||
      cfg->d_min < 0 || cfg->d_max < cfg->d_min || cfg->ba_iters < 0 || cfg->scale_iters < 0)
    return me_set_error(ba, ME_ERR_INVALID, "me_vo_loop_create: bad configuration");
  auto v = std::make_unique<me_vo_loop>();
  v->ctx = ba;
  v->tctx = front;
  const int rc = v->init(*cfg);
  if (rc != ME_OK) {
    v->close();
    return rc;
  }
  *out = v.release();
  return ME_OK;
}

void me_vo_loop_destroy(me_vo_loop* v) {
  if (!v) return;
  v->close();
  delete v;
}

const char* me_vo_loop_last_error(const me_vo_loop* v) { return v ? v->err.c_str() : "null loop"; }

int me_vo_loop_process(me_vo_loop* v, int t, const uint8_t* left, const uint8_t* right, me_mem mem) {
  if (!v || !left || !right) return ME_ERR_INVALID;
  if (t != (v->has_prev ? v->prev_t + 1 : 0)) {
    v->err = "me_vo_loop_process: keyframes must come in order 0, 1, 2, ...";
    return ME_ERR_STATE;
  }
  if (v->failed) {
    v->err = "me_vo_loop_process: an earlier call failed (" + v->err + "); the loop state is undefined";
    return ME_ERR_STATE;
  }
  me_range range_("me_vo_loop_process");
  const int rc = v->process(t, left, right, mem);
  if (rc != ME_OK) v->failed = true;  // the loop may have stopped half-way through a keyframe
  return rc;
}

int me_vo_loop_finish(me_vo_loop* v) {
  if (!v) return ME_ERR_INVALID;
  me_range range_("me_vo_loop_finish");
  return v->finish();
}

int me_vo_loop_results(me_vo_loop* v, me_vo_frame_result* out, int cap, int* n) {
  if (!v || !n) return ME_ERR_INVALID;
  *n = (int)v->results.size();
  if (out)
    for (int i = 0; i < std::min(cap, *n); ++i) out[i] = v->results[i];
  return ME_OK;
}

int me_vo_loop_events(me_vo_loop* v, me_vo_event* out, long cap, long* n) {
  if (!v || !n) return ME_ERR_INVALID;
  *n = (long)v->events.size();
  if (out && cap > 0) std::memcpy(out, v->events.data(), sizeof(me_vo_event) * (size_t)std::min(cap, *n));
  return ME_OK;
}

int me_vo_loop_tracks(me_vo_loop* v, int64_t* ids, double* X, uint8_t* active, int64_t* first, int64_t* last, int cap,
                      int* n) {
  if (!v || !n) return ME_ERR_INVALID;
  *n = (int)v->ntab();
  const int m = std::min(cap, *n);
  for (int i = 0; i < m; ++i) {
    if (ids) ids[i] = v->ids[i];
    if (X)
      for (int q = 0; q < 3; ++q) X[3 * i + q] = v->X[3 * (size_t)i + q];
    if (active) active[i] = v->active[i];
    if (first) first[i] = v->first[i];
    if (last) last[i] = v->last[i];
  }
  return ME_OK;
}

int me_vo_loop_poses(me_vo_loop* v, int32_t* ts, double* poses, int cap, int* n) {
  if (!v || !n) return ME_ERR_INVALID;
  *n = (int)v->poses.size();
  int i = 0;
  for (auto& kv : v->poses) {
    if (i >= cap) break;
    if (ts) ts[i] = kv.first;
    if (poses)
      for (int q = 0; q < 6; ++q) poses[6 * i + q] = kv.second[q];
    ++i;
  }
  return ME_OK;
}

int me_vo_loop_frame_obs(me_vo_loop* v, int t, int64_t* ids, float* feats, int cap, int* n) {
  if (!v || !n) return ME_ERR_INVALID;
  auto it = v->obs.find(t);
  if (it == v->obs.end()) {
    *n = -1;
    return ME_OK;
  }
  *n = (int)it->second.ids.size();
  const int m = std::min(cap, *n);
  if (ids && m > 0) std::memcpy(ids, it->second.ids.data(), 8 * (size_t)m);
  if (feats && m > 0) std::memcpy(feats, it->second.feats.data(), 16 * (size_t)m);
  return ME_OK;
}

int me_vo_loop_frames(me_vo_loop* v, int32_t* ts, int cap, int* n) {
  if (!v || !n) return ME_ERR_INVALID;
  *n = (int)v->obs.size();
  int i = 0;
  for (auto& kv : v->obs) {
    if (i >= cap) break;
    if (ts) ts[i] = kv.first;
    ++i;
  }
  return ME_OK;
}

int me_vo_loop_stats(me_vo_loop* v, double* out, int n) {
  if (!v || !out) return ME_ERR_INVALID;
  const double s[9] = {v->host_s, v->wait_s, (double)v->latest_id, v->wait_stage[0], v->wait_stage[1],
                       v->wait_stage[2], v->wait_stage[3], v->wait_stage[4], v->wait_stage[5]};
  for (int i = 0; i < std::min(n, 9); ++i) out[i] = s[i];
  return ME_OK;
}

}  // extern "C"
