// sanitize_driver.cpp — TEST INFRASTRUCTURE ONLY.  Drives every entry point
// of the CPU restatement (oracle/*.cpp) once on small deterministic inputs,
// built with -fsanitize=address,undefined (oracle/Makefile target
// `sanitize`, run by tests/test_oracle_sanitize.py): out-of-bounds accesses,
// use-after-free, signed overflow, misaligned loads or bad shifts in the
// checker itself abort the run.  Prints a checksum of the outputs.
// (The reference's own build has only -Wall -pedantic, CMakeLists.txt:6.)
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>
#include "oracle.h"

namespace {

uint32_t g_state = 12345u;
uint32_t lcg() {
  g_state = g_state * 1664525u + 1013904223u;
  return g_state >> 8;
}
double urand() { return (lcg() & 0xffffff) / 16777216.0; }

// textured 8-bit image: smooth value noise + a little grain
std::vector<uint8_t> image(int w, int h, double phase) {
  std::vector<uint8_t> img((size_t)w * h);
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      double v = 128 + 60 * std::sin(0.07 * x + phase) * std::cos(0.05 * y - phase) + 30 * std::sin(0.013 * x * y);
      img[(size_t)y * w + x] = (uint8_t)std::max(0.0, std::min(255.0, v + 10 * urand()));
    }
  return img;
}

double sum(const double* v, size_t n) {
  double s = 0;
  for (size_t i = 0; i < n; ++i) s += std::isfinite(v[i]) ? v[i] : 0.0;
  return s;
}

void project(const double* K, double b, const double* cam, const double* X, double* o) {
  // cam {t, angle-axis}: p = R(aa) X + t (Rodrigues)
  const double* aa = cam + 3;
  const double th = std::sqrt(aa[0] * aa[0] + aa[1] * aa[1] + aa[2] * aa[2]);
  double p[3];
  if (th > 1e-12) {
    const double k[3] = {aa[0] / th, aa[1] / th, aa[2] / th}, c = std::cos(th), s = std::sin(th);
    const double kx[3] = {k[1] * X[2] - k[2] * X[1], k[2] * X[0] - k[0] * X[2], k[0] * X[1] - k[1] * X[0]};
    const double kd = k[0] * X[0] + k[1] * X[1] + k[2] * X[2];
    for (int i = 0; i < 3; ++i) p[i] = X[i] * c + kx[i] * s + k[i] * kd * (1 - c);
  } else {
    for (int i = 0; i < 3; ++i) p[i] = X[i];
  }
  for (int i = 0; i < 3; ++i) p[i] += cam[i];
  o[0] = K[0] * p[0] / p[2] + K[2];
  o[1] = K[4] * p[1] / p[2] + K[5];
  o[2] = K[0] * (p[0] - b) / p[2] + K[2];
  o[3] = o[1];
}

}  // namespace

int main() {
  const int W = 160, H = 120;
  double chk = 0;
  std::vector<uint8_t> L = image(W, H, 0.3), R = image(W, H, 0.9), L2 = image(W, H, 0.35);

  // A1/A2/A3
  chk += oracle_mutual_information(L.data(), W, R.data(), W, 11, 11);
  chk += oracle_mutual_information(L.data(), W, L.data(), W, W, H);
  chk += oracle_entropy(L.data(), W, W, H);
  int32_t hl[20], hr[20], hj[400];
  oracle_mi_histograms(L.data(), W, R.data(), W, 10, 10, hl, hr, hj);
  const int n = 64;
  std::vector<int32_t> xyL(2 * n), xyR(2 * n);
  for (int k = 0; k < n; ++k) {
    xyL[2 * k] = (int)(lcg() % (W - 11));
    xyL[2 * k + 1] = (int)(lcg() % (H - 11));
    xyR[2 * k] = (int)(lcg() % (W - 11));
    xyR[2 * k + 1] = xyL[2 * k + 1];
  }
  std::vector<float> mi(n);
  oracle_mi_scores(L.data(), W, R.data(), W, xyL.data(), xyR.data(), n, 11, 11, mi.data());
  for (float v : mi) chk += v;
  std::vector<float> A(4 * 8 * 8), B(4 * 8 * 8), out(4);
  for (auto& v : A) v = (float)urand();
  for (auto& v : B) v = (float)urand();
  oracle_compare_pc(A.data(), B.data(), 4, 8, 8, out.data());
  for (float v : out) chk += v;
  oracle_ccoeff_normed(A.data(), B.data(), 4, 8, 8, out.data());
  for (float v : out) chk += v;
  std::vector<uint8_t> Q = L;
  oracle_quantise(Q.data(), W, W, H, 40, 200);
  chk += Q[777];
  chk += oracle_log2f(3.0f);

  // A11 NMS
  std::vector<double> resp((size_t)W * H);
  for (auto& v : resp) v = std::floor(urand() * 20);  // plateaus
  std::vector<uint8_t> mask((size_t)W * H);
  std::vector<double> maxima(2 * W * H);
  chk += oracle_nms_scanline3x3(resp.data(), W, H, mask.data(), maxima.data(), W * H);

  // A12 KLT
  oracle_klt_params kp{21, 3, 30, 0.01, 1e-4};
  const int nf = 40;
  std::vector<float> pin(2 * nf), pout(2 * nf);
  std::vector<uint8_t> st(nf);
  for (int k = 0; k < nf; ++k) {
    pin[2 * k] = 15 + (float)(urand() * (W - 30));
    pin[2 * k + 1] = 15 + (float)(urand() * (H - 30));
  }
  oracle_klt_track(L.data(), L2.data(), W, H, W, pin.data(), pout.data(), st.data(), nf, &kp);
  for (int k = 0; k < nf; ++k) chk += st[k] ? pout[2 * k] : 0.0;

  // A13-A17 BA: 6 cameras moving forward, 80 points, tracks of >= 2 frames
  const int nc = 6, np = 80;
  double K[9] = {150, 0, 80, 0, 150, 60, 0, 0, 1};
  std::vector<double> cams(6 * nc, 0.0), pts(3 * np), obs;
  std::vector<int32_t> ci, pi;
  for (int c = 0; c < nc; ++c) {
    cams[6 * c + 2] = -0.3 * c;
    cams[6 * c + 4] = 0.002 * c;
  }
  for (int j = 0; j < np; ++j) {
    pts[3 * j] = (urand() - 0.5) * 6;
    pts[3 * j + 1] = (urand() - 0.5) * 4;
    pts[3 * j + 2] = 6 + urand() * 10;
    const int s = (int)(lcg() % (nc - 1)), e = s + 1 + (int)(lcg() % (nc - s - 1));
    for (int c = s; c <= e; ++c) {
      double o[4];
      project(K, 0.5, &cams[6 * c], &pts[3 * j], o);
      for (int k = 0; k < 4; ++k) obs.push_back(o[k] + (urand() - 0.5));
      ci.push_back(c);
      pi.push_back(j);
    }
  }
  for (int c = 2; c < nc; ++c) cams[6 * c] += 0.02;
  for (auto& v : pts) v *= 1.01;
  oracle_ba_problem p{};
  p.n_cams = nc;
  p.n_pts = np;
  p.n_obs = (int)ci.size();
  p.cams = cams.data();
  p.pts = pts.data();
  p.obs = obs.data();
  p.cam_idx = ci.data();
  p.pt_idx = pi.data();
  std::memcpy(p.K0, K, sizeof K);
  std::memcpy(p.K1, K, sizeof K);
  p.baseline = 0.5;
  p.feat_var = 0.25;
  p.fixed_frames = 2;
  p.obs_dim = 4;
  std::vector<double> res(4 * p.n_obs), Jc(24 * p.n_obs), Jp(12 * p.n_obs);
  oracle_ba_evaluate(&p, res.data(), Jc.data(), Jp.data());
  chk += sum(res.data(), res.size()) + oracle_ba_cost(&p);
  const int m6 = 6 * (nc - 2);
  std::vector<double> S((size_t)m6 * m6), b(m6);
  oracle_ba_reduced_system(&p, 1e4, S.data(), b.data());
  chk += sum(S.data(), S.size()) + sum(b.data(), b.size());
  oracle_ba_reduced_system_ex(&p, 1e3, 0, S.data(), b.data());
  chk += sum(b.data(), b.size());
  oracle_ba_options bo;
  oracle_ba_default_options(&bo);
  bo.max_num_iterations = 5;
  oracle_ba_summary bs{};
  std::vector<double> trace(16);
  oracle_ba_solve(&p, &bo, &bs, trace.data(), 16);
  chk += bs.final_cost + sum(cams.data(), cams.size()) + sum(pts.data(), pts.size());
  std::vector<double> cov(36 * nc);
  if (oracle_ba_covariance(&p, cov.data())) chk += sum(cov.data(), cov.size());
  // BundleAdjuster<2>: left / right observations by camID
  std::vector<double> obs2(2 * p.n_obs);
  std::vector<int32_t> cid(p.n_obs);
  for (int o = 0; o < p.n_obs; ++o) {
    cid[o] = o & 1;
    obs2[2 * o] = obs[4 * o + (cid[o] ? 2 : 0)];
    obs2[2 * o + 1] = obs[4 * o + 1];
  }
  oracle_ba_problem p2 = p;
  p2.obs = obs2.data();
  p2.obs_dim = 2;
  p2.cam_id = cid.data();
  oracle_ba_solve(&p2, &bo, &bs, nullptr, 0);
  chk += bs.final_cost;

  // A4-A8 scale LM over the BA points, left tracks seen in the last frame
  std::vector<double> Xh(4 * np);
  std::vector<uint8_t> tri(np, 1);
  std::vector<uint32_t> last(np, nc - 1);
  for (int j = 0; j < np; ++j) {
    for (int a = 0; a < 3; ++a) Xh[4 * j + a] = pts[3 * j + a];
    Xh[4 * j + 3] = 1.0;
  }
  oracle_scale_state ss{};
  ss.n_left = np;
  ss.X_left = Xh.data();
  ss.tri_left = tri.data();
  ss.last_left = last.data();
  ss.lframe = nc - 1;
  std::memcpy(ss.K1, K, sizeof K);
  std::memcpy(ss.K2, K, sizeof K);
  ss.q1[0] = ss.q2[0] = 1.0;
  ss.scale = 1.0;
  ss.baseline = 0.5;
  ss.window_size = 5;
  ss.imgL = L.data();
  ss.imgR = R.data();
  ss.stride = ss.cols = ss.bb_cols = W;
  ss.rows = ss.bb_rows = H;
  std::vector<double> sres(np + 1);
  const int rows = oracle_scale_residuals(&ss, 0, sres.data());
  chk += rows + sum(sres.data(), rows > 0 ? rows : 0);
  double JJ = 0, e = 0;
  oracle_scale_normal_equations(&ss, 0, sres.data(), &JJ, &e);
  oracle_scale_jacobian(&ss, 0, &JJ);
  chk += JJ + e;
  oracle_optim_params op;
  oracle_optim_default_params(&op);
  op.max_nb_iter = 4;
  int it = 0;
  long nmi = 0;
  std::vector<double> st_trace(32);
  chk += oracle_scale_optimise(&ss, &op, 0, &it, st_trace.data(), 16, &nmi) + ss.scale;
  std::vector<int> inl(np + 1);
  chk += oracle_scale_inliers(&ss, 0.5, inl.data(), np + 1);
  double smi = 0;
  int npairs = 0;
  if (oracle_scale_state_mi(&ss, &smi, &npairs) == 0) chk += smi;
  long cnt[3];
  oracle_scale_counters(cnt);

  // A19 StereoVO on noise-free matches of the BA scene (frame 0 -> 1)
  const int nm = 40;
  std::vector<float> matches(8 * nm);
  double cam0[6] = {0, 0, 0, 0, 0, 0}, cam1[6] = {0.01, 0, -0.3, 0, 0.002, 0};
  for (int k = 0; k < nm; ++k) {
    double o0[4], o1[4];
    project(K, 0.5, cam0, &pts[3 * k], o0);
    project(K, 0.5, cam1, &pts[3 * k], o1);
    const float v[8] = {(float)o0[0], (float)o0[1], (float)o0[2], (float)o0[3],
                        (float)o1[0], (float)o1[1], (float)o1[2], (float)o1[3]};
    std::memcpy(&matches[8 * k], v, sizeof v);
  }
  oracle_vo_params vp{};
  vp.method = 0;
  vp.e1 = vp.e2 = vp.e3 = vp.e4 = 1e-7;
  vp.max_iter = 20;
  vp.ransac = 1;
  vp.n_ransac = 20;
  vp.inlier_threshold = 2.0;
  vp.baseline = 0.5;
  vp.fu1 = vp.fu2 = 150;
  vp.fv1 = vp.fv2 = 150;
  vp.cu1 = vp.cu2 = 80;
  vp.cv1 = vp.cv2 = 60;
  std::vector<int> rs(3 * 20);
  for (auto& v : rs) v = (int)(lcg() & 0x7fffffff);
  double init6[6] = {0, 0, 0, 0, 0, 0}, motion[16];
  std::vector<int> vin(nm);
  int nin = 0;
  chk += oracle_vo_process(matches.data(), nm, init6, &vp, rs.data(), (int)rs.size(), motion, vin.data(), &nin, 200);
  chk += nin + sum(motion, 16);

  // pose-covariance helpers
  double q1[4] = {1, 0, 0, 0}, t1[3] = {0.1, 0, 0}, c1[36] = {0}, q2[4] = {0.99, 0.1, 0, 0}, t2[3] = {0, 0.2, 0},
         c2[36] = {0}, q3[4], t3[3], c3[36];
  for (int i = 0; i < 6; ++i) c1[7 * i] = c2[7 * i] = 0.01;
  oracle_pose_mul_cov(q1, t1, c1, q2, t2, c2, 0, q3, t3, c3);
  oracle_pose_invert_cov(q3, t3, c3);
  oracle_pose_scale_cov(t3, c3, 2.0, 0.1);
  chk += sum(c3, 36) + t3[0];

  std::printf("sanitize_driver ok checksum %.6e\n", chk);
  return 0;
}
