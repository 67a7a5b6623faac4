// adapter_cli — a C++ caller of the reference-shaped API in
// include/MotionEstimationAMD/motion_estimation_amd.hpp (which binds the C ABI
// of libme_hip.so).  Used by tests/test_cpp_adapter.py to show that a C++
// host built like the reference's src/ gets the same results as the Python
// mirror and the oracle.
//   adapter_cli ba  <in.bin> <out.bin>   BundleAdjuster<M>-style solve (M = 4 or 2, optional covariance)
//   adapter_cli ba_rccl <in.bin> <out.bin>  the same through a one-rank RCCL amd::Comm (me_ba_solve_comm)
//   adapter_cli mi  <in.bin> <out.bin>   computeMutualInformation / computeEntropy
//   adapter_cli nms <in.bin> <out.bin>   nonMaxSupScanline3x3
//   adapter_cli scale <in.bin> <out.bin> Optimiser<ScaleState,...>: compute_residuals, optimise, compute_inliers,
//                                        getJacobian, ScaleState::compute_residuals (via flatten_scale_state)
//   adapter_cli vo  <in.bin> <out.bin>   StereoVisualOdometry::process / getMotion / getInliers_idx
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <vector>

#include "MotionEstimationAMD/motion_estimation_amd.hpp"

namespace {
struct Reader {
  std::vector<char> buf;
  size_t pos = 0;
  template <class T>
  T get() {
    T v;
    std::memcpy(&v, buf.data() + pos, sizeof(T));
    pos += sizeof(T);
    return v;
  }
  template <class T>
  void get(T* dst, size_t n) {
    std::memcpy(dst, buf.data() + pos, n * sizeof(T));
    pos += n * sizeof(T);
  }
};

Reader read_file(const char* path) {
  std::ifstream f(path, std::ios::binary);
  Reader r;
  r.buf.assign(std::istreambuf_iterator<char>(f), {});
  return r;
}

template <int M>
int solve_ba(Reader& in, FILE* out, int nc, int np, int no, int fixed, int compute_cov, bool rccl) {
  using namespace me::optimisation;
  CalibrationParameters calib;
  calib.K.resize(2);
  in.get(calib.K[0].data(), 9);
  in.get(calib.K[1].data(), 9);
  calib.baseline = in.get<double>();
  calib.feat_var = in.get<double>();
  calib.compute_cov = compute_cov != 0;
  std::vector<std::array<double, 6>> cams(nc);
  std::vector<std::array<double, 3>> pts(np);
  in.get(cams[0].data(), 6 * (size_t)nc);
  in.get(pts[0].data(), 3 * (size_t)np);
  std::vector<double> o(M * (size_t)no);
  in.get(o.data(), o.size());
  std::vector<int32_t> ci(no), pi(no), cid(no, 0);
  in.get(ci.data(), no);
  in.get(pi.data(), no);
  if (M == 2) in.get(cid.data(), no);
  std::vector<Observation<M>> obs(no);
  for (int k = 0; k < no; ++k) {
    for (int a = 0; a < M; ++a) obs[k].xy[a] = o[M * k + a];
    obs[k].camIdx = ci[k];
    obs[k].ptIdx = pi[k];
    obs[k].camID = cid[k];
  }
  BundleAdjuster<M> ba(calib, cams, pts, obs);
  std::unique_ptr<me::amd::Comm> comm;
  if (rccl) comm.reset(new me::amd::Comm(me::amd::Context::thread_default(), 1, 0, me::amd::Comm::unique_id()));
  const auto status = ba.optimise(fixed, comm.get());
  const int32_t st = (int32_t)status, it = ba.summary().iterations;
  const double cost = ba.summary().final_cost;
  fwrite(&st, 4, 1, out);
  fwrite(&it, 4, 1, out);
  fwrite(&cost, 8, 1, out);
  fwrite(ba.getCameraParams()[0].data(), 8, 6 * (size_t)nc, out);
  fwrite(ba.getPoints()[0].data(), 8, 3 * (size_t)np, out);
  const int32_t ncov = (int32_t)ba.getPosesCovariance().size();
  fwrite(&ncov, 4, 1, out);
  for (const auto& c : ba.getPosesCovariance()) fwrite(c.data(), 8, 36, out);
  return 0;
}

// payload: nc np no fixed obs_dim compute_cov | K0 K1 | baseline feat_var | cams pts obs cam_idx pt_idx [cam_id]
int run_ba(Reader& in, FILE* out, bool rccl = false) {
  const int nc = in.get<int32_t>(), np = in.get<int32_t>(), no = in.get<int32_t>(), fixed = in.get<int32_t>();
  const int od = in.get<int32_t>(), cov = in.get<int32_t>();
  return od == 2 ? solve_ba<2>(in, out, nc, np, no, fixed, cov, rccl) : solve_ba<4>(in, out, nc, np, no, fixed, cov, rccl);
}

int run_mi(Reader& in, FILE* out) {
  const int rows = in.get<int32_t>(), cols = in.get<int32_t>();
  std::vector<uint8_t> L((size_t)rows * cols), R((size_t)rows * cols);
  in.get(L.data(), L.size());
  in.get(R.data(), R.size());
  me::amd::ImageView vl{L.data(), rows, cols, cols}, vr{R.data(), rows, cols, cols};
  const float mi = me::computeMutualInformation(vl, vr), h = me::computeEntropy(vl);
  fwrite(&mi, 4, 1, out);
  fwrite(&h, 4, 1, out);
  // invalid input keeps the reference's contract (assert -> exception here)
  int32_t threw = 0;
  try {
    me::computeMutualInformation(me::amd::ImageView{}, vr);
  } catch (const std::invalid_argument&) {
    threw = 1;
  }
  fwrite(&threw, 4, 1, out);
  return 0;
}

int run_nms(Reader& in, FILE* out) {
  const int rows = in.get<int32_t>(), cols = in.get<int32_t>();
  std::vector<double> resp((size_t)rows * cols);
  in.get(resp.data(), resp.size());
  std::vector<uint8_t> mask;
  auto pts = me::nonMaxSupScanline3x3(resp.data(), rows, cols, mask);
  const int32_t n = (int32_t)pts.size();
  fwrite(&n, 4, 1, out);
  for (auto& p : pts) {
    fwrite(&p.first, 8, 1, out);
    fwrite(&p.second, 8, 1, out);
  }
  fwrite(mask.data(), 1, mask.size(), out);
  return 0;
}
// payload: nL nR w lframe fixed10 has_mask rows cols | K1 K2 q1 t1 q2 t2 scale baseline threshold |
//          XL XR | triL triR (u8) | lastL lastR (u32) | [mask u8 nL+nR] | imgL imgR
int run_scale(Reader& in, FILE* out) {
  using namespace me::optimisation;
  const int nL = in.get<int32_t>(), nR = in.get<int32_t>(), w = in.get<int32_t>(), lframe = in.get<int32_t>();
  const int fixed10 = in.get<int32_t>(), has_mask = in.get<int32_t>(), rows = in.get<int32_t>(),
            cols = in.get<int32_t>();
  ScaleState st;
  in.get(st.K.first.val.data(), 9);
  in.get(st.K.second.val.data(), 9);
  me::CamPose_qd p1, p2;
  double q[4];
  in.get(q, 4);
  p1.orientation = me::Quat{q[0], q[1], q[2], q[3]};
  in.get(p1.position.data(), 3);
  in.get(q, 4);
  p2.orientation = me::Quat{q[0], q[1], q[2], q[3]};
  in.get(p2.position.data(), 3);
  st.scale = in.get<double>();
  st.baseline = in.get<double>();
  const double thr = in.get<double>();
  st.window_size = w;
  // a two-keyframe window ending at lframe: poses.first[0].ID + size - 1 == lframe (optimisation.cpp:165)
  me::CamPose_qd p0;
  p0.ID = lframe - 1;
  p1.ID = p2.ID = lframe;
  st.poses.first = {p0, p1};
  st.poses.second = {p0, p2};
  std::vector<double> XL(4 * (size_t)nL), XR(4 * (size_t)nR);
  in.get(XL.data(), XL.size());
  in.get(XR.data(), XR.size());
  std::vector<uint8_t> tL(nL), tR(nR);
  in.get(tL.data(), nL);
  in.get(tR.data(), nR);
  std::vector<uint32_t> lL(nL), lR(nR);
  in.get(lL.data(), nL);
  in.get(lR.data(), nR);
  me::VectorXi mask;
  if (has_mask) {
    std::vector<uint8_t> m(nL + nR);
    in.get(m.data(), m.size());
    mask.v.assign(m.begin(), m.end());
  }
  auto fill = [](std::vector<me::WBA_Ptf>& v, const std::vector<double>& X, const std::vector<uint32_t>& last) {
    v.resize(last.size());
    for (size_t i = 0; i < v.size(); ++i) {
      for (int k = 0; k < 4; ++k) v[i].pt.v[k] = X[4 * i + k];
      v[i].last_frame = last[i];
    }
  };
  fill(st.pts.first, XL, lL);
  fill(st.pts.second, XR, lR);
  std::vector<uint8_t> L((size_t)rows * cols), R((size_t)rows * cols);
  in.get(L.data(), L.size());
  in.get(R.data(), R.size());
  const me::amd::ImageView vl{L.data(), rows, cols, cols}, vr{R.data(), rows, cols, cols};
  const ImagePairs obs{{vl, vr}, {vl, vr}};
  OptimisationParams params;
  if (fixed10) {  // the bench frame: MAX_NB_ITER 10, tolerances off
    params.MAX_NB_ITER = 10;
    params.abs_tol = params.grad_tol = params.incr_tol = params.rel_tol = 0;
  }
  const ScaleState st0 = st;
  Optimiser<ScaleState, ImagePairs> opt(obs, params);
  const std::vector<double> res0 = opt.compute_residuals(st0);
  const int32_t stop = (int32_t)opt.optimise(st, false, mask);
  const int32_t iters = opt.iterations();
  const std::vector<int> inl = opt.compute_inliers(thr);
  const double jac = opt.getJacobian();
  const double smi = st0.compute_residuals(obs);
  fwrite(&stop, 4, 1, out);
  fwrite(&iters, 4, 1, out);
  fwrite(&st.scale, 8, 1, out);
  const int32_t nres = (int32_t)res0.size(), ninl = (int32_t)inl.size();
  fwrite(&nres, 4, 1, out);
  fwrite(res0.data(), 8, res0.size(), out);
  fwrite(&ninl, 4, 1, out);
  fwrite(inl.data(), 4, inl.size(), out);
  fwrite(&jac, 8, 1, out);
  fwrite(&smi, 8, 1, out);
  return 0;
}

// payload: n seed | baseline fu1 fv1 fu2 fv2 cu1 cu2 cv1 cv2 | matches n x 8 floats
int run_vo(Reader& in, FILE* out) {
  const int n = in.get<int32_t>();
  const unsigned seed = (unsigned)in.get<int32_t>();
  me::StereoVisualOdometry::parameters prm;
  prm.baseline = in.get<double>();
  prm.fu1 = in.get<double>();
  prm.fv1 = in.get<double>();
  prm.fu2 = in.get<double>();
  prm.fv2 = in.get<double>();
  prm.cu1 = in.get<double>();
  prm.cu2 = in.get<double>();
  prm.cv1 = in.get<double>();
  prm.cv2 = in.get<double>();
  std::vector<me::StereoOdoMatchesf> m((size_t)n);
  for (auto& q : m) {
    float v[8];
    in.get(v, 8);
    q.f1 = {v[0], v[1]};
    q.f2 = {v[2], v[3]};
    q.f3 = {v[4], v[5]};
    q.f4 = {v[6], v[7]};
  }
  me::StereoVisualOdometry vo(prm);
  vo.srand(seed);
  const int32_t ok = vo.process(m) ? 1 : 0;
  fwrite(&ok, 4, 1, out);
  fwrite(vo.getMotion().data(), 8, 16, out);
  const int32_t ninl = (int32_t)vo.getInliers_idx().size();
  fwrite(&ninl, 4, 1, out);
  fwrite(vo.getInliers_idx().data(), 4, vo.getInliers_idx().size(), out);
  return 0;
}
int run_mono(Reader& in, FILE* out) {
  const int n = in.get<int32_t>();
  me::MonoVisualOdometry::parameters prm;
  prm.ransac = in.get<int32_t>() != 0;
  prm.fu = in.get<double>();
  prm.fv = in.get<double>();
  prm.cu = in.get<double>();
  prm.cv = in.get<double>();
  std::vector<me::StereoMatch<me::Point2f>> m((size_t)n);
  for (auto& q : m) {
    float v[4];
    in.get(v, 4);
    q.f1 = {v[0], v[1]};
    q.f2 = {v[2], v[3]};
  }
  me::MonoVisualOdometry vo(prm);
  const int32_t ok = vo.process(m) ? 1 : 0;
  fwrite(&ok, 4, 1, out);
  fwrite(vo.getMotion().data(), 8, 16, out);
  const int32_t ninl = (int32_t)vo.getInliersIdx().size();
  fwrite(&ninl, 4, 1, out);
  fwrite(vo.getInliersIdx().data(), 4, vo.getInliersIdx().size(), out);
  return 0;
}
}  // namespace

int main(int argc, char** argv) {
  if (argc != 4) {
    std::fprintf(stderr, "usage: %s ba|mi|nms|scale|vo|mono in.bin out.bin\n", argv[0]);
    return 2;
  }
  Reader in = read_file(argv[2]);
  FILE* out = std::fopen(argv[3], "wb");
  if (!out) return 2;
  int rc = 2;
  try {
    if (!std::strcmp(argv[1], "ba")) rc = run_ba(in, out);
    else if (!std::strcmp(argv[1], "ba_rccl")) rc = run_ba(in, out, true);
    else if (!std::strcmp(argv[1], "mi")) rc = run_mi(in, out);
    else if (!std::strcmp(argv[1], "nms")) rc = run_nms(in, out);
    else if (!std::strcmp(argv[1], "scale")) rc = run_scale(in, out);
    else if (!std::strcmp(argv[1], "vo")) rc = run_vo(in, out);
    else if (!std::strcmp(argv[1], "mono")) rc = run_mono(in, out);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "adapter_cli: %s\n", e.what());
    rc = 1;
  }
  std::fclose(out);
  return rc;
}
