// adapter_cli — a C++ caller of the reference-shaped API in
// include/MotionEstimationAMD/motion_estimation_amd.hpp (which binds the C ABI
// of libme_hip.so).  Used by tests/test_cpp_adapter.py to show that a C++
// host built like the reference's src/ gets the same results as the Python
// mirror and the oracle.
//   adapter_cli ba  <in.bin> <out.bin>   BundleAdjuster<M>-style solve (M = 4 or 2, optional covariance)
//   adapter_cli mi  <in.bin> <out.bin>   computeMutualInformation / computeEntropy
//   adapter_cli nms <in.bin> <out.bin>   nonMaxSupScanline3x3
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
int solve_ba(Reader& in, FILE* out, int nc, int np, int no, int fixed, int compute_cov) {
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
  const auto status = ba.optimise(fixed);
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
int run_ba(Reader& in, FILE* out) {
  const int nc = in.get<int32_t>(), np = in.get<int32_t>(), no = in.get<int32_t>(), fixed = in.get<int32_t>();
  const int od = in.get<int32_t>(), cov = in.get<int32_t>();
  return od == 2 ? solve_ba<2>(in, out, nc, np, no, fixed, cov) : solve_ba<4>(in, out, nc, np, no, fixed, cov);
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
}  // namespace

int main(int argc, char** argv) {
  if (argc != 4) {
    std::fprintf(stderr, "usage: %s ba|mi|nms in.bin out.bin\n", argv[0]);
    return 2;
  }
  Reader in = read_file(argv[2]);
  FILE* out = std::fopen(argv[3], "wb");
  if (!out) return 2;
  int rc = 2;
  try {
    if (!std::strcmp(argv[1], "ba")) rc = run_ba(in, out);
    else if (!std::strcmp(argv[1], "mi")) rc = run_mi(in, out);
    else if (!std::strcmp(argv[1], "nms")) rc = run_nms(in, out);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "adapter_cli: %s\n", e.what());
    rc = 1;
  }
  std::fclose(out);
  return rc;
}
