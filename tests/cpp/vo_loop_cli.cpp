// vo_loop_cli -- a compiled C++ host driving the windowed stereo VO loop
// through me::WindowedStereoVO (include/MotionEstimationAMD/
// motion_estimation_amd.hpp over the C ABI): the loop the reference's
// application would run, with no Python in the process.  Used by
// tests/test_pipeline.py (test_native_loop_*, test_cpp_host_drives_the_loop).
//   vo_loop_cli <in.bin> <out.bin> [front_cus]
// in.bin : int32 {width, height, n_feats, window, ba_iters, scale_iters, fixed_frames, d_min, d_max, n_frames,
//          has_velocity}, float64 {baseline, feat_var, K[9], first_pose[6], velocity[6]},
//          then n_frames x (left, right) width x height bytes
// out.bin: int64 n_results, me_vo_frame_result[...], int64 n_events, me_vo_event[...],
//          int64 n_poses, {int32 t, int32 pad, float64 pose[6]}[...], int64 n_tracks, int64 ids[...], float64 X[3 n]
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <vector>

#include "MotionEstimationAMD/motion_estimation_amd.hpp"

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: vo_loop_cli <in.bin> <out.bin> [front_cus]\n");
    return 2;
  }
  std::ifstream f(argv[1], std::ios::binary);
  std::vector<char> buf((std::istreambuf_iterator<char>(f)), {});
  size_t pos = 0;
  auto get = [&](void* dst, size_t n) {
    std::memcpy(dst, buf.data() + pos, n);
    pos += n;
  };
  int32_t iv[11];
  double dv[2 + 9 + 6 + 6];
  get(iv, sizeof iv);
  get(dv, sizeof dv);
  me::WindowedStereoVO::Config cfg;
  cfg.width = iv[0];
  cfg.height = iv[1];
  cfg.n_feats = iv[2];
  cfg.window = iv[3];
  cfg.ba_iters = iv[4];
  cfg.scale_iters = iv[5];
  cfg.fixed_frames = iv[6];
  cfg.d_min = iv[7];
  cfg.d_max = iv[8];
  const int n_frames = iv[9];
  cfg.has_velocity = iv[10];
  cfg.baseline = dv[0];
  cfg.feat_var = dv[1];
  std::memcpy(cfg.K, dv + 2, 9 * sizeof(double));
  std::memcpy(cfg.first_pose, dv + 11, 6 * sizeof(double));
  std::memcpy(cfg.velocity, dv + 17, 6 * sizeof(double));
  cfg.log_events = 1;
  const size_t npx = (size_t)cfg.width * cfg.height;
  if (buf.size() != pos + 2 * npx * n_frames) {
    std::fprintf(stderr, "vo_loop_cli: %zu bytes, expected %zu\n", buf.size(), pos + 2 * npx * n_frames);
    return 2;
  }
  try {
    me::amd::Context ba(0), front(0);
    me::WindowedStereoVO vo(ba, front, cfg, argc > 3 ? std::atoi(argv[3]) : 4);
    for (int t = 0; t < n_frames; ++t) {
      const uint8_t* L = reinterpret_cast<const uint8_t*>(buf.data() + pos + 2 * npx * t);
      me::amd::ImageView left{L, cfg.height, cfg.width, cfg.width}, right{L + npx, cfg.height, cfg.width, cfg.width};
      vo.process(t, left, right);
    }
    vo.finish();
    FILE* o = std::fopen(argv[2], "wb");
    const auto res = vo.results();
    int64_t n = (int64_t)res.size();
    std::fwrite(&n, 8, 1, o);
    std::fwrite(res.data(), sizeof(me_vo_frame_result), res.size(), o);
    const auto ev = vo.events();
    n = (int64_t)ev.size();
    std::fwrite(&n, 8, 1, o);
    std::fwrite(ev.data(), sizeof(me_vo_event), ev.size(), o);
    const auto ps = vo.poses();
    n = (int64_t)ps.size();
    std::fwrite(&n, 8, 1, o);
    for (const auto& p : ps) {
      const int32_t tp[2] = {p.first, 0};
      std::fwrite(tp, 4, 2, o);
      std::fwrite(p.second.data(), 8, 6, o);
    }
    std::vector<int64_t> ids;
    std::vector<std::array<double, 3>> X;
    vo.tracks(ids, X);
    n = (int64_t)ids.size();
    std::fwrite(&n, 8, 1, o);
    std::fwrite(ids.data(), 8, ids.size(), o);
    if (!X.empty()) std::fwrite(X[0].data(), 8, 3 * X.size(), o);
    std::fclose(o);
    std::printf("vo_loop_cli: %d keyframes, %zu results, %zu events\n", n_frames, res.size(), ev.size());
  } catch (const std::exception& e) {
    std::fprintf(stderr, "vo_loop_cli: %s\n", e.what());
    return 1;
  }
  return 0;
}
