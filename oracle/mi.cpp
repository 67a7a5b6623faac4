#include <utility>
// oracle/mi.cpp — TEST INFRASTRUCTURE: CPU restatement of the reference MI
// (src/core/mutual_information.cpp:28-86).  Parity unpinned (see oracle.h).
//
// OpenCV 4 semantics restated:
//  * calcHist(8U, 20 uniform bins over [0,256)): lookup bin = floor(v*20/256)
//    = (5v)>>6 (a = 20/256 is exact in double), integer counts, then float.
//  * `hist /= N` is Mat::convertTo(alpha = 1/N) -> cvt_32f with
//    a = (float)(1.0/N): p = fl32(count * fl32(1/N)).
//  * MI loop (mutual_information.cpp:80-83): i (L bin) outer, j (R bin) inner,
//    float accumulator, term = pJ*log2f(pJ/(pL*pR)) with every op in float and
//    no FMA contraction (x86-64 default build).
//  * log2 is glibc 2.35 log2f: restated below from the published algorithm and
//    checked exhaustively against the host libm by tests/test_oracle.py.
#include "oracle.h"
#include <cmath>
#include <cstring>

namespace {
const double kLog2fTab[16][2] = {
    {0x1.661ec79f8f3bep+0, -0x1.efec65b963019p-2}, {0x1.571ed4aaf883dp+0, -0x1.b0b6832d4fca4p-2},
    {0x1.49539f0f010b0p+0, -0x1.7418b0a1fb77bp-2}, {0x1.3c995b0b80385p+0, -0x1.39de91a6dcf7bp-2},
    {0x1.30d190c8864a5p+0, -0x1.01d9bf3f2b631p-2}, {0x1.25e227b0b8ea0p+0, -0x1.97c1d1b3b7af0p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.2f9e393af3c9fp-3}, {0x1.12358f08ae5bap+0, -0x1.960cbbf788d5cp-4},
    {0x1.0953f419900a7p+0, -0x1.a6f9db6475fcep-5}, {0x1.0000000000000p+0, 0x0.0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.338ca9f24f53dp-4},  {0x1.ca4b31f026aa0p-1, 0x1.476a9543891bap-3},
    {0x1.b2036576afce6p-1, 0x1.e840b4ac4e4d2p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.40645f0c6651cp-2},
    {0x1.886e6037841edp-1, 0x1.88e9c2c1b9ff8p-2},  {0x1.767dcf5534862p-1, 0x1.ce0a44eb17bccp-2}};
const double kLog2fPoly[4] = {-0x1.712b6f70a7e4dp-2, 0x1.ecabf496832e0p-2, -0x1.715479ffae3dep-1,
                              0x1.715475f35c8b8p+0};

inline int bin20(int v) { return (v * 5) >> 6; }
}  // namespace

extern "C" float oracle_log2f(float x) {
  uint32_t ix;
  std::memcpy(&ix, &x, 4);
  if (ix == 0x3f800000u) return 0.0f;
  if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
    if (ix * 2 == 0) return -INFINITY;
    if (ix == 0x7f800000u) return x;
    if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return NAN;
    float y = x * 0x1p23f;
    std::memcpy(&ix, &y, 4);
    ix -= 23u << 23;
  }
  uint32_t tmp = ix - 0x3f330000u;
  int i = (tmp >> (23 - 4)) % 16;
  uint32_t top = tmp & 0xff800000u;
  uint32_t iz = ix - top;
  int k = (int32_t)tmp >> 23;
  float zf;
  std::memcpy(&zf, &iz, 4);
  double z = zf, invc = kLog2fTab[i][0], logc = kLog2fTab[i][1];
  double r = z * invc - 1.0;
  double y0 = logc + (double)k;
  double r2 = r * r;
  double y = kLog2fPoly[1] * r + kLog2fPoly[2];
  y = kLog2fPoly[0] * r2 + y;
  double p = kLog2fPoly[3] * r + y0;
  y = y * r2 + p;
  return (float)y;
}

extern "C" void oracle_mi_histograms(const uint8_t* L, int sL, const uint8_t* R, int sR, int w, int h,
                                     int32_t* hl, int32_t* hr, int32_t* hj) {
  std::memset(hl, 0, 20 * 4);
  std::memset(hr, 0, 20 * 4);
  std::memset(hj, 0, 400 * 4);
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      int bl = bin20(L[(long)y * sL + x]), br = bin20(R[(long)y * sR + x]);
      hl[bl]++;
      hr[br]++;
      hj[bl * 20 + br]++;
    }
}

// mutual_information.cpp:55-86
extern "C" float oracle_mutual_information(const uint8_t* L, int sL, const uint8_t* R, int sR, int w, int h) {
  int32_t hl[20], hr[20], hj[400];
  oracle_mi_histograms(L, sL, R, sR, w, h, hl, hr, hj);
  const float a = (float)(1.0 / (double)(w * h));  // histL/R/Joint /= rows*cols (N of L for the joint)
  float pL[20], pR[20];
  for (int i = 0; i < 20; ++i) {
    pL[i] = (float)hl[i] * a;
    pR[i] = (float)hr[i] * a;
  }
  float MI = 0.0f;
  for (int i = 0; i < 20; ++i)
    for (int j = 0; j < 20; ++j) {
      float pJ = (float)hj[i * 20 + j] * a;
      if (pJ > 0 && pL[i] > 0 && pR[j] > 0) {
        float den = pL[i] * pR[j];
        float q = pJ / den;
        float t = pJ * oracle_log2f(q);
        MI += t;
      }
    }
  return MI;
}

// mutual_information.cpp:28-45
extern "C" float oracle_entropy(const uint8_t* img, int s, int w, int h) {
  int32_t hist[20] = {0};
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) hist[bin20(img[(long)y * s + x])]++;
  const float a = (float)(1.0 / (double)(w * h));
  float e = 0.0f;
  for (int i = 0; i < 20; ++i) {
    float p = (float)hist[i] * a;
    if (p > 0) e += p * oracle_log2f(p);
  }
  return -e;
}

extern "C" void oracle_mi_scores(const uint8_t* imgL, int sL, const uint8_t* imgR, int sR, const int32_t* xyL,
                                 const int32_t* xyR, int n, int pw, int ph, float* out) {
  for (int k = 0; k < n; ++k) {
    const uint8_t* pl = imgL + (long)xyL[2 * k + 1] * sL + xyL[2 * k];
    const uint8_t* pr = imgR + (long)xyR[2 * k + 1] * sR + xyR[2 * k];
    out[k] = oracle_mutual_information(pl, sL, pr, sR, pw, ph);
  }
}

// Exhaustive self-check of the restatement against the host libm log2f over
// the bit patterns [lo, hi) (tests/test_oracle.py runs all positive floats).
extern "C" long oracle_log2f_mismatches(uint32_t lo, uint32_t hi) {
  long bad = 0;
#pragma omp parallel for reduction(+ : bad) schedule(static)
  for (long u = (long)lo; u < (long)hi; ++u) {
    uint32_t v = (uint32_t)u;
    float x;
    std::memcpy(&x, &v, 4);
    float a = log2f(x), b = oracle_log2f(x);
    if (std::memcmp(&a, &b, 4) != 0) bad++;
  }
  return bad;
}


// ---- A3: src/core/mutual_information.cpp:14-25 (comparePC), written with
// the reference's own expressions: pow(float, 2) promotes to double (C++11),
// sqrt(float) is the float overload; compiled without FMA contraction.
static float compare_pc_one(const float* PC1, const float* PC2, int rows, int cols) {
  float sum = 0, sum1 = 0, sum2 = 0;
  for (int i = 0; i < rows; i++)
    for (int j = 0; j < cols; j++) {
      sum += PC1[i * cols + j] * PC2[i * cols + j];
      sum1 += std::pow(PC1[i * cols + j], 2);
      sum2 += std::pow(PC2[i * cols + j], 2);
    }
  return sum / std::sqrt(sum1 * sum2);
}

extern "C" void oracle_compare_pc(const float* A, const float* B, int n, int rows, int cols, float* out) {
  for (int k = 0; k < n; ++k) out[k] = compare_pc_one(A + (long)k * rows * cols, B + (long)k * rows * cols, rows, cols);
}

// :136-140 applyCCOEFFNormed.  (r - 1) / N * sum(r) is one OpenCV MatExpr
// (alpha = sum / N, shift = -sum / N in double) evaluated by convertTo, i.e.
// float src * (float)alpha + (float)shift (fused in OpenCV's SIMD path);
// cv::sum accumulates in double.  OpenCV is not present: parity unpinned.
static float ccoeff_one(const float* r1, const float* r2, int npx) {
  double s1 = 0, s2 = 0;
  for (int i = 0; i < npx; ++i) { s1 += (double)r1[i]; s2 += (double)r2[i]; }
  const double inv = 1.0 / (double)npx;
  const float a1 = (float)(inv * s1), b1 = (float)(-inv * s1), a2 = (float)(inv * s2), b2 = (float)(-inv * s2);
  double s12 = 0, s11 = 0, s22 = 0;
  for (int i = 0; i < npx; ++i) {
    const float u = std::fma(r1[i], a1, b1), v = std::fma(r2[i], a2, b2);
    s12 += (double)(u * v);
    s11 += (double)(u * u);
    s22 += (double)(v * v);
  }
  return (float)(s12 / std::sqrt(s11 * s22));
}

extern "C" void oracle_ccoeff_normed(const float* A, const float* B, int n, int rows, int cols, float* out) {
  for (int k = 0; k < n; ++k) out[k] = ccoeff_one(A + (long)k * rows * cols, B + (long)k * rows * cols, rows * cols);
}

// :48-53 quantise, the reference's expression per pixel (row by row for a strided image)
extern "C" void oracle_quantise(uint8_t* img, int stride, int w, int h, int lo, int hi) {
  const std::pair<uint8_t, uint8_t> range{(uint8_t)lo, (uint8_t)hi};
  for (int y = 0; y < h; ++y) {
    uint8_t* img_ptr = img + (long)y * stride;
    for (int i = 0; i < w; i++)
      img_ptr[i] = (uint8_t)(img_ptr[i] / (256 / (int)(range.second - range.first))) + range.first;
  }
}
