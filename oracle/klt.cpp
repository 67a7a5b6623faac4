// oracle/klt.cpp — TEST INFRASTRUCTURE: CPU restatement of the build-defined
// pyramidal Lucas-Kanade tracker.  The reference has NO
// KLT (the tracking app is absent from the repo), so there is no reference
// file to cite: the algorithm is OpenCV's calcOpticalFlowPyrLK structure
// (Bouguet) with an integer/fixed-point formulation chosen so that the device
// kernel and this restatement agree bit for bit independently of reduction
// order:
//   * pyrDown: 5x5 binomial [1 4 6 4 1]^2 / 256, reflect-101, (s+128)>>8.
//   * Scharr derivatives: 3/10/3 smoothing, reflect-101, int16.
//   * bilinear weights iw = rint(w * 2^14) (iw11 = 2^14 - others), template
//     values descaled by 9 bits, derivatives by 14 bits, all products summed
//     in int64 (exact, order independent).
//   * 2x2 solve and position updates in double/float with fixed op order.
// Parity unpinned by construction (no reference implementation exists).
#include <cmath>
#include <cstring>
#include <vector>
#include "oracle.h"

namespace {
inline int refl(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) { if (i < 0) i = -i; if (i >= n) i = 2 * n - 2 - i; }
  return i;
}
inline int descale(long v, int n) { return (int)((v + (1L << (n - 1))) >> n); }

struct Level { int w, h; std::vector<uint8_t> I; std::vector<int16_t> dx, dy; };

void build(const uint8_t* img, int w, int h, int stride, int maxL, std::vector<Level>& L, bool deriv) {
  L.resize(maxL + 1);
  L[0].w = w; L[0].h = h; L[0].I.resize((size_t)w * h);
  for (int y = 0; y < h; ++y) std::memcpy(&L[0].I[(size_t)y * w], img + (size_t)y * stride, w);
  for (int l = 1; l <= maxL; ++l) {
    L[l].w = (L[l - 1].w + 1) / 2; L[l].h = (L[l - 1].h + 1) / 2;
    L[l].I.resize((size_t)L[l].w * L[l].h);
    oracle_pyr_down(L[l - 1].I.data(), L[l - 1].w, L[l - 1].h, L[l - 1].w, L[l].I.data(), L[l].w, L[l].h, L[l].w);
  }
  if (deriv)
    for (int l = 0; l <= maxL; ++l) {
      L[l].dx.resize((size_t)L[l].w * L[l].h); L[l].dy.resize((size_t)L[l].w * L[l].h);
      oracle_scharr(L[l].I.data(), L[l].w, L[l].h, L[l].w, L[l].dx.data(), L[l].dy.data());
    }
}
}  // namespace

extern "C" void oracle_pyr_down(const uint8_t* src, int w, int h, int ss, uint8_t* dst, int dw, int dh, int ds) {
  static const int k[5] = {1, 4, 6, 4, 1};
  for (int y = 0; y < dh; ++y)
    for (int x = 0; x < dw; ++x) {
      int s = 0;
      for (int a = 0; a < 5; ++a) {
        const uint8_t* row = src + (size_t)refl(2 * y + a - 2, h) * ss;
        int rs = 0;
        for (int b = 0; b < 5; ++b) rs += k[b] * row[refl(2 * x + b - 2, w)];
        s += k[a] * rs;
      }
      dst[(size_t)y * ds + x] = (uint8_t)((s + 128) >> 8);
    }
}

extern "C" void oracle_scharr(const uint8_t* I, int w, int h, int stride, int16_t* dx, int16_t* dy) {
  for (int y = 0; y < h; ++y) {
    const uint8_t* r0 = I + (size_t)refl(y - 1, h) * stride;
    const uint8_t* r1 = I + (size_t)y * stride;
    const uint8_t* r2 = I + (size_t)refl(y + 1, h) * stride;
    for (int x = 0; x < w; ++x) {
      int xm = refl(x - 1, w), xp = refl(x + 1, w);
      int t0m = 3 * (r0[xm] + r2[xm]) + 10 * r1[xm], t0p = 3 * (r0[xp] + r2[xp]) + 10 * r1[xp];
      int t1m = r2[xm] - r0[xm], t1p = r2[xp] - r0[xp], t1 = r2[x] - r0[x];
      dx[(size_t)y * w + x] = (int16_t)(t0p - t0m);
      dy[(size_t)y * w + x] = (int16_t)(3 * (t1p + t1m) + 10 * t1);
    }
  }
}

extern "C" void oracle_klt_track(const uint8_t* prev, const uint8_t* next, int w, int h, int stride, const float* pin,
                                 float* pout, uint8_t* status, int n, const oracle_klt_params* kp) {
  std::vector<Level> P, N;
  build(prev, w, h, stride, kp->max_level, P, true);
  build(next, w, h, stride, kp->max_level, N, false);
  const int win = kp->win, half = (win - 1) / 2;
  const double FLT_SCALE = 1.0 / (1 << 20);
  const double eps2 = kp->eps * kp->eps;
  std::vector<int> iv(win * win), ixv(win * win), iyv(win * win);
  for (int i = 0; i < n; ++i) {
    uint8_t st = 1;
    float nx = 0, ny = 0;
    for (int L = kp->max_level; L >= 0; --L) {
      const Level& lp = P[L];
      const Level& ln = N[L];
      const float sc = 1.0f / (float)(1 << L);
      float px = pin[2 * i] * sc, py = pin[2 * i + 1] * sc;
      if (L == kp->max_level) { nx = px; ny = py; }
      else { nx = nx * 2.0f; ny = ny * 2.0f; }
      float pxw = px - (float)half, pyw = py - (float)half;
      int ix0 = (int)std::floor(pxw), iy0 = (int)std::floor(pyw);
      if (ix0 < 0 || iy0 < 0 || ix0 + win >= lp.w || iy0 + win >= lp.h) { if (L == 0) st = 0; continue; }
      float a = pxw - (float)ix0, b = pyw - (float)iy0;
      int iw00 = (int)std::rint((1.f - a) * (1.f - b) * 16384.f);
      int iw01 = (int)std::rint(a * (1.f - b) * 16384.f);
      int iw10 = (int)std::rint((1.f - a) * b * 16384.f);
      int iw11 = 16384 - iw00 - iw01 - iw10;
      long A11 = 0, A12 = 0, A22 = 0;
      for (int y = 0; y < win; ++y)
        for (int x = 0; x < win; ++x) {
          size_t o = (size_t)(iy0 + y) * lp.w + ix0 + x;
          long v = (long)lp.I[o] * iw00 + (long)lp.I[o + 1] * iw01 + (long)lp.I[o + lp.w] * iw10 + (long)lp.I[o + lp.w + 1] * iw11;
          long gx = (long)lp.dx[o] * iw00 + (long)lp.dx[o + 1] * iw01 + (long)lp.dx[o + lp.w] * iw10 + (long)lp.dx[o + lp.w + 1] * iw11;
          long gy = (long)lp.dy[o] * iw00 + (long)lp.dy[o + 1] * iw01 + (long)lp.dy[o + lp.w] * iw10 + (long)lp.dy[o + lp.w + 1] * iw11;
          int k = y * win + x;
          iv[k] = descale(v, 9); ixv[k] = descale(gx, 14); iyv[k] = descale(gy, 14);
          A11 += (long)ixv[k] * ixv[k]; A12 += (long)ixv[k] * iyv[k]; A22 += (long)iyv[k] * iyv[k];
        }
      double a11 = (double)A11 * FLT_SCALE, a12 = (double)A12 * FLT_SCALE, a22 = (double)A22 * FLT_SCALE;
      double D = a11 * a22 - a12 * a12;
      double minEig = (a22 + a11 - std::sqrt((a11 - a22) * (a11 - a22) + 4.0 * a12 * a12)) / (2.0 * win * win);
      if (minEig < kp->min_eig || D < 1.1920928955078125e-07) { if (L == 0) st = 0; continue; }
      double Dinv = 1.0 / D;
      float nxw = nx - (float)half, nyw = ny - (float)half;
      float pdx = 0, pdy = 0;
      for (int j = 0; j < kp->max_iters; ++j) {
        int jx0 = (int)std::floor(nxw), jy0 = (int)std::floor(nyw);
        if (jx0 < 0 || jy0 < 0 || jx0 + win >= ln.w || jy0 + win >= ln.h) { if (L == 0) st = 0; break; }
        float c = nxw - (float)jx0, d = nyw - (float)jy0;
        int jw00 = (int)std::rint((1.f - c) * (1.f - d) * 16384.f);
        int jw01 = (int)std::rint(c * (1.f - d) * 16384.f);
        int jw10 = (int)std::rint((1.f - c) * d * 16384.f);
        int jw11 = 16384 - jw00 - jw01 - jw10;
        long b1 = 0, b2 = 0;
        for (int y = 0; y < win; ++y)
          for (int x = 0; x < win; ++x) {
            size_t o = (size_t)(jy0 + y) * ln.w + jx0 + x;
            long v = (long)ln.I[o] * jw00 + (long)ln.I[o + 1] * jw01 + (long)ln.I[o + ln.w] * jw10 + (long)ln.I[o + ln.w + 1] * jw11;
            int k = y * win + x;
            long diff = descale(v, 9) - iv[k];
            b1 += diff * ixv[k]; b2 += diff * iyv[k];
          }
        double b1d = (double)b1 * FLT_SCALE, b2d = (double)b2 * FLT_SCALE;
        float dx = (float)((a12 * b2d - a22 * b1d) * Dinv);
        float dy = (float)((a12 * b1d - a11 * b2d) * Dinv);
        nxw += dx; nyw += dy;
        nx = nxw + (float)half; ny = nyw + (float)half;
        if ((double)dx * dx + (double)dy * dy <= eps2) break;
        if (j > 0 && std::fabs(dx + pdx) < 0.01f && std::fabs(dy + pdy) < 0.01f) {
          nx -= dx * 0.5f; ny -= dy * 0.5f;
          break;
        }
        pdx = dx; pdy = dy;
      }
    }
    pout[2 * i] = nx; pout[2 * i + 1] = ny;
    status[i] = st;
  }
}
