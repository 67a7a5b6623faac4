// oracle/nms.cpp — TEST INFRASTRUCTURE: CPU restatement of
// me::nonMaxSupScanline3x3 (src/core/feature_types.cpp:253-351): 8-connected
// scanline non-maximum suppression on a CV_64F response map with two rolling
// skip rows.  Maxima are emitted in scan order as
// (row + 0.5 + dr, col + 0.5 + dc) with the parabola-free sub-pixel offsets
// of the reference.  Parity unpinned (see oracle.h).
#include <cstring>
#include <vector>
#include "oracle.h"

extern "C" int oracle_nms_scanline3x3(const double* in, int w, int h, uint8_t* out, double* maxima, int cap) {
  std::memset(out, 0, (size_t)w * h);
  std::vector<uint8_t> skip(2 * (size_t)w, 0);
  int cur = 0, next = 1, n = 0;
  for (int r = 1; r < h - 1; r++) {
    int c = 1;
    uint8_t* po = out + (size_t)r * w;
    const double* pi = in + (size_t)r * w;
    while (c < w - 1) {
      uint8_t* ps = &skip[(size_t)cur * w];
      if (ps[c]) { c++; continue; }
      if (pi[c] <= pi[c + 1]) {
        c++;
        while (c < w - 1 && pi[c] <= pi[c + 1]) c++;
        if (c == w - 1) break;
      } else if (pi[c] <= pi[c - 1]) {
        c++;
        continue;
      }
      ps[c + 1] = 1;
      ps = &skip[(size_t)next * w];
      const double* pd = in + (size_t)(r + 1) * w;
      if (pi[c] <= pd[c - 1]) { c++; continue; }
      ps[c - 1] = 1;
      if (pi[c] <= pd[c]) { c++; continue; }
      ps[c] = 1;
      if (pi[c] <= pd[c + 1]) { c++; continue; }
      ps[c + 1] = 1;
      const double* pu = in + (size_t)(r - 1) * w;
      if (pi[c] <= pu[c - 1]) { c++; continue; }
      if (pi[c] <= pu[c]) { c++; continue; }
      if (pi[c] <= pu[c + 1]) { c++; continue; }
      po[c] = 255;
      double sub_v = c + 0.5 + (pi[c + 1] - pi[c - 1]) / (pi[c - 1] + pi[c] + pi[c + 1]);
      double sub_u = r + 0.5 + (pd[c] - pu[c]) / (pu[c] + pi[c] + pd[c]);
      if (n < cap) { maxima[2 * n] = sub_u; maxima[2 * n + 1] = sub_v; }
      n++;
      c++;
    }
    int t = cur; cur = next; next = t;
    std::memset(&skip[(size_t)next * w], 0, w);
  }
  return n;
}
