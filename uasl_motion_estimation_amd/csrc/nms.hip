// nms.hip — exact parallel restatement of me::nonMaxSupScanline3x3
// (src/core/feature_types.cpp:253-351).
//
// The reference scan is sequential: row r's skip mask is written by row r-1's
// candidates and its plateau handling depends on the scan state (walk vs
// direct arrival, Appendix A-14).  A strict-max stencil would differ on ties,
// so this kernel runs the SAME per-row state machine for up to 1024 rows at
// once as a wavefront: row-thread t processes column c at step c + 2t, i.e. two
// columns behind the row above, which is exactly the lag after which every
// skip bit of that column has been written.  Skip bits travel through a
// 4-column ring per row in LDS; the last row of a pass hands its bits to the
// next pass through a full-width carry row.  Maxima are emitted per row and
// compacted in row-major order by a second kernel (prefix sum), giving the
// reference's output order bit for bit.
#include <algorithm>
#include <vector>
#include "me_internal.hpp"

namespace {

constexpr int kRows = 1024;

__global__ __launch_bounds__(kRows) void nms_wavefront_kernel(const double* __restrict__ in, int w, int h,
                                                              uint8_t* __restrict__ mask, int row0,
                                                              uint8_t* __restrict__ carry, int* __restrict__ rowcnt,
                                                              double* __restrict__ rowbuf, int rowcap) {
  __shared__ uint8_t ring[kRows + 1][4];
  const int t = threadIdx.x;
  for (int i = t; i < (kRows + 1) * 4; i += kRows) (&ring[0][0])[i] = 0;
  __syncthreads();
  const int r = row0 + t;
  const bool active = r <= h - 2;
  const int last_t = min(kRows - 1, h - 2 - row0);  // last active row-thread of this pass
  const double* pi = in + (long)r * w;
  const double* pd = in + (long)(r + 1) * w;
  const double* pu = in + (long)(r - 1) * w;
  bool walking = false, own_skip = false, row_done = false;
  int cnt = 0;
  double* out = rowbuf + (long)r * 2 * rowcap;
  const int steps = (w - 2) + 2 * (kRows - 1);
  for (int s = 0; s < steps; ++s) {
    const int c = s - 2 * t + 1;
    if (active && c >= 1 && c <= w - 2) {
      uint8_t sk;
      if (t == 0) sk = carry[c];  // bits from the last row of the previous pass
      else {
        sk = ring[t][c & 3];
        ring[t][c & 3] = 0;
      }
      const bool skipped = sk || own_skip;
      own_skip = false;
      if (!row_done) {
        const double v = pi[c];
        bool cand = false;
        if (walking) {
          if (v <= pi[c + 1]) {
            if (c + 1 == w - 1) row_done = true;
          } else {
            walking = false;
            cand = true;
          }
        } else if (skipped) {
        } else if (v <= pi[c + 1]) {
          if (c + 1 == w - 1) row_done = true;
          else walking = true;
        } else if (v <= pi[c - 1]) {
        } else {
          cand = true;
        }
        if (cand) {
          own_skip = true;  // ptrSkip[c+1] = 1 on the current row
          // skip bits for the next row: ring of thread t+1, or the carry row
          // (columns 0 and w-1 are never scanned: their bits are dropped)
          uint8_t* nb = (t == last_t) ? nullptr : ring[t + 1];
          auto setbit = [&](int x) {
            if (x < 1 || x > w - 2) return;
            if (nb) nb[x & 3] = 1;
            else carry[x + w] = 1;
          };
          bool ok = true;
          if (v <= pd[c - 1]) ok = false;
          else {
            setbit(c - 1);
            if (v <= pd[c]) ok = false;
            else {
              setbit(c);
              if (v <= pd[c + 1]) ok = false;
              else {
                setbit(c + 1);
                if (v <= pu[c - 1] || v <= pu[c] || v <= pu[c + 1]) ok = false;
              }
            }
          }
          if (ok) {
            mask[(long)r * w + c] = 255;
            const double sub_v = c + 0.5 + (pi[c + 1] - pi[c - 1]) / (pi[c - 1] + pi[c] + pi[c + 1]);
            const double sub_u = r + 0.5 + (pd[c] - pu[c]) / (pu[c] + pi[c] + pd[c]);
            if (cnt < rowcap) {
              out[2 * cnt] = sub_u;
              out[2 * cnt + 1] = sub_v;
            }
            cnt++;
          }
        }
      }
    }
    __syncthreads();
  }
  if (active) rowcnt[r] = cnt;
}

// carry swap: the bits written for row (row0 + 1024) become the input carry
__global__ void carry_shift_kernel(uint8_t* carry, int w) {
  for (int i = threadIdx.x + blockIdx.x * blockDim.x; i < w; i += blockDim.x * gridDim.x) {
    carry[i] = carry[i + w];
    carry[i + w] = 0;
  }
}

// exclusive scan of row counts (single workgroup) + gather in row-major order
__global__ __launch_bounds__(1024) void nms_compact_kernel(const int* __restrict__ rowcnt, int h,
                                                           const double* __restrict__ rowbuf, int rowcap,
                                                           double* __restrict__ maxima, int cap, int* __restrict__ n_out) {
  __shared__ int chunk_sum[1024];
  const int t = threadIdx.x;
  const int per = (h + 1023) / 1024;
  int s = 0;
  for (int i = 0; i < per; ++i) {
    const int r = t * per + i;
    if (r >= 1 && r <= h - 2) s += rowcnt[r];
  }
  chunk_sum[t] = s;
  __syncthreads();
  if (t == 0) {
    int acc = 0;
    for (int i = 0; i < 1024; ++i) {
      const int v = chunk_sum[i];
      chunk_sum[i] = acc;
      acc += v;
    }
    *n_out = acc;
  }
  __syncthreads();
  int off = chunk_sum[t];
  for (int i = 0; i < per; ++i) {
    const int r = t * per + i;
    if (r >= 1 && r <= h - 2) {
      const int cn = rowcnt[r];
      for (int k = 0; k < cn; ++k) {
        if (off + k < cap && k < rowcap) {
          maxima[2 * (long)(off + k)] = rowbuf[(long)r * 2 * rowcap + 2 * k];
          maxima[2 * (long)(off + k) + 1] = rowbuf[(long)r * 2 * rowcap + 2 * k + 1];
        }
      }
      off += cn;
    }
  }
}

}  // namespace

extern "C" int me_nms_scanline3x3(me_ctx* c, me_mem mem, const double* response, int w, int h, uint8_t* mask_out,
                                  double* maxima, int cap, int* n_out) {
  if (!c) return ME_ERR_INVALID;
  ME_CHECK(c, w > 0 && h > 0 && cap >= 0, "me_nms_scanline3x3: bad sizes");
  ME_HIP(c, hipSetDevice(c->device));
  const int rowcap = w / 2 + 1;
  const size_t npx = (size_t)w * h;
  size_t bytes = 8 * npx + npx + 2 * (size_t)w + 4 * (size_t)h + 16 * (size_t)rowcap * h + 16 * (size_t)std::max(cap, 1) + 64 + 5 * 256;
  void* base;
  ME_TRY(me_scratch(c, SLOT_NMS, bytes, &base));
  char* p = (char*)base;
  auto take = [&](size_t n) { char* q = p; p += (n + 255) / 256 * 256; return q; };
  const double* din = response;
  uint8_t* dmask = mask_out;
  double* dmax = maxima;
  if (mem == ME_HOST) {
    double* t = (double*)take(8 * npx);
    ME_HIP(c, hipMemcpyAsync(t, response, 8 * npx, hipMemcpyHostToDevice, c->stream));
    din = t;
    dmask = (uint8_t*)take(npx);
    dmax = (double*)take(16 * (size_t)std::max(cap, 1));
  } else {
    take(8 * npx);
    take(npx);
    take(16 * (size_t)std::max(cap, 1));
  }
  uint8_t* carry = (uint8_t*)take(2 * (size_t)w);
  int* rowcnt = (int*)take(4 * (size_t)h);
  double* rowbuf = (double*)take(16 * (size_t)rowcap * h);
  int* dn = (int*)take(64);
  ME_HIP(c, hipMemsetAsync(dmask, 0, npx, c->stream));
  ME_HIP(c, hipMemsetAsync(carry, 0, 2 * (size_t)w, c->stream));
  ME_HIP(c, hipMemsetAsync(rowcnt, 0, 4 * (size_t)h, c->stream));
  {
    me_ktimer tk(c, ME_KT_NMS);
    for (int row0 = 1; row0 <= h - 2; row0 += kRows) {
      hipLaunchKernelGGL(nms_wavefront_kernel, dim3(1), dim3(kRows), 0, c->stream, din, w, h, dmask, row0, carry,
                         rowcnt, rowbuf, rowcap);
      hipLaunchKernelGGL(carry_shift_kernel, dim3(1), dim3(256), 0, c->stream, carry, w);
    }
    hipLaunchKernelGGL(nms_compact_kernel, dim3(1), dim3(1024), 0, c->stream, (const int*)rowcnt, h,
                       (const double*)rowbuf, rowcap, dmax, cap, dn);
  }
  ME_TRY(me_check_launch(c, "nms kernels"));
  int n = 0;
  ME_HIP(c, hipMemcpyAsync(&n, dn, 4, hipMemcpyDeviceToHost, c->stream));
  ME_HIP(c, hipStreamSynchronize(c->stream));
  if (mem == ME_HOST) {
    ME_HIP(c, hipMemcpyAsync(mask_out, dmask, npx, hipMemcpyDeviceToHost, c->stream));
    if (std::min(n, cap) > 0)
      ME_HIP(c, hipMemcpyAsync(maxima, dmax, 16 * (size_t)std::min(n, cap), hipMemcpyDeviceToHost, c->stream));
    ME_HIP(c, hipStreamSynchronize(c->stream));
  }
  *n_out = n;
  return ME_OK;
}
