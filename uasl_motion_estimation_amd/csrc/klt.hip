// klt.hip — pyramidal Lucas-Kanade feature tracking.
//
// The reference contains NO tracker (the app that drove it is absent); this
// is the build-defined tracker, specified by oracle/klt.cpp (the CPU
// restatement used as its checker).  MI355X design:
//  * pyramids (pyrDown 5x5 binomial) and Scharr derivatives built once per
//    image by 2-D kernels; levels resident in HBM;
//  * one wavefront per feature: the 21x21 window is spread over 64 lanes
//    (7 pixels each), template values / gradients stay in VGPRs across the
//    LK iterations, the 2x2 normal matrix and the mismatch vector are exact
//    wave sums (int32 DPP stages while the partial sums fit, then FP64 on
//    integers: order-independent and bit-identical to the serial restatement);
//  * the 2x2 solve runs redundantly in every lane; the window position, its
//    bilinear weights and the region tests are wave-uniform and kept in
//    scalar registers (the weight packing runs on the scalar unit).
#include <algorithm>
#include <cstring>
#include <vector>
#include "me_internal.hpp"

namespace {

__device__ __forceinline__ int refl(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) {
    if (i < 0) i = -i;
    if (i >= n) i = 2 * n - 2 - i;
  }
  return i;
}

// one pyramid level of both images (blockIdx.z: 0 prev, 1 next)
__global__ void pyr_down_kernel(const uint8_t* __restrict__ srcI, const uint8_t* __restrict__ srcJ, int w, int h,
                                int ss, uint8_t* __restrict__ dstI, uint8_t* __restrict__ dstJ, int dw, int dh,
                                int ds) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y * blockDim.y + threadIdx.y;
  if (x >= dw || y >= dh) return;
  const uint8_t* src = blockIdx.z ? srcJ : srcI;
  uint8_t* dst = blockIdx.z ? dstJ : dstI;
  const int k[5] = {1, 4, 6, 4, 1};
  int s = 0;
#pragma unroll
  for (int a = 0; a < 5; ++a) {
    const uint8_t* row = src + (long)refl(2 * y + a - 2, h) * ss;
    int rs = 0;
#pragma unroll
    for (int b = 0; b < 5; ++b) rs += k[b] * row[refl(2 * x + b - 2, w)];
    s += k[a] * rs;
  }
  dst[(long)y * ds + x] = (uint8_t)((s + 128) >> 8);
}

constexpr int kMaxLevels = 8;
struct Pyr {
  int nl;
  int w[kMaxLevels], h[kMaxLevels];
  int is[kMaxLevels];                // row stride of I[l] and J[l] (level 0: the caller's images)
  const uint8_t* I[kMaxLevels];      // prev levels (stride = w)
  const int16_t* dx[kMaxLevels];
  const int16_t* dy[kMaxLevels];
  const uint8_t* J[kMaxLevels];      // next levels
};

// Scharr derivatives of every level of the prev pyramid in one launch (blockIdx.z = level)
__global__ void scharr_levels_kernel(Pyr P) {
  const int l = blockIdx.z;
  const int w = P.w[l], h = P.h[l], stride = P.is[l];
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y * blockDim.y + threadIdx.y;
  if (x >= w || y >= h) return;
  const uint8_t* I = P.I[l];
  int16_t* dx = const_cast<int16_t*>(P.dx[l]);
  int16_t* dy = const_cast<int16_t*>(P.dy[l]);
  const uint8_t* r0 = I + (long)refl(y - 1, h) * stride;
  const uint8_t* r1 = I + (long)y * stride;
  const uint8_t* r2 = I + (long)refl(y + 1, h) * stride;
  const int xm = refl(x - 1, w), xp = refl(x + 1, w);
  const int t0m = 3 * (r0[xm] + r2[xm]) + 10 * r1[xm], t0p = 3 * (r0[xp] + r2[xp]) + 10 * r1[xp];
  const int t1m = r2[xm] - r0[xm], t1p = r2[xp] - r0[xp], t1 = r2[x] - r0[x];
  dx[(long)y * w + x] = (int16_t)(t0p - t0m);
  dy[(long)y * w + x] = (int16_t)(3 * (t1p + t1m) + 10 * t1);
}

// Exact wave-wide sum of per-lane int32 partials: every partial sum is an
// integer below 2^53 (|b| <= 64 * 7 * 8160 * 4080, A <= 441 * 4080^2), so the
// FP64 adds are exact and the result equals the int64 sum in any order.
// Within each 16-lane row: quad xor 1, xor 2, half-mirror, mirror (DPP, VALU
// latency); then the four row sums by readlane.  All 64 lanes must be active.
template <int Ctrl>
__device__ __forceinline__ double dpp_f64(double x) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), Ctrl, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), Ctrl, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double readlane_f64(double x, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(x), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(x), l);
  return __hiloint2double(hi, lo);
}
// lanes outside row_mask read 0 (update_dpp's old value)
template <int Ctrl, int RowMask>
__device__ __forceinline__ double dpp_f64_masked(double x) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), Ctrl, RowMask, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), Ctrl, RowMask, 0xf, false);
  return __hiloint2double(hi, lo);
}
template <int Ctrl>
__device__ __forceinline__ int dpp_i32k(int x) {
  return __builtin_amdgcn_mov_dpp(x, Ctrl, 0xf, 0xf, true);  // (bound_ctrl: lets the mov fold into the add)
}
// Exact wave sum of int32 lane values whose sums over any (1 << INT_STAGES)
// lanes still fit int32: the first INT_STAGES butterfly stages add in 32-bit
// integers (one DPP-sourced add each), the rest in FP64 (integers below 2^53:
// exact, so the order does not matter), the four row sums gathered in lane 63
// by row broadcasts (row_bcast15 / row_bcast31) and read once.
template <int INT_STAGES>
__device__ __forceinline__ double wave_sum_exact(int v) {
  uint32_t u = (uint32_t)v;  // (wrapping adds: no overflow for the bounded inputs, none for the compiler either)
  if (INT_STAGES >= 1) u += (uint32_t)dpp_i32k<0xB1>((int)u);   // quad_perm [1,0,3,2]
  if (INT_STAGES >= 2) u += (uint32_t)dpp_i32k<0x4E>((int)u);   // quad_perm [2,3,0,1]
  if (INT_STAGES >= 3) u += (uint32_t)dpp_i32k<0x141>((int)u);  // row_half_mirror
  if (INT_STAGES >= 4) u += (uint32_t)dpp_i32k<0x140>((int)u);  // row_mirror
  double x = (double)(int)u;
  if (INT_STAGES < 1) x += dpp_f64<0xB1>(x);
  if (INT_STAGES < 2) x += dpp_f64<0x4E>(x);
  if (INT_STAGES < 3) x += dpp_f64<0x141>(x);
  if (INT_STAGES < 4) x += dpp_f64<0x140>(x);  // every lane of a row: the row's sum
  x += dpp_f64_masked<0x142, 0xA>(x);          // rows 1, 3 += rows 0, 2 (row_bcast15)
  x += dpp_f64_masked<0x143, 0xC>(x);          // rows 2, 3 += row 1 (row_bcast31): lane 63 holds the total
  return readlane_f64(x, 63);
}
// two sums, stage by stage (the second fills the first's DPP wait states)
template <int INT_STAGES>
__device__ __forceinline__ void wave_sum2_exact(int v1, int v2, double& s1, double& s2) {
  uint32_t u1 = (uint32_t)v1, u2 = (uint32_t)v2;
  if (INT_STAGES >= 1) {
    u1 += (uint32_t)dpp_i32k<0xB1>((int)u1);
    u2 += (uint32_t)dpp_i32k<0xB1>((int)u2);
  }
  if (INT_STAGES >= 2) {
    u1 += (uint32_t)dpp_i32k<0x4E>((int)u1);
    u2 += (uint32_t)dpp_i32k<0x4E>((int)u2);
  }
  if (INT_STAGES >= 3) {
    u1 += (uint32_t)dpp_i32k<0x141>((int)u1);
    u2 += (uint32_t)dpp_i32k<0x141>((int)u2);
  }
  static_assert(INT_STAGES == 3, "the row_mirror stage below is the FP64 one");
  double x1 = (double)(int)u1, x2 = (double)(int)u2;
  x1 += dpp_f64<0x140>(x1);
  x2 += dpp_f64<0x140>(x2);
  x1 += dpp_f64_masked<0x142, 0xA>(x1);
  x2 += dpp_f64_masked<0x142, 0xA>(x2);
  x1 += dpp_f64_masked<0x143, 0xC>(x1);
  x2 += dpp_f64_masked<0x143, 0xC>(x2);
  s1 = readlane_f64(x1, 63);
  s2 = readlane_f64(x2, 63);
}
// 32-bit form: every per-pixel product below fits in int32 (|I w| <= 255 * 16384,
// |DX w| <= 4080 * 16384, |diff * grad| <= 8160 * 4080, 7 pixels per lane), so
// only the wave-wide sums need more than 32 bits -- same integers as the 64-bit form.
__device__ __forceinline__ int descale32(int v, int n) { return (v + (1 << (n - 1))) >> n; }

constexpr int kMaxWinPx = 7;  // pixels per lane: ceil(21*21/64)
// Next-image region staged in LDS per wave: 32x32 pixels around the current
// window (the (win+1)^2 bilinear footprint plus a margin), so the LK
// iterations read LDS instead of making an L2 round trip each.  When the
// window walks out of the region it is restaged around the new position;
// levels narrower or shorter than the region read global memory directly.
// The region holds one 32-bit word per pixel with its whole bilinear
// footprint -- bytes J(x, y), J(x+1, y), J(x, y+1), J(x+1, y+1) -- so a tap
// set is one aligned ds_read_b32 (the byte form's taps were pairs of bytes
// at odd addresses, merged into unaligned ds_read_u16: SQ_LDS_UNALIGNED_STALL
// matched the LDS-active cycles and the LDS waits were 20 % of the wave's
// time, profiles/r05_klt_sq_counters_before.txt; after: r05_klt_sq_counters_after.txt).  Same pixel values either way, so
// results are unchanged bit for bit.
constexpr int kRegion = 32;

// wave-local ordering of this wave's LDS region (no cross-wave sharing)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// lane = (row y = lane>>1, half lane&1): the 16 footprint words of row
// ry0 + y, columns 16 (lane & 1) .. + 15.  Footprints reaching past the
// region's last row or column (x or y = 31, never a tap of a window inside
// the region) are built from clamped addresses: defined, never read.
__device__ __forceinline__ void stage_region(uint32_t* reg, const uint8_t* __restrict__ J, int SI, int rx0, int ry0,
                                             int lane) {
  const int y = lane >> 1, x0 = 16 * (lane & 1);
  const uint8_t* r0 = J + (long)(ry0 + y) * SI + rx0 + x0;
  const uint8_t* r1 = J + (long)(ry0 + min(y + 1, kRegion - 1)) * SI + rx0 + x0;
  // the row segment's 16 bytes as four (unaligned) dwords, the 17th byte
  // (clamped to the region) on its own; each footprint word picks bytes
  // k, k + 1 of both rows (alignbyte + perm)
  uint32_t d0[5], d1[5];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    __builtin_memcpy(&d0[i], r0 + 4 * i, 4);
    __builtin_memcpy(&d1[i], r1 + 4 * i, 4);
  }
  const int x16 = min(x0 + 16, kRegion - 1) - x0;
  d0[4] = r0[x16];
  d1[4] = r1[x16];
  uint32_t w[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t a0 = __builtin_amdgcn_alignbyte(d0[k / 4 + 1], d0[k / 4], k % 4);  // row y: bytes k .. k + 3
    const uint32_t a1 = __builtin_amdgcn_alignbyte(d1[k / 4 + 1], d1[k / 4], k % 4);  // row y + 1
    w[k] = __builtin_amdgcn_perm(a1, a0, 0x05040100u);  // J(k), J(k+1), J'(k), J'(k+1)
  }
  wave_lds_sync();  // earlier reads of the previous region are done
  uint4* dst = reinterpret_cast<uint4*>(reg + y * kRegion + x0);
#pragma unroll
  for (int k = 0; k < 4; ++k) dst[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
  wave_lds_sync();
}

// Every lane loads all of its window pixels unconditionally (pixels past the
// window alias pixel 0 and are masked afterwards), so the loads of one step
// issue back to back behind a single wait instead of one round trip per pixel.
__global__ __launch_bounds__(256) void klt_kernel(Pyr P, const float* __restrict__ pin, float* __restrict__ pout,
                                                  uint8_t* __restrict__ status, int n, int win, int max_iters,
                                                  double eps2, double min_eig) {
  __shared__ __attribute__((aligned(16))) uint32_t regions[4][kRegion * kRegion];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // (scalar: the feature, its region and
  const int f = blockIdx.x * 4 + wv;                                 // its window origin live in scalar registers)
  if (f >= n) return;  // wave-uniform
  uint32_t* reg = regions[wv];
  const int half = (win - 1) / 2, npx = win * win;
  const double FLT_SCALE = 1.0 / (1 << 20);
  uint8_t st = 1;
  float nx = 0, ny = 0;
  int iv[kMaxWinPx], ixv[kMaxWinPx], iyv[kMaxWinPx];
  int wy[kMaxWinPx], wx[kMaxWinPx], roff[kMaxWinPx];  // window coordinates of this lane's pixels, region byte offsets
  bool wok[kMaxWinPx];
#pragma unroll
  for (int q = 0; q < kMaxWinPx; ++q) {
    const int k = lane + 64 * q;
    wok[q] = k < npx;
    const int kk = wok[q] ? k : 0;
    wy[q] = kk / win;
    wx[q] = kk - wy[q] * win;
    roff[q] = 4 * (wy[q] * kRegion + wx[q]);  // (bytes)
    asm volatile("" : "+v"(roff[q]));  // kept in a register: one add per tap address in the LK loop
  }
  const float px0 = pin[2 * f], py0 = pin[2 * f + 1];
  for (int L = P.nl - 1; L >= 0; --L) {
    const int W = P.w[L], H = P.h[L], SI = P.is[L];
    const float sc = 1.0f / (float)(1 << L);
    const float px = px0 * sc, py = py0 * sc;
    if (L == P.nl - 1) {
      nx = px;
      ny = py;
    } else {
      nx = nx * 2.0f;
      ny = ny * 2.0f;
    }
    const float pxw = px - (float)half, pyw = py - (float)half;
    int iv0[2] = {(int)floorf(pxw), (int)floorf(pyw)};
    asm volatile("" : "+v"(iv0[0]), "+v"(iv0[1]));
    const int ix0 = __builtin_amdgcn_readfirstlane(iv0[0]), iy0 = __builtin_amdgcn_readfirstlane(iv0[1]);
    if (ix0 < 0 || iy0 < 0 || ix0 + win >= W || iy0 + win >= H) {
      if (L == 0) st = 0;
      continue;
    }
    const float a = pxw - (float)ix0, b = pyw - (float)iy0;
    const int iw00 = (int)rintf((1.f - a) * (1.f - b) * 16384.f);
    const int iw01 = (int)rintf(a * (1.f - b) * 16384.f);
    const int iw10 = (int)rintf((1.f - a) * b * 16384.f);
    const int iw11 = 16384 - iw00 - iw01 - iw10;
    // window origin as scalar base pointers, the lane's pixels as 32-bit
    // offsets from them (scalar-base loads: no 64-bit address per tap)
    const uint8_t* I = P.I[L] + (long)iy0 * SI + ix0;
    const char* DX = reinterpret_cast<const char*>(P.dx[L] + (long)iy0 * W + ix0);
    const char* DY = reinterpret_cast<const char*>(P.dy[L] + (long)iy0 * W + ix0);
    // horizontal tap pairs as one (unaligned) load each: I(x), I(x+1) as 16
    // bits, DX / DY(x), (x+1) as 32 bits, split in registers
    auto ld_u16 = [](const uint8_t* base, uint32_t off) {
      uint16_t v;
      __builtin_memcpy(&v, base + off, 2);
      return (uint32_t)v;
    };
    auto ld_u32 = [](const char* base, uint32_t off) {
      uint32_t v;
      __builtin_memcpy(&v, base + off, 4);
      return v;
    };
    int i4[kMaxWinPx][4], x4[kMaxWinPx][4], y4[kMaxWinPx][4];
#pragma unroll
    for (int q = 0; q < kMaxWinPx; ++q) {
      const uint32_t o = 2u * (uint32_t)(wy[q] * W + wx[q]), oi = (uint32_t)(wy[q] * SI + wx[q]);  // (bytes)
      const uint32_t oW = o + 2u * (uint32_t)W, oS = oi + (uint32_t)SI;
      const uint32_t i01 = ld_u16(I, oi), i23 = ld_u16(I, oS);
      const uint32_t x01 = ld_u32(DX, o), x23 = ld_u32(DX, oW), y01 = ld_u32(DY, o), y23 = ld_u32(DY, oW);
      i4[q][0] = (int)(i01 & 255u);
      i4[q][1] = (int)(i01 >> 8);
      i4[q][2] = (int)(i23 & 255u);
      i4[q][3] = (int)(i23 >> 8);
      x4[q][0] = (int)(int16_t)(x01 & 0xffffu);
      x4[q][1] = (int)x01 >> 16;
      x4[q][2] = (int)(int16_t)(x23 & 0xffffu);
      x4[q][3] = (int)x23 >> 16;
      y4[q][0] = (int)(int16_t)(y01 & 0xffffu);
      y4[q][1] = (int)y01 >> 16;
      y4[q][2] = (int)(int16_t)(y23 & 0xffffu);
      y4[q][3] = (int)y23 >> 16;
    }
    int a11l = 0, a12l = 0, a22l = 0;
#pragma unroll
    for (int q = 0; q < kMaxWinPx; ++q) {
      const int v = i4[q][0] * iw00 + i4[q][1] * iw01 + i4[q][2] * iw10 + i4[q][3] * iw11;
      const int gx = x4[q][0] * iw00 + x4[q][1] * iw01 + x4[q][2] * iw10 + x4[q][3] * iw11;
      const int gy = y4[q][0] * iw00 + y4[q][1] * iw01 + y4[q][2] * iw10 + y4[q][3] * iw11;
      iv[q] = wok[q] ? descale32(v, 9) : 0;
      ixv[q] = wok[q] ? descale32(gx, 14) : 0;  // masked pixels contribute nothing below
      iyv[q] = wok[q] ? descale32(gy, 14) : 0;
      a11l += ixv[q] * ixv[q];
      a12l += ixv[q] * iyv[q];
      a22l += iyv[q] * iyv[q];
    }
    // (|ix|, |iy| <= 4080, 7 pixels per lane: a 16-lane sum of the products
    // is at most 1.87e9, inside int32 -- four integer stages)
    const double a11 = wave_sum_exact<4>(a11l) * FLT_SCALE, a12 = wave_sum_exact<4>(a12l) * FLT_SCALE,
                 a22 = wave_sum_exact<4>(a22l) * FLT_SCALE;
    const double D = a11 * a22 - a12 * a12;
    const double minEig = (a22 + a11 - sqrt((a11 - a22) * (a11 - a22) + 4.0 * a12 * a12)) / (2.0 * win * win);
    if (minEig < min_eig || D < 1.1920928955078125e-07) {
      if (L == 0) st = 0;
      continue;
    }
    const double Dinv = 1.0 / D;
    float nxw = nx - (float)half, nyw = ny - (float)half;
    float pdx = 0, pdy = 0;
    const uint8_t* J = P.J[L];
    const bool staged = W >= kRegion && H >= kRegion && win + 1 <= kRegion;
    int rx0 = -(1 << 30), ry0 = -(1 << 30);  // no region yet
    for (int j = 0; j < max_iters; ++j) {
      // (the position, its weights and the region test are wave-uniform -- every
      // lane runs the same arithmetic on the same values: scalar registers)
      const int jx0 = __builtin_amdgcn_readfirstlane((int)floorf(nxw));
      const int jy0 = __builtin_amdgcn_readfirstlane((int)floorf(nyw));
      if (jx0 < 0 || jy0 < 0 || jx0 + win >= W || jy0 + win >= H) {
        if (L == 0) st = 0;
        break;
      }
      const float c = nxw - (float)jx0, d = nyw - (float)jy0;
      // (converted in a vector register, then read once into a scalar one: the
      // weight packing below runs on the scalar unit)
      int jv[3] = {(int)rintf((1.f - c) * (1.f - d) * 16384.f), (int)rintf(c * (1.f - d) * 16384.f),
                   (int)rintf((1.f - c) * d * 16384.f)};
      asm volatile("" : "+v"(jv[0]), "+v"(jv[1]), "+v"(jv[2]));
      const int jw00 = __builtin_amdgcn_readfirstlane(jv[0]);
      const int jw01 = __builtin_amdgcn_readfirstlane(jv[1]);
      const int jw10 = __builtin_amdgcn_readfirstlane(jv[2]);
      const int jw11 = 16384 - jw00 - jw01 - jw10;
      // the bilinear sum of a footprint word f (bytes J00 J01 J10 J11) as two
      // packed u8 dot products: w = 128 (w >> 7) + (w & 127), both halves fit
      // a byte (0 <= w <= 16384), the sums are exact in 32 bits.  jw11 =
      // 16384 - the other three comes out -1 in ~1e-5 of the iterations (the
      // three roundings): the dot products then take 0 for it and J11 is
      // subtracted afterwards (a wave-uniform branch; the same integer)
      const int w11 = max(jw11, 0);
      const uint32_t whp = (uint32_t)(jw00 >> 7) | ((uint32_t)(jw01 >> 7) << 8) | ((uint32_t)(jw10 >> 7) << 16) |
                           ((uint32_t)(w11 >> 7) << 24);
      const uint32_t wlp = (uint32_t)(jw00 & 127) | ((uint32_t)(jw01 & 127) << 8) | ((uint32_t)(jw10 & 127) << 16) |
                           ((uint32_t)(w11 & 127) << 24);
      uint32_t f4[kMaxWinPx];
      if (staged) {
        if (jx0 < rx0 || jy0 < ry0 || jx0 + win >= rx0 + kRegion || jy0 + win >= ry0 + kRegion) {
          // centre the region on the window, clamped inside the level
          rx0 = min(max(jx0 - (kRegion - win - 1) / 2, 0), W - kRegion);
          ry0 = min(max(jy0 - (kRegion - win - 1) / 2, 0), H - kRegion);
          stage_region(reg, J, SI, rx0, ry0, lane);
        }
        const char* R0 = reinterpret_cast<const char*>(reg + (jy0 - ry0) * kRegion + (jx0 - rx0));
#pragma unroll
        for (int q = 0; q < kMaxWinPx; ++q) f4[q] = *reinterpret_cast<const uint32_t*>(R0 + roff[q]);
      } else {
#pragma unroll
        for (int q = 0; q < kMaxWinPx; ++q) {
          const uint8_t* r = J + (long)(jy0 + wy[q]) * SI + jx0 + wx[q];
          f4[q] = (uint32_t)r[0] | ((uint32_t)r[1] << 8) | ((uint32_t)r[SI] << 16) | ((uint32_t)r[SI + 1] << 24);
        }
      }
      int vq[kMaxWinPx];
#pragma unroll
      for (int q = 0; q < kMaxWinPx; ++q)
        vq[q] = (int)((__builtin_amdgcn_udot4(f4[q], whp, 0u, false) << 7) + __builtin_amdgcn_udot4(f4[q], wlp, 0u, false));
      if (jw11 < 0) {  // (wave-uniform, rare) jw11 = -1
#pragma unroll
        for (int q = 0; q < kMaxWinPx; ++q) vq[q] -= (int)(f4[q] >> 24);
      }
      int b1l = 0, b2l = 0;
#pragma unroll
      for (int q = 0; q < kMaxWinPx; ++q) {
        const int diff = descale32(vq[q], 9) - iv[q];
        b1l += diff * ixv[q];  // ixv = iyv = 0 on masked pixels
        b2l += diff * iyv[q];
      }
      // (|diff| <= 8160, |ix| <= 4080: an 8-lane sum is at most 1.87e9 -- three integer stages)
      double b1d, b2d;
      wave_sum2_exact<3>(b1l, b2l, b1d, b2d);
      b1d *= FLT_SCALE;
      b2d *= FLT_SCALE;
      const float ddx = (float)((a12 * b2d - a22 * b1d) * Dinv);
      const float ddy = (float)((a12 * b1d - a11 * b2d) * Dinv);
      nxw += ddx;
      nyw += ddy;
      nx = nxw + (float)half;
      ny = nyw + (float)half;
      if ((double)ddx * ddx + (double)ddy * ddy <= eps2) break;
      if (j > 0 && fabsf(ddx + pdx) < 0.01f && fabsf(ddy + pdy) < 0.01f) {
        nx -= ddx * 0.5f;
        ny -= ddy * 0.5f;
        break;
      }
      pdx = ddx;
      pdy = ddy;
    }
  }
  if (lane == 0) {
    pout[2 * f] = nx;
    pout[2 * f + 1] = ny;
    status[f] = st;
  }
}

}  // namespace

extern "C" void me_klt_default_params(me_klt_params* p) {
  p->win = 21;
  p->max_level = 3;
  p->max_iters = 30;
  p->eps = 0.01;
  p->min_eig = 1e-4;
}

// Builds the pyramids of prev (with derivatives) and next into scratch.
static int build_pyramids(me_ctx* c, const uint8_t* dprev, const uint8_t* dnext, int w, int h, int stride, int nl,
                          Pyr& P) {
  std::vector<int> W(nl), H(nl);
  W[0] = w;
  H[0] = h;
  for (int l = 1; l < nl; ++l) {
    W[l] = (W[l - 1] + 1) / 2;
    H[l] = (H[l - 1] + 1) / 2;
  }
  size_t bytes = 0;
  for (int l = 0; l < nl; ++l) bytes += 2 * (size_t)W[l] * H[l] + 4 * (size_t)W[l] * H[l] + 64;
  void* base;
  ME_TRY(me_scratch(c, SLOT_KLT_PYR, bytes + 1024, &base));
  char* p = (char*)base;
  P.nl = nl;
  for (int l = 0; l < nl; ++l) {
    P.w[l] = W[l];
    P.h[l] = H[l];
    size_t npx = (size_t)W[l] * H[l];
    if (l == 0) {  // level 0 is read in place from the caller's images
      P.I[0] = dprev;
      P.J[0] = dnext;
      P.is[0] = stride;
    } else {
      P.I[l] = (const uint8_t*)p;
      p += (npx + 63) / 64 * 64;
      P.J[l] = (const uint8_t*)p;
      p += (npx + 63) / 64 * 64;
      P.is[l] = W[l];
    }
    P.dx[l] = (int16_t*)p;
    p += (2 * npx + 63) / 64 * 64;
    P.dy[l] = (int16_t*)p;
    p += (2 * npx + 63) / 64 * 64;
  }
  hipStream_t s = c->stream;
  me_ktimer t(c, ME_KT_PYR);
  for (int l = 1; l < nl; ++l) {  // both images per launch
    dim3 blk(32, 8), grd((W[l] + 31) / 32, (H[l] + 7) / 8, 2);
    hipLaunchKernelGGL(pyr_down_kernel, grd, blk, 0, s, P.I[l - 1], P.J[l - 1], W[l - 1], H[l - 1], P.is[l - 1],
                       const_cast<uint8_t*>(P.I[l]), const_cast<uint8_t*>(P.J[l]), W[l], H[l], P.is[l]);
  }
  {  // derivatives of every prev level in one launch
    dim3 blk(32, 8), grd((W[0] + 31) / 32, (H[0] + 7) / 8, nl);
    hipLaunchKernelGGL(scharr_levels_kernel, grd, blk, 0, s, P);
  }
  return me_check_launch(c, "pyramid kernels");
}

extern "C" int me_klt_track(me_ctx* c, me_mem mem, const uint8_t* prev, const uint8_t* next, int w, int h,
                            int stride, const float* pin, float* pout, uint8_t* status, int n,
                            const me_klt_params* kp) {
  me_range range_("me_klt_track");
  if (!c || !kp) return ME_ERR_INVALID;
  ME_CHECK(c, w > 0 && h > 0 && stride >= w && n >= 0, "me_klt_track: bad image");
  ME_CHECK(c, kp->win >= 3 && (kp->win & 1) && kp->win * kp->win <= 64 * kMaxWinPx,
           "me_klt_track: window must be odd and <= 21");
  ME_CHECK(c, kp->max_level >= 0 && kp->max_level < kMaxLevels, "me_klt_track: max_level out of range");
  ME_HIP(c, hipSetDevice(c->device));
  const int nl = kp->max_level + 1;
  const uint8_t *dprev = prev, *dnext = next;
  const float* dpin = pin;
  float* dpout = pout;
  uint8_t* dst = status;
  if (mem == ME_HOST) {
    void *a, *b, *pts;
    size_t bytes = (size_t)stride * (h - 1) + w;
    ME_TRY(me_scratch(c, SLOT_IMG_L, bytes, &a));
    ME_TRY(me_scratch(c, SLOT_IMG_R, bytes, &b));
    ME_TRY(me_scratch(c, SLOT_KLT_PTS, 17 * (size_t)std::max(n, 1) + 64, &pts));
    ME_HIP(c, hipMemcpyAsync(a, prev, bytes, hipMemcpyHostToDevice, c->stream));
    ME_HIP(c, hipMemcpyAsync(b, next, bytes, hipMemcpyHostToDevice, c->stream));
    dprev = (const uint8_t*)a;
    dnext = (const uint8_t*)b;
    dpin = (const float*)pts;
    dpout = (float*)pts + 2 * (size_t)std::max(n, 1);
    dst = (uint8_t*)((float*)pts + 4 * (size_t)std::max(n, 1));
    if (n) ME_HIP(c, hipMemcpyAsync((void*)dpin, pin, 8 * (size_t)n, hipMemcpyHostToDevice, c->stream));
  }
  Pyr P;
  ME_TRY(build_pyramids(c, dprev, dnext, w, h, stride, nl, P));
  if (n > 0) {
    me_ktimer t(c, ME_KT_KLT);
    hipLaunchKernelGGL(klt_kernel, dim3((n + 3) / 4), dim3(256), 0, c->stream, P, dpin, dpout, dst, n, kp->win,
                       kp->max_iters, kp->eps * kp->eps, kp->min_eig);
  }
  ME_TRY(me_check_launch(c, "klt_kernel"));
  if (mem == ME_HOST) {
    if (n) {
      ME_HIP(c, hipMemcpyAsync(pout, dpout, 8 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
      ME_HIP(c, hipMemcpyAsync(status, dst, (size_t)n, hipMemcpyDeviceToHost, c->stream));
    }
    ME_HIP(c, hipStreamSynchronize(c->stream));
  }
  return ME_OK;
}
