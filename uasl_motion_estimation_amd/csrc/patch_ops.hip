// patch_ops.hip — the remaining patch utilities of src/core/mutual_information.cpp
// (SURVEY §8a A3), batched over patch pairs:
//   me_compare_pc     <- me::comparePC (:14-25)          one lane per pair, bit-exact
//   me_ccoeff_normed  <- me::applyCCOEFFNormed (:136-140) one lane per pair (parity unpinned:
//                        OpenCV MatExpr / convertTo / cv::sum rounding restated, not linked)
//   me_quantise       <- me::quantise (:48-53)           one thread per 4 pixels, in place
// jointDistribution (:88-134) has no observable output (it draws into local
// images) and is not restated.  The sums follow the reference's row-major
// order, so the parallelism is across pairs, never inside one sum.
#include "me_internal.hpp"

namespace {

constexpr int kPatchBlock = 256;

// comparePC: float sum of products; sum1 / sum2 += pow(x, 2) promotes to double
// (C++11 pow(float, int)) and rounds back to float on each accumulation;
// sqrt(float * float) is the float overload.
__global__ __launch_bounds__(kPatchBlock) void compare_pc_kernel(const float* __restrict__ A,
                                                                 const float* __restrict__ B, int n, int npx,
                                                                 float* __restrict__ out) {
  const int k = blockIdx.x * kPatchBlock + threadIdx.x;
  if (k >= n) return;
  const float* a = A + (long)k * npx;
  const float* b = B + (long)k * npx;
  float sum = 0.f, sum1 = 0.f, sum2 = 0.f;
  for (int i = 0; i < npx; ++i) {
    const float x = a[i], y = b[i];
    sum = __fadd_rn(sum, __fmul_rn(x, y));
    sum1 = (float)__dadd_rn((double)sum1, __dmul_rn((double)x, (double)x));
    sum2 = (float)__dadd_rn((double)sum2, __dmul_rn((double)y, (double)y));
  }
  out[k] = __fdiv_rn(sum, __fsqrt_rn(__fmul_rn(sum1, sum2)));
}

// applyCCOEFFNormed: r_ = (r - 1) / N * sum(r) is one MatExpr (alpha = S / N,
// shift = -S / N, both double) assigned through convertTo (float FMA with the
// float-cast coefficients); cv::sum accumulates in double; the double ratio
// is returned as float.
__global__ __launch_bounds__(kPatchBlock) void ccoeff_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                             int n, int npx, float* __restrict__ out) {
  const int k = blockIdx.x * kPatchBlock + threadIdx.x;
  if (k >= n) return;
  const float* a = A + (long)k * npx;
  const float* b = B + (long)k * npx;
  double sa = 0.0, sb = 0.0;
  for (int i = 0; i < npx; ++i) {
    sa = __dadd_rn(sa, (double)a[i]);
    sb = __dadd_rn(sb, (double)b[i]);
  }
  const double inv = 1.0 / (double)npx;
  const float al = (float)(inv * sa), bl = (float)(-inv * sa);
  const float ar = (float)(inv * sb), br = (float)(-inv * sb);
  double s12 = 0.0, s11 = 0.0, s22 = 0.0;
  for (int i = 0; i < npx; ++i) {
    const float u = __fmaf_rn(a[i], al, bl), v = __fmaf_rn(b[i], ar, br);
    s12 = __dadd_rn(s12, (double)__fmul_rn(u, v));
    s11 = __dadd_rn(s11, (double)__fmul_rn(u, u));
    s22 = __dadd_rn(s22, (double)__fmul_rn(v, v));
  }
  out[k] = (float)__ddiv_rn(s12, __dsqrt_rn(__dmul_rn(s11, s22)));
}

// quantise: v = (uchar)(v / (256 / (int)(hi - lo))) + lo, stored as uchar
__global__ __launch_bounds__(kPatchBlock) void quantise_kernel(uint8_t* __restrict__ img, int stride, int w, int h,
                                                               int lo, int div) {
  const long q = (long)blockIdx.x * kPatchBlock + threadIdx.x;  // 4 pixels per thread
  const int per_row = (w + 3) / 4;
  const long y = q / per_row;
  if (y >= h) return;
  const int x0 = 4 * (int)(q - y * per_row);
  uint8_t* row = img + y * (long)stride;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int x = x0 + k;
    if (x < w) row[x] = (uint8_t)((int)(uint8_t)((int)row[x] / div) + lo);
  }
}

int pairs_entry(me_ctx* c, me_mem mem, const float* A, const float* B, int n, int rows, int cols, float* out,
                bool pc) {
  if (!c) return ME_ERR_INVALID;
  ME_CHECK(c, n >= 0 && rows > 0 && cols > 0, "%s: empty patch (the reference reads PC1.rows x PC1.cols)",
           pc ? "me_compare_pc" : "me_ccoeff_normed");
  ME_CHECK(c, mem == ME_HOST || mem == ME_DEVICE, "bad memory kind");
  if (n == 0) return ME_OK;
  ME_HIP(c, hipSetDevice(c->device));
  const int npx = rows * cols;
  const float *dA = A, *dB = B;
  float* dout = out;
  const size_t pb = 4 * (size_t)npx * n;
  if (mem == ME_HOST) {
    void* d;
    ME_TRY(me_scratch(c, SLOT_GENERIC, 2 * pb + 4 * (size_t)n + 256, &d));
    float* f = (float*)d;
    ME_HIP(c, hipMemcpyAsync(f, A, pb, hipMemcpyHostToDevice, c->stream));
    ME_HIP(c, hipMemcpyAsync(f + (size_t)npx * n, B, pb, hipMemcpyHostToDevice, c->stream));
    dA = f;
    dB = f + (size_t)npx * n;
    dout = f + 2 * (size_t)npx * n;
  }
  const int blocks = (n + kPatchBlock - 1) / kPatchBlock;
  if (pc)
    hipLaunchKernelGGL(compare_pc_kernel, dim3(blocks), dim3(kPatchBlock), 0, c->stream, dA, dB, n, npx, dout);
  else
    hipLaunchKernelGGL(ccoeff_kernel, dim3(blocks), dim3(kPatchBlock), 0, c->stream, dA, dB, n, npx, dout);
  ME_TRY(me_check_launch(c, pc ? "compare_pc_kernel" : "ccoeff_kernel"));
  if (mem == ME_HOST) {
    ME_HIP(c, hipMemcpyAsync(out, dout, 4 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    ME_HIP(c, hipStreamSynchronize(c->stream));
  }
  return ME_OK;
}

}  // namespace

extern "C" int me_compare_pc(me_ctx* c, me_mem mem, const float* A, const float* B, int n, int rows, int cols,
                             float* out) {
  return pairs_entry(c, mem, A, B, n, rows, cols, out, true);
}

extern "C" int me_ccoeff_normed(me_ctx* c, me_mem mem, const float* A, const float* B, int n, int rows, int cols,
                                float* out) {
  return pairs_entry(c, mem, A, B, n, rows, cols, out, false);
}

extern "C" int me_quantise(me_ctx* c, me_mem mem, uint8_t* img, int stride, int w, int h, int lo, int hi) {
  if (!c) return ME_ERR_INVALID;
  ME_CHECK(c, w > 0 && h > 0 && stride >= w, "me_quantise: empty image");
  ME_CHECK(c, lo >= 0 && lo <= 255 && hi >= 0 && hi <= 255, "me_quantise: range is a pair of uchar");
  const int d = hi - lo;  // (int)(range.second - range.first)
  ME_CHECK(c, d != 0, "me_quantise: empty range (the reference divides by zero)");
  ME_CHECK(c, mem == ME_HOST || mem == ME_DEVICE, "bad memory kind");
  ME_HIP(c, hipSetDevice(c->device));
  const int div = 256 / d;
  uint8_t* dimg = img;
  const size_t bytes = (size_t)stride * (h - 1) + w;
  if (mem == ME_HOST) {
    void* t;
    ME_TRY(me_scratch(c, SLOT_GENERIC, bytes, &t));
    ME_HIP(c, hipMemcpyAsync(t, img, bytes, hipMemcpyHostToDevice, c->stream));
    dimg = (uint8_t*)t;
  }
  const long threads = (long)h * ((w + 3) / 4);
  hipLaunchKernelGGL(quantise_kernel, dim3((unsigned)((threads + kPatchBlock - 1) / kPatchBlock)), dim3(kPatchBlock), 0,
                     c->stream, dimg, stride, w, h, lo, div);
  ME_TRY(me_check_launch(c, "quantise_kernel"));
  if (mem == ME_HOST) {
    ME_HIP(c, hipMemcpyAsync(img, dimg, bytes, hipMemcpyDeviceToHost, c->stream));
    ME_HIP(c, hipStreamSynchronize(c->stream));
  }
  return ME_OK;
}
