// mi.hip — batched mutual-information patch scores.
//
// Replaces me::computeMutualInformation (src/core/mutual_information.cpp:55-86)
// and me::computeEntropy (:28-45).  Design (MI355X):
//  * one lane per patch pair: the reference's row-major float accumulation is
//    inherently sequential, so the parallelism is across pairs, never inside
//    one sum (a tree sum would change the float result);
//  * lane-private histograms in LDS, word-interleaved across the workgroup
//    (bank = lane), built with ds_add/ds_or; empty bins are skipped through an
//    occupancy bitmap, so the term loop runs only over non-empty joint bins in
//    ascending code order (= the reference's i-outer / j-inner order);
//  * terms use the glibc log2f restatement (me_device.hpp): bit-exact floats.
#include "me_internal.hpp"
#include "me_device.hpp"

using namespace me_dev;

namespace {

constexpr int kMiBlock = 256;
// below this many pairs the batch cannot fill 256 CUs one pair per lane
constexpr int kGroupThreshold = 65536;

__global__ __launch_bounds__(kMiBlock) void mi_pairs_kernel(const uint8_t* __restrict__ imgL, int strideL,
                                                            const uint8_t* __restrict__ imgR, int strideR,
                                                            const int32_t* __restrict__ xyL,
                                                            const int32_t* __restrict__ xyR, int n, int pw, int ph,
                                                            float invN, float* __restrict__ out) {
  __shared__ uint32_t lds[kHistWords * kMiBlock];
  LaneHist<kMiBlock> h{&lds[threadIdx.x]};
  for (int k = blockIdx.x * kMiBlock + threadIdx.x; k < n; k += gridDim.x * kMiBlock) {
    const int2 cl = reinterpret_cast<const int2*>(xyL)[k];
    const int2 cr = reinterpret_cast<const int2*>(xyR)[k];
    const uint8_t* pl = imgL + (long)cl.y * strideL + cl.x;
    const uint8_t* pr = imgR + (long)cr.y * strideR + cr.x;
    h.clear();
    for (int y = 0; y < ph; ++y) {
      for (int x = 0; x < pw; ++x) h.add(pl[x], pr[x]);
      pl += strideL;
      pr += strideR;
    }
    out[k] = h.mi(invN);
  }
}

// Latency-bound batches: 16 lanes per pair (me_device.hpp GroupHist).
constexpr int kGroupBlock = 256;
__global__ __launch_bounds__(kGroupBlock) void mi_pairs_group_kernel(const uint8_t* __restrict__ imgL, int strideL,
                                                                     const uint8_t* __restrict__ imgR, int strideR,
                                                                     const int32_t* __restrict__ xyL,
                                                                     const int32_t* __restrict__ xyR, int n, int pw,
                                                                     int ph, float invN, float* __restrict__ out) {
  __shared__ uint32_t lds[(kGroupBlock / 16) * kGroupWords];
  const int grp = threadIdx.x >> 4;
  GroupHist<16> h{&lds[grp * kGroupWords], (int)(threadIdx.x & 15)};
  for (int k = blockIdx.x * (kGroupBlock / 16) + grp; k < n; k += gridDim.x * (kGroupBlock / 16)) {
    const int2 cl = reinterpret_cast<const int2*>(xyL)[k];
    const int2 cr = reinterpret_cast<const int2*>(xyR)[k];
    const float mi = group_mi<false>(h, imgL + (long)cl.y * strideL + cl.x, strideL,
                                     imgR + (long)cr.y * strideR + cr.x, strideR, pw, ph, invN);
    if (h.gl == 0) out[k] = mi;
  }
}

// Any patch size: one workgroup per pair, shared u32 histograms.
constexpr int kLargeBlock = 256;
__global__ __launch_bounds__(kLargeBlock) void mi_large_kernel(const uint8_t* __restrict__ L, int sL,
                                                               const uint8_t* __restrict__ R, int sR, int w, int h,
                                                               float invN, float* __restrict__ out) {
  __shared__ uint32_t hj[400], hl[20], hr[20];
  __shared__ float terms[400];
  for (int i = threadIdx.x; i < 400; i += kLargeBlock) hj[i] = 0;
  if (threadIdx.x < 20) { hl[threadIdx.x] = 0; hr[threadIdx.x] = 0; }
  __syncthreads();
  const long npx = (long)w * h;
  for (long p = threadIdx.x; p < npx; p += kLargeBlock) {
    int y = (int)(p / w), x = (int)(p - (long)y * w);
    int bl = bin20(L[(long)y * sL + x]), br = bin20(R[(long)y * sR + x]);
    atomicAdd(&hj[bl * 20 + br], 1u);
    atomicAdd(&hl[bl], 1u);
    atomicAdd(&hr[br], 1u);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 400; c += kLargeBlock) {
    int i = c / 20, j = c - i * 20;
    float pJ = (float)hj[c] * invN, pL = (float)hl[i] * invN, pR = (float)hr[j] * invN;
    terms[c] = (pJ > 0 && pL > 0 && pR > 0) ? pJ * log2f_glibc(pJ / (pL * pR)) : 0.0f;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float MI = 0.0f;
    for (int c = 0; c < 400; ++c)
      if (hj[c]) MI += terms[c];  // skipped bins never enter the sum (mutual_information.cpp:82)
    *out = MI;
  }
}

__global__ __launch_bounds__(kLargeBlock) void entropy_kernel(const uint8_t* __restrict__ I, int s, int w, int h,
                                                              float invN, float* __restrict__ out) {
  __shared__ uint32_t hist[20];
  if (threadIdx.x < 20) hist[threadIdx.x] = 0;
  __syncthreads();
  const long npx = (long)w * h;
  for (long p = threadIdx.x; p < npx; p += kLargeBlock) {
    int y = (int)(p / w), x = (int)(p - (long)y * w);
    atomicAdd(&hist[bin20(I[(long)y * s + x])], 1u);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float e = 0.0f;
    for (int i = 0; i < 20; ++i) {
      float p = (float)hist[i] * invN;
      if (p > 0) e += p * log2f_glibc(p);
    }
    *out = -e;
  }
}

inline float inv_count(long n) { return (float)(1.0 / (double)n); }

}  // namespace

// Shared launcher (also used by scale.hip for raw device buffers).
int me_launch_mi_pairs(me_ctx* c, const uint8_t* dL, int sL, const uint8_t* dR, int sR, const int32_t* dxyL,
                       const int32_t* dxyR, int n, int pw, int ph, float* dout) {
  if (n <= 0) return ME_OK;
  me_ktimer t(c, ME_KT_MI);
  if (n < kGroupThreshold) {
    // fewer pairs than lanes to fill the chip: 16 lanes per pair
    const int per = kGroupBlock / 16;
    int blocks = (n + per - 1) / per;
    hipLaunchKernelGGL(mi_pairs_group_kernel, dim3(blocks), dim3(kGroupBlock), 0, c->stream, dL, sL, dR, sR, dxyL,
                       dxyR, n, pw, ph, inv_count((long)pw * ph), dout);
    return me_check_launch(c, "mi_pairs_group_kernel");
  }
  int blocks = (n + kMiBlock - 1) / kMiBlock;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(mi_pairs_kernel, dim3(blocks), dim3(kMiBlock), 0, c->stream, dL, sL, dR, sR, dxyL, dxyR, n, pw,
                     ph, inv_count((long)pw * ph), dout);
  return me_check_launch(c, "mi_pairs_kernel");
}

extern "C" int me_mi_scores(me_ctx* c, me_mem mem, const uint8_t* imgL, int strideL, const uint8_t* imgR,
                            int strideR, int width, int height, const int32_t* xyL, const int32_t* xyR, int n,
                            int pw, int ph, float* out) {
  if (!c) return ME_ERR_INVALID;
  ME_CHECK(c, n >= 0 && pw > 0 && ph > 0 && width > 0 && height > 0, "me_mi_scores: bad sizes");
  ME_CHECK(c, pw * ph <= 255, "me_mi_scores: patch of %d px exceeds the 255-px lane-histogram limit; use "
                              "me_mutual_information", pw * ph);
  ME_CHECK(c, strideL >= width && strideR >= width, "me_mi_scores: stride < width");
  if (n == 0) return ME_OK;
  ME_HIP(c, hipSetDevice(c->device));
  if (mem == ME_DEVICE) return me_launch_mi_pairs(c, imgL, strideL, imgR, strideR, xyL, xyR, n, pw, ph, out);
  // host path: validate corners (the reference would throw cv::Exception on an out-of-image ROI)
  for (int k = 0; k < n; ++k) {
    int lx = xyL[2 * k], ly = xyL[2 * k + 1], rx = xyR[2 * k], ry = xyR[2 * k + 1];
    ME_CHECK(c, lx >= 0 && ly >= 0 && lx + pw <= width && ly + ph <= height && rx >= 0 && ry >= 0 &&
                    rx + pw <= width && ry + ph <= height,
             "me_mi_scores: pair %d ROI outside the image", k);
  }
  void *dL, *dR, *dxl, *dxr, *dout;
  size_t bl = (size_t)strideL * height, br = (size_t)strideR * height;
  ME_TRY(me_scratch(c, SLOT_IMG_L, bl, &dL));
  ME_TRY(me_scratch(c, SLOT_IMG_R, br, &dR));
  ME_TRY(me_scratch(c, SLOT_XY_L, 8 * (size_t)n, &dxl));
  ME_TRY(me_scratch(c, SLOT_XY_R, 8 * (size_t)n, &dxr));
  ME_TRY(me_scratch(c, SLOT_MI_OUT, 4 * (size_t)n, &dout));
  ME_HIP(c, hipMemcpyAsync(dL, imgL, bl, hipMemcpyHostToDevice, c->stream));
  ME_HIP(c, hipMemcpyAsync(dR, imgR, br, hipMemcpyHostToDevice, c->stream));
  ME_HIP(c, hipMemcpyAsync(dxl, xyL, 8 * (size_t)n, hipMemcpyHostToDevice, c->stream));
  ME_HIP(c, hipMemcpyAsync(dxr, xyR, 8 * (size_t)n, hipMemcpyHostToDevice, c->stream));
  ME_TRY(me_launch_mi_pairs(c, (const uint8_t*)dL, strideL, (const uint8_t*)dR, strideR, (const int32_t*)dxl,
                            (const int32_t*)dxr, n, pw, ph, (float*)dout));
  ME_HIP(c, hipMemcpyAsync(out, dout, 4 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
  ME_HIP(c, hipStreamSynchronize(c->stream));
  return ME_OK;
}

extern "C" int me_mutual_information(me_ctx* c, me_mem mem, const uint8_t* L, int sL, const uint8_t* R, int sR,
                                     int w, int h, float* out) {
  if (!c) return ME_ERR_INVALID;
  ME_CHECK(c, w > 0 && h > 0 && sL >= w && sR >= w, "me_mutual_information: empty or bad image (assert at "
                                                    "mutual_information.cpp:57)");
  ME_HIP(c, hipSetDevice(c->device));
  const float invN = inv_count((long)w * h);
  if (mem == ME_DEVICE) {
    me_ktimer t(c, ME_KT_MI);
    hipLaunchKernelGGL(mi_large_kernel, dim3(1), dim3(kLargeBlock), 0, c->stream, L, sL, R, sR, w, h, invN, out);
    return me_check_launch(c, "mi_large_kernel");
  }
  void *dL, *dR, *dout;
  size_t bl = (size_t)sL * (h - 1) + w, br = (size_t)sR * (h - 1) + w;
  ME_TRY(me_scratch(c, SLOT_IMG_L, bl, &dL));
  ME_TRY(me_scratch(c, SLOT_IMG_R, br, &dR));
  ME_TRY(me_scratch(c, SLOT_MI_OUT, 16, &dout));
  ME_HIP(c, hipMemcpyAsync(dL, L, bl, hipMemcpyHostToDevice, c->stream));
  ME_HIP(c, hipMemcpyAsync(dR, R, br, hipMemcpyHostToDevice, c->stream));
  {
    me_ktimer t(c, ME_KT_MI);
    hipLaunchKernelGGL(mi_large_kernel, dim3(1), dim3(kLargeBlock), 0, c->stream, (const uint8_t*)dL, sL,
                       (const uint8_t*)dR, sR, w, h, invN, (float*)dout);
  }
  ME_TRY(me_check_launch(c, "mi_large_kernel"));
  ME_HIP(c, hipMemcpyAsync(out, dout, 4, hipMemcpyDeviceToHost, c->stream));
  ME_HIP(c, hipStreamSynchronize(c->stream));
  return ME_OK;
}

extern "C" int me_entropy(me_ctx* c, me_mem mem, const uint8_t* I, int s, int w, int h, float* out) {
  if (!c) return ME_ERR_INVALID;
  ME_CHECK(c, w > 0 && h > 0 && s >= w, "me_entropy: empty image");
  ME_HIP(c, hipSetDevice(c->device));
  const float invN = inv_count((long)w * h);
  if (mem == ME_DEVICE) {
    hipLaunchKernelGGL(entropy_kernel, dim3(1), dim3(kLargeBlock), 0, c->stream, I, s, w, h, invN, out);
    return me_check_launch(c, "entropy_kernel");
  }
  void *dI, *dout;
  size_t b = (size_t)s * (h - 1) + w;
  ME_TRY(me_scratch(c, SLOT_IMG_L, b, &dI));
  ME_TRY(me_scratch(c, SLOT_MI_OUT, 16, &dout));
  ME_HIP(c, hipMemcpyAsync(dI, I, b, hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(entropy_kernel, dim3(1), dim3(kLargeBlock), 0, c->stream, (const uint8_t*)dI, s, w, h, invN,
                     (float*)dout);
  ME_TRY(me_check_launch(c, "entropy_kernel"));
  ME_HIP(c, hipMemcpyAsync(out, dout, 4, hipMemcpyDeviceToHost, c->stream));
  ME_HIP(c, hipStreamSynchronize(c->stream));
  return ME_OK;
}
