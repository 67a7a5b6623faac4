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

// below this many pairs the 8-lane batch kernel leaves most CUs idle: 16 lanes per pair
constexpr int kGroupThreshold = 32768;

// Term table: every value the reference's MI term can take for patches of N
// pixels, T(cJ, cL, cR) = pJ * log2f(pJ / (pL * pR)) with p = fl32(c * fl32(1/N)),
// computed once per N by the same device function (so bit-identical), stored
// for cL >= cR (pL * pR commutes exactly) and 1 <= cJ <= cR:
//   index(a, b, cJ) = (a-1) a (a+1) / 6 + b (b-1) / 2 + cJ - 1,  a = max, b = min.
// N = 121: 302 621 floats (1.2 MB, L2-resident per XCD).  It replaces ~35
// instructions (a correctly rounded division and the table-driven double
// polynomial of log2f) per term with one gather.
__host__ __device__ inline long mi_tab_index(int a, int b, int cJ) {
  return (long)(a - 1) * a * (a + 1) / 6 + (long)b * (b - 1) / 2 + cJ - 1;
}
__host__ __device__ inline long mi_tab_size(int N) { return mi_tab_index(N + 1, 1, 1); }

__global__ void mi_table_kernel(int N, float invN, float* __restrict__ tab) {
  const int a = blockIdx.x + 1;  // cL (the larger marginal)
  for (int b = threadIdx.x + 1; b <= a; b += blockDim.x)
    for (int cJ = 1; cJ <= b; ++cJ) tab[mi_tab_index(a, b, cJ)] = mi_term(cJ, a, b, invN);
}

__device__ __forceinline__ int byte_of(uint32_t w, int k) { return (w >> (8 * k)) & 0xff; }

// Batched MI, 8 lanes per patch pair (32 pairs per 256-thread workgroup, ~34 KB
// LDS: 4 workgroups / 16 waves per CU):
//  * histogram: a lane takes whole patch rows (dword loads realigned with
//    v_alignbyte), joint / marginal u8 counts and the occupancy bitmap by LDS
//    atomics in the group's shared histogram;
//  * terms: lane l walks bitmap words l and l + 8, each set bit is one
//    non-empty joint bin in row-major order, its term comes from the table
//    and lands at its rank (prefix of the bitmap popcounts) in a term list;
//  * sum: lane 0 of the group adds the list in order -- the reference's
//    left-to-right float sum over non-empty bins, bit for bit.
constexpr int kMiG = 8;
constexpr int kMiBlock = 256;
constexpr int kMiPairsPerBlock = kMiBlock / kMiG;
constexpr int kMiHistWords = 123;  // joint 100 | left 5 | right 5 | bitmap 13

template <int LIST>
__global__ __launch_bounds__(kMiBlock) void mi_batch_kernel(const uint8_t* __restrict__ imgL, int strideL,
                                                            const uint8_t* __restrict__ imgR, int strideR,
                                                            long bytesL, long bytesR,
                                                            const int32_t* __restrict__ xyL,
                                                            const int32_t* __restrict__ xyR, int n, int pw, int ph,
                                                            const float* __restrict__ tab, float* __restrict__ out) {
  constexpr int W = kMiHistWords + LIST;
  __shared__ uint32_t lds[kMiPairsPerBlock * W];
  const int gl = threadIdx.x & (kMiG - 1), grp = threadIdx.x / kMiG;
  uint32_t* h = lds + grp * W;
  float* list = reinterpret_cast<float*>(h + kMiHistWords);
  for (int k = blockIdx.x * kMiPairsPerBlock + grp; k < n; k += gridDim.x * kMiPairsPerBlock) {
    for (int i = gl; i < kMiHistWords; i += kMiG) h[i] = 0u;
    wave_sync();
    const int2 cl = reinterpret_cast<const int2*>(xyL)[k];
    const int2 cr = reinterpret_cast<const int2*>(xyR)[k];
    if (pw <= 12 && ph <= 2 * kMiG) {
      // rows gl and gl + 8: both rows' loads are issued before any histogram update
      uint32_t pl[2][3], pr[2][3];
      bool fast[2], live[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int r = gl + u * kMiG;
        live[u] = r < ph;
        const long offL = (long)(cl.y + r) * strideL + cl.x, offR = (long)(cr.y + r) * strideR + cr.x;
        // dword-aligned 16-byte windows by absolute address (inputs may be offset views)
        const int sl = (int)(((uintptr_t)imgL + offL) & 3), sr = (int)(((uintptr_t)imgR + offR) & 3);
        const long aL = offL - sl, aR = offR - sr;
        fast[u] = live[u] && aL + 16 <= bytesL && aR + 16 <= bytesR && aL >= 0 && aR >= 0;
        uint4 dl = {0, 0, 0, 0}, dr = {0, 0, 0, 0};
        if (fast[u]) {
          dl = *reinterpret_cast<const uint4*>(imgL + aL);
          dr = *reinterpret_cast<const uint4*>(imgR + aR);
        } else if (live[u]) {  // first / last bytes of an image: byte loads, never outside it
          uint32_t tl[4] = {0, 0, 0, 0}, tr[4] = {0, 0, 0, 0};
          for (int x = 0; x < pw; ++x) {
            const int q = sl + x, qr = sr + x;
            tl[q >> 2] |= (uint32_t)imgL[offL + x] << (8 * (q & 3));
            tr[qr >> 2] |= (uint32_t)imgR[offR + x] << (8 * (qr & 3));
          }
          dl = {tl[0], tl[1], tl[2], tl[3]};
          dr = {tr[0], tr[1], tr[2], tr[3]};
        }
        pl[u][0] = __builtin_amdgcn_alignbyte(dl.y, dl.x, sl);
        pl[u][1] = __builtin_amdgcn_alignbyte(dl.z, dl.y, sl);
        pl[u][2] = __builtin_amdgcn_alignbyte(dl.w, dl.z, sl);
        pr[u][0] = __builtin_amdgcn_alignbyte(dr.y, dr.x, sr);
        pr[u][1] = __builtin_amdgcn_alignbyte(dr.z, dr.y, sr);
        pr[u][2] = __builtin_amdgcn_alignbyte(dr.w, dr.z, sr);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (!live[u]) continue;
#pragma unroll
        for (int x = 0; x < 12; ++x) {
          if (x < pw) {
            const int bl = bin20(byte_of(pl[u][x >> 2], x & 3)), br = bin20(byte_of(pr[u][x >> 2], x & 3));
            const int code = bl * 20 + br;
            atomicAdd(&h[code >> 2], 1u << ((code & 3) * 8));
            atomicAdd(&h[100 + (bl >> 2)], 1u << ((bl & 3) * 8));
            atomicAdd(&h[105 + (br >> 2)], 1u << ((br & 3) * 8));
            atomicOr(&h[110 + (code >> 5)], 1u << (code & 31));
          }
        }
      }
    } else {
      for (int r = gl; r < ph; r += kMiG) {
        const long offL = (long)(cl.y + r) * strideL + cl.x, offR = (long)(cr.y + r) * strideR + cr.x;
        for (int x = 0; x < pw; ++x) {
          const int bl = bin20(imgL[offL + x]), br = bin20(imgR[offR + x]);
          const int code = bl * 20 + br;
          atomicAdd(&h[code >> 2], 1u << ((code & 3) * 8));
          atomicAdd(&h[100 + (bl >> 2)], 1u << ((bl & 3) * 8));
          atomicAdd(&h[105 + (br >> 2)], 1u << ((br & 3) * 8));
          atomicOr(&h[110 + (code >> 5)], 1u << (code & 31));
        }
      }
    }
    wave_sync();
    // ranks: exclusive prefix of the bitmap-word popcounts (words gl, gl + 8)
    const uint32_t b0 = h[110 + gl], b1 = gl + 8 < 13 ? h[118 + gl] : 0u;
    const int c0 = __builtin_popcount(b0), c1 = __builtin_popcount(b1);
    int s0 = c0, s1 = c1;
#pragma unroll
    for (int off = 1; off < kMiG; off <<= 1) {
      const int t0 = __shfl_up(s0, off, kMiG), t1 = __shfl_up(s1, off, kMiG);
      if (gl >= off) {
        s0 += t0;
        s1 += t1;
      }
    }
    const int tot0 = __shfl(s0, kMiG - 1, kMiG);
    const int total = tot0 + __shfl(s1, kMiG - 1, kMiG);
    // (1) table index of every non-empty bin at its rank (LDS only)
    int* slot = reinterpret_cast<int*>(list);
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      uint32_t bits = half ? b1 : b0;
      int idx = half ? tot0 + s1 - c1 : s0 - c0;
      const int wd = half ? gl + 8 : gl;
      while (bits) {
        const int b = __builtin_ctz(bits);
        bits &= bits - 1u;
        const int code = wd * 32 + b;
        const int i = code / 20, j = code - i * 20;
        const int cJ = byte_of(h[code >> 2], code & 3);
        const int cL = byte_of(h[100 + (i >> 2)], i & 3);
        const int cR = byte_of(h[105 + (j >> 2)], j & 3);
        slot[idx++] = (int)mi_tab_index(max(cL, cR), min(cL, cR), cJ);
      }
    }
    wave_sync();
    // (2) gather the terms, ranks strided over the group: 8 independent loads in flight per lane
    for (int r0 = gl; r0 < total; r0 += 8 * kMiG) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int r = r0 + u * kMiG;
        v[u] = r < total ? tab[slot[r]] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int r = r0 + u * kMiG;
        if (r < total) list[r] = v[u];
      }
    }
    wave_sync();
    if (gl == 0) {
      float MI = 0.0f;
      for (int t = 0; t < total; ++t) MI += list[t];
      out[k] = MI;
    }
    wave_sync();
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
int me_launch_mi_pairs(me_ctx* c, const uint8_t* dL, int sL, const uint8_t* dR, int sR, int width, int height,
                       const int32_t* dxyL, const int32_t* dxyR, int n, int pw, int ph, float* dout) {
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
  const int npx = pw * ph;
  const float* tab;
  ME_TRY(me_mi_table(c, npx, &tab));
  int blocks = (n + kMiPairsPerBlock - 1) / kMiPairsPerBlock;
  if (blocks > 4096) blocks = 4096;
  // bounds of the realigned 16-byte row loads: never read past the images
  const long img_bytes_L = (long)sL * (height - 1) + width, img_bytes_R = (long)sR * (height - 1) + width;
  if (npx <= 128)
    hipLaunchKernelGGL(mi_batch_kernel<128>, dim3(blocks), dim3(kMiBlock), 0, c->stream, dL, sL, dR, sR, img_bytes_L,
                       img_bytes_R, dxyL, dxyR, n, pw, ph, tab, dout);
  else
    hipLaunchKernelGGL(mi_batch_kernel<256>, dim3(blocks), dim3(kMiBlock), 0, c->stream, dL, sL, dR, sR, img_bytes_L,
                       img_bytes_R, dxyL, dxyR, n, pw, ph, tab, dout);
  return me_check_launch(c, "mi_batch_kernel");
}

int me_mi_table(me_ctx* c, int npx, const float** out) {
  if (npx < 1 || npx > 255) return me_set_error(c, ME_ERR_INVALID, "MI table: %d px outside [1, 255]", npx);
  if (!c->mi_table[npx]) {
    float* t;
    ME_HIP(c, hipMalloc(&t, 4 * (size_t)mi_tab_size(npx)));
    hipLaunchKernelGGL(mi_table_kernel, dim3(npx), dim3(128), 0, c->stream, npx, inv_count(npx), t);
    ME_TRY(me_check_launch(c, "mi_table_kernel"));
    c->mi_table[npx] = t;
  }
  *out = c->mi_table[npx];
  return ME_OK;
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
  if (mem == ME_DEVICE)
    return me_launch_mi_pairs(c, imgL, strideL, imgR, strideR, width, height, xyL, xyR, n, pw, ph, out);
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
  ME_TRY(me_launch_mi_pairs(c, (const uint8_t*)dL, strideL, (const uint8_t*)dR, strideR, width, height,
                            (const int32_t*)dxl,
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
