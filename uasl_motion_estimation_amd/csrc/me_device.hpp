// me_device.hpp — device-side building blocks shared by the kernels.
//
// Numerics contract (bit-exact parity with the reference's x86-64 build):
//  * this whole library is compiled with -ffp-contract=off, so every float /
//    double expression rounds exactly as written (no implicit FMA);
//  * fp32 division/sqrt are the correctly rounded HIP defaults;
//  * log2f is the glibc 2.35 algorithm (ARM optimized-routines log2f: a
//    16-entry {1/c, log2 c} table and a degree-4 polynomial evaluated in
//    double).  Verified equal to the host libm on all 2^31 positive floats
//    (tests/test_oracle.py::test_log2f_exhaustive runs the same check).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Cross-workgroup hand-offs inside one launch (ba.hip: last_arrival_wt, the
// fused assembly, the multi-workgroup camera solve; scale.hip:
// last_block_arrives, wt_store): the producer stores with agent-scope
// atomics (written through, sc1), every storing wave drains (s_waitcnt
// vmcnt(0)) before the workgroup barrier, one lane arrives with a RELAXED
// agent-scope atomic, and the consumer reads the data only through
// agent-scope atomic loads (a_ld<true> / the coherent loads).  This is
// correct because on gfx950 sc1 stores write through to memory and vmcnt
// counts stores -- under the HIP / C++ memory model alone the relaxed
// arrival would be a data race.  Every cross-workgroup read of same-launch
// data in a reducer must go through such a coherent load; a plain load may
// hit a stale line of another XCD's L2.  -DME_HANDOFF_ACQREL restores
// release / acquire ordering on these operations (A/B checks).
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "the written-through hand-offs rely on gfx950 cache behaviour (build with --offload-arch=gfx950)"
#endif
#ifdef ME_HANDOFF_ACQREL
#define ME_HO_LD __ATOMIC_ACQUIRE
#define ME_HO_ST __ATOMIC_RELEASE
#define ME_HO_RMW __ATOMIC_ACQ_REL
#else
#define ME_HO_LD __ATOMIC_RELAXED
#define ME_HO_ST __ATOMIC_RELAXED
#define ME_HO_RMW __ATOMIC_RELAXED
#endif

namespace me_dev {

__constant__ const double kLog2fInvc[16] = {
    0x1.661ec79f8f3bep+0, 0x1.571ed4aaf883dp+0, 0x1.49539f0f010b0p+0, 0x1.3c995b0b80385p+0,
    0x1.30d190c8864a5p+0, 0x1.25e227b0b8ea0p+0, 0x1.1bb4a4a1a343fp+0, 0x1.12358f08ae5bap+0,
    0x1.0953f419900a7p+0, 0x1.0000000000000p+0, 0x1.e608cfd9a47acp-1, 0x1.ca4b31f026aa0p-1,
    0x1.b2036576afce6p-1, 0x1.9c2d163a1aa2dp-1, 0x1.886e6037841edp-1, 0x1.767dcf5534862p-1};
__constant__ const double kLog2fLogc[16] = {
    -0x1.efec65b963019p-2, -0x1.b0b6832d4fca4p-2, -0x1.7418b0a1fb77bp-2, -0x1.39de91a6dcf7bp-2,
    -0x1.01d9bf3f2b631p-2, -0x1.97c1d1b3b7af0p-3, -0x1.2f9e393af3c9fp-3, -0x1.960cbbf788d5cp-4,
    -0x1.a6f9db6475fcep-5, 0x0.0p+0,              0x1.338ca9f24f53dp-4,  0x1.476a9543891bap-3,
    0x1.e840b4ac4e4d2p-3,  0x1.40645f0c6651cp-2,  0x1.88e9c2c1b9ff8p-2,  0x1.ce0a44eb17bccp-2};

// glibc log2f for the finite positive normal/subnormal inputs MI produces
// (q = pJ/(pL*pR) > 0).  FMA form = glibc's __log2f_fma ifunc variant; both
// variants agree with libm on every float (checked exhaustively).
__device__ __forceinline__ float log2f_glibc(float x) {
  uint32_t ix = __float_as_uint(x);
  if (ix == 0x3f800000u) return 0.0f;
  if (ix < 0x00800000u) {  // subnormal
    ix = __float_as_uint(x * 0x1p23f);
    ix -= 23u << 23;
  }
  uint32_t tmp = ix - 0x3f330000u;
  int i = (tmp >> 19) & 15;
  uint32_t top = tmp & 0xff800000u;
  uint32_t iz = ix - top;
  int k = (int32_t)tmp >> 23;
  double z = (double)__uint_as_float(iz);
  double r = __builtin_fma(z, kLog2fInvc[i], -1.0);
  double y0 = kLog2fLogc[i] + (double)k;
  double r2 = r * r;
  double y = __builtin_fma(0x1.ecabf496832e0p-2, r, -0x1.715479ffae3dep-1);
  y = __builtin_fma(-0x1.712b6f70a7e4dp-2, r2, y);
  double p = __builtin_fma(0x1.715475f35c8b8p+0, r, y0);
  y = __builtin_fma(y, r2, p);
  return (float)y;
}

// calcHist 8U, 20 uniform bins over [0,256): floor(v*20/256) = (5v)>>6
__device__ __forceinline__ int bin20(int v) { return (v * 5) >> 6; }

// (a-1) a (a+1) / 6 for 1 <= a <= 255: the product is < 2^24 (exact in float)
// and the quotient is an integer < 2^22, so the rounded float product is within
// 0.21 of it (checked exhaustively in tests/test_host.py).
// fl32(1/6) > 1/6 and the quotient k < 2^22 is representable, so the rounded
// product lies in [k, k + 0.21] and truncation gives k.
__device__ __forceinline__ int mi_c3(int a) {
  const float af = (float)a;
  const float p = __builtin_fmaf(af, af, -1.0f) * af;  // exact: < 2^24
  return (int)(uint32_t)(p * (1.0f / 6.0f));
}

// v_mul_u32_u24 (full rate); the compiler otherwise folds these into the
// quarter-rate v_mul_lo_u32.
__device__ __forceinline__ uint32_t mul_u24(uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// Index of T(cJ, cL, cR) in the per-N term table (mi.hip mi_table_kernel):
// c3(max) + min (min - 1) / 2 + cJ - 1.
__device__ __forceinline__ int mi_tab_idx(int cJ, int cL, int cR) {
  const int a = max(cL, cR), b = min(cL, cR);
  return mi_c3(a) + (int)(mul_u24((uint32_t)b, (uint32_t)(b - 1)) >> 1) + cJ - 1;
}

// One MI term of mutual_information.cpp:82-83.
__device__ __forceinline__ float mi_term(int cJ, int cL, int cR, float invN) {
  float pJ = (float)cJ * invN;
  float pL = (float)cL * invN;
  float pR = (float)cR * invN;
  float den = pL * pR;
  float q = pJ / den;
  return pJ * log2f_glibc(q);
}

// ---------------------------------------------------------------------
// Lane-private MI histogram in LDS.  Word w of lane t lives at
// lds[w * LANES + t] so a wave's accesses to one word hit 64 distinct banks.
//   words [0,100)   joint counts, 4 x u8 per word (code = bl*20 + br)
//   words [100,105) left marginal, [105,110) right marginal
//   words [110,123) occupancy bitmap of the 400 joint bins
// u8 counts limit a patch to 255 pixels (P <= 15).
constexpr int kHistWords = 123;

template <int LANES>
struct LaneHist {
  uint32_t* base;  // &lds[tid]
  __device__ __forceinline__ uint32_t& w(int i) { return base[i * LANES]; }
  __device__ __forceinline__ void clear() {
#pragma unroll 4
    for (int i = 0; i < kHistWords; ++i) w(i) = 0u;
  }
  __device__ __forceinline__ void add(int vl, int vr) {
    int bl = bin20(vl), br = bin20(vr);
    int code = bl * 20 + br;
    // lane-private words: LDS atomics only to get single ds_add/ds_or ops
    atomicAdd(&w(code >> 2), 1u << ((code & 3) * 8));
    atomicAdd(&w(100 + (bl >> 2)), 1u << ((bl & 3) * 8));
    atomicAdd(&w(105 + (br >> 2)), 1u << ((br & 3) * 8));
    atomicOr(&w(110 + (code >> 5)), 1u << (code & 31));
  }
  // Row-major (i = L bin outer, j = R bin inner) float sum over non-empty bins.
  __device__ __forceinline__ float mi(float invN) {
    float MI = 0.0f;
    for (int wd = 0; wd < 13; ++wd) {
      uint32_t bits = w(110 + wd);
      while (bits) {
        int b = __builtin_ctz(bits);
        bits &= bits - 1u;
        int code = wd * 32 + b;
        int i = code / 20, j = code - i * 20;
        int cJ = (w(code >> 2) >> ((code & 3) * 8)) & 0xff;
        int cL = (w(100 + (i >> 2)) >> ((i & 3) * 8)) & 0xff;
        int cR = (w(105 + (j >> 2)) >> ((j & 3) * 8)) & 0xff;
        MI += mi_term(cJ, cL, cR, invN);
      }
    }
    return MI;
  }
};

// ---------------------------------------------------------------------
// Group MI: G consecutive lanes of one wavefront cooperate on one patch pair
// (latency-bound batches: a few thousand pairs cannot fill 256 CUs at one
// pair per lane).  The histogram is shared by the group (LDS atomics), the
// expensive terms of the non-empty joint bins are computed in parallel (lane
// l of the group owns bitmap word l) and stored in row-major order, and the
// group's lane 0 adds them sequentially -- the reference's float summation
// order is preserved bit for bit.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr int kGroupTerms = 256;  // >= max non-empty joint bins (<= pixels <= 255)
constexpr int kGroupWords = kHistWords + kGroupTerms + 16;  // + the balanced walk's 16 start words

template <int G>
struct GroupHist {
  static_assert(G == 16, "group MI is written for 16-lane groups (13 bitmap words)");
  uint32_t* h;  // kGroupWords words of this group: histogram then float terms
  int gl;       // lane within the group
  __device__ __forceinline__ void clear() {
    for (int i = gl; i < 100; i += G) h[i] = 0u;  // the joint words (mi() rewrites the rest)
    wave_sync();
  }
  // one packed-byte joint update per pixel; the marginals and the occupancy
  // bitmap are derived from the joint words in mi() (round 6: the marginal and
  // bitmap atomics, 16 lanes hammering 10 + 13 words, were three quarters of
  // the LDS atomics)
  __device__ __forceinline__ void add(int vl, int vr) {
    int bl = bin20(vl), br = bin20(vr);
    int code = bl * 20 + br;
    atomicAdd(&h[code >> 2], 1u << ((code & 3) * 8));
  }
  // packed-byte sum over the group's 16 lanes (one DPP row; every byte sum
  // <= 121 pixels: no carry crosses a byte)
  __device__ __forceinline__ static uint32_t row_sum_u8x4(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false);   // quad [1,0,3,2]
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, false);   // quad [2,3,0,1]
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xf, 0xf, false);  // row half mirror
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xf, 0xf, false);  // row mirror
    return v;
  }
  // Left marginals (row sums), right marginals (column sums) and the bitmap of
  // non-empty bins from the joint words; returns this lane's bitmap word
  // (codes 32 gl .. 32 gl + 31).  Called by all 16 lanes after a wave_sync.
  __device__ __forceinline__ uint32_t derive() {
    uint32_t col[5] = {0u, 0u, 0u, 0u, 0u};
    uint8_t* lm = reinterpret_cast<uint8_t*>(h + 100);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int r = gl + 16 * k;
      if (r < 20) {
        uint32_t s = 0u;
#pragma unroll
        for (int m = 0; m < 5; ++m) {
          const uint32_t w = h[5 * r + m];
          s = __builtin_amdgcn_sad_u8(w, 0u, s);
          col[m] += w;
        }
        lm[r] = (uint8_t)s;
      }
    }
#pragma unroll
    for (int m = 0; m < 5; ++m) col[m] = row_sum_u8x4(col[m]);
    if (gl < 5) {
      uint32_t c = col[0];
#pragma unroll
      for (int m = 1; m < 5; ++m) c = gl == m ? col[m] : c;
      h[105 + gl] = c;
    }
    uint32_t bits = 0u;
    if (gl < 13) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int w8 = 8 * gl + k;
        if (w8 < 100) {
          const uint32_t f = (h[w8] + 0x7f7f7f7fu) & 0x80808080u;  // bit 7 of a byte: count > 0
          bits |= ((f * 0x00204081u) >> 28) << (4 * k);
        }
      }
    }
    return bits;
  }
  // Returns the MI in lane gl == 0 of the group (other lanes: unspecified).
  // tab: the per-N term table (bit-identical values, one gather per term) or null.
  __device__ __forceinline__ float mi(float invN, const float* __restrict__ tab = nullptr) {
    wave_sync();
    float* terms = reinterpret_cast<float*>(h + kHistWords);
    uint32_t bits = derive();
    wave_sync();  // the marginals visible to the group
    const int cnt = __builtin_popcount(bits);
    int pre = cnt;
#pragma unroll
    for (int off = 1; off < G; off <<= 1) {
      const int t = __shfl_up(pre, off, G);
      if (gl >= off) pre += t;
    }
    const int total = __shfl(pre, G - 1, G);
    const int excl = pre - cnt;
    // Balanced walk (round 6): lane q takes the slots [q T / 16, (q + 1) T / 16)
    // of the T non-empty bins in code order, crossing bitmap words, instead of
    // the bins of its own word (a patch's bins crowd a few rows: a few lanes
    // had all the terms).  Each word's owner leaves the lanes whose first slot
    // falls in its word their start (word, bins to skip).
    uint32_t* bmw = h + 110;                        // the bitmap words, for the walkers
    uint32_t* starts = h + kHistWords + kGroupTerms;  // one start word per lane
    if (gl < 13) {
      bmw[gl] = bits;
      if (cnt > 0) {
        const int qlo = (16 * excl + total - 1) / total, qhi = min(16, (16 * (excl + cnt) + total - 1) / total);
        for (int q = qlo; q < qhi; ++q) starts[q] = (uint32_t)gl | ((uint32_t)(((q * total) >> 4) - excl) << 8);
      }
    }
    wave_sync();  // bitmap words and starts visible to the group
    const int s0 = (gl * total) >> 4, nq = (((gl + 1) * total) >> 4) - s0;
    int w = 0;
    uint32_t cur = 0u;
    if (nq > 0) {
      const uint32_t st = starts[gl];
      w = (int)(st & 0xffu);
      cur = bmw[w];
      for (uint32_t sk = st >> 8; sk > 0; --sk) cur &= cur - 1u;
    }
    int idx = s0;
    // four bins per pass: the four terms' independent chains (division,
    // log2f table reads, polynomial) overlap instead of running back to back
    for (int t = 0; t < nq; t += 4) {
      int code[4];
      bool ok[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        ok[u] = t + u < nq;
        while (ok[u] && cur == 0u && w < 12) cur = bmw[++w];  // next non-empty word
        code[u] = ok[u] ? w * 32 + __builtin_ctz(cur | 0x80000000u) : 0;
        if (ok[u]) cur &= cur - 1u;
      }
      float tv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = code[u] / 20, j = code[u] - i * 20;
        const int cJ = (h[code[u] >> 2] >> ((code[u] & 3) * 8)) & 0xff;
        const int cL = (h[100 + (i >> 2)] >> ((i & 3) * 8)) & 0xff;
        const int cR = (h[105 + (j >> 2)] >> ((j & 3) * 8)) & 0xff;
        if (tab)
          tv[u] = ok[u] ? tab[mi_tab_idx(cJ, cL, cR)] : 0.0f;
        else
          tv[u] = mi_term(cJ, cL > 0 ? cL : 1, cR > 0 ? cR : 1, invN);  // padded slots: any finite value
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (ok[u]) terms[idx++] = tv[u];
    }
    wave_sync();
    float MI = 0.0f;
    if (gl == 0) {  // in-order float sum; the reads of a batch issue together
      int t = 0;
      for (; t + 8 <= total; t += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = terms[t + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) MI += v[u];
      }
      for (; t < total; ++t) MI += terms[t];
    }
    return MI;
  }
};

// Patch pair MI by a 16-lane group.  Row form (patches up to 12 x 16 whose
// 16-byte row windows lie inside both images, endA / endB = one past each
// image's last byte): lane r loads row r of both patches as one aligned
// 16-byte window each and adds its pixels -- two vector loads per lane instead
// of two byte loads per pixel (round 6: the scattered byte gathers were the
// group MI's address-unit work).  Otherwise pixels strided over the group.
template <bool BIN>
__device__ __forceinline__ float group_mi(GroupHist<16>& h, const uint8_t* A, long astride, const uint8_t* B,
                                          long bstride, int pw, int ph, float invN,
                                          const float* __restrict__ tab = nullptr, const uint8_t* endA = nullptr,
                                          const uint8_t* endB = nullptr) {
  h.clear();
  if (endA && endB && pw <= 12 && ph <= 16) {
    const uint8_t* la = A + (long)(ph - 1) * astride;
    const uint8_t* lb = B + (long)(ph - 1) * bstride;
    if (la - ((uintptr_t)la & 3) + 16 <= endA && lb - ((uintptr_t)lb & 3) + 16 <= endB) {  // (group-uniform)
      if (h.gl < ph) {
        const uint8_t* ra = A + (long)h.gl * astride;
        const uint8_t* rb = B + (long)h.gl * bstride;
        const uint32_t sa = (uint32_t)(uintptr_t)ra & 3u, sb = (uint32_t)(uintptr_t)rb & 3u;
        const uint4 va = *reinterpret_cast<const uint4*>(ra - sa);
        const uint4 vb = *reinterpret_cast<const uint4*>(rb - sb);
        const uint32_t pa[3] = {__builtin_amdgcn_alignbyte(va.y, va.x, sa), __builtin_amdgcn_alignbyte(va.z, va.y, sa),
                                __builtin_amdgcn_alignbyte(va.w, va.z, sa)};
        const uint32_t pb[3] = {__builtin_amdgcn_alignbyte(vb.y, vb.x, sb), __builtin_amdgcn_alignbyte(vb.z, vb.y, sb),
                                __builtin_amdgcn_alignbyte(vb.w, vb.z, sb)};
#pragma unroll
        for (int x = 0; x < 12; ++x) {
          if (x < pw) {
            int a = (int)((pa[x >> 2] >> (8 * (x & 3))) & 0xffu), b = (int)((pb[x >> 2] >> (8 * (x & 3))) & 0xffu);
            if (BIN) {
              a = a ? 255 : 0;
              b = b ? 255 : 0;
            }
            h.add(a, b);
          }
        }
      }
      return h.mi(invN, tab);
    }
  }
  const int npx = pw * ph;
  // Pixels in batches of 8 per lane: every load of a batch is issued before
  // the first histogram update (pixels past the patch alias pixel 0 and are
  // skipped), one memory round trip per batch instead of one per pixel.
  constexpr int kB = 8;
  for (int p0 = h.gl; p0 < npx; p0 += 16 * kB) {
    int va[kB], vb[kB];
#pragma unroll
    for (int u = 0; u < kB; ++u) {
      const int p = p0 + 16 * u < npx ? p0 + 16 * u : 0;
      const int y = p / pw, x = p - y * pw;
      va[u] = A[y * astride + x];
      vb[u] = B[y * bstride + x];
    }
#pragma unroll
    for (int u = 0; u < kB; ++u) {
      if (p0 + 16 * u < npx) {
        int a = va[u], b = vb[u];
        if (BIN) {
          a = a ? 255 : 0;
          b = b ? 255 : 0;
        }
        h.add(a, b);
      }
    }
  }
  return h.mi(invN, tab);
}

// ---------------------------------------------------------------------
// Pose / projection math for the ScaleState residuals, restating the
// OpenCV Matx evaluation order of optimisation.cpp:172-215 (s = 0; s += ...).
struct Pose44 { double T[16]; };

__device__ __forceinline__ void quat_pose(const double* q, const double* t, double* T) {
  const double w = q[0], x = q[1], y = q[2], z = q[3];
  T[0] = w * w + x * x - y * y - z * z; T[1] = 2 * (x * y - w * z); T[2] = 2 * (x * z + w * y); T[3] = t[0];
  T[4] = 2 * (x * y + w * z); T[5] = w * w - x * x + y * y - z * z; T[6] = 2 * (y * z - w * x); T[7] = t[1];
  T[8] = 2 * (x * z - w * y); T[9] = 2 * (y * z + w * x); T[10] = w * w - x * x - y * y + z * z; T[11] = t[2];
  T[12] = 0; T[13] = 0; T[14] = 0; T[15] = 1;
}

__device__ __forceinline__ void mat44_vec(const double* T, const double* X, double* Y) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    double s = 0;
    s += T[i * 4 + 0] * X[0];
    s += T[i * 4 + 1] * X[1];
    s += T[i * 4 + 2] * X[2];
    s += T[i * 4 + 3] * X[3];
    Y[i] = s;
  }
}

// ((K * I34) * s) * Y
__device__ __forceinline__ void project_scaled(const double* K, double s, const double* Y, double* f) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    double a = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      double kij = 0;
      kij += K[i * 3 + 0] * (k == 0 ? 1.0 : 0.0);
      kij += K[i * 3 + 1] * (k == 1 ? 1.0 : 0.0);
      kij += K[i * 3 + 2] * (k == 2 ? 1.0 : 0.0);
      a += (kij * s) * Y[k];
    }
    f[i] = a;
  }
}

// (K * I34) * Z
__device__ __forceinline__ void project(const double* K, const double* Z, double* f) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    double a = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      double kij = 0;
      kij += K[i * 3 + 0] * (k == 0 ? 1.0 : 0.0);
      kij += K[i * 3 + 1] * (k == 1 ? 1.0 : 0.0);
      kij += K[i * 3 + 2] * (k == 2 ? 1.0 : 0.0);
      a += kij * Z[k];
    }
    f[i] = a;
  }
}

// cv::Rect::contains(Point2f): cvRound (half-even) then half-open test
__device__ __forceinline__ bool rect_contains(int rx, int ry, int rw, int rh, float px, float py) {
  int ix = (int)rintf(px), iy = (int)rintf(py);
  return rx <= ix && ix < rx + rw && ry <= iy && iy < ry + rh;
}
// Rect(feat.x - w, ...): float - int in float, then truncation to int
__device__ __forceinline__ int roi_corner(float c, int w) { return (int)(c - (float)w); }

}  // namespace me_dev
