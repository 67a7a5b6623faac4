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
#include <cstring>

using namespace me_dev;

// quad kernel: walk iterations in flight per lane (table gathers overlapped;
// 2 / 4 / 6 / 8 measured 267.8 / 266.4 / 268.3 / 272.0 us per 1 M pairs)
constexpr int kQuadU = 4;
// lane kernel: histogram update order, pixel p = (k * kMiPerm) mod (PW PH)
constexpr int kMiPerm = 37;

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

// Batched MI, one lane per patch pair (measured on 11x11 patches of the
// synthetic stream: ~26 non-empty joint bins per pair, p90 41, so the 121
// pixel updates dominate and the term walk must stay cheap):
//  * lane-private histogram, word w of lane l at lds[64 w + l]: every LDS
//    access of the wave hits 64 distinct banks whatever the data, no atomics
//    collide and no barrier is ever needed (nothing crosses lanes);
//  * per pixel one packed-u8 ds_add (joint); the marginals and the occupancy
//    bitmap are derived afterwards from one read of the joint words (v_sad_u8
//    row sums, packed-byte column sums, carry-free non-zero-byte flags), and
//    the walk clears each joint word as it leaves it: per pair 121 LDS atomics
//    instead of 242, and no separate clearing pass;
//  * term walk: one flat loop over the lane's set bitmap bits in ascending
//    code order (= the reference's i-outer / j-inner order), int32 index
//    math, terms from the per-N table, summed left to right as they arrive
//    (bit-identical to the reference's float loop).
constexpr int kLaneBlock = 64;
constexpr int kLaneBm = 100, kLaneMarg = 114, kLaneWords = 124;  // joint | bitmap | 0 | marginals
constexpr int kLaneUnroll = 4;

__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = max(v, __shfl_xor(v, off, 64));
  return v;
}

// One patch row (PW <= 12 bytes) as three realigned dwords: FAST = the
// 16-byte window around the row lies inside the image (checked once per pair).
template <bool FAST>
__device__ __forceinline__ void load_row12(const uint8_t* __restrict__ img, long off, int pw, uint32_t d[3]) {
  const int sh = (int)(((uintptr_t)img + off) & 3);
  uint4 v = {0, 0, 0, 0};
  if (FAST) {
    v = *reinterpret_cast<const uint4*>(img + off - sh);
  } else {  // first / last bytes of an image: byte loads, never outside it
    uint32_t t[4] = {0, 0, 0, 0};
    for (int x = 0; x < pw; ++x) {
      const int q = sh + x;
      t[q >> 2] |= (uint32_t)img[off + x] << (8 * (q & 3));
    }
    v = {t[0], t[1], t[2], t[3]};
  }
  d[0] = __builtin_amdgcn_alignbyte(v.y, v.x, sh);
  d[1] = __builtin_amdgcn_alignbyte(v.z, v.y, sh);
  d[2] = __builtin_amdgcn_alignbyte(v.w, v.z, sh);
}

template <int PW>
__device__ __forceinline__ void lane_hist_row(uint32_t* h, const uint32_t pl[3], const uint32_t pr[3], int pw) {
#pragma unroll
  for (int x = 0; x < 12; ++x) {
    if (PW > 0 ? x < PW : x < pw) {
      const int bl = bin20((pl[x >> 2] >> (8 * (x & 3))) & 0xff), br = bin20((pr[x >> 2] >> (8 * (x & 3))) & 0xff);
      const int code = bl * 20 + br;
      atomicAdd(&h[64 * (code >> 2)], 1u << ((code & 3) * 8));
    }
  }
}

template <int PW, int PH, bool FAST>
__device__ __forceinline__ void lane_hist_pair(uint32_t* h, const uint8_t* __restrict__ imgL, int strideL, long oL,
                                               const uint8_t* __restrict__ imgR, int strideR, long oR, int pw,
                                               int ph) {
  if (PH > 0) {  // every row's loads issued before the first histogram update
    uint32_t pl[PH > 0 ? PH : 1][3], pr[PH > 0 ? PH : 1][3];
#pragma unroll
    for (int r = 0; r < PH; ++r) {
      load_row12<FAST>(imgL, oL + (long)r * strideL, PW, pl[r]);
      load_row12<FAST>(imgR, oR + (long)r * strideR, PW, pr[r]);
    }
    // updates in a scattered static order: neighbouring pixels often share a
    // joint bin, and back-to-back atomics on one LDS word serialise
#pragma unroll
    for (int k = 0; k < PW * PH; ++k) {
      const int p = (k * kMiPerm) % (PW * PH), r = p / PW, x = p % PW;
      const int bl = bin20((pl[r][x >> 2] >> (8 * (x & 3))) & 0xff), br = bin20((pr[r][x >> 2] >> (8 * (x & 3))) & 0xff);
      const int code = bl * 20 + br;
      atomicAdd(&h[64 * (code >> 2)], 1u << ((code & 3) * 8));
    }
  } else {
    for (int r = 0; r < ph; ++r) {
      uint32_t pl[3], pr[3];
      load_row12<FAST>(imgL, oL + (long)r * strideL, pw, pl);
      load_row12<FAST>(imgR, oR + (long)r * strideR, pw, pr);
      lane_hist_row<PW>(h, pl, pr, pw);
    }
  }
}

// Candidate pairs of the epipolar matcher (EPI instances): pair k is
// candidate c = k mod nd of feature f = k / nd, left patch at (floor(u - h),
// floor(v - h)), right patch d = lo_f + c pixels to its left; scored iff the
// right patch starts at x >= 0, d <= d_max and the feature passes the gates
// (valid_f; status_f == 1 inside the margin); score -inf otherwise.
struct EpiMap {
  const float* uv;
  const int32_t* lo;
  const uint8_t* valid;
  const uint8_t* status;
  const int32_t* n_dev;  // feature count on the device (or null)
  int nd, d_max, width, height, half;
  float margin;
  double* sc;  // n x nd scores
};

// PW, PH > 0: patch size known at compile time (11x11 residual, 10x10 finite-difference ROIs).
template <int PW, int PH, bool EPI = false>
__global__ __launch_bounds__(kLaneBlock) void mi_lane_kernel(const uint8_t* __restrict__ imgL, int strideL,
                                                             const uint8_t* __restrict__ imgR, int strideR,
                                                             long bytesL, long bytesR,
                                                             const int32_t* __restrict__ xyL,
                                                             const int32_t* __restrict__ xyR, int n, int pw, int ph,
                                                             const float* __restrict__ tab, int tab_bytes,
                                                             float* __restrict__ out, EpiMap em = EpiMap{}) {
  __shared__ uint32_t lds[kLaneWords * kLaneBlock];
  const int lane = threadIdx.x;
  uint32_t* h = lds + lane;
  for (int w = 0; w < kLaneWords; ++w) h[64 * w] = 0u;
  // table entry of (a, b, cJ) is c3(a) + b(b-1)/2 + cJ - 1; buffer loads past tab_bytes return 0
  const __amdgpu_buffer_rsrc_t rtab = __builtin_amdgcn_make_buffer_rsrc((void*)tab, (short)0, tab_bytes, 0x00020000);
  const int ntot = EPI ? (em.n_dev ? min(n, *em.n_dev) : n) * em.nd : n;
  for (int k0 = blockIdx.x * kLaneBlock; k0 < ntot; k0 += gridDim.x * kLaneBlock) {
    const int k = k0 + lane;
    bool live = k < ntot;
    long oL = 0, oR = 0;
    if (EPI && live) {
      const int f = k / em.nd, c = k - f * em.nd;
      const float u = em.uv[2 * f], v = em.uv[2 * f + 1];
      // Rect(x - w, y - w, ..) corner (floor of the FP64 value, as the restatement)
      const int x0 = (int)floor((double)u - em.half), y0 = (int)floor((double)v - em.half);
      bool fv = em.valid ? em.valid[f] != 0 : true;
      if (em.status)  // the KLT gate: status 1 and inside the feature margin
        fv = fv && em.status[f] == 1 && u >= em.margin && u < (float)em.width - em.margin && v >= em.margin &&
             v < (float)em.height - em.margin;
      const int d = em.lo[f] + c, xr = x0 - d;
      // (inside the image: the left patch, and the right one (x >= 0) -- ADVICE r3)
      live = fv && xr >= 0 && d <= em.d_max && x0 >= 0 && y0 >= 0 && x0 + 2 * em.half + 1 <= em.width &&
             y0 + 2 * em.half + 1 <= em.height;
      oL = (long)y0 * strideL + x0;
      oR = (long)y0 * strideR + xr;
    } else if (!EPI && live) {
      const int2 cl = reinterpret_cast<const int2*>(xyL)[k];
      const int2 cr = reinterpret_cast<const int2*>(xyR)[k];
      oL = (long)cl.y * strideL + cl.x;
      oR = (long)cr.y * strideR + cr.x;
    }
    if (live) {
      const int rows = PH > 0 ? PH : ph;
      // 16-byte windows start at most 3 bytes before a row and end at most 16 after its start
      const bool fast = oL >= 3 && oR >= 3 && oL + (long)(rows - 1) * strideL + 16 <= bytesL &&
                        oR + (long)(rows - 1) * strideR + 16 <= bytesR;
      if (fast)
        lane_hist_pair<PW, PH, true>(h, imgL, strideL, oL, imgR, strideR, oR, pw, ph);
      else
        lane_hist_pair<PW, PH, false>(h, imgL, strideL, oL, imgR, strideR, oR, pw, ph);
    }
    // marginals from the joint rows (row i is words 5i..5i+4, bins j = 0..19)
    // and the occupancy bitmap of the joint bins from the same reads: bit c
    // of the 416-bit map <=> joint count of code c non-zero.  Counts are
    // <= 121, so (w + 0x7f7f7f7f) & 0x80808080 flags the non-zero bytes
    // without carries, and one multiply gathers the four flags (bytes 0..3
    // -> bits 28..31, no overlapping partial products) into a nibble placed at
    // the word's static bitmap position.
    uint32_t cl4[5] = {0, 0, 0, 0, 0}, cr4[5] = {0, 0, 0, 0, 0};
    uint32_t bm[13] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 20; ++i) {
      uint32_t s = 0;
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        const int jw = 5 * i + q;
        const uint32_t w = h[64 * jw];
        s = __builtin_amdgcn_sad_u8(w, 0u, s);
        cr4[q] += w;  // byte sums <= 255: no carries between the packed counts
        const uint32_t f = (w + 0x7f7f7f7fu) & 0x80808080u;
        bm[jw >> 3] |= ((f * 0x00204081u) >> 28) << (4 * (jw & 7));
      }
      cl4[i >> 2] |= s << (8 * (i & 3));
    }
    uint32_t nz = 0;  // non-empty bitmap words
    int nnz = 0;
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      h[64 * (kLaneMarg + q)] = cl4[q];
      h[64 * (kLaneMarg + 5 + q)] = cr4[q];
    }
#pragma unroll
    for (int w = 0; w < 13; ++w) {
      h[64 * (kLaneBm + w)] = bm[w];
      nz |= (bm[w] != 0u ? 1u : 0u) << w;
      nnz += __builtin_popcount(bm[w]);
    }
    const int tmax = wave_max(nnz);
    // Branch-free walk.  State: current word wd and its remaining bits, the
    // words still to visit (nz), and the next non-empty word nw with its bits
    // read one step ahead (nxt); word 13 is a permanent zero sentinel.  A
    // finished lane keeps producing in-range garbage codes whose table reads
    // are masked off, so the whole wave runs one uniform loop.  The marginal
    // counts stay in registers (byte select); the table gathers of one
    // iteration are summed in the next one, so their L2 latency overlaps a
    // whole iteration of the walk (same left-to-right order of the float sum).
    int wd = __builtin_ctz(nz | 0x2000u);
    nz &= nz - 1u;
    uint32_t bits = h[64 * (kLaneBm + wd)];
    int nw = __builtin_ctz(nz | 0x2000u);
    uint32_t nxt = h[64 * (kLaneBm + nw)];
    float MI = 0.0f;
    float vp[kLaneUnroll];
#pragma unroll
    for (int u = 0; u < kLaneUnroll; ++u) vp[u] = 0.0f;
    for (int t = 0; t < tmax; t += kLaneUnroll) {
      float v[kLaneUnroll];
#pragma unroll
      for (int u = 0; u < kLaneUnroll; ++u) {
        const int code = (wd << 5) | __builtin_ctz(bits | 0x80000000u);  // < 448
        bits &= bits - 1u;
        const bool z = bits == 0u;
        wd = z ? nw : wd;
        bits = z ? nxt : bits;
        nz = z ? nz & (nz - 1u) : nz;
        nw = __builtin_ctz(nz | 0x2000u);
        nxt = h[64 * (kLaneBm + nw)];  // unchanged unless z: same word as before
        const int i = (int)(mul_u24((uint32_t)code, 205u) >> 12);  // exact code / 20 for code < 1024
        const int j = code - (int)mul_u24((uint32_t)i, 20u);
        const int cw = code >> 2;
        const uint32_t hw = h[64 * cw];
        const int cJ = (hw >> ((code & 3) * 8)) & 0xff;
        // the joint histogram is cleared as the walk leaves each non-empty
        // word (every such word is visited; ascending codes never return);
        // otherwise the word is stored back unchanged (no branch)
        const int ncode = (wd << 5) | __builtin_ctz(bits | 0x80000000u);
        const bool clr = t + u < nnz && ((ncode >> 2) != cw || t + u + 1 >= nnz);
        h[64 * cw] = clr ? 0u : hw;
        const int qi = i >> 2, qj = j >> 2;  // i <= 22 for a finished lane's garbage code
        const uint32_t wl = h[64 * (kLaneMarg + qi)];
        const uint32_t wr = h[64 * (kLaneMarg + 5 + qj)];
        const int cL = (wl >> ((i & 3) * 8)) & 0xff;
        const int cR = (wr >> ((j & 3) * 8)) & 0xff;
        const int a = max(cL, cR), b = min(cL, cR);
        const int idx = mi_c3(a) + (int)(mul_u24((uint32_t)b, (uint32_t)(b - 1)) >> 1) + cJ;
        // out-of-range buffer offsets read 0: a finished lane adds +0.0f, no branch
        const int off = t + u < nnz ? 4 * (idx - 1) : 0x7ffffff0;
        v[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rtab, off, 0, 0));
      }
#pragma unroll
      for (int u = 0; u < kLaneUnroll; ++u) MI += vp[u];  // previous iteration: +0.0f when finished (MI is never -0)
#pragma unroll
      for (int u = 0; u < kLaneUnroll; ++u) vp[u] = v[u];
    }
#pragma unroll
    for (int u = 0; u < kLaneUnroll; ++u) MI += vp[u];
    // the joint words were cleared by the walk; bitmap and marginals are rewritten per pair
    if (EPI) {
      if (k < ntot) em.sc[k] = live ? (double)MI : -INFINITY;
    } else if (k < n) {
      out[k] = MI;
    }
  }
}

// ---------------------------------------------------------------------
// Batched MI, four lanes per patch pair (the default batch kernel).  The
// lane kernel above is LDS-bound at ~1.25 waves per SIMD (124 lane-private
// words).  Here the four lanes q = 0..3 of a quad share one pair's 100 joint
// words, so a wave holds 16 pairs in 16 x (105 + N) words (N = patch pixels,
// the term slots) and ~11 waves fit a CU:
//  * histogram: lane q bins patch rows q, q + 4, ... into the shared joint
//    words (LDS atomics; same-word updates of a quad serialise, counts are
//    order-free);
//  * lane q derives joint rows i = q + 4k (k = 0..4) from one read of their
//    25 words: left marginals, occupancy (20 bits per row), bin counts; the
//    right marginal is the quad sum of the column partials (DPP);
//  * quad prefix sums over the per-row counts give every row its first slot
//    in the reference's i-outer / j-inner order and its index in a compacted
//    table of non-empty rows;
//  * the walk is balanced by bins, not rows: lane q takes the slots
//    [floor(qT/4), floor((q+1)T/4)) of the pair's T non-empty bins, starting
//    from the row the row's owner names, gathers their terms from the per-N
//    table and stores them in their slots;
//  * lane 0 of the quad adds the slots left to right (bit-identical to the
//    reference's float loop, mutual_information.cpp:78-84).
// Group g's word w lives at lds[16 w + g]: the 16 quads of a wave never
// share a bank; lanes of one quad do when their words agree mod 4.
// unpacked group words: [0,100) joint, [100,105) right marginal, [105,126) compacted row table (20 + 1 spare),
// [126,132) its left marginals (bytes), [132,136) lane starts, [136, 136 + N) term slots
// Packed layout (N <= 127 pixels): the right marginal as one word per column
// and the row table's left marginals as words, each m -> c3(m) << 13 | m (m - 1) / 2
// (c3(127) < 2^19, 127 * 126 / 2 < 2^13).  For m >= 1 the words order as m
// does, so the walk's table index is (max >> 13) + (min & 0x1fff) + cJ - 1 --
// five operations instead of the float c3 and the triangle product per term.
// Packed shapes keep the terms in registers and sum them in order by DPP quad
// broadcasts; the group words are [0,100) joint, [100,120) column words,
// [120,140) row table (no spare: the walk's look-ahead stops at entry 19),
// [140,160) its left-marginal words, [160,164) lane starts: 164 words per pair,
// 10.5 KB per workgroup.  Unpacked shapes (N > 127) add N term slots.
constexpr int kQuadBlock = 64, kQuadGroups = 16;

template <int PW, int PH>
struct QuadShape {
  static constexpr bool kPack = PW > 0 && PH > 0 && PW * PH <= 127;
  static constexpr int kN = (PW > 0 && PH > 0) ? PW * PH : 255;               // >= non-empty bins
  static constexpr int kSlots = kPack ? 0 : kN;  // packed: terms in registers
  static constexpr int kMaxT = kPack ? ((kN + 3) / 4 + kQuadU - 1) / kQuadU * kQuadU : 0;  // >= a lane's run
  // packed: 22 row-table entries (up to 20 rows + 2 sentinels), no bound on the walk's look-ahead
  static constexpr int kCR = 100, kRowTab = kPack ? 120 : 105, kRowCL = kPack ? 142 : 126,
                       kStart = kPack ? 164 : 132, kTerms = kStart + 4, kClear = kPack ? kStart : kRowCL,
                       kLastE = kPack ? 21 : 20;  // last row-table entry the walk reads
  static constexpr int kWords = kTerms + kSlots;
  static constexpr int kRows = PH > 0 ? (PH + 3) / 4 : 4;  // patch rows per lane (PH <= 15)
};

__device__ __forceinline__ uint32_t mi_pack(uint32_t m) {
  return ((uint32_t)mi_c3((int)m) << 13) | (mul_u24(m, m - 1u) >> 1);
}

// Quad reductions over lanes 4g..4g+3 by DPP quad permutes (no LDS round trip).
template <int CTRL>
__device__ __forceinline__ uint32_t quad_perm(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}
// lane QQ of each quad's value, to all four lanes
template <int QQ>
__device__ __forceinline__ float bcast_lane(float v) {
  // (old = +0.0f, the add's identity: the DPP folds into the consuming v_add_f32)
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), QQ * 0x55, 0xf, 0xf, false));
}
__device__ __forceinline__ uint32_t quad_sum(uint32_t v) {
  v += quad_perm<0xB1>(v);     // lanes [1,0,3,2]
  return v + quad_perm<0x4E>(v);  // lanes [2,3,0,1]
}
__device__ __forceinline__ uint32_t quad_exscan(uint32_t v, int q) {
  uint32_t s = v;
  const uint32_t a = quad_perm<0x90>(s);  // lanes [0,0,1,2]
  s += q >= 1 ? a : 0u;
  const uint32_t b = quad_perm<0x44>(s);  // lanes [0,1,0,1]
  s += q >= 2 ? b : 0u;
  return s - v;
}

template <int PW, int PH, bool FAST>
__device__ __forceinline__ void quad_hist(uint32_t* hg, const uint8_t* __restrict__ imgL, int strideL, long oL,
                                          const uint8_t* __restrict__ imgR, int strideR, long oR, int pw, int ph,
                                          int q) {
  using QS = QuadShape<PW, PH>;
  if (PH > 0) {
    uint32_t pl[QS::kRows][3], pr[QS::kRows][3];
#pragma unroll
    for (int rr = 0; rr < QS::kRows; ++rr) {
      const int r = q + 4 * rr;
      pl[rr][0] = pl[rr][1] = pl[rr][2] = pr[rr][0] = pr[rr][1] = pr[rr][2] = 0u;
      if (r < PH) {
        load_row12<FAST>(imgL, oL + (long)r * strideL, PW, pl[rr]);
        load_row12<FAST>(imgR, oR + (long)r * strideR, PW, pr[rr]);
      }
    }
#pragma unroll
    for (int rr = 0; rr < QS::kRows; ++rr) {
      if (q + 4 * rr < PH) {
#pragma unroll
        for (int k = 0; k < PW; ++k) {
          // scattered (a multiplier coprime to PW): neighbouring pixels often share a joint word
          const int x = PW > 0 ? (k * (PW % 5 == 0 ? 3 : 5)) % (PW > 0 ? PW : 1) : k;
          const int bl = bin20((pl[rr][x >> 2] >> (8 * (x & 3))) & 0xff);
          const int br = bin20((pr[rr][x >> 2] >> (8 * (x & 3))) & 0xff);
          const int code = bl * 20 + br;
          atomicAdd(&hg[16 * (code >> 2)], 1u << ((code & 3) * 8));
        }
      }
    }
  } else {
    for (int r = q; r < ph; r += 4) {
      uint32_t pl[3], pr[3];
      load_row12<FAST>(imgL, oL + (long)r * strideL, pw, pl);
      load_row12<FAST>(imgR, oR + (long)r * strideR, pw, pr);
#pragma unroll
      for (int x = 0; x < 12; ++x) {
        if (x < pw) {
          const int bl = bin20((pl[x >> 2] >> (8 * (x & 3))) & 0xff), br = bin20((pr[x >> 2] >> (8 * (x & 3))) & 0xff);
          const int code = bl * 20 + br;
          atomicAdd(&hg[16 * (code >> 2)], 1u << ((code & 3) * 8));
        }
      }
    }
  }
}

template <int PW, int PH, bool EPI = false>
__global__ __launch_bounds__(kQuadBlock) void mi_quad_kernel(const uint8_t* __restrict__ imgL, int strideL,
                                                             const uint8_t* __restrict__ imgR, int strideR,
                                                             long bytesL, long bytesR,
                                                             const int32_t* __restrict__ xyL,
                                                             const int32_t* __restrict__ xyR, int n, int pw, int ph,
                                                             const float* __restrict__ tab, int tab_bytes,
                                                             float* __restrict__ out, EpiMap em = EpiMap{}) {
  using QS = QuadShape<PW, PH>;
  __shared__ uint32_t lds[QS::kWords * kQuadGroups];
  const int lane = threadIdx.x, g = lane >> 2, q = lane & 3;
  uint32_t* hg = lds + g;  // word w of this quad's pair: hg[16 w]
  // joint words zero (the walk's clears keep them so); row table entries always name a row of this region
  for (int w = q; w < QS::kClear; w += 4) hg[16 * w] = 0u;
  const __amdgpu_buffer_rsrc_t rtab = __builtin_amdgcn_make_buffer_rsrc((void*)tab, (short)0, tab_bytes, 0x00020000);
  const int ntot = EPI ? (em.n_dev ? min(n, *em.n_dev) : n) * em.nd : n;
  for (int k0 = blockIdx.x * kQuadGroups; k0 < ntot; k0 += gridDim.x * kQuadGroups) {
    const int k = k0 + g;
    bool live = k < ntot;
    long oL = 0, oR = 0;
    if (EPI && live) {
      const int f = k / em.nd, c = k - f * em.nd;
      const float u = em.uv[2 * f], v = em.uv[2 * f + 1];
      const int x0 = (int)floor((double)u - em.half), y0 = (int)floor((double)v - em.half);
      bool fv = em.valid ? em.valid[f] != 0 : true;
      if (em.status)
        fv = fv && em.status[f] == 1 && u >= em.margin && u < (float)em.width - em.margin && v >= em.margin &&
             v < (float)em.height - em.margin;
      const int d = em.lo[f] + c, xr = x0 - d;
      // (inside the image: the left patch, and the right one (x >= 0) -- ADVICE r3)
      live = fv && xr >= 0 && d <= em.d_max && x0 >= 0 && y0 >= 0 && x0 + 2 * em.half + 1 <= em.width &&
             y0 + 2 * em.half + 1 <= em.height;
      oL = (long)y0 * strideL + x0;
      oR = (long)y0 * strideR + xr;
    } else if (!EPI && live) {
      const int2 cl = reinterpret_cast<const int2*>(xyL)[k];
      const int2 cr = reinterpret_cast<const int2*>(xyR)[k];
      oL = (long)cl.y * strideL + cl.x;
      oR = (long)cr.y * strideR + cr.x;
    }
    wave_sync();  // the previous pair's clears and slot reads precede this pair's updates
    if (live) {
      const int rows = PH > 0 ? PH : ph;
      const bool fast = oL >= 3 && oR >= 3 && oL + (long)(rows - 1) * strideL + 16 <= bytesL &&
                        oR + (long)(rows - 1) * strideR + 16 <= bytesR;
      if (fast)
        quad_hist<PW, PH, true>(hg, imgL, strideL, oL, imgR, strideR, oR, pw, ph, q);
      else
        quad_hist<PW, PH, false>(hg, imgL, strideL, oL, imgR, strideR, oR, pw, ph, q);
    }
    wave_sync();
    // Own rows i = q + 4 kk: left marginals (bytes of cl), column partials,
    // occupancy (20 bits per row), bin counts (bytes of c03 / c4).
    uint32_t cr4[5] = {0, 0, 0, 0, 0}, rb[5];
    uint64_t cl = 0;
    uint32_t c03 = 0, c4 = 0;
#pragma unroll
    for (int kk = 0; kk < 5; ++kk) {
      const uint32_t* row = hg + 16 * 5 * (q + 4 * kk);
      uint32_t s = 0, bits = 0;
#pragma unroll
      for (int m = 0; m < 5; ++m) {
        const uint32_t w = row[16 * m];
        s = __builtin_amdgcn_sad_u8(w, 0u, s);
        cr4[m] += w;
        const uint32_t f = (w + 0x7f7f7f7fu) & 0x80808080u;
        bits |= ((f * 0x00204081u) >> 28) << (4 * m);
      }
      rb[kk] = bits;
      cl |= (uint64_t)s << (8 * kk);
      const uint32_t cnt = __builtin_popcount(bits);
      if (kk < 4) c03 |= cnt << (8 * kk);
      else c4 = cnt;
    }
#pragma unroll
    for (int m = 0; m < 5; ++m) cr4[m] = quad_sum(cr4[m]);
    if (QS::kPack) {  // lane q: columns 4m + q
#pragma unroll
      for (int m = 0; m < 5; ++m) hg[16 * (QS::kCR + 4 * m + q)] = mi_pack((cr4[m] >> (8 * q)) & 0xffu);
    } else if (q == 0) {
#pragma unroll
      for (int m = 0; m < 5; ++m) hg[16 * (QS::kCR + m)] = cr4[m];
    }
    // Global order = rows ascending, bins ascending within a row.  Per own row:
    // P = bins in earlier rows (its first slot), E = non-empty rows before it
    // (its index in the compacted row table).  Row i = q + 4 kk comes after
    // all rows of earlier kk and the rows of lanes < q at this kk: quad
    // reductions / exclusive scans of the packed per-kk bytes (no byte ever
    // carries: every partial sum is <= N <= 255).
    const uint32_t a03 = quad_sum(c03), a4 = quad_sum(c4);
    const uint32_t p03 = a03 * 0x01010100u + quad_exscan(c03, q);
    const uint32_t p4 = __builtin_amdgcn_sad_u8(a03, 0u, 0u) + quad_exscan(c4, q);
    const int total = (int)(__builtin_amdgcn_sad_u8(a03, 0u, 0u) + a4);
    const uint32_t n03 = ((c03 + 0x7f7f7f7fu) & 0x80808080u) >> 7, n4 = c4 ? 1u : 0u;
    const uint32_t na03 = quad_sum(n03), na4 = quad_sum(n4);
    const uint32_t e03 = na03 * 0x01010100u + quad_exscan(n03, q);
    const uint32_t e4 = __builtin_amdgcn_sad_u8(na03, 0u, 0u) + quad_exscan(n4, q);
    // Lane q' takes the bins with slots [b_q', b_q'+1), b_q' = floor(q' T / 4): the
    // owner of the row holding slot b_q' leaves lane q' its start (table entry, bins to skip).
    uint32_t* rowtab = hg + 16 * QS::kRowTab;
    uint32_t* rowcw = hg + 16 * QS::kRowCL;  // (packed layout: left-marginal words)
    uint8_t* clc = reinterpret_cast<uint8_t*>(rowcw);
#pragma unroll
    for (int kk = 0; kk < 5; ++kk) {
      const int cnt = kk < 4 ? (int)((c03 >> (8 * kk)) & 0xff) : (int)c4;
      const int P = kk < 4 ? (int)((p03 >> (8 * kk)) & 0xff) : (int)p4;
      const int E = kk < 4 ? (int)((e03 >> (8 * kk)) & 0xff) : (int)e4;
      if (cnt > 0) {
        rowtab[16 * E] = rb[kk] | ((uint32_t)(5 * (q + 4 * kk)) << 20);  // (the row's first joint word)
        if (QS::kPack)
          rowcw[16 * E] = mi_pack((uint32_t)(cl >> (8 * kk)) & 0xffu);
        else
          clc[64 * (E >> 2) + (E & 3)] = (uint8_t)(cl >> (8 * kk));
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int bq = (qq * total) >> 2;
          if (P <= bq && bq < P + cnt) hg[16 * (QS::kStart + qq)] = (uint32_t)E | ((uint32_t)(bq - P) << 8);
        }
      }
    }
    if (QS::kPack && q == 0) {
      // two sentinel rows of 20 bins after the last: a lane's run of <= kMaxT
      // steps never exhausts both, so its look-ahead needs no bound (their
      // terms lie beyond the run: masked loads)
      const uint32_t nrows = __builtin_amdgcn_sad_u8(na03, 0u, 0u) + na4;
      rowtab[16 * nrows] = 0xfffffu;
      rowtab[16 * (nrows + 1)] = 0xfffffu;
    }
    wave_sync();  // right marginal, row table and starts visible to the quad
    const int s0 = (q * total) >> 2, nq = (((q + 1) * total) >> 2) - s0;
    const int tmax = __builtin_amdgcn_readfirstlane(wave_max(nq));  // (uniform: scalar branches)
    const uint8_t* crb = reinterpret_cast<const uint8_t*>(hg + 16 * QS::kCR);
    const uint32_t* colw = hg + 16 * QS::kCR;  // (packed layout)
    const uint8_t* jnt = reinterpret_cast<const uint8_t*>(hg);
    int e = 0;
    uint32_t bits = 0, ent = 0, cL = 0, nxt = 0, ncl = 0;
    if (nq > 0) {
      const uint32_t st = hg[16 * (QS::kStart + q)];
      e = (int)(st & 0xff);
      ent = rowtab[16 * e];
      cL = QS::kPack ? rowcw[16 * e] : clc[64 * (e >> 2) + (e & 3)];
      bits = ent & 0xfffffu;
      for (uint32_t sk = st >> 8; sk > 0; --sk) bits &= bits - 1u;
    }
    nxt = rowtab[16 * min(e + 1, QS::kLastE)];
    ncl = QS::kPack ? rowcw[16 * min(e + 1, QS::kLastE)] : clc[64 * ((e + 1) >> 2) + ((e + 1) & 3)];
    int rowb = 64 * (int)(ent >> 20);  // byte offset of the row's first joint word (group-relative)
    // packed: the look-ahead entry and the row's joint bytes as byte offsets into the
    // workgroup's LDS (group base included: no index arithmetic per term)
    const uint8_t* ldsb = reinterpret_cast<const uint8_t*>(lds);
    const uint32_t gb = 4u * (uint32_t)g;
    uint32_t eb = gb + 64u * (uint32_t)(QS::kRowTab + min(e + 1, QS::kLastE));
    uint32_t rowo = gb + (uint32_t)rowb;
    constexpr int kU = kQuadU;
    // kU terms of the lane's run from its t-th on (finished lanes load +0.0f)
    auto step = [&](int t, float* v) {
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int j = __builtin_ctz(bits | 0x100000u);  // < 21
        bits &= bits - 1u;
        const int jo = 64 * (j >> 2) + (j & 3);
        const uint32_t cJ = QS::kPack ? ldsb[rowo + jo] : jnt[rowb + jo];
        int idx;
        if (QS::kPack) {  // cL, cR: packed marginal words
          const uint32_t cR = colw[16 * j];
          const uint32_t a = max(cL, cR), b = min(cL, cR);
          idx = (int)((a >> 13) + (b & 0x1fffu) + cJ);
        } else {
          const uint32_t cR = crb[jo];
          const int a = (int)max(cL, cR), b = (int)min(cL, cR);
          idx = mi_c3(a) + (int)(mul_u24((uint32_t)b, (uint32_t)(b - 1)) >> 1) + (int)cJ;
        }
        // lanes past their run issue no gather (exec-masked: no address work in the TA)
        float tv = 0.0f;
        if (t + u < nq) tv = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rtab, 4 * (idx - 1), 0, 0));
        v[u] = tv;
        // next non-empty row of the compacted table (read one ahead)
        const bool z = bits == 0u;
        bits = z ? (nxt & 0xfffffu) : bits;
        cL = z ? ncl : cL;
        if (QS::kPack) {
          rowo = z ? gb | ((nxt >> 20) << 6) : rowo;
          eb = z ? eb + 64u : eb;
          nxt = *reinterpret_cast<const uint32_t*>(ldsb + eb);
          ncl = *reinterpret_cast<const uint32_t*>(ldsb + eb + 64 * (QS::kRowCL - QS::kRowTab));
        } else {
          e = z ? min(e + 1, QS::kLastE) : e;
          rowb = z ? 64 * (int)(nxt >> 20) : rowb;
          nxt = rowtab[16 * min(e + 1, QS::kLastE)];
          ncl = clc[64 * ((e + 1) >> 2) + ((e + 1) & 3)];
        }
      }
    };
    float MI = 0.0f;
    if constexpr (QS::kPack) {
      // Terms stay in registers (no LDS slots: 164 words per pair, 15
      // workgroups per CU instead of 9).  Lane q's terms are T[0, nq), then
      // +0.0f up to tmax.  The pair's terms left to right
      // (mutual_information.cpp:78-84) are lane 0's, then lane 1's, 2's, 3's:
      // every lane adds the quad's lane-qq terms by a DPP broadcast, and
      // adding the +0.0f tail leaves a sum unchanged (no term and no partial
      // sum is -0.0f: pJ > 0 and log2f(x) = +0.0f only at x = 1).
      float T[QS::kMaxT];
#pragma unroll
      for (int t = 0; t < QS::kMaxT; t += kU) {
        if (t < tmax) {  // (wave-uniform; no early exit: a break copies T at every exit)
          step(t, T + t);
        } else {
#pragma unroll
          for (int u = 0; u < kU; ++u) T[t + u] = 0.0f;
        }
      }
#pragma unroll
      for (int t = 0; t < QS::kMaxT; t += kU) {
        if (t < tmax) {  // (uniform guards, not breaks: the sums stay unrolled, T stays in registers)
#pragma unroll
          for (int u = 0; u < kU; ++u) MI += T[t + u];
        }
      }
#pragma unroll
      for (int t = 0; t < QS::kMaxT; t += kU) {
        if (t < tmax) {
#pragma unroll
          for (int u = 0; u < kU; ++u) MI += bcast_lane<1>(T[t + u]);
        }
      }
#pragma unroll
      for (int t = 0; t < QS::kMaxT; t += kU) {
        if (t < tmax) {
#pragma unroll
          for (int u = 0; u < kU; ++u) MI += bcast_lane<2>(T[t + u]);
        }
      }
#pragma unroll
      for (int t = 0; t < QS::kMaxT; t += kU) {
        if (t < tmax) {
#pragma unroll
          for (int u = 0; u < kU; ++u) MI += bcast_lane<3>(T[t + u]);
        }
      }
      wave_sync();  // the walk's joint reads precede the clears
#pragma unroll
      for (int kk = 0; kk < 5; ++kk) {
        uint32_t* row = hg + 16 * 5 * (q + 4 * kk);
#pragma unroll
        for (int m = 0; m < 5; ++m) row[16 * m] = 0u;
      }
    } else {
      // unpacked (N > 127): each lane stores its terms in the pair's slots, lane 0 sums them in order
      float* slots = reinterpret_cast<float*>(hg + 16 * QS::kTerms);
      float vp[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) vp[u] = 0.0f;
      for (int t = 0; t < tmax; t += kU) {
        float v[kU];
        step(t, v);
#pragma unroll
        for (int u = 0; u < kU; ++u)
          if (t - kU + u >= 0 && t - kU + u < nq) slots[16 * (s0 + t - kU + u)] = vp[u];
#pragma unroll
        for (int u = 0; u < kU; ++u) vp[u] = v[u];
      }
      {
        const int t = (tmax + kU - 1) / kU * kU;
#pragma unroll
        for (int u = 0; u < kU; ++u)
          if (t - kU + u >= 0 && t - kU + u < nq) slots[16 * (s0 + t - kU + u)] = vp[u];
      }
      wave_sync();  // the walk's joint reads precede the clears
#pragma unroll
      for (int kk = 0; kk < 5; ++kk) {
        uint32_t* row = hg + 16 * 5 * (q + 4 * kk);
#pragma unroll
        for (int m = 0; m < 5; ++m) row[16 * m] = 0u;
      }
      wave_sync();  // slots written by the quad
      if (q == 0) {
        int s = 0;
        for (; s + 8 <= total; s += 8) {
          float x[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) x[u] = slots[16 * (s + u)];
#pragma unroll
          for (int u = 0; u < 8; ++u) MI += x[u];
        }
        for (; s < total; ++s) MI += slots[16 * s];
      }
    }
    if (q == 0) {
      if (EPI) {
        if (k < ntot) em.sc[k] = live ? (double)MI : -INFINITY;
      } else if (k < n) {
        out[k] = MI;
      }
    }
  }
}

// Latency-bound batches: 16 lanes per pair (me_device.hpp GroupHist).
constexpr int kGroupBlock = 256;
__global__ __launch_bounds__(kGroupBlock) void mi_pairs_group_kernel(const uint8_t* __restrict__ imgL, int strideL,
                                                                     const uint8_t* __restrict__ imgR, int strideR,
                                                                     const int32_t* __restrict__ xyL,
                                                                     const int32_t* __restrict__ xyR, int n, int pw,
                                                                     int ph, float invN, const float* __restrict__ tab,
                                                                     float* __restrict__ out, long bytesL, long bytesR) {
  __shared__ uint32_t lds[(kGroupBlock / 16) * kGroupWords];
  const int grp = threadIdx.x >> 4;
  GroupHist<16> h{&lds[grp * kGroupWords], (int)(threadIdx.x & 15)};
  for (int k = blockIdx.x * (kGroupBlock / 16) + grp; k < n; k += gridDim.x * (kGroupBlock / 16)) {
    const int2 cl = reinterpret_cast<const int2*>(xyL)[k];
    const int2 cr = reinterpret_cast<const int2*>(xyR)[k];
    const float mi = group_mi<false>(h, imgL + (long)cl.y * strideL + cl.x, strideL,
                                     imgR + (long)cr.y * strideR + cr.x, strideR, pw, ph, invN, tab, imgL + bytesL,
                                     imgR + bytesR);
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

// ME_MI_KERNEL=lane selects the one-lane-per-pair kernel (A/B timing; same results)
inline bool mi_use_lane_kernel() {
  static const bool lane = [] {
    const char* e = getenv("ME_MI_KERNEL");
    return e && strcmp(e, "lane") == 0;
  }();
  return lane;
}

// Epipolar MI stereo matcher of the VO loop (pipeline.WindowedStereoVO.
// stereo_match / _pick, restated on the device).  Two passes:
//  * score: every (feature, candidate disparity) pair is one 16-lane group's
//    MI (group_mi: the bits of me_mi_scores), dealt flat over a grid-stride
//    loop -- a feature's candidates run side by side, not on one workgroup's
//    chain (the full-range search of new features has 127 of them);
//  * pick: one thread per feature, exactly as the numpy restatement, in FP64
//    (first maximum, interior, parabola vertex, uniqueness against the best
//    outside +-2 candidates, x_r = u - disparity, margin test).
// n_dev (optional): the feature count a preceding kernel left on the device.
constexpr int kEpiMaxNd = 512, kEpiBlock = 256, kEpiGroups = kEpiBlock / 16, kBlockPick = 256;
__global__ __launch_bounds__(kEpiBlock) void mi_epi_score_kernel(
    const uint8_t* __restrict__ L, const uint8_t* __restrict__ R, int stride, int width, int height,
    const float* __restrict__ uv, const int32_t* __restrict__ lo, const uint8_t* __restrict__ valid,
    const uint8_t* __restrict__ status, int n, const int32_t* __restrict__ n_dev, int nd, int patch, int d_max,
    float margin, float invN, double* __restrict__ sc) {
  __shared__ uint32_t lds[kEpiGroups * kGroupWords];
  const int grp = threadIdx.x >> 4;
  GroupHist<16> h{&lds[grp * kGroupWords], (int)(threadIdx.x & 15)};
  const int nf = n_dev ? min(n, *n_dev) : n;
  const long total = (long)nf * nd;
  const int half = patch / 2;
  for (long q = (long)blockIdx.x * kEpiGroups + grp; q < total; q += (long)gridDim.x * kEpiGroups) {
    const int f = (int)(q / nd), c = (int)(q - (long)f * nd);
    const float u = uv[2 * f], v = uv[2 * f + 1];
    // Rect(x - w, y - w, ..) corner (floor of the FP64 value, as the restatement)
    const int x0 = (int)floor((double)u - half), y0 = (int)floor((double)v - half);
    bool fv = valid ? valid[f] != 0 : true;
    if (status)  // the KLT gate: status 1 and inside the feature margin
      fv = fv && status[f] == 1 && u >= margin && u < (float)width - margin && v >= margin &&
           v < (float)height - margin;
    const int d = lo[f] + c, xr = x0 - d;
    const bool ok = fv && xr >= 0 && d <= d_max && x0 >= 0 && y0 >= 0 && x0 + patch <= width &&
                    y0 + patch <= height;  // (group-uniform; both patches inside the image)
    float s = 0.0f;
    const long end = (long)(height - 1) * stride + width;  // one past each image's last byte
    if (ok) s = group_mi<false>(h, L + (long)y0 * stride + x0, stride, R + (long)y0 * stride + xr, stride, patch, patch,
                                invN, nullptr, L + end, R + end);
    if (h.gl == 0) sc[q] = ok ? (double)s : -INFINITY;
  }
}

// One wave per feature: lanes take candidates lane, lane + 64, ...; the first
// maximum (largest score, smallest index on ties: np.argmax) and the best
// outside +-2 candidates by wave reductions (exact: max / compare only).
__global__ __launch_bounds__(kBlockPick) void mi_epi_pick_kernel(const float* __restrict__ uv,
                                                                 const int32_t* __restrict__ lo, int n,
                                                                 const int32_t* __restrict__ n_dev, int nd, int unique,
                                                                 double ratio, float margin,
                                                                 const double* __restrict__ scores,
                                                                 float* __restrict__ xr_out,
                                                                 uint8_t* __restrict__ ok_out) {
  const int lane = threadIdx.x & 63;
  const int f = blockIdx.x * (kBlockPick / 64) + (threadIdx.x >> 6);
  if (f >= (n_dev ? min(n, *n_dev) : n)) return;  // (wave-uniform)
  const double* sc = scores + (long)f * nd;
  double bv = -INFINITY;
  int bi = nd;  // (no score above -inf: np.argmax gives 0)
  for (int c = lane; c < nd; c += 64) {
    const double x = sc[c];
    if (x > bv) {
      bv = x;
      bi = c;
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double ov = __shfl_xor(bv, off, 64);
    const int oi = __shfl_xor(bi, off, 64);
    if (ov > bv || (ov == bv && oi < bi)) {
      bv = ov;
      bi = oi;
    }
  }
  const int k = bi == nd ? 0 : bi;
  const double best = bi == nd ? -INFINITY : bv;
  double second = -INFINITY;
  if (unique) {
    for (int c = lane; c < nd; c += 64)
      if (c < k - 2 || c > k + 2) second = fmax(second, sc[c]);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) second = fmax(second, __shfl_xor(second, off, 64));
  }
  if (lane != 0) return;
  bool ok = k > 0 && k < nd - 1 && isfinite(best);
  const int kk = min(max(k, 1), nd - 2);
  const double sm = sc[kk - 1], s0 = sc[kk], sp = sc[kk + 1];
  const double den = sm - 2.0 * s0 + sp;
  ok = ok && isfinite(sm) && isfinite(sp) && den < 0.0;
  if (unique) ok = ok && best >= ratio * second;
  const double den_s = ok ? den : -1.0;
  const double delta = ok ? 0.5 * (sm - sp) / den_s : 0.0;
  const double disp = (double)(lo[f] + kk) + delta;
  const float xr_f = (float)((double)uv[2 * f] - disp);
  ok = ok && xr_f >= margin;
  xr_out[f] = xr_f;
  ok_out[f] = ok ? 1 : 0;
}

}  // namespace

static int epipolar_launch(me_ctx* c, const uint8_t* imgL, const uint8_t* imgR, int width, int height, int stride,
                           const float* uv, const int32_t* lo, const uint8_t* valid, const uint8_t* status, int n,
                           const int32_t* n_dev, int nd, int patch, int d_max, int unique, double ratio, float margin,
                           float* xr_out, uint8_t* ok_out) {
  if (!c) return ME_ERR_INVALID;
  ME_CHECK(c, n >= 0 && nd >= 3 && nd <= kEpiMaxNd && patch > 0 && patch * patch <= 255 && width > 0 && height > 0 &&
                  stride >= width,
           "me_mi_epipolar_match: bad sizes (3 <= nd <= %d, patch <= 15)", kEpiMaxNd);
  if (n == 0) return ME_OK;
  ME_HIP(c, hipSetDevice(c->device));
  ME_CHECK(c, (long)n * nd < (1L << 31), "me_mi_epipolar_match: too many candidates");
  void* sc;
  ME_TRY(me_scratch(c, SLOT_EPI, 8 * (size_t)n * nd, &sc));
  const float* tab = nullptr;
  if (patch == 11) ME_TRY(me_mi_table(c, 121, &tab));
  me_ktimer t(c, ME_KT_MI);
  const long pairs = (long)n * nd;
  if (patch == 11) {
    // one lane per candidate pair (table-driven terms, the batch kernel's bits)
    EpiMap em{uv, lo, valid, status, n_dev, nd, d_max, width, height, patch / 2, margin, (double*)sc};
    const long img_bytes = (long)stride * (height - 1) + width;
    if (!mi_use_lane_kernel()) {
      const int qb = (int)std::min<long>((pairs + kQuadGroups - 1) / kQuadGroups, 16384);
      hipLaunchKernelGGL((mi_quad_kernel<11, 11, true>), dim3(qb), dim3(kQuadBlock), 0, c->stream, imgL, stride, imgR,
                         stride, img_bytes, img_bytes, nullptr, nullptr, n, 11, 11, tab, (int)(4 * mi_tab_size(121)),
                         nullptr, em);
      ME_TRY(me_check_launch(c, "mi_quad_kernel<epi>"));
    } else {
      const int blocks = (int)std::min<long>((pairs + kLaneBlock - 1) / kLaneBlock, 8192);
      hipLaunchKernelGGL((mi_lane_kernel<11, 11, true>), dim3(blocks), dim3(kLaneBlock), 0, c->stream, imgL, stride,
                         imgR, stride, img_bytes, img_bytes, nullptr, nullptr, n, 11, 11, tab,
                         (int)(4 * mi_tab_size(121)), nullptr, em);
      ME_TRY(me_check_launch(c, "mi_lane_kernel<epi>"));
    }
  } else {
    // grid-stride over n x nd 16-lane groups: at most ~8 workgroups per CU (28 KB of LDS each)
    const int blocks = (int)std::min<long>((pairs + kEpiGroups - 1) / kEpiGroups, 8L * std::max(c->num_cu, 1));
    hipLaunchKernelGGL(mi_epi_score_kernel, dim3(blocks), dim3(kEpiBlock), 0, c->stream, imgL, imgR, stride, width,
                       height, uv, lo, valid, status, n, n_dev, nd, patch, d_max, margin,
                       inv_count((long)patch * patch), (double*)sc);
    ME_TRY(me_check_launch(c, "mi_epi_score_kernel"));
  }
  hipLaunchKernelGGL(mi_epi_pick_kernel, dim3((n + kBlockPick / 64 - 1) / (kBlockPick / 64)), dim3(kBlockPick), 0,
                     c->stream, uv,
                     lo, n, n_dev, nd, unique, ratio, margin, (const double*)sc, xr_out, ok_out);
  return me_check_launch(c, "mi_epi_pick_kernel");
}

extern "C" int me_mi_epipolar_match(me_ctx* c, const uint8_t* imgL, const uint8_t* imgR, int width, int height,
                                    int stride, const float* uv, const int32_t* lo, const uint8_t* valid,
                                    const uint8_t* status, int n, int nd, int patch, int d_max, int unique,
                                    double ratio, float margin, float* xr_out, uint8_t* ok_out) {
  me_range range_("me_mi_epipolar_match");
  return epipolar_launch(c, imgL, imgR, width, height, stride, uv, lo, valid, status, n, nullptr, nd, patch, d_max,
                         unique, ratio, margin, xr_out, ok_out);
}

extern "C" int me_mi_epipolar_match_count(me_ctx* c, const uint8_t* imgL, const uint8_t* imgR, int width, int height,
                                          int stride, const float* uv, const int32_t* lo, const int32_t* n_dev,
                                          int n_max, int nd, int patch, int d_max, int unique, double ratio,
                                          float margin, float* xr_out, uint8_t* ok_out) {
  me_range range_("me_mi_epipolar_match_count");
  if (!c) return ME_ERR_INVALID;
  ME_CHECK(c, n_dev != nullptr, "me_mi_epipolar_match_count: null count");
  return epipolar_launch(c, imgL, imgR, width, height, stride, uv, lo, nullptr, nullptr, n_max, n_dev, nd, patch, d_max,
                         unique, ratio, margin, xr_out, ok_out);
}

// Batch launcher.
int me_launch_mi_pairs(me_ctx* c, const uint8_t* dL, int sL, const uint8_t* dR, int sR, int width, int height,
                       const int32_t* dxyL, const int32_t* dxyR, int n, int pw, int ph, float* dout) {
  if (n <= 0) return ME_OK;
  me_ktimer t(c, ME_KT_MI);
  const float* gtab;  // the group kernels' terms come from the same per-N table
  ME_TRY(me_mi_table(c, pw * ph, &gtab));
  // one past each image's last byte (the row windows' bound)
  const long endL = (long)sL * (height - 1) + width, endR = (long)sR * (height - 1) + width;
  if (n < kGroupThreshold) {
    // fewer pairs than lanes to fill the chip: 16 lanes per pair
    const int per = kGroupBlock / 16;
    int blocks = (n + per - 1) / per;
    hipLaunchKernelGGL(mi_pairs_group_kernel, dim3(blocks), dim3(kGroupBlock), 0, c->stream, dL, sL, dR, sR, dxyL,
                       dxyR, n, pw, ph, inv_count((long)pw * ph), gtab, dout, endL, endR);
    return me_check_launch(c, "mi_pairs_group_kernel");
  }
  const int npx = pw * ph;
  if (pw > 12) {  // wider than one realigned 16-byte row load: the group kernel handles any shape
    const int per = kGroupBlock / 16;
    hipLaunchKernelGGL(mi_pairs_group_kernel, dim3((n + per - 1) / per), dim3(kGroupBlock), 0, c->stream, dL, sL, dR,
                       sR, dxyL, dxyR, n, pw, ph, inv_count((long)npx), gtab, dout, endL, endR);
    return me_check_launch(c, "mi_pairs_group_kernel");
  }
  const float* tab;
  ME_TRY(me_mi_table(c, npx, &tab));
  // bounds of the realigned 16-byte row loads: never read past the images
  const long img_bytes_L = (long)sL * (height - 1) + width, img_bytes_R = (long)sR * (height - 1) + width;
  if (!mi_use_lane_kernel()) {
    const int qb = (int)std::min<long>(((long)n + kQuadGroups - 1) / kQuadGroups, 16384);
    const int tb = (int)(4 * mi_tab_size(npx));
    if (pw == 11 && ph == 11)
      hipLaunchKernelGGL((mi_quad_kernel<11, 11>), dim3(qb), dim3(kQuadBlock), 0, c->stream, dL, sL, dR, sR,
                         img_bytes_L, img_bytes_R, dxyL, dxyR, n, pw, ph, tab, tb, dout);
    else if (pw == 10 && ph == 10)
      hipLaunchKernelGGL((mi_quad_kernel<10, 10>), dim3(qb), dim3(kQuadBlock), 0, c->stream, dL, sL, dR, sR,
                         img_bytes_L, img_bytes_R, dxyL, dxyR, n, pw, ph, tab, tb, dout);
    else
      hipLaunchKernelGGL((mi_quad_kernel<0, 0>), dim3(qb), dim3(kQuadBlock), 0, c->stream, dL, sL, dR, sR,
                         img_bytes_L, img_bytes_R, dxyL, dxyR, n, pw, ph, tab, tb, dout);
    return me_check_launch(c, "mi_quad_kernel");
  }
  int blocks = (n + kLaneBlock - 1) / kLaneBlock;
  if (blocks > 8192) blocks = 8192;
  if (pw == 11 && ph == 11)
    hipLaunchKernelGGL((mi_lane_kernel<11, 11>), dim3(blocks), dim3(kLaneBlock), 0, c->stream, dL, sL, dR, sR, img_bytes_L,
                       img_bytes_R, dxyL, dxyR, n, pw, ph, tab, (int)(4 * mi_tab_size(npx)), dout);
  else if (pw == 10 && ph == 10)
    hipLaunchKernelGGL((mi_lane_kernel<10, 10>), dim3(blocks), dim3(kLaneBlock), 0, c->stream, dL, sL, dR, sR, img_bytes_L,
                       img_bytes_R, dxyL, dxyR, n, pw, ph, tab, (int)(4 * mi_tab_size(npx)), dout);
  else
    hipLaunchKernelGGL((mi_lane_kernel<0, 0>), dim3(blocks), dim3(kLaneBlock), 0, c->stream, dL, sL, dR, sR, img_bytes_L,
                       img_bytes_R, dxyL, dxyR, n, pw, ph, tab, (int)(4 * mi_tab_size(npx)), dout);
  return me_check_launch(c, "mi_lane_kernel");
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
  me_range range_("me_mi_scores");
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
