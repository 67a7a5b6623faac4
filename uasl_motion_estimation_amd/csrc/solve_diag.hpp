// solve_diag.hpp -- the camera solve's diagonal-block factorisation (ba.hip),
// kept in a header so tools/ubench/diag.hip times the same code in isolation.
#pragma once
#include <hip/hip_runtime.h>

typedef double double4_t __attribute__((ext_vector_type(4)));

// wave-local ordering of LDS (and, for the global fallback, L1) traffic
__device__ __forceinline__ void solve_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
#ifndef ME_RSQ_NR
#define ME_RSQ_NR 1
#endif
__device__ __forceinline__ double rsqrt_nr(double p) {
  double r = __builtin_amdgcn_rsq(p);
  r = r * fma(-0.5 * p * r, r, 1.5);
  if (ME_RSQ_NR > 1) r = r * fma(-0.5 * p * r, r, 1.5);
  return r;
}
// Diagonal block on ONE wave with the rank-4 updates on the matrix cores.  The block [A | Y] (Y -> X = L^-1) sits in two
// v_mfma_f64_16x16x4f64 accumulators: lane l = 16 q + c holds A[q + 4i][c] and
// Y[q + 4i][c] in register i.  Round R (pivots p0 = 4R .. p0 + 3):
//  * register R holds the round's pivot rows: A[p0 + q][c] (= A[c][p0 + q],
//    symmetry) and Y[p0 + q][c].  Every lane gathers the four values of its
//    column c from the four 16-lane rows with v_permlane16/32_swap (no LDS),
//    and the 4 x 4 pivot block by readlane (uniform values);
//  * the pivot block is factored redundantly by every lane, and each lane
//    forms its row of the panel, L[c][p0 .. p0+3], and its column of the pivot
//    rows of X, X[p0 .. p0+3][c], by 4-step substitutions (for c inside the
//    pivot block the same recurrence yields the block's own L entries);
//  * the trailing part of [A | Y] is updated by two MFMAs:
//    A -= Lp Lp^T and Y -= Lp X_p, with Lp = the panel (rows >= p0 + 4, zero
//    above), whose operand in lane l is L[c][p0 + q] for both A and B.
// No workgroup barrier and no LDS round trip inside the block: per round the
// uniform pivot chain, the substitutions and two MFMAs.
#ifndef ME_DIAG_EXP
#define ME_DIAG_EXP 0  // timing experiments only (tools/ubench/diag.hip), results invalid: 1 no Newton step, 2 no MFMA, 4 no rsq, 8 no substitutions
#endif
#ifndef ME_DIAG_GATHER
#define ME_DIAG_GATHER 1  // 1: permlane swaps + readlane, 0: wave-private LDS scratch (3.34k vs 3.49k ticks per block in
                          // isolation, tools/ubench/diag.hip; DPP row broadcasts instead of readlane: 3.64k, dropped)
#endif
__device__ __forceinline__ double lane_read(double x, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), l),
                          __builtin_amdgcn_readlane(__double2loint(x), l));
}
// x held as x[q][c] by lane 16 q + c  ->  o[u] = x[u][c] on every lane
__device__ __forceinline__ void col_gather4(double x, double o[4]) {
  const int lo = __double2loint(x), hi = __double2hiint(x);
  const auto sl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);  // [0]: row q & 2, [1]: row (q & 2) | 1
  const auto sh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  const auto al = __builtin_amdgcn_permlane32_swap(sl[0], sl[0], false, false);  // [0]: row 0, [1]: row 2
  const auto ah = __builtin_amdgcn_permlane32_swap(sh[0], sh[0], false, false);
  const auto bl = __builtin_amdgcn_permlane32_swap(sl[1], sl[1], false, false);  // [0]: row 1, [1]: row 3
  const auto bh = __builtin_amdgcn_permlane32_swap(sh[1], sh[1], false, false);
  o[0] = __hiloint2double((int)ah[0], (int)al[0]);
  o[1] = __hiloint2double((int)bh[0], (int)bl[0]);
  o[2] = __hiloint2double((int)ah[1], (int)al[1]);
  o[3] = __hiloint2double((int)bh[1], (int)bl[1]);
}
// Rounds whose pivots are all padding or the right-hand-side row (p0 >= nreal:
// the last diagonal block of a system whose n + 1 rows end inside it) are
// skipped: nothing reads their L entries (no trailing block follows, the
// backward solve starts at block (n - 1) / 16), and their X rows are written
// as zeros -- the backward solve multiplies them by the zero entries of u
// past n.  Config 3 (n = 108): the last block's fourth round; config 5
// (n = 288): the whole last block.
#ifndef ME_DIAG_SKIP_PAD
#define ME_DIAG_SKIP_PAD 1
#endif
template <int R>
__device__ __forceinline__ void diag_round_mfma(double4_t& A4, double4_t& Y4, int q, int c, int nreal, bool& ok,
                                                double* Lblk, int lld, double* X, double* gx) {
  constexpr int p0 = 4 * R;
  if (ME_DIAG_SKIP_PAD && p0 >= nreal) {  // (wave-uniform)
    X[(p0 + q) * 16 + c] = 0.0;
    return;
  }
  double acol[4], ycol[4], Lq[4][4];
  if (ME_DIAG_GATHER) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v <= u; ++v) Lq[u][v] = lane_read(A4[R], 16 * u + p0 + v);  // A[p0+u][p0+v]
    col_gather4(A4[R], acol);  // A[p0+u][c]
    col_gather4(Y4[R], ycol);  // Y[p0+u][c]
  } else {
    double* g = gx + 128 * (R & 1);  // [c][u]: A column values | Y column values at +64
    g[4 * c + q] = A4[R];
    g[64 + 4 * c + q] = Y4[R];
    solve_wave_sync();
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      acol[u] = g[4 * c + u];
      ycol[u] = g[64 + 4 * c + u];
#pragma unroll
      for (int v = 0; v <= u; ++v) Lq[u][v] = g[4 * (p0 + v) + u];  // uniform address
    }
  }
  double Lr[4], Xg[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    double piv = Lq[t][t];
#pragma unroll
    for (int u = 0; u < t; ++u) piv = fma(-Lq[t][u], Lq[t][u], piv);
    const bool pad = p0 + t >= nreal;  // padding / right-hand-side row: never a failure
    ok = ok && (pad || piv > 0);
    piv = (pad && !(piv > 0)) ? 1.0 : piv;
    const double r = (ME_DIAG_EXP & 4) ? piv : (ME_DIAG_EXP & 1) ? __builtin_amdgcn_rsq(piv) : rsqrt_nr(piv);
    Lq[t][t] = piv * r;
#pragma unroll
    for (int v = t + 1; v < 4; ++v) {
      double x = Lq[v][t];
#pragma unroll
      for (int u = 0; u < t; ++u) x = fma(-Lq[v][u], Lq[t][u], x);
      Lq[v][t] = x * r;
    }
    double sr = acol[t], sx = ycol[t];
#pragma unroll
    for (int u = 0; u < ((ME_DIAG_EXP & 8) ? 0 : t); ++u) {
      sr = fma(-Lr[u], Lq[t][u], sr);
      sx = fma(-Lq[t][u], Xg[u], sx);
    }
    Lr[t] = sr * r;  // L[c][p0+t]
    Xg[t] = sx * r;  // X[p0+t][c]
  }
  double lq = Lr[0], xq = Xg[0];
#pragma unroll
  for (int t = 1; t < 4; ++t) {
    lq = q == t ? Lr[t] : lq;
    xq = q == t ? Xg[t] : xq;
  }
  if (c >= p0 + q) Lblk[c * lld + p0 + q] = lq;  // L[c][p0+q], lower part
  X[(p0 + q) * 16 + c] = xq;                     // X[p0+q][c]
  if (R < 3 && !(ME_DIAG_EXP & 2)) {
    const double lop = c >= p0 + 4 ? lq : 0.0;  // rows above the trailing part stay as they are
    A4 = __builtin_amdgcn_mfma_f64_16x16x4f64(-lop, lop, A4, 0, 0, 0);
    Y4 = __builtin_amdgcn_mfma_f64_16x16x4f64(-lop, xq, Y4, 0, 0, 0);
  }
}

