// ba_kernels.hpp — device kernels of the windowed stereo bundle adjuster
// (SURVEY §8a A13-A17).  Included by ba.hip only.
//
// Replaces the Ceres solve behind BundleAdjuster<4>::optimise
// (include/MotionEstimation/optimisation/BundleAdjuster.h:431-476) and
// BundleAdjuster<2>::optimise (:378-429):
//   linearize      per observation: StereoReprojectionError (:153-171), or
//                  StandardReprojectionError (:71-103) / StereoRightError
//                  (:106-139) chosen by camID for <2>, value + analytic
//                  Jacobian (2-row residuals padded with zero rows, so every
//                  later stage is shared), HuberLoss(1.0) corrector, cost;
//                  stores only the normal-equation pieces (J^T J, J^T r
//                  blocks), never the Jacobian itself.
//   cam_assemble   ck workgroups per variable camera, the last to finish
//                  reduces: Jacobi column norms (iteration 0), scaled
//                  U = Jc'Jc, g_c = Jc'r.
//   pt_schur       per landmark sub-chunk: V = Jp'Jp, g_p, V + D/radius ->
//                  Cholesky L_p, z_p = L_p^-1 g_p, the landmark's rows of
//                  Y = W L_p^-T (and z_p) in LDS, partial tiles of Y^T [Y | z]
//                  on v_mfma_f64_16x16x4f64 (deterministic, no atomics).
//   s_assemble     S = U - sum of the partial tiles, b = g - Y^T z.
//   cam_solve      one workgroup: S = U + D/radius - sum(partials), dense
//                  Cholesky, y_c = -S^-1 b, candidate cameras.
//   pt_step        16 lanes per point: y_p, candidate point (bounds
//                  projection), step norms, the point's part of the model
//                  cost change (normal-equation form) and the candidate
//                  cost of the point's observations; its last
//                  workgroup reduces them and runs decide (Ceres LM
//                  acceptance / radius / termination).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ba {

typedef double double4_t __attribute__((ext_vector_type(4)));

constexpr int kBlock = 256;
constexpr int kObsxStride = 9;   // V_o (6 unique) + g_o (3), unscaled

struct Opts {
  int max_num_iterations;
  double function_tolerance, gradient_tolerance, parameter_tolerance;
  double initial_radius, max_radius, min_radius, min_diag, max_diag, min_rel_decrease;
  int max_invalid;
};

struct State {
  int cur;            // parameter buffer holding x
  int need_lin;       // linearize at the start of this iteration
  int done;
  int termination;    // 0 CONVERGENCE, 1 NO_CONVERGENCE, 2 FAILURE
  int iterations, successful, invalid_count;
  int fail;           // linear solver failure in this iteration
  int scaled;         // jacobi scaling computed
  int accepted;
  int bad_input;      // device-resident input: an observation indexes outside the window
  int infeasible;     // a starting point violates the box bounds (Ceres IsFeasible -> FAILURE)
  int final_pass;     // set by pt_schur: this linearisation only feeds the closing gradient test
  int spin_err;       // a bounded cross-workgroup wait timed out (partner not co-resident): the solve ends in error
  int pad[2];
  double radius, decrease;
  double x_cost, cand_cost, model_change, initial_cost;
  double cam_step2, cam_xn2, cam_model;  // cam_model: -(g_c.y_c + y_c^T U y_c / 2), this rank's camera part
  double last_q;
  long long stamps[16];  // s_memtime at cam_solve phase ends (ME_SOLVE_SKIP & 256)
};

// Scalars reduced from block partials (one slot per quantity).
enum { R_COST = 0, R_GMAX_PT, R_MODEL, R_CAND, R_STEP2, R_XN2, R_COUNT };

struct Geo {
  int nc, np, no, nf, m, n6, Rpad, T, Ts, spts, nsub, ksplit, npairs, nblk_obs, nblk_lin, nblk_pts, nblk_step, pstride, jacobi,
      ck;
  // band-sorted Schur pass (plan_band / plan_order): landmark runs of rlen = spts x rsub landmarks in
  // (first tile, last tile) order, each split into sgrp tile groups of stpw tiles (ksplit = nruns x sgrp)
  int nruns, rlen, rsub, sgrp, stpw, nblkp;
  int sorted;              // 0: runs in landmark order, every run takes the whole tile set (small windows)
  int od;                  // residual rows per observation: 4 StereoReprojectionError, 2 Standard/StereoRight
  int xslots, xrank;       // sharded: gradient max-norm slots in the exchange (one per rank) and this rank's
  double K0[9], K1[9];
  double baseline, sinv;
  double lo[3], hi[3];     // point bounds (BundleAdjuster.h:442-460)
};

struct Bufs {
  double* cams[2];
  double* pts[2];
  const double* obs;
  const int* cam_idx;
  const int* pt_idx;
  const int* cam_id;  // od == 2: Observation::camID (0 left -> StandardReprojectionError, else StereoRightError)
  int* p_off;         // CSR by point (obs sorted by cam inside a point)
  int* p_obs;
  int* pos;           // obs -> CSR slot
  int* p_cam;         // CSR slot -> variable camera index (-1 fixed)
  int* c_off;         // CSR by variable camera (original observation order inside a camera)
  int* c_obs;
  int* tmp_obs;       // plan: unsorted CSR-by-point slots
  int* cpos;          // obs -> slot in c_obs (-1: fixed camera)
  double* obsx;       // no * 9  (V_o, g_o unscaled)
  uint8_t* dup;       // obs shares (point, camera) with another obs
  double* Abuf;       // n6 * (n6|1) factorisation workspace (when S does not fit LDS)
  double* Wo;         // no * 18 (unscaled Jc^T Jp, row-major 6x3)
  double* csc;        // 6m jacobi scaling (cameras)
  double* psc;        // 3np (points)
  double* U;          // m * 36 scaled Jc^T Jc
  double* gcs;        // 6m scaled gradient
  double* V;          // np * 9 scaled Jp^T Jp
  double* gps;        // 3np scaled gradient
  double* Lp;         // np * 9 Cholesky of V + D/radius
  double* zp;         // 3np
  double* Spart;      // nruns * npairs * 256 partial tiles of Y^T [Y | z]: run r's tile c at slot r * npairs + c
  int* order;         // np landmarks in band order (the Schur runs)
  int* rband;         // 2 * nruns: first / last tile of each run's camera band (its tile set adds the z tile T-1)
  int* tl;            // npairs * nruns: per tile pair, the partial slots of the runs covering it, in run order
  int* tcnt;          // npairs: entries of tl per tile pair
  int* pkey;          // plan: per landmark band key (first tile * T + last tile)
  int* prank;         // plan: stable rank of the key inside its 256-landmark block
  int* phist;         // plan: T^2 x nblkp key counts per block, scanned in place into offsets
  double* S;          // n6 * n6 (assembled / reduced)
  double* bvec;       // n6
  double* diagU;      // n6 (for the sharded all-reduce)
  double* yc;         // n6
  double* dp;         // 3np point step (unscaled)
  double* part;       // R_COUNT * max(nblk_obs, nblk_pts)
  double* scal;       // R_COUNT reduced scalars (all-reduce target in sharded mode)
  State* st;
  int* work;          // plan build: cnt_p[np] | fill_p[np] | blk_cam[nblk_obs*nc] | flags[4] (zeroed)
  unsigned* cnt;      // last-arrival counters: m (cam_assemble, per camera) + 1 (pt_step); re-armed by the last
  unsigned* ssync;    // camera solve, global-memory form: {step epoch, worker step count} (zeroed by s_assemble)
  unsigned* roster;   // camera solve: the trailing workers' roster (roster.hpp; 2 words, re-zeroed by pt_step)
  unsigned* asm_claim;  // fused assembly: per unit, the generation of the launch whose workgroup claimed it
  double* out;        // State | cams[cur] | pts[cur] for the single read-back
  double* xch;        // sharded only (else null): the packed per-iteration exchange, see xo_* below
};

// Layout of the sharded exchange buffer (one all-reduce per LM iteration after
// the Schur pass): the reduced camera system in the Schur tile layout
// [npairs x 16 x 16: the upper block triangle of [S | b], tile pair p = (I <= J)]
// | diag(U) (n6) | raw camera gradient (n6, the gradient-tolerance test) |
// cost | failure count | one gradient max-norm slot per rank (a max carried by
// a sum: every rank writes its own slot, the others hold 0).
__host__ __device__ inline long xo_diag(const Geo& g) { return (long)g.npairs * 256; }
__host__ __device__ inline long xo_gc(const Geo& g) { return xo_diag(g) + g.n6; }
__host__ __device__ inline long xo_cost(const Geo& g) { return xo_gc(g) + g.n6; }
__host__ __device__ inline long xo_fail(const Geo& g) { return xo_cost(g) + 1; }
__host__ __device__ inline long xo_gmax(const Geo& g) { return xo_fail(g) + 1; }
__host__ __device__ inline long xo_total(const Geo& g) { return xo_gmax(g) + g.xslots; }

}  // namespace ba
