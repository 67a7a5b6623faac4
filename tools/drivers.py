"""GPU workload drivers for profiling and A/B timing (run on the GPU box,
usually through tools/gpu.sh): each subcommand runs one hot-path workload of
the bench's configurations and prints its timing; `--lib LIB` (or ME_LIB)
loads another build of libme_hip.so (tools/build_variant.sh).

  ba_wall [CONFIGS]      wall time of one 10-iteration BA solve (configs 3,4,5 or NFxW at 1280x720)
  klt [--reps --check]   klt_kernel on the config-3 frame (2000 features), bit-exact check vs the oracle
  mi [--pairs --reps --check]
                         batch MI kernel (1M 11x11 pairs), self-check vs the group kernel
  coop [--reps]          scale LM (config 3) and config-5 BA wall clocks (tools/gpu.sh coop: plain vs
                         cooperative launch build)
  solve_ts               cam_solve_kernel phase stamps (a -DME_SOLVE_TS build), configs 3 and 5
  scale_ts [--front F]   persistent scale LM phase split (a -DME_SCALE_TS build)
  schur_stamps           pt_schur_kernel workgroup-0 stamps (a -DME_SCHUR_STAMPS build)
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _setup(lib):
    import torch  # noqa: F401  (device runtime up before the library)

    from uasl_motion_estimation_amd import _lib
    if lib:
        _lib.load_library(lib)
    from uasl_motion_estimation_amd._lib import Context
    return Context(0)


def _ba_problem(c):
    from uasl_motion_estimation_amd import synthetic as S
    if "x" in c:  # NFEATSxWINDOW at 1280x720
        nf, w = (int(v) for v in c.split("x"))
        return S.ba_problem(S.SEED0 * 7 + w, nf, w, 1280, 720)
    cfg = S.CONFIGS[int(c)]
    return S.ba_problem(S.SEED0 * 7 + int(c), cfg["n_feats"], cfg["window"], cfg["width"], cfg["height"])


def cmd_ba_wall(a):
    from uasl_motion_estimation_amd.optimisation import DeviceBAProblem, SolverOptions
    ctx = _setup(a.lib)
    out = {}
    for c in a.configs.split(","):
        d = DeviceBAProblem(_ba_problem(c), ctx)
        o = SolverOptions.fixed_iterations(10)
        for _ in range(3):
            d.reset()
            s = d.solve(o)
        best = []
        for _ in range(3):
            ctx.synchronize()
            w0 = time.perf_counter()
            for _ in range(20):
                d.reset()
                s = d.solve(o)
            ctx.synchronize()
            best.append((time.perf_counter() - w0) / 20 * 1e3)
        out[c] = {"ms": round(min(best), 4), "iterations": s["iterations"], "cost": s["final_cost"]}
    print(json.dumps(out))


def cmd_klt(a):
    from uasl_motion_estimation_amd import synthetic as S
    from uasl_motion_estimation_amd._lib import ME_DEVICE
    from uasl_motion_estimation_amd.klt import klt_params
    ctx = _setup(a.lib)
    W, H, N = 1280, 720, 2000
    scene, K, stream = S.stereo_stream(20261018, W, H, 2)
    pts = S.grid_features(np.random.default_rng(0), N, W, H, 12).astype(np.float32)
    dp, dn, din, dout, dst = ctx.malloc(W * H), ctx.malloc(W * H), ctx.malloc(8 * N), ctx.malloc(8 * N), ctx.malloc(N)
    L0, L1 = np.ascontiguousarray(stream[0].left), np.ascontiguousarray(stream[1].left)
    ctx.h2d(dp, L0)
    ctx.h2d(dn, L1)
    ctx.h2d(din, pts)
    kp = klt_params()

    def run():
        ctx.check(ctx.lib.me_klt_track(ctx.h, ME_DEVICE, ctypes.c_void_p(dp), ctypes.c_void_p(dn), W, H, W,
                                       ctypes.c_void_p(din), ctypes.c_void_p(dout), ctypes.c_void_p(dst), N,
                                       ctypes.byref(kp)), "klt")
    for _ in range(3):
        run()
    ctx.synchronize()
    ctx.timing_reset()
    ctx.timing(True, ["KLT"])
    for _ in range(a.reps):
        run()
    ctx.synchronize()
    ctx.timing(False)
    cnt, ms = ctx.timing_read("KLT")
    print(f"klt_kernel: {1000 * ms / max(cnt, 1):.2f} us/launch ({N} features, {W}x{H})", flush=True)
    if a.check:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle as O  # checker only
        got, gst = np.zeros(2 * N, np.float32), np.zeros(N, np.uint8)
        ctx.d2h(got, dout)
        ctx.d2h(gst, dst)
        ref_pts, ref_st = O.klt(L0, L1, pts)
        same = np.array_equal(got.view(np.uint32), np.ascontiguousarray(ref_pts, np.float32).ravel().view(np.uint32)) \
            and np.array_equal(gst, ref_st)
        print(f"klt parity vs oracle: {'bit-exact' if same else 'MISMATCH'}", flush=True)
        if not same:
            sys.exit(1)


def cmd_mi(a):
    from uasl_motion_estimation_amd import synthetic as S
    from uasl_motion_estimation_amd.mutual_information import mi_scores_device
    ctx = _setup(a.lib)
    cfg = S.CONFIGS[3]
    scene, K, stream = S.stereo_stream(S.SEED0 + 3, cfg["width"], cfg["height"], 2)
    L, R = np.ascontiguousarray(stream[1].left), np.ascontiguousarray(stream[1].right)
    H, W = L.shape
    n = a.pairs
    rng = np.random.default_rng(7)
    xyL = np.stack([rng.integers(0, W - 11, n), rng.integers(0, H - 11, n)], -1).astype(np.int32)
    xyR = xyL.copy()
    xyR[:, 0] = np.clip(xyL[:, 0] - rng.integers(0, 40, n), 0, W - 11)
    dLi, dRi = ctx.malloc(L.nbytes), ctx.malloc(R.nbytes)
    ctx.h2d(dLi, L)
    ctx.h2d(dRi, R)
    dL, dR, dout = ctx.malloc(xyL.nbytes), ctx.malloc(xyR.nbytes), ctx.malloc(4 * n)
    ctx.h2d(dL, xyL)
    ctx.h2d(dR, xyR)
    run = lambda: mi_scores_device(ctx, dLi, W, dRi, W, W, H, dL, dR, n, (11, 11), dout)  # noqa: E731
    run()
    ctx.synchronize()
    ctx.timing_reset()
    ctx.timing(True)
    for _ in range(a.reps):
        run()
    ctx.synchronize()
    ctx.timing(False)
    cnt, ms = ctx.timing_read("MI")
    avg = ms / cnt
    print("pairs %d  avg %.4f ms  %.3f Gpairs/s  %.1f GB/s (262 B/pair)  frac %.4f" %
          (n, avg, n / avg / 1e6, 262 * n / avg / 1e6, 262 * n / avg / 1e6 / 8000), flush=True)
    if a.check:
        got = np.zeros(n, np.float32)
        ctx.d2h(got, dout)
        m = min(n, 200000)
        ref = np.zeros(m, np.float32)
        for s in range(0, m, 30000):  # below the batch kernel's threshold: the group kernel (parity-tested)
            e = min(m, s + 30000)
            mi_scores_device(ctx, dLi, W, dRi, W, W, H, dL + 8 * s, dR + 8 * s, e - s, (11, 11), dout + 4 * s)
        ctx.synchronize()
        ctx.d2h(ref, dout)
        bad = np.flatnonzero(got[:m].view(np.uint32) != ref.view(np.uint32))
        print("self-check vs group kernel on %d pairs: %d mismatches" % (m, len(bad)))
        if len(bad):
            sys.exit(1)


def cmd_coop(a):
    from uasl_motion_estimation_amd import synthetic as S
    from uasl_motion_estimation_amd.optimisation import (DeviceBAProblem, OptimisationParams, SolverOptions,
                                                         scale_optimise)
    ctx = _setup(a.lib)
    cfg = S.CONFIGS[3]
    seed = S.SEED0 + 3
    scene, K, stream = S.stereo_stream(seed, cfg["width"], cfg["height"], 2)
    sp = S.scale_problem(seed, cfg["width"], cfg["height"], cfg["n_feats"], window=cfg["window"], w=5,
                         frames=stream[:2], scene=scene)
    out = {"lib": a.lib or os.environ.get("ME_LIB", "tree")}
    for _ in range(3):
        r = scale_optimise(sp, OptimisationParams(), ctx=ctx)
    t0 = time.perf_counter()
    for _ in range(a.reps):
        r = scale_optimise(sp, OptimisationParams(), ctx=ctx)
    out["scale_lm_ms"] = round((time.perf_counter() - t0) / a.reps * 1e3, 4)
    out["scale_lm"] = {k: r[k] for k in ("iterations", "res_evals", "rejections")}
    d = DeviceBAProblem(_ba_problem("5"), ctx)
    o = SolverOptions.fixed_iterations(10)
    for _ in range(3):
        d.reset()
        s = d.solve(o)
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        d.reset()
        s = d.solve(o)
    ctx.synchronize()
    out["ba_config5_ms"] = round((time.perf_counter() - t0) / a.reps * 1e3, 4)
    out["ba_config5_iterations"] = s["iterations"]
    print(json.dumps(out))


def cmd_solve_ts(a):
    from uasl_motion_estimation_amd.optimisation import SolverOptions, ba_solve
    ctx = _setup(a.lib)
    fn = ctx.lib.me_solve_ts
    fn.argtypes = [ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]
    buf = (ctypes.c_longlong * 24)()
    names = {1: "lin_finalize", 2: "asm_wait", 11: "ts_asm_probe", 12: "load_issue", 13: "load_diag_barrier",
             3: "load_rest", 4: "factor", 5: "backward", 6: "tail", 8: "asm_last_exit", 9: "asm_first_entry",
             19: "f_diag0", 16: "f_w0_panel", 17: "f_w0_diag", 18: "f_barrier_wait"}
    names5 = {**names, 16: "m2_w0_diag", 17: "m2_count_wait", 18: "m2_panel", 19: "m2_drain_publish"}
    for c in a.configs.split(","):
        bp = _ba_problem(c)
        for _ in range(3):
            ba_solve(bp.copy(), SolverOptions.fixed_iterations(10), ctx=ctx)
        fn(buf, 1)
        for _ in range(20):
            ba_solve(bp.copy(), SolverOptions.fixed_iterations(10), ctx=ctx)
        fn(buf, 1)
        calls = max(buf[15], 1)
        us = {nm: round(buf[i] / calls / 100.0, 2) for i, nm in (names5 if c == "5" else names).items()}
        tot = sum(buf[i] for i in (1, 2, 3, 4, 5, 6, 11, 12, 13, 16, 17, 18, 19)) / calls / 100.0
        print(f"config {c}: calls {calls} us/launch {us} wg0 total {tot:.2f} us", flush=True)


def cmd_scale_ts(a):
    from uasl_motion_estimation_amd import synthetic as S
    from uasl_motion_estimation_amd._lib import cu_split
    from uasl_motion_estimation_amd.optimisation import OptimisationParams, ScaleCall
    import torch
    ctx = _setup(a.lib)
    if a.front:  # the bench's front-end share: front of every 16 CUs, whole XCDs
        ctx.set_cu_mask(cu_split(torch.cuda.get_device_properties(0).multi_processor_count, a.front)[0])
    fn = ctx.lib.me_scale_ts
    fn.argtypes = [ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]
    buf = (ctypes.c_longlong * 16)()
    cfg = S.CONFIGS[3]
    W, H, N, win = cfg["width"], cfg["height"], cfg["n_feats"], cfg["window"]
    seed = S.SEED0 + 3
    scene, K, stream = S.stereo_stream(seed, W, H, 3)
    sp = S.scale_problem(seed, W, H, N, window=win, w=5, frames=stream[:2], scene=scene)
    params = OptimisationParams.fixed_iterations(10)
    for rep in range(2):
        fn(buf, 1)
        for _ in range(3 if rep == 0 else 20):
            c = ScaleCall(sp, params, ctx=ctx)
            c.run()
            r = c.result()
        evals = r["executed_evals"] * N
        fn(buf, 1)
    L = max(buf[1], 1)
    us = lambda k: round(buf[k] / L / 100.0, 2)  # noqa: E731
    print(f"front_cus {a.front or 16}/16: launches {buf[1]}, phases/launch {buf[0] / L:.1f} "
          f"(A/D {buf[7] / L:.1f}, B {buf[8] / L:.1f}, C {buf[9] / L:.1f}); executed track evaluations/launch {evals}")
    print(f"  wall {us(2)} us/launch: wg0 track work A/D {us(3)} B {us(4)} C {us(5)}; wg0 waits for control {us(6)}; "
          f"control (reduce + decide) {us(10)} over {buf[11] / L:.1f} reductions")
    n7 = max(buf[7], 1)
    print(f"  A/D controls: acquire {buf[12] / n7 / 100:.2f}, reduce {buf[13] / n7 / 100:.2f}, "
          f"control {buf[14] / n7 / 100:.2f}, publish {buf[15] / n7 / 100:.2f} us")
    print(f"  ns per executed track evaluation: {1e3 * buf[2] / L / 100.0 / max(evals, 1):.2f}")


def cmd_cam_ts(a):
    """Camera (0, 0)'s assembly workgroup phases (a -DME_CAM_TS=1 build): the
    slot loop (loads + residual/Jacobian + sums), block_sum<27>, partial stores +
    arrival, and (when last) the camera reduce; s_memtime ticks per execution."""
    from uasl_motion_estimation_amd.optimisation import DeviceBAProblem, SolverOptions
    ctx = _setup(a.lib)
    fn = ctx.lib.me_cam_ts
    fn.argtypes = [ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]
    buf = (ctypes.c_longlong * 8)()
    d = DeviceBAProblem(_ba_problem(a.config), ctx)
    o = SolverOptions.fixed_iterations(10)
    for _ in range(3):
        d.reset()
        d.solve(o)
    ctx.synchronize()
    fn(buf, 1)
    for _ in range(20):
        d.reset()
        d.solve(o)
    ctx.synchronize()
    fn(buf, 0)
    n = max(buf[0], 1)
    print(json.dumps({"executions": buf[0], "slot_loop": round(buf[1] / n), "block_sum27": round(buf[2] / n),
                      "store_arrive": round(buf[3] / n), "times_last": buf[5],
                      "reduce_when_last": round(buf[4] / max(buf[5], 1))}))


def cmd_step_ts(a):
    """pt_step workgroup 0's phases and the finalizing workgroup's tail (a
    -DME_STEP_TS=1 build), s_memtime ticks per launch."""
    from uasl_motion_estimation_amd.optimisation import DeviceBAProblem, SolverOptions
    ctx = _setup(a.lib)
    fn = ctx.lib.me_step_ts
    fn.argtypes = [ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]
    buf = (ctypes.c_longlong * 12)()
    d = DeviceBAProblem(_ba_problem(a.config), ctx)
    o = SolverOptions.fixed_iterations(10)
    for _ in range(3):
        d.reset()
        d.solve(o)
    ctx.synchronize()
    fn(buf, 1)
    for _ in range(20):
        d.reset()
        d.solve(o)
    ctx.synchronize()
    fn(buf, 0)
    n = max(buf[0], 1)
    nf = max(buf[7], 1)
    names = ["issue", "slot_sums", "point_solve", "cand_cost", "blocksum_store"]
    out = {k: round(buf[i + 1] / n) for i, k in enumerate(names)}
    out["launches"] = buf[0]
    out["finalize"] = round(buf[6] / nf)
    out["fin_loads"], out["fin_blocksum"], out["fin_decide"] = (round(buf[k] / nf) for k in (8, 9, 10))
    print(json.dumps(out))


def cmd_schur_stamps(a):
    from uasl_motion_estimation_amd.optimisation import SolverOptions, ba_solve
    ctx = _setup(a.lib)
    ctx.lib.me_debug_read.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]
    for c in a.configs.split(","):
        ba_solve(_ba_problem(c), SolverOptions.fixed_iterations(10), ctx=ctx)
        buf = (ctypes.c_longlong * 16)()
        ctx.lib.me_debug_read(ctx.h, buf, 16)
        calls = max(buf[12], 1)
        print("config", c, "pt_schur wg0 ticks/launch:", {nm: round(buf[i] / calls) for i, nm in
              zip([6, 7, 8, 9, 10], ["loads", "sums+chol", "Y+barrier", "mfma", "tail+stores"])}, "launches", calls,
              flush=True)


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--lib", default=os.environ.get("ME_LIB"))
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("ba_wall")
    p.add_argument("configs", nargs="?", default="3,4,5")
    p = sub.add_parser("klt")
    p.add_argument("--reps", type=int, default=50)
    p.add_argument("--check", type=int, default=1)
    p = sub.add_parser("mi")
    p.add_argument("--pairs", type=int, default=1 << 20)
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--check", type=int, default=1)
    p = sub.add_parser("coop")
    p.add_argument("--reps", type=int, default=20)
    p = sub.add_parser("solve_ts")
    p.add_argument("configs", nargs="?", default="3,5")
    p = sub.add_parser("scale_ts")
    p.add_argument("--front", type=int, default=0)
    p = sub.add_parser("step_ts")
    p.add_argument("--config", default="3")
    p = sub.add_parser("cam_ts")
    p.add_argument("--config", default="3")
    p = sub.add_parser("schur_stamps")
    p.add_argument("configs", nargs="?", default="3,4")
    a = ap.parse_args()
    globals()["cmd_" + a.cmd](a)


if __name__ == "__main__":
    main()
