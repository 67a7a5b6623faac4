"""Long-sequence run of the windowed stereo VO loop (config 5: 1280x720, 2000
features, W = 50 sliding window, 10-iteration BA per keyframe) on one GPU,
frames rendered on the GPU in chunks (synthetic.corridor_frames_torch: the
ring-corridor arc, any length) and handed to the loop device-resident.  The
first --parity-frames keyframes also run, sequentially, on the oracle backend
(tests/pipeline_oracle.py, the checker): events bit-exact, poses 1e-6.
Reports frames/s (loop only and with rendering), per-segment rates, drift
against the ground-truth trajectory and the window sizes.
--loop native (default) runs the C++ loop (me_vo_loop_*, NativeStereoVO); its
parity prefix is a separate native run of the first keyframes with the event
log on.  Usage: tools/long_run.py [--frames 10000] [--config 5] [--loop native|python] [--out FILE]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=10000)
    ap.add_argument("--config", type=int, default=5)
    ap.add_argument("--chunk", type=int, default=100)
    ap.add_argument("--parity-frames", type=int, default=60)
    ap.add_argument("--segment", type=int, default=1000)
    ap.add_argument("--out", default=None)
    ap.add_argument("--trace", type=int, default=0, help="print tracking / drift stats every N keyframes")
    ap.add_argument("--loop", choices=("native", "python"), default="native")
    args = ap.parse_args()
    import torch

    from uasl_motion_estimation_amd import pipeline as PL
    from uasl_motion_estimation_amd import synthetic as S
    from uasl_motion_estimation_amd._lib import default_context

    c, n = args.config, args.frames
    cfg = PL.PipelineConfig.from_config(c)
    seed = S.SEED0 + c
    arc = S.trajectory_arc(max(n, 2))
    truth = [np.concatenate([t, S.R_to_aa_robust(R)]) for (R, t) in arc]
    centres = [-R.T @ t for (R, t) in arc]
    K = S.intrinsics(cfg.width, cfg.height)
    ctx = default_context()
    native = args.loop == "native"
    if native:
        be = None
        vo = PL.NativeStereoVO(cfg, ctx, K, truth[0], truth[1] - truth[0], log_events=False, overlap=True)
    else:
        be = PL.GPUBackend(ctx)
        vo = PL.WindowedStereoVO(cfg, be, K, truth[0], truth[1] - truth[0], log_events=args.parity_frames > 0,
                                 overlap=True)
    host_frames = []  # the parity prefix's images on the host (for the oracle backend)
    t_loop = t_render = 0.0
    seg_t0, seg_f0, segs = time.perf_counter(), 0, []
    t_all = time.perf_counter()
    pending = {}
    for c0 in range(0, n, args.chunk):
        t1 = time.perf_counter()
        _, fr = S.corridor_frames_torch(seed, cfg.width, cfg.height, c0, min(args.chunk, n - c0))
        torch.cuda.synchronize()
        t_render += time.perf_counter() - t1
        t1 = time.perf_counter()
        for k, (L, R, _, _) in enumerate(fr):
            t = c0 + k
            if t < args.parity_frames:
                host_frames.append((L.cpu().numpy(), R.cpu().numpy()))
            if native:
                vo.process(t, L.contiguous(), R.contiguous())  # (the loop keeps the last two keyframes' images)
            else:
                be.frame_images_device(t, L, R)
                pending[t] = (L, R)
                vo.process(t, None, None)
                if t == args.parity_frames:
                    vo.log_events = False  # (the event log of the prefix only: frames < P and their pops)
                for old in [f for f in pending if f < t - 1]:
                    be.release(old)
                    del pending[old]
            if args.trace and t % args.trace == 0 and vo.results:
                r = vo.results[-1]
                e = np.abs(PL.camera_centre(vo.poses[r.t]) - centres[r.t]).max()
                print(f"t={r.t} tracked={r.n_tracked} new={r.n_new} win_pts={r.n_window_pts} "
                      f"ba_cost={r.ba_cost:.4g} err={e:.4f}", flush=True)
            if (t + 1) % args.segment == 0:
                now = time.perf_counter()
                segs.append({"frames": f"{seg_f0}-{t}", "frames_per_s_with_render": round((t + 1 - seg_f0) / (now - seg_t0), 2)})
                seg_t0, seg_f0 = now, t + 1
                print(f"{t + 1} keyframes, {segs[-1]}", flush=True)
        t_loop += time.perf_counter() - t1
    vo.finish()
    wall = time.perf_counter() - t_all
    poses, res, host_s, latest = vo.poses, vo.results, vo.stage_s["host"], vo.latest_id
    if native:
        vo.close()
    else:
        be.close()
    err = np.array([np.abs(PL.camera_centre(poses[t]) - centres[t]).max() for t in range(n)])
    out = {"workload": f"config {c}: {cfg.width}x{cfg.height} stereo, {cfg.n_feats} features, {cfg.window}-keyframe "
                       f"sliding window, {n} keyframes on the ring-corridor arc, 10-iteration BA per keyframe, "
                       f"pipelined loop on one MI355X (front end 4/16 CUs, BA 12/16)",
           "host_loop": "native (me_vo_loop_*, C++)" if native else "python (WindowedStereoVO)",
           "keyframes": n, "frames_per_s": round(n / t_loop, 2), "frames_per_s_with_render": round(n / wall, 2),
           "render_s": round(t_render, 1), "loop_s": round(t_loop, 1),
           "host_ms_per_frame": round(1e3 * host_s / n, 3),
           "segments": segs,
           "drift_m": {"last": round(float(err[-1]), 4), "max": round(float(err.max()), 4),
                       "per_1000_frames_max": [round(float(err[i:i + 1000].max()), 4) for i in range(0, n, 1000)],
                       "path_length_m": round(0.5 * n, 1)},
           "tracked_per_frame": {"min": int(min(r.n_tracked for r in res[2:])),
                                 "mean": round(float(np.mean([r.n_tracked for r in res[2:]])), 1)},
           "window_landmarks": {"mean": round(float(np.mean([r.n_window_pts for r in res[cfg.window:]] or [0])), 1),
                                "max": int(max([r.n_window_pts for r in res] or [0]))},
           "window_observations_max": int(max([r.n_window_obs for r in res] or [0])),
           "tracks_created": int(latest)}
    if args.parity_frames > 0:
        from pipeline_oracle import OracleBackend  # the checker

        P = args.parity_frames
        ov = PL.WindowedStereoVO(cfg, OracleBackend(), K, truth[0], truth[1] - truth[0], log_events=True)
        t1 = time.perf_counter()
        for t in range(P):
            ov.process(t, *host_frames[t])
        ov.finish()
        ct = time.perf_counter() - t1
        if native:  # the prefix again on a native loop with the event log on
            vp = PL.NativeStereoVO(cfg, ctx, K, truth[0], truth[1] - truth[0], log_events=True, overlap=True)
            for t in range(P):
                vp.process(t, *host_frames[t])
            vp.finish()
            gev, gres = vp.events, vp.results
            vp.close()
        else:
            gev, gres = vo.events, res
        # each frame's pose as its own BA left it (later windows refine it again on the GPU run only)
        pose_rel = max(float(np.max(np.abs(gres[t].pose - ov.results[t].pose) / (np.abs(ov.results[t].pose) + 1e-3)))
                       for t in range(P))
        out["parity_prefix"] = {"keyframes": P, "events_bit_exact": gev[:len(ov.events)] == ov.events,
                                "events_compared": len(ov.events),
                                "pose_max_rel_diff": float("%.3g" % pose_rel)}
        out["cpu_baseline_prefix"] = {"frames_per_s": round(P / ct, 3), "cores": 1, "kind": "port",
                                      "sample": f"the first {P} keyframes on the oracle backend, 1 thread; {ct:.1f} s"}
    bad = np.flatnonzero(err > max(1.0, 20 * np.median(err)))
    out["drift_outlier_frames"] = [int(x) for x in bad[:20]]
    if len(bad):
        out["drift_outliers"] = [{"t": int(t), "err": round(float(err[t]), 3),
                                  "ba_iters": res[t].ba_iters, "ba_cost": res[t].ba_cost,
                                  "tracked": res[t].n_tracked} for t in bad[:5]]
    line = json.dumps(out)
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
