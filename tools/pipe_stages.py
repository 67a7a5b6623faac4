"""Per-stage time of the windowed VO loop (pipeline.WindowedStereoVO): wall
time inside each backend call vs the host bookkeeping around them.
Usage: tools/pipe_stages.py CONFIG NFRAMES [oracle|gpu]"""
import os
import sys
import time
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from uasl_motion_estimation_amd import pipeline as PL  # noqa: E402


def wrap(be, acc):
    for name in ("klt", "mi_scores", "scale_optimise", "ba_solve", "frame_images", "klt_match", "match",
                 "ba_window", "ba_wait", "scale_async", "scale_wait"):
        fn = getattr(be, name, None)
        if fn is None:
            continue

        def timed(*a, _fn=fn, _n=name, **k):
            t0 = time.perf_counter()
            r = _fn(*a, **k)
            acc[_n] += time.perf_counter() - t0
            return r

        setattr(be, name, timed)


def main():
    c, n = int(sys.argv[1]), int(sys.argv[2])
    kind = sys.argv[3] if len(sys.argv) > 3 else "oracle"
    fr, K, p0, v, truth = PL.synthetic_sequence(c, n)
    if kind == "gpu":
        be = PL.GPUBackend()
    else:
        from pipeline_oracle import OracleBackend
        be = OracleBackend()
    for t in range(n):
        be.frame_images(t, fr[t].left, fr[t].right)
    acc = defaultdict(float)
    wrap(be, acc)
    vo = PL.WindowedStereoVO(PL.PipelineConfig.from_config(c), be, K, p0, v)
    warm = min(4, n // 2)
    tot = 0.0
    for t in range(n):
        if t == warm:
            acc.clear()
            tot = 0.0
        t0 = time.perf_counter()
        vo.process(t, fr[t].left, fr[t].right)
        tot += time.perf_counter() - t0
    m = n - warm
    calls = sum(acc.values())
    print(f"config {c}, {m} keyframes timed: {1e3 * tot / m:.3f} ms/keyframe, backend calls {1e3 * calls / m:.3f}, "
          f"host bookkeeping {1e3 * (tot - calls) / m:.3f}")
    for k, s in sorted(acc.items(), key=lambda kv: -kv[1]):
        print(f"  {k:16s} {1e3 * s / m:8.3f} ms/keyframe")
    r = vo.results[-1]
    print("last:", r.n_tracked, r.n_new, r.n_window_pts, r.n_window_obs)


if __name__ == "__main__":
    main()
