"""Host timeline of the pipelined VO loop with the GPU backend: per keyframe,
the average wall time of each stage between the BA result of frame t-1 and
the BA submission of frame t (the loop's critical path), and of the work the
host does beside the BA.  Frames resident before timing (as bench.py).
Usage: tools/pipe_timeline.py [CONFIG] [NFRAMES]"""
import os
import sys
import time
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402

from uasl_motion_estimation_amd import pipeline as PL  # noqa: E402

c = int(sys.argv[1]) if len(sys.argv) > 1 else 3
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
fr, K, p0, v, truth = PL.synthetic_sequence(c, n)
be = PL.GPUBackend()
for t in range(n):
    be.frame_images(t, fr[t].left, fr[t].right)  # resident before timing
vo = PL.WindowedStereoVO(PL.PipelineConfig.from_config(c), be, K, p0, v, overlap=True)
ev = []


def wrap(obj, name):
    fn = getattr(obj, name)

    def w(*a, **k):
        ev.append((name, "b", time.perf_counter()))
        r = fn(*a, **k)
        ev.append((name, "e", time.perf_counter()))
        return r

    setattr(obj, name, w)


for nm in ("klt_submit", "klt_match", "klt_match_new", "match", "ba_submit_window", "scale_submit", "ba_result", "scale_result",
           "window_add", "frame_images", "frame_images_device"):
    wrap(be, nm)
for nm in ("process", "_complete", "_pop"):
    wrap(vo, nm)
warm = 8
span = defaultdict(float)
cnt = 0
for t in range(n):
    ev.clear()
    vo.process(t, fr[t].left, fr[t].right)
    if t < warm:
        continue
    cnt += 1
    t0 = ev[0][2]
    for name, be_, ts in ev:
        span[(name, be_)] += ts - t0
    span[("end", "e")] += ev[-1][2] - t0
print(f"config {c}, {cnt} keyframes: mean offsets from process() start (ms)")
for (name, be_), s in sorted(span.items(), key=lambda kv: kv[1]):
    print(f"  {1e3 * s / cnt:8.3f}  {name}:{be_}")
