"""cProfile of the windowed VO loop with the GPU backend (config 3 by default):
where the host time per keyframe goes (Python bookkeeping vs backend calls).
Usage: tools/pipe_hostprof.py [CONFIG] [NFRAMES]"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402

from uasl_motion_estimation_amd import pipeline as PL  # noqa: E402

c = int(sys.argv[1]) if len(sys.argv) > 1 else 3
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
fr, K, p0, v, truth = PL.synthetic_sequence(c, n)
be = PL.GPUBackend()
vo = PL.WindowedStereoVO(PL.PipelineConfig.from_config(c), be, K, p0, v, overlap=True)
for t in range(n):  # images resident before timing (as the bench line)
    be.frame_images(t, fr[t].left, fr[t].right)
warm = 8
for t in range(warm):
    vo.process(t, fr[t].left, fr[t].right)
vo.stage_s = {"host": 0.0, "wait": 0.0}
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
for t in range(warm, n):
    vo.process(t, fr[t].left, fr[t].right)
pr.disable()
vo.finish()
dt = time.perf_counter() - t0
m = n - warm
print(f"config {c}: {1e3 * dt / m:.3f} ms/keyframe, host {1e3 * vo.stage_s['host'] / m:.3f}, "
      f"wait {1e3 * vo.stage_s['wait'] / m:.3f} (profiled)")
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(30)
st.sort_stats("cumtime").print_stats(30)
