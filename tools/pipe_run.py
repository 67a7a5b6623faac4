"""The pipelined VO loop alone (GPU backend, frames resident), for a kernel
trace: tools/pipe_ktrace.py reads rocprofv3 --kernel-trace of this.
Usage: tools/pipe_run.py [CONFIG] [NFRAMES]"""
import os
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
for t in range(n):
    be.frame_images(t, fr[t].left, fr[t].right)
vo = PL.WindowedStereoVO(PL.PipelineConfig.from_config(c), be, K, p0, v, overlap=True)
warm = 8
be.tlog = []
tin = []
for t in range(n):
    if t == warm:
        t0 = time.perf_counter()
    tin.append(time.perf_counter())
    vo.process(t, fr[t].left, fr[t].right)
vo.finish()
dt = time.perf_counter() - t0
print(f"config {c}: {1e3 * dt / (n - warm):.3f} ms/keyframe", flush=True)
# BA(t) enqueued vs BA(t-1) completed: a positive lead means the BA stream never waits for the host
enq = {f: x for k, f, x in be.tlog if k == "enq"}
enq0 = {f: x for k, f, x in be.tlog if k == "enq0"}
fs = [f for f in enq if f >= warm and f in enq0]
if fs:
    print("enqueue: start at %.3f ms into the keyframe, me_vo_window_submit %.3f ms (means)" % (
        1e3 * sum(enq0[f] - tin[f] for f in fs) / len(fs), 1e3 * sum(enq[f] - enq0[f] for f in fs) / len(fs)))
done = [x for k, f, x in be.tlog if k == "done"]
ts = sorted(enq)
for i, f in enumerate(ts[1:], 1):
    if f >= warm and i < len(done):
        print(f"frame {f}: enqueue done at {1e3 * (enq[f] - tin[f]):.3f} ms, BA({ts[i - 1]}) completed at "
              f"{1e3 * (done[i - 1] - tin[f]):.3f} ms, BA({f}) completed {1e3 * (done[i] - done[i - 1]):.3f} ms later")
be.close()
