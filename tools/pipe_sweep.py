"""Frames/s of the pipelined VO loop (GPU backend) over front-end CU shares
and matcher placement.  Usage: tools/pipe_sweep.py CONFIG NFRAMES"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]

from uasl_motion_estimation_amd import pipeline as PL  # noqa: E402
from uasl_motion_estimation_amd._lib import default_context  # noqa: E402


def run(fr, K, p0, v, c, n, warm, **kw):
    ctx = default_context()
    be = PL.GPUBackend(ctx, **kw)
    for t in range(n):
        be.frame_images(t, fr[t].left, fr[t].right)
    vo = PL.WindowedStereoVO(PL.PipelineConfig.from_config(c), be, K, p0, v, overlap=True)
    for t in range(warm):
        vo.process(t, fr[t].left, fr[t].right)
    vo.finish()
    h0, w0 = vo.stage_s["host"], vo.stage_s["wait"]
    t0 = time.perf_counter()
    for t in range(warm, n):
        vo.process(t, fr[t].left, fr[t].right)
    vo.finish()
    el = time.perf_counter() - t0
    be.close()
    m = n - warm
    return m / el, 1e3 * (vo.stage_s["host"] - h0) / m, 1e3 * (vo.stage_s["wait"] - w0) / m


def main():
    c, n = int(sys.argv[1]), int(sys.argv[2])
    fr, K, p0, v, truth = PL.synthetic_sequence(c, n)
    for kw in (dict(front_cus=8, match_on_ba=False), dict(front_cus=8), dict(front_cus=6), dict(front_cus=4),
               dict(front_cus=8), dict(front_cus=4)):
        fps, host, wait = run(fr, K, p0, v, c, n, 6, **kw)
        print(f"{kw}: {fps:.1f} frames/s, host {host:.3f} ms, wait {wait:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
