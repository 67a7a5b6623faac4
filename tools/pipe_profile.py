"""cProfile of the pipelined VO loop on the GPU backend (host-side costs).
Usage: tools/pipe_profile.py CONFIG NFRAMES"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]

from uasl_motion_estimation_amd import pipeline as PL  # noqa: E402


def main():
    c, n = int(sys.argv[1]), int(sys.argv[2])
    warm = 6
    fr, K, p0, v, truth = PL.synthetic_sequence(c, n)
    be = PL.GPUBackend()
    for t in range(n):
        be.frame_images(t, fr[t].left, fr[t].right)
    vo = PL.WindowedStereoVO(PL.PipelineConfig.from_config(c), be, K, p0, v, overlap=True)
    for t in range(warm):
        vo.process(t, fr[t].left, fr[t].right)
    vo.finish()
    pr = cProfile.Profile()
    h0, w0 = vo.stage_s["host"], vo.stage_s["wait"]
    t0 = time.perf_counter()
    pr.enable()
    for t in range(warm, n):
        vo.process(t, fr[t].left, fr[t].right)
    vo.finish()
    pr.disable()
    el = time.perf_counter() - t0
    m = n - warm
    print(f"{1e3 * el / m:.3f} ms/frame (profiled), host {1e3 * (vo.stage_s['host'] - h0) / m:.3f}, "
          f"wait {1e3 * (vo.stage_s['wait'] - w0) / m:.3f}")
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)
    be.close()


if __name__ == "__main__":
    main()
