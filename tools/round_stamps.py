"""Per-round phase times (s_memtime ticks) of the camera solve's diagonal factor (ME_ROUND_STAMPS build)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401
from uasl_motion_estimation_amd import _lib
_lib.load_library(os.path.join(ROOT, "tools/abl/rst/libme_hip.so"))
from uasl_motion_estimation_amd import synthetic as S
from uasl_motion_estimation_amd._lib import Context
from uasl_motion_estimation_amd.optimisation import DeviceBAProblem, SolverOptions
ctx = Context(0)
L = ctx.lib
L.me_round_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
buf = (ctypes.c_ulonglong * 8)()
for c in (3, 5):
    cfg = S.CONFIGS[c]
    bp = S.ba_problem(S.SEED0 * 7 + c, cfg["n_feats"], cfg["window"], cfg["width"], cfg["height"])
    d = DeviceBAProblem(bp, ctx)
    d.solve(SolverOptions.fixed_iterations(10)); ctx.synchronize()
    L.me_round_stamps(buf, 1)
    ctx.timing_reset(); ctx.timing(True, ["BA_SOLVE"])
    d.reset(); d.solve(SolverOptions.fixed_iterations(10)); ctx.synchronize(); ctx.timing(False)
    n, ms = ctx.timing_read("BA_SOLVE")
    L.me_round_stamps(buf, 1)
    n6 = 6 * (len(bp.cams) - bp.fixed_frames)
    Ts = (n6 + 1 + 15) // 16
    rounds = n * Ts * 4
    names = ["store+barrier", "pivot chain", "inverse+L", "updates"]
    print("config", c, "solves", n, "us/solve", round(1e3 * ms / n, 1), "rounds/solve", Ts * 4,
          {nm: round(buf[k] / rounds, 1) for k, nm in enumerate(names)}, "ticks/round total",
          round(sum(buf[:4]) / rounds, 1), "diag us/solve at 2.1GHz", round(sum(buf[:4]) / n / 2100, 1), flush=True)
