"""Per-phase s_memtime stamps of cam_solve (diagnostic path ME_SOLVE_SKIP=256):
load, diag, panel, trailing, backward solve -- ticks per solve, config 3 and 5.
Usage: solve_stamps.py [LIB|default]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402
from uasl_motion_estimation_amd import _lib  # noqa: E402
if len(sys.argv) > 1 and sys.argv[1] != "default":
    _lib.load_library(sys.argv[1])
from uasl_motion_estimation_amd import synthetic as S  # noqa: E402
from uasl_motion_estimation_amd._lib import Context  # noqa: E402
from uasl_motion_estimation_amd.optimisation import SolverOptions, ba_solve  # noqa: E402

ctx = Context(0)
ctx.lib.me_debug_read.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]
for c in (3, 5):
    cfg = S.CONFIGS[c]
    bp = S.ba_problem(S.SEED0 * 7 + c, cfg["n_feats"], cfg["window"], cfg["width"], cfg["height"])
    os.environ["ME_SOLVE_SKIP"] = "256"
    ba_solve(bp.copy(), SolverOptions.fixed_iterations(10), ctx=ctx)
    buf = (ctypes.c_longlong * 16)()
    ctx.lib.me_debug_read(ctx.h, buf, 16)
    calls = max(buf[15], 1)
    ph = {nm: round(buf[i] / calls) for i, nm in zip([0, 1, 2, 3, 5], ["load", "diag", "panel", "trail", "solves"])}
    print(sys.argv[1] if len(sys.argv) > 1 else "default", "config", c, "cam_solve ticks/solve", ph,
          "sum", sum(ph.values()), "calls", calls, flush=True)
    os.environ.pop("ME_SOLVE_SKIP")
