"""Per-phase s_memtime stamps of pt_schur_kernel workgroup 0 (a build with
-DME_SCHUR_STAMPS, e.g. tools/abl/schst/libme_hip.so): ticks per launch.
Usage: schur_stamps.py LIB"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402
from uasl_motion_estimation_amd import _lib  # noqa: E402
_lib.load_library(sys.argv[1])
from uasl_motion_estimation_amd import synthetic as S  # noqa: E402
from uasl_motion_estimation_amd._lib import Context  # noqa: E402
from uasl_motion_estimation_amd.optimisation import SolverOptions, ba_solve  # noqa: E402

ctx = Context(0)
ctx.lib.me_debug_read.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]
for c in (3, 4):
    cfg = S.CONFIGS[c]
    bp = S.ba_problem(S.SEED0 * 7 + c, cfg["n_feats"], cfg["window"], cfg["width"], cfg["height"])
    ba_solve(bp.copy(), SolverOptions.fixed_iterations(10), ctx=ctx)
    buf = (ctypes.c_longlong * 16)()
    ctx.lib.me_debug_read(ctx.h, buf, 16)
    calls = max(buf[12], 1)
    print("config", c, "pt_schur wg0 ticks/launch:", {nm: round(buf[i] / calls) for i, nm in
          zip([6, 7, 8, 9, 10], ["loads", "sums+chol", "Y+barrier", "mfma", "tail+stores"])}, "launches", calls,
          flush=True)
