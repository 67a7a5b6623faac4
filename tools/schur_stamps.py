"""Per-phase s_memtime stamps of pt_schur_kernel workgroup 0 (diagnostic path, ME_SOLVE_SKIP=256)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from uasl_motion_estimation_amd import synthetic as S  # noqa: E402
from uasl_motion_estimation_amd._lib import Context  # noqa: E402
from uasl_motion_estimation_amd.optimisation import SolverOptions, ba_solve  # noqa: E402

ctx = Context(0)
ctx.lib.me_debug_read.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]
c = S.CONFIGS[3]
bp = S.ba_problem(7, c["n_feats"], c["window"], c["width"], c["height"])
os.environ["ME_SOLVE_SKIP"] = "256"
ba_solve(bp, SolverOptions.fixed_iterations(10), ctx=ctx)
buf = (ctypes.c_longlong * 16)()
ctx.lib.me_debug_read(ctx.h, buf, 16)
calls = max(buf[12], 1)
print("pt_schur wg0 ticks/call:", {nm: round(buf[i] / calls) for i, nm in
                                  zip([6, 7, 13, 14, 8, 9, 10, 11], ["zero", "loads", "gsum", "chol", "Y", "sync", "mfma", "tail"])}, "calls", calls)
