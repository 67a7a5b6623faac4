"""Per-phase s_memtime stamps of the BA camera solve (diagnostic build path, ME_SOLVE_SKIP=256)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from uasl_motion_estimation_amd import synthetic as S
from uasl_motion_estimation_amd._lib import Context
from uasl_motion_estimation_amd.optimisation import SolverOptions, ba_solve

ctx = Context(0)
ctx.lib.me_debug_read.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]
for cfg in (2, 3, 4):
    c = S.CONFIGS[cfg]
    bp = S.ba_problem(7, c["n_feats"], c["window"], c["width"], c["height"])
    os.environ["ME_SOLVE_SKIP"] = "256"
    ba_solve(bp, SolverOptions.fixed_iterations(10), ctx=ctx)
    buf = (ctypes.c_longlong * 16)()
    ctx.lib.me_debug_read(ctx.h, buf, 16)
    calls = max(buf[15], 1)
    names = ["load", "diag", "panel", "trail", "Linv", "solves"]
    os.environ["ME_SOLVE_SKIP"] = "0"
    ctx.timing(True); ctx.timing_reset()
    ba_solve(bp, SolverOptions.fixed_iterations(10), ctx=ctx)
    ns, ms = ctx.timing_read("BA_SOLVE"); ctx.timing(False)
    print(cfg, "solve kernel us", round(1000 * ms / max(ns, 1), 1), "ticks/us", round(sum(buf[:6]) / calls / (1000 * ms / max(ns, 1)), 0))
    print(cfg, "calls", calls, {nm: round(buf[i] / calls / 100.0, 1) for i, nm in enumerate(names)},
          "(us, s_memtime ticks/100 assuming 100 MHz)", flush=True)
