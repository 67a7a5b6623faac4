"""Wall-clock phases of cam_solve_kernel (build with -DME_SOLVE_TS:
tools/build_variant.sh ts -DME_SOLVE_TS), config 3 and 5 windows at 10 LM
iterations, standalone (whole GPU) -- microseconds per launch:
lin_finalize, assembly wait, load, factorisation, backward solve, tail; the
last assembler's exit and the first one's entry relative to workgroup 0's
entry; and the core clock implied by s_memtime / s_memrealtime.
Usage: solve_ts.py LIB"""
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
fn = ctx.lib.me_solve_ts
fn.argtypes = [ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]
buf = (ctypes.c_longlong * 24)()
names = {1: "lin_finalize", 2: "asm_wait", 11: "ts_asm_probe", 12: "load_issue", 13: "load_diag_barrier",
         3: "load_rest", 4: "factor", 5: "backward", 6: "tail", 8: "asm_last_exit", 9: "asm_first_entry",
         19: "f_diag0", 16: "f_w0_panel", 17: "f_w0_diag", 18: "f_barrier_wait"}
names5 = {**names, 16: "m2_w0_diag", 17: "m2_count_wait", 18: "m2_panel", 19: "m2_drain_publish"}
for c in (3, 5):
    cfg = S.CONFIGS[c]
    bp = S.ba_problem(S.SEED0 * 7 + c, cfg["n_feats"], cfg["window"], cfg["width"], cfg["height"])
    for _ in range(3):
        ba_solve(bp.copy(), SolverOptions.fixed_iterations(10), ctx=ctx)
    fn(buf, 1)
    for _ in range(20):
        ba_solve(bp.copy(), SolverOptions.fixed_iterations(10), ctx=ctx)
    fn(buf, 1)
    calls = max(buf[15], 1)
    us = {nm: round(buf[i] / calls / 100.0, 2) for i, nm in (names5 if c == 5 else names).items()}
    tot = sum(buf[i] for i in (1, 2, 3, 4, 5, 6, 11, 12, 13, 16, 17, 18, 19)) / calls / 100.0
    clk = buf[10] / calls / (tot * 1e-6) / 1e9 if tot > 0 else 0.0
    print(f"config {c}: calls {calls} us/launch {us} wg0 total {tot:.2f} us, core clock {clk:.2f} GHz", flush=True)
