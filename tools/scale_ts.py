"""Phase split of the persistent scale LM (scale_lm_kernel) on the bench's
config-3 frames at the frame definition (LM, MAX_NB_ITER 10, tolerances off):
workgroup (0, 0)'s track work per phase type, its waits for each phase's
control, and the controlling workgroup's reduce + control time, from a
-DME_SCALE_TS build (tools/build_variant.sh sts -DME_SCALE_TS).  Microseconds
per launch (s_memrealtime, 100 MHz).  Usage: scale_ts.py LIB [front_cus]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402
from uasl_motion_estimation_amd import _lib  # noqa: E402

_lib.load_library(sys.argv[1])
from uasl_motion_estimation_amd import synthetic as S  # noqa: E402
from uasl_motion_estimation_amd._lib import ME_DEVICE, Context, cu_split  # noqa: E402
from uasl_motion_estimation_amd.optimisation import OptimisationParams, ScaleCall  # noqa: E402

front = int(sys.argv[2]) if len(sys.argv) > 2 else 0
ctx = Context(0)
if front:  # the bench's front-end share: front of every 16 CUs, whole XCDs
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    ctx.set_cu_mask(cu_split(ncu, front)[0])
fn = ctx.lib.me_scale_ts
fn.argtypes = [ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]
buf = (ctypes.c_longlong * 16)()
cfg = S.CONFIGS[3]
W, H, N, win = cfg["width"], cfg["height"], cfg["n_feats"], cfg["window"]
seed = S.SEED0 + 3
scene, K, stream = S.stereo_stream(seed, W, H, 3)
sp = S.scale_problem(seed, W, H, N, window=win, w=5, frames=stream[:2], scene=scene)
params = OptimisationParams.fixed_iterations(10)
evals = 0
for rep in range(2):
    fn(buf, 1)
    runs = 3 if rep == 0 else 20
    for _ in range(runs):
        c = ScaleCall(sp, params, ctx=ctx)
        c.run()
        r = c.result()
    evals = r["executed_evals"] * N
    fn(buf, 1)
L = max(buf[1], 1)
us = lambda k: round(buf[k] / L / 100.0, 2)  # noqa: E731
print(f"front_cus {front or 16}/16: launches {buf[1]}, phases/launch {buf[0] / L:.1f} "
      f"(A/D {buf[7] / L:.1f}, B {buf[8] / L:.1f}, C {buf[9] / L:.1f}); executed track evaluations/launch {evals}")
print(f"  wall {us(2)} us/launch: wg0 track work A/D {us(3)} B {us(4)} C {us(5)}; wg0 waits for control {us(6)}; "
      f"control (reduce + decide, controlling wg) {us(10)} over {buf[11] / L:.1f} reductions")
print(f"  A/D controls (per control): acquire {buf[12] / max(buf[7], 1) / 100.0:.2f}, reduce {buf[13] / max(buf[7], 1) / 100.0:.2f}, "
      f"control {buf[14] / max(buf[7], 1) / 100.0:.2f}, publish {buf[15] / max(buf[7], 1) / 100.0:.2f} us")
print(f"  ns per executed track evaluation: {1e3 * buf[2] / L / 100.0 / max(evals, 1):.2f}")
