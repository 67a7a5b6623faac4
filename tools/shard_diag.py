"""Diagnostic: sharded BA summaries vs the single-device solve (config 2)."""
import os, sys, threading
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
import torch  # noqa: F401
import oracle as O
from uasl_motion_estimation_amd import synthetic as S
from uasl_motion_estimation_amd._lib import Context
from uasl_motion_estimation_amd.optimisation import (SolverOptions, ba_solve, ba_solve_sharded, shard_landmarks,
                                                     ThreadAllReduce)
c = S.CONFIGS[2]
bp = S.ba_problem(S.SEED0 + 2, c["n_feats"], c["window"], c["width"], c["height"])
for iters in (4, 6, 8):
    opts = SolverOptions.fixed_iterations(iters)
    ctx = Context(0)
    _, _, s1 = ba_solve(bp.copy(), opts, ctx=ctx)
    r = O.ba_solve(bp, max_num_iterations=iters, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)[2]
    for world in (1, 2):
        ar = ThreadAllReduce(world)
        ctxs = [Context(0) for _ in range(world)]
        res = [None] * world
        def run(k):
            loc, _ = shard_landmarks(bp, k, world)
            res[k] = ba_solve_sharded(loc, ar.callback(k, ctxs[k]), opts, ctx=ctxs[k])[2]
        th = [threading.Thread(target=run, args=(k,)) for k in range(world)]
        [t.start() for t in th]; [t.join() for t in th]
        print(iters, "world", world, "single", s1, "oracle", r, "sharded", res[0], flush=True)
