"""Worker of tests/test_distributed.py::test_ba_solve_distributed_world2_on_device0:
one rank of a landmark-sharded BA (ba_solve_distributed -> me_ba_solve_sharded)
over a gloo process group, both ranks on HIP device 0, host-staged exchange.
Usage: dist_ba_worker.py RANK WORLD PORT OUT_DIR ITERS"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rank, world, port, out, iters = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4], int(sys.argv[5])
    import numpy as np
    import torch
    import torch.distributed as dist

    from uasl_motion_estimation_amd import synthetic as S
    from uasl_motion_estimation_amd._lib import Context
    from uasl_motion_estimation_amd.optimisation import SolverOptions, ba_solve_distributed

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    ctx = Context(0)
    c = S.CONFIGS[2]
    bp = S.ba_problem(S.SEED0 + 2, c["n_feats"], c["window"], c["width"], c["height"])
    opts = SolverOptions.fixed_iterations(iters)
    cams, pts, (lo, hi), s = ba_solve_distributed(bp, opts, ctx=ctx, shard=True)
    # the landmark-count gate: config 2 (~5k observations) is below the
    # crossover, so "auto" solves the whole window on every rank, no exchange
    gcams, gpts, grng, gs = ba_solve_distributed(bp, opts, ctx=ctx)
    np.savez(os.path.join(out, f"rank{rank}.npz"), cams=cams, pts=pts, lo=lo, hi=hi, iterations=s["iterations"],
             successful=s["successful_steps"], backend=dist.get_backend(), world=dist.get_world_size(),
             sharded=s["sharded"], gate_sharded=gs["sharded"], gate_cams=gcams, gate_pts=gpts,
             gate_rng=np.array(grng), gate_iterations=gs["iterations"])
    dist.barrier()
    dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
