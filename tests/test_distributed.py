"""Multi-rank BA: landmark shards, one all-reduce of the reduced
camera system per LM iteration.

CPU (gloo, world size 2): the shard partition and the exchange itself —
S and b of the shards, summed by torch.distributed, equal the full system.
GPU: me_ba_solve_sharded on two contexts of one device with a host-side
all-reduce reproduces the single-device solve.
"""
import os
import socket
import threading

import numpy as np
import pytest

from uasl_motion_estimation_amd import synthetic as S
from uasl_motion_estimation_amd.optimisation import shard_landmarks


def _problem():
    return S.ba_problem(20261019, 300, 8, 640, 480)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_partition_covers_every_landmark_once(world):
    bp = _problem()
    seen_pts, seen_obs, sizes = 0, 0, []
    for r in range(world):
        local, (lo, hi) = shard_landmarks(bp, r, world)
        assert lo == seen_pts  # contiguous, in order
        seen_pts = hi
        np.testing.assert_array_equal(local.pts, bp.pts[lo:hi])
        assert local.pt_idx.min(initial=0) >= 0 and local.pt_idx.max(initial=-1) < hi - lo
        np.testing.assert_array_equal(local.cams, bp.cams)
        seen_obs += len(local.obs)
        sizes.append(len(local.obs))
    assert seen_pts == len(bp.pts) and seen_obs == len(bp.obs)
    assert max(sizes) - min(sizes) <= 2 * S.CONFIGS[2]["window"]  # balanced to within a track or two


def test_shard_gate_model():
    """The landmark-count gate (me_ba_shard_worthwhile, host only): the
    windows the bench's crossover model measured -- config 3 (19k
    observations) never shards, config 4 (100k) and the W = 50 VO window
    (134k) shard at 2 ranks; one rank never; a slow exchange closes it."""
    from uasl_motion_estimation_amd._lib import load_library
    from uasl_motion_estimation_amd.optimisation import shard_worthwhile

    lib = load_library()
    assert lib.me_ba_shard_exchange_us(1) == 0.0
    us = [lib.me_ba_shard_exchange_us(w) for w in (2, 4, 8)]
    assert 0 < us[0] < us[1] < us[2]
    for w in (1, 2, 4, 8):
        assert not shard_worthwhile(19012, w)  # config 3
        assert not shard_worthwhile(0, w)
    assert not shard_worthwhile(100010, 1)
    assert shard_worthwhile(100010, 2) and shard_worthwhile(134053, 2)
    assert not shard_worthwhile(100010, 2, xch_us=1000.0)
    # monotone in the observation count at fixed world size and exchange cost
    dec = [shard_worthwhile(n, 4, 25.0) for n in range(0, 400000, 5000)]
    assert dec == sorted(dec) and dec[-1] and not dec[0]
    # the model itself: t(n) - t(n / world) > 2 xch_us, t(n) = max(floor, n * ns / 1000)
    def model(n, w, x):
        t = lambda m: max(40.0, m * 1.0e-3)  # ME_SHARD_FLOOR_US, ME_SHARD_OBS_NS
        return t(n) - t(-(-n // w)) > 2 * x
    for n in (30000, 60000, 90000, 150000, 1000000):
        for w in (2, 4, 8):
            assert shard_worthwhile(n, w, 20.0) == model(n, w, 20.0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_rank(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist

    import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bp = _problem()
    local, _ = shard_landmarks(bp, rank, world)
    Sg, bg, rc = O.ba_reduced_system_unscaled(local)
    t = torch.from_numpy(np.concatenate([Sg.ravel(), bg]))
    dist.all_reduce(t)
    if rank == 0:
        np.save(os.path.join(out_dir, "sum.npy"), t.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_exchange_sums_to_full_reduced_system(tmp_path, oracle):
    import torch.multiprocessing as mp

    mp.spawn(_gloo_rank, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    got = np.load(tmp_path / "sum.npy")
    bp = _problem()
    Sf, bf, rc = oracle.ba_reduced_system_unscaled(bp)
    assert rc == 0
    n = len(bf)
    np.testing.assert_allclose(got[:n * n].reshape(n, n), Sf, rtol=1e-10, atol=1e-10 * np.abs(Sf).max())
    np.testing.assert_allclose(got[n * n:], bf, rtol=1e-10, atol=1e-10 * np.abs(bf).max())


# ------------------------------------------------------------------ GPU
class _HostAllReduce:
    """All-reduce of device buffers between threads (stands in for RCCL)."""

    def __init__(self, world):
        self.world = world
        self.barrier = threading.Barrier(world)
        self.bufs = [None] * world

    def callback(self, rank, ctx):
        def _ar(ptr, n):
            ctx.synchronize()
            a = np.zeros(abs(n))
            ctx.check(ctx.lib.me_memcpy_d2h(ctx.h, a.ctypes.data, ptr, 8 * abs(n)))
            self.bufs[rank] = a
            self.barrier.wait()
            tot = np.max(self.bufs, axis=0) if n < 0 else np.sum(self.bufs, axis=0)
            self.barrier.wait()
            ctx.check(ctx.lib.me_memcpy_h2d(ctx.h, ptr, np.ascontiguousarray(tot).ctypes.data, 8 * abs(n)))
            ctx.synchronize()

        return _ar


@pytest.mark.gpu
@pytest.mark.parametrize("jacobi", [True, False])
def test_gpu_sharded_solve_matches_single_device(ctx, jacobi):
    from uasl_motion_estimation_amd._lib import Context
    from uasl_motion_estimation_amd.optimisation import SolverOptions, ba_solve, ba_solve_sharded

    bp = _problem()
    opts = SolverOptions.fixed_iterations(8)
    opts.jacobi_scaling = jacobi
    ref_c, ref_p, ref_s = ba_solve(bp.copy(), opts, ctx=ctx)
    world = 2
    ar = _HostAllReduce(world)
    ctxs = [Context(0) for _ in range(world)]
    res = [None] * world

    def run(r):
        local, rng = shard_landmarks(bp, r, world)
        res[r] = (ba_solve_sharded(local, ar.callback(r, ctxs[r]), opts, ctx=ctxs[r]), rng)

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    pts = np.zeros_like(ref_p)
    for r in range(world):
        (cams, p, s), (lo, hi) = res[r]
        np.testing.assert_allclose(cams, ref_c, rtol=1e-6, atol=1e-9)
        assert s["iterations"] == ref_s["iterations"]
        pts[lo:hi] = p
    np.testing.assert_allclose(pts, ref_p, rtol=1e-6, atol=1e-9)


@pytest.mark.gpu
def test_ba_solve_distributed_world2_on_device0(tmp_path, oracle):
    """ba_solve_distributed (torch.distributed glue + me_ba_solve_sharded) in
    two processes on device 0 over gloo (host-staged exchange): the gathered
    landmarks and the cameras match the oracle's unsharded solve."""
    import subprocess
    import sys

    iters = 6
    port = str(_free_port())
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dist_ba_worker.py")
    procs = [subprocess.Popen([sys.executable, worker, str(r), "2", port, str(tmp_path), str(iters)],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(2)]
    outs = [p.communicate(timeout=240)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    c = S.CONFIGS[2]
    bp = S.ba_problem(S.SEED0 + 2, c["n_feats"], c["window"], c["width"], c["height"])
    rc, rp, rs = oracle.ba_solve(bp, max_num_iterations=iters, function_tolerance=0.0, gradient_tolerance=0.0,
                                 parameter_tolerance=0.0)
    pts = np.full_like(rp, np.nan)
    for r in range(2):
        d = np.load(tmp_path / f"rank{r}.npz")
        assert str(d["backend"]) == "gloo" and int(d["world"]) == 2
        assert int(d["iterations"]) == rs["iterations"] and int(d["successful"]) == rs["successful_steps"]
        np.testing.assert_allclose(d["cams"], rc, rtol=1e-6, atol=1e-9)
        pts[int(d["lo"]):int(d["hi"])] = d["pts"]
        # gate: below the crossover every rank solved the whole window itself
        assert bool(d["sharded"]) and not bool(d["gate_sharded"])
        assert list(d["gate_rng"]) == [int(d["lo"]), int(d["hi"])] and int(d["gate_iterations"]) == rs["iterations"]
        np.testing.assert_allclose(d["gate_cams"], rc, rtol=1e-6, atol=1e-9)
        np.testing.assert_allclose(d["gate_pts"], rp[int(d["lo"]):int(d["hi"])], rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(pts, rp, rtol=1e-6, atol=1e-9)


# ------------------------------------------------------------------ me_comm (ABI v3)
def _two_ctx_comm_solve(bp, opts, world=2, device=0):
    """Landmark-sharded solve over `world` contexts of one device through
    me_comm_create_callback (threads + host exchange): returns the gathered
    cameras per rank, the assembled points and the summaries."""
    from uasl_motion_estimation_amd._lib import Context
    from uasl_motion_estimation_amd.optimisation import Comm, ThreadAllReduce, ba_solve_comm

    ar = ThreadAllReduce(world)
    ctxs = [Context(device) for _ in range(world)]
    res, errs = [None] * world, []

    def run(r):
        try:
            local, rng = shard_landmarks(bp, r, world)
            comm = Comm.callback(ctxs[r], world, r, ar.callback(r, ctxs[r]))
            res[r] = (ba_solve_comm(local, comm, opts, ctx=ctxs[r]), rng)
            comm.close()
        except Exception as e:  # pragma: no cover
            errs.append(e)
            ar.barrier.abort()

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    for c in ctxs:
        c.close()
    assert not errs, errs
    pts = np.full_like(np.asarray(bp.pts, np.float64), np.nan)
    cams, summ = [], []
    for r in range(world):
        (c, p, s), (lo, hi) = res[r]
        cams.append(c)
        summ.append(s)
        pts[lo:hi] = p
    return cams, pts, summ


@pytest.mark.gpu
@pytest.mark.parametrize("jacobi", [True, False])
def test_gpu_comm_sharded_solve_matches_single_device(ctx, jacobi):
    """me_ba_solve_comm over a 2-rank callback communicator (packed exchange:
    one all-reduce after the Schur pass, one after the step) = the unsharded
    device solve."""
    from uasl_motion_estimation_amd.optimisation import SolverOptions, ba_solve

    bp = _problem()
    opts = SolverOptions.fixed_iterations(8)
    opts.jacobi_scaling = jacobi
    ref_c, ref_p, ref_s = ba_solve(bp.copy(), opts, ctx=ctx)
    cams, pts, summ = _two_ctx_comm_solve(bp, opts)
    for c, s in zip(cams, summ):
        np.testing.assert_allclose(c, ref_c, rtol=1e-6, atol=1e-9)
        assert (s["iterations"], s["successful_steps"]) == (ref_s["iterations"], ref_s["successful_steps"])
        assert s["final_cost"] == pytest.approx(ref_s["final_cost"], rel=1e-9)
    np.testing.assert_allclose(pts, ref_p, rtol=1e-6, atol=1e-9)


@pytest.mark.gpu
def test_gpu_comm_sharded_config4_8000x30_matches_single_and_oracle(ctx, oracle):
    """Config 4 (8000 landmarks x 30 keyframes, 10 fixed LM iterations),
    landmark-sharded over 2 contexts of one GPU: same iterations and
    successful steps as the unsharded device solve and the oracle, cameras
    and points within 1e-6 of both."""
    from uasl_motion_estimation_amd.optimisation import SolverOptions, ba_solve

    c = S.CONFIGS[4]
    bp = S.ba_problem(S.SEED0 + 4, c["n_feats"], c["window"], c["width"], c["height"])
    assert len(bp.pts) == 8000 and len(bp.cams) == 30
    opts = SolverOptions.fixed_iterations(10)
    ref_c, ref_p, ref_s = ba_solve(bp.copy(), opts, ctx=ctx)
    oc, op, os_ = oracle.ba_solve(bp, max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0,
                                  parameter_tolerance=0.0)
    cams, pts, summ = _two_ctx_comm_solve(bp, opts)
    for cm, s in zip(cams, summ):
        for rc, rs in ((ref_c, ref_s), (oc, os_)):
            np.testing.assert_allclose(cm, rc, rtol=1e-6, atol=1e-9)
            assert (s["iterations"], s["successful_steps"]) == (rs["iterations"], rs["successful_steps"])
    np.testing.assert_allclose(pts, ref_p, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(pts, op, rtol=1e-6, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,iters", [(3, 10), (4, 4)])
def test_gpu_rccl_one_rank_bit_identical_to_single_device(ctx, cfg, iters):
    """Native RCCL communicator at one rank (me_comm_create_rccl): the packed
    exchange reduces in the single-device order, so the sharded solve equals
    me_ba_solve bit for bit."""
    from uasl_motion_estimation_amd.optimisation import Comm, SolverOptions, ba_solve, ba_solve_comm

    c = S.CONFIGS[cfg]
    bp = S.ba_problem(S.SEED0 + cfg, c["n_feats"], c["window"], c["width"], c["height"])
    opts = SolverOptions.fixed_iterations(iters)
    ref_c, ref_p, ref_s = ba_solve(bp.copy(), opts, ctx=ctx)
    comm = Comm.rccl(ctx, 1, 0, Comm.unique_id())
    try:
        assert comm.info() == {"world": 1, "rank": 0, "native": True}
        cams, pts, s = ba_solve_comm(bp.copy(), comm, opts, ctx=ctx)
    finally:
        comm.close()
    assert np.array_equal(cams, ref_c) and np.array_equal(pts, ref_p)
    assert (s["iterations"], s["successful_steps"], s["final_cost"]) == \
        (ref_s["iterations"], ref_s["successful_steps"], ref_s["final_cost"])


@pytest.mark.gpu
def test_gpu_comm_allreduce_native_and_callback(ctx):
    from uasl_motion_estimation_amd.optimisation import Comm

    x = np.arange(1, 1001, dtype=np.float64) * 0.5
    d = ctx.malloc(x.nbytes)
    try:
        ctx.h2d(d, x)
        comm = Comm.rccl(ctx, 1, 0, Comm.unique_id())
        comm.allreduce(d, len(x))
        comm.allreduce(d, len(x), "max")
        comm.close()
        y = np.zeros_like(x)
        ctx.d2h(y, d)
        assert np.array_equal(x, y)  # one rank: identity
        seen = []
        cb = Comm.callback(ctx, 3, 1, lambda ptr, n: seen.append((ptr, n)))
        # creation calibrates: (3 untimed + 10 timed) sums of each exchange size, then one max of the two costs
        sizes = [n for _, n in seen]
        assert sizes == [17000] * 13 + [5] * 13 + [-2], sizes
        assert cb.exchange_us()["system"] > 0 and cb.exchange_us()["scalars"] > 0
        seen.clear()
        cb.allreduce(d, 7)
        cb.allreduce(d, 5, "max")
        assert seen == [(d, 7), (d, -5)] and cb.info() == {"world": 3, "rank": 1, "native": False}
        cb.close()
    finally:
        ctx.free(d)


@pytest.mark.gpu
def test_gpu_comm_calibration_feeds_the_gate():
    """two ranks (two contexts of one GPU, threads, a
    host-staged exchange) create their communicators concurrently; each
    measures its exchanges at creation and takes the max over the ranks, so
    both hold the same costs, and me_ba_shard_worthwhile_comm decides with
    them (equal to the host gate at their mean) -- the same on both ranks."""
    import threading

    from uasl_motion_estimation_amd._lib import Context
    from uasl_motion_estimation_amd.optimisation import Comm, ThreadAllReduce, shard_worthwhile

    world = 2
    ar = ThreadAllReduce(world)
    ctxs = [Context(0) for _ in range(world)]
    comms, errs = [None] * world, []

    def mk(r):
        try:
            comms[r] = Comm.callback(ctxs[r], world, r, ar.callback(r, ctxs[r]))
        except Exception as e:  # pragma: no cover
            errs.append(e)
            ar.barrier.abort()

    th = [threading.Thread(target=mk, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    try:
        assert not errs, errs
        cal = [c.exchange_us() for c in comms]
        assert cal[0] == cal[1] and cal[0]["system"] > 0 and cal[0]["scalars"] > 0
        x = 0.5 * (cal[0]["system"] + cal[0]["scalars"])
        for n in (19012, 100010, 134053, 10 ** 6, 10 ** 8):
            want = shard_worthwhile(n, world, x)
            assert comms[0].shard_worthwhile(n) == comms[1].shard_worthwhile(n) == want, n
        assert comms[0].shard_worthwhile(10 ** 8)  # a window big enough always pays
    finally:
        for c in comms:
            if c is not None:
                c.close()
        for c in ctxs:
            c.close()


@pytest.mark.gpu
def test_gpu_sharded_infeasible_shard_fails_every_rank(ctx):
    """A starting point outside the box bounds in ONE shard: every rank ends
    the solve as FAILURE (the input flags ride in the first exchange), none
    waits for an exchange the other skipped."""
    from uasl_motion_estimation_amd.optimisation import SolverOptions

    bp = _problem()
    bp.pts = np.array(bp.pts, np.float64, copy=True)
    bp.pts[-1, 2] = -5.0  # behind the camera: Z < Zmin, in the last rank's range
    cams, pts, summ = _two_ctx_comm_solve(bp, SolverOptions.fixed_iterations(4))
    for s in summ:
        assert s["status"] == 3 and s["iterations"] == 0


_C4 = {}


def _config4_refs(ctx, oracle):
    """Config 4 window, its unsharded device solve and the oracle's (10 fixed
    LM iterations), computed once for the N-rank tests."""
    if not _C4:
        from uasl_motion_estimation_amd.optimisation import SolverOptions, ba_solve

        c = S.CONFIGS[4]
        bp = S.ba_problem(S.SEED0 + 4, c["n_feats"], c["window"], c["width"], c["height"])
        opts = SolverOptions.fixed_iterations(10)
        _C4["bp"], _C4["opts"] = bp, opts
        _C4["dev"] = ba_solve(bp.copy(), opts, ctx=ctx)
        _C4["oracle"] = oracle.ba_solve(bp, max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0,
                                        parameter_tolerance=0.0)
    return _C4


@pytest.mark.gpu
@pytest.mark.parametrize("world", [4, 8])
def test_gpu_comm_sharded_config4_n_ranks(ctx, oracle, world):
    """Config 4 (8000 x 30, 10 LM iterations) landmark-sharded over 4 and 8
    contexts of one GPU (me_comm_create_callback, thread exchange): the
    packed exchange's per-rank gradient slots and the partition edges at 4
    and 8 ranks give the unsharded solve's iterations and successful steps,
    cameras and points within 1e-6 of it and of the oracle."""
    r = _config4_refs(ctx, oracle)
    ref_c, ref_p, ref_s = r["dev"]
    oc, op, os_ = r["oracle"]
    cams, pts, summ = _two_ctx_comm_solve(r["bp"], r["opts"], world=world)
    assert not np.isnan(pts).any()  # every landmark is in exactly one shard
    for cm, s in zip(cams, summ):
        assert np.array_equal(cm, cams[0])  # the redundant camera solve is identical on every rank
        for rc, rs in ((ref_c, ref_s), (oc, os_)):
            np.testing.assert_allclose(cm, rc, rtol=1e-6, atol=1e-9)
            assert (s["iterations"], s["successful_steps"]) == (rs["iterations"], rs["successful_steps"])
    np.testing.assert_allclose(pts, ref_p, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(pts, op, rtol=1e-6, atol=1e-9)


@pytest.mark.gpu
def test_gpu_sharded_handoff_timeout_on_one_rank_fails_every_rank(ctx):
    """a camera-solve hand-off that times out on ONE rank of a
    sharded solve (forced through the test hook me_debug_solve_flags(512):
    the fused-assembly wait gives up at once) must not leave the other rank
    waiting in a collective: both ranks return ME_ERR_STATE, neither hangs."""
    import ctypes

    from uasl_motion_estimation_amd._lib import Context, MEError
    from uasl_motion_estimation_amd.optimisation import Comm, SolverOptions, ThreadAllReduce, ba_solve_comm

    bp = _problem()
    world = 2
    ar = ThreadAllReduce(world)
    ctxs = [Context(0) for _ in range(world)]
    hook = ctxs[1].lib.me_debug_solve_flags
    hook.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert hook(ctxs[1].h, 512) == 0
    out = [None] * world

    def run(r):
        local, _ = shard_landmarks(bp, r, world)
        comm = Comm.callback(ctxs[r], world, r, ar.callback(r, ctxs[r]))
        try:
            ba_solve_comm(local, comm, SolverOptions.fixed_iterations(6), ctx=ctxs[r])
            out[r] = "ok"
        except MEError as e:
            out[r] = e.code
        finally:
            comm.close()

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    alive = [t.is_alive() for t in th]
    hook(ctxs[1].h, 0)
    if not any(alive):
        for c in ctxs:
            c.close()
    assert not any(alive), "a rank is stuck in the exchange"
    ME_ERR_STATE = -5
    assert out == [ME_ERR_STATE, ME_ERR_STATE], out


@pytest.mark.gpu
def test_bench_world2_gloo_sharded_branch(tmp_path):
    """bench.py's N-rank sharded-BA branch (sharded_ba_line, `dist is not None`) at world size 2 --
    both ranks on GPU 0 over gloo (--comm gloo --rank-device zero: the exchange host-staged through
    me_comm_create_callback) -- so its first N-rank run is not the driver's 8-GPU one: the bench
    line completes and the shards' solve equals the single-GPU solve (its parity field)."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"), "--gpus", "2", "--comm",
           "gloo", "--rank-device", "zero", "--steps", "2", "--warmup", "1", "--frames", "1", "--no-pipeline",
           "--pipeline-frames", "0", "--mi-pairs", "0", "--vo-matches", "0", "--sharded-reps", "1",
           "--profile-steps", "1", "--no-cpu-baseline"]
    r = subprocess.run(cmd, env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["value"] > 0
    sb = line["sharded_ba"]
    assert "error" not in sb, sb
    assert sb["ranks"] == 2 and "gloo" in sb["mode"], sb
    assert sb["parity_vs_single_gpu"]["ok"], sb["parity_vs_single_gpu"]
    assert set(sb["exchange_us"]) == {"17000", "5"}
    # the gate reads the communicator's own calibration
    gi = sb["gate_inputs"]
    cal = gi["calibrated_exchange_us"]
    assert cal["system"] > 0 and cal["scalars"] > 0
    # (both sides rounded to 0.01 us: compare within one rounding step)
    assert abs(gi["per_exchange_us"] - 0.5 * (cal["system"] + cal["scalars"])) <= 0.011
    from uasl_motion_estimation_amd.optimisation import shard_worthwhile
    assert sb["gate_would_shard"] == shard_worthwhile(100010, 2, 0.5 * (cal["system"] + cal["scalars"]))
