"""Host-side logic (no GPU): track-ID bookkeeping, rotation helpers, the
reference's option defaults, and the ctypes mirror of the C ABI structs."""
import ctypes
import math
import os
import subprocess

import numpy as np
import pytest

from uasl_motion_estimation_amd import _lib
from uasl_motion_estimation_amd.feature_types import CamPose, WBA_Point
from uasl_motion_estimation_amd.optimisation import OptimisationParams, OptimType, SolverOptions
from uasl_motion_estimation_amd.rotation_utils import PI, Quat, deg2Rad, exp_map_Quat, log_map_Quat

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# --------------------------------------------------- WBA_Point (feature_types.h:121-197)
def test_wba_point_ids_one_counter_per_feature_type():
    WBA_Point.reset_ids()
    m0 = WBA_Point((1.0, 2.0), 0)
    s0 = WBA_Point(((1.0, 2.0), (0.5, 2.0)), 0)
    m1 = WBA_Point((3.0, 4.0), 0)
    s1 = WBA_Point(((3.0, 4.0), (2.5, 4.0)), 3)
    assert (m0.getID(), m1.getID()) == (0, 1)
    assert (s0.getID(), s1.getID()) == (0, 1)
    assert WBA_Point.latest_id("mono") == 2 and WBA_Point.latest_id("stereo") == 2


def test_wba_point_copy_keeps_id_and_assignment_swaps_id_not_count():
    WBA_Point.reset_ids()
    a = WBA_Point((1.0, 1.0), 5, camIDber=1)
    b = WBA_Point((2.0, 2.0), 7, camIDber=2)
    b.addMatch((2.5, 2.0), 8)
    c = a.copy()
    assert c.getID() == a.getID() == 0 and c.getCount() == 1 and c.getCameraID() == 1
    assert WBA_Point.latest_id("mono") == 2  # copies do not draw IDs
    a.assign(b)
    assert a.getID() == 1 and a.getNbFeatures() == 2 and a.getFrameIdx(1) == 8
    assert a.getCount() == 1 and a.getCameraID() == 1  # operator= keeps count and camID


def test_wba_point_contiguity_pop_and_empty_indices():
    p = WBA_Point((0.0, 0.0), 3)
    p.addMatch((1.0, 0.0), 4)
    with pytest.raises(AssertionError):
        p.addMatch((2.0, 0.0), 6)  # feature_types.h:140 asserts contiguous frames
    p.removeLastFeat()  # undo the offending append
    p.pop()
    assert p.getFirstFrameIdx() == 4 and p.getLastFrameIdx() == 4
    p.pop()
    assert not p.isValid()
    assert p.getLastFrameIdx() == 0xFFFFFFFF  # (unsigned)-1 on an empty track (:164)
    assert not p.isTriangulated()
    p.set3DLocation([1.0, 2.0, 3.0, 1.0])
    assert p.isTriangulated()


def test_campose_trmat():
    q = exp_map_Quat([0.0, 0.1, 0.0])
    cp = CamPose(ID=3, orientation=q, position=np.array([1.0, 2.0, 3.0]))
    T = cp.TrMat()
    np.testing.assert_allclose(T[:3, :3] @ T[:3, :3].T, np.eye(3), atol=1e-12)
    np.testing.assert_array_equal(T[:3, 3], [1.0, 2.0, 3.0])


# --------------------------------------------------- rotation_utils.h
def test_reference_pi_constant_is_kept():
    assert PI == 3.14156592  # rotation_utils.h:15 (sic)
    assert deg2Rad(180.0) == PI


def test_exp_log_map_round_trip_and_floor():
    rng = np.random.default_rng(0)
    for _ in range(50):
        v = rng.normal(0, 0.5, 3)
        np.testing.assert_allclose(log_map_Quat(exp_map_Quat(v)), v, atol=1e-12)
    q = exp_map_Quat([0.0, 0.0, 0.0])  # theta floor 1e-10 (rotation_utils.h:192-196)
    assert (q.w, q.x, q.y, q.z) == (1.0, 0.0, 0.0, 0.0)
    R = exp_map_Quat([0.0, 0.0, math.pi / 2]).getR3()
    np.testing.assert_allclose(R @ [1, 0, 0], [0, 1, 0], atol=1e-12)


def test_quat_is_normalised_on_construction():
    q = Quat(2.0, 0.0, 0.0, 0.0)
    assert q.w == 1.0


# --------------------------------------------------- option defaults
def test_optimisation_params_defaults_match_reference():
    p = OptimisationParams()  # optimisation.h:31
    assert p.type == OptimType.LM and p.minim and p.MAX_NB_ITER == 20
    assert (p.v, p.mu, p.abs_tol, p.grad_tol, p.incr_tol, p.rel_tol, p.alpha) == (2.0, 1e-20, 1e-4, 1e-4, 1e-3,
                                                                                  1e-4, 1.0)


def test_solver_options_match_bundle_adjuster_and_ceres_defaults():
    o = SolverOptions()  # BundleAdjuster.h:463-466 + Ceres defaults
    assert o.function_tolerance == 1e-3 and o.gradient_tolerance == 1e-10 and o.parameter_tolerance == 1e-8
    assert o.initial_trust_region_radius == 1e4 and o.min_relative_decrease == 1e-3
    assert o.min_lm_diagonal == 1e-6 and o.max_lm_diagonal == 1e32 and o.max_num_iterations == 50
    f = SolverOptions.fixed_iterations(10)
    assert f.max_num_iterations == 10 and f.function_tolerance == 0.0


# --------------------------------------------------- ctypes mirror == C header layout
_STRUCTS = {"me_scale_state": "ScaleStateC", "me_optim_params": "OptimParamsC", "me_ba_problem": "BAProblemC",
            "me_ba_options": "BAOptionsC", "me_ba_summary": "BASummaryC", "me_klt_params": "KLTParamsC"}


def test_ctypes_struct_layout_matches_header(tmp_path):
    src = tmp_path / "sz.c"
    body = "".join(f'  printf("{k} %zu\\n", sizeof({k}));\n' for k in _STRUCTS)
    src.write_text(f'#include <stdio.h>\n#include "me_hip.h"\nint main(void) {{\n{body}  return 0;\n}}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    sizes = dict(zip(out[0::2], map(int, out[1::2])))
    for cname, pyname in _STRUCTS.items():
        assert sizes[cname] == ctypes.sizeof(getattr(_lib, pyname)), cname


def test_mi_table_index_arithmetic_is_exact():
    """mi.hip mi_c3: (a-1)a(a+1)/6 as trunc(fl32((a*a - 1) * a) * fl32(1/6)),
    and code/20 as (205 code) >> 12, for every value the kernels can see."""
    a = np.arange(1, 256, dtype=np.int64)
    p = (a - 1) * a * (a + 1)
    assert p.max() < 2 ** 24
    af = a.astype(np.float32)
    pf = (af * af - np.float32(1.0)) * af
    assert np.array_equal(pf.astype(np.int64), p)
    q = (pf * np.float32(1.0 / 6.0)).astype(np.uint32).astype(np.int64)
    assert np.array_equal(q, p // 6)
    code = np.arange(400)
    assert np.array_equal((code * 205) >> 12, code // 20)


@pytest.mark.parametrize("front", [2, 4, 6, 8, 10, 3])
@pytest.mark.parametrize("mode", ["xcd", "interleaved"])
def test_cu_split_is_a_disjoint_cover(front, mode):
    """_lib.cu_split: the two contexts' CU sets are disjoint, cover the device
    and give the front end front/16 of it; the XCD mode (CU i on XCD i mod 8)
    never puts both sides on one XCD (odd shares fall back to interleaving)."""
    ncu = 256
    f, b = _lib.cu_split(ncu, front, mode)
    assert not set(f) & set(b) and sorted(f + b) == list(range(ncu))
    assert len(f) == ncu * front // 16
    if mode == "xcd" and front % 2 == 0:
        xf, xb = {i % 8 for i in f}, {i % 8 for i in b}
        assert not xf & xb and len(xf) == front // 2


# --------------------------------------------------- co-residency roster (csrc/roster.hpp)
def test_roster_protocol_host_threads():
    """The roster the cross-workgroup kernels join (scale_lm_kernel, the camera
    solve's workers and fused assemblers), run by tests/cpp/roster_test over
    std atomics with threads as workgroups, some dispatched after the close:
    every unit of every phase runs exactly once, late workgroups run nothing,
    nobody waits for a workgroup that did not join, and with no participant
    the decider does every unit itself."""
    exe = os.path.join(ROOT, "tests", "cpp", "roster_test")
    assert os.path.exists(exe), "build() compiles tests/cpp/roster_test"
    p = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    assert "roster_test: ok" in p.stdout


def test_scale_lm_launch_form_selection():
    """me_scale_persistent (host only): the one persistent scale-LM launch
    while its nb x 2 workgroups take at most half of the co-resident capacity,
    else the per-phase launches; no capacity (occupancy query failed) always
    takes the per-phase launches.  No environment variable enters the choice
    (bench.py no longer sets ME_SCALE_BLOCKS)."""
    lib = _lib.load_library()
    assert lib.me_scale_persistent(125, 2048) == 1  # config 3: 2 000 tracks, 16 per block
    assert lib.me_scale_persistent(256, 1024) == 1  # exactly half
    assert lib.me_scale_persistent(257, 1024) == 0
    assert lib.me_scale_persistent(1000, 2048) == 0  # config 4 size: per-phase launches
    assert lib.me_scale_persistent(1, 0) == 0
    assert lib.me_scale_persistent(1, -1) == 0
    os.environ["ME_SCALE_BLOCKS"] = "1"  # ignored by the library
    try:
        assert lib.me_scale_persistent(125, 2048) == 1
    finally:
        del os.environ["ME_SCALE_BLOCKS"]
    src = open(os.path.join(ROOT, "uasl_motion_estimation_amd", "csrc", "scale.hip")).read()
    assert "ME_SCALE_BLOCKS" not in src and "getenv(\"ME_SCALE" not in src
    assert "ME_SCALE_BLOCKS" not in open(os.path.join(ROOT, "bench.py")).read()

