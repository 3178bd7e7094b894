"""Workgroup-per-instance kernels (csrc/ipm_wg_impl.hpp): blocked LU with partial
pivoting and MFMA trailing updates for KKT systems beyond one wave's 64 rows
(SURVEY.md §8(f) #2).  Bar as everywhere: every output bit-identical to the
oracle (oracle/ipm_oracle.c, same linear solver), at N ∈ {128, 256, 700}, on
the lane-change game at T = 10 (KKT dimension 700, the reference's
benchmark/trajectory_game_benchmark.jl:38 horizon), and — forced onto the
workgroup kernels with mcpx_params.kernel — on the small cases the one-wave
kernels also cover."""

from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

from mcp_amd import _abi
from mcp_amd.qp_benchmark import generate_random_parameter

FP = ("x", "y", "s", "kkt_error", "eps")
INT = ("outer_iters", "status", "newton_iters")
TRACE = 1024


def assert_bit_exact(got, ref):
    for k in INT:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    if got.get("fail_reason") is not None and ref.get("fail_reason") is not None:
        np.testing.assert_array_equal(np.asarray(got["fail_reason"]), ref["fail_reason"], err_msg="fail_reason")
    if got.get("active_mask") is not None:
        np.testing.assert_array_equal(got["active_mask"], ref["active_mask"], err_msg="active_mask")
    if got.get("alpha_trace") is not None and got["alpha_trace"].size:
        np.testing.assert_array_equal(got["alpha_trace"], ref["alpha_trace"], err_msg="alpha_trace")
    for k in FP:
        g, r = np.asarray(got[k]), np.asarray(ref[k])
        same = (g == r) | (np.isnan(g) & np.isnan(r))
        assert same.all(), f"{k}: {int((~same).sum())} of {same.size} entries differ"


# ---------------------------------------------------------------- CPU


def test_lane_change_t10_gets_workgroup_kernels():
    from mcp_amd.lane_change import LaneChangeGame

    nl = LaneChangeGame(10).mcp.nl
    assert (nl.n, nl.m, nl.n + 2 * nl.m) == (200, 250, 700)
    assert not any(nl.solvers().values())  # beyond every one-wave kernel
    assert nl.wg_solvers() == {"schur": True, "reduced": True, "dense": True}
    assert nl.default_solver() == "schur"
    small = LaneChangeGame(2).mcp.nl
    assert small.solvers()["schur"] and all(small.wg_solvers().values())


def _host_call(n, m, family=0, **kw):
    from mcp_amd._lib import lib

    B = 1
    p = _abi.theta_dim(family, n, m)
    theta = np.zeros((B, p))
    outs = [np.empty(B * max(n, m, 1)) for _ in range(5)] + [np.empty(B, np.int32) for _ in range(2)]
    o = _abi.Out(*[a.ctypes.data for a in outs], None, None, None, 0, 0)
    desc = _abi.Desc(family, n, m, 0, B, p)
    prm = _abi.make_params(**kw)
    return lib().mcpx_solve_batch(C.byref(desc), theta.ctypes.data, None, None, None, C.byref(prm), 1, C.byref(o))


def test_kernel_selection_errors_before_any_device_work():
    """Argument checks of the kernel selector run before the device is touched."""
    assert _host_call(4, 2, kernel=7) == _abi.MCPX_EINVAL
    assert _host_call(300, 200, linear_solver="dense", kernel="wave") == _abi.MCPX_EUNSUPPORTED  # N = 700 > 64
    assert _host_call(300, 300, linear_solver="dense") == _abi.MCPX_EUNSUPPORTED  # N = 900 > 768
    assert _host_call(130, 20, linear_solver="schur") == _abi.MCPX_EUNSUPPORTED  # QP schur: n ≤ 128
    assert _host_call(100, 20, family=1, linear_solver="schur") == _abi.MCPX_EUNSUPPORTED  # affine: one wave only


def test_default_params_select_auto():
    from mcp_amd._lib import lib

    p = _abi.Params()
    p.kernel = 5
    p.linear_solver = 9
    lib().mcpx_default_params(C.byref(p))
    assert p.kernel == _abi.KERNEL_AUTO and p.linear_solver == _abi.LINSOLVE_REDUCED


# ---------------------------------------------------------------- GPU


@pytest.mark.gpu
@pytest.mark.parametrize("ls", ["reduced", "dense"])
@pytest.mark.parametrize("n,m,sp,B,seed", [(16, 8, 0.0, 96, 41), (5, 3, 0.3, 300, 42), (16, 8, 0.9, 64, 43),
                                           (7, 0, 0.0, 16, 44)])
def test_forced_workgroup_equals_oracle_small(gpu, oracle_lib, n, m, sp, B, seed, ls):
    """Small systems the one-wave kernels also solve, forced onto the workgroup path:
    same bits as the oracle and as the one-wave kernel (failing sparse instances
    included — up to 931 Newton steps, so the work queue sees ragged instances)."""
    from mcp_amd.batch import solve_batch

    th = generate_random_parameter(np.random.default_rng(seed), n, m, sp, batch=B)
    ref = oracle_lib.solve_batch(0, n, m, th, tol=1e-6, linear_solver=ls, trace_len=TRACE, nthreads=8)
    got = solve_batch(0, n, m, th, tol=1e-6, linear_solver=ls, trace_len=TRACE, kernel="workgroup")
    assert_bit_exact(got, ref)
    wave = solve_batch(0, n, m, th, tol=1e-6, linear_solver=ls, trace_len=TRACE, kernel="wave")
    assert_bit_exact(got, wave)


@pytest.mark.gpu
@pytest.mark.parametrize("n,m,ls,B", [(64, 32, "dense", 16), (64, 32, "reduced", 16), (128, 64, "dense", 6),
                                      (100, 78, "reduced", 6), (128, 64, "reduced", 6), (300, 200, "dense", 2)],
                         ids=["N128-dense", "N128-reduced", "N256-dense", "N256-reduced", "N256-reduced192",
                              "N700-dense"])
def test_large_qp_vs_oracle(gpu, oracle_lib, n, m, ls, B):
    """Dense random QPs beyond one wave (N = n + 2m = 128, 256, 700): the blocked LU
    with MFMA trailing updates against the oracle's unblocked LU, bit for bit."""
    from mcp_amd.batch import solve_batch

    th = generate_random_parameter(np.random.default_rng(n + m), n, m, 0.0, batch=B)
    ref = oracle_lib.solve_batch(0, n, m, th, tol=1e-6, linear_solver=ls, trace_len=TRACE, nthreads=8)
    got = solve_batch(0, n, m, th, tol=1e-6, linear_solver=ls, trace_len=TRACE)
    assert np.all(got["status"] == 0)
    assert_bit_exact(got, ref)


def _indefinite(th, n, m, scale):
    """M ← M − scale·I: symmetric, so the Gauss-Jordan is tried, but S loses positive definiteness
    on some Newton steps (a pivot ≤ 0: the step falls back to the pivoting LU, as the oracle)."""
    th = th.copy()
    idx = np.arange(n) * (n + 1)
    th[:, idx] -= scale
    return th


@pytest.mark.gpu
@pytest.mark.parametrize("n,m,B,case", [(128, 64, 48, "spd"), (100, 37, 32, "spd"), (70, 10, 32, "spd"),
                                        (33, 40, 32, "spd"), (128, 64, 8, "asym"), (60, 20, 16, "indef"),
                                        (128, 64, 8, "sparse"), (100, 150, 16, "spd")])
def test_qp_schur_workgroup_vs_oracle(gpu, oracle_lib, n, m, B, case):
    """The QP family's workgroup SCHUR step (csrc/gj_vr.hpp: the Schur complement on the matrix
    cores, blocked Gauss-Jordan with MFMA trailing updates) beyond the one-wave kernel's
    n + m ≤ 64: bit-exact against the oracle's SCHUR step (solve_one: S with the MFMA K padding,
    gj_spd_solve) — ragged n and m (panels and K-chunks not multiples of 16 / 4), M not symmetric
    (the pivoting LU at every step), M − c·I (pivots ≤ 0 on some steps: the LU fallback), sparse
    QPs (failing instances, 931 Newton steps); n = 100, m = 150 (bucket 512) reads A from θ, its
    n·kGjLda(m) past the LDS copy's capacity."""
    from mcp_amd.batch import solve_batch

    sp = 0.9 if case == "sparse" else 0.0
    th = generate_random_parameter(np.random.default_rng(n * 7 + m), n, m, sp, batch=B)
    if case == "asym":
        th[:, 1] += 1e-3  # M_21 ≠ M_12
    if case == "indef":
        th = _indefinite(th, n, m, 3.0)
    ref = oracle_lib.solve_batch(0, n, m, th, tol=1e-6, linear_solver="schur", trace_len=TRACE, nthreads=8)
    got = solve_batch(0, n, m, th, tol=1e-6, linear_solver="schur", trace_len=TRACE)
    assert_bit_exact(got, ref)
    if case in ("spd", "asym"):
        assert np.all(ref["status"] == 0)


@pytest.mark.gpu
def test_qp_schur_workgroup_forced_equals_one_wave(gpu, oracle_lib):
    """A size the one-wave SCHUR kernel solves (n = 32, m = 16), forced onto the workgroup SCHUR
    kernel: the same bits as the one-wave kernel and the oracle (the two kernels' Gauss-Jordan
    eliminations are the same chains)."""
    from mcp_amd.batch import solve_batch

    n, m, B = 32, 16, 64
    th = generate_random_parameter(np.random.default_rng(9), n, m, 0.0, batch=B)
    ref = oracle_lib.solve_batch(0, n, m, th, tol=1e-6, linear_solver="schur", trace_len=TRACE, nthreads=8)
    got = solve_batch(0, n, m, th, tol=1e-6, linear_solver="schur", trace_len=TRACE, kernel="workgroup")
    assert_bit_exact(got, ref)
    wave = solve_batch(0, n, m, th, tol=1e-6, linear_solver="schur", trace_len=TRACE, kernel="wave")
    assert_bit_exact(got, wave)


@pytest.mark.gpu
@pytest.mark.parametrize("ls", ["reduced", "dense"])
def test_large_affine_warm_start_vs_oracle(gpu, oracle_lib, ls):
    """Affine family (G = P x + Q y + g, H = R x + S y + h) at n = 60, m = 40 (N = 140),
    warm-started, against the oracle."""
    from mcp_amd.batch import solve_batch

    n, m, B = 60, 40, 8
    rng = np.random.default_rng(5)
    P = rng.standard_normal((B, n, n))
    P = np.einsum("bki,bkj->bij", P, P) + np.eye(n)
    Q = rng.standard_normal((B, n, m))
    R = -Q.transpose(0, 2, 1)
    S = 0.1 * np.eye(m)[None].repeat(B, 0)
    g, h = rng.standard_normal((B, n)), rng.standard_normal((B, m))
    th = np.concatenate([P.transpose(0, 2, 1).reshape(B, -1), Q.transpose(0, 2, 1).reshape(B, -1),
                         R.transpose(0, 2, 1).reshape(B, -1), S.transpose(0, 2, 1).reshape(B, -1), g, h], 1)
    x0, y0 = 0.1 * rng.standard_normal((B, n)), rng.uniform(0.5, 2.0, (B, m))
    ref = oracle_lib.solve_batch(1, n, m, th, x0=x0, y0=y0, tol=1e-6, linear_solver=ls, trace_len=TRACE, nthreads=8)
    got = solve_batch(1, n, m, th, x0=x0, y0=y0, tol=1e-6, linear_solver=ls, trace_len=TRACE)
    assert_bit_exact(got, ref)


@pytest.mark.gpu
def test_large_edge_inputs(gpu, oracle_lib):
    """NaN θ, a zero row (singular Newton system) and a well-posed instance in one
    workgroup-path batch (N = 132)."""
    from mcp_amd.batch import solve_batch

    n, m = 66, 33
    th = generate_random_parameter(np.random.default_rng(9), n, m, 0.0, batch=3)
    th[0, 5] = np.nan
    th[1, : n * n] = 0.0  # M = 0 and …
    th[1, n * n: n * n + n * m] = 0.0  # … A = 0: the Newton matrix has zero rows up to tol·I
    for ls in ("reduced", "dense"):
        ref = oracle_lib.solve_batch(0, n, m, th, tol=1e-6, linear_solver=ls, trace_len=TRACE)
        got = solve_batch(0, n, m, th, tol=1e-6, linear_solver=ls, trace_len=TRACE)
        assert_bit_exact(got, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("ls", ["schur", "reduced", "dense"])
def test_lane_change_t2_forced_workgroup(gpu, oracle_lib, ls):
    """BASELINE C4's game (T = 2, KKT 140) through the module's workgroup kernels."""
    from mcp_amd.batch import solve_batch
    from mcp_amd.lane_change import LaneChangeGame

    game = LaneChangeGame(2)
    mcp = game.mcp
    th = game.generate_random_parameter(np.random.default_rng(11), 48)
    tp, x0 = mcp.theta_map(th), game.initial_guess(th)
    # the oracle follows the kernel: SCHUR solves S by LU on the workgroup kernels (by Gauss-Jordan
    # on the one-wave ones, oracle lu_solve_x rcp = 2)
    ref = oracle_lib.solve_batch_nl(mcp.nl, tp, x0=x0, linear_solver=ls, trace_len=TRACE, nthreads=8,
                                    kernel="workgroup")
    got = solve_batch(_abi.FAMILY_NONLINEAR, mcp.nl.n, mcp.nl.m, tp, x0=x0, linear_solver=ls, trace_len=TRACE,
                      kernel="workgroup", module=mcp.module())
    assert_bit_exact(got, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("ls,B", [("schur", 8), ("reduced", 1), ("dense", 1)])
def test_lane_change_t10_vs_oracle(gpu, oracle_lib, ls, B):
    """The reference's trajectory-benchmark horizon T = 10 (n = 200, m = 250, KKT 700):
    beyond every one-wave kernel; SCHUR forms S (200×200) on the matrix cores.
    REDUCED / DENSE (LU of 450 / 700 rows per Newton step) on the example's θ
    (lane_change.jl:58), which the CPU oracle finishes in seconds."""
    from mcp_amd.batch import solve_batch
    from mcp_amd.lane_change import LaneChangeGame

    game = LaneChangeGame(10)
    mcp = game.mcp
    th = (game.generate_random_parameter(np.random.default_rng(12), B) if ls == "schur"
          else game.example_parameters()[None])
    tp, x0 = mcp.theta_map(th), game.initial_guess(th)
    ref = oracle_lib.solve_batch_nl(mcp.nl, tp, x0=x0, linear_solver=ls, trace_len=TRACE, nthreads=8)
    got = solve_batch(_abi.FAMILY_NONLINEAR, mcp.nl.n, mcp.nl.m, tp, x0=x0, linear_solver=ls, trace_len=TRACE,
                      module=mcp.module())
    assert_bit_exact(got, ref)
