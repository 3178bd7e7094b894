"""CPU tests of the oracle (test infrastructure): pinned by the reference's own
test assertions, cross-checked against the independent LAPACK restatement, and
reproducing the committed golden vectors bit-for-bit."""

from __future__ import annotations

import glob
import os

import numpy as np
import pytest

from mcp_amd.qp_benchmark import generate_random_parameter
from oracle import ipm_ref

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = sorted(p for p in glob.glob(os.path.join(HERE, "golden", "*.npz")) if not os.path.basename(p).startswith(("sens_", "nl_")))
FIELDS = ("x", "y", "s", "kkt_error", "eps", "outer_iters", "status", "newton_iters", "active_mask")


def _params(d):
    return {k[len("param_"):]: d[k].item() for k in d.files if k.startswith("param_")}


@pytest.mark.parametrize("path", GOLDEN, ids=lambda p: os.path.basename(p)[:-4])
def test_oracle_reproduces_golden(oracle_lib, path):
    d = np.load(path, allow_pickle=False)
    r = oracle_lib.solve_batch(int(d["family"]), int(d["n"]), int(d["m"]), d["theta"],
                               trace_len=d["out_alpha_trace"].shape[1], **_params(d))
    for f in FIELDS + ("alpha_trace",):
        g, e = r[f], d["out_" + f]
        same = (g == e) | (np.isnan(g) & np.isnan(e)) if g.dtype.kind == "f" else (g == e)
        assert np.all(same), f


@pytest.mark.parametrize("ls", ["reduced", "dense", "schur"])
def test_readme_qp_reference_assertions(oracle_lib, ls):
    """test/runtests.jl:30-38 (check_solution) on the README QP (θ = [-0.5, 0.5])."""
    M = np.array([[2.0, 1.0], [1.0, 2.0]]); A = np.eye(2); b = np.ones(2); theta = np.array([-0.5, 0.5])
    th = np.concatenate([M.flatten("F"), A.flatten("F"), b, theta])
    r = oracle_lib.solve_batch(0, 2, 2, th, linear_solver=ls)
    x, y, s = r["x"][0], r["y"][0], r["s"][0]
    G = M @ x - theta - A.T @ y
    H = A @ x - b
    assert np.all(np.abs(G) <= 5e-3)
    assert np.all(H >= 0) and np.all(y >= 0)
    assert np.sum(y * H) <= 5e-3
    assert np.all(s <= 5e-3) and r["kkt_error"][0] <= 5e-3
    assert r["status"][0] == 0
    # analytic solution x* = [1, 1], y* = [3.5, 2.5] (both constraints active)
    np.testing.assert_allclose(x, [1.0, 1.0], atol=1e-3)
    np.testing.assert_allclose(y, [3.5, 2.5], atol=1e-3)
    assert int(r["active_mask"][0, 0]) == 0b11


@pytest.mark.parametrize("ls", ["reduced", "dense"])
def test_game_clamp_reference_assertion(oracle_lib, ls):
    """test/runtests.jl:88-116: primals ≈ clamp(θ_i, −0.5, 0.5) at atol = 10·tol, status solved."""
    from tests.golden.make_golden import game_clamp_theta

    theta = np.array([-1.0, 0.0, 1.0, 1.0])
    r = oracle_lib.solve_batch(1, 4, 8, game_clamp_theta(theta), tol=1e-4, linear_solver=ls)
    np.testing.assert_allclose(r["x"][0], np.clip(theta, -0.5, 0.5), atol=10 * 1e-4)
    assert r["status"][0] == 0


@pytest.mark.parametrize("n,m,sp,B,seed", [(16, 8, 0.0, 24, 1), (32, 16, 0.0, 8, 2), (16, 8, 0.9, 8, 3),
                                           (5, 3, 0.3, 24, 4)])
@pytest.mark.parametrize("ls", ["reduced", "dense", "schur"])
def test_oracle_matches_lapack_restatement(oracle_lib, n, m, sp, B, seed, ls):
    """Independent restatement (numpy + LAPACK getrf on the full system) agrees on
    status / outer / Newton counts and to ≤1e-8 on the iterates."""
    th = generate_random_parameter(np.random.default_rng(seed), n, m, sp, batch=B)
    r = oracle_lib.solve_batch(0, n, m, th, tol=1e-6, linear_solver=ls)
    agree = 0
    for b in range(B):
        ref = ipm_ref.solve(0, th[b], n, m, tol=1e-6)
        ok = (int(r["status"][b]) == (0 if ref.status == "solved" else 1)
              and r["outer_iters"][b] == ref.outer_iters and r["newton_iters"][b] == ref.newton_iters)
        agree += ok
        if ok and ref.status == "solved":
            z = np.concatenate([r["x"][b], r["y"][b], r["s"][b]])
            zr = np.concatenate([ref.x, ref.y, ref.s])
            assert np.max(np.abs(z - zr)) / max(1.0, np.max(np.abs(zr))) <= 1e-8
    assert agree == B  # rounding-level LU differences never flip a count on these sets


def test_linesearch_restatement():
    """fraction_to_the_boundary_linesearch, src/solver.jl:127-138: α ∈ {2^-e}, NaN past min_stepsize."""
    v = np.array([1.0, 2.0])
    assert ipm_ref.fraction_to_the_boundary_linesearch(v, np.array([1.0, 1.0]))[0] == 1.0
    a, e = ipm_ref.fraction_to_the_boundary_linesearch(v, np.array([-1.0, 0.0]))
    assert a == 0.5 and e == 1  # 1 − 1 = 0 < 0.005 → halve once
    a, _ = ipm_ref.fraction_to_the_boundary_linesearch(v, np.array([-1e9, 0.0]))
    assert np.isnan(a)


def test_oracle_param_validation(oracle_lib):
    th = generate_random_parameter(np.random.default_rng(0), 3, 2, 0.0, batch=1)
    for bad in (dict(tol=0.0), dict(decay=1.0), dict(min_stepsize=-1.0), dict(max_inner_iters=0),
                dict(max_inner_iters=1000), dict(linear_solver=7)):
        with pytest.raises(ValueError):
            oracle_lib.solve_batch(0, 3, 2, th, **bad)
    tha = np.zeros((1, 4 * 4 + 2 * 4 * 4 + 4 * 4 + 8))
    r = oracle_lib.solve_batch(1, 4, 4, tha, linear_solver="schur")  # affine SCHUR: ∂H/∂y taken as 0
    assert r["status"].shape == (1,)


def test_oracle_threads_deterministic(oracle_lib):
    th = generate_random_parameter(np.random.default_rng(5), 16, 8, 0.0, batch=64)
    a = oracle_lib.solve_batch(0, 16, 8, th, tol=1e-6, nthreads=1)
    b = oracle_lib.solve_batch(0, 16, 8, th, tol=1e-6, nthreads=4)
    for f in FIELDS:
        np.testing.assert_array_equal(a[f], b[f])
