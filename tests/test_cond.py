"""The ill-conditioning flag of the sensitivities: mcpx_cond_batch[_module] (include/mcpx.h), the
Hager–Higham reciprocal 1-norm condition estimate of ∇F_z at the returned iterate — the matrix the
reference's rrule factors with a column-pivoted QR (src/AutoDiff.jl:39), where QR and LU answers can
part at degenerate solutions.

* CPU: the oracle's estimate (oracle/ipm_oracle.c cond_estimate) against numpy's exact cond₁ on the
  sensitivity fixtures, on random QP solutions and on lane-change game solutions: the estimate
  never exceeds ‖∇F_z⁻¹‖₁, so rcond · cond₁ ≥ 1, and it is within a small factor of it; an exactly
  singular ∇F_z gives status 1 and rcond 0.
* GPU: the workgroup kernels' estimate bit-exact against the oracle (QP C3 and KKT 256, affine,
  the lane-change module)."""

from __future__ import annotations

import glob
import os

import numpy as np
import pytest

from mcp_amd import _abi
from mcp_amd.qp_benchmark import generate_random_parameter
from oracle import ipm_ref

HERE = os.path.dirname(os.path.abspath(__file__))


def _cond1(fam, n, m, th, x, y, s):
    _, J = ipm_ref.F_and_jacobian(ipm_ref.unpack(fam, th, n, m), x, y, s, 0.0)
    return np.linalg.cond(J, 1)


def _ratios(fam, n, m, th, x, y, s, rc):
    return np.array([rc[b] * _cond1(fam, n, m, th[b], x[b], y[b], s[b]) for b in range(th.shape[0])])


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(HERE, "golden", "sens_*.npz"))),
                         ids=lambda p: os.path.basename(p))
def test_oracle_estimate_on_sensitivity_fixtures(oracle_lib, path):
    d = np.load(path)
    fam, n, m = int(d["family"]), int(d["n"]), int(d["m"])
    rc, st = oracle_lib.cond_batch(fam, n, m, d["theta"], d["x"], d["y"], d["s"])
    assert not st.any()
    r = _ratios(fam, n, m, d["theta"], d["x"], d["y"], d["s"], rc)
    assert (r >= 1.0 - 1e-9).all() and (r <= 3.0).all(), r


@pytest.mark.parametrize("n,m", [(16, 8), (32, 16), (128, 64)])
def test_oracle_estimate_on_qp_solutions(oracle_lib, n, m):
    B = 32 if n < 64 else 4
    th = generate_random_parameter(np.random.default_rng(n), n, m, 0.0, batch=B)
    sol = oracle_lib.solve_batch(0, n, m, th, tol=1e-6, nthreads=8)
    rc, st = oracle_lib.cond_batch(0, n, m, th, sol["x"], sol["y"], sol["s"], nthreads=8)
    assert not st.any()
    r = _ratios(0, n, m, th, sol["x"], sol["y"], sol["s"], rc)
    assert (r >= 1.0 - 1e-9).all() and (r <= 3.0).all(), (r.min(), r.max())


def test_oracle_singular_is_flagged(oracle_lib):
    """P = 0, m = 0: ∇F_z = 0 — the LU's first pivot is an exact zero."""
    n, m = 3, 0
    th = np.zeros((2, _abi.theta_dim(_abi.FAMILY_AFFINE, n, m)))
    rc, st = oracle_lib.cond_batch(_abi.FAMILY_AFFINE, n, m, th, np.zeros((2, n)), np.zeros((2, 0)), np.zeros((2, 0)))
    assert st.tolist() == [1, 1] and rc.tolist() == [0.0, 0.0]


def test_oracle_estimate_on_lane_change_solutions(oracle_lib):
    """The lane-change game's solutions (T = 2, KKT 140): the estimate against numpy's cond₁ of the
    generated Jacobian, and the share of games the flag marks (cond₁ > 1e12)."""
    from mcp_amd.lane_change import LaneChangeGame

    game = LaneChangeGame(2)
    nl = game.mcp.nl
    th = np.ascontiguousarray(game.mcp.theta_map(game.generate_random_parameter(np.random.default_rng(11), 24)))
    sol = oracle_lib.solve_batch_nl(nl, th, tol=1e-6, nthreads=8)
    rc, st = oracle_lib.cond_batch(0, 0, 0, th, sol["x"], sol["y"], sol["s"], nthreads=8, nl=nl)
    ok = (sol["status"] == 0) & (st == 0)
    assert ok.sum() >= 16
    for b in np.nonzero(ok)[0]:
        J = game.mcp.jacobian_z(sol["x"][b], sol["y"][b], sol["s"][b], θ=th[b])
        c = np.linalg.cond(J, 1)
        assert 1.0 - 1e-6 <= rc[b] * c <= 3.0 or (c > 1e15 and rc[b] * c >= 1.0 - 1e-6), (b, rc[b], c)
    # every solved game sits at cond₁ ≈ 1e15–1e16 (degenerate complementarity): all flagged
    from mcp_amd.batch import ILL_CONDITIONED

    assert (rc[ok] < ILL_CONDITIONED).all()


# ---------------------------------------------------------------- GPU


@pytest.mark.gpu
@pytest.mark.parametrize("fam,n,m,B", [(0, 32, 16, 256), (0, 128, 64, 16), (1, 8, 4, 64)])
def test_gpu_cond_matches_oracle(gpu, oracle_lib, fam, n, m, B):
    from mcp_amd.batch import cond_batch, solve_batch
    from tests.test_affine_schur import perturbed

    th = (generate_random_parameter(np.random.default_rng(n), n, m, 0.0, batch=B) if fam == 0
          else perturbed(n, m, B, seed=4))
    sol = oracle_lib.solve_batch(fam, n, m, th, tol=1e-6, nthreads=8)
    ref, rst = oracle_lib.cond_batch(fam, n, m, th, sol["x"], sol["y"], sol["s"], nthreads=8)
    got, gst = cond_batch(fam, n, m, th, sol["x"], sol["y"], sol["s"])
    np.testing.assert_array_equal(gst, rst)
    assert np.array_equal(got.view(np.int64), ref.view(np.int64)), np.abs(got - ref).max()
    del solve_batch


@pytest.mark.gpu
def test_gpu_cond_lane_change_module(gpu, oracle_lib):
    from mcp_amd.batch import cond_batch
    from mcp_amd.lane_change import LaneChangeGame

    game = LaneChangeGame(2)
    nl = game.mcp.nl
    th = np.ascontiguousarray(game.mcp.theta_map(game.generate_random_parameter(np.random.default_rng(11), 64)))
    sol = oracle_lib.solve_batch_nl(nl, th, tol=1e-6, nthreads=8)
    ref, rst = oracle_lib.cond_batch(0, 0, 0, th, sol["x"], sol["y"], sol["s"], nthreads=8, nl=nl)
    got, gst = cond_batch(_abi.FAMILY_NONLINEAR, nl.n, nl.m, th, sol["x"], sol["y"], sol["s"], module=game.mcp.module())
    np.testing.assert_array_equal(gst, rst)
    assert np.array_equal(got.view(np.int64), ref.view(np.int64)), np.abs(got - ref).max()
