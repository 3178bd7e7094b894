"""The SCHUR solve of the affine family (∂H/∂y ≡ 0): θ' = [P; Q; R; S; g; h] with the S block
exactly zero (an instance with a nonzero S entry is not solved: MCPX_FAIL_INPUT), S_ij = P_ij + Σ_k (−Q_ik)·(R_kj·D_k⁻¹) formed on the matrix cores (ipm_kernel_impl.hpp,
AFF), the same kernel as the QP family's with R in A's place and −Qᵀ, −h, −g in LDS.

This is the path a reference user's MCP takes through the C ABI: the Julia shim
 hands every traced PrimalDualMCP over as affine θ' (src/mcp.jl:27-52 →
`affine_parameters`), and the QP benchmark's MCP (benchmark/quadratic_program_benchmark.jl:12-32)
arrives as P = M, Q = −Aᵀ, R = A, S = 0, g = −ϕ, h = −b.

* CPU: that embedding is bit-identical to the QP family's SCHUR solve in the oracle (every
  field); a perturbed, non-symmetric coupling (−Q ≠ Rᵀ: the pivoting-LU pass) agrees with the
  REDUCED elimination on solved instances; a nonzero or NaN S entry gives the MCPX_FAIL_INPUT
  record; the Python API defaults to REDUCED for the affine family (its SCHUR instances never
  take the SPD pass: the QP-shaped ones are classified QP) and accepts SCHUR when S ≡ 0.
* GPU: bit-exact against the oracle at C3's shape (the compile-time kernel) and the runtime
  buckets, symmetric and not, with NaN / Inf / huge inputs; and equal to the QP kernel's bits
  on the embedding.
"""

from __future__ import annotations

import numpy as np
import pytest

from mcp_amd import _abi
from mcp_amd.qp_benchmark import affine_embedding, generate_random_parameter

AFF = _abi.FAMILY_AFFINE
TRACE = 256
FIELDS = ("x", "y", "s", "kkt_error", "eps", "outer_iters", "status", "newton_iters", "active_mask",
          "alpha_trace", "fail_reason")


def qp_to_affine(th: np.ndarray, n: int, m: int, s_fill: float = 0.0) -> np.ndarray:
    """mcp_amd.qp_benchmark.affine_embedding, with the S block filled with `s_fill`."""
    out = affine_embedding(th, n, m)
    out[:, n * n + 2 * n * m:n * n + 2 * n * m + m * m] = s_fill
    return out


def perturbed(n, m, B, seed, scale=0.05, sparsity=0.0):
    """A QP embedding whose G-side coupling is perturbed: −Q ≠ Rᵀ, S not symmetric."""
    rng = np.random.default_rng(seed)
    th = qp_to_affine(generate_random_parameter(rng, n, m, sparsity, batch=B), n, m)
    th[:, n * n:n * n + n * m] += scale * rng.standard_normal((B, n * m))
    return th


def _same(a, b):
    return np.array_equal(a, b) or (a.dtype.kind == "f" and np.array_equal(a, b, equal_nan=True))


@pytest.mark.parametrize("n,m,sp", [(32, 16, 0.0), (8, 4, 0.0), (20, 12, 0.5)])
def test_oracle_qp_embedding_is_bit_identical(oracle_lib, n, m, sp):
    th = generate_random_parameter(np.random.default_rng(n + m), n, m, sp, batch=128)
    q = oracle_lib.solve_batch(_abi.FAMILY_QP, n, m, th, tol=1e-6, linear_solver="schur", trace_len=TRACE, nthreads=8)
    a = oracle_lib.solve_batch(AFF, n, m, qp_to_affine(th, n, m), tol=1e-6, linear_solver="schur", trace_len=TRACE,
                               nthreads=8)
    for f in FIELDS:
        assert _same(q[f], a[f]), f


def test_oracle_nonzero_s_block_is_rejected(oracle_lib):
    """SCHUR eliminates y through the diagonal D, exact only for ∂H/∂y ≡ 0: an instance whose
    S block holds any nonzero or NaN entry returns the MCPX_FAIL_INPUT record (status failed,
    kkt NaN, the initial point, outer 1, no Newton step); S = −0.0 is zero."""
    n, m = 8, 4
    th = generate_random_parameter(np.random.default_rng(7), n, m, 0.0, batch=32)
    a = oracle_lib.solve_batch(AFF, n, m, qp_to_affine(th, n, m), linear_solver="schur", trace_len=TRACE)
    z = oracle_lib.solve_batch(AFF, n, m, qp_to_affine(th, n, m, s_fill=-0.0), linear_solver="schur",
                               trace_len=TRACE)
    for f in FIELDS:
        assert _same(a[f], z[f]), f
    th_bad = qp_to_affine(th, n, m)
    s0 = n * n + 2 * n * m
    th_bad[0, s0] = np.nan
    th_bad[1, s0 + m * m - 1] = 1e-300
    th_bad[2, s0:s0 + m * m] = 7.0
    b = oracle_lib.solve_batch(AFF, n, m, th_bad, linear_solver="schur", trace_len=TRACE)
    assert (a["status"][:3] == 0).all()
    np.testing.assert_array_equal(b["status"][:3], 1)
    np.testing.assert_array_equal(b["fail_reason"][:3], _abi.FAIL_INPUT)
    assert np.isnan(b["kkt_error"][:3]).all()
    np.testing.assert_array_equal(b["outer_iters"][:3], 1)
    np.testing.assert_array_equal(b["newton_iters"][:3], 0)
    np.testing.assert_array_equal(b["x"][:3], 0.0)
    np.testing.assert_array_equal(b["y"][:3], 1.0)
    for f in FIELDS:  # the other instances are untouched
        assert _same(a[f][3:], b[f][3:]), f
    # REDUCED reads S: the same θ solves there
    r = oracle_lib.solve_batch(AFF, n, m, th_bad[1:3], linear_solver="reduced")
    assert (r["fail_reason"] & _abi.FAIL_INPUT == 0).all()


@pytest.mark.parametrize("n,m", [(32, 16), (12, 8)])
def test_oracle_nonsymmetric_coupling_matches_reduced(oracle_lib, n, m):
    """−Q ≠ Rᵀ: S is not symmetric, every step takes the pivoting LU of the Schur complement.
    Against the REDUCED elimination of the (n+m) system: solved instances agree in status and
    outer count, iterates within 1e-8 relative."""
    th = perturbed(n, m, 256, seed=n)
    s = oracle_lib.solve_batch(AFF, n, m, th, tol=1e-6, linear_solver="schur", nthreads=8)
    r = oracle_lib.solve_batch(AFF, n, m, th, tol=1e-6, linear_solver="reduced", nthreads=8)
    ok = (s["status"] == 0) & (r["status"] == 0)
    assert ok.mean() > 0.9
    assert np.array_equal(s["status"], r["status"])
    z = lambda d: np.concatenate([d["x"], d["y"], d["s"]], 1)[ok]
    rel = np.abs(z(s) - z(r)).max(1) / np.maximum(1.0, np.abs(z(r)).max(1))
    assert rel.max() <= 1e-8


def _sym_mcp(S_zero: bool):
    """A two-player affine game: player i minimises ½x_i² − θ_i·x_i s.t. x_i + ½·x_j ≥ θ_3
    (the other player's decision enters its constraint, so −Q = I ≠ Rᵀ); with S_zero false the
    second constraint also carries 0.1·y_1 (∂H/∂y ≠ 0)."""
    from mcp_amd.api import PrimalDualMCP

    def G(x, y, θ):
        return np.array([x[0] - θ[0] - y[0], x[1] - θ[1] - y[1]])

    def H(x, y, θ):
        h1 = x[1] + 0.5 * x[0] - θ[2]
        return np.array([x[0] + 0.5 * x[1] - θ[2], h1 if S_zero else h1 + 0.1 * y[0]])

    return PrimalDualMCP(G, H, unconstrained_dimension=2, constrained_dimension=2, parameter_dimension=3)


def test_api_affine_defaults_to_reduced_and_accepts_schur_when_h_does_not_depend_on_y():
    """An affine-family MCP from the front end has −Q ≠ Rᵀ symbolically (else it is classified
    QP), so SCHUR would always run its pivoting-LU pass: the default stays REDUCED, and SCHUR is
    accepted on request when ∂H/∂y ≡ 0."""
    from mcp_amd.api import InteriorPoint, _linear_solver, solve

    mcp = _sym_mcp(True)
    assert mcp.family == AFF and mcp.h_independent_of_y
    assert _linear_solver(mcp, None) == "reduced"
    assert _linear_solver(mcp, "schur") == "schur"
    mcp_s = _sym_mcp(False)
    assert mcp_s.family == AFF and not mcp_s.h_independent_of_y
    assert _linear_solver(mcp_s, None) == "reduced"
    with pytest.raises(ValueError):
        solve(InteriorPoint(), mcp_s, np.zeros(3), linear_solve_algorithm="schur")


# ---------------------------------------------------------------- GPU


@pytest.mark.gpu
@pytest.mark.parametrize("n,m,B", [(32, 16, 2048), (8, 4, 256), (20, 12, 256), (40, 24, 128), (2, 2, 64)])
def test_gpu_affine_schur_parity(gpu, oracle_lib, n, m, B):
    """C3's shape runs the compile-time kernel, the others the runtime buckets (8 … 48):
    the QP embedding (SPD Gauss-Jordan pass) and the perturbed coupling (pivoting-LU pass)."""
    from mcp_amd.batch import solve_batch
    from tests.test_gpu_parity import assert_parity

    th_qp = generate_random_parameter(np.random.default_rng(n * m), n, m, 0.0, batch=B // 2)
    th = np.concatenate([qp_to_affine(th_qp, n, m), perturbed(n, m, B - B // 2, seed=n + 1)])
    got = solve_batch(AFF, n, m, th, tol=1e-6, linear_solver="schur", trace_len=TRACE)
    ref = oracle_lib.solve_batch(AFF, n, m, th, tol=1e-6, linear_solver="schur", trace_len=TRACE, nthreads=8)
    assert_parity(got, ref)
    assert (ref["status"] == 0).mean() > 0.8
    # the embedding: the QP kernel's bits
    q = solve_batch(_abi.FAMILY_QP, n, m, th_qp, tol=1e-6, linear_solver="schur", trace_len=TRACE)
    half = {k: (v[:B // 2] if isinstance(v, np.ndarray) and v.ndim and v.shape[0] == B else v) for k, v in got.items()}
    assert_parity(half, q)


@pytest.mark.gpu
def test_gpu_affine_schur_edge_inputs(gpu, oracle_lib):
    from mcp_amd.batch import solve_batch
    from tests.test_gpu_parity import assert_parity

    n, m = 32, 16
    th = perturbed(n, m, 8, seed=3)
    th[0, 0] = np.nan
    th[1, n * n + 3] = np.inf  # Q
    th[2, :] = 0.0
    th[3, n * n + n * m + 5] = 1e200  # R
    th[4, -1] = -np.inf  # h
    th[5, n * n + 2 * n * m:n * n + 2 * n * m + m * m] = 7.0  # S ≠ 0: MCPX_FAIL_INPUT
    th[7, n * n + 2 * n * m + 3] = np.nan  # likewise
    th[6, -m - 1] = 1e-300  # g
    got = solve_batch(AFF, n, m, th, linear_solver="schur", trace_len=TRACE)
    ref = oracle_lib.solve_batch(AFF, n, m, th, linear_solver="schur", trace_len=TRACE)
    assert_parity(got, ref)
    np.testing.assert_array_equal(got["fail_reason"][[5, 7]], _abi.FAIL_INPUT)
    assert (got["fail_reason"][[1, 2, 3, 4, 6]] & _abi.FAIL_INPUT == 0).all()


@pytest.mark.gpu
def test_gpu_api_game_takes_affine_schur(gpu, oracle_lib):
    """solve() on an affine MCP with ∂H/∂y ≡ 0 runs SCHUR on request with the oracle's bits."""
    from mcp_amd.api import InteriorPoint, solve

    mcp = _sym_mcp(True)
    th = np.random.default_rng(2).standard_normal((64, 3))
    sol = solve(InteriorPoint(), mcp, th, tol=1e-6, linear_solve_algorithm="schur")
    ref = oracle_lib.solve_batch(AFF, 2, 2, mcp.theta_map(th), tol=1e-6, linear_solver="schur")
    np.testing.assert_array_equal(sol.x, ref["x"])
    np.testing.assert_array_equal(sol.y, ref["y"])
    np.testing.assert_array_equal(np.asarray(sol.outer_iters), ref["outer_iters"])
