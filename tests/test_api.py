"""The reference API mirror (mcp_amd.api), tested the way test/runtests.jl tests the
reference: the QP test problem through both callable constructors and the
ParametricGame test.  CPU tests check the tracing/θ-map; GPU tests solve through
the C ABI and compare with the reference's assertions and with the oracle."""

from __future__ import annotations

import numpy as np
import pytest

from mcp_amd import _abi
from mcp_amd.api import (Block, InteriorPoint, NotAffineError, OptimizationProblem, ParametricGame,
                         PrimalDualMCP, ThetaMap, make_variables, mortar, solve)
from tests.golden.make_golden import game_clamp_theta, readme_qp_theta

# test/runtests.jl:8-26
M = np.array([[2, 1], [1, 2]])
A = np.array([[1, 0], [0, 1]])
b = np.array([1, 1])
θ = np.array([-0.5, 0.5])


def G(x, y, θ):
    return M @ x - θ - A.T @ y


def H(x, y, θ):
    return A @ x - b


def K(z, θ):
    x = z[:M.shape[0]]
    y = z[M.shape[0]:]
    return np.concatenate([G(x, y, θ=θ), H(x, y, θ=θ)])


def check_solution(sol):
    """test/runtests.jl:30-38."""
    assert np.all(np.abs(G(sol.x, sol.y, θ)) <= 5e-3)
    assert np.all(H(sol.x, sol.y, θ) >= 0)
    assert np.all(sol.y >= 0)
    assert np.sum(sol.y * H(sol.x, sol.y, θ)) <= 5e-3
    assert np.all(sol.s <= 5e-3)
    assert sol.kkt_error <= 5e-3
    assert sol.status == "solved"


def basic_mcp():
    return PrimalDualMCP(G, H, unconstrained_dimension=M.shape[0], constrained_dimension=len(b),
                         parameter_dimension=M.shape[0])


def alternative_mcp():
    return PrimalDualMCP(K, [-np.inf] * M.shape[0] + [0] * len(b), [np.inf] * (M.shape[0] + len(b)),
                         parameter_dimension=M.shape[0])


LIM = 0.5


def clamp_game():
    """test/runtests.jl:88-107."""
    return ParametricGame(
        test_point=mortar([[1, 1], [1, 1]]),
        test_parameter=mortar([[1, 1], [1, 1]]),
        problems=[
            OptimizationProblem(objective=lambda x, θi: np.sum((x[Block(1)] - θi) ** 2),
                                private_inequality=lambda x, θi: np.concatenate([-x[Block(1)] + LIM,
                                                                                  x[Block(1)] + LIM])),
            OptimizationProblem(objective=lambda x, θi: np.sum((x[Block(2)] - θi) ** 2),
                                private_inequality=lambda x, θi: np.concatenate([-x[Block(2)] + LIM,
                                                                                  x[Block(2)] + LIM])),
        ])


# ---------------------------------------------------------------- CPU: tracing


@pytest.mark.parametrize("ctor", [basic_mcp, alternative_mcp])
def test_qp_test_problem_traces_to_qp_family(ctor):
    mcp = ctor()
    assert (mcp.unconstrained_dimension, mcp.constrained_dimension, mcp.parameter_dimension) == (2, 2, 2)
    assert mcp.family == _abi.FAMILY_QP
    np.testing.assert_array_equal(mcp.theta_map(θ)[0], readme_qp_theta(θ))


def test_game_traces_to_affine_family():
    game = clamp_game()
    assert game.num_players() == 2
    assert game.dims["x"] == [2, 2] and game.dims["μ"] == [4, 4] and game.dims["λ"] == [0, 0]
    mcp = game.mcp
    assert mcp.family == _abi.FAMILY_AFFINE
    assert (mcp.unconstrained_dimension, mcp.constrained_dimension) == (4, 8)
    th = np.array([-1.0, 0.0, 1.0, 1.0])
    np.testing.assert_array_equal(mcp.theta_map(th)[0], game_clamp_theta(th))


def test_benchmark_qp_family_is_an_identity_map():
    """benchmark/quadratic_program_benchmark.jl:12-32 written against θ: the traced map is θ' = θ."""
    n, m = 5, 3

    def Gq(x, y, θ):
        Mq = θ[:n * n].reshape(n, n, order="F")
        Aq = θ[n * n:n * n + m * n].reshape(m, n, order="F")
        return Mq @ x - θ[n * n + m * n + m:] - Aq.T @ y

    def Hq(x, y, θ):
        return θ[n * n:n * n + m * n].reshape(m, n, order="F") @ x - θ[n * n + m * n:n * n + m * n + m]

    mcp = PrimalDualMCP(Gq, Hq, unconstrained_dimension=n, constrained_dimension=m,
                        parameter_dimension=n * n + m * n + m + n)
    assert mcp.family == _abi.FAMILY_QP and mcp.theta_map.identity


def test_symbolic_constructors():
    x, y, t = make_variables("x", 2), make_variables("y", 2), make_variables("θ", 2)
    mcp = PrimalDualMCP.from_symbolic(G(x, y, t), H(x, y, t), x, y, t)
    np.testing.assert_array_equal(mcp.theta_map(θ)[0], readme_qp_theta(θ))
    z = make_variables("z", 4)
    mcp2 = PrimalDualMCP.from_symbolic_K(K(z, t), z, t, [-np.inf, -np.inf, 0, 0], [np.inf] * 4)
    np.testing.assert_array_equal(mcp2.theta_map(θ)[0], readme_qp_theta(θ))


def test_non_affine_goes_to_the_nonlinear_family():
    """G/H that are not affine become generated device code (MCPX_FAMILY_NONLINEAR)."""
    mcp = PrimalDualMCP(lambda x, y, θ: x ** 3 - θ, lambda x, y, θ: x - y, unconstrained_dimension=1,
                        constrained_dimension=1, parameter_dimension=1)
    assert mcp.family == _abi.FAMILY_NONLINEAR and mcp.nl.has_s  # H = x − y depends on y
    assert mcp.nl.default_solver() == "reduced"
    assert issubclass(NotAffineError, NotImplementedError)


def test_bounds_assertion():
    """src/mcp.jl:191: upper bounds Inf, lower bounds −Inf or 0."""
    with pytest.raises(ValueError):
        PrimalDualMCP(K, [-np.inf, -np.inf, 1, 0], [np.inf] * 4, parameter_dimension=2)
    with pytest.raises(ValueError):
        PrimalDualMCP(K, [-np.inf, -np.inf, 0, 0], [np.inf, np.inf, np.inf, 5.0], parameter_dimension=2)


def test_missing_dimensions():
    with pytest.raises(TypeError):
        PrimalDualMCP(G, H, unconstrained_dimension=2, constrained_dimension=2)


def test_affine_family_with_coupled_y_and_theta_products():
    """A non-QP affine MCP (∂H/∂y ≠ 0, θ-scaled coefficients, a nonlinear θ entry):
    blocks, F and ∇F_z agree with direct evaluation; the θ-map VJP matches finite differences."""
    def Ga(x, y, θ):
        return np.array([θ[0] * x[0] + 2 * x[1] - y[0] + θ[1], x[1] - θ[0] * θ[1] * y[1] + 1.5])

    def Ha(x, y, θ):
        return np.array([x[0] + 0.5 * y[1] - θ[2], -x[1] + θ[2] * y[0] + 3])

    mcp = PrimalDualMCP(Ga, Ha, unconstrained_dimension=2, constrained_dimension=2, parameter_dimension=3)
    assert mcp.family == _abi.FAMILY_AFFINE
    th = np.array([0.7, -1.3, 2.1])
    P, Q, R, S, g, h = mcp.blocks(th)
    np.testing.assert_allclose(P, [[0.7, 2], [0, 1]])
    np.testing.assert_allclose(Q, [[-1, 0], [0, 0.7 * 1.3]])
    np.testing.assert_allclose(R, [[1, 0], [0, -1]])
    np.testing.assert_allclose(S, [[0, 0.5], [2.1, 0]])
    np.testing.assert_allclose(g, [-1.3, 1.5])
    np.testing.assert_allclose(h, [-2.1, 3])
    x, y, s = np.array([0.3, -0.2]), np.array([1.1, 0.4]), np.array([0.5, 0.9])
    F = mcp.F(x, y, s, θ=th, ϵ=0.1)
    np.testing.assert_allclose(F[:2], Ga(x, y, th))
    np.testing.assert_allclose(F[2:4], Ha(x, y, th) - s)
    np.testing.assert_allclose(F[4:], s * y - 0.1)
    J = mcp.jacobian_z(x, y, s, θ=th)
    eps = 1e-7
    for j in range(6):
        dz = np.zeros(6)
        dz[j] = eps
        z = np.concatenate([x, y, s]) + dz
        Fp = mcp.F(z[:2], z[2:4], z[4:], θ=th, ϵ=0.1)
        np.testing.assert_allclose((Fp - F) / eps, J[:, j], atol=1e-6)
    # θ-map adjoint vs finite differences
    rng = np.random.default_rng(0)
    gout = rng.standard_normal((1, mcp.theta_map.p_out))
    vj = mcp.theta_map.vjp(th[None], gout)[0]
    for k in range(3):
        d = np.zeros(3)
        d[k] = 1e-6
        fd = (mcp.theta_map(th + d)[0] - mcp.theta_map(th - d)[0]) / 2e-6
        assert abs(fd @ gout[0] - vj[k]) <= 1e-6 * max(1.0, abs(vj[k]))


def test_theta_map_linear_combinations_fixed_order():
    t = make_variables("θ", 3)
    tm = ThetaMap([t[0], -t[1], 2 * t[0] + t[2] - 1.5, 4.0, t[1] * t[2]], list(t))
    th = np.array([[1.0, 2.0, 3.0], [-0.5, 0.25, 8.0]])
    out = tm(th)
    np.testing.assert_array_equal(out[:, 0], th[:, 0])
    np.testing.assert_array_equal(out[:, 1], -th[:, 1])
    np.testing.assert_array_equal(out[:, 2], 2 * th[:, 0] + th[:, 2] - 1.5)
    np.testing.assert_array_equal(out[:, 3], [4.0, 4.0])
    np.testing.assert_array_equal(out[:, 4], th[:, 1] * th[:, 2])


def test_theta_map_torch_matches_numpy():
    torch = pytest.importorskip("torch")
    t = make_variables("θ", 3)
    tm = ThetaMap([t[0], -t[1], 2 * t[0] + t[2] - 1.5, 4.0, t[1] * t[2]], list(t))
    th = np.random.default_rng(1).standard_normal((5, 3))
    np.testing.assert_array_equal(tm(torch.from_numpy(th)).numpy(), tm(th))
    g = np.random.default_rng(2).standard_normal((5, 5))
    np.testing.assert_allclose(tm.vjp(torch.from_numpy(th), torch.from_numpy(g)).numpy(), tm.vjp(th, g))


def test_solve_argument_checks():
    mcp = basic_mcp()
    with pytest.raises(TypeError):
        solve("InteriorPoint", mcp, θ)
    with pytest.raises(ValueError):
        solve(InteriorPoint(), mcp, θ, linear_solve_algorithm="umfpack")
    with pytest.raises(ValueError):
        solve(InteriorPoint(), mcp, np.zeros(3))


def test_solve_without_gpu_fails_loudly():
    from mcp_amd._lib import MCPXError, lib

    if lib().mcpx_device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(MCPXError):
        solve(InteriorPoint(), basic_mcp(), θ)


# ---------------------------------------------------------------- GPU: runtests.jl


@pytest.mark.gpu
def test_basic_callable_constructor(gpu):
    """test/runtests.jl:40-50."""
    check_solution(solve(InteriorPoint(), basic_mcp(), θ))


@pytest.mark.gpu
def test_alternative_callable_constructor(gpu):
    """test/runtests.jl:52-62."""
    check_solution(solve(InteriorPoint(), alternative_mcp(), θ))


@pytest.mark.gpu
@pytest.mark.parametrize("algo", ["reduced", "dense", "schur"])
def test_api_solution_is_the_oracles(gpu, oracle_lib, algo):
    sol = solve(InteriorPoint(), basic_mcp(), θ, linear_solve_algorithm=algo)
    ref = oracle_lib.solve_batch(0, 2, 2, readme_qp_theta(θ), linear_solver=algo)
    np.testing.assert_array_equal(sol.x, ref["x"][0])
    np.testing.assert_array_equal(sol.y, ref["y"][0])
    assert sol.kkt_error == ref["kkt_error"][0] and sol.ϵ == ref["eps"][0]
    assert sol.outer_iters == ref["outer_iters"][0]


@pytest.mark.gpu
def test_parametric_game(gpu):
    """test/runtests.jl:88-116."""
    game = clamp_game()
    th = mortar([[-1, 0], [1, 1]])
    tol = 1e-4
    res = solve(game, th, tol=tol)
    for ii in range(2):
        np.testing.assert_allclose(res.primals[ii], np.clip(th[Block(ii + 1)], -LIM, LIM), atol=10 * tol)
    assert res.status == "solved"


@pytest.mark.gpu
def test_batched_theta_and_warm_start_aliasing(gpu, oracle_lib):
    """A (B, p) θ solves the batch; caller x₀/y₀/s₀ are updated in place (src/solver.jl:64-66)."""
    mcp = basic_mcp()
    rng = np.random.default_rng(3)
    th = rng.standard_normal((64, 2))
    x0 = np.zeros((64, 2))
    y0 = np.ones((64, 2))
    s0 = np.ones((64, 2))
    sol = solve(InteriorPoint(), mcp, th, x0=x0, y0=y0, s0=s0, tol=1e-6)
    assert sol.x is x0 and sol.y is y0 and sol.s is s0
    ref = oracle_lib.solve_batch(0, 2, 2, np.stack([readme_qp_theta(t) for t in th]), tol=1e-6,
                                 linear_solver="schur")
    np.testing.assert_array_equal(x0, ref["x"])
    assert list(sol.status) == ["solved" if s == 0 else "failed" for s in ref["status"]]


@pytest.mark.gpu
def test_device_theta(gpu):
    import torch

    mcp = basic_mcp()
    th = torch.tensor([[-0.5, 0.5], [0.3, 0.1]], dtype=torch.float64, device="cuda")
    sol = solve(InteriorPoint(), mcp, th)
    torch.cuda.synchronize()
    host = solve(InteriorPoint(), mcp, th.cpu().numpy())
    np.testing.assert_array_equal(sol.x.cpu().numpy(), host.x)
    assert sol.status.cpu().tolist() == [0, 0]


# ---------------------------------------------------------------- AutoDiff mirror (src/AutoDiff.jl)


def test_theta_map_jvp_is_the_adjoint_of_vjp():
    t = make_variables("θ", 3)
    tm = ThetaMap([t[0], -t[1], 2 * t[0] + t[2] - 1.5, 4.0, t[1] * t[2]], list(t))
    rng = np.random.default_rng(4)
    th, td, g = rng.standard_normal((5, 3)), rng.standard_normal((5, 2, 3)), rng.standard_normal((5, 5))
    np.testing.assert_allclose(np.einsum("bkp,bp->bk", tm.jvp(th, td), g),
                               np.einsum("bkq,bq->bk", td, tm.vjp(th, g)), rtol=1e-12)


def test_missing_sensitivities_is_an_argument_error():
    """src/AutoDiff.jl:19-23."""
    from mcp_amd.autodiff import rrule

    mcp = PrimalDualMCP(G, H, unconstrained_dimension=2, constrained_dimension=2, parameter_dimension=2,
                        compute_sensitivities=False)
    with pytest.raises(ValueError, match="compute_sensitivities"):
        rrule(solve, InteriorPoint(), mcp, θ)


def _readme_f(sol):
    return float(np.sum(sol.x ** 2) + np.sum(sol.y ** 2))


@pytest.mark.gpu
def test_autodiff_reference_test(gpu):
    """test/runtests.jl:65-85: reverse (rrule) vs forward (Dual) vs finite differences, atol 1e-3."""
    from mcp_amd.autodiff import NoTangent, rrule, solve_dual

    mcp = basic_mcp()
    sol, pullback = rrule(solve, InteriorPoint(), mcp, θ)
    grads = pullback({"x": 2 * sol.x, "y": 2 * sol.y})
    assert grads[:3] == (NoTangent(), NoTangent(), NoTangent())
    g_rev = grads[3]
    h = 1e-6
    g_fd = np.array([(_readme_f(solve(InteriorPoint(), mcp, θ + h * e)) -
                      _readme_f(solve(InteriorPoint(), mcp, θ - h * e))) / (2 * h) for e in np.eye(2)])
    np.testing.assert_allclose(g_rev, g_fd, atol=1e-3)
    d = solve_dual(InteriorPoint(), mcp, θ, np.eye(2))  # partials: the identity seeds
    g_fwd = 2 * d.x @ d.x_partials + 2 * d.y @ d.y_partials
    np.testing.assert_allclose(g_rev, g_fwd, atol=1e-3)
    np.testing.assert_array_equal(d.s, d.y)  # src/AutoDiff.jl:112 quirk kept
    np.testing.assert_array_equal(d.s_value_true, sol.s)


@pytest.mark.gpu
def test_pullback_is_the_oracles_through_the_theta_map(gpu, oracle_lib):
    """Alternative (K-form) constructor, batched θ: the API pullback is the kernel's
    θ'-pullback (bit-exact vs the oracle) chained through ThetaMap.vjp."""
    from mcp_amd.autodiff import solve_pullback

    mcp = alternative_mcp()
    rng = np.random.default_rng(8)
    th = rng.standard_normal((16, 2))
    sol = solve(InteriorPoint(), mcp, th, tol=1e-6)
    gx, gy = rng.standard_normal((16, 2)), rng.standard_normal((16, 2))
    dθ = solve_pullback(sol, gx, gy)
    tp = mcp.theta_map(th)
    ref, _ = oracle_lib.vjp_batch(0, 2, 2, tp, sol.x, sol.y, sol.s, gx, gy, None)
    np.testing.assert_array_equal(dθ, mcp.theta_map.vjp(th, ref))


@pytest.mark.gpu
def test_torch_autograd_through_the_gpu_pullback(gpu):
    import torch

    from mcp_amd.autodiff import solve_pullback, solve_torch

    mcp = basic_mcp()
    th = torch.tensor([[-0.5, 0.5], [0.2, -0.1]], dtype=torch.float64, device="cuda", requires_grad=True)
    x, y, s, status = solve_torch(mcp, th, tol=1e-6)
    loss = (x ** 2).sum() + (y ** 2).sum()
    loss.backward()
    assert status.cpu().tolist() == [0, 0]
    host = solve(InteriorPoint(), mcp, th.detach().cpu().numpy(), tol=1e-6)
    ref = solve_pullback(host, 2 * host.x, 2 * host.y)
    np.testing.assert_array_equal(th.grad.cpu().numpy(), ref)
