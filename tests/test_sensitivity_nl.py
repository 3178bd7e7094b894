"""Sensitivities of nonlinear-family MCPs (reference src/AutoDiff.jl on a
PrimalDualMCP whose ∇F_θ comes from src/mcp.jl:122-147) — the trajectory games
of src/game.jl, differentiated by examples/utils.jl:233-269 — and of QP / affine
systems beyond the one-wave kernels' 64 rows.

CPU (oracle, test infrastructure):
  * the generated ∇F_θ code (mcp_amd/codegen.py, compiled by gcc) against the
    sympy Jacobian of the traced G/H;
  * the oracle's pullback / tangents against an independent pivoted-QR
    restatement of `_solve_jacobian_θ` (LAPACK geqp3 of −∇F_z, as the reference,
    src/AutoDiff.jl:39) on well-conditioned nonlinear MCPs, 1e-8 relative;
  * the clamp game of test/runtests.jl:88-107 forced through generated code
    against the affine family's (pinned) sensitivities;
  * the reference's AD test (test/runtests.jl:65-85: reverse vs forward vs finite
    differences, atol 1e-3) restated on the clamp game and on the lane-change game.
    The lane change's solutions are degenerate (weakly active bounds; cond(∇F_z) ≈
    1e15), so its θ → x map is not differentiable in every direction there: the
    finite-difference leg is asserted on the directions whose one-sided differences
    agree (differentiable), reverse = forward on all.
GPU (MI355X, through the C ABI): bit-exact against the oracle — the BASELINE C4
batch at T = 2 (1,024 games, failed ones included), T = 10, small modules, QP /
affine at KKT 96 and 256, NULL cotangent blocks, K beyond one factorisation's
partials — plus rrule / solve_dual / solve_torch through a game.
"""

from __future__ import annotations

import numpy as np
import pytest
import scipy.linalg as sl

from mcp_amd import _abi
from mcp_amd.api import PrimalDualMCP
from mcp_amd.lane_change import LaneChangeGame
from mcp_amd.qp_benchmark import generate_random_parameter
from tests.test_api import clamp_game
from tests.test_nonlinear import cubic_mcp, trig_mcp
from tests.test_sensitivity import _same, random_affine_theta


def poly_mcp(n, m, p=6, seed=0):
    """A smooth, strongly monotone polynomial MCP with θ entering G and H nonlinearly:
    G = P x + 0.1 x³ − Aᵀ y + C θ + 0.05 θ₀ x,  H = A x + D θ + 0.05 x[:m]² + 0.5."""
    rng = np.random.default_rng(seed)
    L = rng.standard_normal((n, n))
    P = L @ L.T / n + np.eye(n)
    A = rng.standard_normal((m, n)) / np.sqrt(n)
    C = rng.standard_normal((n, p))
    D = rng.standard_normal((m, p))
    G = lambda x, y, θ: P @ x + 0.1 * x ** 3 - A.T @ y + C @ θ + 0.05 * θ[0] * x
    H = lambda x, y, θ: A @ x + D @ θ + 0.05 * x[:m] ** 2 + 0.5
    return PrimalDualMCP(G, H, unconstrained_dimension=n, constrained_dimension=m, parameter_dimension=p)


def nl_clamp():
    aff = clamp_game().mcp
    return aff, PrimalDualMCP.from_symbolic(aff.G_symbolic, aff.H_symbolic, aff.x_symbolic, aff.y_symbolic,
                                            aff.θ_symbolic, backend_options={"family": "nonlinear"})


def qr_dz_dtheta(mcp, x, y, s, θ):
    """src/AutoDiff.jl:18-40 restated independently: qr(−∇F_z, ColumnNorm()) \\ ∇F_θ with the
    host (sympy) Jacobians of the traced F."""
    J = mcp.jacobian_z(x, y, s, θ=θ)
    Jt = mcp.jacobian_theta(x, y, s, θ=θ)
    Q, R, piv = sl.qr(-J, pivoting=True)
    sol = sl.solve_triangular(R, Q.T @ Jt)
    out = np.empty_like(sol)
    out[piv] = sol
    return out, np.linalg.cond(J)


@pytest.fixture(scope="module")
def lane():
    return LaneChangeGame(2)


# ---------------------------------------------------------------------------
# CPU


def test_generated_dtheta_matches_sympy_jacobian(oracle_lib, lane):
    import ctypes as C

    for mcp in (lane.mcp, poly_mcp(7, 4), trig_mcp()):
        nl = mcp.nl
        G = oracle_lib.nl_lib(nl)
        rng = np.random.default_rng(1)
        nr = nl.n + nl.m
        for _ in range(3):
            th = rng.standard_normal(nl.p)
            z = rng.standard_normal(nr)
            dth = np.zeros(nr * max(nl.p, 1))
            G.oracle_nl_eval_theta(C.c_void_p(th.ctypes.data), C.c_void_p(z.ctypes.data),
                                   C.c_void_p(dth.ctypes.data))
            ref = mcp.jacobian_theta(z[:nl.n], z[nl.n:], np.ones(nl.m), θ=th)[:nr]
            np.testing.assert_allclose(dth[:nr * nl.p].reshape(nl.p, nr).T, ref, rtol=1e-13, atol=1e-13)
        (cp, ci), (rp, ri) = nl.theta_structure()
        assert cp[-1] == rp[-1] == nl.nnz_theta


@pytest.mark.parametrize("n,m", [(6, 3), (40, 30)])
def test_oracle_nl_matches_pivoted_qr(oracle_lib, n, m):
    mcp = poly_mcp(n, m)
    nl = mcp.nl
    B = 6
    rng = np.random.default_rng(n)
    th = rng.standard_normal((B, nl.p))
    r = oracle_lib.solve_batch_nl(nl, th, tol=1e-9, linear_solver="reduced" if n + m <= 64 else "dense")
    gx, gy, gs = rng.standard_normal((B, n)), rng.standard_normal((B, m)), rng.standard_normal((B, m))
    dth, st = oracle_lib.vjp_batch_nl(nl, th, r["x"], r["y"], r["s"], gx, gy, gs)
    td = rng.standard_normal((B, 3, nl.p))
    zd, stj = oracle_lib.jvp_batch_nl(nl, th, r["x"], r["y"], r["s"], td)
    checked = 0
    for b in range(B):
        D, cond = qr_dz_dtheta(mcp, r["x"][b], r["y"][b], r["s"][b], th[b])
        if r["status"][b] != 0 or cond > 1e8:
            continue
        assert st[b] == 0 and stj[b] == 0
        ref = D[:n].T @ gx[b] + D[n:n + m].T @ gy[b] + D[n + m:].T @ gs[b]
        assert np.abs(ref - dth[b]).max() <= 1e-8 * max(1.0, np.abs(ref).max())
        refj = (D @ td[b].T).T
        assert np.abs(refj - zd[b]).max() <= 1e-8 * max(1.0, np.abs(refj).max())
        checked += 1
    assert checked >= 4


def test_oracle_nl_clamp_game_matches_affine_family(oracle_lib):
    """The same game traced into the affine family (θ' layout, analytic ∇F_θ chained with
    ∂θ'/∂θ) and into generated code (∇F_θ w.r.t. θ directly): same sensitivities."""
    aff, nlm = nl_clamp()
    rng = np.random.default_rng(4)
    th = rng.uniform(-1, 1, (16, 4))
    r = oracle_lib.solve_batch(_abi.FAMILY_AFFINE, 4, 8, aff.theta_map(th), tol=1e-8)
    n, m = 4, 8
    gx, gy = rng.standard_normal((16, n)), rng.standard_normal((16, m))
    dtp, st = oracle_lib.vjp_batch(_abi.FAMILY_AFFINE, n, m, aff.theta_map(th), r["x"], r["y"], r["s"], gx, gy)
    d_aff = aff.theta_map.vjp(th, dtp)
    d_nl, st2 = oracle_lib.vjp_batch_nl(nlm.nl, th, r["x"], r["y"], r["s"], gx, gy)
    np.testing.assert_array_equal(st, st2)
    np.testing.assert_allclose(d_nl, d_aff, rtol=1e-9, atol=1e-9)
    td = rng.standard_normal((16, 2, 4))
    za, _ = oracle_lib.jvp_batch(_abi.FAMILY_AFFINE, n, m, aff.theta_map(th), r["x"], r["y"], r["s"],
                                 aff.theta_map.jvp(th, td))
    zn, _ = oracle_lib.jvp_batch_nl(nlm.nl, th, r["x"], r["y"], r["s"], td)
    np.testing.assert_allclose(zn, za, rtol=1e-9, atol=1e-9)


def _ad_test(oracle_lib, mcp, th, solve_kw, x0=None, h=1e-5, differentiable_only=False, loss_rows=None):
    """test/runtests.jl:65-85 on an oracle solve: ∇f by the pullback (Zygote rrule) against
    forward mode (ForwardDiff Dual) and central finite differences, atol 1e-3.  Loss
    f(θ) = Σ w⊙x (+ Σ y² when loss_rows is None: Σx² + Σy² as the reference)."""
    nl = mcp.nl
    n, m = nl.n, nl.m

    def sol(t):
        t = t[None]
        return oracle_lib.solve_batch_nl(nl, t, x0=None if x0 is None else x0(t), **solve_kw)

    rng = np.random.default_rng(0)
    w = None if loss_rows is None else rng.standard_normal(loss_rows)

    def f(r):
        if w is None:
            return float((r["x"] ** 2).sum() + (r["y"] ** 2).sum())
        return float(w @ r["x"][0, :loss_rows])

    r = sol(th)
    assert r["status"][0] == 0
    gx = np.zeros((1, n))
    gy = None
    if w is None:
        gx, gy = 2 * r["x"], 2 * r["y"]
    else:
        gx[0, :loss_rows] = w
    grad_rev, st = oracle_lib.vjp_batch_nl(nl, th[None], r["x"], r["y"], r["s"], gx, gy)
    assert st[0] == 0
    grad_rev = grad_rev[0]
    zd, _ = oracle_lib.jvp_batch_nl(nl, th[None], r["x"], r["y"], r["s"], np.eye(nl.p)[None])
    grad_fwd = zd[0, :, :n] @ gx[0] + (0 if gy is None else zd[0, :, n:n + m] @ gy[0])
    np.testing.assert_allclose(grad_rev, grad_fwd, rtol=1e-9, atol=1e-9)
    fp = np.array([f(sol(th + h * e)) for e in np.eye(nl.p)])
    fm = np.array([f(sol(th - h * e)) for e in np.eye(nl.p)])
    f0 = f(r)
    central = (fp - fm) / (2 * h)
    if differentiable_only:  # one-sided differences agree ⇒ differentiable in that direction
        ok = np.abs((fp - f0) / h - (f0 - fm) / h) <= 1e-3
        assert ok.sum() >= nl.p // 2
        np.testing.assert_allclose(grad_rev[ok], central[ok], atol=1e-3)
    else:
        np.testing.assert_allclose(grad_rev, central, atol=1e-3)


def test_reference_ad_test_on_clamp_game(oracle_lib):
    _, nlm = nl_clamp()
    _ad_test(oracle_lib, nlm, np.array([0.3, -0.7, 0.1, 0.9]), dict(tol=1e-8, linear_solver="reduced"))


def test_reference_ad_test_on_lane_change(oracle_lib, lane):
    th = lane.generate_random_parameter(np.random.default_rng(1), 4)[1]
    _ad_test(oracle_lib, lane.mcp, th, dict(tol=1e-8, linear_solver="schur"), x0=lane.initial_guess, h=1e-4,
             differentiable_only=True, loss_rows=24)


def test_nl_sensitivities_python_api_requires_module_kernels(lane):
    """The API no longer refuses nonlinear MCPs; the module reports its kernels."""
    from mcp_amd import autodiff

    autodiff._require_sensitivities(lane.mcp)  # no NotImplementedError any more
    ws = lane.mcp.nl.wg_solvers()
    assert ws["reduced"] and ws["dense"]  # → mcpx_nl_vjp_wg / mcpx_nl_jvp_wg are compiled in


# ---------------------------------------------------------------------------
# GPU


def _gpu_vs_oracle_nl(oracle_lib, mcp, tp, x, y, s, rng, K=3, null=None):
    from mcp_amd.batch import jvp_batch, vjp_batch

    nl, mod = mcp.nl, mcp.module()
    B = tp.shape[0]
    n, m = nl.n, nl.m
    g = dict(gx=rng.standard_normal((B, n)), gy=rng.standard_normal((B, m)), gs=rng.standard_normal((B, m)))
    if null:
        g[null] = None
    dth, st = vjp_batch(_abi.FAMILY_NONLINEAR, n, m, tp, x, y, s, **g, module=mod)
    rdth, rst = oracle_lib.vjp_batch_nl(nl, tp, x, y, s, **g, nthreads=8)
    np.testing.assert_array_equal(st, rst)
    assert _same(dth, rdth)
    td = rng.standard_normal((B, K, nl.p))
    zd, stj = jvp_batch(_abi.FAMILY_NONLINEAR, n, m, tp, x, y, s, td, module=mod)
    rzd, rstj = oracle_lib.jvp_batch_nl(nl, tp, x, y, s, td, nthreads=8)
    np.testing.assert_array_equal(stj, rstj)
    assert _same(zd, rzd)


@pytest.mark.gpu
def test_gpu_lane_change_c4_sensitivities_bit_exact(gpu, lane, oracle_lib):
    """The BASELINE C4 batch (1,024 games, the bench's θ stream) solved on the GPU, then the
    pullback and 10 tangents (one per θ entry; two factorisations' worth of partials) of
    every game — failed games included — bit-exact against the oracle."""
    from mcp_amd.batch import solve_batch
    from mcp_amd.qp_benchmark import chunked_slice

    mcp = lane.mcp
    th = chunked_slice(lambda rng, k: lane.generate_random_parameter(rng, k), 1, 0, 1024)
    tp = np.ascontiguousarray(mcp.theta_map(th))
    r = solve_batch(_abi.FAMILY_NONLINEAR, 40, 50, tp, linear_solver="schur", tol=1e-6, module=mcp.module())
    assert (r["status"] != 0).sum() >= 10  # failed games are in the batch
    _gpu_vs_oracle_nl(oracle_lib, mcp, tp, r["x"], r["y"], r["s"], np.random.default_rng(3), K=10)


@pytest.mark.gpu
@pytest.mark.parametrize("null", ["gx", "gy", "gs"])
def test_gpu_lane_change_null_cotangents(gpu, lane, oracle_lib, null):
    from mcp_amd.batch import solve_batch

    mcp = lane.mcp
    th = lane.generate_random_parameter(np.random.default_rng(8), 64)
    tp = mcp.theta_map(th)
    r = solve_batch(_abi.FAMILY_NONLINEAR, 40, 50, tp, x0=lane.initial_guess(th), linear_solver="schur",
                    module=mcp.module())
    _gpu_vs_oracle_nl(oracle_lib, mcp, tp, r["x"], r["y"], r["s"], np.random.default_rng(9), K=1, null=null)


@pytest.mark.gpu
def test_gpu_lane_change_t10_sensitivities_bit_exact(gpu, oracle_lib):
    """Horizon T = 10 (n = 200, m = 250: a 450-dim adjoint system, a 700-dim tangent system)."""
    from mcp_amd.batch import solve_batch

    game = LaneChangeGame(10)
    mcp = game.mcp
    th = game.generate_random_parameter(np.random.default_rng(2), 6)
    tp = mcp.theta_map(th)
    r = solve_batch(_abi.FAMILY_NONLINEAR, 200, 250, tp, x0=game.initial_guess(th), linear_solver="schur",
                    module=mcp.module())
    _gpu_vs_oracle_nl(oracle_lib, mcp, tp, r["x"], r["y"], r["s"], np.random.default_rng(10), K=9)


@pytest.mark.gpu
@pytest.mark.parametrize("make", [cubic_mcp, trig_mcp, lambda: poly_mcp(40, 30)], ids=["cubic", "trig", "poly70"])
def test_gpu_small_modules_sensitivities(gpu, oracle_lib, make):
    """Polynomial modules are bit-exact; the transcendental one is compared bit-exact too
    because both sides evaluate ∇F_θ / ∇F_z from the same z with the same libm-free
    arithmetic except sin/exp (held to 1e-8 when they differ by an ulp)."""
    from mcp_amd.batch import jvp_batch, vjp_batch

    mcp = make()
    nl = mcp.nl
    rng = np.random.default_rng(11)
    B = 96
    th = rng.uniform(-1, 1, (B, nl.p))
    r = oracle_lib.solve_batch_nl(nl, th, tol=1e-8, linear_solver="dense" if nl.n + 2 * nl.m <= 64 else "reduced"
                                  if nl.n + nl.m <= 64 else "dense", nthreads=8)
    if make is trig_mcp:
        gx = rng.standard_normal((B, nl.n))
        dth, st = vjp_batch(_abi.FAMILY_NONLINEAR, nl.n, nl.m, th, r["x"], r["y"], r["s"], gx, module=mcp.module())
        rdth, rst = oracle_lib.vjp_batch_nl(nl, th, r["x"], r["y"], r["s"], gx)
        np.testing.assert_array_equal(st, rst)
        np.testing.assert_allclose(dth, rdth, rtol=1e-8, atol=1e-10)
        td = rng.standard_normal((B, 2, nl.p))
        zd, _ = jvp_batch(_abi.FAMILY_NONLINEAR, nl.n, nl.m, th, r["x"], r["y"], r["s"], td, module=mcp.module())
        rzd, _ = oracle_lib.jvp_batch_nl(nl, th, r["x"], r["y"], r["s"], td)
        np.testing.assert_allclose(zd, rzd, rtol=1e-8, atol=1e-10)
        return
    _gpu_vs_oracle_nl(oracle_lib, mcp, th, r["x"], r["y"], r["s"], rng, K=13)


@pytest.mark.gpu
@pytest.mark.parametrize("fam,n,m", [(0, 48, 24), (1, 40, 30), (0, 128, 64)])
def test_gpu_large_qp_affine_sensitivities(gpu, oracle_lib, fam, n, m):
    """QP / affine systems beyond 64 KKT rows: the workgroup sensitivity kernels
    (sens_inst_wg.hip), bit-exact against the same oracle as the one-wave kernels."""
    from mcp_amd.batch import jvp_batch, vjp_batch

    rng = np.random.default_rng(n + m)
    B = 24
    th = generate_random_parameter(rng, n, m, 0.0, batch=B) if fam == 0 else random_affine_theta(rng, n, m, B)
    r = oracle_lib.solve_batch(fam, n, m, th, tol=1e-6, nthreads=8)
    gx, gy, gs = rng.standard_normal((B, n)), rng.standard_normal((B, m)), rng.standard_normal((B, m))
    dth, st = vjp_batch(fam, n, m, th, r["x"], r["y"], r["s"], gx, gy, gs)
    rdth, rst = oracle_lib.vjp_batch(fam, n, m, th, r["x"], r["y"], r["s"], gx, gy, gs, nthreads=8)
    np.testing.assert_array_equal(st, rst)
    assert _same(dth, rdth)
    td = rng.standard_normal((B, 3, th.shape[1]))
    zd, stj = jvp_batch(fam, n, m, th, r["x"], r["y"], r["s"], td)
    rzd, rstj = oracle_lib.jvp_batch(fam, n, m, th, r["x"], r["y"], r["s"], td, nthreads=8)
    np.testing.assert_array_equal(stj, rstj)
    assert _same(zd, rzd)


@pytest.mark.gpu
def test_gpu_qp_vjp_nonfinite_cotangents(gpu, oracle_lib):
    """the QP y-rows' structural zeros are skipped on both sides, so Inf / NaN
    in gs (and y) give the same bits."""
    from mcp_amd.batch import vjp_batch

    rng = np.random.default_rng(12)
    n, m, B = 16, 8, 16
    th = generate_random_parameter(rng, n, m, 0.0, batch=B)
    r = oracle_lib.solve_batch(0, n, m, th, tol=1e-6)
    gx, gy, gs = rng.standard_normal((B, n)), rng.standard_normal((B, m)), rng.standard_normal((B, m))
    gs[0, 0], gs[1, 3], gs[2, :] = np.inf, np.nan, -np.inf
    y = r["y"].copy()
    y[3, 1] = np.inf
    for nmax_big in (False, True):
        if nmax_big:  # the same instances through the workgroup kernel (n + 2m > 64)
            n2, m2 = 48, 24
            th2 = generate_random_parameter(rng, n2, m2, 0.0, batch=4)
            r2 = oracle_lib.solve_batch(0, n2, m2, th2, tol=1e-6)
            g2 = rng.standard_normal((4, m2))
            g2[0, 0], g2[1, 1] = np.inf, np.nan
            got = vjp_batch(0, n2, m2, th2, r2["x"], r2["y"], r2["s"], None, None, g2)
            ref = oracle_lib.vjp_batch(0, n2, m2, th2, r2["x"], r2["y"], r2["s"], None, None, g2)
        else:
            got = vjp_batch(0, n, m, th, r["x"], y, r["s"], gx, gy, gs)
            ref = oracle_lib.vjp_batch(0, n, m, th, r["x"], y, r["s"], gx, gy, gs)
        np.testing.assert_array_equal(got[1], ref[1])
        assert _same(got[0], ref[0])


@pytest.mark.gpu
def test_gpu_game_rrule_and_dual(gpu, lane, oracle_lib):
    """rrule(solve, game, θ) (the Zygote path of examples/utils.jl:233-269) and the Dual
    method through the lane-change game: both against the oracle, and reverse ≡ forward."""
    from mcp_amd.api import InteriorPoint, solve
    from mcp_amd.autodiff import rrule, solve_dual

    th = lane.generate_random_parameter(np.random.default_rng(1), 4)[1]
    x0 = lane.initial_guess(th[None])[0]
    sol, back = rrule(solve, lane.game, th, x0=x0, tol=1e-8, linear_solve_algorithm="schur")
    assert sol.status == "solved"
    w = np.random.default_rng(2).standard_normal(12)
    _, _, dθ = back({"primals": [w, None]})
    nl = lane.mcp.nl
    gx = np.zeros((1, nl.n))
    gx[0, :12] = w
    rdθ, _ = oracle_lib.vjp_batch_nl(nl, th[None], sol.variables["x"][None], sol.variables["y"][None],
                                     sol.variables["s"][None], gx)
    assert _same(dθ, rdθ[0])
    ds = solve_dual(InteriorPoint(), lane.mcp, th, np.eye(nl.p), x0=x0, tol=1e-8, linear_solve_algorithm="schur")
    np.testing.assert_allclose(ds.x_partials[:12].T @ w, dθ, rtol=1e-9, atol=1e-9)


@pytest.mark.gpu
def test_gpu_solve_torch_through_game(gpu, lane, oracle_lib):
    """torch autograd through a batch of lane-change solves on the device (the torch
    analogue of Zygote.gradient over game solves)."""
    import torch

    from mcp_amd.autodiff import solve_torch

    th = lane.generate_random_parameter(np.random.default_rng(6), 32)
    t = torch.from_numpy(th).cuda().requires_grad_(True)
    x, y, s, status = solve_torch(lane.mcp, t, x0=torch.from_numpy(lane.initial_guess(th)).cuda(),
                                  linear_solve_algorithm="schur")
    loss = (x[:, :24] ** 2).sum()
    loss.backward()
    nl = lane.mcp.nl
    xh = x.detach().cpu().numpy()
    gx = np.zeros_like(xh)
    gx[:, :24] = 2 * xh[:, :24]
    ref, _ = oracle_lib.vjp_batch_nl(nl, th, xh, y.detach().cpu().numpy(), s.detach().cpu().numpy(), gx,
                                     nthreads=8)
    assert _same(t.grad.cpu().numpy(), ref)
