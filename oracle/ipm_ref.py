"""ORACLE — TEST INFRASTRUCTURE ONLY.

Independent numpy/LAPACK restatement of the reference interior-point solver
(MixedComplementarityProblems.jl, src/solver.jl:35-138), written directly from
the Julia source and sharing no code with oracle/ipm_oracle.c.  It differs from
the C oracle deliberately in the one place the reference itself is
implementation-defined — the Newton linear solve: the reference calls UMFPACK
through LinearSolve.jl (src/solver.jl:50,61,83), this module calls LAPACK
dgetrf/dgetrs (scipy.linalg.lu_factor) on the dense ∇F + tol·I, the C oracle
uses its own unblocked LU.  Agreement of the two is therefore evidence that the
C oracle restates the reference *algorithm* (loop bounds, ϵ schedule, line
search, update order, status logic), independent of LU rounding.

Used only by tests/ (never by the product package mcp_amd/).
"""

from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import scipy.linalg

QP, AFFINE = 0, 1


def theta_dim(family: int, n: int, m: int) -> int:
    if family == QP:  # benchmark/quadratic_program_benchmark.jl:77-90
        return n * n + m * n + m + n
    return n * n + 2 * n * m + m * m + n + m


def unpack(family: int, theta: np.ndarray, n: int, m: int):
    """θ → (P, Q, R, S, g, h) with G = P x + Q y + g, H = R x + S y + h."""
    th = np.asarray(theta, dtype=np.float64)
    if family == QP:
        # unpack_parameters, benchmark/quadratic_program_benchmark.jl:77-90 (column-major)
        M = th[: n * n].reshape(n, n, order="F")
        A = th[n * n : n * n + m * n].reshape(m, n, order="F")
        b = th[n * n + m * n : n * n + m * n + m]
        phi = th[n * n + m * n + m : n * n + m * n + m + n]
        # G = M x − ϕ − Aᵀ y, H = A x − b  (:12-32)
        return M, -A.T, A, np.zeros((m, m)), -phi, -b
    o = 0
    P = th[o : o + n * n].reshape(n, n, order="F"); o += n * n
    Q = th[o : o + n * m].reshape(n, m, order="F"); o += n * m
    R = th[o : o + m * n].reshape(m, n, order="F"); o += m * n
    S = th[o : o + m * m].reshape(m, m, order="F"); o += m * m
    g = th[o : o + n]; o += n
    h = th[o : o + m]
    return P, Q, R, S, g, h


def F_and_jacobian(blocks, x, y, s, eps):
    """F = [G; H − s; s⊙y − ϵ] (src/mcp.jl:76-80) and ∇_z F (src/mcp.jl:97-120)."""
    P, Q, R, S, g, h = blocks
    n, m = len(x), len(y)
    G = P @ x + Q @ y + g
    H = R @ x + S @ y + h
    F = np.concatenate([G, H - s, s * y - eps])
    N = n + 2 * m
    J = np.zeros((N, N))
    J[:n, :n] = P
    J[:n, n : n + m] = Q
    J[n : n + m, :n] = R
    J[n : n + m, n : n + m] = S
    J[n : n + m, n + m :] = -np.eye(m)
    J[n + m :, n : n + m] = np.diag(s)
    J[n + m :, n + m :] = np.diag(y)
    return F, J


def fraction_to_the_boundary_linesearch(v, d, tau=0.995, decay=0.5, tol=1e-4):
    """src/solver.jl:127-138, literally.  Returns (α, number of halvings)."""
    alpha = 1.0
    e = 0
    while np.any(v + alpha * d < (1 - tau) * v):
        if alpha < tol:
            return math.nan, -1
        alpha *= decay
        e += 1
    return alpha, e


@dataclass
class Solution:
    status: str
    x: np.ndarray
    y: np.ndarray
    s: np.ndarray
    kkt_error: float
    eps: float
    outer_iters: int
    newton_iters: int
    alpha_trace: list


def solve(family, theta, n, m, **kw):
    """src/solver.jl:35-122 for one instance of the QP / affine family."""
    blocks = unpack(family, theta, n, m)
    return solve_fj(lambda x, y, s, eps: F_and_jacobian(blocks, x, y, s, eps), n, m, **kw)


def nl_callbacks(G, H, xs, ys, ts):
    """Independent evaluation of a nonlinear MCP — sympy.lambdify of G, H and their
    Jacobian, sharing nothing with the generated C of mcp_amd/codegen.py: returns
    θ ↦ FJ(x, y, s, ϵ) = (F, ∇F_z) for solve_fj (src/mcp.jl:72-120)."""
    import sympy as sp

    n, m = len(xs), len(ys)
    zs = list(xs) + list(ys)
    args = zs + list(ts)
    GH = list(G) + list(H)
    f = sp.lambdify(args, GH, "numpy")
    jac = sp.lambdify(args, sp.Matrix(GH).jacobian(zs), "numpy")

    def bind(theta):
        th = [float(t) for t in np.asarray(theta, dtype=np.float64)]

        def FJ(x, y, s, eps):
            a = [float(v) for v in x] + [float(v) for v in y] + th
            gh = np.array(f(*a), dtype=np.float64).reshape(n + m)
            J = np.zeros((n + 2 * m, n + 2 * m))
            J[:n + m, :n + m] = np.array(jac(*a), dtype=np.float64).reshape(n + m, n + m)
            J[n:n + m, n + m:] = -np.eye(m)
            J[n + m:, n:n + m] = np.diag(s)
            J[n + m:, n + m:] = np.diag(y)
            return np.concatenate([gh[:n], gh[n:] - s, s * y - eps]), J

        return FJ

    return bind


def solve_fj(FJ, n, m, *, x0=None, y0=None, s0=None, tol=1e-4, max_inner_iters=20, max_outer_iters=50,
             tightening_rate=0.1, loosening_rate=0.5, min_stepsize=1e-4):
    """The loop of src/solver.jl:35-122 on a callback FJ(x, y, s, ϵ) → (F, ∇F_z)."""
    N = n + 2 * m
    x = np.zeros(n) if x0 is None else np.array(x0, dtype=np.float64)
    y = np.ones(m) if y0 is None else np.array(y0, dtype=np.float64)
    s = np.ones(m) if s0 is None else np.array(s0, dtype=np.float64)
    eps = 1.0
    kkt_error = math.inf
    status = "solved"
    outer_iters = 1
    newton = 0
    trace = []
    while kkt_error > tol and eps > tol and outer_iters < max_outer_iters:
        inner_iters = 1
        status = "solved"
        while kkt_error > eps and inner_iters < max_inner_iters:
            F, J = FJ(x, y, s, eps)
            A = J + tol * np.eye(N)
            try:
                with np.errstate(all="ignore"):
                    lu = scipy.linalg.lu_factor(A, check_finite=False)
                if np.any(np.diag(lu[0]) == 0.0):
                    raise np.linalg.LinAlgError("singular")
                dz = scipy.linalg.lu_solve(lu, -F, check_finite=False)
            except (np.linalg.LinAlgError, ValueError):
                status = "failed"
                break
            dx, dy, ds = dz[:n], dz[n : n + m], dz[n + m :]
            a_s, es = fraction_to_the_boundary_linesearch(s, ds, tol=min_stepsize)
            a_y, ey = fraction_to_the_boundary_linesearch(y, dy, tol=min_stepsize)
            trace.append((es if es >= 0 else 255, ey if ey >= 0 else 255))
            if math.isnan(a_s) or math.isnan(a_y):
                status = "failed"
                break
            x = x + a_s * dx
            s = s + a_s * ds
            y = y + a_y * dy
            absF = np.abs(F)
            kkt_error = math.nan if np.any(np.isnan(absF)) else float(absF.max())
            inner_iters += 1
            newton += 1
        eps *= (1 - math.exp(-tightening_rate * inner_iters)) if status == "solved" else (
            1 + math.exp(-loosening_rate * inner_iters))
        outer_iters += 1
    if outer_iters == max_outer_iters:
        status = "failed"
    return Solution(status, x, y, s, kkt_error, eps, outer_iters, newton, trace)


# ---------------------------------------------------------------------------
# sensitivities (src/AutoDiff.jl)


def jacobian_theta(family, theta, n, m, x, y, s):
    """∇F_θ (N × p) at (x, y, s).  F is affine in θ for both families, so column t
    is F(z; e_t) − F(z; 0) (with the θ-free terms cancelling exactly)."""
    p = theta_dim(family, n, m)
    z0 = F_and_jacobian(unpack(family, np.zeros(p), n, m), x, y, s, 0.0)[0]
    cols = np.empty((n + 2 * m, p))
    for t in range(p):
        e = np.zeros(p)
        e[t] = 1.0
        cols[:, t] = F_and_jacobian(unpack(family, e, n, m), x, y, s, 0.0)[0] - z0
    return cols


def dz_dtheta(family, theta, n, m, x, y, s):
    """src/AutoDiff.jl:18-40: `qr(−∇F_z, ColumnNorm()) \\ ∇F_θ` (LAPACK geqp3, as
    the reference), evaluated at the solution WITHOUT tol·I.  For a full-rank
    ∇F_z the pivoted-QR solve is P R⁻¹ Qᵀ B."""
    _, J = F_and_jacobian(unpack(family, theta, n, m), x, y, s, 0.0)
    B = jacobian_theta(family, theta, n, m, x, y, s)
    Q, R, piv = scipy.linalg.qr(-J, pivoting=True)
    sol = scipy.linalg.solve_triangular(R, Q.T @ B)
    out = np.empty_like(sol)
    out[piv] = sol
    return out


def vjp(family, theta, n, m, x, y, s, gx, gy, gs):
    """rrule pullback, src/AutoDiff.jl:59-76: ∂z∂θ[x rows]ᵀ ∂l∂x + ∂z∂θ[y rows]ᵀ ∂l∂y + ∂z∂θ[s rows]ᵀ ∂l∂s."""
    D = dz_dtheta(family, theta, n, m, x, y, s)
    return D[:n].T @ gx + D[n : n + m].T @ gy + D[n + m :].T @ gs


def jvp(family, theta, n, m, x, y, s, theta_dot):
    """ForwardDiff Dual method, src/AutoDiff.jl:94-100: z_p = ∂z∂θ · θ_p; theta_dot (K, p) → (K, N)."""
    D = dz_dtheta(family, theta, n, m, x, y, s)
    return (D @ np.atleast_2d(theta_dot).T).T
