"""Generates the committed fixtures in tests/golden/*.npz.

Inputs are the reference's own test problems (test/runtests.jl) and synthetic
draws of the reference benchmark family (benchmark/quadratic_program_benchmark.jl,
numpy PCG64 with the seeds below — the reference's MersenneTwister(1) stream
cannot be reproduced without Julia).  Expected outputs are produced by the C
oracle (oracle/ipm_oracle.c), whose algorithm is pinned by the reference's
analytic assertions (tests/test_oracle.py) and by the independent LAPACK
restatement (oracle/ipm_ref.py).  The reference itself (Julia) cannot run
here, so these vectors are oracle outputs, not reference outputs.

    python tests/golden/make_golden.py
"""

from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from mcp_amd.qp_benchmark import generate_random_parameter  # noqa: E402
from oracle import coracle  # noqa: E402

TRACE = 1024
FIELDS = ("x", "y", "s", "kkt_error", "eps", "outer_iters", "status", "newton_iters", "active_mask",
          "alpha_trace")


def readme_qp_theta(phi):
    """README.md:51-57 / test/runtests.jl:16-19 QP in the QP-family layout:
    M=[2 1;1 2], A=I, b=[1,1], ϕ=θ."""
    M = np.array([[2.0, 1.0], [1.0, 2.0]])
    A = np.eye(2)
    b = np.ones(2)
    return np.concatenate([M.flatten("F"), A.flatten("F"), b, np.asarray(phi, float)])


def game_clamp_theta(theta, lim=0.5):
    """test/runtests.jl:88-116 ParametricGame (two players, |x_i| ≤ lim, objective ‖x_i − θ_i‖²)
    as the affine MCP produced by src/game.jl:47-157:
    G = ∇_x L = 2x − 2θ + [I −I] μ (per player), H = [−x + lim; x + lim]."""
    n, m = 4, 8
    P = 2.0 * np.eye(n)
    Q = np.zeros((n, m))
    R = np.zeros((m, n))
    for i in range(2):  # player blocks
        xs = slice(2 * i, 2 * i + 2)
        Q[xs, 4 * i: 4 * i + 2] = np.eye(2)       # −(∂h/∂x)ᵀ μ with ∂h_a/∂x = −I
        Q[xs, 4 * i + 2: 4 * i + 4] = -np.eye(2)  # ∂h_b/∂x = +I
        R[4 * i: 4 * i + 2, xs] = -np.eye(2)
        R[4 * i + 2: 4 * i + 4, xs] = np.eye(2)
    S = np.zeros((m, m))
    g = -2.0 * np.asarray(theta, float)
    h = lim * np.ones(m)
    return np.concatenate([P.flatten("F"), Q.flatten("F"), R.flatten("F"), S.flatten("F"), g, h])


def qp_theta_with_M(rng, n, m, B, kind):
    """Random QPs whose M is non-symmetric ("asym": the SCHUR solve falls back to the
    pivoting LU every step) or symmetric indefinite ("indef": the pivot-free SPD
    Gauss-Jordan meets a pivot ≤ 0 and that step falls back)."""
    th = generate_random_parameter(rng, n, m, 0.0, batch=B)
    M = th[:, :n * n].reshape(B, n, n).transpose(0, 2, 1)  # column-major blocks
    if kind == "asym":
        M = M + 0.5 * rng.standard_normal((B, n, n))
    else:
        M = M - np.trace(M, axis1=1, axis2=2)[:, None, None] / n * np.eye(n)
    th[:, :n * n] = M.transpose(0, 2, 1).reshape(B, n * n)
    return th


def case(name, family, n, m, theta, **kw):
    theta = np.atleast_2d(np.asarray(theta, dtype=np.float64))
    r = coracle.solve_batch(family, n, m, theta, trace_len=TRACE, **kw)
    d = dict(family=np.int32(family), n=np.int32(n), m=np.int32(m), theta=theta)
    for k, v in kw.items():
        d["param_" + k] = np.asarray(v)
    for f in FIELDS:
        d["out_" + f] = r[f]
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
    print(f"{name}: B={theta.shape[0]} N={n + 2 * m} solved={int((r['status'] == 0).sum())} "
          f"newton mean={r['newton_iters'].mean():.1f}")


def main():
    coracle.build(force=True)
    # C1: README / test QP (θ = ϕ = [−0.5, 0.5]) with the default tol=1e-4 and the benchmark tol
    case("readme_qp", 0, 2, 2, readme_qp_theta([-0.5, 0.5]))
    case("readme_qp_tol1e-6", 0, 2, 2, readme_qp_theta([-0.5, 0.5]), tol=1e-6)
    rng = np.random.default_rng(20250808)
    case("readme_qp_rand", 0, 2, 2, np.stack([readme_qp_theta(rng.random(2)) for _ in range(8)]))
    # C2 / C3 shapes, dense QPs, benchmark tol (benchmark/path.jl:8)
    case("qp_n16_m8_dense", 0, 16, 8, generate_random_parameter(np.random.default_rng(1), 16, 8, 0.0, batch=16),
         tol=1e-6)
    case("qp_n32_m16_dense", 0, 32, 16, generate_random_parameter(np.random.default_rng(2), 32, 16, 0.0, batch=8),
         tol=1e-6)
    # reference-default sparsity 0.9: mostly :failed, long iteration counts
    case("qp_n16_m8_sparse", 0, 16, 8, generate_random_parameter(np.random.default_rng(3), 16, 8, 0.9, batch=8),
         tol=1e-6)
    # game → MCP clamp test (affine family), tol=1e-4 as in test/runtests.jl:94
    case("game_clamp", 1, 4, 8, game_clamp_theta([-1.0, 0.0, 1.0, 1.0]), tol=1e-4)
    # the full-system dense LU (MCPX_LINSOLVE_DENSE) on the same inputs
    case("readme_qp_dense", 0, 2, 2, readme_qp_theta([-0.5, 0.5]), linear_solver="dense")
    case("qp_n16_m8_dense_lu", 0, 16, 8, generate_random_parameter(np.random.default_rng(1), 16, 8, 0.0, batch=16),
         tol=1e-6, linear_solver="dense")
    case("qp_n32_m16_dense_lu", 0, 32, 16, generate_random_parameter(np.random.default_rng(2), 32, 16, 0.0, batch=8),
         tol=1e-6, linear_solver="dense")
    case("qp_n16_m8_sparse_dense_lu", 0, 16, 8,
         generate_random_parameter(np.random.default_rng(3), 16, 8, 0.9, batch=8), tol=1e-6, linear_solver="dense")
    case("game_clamp_dense", 1, 4, 8, game_clamp_theta([-1.0, 0.0, 1.0, 1.0]), tol=1e-4, linear_solver="dense")
    # the MFMA Schur-complement solve (QP family)
    case("readme_qp_schur", 0, 2, 2, readme_qp_theta([-0.5, 0.5]), linear_solver="schur")
    case("qp_n16_m8_schur", 0, 16, 8, generate_random_parameter(np.random.default_rng(1), 16, 8, 0.0, batch=16),
         tol=1e-6, linear_solver="schur")
    case("qp_n32_m16_schur", 0, 32, 16, generate_random_parameter(np.random.default_rng(2), 32, 16, 0.0, batch=8),
         tol=1e-6, linear_solver="schur")
    case("qp_n16_m8_sparse_schur", 0, 16, 8,
         generate_random_parameter(np.random.default_rng(3), 16, 8, 0.9, batch=8), tol=1e-6, linear_solver="schur")
    # the SCHUR solve's fallback from the SPD Gauss-Jordan to the pivoting LU
    case("qp_n16_m8_asym_schur", 0, 16, 8, qp_theta_with_M(np.random.default_rng(4), 16, 8, 8, "asym"), tol=1e-6,
         linear_solver="schur")
    case("qp_n16_m8_indef_schur", 0, 16, 8, qp_theta_with_M(np.random.default_rng(5), 16, 8, 8, "indef"), tol=1e-6,
         linear_solver="schur")


if __name__ == "__main__":
    main()
