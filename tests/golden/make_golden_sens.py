"""Generates the committed sensitivity fixtures tests/golden/sens_*.npz.

For each case: θ, the oracle's solution (x, y, s), seeded cotangents
(gx, gy, gs) and tangents θ̇, and the oracle's pullback ∂θ
(oracle_vjp_batch) and tangents ż (oracle_jvp_batch) with their status.
The oracle's sensitivity restatement (oracle/ipm_oracle.c, src/AutoDiff.jl) is
cross-checked against the independent pivoted-QR restatement
(oracle/ipm_ref.py dz_dtheta) before writing; the reference (Julia) cannot
run here, so these are oracle outputs, not reference outputs.

    python tests/golden/make_golden_sens.py
"""

from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from mcp_amd.qp_benchmark import generate_random_parameter  # noqa: E402
from oracle import coracle, ipm_ref  # noqa: E402
from tests.golden.make_golden import game_clamp_theta, readme_qp_theta  # noqa: E402


def case(name, family, n, m, theta, tol, K, seed):
    theta = np.atleast_2d(theta)
    B, p = theta.shape[0], theta.shape[1]
    rng = np.random.default_rng(seed)
    r = coracle.solve_batch(family, n, m, theta, tol=tol)
    gx, gy, gs = rng.standard_normal((B, n)), rng.standard_normal((B, m)), rng.standard_normal((B, m))
    td = rng.standard_normal((B, K, p))
    dth, st = coracle.vjp_batch(family, n, m, theta, r["x"], r["y"], r["s"], gx, gy, gs)
    zd, stj = coracle.jvp_batch(family, n, m, theta, r["x"], r["y"], r["s"], td)
    for b in range(B):  # cross-check before writing
        if st[b] == 0 and r["status"][b] == 0:
            ref = ipm_ref.vjp(family, theta[b], n, m, r["x"][b], r["y"][b], r["s"][b], gx[b], gy[b], gs[b])
            assert np.abs(ref - dth[b]).max() <= 1e-8 * max(1.0, np.abs(ref).max()), (name, b)
            refj = ipm_ref.jvp(family, theta[b], n, m, r["x"][b], r["y"][b], r["s"][b], td[b])
            assert np.abs(refj - zd[b]).max() <= 1e-8 * max(1.0, np.abs(refj).max()), (name, b)
    np.savez_compressed(os.path.join(HERE, f"sens_{name}.npz"), family=family, n=n, m=m, tol=tol, theta=theta,
                        x=r["x"], y=r["y"], s=r["s"], gx=gx, gy=gy, gs=gs, theta_dot=td, dtheta=dth,
                        vjp_status=st, zdot=zd, jvp_status=stj)
    print(name, B, "vjp status", np.bincount(st), "jvp status", np.bincount(stj))


def main():
    case("readme_qp", 0, 2, 2, readme_qp_theta([-0.5, 0.5]), 1e-4, 3, 1)
    case("qp_n16_m8", 0, 16, 8, generate_random_parameter(np.random.default_rng(11), 16, 8, 0.0, batch=4), 1e-6,
         9, 2)
    case("qp_n32_m16", 0, 32, 16, generate_random_parameter(np.random.default_rng(12), 32, 16, 0.0, batch=4),
         1e-6, 2, 3)
    case("game_clamp", 1, 4, 8, game_clamp_theta([-1.0, 0.0, 1.0, 1.0]), 1e-4, 4, 4)


if __name__ == "__main__":
    main()
