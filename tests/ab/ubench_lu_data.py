"""Dumps Schur complements S (and rhs) of the lane-change game at T = 2 for tools/ubench_lu.hip:
S = (P + tol·I) − Q D⁻¹ R at the iterate after a few outer iterations (oracle), rows
canonicalised as the kernel does; and the oracle LU's solution for checking.
    python tests/ab/ubench_lu_data.py B   → tools/ubench_data/lu_S.bin (B×40×41 doubles, row-major [S | rhs])"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from mcp_amd.lane_change import LaneChangeGame
from mcp_amd.qp_benchmark import chunked_slice
from oracle import coracle

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
g = LaneChangeGame(2); mcp = g.mcp; nl = mcp.nl; n, m = nl.n, nl.m
th = chunked_slice(lambda rng, k: g.generate_random_parameter(rng, k), 1, 0, B)
tol = 1e-6
out = np.zeros((B, n, n + 1))
rng = np.random.default_rng(0)
for b in range(B):
    r = coracle.solve_batch_nl(nl, th[b:b + 1], linear_solver="schur", tol=tol, max_outer_iters=int(rng.integers(2, 8)))
    x, y, s = r["x"][0], r["y"][0], r["s"][0]
    J = mcp.jacobian_z(x, y, s, θ=th[b])
    P = J[:n, :n]; Q = J[:n, n:n + m]; R = J[n:n + m, :n]
    D = tol + s / (y + tol)
    S = P + tol * np.eye(n) - Q @ np.diag(1 / D) @ R
    out[b, :, :n] = S + 0.0
    out[b, :, n] = rng.standard_normal(n)
os.makedirs(os.path.join(ROOT, "tools", "ubench_data"), exist_ok=True)
out.tofile(os.path.join(ROOT, "tools", "ubench_data", "lu_S.bin"))
pat = np.full(n, (1 << 64) - 1, dtype=np.uint64)  # dense pattern (the sparse variant 6 reads it)
pat.tofile(os.path.join(ROOT, "tools", "ubench_data", "lu_pat.bin"))
print("wrote", out.shape)
