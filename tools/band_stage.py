"""One bounded run of the band SCHUR kernel (diagnostic): python tools/band_stage.py T B OUTER INNER
prints the time of the GPU solve and its mismatches against the oracle's lu_band_solve."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mcp_amd import _abi
from mcp_amd.batch import solve_batch
from oracle import coracle
from tests.test_band import _c4

T, B, OUTER, INNER = (int(a) for a in sys.argv[1:5])
t0 = time.time()
game, tp = _c4(T, B)
nl = game.mcp.nl
mod = game.mcp.module()
print(f"T={T} B={B} outer={OUTER} inner={INNER}: setup {time.time() - t0:.1f}s", flush=True)
kw = dict(linear_solver="schur", trace_len=1024, max_outer_iters=OUTER, max_inner_iters=INNER)
t0 = time.time()
got = solve_batch(_abi.FAMILY_NONLINEAR, nl.n, nl.m, tp, module=mod, kernel="band", **kw)
t1 = time.time()
ref = coracle.solve_batch_nl(nl, tp, nthreads=8, kernel="band", **kw)
bad = {}
for k in ("x", "y", "s", "kkt_error", "eps", "status", "newton_iters", "outer_iters", "alpha_trace"):
    g, r = np.asarray(got[k]), np.asarray(ref[k])
    same = (g == r) | (np.isnan(g) & np.isnan(r)) if g.dtype.kind == "f" else (g == r)
    bad[k] = int((~same.reshape(B, -1).all(1)).sum())
print(f"  gpu {t1 - t0:.3f}s newton {int(np.sum(got['newton_iters']))} (oracle {int(np.sum(ref['newton_iters']))}) "
      f"mismatching instances {bad}", flush=True)
if bad["x"]:
    i = int(np.nonzero(~(np.asarray(got["x"]) == ref["x"]).all(1))[0][0])
    print("  instance", i, "x gpu", got["x"][i][:6], "oracle", ref["x"][i][:6], flush=True)
