"""GPU vs oracle on a small C3/C2 SCHUR batch, per-field mismatch counts (diagnostic):
    MCPX_LIB_PATH=... python tools/parity_probe.py [n m B]"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mcp_amd.batch import solve_batch
from mcp_amd.qp_benchmark import generate_random_parameter
from oracle import coracle

n, m, B = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (32, 16, 256)))
th = generate_random_parameter(np.random.default_rng(3), n, m, 0.0, batch=B)
got = solve_batch(0, n, m, th, tol=1e-6, linear_solver="schur", trace_len=64)
ref = coracle.solve_batch(0, n, m, th, tol=1e-6, linear_solver="schur", trace_len=64, nthreads=8)
lib = os.path.basename(os.environ.get("MCPX_LIB_PATH", "default"))
for k in ("x", "y", "s", "kkt_error", "eps", "outer_iters", "status", "newton_iters", "alpha_trace"):
    g, r = np.asarray(got[k]), np.asarray(ref[k])
    same = (g == r) | (np.isnan(g) & np.isnan(r)) if g.dtype.kind == "f" else (g == r)
    bad = ~same.reshape(B, -1).all(1)
    print(lib, n, m, k, int(bad.sum()), (np.nonzero(bad)[0][:5]).tolist(), flush=True)
i = int(np.nonzero(~(np.asarray(got["x"]) == ref["x"]).all(1))[0][0]) if (~(np.asarray(got["x"]) == ref["x"]).all(1)).any() else -1
if i >= 0:
    print("instance", i, "newton gpu/oracle", got["newton_iters"][i], ref["newton_iters"][i])
    print("trace gpu", got["alpha_trace"][i][:8].tolist(), "oracle", ref["alpha_trace"][i][:8].tolist())
    print("x gpu", got["x"][i][:4], "oracle", ref["x"][i][:4])
