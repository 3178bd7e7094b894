"""Host-buffer API (mcpx_solve_batch) timing at C3: pageable vs page-locked θ, fresh vs reused
(pre-touched) result buffers, per θ-buffer count and chunk size (MCPX_HOST_BUFFERS /
MCPX_HOST_CHUNK are read per call).  One JSON line per variant; median of 5 after a warm-up."""
import json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mcp_amd.batch import solve_batch, pinned, alloc_host_outputs
from mcp_amd.qp_benchmark import generate_global_slice

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
th = generate_global_slice(1, 32, 16, 0.0, 0, B)
out = alloc_host_outputs(B, 32, 16)
def runs(reuse, k=5):
    solve_batch(0, 32, 16, th[:1024], tol=1e-6, linear_solver="schur", num_devices=1)
    r = []
    for _ in range(k):
        t = time.perf_counter()
        solve_batch(0, 32, 16, th, tol=1e-6, linear_solver="schur", num_devices=1, out=out if reuse else None)
        r.append(time.perf_counter() - t)
    return float(np.median(r)) * 1e3
for S, CH in ((2, 8192), (3, 8192), (4, 8192), (3, 4096), (3, 16384)):
    os.environ["MCPX_HOST_BUFFERS"] = str(S)
    os.environ["MCPX_HOST_CHUNK"] = str(CH)
    rec = {"buffers": S, "chunk": CH, "pageable_fresh_ms": runs(False), "pageable_reused_ms": runs(True)}
    with pinned(th):
        rec["registered_reused_ms"] = runs(True)
    rec["best_solves_per_s"] = B / (min(v for k, v in rec.items() if k.endswith("_ms")) * 1e-3)
    print(json.dumps(rec), flush=True)
