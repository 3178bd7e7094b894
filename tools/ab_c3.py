"""Timing A/B of alternative libmcpx.so builds (MCPX_LIB_PATH) on QP batches, one process per
library: kernel ms per batched solve (HIP events, median of --reps) and a digest of every
output, so a variant that changes any bit shows a different digest.

    MCPX_LIB_PATH=tools/exp/libX.so python tools/ab_c3.py --batch 65536 8192 [--n 32 --m 16]
"""
import argparse, hashlib, json, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mcp_amd.batch import solve_batch_device, alloc_device_outputs
from mcp_amd.qp_benchmark import generate_global_slice

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, nargs="+", default=[65536, 8192])
ap.add_argument("--n", type=int, default=32)
ap.add_argument("--m", type=int, default=16)
ap.add_argument("--solver", default="schur")
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--family", default="qp", choices=["qp", "affine"], help="affine: the QPs as affine-family data")
a = ap.parse_args()
lib = os.environ.get("MCPX_LIB_PATH", "default")
for B in a.batch:
    fam = 1 if a.family == "affine" else 0
    thh = generate_global_slice(1, a.n, a.m, 0.0, 0, B)
    if fam:
        from mcp_amd.qp_benchmark import affine_embedding
        thh = affine_embedding(thh, a.n, a.m)
    th = torch.from_numpy(thh).cuda()
    out = alloc_device_outputs(B, a.n, a.m, th.device)
    run = lambda: solve_batch_device(fam, a.n, a.m, th, out, tol=1e-6, linear_solver=a.solver)
    run(); torch.cuda.synchronize()
    ms = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); run(); e1.record(); torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    h = hashlib.sha256()
    for k in sorted(out):
        if out[k] is not None:
            h.update(out[k].cpu().numpy().tobytes())
    print(json.dumps({"lib": os.path.basename(lib), "family": a.family, "B": B, "ms_median": float(np.median(ms)), "ms_min": min(ms),
                      "solves_per_s": B / (np.median(ms) * 1e-3), "digest": h.hexdigest()[:16]}), flush=True)
