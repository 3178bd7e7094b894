"""C4 diagnostic: Newton-count distribution and per-step cost of the lane-change kernel."""
import os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mcp_amd import _abi
from mcp_amd.batch import alloc_device_outputs, solve_batch_device
from mcp_amd.lane_change import LaneChangeGame

g = LaneChangeGame(2); mcp = g.mcp; n, m = mcp.unconstrained_dimension, mcp.constrained_dimension
rng = np.random.default_rng(np.random.SeedSequence(1, spawn_key=(0,)))
th = torch.from_numpy(np.ascontiguousarray(mcp.theta_map(g.generate_random_parameter(rng, 1024)))).cuda()
mod = mcp.module()
for B, sel in [(1024, None), (1024, "solved"), (64, "solved"), (1, "solved")]:
    t = th
    if sel == "solved":
        idx = torch.nonzero(out0["status"] == 0).flatten()[:B]
        t = th[idx].contiguous()
    out = alloc_device_outputs(t.shape[0], n, m, t.device)
    run = lambda: solve_batch_device(_abi.FAMILY_NONLINEAR, n, m, t, out, tol=1e-6, linear_solver="schur", module=mod)
    run(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); run(); e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    nw = out["newton_iters"].cpu().numpy()
    if sel is None:
        out0 = out
    print(f"B={t.shape[0]} sel={sel} ms={ms:.3f} newton mean={nw.mean():.1f} max={nw.max()} "
          f"us/step(max)={ms * 1e3 / nw.max():.2f} failed={(out['status'] != 0).sum().item()}", flush=True)
