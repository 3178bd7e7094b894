"""C4 diagnostic: lane-change T=2 on the one-wave kernel vs the workgroup-per-instance
kernel, whole batch and the failing (931-step) games alone."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mcp_amd import _abi
from mcp_amd.batch import alloc_device_outputs, solve_batch_device
from mcp_amd.lane_change import LaneChangeGame

T = int(sys.argv[1]) if len(sys.argv) > 1 else 2
g = LaneChangeGame(T); mcp = g.mcp; n, m = mcp.unconstrained_dimension, mcp.constrained_dimension
rng = np.random.default_rng(np.random.SeedSequence(1, spawn_key=(0,)))
th = torch.from_numpy(np.ascontiguousarray(mcp.theta_map(g.generate_random_parameter(rng, 1024)))).cuda()
mod = mcp.module()
out0 = None
for sel in [None, "failed"]:
    for kern in ["wave", "workgroup"]:
        t = th
        if sel == "failed":
            t = th[torch.nonzero(out0["status"] != 0).flatten()].contiguous()
        out = alloc_device_outputs(t.shape[0], n, m, t.device)
        run = lambda: solve_batch_device(_abi.FAMILY_NONLINEAR, n, m, t, out, tol=1e-6, linear_solver="schur",
                                         module=mod, kernel=kern)
        run(); torch.cuda.synchronize()
        ms = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(); run(); e1.record(); torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        nw = out["newton_iters"].cpu().numpy()
        if sel is None and kern == "wave":
            out0 = out
        print(f"T={T} B={t.shape[0]} sel={sel} kernel={kern} ms={np.median(ms):.3f} newton mean={nw.mean():.1f} "
              f"max={nw.max()} us/step(max)={np.median(ms) * 1e3 / nw.max():.2f} "
              f"failed={(out['status'] != 0).sum().item()}", flush=True)
