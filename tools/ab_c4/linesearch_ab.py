import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from mcp_amd import _abi
from mcp_amd.batch import Module, alloc_device_outputs, solve_batch_device
from mcp_amd.lane_change import LaneChangeGame
from mcp_amd.qp_benchmark import chunked_slice
g = LaneChangeGame(2); mcp = g.mcp; n, m = mcp.unconstrained_dimension, mcp.constrained_dimension
th = torch.from_numpy(np.ascontiguousarray(mcp.theta_map(chunked_slice(lambda rng, k: g.generate_random_parameter(rng, k), 1, 0, 8192)))).cuda()
ref = {}
for rnd in range(2):
    for name in ("ls_old", "ls_new"):
        mod = Module(os.path.join(ROOT, "tools", "abx", name + ".hsaco"))
        for B in (1024, 8192):
            t = th[:B].contiguous(); out = alloc_device_outputs(B, n, m, t.device)
            run = lambda: solve_batch_device(_abi.FAMILY_NONLINEAR, n, m, t, out, tol=1e-6, linear_solver="schur", module=mod)
            run(); torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(); run(); run(); run(); e1.record(); torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 3
            x = torch.cat([out["x"], out["y"], out["s"]], 1).clone()
            same = torch.equal(ref.setdefault(B, x), x) and True
            print(f"{name} B={B} ms={ms:.3f} solves/s={B / ms * 1e3:.0f} identical={same}", flush=True)
