"""GPU check of the ×5-unrolled C4 Schur formation built from the fixed sources
(tools/ab_c4/su5_fixed.hsaco: the lane-change T=2 module with `#pragma unroll 5`
on the Schur k-loop of csrc/ipm_nl_kernel.hpp, otherwise the tree's sources and
codegen flags).  In r01 this variant returned wrong iterates; with the broadcast
moved out of divergent control flow it must equal the oracle bit for bit.
Prints one JSON line per batch: bit-exactness vs the oracle and the time per
launch next to the shipped ×2 module."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from mcp_amd import _abi  # noqa: E402
from mcp_amd.batch import Module, alloc_device_outputs, solve_batch_device  # noqa: E402
from mcp_amd.lane_change import LaneChangeGame  # noqa: E402
from mcp_amd.qp_benchmark import chunked_slice  # noqa: E402
from oracle import coracle  # noqa: E402

g = LaneChangeGame(2)
mcp = g.mcp
n, m = mcp.unconstrained_dimension, mcp.constrained_dimension
th_host = np.ascontiguousarray(mcp.theta_map(chunked_slice(lambda r, k: g.generate_random_parameter(r, k), 1, 0, 1024)))
mods = {"x2_shipped": mcp.module(), "x5_fixed": Module(os.path.join(ROOT, "tools", "ab_c4", "su5_fixed.hsaco"))}
FIELDS = ("x", "y", "s", "kkt_error", "eps", "outer_iters", "status", "newton_iters")
for B in (1, 1024):
    ref = coracle.solve_batch_nl(mcp.nl, th_host[:B], tol=1e-6, linear_solver="schur", nthreads=16)
    t = torch.from_numpy(th_host[:B]).cuda()
    for name, mod in mods.items():
        out = alloc_device_outputs(B, n, m, t.device)
        run = lambda: solve_batch_device(_abi.FAMILY_NONLINEAR, n, m, t, out, tol=1e-6, linear_solver="schur",
                                         module=mod)
        run()
        torch.cuda.synchronize()
        exact = {k: bool(np.array_equal(out[k].cpu().numpy(), ref[k])) for k in FIELDS}
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            run()
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"variant": name, "B": B, "bit_exact_vs_oracle": all(exact.values()), "fields": exact,
                          "ms_per_launch": e0.elapsed_time(e1) / 3,
                          "newton_max": int(out["newton_iters"].max().item())}), flush=True)
