"""Timing-only A/B of the C4 kernel: generated eval 1×/2×/4× per Newton step, LU twice (lu2),
Schur-complement formation twice (s2).  Results must stay identical; only the time moves.

The variants are throwaway copies of the generated module / csrc/ipm_nl_kernel.hpp with
one phase repeated behind empty asm barriers, built next to this file with the
module build flags of mcp_amd/codegen.py (not kept in the tree).  Output:
profiles/r01/ab_c4_phase_costs.txt."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from mcp_amd import _abi
from mcp_amd.batch import Module, alloc_device_outputs, solve_batch_device
from mcp_amd.lane_change import LaneChangeGame

g = LaneChangeGame(2); mcp = g.mcp; n, m = mcp.unconstrained_dimension, mcp.constrained_dimension
rng = np.random.default_rng(np.random.SeedSequence(1, spawn_key=(0,)))
th = torch.from_numpy(np.ascontiguousarray(mcp.theta_map(g.generate_random_parameter(rng, 1024)))).cuda()
here = os.path.dirname(os.path.abspath(__file__))
mods = {"x1": mcp.module(), "x2": Module(os.path.join(here, "eval_x2.hsaco")), "x4": Module(os.path.join(here, "eval_x4.hsaco")),
        "lu2": Module(os.path.join(here, "lu2.hsaco")), "s2": Module(os.path.join(here, "s2.hsaco")),
        "su2": Module(os.path.join(here, "su2.hsaco")), "su5": Module(os.path.join(here, "su5.hsaco"))}
ref = None
for name, mod in mods.items():
    for B in (1, 1024):
        t = th[:B].contiguous()
        out = alloc_device_outputs(B, n, m, t.device)
        run = lambda: solve_batch_device(_abi.FAMILY_NONLINEAR, n, m, t, out, tol=1e-6, linear_solver="schur", module=mod)
        run(); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); run(); run(); run(); e1.record(); torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 3
        nw = out["newton_iters"].cpu().numpy()
        same = ""
        if B == 1024:
            if ref is None:
                ref = out["x"].clone()
            same = f"x identical to x1: {torch.equal(ref, out['x'])}"
        print(f"{name} B={B} ms={ms:.3f} newton max={nw.max()} us/step={ms * 1e3 / nw.max():.2f} {same}", flush=True)
