"""Diagnostic builds of the T = 2 lane-change module's band kernel with early exits
(MCPX_BAND_DEBUG_EXIT, csrc/ipm_nl_band.hpp) and their runs.
    python tools/band_debug.py build          (CPU: tools/bandv/band_exit<N>.hsaco, N = 0..4)
    python tools/band_debug.py run N          (GPU: one game through variant N, timed)"""
import os, subprocess, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tools", "bandv")

if sys.argv[1] == "build":
    from mcp_amd import codegen
    from mcp_amd.lane_change import LaneChangeGame

    src = os.path.join(OUT, "t2.hip")
    open(src, "w").write(LaneChangeGame(2).mcp.nl.hip_source())
    procs = []
    for N in range(5):
        cmd = [codegen.HIPCC, *codegen._MODULE_FLAGS, "-I", codegen.CSRC, "-DMCPX_NL_ONLY_BAND",
               f"-DMCPX_BAND_DEBUG_EXIT={N}", "-o", os.path.join(OUT, f"band_exit{N}.hsaco"), src]
        procs.append(subprocess.Popen(cmd))
    sys.exit(max(p.wait() for p in procs))

from mcp_amd import _abi
from mcp_amd.batch import Module, solve_batch
from tests.test_band import _c4

N = int(sys.argv[2])
game, tp = _c4(2, 1)
nl = game.mcp.nl
mod = Module(os.path.join(OUT, f"band_exit{N}.hsaco"))
print(f"variant {N}: loaded", flush=True)
t0 = time.time()
r = solve_batch(_abi.FAMILY_NONLINEAR, nl.n, nl.m, tp, linear_solver="schur", module=mod, kernel="band")
print(f"variant {N}: returned in {time.time() - t0:.3f}s status {r['status']} newton {r['newton_iters']}", flush=True)
