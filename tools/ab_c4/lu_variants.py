"""Timing-only A/B of the LU inside the C4 kernel (mcpx_nl_solve_schur, lane change T=2).

build (CPU):  python tools/ab_c4/lu_variants.py build   -> tools/abx/lu_<name>.hsaco
run (GPU):    python tools/ab_c4/lu_variants.py run     -> one line per variant
Variants are the product module's generated text compiled with -D knobs of
csrc/ipm_kernel_impl.hpp (MCPX_LU_NO_SPEC: pivot search at every step instead of
the previous Newton step's pivots).  x must stay identical across variants; only
time moves.  Results, with the variants measured and dropped since (8-column
broadcast groups, division behind the first broadcast, pivot row through LDS):
profiles/r02/ab_c4_lu_variants.txt."""
import os, subprocess, sys
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tools", "abx")
VARIANTS = {
    "base": [],
    "nospec": ["-DMCPX_LU_NO_SPEC=1"],
}


def build():
    from mcp_amd import codegen
    from mcp_amd.lane_change import LaneChangeGame
    nl = LaneChangeGame(2).mcp.nl
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(OUT, "lu_t2.hip")
    open(src, "w").write(nl.hip_source())
    procs = []
    for name, flags in VARIANTS.items():
        cmd = [codegen.HIPCC, *codegen._MODULE_FLAGS, *flags, "-I", codegen.CSRC, "-o",
               os.path.join(OUT, f"lu_{name}.hsaco"), src]
        procs.append((name, subprocess.Popen(cmd)))
    for name, p in procs:
        if p.wait() != 0:
            raise SystemExit(f"build of {name} failed")


def run():
    import torch
    from mcp_amd import _abi
    from mcp_amd.batch import Module, alloc_device_outputs, solve_batch_device
    from mcp_amd.lane_change import LaneChangeGame
    from mcp_amd.qp_benchmark import chunked_slice
    g = LaneChangeGame(2); mcp = g.mcp; n, m = mcp.unconstrained_dimension, mcp.constrained_dimension
    th_all = torch.from_numpy(np.ascontiguousarray(mcp.theta_map(
        chunked_slice(lambda rng, k: g.generate_random_parameter(rng, k), 1, 0, 8192)))).cuda()
    ref = {}
    for name in VARIANTS:
        mod = Module(os.path.join(OUT, f"lu_{name}.hsaco"))
        for B in (1024, 8192):
            t = th_all[:B].contiguous()
            out = alloc_device_outputs(B, n, m, t.device)
            run1 = lambda: solve_batch_device(_abi.FAMILY_NONLINEAR, n, m, t, out, tol=1e-6, linear_solver="schur",
                                              module=mod)
            run1(); torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(); run1(); run1(); run1(); e1.record(); torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 3
            x = out["x"].clone()
            same = torch.equal(ref.setdefault(B, x), x)
            print(f"{name:12s} B={B:5d} ms={ms:8.3f} solves/s={B / ms * 1e3:10.0f} x identical to base: {same}",
                  flush=True)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
