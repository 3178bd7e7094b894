"""A/B of generated-module kernel variants on the lane-change game (BASELINE C4).

    python tests/ab/ab_module.py build NAME CSRC_DIR [T]   # CPU: module text of T (default 2) + CSRC_DIR headers
    python tests/ab/ab_module.py run NAME... [--T T] [--B B]  # GPU: time each, compare with the oracle

Variants are throwaway code objects under tools/abx/ or $MCPX_AB_OUT (not kept in the tree); the
generated text is the product's (mcp_amd/codegen.py), only the kernel headers differ."""
import os, subprocess, sys, time
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
OUT = os.environ.get("MCPX_AB_OUT", os.path.join(ROOT, "tools", "abx"))


def build(name, csrc, T=2):
    from mcp_amd import codegen
    from mcp_amd.lane_change import LaneChangeGame

    g = LaneChangeGame(T)
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(OUT, f"{name}_t{T}.hip")
    with open(src, "w") as f:
        f.write(g.mcp.nl.hip_source())
    cmd = [codegen.HIPCC, *codegen._MODULE_FLAGS, "-I", csrc, "-o", os.path.join(OUT, f"{name}_t{T}.hsaco"), src]
    subprocess.run(cmd, check=True)


def run(names, T=2, B=1024, reps=3):
    import torch

    from mcp_amd import _abi
    from mcp_amd.batch import Module, alloc_device_outputs, solve_batch_device
    from mcp_amd.lane_change import LaneChangeGame
    from mcp_amd.qp_benchmark import chunked_slice
    from oracle import coracle

    g = LaneChangeGame(T)
    mcp = g.mcp
    n, m = mcp.unconstrained_dimension, mcp.constrained_dimension
    thh = np.ascontiguousarray(mcp.theta_map(chunked_slice(lambda rng, k: g.generate_random_parameter(rng, k), 1, 0, B)))
    t0 = time.time()
    ref = coracle.solve_batch_nl(mcp.nl, thh, tol=1e-6, linear_solver="schur", nthreads=16)
    print(f"oracle {time.time() - t0:.1f}s", flush=True)
    th = torch.from_numpy(thh).cuda()
    for name in names:
        mod = Module(os.path.join(OUT, f"{name}_t{T}.hsaco")) if name != "product" else mcp.module()
        out = alloc_device_outputs(B, n, m, th.device)
        f = lambda: solve_batch_device(_abi.FAMILY_NONLINEAR, n, m, th, out, tol=1e-6, linear_solver="schur", module=mod)
        f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        nw = out["newton_iters"].cpu().numpy()
        same = {k: bool(np.array_equal(out[k].cpu().numpy(), ref[k])) for k in ("x", "y", "s", "status", "newton_iters",
                                                                                 "kkt_error", "eps")}
        print(f"{name:12s} T={T} B={B} ms={ms:8.3f} solves/s={B / ms * 1e3:9.0f} newton max={nw.max()} "
              f"us/step(max)={ms * 1e3 / nw.max():.2f} oracle-identical={all(same.values())} {'' if all(same.values()) else same}",
              flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2], sys.argv[3], int(sys.argv[4]) if len(sys.argv) > 4 else 2)
    else:
        args = sys.argv[2:]
        T = int(args[args.index("--T") + 1]) if "--T" in args else 2
        B = int(args[args.index("--B") + 1]) if "--B" in args else 1024
        names = [a for i, a in enumerate(args) if not a.startswith("--") and (i == 0 or args[i - 1] not in ("--T", "--B"))]
        run(names, T, B)
