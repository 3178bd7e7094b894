"""Benchmark: batched interior-point MCP solves on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--n 32 --m 16]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

A "step" is one full batched solve (src/solver.jl:35-122 for every instance:
ϵ-continuation, Newton steps, LU, line search) of B random dense QP-KKT
instances per GPU (benchmark/quadratic_program_benchmark.jl family, fp64,
tol = 1e-6 as benchmark/path.jl:8), θ generated on the host (numpy PCG64,
documented seed) and uploaded before the timed region, so it is
resident in HBM when timing starts; with N > 1
ranks each rank solves its own shard (weak scaling: B instances per GPU) and
the packed per-instance results are all-gathered over RCCL (north_star:
collective only for solution collection).  Rank 0 prints one JSON line.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "MCP solves/sec (batched QP-KKT, n=64) at 1/2/4/8 GPUs; % LU roofline"
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector = FP64 matrix peak (AMD datasheet)
# rocprofv3 PMC pass of this same bench command (tools/gpu_profile.sh), per kernel dispatch
PMC_SUMMARY = os.path.join(ROOT, "profiles", "r01", "pmc_c3_schur.json")


def pmc_traffic(n: int, m: int, B: int, ls: str):
    """HBM-side bytes per launch from the committed PMC summary when it was taken on
    this exact configuration: (FETCH_SIZE + WRITE_SIZE) KB × 1024.  FETCH_SIZE counts
    L2 misses served by the Infinity Cache too (MI355X_MICROARCH.md, HBM section)."""
    try:
        d = json.load(open(PMC_SUMMARY))
    except (OSError, ValueError):
        return None, None
    want = {"schur": 2, "reduced": 0, "dense": 1}[ls]
    k = d.get("kernel", "")
    if int(d.get("Grid_Size", 0)) != 64 * B or f", 0, {n}, {m}, {want}" not in k:
        return None, None
    return (d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024.0, os.path.relpath(PMC_SUMMARY, ROOT)


def lu_flops(N: int) -> float:
    """FLOPs of one dense LU with partial pivoting + the two triangular solves of an
    N-dim system: 2N³/3 + 2N²."""
    return 2.0 * N ** 3 / 3.0 + 2.0 * N ** 2


def solve_dim(n: int, m: int, linear_solver: str) -> int:
    """Dimension of the system the kernel LU-factors per Newton step: n + m after the
    exact slack elimination (reduced), n + 2m for the full dense LU, n for the
    Schur complement."""
    return {"reduced": n + m, "dense": n + 2 * m, "schur": n}[linear_solver]


def executed_flops(n: int, m: int, linear_solver: str) -> float:
    """FLOPs the kernel actually spends on the Newton linear solve per step: the LU of
    the factored system, plus the Schur-complement GEMM (2n²m, fp64 MFMA) for schur."""
    f = lu_flops(solve_dim(n, m, linear_solver))
    return f + (2.0 * n * n * m if linear_solver == "schur" else 0.0)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=65536, help="instances per GPU")
    ap.add_argument("--n", type=int, default=32)
    ap.add_argument("--m", type=int, default=16)
    ap.add_argument("--tol", type=float, default=1e-6)
    ap.add_argument("--sparsity", type=float, default=0.0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--linear-solver", default="schur", choices=["reduced", "dense", "schur"])
    ap.add_argument("--cpu-sample", type=int, default=32768, help="instances in the CPU-baseline sample (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, cpu_count)")
    ap.add_argument("--sens", action="store_true",
                    help="BASELINE C5: each step is the batched solve + the rrule pullback (VJP kernel) of "
                         "f = Σx² + Σy² (src/AutoDiff.jl:42-82, test/runtests.jl:72-75)")
    ap.add_argument("--gather", action="store_true",
                    help="run the RCCL result collection even at world size 1 (rehearsal under torchrun)")
    ap.add_argument("--lane-change", type=int, default=0, metavar="T",
                    help="BASELINE C4: each step solves --batch lane-change games of horizon T (generated "
                         "nonlinear module; examples/lane_change.jl, benchmark/trajectory_game_benchmark.jl)")
    return ap.parse_args()


def main_lane_change(a):
    """BASELINE C4: B lane-change trajectory games (θ from the sampler of
    benchmark/trajectory_game_benchmark.jl:62-87) solved per step by the generated
    nonlinear module, x₀ = y₀ = s₀ defaults and tol as benchmark/path.jl:8,67-84.
    Instances shard over ranks (weak scaling); no collective on the data path."""
    import torch
    import torch.distributed as dist

    from mcp_amd import _abi
    from mcp_amd.batch import alloc_device_outputs, solve_batch_device
    from mcp_amd.lane_change import LaneChangeGame

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("NCCL_DEBUG", "WARN")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    game = LaneChangeGame(a.lane_change)
    mcp = game.mcp
    n, m, B = mcp.unconstrained_dimension, mcp.constrained_dimension, a.batch
    N = n + 2 * m
    module = mcp.module()
    rng = np.random.default_rng(np.random.SeedSequence(a.seed, spawn_key=(rank,)))
    theta_host = np.ascontiguousarray(mcp.theta_map(game.generate_random_parameter(rng, B)))
    theta = torch.from_numpy(theta_host).to(dev)
    out = alloc_device_outputs(B, n, m, dev)
    stream = torch.cuda.current_stream(dev)
    ls = mcp.nl.default_solver()

    def step():
        solve_batch_device(_abi.FAMILY_NONLINEAR, n, m, theta, out, tol=a.tol, linear_solver=ls, stream=stream,
                           module=module)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(a.steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
    newton = out["newton_iters"].to(torch.float64).sum().item()
    solved = (out["status"] == 0).to(torch.float64).mean().item()
    if world > 1:
        t = torch.tensor([elapsed, kern_ms, newton, solved], dtype=torch.float64, device=dev)
        t2 = t.clone()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(t2, op=dist.ReduceOp.SUM)
        elapsed, kern_ms, newton, solved = float(t[0]), float(t[1]), float(t2[2]), float(t2[3]) / world
    if rank == 0:
        flops_launch = newton / world * lu_flops(N)
        achieved = flops_launch / (kern_ms * 1e-3) / 1e12
        traffic, traffic_src = None, None
        pmc_path = os.path.join(ROOT, "profiles", "r01", "pmc_c4_lane.json")
        try:  # tools/gpu_c4_pmc.sh on this exact configuration: (FETCH_SIZE + WRITE_SIZE) KB per launch
            d = json.load(open(pmc_path))
            if d.get("kernel") == "mcpx_nl_solve_" + ls and int(d.get("Grid_Size", 0)) == 64 * B \
                    and a.lane_change == 2:
                traffic, traffic_src = (d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024.0, os.path.relpath(pmc_path, ROOT)
        except (OSError, ValueError, KeyError):
            pass
        res = {
            "metric": "MCP solves/sec (lane-change trajectory game, generated nonlinear module)",
            "value": a.steps * B * world / elapsed, "unit": "solves/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic θ (benchmark/trajectory_game_benchmark.jl:62-87 sampler, numpy PCG64 "
                    f"SeedSequence({a.seed}, spawn_key=(rank,))), uploaded to HBM before timing",
            "config": {"workload": f"BASELINE C4: 2-player lane-change game T={a.lane_change} "
                                   f"(n={n}, m={m}, KKT dim {N}), fp64, {B} games per GPU, tol={a.tol:g}",
                       "n": n, "m": m, "kkt_dim": N, "linear_solver": ls, "batch_per_gpu": B,
                       "global_batch": B * world, "parallelism": f"dp{world} (instance shards)"},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "mcpx_nl_solve_" + ls,
                         "kernel_ms": kern_ms, "flops_per_launch": flops_launch,
                         "note": f"SURVEY.md §8(d) algorithmic FLOPs: dense LU of the N={N} KKT system per "
                                 "Newton step x the run's own Newton counts / HIP-event kernel time"},
            "newton_iters_mean": newton / (B * world), "success_rate": solved,
        }
        if world == 1 and a.cpu_sample > 0:
            from oracle import coracle

            coracle.build()
            th = int(a.cpu_threads) or min(16, os.cpu_count() or 1)
            S = min(a.cpu_sample, B)
            t1 = time.perf_counter()
            r = coracle.solve_batch_nl(mcp.nl, theta_host[:S], tol=a.tol, linear_solver=ls, nthreads=th)
            dt = time.perf_counter() - t1
            res["cpu_baseline"] = dict(value=S / dt, unit="solves/s", cores=th, kind="port",
                                       sample=f"first {S} games of rank 0, C oracle with the generated host "
                                              f"G/H code, {th} threads, {dt:.2f} s wall",
                                       status_match=bool(np.array_equal(r["status"],
                                                                        out["status"][:S].cpu().numpy())))
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(theta_host: np.ndarray, n: int, m: int, tol: float, threads: int, ls: str) -> dict:
    """Times the C oracle (oracle/ipm_oracle.c, same algorithm) on host cores."""
    from oracle import coracle

    coracle.build()
    coracle.solve_batch(0, n, m, theta_host[: min(64, len(theta_host))], tol=tol, nthreads=threads,
                        linear_solver=ls)  # warm
    t0 = time.perf_counter()
    r = coracle.solve_batch(0, n, m, theta_host, tol=tol, nthreads=threads, linear_solver=ls)
    dt = time.perf_counter() - t0
    model = ""
    try:
        model = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    return dict(value=len(theta_host) / dt, unit="solves/s", cores=threads, kind="port",
                host_cpu=model, host_nproc=os.cpu_count(),
                sample=f"{len(theta_host)} instances of the same workload (first {len(theta_host)} θ of rank 0), "
                       f"C oracle (oracle/ipm_oracle.c, same algorithm and linear solver) on {threads} host threads, "
                       f"{dt:.2f} s wall = {dt * threads:.1f} thread-s",
                newton_mean=float(r["newton_iters"].mean()))


def main():
    a = parse()
    if a.lane_change:
        return main_lane_change(a)
    import torch
    import torch.distributed as dist

    from mcp_amd.batch import solve_batch_device
    from mcp_amd.distributed import Gatherer, alloc_packed
    from mcp_amd.batch import solve_batch
    from mcp_amd.qp_benchmark import generate_random_parameter

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1 or (a.gather and "RANK" in os.environ)
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("NCCL_DEBUG", "WARN")  # keep RCCL's banner off stdout (one JSON line)
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    n, m, B = a.n, a.m, a.batch
    N = n + 2 * m

    # host RNG, one independent stream per rank (SeedSequence(seed, spawn_key=(rank,))), uploaded once
    rng = np.random.default_rng(np.random.SeedSequence(a.seed, spawn_key=(rank,)))
    theta_host = generate_random_parameter(rng, n, m, a.sparsity, batch=B)
    theta = torch.from_numpy(theta_host).to(dev)
    # outputs written straight into one packed fp64 record buffer + one int32 buffer
    # (x | y | s | kkt | ϵ and outer | status | newton), so the collection is 2 all-gathers
    packed = alloc_packed(B, n, m, dev)
    out = packed.views()
    gather = Gatherer(packed) if distributed else None

    stream = torch.cuda.current_stream(dev)

    if a.sens:
        from mcp_amd.batch import vjp_batch_device

        p = theta.shape[1]
        dtheta = torch.empty(B, p, dtype=torch.float64, device=dev)
        vstat = torch.empty(B, dtype=torch.int32, device=dev)
        zeros_m = torch.zeros(B, m, dtype=torch.float64, device=dev)
        gx = torch.empty(B, n, dtype=torch.float64, device=dev)
        gy = torch.empty(B, m, dtype=torch.float64, device=dev)

    def pullback():
        # cotangent of f = Σx² + Σy² (test/runtests.jl:72-75): ∂x = 2x, ∂y = 2y, ∂s = 0
        torch.mul(out["x"], 2.0, out=gx)
        torch.mul(out["y"], 2.0, out=gy)
        vjp_batch_device(0, n, m, theta, out["x"], out["y"], out["s"], gx, gy, zeros_m, dtheta, vstat,
                         stream=stream)

    def step():
        solve_batch_device(0, n, m, theta, out, tol=a.tol, linear_solver=a.linear_solver, stream=stream)
        if a.sens:
            pullback()
        if gather is not None:
            gather()

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(a.steps):
        ev[i][0].record(stream)
        solve_batch_device(0, n, m, theta, out, tol=a.tol, linear_solver=a.linear_solver, stream=stream)
        ev[i][1].record(stream)
        if a.sens:
            evs[i][0].record(stream)
            pullback()
            evs[i][1].record(stream)
        if gather is not None:
            gather()
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
    vjp_ms = float(np.mean([s.elapsed_time(e) for s, e in evs])) if a.sens else None
    # PCIe-inclusive rate of the host-buffer API (mcpx_solve_batch: H→D θ, solve, D→H
    # results) — reported beside `value`, never as it
    host_rate = None
    if world == 1:
        solve_batch(0, n, m, theta_host[:1024], tol=a.tol, linear_solver=a.linear_solver, num_devices=1)
        t1 = time.perf_counter()
        solve_batch(0, n, m, theta_host, tol=a.tol, linear_solver=a.linear_solver, num_devices=1)
        host_rate = B / (time.perf_counter() - t1)
    newton = out["newton_iters"].to(torch.float64).sum().item()
    solved = (out["status"] == 0).to(torch.float64).mean().item()
    if distributed:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
        s = torch.tensor([newton, solved], dtype=torch.float64, device=dev)
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        newton, solved = float(s[0]), float(s[1]) / world

    if rank == 0:
        NS = solve_dim(n, m, a.linear_solver)
        # algorithmic FLOPs per Newton step = dense LU of the N = n+2m
        # KKT system, 2N³/3 + 2N², × the run's own Newton counts, per launch (per GPU)
        flops_launch = newton / world * lu_flops(N)
        traffic, traffic_src = pmc_traffic(n, m, B, a.linear_solver)
        achieved = flops_launch / (kern_ms * 1e-3) / 1e12
        executed = newton / world * executed_flops(n, m, a.linear_solver) / (kern_ms * 1e-3) / 1e12
        res = {
            "metric": METRIC,
            "value": a.steps * B * world / elapsed,
            "unit": "solves/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (random dense QPs of benchmark/quadratic_program_benchmark.jl, host numpy PCG64 "
                    f"SeedSequence({a.seed}, spawn_key=(rank,)), uploaded to HBM before timing)",
            "config": {"workload": f"BASELINE C3: random dense QP-KKT n={n} m={m} (KKT dim {N}), fp64, "
                                   f"{B} instances per GPU, tol={a.tol:g}",
                       "n": n, "m": m, "kkt_dim": N, "linear_solver": a.linear_solver, "solve_dim": NS,
                       "batch_per_gpu": B, "global_batch": B * world,
                       "sparsity": a.sparsity,
                       "parallelism": f"dp{world} (instance shards, RCCL all-gather of results)" if distributed
                       else "dp1"},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic,
                         "traffic_source": traffic_src,
                         "algorithmic_bytes": B * (8 * (n * n + m * n + m + n) + 8 * (n + 2 * m + 2) + 12),
                         "kernel": "ipm_solve_kernel", "kernel_ms": kern_ms,
                         "flops_per_launch": flops_launch,
                         "executed_tflops": executed, "executed_frac": executed / FP64_PEAK_TFLOPS,
                         "note": f"achieved = SURVEY.md §8(d) algorithmic FLOPs (dense LU of the N={N} KKT "
                                 f"system, 2N^3/3+2N^2 per Newton step) x the run's own Newton counts / "
                                 f"HIP-event kernel time; executed_tflops counts what the kernel really does "
                                 f"({a.linear_solver}: LU of dim {NS}" + (f" + 2n^2m Schur GEMM on fp64 MFMA"
                                 if a.linear_solver == "schur" else "") + "); FP64 vector = matrix peak on MI355X"},
            "newton_iters_mean": newton / (B * world),
            "success_rate": solved,
            "host_api_solves_per_s": host_rate,
        }
        if a.sens:
            p = n * n + m * n + m + n
            vbytes = B * 8 * (2 * p + 3 * N + 2 * N)  # θ read, ∂θ written, (x,y,s) + cotangents read
            vflops = B * lu_flops(N)
            res["config"]["workload"] = (f"BASELINE C5: batched solve + rrule pullback (VJP kernel) of f = Σx²+Σy², "
                                         f"QP-KKT n={n} m={m} (KKT dim {N}), fp64, {B} instances per GPU, tol={a.tol:g}")
            res["sensitivity"] = {
                "vjp_kernel_ms": vjp_ms, "solve_kernel_ms": kern_ms,
                "vjp_per_s": B / (vjp_ms * 1e-3),
                "vjp_failed": int((vstat != 0).sum().item()),
                "vjp_roofline": {"flops_per_launch": vflops, "achieved_tflops": vflops / (vjp_ms * 1e-3) / 1e12,
                                 "frac_fp64": vflops / (vjp_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
                                 "algorithmic_bytes": vbytes, "achieved_gbs": vbytes / (vjp_ms * 1e-3) / 1e9,
                                 "frac_hbm": vbytes / (vjp_ms * 1e-3) / 8.0e12,
                                 "note": "one dense LU of the N-dim ∇F_zᵀ (2N³/3+2N²) per instance; bytes = θ read + "
                                         "∂θ written + z and cotangents"},
            }
        if world == 1 and a.cpu_sample > 0:
            th = int(a.cpu_threads) or min(16, os.cpu_count() or 1)
            res["cpu_baseline"] = cpu_baseline(theta_host[: a.cpu_sample], n, m, a.tol, th, a.linear_solver)
        print(json.dumps(res), flush=True)
    if distributed:
        if a.gather and world == 1:  # rehearsal: the gathered batch must equal the local results
            full = gather.unpack()
            assert all(torch.equal(full[k], packed.views()[k].reshape(full[k].shape)) for k in full)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
