"""Benchmark: batched interior-point MCP solves on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--n 32 --m 16]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

A "step" is one full batched solve (src/solver.jl:35-122 for every instance:
ϵ-continuation, Newton steps, LU, line search) of B random dense QP-KKT
instances per GPU (benchmark/quadratic_program_benchmark.jl family, fp64,
tol = 1e-6 as benchmark/path.jl:8), θ already resident in HBM; with N > 1
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
    return ap.parse_args()


def cpu_baseline(theta_host: np.ndarray, n: int, m: int, tol: float, threads: int, ls: str) -> dict:
    """Times the C oracle (oracle/ipm_oracle.c, same algorithm) on host cores."""
    from oracle import coracle

    coracle.build()
    coracle.solve_batch(0, n, m, theta_host[: min(64, len(theta_host))], tol=tol, nthreads=threads,
                        linear_solver=ls)  # warm
    t0 = time.perf_counter()
    r = coracle.solve_batch(0, n, m, theta_host, tol=tol, nthreads=threads, linear_solver=ls)
    dt = time.perf_counter() - t0
    return dict(value=len(theta_host) / dt, unit="solves/s", cores=threads, kind="port",
                sample=f"{len(theta_host)} instances of the same workload (first {len(theta_host)} θ of rank 0), "
                       f"C oracle (oracle/ipm_oracle.c, same algorithm and linear solver) on {threads} host threads, "
                       f"{dt:.2f} s wall = {dt * threads:.1f} thread-s",
                newton_mean=float(r["newton_iters"].mean()))


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    from mcp_amd.batch import alloc_device_outputs, solve_batch_device
    from mcp_amd.qp_benchmark import generate_random_parameter_torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    n, m, B = a.n, a.m, a.batch
    N = n + 2 * m

    g = torch.Generator(device=dev).manual_seed(a.seed * 1000003 + rank)
    theta = generate_random_parameter_torch(g, n, m, B, sparsity_rate=a.sparsity, device=dev)
    # outputs written straight into one packed fp64 record buffer + one int32 buffer
    # (x | y | s | kkt | ϵ and outer | status | newton), so the collection is 2 all-gathers
    rec = torch.empty(B * (N + 2), dtype=torch.float64, device=dev)
    irec = torch.empty(3 * B, dtype=torch.int32, device=dev)
    out = alloc_device_outputs(B, n, m, dev, newton=True, active=False)
    o = 0
    for k, w in (("x", n), ("y", m), ("s", m), ("kkt_error", 1), ("eps", 1)):
        out[k] = rec[o:o + B * w].view(B, w) if w > 1 else rec[o:o + B]
        o += B * w
    out["outer_iters"], out["status"], out["newton_iters"] = irec[:B], irec[B:2 * B], irec[2 * B:]
    if world > 1:
        grec = torch.empty(world * rec.numel(), dtype=rec.dtype, device=dev)
        girec = torch.empty(world * irec.numel(), dtype=irec.dtype, device=dev)

    stream = torch.cuda.current_stream(dev)

    def step():
        solve_batch_device(0, n, m, theta, out, tol=a.tol, linear_solver=a.linear_solver, stream=stream)
        if world > 1:
            dist.all_gather_into_tensor(grec, rec)
            dist.all_gather_into_tensor(girec, irec)

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
        solve_batch_device(0, n, m, theta, out, tol=a.tol, linear_solver=a.linear_solver, stream=stream)
        ev[i][1].record(stream)
        if world > 1:
            dist.all_gather_into_tensor(grec, rec)
            dist.all_gather_into_tensor(girec, irec)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
    newton = out["newton_iters"].to(torch.float64).sum().item()
    solved = (out["status"] == 0).to(torch.float64).mean().item()
    if world > 1:
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
            "data": "synthetic (random dense QPs of benchmark/quadratic_program_benchmark.jl, torch Philox seed "
                    f"{a.seed}+rank, generated in HBM)",
            "config": {"workload": f"BASELINE C3: random dense QP-KKT n={n} m={m} (KKT dim {N}), fp64, "
                                   f"{B} instances per GPU, tol={a.tol:g}",
                       "n": n, "m": m, "kkt_dim": N, "linear_solver": a.linear_solver, "solve_dim": NS,
                       "batch_per_gpu": B, "global_batch": B * world,
                       "sparsity": a.sparsity,
                       "parallelism": f"dp{world} (instance shards, RCCL all-gather of results)" if world > 1
                       else "dp1"},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / FP64_PEAK_TFLOPS, "traffic": None,
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
        }
        if world == 1 and a.cpu_sample > 0:
            th = int(a.cpu_threads) or min(16, os.cpu_count() or 1)
            res["cpu_baseline"] = cpu_baseline(theta[: a.cpu_sample].cpu().numpy(), n, m, a.tol, th,
                                               a.linear_solver)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
