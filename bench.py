"""Benchmark: batched interior-point MCP solves on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--global-batch G | --batch B] ...
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

A "step" is one full batched solve (src/solver.jl:35-122 for every instance:
ϵ-continuation, Newton steps, linear solve, line search) of random dense QP-KKT
instances (benchmark/quadratic_program_benchmark.jl family, fp64, tol = 1e-6 as
benchmark/path.jl:8).  θ is generated on the host (numpy PCG64 in chunks of
4096 instances, chunk c seeded SeedSequence(seed, spawn_key=(c,)), so instance i
is the same at every GPU count) and uploaded before the timed region, so it is
resident in HBM when timing starts.

Workload (BASELINE.json configs):
  default         C3: global batch 65,536 (n=32, m=16, KKT dim 64), sharded over
                  the N GPUs (strong scaling: 65,536 at N=1, 8,192 per GPU at N=8);
  --batch B       B instances per GPU instead (weak scaling);
  --sens          C5: solve + rrule pullback (VJP kernel), global batch 4,096;
  --lane-change T C4: the lane-change trajectory game, global batch 1,024.
With N > 1 ranks the packed per-instance results are all-gathered over RCCL
inside the timed step (north_star: collective only for solution collection).

`--gpus N` without torchrun's RANK in the environment starts N ranks itself
(torch.distributed.run as a child process, before this process touches the
GPU) and fails if fewer than N GPUs are visible.  Rank 0 prints one JSON line.
"""

from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "MCP solves/sec (batched QP-KKT, n=64) at 1/2/4/8 GPUs; % LU roofline"
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector = FP64 matrix peak (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0
XCDS, SIMDS = 8, 256 * 4  # MI355X: 8 XCDs, 256 CUs × 4 SIMDs
# rocprofv3 evidence of this round's kernels (tools/gpu_profile.sh + tools/prof_summary.py)
PROFILE_DIR = os.environ.get("MCPX_PROFILE_DIR") or os.path.join(ROOT, "profiles", "r06")
DEFAULT_GLOBAL = {"c3": 65536, "c5": 4096, "c4": 1024}
QP_FIELDS = ("x", "y", "s", "kkt_error", "eps", "outer_iters", "status", "newton_iters")
C4_FIELDS = QP_FIELDS


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
    """FP64 FLOPs the QP kernels execute per Newton step (executed roofline):
    the residual F (G rows n·(n+m) fmas, H rows m·n) plus the linear solve —
      dense / reduced: LU with partial pivoting of the N = n+2m / n+m system (2N³/3 + 2N²);
      schur: the Schur complement S = M + tol·I + Aᵀ D⁻¹ A on the matrix cores (2n²·4⌈m/4⌉,
      K padded to the MFMA's 4), rr and δy (2nm each) and the pivot-free Gauss-Jordan
      elimination of the SPD S, every other row updated at every step ((n−1)·n·(n+1)).
    The one-wave kernels run every instance of the bench on these paths (M = PᵀP is
    symmetric, S is SPD)."""
    resid = 2.0 * (n * (n + m) + m * n)
    if linear_solver == "schur":
        return resid + 2.0 * n * n * 4 * ((m + 3) // 4) + 4.0 * n * m + (n - 1.0) * n * (n + 1.0)
    return resid + lu_flops(solve_dim(n, m, linear_solver))


def executed_flops_nl(nl, linear_solver: str, band: bool = False) -> float:
    """Same for a generated nonlinear module: the linear solve only (the generated G/H
    evaluation is not counted) — schur: R·D⁻¹ (m·n products), S from Q's structural
    nonzeros (2n per term), rr and δy over the Q / R patterns, LU of S; with the band kernel
    (csrc/ipm_nl_band.hpp) the LU of S is the band elimination: per step one reciprocal, NS
    multipliers and the NS × WC window update (2 flops each), and the back substitution's WC
    updates per row."""
    n, m = nl.n, nl.m
    if linear_solver != "schur":
        return lu_flops(solve_dim(n, m, linear_solver))
    (qp, qi), (rp, ri) = nl.structure()
    form = m * n + 2.0 * n * len(qi) + 2.0 * len(qi) + 2.0 * len(ri)
    if band:
        b = nl.band
        return form + n * (1.0 + b.ns + 2.0 * b.ns * b.wc + 2.0 * b.wc)
    return form + lu_flops(n)


def band_kernel_runs(nl, linear_solver: str, kernel: str) -> bool:
    """Whether the C ABI runs a module's band SCHUR kernel (mcpx_api.cpp prepare: forced, or
    AUTO when the module prefers it or has no one-wave SCHUR kernel)."""
    return linear_solver == "schur" and nl.band_can and (
        kernel == "band" or (kernel == "auto" and (nl.band_auto or not nl.solvers()["schur"])))


def one_wave(n: int, m: int, linear_solver: str) -> bool:
    """Whether the C ABI's default kernel selector (MCPX_KERNEL_AUTO) runs this QP size on
    the one-wave register kernels (≤ 64 rows) rather than the workgroup-per-instance ones."""
    lanes = n + 2 * m if linear_solver == "dense" else n + m
    return solve_dim(n, m, linear_solver) <= 64 and lanes <= 64


def roofline_bound(ev: dict, kern_ms: float, fallback: str) -> tuple:
    """What limits the kernel, from the committed PMC counters of this configuration and
    build (tools/gpu_profile.sh): the largest of
      hbm  = (FETCH_SIZE + WRITE_SIZE) / kernel time / 8 TB/s,
      mfma = MFMA-busy SIMD-cycles / (active cycles × SIMDs),
      valu = SQ_INSTS_VALU × 4 cycles (a wave64 VALU op, FP64 at full rate) / (active cycles × SIMDs);
    "latency" when none reaches 0.3 (waves stall on dependencies, not on a unit).  Without
    PMC evidence for this build: `fallback`, marked as such."""
    p = ev.get("pmc") or {}
    if not p.get("GRBM_GUI_ACTIVE"):
        return fallback, {"source": "assumed: no PMC summary of this configuration and build"}
    sim_cycles = p["GRBM_GUI_ACTIVE"] / XCDS * SIMDS
    fr = {}
    if "FETCH_SIZE" in p and "WRITE_SIZE" in p:
        fr["hbm"] = (p["FETCH_SIZE"] + p["WRITE_SIZE"]) * 1024.0 / (kern_ms * 1e-3) / (HBM_PEAK_GBS * 1e9)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in p:
        fr["mfma"] = p["SQ_VALU_MFMA_BUSY_CYCLES"] / sim_cycles
    if "SQ_INSTS_VALU" in p:
        fr["valu"] = p["SQ_INSTS_VALU"] * 4.0 / sim_cycles
    best = max(fr, key=fr.get) if fr else fallback
    bound = best if fr and fr[best] >= 0.3 else "latency"
    return bound, {"source": p.get("_source"), "utilisation": fr}


def parity_report(got: dict, ref: dict, fields, count: int, what: str) -> dict:
    """Bit-exact comparison of the GPU outputs of the first `count` instances with the
    oracle's (parity pass/fail in every bench line): per field the
    number of instances with any differing entry (NaN = NaN)."""
    mism = {}
    for f in fields:
        g = np.asarray(got[f])[:count]
        r = np.asarray(ref[f])[:count]
        same = (g == r)
        if np.issubdtype(g.dtype, np.floating):
            same |= np.isnan(g) & np.isnan(r)
        mism[f] = int((~same.reshape(count, -1).all(1)).sum())
    return {"instances": int(count), "bit_exact_fields": [f for f in fields if mism[f] == 0],
            "mismatches": mism, "pass": all(v == 0 for v in mism.values()), "reference": what}


def fixture_parity() -> dict:
    """The committed golden vectors of the QP family (tests/golden/qp_*.npz, readme_qp*.npz:
    inputs and the oracle's outputs, tests/golden/make_golden.py) through the GPU host API,
    bit-exact on every output field."""
    import glob

    from mcp_amd.batch import solve_batch

    files = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "qp_*.npz"))
                   + glob.glob(os.path.join(ROOT, "tests", "golden", "readme_qp*.npz")))
    bad, inst = [], 0
    fields = ("x", "y", "s", "kkt_error", "eps", "outer_iters", "status", "newton_iters")
    for f in files:
        d = np.load(f, allow_pickle=False)
        kw = {k[len("param_"):]: d[k].item() for k in d.files if k.startswith("param_")}
        got = solve_batch(int(d["family"]), int(d["n"]), int(d["m"]), d["theta"], num_devices=1, **kw)
        rep = parity_report(got, {k: d["out_" + k] for k in fields}, fields, d["theta"].shape[0], "")
        inst += rep["instances"]
        if not rep["pass"]:
            bad.append(os.path.basename(f))
    return {"files": len(files), "instances": inst, "failed_files": bad, "pass": not bad and bool(files)}


def host_cpus() -> dict:
    """CPUs this process can actually use: its affinity set, capped by the cgroup CPU
    quota (a GPU box grants 16 of the machine's 256 hardware threads; GNU `nproc`
    prints 16 there too, via OMP_NUM_THREADS), plus the machine total and model."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count() or 1
    info = {"affinity_cpus": affinity, "machine_cpus": os.cpu_count()}
    usable = affinity
    try:
        q = open("/sys/fs/cgroup/cpu.max").read().split()
        if q and q[0] != "max":
            info["cgroup_cpus"] = float(q[0]) / float(q[1])
            usable = max(1, min(usable, int(info["cgroup_cpus"] + 0.999)))
    except (OSError, ValueError, IndexError):
        pass
    info["nproc"] = usable
    try:
        info["model"] = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    return info


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--global-batch", type=int, default=0,
                    help="instances over all GPUs, sharded (strong scaling); 0 = the BASELINE config's")
    ap.add_argument("--batch", type=int, default=0, help="instances per GPU (weak scaling) instead")
    ap.add_argument("--n", type=int, default=32)
    ap.add_argument("--m", type=int, default=16)
    ap.add_argument("--tol", type=float, default=1e-6)
    ap.add_argument("--sparsity", type=float, default=0.0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--linear-solver", default="schur", choices=["reduced", "dense", "schur"])
    ap.add_argument("--family", default="qp", choices=["qp", "affine"],
                    help="affine: the same QPs handed over as affine-family data (P = M, Q = -A^T, R = A, S = 0, "
                         "g = -phi, h = -b), the layout the Julia shim's affine_parameters produces (INTEGRATION.md)")
    ap.add_argument("--cpu-sample", type=int, default=-1,
                    help="instances in the CPU-baseline sample (-1 = 2048 per thread, 0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every CPU this process may use (nproc)")
    ap.add_argument("--host-runs", type=int, default=5, help="timed runs of the host-buffer API (median)")
    ap.add_argument("--sens", action="store_true",
                    help="BASELINE C5: each step is the batched solve + the rrule pullback (VJP kernel) of "
                         "f = Σx² + Σy² (src/AutoDiff.jl:42-82, test/runtests.jl:72-75)")
    ap.add_argument("--unfused", action="store_true",
                    help="with --sens: solve and pullback as two calls (solve, torch cotangent, "
                         "mcpx_vjp_batch_device) instead of mcpx_solve_vjp_batch_device")
    ap.add_argument("--gather", action="store_true",
                    help="run the RCCL result collection even at world size 1 (rehearsal under torchrun)")
    ap.add_argument("--kernel", default="auto", choices=["auto", "wave", "workgroup", "multiwave", "band"],
                    help="with --lane-change: the generated module's kernel (mcpx_params.kernel)")
    ap.add_argument("--lane-change", type=int, default=0, metavar="T",
                    help="BASELINE C4: each step solves lane-change games of horizon T (generated "
                         "nonlinear module; examples/lane_change.jl, benchmark/trajectory_game_benchmark.jl)")
    return ap.parse_args(argv)


def mode_of(a) -> str:
    return "c4" if a.lane_change else ("c5" if a.sens else "c3")


def plan(a, world: int, rank: int) -> dict:
    """This rank's instances: a contiguous shard of the global batch (strong scaling,
    the BASELINE configs) or `--batch` per GPU (weak scaling)."""
    from mcp_amd.distributed import shard_capacity, shard_range

    if a.batch > 0:
        return dict(start=rank * a.batch, count=a.batch, cap=a.batch, global_batch=a.batch * world,
                    scaling="weak")
    G = a.global_batch or DEFAULT_GLOBAL[mode_of(a)]
    start, count = shard_range(G, world, rank)
    return dict(start=start, count=count, cap=shard_capacity(G, world), global_batch=G, scaling="strong")


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(nranks: int, script: str, argv, have_devices: int | None = None) -> int:
    """`--gpus N` outside torchrun: N ranks of `script`, one per GPU, through
    torch.distributed.run started as a child process; this process only counts the
    devices (torch.cuda.device_count does not initialise the GPU) and fails if fewer
    than N are visible.  Returns the child's exit code."""
    if have_devices is None:
        import torch

        have_devices = torch.cuda.device_count()
    if have_devices < nranks:
        print(f"bench.py: --gpus {nranks} but only {have_devices} GPU(s) are visible", file=sys.stderr)
        return 2
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nranks}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), script, *argv]
    return subprocess.call(cmd, env=env)


def evidence(name: str, cfg: dict) -> dict:
    """The committed rocprofv3 summaries of this configuration (profiles/r06/ or MCPX_PROFILE_DIR:
    trace_<name>.json, pmc_<name>.json; tools/prof_summary.py), if they were taken on
    exactly this configuration and this build of libmcpx.so; else {}."""
    from mcp_amd.build import built_hash

    out = {}
    for kind in ("trace", "pmc"):
        path = os.path.join(PROFILE_DIR, f"{kind}_{name}.json")
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if d.get("config") != cfg or d.get("lib_hash") != built_hash():
            continue
        d["_source"] = os.path.relpath(path, ROOT)
        out[kind] = d
    return out


def evidence_id(key: str, cfg: dict) -> dict:
    """What tools/prof_summary.py stamps on the profile summaries of this run."""
    from mcp_amd.build import built_hash

    return {"key": key, "config": cfg, "lib_hash": built_hash()}


def pmc_traffic(ev: dict):
    """HBM-side bytes per launch of the dominant kernel from the PMC summary:
    (FETCH_SIZE + WRITE_SIZE) KB × 1024 (MI355X_MICROARCH.md: FETCH_SIZE also counts
    reads served by the Infinity Cache)."""
    p = ev.get("pmc")
    if not p or "FETCH_SIZE" not in p or "WRITE_SIZE" not in p:
        return None, None
    return (p["FETCH_SIZE"] + p["WRITE_SIZE"]) * 1024.0, p["_source"]


def summary_statistics(step_s, count: int, success_rate: float) -> dict:
    """benchmark/path.jl:101-126 (summary_statistics / runtime_stats / fraction_solved)
    for a batched solver: the reference times each solve alone; a batched step solves
    `count` instances at once, so μ and σ are the per-step device times (HIP events)
    ÷ count (seconds per solve, amortised over the batch) over the timed steps."""
    per = np.asarray(step_s, dtype=np.float64) / max(count, 1)
    return {"ip": {"success_rate": success_rate, "μ": float(per.mean()),
                   "σ": float(per.std(ddof=1)) if len(per) > 1 else 0.0,
                   "unit": "s per solve (step time / instances per GPU)", "steps": len(per)}}


def cpu_baseline(solve, count_avail: int, a, threads_all: int, label: str, per_thread: int = 2048) -> dict:
    """Times the C oracle (the same algorithm as the kernel, oracle/ipm_oracle.c) on
    every CPU this process may use, on a bounded sample of the workload, plus one
    core alone.  `solve(k, threads)` solves the first k instances."""
    solve(min(threads_all, count_avail), threads_all)  # warm: library load, generated code compiled
    S = min(count_avail, a.cpu_sample if a.cpu_sample > 0 else per_thread * threads_all)
    t0 = time.perf_counter()
    r = solve(S, threads_all)
    dt = time.perf_counter() - t0
    S1 = min(count_avail, max(1, S // max(threads_all, 1)))
    t1 = time.perf_counter()
    solve(S1, 1)
    dt1 = time.perf_counter() - t1
    info = host_cpus()
    return dict(value=S / dt, unit="solves/s", cores=threads_all, kind="port",
                single_core_value=S1 / dt1, nproc=info["nproc"], machine_cpus=info["machine_cpus"],
                affinity_cpus=info["affinity_cpus"], host_cpu=info.get("model", ""),
                cgroup_cpus=info.get("cgroup_cpus"),
                sample=f"{S} instances of the same workload (the first {S} of rank 0), {label}, "
                       f"{threads_all} threads = usable CPUs (cgroup quota / affinity), {dt:.2f} s wall; single core: {S1} instances in {dt1:.2f} s",
                _result=r)


def timed_steps(step, a, stream, world, dist, dev, sub_events: int = 1):
    """W untimed warm-up steps, then exactly K steps between barrier + synchronize;
    HIP events around each launch, recorded on the kernels' own stream.  Returns
    (elapsed wall time of the K steps, per-launch ms lists, one per event pair)."""
    import torch

    for _ in range(a.warmup):
        step(None)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    ev = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
          for _ in range(sub_events)]
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(a.steps):
        step([e[i] for e in ev])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    return elapsed, [[s.elapsed_time(e) for s, e in evs] for evs in ev]


def reduce_max_sum(dist, dev, world, maxes, sums):
    import torch

    if world == 1:
        return list(maxes), list(sums)
    t = torch.tensor(list(maxes), dtype=torch.float64, device=dev)
    s = torch.tensor(list(sums), dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    return t.tolist(), s.tolist()


def roofline(kern_ms: float, flops_launch: float, exec_flops_launch: float, alg_bytes: float, ev: dict,
             kernel: str, bound, note: str, structural: bool = False) -> dict:
    """The line's roofline record.  `frac` is SURVEY.md §8(d)'s: the dense-LU FLOPs of the full KKT
    system per Newton step over the kernel time.  A fraction above 1 means that count is not a
    roofline for the kernel (an exact elimination that skips structural zeros — the generated
    modules' band and Schur solves, as the reference's sparse UMFPACK does): `frac` is then the
    structural count (the elimination the kernel performs, `executed`), and the dense figure is
    kept as `frac_dense_kkt` with `dense_count_exceeds_peak`.  `structural` takes that basis
    whatever the dense fraction: the generated modules' lines, whose systems the reference
    factors with a sparse LU (UMFPACK), so the dense count is not their algorithm either.  A
    fraction above 1 on the structural count too is an error in the line (`frac` null, `frac_error`)."""
    achieved = flops_launch / (kern_ms * 1e-3) / 1e12
    executed = exec_flops_launch / (kern_ms * 1e-3) / 1e12
    traffic, traffic_src = pmc_traffic(ev)
    bound, bound_ev = bound
    basis = ("algorithmic: SURVEY.md §8(d) dense-LU FLOPs of the full KKT system (not the FLOPs the "
             "kernel executes: executed_frac)")
    dense_frac = achieved / FP64_PEAK_TFLOPS
    extra = {}
    if dense_frac > 1.0 or structural:
        extra = {"frac_dense_kkt": dense_frac, "dense_count_exceeds_peak": dense_frac > 1.0}
        achieved = executed
        basis = ("structural: the FLOPs of the elimination the kernel performs (" +
                 ("the dense KKT count exceeds the FP64 peak, so it is not a roofline for this kernel"
                  if dense_frac > 1.0 else "a structurally sparse system, factored by the reference with a sparse "
                  "LU: the dense KKT count is not its algorithm") + "; frac_dense_kkt)")
    frac = achieved / FP64_PEAK_TFLOPS
    if frac > 1.0:
        extra["frac_error"] = f"structural FLOPs over the kernel time exceed the FP64 peak ({frac:.3f})"
        frac = None
    r = {"bound": bound, "bound_evidence": bound_ev, "achieved": achieved, "peak": FP64_PEAK_TFLOPS,
         "unit": "TFLOP/s", "frac": frac, "frac_basis": basis, **extra,
         "traffic": traffic, "traffic_source": traffic_src,
         "executed_tflops": executed, "executed_frac": executed / FP64_PEAK_TFLOPS,
         "algorithmic_bytes": alg_bytes, "hbm_gbs_algorithmic": alg_bytes / (kern_ms * 1e-3) / 1e9,
         "kernel": kernel, "kernel_ms": kern_ms, "flops_per_launch": flops_launch,
         "executed_flops_per_launch": exec_flops_launch, "note": note}
    tr = ev.get("trace")
    if tr:
        t_ms = float(tr.get("launch_avg_ms_all_passes", tr["avg_ms"]))
        num = exec_flops_launch if extra else flops_launch
        r.update(trace_kernel_ms=t_ms, frac_trace=num / (t_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
                 executed_frac_trace=exec_flops_launch / (t_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
                 trace_source=tr["_source"])
    if traffic:
        r["traffic_over_algorithmic"] = traffic / alg_bytes
    p = ev.get("pmc") or {}
    if "SQ_VALU_MFMA_BUSY_CYCLES" in p and p.get("GRBM_GUI_ACTIVE"):
        # rocprofv3's MfmaUtil: Σ MFMA-busy SIMD-cycles / (GPU-active cycles × SIMDs); the per-dispatch
        # GRBM_GUI_ACTIVE of the CSV is the sum over the 8 XCDs, hence / 8
        r["mfma_util"] = p["SQ_VALU_MFMA_BUSY_CYCLES"] / (p["GRBM_GUI_ACTIVE"] / XCDS * SIMDS)
        r["mfma_tflops_pmc"] = p.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0) * 512 / (kern_ms * 1e-3) / 1e12
    return r


def main_lane_change(a, world, rank, local, dist, pl):
    """BASELINE C4: lane-change trajectory games (θ from the sampler of
    benchmark/trajectory_game_benchmark.jl:62-87) solved per step by the generated
    nonlinear module, x₀ = y₀ = s₀ defaults and tol as benchmark/path.jl:8,67-84.
    Instances shard over ranks; no collective on the data path."""
    import torch

    from mcp_amd import _abi
    from mcp_amd.batch import alloc_device_outputs, solve_batch_device, vjp_batch_device
    from mcp_amd.lane_change import LaneChangeGame
    from mcp_amd.qp_benchmark import chunked_slice

    dev = torch.device("cuda", local)
    game = LaneChangeGame(a.lane_change)
    mcp = game.mcp
    n, m, B = mcp.unconstrained_dimension, mcp.constrained_dimension, pl["count"]
    N = n + 2 * m
    module = mcp.module()
    theta_host = np.ascontiguousarray(mcp.theta_map(
        chunked_slice(lambda rng, k: game.generate_random_parameter(rng, k), a.seed, pl["start"], B)))
    theta = torch.from_numpy(theta_host).to(dev)
    out = alloc_device_outputs(B, n, m, dev)
    stream = torch.cuda.current_stream(dev)
    ls = mcp.nl.default_solver()

    # --sens: the application's solve + gradient (examples/utils.jl:236-261): Zygote's gradient of
    # x₁ of the game solution w.r.t. θ, i.e. the rrule pullback of the cotangent e₁ on x
    # (src/AutoDiff.jl:42-82) at each game's returned iterate, by mcpx_vjp_batch_module_device
    gx = torch.zeros(B, n, dtype=torch.float64, device=dev)
    gx[:, 0] = 1.0
    dth = torch.empty(B, mcp.nl.p, dtype=torch.float64, device=dev)
    vst = torch.empty(B, dtype=torch.int32, device=dev)

    def step(evs):
        if evs:
            evs[0][0].record(stream)
        solve_batch_device(_abi.FAMILY_NONLINEAR, n, m, theta, out, tol=a.tol, linear_solver=ls, stream=stream,
                           module=module, kernel=a.kernel)
        if evs:
            evs[0][1].record(stream)
        if a.sens:
            if evs:
                evs[1][0].record(stream)
            vjp_batch_device(_abi.FAMILY_NONLINEAR, n, m, theta, out["x"], out["y"], out["s"], gx, None, None,
                             dtheta=dth, status=vst, stream=stream, module=module)
            if evs:
                evs[1][1].record(stream)

    elapsed, ms = timed_steps(step, a, stream, world, dist, dev, 2 if a.sens else 1)
    kern_ms = float(np.mean(ms[0]))
    vjp_ms = float(np.mean(ms[1])) if a.sens else 0.0
    step_s = [t * 1e-3 for t in ms[0]]
    newton = out["newton_iters"].to(torch.float64).sum().item()
    solved = (out["status"] == 0).to(torch.float64).sum().item()
    (elapsed, kern_ms), (newton_all, solved_all) = reduce_max_sum(dist, dev, world, [elapsed, kern_ms],
                                                                  [newton, solved])
    if rank != 0:
        return
    # the generated module's content hash (its kernel headers included) keys the evidence too:
    # the nonlinear kernels live in the module, not in libmcpx.so
    cfg = {"mode": "c4s" if a.sens else "c4", "horizon": a.lane_change, "batch_per_gpu": B, "linear_solver": ls,
           "module": mcp.nl.module_key(), "kernel": a.kernel}
    key = f"c4{'s' if a.sens else ''}_lane_t{a.lane_change}_b{B}"
    ev = evidence(key, cfg)
    mw = ls == "schur" and a.kernel == "multiwave" and module.has_schur_mw
    bandk = band_kernel_runs(mcp.nl, ls, a.kernel)
    kernel = "mcpx_nl_solve_band" if bandk else "mcpx_nl_solve_" + ls + (
        "_mw" if mw else ("" if mcp.nl.solvers()[ls] and a.kernel != "workgroup" else "_wg"))
    rl = roofline(kern_ms, newton * lu_flops(N), newton * executed_flops_nl(mcp.nl, ls, bandk),
                  B * 8.0 * (mcp.nl.p + n + 2 * m + 2) + 12.0 * B, ev, kernel, roofline_bound(ev, kern_ms, "latency"),
                  f"achieved = SURVEY.md §8(d) algorithmic FLOPs (dense LU of the N={N} KKT system per Newton step) "
                  f"x rank 0's own Newton counts / HIP-event kernel time; executed = the linear solve the kernel "
                  f"performs ({ls}: " + (f"band LU of the reordered {n}x{n} S, window {mcp.nl.band.ns}x"
                  f"{mcp.nl.band.wc}" if bandk else f"LU of dim {solve_dim(n, m, ls)}") +
                  (" + the Schur complement from Q's structural nonzeros" if ls == "schur" else "") +
                  "); bound: per-wave latency (PMC: waves stall on LDS/VALU dependencies, DESIGN.md §4)",
                  structural=True)
    rl["frac_structural"] = rl["executed_frac"]
    # critical path: the game with the most Newton steps solved alone (one wave on an idle GPU,
    # the same kernel): its time over the launch's says how much of the launch is that one
    # game's chain of dependent steps (≈ 1: tail-bound, the rest of the batch fits beside it)
    imax = int(torch.argmax(out["newton_iters"]).item())
    nmax = int(out["newton_iters"][imax].item())
    one = alloc_device_outputs(1, n, m, dev)
    th1 = theta[imax:imax + 1].contiguous()
    lone = []
    for rep in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        solve_batch_device(_abi.FAMILY_NONLINEAR, n, m, th1, one, tol=a.tol, linear_solver=ls, stream=stream,
                           module=module, kernel=a.kernel)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        if rep:
            lone.append(e0.elapsed_time(e1))
    lone_ms = float(np.mean(lone))
    rl["critical_path"] = {"longest_game_newton": nmax, "lone_game_ms": lone_ms,
                           "lone_step_us": lone_ms * 1e3 / max(nmax, 1), "frac_of_launch": lone_ms / kern_ms,
                           "note": "the longest game of rank 0's batch solved alone (B = 1, same kernel) over the "
                                   "batch launch's kernel time: the share of the launch its dependent chain sets"}
    res = {
        "metric": ("MCP solve+VJP/sec (lane-change trajectory game, generated nonlinear module, rrule pullback of "
                   "x₁ as examples/utils.jl:236-261)" if a.sens else
                   "MCP solves/sec (lane-change trajectory game, generated nonlinear module)"),
        "value": a.steps * pl["global_batch"] / elapsed, "unit": "solves/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True,
        "scaling": pl["scaling"], "vs_baseline": None, "dtype": "f64",
        "data": "synthetic θ (benchmark/trajectory_game_benchmark.jl:62-87 sampler, numpy PCG64 in chunks of 4096 "
                f"seeded SeedSequence({a.seed}, spawn_key=(chunk,))), uploaded to HBM before timing",
        "config": {"workload": f"BASELINE C4: 2-player lane-change game T={a.lane_change} "
                               f"(n={n}, m={m}, KKT dim {N}), fp64, global batch {pl['global_batch']}, tol={a.tol:g}",
                   "n": n, "m": m, "kkt_dim": N, "linear_solver": ls, "batch_per_gpu": B, "kernel": kernel,
                   "global_batch": pl["global_batch"], "parallelism": f"dp{world} (instance shards)"},
        "roofline": rl,
        "newton_iters_mean": newton_all / pl["global_batch"], "success_rate": solved_all / pl["global_batch"],
        "summary_statistics": summary_statistics(step_s, B, solved_all / pl["global_batch"]),
        "evidence": evidence_id(key, cfg),
    }
    if a.sens:
        res["solve_kernel_ms"] = kern_ms
        res["vjp_kernel_ms"] = vjp_ms
        res["vjp_kernel"] = "mcpx_nl_vjp_wg"
        res["vjp_status_nonzero"] = int((vst != 0).sum().item())
    if world == 1 and a.cpu_sample != 0:
        from oracle import coracle

        coracle.build()
        th = a.cpu_threads or host_cpus()["nproc"]
        cb = cpu_baseline(lambda k, t: coracle.solve_batch_nl(mcp.nl, theta_host[:k], tol=a.tol, linear_solver=ls,
                                                              kernel=a.kernel, nthreads=t),
                          B, a, th, "C oracle with the generated host G/H code (same algorithm and linear solver)",
                          per_thread=256 if a.lane_change <= 2 else 32)
        r = cb.pop("_result")
        k = len(r["status"])
        got = {f: out[f][:k].cpu().numpy() for f in C4_FIELDS}
        res["parity"] = parity_report(got, r, C4_FIELDS, k, "oracle/ipm_oracle.c with the same generated G/H "
                                      "code (cpu_baseline sample)")
        if a.sens:  # the pullback of the same games against oracle_vjp_batch_nl at the GPU's solutions
            x, y, s_ = (out[f][:k].cpu().numpy() for f in ("x", "y", "s"))
            gxh = np.zeros((k, n))
            gxh[:, 0] = 1.0
            rd, rs = coracle.vjp_batch_nl(mcp.nl, theta_host[:k], x, y, s_, gxh, None, None, nthreads=th)
            res["vjp_parity"] = parity_report({"dtheta": dth[:k].cpu().numpy(), "status": vst[:k].cpu().numpy()},
                                              {"dtheta": rd, "status": rs}, ("dtheta", "status"), k,
                                              "oracle_vjp_batch_nl on the GPU's solutions")
        res["cpu_baseline"] = cb
    print(json.dumps(res), flush=True)


def main_qp(a, world, rank, local, dist, pl, distributed):
    import torch

    from mcp_amd.batch import solve_batch, solve_batch_device
    from mcp_amd.distributed import Gatherer, alloc_packed, shard_range
    from mcp_amd.qp_benchmark import generate_global_slice

    dev = torch.device("cuda", local)
    n, m, B = a.n, a.m, pl["count"]
    N = n + 2 * m
    theta_host = generate_global_slice(a.seed, n, m, a.sparsity, pl["start"], B)
    fam = 1 if a.family == "affine" else 0  # MCPX_FAMILY_AFFINE / _QP
    if fam:
        if a.sens:
            raise SystemExit("bench.py: --family affine has no --sens (the fused pullback is the QP family's)")
        from mcp_amd.qp_benchmark import affine_embedding

        theta_host = affine_embedding(theta_host, n, m)
    theta = torch.from_numpy(theta_host).to(dev)
    # outputs written straight into one packed fp64 record buffer + one int32 buffer
    # (x | y | s | kkt | ϵ and outer | status | newton), so the collection is 2 all-gathers
    packed = alloc_packed(B, n, m, dev, capacity=pl["cap"])
    out = packed.views()
    gather = Gatherer(packed) if distributed else None
    stream = torch.cuda.current_stream(dev)

    fused = a.sens and not a.unfused
    if a.sens:
        from mcp_amd.batch import solve_vjp_batch_device, vjp_batch_device

        p = theta.shape[1]
        dtheta = torch.empty(B, p, dtype=torch.float64, device=dev)
        vstat = torch.empty(B, dtype=torch.int32, device=dev)
        gx = torch.empty(B, n, dtype=torch.float64, device=dev)
        gy = torch.empty(B, m, dtype=torch.float64, device=dev)

    def pullback():
        # cotangent of f = Σx² + Σy² (test/runtests.jl:72-75): ∂x = 2x, ∂y = 2y, ∂s = 0
        torch.mul(out["x"], 2.0, out=gx)
        torch.mul(out["y"], 2.0, out=gy)
        vjp_batch_device(0, n, m, theta, out["x"], out["y"], out["s"], gx, gy, None, dtheta, vstat, stream=stream)

    def step(evs):
        if evs:
            evs[0][0].record(stream)
        if fused:  # one call: the pullback runs in the solve kernel's epilogue
            solve_vjp_batch_device(0, n, m, theta, out, ct=(2.0, 2.0, 0.0), dtheta=dtheta, status=vstat,
                                   tol=a.tol, linear_solver=a.linear_solver, stream=stream)
        else:
            solve_batch_device(fam, n, m, theta, out, tol=a.tol, linear_solver=a.linear_solver, stream=stream)
        if evs:
            evs[0][1].record(stream)
        if a.sens and not fused:
            if evs:
                evs[1][0].record(stream)
            pullback()
            if evs:
                evs[1][1].record(stream)
        if gather is not None:
            gather()

    elapsed, ms = timed_steps(step, a, stream, world, dist, dev, 2 if (a.sens and not fused) else 1)
    kern_ms = float(np.mean(ms[0]))
    vjp_ms = float(np.mean(ms[1])) if (a.sens and not fused) else 0.0
    step_s = [sum(t) * 1e-3 for t in zip(*ms)]  # per-step device time of the solve (+ pullback)
    # PCIe-inclusive rate of the host-buffer API (mcpx_solve_batch: H→D θ, solve, D→H
    # results), median of --host-runs runs after one warm-up;
    # reported beside `value`, never as it
    host = None
    if world == 1 and a.host_runs > 0 and not a.sens:
        from mcp_amd.batch import alloc_host_outputs, pinned

        def host_runs(out=None):
            solve_batch(fam, n, m, theta_host[:1024], tol=a.tol, linear_solver=a.linear_solver, num_devices=1)
            runs = []
            for _ in range(a.host_runs):
                t1 = time.perf_counter()
                solve_batch(fam, n, m, theta_host, tol=a.tol, linear_solver=a.linear_solver, num_devices=1, out=out)
                runs.append(time.perf_counter() - t1)
            return runs

        runs = host_runs()
        hout = alloc_host_outputs(B, n, m)
        runs_reuse = host_runs(hout)
        t_reg = time.perf_counter()
        with pinned(theta_host):
            t_reg = time.perf_counter() - t_reg
            runs_reg = host_runs(hout)
        host = {"median_solves_per_s": B / float(np.median(runs)), "runs_s": runs,
                "reused_outputs_median_solves_per_s": B / float(np.median(runs_reuse)), "reused_outputs_runs_s": runs_reuse,
                "registered_median_solves_per_s": B / float(np.median(runs_reg)), "registered_runs_s": runs_reg,
                "register_s": t_reg, "theta_bytes": int(theta_host.nbytes),
                "note": "mcpx_solve_batch on host numpy buffers (theta uploaded chunk by chunk on one copy stream "
                        "while earlier chunks solve, D->H of the results at the end), median of runs after a warm-up; "
                        "median_solves_per_s: fresh numpy result arrays per call (their pages fault during the call); "
                        "reused_outputs: result buffers from alloc_host_outputs reused across calls; registered: "
                        "theta page-locked once with mcpx_host_register (register_s, outside the runs), reused outputs"}
    newton = out["newton_iters"].to(torch.float64).sum().item()
    solved = (out["status"] == 0).to(torch.float64).sum().item()
    (elapsed, kern_ms, vjp_ms), (newton_all, solved_all) = reduce_max_sum(
        dist, dev, world, [elapsed, kern_ms, vjp_ms], [newton, solved])
    if distributed:
        full = gather.unpack([shard_range(pl["global_batch"], world, r)[1] for r in range(world)]
                             if pl["scaling"] == "strong" else None)
        assert int(full["status"].numel()) == pl["global_batch"], "gathered batch has the wrong size"
        for k in ("status", "newton_iters", "active_mask", "fail_reason", "x"):  # x by bits (NaN included)
            mine, own = full[k][pl["start"]:pl["start"] + B].to(dev), out[k]
            if mine.dtype == torch.float64:
                mine, own = mine.view(torch.int64), own.view(torch.int64)
            assert torch.equal(mine, own), f"gathered {k} differs from this rank's"
    if rank != 0:
        return
    G = pl["global_batch"]
    ls = a.linear_solver
    NS = solve_dim(n, m, ls)
    cfg = {"mode": ("c5" if fused else "c5u") if a.sens else "c3", "n": n, "m": m, "batch_per_gpu": B, "linear_solver": ls,
           "sparsity": a.sparsity}
    key = f"{cfg['mode']}_n{n}_m{m}_b{B}_{ls}"
    if fam:
        cfg["family"] = "affine"
        key += "_affine"
    ev = evidence(key, cfg)
    p = theta_host.shape[1]
    rl = roofline(kern_ms, newton * lu_flops(N), newton * executed_flops(n, m, ls),
                  B * (8.0 * (p + n + 2 * m + 2) + 12.0), ev,
                  "ipm_solve_kernel" if one_wave(n, m, ls) else "ipm_wg",  # ipm_wg_kernel_t / ipm_wg_vr_kernel_t
                  roofline_bound(ev, kern_ms, "valu" if one_wave(n, m, ls) else "latency"),
                  f"achieved = SURVEY.md §8(d) algorithmic FLOPs (dense LU of the N={N} KKT system, 2N^3/3+2N^2 per "
                  f"Newton step) x rank 0's own Newton counts / HIP-event time of the solve launch; executed = the FP64 "
                  f"work the kernel performs per step (residual + " + ("MFMA Schur complement + Gauss-Jordan of the "
                  f"{NS}-dim SPD S" if ls == "schur" else f"LU of dim {NS}") + ", bench.executed_flops); "
                  "bound: FP64 VALU issue (PMC, DESIGN.md §4); FP64 vector = matrix peak on MI355X; "
                  "frac_trace: same FLOPs over the committed rocprofv3 trace of this configuration and build")
    res = {
        "metric": METRIC,
        "value": a.steps * G / elapsed,
        "unit": "solves/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": pl["scaling"],
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (random dense QPs of benchmark/quadratic_program_benchmark.jl, host numpy PCG64 in chunks "
                f"of 4096 seeded SeedSequence({a.seed}, spawn_key=(chunk,)), uploaded to HBM before timing)",
        "config": {"workload": (f"BASELINE {'C5' if a.sens else ('C2' if (n, m) == (16, 8) else 'C3')}: random dense "
                                f"QP-KKT n={n} m={m} (KKT dim {N}), "
                                f"fp64, global batch {G} ({B} on rank 0), tol={a.tol:g}"
                                + (", passed as the affine family (P=M, Q=-A^T, R=A, S=0, g=-phi, h=-b: the "
                                   "Julia shim's layout)" if fam else "")
                                + ((", solve + rrule pullback of f = Σx²+Σy² "
                                    + ("fused in one kernel" if fused else "(solve, then VJP kernel)"))
                                   if a.sens else "")),
                   "n": n, "m": m, "kkt_dim": N, "linear_solver": ls, "solve_dim": NS, "family": a.family,
                   "batch_per_gpu": B, "global_batch": G, "sparsity": a.sparsity,
                   "parallelism": f"dp{world} (instance shards, RCCL all-gather of results)" if distributed
                   else "dp1"},
        "roofline": rl,
        "newton_iters_mean": newton_all / G,
        "success_rate": solved_all / G,
        "summary_statistics": summary_statistics(step_s, B, solved_all / G),
        "host_api": host,
        "evidence": evidence_id(key, cfg),
    }
    if fused:
        res["sensitivity"] = {
            "fused": True, "solve_vjp_kernel_ms": kern_ms, "solve_vjp_per_s": B / (kern_ms * 1e-3),
            "vjp_failed": int((vstat != 0).sum().item()),
            "note": "mcpx_solve_vjp_batch_device: the rrule pullback of f = Σx²+Σy² runs in the epilogue of the "
                    "SCHUR solve kernel (csrc/ipm_inst_fused.hip), one launch pair for solve + VJP; roofline = "
                    "the solve's Newton-step FLOPs over the fused launch (the pullback's one LU per instance "
                    "is not counted); --unfused times the two-call path"}
    elif a.sens:
        vbytes = B * 8 * (2 * p + 3 * N + 2 * N)  # θ read, ∂θ written, (x,y,s) + cotangents read
        vflops = B * lu_flops(N)
        vexec = B * lu_flops(n + m)
        res["sensitivity"] = {"fused": False,
            "vjp_kernel_ms": vjp_ms, "solve_kernel_ms": kern_ms, "vjp_per_s": B / (vjp_ms * 1e-3),
            "vjp_failed": int((vstat != 0).sum().item()),
            "vjp_roofline": {"flops_per_launch": vflops, "achieved_tflops": vflops / (vjp_ms * 1e-3) / 1e12,
                             "frac_fp64": vflops / (vjp_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
                             "executed_frac_fp64": vexec / (vjp_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
                             "algorithmic_bytes": vbytes, "achieved_gbs": vbytes / (vjp_ms * 1e-3) / 1e9,
                             "frac_hbm": vbytes / (vjp_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                             "note": "algorithmic: one dense LU of the N-dim ∇F_zᵀ (2N³/3+2N²) per instance; "
                                     "executed: the LU of the slack-eliminated (n+m)-dim system the kernel "
                                     "factors; bytes = θ read + ∂θ written + z and cotangents"},
        }
    if world == 1 and a.cpu_sample != 0:
        from oracle import coracle

        coracle.build()
        th = a.cpu_threads or host_cpus()["nproc"]
        cb = cpu_baseline(lambda k, t: coracle.solve_batch(fam, n, m, theta_host[:k], tol=a.tol, nthreads=t,
                                                           linear_solver=ls),
                          B, a, th, "C oracle (oracle/ipm_oracle.c, same algorithm and linear solver)")
        r = cb.pop("_result")
        cb["newton_mean"] = float(r["newton_iters"].mean())
        k = len(r["status"])
        got = {f: out[f][:k].cpu().numpy() for f in QP_FIELDS}
        res["parity"] = parity_report(got, r, QP_FIELDS, k, "oracle/ipm_oracle.c, same linear solver "
                                      "(cpu_baseline sample)")
        if a.sens:  # the pullback of the same instances against oracle_vjp_batch
            kv = min(k, 1024)
            x, y, s_ = (out[f][:kv].cpu().numpy() for f in ("x", "y", "s"))
            rd, rs = coracle.vjp_batch(0, n, m, theta_host[:kv], x, y, s_, 2.0 * x, 2.0 * y, None, nthreads=th)
            res["parity"]["vjp"] = parity_report({"dtheta": dtheta[:kv].cpu().numpy(), "status": vstat[:kv].cpu().numpy()},
                                                 {"dtheta": rd, "status": rs}, ("dtheta", "status"), kv,
                                                 "oracle_vjp_batch on the GPU's solutions")
        res["cpu_baseline"] = cb
    if world == 1 and not a.sens and not fam:
        res["parity_fixtures"] = fixture_parity()
    print(json.dumps(res), flush=True)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if a.gpus > 1 and "RANK" not in os.environ:
        return launch_ranks(a.gpus, os.path.abspath(__file__), argv)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus > 1 and a.gpus != world:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    # MCPX_BENCH_SHARED_GPU=1: rehearsal of the N-rank path on a one-GPU box — every rank on
    # cuda:0, gloo instead of RCCL (the sharding, the solves, the gather and the max-over-ranks
    # timing run as on N GPUs; the rate is not an N-GPU rate)
    shared = os.environ.get("MCPX_BENCH_SHARED_GPU") == "1"
    if world > 1 and not shared and torch.cuda.device_count() < world:
        print(f"bench.py: {world} ranks but only {torch.cuda.device_count()} GPU(s) visible", file=sys.stderr)
        return 2
    distributed = world > 1 or (a.gather and "RANK" in os.environ)
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("NCCL_DEBUG", "WARN")  # keep RCCL's banner off stdout (one JSON line)
        if shared:
            local = 0
            torch.cuda.set_device(0)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    pl = plan(a, world, rank)
    try:
        if a.lane_change:
            main_lane_change(a, world, rank, local, dist, pl)
        else:
            main_qp(a, world, rank, local, dist, pl, distributed)
    finally:
        if distributed:
            dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
