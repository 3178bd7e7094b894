"""The N > 1 paths with the HIP kernels on a one-GPU box.

* In-process (C ABI): `mcpx_solve_batch` / `mcpx_vjp_batch` / `mcpx_jvp_batch` /
  `mcpx_solve_batch_module` with `num_devices > 1` run one host thread per device on
  contiguous shards.  `MCPX_HOST_SHARDS = k` forces k shards over the visible devices
  (round-robin), so the threaded shard path, the per-shard pipelines and the stitching
  of the results run here; the results must be bit-identical to one shard.
* One process per GPU (bench.py under torch.distributed.run): `MCPX_BENCH_SHARED_GPU = 1`
  puts every rank on cuda:0 and uses gloo instead of RCCL (RCCL needs one GPU per rank),
  so the sharding, the per-rank HIP solves, the packed-record all-gather
  (`mcp_amd.distributed.Gatherer`, staged through host copies for gloo) with bench.py's own
  check of each rank's slice, and the max-over-ranks timing run for world size 2.
"""

from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from mcp_amd import _abi
from mcp_amd.qp_benchmark import generate_random_parameter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ("x", "y", "s", "kkt_error", "eps", "outer_iters", "status", "newton_iters")


def _same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and bool(np.all((a == b) | (np.isnan(a) & np.isnan(b))))


class _shards:
    def __init__(self, k):
        self.k = k

    def __enter__(self):
        self.old = os.environ.get("MCPX_HOST_SHARDS")
        os.environ["MCPX_HOST_SHARDS"] = str(self.k)

    def __exit__(self, *exc):
        if self.old is None:
            os.environ.pop("MCPX_HOST_SHARDS", None)
        else:
            os.environ["MCPX_HOST_SHARDS"] = self.old


@pytest.mark.gpu
@pytest.mark.parametrize("ls", ["schur", "reduced"])
def test_gpu_host_shards_bit_identical(gpu, ls):
    from mcp_amd.batch import jvp_batch, solve_batch, vjp_batch

    rng = np.random.default_rng(44)
    n, m, B = 32, 16, 1001  # ragged: 3 shards of 334 / 334 / 333
    th = generate_random_parameter(rng, n, m, 0.0, batch=B)
    ref = solve_batch(0, n, m, th, tol=1e-6, linear_solver=ls)
    with _shards(3):
        got = solve_batch(0, n, m, th, tol=1e-6, linear_solver=ls)
    for f in FIELDS:
        assert _same(got[f], ref[f]), f
    gx = rng.standard_normal((B, n))
    td = rng.standard_normal((B, 2, th.shape[1]))
    rd, rs = vjp_batch(0, n, m, th, ref["x"], ref["y"], ref["s"], gx)
    rz, rzs = jvp_batch(0, n, m, th, ref["x"], ref["y"], ref["s"], td)
    with _shards(4):
        d, s_ = vjp_batch(0, n, m, th, ref["x"], ref["y"], ref["s"], gx)
        z, zs = jvp_batch(0, n, m, th, ref["x"], ref["y"], ref["s"], td)
    assert _same(d, rd) and _same(s_, rs) and _same(z, rz) and _same(zs, rzs)


@pytest.mark.gpu
def test_gpu_host_shards_module(gpu):
    from mcp_amd.batch import solve_batch
    from mcp_amd.lane_change import LaneChangeGame

    g = LaneChangeGame(2)
    mcp = g.mcp
    n, m = mcp.unconstrained_dimension, mcp.constrained_dimension
    th = mcp.theta_map(g.generate_random_parameter(np.random.default_rng(3), 97))
    mod = mcp.module()
    fam = _abi.FAMILY_NONLINEAR
    ref = solve_batch(fam, n, m, th, tol=1e-6, linear_solver="schur", module=mod)
    with _shards(2):
        got = solve_batch(fam, n, m, th, tol=1e-6, linear_solver="schur", module=mod)
    for f in FIELDS:
        assert _same(got[f], ref[f]), f


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["--sens"]], ids=["c3", "c5"])
def test_gpu_two_rank_rehearsal(gpu, extra):
    env = dict(os.environ, MCPX_BENCH_SHARED_GPU="1", MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--global-batch", "4097", "--cpu-sample", "0",
           "--host-runs", "0", *extra]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 4097 and d["success_rate"] == 1.0
    assert d["config"]["parallelism"].startswith("dp2")
