"""The N > 1 path on CPU: world-size-2 gloo process group, instances sharded
contiguously (ragged: 13 + 12, as a strong-scaling global batch splits), per-rank solves (the C oracle stands in for the GPU kernel here —
test-only injection; the product path is the HIP kernel), packed records
all-gathered with mcp_amd.distributed.Gatherer, and rank 0 checks the gathered
whole-batch results against a single-process solve."""

from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mcp_amd.distributed import Gatherer, alloc_packed, shard_capacity, shard_range
from mcp_amd.qp_benchmark import generate_random_parameter

N_, M_, B_TOTAL = 16, 8, 25  # ragged: 13 + 12 instances


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, ret):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import coracle

        th_all = generate_random_parameter(np.random.default_rng(3), N_, M_, 0.0, batch=B_TOTAL)
        start, cnt = shard_range(len(th_all), world, rank)
        packed = alloc_packed(cnt, N_, M_, "cpu", capacity=shard_capacity(B_TOTAL, world))
        out = packed.views()
        r = coracle.solve_batch(0, N_, M_, th_all[start:start + cnt], tol=1e-6, linear_solver="schur")
        for k in ("x", "y", "s", "kkt_error", "eps", "outer_iters", "status", "newton_iters"):
            out[k].copy_(torch.from_numpy(np.ascontiguousarray(r[k]).reshape(out[k].shape)))
        g = Gatherer(packed)
        g()
        full = g.unpack([shard_range(B_TOTAL, world, r)[1] for r in range(world)])
        if rank == 0:
            ref = coracle.solve_batch(0, N_, M_, th_all, tol=1e-6, linear_solver="schur")
            ok = all(np.array_equal(full[k].numpy(), ref[k].reshape(full[k].shape))
                     for k in ("x", "y", "s", "kkt_error", "eps", "outer_iters", "status", "newton_iters"))
            ret.put(ok)
    finally:
        dist.destroy_process_group()


def test_shard_range_covers_batch():
    for total in (0, 1, 7, 65536, 65537):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, world, r) for r in range(world)]
            assert sum(c for _, c in spans) == total
            assert all(spans[i][0] + spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


@pytest.mark.slow
def test_gloo_world2_sharded_solve_and_gather(oracle_lib):
    ctx = mp.get_context("spawn")
    ret = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, ret)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
        assert p.exitcode == 0
    assert ret.get(timeout=10) is True


def test_packed_views_with_padding():
    """A rank's packed buffers hold `capacity` instances; its views cover its own B."""
    p = alloc_packed(3, 4, 2, "cpu", capacity=5)
    v = p.views()
    assert v["x"].shape == (3, 4) and v["y"].shape == (3, 2) and v["status"].shape == (3,)
    assert p.rec.numel() == 5 * (4 + 2 * 2 + 2) and p.irec.numel() == 15
    v["s"].fill_(7.0)
    assert float(p.rec[5 * 4 + 5 * 2:5 * 4 + 5 * 2 + 6].sum()) == 42.0  # s block starts after cap·(n + m)
    with pytest.raises(ValueError):
        alloc_packed(6, 4, 2, "cpu", capacity=5)
