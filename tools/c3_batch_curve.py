"""Latency / throughput curve of the C3 SCHUR kernel over the batch size.

For B in a sweep: device time of one solve launch pair (HIP events, median of
repeats), solves/s, the Newton-count distribution (mean, max) and the number of
instances the fast pass deferred.  At B = 1 the time is one wave's latency; at
B = 1,024 every SIMD holds one wave; the C5 batch (4,096) is 4 waves per SIMD.

    python tools/c3_batch_curve.py [--n 32 --m 16] [--fused]
"""

from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=32)
    ap.add_argument("--m", type=int, default=16)
    ap.add_argument("--batches", default="1,64,256,1024,2048,4096,8192,16384,65536")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--fused", action="store_true", help="time mcpx_solve_vjp_batch_device instead")
    a = ap.parse_args()
    import torch

    from mcp_amd.batch import alloc_device_outputs, solve_batch_device, solve_vjp_batch_device
    from mcp_amd.qp_benchmark import generate_random_parameter

    dev = torch.device("cuda", 0)
    n, m = a.n, a.m
    Bmax = max(int(b) for b in a.batches.split(","))
    th_all = torch.from_numpy(generate_random_parameter(np.random.default_rng(1), n, m, 0.0, batch=Bmax)).to(dev)
    st = torch.cuda.current_stream(dev)
    for B in (int(b) for b in a.batches.split(",")):
        th = th_all[:B].contiguous()
        out = alloc_device_outputs(B, n, m, dev)
        dth = torch.empty(B, th.shape[1], dtype=torch.float64, device=dev)
        vst = torch.empty(B, dtype=torch.int32, device=dev)

        def run():
            if a.fused:
                solve_vjp_batch_device(0, n, m, th, out, ct=(2.0, 2.0, 0.0), dtheta=dth, status=vst, tol=1e-6,
                                       linear_solver="schur", stream=st)
            else:
                solve_batch_device(0, n, m, th, out, tol=1e-6, linear_solver="schur", stream=st)

        run()
        torch.cuda.synchronize()
        ms = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            run()
            e1.record(st)
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        newton = out["newton_iters"].cpu().numpy()
        t = float(np.median(ms))
        print(json.dumps({"B": B, "ms": t, "solves_per_s": B / (t * 1e-3), "newton_mean": float(newton.mean()),
                          "newton_max": int(newton.max()), "newton_p99": float(np.percentile(newton, 99)),
                          "us_per_step_of_longest": t * 1e3 / max(int(newton.max()), 1),
                          "status_nonzero": int((out["status"] != 0).sum().item())}), flush=True)


if __name__ == "__main__":
    main()
