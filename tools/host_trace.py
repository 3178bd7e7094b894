"""Three host-buffer C3 solves (2 streams, 8192-instance chunks, reused result buffers,
page-locked θ) for a rocprofv3 kernel + memory-copy trace of the pipeline."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mcp_amd.batch import solve_batch, pinned, alloc_host_outputs
from mcp_amd.qp_benchmark import generate_global_slice
B = 65536
th = generate_global_slice(1, 32, 16, 0.0, 0, B)
out = alloc_host_outputs(B, 32, 16)
with pinned(th):
    for _ in range(3):
        t = time.perf_counter()
        solve_batch(0, 32, 16, th, tol=1e-6, linear_solver="schur", num_devices=1, out=out)
        print(f"{(time.perf_counter() - t) * 1e3:.2f} ms", flush=True)
