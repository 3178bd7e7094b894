"""Builds the lane-change module with -DMCPX_STAMPS=1 and tools/nl_phase (CPU side), and writes
θ (benchmark sampler, the bench's seed) for the GPU run:  python tools/nl_phase.py T B"""
import os, subprocess, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mcp_amd import codegen
from mcp_amd.lane_change import LaneChangeGame
from mcp_amd.qp_benchmark import chunked_slice

T, B = int(sys.argv[1]), int(sys.argv[2])
g = LaneChangeGame(T)
mcp = g.mcp
th = np.ascontiguousarray(mcp.theta_map(chunked_slice(lambda rng, k: g.generate_random_parameter(rng, k), 1, 0, B)))
out = os.path.join(ROOT, "tools", "phase_data")  # shipped to the box (ubench_data is not)
os.makedirs(out, exist_ok=True)
th.tofile(os.path.join(out, f"theta_lane_t{T}_b{B}.bin"))
mcp.nl.build_module()  # the product module (and its .hip text)
src = mcp.nl.module_path().replace(".hsaco", ".hip")
flags = [f for f in codegen._MODULE_FLAGS]
cmd = [codegen.HIPCC, *flags, "-DMCPX_STAMPS=1", "-I", codegen.CSRC, "-o", os.path.join(out, f"nl_t{T}_stamps.hsaco"), src]
subprocess.run(cmd, check=True)
print(f"n={mcp.unconstrained_dimension} m={mcp.constrained_dimension} p={th.shape[1]} B={B}")
