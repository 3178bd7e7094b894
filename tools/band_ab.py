"""A/B of band-kernel build variants (diagnostic): the lane-change module at horizon T compiled with
extra -D flags (only the band kernel, MCPX_NL_ONLY_BAND), timed on the C4 batch through
MCPX_KERNEL_BAND, outputs compared bit for bit with the first variant.
    python tools/band_ab.py build T name "-DFLAG=1 ..." [name "-D..."] ...   (CPU)
    python tools/band_ab.py run T B name [name ...]                          (GPU)"""
import hashlib, json, os, subprocess, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tools", "bandv")

if sys.argv[1] == "build":
    from mcp_amd import codegen
    from mcp_amd.lane_change import LaneChangeGame

    T = int(sys.argv[2])
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(OUT, f"t{T}.hip")
    open(src, "w").write(LaneChangeGame(T).mcp.nl.hip_source())
    procs = []
    args = sys.argv[3:]
    for name, flags in zip(args[0::2], args[1::2]):
        cmd = [codegen.HIPCC, *codegen._MODULE_FLAGS, "-I", codegen.CSRC, "-DMCPX_NL_ONLY_BAND", *flags.split(),
               "-o", os.path.join(OUT, f"band_t{T}_{name}.hsaco"), src]
        procs.append(subprocess.Popen(cmd))
    sys.exit(max(p.wait() for p in procs))

from mcp_amd import _abi
from mcp_amd.batch import Module, solve_batch
from tests.test_band import _c4

T, B = int(sys.argv[2]), int(sys.argv[3])
game, tp = _c4(T, B)
nl = game.mcp.nl
ref = None
for name in sys.argv[4:]:
    mod = Module(os.path.join(OUT, f"band_t{T}_{name}.hsaco"))
    run = lambda: solve_batch(_abi.FAMILY_NONLINEAR, nl.n, nl.m, tp, linear_solver="schur", module=mod, kernel="band",
                              trace_len=64)
    r = run()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        r = run()
        ts.append(time.perf_counter() - t0)
    h = hashlib.sha256()
    for k in sorted(r):
        if isinstance(r[k], np.ndarray):
            h.update(r[k].tobytes())
    d = h.hexdigest()[:16]
    ref = ref or d
    print(json.dumps({"T": T, "B": B, "variant": name, "s_median": float(np.median(ts)),
                      "games_per_s": B / float(np.median(ts)), "newton": int(r["newton_iters"].sum()),
                      "digest": d, "same_as_first": d == ref}), flush=True)
