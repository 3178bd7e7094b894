"""A/B of compile-time variants of the C4 lane-change module (T = 2, SCHUR, one wave).

Build (CPU, here):   python tools/ab_c4/variants.py build NAME=-DFLAG=1[,-DFLAG2=0] ... [--T 2]
Run (GPU box):       python tools/ab_c4/variants.py run NAME ... [--out file.jsonl] [--T 2]

`build` compiles the product module's generated .hip with the module flags of
mcp_amd/codegen.py plus the variant's -D flags into tools/ab_c4/<NAME>.hsaco (not kept in
git).  `run` times each variant on the bench's 1,024 games (HIP events, 3 launches after a
warm-up) and compares every output field bitwise with the product module's (the product
module itself is the reference: a variant must change the time only).
"""
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

FIELDS = ("x", "y", "s", "kkt_error", "eps", "outer_iters", "status", "newton_iters")


T = 2  # horizon (--T)


def game():
    from mcp_amd.lane_change import LaneChangeGame

    return LaneChangeGame(T)


def build(specs):
    from mcp_amd import codegen

    mcp = game().mcp
    mcp.nl.build_module()
    src = mcp.nl.module_path().replace(".hsaco", ".hip")
    for spec in specs:
        name, _, flags = spec.partition("=")
        fl = [f for f in flags.split(",") if f]
        out = os.path.join(HERE, f"{name}.hsaco")
        inc = os.environ.get("AB_CSRC", codegen.CSRC)  # a modified copy of csrc/ for kernel variants
        subprocess.run([codegen.HIPCC, *codegen._MODULE_FLAGS, *fl, "-I", inc, "-o", out, src], check=True)
        print(f"built {out} {' '.join(fl)}", flush=True)


def run(names, out_path=None):
    import torch

    from mcp_amd import _abi
    from mcp_amd.batch import Module, alloc_device_outputs, solve_batch_device
    from mcp_amd.qp_benchmark import chunked_slice

    g = game()
    mcp = g.mcp
    n, m = mcp.unconstrained_dimension, mcp.constrained_dimension
    th_h = np.ascontiguousarray(mcp.theta_map(chunked_slice(lambda rng, k: g.generate_random_parameter(rng, k), 1, 0, 1024)))
    th = torch.from_numpy(th_h).cuda()
    mods = {"product": mcp.module()}
    for nm in names:
        mods[nm] = Module(os.path.join(HERE, f"{nm}.hsaco"))
    ref = None
    recs = []
    for name, mod in mods.items():
        out = alloc_device_outputs(1024, n, m, th.device)
        go = lambda: solve_batch_device(_abi.FAMILY_NONLINEAR, n, m, th, out, tol=1e-6,
                                        linear_solver=mcp.nl.default_solver(), module=mod)
        go()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            go()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 3
        got = {f: out[f].cpu().numpy() for f in FIELDS}
        if ref is None:
            ref = got
        same = all(np.array_equal(got[f], ref[f], equal_nan=True) for f in FIELDS)
        nw = got["newton_iters"]
        rec = {"variant": name, "ms": ms, "games_per_s": 1024 / (ms * 1e-3), "newton_max": int(nw.max()),
               "us_per_step_longest": ms * 1e3 / int(nw.max()), "identical_to_product": bool(same)}
        print(json.dumps(rec), flush=True)
        recs.append(rec)
    if out_path:
        with open(out_path, "w") as f:
            for r in recs:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    mode, rest = sys.argv[1], sys.argv[2:]
    outp = None
    if "--T" in rest:
        i = rest.index("--T")
        T = int(rest[i + 1])
        rest = rest[:i] + rest[i + 2:]
    if "--out" in rest:
        i = rest.index("--out")
        outp = rest[i + 1]
        rest = rest[:i] + rest[i + 2:]
    build(rest) if mode == "build" else run(rest, outp)
