"""Determinism and parity of band-kernel build variants on the whole C4 batch (diagnostic), one
process, the variants in the order given (a name may repeat):
    python tools/band_det.py T B name [name ...]   (tools/bandv/band_t<T>_<name>.hsaco, tools/band_ab.py build)"""
import json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mcp_amd import _abi
from mcp_amd.batch import Module, solve_batch
from oracle import coracle
from tests.test_band import _c4

T, B, names = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3:]
game, tp = _c4(T, B)
nl = game.mcp.nl
mods = {nm: Module(os.path.join(ROOT, "tools", "bandv", f"band_t{T}_{nm}.hsaco")) for nm in set(names)}
kw = dict(linear_solver="schur", kernel="band", trace_len=64)
runs = [solve_batch(_abi.FAMILY_NONLINEAR, nl.n, nl.m, tp, module=mods[nm], **kw) for nm in names]
t0 = time.time()
ref = coracle.solve_batch_nl(nl, tp, nthreads=16, **kw)
print(f"oracle {time.time() - t0:.1f}s", flush=True)
def bad(a, b):
    m = np.zeros(B, bool)
    for k in ("x", "y", "s", "status", "newton_iters", "outer_iters"):
        g, r = np.asarray(a[k]).reshape(B, -1), np.asarray(b[k]).reshape(B, -1)
        same = (g == r) | (np.isnan(g) & np.isnan(r)) if g.dtype.kind == "f" else (g == r)
        m |= ~same.all(1)
    return m
for i, r in enumerate(runs):
    vo = bad(r, ref)
    vr = bad(r, runs[0])
    print(json.dumps({"run": i, "variant": names[i], "vs_oracle": int(vo.sum()), "vs_run0": int(vr.sum()), "first_bad": np.nonzero(vo)[0][:10].tolist(),
                      "newton": int(r["newton_iters"].sum())}), flush=True)
print("oracle newton", int(ref["newton_iters"].sum()))
