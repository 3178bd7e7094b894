"""Repeat-call determinism of a generated module's solve (diagnostic): the C4 batch solved `count`
times in one process, every call's outputs compared bit for bit with the CPU oracle's.
    python tools/band_stress.py T B kernel count reuse|reload|device|pinned [hsaco]
kernel: band | workgroup | auto; reuse: one Module for every call; reload: a new Module per call
(the pattern of tools/band_ab.py); device: one Module, θ and outputs as device tensors
(solve_batch_device); pinned: one Module, θ page-locked.  hsaco: a tools/bandv build instead of
the module cache's.  Each call is compared with the oracle and with call 0.
STRESS_FLUSH=1: a 512 MiB device fill between calls (evicts the L2s); STRESS_ALT=1: odd calls solve
a second parameter batch (compared with its own oracle solution).  MCPX_POISON=1: the library's
device blocks come NaN-filled with a checked canary after them ("canary" = blocks overwritten)."""
import json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mcp_amd import _abi
from mcp_amd.batch import Module, solve_batch
from oracle import coracle
from tests.test_band import _c4

T, B, kernel, count, mode = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], int(sys.argv[4]), sys.argv[5]
FLUSH, ALT = os.environ.get("STRESS_FLUSH") == "1", os.environ.get("STRESS_ALT") == "1"
if mode == "device" or FLUSH or os.environ.get("STRESS_TORCH") == "1":  # torch's HIP runtime first (tests/conftest.py)
    import torch
    torch.zeros(1, device="cuda")
path = sys.argv[6] if len(sys.argv) > 6 else None
PRE = os.environ.get("STRESS_PREINIT", "")
if PRE == "import":  # torch imported, its HIP runtime not initialised
    import torch
if PRE == "hipmalloc":  # one plain hipMalloc before the library's first call
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    _p = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(_p), ctypes.c_size_t(2 << 20)) == 0
game, tp = _c4(T, B)
nl = game.mcp.nl
kw = dict(linear_solver="schur", trace_len=64)
ref = coracle.solve_batch_nl(nl, tp, nthreads=16, **kw)
if ALT:
    tq = np.ascontiguousarray(_c4(T, 2 * B)[1][B:], dtype=np.float64)
    refq = coracle.solve_batch_nl(nl, tq, nthreads=16, **kw)


def load():
    return Module(path) if path else game.mcp.module()


def bad(a, b):
    m = np.zeros(B, bool)
    for k in ("x", "y", "s", "status", "newton_iters", "outer_iters"):
        g, r = np.asarray(a[k]).reshape(B, -1), np.asarray(b[k]).reshape(B, -1)
        same = (g == r) | (np.isnan(g) & np.isnan(r)) if g.dtype.kind == "f" else (g == r)
        m |= ~same.all(1)
    return m


mod = load()
tp = np.ascontiguousarray(tp, dtype=np.float64)
if mode == "device":
    from mcp_amd.batch import alloc_device_outputs, solve_batch_device
    td = torch.from_numpy(tp).cuda()
if mode == "pinned":
    from mcp_amd.batch import pinned
    pin = pinned(tp)
    pin.__enter__()
r0 = None
ob = None
tp0, ref0 = tp, ref
for i in range(count):
    if ALT:
        tp, ref = (tq, refq) if i % 2 else (tp0, ref0)
    if FLUSH and i:
        junk = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
        junk.fill_(7)
        torch.cuda.synchronize()
        del junk
    if mode == "reload" and i:
        mod = load() if path else Module(mod.path)
    t0 = time.perf_counter()
    if mode == "device":
        o = alloc_device_outputs(B, nl.n, nl.m, td.device, trace_len=64)
        solve_batch_device(_abi.FAMILY_NONLINEAR, nl.n, nl.m, td, o, module=mod, kernel=kernel, linear_solver="schur")
        torch.cuda.synchronize()
        r = {k: v.cpu().numpy() for k, v in o.items() if v is not None}
    else:
        if PRE == "outbuf":  # host result buffers allocated once, reused
            from mcp_amd.batch import alloc_host_outputs
            ob = ob if i else alloc_host_outputs(B, nl.n, nl.m, 64)
            r = solve_batch(_abi.FAMILY_NONLINEAR, nl.n, nl.m, tp, module=mod, kernel=kernel, out=ob, **kw)
            r = {k: np.copy(v) for k, v in r.items()}
        else:
            r = solve_batch(_abi.FAMILY_NONLINEAR, nl.n, nl.m, tp, module=mod, kernel=kernel, **kw)
    dt = time.perf_counter() - t0
    r0 = r0 or r
    vo, v0 = bad(r, ref), (bad(r, r0) if not ALT else bad(r, ref))
    det = []
    for b in np.nonzero(vo)[0][:4]:  # the first Newton step whose line-search record differs
        ta, tb = r["alpha_trace"][b].reshape(-1, 2), ref["alpha_trace"][b].reshape(-1, 2)
        dif = np.nonzero((ta != tb).any(1))[0]
        fields = [k for k in ("x", "y", "s", "status", "newton_iters", "outer_iters", "kkt_error", "eps")
                  if not np.array_equal(np.asarray(r[k][b]), np.asarray(ref[k][b]))]
        other = [int(c) for c in range(B) if np.array_equal(r["x"][b], ref["x"][c])][:3]
        det.append([int(b), int(r["newton_iters"][b]), int(ref["newton_iters"][b]), int(r["status"][b]),
                    int(dif[0]) if len(dif) else -1, fields, other,
                    float(r["kkt_error"][b]), float(ref["kkt_error"][b]), float(r["eps"][b]), float(ref["eps"][b])])
    from mcp_amd._lib import lib as _mcpx

    print(json.dumps({"call": i, "s": round(dt, 4), "vs_oracle": int(vo.sum()), "vs_call0": int(v0.sum()),
                      "canary": int(_mcpx().mcpx_debug_canary_violations()),
                      "first_bad": np.nonzero(v0 if v0.any() else vo)[0][:8].tolist(),
                      "newton": int(r["newton_iters"].sum()), "bad[inst,newton,ref,status,step]": det}), flush=True)
print("oracle newton", int(ref["newton_iters"].sum()), flush=True)
