"""Batched solves through the C ABI (include/mcpx.h).

Two entry points, both running the HIP kernel (never a CPU fallback):

* :func:`solve_batch` — numpy host arrays in, numpy arrays out
  (``mcpx_solve_batch``: H→D copy, solve, D→H copy; shards over GPUs).
* :func:`solve_batch_device` — torch device tensors in and out, enqueued on
  the current HIP stream (``mcpx_solve_batch_device``); the benchmark's hot path.

Both return the per-instance fields of the reference's result NamedTuple
(src/solver.jl:121: status, x, y, s, kkt_error, ϵ, outer_iters) plus
``newton_iters``, ``active_mask`` and an optional ``alpha_trace``.
"""

from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _abi
from ._lib import check, lib


def _ptr(a):
    return None if a is None else a.ctypes.data


def _params(params=None, **kw) -> _abi.Params:
    return params if params is not None else _abi.make_params(**kw)


class Module:
    """A generated nonlinear-MCP code object (mcp_amd/codegen.py) loaded through
    the C ABI (mcpx_module_load, include/mcpx.h MCPX_FAMILY_NONLINEAR).  Kept for
    the process lifetime unless close() is called."""

    def __init__(self, path: str):
        h = C.c_void_p()
        check(lib().mcpx_module_load(os.fsencode(path), C.byref(h)))
        self.handle = h
        v = [C.c_int32() for _ in range(4)]
        check(lib().mcpx_module_dims(h, *(C.byref(x) for x in v)))
        self.n, self.m, self.p, self.solvers = (x.value for x in v)
        self.path = path

    @property
    def has_vjp(self) -> bool:
        return bool((self.solvers >> _abi.MODULE_VJP) & 1)

    @property
    def has_jvp(self) -> bool:
        return bool((self.solvers >> _abi.MODULE_JVP) & 1)

    @property
    def has_schur_mw(self) -> bool:
        return bool((self.solvers >> _abi.MODULE_SCHUR_MW) & 1)

    def close(self) -> None:
        if self.handle:
            lib().mcpx_module_unload(self.handle)
            self.handle = None


def alloc_host_outputs(B: int, n: int, m: int, trace_len: int = 0) -> dict:
    """Host result buffers of solve_batch(out=...), first-touched here: reused across
    calls they spare the D→H copy the page faults of fresh numpy pages."""
    words = max(1, (m + 63) // 64)
    r = dict(
        x=np.zeros((B, n)), y=np.zeros((B, m)), s=np.zeros((B, m)), kkt_error=np.zeros(B),
        eps=np.zeros(B), outer_iters=np.zeros(B, np.int32), status=np.zeros(B, np.int32),
        newton_iters=np.zeros(B, np.int32),
        active_mask=np.zeros((B, words), np.uint64),
        alpha_trace=np.full((B, max(trace_len, 0), 2), 254, np.uint8),
        fail_reason=np.zeros(B, np.uint8),
    )
    return r


def solve_batch(family: int, n: int, m: int, theta, *, x0=None, y0=None, s0=None, params=None,
                num_devices: int = 0, trace_len: int = 0, module: Module | None = None, out: dict | None = None,
                **kw) -> dict:
    """Solve B instances on the GPU(s).  theta: (B, ≥p) float64 host array.  `out`: result
    buffers from alloc_host_outputs (filled in place and returned), else fresh arrays."""
    theta = np.ascontiguousarray(theta, dtype=np.float64)
    if theta.ndim == 1:
        theta = theta[None, :]
    B, ld = theta.shape
    prm = _params(params, **kw)
    conv = lambda a, k: None if a is None else np.ascontiguousarray(np.broadcast_to(a, (B, k)), dtype=np.float64)
    x0, y0, s0 = conv(x0, n), conv(y0, m), conv(s0, m)
    words = max(1, (m + 63) // 64)
    if out is not None:
        r = out
        if r["x"].shape != (B, n) or r["y"].shape != (B, m) or r["status"].shape != (B,) or (
                trace_len > 0 and r["alpha_trace"].shape[1] < trace_len):
            raise ValueError("out buffers do not match the batch (alloc_host_outputs(B, n, m, trace_len))")
    else:
        r = dict(
            x=np.empty((B, n)), y=np.empty((B, m)), s=np.empty((B, m)), kkt_error=np.empty(B),
            eps=np.empty(B), outer_iters=np.empty(B, np.int32), status=np.empty(B, np.int32),
            newton_iters=np.empty(B, np.int32),
            active_mask=np.empty((B, words), np.uint64),
            alpha_trace=np.full((B, max(trace_len, 0), 2), 254, np.uint8),
            fail_reason=np.empty(B, np.uint8),
        )
    fr = r.get("fail_reason")
    out = _abi.Out(_ptr(r["x"]), _ptr(r["y"]), _ptr(r["s"]), _ptr(r["kkt_error"]), _ptr(r["eps"]),
                   _ptr(r["outer_iters"]), _ptr(r["status"]), _ptr(r["newton_iters"]),
                   _ptr(r["active_mask"]), _ptr(r["alpha_trace"]) if trace_len > 0 else None,
                   int(trace_len), 0, _ptr(fr) if fr is not None else None)
    desc = _abi.Desc(int(family), int(n), int(m), 0, int(B), int(ld))
    if module is not None:  # MCPX_FAMILY_NONLINEAR: the problem's generated code object
        check(lib().mcpx_solve_batch_module(module.handle, C.byref(desc), _ptr(theta), _ptr(x0), _ptr(y0),
                                            _ptr(s0), C.byref(prm), int(num_devices), C.byref(out)))
    else:
        check(lib().mcpx_solve_batch(C.byref(desc), _ptr(theta), _ptr(x0), _ptr(y0), _ptr(s0),
                                     C.byref(prm), int(num_devices), C.byref(out)))
    return r


class pinned:
    """Context manager that page-locks a host numpy array for the host-buffer calls
    (mcpx_host_register / mcpx_host_unregister): θ is then read by asynchronous DMA
    straight from it while earlier chunks solve.  For long-lived input batches."""

    def __init__(self, array: np.ndarray):
        if not (isinstance(array, np.ndarray) and array.flags.c_contiguous):
            raise ValueError("pinned() needs a C-contiguous numpy array")
        self.array = array

    def __enter__(self):
        check(lib().mcpx_host_register(self.array.ctypes.data, self.array.nbytes))
        return self.array

    def __exit__(self, *exc):
        check(lib().mcpx_host_unregister(self.array.ctypes.data))
        return False


def alloc_device_outputs(B: int, n: int, m: int, device, trace_len: int = 0, newton: bool = True,
                         active: bool = True) -> dict:
    import torch

    f64 = dict(dtype=torch.float64, device=device)
    i32 = dict(dtype=torch.int32, device=device)
    return dict(
        x=torch.empty(B, n, **f64), y=torch.empty(B, m, **f64), s=torch.empty(B, m, **f64),
        kkt_error=torch.empty(B, **f64), eps=torch.empty(B, **f64),
        outer_iters=torch.empty(B, **i32), status=torch.empty(B, **i32),
        newton_iters=torch.empty(B, **i32) if newton else None,
        # (B, W) uint64 words, W = max(1, ⌈m/64⌉) — the host path's and distributed.py's shape
        active_mask=torch.empty(B, max(1, (m + 63) // 64), dtype=torch.int64, device=device) if active else None,
        alpha_trace=torch.full((B, trace_len, 2), 254, dtype=torch.uint8, device=device) if trace_len > 0 else None,
        fail_reason=torch.empty(B, dtype=torch.uint8, device=device),
    )


def solve_batch_device(family: int, n: int, m: int, theta, out: dict | None = None, *, x0=None, y0=None,
                       s0=None, params=None, trace_len: int = 0, stream=None, module: Module | None = None,
                       **kw) -> dict:
    """Enqueue a batched solve on torch device tensors (no synchronisation).

    theta: (B, ≥p) contiguous float64 CUDA(HIP) tensor.  `out` (from
    :func:`alloc_device_outputs`) is reused when given — nothing is allocated
    on the hot path then.
    """
    import torch

    if not (theta.is_cuda and theta.dtype == torch.float64 and theta.dim() == 2 and theta.is_contiguous()):
        raise ValueError("theta must be a contiguous (B, p) float64 device tensor")
    B, ld = theta.shape
    if out is None:
        out = alloc_device_outputs(B, n, m, theta.device, trace_len)
    for t in (x0, y0, s0):
        if t is not None and not (t.is_cuda and t.dtype == torch.float64 and t.is_contiguous()):
            raise ValueError("warm starts must be contiguous float64 device tensors")
    dp = lambda t: None if t is None else t.data_ptr()
    tl = 0 if out.get("alpha_trace") is None else out["alpha_trace"].shape[1]
    o = _abi.Out(dp(out["x"]), dp(out["y"]), dp(out["s"]), dp(out["kkt_error"]), dp(out["eps"]),
                 dp(out["outer_iters"]), dp(out["status"]), dp(out.get("newton_iters")),
                 dp(out.get("active_mask")), dp(out.get("alpha_trace")), int(tl), 0, dp(out.get("fail_reason")))
    prm = _params(params, **kw)
    desc = _abi.Desc(int(family), int(n), int(m), 0, int(B), int(ld))
    st = stream if stream is not None else torch.cuda.current_stream(theta.device)
    if module is not None:
        check(lib().mcpx_solve_batch_module_device(module.handle, C.byref(desc), dp(theta), dp(x0), dp(y0), dp(s0),
                                                   C.byref(prm), C.byref(o), C.c_void_p(st.cuda_stream)))
    else:
        check(lib().mcpx_solve_batch_device(C.byref(desc), dp(theta), dp(x0), dp(y0), dp(s0), C.byref(prm),
                                            C.byref(o), C.c_void_p(st.cuda_stream)))
    return out


# ---------------------------------------------------------------------------
# sensitivities (reference src/AutoDiff.jl; include/mcpx.h mcpx_vjp_* / mcpx_jvp_*)


def _host_f64(a, shape):
    return None if a is None else np.ascontiguousarray(np.broadcast_to(a, shape), dtype=np.float64)


def _pdim(family: int, n: int, m: int, module: Module | None) -> int:
    return module.p if module is not None else _abi.theta_dim(family, n, m)


def vjp_batch(family: int, n: int, m: int, theta, x, y, s, gx=None, gy=None, gs=None,
              num_devices: int = 0, module: Module | None = None) -> tuple:
    """rrule pullback on the GPU(s) for host arrays: ∂θ = (∂z/∂θ)ᵀ [gx; gy; gs]
    (src/AutoDiff.jl:59-76).  None cotangents are zero.  Returns
    (dtheta (B, p) in the family's θ layout, status (B,) int32: 1 = ∇F_z singular).
    `module`: the generated module of a nonlinear-family MCP (mcpx_vjp_batch_module)."""
    theta = np.ascontiguousarray(np.atleast_2d(theta), dtype=np.float64)
    B, ld = theta.shape
    p = _pdim(family, n, m, module)
    x, y, s = _host_f64(x, (B, n)), _host_f64(y, (B, m)), _host_f64(s, (B, m))
    gx, gy, gs = _host_f64(gx, (B, n)), _host_f64(gy, (B, m)), _host_f64(gs, (B, m))
    dth = np.empty((B, p))
    st = np.empty(B, np.int32)
    desc = _abi.Desc(int(family), int(n), int(m), 0, int(B), int(ld))
    if module is not None:
        check(lib().mcpx_vjp_batch_module(module.handle, C.byref(desc), _ptr(theta), _ptr(x), _ptr(y), _ptr(s),
                                          _ptr(gx), _ptr(gy), _ptr(gs), int(num_devices), _ptr(dth), _ptr(st)))
    else:
        check(lib().mcpx_vjp_batch(C.byref(desc), _ptr(theta), _ptr(x), _ptr(y), _ptr(s), _ptr(gx), _ptr(gy),
                                   _ptr(gs), int(num_devices), _ptr(dth), _ptr(st)))
    return dth, st


def jvp_batch(family: int, n: int, m: int, theta, x, y, s, theta_dot, num_devices: int = 0,
              module: Module | None = None) -> tuple:
    """ForwardDiff-Dual tangents on the GPU(s): ż = (∂z/∂θ) θ̇ (src/AutoDiff.jl:94-100).
    theta_dot (B, K, p) → (zdot (B, K, n+2m), status (B,))."""
    theta = np.ascontiguousarray(np.atleast_2d(theta), dtype=np.float64)
    B, ld = theta.shape
    p = _pdim(family, n, m, module)
    td = np.ascontiguousarray(theta_dot, dtype=np.float64).reshape(B, -1, p)
    K = td.shape[1]
    x, y, s = _host_f64(x, (B, n)), _host_f64(y, (B, m)), _host_f64(s, (B, m))
    zd = np.empty((B, K, n + 2 * m))
    st = np.empty(B, np.int32)
    desc = _abi.Desc(int(family), int(n), int(m), 0, int(B), int(ld))
    if module is not None:
        check(lib().mcpx_jvp_batch_module(module.handle, C.byref(desc), _ptr(theta), _ptr(x), _ptr(y), _ptr(s),
                                          int(K), _ptr(td), int(num_devices), _ptr(zd), _ptr(st)))
    else:
        check(lib().mcpx_jvp_batch(C.byref(desc), _ptr(theta), _ptr(x), _ptr(y), _ptr(s), int(K), _ptr(td),
                                   int(num_devices), _ptr(zd), _ptr(st)))
    return zd, st


# rcond below which an instance's sensitivities count as ill-conditioned (include/mcpx.h
# mcpx_cond_batch): cond₁(∇F_z) > 1e12 leaves fewer than ~4 significant digits in ∂z/∂θ
ILL_CONDITIONED = 1e-12


def cond_batch(family: int, n: int, m: int, theta, x, y, s, num_devices: int = 0,
               module: Module | None = None) -> tuple:
    """Reciprocal 1-norm condition estimate of ∇F_z at the solutions (the matrix of the rrule's
    solve, src/AutoDiff.jl:39) on the GPU(s) → (rcond (B,), status (B,): 1 = exactly singular).
    `rcond < ILL_CONDITIONED` is the per-instance ill-conditioning flag."""
    theta = np.ascontiguousarray(np.atleast_2d(theta), dtype=np.float64)
    B, ld = theta.shape
    x, y, s = _host_f64(x, (B, n)), _host_f64(y, (B, m)), _host_f64(s, (B, m))
    rc = np.empty(B)
    st = np.empty(B, np.int32)
    desc = _abi.Desc(int(family), int(n), int(m), 0, int(B), int(ld))
    if module is not None:
        check(lib().mcpx_cond_batch_module(module.handle, C.byref(desc), _ptr(theta), _ptr(x), _ptr(y), _ptr(s),
                                           int(num_devices), _ptr(rc), _ptr(st)))
    else:
        check(lib().mcpx_cond_batch(C.byref(desc), _ptr(theta), _ptr(x), _ptr(y), _ptr(s), int(num_devices),
                                    _ptr(rc), _ptr(st)))
    return rc, st


def _dev_f64(t, what):
    import torch

    if t is None:
        return None
    if not (t.is_cuda and t.dtype == torch.float64 and t.is_contiguous()):
        raise ValueError(f"{what} must be a contiguous float64 device tensor")
    return t.data_ptr()


def vjp_batch_device(family: int, n: int, m: int, theta, x, y, s, gx=None, gy=None, gs=None, dtheta=None,
                     status=None, stream=None, module: Module | None = None):
    """Device-tensor pullback enqueued on the current stream (no sync).
    Returns (dtheta (B, p), status (B,) int32) tensors."""
    import torch

    if not (theta.is_cuda and theta.dtype == torch.float64 and theta.dim() == 2 and theta.is_contiguous()):
        raise ValueError("theta must be a contiguous (B, p) float64 device tensor")
    B, ld = theta.shape
    p = _pdim(family, n, m, module)
    dev = theta.device
    if dtheta is None:
        dtheta = torch.empty(B, p, dtype=torch.float64, device=dev)
    if status is None:
        status = torch.empty(B, dtype=torch.int32, device=dev)
    ptrs = [_dev_f64(t, k) for t, k in ((x, "x"), (y, "y"), (s, "s"), (gx, "gx"), (gy, "gy"), (gs, "gs"))]
    desc = _abi.Desc(int(family), int(n), int(m), 0, int(B), int(ld))
    st = stream if stream is not None else torch.cuda.current_stream(dev)
    if module is not None:
        check(lib().mcpx_vjp_batch_module_device(module.handle, C.byref(desc), theta.data_ptr(), *ptrs,
                                                 _dev_f64(dtheta, "dtheta"), status.data_ptr(),
                                                 C.c_void_p(st.cuda_stream)))
    else:
        check(lib().mcpx_vjp_batch_device(C.byref(desc), theta.data_ptr(), *ptrs, _dev_f64(dtheta, "dtheta"),
                                          status.data_ptr(), C.c_void_p(st.cuda_stream)))
    return dtheta, status


def solve_vjp_batch_device(family: int, n: int, m: int, theta, out: dict | None = None, *, ct=(0.0, 0.0, 0.0),
                           bx=None, by=None, bs=None, dtheta=None, status=None, x0=None, y0=None, s0=None,
                           params=None, stream=None, **kw):
    """Solve and pull back in one call (mcpx_solve_vjp_batch_device): the solve into
    `out` (as :func:`solve_batch_device`), then ∂θ of the loss whose cotangent is
    ∂l/∂x = ct[0]·x + bx, ∂l/∂y = ct[1]·y + by, ∂l/∂s = ct[2]·s + bs (b tensors or
    None = 0).  The README / C5 loss f = Σx² + Σy² is ct = (2, 2, 0).  SCHUR QPs at the
    benchmark sizes run the pullback inside the solve kernel.  Returns
    (out, dtheta (B, p), status (B,))."""
    import torch

    if not (theta.is_cuda and theta.dtype == torch.float64 and theta.dim() == 2 and theta.is_contiguous()):
        raise ValueError("theta must be a contiguous (B, p) float64 device tensor")
    B, ld = theta.shape
    dev = theta.device
    if out is None:
        out = alloc_device_outputs(B, n, m, dev)
    if dtheta is None:
        dtheta = torch.empty(B, _abi.theta_dim(family, n, m), dtype=torch.float64, device=dev)
    if status is None:
        status = torch.empty(B, dtype=torch.int32, device=dev)
    for t in (x0, y0, s0):
        if t is not None and not (t.is_cuda and t.dtype == torch.float64 and t.is_contiguous()):
            raise ValueError("warm starts must be contiguous float64 device tensors")
    dp = lambda t: None if t is None else t.data_ptr()
    tl = 0 if out.get("alpha_trace") is None else out["alpha_trace"].shape[1]
    o = _abi.Out(dp(out["x"]), dp(out["y"]), dp(out["s"]), dp(out["kkt_error"]), dp(out["eps"]),
                 dp(out["outer_iters"]), dp(out["status"]), dp(out.get("newton_iters")),
                 dp(out.get("active_mask")), dp(out.get("alpha_trace")), int(tl), 0, dp(out.get("fail_reason")))
    cot = _abi.Cotangent(float(ct[0]), float(ct[1]), float(ct[2]), _dev_f64(bx, "bx"), _dev_f64(by, "by"),
                         _dev_f64(bs, "bs"))
    prm = _params(params, **kw)
    desc = _abi.Desc(int(family), int(n), int(m), 0, int(B), int(ld))
    st = stream if stream is not None else torch.cuda.current_stream(dev)
    check(lib().mcpx_solve_vjp_batch_device(C.byref(desc), dp(theta), dp(x0), dp(y0), dp(s0), C.byref(prm),
                                            C.byref(o), C.byref(cot), _dev_f64(dtheta, "dtheta"), dp(status),
                                            C.c_void_p(st.cuda_stream)))
    return out, dtheta, status


def jvp_batch_device(family: int, n: int, m: int, theta, x, y, s, theta_dot, zdot=None, status=None,
                     stream=None, module: Module | None = None):
    """Device-tensor tangents: theta_dot (B, K, p) → (zdot (B, K, n+2m), status (B,))."""
    import torch

    if not (theta.is_cuda and theta.dtype == torch.float64 and theta.dim() == 2 and theta.is_contiguous()):
        raise ValueError("theta must be a contiguous (B, p) float64 device tensor")
    B, ld = theta.shape
    p = _pdim(family, n, m, module)
    td = theta_dot.reshape(B, -1, p)
    K = td.shape[1]
    dev = theta.device
    if zdot is None:
        zdot = torch.empty(B, K, n + 2 * m, dtype=torch.float64, device=dev)
    if status is None:
        status = torch.empty(B, dtype=torch.int32, device=dev)
    desc = _abi.Desc(int(family), int(n), int(m), 0, int(B), int(ld))
    st = stream if stream is not None else torch.cuda.current_stream(dev)
    fn = lib().mcpx_jvp_batch_device if module is None else (
        lambda *a: lib().mcpx_jvp_batch_module_device(module.handle, *a))
    check(fn(C.byref(desc), theta.data_ptr(), _dev_f64(x, "x"), _dev_f64(y, "y"), _dev_f64(s, "s"), int(K),
             _dev_f64(td.contiguous(), "theta_dot"), _dev_f64(zdot, "zdot"), status.data_ptr(),
             C.c_void_p(st.cuda_stream)))
    return zdot, status
