"""mcpx_solve_vjp_batch_device — the solve with the rrule pullback in one call
(BASELINE C5; reference src/AutoDiff.jl:42-82 applied to src/solver.jl's solve).

The SCHUR QP kernels at the benchmark sizes run the pullback in the solve kernel's
epilogue (csrc/ipm_inst_fused.hip); every other configuration composes the solve and
the VJP launches.  Either way the outputs must be the bits of mcpx_solve_batch_device
followed by mcpx_vjp_batch_device with the cotangent a·z + b formed outside (and those
are the oracle's bits, tests/test_sensitivity.py).
"""

from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

from mcp_amd import _abi
from mcp_amd.qp_benchmark import generate_random_parameter

QP_FIELDS = ("x", "y", "s", "kkt_error", "eps", "outer_iters", "status", "newton_iters")


def _same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and bool(np.all((a == b) | (np.isnan(a) & np.isnan(b))))


def test_abi_solve_vjp_argument_errors():
    from mcp_amd._lib import lib

    L = lib()
    prm = _abi.make_params(linear_solver="schur")
    desc = _abi.Desc(0, 2, 2, 0, 1, _abi.theta_dim(0, 2, 2))
    buf = np.zeros(64)
    ptr = buf.ctypes.data
    o = _abi.Out(*([ptr] * 8), None, None, 0, 0)
    ct = _abi.Cotangent(2.0, 2.0, 0.0, None, None, None)
    # no cotangent
    assert L.mcpx_solve_vjp_batch_device(C.byref(desc), ptr, None, None, None, C.byref(prm), C.byref(o), None,
                                         ptr, None, None) == _abi.MCPX_EINVAL
    # nonlinear family has no generic kernels
    nl = _abi.Desc(_abi.FAMILY_NONLINEAR, 2, 2, 0, 1, 8)
    assert L.mcpx_solve_vjp_batch_device(C.byref(nl), ptr, None, None, None, C.byref(prm), C.byref(o),
                                         C.byref(ct), ptr, None, None) == _abi.MCPX_EINVAL
    # missing output arrays
    o_bad = _abi.Out(None, *([ptr] * 7), None, None, 0, 0)
    assert L.mcpx_solve_vjp_batch_device(C.byref(desc), ptr, None, None, None, C.byref(prm), C.byref(o_bad),
                                         C.byref(ct), ptr, None, None) == _abi.MCPX_EINVAL
    if L.mcpx_device_count() == 0:  # no CPU fallback
        assert L.mcpx_solve_vjp_batch_device(C.byref(desc), ptr, None, None, None, C.byref(prm), C.byref(o),
                                             C.byref(ct), ptr, None, None) == _abi.MCPX_ENODEV


# (family, n, m, linear solver): the first three run the fused kernels, the rest compose
CASES = [(0, 2, 2, "schur"), (0, 16, 8, "schur"), (0, 32, 16, "schur"),
         (0, 8, 4, "schur"), (0, 16, 8, "reduced"), (0, 12, 6, "dense"), (1, 6, 4, "reduced"),
         (0, 40, 16, "reduced")]


def _theta(rng, fam, n, m, B):
    if fam == 0:
        return generate_random_parameter(rng, n, m, 0.0, batch=B)
    from tests.test_sensitivity import random_affine_theta

    return random_affine_theta(rng, n, m, B)


@pytest.mark.gpu
@pytest.mark.parametrize("fam,n,m,ls", CASES)
@pytest.mark.parametrize("cot", ["loss", "affine", "plain"])
def test_gpu_solve_vjp_matches_solve_then_vjp(gpu, oracle_lib, fam, n, m, ls, cot):
    import torch

    from mcp_amd.batch import alloc_device_outputs, solve_batch_device, solve_vjp_batch_device, vjp_batch_device

    rng = np.random.default_rng(31 * n + m + len(cot))
    B = 1024 if (n, m) == (32, 16) else 256
    th_h = _theta(rng, fam, n, m, B)
    dev = torch.device("cuda", 0)
    th = torch.from_numpy(th_h).to(dev)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    if cot == "loss":  # f = Σx² + Σy² (test/runtests.jl:72-75)
        ct, b = (2.0, 2.0, 0.0), (None, None, None)
    elif cot == "affine":
        ct, b = (0.5, -1.5, 3.0), (T(rng.standard_normal((B, n))), T(rng.standard_normal((B, m))),
                                   T(rng.standard_normal((B, m))))
    else:  # plain cotangent arrays (a = 0)
        ct, b = (0.0, 0.0, 0.0), (T(rng.standard_normal((B, n))), None, T(rng.standard_normal((B, m))))
    kw = dict(tol=1e-6, linear_solver=ls)
    out, dth, st = solve_vjp_batch_device(fam, n, m, th, ct=ct, bx=b[0], by=b[1], bs=b[2], **kw)
    ref = solve_batch_device(fam, n, m, th, alloc_device_outputs(B, n, m, dev), **kw)

    def g(a, z, bb):  # a·z + b, two roundings (torch: separate mul and add kernels)
        if a == 0.0:
            return bb
        return a * z if bb is None else a * z + bb

    gx, gy, gs = g(ct[0], ref["x"], b[0]), g(ct[1], ref["y"], b[1]), g(ct[2], ref["s"], b[2])
    rdth, rst = vjp_batch_device(fam, n, m, th, ref["x"], ref["y"], ref["s"], gx, gy, gs)
    torch.cuda.synchronize()
    for f in QP_FIELDS:
        assert _same(out[f].cpu().numpy(), ref[f].cpu().numpy()), f
    assert _same(st.cpu().numpy(), rst.cpu().numpy())
    assert _same(dth.cpu().numpy(), rdth.cpu().numpy())
    if cot == "loss":  # and the oracle's pullback at the GPU's solution
        x, y, s = (ref[f].cpu().numpy() for f in ("x", "y", "s"))
        odth, ost = oracle_lib.vjp_batch(fam, n, m, th_h, x, y, s, 2.0 * x, 2.0 * y, None)
        assert _same(dth.cpu().numpy(), odth) and _same(st.cpu().numpy(), ost)


@pytest.mark.gpu
def test_gpu_solve_vjp_warm_start_and_failures(gpu):
    """Warm starts reach the fused kernel, and instances whose solve fails still get the
    pullback at their returned iterate, exactly as the composed calls do."""
    import torch

    from mcp_amd.batch import alloc_device_outputs, solve_batch_device, solve_vjp_batch_device, vjp_batch_device

    rng = np.random.default_rng(77)
    n, m, B = 16, 8, 512
    dev = torch.device("cuda", 0)
    th = torch.from_numpy(generate_random_parameter(rng, n, m, 0.0, batch=B)).to(dev)
    x0 = torch.from_numpy(rng.standard_normal((B, n))).to(dev)
    y0 = torch.from_numpy(rng.uniform(0.5, 2.0, (B, m))).to(dev)
    s0 = torch.from_numpy(rng.uniform(0.5, 2.0, (B, m))).to(dev)
    kw = dict(tol=1e-9, linear_solver="schur", max_outer_iters=3)  # many instances stop unsolved
    out, dth, st = solve_vjp_batch_device(0, n, m, th, ct=(2.0, 2.0, 0.0), x0=x0, y0=y0, s0=s0, **kw)
    ref = solve_batch_device(0, n, m, th, alloc_device_outputs(B, n, m, dev), x0=x0, y0=y0, s0=s0, **kw)
    rdth, rst = vjp_batch_device(0, n, m, th, ref["x"], ref["y"], ref["s"], 2.0 * ref["x"], 2.0 * ref["y"])
    torch.cuda.synchronize()
    assert (ref["status"] != 0).any()
    for f in QP_FIELDS:
        assert _same(out[f].cpu().numpy(), ref[f].cpu().numpy()), f
    assert _same(dth.cpu().numpy(), rdth.cpu().numpy()) and _same(st.cpu().numpy(), rst.cpu().numpy())


@pytest.mark.gpu
def test_gpu_solve_vjp_asymmetric_m_takes_the_lu_pass(gpu, oracle_lib):
    """M not exactly symmetric: the solve and the pullback both leave the Gauss-Jordan /
    Schur paths (fast pass defers, second pass uses the LU fallbacks); same bits as the
    composed calls and the oracle."""
    import torch

    from mcp_amd.batch import alloc_device_outputs, solve_batch_device, solve_vjp_batch_device, vjp_batch_device

    rng = np.random.default_rng(5)
    n, m, B = 32, 16, 256
    th_h = generate_random_parameter(rng, n, m, 0.0, batch=B)
    th_h[::2, 1] += 1e-3  # M[1, 0] != M[0, 1] in every other instance
    dev = torch.device("cuda", 0)
    th = torch.from_numpy(th_h).to(dev)
    kw = dict(tol=1e-6, linear_solver="schur")
    out, dth, st = solve_vjp_batch_device(0, n, m, th, ct=(2.0, 2.0, 0.0), **kw)
    ref = solve_batch_device(0, n, m, th, alloc_device_outputs(B, n, m, dev), **kw)
    rdth, rst = vjp_batch_device(0, n, m, th, ref["x"], ref["y"], ref["s"], 2.0 * ref["x"], 2.0 * ref["y"])
    torch.cuda.synchronize()
    for f in QP_FIELDS:
        assert _same(out[f].cpu().numpy(), ref[f].cpu().numpy()), f
    assert _same(dth.cpu().numpy(), rdth.cpu().numpy()) and _same(st.cpu().numpy(), rst.cpu().numpy())
    x, y, s = (ref[f].cpu().numpy() for f in ("x", "y", "s"))
    odth, ost = oracle_lib.vjp_batch(0, n, m, th_h, x, y, s, 2.0 * x, 2.0 * y, None)
    assert _same(dth.cpu().numpy(), odth) and _same(st.cpu().numpy(), ost)


@pytest.mark.gpu
def test_gpu_solve_vjp_warm_start_in_place(gpu):
    """Warm start read from the output buffers (x0 = out.x, y0 = out.y, s0 = out.s, the
    receding-horizon pattern) on instances the fused fast pass defers at the pullback
    (y < 0 at the returned iterate: the Schur pullback does not apply, so pass 2 solves
    them again from x0/y0/s0).  The fast pass must not have overwritten those buffers
    first: the bits equal the composed calls on separate warm-start buffers."""
    import torch

    from mcp_amd.batch import alloc_device_outputs, solve_batch_device, solve_vjp_batch_device, vjp_batch_device

    rng = np.random.default_rng(2024)
    n, m, B = 16, 8, 256
    dev = torch.device("cuda", 0)
    th = torch.from_numpy(generate_random_parameter(rng, n, m, 0.0, batch=B)).to(dev)
    x0 = torch.from_numpy(rng.standard_normal((B, n))).to(dev)
    yh = rng.uniform(0.5, 2.0, (B, m))
    yh[::2] *= -1.0  # every other instance starts (and stays) with y < 0
    y0 = torch.from_numpy(yh).to(dev)
    s0 = torch.from_numpy(rng.uniform(0.5, 2.0, (B, m))).to(dev)
    kw = dict(tol=1e-6, linear_solver="schur", max_outer_iters=4)
    ref = solve_batch_device(0, n, m, th, alloc_device_outputs(B, n, m, dev), x0=x0, y0=y0, s0=s0, **kw)
    rdth, rst = vjp_batch_device(0, n, m, th, ref["x"], ref["y"], ref["s"], 2.0 * ref["x"], 2.0 * ref["y"])
    out = alloc_device_outputs(B, n, m, dev)
    out["x"].copy_(x0)
    out["y"].copy_(y0)
    out["s"].copy_(s0)
    out, dth, st = solve_vjp_batch_device(0, n, m, th, out, ct=(2.0, 2.0, 0.0), x0=out["x"], y0=out["y"],
                                          s0=out["s"], **kw)
    torch.cuda.synchronize()
    ry = ref["y"].cpu().numpy()
    assert (ry < 0).any(axis=1).sum() > 0  # some instances do take the deferred pullback
    assert not np.array_equal(ref["x"].cpu().numpy(), x0.cpu().numpy())  # and their solves moved x
    for f in QP_FIELDS:
        assert _same(out[f].cpu().numpy(), ref[f].cpu().numpy()), f
    assert _same(dth.cpu().numpy(), rdth.cpu().numpy()) and _same(st.cpu().numpy(), rst.cpu().numpy())
