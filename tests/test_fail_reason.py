"""Per-instance failure reasons (mcpx_out.fail_reason, include/mcpx.h MCPX_FAIL_*): the
events behind the reference's `verbose` warnings — a failed linear solve
(src/solver.jl:84-88), a failed line search (:93-99) — and the outer-iteration limit
(:117-119).  CPU: the oracle's semantics on inputs built to trigger each event; GPU:
every kernel family reports the oracle's bits (assert_parity compares fail_reason)."""

from __future__ import annotations

import numpy as np
import pytest

from mcp_amd import _abi
from mcp_amd.qp_benchmark import generate_random_parameter

LIN, LS, MO = _abi.FAIL_LINSOLVE, _abi.FAIL_LINESEARCH, _abi.FAIL_MAX_OUTER
TOL = 2.0 ** -10  # exactly representable: P = −tol·I cancels the regularisation to 0


def singular_affine(B=3):
    """Affine MCP with P = −tol·I and Q = R = S = 0: every x column of ∇F + tol·I is zero,
    so the LU meets an exact zero pivot (the failed solve of :84-88)."""
    n, m = 2, 1
    th = np.zeros((B, _abi.theta_dim(_abi.FAMILY_AFFINE, n, m)))
    th[:, 0] = th[:, 3] = -TOL  # P (column-major 2×2)
    th[:, -3:] = np.arange(1.0, 4.0)  # g, h
    return n, m, th


def qp_batch(B=64, seed=3):
    return 8, 4, generate_random_parameter(np.random.default_rng(seed), 8, 4, 0.0, batch=B)


def cases():
    """(label, family, n, m, θ, kwargs, bit the case must show somewhere)."""
    n, m, th = singular_affine()
    yield "linsolve", _abi.FAMILY_AFFINE, n, m, th, dict(tol=TOL), LIN
    n, m, th = qp_batch()
    yield "linesearch", _abi.FAMILY_QP, n, m, th, dict(tol=1e-6, min_stepsize=0.99), LS
    yield "max_outer", _abi.FAMILY_QP, n, m, th, dict(tol=1e-12, max_outer_iters=3), MO
    yield "default", _abi.FAMILY_QP, n, m, th, dict(tol=1e-6), 0


CASES = list(cases())


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("ls", ["reduced", "dense", "schur"])
def test_oracle_fail_reason(oracle_lib, case, ls):
    label, fam, n, m, th, kw, bit = case
    r = oracle_lib.solve_batch(fam, n, m, th, linear_solver=ls, **kw)
    fr, st, outer = r["fail_reason"], r["status"], r["outer_iters"]
    maxo = kw.get("max_outer_iters", 50)
    assert ((fr & MO) != 0).tolist() == (outer == maxo).tolist()  # :117-119
    assert np.all(fr[st == _abi.STATUS_FAILED] != 0)  # a failed solve says why
    assert np.all(fr < 8)
    if bit:
        assert np.any(fr & bit), label
    else:
        assert np.all(fr[st == _abi.STATUS_SOLVED] & MO == 0)
    if label == "linsolve":
        assert np.all(fr & LIN) and np.all(st == _abi.STATUS_FAILED)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("ls", ["reduced", "dense", "schur"])
def test_gpu_fail_reason_vs_oracle(gpu, oracle_lib, case, ls):
    from mcp_amd.batch import solve_batch

    from tests.test_gpu_parity import assert_parity

    label, fam, n, m, th, kw, _ = case
    got = solve_batch(fam, n, m, th, linear_solver=ls, trace_len=64, **kw)
    ref = oracle_lib.solve_batch(fam, n, m, th, linear_solver=ls, trace_len=64, **kw)
    assert_parity(got, ref)
    np.testing.assert_array_equal(got["fail_reason"], ref["fail_reason"])


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES[1:], ids=[c[0] for c in CASES[1:]])
def test_gpu_fail_reason_workgroup_and_device(gpu, oracle_lib, case):
    """The workgroup-per-instance kernel (forced) and the device-tensor path."""
    import torch

    from mcp_amd.batch import alloc_device_outputs, solve_batch, solve_batch_device

    label, fam, n, m, th, kw, _ = case
    ref = oracle_lib.solve_batch(fam, n, m, th, linear_solver="dense", **kw)
    got = solve_batch(fam, n, m, th, linear_solver="dense", kernel="workgroup", **kw)
    np.testing.assert_array_equal(got["fail_reason"], ref["fail_reason"])
    out = alloc_device_outputs(th.shape[0], n, m, "cuda")
    solve_batch_device(fam, n, m, torch.from_numpy(th).cuda(), out, linear_solver="dense", **kw)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out["fail_reason"].cpu().numpy(), ref["fail_reason"])
