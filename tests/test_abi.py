"""The C-ABI library builds for gfx950, loads, exports every symbol include/mcpx.h
declares, and rejects bad arguments loudly — no GPU needed (no compute calls)."""

from __future__ import annotations

import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from mcp_amd import _abi
from mcp_amd._lib import EXPORTS, LIB_PATH, MCPXError, check, lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mcpx.h")


def header_functions():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z0-9_]+\s*\*?\s*(mcpx_[a-z_]+)\(", txt, re.M)))


def test_header_functions_are_exported():
    L = lib()
    names = header_functions()
    assert set(names) == set(EXPORTS), (names, EXPORTS)
    for name in names:
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], capture_output=True, text=True).stdout
    for name in names:
        assert re.search(rf"\bT {name}$", out, re.M), f"{name} not a defined text symbol"


def test_library_has_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", LIB_PATH], capture_output=True,
                         text=True)
    blob = out.stdout + out.stderr
    if "gfx950" not in blob:  # older objdump: look into the bundle section directly
        data = open(LIB_PATH, "rb").read()
        assert b"gfx950" in data


def test_version_and_constants():
    L = lib()
    assert L.mcpx_version() == 20200
    for fam, (n, m) in [(0, (2, 2)), (0, (32, 16)), (1, (4, 8))]:
        assert L.mcpx_theta_dim(fam, n, m) == _abi.theta_dim(fam, n, m)
    assert L.mcpx_theta_dim(9, 2, 2) < 0 and L.mcpx_theta_dim(0, -1, 2) < 0


def test_default_params_match_reference_defaults():
    """src/solver.jl:42-48 and the fraction_to_the_boundary_linesearch defaults (:127)."""
    p = _abi.Params()
    lib().mcpx_default_params(C.byref(p))
    ref = _abi.make_params()
    for f, _ in _abi.Params._fields_:
        assert getattr(p, f) == getattr(ref, f), f
    assert (p.tol, p.max_inner_iters, p.max_outer_iters) == (1e-4, 20, 50)
    assert (p.tightening_rate, p.loosening_rate, p.min_stepsize, p.tau, p.decay) == (0.1, 0.5, 1e-4, 0.995, 0.5)


def _call(desc, theta, params):
    B = desc.batch
    outs = [np.empty(max(B, 1) * 64) for _ in range(5)] + [np.empty(max(B, 1), np.int32) for _ in range(2)]
    o = _abi.Out(*[a.ctypes.data for a in outs], None, None, None, 0, 0)
    rc = lib().mcpx_solve_batch(C.byref(desc), theta.ctypes.data if theta is not None else None, None, None, None,
                                C.byref(params), 1, C.byref(o))
    return rc


@pytest.mark.parametrize("bad", [
    dict(family=5), dict(n=-1), dict(n=0, m=0), dict(theta_ld=3), dict(batch=-1),
])
def test_argument_errors(bad):
    d = dict(family=0, n=2, m=2, batch=1, theta_ld=_abi.theta_dim(0, 2, 2))
    d.update(bad)
    desc = _abi.Desc(d["family"], d["n"], d["m"], 0, d["batch"], d["theta_ld"])
    rc = _call(desc, np.zeros(64), _abi.make_params())
    assert rc == _abi.MCPX_EINVAL
    assert lib().mcpx_last_error()


@pytest.mark.parametrize("kw,code", [
    (dict(tol=0.0), _abi.MCPX_EINVAL), (dict(decay=1.5), _abi.MCPX_EINVAL),
    (dict(max_outer_iters=0), _abi.MCPX_EINVAL), (dict(linear_solver=9), _abi.MCPX_EINVAL),
    (dict(max_inner_iters=4096), _abi.MCPX_EUNSUPPORTED), (dict(min_stepsize=1e-300), _abi.MCPX_EUNSUPPORTED),
])
def test_param_errors(kw, code):
    desc = _abi.Desc(0, 2, 2, 0, 1, _abi.theta_dim(0, 2, 2))
    assert _call(desc, np.zeros(64), _abi.make_params(**kw)) == code


def test_size_limits():
    # one wave: reduced n + m <= 64, dense n + 2m <= 64 (MCPX_KERNEL_WAVE refuses beyond);
    # workgroup kernels: n + 2m <= 768 (beyond: refused whatever the selector)
    desc = _abi.Desc(0, 40, 30, 0, 1, _abi.theta_dim(0, 40, 30))
    assert _call(desc, np.zeros(_abi.theta_dim(0, 40, 30)), _abi.make_params(kernel="wave")) == _abi.MCPX_EUNSUPPORTED
    desc = _abi.Desc(0, 32, 32, 0, 1, _abi.theta_dim(0, 32, 32))
    assert _call(desc, np.zeros(_abi.theta_dim(0, 32, 32)),
                 _abi.make_params(linear_solver="dense", kernel="wave")) == _abi.MCPX_EUNSUPPORTED
    desc = _abi.Desc(0, 400, 200, 0, 1, _abi.theta_dim(0, 400, 200))
    assert _call(desc, np.zeros(_abi.theta_dim(0, 400, 200)), _abi.make_params()) == _abi.MCPX_EUNSUPPORTED


def test_schur_takes_the_affine_family_on_one_wave():
    """SCHUR accepts the affine family (∂H/∂y taken as 0, include/mcpx.h); it is one wave only."""
    desc = _abi.Desc(1, 2, 2, 0, 1, _abi.theta_dim(1, 2, 2))
    assert _call(desc, np.zeros(64), _abi.make_params(linear_solver="schur")) in (_abi.MCPX_OK, _abi.MCPX_ENODEV)
    desc = _abi.Desc(1, 40, 30, 0, 1, _abi.theta_dim(1, 40, 30))
    assert _call(desc, np.zeros(_abi.theta_dim(1, 40, 30)),
                 _abi.make_params(linear_solver="schur")) == _abi.MCPX_EUNSUPPORTED


def test_no_device_is_an_error_not_a_fallback():
    """Without a GPU the product path fails loudly (there is no CPU fallback)."""
    if lib().mcpx_device_count() > 0:
        pytest.skip("a GPU is visible")
    desc = _abi.Desc(0, 2, 2, 0, 1, _abi.theta_dim(0, 2, 2))
    assert _call(desc, np.zeros(16), _abi.make_params()) == _abi.MCPX_ENODEV
    with pytest.raises(MCPXError):
        check(_abi.MCPX_ENODEV)


def test_host_register_argument_errors():
    assert lib().mcpx_host_register(None, 16) == _abi.MCPX_EINVAL
    buf = np.zeros(4)
    assert lib().mcpx_host_register(buf.ctypes.data, 0) == _abi.MCPX_EINVAL
    assert lib().mcpx_host_unregister(None) == _abi.MCPX_EINVAL
