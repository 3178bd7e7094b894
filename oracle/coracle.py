"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes wrapper around oracle/_build/libipm_oracle.so (the C restatement of
src/solver.jl, oracle/ipm_oracle.c).  Used by tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg; never by mcp_amd/.
"""

from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from mcp_amd._abi import Desc, Out, Params, make_params, theta_dim

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libipm_oracle.so")
_lib = None


def build(force: bool = False) -> str:
    """Compile the oracle with oracle/Makefile (gcc)."""
    if force:
        subprocess.run(["make", "-s", "-B", "-C", _HERE], check=True)
    else:  # incremental: rebuilds when ipm_oracle.c / mcpx.h are newer than the library
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        L.oracle_solve_batch.restype = C.c_int
        L.oracle_solve_batch.argtypes = [C.POINTER(Desc), C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.c_void_p, C.POINTER(Params), C.POINTER(Out), C.c_int]
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data


def solve_batch(family: int, n: int, m: int, theta: np.ndarray, *, x0=None, y0=None, s0=None,
                params: Params | None = None, trace_len: int = 0, nthreads: int = 1, **kw) -> dict:
    """Batched oracle solve.  theta: (B, p) float64.  Returns a dict of numpy arrays."""
    theta = np.ascontiguousarray(theta, dtype=np.float64)
    if theta.ndim == 1:
        theta = theta[None, :]
    B, ld = theta.shape
    p = theta_dim(family, n, m)
    if ld < p:
        raise ValueError(f"theta has {ld} columns, family needs {p}")
    prm = params if params is not None else make_params(**kw)
    conv = lambda a, k: None if a is None else np.ascontiguousarray(np.broadcast_to(a, (B, k)), dtype=np.float64)
    x0, y0, s0 = conv(x0, n), conv(y0, m), conv(s0, m)
    words = max(1, (m + 63) // 64)
    r = dict(
        x=np.empty((B, n)), y=np.empty((B, m)), s=np.empty((B, m)), kkt_error=np.empty(B),
        eps=np.empty(B), outer_iters=np.empty(B, np.int32), status=np.empty(B, np.int32),
        newton_iters=np.empty(B, np.int32), active_mask=np.empty((B, words), np.uint64),
        alpha_trace=np.full((B, max(trace_len, 0), 2), 254, np.uint8), fail_reason=np.empty(B, np.uint8),
    )
    out = Out(_ptr(r["x"]), _ptr(r["y"]), _ptr(r["s"]), _ptr(r["kkt_error"]), _ptr(r["eps"]),
              _ptr(r["outer_iters"]), _ptr(r["status"]), _ptr(r["newton_iters"]),
              _ptr(r["active_mask"]), _ptr(r["alpha_trace"]) if trace_len > 0 else None,
              int(trace_len), 0, _ptr(r["fail_reason"]))
    desc = Desc(family, n, m, 0, B, ld)
    rc = lib().oracle_solve_batch(C.byref(desc), _ptr(theta), _ptr(x0), _ptr(y0), _ptr(s0),
                                  C.byref(prm), C.byref(out), int(nthreads))
    if rc != 0:
        raise ValueError(f"oracle_solve_batch failed with code {rc}")
    return r


class OracleNL(C.Structure):
    """oracle_nl of ipm_oracle.c: the generated init/eval of one nonlinear MCP."""

    _fields_ = [("init", C.c_void_p), ("eval", C.c_void_p), ("p", C.c_int32), ("has_s", C.c_int32),
                ("size", C.c_int32), ("wave_schur", C.c_int32), ("qk_ptr", C.c_void_p), ("qk_idx", C.c_void_p),
                ("rj_ptr", C.c_void_p), ("rj_idx", C.c_void_p), ("eval_theta", C.c_void_p),
                ("tc_ptr", C.c_void_p), ("tc_idx", C.c_void_p), ("tr_ptr", C.c_void_p), ("tr_idx", C.c_void_p),
                ("band", C.c_int32), ("band_ns", C.c_int32), ("band_wc", C.c_int32), ("band_auto", C.c_int32),
                ("band_rperm", C.c_void_p), ("band_cperm", C.c_void_p)]


_GEN_DIR = os.path.join(_HERE, "_build", "gen")
_nl_libs: dict = {}


def nl_lib(nl):
    """gcc-compile the SAME generated text the gfx950 module is built from
    (mcp_amd/codegen.py NLSystem.body) into oracle/_build/gen/nl_<key>.so."""
    if nl.key in _nl_libs:
        return _nl_libs[nl.key]
    os.makedirs(_GEN_DIR, exist_ok=True)
    so = os.path.join(_GEN_DIR, f"nl_{nl.key}.so")
    if not os.path.exists(so):
        src = os.path.join(_GEN_DIR, f"nl_{nl.key}.c")
        with open(src, "w") as f:
            f.write("#include <math.h>\n#include <stdint.h>\n#define MCPX_NL_FN static inline\n"
                    "#define MCPX_NL_RESTRICT restrict\n#define MCPX_NL_TABLE static const\n"
                    "#define MCPX_NL_Z(j) (z[j])\n")
            f.write(nl.body)
            f.write("\nvoid oracle_nl_init(const double* th, double* blk) { mcpx_nl_init(th, blk); }\n"
                    "void oracle_nl_eval(const double* th, const double* z, double* blk) "
                    "{ mcpx_nl_eval(th, z, blk); }\n"
                    "void oracle_nl_eval_theta(const double* th, const double* z, double* dth) "
                    "{ mcpx_nl_eval_theta(th, z, dth); }\n"
                    "const int32_t* oracle_nl_table(int which) {\n"
                    "  switch (which) { case 0: return mcpx_nl_qk_ptr; case 1: return mcpx_nl_qk_idx;\n"
                    "    case 2: return mcpx_nl_rj_ptr; case 3: return mcpx_nl_rj_idx;\n"
                    "    case 4: return mcpx_nl_tc_ptr; case 5: return mcpx_nl_tc_idx;\n"
                    "    case 6: return mcpx_nl_tr_ptr; case 7: return mcpx_nl_tr_idx;\n"
                    "    case 8: return mcpx_nl_band_info; case 9: return mcpx_nl_band_rperm;\n"
                    "    default: return mcpx_nl_band_cperm; }\n}\n")
        tmp = f"{so}.{os.getpid()}.tmp"
        subprocess.run(["gcc", "-O2", "-std=c11", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared",
                        "-o", tmp, src, "-lm"], check=True)
        os.replace(tmp, so)
    L = C.CDLL(so)
    _nl_libs[nl.key] = L
    return L


def _nl_spec(nl) -> OracleNL:
    G = nl_lib(nl)
    G.oracle_nl_table.restype = C.c_void_p
    G.oracle_nl_table.argtypes = [C.c_int]
    fn = lambda f: C.cast(f, C.c_void_p).value
    t = [G.oracle_nl_table(w) for w in range(11)]
    info = (C.c_int32 * 4).from_address(t[8])  # mcpx_nl_band_info of the same generated text
    return OracleNL(fn(G.oracle_nl_init), fn(G.oracle_nl_eval), nl.p, int(nl.has_s), nl.size,
                    int(nl.solvers()["schur"]), *t[:4],
                    fn(G.oracle_nl_eval_theta), *t[4:8], info[0], info[1], info[2], info[3], t[9], t[10])


def solve_batch_nl(nl, theta: np.ndarray, *, x0=None, y0=None, s0=None, params: Params | None = None,
                   trace_len: int = 0, nthreads: int = 1, **kw) -> dict:
    """Oracle of mcpx_solve_batch_module: nl is the problem's codegen.NLSystem."""
    from mcp_amd._abi import FAMILY_NONLINEAR

    theta = np.ascontiguousarray(np.atleast_2d(theta), dtype=np.float64)
    B, ld = theta.shape
    n, m = nl.n, nl.m
    if ld < nl.p:
        raise ValueError(f"theta has {ld} columns, the problem needs {nl.p}")
    prm = params if params is not None else make_params(**kw)
    conv = lambda a, k: None if a is None else np.ascontiguousarray(np.broadcast_to(a, (B, k)), dtype=np.float64)
    x0, y0, s0 = conv(x0, n), conv(y0, m), conv(s0, m)
    words = max(1, (m + 63) // 64)
    r = dict(
        x=np.empty((B, n)), y=np.empty((B, m)), s=np.empty((B, m)), kkt_error=np.empty(B),
        eps=np.empty(B), outer_iters=np.empty(B, np.int32), status=np.empty(B, np.int32),
        newton_iters=np.empty(B, np.int32), active_mask=np.empty((B, words), np.uint64),
        alpha_trace=np.full((B, max(trace_len, 0), 2), 254, np.uint8), fail_reason=np.empty(B, np.uint8),
    )
    out = Out(_ptr(r["x"]), _ptr(r["y"]), _ptr(r["s"]), _ptr(r["kkt_error"]), _ptr(r["eps"]),
              _ptr(r["outer_iters"]), _ptr(r["status"]), _ptr(r["newton_iters"]),
              _ptr(r["active_mask"]), _ptr(r["alpha_trace"]) if trace_len > 0 else None,
              int(trace_len), 0, _ptr(r["fail_reason"]))
    spec = _nl_spec(nl)
    L = lib()
    L.oracle_solve_batch_nl.restype = C.c_int
    L.oracle_solve_batch_nl.argtypes = [C.POINTER(Desc), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.POINTER(Params), C.POINTER(Out), C.c_int, C.POINTER(OracleNL)]
    desc = Desc(FAMILY_NONLINEAR, n, m, 0, B, ld)
    rc = L.oracle_solve_batch_nl(C.byref(desc), _ptr(theta), _ptr(x0), _ptr(y0), _ptr(s0), C.byref(prm),
                                 C.byref(out), int(nthreads), C.byref(spec))
    if rc != 0:
        raise ValueError(f"oracle_solve_batch_nl failed with code {rc}")
    return r


def _sens_lib():
    L = lib()
    if not hasattr(L, "_sens_ready"):
        L.oracle_vjp_batch.restype = C.c_int
        L.oracle_vjp_batch.argtypes = [C.POINTER(Desc)] + [C.c_void_p] * 9 + [C.c_int]
        L.oracle_jvp_batch.restype = C.c_int
        L.oracle_jvp_batch.argtypes = [C.POINTER(Desc), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L._sens_ready = True
    return L


def _f64(a, shape):
    return None if a is None else np.ascontiguousarray(np.broadcast_to(a, shape), dtype=np.float64)


def vjp_batch(family: int, n: int, m: int, theta, x, y, s, gx=None, gy=None, gs=None, nthreads: int = 1):
    """Oracle of mcpx_vjp_batch: returns (dtheta (B, p), status (B,))."""
    theta = np.ascontiguousarray(np.atleast_2d(theta), dtype=np.float64)
    B, ld = theta.shape
    p = theta_dim(family, n, m)
    x, y, s = _f64(x, (B, n)), _f64(y, (B, m)), _f64(s, (B, m))
    gx, gy, gs = _f64(gx, (B, n)), _f64(gy, (B, m)), _f64(gs, (B, m))
    dth = np.empty((B, p))
    st = np.empty(B, np.int32)
    desc = Desc(family, n, m, 0, B, ld)
    rc = _sens_lib().oracle_vjp_batch(C.byref(desc), _ptr(theta), _ptr(x), _ptr(y), _ptr(s), _ptr(gx), _ptr(gy),
                                      _ptr(gs), _ptr(dth), _ptr(st), int(nthreads))
    if rc != 0:
        raise ValueError(f"oracle_vjp_batch failed with code {rc}")
    return dth, st


def jvp_batch(family: int, n: int, m: int, theta, x, y, s, theta_dot, nthreads: int = 1):
    """Oracle of mcpx_jvp_batch: theta_dot (B, K, p) → (zdot (B, K, n+2m), status (B,))."""
    theta = np.ascontiguousarray(np.atleast_2d(theta), dtype=np.float64)
    B, ld = theta.shape
    p = theta_dim(family, n, m)
    td = np.ascontiguousarray(theta_dot, dtype=np.float64).reshape(B, -1, p)
    K = td.shape[1]
    x, y, s = _f64(x, (B, n)), _f64(y, (B, m)), _f64(s, (B, m))
    zd = np.empty((B, K, n + 2 * m))
    st = np.empty(B, np.int32)
    desc = Desc(family, n, m, 0, B, ld)
    rc = _sens_lib().oracle_jvp_batch(C.byref(desc), _ptr(theta), _ptr(x), _ptr(y), _ptr(s), int(K), _ptr(td),
                                      _ptr(zd), _ptr(st), int(nthreads))
    if rc != 0:
        raise ValueError(f"oracle_jvp_batch failed with code {rc}")
    return zd, st


def _sens_nl_lib():
    L = lib()
    if not hasattr(L, "_sens_nl_ready"):
        L.oracle_vjp_batch_nl.restype = C.c_int
        L.oracle_vjp_batch_nl.argtypes = [C.POINTER(Desc)] + [C.c_void_p] * 9 + [C.c_int, C.POINTER(OracleNL)]
        L.oracle_jvp_batch_nl.restype = C.c_int
        L.oracle_jvp_batch_nl.argtypes = [C.POINTER(Desc), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                          C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                          C.POINTER(OracleNL)]
        L._sens_nl_ready = True
    return L


def vjp_batch_nl(nl, theta, x, y, s, gx=None, gy=None, gs=None, nthreads: int = 1):
    """Oracle of mcpx_vjp_batch_module: returns (dtheta (B, p), status (B,))."""
    from mcp_amd._abi import FAMILY_NONLINEAR

    theta = np.ascontiguousarray(np.atleast_2d(theta), dtype=np.float64)
    B, ld = theta.shape
    n, m, p = nl.n, nl.m, nl.p
    x, y, s = _f64(x, (B, n)), _f64(y, (B, m)), _f64(s, (B, m))
    gx, gy, gs = _f64(gx, (B, n)), _f64(gy, (B, m)), _f64(gs, (B, m))
    dth = np.empty((B, p))
    st = np.empty(B, np.int32)
    desc = Desc(FAMILY_NONLINEAR, n, m, 0, B, ld)
    rc = _sens_nl_lib().oracle_vjp_batch_nl(C.byref(desc), _ptr(theta), _ptr(x), _ptr(y), _ptr(s), _ptr(gx),
                                            _ptr(gy), _ptr(gs), _ptr(dth), _ptr(st), int(nthreads),
                                            C.byref(_nl_spec(nl)))
    if rc != 0:
        raise ValueError(f"oracle_vjp_batch_nl failed with code {rc}")
    return dth, st


def jvp_batch_nl(nl, theta, x, y, s, theta_dot, nthreads: int = 1):
    """Oracle of mcpx_jvp_batch_module: theta_dot (B, K, p) → (zdot (B, K, n+2m), status (B,))."""
    from mcp_amd._abi import FAMILY_NONLINEAR

    theta = np.ascontiguousarray(np.atleast_2d(theta), dtype=np.float64)
    B, ld = theta.shape
    n, m, p = nl.n, nl.m, nl.p
    td = np.ascontiguousarray(theta_dot, dtype=np.float64).reshape(B, -1, p)
    K = td.shape[1]
    x, y, s = _f64(x, (B, n)), _f64(y, (B, m)), _f64(s, (B, m))
    zd = np.empty((B, K, n + 2 * m))
    st = np.empty(B, np.int32)
    desc = Desc(FAMILY_NONLINEAR, n, m, 0, B, ld)
    rc = _sens_nl_lib().oracle_jvp_batch_nl(C.byref(desc), _ptr(theta), _ptr(x), _ptr(y), _ptr(s), int(K),
                                            _ptr(td), _ptr(zd), _ptr(st), int(nthreads), C.byref(_nl_spec(nl)))
    if rc != 0:
        raise ValueError(f"oracle_jvp_batch_nl failed with code {rc}")
    return zd, st


def cond_batch(family: int, n: int, m: int, theta, x, y, s, nthreads: int = 1, nl=None):
    """Oracle of mcpx_cond_batch[_module]: the Hager–Higham reciprocal 1-norm condition estimate
    of ∇F_z at (x, y, s) (oracle/ipm_oracle.c cond_estimate) → (rcond (B,), status (B,))."""
    theta = np.ascontiguousarray(np.atleast_2d(theta), dtype=np.float64)
    B, ld = theta.shape
    if nl is not None:
        n, m = nl.n, nl.m
    x, y, s = _f64(x, (B, n)), _f64(y, (B, m)), _f64(s, (B, m))
    rc_ = np.empty(B)
    st = np.empty(B, np.int32)
    L = lib()
    if not hasattr(L, "_cond_ready"):
        L.oracle_cond_batch.restype = C.c_int
        L.oracle_cond_batch.argtypes = [C.POINTER(Desc)] + [C.c_void_p] * 6 + [C.c_int]
        L.oracle_cond_batch_nl.restype = C.c_int
        L.oracle_cond_batch_nl.argtypes = [C.POINTER(Desc)] + [C.c_void_p] * 6 + [C.c_int, C.POINTER(OracleNL)]
        L._cond_ready = True
    args = (_ptr(theta), _ptr(x), _ptr(y), _ptr(s), _ptr(rc_), _ptr(st), int(nthreads))
    if nl is not None:
        from mcp_amd._abi import FAMILY_NONLINEAR

        desc = Desc(FAMILY_NONLINEAR, n, m, 0, B, ld)
        rc = L.oracle_cond_batch_nl(C.byref(desc), *args, C.byref(_nl_spec(nl)))
    else:
        desc = Desc(family, n, m, 0, B, ld)
        rc = L.oracle_cond_batch(C.byref(desc), *args)
    if rc != 0:
        raise ValueError(f"oracle_cond_batch failed with code {rc}")
    return rc_, st
