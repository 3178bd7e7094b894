"""ctypes mirror of include/mcpx.h (struct layouts and constants only — no loading)."""

import ctypes as C

MCPX_OK = 0
MCPX_EINVAL = -1
MCPX_EHIP = -2
MCPX_ENODEV = -3
MCPX_EUNSUPPORTED = -4

STATUS_SOLVED = 0
STATUS_FAILED = 1
# fail_reason bits (include/mcpx.h MCPX_FAIL_*)
FAIL_LINSOLVE = 1
FAIL_LINESEARCH = 2
FAIL_MAX_OUTER = 4
FAIL_INPUT = 8  # SCHUR on an affine θ with a nonzero S block: not solved

FAMILY_QP = 0
FAMILY_AFFINE = 1
FAMILY_NONLINEAR = 2  # generated device code per problem (mcp_amd/codegen.py)

MAX_KKT_DIM = 64
MAX_WG_KKT_DIM = 768  # MCPX_MAX_WG_KKT_DIM: workgroup-per-instance kernels (QP / affine)
MAX_WG_SCHUR_N = 128  # wg::kGjMax: the QP family's workgroup SCHUR kernels (csrc/gj_vr.hpp)
KERNEL_AUTO, KERNEL_WAVE, KERNEL_WORKGROUP, KERNEL_MULTIWAVE, KERNEL_BAND = 0, 1, 2, 3, 4
KERNELS = {"auto": KERNEL_AUTO, "wave": KERNEL_WAVE, "workgroup": KERNEL_WORKGROUP, "multiwave": KERNEL_MULTIWAVE,
           "band": KERNEL_BAND}
JVP_RHS = 8  # MCPX_JVP_RHS: partials per factorisation of the JVP kernel
MODULE_VJP, MODULE_JVP = 6, 7  # MCPX_MODULE_VJP / _JVP: sensitivity-kernel bits of a module's kernel mask
MODULE_SCHUR_MW = 8  # MCPX_MODULE_SCHUR_MW: the 4-wave SCHUR solve kernel
MODULE_BAND, MODULE_BAND_AUTO = 9, 10  # MCPX_MODULE_BAND / _BAND_AUTO: the band SCHUR kernel

LINSOLVE_REDUCED = 0
LINSOLVE_DENSE = 1
LINSOLVE_SCHUR = 2
LINEAR_SOLVERS = {"reduced": LINSOLVE_REDUCED, "dense": LINSOLVE_DENSE, "schur": LINSOLVE_SCHUR}
MAX_INNER_ITERS = 128
MAX_LS_TRIALS = 64

ERRORS = {
    MCPX_EINVAL: "invalid argument",
    MCPX_EHIP: "HIP runtime error",
    MCPX_ENODEV: "no usable gfx950 device",
    MCPX_EUNSUPPORTED: "unsupported size",
}


class Params(C.Structure):
    """mcpx_params — solver keyword arguments (reference src/solver.jl:42-50)."""

    _fields_ = [
        ("tol", C.c_double),
        ("tightening_rate", C.c_double),
        ("loosening_rate", C.c_double),
        ("min_stepsize", C.c_double),
        ("tau", C.c_double),
        ("decay", C.c_double),
        ("max_inner_iters", C.c_int32),
        ("max_outer_iters", C.c_int32),
        ("linear_solver", C.c_int32),
        ("kernel", C.c_int32),
    ]


class Desc(C.Structure):
    _fields_ = [
        ("family", C.c_int32),
        ("n", C.c_int32),
        ("m", C.c_int32),
        ("pad_", C.c_int32),
        ("batch", C.c_int64),
        ("theta_ld", C.c_int64),
    ]


class Out(C.Structure):
    _fields_ = [
        ("x", C.c_void_p),
        ("y", C.c_void_p),
        ("s", C.c_void_p),
        ("kkt_error", C.c_void_p),
        ("eps", C.c_void_p),
        ("outer_iters", C.c_void_p),
        ("status", C.c_void_p),
        ("newton_iters", C.c_void_p),
        ("active_mask", C.c_void_p),
        ("alpha_trace", C.c_void_p),
        ("trace_len", C.c_int32),
        ("pad_", C.c_int32),
        ("fail_reason", C.c_void_p),
    ]


class Cotangent(C.Structure):
    """mcpx_cotangent: ∂l/∂z = a·z + b per block (b device arrays or NULL)."""
    _fields_ = [
        ("ax", C.c_double),
        ("ay", C.c_double),
        ("as_", C.c_double),
        ("bx", C.c_void_p),
        ("by", C.c_void_p),
        ("bs", C.c_void_p),
    ]


def make_params(tol=1e-4, max_inner_iters=20, max_outer_iters=50, tightening_rate=0.1,
                loosening_rate=0.5, min_stepsize=1e-4, tau=0.995, decay=0.5,
                linear_solver="reduced", kernel="auto") -> Params:
    """Defaults exactly as src/solver.jl:42-48 and :127.  `linear_solver` plays the
    role of the reference's `linear_solve_algorithm` kwarg (src/solver.jl:50);
    `kernel` picks the one-wave or the workgroup-per-instance kernels (MCPX_KERNEL_*)."""
    ls = LINEAR_SOLVERS[linear_solver] if isinstance(linear_solver, str) else int(linear_solver)
    kk = KERNELS[kernel] if isinstance(kernel, str) else int(kernel)
    return Params(float(tol), float(tightening_rate), float(loosening_rate), float(min_stepsize),
                  float(tau), float(decay), int(max_inner_iters), int(max_outer_iters), ls, kk)


def theta_dim(family: int, n: int, m: int) -> int:
    if family == FAMILY_QP:
        return n * n + m * n + m + n
    if family == FAMILY_AFFINE:
        return n * n + 2 * n * m + m * m + n + m
    if family == FAMILY_NONLINEAR:
        raise ValueError("a nonlinear MCP's θ dimension is its own (NLSystem.p, mcpx_module_dims)")
    raise ValueError(f"unknown family {family}")
