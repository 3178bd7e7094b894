"""Loader for the in-tree HIP extension mcp_amd/libmcpx.so (C ABI: include/mcpx.h).

The product path has no CPU fallback: if the library is missing or no gfx950
device is visible, calls fail loudly (MCPXError).
"""

from __future__ import annotations

import ctypes as C
import os

from . import _abi

_HERE = os.path.dirname(os.path.abspath(__file__))
# MCPX_LIB_PATH: load an alternative in-tree build (kernel A/B experiments, tools/)
LIB_PATH = os.environ.get("MCPX_LIB_PATH") or os.path.join(_HERE, "libmcpx.so")
_lib = None


class MCPXError(RuntimeError):
    """Raised for a negative return code of the C ABI (API misuse / HIP error)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"mcpx error {code} ({_abi.ERRORS.get(code, '?')}): {msg}")
        self.code = code


EXPORTS = ("mcpx_version", "mcpx_last_error", "mcpx_default_params", "mcpx_theta_dim",
           "mcpx_device_count", "mcpx_solve_batch", "mcpx_solve_batch_device", "mcpx_vjp_batch",
           "mcpx_vjp_batch_device", "mcpx_jvp_batch", "mcpx_jvp_batch_device", "mcpx_module_load",
           "mcpx_module_dims", "mcpx_module_unload", "mcpx_solve_batch_module", "mcpx_solve_batch_module_device",
           "mcpx_host_register", "mcpx_host_unregister", "mcpx_vjp_batch_module", "mcpx_vjp_batch_module_device",
           "mcpx_jvp_batch_module", "mcpx_jvp_batch_module_device", "mcpx_solve_vjp_batch_device",
           "mcpx_cond_batch", "mcpx_cond_batch_device", "mcpx_cond_batch_module", "mcpx_cond_batch_module_device",
           "mcpx_debug_canary_violations")


ABI_MAJOR = 2  # include/mcpx.h MCPX_VERSION / 10000


def lib():
    """Load libmcpx.so (building it first if only the sources are present)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        from . import build as _build
        _build.build()
    L = C.CDLL(LIB_PATH)
    L.mcpx_version.restype = C.c_int
    if L.mcpx_version() // 10000 != ABI_MAJOR:  # mcpx_out's layout is part of the major version
        raise RuntimeError(f"{LIB_PATH}: ABI {L.mcpx_version()} does not match this package's major {ABI_MAJOR}")
    L.mcpx_last_error.restype = C.c_char_p
    L.mcpx_default_params.argtypes = [C.POINTER(_abi.Params)]
    L.mcpx_theta_dim.restype = C.c_int64
    L.mcpx_theta_dim.argtypes = [C.c_int32, C.c_int32, C.c_int32]
    L.mcpx_device_count.restype = C.c_int
    L.mcpx_debug_canary_violations.restype = C.c_int64
    L.mcpx_solve_batch.restype = C.c_int
    L.mcpx_solve_batch.argtypes = [C.POINTER(_abi.Desc), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                   C.POINTER(_abi.Params), C.c_int, C.POINTER(_abi.Out)]
    L.mcpx_solve_batch_device.restype = C.c_int
    L.mcpx_solve_batch_device.argtypes = [C.POINTER(_abi.Desc), C.c_void_p, C.c_void_p, C.c_void_p,
                                          C.c_void_p, C.POINTER(_abi.Params), C.POINTER(_abi.Out),
                                          C.c_void_p]
    P = C.c_void_p
    L.mcpx_vjp_batch.restype = C.c_int
    L.mcpx_vjp_batch.argtypes = [C.POINTER(_abi.Desc), P, P, P, P, P, P, P, C.c_int, P, P]
    L.mcpx_vjp_batch_device.restype = C.c_int
    L.mcpx_vjp_batch_device.argtypes = [C.POINTER(_abi.Desc), P, P, P, P, P, P, P, P, P, P]
    L.mcpx_jvp_batch.restype = C.c_int
    L.mcpx_jvp_batch.argtypes = [C.POINTER(_abi.Desc), P, P, P, P, C.c_int32, P, C.c_int, P, P]
    L.mcpx_jvp_batch_device.restype = C.c_int
    L.mcpx_jvp_batch_device.argtypes = [C.POINTER(_abi.Desc), P, P, P, P, C.c_int32, P, P, P, P]
    L.mcpx_solve_vjp_batch_device.restype = C.c_int
    L.mcpx_solve_vjp_batch_device.argtypes = [C.POINTER(_abi.Desc), P, P, P, P, C.POINTER(_abi.Params),
                                              C.POINTER(_abi.Out), C.POINTER(_abi.Cotangent), P, P, C.c_void_p]
    I32P = C.POINTER(C.c_int32)
    L.mcpx_module_load.restype = C.c_int
    L.mcpx_module_load.argtypes = [C.c_char_p, C.POINTER(C.c_void_p)]
    L.mcpx_module_dims.restype = C.c_int
    L.mcpx_module_dims.argtypes = [C.c_void_p, I32P, I32P, I32P, I32P]
    L.mcpx_module_unload.restype = None
    L.mcpx_module_unload.argtypes = [C.c_void_p]
    L.mcpx_solve_batch_module.restype = C.c_int
    L.mcpx_solve_batch_module.argtypes = [C.c_void_p, C.POINTER(_abi.Desc), P, P, P, P, C.POINTER(_abi.Params),
                                          C.c_int, C.POINTER(_abi.Out)]
    L.mcpx_solve_batch_module_device.restype = C.c_int
    L.mcpx_solve_batch_module_device.argtypes = [C.c_void_p, C.POINTER(_abi.Desc), P, P, P, P,
                                                 C.POINTER(_abi.Params), C.POINTER(_abi.Out), C.c_void_p]
    L.mcpx_vjp_batch_module.restype = C.c_int
    L.mcpx_vjp_batch_module.argtypes = [C.c_void_p, C.POINTER(_abi.Desc), P, P, P, P, P, P, P, C.c_int, P, P]
    L.mcpx_vjp_batch_module_device.restype = C.c_int
    L.mcpx_vjp_batch_module_device.argtypes = [C.c_void_p, C.POINTER(_abi.Desc), P, P, P, P, P, P, P, P, P, P]
    L.mcpx_jvp_batch_module.restype = C.c_int
    L.mcpx_jvp_batch_module.argtypes = [C.c_void_p, C.POINTER(_abi.Desc), P, P, P, P, C.c_int32, P, C.c_int, P, P]
    L.mcpx_jvp_batch_module_device.restype = C.c_int
    L.mcpx_jvp_batch_module_device.argtypes = [C.c_void_p, C.POINTER(_abi.Desc), P, P, P, P, C.c_int32, P, P, P,
                                               P]
    L.mcpx_cond_batch.restype = C.c_int
    L.mcpx_cond_batch.argtypes = [C.POINTER(_abi.Desc), P, P, P, P, C.c_int, P, P]
    L.mcpx_cond_batch_device.restype = C.c_int
    L.mcpx_cond_batch_device.argtypes = [C.POINTER(_abi.Desc), P, P, P, P, P, P, P]
    L.mcpx_cond_batch_module.restype = C.c_int
    L.mcpx_cond_batch_module.argtypes = [C.c_void_p, C.POINTER(_abi.Desc), P, P, P, P, C.c_int, P, P]
    L.mcpx_cond_batch_module_device.restype = C.c_int
    L.mcpx_cond_batch_module_device.argtypes = [C.c_void_p, C.POINTER(_abi.Desc), P, P, P, P, P, P, P]
    L.mcpx_host_register.restype = C.c_int
    L.mcpx_host_register.argtypes = [C.c_void_p, C.c_size_t]
    L.mcpx_host_unregister.restype = C.c_int
    L.mcpx_host_unregister.argtypes = [C.c_void_p]
    _lib = L
    return L


def check(rc: int) -> None:
    if rc != 0:
        raise MCPXError(rc, lib().mcpx_last_error().decode(errors="replace"))
