"""mcp_amd — MI355X-native batched interior-point MCP solver.

Drop-in for the Newton-step hot path of MixedComplementarityProblems.jl
(TianyuQ/MCP): the reference's API (PrimalDualMCP, solve(InteriorPoint(), …))
on top of hand-written gfx950 HIP kernels behind the C ABI of include/mcpx.h.
"""

from . import _abi  # noqa: F401
from ._lib import MCPXError  # noqa: F401

__version__ = "1.1.0"
