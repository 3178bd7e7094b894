"""Sensitivities of an MCP solution w.r.t. θ — mirror of the reference's
src/AutoDiff.jl on top of the gfx950 sensitivity kernels (include/mcpx.h
mcpx_vjp_* / mcpx_jvp_*).

    ∂z/∂θ = −(∇F_z)⁻¹ ∇F_θ   at the returned (x, y, s), ∇F_z without tol·I
                              (src/AutoDiff.jl:18-40)

* :func:`rrule` / :func:`solve_pullback` — the ChainRulesCore.rrule of `solve`
  (src/AutoDiff.jl:42-82): the pullback maps (∂x, ∂y, ∂s) to ∂θ with one adjoint
  solve ∇F_zᵀ λ = [∂x; ∂y; ∂s] per instance on the GPU, then the θ' → θ chain
  rule of the traced family map (ThetaMap.vjp) on the host or device.
* :func:`solve_dual` — the ForwardDiff.Dual method of `solve`
  (src/AutoDiff.jl:84-117): solution values plus partials ż = (∂z/∂θ) θ̇.
* :func:`solve_torch` — the same pullback as a torch.autograd.Function, so a
  torch loss over (x, y, s) back-propagates into θ (the Zygote use of the
  reference's rrule, test/runtests.jl:65-85).

Every family is covered: QP / affine through the analytic ∇F_θ of their θ
layouts, nonlinear-family MCPs (the trajectory games of src/game.jl) through
their generated module's ∇F_θ code; one wave per instance up to 64 KKT rows,
one workgroup per instance beyond (include/mcpx.h).

Where ∇F_z is exactly singular the kernels report it per instance
(`status` 1) and return NaN; the reference's pivoted QR would return a basic
least-squares solution there.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Any

import numpy as np


class NoTangent:
    """ChainRulesCore.NoTangent(): the pullback's tangent for solve, solver_type, mcp."""

    def __repr__(self):
        return "NoTangent()"

    def __eq__(self, other):
        return isinstance(other, NoTangent)

    __hash__ = object.__hash__


def _require_sensitivities(mcp) -> None:
    # src/AutoDiff.jl:19-23
    if not getattr(mcp, "compute_sensitivities", False):
        raise ValueError("Missing sensitivities. Set `compute_sensitivities = True` when constructing the "
                         "PrimalDualMCP.")


def _module(mcp):
    """The generated module of a nonlinear-family MCP (its ∇F_θ is the generated
    mcpx_nl_eval_theta, src/mcp.jl:122-147), else None (QP / affine kernels)."""
    return mcp.module() if getattr(mcp, "nl", None) is not None else None


def _is_torch(a) -> bool:
    return type(a).__module__.startswith("torch")


def _get(d, k):
    if d is None:
        return None
    if isinstance(d, dict):
        return d.get(k)
    return getattr(d, k, None)


def solve_pullback(solution, dx=None, dy=None, ds=None, *, num_devices: int = 0, return_status: bool = False):
    """∂θ = ∂z∂θ[x]ᵀ ∂x + ∂z∂θ[y]ᵀ ∂y + ∂z∂θ[s]ᵀ ∂s (src/AutoDiff.jl:59-76) for a solution
    returned by `solve(InteriorPoint(), mcp, θ)`.  None cotangents are zero.
    Shapes follow the solution: single instance → (p,), batch → (B, p); torch
    solutions stay on device (enqueued on the current stream)."""
    from .batch import vjp_batch, vjp_batch_device

    mcp = solution.mcp
    _require_sensitivities(mcp)
    n, m = mcp.unconstrained_dimension, mcp.constrained_dimension
    θ = solution.θ
    if _is_torch(θ):
        import torch

        th = θ if θ.dim() == 2 else θ[None, :]
        tp = mcp.theta_map(th).contiguous()
        f = lambda t: None if t is None else t.to(torch.float64).reshape(th.shape[0], -1).contiguous()
        dtp, st = vjp_batch_device(mcp.family, n, m, tp, f(solution.x), f(solution.y), f(solution.s),
                                   f(dx), f(dy), f(ds), module=_module(mcp))
        dθ = mcp.theta_map.vjp(th, dtp)
        return (dθ, st) if return_status else dθ
    th = np.asarray(θ, dtype=np.float64)
    single = th.ndim == 1
    th2 = np.atleast_2d(th)
    B = th2.shape[0]
    tp = mcp.theta_map(th2)
    f = lambda a, k: None if a is None else np.asarray(a, np.float64).reshape(B, k)
    dtp, st = vjp_batch(mcp.family, n, m, tp, f(solution.x, n), f(solution.y, m), f(solution.s, m),
                        f(dx, n), f(dy, m), f(ds, m), num_devices=num_devices, module=_module(mcp))
    dθ = mcp.theta_map.vjp(th2, dtp)
    if single:
        dθ, st = dθ[0], st[0]
    return (dθ, st) if return_status else dθ


def rrule(f, solver_type, mcp, θ=None, **kwargs):
    """ChainRulesCore.rrule(solve, solver_type, mcp, θ; kwargs...) (src/AutoDiff.jl:42-82).
    Returns (solution, pullback); pullback(∂solution) → (NoTangent(), NoTangent(),
    NoTangent(), ∂θ) where ∂solution has fields / keys x, y, s (missing = zero).

    rrule(solve, game, θ; kwargs...) differentiates a game solve (src/game.jl:196-212,
    which calls solve(solver_type, game.mcp, θ) — the path Zygote takes through
    examples/utils.jl:233-269): the solution is the GameSolution, ∂solution carries
    `variables` (x, y, s) and/or `primals` (one block per player, added into ∂x);
    pullback → (NoTangent(), NoTangent(), ∂θ)."""
    from .api import ParametricGame, solve

    if f is not solve:
        raise TypeError("rrule is defined for mcp_amd.api.solve only")
    if isinstance(solver_type, ParametricGame):
        return _game_rrule(solver_type, mcp, **kwargs)
    _require_sensitivities(mcp)
    solution = solve(solver_type, mcp, θ, **kwargs)

    def solve_pullback_(dsolution):
        dθ = solve_pullback(solution, _get(dsolution, "x"), _get(dsolution, "y"), _get(dsolution, "s"))
        return NoTangent(), NoTangent(), NoTangent(), dθ

    return solution, solve_pullback_


def _game_rrule(game, θ, solver_type=None, **kwargs):
    from .api import GameSolution, InteriorPoint, solve

    mcp = game.mcp
    _require_sensitivities(mcp)
    sol_mcp = solve(solver_type or InteriorPoint(), mcp, θ, **kwargs)  # src/game.jl:196-212
    ends = np.cumsum(game.dims["x"])
    starts = np.concatenate([[0], ends[:-1]])
    x = sol_mcp.x
    solution = GameSolution([x[..., a:b] for a, b in zip(starts, ends)],
                            {"x": sol_mcp.x, "y": sol_mcp.y, "s": sol_mcp.s}, sol_mcp.kkt_error, sol_mcp.status)

    def game_pullback(dsolution):
        var = _get(dsolution, "variables") or {}
        dx, dy, ds = _get(var, "x"), _get(var, "y"), _get(var, "s")
        prim = _get(dsolution, "primals")
        if prim is not None:  # ∂primals[i] is the cotangent of x[starts[i]:ends[i]]
            acc = np.zeros(np.shape(x)) if dx is None else np.array(dx, np.float64)
            for a, b, g in zip(starts, ends, prim):
                if g is not None:
                    acc[..., a:b] += np.asarray(g, np.float64)
            dx = acc
        return NoTangent(), NoTangent(), solve_pullback(sol_mcp, dx, dy, ds)

    return solution, game_pullback


@dataclass
class DualSolution:
    """The NamedTuple of src/AutoDiff.jl:116 with ForwardDiff.Dual fields split into
    value and partials: x / y / s values and x_partials (…, n, K), y_partials,
    s_partials.  As the reference (src/AutoDiff.jl:110-114), the value of `s` is
    the solution's **y** (a reference quirk kept for parity; `s_value_true` holds
    the solver's s)."""

    status: Any
    kkt_error: Any
    eps: Any
    x: Any
    y: Any
    s: Any
    x_partials: Any
    y_partials: Any
    s_partials: Any
    s_value_true: Any = None
    sensitivity_status: Any = None


def solve_dual(solver_type, mcp, θ, θ_partials, *, num_devices: int = 0, **kwargs) -> DualSolution:
    """solve(solver_type, mcp, θ::Vector{<:Dual}) (src/AutoDiff.jl:84-117).
    θ: (p,) or (B, p) values; θ_partials: (p, K) or (B, p, K) — the partials of
    each θ entry, as ForwardDiff.partials.(θ) stacked."""
    from .api import solve
    from .batch import jvp_batch

    _require_sensitivities(mcp)
    n, m = mcp.unconstrained_dimension, mcp.constrained_dimension
    th = np.asarray(θ, np.float64)
    single = th.ndim == 1
    th2 = np.atleast_2d(th)
    B, p_in = th2.shape
    tpar = np.asarray(θ_partials, np.float64).reshape(B, p_in, -1)
    sol = solve(solver_type, mcp, th2, num_devices=num_devices, **kwargs)  # forward pass (:94)
    tp = mcp.theta_map(th2)
    tdot = mcp.theta_map.jvp(th2, np.ascontiguousarray(np.swapaxes(tpar, 1, 2)))  # (B, K, p')
    zd, st = jvp_batch(mcp.family, n, m, tp, sol.x, sol.y, sol.s, tdot, num_devices=num_devices,
                       module=_module(mcp))  # (B, K, N)
    zp = np.swapaxes(zd, 1, 2)  # (B, N, K): z_p = ∂z∂θ · θ_p (:98)
    xp, yp, sp_ = zp[:, :n], zp[:, n:n + m], zp[:, n + m:]
    pick = (lambda a: a[0]) if single else (lambda a: a)
    return DualSolution(pick(sol.status), pick(sol.kkt_error), pick(sol.eps), pick(sol.x), pick(sol.y),
                        pick(sol.y),  # src/AutoDiff.jl:112: Dual(solution.y, s partials)
                        pick(xp), pick(yp), pick(sp_), s_value_true=pick(sol.s), sensitivity_status=pick(st))


# ---------------------------------------------------------------------------
# torch autograd


def _autograd_fn():
    import torch

    class _SolveFn(torch.autograd.Function):
        @staticmethod
        def forward(ctx, θ, mcp, kwargs):
            from .api import solve

            kw = dict(kwargs)
            sol = solve(kw.pop("solver_type"), mcp, θ.detach(), **kw)
            ctx.solution = sol
            ctx.mark_non_differentiable(sol.status)
            return sol.x.clone(), sol.y.clone(), sol.s.clone(), sol.status

        @staticmethod
        def backward(ctx, gx, gy, gs, _gstatus):
            dθ = solve_pullback(ctx.solution, gx, gy, gs)
            return dθ.reshape(ctx.solution.θ.shape), None, None

    return _SolveFn


_FN = None


def solve_torch(mcp, θ, *, solver_type=None, **kwargs):
    """Differentiable batched solve on device: θ a (B, p) float64 HIP tensor
    (requires_grad allowed) → (x, y, s, status) with x, y, s differentiable
    w.r.t. θ through the GPU pullback (src/AutoDiff.jl rrule)."""
    global _FN
    from .api import InteriorPoint

    _require_sensitivities(mcp)
    if not (_is_torch(θ) and θ.is_cuda):
        raise ValueError("solve_torch needs a HIP (cuda) tensor θ")
    if _FN is None:
        _FN = _autograd_fn()
    kw = dict(kwargs, solver_type=solver_type or InteriorPoint())
    return _FN.apply(θ if θ.dim() == 2 else θ[None, :], mcp, kw)
