"""Host-side mirror of the reference API: PrimalDualMCP, InteriorPoint, solve,
ParametricGame, OptimizationProblem.

The reference builds an MCP by tracing the user's G/H (or K, or a game) with
Symbolics and compiling F!/∇F_z!/∇F_θ! callbacks that its solver calls per
Newton step (src/mcp.jl:27-153, src/game.jl:47-157).  Here the tracing is done
once, at construction, with sympy (the Symbolics analogue available in this
image), and the traced system is classified into a problem *family* that the
gfx950 kernels evaluate on device per instance (include/mcpx.h):

* MCPX_FAMILY_QP      when G = M x − ϕ − Aᵀ y and H = A x − b (∂H/∂y = 0 and
                      ∂G/∂y = −(∂H/∂x)ᵀ): θ' = [vec(M); vec(A); b; ϕ];
* MCPX_FAMILY_AFFINE  any G, H affine in (x, y):
                      θ' = [vec(P); vec(Q); vec(R); vec(S); g; h].

The coefficients may depend on θ arbitrarily; the θ → θ' map is compiled into
a sparse linear part (gathers/scaled adds, which is what every benchmark family
is) plus lambdified residual expressions, and is evaluated per batch with numpy
(host θ) or torch (device θ).

* MCPX_FAMILY_NONLINEAR  any other G/H — e.g. the reference's trajectory
                      games (examples/lane_change.jl): G, H and their Jacobian
                      blocks become device code generated per problem
                      (mcp_amd/codegen.py, the build_function analogue), which
                      the kernel evaluates every Newton step; θ' = θ.

solve() keeps the reference's keyword arguments and result fields
(src/solver.jl:35-51,121), including the in-place update of caller-supplied
x₀/y₀/s₀ (Appendix A.2).  Every solve runs the HIP kernel through the C ABI;
there is no CPU fallback.
"""

from __future__ import annotations

import math
import warnings
from dataclasses import dataclass, field
from typing import Any, Callable, Sequence

import numpy as np

from . import _abi

# ---------------------------------------------------------------------------
# symbolic tracing (the SymbolicTracingUtils.make_variables analogue)


def _sp():
    import sympy

    return sympy


def make_variables(name: str, n: int) -> np.ndarray:
    """n scalar symbols `name_1 … name_n` as a numpy object array (so that user
    code written with numpy operators — M @ x, x.sum(), x ** 2 — traces)."""
    sp = _sp()
    out = np.empty(int(n), dtype=object)
    for i in range(int(n)):
        out[i] = sp.Symbol(f"{name}_{i + 1}", real=True)
    return out


def _as_exprs(v, what: str) -> list:
    sp = _sp()
    arr = np.asarray(v, dtype=object).reshape(-1)
    return [sp.sympify(e) for e in arr]


class NotAffineError(NotImplementedError):
    """G/H not affine in (x, y): the MCP goes to the nonlinear family (generated device code)."""


def _affine_rows(rows: list, zs: list, what: str):
    """Coefficient matrix C[i][j] = ∂row_i/∂z_j and constants c_i = row_i(z = 0),
    as sympy expressions in θ; raises NotAffineError for higher-degree terms."""
    sp = _sp()
    C, c = [], []
    for i, e in enumerate(rows):
        e = sp.expand(e)
        # the polynomial in the variables this row uses only (a Poly over all n + m generators is
        # a recursion as deep as their number: past ~1,000 it overflows, e.g. the lane change at T = 30)
        # (the coefficients of the other variables: the zero of the polynomial's domain, as
        # coeff_monomial gives over all generators — e.g. Float 0.0 for a row with float
        # constants, which the QP / affine classification then sees exactly as before)
        if zs:
            fs = e.free_symbols
            used = [z for z in zs if z in fs]
            try:
                poly = sp.Poly(e, *(used or zs[:1]))
            except sp.PolynomialError as exc:
                raise NotAffineError(f"{what}[{i}] is not polynomial in the decision variables: {e}") from exc
            if poly.total_degree() > 1:
                raise NotAffineError(f"{what}[{i}] is not affine in the decision variables (degree "
                                     f"{poly.total_degree()}); general nonlinear G/H is SURVEY.md §8(f) #2")
            zero = poly.domain.to_sympy(poly.domain.zero)
            C.append([poly.coeff_monomial(z) if z in fs else zero for z in zs])
            c.append(poly.coeff_monomial(1))
        else:
            C.append([])
            c.append(e)
    return C, c


# ---------------------------------------------------------------------------
# θ → θ' (family parameter) map


class ThetaMap:
    """θ' = T(θ), compiled from sympy expressions in θ.

    Linear entries (every benchmark family: θ' entries are θ_k, −θ_k, constants, or
    small linear combinations) are stored as (dst, src, coef) terms and evaluated
    as gathers + scaled adds; anything else is lambdified.  `vjp` is the adjoint
    map (∂θ'/∂θ)ᵀ used by the sensitivity path."""

    def __init__(self, exprs: Sequence, thetas: Sequence):
        sp = _sp()
        self.p_in = len(thetas)
        self.p_out = len(exprs)
        const = np.zeros(self.p_out)
        dst, src, coef, nonlin = [], [], [], []
        for i, e in enumerate(exprs):
            e = sp.expand(sp.sympify(e))
            if e.is_number:
                const[i] = float(e)
                continue
            fs = [t for t in thetas if t in e.free_symbols]
            lin = False
            try:
                poly = sp.Poly(e, *fs)
                lin = poly.total_degree() <= 1 and all(poly.coeff_monomial(t).is_number for t in fs)
            except sp.PolynomialError:
                pass
            if lin:
                for t in fs:
                    cval = float(poly.coeff_monomial(t))
                    if cval != 0.0:
                        dst.append(i)
                        src.append(thetas.index(t))
                        coef.append(cval)
                const[i] = float(poly.coeff_monomial(1))
            else:
                nonlin.append((i, e))
        self.const = const
        self.dst = np.asarray(dst, np.int64)
        self.src = np.asarray(src, np.int64)
        self.coef = np.asarray(coef, np.float64)
        # terms grouped by their rank within the destination entry (fixed summation order)
        rank = np.zeros(len(dst), np.int64)
        seen: dict = {}
        for t, d in enumerate(dst):
            rank[t] = seen.get(d, 0)
            seen[d] = rank[t] + 1
        self._groups = [np.nonzero(rank == r)[0] for r in range(int(rank.max()) + 1 if len(dst) else 0)]
        self._has_lin = np.zeros(self.p_out, bool)
        self._has_lin[self.dst] = True
        thetas = list(thetas)
        self._nonlin = [(i, sp.lambdify(thetas, e, "numpy"), e) for i, e in nonlin]
        self._nonlin_grad = [(i, [(thetas.index(t), sp.lambdify(thetas, sp.diff(e, t), "numpy"))
                                  for t in e.free_symbols if t in thetas]) for i, e in nonlin]
        self._thetas = thetas
        # identity fast path: θ' is a permutation-free copy of θ
        self.identity = (not nonlin and self.p_in == self.p_out and len(dst) == self.p_out
                         and np.array_equal(self.dst, np.arange(self.p_out))
                         and np.array_equal(self.src, np.arange(self.p_out)) and np.all(self.coef == 1.0)
                         and np.all(const == 0.0))

    # -- evaluation ---------------------------------------------------------
    def __call__(self, theta):
        """theta: (B, p) numpy array or torch tensor → (B, p') of the same kind."""
        if _is_torch(theta):
            return self._eval_torch(theta)
        th = np.ascontiguousarray(theta, dtype=np.float64)
        if th.ndim == 1:
            th = th[None, :]
        if th.shape[1] != self.p_in:
            raise ValueError(f"θ has dimension {th.shape[1]}, the MCP was built with parameter_dimension={self.p_in}")
        if self.identity:
            return th.copy()
        B = th.shape[0]
        out = np.empty((B, self.p_out))
        out[:, ~self._has_lin] = self.const[~self._has_lin]
        for r, g in enumerate(self._groups):
            d, s, c = self.dst[g], self.src[g], self.coef[g]
            term = th[:, s] * c
            if r == 0:
                out[:, d] = term
            else:
                out[:, d] += term
        cl = self._has_lin & (self.const != 0.0)
        out[:, cl] += self.const[cl]
        if self._nonlin:
            cols = [th[:, k] for k in range(self.p_in)]
            for i, f, _ in self._nonlin:
                out[:, i] = np.broadcast_to(f(*cols), (B,))
        return out

    def _eval_torch(self, theta):
        import torch

        th = theta if theta.dim() == 2 else theta[None, :]
        if th.shape[1] != self.p_in:
            raise ValueError(f"θ has dimension {th.shape[1]}, the MCP was built with parameter_dimension={self.p_in}")
        th = th.to(torch.float64).contiguous()
        if self.identity:
            return th.clone()
        dev = th.device
        B = th.shape[0]
        out = torch.empty(B, self.p_out, dtype=torch.float64, device=dev)
        nl = torch.from_numpy(np.nonzero(~self._has_lin)[0]).to(dev)
        out[:, nl] = torch.from_numpy(self.const[~self._has_lin]).to(dev)
        for r, g in enumerate(self._groups):
            d = torch.from_numpy(self.dst[g]).to(dev)
            s = torch.from_numpy(self.src[g]).to(dev)
            c = torch.from_numpy(self.coef[g]).to(dev)
            term = th[:, s] * c
            if r == 0:
                out[:, d] = term
            else:
                out[:, d] += term
        cl = self._has_lin & (self.const != 0.0)
        if cl.any():
            idx = torch.from_numpy(np.nonzero(cl)[0]).to(dev)
            out[:, idx] += torch.from_numpy(self.const[cl]).to(dev)
        if self._nonlin:  # rare: evaluated on the host and uploaded
            host = th.cpu().numpy()
            cols = [host[:, k] for k in range(self.p_in)]
            for i, f, _ in self._nonlin:
                out[:, i] = torch.from_numpy(np.array(np.broadcast_to(f(*cols), (B,)), dtype=np.float64)).to(dev)
        return out

    def vjp(self, theta, g_out):
        """(∂θ'/∂θ)ᵀ g_out per instance: (B, p') → (B, p); numpy or torch."""
        if _is_torch(g_out):
            import torch

            dev = g_out.device
            B = g_out.shape[0]
            res = torch.zeros(B, self.p_in, dtype=torch.float64, device=dev)
            if len(self.dst):
                contrib = g_out[:, torch.from_numpy(self.dst).to(dev)] * torch.from_numpy(self.coef).to(dev)
                res.index_add_(1, torch.from_numpy(self.src).to(dev), contrib)
            if self._nonlin_grad:
                host = self.vjp_nonlin(theta.cpu().numpy(), g_out.cpu().numpy())
                res += torch.from_numpy(host).to(dev)
            return res
        g = np.atleast_2d(np.asarray(g_out, np.float64))
        B = g.shape[0]
        res = np.zeros((B, self.p_in))
        if len(self.dst):
            np.add.at(res.T, self.src, (g[:, self.dst] * self.coef).T)
        if self._nonlin_grad:
            res += self.vjp_nonlin(np.atleast_2d(theta), g)
        return res

    def jvp(self, theta, t_in):
        """(∂θ'/∂θ) θ̇ per instance and tangent: (B, K, p) → (B, K, p') (host numpy),
        the forward-mode counterpart of `vjp` (src/AutoDiff.jl:84-100)."""
        td = np.asarray(t_in, np.float64)
        B, K = td.shape[0], td.shape[1]
        out = np.zeros((B, K, self.p_out))
        if len(self.dst):
            np.add.at(np.moveaxis(out, 2, 0), self.dst, np.moveaxis(td[:, :, self.src] * self.coef, 2, 0))
        if self._nonlin_grad:
            th = np.atleast_2d(np.asarray(theta, np.float64))
            cols = [th[:, k] for k in range(self.p_in)]
            for i, grads in self._nonlin_grad:
                for k, f in grads:
                    out[:, :, i] += np.broadcast_to(f(*cols), (B,))[:, None] * td[:, :, k]
        return out

    def vjp_nonlin(self, theta, g):
        B = g.shape[0]
        res = np.zeros((B, self.p_in))
        cols = [theta[:, k] for k in range(self.p_in)]
        for i, grads in self._nonlin_grad:
            for k, f in grads:
                res[:, k] += g[:, i] * np.broadcast_to(f(*cols), (B,))
        return res


def _is_torch(a) -> bool:
    return type(a).__module__.startswith("torch")


# ---------------------------------------------------------------------------
# PrimalDualMCP


class PrimalDualMCP:
    """The reference's `PrimalDualMCP` (src/mcp.jl:13-24) for
        0 = G(x, y; θ),   0 ≤ H(x, y; θ) ⟂ y ≥ 0,
    with the primal-dual system F = [G; H − s; s⊙y − ϵ] (src/mcp.jl:72-80).

    Constructors, as in the reference:
      PrimalDualMCP(G, H, unconstrained_dimension=, constrained_dimension=,
                    parameter_dimension=)                          (src/mcp.jl:27-52)
      PrimalDualMCP(K, lower_bounds, upper_bounds, parameter_dimension=)
                    K(z; θ) ⟂ z̲ ≤ z ≤ z̅, bounds −Inf/0 below, Inf above  (:155-177)
      PrimalDualMCP.from_symbolic(G_sym, H_sym, x_sym, y_sym, θ_sym)    (:55-70)
      PrimalDualMCP.from_symbolic_K(K_sym, z_sym, θ_sym, lower, upper)  (:182-210)
    G/H are called as G(x, y, θ=θ) (Julia: G(x, y; θ)); x, y, θ are numpy
    object arrays of symbols, so ordinary numpy expressions trace.
    `compute_sensitivities` keeps ∂θ'/∂θ for the sensitivity path (the reference's
    ∇F_θ!, src/mcp.jl:122-140).
    """

    def __init__(self, *args, unconstrained_dimension=None, constrained_dimension=None,
                 parameter_dimension=None, compute_sensitivities=True, backend=None, backend_options=None):
        if len(args) == 2 and callable(args[0]) and callable(args[1]):
            G, H = args
            if unconstrained_dimension is None or constrained_dimension is None or parameter_dimension is None:
                raise TypeError("PrimalDualMCP(G, H; unconstrained_dimension, constrained_dimension, "
                                "parameter_dimension) needs all three dimensions")
            xs = make_variables("x", unconstrained_dimension)
            ys = make_variables("y", constrained_dimension)
            ts = make_variables("θ", parameter_dimension)
            self._init_symbolic(_as_exprs(G(xs, ys, θ=ts), "G"), _as_exprs(H(xs, ys, θ=ts), "H"),
                                list(xs), list(ys), list(ts), compute_sensitivities, backend_options)
        elif len(args) == 3 and callable(args[0]):
            K, lo, hi = args
            if parameter_dimension is None:
                raise TypeError("PrimalDualMCP(K, lower_bounds, upper_bounds; parameter_dimension) "
                                "needs parameter_dimension")
            zs = make_variables("z", len(lo))
            ts = make_variables("θ", parameter_dimension)
            self._init_K(_as_exprs(K(zs, θ=ts), "K"), list(zs), list(ts), lo, hi, compute_sensitivities,
                         backend_options)
        elif len(args) == 0:
            pass  # used by the from_symbolic* class methods
        else:
            raise TypeError("PrimalDualMCP(G, H; dims...) or PrimalDualMCP(K, lower_bounds, upper_bounds; "
                            "parameter_dimension)")

    # -- alternative constructors ------------------------------------------
    @classmethod
    def from_symbolic(cls, G_symbolic, H_symbolic, x_symbolic, y_symbolic, θ_symbolic,
                      compute_sensitivities=True, backend_options=None) -> "PrimalDualMCP":
        self = cls()
        self._init_symbolic(_as_exprs(G_symbolic, "G"), _as_exprs(H_symbolic, "H"), list(x_symbolic),
                            list(y_symbolic), list(θ_symbolic), compute_sensitivities, backend_options)
        return self

    @classmethod
    def from_text(cls, path: str, compute_sensitivities=True, backend_options=None) -> "PrimalDualMCP":
        """The MCP of a GH text file (mcp_amd/symtext.py): G/H printed by the Julia side from
        its Symbolics expressions (src/mcp.jl:55-70), read back in the front end's symbols."""
        from . import symtext

        G, H, xs, ys, ts = symtext.load(path)
        return cls.from_symbolic(G, H, xs, ys, ts, compute_sensitivities, backend_options)

    @classmethod
    def from_symbolic_K(cls, K_symbolic, z_symbolic, θ_symbolic, lower_bounds, upper_bounds,
                        compute_sensitivities=True, backend_options=None) -> "PrimalDualMCP":
        self = cls()
        self._init_K(_as_exprs(K_symbolic, "K"), list(z_symbolic), list(θ_symbolic), lower_bounds, upper_bounds,
                     compute_sensitivities, backend_options)
        return self

    def _init_K(self, K, zs, ts, lower_bounds, upper_bounds, compute_sensitivities, backend_options=None):
        lo = np.asarray(lower_bounds, dtype=float)
        hi = np.asarray(upper_bounds, dtype=float)
        # src/mcp.jl:191 — the reference @asserts this
        if not (np.all(np.isinf(hi)) and np.all(np.isinf(lo) | (lo == 0))):
            raise ValueError("upper bounds must all be Inf and lower bounds -Inf or 0 (src/mcp.jl:191)")
        if len(K) != len(zs) or len(lo) != len(zs) or len(hi) != len(zs):
            raise ValueError("K, z, lower_bounds and upper_bounds must have the same length")
        unc = [i for i in range(len(zs)) if np.isinf(lo[i])]
        con = [i for i in range(len(zs)) if not np.isinf(lo[i])]
        self._init_symbolic([K[i] for i in unc], [K[i] for i in con], [zs[i] for i in unc], [zs[i] for i in con],
                            ts, compute_sensitivities, backend_options)

    def _init_symbolic(self, G, H, xs, ys, ts, compute_sensitivities, backend_options=None):
        sp = _sp()
        n, m = len(xs), len(ys)
        if len(G) != n or len(H) != m:
            raise ValueError(f"G has {len(G)} rows for {n} unconstrained variables, H has {len(H)} rows for "
                             f"{m} constrained variables")
        self.unconstrained_dimension = n
        self.constrained_dimension = m
        self.parameter_dimension = len(ts)
        self.compute_sensitivities = bool(compute_sensitivities)
        self.G_symbolic, self.H_symbolic = G, H
        self.x_symbolic, self.y_symbolic, self.θ_symbolic = xs, ys, ts
        zs = xs + ys
        self.nl = None
        self._module = None
        self.h_independent_of_y = False
        try:
            if (backend_options or {}).get("family") == "nonlinear":  # force the generated-code path
                raise NotAffineError("nonlinear family requested through backend_options")
            CG, cg = _affine_rows(G, zs, "G")
            CH, ch = _affine_rows(H, zs, "H")
        except NotAffineError:
            from . import codegen

            self.family = _abi.FAMILY_NONLINEAR
            self.nl = codegen.NLSystem(G, H, xs, ys, ts)
            self.theta_map = ThetaMap(list(ts), ts)  # θ' = θ
            return
        P = [[CG[i][j] for j in range(n)] for i in range(n)]
        Q = [[CG[i][n + k] for k in range(m)] for i in range(n)]
        R = [[CH[k][j] for j in range(n)] for k in range(m)]
        S = [[CH[k][n + l] for l in range(m)] for k in range(m)]
        # ∂H/∂y ≡ 0: the SCHUR elimination applies (QP family, or the affine family's S block
        # structurally zero — include/mcpx.h MCPX_LINSOLVE_SCHUR)
        self.h_independent_of_y = all(sp.expand(S[k][l]) == 0 for k in range(m) for l in range(m))
        is_qp = (self.h_independent_of_y
                 and all(sp.expand(Q[i][k] + R[k][i]) == 0 for i in range(n) for k in range(m)))
        colmajor = lambda Mx, r, c: [Mx[i][j] for j in range(c) for i in range(r)]
        if is_qp:
            self.family = _abi.FAMILY_QP
            exprs = colmajor(P, n, n) + colmajor(R, m, n) + [-e for e in ch] + [-e for e in cg]
        else:
            self.family = _abi.FAMILY_AFFINE
            exprs = colmajor(P, n, n) + colmajor(Q, n, m) + colmajor(R, m, n) + colmajor(S, m, m) + cg + ch
        self.theta_map = ThetaMap(exprs, ts)
        assert self.theta_map.p_out == _abi.theta_dim(self.family, n, m)

    def module(self):
        """The loaded gfx950 code object of a nonlinear-family MCP: compiled on first
        use (cached in-tree by content hash, mcp_amd/_gen), loaded once per process."""
        if self.nl is None:
            raise TypeError("only nonlinear-family MCPs have a generated module")
        if self._module is None:
            from .batch import Module

            self._module = Module(self.nl.build_module())
        return self._module

    def _nl_host(self):
        """Lambdified (G; H) and its z-Jacobian: host inspection of a nonlinear MCP."""
        if getattr(self, "_nl_fns", None) is None:
            sp = _sp()
            zs = list(self.x_symbolic) + list(self.y_symbolic)
            args = zs + list(self.θ_symbolic)
            GH = list(self.G_symbolic) + list(self.H_symbolic)
            self._nl_fns = (sp.lambdify(args, GH, "numpy"),
                            sp.lambdify(args, sp.Matrix(GH).jacobian(zs), "numpy"))
        return self._nl_fns

    def _nl_host_theta(self):
        """Lambdified ∂(G; H)/∂θ of a nonlinear MCP (host inspection)."""
        if getattr(self, "_nl_tfn", None) is None:
            sp = _sp()
            zs = list(self.x_symbolic) + list(self.y_symbolic)
            args = zs + list(self.θ_symbolic)
            GH = list(self.G_symbolic) + list(self.H_symbolic)
            self._nl_tfn = sp.lambdify(args, sp.Matrix(GH).jacobian(list(self.θ_symbolic)), "numpy")
        return self._nl_tfn

    # -- host evaluation of the reference callbacks (inspection / tests) ----
    def jacobian_theta(self, x, y, s, *, θ, ϵ=None):
        """∇F_θ (src/mcp.jl:122-147) of a nonlinear-family MCP as a dense N×p host array
        (the s⊙y − ϵ rows are 0), w.r.t. the MCP's own parameters θ (host inspection; the
        affine families' ∇F_θ is analytic, oracle/ipm_ref.py jacobian_theta)."""
        if self.family != _abi.FAMILY_NONLINEAR:
            raise TypeError("jacobian_theta is the nonlinear family's host check")
        n, m, p = self.unconstrained_dimension, self.constrained_dimension, self.parameter_dimension
        out = np.zeros((n + 2 * m, p))
        x, y, th = (np.asarray(v, float) for v in (x, y, θ))
        out[:n + m] = np.asarray(self._nl_host_theta()(*x, *y, *th), float).reshape(n + m, p)
        return out

    def family_parameters(self, θ):
        """θ → θ' (the per-instance data the kernel reads), numpy or torch."""
        return self.theta_map(θ)

    def blocks(self, θ):
        """Affine blocks (P, Q, R, S, g, h) of G = P x + Q y + g, H = R x + S y + h at one θ."""
        if self.family == _abi.FAMILY_NONLINEAR:
            raise TypeError("a nonlinear MCP has no constant affine blocks; see F / jacobian_z")
        n, m = self.unconstrained_dimension, self.constrained_dimension
        t = self.theta_map(np.asarray(θ, float).reshape(1, -1))[0]
        if self.family == _abi.FAMILY_QP:
            M = t[:n * n].reshape(n, n, order="F")
            A = t[n * n:n * n + m * n].reshape(m, n, order="F")
            b = t[n * n + m * n:n * n + m * n + m]
            phi = t[n * n + m * n + m:]
            return M, -A.T, A, np.zeros((m, m)), -phi, -b
        o = 0
        out = []
        for r, c in ((n, n), (n, m), (m, n), (m, m)):
            out.append(t[o:o + r * c].reshape(r, c, order="F"))
            o += r * c
        return (*out, t[o:o + n], t[o + n:o + n + m])

    def F(self, x, y, s, *, θ, ϵ):
        """F(x, y, s; θ, ϵ) = [G; H − s; s⊙y − ϵ] (src/mcp.jl:72-80), host numpy."""
        x, y, s = (np.asarray(v, float) for v in (x, y, s))
        if self.family == _abi.FAMILY_NONLINEAR:
            n = self.unconstrained_dimension
            gh = np.asarray(self._nl_host()[0](*x, *y, *np.asarray(θ, float)), float).reshape(-1)
            return np.concatenate([gh[:n], gh[n:] - s, s * y - ϵ])
        P, Q, R, S, g, h = self.blocks(θ)
        return np.concatenate([P @ x + Q @ y + g, R @ x + S @ y + h - s, s * y - ϵ])

    def jacobian_z(self, x, y, s, *, θ, ϵ=None):
        """∇F_z (src/mcp.jl:97-120) as a dense N×N host array."""
        n, m = self.unconstrained_dimension, self.constrained_dimension
        J = np.zeros((n + 2 * m, n + 2 * m))
        if self.family == _abi.FAMILY_NONLINEAR:
            J[:n + m, :n + m] = np.asarray(self._nl_host()[1](*np.asarray(x, float), *np.asarray(y, float),
                                                              *np.asarray(θ, float)), float).reshape(n + m, n + m)
            J[n:n + m, n + m:] = -np.eye(m)
        else:
            P, Q, R, S, g, h = self.blocks(θ)
            J[:n, :n], J[:n, n:n + m] = P, Q
            J[n:n + m, :n], J[n:n + m, n:n + m], J[n:n + m, n + m:] = R, S, -np.eye(m)
        J[n + m:, n:n + m], J[n + m:, n + m:] = np.diag(np.asarray(s, float)), np.diag(np.asarray(y, float))
        return J

    def __repr__(self):
        fam = {_abi.FAMILY_QP: "qp", _abi.FAMILY_AFFINE: "affine", _abi.FAMILY_NONLINEAR: "nonlinear"}[self.family]
        return (f"PrimalDualMCP(n={self.unconstrained_dimension}, m={self.constrained_dimension}, "
                f"parameter_dimension={self.parameter_dimension}, family={fam})")


# ---------------------------------------------------------------------------
# solver


class SolverType:
    """Dispatch hook, src/solver.jl:1-2."""


class InteriorPoint(SolverType):
    """The interior-point solver of src/solver.jl:35-122."""


@dataclass
class MCPSolution:
    """The NamedTuple `(; status, x, y, s, kkt_error, ϵ, outer_iters)` of
    src/solver.jl:121, plus the build's derived outputs (newton_iters,
    active_mask).  `sol.ϵ` works (NFKC maps ϵ to ε)."""

    status: Any
    x: Any
    y: Any
    s: Any
    kkt_error: Any
    eps: Any
    outer_iters: Any
    newton_iters: Any = None
    active_mask: Any = None
    alpha_trace: Any = None
    θ: Any = field(default=None, repr=False)
    params: Any = field(default=None, repr=False)
    mcp: Any = field(default=None, repr=False)

    @property
    def ε(self):  # noqa: N802 — `sol.ϵ` in user code normalises to this name
        return self.eps


_STATUS = np.array(["solved", "failed"])


def _linear_solver(mcp: PrimalDualMCP, linear_solve_algorithm) -> str:
    if linear_solve_algorithm is None:
        if mcp.family == _abi.FAMILY_NONLINEAR:
            return mcp.nl.default_solver()
        # the MFMA Schur-complement kernels for the QP family (one wave: n + m ≤ 64; one
        # workgroup: n ≤ 128, csrc/gj_vr.hpp).  An affine-family MCP here has −Q ≠ Rᵀ
        # symbolically (else it is classified QP), so its SCHUR solve would always take the
        # pivoting-LU pass, whose rate is not the measured one: REDUCED (pivoting over the
        # whole n + m system) stays its default.
        n, m = mcp.unconstrained_dimension, mcp.constrained_dimension
        schur_ok = n + m <= _abi.MAX_KKT_DIM or (n <= _abi.MAX_WG_SCHUR_N and n + 2 * m <= _abi.MAX_WG_KKT_DIM)
        return "schur" if mcp.family == _abi.FAMILY_QP and schur_ok else "reduced"
    if isinstance(linear_solve_algorithm, str):
        if linear_solve_algorithm not in _abi.LINEAR_SOLVERS:
            raise ValueError(f"linear_solve_algorithm must be one of {sorted(_abi.LINEAR_SOLVERS)}")
        if (linear_solve_algorithm == "schur" and mcp.family == _abi.FAMILY_AFFINE
                and not mcp.h_independent_of_y):
            raise ValueError("linear_solve_algorithm='schur' needs ∂H/∂y ≡ 0 (this MCP's H depends on y)")
        return linear_solve_algorithm
    raise TypeError("linear_solve_algorithm: 'reduced' | 'dense' | 'schur' (the kernels' exact eliminations of "
                    "the regularised Newton system; the reference's LinearSolve.jl algorithm objects do not apply)")


def solve(solver_type, mcp=None, θ=None, *, x0=None, y0=None, s0=None, tol=1e-4, max_inner_iters=20,
          max_outer_iters=50, tightening_rate=0.1, loosening_rate=0.5, min_stepsize=1e-4, verbose=False,
          linear_solve_algorithm=None, num_devices=0, trace_len=0, **kwargs):
    """solve(InteriorPoint(), mcp, θ; x₀, y₀, s₀, tol, …)  — src/solver.jl:35-122
    solve(game, θ; solver_type=InteriorPoint(), kwargs…)  — src/game.jl:196-212

    θ: a (p,) vector → one instance (scalar fields, status 'solved'/'failed');
       a (B, p) array → a batch (array fields);
       a torch HIP tensor → the batch stays on device (torch results, status int32:
       0 solved / 1 failed), enqueued on the current stream.
    x0/y0/s0 (aliases x₀/y₀/s₀): warm starts; caller-supplied numpy arrays of the
    result's shape are updated in place and returned, like the reference
    (src/solver.jl:64-66).
    """
    if isinstance(solver_type, ParametricGame):
        game, theta = solver_type, mcp
        return _solve_game(game, theta, **dict(kwargs, x0=x0, y0=y0, s0=s0, tol=tol,
                                                  max_inner_iters=max_inner_iters, max_outer_iters=max_outer_iters,
                                                  tightening_rate=tightening_rate, loosening_rate=loosening_rate,
                                                  min_stepsize=min_stepsize, verbose=verbose,
                                                  linear_solve_algorithm=linear_solve_algorithm,
                                                  num_devices=num_devices, trace_len=trace_len))
    if not isinstance(solver_type, InteriorPoint):
        raise TypeError(f"no solver for {type(solver_type).__name__}; use InteriorPoint()")
    if not isinstance(mcp, PrimalDualMCP):
        raise TypeError("solve(InteriorPoint(), mcp::PrimalDualMCP, θ)")
    x0 = kwargs.pop("x₀", x0)
    y0 = kwargs.pop("y₀", y0)
    s0 = kwargs.pop("s₀", s0)
    if kwargs:
        raise TypeError(f"unexpected keyword arguments {sorted(kwargs)}")
    n, m = mcp.unconstrained_dimension, mcp.constrained_dimension
    ls = _linear_solver(mcp, linear_solve_algorithm)
    prm = _abi.make_params(tol=tol, max_inner_iters=max_inner_iters, max_outer_iters=max_outer_iters,
                           tightening_rate=tightening_rate, loosening_rate=loosening_rate,
                           min_stepsize=min_stepsize, linear_solver=ls)
    if _is_torch(θ):
        return _solve_device(mcp, θ, prm, x0, y0, s0, trace_len)
    from .batch import solve_batch

    th = np.asarray(θ, dtype=np.float64)
    single = th.ndim == 1
    tp = mcp.theta_map(th)
    B = tp.shape[0]
    r = solve_batch(mcp.family, n, m, tp, x0=x0, y0=y0, s0=s0, params=prm, num_devices=num_devices,
                    trace_len=trace_len, module=mcp.module() if mcp.nl is not None else None)
    if verbose:  # the warnings of src/solver.jl:85,97 from the per-instance failure events
        fr = r["fail_reason"]
        for b in np.nonzero(fr & (_abi.FAIL_LINSOLVE | _abi.FAIL_LINESEARCH))[0][:16]:
            what = [w for bit, w in ((_abi.FAIL_LINSOLVE, "Linear solve failed"),
                                     (_abi.FAIL_LINESEARCH, "Linesearch failed")) if fr[b] & bit]
            warnings.warn(f"instance {b}: {'; '.join(what)}. Exiting prematurely "
                          f"(outer_iters={r['outer_iters'][b]}, kkt_error={r['kkt_error'][b]:.3e})")
    # aliasing of caller-supplied warm starts (src/solver.jl:64-66)
    for key, w in (("x", x0), ("y", y0), ("s", s0)):
        if isinstance(w, np.ndarray) and w.dtype == np.float64 and w.shape == (r[key][0].shape if single
                                                                                  else r[key].shape):
            w[...] = r[key][0] if single else r[key]
            r[key] = w[None] if single else w
    status = _STATUS[r["status"]]
    if single:
        return MCPSolution(str(status[0]), r["x"][0], r["y"][0], r["s"][0], float(r["kkt_error"][0]),
                           float(r["eps"][0]), int(r["outer_iters"][0]), int(r["newton_iters"][0]),
                           r["active_mask"][0] if r["active_mask"] is not None else None,
                           r["alpha_trace"][0] if trace_len else None, θ=th, params=prm, mcp=mcp)
    return MCPSolution(status, r["x"], r["y"], r["s"], r["kkt_error"], r["eps"], r["outer_iters"],
                       r["newton_iters"], r["active_mask"], r["alpha_trace"] if trace_len else None,
                       θ=th, params=prm, mcp=mcp)


def _solve_device(mcp, θ, prm, x0, y0, s0, trace_len):
    from .batch import solve_batch_device

    th = θ if θ.dim() == 2 else θ[None, :]
    tp = mcp.theta_map(th)
    n, m = mcp.unconstrained_dimension, mcp.constrained_dimension
    out = solve_batch_device(mcp.family, n, m, tp, x0=x0, y0=y0, s0=s0, params=prm, trace_len=trace_len,
                             module=mcp.module() if mcp.nl is not None else None)
    return MCPSolution(out["status"], out["x"], out["y"], out["s"], out["kkt_error"], out["eps"],
                       out["outer_iters"], out.get("newton_iters"), out.get("active_mask"),
                       out.get("alpha_trace"), θ=th, params=prm, mcp=mcp)


# ---------------------------------------------------------------------------
# games (src/game.jl)


class Block:
    """BlockArrays.jl-style block index (1-based, as in the reference's tests)."""

    def __init__(self, i: int):
        self.i = int(i)


class BlockVector:
    """Minimal BlockArrays `BlockVector`: a flat vector with block sizes; x[Block(i)]
    is the i-th block (1-based), any other index goes to the flat vector."""

    def __init__(self, data, sizes):
        self.data = np.asarray(data) if not isinstance(data, np.ndarray) else data
        self.sizes = [int(s) for s in sizes]
        self.offsets = np.concatenate([[0], np.cumsum(self.sizes)]).astype(int)
        if self.offsets[-1] != len(self.data):
            raise ValueError("block sizes do not add up to the vector length")

    def __getitem__(self, k):
        if isinstance(k, Block):
            return self.data[self.offsets[k.i - 1]:self.offsets[k.i]]
        return self.data[k]

    def __len__(self):
        return len(self.data)

    def __array__(self, dtype=None, copy=None):
        return np.asarray(self.data, dtype=dtype)

    def blocks(self):
        return [self[Block(i + 1)] for i in range(len(self.sizes))]


def mortar(blocks) -> BlockVector:
    """BlockArrays.mortar for vectors."""
    blocks = [np.asarray(b) for b in blocks]
    data = np.concatenate(blocks) if blocks else np.zeros(0)
    return BlockVector(data, [len(b) for b in blocks])


def _blocks_of(v) -> list:
    return v.blocks() if isinstance(v, BlockVector) else [np.asarray(v)]


@dataclass
class OptimizationProblem:
    """src/game.jl:2-6: objective(x, θi), optional private_equality / private_inequality
    (x, θi) ↦ vector (equalities = 0, inequalities ≥ 0)."""

    objective: Callable
    private_equality: Callable | None = None
    private_inequality: Callable | None = None


class ParametricGame:
    """src/game.jl:16-46: N players, player i's decision block x[Block(i)] and parameter
    block θ[Block(i)]; shared constraints see the whole x and θ.  The game's KKT
    system is turned into an MCP exactly as game_to_mcp (src/game.jl:47-157):
      K = [∇_{x_i} L_i ...; g...; g̃; h...; h̃],  z = [x; λ; λ̃; μ; μ̃],
      L_i = f_i − λ_iᵀ g_i − μ_iᵀ h_i − λ̃ᵀ g̃ − μ̃ᵀ h̃,
      lower bounds −Inf for x, λ, λ̃ and 0 for μ, μ̃."""

    def __init__(self, *, test_point, test_parameter, problems, shared_equality=None, shared_inequality=None,
                 backend_options=None):
        sp = _sp()
        self.problems = list(problems)
        self.shared_equality = shared_equality
        self.shared_inequality = shared_inequality
        N = len(self.problems)
        tp = test_point if isinstance(test_point, BlockVector) else mortar(test_point)
        tt = test_parameter if isinstance(test_parameter, BlockVector) else mortar(test_parameter)
        if len(tp.sizes) != N:
            raise ValueError("test_point must have one block per player (src/game.jl:57)")
        self.dims = self._dimensions(tp, tt)
        d = self.dims
        x = BlockVector(make_variables("x", sum(d["x"])), d["x"])
        lam = BlockVector(make_variables("λ", sum(d["λ"])), d["λ"])
        mu = BlockVector(make_variables("μ", sum(d["μ"])), d["μ"])
        lam_s = make_variables("λ̃", d["λ̃"])
        mu_s = make_variables("μ̃", d["μ̃"])
        th = BlockVector(make_variables("θ", sum(d["θ"])), d["θ"])
        th_blocks = th.blocks()
        fs = [p.objective(x, ti) for p, ti in zip(self.problems, th_blocks)]
        gs = [None if p.private_equality is None else _as_exprs(p.private_equality(x, ti), "g")
              for p, ti in zip(self.problems, th_blocks)]
        hs = [None if p.private_inequality is None else _as_exprs(p.private_inequality(x, ti), "h")
              for p, ti in zip(self.problems, th_blocks)]
        gt = None if shared_equality is None else _as_exprs(shared_equality(x, th), "g̃")
        ht = None if shared_inequality is None else _as_exprs(shared_inequality(x, th), "h̃")
        grads = []
        for i in range(N):
            L = sp.sympify(fs[i])
            if gs[i] is not None:
                L -= sum(l * g for l, g in zip(lam[Block(i + 1)], gs[i]))
            if hs[i] is not None:
                L -= sum(u * h for u, h in zip(mu[Block(i + 1)], hs[i]))
            if gt is not None:
                L -= sum(l * g for l, g in zip(lam_s, gt))
            if ht is not None:
                L -= sum(u * h for u, h in zip(mu_s, ht))
            grads += [sp.diff(L, xv) for xv in x[Block(i + 1)]]
        K = grads + [e for g in gs if g is not None for e in g] + (gt or []) + \
            [e for h in hs if h is not None for e in h] + (ht or [])
        z = list(x.data) + list(lam.data) + list(lam_s) + list(mu.data) + list(mu_s)
        nx, nl, nls, nm, nms = len(x), len(lam), len(lam_s), len(mu), len(mu_s)
        lo = [-math.inf] * (nx + nl + nls) + [0.0] * (nm + nms)
        hi = [math.inf] * len(z)
        self.mcp = PrimalDualMCP.from_symbolic_K(K, z, list(th.data), lo, hi, backend_options=backend_options)

    def _dimensions(self, tp: BlockVector, tt: BlockVector) -> dict:
        """src/game.jl:159-187 (evaluated numerically on the test point)."""
        blocks_t = tt.blocks()
        lam = [0 if p.private_equality is None else len(np.atleast_1d(p.private_equality(tp, ti)))
               for p, ti in zip(self.problems, blocks_t)]
        mu = [0 if p.private_inequality is None else len(np.atleast_1d(p.private_inequality(tp, ti)))
              for p, ti in zip(self.problems, blocks_t)]
        lt = 0 if self.shared_equality is None else len(np.atleast_1d(self.shared_equality(tp, tt)))
        mt = 0 if self.shared_inequality is None else len(np.atleast_1d(self.shared_inequality(tp, tt)))
        return {"x": tp.sizes, "θ": tt.sizes, "λ": lam, "μ": mu, "λ̃": lt, "μ̃": mt}

    def num_players(self) -> int:
        return len(self.problems)


@dataclass
class GameSolution:
    """`(; primals, variables = (; x, y, s), kkt_error, status)` of src/game.jl:196-212."""

    primals: Any
    variables: Any
    kkt_error: Any
    status: Any


def num_players(game: ParametricGame) -> int:
    return game.num_players()


def _solve_game(game: ParametricGame, θ, solver_type=None, **kw):
    solver_type = solver_type or InteriorPoint()
    th = np.concatenate([np.asarray(b, float) for b in _blocks_of(θ)]) if isinstance(θ, BlockVector) \
        else θ
    sol = solve(solver_type, game.mcp, th, **kw)
    ends = np.cumsum(game.dims["x"])
    starts = np.concatenate([[0], ends[:-1]])
    x = sol.x
    primals = [x[..., a:b] for a, b in zip(starts, ends)]
    return GameSolution(primals, {"x": sol.x, "y": sol.y, "s": sol.s}, sol.kkt_error, sol.status)
