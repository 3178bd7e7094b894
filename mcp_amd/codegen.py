"""Device code generation for general (nonlinear) G/H — MCPX_FAMILY_NONLINEAR.

The reference compiles F!, ∇F_z! (and ∇F_θ!) from Symbolics expressions with
`build_function` once per problem (src/mcp.jl:82-120).  This module is that
step for the GPU: it turns the traced G(x, y; θ), H(x, y; θ) into straight-line
C that both the gfx950 kernel (hipcc, compiled with the solver template
csrc/ipm_nl_kernel.hpp into a code object the C ABI loads with
`mcpx_module_load`) and the CPU oracle (gcc, tests only) compile from the very
same text, so the evaluation order — and with -ffp-contract=off every
rounding — is identical on both sides.

Generated functions (MCPX_NL_FN is `__device__` on the GPU, `static inline` in C)
and tables (MCPX_NL_TABLE: `__constant__` on the GPU, `static const` in C):

  mcpx_nl_init(th, blk)      the Jacobian entries that do not depend on z
                             (θ-only and constant entries — the reference's
                             `constant_entries`, src/mcp.jl:111-112), once per
                             instance;
  mcpx_nl_eval(th, z, blk)   G, H and the z-dependent Jacobian entries at
                             z = [x; y], once per Newton step;
  mcpx_nl_qk_ptr / _idx      K(i): the structural nonzeros of row i of Q;
  mcpx_nl_rj_ptr / _idx      J(k): the structural nonzeros of row k of R
                             (the SCHUR elimination's sparse terms);
  mcpx_nl_eval_theta(th, z, dth)  ∇F_θ at z = [x; y] — the reference's ∇F_θ!
                             (src/mcp.jl:122-147), used by the sensitivity
                             kernels (src/AutoDiff.jl:18-40): the G and H rows
                             (the s⊙y − ϵ rows do not depend on θ) as an
                             (n+m)×p column-major block, dth[t·(n+m) + i] =
                             ∂[G; H]_i/∂θ_t, structural nonzeros only;
  mcpx_nl_tc_ptr / _idx      rows of column t of ∇F_θ with a structural
                             nonzero (CSR by θ column, ascending): the pullback
                             ∂θ_t = −Σ_i ∇F_θ[i, t] λ_i takes exactly these terms;
  mcpx_nl_tr_ptr / _idx      θ columns of row i (CSR by row, ascending): the
                             tangent (∇F_θ θ̇)_i of the JVP.

Block layout of `blk` (doubles, column-major blocks like the affine family):

  P = ∂G/∂x  n×n  at OFF_P = 0              P[i, j] = blk[j·n + i]
  Q = ∂G/∂y  n×m  at OFF_Q = n²             Q[i, k] = blk[OFF_Q + k·n + i]
  R = ∂H/∂x  m×n  at OFF_R = n² + nm        R[k, j] = blk[OFF_R + j·m + k]
  g = G      n    at OFF_G = n² + 2nm
  h = H      m    at OFF_H = OFF_G + n
  S = ∂H/∂y  m×m  at OFF_S = OFF_H + m      S[k, q] = blk[OFF_S + q·m + k]
                  (written only when ∂H/∂y is not structurally zero: HAS_S)

Structural zeros are never written (the kernel zeroes the block once).

Op order: after common-subexpression elimination (sympy.cse) every node is
printed fully parenthesised as a left fold over sympy's canonical argument
order; integer powers become repeated products, x**-k a division of 1 by the
product, x**(±1/2) sqrt; numbers are exact hex-float literals.  Polynomial and
rational G/H are therefore bit-identical between GPU and oracle (+ − × ÷ and
sqrt are correctly rounded on both); for transcendental functions (sin, exp, …)
device libm (ocml) and glibc may differ by an ulp, and parity is then the
north_star's 1e-8 bar only.
"""

from __future__ import annotations

import glob
import hashlib
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
GEN_DIR = os.environ.get("MCPX_GEN_DIR") or os.path.join(HERE, "_gen")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# x + y entries above which the generated code re-reads z per use (register pressure)
Z_VOLATILE_ABOVE = int(os.environ.get("MCPX_NL_Z_VOLATILE_ABOVE", "128"))
ARCH = "gfx950"
# bump when the generated text or csrc/ipm_nl_kernel.hpp changes meaning (part of the cache key)
GEN_VERSION = 8
EVAL_PARTS = 4  # mcpx_nl_eval_p0..p3: the generated eval split over the 4-wave SCHUR kernel
_MODULE_FLAGS = ("--genco", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-ffp-contract=off", "-Wno-unused-function",
                 "-mllvm", "-amdgpu-mfma-vgpr-form=1")
_MODULE_DEPS = ("ipm_nl_kernel.hpp", "ipm_nl_band.hpp", "ipm_kernel_impl.hpp", "ipm_kernel.h", "bcast_group.inc", "ipm_wg.h",
                "ipm_wg_impl.hpp", "lu_vr.hpp", "gj_vr.hpp", "sens_wg_impl.hpp", "sens_kernel.h", "../../include/mcpx.h")
WG_LDS_LIMIT = 160 * 1024 - 2048  # MCPX_NL_WG_LIMIT of csrc/ipm_nl_kernel.hpp
LDS_LIMIT = 160 * 1024 - 2048  # bytes of static LDS one workgroup may declare on gfx950 (minus headroom)
# band kernel (csrc/ipm_nl_band.hpp): as much LDS as one workgroup may declare.  The launch sizes
# its persistent grid by the kernel's occupancy (mcpx_api.cpp launch_band), so a longer horizon
# runs fewer games per CU at once (T = 10: 40 KB, four per CU; T = 15: 60 KB, two) rather than
# falling back to the workgroup LU — a tail-bound launch (the 931-step failing games set its
# length) loses little by it
BAND_LDS_LIMIT = LDS_LIMIT
BAND_KERNEL = True  # the band kernel is compiled into modules (csrc/ipm_nl_band.hpp)

_FUNCS = {  # sympy function → C name (both libm and HIP device math)
    "sin": "sin", "cos": "cos", "tan": "tan", "exp": "exp", "log": "log", "tanh": "tanh",
    "sinh": "sinh", "cosh": "cosh", "asin": "asin", "acos": "acos", "atan": "atan",
    "Abs": "fabs", "atan2": "atan2",
}


def _sp():
    import sympy

    return sympy


def _lit(v) -> str:
    f = float(v)
    if f != f or f in (float("inf"), float("-inf")):
        raise ValueError(f"non-finite constant {v} in a generated expression")
    s = f.hex()
    return f"({s})" if f < 0 else s


class _Printer:
    """sympy expression → fully parenthesised C expression with a fixed op order."""

    def __init__(self, names: dict):
        self.names = names  # Symbol → C operand

    def __call__(self, e) -> str:
        sp = _sp()
        if e in self.names:
            return self.names[e]
        if e.is_Number:
            return _lit(e)
        if e.is_Symbol:
            raise ValueError(f"free symbol {e} is neither a decision variable nor a parameter")
        if e.is_Add:
            out = None
            for t in e.as_ordered_terms():
                neg = False
                c, rest = t.as_coeff_Mul()
                if c == -1 and rest != 1:
                    neg, t = True, rest
                s = self(t)
                if out is None:
                    out = f"(-{s})" if neg else s
                else:
                    out = f"({out} {'-' if neg else '+'} {s})"
            return out
        if e.is_Mul:
            c, rest = e.as_coeff_Mul()
            if c == -1:
                return f"(-{self(rest)})"
            facs = list(e.as_ordered_factors())
            recip = lambda f: f.is_Pow and f.exp.is_Integer and f.exp < 0
            num = [f for f in facs if not recip(f)]
            den = [f.base ** (-f.exp) for f in facs if recip(f)]
            out = None
            for f in num:
                s = self(f)
                out = s if out is None else f"({out} * {s})"
            if out is None:
                out = _lit(1.0)
            for f in den:  # x·y⁻ᵏ prints as a division by the product yᵏ
                out = f"({out} / {self(f)})"
            return out
        if e.is_Pow:
            b, x = e.base, e.exp
            if x.is_Integer:
                k = int(x)
                if k == 0:
                    return _lit(1.0)
                bs = self(b)
                prod = bs
                for _ in range(abs(k) - 1):
                    prod = f"({prod} * {bs})"
                return prod if k > 0 else f"({_lit(1.0)} / {prod})"
            if x == sp.Rational(1, 2):
                return f"sqrt({self(b)})"
            if x == sp.Rational(-1, 2):
                return f"({_lit(1.0)} / sqrt({self(b)}))"
            return f"pow({self(b)}, {self(x)})"
        if isinstance(e, sp.Function):
            name = type(e).__name__
            if name not in _FUNCS:
                raise NotImplementedError(f"function {name} has no generated-code mapping")
            return f"{_FUNCS[name]}({', '.join(self(a) for a in e.args)})"
        raise NotImplementedError(f"cannot generate code for {type(e).__name__}: {e}")


class NLSystem:
    """The generated evaluation code of one nonlinear PrimalDualMCP.

    G (n), H (m): sympy expressions in the decision variables xs (n), ys (m)
    and the parameters ts (p)."""

    def __init__(self, G, H, xs, ys, ts):
        sp = _sp()
        self.n, self.m, self.p = len(xs), len(ys), len(ts)
        n, m = self.n, self.m
        # The variables are renamed by position (x00000…, y00000…, θ00000…) before anything is
        # generated: sympy orders the terms of a sum by the names of their symbols, and that order
        # is the generated code's op order.  So the module depends on G/H and the positions of the
        # variables only, not on what a front end called them — the sympy tracer's x_1, λ̃_1, μ̃_1
        # and the names in a GH text from Julia (mcp_amd/symtext.py) give the same code object.
        canon = ([sp.Symbol(f"x{i:05d}", real=True) for i in range(n)],
                 [sp.Symbol(f"y{k:05d}", real=True) for k in range(m)],
                 [sp.Symbol(f"θ{t:05d}", real=True) for t in range(self.p)])
        sub = dict(zip(list(xs) + list(ys) + list(ts), canon[0] + canon[1] + canon[2]))
        if len(sub) != n + m + self.p:
            raise ValueError("the decision variables and parameters must be distinct symbols")
        self.G = [sp.sympify(e).xreplace(sub) for e in G]
        self.H = [sp.sympify(e).xreplace(sub) for e in H]
        self.xs, self.ys, self.ts = canon
        zset = set(self.xs) | set(self.ys)
        nn, nm = n * n, n * m
        self.OFF_P, self.OFF_Q, self.OFF_R = 0, nn, nn + nm
        self.OFF_G = nn + 2 * nm
        self.OFF_H = self.OFF_G + n
        self.OFF_S = self.OFF_H + m
        const_entries, var_entries = [], []

        def put(idx, e):
            if e == 0:
                return
            (var_entries if (e.free_symbols & zset) else const_entries).append((idx, e))

        for i, g in enumerate(self.G):
            for j, xj in enumerate(self.xs):
                put(self.OFF_P + j * n + i, sp.diff(g, xj))
            for k, yk in enumerate(self.ys):
                put(self.OFF_Q + k * n + i, sp.diff(g, yk))
        S_entries = []
        for k, h in enumerate(self.H):
            for j, xj in enumerate(self.xs):
                put(self.OFF_R + j * m + k, sp.diff(h, xj))
            for q, yq in enumerate(self.ys):
                d = sp.diff(h, yq)
                if d != 0:
                    S_entries.append((self.OFF_S + q * m + k, d))
        self.has_s = bool(S_entries)
        for idx, d in S_entries:
            put(idx, d)
        self.size = self.OFF_S + (m * m if self.has_s else 0)
        self.const_entries = sorted(const_entries, key=lambda t: t[0])
        self.var_entries = sorted(var_entries, key=lambda t: t[0])
        # residual values: per step (they carry z)
        self.residuals = ([(self.OFF_G + i, g) for i, g in enumerate(self.G)]
                          + [(self.OFF_H + k, h) for k, h in enumerate(self.H)])
        self.nnz = len(self.const_entries) + len(self.var_entries)
        # ∇F_θ of the G and H rows (src/mcp.jl:122-147), dth[t·(n+m) + i]
        nr = n + m
        self.theta_entries = sorted(
            [(t * nr + i, d) for i, e in enumerate(self.G + self.H) for t, th in enumerate(self.ts)
             if (d := sp.diff(e, th)) != 0], key=lambda t: t[0])
        self.nnz_theta = len(self.theta_entries)
        self.body = self._emit()
        self.key = hashlib.sha256(f"v{GEN_VERSION}\n{self.body}".encode()).hexdigest()[:24]

    # ---- which one-wave kernels the module gets (csrc/ipm_nl_kernel.hpp) -------
    def schur_lds_bytes(self) -> int:
        """MCPX_NL_SCHUR_LDS of csrc/ipm_nl_kernel.hpp: the blocks up to S, the n×(n+1) rows
        of [S | rr], z / δz / F and the four per-constraint arrays (tests/test_codegen_masks.py
        evaluates the C macros against these formulas)."""
        n, m = self.n, self.m
        return 8 * (self.OFF_S + n * (n + 1) + 3 * (n + 2 * m) + 4 * m)

    def solvers(self) -> dict:
        n, m = self.n, self.m
        return {
            "schur": (not self.has_s) and 1 <= n <= 64 and m <= 128 and self.schur_lds_bytes() <= LDS_LIMIT,
            "reduced": 1 <= n + m <= 64,
            "dense": 1 <= n + 2 * m <= 64,
        }

    def wg_solvers(self) -> dict:
        """Workgroup-per-instance kernels of the module (MCPX_NL_CAN_WG_* of
        csrc/ipm_nl_kernel.hpp): LDS = 3·8·(n+2m) + NS·(16·8 + 7) + 512 bytes."""
        n, m = self.n, self.m
        lds = lambda ns: 8 * 3 * (n + 2 * m) + ns * (8 * 16 + 7) + 512
        return {
            "schur": (not self.has_s) and n >= 1 and lds(n) <= WG_LDS_LIMIT,
            "reduced": n + m >= 1 and lds(n + m) <= WG_LDS_LIMIT,
            "dense": n + 2 * m >= 1 and lds(n + 2 * m) <= WG_LDS_LIMIT,
        }

    def default_solver(self) -> str:
        """The cheapest elimination a kernel exists for: SCHUR, then REDUCED, then
        DENSE; the one-wave kernels when the system fits them, else the
        workgroup-per-instance ones (the C ABI picks the kernel the same way)."""
        for ok in (self.solvers(), self.wg_solvers()):
            for s in ("schur", "reduced", "dense"):
                if ok[s]:
                    return s
        raise NotImplementedError(f"nonlinear MCP with n={self.n}, m={self.m} exceeds every kernel's LDS budget")

    # ---- emission ------------------------------------------------------------
    def _block(self, entries, with_z: bool, out: str = "blk", cse_out: dict | None = None) -> list:
        """Straight-line C for `entries` after common-subexpression elimination.  Each
        CSE temporary is emitted right before the first statement that needs it
        (dependency order kept), not all at the top: at horizon T = 10 the
        all-at-the-top form kept ~170 temporaries and every z load live at once, and
        the kernel it is inlined into spilled (512 registers + scratch)."""
        sp = _sp()
        names = {t: f"th[{k}]" for k, t in enumerate(self.ts)}
        if with_z:  # MCPX_NL_Z: a fresh load per use on the GPU (see hip_source), plain z[j] in C
            names.update({x: f"MCPX_NL_Z({j})" for j, x in enumerate(self.xs)})
            names.update({y: f"MCPX_NL_Z({self.n + k})" for k, y in enumerate(self.ys)})
        if not entries:
            return []
        reps, red = sp.cse([e for _, e in entries], symbols=sp.numbered_symbols("c"), order="canonical")
        if cse_out is not None:  # the same CSE for the lane-parallel eval (nl_vec)
            cse_out.update(reps=reps, red=red, names=dict(names))
        pr = _Printer(names)
        rep_of = {sym: e for sym, e in reps}
        order = {sym: i for i, (sym, _) in enumerate(reps)}
        emitted, lines = set(), []

        def need(e):  # CSE temporaries e depends on, transitively, in definition order
            out, stack = set(), [e]
            while stack:
                for f in stack.pop().free_symbols:
                    if f in rep_of and f not in out and f not in emitted:
                        out.add(f)
                        stack.append(rep_of[f])
            return sorted(out, key=order.get)

        for (idx, _), e in zip(entries, red):
            for sym in need(e):
                lines.append(f"  const double {sym} = {pr(rep_of[sym])};")
                names[sym] = str(sym)
                emitted.add(sym)
            lines.append(f"  {out}[{idx}] = {pr(e)};")
        return lines

    def _block_parts(self, entries, with_z: bool, parts: int, out: str = "blk") -> list:
        """`entries` split into `parts` straight-line functions' bodies for the 4-wave
        SCHUR kernel (one wave's lane 0 runs each): the same CSE as _block, so every
        output is the same expression tree (same bits); contiguous runs of entries (they
        share temporaries) of about equal operation count; a temporary a part needs is
        recomputed in that part."""
        sp = _sp()
        names = {t: f"th[{k}]" for k, t in enumerate(self.ts)}
        if with_z:
            names.update({x: f"MCPX_NL_Z({j})" for j, x in enumerate(self.xs)})
            names.update({y: f"MCPX_NL_Z({self.n + k})" for k, y in enumerate(self.ys)})
        if not entries:
            return [[] for _ in range(parts)]
        reps, red = sp.cse([e for _, e in entries], symbols=sp.numbered_symbols("c"), order="canonical")
        rep_of = {sym: e for sym, e in reps}
        order = {sym: i for i, (sym, _) in enumerate(reps)}

        def need(e, have):
            got, stack = set(), [e]
            while stack:
                for f in stack.pop().free_symbols:
                    if f in rep_of and f not in got and f not in have:
                        got.add(f)
                        stack.append(rep_of[f])
            return sorted(got, key=order.get)

        # cost of each entry in sequence (its new temporaries included), then equal-cost runs
        have, cost = set(), []
        for e in red:
            new = need(e, have)
            have.update(new)
            cost.append(1 + sp.count_ops(e) + sum(sp.count_ops(rep_of[t]) for t in new))
        total, acc, cut, bounds = sum(cost), 0, 1, [0]
        for i, c in enumerate(cost):
            acc += c
            if cut < parts and acc >= total * cut / parts:
                bounds.append(i + 1)
                cut += 1
        while len(bounds) < parts:
            bounds.append(len(red))
        bounds.append(len(red))
        bodies = []
        for w in range(parts):
            pr = _Printer(dict(names))
            emitted, lines = set(), []
            for (idx, _), e in list(zip(entries, red))[bounds[w]:bounds[w + 1]]:
                for sym in need(e, emitted):
                    lines.append(f"  const double {sym} = {pr(rep_of[sym])};")
                    pr.names[sym] = str(sym)
                    emitted.add(sym)
                lines.append(f"  {out}[{idx}] = {pr(e)};")
            bodies.append(lines)
        return bodies

    def structure(self):
        """Structural nonzeros of Q = ∂G/∂y by rows (K(i): the k with Q_ik written by the
        generated code, ascending) and of R = ∂H/∂x by rows (J(k), ascending), as CSR
        (ptr, idx) pairs.  The SCHUR elimination forms S = (P + tol·I) − Q D⁻¹ R and
        recovers δy from these terms only (oracle and kernels alike): structural zeros
        are exact zeros, so they are never multiplied (as a sparse LU never touches them)."""
        n, m = self.n, self.m
        ents = {i for i, _ in self.const_entries} | {i for i, _ in self.var_entries}
        qk = [[k for k in range(m) if self.OFF_Q + k * n + i in ents] for i in range(n)]
        rj = [[j for j in range(n) if self.OFF_R + j * m + k in ents] for k in range(m)]
        csr = lambda rows: ([0] + list(__import__("itertools").accumulate(len(r) for r in rows)),
                            [x for r in rows for x in r])
        return csr(qk), csr(rj)

    def schur_entries(self):
        """The entries of [S | rr] the SCHUR elimination changes beyond P + tol·I and −F_G:
        (position i·(n+1) + j, [k ascending]) for each structural nonzero (i, j) of Q D⁻¹ R
        (k ∈ K(i) with j ∈ J(k)) and (i·(n+1) + n, K(i)) for each rr_i with K(i) ≠ ∅,
        sorted by position.  The one-wave SCHUR kernel gives each entry's fma chain to one
        lane (csrc/ipm_nl_kernel.hpp schur_form_entries)."""
        (qp, qi), (rp, ri) = self.structure()
        n, ldr, out = self.n, self.n + 1, []
        for i in range(n):
            K = qi[qp[i]:qp[i + 1]]
            cols = {}
            for k in K:
                for j in ri[rp[k]:rp[k + 1]]:
                    cols.setdefault(j, []).append(k)
            out += [(i * ldr + j, cols[j]) for j in sorted(cols)]
            if K:
                out.append((i * ldr + n, list(K)))
        return out

    def theta_structure(self):
        """Structural nonzeros of ∇F_θ's G/H rows: (ptr, idx) CSR by θ column (rows i
        ascending) and by row (θ columns t ascending)."""
        nr, p = self.n + self.m, self.p
        ents = [idx for idx, _ in self.theta_entries]
        cols = [[idx - t * nr for idx in ents if idx // nr == t] for t in range(p)]
        rows = [[idx // nr for idx in ents if idx % nr == i] for i in range(nr)]
        acc = __import__("itertools").accumulate
        csr = lambda rr: ([0] + list(acc(len(r) for r in rr)), [x for r in rr for x in r])
        return csr(cols), csr(rows)

    def _emit(self) -> str:
        init = self._block(self.const_entries, with_z=False)
        cse = {}
        ev = self._block(self.var_entries + self.residuals, with_z=True, cse_out=cse)
        from . import nl_vec

        self.vec = (nl_vec.build(self, cse["reps"], cse["red"], self.var_entries + self.residuals, cse["names"])
                    if cse else None)
        band_lines = self._emit_band()
        evt = self._block(self.theta_entries, with_z=True, out="dth")
        evp = self._block_parts(self.var_entries + self.residuals, True, EVAL_PARTS)
        parts = []
        for w, body in enumerate(evp):
            parts += [f"MCPX_NL_FN void mcpx_nl_eval_p{w}(const double* MCPX_NL_RESTRICT th, "
                      "const double* MCPX_NL_RESTRICT z, double* MCPX_NL_RESTRICT blk) {",
                      "  (void)th;", "  (void)z;", "  (void)blk;", *body, "}"]
        (qp, qi), (rp, ri) = self.structure()
        (tcp, tci), (trp, tri) = self.theta_structure()
        se = self.schur_entries()
        se_er = max(1, -(-len(se) // 64))
        se_kt = max([1] + [len(ks) for _, ks in se])
        se_pos = [-1] * (64 * se_er)
        se_k = [-1] * (64 * se_er * se_kt)
        for e, (pos, ks) in enumerate(se):
            r, ln = divmod(e, 64)
            se_pos[e] = pos
            for t, k in enumerate(ks):
                se_k[(r * se_kt + t) * 64 + ln] = k
        arr = lambda name, v: f"MCPX_NL_TABLE int32_t {name}[{max(len(v), 1)}] = {{{', '.join(map(str, v)) or '0'}}};"
        return "\n".join([
            "/* generated by mcp_amd/codegen.py — do not edit */",
            f"#define MCPX_NL_N {self.n}",
            f"#define MCPX_NL_M {self.m}",
            f"#define MCPX_NL_P {self.p}",
            f"#define MCPX_NL_HAS_S {int(self.has_s)}",
            f"#define MCPX_NL_SIZE {self.size}",
            f"#define MCPX_NL_NNZ {self.nnz}",
            f"#define MCPX_NL_NNZ_Q {len(qi)}",
            f"#define MCPX_NL_NNZ_R {len(ri)}",
            f"#define MCPX_NL_NNZ_T {self.nnz_theta}",
            "/* structural nonzeros: K(i) of Q row i, J(k) of R row k (CSR, ascending) */",
            arr("mcpx_nl_qk_ptr", qp),
            arr("mcpx_nl_qk_idx", qi),
            arr("mcpx_nl_rj_ptr", rp),
            arr("mcpx_nl_rj_idx", ri),
            "/* entries of [S | rr] beyond P + tol·I and −F_G (schur_entries): slot e = lane + 64r holds",
            "   position mcpx_nl_se_pos[e] (−1: none) and its k ascending, mcpx_nl_se_k[(r·KT + t)·64 + lane] */",
            f"#define MCPX_NL_SE_ER {se_er}",
            f"#define MCPX_NL_SE_KT {se_kt}",
            arr("mcpx_nl_se_pos", se_pos),
            arr("mcpx_nl_se_k", se_k),
            "/* structural nonzeros of ∇F_θ (G/H rows): rows of column t, columns of row i (CSR) */",
            arr("mcpx_nl_tc_ptr", tcp),
            arr("mcpx_nl_tc_idx", tci),
            arr("mcpx_nl_tr_ptr", trp),
            arr("mcpx_nl_tr_idx", tri),
            *(nl_vec.emit(self.vec) if self.vec is not None else []),
            *band_lines,
            "MCPX_NL_FN void mcpx_nl_init(const double* MCPX_NL_RESTRICT th, double* MCPX_NL_RESTRICT blk) {",
            "  (void)th;",
            "  (void)blk;",
            *init,
            "}",
            "MCPX_NL_FN void mcpx_nl_eval(const double* MCPX_NL_RESTRICT th, const double* MCPX_NL_RESTRICT z,",
            "                             double* MCPX_NL_RESTRICT blk) {",
            "  (void)th;",
            "  (void)z;",
            *ev,
            "}",
            f"/* the same outputs in {EVAL_PARTS} parts (one per wave of mcpx_nl_solve_schur_mw) */",
            f"#define MCPX_NL_EVAL_PARTS {EVAL_PARTS}",
            *parts,
            "MCPX_NL_FN void mcpx_nl_eval_theta(const double* MCPX_NL_RESTRICT th, const double* MCPX_NL_RESTRICT z,",
            "                                   double* MCPX_NL_RESTRICT dth) {",
            "  (void)th;",
            "  (void)z;",
            "  (void)dth;",
            *evt,
            "}",
            "",
        ])

    def _emit_band(self) -> list:
        """The band kernel's part of the text (mcp_amd/band.py, csrc/ipm_nl_band.hpp): its tables,
        mcpx_nl_init_c / mcpx_nl_eval_c — the generated code writing the compact array `cb`
        (structural entries in block order, then G, then H) with the same CSE and expression
        trees as mcpx_nl_init / mcpx_nl_eval, hence the same bits — and the lane-parallel
        program on cb (MCPX_NL_CVEC).  MCPX_NL_CAN_BAND (whether the module gets the kernel)
        and MCPX_NL_BAND_AUTO (whether MCPX_KERNEL_AUTO prefers it) are decided here, and
        mcpx_nl_band_info carries them to the oracle's gcc build of the same text."""
        from . import band as _band
        from . import nl_vec

        self.band = bp = _band.plan(self)
        self.cvec = None
        self.band_can = self.band_auto = False
        if bp is None:
            return ["#define MCPX_NL_CAN_BAND 0", "#define MCPX_NL_BAND_AUTO 0",
                    "MCPX_NL_TABLE int32_t mcpx_nl_band_info[4] = {0, 0, 0, 0};",
                    "MCPX_NL_TABLE int32_t mcpx_nl_band_rperm[1] = {0};",
                    "MCPX_NL_TABLE int32_t mcpx_nl_band_cperm[1] = {0};"]
        ci = lambda entries: [(bp.compact_index(self, i), e) for i, e in entries]
        init = self._block(ci(self.const_entries), with_z=False, out="cb")
        cse = {}
        ev_entries = ci(self.var_entries + self.residuals)
        ev = self._block(ev_entries, with_z=True, out="cb", cse_out=cse)
        if cse:
            self.cvec = nl_vec.build(self, cse["reps"], cse["red"], ev_entries, cse["names"], size=bp.csize)
        ev_size = self.cvec.ev_size if self.cvec is not None else bp.csize + self.n + 2 * self.m
        lds = bp.lds_bytes(ev_size)
        self.band_lds = lds
        can = BAND_KERNEL and lds <= BAND_LDS_LIMIT
        auto = can and self.n > 64  # measured per size class: DESIGN.md §4 (band kernel)
        self.band_can, self.band_auto = can, auto
        return [
            *bp.tables(),
            f"#define MCPX_NL_CAN_BAND {int(can)}",
            f"#define MCPX_NL_BAND_AUTO {int(auto)}",
            f"MCPX_NL_TABLE int32_t mcpx_nl_band_info[4] = {{{int(can)}, {bp.ns}, {bp.wc}, {int(auto)}}};",
            *(nl_vec.emit(self.cvec, "MCPX_NL_CVEC", "mcpx_nl_cvec") if self.cvec is not None else []),
            "MCPX_NL_FN void mcpx_nl_init_c(const double* MCPX_NL_RESTRICT th, double* MCPX_NL_RESTRICT cb) {",
            "  (void)th;",
            "  (void)cb;",
            *init,
            "}",
            "MCPX_NL_FN void mcpx_nl_eval_c(const double* MCPX_NL_RESTRICT th, const double* MCPX_NL_RESTRICT z,",
            "                               double* MCPX_NL_RESTRICT cb) {",
            "  (void)th;",
            "  (void)z;",
            "  (void)cb;",
            *ev,
            "}",
        ]

    # ---- device module ---------------------------------------------------------
    def hip_source(self) -> str:
        return "\n".join([
            "// generated gfx950 module of one nonlinear MCP (mcp_amd/codegen.py)",
            "#include <hip/hip_runtime.h>",
            "#define MCPX_NL_FN __device__ __forceinline__",
            "#define MCPX_NL_RESTRICT __restrict__",
            "#define MCPX_NL_TABLE static __constant__ const",
            "// z lives in LDS (the address space makes its reads ds_read; a generic pointer compiled",
            "// them to flat loads).  Large problems read it afresh at every use (volatile): kept in",
            "// registers from its first use, the ~450 z values of a T = 10 game made the kernel spill;",
            "// small ones let the compiler batch the loads.",
            "#define MCPX_NL_Z(j) (((const " + ("volatile " if self.n + self.m > Z_VOLATILE_ABOVE else "")
            + "__attribute__((address_space(3))) double*)z)[j])",
            self.body,
            '#include "ipm_nl_kernel.hpp"',
            "",
        ])

    def module_key(self) -> str:
        """Content hash of everything the code object is built from: the generated
        text, the kernel headers it includes and the compiler flags (self.key, the
        oracle's cache key, covers the generated text only)."""
        h = hashlib.sha256(self.key.encode())
        h.update(deps_hash().encode())
        return h.hexdigest()[:24]

    def module_path(self) -> str:
        return os.path.join(GEN_DIR, f"nl_{self.module_key()}.hsaco")

    def build_module(self, verbose: bool = False) -> str:
        """Compile (or reuse, by content hash) the gfx950 code object; returns its path."""
        path = self.module_path()
        if os.path.exists(path):
            return path
        os.makedirs(GEN_DIR, exist_ok=True)
        src = os.path.join(GEN_DIR, f"nl_{self.module_key()}.hip")
        with open(src, "w") as f:
            f.write(self.hip_source())
        tmp_dir = tempfile.mkdtemp(prefix="mcpx_gen_")
        tmp = os.path.join(tmp_dir, os.path.basename(path))
        cmd = [HIPCC, *_MODULE_FLAGS, "-I", CSRC, "-save-temps", "-o", tmp, src]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True, cwd=tmp_dir)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on the generated module {src}:\n{r.stderr[-6000:]}")
        _check_hazards(tmp_dir)
        os.replace(tmp, path)
        with open(os.path.splitext(path)[0] + ".dep", "w") as f:  # what __graft_entry__ prunes by
            f.write(deps_hash())
        shutil.rmtree(tmp_dir, ignore_errors=True)
        return path


def deps_hash() -> str:
    """Hash of the kernel headers and compiler flags every module is built with: the part of
    module_key() beyond the generated text.  A code object whose `.dep` record differs was built
    from other headers and can never be loaded again."""
    h = hashlib.sha256()
    for f in _MODULE_DEPS:
        h.update(f.encode() + b"\0" + open(os.path.join(CSRC, f), "rb").read())
    h.update(" ".join(_MODULE_FLAGS).encode())
    return h.hexdigest()[:24]


def _check_hazards(tmp_dir: str) -> None:
    """The inline-asm hazard check of the main build (mcp_amd/build.py) on the module's ISA."""
    checker = os.path.join(os.path.dirname(HERE), "tools", "check_dpp_hazards.py")
    if not os.path.exists(checker):
        raise RuntimeError(f"the inline-asm hazard checker {checker} is missing: refusing an unchecked module")
    asms = glob.glob(os.path.join(tmp_dir, "*gfx950*.s"))
    if not asms:
        raise RuntimeError(f"no device .s under {tmp_dir} for the hazard check (-save-temps naming changed?)")
    for asm in asms:
        r = subprocess.run([sys.executable, checker, asm], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"inline-asm hazard in the generated module:\n{r.stdout[-2000:]}")
