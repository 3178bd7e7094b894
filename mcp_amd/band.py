"""Banded elimination plan of a generated module's SCHUR step (csrc/ipm_nl_band.hpp).

The reference factors the Newton system with UMFPACK, a sparse LU whose symbolic phase
orders the columns for sparsity before the numeric factorisation with partial pivoting
(src/solver.jl:50,61,83).  The generated modules' n×n Schur complement

    S = (P + tol·I) − Q D⁻¹ R            (∂H/∂y ≡ 0, P = ∂G/∂x, Q = ∂G/∂y, R = ∂H/∂x)

has a structure known at codegen time, and for trajectory games it is very sparse (the
lane-change game: 136 of 1,600 entries at horizon T = 2, 840 of 40,000 at T = 10; every
row has at most 6).  This module is that symbolic phase for the GPU:

* a symmetric permutation π (S' = S[π][:, π]) from Cuthill-McKee orderings of the pattern
  of S + Sᵀ, one per connected component, the start vertex and direction with the
  smallest bandwidth (the lane-change game: 9 at T = 2, 16 at T = 10);
* the lower / upper bandwidths pl, pu of S' and the window width WC (pl + pu + 1 rounded up
  to a multiple of 4): partial pivoting by row interchanges keeps every row that can be a
  pivot candidate at step k among the rows ≤ k + pl, and every row of the window inside
  the columns [k, k + pl + pu] (the band LU of LAPACK gbtrf, with implicit pivoting here);
* the compact storage of the generated Jacobian (structural nonzeros only, in the dense
  block order) and the formation tables of S' and rr' on it.

The elimination itself — partial pivoting over the window rows, first-max rule, the
oracle's `lu_solve_x(rcp = 1)` arithmetic restricted to the window columns — is restated
in oracle/ipm_oracle.c (`lu_band_solve`); on finite values it equals the dense LU of S'
(out-of-band entries are exact zeros) and therefore differs from the dense LU of S only by
the order of the columns, as UMFPACK's does.
"""

from __future__ import annotations

import numpy as np

MAX_SLOTS = 64    # window rows (pl + 1): 16-lane DPP rows × NJ ≤ 4 register blocks
MAX_WC = 64       # window columns: NCB = WC / 4 ≤ 16 registers per slot block


def s_pattern(nl) -> np.ndarray:
    """Structural pattern of S = (P + tol·I) − Q D⁻¹ R (the diagonal always)."""
    n = nl.n
    (qp, qi), (rp, ri) = nl.structure()
    ents = {i for i, _ in nl.const_entries} | {i for i, _ in nl.var_entries}
    S = np.zeros((n, n), bool)
    for idx in ents:
        if nl.OFF_P <= idx < nl.OFF_Q:
            j, i = divmod(idx - nl.OFF_P, n)
            S[i, j] = True
    for i in range(n):
        for k in qi[qp[i]:qp[i + 1]]:
            for j in ri[rp[k]:rp[k + 1]]:
                S[i, j] = True
    np.fill_diagonal(S, True)
    return S


def window(S: np.ndarray, cperm, rperm=None) -> tuple[int, int]:
    """(rows, columns) of the elimination window for column order `cperm` and row order
    `rperm` (default: rows by their first nonzero column).  Rows enter one per step in row
    order (rows 0 .. W − 1 before step 0, row k + W after step k), so W must cover
    i + 1 − f(i) for every row i (f = first nonzero column): every row with a nonzero in
    column k is in the window at step k.  Columns: the window rows at step k reach column
    max l(r) over r ≤ k + W − 1 (l = last nonzero column; fill stays inside, as in a band
    LU), so WC − 1 ≥ that − k."""
    n = S.shape[0]
    Sc = S[:, cperm]
    f = Sc.argmax(1)                      # first nonzero column (every row has its diagonal)
    l = n - 1 - Sc[:, ::-1].argmax(1)     # last nonzero column
    rp = np.lexsort((np.arange(n), f)) if rperm is None else np.asarray(rperm)
    fs, ls = f[rp], l[rp]
    k = np.arange(n)
    W = int((k + 1 - fs).max())
    lmax = np.maximum.accumulate(ls)
    Wc = int((lmax[np.minimum(n, k + W) - 1] - k + 1).max())
    return W, Wc


def row_order(S: np.ndarray, cperm) -> np.ndarray:
    """Rows by their first nonzero column in `cperm` order, ties by row index."""
    n = S.shape[0]
    f = np.array([np.nonzero(S[r][cperm])[0].min() for r in range(n)])
    return np.lexsort((np.arange(n), f)).astype(np.int64)


CM_EXHAUSTIVE = 1024
CM_STARTS = 16


def cm_order(S: np.ndarray) -> np.ndarray:
    """Column order: Cuthill-McKee per connected component of S + Sᵀ (components by their
    smallest vertex; isolated vertices last), each from the start vertex and direction whose
    whole order gives the smallest window (rows first, then columns; ties: the smaller
    start, forward before reverse).  Deterministic."""
    n = S.shape[0]
    A = S | S.T
    np.fill_diagonal(A, False)
    adj = [np.nonzero(A[i])[0].tolist() for i in range(n)]
    deg = [len(a) for a in adj]
    seen, comps = [False] * n, []
    for s in range(n):
        if seen[s]:
            continue
        comp, stack = [], [s]
        seen[s] = True
        while stack:
            v = stack.pop()
            comp.append(v)
            for w in adj[v]:
                if not seen[w]:
                    seen[w] = True
                    stack.append(w)
        comps.append(sorted(comp))
    order = [v for c in comps if len(c) == 1 for v in c]  # isolated vertices go last
    big = [c for c in comps if len(c) > 1]
    head = []
    for ci, comp in enumerate(big):
        best = None
        # every start vertex up to CM_EXHAUSTIVE vertices (each trial is an O(n²) window);
        # beyond that the CM_STARTS lowest-degree vertices (the pseudo-peripheral candidates)
        starts = comp if len(comp) <= CM_EXHAUSTIVE else sorted(comp, key=lambda v: (deg[v], v))[:CM_STARTS]
        for s in starts:
            o, mark, q = [s], {s}, 0
            while q < len(o):
                v = o[q]
                q += 1
                for w in sorted(adj[v], key=lambda w: (deg[w], w)):
                    if w not in mark:
                        mark.add(w)
                        o.append(w)
            for rev in (False, True):
                oo = o[::-1] if rev else o
                trial = np.asarray(head + oo + [v for c in big[ci + 1:] for v in c] + order)
                key = (*window(S, trial), s, rev)
                if best is None or key < best[0]:
                    best = (key, list(oo))
        head += best[1]
    return np.asarray(head + order, dtype=np.int64)


class BandPlan:
    """π, the bandwidths and the tables of the band kernel for one generated module."""

    def __init__(self, nl):
        n, m = nl.n, nl.m
        self.n, self.m = n, m
        S = s_pattern(nl)
        self.cperm = cm_order(S)                     # S' column → original variable
        self.rperm = row_order(S, self.cperm)        # S' row → original row
        self.iperm = np.empty(n, np.int64)
        self.iperm[self.cperm] = np.arange(n)        # original variable → S' column (δx order)
        self.ns, wcols = window(S, self.cperm, self.rperm)  # window rows (slots) and columns
        self.wc = max(4, -(-wcols // 4) * 4)
        self.nj = -(-self.ns // 16)
        self.ncb = self.wc // 4
        # compact storage: the structural entries in dense block order, then G, then H
        dense = sorted(i for i, _ in nl.const_entries + nl.var_entries)
        self.cslot = {idx: s for s, idx in enumerate(dense)}
        self.nnz = len(dense)
        self.c_g, self.c_h = self.nnz, self.nnz + n
        self.csize = self.nnz + n + m
        # S' entries, row-major in S' order: (r', c', P slot or −1, diag, [(Q slot, R slot, k)])
        terms = {pos: ks for pos, ks in nl.schur_entries()}
        Sp = S[np.ix_(self.rperm, self.cperm)]
        self.entries = []
        self.rowptr = [0]
        for r in range(n):
            i = int(self.rperm[r])
            for c in np.nonzero(Sp[r])[0]:
                j = int(self.cperm[c])
                ps = self.cslot.get(nl.OFF_P + j * n + i, -1)
                ks = terms.get(i * (n + 1) + j, [])
                tl = [(self.cslot[nl.OFF_Q + k * n + i], self.cslot[nl.OFF_R + j * m + k], k) for k in ks]
                self.entries.append((r, int(c), ps, i == j, tl))
            self.rowptr.append(len(self.entries))
        self.nnz_s = len(self.entries)
        (qp, qi), (rp, ri) = nl.structure()
        # rr' entries by S' row: G slot of i = π(r'), then −Q_ik·ty_k over K(i) ascending
        self.rr = [(self.c_g + int(i), [(self.cslot[nl.OFF_Q + k * n + int(i)], k) for k in qi[qp[i]:qp[i + 1]]])
                   for i in (int(v) for v in self.rperm)]
        # δy_k: R_kj over J(k) ascending, with the S' index of j (δx lives in S' order)
        self.dy = [[(self.cslot[nl.OFF_R + j * m + k], int(self.iperm[j])) for j in ri[rp[k]:rp[k + 1]]]
                   for k in range(m)]

    def fits(self) -> bool:
        # compact slots are packed two per 32-bit table word (Q slot | R slot << 16); entries
        # eight bits up in the entering-row table
        return (self.ns <= MAX_SLOTS and self.wc <= MAX_WC and self.n >= 2 and self.csize < 32768
                and self.nnz_s < (1 << 23))

    # ---- tables of the generated text (per-lane slots: entry e = lane + 64·r) ---------------
    @staticmethod
    def _lanes(items, width, pad):
        """items (list of tuples of `width` ints) → flat [(r·width + f)·64 + lane] tables."""
        R = max(1, -(-len(items) // 64))
        out = [pad] * (R * width * 64)
        for e, it in enumerate(items):
            r, ln = divmod(e, 64)
            for f, v in enumerate(it):
                out[(r * width + f) * 64 + ln] = v
        return R, out

    def tables(self) -> list:
        """C lines of the band kernel's tables (MCPX_NL_TABLE arrays)."""
        arr = lambda name, v, t="int32_t": f"MCPX_NL_TABLE {t} {name}[{max(len(v), 1)}] = {{{', '.join(map(str, v)) or '0'}}};"
        KT = max([1] + [len(e[4]) for e in self.entries])
        # S' formation: word 0 = P slot + 1 (0: none) | diag << 30; then KT × (Q slot | R slot << 16, k)
        form = []
        for (_, _, ps, dg, tl) in self.entries:
            w = [(ps + 1) | (int(dg) << 30)]
            for t in range(KT):
                if t < len(tl):
                    q, r, k = tl[t]
                    w += [q | (r << 16), k]
                else:
                    w += [-1, -1]
            form.append(tuple(w))
        fr, ftab = self._lanes(form, 1 + 2 * KT, -1)
        KQ = max([1] + [len(t) for _, t in self.rr])
        rrw = [tuple([g] + [x for t in range(KQ) for x in (tl[t] if t < len(tl) else (-1, -1))]) for g, tl in self.rr]
        rrr, rtab = self._lanes(rrw, 1 + 2 * KQ, -1)
        KR = max([1] + [len(t) for t in self.dy])
        dyw = [tuple(x for t in range(KR) for x in (tl[t] if t < len(tl) else (-1, -1))) for tl in self.dy]
        dyr, dtab = self._lanes(dyw, 2 * KR, -1)
        # entering rows: per S' row its (window index | entry << 8) pairs, EMAX per row, −1 padding
        emax = max(1, max(self.rowptr[r + 1] - self.rowptr[r] for r in range(self.n)))
        bent = []
        for r in range(self.n):
            row = [(self.entries[e][1] % self.wc) | (e << 8) for e in range(self.rowptr[r], self.rowptr[r + 1])]
            bent += row + [-1] * (emax - len(row))
        return [
            "/* band kernel (mcp_amd/band.py): S' = S[σ][:, π], a window of NS rows and WC columns */",
            "#define MCPX_NL_BAND 1",
            f"#define MCPX_NL_BAND_NS {self.ns}",
            f"#define MCPX_NL_BAND_WC {self.wc}",
            f"#define MCPX_NL_BAND_NNZ {self.nnz_s}",
            f"#define MCPX_NL_CSIZE {self.csize}",
            f"#define MCPX_NL_C_G {self.c_g}",
            f"#define MCPX_NL_C_H {self.c_h}",
            f"#define MCPX_NL_BF_R {fr}",
            f"#define MCPX_NL_BF_KT {KT}",
            f"#define MCPX_NL_BR_R {rrr}",
            f"#define MCPX_NL_BR_KQ {KQ}",
            f"#define MCPX_NL_BD_R {dyr}",
            f"#define MCPX_NL_BD_KR {KR}",
            f"#define MCPX_NL_BAND_EMAX {emax}",
            arr("mcpx_nl_band_rperm", self.rperm.tolist()),
            arr("mcpx_nl_band_cperm", self.cperm.tolist()),
            arr("mcpx_nl_band_iperm", self.iperm.tolist()),
            arr("mcpx_nl_bf_tab", ftab),
            arr("mcpx_nl_br_tab", rtab),
            arr("mcpx_nl_bd_tab", dtab),
            arr("mcpx_nl_bent_tab", bent),
        ]

    def compact_index(self, nl, idx: int) -> int:
        """Compact position of dense block index `idx` (structural entry, G or H)."""
        if idx in self.cslot:
            return self.cslot[idx]
        if nl.OFF_G <= idx < nl.OFF_G + self.n:
            return self.c_g + idx - nl.OFF_G
        if nl.OFF_H <= idx < nl.OFF_H + self.m:
            return self.c_h + idx - nl.OFF_H
        raise KeyError(idx)

    def lds_bytes(self, ev_size: int) -> int:
        """Static LDS of mcpx_nl_solve_band (the static_assert of csrc/ipm_nl_band.hpp): ev, S'
        values + a zero, rr', D⁻¹ and ty, δx (S' order), two entering-row images, and the U rows
        (WC + 2 doubles each) when they take at most 8 KB (else the slot's HBM workspace, and each
        row's rhs and 1 / u_kk in LDS for the back substitution: 2n doubles)."""
        u = self.n * (self.wc + 2)
        lds_u = u if 8 * u <= 8 * 1024 else 2 * self.n
        return 8 * (ev_size + self.nnz_s + 1 + self.n + 2 * self.m + self.n + 2 * self.wc + lds_u)


def plan(nl) -> BandPlan | None:
    if nl.has_s or nl.n < 2:
        return None
    bp = BandPlan(nl)
    return bp if bp.fits() else None


__all__ = ["BandPlan", "plan", "cm_order", "row_order", "s_pattern", "window"]
