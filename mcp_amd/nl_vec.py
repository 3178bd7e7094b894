"""Lane-parallel form of a generated module's per-step evaluation (mcpx_nl_eval).

The generated C evaluates G, H and the z-dependent Jacobian entries as straight-line code
(codegen.py, one lane of the wave runs it, since its values are wave-uniform): ~270
dependent double operations a Newton step at the lane-change horizon T = 2, ~5 K cycles
of a lone wave's ~24 K.  Here the SAME expression trees (the printer's operation order,
the same CSE temporaries) are rewritten as chains

    acc = A₀·B₀;  acc = acc + A₁·B₁;  …           (every product and sum rounded once)

whose operands are atoms: a constant, an entry of z or θ, or an earlier chain's result.
The rewrite is exact — it changes no rounding:

* ``x + y`` and ``x − y`` of the C text are ``acc + (±y)``: IEEE subtraction is the addition
  of the negation, and a negation is exact;
* a plain operand ``v`` becomes the product ``1.0·v`` (exact, signed zeros and NaN kept);
* a negated product ``−(a·b)`` folds its sign into a constant factor (``(−c)·b``: rounding
  is sign-symmetric); two non-constant factors take a ``(−1.0)·a`` chain first;
* any operand that is not an atom (a nested sum, a product of three factors, …) becomes a
  chain of its own, evaluated one level earlier.

Chains of one level are independent, so the wave evaluates up to 64 of them per
instruction (lane = chain, with `slots` rounds of 64 per level); lanes with a shorter or no
chain add ``(−0)·1 = −0``, which leaves every value unchanged (``x + (−0) = x`` for all x,
±0 included).  The oracle keeps compiling the straight-line C text; tests/test_nonlinear.py
checks the emulation below against it bit for bit, and the GPU tests the kernel.

Only polynomial expressions (sums, products, integer powers ≥ 0) are rewritten; a module
with a division, a square root or a transcendental function keeps the straight-line eval.
"""

from __future__ import annotations

import numpy as np

# atoms: ("c", value) constant | ("z", j) decision variable | ("t", k) parameter θ_k |
#        ("T", i) chain i's result
ONE = ("c", 1.0)


class Unsupported(Exception):
    pass


class _Builder:
    def __init__(self, names):
        self.names = names  # sympy Symbol → atom
        self.chains = []  # list of list of (A, B) terms (sign folded into constants)

    # --- the printer's operation trees (codegen._Printer, same ordering calls) ------------
    def tree(self, e):
        import sympy as sp

        if e in self.names:
            return ("atom", self.names[e])
        if e.is_Number:
            return ("atom", ("c", float(e)))
        if e.is_Add:
            out = None
            for t in e.as_ordered_terms():
                neg = False
                c, rest = t.as_coeff_Mul()
                if c == -1 and rest != 1:
                    neg, t = True, rest
                s = self.tree(t)
                if out is None:
                    out = ("neg", s) if neg else s
                else:
                    out = ("sub" if neg else "add", out, s)
            return out
        if e.is_Mul:
            c, rest = e.as_coeff_Mul()
            if c == -1:
                return ("neg", self.tree(rest))
            facs = list(e.as_ordered_factors())
            if any(f.is_Pow and f.exp.is_Integer and f.exp < 0 for f in facs):
                raise Unsupported("division")
            out = None
            for f in facs:
                s = self.tree(f)
                out = s if out is None else ("mul", out, s)
            return out if out is not None else ("atom", ONE)
        if e.is_Pow and e.exp.is_Integer and int(e.exp) >= 0:
            k = int(e.exp)
            if k == 0:
                return ("atom", ONE)
            b = self.tree(e.base)
            out = b
            for _ in range(k - 1):
                out = ("mul", out, b)
            return out
        raise Unsupported(type(e).__name__)

    # --- chains -------------------------------------------------------------------------
    def new_chain(self, terms) -> tuple:
        self.chains.append(terms)
        return ("T", len(self.chains) - 1)

    def atomize(self, t):
        """An atom holding the value of tree t (a new chain unless t is an atom)."""
        if t[0] == "atom":
            return t[1]
        return self.new_chain(self.chain(t))

    def signed_atom(self, t):
        """(sign, atom) with value sign·atom for t = atom or neg(…)."""
        if t[0] == "neg":
            s, a = self.signed_atom(t[1])
            return -s, a
        return 1, self.atomize(t)

    def term(self, t, sign=1):
        """One chain term (A, B) with value sign·(tree t), a single rounding."""
        if t[0] == "neg":
            return self.term(t[1], -sign)
        if t[0] == "mul":
            sa, a = self.signed_atom(t[1])
            sb, b = self.signed_atom(t[2])
            return self.fold(sign * sa * sb, a, b)
        if t[0] == "atom":
            return self.fold(sign, t[1], ONE)
        return self.fold(sign, self.atomize(t), ONE)  # a sum as a term: its own chain

    def fold(self, sign, a, b):
        """(A, B) with A·B = sign·a·b exactly: the sign goes into a constant factor."""
        if b[0] == "c" and a[0] != "c":
            a, b = b, a  # the constant first (a product commutes exactly)
        if sign < 0:
            if a[0] == "c":
                a = ("c", -a[1])
            else:  # two non-constant factors: −a as a chain of its own
                a = self.new_chain([(("c", -1.0), a)])
        return (a, b)

    def chain(self, t):
        if t[0] == "add":
            return self.chain(t[1]) + [self.term(t[2])]
        if t[0] == "sub":
            return self.chain(t[1]) + [self.term(t[2], -1)]
        return [self.term(t)]


class Program:
    """Chains, their levels and the per-lane tables of the device evaluation."""

    def __init__(self, n, m, p, size, chains, outputs):
        self.n, self.m, self.p, self.size = n, m, p, size
        self.chains = chains  # list of term lists
        self.outputs = outputs  # chain index → blk index (outputs), others are temporaries
        lv = [0] * len(chains)
        for i, terms in enumerate(chains):  # chains only refer to earlier chains
            deps = [x[1] for t in terms for x in t if x[0] == "T"]
            assert all(d < i for d in deps)
            lv[i] = 1 + max([lv[d] for d in deps] + [0])
        self.level = lv
        # distinct constants by bit pattern (−0.0 ≠ +0.0; a set of floats would merge them)
        seen, self.consts = set(), []
        for v in [1.0, -0.0] + [x[1] for terms in chains for t in terms for x in t if x[0] == "c"]:
            k = np.float64(v).tobytes()
            if k not in seen:
                seen.add(k)
                self.consts.append(v)
        self.temps = [i for i in range(len(chains)) if i not in outputs]
        # ev layout (doubles): blk | z (n + 2m) | θ (p) | constants | temporaries | dummy
        self.off_z = size
        self.off_t = self.off_z + n + 2 * m
        self.off_c = self.off_t + p
        self.off_tmp = self.off_c + len(self.consts)
        tmp_slot = {c: k for k, c in enumerate(self.temps)}
        self.off_dummy = self.off_tmp + len(self.temps)
        self.ev_size = self.off_dummy + 1
        cidx = {np.float64(v).tobytes(): k for k, v in enumerate(self.consts)}

        def addr(x):  # ev index of an atom
            if x[0] == "c":
                return self.off_c + cidx[np.float64(x[1]).tobytes()]
            if x[0] == "z":
                return self.off_z + x[1]
            if x[0] == "t":
                return self.off_t + x[1]
            return self.dst(x[1], tmp_slot)

        self._addr = addr
        self._tmp_slot = tmp_slot
        # schedule: per level, chains by length (longest first), 64 per slot
        self.schedule = []  # [(level, [ [chain or None] * 64 per slot ])]
        for L in range(1, max(lv + [0]) + 1):
            cs = sorted((i for i in range(len(chains)) if lv[i] == L), key=lambda i: -len(chains[i]))
            slots = [cs[k:k + 64] for k in range(0, len(cs), 64)]
            self.schedule.append([s + [None] * (64 - len(s)) for s in slots])

    def dst(self, i, tmp_slot=None):
        tmp_slot = tmp_slot if tmp_slot is not None else self._tmp_slot
        return self.outputs[i] if i in self.outputs else self.off_tmp + tmp_slot[i]

    def tables(self):
        """(steps, words, dsts): per slot its number of term steps; per (slot, step) 64 words
        (ev index of A | ev index of B << 16, as byte offsets); per slot 64 destination byte
        offsets.  Padding lanes read (−0)·1 and write the dummy slot."""
        pad = (self._addr(("c", -0.0)) * 8) | ((self._addr(ONE) * 8) << 16)
        steps, words, dsts = [], [], []
        for level in self.schedule:
            for slot in level:
                k = max(len(self.chains[c]) for c in slot if c is not None)
                steps.append(k)
                for t in range(k):
                    row = []
                    for c in slot:
                        if c is None or t >= len(self.chains[c]):
                            row.append(pad)
                        else:
                            a, b = self.chains[c][t]
                            row.append((self._addr(a) * 8) | ((self._addr(b) * 8) << 16))
                    words.append(row)
                dsts.append([(self.dst(c) if c is not None else self.off_dummy) * 8 for c in slot])
        return steps, words, dsts

    def levels(self):
        return [len(level) for level in self.schedule]

    def emulate(self, th, z, blk):
        """numpy restatement of the device evaluation (float64, every operation rounded):
        writes the outputs into blk (a copy is not made)."""
        ev = np.zeros(self.ev_size)
        ev[:self.size] = blk
        ev[self.off_z:self.off_z + len(z)] = z
        ev[self.off_t:self.off_t + self.p] = th[:self.p]
        ev[self.off_c:self.off_c + len(self.consts)] = self.consts
        steps, words, dsts = self.tables()
        si = wi = 0
        for level in self.schedule:
            for slot in level:
                acc = None
                for t in range(steps[si]):
                    w = np.array(words[wi], dtype=np.int64)
                    a, b = ev[(w & 0xFFFF) // 8], ev[(w >> 16) // 8]
                    prod = a * b
                    acc = prod if acc is None else acc + prod
                    wi += 1
                ev[np.array(dsts[si]) // 8] = acc  # lanes write distinct slots (padding: dummy)
                si += 1
        blk[:] = ev[:self.size]
        return blk


def build(nl, reps, red, entries, names, size: int | None = None) -> Program | None:
    """The chain program of the eval block (entries = [(blk index, expr)], reps/red = the CSE
    the C text was printed from, names = the printer's Symbol → operand map of z / θ; `size` =
    doubles of the block array the entries index, nl.size by default — the band kernel's
    compact array is smaller).  None when an expression is not polynomial or the ev array
    would not fit 16-bit byte offsets."""
    atom_of = {}
    for sym, txt in names.items():
        if txt.startswith("th["):
            atom_of[sym] = ("t", int(txt[3:-1]))
        elif txt.startswith("MCPX_NL_Z("):
            atom_of[sym] = ("z", int(txt[len("MCPX_NL_Z("):-1]))
    b = _Builder(atom_of)
    outputs = {}
    try:
        for sym, e in reps:
            # a CSE temporary: its own chain, referenced by later chains as an atom (a
            # temporary that is a bare atom is an alias of it)
            b.names[sym] = b.atomize(b.tree(e))
        for (idx, _), e in zip(entries, red):
            terms = b.chain(b.tree(e))  # may add chains of its operands first
            outputs[len(b.chains)] = idx
            b.chains.append(terms)
    except Unsupported:
        return None
    prog = Program(nl.n, nl.m, nl.p, nl.size if size is None else size, b.chains, outputs)
    if prog.ev_size * 8 >= 65536:
        return None
    steps, _, _ = prog.tables()
    # the one-wave kernel keeps one operand word per term step and one destination per slot in
    # VGPRs for the whole solve (eval_vec): beyond these caps they would spill to scratch
    if sum(steps) > MAX_WORDS or len(steps) > MAX_SLOTS:
        return None
    return prog


MAX_WORDS, MAX_SLOTS = 64, 32  # VGPR budget of eval_vec's word and destination tables


def emit(prog: Program, macro: str = "MCPX_NL_VEC", name: str = "mcpx_nl_vec") -> list:
    """C lines of the tables (generated module text): the ev layout, the constants, the term
    steps per slot (a macro list, for compile-time unrolling), per (slot, step) the 64 lanes'
    operand words and per slot the 64 destinations.  (`macro` / `name`: MCPX_NL_CVEC /
    mcpx_nl_cvec for the band kernel's program on the compact array.)"""
    steps, words, dsts = prog.tables()
    lit = lambda v: ("-" if np.signbit(v) else "") + float(abs(v)).hex()
    flat = lambda rows: ", ".join(str(x) for r in rows for x in r)
    return [
        "/* lane-parallel eval (mcp_amd/nl_vec.py): chains of one rounding per product and sum, the",
        "   outputs and CSE temporaries of mcpx_nl_eval in the same operation order, 64 chains per slot */",
        f"#define {macro} 1",
        f"#define {macro}_EV {prog.ev_size}",
        f"#define {macro}_OFF_Z {prog.off_z}",
        f"#define {macro}_OFF_T {prog.off_t}",
        f"#define {macro}_OFF_C {prog.off_c}",
        f"#define {macro}_NC {len(prog.consts)}",
        f"#define {macro}_NSLOT {len(steps)}",
        f"#define {macro}_NWORD {len(words)}",
        f"#define {macro}_STEPS {', '.join(map(str, steps))}",
        f"MCPX_NL_TABLE double {name}_const[{len(prog.consts)}] = {{{', '.join(lit(v) for v in prog.consts)}}};",
        f"MCPX_NL_TABLE uint32_t {name}_word[{len(words) * 64}] = {{{flat(words)}}};",
        f"MCPX_NL_TABLE uint32_t {name}_dst[{len(dsts) * 64}] = {{{flat(dsts)}}};",
    ]
