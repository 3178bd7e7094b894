"""G/H as text: the language-neutral route from a Julia `PrimalDualMCP` to a device module.

The reference builds F!, ∇F_z! and ∇F_θ! from Symbolics expressions of G and H
(`PrimalDualMCP(G_symbolic, H_symbolic, x_symbolic, y_symbolic, θ_symbolic)`,
src/mcp.jl:55-120; the games reach it through src/game.jl:42 → :182-210).  A Julia
caller of the C ABI has those expressions but no sympy: it prints them, one row a
line, in Julia's own syntax (what `string(::Num)` / `print` of Symbolics gives), and
this module parses the text into the expressions `mcp_amd.codegen.NLSystem` compiles.
The same text always gives the same module (content hash), the one the Python front
end's sympy tracing gives for the same G/H.

GH text (`*.gh`), one item per line, `#` starts a comment:

    n = 40                      unconstrained_dimension
    m = 50                      constrained_dimension
    p = 10                      parameter_dimension
    G[1] = x[1] - θ[1] + 2(x[2]^2)
    ...                         G[1..n], H[1..m], any order, each once
    H[50] = (x₁ - x₅)^2 + (x₂ - x₆)^2 - 4

Optional declarations give the scalars' own names, in order, as Symbolics prints them
(the games of src/game.jl:66-80 call them x, λ̃, μ̃, θ):

    x = [x₁, x₂, …, λ̃₁, …]     the n unconstrained scalars
    y = [μ̃₁, …]                the m constrained ones
    θ = [θ₁, …]                the p parameters

Without a declaration a role's scalars are written by position: `x[i]`, `x₁₂` or `x_12`
(likewise y, θ or theta; 1-based).  The module does not depend on the names
(mcp_amd/codegen.py renames by position).  Expressions are Julia syntax:

* numbers: integers (exact), decimal floats (`0.1`, `1.0e-5`: the Float64 they denote,
  as Julia reads them), rationals `a//b` (exact);
* `+ - * / ^ //`, unary ±, parentheses, Julia precedence (`^` right-associative and
  above unary minus: `-x^2` = −(x²); `//` above `*` `/`);
* juxtaposition of a numeric literal with what follows (`2x`, `0.5(x + y)`, `2x^2` =
  2·x²), binding tighter than `*` `/` as in Julia (`1/2x` = 1/(2x));
* elementary calls `sin cos tan exp log sqrt abs tanh sinh cosh asin acos atan` and
  `atan(y, x)`;
* Symbolics' prefix call form `(+)(a, b, …)`, `(*)(…)`, `(-)(a)`, `(-)(a, b)`, `(/)(a, b)`,
  `(^)(a, b)` (the `toexpr` spelling).

A line whose parentheses do not balance continues on the next one.

    python -m mcp_amd.symtext build problem.gh     # → JSON: the code object's path, n, m, p, key

builds (or reuses) the gfx950 code object that `mcpx_module_load` takes (INTEGRATION.md
shows the Julia side).  `load(path)` returns the parsed rows and symbols;
`mcp_amd.api.PrimalDualMCP.from_text(path)` the front-end MCP; `write(path, G, H, xs, ys, ts)`
prints sympy rows in the same syntax (tests, and the round trip).
"""

from __future__ import annotations

import json
import re
import sys

_SUB = "₀₁₂₃₄₅₆₇₈₉"
_FUNCS1 = {"sin", "cos", "tan", "exp", "log", "sqrt", "abs", "tanh", "sinh", "cosh", "asin", "acos", "atan"}
_VARS = {"x": "x", "y": "y", "θ": "θ", "theta": "θ"}

_TOKEN = re.compile(r"""
    (?P<ws>[ \t\r\n]+)
  | (?P<num>(?:\d+\.\d*|\.\d+)(?:[eE][+-]?\d+)?|\d+[eE][+-]?\d+|\d+)
  | (?P<id>[^\W\d][\w\u0300-\u036f]*)
  | (?P<op>//|[-+*/^(),\[\]])
""", re.VERBOSE)


class GHSyntaxError(ValueError):
    pass


def _sp():
    import sympy

    return sympy


def _tokens(text: str):
    """(kind, text, adjacent-to-previous) triples."""
    out, pos, gap = [], 0, True
    while pos < len(text):
        mt = _TOKEN.match(text, pos)
        if not mt:
            raise GHSyntaxError(f"unexpected character {text[pos]!r} at {pos}: {text}")
        pos = mt.end()
        kind = mt.lastgroup
        if kind == "ws":
            gap = True
            continue
        out.append((kind, mt.group(), not gap))
        gap = False
    out.append(("end", "", False))
    return out


def _split_name(name: str):
    """`x₁₂` / `x_12` → ("x", 12); `x` → ("x", None)."""
    i = len(name)
    while i > 0 and name[i - 1] in _SUB:
        i -= 1
    if i < len(name):
        return name[:i], int("".join(str(_SUB.index(c)) for c in name[i:]))
    base, sep, idx = name.rpartition("_")
    if sep and base and idx.isdigit():
        return base, int(idx)
    return name, None


class _Parser:
    """Pratt parser of one Julia expression (module docstring) into a sympy expression."""

    # binding powers: + - 10, * / 20, // 25, unary ± 30, juxtaposition 35, ^ 40 (right)
    _BIN = {"+": (10, 11), "-": (10, 11), "*": (20, 21), "/": (20, 21), "//": (25, 26), "^": (41, 40)}

    def __init__(self, text: str, symbols: dict):
        self.toks = _tokens(text)
        self.i = 0
        self.text = text
        self.symbols = symbols  # ("x", i) → Symbol

    def peek(self, k=0):
        return self.toks[self.i + k]

    def take(self, want=None):
        t = self.toks[self.i]
        if want is not None and t[1] != want:
            raise GHSyntaxError(f"expected {want!r}, got {t[1] or 'end of line'!r} in: {self.text}")
        self.i += 1
        return t

    def parse(self):
        e = self.expr(0)
        if self.peek()[0] != "end":
            raise GHSyntaxError(f"unexpected {self.peek()[1]!r} in: {self.text}")
        return e

    def expr(self, min_bp: int):
        lhs = self.prefix()
        while True:
            kind, tok, adj = self.peek()
            if kind == "op" and tok in self._BIN:
                lbp, rbp = self._BIN[tok]
                if lbp < min_bp:
                    break
                self.take()
                lhs = self.binary(tok, lhs, self.expr(rbp))
                continue
            break
        return lhs

    def binary(self, op, a, b):
        sp = _sp()
        if op == "+":
            return a + b
        if op == "-":
            return a - b
        if op == "*":
            return a * b
        if op == "/":
            return a / b
        if op == "^":
            return a ** b
        if op == "//":
            if not (a.is_Integer and b.is_Integer):
                raise GHSyntaxError(f"// takes two integers (a Julia Rational) in: {self.text}")
            return sp.Rational(int(a), int(b))
        raise AssertionError(op)

    def args(self):
        self.take("(")
        out = []
        if self.peek()[1] != ")":
            out.append(self.expr(0))
            while self.peek()[1] == ",":
                self.take()
                out.append(self.expr(0))
        self.take(")")
        return out

    def prefix(self):
        sp = _sp()
        kind, tok, _ = self.take()
        if kind == "num":
            v = sp.Integer(int(tok)) if re.fullmatch(r"\d+", tok) else sp.Float(float(tok))
            return self.juxtapose(v)
        if kind == "op" and tok in "+-":
            v = self.expr(30)
            return v if tok == "+" else -v
        if kind == "op" and tok == "(":
            k2, t2, _ = self.peek()
            # Symbolics' prefix call form: (+)(a, b, …)
            if k2 == "op" and t2 in ("+", "-", "*", "/", "^", "//") and self.peek(1)[1] == ")" \
                    and self.peek(2)[1] == "(":
                self.take()
                self.take(")")
                return self.call_op(t2, self.args())
            e = self.expr(0)
            self.take(")")
            return e
        if kind == "id":
            if self.peek()[1] == "(" and self.peek()[2]:
                return self.call(tok, self.args())
            if self.peek()[1] == "[":
                self.take("[")
                e = self.expr(0)
                self.take("]")
                if not e.is_Integer:
                    raise GHSyntaxError(f"{tok}[…] needs an integer index in: {self.text}")
                tok = f"{tok}[{int(e)}]"
            return self.variable(tok)
        raise GHSyntaxError(f"unexpected {tok or 'end of line'!r} in: {self.text}")

    def juxtapose(self, v):
        """A numeric literal directly followed by a name or '(' multiplies it (Julia)."""
        kind, tok, adj = self.peek()
        if adj and (kind == "id" or tok == "("):
            return v * self.expr(35)
        return v

    def variable(self, spelling):
        sym = self.symbols.get(spelling)
        if sym is None:
            base, idx = _split_name(spelling.split("[")[0])
            if "[" in spelling:
                idx = int(spelling.split("[")[1].rstrip("]"))
            sym = self.symbols.get((_VARS.get(base), idx))
        if sym is None:
            raise GHSyntaxError(f"unknown name {spelling!r} (x[i], y[i], θ[i] by position, or the names the "
                                f"header declares; within n, m, p) in: {self.text}")
        return sym

    def call(self, name, a):
        sp = _sp()
        if name == "atan" and len(a) == 2:
            return sp.atan2(a[0], a[1])
        if name not in _FUNCS1 or len(a) != 1:
            raise GHSyntaxError(f"unsupported call {name}({len(a)} args) in: {self.text}")
        if name == "sqrt":
            return sp.sqrt(a[0])
        if name == "abs":
            return sp.Abs(a[0])
        return getattr(sp, name)(a[0])

    def call_op(self, op, a):
        if op in ("+", "*") and a:
            out = a[0]
            for b in a[1:]:
                out = self.binary(op, out, b)
            return out
        if op == "-" and len(a) == 1:
            return -a[0]
        if len(a) == 2:
            return self.binary(op, a[0], a[1])
        raise GHSyntaxError(f"({op}) with {len(a)} arguments in: {self.text}")


def symbols(n: int, m: int, p: int):
    """The front end's scalars (mcp_amd.api.make_variables): x_1…x_n, y_1…y_m, θ_1…θ_p."""
    from .api import make_variables

    return list(make_variables("x", n)), list(make_variables("y", m)), list(make_variables("θ", p))


def _lines(text: str):
    """Logical lines: comments stripped, lines with open parentheses joined to the next."""
    buf, depth = "", 0
    for raw in text.splitlines():
        line = raw.split("#", 1)[0]
        if not line.strip() and not buf:
            continue
        buf = f"{buf} {line}" if buf else line
        depth = buf.count("(") + buf.count("[") - buf.count(")") - buf.count("]")
        if depth <= 0:
            yield buf.strip()
            buf = ""
    if buf.strip():
        raise GHSyntaxError(f"unbalanced parentheses at the end: {buf.strip()[:80]}")


def loads(text: str):
    """GH text → (G, H, xs, ys, ts): sympy rows and the scalars they are written in."""
    dims, rows = {}, {"G": {}, "H": {}}
    items = []
    decl = {}
    for line in _lines(text):
        lhs, eq, rhs = line.partition("=")
        if not eq:
            raise GHSyntaxError(f"expected `name = …`: {line}")
        lhs = lhs.strip()
        if lhs in ("n", "m", "p"):
            if lhs in dims:
                raise GHSyntaxError(f"{lhs} given twice")
            dims[lhs] = int(rhs.strip())
            continue
        if lhs in _VARS:  # x = [name, name, …]: the spellings of the role's scalars, in order
            role, body = _VARS[lhs], rhs.strip()
            if role in decl or not (body.startswith("[") and body.endswith("]")):
                raise GHSyntaxError(f"expected one `{lhs} = [name, …]` declaration: {line[:80]}")
            decl[role] = ["".join(v.split()) for v in body[1:-1].split(",") if v.strip()]
            continue
        mt = re.fullmatch(r"([GH])\s*\[\s*(\d+)\s*\]|([GH])([₀-₉]+)|([GH])_(\d+)", lhs)
        if not mt:
            raise GHSyntaxError(f"expected n, m, p, G[i] or H[k] on the left: {line}")
        which = mt.group(1) or mt.group(3) or mt.group(5)
        idx = mt.group(2) or mt.group(6)
        idx = int(idx) if idx else int("".join(str(_SUB.index(c)) for c in mt.group(4)))
        items.append((which, idx, rhs, line))
    for k in ("n", "m", "p"):
        if k not in dims or dims[k] < 0:
            raise GHSyntaxError(f"the header must give {k} = <count>")
    n, m, p = dims["n"], dims["m"], dims["p"]
    xs, ys, ts = symbols(n, m, p)
    table = {}
    for role, syms in (("x", xs), ("y", ys), ("θ", ts)):
        if role in decl:  # declared spellings only
            if len(decl[role]) != len(syms):
                raise GHSyntaxError(f"{role} declares {len(decl[role])} names for {len(syms)} scalars")
            for name, sym in zip(decl[role], syms):
                if name in table:
                    raise GHSyntaxError(f"name {name} declared twice")
                table[name] = sym
        else:  # by position: x[i], x₁, x_1
            table.update({(role, i + 1): sym for i, sym in enumerate(syms)})
    for which, idx, rhs, line in items:
        size = n if which == "G" else m
        if not 1 <= idx <= size:
            raise GHSyntaxError(f"{which}[{idx}] is outside 1..{size}: {line}")
        if idx in rows[which]:
            raise GHSyntaxError(f"{which}[{idx}] given twice")
        rows[which][idx] = _Parser(rhs.strip(), table).parse()
    for which, size in (("G", n), ("H", m)):
        missing = [i for i in range(1, size + 1) if i not in rows[which]]
        if missing:
            raise GHSyntaxError(f"{which} rows missing: {missing[:8]}{' …' if len(missing) > 8 else ''}")
    G = [rows["G"][i] for i in range(1, n + 1)]
    H = [rows["H"][i] for i in range(1, m + 1)]
    return G, H, xs, ys, ts


def load(path: str):
    with open(path, encoding="utf-8") as f:
        return loads(f.read())


# ---- printing (sympy → Julia syntax) --------------------------------------------------


class _Julia:
    """sympy → Julia text that `loads` reads back to the same expression tree."""

    _FN = {"sin": "sin", "cos": "cos", "tan": "tan", "exp": "exp", "log": "log", "tanh": "tanh",
           "sinh": "sinh", "cosh": "cosh", "asin": "asin", "acos": "acos", "atan": "atan", "Abs": "abs"}

    def __init__(self, names: dict):
        self.names = names

    def atom(self, e) -> str:
        """e printed so that it can be an operand of any operator."""
        sp = _sp()
        s = self(e)
        if e in self.names or isinstance(e, sp.Function) or (e.is_Pow and e.exp == sp.Rational(1, 2)):
            return s  # a name or a call
        if (e.is_Integer or e.is_Float) and e >= 0:
            return s
        return f"({s})"

    def __call__(self, e) -> str:
        sp = _sp()
        if e in self.names:
            return self.names[e]
        if e.is_Integer:
            return str(int(e))
        if e.is_Rational:
            return f"({int(e.p)}//{int(e.q)})"
        if e.is_Float:
            f = float(e)
            if f != f or f in (float("inf"), float("-inf")):
                raise ValueError(f"non-finite constant {e}")
            return repr(f)
        if e.is_Add:  # one n-ary sum: reads back to the same Add
            return " + ".join(self.atom(t) if t.is_Number else self(t) for t in e.args)
        if e.is_Mul:
            # the numeric coefficient last: with two factors a coefficient first would
            # distribute over a sum when read back (2*(a + b) → 2a + 2b)
            c, rest = e.as_coeff_Mul()
            facs = list(rest.args) if rest.is_Mul else [rest]
            parts = [self.atom(f) for f in facs]
            if c != 1:
                parts.append(self.atom(c))
            return "*".join(parts)
        if e.is_Pow:
            b, x = e.base, e.exp
            if x == sp.Rational(1, 2):
                return f"sqrt({self(b)})"
            return f"{self.atom(b)}^{self.atom(x) if not (x.is_Integer and x >= 0) else str(int(x))}"
        if isinstance(e, sp.Function):
            name = type(e).__name__
            if name == "atan2":
                return f"atan({self(e.args[0])}, {self(e.args[1])})"
            if name not in self._FN:
                raise NotImplementedError(f"no GH-text spelling for {name}")
            return f"{self._FN[name]}({', '.join(self(a) for a in e.args)})"
        raise NotImplementedError(f"no GH-text spelling for {type(e).__name__}: {e}")


def _julia_name(sym) -> str:
    """A front-end symbol `base_12` as Symbolics prints its scalar: `base₁₂`."""
    base, idx = _split_name(sym.name)
    return sym.name if idx is None else base + "".join(_SUB[int(c)] for c in str(idx))


def dumps(G, H, xs, ys, ts, style: str = "index") -> str:
    """sympy rows → GH text.  style "index": x[1] by position; "subscript": x₁ by position;
    "names": the symbols' own names in Symbolics' spelling (x₁ … λ̃₁₆, μ̃₁ …), declared in the
    header — what the Julia side writes."""
    def nm(base, i):
        return f"{base}[{i}]" if style == "index" else base + "".join(_SUB[int(c)] for c in str(i))

    if style == "names":
        names = {s: _julia_name(s) for s in list(xs) + list(ys) + list(ts)}
        if len(set(names.values())) != len(names):
            raise ValueError("two symbols print to the same name")
    else:
        names = {s: nm("x", i + 1) for i, s in enumerate(xs)}
        names.update({s: nm("y", i + 1) for i, s in enumerate(ys)})
        names.update({s: nm("θ", i + 1) for i, s in enumerate(ts)})
    pr = _Julia(names)
    out = ["# mcpx GH text (mcp_amd/symtext.py)", f"n = {len(xs)}", f"m = {len(ys)}", f"p = {len(ts)}"]
    if style == "names":
        out += [f"{role} = [{', '.join(names[s] for s in syms)}]" for role, syms in (("x", xs), ("y", ys), ("θ", ts))]
    out += [f"G[{i + 1}] = {pr(_sp().sympify(e))}" for i, e in enumerate(G)]
    out += [f"H[{k + 1}] = {pr(_sp().sympify(e))}" for k, e in enumerate(H)]
    return "\n".join(out) + "\n"


def write(path: str, G, H, xs, ys, ts, style: str = "index") -> None:
    with open(path, "w", encoding="utf-8") as f:
        f.write(dumps(G, H, xs, ys, ts, style))


# ---- the module ------------------------------------------------------------------------


def nl_system(path: str):
    """The generated-code system (mcp_amd.codegen.NLSystem) of a GH file, whatever its G/H
    (affine ones included: the C ABI's module route takes every MCP)."""
    from .codegen import NLSystem

    return NLSystem(*load(path))


def build(path: str, verbose: bool = False) -> dict:
    """Compile (or reuse by content hash) the gfx950 code object of a GH file."""
    nl = nl_system(path)
    mod = nl.build_module(verbose=verbose)
    return {"module": mod, "n": nl.n, "m": nl.m, "p": nl.p, "key": nl.key}


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if len(argv) != 2 or argv[0] not in ("build", "check"):
        print("usage: python -m mcp_amd.symtext {build|check} FILE.gh", file=sys.stderr)
        return 2
    if argv[0] == "check":
        G, H, xs, ys, ts = load(argv[1])
        print(json.dumps({"n": len(xs), "m": len(ys), "p": len(ts)}))
        return 0
    print(json.dumps(build(argv[1])))
    return 0


if __name__ == "__main__":
    sys.exit(main())
