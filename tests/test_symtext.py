"""GH text: G/H from the Julia side to a device module (mcp_amd/symtext.py).

The reference builds F!/∇F_z!/∇F_θ! from Symbolics expressions (src/mcp.jl:55-120; the games
through src/game.jl:42, 66-80).  A Julia caller of the C ABI prints those expressions as text
("Nonlinear G/H"); `symtext` parses the text into the expressions the code
generator compiles.  CPU: Julia's operator precedence, juxtaposition, the prefix call form of
Symbolics' `toexpr`, Unicode subscripts and declared names; errors that must be loud; a
hand-written file in Symbolics' print style and the committed lane-change file (the game's own
names λ̃, μ̃ declared) give the very module key of the sympy-traced MCP, so the same code object
and the same bits (checked on the oracle, which compiles the same generated text); the CLI.
GPU: the module built from the text solves the C4 batch bit-exactly against the oracle and
equals the traced game's solve.
"""

from __future__ import annotations

import json
import os
import subprocess
import sys

import numpy as np
import pytest

from mcp_amd import symtext
from mcp_amd.api import PrimalDualMCP

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
ROOT = os.path.dirname(HERE)


def _parse(expr, n=3, m=2, p=3):
    text = f"n = {n}\nm = {m}\np = {p}\n" + "".join(f"G[{i}] = 0\n" for i in range(2, n + 1)) \
        + "".join(f"H[{k}] = 0\n" for k in range(1, m + 1)) + f"G[1] = {expr}\n"
    G, H, xs, ys, ts = symtext.loads(text)
    return G[0], xs, ys, ts


@pytest.mark.parametrize("expr,want", [
    ("-x[1]^2", lambda x, y, t: -(x[0] ** 2)),
    ("2x[1]^2", lambda x, y, t: 2 * x[0] ** 2),
    ("1/2x[1]", lambda x, y, t: 1 / (2 * x[0])),
    ("x[1]^2^2", lambda x, y, t: x[0] ** 4),
    ("2^-1*x₂", lambda x, y, t: x[1] / 2),
    ("(1//3)*x_3 - θ[1]", lambda x, y, t: x[2] / 3 - t[0]),
    ("1.0e-5x₁ + 0.5(y₁ + y₂)", lambda x, y, t: 1.0e-5 * x[0] + 0.5 * (y[0] + y[1])),
    ("x[1]*-y[2]", lambda x, y, t: -x[0] * y[1]),
    ("(+)(x[1], (*)(-2, x[2], y[1]), 3)", lambda x, y, t: x[0] - 2 * x[1] * y[0] + 3),
    ("(-)(x[1]) + (-)(x[2], x[3]) + (/)(θ₂, x₁) + (^)(x₁, 3)",
     lambda x, y, t: -x[0] + x[1] - x[2] + t[1] / x[0] + x[0] ** 3),
    ("sin(x[1]) + atan(x[2], x[3]) + sqrt(abs(θ[3])) + exp(-x[1]^2)",
     lambda x, y, t: __import__("sympy").sin(x[0]) + __import__("sympy").atan2(x[1], x[2])
     + __import__("sympy").sqrt(__import__("sympy").Abs(t[2])) + __import__("sympy").exp(-x[0] ** 2)),
    ("theta_2*x[3]", lambda x, y, t: t[1] * x[2]),
])
def test_julia_syntax(expr, want):
    import sympy as sp

    e, xs, ys, ts = _parse(expr)
    assert sp.simplify(e - want(xs, ys, ts)) == 0, (expr, e)


def test_float_literals_are_the_doubles_julia_reads():
    import sympy as sp

    e, xs, _, _ = _parse("0.1x[1] + 0.30000000000000004")
    c = dict(e.as_coefficients_dict())
    assert float(c[xs[0]]) == 0.1 and float(c[sp.Integer(1)]) == 0.30000000000000004


@pytest.mark.parametrize("expr,msg", [
    ("x[4]", "unknown name"), ("z[1]", "unknown name"), ("x[1] +", "unexpected"),
    ("(x[1]", "unbalanced"), ("x[1])", "unexpected"), ("x[1]//2", "two integers"), ("foo(x[1])", "unsupported call"),
    ("x[1] $ 2", "unexpected character"), ("2 x[1]", "unexpected"),
])
def test_errors_are_loud(expr, msg):
    with pytest.raises(symtext.GHSyntaxError, match=msg):
        _parse(expr)


def test_header_errors():
    with pytest.raises(symtext.GHSyntaxError, match="must give p"):
        symtext.loads("n = 1\nm = 0\nG[1] = x[1]\n")
    with pytest.raises(symtext.GHSyntaxError, match="rows missing"):
        symtext.loads("n = 2\nm = 0\np = 0\nG[1] = x[1]\n")
    with pytest.raises(symtext.GHSyntaxError, match="twice"):
        symtext.loads("n = 1\nm = 0\np = 0\nG[1] = x[1]\nG[1] = x[1]\n")
    with pytest.raises(symtext.GHSyntaxError, match="outside"):
        symtext.loads("n = 1\nm = 0\np = 0\nG[1] = x[1]\nG[2] = x[1]\n")
    with pytest.raises(symtext.GHSyntaxError, match="declares"):
        symtext.loads("n = 2\nm = 0\np = 0\nx = [a₁]\nG[1] = a₁\nG[2] = a₁\n")
    # continuation lines and comments
    G, H, xs, ys, ts = symtext.loads("n = 1  # one\nm = 1\np = 1\nG[1] = (x[1] +\n   θ[1])\nH[1] = y[1]\n")
    assert G[0] == xs[0] + ts[0] and H[0] == ys[0]


def _cubic_python():
    """tests/golden/two_player_cubic.gh through the Python front end's tracer."""
    return PrimalDualMCP(
        lambda x, y, θ: np.array([x[0] - θ[0] + x[0] ** 3 + 2 * x[0] * y[0],
                                  x[1] - θ[1] + x[1] ** 3 + 2 * x[1] * y[0]]),
        lambda x, y, θ: np.array([θ[2] - x[0] ** 2 - x[1] ** 2]),
        unconstrained_dimension=2, constrained_dimension=1, parameter_dimension=3)


def _theta_cubic(B, seed=3):
    rng = np.random.default_rng(seed)
    return np.stack([rng.uniform(-2, 2, B), rng.uniform(-2, 2, B), rng.uniform(0.1, 1.0, B)], 1)


def test_hand_written_file_is_the_traced_mcp(oracle_lib):
    """The hand-written Symbolics-style file gives the traced MCP's module key, and the oracle
    (the same generated text under gcc) the same bits."""
    mt = PrimalDualMCP.from_text(os.path.join(GOLD, "two_player_cubic.gh"))
    mp = _cubic_python()
    assert mt.nl is not None and mp.nl is not None
    assert mt.nl.key == mp.nl.key
    th = _theta_cubic(64)
    a = oracle_lib.solve_batch_nl(mt.nl, mt.theta_map(th), tol=1e-6, linear_solver="reduced")
    b = oracle_lib.solve_batch_nl(mp.nl, mp.theta_map(th), tol=1e-6, linear_solver="reduced")
    assert (a["status"] == 0).mean() > 0.9
    assert ((a["y"][:, 0] > a["s"][:, 0]) & (a["status"] == 0)).mean() > 0.2  # the constraint binds on some
    for k in ("x", "y", "s", "status", "newton_iters"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


def test_lane_change_file_is_the_traced_game():
    """The committed lane-change file (T = 2; the game's names x, λ̃, μ̃, θ declared as Symbolics
    prints them) gives the traced game's module key; the other spellings at T = 2 and the declared
    names at T = 10 (KKT 700) round-trip to the same key."""
    from mcp_amd.lane_change import LaneChangeGame

    game = LaneChangeGame(2).mcp
    mt = PrimalDualMCP.from_text(os.path.join(GOLD, "lane_change_t2.gh"))
    assert (mt.unconstrained_dimension, mt.constrained_dimension, mt.parameter_dimension) == (40, 50, 10)
    assert mt.nl.key == game.nl.key
    from mcp_amd.codegen import NLSystem

    args = (game.G_symbolic, game.H_symbolic, game.x_symbolic, game.y_symbolic, game.θ_symbolic)
    for style in ("subscript", "index"):
        assert NLSystem(*symtext.loads(symtext.dumps(*args, style=style))).key == game.nl.key, style
    g10 = LaneChangeGame(10).mcp
    args = (g10.G_symbolic, g10.H_symbolic, g10.x_symbolic, g10.y_symbolic, g10.θ_symbolic)
    assert NLSystem(*symtext.loads(symtext.dumps(*args, style="names"))).key == g10.nl.key


def test_module_does_not_depend_on_names():
    """codegen renames by position: the same G/H in other symbols is the same module."""
    import sympy as sp

    from mcp_amd.codegen import NLSystem

    a, b, t = sp.symbols("a b t", real=True)
    u, v, w = sp.symbols("zz aa mm", real=True)
    k1 = NLSystem([a ** 3 - t + b * a], [a - 2 * b], [a], [b], [t]).key
    k2 = NLSystem([u ** 3 - w + v * u], [u - 2 * v], [u], [v], [w]).key
    assert k1 == k2


def test_cli_check_and_build():
    env = dict(os.environ, PYTHONPATH=ROOT)
    path = os.path.join(GOLD, "lane_change_t2.gh")
    r = subprocess.run([sys.executable, "-m", "mcp_amd.symtext", "check", path], capture_output=True, text=True,
                       env=env, cwd=ROOT, timeout=300)
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout) == {"n": 40, "m": 50, "p": 10}
    # build reuses the prebuilt C4 code object (__graft_entry__.build) — the path mcpx_module_load takes
    r = subprocess.run([sys.executable, "-m", "mcp_amd.symtext", "build", path], capture_output=True, text=True,
                       env=env, cwd=ROOT, timeout=600)
    assert r.returncode == 0, r.stderr
    info = json.loads(r.stdout)
    from mcp_amd.lane_change import LaneChangeGame

    assert info["module"] == LaneChangeGame(2).mcp.nl.module_path() and os.path.exists(info["module"])
    r = subprocess.run([sys.executable, "-m", "mcp_amd.symtext", "build"], capture_output=True, text=True,
                       env=env, cwd=ROOT, timeout=300)
    assert r.returncode == 2


# ---------------------------------------------------------------- GPU


@pytest.mark.gpu
def test_gpu_module_from_text_matches_oracle_and_traced_game(gpu, oracle_lib):
    from mcp_amd.api import InteriorPoint, solve
    from mcp_amd.lane_change import LaneChangeGame
    from tests.test_gpu_parity import assert_parity

    lane = LaneChangeGame(2)
    mt = PrimalDualMCP.from_text(os.path.join(GOLD, "lane_change_t2.gh"))
    th = lane.generate_random_parameter(np.random.default_rng(11), 256)
    x0 = lane.initial_guess(th)
    from mcp_amd.batch import solve_batch

    got = solve_batch(2, 40, 50, mt.theta_map(th), x0=x0, tol=1e-6, linear_solver="schur", trace_len=256,
                      module=mt.module())
    ref = oracle_lib.solve_batch_nl(mt.nl, mt.theta_map(th), x0=x0, tol=1e-6, linear_solver="schur",
                                    trace_len=256, nthreads=8)
    assert_parity(got, ref)
    traced = solve(InteriorPoint(), lane.mcp, th, x0=x0.copy(), tol=1e-6)
    np.testing.assert_array_equal(traced.x, got["x"])
    np.testing.assert_array_equal(np.asarray(traced.newton_iters), got["newton_iters"])
    # and the hand-written cubic game through its text module
    mc = PrimalDualMCP.from_text(os.path.join(GOLD, "two_player_cubic.gh"))
    thc = _theta_cubic(128)
    for ls in ("reduced", "schur"):
        sol = solve(InteriorPoint(), mc, thc, tol=1e-6, linear_solve_algorithm=ls)
        refc = oracle_lib.solve_batch_nl(mc.nl, mc.theta_map(thc), tol=1e-6, linear_solver=ls)
        np.testing.assert_array_equal(sol.x, refc["x"])
        np.testing.assert_array_equal(np.asarray(sol.outer_iters), refc["outer_iters"])
