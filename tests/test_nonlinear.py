"""The nonlinear family (MCPX_FAMILY_NONLINEAR): general G/H turned into generated
code (mcp_amd/codegen.py) that both the gfx950 module and the C oracle compile.

CPU: the BASELINE C4 lane-change game (examples/lane_change.jl) traces to the
expected sizes, the oracle solves the reference example and satisfies its KKT
conditions, the nonlinear oracle path agrees with the pinned affine-family
oracle on the reference's clamp game (test/runtests.jl:88-107) forced through
generated code, and the generated modules compile for gfx950.
GPU: the generated kernels against the oracle, bit for bit (every solver a
module carries), through the C ABI and the torch device path.
"""

from __future__ import annotations

import numpy as np
import pytest

from mcp_amd import _abi
from mcp_amd.api import InteriorPoint, PrimalDualMCP, solve
from mcp_amd.lane_change import LaneChangeGame
from tests.test_api import clamp_game
from tests.test_gpu_parity import assert_parity

TRACE = 256


@pytest.fixture(scope="module")
def lane():
    return LaneChangeGame(2)


def cubic_mcp():
    """x³ − θ₀ − y = 0, y ⟂ x − θ₁ y ≥ 0 (∂H/∂y ≠ 0: REDUCED / DENSE only)."""
    return PrimalDualMCP(lambda x, y, θ: x ** 3 - θ[0] - y, lambda x, y, θ: x - θ[1] * y,
                         unconstrained_dimension=1, constrained_dimension=1, parameter_dimension=2)


def trig_mcp():
    """A smooth transcendental G (sin/exp): parity is the 1e-8 bar, not bitwise (codegen.py header)."""
    import sympy as sp

    return PrimalDualMCP(lambda x, y, θ: np.array([x[0] + 0.3 * sp.sin(x[1]) - θ[0] - y[0],
                                                   x[1] + 0.1 * sp.exp(-x[0] * x[0]) - θ[1]]),
                         lambda x, y, θ: np.array([x[0] - 0.5]),
                         unconstrained_dimension=2, constrained_dimension=1, parameter_dimension=2)


def _cubic_theta(B, seed=0):
    rng = np.random.default_rng(seed)
    return np.stack([rng.uniform(-2, 2, B), rng.uniform(0.1, 1.0, B)], 1)


# ---------------------------------------------------------------- CPU


def test_lane_change_traces_to_nonlinear_family(lane):
    mcp = lane.mcp
    assert mcp.family == _abi.FAMILY_NONLINEAR
    nl = mcp.nl
    # n = 12T primals + 8T λ̃, m = 25T μ̃ (lane_change.py header), θ = 2 × (state + preference)
    assert (nl.n, nl.m, nl.p) == (40, 50, 10)
    assert not nl.has_s and nl.default_solver() == "schur"
    # collision rows are the only z-dependent entries of R: 2 players × 2 coords × T
    assert any(idx >= nl.OFF_R and idx < nl.OFF_G for idx, _ in nl.var_entries)


def test_oracle_solves_lane_change_example(lane, oracle_lib):
    """run_lane_change_example's θ (lane_change.jl:57-73): solved, and the solution
    satisfies the complementarity conditions checked against the host F (src/mcp.jl:72-80)."""
    mcp, nl = lane.mcp, lane.mcp.nl
    th = lane.example_parameters()
    r = oracle_lib.solve_batch_nl(nl, mcp.theta_map(th), x0=lane.initial_guess(th), linear_solver="schur")
    assert r["status"][0] == 0 and r["kkt_error"][0] <= 1e-4
    x, y, s = r["x"][0], r["y"][0], r["s"][0]
    F = mcp.F(x, y, s, θ=th, ϵ=0.0)
    n, m = mcp.nl.n, mcp.nl.m
    assert np.max(np.abs(F[:n + m])) <= 1e-3  # G = 0, H = s
    assert np.max(F[n + m:]) <= 5e-3  # s ⊙ y → 0 (test/runtests.jl:30-38 bar)
    assert np.all(y >= 0) and np.all(s >= 0)
    (p1, _), (p2, _) = lane.trajectories(x)
    assert np.all(np.sum((p1[:, :2] - p2[:, :2]) ** 2, 1) - 4 >= -1e-3)  # collision avoidance
    np.testing.assert_allclose(p1[0], th[:4], atol=1e-6)  # initial-state equality rows


def test_nonlinear_oracle_matches_affine_oracle(oracle_lib):
    """The clamp game through generated code vs the affine family (pinned by the golden
    vectors): same iteration path, iterates within rounding."""
    aff = clamp_game().mcp
    from mcp_amd.api import ParametricGame, OptimizationProblem, mortar  # noqa: F401

    g = clamp_game()
    nlm = PrimalDualMCP.from_symbolic(aff.G_symbolic, aff.H_symbolic, aff.x_symbolic, aff.y_symbolic,
                                      aff.θ_symbolic, backend_options={"family": "nonlinear"})
    assert nlm.family == _abi.FAMILY_NONLINEAR and g.mcp.family == _abi.FAMILY_AFFINE
    rng = np.random.default_rng(3)
    th = rng.uniform(-1, 1, (16, 4))
    for ls in ("reduced", "dense"):
        ra = oracle_lib.solve_batch(_abi.FAMILY_AFFINE, 4, 8, aff.theta_map(th), linear_solver=ls)
        rn = oracle_lib.solve_batch_nl(nlm.nl, nlm.theta_map(th), linear_solver=ls)
        np.testing.assert_array_equal(ra["status"], rn["status"])
        np.testing.assert_array_equal(ra["outer_iters"], rn["outer_iters"])
        for k in ("x", "y", "s"):
            np.testing.assert_allclose(rn[k], ra[k], rtol=1e-8, atol=1e-10)


def test_oracle_nl_rejects_schur_with_dh_dy(oracle_lib):
    nl = cubic_mcp().nl
    assert nl.has_s and not nl.solvers()["schur"]
    with pytest.raises(ValueError):
        oracle_lib.solve_batch_nl(nl, _cubic_theta(2), linear_solver="schur")


def test_generated_modules_compile(lane):
    """hipcc --genco of the generated text + csrc/ipm_nl_kernel.hpp (cached by content hash)."""
    import os

    for mcp in (lane.mcp, cubic_mcp(), trig_mcp()):
        path = mcp.nl.build_module()
        assert os.path.getsize(path) > 0
        blob = open(path, "rb").read()
        for s, ok in mcp.nl.solvers().items():  # symbol names are NUL-terminated in the ELF string table
            assert (f"mcpx_nl_solve_{s}\0".encode() in blob) == ok, s
        for s, ok in mcp.nl.wg_solvers().items():
            assert (f"mcpx_nl_solve_{s}_wg\0".encode() in blob) == ok, s


def test_lane_parallel_eval_matches_generated_c(lane, oracle_lib):
    """The chain rewrite of mcpx_nl_eval (mcp_amd/nl_vec.py) that the one-wave SCHUR kernel
    evaluates lane-parallel is bitwise the generated C text the oracle compiles: random z over
    wide magnitudes with ±0, Inf and NaN entries, every output entry of blk compared by bits
    (NaN = NaN whatever its payload, as in every parity test).
    Transcendental modules keep the straight-line eval (no program)."""
    import ctypes as C

    from oracle import coracle

    assert trig_mcp().nl.vec is None
    rng = np.random.default_rng(7)
    for mcp, theta_of in ((lane.mcp, lambda k: lane.mcp.theta_map(lane.generate_random_parameter(rng, k))),
                          (cubic_mcp(), _cubic_theta)):
        nl = mcp.nl
        prog = nl.vec
        assert prog is not None and prog.levels()
        G = coracle.nl_lib(nl)
        ev = G.oracle_nl_eval
        ev.restype, ev.argtypes = None, [C.c_void_p] * 3
        ini = G.oracle_nl_init
        ini.restype, ini.argtypes = None, [C.c_void_p] * 2
        ths = np.atleast_2d(theta_of(300))
        for trial in range(300):
            th = np.ascontiguousarray(ths[trial % len(ths)], dtype=np.float64)
            z = rng.standard_normal(nl.n + 2 * nl.m) * 10.0 ** rng.integers(-6, 7)
            sel = rng.integers(0, len(z), 3)
            z[sel] = [0.0, -0.0, [np.inf, -np.inf, np.nan][trial % 3]] if trial % 5 == 0 else z[sel]
            ref = np.zeros(nl.size + 1)
            ini(th.ctypes.data, ref.ctypes.data)
            got = ref[:nl.size].copy()
            ev(th.ctypes.data, z.ctypes.data, ref.ctypes.data)
            prog.emulate(th, z, got)
            r = ref[:nl.size]
            same_bits = got.view(np.uint64) == r.view(np.uint64)
            assert (same_bits | (np.isnan(got) & np.isnan(r))).all(), trial  # NaN payloads aside


# ---------------------------------------------------------------- GPU


@pytest.mark.gpu
@pytest.mark.parametrize("B", [1, 257])
@pytest.mark.parametrize("kernel", ["multiwave", "auto"])
def test_gpu_lane_change_bit_exact(gpu, lane, oracle_lib, B, kernel):
    """multiwave = the 4-wave SCHUR kernel (mcpx_nl_solve_schur_mw), auto = the one-wave kernel."""
    from mcp_amd.batch import solve_batch

    mcp = lane.mcp
    assert mcp.module().has_schur_mw
    th = lane.example_parameters()[None] if B == 1 else lane.generate_random_parameter(np.random.default_rng(7), B)
    tp, x0 = mcp.theta_map(th), lane.initial_guess(th)
    got = solve_batch(_abi.FAMILY_NONLINEAR, 40, 50, tp, x0=x0, linear_solver="schur", trace_len=TRACE,
                      module=mcp.module(), kernel=kernel)
    ref = oracle_lib.solve_batch_nl(mcp.nl, tp, x0=x0, linear_solver="schur", trace_len=TRACE, nthreads=8)
    assert_parity(got, ref)
    if B == 1:
        assert got["status"][0] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("ls", ["reduced", "dense"])
def test_gpu_cubic_bit_exact(gpu, oracle_lib, ls):
    from mcp_amd.batch import solve_batch

    mcp = cubic_mcp()
    th = _cubic_theta(130)
    got = solve_batch(_abi.FAMILY_NONLINEAR, 1, 1, th, linear_solver=ls, trace_len=TRACE, module=mcp.module())
    ref = oracle_lib.solve_batch_nl(mcp.nl, th, linear_solver=ls, trace_len=TRACE)
    assert_parity(got, ref)
    # x³ has a zero Jacobian at the x₀ = 0 start: the reference algorithm fails on part of
    # this family (status parity above is the bar); most instances still solve
    assert (got["status"] == 0).mean() > 0.5


@pytest.mark.gpu
def test_gpu_transcendental_within_tolerance(gpu, oracle_lib):
    """sin/exp: device ocml vs glibc may differ by an ulp → the north_star's 1e-8 bar."""
    from mcp_amd.batch import solve_batch

    mcp = trig_mcp()
    th = np.random.default_rng(5).uniform(-1, 1, (64, 2))
    for ls in ("schur", "reduced", "dense"):
        got = solve_batch(_abi.FAMILY_NONLINEAR, 2, 1, th, linear_solver=ls, module=mcp.module())
        ref = oracle_lib.solve_batch_nl(mcp.nl, th, linear_solver=ls)
        np.testing.assert_array_equal(got["status"], ref["status"])
        for k in ("x", "y", "s"):
            np.testing.assert_allclose(got[k], ref[k], rtol=1e-8, atol=1e-10)


@pytest.mark.gpu
def test_gpu_module_rejects_missing_solver(gpu):
    from mcp_amd._lib import MCPXError
    from mcp_amd.batch import solve_batch

    mcp = cubic_mcp()
    with pytest.raises(MCPXError):
        solve_batch(_abi.FAMILY_NONLINEAR, 1, 1, _cubic_theta(4), linear_solver="schur", module=mcp.module())
    with pytest.raises(MCPXError):  # no multi-wave kernel for n < 4
        solve_batch(_abi.FAMILY_NONLINEAR, 1, 1, _cubic_theta(4), linear_solver="reduced", module=mcp.module(),
                    kernel="multiwave")


@pytest.mark.gpu
def test_gpu_lane_change_api_device_path(gpu, lane, oracle_lib):
    """solve(game, θ) on a torch HIP tensor: the generated module on the current stream."""
    import torch

    mcp = lane.mcp
    th = lane.generate_random_parameter(np.random.default_rng(11), 64)
    x0 = lane.initial_guess(th)
    sol = solve(InteriorPoint(), mcp, torch.from_numpy(th).cuda(), x0=torch.from_numpy(x0).cuda())
    torch.cuda.synchronize()
    ref = oracle_lib.solve_batch_nl(mcp.nl, mcp.theta_map(th), x0=x0, linear_solver="schur", nthreads=8)
    np.testing.assert_array_equal(sol.x.cpu().numpy(), ref["x"])
    np.testing.assert_array_equal(sol.status.cpu().numpy(), ref["status"])


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["multiwave", "wave"])
def test_gpu_lane_change_c4_batch_and_edge_inputs(gpu, lane, oracle_lib, kernel):
    """The BASELINE C4 batch itself (1,024 games of the bench's θ stream, 45-50 of which run
    all 931 Newton steps) plus games with NaN / Inf / huge / zeroed parameters, bit-exact vs
    the oracle.  Exercises the guessed-pivot LU of mcpx_nl_solve_schur on every path: guesses
    that hold, guesses that miss (re-factored with the search), and NaN or zero guessed
    pivots (csrc/ipm_kernel_impl.hpp, lu_solve_rows_core)."""
    from mcp_amd.batch import solve_batch
    from mcp_amd.qp_benchmark import chunked_slice

    mcp = lane.mcp
    th = chunked_slice(lambda rng, k: lane.generate_random_parameter(rng, k), 1, 0, 1024)
    edge = np.repeat(th[:1], 8, 0)
    edge[0, 0] = np.nan
    edge[1, 3] = np.inf
    edge[2, :] = 0.0
    edge[3, 1] = 1e200
    edge[4, 5] = -1e-300
    edge[5, :4] = edge[5, 5:9]  # both players start in the same state
    edge[6, 2] = -np.inf
    edge[7, 9] = 1e6
    th = np.concatenate([th, edge])
    tp = np.ascontiguousarray(mcp.theta_map(th))
    got = solve_batch(_abi.FAMILY_NONLINEAR, 40, 50, tp, linear_solver="schur", trace_len=TRACE, module=mcp.module(),
                      kernel=kernel)
    ref = oracle_lib.solve_batch_nl(mcp.nl, tp, linear_solver="schur", trace_len=TRACE, nthreads=8)
    assert_parity(got, ref)
    assert (ref["newton_iters"][:1024] == 931).sum() >= 30  # the tail really ran
