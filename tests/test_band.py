"""The band SCHUR elimination of generated modules (mcp_amd/band.py, csrc/ipm_nl_band.hpp,
oracle/ipm_oracle.c lu_band_solve).

* CPU: the ordering's window really holds the elimination — every row with a structural
  nonzero in column k is a window row at step k, and the row-merge fill of partial pivoting
  (George & Ng: every candidate row may take the union of the candidates' patterns) never
  leaves the WC window columns — so lu_band_solve is the dense LU with partial pivoting of
  S' = S[σ][:, π] on finite values; and at scale the band oracle agrees with the literal
  full-system LU (src/solver.jl:81-83) on every solved C4 game, with the divergences on the
  failing games recorded exactly.
* GPU: mcpx_nl_solve_band bit-exact against the oracle's lu_band_solve mode on the C4 batch
  with edge games, at the reference benchmark's horizon T = 10, with warm starts, and over
  back-to-back host-buffer calls on both HIP runtimes (torch's and /opt/rocm's).
"""

from __future__ import annotations

import os

import numpy as np
import pytest

from mcp_amd import _abi, band

TRACE = 1024
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _z(r):
    return np.concatenate([r["x"], r["y"], r["s"]], 1)


def _row_merge_fits(S, rperm, cperm, ns, wc):
    """Symbolic band LU with the worst-case row merge: True when every step's candidates are
    window rows and every merged pattern stays inside [k, k + wc − 1]."""
    Sp = S[np.ix_(rperm, cperm)]
    n = Sp.shape[0]
    pat = [set(np.nonzero(Sp[r])[0]) for r in range(n)]
    rem = set(range(n))
    for k in range(n):
        cand = [r for r in rem if k in pat[r]]
        if any(r > k + ns - 1 for r in cand):
            return False
        union = set().union(*[pat[r] for r in cand]) - {c for c in range(k + 1)}
        if any(c > k + wc - 1 for c in union):
            return False
        p = min(cand) if cand else min(r for r in rem if r <= k + ns - 1)
        rem.discard(p)
        for r in cand:
            if r != p:
                pat[r] = (pat[r] - {k}) | union
    return True


@pytest.mark.parametrize("T", [2, 10])
def test_window_holds_the_elimination(T):
    from mcp_amd.lane_change import LaneChangeGame

    nl = LaneChangeGame(T).mcp.nl
    bp = nl.band
    assert bp is not None and nl.band_can
    assert (bp.ns, bp.wc) == {2: (7, 20), 10: (13, 32)}[T]
    S = band.s_pattern(nl)
    assert sorted(bp.rperm.tolist()) == list(range(nl.n)) and sorted(bp.cperm.tolist()) == list(range(nl.n))
    assert _row_merge_fits(S, bp.rperm, bp.cperm, bp.ns, bp.wc)
    # a window one row or four columns smaller does not hold it
    assert not _row_merge_fits(S, bp.rperm, bp.cperm, bp.ns - 1, bp.wc) or \
        not _row_merge_fits(S, bp.rperm, bp.cperm, bp.ns, bp.wc - 4)


def test_window_on_random_patterns():
    rng = np.random.default_rng(0)
    for n in (5, 17, 40):
        S = rng.random((n, n)) < 3.0 / n
        S |= S.T
        np.fill_diagonal(S, True)
        cp = band.cm_order(S)
        rp = band.row_order(S, cp)
        ns, wc = band.window(S, cp, rp)
        assert _row_merge_fits(S, rp, cp, ns, -(-wc // 4) * 4)


def _c4(T, B):
    from mcp_amd.lane_change import LaneChangeGame
    from mcp_amd.qp_benchmark import chunked_slice

    game = LaneChangeGame(T)
    th = chunked_slice(lambda rng, k: game.generate_random_parameter(rng, k), 1, 0, B)
    return game, np.ascontiguousarray(game.mcp.theta_map(th))


@pytest.mark.slow
@pytest.mark.parametrize("T,B,ref_mode,expect", [(2, 1024, "dense", (974, 14, 11, 24)),
                                                 (10, 64, "workgroup", (62, 2, 2, 2))])
def test_band_oracle_equals_full_lu_on_solved_games(oracle_lib, T, B, ref_mode, expect):
    """The band elimination against the literal LU: the full (n + 2m)-dim ∇F + tol·I at T = 2
    (KKT 140), the workgroup kernels' LU of the 200-dim S at T = 10 (the full 700-dim LU takes
    minutes there).  Solved games: every discrete output identical, iterates ≤ 1e-10 relative.
    Failing games (all 931 Newton steps) fail under both; rounding moves some trajectories
    (Newton counts, active sets, α traces), counted exactly."""
    game, tp = _c4(T, B)
    nl = game.mcp.nl
    run = lambda **kw: oracle_lib.solve_batch_nl(nl, tp, tol=1e-6, nthreads=8, trace_len=TRACE, **kw)
    b = run(linear_solver="schur", kernel="band")
    d = run(linear_solver="dense") if ref_mode == "dense" else run(linear_solver="schur", kernel="workgroup")
    ok = d["status"] == 0
    assert np.array_equal(b["status"], d["status"]) and np.array_equal(b["outer_iters"], d["outer_iters"])
    diff = {k: (b[k] != d[k]).reshape(B, -1).any(1) for k in ("newton_iters", "active_mask", "alpha_trace")}
    for k, v in diff.items():
        assert not v[ok].any(), k
    assert (int(ok.sum()), *(int(v.sum()) for v in diff.values())) == expect
    rel = np.abs(_z(b)[ok] - _z(d)[ok]).max(1) / np.maximum(1.0, np.abs(_z(d)[ok]).max(1))
    assert rel.max() <= 1e-10


@pytest.mark.slow
def test_t10_band_and_workgroup_equal_the_full_700_dim_lu(oracle_lib):
    """C4 at the reference benchmark's horizon (T = 10, benchmark/trajectory_game_benchmark.jl:38):
    the band elimination (what AUTO runs) and the workgroup LU of the 200-dim S against the literal
    LU of the full (n + 2m) = 700-dim ∇F + tol·I (src/solver.jl:81-83), on the first 48 games of
    the bench's θ stream.  The dense run takes the games both other modes solve (47; no 931-step
    dense solves).  On them every discrete output (status, outer and Newton counts, α traces,
    active sets) is identical, and the iterates agree to ≤ 1e-10 relative (observed 4.3e-13 band,
    1.2e-13 workgroup)."""
    game, tp = _c4(10, 48)
    nl = game.mcp.nl
    run = lambda th, **kw: oracle_lib.solve_batch_nl(nl, th, tol=1e-6, nthreads=8, trace_len=TRACE, **kw)
    r = {"band": run(tp, linear_solver="schur", kernel="band"),
         "wg": run(tp, linear_solver="schur", kernel="workgroup")}
    both = (r["band"]["status"] == 0) & (r["wg"]["status"] == 0)
    idx = np.nonzero(both)[0]
    assert len(idx) == 47
    d = run(np.ascontiguousarray(tp[idx]), linear_solver="dense")
    assert (d["status"] == 0).all()
    for mode, a in r.items():
        for k in ("status", "outer_iters", "newton_iters", "active_mask", "alpha_trace"):
            np.testing.assert_array_equal(a[k][idx], d[k], err_msg=f"{mode} {k}")
        rel = np.abs(_z(a)[idx] - _z(d)).max(1) / np.maximum(1.0, np.abs(_z(d)).max(1))
        assert rel.max() <= 1e-10, (mode, rel.max())


def test_band_mode_follows_the_kernel_choice(oracle_lib):
    """AUTO takes the band kernel at T = 10 (no one-wave SCHUR kernel: n = 200) and the one-wave
    Gauss-Jordan at T = 2 (the module does not prefer the band kernel there); the oracle picks its
    elimination by the same rule as the C ABI (mcpx_api.cpp prepare / ipm_oracle.c solve_one)."""
    from mcp_amd.lane_change import LaneChangeGame

    for T, auto in ((2, "wave"), (10, "band")):
        game = LaneChangeGame(T)
        nl = game.mcp.nl
        assert nl.band_can and nl.band_auto == (T == 10)
        th = np.ascontiguousarray(game.mcp.theta_map(game.generate_random_parameter(np.random.default_rng(3), 2)))
        a = oracle_lib.solve_batch_nl(nl, th, linear_solver="schur", trace_len=TRACE)
        b = oracle_lib.solve_batch_nl(nl, th, linear_solver="schur", trace_len=TRACE, kernel=auto)
        for k in ("x", "y", "s", "newton_iters", "alpha_trace"):
            assert np.array_equal(a[k], b[k]), (T, k)


# ---------------------------------------------------------------- GPU


@pytest.mark.gpu
def test_gpu_band_c4_batch_and_edge_inputs(gpu, oracle_lib):
    """The C4 batch (1,024 games of the bench's θ stream, ~50 of them 931 Newton steps) plus
    NaN / Inf / huge / zeroed parameters through mcpx_nl_solve_band, bit-exact against the
    oracle's lu_band_solve."""
    from mcp_amd.batch import solve_batch

    game, tp = _c4(2, 1024)
    mcp = game.mcp
    edge = np.repeat(tp[:1], 8, 0)
    edge[0, 0] = np.nan
    edge[1, 3] = np.inf
    edge[2, :] = 0.0
    edge[3, 1] = 1e200
    edge[4, 5] = -1e-300
    edge[5, :4] = edge[5, 5:9]
    edge[6, 2] = -np.inf
    edge[7, 9] = 1e6
    tp = np.ascontiguousarray(np.concatenate([tp, edge]))
    got = solve_batch(_abi.FAMILY_NONLINEAR, mcp.nl.n, mcp.nl.m, tp, linear_solver="schur", trace_len=TRACE,
                      module=mcp.module(), kernel="band")
    ref = oracle_lib.solve_batch_nl(mcp.nl, tp, linear_solver="schur", trace_len=TRACE, nthreads=8, kernel="band")
    from tests.test_gpu_parity import assert_parity

    assert_parity(got, ref)
    assert (ref["newton_iters"][:1024] == 931).sum() >= 30


@pytest.mark.gpu
@pytest.mark.parametrize("B,warm", [(64, False), (16, True)])
def test_gpu_band_t10(gpu, oracle_lib, B, warm):
    """The reference benchmark's horizon (T = 10: S is 200 × 200, KKT 700): AUTO runs the band
    kernel; cold starts (x₀ = 0) on the bench's θ and warm starts from the zero-input rollout."""
    from mcp_amd.batch import solve_batch

    game, tp = _c4(10, B)
    mcp = game.mcp
    x0 = game.initial_guess(game.generate_random_parameter(np.random.default_rng(5), B)) if warm else None
    got = solve_batch(_abi.FAMILY_NONLINEAR, mcp.nl.n, mcp.nl.m, tp, x0=x0, linear_solver="schur", trace_len=TRACE,
                      module=mcp.module())
    ref = oracle_lib.solve_batch_nl(mcp.nl, tp, x0=x0, linear_solver="schur", trace_len=TRACE, nthreads=8)
    from tests.test_gpu_parity import assert_parity

    assert_parity(got, ref)
    if not warm:  # the bench's θ from x₀ = 0 (the zero-input warm start solves fewer: parity only)
        assert (ref["status"] == 0).mean() > 0.8


@pytest.mark.gpu
@pytest.mark.parametrize("T", [12, 15])
def test_gpu_band_past_the_benchmark_horizon(gpu, oracle_lib, T):
    """Past T = 10 the band kernel's LDS grows (48 KB at T = 12, 60 KB at T = 15): it still runs,
    with fewer games per CU (the launch sizes its grid by occupancy), instead of AUTO falling back
    to the workgroup LU (the research application runs horizon 30,
    examples/train_and_test_utils.jl:585).  AUTO takes it, bit-exact against lu_band_solve."""
    from mcp_amd.batch import solve_batch
    from tests.test_gpu_parity import assert_parity

    game, tp = _c4(T, 32)
    mcp = game.mcp
    assert mcp.nl.band_can and mcp.nl.band_auto
    got = solve_batch(_abi.FAMILY_NONLINEAR, mcp.nl.n, mcp.nl.m, tp, linear_solver="schur", trace_len=TRACE,
                      module=mcp.module())
    ref = oracle_lib.solve_batch_nl(mcp.nl, tp, linear_solver="schur", trace_len=TRACE, nthreads=8)
    assert_parity(got, ref)
    assert (ref["status"] == 0).mean() > 0.8


@pytest.mark.gpu
@pytest.mark.parametrize("runtime", ["torch", "system"])
def test_gpu_host_calls_repeat_bit_exact(gpu, oracle_lib, runtime):
    """Back-to-back host-buffer calls in one process (T = 10, 1,024 games): every call bit-exact
    against the oracle.  "torch": this process (torch's bundled HIP runtime), two θ batches in
    turn.  "system": a child process that never imports torch, so libmcpx.so runs on
    /opt/rocm's HIP runtime — where the stream-ordered pool the library used to allocate from
    (hipMallocFromPoolAsync, VM heap) returned wrong games from the fourth call on, every other
    call (tools/band_stress.py); the library's block cache replaced it."""
    if runtime == "system":
        import json
        import subprocess
        import sys

        env = {k: v for k, v in os.environ.items() if k != "PYTHONPATH"}
        p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tools", "band_stress.py"), "10", "1024", "band",
                            "6", "reuse"], capture_output=True, text=True, timeout=150, env=env, cwd=ROOT)
        assert p.returncode == 0, p.stderr[-2000:]
        calls = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
        assert len(calls) == 6 and all(c["vs_oracle"] == 0 for c in calls), calls
        return
    from mcp_amd.batch import solve_batch
    from tests.test_gpu_parity import assert_parity

    game, tp = _c4(10, 2048)
    mcp = game.mcp
    batches = [np.ascontiguousarray(tp[:1024]), np.ascontiguousarray(tp[1024:])]
    refs = [oracle_lib.solve_batch_nl(mcp.nl, t, linear_solver="schur", trace_len=TRACE, nthreads=8) for t in batches]
    for call in range(6):
        got = solve_batch(_abi.FAMILY_NONLINEAR, mcp.nl.n, mcp.nl.m, batches[call % 2], linear_solver="schur",
                          trace_len=TRACE, module=mcp.module())
        assert_parity(got, refs[call % 2])


@pytest.mark.gpu
def test_gpu_host_calls_repeat_poisoned(gpu):
    """the repeated host calls of the system-runtime case once more with
    MCPX_POISON=1 — every library block handed out NaN-filled up to its requested size, a canary
    after it checked at release.  A kernel that read workspace before writing it would change its
    games, one that wrote past a block's end would trip the canary: all 6 calls stay bit-exact
    against the oracle with every canary intact, so the wrong games of the HIP 7.2 pool were not
    a kernel-side read or write."""
    import json
    import subprocess
    import sys

    env = {k: v for k, v in os.environ.items() if k != "PYTHONPATH"}
    env["MCPX_POISON"] = "1"
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tools", "band_stress.py"), "10", "1024", "band",
                        "6", "reuse"], capture_output=True, text=True, timeout=200, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    assert "MCPX_POISON canary" not in p.stderr, p.stderr[-2000:]
    calls = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(calls) == 6 and all(c["vs_oracle"] == 0 and c["canary"] == 0 for c in calls), calls


@pytest.mark.gpu
def test_gpu_band_kernel_selector_errors(gpu):
    from mcp_amd._lib import MCPXError
    from mcp_amd.batch import solve_batch
    from mcp_amd.qp_benchmark import generate_random_parameter
    from tests.test_nonlinear import _cubic_theta, cubic_mcp

    th = generate_random_parameter(np.random.default_rng(1), 4, 2, 0.0, batch=2)
    with pytest.raises(MCPXError):  # the band kernel is a generated module's
        solve_batch(0, 4, 2, th, linear_solver="schur", kernel="band")
    with pytest.raises(MCPXError):  # ∂H/∂y ≠ 0: no SCHUR elimination, no band kernel
        solve_batch(_abi.FAMILY_NONLINEAR, 1, 1, _cubic_theta(2), linear_solver="schur", module=cubic_mcp().module(),
                    kernel="band")
