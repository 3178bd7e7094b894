"""The batched receding-horizon driver (mcp_amd/receding_horizon.py) against a
literal one-simulation-at-a-time restatement of WarmStartRecedingHorizonStrategy /
solve_trajectory_game! / rollout (examples/utils.jl:195-308), both on the oracle
(CPU), and the GPU-solved driver against the oracle-solved one (bit-exact)."""

from __future__ import annotations

import numpy as np
import pytest

from mcp_amd.lane_change import NUM_PLAYERS, STATE_DIM, LaneChangeGame
from mcp_amd.receding_horizon import WarmStartRecedingHorizon, product_dynamics, rollout

B, STEPS, TURN = 6, 7, 2


def _initial(game, rng):
    th = game.generate_random_parameter(rng, B)  # positions on the road, zero velocity
    states = np.concatenate([th[:, :STATE_DIM], th[:, STATE_DIM + 1:2 * STATE_DIM + 1]], 1)
    states[:, 3] = 1.0  # forward speed 1 (lane_change.jl:58 starts at 1 m/s)
    states[:, 7] = 1.0
    prefs = np.stack([th[:, STATE_DIM], th[:, 2 * STATE_DIM + 1]], 1)
    return states, prefs


def _oracle_solver(game, oracle_lib):
    mcp = game.mcp

    def solve(theta_mcp, x0, y0):
        return oracle_lib.solve_batch_nl(mcp.nl, theta_mcp, x0=x0, y0=y0, linear_solver=mcp.nl.default_solver(),
                                         nthreads=8)

    return solve


def _serial_reference(game, oracle_lib, state, prefs):
    """utils.jl:195-308 + TrajectoryGamesBase.rollout, one simulation, literally."""
    mcp = game.mcp
    last, plan, t_last = None, None, 0
    xs, us, statuses = [state], [], []
    for t in range(1, STEPS):
        tap = t - t_last + 1
        if plan is None or not (1 <= tap <= TURN):
            theta = game.pack_parameters(state.reshape(NUM_PLAYERS, STATE_DIM), prefs)[None]
            if last is not None:  # warm start from the last :solved solution
                sol = oracle_lib.solve_batch_nl(mcp.nl, theta, x0=last["x"], y0=last["y"],
                                                linear_solver=mcp.nl.default_solver())
            else:  # zero-input rollout, zero multipliers; y₀ default
                sol = oracle_lib.solve_batch_nl(mcp.nl, theta, x0=game.initial_guess(theta),
                                                linear_solver=mcp.nl.default_solver())
            statuses.append(int(sol["status"][0]))
            if sol["status"][0] == 0:
                last = sol
            trajs = game.trajectories(sol["x"][0])
            plan = np.concatenate([u for _, u in trajs], axis=-1)
            t_last, tap = t, 1
        u = plan[tap - 1]
        us.append(u)
        state = product_dynamics(state[None], u[None])[0]
        xs.append(state)
    return np.stack(xs), np.stack(us), statuses


@pytest.mark.slow
def test_batched_driver_equals_serial_restatement(oracle_lib):
    game = LaneChangeGame(2)
    states, prefs = _initial(game, np.random.default_rng(3))
    strat = WarmStartRecedingHorizon(game, TURN, prefs, solve=_oracle_solver(game, oracle_lib))
    xs, us = rollout(strat, states, STEPS)
    assert xs.shape == (B, STEPS, 8) and us.shape == (B, STEPS - 1, 4)
    assert len(strat.statuses) == 3  # re-solves at t = 1, 3, 5
    for b in range(B):
        rx, ru, rs = _serial_reference(game, oracle_lib, states[b], prefs[b])
        np.testing.assert_array_equal(xs[b], rx)
        np.testing.assert_array_equal(us[b], ru)
        assert [int(s[b]) for s in strat.statuses] == rs
    assert any(np.all(s == 0) for s in strat.statuses)


@pytest.mark.gpu
def test_gpu_driver_equals_oracle_driver(gpu, oracle_lib):
    game = LaneChangeGame(2)
    states, prefs = _initial(game, np.random.default_rng(4))
    g = WarmStartRecedingHorizon(game, TURN, prefs)  # default: the GPU through the C ABI
    o = WarmStartRecedingHorizon(game, TURN, prefs, solve=_oracle_solver(game, oracle_lib))
    gx, gu = rollout(g, states, STEPS)
    ox, ou = rollout(o, states, STEPS)
    np.testing.assert_array_equal(gx, ox)
    np.testing.assert_array_equal(gu, ou)
    for a, b in zip(g.statuses, o.statuses):
        np.testing.assert_array_equal(a, b)
