"""Batched receding-horizon simulation with warm starts — the host-side caller of
the solver in the reference's examples:

  * WarmStartRecedingHorizonStrategy (examples/utils.jl:280-308): a plan is
    re-solved every `turn_length` steps and followed in between;
  * solve_trajectory_game! (examples/utils.jl:195-278): the re-solve is warm
    started from the last *successful* solution (x₀ = its x, y₀ = its y); without
    one, x₀ is the zero-input rollout from the current state followed by zero
    multipliers (utils.jl:218-227); the plan is replaced by the new solution's
    trajectories whatever its status, and only a :solved solution becomes the
    next warm start;
  * TrajectoryGamesBase.rollout (not vendored; its published loop): for
    t = 1 … T−1, u_t = strategy(x_t, t), x_{t+1} = dynamics(x_t, u_t).

The reference runs one simulation at a time.  Here B simulations advance in
lock step, so every re-solve is ONE batched call of the C ABI (one wave or one
workgroup per game on the GPU) with per-instance warm starts.  Not restated:
the Zygote gradient that solve_trajectory_game! also computes (utils.jl:233-269,
an AD test of the example); the rrule path of mcp_amd.autodiff covers the QP
and affine families.
"""

from __future__ import annotations

import numpy as np

from .lane_change import CONTROL_DIM, NUM_PLAYERS, STATE_DIM, LaneChangeGame, double_integrator


def gpu_solver(game: LaneChangeGame, linear_solver: str | None = None, **kw):
    """The batched solve of the game's generated module through the C ABI."""
    from . import _abi
    from .batch import solve_batch

    mcp = game.mcp
    ls = linear_solver or mcp.nl.default_solver()

    def solve(theta_mcp, x0, y0):
        return solve_batch(_abi.FAMILY_NONLINEAR, mcp.nl.n, mcp.nl.m, theta_mcp, x0=x0, y0=y0, linear_solver=ls,
                           module=mcp.module(), **kw)

    return solve


class WarmStartRecedingHorizon:
    """B lock-step copies of WarmStartRecedingHorizonStrategy (utils.jl:280-308).

    `preferences`: (B, 2) lane preference per player (the strategy's
    `parameters`); `solve(theta_mcp (B, p), x0 (B, n), y0 (B, m)) -> dict` is the
    batched solver (default: the GPU, :func:`gpu_solver`)."""

    def __init__(self, game: LaneChangeGame, turn_length: int, preferences, solve=None):
        self.game = game
        self.turn_length = int(turn_length)
        self.preferences = np.atleast_2d(np.asarray(preferences, float))
        self.B = self.preferences.shape[0]
        self.solve = solve or gpu_solver(game)
        n, m = game.mcp.unconstrained_dimension, game.mcp.constrained_dimension
        self.last_x = np.zeros((self.B, n))  # last :solved solution (utils.jl:272-274)
        self.last_y = np.ones((self.B, m))
        self.has_last = np.zeros(self.B, bool)
        self.plan_us = None                   # (B, T, 4): the current plan's joint controls
        self.time_last_updated = 0
        self.statuses = []                    # status of every re-solve, (B,) each

    def _resolve(self, states: np.ndarray) -> None:
        """solve_trajectory_game! for every simulation (utils.jl:195-278)."""
        g, T = self.game, self.game.horizon
        theta = np.stack([g.pack_parameters(states[b].reshape(NUM_PLAYERS, STATE_DIM), self.preferences[b])
                          for b in range(self.B)])
        cold_x = g.initial_guess(theta)  # zero-input rollout, zero multipliers (utils.jl:218-227)
        x0 = np.where(self.has_last[:, None], self.last_x, cold_x)
        y0 = np.where(self.has_last[:, None], self.last_y, 1.0)  # y₀ default 1 (src/solver.jl:40)
        r = self.solve(g.mcp.theta_map(theta), x0, y0)
        ok = np.asarray(r["status"]) == 0
        self.last_x = np.where(ok[:, None], r["x"], self.last_x)
        self.last_y = np.where(ok[:, None], r["y"], self.last_y)
        self.has_last |= ok
        self.statuses.append(np.asarray(r["status"]).copy())
        # the plan follows the new solution whatever its status (utils.jl:276-277)
        trajs = g.trajectories(np.asarray(r["x"]))  # per player (states (B,T,4), controls (B,T,2))
        self.plan_us = np.concatenate([us for _, us in trajs], axis=-1)  # (B, T, 2·CONTROL_DIM)
        assert self.plan_us.shape[1] == T

    def __call__(self, states: np.ndarray, time: int) -> np.ndarray:
        """Joint controls (B, 4) at simulation time `time` (1-based), utils.jl:293-308."""
        plan_exists = self.plan_us is not None
        time_along_plan = time - self.time_last_updated + 1
        if not plan_exists or not (1 <= time_along_plan <= self.turn_length):
            self._resolve(np.asarray(states, float))
            self.time_last_updated = time
            time_along_plan = 1
        return self.plan_us[:, time_along_plan - 1, :]


def product_dynamics(states: np.ndarray, controls: np.ndarray) -> np.ndarray:
    """ProductDynamics of two planar double integrators (lane_change.py): (B, 8), (B, 4) → (B, 8)."""
    out = np.empty_like(states)
    for ii in range(NUM_PLAYERS):
        x = states[:, STATE_DIM * ii:STATE_DIM * (ii + 1)].T
        u = controls[:, CONTROL_DIM * ii:CONTROL_DIM * (ii + 1)].T
        out[:, STATE_DIM * ii:STATE_DIM * (ii + 1)] = np.array(double_integrator(x, u)).T
    return out


def rollout(strategy: WarmStartRecedingHorizon, initial_states, num_steps: int):
    """TrajectoryGamesBase.rollout: xs (B, num_steps, 8), us (B, num_steps − 1, 4)."""
    xs = [np.atleast_2d(np.asarray(initial_states, float))]
    us = []
    for t in range(1, num_steps):
        u = strategy(xs[-1], t)
        us.append(u)
        xs.append(product_dynamics(xs[-1], u))
    B = xs[0].shape[0]
    return np.stack(xs, 1), (np.stack(us, 1) if us else np.zeros((B, 0, 2 * CONTROL_DIM)))
