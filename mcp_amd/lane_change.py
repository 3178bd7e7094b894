"""BASELINE C4 workload: the two-player lane-change trajectory game of the
reference's examples/lane_change.jl, built into a ParametricGame the way
examples/utils.jl builds it (build_mcp_components / build_parametric_game,
:52-178), with the θ generator of benchmark/trajectory_game_benchmark.jl:62-87.

The collision-avoidance constraint ‖p¹_t − p²_t‖² − 4 ≥ 0 (lane_change.jl:39-46)
makes H quadratic and G bilinear in (x, μ̃), so the game lands in the nonlinear
family (MCPX_FAMILY_NONLINEAR, generated device code).  Horizon T gives
n = 12T primals + 8T shared-equality multipliers λ̃ = 20T and
m = T + 8T + 8T + 8T = 25T inequality multipliers μ̃ (40 and 50 at T = 2).

Pieces the example takes from packages that are not vendored in
/root/reference (TrajectoryGamesBase, TrajectoryGamesExamples, LazySets) are
restated from their published definitions, unverified against those packages
(absent here):
  * planar_double_integrator(; dt = 0.1, m = 1): x = (px, py, vx, vy),
    u = (Fx, Fy), x⁺ = A x + B u, A = [I dt·I; 0 I], B = [dt²/2·I; dt·I] / m;
  * PolygonEnvironment constraints: for every player's position p and every
    edge a·p ≤ b of the road polygon (LazySets' outward edge normals of the
    counter-clockwise vertex list, unnormalised), −a·p + b ≥ 0, edges varying
    fastest (the Iterators.product order);
  * get_constraints_from_box_bounds: [v − lb; −(v − ub)] over the finite bounds;
  * LazySets.sample on the road rectangle: uniform.
"""

from __future__ import annotations

import math

import numpy as np

from .api import OptimizationProblem, ParametricGame, mortar

STATE_DIM, CONTROL_DIM, NUM_PLAYERS = 4, 2, 2
DT, MASS = 0.1, 1.0
STATE_LB, STATE_UB = (-math.inf, -math.inf, -10.0, 0.0), (math.inf, math.inf, 10.0, 10.0)  # lane_change.jl:49
CONTROL_LB, CONTROL_UB = (-5.0, -5.0), (3.0, 3.0)  # lane_change.jl:50
INITIAL_STATE = ((1.0, 1.0, 0.0, 1.0), (3.2, 0.9, 0.0, 1.0))  # lane_change.jl:58


def setup_road_environment(lane_width=2.0, num_lanes=2, height=50.0):
    """examples/lane_change.jl:2-12: lane centres and the road polygon (counter-clockwise)."""
    centers = [(i - 0.5) * lane_width for i in range(1, num_lanes + 1)]
    left, right = centers[0] - 0.5 * lane_width, centers[-1] + 0.5 * lane_width
    return centers, [(left, 0.0), (right, 0.0), (right, height), (left, height)]


def polygon_halfplanes(vertices):
    """a·p ≤ b per edge v_i → v_{i+1} of a counter-clockwise convex polygon:
    a = (Δy, −Δx) (outward, unnormalised), b = a·v_i."""
    out = []
    for i, (x1, y1) in enumerate(vertices):
        x2, y2 = vertices[(i + 1) % len(vertices)]
        a = (y2 - y1, x1 - x2)
        out.append((a, a[0] * x1 + a[1] * y1))
    return out


def double_integrator(x, u, dt=DT, mass=MASS):
    """planar_double_integrator's step x⁺ = A x + B u (restated, module docstring)."""
    h = 0.5 * dt * dt / mass
    return [x[0] + dt * x[2] + h * u[0], x[1] + dt * x[3] + h * u[1], x[2] + dt / mass * u[0],
            x[3] + dt / mass * u[1]]


def box_constraints(v, lb, ub):
    """get_constraints_from_box_bounds: [v − lb; −(v − ub)] over the finite bounds."""
    return ([v[i] - lb[i] for i in range(len(v)) if not math.isinf(lb[i])]
            + [-(v[i] - ub[i]) for i in range(len(v)) if not math.isinf(ub[i])])


def _split(v, size, count):
    if hasattr(v, "blocks"):
        return v.blocks()
    v = np.asarray(v)
    return [v[size * i:size * (i + 1)] for i in range(count)]


class LaneChangeGame:
    """The lane-change ParametricGame at horizon T (lane_change.jl:57-73 with the
    road of :2-12, the game of :15-55 and the MCP components of utils.jl:87-178)."""

    def __init__(self, horizon: int = 2, lane_width: float = 2.0, num_lanes: int = 2, height: float = 50.0,
                 backend_options=None):
        self.horizon = int(horizon)
        self.lane_centers, self.vertices = setup_road_environment(lane_width, num_lanes, height)
        self.halfplanes = polygon_halfplanes(self.vertices)
        self.primal_dim = self.horizon * (STATE_DIM + CONTROL_DIM)  # per player, utils.jl:157-160
        self.param_dim = STATE_DIM + 1  # initial state + one lane preference (params_per_player = 1)
        problems = [OptimizationProblem(objective=self._objective(ii)) for ii in range(NUM_PLAYERS)]
        self.game = ParametricGame(
            test_point=mortar([np.zeros(self.primal_dim) for _ in range(NUM_PLAYERS)]),
            test_parameter=mortar([np.zeros(self.param_dim) for _ in range(NUM_PLAYERS)]),
            problems=problems, shared_equality=self._shared_equality,
            shared_inequality=self._shared_inequality, backend_options=backend_options)
        self.mcp = self.game.mcp

    # ---- the game (utils.jl:2-16, 87-155) -------------------------------------
    def unpack_trajectory(self, tau):
        """utils.jl:2-16: per time step t the players' states xs[t][i] and controls us[t][i]."""
        T, S, C = self.horizon, STATE_DIM, CONTROL_DIM
        trajs = _split(tau, self.primal_dim, NUM_PLAYERS)
        xs = [[tr[S * t:S * (t + 1)] for tr in trajs] for t in range(T)]
        us = [[tr[S * T + C * t:S * T + C * (t + 1)] for tr in trajs] for t in range(T)]
        return xs, us

    def _objective(self, ii):
        def player_cost(tau, theta_i):  # utils.jl:96-102, stage cost lane_change.jl:17-25
            xs, us = self.unpack_trajectory(tau)
            pref = theta_i[-1]
            total = None
            for t in range(self.horizon):  # discount factor 1 (lane_change.jl:35)
                x, u = xs[t][ii], us[t][ii]
                c = ((x[0] - pref) ** 2 + 0.5 * ((x[2] - 0.0) ** 2 + (x[3] - 2.0) ** 2)
                     + 0.1 * (u[0] ** 2 + u[1] ** 2))
                total = c if total is None else total + c
            return total / self.horizon  # reducer: reduce(+) / length (lane_change.jl:27-29)
        return player_cost

    def _shared_equality(self, tau, theta):  # utils.jl:109-123: initial state, then dynamics
        xs, us = self.unpack_trajectory(tau)
        th = _split(theta, self.param_dim, NUM_PLAYERS)
        g = [xs[0][ii][j] - th[ii][j] for ii in range(NUM_PLAYERS) for j in range(STATE_DIM)]
        for t in range(1, self.horizon):
            for ii in range(NUM_PLAYERS):
                nxt = double_integrator(xs[t - 1][ii], us[t - 1][ii])
                g += [xs[t][ii][j] - nxt[j] for j in range(STATE_DIM)]
        return g

    def _shared_inequality(self, tau, theta):  # utils.jl:126-155
        xs, us = self.unpack_trajectory(tau)
        T = self.horizon
        # collision avoidance (lane_change.jl:39-46)
        h = [(xs[t][0][0] - xs[t][1][0]) ** 2 + (xs[t][0][1] - xs[t][1][1]) ** 2 - 4 for t in range(T)]
        for t in range(T):  # environment: every player's position, every edge
            for ii in range(NUM_PLAYERS):
                p = xs[t][ii]
                h += [-(a[0] * p[0] + a[1] * p[1]) + b for a, b in self.halfplanes]
        for t in range(T):  # actuator limits
            h += box_constraints(list(us[t][0]) + list(us[t][1]), CONTROL_LB * 2, CONTROL_UB * 2)
        for t in range(T):  # state limits
            h += box_constraints(list(xs[t][0]) + list(xs[t][1]), STATE_LB * 2, STATE_UB * 2)
        return h

    # ---- parameters, initial guesses, solutions ---------------------------------
    def pack_parameters(self, initial_states, preferences):
        """utils.jl:27-29: per player [initial state; lane preference]."""
        return np.concatenate([np.concatenate([np.asarray(x, float), [float(p)]])
                               for x, p in zip(initial_states, preferences)])

    def example_parameters(self):
        """θ of run_lane_change_example: INITIAL_STATE and lane_centers[1] for both (lane_change.jl:58,72)."""
        return self.pack_parameters(INITIAL_STATE, [self.lane_centers[0]] * NUM_PLAYERS)

    def generate_random_parameter(self, rng, batch: int):
        """benchmark/trajectory_game_benchmark.jl:62-87: per player a position sampled on
        the road (uniform on the rectangle), zero velocity and a lane reference drawn
        from the lane centres.  numpy PCG64 stands in for the reference's
        MersenneTwister(1), which cannot be reproduced without Julia.  (B, 10)."""
        th = np.zeros((batch, NUM_PLAYERS * self.param_dim))
        (x_lo, _), (x_hi, _), (_, y_hi) = self.vertices[0], self.vertices[1], self.vertices[2]
        for ii in range(NUM_PLAYERS):
            o = ii * self.param_dim
            th[:, o] = rng.uniform(x_lo, x_hi, batch)
            th[:, o + 1] = rng.uniform(0.0, y_hi, batch)
            th[:, o + STATE_DIM] = rng.choice(self.lane_centers, batch)
        return th

    def initial_guess(self, theta):
        """x₀ of solve_trajectory_game! without a warm start (utils.jl:218-227): the
        zero-input rollout from the initial state (T states, T zero controls) per
        player, then zero multipliers λ̃.  (B, n)."""
        th = np.atleast_2d(np.asarray(theta, float))
        B, T = th.shape[0], self.horizon
        x0 = np.zeros((B, self.mcp.unconstrained_dimension))
        zero_u = np.zeros((CONTROL_DIM, B))
        for ii in range(NUM_PLAYERS):
            s = th[:, ii * self.param_dim: ii * self.param_dim + STATE_DIM].T
            base = ii * self.primal_dim
            for t in range(T):
                x0[:, base + STATE_DIM * t: base + STATE_DIM * (t + 1)] = s.T
                s = np.array(double_integrator(s, zero_u))
        return x0

    def trajectories(self, x):
        """Per player (states (…, T, 4), controls (…, T, 2)) of a solution's x."""
        x = np.asarray(x)
        T = self.horizon
        out = []
        for ii in range(NUM_PLAYERS):
            tr = x[..., ii * self.primal_dim:(ii + 1) * self.primal_dim]
            out.append((tr[..., :STATE_DIM * T].reshape(*tr.shape[:-1], T, STATE_DIM),
                        tr[..., STATE_DIM * T:].reshape(*tr.shape[:-1], T, CONTROL_DIM)))
        return out


def prebuild(horizons=(2,), verbose: bool = False) -> list:
    """Compile the C4 modules ahead of time (in-tree, by __graft_entry__.build())."""
    return [LaneChangeGame(T).mcp.nl.build_module(verbose=verbose) for T in horizons]
