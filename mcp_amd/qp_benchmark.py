"""Random convex-QP family of the reference benchmark.

Restates benchmark/quadratic_program_benchmark.jl:
  - generate_random_parameter (:51-74):  P ~ N(0,1)^{n×n} ⊙ Bernoulli(1−sparsity),
    M = PᵀP, A ~ N(0,1)^{m×n} ⊙ Bernoulli(1−sparsity), b ~ N(0,1)^m, ϕ ~ N(0,1)^n,
    θ = [vec(M); vec(A); b; ϕ] (column-major vec, :73);
  - unpack_parameters (:77-90).
The reference draws from Julia's MersenneTwister(1) (benchmark/path.jl:14),
which cannot be reproduced without Julia; we use numpy's PCG64 (host) or
torch's Philox (device) with a documented seed instead.  θ layout and the
distribution are identical.
"""

from __future__ import annotations

import numpy as np


def theta_dim(n: int, m: int) -> int:
    return n * n + m * n + m + n


def generate_random_parameter(rng: np.random.Generator, num_primals: int = 100,
                              num_inequalities: int = 100, sparsity_rate: float = 0.9,
                              batch: int | None = None) -> np.ndarray:
    """One θ (batch=None) or a (batch, p) array of θs, column-major blocks."""
    n, m = num_primals, num_inequalities
    B = 1 if batch is None else int(batch)
    keep = 1.0 - sparsity_rate
    P = rng.standard_normal((B, n, n))
    if sparsity_rate > 0:
        P *= rng.random((B, n, n)) < keep
    M = np.einsum("bki,bkj->bij", P, P)  # PᵀP
    A = rng.standard_normal((B, m, n))
    if sparsity_rate > 0:
        A *= rng.random((B, m, n)) < keep
    b = rng.standard_normal((B, m))
    phi = rng.standard_normal((B, n))
    theta = np.concatenate([
        M.transpose(0, 2, 1).reshape(B, n * n),  # vec(M), column-major
        A.transpose(0, 2, 1).reshape(B, m * n),  # vec(A), column-major
        b, phi], axis=1)
    return theta[0] if batch is None else theta


def unpack_parameters(theta: np.ndarray, num_primals: int, num_inequalities: int):
    """(:77-90) → dict(M, A, b, ϕ)."""
    n, m = num_primals, num_inequalities
    th = np.asarray(theta)
    M = th[: n * n].reshape(n, n, order="F")
    A = th[n * n : n * n + m * n].reshape(m, n, order="F")
    b = th[n * n + m * n : n * n + m * n + m]
    phi = th[n * n + m * n + m :]
    return dict(M=M, A=A, b=b, phi=phi)


def affine_embedding(theta: np.ndarray, num_primals: int, num_inequalities: int) -> np.ndarray:
    """The QP θ = [vec M; vec A; b; ϕ] as affine-family data θ' = [vec P; vec Q; vec R; vec S; g; h]
    (include/mcpx.h): P = M, Q = −Aᵀ, R = A, S = 0, g = −ϕ, h = −b — what the Julia shim's
    `affine_parameters` hands over for the benchmark's PrimalDualMCP."""
    n, m = num_primals, num_inequalities
    th = np.atleast_2d(np.asarray(theta, dtype=np.float64))
    B = th.shape[0]
    M = th[:, :n * n]
    A = th[:, n * n:n * n + m * n].reshape(B, n, m)  # [b, i, k] = A_ki (column-major m×n)
    b = th[:, n * n + m * n:n * n + m * n + m]
    phi = th[:, n * n + m * n + m:n * n + m * n + m + n]
    Q = -A.transpose(0, 2, 1)  # [b, k, i] = Q_ik (column-major n×m)
    return np.ascontiguousarray(np.concatenate([M, Q.reshape(B, -1), A.reshape(B, -1), np.zeros((B, m * m)),
                                                -phi, -b], 1))


def generate_random_parameter_torch(generator, num_primals: int, num_inequalities: int,
                                    batch: int, sparsity_rate: float = 0.0, device="cuda"):
    """Same distribution and layout, generated directly in device memory with torch
    (used by bench.py so that 65536×12.7 KB of θ never crosses PCIe)."""
    import torch

    n, m, B = num_primals, num_inequalities, int(batch)
    kw = dict(generator=generator, device=device, dtype=torch.float64)
    P = torch.randn(B, n, n, **kw)
    A = torch.randn(B, m, n, **kw)
    if sparsity_rate > 0:
        P *= (torch.rand(B, n, n, **kw) < 1.0 - sparsity_rate)
        A *= (torch.rand(B, m, n, **kw) < 1.0 - sparsity_rate)
    M = torch.bmm(P.transpose(1, 2), P)
    b = torch.randn(B, m, **kw)
    phi = torch.randn(B, n, **kw)
    return torch.cat([M.transpose(1, 2).reshape(B, n * n), A.transpose(1, 2).reshape(B, m * n),
                      b, phi], dim=1).contiguous()


# Instances of a benchmark batch are drawn in fixed chunks, chunk c from its own
# stream SeedSequence(seed, spawn_key=(c,)), so that instance i of the global batch
# is the same whichever rank (and however many ranks) generates it: strong- and
# weak-scaling runs at any GPU count solve identical θ.
SEED_CHUNK = 4096


def chunked_slice(draw, seed: int, start: int, count: int, chunk: int = SEED_CHUNK) -> np.ndarray:
    """Rows [start, start + count) of a batch drawn chunk by chunk: `draw(rng, k)`
    returns k rows, chunk c is drawn from SeedSequence(seed, spawn_key=(c,))."""
    parts, i, end = [], int(start), int(start) + int(count)
    while i < end:
        c = i // chunk
        block = draw(np.random.default_rng(np.random.SeedSequence(seed, spawn_key=(c,))), chunk)
        lo, hi = i - c * chunk, min(end, (c + 1) * chunk) - c * chunk
        parts.append(np.asarray(block)[lo:hi])
        i += hi - lo
    if not parts:
        return np.empty((0, 0))
    return np.ascontiguousarray(np.concatenate(parts, 0))


def generate_global_slice(seed: int, num_primals: int, num_inequalities: int, sparsity_rate: float,
                          start: int, count: int, chunk: int = SEED_CHUNK) -> np.ndarray:
    """θ of global instances [start, start + count) of the QP batch seeded by `seed`."""
    n, m = num_primals, num_inequalities
    if count == 0:
        return np.empty((0, theta_dim(n, m)))
    return chunked_slice(lambda rng, k: generate_random_parameter(rng, n, m, sparsity_rate, batch=k),
                         seed, start, count, chunk)
