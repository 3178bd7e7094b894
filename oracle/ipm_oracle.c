/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C, single-instance-at-a-time restatement of the reference
 * interior-point solver of MixedComplementarityProblems.jl (TianyuQ/MCP),
 * src/solver.jl:35-138, for the problem families of include/mcpx.h.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this; the product path (mcp_amd/) never does.
 *
 * Parity status: the reference is Julia and cannot run here (no Julia
 * toolchain, dependencies not vendored), and it holds no golden vectors.
 * This restatement is pinned only by the reference's own analytic test
 * assertions (test/runtests.jl:30-38, :112-114, see tests/test_oracle.py) and
 * cross-checked against an independent numpy/LAPACK restatement
 * (oracle/ipm_ref.py).  Iterate-level (1e-8) parity with the Julia solver is
 * therefore "parity unpinned"; see DESIGN.md §Oracle.
 *
 * Arithmetic contract (shared bit-for-bit with the HIP kernel):
 *  - residual F per src/mcp.jl:76-80 with z = [x; y; s] (src/mcp.jl:74);
 *    dot products are fma chains in ascending column order;
 *  - Jacobian per src/mcp.jl:97-120 plus tol·I on the whole diagonal
 *    (src/solver.jl:81);
 *  - the Newton system is solved by dense LU with partial pivoting on the
 *    augmented matrix [∇F + tol·I | −F]: rows are never physically swapped;
 *    the pivot of column k is the first remaining row (ascending index) of
 *    largest |a_ik| (NaN never wins; if all remaining are NaN the first
 *    remaining row is taken); an exactly-zero pivot is the linear-solve
 *    failure (the UMFPACK "singular" retcode of src/solver.jl:84);
 *    elimination a_ij ← fma(−l_i, u_j, a_ij) with l_i = a_ik / pivot;
 *    back substitution column-oriented with x_k = b_p / u_pk;
 *  - linear_solver = MCPX_LINSOLVE_REDUCED (default) first eliminates the
 *    slack block exactly: w_k = y_k + tol (the ∂F_C/∂s diagonal entry),
 *    d_k = s_k / w_k added to the (H_k, y_k) diagonal entry after its tol,
 *    rhs_Hk = (−F_Hk) − (F_Ck / w_k); the (n+m) system is solved by the LU
 *    above and δs_k = fma(−s_k, δy_k, −F_Ck) / w_k;
 *  - linear_solver = MCPX_LINSOLVE_SCHUR (QP family) works with reciprocals:
 *    r_k = 1 / w_k, D_k = (0 + tol) + s_k·r_k, Dⁱ_k = 1 / D_k,
 *    ry_k = (−F_Hk) − (F_Ck·r_k), ty_k = ry_k·Dⁱ_k; S_ij = fma chain over
 *    k = 0 .. 4⌈m/4⌉−1 starting at (M_ij + tol·[i=j]) of A_ki · (A_kj·Dⁱ_k)
 *    (k ≥ m contributes fma(0, 0, ·),
 *    the zero padding of the fp64 MFMA K-chunks); rr_i = fma chain over k of
 *    A_ki · ty_k starting at −F_Gi; δx = S \ rr; δy_k = (fma chain over j
 *    of −A_kj · δx_j starting at ry_k)·Dⁱ_k; δs_k = fma(−s_k, δy_k, −F_Ck)·r_k.  S \ rr: when M is
 *    exactly symmetric (checked once per instance), S is symmetric and — if
 *    every pivot of elimination without pivoting is > 0 — positive definite,
 *    so it is solved by pivot-free Gauss-Jordan elimination (gj_spd_solve:
 *    pivot k is row k; every other row i, above and below, is updated with
 *    l_i = a_ik · r_k with r_k = 1 / a_kk, a_ij ← fma(−l_i, a_kj, a_ij) for j > k and the rhs,
 *    then the pivot row itself a_kj ← fma(a_kj, +0, a_kj) (identity unless
 *    non-finite; the GPU updates every lane uniformly); x_i = b_i / a_ii).  If M is not symmetric or a pivot is not
 *    > 0 (indefinite / NaN), that Newton step falls back to the partial-
 *    pivoting LU below on the same S and rr;
 *    (UMFPACK itself, LinearSolve 2.38 UMFPACKFactorization, is a third-party
 *    sparse LU not present here: this dense LU replaces it, results differ in
 *    rounding only);
 *  - line search α = decayᵉ by repeated multiplication, predicate
 *    v + α·δ < (1−τ)·v evaluated without contraction (src/solver.jl:127-138);
 *  - ϵ factors 1 − exp(−t·k) / 1 + exp(−l·k) from libm (src/solver.jl:111-113);
 *  - family MCPX_FAMILY_NONLINEAR: the per-step Jacobian blocks and G, H come
 *    from the problem's generated code (oracle_nl.init / .eval — the text of
 *    mcp_amd/codegen.py compiled by gcc, oracle/nl.py); rows are read from
 *    them as the affine family reads θ (G rows: P, Q and g = G(z) itself; H
 *    rows: R, S and h − s); SCHUR (∂H/∂y ≡ 0) without the QP family's K
 *    padding and SPD attempt.
 * Build with -ffp-contract=off (oracle/Makefile) so that only the explicit
 * fma() calls fuse.
 */
#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/mcpx.h"

typedef struct oracle_tables {
  double alpha[MCPX_MAX_LS_TRIALS];
  int n_trials; /* E + 1 */
  double c_tau; /* (1 - τ) */
  double tight[MCPX_MAX_INNER_ITERS + 1];
  double loose[MCPX_MAX_INNER_ITERS + 1];
} oracle_tables;

/* MCPX_FAMILY_NONLINEAR: the generated evaluation code of one problem.  `blk`
 * holds the blocks P, Q, R, g, h, S of mcp_amd/codegen.py's layout; init
 * writes the θ-only Jacobian entries once per instance, eval G, H and the
 * z-dependent entries at z = [x; y]. */
typedef struct oracle_nl {
  void (*init)(const double* th, double* blk);
  void (*eval)(const double* th, const double* z, double* blk);
  int32_t p, has_s, size;
  /* the module has the one-wave SCHUR kernel (codegen.py NLSystem.solvers()["schur"]): with
   * linear_solver = SCHUR and kernel != MCPX_KERNEL_WORKGROUP the product solves S by the
   * one-wave Gauss-Jordan (lu_solve_x rcp = 2), else by the workgroup kernels' LU (rcp = 1) */
  int32_t wave_schur;
  /* structural nonzeros (mcp_amd/codegen.py NLSystem.structure): K(i) of row i of
   * Q = ∂G/∂y and J(k) of row k of R = ∂H/∂x, CSR with ascending indices */
  const int32_t *qk_ptr, *qk_idx, *rj_ptr, *rj_idx;
  /* ∇F_θ of the G/H rows (src/mcp.jl:122-147): eval_theta writes the structural nonzeros
   * of the (n+m)×p column-major block dth[t·(n+m) + i] at z = [x; y]; tc = rows of
   * column t, tr = columns of row i (CSR, ascending).  Sensitivities only (may be NULL
   * for a solve). */
  void (*eval_theta)(const double* th, const double* z, double* dth);
  const int32_t *tc_ptr, *tc_idx, *tr_ptr, *tr_idx;
  /* the band kernel (mcp_amd/band.py, csrc/ipm_nl_band.hpp; mcpx_nl_band_info of the generated
   * text): band = the module has it, band_auto = MCPX_KERNEL_AUTO prefers it; S' = S[σ][:, π]
   * with σ = band_rperm, π = band_cperm (S' row / column → original index), window rows
   * ≤ k + band_ns − 1, window columns [k, k + band_wc − 1] */
  int32_t band, band_ns, band_wc, band_auto;
  const int32_t *band_rperm, *band_cperm;
} oracle_nl;

/* doubles of the block array, the S block always included (zero when absent) */
static size_t nl_blk_doubles(int n, int m) {
  return (size_t)n * n + 2 * (size_t)n * m + n + m + (size_t)m * m;
}

/* Validates the keyword arguments and precomputes what the reference computes
 * inline.  Returns 0 or MCPX_EINVAL / MCPX_EUNSUPPORTED. */
int oracle_build_tables(const mcpx_params* p, oracle_tables* t) {
  if (!(p->tol > 0) || !(p->min_stepsize > 0) || !(p->decay > 0 && p->decay < 1) ||
      !(p->tau == p->tau) || !(p->tightening_rate == p->tightening_rate) ||
      !(p->loosening_rate == p->loosening_rate) || p->max_inner_iters < 1 ||
      p->max_outer_iters < 1 ||
      (p->linear_solver != MCPX_LINSOLVE_REDUCED && p->linear_solver != MCPX_LINSOLVE_DENSE &&
       p->linear_solver != MCPX_LINSOLVE_SCHUR))
    return MCPX_EINVAL;
  if (p->max_inner_iters > MCPX_MAX_INNER_ITERS) return MCPX_EUNSUPPORTED;
  /* src/solver.jl:128-135: α = 1; while violated: if α < tol → NaN; α *= decay */
  double a = 1.0;
  int e = 0;
  for (;;) {
    if (e >= MCPX_MAX_LS_TRIALS) return MCPX_EUNSUPPORTED;
    t->alpha[e] = a;
    if (a < p->min_stepsize) break;
    a *= p->decay;
    ++e;
  }
  t->n_trials = e + 1;
  t->c_tau = 1.0 - p->tau; /* src/solver.jl:129 (1 - τ) */
  for (int k = 0; k <= p->max_inner_iters; ++k) {
    /* src/solver.jl:111-113 */
    t->tight[k] = 1.0 - exp(-p->tightening_rate * (double)k);
    t->loose[k] = 1.0 + exp(-p->loosening_rate * (double)k);
  }
  return 0;
}

/* ---- problem families: residual row + Jacobian row (src/mcp.jl:72-120) ---- */

/* The affine family under linear_solver = SCHUR: ∂H/∂y is taken as 0, the S block of θ'
 * is not read (include/mcpx.h) — family_row skips it; oracle-internal code. */
#define FAMILY_AFFINE_NOS 100

/* Row i of F and of ∇F (without tol·I) at z = [x; y; s]. */
static double family_row(int family, int n, int m, const double* th, const double* z,
                         double eps, int i, double* row) {
  const int N = n + 2 * m;
  const double* x = z;
  const double* y = z + n;
  const double* s = z + n + m;
  for (int j = 0; j < N; ++j) row[j] = 0.0;
  if (i < n) { /* G rows */
    double acc = 0.0;
    if (family == MCPX_FAMILY_QP) {
      /* G = M x − ϕ − Aᵀ y (benchmark/quadratic_program_benchmark.jl:12-32) */
      const double* M = th;
      const double* A = th + (size_t)n * n;
      const double* phi = th + (size_t)n * n + (size_t)m * n + m;
      for (int j = 0; j < n; ++j) {
        row[j] = M[(size_t)j * n + i];
        acc = fma(row[j], x[j], acc);
      }
      for (int k = 0; k < m; ++k) {
        row[n + k] = -A[(size_t)i * m + k];
        acc = fma(row[n + k], y[k], acc);
      }
      return acc - phi[i];
    } else if (family == MCPX_FAMILY_NONLINEAR) {
      /* generated blocks (mcp_amd/codegen.py): P = ∂G/∂x, Q = ∂G/∂y, g = G(x, y; θ) */
      const double* P = th;
      const double* Q = th + (size_t)n * n;
      for (int j = 0; j < n; ++j) row[j] = P[(size_t)j * n + i];
      for (int k = 0; k < m; ++k) row[n + k] = Q[(size_t)k * n + i];
      return th[(size_t)n * n + 2 * (size_t)n * m + i];
    } else { /* G = P x + Q y + g (FAMILY_AFFINE_NOS too) */
      const double* P = th;
      const double* Q = th + (size_t)n * n;
      const double* g = th + (size_t)n * n + 2 * (size_t)n * m + (size_t)m * m;
      for (int j = 0; j < n; ++j) {
        row[j] = P[(size_t)j * n + i];
        acc = fma(row[j], x[j], acc);
      }
      for (int k = 0; k < m; ++k) {
        row[n + k] = Q[(size_t)k * n + i];
        acc = fma(row[n + k], y[k], acc);
      }
      return acc + g[i];
    }
  } else if (i < n + m) { /* H − s rows */
    const int k = i - n;
    double acc = 0.0;
    row[n + m + k] = -1.0;
    if (family == MCPX_FAMILY_QP) {
      const double* A = th + (size_t)n * n;
      const double* b = th + (size_t)n * n + (size_t)m * n;
      for (int j = 0; j < n; ++j) {
        row[j] = A[(size_t)j * m + k];
        acc = fma(row[j], x[j], acc);
      }
      return (acc - b[k]) - s[k];
    } else if (family == MCPX_FAMILY_NONLINEAR) {
      /* R = ∂H/∂x, S = ∂H/∂y (a zero block when H does not depend on y), h = H(x, y; θ) */
      const double* R = th + (size_t)n * n + (size_t)n * m;
      const double* S = th + (size_t)n * n + 2 * (size_t)n * m + n + m;
      for (int j = 0; j < n; ++j) row[j] = R[(size_t)j * m + k];
      for (int q = 0; q < m; ++q) row[n + q] = S[(size_t)q * m + k];
      return th[(size_t)n * n + 2 * (size_t)n * m + n + k] - s[k];
    } else {
      const double* R = th + (size_t)n * n + (size_t)n * m;
      const double* S = th + (size_t)n * n + 2 * (size_t)n * m;
      const double* h = th + (size_t)n * n + 2 * (size_t)n * m + (size_t)m * m + n;
      for (int j = 0; j < n; ++j) {
        row[j] = R[(size_t)j * m + k];
        acc = fma(row[j], x[j], acc);
      }
      if (family == MCPX_FAMILY_AFFINE) /* FAMILY_AFFINE_NOS: S not read (SCHUR, ∂H/∂y ≡ 0) */
        for (int q = 0; q < m; ++q) {
          row[n + q] = S[(size_t)q * m + k];
          acc = fma(row[n + q], y[q], acc);
        }
      return (acc + h[k]) - s[k];
    }
  } else { /* s ⊙ y − ϵ rows */
    const int k = i - n - m;
    row[n + k] = s[k];
    row[n + m + k] = y[k];
    return s[k] * y[k] - eps;
  }
}

/* ---- dense LU with partial pivoting on [J | b]; returns 0 ok, 1 singular ---- */
/* rcp = 1 (the SCHUR step of generated nonlinear modules on the workgroup-per-instance
 * kernels): multipliers a_ik · (1 / piv) and back substitution x_k = b_p · (1 / u_kk), one
 * correctly rounded reciprocal per pivot (csrc/ipm_wg_impl.hpp, lu_vr.hpp).
 * rcp = 2 (the same step on the one-wave kernels, csrc/ipm_nl_kernel.hpp): Gauss-Jordan with
 * the same partial pivoting — the pivot of column k is searched over the remaining rows as
 * above, so the pivot sequence is the LU's — but every other row, pivoted before or not,
 * takes the update a_ij ← fma(−l_i, u_j, a_ij) for j > k and the rhs (l_i = a_ik · (1 / piv)),
 * and the pivot row itself takes it with multiplier +0 (a_pj ← fma(a_pj, +0, a_pj): the
 * identity unless non-finite; the GPU updates its lanes uniformly); then x_k = b_p · (1 / u_pk)
 * with no back substitution (the 40-step dependent chain it replaces was a third of a
 * lone wave's Newton step on the lane-change game). */
static int lu_solve_x(int N, double* J /* N×N row-major, destroyed */, double* b /* destroyed */,
                      double* dz, int* remaining, int* step_of, int* prow, int rcp) {
  for (int i = 0; i < N; ++i) remaining[i] = 1;
  for (int k = 0; k < N; ++k) {
    int best = -1;
    double bv = -1.0;
    for (int i = 0; i < N; ++i) {
      if (!remaining[i]) continue;
      const double v = fabs(J[(size_t)i * N + k]);
      if (v > bv) { bv = v; best = i; }
    }
    if (best < 0)
      for (int i = 0; i < N; ++i)
        if (remaining[i]) { best = i; break; }
    const double piv = J[(size_t)best * N + k];
    if (piv == 0.0) return 1;
    remaining[best] = 0;
    step_of[best] = k;
    prow[k] = best;
    double* u = J + (size_t)best * N;
    const double rp = 1.0 / piv;
    for (int i = 0; i < N; ++i) {
      if (rcp == 2 ? i == best : !remaining[i]) continue;
      double* a = J + (size_t)i * N;
      const double l = rcp ? a[k] * rp : a[k] / piv;
      for (int j = k + 1; j < N; ++j) a[j] = fma(-l, u[j], a[j]);
      b[i] = fma(-l, b[best], b[i]);
    }
    if (rcp == 2) { /* the pivot row, multiplier +0 */
      for (int j = k + 1; j < N; ++j) u[j] = fma(u[j], 0.0, u[j]);
      b[best] = fma(b[best], 0.0, b[best]);
    }
  }
  if (rcp == 2) {
    for (int k = 0; k < N; ++k) {
      const int p = prow[k];
      dz[k] = b[p] * (1.0 / J[(size_t)p * N + k]);
    }
    return 0;
  }
  for (int k = N - 1; k >= 0; --k) {
    const int p = prow[k];
    const double xk = rcp ? b[p] * (1.0 / J[(size_t)p * N + k]) : b[p] / J[(size_t)p * N + k];
    dz[k] = xk;
    for (int i = 0; i < N; ++i)
      if (step_of[i] < k) b[i] = fma(-J[(size_t)i * N + k], xk, b[i]);
  }
  return 0;
}

/* Pivot-free Gauss-Jordan on [S | b] for symmetric positive definite S (see the
 * header); returns 0 ok, 1 when a pivot is not > 0 (caller falls back to lu_solve). */
static int gj_spd_solve(int n, double* S /* n×n row-major, destroyed */, double* b /* destroyed */,
                        double* dz) {
  for (int k = 0; k < n; ++k) {
    const double piv = S[(size_t)k * n + k];
    if (!(piv > 0.0)) return 1;
    const double rp = 1.0 / piv; /* one reciprocal per pivot, off the GPU's multiplier chain */
    const double* u = S + (size_t)k * n;
    for (int i = 0; i < n; ++i) {
      if (i == k) continue;
      double* a = S + (size_t)i * n;
      const double l = a[k] * rp;
      for (int j = k + 1; j < n; ++j) a[j] = fma(-l, u[j], a[j]);
      b[i] = fma(-l, b[k], b[i]);
    }
    /* the pivot row takes the same update with multiplier +0 (the GPU's lane-uniform
       update; identity for finite entries, Inf → NaN otherwise) */
    double* a = S + (size_t)k * n;
    for (int j = k + 1; j < n; ++j) a[j] = fma(a[j], 0.0, a[j]);
    b[k] = fma(b[k], 0.0, b[k]);
  }
  for (int i = 0; i < n; ++i) dz[i] = b[i] / S[(size_t)i * n + i];
  return 0;
}

/* Band LU with partial pivoting of S' = S[σ][:, π] (the generated modules' band kernel,
 * csrc/ipm_nl_band.hpp; mcp_amd/band.py orders the columns for a narrow elimination window, as
 * UMFPACK's symbolic phase orders the columns of its sparse LU, src/solver.jl:50,61,83, and the
 * rows by their first nonzero column).  Rows enter the window in S' row order: rows 0 .. ns − 1
 * before step 0, row k + ns after step k; every row with a nonzero in column k is in the window
 * at step k, and every window row lies inside the columns [k, k + wc − 1].  Step k searches the
 * remaining window rows with lu_solve_x's first-max rule (largest |a_ik|, ties to the lowest S'
 * row, NaN never wins, all-NaN → the first remaining window row; an exact zero pivot is the
 * failed solve) and updates every other remaining window row in the columns k + 1 .. k + wc − 1
 * and the rhs with lu_solve_x's rcp = 1 arithmetic (l_i = a_ik · (1 / piv),
 * a_ij ← fma(−l_i, u_j, a_ij)); the back substitution takes x_k = b_p · (1 / u_pk) and updates
 * the pivot rows of steps k − wc + 1 .. k − 1.  On finite values the skipped terms are exact
 * zeros, so this is the dense LU with partial pivoting of S' (a row permutation only changes
 * which of equal |a_ik| wins).  S, rr: original order; dz: the solution in original order.
 * Returns 0 ok, 1 on a zero pivot. */
static int lu_band_solve(int n, const double* S, const double* rr, double* dz, const int32_t* rperm,
                         const int32_t* cperm, int ns, int wc, double* Sp, double* b, double* x, int* rem,
                         int* prow) {
  for (int r = 0; r < n; ++r) {
    for (int c = 0; c < n; ++c) Sp[(size_t)r * n + c] = S[(size_t)rperm[r] * n + cperm[c]];
    b[r] = rr[rperm[r]];
    rem[r] = 1;
  }
  for (int k = 0; k < n; ++k) {
    const int hi = k + ns - 1 < n - 1 ? k + ns - 1 : n - 1;
    int best = -1;
    double bv = -1.0;
    for (int i = 0; i <= hi; ++i) {
      if (!rem[i]) continue;
      const double v = fabs(Sp[(size_t)i * n + k]);
      if (v > bv) { bv = v; best = i; }
    }
    if (best < 0)
      for (int i = 0; i <= hi; ++i)
        if (rem[i]) { best = i; break; }
    const double piv = Sp[(size_t)best * n + k];
    if (piv == 0.0) return 1;
    rem[best] = 0;
    prow[k] = best;
    const double rp = 1.0 / piv;
    const int jhi = k + wc - 1 < n - 1 ? k + wc - 1 : n - 1;
    const double* u = Sp + (size_t)best * n;
    for (int i = 0; i <= hi; ++i) {
      if (!rem[i]) continue;
      double* a = Sp + (size_t)i * n;
      const double l = a[k] * rp;
      for (int j = k + 1; j <= jhi; ++j) a[j] = fma(-l, u[j], a[j]);
      b[i] = fma(-l, b[best], b[i]);
    }
  }
  for (int k = n - 1; k >= 0; --k) {
    const int p = prow[k];
    const double xk = b[p] * (1.0 / Sp[(size_t)p * n + k]);
    x[k] = xk;
    for (int t = (k - wc + 1 > 0 ? k - wc + 1 : 0); t < k; ++t) {
      const int q = prow[t];
      b[q] = fma(-Sp[(size_t)q * n + k], xk, b[q]);
    }
  }
  for (int k = 0; k < n; ++k) dz[cperm[k]] = x[k];
  return 0;
}

static int lu_solve(int N, double* J, double* b, double* dz, int* remaining, int* step_of, int* prow) {
  return lu_solve_x(N, J, b, dz, remaining, step_of, prow, 0);
}

/* first e in [0, n_trials) with no violation, or -1 (the NaN of src/solver.jl:131) */
static int linesearch_exponent(const double* v, const double* d, int cnt, const oracle_tables* t) {
  for (int e = 0; e < t->n_trials; ++e) {
    const double a = t->alpha[e];
    int viol = 0;
    for (int i = 0; i < cnt; ++i) {
      const double lhs = v[i] + a * d[i];
      const double rhs = t->c_tau * v[i];
      if (lhs < rhs) { viol = 1; break; }
    }
    if (!viol) return e;
  }
  return -1;
}

typedef struct ws {
  double *J, *Jr, *Js, *bs, *row, *F, *b, *dz, *z, *sD, *srw, *sry, *sty;
  double* blk; /* MCPX_FAMILY_NONLINEAR: the generated blocks */
  int *remaining, *step_of, *prow;
} ws;

static int ws_alloc(ws* w, int N) {
  w->blk = NULL;
  w->J = (double*)malloc(sizeof(double) * (size_t)N * N);
  w->Jr = (double*)malloc(sizeof(double) * (size_t)N * N);
  w->Js = (double*)malloc(sizeof(double) * (size_t)N * N);
  w->bs = (double*)malloc(sizeof(double) * N);
  w->row = (double*)malloc(sizeof(double) * N);
  w->sD = (double*)malloc(sizeof(double) * N);
  w->sry = (double*)malloc(sizeof(double) * N);
  w->srw = (double*)malloc(sizeof(double) * N);
  w->sty = (double*)malloc(sizeof(double) * N);
  w->F = (double*)malloc(sizeof(double) * N);
  w->b = (double*)malloc(sizeof(double) * N);
  w->dz = (double*)malloc(sizeof(double) * N);
  w->z = (double*)malloc(sizeof(double) * N);
  w->remaining = (int*)malloc(sizeof(int) * N);
  w->step_of = (int*)malloc(sizeof(int) * N);
  w->prow = (int*)malloc(sizeof(int) * N);
  return (w->J && w->Jr && w->Js && w->bs && w->sD && w->srw && w->sry && w->sty && w->row && w->F && w->b && w->dz && w->z && w->remaining && w->step_of && w->prow) ? 0 : -1;
}
static void ws_free(ws* w) {
  free(w->J); free(w->Jr); free(w->Js); free(w->bs); free(w->sD); free(w->srw); free(w->sry); free(w->sty); free(w->row); free(w->F); free(w->b); free(w->dz); free(w->z);
  free(w->remaining); free(w->step_of); free(w->prow);
  free(w->blk);
}

/* One instance: src/solver.jl:35-122. */
static void solve_one(const mcpx_desc* d, const double* th, const double* x0, const double* y0,
                      const double* s0, const mcpx_params* p, const oracle_tables* t, ws* w,
                      int64_t inst, const mcpx_out* o, const oracle_nl* nl) {
  const int n = d->n, m = d->m, N = n + 2 * m;
  double* z = w->z;
  /* src/solver.jl:39-41,64-66 */
  for (int i = 0; i < n; ++i) z[i] = x0 ? x0[inst * n + i] : 0.0;
  for (int k = 0; k < m; ++k) z[n + k] = y0 ? y0[inst * m + k] : 1.0;
  for (int k = 0; k < m; ++k) z[n + m + k] = s0 ? s0[inst * m + k] : 1.0;
  double eps = 1.0;           /* :67 */
  double kkt = INFINITY;      /* :68 */
  int status = MCPX_STATUS_SOLVED; /* :69 */
  int outer = 1;              /* :70 */
  int newton = 0;
  unsigned reason = 0;        /* MCPX_FAIL_* events (the `verbose` warnings of :85, :97) */
  int m_sym = 0; /* SCHUR: M exactly symmetric → try the SPD Gauss-Jordan first */
  /* MCPX_FAMILY_NONLINEAR: family_row reads the generated blocks instead of θ */
  const double* fth = th;
  if (nl) {
    memset(w->blk, 0, sizeof(double) * nl_blk_doubles(n, m));
    nl->init(th, w->blk);
    fth = w->blk;
  }
  const int schur_dense = p->linear_solver == MCPX_LINSOLVE_SCHUR && !nl;
  const int fam = (schur_dense && d->family == MCPX_FAMILY_AFFINE) ? FAMILY_AFFINE_NOS : d->family;
  if (schur_dense) {
    m_sym = 1;
    for (int i = 0; i < n && m_sym; ++i)
      for (int j = 0; j < n; ++j)
        if (!(th[(size_t)j * n + i] == th[(size_t)i * n + j])) { m_sym = 0; break; }
    /* affine: and −Q = Rᵀ exactly (then S = P − Q·D⁻¹·R is symmetric for every D) */
    if (d->family == MCPX_FAMILY_AFFINE)
      for (int i = 0; i < n && m_sym; ++i)
        for (int k = 0; k < m; ++k)
          if (!(-th[(size_t)n * n + (size_t)k * n + i] == th[(size_t)n * n + (size_t)n * m + (size_t)i * m + k])) {
            m_sym = 0;
            break;
          }
  }
  if (schur_dense && d->family == MCPX_FAMILY_AFFINE) {
    /* SCHUR takes ∂H/∂y ≡ 0: an affine θ with an S entry ≠ 0 (or NaN) is not solved
       (MCPX_FAIL_INPUT, include/mcpx.h) — the loop below does not run on a NaN kkt */
    const double* S = th + (size_t)n * n + 2 * (size_t)n * m;
    for (size_t i = 0; i < (size_t)m * m; ++i)
      if (!(S[i] == 0.0)) {
        kkt = NAN;
        status = MCPX_STATUS_FAILED;
        reason = MCPX_FAIL_INPUT;
        break;
      }
  }
  while (kkt > p->tol && eps > p->tol && outer < p->max_outer_iters) { /* :71 */
    int inner = 1;            /* :72 */
    status = MCPX_STATUS_SOLVED; /* :73 */
    while (kkt > eps && inner < p->max_inner_iters) { /* :75 */
      /* :79-82 F!, ∇F_z!, A = ∇F + tol I, b = −F */
      if (nl) nl->eval(th, z, w->blk);
      for (int i = 0; i < N; ++i) {
        w->F[i] = family_row(fam, n, m, fth, z, eps, i, w->J + (size_t)i * N);
        w->J[(size_t)i * N + i] += p->tol;
        w->b[i] = -w->F[i];
      }
      /* :83-88 */
      if (p->linear_solver == MCPX_LINSOLVE_DENSE) {
        if (lu_solve(N, w->J, w->b, w->dz, w->remaining, w->step_of, w->prow)) {
          status = MCPX_STATUS_FAILED;
          reason |= MCPX_FAIL_LINSOLVE;
          break;
        }
      } else if (p->linear_solver == MCPX_LINSOLVE_SCHUR) {
        /* slack block, then the diagonal y block: n×n Schur complement (QP / affine family:
           S_ij = P_ij + Σ_k (−Q_ik)·(R_kj·D_k⁻¹), the QP's A_ki·(A_kj·D_k⁻¹)) */
        const int m4 = !nl ? (m + 3) / 4 * 4 : m; /* QP / affine: the MFMA's K padding */
        for (int k = 0; k < m; ++k) {
          const int h = n + k, c = n + m + k;
          const double rwk = 1.0 / w->J[(size_t)c * N + c];  /* 1 / (y_k + tol) */
          const double D = w->J[(size_t)h * N + h] + z[c] * rwk;
          const double Di = 1.0 / D;
          const double ry = w->b[h] - (w->F[c] * rwk);
          w->sD[k] = Di;   /* D_k⁻¹ */
          w->srw[k] = rwk;
          w->sry[k] = ry;
          w->sty[k] = ry * Di;
        }
        if (nl) {
          /* nonlinear family: only the structural nonzeros enter S and rr — entry (i, j)
             takes the terms k ∈ K(i) (Q's row pattern) with j ∈ J(k) (R's row pattern),
             k ascending (structural zeros are exact zeros; a sparse elimination never
             touches them) */
          for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) {
              double acc = w->J[(size_t)i * N + j]; /* P_ij (+ tol) */
              for (int t = nl->qk_ptr[i]; t < nl->qk_ptr[i + 1]; ++t) {
                const int k = nl->qk_idx[t];
                for (int u = nl->rj_ptr[k]; u < nl->rj_ptr[k + 1]; ++u)
                  if (nl->rj_idx[u] == j) {
                    acc = fma(-w->J[(size_t)i * N + n + k], w->J[(size_t)(n + k) * N + j] * w->sD[k], acc);
                    break;
                  }
              }
              w->Jr[(size_t)i * n + j] = acc;
            }
          for (int i = 0; i < n; ++i) {
            double acc = w->b[i]; /* −F_Gi */
            for (int t = nl->qk_ptr[i]; t < nl->qk_ptr[i + 1]; ++t) {
              const int k = nl->qk_idx[t];
              acc = fma(-w->J[(size_t)i * N + n + k], w->sty[k], acc);
            }
            w->b[i] = acc;
          }
        } else {
        for (int i = 0; i < n; ++i)
          for (int j = 0; j < n; ++j) {
            double acc = w->J[(size_t)i * N + j]; /* M_ij (+ tol) */
            for (int k = 0; k < m4; ++k) {
              if (k < m) {
                const double aki = -w->J[(size_t)i * N + n + k]; /* A_ki */
                const double akj = w->J[(size_t)(n + k) * N + j];  /* A_kj */
                acc = fma(aki, akj * w->sD[k], acc);
              } else {
                acc = fma(0.0, 0.0, acc);
              }
            }
            w->Jr[(size_t)i * n + j] = acc;
          }
        for (int i = 0; i < n; ++i) {
          double acc = w->b[i]; /* −F_Gi */
          for (int k = 0; k < m; ++k) acc = fma(-w->J[(size_t)i * N + n + k], w->sty[k], acc);
          w->b[i] = acc;
        }
        }
        int spd_ok = 0;
        if (m_sym) {
          memcpy(w->Js, w->Jr, sizeof(double) * (size_t)n * n);
          memcpy(w->bs, w->b, sizeof(double) * n);
          spd_ok = gj_spd_solve(n, w->Js, w->bs, w->dz) == 0;
        }
        /* generated modules, as the C ABI picks the kernel (mcpx_api.cpp prepare): the band kernel
           (MCPX_KERNEL_BAND, or AUTO when the module prefers it or has no one-wave SCHUR kernel),
           the one-wave Gauss-Jordan (rcp = 2), else the workgroup kernels' LU (rcp = 1) */
        const int band = nl && nl->band &&
                         (p->kernel == MCPX_KERNEL_BAND ||
                          (p->kernel == MCPX_KERNEL_AUTO && (nl->band_auto || !nl->wave_schur)));
        const int xmode = !nl ? 0 : ((nl->wave_schur && p->kernel != MCPX_KERNEL_WORKGROUP) ? 2 : 1);
        if (band) {
          if (lu_band_solve(n, w->Jr, w->b, w->dz, nl->band_rperm, nl->band_cperm, nl->band_ns, nl->band_wc, w->Js,
                            w->bs, w->row, w->remaining, w->prow)) {
            status = MCPX_STATUS_FAILED;
            reason |= MCPX_FAIL_LINSOLVE;
            break;
          }
        } else if (!spd_ok && lu_solve_x(n, w->Jr, w->b, w->dz, w->remaining, w->step_of, w->prow, xmode)) {
          status = MCPX_STATUS_FAILED;
          reason |= MCPX_FAIL_LINSOLVE;
          break;
        }
        for (int k = 0; k < m; ++k) {
          double acc = w->sry[k];
          if (nl) { /* R's structural nonzeros J(k) only */
            for (int t = nl->rj_ptr[k]; t < nl->rj_ptr[k + 1]; ++t) {
              const int j = nl->rj_idx[t];
              acc = fma(-w->J[(size_t)(n + k) * N + j], w->dz[j], acc);
            }
          } else {
            for (int j = 0; j < n; ++j) acc = fma(-w->J[(size_t)(n + k) * N + j], w->dz[j], acc);
          }
          w->dz[n + k] = acc * w->sD[k];
        }
        for (int k = 0; k < m; ++k) {
          const int c = n + m + k;
          w->dz[c] = fma(-z[c], w->dz[n + k], -w->F[c]) * w->srw[k];
        }
      } else {
        /* exact elimination of the slack block, then LU of the (n+m) Schur complement */
        const int Nr = n + m;
        for (int k = 0; k < m; ++k) {
          const int h = n + k, c = n + m + k;
          const double wk = w->J[(size_t)c * N + c]; /* y_k + tol */
          const double dk = z[c] / wk;               /* s_k / w_k */
          w->J[(size_t)h * N + h] += dk;
          w->b[h] = w->b[h] - (w->F[c] / wk);
        }
        for (int i = 0; i < Nr; ++i)
          for (int j = 0; j < Nr; ++j) w->Jr[(size_t)i * Nr + j] = w->J[(size_t)i * N + j];
        if (lu_solve(Nr, w->Jr, w->b, w->dz, w->remaining, w->step_of, w->prow)) {
          status = MCPX_STATUS_FAILED;
          reason |= MCPX_FAIL_LINSOLVE;
          break;
        }
        for (int k = 0; k < m; ++k) {
          const int c = n + m + k;
          const double wk = w->J[(size_t)c * N + c];
          w->dz[c] = fma(-z[c], w->dz[n + k], -w->F[c]) / wk;
        }
      }
      /* :93-100 */
      const int es = linesearch_exponent(z + n + m, w->dz + n + m, m, t);
      const int ey = linesearch_exponent(z + n, w->dz + n, m, t);
      if (es < 0 || ey < 0) {
        status = MCPX_STATUS_FAILED;
        reason |= MCPX_FAIL_LINESEARCH;
        break;
      }
      if (o->alpha_trace && newton < o->trace_len) { /* accepted steps only */
        uint8_t* tr = o->alpha_trace + ((size_t)inst * o->trace_len + newton) * 2;
        tr[0] = (uint8_t)es;
        tr[1] = (uint8_t)ey;
      }
      const double as = t->alpha[es], ay = t->alpha[ey];
      /* :103-105 (x moves with α_s) */
      for (int i = 0; i < n; ++i) z[i] = z[i] + as * w->dz[i];
      for (int k = 0; k < m; ++k) z[n + m + k] = z[n + m + k] + as * w->dz[n + m + k];
      for (int k = 0; k < m; ++k) z[n + k] = z[n + k] + ay * w->dz[n + k];
      /* :107 kkt_error = ‖F‖∞ of the pre-step F, NaN-propagating */
      double mx = fabs(w->F[0]);
      for (int i = 1; i < N; ++i) {
        const double v = fabs(w->F[i]);
        if (v != v || v > mx) mx = v;
        if (mx != mx) break;
      }
      kkt = mx;
      ++inner;
      ++newton;
    }
    eps *= (status == MCPX_STATUS_SOLVED) ? t->tight[inner] : t->loose[inner]; /* :111-113 */
    ++outer; /* :114 */
  }
  if (outer == p->max_outer_iters) { /* :117-119 */
    status = MCPX_STATUS_FAILED;
    reason |= MCPX_FAIL_MAX_OUTER;
  }
  for (int i = 0; i < n; ++i) o->x[inst * n + i] = z[i];
  for (int k = 0; k < m; ++k) o->y[inst * m + k] = z[n + k];
  for (int k = 0; k < m; ++k) o->s[inst * m + k] = z[n + m + k];
  o->kkt_error[inst] = kkt;
  o->eps[inst] = eps;
  o->outer_iters[inst] = outer;
  o->status[inst] = status;
  if (o->newton_iters) o->newton_iters[inst] = newton;
  if (o->fail_reason) o->fail_reason[inst] = (uint8_t)reason;
  if (o->active_mask) {
    const int words = m > 64 ? (m + 63) / 64 : 1;
    uint64_t* am = o->active_mask + (size_t)inst * words;
    for (int q = 0; q < words; ++q) am[q] = 0;
    for (int k = 0; k < m; ++k)
      if (z[n + k] > z[n + m + k]) am[k / 64] |= (uint64_t)1 << (k % 64);
  }
}

typedef struct job {
  const mcpx_desc* d;
  const double *theta, *x0, *y0, *s0;
  const mcpx_params* p;
  const oracle_tables* t;
  const mcpx_out* o;
  const oracle_nl* nl; /* MCPX_FAMILY_NONLINEAR, else NULL */
  int64_t next; /* shared work counter */
  pthread_mutex_t mu;
  int err;
} job;

static void* worker(void* arg) {
  job* j = (job*)arg;
  ws w;
  int bad = ws_alloc(&w, j->d->n + 2 * j->d->m);
  if (!bad && j->nl) {
    w.blk = (double*)malloc(sizeof(double) * (nl_blk_doubles(j->d->n, j->d->m) + 1));
    bad = w.blk == NULL;
  }
  if (bad) {
    pthread_mutex_lock(&j->mu);
    j->err = 1;
    pthread_mutex_unlock(&j->mu);
    ws_free(&w);
    return NULL;
  }
  for (;;) {
    pthread_mutex_lock(&j->mu);
    const int64_t b = j->next++;
    pthread_mutex_unlock(&j->mu);
    if (b >= j->d->batch) break;
    solve_one(j->d, j->theta + b * j->d->theta_ld, j->x0, j->y0, j->s0, j->p, j->t, &w, b, j->o, j->nl);
  }
  ws_free(&w);
  return NULL;
}

int64_t oracle_theta_dim(int family, int n, int m) {
  if (n < 0 || m < 0) return -1;
  if (family == MCPX_FAMILY_QP) return (int64_t)n * n + (int64_t)m * n + m + n;
  if (family == MCPX_FAMILY_AFFINE) return (int64_t)n * n + 2 * (int64_t)n * m + (int64_t)m * m + n + m;
  return -1;
}

static int run_batch(const mcpx_desc* d, const double* theta, const double* x0, const double* y0,
                     const double* s0, const mcpx_params* p, mcpx_out* o, int nthreads,
                     const oracle_nl* nl) {
  oracle_tables t;
  const int rc = oracle_build_tables(p, &t);
  if (rc) return rc;
  job j;
  j.d = d; j.theta = theta; j.x0 = x0; j.y0 = y0; j.s0 = s0; j.p = p; j.t = &t; j.o = o; j.nl = nl;
  j.next = 0; j.err = 0;
  pthread_mutex_init(&j.mu, NULL);
  if (nthreads < 1) nthreads = 1;
  if (nthreads == 1) {
    worker(&j);
  } else {
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
    for (int i = 0; i < nthreads; ++i) pthread_create(&th[i], NULL, worker, &j);
    for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
    free(th);
  }
  pthread_mutex_destroy(&j.mu);
  return j.err ? MCPX_EINVAL : 0;
}

static int outputs_ok(const mcpx_out* o) {
  return o && o->x && o->y && o->s && o->kkt_error && o->eps && o->outer_iters && o->status;
}

/* Batched entry: same argument meaning as mcpx_solve_batch (host buffers),
 * instances distributed over `nthreads` POSIX threads (one instance per task). */
int oracle_solve_batch(const mcpx_desc* d, const double* theta, const double* x0,
                       const double* y0, const double* s0, const mcpx_params* p,
                       mcpx_out* o, int nthreads) {
  if (!d || !theta || !p || !outputs_ok(o)) return MCPX_EINVAL;
  const int64_t pd = oracle_theta_dim(d->family, d->n, d->m);
  if (pd < 0 || d->n + d->m < 1 || d->batch < 0 || d->theta_ld < pd) return MCPX_EINVAL;
  if (p->linear_solver == MCPX_LINSOLVE_SCHUR && d->family != MCPX_FAMILY_QP && d->family != MCPX_FAMILY_AFFINE)
    return MCPX_EINVAL;
  return run_batch(d, theta, x0, y0, s0, p, o, nthreads, NULL);
}

/* MCPX_FAMILY_NONLINEAR: the same with the problem's generated evaluation code. */
int oracle_solve_batch_nl(const mcpx_desc* d, const double* theta, const double* x0,
                          const double* y0, const double* s0, const mcpx_params* p,
                          mcpx_out* o, int nthreads, const oracle_nl* nl) {
  if (!d || !theta || !p || !outputs_ok(o) || !nl || !nl->init || !nl->eval) return MCPX_EINVAL;
  if (d->family != MCPX_FAMILY_NONLINEAR || d->n + d->m < 1 || d->batch < 0 || d->theta_ld < nl->p)
    return MCPX_EINVAL;
  if (p->linear_solver == MCPX_LINSOLVE_SCHUR && nl->has_s) return MCPX_EINVAL;
  return run_batch(d, theta, x0, y0, s0, p, o, nthreads, nl);
}

/* ======================================================================
 * Sensitivities (reference src/AutoDiff.jl) — see include/mcpx.h.
 *
 * ∂z/∂θ = −(∇F_z)⁻¹ ∇F_θ at the returned (x, y, s), ∇F_z WITHOUT tol·I
 * (src/AutoDiff.jl:18-40; Appendix A.10 of SURVEY.md).  The reference solves
 * with a column-pivoted QR of −∇F_z (LAPACK geqp3, :39); this restatement uses
 * lu_solve() above on ∇F_z (JVP) or on the slack-eliminated (n+m)-dim rows of
 * ∇F_zᵀ (VJP, exact elimination through the −1 entries): equal for nonsingular ∇F_z up
 * to rounding (tests/test_oracle.py cross-checks against a numpy pivoted-QR
 * restatement, oracle/ipm_ref.py).  Exactly singular ⇒ status 1, NaN outputs.
 * ====================================================================== */

/* (∇F_θ θ̇)_i: row i of F's θ-derivative applied to the tangent d (QP:
 * ∂G/∂θ·d = Ṁx − ϕ̇ − Ȧᵀy, ∂H/∂θ·d = Ȧx − ḃ; affine: Ṗx + Q̇y + ġ,
 * Ṙx + Ṡy + ḣ; complementarity rows 0).  fma chains as family_row(). */
static double dtheta_row(int family, int n, int m, const double* d, const double* z, int i) {
  const double* x = z;
  const double* y = z + n;
  const size_t nn = (size_t)n * n, nm = (size_t)n * m, mm = (size_t)m * m;
  double acc = 0.0;
  if (i < n) {
    if (family == MCPX_FAMILY_QP) {
      for (int j = 0; j < n; ++j) acc = fma(d[(size_t)j * n + i], x[j], acc);
      for (int k = 0; k < m; ++k) acc = fma(-d[nn + (size_t)i * m + k], y[k], acc);
      return acc - d[nn + nm + m + i];
    }
    for (int j = 0; j < n; ++j) acc = fma(d[(size_t)j * n + i], x[j], acc);
    for (int k = 0; k < m; ++k) acc = fma(d[nn + (size_t)k * n + i], y[k], acc);
    return acc + d[nn + 2 * nm + mm + i];
  }
  if (i < n + m) {
    const int k = i - n;
    if (family == MCPX_FAMILY_QP) {
      for (int j = 0; j < n; ++j) acc = fma(d[nn + (size_t)j * m + k], x[j], acc);
      return acc - d[nn + nm + k];
    }
    for (int j = 0; j < n; ++j) acc = fma(d[nn + nm + (size_t)j * m + k], x[j], acc);
    for (int q = 0; q < m; ++q) acc = fma(d[nn + 2 * nm + (size_t)q * m + k], y[q], acc);
    return acc + d[nn + 2 * nm + mm + n + k];
  }
  return 0.0;
}

typedef struct sens_ws {
  double *J, *JT, *b, *dz, *z, *row;
  double *blk, *dth; /* MCPX_FAMILY_NONLINEAR: generated blocks and ∇F_θ */
  int *rem, *step, *prow;
} sens_ws;

static int sens_ws_alloc(sens_ws* w, int N) {
  const size_t NN = (size_t)(N > 0 ? N : 1);
  w->J = (double*)malloc(sizeof(double) * NN * NN);
  w->JT = (double*)malloc(sizeof(double) * (NN * NN > 4 * NN ? NN * NN : 4 * NN)); /* also cond_estimate's 4 vectors */
  w->b = (double*)malloc(sizeof(double) * NN);
  w->dz = (double*)malloc(sizeof(double) * NN);
  w->z = (double*)malloc(sizeof(double) * NN);
  w->row = (double*)malloc(sizeof(double) * NN);
  w->rem = (int*)malloc(sizeof(int) * NN);
  w->step = (int*)malloc(sizeof(int) * NN);
  w->prow = (int*)malloc(sizeof(int) * NN);
  w->blk = NULL;
  w->dth = NULL;
  return !(w->J && w->JT && w->b && w->dz && w->z && w->row && w->rem && w->step && w->prow);
}

static void sens_ws_free(sens_ws* w) {
  free(w->J); free(w->JT); free(w->b); free(w->dz); free(w->z); free(w->row);
  free(w->rem); free(w->step); free(w->prow);
  free(w->blk); free(w->dth);
}

/* MCPX_FAMILY_NONLINEAR: (∇F_θ θ̇)_i from the generated block, θ columns of row i
 * ascending (tr); 0 for the s⊙y − ϵ rows. */
static double dtheta_row_nl(const oracle_nl* nl, int n, int m, const double* dth, const double* d, int i) {
  if (i >= n + m) return 0.0;
  const int nr = n + m;
  double acc = 0.0;
  for (int u = nl->tr_ptr[i]; u < nl->tr_ptr[i + 1]; ++u) {
    const int t = nl->tr_idx[u];
    acc = fma(dth[(size_t)t * nr + i], d[t], acc);
  }
  return acc;
}

/* ∇F_z (no tol·I) at z, N×N row-major, via family_row (src/mcp.jl:97-120). */
static void jacobian_z(int family, int n, int m, const double* th, const double* z, double* J) {
  const int N = n + 2 * m;
  for (int i = 0; i < N; ++i) (void)family_row(family, n, m, th, z, 0.0, i, J + (size_t)i * N);
}

/* ---- condition estimate of ∇F_z (the matrix of the rrule's solve, src/AutoDiff.jl:39) ----
 * The reference solves qr(−∇F_z, ColumnNorm()) \ ∇F_θ; at degenerate solutions ∇F_z is nearly
 * singular and QR and LU answers can differ at O(1).  rcond = 1 / (‖∇F_z‖₁ · est‖∇F_z⁻¹‖₁), the
 * Hager–Higham 1-norm estimate (Higham, "FORTRAN codes for estimating the one-norm of a real or
 * complex matrix", ACM TOMS 14 (1988), Algorithm 4.1 with its alternative lower bound) from one
 * LU with partial pivoting — the kernels' (csrc/sens_wg_impl.hpp cond_instances) op for op:
 *   factor   lu_solve's elimination (division multipliers, first-max pivots) with l_ik kept in
 *            A[i][k]; an exact zero pivot: rcond = 0, status 1;
 *   A x = b  forward: for k ascending, rows pivoted later take b_i = fma(−l_ik, b_{p_k}, b_i);
 *            back: x_k = b_{p_k} / u_{p_k k}, rows pivoted earlier b_i = fma(−u_ik, x_k, b_i);
 *   Aᵀz = c  (PA = LU) Uᵀ: u_k = c_k / u_{p_k k}, columns i > k take c_i = fma(−u_{p_k i}, u_k, c_i);
 *            Lᵀ: for k descending, v_k = u_k, j < k take u_j = fma(−l_{p_k j}, v_k, u_j); z_{p_k} = v_k;
 *   Hager    x = 1/N; at most 5 rounds: y = A⁻¹x, γ = Σ|y_k| (ascending); stop if round > 0 and
 *            not γ > γ_prev; ξ = sign(y) (+1 for y ≥ 0); stop if round > 0 and ξ is unchanged;
 *            z = A⁻ᵀξ; j = first argmax |z_i| (NaN never wins, none: 0); stop if round > 0 and
 *            not |z_j| > z_{j_prev}; x = e_j;
 *   alt      b_i = (−1)ⁱ (1 + i/(N−1)), γ = max(γ, 2·Σ|A⁻¹b| / (3N));
 *   rcond    ‖A‖₁ = max over columns of the column sums of |a_ij| (rows ascending); rcond =
 *            1 / (‖A‖₁ · γ), 0 when that product is 0 or not finite. */
static int lu_factor_keep(int N, double* J, int* remaining, int* step_of, int* prow) {
  for (int i = 0; i < N; ++i) remaining[i] = 1;
  for (int k = 0; k < N; ++k) {
    int best = -1;
    double bv = -1.0;
    for (int i = 0; i < N; ++i) {
      if (!remaining[i]) continue;
      const double v = fabs(J[(size_t)i * N + k]);
      if (v > bv) { bv = v; best = i; }
    }
    if (best < 0)
      for (int i = 0; i < N; ++i)
        if (remaining[i]) { best = i; break; }
    const double piv = J[(size_t)best * N + k];
    if (piv == 0.0) return 1;
    remaining[best] = 0;
    step_of[best] = k;
    prow[k] = best;
    const double* u = J + (size_t)best * N;
    for (int i = 0; i < N; ++i) {
      if (!remaining[i]) continue;
      double* a = J + (size_t)i * N;
      const double l = a[k] / piv;
      for (int j = k + 1; j < N; ++j) a[j] = fma(-l, u[j], a[j]);
      a[k] = l;
    }
  }
  return 0;
}

static void lu_apply(int N, const double* J, const int* step_of, const int* prow, double* b, double* x) {
  for (int k = 0; k < N; ++k) {
    const double bp = b[prow[k]];
    for (int i = 0; i < N; ++i)
      if (step_of[i] > k) b[i] = fma(-J[(size_t)i * N + k], bp, b[i]);
  }
  for (int k = N - 1; k >= 0; --k) {
    const int p = prow[k];
    const double xk = b[p] / J[(size_t)p * N + k];
    x[k] = xk;
    for (int i = 0; i < N; ++i)
      if (step_of[i] < k) b[i] = fma(-J[(size_t)i * N + k], xk, b[i]);
  }
}

static void lu_apply_t(int N, const double* J, const int* prow, double* c, double* z) {
  for (int k = 0; k < N; ++k) {
    const double* u = J + (size_t)prow[k] * N;
    const double uk = c[k] / u[k];
    c[k] = uk;
    for (int i = k + 1; i < N; ++i) c[i] = fma(-u[i], uk, c[i]);
  }
  for (int k = N - 1; k >= 0; --k) {
    const double* l = J + (size_t)prow[k] * N;
    const double vk = c[k];
    for (int j = 0; j < k; ++j) c[j] = fma(-l[j], vk, c[j]);
    z[prow[k]] = vk;
  }
}

/* J: N×N row-major ∇F_z (destroyed); v: 4·N doubles of scratch.  Returns rcond, *singular. */
static double cond_estimate(int N, double* J, int* remaining, int* step_of, int* prow, double* v, int* singular) {
  double anorm = 0.0;
  for (int j = 0; j < N; ++j) {
    double c = 0.0;
    for (int i = 0; i < N; ++i) c = c + fabs(J[(size_t)i * N + j]);
    if (c > anorm || c != c) anorm = c;
    if (anorm != anorm) break;
  }
  *singular = lu_factor_keep(N, J, remaining, step_of, prow);
  if (*singular) return 0.0;
  double *x = v, *y = v + N, *xi = v + 2 * N, *z = v + 3 * N;
  const double inv = 1.0 / (double)N;
  for (int i = 0; i < N; ++i) x[i] = inv;
  double est = 0.0;
  int jprev = -1;
  for (int it = 0; it < 5; ++it) {
    lu_apply(N, J, step_of, prow, x, y); /* x destroyed */
    double g = 0.0;
    for (int k = 0; k < N; ++k) g = g + fabs(y[k]);
    if (it > 0 && !(g > est)) break;
    est = g;
    int same = it > 0;
    for (int k = 0; k < N; ++k) {
      const double sg = y[k] >= 0.0 ? 1.0 : -1.0;
      if (sg != xi[k]) same = 0;
      xi[k] = sg;
    }
    if (same) break;
    for (int k = 0; k < N; ++k) x[k] = xi[k]; /* x: the rhs of the transposed solve */
    lu_apply_t(N, J, prow, x, z);
    int jm = -1;
    double bz = -1.0;
    for (int i = 0; i < N; ++i)
      if (fabs(z[i]) > bz) { bz = fabs(z[i]); jm = i; }
    if (jm < 0) jm = 0;
    if (it > 0 && !(fabs(z[jm]) > z[jprev])) break;
    for (int i = 0; i < N; ++i) x[i] = 0.0;
    x[jm] = 1.0;
    jprev = jm;
  }
  for (int i = 0; i < N; ++i) x[i] = (i & 1 ? -1.0 : 1.0) * (1.0 + (N > 1 ? (double)i / (double)(N - 1) : 0.0));
  lu_apply(N, J, step_of, prow, x, y);
  double g = 0.0;
  for (int k = 0; k < N; ++k) g = g + fabs(y[k]);
  const double alt = 2.0 * g / (3.0 * (double)N);
  if (alt > est) est = alt;
  const double den = anorm * est;
  return (den > 0.0 && den <= DBL_MAX) ? 1.0 / den : 0.0;
}

typedef struct sens_job {
  int jvp; /* 0 VJP, 1 JVP, 2 condition estimate (out[b] = rcond) */
  const mcpx_desc* d;
  const double *theta, *x, *y, *s, *gx, *gy, *gs, *tdot;
  int K;
  double* out;
  int32_t* status;
  const oracle_nl* nl; /* MCPX_FAMILY_NONLINEAR, else NULL */
  int64_t p;           /* θ dimension (dense stride of dtheta / theta_dot) */
  int64_t next;
  pthread_mutex_t mu;
  int err;
} sens_job;

/* QP family pullback by the Schur complement, for the one-wave sizes (n + 2m <=
 * MCPX_MAX_KKT_DIM) with M exactly symmetric, every s_k > 0, y_k >= 0 and y_k / s_k
 * finite.  The reduced system of sens_one (u = [λx; λc]) is, for the QP family,
 *     M λx + Aᵀ diag(y) λc = gx + Aᵀ gs,      −A λx + diag(s) λc = gy;
 * λc = (gy + A λx) / s leaves the n×n SPD system
 *     (M + Aᵀ diag(d) A) λx = gx + Aᵀ (gs − d ⊙ gy),   d = y / s,
 * whose matrix is formed exactly as the SCHUR solver forms S (tol = 0, D⁻¹ = d, the
 * MFMA's K padding) and solved by gj_spd_solve.  Absent cotangent blocks are zeros here.
 * On return 0, w->dz = [λx; λc]; 1: a condition or a pivot failed (→ the LU path). */
static int vjp_qp_schur(int n, int m, const double* th, const double* z, const double* gx, const double* gy,
                        const double* gs, sens_ws* w) {
  if (n < 1 || n + 2 * m > MCPX_MAX_KKT_DIM) return 1;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j)
      if (!(th[(size_t)j * n + i] == th[(size_t)i * n + j])) return 1;
  const double* y = z + n;
  const double* s = z + n + m;
  const double* A = th + (size_t)n * n; /* A_kj = A[j·m + k] */
  double* d = w->row;
  double* t = w->b + n;                 /* gs − d ⊙ gy */
  for (int k = 0; k < m; ++k) {
    if (!(s[k] > 0.0) || !(y[k] >= 0.0)) return 1;
    d[k] = y[k] / s[k];
    if (!isfinite(d[k])) return 1;
    t[k] = fma(-d[k], gy ? gy[k] : 0.0, gs ? gs[k] : 0.0);
  }
  double* S = w->J;
  const int m4 = (m + 3) / 4 * 4;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double acc = th[(size_t)j * n + i]; /* M_ij */
      if (i == j) acc = acc + 0.0;        /* the solver's + tol, tol = 0 */
      for (int k = 0; k < m4; ++k)
        acc = k < m ? fma(A[(size_t)i * m + k], A[(size_t)j * m + k] * d[k], acc) : fma(0.0, 0.0, acc);
      S[(size_t)i * n + j] = acc;
    }
  double* r = w->b;
  for (int j = 0; j < n; ++j) {
    double acc = gx ? gx[j] : 0.0;
    for (int k = 0; k < m; ++k) acc = fma(A[(size_t)j * m + k], t[k], acc);
    r[j] = acc;
  }
  if (gj_spd_solve(n, S, r, w->dz)) return 1;
  for (int k = 0; k < m; ++k) {
    double acc = gy ? gy[k] : 0.0;
    for (int j = 0; j < n; ++j) acc = fma(A[(size_t)j * m + k], w->dz[j], acc);
    w->dz[n + k] = acc / s[k];
  }
  return 0;
}

static void sens_one(const sens_job* j, sens_ws* w, int64_t b) {
  const mcpx_desc* d = j->d;
  const int n = d->n, m = d->m, N = n + 2 * m;
  const double* th = j->theta + b * d->theta_ld;
  const int64_t p = j->p;
  for (int i = 0; i < n; ++i) w->z[i] = j->x[b * n + i];
  for (int k = 0; k < m; ++k) {
    w->z[n + k] = j->y[b * m + k];
    w->z[n + m + k] = j->s[b * m + k];
  }
  /* MCPX_FAMILY_NONLINEAR: ∇F_z from the generated blocks at z (family_row reads them as
     the affine family reads θ), ∇F_θ from the generated eval_theta */
  const double* fth = th;
  if (j->nl) {
    memset(w->blk, 0, sizeof(double) * nl_blk_doubles(n, m));
    j->nl->init(th, w->blk);
    j->nl->eval(th, w->z, w->blk);
    memset(w->dth, 0, sizeof(double) * (size_t)(n + m) * (size_t)(p > 0 ? p : 1));
    j->nl->eval_theta(th, w->z, w->dth);
    fth = w->blk;
  }
  const double nanv = __builtin_nan("");
  int failed = 0;
  if (!j->jvp) {
    /* rrule pullback, src/AutoDiff.jl:59-76: ∇F_zᵀ λ = g, ∂θ = −∇F_θᵀ λ, solved on the
       slack-eliminated (n+m) system.  Row n+m+r of ∇F_zᵀ is [−1 at λh_r, y_r at λc_r] = gs_r:
       its −1 eliminates λh_r = y_r·λc_r − gs_r exactly (no division), leaving for
       u = [λx; λc]:
         row j < n:  Σ_i ∇F_z[i][j] λx_i + Σ_k (∇F_z[n+k][j]·y_k) λc_k = gx_j + Σ_k ∇F_z[n+k][j] gs_k
         row n+q:    Σ_i ∇F_z[i][n+q] λx_i + Σ_k (∇F_z[n+k][n+q]·y_k) λc_k (+ s_q at k = q) = gy_q
                     + Σ_k ∇F_z[n+k][n+q] gs_k
       (gs = NULL: the Σ gs chains are skipped), factored by lu_solve like the solver's
       REDUCED Newton system.  The GPU's vjp_kernel forms the same rows. */
    const double* yv = w->z + n;
    const double* sv = w->z + n + m;
    const int Nr = n + m;
    int schur = !j->nl && d->family == MCPX_FAMILY_QP &&
                vjp_qp_schur(n, m, th, w->z, j->gx ? j->gx + b * n : NULL, j->gy ? j->gy + b * m : NULL,
                             j->gs ? j->gs + b * m : NULL, w) == 0;
    if (!schur) jacobian_z(d->family, n, m, fth, w->z, w->J);
    for (int r = 0; r < Nr && !schur; ++r) {
      double* row = w->JT + (size_t)r * Nr;
      /* QP family, y-rows: ∂H/∂y ≡ 0 is a structural zero block — never multiplied, neither
         into the row (0 instead of 0·y_k) nor into the rhs (no fma(0, gs_k, ·)); the kernel
         (sens_kernel_impl.hpp vjp_reduced_row) skips the same terms, so Inf/NaN in y or gs
         give the same bits on both sides */
      const int qp_y = d->family == MCPX_FAMILY_QP && r >= n;
      for (int i = 0; i < n; ++i) row[i] = w->J[(size_t)i * N + r];
      for (int k = 0; k < m; ++k) {
        double v = qp_y ? 0.0 : w->J[(size_t)(n + k) * N + r] * yv[k];
        if (r == n + k) v = v + sv[k];
        row[n + k] = v;
      }
      double acc = r < n ? (j->gx ? j->gx[b * n + r] : 0.0) : (j->gy ? j->gy[b * m + (r - n)] : 0.0);
      if (j->gs && !qp_y)
        for (int k = 0; k < m; ++k) acc = fma(w->J[(size_t)(n + k) * N + r], j->gs[b * m + k], acc);
      w->b[r] = acc;
    }
    failed = schur ? 0 : lu_solve(Nr, w->JT, w->b, w->dz, w->rem, w->step, w->prow);
    if (failed) {
      for (int i = 0; i < N; ++i) w->dz[i] = nanv;
    } else {  /* [λx; λc] → [λx; λh]: λh_k = y_k·λc_k − gs_k */
      for (int k = 0; k < m; ++k) {
        const double lc = w->dz[n + k];
        w->dz[n + k] = j->gs ? fma(yv[k], lc, -j->gs[b * m + k]) : yv[k] * lc;
      }
    }
    const double* lx = w->dz;      /* λ of the G rows */
    const double* ly = w->dz + n;  /* λ of the H − s rows */
    const double* x = w->z;
    const double* y = w->z + n;
    double* o = j->out + b * p;
    const size_t nn = (size_t)n * n, nm = (size_t)n * m, mm = (size_t)m * m;
    if (j->nl) {
      /* ∂θ_t = −Σ_i ∇F_θ[i, t] λ_i over the structural nonzeros of column t, rows ascending
         (λ = [λx; λh]: the G rows, then the H − s rows) */
      const int nr = n + m;
      for (int64_t t = 0; t < p; ++t) {
        double acc = 0.0;
        for (int u = j->nl->tc_ptr[t]; u < j->nl->tc_ptr[t + 1]; ++u) {
          const int i = j->nl->tc_idx[u];
          acc = fma(w->dth[(size_t)t * nr + i], w->dz[i], acc);
        }
        o[t] = failed ? nanv : -acc;
      }
    } else if (d->family == MCPX_FAMILY_QP) {
      for (int c = 0; c < n; ++c)
        for (int r = 0; r < n; ++r) o[(size_t)c * n + r] = -(lx[r] * x[c]);               /* ∂M_rc */
      for (int c = 0; c < n; ++c)
        for (int k = 0; k < m; ++k) o[nn + (size_t)c * m + k] = fma(lx[c], y[k], -(ly[k] * x[c]));  /* ∂A_kc */
      for (int k = 0; k < m; ++k) o[nn + nm + k] = ly[k];                                  /* ∂b_k */
      for (int i = 0; i < n; ++i) o[nn + nm + m + i] = lx[i];                              /* ∂ϕ_i */
    } else {
      for (int c = 0; c < n; ++c)
        for (int r = 0; r < n; ++r) o[(size_t)c * n + r] = -(lx[r] * x[c]);               /* ∂P */
      for (int c = 0; c < m; ++c)
        for (int r = 0; r < n; ++r) o[nn + (size_t)c * n + r] = -(lx[r] * y[c]);          /* ∂Q */
      for (int c = 0; c < n; ++c)
        for (int k = 0; k < m; ++k) o[nn + nm + (size_t)c * m + k] = -(ly[k] * x[c]);     /* ∂R */
      for (int c = 0; c < m; ++c)
        for (int k = 0; k < m; ++k) o[nn + 2 * nm + (size_t)c * m + k] = -(ly[k] * y[c]); /* ∂S */
      for (int i = 0; i < n; ++i) o[nn + 2 * nm + mm + i] = -lx[i];                        /* ∂g */
      for (int k = 0; k < m; ++k) o[nn + 2 * nm + mm + n + k] = -ly[k];                    /* ∂h */
    }
  } else if (j->jvp == 2) {
    jacobian_z(d->family, n, m, fth, w->z, w->J);
    int sing = 0;
    j->out[b] = cond_estimate(N, w->J, w->rem, w->step, w->prow, w->JT, &sing);
    failed = sing;
  } else {
    /* ForwardDiff Dual method, src/AutoDiff.jl:94-100: ż = −(∇F_z)⁻¹ ∇F_θ θ̇ per partial */
    for (int c = 0; c < j->K; ++c) {
      const double* dd = j->tdot + (b * j->K + c) * p;
      double* o = j->out + (b * j->K + c) * N;
      jacobian_z(d->family, n, m, fth, w->z, w->J);
      for (int i = 0; i < N; ++i)
        w->b[i] = j->nl ? -dtheta_row_nl(j->nl, n, m, w->dth, dd, i) : -dtheta_row(d->family, n, m, dd, w->z, i);
      const int f = lu_solve(N, w->J, w->b, w->dz, w->rem, w->step, w->prow);
      failed |= f;
      for (int i = 0; i < N; ++i) o[i] = f ? nanv : w->dz[i];
    }
  }
  if (j->status) j->status[b] = failed ? 1 : 0;
}

static void* sens_worker(void* arg) {
  sens_job* j = (sens_job*)arg;
  sens_ws w;
  int bad = sens_ws_alloc(&w, j->d->n + 2 * j->d->m);
  if (!bad && j->nl) {
    w.blk = (double*)malloc(sizeof(double) * (nl_blk_doubles(j->d->n, j->d->m) + 1));
    w.dth = (double*)malloc(sizeof(double) * ((size_t)(j->d->n + j->d->m) * (size_t)(j->p > 0 ? j->p : 1) + 1));
    bad = !w.blk || !w.dth;
  }
  if (bad) {
    pthread_mutex_lock(&j->mu);
    j->err = 1;
    pthread_mutex_unlock(&j->mu);
    sens_ws_free(&w);
    return NULL;
  }
  for (;;) {
    pthread_mutex_lock(&j->mu);
    const int64_t b = j->next++;
    pthread_mutex_unlock(&j->mu);
    if (b >= j->d->batch) break;
    sens_one(j, &w, b);
  }
  sens_ws_free(&w);
  return NULL;
}

static int sens_run(sens_job* j, int nthreads) {
  const mcpx_desc* d = j->d;
  const int64_t pd = j->nl ? j->nl->p : oracle_theta_dim(d->family, d->n, d->m);
  if (pd < 0 || d->n + d->m < 1 || d->batch < 0 || d->theta_ld < pd || !j->theta || !j->out) return MCPX_EINVAL;
  if (j->nl ? (d->family != MCPX_FAMILY_NONLINEAR || !j->nl->eval_theta || !j->nl->tc_ptr || !j->nl->tr_ptr)
            : d->family == MCPX_FAMILY_NONLINEAR)
    return MCPX_EINVAL;
  j->p = pd;
  j->next = 0;
  j->err = 0;
  pthread_mutex_init(&j->mu, NULL);
  if (nthreads < 1) nthreads = 1;
  if (nthreads == 1) {
    sens_worker(j);
  } else {
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
    for (int i = 0; i < nthreads; ++i) pthread_create(&th[i], NULL, sens_worker, j);
    for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
    free(th);
  }
  pthread_mutex_destroy(&j->mu);
  return j->err ? MCPX_EINVAL : 0;
}

/* Same argument meaning as mcpx_vjp_batch / mcpx_jvp_batch (host buffers). */
int oracle_vjp_batch(const mcpx_desc* d, const double* theta, const double* x, const double* y,
                     const double* s, const double* gx, const double* gy, const double* gs,
                     double* dtheta, int32_t* status, int nthreads) {
  if (!d) return MCPX_EINVAL;
  sens_job j;
  memset(&j, 0, sizeof j);
  j.jvp = 0; j.d = d; j.theta = theta; j.x = x; j.y = y; j.s = s;
  j.gx = gx; j.gy = gy; j.gs = gs; j.out = dtheta; j.status = status;
  return sens_run(&j, nthreads);
}

/* MCPX_FAMILY_NONLINEAR: the same with the problem's generated ∇F_z / ∇F_θ code. */
int oracle_vjp_batch_nl(const mcpx_desc* d, const double* theta, const double* x, const double* y,
                        const double* s, const double* gx, const double* gy, const double* gs,
                        double* dtheta, int32_t* status, int nthreads, const oracle_nl* nl) {
  if (!d || !nl || !nl->init || !nl->eval) return MCPX_EINVAL;
  sens_job j;
  memset(&j, 0, sizeof j);
  j.jvp = 0; j.d = d; j.theta = theta; j.x = x; j.y = y; j.s = s; j.nl = nl;
  j.gx = gx; j.gy = gy; j.gs = gs; j.out = dtheta; j.status = status;
  return sens_run(&j, nthreads);
}

int oracle_jvp_batch_nl(const mcpx_desc* d, const double* theta, const double* x, const double* y,
                        const double* s, int32_t n_partials, const double* theta_dot, double* zdot,
                        int32_t* status, int nthreads, const oracle_nl* nl) {
  if (!d || !nl || !nl->init || !nl->eval || n_partials < 0 || (n_partials > 0 && !theta_dot)) return MCPX_EINVAL;
  sens_job j;
  memset(&j, 0, sizeof j);
  j.jvp = 1; j.d = d; j.theta = theta; j.x = x; j.y = y; j.s = s; j.nl = nl;
  j.tdot = theta_dot; j.K = n_partials; j.out = zdot; j.status = status;
  return sens_run(&j, nthreads);
}

/* rcond [B] and status [B] (1: ∇F_z exactly singular) at the returned iterate (cond_estimate). */
int oracle_cond_batch(const mcpx_desc* d, const double* theta, const double* x, const double* y,
                      const double* s, double* rcond, int32_t* status, int nthreads) {
  if (!d) return MCPX_EINVAL;
  sens_job j;
  memset(&j, 0, sizeof j);
  j.jvp = 2; j.d = d; j.theta = theta; j.x = x; j.y = y; j.s = s; j.out = rcond; j.status = status;
  return sens_run(&j, nthreads);
}

int oracle_cond_batch_nl(const mcpx_desc* d, const double* theta, const double* x, const double* y,
                         const double* s, double* rcond, int32_t* status, int nthreads, const oracle_nl* nl) {
  if (!d || !nl || !nl->init || !nl->eval) return MCPX_EINVAL;
  sens_job j;
  memset(&j, 0, sizeof j);
  j.jvp = 2; j.d = d; j.theta = theta; j.x = x; j.y = y; j.s = s; j.nl = nl; j.out = rcond; j.status = status;
  return sens_run(&j, nthreads);
}

int oracle_jvp_batch(const mcpx_desc* d, const double* theta, const double* x, const double* y,
                     const double* s, int32_t n_partials, const double* theta_dot, double* zdot,
                     int32_t* status, int nthreads) {
  if (!d || n_partials < 0 || (n_partials > 0 && !theta_dot)) return MCPX_EINVAL;
  sens_job j;
  memset(&j, 0, sizeof j);
  j.jvp = 1; j.d = d; j.theta = theta; j.x = x; j.y = y; j.s = s;
  j.tdot = theta_dot; j.K = n_partials; j.out = zdot; j.status = status;
  return sens_run(&j, nthreads);
}
