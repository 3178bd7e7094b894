/*
 * mcpx.h — C ABI of the MI355X-native batched interior-point MCP solver.
 *
 * This is the drop-in boundary for the Newton-step hot path of
 * MixedComplementarityProblems.jl (TianyuQ/MCP).  One call replaces, for a
 * whole batch of parameter vectors θ, the host loop of
 *
 *     solve(::InteriorPoint, mcp::PrimalDualMCP, θ; x₀, y₀, s₀, tol,
 *           max_inner_iters, max_outer_iters, tightening_rate,
 *           loosening_rate, min_stepsize, verbose, linear_solve_algorithm)
 *                                                  reference src/solver.jl:35-51
 *
 * i.e. the per-instance block src/solver.jl:53-121 (residual F! and Jacobian
 * ∇F_z! callbacks of src/mcp.jl:82-120, the regularised Newton solve
 * src/solver.jl:81-90, the fraction-to-the-boundary line search
 * src/solver.jl:93-100,127-138, the update src/solver.jl:103-108 and the
 * ϵ-continuation src/solver.jl:71-121).  The reference binds nothing over an
 * FFI today (it is pure Julia); the `ccall` a maintainer would add is shown in
 * INTEGRATION.md.
 *
 * Problem families (how F and ∇F are evaluated on device per instance):
 *
 *   MCPX_FAMILY_QP      the convex-QP family of
 *                       benchmark/quadratic_program_benchmark.jl:7-90:
 *                         G(x,y;θ) = M x − ϕ − Aᵀ y,  H(x,y;θ) = A x − b,
 *                       θ = [vec(M); vec(A); b; ϕ] column-major
 *                       (unpack_parameters, :77-90), p = n² + m n + m + n.
 *   MCPX_FAMILY_AFFINE  general affine MCP (any G/H affine in (x,y)):
 *                         G = P x + Q y + g,  H = R x + S y + h,
 *                       θ = [vec(P); vec(Q); vec(R); vec(S); g; h]
 *                       column-major, p = n² + 2 n m + m² + n + m.
 *                       (The Python front-end traces user G/H callables —
 *                       src/mcp.jl:27-52, :155-210 — into this layout.)
 *   MCPX_FAMILY_NONLINEAR  general G(x,y;θ), H(x,y;θ) (e.g. the trajectory games of
 *                       src/game.jl): device code generated per problem and run
 *                       through an mcpx_module (end of this header); θ is the
 *                       problem's own parameter vector.
 *
 * Conventions: all arrays are instance-major (instance b's data is contiguous,
 * stride `theta_ld` for θ); all buffers are caller-owned; the library keeps no
 * pointer after returning.  Return value 0 = OK, < 0 = API misuse / HIP error
 * (message via mcpx_last_error(), thread-local).  Numerical failure is never
 * an error: it is status[b] = MCPX_STATUS_FAILED, as in src/solver.jl:84-100,
 * 117-119, which never throws.
 */
#ifndef MCPX_H
#define MCPX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2.0.0: mcpx_out gained the trailing fail_reason pointer (1.6), which changes the
 * struct's size and layout: a caller built against a 1.x header passes a shorter
 * struct, so the major version moved.  Callers check mcpx_version() / 10000 against
 * MCPX_VERSION / 10000 before the first call (mcp_amd/_lib.py does). */
#define MCPX_VERSION 20200 /* 2.1.0: mcpx_cond_batch*; 2.2.0: MCPX_FAIL_INPUT */

/* error codes */
#define MCPX_OK 0
#define MCPX_EINVAL (-1)      /* argument check failed (reference: ArgumentError / @assert) */
#define MCPX_EHIP (-2)        /* HIP runtime error */
#define MCPX_ENODEV (-3)      /* no usable gfx950 device */
#define MCPX_EUNSUPPORTED (-4) /* size outside what the compiled kernels cover */

/* per-instance status (reference: :solved / :failed, src/solver.jl:69,86,98,118) */
#define MCPX_STATUS_SOLVED 0
#define MCPX_STATUS_FAILED 1
/* mcpx_out.fail_reason bits: the events behind the reference's `verbose` warnings
 * (src/solver.jl), each set when it happened at least once during the solve */
#define MCPX_FAIL_LINSOLVE 1u   /* a Newton system was singular, a zero pivot (:84-88) */
#define MCPX_FAIL_LINESEARCH 2u /* the fraction-to-the-boundary line search gave NaN (:93-99) */
#define MCPX_FAIL_MAX_OUTER 4u  /* outer_iters reached max_outer_iters (:117-119) */
/* the instance is outside what the chosen elimination is exact for, so it was not solved:
 * MCPX_LINSOLVE_SCHUR on an affine θ whose S block (∂H/∂y) is not exactly zero.  The record
 * is status FAILED, kkt_error NaN, the initial point, outer_iters 1, newton_iters 0. */
#define MCPX_FAIL_INPUT 8u

#define MCPX_FAMILY_QP 0
#define MCPX_FAMILY_AFFINE 1
#define MCPX_FAMILY_NONLINEAR 2

/* largest linear-system dimension of the register-resident one-wave kernels
 * (n + m for MCPX_LINSOLVE_REDUCED, n + 2m for MCPX_LINSOLVE_DENSE) */
#define MCPX_MAX_KKT_DIM 64
/* largest KKT dimension n + 2m of the workgroup-per-instance kernels of the QP
 * and affine families (blocked LU with MFMA trailing updates, REDUCED / DENSE);
 * a generated nonlinear module sizes its own (mcpx_module_dims) */
#define MCPX_MAX_WG_KKT_DIM 768

/* Which kernel family runs a solve (mcpx_params.kernel):
 *  MCPX_KERNEL_AUTO       one wave per instance when the system fits its 64 rows,
 *                         else one workgroup per instance;
 *  MCPX_KERNEL_WAVE       only the one-wave kernels (MCPX_EUNSUPPORTED beyond);
 *  MCPX_KERNEL_WORKGROUP  the workgroup-per-instance kernels at any size they
 *                         support (REDUCED / DENSE, and SCHUR for generated
 *                         modules) — bit-identical results to the one-wave path;
 *  MCPX_KERNEL_MULTIWAVE  generated modules, SCHUR: one 4-wave workgroup per
 *                         instance, S in LDS, the LU's columns split over the waves
 *                         (module kernel-mask bit MCPX_MODULE_SCHUR_MW); same bits,
 *                         opt-in (slower than one wave on the lane-change game);
 *  MCPX_KERNEL_BAND       generated modules, SCHUR: one wave per instance, the band LU
 *                         of the symmetrically reordered Schur complement (module bit
 *                         MCPX_MODULE_BAND; the oracle's lu_band_solve).  AUTO takes it
 *                         when the module prefers it (bit MCPX_MODULE_BAND_AUTO) or has
 *                         no one-wave SCHUR kernel. */
#define MCPX_KERNEL_AUTO 0
#define MCPX_KERNEL_WAVE 1
#define MCPX_KERNEL_WORKGROUP 2
#define MCPX_KERNEL_MULTIWAVE 3
#define MCPX_KERNEL_BAND 4
/* largest max_inner_iters (ϵ-schedule table length) */
#define MCPX_MAX_INNER_ITERS 128
/* largest number of line-search trials (α = decayᵉ, e = 0..E) */
#define MCPX_MAX_LS_TRIALS 64

/* Newton linear solve (∇F + tol·I) δz = −F, src/solver.jl:81-83:
 *  MCPX_LINSOLVE_REDUCED  exact block elimination of the slack block first —
 *                         ∂(s⊙y − ϵ)/∂s = Y + tol·I is diagonal for every MCP of
 *                         the form F = [G; H − s; s⊙y − ϵ] (src/mcp.jl:76-80) —
 *                         then dense LU with partial pivoting of the (n+m)-dim
 *                         Schur complement (default; N ≤ 64 means n + m ≤ 64);
 *  MCPX_LINSOLVE_DENSE    dense LU with partial pivoting of the full
 *                         (n+2m)-dim system (n + 2m ≤ 64);
 *  MCPX_LINSOLVE_SCHUR    ∂H/∂y = 0 (QP family; affine family, whose S block must
 *                         then be exactly 0 — an instance with any nonzero (or NaN)
 *                         S entry is not solved and reports MCPX_FAIL_INPUT; generated modules
 *                         without an ∂H/∂y block): after the slack block, the
 *                         now-diagonal y block is eliminated as well, leaving the
 *                         n×n Schur complement S = (M + tol·I) + Aᵀ D⁻¹ A (affine:
 *                         (P + tol·I) − Q D⁻¹ R; both formed on the matrix cores,
 *                         fp64 MFMA).  M (affine: P) exactly symmetric (affine:
 *                         and −Q = Rᵀ exactly): S is solved by pivot-free
 *                         Gauss-Jordan while every pivot is > 0 (S SPD), and by
 *                         dense LU with partial pivoting otherwise — the oracle
 *                         takes the same branch (gj_spd_solve / lu_solve); a QP
 *                         passed as affine (P = M, Q = −Aᵀ, R = A, g = −ϕ, h = −b)
 *                         gives the QP solve's bits.  Modules: dense LU with
 *                         partial pivoting.  One wave: n + m ≤ 64; the QP family
 *                         also on one workgroup per instance up to n = 128 (S formed
 *                         on MFMA, blocked Gauss-Jordan with MFMA trailing updates,
 *                         the same bits). */
#define MCPX_LINSOLVE_REDUCED 0
#define MCPX_LINSOLVE_DENSE 1
#define MCPX_LINSOLVE_SCHUR 2

/* Solver keyword arguments, same names and defaults as src/solver.jl:42-50;
 * tau and decay are the hard-coded defaults of
 * fraction_to_the_boundary_linesearch (src/solver.jl:127). */
typedef struct mcpx_params {
  double tol;               /* 1e-4 */
  double tightening_rate;   /* 0.1  */
  double loosening_rate;    /* 0.5  */
  double min_stepsize;      /* 1e-4 (the docstring's 1e-2 is stale, src/solver.jl:31 vs :48) */
  double tau;               /* 0.995 */
  double decay;             /* 0.5  */
  int32_t max_inner_iters;  /* 20 */
  int32_t max_outer_iters;  /* 50 */
  int32_t linear_solver;    /* MCPX_LINSOLVE_* — the reference's linear_solve_algorithm kwarg (src/solver.jl:50) */
  int32_t kernel;           /* MCPX_KERNEL_* (0 = auto) */
} mcpx_params;

/* Batch descriptor. */
typedef struct mcpx_desc {
  int32_t family;   /* MCPX_FAMILY_* */
  int32_t n;        /* unconstrained_dimension (src/mcp.jl:22) */
  int32_t m;        /* constrained_dimension   (src/mcp.jl:23) */
  int32_t pad_;
  int64_t batch;    /* number of instances B */
  int64_t theta_ld; /* doubles between consecutive instances' θ (>= mcpx_theta_dim) */
} mcpx_desc;

/* Outputs, one record per instance.  Required: x, y, s, kkt_error, eps,
 * outer_iters, status (the NamedTuple of src/solver.jl:121).  Optional
 * (NULL = not wanted): newton_iters (total Newton steps taken),
 * active_mask (bit k of word b*W + k/64 set iff y_k > s_k at return, W = max(1, ⌈m/64⌉)),
 * alpha_trace (per accepted Newton step two bytes (e_s, e_y): α = decay^e;
 * at most trace_len steps recorded per instance), fail_reason (MCPX_FAIL_* bits of the
 * failure events seen; status is FAILED iff MCPX_FAIL_MAX_OUTER is set or the last
 * outer iteration ended in one of the other two). */
typedef struct mcpx_out {
  double* x;            /* [B*n] */
  double* y;            /* [B*m] */
  double* s;            /* [B*m] */
  double* kkt_error;    /* [B] */
  double* eps;          /* [B] */
  int32_t* outer_iters; /* [B] */
  int32_t* status;      /* [B] */
  int32_t* newton_iters;  /* [B] or NULL */
  uint64_t* active_mask;  /* [B*W] or NULL */
  uint8_t* alpha_trace;   /* [B*trace_len*2] or NULL */
  int32_t trace_len;
  int32_t pad_;
  uint8_t* fail_reason;   /* [B] or NULL */
} mcpx_out;

int mcpx_version(void);
const char* mcpx_last_error(void);
void mcpx_default_params(mcpx_params* prm);
/* θ dimension p of a family at (n, m); < 0 on bad input. */
int64_t mcpx_theta_dim(int32_t family, int32_t n, int32_t m);
/* number of visible HIP devices (0 when none) */
int mcpx_device_count(void);
/* Debug: with MCPX_POISON=1 in the environment every device block the library allocates for
 * itself is filled with NaN bytes up to its requested size and a canary after it, checked when
 * the block is released; this returns the number of blocks found overwritten past their size
 * (each also reported on stderr).  0 without MCPX_POISON. */
int64_t mcpx_debug_canary_violations(void);

/* Host-buffer batched solve (what the Julia ccall / Python API drive).
 * Copies θ (and optional warm starts x0/y0/s0, each [B*n] / [B*m], NULL ⇒
 * the defaults x₀=0, y₀=1, s₀=1 of src/solver.jl:39-41) to `num_devices`
 * GPUs (0 ⇒ all visible), shards the batch contiguously, solves and copies
 * the outputs back.  Blocking.  Per device the shard is pipelined in chunks on
 * two streams (the upload of chunk c+1 overlaps the solve of chunk c); θ in a
 * range registered with mcpx_host_register is read by DMA straight from the
 * caller's pages, any other θ is staged by the HIP runtime.  The environment
 * variable MCPX_HOST_SHARDS = k (tests) splits the batch into k shards over the
 * visible devices round-robin, one host thread each, as k devices would. */
int mcpx_solve_batch(const mcpx_desc* desc, const double* theta,
                     const double* x0, const double* y0, const double* s0,
                     const mcpx_params* prm, int num_devices, mcpx_out* out);

/* Page-lock a caller-owned host range (hipHostRegister, all devices) so that the
 * host-buffer calls read it by asynchronous DMA; optional, for long-lived θ
 * batches.  The range must stay allocated until mcpx_host_unregister(ptr).
 * MCPX_OK, MCPX_EINVAL (NULL / empty), MCPX_EHIP. */
int mcpx_host_register(void* ptr, size_t bytes);
int mcpx_host_unregister(void* ptr);

/* Device-buffer batched solve on the current device: every pointer in the
 * call (theta, x0/y0/s0 and every mcpx_out array) is device memory.
 * Enqueued on `stream` (a hipStream_t; NULL = default stream); returns
 * without synchronising.  This is the hot path the benchmark times. */
int mcpx_solve_batch_device(const mcpx_desc* desc, const double* theta,
                            const double* x0, const double* y0, const double* s0,
                            const mcpx_params* prm, const mcpx_out* out,
                            void* stream);


/* ---------------------------------------------------------------------------
 * Sensitivities of a solution w.r.t. θ (reference src/AutoDiff.jl).
 *
 * The reference differentiates F(z; θ) = 0 at the returned iterate:
 *     ∂z/∂θ = −(∇F_z)⁻¹ ∇F_θ      (src/AutoDiff.jl:18-40; `qr(−∇F_z, ColumnNorm()) \ ∇F_θ`)
 * with ∇F_z WITHOUT the tol·I regularisation, at the final (x, y, s)
 * (SURVEY.md Appendix A.10).  For both families ∇F_z and ∇F_θ do not depend on ϵ.
 * The kernels solve the same square system by dense LU with partial pivoting:
 * the JVP factors the full (n+2m)-dim ∇F_z, the VJP the (n+m)-dim system left
 * after eliminating λ_s of ∇F_zᵀ exactly through its −1 entries (no division);
 * for a nonsingular ∇F_z that equals the reference's pivoted-QR solve up to
 * rounding (amplified by cond(∇F_z), which is large at degenerate solutions).  An exactly zero
 * pivot (∇F_z singular, where the reference's QR would return a basic
 * least-squares solution) is reported per instance: status[b] = 1 and the
 * instance's outputs are NaN.
 *
 * Reverse mode — the ChainRulesCore.rrule pullback (src/AutoDiff.jl:42-82):
 *     ∂θ = (∂z/∂θ)ᵀ [∂l/∂x; ∂l/∂y; ∂l/∂s] = −∇F_θᵀ λ,  ∇F_zᵀ λ = [∂l/∂x; ∂l/∂y; ∂l/∂s].
 * Inputs (instance-major): θ (stride theta_ld), x [B*n], y [B*m], s [B*m],
 * gx [B*n], gy [B*m], gs [B*m] (any of gx/gy/gs may be NULL = zero cotangent,
 * ChainRulesCore's ZeroTangent).  Output: dtheta [B*p] (p = mcpx_theta_dim,
 * dense stride p, the family's θ layout), status [B] or NULL.
 * n + 2m <= MCPX_MAX_KKT_DIM runs one wave per instance (the system in registers),
 * larger systems up to MCPX_MAX_WG_KKT_DIM one workgroup per instance: blocked LU
 * with partial pivoting and MFMA trailing updates, on a per-slot HBM workspace
 * holding [K | rhs] (the register-resident LU of the solve kernels, lu_vr.hpp, is
 * not used by the sensitivity kernels); both give the same bits. */
int mcpx_vjp_batch(const mcpx_desc* desc, const double* theta, const double* x, const double* y,
                   const double* s, const double* gx, const double* gy, const double* gs,
                   int num_devices, double* dtheta, int32_t* status);
/* Same on device buffers of the current device, enqueued on `stream`. */
int mcpx_vjp_batch_device(const mcpx_desc* desc, const double* theta, const double* x,
                          const double* y, const double* s, const double* gx, const double* gy,
                          const double* gs, double* dtheta, int32_t* status, void* stream);

/* Solve and pullback in one call — the rrule of solve (src/AutoDiff.jl:42-82) applied
 * at the returned iterate, for a loss whose cotangent is given per block as
 *     ∂l/∂x = ax·x + bx,  ∂l/∂y = ay·y + by,  ∂l/∂s = as·s + bs
 * (b arrays [B*n] / [B*m] on the device, NULL = 0; a = 0 with b = NULL is
 * ChainRulesCore's ZeroTangent; a·z + b is rounded twice, no fma).  The AD test's
 * f = Σx² + Σy² (test/runtests.jl:72-75) is {ax = 2, ay = 2, as = 0, NULLs}. */
typedef struct mcpx_cotangent {
  double ax, ay, as;
  const double* bx; /* [B*n] or NULL */
  const double* by; /* [B*m] or NULL */
  const double* bs; /* [B*m] or NULL */
} mcpx_cotangent;

/* mcpx_solve_batch_device into `out`, then the pullback of `ct` at the solution into
 * dtheta [B*p] / vjp_status [B] (or NULL), device buffers of the current device,
 * enqueued on `stream`.  For the QP family with linear_solver = SCHUR at the
 * compiled (n, m) of the benchmarks ((2,2), (16,8), (32,16)) the pullback runs in
 * the epilogue of the solve kernel (one launch, the iterate never leaves the wave);
 * every other configuration runs the solve and mcpx_vjp_batch_device on `stream`.
 * Both give the bits of mcpx_solve_batch_device followed by mcpx_vjp_batch_device
 * with gx = ax·x + bx, gy = ay·y + by, gs = as·s + bs. */
int mcpx_solve_vjp_batch_device(const mcpx_desc* desc, const double* theta,
                                const double* x0, const double* y0, const double* s0,
                                const mcpx_params* prm, const mcpx_out* out,
                                const mcpx_cotangent* ct, double* dtheta,
                                int32_t* vjp_status, void* stream);

/* Conditioning of the pullback's matrix.  The reference's rrule solves with a column-pivoted QR
 * of −∇F_z (src/AutoDiff.jl:39); at degenerate solutions ∇F_z is nearly singular and QR and LU
 * sensitivities can differ at O(1).  rcond[b] = 1 / (‖∇F_z‖₁ · est‖∇F_z⁻¹‖₁) at (x, y, s), ∇F_z
 * without tol·I: the Hager–Higham estimate (≤ 5 rounds of solves with the LU factors and
 * their transpose, plus the alternating-sign lower bound), which never exceeds the true
 * ‖∇F_z⁻¹‖₁, so rcond[b] ≥ 1 / cond₁(∇F_z).  status[b] = 1 and rcond[b] = 0: ∇F_z exactly
 * singular.  A caller flags an instance as ill-conditioned when rcond[b] < its threshold
 * (mcp_amd.batch.ILL_CONDITIONED = 1e-12: fewer than ~4 significant digits in the
 * sensitivities).  Every size runs one workgroup per instance (n + 2m <= MCPX_MAX_WG_KKT_DIM). */
int mcpx_cond_batch(const mcpx_desc* desc, const double* theta, const double* x, const double* y,
                    const double* s, int num_devices, double* rcond, int32_t* status);
int mcpx_cond_batch_device(const mcpx_desc* desc, const double* theta, const double* x, const double* y,
                           const double* s, double* rcond, int32_t* status, void* stream);

/* Forward mode — the ForwardDiff.Dual method of solve (src/AutoDiff.jl:84-117):
 *     ż_c = (∂z/∂θ) θ̇_c = −(∇F_z)⁻¹ (∇F_θ θ̇_c),   c = 0 .. n_partials−1.
 * theta_dot [B*n_partials*p] (instance-major, then partial-major, stride p);
 * zdot [B*n_partials*(n+2m)], z = [x; y; s] ordering (src/mcp.jl:74);
 * status [B] or NULL.  One factorisation of ∇F_z serves up to
 * MCPX_JVP_RHS partials at a time. */
#define MCPX_JVP_RHS 8
int mcpx_jvp_batch(const mcpx_desc* desc, const double* theta, const double* x, const double* y,
                   const double* s, int32_t n_partials, const double* theta_dot, int num_devices,
                   double* zdot, int32_t* status);
int mcpx_jvp_batch_device(const mcpx_desc* desc, const double* theta, const double* x,
                          const double* y, const double* s, int32_t n_partials,
                          const double* theta_dot, double* zdot, int32_t* status, void* stream);

/* ---------------------------------------------------------------------------
 * Nonlinear G/H — MCPX_FAMILY_NONLINEAR (BASELINE C4: games, src/game.jl).
 *
 * The reference compiles F!/∇F_z! from Symbolics expressions once per problem
 * (build_function, src/mcp.jl:82-120).  The front-end does the same for the
 * GPU (mcp_amd/codegen.py): straight-line device code for G, H and their
 * Jacobian blocks, compiled with the solver template
 * (mcp_amd/csrc/ipm_nl_kernel.hpp) into one gfx950 code object per problem.
 * These calls load and run it.  A module holds the kernels its size admits:
 * one-wave MCPX_LINSOLVE_SCHUR (∂H/∂y ≡ 0, n ≤ 64, m ≤ 128), _REDUCED
 * (n + m ≤ 64), _DENSE (n + 2m ≤ 64), and workgroup-per-instance kernels of
 * each of them (SCHUR: ∂H/∂y ≡ 0) whose LDS footprint fits
 * (e.g. the lane change at T = 10: n = 200, m = 250, KKT dimension 700), and
 * the one-wave band SCHUR kernel when the reordered Schur complement has a
 * narrow band (MCPX_KERNEL_BAND); another linear_solver is MCPX_EUNSUPPORTED.
 */
typedef struct mcpx_module mcpx_module;
/* Sensitivity kernels of a module (bits of the mcpx_module_dims kernel mask) */
#define MCPX_MODULE_VJP 6
#define MCPX_MODULE_JVP 7
#define MCPX_MODULE_SCHUR_MW 8  /* the 4-wave SCHUR solve kernel (MCPX_KERNEL_MULTIWAVE) */
#define MCPX_MODULE_BAND 9       /* the band SCHUR solve kernel (MCPX_KERNEL_BAND) */
#define MCPX_MODULE_BAND_AUTO 10 /* MCPX_KERNEL_AUTO prefers the band kernel */
/* Loads the code object at `path` on the current device (other devices load
 * it on first use).  No usable GPU: MCPX_ENODEV. */
int mcpx_module_load(const char* path, mcpx_module** mod);
/* The module's n, m, θ dimension p and kernel mask: bit MCPX_LINSOLVE_* for the
 * one-wave kernels, bit 3 + MCPX_LINSOLVE_* for the workgroup kernels, bits
 * MCPX_MODULE_VJP / MCPX_MODULE_JVP for the sensitivity kernels; NULL pointers
 * are skipped. */
int mcpx_module_dims(const mcpx_module* mod, int32_t* n, int32_t* m, int32_t* p, int32_t* solvers);
void mcpx_module_unload(mcpx_module* mod);
/* mcpx_solve_batch / mcpx_solve_batch_device for the module's problem:
 * desc->family = MCPX_FAMILY_NONLINEAR, desc->n / m = the module's, theta_ld >= p. */
int mcpx_solve_batch_module(mcpx_module* mod, const mcpx_desc* desc, const double* theta,
                            const double* x0, const double* y0, const double* s0,
                            const mcpx_params* prm, int num_devices, mcpx_out* out);
int mcpx_solve_batch_module_device(mcpx_module* mod, const mcpx_desc* desc, const double* theta,
                                   const double* x0, const double* y0, const double* s0,
                                   const mcpx_params* prm, const mcpx_out* out, void* stream);

/* Sensitivities of the module's problem — the rrule pullback and the Dual method of
 * src/AutoDiff.jl for any PrimalDualMCP built with compute_sensitivities = true
 * (src/mcp.jl:122-147: ∇F_θ from the generated mcpx_nl_eval_theta), e.g. the
 * trajectory games of src/game.jl.  Same argument meaning as mcpx_vjp_batch /
 * mcpx_jvp_batch with p = the module's θ dimension; one workgroup per instance
 * (VJP: the (n+m)-dim reduced ∇F_zᵀ system, JVP: the (n+2m)-dim ∇F_z, blocked LU
 * with partial pivoting).  MCPX_EUNSUPPORTED when the module has no such kernel
 * (mask bits MCPX_MODULE_VJP / MCPX_MODULE_JVP). */
int mcpx_vjp_batch_module(mcpx_module* mod, const mcpx_desc* desc, const double* theta, const double* x,
                          const double* y, const double* s, const double* gx, const double* gy,
                          const double* gs, int num_devices, double* dtheta, int32_t* status);
int mcpx_vjp_batch_module_device(mcpx_module* mod, const mcpx_desc* desc, const double* theta,
                                 const double* x, const double* y, const double* s, const double* gx,
                                 const double* gy, const double* gs, double* dtheta, int32_t* status,
                                 void* stream);
int mcpx_jvp_batch_module(mcpx_module* mod, const mcpx_desc* desc, const double* theta, const double* x,
                          const double* y, const double* s, int32_t n_partials, const double* theta_dot,
                          int num_devices, double* zdot, int32_t* status);
int mcpx_jvp_batch_module_device(mcpx_module* mod, const mcpx_desc* desc, const double* theta,
                                 const double* x, const double* y, const double* s, int32_t n_partials,
                                 const double* theta_dot, double* zdot, int32_t* status, void* stream);
int mcpx_cond_batch_module(mcpx_module* mod, const mcpx_desc* desc, const double* theta, const double* x,
                           const double* y, const double* s, int num_devices, double* rcond, int32_t* status);
int mcpx_cond_batch_module_device(mcpx_module* mod, const mcpx_desc* desc, const double* theta,
                                  const double* x, const double* y, const double* s, double* rcond,
                                  int32_t* status, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* MCPX_H */
