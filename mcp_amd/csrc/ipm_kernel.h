// ipm_kernel.h — kernel argument block shared by the launcher (mcpx_api.cpp)
// and the kernels (ipm_kernel.hip).  Passed by value (kernarg segment, ~2.3 KB).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mcpx.h"

namespace mcpx {

// Internal per-instance status of the two-pass SCHUR launch (ipm_solve_kernel
// PASS 1 → 2); never returned: the second pass overwrites it with 0 / 1.
constexpr int32_t STATUS_DEFERRED = 2;

struct KernelArgs {
  const double* theta;
  int64_t theta_ld;
  const double* x0;
  const double* y0;
  const double* s0;
  double* x;
  double* y;
  double* s;
  double* kkt_error;
  double* eps;
  int32_t* outer_iters;
  int32_t* status;
  int32_t* newton_iters;
  uint64_t* active_mask;
  uint8_t* alpha_trace;
  uint8_t* fail_reason;  // MCPX_FAIL_* bits per instance, or NULL
  uint64_t* stamps;  // diagnostic builds only (MCPX_STAMPS); NULL otherwise
  int32_t trace_len;
  int32_t n, m;
  int32_t family;   // MCPX_FAMILY_*
  int32_t solver;   // MCPX_LINSOLVE_*
  int32_t max_inner, max_outer;
  int32_t n_trials;  // line-search trials e = 0 .. n_trials-1 (α_e = decayᵉ)
  double tol;
  double c_tau;  // (1 − τ), src/solver.jl:129
  double decay;
  double tight[MCPX_MAX_INNER_ITERS + 1];  // 1 − exp(−t·k), src/solver.jl:112
  double loose[MCPX_MAX_INNER_ITERS + 1];  // 1 + exp(−l·k), src/solver.jl:113
  // fused rrule pullback (mcpx_solve_vjp_batch_device, the FUSE kernels only): ∂θ of the
  // instance right after its solve, cotangent g = a ⊙ z + b (sens_kernel.h SensArgs)
  double* vjp_dtheta;
  int32_t* vjp_status;
  const double* ct_bx;  // b of the x / y / s cotangent blocks, [B*n] / [B*m] / [B*m] or NULL = 0
  const double* ct_by;
  const double* ct_bs;
  double ct_ax, ct_ay, ct_as;  // a (scalars)
};

// Launchers of the register-resident solver: one 64-lane wave (= one
// workgroup) per instance.  nmax ∈ {8,16,24,32,48,64} ≥ the linear-system dimension
// (n + m reduced, n + 2m dense, n Schur).  Each returns hipErrorNotFound /
// hipErrorInvalidValue when it has no matching kernel.
hipError_t launch_ipm_spec(int family, int solver, int n, int m, const KernelArgs& a, int64_t batch,
                           hipStream_t st);
hipError_t launch_ipm_schur_qp(int nmax, const KernelArgs& a, int64_t batch, hipStream_t st);
hipError_t launch_ipm_schur_aff(int nmax, const KernelArgs& a, int64_t batch, hipStream_t st);
hipError_t launch_ipm_red_qp(int nmax, const KernelArgs& a, int64_t batch, hipStream_t st);
hipError_t launch_ipm_red_aff(int nmax, const KernelArgs& a, int64_t batch, hipStream_t st);
hipError_t launch_ipm_dense_qp(int nmax, const KernelArgs& a, int64_t batch, hipStream_t st);
hipError_t launch_ipm_dense_aff(int nmax, const KernelArgs& a, int64_t batch, hipStream_t st);
// The SCHUR QP solve with the rrule pullback fused into its epilogue (ipm_inst_fused.hip):
// compile-time (n, m) ∈ {(2, 2), (16, 8), (32, 16)}; hipErrorNotFound otherwise.
hipError_t launch_ipm_fused_vjp(int family, int solver, int n, int m, const KernelArgs& a, int64_t batch,
                                hipStream_t st);
bool has_fused_vjp(int family, int solver, int n, int m);

}  // namespace mcpx
