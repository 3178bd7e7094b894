// ipm_kernel.h — kernel argument block shared by the launcher (mcpx_api.cpp)
// and the kernels (ipm_kernel.hip).  Passed by value (kernarg segment, ~2.3 KB).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mcpx.h"

namespace mcpx {

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
  uint64_t* stamps;  // diagnostic builds only (MCPX_STAMPS); NULL otherwise
  int32_t trace_len;
  int32_t n, m;
  int32_t max_inner, max_outer;
  int32_t n_trials;  // line-search trials e = 0 .. n_trials-1 (α_e = decayᵉ)
  double tol;
  double c_tau;  // (1 − τ), src/solver.jl:129
  double decay;
  double tight[MCPX_MAX_INNER_ITERS + 1];  // 1 − exp(−t·k), src/solver.jl:112
  double loose[MCPX_MAX_INNER_ITERS + 1];  // 1 + exp(−l·k), src/solver.jl:113
};

// Launches the register-resident solver: one 64-lane wave (= one workgroup)
// per instance.  nmax ∈ {8,16,32,64} ≥ n + 2m; family = MCPX_FAMILY_*.
// allow_specialized: use a compile-time-(n, m) kernel when one matches.
hipError_t launch_ipm(int nmax, int family, const KernelArgs& args, int64_t batch, hipStream_t stream,
                      bool allow_specialized);

}  // namespace mcpx
