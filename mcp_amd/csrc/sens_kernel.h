// sens_kernel.h — argument block and launchers of the sensitivity kernels
// (reference src/AutoDiff.jl): the reverse-mode pullback (rrule, :42-82) and the
// forward-mode Dual path (:84-117).  Shared by mcpx_api.cpp and sens_inst_*.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mcpx.h"

namespace mcpx {

struct SensArgs {
  const double* theta;
  int64_t theta_ld;
  const double* x;  // [B*n] solution (src/AutoDiff.jl:25 `(; x, y, s, ϵ) = solution`)
  const double* y;  // [B*m]
  const double* s;  // [B*m]
  const double* gx;  // VJP cotangents ∂l/∂x [B*n] (NULL = 0)
  const double* gy;  // ∂l/∂y [B*m]
  const double* gs;  // ∂l/∂s [B*m]
  const double* theta_dot;  // JVP tangents [B*K*p]
  double* out;              // VJP: dtheta [B*p]; JVP: zdot [B*K*(n+2m)]
  int32_t* status;          // [B] or NULL: 0 ok, 1 ∇F_z singular (outputs NaN)
  int64_t p;                // θ dimension of the family (dense stride of dtheta / theta_dot)
  int32_t n, m;
  int32_t n_partials;       // K (JVP)
  int32_t family;
  int32_t mode;             // workgroup JVP kernels: 1 = condition estimate (out = rcond [B], mcpx_cond_batch)
  int32_t pad_;
  // VJP cotangent g = a ⊙ z + b per block (b = gx / gy / gs above, NULL = 0): a = 0 is the
  // plain cotangent arrays; a ≠ 0 the gradient of a separable quadratic loss
  // l = Σ ½ a z² + b·z (e.g. a = 2, b = 0: f = Σx² + Σy², test/runtests.jl:72-75),
  // computed in the kernel as a·z + b (two roundings, no fma)
  double ga_x, ga_y, ga_s;
};

// One cotangent entry g = a·z + b (a = 0 → b, 0 when b is absent; b absent → a·z).
__device__ __forceinline__ double affine_ct(double a, double z, const double* b) {
  if (a == 0.0) return b ? *b : 0.0;
  return b ? a * z + *b : a * z;
}

// One 64-lane wave per instance; nmax ∈ {8,16,24,32,48,64} ≥ n + 2m.
// hipErrorInvalidValue when no kernel matches.
hipError_t launch_vjp(int nmax, const SensArgs& a, int64_t batch, hipStream_t st);
hipError_t launch_jvp(int nmax, const SensArgs& a, int64_t batch, hipStream_t st);

}  // namespace mcpx
