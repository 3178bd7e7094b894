// ipm_wg.h — launch record and launchers of the workgroup-per-instance solver
// (ipm_wg_impl.hpp) for KKT systems beyond the one-wave kernels' 64 rows.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ipm_kernel.h"
#include "sens_kernel.h"

namespace mcpx {
namespace wg {

// The one-wave kernels' KernelArgs plus the work queue and the per-slot workspace
// (mcpx_api.cpp sizes it; one slot per resident workgroup).
struct WgArgs {
  KernelArgs k;
  double* work;         // grid slots × slot_stride doubles
  int32_t* counter;     // work-queue head, zeroed before the launch
  int64_t batch;        // instances
  int64_t slot_stride;  // doubles per slot
  int64_t off_blk;      // nonlinear family: generated Jacobian blocks (MCPX_NL_SIZE doubles)
  int64_t off_rd;       // SCHUR: R·D⁻¹ (m × n, row k = constraint k)
  int64_t off_aux;      // SCHUR: D⁻¹, 1/w, ry, ty (4 × m)
  int32_t ld;           // row stride of [K | rhs] (≥ ns + 1)
  int32_t pad_;
};

// Sensitivity kernels of the workgroup-per-instance layout (sens_wg_impl.hpp): the
// one-wave SensArgs plus the work queue and the per-slot workspace — [K | rhs] of the
// slack-eliminated (n+m)-dim ∇F_zᵀ system (VJP) or of the full (n+2m)-dim ∇F_z (JVP,
// `nrhs` partials per factorisation), and for a generated module its Jacobian blocks
// and ∇F_θ.
struct WgSensArgs {
  SensArgs s;
  double* work;         // grid slots × slot_stride doubles
  int32_t* counter;     // work-queue head, zeroed before the launch
  int64_t batch;        // instances
  int64_t slot_stride;  // doubles per slot
  int64_t off_blk;      // nonlinear family: generated Jacobian blocks (MCPX_NL_SIZE doubles)
  int64_t off_dth;      // nonlinear family: ∇F_θ of the G/H rows, (n+m) × p column-major
  int64_t off_sol;      // JVP: the nrhs solutions (nrhs × ns)
  int32_t ld;           // row stride of [K | rhs] (≥ ns + nrhs)
  int32_t nrhs;         // right-hand sides per factorisation (JVP partials; 1 for the VJP)
};

constexpr int kThreads = 256;       // workgroup size of every workgroup kernel (4 waves)
constexpr int kMaxDim = 768;        // largest system / vector dimension of the QP / affine kernels
constexpr int kDimBuckets[4] = {128, 256, 512, 768};
constexpr int kGjMax = 128;         // largest n of the QP family's workgroup SCHUR kernels (gj_vr.hpp)
// The LDS row stride of that copy: odd, so the lanes' reads of one k over 16 rows (the
// formation's A fragments, rr) fall in different banks (with m = 64 an even stride put all 16
// rows in one bank).
__host__ __device__ constexpr int kGjLda(int m) { return m | 1; }
// doubles of the A block those kernels keep in LDS (n·kGjLda(m) ≤ this): the largest of bucket
// NV (n ≤ 128, n + 2m ≤ NV), capped at 128 · 65 (KKT 256's n = 128, m = 64)
constexpr int kGjACapOf(int nv) {
  int best = 1;
  for (int n = 1; n <= kGjMax && n < nv; ++n) best = (n * kGjLda((nv - n) / 2) > best) ? n * kGjLda((nv - n) / 2) : best;
  return best < 128 * 65 ? best : 128 * 65;
}
template <int NV>
constexpr int kGjACap = kGjACapOf(NV);

}  // namespace wg

// QP / affine families, MCPX_LINSOLVE_REDUCED or _DENSE, vector dimension
// n + 2m ≤ nv ∈ wg::kDimBuckets.  The kernel symbol (for the occupancy query)
// and the launch; hipErrorInvalidValue when no such kernel exists.
// ns: rows of the factored system (a system of at most MCPX_VR_MAX rows is factored in
// registers, lu_vr.hpp).
const void* ipm_wg_kernel(int family, int solver, int nv, int ns);
// The register-resident ones (ipm_inst_wg_vr.hip): bucket 128, and bucket 256 for
// systems of at most MCPX_VR_MAX rows; nullptr otherwise.
const void* ipm_wg_vr_kernel(int family, int solver, int nv);
// The QP family's MCPX_LINSOLVE_SCHUR for n ≤ wg::kGjMax (ipm_inst_wg_gj.hip); nullptr otherwise.
const void* ipm_wg_gj_kernel(int nv);
hipError_t launch_ipm_wg(int family, int solver, int nv, int ns, const wg::WgArgs& a, int grid, hipStream_t st);
// Sensitivity kernels of the QP and affine families beyond the one-wave kernels'
// 64 rows (sens_inst_wg.hip): VJP (jvp = false) or JVP at vector dimension
// n + 2m ≤ nv ∈ wg::kDimBuckets.
const void* sens_wg_kernel(int family, bool jvp, int nv);
hipError_t launch_sens_wg(int family, bool jvp, int nv, const wg::WgSensArgs& a, int grid, hipStream_t st);

}  // namespace mcpx
