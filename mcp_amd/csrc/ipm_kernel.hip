// ipm_kernel.hip — gfx950 (CDNA4) kernels of the batched interior-point MCP solver.
//
// One 64-lane wavefront solves one MCP instance end to end: the whole
// ϵ-continuation / Newton loop of the reference, src/solver.jl:64-121, runs on
// the device with no host round trip.  Lane i owns row i of the KKT system:
//   z_i (iterate), F_i (residual, src/mcp.jl:76-80), the row i of
//   ∇F_z + tol·I (src/mcp.jl:97-120, src/solver.jl:81) held in NMAX fp64
//   VGPRs, and the right-hand side −F_i.
// The Newton system (src/solver.jl:81-90, UMFPACK in the reference) is solved
// by a register-resident dense LU with partial pivoting on the augmented
// matrix: rows stay in their lanes; the pivot search is a 32-bit DPP max over
// the high word of |a_ik| (exact two-phase tie resolution on the low word);
// the pivot row is broadcast to the wave through SGPRs (v_readlane) and every
// remaining lane eliminates with v_fma_f64.  Back substitution is
// column-oriented with one SGPR broadcast per column.  The fraction-to-the-
// boundary line search (src/solver.jl:127-138) evaluates every trial step
// α = decayᵉ at once (one ballot per e) and takes the first all-clear e.
//
// Arithmetic is the contract of oracle/ipm_oracle.c (same op order, explicit
// fma, -ffp-contract=off), so results are bit-identical to the CPU oracle.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ipm_kernel.h"

// Diagnostic phase stamps (tools/phase_profile.hip builds with MCPX_STAMPS=1;
// the product build compiles them away).
#ifndef MCPX_STAMPS
#define MCPX_STAMPS 0
#endif
#if MCPX_STAMPS
#define MCPX_STAMP(i)                                   \
  do {                                                  \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();   \
    st_acc[i] += t_ - st_last;                          \
    st_last = t_;                                       \
  } while (0)
#else
#define MCPX_STAMP(i) \
  do {                \
  } while (0)
#endif

namespace mcpx {

namespace {

__device__ __forceinline__ double bcast(double v, int src) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), src);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), src);
  return __hiloint2double(hi, lo);
}

// Broadcast 4 doubles of lane `p` to the wave through SGPRs.  A dynamic-lane
// v_readlane costs ≈8.5 cycles per dword on gfx950 (tools/ubench_mfma64.hip);
// v_readfirstlane under an EXEC mask holding only lane p costs ≈3.5, so the
// pivot-row broadcast runs with EXEC switched to the pivot lane.  The trailing
// s_nop 1 covers the VALU-writes-SGPR → VALU-reads-SGPR hazard that hipcc does
// not see through inline asm.
__device__ __forceinline__ void bcast4(double v0, double v1, double v2, double v3, uint64_t pmask,
                                       double& u0, double& u1, double& u2, double& u3) {
  int o0, o1, o2, o3, o4, o5, o6, o7;
  uint64_t saved;
  asm volatile(
      "s_mov_b64 %[sv], exec\n\t"
      "s_mov_b64 exec, %[pm]\n\t"
      "v_readfirstlane_b32 %0, %[a0]\n\t"
      "v_readfirstlane_b32 %1, %[a1]\n\t"
      "v_readfirstlane_b32 %2, %[a2]\n\t"
      "v_readfirstlane_b32 %3, %[a3]\n\t"
      "v_readfirstlane_b32 %4, %[a4]\n\t"
      "v_readfirstlane_b32 %5, %[a5]\n\t"
      "v_readfirstlane_b32 %6, %[a6]\n\t"
      "v_readfirstlane_b32 %7, %[a7]\n\t"
      "s_mov_b64 exec, %[sv]\n\t"
      "s_nop 1"
      : "=s"(o0), "=s"(o1), "=s"(o2), "=s"(o3), "=s"(o4), "=s"(o5), "=s"(o6), "=s"(o7), [sv] "=&s"(saved)
      : [a0] "v"(__double2loint(v0)), [a1] "v"(__double2hiint(v0)), [a2] "v"(__double2loint(v1)),
        [a3] "v"(__double2hiint(v1)), [a4] "v"(__double2loint(v2)), [a5] "v"(__double2hiint(v2)),
        [a6] "v"(__double2loint(v3)), [a7] "v"(__double2hiint(v3)), [pm] "s"(pmask));
  u0 = __hiloint2double(o1, o0);
  u1 = __hiloint2double(o3, o2);
  u2 = __hiloint2double(o5, o4);
  u3 = __hiloint2double(o7, o6);
}

// Wave-wide max of an unsigned 32-bit key, result uniform.  DPP row_shr
// 1/2/4/8 then row_bcast 15/31 (GFX9 DPP; 0 is the identity for `max`).
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false));
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

// Hides a uniform value from the optimiser for one loop iteration so that the
// ~3·NMAX uniform predicates derived from it (j < n, k < N, …) are recomputed
// where used instead of being hoisted out of the Newton loop and kept live in
// SGPRs (which spills them into VGPR lanes).
__device__ __forceinline__ int opaque(int v) {
  asm volatile("" : "+s"(v));
  return v;
}
// Same for the θ base pointer and the lane index: keeps the NMAX per-lane θ
// addresses of the Jacobian assembly from being hoisted out of the Newton loop
// (they would occupy 2·NMAX registers for the whole solve).
__device__ __forceinline__ int64_t opaque64(int64_t v) {
  asm volatile("" : "+s"(v));
  return v;
}
__device__ __forceinline__ int opaque_lane(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

__device__ __forceinline__ int lowest_lane(uint64_t mask) { return __ffsll((unsigned long long)mask) - 1; }

// Exact wave max of non-negative, non-NaN doubles (bit patterns are monotone).
__device__ __forceinline__ double wave_max_nonneg(double v) {
  const uint32_t hi = (uint32_t)__double2hiint(v);
  const uint32_t lo = (uint32_t)__double2loint(v);
  const uint32_t mhi = wave_max_u32(hi);
  const uint32_t mlo = wave_max_u32(hi == mhi ? lo : 0u);
  return __hiloint2double((int)mhi, (int)mlo);
}

// Row `lane` of F and of ∇F_z + tol·I for the problem family (src/mcp.jl:72-120).
// `zs` is the wave's copy of z in LDS.  Same op order as family_row() of
// oracle/ipm_oracle.c.  Every lane streams its row of θ through one per-lane
// base pointer and stride per column block (no per-column branches); lanes
// that read nothing in a block get stride 0 on a valid address and a masked
// value.
template <int NMAX, int FAMILY>
__device__ __forceinline__ double assemble_row(const double* __restrict__ th, const double* zs,
                                               int lane, int n, int m, double eps, double tol,
                                               double (&a)[NMAX]) {
  const int N = n + 2 * m;
  const bool rg = lane < n;                       // G rows
  const bool rh = lane >= n && lane < n + m;      // H − s rows
  const bool rc = lane >= n + m && lane < N;      // s⊙y − ϵ rows
  const int kh = lane - n;                        // H row index
  const int kc = lane - n - m;                    // complementarity index
  const int nn = n * n, nm = n * m, mm = m * m;
  // x-column block: G rows read M[i,:] / P[i,:], H rows A[k,:] / R[k,:]
  const double* px = th;
  int sx = 0;
  if (rg) { px = th + lane; sx = n; }
  if (rh) { px = th + (FAMILY == 0 ? nn : nn + nm) + kh; sx = m; }
  // y-column block: QP G rows read A[:,i] (contiguous); affine G rows Q[i,:], H rows S[k,:]
  const double* py = th;
  int sy = 0;
  if (FAMILY == 0) {
    if (rg) { py = th + nn + lane * m; sy = 1; }
  } else {
    if (rg) { py = th + nn + lane; sy = n; }
    if (rh) { py = th + nn + 2 * nm + kh; sy = m; }
  }
  const bool use_x = rg || rh;
  const bool use_y = (FAMILY == 0) ? rg : (rg || rh);
  const double s_own = zs[min(n + m + (rc ? kc : max(kh, 0)), 63)];  // s_k of a C or H row
  const double y_own = zs[min(n + max(kc, 0), 63)];                   // y_k of a C row
  double acc = 0.0;
#pragma unroll
  for (int j = 0; j < NMAX; ++j) {
    double v = 0.0;
    if (j < n) {  // x columns
      const double t = px[j * sx];
      v = use_x ? t : 0.0;
      acc = fma(v, zs[j], acc);
    } else if (j < n + m) {  // y columns
      const int q = j - n;
      const double t = py[q * sy];
      if (use_y) v = (FAMILY == 0) ? -t : t;
      if (rc && q == kc) v = s_own;  // ∂(s⊙y)/∂y = diag(s)
      const double na = fma(v, zs[j], acc);
      acc = use_y ? na : acc;
    } else if (j < N) {  // s columns
      const int q = j - n - m;
      if (rh && q == kh) v = -1.0;    // ∂(H − s)/∂s = −I
      if (rc && q == kc) v = y_own;   // ∂(s⊙y)/∂s = diag(y)
    }
    if (j == lane) v += tol;  // src/solver.jl:81 ∇F + tol*I
    a[j] = v;
    if ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);  // bound the load look-ahead
  }
  double F = 0.0;
  if (FAMILY == 0) {
    if (rg) F = acc - th[nn + nm + m + lane];                    // G = Mx − Aᵀy − ϕ
    if (rh) F = (acc - th[nn + nm + kh]) - s_own;                // H − s = (Ax − b) − s
  } else {
    if (rg) F = acc + th[nn + 2 * nm + mm + lane];               // G = Px + Qy + g
    if (rh) F = (acc + th[nn + 2 * nm + mm + n + kh]) - s_own;
  }
  if (rc) F = s_own * y_own - eps;                               // s⊙y − ϵ
  return F;
}

}  // namespace

// NC, MC > 0: compile-time (n, m) specialisation; 0: runtime n, m (N ≤ NMAX).
template <int NMAX, int FAMILY, int NC, int MC>
__global__ __launch_bounds__(64) void ipm_solve_kernel(const KernelArgs args) {
  __shared__ double zs[64];
  const int lane = threadIdx.x;
  const int64_t inst = blockIdx.x;
  const int n0 = NC ? NC : args.n, m0 = MC ? MC : args.m;
  const int n = n0, m = m0, N = n + 2 * m;
  const double* const th0 = args.theta + inst * args.theta_ld;
  const bool rx = lane < n;
  const bool ry = lane >= n && lane < n + m;
  const bool rs = lane >= n + m && lane < N;
  const double tol = args.tol;

  // src/solver.jl:39-41, 64-66: x₀ = 0, y₀ = 1, s₀ = 1 unless warm-started
  double z = 0.0;
  if (rx) z = args.x0 ? args.x0[inst * n + lane] : 0.0;
  if (ry) z = args.y0 ? args.y0[inst * m + (lane - n)] : 1.0;
  if (rs) z = args.s0 ? args.s0[inst * m + (lane - n - m)] : 1.0;

  double eps = 1.0;                    // :67
  double kkt = __builtin_huge_val();   // :68
  int status = 0;                      // :69
  int outer = 1;                       // :70
  int newton = 0;
#if MCPX_STAMPS
  uint64_t st_acc[4] = {0, 0, 0, 0};
  uint64_t st_last = __builtin_amdgcn_s_memtime();
#endif

  while (kkt > tol && eps > tol && outer < args.max_outer) {  // :71
    int inner = 1;   // :72
    status = 0;      // :73
    while (kkt > eps && inner < args.max_inner) {  // :75
      const int n = NC ? NC : opaque(n0), m = MC ? MC : opaque(m0), N = n + 2 * m;
      const double* __restrict__ th = th0 + opaque64(0);  // stays a global pointer
      const int ln = opaque_lane(lane);
      // ---- F!, ∇F_z! (:79-81) -------------------------------------------
      __syncthreads();
      zs[ln] = z;
      __syncthreads();
      double a[NMAX];
      const double F = assemble_row<NMAX, FAMILY>(th, zs, ln, n, m, eps, tol, a);
      double rhs = -F;  // :82
      // ‖F‖∞ with NaN propagation (:107), taken now, committed after the step
      const double aF = (ln < N) ? fabs(F) : 0.0;
      const bool any_nan = ballot(aF != aF) != 0ull;
      const double kkt_step = any_nan ? __builtin_nan("") : wave_max_nonneg(aF);

      MCPX_STAMP(0);
      // ---- dense LU with partial pivoting on [∇F + tol I | −F] (:81-83) --
      uint64_t rem = (N >= 64) ? ~0ull : ((1ull << N) - 1ull);
      int my_step = 1 << 30;  // LU step at which this row became a pivot row
      int pk = 0;             // ln k: pivot row of step k
      bool singular = false;
#pragma clang loop unroll(full)
      for (int k = 0; k < NMAX; ++k) {
        if (k >= N || singular) continue;  // uniform; no `break` so the loop fully unrolls
        const double ak = a[k];
        const double av = fabs(ak);
        const bool valid = ((rem >> ln) & 1ull) && !(av != av);
        const uint32_t khi = valid ? (uint32_t)__double2hiint(av) + 1u : 0u;
        const uint32_t mhi = wave_max_u32(khi);
        int p;
        if (mhi == 0u) {
          p = lowest_lane(rem);  // every remaining entry is NaN
        } else {
          const uint64_t cand = ballot(khi == mhi);
          if (__popcll(cand) == 1) {
            p = lowest_lane(cand);
          } else {  // exact tie-break on the low word, lowest ln wins
            const uint32_t klo = (khi == mhi) ? (uint32_t)__double2loint(av) : 0u;
            const uint32_t mlo = wave_max_u32(klo);
            p = lowest_lane(ballot(khi == mhi && klo == mlo));
          }
        }
        const double piv = bcast(ak, p);
        if (piv == 0.0) {  // singular: the failed linear solve of :84-88
          singular = true;
          continue;
        }
        rem &= ~(1ull << p);
        if (ln == p) my_step = k;
        if (ln == k) pk = p;
        if ((rem >> ln) & 1ull) {
          const double l = ak / piv;
          const uint64_t pm = 1ull << p;
          // columns k+1 .. NMAX-1 and the right-hand side (index NMAX), 4 per broadcast
#pragma clang loop unroll(full)
          for (int g = 0; g <= NMAX / 4; ++g) {
            if (4 * g + 3 <= k) continue;  // static: group entirely left of the pivot column
            double v[4], u[4];
#pragma clang loop unroll(full)
            for (int t = 0; t < 4; ++t) {
              const int j = 4 * g + t;
              v[t] = (j < NMAX) ? a[j < NMAX ? j : 0] : (j == NMAX ? rhs : 0.0);
            }
            bcast4(v[0], v[1], v[2], v[3], pm, u[0], u[1], u[2], u[3]);
#pragma clang loop unroll(full)
            for (int t = 0; t < 4; ++t) {
              const int j = 4 * g + t;
              if (j > k && j < NMAX) a[j < NMAX ? j : 0] = fma(-l, u[t], a[j < NMAX ? j : 0]);
              if (j == NMAX) rhs = fma(-l, u[t], rhs);
            }
          }
        }
      }
      MCPX_STAMP(1);
      if (singular) {
        status = 1;
        break;
      }
      // ---- back substitution, column oriented ----------------------------
      double dz = 0.0;
#pragma unroll
      for (int k = NMAX - 1; k >= 0; --k) {
        if (k < N) {
          const int p = __builtin_amdgcn_readlane(pk, k);
          const double t = rhs / a[k];
          const double xk = bcast(t, p);
          if (ln == k) dz = xk;
          if (my_step < k) rhs = fma(-a[k], xk, rhs);
        }
      }

      MCPX_STAMP(2);
      // ---- fraction-to-the-boundary line search (:93-100, :127-138) -----
      const bool ry = ln >= n && ln < n + m;
      const bool rs = ln >= n + m && ln < N;
      const double cv = args.c_tau * z;
      uint64_t vs = 0ull, vy = 0ull;
      double alpha = 1.0;
      for (int e = 0; e < args.n_trials; ++e) {
        const double t = alpha * dz;
        const double lhs = z + t;
        const bool viol = lhs < cv;
        if (ballot(viol && rs)) vs |= 1ull << e;
        if (ballot(viol && ry)) vy |= 1ull << e;
        alpha *= args.decay;
      }
      const int es = (~vs) ? lowest_lane(~vs) : 64;
      const int ey = (~vy) ? lowest_lane(~vy) : 64;
      if (es >= args.n_trials || ey >= args.n_trials) {  // α = NaN
        status = 1;
        break;
      }
      double as = 1.0, ay = 1.0;
      for (int e = 0; e < es; ++e) as *= args.decay;
      for (int e = 0; e < ey; ++e) ay *= args.decay;
      if (args.alpha_trace && newton < args.trace_len && ln == 0) {
        uint8_t* tr = args.alpha_trace + ((size_t)inst * args.trace_len + newton) * 2;
        tr[0] = (uint8_t)es;
        tr[1] = (uint8_t)ey;
      }
      // ---- update (:103-105; x moves with α_s) --------------------------
      const bool rx = ln < n;
      if (rx || rs) z = z + as * dz;
      if (ry) z = z + ay * dz;
      kkt = kkt_step;  // :107
      MCPX_STAMP(3);
      ++inner;         // :108
      ++newton;
    }
    eps *= (status == 0) ? args.tight[inner] : args.loose[inner];  // :111-113
    ++outer;                                                        // :114
  }
  if (outer == args.max_outer) status = 1;  // :117-119

  // ---- outputs (:121) -----------------------------------------------------
  if (rx) args.x[inst * n + lane] = z;
  if (ry) args.y[inst * m + (lane - n)] = z;
  if (rs) args.s[inst * m + (lane - n - m)] = z;
  if (args.active_mask) {
    __syncthreads();
    zs[lane] = z;
    __syncthreads();
    const uint64_t act = ballot(ry && z > zs[min(lane + m, 63)]);
    if (lane == 0) args.active_mask[inst] = act >> n;
  }
#if MCPX_STAMPS
  if (lane == 0 && args.stamps)
    for (int i = 0; i < 4; ++i) args.stamps[inst * 4 + i] = st_acc[i];
#endif
  if (lane == 0) {
    args.kkt_error[inst] = kkt;
    args.eps[inst] = eps;
    args.outer_iters[inst] = outer;
    args.status[inst] = status;
    if (args.newton_iters) args.newton_iters[inst] = newton;
  }
}

hipError_t launch_ipm(int nmax, int family, const KernelArgs& args, int64_t batch, hipStream_t stream,
                      bool allow_specialized) {
  const dim3 grid((unsigned)batch), block(64);
#define MCPX_LAUNCH(NM, FAM, NC, MC)                                                    \
  if (nmax == NM && family == FAM &&                                                  \
      (NC == 0 || (allow_specialized && args.n == NC && args.m == MC))) {              \
    hipLaunchKernelGGL((ipm_solve_kernel<NM, FAM, NC, MC>), grid, block, 0, stream, args); \
    return hipGetLastError();                                                          \
  }
  // compile-time specialisations: README QP (n=m=2), benchmark C2 (16,8), C3 (32,16)
  MCPX_LAUNCH(8, 0, 2, 2)
  MCPX_LAUNCH(32, 0, 16, 8)
  MCPX_LAUNCH(64, 0, 32, 16)
  MCPX_LAUNCH(8, 1, 2, 2)
  // generic runtime-(n, m) kernels
  MCPX_LAUNCH(8, 0, 0, 0)
  MCPX_LAUNCH(16, 0, 0, 0)
  MCPX_LAUNCH(32, 0, 0, 0)
  MCPX_LAUNCH(64, 0, 0, 0)
  MCPX_LAUNCH(8, 1, 0, 0)
  MCPX_LAUNCH(16, 1, 0, 0)
  MCPX_LAUNCH(32, 1, 0, 0)
  MCPX_LAUNCH(64, 1, 0, 0)
#undef MCPX_LAUNCH
  return hipErrorInvalidValue;
}

}  // namespace mcpx
