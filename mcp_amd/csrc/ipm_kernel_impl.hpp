// ipm_kernel_impl.hpp — gfx950 (CDNA4) kernel templates of the batched interior-point
// MCP solver.  Instantiated by ipm_inst_*.hip (one translation unit per kernel
// group so the build compiles them in parallel).
//
// One 64-lane wavefront solves one MCP instance end to end: the whole
// ϵ-continuation / Newton loop of the reference, src/solver.jl:64-121, runs on
// the device with no host round trip.  Lane i owns row i of the Newton system
// (∇F + tol·I) δz = −F (src/mcp.jl:76-120, src/solver.jl:81-82):
//
//  * RED (default, MCPX_LINSOLVE_REDUCED): the slack block is eliminated
//    exactly first — ∂(s⊙y − ϵ)/∂s = Y + tol·I is diagonal for every MCP of the
//    reference's form — so lanes [0, n) hold x-rows (G) and lanes [n, n+m)
//    hold y-rows (H − s) together with y_k and s_k; the system is (n+m)-dim.
//  * DENSE (MCPX_LINSOLVE_DENSE): lanes [0, n+2m) hold the rows of the full
//    system, z = [x; y; s] one entry per lane.
//
// The Newton system (src/solver.jl:81-90, UMFPACK in the reference) is solved
// by a register-resident dense LU with partial pivoting on the augmented
// matrix [K | rhs]: rows stay in their lanes (NMAX fp64 VGPRs each); the pivot
// search is a 32-bit DPP max over the high word of |a_ik| with exact two-phase
// tie resolution on the low word; the pivot row is broadcast through SGPRs
// (EXEC-masked v_readfirstlane, bcast_group.inc, ≤16 columns per EXEC switch)
// and every remaining lane eliminates with v_fma_f64.  Back substitution is
// column-oriented.  The fraction-to-the-boundary line search
// (src/solver.jl:127-138) evaluates every trial step α = decayᵉ at once (one
// ballot per e) and takes the first all-clear e.
//
// Arithmetic is the contract of oracle/ipm_oracle.c (same op order, explicit
// fma, -ffp-contract=off), so results are bit-identical to the CPU oracle.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "ipm_kernel.h"

// A DPP read of a VGPR needs 2 wait states after a VALU write of it, and hipcc
// does not pad hazards whose reader is inside an asm statement: a register copy
// it places right before a DPP fmac would feed the fmac a stale source
// (tools/check_dpp_hazards.py finds them in the .s, and the build refuses such
// an object).  The DPP fmacs of the Gauss-Jordan take a PAD template flag: the
// compile-time-(n, m) kernels run unpadded (the checker passes them; the pads
// cost 2-3 % at C3, profiles/r02/ab_c3_pad_waves.jsonl), the generic kernels,
// where the allocator does place copies right before the asm, keep an
// s_nop 1 per fmac.  MCPX_DPP_PAD_ON=1 pads every kernel.
#ifndef MCPX_DPP_PAD_ON
#define MCPX_DPP_PAD_ON 0
#endif

// SCHUR kernels with compile-time (n, m) keep A, b, ϕ in LDS (A/B knob).
#ifndef MCPX_LDS_A
#define MCPX_LDS_A 1
#endif

// SCHUR kernels with compile-time n ≤ 16 (C2) keep M in LDS as well (A/B knob): its 2 KB per
// wave fit beside A at the occupancy those kernels run at, and the residual's and the Schur
// accumulator's M reads stop paying an L2 round trip (C2 +3 to +6 %, ab_c2_lds_m.jsonl).
#ifndef MCPX_LDS_M
#define MCPX_LDS_M 1
#endif

// kkt and ϵ re-read into SGPRs after each update (A/B knob).
#ifndef MCPX_SREG_KKT
#define MCPX_SREG_KKT 0
#endif

// θ loads in flight per lane in the SCHUR residual dot products (A/B knob).
#ifndef MCPX_RES_BATCH
#define MCPX_RES_BATCH 8
#endif

// Waves per SIMD the register allocator targets in the SCHUR fast pass (A/B knob).
#ifndef MCPX_FAST_WAVES
#define MCPX_FAST_WAVES 5
#endif

// Dispatch-order priority levels (A/B knob; 0 = off): see ipm_solve_kernel.
#ifndef MCPX_AFF_LDS_R
#define MCPX_AFF_LDS_R 1
#endif
#ifndef MCPX_PRIO
#define MCPX_PRIO 0
#endif

// Diagnostic phase stamps (tools/phase_profile.hip builds with MCPX_STAMPS=1;
// the product build compiles them away).
#ifndef MCPX_STAMPS
#define MCPX_STAMPS 0
#endif
#define MCPX_NSTAMP 6  // residuals | ‖F‖∞ + rr | Schur form | LU / GJ | back-substitution | line search + update
// MCPX_STAMPS=2 (tools/timeline.hip): the wave's start and end on the 100 MHz constant clock
// and where it ran (HW_ID, XCC_ID) instead — the residency timeline of a launch.
#if MCPX_STAMPS == 1
#define MCPX_STAMP(i)                                 \
  do {                                                \
    const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    st_acc[i] += t_ - st_last;                        \
    st_last = t_;                                     \
  } while (0)
#else
#define MCPX_STAMP(i) \
  do {                \
  } while (0)
#endif

namespace mcpx {

namespace {

#include "bcast_group.inc"

__device__ __forceinline__ double bcast(double v, int src) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), src);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), src);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

__device__ __forceinline__ int lowest_lane(uint64_t mask) { return __ffsll((unsigned long long)mask) - 1; }

// Hides a uniform value from the optimiser for one loop iteration so that the
// ~3·NMAX uniform predicates derived from it (j < n, k < N, …) are recomputed
// where used instead of being hoisted out of the Newton loop and kept live in
// SGPRs (which spills them into VGPR lanes).
__device__ __forceinline__ int opaque(int v) {
  asm volatile("" : "+s"(v));
  return v;
}
// Same for an offset on the θ pointer and for the lane index: keeps the NMAX
// per-lane θ addresses of the Jacobian assembly from being hoisted out of the
// Newton loop (they would occupy 2·NMAX registers for the whole solve).
__device__ __forceinline__ int64_t opaque64(int64_t v) {
  asm volatile("" : "+s"(v));
  return v;
}
__device__ __forceinline__ int opaque_lane(int v) {
  asm volatile("" : "+v"(v));
  return v;
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

// Exact wave max of non-negative, non-NaN doubles (bit patterns are monotone).
__device__ __forceinline__ double wave_max_nonneg(double v) {
  const uint32_t hi = (uint32_t)__double2hiint(v);
  const uint32_t lo = (uint32_t)__double2loint(v);
  const uint32_t mhi = wave_max_u32(hi);
  const uint32_t mlo = wave_max_u32(hi == mhi ? lo : 0u);
  return __hiloint2double((int)mhi, (int)mlo);
}

// 1 / b, correctly rounded (== the IEEE quotient the oracle's C division takes),
// for a wave-uniform b.  The compiler's f64 division is v_div_scale ×2, v_rcp,
// two Newton steps, a product, the remainder, v_div_fmas and v_div_fixup: 11
// VALU instructions.  For 2⁻⁵⁰⁰ ≤ |b| ≤ 2⁵⁰⁰ (numerator 1) the scales are the
// identity, v_div_fmas is a plain fma and v_div_fixup returns its input, so the
// same chain without them (7 instructions) gives the same bits; other b (0,
// subnormal, huge, Inf, NaN) take the full division.  The test is on the SGPR
// copy of b, so the branch is scalar.
__device__ __forceinline__ bool rcp_fast_ok(double b) {
  const uint32_t e = ((uint32_t)__double2hiint(b) >> 20) & 0x7ffu;  // biased exponent
  return e - 523u <= 1000u;
}
// The 7-instruction chain alone: == 1.0 / b whenever rcp_fast_ok(b).
__device__ __forceinline__ double rcp_fast(double b) {
  double y = __builtin_amdgcn_rcp(b);
  double t = fma(-b, y, 1.0);
  y = fma(y, t, y);
  t = fma(-b, y, 1.0);
  y = fma(y, t, y);
  t = fma(-b, y, 1.0);  // remainder of the quotient 1·y
  return fma(t, y, y);
}
__device__ __forceinline__ double rcp_uniform(double b) {
  if (__builtin_expect(rcp_fast_ok(b), 1)) return rcp_fast(b);
  return 1.0 / b;
}

// A wave-uniform double moved to SGPRs (readfirstlane of both halves): keeps loop-carried
// uniform values (kkt, ϵ) out of the VGPR budget.
__device__ __forceinline__ double uniform_f64(double v) {
  const int lo = __builtin_amdgcn_readfirstlane(__double2loint(v));
  const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
  return __hiloint2double(hi, lo);
}

// NaN-propagating max (Julia `max`, as in norm(F, Inf), src/solver.jl:107)
__device__ __forceinline__ double max_nan(double a, double b) { return (a != a || b != b) ? a + b : fmax(a, b); }

// Row `lane` of F and of ∇F_z + tol·I (DENSE) or of the slack-eliminated
// system (RED), src/mcp.jl:72-120.  `zs` is the wave's copy of z in LDS:
// zs[j] = x_j (j < n), zs[n+q] = y_q, and for DENSE zs[n+m+q] = s_q.
// `s_own` is s_k of a RED y-row.  Same op order as family_row() and the slack
// elimination of oracle/ipm_oracle.c.  Every lane streams its row of θ
// through one per-lane base pointer and stride per column block (no
// per-column branches); lanes that read nothing in a block get stride 0 on a
// valid address and a masked value.
template <int NMAX, int FAMILY, bool RED, bool CT>
__device__ __forceinline__ void assemble_row(const double* __restrict__ th, const double* zs, int lane, int n,
                                             int m, double eps, double tol, double s_own, double (&a)[NMAX],
                                             double& F, double& Fc, double& rhs, double& w) {
  const int N = RED ? n + m : n + 2 * m;
  const bool rg = lane < n;                           // G rows
  const bool rh = lane >= n && lane < n + m;          // H − s rows
  const bool rc = !RED && lane >= n + m && lane < N;  // s⊙y − ϵ rows (DENSE only)
  const int kh = lane - n;                            // H row index
  const int kc = lane - n - m;                        // complementarity index (DENSE)
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
  // s_k / y_k of this row's complementarity pair
  const double s_k = RED ? s_own : zs[min(n + m + (rc ? kc : max(kh, 0)), 63)];
  const double y_k = zs[min(n + (RED ? max(kh, 0) : max(kc, 0)), 63)];
  // RED: pivot w_k = y_k + tol of the eliminated δs_k and the Schur term d_k = s_k / w_k
  w = y_k + tol;
  const double d = (RED && rh) ? s_k / w : 0.0;
  double acc = 0.0;
  if constexpr (CT) {
    // Compile-time (n, m): branch-free over columns, so the compiler batches
    // the θ loads of neighbouring columns.  Every lane issues one load per
    // column from a valid address and masks the value.
#pragma unroll
    for (int j = 0; j < NMAX; ++j) {
      const int q = j - n, qs = q - m;  // column class, folded at compile time
      const bool cx = q < 0;
      const bool cy = q >= 0 && q < m;
      const bool cs = !RED && qs >= 0 && qs < m;
      const double* pa = cx ? px + j * sx : (cy ? py + q * sy : th);
      const double t = *pa;
      const double zj = zs[j];
      double v = 0.0;
      v = (cx && use_x) ? t : v;
      v = (cy && use_y) ? ((FAMILY == 0) ? -t : t) : v;
      v = (cy && rc && q == kc) ? s_k : v;   // ∂(s⊙y)/∂y = diag(s)
      v = (cs && rh && qs == kh) ? -1.0 : v; // ∂(H − s)/∂s = −I
      v = (cs && rc && qs == kc) ? y_k : v;  // ∂(s⊙y)/∂s = diag(y)
      const double na = fma(v, zj, acc);
      acc = (cx || (cy && use_y)) ? na : acc;
      if (j == lane) {
        v += tol;                 // src/solver.jl:81 ∇F + tol*I
        if (RED && rh) v += d;    // + s_k / w_k from the slack elimination
      }
      a[j] = v;
      if ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);  // bound the load look-ahead
    }
  } else {
    // Runtime (n, m): per-column uniform branches keep the register pressure
    // of the generic kernels low (a branch-free stream raises it by ~60 VGPRs).
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
        if (rc && q == kc) v = s_k;  // ∂(s⊙y)/∂y = diag(s)
        const double na = fma(v, zs[j], acc);
        acc = use_y ? na : acc;
      } else if (!RED && j < N) {  // s columns (DENSE)
        const int q = j - n - m;
        if (rh && q == kh) v = -1.0;  // ∂(H − s)/∂s = −I
        if (rc && q == kc) v = y_k;   // ∂(s⊙y)/∂s = diag(y)
      }
      if (j == lane) {
        v += tol;               // src/solver.jl:81 ∇F + tol*I
        if (RED && rh) v += d;  // + s_k / w_k from the slack elimination
      }
      a[j] = v;
      if ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);
    }
  }
  F = 0.0;
  if (FAMILY == 0) {
    if (rg) F = acc - th[nn + nm + m + lane];           // G = Mx − Aᵀy − ϕ
    if (rh) F = (acc - th[nn + nm + kh]) - s_k;         // H − s = (Ax − b) − s
  } else {
    if (rg) F = acc + th[nn + 2 * nm + mm + lane];      // G = Px + Qy + g
    if (rh) F = (acc + th[nn + 2 * nm + mm + n + kh]) - s_k;
  }
  Fc = 0.0;
  if (RED) {
    if (rh) {  // exact elimination of δs_k: rhs_H = −F_H − F_C / w_k
      Fc = s_k * y_k - eps;
      rhs = (-F) - (Fc / w);
    } else {
      rhs = -F;
    }
  } else {
    if (rc) F = s_k * y_k - eps;  // s⊙y − ϵ
    rhs = -F;
  }
}

// a[j] ← fma(−l, u_j, a[j]) for j in (k, NMAX) and rhs ← fma(−l, u_rhs, rhs) in
// the lanes where `upd` holds, where u is the row held by the lane in `pm`,
// broadcast through SGPRs in groups of ≤16 columns (bcast_group.inc).
//
// The broadcast runs in uniform control flow (full EXEC) and only the fmas are
// predicated.  The asm switches EXEC to the pivot lane and reads its VGPRs; the
// pivot lane is never among the updated lanes, so under a compiler-narrowed EXEC
// any copy the compiler places into the asm's input registers (a reload of a
// spilled a[j] from an AGPR, a register move) would skip the pivot lane and the
// asm would broadcast a stale value.  That is what the ×5-unrolled C4 Schur
// formation did; tools/check_dpp_hazards.py rejects the pattern.
template <int NMAX>
__device__ __forceinline__ void eliminate_row(double (&a)[NMAX], double& rhs, int k, double l, uint64_t pm,
                                              bool upd) {
  constexpr int G = 16;  // columns per EXEC-masked broadcast (8: 2-4 % slower on C4, r02 A/B)
  // columns k+1 .. NMAX-1 and the right-hand side (index NMAX)
#pragma clang loop unroll(full)
  for (int g = 0; g <= NMAX / G; ++g) {
    const int lo = max(G * g, k + 1);        // static after unrolling
    const int hi = min(G * g + G, NMAX + 1);  // exclusive
    if (lo >= hi) continue;
    const int cnt = hi - lo;  // 1..16
    double v[16], u[16];
#pragma clang loop unroll(full)
    for (int t = 0; t < 16; ++t) {
      const int j = lo + t;
      v[t] = (t < cnt) ? ((j < NMAX) ? a[j < NMAX ? j : 0] : rhs) : 0.0;
    }
    bcast_n(cnt, v, pm, u);
    if (upd) {
#pragma clang loop unroll(full)
      for (int t = 0; t < 16; ++t) {
        const int j = lo + t;
        if (t < cnt && j < NMAX) a[j < NMAX ? j : 0] = fma(-l, u[t], a[j < NMAX ? j : 0]);
        if (t < cnt && j == NMAX) rhs = fma(-l, u[t], rhs);
      }
    }
  }
}

// Dense LU with partial pivoting of the rows held in lanes [0, N) plus the
// augmented right-hand side, then column-oriented back substitution.  On
// success returns true and the solution entry of column `ln` in dz; returns
// false if a pivot is exactly 0.  Measured on the lone-wave lane-change LU (r02):
// a pivot-row broadcast through LDS instead of SGPRs was 24 % slower (30-45 % in a
// second A/B, profiles/r02/ab_c4_lu_variants.txt), and a
// look-ahead that starts step k+1's pivot search right after updating column k+1
// (to overlap its DPP chain with the rest of the update) 4 % slower.
//
// Guessed pivots (`spec`, the nonlinear SCHUR kernel): lane k of `pk` holds on entry
// the pivot row of step k of an earlier factorisation (the previous Newton step's).
// Step k then skips the pivot search and only checks, lane by lane, that the
// first-max rule above would have picked the guessed row; the arithmetic is the
// searched LU's, so when every check holds the bits are the same.  A failed check,
// or a guessed pivot that is 0 or NaN (singular / all-NaN cases the search decides),
// sets `miss`: the caller restores the rows and runs the search.
#ifndef MCPX_LU_NO_SPEC
#define MCPX_LU_NO_SPEC 0
#endif
// RCP (the SCHUR step of generated nonlinear modules, oracle lu_solve_x rcp = 2): Gauss-Jordan
// with the same pivot search — multipliers a_ik · (1 / piv), one correctly rounded reciprocal
// (rcp_uniform) per pivot, every row but the pivot row updated, the pivot row with
// multiplier +0 (l = −0: fma(+0, u, a)) — and x_k = b_p · (1 / u_pk), no back substitution.
template <int NMAX, bool RCP = false>
__device__ __forceinline__ bool lu_solve_rows_core(double (&a)[NMAX], double rhs, int N, int ln, double& dz,
                                                   int& pk, bool spec, bool& miss) {
  uint64_t rem = (N >= 64) ? ~0ull : ((1ull << N) - 1ull);
  int my_step = 1 << 30;  // LU step at which this row became a pivot row
  bool singular = false;
  bool viol = false;  // spec: a remaining row beats the guessed pivot under the first-max rule
  double rcpd = 1.0;  // RCP: lane k holds 1 / u_kk of step k
  miss = false;
#pragma clang loop unroll(full)
  for (int k = 0; k < NMAX; ++k) {
    if (k >= N || singular) continue;  // uniform; no `break` so the loop fully unrolls
    const double ak = a[k];
    const double av = fabs(ak);
    int p;
    double piv;
    if (spec && !MCPX_LU_NO_SPEC) {
      p = __builtin_amdgcn_readlane(pk, k);
      piv = bcast(ak, p);
      const double ap = fabs(piv);
      if (!(ap > 0.0)) {  // 0 or NaN: let the search decide
        miss = true;
        singular = true;
        continue;
      }
      // NaN entries never win the search (av > ap is false for them); bitwise, no branches
      const bool beats = (av > ap) | ((av == ap) & (ln < p));
      viol = viol | ((((rem >> ln) & 1ull) != 0) & (ln != p) & beats);
    } else {
      const bool valid = ((rem >> ln) & 1ull) && !(av != av);
      const uint32_t khi = valid ? (uint32_t)__double2hiint(av) + 1u : 0u;
      const uint32_t mhi = wave_max_u32(khi);
      if (mhi == 0u) {
        p = lowest_lane(rem);  // every remaining entry is NaN
      } else {
        const uint64_t cand = ballot(khi == mhi);
        if (__popcll(cand) == 1) {
          p = lowest_lane(cand);
        } else {  // exact tie-break on the low word, lowest lane wins
          const uint32_t klo = (khi == mhi) ? (uint32_t)__double2loint(av) : 0u;
          const uint32_t mlo = wave_max_u32(klo);
          p = lowest_lane(ballot(khi == mhi && klo == mlo));
        }
      }
      piv = bcast(ak, p);
      if (piv == 0.0) {  // singular: the failed linear solve of src/solver.jl:84-88
        singular = true;
        continue;
      }
    }
    rem &= ~(1ull << p);
    if (ln == p) my_step = k;
    if (ln == k) pk = p;
    double l;
    if constexpr (RCP) {
      const double rp = rcp_uniform(piv);
      if (ln == p) rcpd = rp;
      l = (ln == p) ? -0.0 : ak * rp;  // Gauss-Jordan: the pivot row takes fma(+0, u, a)
      eliminate_row<NMAX>(a, rhs, k, l, 1ull << p, true);
    } else {
      l = ak / piv;
      eliminate_row<NMAX>(a, rhs, k, l, 1ull << p, (rem >> ln) & 1ull);
    }
  }
  if (spec && ballot(viol)) miss = true;
  if (singular || miss) return false;
  if constexpr (RCP) {  // x_k = b_p · (1 / u_pk) in lane p = pk of lane k
    const double xp = rhs * rcpd;
    const int lo = __builtin_amdgcn_ds_bpermute(pk << 2, __double2loint(xp));
    const int hi = __builtin_amdgcn_ds_bpermute(pk << 2, __double2hiint(xp));
    dz = __hiloint2double(hi, lo);
    return true;
  }
  dz = 0.0;
#pragma clang loop unroll(full)
  for (int k = NMAX - 1; k >= 0; --k) {
    if (k < N) {
      const int p = __builtin_amdgcn_readlane(pk, k);
      const double xk = bcast(rhs / a[k], p);
      if (ln == k) dz = xk;
      if (my_step < k) rhs = fma(-a[k], xk, rhs);
    }
  }
  return true;
}

template <int NMAX>
__device__ __forceinline__ bool lu_solve_rows(double (&a)[NMAX], double rhs, int N, int ln, double& dz) {
  int pk = 0;
  bool miss;
  return lu_solve_rows_core<NMAX>(a, rhs, N, ln, dz, pk, false, miss);
}

typedef double d4 __attribute__((ext_vector_type(4)));

// acc ← fma chain over j < cnt of (±p[j·st]) · q[j], q in LDS.  The global
// loads are issued BATCH at a time from clamped (always valid) addresses and
// consumed afterwards, so a batch pays one memory latency instead of BATCH
// (a plain loop compiles to load → s_waitcnt vmcnt(0) → fma per element).
template <int BATCH, bool NEG>
__device__ __forceinline__ double dot_strided(const double* __restrict__ p, int st, const double* q, int cnt,
                                              double acc) {
  for (int j0 = 0; j0 < cnt; j0 += BATCH) {
    double t[BATCH];
#pragma unroll
    for (int b = 0; b < BATCH; ++b) t[b] = p[min(j0 + b, cnt - 1) * st];
#pragma unroll
    for (int b = 0; b < BATCH; ++b)
      if (j0 + b < cnt) acc = fma(NEG ? -t[b] : t[b], q[j0 + b], acc);
    __builtin_amdgcn_sched_barrier(0);  // at most BATCH loads in flight (register budget)
  }
  return acc;
}

#ifndef MCPX_RES_INC
#define MCPX_RES_INC 1
#endif
// dot_strided (NEG = false) with the addresses formed by a running pointer, one 64-bit add
// per element (the empty asm keeps the compiler from re-deriving p + j·st with a multiply).
// The residual's M·x | A·x reads a lane-dependent pointer and stride (M column in θ, A row
// in LDS); from p + j·st the compiler spent a multiply, a shift and a 64-bit add on each
// element (≈ 96 VALU a Newton step at C3), here one add (MCPX_RES_INC; same loads, same
// bits; C3 8,192: 12.56 against 12.21 M solves/s, profiles/r05/ab_res_inc.jsonl).
template <int BATCH>
__device__ __forceinline__ double dot_strided_inc(const double* __restrict__ p, int st, const double* q, int cnt,
                                                  double acc) {
  const int64_t sb = (int64_t)st * 8;
  const char* pc = (const char*)p;
  for (int j0 = 0; j0 < cnt; j0 += BATCH) {
    double t[BATCH];
#pragma unroll
    for (int b = 0; b < BATCH; ++b) {
      t[b] = *(const double*)pc;
      if (j0 + b + 1 < cnt) pc += sb;  // the last element repeats (clamped, always valid)
      asm volatile("" : "+v"(pc));
    }
#pragma unroll
    for (int b = 0; b < BATCH; ++b)
      if (j0 + b < cnt) acc = fma(t[b], q[j0 + b], acc);
    __builtin_amdgcn_sched_barrier(0);  // at most BATCH loads in flight (register budget)
  }
  return acc;
}

// SCHUR path (QP family, and the affine family with ∂H/∂y ≡ 0), part 1: residuals.
// x-lanes compute F_G, y-lanes (which also own s_k) F_H and F_C; same fma order as
// family_row() of the oracle.  `ta` is the H-side coupling (QP: A; affine: R) with
// leading dimension `lda` (A_ki = ta[i·lda + k]); `tq` / `ldq` the G-side coupling
// negated in the same layout (QP: A again, since ∂G/∂y = −Aᵀ; affine: −Qᵀ); `tb` the
// constants b then ϕ (affine: −h then −g, so that acc − b = acc + h bit for bit).
// QP: θ itself (lda = m) or the wave's LDS copy, tq = ta, tb = ta + n·lda.
template <int BATCH>
__device__ __forceinline__ void qp_residuals(const double* __restrict__ th, const double* ta, int lda,
                                             const double* tq, int ldq, const double* tb, const double* zs,
                                             int ln, int n, int m, double eps, double s_own, double& F, double& Fc) {
  const bool rg = ln < n, rh = ln >= n && ln < n + m;
  const int kh = ln - n;
  const double* px = rg ? th + ln : (rh ? ta + kh : th);  // M column (θ) | A row
  const int sx = rg ? n : (rh ? lda : 0);
  double acc = MCPX_RES_INC ? dot_strided_inc<BATCH>(px, sx, zs, n, 0.0)   // M_ij x_j  |  A_kj x_j
                            : dot_strided<BATCH, false>(px, sx, zs, n, 0.0);
  const double acc_y = dot_strided<BATCH, true>(tq + (rg ? ln * ldq : 0), 1, zs + n, m, acc);  // − A_ki y_k
  if (rg) acc = acc_y;
  F = 0.0;
  Fc = 0.0;
  if (rg) F = acc - tb[m + ln];                                 // G = Mx − Aᵀy − ϕ
  if (rh) {
    F = (acc - tb[kh]) - s_own;                                 // H − s
    Fc = s_own * zs[n + kh] - eps;                              // s⊙y − ϵ
  }
}

// ---- 2-D Gauss-Jordan on the matrix-core output layout (SCHUR, SPD) --------
//
// The Schur complement is formed transposed on the matrix cores (the A fragment
// carries A_kj / D_k, the B fragment A_ki, the accumulator starts at Mᵀ), so
// that accumulator tile (I, J), element r of lane (lr, lc) = (l >> 4, l & 15)
// holds S[16J + lc][16I + lr + 4r]: lane (lr, lc) owns rows lc + 16J of S at
// the columns ≡ lr (mod 4), and every DPP row of 16 lanes holds all rows.
// (fma(a, b, c) = fma(b, a, c), so every entry is bit-identical to the oracle's
// S_ij chain.)  In this layout a Gauss-Jordan step needs the pivot row's entry
// of the lane's own column — one DPP row_newbcast source operand of the fma —
// and two row multipliers per lane, moved across DPP rows with
// v_permlane16/32_swap.  Compared with the lane-per-row layout this replaces
// two v_readfirstlane + one fma per element by one v_fmac_f64_dpp, keeps S in
// NT²·8 instead of 32·NT·2 VGPRs, and needs no LDS round trip of the tile.

// v from DPP row Q (lanes 16Q .. 16Q+15) in every DPP row, lane position kept:
// v_permlane16_swap replicates the even / odd DPP rows, v_permlane32_swap the
// lower / upper half (semantics checked by tools/ubench_lanes.hip).  Written as
// inline asm so that it stays ordered after the asm fmacs of the previous step
// (FIRST: the step right after the MFMAs, whose results need wait states before
// a VALU read that the compiler cannot see through the asm).
template <int Q, bool FIRST>
__device__ __forceinline__ double from_dpp_row(double v) {
  unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  unsigned a0, a1, b0, b1, c0, c1, d0, d1;
#define MCPX_PL_STAGE1(SEL_LO, SEL_HI)                                                     \
  "v_mov_b32 %0, %8\n v_mov_b32 %1, %8\n v_mov_b32 %2, %9\n v_mov_b32 %3, %9\n s_nop 1\n" \
  "v_permlane16_swap_b32 %0, %1\n v_permlane16_swap_b32 %2, %3\n s_nop 1\n"              \
  "v_mov_b32 %4, " SEL_LO "\n v_mov_b32 %5, " SEL_LO "\n"                                \
  "v_mov_b32 %6, " SEL_HI "\n v_mov_b32 %7, " SEL_HI "\n s_nop 1\n"                     \
  "v_permlane32_swap_b32 %4, %5\n v_permlane32_swap_b32 %6, %7\n s_nop 1"
#define MCPX_PL_ASM(PRE, SEL_LO, SEL_HI)                                                   \
  asm volatile(PRE MCPX_PL_STAGE1(SEL_LO, SEL_HI)                                          \
               : "=&v"(a0), "=&v"(a1), "=&v"(b0), "=&v"(b1), "=&v"(c0), "=&v"(c1), "=&v"(d0), \
                 "=&v"(d1)                                                                 \
               : "v"(lo), "v"(hi))
  if (FIRST) {
    if (Q & 1) MCPX_PL_ASM("s_nop 7\n s_nop 7\n s_nop 7\n", "%1", "%3");
    else MCPX_PL_ASM("s_nop 7\n s_nop 7\n s_nop 7\n", "%0", "%2");
  } else {
    if (Q & 1) MCPX_PL_ASM("", "%1", "%3");
    else MCPX_PL_ASM("", "%0", "%2");
  }
#undef MCPX_PL_ASM
#undef MCPX_PL_STAGE1
  // c0/d0: lower half replicated (Q < 2), c1/d1: upper half replicated (Q ≥ 2)
  return (Q & 2) ? __hiloint2double((int)d1, (int)c1) : __hiloint2double((int)d0, (int)c0);
}

// (v_permlane*_swap reads its operands 2 wait states after a VALU write at the
// earliest: the s_nop 1 ahead of each swap in the asm blocks.)
//
// NT = 2: both row halves' negated multipliers with ONE multiplication by the
// pivot's reciprocal rp (computed from the pivot alone, so its division runs
// beside the column distribution instead of after it).  v0 / v1 = the pivot
// column entries of half 0 / 1, valid in DPP row Q.  permlane32_swap puts half
// 0's values in the lower and half 1's in the upper 32 lanes (same DPP-row
// offset), permlane16_swap then spreads DPP row Q within each half, so lane l
// holds w = a_{16·(l≥32) + lc, k}; one product gives t = −w · rp, and a final
// permlane32_swap hands every lane both t's (lower → half 0, upper → half 1).
template <int Q, bool FIRST>
__device__ __forceinline__ void col_quot_nt2(double v0, double v1, double rp, double& q0, double& q1) {
  const unsigned a0 = (unsigned)__double2loint(v0), a1 = (unsigned)__double2hiint(v0);
  const unsigned b0 = (unsigned)__double2loint(v1), b1 = (unsigned)__double2hiint(v1);
  unsigned x0, y0, z0, x1, y1, z1;  // per dword (0 = low, 1 = high)
  // rows 0/1 of half 0 and 1 end up in x (Q < 2), rows 2/3 in y (Q ≥ 2); after the
  // 16-swap the selected register holds the even DPP rows replicated, z the odd ones.
  // Both dword chains interleaved, so each swap's wait states overlap the other's.
#define MCPX_NT2_ASM(PRE, S0, S1)                                                                      \
  asm volatile(PRE "v_mov_b32 %0, %6\n v_mov_b32 %1, %7\n v_mov_b32 %3, %8\n v_mov_b32 %4, %9\n"     \
               "s_nop 1\n v_permlane32_swap_b32 %0, %1\n v_permlane32_swap_b32 %3, %4\n s_nop 0\n"   \
               "v_mov_b32 %2, " S0 "\n v_mov_b32 %5, " S1 "\n s_nop 1\n"                              \
               "v_permlane16_swap_b32 " S0 ", %2\n v_permlane16_swap_b32 " S1 ", %5\n s_nop 1"         \
               : "=&v"(x0), "=&v"(y0), "=&v"(z0), "=&v"(x1), "=&v"(y1), "=&v"(z1)                     \
               : "v"(a0), "v"(b0), "v"(a1), "v"(b1))
  if (FIRST) {  // right after the MFMAs: their results need more wait states before a VALU read
    if (Q < 2) MCPX_NT2_ASM("s_nop 7\n s_nop 7\n s_nop 7\n", "%0", "%3");
    else MCPX_NT2_ASM("s_nop 7\n s_nop 7\n s_nop 7\n", "%1", "%4");
  } else {
    if (Q < 2) MCPX_NT2_ASM("", "%0", "%3");
    else MCPX_NT2_ASM("", "%1", "%4");
  }
#undef MCPX_NT2_ASM
  const unsigned w0 = (Q & 1) ? z0 : ((Q < 2) ? x0 : y0);
  const unsigned w1 = (Q & 1) ? z1 : ((Q < 2) ? x1 : y1);
  const double t = (-__hiloint2double((int)w1, (int)w0)) * rp;  // −l = (−w)·(1/piv), exact negation
  const unsigned tl = (unsigned)__double2loint(t), thi = (unsigned)__double2hiint(t);
  const auto pl = __builtin_amdgcn_permlane32_swap(tl, tl, false, false);
  const auto ph = __builtin_amdgcn_permlane32_swap(thi, thi, false, false);
  q0 = __hiloint2double((int)ph[0], (int)pl[0]);  // lower half replicated: half 0
  q1 = __hiloint2double((int)ph[1], (int)pl[1]);  // upper half replicated: half 1
}

// acc ← fma(nl, u, acc), u = lane (16·row + R)'s `src` (DPP row_newbcast:R).
// The DPP source is the pivot row, last written one step earlier: the column
// distribution and the multiplication lie between (≥ 2 wait states) unless the
// compiler copies it right before the asm (PAD: s_nop 1 first).
#define MCPX_FMAC_NB(R)                                                                                     \
  case R:                                                                                                   \
    if (pad)                                                                                                \
      asm volatile("s_nop 1\n v_fmac_f64_dpp %0, %1, %2 row_newbcast:" #R " row_mask:0xf bank_mask:0xf"    \
                   : "+v"(acc) : "v"(src), "v"(nl));                                                        \
    else                                                                                                    \
      asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:" #R " row_mask:0xf bank_mask:0xf"               \
                   : "+v"(acc) : "v"(src), "v"(nl));                                                        \
    break;
template <int R, bool PAD>
__device__ __forceinline__ void fmac_row_bcast(double& acc, double src, double nl) {
  const bool pad = PAD || MCPX_DPP_PAD_ON;
  switch (R) {
    MCPX_FMAC_NB(0) MCPX_FMAC_NB(1) MCPX_FMAC_NB(2) MCPX_FMAC_NB(3) MCPX_FMAC_NB(4) MCPX_FMAC_NB(5)
    MCPX_FMAC_NB(6) MCPX_FMAC_NB(7) MCPX_FMAC_NB(8) MCPX_FMAC_NB(9) MCPX_FMAC_NB(10) MCPX_FMAC_NB(11)
    MCPX_FMAC_NB(12) MCPX_FMAC_NB(13) MCPX_FMAC_NB(14) MCPX_FMAC_NB(15)
  }
}
#undef MCPX_FMAC_NB

// Same with the destination as its own DPP source (the pivot half; a DPP read
// happens before the write, so every lane sees the pivot lane's old value).
#define MCPX_FMAC_NB_SELF(R)                                                                                \
  case R:                                                                                                   \
    if (pad)                                                                                                \
      asm volatile("s_nop 1\n v_fmac_f64_dpp %0, %0, %1 row_newbcast:" #R " row_mask:0xf bank_mask:0xf"    \
                   : "+v"(acc) : "v"(nl));                                                                  \
    else                                                                                                    \
      asm volatile("v_fmac_f64_dpp %0, %0, %1 row_newbcast:" #R " row_mask:0xf bank_mask:0xf"               \
                   : "+v"(acc) : "v"(nl));                                                                  \
    break;
template <int R, bool PAD>
__device__ __forceinline__ void fmac_row_bcast_self(double& acc, double nl) {
  const bool pad = PAD || MCPX_DPP_PAD_ON;
  switch (R) {
    MCPX_FMAC_NB_SELF(0) MCPX_FMAC_NB_SELF(1) MCPX_FMAC_NB_SELF(2) MCPX_FMAC_NB_SELF(3) MCPX_FMAC_NB_SELF(4)
    MCPX_FMAC_NB_SELF(5) MCPX_FMAC_NB_SELF(6) MCPX_FMAC_NB_SELF(7) MCPX_FMAC_NB_SELF(8) MCPX_FMAC_NB_SELF(9)
    MCPX_FMAC_NB_SELF(10) MCPX_FMAC_NB_SELF(11) MCPX_FMAC_NB_SELF(12) MCPX_FMAC_NB_SELF(13)
    MCPX_FMAC_NB_SELF(14) MCPX_FMAC_NB_SELF(15)
  }
}
#undef MCPX_FMAC_NB_SELF

// Transposed Schur complement in the 2-D layout (see above).  acc[I][J][r].
// `ta` / `lda`: the A block as in qp_residuals.  TWO (affine family): the B fragment
// comes from the negated G-side coupling tq / ldq (−Q_ik) instead of A_ki, so the
// entries are S_ij = P_ij + Σ_k (−Q_ik)·(R_kj·D_k⁻¹) — the oracle's chain for either family.
template <int NT, bool TWO = false>
__device__ __forceinline__ void qp_schur_form_2d(const double* __restrict__ th, const double* ta, int lda,
                                                 const double* sD, int ln, int n, int m, double tol,
                                                 d4 (&acc)[NT][NT], const double* tq = nullptr, int ldq = 0) {
  // lr ∈ [0, 3] made visible to the compiler (ln is opaque_lane in the Newton loop): with
  // compile-time (n, m) the range checks of the loads and masks below then fold away
  const int lr = (ln >> 4) & 3, lc = ln & 15;
  {  // C = Mᵀ blocks: element (p = lr + 4r, q = lc) of tile (I, J) is M[16J+q][16I+p] = θ[(16I+p)·n + 16J+q]
    double mv[NT][NT][4];
#pragma unroll
    for (int I = 0; I < NT; ++I)
#pragma unroll
      for (int J = 0; J < NT; ++J)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int col = min(16 * I + lr + 4 * r, n - 1), row = min(16 * J + lc, n - 1);
          mv[I][J][r] = th[col * n + row];
        }
#pragma unroll
    for (int I = 0; I < NT; ++I)
#pragma unroll
      for (int J = 0; J < NT; ++J)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int col = 16 * I + lr + 4 * r, row = 16 * J + lc;
          const bool in = row < n && col < n;
          const double v = mv[I][J][r];
          acc[I][J][r] = in ? (row == col ? v + tol : v) : 0.0;  // M_ij (+ tol on the diagonal)
        }
  }
  const int kc = (m + 3) / 4;
  double nxt[NT], nxq[TWO ? NT : 1];
#pragma unroll
  for (int X = 0; X < NT; ++X) nxt[X] = ta[min(16 * X + lc, n - 1) * lda + min(lr, max(m - 1, 0))];
  if constexpr (TWO) {
#pragma unroll
    for (int X = 0; X < NT; ++X) nxq[X] = tq[min(16 * X + lc, n - 1) * ldq + min(lr, max(m - 1, 0))];
  }
  for (int c = 0; c < kc; ++c) {
    const int k = 4 * c + lr;
    const bool kin = k < m;
    const double dk = sD[kin ? k : 0];  // D_k⁻¹
    double cur[NT], curq[TWO ? NT : 1];
#pragma unroll
    for (int X = 0; X < NT; ++X) cur[X] = nxt[X];
    if constexpr (TWO) {
#pragma unroll
      for (int X = 0; X < NT; ++X) curq[X] = nxq[X];
    }
    if (c + 1 < kc) {
      const int k1 = min(k + 4, m - 1);
#pragma unroll
      for (int X = 0; X < NT; ++X) nxt[X] = ta[min(16 * X + lc, n - 1) * lda + k1];
      if constexpr (TWO) {
#pragma unroll
        for (int X = 0; X < NT; ++X) nxq[X] = tq[min(16 * X + lc, n - 1) * ldq + k1];
      }
    }
    double af[NT], bf[NT];
#pragma unroll
    for (int X = 0; X < NT; ++X) {
      const bool in = kin && 16 * X + lc < n;
      af[X] = in ? cur[X] * dk : 0.0;                    // A_kj · D_k⁻¹   (j = 16I + p)
      bf[X] = in ? (TWO ? curq[X] : cur[X]) : 0.0;       // A_ki         (i = 16J + q)
    }
#pragma unroll
    for (int I = 0; I < NT; ++I)
#pragma unroll
      for (int J = 0; J < NT; ++J) acc[I][J] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[I], bf[J], acc[I][J], 0, 0, 0);
  }
}

// Pivot-free Gauss-Jordan of [S | rh] in the 2-D layout; gj_spd_solve() of the
// oracle step for step (pivot k = row k; rows ≠ k: l = a_ik · (1 / a_kk),
// a_ij ← fma(−l, a_kj, a_ij) for j > k, rh_i ← fma(−l, rh_k, rh_i); then the
// pivot row a_kj ← fma(a_kj, +0, a_kj), rh_k likewise; x_i = rh_i / a_ii).  Entries of columns ≤ k are also touched in a lane
// whose local column block straddles k; those are never read again.
// rh[J] / x[J]: row 16J + lc, replicated over the four DPP rows.
// Gauss-Jordan knobs (A/B: profiles/r03/ab_c3_gj_bperm.jsonl, same bits either way):
// MCPX_GJ_BPERM = 1 hands every lane its rows' pivot-column entries with ds_bpermute
// (LDS crossbar: 2 LDS instructions and 1 product per row half, instead of the
// 17-VALU permlane chain of col_quot_nt2 / from_dpp_row); MCPX_GJ_DGLANE = 1 records
// pivot k in lane k (two v_writelane) instead of a compare-and-select per pivot.
// C3 at 65,536: 13.1 → 15.0 M solves/s; a lone wave's step 10 % shorter.
#ifndef MCPX_GJ_BPERM
#define MCPX_GJ_BPERM 1
#endif
#ifndef MCPX_GJ_DGLANE
#define MCPX_GJ_DGLANE 1
#endif

// v of the lane whose byte address (4 × lane) is `addr` (ds_bpermute, no LDS allocation).
__device__ __forceinline__ double bperm_f64_addr(double v, int addr) {
  const int lo = __builtin_amdgcn_ds_bpermute(addr, __double2loint(v));
  const int hi = __builtin_amdgcn_ds_bpermute(addr, __double2hiint(v));
  return __hiloint2double(hi, lo);
}

// v with lane `k` replaced by the wave-uniform u (two v_writelane_b32; u in SGPRs, the
// lane select an inline constant: k is static after the caller's unrolling).
__device__ __forceinline__ double writelane_f64(double v, double u, int k) {
  int lo = __double2loint(v), hi = __double2hiint(v);
  const int ulo = __builtin_amdgcn_readfirstlane(__double2loint(u));
  const int uhi = __builtin_amdgcn_readfirstlane(__double2hiint(u));
#define C(K) \
  case K: asm volatile("v_writelane_b32 %0, %2, " #K "\n v_writelane_b32 %1, %3, " #K : "+v"(lo), "+v"(hi) : "s"(ulo), "s"(uhi)); break;
  switch (k) { C(0) C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8) C(9) C(10) C(11) C(12) C(13) C(14) C(15) C(16) C(17) C(18) C(19) C(20) C(21) C(22) C(23) C(24) C(25) C(26) C(27) C(28) C(29) C(30) C(31) C(32) C(33) C(34) C(35) C(36) C(37) C(38) C(39) C(40) C(41) C(42) C(43) C(44) C(45) C(46) C(47) C(48) C(49) C(50) C(51) C(52) C(53) C(54) C(55) C(56) C(57) C(58) C(59) C(60) C(61) C(62) C(63)
  }
#undef C
  return __hiloint2double(hi, lo);
}

// xo: the solution entry of row ln (lanes < N; lane 16J + lc is row 16J + lc).
template <int NT, bool PAD>
__device__ __forceinline__ bool gj2d_spd(double (&acc)[NT][NT][4], double (&rh)[NT], int N, int ln, double& xo) {
  const int lc = ln & 15;
  double dg[NT];
#pragma unroll
  for (int J = 0; J < NT; ++J) dg[J] = 1.0;
  double dgl = 1.0;  // MCPX_GJ_DGLANE: pivot k in lane k
  int ad[4];         // MCPX_GJ_BPERM: byte address of lane 16·Q + lc
#pragma unroll
  for (int Q = 0; Q < 4; ++Q) ad[Q] = (16 * Q + lc) << 2;
  // A pivot that is not > 0 (not numerically SPD, or NaN) is only recorded: the
  // remaining steps run on (discarded) values instead of branching on every pivot,
  // which keeps the compare off the step's dependency chain.
  bool bad = false;
#pragma clang loop unroll(full)
  for (int k = 0; k < 16 * NT; ++k) {
    if (k >= N) continue;
    const int Jk = k >> 4, Rk = k & 15;        // pivot row 16·Jk + Rk
    const int Qk = k & 3, Ck = k >> 2;         // pivot column: DPP row Qk, local column Ck
    const int Ik = Ck >> 2, rk = Ck & 3;       // local column Ck = accumulator tile Ik, element rk
    const double piv = bcast(acc[Ik][Jk][rk], 16 * Qk + Rk);
    bad |= !(piv > 0.0);
    const double rp = rcp_uniform(piv);  // oracle gj_spd_solve: l_i = a_ik · (1 / a_kk)
    const bool prow = lc == Rk;  // this lane holds the pivot row in half Jk
    if constexpr (MCPX_GJ_DGLANE) dgl = writelane_f64(dgl, piv, k);
    else if (prow) dg[Jk] = piv;
    double nl[NT];
    if constexpr (MCPX_GJ_BPERM) {  // column k: DPP row Qk of every half register
#pragma unroll
      for (int J = 0; J < NT; ++J) nl[J] = (-bperm_f64_addr(acc[Ik][J][rk], ad[Qk])) * rp;
    } else if constexpr (NT == 2) {
      double q0, q1;  // −l of rows lc and 16 + lc: the fma takes −l · u exactly as fma(−l, u, a)
      switch (Qk + (k == 0 ? 4 : 0)) {  // static after unrolling
        case 0: col_quot_nt2<0, false>(acc[Ik][0][rk], acc[Ik][1][rk], rp, q0, q1); break;
        case 1: col_quot_nt2<1, false>(acc[Ik][0][rk], acc[Ik][1][rk], rp, q0, q1); break;
        case 2: col_quot_nt2<2, false>(acc[Ik][0][rk], acc[Ik][1][rk], rp, q0, q1); break;
        case 3: col_quot_nt2<3, false>(acc[Ik][0][rk], acc[Ik][1][rk], rp, q0, q1); break;
        default: col_quot_nt2<0, true>(acc[Ik][0][rk], acc[Ik][1][rk], rp, q0, q1); break;
      }
      nl[0] = q0;
      nl[1] = q1;
    } else {
#pragma unroll
      for (int J = 0; J < NT; ++J) {
        double colv;
        const bool first = k == 0 && J == 0;
        switch (Qk + (first ? 4 : 0)) {  // static after unrolling
          case 0: colv = from_dpp_row<0, false>(acc[Ik][J][rk]); break;
          case 1: colv = from_dpp_row<1, false>(acc[Ik][J][rk]); break;
          case 2: colv = from_dpp_row<2, false>(acc[Ik][J][rk]); break;
          case 3: colv = from_dpp_row<3, false>(acc[Ik][J][rk]); break;
          default: colv = from_dpp_row<0, true>(acc[Ik][J][rk]); break;  // k = 0: DPP row 0
        }
        nl[J] = (-colv) * rp;
      }
    }
    // The pivot row takes the same fma with multiplier +0 (a_kj ← fma(a_kj, +0, a_kj),
    // mirrored by the oracle): masking its lanes off instead would make them
    // invalid DPP sources for the other lanes of the pivot half.
    if (prow) nl[Jk] = 0.0;
#pragma unroll
    for (int J = 0; J < NT; ++J) {
      if (J == Jk) continue;  // the pivot half last
#pragma unroll
      for (int c = 0; c < 4 * NT; ++c) {
        if (4 * c + 3 <= k) continue;  // every column of this local block ≤ k
        switch (Rk) {
#define MCPX_CASE(R) case R: fmac_row_bcast<R, PAD>(acc[c >> 2][J][c & 3], acc[c >> 2][Jk][c & 3], nl[J]); break;
          MCPX_CASE(0) MCPX_CASE(1) MCPX_CASE(2) MCPX_CASE(3) MCPX_CASE(4) MCPX_CASE(5) MCPX_CASE(6) MCPX_CASE(7)
          MCPX_CASE(8) MCPX_CASE(9) MCPX_CASE(10) MCPX_CASE(11) MCPX_CASE(12) MCPX_CASE(13) MCPX_CASE(14)
          MCPX_CASE(15)
#undef MCPX_CASE
        }
      }
      switch (Rk) {
#define MCPX_CASE(R) case R: fmac_row_bcast<R, PAD>(rh[J], rh[Jk], nl[J]); break;
        MCPX_CASE(0) MCPX_CASE(1) MCPX_CASE(2) MCPX_CASE(3) MCPX_CASE(4) MCPX_CASE(5) MCPX_CASE(6) MCPX_CASE(7)
        MCPX_CASE(8) MCPX_CASE(9) MCPX_CASE(10) MCPX_CASE(11) MCPX_CASE(12) MCPX_CASE(13) MCPX_CASE(14) MCPX_CASE(15)
#undef MCPX_CASE
      }
    }
    {  // half Jk (pivot lanes: multiplier +0), after the other halves have read the pivot row
#pragma unroll
      for (int c = 0; c < 4 * NT; ++c) {
        if (4 * c + 3 <= k) continue;
        switch (Rk) {
#define MCPX_CASE(R) case R: fmac_row_bcast_self<R, PAD>(acc[c >> 2][Jk][c & 3], nl[Jk]); break;
          MCPX_CASE(0) MCPX_CASE(1) MCPX_CASE(2) MCPX_CASE(3) MCPX_CASE(4) MCPX_CASE(5) MCPX_CASE(6) MCPX_CASE(7)
          MCPX_CASE(8) MCPX_CASE(9) MCPX_CASE(10) MCPX_CASE(11) MCPX_CASE(12) MCPX_CASE(13) MCPX_CASE(14)
          MCPX_CASE(15)
#undef MCPX_CASE
        }
      }
      switch (Rk) {
#define MCPX_CASE(R) case R: fmac_row_bcast_self<R, PAD>(rh[Jk], nl[Jk]); break;
        MCPX_CASE(0) MCPX_CASE(1) MCPX_CASE(2) MCPX_CASE(3) MCPX_CASE(4) MCPX_CASE(5) MCPX_CASE(6) MCPX_CASE(7)
        MCPX_CASE(8) MCPX_CASE(9) MCPX_CASE(10) MCPX_CASE(11) MCPX_CASE(12) MCPX_CASE(13) MCPX_CASE(14) MCPX_CASE(15)
#undef MCPX_CASE
      }
    }
  }
  if (bad) return false;
  double r = rh[0], d = dg[0];
#pragma unroll
  for (int J = 1; J < NT; ++J)
    if ((ln >> 4) == J) {
      r = rh[J];
      d = dg[J];
    }
  xo = r / (MCPX_GJ_DGLANE ? dgl : d);
  return true;
}

// The same Gauss-Jordan with compile-time dimension NN and one step of lookahead (the fast
// pass of the compile-time-(n, m) SCHUR kernels, MCPX_GJ_LOOKAHEAD).  Step K updates the local
// column block holding column K + 1 first (every half, the pivot half last), then reads pivot
// K + 1, starts its reciprocal and fetches its column by ds_bpermute, and only then updates
// the other blocks, so the reciprocal's dependent chain and the LDS latency of the column
// run beside the bulk of step K's fmas instead of heading step K + 1.  Every entry takes the
// same fma in the same order as gj2d_spd.  The reciprocal is the branch-free fast form, and
// the pivots are checked once at the end: a pivot ≤ 0 or outside the fast reciprocal's exact
// range (|piv| ∉ [2⁻⁵⁰⁰, 2⁵⁰⁰]) makes the caller (pass 1) defer the instance to the second
// pass, which takes the exact rcp_uniform of gj2d_spd — so the bits stay the oracle's.  Per
// pivot the bookkeeping is 2 readlanes, the 7-instruction reciprocal, one product per half, the
// pivot-row zeroing by a constant lane mask (2 v_cndmask, no compare) and the pivot recorded in
// its lane by 2 v_writelane for the final division.
//
// MCPX_GJ_PIVREC = 1 (diagnostic, off): the round-4 variant that records each pivot by a
// one-lane ds_write under an EXEC switch instead (record_pivot).  It gave wrong last bits in
// every instance.  Cause: pivot 0's ds_write reads the accumulator register the Schur MFMA has
// just written, 2-6 instructions later, where a 16x16x4 f64 MFMA result needs 19 before an LDS
// store reads it as data — hipcc pads that for its own instructions, not inside asm, and the
// store took the register's stale value (tools/check_dpp_hazards.py rule 4).
// MCPX_GJ_PIVREC_PAD = 1 adds that distance (s_nop) ahead of pivot 0's store; the EXEC write →
// store s_nop 4 of round 4 is always there.
#ifndef MCPX_GJ_LOOKAHEAD
#define MCPX_GJ_LOOKAHEAD 1
#endif
#ifndef MCPX_GJ_ZMASK
#define MCPX_GJ_ZMASK 1
#endif
#ifndef MCPX_GJ_PIVREC
#define MCPX_GJ_PIVREC 0
#endif
#ifndef MCPX_GJ_PIVREC_PAD
#define MCPX_GJ_PIVREC_PAD 0
#endif
#ifndef MCPX_GJ_PIVREC_SETPAD  // s_nop 4 between the EXEC write and the store
#define MCPX_GJ_PIVREC_SETPAD 1
#endif
#ifndef MCPX_GJ_PIVREC_EXECPAD  // s_nop 4 after the EXEC restore (ahead of the next DPP fmac)
#define MCPX_GJ_PIVREC_EXECPAD 1
#endif
#define MCPX_PR_STR2(x) #x
#define MCPX_PR_STR(x) MCPX_PR_STR2(x)
#define MCPX_PR_SET MCPX_PR_STR(MCPX_GJ_PIVREC_SETPAD)
#define MCPX_PR_EXEC MCPX_PR_STR(MCPX_GJ_PIVREC_EXECPAD)
typedef __attribute__((address_space(3))) double lds_f64;
// The pivot of step K, the entry `v` holds in lane LANE, to LDS slot K of `base` by a one-lane
// ds_write under a constant EXEC mask.  (The lane mask passes through an opaque asm first: as a
// plain "s" constant the compiler hoists all the distinct masks out of the Newton loop.)
template <int K, int LANE, bool PAD>
__device__ __forceinline__ void record_pivot(uint32_t base, double v) {
  uint64_t save, msk = 1ull << LANE;
  asm volatile("" : "+s"(msk));
  // (".rept 0" emits nothing: the pads are switched by the macros above)
  if (PAD)
    asm volatile("s_nop 7\n s_nop 7\n s_nop 3\n s_mov_b64 %0, exec\n s_mov_b64 exec, %3\n"
                 " .rept " MCPX_PR_SET "\n s_nop 4\n .endr\n"
                 " ds_write_b64 %1, %2 offset:%4\n s_mov_b64 exec, %0\n .rept " MCPX_PR_EXEC "\n s_nop 4\n .endr"
                 : "=&s"(save) : "v"(base), "v"(v), "s"(msk), "n"(8 * K) : "memory");
  else
    asm volatile("s_mov_b64 %0, exec\n s_mov_b64 exec, %3\n .rept " MCPX_PR_SET "\n s_nop 4\n .endr\n"
                 " ds_write_b64 %1, %2 offset:%4\n s_mov_b64 exec, %0\n .rept " MCPX_PR_EXEC "\n s_nop 4\n .endr"
                 : "=&s"(save) : "v"(base), "v"(v), "s"(msk), "n"(8 * K) : "memory");
}
// v with the lanes lc = R of every DPP row replaced by +0: two v_cndmask_b32, no compare.
template <int R>
__device__ __forceinline__ double zero_lanes(double v) {
  int lo = __double2loint(v), hi = __double2hiint(v);
  uint64_t msk = 0x0001000100010001ull << R;
  asm volatile("" : "+s"(msk));
  asm volatile("v_cndmask_b32_e64 %0, %0, 0, %2\n v_cndmask_b32_e64 %1, %1, 0, %2" : "+v"(lo), "+v"(hi) : "s"(msk));
  return __hiloint2double(hi, lo);
}

template <int NT, int NN, int K>
__device__ __forceinline__ void gj2d_la_step(double (&acc)[NT][NT][4], double (&rh)[NT], int ln, double& piv,
                                             double& rp, double (&col)[NT], double& dgl, uint32_t pbase) {
  constexpr int Jk = K >> 4, Rk = K & 15;
  constexpr bool NX = K + 1 < NN;
  constexpr int K1 = NX ? K + 1 : K;
  constexpr int Jn = K1 >> 4, Rn = K1 & 15, Qn = K1 & 3, Cn = K1 >> 2, In = Cn >> 2, rn = Cn & 3;
  __builtin_amdgcn_sched_barrier(0);  // one step at a time
  const int lc = ln & 15;
  double nl[NT];
#pragma unroll
  for (int J = 0; J < NT; ++J) nl[J] = (-col[J]) * rp;
  if constexpr (MCPX_GJ_ZMASK) nl[Jk] = zero_lanes<Rk>(nl[Jk]);  // the pivot row (lc = Rk): multiplier +0
  else if (lc == Rk) nl[Jk] = 0.0;
  if constexpr (NX) {
    if (4 * Cn + 3 > K) {  // the block of column K + 1 (always live at step K)
#pragma unroll
      for (int J = 0; J < NT; ++J) {
        if (J == Jk) continue;
        switch (Rk) {
#define MCPX_CASE(R) case R: fmac_row_bcast<R, false>(acc[In][J][rn], acc[In][Jk][rn], nl[J]); break;
          MCPX_CASE(0) MCPX_CASE(1) MCPX_CASE(2) MCPX_CASE(3) MCPX_CASE(4) MCPX_CASE(5) MCPX_CASE(6) MCPX_CASE(7)
          MCPX_CASE(8) MCPX_CASE(9) MCPX_CASE(10) MCPX_CASE(11) MCPX_CASE(12) MCPX_CASE(13) MCPX_CASE(14)
          MCPX_CASE(15)
#undef MCPX_CASE
        }
      }
      switch (Rk) {
#define MCPX_CASE(R) case R: fmac_row_bcast_self<R, false>(acc[In][Jk][rn], nl[Jk]); break;
        MCPX_CASE(0) MCPX_CASE(1) MCPX_CASE(2) MCPX_CASE(3) MCPX_CASE(4) MCPX_CASE(5) MCPX_CASE(6) MCPX_CASE(7)
        MCPX_CASE(8) MCPX_CASE(9) MCPX_CASE(10) MCPX_CASE(11) MCPX_CASE(12) MCPX_CASE(13) MCPX_CASE(14)
        MCPX_CASE(15)
#undef MCPX_CASE
      }
    }
#pragma unroll
    for (int J = 0; J < NT; ++J) col[J] = bperm_f64_addr(acc[In][J][rn], (16 * Qn + lc) << 2);
    piv = bcast(acc[In][Jn][rn], 16 * Qn + Rn);
    if constexpr (MCPX_GJ_PIVREC) record_pivot<K1, 16 * Qn + Rn, false>(pbase, acc[In][Jn][rn]);
    else dgl = writelane_f64(dgl, piv, K1);  // pivot K + 1 in lane K + 1 (the final division)
    rp = rcp_fast(piv);
  }
#pragma unroll
  for (int J = 0; J < NT; ++J) {
    if (J == Jk) continue;  // the pivot half last
#pragma unroll
    for (int c = 0; c < 4 * NT; ++c) {
      if (4 * c + 3 <= K || (NX && c == Cn)) continue;
      switch (Rk) {
#define MCPX_CASE(R) case R: fmac_row_bcast<R, false>(acc[c >> 2][J][c & 3], acc[c >> 2][Jk][c & 3], nl[J]); break;
        MCPX_CASE(0) MCPX_CASE(1) MCPX_CASE(2) MCPX_CASE(3) MCPX_CASE(4) MCPX_CASE(5) MCPX_CASE(6) MCPX_CASE(7)
        MCPX_CASE(8) MCPX_CASE(9) MCPX_CASE(10) MCPX_CASE(11) MCPX_CASE(12) MCPX_CASE(13) MCPX_CASE(14)
        MCPX_CASE(15)
#undef MCPX_CASE
      }
    }
    switch (Rk) {
#define MCPX_CASE(R) case R: fmac_row_bcast<R, false>(rh[J], rh[Jk], nl[J]); break;
      MCPX_CASE(0) MCPX_CASE(1) MCPX_CASE(2) MCPX_CASE(3) MCPX_CASE(4) MCPX_CASE(5) MCPX_CASE(6) MCPX_CASE(7)
      MCPX_CASE(8) MCPX_CASE(9) MCPX_CASE(10) MCPX_CASE(11) MCPX_CASE(12) MCPX_CASE(13) MCPX_CASE(14) MCPX_CASE(15)
#undef MCPX_CASE
    }
  }
#pragma unroll
  for (int c = 0; c < 4 * NT; ++c) {
    if (4 * c + 3 <= K || (NX && c == Cn)) continue;
    switch (Rk) {
#define MCPX_CASE(R) case R: fmac_row_bcast_self<R, false>(acc[c >> 2][Jk][c & 3], nl[Jk]); break;
      MCPX_CASE(0) MCPX_CASE(1) MCPX_CASE(2) MCPX_CASE(3) MCPX_CASE(4) MCPX_CASE(5) MCPX_CASE(6) MCPX_CASE(7)
      MCPX_CASE(8) MCPX_CASE(9) MCPX_CASE(10) MCPX_CASE(11) MCPX_CASE(12) MCPX_CASE(13) MCPX_CASE(14) MCPX_CASE(15)
#undef MCPX_CASE
    }
  }
  switch (Rk) {
#define MCPX_CASE(R) case R: fmac_row_bcast_self<R, false>(rh[Jk], nl[Jk]); break;
    MCPX_CASE(0) MCPX_CASE(1) MCPX_CASE(2) MCPX_CASE(3) MCPX_CASE(4) MCPX_CASE(5) MCPX_CASE(6) MCPX_CASE(7)
    MCPX_CASE(8) MCPX_CASE(9) MCPX_CASE(10) MCPX_CASE(11) MCPX_CASE(12) MCPX_CASE(13) MCPX_CASE(14) MCPX_CASE(15)
#undef MCPX_CASE
  }
}

template <int NT, int NN, int... K>
__device__ __forceinline__ bool gj2d_spd_la(std::integer_sequence<int, K...>, double (&acc)[NT][NT][4],
                                            double (&rh)[NT], int ln, double& xo) {
  const int lc = ln & 15;
  double col[NT];
  __shared__ double spiv[MCPX_GJ_PIVREC ? NN : 1];  // MCPX_GJ_PIVREC: pivot k in slot k
  const uint32_t pbase = (uint32_t)(uintptr_t)(lds_f64*)spiv;
  double piv = bcast(acc[0][0][0], 0);  // pivot 0: column 0 = tile 0, element 0, DPP row 0
  double dgl = 1.0;
  if constexpr (MCPX_GJ_PIVREC) record_pivot<0, 0, MCPX_GJ_PIVREC_PAD>(pbase, acc[0][0][0]);
  else dgl = writelane_f64(1.0, piv, 0);  // pivot k in lane k
  double rp = rcp_fast(piv);
#pragma unroll
  for (int J = 0; J < NT; ++J) col[J] = bperm_f64_addr(acc[0][J][0], lc << 2);
  (gj2d_la_step<NT, NN, K>(acc, rh, ln, piv, rp, col, dgl, pbase), ...);
  // every pivot > 0 and inside the fast reciprocal's exact range, checked once at the end
  // (a bad pivot only made the later steps compute discarded values); lane i holds pivot i
  if constexpr (MCPX_GJ_PIVREC) {
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the asm ds_writes
    __builtin_amdgcn_wave_barrier();
    dgl = spiv[ln < NN ? ln : 0];
  }
  const double d = dgl;
  if (ballot((ln < NN) & !((d > 0.0) & rcp_fast_ok(d)))) return false;
  double r = rh[0];
#pragma unroll
  for (int J = 1; J < NT; ++J)
    if ((ln >> 4) == J) r = rh[J];
  xo = r / d;
  return true;
}

// The rrule pullback fused into the solve kernel's epilogue (defined in
// sens_kernel_impl.hpp; only the FUSE instantiations of ipm_inst_fused.hip use it).
template <int NV, int FAMILY, int NT, bool LU>
__device__ __forceinline__ bool fused_vjp(const KernelArgs& A, int64_t inst, int ln, int n, int m, double z, double s,
                                          const double* th, const double* ta, int lda, bool msym,
                                          double* const (&lds)[5]);

}  // namespace

// v of lane `src` (ds_bpermute through the LDS crossbar; no LDS allocation).
__device__ __forceinline__ double bperm_f64(double v, int src) {
  const int lo = __builtin_amdgcn_ds_bpermute(src << 2, __double2loint(v));
  const int hi = __builtin_amdgcn_ds_bpermute(src << 2, __double2hiint(v));
  return __hiloint2double(hi, lo);
}

// Row `ln` of S (lane-per-row layout of the pivoting LU) from the 2-D matrix-core
// layout of qp_schur_form_2d: S[i][j] sits in tile (j >> 4, i >> 4), element
// (j >> 2) & 3 of lane 16·(j & 3) + (i & 15).  Entries outside n×n are 0.
template <int NT, int NMAX>
__device__ __forceinline__ void schur_rows_from_2d(const d4 (&acc)[NT][NT], int ln, int n, double (&a)[NMAX]) {
  const int half = ln >> 4, lc = ln & 15;
#pragma unroll
  for (int j = 0; j < NMAX; ++j) {
    const int I = j >> 4, r = (j >> 2) & 3, src = 16 * (j & 3) + lc;
    double v = 0.0;
#pragma unroll
    for (int J = 0; J < NT; ++J) {
      const double t = bperm_f64(acc[I][J][r], src);
      if (half == J) v = t;
    }
    a[j] = (ln < n && j < n) ? v : 0.0;
  }
}

// NC, MC > 0: compile-time (n, m) specialisation; 0: runtime n, m.
// SOLVER: MCPX_LINSOLVE_REDUCED (slack-eliminated (n+m)-dim system), _DENSE
// (full (n+2m)-dim system) or _SCHUR (QP family, n×n Schur complement on MFMA).
//
// PASS (SCHUR only; 0 otherwise) splits the solve over two launches so that the
// common path is compiled without the pivoting-LU fallback, whose row-per-lane
// S adds ~22 VGPRs to the whole kernel (94 → 116 at C3: 5 → 4 waves/SIMD):
//   1  fast pass: SPD Gauss-Jordan only.  An instance whose M is not symmetric,
//      or whose S stops being numerically SPD at some Newton step, is abandoned
//      with status = STATUS_DEFERRED;
//   2  second pass over the same grid: the instances marked deferred are solved
//      again from the start with every path compiled in (the computation is
//      deterministic, so they end bit-identical to a single complete pass); all
//      others exit at once.
// FUSE > 0 (ipm_inst_fused.hip): the instance's rrule pullback runs in the epilogue
// (fused_vjp, register width FUSE ≥ n + m) once its solve is final — mcpx_solve_vjp_batch_device.
template <int NMAX, int FAMILY, int NC, int MC, int SOLVER, int PASS, int FUSE = 0>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(PASS == 1 ? MCPX_FAST_WAVES : 1, 8))) void ipm_solve_kernel(const KernelArgs args) {
  constexpr bool RED = SOLVER != MCPX_LINSOLVE_DENSE;  // lanes [0,n) x, [n,n+m) (y, s)
  constexpr bool SCH = SOLVER == MCPX_LINSOLVE_SCHUR;
  static_assert(SCH || PASS == 0, "two-pass launch is for the SCHUR solver only");
  if constexpr (PASS == 2) {
    if (__builtin_amdgcn_readfirstlane(args.status[blockIdx.x]) != STATUS_DEFERRED) return;
  }
#if MCPX_STAMPS == 2
  const uint64_t tl_start = __builtin_amdgcn_s_memrealtime();
#endif
  if constexpr (MCPX_PRIO > 0) {
    // VALU issue on a SIMD is arbitrated by priority, then age: with equal priorities the
    // oldest resident wave wins, so the waves dispatched last — the ones that set the end of
    // a launch that needs more than one round of residency — get the leftover issue slots.
    // Static priority graded by dispatch order (blockIdx): quarter q of the grid runs at q.
    const unsigned q = (unsigned)(((uint64_t)blockIdx.x * MCPX_PRIO) / gridDim.x);
    if (q == 1) __builtin_amdgcn_s_setprio(1);
    else if (q == 2) __builtin_amdgcn_s_setprio(2);
    else if (q >= 3) __builtin_amdgcn_s_setprio(3);
  }
  __shared__ double zs[64];
  __shared__ double sD[SCH ? 64 : 1], sT[SCH ? 64 : 1];  // SCHUR: D_k⁻¹, ty_k
  __shared__ double sB[SCH ? 64 : 1];  // rr, restored for the LU fallback
  __shared__ double sF[FUSE > 0 ? 64 : 1];  // the fused pullback's fifth LDS array
  // SCHUR with compile-time (n, m): A (row i of Aᵀ at sA[i·LDA], odd stride: the
  // lanes' row reads fall in different banks), b and ϕ copied into LDS once per
  // instance; they are read five times per Newton step (residual rows of G and of H,
  // rr, the Schur complement's MFMA fragments, δy), and from θ that traffic misses
  // L2 (PMC).  M stays in θ: with it the copy would cap occupancy.
  // Affine family under SCHUR (∂H/∂y ≡ 0, θ' = [P; Q; R; S; g; h], the S block not read):
  // the same kernel with R in A's place and the G-side coupling −Qᵀ, with −h and −g, in
  // the wave's LDS (sQ, odd stride) — Q is column-major in θ, so its rows are strided there.
  constexpr bool AFF = SCH && FAMILY == MCPX_FAMILY_AFFINE;
  // (MCPX_AFF_LDS_R: the affine kernel's R in LDS too, in A's slot — more LDS per wave)
  constexpr bool LDSA = SCH && (!AFF || MCPX_AFF_LDS_R) && NC > 0 && MC > 0 && MCPX_LDS_A;
  constexpr int LDA = LDSA ? MC + 1 : 1;
  __shared__ double sA[LDSA ? NC * LDA + MC + NC : 1];
  constexpr bool LDSM = LDSA && NC <= 16 && MCPX_LDS_M;  // M (column-major, as in θ) in LDS too
  __shared__ double sM[LDSM ? NC * NC : 1];
  // n·(m + 1) + m + n doubles for n + m ≤ 64, n ≤ NMAX
  constexpr int LQ = !AFF ? 1 : (NC > 0 ? NC * (MC + 1) + MC + NC : (NMAX >= 32 ? 1120 : NMAX * (65 - NMAX) + 64));
  __shared__ double sQ[LQ];
  const int lane = threadIdx.x;
  const int64_t inst = blockIdx.x;
  const int n0 = NC ? NC : args.n, m0 = MC ? MC : args.m;
  const double* const th0 = args.theta + inst * args.theta_ld;
  const double tol = args.tol;
  if constexpr (AFF) {  // −Qᵀ (row i at sQ[i·(m+1)]), then −h, −g
    const int n = n0, m = m0, ldq = m + 1;
    const double* tg = th0 + n * n;
    for (int i = lane; i < n * m; i += 64) {
      const int k = i / n, r = i - k * n;
      sQ[r * ldq + k] = -tg[i];
    }
    const double* tc = th0 + n * n + 2 * n * m + m * m;  // g (n), h (m)
    for (int i = lane; i < n + m; i += 64) sQ[n * ldq + (i < n ? m + i : i - n)] = -tc[i];
    __syncthreads();
  }

  // src/solver.jl:39-41, 64-66: x₀ = 0, y₀ = 1, s₀ = 1 unless warm-started.
  // DENSE: z = [x; y; s] one per lane.  RED: lanes [0,n) x, [n,n+m) (y, s).
  double z = 0.0, s = 1.0;
  {
    const int n = n0, m = m0;
    if (lane < n) z = args.x0 ? args.x0[inst * n + lane] : 0.0;
    if (lane >= n && lane < n + m) {
      z = args.y0 ? args.y0[inst * m + (lane - n)] : 1.0;
      if (RED) s = args.s0 ? args.s0[inst * m + (lane - n)] : 1.0;
    }
    if (!RED && lane >= n + m && lane < n + 2 * m) z = args.s0 ? args.s0[inst * m + (lane - n - m)] : 1.0;
  }

  if constexpr (LDSA) {  // read before the first step's barrier
    const double* tg = th0 + NC * NC + (AFF ? NC * MC : 0);  // A | the affine R
#pragma unroll
    for (int i = lane; i < NC * MC; i += 64) sA[(i / MC) * LDA + i % MC] = tg[i];
    if constexpr (!AFF)
      for (int i = lane; i < MC + NC; i += 64) sA[NC * LDA + i] = tg[NC * MC + i];
  }
  if constexpr (LDSM) {
#pragma unroll
    for (int i = lane; i < NC * NC; i += 64) sM[i] = th0[i];
  }

  // SCHUR: M exactly symmetric ⇒ S symmetric ⇒ try the pivot-free SPD
  // Gauss-Jordan first (oracle: m_sym).  Once per instance.
  bool spd_try = false;
  bool s_bad = false;  // affine SCHUR: an S entry ≠ 0 (or NaN) — not solved, MCPX_FAIL_INPUT
  if constexpr (SCH) {
    const int n = n0;
    if constexpr (AFF) {
      const int m = m0;
      const double* ts = th0 + n * n + 2 * n * m;
      bool nz = false;
      for (int i = lane; i < m * m; i += 64) nz |= !(ts[i] == 0.0);
      s_bad = ballot(nz) != 0ull;
    }
    bool asym = false;
    const int r = min(lane, max(n - 1, 0));
#pragma clang loop unroll(disable)
    for (int j0 = 0; j0 < n; j0 += 8) {  // 8 (column, row) pairs in flight
      double c[8], t[8];
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const int j = min(j0 + b, n - 1);
        c[b] = th0[j * n + r];
        t[b] = th0[r * n + j];
      }
#pragma unroll
      for (int b = 0; b < 8; ++b) asym |= (lane < n && j0 + b < n) && !(c[b] == t[b]);
    }
    if constexpr (AFF) {  // and −Q = Rᵀ exactly (S symmetric for every D)
      const int m = m0;
      for (int i = lane; i < n * m; i += 64) {
        const int r = i / m, k = i - r * m;
        asym |= !(sQ[r * (m + 1) + k] == th0[n * n + n * m + i]);
      }
    }
    spd_try = ballot(asym) == 0ull || s_bad;  // (s_bad: no Newton step is taken)
    if constexpr (PASS == 1) {
      if (!spd_try) {  // needs the pivoting LU at every step: second pass
        if (lane == 0) args.status[inst] = STATUS_DEFERRED;
        return;
      }
    }
  }

  double eps = 1.0;                    // :67
  double kkt = __builtin_huge_val();   // :68
  int status = 0;                      // :69
  int outer = 1;                       // :70
  int newton = 0;
  unsigned reason = 0;  // MCPX_FAIL_* events
  if (s_bad) {  // the while condition is false on a NaN kkt: the initial point is returned
    kkt = __builtin_nan("");
    status = MCPX_STATUS_FAILED;
    reason = MCPX_FAIL_INPUT;
  }
#if MCPX_STAMPS == 1
  uint64_t st_acc[MCPX_NSTAMP] = {};
  uint64_t st_last = __builtin_amdgcn_s_memtime();
#endif

  while (kkt > tol && eps > tol && outer < args.max_outer) {  // :71
    int inner = 1;   // :72
    status = 0;      // :73
    while (kkt > eps && inner < args.max_inner) {  // :75
      const int n = NC ? NC : opaque(n0), m = MC ? MC : opaque(m0);
      const int NS = SCH ? n : (RED ? n + m : n + 2 * m);  // rows of the linear system
      const double* __restrict__ th = th0 + opaque64(0);  // stays a global pointer
      // SCHUR: the A block (then b, ϕ), from the wave's LDS copy when it has one
      const double* const ta = LDSA ? (const double*)sA : th + (AFF ? n * n + n * m : n * n);
      const int lda = LDSA ? LDA : m;
      // the negated G-side coupling and the constants (QP: A itself, then b, ϕ)
      const int ldq = AFF ? m + 1 : lda;
      const double* const tq = AFF ? (const double*)sQ : ta;
      const double* const tb = AFF ? (const double*)sQ + n * ldq : ta + n * lda;
      const double* const tm = LDSM ? (const double*)sM : th;  // the M block
      const int ln = opaque_lane(lane);
      // ---- F!, ∇F_z! (:79-81) --------------------------------------------
      __syncthreads();
      zs[ln] = z;
      __syncthreads();
      double a[NMAX];
      double F, Fc, rhs, w = 1.0;
      const bool rh = ln >= n && ln < n + m;
      // SCHUR: reciprocals of the slack pivot w_k and the y-block pivot D_k, and the
      // reduced y right-hand side.  Two divisions per lane replace the 13 per step a
      // quotient-per-use form costs (8 of them in the Schur K-loop).
      double rw = 1.0, Di = 1.0, ryr = 0.0;
      if constexpr (SCH) {
        qp_residuals<MCPX_RES_BATCH>(tm, ta, lda, tq, ldq, tb, zs, ln, n, m, eps, s, F, Fc);
        rhs = -F;
        if (rh) {  // eliminate δs_k (pivot w_k) and then δy_k (pivot D_k)
          w = zs[ln] + tol;
          rw = 1.0 / w;
          const double D = tol + s * rw;
          Di = 1.0 / D;
          ryr = (-F) - (Fc * rw);
          sD[ln - n] = Di;
          sT[ln - n] = ryr * Di;
        }
      } else {
        assemble_row<NMAX, FAMILY, RED, (NC > 0)>(th, zs, ln, n, m, eps, tol, s, a, F, Fc, rhs, w);
      }
      MCPX_STAMP(0);
      // ‖F‖∞ with NaN propagation (:107), taken now, committed after the step
      double aF = (ln < (RED ? n + m : NS)) ? fabs(F) : 0.0;
      if (RED && rh) aF = max_nan(aF, fabs(Fc));
      const bool any_nan = ballot(aF != aF) != 0ull;
      const double kkt_step = any_nan ? __builtin_nan("") : wave_max_nonneg(aF);
      if constexpr (SCH) {
        __syncthreads();
        // rr_i = −F_Gi + Σ_k A_ki ty_k  (x-lanes; other lanes' value unused)
        rhs = dot_strided<8, false>(tq + (ln < n ? ln : 0) * ldq, 1, sT, m, rhs);
        sB[ln] = rhs;
      }
      MCPX_STAMP(1);

      // ---- dense LU with partial pivoting (:81-83) -----------------------
      double dz = 0.0;
      // the LU gets an opaque dimension even in the compile-time kernels: with a
      // constant N the allocator keeps ~40 more VGPRs live (fewer waves/SIMD)
      bool ok = false;
      if constexpr (SCH) {
        constexpr int NT = (NMAX + 15) / 16;
        if (spd_try) {  // S formed transposed on the matrix cores, Gauss-Jordan in that layout
          d4 acc4[NT][NT];
          qp_schur_form_2d<NT, AFF>(tm, ta, lda, sD, ln, n, m, tol, acc4, tq, ldq);
          MCPX_STAMP(2);
          double acc[NT][NT][4];
#pragma unroll
          for (int I = 0; I < NT; ++I)
#pragma unroll
            for (int J = 0; J < NT; ++J)
#pragma unroll
              for (int r = 0; r < 4; ++r) acc[I][J][r] = acc4[I][J][r];
          __syncthreads();  // rr (sB) of every row
          double rh2[NT];
#pragma unroll
          for (int J = 0; J < NT; ++J) rh2[J] = (16 * J + (ln & 15) < n) ? sB[16 * J + (ln & 15)] : 0.0;
          // lane 16J + lc owns row 16J + lc.  Opaque dimension: with a constant one the
          // scheduler merges the 32 steps (+5 % VALU in the fast pass)
          if constexpr (PASS == 1 && NC > 0 && MCPX_GJ_LOOKAHEAD)
            ok = gj2d_spd_la<NT, NC>(std::make_integer_sequence<int, NC>{}, acc, rh2, ln, dz);
          else
            ok = gj2d_spd<NT, (NC == 0)>(acc, rh2, (NC > 0) ? opaque(NS) : NS, ln, dz);
        }
        if constexpr (PASS == 1) {
          if (!ok) {  // S not numerically SPD at this step: second pass
            if (lane == 0) args.status[inst] = STATUS_DEFERRED;
            return;
          }
        } else if (!ok) {  // M not symmetric, or S not numerically SPD: pivoting LU on the same S
          // S again in the matrix-core layout, rows gathered across lanes with
          // ds_bpermute: no n×n LDS tile, so LDS (2 KB per wave) does not cap occupancy
          constexpr int NT = (NMAX + 15) / 16;
          d4 acc4[NT][NT];
          qp_schur_form_2d<NT, AFF>(tm, ta, lda, sD, ln, n, m, tol, acc4, tq, ldq);
          schur_rows_from_2d<NT, NMAX>(acc4, ln, n, a);
          rhs = sB[ln];
          ok = lu_solve_rows<NMAX>(a, rhs, (NC > 0) ? opaque(NS) : NS, ln, dz);
        }
      } else {
        ok = lu_solve_rows<NMAX>(a, rhs, (NC > 0) ? opaque(NS) : NS, ln, dz);
      }
      MCPX_STAMP(3);
      if (!ok) {
        status = 1;
        reason |= MCPX_FAIL_LINSOLVE;
        break;
      }
      if constexpr (SCH) {  // δy_k = (ry_k − Σ_j A_kj δx_j) / D_k
        __syncthreads();
        zs[ln] = dz;
        __syncthreads();
        const double acc = dot_strided<8, true>(ta + (rh ? ln - n : 0), lda, zs, n, ryr);
        // branch-free consumer: under `if (rh)` the compiler sinks all n loads of
        // the dot into that block at once (n more live registers)
        const double dzy = acc * Di;
        dz = rh ? dzy : dz;
      }
      double ds = 0.0;
      if (RED && rh) ds = SCH ? fma(-s, dz, -Fc) * rw : fma(-s, dz, -Fc) / w;  // δs_k = (−F_Ck − s_k δy_k) / w_k
      MCPX_STAMP(4);

      // ---- fraction-to-the-boundary line search (:93-100, :127-138) -----
      const bool ry = rh;
      const bool rs = RED ? rh : (ln >= n + m && ln < NS);
      const double sv = RED ? s : z, sd = RED ? ds : dz;  // this lane's s entry and δs
      const double cvy = args.c_tau * z, cvs = args.c_tau * sv;
      uint64_t vs = 0ull, vy = 0ull;
      double alpha = 1.0;
      bool clean_s = false, clean_y = false;  // a trial without violation seen (uniform)
      for (int e = 0; e < args.n_trials; ++e) {
        const double ty = alpha * dz, ts = alpha * sd;
        const double ly = z + ty, ls = sv + ts;
        const bool bs = ballot(rs && ls < cvs) != 0ull, by = ballot(ry && ly < cvy) != 0ull;
        if (bs) vs |= 1ull << e;
        if (by) vy |= 1ull << e;
        clean_s = clean_s || !bs;
        clean_y = clean_y || !by;
        // e_s / e_y are the lowest clear bits: once both exist, later trials cannot move them
        if (clean_s && clean_y) break;
        alpha *= args.decay;
      }
      const int es = (~vs) ? lowest_lane(~vs) : 64;
      const int ey = (~vy) ? lowest_lane(~vy) : 64;
      if (es >= args.n_trials || ey >= args.n_trials) {  // α = NaN
        status = 1;
        reason |= MCPX_FAIL_LINESEARCH;
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
      if (RED) {
        if (rx) z = z + as * dz;
        if (rh) {
          s = s + as * ds;
          z = z + ay * dz;
        }
      } else {
        if (rx || rs) z = z + as * dz;
        if (ry) z = z + ay * dz;
      }
      kkt = MCPX_SREG_KKT ? uniform_f64(kkt_step) : kkt_step;  // :107
      MCPX_STAMP(5);
      ++inner;         // :108
      ++newton;
    }
    eps *= (status == 0) ? args.tight[inner] : args.loose[inner];  // :111-113
    if (MCPX_SREG_KKT) eps = uniform_f64(eps);
    ++outer;                                                        // :114
  }
  if (outer == args.max_outer) {  // :117-119
    status = 1;
    reason |= MCPX_FAIL_MAX_OUTER;
  }

  if constexpr (FUSE > 0) {
    static_assert(RED && FAMILY == MCPX_FAMILY_QP, "the fused pullback follows the QP REDUCED / SCHUR lane layout");
    // The pullback runs before the outputs are written: an instance the fast pass defers
    // must leave x/y/s untouched, since pass 2 re-solves it from x0/y0/s0, which a caller
    // may have aliased to the output buffers (warm start in place).
    // The pullback's Schur path reuses the solve's A block (LDS copy) and its M-symmetry test
    // (opaque sizes: with constant ones the pullback's loops unroll into spills)
    double* const lds[5] = {zs, sD, sT, sB, sF};
    const bool done = fused_vjp<FUSE, FAMILY, (NMAX + 15) / 16, PASS != 1>(
        args, inst, lane, opaque(n0), opaque(m0), z, s, th0, LDSA ? (const double*)sA : th0 + n0 * n0,
        LDSA ? LDA : m0, spd_try, lds);
    if (!done) {  // PASS 1 only (the LU pass always completes)
      if (lane == 0) args.status[inst] = STATUS_DEFERRED;
      return;
    }
  }

  // ---- outputs (:121) -----------------------------------------------------
  const int n = n0, m = m0;
  const bool rx = lane < n, ry = lane >= n && lane < n + m;
  if (rx) args.x[inst * n + lane] = z;
  if (ry) args.y[inst * m + (lane - n)] = z;
  if (RED) {
    if (ry) args.s[inst * m + (lane - n)] = s;
    if (args.active_mask) {
      const uint64_t act = ballot(ry && z > s);
      if (lane == 0) args.active_mask[inst] = act >> n;
    }
  } else {
    const bool rs = lane >= n + m && lane < n + 2 * m;
    if (rs) args.s[inst * m + (lane - n - m)] = z;
    if (args.active_mask) {
      __syncthreads();
      zs[lane] = z;
      __syncthreads();
      const uint64_t act = ballot(ry && z > zs[min(lane + m, 63)]);
      if (lane == 0) args.active_mask[inst] = act >> n;
    }
  }
#if MCPX_STAMPS == 1
  if (lane == 0 && args.stamps)
    for (int i = 0; i < MCPX_NSTAMP; ++i) args.stamps[inst * MCPX_NSTAMP + i] = st_acc[i];
#elif MCPX_STAMPS == 2
  if (lane == 0 && args.stamps) {
    uint64_t* t = args.stamps + inst * MCPX_NSTAMP;
    t[0] = tl_start;
    t[1] = __builtin_amdgcn_s_memrealtime();
    t[2] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
    t[3] = (uint64_t)__builtin_amdgcn_s_getreg((15 << 11) | 20);  // HW_REG_XCC_ID
    t[4] = PASS;
  }
#endif
  if (lane == 0) {
    args.kkt_error[inst] = kkt;
    args.eps[inst] = eps;
    args.outer_iters[inst] = outer;
    args.status[inst] = status;
    if (args.newton_iters) args.newton_iters[inst] = newton;
    if (args.fail_reason) args.fail_reason[inst] = (uint8_t)reason;
  }
}

// Launch helper used by the instantiation units.
template <int NMAX, int FAMILY, int NC, int MC, int SOLVER, int FUSE = 0>
hipError_t launch_one(const KernelArgs& args, int64_t batch, hipStream_t stream) {
  if constexpr (SOLVER == MCPX_LINSOLVE_SCHUR) {  // fast pass, then the deferred instances
    hipLaunchKernelGGL((ipm_solve_kernel<NMAX, FAMILY, NC, MC, SOLVER, 1, FUSE>), dim3((unsigned)batch), dim3(64), 0,
                       stream, args);
    hipLaunchKernelGGL((ipm_solve_kernel<NMAX, FAMILY, NC, MC, SOLVER, 2, FUSE>), dim3((unsigned)batch), dim3(64), 0,
                       stream, args);
  } else {
    hipLaunchKernelGGL((ipm_solve_kernel<NMAX, FAMILY, NC, MC, SOLVER, 0, FUSE>), dim3((unsigned)batch), dim3(64), 0,
                       stream, args);
  }
  return hipGetLastError();
}

}  // namespace mcpx
