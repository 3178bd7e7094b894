// ipm_nl_kernel.hpp — gfx950 solver kernels of the nonlinear family
// (MCPX_FAMILY_NONLINEAR): general G(x, y; θ), H(x, y; θ) evaluated by code
// generated per problem (mcp_amd/codegen.py), the GPU side of the reference's
// Symbolics-compiled F!/∇F_z! callbacks (src/mcp.jl:82-120).
//
// A generated module is one translation unit:
//     #define MCPX_NL_N / _M / _P / _HAS_S / _SIZE / _NNZ
//     mcpx_nl_init(th, blk)      θ-only Jacobian entries, once per instance
//     mcpx_nl_eval(th, z, blk)   G, H and the z-dependent entries, per Newton step
//     #include "ipm_nl_kernel.hpp"
// and this header adds the extern "C" kernels mcpx_nl_solve_{reduced,dense,
// schur} that the problem's size admits, and the record mcpx_nl_meta that
// mcpx_module_load (mcpx_api.cpp) reads.
//
// One 64-lane wave per instance runs the whole ϵ-continuation / Newton loop
// (src/solver.jl:64-121), as ipm_solve_kernel does for the QP / affine
// families.  The generated code is straight-line and its values are
// wave-uniform, so lane 0 alone runs it and stores the blocks (column-major
// P = ∂G/∂x, Q = ∂G/∂y, R = ∂H/∂x, S = ∂H/∂y, and G, H) into LDS.  The iterate
// z = [x; y; s], δz and F live in LDS too, so each linear solver has its own
// lane ↔ row map:
//   SCHUR   (∂H/∂y ≡ 0) δs, then δy eliminated exactly; lane i < n owns row i
//           of S = (P + tol·I) − Q D⁻¹ R, D = tol + s/(y + tol)  (n ≤ 64, m ≤ 128),
//           formed from Q's and R's structural nonzeros only (oracle: the same terms);
//   REDUCED δs eliminated; lanes [0, n+m) own the (n+m)-dim system;
//   DENSE   lanes [0, n+2m) own the rows of ∇F + tol·I;
// all three factor with the register LU with partial pivoting of the QP /
// affine kernels (lu_solve_rows).  Arithmetic follows oracle/ipm_oracle.c
// (family MCPX_FAMILY_NONLINEAR) op for op, and the oracle runs the same
// generated text compiled by gcc, so results are bit-identical.
#pragma once

#include "ipm_kernel_impl.hpp"

#ifndef MCPX_NL_N
#error "ipm_nl_kernel.hpp closes a generated module: MCPX_NL_* and mcpx_nl_init/eval come first"
#endif

#include <utility>

namespace mcpx {
namespace nl {

constexpr int n = MCPX_NL_N, m = MCPX_NL_M, N = n + 2 * m;
constexpr bool HAS_S = MCPX_NL_HAS_S != 0;
// block offsets in doubles (mcp_amd/codegen.py)
constexpr int OFF_P = 0, OFF_Q = n * n, OFF_R = n * n + n * m, OFF_G = n * n + 2 * n * m;
constexpr int OFF_H = OFF_G + n, OFF_S = OFF_H + m;
constexpr int RM = (m + 63) / 64;  // (y, s) entries per lane: lane l owns k = l, l + 64
constexpr int RN = (N + 63) / 64;  // z entries per lane

constexpr int imax(int a, int b) { return a > b ? a : b; }
constexpr int imin(int a, int b) { return a < b ? a : b; }
constexpr int rows_of(int solver) {
  return solver == MCPX_LINSOLVE_DENSE ? N : (solver == MCPX_LINSOLVE_REDUCED ? n + m : n);
}

// ---- 2-D Gauss-Jordan of the one-wave SCHUR kernel ------------------------------------
// Gauss-Jordan with partial pivoting of [S | rr] (oracle lu_solve_x, rcp = 2) with the
// previous Newton step's pivot sequence (lane k of pk = row p_k) as the guess, in the
// matrix-core layout of the QP Gauss-Jordan (csrc/ipm_kernel_impl.hpp, gj2d_spd): lane
// (lr, lc) holds position q = lc + 16J (J < NJ) at columns lr + 4c (c < NCB), position q
// being row p_q, so step k's pivot is position k and its row reaches every lane through DPP
// row_newbcast operands of the fmas; the pivot column goes to every lane by ds_bpermute.
// Multipliers a_qk · (1 / piv); every position but the pivot's takes the update, the pivot
// row itself with multiplier +0 (its lanes are the DPP sources; the oracle does the same);
// columns ≤ k of a straddling 4-column block are updated too and never read again.  Each
// step checks the first-max rule against the guess over the remaining positions (a NaN
// entry counts as a violation); a violation or a zero / NaN / out of
// range guessed pivot returns false, Srow untouched, for the searched Gauss-Jordan.  On
// success x_k = b_k · (1 / u_kk) needs no substitution: lane k holds position k's rhs
// (rh[lr]) and 1 / u_kk.  (The LU with back substitution this replaced spent a third of a
// failing lane-change game's Newton step in the 40-step dependent substitution chain.)
template <int NM>
struct Lu2d {
  static constexpr int NJ = (NM + 15) / 16, NCB = (NM + 3) / 4;
};

// Lanes 0..15 (DPP row 0; every DPP row holds the same column entries) whose position
// q = lane + 16J is still remaining at step K: q > K, q < NM.
template <int NM, int K, int J>
constexpr uint64_t remaining_lanes() {
  uint64_t m = 0;
  for (int l = 0; l < 16; ++l)
    if (l + 16 * J > K && l + 16 * J < NM) m |= 1ull << l;
  return m;
}

#ifndef MCPX_NL_FIX
#define MCPX_NL_FIX 1  // a violated guess is repaired at its step (0: the whole solve falls back)
#endif
#ifndef MCPX_NL_SCOL
#define MCPX_NL_SCOL 1  // one-wave SCHUR: S column-major in LDS (the P copy is a straight b128 copy)
#endif
#ifndef MCPX_NL_SEHOIST
#define MCPX_NL_SEHOIST 1  // the Schur-entry tables in VGPRs for the whole solve
#endif
#ifndef MCPX_NL_PREC
#define MCPX_NL_PREC 1  // pivots recorded by v_writelane; range check and 1/u_kk once at the end
#endif

// Exchange positions K = 16·Jk + Rk and q = 16·JQ + Rq (Rq uniform) of a per-position
// register array: `addr` = the byte address of the partner lane (lanes Rk ↔ Rq of every DPP
// row, the others themselves).  JQ is a template argument (the caller dispatches on the
// uniform half index), so every index is static and the arrays stay in VGPRs.
__device__ __forceinline__ double bperm_any(double v, int addr) { return bperm_f64_addr(v, addr); }
__device__ __forceinline__ int bperm_any(int v, int addr) { return __builtin_amdgcn_ds_bpermute(addr, v); }
template <int NJ, int Jk, int Rk, int JQ, class T>
__device__ __forceinline__ void swap_positions(T (&v)[NJ], int Rq, int addr, int lc) {
  const T t1 = bperm_any(v[JQ], addr);  // position q's entry, at K's lanes
  const T t2 = bperm_any(v[Jk], addr);  // position K's entry, at q's lanes
  if (lc == Rk) v[Jk] = t1;
  if (lc == Rq) v[JQ] = t2;
}
template <int NM, int K, int JQ>
__device__ __forceinline__ void lu2d_swap(double (&acc)[Lu2d<NM>::NJ][Lu2d<NM>::NCB], double (&rh)[Lu2d<NM>::NJ],
                                          int (&pv)[Lu2d<NM>::NJ], double (&col)[Lu2d<NM>::NJ], int Rq, int addr,
                                          int lc) {
  constexpr int NJ = Lu2d<NM>::NJ, NCB = Lu2d<NM>::NCB;
  constexpr int Jk = K >> 4, Rk = K & 15, Ck = K >> 2;
#pragma unroll
  for (int c = Ck; c < NCB; ++c) {
    double v[NJ];
#pragma unroll
    for (int J = 0; J < NJ; ++J) v[J] = acc[J][c];
    swap_positions<NJ, Jk, Rk, JQ>(v, Rq, addr, lc);
#pragma unroll
    for (int J = 0; J < NJ; ++J) acc[J][c] = v[J];
  }
  swap_positions<NJ, Jk, Rk, JQ>(rh, Rq, addr, lc);
  swap_positions<NJ, Jk, Rk, JQ>(col, Rq, addr, lc);
  swap_positions<NJ, Jk, Rk, JQ>(pv, Rq, addr, lc);
}

// Position K's guessed pivot broke the first-max rule: search column K over the remaining
// positions q ≥ K as the oracle does (largest |a_qk|, ties to the lowest row index p_q) and
// swap that position's row into position K — its entries in the columns still live (blocks
// ≥ K / 4), its rhs, its row index and its column-K entry — then take the new pivot and its
// reciprocal.  The elimination then goes on exactly as if the guess had been right, so a
// wrong guess costs ~one swap instead of a second, searched factorisation.  A NaN among the
// candidates or an all-zero column sets `bad` (the searched Gauss-Jordan decides those).
template <int NM, int K>
__device__ __forceinline__ void lu2d_fix(double (&acc)[Lu2d<NM>::NJ][Lu2d<NM>::NCB], double (&rh)[Lu2d<NM>::NJ],
                                         int (&pv)[Lu2d<NM>::NJ], double (&col)[Lu2d<NM>::NJ], double& piv,
                                         double& rp, bool& bad, int ln) {
  constexpr int NJ = Lu2d<NM>::NJ, NCB = Lu2d<NM>::NCB;
  constexpr int Jk = K >> 4, Rk = K & 15, Ck = K >> 2, Qk = K & 3;
  constexpr uint64_t RK[4] = {remaining_lanes<NM, K - 1, 0>(), remaining_lanes<NM, K - 1, 1>(),
                              remaining_lanes<NM, K - 1, 2>(), remaining_lanes<NM, K - 1, 3>()};
  const int lc = ln & 15;
  double mloc = 0.0;
  bool nan = false;
#pragma unroll
  for (int J = Jk; J < NJ; ++J) {
    if (RK[J & 3] == 0) continue;
    const bool live = (RK[J & 3] >> lc) & 1;
    const double av = fabs(col[J]);
    nan |= live && (av != av);
    if (live && av > mloc) mloc = av;
  }
  const double mx = wave_max_nonneg(nan ? 0.0 : mloc);
  if (ballot(nan) != 0ull || !(mx > 0.0)) {
    bad = true;
    return;
  }
  uint32_t key = 0u;  // ~p_q of the candidates: the wave max is the lowest row index
#pragma unroll
  for (int J = Jk; J < NJ; ++J) {
    if (RK[J & 3] == 0) continue;
    const bool live = (RK[J & 3] >> lc) & 1;
    if (live && fabs(col[J]) == mx) key = max(key, ~(uint32_t)pv[J]);
  }
  const uint32_t pbest = ~wave_max_u32(key);
  int qs = K;
#pragma unroll
  for (int J = NJ - 1; J >= Jk; --J) {
    if (RK[J & 3] == 0) continue;
    const uint64_t b = ballot((uint32_t)pv[J] == pbest) & RK[J & 3];
    if (b) qs = 16 * J + lowest_lane(b);
  }
  qs = __builtin_amdgcn_readfirstlane(qs);
  if (qs != K) {
    const int Jq = qs >> 4, Rq = qs & 15;
    const int addr = ((ln & 48) | (lc == Rk ? Rq : (lc == Rq ? Rk : lc))) << 2;
    // q > K, so its half is Jk or later (static dispatch on the uniform half index)
    if (Jq == Jk) lu2d_swap<NM, K, Jk>(acc, rh, pv, col, Rq, addr, lc);
    else if constexpr (Jk + 1 < NJ) {
      if (Jq == Jk + 1) lu2d_swap<NM, K, (Jk + 1 < NJ ? Jk + 1 : Jk)>(acc, rh, pv, col, Rq, addr, lc);
      else if constexpr (Jk + 2 < NJ) {
        if (Jq == Jk + 2) lu2d_swap<NM, K, (Jk + 2 < NJ ? Jk + 2 : Jk)>(acc, rh, pv, col, Rq, addr, lc);
        else if constexpr (Jk + 3 < NJ) lu2d_swap<NM, K, (Jk + 3 < NJ ? Jk + 3 : Jk)>(acc, rh, pv, col, Rq, addr, lc);
      }
    }
  }
  piv = bcast(acc[Jk][Ck], 16 * Qk + Rk);
  rp = rcp_fast(piv);
}

// Step K with one step of lookahead: `piv` (uniform), its reciprocal `rp` and `col` (column
// K by position, from ds_bpermute) were produced by step K − 1 right after it updated column
// K, so the LDS latency and the reciprocal's 7-deep dependent chain hide behind the rest of
// that step's update.  Step K first checks the guessed pivot against the first-max rule over
// the remaining positions (three compares per half into lane masks: |a_qk| > |piv| or NaN;
// equal with a lower row index) and repairs a violation in place (lu2d_fix).  It then
// updates the column block of column K + 1, fetches pivot K + 1, starts its reciprocal and
// fetches its column, then updates the other blocks.  Each entry still takes the same fma
// in the same order.  1 / piv is the uniform fast reciprocal with no branch; the pivot itself
// goes to lane K (v_writelane, MCPX_NL_PREC), and after the last step every lane checks its
// pivot at once: one that is zero, NaN or outside the reciprocal's exact range means the
// remaining steps ran on (discarded) values, and the caller falls back to the searched
// Gauss-Jordan.  Lane k's 1 / u_kk for x_k is taken there too, all lanes at once.
template <int NM, int K>
__device__ __forceinline__ void lu2d_step(double (&acc)[Lu2d<NM>::NJ][Lu2d<NM>::NCB], double (&rh)[Lu2d<NM>::NJ],
                                          int (&pv)[Lu2d<NM>::NJ], int ln, uint64_t& viol,
                                          double& rpv, bool& bad, double& piv, double& rp,
                                          double (&col)[Lu2d<NM>::NJ]) {
  constexpr int NJ = Lu2d<NM>::NJ, NCB = Lu2d<NM>::NCB;
  constexpr int Jk = K >> 4, Rk = K & 15;
  constexpr bool NX = K + 1 < NM;  // a next pivot to fetch
  constexpr int Jn = (K + 1) >> 4, Rn = (K + 1) & 15, Qn = (K + 1) & 3, Cn = (K + 1) >> 2;
  // (a sched_barrier here — one step at a time — cost 2.6 %: the scheduler may overlap a step's
  // tail with the next step's check; the one wave per SIMD has registers to spare,
  // profiles/r04/ab_c4_sched_barrier.jsonl)
  const int lc = ln & 15;
  {  // the first-max rule over the remaining positions
    const int pkk = __builtin_amdgcn_readlane(pv[Jk], Rk);
    const double ap = fabs(piv);
    uint64_t vk = 0;
#pragma unroll
    for (int J = 0; J < NJ; ++J) {
      constexpr uint64_t REM[4] = {remaining_lanes<NM, K, 0>(), remaining_lanes<NM, K, 1>(),
                                   remaining_lanes<NM, K, 2>(), remaining_lanes<NM, K, 3>()};
      if (J >= Jk && REM[J & 3] != 0) {
        const double av = fabs(col[J]);
        vk |= (ballot(!(av <= ap)) | (ballot(av == ap) & ballot(pv[J] < pkk))) & REM[J & 3];
      }
    }
    if constexpr (MCPX_NL_FIX) {
      // unlikely: the repair's code goes out of the steps' straight line (taken on every step, the
      // branch around it cost 6 %: profiles/r04/ab_c4_repair_layout.jsonl)
      if (__builtin_expect(vk != 0ull, 0)) lu2d_fix<NM, K>(acc, rh, pv, col, piv, rp, bad, ln);
    } else {
      viol |= vk;
    }
    if constexpr (!MCPX_NL_PREC) bad |= !(fabs(piv) > 0.0) || !rcp_fast_ok(piv);
  }
  if constexpr (MCPX_NL_PREC) rpv = writelane_f64(rpv, piv, K);  // lane K: pivot K (1 / u_kk at the end)
  else if (ln == K) rpv = rp;
  double nlm[NJ];
#pragma unroll
  for (int J = 0; J < NJ; ++J) nlm[J] = -(col[J] * rp);  // padding positions: col = 0, rows stay 0
  nlm[Jk] = zero_lanes<Rk>(nlm[Jk]);  // the pivot row: multiplier +0
  if constexpr (NX) {  // column block of column K + 1, then pivot K + 1, its reciprocal and column
#pragma unroll
    for (int J = 0; J < NJ; ++J)
      if (J != Jk) fmac_row_bcast<Rk, false>(acc[J][Cn], acc[Jk][Cn], nlm[J]);
    fmac_row_bcast_self<Rk, false>(acc[Jk][Cn], nlm[Jk]);
    piv = bcast(acc[Jn][Cn], 16 * Qn + Rn);
    rp = rcp_fast(piv);
#pragma unroll
    for (int J = 0; J < NJ; ++J) col[J] = bperm_f64_addr(acc[J][Cn], (16 * Qn + lc) << 2);
  }
#pragma unroll
  for (int J = 0; J < NJ; ++J) {
    if (J == Jk) continue;
#pragma unroll
    for (int c = 0; c < NCB; ++c) {
      if (4 * c + 3 <= K || (NX && c == Cn)) continue;
      fmac_row_bcast<Rk, false>(acc[J][c], acc[Jk][c], nlm[J]);
    }
    fmac_row_bcast<Rk, false>(rh[J], rh[Jk], nlm[J]);
  }
#pragma unroll
  for (int c = 0; c < NCB; ++c) {
    if (4 * c + 3 <= K || (NX && c == Cn)) continue;
    fmac_row_bcast_self<Rk, false>(acc[Jk][c], nlm[Jk]);
  }
  fmac_row_bcast_self<Rk, false>(rh[Jk], nlm[Jk]);
}

template <int NM, int... K>
__device__ __forceinline__ void lu2d_steps(std::integer_sequence<int, K...>,
                                           double (&acc)[Lu2d<NM>::NJ][Lu2d<NM>::NCB], double (&rh)[Lu2d<NM>::NJ],
                                           int (&pv)[Lu2d<NM>::NJ], int ln, uint64_t& viol, double& rpv,
                                           bool& bad) {
  constexpr int NJ = Lu2d<NM>::NJ;
  const int lc = ln & 15;
  double piv = bcast(acc[0][0], 0), col[NJ];  // pivot 0, its reciprocal and column 0
  double rp = rcp_fast(piv);
#pragma unroll
  for (int J = 0; J < NJ; ++J) col[J] = bperm_f64_addr(acc[J][0], lc << 2);
  (lu2d_step<NM, K>(acc, rh, pv, ln, viol, rpv, bad, piv, rp, col), ...);
}

template <int NM, bool COL = false>
__device__ __forceinline__ bool lu2d_solve(double* Srow, int LDR, int ln, int& pk, double& dz) {
  constexpr int NJ = Lu2d<NM>::NJ, NCB = Lu2d<NM>::NCB;
  const int lr = ln >> 4, lc = ln & 15;
  double acc[NJ][NCB], rh[NJ];
  int pv[NJ];
#pragma unroll
  for (int J = 0; J < NJ; ++J) {
    const int q = lc + 16 * J;
    const int p = __builtin_amdgcn_ds_bpermute(min(q, 63) << 2, pk);  // row p_q of position q
    pv[J] = q < NM ? p : 1 << 20;
    const int pr = q < NM ? p : 0;
    if constexpr (COL) {
#pragma unroll
      for (int c = 0; c < NCB; ++c) acc[J][c] = (q < NM && lr + 4 * c < NM) ? Srow[(lr + 4 * c) * NM + pr] : 0.0;
      rh[J] = q < NM ? Srow[NM * NM + pr] : 0.0;
    } else {
      const double* row = Srow + pr * LDR;
#pragma unroll
      for (int c = 0; c < NCB; ++c) acc[J][c] = (q < NM && lr + 4 * c < NM) ? row[lr + 4 * c] : 0.0;
      rh[J] = q < NM ? row[NM] : 0.0;
    }
  }
  uint64_t viol = 0;
  double rpv = 0.0;
  bool bad = false;
  lu2d_steps<NM>(std::make_integer_sequence<int, NM>{}, acc, rh, pv, ln, viol, rpv, bad);
  if constexpr (MCPX_NL_PREC) {  // lane k holds pivot k: the range check and 1 / u_kk, all lanes at once
    bad |= ballot(ln < NM && !((fabs(rpv) > 0.0) & rcp_fast_ok(rpv))) != 0ull;
    rpv = rcp_fast(rpv);
  }
  if (bad || viol != 0) return false;
  if constexpr (MCPX_NL_FIX) {  // the pivot sequence taken (repairs included): next step's guess
    int t[NJ];
#pragma unroll
    for (int J = 0; J < NJ; ++J) t[J] = __builtin_amdgcn_ds_bpermute(lc << 2, pv[J]);
    int p = t[0];
#pragma unroll
    for (int J = 1; J < NJ; ++J)
      if (lr == J) p = t[J];
    pk = p;
  }
  // x_k = b_k · (1 / u_kk): lane k = (lr, lc) holds position lc + 16·lr = k in rh[lr]
  double r = rh[0];
#pragma unroll
  for (int J = 1; J < NJ; ++J)
    if (lr == J) r = rh[J];
  dz = r * rpv;
  return true;
}

// ---- Schur complement into LDS, entry-parallel ---------------------------------------
// [S | rr], S = (P + tol·I) − Q D⁻¹ R, rr_i = −F_Gi − Σ_k Q_ik ty_k: row i at Srow[i·LDR], or
// with COL (the one-wave kernel, MCPX_NL_SCOL) column-major, entry (i, j) at Srow[j·n + i] and
// rr at Srow[n·n + i] — the layout P has in blk, so P is a straight two-doubles-per-lane copy
// and the diagonal's + tol a second pass (+6.6 % on the C4 batch with the entry tables held
// in VGPRs, MCPX_NL_SEHOIST: profiles/r04/ab_c4_formation.jsonl).
// First P + tol·I and −F_G, one P entry per lane and slot (column-major P: coalesced);
// then each structural nonzero of Q D⁻¹ R and each rr_i with K(i) ≠ ∅ — an "entry" of the
// generated tables mcpx_nl_se_pos / mcpx_nl_se_k (codegen.py: slot e = lane + 64r, its
// position i·LDR + j and its k ascending) — takes its fma chain in one lane:
// fma(−Q_ik, R_kj·D_k⁻¹, ·) (rr: fma(−Q_ik, ty_k, ·)), k ascending: the oracle's chain
// for that entry (oracle/ipm_oracle.c, the row-wise loop over K(i) and J(k)).
struct SeTables {
  int pos[MCPX_NL_SE_ER], ks[MCPX_NL_SE_ER][MCPX_NL_SE_KT];
  __device__ __forceinline__ void load(int ln) {
#pragma unroll
    for (int r = 0; r < MCPX_NL_SE_ER; ++r) {
      pos[r] = mcpx_nl_se_pos[64 * r + ln];
#pragma unroll
      for (int t = 0; t < MCPX_NL_SE_KT; ++t) ks[r][t] = mcpx_nl_se_k[(r * MCPX_NL_SE_KT + t) * 64 + ln];
    }
  }
};

// COL: S column-major, entry (i, j) at Srow[j·n + i], the rr column at Srow[n·n + i].
template <int LDR, bool COL = false>
__device__ __forceinline__ void schur_form_entries(double* Srow, const double* blk, const double* Fs,
                                                   const double* sDi, const double* sTy, double tol, int ln,
                                                   const SeTables* se_in = nullptr) {
  constexpr int NP = n * n, RP = (NP + 63) / 64;
  if constexpr (COL) {  // P as it lies in blk (column-major), two doubles per lane and access
    typedef double d2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int r = 0; r < (NP + 127) / 128; ++r) {
      const int t = 2 * ln + 128 * r;
      if (t + 1 < NP) *(d2*)(Srow + t) = *(const d2*)(blk + OFF_P + t);
      else if (t < NP) Srow[t] = blk[OFF_P + t];
    }
    if (ln < n) Srow[NP + ln] = -Fs[ln];
    __syncthreads();
    if (ln < n) Srow[ln * n + ln] = Srow[ln * n + ln] + tol;  // the diagonal's + tol (the row-major copy's v + tol)
  } else {
#pragma unroll
    for (int r = 0; r < RP; ++r) {
      const int t = ln + 64 * r;
      if (t < NP) {
        const int j = t / n, i = t - j * n;  // P_ij = blk[OFF_P + j·n + i]
        const double v = blk[OFF_P + t];
        Srow[i * LDR + j] = (i == j) ? v + tol : v;
      }
    }
    if (ln < n) Srow[ln * LDR + n] = -Fs[ln];
  }
  __syncthreads();
  SeTables own;
  if (!se_in) own.load(ln);
  const SeTables& se = se_in ? *se_in : own;
#pragma unroll
  for (int r = 0; r < MCPX_NL_SE_ER; ++r) {
    if (se.pos[r] < 0) continue;
    const int i = se.pos[r] / LDR, j = se.pos[r] - i * LDR;
    const int at = COL ? j * n + i : se.pos[r];
    double v = Srow[at];
#pragma unroll
    for (int t = 0; t < MCPX_NL_SE_KT; ++t) {
      const int k = se.ks[r][t];
      if (k < 0) continue;
      const double q = -blk[OFF_Q + k * n + i];
      const double f = (j == n) ? sTy[k] : blk[OFF_R + j * m + k] * sDi[k];
      v = fma(q, f, v);
    }
    Srow[at] = v;
  }
}

// ---- multi-wave LU of the SCHUR kernel (mcpx_nl_solve_schur_mw) ---------------------
// First-max partial pivoting over the remaining rows (lu_solve_rows_core's search: keys
// hi32(|a|)+1, NaN never wins, ties to the lowest row).
__device__ __forceinline__ int pivot_search(double ak, uint64_t rem, int ln) {
  const double av = fabs(ak);
  const bool valid = ((rem >> ln) & 1ull) && !(av != av);
  const uint32_t khi = valid ? (uint32_t)__double2hiint(av) + 1u : 0u;
  const uint32_t mhi = wave_max_u32(khi);
  if (mhi == 0u) return lowest_lane(rem);  // every remaining entry is NaN
  const uint64_t cand = ballot(khi == mhi);
  if (__popcll(cand) == 1) return lowest_lane(cand);
  const uint32_t klo = (khi == mhi) ? (uint32_t)__double2loint(av) : 0u;
  const uint32_t mlo = wave_max_u32(klo);
  return lowest_lane(ballot(khi == mhi && klo == mlo));
}

// Pivot k from its column (this lane's entry ak): the multipliers a_ik · (1 / piv), −0 for
// the pivot row (Gauss-Jordan: it takes fma(+0, u, a)), and the pivot row (−1: a zero pivot,
// the failed solve of src/solver.jl:84-88) into the LDS buffers of parity k.
__device__ __forceinline__ void publish_pivot(int k, double ak, uint64_t rem, int ln, double* Lb, int* Pb) {
  const int p = pivot_search(ak, rem, ln);
  const double piv = bcast(ak, p);
  Lb[(k & 1) * 64 + ln] = (ln == p) ? -0.0 : ak * rcp_uniform(piv);  // oracle lu_solve_x, rcp = 2
  if (ln == 0) Pb[k & 1] = (piv == 0.0) ? -1 : p;
}

// Gauss-Jordan with partial pivoting of [S | rhs] (row i at Srow[i·LDR], rhs in column NC)
// on W waves: the oracle's lu_solve_x (rcp = 2) operation for operation (bit-identical).
// Wave w owns columns [w·CW, (w+1)·CW) of every row (lane i = row i), the last wave also the
// right-hand side.  Per pivot the owner of the pivot column searches it and publishes the
// multipliers and the pivot row through LDS (double-buffered: one barrier per pivot); every
// wave then updates its columns of every row with the pivot row broadcast from lane p.  The
// owner of column k+1 updates that column first and publishes pivot k+1 before its other
// columns, so the pivot chain runs ahead of the bulk of the update.  Then x_k = b_p / u_pk
// (reciprocal) in lane p, handed to lane k.  dz: the solution entry of row `ln` on wave 0.
template <int NC, int W, int NMAX>
__device__ __forceinline__ bool lu_solve_mw(double* Srow, int LDR, double* Lb, int* Pb, int* pv, int wv, int ln,
                                            double& dz) {
  constexpr int CW = (NC + W - 1) / W;
  static_assert(CW + 1 <= 16, "one broadcast group per wave and pivot");
  double acol[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const int j = wv * CW + c;
    acol[c] = (c < CW && ln < NC && j < NC) ? Srow[ln * LDR + j] : 0.0;
  }
  const bool rhs_wave = wv == W - 1;
  if (rhs_wave) acol[CW] = ln < NC ? Srow[ln * LDR + NC] : 0.0;
  uint64_t rem = (NC >= 64) ? ~0ull : ((1ull << NC) - 1ull);
  int my_step = 1 << 30;
  if (wv == 0) publish_pivot(0, acol[0], rem, ln, Lb, Pb);
#pragma clang loop unroll(full)
  for (int k = 0; k < NC; ++k) {
    __syncthreads();
    const int p = __builtin_amdgcn_readfirstlane(Pb[k & 1]);
    if (p < 0) return false;
    const double l = Lb[(k & 1) * 64 + ln];
    rem &= ~(1ull << p);
    if (ln == p) my_step = k;
    // Gauss-Jordan: every row, the pivot row with multiplier −0, in uniform control flow (lanes
    // ≥ NC hold zeros with a zero multiplier; an EXEC-narrowed update would put the broadcast
    // groups below inside a divergent region, tools/check_dpp_hazards.py)
    const int wn = (k + 1) / CW, cn = (k + 1) % CW;  // owner of the next pivot column (static after unrolling)
    const bool next_owner = k + 1 < NC && wv == wn;
    if (next_owner) {
      const double u = bcast(acol[cn], p);
      acol[cn] = fma(-l, u, acol[cn]);
      publish_pivot(k + 1, acol[cn], rem, ln, Lb, Pb);
    }
    double u[16];
    bcast_n(CW + 1, acol, 1ull << p, u);
#pragma unroll
    for (int c = 0; c <= CW; ++c) {
      const int j = c < CW ? wv * CW + c : NC;  // the rhs slot: column NC of the last wave
      const bool live = (c < CW ? (j > k && j < NC && !(next_owner && c == cn)) : rhs_wave);
      if (live) acol[c] = fma(-l, u[c], acol[c]);
    }
  }
  // row i was the pivot row of step my_step: x_{my_step} = b_i · (1 / u_{i, my_step}) in lane i
  // (u from the wave owning column my_step, b from the rhs wave; the multiplier buffers are
  // free once every wave is past the last step), then to lane my_step
  __syncthreads();
#pragma unroll
  for (int c = 0; c < CW; ++c) {
    const int j = wv * CW + c;
    if (ln < NC && j < NC && j == my_step) Lb[ln] = acol[c];
  }
  if (rhs_wave && ln < NC) Lb[64 + ln] = acol[CW];
  if (wv == 0 && ln < NC) pv[my_step] = ln;
  __syncthreads();
  if (wv == 0) {
    const double xi = ln < NC ? Lb[64 + ln] * (1.0 / Lb[ln]) : 0.0;
    const int p = ln < NC ? pv[ln] : 0;
    const int lo = __builtin_amdgcn_ds_bpermute(p << 2, __double2loint(xi));
    const int hi = __builtin_amdgcn_ds_bpermute(p << 2, __double2hiint(xi));
    dz = ln < NC ? __hiloint2double(hi, lo) : 0.0;
  }
  return true;
}

// ---- lane-parallel eval (mcp_amd/nl_vec.py) ----------------------------------------------
// The generated mcpx_nl_eval rewritten as chains acc = A₀·B₀ + A₁·B₁ + … (each product and
// sum rounded once, the C text's operation order; exact, see nl_vec.py), one chain per lane
// and slot, levels in order.  Operands and destinations are byte offsets into the wave's `ev`
// LDS array (blk | z | θ | constants | temporaries | dummy): per lane and term one word
// (A | B << 16), held in VGPRs for the whole solve.  One wave: LDS ops complete in order, so
// no barrier between levels.
#if defined(MCPX_NL_VEC)
constexpr bool VEC = true;
constexpr int kVecSteps[] = {MCPX_NL_VEC_STEPS};
__device__ __forceinline__ double ev_at(const double* ev, uint32_t byte_off) {
  return *(const double*)((const char*)ev + byte_off);
}
template <int S = 0, int W = 0>
__device__ __forceinline__ void eval_vec(double* ev, const uint32_t (&w)[MCPX_NL_VEC_NWORD],
                                         const uint32_t (&d)[MCPX_NL_VEC_NSLOT]) {
  if constexpr (S < MCPX_NL_VEC_NSLOT) {
    constexpr int K = kVecSteps[S];
    double acc = 0.0;
#pragma unroll
    for (int t = 0; t < K; ++t) {
      const uint32_t x = w[W + t];
      const double prod = ev_at(ev, x & 0xffffu) * ev_at(ev, x >> 16);
      acc = t == 0 ? prod : acc + prod;
    }
    *(double*)((char*)ev + d[S]) = acc;
    eval_vec<S + 1, W + K>(ev, w, d);
  }
}
#else
constexpr bool VEC = false;
#endif

// MW = true (SCHUR only): one 4-wave workgroup per instance (mcpx_nl_solve_schur_mw).  The
// LU runs on all four waves (lu_solve_mw); wave 0 does the rest, the other waves follow the
// same control flow from the shared state in LDS (every branch below depends only on LDS
// contents and lane indices, so all waves take it alike) and write nothing else.
template <int SOLVER, bool MW = false>
__device__ __forceinline__ void solve(const KernelArgs& args) {
  constexpr bool SCH = SOLVER == MCPX_LINSOLVE_SCHUR, RED = SOLVER == MCPX_LINSOLVE_REDUCED;
  constexpr int NR = rows_of(SOLVER);                 // rows of the factored system
  constexpr int NMAX = imax(8, (NR + 7) / 8 * 8);     // register-row width
  static_assert(NR >= 1 && NR <= 64, "the linear system must fit one wave");
  static_assert(!SCH || !HAS_S, "SCHUR needs dH/dy = 0");
  static_assert(SCH || m <= 64, "REDUCED / DENSE hold every constraint in a lane");
  constexpr int BLK = imax(1, OFF_S + (SCH ? 0 : m * m));  // RED / DENSE read S (a zero block if absent)
  constexpr int NZ = imax(1, N), MZ = imax(1, m);
  // the one-wave SCHUR kernel with a lane-parallel eval: blk and z inside its `ev` array
  constexpr bool EV = VEC && SCH && !MW;
#if defined(MCPX_NL_VEC)
  static_assert(!EV || (MCPX_NL_VEC_OFF_Z >= BLK && MCPX_NL_VEC_OFF_T >= MCPX_NL_VEC_OFF_Z + NZ), "ev layout");
  __shared__ __attribute__((aligned(16))) double ev[EV ? MCPX_NL_VEC_EV : 1];
  uint32_t vw[MCPX_NL_VEC_NWORD], vd[MCPX_NL_VEC_NSLOT];
#else
  __shared__ double ev[1];
#endif
  __shared__ __attribute__((aligned(16))) double blk_own[EV ? 1 : BLK];
  __shared__ double zs_own[EV ? 1 : NZ];
  double* const blk = EV ? ev : blk_own;
#if defined(MCPX_NL_VEC)
  double* const zs = EV ? ev + MCPX_NL_VEC_OFF_Z : zs_own;
#else
  double* const zs = zs_own;
#endif
  __shared__ double dzs[NZ], Fs[NZ];
  constexpr int LDR = n + 1;  // SCHUR: lane-private LDS rows of S (odd stride: 2-way bank conflicts at most)
  __shared__ __attribute__((aligned(16))) double Srow[SCH ? imax(1, n * LDR) : 1];
  __shared__ double sRw[SCH ? MZ : 1], sDi[SCH ? MZ : 1], sRy[SCH ? MZ : 1], sTy[SCH ? MZ : 1];
  constexpr int WV = MW ? 4 : 1;  // waves per instance
  static_assert(!MW || SCH, "the multi-wave kernel is the SCHUR one");
  __shared__ double mwL[MW ? 128 : 1];
  __shared__ int mwP[MW ? 2 : 1], mwPv[MW ? 64 : 1];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = MW ? __builtin_amdgcn_readfirstlane(tid >> 6) : 0;  // uniform: scalar branches
  const bool w0 = wv == 0;  // wave 0 owns every write to the shared state
  const int64_t inst = blockIdx.x;
  const double* __restrict__ th = args.theta + inst * args.theta_ld;
  const double tol = args.tol;
  const bool lx = lane < n;

  for (int i = tid; i < BLK; i += 64 * WV) blk[i] = 0.0;  // structural zeros, never written again
  // src/solver.jl:39-41, 64-66: x₀ = 0, y₀ = 1, s₀ = 1 unless warm-started
  if (w0 && lx) zs[lane] = args.x0 ? args.x0[inst * n + lane] : 0.0;
#pragma unroll
  for (int r = 0; r < RM; ++r) {
    const int k = lane + 64 * r;
    if (w0 && k < m) {
      zs[n + k] = args.y0 ? args.y0[inst * m + k] : 1.0;
      zs[n + m + k] = args.s0 ? args.s0[inst * m + k] : 1.0;
    }
  }
#if defined(MCPX_NL_VEC)
  if constexpr (EV) {  // θ and the constants into ev, the lane's operand words into VGPRs
    for (int k = lane; k < MCPX_NL_P; k += 64) ev[MCPX_NL_VEC_OFF_T + k] = th[k];
    for (int k = lane; k < MCPX_NL_VEC_NC; k += 64) ev[MCPX_NL_VEC_OFF_C + k] = mcpx_nl_vec_const[k];
#pragma unroll
    for (int k = 0; k < MCPX_NL_VEC_NWORD; ++k) vw[k] = mcpx_nl_vec_word[k * 64 + lane];
#pragma unroll
    for (int k = 0; k < MCPX_NL_VEC_NSLOT; ++k) vd[k] = mcpx_nl_vec_dst[k * 64 + lane];
  }
#endif
  __syncthreads();
  if (tid == 0) mcpx_nl_init(th, blk);

  double eps = 1.0;                   // :67
  double kkt = __builtin_huge_val();  // :68
  int status = 0;                     // :69
  int outer = 1;                      // :70
  int newton = 0;
  unsigned reason = 0;  // MCPX_FAIL_* events
  SeTables se_tab;
  if constexpr (SCH && !MW && MCPX_NL_SEHOIST) se_tab.load(lane);
  int piv_guess = 0;        // SCHUR: lane k = pivot row of LU step k at the last Newton step
  bool have_guess = false;  // (lu_solve_rows_core)
#if MCPX_STAMPS
  uint64_t st_acc[4] = {0, 0, 0, 0};
  uint64_t st_last = __builtin_amdgcn_s_memtime();
#endif
  while (kkt > tol && eps > tol && outer < args.max_outer) {  // :71
    int inner = 1;                                             // :72
    status = 0;                                                // :73
    while (kkt > eps && inner < args.max_inner) {              // :75
      // ---- F!, ∇F_z! (:79-81): the generated code, then F = [G; H − s; s⊙y − ϵ] (src/mcp.jl:76-80)
      __syncthreads();
#if defined(MCPX_NL_EVAL_PARTS) && MCPX_NL_EVAL_PARTS == 4
      if constexpr (MW) {  // the generated eval's four parts (disjoint outputs), one per wave
        if (lane == 0) {
          if (wv == 0) mcpx_nl_eval_p0(th, zs, blk);
          else if (wv == 1) mcpx_nl_eval_p1(th, zs, blk);
          else if (wv == 2) mcpx_nl_eval_p2(th, zs, blk);
          else mcpx_nl_eval_p3(th, zs, blk);
        }
      } else {
#if defined(MCPX_NL_VEC)
        if constexpr (EV) eval_vec(ev, vw, vd);
        else
#endif
        if (tid == 0) mcpx_nl_eval(th, zs, blk);
      }
#else
      if (tid == 0) mcpx_nl_eval(th, zs, blk);
#endif
      __syncthreads();
      double aF = 0.0;
#pragma unroll
      for (int r = 0; r < RN; ++r) {
        const int i = lane + 64 * r;
        if (i < N) {
          double f;
          if (i < n) f = blk[OFF_G + i];
          else if (i < n + m) f = blk[OFF_H + (i - n)] - zs[i + m];  // H_k − s_k
          else f = zs[i] * zs[i - m] - eps;                          // s_k·y_k − ϵ
          if (w0) Fs[i] = f;
          aF = max_nan(aF, fabs(f));
        }
      }
      // ‖F‖∞ with NaN propagation (:107), taken now, committed after the step
      const double kkt_step = ballot(aF != aF) ? __builtin_nan("") : wave_max_nonneg(aF);
      __syncthreads();
      MCPX_STAMP(0);

      // ---- Newton system (∇F + tol·I) δz = −F (:81-90) ----------------------
      double dz = 0.0;
      bool ok;
      if constexpr (SCH) {
        // eliminate δs_k (pivot w_k = y_k + tol), then δy_k (pivot D_k = (0 + tol) + s_k / w_k)
#pragma unroll
        for (int r = 0; r < RM; ++r) {
          const int k = lane + 64 * r;
          if (w0 && k < m) {
            const double rw = 1.0 / (zs[n + k] + tol);
            const double Di = 1.0 / (tol + zs[n + m + k] * rw);
            const double ry = (-Fs[n + k]) - (Fs[n + m + k] * rw);
            sRw[k] = rw;
            sDi[k] = Di;
            sRy[k] = ry;
            sTy[k] = ry * Di;
          }
        }
        __syncthreads();
        // row i of S = (P + tol·I) − Q D⁻¹ R and rr_i = −F_Gi − Σ_k Q_ik ty_k, k ascending
        // (MW: wave 0 forms the rows into Srow for lu_solve_mw)
        const int i = lx ? lane : 0;
        if constexpr (!MW) {
          schur_form_entries<LDR, (bool)MCPX_NL_SCOL>(Srow, blk, Fs, sDi, sTy, tol, lane,
                                                       MCPX_NL_SEHOIST ? &se_tab : nullptr);
          __syncthreads();
          MCPX_STAMP(1);
          // Gauss-Jordan with partial pivoting of [S | rr] (oracle lu_solve_x, rcp = 2) with the
          // previous Newton step's pivot sequence as the guess (the lane-change game keeps it on
          // 86 % of steps), repaired in place at a step whose guess breaks the first-max rule
          // (lu2d_fix): the 2-D elimination (lu2d_solve) reads the rows in the guessed order.  A
          // zero, NaN or out-of-range pivot leaves Srow as it was and the searched Gauss-Jordan
          // of lu_solve_rows_core (GJ = true) factors its rows.  Bits equal the oracle's rcp = 2
          // elimination either way.  Lanes ≥ n hold a copy of row 0: the GJ updates every lane
          // uniformly, so they are updated too, but never a pivot row and never read.
          bool miss = true;
          if (have_guess) {
            miss = !lu2d_solve<n, (bool)MCPX_NL_SCOL>(Srow, LDR, lane, piv_guess, dz);
            ok = !miss;
          }
          if (miss) {
            double a[NMAX];
#pragma unroll
            for (int j = 0; j < NMAX; ++j) a[j] = (j < n) ? Srow[MCPX_NL_SCOL ? j * n + i : i * LDR + j] : 0.0;
            const double rhs = Srow[MCPX_NL_SCOL ? n * n + i : i * LDR + n];
            bool unused;
            ok = lu_solve_rows_core<NMAX, true>(a, rhs, opaque(n), lane, dz, piv_guess, false, unused);
          }
          have_guess = ok;
        } else {
        if (w0) {
        const double dg = blk[OFF_P + i * n + i] + tol;  // the diagonal entry, one add
        double a[NMAX];
#pragma unroll
        for (int j = 0; j < NMAX; ++j) {
          const double v = (j < n) ? blk[OFF_P + j * n + i] : 0.0;
          a[j] = (j == lane) ? dg : v;
        }
        double rhs = lx ? -Fs[i] : 0.0;
        // − Q D⁻¹ R over the structural nonzeros only (mcpx_nl_qk_* / mcpx_nl_rj_*, generated):
        // entry (i, j) takes fma(−Q_ik, R_kj·D_k⁻¹, ·) for k ∈ K(i) with j ∈ J(k), k ascending
        // (the oracle's chain; at most 3 × 4 terms a row in the lane-change game).  The row
        // indices are per lane, so the row goes through its lane's own LDS row and back.
        const int t0 = lx ? mcpx_nl_qk_ptr[i] : 0, t1 = lx ? mcpx_nl_qk_ptr[i + 1] : 0;
        if (MW || t1 > t0) {
          double* row = Srow + i * LDR;
#pragma unroll
          for (int j = 0; j < n; ++j)
            if (!MW || lx) row[j] = a[j];
          for (int t = t0; t < t1; ++t) {
            const int k = mcpx_nl_qk_idx[t];
            const double q = -blk[OFF_Q + k * n + i], Di = sDi[k];
            for (int u = mcpx_nl_rj_ptr[k]; u < mcpx_nl_rj_ptr[k + 1]; ++u) {
              const int j = mcpx_nl_rj_idx[u];
              row[j] = fma(q, blk[OFF_R + j * m + k] * Di, row[j]);
            }
            rhs = fma(q, sTy[k], rhs);
          }
          if (MW && lx) row[n] = rhs;
#pragma unroll
          for (int j = 0; j < n; ++j) a[j] = row[j];
        }
        MCPX_STAMP(1);
        }  // w0: S formed
        __syncthreads();  // every row of [S | rr] in Srow
        ok = lu_solve_mw<n, 4, NMAX>(Srow, LDR, mwL, mwP, mwPv, wv, lane, dz);
        }  // MW
        MCPX_STAMP(2);
        if (ok) {
          if (w0 && lx) dzs[lane] = dz;
          __syncthreads();
          // δy_k = (ry_k − Σ_j R_kj δx_j)·D_k⁻¹, δs_k = (−F_Ck − s_k δy_k)·w_k⁻¹
#pragma unroll
          for (int r = 0; r < RM; ++r) {
            const int k = lane + 64 * r;
            if (w0 && k < m) {
              double acc = sRy[k];
              for (int t = mcpx_nl_rj_ptr[k]; t < mcpx_nl_rj_ptr[k + 1]; ++t) {  // R's structural nonzeros J(k)
                const int j = mcpx_nl_rj_idx[t];
                acc = fma(-blk[OFF_R + j * m + k], dzs[j], acc);
              }
              const double dy = acc * sDi[k];
              dzs[n + k] = dy;
              dzs[n + m + k] = fma(-zs[n + m + k], dy, -Fs[n + m + k]) * sRw[k];
            }
          }
        }
      } else if constexpr (RED) {
        // slack block eliminated exactly: lanes [0, n) x-rows, [n, n+m) y-rows
        const int i = lane;
        const bool rx = i < n, ry = i >= n && i < n + m;
        const int kh = ry ? i - n : 0;
        const double* px = rx ? blk + OFF_P + i : (ry ? blk + OFF_R + kh : blk);
        const int sx = rx ? n : (ry ? m : 0);
        const double* py = rx ? blk + OFF_Q + i : (ry ? blk + OFF_S + kh : blk);
        const int sy = rx ? n : (ry ? m : 0);
        const double yk = ry ? zs[imin(n + kh, NZ - 1)] : 1.0;
        const double sk = ry ? zs[imin(n + m + kh, NZ - 1)] : 1.0;
        const double w = yk + tol;  // pivot of the eliminated δs_k
        const double d = sk / w;
        double a[NMAX];
#pragma unroll
        for (int j = 0; j < NMAX; ++j) {
          double v = 0.0;
          if (j < n) v = px[j * sx];
          else if (j < n + m) v = (rx || HAS_S) ? py[(j - n) * sy] : 0.0;
          if (!(rx || ry)) v = 0.0;
          if (j == i) {
            v += tol;        // src/solver.jl:81 ∇F + tol*I
            if (ry) v += d;  // + s_k / w_k
          }
          a[j] = v;
        }
        double rhs = 0.0;
        if (rx) rhs = -Fs[i];
        if (ry) rhs = (-Fs[i]) - (Fs[imin(i + m, NZ - 1)] / w);  // −F_H − F_C / w
        ok = lu_solve_rows<NMAX>(a, rhs, opaque(n + m), lane, dz);
        if (ok) {
          if (rx || ry) dzs[i] = dz;
          if (ry) dzs[i + m] = fma(-sk, dz, -Fs[i + m]) / w;  // δs_k = (−F_Ck − s_k δy_k) / w_k
        }
      } else {
        // full (n+2m)-dim system, lane i owns row i of ∇F + tol·I
        const int i = lane;
        const bool rx = i < n, ry = i >= n && i < n + m, rc = i >= n + m && i < N;
        const int kh = ry ? i - n : 0, kc = rc ? i - n - m : 0;
        const double* px = rx ? blk + OFF_P + i : (ry ? blk + OFF_R + kh : blk);
        const int sx = rx ? n : (ry ? m : 0);
        const double* py = rx ? blk + OFF_Q + i : (ry ? blk + OFF_S + kh : blk);
        const int sy = rx ? n : (ry ? m : 0);
        const bool use_y = rx || (ry && HAS_S);
        const double sk = rc ? zs[imin(i, NZ - 1)] : 0.0;      // s_k
        const double yk = rc ? zs[imin(i - m, NZ - 1)] : 0.0;  // y_k
        double a[NMAX];
#pragma unroll
        for (int j = 0; j < NMAX; ++j) {
          double v = 0.0;
          if (j < n) {
            v = (rx || ry) ? px[j * sx] : 0.0;
          } else if (j < n + m) {
            const int q = j - n;
            v = use_y ? py[q * sy] : 0.0;
            if (rc && q == kc) v = sk;  // ∂(s⊙y)/∂y = diag(s)
          } else if (j < N) {
            const int q = j - n - m;
            if (ry && q == kh) v = -1.0;  // ∂(H − s)/∂s = −I
            if (rc && q == kc) v = yk;    // ∂(s⊙y)/∂s = diag(y)
          }
          if (j == i) v += tol;
          a[j] = v;
        }
        const double rhs = (i < N) ? -Fs[imin(i, NZ - 1)] : 0.0;
        ok = lu_solve_rows<NMAX>(a, rhs, opaque(N), lane, dz);
        if (ok && i < N) dzs[i] = dz;
      }
      if (!ok) {  // the failed linear solve of :84-88
        status = 1;
        reason |= MCPX_FAIL_LINSOLVE;
        break;
      }
      __syncthreads();

      // ---- fraction-to-the-boundary line search (:93-100, :127-138) -------
      double yv[RM > 0 ? RM : 1], sv[RM > 0 ? RM : 1], dyv[RM > 0 ? RM : 1], dsv[RM > 0 ? RM : 1];
      bool own[RM > 0 ? RM : 1];
#pragma unroll
      for (int r = 0; r < RM; ++r) {
        const int k = lane + 64 * r;
        own[r] = k < m;
        const int kk = own[r] ? k : 0;
        yv[r] = zs[n + kk];
        sv[r] = zs[n + m + kk];
        dyv[r] = dzs[n + kk];
        dsv[r] = dzs[n + m + kk];
      }
      uint64_t vs = 0ull, vy = 0ull;
      double alpha = 1.0;
      bool clean_s = false, clean_y = false;  // a trial without violation seen (uniform)
      for (int e = 0; e < args.n_trials; ++e) {
        bool bs = false, by = false;
#pragma unroll
        for (int r = 0; r < RM; ++r) {
          if (own[r]) {
            bs = bs || (sv[r] + alpha * dsv[r] < args.c_tau * sv[r]);
            by = by || (yv[r] + alpha * dyv[r] < args.c_tau * yv[r]);
          }
        }
        const bool ws = ballot(bs) != 0ull, wy = ballot(by) != 0ull;
        if (ws) vs |= 1ull << e;
        if (wy) vy |= 1ull << e;
        clean_s = clean_s || !ws;
        clean_y = clean_y || !wy;
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
      if (args.alpha_trace && newton < args.trace_len && tid == 0) {
        uint8_t* tr = args.alpha_trace + ((size_t)inst * args.trace_len + newton) * 2;
        tr[0] = (uint8_t)es;
        tr[1] = (uint8_t)ey;
      }
      // ---- update (:103-105; x moves with α_s) ------------------------------
      if constexpr (MW) __syncthreads();  // every wave has read z for its line search
      if (w0 && lx) zs[lane] = zs[lane] + as * dzs[lane];
#pragma unroll
      for (int r = 0; r < RM; ++r) {
        if (w0 && own[r]) {
          const int k = lane + 64 * r;
          zs[n + m + k] = sv[r] + as * dsv[r];
          zs[n + k] = yv[r] + ay * dyv[r];
        }
      }
      kkt = kkt_step;  // :107
      MCPX_STAMP(3);
      ++inner;         // :108
      ++newton;
    }
    eps *= (status == 0) ? args.tight[inner] : args.loose[inner];  // :111-113
    ++outer;                                                        // :114
  }
  if (outer == args.max_outer) {  // :117-119
    status = 1;
    reason |= MCPX_FAIL_MAX_OUTER;
  }

  // ---- outputs (:121) -------------------------------------------------------
  __syncthreads();
  if (w0 && lx) args.x[inst * n + lane] = zs[lane];
#pragma unroll
  for (int r = 0; r < RM; ++r) {
    const int k = lane + 64 * r;
    if (w0 && k < m) {
      args.y[inst * m + k] = zs[n + k];
      args.s[inst * m + k] = zs[n + m + k];
    }
  }
  if (args.active_mask) {  // W = ⌈m/64⌉ words (include/mcpx.h): one ballot per word
#pragma unroll
    for (int r = 0; r < imax(RM, 1); ++r) {
      const int k = lane + 64 * r;
      bool act = false;
      if (k < m) act = zs[n + imin(k, MZ - 1)] > zs[n + m + imin(k, MZ - 1)];
      const uint64_t bits = ballot(act);
      if (tid == 0) args.active_mask[inst * imax(RM, 1) + r] = bits;
    }
  }
#if MCPX_STAMPS
  if (tid == 0 && args.stamps)
    for (int i = 0; i < 4; ++i) args.stamps[inst * 4 + i] = st_acc[i];
#endif
  if (tid == 0) {
    args.kkt_error[inst] = kkt;
    args.eps[inst] = eps;
    args.outer_iters[inst] = outer;
    args.status[inst] = status;
    if (args.newton_iters) args.newton_iters[inst] = newton;
    if (args.fail_reason) args.fail_reason[inst] = (uint8_t)reason;
  }
}

}  // namespace nl
}  // namespace mcpx

#define MCPX_NL_CAN_REDUCED (MCPX_NL_N + MCPX_NL_M >= 1 && MCPX_NL_N + MCPX_NL_M <= 64)
#define MCPX_NL_CAN_DENSE (MCPX_NL_N + 2 * MCPX_NL_M >= 1 && MCPX_NL_N + 2 * MCPX_NL_M <= 64)
#define MCPX_NL_SCHUR_LDS                                                                             \
  (8 * (MCPX_NL_N * MCPX_NL_N + 2 * MCPX_NL_N * MCPX_NL_M + MCPX_NL_N + MCPX_NL_M +                   \
        MCPX_NL_N * (MCPX_NL_N + 1) + 3 * (MCPX_NL_N + 2 * MCPX_NL_M) + 4 * MCPX_NL_M))
#define MCPX_NL_CAN_SCHUR                                                                             \
  (!MCPX_NL_HAS_S && MCPX_NL_N >= 1 && MCPX_NL_N <= 64 && MCPX_NL_M <= 128 &&                         \
   MCPX_NL_SCHUR_LDS <= 160 * 1024 - 2048)
// the 4-wave SCHUR kernel: each wave's columns plus the rhs in one broadcast group (≤ 16)
#define MCPX_NL_CAN_SCHUR_MW (MCPX_NL_CAN_SCHUR && MCPX_NL_N >= 4 && (MCPX_NL_N + 3) / 4 + 1 <= 16)

// ---- workgroup-per-instance kernels (ipm_wg_impl.hpp) for systems beyond one wave --
// LDS of solve_instances<…, NV = n + 2m, NS>: z, F, δz (3·NV doubles) and the LU
// panel + row lists (NS·(16·8 + 7) bytes), plus reduction scratch.
#define MCPX_NL_NV (MCPX_NL_N + 2 * MCPX_NL_M)
#define MCPX_NL_WG_LDS(NS) (8 * 3 * MCPX_NL_NV + (NS) * (8 * 16 + 7) + 512)
#define MCPX_NL_WG_LIMIT (160 * 1024 - 2048)
#define MCPX_NL_CAN_WG_REDUCED (MCPX_NL_N + MCPX_NL_M >= 1 && MCPX_NL_WG_LDS(MCPX_NL_N + MCPX_NL_M) <= MCPX_NL_WG_LIMIT)
#define MCPX_NL_CAN_WG_DENSE (MCPX_NL_NV >= 1 && MCPX_NL_WG_LDS(MCPX_NL_NV) <= MCPX_NL_WG_LIMIT)
#define MCPX_NL_CAN_WG_SCHUR (!MCPX_NL_HAS_S && MCPX_NL_N >= 1 && MCPX_NL_WG_LDS(MCPX_NL_N) <= MCPX_NL_WG_LIMIT)

#include "sens_wg_impl.hpp"
#include "ipm_nl_band.hpp"

namespace mcpx {
namespace nl {
// the generated code, as the workgroup solver's GEN policy
struct Gen {
  static constexpr int OFF_P = nl::OFF_P, OFF_Q = nl::OFF_Q, OFF_R = nl::OFF_R, OFF_G = nl::OFF_G,
                       OFF_H = nl::OFF_H, OFF_S = nl::OFF_S, SIZE = MCPX_NL_SIZE;
  static constexpr bool HAS_S = nl::HAS_S;
  __device__ static void init(const double* th, double* blk) { mcpx_nl_init(th, blk); }
  __device__ static void eval(const double* th, const double* z, double* blk) { mcpx_nl_eval(th, z, blk); }
  __device__ static const int32_t* qk_ptr() { return mcpx_nl_qk_ptr; }
  __device__ static const int32_t* qk_idx() { return mcpx_nl_qk_idx; }
  __device__ static const int32_t* rj_ptr() { return mcpx_nl_rj_ptr; }
  __device__ static const int32_t* rj_idx() { return mcpx_nl_rj_idx; }
  static constexpr int SE_ER = MCPX_NL_SE_ER, SE_KT = MCPX_NL_SE_KT;
  __device__ static const int32_t* se_pos() { return mcpx_nl_se_pos; }
  __device__ static const int32_t* se_k() { return mcpx_nl_se_k; }
  __device__ static void eval_theta(const double* th, const double* z, double* dth) { mcpx_nl_eval_theta(th, z, dth); }
  __device__ static const int32_t* tc_ptr() { return mcpx_nl_tc_ptr; }
  __device__ static const int32_t* tc_idx() { return mcpx_nl_tc_idx; }
  __device__ static const int32_t* tr_ptr() { return mcpx_nl_tr_ptr; }
  __device__ static const int32_t* tr_idx() { return mcpx_nl_tr_idx; }
};
constexpr int NVW = imax(1, N);
}  // namespace nl
}  // namespace mcpx

// mcpx_nl_meta: {layout version, n, m, p, has_s, kernel mask, block size, nnz, nnz of ∇F_θ,
// the band kernel's workspace doubles per slot, 0, 0}; kernel mask: bit MCPX_LINSOLVE_* = one-wave kernel, bit 3 + MCPX_LINSOLVE_* =
// workgroup kernel, bit MCPX_MODULE_VJP / MCPX_MODULE_JVP = sensitivity kernels (the
// VJP factors the (n+m)-dim system of the REDUCED workgroup solver, the JVP the full
// (n+2m)-dim ∇F_z of the DENSE one: they exist when those fit LDS), bit MCPX_MODULE_SCHUR_MW =
// the 4-wave SCHUR kernel mcpx_nl_solve_schur_mw (layout 4); bits MCPX_MODULE_BAND /
// MCPX_MODULE_BAND_AUTO = the band SCHUR kernel mcpx_nl_solve_band (ipm_nl_band.hpp) and whether
// MCPX_KERNEL_AUTO prefers it (both decided by codegen.py: MCPX_NL_CAN_BAND, MCPX_NL_BAND_AUTO)
extern "C" {
__device__ int32_t mcpx_nl_meta[12] = {
    4, MCPX_NL_N, MCPX_NL_M, MCPX_NL_P, MCPX_NL_HAS_S,
    (MCPX_NL_CAN_REDUCED << MCPX_LINSOLVE_REDUCED) | (MCPX_NL_CAN_DENSE << MCPX_LINSOLVE_DENSE) |
        (MCPX_NL_CAN_SCHUR << MCPX_LINSOLVE_SCHUR) | (MCPX_NL_CAN_WG_REDUCED << (3 + MCPX_LINSOLVE_REDUCED)) |
        (MCPX_NL_CAN_WG_DENSE << (3 + MCPX_LINSOLVE_DENSE)) | (MCPX_NL_CAN_WG_SCHUR << (3 + MCPX_LINSOLVE_SCHUR)) |
        (MCPX_NL_CAN_WG_REDUCED << MCPX_MODULE_VJP) | (MCPX_NL_CAN_WG_DENSE << MCPX_MODULE_JVP) |
        (MCPX_NL_CAN_SCHUR_MW << MCPX_MODULE_SCHUR_MW) | (MCPX_NL_CAN_BAND << MCPX_MODULE_BAND) |
        ((MCPX_NL_CAN_BAND && MCPX_NL_BAND_AUTO) << MCPX_MODULE_BAND_AUTO),
    MCPX_NL_SIZE, MCPX_NL_NNZ, MCPX_NL_NNZ_T,
#if MCPX_NL_CAN_BAND
    (int32_t)mcpx::nl::band::WS,
#else
    0,
#endif
    0, 0};

// MCPX_NL_ONLY_BAND (experiments, never set by codegen.py): compile the band kernel alone
#ifndef MCPX_NL_ONLY_BAND
#if MCPX_NL_CAN_WG_REDUCED
__global__ __launch_bounds__(mcpx::wg::kThreads) void mcpx_nl_vjp_wg(const mcpx::wg::WgSensArgs args) {
  mcpx::wg::sens_instances<MCPX_FAMILY_NONLINEAR, false, mcpx::nl::NVW, MCPX_NL_N + MCPX_NL_M, mcpx::nl::Gen>(args);
}
#endif
#if MCPX_NL_CAN_WG_DENSE
__global__ __launch_bounds__(mcpx::wg::kThreads) void mcpx_nl_jvp_wg(const mcpx::wg::WgSensArgs args) {
  mcpx::wg::sens_instances<MCPX_FAMILY_NONLINEAR, true, mcpx::nl::NVW, mcpx::nl::NVW, mcpx::nl::Gen>(args);
}
#endif

#if MCPX_NL_CAN_WG_REDUCED
__global__ __launch_bounds__(mcpx::wg::kThreads) void mcpx_nl_solve_reduced_wg(const mcpx::wg::WgArgs args) {
  mcpx::wg::solve_instances<MCPX_FAMILY_NONLINEAR, MCPX_LINSOLVE_REDUCED, mcpx::nl::NVW, MCPX_NL_N + MCPX_NL_M,
                            mcpx::nl::Gen>(args);
}
#endif
#if MCPX_NL_CAN_WG_DENSE
__global__ __launch_bounds__(mcpx::wg::kThreads) void mcpx_nl_solve_dense_wg(const mcpx::wg::WgArgs args) {
  mcpx::wg::solve_instances<MCPX_FAMILY_NONLINEAR, MCPX_LINSOLVE_DENSE, mcpx::nl::NVW, mcpx::nl::NVW,
                            mcpx::nl::Gen>(args);
}
#endif
#if MCPX_NL_CAN_WG_SCHUR
__global__ __launch_bounds__(mcpx::wg::kThreads) void mcpx_nl_solve_schur_wg(const mcpx::wg::WgArgs args) {
  mcpx::wg::solve_instances<MCPX_FAMILY_NONLINEAR, MCPX_LINSOLVE_SCHUR, mcpx::nl::NVW, MCPX_NL_N, mcpx::nl::Gen>(args);
}
#endif

#endif  // MCPX_NL_ONLY_BAND
#if MCPX_NL_CAN_BAND
__global__ __launch_bounds__(64) void mcpx_nl_solve_band(const mcpx::wg::WgArgs args) { mcpx::nl::band::solve(args); }
#endif
#ifndef MCPX_NL_ONLY_BAND
#if MCPX_NL_CAN_REDUCED
__global__ __launch_bounds__(64) void mcpx_nl_solve_reduced(const mcpx::KernelArgs args) {
  mcpx::nl::solve<MCPX_LINSOLVE_REDUCED>(args);
}
#endif
#if MCPX_NL_CAN_DENSE
__global__ __launch_bounds__(64) void mcpx_nl_solve_dense(const mcpx::KernelArgs args) {
  mcpx::nl::solve<MCPX_LINSOLVE_DENSE>(args);
}
#endif
#if MCPX_NL_CAN_SCHUR
__global__ __launch_bounds__(64) void mcpx_nl_solve_schur(const mcpx::KernelArgs args) {
  mcpx::nl::solve<MCPX_LINSOLVE_SCHUR>(args);
}
#endif
#if MCPX_NL_CAN_SCHUR_MW
__global__ __launch_bounds__(256) void mcpx_nl_solve_schur_mw(const mcpx::KernelArgs args) {
  mcpx::nl::solve<MCPX_LINSOLVE_SCHUR, true>(args);
}
#endif
#endif  // MCPX_NL_ONLY_BAND
}  // extern "C"
