// gj_vr.hpp — the QP family's SCHUR step on the workgroup-per-instance kernels (n ≤ 128,
// beyond the one-wave kernel's 64 rows): the Schur complement formed on the matrix cores and
// solved by a blocked pivot-free Gauss-Jordan elimination whose trailing update runs on the
// matrix cores too, in registers, bit for bit oracle/ipm_oracle.c's SCHUR step
// (solve_one: S = (M + tol·I) + Aᵀ D⁻¹ A with the MFMA's K padding, gj_spd_solve).
//
// Layout: [S | rr] in the f64 MFMA accumulator layout of lu_vr.hpp — 16×16 tiles, tile
// t = tj·R + ti on wave t mod 4, lane (lr, lc) holding rows 16ti + lr + 4e (e < 4) of column
// 16tj + lc.  At n = 128: 8 × 9 tiles, 18 per wave, 72 doubles per lane; no scratch.
//
//   formation  C ← M + tol·I (the oracle's J[i][i] += tol rounding), then per K-chunk of 4
//              constraints v_mfma_f64_16x16x4_f64 with A-fragment A_ki and B-fragment
//              A_kj·D_k⁻¹ (one rounding, as the oracle's akj·sD[k]); chunks past m are zeros,
//              the oracle's fma(0, 0, acc) padding; rr on the VALU (no padding there).
//   panel k0   (16 columns; every row of S takes every step's update in Gauss-Jordan):
//              1. the 16 pivot rows' panel block (rows k0 .. k0+15) is eliminated by one
//                 wave, lane = row: per step the pivot (pivot-free: S SPD, row k at step k;
//                 a pivot ≤ 0 or NaN abandons the elimination), one correctly rounded
//                 reciprocal, l = a_ik·(1/piv), a_ij ← fma(−l, u_kj, a_ij), the pivot row
//                 itself fma(a, 0, a) (gj_spd_solve's multiplier +0 update);
//              2. every other row, thread = row: its 16 multipliers and panel entries with the
//                 step's u_kj from step 1 — no barrier per column;
//              3. thread = trailing column (the rhs included): the 16 pivot rows' chains over
//                 the panel's steps, in order — each pivot row's value at its own step is the
//                 B operand U12, its value after the panel is final;
//              4. every other row's trailing columns: C ← C + (−L)·U12 on the matrix cores,
//                 K-chunks in step order, i.e. the oracle's fma(−l_ik, u_kj, a_ij) chain k
//                 ascending (a panel narrower than 16 finishes on the VALU in that order).
//   solution   x_i = b_i / S_ii (gj_spd_solve's final division by the step-i pivot).
#pragma once

// MCPX_GJ_STAMPS (diagnostic builds only, tools/gj_phase.hip): thread 0 of each workgroup adds
// s_memtime cycles per phase into gj_stamp_acc[block][phase] — 0 panel staging, 1 the pivot
// block (one wave), 2 the other rows' multipliers and the pivot rows' chains, 3 the MFMA
// trailing update, 4 the solution, 5 the formation of S.
#ifndef MCPX_GJ_STAMPS
#define MCPX_GJ_STAMPS 0
#endif

namespace mcpx {
namespace wg {

#if MCPX_GJ_STAMPS
__device__ uint64_t gj_stamp_acc[2048 * 8];
#define GJ_STAMP(i)                                                 \
  do {                                                              \
    if (threadIdx.x == 0) {                                         \
      const uint64_t t_ = __builtin_amdgcn_s_memtime();             \
      gj_stamp_acc[blockIdx.x * 8 + (i)] += t_ - gj_t0;             \
      gj_t0 = t_;                                                   \
    }                                                               \
  } while (0)
#else
#define GJ_STAMP(i) \
  do {              \
  } while (0)
#endif

// The wave index, opaque to the optimiser (recomputed per tile, as lu_vr.hpp's vr_opaque) and
// uniform by readfirstlane.  (vr_opaque's "+s" constraint here, next to the LU fallback,
// failed instruction selection: illegal VGPR to SGPR copies.)
__device__ __forceinline__ int gj_opaque(int v) {
  asm volatile("" : "+v"(v));
  return __builtin_amdgcn_readfirstlane(v);
}

template <int NSMAX>
struct GjDims {
  static constexpr int R = (NSMAX + 15) / 16;           // row tiles
  static constexpr int T = (NSMAX + 1 + 15) / 16;       // column tiles, the rhs included
  static constexpr int TPW = (R * T + NWAVE - 1) / NWAVE;
  static constexpr int PL = 17;                          // LDS row stride of the panel
  static constexpr int UL = 16 * T;                      // LDS row stride of U12 / the pivot rows
};

template <int NSMAX>
struct GjShared {
  double pan[NSMAX * GjDims<NSMAX>::PL];   // the panel, then the rows' multipliers in place
  double u12[16 * GjDims<NSMAX>::UL];      // pivot row s at its step s (B operand), trailing columns
  double fb[16 * GjDims<NSMAX>::UL];       // the pivot rows' trailing values (their tiles' source)
  double ud[16 * 16];                      // step 1's u_kj inside the panel (for step 2)
  double rp[NSMAX];                        // 1 / pivot per step
  double piv[NSMAX];                       // pivot per step (S_kk)
  double xb[NSMAX];                        // the final rhs column
  int32_t fail;
};

// C ← M + tol·I, then Σ_k A_ki (A_kj·D_k⁻¹) on the MFMA; column n = rr (LDS); the rest 0.
// th: the instance's θ (QP layout: M n×n column-major, then A m×n column-major).
// tA: the A block (m × n column-major) — θ's, or the instance's copy in LDS when it fits.
template <int NSMAX>
__device__ __forceinline__ void gj_form(d4 (&acc)[GjDims<NSMAX>::TPW], const double* __restrict__ th,
                                        const double* __restrict__ tA, int n, int m, double tol, const double* Di,
                                        const double* rr) {
  using D = GjDims<NSMAX>;
  constexpr int R = D::R;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m4 = (m + 3) & ~3;
  uint64_t gj_t0 = MCPX_GJ_STAMPS ? __builtin_amdgcn_s_memtime() : 0;
  (void)gj_t0;
#pragma unroll
  for (int u = 0; u < D::TPW; ++u) {
    __builtin_amdgcn_sched_barrier(0);  // one tile at a time
    const int t = gj_opaque(wave) + NWAVE * u, ti = t % R, tj = t / R;
    const int ln_ = vr_opaque_lane(lane), lr = ln_ >> 4, lc = ln_ & 15;
    const int col = 16 * tj + lc;
    d4 c;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = 16 * ti + lr + 4 * e;
      double v = 0.0;
      if (row < n && col < n) {
        v = th[(int64_t)col * n + row];  // M_ij = J[i][j]
        if (row == col) v += tol;        // J[i][i] += tol
      }
      c[e] = v;
    }
    if (16 * ti < n && 16 * tj < n) {  // uniform: the tile holds S entries
      const int ra = 16 * ti + lc;      // A-fragment row (an S row)
      const bool oka = ra < n, okb = col < n;
      const double* pa = tA + (int64_t)(oka ? ra : 0) * m;
      const double* pb = tA + (int64_t)(okb ? col : 0) * m;
#pragma unroll 4
      for (int q = 0; q < m4; q += 4) {
        const int k = q + lr;
        const bool in = k < m;
        const double a = (oka && in) ? pa[in ? k : 0] : 0.0;                // A_ki
        const double b = (okb && in) ? pb[in ? k : 0] * Di[in ? k : 0] : 0.0;  // A_kj·D_k⁻¹
        c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {  // the rhs column and the padding (the MFMA's values there are discarded)
      const int row = 16 * ti + lr + 4 * e;
      if (col == n) c[e] = row < n ? rr[row] : 0.0;
      else if (col > n || row >= n) c[e] = 0.0;
    }
    acc[u] = c;
  }
  GJ_STAMP(5);
}

// gj_spd_solve on the tiles: x (LDS, ≥ n) = S⁻¹ rr.  False: a pivot that is not > 0 (the
// caller then solves with the pivoting LU, as the oracle does).
template <int NSMAX>
__device__ __forceinline__ bool gj_solve(d4 (&acc)[GjDims<NSMAX>::TPW], int n, double* x, GjShared<NSMAX>& L) {
  using D = GjDims<NSMAX>;
  constexpr int R = D::R, TPW = D::TPW, PL = D::PL, UL = D::UL;
  static_assert(NSMAX <= WG, "one thread per row");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (tid == 0) L.fail = 0;
  uint64_t gj_t0 = MCPX_GJ_STAMPS ? __builtin_amdgcn_s_memtime() : 0;
  (void)gj_t0;
  for (int k0 = 0; k0 < n; k0 += 16) {
    const int tc = k0 >> 4, kb = min(16, n - k0), j_lo = k0 + kb;
    // ---- the panel (columns k0 .. k0+kb−1 of every row) and the pivot rows' trailing
    //      columns into LDS -------------------------------------------------------------
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
      __builtin_amdgcn_sched_barrier(0);
      const int t = gj_opaque(wave) + NWAVE * u, ti = t % R, tj = t / R;
      const int ln_ = vr_opaque_lane(lane), lr = ln_ >> 4, lc = ln_ & 15;
      if (16 * ti >= n || 16 * tj > n || tj < tc) continue;  // uniform
      const int col = 16 * tj + lc;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = 16 * ti + lr + 4 * e;
        if (row >= n) continue;
        if (tj == tc && lc < kb) L.pan[row * PL + lc] = acc[u][e];
        if (ti == tc && col >= j_lo && col <= n) L.fb[(row - k0) * UL + col] = acc[u][e];
      }
    }
    __syncthreads();
    GJ_STAMP(0);
    // ---- 1. the pivot rows' block, one wave, lane = block row ----------------------------
    if (wave == 0) {
      double pr[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) pr[q] = (lane < kb && q < kb) ? L.pan[(k0 + lane) * PL + q] : 0.0;
      bool bad = false;
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) {
        if (kk >= kb) continue;  // uniform
        const double piv = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(pr[kk]), kk),
                                            __builtin_amdgcn_readlane(__double2loint(pr[kk]), kk));
        bad |= !(piv > 0.0);
        const double rp = 1.0 / piv;
        double u[16];
#pragma unroll
        for (int jj = kk + 1; jj < 16; ++jj)
          u[jj] = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(pr[jj]), kk),
                                   __builtin_amdgcn_readlane(__double2loint(pr[jj]), kk));
        if (lane == kk) {
#pragma unroll
          for (int jj = kk + 1; jj < 16; ++jj) pr[jj] = fma(pr[jj], 0.0, pr[jj]);
          L.pan[(k0 + lane) * PL + kk] = 0.0;  // (the pivot row's own step: not a multiplier)
        } else {
          const double l = pr[kk] * rp;
#pragma unroll
          for (int jj = kk + 1; jj < 16; ++jj) pr[jj] = fma(-l, u[jj], pr[jj]);
          if (lane < kb) L.pan[(k0 + lane) * PL + kk] = l;
        }
        if (lane == 0) {
#pragma unroll
          for (int jj = kk + 1; jj < 16; ++jj) L.ud[kk * 16 + jj] = u[jj];
          L.rp[k0 + kk] = rp;
          L.piv[k0 + kk] = piv;
        }
      }
      if (bad && lane == 0) L.fail = 1;
    }
    __syncthreads();
    GJ_STAMP(1);
    // uniform by construction (readfirstlane): an LDS value as the branch condition made the
    // rest of the elimination divergent, and the tiles' uniform indices illegal VGPR→SGPR copies
    if (__builtin_amdgcn_readfirstlane(L.fail)) break;
    // ---- 2. every other row: its multipliers (in place of its panel entries) ----------
    {
      const int row = tid;
      if (row < n && (row < k0 || row >= j_lo)) {
        double pr[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) pr[q] = q < kb ? L.pan[row * PL + q] : 0.0;
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) {
          if (kk >= kb) continue;  // uniform
          const double l = pr[kk] * L.rp[k0 + kk];
#pragma unroll
          for (int jj = kk + 1; jj < 16; ++jj)
            if (jj < kb) pr[jj] = fma(-l, L.ud[kk * 16 + jj], pr[jj]);
          L.pan[row * PL + kk] = l;
        }
      }
    }
    // ---- 3. thread = trailing column: the pivot rows' chains over the panel's steps ----
    for (int j = j_lo + tid; j <= n; j += WG) {
      double v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = r < kb ? L.fb[r * UL + j] : 0.0;
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        if (s >= kb) continue;  // uniform
        const double us = v[s];
        L.u12[s * UL + j] = us;
        v[s] = fma(us, 0.0, us);
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (r != s && r < kb) v[r] = fma(-L.pan[(k0 + r) * PL + s], us, v[r]);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (r < kb) L.fb[r * UL + j] = v[r];
    }
    __syncthreads();
    GJ_STAMP(2);
    // ---- 4. trailing update of every other row on the matrix cores; the pivot rows'
    //      final values into their tiles -------------------------------------------------
    const int kfull = kb & ~3;
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
      __builtin_amdgcn_sched_barrier(0);
      const int t = gj_opaque(wave) + NWAVE * u, ti = t % R, tj = t / R;
      const int ln_ = vr_opaque_lane(lane), lr = ln_ >> 4, lc = ln_ & 15;
      if (16 * ti >= n || 16 * tj > n || 16 * tj + 15 < j_lo) continue;  // uniform: no trailing column
      const int col = 16 * tj + lc;
      const bool ctr = col >= j_lo && col <= n;  // a trailing column (the rhs included)
      if (ti == tc) {  // uniform: the panel's pivot rows
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = lr + 4 * e;
          if (ctr && r < kb) acc[u][e] = L.fb[r * UL + col];
        }
        continue;
      }
      const int ra = 16 * ti + lc;  // A-fragment row
      const bool oka = ra < n;
      d4 c = acc[u];
      double fa[4], fb[4];  // the fragments of all four K-chunks first: one LDS round trip
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int kk = 4 * q + lr;
        fa[q] = (oka && 4 * q < kfull) ? -L.pan[ra * PL + kk] : 0.0;
        fb[q] = (ctr && 4 * q < kfull) ? L.u12[kk * UL + col] : 0.0;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (4 * q < kfull) c = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[q], fb[q], c, 0, 0, 0);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = 16 * ti + lr + 4 * e;
        if (row >= n || !ctr) continue;
        double v = c[e];
        for (int kk = kfull; kk < kb; ++kk) v = fma(-L.pan[row * PL + kk], L.u12[kk * UL + col], v);
        acc[u][e] = v;
      }
    }
    __syncthreads();
    GJ_STAMP(3);
  }
  if (__builtin_amdgcn_readfirstlane(L.fail)) return false;
  // ---- x_i = b_i / S_ii -----------------------------------------------------------------
#pragma unroll
  for (int u = 0; u < TPW; ++u) {
    __builtin_amdgcn_sched_barrier(0);
    const int t = gj_opaque(wave) + NWAVE * u, ti = t % R, tj = t / R;
    const int ln_ = vr_opaque_lane(lane), lr = ln_ >> 4, lc = ln_ & 15;
    if (tj != (n >> 4) || 16 * ti >= n) continue;  // uniform
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = 16 * ti + lr + 4 * e;
      if (row < n && lc == (n & 15)) L.xb[row] = acc[u][e];
    }
  }
  __syncthreads();
  for (int i = tid; i < n; i += WG) x[i] = L.xb[i] / L.piv[i];
  __syncthreads();
  GJ_STAMP(4);
  return true;
}

}  // namespace wg
}  // namespace mcpx
