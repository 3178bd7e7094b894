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
//              the oracle's fma(0, 0, acc) padding; rr on the VALU (no padding there).  A
//              wave's two tiles of one column tile are formed together (one B fragment, two
//              interleaved chains), four K-chunks' LDS reads ahead of their MFMAs; the A copy in
//              LDS has an odd row stride (kGjLda) so a fragment's 16 rows hit 16 banks.
//   panel k0   (16 columns; every row of S takes every step's update in Gauss-Jordan):
//              1. the 16 pivot rows' panel block (rows k0 .. k0+15) is eliminated by one
//                 wave, lane = row (the pivot row reaches the fmas as a DPP row_newbcast
//                 operand): per step the pivot (pivot-free: S SPD, row k at step k;
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

#include <type_traits>

// MCPX_GJ_STAMPS (diagnostic builds only, tools/gj_phase.hip): thread 0 of each workgroup adds
// s_memtime cycles per phase into gj_stamp_acc[block][phase] — 0 panel staging, 1 the pivot
// block (one wave), 2 the other rows' multipliers and the pivot rows' chains, 3 the MFMA
// trailing update, 4 the solution, 5 the formation of S.
#ifndef MCPX_GJ_STAMPS
#define MCPX_GJ_STAMPS 0
#endif
// MCPX_GJ_FORM_PAIR: the formation takes a wave's two tiles of one column tile together (they
// share the B fragment; two independent MFMA chains).  0: one tile at a time.
#ifndef MCPX_GJ_FORM_PAIR
#define MCPX_GJ_FORM_PAIR 1
#endif
// MCPX_GJ_DPP_NOP: s_nop 1 ahead of each of the pivot block's DPP fmacs (0: the first of each
// step only).  Their DPP source was last written a step earlier; tools/check_dpp_hazards.py
// refuses a build in which the compiler placed a write of it right before.
#ifndef MCPX_GJ_DPP_NOP
#define MCPX_GJ_DPP_NOP 0
#endif

namespace mcpx {
namespace wg {

#if MCPX_GJ_STAMPS
// [block][wave][slot]: lane 0 of every wave; slots 0-5 the phases' work, 8-13 the barrier
// waits that end them (GJ_WAIT)
__device__ uint64_t gj_stamp_acc[2048 * 4 * 16];
#define GJ_STAMP(i)                                                                      \
  do {                                                                                   \
    if ((threadIdx.x & 63) == 0) {                                                       \
      const uint64_t t_ = __builtin_amdgcn_s_memtime();                                  \
      gj_stamp_acc[(blockIdx.x * 4 + (threadIdx.x >> 6)) * 16 + (i)] += t_ - gj_t0;      \
      gj_t0 = t_;                                                                        \
    }                                                                                    \
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

template <int K, int E, class F>
__device__ __forceinline__ void gj_static_for(F&& f) {
  if constexpr (K < E) {
    f(std::integral_constant<int, K>{});
    gj_static_for<K + 1, E>(f);
  }
}

// acc ← fma(nl, u, acc) with u = lane R of acc's 16-lane row (v_fmac_f64_dpp row_newbcast:R; the
// DPP read precedes the write, so every lane sees lane R's old value).  PAD: s_nop 1 first — a
// VALU write needs two wait states before a DPP read of its register, an EXEC write five before
// any DPP instruction (the pivot block pads the first fmac of each step, which follows the
// EXEC restore of the pivot lane's U stores; MCPX_GJ_DPP_NOP = 1 pads every one).
#define GJ_FMAC_NB(R)                                                                                   \
  case R:                                                                                               \
    if (PAD)                                                                                            \
      asm volatile("s_nop 1\n v_fmac_f64_dpp %0, %0, %1 row_newbcast:" #R " row_mask:0xf bank_mask:0xf" \
                   : "+v"(acc)                                                                          \
                   : "v"(nl));                                                                          \
    else                                                                                                \
      asm volatile("v_fmac_f64_dpp %0, %0, %1 row_newbcast:" #R " row_mask:0xf bank_mask:0xf"           \
                   : "+v"(acc)                                                                          \
                   : "v"(nl));                                                                          \
    break;
template <int R, bool PAD>
__device__ __forceinline__ void gj_fmac_bcast_self(double& acc, double nl) {
  switch (R) {
    GJ_FMAC_NB(0) GJ_FMAC_NB(1) GJ_FMAC_NB(2) GJ_FMAC_NB(3) GJ_FMAC_NB(4) GJ_FMAC_NB(5) GJ_FMAC_NB(6)
    GJ_FMAC_NB(7) GJ_FMAC_NB(8) GJ_FMAC_NB(9) GJ_FMAC_NB(10) GJ_FMAC_NB(11) GJ_FMAC_NB(12) GJ_FMAC_NB(13)
    GJ_FMAC_NB(14) GJ_FMAC_NB(15)
  }
}
#undef GJ_FMAC_NB

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
  double lb[16 * 16];                      // the pivot rows' multipliers, [row][step] (0 at its own)
  double rp[NSMAX];                        // 1 / pivot per step
  double piv[NSMAX];                       // pivot per step (S_kk)
  double xb[NSMAX];                        // the final rhs column
  int32_t fail;
};

// C ← M + tol·I, then Σ_k A_ki (A_kj·D_k⁻¹) on the MFMA; column n = rr (LDS); the rest 0.
// th: the instance's θ (QP layout: M n×n column-major, then A m×n column-major).
// tA: the A block, row j of Aᵀ (column j of A) at tA[j·la] — θ's (la = m), or the instance's
// copy in LDS when it fits (la = kGjLda(m)).
template <int NSMAX>
__device__ __forceinline__ void gj_form(d4 (&acc)[GjDims<NSMAX>::TPW], const double* __restrict__ th,
                                        const double* __restrict__ tA, int la, int n, int m, double tol, const double* Di,
                                        const double* rr) {
  using D = GjDims<NSMAX>;
  constexpr int R = D::R;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m4 = (m + 3) & ~3;
  uint64_t gj_t0 = MCPX_GJ_STAMPS ? __builtin_amdgcn_s_memtime() : 0;
  (void)gj_t0;
  // the tile's M entries (clamped addresses: every lane loads, the caller selects), one tile
  // ahead: their global-memory latency hides behind the previous tile's MFMA chain
  auto mload = [&](int u) {
    const int t = gj_opaque(wave) + NWAVE * u, ti = t % R, tj = t / R;
    const int ln_ = vr_opaque_lane(lane), lr = ln_ >> 4, lc = ln_ & 15;
    const int colc = min(16 * tj + lc, n - 1);
    d4 mv;
#pragma unroll
    for (int e = 0; e < 4; ++e) mv[e] = th[(int64_t)colc * n + min(16 * ti + lr + 4 * e, n - 1)];  // M_ij = J[i][j]
    return mv;
  };
  if constexpr (MCPX_GJ_FORM_PAIR && R == 2 * NWAVE && D::TPW % 2 == 0) {
    // Tiles 2v and 2v + 1 of a wave are row tiles `wave` and `wave` + 4 of column tile v: they
    // share the B fragment A_kj·D_k⁻¹, so a K-chunk loads it once, and the two accumulators' MFMA
    // chains interleave (each tile's chain is the same, in the same order: the same bits).
    d4 mn0 = mload(0), mn1 = mload(1);
#pragma unroll
    for (int v = 0; v < D::TPW / 2; ++v) {
      __builtin_amdgcn_sched_barrier(0);  // one column tile at a time
      const d4 mc0 = mn0, mc1 = mn1;
      if (2 * v + 2 < D::TPW) {
        mn0 = mload(2 * v + 2);
        mn1 = mload(2 * v + 3);
      }
      const int ti0 = gj_opaque(wave), ti1 = ti0 + NWAVE, tj = v;
      const int ln_ = vr_opaque_lane(lane), lr = ln_ >> 4, lc = ln_ & 15;
      const int col = 16 * tj + lc, colc = min(col, n - 1);
      // uniform: both tiles inside S (no padding, not the rhs column) — the selects below are
      // identities there except on the diagonal (behind a branch, the compiler sank the rhs
      // column's LDS reads into divergent blocks that re-wrote the accumulators)
      const bool inner = 16 * tj + 16 <= n && 16 * ti1 + 16 <= n;
      d4 c0 = mc0, c1 = mc1;
      if (!inner || ti0 == tj || ti1 == tj) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r0 = 16 * ti0 + lr + 4 * e, r1 = 16 * ti1 + lr + 4 * e;
          const double v0 = r0 == col ? mc0[e] + tol : mc0[e], v1 = r1 == col ? mc1[e] + tol : mc1[e];
          c0[e] = (r0 < n && col < n) ? v0 : 0.0;
          c1[e] = (r1 < n && col < n) ? v1 : 0.0;
        }
      }
      const bool okb = col < n;
      const double* pb = tA + (int64_t)colc * la;
      const int ra0 = 16 * ti0 + lc, ra1 = 16 * ti1 + lc;
      const bool oka0 = ra0 < n, oka1 = ra1 < n;
      const double* pa0 = tA + (int64_t)min(ra0, n - 1) * la;
      const double* pa1 = tA + (int64_t)min(ra1, n - 1) * la;
      if (16 * ti1 < n && 16 * tj < n) {  // uniform: both tiles hold S entries
        // four K-chunks at a time, their 16 LDS reads issued ahead of the 8 MFMAs (the loop does
        // not unroll at a run-time m, and a chunk that waited for its own reads serialised two
        // LDS round trips with every MFMA pair); chunks past m4 only read (clamped addresses)
        for (int q0 = 0; q0 < m4; q0 += 16) {
          double gb[4], gd[4], g0[4], g1[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int kc = min(q0 + 4 * j + lr, m - 1);
            gb[j] = pb[kc];
            gd[j] = Di[kc];
            g0[j] = pa0[kc];
            g1[j] = pa1[kc];
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int q = q0 + 4 * j;
            if (q < m4) {  // uniform
              const bool in = q + lr < m;
              const double b = (okb && in) ? gb[j] * gd[j] : 0.0;
              c0 = __builtin_amdgcn_mfma_f64_16x16x4f64((oka0 && in) ? g0[j] : 0.0, b, c0, 0, 0, 0);
              c1 = __builtin_amdgcn_mfma_f64_16x16x4f64((oka1 && in) ? g1[j] : 0.0, b, c1, 0, 0, 0);
            }
          }
        }
      } else if (16 * ti0 < n && 16 * tj < n) {  // the first only (n ≤ 16·(wave + 4))
#pragma unroll 4
        for (int q = 0; q < m4; q += 4) {
          const int k = q + lr, kc = min(k, m - 1);
          const bool in = k < m;
          const double bv = pb[kc] * Di[kc], av0 = pa0[kc];
          c0 = __builtin_amdgcn_mfma_f64_16x16x4f64((oka0 && in) ? av0 : 0.0, (okb && in) ? bv : 0.0, c0, 0, 0, 0);
        }
      }
      if (!inner) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {  // the rhs column and the padding (as below)
          const int r0 = 16 * ti0 + lr + 4 * e, r1 = 16 * ti1 + lr + 4 * e;
          const double rv0 = rr[min(r0, n - 1)], rv1 = rr[min(r1, n - 1)];
          c0[e] = col == n ? (r0 < n ? rv0 : 0.0) : ((col > n || r0 >= n) ? 0.0 : c0[e]);
          c1[e] = col == n ? (r1 < n ? rv1 : 0.0) : ((col > n || r1 >= n) ? 0.0 : c1[e]);
        }
      }
      acc[2 * v] = c0;
      acc[2 * v + 1] = c1;
    }
    GJ_STAMP(5);
    return;
  }
  d4 mnext = mload(0);
#pragma unroll
  for (int u = 0; u < D::TPW; ++u) {
    __builtin_amdgcn_sched_barrier(0);  // one tile at a time
    const d4 mcur = mnext;
    if (u + 1 < D::TPW) mnext = mload(u + 1);
    const int t = gj_opaque(wave) + NWAVE * u, ti = t % R, tj = t / R;
    const int ln_ = vr_opaque_lane(lane), lr = ln_ >> 4, lc = ln_ & 15;
    // every lane loads from a clamped (valid) address and selects: a load behind a per-lane
    // branch costs an EXEC-mask round trip per entry and waits the memory counter out
    const int col = 16 * tj + lc, colc = min(col, n - 1);
    d4 c;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = 16 * ti + lr + 4 * e;
      const double v = row == col ? mcur[e] + tol : mcur[e];  // J[i][i] += tol
      c[e] = (row < n && col < n) ? v : 0.0;
    }
    if (16 * ti < n && 16 * tj < n) {  // uniform: the tile holds S entries
      const int ra = 16 * ti + lc;      // A-fragment row (an S row)
      const bool oka = ra < n, okb = col < n;
      const double* pa = tA + (int64_t)min(ra, n - 1) * la;
      const double* pb = tA + (int64_t)colc * la;
#pragma unroll 4
      for (int q = 0; q < m4; q += 4) {
        const int k = q + lr, kc = min(k, m - 1);
        const bool in = k < m;
        const double av = pa[kc], bv = pb[kc] * Di[kc];
        const double a = (oka && in) ? av : 0.0;  // A_ki
        const double b = (okb && in) ? bv : 0.0;  // A_kj·D_k⁻¹
        c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {  // the rhs column and the padding (the MFMA's values there are discarded)
      const int row = 16 * ti + lr + 4 * e;
      const double r = rr[min(row, n - 1)];
      c[e] = col == n ? (row < n ? r : 0.0) : ((col > n || row >= n) ? 0.0 : c[e]);
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
  static_assert(NSMAX <= 128, "rows on threads 0-127, trailing columns on threads 128-255");
  // one panel; KB = 16 (full panels: every width test folds) or 0 (the last, kb < 16)
  auto panel = [&](const int k0, auto KBc) -> bool {
    constexpr int KB = decltype(KBc)::value;
    const int tc = k0 >> 4, kb = KB ? KB : min(16, n - k0), j_lo = k0 + kb;
    // ---- the panel (columns k0 .. k0+15 of every row) and the pivot rows' trailing
    //      columns into LDS (whole tiles: entries outside are never read) ------------------
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
      __builtin_amdgcn_sched_barrier(0);
      const int t = gj_opaque(wave) + NWAVE * u, ti = t % R, tj = t / R;
      const int ln_ = vr_opaque_lane(lane), lr = ln_ >> 4, lc = ln_ & 15;
      if (16 * ti >= n || 16 * tj > n || tj < tc) continue;  // uniform
      if (tj == tc) {  // uniform
#pragma unroll
        for (int e = 0; e < 4; ++e) L.pan[(16 * ti + lr + 4 * e) * PL + lc] = acc[u][e];
      }
      if (ti == tc) {  // uniform
#pragma unroll
        for (int e = 0; e < 4; ++e) L.fb[(lr + 4 * e) * UL + 16 * tj + lc] = acc[u][e];
      }
    }
    GJ_STAMP(0);
    __syncthreads();
    GJ_STAMP(8);
    // ---- 1. the pivot rows' block, one wave, lane = block row ----------------------------
    if (wave == 0) {
      double pr[16];
      const int br = k0 + min(lane, 15);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const double v = L.pan[br * PL + q];
        pr[q] = (KB || (lane < kb && q < kb)) ? v : 0.0;
      }
      bool bad = false;
      gj_static_for<0, 16>([&](auto KKc) {
        constexpr int kk = decltype(KKc)::value;
        if (!KB && kk >= kb) return;  // uniform
        const double piv = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(pr[kk]), kk),
                                            __builtin_amdgcn_readlane(__double2loint(pr[kk]), kk));
        bad |= !(piv > 0.0);
        const double rp = 1.0 / piv;
        const bool me = lane == kk;
        if (me) {  // row kk at its step: U for step 2
#pragma unroll
          for (int jj = kk + 1; jj < 16; ++jj) L.ud[kk * 16 + jj] = pr[jj];
        }
        // the pivot row: multiplier +0 (fma(+0, a, a) = fma(a, 0, a)); the others: l = a_ik·(1/piv),
        // a_ij ← fma(−l, u_kj, a_ij) with u_kj from lane kk by the fma's DPP operand
        const double l = pr[kk] * rp;
        const double nl = me ? 0.0 : -l;
#pragma unroll
        for (int jj = kk + 1; jj < 16; ++jj) {
          if (MCPX_GJ_DPP_NOP || jj == kk + 1) gj_fmac_bcast_self<kk, true>(pr[jj], nl);
          else gj_fmac_bcast_self<kk, false>(pr[jj], nl);
        }
        if (lane < 16) L.lb[lane * 16 + kk] = me ? 0.0 : l;  // (lanes kb … 15: rows beyond, never read)
        if (lane == 0) {
          L.rp[k0 + kk] = rp;
          L.piv[k0 + kk] = piv;
        }
      });
      if (bad && lane == 0) L.fail = 1;
    }
    GJ_STAMP(1);
    __syncthreads();
    GJ_STAMP(9);
    // uniform by construction (readfirstlane): an LDS value as the branch condition made the
    // rest of the elimination divergent, and the tiles' uniform indices illegal VGPR→SGPR copies
    if (__builtin_amdgcn_readfirstlane(L.fail)) return false;
    if (tid < 128) {
      // ---- 2. threads 0-127, row = thread: the other rows' multipliers (in place of their
      //      panel entries: the MFMA's A fragments) ----------------------------------------
      const int row = tid;
      if (row < n && (row < k0 || row >= j_lo)) {
        double pr[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) pr[q] = L.pan[row * PL + q];
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) {
          if (!KB && kk >= kb) continue;  // uniform
          const double l = pr[kk] * L.rp[k0 + kk];
#pragma unroll
          for (int jj = kk + 1; jj < 16; ++jj)
            if (KB || jj < kb) pr[jj] = fma(-l, L.ud[kk * 16 + jj], pr[jj]);
          L.pan[row * PL + kk] = l;
        }
      }
    } else {
      // ---- 3. threads 128-255, trailing column = thread: the pivot rows' chains over the
      //      panel's steps (each pivot row's value at its own step is U12, the B operand) ----
      // columns interleaved over the two waves (the trailing set shrinks panel by panel)
      const int q = tid - 128, j = j_lo + 2 * (q & 63) + (q >> 6);
      if (j <= n) {
        double v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = (KB || r < kb) ? L.fb[r * UL + j] : 0.0;
        double lc[16], ln[16];  // step s's multipliers (column s of lb), the next step's loaded ahead
#pragma unroll
        for (int r = 0; r < 16; ++r) lc[r] = L.lb[r * 16];
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          if (!KB && s >= kb) continue;  // uniform
          if (s + 1 < 16) {
#pragma unroll
            for (int r = 0; r < 16; ++r) ln[r] = L.lb[r * 16 + s + 1];
          }
          const double us = v[s];
          L.u12[s * UL + j] = us;
          v[s] = fma(us, 0.0, us);
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (r != s && (KB || r < kb)) v[r] = fma(-lc[r], us, v[r]);
#pragma unroll
          for (int r = 0; r < 16; ++r) lc[r] = ln[r];
        }
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (KB || r < kb) L.fb[r * UL + j] = v[r];
      }
    }
    GJ_STAMP(2);
    __syncthreads();
    GJ_STAMP(10);
    // ---- 4. trailing update of every other row on the matrix cores; the pivot rows'
    //      final values into their tiles (per lane by selects, no per-lane branch) ----------
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
          const double f = L.fb[r * UL + col];
          acc[u][e] = (ctr && (KB || r < kb)) ? f : acc[u][e];
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
        const double av = -L.pan[ra * PL + kk], bv = L.u12[kk * UL + col];
        fa[q] = oka ? av : 0.0;
        fb[q] = ctr ? bv : 0.0;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (KB || 4 * q < kfull) c = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[q], fb[q], c, 0, 0, 0);
      if (!KB && kfull < kb) {  // uniform: a width not a multiple of 4, the rest on the VALU
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = min(16 * ti + lr + 4 * e, n - 1);
          double v = c[e];
          for (int kk = kfull; kk < kb; ++kk) v = fma(-L.pan[row * PL + kk], L.u12[kk * UL + col], v);
          c[e] = v;
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = 16 * ti + lr + 4 * e;
        acc[u][e] = (row < n && ctr) ? c[e] : acc[u][e];
      }
    }
    GJ_STAMP(3);
    __syncthreads();
    GJ_STAMP(11);
    return true;
  };
  bool ok = true;
  for (int k0 = 0; k0 < n && ok; k0 += 16)
    ok = n - k0 >= 16 ? panel(k0, std::integral_constant<int, 16>{}) : panel(k0, std::integral_constant<int, 0>{});
  if (!ok) return false;
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
