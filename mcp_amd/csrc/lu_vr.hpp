// lu_vr.hpp — register-resident blocked LU of the workgroup-per-instance kernels
// (ipm_wg_impl.hpp) for systems up to MCPX_VR_MAX rows: the same elimination as
// wg::lu_solve — implicit partial pivoting (first remaining row of largest |a|, NaN
// never wins), 16-column panels factored in LDS, U12 by in-panel forward substitution,
// trailing update C ← C + (−L21)·U12 on v_mfma_f64_16x16x4_f64 (an ordered k-ascending
// fma chain bitwise), column-oriented back substitution — so the bits
// equal oracle/ipm_oracle.c::lu_solve (lu_solve_x with RCP) like wg::lu_solve's.
//
// The difference is where [K | rhs] lives while it is factored: wg::lu_solve streams
// it through the slot's HBM workspace at every panel (the trailing update reads and
// writes the whole trailing matrix once per 16 columns), while here its entries are
// computed straight into the VGPRs of the workgroup's WG threads, in the MFMA
// accumulator layout, and the matrix never touches memory.  Tile (ti, tj) of 16×16
// (rows 16ti.., columns 16tj.., right-hand sides as trailing columns) belongs to wave
// t mod NWAVE with t = tj·R + ti (column-major:
// every column tile spreads over the waves, so each panel's trailing update is
// balanced); in it lane (lr, lc) holds rows 16ti + lr + 4e (e < 4) of column 16tj + lc,
// the f64 MFMA's C layout.  Only the panel (all rows × 16 columns), the panel's U12 rows
// and the per-row bookkeeping pass through LDS.  At NSMAX = 200 on 4 waves: 44 tiles = 176
// doubles per lane (VGPRs and AGPRs; one workgroup per CU).
#pragma once

// MCPX_VR_TWICE (diagnostic builds only, tools/ab_build.py): one phase of lu_solve_vr runs twice
// — 1 the staging of [K | rhs] into the tiles, 2 the back substitution.  Both are idempotent, so
// the bits stay the product's and the time added is the phase's cost.
#ifndef MCPX_VR_TWICE
#define MCPX_VR_TWICE 0
#endif

namespace mcpx {
namespace wg {

// The wave index through an empty asm: tile indices and the LDS addresses derived from
// them are recomputed where used instead of being hoisted out of the panel loop, where
// 4·TPW addresses would stay live beside the tiles.
__device__ __forceinline__ int vr_opaque(int v) {
  asm volatile("" : "+s"(v));
  return v;
}
// Same for the lane's (lr, lc): its per-tile LDS offsets are recomputed in each tile's
// iteration instead of being hoisted to the kernel entry (where they spilled).
__device__ __forceinline__ int vr_opaque_lane(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

template <int NSMAX, int NRHS>
struct VrDims {
  static constexpr int R = (NSMAX + 15) / 16;           // row tiles
  static constexpr int T = (NSMAX + NRHS + 15) / 16;    // column tiles, right-hand sides included
  static constexpr int TPW = (R * T + NWAVE - 1) / NWAVE;  // tiles per wave
  static constexpr int PL = 17;                          // LDS row stride of the panel (odd: no bank conflicts)
  static constexpr int UL = 16 * T;                      // LDS row stride of U12
};

template <int NSMAX, int NRHS>
struct VrShared {
  double pan[NSMAX * VrDims<NSMAX, NRHS>::PL];  // panel (factorisation) / U column block (back substitution)
  double u12[16 * VrDims<NSMAX, NRHS>::UL];     // the panel's pivot rows, trailing columns from j_lo
  double bv[NSMAX];                             // back substitution: right-hand side by row
  uint64_t key[2][NWAVE];                       // pivot search, double-buffered by step parity
  int32_t kpos[2][NWAVE];
  int16_t step_of[NSMAX];  // LU step at which the row became a pivot row, −1 while remaining
  int16_t prow[NSMAX];     // pivot row of each step
  int8_t ps[NSMAX];        // the row's step within the current panel, −1 otherwise
};

// Wave-wide max of an unsigned 32-bit key (DPP row_shr 1/2/4/8, row_bcast 15/31), uniform.
__device__ __forceinline__ uint32_t vr_wave_max_u32(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false));
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// Pivot among the remaining rows (thread = row; key 0 = not a candidate, pivot_key
// otherwise): the largest key, ties to the smallest row.  Each wave reduces by DPP (the
// 64-bit key as two 32-bit maxima, then the lowest lane holding it: rows ascend with the
// lane), then the wave results meet in LDS (double-buffered by step parity): one barrier.
template <int NSMAX, int NRHS>
__device__ __forceinline__ int vr_pivot(VrShared<NSMAX, NRHS>& L, uint64_t key, int step) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t khi = (uint32_t)(key >> 32), klo = (uint32_t)key;
  const uint32_t mhi = vr_wave_max_u32(khi);
  const uint32_t mlo = vr_wave_max_u32(khi == mhi ? klo : 0u);
  const uint64_t win = __ballot(khi == mhi && klo == mlo);
  if (lane == 0) {
    const uint64_t wk = ((uint64_t)mhi << 32) | mlo;
    L.key[step & 1][wave] = wk;
    L.kpos[step & 1][wave] = wk ? (wave << 6) + (int)__ffsll((unsigned long long)win) - 1 : -1;
  }
  __syncthreads();
  uint64_t k = L.key[step & 1][0];
  int p = L.kpos[step & 1][0];
#pragma unroll
  for (int q = 1; q < NWAVE; ++q) better(k, p, L.key[step & 1][q], L.kpos[step & 1][q]);
  return p;
}

// entry(i, j): entry (i, j) of [K | rhs] (i < ns, j < ns + nrhs), computed once each, one
// column tile at a time into LDS and from there into the owners' tiles — the matrix is
// never written to memory.  x (LDS, ≥ ns): the solution of the last right-hand side; with
// xout also every right-hand side's at xout[c·ns + k].  false: an exact zero pivot (the
// failed solve of src/solver.jl:84-88).
struct NoPatch {
  static constexpr bool active = false;
  __device__ void operator()(int, double*, int) const {}
};

// `patch(tc, pan, PL)` (when active): every thread writes entries of column tile tc that
// differ from `entry` into the staged tile (pan[i·PL + j − 16·tc]) — the nonlinear SCHUR
// step's sparse Q D⁻¹ R terms, computed once per step beside the dense P + tol·I.
template <int NSMAX, int NRHS, bool RCP, class Entry, class Patch = NoPatch>
__device__ __forceinline__ bool lu_solve_vr(const Entry& entry, int ns, double* x, VrShared<NSMAX, NRHS>& L,
                                            int nrhs = 1, double* __restrict__ xout = nullptr,
                                            const Patch& patch = Patch{}) {
  using D = VrDims<NSMAX, NRHS>;
  constexpr int R = D::R, T = D::T, TPW = D::TPW, PL = D::PL, UL = D::UL;
  static_assert(NSMAX <= WG, "one thread per row");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ncols = ns + nrhs;
  d4 acc[TPW];
  // ---- [K | rhs] into the tiles, one column tile at a time through the panel buffer --
  for (int rep = 0; rep < (MCPX_VR_TWICE == 1 ? 2 : 1); ++rep)
  for (int tc = 0; tc < T; ++tc) {
    if (16 * tc >= ncols) break;  // uniform
    for (int q = tid; q < ns * 16; q += WG) {  // column-major: consecutive threads, consecutive rows
      const int c = q / ns, i = q - c * ns, j = 16 * tc + c;
      L.pan[i * PL + c] = j < ncols ? entry(i, j) : 0.0;
    }
    __syncthreads();
    if constexpr (Patch::active) {
      patch(tc, L.pan, PL);
      __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
      __builtin_amdgcn_sched_barrier(0);
      const int t = vr_opaque(wave) + NWAVE * u, ti = t % R, tj = t / R;
      const int ln_ = vr_opaque_lane(lane), lr = ln_ >> 4, lc = ln_ & 15;
      if (tj != tc) continue;  // uniform
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = 16 * ti + lr + 4 * e;
        acc[u][e] = row < ns ? L.pan[row * PL + lc] : 0.0;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int u = 0; u < TPW; ++u) {  // tiles beyond the last column: zero
    const int t = vr_opaque(wave) + NWAVE * u, tj = t / R;
    if (16 * tj >= ncols) acc[u] = d4{0.0, 0.0, 0.0, 0.0};
  }
  if (tid < NSMAX) L.step_of[tid] = -1;
  int step = 0;
  for (int k0 = 0; k0 < ns; k0 += 16) {
    const int tc = k0 >> 4, kb = min(16, ns - k0), j_lo = k0 + kb;
    // ---- the panel (columns k0 .. k0+kb−1 of every row) into LDS -------------------
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
      __builtin_amdgcn_sched_barrier(0);  // one tile at a time
      const int t = vr_opaque(wave) + NWAVE * u, ti = t % R, tj = t / R;
      const int ln_ = vr_opaque_lane(lane), lr = ln_ >> 4, lc = ln_ & 15;
      if (tj != tc || 16 * ti >= ns) continue;  // uniform
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = 16 * ti + lr + 4 * e;
        if (row < ns && lc < kb) L.pan[row * PL + lc] = acc[u][e];
      }
    }
    if (tid < NSMAX) L.ps[tid] = -1;
    __syncthreads();  // the staged panel before the first pivot search reads other tiles' rows
    // ---- factor it column by column: thread = row, its panel row in registers; after
    //      each column a remaining row stores its updated entries back, so the next
    //      pivot row is in LDS for everyone (one barrier per column) --------------------
    {
      double pr[16];
      const bool own = tid < ns;
      bool rem = own && L.step_of[own ? tid : 0] < 0;
#pragma unroll
      for (int q = 0; q < 16; ++q) pr[q] = (own && q < kb) ? L.pan[tid * PL + q] : 0.0;
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) {
        if (kk >= kb) continue;  // uniform
        const int pp = vr_pivot(L, rem ? pivot_key(pr[kk]) : 0ull, step);  // barrier inside
        ++step;
        const double* prw = L.pan + pp * PL;
        const double piv = prw[kk];
        if (piv == 0.0) return false;  // the failed linear solve of src/solver.jl:84-88
        if (tid == pp) {
          rem = false;
          L.step_of[pp] = (int16_t)(k0 + kk);
          L.prow[k0 + kk] = (int16_t)pp;
          L.ps[pp] = (int8_t)kk;
        } else if (rem) {
          const double l = RCP ? pr[kk] * (1.0 / piv) : pr[kk] / piv;
          double* row = L.pan + tid * PL;
#pragma unroll
          for (int jj = kk + 1; jj < 16; ++jj) {
            if (jj >= kb) continue;
            pr[jj] = fma(-l, prw[jj], pr[jj]);
            row[jj] = pr[jj];
          }
          pr[kk] = l;  // a_ik of a remaining row is never read again: keep l_ik there
          row[kk] = l;
        }
      }
    }
    __syncthreads();
    // ---- panel back into the tiles; U12 rows of the panel's pivot rows into LDS ----
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
      __builtin_amdgcn_sched_barrier(0);  // one tile at a time
      const int t = vr_opaque(wave) + NWAVE * u, ti = t % R, tj = t / R;
      const int ln_ = vr_opaque_lane(lane), lr = ln_ >> 4, lc = ln_ & 15;
      if (tj < tc || 16 * ti >= ns || 16 * tj >= ncols) continue;  // uniform
      const int col = 16 * tj + lc;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = 16 * ti + lr + 4 * e;
        if (row >= ns) continue;
        if (tj == tc && lc < kb) acc[u][e] = L.pan[row * PL + lc];
        const int s = L.ps[row];
        if (s >= 0 && col >= j_lo && col < ncols) L.u12[s * UL + col] = acc[u][e];
      }
    }
    __syncthreads();
    // ---- U12: in-panel forward substitution (thread = trailing column) -------------
    for (int j = j_lo + tid; j < ncols; j += WG) {  // (u_k2j re-read from LDS: the tiles hold the registers)
#pragma unroll
      for (int kk = 1; kk < 16; ++kk) {
        if (kk >= kb) continue;  // uniform
        const double* lrow = L.pan + L.prow[k0 + kk] * PL;
        double v = L.u12[kk * UL + j];
#pragma unroll
        for (int k2 = 0; k2 < kk; ++k2) v = fma(-lrow[k2], L.u12[k2 * UL + j], v);
        L.u12[kk * UL + j] = v;
      }
    }
    __syncthreads();
    // ---- trailing update of the remaining rows on the matrix cores; U12 into the
    //      pivot rows' tiles ------------------------------------------------------------
    const int kfull = kb & ~3;
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
      __builtin_amdgcn_sched_barrier(0);  // one tile at a time
      const int t = vr_opaque(wave) + NWAVE * u, ti = t % R, tj = t / R;
      const int ln_ = vr_opaque_lane(lane), lr = ln_ >> 4, lc = ln_ & 15;
      if (tj < tc || 16 * ti >= ns || 16 * tj + 15 < j_lo || 16 * tj >= ncols) continue;  // uniform
      const int col = 16 * tj + lc;
      const bool ctr = col >= j_lo && col < ncols;  // a trailing column
      const int ra = 16 * ti + lc;                   // A-fragment row of this lane
      const bool rema = ra < ns && L.step_of[ra] < 0;
      d4 c = acc[u];
      for (int q = 0; q < kfull; q += 4) {
        const int kk = q + lr;
        const double a = rema ? -L.pan[ra * PL + kk] : 0.0;
        const double b = ctr ? L.u12[kk * UL + col] : 0.0;
        c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = 16 * ti + lr + 4 * e;
        if (row >= ns || !ctr) continue;
        if (L.step_of[row] < 0) {
          double v = c[e];
          for (int kk = kfull; kk < kb; ++kk)  // width not a multiple of 4: same order on the VALU
            v = fma(-L.pan[row * PL + kk], L.u12[kk * UL + col], v);
          acc[u][e] = v;
        } else {
          const int s = L.ps[row];
          if (s >= 0) acc[u][e] = L.u12[s * UL + col];
        }
      }
    }
    __syncthreads();
  }
  // ---- back substitution, blocked by 16 columns (oracle order: row i takes
  //      fma(−u_ik, x_k, b_i) for k = ns−1 down to step_of(i)+1) -----------------------
  for (int rep = 0; rep < (MCPX_VR_TWICE == 2 ? 2 : 1); ++rep)
  for (int rc = 0; rc < nrhs; ++rc) {
    const int cb = ns + rc;
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
      __builtin_amdgcn_sched_barrier(0);  // one tile at a time
      const int t = vr_opaque(wave) + NWAVE * u, ti = t % R, tj = t / R;
      const int ln_ = vr_opaque_lane(lane), lr = ln_ >> 4, lc = ln_ & 15;
      if (tj != (cb >> 4) || 16 * ti >= ns) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = 16 * ti + lr + 4 * e;
        if (row < ns && lc == (cb & 15)) L.bv[row] = acc[u][e];
      }
    }
    for (int k0 = ((ns - 1) >> 4) << 4; k0 >= 0; k0 -= 16) {
      const int tc = k0 >> 4, kb = min(16, ns - k0);
#pragma unroll
      for (int u = 0; u < TPW; ++u) {  // U columns k0 .. k0+kb−1 of every row into LDS
        __builtin_amdgcn_sched_barrier(0);
        const int t = vr_opaque(wave) + NWAVE * u, ti = t % R, tj = t / R;
      const int ln_ = vr_opaque_lane(lane), lr = ln_ >> 4, lc = ln_ & 15;
        if (tj != tc || 16 * ti >= ns) continue;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = 16 * ti + lr + 4 * e;
          if (row < ns && lc < kb) L.pan[row * PL + lc] = acc[u][e];
        }
      }
      __syncthreads();
      if (wave == 0) {  // the block's pivot rows, serially: lane j holds pivot row p_{k0+j}
        const int j = lane < kb ? lane : 0;
        const int p = L.prow[k0 + j];
        const double* up = L.pan + p * PL;
        double bj = L.bv[p];
#pragma unroll
        for (int q = 15; q >= 0; --q) {
          if (q >= kb) continue;  // uniform
          const double uq = up[q];
          const double tq = RCP ? bj * (1.0 / uq) : bj / uq;  // lane q: x_{k0+q} = b_p / u_pk
          const double xq = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(tq), q),
                                             __builtin_amdgcn_readlane(__double2loint(tq), q));
          if (lane == q) x[k0 + q] = xq;
          if (lane < q) bj = fma(-uq, xq, bj);
        }
      }
      __syncthreads();
      if (tid < ns && L.step_of[tid] < k0) {  // every row of an earlier step: the block's terms
        double b = L.bv[tid];
        const double* ur = L.pan + tid * PL;
#pragma unroll
        for (int q = 15; q >= 0; --q)
          if (q < kb) b = fma(-ur[q], x[k0 + q], b);
        L.bv[tid] = b;
      }
      __syncthreads();
    }
    if (xout) {
      for (int k = tid; k < ns; k += WG) xout[(int64_t)rc * ns + k] = x[k];
      __syncthreads();
    }
  }
  return true;
}

}  // namespace wg
}  // namespace mcpx
