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
// writes the whole trailing matrix once per 16 columns), while here it is read once
// into the VGPRs of the workgroup's WG threads in the MFMA accumulator layout and never
// written back.  Tile (ti, tj) of 16×16 (rows 16ti.., columns 16tj.., right-hand sides
// as trailing columns) belongs to wave t mod NWAVE with t = tj·R + ti (column-major:
// every column tile spreads over the waves, so each panel's trailing update is
// balanced); in it lane (lr, lc) holds rows 16ti + lr + 4e (e < 4) of column 16tj + lc,
// the f64 MFMA's C layout.  Only the panel (all rows × 16 columns), the panel's U12 rows
// and the per-row bookkeeping pass through LDS.  At NSMAX = 208, 8 waves: 23 tiles = 92
// doubles per lane.
#pragma once

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

// Pivot of panel column kk among the remaining rows (thread = row), one barrier.
template <int NSMAX, int NRHS>
__device__ __forceinline__ int vr_pivot(VrShared<NSMAX, NRHS>& L, int ns, int kk, int step) {
  constexpr int PL = VrDims<NSMAX, NRHS>::PL;
  const int tid = threadIdx.x, wave = tid >> 6;
  uint64_t key = 0;
  int pos = -1;
  if (tid < ns && L.step_of[tid] < 0) {
    key = pivot_key(L.pan[tid * PL + kk]);
    pos = tid;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const uint64_t k2 = shfl_xor_u64(key, o);
    const int p2 = __shfl_xor(pos, o);
    better(key, pos, k2, p2);
  }
  if ((tid & 63) == 0) {
    L.key[step & 1][wave] = key;
    L.kpos[step & 1][wave] = pos;
  }
  __syncthreads();
  uint64_t k = L.key[step & 1][0];
  int p = L.kpos[step & 1][0];
#pragma unroll
  for (int q = 1; q < NWAVE; ++q) better(k, p, L.key[step & 1][q], L.kpos[step & 1][q]);
  return p;
}

// A: ns × (ns + nrhs) row-major (stride ld), read once, not modified.  x (LDS, ≥ ns):
// the solution of the last right-hand side; with xout also every right-hand side's at
// xout[c·ns + k].  false: an exact zero pivot (the failed solve of src/solver.jl:84-88).
template <int NSMAX, int NRHS, bool RCP>
__device__ __forceinline__ bool lu_solve_vr(const double* __restrict__ A, int ld, int ns, double* x,
                                            VrShared<NSMAX, NRHS>& L, int nrhs = 1,
                                            double* __restrict__ xout = nullptr) {
  using D = VrDims<NSMAX, NRHS>;
  constexpr int R = D::R, TPW = D::TPW, PL = D::PL, UL = D::UL;
  static_assert(NSMAX <= WG, "one thread per row");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane >> 4, lc = lane & 15;
  const int ncols = ns + nrhs;
  d4 acc[TPW];
  // ---- [K | rhs] into the tiles (the only read of A) -------------------------------
#pragma unroll
  for (int u = 0; u < TPW; ++u) {
    const int t = vr_opaque(wave) + NWAVE * u, ti = t % R, tj = t / R;
      const int ln_ = vr_opaque_lane(lane), lr = ln_ >> 4, lc = ln_ & 15;
    const int col = 16 * tj + lc;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = 16 * ti + lr + 4 * e;
      acc[u][e] = (row < ns && col < ncols) ? A[(int64_t)row * ld + col] : 0.0;
    }
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
    // ---- factor it column by column (thread = row; one barrier per column) ---------
    for (int kk = 0; kk < kb; ++kk, ++step) {
      const int pp = vr_pivot(L, ns, kk, step);  // barrier inside: the previous update is visible
      const double piv = L.pan[pp * PL + kk];
      if (piv == 0.0) return false;
      const double rp = RCP ? 1.0 / piv : 1.0;
      if (tid == pp) {
        L.step_of[pp] = (int16_t)(k0 + kk);
        L.prow[k0 + kk] = (int16_t)pp;
        L.ps[pp] = (int8_t)kk;
      } else if (tid < ns && L.step_of[tid] < 0) {
        double* row = L.pan + tid * PL;
        const double l = RCP ? row[kk] * rp : row[kk] / piv;
        for (int jj = kk + 1; jj < kb; ++jj) row[jj] = fma(-l, L.pan[pp * PL + jj], row[jj]);
        row[kk] = l;  // a_ik of a remaining row is never read again: keep l_ik there
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
      for (int kk = 1; kk < kb; ++kk) {
        const double* lrow = L.pan + L.prow[k0 + kk] * PL;
        double v = L.u12[kk * UL + j];
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
        for (int q = kb - 1; q >= 0; --q) {
          const double uq = up[q];
          const double tq = RCP ? bj * (1.0 / uq) : bj / uq;  // lane q: x_{k0+q} = b_p / u_pk
          const double xq = __shfl(tq, q);
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
