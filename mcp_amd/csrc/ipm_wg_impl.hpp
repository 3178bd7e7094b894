// ipm_wg_impl.hpp — workgroup-per-instance solver for KKT systems too large for
// one wave (the register-resident kernels of ipm_kernel_impl.hpp stop at 64
// rows).  SURVEY.md §8(f) #2: the reference's trajectory games reach KKT
// dimension 700 at horizon T = 10 (benchmark/trajectory_game_benchmark.jl:38).
//
// One workgroup of 256 threads (4 waves) runs the whole ϵ-continuation / Newton
// loop of src/solver.jl:64-121 for one instance at a time, taking instances from
// an atomic work queue (grid = the resident workgroups, so imbalance between
// instances — 12 to 931 Newton steps — evens out).  Per workgroup slot the host
// allocates a workspace in HBM: the linear system [K | rhs] row-major (ld ≥ NS+1)
// and, for the nonlinear family, the generated Jacobian blocks.  Systems of at most
// MCPX_VR_MAX rows skip the [K | rhs] workspace: their entries go straight into the
// registers of the register-resident LU (lu_vr.hpp), same arithmetic.
//
// The Newton system is factored by a right-looking blocked LU with partial
// pivoting that reproduces oracle/ipm_oracle.c::lu_solve bit for bit:
//   * implicit pivoting: rows are never moved; the remaining rows are kept as a
//     list in ascending row order, and the pivot of column k is the first
//     remaining row of largest |a_ik| (NaN never wins; all-NaN → first row);
//   * panel of NB = 16 columns staged in LDS and factored column by column
//     (multipliers l_i = a_ik / pivot, a_ij ← fma(−l_i, u_j, a_ij));
//   * the panel's pivot rows get their trailing part (U12, the rhs included) by
//     the in-panel forward substitution — the same fma chain the unblocked
//     elimination applies to them;
//   * every other remaining row gets the trailing update C ← C + (−L21)·U12 on
//     the matrix cores: v_mfma_f64_16x16x4_f64 equals an ordered k-ascending fma
//     chain bitwise (tools/ubench_mfma64.hip), so each entry sees
//     exactly the oracle's sequence fma(−l_ik, u_kj, ·), k ascending; a panel
//     width that is not a multiple of 4 finishes on the VALU in the same order;
//   * column-oriented back substitution, x_k = b_p / u_pk.
// Residual, Jacobian rows, slack / y eliminations, line search and update follow
// the oracle's solve_one() op for op (same fma chains, same order); the nonlinear
// SCHUR elimination takes the terms of Q's and R's structural nonzeros only, as
// the oracle does (the generated mcpx_nl_qk_* / mcpx_nl_rj_* tables).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "ipm_wg.h"

namespace mcpx {
namespace wg {

constexpr int WG = kThreads;  // threads per workgroup
constexpr int NWAVE = WG / 64;
constexpr int NB = 16;   // LU panel width

typedef double d4 __attribute__((ext_vector_type(4)));

// ---- workgroup reductions (all threads call; result uniform) ----------------

struct Scratch {
  double d[NWAVE];
  uint64_t u[NWAVE];
  uint64_t u2[NWAVE];
  int32_t i[NWAVE];
  int32_t inst;
};

__device__ __forceinline__ double max_nan(double a, double b) { return (a != a || b != b) ? a + b : fmax(a, b); }

__device__ __forceinline__ double shfl_xor_d(double v, int m) {
  const int lo = __shfl_xor(__double2loint(v), m), hi = __shfl_xor(__double2hiint(v), m);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m), hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m);
  return ((uint64_t)hi << 32) | lo;
}

// NaN-propagating max of non-negative values (‖F‖∞ of src/solver.jl:107).
__device__ __forceinline__ double wg_max_nan(double v, Scratch& s) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = max_nan(v, shfl_xor_d(v, o));
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) s.d[w] = v;
  __syncthreads();
  double r = s.d[0];
#pragma unroll
  for (int q = 1; q < NWAVE; ++q) r = max_nan(r, s.d[q]);
  return r;
}

__device__ __forceinline__ uint64_t wg_or(uint64_t v, Scratch& s) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v |= shfl_xor_u64(v, o);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) s.u[w] = v;
  __syncthreads();
  uint64_t r = 0;
#pragma unroll
  for (int q = 0; q < NWAVE; ++q) r |= s.u[q];
  return r;
}

// Largest key, ties to the smallest position (pos < 0: no candidate).
__device__ __forceinline__ void better(uint64_t& k, int& p, uint64_t k2, int p2) {
  if (k2 > k || (k2 == k && p2 >= 0 && (p < 0 || p2 < p))) {
    k = k2;
    p = p2;
  }
}
__device__ __forceinline__ int wg_argmax(uint64_t key, int pos, Scratch& s) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const uint64_t k2 = shfl_xor_u64(key, o);
    const int p2 = __shfl_xor(pos, o);
    better(key, pos, k2, p2);
  }
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    s.u2[w] = key;
    s.i[w] = pos;
  }
  __syncthreads();
  uint64_t k = s.u2[0];
  int p = s.i[0];
#pragma unroll
  for (int q = 1; q < NWAVE; ++q) better(k, p, s.u2[q], s.i[q]);
  return p;
}

// Pivot-search key of a remaining row: NaN never wins over a number (oracle:
// `v > bv` is false for NaN), an all-NaN column takes the first remaining row.
__device__ __forceinline__ uint64_t pivot_key(double a) {
  const double v = fabs(a);
  if (v != v) return 1ull;
  return (uint64_t)__double_as_longlong(v) + 2ull;
}

// ---- blocked LU with partial pivoting (oracle lu_solve) --------------------
//
// A: ns × (ns + nrhs) row-major with stride ld, columns ns .. ns+nrhs−1 = right-hand
// sides (each sees exactly the oracle's single-rhs chain: they are trailing columns of the
// same elimination); destroyed.  x (LDS, ≥ ns): the solution of the last right-hand side,
// x[k] = δz_k; with xout, the solution of right-hand side c is also stored at
// xout[c·ns + k] (the sensitivity kernels' several partials).
template <int NSMAX>
struct LuShared {
  double pan[NSMAX * NB];     // the panel, row q = remaining-list position q
  double bb[NB];              // back substitution: rhs of the block's pivot rows
  uint64_t key[2][NWAVE];     // pivot search, double-buffered by step parity
  int32_t kpos[2][NWAVE];
  int16_t rem[NSMAX];         // remaining rows, ascending
  int16_t step_of[NSMAX];
  int16_t prow[NSMAX];
  int16_t pivpos[NB];
  uint8_t ispiv[NSMAX];
  int32_t cnt[NWAVE];
};

// One pivot search per column with a single barrier: every thread owns the panel
// rows q ≡ tid (mod 256) for the whole panel (their updates and pivot flags are
// its own), so the only cross-thread data of a step are the 4 wave maxima and the
// pivot row, both published before the barrier of the step's search.
template <int NSMAX>
__device__ __forceinline__ int panel_pivot(LuShared<NSMAX>& L, int r, int kk, int step) {
  const int tid = threadIdx.x, wave = tid >> 6;
  uint64_t key = 0;
  int pos = -1;
  for (int q = tid; q < r; q += WG)
    if (!L.ispiv[q]) better(key, pos, pivot_key(L.pan[q * NB + kk]), q);
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

// RCP: the reciprocal-multiplier arithmetic of oracle lu_solve_x (rcp = 1; the SCHUR step of
// generated nonlinear modules): l = a_ik · (1 / piv), x_k = b_p · (1 / u_kk).
template <int NSMAX, bool RCP = false>
__device__ __forceinline__ bool lu_solve(double* __restrict__ A, int ld, int ns, double* x, LuShared<NSMAX>& L,
                                         int nrhs = 1, double* __restrict__ xout = nullptr) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < ns; i += WG) L.rem[i] = (int16_t)i;
  int r = ns;  // remaining rows (list length)
  int step = 0;
  __syncthreads();
  for (int k0 = 0; k0 < ns; k0 += NB) {
    const int kb = min(NB, ns - k0);
    // ---- stage the panel columns [k0, k0+kb) of the remaining rows (own rows) ----
    for (int q = tid; q < r; q += WG) {
      const double* src = A + (int64_t)L.rem[q] * ld + k0;
#pragma unroll
      for (int kk = 0; kk < NB; ++kk)
        if (kk < kb) L.pan[q * NB + kk] = src[kk];
      L.ispiv[q] = 0;
    }
    // ---- factor the panel column by column (one barrier per column) -----------
    for (int kk = 0; kk < kb; ++kk, ++step) {
      const int pp = panel_pivot(L, r, kk, step);  // barrier inside: the previous update is visible
      const double piv = L.pan[pp * NB + kk];
      if (piv == 0.0) return false;  // the failed linear solve of src/solver.jl:84-88
      const double rp = RCP ? 1.0 / piv : 1.0;
      if (tid == (pp & (WG - 1))) {  // the owner of the pivot row
        L.ispiv[pp] = 1;
        L.pivpos[kk] = (int16_t)pp;
        L.prow[k0 + kk] = L.rem[pp];
        L.step_of[L.rem[pp]] = (int16_t)(k0 + kk);
      }
      for (int q = tid; q < r; q += WG) {
        if (q == pp || L.ispiv[q]) continue;
        double* row = L.pan + q * NB;
        const double l = RCP ? row[kk] * rp : row[kk] / piv;
        for (int jj = kk + 1; jj < kb; ++jj) row[jj] = fma(-l, L.pan[pp * NB + jj], row[jj]);
        row[kk] = l;  // a_ik of a remaining row is never read again: keep l_ik there
      }
    }
    __syncthreads();
    // panel back to A: U11 in the pivot rows (their left part holds multipliers, never read)
    for (int q = tid; q < r; q += WG) {
      double* dst = A + (int64_t)L.rem[q] * ld + k0;
#pragma unroll
      for (int kk = 0; kk < NB; ++kk)
        if (kk < kb) dst[kk] = L.pan[q * NB + kk];
    }
    // ---- U12: in-panel forward substitution of the pivot rows' trailing part -
    const int j_lo = k0 + kb;  // trailing columns j_lo .. ns+nrhs−1 (right-hand sides from column ns)
    const int jend = ns + nrhs;
    for (int j = j_lo + tid; j < jend; j += WG) {
      double u[NB];
#pragma unroll
      for (int kk = 0; kk < NB; ++kk) {
        if (kk >= kb) continue;
        const int pp = L.pivpos[kk];
        double v = A[(int64_t)L.rem[pp] * ld + j];
#pragma unroll
        for (int k2 = 0; k2 < NB; ++k2)
          if (k2 < kk) v = fma(-L.pan[pp * NB + k2], u[k2], v);
        u[kk] = v;
        A[(int64_t)L.rem[pp] * ld + j] = v;
      }
    }
    __syncthreads();
    // ---- trailing update of the other remaining rows on the matrix cores -----
    const int ncol = jend - j_lo;
    if (ncol > 0 && r > kb) {
      const int rt = (r + 15) / 16, ct = (ncol + 15) / 16;
      const int lr = lane >> 4, lc = lane & 15;
      // U12 row of panel step kk: A + rem[pivpos[kk]]·ld (read from LDS where needed: kk is per lane)
      auto urow = [&](int kk) { return (int64_t)L.rem[L.pivpos[kk]] * ld; };
      for (int t = wave; t < rt * ct; t += NWAVE) {
        const int ti = t / ct, tj = t - ti * ct;
        const int j = j_lo + 16 * tj + lc;
        const bool jin = j < jend;
        d4 acc;
        int64_t rowo[4];
        bool rin[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int pos = 16 * ti + lr + 4 * e;
          rin[e] = pos < r && !L.ispiv[pos < r ? pos : 0];
          rowo[e] = pos < r ? (int64_t)L.rem[pos] * ld : 0;
          acc[e] = (rin[e] && jin) ? A[rowo[e] + j] : 0.0;
        }
        const int pa = 16 * ti + lc;  // A-fragment row of this lane
        if (kb == NB) {  // the common full panel: 4 K-chunks, loads hoisted ahead of the MFMA chain
          double av[NB / 4], bv[NB / 4];
#pragma unroll
          for (int c = 0; c < NB / 4; ++c) {
            const int kk = 4 * c + lr;
            av[c] = pa < r ? -L.pan[pa * NB + kk] : 0.0;
            bv[c] = jin ? A[urow(kk) + j] : 0.0;
          }
#pragma unroll
          for (int c = 0; c < NB / 4; ++c) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[c], bv[c], acc, 0, 0, 0);
        } else {
          const int kfull = kb & ~3;
          for (int c = 0; c < kfull; c += 4) {
            const int kk = c + lr;
            const double a = pa < r ? -L.pan[pa * NB + kk] : 0.0;
            const double b = jin ? A[urow(kk) + j] : 0.0;
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
          }
          for (int kk = kfull; kk < kb; ++kk) {  // width not a multiple of 4: same order on the VALU
            const double b = jin ? A[urow(kk) + j] : 0.0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int pos = 16 * ti + lr + 4 * e;
              const double l = pos < r ? L.pan[pos * NB + kk] : 0.0;
              acc[e] = fma(-l, b, acc[e]);
            }
          }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (rin[e] && jin) A[rowo[e] + j] = acc[e];
      }
    }
    __syncthreads();
    // ---- drop the panel's pivot rows from the remaining list (stable) --------
    // A kept row only moves left (dst ≤ pos), and every source of a chunk is read
    // before the barrier that precedes its writes, so the list compacts in place.
    int base = 0;
    for (int c0 = 0; c0 < r; c0 += WG) {
      const int pos = c0 + tid;
      const bool f = pos < r && !L.ispiv[pos < r ? pos : 0];
      const int16_t v = pos < r ? L.rem[pos] : (int16_t)0;
      const uint64_t bal = __ballot(f);
      const int before = __popcll(bal & ((1ull << lane) - 1ull));
      if (lane == 0) L.cnt[wave] = __popcll(bal);
      __syncthreads();
      int off = base, tot = 0;
#pragma unroll
      for (int q = 0; q < NWAVE; ++q) {
        off += (q < wave) ? L.cnt[q] : 0;
        tot += L.cnt[q];
      }
      __syncthreads();  // every thread has read cnt and its source entry
      if (f) L.rem[off + before] = v;
      base += tot;
    }
    r = base;
    __syncthreads();
  }
  // ---- back substitution, blocked by 16 columns ---------------------------------
  // Oracle order: row i takes fma(−u_ik, x_k, b_i) for k = ns−1 down to step_of(i)+1.
  // Per block [k0, k0+16), descending: wave 0 solves the block's 16 pivot rows
  // (each already updated by every later block) serially in registers, then every
  // row of an earlier step takes the block's 16 updates, k descending.
  constexpr int RPT = (NSMAX + WG - 1) / WG;  // rows per thread (rows i ≡ tid mod 256)
  double b[RPT];
  int st[RPT];
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int i = q * WG + tid;
    st[q] = i < ns ? L.step_of[i] : 0x7fff;
  }
  const int nblk = (ns + NB - 1) / NB;
  for (int rc = 0; rc < nrhs; ++rc) {  // one back substitution per right-hand side
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int i = q * WG + tid;
    b[q] = i < ns ? A[(int64_t)i * ld + ns + rc] : 0.0;
  }
  for (int blk = nblk - 1; blk >= 0; --blk) {
    const int k0 = blk * NB, kb = min(NB, ns - k0);
    // the block's pivot rows publish their rhs (final but for the block's own terms)
#pragma unroll
    for (int q = 0; q < RPT; ++q)
      if (st[q] >= k0 && st[q] < k0 + kb) L.bb[st[q] - k0] = b[q];
    __syncthreads();
    if (wave == 0) {
      // lane j (< kb) holds pivot row p_{k0+j}: its rhs and u_{p, k0..k0+kb-1}
      const int j = lane < kb ? lane : 0;
      const int64_t ro = (int64_t)L.prow[k0 + j] * ld + k0;
      double bj = L.bb[j];
      double uj[NB];
#pragma unroll
      for (int c = 0; c < NB; ++c) uj[c] = (c < kb) ? A[ro + c] : 0.0;
#pragma unroll
      for (int c = NB - 1; c >= 0; --c) {
        if (c >= kb) continue;
        const double t = RCP ? bj * (1.0 / uj[c]) : bj / uj[c];  // lane c: x_{k0+c} = b_p / u_pk
        const double xc = __shfl(t, c);
        if (lane == c) x[k0 + c] = xc;
        if (lane < c) bj = fma(-uj[c], xc, bj);
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const int i = q * WG + tid;
      if (i >= ns || st[q] >= k0) continue;
      const double* ur = A + (int64_t)i * ld + k0;
#pragma unroll
      for (int c = NB - 1; c >= 0; --c)
        if (c < kb) b[q] = fma(-ur[c], x[k0 + c], b[q]);
    }
  }
  __syncthreads();
  if (xout) {
    for (int k = tid; k < ns; k += WG) xout[(int64_t)rc * ns + k] = x[k];
    __syncthreads();
  }
  }  // right-hand side c
  return true;
}

}  // namespace wg
}  // namespace mcpx

#include "lu_vr.hpp"  // the register-resident LU (uses the helpers above)
#include "gj_vr.hpp"  // the QP family's SCHUR step: MFMA Schur complement + blocked Gauss-Jordan

namespace mcpx {
namespace wg {

// ---- the solver -------------------------------------------------------------

// The generated code of a nonlinear module (csrc/ipm_nl_kernel.hpp) or nothing.
struct NoGen {
  static constexpr int OFF_P = 0, OFF_Q = 0, OFF_R = 0, OFF_G = 0, OFF_H = 0, OFF_S = 0, SIZE = 0;
  static constexpr bool HAS_S = false;
  __device__ static void init(const double*, double*) {}
  __device__ static void eval(const double*, const double*, double*) {}
  __device__ static void eval_theta(const double*, const double*, double*) {}
  __device__ static const int32_t* tc_ptr() { return nullptr; }
  __device__ static const int32_t* tc_idx() { return nullptr; }
  __device__ static const int32_t* tr_ptr() { return nullptr; }
  __device__ static const int32_t* tr_idx() { return nullptr; }
  __device__ static const int32_t* qk_ptr() { return nullptr; }
  __device__ static const int32_t* qk_idx() { return nullptr; }
  __device__ static const int32_t* rj_ptr() { return nullptr; }
  __device__ static const int32_t* rj_idx() { return nullptr; }
  static constexpr int SE_ER = 1, SE_KT = 1;
  __device__ static const int32_t* se_pos() { return nullptr; }
  __device__ static const int32_t* se_k() { return nullptr; }
};

// Row i of F (src/mcp.jl:76-80) at z = zs, oracle family_row() op for op.
template <int FAMILY, class GEN>
__device__ __forceinline__ double residual(const double* __restrict__ th, const double* __restrict__ blk,
                                           const double* zs, int n, int m, double eps, int i) {
  const int nn = n * n, nm = n * m, mm = m * m;
  if (i < n) {
    if constexpr (FAMILY == MCPX_FAMILY_NONLINEAR) {
      return blk[GEN::OFF_G + i];
    } else {
      double acc = 0.0;
      for (int j = 0; j < n; ++j) acc = fma(th[j * n + i], zs[j], acc);  // M_ij / P_ij
      if constexpr (FAMILY == MCPX_FAMILY_QP) {
        for (int k = 0; k < m; ++k) acc = fma(-th[nn + i * m + k], zs[n + k], acc);  // −A_ki
        return acc - th[nn + nm + m + i];                                           // − ϕ_i
      } else {
        for (int k = 0; k < m; ++k) acc = fma(th[nn + k * n + i], zs[n + k], acc);   // Q_ik
        return acc + th[nn + 2 * nm + mm + i];                                      // + g_i
      }
    }
  } else if (i < n + m) {
    const int k = i - n;
    if constexpr (FAMILY == MCPX_FAMILY_NONLINEAR) {
      return blk[GEN::OFF_H + k] - zs[n + m + k];
    } else {
      double acc = 0.0;
      if constexpr (FAMILY == MCPX_FAMILY_QP) {
        for (int j = 0; j < n; ++j) acc = fma(th[nn + j * m + k], zs[j], acc);  // A_kj
        return (acc - th[nn + nm + k]) - zs[n + m + k];
      } else {
        for (int j = 0; j < n; ++j) acc = fma(th[nn + nm + j * m + k], zs[j], acc);  // R_kj
        for (int q = 0; q < m; ++q) acc = fma(th[nn + 2 * nm + q * m + k], zs[n + q], acc);  // S_kq
        return (acc + th[nn + 2 * nm + mm + n + k]) - zs[n + m + k];
      }
    }
  }
  const int k = i - n - m;
  return zs[n + m + k] * zs[n + k] - eps;  // s ⊙ y − ϵ
}

// ∇F_z[i][j] without tol·I (src/mcp.jl:97-120), oracle family_row() entries.
template <int FAMILY, class GEN>
__device__ __forceinline__ double jac(const double* __restrict__ th, const double* __restrict__ blk,
                                      const double* zs, int n, int m, int i, int j) {
  const int nn = n * n, nm = n * m;
  if (i < n) {  // G rows
    if (j < n) return FAMILY == MCPX_FAMILY_NONLINEAR ? blk[GEN::OFF_P + j * n + i] : th[j * n + i];
    if (j < n + m) {
      const int k = j - n;
      if constexpr (FAMILY == MCPX_FAMILY_QP) return -th[nn + i * m + k];
      else if constexpr (FAMILY == MCPX_FAMILY_NONLINEAR) return blk[GEN::OFF_Q + k * n + i];
      else return th[nn + k * n + i];
    }
    return 0.0;
  }
  if (i < n + m) {  // H − s rows
    const int k = i - n;
    if (j < n) {
      if constexpr (FAMILY == MCPX_FAMILY_QP) return th[nn + j * m + k];
      else if constexpr (FAMILY == MCPX_FAMILY_NONLINEAR) return blk[GEN::OFF_R + j * m + k];
      else return th[nn + nm + j * m + k];
    }
    if (j < n + m) {
      const int q = j - n;
      if constexpr (FAMILY == MCPX_FAMILY_QP) return 0.0;
      else if constexpr (FAMILY == MCPX_FAMILY_NONLINEAR) return GEN::HAS_S ? blk[GEN::OFF_S + q * m + k] : 0.0;
      else return th[nn + 2 * nm + q * m + k];
    }
    return (j - n - m == k) ? -1.0 : 0.0;
  }
  const int k = i - n - m;  // s ⊙ y − ϵ rows
  if (j == n + k) return zs[n + m + k];
  if (j == n + m + k) return zs[n + k];
  return 0.0;
}

// MCPX_WG_TWICE (diagnostic builds only, tools/ab_build.py): 1 the register LU (lu_solve_vr)
// of the QP / affine step runs twice, 2 the residual F; the QP SCHUR step (gj_vr.hpp): 3 the
// formation and the Gauss-Jordan, 4 the formation, 5 rr, 6 δy and δs — all idempotent (same
// bits, the added time is the phase's cost).
#ifndef MCPX_WG_TWICE
#define MCPX_WG_TWICE 0
#endif
// Systems of up to MCPX_VR_MAX rows are factored in registers (lu_vr.hpp), larger ones
// through the slot's HBM workspace (lu_solve above).
#ifndef MCPX_VR_MAX
#define MCPX_VR_MAX 200
#endif
template <int NSMAX>
constexpr bool kVr = NSMAX <= MCPX_VR_MAX;

// lu_solve_vr's patch of the nonlinear SCHUR step: the entries of column tile tc among the
// generated mcpx_nl_se_* entries (position i·(n+1) + j, value sv[e]).
template <class GEN>
struct SePatch {
  static constexpr bool active = true;
  const double* sv;
  int n;
  __device__ void operator()(int tc, double* pan, int PL) const {
    const int32_t* sp = GEN::se_pos();
    for (int e = threadIdx.x; e < 64 * GEN::SE_ER; e += WG) {
      const int pos = sp[e];
      if (pos < 0) continue;
      const int i = pos / (n + 1), j = pos - i * (n + 1);
      if ((j >> 4) == tc) pan[i * PL + (j & 15)] = sv[e];
    }
  }
};

// The QP SCHUR step (gj_vr.hpp) and its pivoting-LU fallback share their LDS: one or the other
// is live.
template <int NSMAX>
union VrGjShared {
  VrShared<NSMAX, 1> vr;
  GjShared<NSMAX> gj;
};

template <int NVMAX, int NSMAX, bool VR = kVr<NSMAX>, bool GJ = false>
struct SolveShared {
  double zs[NVMAX], Fs[NVMAX], dzs[NVMAX];
  std::conditional_t<GJ, VrGjShared<NSMAX>, std::conditional_t<VR, VrShared<NSMAX, 1>, LuShared<NSMAX>>> lu;
  Scratch sc;
};

template <int FAMILY, int SOLVER, int NVMAX, int NSMAX, class GEN>
__device__ __forceinline__ void solve_instances(const WgArgs& W) {
  constexpr bool SCH = SOLVER == MCPX_LINSOLVE_SCHUR, RED = SOLVER == MCPX_LINSOLVE_REDUCED;
  constexpr bool NL = FAMILY == MCPX_FAMILY_NONLINEAR;
  // QP SCHUR (gj_vr.hpp): the Schur complement on the matrix cores, blocked Gauss-Jordan
  constexpr bool QPS = SCH && FAMILY == MCPX_FAMILY_QP;
  constexpr bool NLS = SCH && NL;  // the nonlinear family's SCHUR (generated tables; GEN's null tables otherwise)
  static_assert(!SCH || QPS || (NL && !GEN::HAS_S), "the workgroup SCHUR path: QP, or the nonlinear family's dH/dy = 0");
  static_assert(!QPS || kVr<NSMAX>, "the QP SCHUR step is register-resident");
  __shared__ SolveShared<NVMAX, NSMAX, kVr<NSMAX>, QPS> S;
  // QP SCHUR: D⁻¹, 1 / w, ry, ty per constraint and rr per row, in LDS
  __shared__ double qd[QPS ? NVMAX / 2 : 1], qw[QPS ? NVMAX / 2 : 1], qy[QPS ? NVMAX / 2 : 1],
      qt[QPS ? NVMAX / 2 : 1], qr[QPS ? NSMAX : 1];
  // QP SCHUR: the instance's A block in LDS when it fits (every Newton step reads it five times:
  // the residual's H rows aside, rr, the Schur complement's two fragments, δy)
  __shared__ double sA[QPS ? kGjACap<NVMAX> : 1];
  const KernelArgs& a = W.k;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = a.n, m = a.m, N = n + 2 * m;
  const int ns = SCH ? n : (RED ? n + m : N);
  const int ld = W.ld;
  const double tol = a.tol;
  double* const slot = W.work + (int64_t)blockIdx.x * W.slot_stride;
  double* const Am = slot;
  double* const blk = slot + W.off_blk;
  double* const sD = slot + W.off_aux;
  double* const srw = sD + m;
  double* const sry = sD + 2 * m;
  double* const sty = sD + 3 * m;
  double* const zs = S.zs;
  double* const Fs = S.Fs;
  double* const dzs = S.dzs;
  __shared__ double sv[NLS && kVr<NSMAX> ? 64 * GEN::SE_ER : 1];  // VR SCHUR: the sparse entries of [S | rr]

  for (;;) {
    if (tid == 0) S.sc.inst = atomicAdd(W.counter, 1);  // the work queue
    __syncthreads();
    const int64_t inst = S.sc.inst;
    __syncthreads();
    if (inst >= W.batch) break;  // every workgroup reaches this exit
    const double* __restrict__ th = a.theta + inst * a.theta_ld;

    // src/solver.jl:39-41, 64-66: x₀ = 0, y₀ = 1, s₀ = 1 unless warm-started
    for (int i = tid; i < N; i += WG) {
      double v;
      if (i < n) v = a.x0 ? a.x0[inst * n + i] : 0.0;
      else if (i < n + m) v = a.y0 ? a.y0[inst * m + (i - n)] : 1.0;
      else v = a.s0 ? a.s0[inst * m + (i - n - m)] : 1.0;
      zs[i] = v;
    }
    if constexpr (NL) {
      for (int i = tid; i < GEN::SIZE; i += WG) blk[i] = 0.0;  // structural zeros
      __syncthreads();
      if (tid == 0) GEN::init(th, blk);
    }
    __syncthreads();
    // QP SCHUR: M exactly symmetric ⇒ S symmetric ⇒ the pivot-free Gauss-Jordan first (the
    // oracle's m_sym), else the pivoting LU at every step.  Once per instance.
    bool msym = false, a_lds = false;
    if constexpr (QPS) {
      a_lds = n * kGjLda(m) <= kGjACap<NVMAX>;
      if (a_lds)
        for (int q = tid; q < n * m; q += WG) sA[(q / m) * kGjLda(m) + q % m] = th[(int64_t)n * n + q];
      uint64_t asym = 0;
      for (int q = tid; q < n * n; q += WG) {
        const int j = q / n, i = q - j * n;
        asym |= !(th[(int64_t)j * n + i] == th[(int64_t)i * n + j]);
      }
      msym = wg_or(asym, S.sc) == 0;
    }

    double eps = 1.0;                   // :67
    double kkt = __builtin_huge_val();  // :68
    int status = 0;                     // :69
    int outer = 1;                      // :70
    int newton = 0;
    unsigned reason = 0;  // MCPX_FAIL_* events
    while (kkt > tol && eps > tol && outer < a.max_outer) {  // :71
      int inner = 1;                                          // :72
      status = 0;                                             // :73
      while (kkt > eps && inner < a.max_inner) {              // :75
        // ---- F!, ∇F_z! (:79-81) ------------------------------------------------
        if constexpr (NL) {
          if (tid == 0) GEN::eval(th, zs, blk);
          __syncthreads();
        }
        double mx = 0.0;
        for (int rep = 0; rep < (MCPX_WG_TWICE == 2 ? 2 : 1); ++rep)
        for (int i = tid; i < N; i += WG) {
          const double f = residual<FAMILY, GEN>(th, blk, zs, n, m, eps, i);
          Fs[i] = f;
          mx = max_nan(mx, fabs(f));
        }
        const double kkt_step = wg_max_nan(mx, S.sc);  // ‖F‖∞ (:107), committed after the step
        // ---- the Newton system (:81-83) as [K | rhs] -------------------------------
        if constexpr (QPS) {  // the oracle's SCHUR branch (solve_one), QP family
          for (int k = tid; k < m; k += WG) {
            const double rw = 1.0 / (zs[n + k] + tol);  // 1 / J[c][c], J[c][c] = y_k + tol
            const double D = (0.0 + tol) + zs[n + m + k] * rw;
            const double Di = 1.0 / D;
            const double ry = (-Fs[n + k]) - (Fs[n + m + k] * rw);
            qd[k] = Di;
            qw[k] = rw;
            qy[k] = ry;
            qt[k] = ry * Di;
          }
          __syncthreads();
          // tA: row j of Aᵀ at tA[j·la] (θ: la = m; the LDS copy: kGjLda(m))
          auto rr = [&](const double* __restrict__ tA, int la) {
            for (int i = tid; i < n; i += WG) {  // rr_i = −F_Gi + Σ_k A_ki ty_k
              double acc = -Fs[i];
              for (int k = 0; k < m; ++k) acc = fma(tA[(int64_t)i * la + k], qt[k], acc);
              qr[i] = acc;
            }
          };
          for (int rep = 0; rep < (MCPX_WG_TWICE == 5 ? 2 : 1); ++rep) {
            if (a_lds) rr(sA, kGjLda(m));
            else rr(th + (int64_t)n * n, m);
          }
          __syncthreads();
        } else if constexpr (SCH) {
          // eliminate δs_k (pivot w_k = y_k + tol), then δy_k (pivot D_k = (0 + tol) + s_k / w_k)
          for (int k = tid; k < m; k += WG) {
            const double rw = 1.0 / (zs[n + k] + tol);
            const double D = (0.0 + tol) + zs[n + m + k] * rw;
            const double Di = 1.0 / D;
            const double ry = (-Fs[n + k]) - (Fs[n + m + k] * rw);
            sD[k] = Di;
            srw[k] = rw;
            sry[k] = ry;
            sty[k] = ry * Di;
          }
          __syncthreads();
        }
        // VR SCHUR: the entries of [S | rr] beyond P + tol·I and −F_G (the generated
        // mcpx_nl_se_* tables: 360 at T = 10), each with its fma chain, once per step into
        // LDS; the LU's staging writes them over the dense part (`patch`)
        if constexpr (NLS && kVr<NSMAX>) {
          const int32_t* sp = GEN::se_pos();
          const int32_t* sk = GEN::se_k();
          for (int e = tid; e < 64 * GEN::SE_ER; e += WG) {
            const int pos = sp[e];
            if (pos < 0) continue;
            const int i = pos / (n + 1), j = pos - i * (n + 1), r = e >> 6, l = e & 63;
            double v = j < n ? blk[GEN::OFF_P + j * n + i] : -Fs[i];
            if (i == j) v += tol;
#pragma unroll
            for (int t = 0; t < GEN::SE_KT; ++t) {
              const int k = sk[(r * GEN::SE_KT + t) * 64 + l];
              if (k < 0) continue;
              v = fma(-blk[GEN::OFF_Q + k * n + i], j < n ? blk[GEN::OFF_R + j * m + k] * sD[k] : sty[k], v);
            }
            sv[e] = v;
          }
          __syncthreads();
        }
        // ---- entry (i, j) of [K | rhs] ------------------------------------------------
        // SCHUR: S = (P + tol·I) + Σ (−Q_ik)(R_kj·D_k⁻¹) over k ∈ K(i) (Q's structural
        // nonzeros of row i) with j ∈ J(k) (R's of row k), k ascending (the oracle's terms),
        // and rr_i = −F_Gi + Σ_{k ∈ K(i)} (−Q_ik) ty_k; otherwise ∇F_z + tol·I (RED: with
        // the slack block eliminated) and −F.
        auto entry = [&](int i, int j) -> double {
          if constexpr (NLS && kVr<NSMAX>) {  // the dense part; sv patches the rest
            if (j < n) return i == j ? blk[GEN::OFF_P + j * n + i] + tol : blk[GEN::OFF_P + j * n + i];
            return -Fs[i];
          } else if constexpr (SCH) {
            const int32_t* qp = GEN::qk_ptr();
            const int32_t* qi = GEN::qk_idx();
            const int32_t* rp = GEN::rj_ptr();
            const int32_t* ri = GEN::rj_idx();
            double acc;
            if (j < n) {
              acc = blk[GEN::OFF_P + j * n + i];
              if (i == j) acc += tol;
              for (int t = qp[i]; t < qp[i + 1]; ++t) {
                const int k = qi[t];
                bool nz = false;
                for (int u = rp[k]; u < rp[k + 1]; ++u) nz |= ri[u] == j;
                if (nz) acc = fma(-blk[GEN::OFF_Q + k * n + i], blk[GEN::OFF_R + j * m + k] * sD[k], acc);
              }
            } else {
              acc = -Fs[i];
              for (int t = qp[i]; t < qp[i + 1]; ++t) {
                const int k = qi[t];
                acc = fma(-blk[GEN::OFF_Q + k * n + i], sty[k], acc);
              }
            }
            return acc;
          } else {
            double v;
            if (j < ns) {
              v = jac<FAMILY, GEN>(th, blk, zs, n, m, i, j);
              if (i == j) {
                v += tol;  // src/solver.jl:81 ∇F + tol*I
                if (RED && i >= n) v += zs[n + m + (i - n)] / (zs[i] + tol);  // + s_k / w_k
              }
            } else {
              v = -Fs[i];
              if (RED && i >= n) v = v - (Fs[i + m] / (zs[i] + tol));  // −F_H − F_C / w_k
            }
            return v;
          }
        };
        // ---- LU with partial pivoting (:83-88) ------------------------------------
        // generated nonlinear modules' SCHUR step: reciprocal multipliers (oracle lu_solve_x)
        constexpr bool RCP = FAMILY == MCPX_FAMILY_NONLINEAR && SOLVER == MCPX_LINSOLVE_SCHUR;
        bool lu_ok;
        if constexpr (QPS) {
          bool gj_ok = false;
          if (msym) {
            for (int rep = 0; rep < (MCPX_WG_TWICE == 3 ? 2 : 1); ++rep) {
              d4 acc[GjDims<NSMAX>::TPW];
              for (int r2 = 0; r2 < (MCPX_WG_TWICE == 4 ? 2 : 1); ++r2) {
                if (a_lds) gj_form<NSMAX>(acc, th, sA, kGjLda(m), n, m, tol, qd, qr);
                else gj_form<NSMAX>(acc, th, th + (int64_t)n * n, m, n, m, tol, qd, qr);
              }
              gj_ok = gj_solve<NSMAX>(acc, n, dzs, S.lu.gj);
            }
          }
          lu_ok = true;
          if (!gj_ok) {  // the oracle's lu_solve of S (recomputed: the tiles were overwritten)
            __syncthreads();
            const int m4 = (m + 3) & ~3;
            const double* __restrict__ tA = th + (int64_t)n * n;
            auto sentry = [&](int i, int j) -> double {
              if (j == n) return qr[i];
              double acc = th[(int64_t)j * n + i];
              if (i == j) acc += tol;
              for (int k = 0; k < m4; ++k)
                acc = k < m ? fma(tA[(int64_t)i * m + k], tA[(int64_t)j * m + k] * qd[k], acc) : fma(0.0, 0.0, acc);
              return acc;
            };
            lu_ok = lu_solve_vr<NSMAX, 1, false>(sentry, n, dzs, S.lu.vr);
          }
        } else if constexpr (kVr<NSMAX> && SCH) {  // entries straight into registers (lu_vr.hpp)
          lu_ok = lu_solve_vr<NSMAX, 1, RCP>(entry, ns, dzs, S.lu, 1, nullptr, SePatch<GEN>{sv, n});
        } else if constexpr (kVr<NSMAX>) {
          lu_ok = lu_solve_vr<NSMAX, 1, RCP>(entry, ns, dzs, S.lu);
          if (MCPX_WG_TWICE == 1) {
            __syncthreads();
            lu_ok = lu_solve_vr<NSMAX, 1, RCP>(entry, ns, dzs, S.lu);
          }
        } else {  // [K | rhs] into the slot's workspace, then the HBM LU
          for (int i = wave; i < ns; i += NWAVE)
            for (int j = lane; j <= ns; j += 64) Am[(int64_t)i * ld + j] = entry(i, j);  // wave per row
          __syncthreads();
          lu_ok = lu_solve<NSMAX, RCP>(Am, ld, ns, dzs, S.lu);
        }
        if (!lu_ok) {
          status = 1;
          reason |= MCPX_FAIL_LINSOLVE;
          break;
        }
        if constexpr (QPS) {  // δy_k = (ry_k − Σ_j A_kj δx_j)·D_k⁻¹, δs_k = (−F_Ck − s_k δy_k)·w_k⁻¹
          auto dyds = [&](const double* __restrict__ tA, int la) {
            for (int k = tid; k < m; k += WG) {
              double acc = qy[k];
              for (int j = 0; j < n; ++j) acc = fma(-tA[(int64_t)j * la + k], dzs[j], acc);
              const double dy = acc * qd[k];
              dzs[n + k] = dy;
              dzs[n + m + k] = fma(-zs[n + m + k], dy, -Fs[n + m + k]) * qw[k];
            }
          };
          for (int rep = 0; rep < (MCPX_WG_TWICE == 6 ? 2 : 1); ++rep) {
            if (a_lds) dyds(sA, kGjLda(m));
            else dyds(th + (int64_t)n * n, m);
          }
        } else if constexpr (SCH) {  // δy_k = (ry_k − Σ_j R_kj δx_j)·D_k⁻¹, δs_k = (−F_Ck − s_k δy_k)·w_k⁻¹
          const int32_t* rp = GEN::rj_ptr();
          const int32_t* ri = GEN::rj_idx();
          for (int k = tid; k < m; k += WG) {
            double acc = sry[k];
            for (int t = rp[k]; t < rp[k + 1]; ++t) {  // R's structural nonzeros J(k)
              const int j = ri[t];
              acc = fma(-blk[GEN::OFF_R + j * m + k], dzs[j], acc);
            }
            const double dy = acc * sD[k];
            dzs[n + k] = dy;
            dzs[n + m + k] = fma(-zs[n + m + k], dy, -Fs[n + m + k]) * srw[k];
          }
        } else if constexpr (RED) {  // δs_k = (−F_Ck − s_k δy_k) / w_k
          for (int k = tid; k < m; k += WG)
            dzs[n + m + k] = fma(-zs[n + m + k], dzs[n + k], -Fs[n + m + k]) / (zs[n + k] + tol);
        }
        __syncthreads();
        // ---- fraction-to-the-boundary line search (:93-100, :127-138) ---------------
        uint64_t vs = 0ull, vy = 0ull;
        for (int k = tid; k < m; k += WG) {
          const double s = zs[n + m + k], ds = dzs[n + m + k], y = zs[n + k], dy = dzs[n + k];
          const double cs = a.c_tau * s, cy = a.c_tau * y;
          double alpha = 1.0;
          for (int e = 0; e < a.n_trials; ++e) {
            if (s + alpha * ds < cs) vs |= 1ull << e;
            if (y + alpha * dy < cy) vy |= 1ull << e;
            alpha *= a.decay;
          }
        }
        vs = wg_or(vs, S.sc);
        vy = wg_or(vy, S.sc);
        const int es = (~vs) ? __ffsll((unsigned long long)~vs) - 1 : 64;
        const int ey = (~vy) ? __ffsll((unsigned long long)~vy) - 1 : 64;
        if (es >= a.n_trials || ey >= a.n_trials) {  // α = NaN
          status = 1;
          reason |= MCPX_FAIL_LINESEARCH;
          break;
        }
        double as = 1.0, ay = 1.0;
        for (int e = 0; e < es; ++e) as *= a.decay;
        for (int e = 0; e < ey; ++e) ay *= a.decay;
        if (a.alpha_trace && newton < a.trace_len && tid == 0) {
          uint8_t* tr = a.alpha_trace + ((size_t)inst * a.trace_len + newton) * 2;
          tr[0] = (uint8_t)es;
          tr[1] = (uint8_t)ey;
        }
        // ---- update (:103-105; x moves with α_s) ------------------------------------
        for (int i = tid; i < N; i += WG) zs[i] = zs[i] + ((i >= n && i < n + m) ? ay : as) * dzs[i];
        kkt = kkt_step;  // :107
        ++inner;         // :108
        ++newton;
        __syncthreads();
      }
      eps *= (status == 0) ? a.tight[inner] : a.loose[inner];  // :111-113
      ++outer;                                                  // :114
    }
    if (outer == a.max_outer) {  // :117-119
      status = 1;
      reason |= MCPX_FAIL_MAX_OUTER;
    }
    __syncthreads();

    // ---- outputs (:121) -------------------------------------------------------------
    for (int i = tid; i < N; i += WG) {
      if (i < n) a.x[inst * n + i] = zs[i];
      else if (i < n + m) a.y[inst * m + (i - n)] = zs[i];
      else a.s[inst * m + (i - n - m)] = zs[i];
    }
    if (a.active_mask && tid < 64) {  // W = ⌈m/64⌉ words (include/mcpx.h), wave 0 by ballots
      const int W = m > 64 ? (m + 63) / 64 : 1;
      for (int q = 0; q < W; ++q) {
        const int k = 64 * q + tid, kk = k < m ? k : 0;
        const uint64_t act = __ballot(k < m && zs[n + kk] > zs[n + m + kk]);
        if (tid == 0) a.active_mask[inst * W + q] = act;
      }
    }
    if (tid == 0) {
      a.kkt_error[inst] = kkt;
      a.eps[inst] = eps;
      a.outer_iters[inst] = outer;
      a.status[inst] = status;
      if (a.newton_iters) a.newton_iters[inst] = newton;
      if (a.fail_reason) a.fail_reason[inst] = (uint8_t)reason;
    }
    __syncthreads();
  }
}

}  // namespace wg
}  // namespace mcpx
