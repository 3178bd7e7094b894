// sens_kernel_impl.hpp — gfx950 kernels of the solution sensitivities
// (reference src/AutoDiff.jl).  Instantiated by sens_inst_vjp.hip / sens_inst_jvp.hip.
//
// The reference differentiates F(z; θ) = 0 at the returned iterate (x, y, s):
//     ∂z/∂θ = −(∇F_z)⁻¹ ∇F_θ           (src/AutoDiff.jl:18-40, pivoted QR of −∇F_z)
// with ∇F_z taken WITHOUT the solver's tol·I (src/AutoDiff.jl:25-31).
//
//  * vjp_kernel — the rrule pullback (src/AutoDiff.jl:42-82):
//        ∂θ = (∂z/∂θ)ᵀ g = −∇F_θᵀ λ,   ∇F_zᵀ λ = g = [∂l/∂x; ∂l/∂y; ∂l/∂s].
//    The s-rows of ∇F_zᵀ carry −1 at λh: eliminated exactly (λh = y⊙λc − gs),
//    leaving an (n+m)-dim system; lane j owns its row j plus the rhs, the register
//    LU of the Newton step (lu_solve_rows, ipm_kernel_impl.hpp) solves it, and λ
//    goes to LDS with z; ∂θ is then written as coalesced rank-1 blocks
//    (∂M = −λ_x xᵀ, ∂A_kj = λ_x,j y_k − λ_y,k x_j, ∂b = λ_y, ∂ϕ = λ_x for the QP
//    family; −λ ⊗ z blocks for the affine family).
//  * jvp_kernel — the ForwardDiff.Dual method (src/AutoDiff.jl:84-117):
//        ż_c = −(∇F_z)⁻¹ (∇F_θ θ̇_c)  for K partials.
//    Lane i owns row i of ∇F_z plus up to R right-hand sides −(∇F_θ θ̇_c)_i; one
//    LU of ∇F_z serves R partials (lu_solve_rows_multi).
//
// One 64-lane wave per instance, as the solver.  The ∇F_z rows are assembled
// straight from θ in registers (no Jacobian in HBM).  Arithmetic follows
// oracle_vjp_batch / oracle_jvp_batch of oracle/ipm_oracle.c op for op, so the
// results are bit-identical to the oracle.
#pragma once

#include "ipm_kernel_impl.hpp"
#include "sens_kernel.h"

namespace mcpx {
namespace {

// Row `ln` of ∇F_z (TR = false) or of ∇F_zᵀ (TR = true) at z = zs (LDS:
// x at 0, y at n, s at n+m), WITHOUT tol·I (src/AutoDiff.jl:27-31).  Entries of
// the x-column block (j < n) are ±px[j·sx], of the y-column block ±py[(j−n)·sy];
// the θ-independent entries (−I, diag(s), diag(y), src/mcp.jl:76-80) are the two
// (c1, v1), (c2, v2) pairs.  `RowPattern` is reused by the JVP right-hand side
// (the same θ pattern applied to a tangent θ̇).
struct RowPattern {
  int64_t ox, oy;  // offsets of the row's x / y column blocks in θ
  int sx, sy;      // strides (0 with use = false)
  bool usex, usey, negx, negy;
  int c1, c2;
  double v1, v2;
};

template <int FAMILY, bool TR>
__device__ __forceinline__ RowPattern row_pattern(const double* zs, int ln, int n, int m) {
  const int N = n + 2 * m;
  const int64_t nn = (int64_t)n * n, nm = (int64_t)n * m;
  const bool lx = ln < n, ly = ln >= n && ln < n + m, lz = ln >= n + m && ln < N;
  const int q = ln - n, r = ln - n - m;
  RowPattern P{0, 0, 0, 0, false, false, false, false, -1, -1, 0.0, 0.0};
  if (!TR) {  // row ln of ∇F_z = [[M, −Aᵀ, 0], [A, 0, −I], [0, diag(s), diag(y)]] (QP)
    if (lx) {
      P.usex = true; P.ox = ln; P.sx = n;                       // M[i,j] / P[i,j] = θ[j·n + i]
      P.usey = true;
      if (FAMILY == 0) { P.oy = nn + (int64_t)ln * m; P.sy = 1; P.negy = true; }  // −A[k,i]
      else { P.oy = nn + ln; P.sy = n; }                        // Q[i,k] = θ[n² + k·n + i]
    }
    if (ly) {
      P.usex = true; P.sx = m;
      P.ox = (FAMILY == 0 ? nn : nn + nm) + q;                  // A[q,j] / R[q,j]
      if (FAMILY != 0) { P.usey = true; P.oy = nn + 2 * nm + q; P.sy = m; }  // S[q,l]
      P.c1 = n + m + q; P.v1 = -1.0;                            // ∂(H − s)/∂s = −I
    }
    if (lz) {
      P.c1 = n + r; P.v1 = zs[n + m + r];                       // ∂(s⊙y)/∂y = diag(s)
      P.c2 = n + m + r; P.v2 = zs[n + r];                       // ∂(s⊙y)/∂s = diag(y)
    }
  } else {  // row ln of ∇F_zᵀ = column ln of ∇F_z
    if (lx) {
      P.usex = true; P.ox = (int64_t)ln * n; P.sx = 1;          // M[i,ln] / P[i,ln]
      P.usey = true; P.sy = 1;
      P.oy = (FAMILY == 0 ? nn : nn + nm) + (int64_t)ln * m;    // A[k,ln] / R[k,ln]
    }
    if (ly) {
      P.usex = true;
      if (FAMILY == 0) { P.ox = nn + q; P.sx = m; P.negx = true; }  // −A[q,i]
      else { P.ox = nn + (int64_t)q * n; P.sx = 1; }                // Q[i,q]
      if (FAMILY != 0) { P.usey = true; P.oy = nn + 2 * nm + (int64_t)q * m; P.sy = 1; }  // S[k,q]
      P.c1 = n + m + q; P.v1 = zs[n + m + q];                   // ∂(s⊙y)_q/∂y_q = s_q
    }
    if (lz) {
      P.c1 = n + r; P.v1 = -1.0;                                // ∂(H − s)_r/∂s_r
      P.c2 = n + m + r; P.v2 = zs[n + r];                       // ∂(s⊙y)_r/∂s_r = y_r
    }
  }
  return P;
}

template <int NMAX>
__device__ __forceinline__ void assemble_pattern_row(const double* __restrict__ th, const RowPattern& P, int n,
                                                     int m, double (&a)[NMAX]) {
  const double* px = th + (P.usex ? P.ox : 0);
  const double* py = th + (P.usey ? P.oy : 0);
  const int sx = P.usex ? P.sx : 0, sy = P.usey ? P.sy : 0;
#pragma unroll
  for (int j = 0; j < NMAX; ++j) {
    double v = 0.0;
    if (j < n) {
      const double t = px[j * sx];
      if (P.usex) v = P.negx ? -t : t;
    } else if (j < n + m) {
      const double t = py[(j - n) * sy];
      if (P.usey) v = P.negy ? -t : t;
    }
    if (j == P.c1) v = P.v1;
    if (j == P.c2) v = P.v2;
    a[j] = v;
  }
}

// (∇F_θ θ̇)_ln for the row pattern of ∇F_z (TR = false) applied to the tangent
// θ̇: the x-block chain, then the y-block chain, then the θ-only term
// (QP: −ϕ̇_i / −ḃ_q, affine: +ġ_i / +ḣ_q); complementarity rows: 0.
// fma_chain order of oracle dtheta_row().
template <int FAMILY>
__device__ __forceinline__ double dtheta_row(const double* __restrict__ d, const RowPattern& P, const double* zs,
                                             int ln, int n, int m) {
  const int64_t nn = (int64_t)n * n, nm = (int64_t)n * m, mm = (int64_t)m * m;
  double acc = 0.0;
  if (P.usex)
    for (int j = 0; j < n; ++j) {
      const double t = d[P.ox + (int64_t)j * P.sx];
      acc = fma(P.negx ? -t : t, zs[j], acc);
    }
  if (P.usey)
    for (int k = 0; k < m; ++k) {
      const double t = d[P.oy + (int64_t)k * P.sy];
      acc = fma(P.negy ? -t : t, zs[n + k], acc);
    }
  if (ln < n) return FAMILY == 0 ? acc - d[nn + nm + m + ln] : acc + d[nn + 2 * nm + mm + ln];
  if (ln < n + m) return FAMILY == 0 ? acc - d[nn + nm + (ln - n)] : acc + d[nn + 2 * nm + mm + n + (ln - n)];
  return 0.0;
}

// a[j] ← fma(−l, u_j, a[j]) for j in (k, NMAX) and r[c] ← fma(−l, u_{NMAX+c}, r[c])
// in the lanes where `upd` holds: eliminate_row() of the solver, widened to R
// right-hand sides (broadcast at full EXEC, only the fmas predicated — see there).
template <int NMAX, int R>
__device__ __forceinline__ void eliminate_row_multi(double (&a)[NMAX], double (&r)[R], int k, double l,
                                                    uint64_t pm, bool upd) {
  constexpr int G = 16;
  constexpr int W = NMAX + R;
#pragma clang loop unroll(full)
  for (int g = 0; g <= (W - 1) / G; ++g) {
    const int lo = max(G * g, k + 1);
    const int hi = min(G * g + G, W);
    if (lo >= hi) continue;
    const int cnt = hi - lo;
    double v[16], u[16];
#pragma clang loop unroll(full)
    for (int t = 0; t < 16; ++t) {
      const int j = lo + t;
      v[t] = (t < cnt) ? ((j < NMAX) ? a[j < NMAX ? j : 0] : r[j >= NMAX && j - NMAX < R ? j - NMAX : 0]) : 0.0;
    }
    bcast_n(cnt, v, pm, u);
    if (upd) {
#pragma clang loop unroll(full)
      for (int t = 0; t < 16; ++t) {
        const int j = lo + t;
        if (t < cnt && j < NMAX) a[j < NMAX ? j : 0] = fma(-l, u[t], a[j < NMAX ? j : 0]);
        if (t < cnt && j >= NMAX) r[j - NMAX < R ? j - NMAX : 0] = fma(-l, u[t], r[j - NMAX < R ? j - NMAX : 0]);
      }
    }
  }
}

// lu_solve_rows() with R right-hand sides: same pivot rule (first remaining row
// of largest |a_ik|, NaN never wins), same elimination and back substitution
// per right-hand side, so every column equals the single-rhs solve bitwise.
template <int NMAX, int R>
__device__ __forceinline__ bool lu_solve_rows_multi(double (&a)[NMAX], double (&r)[R], int N, int ln,
                                                    double (&dz)[R]) {
  uint64_t rem = (N >= 64) ? ~0ull : ((1ull << N) - 1ull);
  int my_step = 1 << 30;
  int pk = 0;
  bool singular = false;
#pragma clang loop unroll(full)
  for (int k = 0; k < NMAX; ++k) {
    if (k >= N || singular) continue;
    const double ak = a[k];
    const double av = fabs(ak);
    const bool valid = ((rem >> ln) & 1ull) && !(av != av);
    const uint32_t khi = valid ? (uint32_t)__double2hiint(av) + 1u : 0u;
    const uint32_t mhi = wave_max_u32(khi);
    int p;
    if (mhi == 0u) {
      p = lowest_lane(rem);
    } else {
      const uint64_t cand = ballot(khi == mhi);
      if (__popcll(cand) == 1) {
        p = lowest_lane(cand);
      } else {
        const uint32_t klo = (khi == mhi) ? (uint32_t)__double2loint(av) : 0u;
        const uint32_t mlo = wave_max_u32(klo);
        p = lowest_lane(ballot(khi == mhi && klo == mlo));
      }
    }
    const double piv = bcast(ak, p);
    if (piv == 0.0) {
      singular = true;
      continue;
    }
    rem &= ~(1ull << p);
    if (ln == p) my_step = k;
    if (ln == k) pk = p;
    eliminate_row_multi<NMAX, R>(a, r, k, ak / piv, 1ull << p, (rem >> ln) & 1ull);
  }
  if (singular) return false;
#pragma unroll
  for (int c = 0; c < R; ++c) dz[c] = 0.0;
#pragma clang loop unroll(full)
  for (int k = NMAX - 1; k >= 0; --k) {
    if (k < N) {
      const int p = __builtin_amdgcn_readlane(pk, k);
      const double akk = a[k];
#pragma unroll
      for (int c = 0; c < R; ++c) {
        const double xk = bcast(r[c] / akk, p);
        if (ln == k) dz[c] = xk;
        if (my_step < k) r[c] = fma(-akk, xk, r[c]);
      }
    }
  }
  return true;
}

// out[t] = f(row, col) for t = row + rows·col < rows·cols, 64 lanes at a time
// (coalesced stores of a column-major block).
template <class Fn>
__device__ __forceinline__ void write_block(double* __restrict__ out, int rows, int cols, int ln, Fn f) {
  const int total = rows * cols;
  if (total <= 0) return;
  int r = ln % rows, c = ln / rows;
  const int dr = 64 % rows, dc = 64 / rows;
  for (int t = ln; t < total; t += 64) {
    out[t] = f(r, c);
    r += dr;
    c += dc;
    if (r >= rows) {
      r -= rows;
      ++c;
    }
  }
}

// Load z = [x; y; s] of instance `inst` into LDS (zs[0, n+2m)).
__device__ __forceinline__ void load_z(const SensArgs& A, int64_t inst, int ln, double* zs) {
  const int n = A.n, m = A.m;
  double v = 0.0;
  if (ln < n) v = A.x[inst * n + ln];
  else if (ln < n + m) v = A.y[inst * m + (ln - n)];
  else if (ln < n + 2 * m) v = A.s[inst * m + (ln - n - m)];
  zs[ln] = v;
}

// Row `ln` (< n + m) of the slack-eliminated ∇F_zᵀ system of the VJP (oracle
// sens_one): unknowns u = [λx; λc]; λh = y⊙λc − gs follows from the −1 entries of
// the s-rows.  Row j < n: [∇F_z[i][j] (i < n) | ∇F_z[n+k][j]·y_k]; row n+q:
// [∇F_z[i][n+q] | ∇F_z[n+k][n+q]·y_k (+ s_q at k = q)]; rhs g_ln + Σ_k ∇F_z[n+k][ln]·gs_k.
template <int NMAX, int FAMILY>
__device__ __forceinline__ void vjp_reduced_row(const double* __restrict__ th, const double* zs, const double* gsv,
                                                int ln, int n, int m, double (&a)[NMAX], double& rhs) {
  const int64_t nn = (int64_t)n * n, nm = (int64_t)n * m;
  const bool lx = ln < n, lq = ln >= n && ln < n + m;
  const int q = ln - n;
  // column block of the G rows (∇F_z[i][ln], i < n) and of the H rows (∇F_z[n+k][ln], k < m)
  const double* pg = th;  // stride sg over i
  int sg = 0;
  bool ng = false;
  const double* ph = th;  // stride sh over k
  int sh = 0;
  bool uh = false;
  if (lx) {
    pg = th + (int64_t)ln * n; sg = 1;                                      // M[i,ln] / P[i,ln]
    ph = th + (FAMILY == 0 ? nn : nn + nm) + (int64_t)ln * m; sh = 1; uh = true;  // A[k,ln] / R[k,ln]
  }
  if (lq) {
    if (FAMILY == 0) { pg = th + nn + q; sg = m; ng = true; }              // −A[q,i]
    else { pg = th + nn + (int64_t)q * n; sg = 1; }                         // Q[i,q]
    if (FAMILY != 0) { ph = th + nn + 2 * nm + (int64_t)q * m; sh = 1; uh = true; }  // S[k,q]
  }
  const bool ug = lx || lq;
#pragma unroll
  for (int j = 0; j < NMAX; ++j) {
    double v = 0.0;
    if (j < n) {
      const double t = pg[j * sg];
      if (ug) v = ng ? -t : t;
    } else if (j < n + m) {
      const int k = j - n;
      const double t = ph[k * sh];
      if (uh) v = t * zs[n + k];          // ∇F_z[n+k][ln] · y_k
      if (lq && k == q) v = v + zs[n + m + q];  // + s_q
    }
    a[j] = v;
  }
  if (gsv && uh)
    for (int k = 0; k < m; ++k) rhs = fma(ph[k * sh], gsv[k], rhs);
}

// M exactly symmetric (the SCHUR solver's spd_try test; uniform).
__device__ __forceinline__ bool m_symmetric(const double* __restrict__ th, int ln, int n) {
  bool asym = false;
  const int r = min(ln, max(n - 1, 0));
  for (int j = 0; j < n; ++j) asym |= ln < n && !(th[j * n + r] == th[r * n + j]);
  return ballot(asym) == 0ull;
}

// QP pullback by the Schur complement (oracle vjp_qp_schur): with d = y / s,
//   (M + Aᵀ diag(d) A) λx = gx + Aᵀ (gs − d ⊙ gy),   λc = (gy + A λx) / s,
// S' formed on the matrix cores exactly as the SCHUR solver forms S (tol = 0, D⁻¹ = d)
// and solved by the 2-D Gauss-Jordan.  Needs M symmetric (msym), s > 0, y ≥ 0 and d
// finite; false (→ the LU of the reduced system) otherwise or on a pivot ≤ 0.  On true,
// l = this lane's entry of u = [λx; λc].  ta / lda: the A block (A_kj = ta[j·lda + k]);
// LDS scratch of 64 doubles each: sd (d_k), tk (gs_k − d_k·gy_k, then λx_j), gxl (gx_j;
// free again on return).
template <int NT>
__device__ __forceinline__ bool vjp_qp_schur(const double* __restrict__ th, const double* ta, int lda,
                                             const double* zs, const double* gsv, double g, int ln, int n, int m,
                                             bool msym, double* sd, double* tk, double* gxl, double& l) {
  const bool rh = ln >= n && ln < n + m;
  const int k = ln - n;
  const double yk = rh ? zs[ln] : 1.0, sk = rh ? zs[ln + m] : 1.0;
  const double d = yk / sk;
  const bool okk = sk > 0.0 && yk >= 0.0 && __builtin_isfinite(d);
  if (!msym || n < 1 || n > 16 * NT || ballot(rh && !okk) != 0ull) return false;
  __syncthreads();  // scr may still be read by the caller's previous use
  if (rh) {
    sd[k] = d;
    tk[k] = fma(-d, g, gsv ? gsv[k] : 0.0);
  }
  if (ln < n) gxl[ln] = g;
  __syncthreads();
  const int lc = ln & 15;
  double rh2[NT];
#pragma unroll
  for (int J = 0; J < NT; ++J) {
    const int j = 16 * J + lc;
    rh2[J] = j < n ? dot_strided<8, false>(ta + j * lda, 1, tk, m, gxl[j]) : 0.0;
  }
  d4 acc4[NT][NT];
  qp_schur_form_2d<NT>(th, ta, lda, sd, ln, n, m, 0.0, acc4);
  double acc[NT][NT][4];
#pragma unroll
  for (int I = 0; I < NT; ++I)
#pragma unroll
    for (int J = 0; J < NT; ++J)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[I][J][r] = acc4[I][J][r];
  double xo = 0.0;
  if (!gj2d_spd<NT, true>(acc, rh2, n, ln, xo)) return false;
  __syncthreads();  // every read of tk done
  if (ln < n) tk[ln] = xo;
  __syncthreads();
  l = ln < n ? xo : 0.0;
  if (rh) l = dot_strided<8, false>(ta + k, lda, tk, n, g) / sk;
  return true;
}

// The pullback of one instance (the rrule of src/AutoDiff.jl:42-82), one wave: zs = z =
// [x; y; s] in LDS, `lam` LDS scratch (≥ n+m), g = this lane's cotangent entry of the x / y
// rows, gsv = the s block's cotangent (any address space) or NULL = zero.  Writes ∂θ
// (family layout, stride p) to `o` and 0 / 1 (∇F_z singular) to *st.  QP family with
// NT > 0: the Schur-complement path first (vjp_qp_schur; ta / lda, msym, sd / tk as
// there, `lam` its gxl).
// LU = false (the fused fast pass): no LU fallback — returns false, writing nothing,
// when the Schur path does not apply.
template <int NMAX, int FAMILY, int NT = 0, bool LU = true>
__device__ __forceinline__ bool vjp_instance(const double* __restrict__ th, const double* zs, double* lam,
                                             const double* gsv, double g, int ln, int n, int m, double* __restrict__ o,
                                             int32_t* st, const double* ta = nullptr, int lda = 0, bool msym = false,
                                             double* sd = nullptr, double* tk = nullptr) {
  double l = 0.0;
  bool ok = false;
  if constexpr (FAMILY == MCPX_FAMILY_QP && NT > 0)
    ok = vjp_qp_schur<NT>(th, ta, lda, zs, gsv, g, ln, n, m, msym, sd, tk, lam, l);
  if constexpr (LU) {
    if (!ok) {
      double a[NMAX];
      vjp_reduced_row<NMAX, FAMILY>(th, zs, gsv, ln, n, m, a, g);
      ok = lu_solve_rows<NMAX>(a, g, n + m, ln, l);
    }
  } else {
    if (!ok) return false;
  }
  // [λx; λc] → [λx; λh], λh_q = y_q·λc_q − gs_q
  double lv = l;
  if (ln >= n && ln < n + m) {
    const int q = ln - n;
    lv = gsv ? fma(zs[n + q], l, -gsv[q]) : zs[n + q] * l;
  }
  lam[ln] = ok ? lv : __builtin_nan("");
  __syncthreads();
  if (st && ln == 0) *st = ok ? 0 : 1;
  const int64_t nn = (int64_t)n * n, nm = (int64_t)n * m, mm = (int64_t)m * m;
  const double* x = zs;
  const double* y = zs + n;
  const double* lx = lam;      // λ of the G rows
  const double* ly = lam + n;  // λ of the H − s rows
  if (FAMILY == 0) {
    write_block(o, n, n, ln, [&](int i, int j) { return -(lx[i] * x[j]); });               // ∂M_ij
    write_block(o + nn, m, n, ln, [&](int k, int j) { return fma(lx[j], y[k], -(ly[k] * x[j])); });  // ∂A_kj
    write_block(o + nn + nm, m, 1, ln, [&](int k, int) { return ly[k]; });                 // ∂b_k
    write_block(o + nn + nm + m, n, 1, ln, [&](int i, int) { return lx[i]; });             // ∂ϕ_i
  } else {
    write_block(o, n, n, ln, [&](int i, int j) { return -(lx[i] * x[j]); });               // ∂P_ij
    write_block(o + nn, n, m, ln, [&](int i, int k) { return -(lx[i] * y[k]); });          // ∂Q_ik
    write_block(o + nn + nm, m, n, ln, [&](int k, int j) { return -(ly[k] * x[j]); });     // ∂R_kj
    write_block(o + nn + 2 * nm, m, m, ln, [&](int k, int q) { return -(ly[k] * y[q]); }); // ∂S_kq
    write_block(o + nn + 2 * nm + mm, n, 1, ln, [&](int i, int) { return -lx[i]; });       // ∂g_i
    write_block(o + nn + 2 * nm + mm + n, m, 1, ln, [&](int k, int) { return -ly[k]; });   // ∂h_k
  }
  return true;
}

template <int NMAX, int FAMILY>
__global__ __launch_bounds__(64) void vjp_kernel(const SensArgs A) {
  constexpr bool QP = FAMILY == MCPX_FAMILY_QP;
  constexpr int NT = QP ? (NMAX + 15) / 16 : 0;  // Schur path: n < NMAX
  __shared__ double zs[64];
  __shared__ double lam[64];
  __shared__ double gsl[64];
  __shared__ double scr[QP ? 128 : 1];
  const int ln = threadIdx.x;
  const int64_t inst = blockIdx.x;
  const int n = A.n, m = A.m;
  const double* th = A.theta + inst * A.theta_ld;
  load_z(A, inst, ln, zs);
  __syncthreads();
  // ∂l/∂z_ln of the x / y rows (NULL block with a = 0: ZeroTangent)
  double g = 0.0;
  if (ln < n) g = affine_ct(A.ga_x, zs[ln], A.gx ? A.gx + inst * n + ln : nullptr);
  else if (ln < n + m) g = affine_ct(A.ga_y, zs[ln], A.gy ? A.gy + inst * m + (ln - n) : nullptr);
  const double* gsv = A.gs ? A.gs + inst * m : nullptr;
  if (A.ga_s != 0.0) {  // the s block's cotangent a·s + b, materialised for the row chains
    if (ln < m) gsl[ln] = affine_ct(A.ga_s, zs[n + m + ln], A.gs ? A.gs + inst * m + ln : nullptr);
    __syncthreads();
    gsv = gsl;
  }
  const bool msym = QP && m_symmetric(th, ln, n);
  vjp_instance<NMAX, FAMILY, NT>(th, zs, lam, gsv, g, ln, n, m, A.out + inst * A.p, A.status ? A.status + inst : nullptr,
                                 th + (int64_t)n * n, m, msym, scr, scr + 64);
}

// The pullback fused into the solve kernel's epilogue (ipm_solve_kernel<…, FUSE = NV>):
// the solve's lane layout (lanes [0, n) x, [n, n+m) y with s in `s`) into LDS, the
// cotangent a ⊙ z + b of KernelArgs, vjp_instance with register width NV ≥ n + m.
// LU = false (fast pass): returns false, having written nothing, when the Schur path cannot
// take the instance; the caller then defers it to the second pass, which solves it again
// (same bits) and pulls back with the LU fallback.  The caller runs this BEFORE writing the
// solve's outputs, so a deferred instance leaves x/y/s untouched and a warm start read from
// the output buffers (x0 = out.x, the receding-horizon pattern) is still intact for pass 2.
// lds: five 64-double LDS arrays of the solve kernel, dead once its Newton loop is done.
template <int NV, int FAMILY, int NT, bool LU>
__device__ __forceinline__ bool fused_vjp(const KernelArgs& A, int64_t inst, int ln, int n, int m, double z, double s,
                                          const double* th, const double* ta, int lda, bool msym,
                                          double* const (&lds)[5]) {
  double* const zs = lds[0];
  double* const lam = lds[1];
  double* const gsl = lds[2];
  __syncthreads();
  if (ln < n + m) zs[ln] = z;
  if (ln >= n && ln < n + m) zs[ln + m] = s;
  __syncthreads();
  double g = 0.0;
  if (ln < n) g = affine_ct(A.ct_ax, zs[ln], A.ct_bx ? A.ct_bx + inst * n + ln : nullptr);
  else if (ln < n + m) g = affine_ct(A.ct_ay, zs[ln], A.ct_by ? A.ct_by + inst * m + (ln - n) : nullptr);
  const double* gsv = nullptr;
  if (A.ct_as != 0.0 || A.ct_bs) {
    if (ln < m) gsl[ln] = affine_ct(A.ct_as, zs[n + m + ln], A.ct_bs ? A.ct_bs + inst * m + ln : nullptr);
    __syncthreads();
    gsv = gsl;
  }
  const int64_t p = (int64_t)n * n + (int64_t)m * n + m + n;  // QP θ dimension (mcpx_theta_dim)
  const bool done = vjp_instance<NV, FAMILY, NT, LU>(th, zs, lam, gsv, g, ln, n, m, A.vjp_dtheta + inst * p,
                                                     A.vjp_status ? A.vjp_status + inst : nullptr, ta, lda, msym,
                                                     lds[3], lds[4]);
  return done;
}

template <int NMAX, int FAMILY>
__global__ __launch_bounds__(64) void jvp_kernel(const SensArgs A) {
  constexpr int R = MCPX_JVP_RHS;
  __shared__ double zs[64];
  const int ln = threadIdx.x;
  const int64_t inst = blockIdx.x;
  const int n = A.n, m = A.m, N = n + 2 * m, K = A.n_partials;
  const double* th = A.theta + inst * A.theta_ld;
  load_z(A, inst, ln, zs);
  __syncthreads();
  const RowPattern P = row_pattern<FAMILY, false>(zs, ln, n, m);
  bool all_ok = true;
  for (int c0 = 0; c0 < K; c0 += R) {  // one factorisation of ∇F_z per R partials
    double a[NMAX], r[R], dz[R];
    assemble_pattern_row<NMAX>(th, P, n, m, a);
#pragma unroll
    for (int c = 0; c < R; ++c) {
      r[c] = 0.0;
      if (c0 + c < K) {
        const double* d = A.theta_dot + (inst * K + c0 + c) * A.p;
        r[c] = -dtheta_row<FAMILY>(d, P, zs, ln, n, m);
      }
    }
    const bool ok = lu_solve_rows_multi<NMAX, R>(a, r, N, ln, dz);
    all_ok = all_ok && ok;
#pragma unroll
    for (int c = 0; c < R; ++c)
      if (c0 + c < K && ln < N) A.out[(inst * K + c0 + c) * N + ln] = ok ? dz[c] : __builtin_nan("");
  }
  if (A.status && ln == 0) A.status[inst] = all_ok ? 0 : 1;
}

}  // namespace
}  // namespace mcpx
