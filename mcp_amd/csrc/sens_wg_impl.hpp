// sens_wg_impl.hpp — sensitivity kernels (reference src/AutoDiff.jl) in the
// workgroup-per-instance layout of ipm_wg_impl.hpp, for systems beyond the
// one-wave kernels' 64 rows and for every generated nonlinear module (the
// trajectory games of src/game.jl, whose ∇F_θ comes from the generated
// mcpx_nl_eval_theta — the reference's ∇F_θ!, src/mcp.jl:122-147).
//
// At the returned (x, y, s), ∇F_z WITHOUT tol·I (src/AutoDiff.jl:25-31):
//  * VJP — the rrule pullback (src/AutoDiff.jl:42-82): ∇F_zᵀ λ = g, ∂θ = −∇F_θᵀ λ,
//    on the slack-eliminated (n+m)-dim system of oracle sens_one (the s-rows of ∇F_zᵀ
//    carry −1 at λh: λh = y⊙λc − gs exactly), one right-hand side;
//  * JVP — the ForwardDiff.Dual method (src/AutoDiff.jl:84-117): ∇F_z ż = −∇F_θ θ̇
//    on the full (n+2m)-dim ∇F_z, `nrhs` partials per factorisation (each a trailing
//    column of the same elimination: the oracle's per-partial lu_solve bit for bit).
//  * condition estimate (SensArgs::mode = 1, the JVP kernels: mcpx_cond_batch) — rcond of
//    ∇F_z by the Hager–Higham 1-norm estimate from one LU (cond_one below).
// The system [K | rhs] is written into the slot's HBM workspace and factored by
// wg::lu_solve (blocked LU with partial pivoting, MFMA trailing update).  Entries,
// right-hand sides and the ∂θ contraction follow oracle/ipm_oracle.c sens_one op for
// op, so the results are bit-identical to oracle_{vjp,jvp}_batch[_nl].
#pragma once

#include "ipm_wg_impl.hpp"

namespace mcpx {
namespace wg {

// (∇F_θ θ̇)_i of the QP / affine families (oracle dtheta_row): the θ-pattern of row i
// applied to the tangent d, fma chains over x then y, then the θ-only term.
template <int FAMILY>
__device__ __forceinline__ double dtheta_row_aff(const double* __restrict__ d, const double* zs, int n, int m,
                                                 int i) {
  const int64_t nn = (int64_t)n * n, nm = (int64_t)n * m, mm = (int64_t)m * m;
  double acc = 0.0;
  if (i < n) {
    for (int j = 0; j < n; ++j) acc = fma(d[(int64_t)j * n + i], zs[j], acc);
    if constexpr (FAMILY == MCPX_FAMILY_QP) {
      for (int k = 0; k < m; ++k) acc = fma(-d[nn + (int64_t)i * m + k], zs[n + k], acc);
      return acc - d[nn + nm + m + i];
    } else {
      for (int k = 0; k < m; ++k) acc = fma(d[nn + (int64_t)k * n + i], zs[n + k], acc);
      return acc + d[nn + 2 * nm + mm + i];
    }
  }
  if (i < n + m) {
    const int k = i - n;
    if constexpr (FAMILY == MCPX_FAMILY_QP) {
      for (int j = 0; j < n; ++j) acc = fma(d[nn + (int64_t)j * m + k], zs[j], acc);
      return acc - d[nn + nm + k];
    } else {
      for (int j = 0; j < n; ++j) acc = fma(d[nn + nm + (int64_t)j * m + k], zs[j], acc);
      for (int q = 0; q < m; ++q) acc = fma(d[nn + 2 * nm + (int64_t)q * m + k], zs[n + q], acc);
      return acc + d[nn + 2 * nm + mm + n + k];
    }
  }
  return 0.0;
}

// (∇F_θ θ̇)_i of a generated module (oracle dtheta_row_nl): the θ columns of row i ascending.
template <class GEN>
__device__ __forceinline__ double dtheta_row_nl(const double* __restrict__ dth, const double* __restrict__ d,
                                                int nr, int i) {
  if (i >= nr) return 0.0;
  const int32_t* tp = GEN::tr_ptr();
  const int32_t* ti = GEN::tr_idx();
  double acc = 0.0;
  for (int u = tp[i]; u < tp[i + 1]; ++u) {
    const int t = ti[u];
    acc = fma(dth[(int64_t)t * nr + i], d[t], acc);
  }
  return acc;
}

// ∂θ_t of the pullback from λ = [λx; λh] (oracle sens_one): the QP / affine rank-1
// blocks, or −Σ_i ∇F_θ[i, t] λ_i over the structural nonzeros of column t.
template <int FAMILY, class GEN>
__device__ __forceinline__ double dtheta_entry(int64_t t, const double* lam, const double* zs,
                                               const double* __restrict__ dth, int n, int m) {
  const double* lx = lam;
  const double* ly = lam + n;
  const double* x = zs;
  const double* y = zs + n;
  if constexpr (FAMILY == MCPX_FAMILY_NONLINEAR) {
    const int nr = n + m;
    const int32_t* cp = GEN::tc_ptr();
    const int32_t* ci = GEN::tc_idx();
    double acc = 0.0;
    for (int u = cp[t]; u < cp[t + 1]; ++u) {
      const int i = ci[u];
      acc = fma(dth[t * nr + i], lam[i], acc);
    }
    return -acc;
  } else {
    const int64_t nn = (int64_t)n * n, nm = (int64_t)n * m, mm = (int64_t)m * m;
    if (t < nn) return -(lx[t % n] * x[t / n]);  // ∂M_rc / ∂P_rc
    if constexpr (FAMILY == MCPX_FAMILY_QP) {
      if (t < nn + nm) {
        const int64_t u = t - nn;
        const int c = (int)(u / m), k = (int)(u % m);
        return fma(lx[c], y[k], -(ly[k] * x[c]));  // ∂A_kc
      }
      if (t < nn + nm + m) return ly[t - nn - nm];  // ∂b_k
      return lx[t - nn - nm - m];                   // ∂ϕ_i
    } else {
      if (t < nn + nm) {  // ∂Q_rc
        const int64_t u = t - nn;
        return -(lx[u % n] * y[u / n]);
      }
      if (t < nn + 2 * nm) {  // ∂R_kc
        const int64_t u = t - nn - nm;
        return -(ly[u % m] * x[u / m]);
      }
      if (t < nn + 2 * nm + mm) {  // ∂S_kc
        const int64_t u = t - nn - 2 * nm;
        return -(ly[u % m] * y[u / m]);
      }
      if (t < nn + 2 * nm + mm + n) return -lx[t - nn - 2 * nm - mm];  // ∂g_i
      return -ly[t - nn - 2 * nm - mm - n];                             // ∂h_k
    }
  }
}

// ---- condition estimate of ∇F_z (oracle/ipm_oracle.c cond_estimate, op for op) -------------
// After lu_solve with no right-hand side, row i of A holds the multipliers l_ik (k < step(i))
// and u_ik (k ≥ step(i)); L.prow / L.step_of give the pivot order.  Solves are column-oriented,
// one barrier per step (each thread owns the rows i ≡ tid mod 256); the short sequential parts
// (sums, sign vector, argmax) run on thread 0 in the oracle's order.

// A x = b: b (row-indexed) destroyed, x (column-indexed).
template <int NSMAX>
__device__ __forceinline__ void lu_apply(const double* __restrict__ A, int ld, int N, const LuShared<NSMAX>& L,
                                         double* b, double* x) {
  const int tid = threadIdx.x;
  for (int k = 0; k < N; ++k) {
    const double bp = b[L.prow[k]];
    for (int i = tid; i < N; i += WG)
      if (L.step_of[i] > k) b[i] = fma(-A[(int64_t)i * ld + k], bp, b[i]);
    __syncthreads();
  }
  for (int k = N - 1; k >= 0; --k) {
    const int p = L.prow[k];
    const double xk = b[p] / A[(int64_t)p * ld + k];
    if (tid == 0) x[k] = xk;
    for (int i = tid; i < N; i += WG)
      if (L.step_of[i] < k) b[i] = fma(-A[(int64_t)i * ld + k], xk, b[i]);
    __syncthreads();
  }
}

// Aᵀ z = c (PA = LU): c (column-indexed) destroyed, u (N scratch), z (row-indexed).
template <int NSMAX>
__device__ __forceinline__ void lu_apply_t(const double* __restrict__ A, int ld, int N, const LuShared<NSMAX>& L,
                                           double* c, double* u, double* z) {
  const int tid = threadIdx.x;
  for (int k = 0; k < N; ++k) {  // Uᵀ
    const double* ur = A + (int64_t)L.prow[k] * ld;
    const double uk = c[k] / ur[k];
    if (tid == 0) u[k] = uk;
    for (int i = k + 1 + tid; i < N; i += WG) c[i] = fma(-ur[i], uk, c[i]);
    __syncthreads();
  }
  for (int k = N - 1; k >= 0; --k) {  // Lᵀ
    const double* lr = A + (int64_t)L.prow[k] * ld;
    const double vk = u[k];
    for (int j = tid; j < k; j += WG) u[j] = fma(-lr[j], vk, u[j]);
    if (tid == 0) z[L.prow[k]] = vk;
    __syncthreads();
  }
}

// rcond of the N×N ∇F_z in A (destroyed); v0..v2: LDS vectors, h: 2·N doubles of HBM scratch.
template <int NSMAX>
__device__ __forceinline__ double cond_one(double* __restrict__ A, int ld, int N, LuShared<NSMAX>& L, double* v0,
                                           double* v1, double* v2, double* h, double* xs, Scratch& sc, bool& singular) {
  const int tid = threadIdx.x;
  for (int j = tid; j < N; j += WG) {  // column sums of |a_ij|, rows ascending
    double c = 0.0;
    for (int i = 0; i < N; ++i) c = c + fabs(A[(int64_t)i * ld + j]);
    h[j] = c;
  }
  __syncthreads();
  double anorm = 0.0;  // (thread 0's value is the one used)
  if (tid == 0) {
    for (int j = 0; j < N; ++j) {
      const double c = h[j];
      if (c > anorm || c != c) anorm = c;
      if (anorm != anorm) break;
    }
  }
  __syncthreads();
  singular = !lu_solve<NSMAX>(A, ld, N, xs, L, 0, nullptr);
  if (singular) return 0.0;
  double* const x = v0;   // the rhs of the next solve (destroyed by it)
  double* const y = v1;   // A⁻¹x
  double* const xi = v2;  // sign(y) of the previous round
  double* const z = h;    // A⁻ᵀξ
  double* const u = h + N;
  const double inv = 1.0 / (double)N;
  for (int i = tid; i < N; i += WG) x[i] = inv;
  __syncthreads();
  double est = 0.0;  // thread 0 holds the estimate; the stop decisions go through sc.i[0]
  int jprev = -1;
  for (int it = 0; it < 5; ++it) {
    lu_apply<NSMAX>(A, ld, N, L, x, y);
    if (tid == 0) {
      double g = 0.0;
      for (int k = 0; k < N; ++k) g = g + fabs(y[k]);
      int stop = it > 0 && !(g > est);
      if (!stop) {
        est = g;
        int same = it > 0;
        for (int k = 0; k < N; ++k) {
          const double sg = y[k] >= 0.0 ? 1.0 : -1.0;
          if (sg != xi[k]) same = 0;
          xi[k] = sg;
        }
        stop = same;
      }
      sc.i[0] = stop;
    }
    __syncthreads();
    if (sc.i[0]) break;
    for (int k = tid; k < N; k += WG) x[k] = xi[k];
    __syncthreads();
    lu_apply_t<NSMAX>(A, ld, N, L, x, u, z);
    if (tid == 0) {
      int jm = -1;
      double bz = -1.0;
      for (int i = 0; i < N; ++i)
        if (fabs(z[i]) > bz) {
          bz = fabs(z[i]);
          jm = i;
        }
      if (jm < 0) jm = 0;
      const int stop = it > 0 && !(fabs(z[jm]) > z[jprev]);
      if (!stop) jprev = jm;
      sc.i[0] = stop;
      sc.i[1] = jm;
    }
    __syncthreads();
    if (sc.i[0]) break;
    const int jm = sc.i[1];
    for (int i = tid; i < N; i += WG) x[i] = i == jm ? 1.0 : 0.0;
    __syncthreads();
  }
  for (int i = tid; i < N; i += WG) x[i] = (i & 1 ? -1.0 : 1.0) * (1.0 + (N > 1 ? (double)i / (double)(N - 1) : 0.0));
  __syncthreads();
  lu_apply<NSMAX>(A, ld, N, L, x, y);
  double rc = 0.0;
  if (tid == 0) {
    double g = 0.0;
    for (int k = 0; k < N; ++k) g = g + fabs(y[k]);
    const double alt = 2.0 * g / (3.0 * (double)N);
    if (alt > est) est = alt;
    const double den = anorm * est;
    rc = (den > 0.0 && den <= __DBL_MAX__) ? 1.0 / den : 0.0;
  }
  return rc;  // thread 0's
}

template <int FAMILY, bool JVP, int NVMAX, int NSMAX, class GEN>
__device__ __forceinline__ void sens_instances(const WgSensArgs& W) {
  constexpr bool NL = FAMILY == MCPX_FAMILY_NONLINEAR;
  __shared__ SolveShared<NVMAX, NSMAX, false> S;  // several right-hand sides: the HBM LU
  const SensArgs& a = W.s;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = a.n, m = a.m, N = n + 2 * m, nr = n + m;
  const int ns = JVP ? N : nr;  // dimension of the factored system
  const int64_t p = a.p;
  const int K = JVP ? a.n_partials : 1;
  const int ld = W.ld;
  double* const slot = W.work + (int64_t)blockIdx.x * W.slot_stride;
  double* const Am = slot;
  double* const blk = slot + W.off_blk;
  double* const dth = slot + W.off_dth;
  double* const sol = slot + W.off_sol;
  double* const zs = S.zs;
  double* const lam = S.Fs;
  double* const xs = S.dzs;

  for (;;) {
    if (tid == 0) S.sc.inst = atomicAdd(W.counter, 1);  // the work queue
    __syncthreads();
    const int64_t inst = S.sc.inst;
    __syncthreads();
    if (inst >= W.batch) break;  // every workgroup reaches this exit
    const double* __restrict__ th = a.theta + inst * a.theta_ld;
    const bool has_gs = a.gs || a.ga_s != 0.0;  // else ∂l/∂s = ZeroTangent
    auto gs_at = [&](int k) { return affine_ct(a.ga_s, zs[nr + k], a.gs ? a.gs + inst * m + k : nullptr); };

    // z = [x; y; s] at the returned iterate (src/AutoDiff.jl:25)
    for (int i = tid; i < N; i += WG)
      zs[i] = i < n ? a.x[inst * n + i] : (i < nr ? a.y[inst * m + (i - n)] : a.s[inst * m + (i - nr)]);
    if constexpr (NL) {
      for (int i = tid; i < GEN::SIZE; i += WG) blk[i] = 0.0;  // structural zeros
      for (int64_t i = tid; i < (int64_t)nr * p; i += WG) dth[i] = 0.0;
      __syncthreads();
      if (tid == 0) {  // ∇F_z! and ∇F_θ! at z (src/AutoDiff.jl:27-37)
        GEN::init(th, blk);
        GEN::eval(th, zs, blk);
        GEN::eval_theta(th, zs, dth);
      }
    }
    __syncthreads();

    if constexpr (JVP) {
      if (a.mode == 1) {  // mcpx_cond_batch: rcond of ∇F_z at the returned iterate
        for (int r = wave; r < N; r += NWAVE)
          for (int j = lane; j < N; j += 64) Am[(int64_t)r * ld + j] = jac<FAMILY, GEN>(th, blk, zs, n, m, r, j);
        __syncthreads();
        bool sing = false;
        const double rc = cond_one<NSMAX>(Am, ld, N, S.lu, S.zs, S.Fs, S.dzs, sol, xs, S.sc, sing);
        if (tid == 0) {
          a.out[inst] = rc;
          if (a.status) a.status[inst] = sing ? 1 : 0;
        }
        __syncthreads();
        continue;
      }
    }

    bool ok_all = true;
    for (int c0 = 0; c0 < K; c0 += W.nrhs) {
      const int R = JVP ? min(W.nrhs, K - c0) : 1;
      // ---- [K | rhs] ----------------------------------------------------------------
      for (int r = wave; r < ns; r += NWAVE) {  // wave per row, lanes over the columns
        const bool qp_y = FAMILY == MCPX_FAMILY_QP && r >= n;  // ∂H/∂y ≡ 0: structural zeros
        for (int j = lane; j < ns + R; j += 64) {
          double v;
          if constexpr (JVP) {
            if (j < ns) {
              v = jac<FAMILY, GEN>(th, blk, zs, n, m, r, j);
            } else {
              const double* d = a.theta_dot + (inst * K + c0 + (j - ns)) * p;
              v = -(NL ? dtheta_row_nl<GEN>(dth, d, nr, r) : dtheta_row_aff<FAMILY>(d, zs, n, m, r));
            }
          } else {
            if (j < n) {
              v = jac<FAMILY, GEN>(th, blk, zs, n, m, j, r);  // ∇F_z[j][r]
            } else if (j < ns) {
              const int k = j - n;
              v = qp_y ? 0.0 : jac<FAMILY, GEN>(th, blk, zs, n, m, n + k, r) * zs[n + k];  // ∇F_z[n+k][r]·y_k
              if (r == n + k) v = v + zs[nr + k];                                          // + s_k
            } else {  // g_r + Σ_k ∇F_z[n+k][r]·gs_k, k ascending (g = a ⊙ z + b, SensArgs ga_*)
              double acc = r < n ? affine_ct(a.ga_x, zs[r], a.gx ? a.gx + inst * n + r : nullptr)
                                 : affine_ct(a.ga_y, zs[r], a.gy ? a.gy + inst * m + (r - n) : nullptr);
              if (has_gs && !qp_y)
                for (int k = 0; k < m; ++k)
                  acc = fma(jac<FAMILY, GEN>(th, blk, zs, n, m, n + k, r), gs_at(k), acc);
              v = acc;
            }
          }
          Am[(int64_t)r * ld + j] = v;
        }
      }
      __syncthreads();
      // ---- LU with partial pivoting (oracle lu_solve) -------------------------------
      const bool ok = lu_solve<NSMAX>(Am, ld, ns, xs, S.lu, R, JVP ? sol : nullptr);
      ok_all = ok_all && ok;
      if constexpr (JVP) {
        for (int c = 0; c < R; ++c)
          for (int i = tid; i < N; i += WG)
            a.out[(inst * K + c0 + c) * N + i] = ok ? sol[(int64_t)c * ns + i] : __builtin_nan("");
        __syncthreads();  // every read of sol / Am done before the next chunk rebuilds them
      }
    }
    if constexpr (!JVP) {
      // [λx; λc] → [λx; λh], λh_k = y_k·λc_k − gs_k
      for (int i = tid; i < nr; i += WG) {
        double u = xs[i];
        if (i >= n) {
          const int k = i - n;
          u = has_gs ? fma(zs[n + k], u, -gs_at(k)) : zs[n + k] * u;
        }
        lam[i] = u;
      }
      __syncthreads();
      for (int64_t t = tid; t < p; t += WG)
        a.out[inst * p + t] = ok_all ? dtheta_entry<FAMILY, GEN>(t, lam, zs, dth, n, m) : __builtin_nan("");
    }
    if (a.status && tid == 0) a.status[inst] = ok_all ? 0 : 1;
    __syncthreads();
  }
}

}  // namespace wg
}  // namespace mcpx
