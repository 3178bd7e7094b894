// ipm_nl_band.hpp — the band SCHUR kernel of generated modules (mcpx_nl_solve_band,
// MCPX_KERNEL_BAND): the reference's sparse Newton solve (UMFPACK, src/solver.jl:50,61,83)
// for problems whose Schur complement S = (P + tol·I) − Q D⁻¹ R has a narrow elimination
// window after mcp_amd/band.py's ordering (S' = S[σ][:, π]; the lane-change game: 7 rows ×
// 20 columns at horizon T = 2, 13 × 32 at T = 10, where S is 200 × 200 with 840 nonzeros).
//
// One 64-lane wave per instance, a persistent grid on the work queue of the workgroup
// kernels (wg::WgArgs; no workspace: everything lives in LDS and VGPRs).  The Newton loop is
// the one-wave SCHUR kernel's (ipm_nl_kernel.hpp solve<SCHUR>), on the compact Jacobian: the
// generated code writes the structural entries only (mcpx_nl_init_c / mcpx_nl_eval_c, or the
// lane-parallel program MCPX_NL_CVEC), S' and rr' are formed entry-parallel from the
// generated tables, and the elimination is oracle/ipm_oracle.c lu_band_solve op for op:
//
//   window   NS slots × WC columns in the matrix-core layout of the 2-D Gauss-Jordan:
//            lane (lr, lc) holds slot lc (+ 16J) at the columns j with j mod WC = 4c + lr
//            (register c); a column's registers are recycled for column j + WC once
//            column j has been eliminated.  Slots hold rows in any order; each slot knows
//            its S' row (pv, the tie-break of the first-max rule).
//   step k   column k of every slot to every lane (ds_bpermute), the first-max pivot slot
//            (DPP 16-lane maximum of the |a| key; a tie goes through the full rule behind a
//            uniform branch), l = a · (1 / piv) (correctly rounded reciprocal), the pivot row
//            to every lane (ds_bpermute from the pivot slot), the rank-1 update of the other
//            slots, column k zeroed, then row k + NS of S' enters the free slot from its
//            image in LDS (its WC window entries, built one step ahead from the S' entries by
//            the row's table of (window index, entry) pairs).
//   loop     the steps run in blocks of WC, so every register index is static (k mod WC)
//            and the code is WC steps long, whatever n.
//   U        row k (its window entries, its rhs and 1 / u_kk) goes to U (LDS when small, the
//            slot's HBM workspace otherwise); the back substitution is the oracle's
//            column-oriented one: lane t mod 64 holds the rhs of row t while the row is in
//            the window [k − WC + 1, k − 1], x_k comes by a readlane, the U_tk by loads issued
//            WC steps ahead.
#pragma once

#if MCPX_NL_CAN_BAND

#include <type_traits>
#include <utility>

namespace mcpx {
namespace nl {
namespace band {

constexpr int NS = MCPX_NL_BAND_NS, WC = MCPX_NL_BAND_WC, NCB = WC / 4, NJ = (NS + 15) / 16;
constexpr int NNZ = MCPX_NL_BAND_NNZ, CS = MCPX_NL_CSIZE, C_G = MCPX_NL_C_G, C_H = MCPX_NL_C_H;
constexpr int SENT = 1 << 20;  // pv of an empty slot
constexpr int RNB = (n + 63) / 64, RMB = imax(1, (m + 63) / 64);
static_assert(NS >= 1 && NS <= 64 && WC >= 4 && WC <= 64 && WC % 4 == 0, "band window");
static_assert(CS < 32768, "compact slots are packed in 16 bits (mcp_amd/band.py)");
#if defined(MCPX_NL_CVEC)
constexpr int EVN = MCPX_NL_CVEC_EV, OFFZ = MCPX_NL_CVEC_OFF_Z;
constexpr int kCVecSteps[] = {MCPX_NL_CVEC_STEPS};
#else
constexpr int EVN = CS + N, OFFZ = CS;
#endif
// the LDS codegen.py budgets for (NLSystem._emit_band: band.BandPlan.lds_bytes)


__device__ __forceinline__ const int* opaque_ptr(const int* p) {
  asm volatile("" : "+s"(p));
  return p;
}

template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// Max over the 16 lanes of a DPP row (every row holds the same slots), uniform.
__device__ __forceinline__ uint32_t row_max_u32(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false));
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 15);
}

// The pivot slot of column k (col: this lane's slot entries): largest |a| by the key
// hi32(|a|) + 1 (0 for an empty slot or NaN: NaN never wins); 16·J + lc, uniform.  `tie`: the
// key maximum is not unique or is 0 (equal hi32 halves, every remaining entry NaN) — the step
// then takes pivot_exact, which breaks the tie as lu_band_solve does.
__device__ __forceinline__ int pivot_fast(const double (&col)[NJ], const int (&pv)[NJ], bool& tie) {
  uint32_t kh[NJ], mx = 0u;
#pragma unroll
  for (int J = 0; J < NJ; ++J) {
    const double a = fabs(col[J]);
    kh[J] = (pv[J] < SENT && !(a != a)) ? (uint32_t)__double2hiint(a) + 1u : 0u;
    mx = max(mx, kh[J]);
  }
  mx = row_max_u32(mx);
  int cnt = 0, ps = 0;
#pragma unroll
  for (int J = NJ - 1; J >= 0; --J) {
    const uint64_t c = ballot(kh[J] == mx) & 0xFFFFull;
    cnt += __popcll(c);
    if (c) ps = 16 * J + lowest_lane(c);
  }
  tie |= (cnt != 1) | (mx == 0u);
  return ps;
}

// lu_band_solve's first-max rule in full: largest |a| (NaN never wins), ties to the lowest S'
// row; all-NaN → the lowest remaining row.  Keys hi32(|a|) + 1 first, then lo32, then the rows.
__device__ __forceinline__ int pivot_exact(const double (&col)[NJ], const int (&pv)[NJ]) {
  uint32_t kh[NJ], mx = 0u;
#pragma unroll
  for (int J = 0; J < NJ; ++J) {
    const double a = fabs(col[J]);
    kh[J] = (pv[J] < SENT && !(a != a)) ? (uint32_t)__double2hiint(a) + 1u : 0u;
    mx = max(mx, kh[J]);
  }
  mx = row_max_u32(mx);
  // the lo32 halves of the largest, then the rows; every remaining entry NaN (mx = 0): the
  // lowest remaining row
  uint32_t key[NJ], k2 = 0u, lo[NJ], ml = 0u;
#pragma unroll
  for (int J = 0; J < NJ; ++J) {
    lo[J] = (kh[J] == mx && mx != 0u) ? (uint32_t)__double2loint(fabs(col[J])) : 0u;
    ml = max(ml, lo[J]);
  }
  ml = row_max_u32(ml);
#pragma unroll
  for (int J = 0; J < NJ; ++J)
    key[J] = (mx != 0u ? (kh[J] == mx && lo[J] == ml) : pv[J] < SENT) ? ~(uint32_t)pv[J] : 0u;
#pragma unroll
  for (int J = 0; J < NJ; ++J) k2 = max(k2, key[J]);
  k2 = row_max_u32(k2);
  int ps = 0;
#pragma unroll
  for (int J = NJ - 1; J >= 0; --J) {
    const uint64_t b = ballot(key[J] == k2 && key[J] != 0u) & 0xFFFFull;
    if (b) ps = 16 * J + lowest_lane(b);
  }
  return ps;
}

// MCPX_BAND_TWICE (diagnostic builds only, tools/band_ab.py): one phase of the Newton step
// runs twice — 1 factorisation and back substitution, 2 formation of S' and rr', 3 the
// generated eval, 4 back substitution.  Each phase is idempotent, so the bits stay the
// product's and the time added is the phase's cost.
#ifndef MCPX_BAND_BS_NOBR
#define MCPX_BAND_BS_NOBR 1
#endif
#ifndef MCPX_BAND_TWICE
#define MCPX_BAND_TWICE 0
#endif

constexpr int US = WC + 2;   // U row stride: the WC window entries, the rhs, 1 / u_kk
constexpr int EMAX = MCPX_NL_BAND_EMAX;  // nonzeros per S' row (the entering-row table's width)
constexpr bool ULDS = (int64_t)n * US * 8 <= 8 * 1024;
constexpr int UD = ULDS ? 4 : WC;  // back-substitution prefetch distance (divides WC)
// the slot's HBM workspace in doubles (mcpx_nl_meta[9]): U rows, 64 spare rows for the
// prefetch of rows that are read and discarded
constexpr int64_t WS = ULDS ? 0 : (int64_t)(n + 64) * US;
static_assert(WC % UD == 0 && EMAX <= 64, "band tables");
// MCPX_BAND_BS_NOBR with the U rows in HBM: each row's rhs and 1 / u_kk also go to LDS (sBR,
// 2n doubles), so the back substitution's entering rows come from LDS, not from branch-guarded
// loads (see factor_solve).
constexpr bool BSL = !ULDS && MCPX_BAND_BS_NOBR;
static_assert(8 * (EVN + NNZ + 1 + n + 2 * m + n + 2 * WC + (ULDS ? n * US : 0) + (BSL ? 2 * n : 0)) <=
                  160 * 1024 - 2048,
              "band kernel LDS (mcp_amd/band.py BandPlan.lds_bytes, codegen.BAND_LDS_LIMIT)");

struct Win {
  double acc[NJ][NCB], rh[NJ];
  int pv[NJ];
};

// Row R's window image into img (WC doubles, indexed by column mod WC): zeros, then its nonzeros
// (ent: this lane's packed (window index | entry << 8) of row R, −1 = none; one lane per entry).
__device__ __forceinline__ void build_image(double* img, int ent, const double* Sc, int ln) {
  if (ln < WC) img[ln] = 0.0;
  if (ent >= 0) img[ent & 0xff] = Sc[ent >> 8];
}

// Slot (J, ls) takes row R from its image (the lanes lc == ls load their window entries).
template <int J>
__device__ __forceinline__ void enter(Win& w, int R, int ls, const double* img, const double* rrp, int lc, int lr) {
  if (lc == ls) {
    if (R < n) {
#pragma unroll
      for (int c = 0; c < NCB; ++c) w.acc[J][c] = img[4 * c + lr];
      w.rh[J] = rrp[R];
      w.pv[J] = R;
    } else {
      w.pv[J] = SENT;
    }
  }
}

// Elimination step k (lu_band_solve's step k), W = k mod WC static.  `fail`: a zero pivot.
template <int W>
__device__ __forceinline__ void step(Win& w, int k, const double* Sc, const double* rrp, double* img2,
                                     double* U, double* sBR, const int* ent_tab, int& ent, int ln, bool& fail) {
  constexpr int CK = W >> 2, QK = W & 3;
  const int lc = ln & 15, lr = ln >> 4;
  double col[NJ];
#pragma unroll
  for (int J = 0; J < NJ; ++J) col[J] = bperm_f64_addr(w.acc[J][CK], ((QK << 4) | lc) << 2);
  bool tie = false;
  int ps = __builtin_amdgcn_readfirstlane(pivot_fast(col, w.pv, tie));
  if (__builtin_expect(tie, 0)) ps = __builtin_amdgcn_readfirstlane(pivot_exact(col, w.pv));
  const int Jp = NJ == 1 ? 0 : ps >> 4, lp = ps & 15;
  double cp = col[0];
#pragma unroll
  for (int J = 1; J < NJ; ++J) cp = Jp == J ? col[J] : cp;
  const double piv = bcast(cp, lp);
  fail |= piv == 0.0;  // the failed solve (the remaining steps run on discarded values)
  double rp = rcp_fast(piv);
  if (__builtin_expect(!rcp_fast_ok(piv), 0)) rp = 1.0 / piv;  // zero, subnormal, huge, Inf, NaN
  double lm[NJ];
#pragma unroll
  for (int J = 0; J < NJ; ++J) lm[J] = -(col[J] * rp);
  // the pivot row to every lane (each lane its own columns) and its rhs
  double u[NCB], ub = 0.0;
  const int addr = ((ln & 48) | lp) << 2;
  static_for<0, NJ>([&](auto J) {
    if (NJ == 1 || Jp == decltype(J)::value) {
#pragma unroll
      for (int c = 0; c < NCB; ++c) u[c] = bperm_f64_addr(w.acc[decltype(J)::value][c], addr);
      ub = bcast(w.rh[decltype(J)::value], lp);
    }
  });
  // U row k: the window entries (lanes lc == 0), the rhs and 1 / u_kk (lane 0)
  double* const Uk = U + (int64_t)k * US;
  if (lc == 0) {
#pragma unroll
    for (int c = 0; c < NCB; ++c) Uk[4 * c + lr] = u[c];
  }
  if (ln == 0) {
    if constexpr (BSL) {
      sBR[2 * k] = ub;
      sBR[2 * k + 1] = rp;
    } else {
      Uk[WC] = ub;
      Uk[WC + 1] = rp;
    }
  }
#pragma unroll
  for (int J = 0; J < NJ; ++J) {
#pragma unroll
    for (int c = 0; c < NCB; ++c) w.acc[J][c] = fma(lm[J], u[c], w.acc[J][c]);
    w.rh[J] = fma(lm[J], ub, w.rh[J]);
  }
  const bool retire = lr == QK;  // column k is eliminated: its registers become column k + WC
#pragma unroll
  for (int J = 0; J < NJ; ++J) w.acc[J][CK] = retire ? 0.0 : w.acc[J][CK];
  // row k + NS enters the free slot; the image of row k + NS + 1 is built for the next step
  const int R = k + NS;
  const double* img = img2 + (R & 1) * WC;
  static_for<0, NJ>([&](auto J) {
    if (NJ == 1 || Jp == decltype(J)::value) enter<decltype(J)::value>(w, R, lp, img, rrp, lc, lr);
  });
  build_image(img2 + ((R + 1) & 1) * WC, ent, Sc, ln);
  ent = (ln < EMAX && R + 2 < n) ? ent_tab[(R + 2) * EMAX + ln] : -1;  // row R + 2's entries, a step ahead
}

// lu_band_solve on S' (Sc: the entries in S' row-major order, ent_tab: each row's (window index,
// entry) pairs) and rr' (rrp, S' row order): x' (S' column order) into dxp.  False: a zero pivot.
__device__ __forceinline__ bool factor_solve(const double* Sc, const double* rrp, double* dxp, double* img2,
                                             double* U, double* sBR, const int* ent_tab, int ln) {
  const int lc = ln & 15, lr = ln >> 4;
  Win w;
#pragma unroll
  for (int J = 0; J < NJ; ++J) {
#pragma unroll
    for (int c = 0; c < NCB; ++c) w.acc[J][c] = 0.0;
    w.rh[J] = 0.0;
    w.pv[J] = SENT;
  }
  // rows 0 .. NS − 1 before step 0 (slot = row), then the image of row NS
#pragma unroll 1
  for (int r = 0; r < (NS < n ? NS : n); ++r) {
    build_image(img2, ln < EMAX ? ent_tab[r * EMAX + ln] : -1, Sc, ln);
    static_for<0, NJ>([&](auto J) {
      if ((r >> 4) == decltype(J)::value) enter<decltype(J)::value>(w, r, r & 15, img2, rrp, lc, lr);
    });
  }
  build_image(img2 + (NS & 1) * WC, (ln < EMAX && NS < n) ? ent_tab[NS * EMAX + ln] : -1, Sc, ln);
  int ent = (ln < EMAX && NS + 1 < n) ? ent_tab[(NS + 1) * EMAX + ln] : -1;
  bool fail = false;
#pragma unroll 1
  for (int k0 = 0; k0 < n; k0 += WC) {
    static_for<0, WC>([&](auto W) {
      if (k0 + decltype(W)::value < n) step<decltype(W)::value>(w, k0 + decltype(W)::value, Sc, rrp, img2, U, sBR,
                                                                ent_tab, ent, ln, fail);
    });
  }
  if (fail) return false;
  for (int rep = 0; rep < (MCPX_BAND_TWICE == 4 ? 2 : 1); ++rep) {
  // ---- back substitution, k = n − 1 .. 0 (lane l: the rhs and 1 / u_tt of row t ≡ l mod 64,
  // the largest such t ≤ k; rows enter the update window [k − WC + 1, k − 1] WC − 1 steps
  // before their x) --------------------------------------------------------------------------
  if constexpr (!ULDS) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the U rows are stored
  __syncthreads();
  constexpr int top = n - 1;
  int t = top - ((top - ln) & 63);  // this lane's row
  double bs = 0.0, rd = 0.0, nb = 0.0, nr = 0.0;
  if (t >= 0) {
    bs = BSL ? sBR[2 * t] : U[(int64_t)t * US + WC];
    rd = BSL ? sBR[2 * t + 1] : U[(int64_t)t * US + WC + 1];
  }
  // BSL: the pair (rhs, 1 / u) of the row entering at the next step, read from LDS a step ahead
  double pb = 0.0, pc = 0.0;
  if constexpr (BSL) {
    const int i = top - WC + 1 > 0 ? top - WC + 1 : 0;
    pb = sBR[2 * i];
    pc = sBR[2 * i + 1];
  }
  double ring[UD];
  // MCPX_BAND_BS_NOBR: the back substitution's loads are issued by every lane from a valid
  // (clamped) address and selected afterwards.  Behind a branch, a load the compiler cannot
  // count through made it wait vmcnt(0) at every step — for the prefetches issued UD steps
  // ahead too, a memory round trip per step.
  auto prefetch = [&](int kk) {  // U_{t(kk), kk} of step kk into ring[kk mod UD] (rows outside the window: discarded)
    const int tt = kk - ((kk - ln) & 63);
    if constexpr (MCPX_BAND_BS_NOBR) {  // raw: a lane without a row (tt < 0) never feeds an x
      const bool ok = tt >= 0 && kk >= 0;
      return U[(int64_t)(ok ? tt : 0) * US + (kk >= 0 ? kk % WC : 0)];
    }
    return tt >= 0 && kk >= 0 ? U[(int64_t)tt * US + kk % WC] : 0.0;
  };
#pragma unroll
  for (int d = 0; d < UD; ++d) ring[(top - d) % UD] = prefetch(top - d);
  // k = top, top − 1, …, in blocks of WC steps (k mod WC static in a block); the last block's
  // steps past k = 0 run as no-ops (no row takes part, no x is stored) instead of behind a
  // branch: a branch around the prefetches would again cost a vmcnt(0) at every step
#pragma unroll 1
  for (int s0 = 0; s0 < n; s0 += WC) {
    static_for<0, WC>([&](auto JJ) {
      constexpr int W = ((top - decltype(JJ)::value) % WC + WC) % WC;  // k mod WC
      const int k = top - s0 - decltype(JJ)::value;
      {
        // row k − WC + 1 enters the update window: its lane (done with row k − WC + 65) takes its
        // rhs and 1 / u, loaded when that row finished (WC − 1 steps before the lane row's x)
        const int ta = k - WC + 1;
        if constexpr (BSL) {
          const bool tk = ta >= 0 && ta + 64 <= top && (ta & 63) == ln;
          bs = tk ? pb : bs;
          rd = tk ? pc : rd;
        } else if (ta >= 0 && ta + 64 <= top && (ta & 63) == ln) {
          bs = nb;
          rd = nr;
        }
        const double xk = bcast(bs * rd, k & 63);
        if (ln == 0 && k >= 0) dxp[k] = xk;
        const int tl = k - ((k - ln) & 63);  // this lane's row at step k
        const double uv = ring[W % UD];
        const double nbs = fma(-uv, xk, bs);
        bs = (tl >= k - WC + 1 && tl <= k - 1) ? nbs : bs;
        ring[W % UD] = prefetch(k - UD);
        if constexpr (BSL) {  // the next step's entering row
          const int i = ta - 1 > 0 ? ta - 1 : 0;
          pb = sBR[2 * i];
          pc = sBR[2 * i + 1];
        } else if ((k & 63) == ln && k >= 64) {  // row k is done: its lane's next row is k − 64
          nb = U[(int64_t)(k - 64) * US + WC];
          nr = U[(int64_t)(k - 64) * US + WC + 1];
        }
      }
    });
  }
  }
  return true;
}

#if defined(MCPX_NL_CVEC)
__device__ __forceinline__ double ev_at(const double* ev, uint32_t byte_off) {
  return *(const double*)((const char*)ev + byte_off);
}
template <int S = 0, int W = 0>
__device__ __forceinline__ void eval_cvec(double* ev, const uint32_t (&w)[MCPX_NL_CVEC_NWORD],
                                          const uint32_t (&d)[MCPX_NL_CVEC_NSLOT]) {
  if constexpr (S < MCPX_NL_CVEC_NSLOT) {
    constexpr int K = kCVecSteps[S];
    double acc = 0.0;
#pragma unroll
    for (int t = 0; t < K; ++t) {
      uint32_t x = w[W + t];
      asm volatile("" : "+v"(x));  // decoded here: hoisted, the two halves would double the table's VGPRs
      const double prod = ev_at(ev, x & 0xffffu) * ev_at(ev, x >> 16);
      acc = t == 0 ? prod : acc + prod;
    }
    *(double*)((char*)ev + d[S]) = acc;
    eval_cvec<S + 1, W + K>(ev, w, d);
  }
}
#endif

// MCPX_BAND_DEBUG_EXIT (diagnostic builds only, tools/band_debug.py): 1 return at entry, 2 leave
// the work loop at its first instance, 3 no Jacobian init and no Newton loop, 4 no Newton loop.
#ifndef MCPX_BAND_DEBUG_EXIT
#define MCPX_BAND_DEBUG_EXIT 0
#endif

// The Newton loop of one instance after another (work queue), src/solver.jl:35-121.
__device__ __forceinline__ void solve(const wg::WgArgs& A) {
  if (MCPX_BAND_DEBUG_EXIT == 1) return;
  const KernelArgs& args = A.k;
  __shared__ __attribute__((aligned(16))) double ev[EVN];
  __shared__ double Sc[NNZ + 1], rrp[n], sDi[imax(1, m)], sTy[imax(1, m)], dxp[n], img2[2 * WC];
  __shared__ double Ush[ULDS ? n * US : 1];
  __shared__ double sBR[BSL ? 2 * n : 1];
  double* const cb = ev;
  double* const zs = ev + OFFZ;
  const int ln0 = threadIdx.x;
  const double tol = args.tol;
  double* const U = ULDS ? Ush : A.work + (int64_t)blockIdx.x * A.slot_stride;  // the U rows
#if defined(MCPX_NL_CVEC)
  uint32_t vw[MCPX_NL_CVEC_NWORD], vd[MCPX_NL_CVEC_NSLOT];
#pragma unroll
  for (int k = 0; k < MCPX_NL_CVEC_NWORD; ++k) vw[k] = mcpx_nl_cvec_word[k * 64 + ln0];
#pragma unroll
  for (int k = 0; k < MCPX_NL_CVEC_NSLOT; ++k) vd[k] = mcpx_nl_cvec_dst[k * 64 + ln0];
  for (int k = ln0; k < MCPX_NL_CVEC_NC; k += 64) ev[MCPX_NL_CVEC_OFF_C + k] = mcpx_nl_cvec_const[k];
#endif
  int ipx[RNB];  // S' column of x_j, j = ln + 64r (δx lives in S' column order)
#pragma unroll
  for (int r = 0; r < RNB; ++r) ipx[r] = ln0 + 64 * r < n ? mcpx_nl_band_iperm[ln0 + 64 * r] : 0;
  for (;;) {
    const int ln = ln0;
    // the next instance, taken in uniform control flow: every lane adds (lane 0 one, the others
    // zero) and lane 0's old value is the wave's.  (A one-lane `if (ln == 0)` atomic through LDS, as
    // the workgroup kernels do, let the compiler — its barrier being a no-op for a one-wave
    // workgroup — thread the loop's end-of-instance `if (ln == 0)` stores straight into that
    // atomic, so the other 63 lanes re-read the old instance forever: a hang.)
    const int got = atomicAdd(A.counter, ln == 0 ? 1 : 0);
    const int64_t inst = __builtin_amdgcn_readfirstlane(got);
    if (inst >= A.batch || MCPX_BAND_DEBUG_EXIT == 2) break;
    const double* __restrict__ th = args.theta + inst * args.theta_ld;
    // src/solver.jl:39-41, 64-66
#pragma unroll
    for (int r = 0; r < RNB; ++r) {
      const int j = ln + 64 * r;
      if (j < n) zs[j] = args.x0 ? args.x0[inst * n + j] : 0.0;
    }
#pragma unroll
    for (int r = 0; r < RMB; ++r) {
      const int k = ln + 64 * r;
      if (k < m) {
        zs[n + k] = args.y0 ? args.y0[inst * m + k] : 1.0;
        zs[n + m + k] = args.s0 ? args.s0[inst * m + k] : 1.0;
      }
    }
#if defined(MCPX_NL_CVEC)
    for (int k = ln; k < MCPX_NL_P; k += 64) ev[MCPX_NL_CVEC_OFF_T + k] = th[k];
#endif
    __syncthreads();
    if (ln == 0 && MCPX_BAND_DEBUG_EXIT != 3) mcpx_nl_init_c(th, cb);
    double eps = 1.0, kkt = __builtin_huge_val();  // :67-68
    int status = 0, outer = 1, newton = 0;         // :69-70
    unsigned reason = 0;
    while (kkt > tol && eps > tol && outer < args.max_outer && MCPX_BAND_DEBUG_EXIT < 3) {  // :71
      int inner = 1;
      status = 0;
      while (kkt > eps && inner < args.max_inner) {  // :75
        // the tables' base addresses and the lane index, opaque per Newton step: hoisted out of
        // the loops, their ~100 per-lane addresses would stay live for the whole solve (spills)
        const int* const bf_tab = opaque_ptr(mcpx_nl_bf_tab);
        const int* const br_tab = opaque_ptr(mcpx_nl_br_tab);
        const int* const bd_tab = opaque_ptr(mcpx_nl_bd_tab);
        const int* const ent_tab = opaque_ptr(mcpx_nl_bent_tab);
        const int ln = opaque_lane(ln0);
        __syncthreads();
#if defined(MCPX_NL_CVEC)
        for (int rep = 0; rep < (MCPX_BAND_TWICE == 3 ? 2 : 1); ++rep) eval_cvec(ev, vw, vd);
#else
        if (ln == 0) mcpx_nl_eval_c(th, zs, cb);
#endif
        __syncthreads();
        // F = [G; H − s; s⊙y − ϵ] (src/mcp.jl:76-80), ‖F‖∞ NaN-propagating (:107); the Schur
        // eliminations of δs_k (pivot y_k + tol) and δy_k (pivot D_k = tol + s_k / (y_k + tol))
        double aF = 0.0;
#pragma unroll
        for (int r = 0; r < RNB; ++r) {
          const int j = ln + 64 * r;
          if (j < n) aF = max_nan(aF, fabs(cb[C_G + j]));
        }
        double rw[RMB], ry[RMB];
#pragma unroll
        for (int r = 0; r < RMB; ++r) {
          const int k = ln + 64 * r;
          rw[r] = ry[r] = 0.0;
          if (k < m) {
            const double y = zs[n + k], s = zs[n + m + k];
            const double fh = cb[C_H + k] - s, fc = s * y - eps;
            aF = max_nan(aF, fabs(fh));
            aF = max_nan(aF, fabs(fc));
            rw[r] = 1.0 / (y + tol);
            const double Di = 1.0 / (tol + s * rw[r]);
            ry[r] = (-fh) - (fc * rw[r]);
            sDi[k] = Di;
            sTy[k] = ry[r] * Di;
          }
        }
        const double kkt_step = ballot(aF != aF) ? __builtin_nan("") : wave_max_nonneg(aF);
        __syncthreads();
        // S' entries and rr' (oracle: the row-wise loops over K(i) and J(k), the same chains);
        // rounds one at a time (unrolled, all their table loads would be in flight at once)
        for (int rep = 0; rep < (MCPX_BAND_TWICE == 2 ? 2 : 1); ++rep) {
#pragma unroll 1
        for (int r = 0; r < MCPX_NL_BF_R; ++r) {
          constexpr int WD = 1 + 2 * MCPX_NL_BF_KT;
          const int e = ln + 64 * r;
          const int w0 = bf_tab[(r * WD) * 64 + ln];
          if (e < NNZ) {
            const int ps = (w0 & 0x3fffffff) - 1;
            double v = ps >= 0 ? cb[ps] : 0.0;
            if (w0 >> 30) v = v + tol;
#pragma unroll
            for (int t = 0; t < MCPX_NL_BF_KT; ++t) {
              const int q = bf_tab[(r * WD + 1 + 2 * t) * 64 + ln];  // Q slot | R slot << 16
              const int k = bf_tab[(r * WD + 2 + 2 * t) * 64 + ln];  // −1: no term
              if (k >= 0) v = fma(-cb[q & 0xffff], cb[(q >> 16) & 0xffff] * sDi[k], v);
            }
            Sc[e] = v;
          }
        }
#pragma unroll 1
        for (int r = 0; r < MCPX_NL_BR_R; ++r) {
          constexpr int WD = 1 + 2 * MCPX_NL_BR_KQ;
          const int i = ln + 64 * r;
          if (i < n) {
            double v = -cb[br_tab[(r * WD) * 64 + ln]];
#pragma unroll
            for (int t = 0; t < MCPX_NL_BR_KQ; ++t) {
              const int q = br_tab[(r * WD + 1 + 2 * t) * 64 + ln];
              const int k = br_tab[(r * WD + 2 + 2 * t) * 64 + ln];
              if (k >= 0) v = fma(-cb[q], sTy[k], v);
            }
            rrp[i] = v;
          }
        }
        }
        __syncthreads();
        bool ok = factor_solve(Sc, rrp, dxp, img2, U, sBR, ent_tab, ln);
        if (MCPX_BAND_TWICE == 1) ok = factor_solve(Sc, rrp, dxp, img2, U, sBR, ent_tab, ln);
        if (!ok) {  // the failed linear solve of :84-88
          status = 1;
          reason |= MCPX_FAIL_LINSOLVE;
          break;
        }
        __syncthreads();
        // δy_k = (ry_k − Σ_j R_kj δx_j)·D_k⁻¹, δs_k = (−F_Ck − s_k δy_k)·(y_k + tol)⁻¹
        double yv[RMB], sv[RMB], dyv[RMB], dsv[RMB];
        bool own[RMB];
#pragma unroll
        for (int r = 0; r < RMB; ++r) {
          constexpr int WD = 2 * MCPX_NL_BD_KR;
          const int k = ln + 64 * r;
          own[r] = k < m;
          const int kk = own[r] ? k : 0;
          yv[r] = zs[n + kk];
          sv[r] = zs[n + m + kk];
          double acc = ry[r];
#pragma unroll
          for (int t = 0; t < MCPX_NL_BD_KR; ++t) {
            const int rs = bd_tab[(r * WD + 2 * t) * 64 + ln];
            const int sj = bd_tab[(r * WD + 2 * t + 1) * 64 + ln];
            if (own[r] && rs >= 0) acc = fma(-cb[rs], dxp[sj], acc);
          }
          dyv[r] = acc * sDi[kk];
          dsv[r] = fma(-sv[r], dyv[r], -(sv[r] * yv[r] - eps)) * rw[r];
        }
        // fraction-to-the-boundary line search (:93-100, :127-138)
        uint64_t vs = 0ull, vy = 0ull;
        double alpha = 1.0;
        bool clean_s = false, clean_y = false;
        for (int e = 0; e < args.n_trials; ++e) {
          bool bs = false, by = false;
#pragma unroll
          for (int r = 0; r < RMB; ++r) {
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
        // update (:103-105; x moves with α_s)
#pragma unroll
        for (int r = 0; r < RNB; ++r) {
          const int j = ln + 64 * r;
          if (j < n) zs[j] = zs[j] + as * dxp[ipx[r]];
        }
#pragma unroll
        for (int r = 0; r < RMB; ++r) {
          if (own[r]) {
            const int k = ln + 64 * r;
            zs[n + m + k] = sv[r] + as * dsv[r];
            zs[n + k] = yv[r] + ay * dyv[r];
          }
        }
        kkt = kkt_step;  // :107
        ++inner;
        ++newton;
      }
      eps *= (status == 0) ? args.tight[inner] : args.loose[inner];  // :111-113
      ++outer;                                                        // :114
    }
    if (outer == args.max_outer) {  // :117-119
      status = 1;
      reason |= MCPX_FAIL_MAX_OUTER;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RNB; ++r) {
      const int j = ln + 64 * r;
      if (j < n) args.x[inst * n + j] = zs[j];
    }
#pragma unroll
    for (int r = 0; r < RMB; ++r) {
      const int k = ln + 64 * r;
      if (k < m) {
        args.y[inst * m + k] = zs[n + k];
        args.s[inst * m + k] = zs[n + m + k];
      }
      if (args.active_mask) {  // W = ⌈m/64⌉ words (include/mcpx.h)
        const int kk = k < m ? k : 0;
        const uint64_t bits = ballot(k < m && zs[n + kk] > zs[n + m + kk]);
        if (ln == 0) args.active_mask[inst * RMB + r] = bits;
      }
    }
    if (ln == 0) {
      args.kkt_error[inst] = kkt;
      args.eps[inst] = eps;
      args.outer_iters[inst] = outer;
      args.status[inst] = status;
      if (args.newton_iters) args.newton_iters[inst] = newton;
      if (args.fail_reason) args.fail_reason[inst] = (uint8_t)reason;
    }
  }
}

}  // namespace band
}  // namespace nl
}  // namespace mcpx

#endif  // MCPX_NL_CAN_BAND
