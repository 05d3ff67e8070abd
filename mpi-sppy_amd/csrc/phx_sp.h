// phx_sp.h — workgroup-per-scenario sparse KKT solver ("sp") for subproblems too
// large for the register lane solver (phx_lane.h) and the LDS-dense workgroup
// solver (phx_wg.h): netdes network-50-30-H (n = 2,940, m = 1,520, 1,470 nonants).
//
// Reference semantics being replaced: SPOpt.solve_one (mpisppy/spopt.py:85-223),
// one external LP/QP solve per scenario, called from PHBase.solve_loop
// (phbase.py:494-568) in Iter0 (W, prox off: an LP) and in every PH iteration
// (prox on: strictly convex in the nonants, phbase.py:617-699).
//
// Linear algebra.  Every Newton / KKT system of the solver reduces to the normal
// matrix over the rows
//      M = A H^-1 A' + D          (H: column weights, D: row diagonal;
//                                  rows with D < 0 are inactive: identity rows)
// Rows are split ONCE on the host (phx_setup.h build_sp_sym) into B, a maximal
// set of rows no two of which share a column, and the separator C (the rest).
// M_BB is then diagonal and M t = r is solved by block elimination with the
// dense separator Schur complement
//      S_C = M_CC - M_CB M_BB^-1 M_BC      (|C| x |C|, LDS, Cholesky)
// netdes: B = the 1,470 capacity rows (y_e <= u_e x_e touch x_e and y_e only),
// C = the 50 flow-balance rows; sslp: B = 45 client rows, C = 15 facility rows;
// farmer crops_multiplier=10: C = 31 rows.
//
// Algorithm per scenario (one workgroup, phx_kernels.hip k_sp_solve):
//   warm (PH iterations >= 1): classify the previous solution's bounds / rows
//     (polish_lane's rule) and run up to `rounds` active-set rounds: regularised
//     KKT solve for the active set + iterative refinement on the unregularised
//     system (proximal-point) -> KKT certificate (relative 1e-9, unscaled) ->
//     primal-dual active-set update (the phx_wg.h / phx_lane.h rounds);
//   cold (Iter0, or a warm start that did not certify): Mehrotra predictor-
//     corrector interior point (ipm_lane of phx_core.h, same steps) on the same
//     normal matrix, then the active set read off the interior point and the
//     same rounds.
// A certified lane is exactly as exact as a lane of the other solvers (same
// certificate); the rest are handed to the generic path.
//
// Parallel layout: thread t owns columns t, t+NT, ... and rows t, t+NT, ...;
// vectors that sparse products gather (x, z/y, column weights, row rhs) live in
// LDS; owner-only state lives in a per-workgroup global scratch slot
// (scenario-major, contiguous: L2-resident while the workgroup runs).  Phases
// are separated by workgroup barriers; each phase writes only owned elements and
// reads values published before its barrier, so the test emulation (tests/emu,
// SP_NT = 1) runs the same code serially.  Reductions: wave butterflies (the
// same value in every lane) + a fixed-order sum over the waves.
#pragma once
#include "phx_core.h"

namespace phx {

#if defined(__HIP_DEVICE_COMPILE__)
#define SP_TID ((int)threadIdx.x)
#define SP_NT ((int)blockDim.x)
#define SP_SYNC() __syncthreads()
#else
#define SP_TID 0
#define SP_NT 1
#define SP_SYNC() ((void)0)
#endif

// Separator rows are the long ones (netdes: the 50 flow balances, ~60 entries
// each, against 2 in a capacity row; sslp: the 15 facility rows, 47 against 15):
// with a thread per row they were each row phase's serial chain.  They get a
// quad each instead (four adjacent threads, the row's entries interleaved,
// combined by two lane shuffles), the B rows a thread each (sp_rows).
#if defined(__HIP_DEVICE_COMPILE__)
#define SP_QW 4
#define SP_QL ((int)threadIdx.x & 3)
#define SP_QID ((int)threadIdx.x >> 2)
#define SP_QN ((int)blockDim.x >> 2)
#else
#define SP_QW 1
#define SP_QL 0
#define SP_QID 0
#define SP_QN 1
#endif
PHX_HD double sp_quad_sum(double v) {
#if defined(__HIP_DEVICE_COMPILE__)
    v = quad_reduce<0>(v);
#endif
    return v;
}

constexpr int SP_MAX_C = 64;      // separator rows: one wavefront's lanes (sp_csolve)
constexpr int SP_RED = 16;        // reduction slots per value (<= 16 waves per workgroup)

// Host-built symbolic structure (phx_setup.h build_sp_sym), device pointers.
struct SpSym {
    int32_t nC, nlink, ld, nvar;
    const int32_t* cpos;   // [m]   row -> separator position, -1 for a B row
    const int32_t* crow;   // [nC]  separator position -> row
    const int32_t* lptr;   // [m+1] links (B row, C row sharing columns) of each B row
    const int32_t* lc;     // [nlink] separator position of the link
    const int32_t* lrow;   // [nlink] B row of the link
    const int32_t* lkp;    // [nlink+1] shared columns of the link, as CSR positions
    const int32_t* lkb;    //   ... in the B row
    const int32_t* lkc;    //   ... in the C row
    const int32_t* clp;    // [nC+1] links into each separator row
    const int32_t* cll;    // [nlink] link ids
    const int32_t* eap;    // [nC*nC+1] direct terms of S_C entry (c1, c2), c1 >= c2, at c1*nC + c2:
    const int32_t* eka;    //   CSR position in row crow[c1]
    const int32_t* ekb;    //   CSR position in row crow[c2] (same column)
    const int32_t* ebp;    // [nC*nC+1] B-row terms of entry (c1, c2):
    const int32_t* el1;    //   link of a B row into c1
    const int32_t* el2;    //   link of the same B row into c2
    const double* AvT;     // [S][nvar] scaled scenario-varying A values, scenario-major
    // gather tables (phx_setup.h build_sp_tables)
    const double* eab;     // [eap[nC*nC]] A[eka] A[ekb] of a direct term, NaN: either varies
    const int32_t* ecol;   //   its column
    const double* lab;     // [lkp[nlink]] A[lkb] A[lkc] of a link term, NaN: either varies
    const int32_t* lcol;   //   its column
    const double* Acsc;    // [nnz] scaled constant A in CSC order
    const int32_t* kvcsc;  // [nnz] its variation index (-1: constant) in CSC order
};

// One scenario's LDS.
struct SpLds {
    double *Sm;    // [nC * ld] separator Schur complement / Cholesky factor
    double *dg;    // [nC] 1 / L_kk
    double *cv;    // [nC] separator right-hand side / solution
    double *lv;    // [nlink] M_bc of each link
    double *Mbb;   // [m] 1 / (the diagonal of M) on the B rows (one division per B row per
                   //     factorisation; the Schur terms and the M solves multiply)
    double *hv;    // [n] column weights H^-1 / gathered column vector
    double *xv;    // [n] x (scaled)
    double *yv;    // [m] y (interior point) or z = -y (active set)
    double *tv;    // [m] row right-hand side / solution
    double *red;   // [8 * SP_RED] reduction slots
    // PHX_SP_PROF: 16 LDS slots of thread 0's phase clocks (15: the last stamp),
    // null when off (k_sp_solve_t / k_sp_polish add them to the global sums)
    unsigned long long* prof = nullptr;
};

// Phase clocks (PHX_SP_PROF=1): the cycles since the last stamp go to phase ph.
// Phases: 0 load / classify, 1 B rows + separator Schur assembly, 2 separator
// Cholesky, 3-6 a refinement step's column residual, row products, M solve,
// update + stop test, 7 certificate, 8 active-set update, 9-11 interior point:
// KKT error + mu, a direction's products before / after its M solve (+ steps);
// counters 12 refinement steps, 13 interior-point iterations, 14 rounds.
#if defined(__HIP_DEVICE_COMPILE__)
#define SP_TP(ph)                                                                       \
    do {                                                                                \
        if (L.prof && threadIdx.x == 0) {                                               \
            const unsigned long long _n = (unsigned long long)clock64();                \
            L.prof[ph] += _n - L.prof[15];                                              \
            L.prof[15] = _n;                                                            \
        }                                                                               \
    } while (0)
#define SP_CNT(ph) do { if (L.prof && threadIdx.x == 0) L.prof[ph] += 1ull; } while (0)
#else
#define SP_TP(ph) ((void)0)
#define SP_CNT(ph) ((void)0)
#endif

// Split layout (split = true): the link / B-row / column vectors (lv, Mbb,
// hv, xv: nlink + m + 2n doubles) live in the workgroup's global scratch slot
// instead of LDS, so that more workgroups fit a CU (netdes 50-30-H: 129 KB of
// LDS per workgroup, one per CU, against 46 KB, three).
// Level 2 (round 5): the row right-hand side / solution tv too (netdes: 46 ->
// 34 KB of LDS, four workgroups per CU with k_sp_solve_t<4>'s register cap).
PHX_HD size_t sp_split_doubles(int n, int m, int nlink, int level = 1) {
    return (size_t)nlink + (size_t)m + 2 * (size_t)n + (level >= 2 ? (size_t)m : 0);
}

PHX_HD size_t sp_lds_bytes(int n, int m, int nC, int nlink, int split = 0) {
    const size_t ld = (size_t)(nC | 1);
    size_t d = (size_t)nC * ld + 2 * (size_t)nC + 2 * (size_t)m + 8 * SP_RED;
    if (!split) d += sp_split_doubles(n, m, nlink);
    if (split >= 2) d -= (size_t)m;
    return d * 8;
}

// gbase: the split vectors' place (null: LDS, after the rest); level 2: tv there too
PHX_HD SpLds sp_carve(double* base, int n, int m, int nC, int nlink, double* gbase = nullptr, int level = 1) {
    SpLds L;
    double* d = base;
    L.red = d; d += 8 * SP_RED;
    L.Sm = d; d += (size_t)nC * (nC | 1);
    L.dg = d; d += nC;
    L.cv = d; d += nC;
    L.yv = d; d += m;
    const bool tvg = gbase && level >= 2;
    if (!tvg) { L.tv = d; d += m; }
    double* g = gbase ? gbase : d;
    if (tvg) { L.tv = g; g += m; }
    L.lv = g; g += nlink;
    L.Mbb = g; g += m;
    L.hv = g; g += n;
    L.xv = g; g += n;
    return L;
}

// Owner-only per-column / per-row state of one workgroup slot (global scratch).
struct SpScr {
    double *qq, *pp, *lb, *ub, *r1, *aty, *dx, *zl, *zu, *dzl, *dzu, *cl, *cu, *hx;   // [n]
    double *bl, *bu, *ax, *rdg, *s, *wl, *wu, *ds, *dwl, *dwu, *cwl, *cwu;           // [m]
    int32_t *cc, *rc;                                                               // [n], [m]
};

PHX_HD size_t sp_scr_doubles(int n, int m) {
    return 14 * (size_t)n + 12 * (size_t)m + ((size_t)n + (size_t)m + 1) / 2 + 2;
}

// rows_lds: the twelve row vectors' place when they fit the workgroup's LDS
// (small problems: sslp, 60 rows -- 5.8 KB; null: in the slot)
PHX_HD SpScr sp_scr_carve(double* base, int n, int m, double* rows_lds = nullptr) {
    SpScr G;
    double* d = base;
    double** cols[] = {&G.qq, &G.pp, &G.lb, &G.ub, &G.r1, &G.aty, &G.dx, &G.zl, &G.zu, &G.dzl, &G.dzu,
                       &G.cl, &G.cu, &G.hx};
    for (double** p : cols) { *p = d; d += n; }
    double** rows[] = {&G.bl, &G.bu, &G.ax, &G.rdg, &G.s, &G.wl, &G.wu, &G.ds, &G.dwl, &G.dwu, &G.cwl, &G.cwu};
    double* r = rows_lds ? rows_lds : d;
    for (double** p : rows) { *p = r; r += m; }
    if (!rows_lds) d = r;
    G.cc = (int32_t*)d;
    G.rc = G.cc + n;
    return G;
}

// (branch-free: the constant value, the variation index and -- at a clamped
// index -- the scenario's value are loaded without waiting for each other)
// Column bounds the same in every scenario (no per-scenario fixing): the
// scratch's lb / ub point at the problem's shared arrays (L2-resident, read by
// every workgroup) instead of a per-slot copy re-read from memory
PHX_HD SpScr sp_scr_shared(SpScr G, const Prob& P) {
    if (P.lb.ss == 0 && P.lb.si == 1 && P.ub.ss == 0 && P.ub.si == 1) {
        G.lb = (double*)P.lb.p;      // (never written: sp_load skips them)
        G.ub = (double*)P.ub.p;
    }
    return G;
}

PHX_HD double sp_a(const Prob& P, const SpSym& Y, int k, int s) {
    const int v = P.kvar[k];
    const double ac = P.Ac[k];
    const double av = Y.AvT[(int64_t)s * Y.nvar + (v < 0 ? 0 : v)];
    return v < 0 ? ac : av;
}
// A at CSC position k (the column loops), without the csc2csr hop
PHX_HD double sp_a_csc(const SpSym& Y, int k, int s) {
    const int v = Y.kvcsc[k];
    const double ac = Y.Acsc[k];
    const double av = Y.AvT[(int64_t)s * Y.nvar + (v < 0 ? 0 : v)];
    return v < 0 ? ac : av;
}

// A row phase: body(i, (A v1)_i, (A v2)_i) for every row i, the B rows by a
// thread each, the separator rows by a quad each (every thread of the quad
// computes the sums; body runs on the quad's first) -- every row by a quad when
// there are at most as many rows as quads (sslp: 60 rows, its 45 client rows
// 15 entries each).  v2 null: 0.
template <class F>
PHX_HD void sp_rows(const Prob& P, const SpSym& Y, int s, const double* v1, const double* v2, F&& body) {
    const bool allq = P.m <= SP_QN && SP_QW > 1;
    for (int i = SP_TID; i < (allq ? 0 : P.m); i += SP_NT) {
        if (Y.cpos[i] >= 0) continue;
        double a1 = 0.0, a2 = 0.0;
        for (int k = P.rowptr[i]; k < P.rowptr[i + 1]; ++k) {
            const double a = sp_a(P, Y, k, s);
            const int j = P.colidx[k];
            a1 += a * v1[j];
            if (v2) a2 += a * v2[j];
        }
        body(i, a1, a2);
    }
    for (int c = SP_QID; c < (allq ? P.m : Y.nC); c += SP_QN) {
        const int i = allq ? c : Y.crow[c];
        double a1 = 0.0, a2 = 0.0;
        for (int k = P.rowptr[i] + SP_QL; k < P.rowptr[i + 1]; k += SP_QW) {
            const double a = sp_a(P, Y, k, s);
            const int j = P.colidx[k];
            a1 += a * v1[j];
            if (v2) a2 += a * v2[j];
        }
        a1 = sp_quad_sum(a1);
        if (v2) a2 = sp_quad_sum(a2);
        if (SP_QL == 0) body(i, a1, a2);
    }
}

// ---- workgroup reductions of K values (op 0 sum, 1 max, 2 min); the result in
//      every thread, identical (commutative butterflies, fixed wave order) ----
PHX_HD double sp_op(double a, double b, int op) { return op == 0 ? a + b : (op == 1 ? fmax(a, b) : fmin(a, b)); }

template <int K>
PHX_HD void sp_reduce(double* v, double* red, int op) {
#if defined(__HIP_DEVICE_COMPILE__)
    for (int q = 0; q < K; ++q)
        v[q] = op == 0 ? wave_reduce<0>(v[q]) : (op == 1 ? wave_reduce<1>(v[q]) : wave_reduce<2>(v[q]));
    const int nw = (int)(blockDim.x >> 6), w = (int)(threadIdx.x >> 6);
    __syncthreads();
    if ((threadIdx.x & 63) == 0)
        for (int q = 0; q < K; ++q) red[q * SP_RED + w] = v[q];
    __syncthreads();
    for (int q = 0; q < K; ++q) {
        double t = red[q * SP_RED];
        for (int i = 1; i < nw; ++i) t = sp_op(t, red[q * SP_RED + i], op);
        v[q] = t;
    }
#else
    (void)v; (void)red; (void)op;
#endif
}

// ---------------------------------------------------------------------------
// Factorization of M for column weights L.hv (0: column eliminated) and row
// diagonals G.rdg (< 0: inactive row).  Returns false (uniformly) when the
// separator Schur complement is not positive definite.  ipm_safe (interior
// point): a pivot that collapses relative to the separator row's diagonal of
// M itself (a dependent row of A H^-1 A' near an interior-point optimum; the
// B-row elimination cancels up to 1/reg ~ 1e10) is replaced by a huge value,
// which zeroes that component of the solve — cholesky_ipm's safeguard
// (phx_lane.h).
// ---------------------------------------------------------------------------
PHX_HD bool sp_factor_once(const Prob& P, const SpSym& Y, const SpScr& G, const SpLds& L, int s, bool ipm_safe);
// (PHX_SP_FACTOR_TWICE, an experiment build: every factorization done twice,
// its time measured as the difference)
PHX_HD bool sp_factor(const Prob& P, const SpSym& Y, const SpScr& G, const SpLds& L, int s,
                      bool ipm_safe = false) {
#ifdef PHX_SP_FACTOR_TWICE
    (void)sp_factor_once(P, Y, G, L, s, ipm_safe);
#endif
    return sp_factor_once(P, Y, G, L, s, ipm_safe);
}
PHX_HD bool sp_factor_once(const Prob& P, const SpSym& Y, const SpScr& G, const SpLds& L, int s,
                           bool ipm_safe) {
    const int m = P.m, nC = Y.nC, ld = Y.ld;
    // B-row diagonal and the links M_bc (a quad per B row when there are at
    // most as many rows as quads, as sp_rows: its entries and its links
    // interleaved)
    const bool bq = m <= SP_QN && SP_QW > 1;
    const int b_id = bq ? SP_QID : SP_TID, b_n = bq ? SP_QN : SP_NT, b_l = bq ? SP_QL : 0, b_w = bq ? SP_QW : 1;
    for (int i = b_id; i < m; i += b_n) {
        if (Y.cpos[i] >= 0) continue;
        const double rd = G.rdg[i];
        double v = 1.0;
        if (rd >= 0.0) {
            double t = 0.0;
            for (int k = P.rowptr[i] + b_l; k < P.rowptr[i + 1]; k += b_w) {
                const double a = sp_a(P, Y, k, s);
                t += a * a * L.hv[P.colidx[k]];
            }
            if (bq) t = sp_quad_sum(t);
            v = rd + t;
        }
        if (b_l == 0) L.Mbb[i] = 1.0 / v;
        for (int l = Y.lptr[i] + b_l; l < Y.lptr[i + 1]; l += b_w) {
            double w = 0.0;
            if (rd >= 0.0 && G.rdg[Y.crow[Y.lc[l]]] >= 0.0)
                for (int t = Y.lkp[l]; t < Y.lkp[l + 1]; ++t) {
                    const double ab = Y.lab[t];
                    w += (ab == ab ? ab : sp_a(P, Y, Y.lkb[t], s) * sp_a(P, Y, Y.lkc[t], s)) * L.hv[Y.lcol[t]];
                }
            L.lv[l] = w;
        }
    }
    SP_SYNC();
    // separator Schur complement (lower part, Sm[c1*ld + c2], c1 >= c2): the
    // off-diagonal entries a thread each (a few terms: the columns and B rows
    // two separator rows share), the diagonal ones a quad each (every column
    // and B row of the row: netdes ~60 + ~30 terms)
    // (a quad each too when there are at most twice as many entries as quads:
    // sslp's 105 each sum over all 45 client rows)
    const bool offq = nC * (nC - 1) / 2 <= 2 * SP_QN && SP_QW > 1;
    const int o_id = offq ? SP_QID : SP_TID, o_n = offq ? SP_QN : SP_NT, o_l = offq ? SP_QL : 0, o_w = offq ? SP_QW : 1;
    for (int p = o_id; p < nC * nC; p += o_n) {
        const int c1 = p / nC, c2 = p - c1 * nC;
        if (c2 >= c1) continue;
        const double d1 = G.rdg[Y.crow[c1]], d2 = G.rdg[Y.crow[c2]];
        double v = 0.0, w = 0.0;
        if (!(d1 < 0.0 || d2 < 0.0)) {
            for (int t = Y.eap[p] + o_l; t < Y.eap[p + 1]; t += o_w) {
                const double ab = Y.eab[t];
                v += (ab == ab ? ab : sp_a(P, Y, Y.eka[t], s) * sp_a(P, Y, Y.ekb[t], s)) * L.hv[Y.ecol[t]];
            }
            for (int t = Y.ebp[p] + o_l; t < Y.ebp[p + 1]; t += o_w) {
                const int l1 = Y.el1[t];
                w += L.lv[l1] * L.lv[Y.el2[t]] * L.Mbb[Y.lrow[l1]];
            }
        }
        if (offq) {
            v = sp_quad_sum(v);
            w = sp_quad_sum(w);
        }
        if (o_l == 0) L.Sm[c1 * ld + c2] = v - w;
    }
    for (int c = SP_QID; c < nC; c += SP_QN) {
        const int p = c * nC + c;
        const double d1 = G.rdg[Y.crow[c]];
        if (d1 < 0.0) {
            if (SP_QL == 0) { L.Sm[c * ld + c] = 1.0; L.cv[c] = 1.0; }
            continue;
        }
        double v = 0.0, w = 0.0;
        for (int t = Y.eap[p] + SP_QL; t < Y.eap[p + 1]; t += SP_QW) {
            const double ab = Y.eab[t];
            v += (ab == ab ? ab : sp_a(P, Y, Y.eka[t], s) * sp_a(P, Y, Y.ekb[t], s)) * L.hv[Y.ecol[t]];
        }
        for (int t = Y.ebp[p] + SP_QL; t < Y.ebp[p + 1]; t += SP_QW) {
            const int l1 = Y.el1[t];
            w += L.lv[l1] * L.lv[Y.el2[t]] * L.Mbb[Y.lrow[l1]];
        }
        v = d1 + sp_quad_sum(v);
        w = sp_quad_sum(w);
        if (SP_QL == 0) {
            L.cv[c] = v;      // M_cc: the reference of the pivot safeguard
            L.Sm[c * ld + c] = v - w;
        }
    }
    SP_SYNC();
    SP_TP(1);
    // right-looking Cholesky, every trailing entry its own work item; L[i][k]
    // (i > k) is stored transposed at Sm[k*ld + i], 1/L_kk in dg.
    // Pivots in pairs (a, b = a+1), one barrier per pair: every trailing
    // entry applies both updates, with b's column and diagonal corrected for a
    // by the very expressions the one-pivot step stores (the same factor)
    int j2 = 0;
    for (; j2 + 1 < nC; j2 += 2) {
        const int a = j2, b = j2 + 1;
        double d0 = L.Sm[a * ld + a];
        if (ipm_safe) {
            const double c0 = L.cv[a];
            if (!(c0 > 0.0 && c0 < 1e300)) return false;
            if (!(d0 > 1e-13 * c0)) d0 = 1e128;
        }
        if (!(d0 > 0.0)) return false;
        const double e = L.Sm[b * ld + a], id0 = 1.0 / d0;
        double d1 = L.Sm[b * ld + b] - e * e * id0;
        if (ipm_safe) {
            const double c1 = L.cv[b];
            if (!(c1 > 0.0 && c1 < 1e300)) return false;
            if (!(d1 > 1e-13 * c1)) d1 = 1e128;
        }
        if (!(d1 > 0.0)) return false;
        const double sd0 = sqrt(d0), sd1 = sqrt(d1), id1 = 1.0 / d1;
        const int R = nC - b - 1;
        for (int p = SP_TID; p < R * R; p += SP_NT) {
            const int i = b + 1 + p / R, k = b + 1 + (p - (p / R) * R);
            if (k > i) continue;
            const double sia = L.Sm[i * ld + a];
            const double sib = L.Sm[i * ld + b] - sia * e * id0;
            if (k == i) {
                L.Sm[a * ld + i] = sia / sd0;
                L.Sm[b * ld + i] = sib / sd1;
            }
            const double ska = L.Sm[k * ld + a];
            const double hk = L.Sm[k * ld + b] - ska * e * id0;
            const double t = L.Sm[i * ld + k] - sia * ska * id0;
            L.Sm[i * ld + k] = t - sib * hk * id1;
        }
        if (SP_TID == 0) {
            L.dg[a] = 1.0 / sd0;
            L.dg[b] = 1.0 / sd1;
            L.Sm[a * ld + b] = e / sd0;
        }
        SP_SYNC();
    }
    for (int jj = j2; jj < nC; ++jj) {
        double d = L.Sm[jj * ld + jj];
        if (ipm_safe) {
            const double d0 = L.cv[jj];
            if (!(d0 > 0.0 && d0 < 1e300)) return false;
            if (!(d > 1e-13 * d0)) d = 1e128;
        }
        if (!(d > 0.0)) return false;
        const double sd = sqrt(d), id = 1.0 / d;
        const int R = nC - jj - 1;
        for (int p = SP_TID; p < R * R; p += SP_NT) {
            const int i = jj + 1 + p / R, k = jj + 1 + (p - (p / R) * R);
            if (k > i) continue;
            const double sij = L.Sm[i * ld + jj];
            if (k == i) L.Sm[jj * ld + i] = sij / sd;
            L.Sm[i * ld + k] -= sij * L.Sm[k * ld + jj] * id;
        }
        if (SP_TID == 0) L.dg[jj] = 1.0 / sd;
        SP_SYNC();
    }
    SP_TP(2);
    return true;
}

#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ double sp_readlane64(double v, int lane) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u & 0xffffffffull), lane);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), lane);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
#endif
// S_C^-1 cv in place (forward + backward substitution), one wavefront: lane i
// holds separator row i; the other waves wait at the closing barrier.
PHX_HD void sp_csolve(const SpSym& Y, const SpLds& L) {
    const int nC = Y.nC, ld = Y.ld;
#if defined(__HIP_DEVICE_COMPILE__)
    if (threadIdx.x < 64) {
        const int i = (int)threadIdx.x;
        double r = i < nC ? L.cv[i] : 0.0;
        // (lane k's value by v_readlane -- k is uniform -- instead of a
        // ds_bpermute shuffle: the substitution is a chain of 2 nC of them)
        for (int k = 0; k < nC; ++k) {
            const double uk = sp_readlane64(r, k) * L.dg[k];
            if (i > k && i < nC) r -= L.Sm[k * ld + i] * uk;
            if (i == k) r = uk;
        }
        for (int k = nC - 1; k >= 0; --k) {
            const double tk = sp_readlane64(r, k) * L.dg[k];
            if (i < k) r -= L.Sm[i * ld + k] * tk;
            if (i == k) r = tk;
        }
        if (i < nC) L.cv[i] = r;
    }
    __syncthreads();
#else
    for (int k = 0; k < nC; ++k) {
        const double uk = L.cv[k] * L.dg[k];
        L.cv[k] = uk;
        for (int i = k + 1; i < nC; ++i) L.cv[i] -= L.Sm[k * ld + i] * uk;
    }
    for (int k = nC - 1; k >= 0; --k) {
        const double tk = L.cv[k] * L.dg[k];
        L.cv[k] = tk;
        for (int i = 0; i < k; ++i) L.cv[i] -= L.Sm[i * ld + k] * tk;
    }
#endif
}

// M t = r with r in L.tv (rows), solution in L.tv.  Inactive rows: t = r.
PHX_HD void sp_msolve(const Prob& P, const SpSym& Y, const SpLds& L) {
    const int nC = Y.nC;
    // (a quad per separator row: its links -- netdes ~30 B rows -- interleaved)
    for (int c = SP_QID; c < nC; c += SP_QN) {
        double v = 0.0;
        for (int q = Y.clp[c] + SP_QL; q < Y.clp[c + 1]; q += SP_QW) {
            const int l = Y.cll[q];
            const int b = Y.lrow[l];
            v += L.lv[l] * L.tv[b] * L.Mbb[b];
        }
        v = sp_quad_sum(v);
        if (SP_QL == 0) L.cv[c] = L.tv[Y.crow[c]] - v;
    }
    SP_SYNC();
    sp_csolve(Y, L);
    for (int i = SP_TID; i < P.m; i += SP_NT) {
        const int c = Y.cpos[i];
        if (c >= 0) { L.tv[i] = L.cv[c]; continue; }
        double v = L.tv[i];
        for (int l = Y.lptr[i]; l < Y.lptr[i + 1]; ++l) v -= L.lv[l] * L.cv[Y.lc[l]];
        L.tv[i] = v * L.Mbb[i];
    }
    SP_SYNC();
    SP_TP(5);
}

// ---------------------------------------------------------------------------
// Scenario data into the scratch slot (scaled): effective cost / prox weight
// of each column (col_cost), column and row bounds.  Returns max |q / dc|.
// ---------------------------------------------------------------------------
PHX_HD double sp_load(const Prob& P, const SpScr& G, const SpLds& L, int s) {
    double qm = 0.0;
    for (int j = SP_TID; j < P.n; j += SP_NT) {
        double q, p;
        col_cost(P, j, s, q, p);
        G.qq[j] = q;
        G.pp[j] = p;
        if (G.lb != P.lb.p) {
            G.lb[j] = P.lb.at(j, s);
            G.ub[j] = P.ub.at(j, s);
        }
        qm = fmax(qm, fabs(q / P.dc[j]));
    }
    for (int i = SP_TID; i < P.m; i += SP_NT) {
        G.bl[i] = P.bl.at(i, s);
        G.bu[i] = P.bu.at(i, s);
    }
    double v[1] = {qm};
    sp_reduce<1>(v, L.red, 1);
    SP_SYNC();
    return v[0];
}

// Relative KKT error (kkt_error of phx_core.h) of the scaled point (xv, yv);
// leaves A x in G.ax and A'y in G.aty.
PHX_HD double sp_kkt_error(const Prob& P, const SpSym& Y, const SpScr& G, const SpLds& L, int s) {
    double acc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};   // rp2 bn2 rd2 qn2 pobj dobj
    sp_rows(P, Y, s, L.xv, nullptr, [&](int i, double ax, double) {
        G.ax[i] = ax;
        const double dr = P.dr[i], bl = G.bl[i], bu = G.bu[i];
        const double axu = ax / dr;
        const double r = axu - clampd(axu, bl / dr, bu / dr);
        acc[0] += r * r;
        if (isfinite(bl)) acc[1] += (bl / dr) * (bl / dr);
        if (isfinite(bu)) acc[1] += (bu / dr) * (bu / dr);
        const double y = L.yv[i];
        if (y > 0.0 && isfinite(bl)) acc[5] += bl * y;
        else if (y < 0.0 && isfinite(bu)) acc[5] += bu * y;
    });
    for (int j = SP_TID; j < P.n; j += SP_NT) {
        const double q = G.qq[j], p = G.pp[j], x = L.xv[j], dc = P.dc[j], l = G.lb[j], u = G.ub[j];
        double aty = 0.0;
        for (int k = P.colptr[j]; k < P.colptr[j + 1]; ++k)
            aty += sp_a_csc(Y, k, s) * L.yv[P.rowidx[k]];
        G.aty[j] = aty;
        const double lam_s = q + p * x - aty;
        const double lam = lam_s / dc;
        double rd = lam;
        if (isfinite(l) && lam > 0.0) { rd = 0.0; acc[5] += l * lam_s; }
        if (isfinite(u) && lam < 0.0) { rd = 0.0; acc[5] += u * lam_s; }
        acc[2] += rd * rd;
        acc[3] += (q / dc) * (q / dc);
        acc[4] += q * x + 0.5 * p * x * x;
        acc[5] -= 0.5 * p * x * x;
    }
    sp_reduce<6>(acc, L.red, 0);
    const double ep = sqrt(acc[0]) / (1.0 + sqrt(acc[1]));
    const double ed = sqrt(acc[2]) / (1.0 + sqrt(acc[3]));
    const double eg = fabs(acc[4] - acc[5]) / (1.0 + fabs(acc[4]) + fabs(acc[5]));
    // (fmax drops a NaN operand: the sum of the terms catches a non-finite one)
    const double e = fmax(ep, fmax(ed, eg));
    return isfinite(ep + ed + eg) && isfinite(e) ? e : 1e300;
}

// ---------------------------------------------------------------------------
// Interior point (ipm_lane of phx_core.h on the workgroup): x in L.xv, y in
// L.yv (y > 0 <=> lower side active).  The direction of ipm_direction with
// the normal matrix solved by sp_factor / sp_msolve.
// ---------------------------------------------------------------------------
PHX_HD void sp_direction(const Prob& P, const SpSym& Y, const SpScr& G, const SpLds& L, int s) {
    // (the interior point's column / row loops load everything they may use
    // before their branches: one memory round trip per element instead of a
    // chain of them; the arithmetic is unchanged)
    for (int j = SP_TID; j < P.n; j += SP_NT) {
        const double l = G.lb[j], u = G.ub[j], x = L.xv[j];
        const double pp = G.pp[j], qq = G.qq[j], aty = G.aty[j], zl = G.zl[j], zu = G.zu[j], cl = G.cl[j],
                     cu = G.cu[j], hx = G.hx[j];
        if (l == u) { G.dx[j] = 0.0; L.hv[j] = 0.0; continue; }
        double rd = pp * x + qq - aty;
        double rho = 0.0;
        if (isfinite(l)) { rd -= zl; rho += cl / (x - l); }
        if (isfinite(u)) { rd += zu; rho -= cu / (u - x); }
        G.dx[j] = rho - rd;
        L.hv[j] = (rho - rd) / hx;
    }
    SP_SYNC();
    sp_rows(P, Y, s, L.hv, nullptr, [&](int i, double adr, double) {
        const double bl = G.bl[i], bu = G.bu[i];
        const double ax = G.ax[i];
        double rhs;
        if (!isfinite(bl) && !isfinite(bu)) {
            rhs = 0.0;
            G.ds[i] = 0.0;
        } else if (bl == bu) {
            rhs = -(ax - bl) - adr;
            G.ds[i] = 0.0;
        } else {
            const double sv = G.s[i], y = L.yv[i];
            const double wl = G.wl[i], wu = G.wu[i], cwl = G.cwl[i], cwu = G.cwu[i];
            double rs = y, rhos = 0.0, sig = 0.0;
            if (isfinite(bl)) { rs -= wl; rhos += cwl / (sv - bl); sig += wl / (sv - bl); }
            if (isfinite(bu)) { rs += wu; rhos -= cwu / (bu - sv); sig += wu / (bu - sv); }
            rhos -= rs;
            G.ds[i] = rhos;
            rhs = -(ax - sv) + rhos / sig - adr;
        }
        L.tv[i] = rhs;
    });
    SP_SYNC();
    SP_TP(10);
    sp_msolve(P, Y, L);
    for (int i = SP_TID; i < P.m; i += SP_NT) {
        const double bl = G.bl[i], bu = G.bu[i];
        const double dy = L.tv[i], sv = G.s[i], wl = G.wl[i], wu = G.wu[i], ds = G.ds[i], cwl = G.cwl[i],
                     cwu = G.cwu[i];
        if (bl == bu || (!isfinite(bl) && !isfinite(bu))) continue;
        double sig = 0.0;
        if (isfinite(bl)) sig += wl / (sv - bl);
        if (isfinite(bu)) sig += wu / (bu - sv);
        const double dsv = (ds - dy) / sig;
        G.ds[i] = dsv;
        if (isfinite(bl)) G.dwl[i] = (cwl - wl * dsv) / (sv - bl);
        if (isfinite(bu)) G.dwu[i] = (cwu + wu * dsv) / (bu - sv);
    }
    for (int j = SP_TID; j < P.n; j += SP_NT) {
        const double l = G.lb[j], u = G.ub[j], x = L.xv[j];
        const double dx = G.dx[j], hx = G.hx[j], cl = G.cl[j], zl = G.zl[j], cu = G.cu[j], zu = G.zu[j];
        if (l == u) continue;
        double atdy = 0.0;
        for (int k = P.colptr[j]; k < P.colptr[j + 1]; ++k)
            atdy += sp_a_csc(Y, k, s) * L.tv[P.rowidx[k]];
        const double dxv = (dx + atdy) / hx;
        G.dx[j] = dxv;
        if (isfinite(l)) G.dzl[j] = (cl - zl * dxv) / (x - l);
        if (isfinite(u)) G.dzu[j] = (cu + zu * dxv) / (u - x);
    }
    SP_TP(11);
}

PHX_HD void sp_steps(const Prob& P, const SpScr& G, const SpLds& L, double& ap, double& ad) {
    double v[2] = {1.0, 1.0};
    for (int j = SP_TID; j < P.n; j += SP_NT) {
        const double l = G.lb[j], u = G.ub[j], x = L.xv[j], d = G.dx[j];
        const double dzl = G.dzl[j], zl = G.zl[j], dzu = G.dzu[j], zu = G.zu[j];
        if (l == u) continue;
        if (isfinite(l)) {
            if (d < 0.0) v[0] = fmin(v[0], -(x - l) / d);
            if (dzl < 0.0) v[1] = fmin(v[1], -zl / dzl);
        }
        if (isfinite(u)) {
            if (d > 0.0) v[0] = fmin(v[0], (u - x) / d);
            if (dzu < 0.0) v[1] = fmin(v[1], -zu / dzu);
        }
    }
    for (int i = SP_TID; i < P.m; i += SP_NT) {
        const double bl = G.bl[i], bu = G.bu[i], sv = G.s[i], d = G.ds[i];
        const double dwl = G.dwl[i], wl = G.wl[i], dwu = G.dwu[i], wu = G.wu[i];
        if (bl == bu) continue;
        if (isfinite(bl)) {
            if (d < 0.0) v[0] = fmin(v[0], -(sv - bl) / d);
            if (dwl < 0.0) v[1] = fmin(v[1], -wl / dwl);
        }
        if (isfinite(bu)) {
            if (d > 0.0) v[0] = fmin(v[0], (bu - sv) / d);
            if (dwu < 0.0) v[1] = fmin(v[1], -wu / dwu);
        }
    }
    sp_reduce<2>(v, L.red, 2);
    ap = v[0];
    ad = v[1];
}

PHX_HD double sp_ipm(const Prob& P, const SpSym& Y, const SpScr& G, const SpLds& L, int s, int max_it,
                     double tol, double reg, int* its) {
    const int n = P.n, m = P.m;
    SP_TP(0);
    for (int j = SP_TID; j < n; j += SP_NT) {
        const double l = G.lb[j], u = G.ub[j];
        double x;
        if (l == u) x = l;
        else if (isfinite(l) && isfinite(u)) x = (u - l <= 2.0) ? 0.5 * (l + u) : clampd(0.0, l + 1.0, u - 1.0);
        else x = clampd(0.0, isfinite(l) ? l + 1.0 : -1e300, isfinite(u) ? u - 1.0 : 1e300);
        L.xv[j] = x;
        const double g = G.qq[j] + G.pp[j] * x;
        G.zl[j] = isfinite(l) && l != u ? fmax(g, 0.0) + 1.0 : 0.0;
        G.zu[j] = isfinite(u) && l != u ? fmax(-g, 0.0) + 1.0 : 0.0;
        G.dzl[j] = G.dzu[j] = 0.0;
    }
    SP_SYNC();
    sp_rows(P, Y, s, L.xv, nullptr, [&](int i, double ax, double) {
        const double bl = G.bl[i], bu = G.bu[i];
        double sv;
        const bool eq = (bl == bu);
        if (eq) sv = bl;
        else if (isfinite(bl) && isfinite(bu)) sv = (bu - bl <= 2.0) ? 0.5 * (bl + bu) : clampd(ax, bl + 1.0, bu - 1.0);
        else sv = clampd(ax, isfinite(bl) ? bl + 1.0 : -1e300, isfinite(bu) ? bu - 1.0 : 1e300);
        G.s[i] = sv;
        G.wl[i] = (isfinite(bl) && !eq) ? 1.0 : 0.0;
        G.wu[i] = (isfinite(bu) && !eq) ? 1.0 : 0.0;
        G.dwl[i] = G.dwu[i] = 0.0;
        L.yv[i] = G.wl[i] - G.wu[i];
    });
    SP_SYNC();
    double err = 1e300;
    int it = 0;
    for (; it < max_it; ++it) {
        err = sp_kkt_error(P, Y, G, L, s);
        double mu_acc[2] = {0.0, 0.0};
        for (int j = SP_TID; j < n; j += SP_NT) {
            const double l = G.lb[j], u = G.ub[j], x = L.xv[j], zl = G.zl[j], zu = G.zu[j];
            if (l == u) continue;
            if (isfinite(l)) { mu_acc[0] += (x - l) * zl; mu_acc[1] += 1.0; }
            if (isfinite(u)) { mu_acc[0] += (u - x) * zu; mu_acc[1] += 1.0; }
        }
        for (int i = SP_TID; i < m; i += SP_NT) {
            const double bl = G.bl[i], bu = G.bu[i], sv = G.s[i], wl = G.wl[i], wu = G.wu[i];
            if (bl == bu) continue;
            if (isfinite(bl)) { mu_acc[0] += (sv - bl) * wl; mu_acc[1] += 1.0; }
            if (isfinite(bu)) { mu_acc[0] += (bu - sv) * wu; mu_acc[1] += 1.0; }
        }
        sp_reduce<2>(mu_acc, L.red, 0);
        SP_TP(9);
        SP_CNT(13);
        const double ncomp = mu_acc[1];
        const double mu = ncomp > 0.0 ? mu_acc[0] / ncomp : 0.0;
        if (err < tol || !(err < 1e300)) break;
        // column weights H^-1 and row diagonals of the normal matrix
        for (int j = SP_TID; j < n; j += SP_NT) {
            const double l = G.lb[j], u = G.ub[j], x = L.xv[j], zl = G.zl[j], zu = G.zu[j];
            double h = G.pp[j] + reg;
            if (l == u) h = 1e300;
            else {
                if (isfinite(l)) h += zl / (x - l);
                if (isfinite(u)) h += zu / (u - x);
            }
            G.hx[j] = h;
            L.hv[j] = (l == u) ? 0.0 : 1.0 / h;
        }
        for (int i = SP_TID; i < m; i += SP_NT) {
            const double bl = G.bl[i], bu = G.bu[i];
            double dg;
            if (!isfinite(bl) && !isfinite(bu)) dg = -1.0;
            else if (bl == bu) dg = reg;
            else {
                const double sv = G.s[i], wl = G.wl[i], wu = G.wu[i];
                double sig = 0.0;
                if (isfinite(bl)) sig += wl / (sv - bl);
                if (isfinite(bu)) sig += wu / (bu - sv);
                dg = 1.0 / sig + reg;
            }
            G.rdg[i] = dg;
        }
        SP_SYNC();
        if (!sp_factor(P, Y, G, L, s, true)) break;
        // ---- predictor ----
        for (int j = SP_TID; j < n; j += SP_NT) {
            const double l = G.lb[j], u = G.ub[j], x = L.xv[j], zl = G.zl[j], zu = G.zu[j];
            G.cl[j] = isfinite(l) ? -(x - l) * zl : 0.0;
            G.cu[j] = isfinite(u) ? -(u - x) * zu : 0.0;
        }
        for (int i = SP_TID; i < m; i += SP_NT) {
            const double bl = G.bl[i], bu = G.bu[i], sv = G.s[i], wl = G.wl[i], wu = G.wu[i];
            G.cwl[i] = (isfinite(bl) && bl != bu) ? -(sv - bl) * wl : 0.0;
            G.cwu[i] = (isfinite(bu) && bl != bu) ? -(bu - sv) * wu : 0.0;
        }
        sp_direction(P, Y, G, L, s);
        double ap, ad;
        sp_steps(P, G, L, ap, ad);
        double maff[1] = {0.0};
        for (int j = SP_TID; j < n; j += SP_NT) {
            const double l = G.lb[j], u = G.ub[j], x = L.xv[j];
            const double dx = G.dx[j], zl = G.zl[j], dzl = G.dzl[j], zu = G.zu[j], dzu = G.dzu[j];
            if (l == u) continue;
            if (isfinite(l)) maff[0] += (x - l + ap * dx) * (zl + ad * dzl);
            if (isfinite(u)) maff[0] += (u - x - ap * dx) * (zu + ad * dzu);
        }
        for (int i = SP_TID; i < m; i += SP_NT) {
            const double bl = G.bl[i], bu = G.bu[i], sv = G.s[i];
            const double ds = G.ds[i], wl = G.wl[i], dwl = G.dwl[i], wu = G.wu[i], dwu = G.dwu[i];
            if (bl == bu) continue;
            if (isfinite(bl)) maff[0] += (sv - bl + ap * ds) * (wl + ad * dwl);
            if (isfinite(bu)) maff[0] += (bu - sv - ap * ds) * (wu + ad * dwu);
        }
        sp_reduce<1>(maff, L.red, 0);
        const double ma = ncomp > 0.0 ? maff[0] / ncomp : 0.0;
        const double ratio = mu > 0.0 ? ma / mu : 0.0;
        const double smu = ratio * ratio * ratio * mu;
        // ---- corrector ----
        for (int j = SP_TID; j < n; j += SP_NT) {
            const double l = G.lb[j], u = G.ub[j], x = L.xv[j];
            const double dx = G.dx[j], zl = G.zl[j], dzl = G.dzl[j], zu = G.zu[j], dzu = G.dzu[j];
            G.cl[j] = isfinite(l) ? smu - (x - l) * zl - dx * dzl : 0.0;
            G.cu[j] = isfinite(u) ? smu - (u - x) * zu + dx * dzu : 0.0;
        }
        for (int i = SP_TID; i < m; i += SP_NT) {
            const double bl = G.bl[i], bu = G.bu[i], sv = G.s[i];
            const double ds = G.ds[i], wl = G.wl[i], dwl = G.dwl[i], wu = G.wu[i], dwu = G.dwu[i];
            G.cwl[i] = (isfinite(bl) && bl != bu) ? smu - (sv - bl) * wl - ds * dwl : 0.0;
            G.cwu[i] = (isfinite(bu) && bl != bu) ? smu - (bu - sv) * wu + ds * dwu : 0.0;
        }
        SP_SYNC();
        sp_direction(P, Y, G, L, s);
        sp_steps(P, G, L, ap, ad);
        ap = fmin(1.0, 0.995 * ap);
        ad = fmin(1.0, 0.995 * ad);
        // keep the last finite iterate (an infeasible subproblem's diverging
        // multipliers are its Farkas ray; a NaN step would erase them)
        double fin[1] = {0.0};
        for (int j = SP_TID; j < n; j += SP_NT) fin[0] += G.dx[j] + G.dzl[j] + G.dzu[j];
        for (int i = SP_TID; i < m; i += SP_NT) fin[0] += G.ds[i] + G.dwl[i] + G.dwu[i] + L.tv[i];
        sp_reduce<1>(fin, L.red, 0);
        if (!isfinite(fin[0] + ap + ad)) break;
        for (int j = SP_TID; j < n; j += SP_NT) {
            L.xv[j] += ap * G.dx[j];
            G.zl[j] += ad * G.dzl[j];
            G.zu[j] += ad * G.dzu[j];
        }
        for (int i = SP_TID; i < m; i += SP_NT) {
            G.s[i] += ap * G.ds[i];
            G.wl[i] += ad * G.dwl[i];
            G.wu[i] += ad * G.dwu[i];
            L.yv[i] += ad * L.tv[i];
        }
        SP_SYNC();
        SP_TP(11);
    }
    *its = it;
    return err;
}

// ---------------------------------------------------------------------------
// Active set of the point (xv, yv) (polish_lane's rule, relative tolerance
// tol): column codes cc (0 free, 1 at l, 2 at u), row codes rc (0 inactive,
// 1 at bl, 2 at bu); xv <- the bound value on bound-active columns, yv <- z
// (= -y on active rows, 0 elsewhere).
// ---------------------------------------------------------------------------
PHX_HD void sp_classify(const Prob& P, const SpSym& Y, const SpScr& G, const SpLds& L, int s, double tol) {
    for (int j = SP_TID; j < P.n; j += SP_NT) {
        const double x = L.xv[j], l = G.lb[j], u = G.ub[j], qq = G.qq[j], pp = G.pp[j];
        double aty = 0.0;
        for (int k = P.colptr[j]; k < P.colptr[j + 1]; ++k)
            aty += sp_a_csc(Y, k, s) * L.yv[P.rowidx[k]];
        const double lam = qq + pp * x - aty;
        int c = 0;
        if (isfinite(l) && (x - l <= tol * (1.0 + fabs(l)) || x - l < lam)) c = 1;
        else if (isfinite(u) && (u - x <= tol * (1.0 + fabs(u)) || u - x < -lam)) c = 2;
        G.cc[j] = c;
        G.dx[j] = c == 1 ? l : (c == 2 ? u : x);
    }
    sp_rows(P, Y, s, L.xv, nullptr, [&](int i, double ax, double) {
        const double bl = G.bl[i], bu = G.bu[i], yv = L.yv[i];
        int r = 0;
        if (isfinite(bl) && (ax - bl <= tol * (1.0 + fabs(bl)) || ax - bl < yv)) r = 1;
        else if (isfinite(bu) && (bu - ax <= tol * (1.0 + fabs(bu)) || bu - ax < -yv)) r = 2;
        G.rc[i] = r;
        G.ds[i] = r ? -yv : 0.0;
    });
    SP_SYNC();
    for (int j = SP_TID; j < P.n; j += SP_NT) L.xv[j] = G.dx[j];
    for (int i = SP_TID; i < P.m; i += SP_NT) L.yv[i] = G.ds[i];
    SP_SYNC();
}

// Up to `rounds` active-set rounds from the codes in G.cc / G.rc and the point
// (xv, z in yv); returns the rounds used when the point passes the KKT
// certificate (polish_lane's, unscaled quantities, relative kkt_tol), else 0.
PHX_HD int sp_rounds(const Prob& P, const SpSym& Y, const SpScr& G, const SpLds& L, const Opts& O, int s,
                     int rounds, double qmax, int* refine_total) {
    const int n = P.n, m = P.m;
    const double reg = O.reg;
    const double dtol = O.kkt_tol * (1.0 + qmax);
    const double ptol = O.kkt_tol;
    SP_TP(0);
    for (int round = 0; round < rounds; ++round) {
        SP_CNT(14);
        for (int j = SP_TID; j < n; j += SP_NT) L.hv[j] = G.cc[j] == 0 ? 1.0 / (G.pp[j] + reg) : 0.0;
        for (int i = SP_TID; i < m; i += SP_NT) G.rdg[i] = G.rc[i] ? reg : -1.0;
        SP_SYNC();
        if (!sp_factor(P, Y, G, L, s)) return 0;
        // ---- iterative refinement on the unregularised KKT (proximal point) ----
        for (int it = 0; it < O.refine_steps; ++it) {
            // the column residual from the data on the first step only: after
            // a step it is reg dx exactly (phx_wg.h's refinement), written by
            // the update below, so this phase and its barrier go
            for (int j = SP_TID; j < (it == 0 ? n : 0); j += SP_NT) {
                const int cc = G.cc[j];
                const double qq = G.qq[j], pp = G.pp[j], xj = L.xv[j];
                if (cc) { G.r1[j] = 0.0; L.hv[j] = 0.0; continue; }
                double atz = 0.0;
                for (int k = P.colptr[j]; k < P.colptr[j + 1]; ++k)
                    atz += sp_a_csc(Y, k, s) * L.yv[P.rowidx[k]];
                const double r1 = -qq - pp * xj - atz;
                G.r1[j] = r1;
                L.hv[j] = r1 / (pp + reg);
            }
            if (it == 0) SP_SYNC();
            SP_TP(3);
            sp_rows(P, Y, s, L.xv, L.hv, [&](int i, double ax, double adr) {
                const int rc = G.rc[i];
                if (!rc) { L.tv[i] = 0.0; return; }
                const double b = rc == 1 ? G.bl[i] : G.bu[i];
                L.tv[i] = adr - (b - ax);
            });
            SP_SYNC();
            SP_TP(4);
            sp_msolve(P, Y, L);
            double mx[2] = {0.0, 0.0};   // max |correction|, max |value|
            for (int j = SP_TID; j < n; j += SP_NT) {
                const int cc = G.cc[j];
                const double r1 = G.r1[j], pp = G.pp[j], xj = L.xv[j];
                if (cc) continue;
                double atz = 0.0;
                for (int k = P.colptr[j]; k < P.colptr[j + 1]; ++k)
                    atz += sp_a_csc(Y, k, s) * L.tv[P.rowidx[k]];
                const double ih = 1.0 / (pp + reg);
                const double dx = (r1 - atz) * ih;
                const double x = xj + dx;
                L.xv[j] = x;
                // -q - P x' - A'z' = r1 - P dx - A'dz = reg dx
                const double rn = reg * dx;
                G.r1[j] = rn;
                L.hv[j] = rn * ih;
                mx[0] = fmax(mx[0], fabs(dx));
                mx[1] = fmax(mx[1], fabs(x));
            }
            for (int i = SP_TID; i < m; i += SP_NT) {
                const int rc = G.rc[i];
                const double dz = L.tv[i], yi = L.yv[i];
                if (!rc) continue;
                const double zn = yi + dz;
                L.yv[i] = zn;
                mx[0] = fmax(mx[0], fabs(dz));
                mx[1] = fmax(mx[1], fabs(zn));
            }
            sp_reduce<2>(mx, L.red, 1);
            if (SP_TID == 0 && refine_total) ++*refine_total;
            SP_SYNC();
            SP_TP(6);
            SP_CNT(12);
            if (mx[0] <= 1e-10 * (1.0 + mx[1])) break;
        }
        // ---- certificate; keeps the multipliers (r1) and row activities (ax) ----
        double bad[1] = {0.0};
        for (int j = SP_TID; j < n; j += SP_NT) {
            const double x = L.xv[j], l = G.lb[j], u = G.ub[j], dc = P.dc[j];
            const double qq = G.qq[j], pp = G.pp[j];
            const int c = G.cc[j];
            if (x < l && (l - x) * dc > ptol * (1.0 + fabs(l * dc))) bad[0] = 1.0;
            if (x > u && (x - u) * dc > ptol * (1.0 + fabs(u * dc))) bad[0] = 1.0;
            double atz = 0.0;
            for (int k = P.colptr[j]; k < P.colptr[j + 1]; ++k)
                atz += sp_a_csc(Y, k, s) * L.yv[P.rowidx[k]];
            const double lam = (qq + pp * x + atz) / dc;
            G.r1[j] = lam;
            if (!(lam - lam == 0.0)) bad[0] = 1.0;   // non-finite x or y: no comparison would fail
            if (c == 0) {
                if (fabs(lam) > dtol) bad[0] = 1.0;
            } else if (!(l == u)) {
                if (c == 1 && lam < -dtol) bad[0] = 1.0;
                if (c == 2 && lam > dtol) bad[0] = 1.0;
            }
        }
        sp_rows(P, Y, s, L.xv, nullptr, [&](int i, double ax, double) {
            G.ax[i] = ax;
            const double dr = P.dr[i], bl = G.bl[i], bu = G.bu[i];
            if (!(ax - ax == 0.0) || !(L.yv[i] - L.yv[i] == 0.0)) bad[0] = 1.0;
            if (ax < bl && (bl - ax) / dr > ptol * (1.0 + fabs(bl / dr))) bad[0] = 1.0;
            if (ax > bu && (ax - bu) / dr > ptol * (1.0 + fabs(bu / dr))) bad[0] = 1.0;
            if (G.rc[i] && !(bl == bu)) {
                const double y = -L.yv[i] * dr;
                if (G.rc[i] == 1 && y < -dtol) bad[0] = 1.0;
                if (G.rc[i] == 2 && y > dtol) bad[0] = 1.0;
            }
        });
        sp_reduce<1>(bad, L.red, 1);
        SP_TP(7);
        if (bad[0] == 0.0) return round + 1;
        if (round + 1 == rounds) break;
        SP_SYNC();
        // ---- primal-dual active-set update ----
        for (int j = SP_TID; j < n; j += SP_NT) {
            const double l = G.lb[j], u = G.ub[j];
            const double x = L.xv[j], lam = G.r1[j], dc = P.dc[j];
            const int c = G.cc[j];
            if (l == u) continue;
            if (c == 1 && lam < -dtol) G.cc[j] = 0;
            else if (c == 2 && lam > dtol) G.cc[j] = 0;
            else if (c == 0 && x < l && (l - x) * dc > ptol * (1.0 + fabs(l * dc))) { G.cc[j] = 1; L.xv[j] = l; }
            else if (c == 0 && x > u && (x - u) * dc > ptol * (1.0 + fabs(u * dc))) { G.cc[j] = 2; L.xv[j] = u; }
        }
        for (int i = SP_TID; i < m; i += SP_NT) {
            const double bl = G.bl[i], bu = G.bu[i];
            const double ax = G.ax[i], dr = P.dr[i], yi = L.yv[i];
            const int r = G.rc[i];
            if (bl == bu) continue;
            const double y = -yi * dr;
            if (r == 1 && y < -dtol) { G.rc[i] = 0; L.yv[i] = 0.0; }
            else if (r == 2 && y > dtol) { G.rc[i] = 0; L.yv[i] = 0.0; }
            else if (r == 0 && ax < bl && (bl - ax) / dr > ptol * (1.0 + fabs(bl / dr))) G.rc[i] = 1;
            else if (r == 0 && ax > bu && (ax - bu) / dr > ptol * (1.0 + fabs(bu / dr))) G.rc[i] = 2;
        }
        SP_SYNC();
        SP_TP(8);
    }
    return 0;
}

// Farkas test (phx_core.h farkas_lane) of the interior point's multipliers in
// L.yv: a failed IPM on an infeasible subproblem diverges along such a ray.
PHX_HD bool sp_farkas(const Prob& P, const SpSym& Y, const SpScr& G, const SpLds& L, int s) {
    double ym[1] = {0.0};
    for (int i = SP_TID; i < P.m; i += SP_NT) ym[0] = fmax(ym[0], fabs(L.yv[i]));
    sp_reduce<1>(ym, L.red, 1);
    if (!(ym[0] > 0.0) || !isfinite(ym[0])) return false;
    const double iy = -1.0 / ym[0];     // r = -y / |y|_inf (farkas_lane)
    Farkas F;
    for (int j = SP_TID; j < P.n; j += SP_NT) {
        double g = 0.0;
        for (int k = P.colptr[j]; k < P.colptr[j + 1]; ++k)
            g += sp_a_csc(Y, k, s) * L.yv[P.rowidx[k]] * iy;
        farkas_col(F, g, G.lb[j], G.ub[j]);
    }
    for (int i = SP_TID; i < P.m; i += SP_NT) farkas_row(F, L.yv[i] * iy, G.bl[i], G.bu[i]);
    double v[4] = {F.lo, F.hi, F.mag, F.ok ? 0.0 : 1.0};
    sp_reduce<3>(v, L.red, 0);
    double bad[1] = {v[3]};
    sp_reduce<1>(bad, L.red, 1);
    Farkas T;
    T.lo = v[0]; T.hi = v[1]; T.mag = v[2]; T.ok = bad[0] == 0.0;
    return farkas_margin_ok(T);
}

// Per-lane counters of one sp solve (for statistics; summed by the host).
struct SpCount {
    int warm_rounds, ipm_its, cold_rounds, refine;
};

// One scenario.  warm: start from the previous solution (St.xT / St.yT); a
// warm start that does not certify falls back to the interior point.  Returns
// > 0 (the active-set rounds + interior-point iterations used) when certified;
// the point is then in L.xv (x, scaled) and L.yv (z = -y, scaled);
// SP_INFEASIBLE when the failed interior point's multipliers prove the
// subproblem infeasible (sp_farkas); 0 otherwise.
constexpr int SP_INFEASIBLE = -1;
PHX_HD int sp_solve_one(const Prob& P, const State& St, const SpSym& Y, const SpScr& G, const SpLds& L,
                        const Opts& O, int s, bool warm, int warm_rounds, int cold_rounds, SpCount* cnt) {
    const int S = P.S;
    const double qmax = sp_load(P, G, L, s);
    if (warm) {
        for (int j = SP_TID; j < P.n; j += SP_NT) L.xv[j] = St.xT[ix(j, s, S)];
        for (int i = SP_TID; i < P.m; i += SP_NT) L.yv[i] = St.yT[ix(i, s, S)];
        SP_SYNC();
        sp_classify(P, Y, G, L, s, 1e-9);
        const int r = sp_rounds(P, Y, G, L, O, s, warm_rounds, qmax, cnt ? &cnt->refine : nullptr);
        if (cnt && SP_TID == 0) cnt->warm_rounds += r > 0 ? r : warm_rounds;
        if (r > 0) return r;
    }
    int its = 0;
    const double e = sp_ipm(P, Y, G, L, s, O.ipm_max_it, O.ipm_tol, 1e-10, &its);
    if (cnt && SP_TID == 0) cnt->ipm_its += its;
    if (!(e < 1e-4) && sp_farkas(P, Y, G, L, s)) return SP_INFEASIBLE;
    if (e < 1e-4) {
        const double tol = fmin(1e-4, fmax(1e-9, 10.0 * e));
        sp_classify(P, Y, G, L, s, tol);
        const int r = sp_rounds(P, Y, G, L, O, s, cold_rounds, qmax, cnt ? &cnt->refine : nullptr);
        if (cnt && SP_TID == 0) cnt->cold_rounds += r > 0 ? r : cold_rounds;
        if (r > 0) return r + its;
    }
    return 0;
}

// A certified lane: outputs as finalize_lane writes them (unscaled x, row
// duals y = -z, objective incl. PH terms) and the point as the next warm start.
PHX_HD void sp_write_out(const Prob& P, const State& St, const SpLds& L, const double* c_unscaled_p, int64_t c_si,
                         int64_t c_ss, int s, double* x_out, double* y_out, double* obj_out) {
    const int S = P.S;
    double f[1] = {0.0};
    for (int j = SP_TID; j < P.n; j += SP_NT) {
        const int64_t o = ix(j, s, S);
        const double xs = L.xv[j];
        St.xT[o] = xs; St.x[o] = xs; St.x0[o] = xs;
        const double x = xs * P.dc[j];
        x_out[o] = x;
        f[0] += c_unscaled_p[(int64_t)j * c_si + (int64_t)s * c_ss] * x;
        const int sl = P.col_slot[j];
        if (sl >= 0) f[0] += P.qN[ix(sl, s, S)] * x + 0.5 * P.pN[ix(sl, s, S)] * x * x;
    }
    for (int i = SP_TID; i < P.m; i += SP_NT) {
        const int64_t o = ix(i, s, S);
        const double ys = -L.yv[i];
        St.yT[o] = ys; St.y[o] = ys; St.y0[o] = ys;
        if (y_out) y_out[o] = ys * P.dr[i];
    }
    sp_reduce<1>(f, L.red, 0);
    if (SP_TID == 0) obj_out[s] = P.kN[s] + f[0];
}

}  // namespace phx
