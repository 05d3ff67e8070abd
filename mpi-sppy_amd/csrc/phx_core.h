// phx_core.h — per-scenario ("lane") math of the batched PH subproblem solver.
//
// One lane = one scenario.  Every per-scenario array is scenario-minor
// ([i*S + s]), so the 64 lanes of a wavefront touch 64 consecutive doubles of
// one row/column: fully coalesced 512-B accesses, while the shared sparsity
// pattern (rowptr/colidx/...) is wave-uniform and rides the scalar cache.
//
// These functions are pure arithmetic on pointers.  The HIP kernels in
// phx_kernels.hip call them with s = global thread index; the same header is
// compiled for the host by tests/emu (test infrastructure only) so the math
// can be checked against the CPU oracle without a GPU.
//
// Reference semantics being replaced: SPOpt.solve_one (mpisppy/spopt.py:85-223)
// solves one scenario's LP/QP with an external solver.  Here: restarted,
// reflected Halpern PDHG on the Ruiz/Pock-Chambolle scaled problem,
// followed by an active-set KKT polish that certifies exact optimality.
#pragma once
#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#define PHX_HD __host__ __device__ __forceinline__
#else
#define PHX_HD inline
#endif

namespace phx {

#if defined(__HIP_DEVICE_COMPILE__)
// Cross-lane reductions of one wavefront by DPP moves (VALU, a few cycles each)
// instead of __shfl_xor's ds_bpermute (an LDS round trip per step and 32-bit
// half).  OP 0: sum, 1: max, 2: min.  The butterfly's pairing is kept (quad_perm
// [1,0,3,2] = xor 1, [2,3,0,1] = xor 2; on values equal within each quad,
// row_half_mirror = xor 4 and row_mirror = xor 8), so the results are the
// same bits as the __shfl_xor butterflies they replace.
template <int OP, int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_op(double v) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(u & 0xffffffffull), CTRL, ROWMASK, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, ROWMASK, 0xf, false);
    const double w = __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
    return OP == 0 ? v + w : (OP == 1 ? fmax(v, w) : fmin(v, w));
}
// over a quad (four adjacent lanes; all four end with it)
template <int OP>
__device__ __forceinline__ double quad_reduce(double v) {
    v = dpp_op<OP, 0xB1, 0xf>(v);
    return dpp_op<OP, 0x4E, 0xf>(v);
}
// over the wavefront (every lane active): rows by mirrors, then the row
// broadcasts of lanes 15 and 31 leave the total in lane 63, read back
// uniformly (readlane is 32-bit: both halves)
template <int OP>
__device__ __forceinline__ double wave_reduce(double v) {
    v = quad_reduce<OP>(v);
    v = dpp_op<OP, 0x141, 0xf>(v);    // row_half_mirror
    v = dpp_op<OP, 0x140, 0xf>(v);    // row_mirror
    v = dpp_op<OP, 0x142, 0xa>(v);    // row_bcast:15 into rows 1, 3
    v = dpp_op<OP, 0x143, 0xc>(v);    // row_bcast:31 into rows 2, 3
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u & 0xffffffffull), 63);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), 63);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
#endif

// INFEASIBLE: a Farkas certificate proves the subproblem's feasible set empty
// (the reference's infeasible termination, spopt.py:175-194: scenario_feasible
// = False); ITER_LIMIT / NUMERIC_FAIL are solve failures, not infeasibility.
enum Status : int32_t { RUNNING = 0, OPTIMAL = 1, ITER_LIMIT = 2, NUMERIC_FAIL = 3, INFEASIBLE = 4 };

// Farkas test for row weights r: with g = A'r,
//   min over the column box of g'x  >  max over the row box of r's
// proves {bl <= A x <= bu, l <= x <= u} empty (every feasible x gives
// r'A x = r's).  An infeasible problem's interior-point multipliers y
// (y > 0: lower side, the dual ray of the infeasibility) diverge along such
// a ray with r = -y, so the failed IPM's -y (normalised) is the candidate.
// Components below 1e-9 of the largest are taken as zero (an exact ray has
// zeros there; an infinite bound with a nonzero coefficient voids the test).
// Accumulate with farkas_col / farkas_row, decide with farkas_margin_ok.
struct Farkas {
    double lo = 0.0, hi = 0.0, mag = 0.0;
    bool ok = true;
};
PHX_HD void farkas_col(Farkas& F, double g, double l, double u) {
    if (fabs(g) <= 1e-9) return;
    const double b = g > 0.0 ? l : u;
    if (!isfinite(b)) { F.ok = false; return; }
    F.lo += g * b;
    F.mag += fabs(g * b);
}
PHX_HD void farkas_row(Farkas& F, double y, double bl, double bu) {
    if (fabs(y) <= 1e-9) return;
    const double b = y > 0.0 ? bu : bl;
    if (!isfinite(b)) { F.ok = false; return; }
    F.hi += y * b;
    F.mag += fabs(y * b);
}
PHX_HD bool farkas_margin_ok(const Farkas& F) { return F.ok && F.lo - F.hi > 1e-7 * (1.0 + F.mag); }



// strided scenario vector: element i of scenario s at p[i*si + s*ss]
struct SVec {
    const double* p;
    int64_t si, ss;
    PHX_HD double at(int i, int s) const { return p[(int64_t)i * si + (int64_t)s * ss]; }
};

// Scaled problem (device pointers), passed by value to kernels.
struct Prob {
    int32_t S, n, m, nnz, N;
    const int32_t* rowptr;   // [m+1]
    const int32_t* colidx;   // [nnz]
    const int32_t* colptr;   // [n+1]  CSC view
    const int32_t* rowidx;   // [nnz]
    const int32_t* csc2csr;  // [nnz]
    const int32_t* kvar;     // [nnz]
    const double* Ac;        // [nnz]  scaled invariant values
    const double* Av;        // [nvar*S] scaled varying values
    SVec c, lb, ub, bl, bu;  // scaled
    const double* dr;        // [m] row scaling
    const double* dc;        // [n] column scaling
    const int32_t* col_slot; // [n] slot of a nonant column, else -1
    const int32_t* slot_col; // [N]
    const double* qN;        // [N*S] unscaled PH linear term
    const double* pN;        // [N*S] unscaled PH diagonal quadratic
    const double* kN;        // [S]   PH constant
};

struct State {
    double *x, *y, *x0, *y0, *xT, *yT, *xb;  // scaled iterates [n|m][S]
    double *omega, *eta, *r0, *rprev, *err;  // [S]
    int32_t *hk, *status, *iters;            // [S]
    int32_t *flags;                          // [S] bit0: interior-point finisher tried
};

struct Opts {
    int32_t iters;        // PDHG iterations in this chunk
    int32_t restart_max;  // artificial restart length
    double polish_below;
    double opt_tol;
    double kkt_tol;
    double reg;
    int32_t refine_steps;
    int32_t polish;
    int32_t max_iters;
    int32_t ipm_after;    // PDHG iterations before a lane switches to the IPM finisher (<0: never)
    int32_t ipm_max_it;
    double ipm_tol;
};

struct Polish {   // polish workspace, all [.][S]
    double* L;    // packed lower-triangular Schur factor [m(m+1)/2][S]
    double* z;    // [m]  row multipliers (z = -y)
    double* r1;   // [n]
    double* t;    // [m]
    double* xp;   // [n]  polished x (scaled)
    double* xfix; // [n]  bound value of bound-active columns
    double* brhs; // [m]  active row right-hand side
    unsigned char* F;  // [n] 1 = free column
    unsigned char* R;  // [m] 1 = active row
};

struct Ipm {      // interior-point finisher workspace, all [.][S]
    double *s, *zl, *zu, *wl, *wu;            // row activity, bound multipliers
    double *dx, *dzl, *dzu, *cl, *cu, *hx;    // [n]
    double *ds, *dwl, *dwu, *dy, *cwl, *cwu;  // [m]
};

PHX_HD int64_t ix(int i, int s, int S) { return (int64_t)i * S + s; }

PHX_HD double aval(const Prob& P, int k, int s) {
    const int v = P.kvar[k];
    return v < 0 ? P.Ac[k] : P.Av[(int64_t)v * P.S + s];
}

PHX_HD double clampd(double v, double lo, double hi) { return fmin(fmax(v, lo), hi); }

// Farkas test of lane s's multipliers y ([m][S], scaled problem).
PHX_HD bool farkas_lane(const Prob& P, const double* y, int s) {
    const int S = P.S;
    double ym = 0.0;
    for (int i = 0; i < P.m; ++i) ym = fmax(ym, fabs(y[(int64_t)i * S + s]));
    if (!(ym > 0.0) || !isfinite(ym)) return false;
    const double iy = -1.0 / ym;        // r = -y / |y|_inf
    Farkas F;
    for (int j = 0; j < P.n; ++j) {
        double g = 0.0;
        for (int k = P.colptr[j]; k < P.colptr[j + 1]; ++k) {
            const int kk = P.csc2csr[k];
            const int v = P.kvar[kk];
            g += (v < 0 ? P.Ac[kk] : P.Av[(int64_t)v * S + s]) * y[(int64_t)P.rowidx[k] * S + s] * iy;
        }
        farkas_col(F, g, P.lb.at(j, s), P.ub.at(j, s));
    }
    for (int i = 0; i < P.m; ++i) farkas_row(F, y[(int64_t)i * S + s] * iy, P.bl.at(i, s), P.bu.at(i, s));
    return farkas_margin_ok(F);
}

// effective scaled linear cost and diagonal quadratic of column j
PHX_HD void col_cost(const Prob& P, int j, int s, double& q, double& p) {
    q = P.c.at(j, s);
    p = 0.0;
    const int sl = P.col_slot[j];
    if (sl >= 0) {
        const double d = P.dc[j];
        q += d * P.qN[ix(sl, s, P.S)];
        p = d * d * P.pN[ix(sl, s, P.S)];
    }
}

// ---------------------------------------------------------------------------
// One PDHG operator application T(z) followed by the reflected Halpern step
//   z+ = a*((1+g)T(z) - g z) + (1-a) z0,  a = (k+1)/(k+2), g = 1
// primal: xT = proj_[l,u]((x - tau(q - A'y)) / (1 + tau p)),  xb = 2xT - x
// dual:   t = A xb - y/sigma,  yT = sigma (proj_[bl,bu](t) - t)
// On the last iteration of a chunk (want_res) the fixed-point residual
// ||z - T(z)||^2 parts are returned in dx2/dy2.
// ---------------------------------------------------------------------------
PHX_HD void pdhg_iter(const Prob& P, const State& St, int s, int hk,
                      double tau, double sigma, bool want_res,
                      double& dx2, double& dy2) {
    const int S = P.S;
    const double a = (double)(hk + 1) / (double)(hk + 2);
    const double b = 1.0 - a;
    dx2 = 0.0;
    dy2 = 0.0;
    for (int j = 0; j < P.n; ++j) {
        double aty = 0.0;
        for (int k = P.colptr[j]; k < P.colptr[j + 1]; ++k) {
            const int kk = P.csc2csr[k];
            aty += aval(P, kk, s) * St.y[ix(P.rowidx[k], s, S)];
        }
        double q, p;
        col_cost(P, j, s, q, p);
        const int64_t o = ix(j, s, S);
        const double xo = St.x[o];
        double xt = (xo - tau * (q - aty)) / (1.0 + tau * p);
        xt = clampd(xt, P.lb.at(j, s), P.ub.at(j, s));
        St.xT[o] = xt;
        St.xb[o] = 2.0 * xt - xo;
        St.x[o] = a * (2.0 * xt - xo) + b * St.x0[o];
        if (want_res) dx2 += (xt - xo) * (xt - xo);
    }
    for (int i = 0; i < P.m; ++i) {
        double ax = 0.0;
        for (int k = P.rowptr[i]; k < P.rowptr[i + 1]; ++k)
            ax += aval(P, k, s) * St.xb[ix(P.colidx[k], s, S)];
        const int64_t o = ix(i, s, S);
        const double yo = St.y[o];
        const double t = ax - yo / sigma;
        const double yt = sigma * (clampd(t, P.bl.at(i, s), P.bu.at(i, s)) - t);
        St.yT[o] = yt;
        St.y[o] = a * (2.0 * yt - yo) + b * St.y0[o];
        if (want_res) dy2 += (yt - yo) * (yt - yo);
    }
}

// Relative KKT error of the scaled point (xs, ys), measured in the unscaled
// problem (PDLP-style: max of primal residual, dual residual, duality gap).
PHX_HD double kkt_error(const Prob& P, const double* xs, const double* ys, int s) {
    const int S = P.S;
    double rp2 = 0.0, bn2 = 0.0, rd2 = 0.0, qn2 = 0.0;
    double pobj = 0.0, dobj = 0.0;
    for (int i = 0; i < P.m; ++i) {
        double ax = 0.0;
        for (int k = P.rowptr[i]; k < P.rowptr[i + 1]; ++k)
            ax += aval(P, k, s) * xs[ix(P.colidx[k], s, S)];
        const double dr = P.dr[i];
        const double bl = P.bl.at(i, s), bu = P.bu.at(i, s);
        const double axu = ax / dr;
        const double r = axu - clampd(axu, bl / dr, bu / dr);
        rp2 += r * r;
        if (isfinite(bl)) bn2 += (bl / dr) * (bl / dr);
        if (isfinite(bu)) bn2 += (bu / dr) * (bu / dr);
        const double y = ys[ix(i, s, S)];
        if (y > 0.0 && isfinite(bl)) dobj += bl * y;
        else if (y < 0.0 && isfinite(bu)) dobj += bu * y;
    }
    for (int j = 0; j < P.n; ++j) {
        double aty = 0.0;
        for (int k = P.colptr[j]; k < P.colptr[j + 1]; ++k)
            aty += aval(P, P.csc2csr[k], s) * ys[ix(P.rowidx[k], s, S)];
        double q, p;
        col_cost(P, j, s, q, p);
        const double x = xs[ix(j, s, S)];
        const double lam_s = q + p * x - aty;   // scaled reduced cost
        const double dc = P.dc[j];
        const double lam = lam_s / dc;
        const double l = P.lb.at(j, s), u = P.ub.at(j, s);
        double rd = lam;
        if (isfinite(l) && lam > 0.0) { rd = 0.0; dobj += l * lam_s; }
        if (isfinite(u) && lam < 0.0) { rd = 0.0; dobj += u * lam_s; }
        rd2 += rd * rd;
        qn2 += (q / dc) * (q / dc);
        pobj += q * x + 0.5 * p * x * x;
        dobj -= 0.5 * p * x * x;
    }
    const double ep = sqrt(rp2) / (1.0 + sqrt(bn2));
    const double ed = sqrt(rd2) / (1.0 + sqrt(qn2));
    const double eg = fabs(pobj - dobj) / (1.0 + fabs(pobj) + fabs(dobj));
    // (fmax drops a NaN operand: the sum of the terms catches a non-finite one)
    const double e = fmax(ep, fmax(ed, eg));
    return isfinite(ep + ed + eg) && isfinite(e) ? e : 1e300;
}

// Restart / primal-weight logic after a chunk; sets St.err[s].
PHX_HD void check_and_restart(const Prob& P, const State& St, const Opts& O, int s,
                              double dx2, double dy2) {
    const int S = P.S;
    const double w = St.omega[s];
    const double r = sqrt(w * dx2 + dy2 / w);
    const double r0 = St.r0[s];
    const double rprev = St.rprev[s];
    const bool first = !(r0 < 1e300);
    bool restart = first || (r <= 0.2 * r0) || (r <= 0.8 * r0 && r > rprev) ||
                   (St.hk[s] >= O.restart_max);
    St.rprev[s] = r;
    if (restart) {
        double ddx = 0.0, ddy = 0.0;
        for (int j = 0; j < P.n; ++j) {
            const double d = St.xT[ix(j, s, S)] - St.x0[ix(j, s, S)];
            ddx += d * d;
        }
        for (int i = 0; i < P.m; ++i) {
            const double d = St.yT[ix(i, s, S)] - St.y0[ix(i, s, S)];
            ddy += d * d;
        }
        ddx = sqrt(ddx);
        ddy = sqrt(ddy);
        if (!first && ddx > 1e-10 && ddy > 1e-10) {
            const double nw = exp(0.5 * log(ddy / ddx) + 0.5 * log(w));
            if (isfinite(nw) && nw > 1e-8 && nw < 1e8) St.omega[s] = nw;
        }
        for (int j = 0; j < P.n; ++j) {
            const int64_t o = ix(j, s, S);
            St.x[o] = St.x0[o] = St.xT[o];
        }
        for (int i = 0; i < P.m; ++i) {
            const int64_t o = ix(i, s, S);
            St.y[o] = St.y0[o] = St.yT[o];
        }
        St.hk[s] = 0;
        St.r0[s] = r;
    }
    St.err[s] = kkt_error(P, St.xT, St.yT, s);
}

// ---------------------------------------------------------------------------
// Active-set KKT polish.  Given the PDHG point (xT, yT) classify bounds and
// rows as active with a relative tolerance, eliminate bound-active columns and
// solve the equality-constrained KKT system
//      [ P_FF   A_RF' ] [x_F]   [ -q_F        ]
//      [ A_RF   0     ] [ z ] = [ b_R - A_RB x_B ]     (z = -y_R)
// by its quasi-definite regularisation (P+reg, -reg) + iterative refinement,
// seeded with the PDHG point (a proximal-point iteration that converges to
// the KKT solution nearest the sign-consistent PDHG duals — this is what makes
// degenerate vertices certify).  The Schur complement
//      Sm = A_RF (P_FF+reg)^-1 A_RF' + reg I   (identity on inactive rows)
// is factored in place (packed, scenario-minor, uniform loops over all m rows).
// Returns true iff the polished point passes the KKT certificate.
// ---------------------------------------------------------------------------
PHX_HD int64_t tri(int i, int k) { return (int64_t)i * (i + 1) / 2 + k; }   // i >= k

PHX_HD bool polish_lane(const Prob& P, const State& St, const Polish& W, const Opts& O,
                        int s, double tol) {
    const int S = P.S, n = P.n, m = P.m;
    const double reg = O.reg;
    // ---- classify ----
    // A bound/row is active when its slack is within tol (relative), or when
    // its slack is smaller than its correctly-signed multiplier (OSQP's
    // polish rule, sharp at interior-point points by strict complementarity).
    for (int j = 0; j < n; ++j) {
        const int64_t o = ix(j, s, S);
        const double x = St.xT[o];
        const double l = P.lb.at(j, s), u = P.ub.at(j, s);
        double aty = 0.0;
        for (int k = P.colptr[j]; k < P.colptr[j + 1]; ++k)
            aty += aval(P, P.csc2csr[k], s) * St.yT[ix(P.rowidx[k], s, S)];
        double q, p;
        col_cost(P, j, s, q, p);
        const double lam = q + p * x - aty;
        unsigned char f = 1;
        double xf = 0.0;
        if (isfinite(l) && (x - l <= tol * (1.0 + fabs(l)) || x - l < lam)) { f = 0; xf = l; }
        else if (isfinite(u) && (u - x <= tol * (1.0 + fabs(u)) || u - x < -lam)) { f = 0; xf = u; }
        W.F[o] = f;
        W.xfix[o] = xf;
        W.xp[o] = f ? x : xf;
    }
    for (int i = 0; i < m; ++i) {
        double ax = 0.0;
        for (int k = P.rowptr[i]; k < P.rowptr[i + 1]; ++k)
            ax += aval(P, k, s) * St.xT[ix(P.colidx[k], s, S)];
        const double bl = P.bl.at(i, s), bu = P.bu.at(i, s);
        const int64_t o = ix(i, s, S);
        unsigned char r = 0;
        double b = 0.0;
        const double yv = St.yT[o];
        if (isfinite(bl) && (ax - bl <= tol * (1.0 + fabs(bl)) || ax - bl < yv)) { r = 1; b = bl; }
        else if (isfinite(bu) && (bu - ax <= tol * (1.0 + fabs(bu)) || bu - ax < -yv)) { r = 1; b = bu; }
        W.R[o] = r;
        W.brhs[o] = b;
        W.z[o] = r ? -St.yT[o] : 0.0;
    }
    // ---- Schur complement (packed lower) ----
    for (int i = 0; i < m; ++i)
        for (int k = 0; k <= i; ++k)
            W.L[ix((int)tri(i, k), s, S)] = (i == k) ? (W.R[ix(i, s, S)] ? reg : 1.0) : 0.0;
    for (int j = 0; j < n; ++j) {
        if (!W.F[ix(j, s, S)]) continue;
        double q, p;
        col_cost(P, j, s, q, p);
        const double D = 1.0 / (p + reg);
        for (int ka = P.colptr[j]; ka < P.colptr[j + 1]; ++ka) {
            const int ia = P.rowidx[ka];
            if (!W.R[ix(ia, s, S)]) continue;
            const double va = aval(P, P.csc2csr[ka], s) * D;
            for (int kb = P.colptr[j]; kb <= ka; ++kb) {
                const int ib = P.rowidx[kb];
                if (!W.R[ix(ib, s, S)]) continue;
                const double vb = aval(P, P.csc2csr[kb], s);
                const int hi = ia > ib ? ia : ib, lo = ia > ib ? ib : ia;
                W.L[ix((int)tri(hi, lo), s, S)] += va * vb;
            }
        }
    }
    // ---- Cholesky (in place, packed lower) ----
    for (int jj = 0; jj < m; ++jj) {
        double d = W.L[ix((int)tri(jj, jj), s, S)];
        for (int k = 0; k < jj; ++k) {
            const double v = W.L[ix((int)tri(jj, k), s, S)];
            d -= v * v;
        }
        if (!(d > 0.0)) return false;
        d = sqrt(d);
        W.L[ix((int)tri(jj, jj), s, S)] = d;
        for (int i = jj + 1; i < m; ++i) {
            double v = W.L[ix((int)tri(i, jj), s, S)];
            for (int k = 0; k < jj; ++k)
                v -= W.L[ix((int)tri(i, k), s, S)] * W.L[ix((int)tri(jj, k), s, S)];
            W.L[ix((int)tri(i, jj), s, S)] = v / d;
        }
    }
    // ---- iterative refinement on the unregularised KKT ----
    for (int it = 0; it < O.refine_steps; ++it) {
        // r1 = -q - p x - A' z   (free columns)
        for (int j = 0; j < n; ++j) {
            const int64_t o = ix(j, s, S);
            if (!W.F[o]) { W.r1[o] = 0.0; continue; }
            double atz = 0.0;
            for (int k = P.colptr[j]; k < P.colptr[j + 1]; ++k)
                atz += aval(P, P.csc2csr[k], s) * W.z[ix(P.rowidx[k], s, S)];
            double q, p;
            col_cost(P, j, s, q, p);
            W.r1[o] = -q - p * W.xp[o] - atz;
        }
        // t = A_RF D r1 - r2,  r2 = b - A x   (active rows)
        for (int i = 0; i < m; ++i) {
            const int64_t o = ix(i, s, S);
            if (!W.R[o]) { W.t[o] = 0.0; continue; }
            double adr = 0.0, ax = 0.0;
            for (int k = P.rowptr[i]; k < P.rowptr[i + 1]; ++k) {
                const int j = P.colidx[k];
                const int64_t oj = ix(j, s, S);
                const double a = aval(P, k, s);
                ax += a * W.xp[oj];
                if (W.F[oj]) {
                    double q, p;
                    col_cost(P, j, s, q, p);
                    adr += a * W.r1[oj] / (p + reg);
                }
            }
            W.t[o] = adr - (W.brhs[o] - ax);
        }
        // solve L L' dz = t  (forward then backward, packed)
        for (int i = 0; i < m; ++i) {
            double v = W.t[ix(i, s, S)];
            for (int k = 0; k < i; ++k) v -= W.L[ix((int)tri(i, k), s, S)] * W.t[ix(k, s, S)];
            W.t[ix(i, s, S)] = v / W.L[ix((int)tri(i, i), s, S)];
        }
        for (int i = m - 1; i >= 0; --i) {
            double v = W.t[ix(i, s, S)];
            for (int k = i + 1; k < m; ++k) v -= W.L[ix((int)tri(k, i), s, S)] * W.t[ix(k, s, S)];
            W.t[ix(i, s, S)] = v / W.L[ix((int)tri(i, i), s, S)];
        }
        // dx = D (r1 - A' dz);  x += dx; z += dz
        for (int j = 0; j < n; ++j) {
            const int64_t o = ix(j, s, S);
            if (!W.F[o]) continue;
            double atz = 0.0;
            for (int k = P.colptr[j]; k < P.colptr[j + 1]; ++k)
                atz += aval(P, P.csc2csr[k], s) * W.t[ix(P.rowidx[k], s, S)];
            double q, p;
            col_cost(P, j, s, q, p);
            W.xp[o] += (W.r1[o] - atz) / (p + reg);
        }
        for (int i = 0; i < m; ++i) {
            const int64_t o = ix(i, s, S);
            if (W.R[o]) W.z[o] += W.t[o];
        }
    }
    // ---- certificate (unscaled quantities) ----
    double qmax = 0.0;
    for (int j = 0; j < n; ++j) {
        double q, p;
        col_cost(P, j, s, q, p);
        qmax = fmax(qmax, fabs(q / P.dc[j]));
    }
    const double dtol = O.kkt_tol * (1.0 + qmax);
    const double ptol = O.kkt_tol;
    for (int j = 0; j < n; ++j) {
        const int64_t o = ix(j, s, S);
        const double x = W.xp[o];
        const double l = P.lb.at(j, s), u = P.ub.at(j, s);
        const double dc = P.dc[j];
        if (x < l && (l - x) * dc > ptol * (1.0 + fabs(l * dc))) return false;
        if (x > u && (x - u) * dc > ptol * (1.0 + fabs(u * dc))) return false;
        double atz = 0.0;
        for (int k = P.colptr[j]; k < P.colptr[j + 1]; ++k)
            atz += aval(P, P.csc2csr[k], s) * W.z[ix(P.rowidx[k], s, S)];
        double q, p;
        col_cost(P, j, s, q, p);
        const double lam = (q + p * x + atz) / dc;   // y = -z
        if (!(lam - lam == 0.0)) return false;       // non-finite x or z: no comparison would fail
        if (W.F[o]) {
            if (fabs(lam) > dtol) return false;
        } else if (!(l == u)) {
            const bool atl = (W.xfix[o] == l);
            if (atl && lam < -dtol) return false;
            if (!atl && lam > dtol) return false;
        }
    }
    for (int i = 0; i < m; ++i) {
        const int64_t o = ix(i, s, S);
        double ax = 0.0;
        for (int k = P.rowptr[i]; k < P.rowptr[i + 1]; ++k)
            ax += aval(P, k, s) * W.xp[ix(P.colidx[k], s, S)];
        const double dr = P.dr[i];
        const double bl = P.bl.at(i, s), bu = P.bu.at(i, s);
        if (!(ax - ax == 0.0) || !(W.z[o] - W.z[o] == 0.0)) return false;
        if (ax < bl && (bl - ax) / dr > ptol * (1.0 + fabs(bl / dr))) return false;
        if (ax > bu && (ax - bu) / dr > ptol * (1.0 + fabs(bu / dr))) return false;
        if (W.R[o] && !(bl == bu)) {
            const double y = -W.z[o] * dr;
            const bool atl = (W.brhs[o] == bl);
            if (atl && y < -dtol) return false;
            if (!atl && y > dtol) return false;
        }
    }
    return true;
}

// ---------------------------------------------------------------------------
// Interior-point finisher (Mehrotra predictor-corrector), one lane per
// scenario, for lanes PDHG has not certified.  Problem (scaled space):
//   min 0.5 x'Px + q'x  s.t.  A x - s = 0,  l <= x <= u,  bl <= s <= bu
// with bound multipliers z_l, z_u (columns) and w_l, w_u (rows); equality rows
// carry no slack, free rows keep y = 0.  Newton systems reduce to the m x m
// normal matrix  M = A (P + Sigma_x)^-1 A' + Sigma_s^-1,  factored in place with
// the same packed, scenario-minor Cholesky as the polish.  The iterate lands
// in St.xT / St.yT (y > 0 <=> lower side active, the PDHG convention) so the
// polish certifies it.  Returns the final relative KKT error.
// ---------------------------------------------------------------------------
PHX_HD bool ipm_fixed(double l, double u) { return l == u; }

PHX_HD double ipm_mu(const Prob& P, const State& St, const Ipm& I, int s, int& ncomp) {
    const int S = P.S;
    double acc = 0.0;
    ncomp = 0;
    for (int j = 0; j < P.n; ++j) {
        const int64_t o = ix(j, s, S);
        const double l = P.lb.at(j, s), u = P.ub.at(j, s), x = St.xT[o];
        if (ipm_fixed(l, u)) continue;
        if (isfinite(l)) { acc += (x - l) * I.zl[o]; ++ncomp; }
        if (isfinite(u)) { acc += (u - x) * I.zu[o]; ++ncomp; }
    }
    for (int i = 0; i < P.m; ++i) {
        const int64_t o = ix(i, s, S);
        const double bl = P.bl.at(i, s), bu = P.bu.at(i, s), sv = I.s[o];
        if (bl == bu) continue;
        if (isfinite(bl)) { acc += (sv - bl) * I.wl[o]; ++ncomp; }
        if (isfinite(bu)) { acc += (bu - sv) * I.wu[o]; ++ncomp; }
    }
    return ncomp ? acc / ncomp : 0.0;
}

// Solve the Newton system for given complementarity targets (cl, cu, cwl, cwu
// already in I); M must hold the Cholesky factor.  Writes the direction.
PHX_HD void ipm_direction(const Prob& P, const State& St, const Polish& W, const Ipm& I, int s) {
    const int S = P.S, n = P.n, m = P.m;
    // rho_x -> I.dx (temporarily), rho_s -> I.ds (temporarily)
    for (int j = 0; j < n; ++j) {
        const int64_t o = ix(j, s, S);
        const double l = P.lb.at(j, s), u = P.ub.at(j, s), x = St.xT[o];
        if (ipm_fixed(l, u)) { I.dx[o] = 0.0; continue; }
        double aty = 0.0;
        for (int k = P.colptr[j]; k < P.colptr[j + 1]; ++k)
            aty += aval(P, P.csc2csr[k], s) * St.yT[ix(P.rowidx[k], s, S)];
        double q, p;
        col_cost(P, j, s, q, p);
        double rd = p * x + q - aty;
        double rho = 0.0;
        if (isfinite(l)) { rd -= I.zl[o]; rho += I.cl[o] / (x - l); }
        if (isfinite(u)) { rd += I.zu[o]; rho -= I.cu[o] / (u - x); }
        I.dx[o] = rho - rd;
    }
    for (int i = 0; i < m; ++i) {
        const int64_t o = ix(i, s, S);
        const double bl = P.bl.at(i, s), bu = P.bu.at(i, s);
        double ax = 0.0;
        for (int k = P.rowptr[i]; k < P.rowptr[i + 1]; ++k)
            ax += aval(P, k, s) * St.xT[ix(P.colidx[k], s, S)];
        double adr = 0.0;   // (A H^-1 rho_x)_i
        for (int k = P.rowptr[i]; k < P.rowptr[i + 1]; ++k) {
            const int64_t oj = ix(P.colidx[k], s, S);
            adr += aval(P, k, s) * I.dx[oj] / I.hx[oj];
        }
        double rhs;
        if (!isfinite(bl) && !isfinite(bu)) {
            rhs = 0.0;                      // free row: y stays 0
            I.ds[o] = 0.0;
        } else if (bl == bu) {
            rhs = -(ax - bl) - adr;
            I.ds[o] = 0.0;
        } else {
            const double sv = I.s[o];
            const double y = St.yT[o];
            double rs = y, rhos = 0.0, sig = 0.0;
            if (isfinite(bl)) { rs -= I.wl[o]; rhos += I.cwl[o] / (sv - bl); sig += I.wl[o] / (sv - bl); }
            if (isfinite(bu)) { rs += I.wu[o]; rhos -= I.cwu[o] / (bu - sv); sig += I.wu[o] / (bu - sv); }
            rhos -= rs;
            I.ds[o] = rhos;                 // rho_s kept for the back-substitution
            rhs = -(ax - sv) + rhos / sig - adr;
        }
        W.t[o] = rhs;
    }
    // dy = M^-1 rhs
    for (int i = 0; i < m; ++i) {
        double v = W.t[ix(i, s, S)];
        for (int k = 0; k < i; ++k) v -= W.L[ix((int)tri(i, k), s, S)] * W.t[ix(k, s, S)];
        W.t[ix(i, s, S)] = v / W.L[ix((int)tri(i, i), s, S)];
    }
    for (int i = m - 1; i >= 0; --i) {
        double v = W.t[ix(i, s, S)];
        for (int k = i + 1; k < m; ++k) v -= W.L[ix((int)tri(k, i), s, S)] * W.t[ix(k, s, S)];
        W.t[ix(i, s, S)] = v / W.L[ix((int)tri(i, i), s, S)];
    }
    for (int i = 0; i < m; ++i) {
        const int64_t o = ix(i, s, S);
        const double bl = P.bl.at(i, s), bu = P.bu.at(i, s);
        const double dy = W.t[o];
        I.dy[o] = dy;
        if (isfinite(bl) && isfinite(bu) && bl == bu) continue;
        if (!isfinite(bl) && !isfinite(bu)) continue;
        const double sv = I.s[o];
        double sig = 0.0;
        if (isfinite(bl)) sig += I.wl[o] / (sv - bl);
        if (isfinite(bu)) sig += I.wu[o] / (bu - sv);
        const double dsv = (I.ds[o] - dy) / sig;
        I.ds[o] = dsv;
        if (isfinite(bl)) I.dwl[o] = (I.cwl[o] - I.wl[o] * dsv) / (sv - bl);
        if (isfinite(bu)) I.dwu[o] = (I.cwu[o] + I.wu[o] * dsv) / (bu - sv);
    }
    for (int j = 0; j < n; ++j) {
        const int64_t o = ix(j, s, S);
        const double l = P.lb.at(j, s), u = P.ub.at(j, s), x = St.xT[o];
        if (ipm_fixed(l, u)) { I.dx[o] = 0.0; continue; }
        double atdy = 0.0;
        for (int k = P.colptr[j]; k < P.colptr[j + 1]; ++k)
            atdy += aval(P, P.csc2csr[k], s) * I.dy[ix(P.rowidx[k], s, S)];
        const double dxv = (I.dx[o] + atdy) / I.hx[o];
        I.dx[o] = dxv;
        if (isfinite(l)) I.dzl[o] = (I.cl[o] - I.zl[o] * dxv) / (x - l);
        if (isfinite(u)) I.dzu[o] = (I.cu[o] + I.zu[o] * dxv) / (u - x);
    }
}

PHX_HD void ipm_steps(const Prob& P, const State& St, const Ipm& I, int s, double& ap, double& ad) {
    const int S = P.S;
    ap = 1.0;
    ad = 1.0;
    for (int j = 0; j < P.n; ++j) {
        const int64_t o = ix(j, s, S);
        const double l = P.lb.at(j, s), u = P.ub.at(j, s), x = St.xT[o], d = I.dx[o];
        if (ipm_fixed(l, u)) continue;
        if (isfinite(l)) {
            if (d < 0.0) ap = fmin(ap, -(x - l) / d);
            if (I.dzl[o] < 0.0) ad = fmin(ad, -I.zl[o] / I.dzl[o]);
        }
        if (isfinite(u)) {
            if (d > 0.0) ap = fmin(ap, (u - x) / d);
            if (I.dzu[o] < 0.0) ad = fmin(ad, -I.zu[o] / I.dzu[o]);
        }
    }
    for (int i = 0; i < P.m; ++i) {
        const int64_t o = ix(i, s, S);
        const double bl = P.bl.at(i, s), bu = P.bu.at(i, s), sv = I.s[o], d = I.ds[o];
        if (bl == bu) continue;
        if (isfinite(bl)) {
            if (d < 0.0) ap = fmin(ap, -(sv - bl) / d);
            if (I.dwl[o] < 0.0) ad = fmin(ad, -I.wl[o] / I.dwl[o]);
        }
        if (isfinite(bu)) {
            if (d > 0.0) ap = fmin(ap, (bu - sv) / d);
            if (I.dwu[o] < 0.0) ad = fmin(ad, -I.wu[o] / I.dwu[o]);
        }
    }
}

PHX_HD double ipm_lane(const Prob& P, const State& St, const Polish& W, const Ipm& I, int s,
                       int max_it, double tol, double reg) {
    const int S = P.S, n = P.n, m = P.m;
    // ---- start point ----
    for (int j = 0; j < n; ++j) {
        const int64_t o = ix(j, s, S);
        const double l = P.lb.at(j, s), u = P.ub.at(j, s);
        double x;
        if (ipm_fixed(l, u)) x = l;
        else if (isfinite(l) && isfinite(u)) x = (u - l <= 2.0) ? 0.5 * (l + u) : clampd(0.0, l + 1.0, u - 1.0);
        else x = clampd(0.0, isfinite(l) ? l + 1.0 : -1e300, isfinite(u) ? u - 1.0 : 1e300);
        St.xT[o] = x;
        // cost-aware start: bound multipliers absorb the linear cost so the
        // initial dual residual is O(1) even with costs spanning 1e1..1e5
        double q, p;
        col_cost(P, j, s, q, p);
        const double g = q + p * x;
        I.zl[o] = isfinite(l) && !ipm_fixed(l, u) ? fmax(g, 0.0) + 1.0 : 0.0;
        I.zu[o] = isfinite(u) && !ipm_fixed(l, u) ? fmax(-g, 0.0) + 1.0 : 0.0;
        I.dzl[o] = I.dzu[o] = 0.0;
    }
    for (int i = 0; i < m; ++i) {
        const int64_t o = ix(i, s, S);
        const double bl = P.bl.at(i, s), bu = P.bu.at(i, s);
        double ax = 0.0;
        for (int k = P.rowptr[i]; k < P.rowptr[i + 1]; ++k)
            ax += aval(P, k, s) * St.xT[ix(P.colidx[k], s, S)];
        double sv = ax;
        const bool eq = (bl == bu);
        if (eq) sv = bl;
        else if (isfinite(bl) && isfinite(bu)) sv = (bu - bl <= 2.0) ? 0.5 * (bl + bu) : clampd(ax, bl + 1.0, bu - 1.0);
        else sv = clampd(ax, isfinite(bl) ? bl + 1.0 : -1e300, isfinite(bu) ? bu - 1.0 : 1e300);
        I.s[o] = sv;
        I.wl[o] = (isfinite(bl) && !eq) ? 1.0 : 0.0;
        I.wu[o] = (isfinite(bu) && !eq) ? 1.0 : 0.0;
        I.dwl[o] = I.dwu[o] = 0.0;
        St.yT[o] = I.wl[o] - I.wu[o];
    }
    double err = 1e300;
    for (int it = 0; it < max_it; ++it) {
        err = kkt_error(P, St.xT, St.yT, s);
        int ncomp;
        const double mu = ipm_mu(P, St, I, s, ncomp);
#if defined(PHX_IPM_TRACE)
        if (s == PHX_IPM_TRACE) printf("[ipm s=%d] it=%d err=%.3e mu=%.3e\n", s, it, err, mu);
#endif
        if (err < tol || !(err < 1e300)) break;
        // ---- H_x, normal matrix, Cholesky ----
        for (int j = 0; j < n; ++j) {
            const int64_t o = ix(j, s, S);
            const double l = P.lb.at(j, s), u = P.ub.at(j, s), x = St.xT[o];
            double q, p;
            col_cost(P, j, s, q, p);
            double h = p + reg;
            if (ipm_fixed(l, u)) h = 1e300;
            else {
                if (isfinite(l)) h += I.zl[o] / (x - l);
                if (isfinite(u)) h += I.zu[o] / (u - x);
            }
            I.hx[o] = h;
        }
        for (int i = 0; i < m; ++i) {
            const double bl = P.bl.at(i, s), bu = P.bu.at(i, s);
            const int64_t o = ix(i, s, S);
            double dg;
            if (!isfinite(bl) && !isfinite(bu)) dg = 1.0;
            else if (bl == bu) dg = reg;
            else {
                const double sv = I.s[o];
                double sig = 0.0;
                if (isfinite(bl)) sig += I.wl[o] / (sv - bl);
                if (isfinite(bu)) sig += I.wu[o] / (bu - sv);
                dg = 1.0 / sig + reg;
            }
            for (int k = 0; k < i; ++k) W.L[ix((int)tri(i, k), s, S)] = 0.0;
            W.L[ix((int)tri(i, i), s, S)] = dg;
        }
        for (int j = 0; j < n; ++j) {
            const double D = 1.0 / I.hx[ix(j, s, S)];
            for (int ka = P.colptr[j]; ka < P.colptr[j + 1]; ++ka) {
                const int ia = P.rowidx[ka];
                const double bla = P.bl.at(ia, s), bua = P.bu.at(ia, s);
                if (!isfinite(bla) && !isfinite(bua)) continue;
                const double va = aval(P, P.csc2csr[ka], s) * D;
                for (int kb = P.colptr[j]; kb <= ka; ++kb) {
                    const int ib = P.rowidx[kb];
                    const double blb = P.bl.at(ib, s), bub = P.bu.at(ib, s);
                    if (!isfinite(blb) && !isfinite(bub)) continue;
                    const int hi = ia > ib ? ia : ib, lo = ia > ib ? ib : ia;
                    W.L[ix((int)tri(hi, lo), s, S)] += va * aval(P, P.csc2csr[kb], s);
                }
            }
        }
        bool okc = true;
        for (int jj = 0; jj < m && okc; ++jj) {
            double d = W.L[ix((int)tri(jj, jj), s, S)];
            for (int k = 0; k < jj; ++k) {
                const double v = W.L[ix((int)tri(jj, k), s, S)];
                d -= v * v;
            }
            if (!(d > 0.0)) { okc = false; break; }
            d = sqrt(d);
            W.L[ix((int)tri(jj, jj), s, S)] = d;
            for (int i = jj + 1; i < m; ++i) {
                double v = W.L[ix((int)tri(i, jj), s, S)];
                for (int k = 0; k < jj; ++k)
                    v -= W.L[ix((int)tri(i, k), s, S)] * W.L[ix((int)tri(jj, k), s, S)];
                W.L[ix((int)tri(i, jj), s, S)] = v / d;
            }
        }
        if (!okc) break;
        // ---- predictor ----
        for (int j = 0; j < n; ++j) {
            const int64_t o = ix(j, s, S);
            const double l = P.lb.at(j, s), u = P.ub.at(j, s), x = St.xT[o];
            I.cl[o] = isfinite(l) ? -(x - l) * I.zl[o] : 0.0;
            I.cu[o] = isfinite(u) ? -(u - x) * I.zu[o] : 0.0;
        }
        for (int i = 0; i < m; ++i) {
            const int64_t o = ix(i, s, S);
            const double bl = P.bl.at(i, s), bu = P.bu.at(i, s), sv = I.s[o];
            I.cwl[o] = (isfinite(bl) && bl != bu) ? -(sv - bl) * I.wl[o] : 0.0;
            I.cwu[o] = (isfinite(bu) && bl != bu) ? -(bu - sv) * I.wu[o] : 0.0;
        }
        ipm_direction(P, St, W, I, s);
        double ap, ad;
        ipm_steps(P, St, I, s, ap, ad);
        // affine complementarity
        double maff = 0.0;
        for (int j = 0; j < n; ++j) {
            const int64_t o = ix(j, s, S);
            const double l = P.lb.at(j, s), u = P.ub.at(j, s), x = St.xT[o];
            if (ipm_fixed(l, u)) continue;
            if (isfinite(l)) maff += (x - l + ap * I.dx[o]) * (I.zl[o] + ad * I.dzl[o]);
            if (isfinite(u)) maff += (u - x - ap * I.dx[o]) * (I.zu[o] + ad * I.dzu[o]);
        }
        for (int i = 0; i < m; ++i) {
            const int64_t o = ix(i, s, S);
            const double bl = P.bl.at(i, s), bu = P.bu.at(i, s), sv = I.s[o];
            if (bl == bu) continue;
            if (isfinite(bl)) maff += (sv - bl + ap * I.ds[o]) * (I.wl[o] + ad * I.dwl[o]);
            if (isfinite(bu)) maff += (bu - sv - ap * I.ds[o]) * (I.wu[o] + ad * I.dwu[o]);
        }
        maff = ncomp ? maff / ncomp : 0.0;
        const double ratio = mu > 0.0 ? maff / mu : 0.0;
        const double smu = ratio * ratio * ratio * mu;
        // ---- corrector ----
        for (int j = 0; j < n; ++j) {
            const int64_t o = ix(j, s, S);
            const double l = P.lb.at(j, s), u = P.ub.at(j, s), x = St.xT[o];
            I.cl[o] = isfinite(l) ? smu - (x - l) * I.zl[o] - I.dx[o] * I.dzl[o] : 0.0;
            I.cu[o] = isfinite(u) ? smu - (u - x) * I.zu[o] + I.dx[o] * I.dzu[o] : 0.0;
        }
        for (int i = 0; i < m; ++i) {
            const int64_t o = ix(i, s, S);
            const double bl = P.bl.at(i, s), bu = P.bu.at(i, s), sv = I.s[o];
            I.cwl[o] = (isfinite(bl) && bl != bu) ? smu - (sv - bl) * I.wl[o] - I.ds[o] * I.dwl[o] : 0.0;
            I.cwu[o] = (isfinite(bu) && bl != bu) ? smu - (bu - sv) * I.wu[o] + I.ds[o] * I.dwu[o] : 0.0;
        }
        ipm_direction(P, St, W, I, s);
        ipm_steps(P, St, I, s, ap, ad);
        ap = fmin(1.0, 0.995 * ap);
        ad = fmin(1.0, 0.995 * ad);
        // keep the last finite iterate (an infeasible lane's diverging multipliers
        // are its Farkas ray; a NaN step would erase them)
        double fin = ap + ad;
        for (int j = 0; j < n; ++j) {
            const int64_t o = ix(j, s, S);
            fin += I.dx[o] + I.dzl[o] + I.dzu[o];
        }
        for (int i = 0; i < m; ++i) {
            const int64_t o = ix(i, s, S);
            fin += I.ds[o] + I.dwl[o] + I.dwu[o] + I.dy[o];
        }
        if (!isfinite(fin)) break;
        for (int j = 0; j < n; ++j) {
            const int64_t o = ix(j, s, S);
            St.xT[o] += ap * I.dx[o];
            I.zl[o] += ad * I.dzl[o];
            I.zu[o] += ad * I.dzu[o];
        }
        for (int i = 0; i < m; ++i) {
            const int64_t o = ix(i, s, S);
            I.s[o] += ap * I.ds[o];
            I.wl[o] += ad * I.dwl[o];
            I.wu[o] += ad * I.dwu[o];
            St.yT[o] += ad * I.dy[o];
        }
    }
    return err;
}

// After a successful polish: adopt the polished point as the solution and as
// the warm start for the next solve.
PHX_HD void adopt_polished(const Prob& P, const State& St, const Polish& W, int s) {
    const int S = P.S;
    for (int j = 0; j < P.n; ++j) {
        const int64_t o = ix(j, s, S);
        const double v = W.xp[o];
        St.xT[o] = v; St.x[o] = v; St.x0[o] = v;
    }
    for (int i = 0; i < P.m; ++i) {
        const int64_t o = ix(i, s, S);
        const double v = -W.z[o];
        St.yT[o] = v; St.y[o] = v; St.y0[o] = v;
    }
}

// IPM finisher for one lane + polish; returns the lane's final status
// (OPTIMAL, or INFEASIBLE with a Farkas certificate from the failed interior
// point's multipliers), RUNNING when the lane goes on with PDHG.
PHX_HD int finish_lane(const Prob& P, const State& St, const Polish& W, const Ipm& I, const Opts& O, int s) {
    St.flags[s] |= 1;
    const double e = ipm_lane(P, St, W, I, s, O.ipm_max_it, O.ipm_tol, 1e-10);
    St.err[s] = e;
    if (!(e < 1e-4) && farkas_lane(P, St.yT, s)) return INFEASIBLE;
    bool done = false;
    if (e < 1e-4 && O.polish) {
        const double tol = fmin(1e-4, fmax(1e-9, 10.0 * e));
        if (polish_lane(P, St, W, O, s, tol)) {
            adopt_polished(P, St, W, s);
            done = true;
        }
    }
    if (!done && e < O.opt_tol) done = true;
    // warm start / restart PDHG from the IPM point either way
    for (int j = 0; j < P.n; ++j) {
        const int64_t o = ix(j, s, P.S);
        St.x[o] = St.x0[o] = St.xT[o];
    }
    for (int i = 0; i < P.m; ++i) {
        const int64_t o = ix(i, s, P.S);
        St.y[o] = St.y0[o] = St.yT[o];
    }
    St.hk[s] = 0;
    St.r0[s] = 1e301;
    St.rprev[s] = 1e301;
    return done ? OPTIMAL : RUNNING;
}

// Unscaled outputs + objective (c'x + qN'x_N + 0.5 pN x_N^2 + kN), the value
// the reference reads back as pyo.value(objective) and outer_bound
// (spopt.py:197-206, 327-343).
PHX_HD void finalize_lane(const Prob& P, const State& St, const double* c_unscaled_p,
                          int64_t c_si, int64_t c_ss, int s,
                          double* x_out, double* y_out, double* obj_out) {
    const int S = P.S;
    double f = P.kN[s];
    for (int j = 0; j < P.n; ++j) {
        const int64_t o = ix(j, s, S);
        const double x = St.xT[o] * P.dc[j];
        x_out[o] = x;
        f += c_unscaled_p[(int64_t)j * c_si + (int64_t)s * c_ss] * x;
        const int sl = P.col_slot[j];
        if (sl >= 0) f += P.qN[ix(sl, s, S)] * x + 0.5 * P.pN[ix(sl, s, S)] * x * x;
    }
    if (y_out)
        for (int i = 0; i < P.m; ++i) {
            const int64_t o = ix(i, s, S);
            y_out[o] = St.yT[o] * P.dr[i];
        }
    obj_out[s] = f;
}

// Objective of an unscaled point x ([n][S]) under the current PH terms.
PHX_HD double objective_lane(const Prob& P, const double* c_unscaled_p, int64_t c_si, int64_t c_ss,
                             const double* x, int s) {
    const int S = P.S;
    double f = P.kN[s];
    for (int j = 0; j < P.n; ++j) {
        const double v = x[ix(j, s, S)];
        f += c_unscaled_p[(int64_t)j * c_si + (int64_t)s * c_ss] * v;
        const int sl = P.col_slot[j];
        if (sl >= 0) f += P.qN[ix(sl, s, S)] * v + 0.5 * P.pN[ix(sl, s, S)] * v * v;
    }
    return f;
}

// Power iteration for ||A_s||_2 of the scaled matrix (per lane), using the
// xb / yT state rows as scratch.
PHX_HD double spectral_norm(const Prob& P, const State& St, int s, int iters) {
    const int S = P.S;
    for (int j = 0; j < P.n; ++j) St.xb[ix(j, s, S)] = 1.0 + 0.01 * (double)(j % 7);
    double nrm = 0.0;
    for (int it = 0; it < iters; ++it) {
        for (int i = 0; i < P.m; ++i) {
            double ax = 0.0;
            for (int k = P.rowptr[i]; k < P.rowptr[i + 1]; ++k)
                ax += aval(P, k, s) * St.xb[ix(P.colidx[k], s, S)];
            St.yT[ix(i, s, S)] = ax;
        }
        double nn = 0.0;
        for (int j = 0; j < P.n; ++j) {
            double aty = 0.0;
            for (int k = P.colptr[j]; k < P.colptr[j + 1]; ++k)
                aty += aval(P, P.csc2csr[k], s) * St.yT[ix(P.rowidx[k], s, S)];
            St.xb[ix(j, s, S)] = aty;
            nn += aty * aty;
        }
        nn = sqrt(nn);
        if (!(nn > 0.0)) return 1.0;
        for (int j = 0; j < P.n; ++j) St.xb[ix(j, s, S)] /= nn;
        nrm = sqrt(nn);
    }
    return nrm;
}

}  // namespace phx
