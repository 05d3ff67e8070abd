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

enum Status : int32_t { RUNNING = 0, OPTIMAL = 1, ITER_LIMIT = 2, NUMERIC_FAIL = 3 };

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

PHX_HD int64_t ix(int i, int s, int S) { return (int64_t)i * S + s; }

PHX_HD double aval(const Prob& P, int k, int s) {
    const int v = P.kvar[k];
    return v < 0 ? P.Ac[k] : P.Av[(int64_t)v * P.S + s];
}

PHX_HD double clampd(double v, double lo, double hi) { return fmin(fmax(v, lo), hi); }

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
    const double e = fmax(ep, fmax(ed, eg));
    return isfinite(e) ? e : 1e300;
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
    for (int j = 0; j < n; ++j) {
        const int64_t o = ix(j, s, S);
        const double x = St.xT[o];
        const double l = P.lb.at(j, s), u = P.ub.at(j, s);
        unsigned char f = 1;
        double xf = 0.0;
        if (isfinite(l) && x - l <= tol * (1.0 + fabs(l))) { f = 0; xf = l; }
        else if (isfinite(u) && u - x <= tol * (1.0 + fabs(u))) { f = 0; xf = u; }
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
        if (isfinite(bl) && ax - bl <= tol * (1.0 + fabs(bl))) { r = 1; b = bl; }
        else if (isfinite(bu) && bu - ax <= tol * (1.0 + fabs(bu))) { r = 1; b = bu; }
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
