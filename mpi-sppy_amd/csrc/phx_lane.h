// phx_lane.h — register-resident lane solver for SMALL subproblems.
//
// For subproblems with a few dozen variables/rows (farmer, aircond) the whole
// per-scenario solve fits in the registers of one lane.  The solver is written
// once as templates over a pattern type PT whose accessors are constexpr when
// the kernels are JIT-specialised with hipRTC (phx_jit.h): every loop has a
// compile-time trip count, so hipcc fully unrolls it, constant-folds the
// sparsity pattern and the bound-finiteness structure (the multipliers of
// infinite bounds and their updates vanish) and keeps the per-lane vectors in
// VGPRs.  Scenario-invariant numbers (constant A entries, costs, bounds,
// scaling) are baked in as exact literals (one kernel per problem, compiled at
// phx_set_problem); only scenario-varying values occupy vector registers.  The same templates compile on the host with a runtime pattern
// (tests/emu), which is how the CPU suite checks them.
//
// Two kernels per solve (phx_jit.h emits both):
//   phx_lane_ipm     Mehrotra predictor-corrector IPM on
//                      min 0.5 x'Px + q'x  s.t. Ax - s = 0, l <= x <= u,
//                      bl <= s <= bu
//                    normal matrix M = A (P+Sx)^-1 A' + Ss^-1 (packed
//                    Cholesky).  Bound-multiplier steps are recomputed from
//                    (dx, ds) instead of stored.  Writes (x, y) to xT/yT and
//                    the PDHG warm start (phx_core.h conventions).
//   phx_lane_polish  active-set KKT polish from (xT, yT): classification by
//                    slack-vs-multiplier (sharp at IPM points), quasi-definite
//                    regularised KKT + iterative refinement, KKT certificate.
// Lanes that fail the certificate continue on the generic PDHG path from the
// IPM point.
#pragma once
#if !defined(__HIPCC_RTC__)
#include <stdint.h>
#include <math.h>
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#endif
#else
typedef long long int64_t;   // hipRTC: no libc headers; hip_runtime provides the math
typedef int int32_t;
#endif

#if defined(__HIPCC__) || defined(__HIPCC_RTC__)
#define PHX_LD __host__ __device__ __forceinline__
#define PHX_UNROLL _Pragma("unroll")
#else
#define PHX_LD inline
#define PHX_UNROLL
#endif

namespace phx_lane {

PHX_LD int tri(int i, int k) { return i * (i + 1) / 2 + k; }   // i >= k
PHX_LD double clampd(double v, double lo, double hi) { return fmin(fmax(v, lo), hi); }

// Runtime inputs/outputs (device pointers; per-scenario arrays [i*S + s]).
struct LaneIO {
    int32_t S;
    const double* Ac;      // scaled invariant A values [nnz]
    const double* dr;      // row scaling [m]
    const double* dc;      // column scaling [n]
    const double* Av;      // varying scaled A values [nvar*S]
    const double* c;       // scaled c   [n] or [n*S] (PT::c_vary())
    const double* lb;      // scaled lb  [n] or [n*S] (PT::bnd_vary())
    const double* ub;
    const double* bl;      // scaled bl  [m] or [m*S] (PT::rhs_vary())
    const double* bu;
    const double* qN;      // unscaled PH linear term [N*S]
    const double* pN;      // unscaled PH quadratic   [N*S]
    double* xT;            // scaled x [n*S]
    double* yT;            // scaled y [m*S]
    double* x;             // PDHG warm start (= xT)
    double* y;
    double* x0;
    double* y0;
    double* err;           // [S]
    int32_t* status;       // [S]: 1 certified, 0 hand over to PDHG
    int32_t* iters;        // [S]: IPM iterations used
    int32_t* flags;        // [S]: bit0 set (IPM attempted)
    int32_t max_it;
    double ipm_tol;
    double kkt_tol;
    double reg;
    int32_t refine;
};

// Data access for one lane: scenario-varying numbers in registers; the
// invariant ones are literals of the specialised kernel (PT tables), which the
// compiler rematerialises with scalar moves instead of keeping them live.
template <class PT>
struct Data {
    const LaneIO& io;
    const int sc;
    double av[PT::NMAX_V];
    double qn[PT::NMAX_S], pn[PT::NMAX_S];

    PHX_LD Data(const LaneIO& io_, int sc_) : io(io_), sc(sc_) {
        const int S = io.S;
        PHX_UNROLL for (int v = 0; v < PT::nvar(); ++v) av[v] = io.Av[(int64_t)v * S + sc];
        PHX_UNROLL for (int t = 0; t < PT::nslot(); ++t) {
            qn[t] = io.qN[(int64_t)t * S + sc];
            pn[t] = io.pN[(int64_t)t * S + sc];
        }
    }
    PHX_LD double A(int k) const { return PT::kvar(k) < 0 ? PT::Ac(k) : av[PT::kvar(k)]; }
    PHX_LD double dc(int j) const { return PT::dcs(j); }
    PHX_LD double dr(int i) const { return PT::drs(i); }
    PHX_LD double q(int j) const {
        const double c = PT::c_vary() ? io.c[(int64_t)j * io.S + sc] : PT::cs(j);
        return PT::col_slot(j) >= 0 ? c + dc(j) * qn[PT::col_slot(j)] : c;
    }
    PHX_LD double p(int j) const {
        return PT::col_slot(j) >= 0 ? dc(j) * dc(j) * pn[PT::col_slot(j)] : 0.0;
    }
    PHX_LD double l(int j) const { return PT::bnd_vary() ? io.lb[(int64_t)j * io.S + sc] : PT::lbs(j); }
    PHX_LD double u(int j) const { return PT::bnd_vary() ? io.ub[(int64_t)j * io.S + sc] : PT::ubs(j); }
    PHX_LD double bl(int i) const { return PT::rhs_vary() ? io.bl[(int64_t)i * io.S + sc] : PT::bls(i); }
    PHX_LD double bu(int i) const { return PT::rhs_vary() ? io.bu[(int64_t)i * io.S + sc] : PT::bus(i); }

    PHX_LD void matvec(const double* xv, double* ax) const {
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) ax[i] = 0.0;
        PHX_UNROLL for (int k = 0; k < PT::nnz(); ++k) ax[PT::row(k)] += A(k) * xv[PT::col(k)];
    }
    PHX_LD void matvec_t(const double* yv, double* aty) const {
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) aty[j] = 0.0;
        PHX_UNROLL for (int k = 0; k < PT::nnz(); ++k) aty[PT::col(k)] += A(k) * yv[PT::row(k)];
    }

    // relative KKT error, unscaled measure (phx_core.h kkt_error)
    PHX_LD double kkt(const double* xv, const double* yv) const {
        double rp2 = 0.0, bn2 = 0.0, rd2 = 0.0, qn2 = 0.0, pobj = 0.0, dobj = 0.0;
        {
            double ax[PT::NMAX_M];
            matvec(xv, ax);
            PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
                const double d = dr(i);
                const double axu = ax[i] / d;
                double r = 0.0;
                if (PT::blfin(i)) r = fmin(axu - bl(i) / d, 0.0);
                if (PT::bufin(i)) r += fmax(axu - bu(i) / d, 0.0);
                rp2 += r * r;
                if (PT::blfin(i)) bn2 += (bl(i) / d) * (bl(i) / d);
                if (PT::bufin(i)) bn2 += (bu(i) / d) * (bu(i) / d);
                if (PT::blfin(i) && yv[i] > 0.0) dobj += bl(i) * yv[i];
                if (PT::bufin(i) && yv[i] < 0.0) dobj += bu(i) * yv[i];
            }
        }
        double aty[PT::NMAX_N];
        matvec_t(yv, aty);
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
            const double qj = q(j), pj = p(j), d = dc(j);
            const double lam_s = qj + pj * xv[j] - aty[j];
            const double lam = lam_s / d;
            double rd = lam;
            if (PT::lfin(j) && lam > 0.0) { rd = 0.0; dobj += l(j) * lam_s; }
            if (PT::ufin(j) && lam < 0.0) { rd = 0.0; dobj += u(j) * lam_s; }
            rd2 += rd * rd;
            qn2 += (qj / d) * (qj / d);
            pobj += qj * xv[j] + 0.5 * pj * xv[j] * xv[j];
            dobj -= 0.5 * pj * xv[j] * xv[j];
        }
        const double ep = sqrt(rp2) / (1.0 + sqrt(bn2));
        const double ed = sqrt(rd2) / (1.0 + sqrt(qn2));
        const double eg = fabs(pobj - dobj) / (1.0 + fabs(pobj) + fabs(dobj));
        const double e = fmax(ep, fmax(ed, eg));
        return (e == e && e < 1e300) ? e : 1e300;
    }
};

// packed Cholesky (lower, in place); false if not positive definite
template <class PT>
PHX_LD bool cholesky(double* M) {
    bool ok = true;
    PHX_UNROLL for (int jj = 0; jj < PT::m(); ++jj) {
        double d = M[tri(jj, jj)];
        PHX_UNROLL for (int k = 0; k < PT::m(); ++k)
            if (k < jj) d -= M[tri(jj, k)] * M[tri(jj, k)];
        ok = ok && (d > 0.0);
        d = sqrt(fmax(d, 1e-300));
        M[tri(jj, jj)] = d;
        const double inv = 1.0 / d;
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
            if (i > jj) {
                double v = M[tri(i, jj)];
                PHX_UNROLL for (int k = 0; k < PT::m(); ++k)
                    if (k < jj) v -= M[tri(i, k)] * M[tri(jj, k)];
                M[tri(i, jj)] = v * inv;
            }
        }
    }
    return ok;
}

// solve (L L') t = t ; diagonal stored as its reciprocal is not assumed
template <class PT>
PHX_LD void chol_solve(const double* M, double* t) {
    PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
        double v = t[i];
        PHX_UNROLL for (int k = 0; k < PT::m(); ++k)
            if (k < i) v -= M[tri(i, k)] * t[k];
        t[i] = v / M[tri(i, i)];
    }
    PHX_UNROLL for (int ii = 0; ii < PT::m(); ++ii) {
        const int i = PT::m() - 1 - ii;
        double v = t[i];
        PHX_UNROLL for (int k = 0; k < PT::m(); ++k)
            if (k > i) v -= M[tri(k, i)] * t[k];
        t[i] = v / M[tri(i, i)];
    }
}

// Complementarity right-hand sides with Mehrotra's second-order term.
// Lower side (slack sl = x - l, multiplier z, affine step da):
//   dz_aff = -z (sl + da) / sl,  c = smu - sl z - da dz_aff,  dz = (c - z dx) / sl
// Upper side (slack sl = u - x):
//   dz_aff =  z (da - sl) / sl,  c = smu - sl z + da dz_aff,  dz = (c + z dx) / sl
// (da = 0 in the predictor pass gives the plain affine system.)
PHX_LD double comp_lo(double sl, double z, double smu, double da) { return smu - sl * z + da * z * (sl + da) / sl; }
PHX_LD double comp_up(double sl, double z, double smu, double da) { return smu - sl * z + da * z * (da - sl) / sl; }

template <class PT>
PHX_LD bool has_lo(int j) { return PT::lfin(j) && !PT::fixed(j); }
template <class PT>
PHX_LD bool has_up(int j) { return PT::ufin(j) && !PT::fixed(j); }
template <class PT>
PHX_LD bool row_lo(int i) { return PT::blfin(i) && !PT::eq(i); }
template <class PT>
PHX_LD bool row_up(int i) { return PT::bufin(i) && !PT::eq(i); }
template <class PT>
PHX_LD bool row_free(int i) { return !PT::blfin(i) && !PT::bufin(i); }

// ---------------------------------------------------------------------------
// IPM kernel body
// ---------------------------------------------------------------------------
template <class PT>
PHX_LD void ipm_lane(const LaneIO& io, int sc) {
    constexpr int NN = PT::NMAX_N, MM = PT::NMAX_M, TT = PT::NMAX_M * (PT::NMAX_M + 1) / 2;
    const Data<PT> D(io, sc);
    const double reg = 1e-10;
    double x[NN], zl[NN], zu[NN], s[MM], y[MM], wl[MM], wu[MM];
    // start point (cost-aware multipliers, phx_core.h ipm_lane)
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
        double xv = 0.0;
        if (PT::fixed(j)) xv = D.l(j);
        else if (PT::lfin(j) && PT::ufin(j)) {
            const double lo = D.l(j), hi = D.u(j);
            xv = (hi - lo <= 2.0) ? 0.5 * (lo + hi) : clampd(0.0, lo + 1.0, hi - 1.0);
        } else if (PT::lfin(j)) xv = fmax(0.0, D.l(j) + 1.0);
        else if (PT::ufin(j)) xv = fmin(0.0, D.u(j) - 1.0);
        x[j] = xv;
        const double g = D.q(j) + D.p(j) * xv;
        zl[j] = has_lo<PT>(j) ? fmax(g, 0.0) + 1.0 : 0.0;
        zu[j] = has_up<PT>(j) ? fmax(-g, 0.0) + 1.0 : 0.0;
    }
    {
        double ax[MM];
        D.matvec(x, ax);
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
            double sv = ax[i];
            if (PT::eq(i)) sv = D.bl(i);
            else if (PT::blfin(i) && PT::bufin(i)) {
                const double lo = D.bl(i), hi = D.bu(i);
                sv = (hi - lo <= 2.0) ? 0.5 * (lo + hi) : clampd(ax[i], lo + 1.0, hi - 1.0);
            } else if (PT::blfin(i)) sv = fmax(ax[i], D.bl(i) + 1.0);
            else if (PT::bufin(i)) sv = fmin(ax[i], D.bu(i) - 1.0);
            s[i] = sv;
            wl[i] = row_lo<PT>(i) ? 1.0 : 0.0;
            wu[i] = row_up<PT>(i) ? 1.0 : 0.0;
            y[i] = wl[i] - wu[i];
        }
    }
    double ncomp = 0.0;
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) ncomp += (has_lo<PT>(j) ? 1.0 : 0.0) + (has_up<PT>(j) ? 1.0 : 0.0);
    PHX_UNROLL for (int i = 0; i < PT::m(); ++i) ncomp += (row_lo<PT>(i) ? 1.0 : 0.0) + (row_up<PT>(i) ? 1.0 : 0.0);
    double err = 1e300;
    int it = 0;
    for (; it < io.max_it; ++it) {
        err = D.kkt(x, y);
        if (err < io.ipm_tol || !(err < 1e300)) break;
        double mu = 0.0;
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
            if (has_lo<PT>(j)) mu += (x[j] - D.l(j)) * zl[j];
            if (has_up<PT>(j)) mu += (D.u(j) - x[j]) * zu[j];
        }
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
            if (row_lo<PT>(i)) mu += (s[i] - D.bl(i)) * wl[i];
            if (row_up<PT>(i)) mu += (D.bu(i) - s[i]) * wu[i];
        }
        mu = ncomp > 0.0 ? mu / ncomp : 0.0;
        // normal matrix
        double Dx[NN], sig[MM], M[TT];
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
            double h = D.p(j) + reg;
            if (has_lo<PT>(j)) h += zl[j] / (x[j] - D.l(j));
            if (has_up<PT>(j)) h += zu[j] / (D.u(j) - x[j]);
            Dx[j] = PT::fixed(j) ? 0.0 : 1.0 / h;
        }
        PHX_UNROLL for (int t = 0; t < TT; ++t) M[t] = 0.0;
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
            double sg = 0.0;
            if (row_lo<PT>(i)) sg += wl[i] / (s[i] - D.bl(i));
            if (row_up<PT>(i)) sg += wu[i] / (D.bu(i) - s[i]);
            sig[i] = sg;
            M[tri(i, i)] = row_free<PT>(i) ? 1.0 : (PT::eq(i) ? reg : 1.0 / sg + reg);
        }
        PHX_UNROLL for (int t = 0; t < PT::npairs(); ++t) {
            const int ka = PT::pair_a(t), kb = PT::pair_b(t);
            if (!row_free<PT>(PT::row(ka)) && !row_free<PT>(PT::row(kb)))
                M[PT::pair_pos(t)] += D.A(ka) * Dx[PT::col(ka)] * D.A(kb);
        }
        if (!cholesky<PT>(M)) break;
        // predictor (pass 0, smu = 0) then corrector (pass 1)
        double smu = 0.0, ap = 1.0, ad = 1.0;
        double dx[NN], ds[MM], dy[MM], dxa[NN], dsa[MM];
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) dxa[j] = 0.0;
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) dsa[i] = 0.0;
        for (int pass = 0; pass < 2; ++pass) {
            {
                double ax[MM], aty[NN];
                D.matvec(x, ax);
                D.matvec_t(y, aty);
                PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
                    double r = aty[j] - D.p(j) * x[j] - D.q(j);
                    if (has_lo<PT>(j)) {
                        const double sl = x[j] - D.l(j);
                        r += zl[j] + comp_lo(sl, zl[j], smu, dxa[j]) / sl;
                    }
                    if (has_up<PT>(j)) {
                        const double sl = D.u(j) - x[j];
                        r -= zu[j] + comp_up(sl, zu[j], smu, dxa[j]) / sl;
                    }
                    dx[j] = PT::fixed(j) ? 0.0 : r * Dx[j];      // H^-1 rho_x
                }
                double ahr[MM];
                D.matvec(dx, ahr);
                PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
                    double rhos = -y[i];
                    if (row_lo<PT>(i)) {
                        const double sl = s[i] - D.bl(i);
                        rhos += wl[i] + comp_lo(sl, wl[i], smu, dsa[i]) / sl;
                    }
                    if (row_up<PT>(i)) {
                        const double sl = D.bu(i) - s[i];
                        rhos -= wu[i] + comp_up(sl, wu[i], smu, dsa[i]) / sl;
                    }
                    ds[i] = rhos;
                    if (row_free<PT>(i)) dy[i] = 0.0;
                    else if (PT::eq(i)) dy[i] = -(ax[i] - D.bl(i)) - ahr[i];
                    else dy[i] = -(ax[i] - s[i]) + rhos / sig[i] - ahr[i];
                }
            }
            chol_solve<PT>(M, dy);
            {
                double atdy[NN];
                D.matvec_t(dy, atdy);
                PHX_UNROLL for (int j = 0; j < PT::n(); ++j)
                    if (!PT::fixed(j)) dx[j] += Dx[j] * atdy[j];
            }
            PHX_UNROLL for (int i = 0; i < PT::m(); ++i)
                ds[i] = (PT::eq(i) || row_free<PT>(i)) ? 0.0 : (ds[i] - dy[i]) / sig[i];
            // step lengths (multiplier steps recomputed from dx, ds)
            ap = 1.0;
            ad = 1.0;
            double maff = 0.0;
            PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
                if (has_lo<PT>(j)) {
                    const double sl = x[j] - D.l(j);
                    const double dz = (comp_lo(sl, zl[j], smu, dxa[j]) - zl[j] * dx[j]) / sl;
                    if (dx[j] < 0.0) ap = fmin(ap, -sl / dx[j]);
                    if (dz < 0.0) ad = fmin(ad, -zl[j] / dz);
                }
                if (has_up<PT>(j)) {
                    const double sl = D.u(j) - x[j];
                    const double dz = (comp_up(sl, zu[j], smu, dxa[j]) + zu[j] * dx[j]) / sl;
                    if (dx[j] > 0.0) ap = fmin(ap, sl / dx[j]);
                    if (dz < 0.0) ad = fmin(ad, -zu[j] / dz);
                }
            }
            PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
                if (row_lo<PT>(i)) {
                    const double sl = s[i] - D.bl(i);
                    const double dw = (comp_lo(sl, wl[i], smu, dsa[i]) - wl[i] * ds[i]) / sl;
                    if (ds[i] < 0.0) ap = fmin(ap, -sl / ds[i]);
                    if (dw < 0.0) ad = fmin(ad, -wl[i] / dw);
                }
                if (row_up<PT>(i)) {
                    const double sl = D.bu(i) - s[i];
                    const double dw = (comp_up(sl, wu[i], smu, dsa[i]) + wu[i] * ds[i]) / sl;
                    if (ds[i] > 0.0) ap = fmin(ap, sl / ds[i]);
                    if (dw < 0.0) ad = fmin(ad, -wu[i] / dw);
                }
            }
            if (pass == 0) {
                PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
                    if (has_lo<PT>(j)) {
                        const double sl = x[j] - D.l(j);
                        const double dz = -zl[j] * (sl + dx[j]) / sl;
                        maff += (sl + ap * dx[j]) * (zl[j] + ad * dz);
                    }
                    if (has_up<PT>(j)) {
                        const double sl = D.u(j) - x[j];
                        const double dz = zu[j] * (dx[j] - sl) / sl;
                        maff += (sl - ap * dx[j]) * (zu[j] + ad * dz);
                    }
                    dxa[j] = dx[j];
                }
                PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
                    if (row_lo<PT>(i)) {
                        const double sl = s[i] - D.bl(i);
                        const double dw = -wl[i] * (sl + ds[i]) / sl;
                        maff += (sl + ap * ds[i]) * (wl[i] + ad * dw);
                    }
                    if (row_up<PT>(i)) {
                        const double sl = D.bu(i) - s[i];
                        const double dw = wu[i] * (ds[i] - sl) / sl;
                        maff += (sl - ap * ds[i]) * (wu[i] + ad * dw);
                    }
                    dsa[i] = ds[i];
                }
                maff = ncomp > 0.0 ? maff / ncomp : 0.0;
                const double ratio = mu > 0.0 ? maff / mu : 0.0;
                smu = ratio * ratio * ratio * mu;
            }
        }
        // update (multipliers first: they use the old slacks)
        ap = fmin(1.0, 0.995 * ap);
        ad = fmin(1.0, 0.995 * ad);
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
            if (has_lo<PT>(j)) {
                const double sl = x[j] - D.l(j);
                zl[j] += ad * (comp_lo(sl, zl[j], smu, dxa[j]) - zl[j] * dx[j]) / sl;
            }
            if (has_up<PT>(j)) {
                const double sl = D.u(j) - x[j];
                zu[j] += ad * (comp_up(sl, zu[j], smu, dxa[j]) + zu[j] * dx[j]) / sl;
            }
            x[j] += ap * dx[j];
        }
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
            if (row_lo<PT>(i)) {
                const double sl = s[i] - D.bl(i);
                wl[i] += ad * (comp_lo(sl, wl[i], smu, dsa[i]) - wl[i] * ds[i]) / sl;
            }
            if (row_up<PT>(i)) {
                const double sl = D.bu(i) - s[i];
                wu[i] += ad * (comp_up(sl, wu[i], smu, dsa[i]) + wu[i] * ds[i]) / sl;
            }
            s[i] += ap * ds[i];
            y[i] += ad * dy[i];
        }
    }
    const int S = io.S;
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
        const int64_t o = (int64_t)j * S + sc;
        io.xT[o] = x[j]; io.x[o] = x[j]; io.x0[o] = x[j];
    }
    PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
        const int64_t o = (int64_t)i * S + sc;
        io.yT[o] = y[i]; io.y[o] = y[i]; io.y0[o] = y[i];
    }
    io.err[sc] = err;
    io.iters[sc] = it;
    io.status[sc] = 0;
    io.flags[sc] = io.flags[sc] | 1;
}

// ---------------------------------------------------------------------------
// Polish kernel body: from (xT, yT) written by ipm_lane.  Returns 1 if the
// certificate holds (then the polished point replaces xT/yT and the warm start).
// ---------------------------------------------------------------------------
template <class PT>
PHX_LD int polish_lane(const LaneIO& io, int sc) {
    constexpr int NN = PT::NMAX_N, MM = PT::NMAX_M, TT = PT::NMAX_M * (PT::NMAX_M + 1) / 2;
    const double e = io.err[sc];
    if (!(e < 1e-4)) { io.status[sc] = 0; return 0; }
    const Data<PT> D(io, sc);
    const int S = io.S;
    const double tol = fmin(1e-4, fmax(1e-9, 10.0 * e));
    const double reg = io.reg;
    double xp[NN], z[MM];
    bool F[NN], R[MM], lowside[MM];
    {
        double xv[NN], yv[MM];
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) xv[j] = io.xT[(int64_t)j * S + sc];
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) yv[i] = io.yT[(int64_t)i * S + sc];
        double aty[NN];
        D.matvec_t(yv, aty);
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
            const double lam = D.q(j) + D.p(j) * xv[j] - aty[j];
            bool fr = true;
            double v = xv[j];
            if (PT::lfin(j)) {
                const double lo = D.l(j);
                if (xv[j] - lo <= tol * (1.0 + fabs(lo)) || xv[j] - lo < lam) { fr = false; v = lo; }
            }
            if (fr && PT::ufin(j)) {
                const double hi = D.u(j);
                if (hi - xv[j] <= tol * (1.0 + fabs(hi)) || hi - xv[j] < -lam) { fr = false; v = hi; }
            }
            F[j] = fr;
            xp[j] = v;
        }
        double ax[MM];
        D.matvec(xv, ax);
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
            bool lo_act = false, up_act = false;
            if (PT::blfin(i)) {
                const double lo = D.bl(i);
                lo_act = ax[i] - lo <= tol * (1.0 + fabs(lo)) || ax[i] - lo < yv[i];
            }
            if (!lo_act && PT::bufin(i)) {
                const double hi = D.bu(i);
                up_act = hi - ax[i] <= tol * (1.0 + fabs(hi)) || hi - ax[i] < -yv[i];
            }
            R[i] = lo_act || up_act;
            lowside[i] = lo_act;
            z[i] = R[i] ? -yv[i] : 0.0;
        }
    }
    double Dx[NN], M[TT];
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) Dx[j] = F[j] ? 1.0 / (D.p(j) + reg) : 0.0;
    PHX_UNROLL for (int t = 0; t < TT; ++t) M[t] = 0.0;
    PHX_UNROLL for (int i = 0; i < PT::m(); ++i) M[tri(i, i)] = R[i] ? reg : 1.0;
    PHX_UNROLL for (int t = 0; t < PT::npairs(); ++t) {
        const int ka = PT::pair_a(t), kb = PT::pair_b(t);
        if (R[PT::row(ka)] && R[PT::row(kb)]) M[PT::pair_pos(t)] += D.A(ka) * Dx[PT::col(ka)] * D.A(kb);
    }
    bool ok = cholesky<PT>(M);
    if (ok) {
        for (int it = 0; it < io.refine; ++it) {
            double r1[NN], t[MM];
            {
                double atz[NN];
                D.matvec_t(z, atz);
                PHX_UNROLL for (int j = 0; j < PT::n(); ++j)
                    r1[j] = F[j] ? -D.q(j) - D.p(j) * xp[j] - atz[j] : 0.0;
            }
            {
                double axp[MM], hr[NN], ahr[MM];
                D.matvec(xp, axp);
                PHX_UNROLL for (int j = 0; j < PT::n(); ++j) hr[j] = r1[j] * Dx[j];
                D.matvec(hr, ahr);
                PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
                    const double b = lowside[i] ? D.bl(i) : D.bu(i);
                    t[i] = R[i] ? ahr[i] - (b - axp[i]) : 0.0;
                }
            }
            chol_solve<PT>(M, t);
            double atdz[NN];
            D.matvec_t(t, atdz);
            PHX_UNROLL for (int j = 0; j < PT::n(); ++j)
                if (F[j]) xp[j] += (r1[j] - atdz[j]) * Dx[j];
            PHX_UNROLL for (int i = 0; i < PT::m(); ++i)
                if (R[i]) z[i] += t[i];
        }
        // certificate (unscaled, relative kkt_tol)
        double qmax = 0.0;
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) qmax = fmax(qmax, fabs(D.q(j) / D.dc(j)));
        const double dtol = io.kkt_tol * (1.0 + qmax);
        const double ptol = io.kkt_tol;
        {
            double atz[NN];
            D.matvec_t(z, atz);
            PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
                const double d = D.dc(j);
                if (PT::lfin(j)) {
                    const double lo = D.l(j);
                    if (xp[j] < lo && (lo - xp[j]) * d > ptol * (1.0 + fabs(lo * d))) ok = false;
                }
                if (PT::ufin(j)) {
                    const double hi = D.u(j);
                    if (xp[j] > hi && (xp[j] - hi) * d > ptol * (1.0 + fabs(hi * d))) ok = false;
                }
                const double lam = (D.q(j) + D.p(j) * xp[j] + atz[j]) / d;
                if (F[j]) {
                    if (fabs(lam) > dtol) ok = false;
                } else if (!PT::fixed(j)) {
                    const bool atl = PT::lfin(j) && (xp[j] == D.l(j));
                    if (atl && lam < -dtol) ok = false;
                    if (!atl && lam > dtol) ok = false;
                }
            }
        }
        double axp[MM];
        D.matvec(xp, axp);
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
            const double d = D.dr(i);
            if (PT::blfin(i)) {
                const double lo = D.bl(i);
                if (axp[i] < lo && (lo - axp[i]) / d > ptol * (1.0 + fabs(lo / d))) ok = false;
            }
            if (PT::bufin(i)) {
                const double hi = D.bu(i);
                if (axp[i] > hi && (axp[i] - hi) / d > ptol * (1.0 + fabs(hi / d))) ok = false;
            }
            if (R[i] && !PT::eq(i)) {
                const double yy = -z[i] * d;
                if (lowside[i] && yy < -dtol) ok = false;
                if (!lowside[i] && yy > dtol) ok = false;
            }
        }
    }
    io.status[sc] = ok ? 1 : 0;
    if (ok) {
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
            const int64_t o = (int64_t)j * S + sc;
            io.xT[o] = xp[j]; io.x[o] = xp[j]; io.x0[o] = xp[j];
        }
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
            const int64_t o = (int64_t)i * S + sc;
            io.yT[o] = -z[i]; io.y[o] = -z[i]; io.y0[o] = -z[i];
        }
    }
    return ok ? 1 : 0;
}

}  // namespace phx_lane
