// phx_emu.cpp — TEST INFRASTRUCTURE ONLY.
//
// Host (CPU) emulation of the libphx C ABI (include/phx.h) built from the very
// same per-lane math (mpi-sppy_amd/csrc/phx_core.h) and setup
// (phx_setup.h) as the HIP kernels: every "device pointer" is a host pointer
// and every kernel is a loop over lanes.  It lets the CPU test suite check the
// solver algorithm (PDHG + KKT polish) and the PH reductions against the CPU
// oracle without a GPU.  The product package never loads this library; on a
// GPU box the -m gpu tests exercise the real kernels instead.
//
// Symbols: emu_phx_<name>, same signatures as phx_<name>.
#include <stdint.h>
#include <string.h>
#include <math.h>
#include <string>
#include <vector>
#include <algorithm>
#include <stdio.h>
#include <stdlib.h>
#include "../../include/phx.h"
#include "../../mpi-sppy_amd/csrc/phx_core.h"
#include "../../mpi-sppy_amd/csrc/phx_setup.h"

using namespace phx;

struct emu_ctx {
    std::string err;
    bool have = false;
    int S = 0, n = 0, m = 0, nnz = 0, N = 0, nvar = 0;
    int c_vary = 0;
    HostSetup hs;
    std::vector<double> Av, cs, lbs, ubs, bls, bus, qN, pN, kN, c_user;
    std::vector<double> x, y, x0, y0, xT, yT, xb, omega, eta, r0, rprev, errv;
    std::vector<int32_t> hk, status, iters, flags;
    std::vector<double> ipm_buf;
    Ipm Iw{};
    std::vector<double> L, z, r1, t, xp, xfix, brhs;
    std::vector<unsigned char> F, R;
    Prob P{};
    State St{};
    Polish Pw{};
    bool solved_once = false;
    double lane_iters = 0;
    int launches = 0;
};

static void scale_rows(const double* src, double* dst, const double* sc, int64_t nrows, int64_t S, int mode) {
    for (int64_t r = 0; r < nrows; ++r)
        for (int64_t s = 0; s < S; ++s) {
            const double v = src[r * S + s];
            dst[r * S + s] = mode == 0 ? v * sc[r] : v / sc[r];
        }
}

extern "C" {

int emu_phx_create(int32_t device, emu_ctx** out) {
    (void)device;
    *out = new emu_ctx();
    return 0;
}

int emu_phx_destroy(emu_ctx* c) {
    delete c;
    return 0;
}

const char* emu_phx_last_error(const emu_ctx* c) { return c ? c->err.c_str() : "null"; }

const char* emu_phx_build_info(void) { return "phx-emu: host emulation of the phx C ABI (tests only)"; }

int emu_phx_set_problem(emu_ctx* c, const phx_problem_desc* d) {
    const int S = d->S, n = d->n, m = d->m, nnz = d->nnz, N = d->N, nvar = d->nvar;
    c->S = S; c->n = n; c->m = m; c->nnz = nnz; c->N = N; c->nvar = nvar; c->c_vary = d->c_vary;
    HostSetup& hs = c->hs;
    hs.rowptr.assign(d->rowptr, d->rowptr + m + 1);
    hs.colidx.assign(d->colidx, d->colidx + nnz);
    hs.kvar.assign(d->kvar, d->kvar + nnz);
    hs.Aconst.assign(d->Aconst, d->Aconst + nnz);
    hs.slot_col.assign(d->slot_col, d->slot_col + N);
    std::vector<double> vmax(std::max(nvar, 1), 0.0);
    for (int v = 0; v < nvar; ++v)
        for (int s = 0; s < S; ++s) vmax[v] = std::max(vmax[v], fabs(d->Avar[(size_t)v * S + s]));
    std::string e = build_setup(hs, n, m, nnz, N, nvar, vmax);
    if (!e.empty()) { c->err = e; return 1; }
    const int64_t cS = d->c_vary ? S : 1, bS = d->bnd_vary ? S : 1, rS = d->rhs_vary ? S : 1;
    c->Av.assign((size_t)nvar * S, 0.0);
    scale_rows(d->Avar, c->Av.data(), hs.vscale.data(), nvar, S, 0);
    c->cs.assign(n * cS, 0.0); scale_rows(d->c, c->cs.data(), hs.dc.data(), n, cS, 0);
    c->c_user.assign(d->c, d->c + n * cS);
    c->lbs.assign(n * bS, 0.0); scale_rows(d->lb, c->lbs.data(), hs.dc.data(), n, bS, 1);
    c->ubs.assign(n * bS, 0.0); scale_rows(d->ub, c->ubs.data(), hs.dc.data(), n, bS, 1);
    c->bls.assign(std::max<int64_t>(m * rS, 1), 0.0);
    c->bus.assign(std::max<int64_t>(m * rS, 1), 0.0);
    if (m) {
        scale_rows(d->bl, c->bls.data(), hs.dr.data(), m, rS, 0);
        scale_rows(d->bu, c->bus.data(), hs.dr.data(), m, rS, 0);
    }
    c->qN.assign((size_t)std::max(N, 1) * S, 0.0);
    c->pN.assign((size_t)std::max(N, 1) * S, 0.0);
    c->kN.assign(S, 0.0);
    Prob& P = c->P;
    P.S = S; P.n = n; P.m = m; P.nnz = nnz; P.N = N;
    P.rowptr = hs.rowptr.data(); P.colidx = hs.colidx.data(); P.colptr = hs.colptr.data();
    P.rowidx = hs.rowidx.data(); P.csc2csr = hs.csc2csr.data(); P.kvar = hs.kvar.data();
    P.Ac = hs.Acs.data(); P.Av = c->Av.data();
    P.c = SVec{c->cs.data(), d->c_vary ? S : 1, d->c_vary ? 1 : 0};
    P.lb = SVec{c->lbs.data(), d->bnd_vary ? S : 1, d->bnd_vary ? 1 : 0};
    P.ub = SVec{c->ubs.data(), d->bnd_vary ? S : 1, d->bnd_vary ? 1 : 0};
    P.bl = SVec{c->bls.data(), d->rhs_vary ? S : 1, d->rhs_vary ? 1 : 0};
    P.bu = SVec{c->bus.data(), d->rhs_vary ? S : 1, d->rhs_vary ? 1 : 0};
    P.dr = hs.dr.data(); P.dc = hs.dc.data(); P.col_slot = hs.col_slot.data(); P.slot_col = hs.slot_col.data();
    P.qN = c->qN.data(); P.pN = c->pN.data(); P.kN = c->kN.data();
    const size_t nS = (size_t)n * S, mS = (size_t)std::max(m, 1) * S;
    for (auto* v : {&c->x, &c->x0, &c->xT, &c->xb, &c->r1, &c->xp, &c->xfix}) v->assign(nS, 0.0);
    for (auto* v : {&c->y, &c->y0, &c->yT, &c->z, &c->t, &c->brhs}) v->assign(mS, 0.0);
    for (auto* v : {&c->omega, &c->eta, &c->r0, &c->rprev, &c->errv}) v->assign(S, 0.0);
    c->hk.assign(S, 0); c->status.assign(S, 0); c->iters.assign(S, 0); c->flags.assign(S, 0);
    c->L.assign((size_t)m * (m + 1) / 2 * S + 1, 0.0);
    c->F.assign(nS, 0); c->R.assign(mS, 0);
    State& St = c->St;
    St.x = c->x.data(); St.y = c->y.data(); St.x0 = c->x0.data(); St.y0 = c->y0.data();
    St.xT = c->xT.data(); St.yT = c->yT.data(); St.xb = c->xb.data();
    St.omega = c->omega.data(); St.eta = c->eta.data(); St.r0 = c->r0.data(); St.rprev = c->rprev.data();
    St.err = c->errv.data(); St.hk = c->hk.data(); St.status = c->status.data(); St.iters = c->iters.data();
    St.flags = c->flags.data();
    c->ipm_buf.assign((size_t)(8 * n + 9 * std::max(m, 1)) * S, 0.0);
    {
        double* b = c->ipm_buf.data();
        auto take = [&](size_t k) { double* r = b; b += k; return r; };
        Ipm& I = c->Iw;
        I.s = take(mS); I.zl = take(nS); I.zu = take(nS); I.wl = take(mS); I.wu = take(mS);
        I.dx = take(nS); I.dzl = take(nS); I.dzu = take(nS); I.cl = take(nS); I.cu = take(nS); I.hx = take(nS);
        I.ds = take(mS); I.dwl = take(mS); I.dwu = take(mS); I.dy = take(mS); I.cwl = take(mS); I.cwu = take(mS);
    }
    Polish& W = c->Pw;
    W.L = c->L.data(); W.z = c->z.data(); W.r1 = c->r1.data(); W.t = c->t.data(); W.xp = c->xp.data();
    W.xfix = c->xfix.data(); W.brhs = c->brhs.data(); W.F = c->F.data(); W.R = c->R.data();
    for (int s = 0; s < S; ++s) {
        const double nrm = spectral_norm(P, St, s, 100);
        St.eta[s] = 0.998 / (1.02 * nrm);
        St.omega[s] = 1.0;
        for (int j = 0; j < n; ++j) {
            const double v = clampd(0.0, P.lb.at(j, s), P.ub.at(j, s));
            St.x[ix(j, s, S)] = St.x0[ix(j, s, S)] = St.xT[ix(j, s, S)] = v;
        }
        for (int i = 0; i < m; ++i) St.y[ix(i, s, S)] = St.y0[ix(i, s, S)] = St.yT[ix(i, s, S)] = 0.0;
    }
    c->have = true;
    return 0;
}

int emu_phx_set_ph_terms(emu_ctx* c, const double* W, const double* rho, const double* xbar_node,
                         const int32_t* xbar_idx, int32_t W_on, int32_t prox_on, void*) {
    const int S = c->S;
    for (int s = 0; s < S; ++s) {
        double k = 0.0;
        for (int j = 0; j < c->N; ++j) {
            const int64_t o = ix(j, s, S);
            double q = 0.0, p = 0.0;
            if (W_on) q += W[o];
            if (prox_on) {
                const double r = rho[o], xb = xbar_node[xbar_idx[o]];
                q -= r * xb;
                p = r;
                k += 0.5 * r * xb * xb;
            }
            c->qN[o] = q;
            c->pN[o] = p;
        }
        c->kN[s] = k;
    }
    return 0;
}

int emu_phx_solve(emu_ctx* c, const phx_solve_opts* o, double* x_out, double* y_out, double* obj_out,
                  int32_t* status_out, int32_t* iters_out, int32_t* total_iters, void*) {
    const int S = c->S;
    const Prob& P = c->P;
    const State& St = c->St;
    Opts O;
    O.iters = o->check_every; O.restart_max = o->restart_max; O.polish_below = o->polish_below;
    O.opt_tol = o->opt_tol; O.kkt_tol = o->kkt_tol; O.reg = o->reg; O.refine_steps = o->refine_steps;
    O.polish = o->polish; O.max_iters = o->max_iters;
    O.ipm_after = o->ipm_after; O.ipm_max_it = o->ipm_max_it; O.ipm_tol = o->ipm_tol;
    const bool warm = o->warm_start && c->solved_once;
    for (int s = 0; s < S; ++s) {
        if (!warm) {
            for (int j = 0; j < P.n; ++j) {
                const double v = clampd(0.0, P.lb.at(j, s), P.ub.at(j, s));
                St.x[ix(j, s, S)] = St.x0[ix(j, s, S)] = St.xT[ix(j, s, S)] = v;
            }
            for (int i = 0; i < P.m; ++i) St.y[ix(i, s, S)] = St.y0[ix(i, s, S)] = St.yT[ix(i, s, S)] = 0.0;
        } else {
            for (int j = 0; j < P.n; ++j) St.x0[ix(j, s, S)] = St.x[ix(j, s, S)];
            for (int i = 0; i < P.m; ++i) St.y0[ix(i, s, S)] = St.y[ix(i, s, S)];
        }
        St.hk[s] = 0; St.r0[s] = 1e301; St.rprev[s] = 1e301; St.status[s] = RUNNING; St.iters[s] = 0;
        St.err[s] = 1e300;
        St.flags[s] = 0;
    }
    int total = 0, running = S;
    c->lane_iters = 0;
    c->launches = 0;
    while (running > 0 && total < o->max_iters) {
        c->lane_iters += (double)running * o->check_every;
        ++c->launches;
        running = 0;
        for (int s = 0; s < S; ++s) {
            if (St.status[s] != RUNNING) continue;
            if (O.ipm_after >= 0 && St.iters[s] >= O.ipm_after && !(St.flags[s] & 1)) {
                if (finish_lane(P, St, c->Pw, c->Iw, O, s)) { St.status[s] = OPTIMAL; continue; }
            }
            int hk = St.hk[s];
            const double tau = St.eta[s] / St.omega[s], sigma = St.eta[s] * St.omega[s];
            double dx2 = 0, dy2 = 0;
            for (int it = 0; it < O.iters; ++it) {
                pdhg_iter(P, St, s, hk, tau, sigma, it == O.iters - 1, dx2, dy2);
                ++hk;
            }
            St.hk[s] = hk;
            St.iters[s] += O.iters;
            check_and_restart(P, St, O, s, dx2, dy2);
            const double e = St.err[s];
            if (!O.polish && e < O.opt_tol) St.status[s] = OPTIMAL;
            if (!(e < 1e300)) St.status[s] = NUMERIC_FAIL;
            bool tried = false, okp = false;
            if (St.status[s] == RUNNING && O.polish && e < O.polish_below) {
                const double tol = fmin(1e-4, fmax(1e-9, 10.0 * e));
                tried = true;
                if (polish_lane(P, St, c->Pw, O, s, tol)) {
                    adopt_polished(P, St, c->Pw, s);
                    St.status[s] = OPTIMAL;
                    okp = true;
                }
            }
            static int trace_s = getenv("PHX_EMU_TRACE") ? atoi(getenv("PHX_EMU_TRACE")) : -1;
            if (s == trace_s)
                fprintf(stderr, "[emu s=%d] it=%d err=%.3e omega=%.3e hk=%d r0=%.3e polish=%s\n", s, St.iters[s], e,
                        St.omega[s], St.hk[s], St.r0[s], tried ? (okp ? "OK" : "fail") : "-");
            if (St.status[s] == RUNNING) {
                if (St.iters[s] >= O.max_iters) St.status[s] = ITER_LIMIT;
                else ++running;
            }
        }
        total += o->check_every;
    }
    const int64_t c_si = c->c_vary ? S : 1, c_ss = c->c_vary ? 1 : 0;
    for (int s = 0; s < S; ++s) {
        finalize_lane(P, St, c->c_user.data(), c_si, c_ss, s, x_out, y_out, obj_out);
        if (status_out) status_out[s] = St.status[s];
        if (iters_out) iters_out[s] = St.iters[s];
    }
    c->solved_once = true;
    if (total_iters) *total_iters = total;
    return 0;
}

int emu_phx_objective(emu_ctx* c, const double* x, double* obj, void*) {
    const int64_t c_si = c->c_vary ? c->S : 1, c_ss = c->c_vary ? 1 : 0;
    for (int s = 0; s < c->S; ++s) obj[s] = objective_lane(c->P, c->c_user.data(), c_si, c_ss, x, s);
    return 0;
}

int emu_phx_xbar(emu_ctx* c, const phx_tree_desc* T, const double* x, const double* pc, double* partial,
                 double* node_sums, void*) {
    const int S = c->S;
    for (int e = 0; e < 2 * T->NNS; ++e) node_sums[e] = 0.0;
    for (int t = 0; t < T->ntiles; ++t) {
        const int nl = T->tile_nlen[t];
        for (int l = 0; l < nl; ++l) {
            const int j = T->tile_slot[t] + l;
            const int col = c->hs.slot_col[j];
            double a = 0, a2 = 0;
            for (int s = T->tile_s0[t]; s < T->tile_s1[t]; ++s) {
                const double xv = x[ix(col, s, S)];
                const double v = pc[ix(j, s, S)] * xv;
                a += v;
                a2 += v * xv;
            }
            partial[T->tile_out[t] + l] = a;
            partial[T->tile_out[t] + nl + l] = a2;
        }
    }
    for (int v = 0; v < T->nnodes; ++v) {
        const int nl = T->node_nlen[v];
        for (int l = 0; l < nl; ++l) {
            double a = 0, a2 = 0;
            for (int t = T->node_tile_ptr[v]; t < T->node_tile_ptr[v + 1]; ++t) {
                a += partial[T->tile_out[t] + l];
                a2 += partial[T->tile_out[t] + nl + l];
            }
            node_sums[T->node_off[v] + l] = a;
            node_sums[T->NNS + T->node_off[v] + l] = a2;
        }
    }
    return 0;
}

int emu_phx_update_w(emu_ctx* c, const double* x, const double* xbar_node, const int32_t* xbar_idx,
                     const double* rho, double* W, int32_t update_w, double* dsum, int32_t nseg,
                     const int32_t* seg_s0, const int32_t* seg_s1, double* seg_sums, void*) {
    const int S = c->S;
    for (int s = 0; s < S; ++s) {
        double d = 0;
        for (int j = 0; j < c->N; ++j) {
            const int64_t o = ix(j, s, S);
            const double diff = x[ix(c->hs.slot_col[j], s, S)] - xbar_node[xbar_idx[o]];
            if (update_w) W[o] += rho[o] * diff;
            d += fabs(diff);
        }
        dsum[s] = d;
    }
    for (int g = 0; g < nseg; ++g) {
        double a = 0;
        for (int s = seg_s0[g]; s < seg_s1[g]; ++s) a += dsum[s];
        seg_sums[g] = a;
    }
    return 0;
}

int emu_phx_expect(emu_ctx* c, const double* prob, const double* obj, const int32_t* status, double* out,
                   void*) {
    double a = 0, b = 0, d = 0;
    for (int s = 0; s < c->S; ++s) {
        a += prob[s] * obj[s];
        b += prob[s];
        d += status[s] == OPTIMAL ? prob[s] : 0.0;
    }
    out[0] = a; out[1] = b; out[2] = d;
    return 0;
}

int emu_phx_export_slots(emu_ctx* c, const double* src, double* out, void*) {
    for (int j = 0; j < c->N; ++j)
        for (int s = 0; s < c->S; ++s) out[(int64_t)s * c->N + j] = src[(int64_t)j * c->S + s];
    return 0;
}

int emu_phx_last_solve_timing(const emu_ctx* c, double* ms, int32_t* launches, double* lane_iters,
                              double* pms, double* ims) {
    if (ims) *ims = 0;
    if (ms) *ms = 0;
    if (launches) *launches = c->launches;
    if (lane_iters) *lane_iters = c->lane_iters;
    if (pms) *pms = 0;
    return 0;
}

}  // extern "C"
