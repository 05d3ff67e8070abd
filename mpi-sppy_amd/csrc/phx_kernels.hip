// phx_kernels.hip — CDNA4 (gfx950) kernels + C ABI of the batched PH engine.
//
// Layout: one lane = one scenario; every per-scenario array is
// scenario-minor [i*S + s]; the sparsity pattern is shared and wave-uniform.
// Kernels:
//   k_chunk        `check_every` PDHG iterations + restart check per lane   (hot)
//   k_polish       active-set KKT polish + certificate per lane
//   k_finalize     unscaled x, y, objective per lane
//   k_ph_terms     qN/pN/kN from W, rho, xbar        (attach_PH_to_objective)
//   k_xbar_*       per-tree-node segmented reduction (Compute_Xbar)
//   k_update_w     W += rho (x - xbar), |x - xbar|   (Update_W, convergence_diff)
//   k_seg_*        deterministic segmented sums (conv per emulated rank)
//   k_expect       sum p*obj, sum p, sum p*feasible  (Eobjective/Ebound/E1/feas)
// All reductions are fixed-order trees (no float atomics), so results are
// bitwise reproducible run to run.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <math.h>
#include <string>
#include <vector>
#include <algorithm>
#include "../../include/phx.h"
#include "phx_core.h"
#include "phx_setup.h"

using namespace phx;

#define PHX_BLOCK 64   // lane-per-scenario kernels: one wavefront per block

// ------------------------------------------------------------------ kernels
// Lane lists: launches cover only still-running scenarios.  lanes[0..*count)
// holds scenario ids (ascending within a wavefront), rebuilt by k_polish.
__global__ __launch_bounds__(PHX_BLOCK) void k_chunk(Prob P, State St, Opts O, const int32_t* lanes,
                                                    const int32_t* count) {
    const int t = blockIdx.x * PHX_BLOCK + threadIdx.x;
    if (t >= *count) return;
    const int s = lanes[t];
    if (St.status[s] != RUNNING) return;
    int hk = St.hk[s];
    const double eta = St.eta[s];
    const double w = St.omega[s];
    const double tau = eta / w, sigma = eta * w;
    double dx2 = 0.0, dy2 = 0.0;
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
}

// Interior-point finisher for lanes that PDHG has not certified after
// O.ipm_after iterations (O.ipm_after = 0: IPM first), followed by the polish.
__global__ __launch_bounds__(PHX_BLOCK) void k_ipm(Prob P, State St, Polish W, Ipm I, Opts O,
                                                  const int32_t* lanes, const int32_t* count) {
    const int t = blockIdx.x * PHX_BLOCK + threadIdx.x;
    if (t >= *count) return;
    const int s = lanes[t];
    if (St.status[s] != RUNNING || St.iters[s] < O.ipm_after || (St.flags[s] & 1)) return;
    if (finish_lane(P, St, W, I, O, s)) St.status[s] = OPTIMAL;
}

__global__ __launch_bounds__(PHX_BLOCK) void k_polish(Prob P, State St, Polish W, Opts O,
                                                     const int32_t* lanes, const int32_t* count,
                                                     int32_t* lanes_out, int32_t* running) {
    const int t = blockIdx.x * PHX_BLOCK + threadIdx.x;
    const int s = t < *count ? lanes[t] : -1;
    bool still = false;
    if (s >= 0 && St.status[s] == RUNNING) {
        const double e = St.err[s];
        if (O.polish && e < O.polish_below) {
            const double tol = fmin(1e-4, fmax(1e-9, 10.0 * e));
            if (polish_lane(P, St, W, O, s, tol)) {
                adopt_polished(P, St, W, s);
                St.status[s] = OPTIMAL;
            }
        }
        if (St.status[s] == RUNNING) {
            if (St.iters[s] >= O.max_iters) St.status[s] = ITER_LIMIT;
            else still = true;
        }
    }
    // compact the still-running lanes: one atomic per wavefront, lane order kept
    const unsigned long long b = __ballot(still);
    const int lane = threadIdx.x & 63;
    int base = 0;
    if (lane == 0 && b) base = atomicAdd(running, (int32_t)__popcll(b));
    base = __shfl(base, 0, 64);
    if (still) {
        const unsigned long long below = b & ((1ull << lane) - 1ull);
        lanes_out[base + __popcll(below)] = s;
    }
}

__global__ void k_iota(int32_t* lanes, int32_t* count, int S) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < S) lanes[t] = t;
    if (t == 0) *count = S;
}

__global__ __launch_bounds__(PHX_BLOCK) void k_finalize(Prob P, State St, const double* c,
                                                       int64_t c_si, int64_t c_ss,
                                                       double* x_out, double* y_out,
                                                       double* obj_out, int32_t* status_out,
                                                       int32_t* iters_out) {
    const int s = blockIdx.x * PHX_BLOCK + threadIdx.x;
    if (s >= P.S) return;
    finalize_lane(P, St, c, c_si, c_ss, s, x_out, y_out, obj_out);
    if (status_out) status_out[s] = St.status[s];
    if (iters_out) iters_out[s] = St.iters[s];
}

__global__ __launch_bounds__(PHX_BLOCK) void k_objective(Prob P, const double* c, int64_t c_si,
                                                        int64_t c_ss, const double* x, double* obj) {
    const int s = blockIdx.x * PHX_BLOCK + threadIdx.x;
    if (s >= P.S) return;
    obj[s] = objective_lane(P, c, c_si, c_ss, x, s);
}

__global__ void k_begin_solve(Prob P, State St, int warm) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= P.S) return;
    const int S = P.S;
    if (!warm) {
        for (int j = 0; j < P.n; ++j) {
            const int64_t o = ix(j, s, S);
            const double v = clampd(0.0, P.lb.at(j, s), P.ub.at(j, s));
            St.x[o] = St.x0[o] = St.xT[o] = v;
        }
        for (int i = 0; i < P.m; ++i) {
            const int64_t o = ix(i, s, S);
            St.y[o] = St.y0[o] = St.yT[o] = 0.0;
        }
    } else {
        // restart the Halpern anchor at the warm-start point
        for (int j = 0; j < P.n; ++j) {
            const int64_t o = ix(j, s, S);
            St.x0[o] = St.x[o];
        }
        for (int i = 0; i < P.m; ++i) {
            const int64_t o = ix(i, s, S);
            St.y0[o] = St.y[o];
        }
    }
    St.hk[s] = 0;
    St.r0[s] = 1e301;
    St.rprev[s] = 1e301;
    St.status[s] = RUNNING;
    St.iters[s] = 0;
    St.err[s] = 1e300;
    St.flags[s] = 0;
}

__global__ void k_norm(Prob P, State St, int iters) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= P.S) return;
    const double nrm = spectral_norm(P, St, s, iters);
    St.eta[s] = 0.998 / (1.02 * nrm);
    St.omega[s] = 1.0;
}

// scaled copy of the varying A values: Av[v*S+s] = A[v*S+s] * vscale[v]
__global__ void k_scale_rows(const double* src, double* dst, const double* scale,
                             int64_t nrows, int64_t S, int mode) {
    // mode 0: dst = src*scale[row] ; mode 1: dst = src/scale[row]
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nrows * S) return;
    const int64_t r = t / S;
    const double v = src[t];
    dst[t] = mode == 0 ? v * scale[r] : v / scale[r];
}

__global__ void k_ph_terms(int N, int S, const double* W, const double* rho,
                           const double* xbar_node, const int32_t* xbar_idx, int W_on,
                           int prox_on, double* qN, double* pN, double* kN) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    double k = 0.0;
    for (int j = 0; j < N; ++j) {
        const int64_t o = ix(j, s, S);
        double q = 0.0, p = 0.0;
        if (W_on) q += W[o];
        if (prox_on) {
            const double r = rho[o];
            const double xb = xbar_node[xbar_idx[o]];
            q -= r * xb;
            p = r;
            k += 0.5 * r * xb * xb;
        }
        qN[o] = q;
        pN[o] = p;
    }
    kN[s] = k;
}

// ---- block reduction helpers (wave shuffles + LDS, fixed order) ----
template <int NT>
__device__ double block_sum(double v, double* sh) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) sh[wid] = v;
    __syncthreads();
    double r = 0.0;
    if (threadIdx.x == 0) {
        for (int w = 0; w < NT / 64; ++w) r += sh[w];
    }
    __syncthreads();
    return r;   // valid in thread 0
}

#define RED_NT 256
__global__ __launch_bounds__(RED_NT) void k_xbar_partial(
    int S, const int32_t* tile_s0, const int32_t* tile_s1, const int32_t* tile_slot,
    const int32_t* tile_nlen, const int32_t* tile_out, const int32_t* slot_col,
    const double* x, const double* pc, double* partial) {
    __shared__ double sh[RED_NT / 64];
    const int t = blockIdx.x;
    const int s0 = tile_s0[t], s1 = tile_s1[t], sl0 = tile_slot[t], nl = tile_nlen[t];
    const int out = tile_out[t];
    for (int l = 0; l < nl; ++l) {
        const int j = sl0 + l;
        const int col = slot_col[j];
        double a = 0.0, a2 = 0.0;
        for (int s = s0 + (int)threadIdx.x; s < s1; s += RED_NT) {
            const double xv = x[ix(col, s, S)];
            const double v = pc[ix(j, s, S)] * xv;
            a += v;
            a2 += v * xv;
        }
        const double ra = block_sum<RED_NT>(a, sh);
        const double ra2 = block_sum<RED_NT>(a2, sh);
        if (threadIdx.x == 0) {
            partial[out + l] = ra;
            partial[out + nl + l] = ra2;
        }
    }
}

__global__ void k_xbar_finish(int nnodes, const int32_t* node_tile_ptr, const int32_t* node_off,
                              const int32_t* node_nlen, const int32_t* tile_out, int NNS,
                              const double* partial, double* node_sums) {
    const int v = blockIdx.x;
    if (v >= nnodes) return;
    const int nl = node_nlen[v];
    for (int l = threadIdx.x; l < nl; l += blockDim.x) {
        double a = 0.0, a2 = 0.0;
        for (int t = node_tile_ptr[v]; t < node_tile_ptr[v + 1]; ++t) {
            a += partial[tile_out[t] + l];
            a2 += partial[tile_out[t] + nl + l];
        }
        node_sums[node_off[v] + l] = a;
        node_sums[NNS + node_off[v] + l] = a2;
    }
}

__global__ void k_zero(double* p, int64_t n) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) p[t] = 0.0;
}

__global__ void k_update_w(int N, int S, const int32_t* slot_col, const double* x,
                           const double* xbar_node, const int32_t* xbar_idx,
                           const double* rho, double* W, int update, double* dsum) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    double d = 0.0;
    for (int j = 0; j < N; ++j) {
        const int64_t o = ix(j, s, S);
        const double diff = x[ix(slot_col[j], s, S)] - xbar_node[xbar_idx[o]];
        if (update) W[o] += rho[o] * diff;
        d += fabs(diff);
    }
    dsum[s] = d;
}

// segmented sums of a [S] vector: tile t covers [s0,s1) of segment seg[t]
__global__ __launch_bounds__(RED_NT) void k_seg_partial(const double* v, const int32_t* ts0,
                                                        const int32_t* ts1, double* partial) {
    __shared__ double sh[RED_NT / 64];
    const int t = blockIdx.x;
    double a = 0.0;
    for (int s = ts0[t] + (int)threadIdx.x; s < ts1[t]; s += RED_NT) a += v[s];
    const double r = block_sum<RED_NT>(a, sh);
    if (threadIdx.x == 0) partial[t] = r;
}

__global__ void k_seg_finish(int nseg, const int32_t* seg_tile_ptr, const double* partial,
                             double* out) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nseg) return;
    double a = 0.0;
    for (int t = seg_tile_ptr[g]; t < seg_tile_ptr[g + 1]; ++t) a += partial[t];
    out[g] = a;
}

__global__ __launch_bounds__(1024) void k_expect(int S, const double* prob, const double* obj,
                                                 const int32_t* status, double* out) {
    __shared__ double sh[1024 / 64];
    double a = 0.0, b = 0.0, c = 0.0;
    for (int s = threadIdx.x; s < S; s += 1024) {
        const double p = prob[s];
        a += p * obj[s];
        b += p;
        c += (status[s] == OPTIMAL) ? p : 0.0;
    }
    const double ra = block_sum<1024>(a, sh);
    const double rb = block_sum<1024>(b, sh);
    const double rc = block_sum<1024>(c, sh);
    if (threadIdx.x == 0) { out[0] = ra; out[1] = rb; out[2] = rc; }
}

__global__ void k_export_slots(int N, int S, const double* src, double* out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)N * S) return;
    const int j = (int)(t / S), s = (int)(t % S);
    out[(int64_t)s * N + j] = src[t];
}

// ------------------------------------------------------------------ context
struct phx_ctx {
    int device = 0;
    std::string err;
    bool have_problem = false;
    // problem
    int S = 0, n = 0, m = 0, nnz = 0, N = 0, nvar = 0;
    int c_vary = 0, bnd_vary = 0, rhs_vary = 0;
    const double* c_user = nullptr;   // unscaled c (caller-owned)
    // owned device buffers
    std::vector<void*> owned;
    int32_t *colptr = nullptr, *rowidx = nullptr, *csc2csr = nullptr, *col_slot = nullptr;
    double *Ac = nullptr, *Av = nullptr, *cs = nullptr, *lbs = nullptr, *ubs = nullptr;
    double *bls = nullptr, *bus = nullptr, *dr = nullptr, *dc = nullptr;
    double *qN = nullptr, *pN = nullptr, *kN = nullptr;
    int32_t* running = nullptr;
    int32_t* lanesA = nullptr;
    int32_t* lanesB = nullptr;
    int32_t* countA = nullptr;
    int32_t* running_host = nullptr;
    Prob P{};
    State St{};
    Polish Pw{};
    Ipm Iw{};
    bool have_ipm = false;
    // tree/seg caches
    std::vector<int32_t> seg_s0_cache, seg_s1_cache;
    int32_t *seg_ts0 = nullptr, *seg_ts1 = nullptr, *seg_ptr = nullptr;
    double* seg_part = nullptr;
    int seg_ntiles = 0;
    // timing
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr, ev3 = nullptr, ev4 = nullptr;
    double last_ipm_ms = 0.0;
    double last_pdhg_ms = 0.0, last_polish_ms = 0.0;
    int32_t last_launches = 0;
    double last_lane_iters = 0.0;
    bool solved_once = false;
    ~phx_ctx() {
        for (void* p : owned) (void)hipFree(p);
        if (running_host) (void)hipHostFree(running_host);
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
        if (ev2) (void)hipEventDestroy(ev2);
        if (ev3) (void)hipEventDestroy(ev3);
        if (ev4) (void)hipEventDestroy(ev4);
    }
    template <class T> T* alloc(size_t count) {
        void* p = nullptr;
        if (count == 0) count = 1;
        if (hipMalloc(&p, count * sizeof(T)) != hipSuccess) return nullptr;
        owned.push_back(p);
        return (T*)p;
    }
};

#define PHX_CHECK(ctx, expr)                                                      \
    do {                                                                          \
        hipError_t _e = (expr);                                                   \
        if (_e != hipSuccess) {                                                   \
            (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(_e);       \
            return 1;                                                             \
        }                                                                         \
    } while (0)

#define PHX_REQUIRE(ctx, cond, msg)                                               \
    do {                                                                          \
        if (!(cond)) { (ctx)->err = (msg); return 1; }                            \
    } while (0)

static inline unsigned nblk(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

extern "C" {

const char* phx_build_info(void) {
    return "phx: gfx950 HIP kernels, fp64 lane-per-scenario PDHG + KKT polish";
}

int phx_create(int32_t device, phx_ctx** out) {
    if (!out) return 1;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= device) return 2;
    if (hipSetDevice(device) != hipSuccess) return 3;
    phx_ctx* c = new phx_ctx();
    c->device = device;
    if (hipHostMalloc((void**)&c->running_host, sizeof(int32_t)) != hipSuccess) { delete c; return 4; }
    (void)hipEventCreate(&c->ev0);
    (void)hipEventCreate(&c->ev1);
    (void)hipEventCreate(&c->ev2);
    (void)hipEventCreate(&c->ev3);
    (void)hipEventCreate(&c->ev4);
    *out = c;
    return 0;
}

int phx_destroy(phx_ctx* ctx) {
    if (!ctx) return 0;
    (void)hipSetDevice(ctx->device);
    (void)hipDeviceSynchronize();
    delete ctx;
    return 0;
}

const char* phx_last_error(const phx_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int phx_set_problem(phx_ctx* ctx, const phx_problem_desc* d) {
    PHX_REQUIRE(ctx, ctx && d, "null argument");
    PHX_CHECK(ctx, hipSetDevice(ctx->device));
    PHX_REQUIRE(ctx, !ctx->have_problem, "phx_set_problem: problem already set (create a new context)");
    PHX_REQUIRE(ctx, d->S > 0 && d->n > 0 && d->m >= 0 && d->nnz >= 0 && d->N >= 0,
                "phx_set_problem: bad sizes");
    const int S = d->S, n = d->n, m = d->m, nnz = d->nnz, N = d->N, nvar = d->nvar;
    ctx->S = S; ctx->n = n; ctx->m = m; ctx->nnz = nnz; ctx->N = N; ctx->nvar = nvar;
    ctx->c_vary = d->c_vary; ctx->bnd_vary = d->bnd_vary; ctx->rhs_vary = d->rhs_vary;
    // ---- pattern to host; CSC view + scaling (phx_setup.h) ----
    HostSetup hs;
    hs.rowptr.resize(m + 1); hs.colidx.resize(nnz); hs.kvar.resize(nnz); hs.slot_col.resize(N);
    hs.Aconst.resize(nnz);
    PHX_CHECK(ctx, hipMemcpy(hs.rowptr.data(), d->rowptr, sizeof(int32_t) * (m + 1), hipMemcpyDeviceToHost));
    if (nnz) {
        PHX_CHECK(ctx, hipMemcpy(hs.colidx.data(), d->colidx, sizeof(int32_t) * nnz, hipMemcpyDeviceToHost));
        PHX_CHECK(ctx, hipMemcpy(hs.kvar.data(), d->kvar, sizeof(int32_t) * nnz, hipMemcpyDeviceToHost));
        PHX_CHECK(ctx, hipMemcpy(hs.Aconst.data(), d->Aconst, sizeof(double) * nnz, hipMemcpyDeviceToHost));
    }
    if (N) PHX_CHECK(ctx, hipMemcpy(hs.slot_col.data(), d->slot_col, sizeof(int32_t) * N, hipMemcpyDeviceToHost));
    std::vector<double> vmax(std::max(nvar, 1), 0.0);
    if (nvar > 0) {
        std::vector<double> Avh((size_t)nvar * S);
        PHX_CHECK(ctx, hipMemcpy(Avh.data(), d->Avar, sizeof(double) * Avh.size(), hipMemcpyDeviceToHost));
        for (int v = 0; v < nvar; ++v) {
            double mx = 0.0;
            const double* r = Avh.data() + (size_t)v * S;
            for (int s = 0; s < S; ++s) mx = std::max(mx, fabs(r[s]));
            vmax[v] = mx;
        }
    }
    {
        const std::string e = build_setup(hs, n, m, nnz, N, nvar, vmax);
        PHX_REQUIRE(ctx, e.empty(), "phx_set_problem: " + e);
    }
    const auto& rowptr = hs.rowptr; const auto& colidx = hs.colidx; const auto& kvar = hs.kvar;
    const auto& slot_col = hs.slot_col; const auto& colptr = hs.colptr; const auto& rowidx = hs.rowidx;
    const auto& csc2csr = hs.csc2csr; const auto& col_slot = hs.col_slot; const auto& dr = hs.dr;
    const auto& dc = hs.dc; const auto& Acs = hs.Acs; const auto& vscale = hs.vscale;
    // ---- device copies ----
    ctx->colptr = ctx->alloc<int32_t>(n + 1);
    ctx->rowidx = ctx->alloc<int32_t>(nnz);
    ctx->csc2csr = ctx->alloc<int32_t>(nnz);
    ctx->col_slot = ctx->alloc<int32_t>(n);
    ctx->Ac = ctx->alloc<double>(nnz);
    ctx->Av = ctx->alloc<double>((size_t)nvar * S);
    ctx->dr = ctx->alloc<double>(m);
    ctx->dc = ctx->alloc<double>(n);
    double* vsc = ctx->alloc<double>(std::max(nvar, 1));
    const int64_t cS = d->c_vary ? S : 1, bS = d->bnd_vary ? S : 1, rS = d->rhs_vary ? S : 1;
    ctx->cs = ctx->alloc<double>((size_t)n * cS);
    ctx->lbs = ctx->alloc<double>((size_t)n * bS);
    ctx->ubs = ctx->alloc<double>((size_t)n * bS);
    ctx->bls = ctx->alloc<double>((size_t)m * rS);
    ctx->bus = ctx->alloc<double>((size_t)m * rS);
    ctx->qN = ctx->alloc<double>((size_t)N * S);
    ctx->pN = ctx->alloc<double>((size_t)N * S);
    ctx->kN = ctx->alloc<double>(S);
    ctx->running = ctx->alloc<int32_t>(1);
    ctx->lanesA = ctx->alloc<int32_t>(S);
    ctx->lanesB = ctx->alloc<int32_t>(S);
    ctx->countA = ctx->alloc<int32_t>(1);
    PHX_REQUIRE(ctx, ctx->running && ctx->kN && ctx->bus, "phx_set_problem: out of device memory");
    PHX_CHECK(ctx, hipMemcpy(ctx->colptr, colptr.data(), sizeof(int32_t) * (n + 1), hipMemcpyHostToDevice));
    if (nnz) {
        PHX_CHECK(ctx, hipMemcpy(ctx->rowidx, rowidx.data(), sizeof(int32_t) * nnz, hipMemcpyHostToDevice));
        PHX_CHECK(ctx, hipMemcpy(ctx->csc2csr, csc2csr.data(), sizeof(int32_t) * nnz, hipMemcpyHostToDevice));
        PHX_CHECK(ctx, hipMemcpy(ctx->Ac, Acs.data(), sizeof(double) * nnz, hipMemcpyHostToDevice));
    }
    PHX_CHECK(ctx, hipMemcpy(ctx->col_slot, col_slot.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice));
    if (m) PHX_CHECK(ctx, hipMemcpy(ctx->dr, dr.data(), sizeof(double) * m, hipMemcpyHostToDevice));
    PHX_CHECK(ctx, hipMemcpy(ctx->dc, dc.data(), sizeof(double) * n, hipMemcpyHostToDevice));
    PHX_CHECK(ctx, hipMemcpy(vsc, vscale.data(), sizeof(double) * vscale.size(), hipMemcpyHostToDevice));
    const int TB = 256;
    if (nvar)
        hipLaunchKernelGGL(k_scale_rows, dim3(nblk((int64_t)nvar * S, TB)), dim3(TB), 0, 0,
                           d->Avar, ctx->Av, vsc, (int64_t)nvar, (int64_t)S, 0);
    // c~ = dc*c ; l~ = l/dc ; bl~ = dr*bl  (rows of length S if varying, else 1)
    hipLaunchKernelGGL(k_scale_rows, dim3(nblk((int64_t)n * cS, TB)), dim3(TB), 0, 0,
                       d->c, ctx->cs, ctx->dc, (int64_t)n, cS, 0);
    hipLaunchKernelGGL(k_scale_rows, dim3(nblk((int64_t)n * bS, TB)), dim3(TB), 0, 0,
                       d->lb, ctx->lbs, ctx->dc, (int64_t)n, bS, 1);
    hipLaunchKernelGGL(k_scale_rows, dim3(nblk((int64_t)n * bS, TB)), dim3(TB), 0, 0,
                       d->ub, ctx->ubs, ctx->dc, (int64_t)n, bS, 1);
    if (m) {
        hipLaunchKernelGGL(k_scale_rows, dim3(nblk((int64_t)m * rS, TB)), dim3(TB), 0, 0,
                           d->bl, ctx->bls, ctx->dr, (int64_t)m, rS, 0);
        hipLaunchKernelGGL(k_scale_rows, dim3(nblk((int64_t)m * rS, TB)), dim3(TB), 0, 0,
                           d->bu, ctx->bus, ctx->dr, (int64_t)m, rS, 0);
    }
    PHX_CHECK(ctx, hipGetLastError());
    PHX_CHECK(ctx, hipMemset(ctx->qN, 0, sizeof(double) * (size_t)N * S));
    PHX_CHECK(ctx, hipMemset(ctx->pN, 0, sizeof(double) * (size_t)N * S));
    PHX_CHECK(ctx, hipMemset(ctx->kN, 0, sizeof(double) * S));
    // ---- Prob ----
    Prob& P = ctx->P;
    P.S = S; P.n = n; P.m = m; P.nnz = nnz; P.N = N;
    {
        int32_t* rp = ctx->alloc<int32_t>(m + 1);
        int32_t* ci = ctx->alloc<int32_t>(nnz);
        int32_t* kv = ctx->alloc<int32_t>(nnz);
        int32_t* sc = ctx->alloc<int32_t>(N);
        double* cu = ctx->alloc<double>((size_t)n * cS);
        PHX_REQUIRE(ctx, rp && ci && kv && sc && cu, "phx_set_problem: out of device memory");
        PHX_CHECK(ctx, hipMemcpy(rp, rowptr.data(), sizeof(int32_t) * (m + 1), hipMemcpyHostToDevice));
        if (nnz) {
            PHX_CHECK(ctx, hipMemcpy(ci, colidx.data(), sizeof(int32_t) * nnz, hipMemcpyHostToDevice));
            PHX_CHECK(ctx, hipMemcpy(kv, kvar.data(), sizeof(int32_t) * nnz, hipMemcpyHostToDevice));
        }
        if (N) PHX_CHECK(ctx, hipMemcpy(sc, slot_col.data(), sizeof(int32_t) * N, hipMemcpyHostToDevice));
        PHX_CHECK(ctx, hipMemcpy(cu, d->c, sizeof(double) * (size_t)n * cS, hipMemcpyDeviceToDevice));
        P.rowptr = rp; P.colidx = ci; P.kvar = kv; P.slot_col = sc;
        ctx->c_user = cu;
    }
    P.colptr = ctx->colptr; P.rowidx = ctx->rowidx; P.csc2csr = ctx->csc2csr;
    P.Ac = ctx->Ac; P.Av = ctx->Av;
    P.c = SVec{ctx->cs, d->c_vary ? S : 1, d->c_vary ? 1 : 0};
    P.lb = SVec{ctx->lbs, d->bnd_vary ? S : 1, d->bnd_vary ? 1 : 0};
    P.ub = SVec{ctx->ubs, d->bnd_vary ? S : 1, d->bnd_vary ? 1 : 0};
    P.bl = SVec{ctx->bls, d->rhs_vary ? S : 1, d->rhs_vary ? 1 : 0};
    P.bu = SVec{ctx->bus, d->rhs_vary ? S : 1, d->rhs_vary ? 1 : 0};
    P.dr = ctx->dr; P.dc = ctx->dc;
    P.col_slot = ctx->col_slot;
    P.qN = ctx->qN; P.pN = ctx->pN; P.kN = ctx->kN;
    // ---- state + polish workspace ----
    State& St = ctx->St;
    const size_t nS = (size_t)n * S, mS = (size_t)std::max(m, 1) * S;
    St.x = ctx->alloc<double>(nS); St.x0 = ctx->alloc<double>(nS); St.xT = ctx->alloc<double>(nS);
    St.xb = ctx->alloc<double>(nS);
    St.y = ctx->alloc<double>(mS); St.y0 = ctx->alloc<double>(mS); St.yT = ctx->alloc<double>(mS);
    St.omega = ctx->alloc<double>(S); St.eta = ctx->alloc<double>(S); St.r0 = ctx->alloc<double>(S);
    St.rprev = ctx->alloc<double>(S); St.err = ctx->alloc<double>(S);
    St.hk = ctx->alloc<int32_t>(S); St.status = ctx->alloc<int32_t>(S); St.iters = ctx->alloc<int32_t>(S);
    St.flags = ctx->alloc<int32_t>(S);
    Polish& W = ctx->Pw;
    W.L = ctx->alloc<double>((size_t)m * (m + 1) / 2 * S);
    W.z = ctx->alloc<double>(mS); W.r1 = ctx->alloc<double>(nS); W.t = ctx->alloc<double>(mS);
    W.xp = ctx->alloc<double>(nS); W.xfix = ctx->alloc<double>(nS); W.brhs = ctx->alloc<double>(mS);
    W.F = ctx->alloc<unsigned char>(nS); W.R = ctx->alloc<unsigned char>(mS);
    PHX_REQUIRE(ctx, St.x && St.iters && St.flags && W.L && W.R, "phx_set_problem: out of device memory (state)");
    {
        Ipm& I = ctx->Iw;
        I.s = ctx->alloc<double>(mS); I.zl = ctx->alloc<double>(nS); I.zu = ctx->alloc<double>(nS);
        I.wl = ctx->alloc<double>(mS); I.wu = ctx->alloc<double>(mS);
        I.dx = ctx->alloc<double>(nS); I.dzl = ctx->alloc<double>(nS); I.dzu = ctx->alloc<double>(nS);
        I.cl = ctx->alloc<double>(nS); I.cu = ctx->alloc<double>(nS); I.hx = ctx->alloc<double>(nS);
        I.ds = ctx->alloc<double>(mS); I.dwl = ctx->alloc<double>(mS); I.dwu = ctx->alloc<double>(mS);
        I.dy = ctx->alloc<double>(mS); I.cwl = ctx->alloc<double>(mS); I.cwu = ctx->alloc<double>(mS);
        ctx->have_ipm = I.cwu != nullptr;
        PHX_REQUIRE(ctx, ctx->have_ipm, "phx_set_problem: out of device memory (ipm)");
    }
    hipLaunchKernelGGL(k_norm, dim3(nblk(S, PHX_BLOCK)), dim3(PHX_BLOCK), 0, 0, P, St, 100);
    hipLaunchKernelGGL(k_begin_solve, dim3(nblk(S, PHX_BLOCK)), dim3(PHX_BLOCK), 0, 0, P, St, 0);
    PHX_CHECK(ctx, hipGetLastError());
    PHX_CHECK(ctx, hipDeviceSynchronize());
    ctx->have_problem = true;
    return 0;
}

int phx_set_ph_terms(phx_ctx* ctx, const double* W, const double* rho, const double* xbar_node,
                     const int32_t* xbar_idx, int32_t W_on, int32_t prox_on, void* stream) {
    PHX_REQUIRE(ctx, ctx && ctx->have_problem, "phx_set_ph_terms: no problem set");
    PHX_REQUIRE(ctx, !(W_on && !W), "phx_set_ph_terms: W_on without W");
    PHX_REQUIRE(ctx, !(prox_on && (!rho || !xbar_node || !xbar_idx)), "phx_set_ph_terms: prox_on without rho/xbar");
    hipStream_t st = (hipStream_t)stream;
    if (ctx->N == 0) return 0;
    hipLaunchKernelGGL(k_ph_terms, dim3(nblk(ctx->S, 256)), dim3(256), 0, st, ctx->N, ctx->S, W, rho,
                       xbar_node, xbar_idx, (int)W_on, (int)prox_on, ctx->qN, ctx->pN, ctx->kN);
    PHX_CHECK(ctx, hipGetLastError());
    return 0;
}

int phx_solve(phx_ctx* ctx, const phx_solve_opts* o, double* x_out, double* y_out, double* obj_out,
              int32_t* status_out, int32_t* iters_out, int32_t* total_iters_host, void* stream) {
    PHX_REQUIRE(ctx, ctx && ctx->have_problem && o, "phx_solve: no problem set");
    PHX_REQUIRE(ctx, x_out && obj_out, "phx_solve: x_out/obj_out required");
    PHX_REQUIRE(ctx, o->check_every > 0 && o->max_iters > 0, "phx_solve: bad options");
    PHX_CHECK(ctx, hipSetDevice(ctx->device));
    hipStream_t st = (hipStream_t)stream;
    const int S = ctx->S;
    const unsigned G = nblk(S, PHX_BLOCK);
    Opts O;
    O.iters = o->check_every;
    O.restart_max = o->restart_max;
    O.polish_below = o->polish_below;
    O.opt_tol = o->opt_tol;
    O.kkt_tol = o->kkt_tol;
    O.reg = o->reg;
    O.refine_steps = o->refine_steps;
    O.polish = o->polish;
    O.max_iters = o->max_iters;
    O.ipm_after = o->ipm_after;
    O.ipm_max_it = o->ipm_max_it;
    O.ipm_tol = o->ipm_tol;
    const int warm = (o->warm_start && ctx->solved_once) ? 1 : 0;
    hipLaunchKernelGGL(k_begin_solve, dim3(G), dim3(PHX_BLOCK), 0, st, ctx->P, ctx->St, warm);
    PHX_CHECK(ctx, hipGetLastError());
    int total = 0;
    int running = S;
    bool ipm_done = false, ipm_launched = false;
    double pdhg_ms = 0.0, polish_ms = 0.0, lane_iters = 0.0, ipm_ms = 0.0;
    int launches = 0;
    hipLaunchKernelGGL(k_iota, dim3(nblk(S, 256)), dim3(256), 0, st, ctx->lanesA, ctx->countA, S);
    int32_t* lin = ctx->lanesA;
    int32_t* lout = ctx->lanesB;
    int32_t* cin = ctx->countA;
    int32_t* cout = ctx->running;
    while (running > 0 && total < o->max_iters) {
        const unsigned Gr = nblk(running, PHX_BLOCK);
        PHX_CHECK(ctx, hipMemsetAsync(cout, 0, sizeof(int32_t), st));
        if (O.ipm_after >= 0 && total >= O.ipm_after && !ipm_done) {
            PHX_CHECK(ctx, hipEventRecord(ctx->ev3, st));
            hipLaunchKernelGGL(k_ipm, dim3(Gr), dim3(PHX_BLOCK), 0, st, ctx->P, ctx->St, ctx->Pw, ctx->Iw, O,
                               lin, cin);
            PHX_CHECK(ctx, hipEventRecord(ctx->ev4, st));
            ipm_done = true;
            ipm_launched = true;
        }
        PHX_CHECK(ctx, hipEventRecord(ctx->ev0, st));
        hipLaunchKernelGGL(k_chunk, dim3(Gr), dim3(PHX_BLOCK), 0, st, ctx->P, ctx->St, O, lin, cin);
        PHX_CHECK(ctx, hipEventRecord(ctx->ev1, st));
        hipLaunchKernelGGL(k_polish, dim3(Gr), dim3(PHX_BLOCK), 0, st, ctx->P, ctx->St, ctx->Pw, O, lin, cin,
                           lout, cout);
        PHX_CHECK(ctx, hipEventRecord(ctx->ev2, st));
        PHX_CHECK(ctx, hipGetLastError());
        PHX_CHECK(ctx, hipMemcpyAsync(ctx->running_host, cout, sizeof(int32_t), hipMemcpyDeviceToHost, st));
        PHX_CHECK(ctx, hipStreamSynchronize(st));
        float a = 0.f, b = 0.f, c = 0.f;
        (void)hipEventElapsedTime(&a, ctx->ev0, ctx->ev1);
        (void)hipEventElapsedTime(&b, ctx->ev1, ctx->ev2);
        if (ipm_launched) {
            (void)hipEventElapsedTime(&c, ctx->ev3, ctx->ev4);
            ipm_ms += c;
            ipm_launched = false;
        }
        pdhg_ms += a;
        polish_ms += b;
        lane_iters += (double)running * o->check_every;
        ++launches;
        total += o->check_every;
        running = *ctx->running_host;
        std::swap(lin, lout);
        std::swap(cin, cout);
    }
    const int64_t c_si = ctx->c_vary ? S : 1, c_ss = ctx->c_vary ? 1 : 0;
    hipLaunchKernelGGL(k_finalize, dim3(G), dim3(PHX_BLOCK), 0, st, ctx->P, ctx->St, ctx->c_user, c_si,
                       c_ss, x_out, y_out, obj_out, status_out, iters_out);
    PHX_CHECK(ctx, hipGetLastError());
    ctx->solved_once = true;
    ctx->last_pdhg_ms = pdhg_ms;
    ctx->last_polish_ms = polish_ms;
    ctx->last_launches = launches;
    ctx->last_lane_iters = lane_iters;
    ctx->last_ipm_ms = ipm_ms;
    if (total_iters_host) *total_iters_host = total;
    return 0;
}

int phx_objective(phx_ctx* ctx, const double* x, double* obj_out, void* stream) {
    PHX_REQUIRE(ctx, ctx && ctx->have_problem, "phx_objective: no problem set");
    const int S = ctx->S;
    const int64_t c_si = ctx->c_vary ? S : 1, c_ss = ctx->c_vary ? 1 : 0;
    hipLaunchKernelGGL(k_objective, dim3(nblk(S, PHX_BLOCK)), dim3(PHX_BLOCK), 0, (hipStream_t)stream,
                       ctx->P, ctx->c_user, c_si, c_ss, x, obj_out);
    PHX_CHECK(ctx, hipGetLastError());
    return 0;
}

int phx_xbar(phx_ctx* ctx, const phx_tree_desc* T, const double* x, const double* prob_coeff,
             double* partial, double* node_sums, void* stream) {
    PHX_REQUIRE(ctx, ctx && ctx->have_problem && T, "phx_xbar: no problem set");
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_zero, dim3(nblk(2 * (int64_t)T->NNS, 256)), dim3(256), 0, st, node_sums,
                       2 * (int64_t)T->NNS);
    if (T->ntiles > 0) {
        hipLaunchKernelGGL(k_xbar_partial, dim3(T->ntiles), dim3(RED_NT), 0, st, ctx->S, T->tile_s0,
                           T->tile_s1, T->tile_slot, T->tile_nlen, T->tile_out, ctx->P.slot_col, x,
                           prob_coeff, partial);
        hipLaunchKernelGGL(k_xbar_finish, dim3(T->nnodes), dim3(64), 0, st, T->nnodes, T->node_tile_ptr,
                           T->node_off, T->node_nlen, T->tile_out, T->NNS, partial, node_sums);
    }
    PHX_CHECK(ctx, hipGetLastError());
    return 0;
}

int phx_update_w(phx_ctx* ctx, const double* x, const double* xbar_node, const int32_t* xbar_idx,
                 const double* rho, double* W, int32_t update_w, double* dsum, int32_t nseg,
                 const int32_t* seg_s0, const int32_t* seg_s1, double* seg_sums, void* stream) {
    PHX_REQUIRE(ctx, ctx && ctx->have_problem, "phx_update_w: no problem set");
    PHX_REQUIRE(ctx, !(update_w && (!W || !rho)), "phx_update_w: W/rho required");
    hipStream_t st = (hipStream_t)stream;
    const int S = ctx->S;
    hipLaunchKernelGGL(k_update_w, dim3(nblk(S, 256)), dim3(256), 0, st, ctx->N, S, ctx->P.slot_col, x,
                       xbar_node, xbar_idx, rho, W, (int)update_w, dsum);
    PHX_CHECK(ctx, hipGetLastError());
    if (nseg > 0 && seg_sums) {
        std::vector<int32_t> a(seg_s0, seg_s0 + nseg), b(seg_s1, seg_s1 + nseg);
        if (a != ctx->seg_s0_cache || b != ctx->seg_s1_cache) {
            for (int g = 0; g < nseg; ++g)
                PHX_REQUIRE(ctx, a[g] >= 0 && b[g] <= S && a[g] <= b[g], "phx_update_w: bad segment");
            std::vector<int32_t> ts0, ts1, ptr;
            build_seg_tiles(a, b, 8192, ts0, ts1, ptr);
            const int nt = (int)ts0.size();
            ctx->seg_ts0 = ctx->alloc<int32_t>(nt);
            ctx->seg_ts1 = ctx->alloc<int32_t>(nt);
            ctx->seg_ptr = ctx->alloc<int32_t>(nseg + 1);
            ctx->seg_part = ctx->alloc<double>(nt);
            if (nt) {
                PHX_CHECK(ctx, hipMemcpy(ctx->seg_ts0, ts0.data(), 4 * nt, hipMemcpyHostToDevice));
                PHX_CHECK(ctx, hipMemcpy(ctx->seg_ts1, ts1.data(), 4 * nt, hipMemcpyHostToDevice));
            }
            PHX_CHECK(ctx, hipMemcpy(ctx->seg_ptr, ptr.data(), 4 * (nseg + 1), hipMemcpyHostToDevice));
            ctx->seg_ntiles = nt;
            ctx->seg_s0_cache = a;
            ctx->seg_s1_cache = b;
        }
        if (ctx->seg_ntiles > 0)
            hipLaunchKernelGGL(k_seg_partial, dim3(ctx->seg_ntiles), dim3(RED_NT), 0, st, dsum, ctx->seg_ts0,
                               ctx->seg_ts1, ctx->seg_part);
        hipLaunchKernelGGL(k_seg_finish, dim3(nblk(nseg, 64)), dim3(64), 0, st, nseg, ctx->seg_ptr,
                           ctx->seg_part, seg_sums);
        PHX_CHECK(ctx, hipGetLastError());
    }
    return 0;
}

int phx_expect(phx_ctx* ctx, const double* prob, const double* obj, const int32_t* status, double* out,
               void* stream) {
    PHX_REQUIRE(ctx, ctx && ctx->have_problem, "phx_expect: no problem set");
    hipLaunchKernelGGL(k_expect, dim3(1), dim3(1024), 0, (hipStream_t)stream, ctx->S, prob, obj, status, out);
    PHX_CHECK(ctx, hipGetLastError());
    return 0;
}

int phx_export_slots(phx_ctx* ctx, const double* src, double* out, void* stream) {
    PHX_REQUIRE(ctx, ctx && ctx->have_problem, "phx_export_slots: no problem set");
    const int64_t tot = (int64_t)ctx->N * ctx->S;
    if (tot == 0) return 0;
    hipLaunchKernelGGL(k_export_slots, dim3(nblk(tot, 256)), dim3(256), 0, (hipStream_t)stream, ctx->N,
                       ctx->S, src, out);
    PHX_CHECK(ctx, hipGetLastError());
    return 0;
}

int phx_last_solve_timing(const phx_ctx* ctx, double* pdhg_ms, int32_t* launches, double* lane_iters,
                          double* polish_ms, double* ipm_ms) {
    if (!ctx) return 1;
    if (pdhg_ms) *pdhg_ms = ctx->last_pdhg_ms;
    if (launches) *launches = ctx->last_launches;
    if (lane_iters) *lane_iters = ctx->last_lane_iters;
    if (polish_ms) *polish_ms = ctx->last_polish_ms;
    if (ipm_ms) *ipm_ms = ctx->last_ipm_ms;
    return 0;
}

}  // extern "C"
