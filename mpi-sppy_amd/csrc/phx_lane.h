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
// phx_set_problem); only scenario-varying values occupy vector registers.  The
// same templates compile on the host with a runtime pattern (tests/emu), which
// is how the CPU suite checks them.
//
// Two kernels per solve (phx_jit.h emits both):
//   phx_lane_warm   active-set solve seeded with the lane's active set of the
//                   previous solve (PH subproblems change little from one PH
//                   iteration to the next): equality-constrained KKT solve ->
//                   certificate -> primal-dual active-set update, a few rounds.
//   phx_lane_cold   Mehrotra predictor-corrector IPM on
//                      min 0.5 x'Px + q'x  s.t. Ax - s = 0, l <= x <= u,
//                      bl <= s <= bu
//                   (normal matrix M = A (P+Sx)^-1 A' + Ss^-1, packed Cholesky
//                   with dependent-pivot replacement), then the active set read
//                   off the IPM point (slack vs multiplier, sharp by strict
//                   complementarity) and the same KKT/certificate/active-set
//                   rounds.  Runs on the lanes the warm kernel did not certify
//                   (all lanes on a first solve).
// A certified lane writes its unscaled solution, row duals and objective
// straight to the caller's outputs and stores its active set for the next
// solve.  Lanes that fail the certificate continue on the generic PDHG path
// (phx_core.h) from the IPM point.
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
typedef unsigned int uint32_t;
typedef unsigned long long uint64_t;
#endif

#if defined(__HIPCC__) || defined(__HIPCC_RTC__)
#define PHX_LD __host__ __device__ __forceinline__
#define PHX_UNROLL _Pragma("unroll")
#define PHX_NOUNROLL _Pragma("nounroll")
#else
#define PHX_LD inline
#define PHX_UNROLL
#define PHX_NOUNROLL
#endif
// The interior point's predictor / corrector passes, unrolled: the
// predictor's complementarity terms fold (no shift, no second-order term) --
// 17 % fewer VALU instructions per interior-point iteration on farmer, 44 ->
// 28 B of scratch (offline ISA, r04).  PHX_IPM_PASS_ROLLED keeps the loop.
#ifdef PHX_IPM_PASS_ROLLED
#define PHX_IPM_PASS_LOOP PHX_NOUNROLL
#else
#define PHX_IPM_PASS_LOOP PHX_UNROLL
#endif
// Refinement loop: kept as a loop by default (the fully unrolled refinement
// multiplies the straight-line code the instruction cache must stream).
#ifdef PHX_REFINE_UNROLL
#define PHX_REFINE_LOOP PHX_UNROLL
#else
#define PHX_REFINE_LOOP PHX_NOUNROLL
#endif
// The refinement carries its column residual from step to step (kkt_refine's
// CARRY) in every kernel but the two-wave fused build; PHX_REFINE_RECOMPUTE
// recomputes it everywhere, PHX_FZR2_CARRY carries it there too.
#ifdef PHX_REFINE_RECOMPUTE
#define PHX_CARRY_DEF false
#else
#define PHX_CARRY_DEF true
#endif
#ifdef PHX_FZR2_CARRY
#define PHX_FZR2_CARRY_DEF PHX_CARRY_DEF
#else
#define PHX_FZR2_CARRY_DEF false
#endif
// The two-wave fused build parks its round data in LDS (warm_fused PARK);
// PHX_FZR2_NO_PARK keeps them in registers (the round-5 build, 144 B of spill)
#ifdef PHX_FZR2_NO_PARK
#define PHX_FZR2_PARK_DEF false
#else
#define PHX_FZR2_PARK_DEF true
#endif

// Diagnostics hook (the CPU emulation defines it to record why a lane failed;
// a no-op in the GPU kernels).
#ifndef PHX_LANE_FAIL
#define PHX_LANE_FAIL(code, idx)
#endif
#ifndef PHX_LANE_STAT
#define PHX_LANE_STAT(kind)
#endif
#ifndef PHX_REFINE_HOOK
#define PHX_REFINE_HOOK(step, d2, tol2)
#endif

namespace phx_lane {

PHX_LD int tri(int i, int k) { return i * (i + 1) / 2 + k; }   // i >= k
PHX_LD double clampd(double v, double lo, double hi) { return fmin(fmax(v, lo), hi); }
template <bool B, class T, class E> struct Cond { typedef T type; };
template <class T, class E> struct Cond<false, T, E> { typedef E type; };

// active-set words: 2 bits per column (0 free, 1 at lower, 2 at upper) then
// 2 bits per row (0 inactive, 1 lower side active, 2 upper side active)
PHX_LD constexpr int aset_words(int n, int m) { return (2 * (n + m) + 31) / 32; }

// Active-set KKT solves: quasi-definite regularisation and the cap on its
// iterative-refinement steps (compile-time, so the refinement is unrolled and
// 1/(p+reg) of the LP columns folds to a constant).
#ifndef PHX_KKT_REG
#define PHX_KKT_REG 1e-6
#endif
constexpr double KKT_REG = PHX_KKT_REG;
constexpr int KKT_REFINE = 6;
#ifndef PHX_KKT_STOP
#define PHX_KKT_STOP 1e-10
#endif
constexpr double KKT_STOP = PHX_KKT_STOP;

// flags bits shared with the host / generic path
constexpr int32_t FLAG_IPM_TRIED = 1;   // interior point already attempted
constexpr int32_t FLAG_WRITTEN = 2;     // outputs written by a lane kernel
constexpr int32_t FLAG_MAP = 4;         // the lane's affine map (LaneIO::map) matches its stored active set

// phx_iterk's progress word in mapped host memory, polled by the host.
struct IterkProgress {
    uint64_t word;   // (iteration << 8) | stop (0 running, 1 converged, 2 generic-path lanes):
                     // one 8-byte store, so the host never sees a torn pair
    double conv;     // read by the host only after the stream drained
};

// phx_iterk, fused mode (two-stage trees): ONE launch of phx_lane_warm is a
// whole PH iteration k.  Per lane: Update_W (W += rho (x_{k-1} - x-bar_k),
// phbase.py:293-318) and |x_{k-1} - x-bar_k| (convergence_diff,
// phbase.py:321-343), then solve k with the new W; the lane's
// prob_coeff-weighted x and x^2 of solve k are the partial sums of iteration
// k+1's Compute_Xbar (phbase.py:54-80).  Per-block partials are folded by the
// last block of each arrival shard, then by the last shard, into the stage
// buffer of iteration k+1.  The stop test on conv_k runs in the prologue of
// the NEXT launch (after the all-reduce on several ranks), so solve k is
// speculative: it writes the other output buffer set and is simply not
// committed when conv_k < convthresh.
struct FusedW {
    int32_t on;
    int32_t iter;              // k
    int32_t first;             // first iteration of a pipeline segment: no decision on conv_{k-1}
    double* stage;             // [2*nns sums | straggler count | R conv sums]: read as iteration k's,
                               // overwritten by the last block with iteration k+1's
    double* node_sums;         // published x-bar | xsqbar (block 0, once the iteration proceeds)
    int32_t nns;               // node-slot count (= nonant slots: one tree node)
    const double* x_prev;      // solve k-1's x [n][S]
    const double* pc;          // prob_coeff [N][S]
    int32_t* ctl;              // [0] stop flag (the gate of later kernels), [1] stop iteration
    IterkProgress* prog;
    double* part;              // [gridDim.x * NV] block partials, then [TICKET_SHARDS * NV] shard partials
    unsigned int* tk;          // sharded arrival counters (TICKET_SET words)
    int32_t g, R;              // this rank's emulated-rank entry, emulated rank count
    const double* cnt;         // [R] element counts (convergence_diff's denominators)
    double thresh;
    // compacting mode (kernel phx_lane_warm_fzc, warm_fused_c): round 0 in every
    // lane; the lanes it leaves with a changed active set are finished by the
    // last block of their group of chunks (64-lane blocks), so no wavefront runs
    // later rounds for one lane while 63 wait
    double* rx;                // [n][S] a rework lane's x after round 0
    double* rz;                // [m][S] ... and z
    unsigned long long* rmask; // [blocks] rework lanes of each block
    double* gpart;             // [groups * NV] the groups' rework-lane partials
    unsigned int* gcnt;        // [groups] arrival counters (reset by each group's finisher)
    int32_t gsize;             // blocks per group
};

// Runtime inputs/outputs (device pointers; per-scenario arrays [i*S + s]).
// A, c, bounds below are scaled iff PT::scaled() (phx_jit.h LaneStructure).
struct LaneIO {
    int32_t S;
    const double* Av;      // varying A values [nvar*S]
    const double* c;       // c   [n*S] (only read if PT::c_vary())
    const double* lb;      // lb  [n*S] (PT::bnd_vary())
    const double* ub;
    const double* bl;      // bl  [m*S] (PT::rhs_vary())
    const double* bu;
    // PH objective terms (attach_PH_to_objective, phbase.py:617-699), evaluated
    // in registers: q_j += W_on*W - prox_on*rho*xbar, p_j = prox_on*rho,
    // k = prox_on * sum rho/2 xbar^2, xbar = xbar_node[xbar_idx]
    const double* W;       // [N*S]
    const double* rho;     // [N*S]
    const double* xbar_node;
    const int32_t* xbar_idx;  // [N*S]
    int32_t W_on, prox_on;
    double* xT;            // scaled x [n*S]   (generic-path hand-over)
    double* yT;            // scaled y [m*S]
    double* x;             // PDHG warm start (= xT)
    double* y;
    double* x0;
    double* y0;
    double* ipm_x;         // unscaled interior point [n*S] (phx_lane_cold -> phx_lane_cold_as)
    double* ipm_y;         // [m*S]
    double* err;           // [S]
    int32_t* status;       // [S]: 1 certified, 0 running (generic path)
    int32_t* iters;        // [S]: IPM iterations used
    int32_t* flags;        // [S]: FLAG_* bits
    uint32_t* aset;        // [aset_words(n,m)*S] active set of the last certified solve
    double* x_out;         // unscaled x [n*S]
    double* y_out;         // unscaled row duals [m*S] (may be null)
    double* obj_out;       // [S] objective incl. PH terms
    int32_t* status_out;   // [S] caller's status (1 optimal)
    int32_t* iters_out;    // [S] caller's iteration counts
    int32_t* lanes_out;    // compacted uncertified lanes
    int32_t* count_out;    // their number (atomic)
    int32_t* counts_next;  // [16] zeroed by block 0 (the next solve's counters), or null
    int32_t max_it;
    double ipm_tol;
    double kkt_tol;
    double reg;
    int32_t refine;
    int32_t as_rounds;     // active-set rounds after the interior point (phx_lane_cold)
    int32_t warm_rounds;   // active-set rounds per warm pass
    int32_t single_after;  // rounds after which the active-set update changes one violation at a time
    const int32_t* gate;   // *gate != 0: the launch does nothing (phx_iterk past its stop), or null
    double* map;           // [map_words<PT>()][S] affine solution maps (see map_apply), or null
    FusedW fz;             // phx_iterk fused Update_W (fz.on = 0 otherwise)
    uint64_t* stamps;      // diagnostics (PHX_LANE_STAMPS=1): [block][8] wall-clock phase stamps, or null
};

// phx_iterk fused mode, the last iteration: the small results the host reads
// after the drain, stored by the tail kernel (phx_fz_tail) instead of three
// copy dispatches behind it (~5 us each on the loop's stream).  Each pointer
// pair is skipped when its destination is null.
struct TailCopy {
    int32_t* left_dst;          // the last solve's leftover count (mapped host memory)
    const int32_t* left_src;
    double* seg_dst;            // the last test's convergence sums (device)
    const double* seg_src;
    int32_t nseg;
    double* exp_dst;            // Iter0's expectations (mapped host memory)
    const double* exp_src;
};

// Phase stamps of phx_lane_warm (lane 0 of each wavefront; 100 MHz wall clock):
// 0 entry, 1 after the prologue, 2 after Update_W, 3 after the solve,
// 4 after the compaction, 5 after the epilogue.
#if defined(__HIPCC__) || defined(__HIPCC_RTC__)
__device__ __forceinline__ void lane_stamp(const LaneIO& io, int k) {
    if (io.stamps && threadIdx.x == 0) io.stamps[(uint64_t)blockIdx.x * 8 + k] = wall_clock64();
}
#endif

// Per-lane output stores: write-through (`sc1`, agent-scope relaxed atomic
// stores), which leave no dirty L2 line behind -- a dependent kernel boundary
// costs ~1.7 us + the dirty bytes / 6 TB/s (MI355X_MICROARCH.md, "boundary"),
// and a warm pass writes ~23 MB.  Measured (r03 s22, farmer 100k): warm kernel
// 40.8 -> 39.2 us by events, 1.11 -> 1.13 x 10^9 at K = 20, 1.62 -> 1.65 x 10^9
// at K = 50.  PHX_OUT_PLAIN (a JIT define, PHX_LANE_DEFS) restores plain stores.
#if (defined(__HIPCC__) || defined(__HIPCC_RTC__)) && !defined(PHX_OUT_PLAIN)
#define PHX_OUT(lv, v) __hip_atomic_store(&(lv), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
#else
#define PHX_OUT(lv, v) ((lv) = (v))
#endif

// phx_iterk gate: every kernel of an iteration past the device-side stop exits
// at once (one scalar load; the counters stay as the last real solve left them)
PHX_LD bool gated(const int32_t* gate) { return gate && *(const volatile int32_t*)gate; }

// Hide a value's origin from the optimiser (no instruction): values derived
// from it are recomputed where used instead of kept live across a loop.
PHX_LD void opaque(double& v) {
#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC_RTC__)
    __asm__ volatile("" : "+v"(v));
#else
    (void)v;
#endif
}
PHX_LD int opaque_index(int v) {
#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC_RTC__)
    __asm__ volatile("" : "+v"(v));
#endif
    return v;
}
// (an unsigned word likewise: bit masks read per use inside a loop)
PHX_LD uint32_t opaque_u32(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC_RTC__)
    __asm__ volatile("" : "+v"(v));
#endif
    return v;
}
PHX_LD uint64_t opaque_u32(uint64_t v) {
#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC_RTC__)
    __asm__ volatile("" : "+v"(v));
#endif
    return v;
}

// Data access for one lane: scenario-varying numbers in registers; the
// invariant ones are literals of the specialised kernel (PT tables), which the
// compiler rematerialises with scalar moves instead of keeping them live.
template <class PT>
struct Data {
    const LaneIO& io;
    const int sc;
    double av[PT::NMAX_V];
    double qn[PT::NMAX_S], pn[PT::NMAX_S];
    double kn;

    // Every load is unconditional and issued before any is used (the lane
    // kernels run one wavefront per SIMD at small batches, so each dependent
    // memory round trip is paid in full): the PH-term switches select values
    // instead of guarding loads -- guarded, each slot's loads sat in a branch
    // of their own behind the previous slot's wait, ~6 serial L2 round trips
    // per construction (ISA, r04).  The arrays are always readable: lane_io
    // substitutes zero arrays of the full size for absent ones.
    PHX_LD Data(const LaneIO& io_, int sc_) : io(io_), sc(sc_) {
        const int S = io.S;
        double wv[PT::NMAX_S], rv[PT::NMAX_S];
        int32_t xi[PT::NMAX_S];
        PHX_UNROLL for (int v = 0; v < PT::nvar(); ++v) av[v] = io.Av[(int64_t)v * S + sc];
        PHX_UNROLL for (int t = 0; t < PT::nslot(); ++t) {
            const int64_t o = (int64_t)t * S + sc;
            wv[t] = io.W[o];
            rv[t] = io.rho[o];
            xi[t] = io.xbar_idx[o];
        }
        const bool won = io.W_on != 0, pon = io.prox_on != 0, fzon = io.fz.on != 0;
        kn = 0.0;
        PHX_UNROLL for (int t = 0; t < PT::nslot(); ++t) {
            // fused mode (one tree node, node slot = nonant slot): x-bar of
            // slot t is stage[t], no index gather
            const double xb = io.xbar_node[fzon ? t : xi[t]];
            const double r = pon ? rv[t] : 0.0;
            const double w = won ? wv[t] : 0.0;
            qn[t] = w - r * xb;
            pn[t] = r;
            kn += 0.5 * r * xb * xb;
        }
    }
    // From values already in registers (the fused kernel's preloads, phx_lane_warm_fz):
    // the varying A values, W and rho of every slot and x-bar by slot -- the
    // same operations as the loading constructor, so the same bits
    PHX_LD Data(const LaneIO& io_, int sc_, const double* av_, const double* wv, const double* rv, const double* xbv)
        : io(io_), sc(sc_) {
        PHX_UNROLL for (int v = 0; v < PT::nvar(); ++v) av[v] = av_[v];
        const bool won = io.W_on != 0, pon = io.prox_on != 0;
        kn = 0.0;
        PHX_UNROLL for (int t = 0; t < PT::nslot(); ++t) {
            const double xb = xbv[t];
            const double r = pon ? rv[t] : 0.0;
            const double w = won ? wv[t] : 0.0;
            qn[t] = w - r * xb;
            pn[t] = r;
            kn += 0.5 * r * xb * xb;
        }
    }
    // A copy parked in LDS (park(): [av | qn | pn | kn] by lane, stride 64) and
    // read back through an index the optimiser cannot see through: the same
    // values as the Data that was parked, re-read where a round needs them
    // instead of held live across the round loop (phx_lane_warm_fzr2)
    static constexpr int PARK = PT::NMAX_V + 2 * PT::NMAX_S + 1;
    PHX_LD Data(const LaneIO& io_, int sc_, const double* lds, int lane) : io(io_), sc(sc_) {
        const int l = opaque_index(lane);
        PHX_UNROLL for (int v = 0; v < PT::nvar(); ++v) av[v] = lds[v * 64 + l];
        PHX_UNROLL for (int t = 0; t < PT::nslot(); ++t) {
            qn[t] = lds[(PT::NMAX_V + t) * 64 + l];
            pn[t] = lds[(PT::NMAX_V + PT::NMAX_S + t) * 64 + l];
        }
        kn = lds[(PT::NMAX_V + 2 * PT::NMAX_S) * 64 + l];
    }
    PHX_LD void park(double* lds, int lane) const {
        PHX_UNROLL for (int v = 0; v < PT::nvar(); ++v) lds[v * 64 + lane] = av[v];
        PHX_UNROLL for (int t = 0; t < PT::nslot(); ++t) {
            lds[(PT::NMAX_V + t) * 64 + lane] = qn[t];
            lds[(PT::NMAX_V + PT::NMAX_S + t) * 64 + lane] = pn[t];
        }
        lds[(PT::NMAX_V + 2 * PT::NMAX_S) * 64 + lane] = kn;
    }
    PHX_LD double A(int k) const { return PT::kvar(k) < 0 ? PT::Ac(k) : av[PT::kvar(k)]; }
    // scaling of the problem the lane solver works on (1 when unscaled)
    PHX_LD double dc(int j) const { return PT::scaled() ? PT::dcs(j) : 1.0; }
    PHX_LD double dr(int i) const { return PT::scaled() ? PT::drs(i) : 1.0; }
    PHX_LD double idc(int j) const { return PT::scaled() ? PT::idcs(j) : 1.0; }   // 1/dc
    PHX_LD double idr(int i) const { return PT::scaled() ? PT::idrs(i) : 1.0; }   // 1/dr
    PHX_LD double c(int j) const { return PT::c_vary() ? io.c[(int64_t)j * io.S + sc] : PT::cs(j); }
    PHX_LD double q(int j) const {
        return PT::col_slot(j) >= 0 ? c(j) + dc(j) * qn[PT::col_slot(j)] : c(j);
    }
    PHX_LD double p(int j) const {
        return PT::col_slot(j) >= 0 ? dc(j) * dc(j) * pn[PT::col_slot(j)] : 0.0;
    }
    PHX_LD double l(int j) const { return PT::bnd_vary() ? io.lb[(int64_t)j * io.S + sc] : PT::lbs(j); }
    PHX_LD double u(int j) const { return PT::bnd_vary() ? io.ub[(int64_t)j * io.S + sc] : PT::ubs(j); }
    PHX_LD double bl(int i) const { return PT::rhs_vary() ? io.bl[(int64_t)i * io.S + sc] : PT::bls(i); }
    PHX_LD double bu(int i) const { return PT::rhs_vary() ? io.bu[(int64_t)i * io.S + sc] : PT::bus(i); }

    // (each row / column sum starts from its first product: 0.0 + v is an
    // add IEEE arithmetic keeps, one per row and column per mat-vec)
    PHX_LD void matvec(const double* xv, double* ax) const {
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) if (PT::rempty(i)) ax[i] = 0.0;
        PHX_UNROLL for (int k = 0; k < PT::nnz(); ++k) {
            const double v = A(k) * xv[PT::col(k)];
            ax[PT::row(k)] = PT::rfirst(k) ? v : ax[PT::row(k)] + v;
        }
    }
    PHX_LD void matvec_t(const double* yv, double* aty) const {
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) if (PT::cempty(j)) aty[j] = 0.0;
        PHX_UNROLL for (int k = 0; k < PT::nnz(); ++k) {
            const double v = A(k) * yv[PT::row(k)];
            aty[PT::col(k)] = PT::cfirst(k) ? v : aty[PT::col(k)] + v;
        }
    }
    // q_j + p_j x: the prox term's gradient exists on the nonant columns only
    // (p_j = 0 elsewhere: no 0 * x, which IEEE arithmetic keeps)
    PHX_LD double qpx(int j, double x) const { return PT::col_slot(j) >= 0 ? q(j) + p(j) * x : q(j); }

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
            const bool ps = PT::col_slot(j) >= 0;          // (p_j = 0 off the nonant columns)
            const double lam_s = qpx(j, xv[j]) - aty[j];
            const double lam = lam_s / d;
            double rd = lam;
            if (PT::lfin(j) && lam > 0.0) { rd = 0.0; dobj += l(j) * lam_s; }
            if (PT::ufin(j) && lam < 0.0) { rd = 0.0; dobj += u(j) * lam_s; }
            rd2 += rd * rd;
            qn2 += (qj / d) * (qj / d);
            pobj += ps ? qj * xv[j] + 0.5 * pj * xv[j] * xv[j] : qj * xv[j];
            if (ps) dobj -= 0.5 * pj * xv[j] * xv[j];
        }
        const double ep = sqrt(rp2) / (1.0 + sqrt(bn2));
        const double ed = sqrt(rd2) / (1.0 + sqrt(qn2));
        const double eg = fabs(pobj - dobj) / (1.0 + fabs(pobj) + fabs(dobj));
        // (fmax drops a NaN operand: a non-finite point must fail here, not
        // pass on its finite terms -- the sum of the terms is NaN or inf then)
        const double all = ep + ed + eg;
        const double e = fmax(ep, fmax(ed, eg));
        return (all - all == 0.0 && e < 1e300) ? e : 1e300;
    }
};

// 1/sqrt(d), d > 0: on the GPU the hardware reciprocal square root plus one
// Newton step (relative error ~1e-14; a correctly rounded sqrt and divide cost
// ~20 instructions more per pivot, and every solve refines against the
// factor anyway); on the host (tests/emu) the library functions.
PHX_LD double rsqrt_pos(double d) {
#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC_RTC__)
    const double y = __builtin_amdgcn_rsq(d);
    return y * fma(-0.5 * d * y, y, 1.5);
#else
    return 1.0 / sqrt(d);
#endif
}

// 1/d for the interior point's scalings (d != 0): on the GPU the hardware
// reciprocal plus two Newton steps (a correctly rounded division is a
// ~10-instruction dependent chain; the interior point needs no correct
// rounding); rcp_step: one Newton step, for step-length ratios only.
PHX_LD double rcp_fast(double d) {
#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC_RTC__)
    double r = __builtin_amdgcn_rcp(d);
    r = fma(r, fma(-d, r, 1.0), r);
    return fma(r, fma(-d, r, 1.0), r);
#else
    return 1.0 / d;
#endif
}
PHX_LD double rcp_step(double d) {
#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC_RTC__)
    const double r = __builtin_amdgcn_rcp(d);
    return fma(r, fma(-d, r, 1.0), r);
#else
    return 1.0 / d;
#endif
}

// Packed Cholesky (lower, in place).  A pivot that collapses relative to its
// original diagonal (a dependent row of A D A' near an interior-point
// optimum) is replaced by a huge value, which zeroes that component of the
// solve — the classic IPM safeguard.  Returns false only on a non-finite or
// non-positive original diagonal.
template <class PT>
PHX_LD bool cholesky_ipm(double* M) {
    bool ok = true;
    PHX_UNROLL for (int jj = 0; jj < PT::m(); ++jj) {
        const double d0 = M[tri(jj, jj)];
        double d = d0;
        PHX_UNROLL for (int k = 0; k < PT::m(); ++k)
            if (k < jj && PT::lnz(tri(jj, k))) d -= M[tri(jj, k)] * M[tri(jj, k)];
        ok = ok && (d0 > 0.0) && (d0 < 1e300);
        if (!(d > 1e-13 * d0)) d = 1e128;
        const double inv = rsqrt_pos(d);
        M[tri(jj, jj)] = inv;          // the diagonal keeps 1/L_jj
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
            if (i > jj && PT::lnz(tri(i, jj))) {
                double v = M[tri(i, jj)];
                PHX_UNROLL for (int k = 0; k < PT::m(); ++k)
                    if (k < jj && PT::lnz(tri(i, k)) && PT::lnz(tri(jj, k))) v -= M[tri(i, k)] * M[tri(jj, k)];
                M[tri(i, jj)] = v * inv;
            }
        }
    }
    return ok;
}

// Plain packed Cholesky; false if not (numerically) positive definite.
// Every packed routine touches only the entries of L's symbolic pattern
// PT::lnz (the pair positions of A A' plus the Cholesky fill, phx_jit.h):
// entries outside it stay exact zeros, so skipping them changes no bit.
// The diagonal receives 1/L_ii (the solve multiplies).
template <class PT>
PHX_LD bool cholesky(double* M) {
    bool ok = true;
    PHX_UNROLL for (int jj = 0; jj < PT::m(); ++jj) {
        double d = M[tri(jj, jj)];
        PHX_UNROLL for (int k = 0; k < PT::m(); ++k)
            if (k < jj && PT::lnz(tri(jj, k))) d -= M[tri(jj, k)] * M[tri(jj, k)];
        ok = ok && (d > 0.0);
        d = fmax(d, 1e-300);
        const double inv = rsqrt_pos(d);
        M[tri(jj, jj)] = inv;          // the diagonal keeps 1/L_jj
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
            if (i > jj && PT::lnz(tri(i, jj))) {
                double v = M[tri(i, jj)];
                PHX_UNROLL for (int k = 0; k < PT::m(); ++k)
                    if (k < jj && PT::lnz(tri(i, k)) && PT::lnz(tri(jj, k))) v -= M[tri(i, k)] * M[tri(jj, k)];
                M[tri(i, jj)] = v * inv;
            }
        }
    }
    return ok;
}

// solve (L L') t = t (L's diagonal stored as its reciprocal)
template <class PT>
PHX_LD void chol_solve_inv(const double* M, double* t) {
    PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
        double v = t[i];
        PHX_UNROLL for (int k = 0; k < PT::m(); ++k)
            if (k < i && PT::lnz(tri(i, k))) v -= M[tri(i, k)] * t[k];
        t[i] = v * M[tri(i, i)];
    }
    PHX_UNROLL for (int ii = 0; ii < PT::m(); ++ii) {
        const int i = PT::m() - 1 - ii;
        double v = t[i];
        PHX_UNROLL for (int k = 0; k < PT::m(); ++k)
            if (k > i && PT::lnz(tri(k, i))) v -= M[tri(k, i)] * t[k];
        t[i] = v * M[tri(i, i)];
    }
}

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
// Interior point (Mehrotra predictor-corrector).  Complementarity right-hand
// sides with the second-order term, written with the reciprocal slack r = 1/sl
// (one division per bound per iteration):
//   lower:  comp = smu - sl z + da z (sl + da) r,   dz = (comp - z dx) r
//   upper:  comp = smu - sl z + da z (da - sl) r,   dz = (comp + z dx) r
// (da = affine step of the slack's variable, 0 in the predictor pass).
// Returns the relative KKT error of (x, y); *its = iterations used.
// ---------------------------------------------------------------------------

PHX_LD double comp_lo(double sl, double r, double z, double smu, double da) {
    return smu - sl * z + da * z * (sl + da) * r;
}
PHX_LD double comp_up(double sl, double r, double z, double smu, double da) {
    return smu - sl * z + da * z * (da - sl) * r;
}

// the interior point's state, made opaque (only the entries that exist)
template <class PT>
PHX_LD void ipm_opaque(double* x, double* zl, double* zu, double* rl, double* ru, double* s, double* wl,
                       double* wu, double* rwl, double* rwu, double* y) {
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
        opaque(x[j]);
        if (has_lo<PT>(j)) { opaque(zl[j]); opaque(rl[j]); }
        if (has_up<PT>(j)) { opaque(zu[j]); opaque(ru[j]); }
    }
    PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
        opaque(y[i]);
        if (!row_free<PT>(i) && !PT::eq(i)) opaque(s[i]);
        if (row_lo<PT>(i)) { opaque(wl[i]); opaque(rwl[i]); }
        if (row_up<PT>(i)) { opaque(wu[i]); opaque(rwu[i]); }
    }
}

// The interior point's per-iteration arrays read in both passes -- the normal
// matrix's factor, the column and row scalings, the predictor's directions --
// parked in LDS on the GPU (one wavefront per block, [slot][lane]) and read
// back where they are used, through an index the optimiser cannot see
// through: with them held in registers across the passes the iteration's
// live set (farmer: ~340 VGPRs) overflowed into AGPRs, one accvgpr move per
// 32-bit half per use (≈1,000 moves against ≈2,300 FP64 operations per
// iteration, offline ISA).  The values read back are the values stored, so
// the arithmetic is unchanged.  Parked while the block fits 40 KB (one
// wavefront per SIMD, four blocks per CU); PHX_IPM_NO_PARK keeps registers.
// (A two-wave build with a 20 KB budget spills 644 B per lane: offline ISA.)
#if (defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC_RTC__)) && !defined(PHX_IPM_NO_PARK)
#define PHX_IPM_PARK_ON 1
#else
#define PHX_IPM_PARK_ON 0
#endif
#ifndef PHX_IPM_PARK_BYTES
#define PHX_IPM_PARK_BYTES 40960
#endif
template <class PT>
struct IpmPark {
    static constexpr int NN = PT::NMAX_N, MM = PT::NMAX_M, TT = PT::NMAX_M * (PT::NMAX_M + 1) / 2;
    // in priority order while the block's bytes fit PHX_IPM_PARK_BYTES (one
    // wavefront per SIMD: 40 KB; two: 20 KB): M | Dx | isig | dxa | dsa | the
    // reciprocal slacks rl ru rwl rwu (farmer: the first five at 40 KB, aircond
    // the first three.  A 96 KB budget for batches of at most one block per CU,
    // where every array fits, was measured slower: C4 Iter0 0.281 / 0.287 against
    // 0.265 / 0.269 ms, C3s8 0.153 / 0.170 against 0.148 / 0.145, r06_s19)
    static constexpr bool fits(int slots) { return PHX_IPM_PARK_ON && slots * 64 * 8 <= PHX_IPM_PARK_BYTES; }
    static constexpr bool PM = fits(TT), PDX = PM && fits(TT + NN), PIS = PDX && fits(TT + NN + MM),
                          PDXA = PIS && fits(TT + 2 * NN + MM), PDSA = PDXA && fits(TT + 2 * NN + 2 * MM),
                          PR = PDSA && fits(TT + 4 * NN + 4 * MM);
    static constexpr int OM = 0, ODX = TT, OIS = TT + NN, ODXA = TT + NN + MM, ODSA = TT + 2 * NN + MM,
                         ORL = TT + 2 * NN + 2 * MM, ORU = ORL + NN, ORWL = ORU + NN, ORWU = ORWL + MM;
    static constexpr int SIZE = PR ? TT + 4 * NN + 4 * MM : PDSA ? TT + 2 * NN + 2 * MM : PDXA ? TT + 2 * NN + MM
                              : PIS ? TT + NN + MM : PDX ? TT + NN : PM ? TT : 0;
    static constexpr bool ON = SIZE > 0;
    static constexpr bool on(int off) {
        return off == OM ? PM : off == ODX ? PDX : off == OIS ? PIS : off == ODXA ? PDXA : off == ODSA ? PDSA : PR;
    }
};
template <class PT, int K>
PHX_LD void ipm_put(double* lds, const double* v, int off) {
    if (IpmPark<PT>::on(off)) {
#if PHX_IPM_PARK_ON
        const int l = threadIdx.x;
        PHX_UNROLL for (int k = 0; k < K; ++k) lds[(off + k) * 64 + l] = v[k];
#endif
    }
}
template <class PT, int K>
PHX_LD void ipm_get(const double* lds, double* v, int off) {
    if (IpmPark<PT>::on(off)) {
#if PHX_IPM_PARK_ON
        const int l = opaque_index(threadIdx.x);
        PHX_UNROLL for (int k = 0; k < K; ++k) v[k] = lds[(off + k) * 64 + l];
#endif
    }
}
// the reciprocal slacks, all four
template <class PT>
PHX_LD void ipm_put_r(double* lds, const double* rl, const double* ru, const double* rwl, const double* rwu) {
    typedef IpmPark<PT> PK;
    ipm_put<PT, PK::NN>(lds, rl, PK::ORL);
    ipm_put<PT, PK::NN>(lds, ru, PK::ORU);
    ipm_put<PT, PK::MM>(lds, rwl, PK::ORWL);
    ipm_put<PT, PK::MM>(lds, rwu, PK::ORWU);
}
template <class PT>
PHX_LD void ipm_get_r(const double* lds, double* rl, double* ru, double* rwl, double* rwu) {
    typedef IpmPark<PT> PK;
    ipm_get<PT, PK::NN>(lds, rl, PK::ORL);
    ipm_get<PT, PK::NN>(lds, ru, PK::ORU);
    ipm_get<PT, PK::MM>(lds, rwl, PK::ORWL);
    ipm_get<PT, PK::MM>(lds, rwu, PK::ORWU);
}

#ifndef PHX_IPM_CHECK_FROM
#define PHX_IPM_CHECK_FROM 6
#endif

// The start point's scales come from the problem (phx_jit.h: xs a fifth of
// the median bound / row-side magnitude, ws half the median cost magnitude,
// zs a tenth of ws); PHX_IPM_SCALES=0 (a JIT define) restores the unit
// offsets of rounds 1-3.
#if defined(PHX_IPM_SCALES) && PHX_IPM_SCALES == 0
#define PHX_IPM_XS_ 1.0
#define PHX_IPM_ZS_ 1.0
#define PHX_IPM_WS_ 1.0
#else
#define PHX_IPM_XS_ PT::ipm_xs()
#define PHX_IPM_ZS_ PT::ipm_zs()
#define PHX_IPM_WS_ PT::ipm_ws()
#endif
template <class PT>
PHX_LD double ipm_core(const Data<PT>& D, int max_it, double tol, double* x, double* y, int* its,
                       double xs = PHX_IPM_XS_, double zs = PHX_IPM_ZS_, double ws = PHX_IPM_WS_) {
    constexpr int NN = PT::NMAX_N, MM = PT::NMAX_M, TT = PT::NMAX_M * (PT::NMAX_M + 1) / 2;
    typedef IpmPark<PT> PK;
#if PHX_IPM_PARK_ON
    __shared__ double ipm_lds[PK::ON ? PK::SIZE * 64 : 1];
#else
    double* const ipm_lds = nullptr;
#endif
    const double reg = 1e-10;
    double zl[NN], zu[NN], s[MM], wl[MM], wu[MM];
    // start point (cost-aware multipliers)
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
        double xv = 0.0;
        if (PT::fixed(j)) xv = D.l(j);
        else if (PT::lfin(j) && PT::ufin(j)) {
            const double lo = D.l(j), hi = D.u(j);
            xv = (hi - lo <= 2.0 * xs) ? 0.5 * (lo + hi) : clampd(0.0, lo + xs, hi - xs);
        } else if (PT::lfin(j)) xv = fmax(0.0, D.l(j) + xs);
        else if (PT::ufin(j)) xv = fmin(0.0, D.u(j) - xs);
        x[j] = xv;
        const double g = D.q(j) + D.p(j) * xv;
        zl[j] = has_lo<PT>(j) ? fmax(g, 0.0) + zs : 0.0;
        zu[j] = has_up<PT>(j) ? fmax(-g, 0.0) + zs : 0.0;
    }
    {
        double ax[MM];
        D.matvec(x, ax);
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
            double sv = ax[i];
            if (PT::eq(i)) sv = D.bl(i);
            else if (PT::blfin(i) && PT::bufin(i)) {
                const double lo = D.bl(i), hi = D.bu(i);
                sv = (hi - lo <= 2.0 * xs) ? 0.5 * (lo + hi) : clampd(ax[i], lo + xs, hi - xs);
            } else if (PT::blfin(i)) sv = fmax(ax[i], D.bl(i) + xs);
            else if (PT::bufin(i)) sv = fmin(ax[i], D.bu(i) - xs);
            s[i] = sv;
            wl[i] = row_lo<PT>(i) ? ws : 0.0;
            wu[i] = row_up<PT>(i) ? ws : 0.0;
            y[i] = wl[i] - wu[i];
        }
    }
    double ncomp = 0.0;
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) ncomp += (has_lo<PT>(j) ? 1.0 : 0.0) + (has_up<PT>(j) ? 1.0 : 0.0);
    PHX_UNROLL for (int i = 0; i < PT::m(); ++i) ncomp += (row_lo<PT>(i) ? 1.0 : 0.0) + (row_up<PT>(i) ? 1.0 : 0.0);
    const double inv_ncomp = ncomp > 0.0 ? 1.0 / ncomp : 0.0;
    double err = 1e300;
    int it = 0;
    for (; it < max_it; ++it) {
        // (the KKT error from iteration PHX_IPM_CHECK_FROM on, and at the last
        // one: no interior point converges in fewer, and the error of the
        // start's first iterations is ~1/3 of an iteration's work)
        if (it >= PHX_IPM_CHECK_FROM || it == max_it - 1) {
            err = D.kkt(x, y);
            if (err < tol || !(err < 1e300)) break;
        }
        // reciprocal slacks
        double rl[NN], ru[NN], rwl[MM], rwu[MM];
        double mu = 0.0;
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
            rl[j] = has_lo<PT>(j) ? rcp_fast(x[j] - D.l(j)) : 0.0;
            ru[j] = has_up<PT>(j) ? rcp_fast(D.u(j) - x[j]) : 0.0;
            if (has_lo<PT>(j)) mu += (x[j] - D.l(j)) * zl[j];
            if (has_up<PT>(j)) mu += (D.u(j) - x[j]) * zu[j];
        }
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
            rwl[i] = row_lo<PT>(i) ? rcp_fast(s[i] - D.bl(i)) : 0.0;
            rwu[i] = row_up<PT>(i) ? rcp_fast(D.bu(i) - s[i]) : 0.0;
            if (row_lo<PT>(i)) mu += (s[i] - D.bl(i)) * wl[i];
            if (row_up<PT>(i)) mu += (D.bu(i) - s[i]) * wu[i];
        }
        mu *= inv_ncomp;
        // normal matrix
        double Dx[NN], isig[MM], M[TT];
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
            double h = D.p(j) + reg;
            if (has_lo<PT>(j)) h += zl[j] * rl[j];
            if (has_up<PT>(j)) h += zu[j] * ru[j];
            Dx[j] = PT::fixed(j) ? 0.0 : rcp_fast(h);
        }
        PHX_UNROLL for (int t = 0; t < TT; ++t) M[t] = 0.0;
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
            double sg = 0.0;
            if (row_lo<PT>(i)) sg += wl[i] * rwl[i];
            if (row_up<PT>(i)) sg += wu[i] * rwu[i];
            isig[i] = (row_lo<PT>(i) || row_up<PT>(i)) ? rcp_fast(sg) : 0.0;
            M[tri(i, i)] = row_free<PT>(i) ? 1.0 : (PT::eq(i) ? reg : isig[i] + reg);
        }
        PHX_UNROLL for (int t = 0; t < PT::npairs(); ++t) {
            const int ka = PT::pair_a(t), kb = PT::pair_b(t);
            if (!row_free<PT>(PT::row(ka)) && !row_free<PT>(PT::row(kb)))
                M[PT::pair_pos(t)] += D.A(ka) * Dx[PT::col(ka)] * D.A(kb);
        }
        if (!cholesky_ipm<PT>(M)) { PHX_LANE_FAIL(20, it); break; }
        ipm_put<PT, TT>(ipm_lds, M, PK::OM);
        ipm_put<PT, NN>(ipm_lds, Dx, PK::ODX);
        ipm_put<PT, MM>(ipm_lds, isig, PK::OIS);
        ipm_put_r<PT>(ipm_lds, rl, ru, rwl, rwu);
        // predictor (pass 0, smu = 0) then corrector (pass 1)
        double smu = 0.0, ap = 1.0, ad = 1.0;
        double dx[NN], ds[MM], dy[MM], dxa[NN], dsa[MM];
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) dxa[j] = 0.0;
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) dsa[i] = 0.0;
        PHX_IPM_PASS_LOOP for (int pass = 0; pass < 2; ++pass) {
            ipm_get_r<PT>(ipm_lds, rl, ru, rwl, rwu);
            ipm_opaque<PT>(x, zl, zu, rl, ru, s, wl, wu, rwl, rwu, y);
            if (pass == 1) ipm_get<PT, NN>(ipm_lds, dxa, PK::ODXA);
            ipm_get<PT, NN>(ipm_lds, Dx, PK::ODX);
            {
                double ax[MM], aty[NN];
                D.matvec(x, ax);
                D.matvec_t(y, aty);
                PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
                    double r = aty[j] - D.p(j) * x[j] - D.q(j);
                    if (has_lo<PT>(j)) {
                        const double sl = x[j] - D.l(j);
                        r += zl[j] + (pass == 0 ? -(sl * zl[j]) : comp_lo(sl, rl[j], zl[j], smu, dxa[j])) * rl[j];
                    }
                    if (has_up<PT>(j)) {
                        const double sl = D.u(j) - x[j];
                        r -= zu[j] + (pass == 0 ? -(sl * zu[j]) : comp_up(sl, ru[j], zu[j], smu, dxa[j])) * ru[j];
                    }
                    dx[j] = PT::fixed(j) ? 0.0 : r * Dx[j];      // H^-1 rho_x
                }
                double ahr[MM];
                D.matvec(dx, ahr);
                ipm_get<PT, MM>(ipm_lds, isig, PK::OIS);
                if (pass == 1) ipm_get<PT, MM>(ipm_lds, dsa, PK::ODSA);
                PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
                    double rhos = -y[i];
                    if (row_lo<PT>(i)) {
                        const double sl = s[i] - D.bl(i);
                        rhos += wl[i] + (pass == 0 ? -(sl * wl[i]) : comp_lo(sl, rwl[i], wl[i], smu, dsa[i])) * rwl[i];
                    }
                    if (row_up<PT>(i)) {
                        const double sl = D.bu(i) - s[i];
                        rhos -= wu[i] + (pass == 0 ? -(sl * wu[i]) : comp_up(sl, rwu[i], wu[i], smu, dsa[i])) * rwu[i];
                    }
                    ds[i] = rhos;
                    if (row_free<PT>(i)) dy[i] = 0.0;
                    else if (PT::eq(i)) dy[i] = -(ax[i] - D.bl(i)) - ahr[i];
                    else dy[i] = -(ax[i] - s[i]) + rhos * isig[i] - ahr[i];
                }
            }
            ipm_get<PT, TT>(ipm_lds, M, PK::OM);
            chol_solve_inv<PT>(M, dy);
            {
                double atdy[NN];
                D.matvec_t(dy, atdy);
                ipm_get<PT, NN>(ipm_lds, Dx, PK::ODX);
                PHX_UNROLL for (int j = 0; j < PT::n(); ++j)
                    if (!PT::fixed(j)) dx[j] += Dx[j] * atdy[j];
            }
            ipm_get<PT, MM>(ipm_lds, isig, PK::OIS);
            PHX_UNROLL for (int i = 0; i < PT::m(); ++i)
                ds[i] = (PT::eq(i) || row_free<PT>(i)) ? 0.0 : (ds[i] - dy[i]) * isig[i];
            ipm_get_r<PT>(ipm_lds, rl, ru, rwl, rwu);
            ipm_opaque<PT>(x, zl, zu, rl, ru, s, wl, wu, rwl, rwu, y);
            // step lengths as inverse ratios (step = 1 / max(1, max ratio)),
            // multiplier steps recomputed from dx, ds
            double apr = 1.0, adr = 1.0;
            if (pass == 1) {
                ipm_get<PT, NN>(ipm_lds, dxa, PK::ODXA);
                ipm_get<PT, MM>(ipm_lds, dsa, PK::ODSA);
            }
            PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
                // (the predictor's comp = -sl z: -dz / z = (sl + dx) r, no reciprocal of z)
                if (has_lo<PT>(j)) {
                    const double sl = x[j] - D.l(j);
                    apr = fmax(apr, -dx[j] * rl[j]);
                    if (pass == 0) {
                        adr = fmax(adr, (sl + dx[j]) * rl[j]);
                    } else {
                        const double dz = (comp_lo(sl, rl[j], zl[j], smu, dxa[j]) - zl[j] * dx[j]) * rl[j];
                        adr = fmax(adr, -dz * rcp_step(zl[j]));
                    }
                }
                if (has_up<PT>(j)) {
                    const double sl = D.u(j) - x[j];
                    apr = fmax(apr, dx[j] * ru[j]);
                    if (pass == 0) {
                        adr = fmax(adr, (sl - dx[j]) * ru[j]);
                    } else {
                        const double dz = (comp_up(sl, ru[j], zu[j], smu, dxa[j]) + zu[j] * dx[j]) * ru[j];
                        adr = fmax(adr, -dz * rcp_step(zu[j]));
                    }
                }
            }
            PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
                if (row_lo<PT>(i)) {
                    const double sl = s[i] - D.bl(i);
                    apr = fmax(apr, -ds[i] * rwl[i]);
                    if (pass == 0) {
                        adr = fmax(adr, (sl + ds[i]) * rwl[i]);
                    } else {
                        const double dw = (comp_lo(sl, rwl[i], wl[i], smu, dsa[i]) - wl[i] * ds[i]) * rwl[i];
                        adr = fmax(adr, -dw * rcp_step(wl[i]));
                    }
                }
                if (row_up<PT>(i)) {
                    const double sl = D.bu(i) - s[i];
                    apr = fmax(apr, ds[i] * rwu[i]);
                    if (pass == 0) {
                        adr = fmax(adr, (sl - ds[i]) * rwu[i]);
                    } else {
                        const double dw = (comp_up(sl, rwu[i], wu[i], smu, dsa[i]) + wu[i] * ds[i]) * rwu[i];
                        adr = fmax(adr, -dw * rcp_step(wu[i]));
                    }
                }
            }
            ap = rcp_fast(apr);
            ad = rcp_fast(adr);
            if (pass == 0) {
                double maff = 0.0;
                PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
                    if (has_lo<PT>(j)) {
                        const double sl = x[j] - D.l(j);
                        const double dz = -zl[j] * (sl + dx[j]) * rl[j];
                        maff += (sl + ap * dx[j]) * (zl[j] + ad * dz);
                    }
                    if (has_up<PT>(j)) {
                        const double sl = D.u(j) - x[j];
                        const double dz = zu[j] * (dx[j] - sl) * ru[j];
                        maff += (sl - ap * dx[j]) * (zu[j] + ad * dz);
                    }
                    dxa[j] = dx[j];
                }
                PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
                    if (row_lo<PT>(i)) {
                        const double sl = s[i] - D.bl(i);
                        const double dw = -wl[i] * (sl + ds[i]) * rwl[i];
                        maff += (sl + ap * ds[i]) * (wl[i] + ad * dw);
                    }
                    if (row_up<PT>(i)) {
                        const double sl = D.bu(i) - s[i];
                        const double dw = wu[i] * (ds[i] - sl) * rwu[i];
                        maff += (sl - ap * ds[i]) * (wu[i] + ad * dw);
                    }
                    dsa[i] = ds[i];
                }
                maff *= inv_ncomp;
                const double ratio = mu > 0.0 ? maff / mu : 0.0;
                smu = ratio * ratio * ratio * mu;
                ipm_put<PT, NN>(ipm_lds, dxa, PK::ODXA);
                ipm_put<PT, MM>(ipm_lds, dsa, PK::ODSA);
            }
        }
        // update (multipliers first: they use the old slacks)
        ap = fmin(1.0, 0.995 * ap);
        ad = fmin(1.0, 0.995 * ad);
        ipm_get<PT, NN>(ipm_lds, dxa, PK::ODXA);
        ipm_get<PT, MM>(ipm_lds, dsa, PK::ODSA);
        ipm_get_r<PT>(ipm_lds, rl, ru, rwl, rwu);
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
            if (has_lo<PT>(j)) {
                const double sl = x[j] - D.l(j);
                zl[j] += ad * (comp_lo(sl, rl[j], zl[j], smu, dxa[j]) - zl[j] * dx[j]) * rl[j];
            }
            if (has_up<PT>(j)) {
                const double sl = D.u(j) - x[j];
                zu[j] += ad * (comp_up(sl, ru[j], zu[j], smu, dxa[j]) + zu[j] * dx[j]) * ru[j];
            }
            x[j] += ap * dx[j];
        }
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
            if (row_lo<PT>(i)) {
                const double sl = s[i] - D.bl(i);
                wl[i] += ad * (comp_lo(sl, rwl[i], wl[i], smu, dsa[i]) - wl[i] * ds[i]) * rwl[i];
            }
            if (row_up<PT>(i)) {
                const double sl = D.bu(i) - s[i];
                wu[i] += ad * (comp_up(sl, rwu[i], wu[i], smu, dsa[i]) + wu[i] * ds[i]) * rwu[i];
            }
            s[i] += ap * ds[i];
            y[i] += ad * dy[i];
        }
    }
    *its = it;
    return err;
}

// ---------------------------------------------------------------------------
// Active set of one lane.  F[j]: column free; up[j]: a non-free column sits at
// its upper bound (else lower; fixed columns: lower).  R[i]: row active;
// lo[i]: at its lower side (equality rows: always active, lower).
// ---------------------------------------------------------------------------
// Kept as per-lane bit masks in vector registers (per-lane bool arrays would
// become 64-bit exec-style lane masks in scalar registers and spill).

template <class PT>
struct ASet {
    typedef typename Cond<(PT::NMAX_N <= 32), uint32_t, uint64_t>::type CMask;
    CMask f = 0, u = 0;      // column j: bit j
    uint32_t r = 0, l = 0;   // row i: bit i
    PHX_LD bool F(int j) const { return (f >> j) & 1u; }
    PHX_LD bool up(int j) const { return (u >> j) & 1u; }
    PHX_LD bool R(int i) const { return (r >> i) & 1u; }
    PHX_LD bool lo(int i) const { return (l >> i) & 1u; }
    PHX_LD void setF(int j, bool v) { f = v ? (f | ((CMask)1 << j)) : (f & ~((CMask)1 << j)); }
    PHX_LD void setUp(int j, bool v) { u = v ? (u | ((CMask)1 << j)) : (u & ~((CMask)1 << j)); }
    PHX_LD void setR(int i, bool v) { r = v ? (r | (1u << i)) : (r & ~(1u << i)); }
    PHX_LD void setLo(int i, bool v) { l = v ? (l | (1u << i)) : (l & ~(1u << i)); }
};

// A lane's boolean as a 0/1 integer in a vector register.  Every per-lane
// bool is a 64-bit lane mask in scalar registers; the ~40 an active set and
// its certificate keep live spilled to VGPR lanes (v_writelane / v_readlane,
// ~500 of them in the r03 warm kernel).  The empty asm keeps the compiler from
// folding the 0/1 values back into lane-mask logic.
PHX_LD uint32_t vbit(bool b) {
    uint32_t v = b ? 1u : 0u;
#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC_RTC__)
    __asm__ volatile("" : "+v"(v));
#endif
    return v;
}
// bit k of an active-set word as a 0/1 double (a multiplier)
template <class W>
PHX_LD double bitd(W w, int k) { return (double)(uint32_t)((w >> k) & 1u); }

// An active set's bits as multipliers, once per round: the factor and the
// refinement scale by them instead of selecting (x * 1 and x + (+-0) are exact,
// so the factor and the iterates are bit for bit those of the selecting code).
template <class PT>
struct AMul {
    double fF[PT::NMAX_N];   // 1: column free
    double rR[PT::NMAX_M];   // 1: row active
    typename ASet<PT>::CMask fb;   // the same as bit words (kkt_refine's LEAN steps)
    uint32_t rb;
    PHX_LD explicit AMul(const ASet<PT>& a) : fb(a.f), rb(a.r) {
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) fF[j] = bitd(a.f, j);
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) rR[i] = bitd(a.r, i);
    }
};

template <class PT>
PHX_LD void aset_from_words(const uint32_t* w, ASet<PT>& a);
template <class PT>
PHX_LD void aset_load(const LaneIO& io, int sc, ASet<PT>& a) {
    constexpr int NW = aset_words(PT::NMAX_N, PT::NMAX_M);
    uint32_t w[NW];
    PHX_UNROLL for (int k = 0; k < aset_words(PT::n(), PT::m()); ++k) w[k] = io.aset[(int64_t)k * io.S + sc];
    aset_from_words<PT>(w, a);
}
// the active set from its stored words (2 bits per column, then per row)
template <class PT>
PHX_LD void aset_from_words(const uint32_t* w, ASet<PT>& a) {
    // (0/1 integers, vbit: no per-lane bool held live)
    typedef typename ASet<PT>::CMask CM;
    CM fw = 0, uw = 0;
    uint32_t rw = 0, lw = 0;
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
        const uint32_t v = (w[(2 * j) >> 5] >> ((2 * j) & 31)) & 3u;
        uint32_t fr = 0u, upj = 0u;
        if (!PT::fixed(j)) {
            fr = vbit(v == 0u);
            upj = vbit(v == 2u);
            if (!PT::ufin(j)) { fr |= upj; upj = 0u; }              // at an infinite upper bound: free
            if (!PT::lfin(j)) fr |= (fr | upj) ^ 1u;                 // at an infinite lower bound: free
        }
        fw |= (CM)fr << j;
        uw |= (CM)upj << j;
    }
    PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
        const int b = 2 * (PT::n() + i);
        const uint32_t v = (w[b >> 5] >> (b & 31)) & 3u;
        uint32_t R, L;
        if (PT::eq(i)) { R = 1u; L = 1u; }
        else {
            L = vbit(v == 1u);
            R = (PT::blfin(i) ? L : 0u) | (PT::bufin(i) ? vbit(v == 2u) : 0u);
        }
        rw |= R << i;
        lw |= L << i;
    }
    a.f = fw;
    a.u = uw;
    a.r = rw;
    a.l = lw;
}

template <class PT>
PHX_LD void aset_store(const LaneIO& io, int sc, const ASet<PT>& a) {
    constexpr int NW = aset_words(PT::NMAX_N, PT::NMAX_M);
    uint32_t w[NW];
    PHX_UNROLL for (int k = 0; k < NW; ++k) w[k] = 0u;
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
        const uint32_t v = a.F(j) ? 0u : (a.up(j) ? 2u : 1u);
        w[(2 * j) >> 5] |= v << ((2 * j) & 31);
    }
    PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
        const int b = 2 * (PT::n() + i);
        const uint32_t v = a.R(i) ? (a.lo(i) ? 1u : 2u) : 0u;
        w[b >> 5] |= v << (b & 31);
    }
    // (the word addresses recomputed from an opaque index: kept from aset_load
    // across the solve they were spilled to scratch)
    const int so = opaque_index(sc);
    PHX_UNROLL for (int k = 0; k < aset_words(PT::n(), PT::m()); ++k) PHX_OUT(io.aset[(int64_t)k * io.S + so], w[k]);
}

// Classify at an interior-point (x, y): a bound/row is active when its slack
// is within tol (relative) or smaller than its correctly-signed multiplier
// (OSQP's polish rule, sharp at IPM points by strict complementarity).
template <class PT>
PHX_LD void classify(const Data<PT>& D, const double* xv, const double* yv, double tol, ASet<PT>& a) {
    // (the words built from 0/1 integers, vbit: no per-lane bool held live)
    typedef typename ASet<PT>::CMask CM;
    CM fw = 0, uw = 0;
    uint32_t rw = 0, lw = 0;
    double aty[PT::NMAX_N];
    D.matvec_t(yv, aty);
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
        const double lam = D.qpx(j, xv[j]) - aty[j];
        uint32_t fr = PT::fixed(j) ? 0u : 1u, upj = 0u;
        if (PT::lfin(j)) {
            const double lo = D.l(j);
            fr &= vbit(xv[j] - lo <= tol * (1.0 + fabs(lo)) || xv[j] - lo < lam) ^ 1u;
        }
        if (PT::ufin(j)) {
            const double hi = D.u(j);
            upj = fr & vbit(hi - xv[j] <= tol * (1.0 + fabs(hi)) || hi - xv[j] < -lam);
            fr &= upj ^ 1u;
        }
        fw |= (CM)fr << j;
        uw |= (CM)upj << j;
    }
    double ax[PT::NMAX_M];
    D.matvec(xv, ax);
    PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
        uint32_t lo_act = PT::eq(i) ? 1u : 0u, up_act = 0u;
        if (!PT::eq(i) && PT::blfin(i)) {
            const double lo = D.bl(i);
            lo_act = vbit(ax[i] - lo <= tol * (1.0 + fabs(lo)) || ax[i] - lo < yv[i]);
        }
        if (!PT::eq(i) && PT::bufin(i)) {
            const double hi = D.bu(i);
            up_act = (lo_act ^ 1u) & vbit(hi - ax[i] <= tol * (1.0 + fabs(hi)) || hi - ax[i] < -yv[i]);
        }
        rw |= (lo_act | up_act) << i;
        lw |= lo_act << i;
    }
    a.f = fw;
    a.u = uw;
    a.r = rw;
    a.l = lw;
}

// Equality-constrained KKT solve for the active set a:
//      [ P_FF   A_RF' ] [x_F]   [ -q_F        ]
//      [ A_RF   0     ] [ z ] = [ b_R - A_RB x_B ]     (z = -y_R)
// by its quasi-definite regularisation (P+reg, -reg) and iterative refinement
// from the given (xp, z) (a proximal-point iteration that converges to the
// KKT solution nearest the start on degenerate faces).  Non-free columns are
// set to their bound.  false if the Schur complement is not positive definite.
// Factor of one active set: Schur complement A_RF (P_FF + reg)^-1 A_RF' + reg I
// (inactive rows: identity), packed Cholesky, and 1/(p + reg) of the nonant
// columns.
template <class PT>
struct KFactor {
    double M[PT::NMAX_M * (PT::NMAX_M + 1) / 2];
    double ipn[PT::NMAX_S];
    PHX_LD double Hinv(int j) const { return PT::col_slot(j) >= 0 ? ipn[PT::col_slot(j)] : 1.0 / KKT_REG; }
};

template <class PT>
PHX_LD bool kkt_factor(const Data<PT>& D, const AMul<PT>& am, KFactor<PT>& K) {
    constexpr int TT = PT::NMAX_M * (PT::NMAX_M + 1) / 2;
    constexpr double reg = KKT_REG;
    // 1/(p_j + reg): a literal for columns without a PH slot (p = 0), three
    // or so reciprocals for the nonant columns
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j)
        if (PT::col_slot(j) >= 0) K.ipn[PT::col_slot(j)] = 1.0 / (D.p(j) + reg);
    PHX_UNROLL for (int t = 0; t < TT; ++t) K.M[t] = 0.0;
    // active rows reg, inactive 1: rR reg + (1 - rR), exact for rR in {0, 1}
    PHX_UNROLL for (int i = 0; i < PT::m(); ++i) K.M[tri(i, i)] = fma(am.rR[i], reg, 1.0 - am.rR[i]);
    // A's entries of inactive rows and H^-1 of non-free columns as zeros:
    // (gA_a h) gA_b is A_a H^-1 A_b when both rows are active and the column is
    // free, an exact zero otherwise
    double gA[PT::NMAX_K > 0 ? PT::NMAX_K : 1];
    PHX_UNROLL for (int k = 0; k < PT::nnz(); ++k) gA[k] = D.A(k) * am.rR[PT::row(k)];
    PHX_UNROLL for (int t = 0; t < PT::npairs(); ++t) {
        const int ka = PT::pair_a(t), kb = PT::pair_b(t), j = PT::col(ka);
        K.M[PT::pair_pos(t)] += gA[ka] * (K.Hinv(j) * am.fF[j]) * gA[kb];
    }
    if (!cholesky<PT>(K.M)) { PHX_LANE_FAIL(10, -1); return false; }
    return true;
}

// Iterative refinement on the regularised system from (xp, z) towards the KKT
// solution for the right-hand side given by R: R.q(j) linear term, R.xb(j)
// value of a non-free column, R.b(i) the active side of row i (a
// proximal-point iteration: it converges to the solution nearest the start on
// degenerate faces).
// The column residual g = -q - P x - A'z (P: the prox weights of the nonant
// columns) of the right-hand side R at (xp, z).
template <class PT, class RHS>
PHX_LD void col_residual(const Data<PT>& D, const RHS& R, const double* xp, const double* z, double* g) {
    double atz[PT::NMAX_N];
    D.matvec_t(z, atz);
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j)
        g[j] = (PT::col_slot(j) >= 0 ? -R.q(j) - D.p(j) * xp[j] : -R.q(j)) - atz[j];
}

// LEAN (the two-wave fused build): the free-column and active-row multipliers
// of each step from the active set's bit words (read through an opaque copy
// per step) instead of 19 doubles held live across the steps -- the same
// values, so the same bits; 44 -> 20 B of scratch per lane there (offline ISA)
template <class PT, class RHS, bool CARRY = PHX_CARRY_DEF, bool LEAN = false>
PHX_LD void kkt_refine(const Data<PT>& D, const AMul<PT>& am, const KFactor<PT>& K, const RHS& R, double* xp,
                       double* z) {
    constexpr int NN = PT::NMAX_N, MM = PT::NMAX_M;
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) xp[j] = am.fF[j] != 0.0 ? xp[j] : R.xb(j);
    PHX_UNROLL for (int i = 0; i < PT::m(); ++i) z[i] *= am.rR[i];
    // the free columns as a multiplier, once: hf = H^-1 on free columns and 0
    // elsewhere; the column loops then run without selects (non-free
    // components get exact zero corrections, so xp keeps its bound values bit
    // for bit); the active rows' right-hand sides (finite: R.b's finite side)
    double hf[NN], bR[MM];
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) hf[j] = am.fF[j] * K.Hinv(j);
    PHX_UNROLL for (int i = 0; i < PT::m(); ++i) bR[i] = R.b(i);
#ifdef PHX_REFINE_PREDICT
    double dprev2 = 1e300;
#endif
    // x2, the stop's scale, is the first step's (the step that moves the
    // point; the later ones change it by the refinement's corrections only).
    double x2 = 0.0;
    // CARRY: the column residual from the data once; after a step it is reg d
    // exactly -- (P + reg) d = g - A'dz on the free columns, so -q - P x' - A'z'
    // = g - P d - A'dz = reg d (the others are multiplied by hf = 0) -- and is
    // carried to the next step instead of a transposed mat-vec per step.
    // (Carrying A'z instead kept 12 more values live across the loop, 12 -> 72 B
    // of scratch in the warm kernel, r04; g replaces the step's own g.  The
    // two-wave fused build recomputes it: carried, it spilled more, r05 s42.)
    double g[NN];
    if (CARRY) col_residual<PT>(D, R, xp, z, g);
    PHX_REFINE_LOOP for (int it = 0; it < KKT_REFINE; ++it) {
        if (!CARRY) col_residual<PT>(D, R, xp, z, g);
        double t[MM];
        const auto fbo = opaque_u32(am.fb);
        const uint32_t rbo = opaque_u32(am.rb);
        auto hfj = [&](int j) -> double { return LEAN ? bitd(fbo, j) * K.Hinv(j) : hf[j]; };
        auto rRi = [&](int i) -> double { return LEAN ? bitd(rbo, i) : am.rR[i]; };
        {
            // t = A_R (xp + H_F g) - b_R: one mat-vec of the sum (the same
            // rounding as the two products it replaces, to eps |A| |x|)
            double u[NN], au[MM];
            PHX_UNROLL for (int j = 0; j < PT::n(); ++j) u[j] = fma(g[j], hfj(j), xp[j]);
            D.matvec(u, au);
            PHX_UNROLL for (int i = 0; i < PT::m(); ++i) t[i] = rRi(i) * (au[i] - bR[i]);
        }
        chol_solve_inv<PT>(K.M, t);   // inactive rows: identity, t stays 0
        double atdz[NN];
        D.matvec_t(t, atdz);
        double d2 = 0.0;
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
            const double d = (g[j] - atdz[j]) * hfj(j);
            xp[j] += d;
            d2 += d * d;
            if (CARRY) g[j] = KKT_REG * d;
        }
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
            z[i] += t[i];
            d2 += t[i] * t[i];
        }
        if (it == 0) {
            PHX_UNROLL for (int j = 0; j < PT::n(); ++j) x2 += xp[j] * xp[j];
            PHX_UNROLL for (int i = 0; i < PT::m(); ++i) x2 += z[i] * z[i];
        }
        PHX_LANE_STAT(1);
        // stop once the correction vanishes (1e-10 relative, in squared 2-norms:
        // |d|^2 <= stop^2 (1 + |x|^2)): the certificate's tolerance is
        // relative to the problem's scale, so it cannot stand in for this (a
        // looser stop, 1e-5, passed certificates at 1e-7 accuracy).  (Skipping
        // the confirming step on a predicted geometric contraction was tried:
        // it leaves errors at the stop's scale, 1e-9 in aircond's W; so was
        // stopping when a step does not contract: on degenerate LPs the
        // refinement is not monotone, and the cut rounds moved the active set
        // to another optimal vertex.)
        const double tol2 = KKT_STOP * KKT_STOP * (1.0 + x2);
        PHX_REFINE_HOOK(it, d2, tol2);
        if (d2 <= tol2) break;
#ifdef PHX_REFINE_PREDICT
        // (opt-in, measured and not adopted, r04) The refinement contracts
        // geometrically (emulation, farmer: relative corrections 1e-0.3,
        // 1e-4.1, 1e-7.8, 1e-11.6 over a 4-step solve); stopping once the
        // PREDICTED next correction, (d / d_prev) d, passes the stop saves the
        // confirming step (3.67 -> 2.7 steps per round) but leaves errors at the
        // stop's scale instead of 1e-4 below it: 6e-10 in aircond's W, and
        // x-bar points whose rows are violated by ~1e-9 relative, which a
        // fixed-nonant evaluation of x-bar (the x-bar inner bound) rejects.
        if (d2 <= 1e-12 * (1.0 + x2) && d2 <= 1e-4 * dprev2 && d2 * d2 <= tol2 * dprev2) break;
        dprev2 = d2;
#endif
    }
}

// right-hand sides: the lane's own problem; the affine parts of the map
// (xb: the value of a non-free column; b: the active side of a row -- both
// always finite, chosen by the finiteness structure where it decides: a
// non-free column sits at a finite bound and an active row at a finite side,
// so only where both are finite does the active set's bit select; the value
// for a free column / inactive row is never used, only multiplied by 0)
template <class PT>
PHX_LD double bound_of(const Data<PT>& D, const ASet<PT>& a, int j) {
    if (PT::lfin(j) && PT::ufin(j)) return a.up(j) ? D.u(j) : D.l(j);
    return PT::ufin(j) ? D.u(j) : (PT::lfin(j) ? D.l(j) : 0.0);
}
template <class PT>
PHX_LD double side_of(const Data<PT>& D, const ASet<PT>& a, int i) {
    if (PT::blfin(i) && PT::bufin(i)) return a.lo(i) ? D.bl(i) : D.bu(i);
    return PT::blfin(i) ? D.bl(i) : (PT::bufin(i) ? D.bu(i) : 0.0);
}
template <class PT>
struct RhsFull {
    const Data<PT>& D;
    const ASet<PT>& a;
    PHX_LD double q(int j) const { return D.q(j); }
    PHX_LD double xb(int j) const { return bound_of<PT>(D, a, j); }
    PHX_LD double b(int i) const { return side_of<PT>(D, a, i); }
};
template <class PT>
struct RhsBase {      // the PH terms off: q = c
    const Data<PT>& D;
    const ASet<PT>& a;
    PHX_LD double q(int j) const { return D.c(j); }
    PHX_LD double xb(int j) const { return bound_of<PT>(D, a, j); }
    PHX_LD double b(int i) const { return side_of<PT>(D, a, i); }
};
template <class PT>
struct RhsSlot {      // d/dqn[t]: unit linear term on slot t's column, homogeneous otherwise
    const Data<PT>& D;
    int t;
    PHX_LD double q(int j) const { return PT::col_slot(j) == t ? D.dc(j) : 0.0; }
    PHX_LD double xb(int) const { return 0.0; }
    PHX_LD double b(int) const { return 0.0; }
};

// Equality-constrained KKT solve for the active set a:
//      [ P_FF   A_RF' ] [x_F]   [ -q_F        ]
//      [ A_RF   0     ] [ z ] = [ b_R - A_RB x_B ]     (z = -y_R)
// by its quasi-definite regularisation (P+reg, -reg) and iterative refinement
// from the given (xp, z).  Non-free columns are set to their bound.  false if
// the Schur complement is not positive definite.
template <class PT, bool CARRY = PHX_CARRY_DEF, bool LEAN = false>
PHX_LD bool kkt_solve(const Data<PT>& D, const ASet<PT>& a, double* xp, double* z) {
    KFactor<PT> K;
    const AMul<PT> am(a);
#ifdef PHX_EXP_FACTOR_TWICE
    // (measurement builds, PHX_LANE_DEFS: the factor's share of a round)
    (void)kkt_factor<PT>(D, am, K);
    PHX_UNROLL for (int t = 0; t < PT::NMAX_M * (PT::NMAX_M + 1) / 2; ++t) opaque(K.M[t]);
#endif
    if (!kkt_factor<PT>(D, am, K)) return false;
#ifdef PHX_EXP_REFINE_TWICE
    // (... and the refinement's: run from the same start twice)
    {
        double x0[PT::NMAX_N], z0[PT::NMAX_M];
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) x0[j] = xp[j];
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) z0[i] = z[i];
        kkt_refine<PT>(D, am, K, RhsFull<PT>{D, a}, xp, z);
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) { opaque(xp[j]); xp[j] = x0[j]; }
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) { opaque(z[i]); z[i] = z0[i]; }
    }
#endif
    kkt_refine<PT, RhsFull<PT>, CARRY, LEAN>(D, am, K, RhsFull<PT>{D, a}, xp, z);
    return true;
}

// ---------------------------------------------------------------------------
// Affine solution map of one active set.  With the active set and the prox
// weights p fixed, the KKT solution is affine in the nonant linear terms qn:
//      (x, z) = (x0, z0) + sum_t qn[t] (gx_t, gz_t)
// PH changes only qn (W and x-bar) from one iteration to the next, and after
// the first few iterations the active set stays put, so a warm solve becomes
// this evaluation plus the KKT certificate — no factorisation, no refinement.
// Stored per lane (scenario-minor words): [x0 (n) | z0 (m) | gx,gz per slot |
// p per slot]; trusted when FLAG_MAP is set and p is bitwise the same.
// ---------------------------------------------------------------------------
template <class PT>
PHX_LD constexpr int map_words() { return (PT::n() + PT::m()) * (PT::nslot() + 1) + PT::nslot(); }

template <class PT>
PHX_LD bool map_compute(const Data<PT>& D, const ASet<PT>& a, const LaneIO& io, int sc) {
    constexpr int NN = PT::NMAX_N, MM = PT::NMAX_M;
    const int64_t S = io.S;
    const int W = PT::n() + PT::m();
    KFactor<PT> K;
    const AMul<PT> am(a);
    if (!kkt_factor<PT>(D, am, K)) return false;
    PHX_NOUNROLL for (int t = -1; t < PT::nslot(); ++t) {
        double xp[NN], z[MM];
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) xp[j] = 0.0;
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) z[i] = 0.0;
        if (t < 0) kkt_refine<PT>(D, am, K, RhsBase<PT>{D, a}, xp, z);
        else kkt_refine<PT>(D, am, K, RhsSlot<PT>{D, t}, xp, z);
        double* m = io.map + (int64_t)(t + 1) * W * S + sc;
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) m[(int64_t)j * S] = xp[j];
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) m[(int64_t)(PT::n() + i) * S] = z[i];
    }
    double* mp = io.map + (int64_t)(PT::nslot() + 1) * W * S + sc;
    PHX_UNROLL for (int t = 0; t < PT::nslot(); ++t) mp[(int64_t)t * S] = D.pn[t];
    return true;
}

// (x, z) from the map; false if the map does not apply (different p)
template <class PT>
PHX_LD bool map_apply(const Data<PT>& D, const LaneIO& io, int sc, double* xp, double* z) {
    const int64_t S = io.S;
    const int W = PT::n() + PT::m();
    const double* mp = io.map + (int64_t)(PT::nslot() + 1) * W * S + sc;
    bool same = true;
    PHX_UNROLL for (int t = 0; t < PT::nslot(); ++t) same = same && mp[(int64_t)t * S] == D.pn[t];
    if (!same) return false;
    const double* m0 = io.map + sc;
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) xp[j] = m0[(int64_t)j * S];
    PHX_UNROLL for (int i = 0; i < PT::m(); ++i) z[i] = m0[(int64_t)(PT::n() + i) * S];
    PHX_UNROLL for (int t = 0; t < PT::nslot(); ++t) {
        const double q = D.qn[t];
        const double* mt = io.map + (int64_t)(t + 1) * W * S + sc;
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) xp[j] += q * mt[(int64_t)j * S];
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) z[i] += q * mt[(int64_t)(PT::n() + i) * S];
    }
    return true;
}

// The largest violation among the flagged changes (kind * 64 + index; kinds:
// 0/1 column to its lower/upper bound, 2 column freed, 3/4 row to its
// lower/upper side, 5 row released): the larger of the largest relative
// primal violation and the largest relative wrong-signed multiplier.
template <class PT, class CM>
PHX_LD int worst_violation(const Data<PT>& D, CM enter_lo, CM enter_up, CM leave, uint32_t act_lo, uint32_t act_up,
                           uint32_t drop, const double* xp, const double* z, double qmax) {
    const double idt = 1.0 / (1.0 + qmax);
    double bp = -1.0, bd = -1.0;
    int kp = -1, kd = -1;
    double atz[PT::NMAX_N], axp[PT::NMAX_M];
    D.matvec_t(z, atz);
    D.matvec(xp, axp);
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
        const double d = D.dc(j);
        const double lam = (D.qpx(j, xp[j]) + atz[j]) * D.idc(j);
        if (PT::lfin(j)) {
            const double v = (D.l(j) - xp[j]) * d * rcp_step(1.0 + fabs(D.l(j) * d));
            const bool f = ((enter_lo >> j) & 1) && v > bp;
            kp = f ? j : kp;
            bp = f ? v : bp;
        }
        if (PT::ufin(j)) {
            const double v = (xp[j] - D.u(j)) * d * rcp_step(1.0 + fabs(D.u(j) * d));
            const bool f = ((enter_up >> j) & 1) && v > bp;
            kp = f ? 64 + j : kp;
            bp = f ? v : bp;
        }
        const double v = fabs(lam) * idt;
        const bool f = ((leave >> j) & 1) && v > bd;
        kd = f ? 128 + j : kd;
        bd = f ? v : bd;
    }
    PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
        const double id = D.idr(i);
        if (PT::blfin(i)) {
            const double v = (D.bl(i) - axp[i]) * id * rcp_step(1.0 + fabs(D.bl(i) * id));
            const bool f = ((act_lo >> i) & 1u) && v > bp;
            kp = f ? 192 + i : kp;
            bp = f ? v : bp;
        }
        if (PT::bufin(i)) {
            const double v = (axp[i] - D.bu(i)) * id * rcp_step(1.0 + fabs(D.bu(i) * id));
            const bool f = ((act_up >> i) & 1u) && v > bp;
            kp = f ? 256 + i : kp;
            bp = f ? v : bp;
        }
        const double v = fabs(z[i] * D.dr(i)) * idt;
        const bool f = ((drop >> i) & 1u) && v > bd;
        kd = f ? 320 + i : kd;
        bd = f ? v : bd;
    }
    // the larger of the two (both relative): on aircond's rescue rounds the
    // slowest lanes need 13-17 single changes instead of 21-26 with the
    // primal violation always first (emulation, 1,000 scenarios; C4 steady
    // step 167 -> 148 us, r04_s26); farmer's rounds are the same.
    // (PHX_SINGLE_PRIMAL_FIRST: the round-3 rule; PHX_SINGLE_DUAL_FIRST: the
    // multiplier first -- fewer rounds on aircond still, but more cold lanes
    // after farmer's seeded Iter0.)
#if defined(PHX_SINGLE_PRIMAL_FIRST)
    return kp >= 0 ? kp : kd;
#elif defined(PHX_SINGLE_DUAL_FIRST)
    return kd >= 0 ? kd : kp;
#else
    return kp >= 0 && (kd < 0 || bp >= bd) ? kp : kd;
#endif
}

// Bounded multi-change update: the flagged changes whose relative violation is
// at least theta times the largest one (worst_violation's measures) -- between
// the full primal-dual update and a single change.  Used for the first
// PT::multi_rounds() rounds after single_after when the problem's lane
// structure sets PT::multi_theta() > 0 (phx_jit.h LaneStructure; a constexpr 0
// compiles it out).  Aircond 10x10x10 (C4): the early iterations' rescue rounds
// of single changes on 1-3 lanes set phx_lane_all's time; with theta 0.2 for
// 4 rounds the step went 0.121 -> 0.111 ms (r06 s20, two pairs on one box).
template <class PT, class CM>
PHX_LD void multi_violations(const Data<PT>& D, CM& enter_lo, CM& enter_up, CM& leave, uint32_t& act_lo,
                             uint32_t& act_up, uint32_t& drop, const double* xp, const double* z, double qmax,
                             double theta) {
    const double idt = 1.0 / (1.0 + qmax);
    double atz[PT::NMAX_N], axp[PT::NMAX_M];
    D.matvec_t(z, atz);
    D.matvec(xp, axp);
    double vlo[PT::NMAX_N], vup[PT::NMAX_N], vlv[PT::NMAX_N], rlo[PT::NMAX_M], rup[PT::NMAX_M], rdr[PT::NMAX_M];
    double mx = 0.0;
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
        const double d = D.dc(j);
        const double lam = (D.qpx(j, xp[j]) + atz[j]) * D.idc(j);
        vlo[j] = vup[j] = -1.0;
        if (PT::lfin(j) && ((enter_lo >> j) & 1)) vlo[j] = (D.l(j) - xp[j]) * d / (1.0 + fabs(D.l(j) * d));
        if (PT::ufin(j) && ((enter_up >> j) & 1)) vup[j] = (xp[j] - D.u(j)) * d / (1.0 + fabs(D.u(j) * d));
        vlv[j] = ((leave >> j) & 1) ? fabs(lam) * idt : -1.0;
        mx = fmax(mx, fmax(vlo[j], fmax(vup[j], vlv[j])));
    }
    PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
        const double id = D.idr(i);
        rlo[i] = rup[i] = -1.0;
        if (PT::blfin(i) && ((act_lo >> i) & 1u)) rlo[i] = (D.bl(i) - axp[i]) * id / (1.0 + fabs(D.bl(i) * id));
        if (PT::bufin(i) && ((act_up >> i) & 1u)) rup[i] = (axp[i] - D.bu(i)) * id / (1.0 + fabs(D.bu(i) * id));
        rdr[i] = ((drop >> i) & 1u) ? fabs(z[i] * D.dr(i)) * idt : -1.0;
        mx = fmax(mx, fmax(rlo[i], fmax(rup[i], rdr[i])));
    }
    const double cut = theta * mx;
    CM el = 0, eu = 0, lv = 0;
    uint32_t al = 0, au = 0, dr = 0;
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
        el |= (CM)(vlo[j] >= cut && vlo[j] >= 0.0) << j;
        eu |= (CM)(vup[j] >= cut && vup[j] >= 0.0) << j;
        lv |= (CM)(vlv[j] >= cut && vlv[j] >= 0.0) << j;
    }
    PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
        al |= (uint32_t)(rlo[i] >= cut && rlo[i] >= 0.0) << i;
        au |= (uint32_t)(rup[i] >= cut && rup[i] >= 0.0) << i;
        dr |= (uint32_t)(rdr[i] >= cut && rdr[i] >= 0.0) << i;
    }
    enter_lo = el; enter_up = eu; leave = lv; act_lo = al; act_up = au; drop = dr;
}

// KKT certificate of (xp, z) for active set a (unscaled, relative kkt_tol);
// on failure applies the primal-dual active-set update (violated bounds/rows
// enter, wrong-signed multipliers leave).  Returns 0 certified, 1 active set
// changed, 2 not certified and nothing to change.
// single: change only the worst violation (worst_violation: the largest
// relative primal violation or wrong-signed multiplier) -- the anti-cycling
// fallback of the later rounds: the full primal-dual update can cycle on
// degenerate LP faces, one change at a time walks them like a pivot.
template <class PT>
PHX_LD int certify_update(const Data<PT>& D, ASet<PT>& a, const double* xp, const double* z, double kkt_tol,
                          bool single = false, bool multi = false) {
    typedef typename ASet<PT>::CMask CM;
    double qmax = 0.0;
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) qmax = fmax(qmax, fabs(D.q(j) * D.idc(j)));
    const double dtol = kkt_tol * (1.0 + qmax);
    const double ptol = kkt_tol;
    // branch-free: violations are gathered into bit masks, applied at the end;
    // each condition is a 0/1 integer in a vector register (vbit), never a
    // live lane mask
    uint32_t bad = 0;                 // a violation the active set cannot fix
    CM enter_lo = 0, enter_up = 0, leave = 0;
    double atz[PT::NMAX_N];
    D.matvec_t(z, atz);
    // a non-finite point (an infeasible subproblem's refinement can diverge)
    // fails every comparison below, i.e. would pass them all: 0 * v is 0 for
    // finite v only, so fin stays 0 exactly when every multiplier and row
    // activity is finite
    double fin = 0.0;
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
        const double d = D.dc(j);
        const double lam = (D.qpx(j, xp[j]) + atz[j]) * D.idc(j);
        fin = fma(lam, 0.0, fin);
        const uint32_t F = (uint32_t)(a.f >> j) & 1u, U = (uint32_t)(a.u >> j) & 1u;
        uint32_t below = 0, above = 0;
        if (PT::lfin(j)) {
            const double lo = D.l(j);
            below = F & vbit(xp[j] < lo && (lo - xp[j]) * d > ptol * (1.0 + fabs(lo * d)));
        }
        if (PT::ufin(j)) {
            const double hi = D.u(j);
            above = F & (below ^ 1u) & vbit(xp[j] > hi && (xp[j] - hi) * d > ptol * (1.0 + fabs(hi * d)));
        }
        bad |= F & ((below | above) ^ 1u) & vbit(fabs(lam) > dtol);
        const uint32_t lv = PT::fixed(j) ? 0u : (F ^ 1u) & ((U & vbit(lam > dtol)) | ((U ^ 1u) & vbit(lam < -dtol)));
        enter_lo |= (CM)below << j;
        enter_up |= (CM)above << j;
        leave |= (CM)lv << j;
    }
    uint32_t act_lo = 0, act_up = 0, drop = 0;
    double axp[PT::NMAX_M];
    D.matvec(xp, axp);
    PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
        const double d = D.dr(i), id = D.idr(i);
        fin = fma(axp[i], 0.0, fma(z[i], 0.0, fin));
        const uint32_t R = (a.r >> i) & 1u, L = (a.l >> i) & 1u;
        uint32_t below = 0, above = 0;
        if (PT::blfin(i)) {
            const double lo = D.bl(i);
            below = vbit(axp[i] < lo && (lo - axp[i]) * id > ptol * (1.0 + fabs(lo * id)));
        }
        if (PT::bufin(i)) {
            const double hi = D.bu(i);
            above = vbit(axp[i] > hi && (axp[i] - hi) * id > ptol * (1.0 + fabs(hi * id)));
        }
        bad |= R & (below | above);
        const double yy = -z[i] * d;
        const uint32_t dr = PT::eq(i) ? 0u : R & ((L & vbit(yy < -dtol)) | ((L ^ 1u) & vbit(yy > dtol)));
        act_lo |= ((R ^ 1u) & below) << i;
        act_up |= ((R ^ 1u) & (below ^ 1u) & above) << i;
        drop |= dr << i;
    }
    if (!(fin == 0.0)) return 2;      // not certified, and no update can repair it
    const bool changed = (enter_lo | enter_up | leave) != 0 || (act_lo | act_up | drop) != 0;
    if (PT::multi_theta() > 0.0 && multi && changed) {
        multi_violations<PT>(D, enter_lo, enter_up, leave, act_lo, act_up, drop, xp, z, qmax, PT::multi_theta());
    } else if (single && changed) {
        // (the rare path: the violations' sizes are recomputed here so the
        // common certificate carries none of this)
        const int code = worst_violation<PT>(D, enter_lo, enter_up, leave, act_lo, act_up, drop, xp, z, qmax);
        const int kind = code >> 6, ix = code & 63;
        enter_lo = kind == 0 ? (CM)1 << ix : (CM)0;
        enter_up = kind == 1 ? (CM)1 << ix : (CM)0;
        leave = kind == 2 ? (CM)1 << ix : (CM)0;
        act_lo = kind == 3 ? 1u << ix : 0u;
        act_up = kind == 4 ? 1u << ix : 0u;
        drop = kind == 5 ? 1u << ix : 0u;
    }
    // primal-dual active-set update: violated bounds / rows enter, wrong-signed
    // multipliers leave
    a.f = (a.f & ~(enter_lo | enter_up)) | leave;
    a.u = (a.u & ~(enter_lo | leave)) | enter_up;
    a.r = (a.r | act_lo | act_up) & ~drop;
    a.l = (a.l & ~act_up) | act_lo;
    return changed ? 1 : (bad != 0 ? 2 : 0);
}

// KKT solve / certificate / active-set update rounds from (a, xp, z): full
// primal-dual updates for the first io.single_after rounds, single changes
// after (certify_update).
// The lane's data (Data) is loaded afresh in every round, through an index the
// optimiser cannot see through (opaque_index): loaded once before the loop, it
// and the round's pair products / reciprocals hoisted with it stayed live
// across the loop, spilled ~200 B of scratch per lane and doubled the warm
// kernel's memory traffic; re-read, it comes from L2.
// D0: the first round's data when the caller has it in registers already
// (the fused kernel); write_its >= 0: a certified lane's outputs are written
// here from the certifying round's data (write_certified, no reload), and with
// pc its x-bar partials [sum pc x | sum pc x^2 per slot] are added to part.
template <class PT>
PHX_LD void write_certified(const LaneIO& io, const Data<PT>& D, int sc, const ASet<PT>& a, const double* xp,
                            const double* z, int its, bool map_ok = false);
// One round with the given data: KKT solve, certificate, active-set update
// (0 certified, 1 active set changed, 2 not certified and nothing to change,
// 3 the Schur complement was not positive definite).
template <class PT, bool CARRY = PHX_CARRY_DEF, bool LEAN = false>
PHX_LD int as_round(const LaneIO& io, const Data<PT>& D, ASet<PT>& a, double* xp, double* z, int r) {
    PHX_LANE_STAT(0);
    if (!kkt_solve<PT, CARRY, LEAN>(D, a, xp, z)) return 3;
    // the first PT::multi_rounds() rounds after single_after: bounded updates
    // (when the structure sets them)
    return certify_update<PT>(D, a, xp, z, io.kkt_tol, r >= io.single_after,
                              PT::multi_theta() > 0.0 && r >= io.single_after &&
                                  r < io.single_after + PT::multi_rounds());
}
// r0: the index of the first round (the fused kernel runs round 0 itself)
// (a certified lane is written by the caller from re-loaded data: writing it
// inside the loop kept the round's data live through the outputs and spilled
// ~400 B per lane, r04)
template <class PT>
PHX_LD bool as_rounds(const LaneIO& io, int sc, ASet<PT>& a, int rounds, double* xp, double* z, int r0 = 0) {
    PHX_NOUNROLL for (int r = r0; r < rounds; ++r) {
        const Data<PT> D(io, opaque_index(sc));
        const int c = as_round<PT>(io, D, a, xp, z, r);
        if (c == 3) return false;
        if (c == 0) return true;
        if (c == 2) { PHX_LANE_STAT(3); return false; }
    }
    return false;
}
// ... with the round data parked in LDS (pk: Data::PARK x 64 doubles, this
// lane's column threadIdx.x; one wavefront per block) at the first round and
// re-read from there per later round instead of re-loaded from memory: a
// lone lane's rounds (the rescue tails) paid the loads' and the x-bar
// gather's round trips every round.  The same values, so the same results.
#if defined(__HIPCC__) || defined(__HIPCC_RTC__)
template <class PT>
PHX_LD bool as_rounds_pk(const LaneIO& io, int sc, ASet<PT>& a, int rounds, double* xp, double* z, double* pk) {
    const int lane = (int)threadIdx.x;
    if (rounds > 0) {
        const Data<PT> D0(io, sc);
        D0.park(pk, lane);
    }
    PHX_NOUNROLL for (int r = 0; r < rounds; ++r) {
        const Data<PT> D(io, sc, pk, lane);
        const int c = as_round<PT>(io, D, a, xp, z, r);
        if (c == 3) return false;
        if (c == 0) return true;
        if (c == 2) { PHX_LANE_STAT(3); return false; }
    }
    return false;
}
#endif

// ---------------------------------------------------------------------------
// Iter0 seeding (phx_kernels.hip enqueue_seeded_solve): T template lanes spread
// over the batch are solved cold first; every other lane starts its warm
// rounds from the active set of the template whose scenario data are nearest
// to its own -- the scenario-varying numbers (A values, and c / bounds / row
// bounds where they vary), each coordinate divided by its range over the
// templates, squared distance.  Templates that did not certify (status != 1)
// are skipped; -1 if none did.  The loop over templates is wave-uniform, so the
// template data are scalar loads.
// ---------------------------------------------------------------------------
constexpr int SEED_T_MAX = 64;    // template lanes at most (one wavefront)

template <class PT>
PHX_LD constexpr int seed_coords() {
    return PT::nvar() + (PT::c_vary() ? PT::n() : 0) + (PT::bnd_vary() ? 2 * PT::n() : 0) +
           (PT::rhs_vary() ? 2 * PT::m() : 0);
}

template <class PT>
PHX_LD double seed_coord(const LaneIO& io, int e, int sc) {
    const int64_t S = io.S;
    if (e < PT::nvar()) return io.Av[(int64_t)e * S + sc];
    e -= PT::nvar();
    if (PT::c_vary()) {
        if (e < PT::n()) return io.c[(int64_t)e * S + sc];
        e -= PT::n();
    }
    if (PT::bnd_vary()) {
        if (e < PT::n()) return io.lb[(int64_t)e * S + sc];
        e -= PT::n();
        if (e < PT::n()) return io.ub[(int64_t)e * S + sc];
        e -= PT::n();
    }
    if (e < PT::m()) return io.bl[(int64_t)e * S + sc];
    return io.bu[(int64_t)(e - PT::m()) * S + sc];
}

constexpr int SEED_LDS = 4096;

template <class PT>
PHX_LD constexpr int seed_templates_staged() {
    return seed_coords<PT>() == 0 ? SEED_T_MAX
                                  : (SEED_T_MAX * seed_coords<PT>() <= SEED_LDS ? SEED_T_MAX
                                                                                : SEED_LDS / seed_coords<PT>());
}

template <class PT>
PHX_LD int nearest_template(const LaneIO& io, int sc, const int32_t* tl, int T) {
    constexpr int NCMAX = PT::NMAX_V + 3 * PT::NMAX_N + 2 * PT::NMAX_M;   // (entries past NC are dead)
    const int NC = seed_coords<PT>();
    int best = -1;
    double bd = 0.0;
    double mine[NCMAX], irange[NCMAX];
    PHX_UNROLL for (int e = 0; e < NC; ++e) {
        mine[e] = seed_coord<PT>(io, e, sc);
        double lo = 1e300, hi = -1e300;
        for (int k = 0; k < T; ++k) {
            const double v = seed_coord<PT>(io, e, tl[k]);
            lo = fmin(lo, v);
            hi = fmax(hi, v);
        }
        // (infinite bounds: inf - inf = nan, a coordinate that never differs)
        const double r = hi - lo;
        irange[e] = (r > 0.0 && r < 1e300) ? 1.0 / r : 0.0;
    }
    for (int k = 0; k < T; ++k) {
        const int t = tl[k];
        if (io.status[t] != 1) continue;
        double d = 0.0;
        PHX_UNROLL for (int e = 0; e < NC; ++e) {
            const double v = (seed_coord<PT>(io, e, t) - mine[e]) * irange[e];
            d += v == v ? v * v : 0.0;
        }
        if (best < 0 || d < bd) { best = k; bd = d; }
    }
    return best;
}

// The lane's starting active set: the nearest certified template's words (the
// templates' active sets saved by k_aset_save, [T][words]); unchanged if none.
template <class PT>
PHX_LD void seed_fill(const LaneIO& io, int sc, const int32_t* tl, int T, const uint32_t* tmpl) {
    const int TS = seed_templates_staged<PT>();
    const int k = nearest_template<PT>(io, sc, tl, T < TS ? T : TS);
    if (k < 0) return;
    constexpr int NW = aset_words(PT::NMAX_N, PT::NMAX_M);
    const int nw = aset_words(PT::n(), PT::m());
    (void)NW;
    for (int w = 0; w < nw; ++w) io.aset[(int64_t)w * io.S + sc] = tmpl[(int64_t)k * nw + w];
}

// Certified lane: unscaled outputs, objective (incl. PH terms), active set.
template <class PT>
PHX_LD void write_certified(const LaneIO& io, const Data<PT>& D, int sc, const ASet<PT>& a, const double* xp,
                            const double* z, int its, bool map_ok) {
    const int S = io.S;
    double f = D.kn;
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
        const double xu = xp[j] * D.dc(j);
        PHX_OUT(io.x_out[(int64_t)j * S + sc], xu);
        f += D.c(j) * xp[j];
        if (PT::col_slot(j) >= 0) f += D.qn[PT::col_slot(j)] * xu + 0.5 * D.pn[PT::col_slot(j)] * xu * xu;
    }
    if (io.y_out)
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) PHX_OUT(io.y_out[(int64_t)i * S + sc], -z[i] * D.dr(i));
    PHX_OUT(io.obj_out[sc], f);
    PHX_OUT(io.status[sc], 1);
    PHX_OUT(io.iters[sc], its);
    if (io.status_out) PHX_OUT(io.status_out[sc], 1);
    if (io.iters_out) PHX_OUT(io.iters_out[sc], its);
    PHX_OUT(io.flags[sc], (its > 0 ? (FLAG_WRITTEN | FLAG_IPM_TRIED) : FLAG_WRITTEN) | (map_ok ? FLAG_MAP : 0));
    aset_store<PT>(io, sc, a);
}

// the warm pass's rounds: re-loaded per round, or parked (PK, GPU only)
template <class PT, bool PK>
PHX_LD bool warm_rounds_of(const LaneIO& io, int sc, ASet<PT>& a, double* xp, double* z, double* pk) {
#if defined(__HIPCC__) || defined(__HIPCC_RTC__)
    if constexpr (PK) return as_rounds_pk<PT>(io, sc, a, io.warm_rounds, xp, z, pk);
#endif
    return as_rounds<PT>(io, sc, a, io.warm_rounds, xp, z);
}

// ---------------------------------------------------------------------------
// Kernel bodies.  Both return true if the lane still needs the generic path.
// ---------------------------------------------------------------------------
// REG: every round on the data loaded at entry (one wave per SIMD kernels with
// the whole register file, phx_lane_warm_list: no per-round re-load)
template <class PT, bool MAP = true, bool REG = false, bool PK = false>
PHX_LD bool warm_lane(const LaneIO& io, int sc, double* pk = nullptr) {
    constexpr int NN = PT::NMAX_N, MM = PT::NMAX_M;
    const Data<PT> D(io, sc);
    ASet<PT> a;
    aset_load<PT>(io, sc, a);
    double xp[NN], z[MM];
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) xp[j] = 0.0;
    PHX_UNROLL for (int i = 0; i < PT::m(); ++i) z[i] = 0.0;
    if (MAP && io.map && (io.flags[sc] & FLAG_MAP) && map_apply<PT>(D, io, sc, xp, z)) {
        PHX_LANE_STAT(2);
        // the same active set, so the same certificate as a KKT solve's
        const int c = certify_update<PT>(D, a, xp, z, io.kkt_tol);
        if (c == 0) {
            write_certified<PT>(io, D, sc, a, xp, z, 0, true);
            return false;
        }
        // the active set moved: rounds from the updated set, warm from (xp, z)
    }
    if (REG) {
        PHX_NOUNROLL for (int r = 0; r < io.warm_rounds; ++r) {
            const int c = as_round<PT>(io, D, a, xp, z, r);
            if (c == 0) {
                const bool mok = MAP && io.map && map_compute<PT>(D, a, io, sc);
                write_certified<PT>(io, D, sc, a, xp, z, 0, mok);
                return false;
            }
            if (c != 1) { PHX_LANE_STAT(3); break; }
        }
    } else if (warm_rounds_of<PT, PK>(io, sc, a, xp, z, pk)) {
        const Data<PT> Dc(io, opaque_index(sc));
        const bool mok = MAP && io.map && map_compute<PT>(Dc, a, io, sc);
        write_certified<PT>(io, Dc, sc, a, xp, z, 0, mok);
        return false;
    }
    aset_store<PT>(io, sc, a);   // the updated active set seeds the next pass
    io.status[sc] = 0;
    io.flags[sc] = 0;
    return true;
}

// Affine-map pass (phx_lane_map): the lane's stored map evaluated and
// certified; nothing else, so the kernel stays small (registers, occupancy)
// and streams the maps.  true: the lane goes on to the rounds pass.
template <class PT>
PHX_LD bool map_lane(const LaneIO& io, int sc) {
    constexpr int NN = PT::NMAX_N, MM = PT::NMAX_M;
    if (io.flags[sc] & FLAG_MAP) {
        const Data<PT> D(io, sc);
        double xp[NN], z[MM];
        if (map_apply<PT>(D, io, sc, xp, z)) {
            PHX_LANE_STAT(2);
            ASet<PT> a;
            aset_load<PT>(io, sc, a);
            const int c = certify_update<PT>(D, a, xp, z, io.kkt_tol);
            if (c == 0) {
                write_certified<PT>(io, D, sc, a, xp, z, 0, true);
                return false;
            }
            aset_store<PT>(io, sc, a);   // the rounds pass starts from the updated set
        }
    }
    io.status[sc] = 0;
    io.flags[sc] = 0;
    return true;
}

// The cold solve is two kernels over the same lane list, so neither carries
// the other's live state (together they needed ~740 registers per lane and
// spilled to scratch on every IPM iteration):
//   phx_lane_cold     ipm_lane: the interior point, stored (unscaled) with its
//                     error and iteration count;
//   phx_lane_cold_as  cold_rounds_lane: classify at that point, active-set
//                     rounds, certificate; or the hand-off to the generic path.
template <class PT>
PHX_LD void ipm_lane(const LaneIO& io, int sc) {
    constexpr int NN = PT::NMAX_N, MM = PT::NMAX_M;
    const Data<PT> D(io, sc);
    const int64_t S = io.S;
    double x[NN], y[MM];
    int its = 0;
    // the problem-scaled start first; a lane whose interior point fails from it
    // runs again from the unit start (farmer 1M, emulation: 1 of 10^6 lanes
    // broke down from the scaled start and converged from the unit one; the
    // generic path it was left to took 100 ms for it).  (A loop, so the
    // interior point is inlined once.)
    double err = 1e300;
    for (int attempt = 0; attempt < 2 && !(err < 1e-4); ++attempt) {
        const bool unit = attempt > 0;
        err = ipm_core<PT>(D, io.max_it, io.ipm_tol, x, y, &its, unit ? 1.0 : PHX_IPM_XS_, unit ? 1.0 : PHX_IPM_ZS_,
                           unit ? 1.0 : PHX_IPM_WS_);
    }
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) io.ipm_x[j * S + sc] = x[j];
    PHX_UNROLL for (int i = 0; i < PT::m(); ++i) io.ipm_y[i * S + sc] = y[i];
    io.err[sc] = err;
    io.iters[sc] = its;
    io.flags[sc] = FLAG_IPM_TRIED;
}

template <class PT>
PHX_LD bool cold_rounds_lane(const LaneIO& io, int sc) {
    constexpr int NN = PT::NMAX_N, MM = PT::NMAX_M;
    const int S = io.S;
    double x[NN], y[MM];
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) x[j] = io.ipm_x[(int64_t)j * S + sc];
    PHX_UNROLL for (int i = 0; i < PT::m(); ++i) y[i] = io.ipm_y[(int64_t)i * S + sc];
    const double err = io.err[sc];
    const int its = io.iters[sc];
    // classification tolerances: the interior point's own accuracy, then (a
    // lane whose rounds cycle from that set: degenerate faces) looser ones
#ifndef PHX_COLD_TRIES
#define PHX_COLD_TRIES 3
#endif
    // (each retry strictly looser than the attempt before: one at or below it
    // would repeat the classification that already cycled, a whole round
    // budget for nothing)
    double prev_tol = 0.0;
    for (int attempt = 0; attempt < PHX_COLD_TRIES && err < 1e-4; ++attempt) {
        const double tol = attempt == 0 ? fmin(1e-4, fmax(1e-9, 10.0 * err))
                                        : (attempt == 1 ? fmin(1e-4, fmax(1e-6, 10.0 * prev_tol)) : 1e-4);
        if (attempt > 0 && !(tol > prev_tol)) continue;
        prev_tol = tol;
        ASet<PT> a;
        {
            const Data<PT> D(io, sc);
            classify<PT>(D, x, y, tol, a);
        }
        double xp[NN], z[MM];
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) xp[j] = x[j];
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) z[i] = a.R(i) ? -y[i] : 0.0;
        if (as_rounds<PT>(io, sc, a, io.as_rounds, xp, z)) {
            const Data<PT> D(io, opaque_index(sc));
            const bool mok = io.map && map_compute<PT>(D, a, io, sc);
            write_certified<PT>(io, D, sc, a, xp, z, its > 0 ? its : 1, mok);
            return false;
        }
    }
    // hand the IPM point to the generic PDHG path (which works scaled:
    // x_s = x / dc, y_s = y / dr); a non-finite component (the interior point
    // of an infeasible subproblem can diverge) starts at 0 there instead
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
        const int64_t o = (int64_t)j * S + sc;
        double v = PT::scaled() ? x[j] : x[j] * PT::idcs(j);
        v = (v - v == 0.0) ? v : 0.0;
        io.xT[o] = v; io.x[o] = v; io.x0[o] = v;
    }
    PHX_UNROLL for (int i = 0; i < PT::m(); ++i) {
        const int64_t o = (int64_t)i * S + sc;
        double v = PT::scaled() ? y[i] : y[i] * PT::idrs(i);
        v = (v - v == 0.0) ? v : 0.0;
        io.yT[o] = v; io.y[o] = v; io.y0[o] = v;
    }
    io.status[sc] = 0;
    // an interior point that did not converge (an infeasible subproblem's
    // diverges): the generic path's own interior point runs again, whose
    // multipliers carry the Farkas certificate of infeasibility (phx_core.h
    // finish_lane); a converged one whose rounds failed is not repeated
    if (!(err < 1e-4)) io.flags[sc] = 0;
    return true;
}

// The whole warm solve of one lane in one kernel (phx_lane_all), for
// batches of at most one wavefront per SIMD, where every pass is one
// wavefront's latency whatever its lane count: the warm rounds, then on the
// lanes they leave the rescue rounds (single changes from the updated active
// set), then the interior point and its rounds -- the same per-lane functions
// in the same order as the warm, rescue-list and cold passes, so the same
// results, in one launch instead of four (three of them usually empty).
// true: the lane needs the generic path.
// REG: the rounds on the data loaded at entry (phx_lane_all); false: re-loaded
// per round (phx_lane_all_rl, which the host picks when the register build
// spills -- aircond: 740 B/lane of scratch; PHX_ALL_RELOAD forces it)
#ifdef PHX_ALL_RELOAD
#define PHX_ALL_REG_DEF false
#else
#define PHX_ALL_REG_DEF true
#endif
// PK (with REG false; phx_lane_all_pk): the warm and rescue rounds on data
// parked in LDS (as_rounds_pk; pk: Data::PARK x 64 doubles of the block's LDS)
template <class PT, bool REG = PHX_ALL_REG_DEF, bool PK = false>
PHX_LD bool all_lane(const LaneIO& io, int sc, int rescue, double* pk = nullptr) {
    if (!warm_lane<PT, false, REG, PK>(io, sc, pk)) return false;
    if (rescue > 0) {
        LaneIO io2 = io;
        io2.warm_rounds = rescue;
        io2.single_after = 1;
        if (!warm_lane<PT, false, REG, PK>(io2, sc, pk)) return false;
    }
    LaneIO io3 = io;
    io3.single_after = 1;          // (the cold pass after warm passes: single changes, phx_kernels.hip)
    // the rounds after the classification get the rescue budget, as every cold
    // pass of enqueue_lane_solve (and the emulation's)
    if (io3.as_rounds > 0 && rescue > io3.as_rounds) io3.as_rounds = rescue;
    ipm_lane<PT>(io3, sc);
    return cold_rounds_lane<PT>(io3, sc);
}

// Both halves for one lane (the host emulation; the GPU runs them as two
// kernels over the same list).  true: the lane needs the generic path.
template <class PT>
PHX_LD bool cold_lane(const LaneIO& io, int sc) {
    ipm_lane<PT>(io, sc);
    return cold_rounds_lane<PT>(io, sc);
}

#if defined(__HIPCC__) || defined(__HIPCC_RTC__)
// Inter-workgroup hand-off of the per-block partials (cdna_hip_programming.md
// §6 Guideline 16).  Producer = the guide's recipe R1: payload stored
// write-through (`sc1`: agent-scope relaxed atomic stores, store_wt), drained
// by the storing wave's `s_waitcnt vmcnt(0)`, then ONE lane's agent-scope
// atomic ticket add -- no release fence (R1 needs none: an agent release would
// write back the XCD's L2, ≈1.7 us).  Consumer = the arriving-last workgroup,
// told by the value its add returned: ONE agent-scope acquire
// (`buffer_inv sc1`, ≈1.7 us) before it reads the partials -- the guide's
// always-valid consumer form.  PHX_RELAXED_HANDOFF (opt-in, a JIT define via
// PHX_LANE_DEFS or a compile flag) drops that acquire and relies on the `sc1`
// loads alone: the guide allows it only for hand-offs matching a row of its
// measured table (MI355X_MICROARCH.md, inter-workgroup visibility), whose
// "one workgroup per CU" condition the warm kernel does not meet.
// PHX_FENCED_HANDOFF adds the producer's release fence as well (test hook).
// (the wait after the release: ROCm 7.2 can drop the fence's own, Pitfall 12)
#if defined(PHX_FENCED_HANDOFF) || !defined(__gfx950__)
#define PHX_HANDOFF_RELEASE()                                  \
    do {                                                       \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");     \
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");       \
    } while (0)
#else
#define PHX_HANDOFF_RELEASE() ((void)0)
#endif
// (the acquire's invalidate completes asynchronously: the wait after it holds
// the workgroup barrier that follows until it has, Guideline 16 Rule)
#if defined(PHX_RELAXED_HANDOFF) && defined(__gfx950__) && !defined(PHX_FENCED_HANDOFF)
#define PHX_HANDOFF_ACQUIRE() ((void)0)
#else
#define PHX_HANDOFF_ACQUIRE()                                  \
    do {                                                       \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");     \
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");       \
    } while (0)
#endif
__device__ __forceinline__ void store_wt(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double load_wt(const double* p) {
    return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Returns true (block-uniform) in the block that arrives last.  The partials
// must have been stored with store_wt by thread 0 (the thread that adds).
// Arrivals are sharded over TICKET_SHARDS counters on lines of their own (one
// counter serialises its atomics at ~12 ns each: 391 arrivals on one word cost
// ~5 us); the last arriver of each shard adds to the top counter, whose last
// arriver is the last block overall.  The last block resets every counter.
#define TICKET_SHARDS 8
#define TICKET_STRIDE 32                        // 128-B lines
#define TICKET_SET ((TICKET_SHARDS + 1) * TICKET_STRIDE)
__device__ bool arrive_last(unsigned int* tk, unsigned int nblocks) {
    __shared__ unsigned int s_last;
    if (threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        PHX_HANDOFF_RELEASE();
        const unsigned b = blockIdx.x, k = b % TICKET_SHARDS;
        const unsigned nk = (nblocks - k + TICKET_SHARDS - 1) / TICKET_SHARDS;   // blocks of shard k
        const unsigned nsh = nblocks < TICKET_SHARDS ? nblocks : TICKET_SHARDS;   // non-empty shards
        unsigned last = 0;
        if (__hip_atomic_fetch_add(tk + k * TICKET_STRIDE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
            nk - 1u)
            last = __hip_atomic_fetch_add(tk + TICKET_SHARDS * TICKET_STRIDE, 1u, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT) == nsh - 1u;
        if (last)
            for (int q = 0; q <= TICKET_SHARDS; ++q) tk[q * TICKET_STRIDE] = 0u;
        if (last) PHX_HANDOFF_ACQUIRE();
        s_last = last;
    }
    __syncthreads();
    return s_last != 0u;
}

// Sum over a full wavefront (all 64 lanes active), uniform result: DPP
// moves within rows of 16 lanes (quad perms, half-row and row mirrors), then
// the row broadcasts of lanes 15 and 31 -- VALU-only steps, where __shfl_down
// was a chain of six ds_bpermute round trips through the LDS crossbar per
// value.  A fixed order: bitwise reproducible.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_add(double v) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(u & 0xffffffffull), CTRL, ROWMASK, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, ROWMASK, 0xf, false);
    return v + __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ double wave_sum(double v) {
    v = dpp_add<0xB1, 0xf>(v);     // quad_perm [1,0,3,2]
    v = dpp_add<0x4E, 0xf>(v);     // quad_perm [2,3,0,1]
    v = dpp_add<0x141, 0xf>(v);    // row_half_mirror
    v = dpp_add<0x140, 0xf>(v);    // row_mirror: every lane of a row holds its sum
    v = dpp_add<0x142, 0xa>(v);    // row_bcast:15 into rows 1, 3
    v = dpp_add<0x143, 0xc>(v);    // row_bcast:31 into rows 2, 3: lane 63 holds the total
    // (readlane is 32-bit: a 64-bit argument would be truncated to its low half)
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u & 0xffffffffull), 63);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), 63);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// (one wavefront; vector stores)
__device__ __forceinline__ void tail_copy(const TailCopy& tc) {
    const int t = (int)threadIdx.x;
    if (tc.left_dst && t == 0) tc.left_dst[0] = *(const volatile int32_t*)tc.left_src;
    if (tc.seg_dst)
        for (int g = t; g < tc.nseg; g += (int)blockDim.x) tc.seg_dst[g] = tc.seg_src[g];
    if (tc.exp_dst && t < 3) tc.exp_dst[t] = tc.exp_src[t];
}

__device__ __forceinline__ void publish_progress(IterkProgress* p, int iter, int done, double conv) {
    // relaxed system-scope stores: no fence (a system release would write back
    // and invalidate the L2); the host orders nothing else on this word
    __hip_atomic_store(&p->conv, conv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&p->word, ((uint64_t)(uint32_t)iter << 8) | (uint64_t)done, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

// conv_{it} from the stage buffer (phbase.py:330-343: mean over emulated ranks
// of each rank's mean |x - x-bar|, ranks in order); the stop test
// (phbase.py:914-926).  Uniform over the grid: every block reads the same
// numbers.  Block 0 publishes the decision.  true: stopped.
__device__ __forceinline__ bool fz_decide(const FusedW& f, int it) {
    const double* seg = f.stage + 2 * f.nns + 1;
    double tot = 0.0;
    for (int r = 0; r < f.R; ++r)
        if (f.cnt[r] > 0) tot += seg[r] / f.cnt[r];
    const double conv = tot / f.R;
    const bool done = conv < f.thresh;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (done) {
            f.ctl[1] = it;
            *(volatile int32_t*)f.ctl = 1;
        }
        publish_progress(f.prog, it, done ? 1 : 0, conv);
    }
    return done;
}

// Prologue (block-uniform; before anything is written): the decision on
// conv_{k-1}; then a previous solve that left lanes to the generic path stops
// the pipeline at k (every rank sees the same all-reduced count) before W is
// touched.  Block 0 publishes x-bar_k.
__device__ bool fz_prologue(const LaneIO& io) {
    const FusedW& f = io.fz;
    if (!f.first && fz_decide(f, f.iter - 1)) return false;
    if (f.stage[2 * f.nns] > 0.5) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            f.ctl[1] = f.iter;
            *(volatile int32_t*)f.ctl = 2;
            publish_progress(f.prog, f.iter, 2, 0.0);
        }
        return false;
    }
    if (blockIdx.x == 0)
        for (int e = threadIdx.x; e < 2 * f.nns; e += blockDim.x) f.node_sums[e] = f.stage[e];
    return true;
}

// Update_W for one lane (in place, before its Data reads W): returns the
// lane's sum |x_{k-1} - x-bar_k| over its nonant slots.
// (fused mode: one tree node, node slot = nonant slot -- x-bar of slot t is
// stage[t], no index gather; all loads issued before the stores)
template <class PT>
__device__ double fz_update_w(const LaneIO& io, int sc) {
    const FusedW& f = io.fz;
    const int64_t S = io.S;
    constexpr int NS = PT::nslot() > 0 ? PT::nslot() : 1;
    double xv[NS], wv[NS], rv[NS];
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
        const int t = PT::col_slot(j);
        if (t >= 0) {
            const int64_t o = (int64_t)t * S + sc;
            xv[t] = f.x_prev[(int64_t)j * S + sc];
            wv[t] = io.W[o];
            rv[t] = io.rho[o];
        }
    }
    double d = 0.0;
    PHX_UNROLL for (int t = 0; t < PT::nslot(); ++t) {
        const double diff = xv[t] - f.stage[t];
        PHX_OUT(const_cast<double*>(io.W)[(int64_t)t * S + sc], wv[t] + rv[t] * diff);
        d += fabs(diff);
    }
    return d;
}

// Epilogue: the block's partials [sum pc x | sum pc x^2 per slot | sum |d|]
// (one wavefront: shuffles), stored write-through; the last block of each
// arrival shard folds its shard's blocks (shard = blockIdx % 8, which is the
// XCD the block ran on), the last shard's folder folds the shards and writes
// the stage buffer of iteration k+1 (+ the straggler count of solve k and
// this rank's conv sum).  Fixed order: independent of arrival order.
// (the lane's sum |x_{k-1} - x-bar_k| is recomputed here from memory, the same
// operations in the same order as fz_update_w: carried across the solve it was
// one of the values spilled to scratch)
template <class PT>
__device__ void fz_fold(const LaneIO& io, double* v);
template <class PT>
__device__ void fz_epilogue(const LaneIO& io, int sc, bool still) {
    const FusedW& f = io.fz;
    constexpr int NS = PT::nslot() > 0 ? PT::nslot() : 1;
    constexpr int NV = 2 * NS + 1;
    const int64_t S = io.S;
    double v[NV];
    PHX_UNROLL for (int e = 0; e < NV; ++e) v[e] = 0.0;
    if (sc < io.S) {
        // (the same slot order and operations as fz_update_w)
        double xv[NS];
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
            const int t = PT::col_slot(j);
            if (t >= 0) xv[t] = f.x_prev[(int64_t)j * S + sc];
        }
        double dl = 0.0;
        PHX_UNROLL for (int t = 0; t < PT::nslot(); ++t) dl += fabs(xv[t] - f.stage[t]);
        v[2 * NS] = dl;
        if (!still)
            PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
                const int t = PT::col_slot(j);
                if (t >= 0) {
                    const double xu = io.x_out[(int64_t)j * S + sc];
                    const double w = f.pc[(int64_t)t * S + sc] * xu;
                    v[t] += w;
                    v[NS + t] += w * xu;
                }
            }
    }
    fz_fold<PT>(io, v);
}

// The fold of the lanes' partials v[2 NS + 1] (the wavefront's sums, then the
// blocks' and the shards' in fixed orders).  Every lane of the block calls it.
template <class PT>
__device__ void fz_fold(const LaneIO& io, double* v) {
    const FusedW& f = io.fz;
    constexpr int NS = PT::nslot() > 0 ? PT::nslot() : 1;
    constexpr int NV = 2 * NS + 1;
    PHX_UNROLL for (int e = 0; e < NV; ++e) v[e] = wave_sum(v[e]);
    const unsigned nb = gridDim.x, b = blockIdx.x, k = b % TICKET_SHARDS;
    const unsigned nk = (nb - k + TICKET_SHARDS - 1) / TICKET_SHARDS;
    const unsigned nsh = nb < TICKET_SHARDS ? nb : TICKET_SHARDS;
    double* shard_part = f.part + (int64_t)nb * NV;
    __shared__ unsigned s_state;
    if (threadIdx.x == 0) {
        PHX_UNROLL for (int e = 0; e < NV; ++e) store_wt(&f.part[(int64_t)b * NV + e], v[e]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        PHX_HANDOFF_RELEASE();
        s_state = __hip_atomic_fetch_add(f.tk + k * TICKET_STRIDE, 1u, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT) == nk - 1u;
    }
    __syncthreads();
    if (!s_state) return;
    PHX_HANDOFF_ACQUIRE();
    // last of shard k: blocks k, k+8, ... in order (4 blocks' loads in flight)
    PHX_UNROLL for (int e = 0; e < NV; ++e) v[e] = 0.0;
    for (unsigned i0 = threadIdx.x; i0 < nk; i0 += 4 * 64) {
        double l[4][NV];
        PHX_UNROLL for (int u = 0; u < 4; ++u) {
            const unsigned i = i0 + 64u * u;
            PHX_UNROLL for (int e = 0; e < NV; ++e)
                l[u][e] = i < nk ? load_wt(&f.part[(int64_t)(k + TICKET_SHARDS * i) * NV + e]) : 0.0;
        }
        PHX_UNROLL for (int u = 0; u < 4; ++u) PHX_UNROLL for (int e = 0; e < NV; ++e) v[e] += l[u][e];
    }
    PHX_UNROLL for (int e = 0; e < NV; ++e) v[e] = wave_sum(v[e]);
    __syncthreads();
    if (threadIdx.x == 0) {
        PHX_UNROLL for (int e = 0; e < NV; ++e) store_wt(&shard_part[k * NV + e], v[e]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        PHX_HANDOFF_RELEASE();
        const bool last = __hip_atomic_fetch_add(f.tk + TICKET_SHARDS * TICKET_STRIDE, 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT) == nsh - 1u;
        if (last)
            for (int q = 0; q <= TICKET_SHARDS; ++q) f.tk[q * TICKET_STRIDE] = 0u;
        s_state = last ? 2u : 0u;
    }
    __syncthreads();
    if (s_state != 2u) return;
    PHX_HANDOFF_ACQUIRE();
    // the last block overall: shards in order, then iteration k+1's stage
    const int e = threadIdx.x;
    if (e < NV) {
        double a = 0.0;
        for (unsigned q = 0; q < nsh; ++q) a += load_wt(&shard_part[q * NV + e]);
        if (e < NS) f.stage[e] = a;
        else if (e < 2 * NS) f.stage[f.nns + (e - NS)] = a;
        else {
            for (int r = 0; r < f.R; ++r) f.stage[2 * f.nns + 1 + r] = r == f.g ? a : 0.0;
            f.stage[2 * f.nns] =
                (double)__hip_atomic_load(io.count_out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Iter0 seeding on the GPU (kernel phx_lane_seed, one wavefront per block):
// the same choice as seed_fill / nearest_template, with the template table
// staged once per block in LDS.  Read per lane from global memory, the T x NC
// template coordinates were dependent scalar loads through the template list
// (tl[k], then the value): 124 us for farmer 100k; from LDS, broadcast reads.
// Ranges over all T templates, distances over the certified ones, e ascending:
// the same floating-point sums as nearest_template.  At most SEED_LDS doubles
// are staged: problems with more coordinates per template use fewer templates
// (the first SEED_LDS / NC; the host emulation applies the same cap).
template <class PT>
__device__ void seed_block(const LaneIO& io, const int32_t* tl, int T, const uint32_t* tmpl) {
    constexpr int NC = seed_coords<PT>();
    constexpr int TS = seed_templates_staged<PT>() > 0 ? seed_templates_staged<PT>() : 1;
    constexpr int NCP = NC > 0 ? NC : 1;
    __shared__ double tc[TS * NCP];
    __shared__ double irange[NCP];
    __shared__ int tok[TS];
    const int Tn = T < TS ? T : TS;
    for (int i = threadIdx.x; i < Tn * NC; i += blockDim.x) {
        const int k = i / NCP, e = i - k * NCP;
        tc[i] = seed_coord<PT>(io, e, tl[k]);
    }
    for (int k = threadIdx.x; k < Tn; k += blockDim.x) tok[k] = io.status[tl[k]] == 1;
    __syncthreads();
    for (int e = threadIdx.x; e < NC; e += blockDim.x) {
        double lo = 1e300, hi = -1e300;
        for (int k = 0; k < Tn; ++k) {
            const double v = tc[k * NCP + e];
            lo = fmin(lo, v);
            hi = fmax(hi, v);
        }
        const double r = hi - lo;
        irange[e] = (r > 0.0 && r < 1e300) ? 1.0 / r : 0.0;
    }
    __syncthreads();
    const int sc = blockIdx.x * blockDim.x + threadIdx.x;
    if (sc >= io.S) return;
    double mine[NCP];
    PHX_UNROLL for (int e = 0; e < NC; ++e) mine[e] = seed_coord<PT>(io, e, sc);
    int best = -1;
    double bd = 0.0;
    for (int k = 0; k < Tn; ++k) {
        if (!tok[k]) continue;
        double d = 0.0;
        PHX_UNROLL for (int e = 0; e < NC; ++e) {
            const double v = (tc[k * NCP + e] - mine[e]) * irange[e];
            d += v == v ? v * v : 0.0;
        }
        if (best < 0 || d < bd) { best = k; bd = d; }
    }
    if (best < 0) return;
    const int nw = aset_words(PT::n(), PT::m());
    for (int w = 0; w < nw; ++w) io.aset[(int64_t)w * io.S + sc] = tmpl[(int64_t)best * nw + w];
}

// Compact the lanes that still need work into out[0..*count): one atomic per
// wavefront, lane order kept within the wavefront.  Every lane of the
// wavefront must reach this call.
// Zero the next solve's counters (double-buffered, so no memset launch).
__device__ __forceinline__ void zero_next_counts(int32_t* next) {
    if (next && blockIdx.x == 0 && threadIdx.x < 16) next[threadIdx.x] = 0;
}

__device__ __forceinline__ void compact_lane(bool still, int sc, int32_t* out, int32_t* count) {
    const unsigned long long b = __ballot(still);
    const int lane = threadIdx.x & 63;
    int base = 0;
    if (lane == 0 && b) base = atomicAdd(count, (int32_t)__popcll(b));
    base = __shfl(base, 0, 64);
    if (still) out[base + __popcll(b & ((1ull << lane) - 1ull))] = sc;
}
// A whole fused PH iteration (phx_iterk fused mode, kernel phx_lane_warm_fz).
// Every load of the lane's Update_W and of its first active-set round is
// issued at kernel entry, before the gate and the stop decision are known
// (loads have no effects; a gated launch just drops them): the lane's varying
// A values, its active-set words, and per slot x_{k-1}, W, rho and prob_coeff.
// Update_W then runs in registers and hands the new W straight to the first
// round's data (no re-load of what it just stored); a certified lane's
// outputs and x-bar partials come from the certifying round's registers
// (as_rounds), so the epilogue re-reads nothing.  The same operations as
// phx_lane_warm's fused path (fz_update_w, warm_lane, fz_epilogue).
// REG (the one-wave-per-SIMD build, 512 registers): every round runs on the
// data in registers -- the other builds re-load it per round (kept live across
// the round loop it spilled; a re-load is a memory round trip per round)
// PARK (with REG; the two-wave build): the round data parked in LDS after
// round 0 and re-read per later round (Data::park), and the lean refinement
// steps -- held in registers across the round loop they spilled 144 B per lane
// (1.40x the kernel's algorithmic HBM bytes, r05); the same values, the same bits
template <class PT, bool REG = false, bool CARRY = PHX_CARRY_DEF, bool PARK = false>
__device__ __forceinline__ void warm_fused(const LaneIO& io) {
    const FusedW& f = io.fz;
    constexpr int NS = PT::nslot() > 0 ? PT::nslot() : 1;
    constexpr int NV = 2 * NS + 1;
    constexpr int NVA = PT::NMAX_V, NW = aset_words(PT::NMAX_N, PT::NMAX_M);
    const int sc = blockIdx.x * 64 + threadIdx.x;
    const bool live = sc < io.S;
    const int s = live ? sc : 0;            // (tail lanes load lane 0's values: valid addresses, unused)
    const int64_t S = io.S;
    double av[NVA], xv[NS], wv[NS], rv[NS], pcv[NS];
    uint32_t aw[NW];
    PHX_UNROLL for (int v = 0; v < PT::nvar(); ++v) av[v] = io.Av[(int64_t)v * S + s];
    PHX_UNROLL for (int k = 0; k < aset_words(PT::n(), PT::m()); ++k) aw[k] = io.aset[(int64_t)k * S + s];
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
        const int t = PT::col_slot(j);
        if (t >= 0) {
            const int64_t o = (int64_t)t * S + s;
            xv[t] = f.x_prev[(int64_t)j * S + s];
            wv[t] = io.W[o];
            rv[t] = io.rho[o];
            pcv[t] = f.pc[o];
        }
    }
    lane_stamp(io, 0);
    if (gated(io.gate)) return;
    if (!fz_prologue(io)) return;
    zero_next_counts(io.counts_next);
    lane_stamp(io, 1);
    // Update_W (phbase.py:293-318) and |x_{k-1} - x-bar_k| (convergence_diff)
    double xb[NS], dl = 0.0;
    PHX_UNROLL for (int t = 0; t < PT::nslot(); ++t) {
        xb[t] = f.stage[t];
        const double diff = xv[t] - xb[t];
        wv[t] = wv[t] + rv[t] * diff;
        if (live) PHX_OUT(const_cast<double*>(io.W)[(int64_t)t * S + sc], wv[t]);
        dl += fabs(diff);
    }
    lane_stamp(io, 2);
#ifndef PHX_FZ_NO_LDS_KEEP
    // (values needed only after the solve, parked in LDS across it)
    __shared__ double fz_keep[(NS + 1) * 64];
    PHX_UNROLL for (int t = 0; t < PT::nslot(); ++t) fz_keep[t * 64 + threadIdx.x] = pcv[t];
    fz_keep[NS * 64 + threadIdx.x] = dl;
#endif
    bool still = false;
    double xn[NS];                      // the certified lane's unscaled nonant x
    if (live) {
        ASet<PT> a;
        aset_from_words<PT>(aw, a);
        double xp[PT::NMAX_N], z[PT::NMAX_M];
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) xp[j] = 0.0;
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) z[i] = 0.0;
        // round 0 on the data in registers; later rounds re-load (as_rounds),
        // or with REG stay on them
        int c;
        if (REG && PARK) {
            __shared__ double fz_park[Data<PT>::PARK * 64];
            {
                const Data<PT> D0(io, sc, av, wv, rv, xb);
                D0.park(fz_park, threadIdx.x);
                c = io.warm_rounds > 0 ? as_round<PT, CARRY, true>(io, D0, a, xp, z, 0) : 2;
            }
            int nr = 1;
            PHX_NOUNROLL for (int r = 1; r < io.warm_rounds && c == 1; ++r, ++nr) {
                const Data<PT> Dr(io, sc, fz_park, threadIdx.x);
                c = as_round<PT, CARRY, true>(io, Dr, a, xp, z, r);
            }
            if (io.stamps) {
                int wmax = 0;
                for (int q = 1; q <= 8; ++q) wmax = __ballot(nr >= q) ? q : wmax;
                if (threadIdx.x == 0) io.stamps[(uint64_t)blockIdx.x * 8 + 6] = (uint64_t)wmax;
            }
            if (c == 2) PHX_LANE_STAT(3);
            if (c == 0) {
                const Data<PT> Dw(io, sc, fz_park, threadIdx.x);
                write_certified<PT>(io, Dw, sc, a, xp, z, 0);
            }
        } else if (REG) {
            const Data<PT> D0(io, sc, av, wv, rv, xb);
            c = io.warm_rounds > 0 ? as_round<PT, CARRY>(io, D0, a, xp, z, 0) : 2;
            int nr = 1;
            PHX_NOUNROLL for (int r = 1; r < io.warm_rounds && c == 1; ++r, ++nr) c = as_round<PT, CARRY>(io, D0, a, xp, z, r);
            // (diagnostics: the wavefront's most rounds, PHX_LANE_STAMPS=1)
            if (io.stamps) {
                int wmax = 0;
                for (int q = 1; q <= 8; ++q) wmax = __ballot(nr >= q) ? q : wmax;
                if (threadIdx.x == 0) io.stamps[(uint64_t)blockIdx.x * 8 + 6] = (uint64_t)wmax;
            }
            if (c == 2) PHX_LANE_STAT(3);
            if (c == 0) write_certified<PT>(io, D0, sc, a, xp, z, 0);
        } else {
            {
                const Data<PT> D0(io, sc, av, wv, rv, xb);
                c = io.warm_rounds > 0 ? as_round<PT>(io, D0, a, xp, z, 0) : 2;
                if (c == 0) write_certified<PT>(io, D0, sc, a, xp, z, 0);
            }
            if (c == 1 && as_rounds<PT>(io, sc, a, io.warm_rounds, xp, z, 1)) {
                c = 0;
                const Data<PT> Dc(io, opaque_index(sc));
                write_certified<PT>(io, Dc, sc, a, xp, z, 0);
            }
        }
        if (c != 0) {
            aset_store<PT>(io, sc, a);   // the updated active set seeds the next pass
            io.status[sc] = 0;
            io.flags[sc] = 0;
            still = true;
        } else {
            PHX_UNROLL for (int j = 0; j < PT::n(); ++j)
                if (PT::col_slot(j) >= 0) xn[PT::col_slot(j)] = xp[j] * (PT::scaled() ? PT::dcs(j) : 1.0);
        }
    }
    // the lane's x-bar partials (a certified lane's unscaled x as written) and
    // its convergence term
    double v[NV];
    PHX_UNROLL for (int e = 0; e < NV; ++e) v[e] = 0.0;
#ifndef PHX_FZ_NO_LDS_KEEP
    PHX_UNROLL for (int t = 0; t < PT::nslot(); ++t) pcv[t] = fz_keep[t * 64 + threadIdx.x];
    dl = fz_keep[NS * 64 + threadIdx.x];
#endif
    if (live) {
        v[2 * NS] = dl;
        if (!still)
            PHX_UNROLL for (int t = 0; t < PT::nslot(); ++t) {
                const double w = pcv[t] * xn[t];
                v[t] += w;
                v[NS + t] += w * xn[t];
            }
    }
    lane_stamp(io, 3);
    compact_lane(still, sc, io.lanes_out, io.count_out);
    lane_stamp(io, 4);
    fz_fold<PT>(io, v);
    lane_stamp(io, 5);
}

// ---------------------------------------------------------------------------
// The compacting fused iteration (kernel phx_lane_warm_fzc).  A wavefront's
// time is its slowest lane's: in steady PH iterations ~6 % of the lanes need a
// second active-set round, so nearly every wavefront of warm_fused runs two
// or more rounds for one or two lanes.  Here every block (64 lanes = one
// chunk) runs Update_W and round 0 only; a lane that round 0 leaves with a
// changed active set stashes (xp, z) and its active set, and the LAST block
// of its group (gsize consecutive chunks, told by an arrival counter) runs the
// remaining rounds for the group's rework lanes packed into full wavefronts
// (scenario order: a deterministic assignment), from the very state a single
// wavefront would have continued with -- the same data bits (Data from the
// stored W, rho, A values and stage x-bar), the same round numbers, so the
// same x, y, objective and active set per lane as warm_fused.  Only the x-bar
// fold differs in order: the blocks' partials (round-0 lanes and every lane's
// convergence term) folded as in fz_fold, then the groups' rework partials in
// group order -- fixed orders, bitwise reproducible run to run.
// Hand-offs (stash -> group finisher, partials -> last block): Guideline 16
// R1 (write-through stores drained before one relaxed ticket; the consumer's
// agent acquire), as fz_fold's.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void store_wt_u64(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long load_wt_u64(const unsigned long long* p) {
    return __hip_atomic_load(const_cast<unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long readlane_u64(unsigned long long u, int l) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u & 0xffffffffull), l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
    return ((unsigned long long)hi << 32) | lo;
}
// the position of the r-th (0-based) set bit of w (w has more than r set bits)
__device__ __forceinline__ int nth_set_bit(unsigned long long w, int r) {
    for (int k = 0; k < r; ++k) w &= w - 1ull;
    return (int)__builtin_ctzll(w);
}

// The rework lanes of group g (every lane of the block calls it): packed in
// scenario order into wavefront batches; each lane continues its solve from
// round 1.  gacc: the batches' partials [sum pc x | sum pc x^2] in batch order.
template <class PT>
__device__ void fz_rework_group(const LaneIO& io, int g, double* gacc) {
    const FusedW& f = io.fz;
    constexpr int NS = PT::nslot() > 0 ? PT::nslot() : 1;
    constexpr int NV = 2 * NS + 1;
    constexpr int NVA = PT::NMAX_V, NW = aset_words(PT::NMAX_N, PT::NMAX_M);
    const int64_t S = io.S;
    const int nch = (io.S + 63) / 64;
    const int c0 = g * f.gsize;
    const int ng = min(f.gsize, nch - c0);          // (<= 64: phx_kernels.hip caps gsize)
    const int l = threadIdx.x;
    const unsigned long long mine = l < ng ? load_wt_u64(&f.rmask[c0 + l]) : 0ull;
    // inclusive prefix of the chunks' rework counts over the lanes
    int inc = __popcll(mine);
    PHX_UNROLL for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(inc, d, 64);
        if (l >= d) inc += o;
    }
    const int total = __builtin_amdgcn_readlane(inc, 63);
    const int exc = inc - __popcll(mine);
    PHX_UNROLL for (int e = 0; e < NV; ++e) gacc[e] = 0.0;
    for (int base = 0; base < total; base += 64) {
        const int q = base + l;
        int sc = -1;
        for (int j = 0; j < ng; ++j) {              // wave-uniform: the chunk holding rank q
            const int ej = __builtin_amdgcn_readlane(exc, j), ij = __builtin_amdgcn_readlane(inc, j);
            if (ij > ej && q >= ej && q < ij) sc = (c0 + j) * 64 + nth_set_bit(readlane_u64(mine, j), q - ej);
        }
        bool still = false;
        double v[NV];
        PHX_UNROLL for (int e = 0; e < NV; ++e) v[e] = 0.0;
        if (sc >= 0) {
            double av[NVA], wv[NS], rv[NS], xb[NS], pcv[NS];
            uint32_t aw[NW];
            // (what other blocks of this launch wrote -- W, the active set, the
            // stash -- is read with `sc1` loads: valid with the acquire above
            // and without it, PHX_RELAXED_HANDOFF; the rest is launch-constant)
            PHX_UNROLL for (int k = 0; k < PT::nvar(); ++k) av[k] = io.Av[(int64_t)k * S + sc];
            PHX_UNROLL for (int k = 0; k < aset_words(PT::n(), PT::m()); ++k)
                aw[k] = __hip_atomic_load(io.aset + (int64_t)k * S + sc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            PHX_UNROLL for (int t = 0; t < PT::nslot(); ++t) {
                const int64_t o = (int64_t)t * S + sc;
                wv[t] = load_wt(io.W + o);
                rv[t] = io.rho[o];
                pcv[t] = f.pc[o];
                xb[t] = f.stage[t];
            }
            double xp[PT::NMAX_N], z[PT::NMAX_M];
            PHX_UNROLL for (int j = 0; j < PT::n(); ++j) xp[j] = load_wt(f.rx + (int64_t)j * S + sc);
            PHX_UNROLL for (int i = 0; i < PT::m(); ++i) z[i] = load_wt(f.rz + (int64_t)i * S + sc);
            ASet<PT> a;
            aset_from_words<PT>(aw, a);
            const Data<PT> D(io, sc, av, wv, rv, xb);
            int c = 1;
            PHX_NOUNROLL for (int r = 1; r < io.warm_rounds && c == 1; ++r) c = as_round<PT>(io, D, a, xp, z, r);
            if (c == 0) {
                write_certified<PT>(io, D, sc, a, xp, z, 0);
                PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
                    const int t = PT::col_slot(j);
                    if (t >= 0) {
                        const double xn = xp[j] * (PT::scaled() ? PT::dcs(j) : 1.0);
                        const double w = pcv[t] * xn;
                        v[t] += w;
                        v[NS + t] += w * xn;
                    }
                }
            } else {
                if (c == 2) PHX_LANE_STAT(3);
                aset_store<PT>(io, sc, a);   // the updated active set seeds the next pass
                io.status[sc] = 0;
                io.flags[sc] = 0;
                still = true;
            }
        }
        compact_lane(still, sc, io.lanes_out, io.count_out);
        PHX_UNROLL for (int e = 0; e < NV; ++e) gacc[e] += wave_sum(v[e]);
    }
}

// fz_fold with the groups: the block's partial, its group arrival (the last
// block of the group finishes the group's rework lanes), then the sharded
// block arrival; the last block overall folds the shards, then the groups.
template <class PT>
__device__ void fz_fold_c(const LaneIO& io, double* v) {
    const FusedW& f = io.fz;
    constexpr int NS = PT::nslot() > 0 ? PT::nslot() : 1;
    constexpr int NV = 2 * NS + 1;
    PHX_UNROLL for (int e = 0; e < NV; ++e) v[e] = wave_sum(v[e]);
    const unsigned nb = gridDim.x, b = blockIdx.x, k = b % TICKET_SHARDS;
    const unsigned nk = (nb - k + TICKET_SHARDS - 1) / TICKET_SHARDS;
    const unsigned nsh = nb < TICKET_SHARDS ? nb : TICKET_SHARDS;
    const unsigned gs = (unsigned)f.gsize, g = b / gs;
    const unsigned gn = (nb - g * gs) < gs ? (nb - g * gs) : gs;
    double* shard_part = f.part + (int64_t)nb * NV;
    __shared__ unsigned s_state;
    if (threadIdx.x == 0) {
        PHX_UNROLL for (int e = 0; e < NV; ++e) store_wt(&f.part[(int64_t)b * NV + e], v[e]);
        // (this wavefront's stash, W and active-set stores: all write-through,
        // drained here with the partials before the group ticket)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        PHX_HANDOFF_RELEASE();
        s_state = __hip_atomic_fetch_add(f.gcnt + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gn - 1u;
    }
    __syncthreads();
    if (s_state) {
        PHX_HANDOFF_ACQUIRE();
        if (threadIdx.x == 0) __hip_atomic_store(f.gcnt + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        double ga[NV];
        fz_rework_group<PT>(io, (int)g, ga);
        if (threadIdx.x == 0)
            PHX_UNROLL for (int e = 0; e < NV; ++e) store_wt(&f.gpart[(int64_t)g * NV + e], ga[e]);
    }
    if (threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        PHX_HANDOFF_RELEASE();
        s_state = __hip_atomic_fetch_add(f.tk + k * TICKET_STRIDE, 1u, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT) == nk - 1u;
    }
    __syncthreads();
    if (!s_state) return;
    PHX_HANDOFF_ACQUIRE();
    // last of shard k: blocks k, k+8, ... in order (4 blocks' loads in flight)
    PHX_UNROLL for (int e = 0; e < NV; ++e) v[e] = 0.0;
    for (unsigned i0 = threadIdx.x; i0 < nk; i0 += 4 * 64) {
        double l[4][NV];
        PHX_UNROLL for (int u = 0; u < 4; ++u) {
            const unsigned i = i0 + 64u * u;
            PHX_UNROLL for (int e = 0; e < NV; ++e)
                l[u][e] = i < nk ? load_wt(&f.part[(int64_t)(k + TICKET_SHARDS * i) * NV + e]) : 0.0;
        }
        PHX_UNROLL for (int u = 0; u < 4; ++u) PHX_UNROLL for (int e = 0; e < NV; ++e) v[e] += l[u][e];
    }
    PHX_UNROLL for (int e = 0; e < NV; ++e) v[e] = wave_sum(v[e]);
    __syncthreads();
    if (threadIdx.x == 0) {
        PHX_UNROLL for (int e = 0; e < NV; ++e) store_wt(&shard_part[k * NV + e], v[e]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        PHX_HANDOFF_RELEASE();
        const bool last = __hip_atomic_fetch_add(f.tk + TICKET_SHARDS * TICKET_STRIDE, 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT) == nsh - 1u;
        if (last)
            for (int q = 0; q <= TICKET_SHARDS; ++q) f.tk[q * TICKET_STRIDE] = 0u;
        s_state = last ? 2u : 0u;
    }
    __syncthreads();
    if (s_state != 2u) return;
    PHX_HANDOFF_ACQUIRE();
    // the last block overall: the groups' rework partials (lane-strided, then
    // the wave sum), then the shards in order + the groups: iteration k+1's stage
    const unsigned ngr = (nb + gs - 1) / gs;
    double gsum[NV];
    PHX_UNROLL for (int e = 0; e < NV; ++e) gsum[e] = 0.0;
    for (unsigned q = threadIdx.x; q < ngr; q += 64)
        PHX_UNROLL for (int e = 0; e < NV; ++e) gsum[e] += load_wt(&f.gpart[(int64_t)q * NV + e]);
    PHX_UNROLL for (int e = 0; e < NV; ++e) gsum[e] = wave_sum(gsum[e]);
    const int e = threadIdx.x;
    if (e < NV) {
        double a = 0.0;
        for (unsigned q = 0; q < nsh; ++q) a += load_wt(&shard_part[q * NV + e]);
        double ge = 0.0;
        PHX_UNROLL for (int u = 0; u < NV; ++u) ge = u == e ? gsum[u] : ge;
        a += ge;
        if (e < NS) f.stage[e] = a;
        else if (e < 2 * NS) f.stage[f.nns + (e - NS)] = a;
        else {
            for (int r = 0; r < f.R; ++r) f.stage[2 * f.nns + 1 + r] = r == f.g ? a : 0.0;
            f.stage[2 * f.nns] =
                (double)__hip_atomic_load(io.count_out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

template <class PT>
__device__ __forceinline__ void warm_fused_c(const LaneIO& io) {
    const FusedW& f = io.fz;
    constexpr int NS = PT::nslot() > 0 ? PT::nslot() : 1;
    constexpr int NV = 2 * NS + 1;
    constexpr int NVA = PT::NMAX_V, NW = aset_words(PT::NMAX_N, PT::NMAX_M);
    const int sc = blockIdx.x * 64 + threadIdx.x;
    const bool live = sc < io.S;
    const int s = live ? sc : 0;            // (tail lanes load lane 0's values: valid addresses, unused)
    const int64_t S = io.S;
    double av[NVA], xv[NS], wv[NS], rv[NS], pcv[NS];
    uint32_t aw[NW];
    PHX_UNROLL for (int v = 0; v < PT::nvar(); ++v) av[v] = io.Av[(int64_t)v * S + s];
    PHX_UNROLL for (int k = 0; k < aset_words(PT::n(), PT::m()); ++k) aw[k] = io.aset[(int64_t)k * S + s];
    PHX_UNROLL for (int j = 0; j < PT::n(); ++j) {
        const int t = PT::col_slot(j);
        if (t >= 0) {
            const int64_t o = (int64_t)t * S + s;
            xv[t] = f.x_prev[(int64_t)j * S + s];
            wv[t] = io.W[o];
            rv[t] = io.rho[o];
            pcv[t] = f.pc[o];
        }
    }
    if (gated(io.gate)) return;
    if (!fz_prologue(io)) return;
    zero_next_counts(io.counts_next);
    // Update_W (phbase.py:293-318) and |x_{k-1} - x-bar_k| (convergence_diff)
    double xb[NS], dl = 0.0;
    PHX_UNROLL for (int t = 0; t < PT::nslot(); ++t) {
        xb[t] = f.stage[t];
        const double diff = xv[t] - xb[t];
        wv[t] = wv[t] + rv[t] * diff;
        if (live) PHX_OUT(const_cast<double*>(io.W)[(int64_t)t * S + sc], wv[t]);
        dl += fabs(diff);
    }
    bool still = false, rework = false;
    double xn[NS];                      // the certified lane's unscaled nonant x
    if (live) {
        ASet<PT> a;
        aset_from_words<PT>(aw, a);
        double xp[PT::NMAX_N], z[PT::NMAX_M];
        PHX_UNROLL for (int j = 0; j < PT::n(); ++j) xp[j] = 0.0;
        PHX_UNROLL for (int i = 0; i < PT::m(); ++i) z[i] = 0.0;
        const Data<PT> D0(io, sc, av, wv, rv, xb);
        const int c = io.warm_rounds > 0 ? as_round<PT>(io, D0, a, xp, z, 0) : 2;
        if (c == 0) {
            write_certified<PT>(io, D0, sc, a, xp, z, 0);
            PHX_UNROLL for (int j = 0; j < PT::n(); ++j)
                if (PT::col_slot(j) >= 0) xn[PT::col_slot(j)] = xp[j] * (PT::scaled() ? PT::dcs(j) : 1.0);
        } else if (c == 1 && io.warm_rounds > 1) {
            // round 1 onwards in the group's finisher: the state to go on from
            rework = true;
            PHX_UNROLL for (int j = 0; j < PT::n(); ++j) store_wt(&f.rx[(int64_t)j * S + sc], xp[j]);
            PHX_UNROLL for (int i = 0; i < PT::m(); ++i) store_wt(&f.rz[(int64_t)i * S + sc], z[i]);
            aset_store<PT>(io, sc, a);
        } else {
            if (c == 2) PHX_LANE_STAT(3);
            aset_store<PT>(io, sc, a);   // the updated active set seeds the next pass
            io.status[sc] = 0;
            io.flags[sc] = 0;
            still = true;
        }
    }
    double v[NV];
    PHX_UNROLL for (int e = 0; e < NV; ++e) v[e] = 0.0;
    if (live) {
        v[2 * NS] = dl;
        if (!still && !rework)
            PHX_UNROLL for (int t = 0; t < PT::nslot(); ++t) {
                const double w = pcv[t] * xn[t];
                v[t] += w;
                v[NS + t] += w * xn[t];
            }
    }
    compact_lane(still, sc, io.lanes_out, io.count_out);
    const unsigned long long rm = __ballot(rework);
    if (threadIdx.x == 0) store_wt_u64(&f.rmask[blockIdx.x], rm);
    fz_fold_c<PT>(io, v);
}

#endif

}  // namespace phx_lane
