/*
 * phx.h — C ABI of the MI355X-native scenario-batched PH engine (libphx.so).
 *
 * The reference (garg02/mpi-sppy) is pure Python; its PH hot path reaches
 * native code only through an external LP/QP solver behind Pyomo
 * (SPOpt.solve_one, mpisppy/spopt.py:85-223, solver call at :165-172) and
 * through mpi4py collectives.  This header is the drop-in boundary that
 * replaces those per-scenario calls and Python loops with batched HIP kernels
 * over all local scenarios at once.  Each entry point cites the reference
 * interface it replaces.
 *
 * Conventions
 *   - Every array argument is a DEVICE pointer (hipMalloc / torch.cuda memory)
 *     unless the name ends in _host.  Per-scenario arrays are scenario-minor:
 *     element i of local scenario s lives at [i*S + s].
 *   - fp64 everywhere; infinite bounds are IEEE +-inf.
 *   - Every function returns 0 on success, nonzero on failure; the message is
 *     available from phx_last_error(ctx).  No C++ exception crosses the ABI.
 *   - Ownership: the caller owns every array it passes; the context owns only
 *     its own scratch (solver state, scaled copies, polish workspace).
 *   - Threading: one host thread per context.  Work is ordered on the HIP
 *     stream passed in (hipStream_t as void*; NULL = default stream).  Only
 *     phx_set_problem and phx_solve synchronise with the host (documented).
 */
#ifndef PHX_H
#define PHX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct phx_ctx phx_ctx;

/* Per-scenario LP/QP standard form with a pattern shared by all scenarios:
 *      min  c'x + qN'x_N + 0.5 pN' x_N^2     (qN, pN: PH terms, phx_set_ph_terms)
 *      s.t. bl <= A x <= bu,  lb <= x <= ub
 * Replaces what the reference extracts from each Pyomo scenario model
 * (SPBase._create_scenarios, spbase.py:255-291) and the PH objective terms of
 * PHBase.attach_PH_to_objective (phbase.py:617-699).                         */
typedef struct phx_problem_desc {
    int32_t S;              /* local scenarios (lanes)                         */
    int32_t n, m, nnz;      /* columns, rows, nonzeros per scenario            */
    int32_t N;              /* nonant slots per scenario                       */
    int32_t nvar;           /* number of scenario-varying A entries            */
    const int32_t* rowptr;  /* [m+1]  CSR pattern                              */
    const int32_t* colidx;  /* [nnz]                                           */
    const int32_t* kvar;    /* [nnz]  -1: value Aconst[k] for all scenarios;
                                      v>=0: value Avar[v*S+s]                  */
    const double* Aconst;   /* [nnz]                                           */
    const double* Avar;     /* [nvar*S]                                        */
    const double* c;        /* [n] or [n*S] (c_vary)                           */
    const double* lb;       /* [n] or [n*S] (bnd_vary)                         */
    const double* ub;
    const double* bl;       /* [m] or [m*S] (rhs_vary)                         */
    const double* bu;
    int32_t c_vary, bnd_vary, rhs_vary;
    const int32_t* slot_col;/* [N]  column of each nonant slot, in the
                               reference's nonant order (spbase.py:293-302)   */
    /* Lane-solver tuning compiled into the structure-specialised kernels
     * (phx_jit.h); zero-initialised means off.  lane_multi_theta > 0: the
     * first lane_multi_rounds (0: 4) active-set rounds after the full
     * primal-dual updates change every violation within lane_multi_theta of
     * the worst one instead of the worst alone (phx_lane.h multi_violations;
     * the engine's solver option of the same name, SPOpt).                   */
    double  lane_multi_theta;
    int32_t lane_multi_rounds;
} phx_problem_desc;

/* Solver knobs; the engine fills them from options["iter0_solver_options"] /
 * ["iterk_solver_options"] (phbase.py:273-275).                              */
typedef struct phx_solve_opts {
    int32_t max_iters;        /* PDHG iterations before giving up (per solve) */
    int32_t check_every;      /* PDHG iterations per launch between checks    */
    int32_t restart_max;      /* artificial Halpern restart length            */
    int32_t polish;           /* 1: active-set KKT polish (exact optimum)     */
    int32_t refine_steps;     /* iterative-refinement steps in the polish     */
    int32_t warm_start;       /* 1: start from the previous solution          */
    double  polish_below;     /* attempt a polish once rel. KKT err < this    */
    double  opt_tol;          /* accept unpolished point when rel. KKT < this */
    double  kkt_tol;          /* polish certificate tolerance (relative)      */
    double  reg;              /* polish regularisation (scaled units)         */
    int32_t ipm_after;        /* PDHG iterations after which a lane still not
                                 certified switches to the interior-point
                                 finisher (0: IPM first; <0: never)           */
    int32_t ipm_max_it;       /* IPM iteration cap                            */
    double  ipm_tol;          /* IPM relative KKT target                      */
    int32_t lane_solver;      /* 1: run the register-resident, structure-
                                 specialised lane solver (IPM + polish) first
                                 when the context has one (small subproblems) */
    int32_t as_rounds;        /* active-set rounds of the warm pass and after
                                 the interior point; 0 disables the warm
                                 start (each solve starts with the interior
                                 point)                                       */
    int32_t warm_passes;      /* 1 (default): one warm pass over all lanes with
                                 as_rounds rounds in-kernel; k > 1: k passes of
                                 one round each, passes 2..k over the
                                 compacted lanes whose active set changed    */
    int32_t defer;            /* 1: with the lane solver, phx_solve returns
                                 right after enqueueing the lane kernels (no
                                 host synchronisation); phx_solve_finish then
                                 completes the solve (generic path for the
                                 lanes the lane solver could not certify)     */
    int32_t wg_warm;          /* k > 0: a warm generic-path solve (subproblems
                                 above the lane limits) first runs the
                                 workgroup-per-scenario active-set KKT pass,
                                 up to k rounds from the previous solution;
                                 PDHG + polish only for the lanes it does not
                                 certify.  0: off                             */
    int32_t sp;               /* 1: use the sparse workgroup solver (phx_sp.h:
                                 separator Schur complement, interior point +
                                 active-set rounds) when the context has one;
                                 0: skip it (generic PDHG path only)          */
    int32_t sp_rounds;        /* sparse solver: active-set rounds after its
                                 interior point (cold) and from the previous
                                 solution (warm)                              */
    int32_t seed_templates;   /* first solve of a context (Iter0) with the lane
                                 solver: template lanes (interior point, 1..64);
                                 every other lane starts active-set rounds from
                                 the nearest certified template's active set
                                 before its own interior point.  0: unseeded
                                 (the interior point on every lane, then the
                                 rescue round budget)                          */
    int32_t rescue_rounds;    /* lane solver: active-set rounds (single changes)
                                 of the rescue pass before any interior point,
                                 and of the first warm pass after a cold solve;
                                 0: max(16, 8 as_rounds)                      */
    double  lane_ipm_tol;     /* lane solver's interior point: relative KKT
                                 error at which it stops -- it only has to
                                 expose the active set (classification, then
                                 active-set rounds certify to kkt_tol);
                                 0: ipm_tol                                   */
    int32_t wg_first;         /* k > 0: the workgroup pass of the first warm
                                 solve after a cold one (the first PH iteration
                                 after Iter0) runs at most k rounds instead of
                                 wg_warm -- where that solve's active sets move
                                 too far for the pass and the sparse solver's
                                 interior point takes most lanes anyway; 0: wg_warm */
} phx_solve_opts;

/* Statistics of the most recent phx_solve (HIP events on the solve stream). */
typedef struct phx_solve_stats {
    double  pdhg_ms;          /* summed k_chunk (PDHG) kernel time            */
    double  polish_ms;        /* summed k_polish time                         */
    double  ipm_ms;           /* generic interior-point finisher              */
    double  lane_ms;          /* specialised lane kernel: IPM + active set    */
    double  lane_warm_ms;     /* specialised lane kernel: warm active set,
                                 first pass (all lanes)                       */
    double  lane_warm_list_ms;/* further warm passes over compacted lanes     */
    double  lane_iters;       /* PDHG scenario-iterations executed            */
    int32_t pdhg_launches;
    int32_t total_iters;      /* PDHG iterations of the batch loop            */
    int32_t lane_certified;   /* scenarios certified by the lane solver       */
    int32_t lane_warm_certified; /* ... of which by the warm active-set pass  */
    int32_t not_optimal;      /* scenarios without an optimal status          */
    int32_t stragglers;       /* lanes the lane solver handed to the generic
                                 path (their x was final only after it)       */
    int32_t jit;              /* 1 if this context has a specialised kernel   */
    int32_t lane_first_certified; /* certified by the first lane pass (the
                                 affine-map pass when maps are on)            */
    int32_t wg_certified;     /* certified by the workgroup warm pass         */
    double  wg_ms;            /* workgroup warm pass kernel time              */
    int32_t sp_certified;     /* certified by the sparse workgroup solver     */
    int32_t sp_warm_rounds;   /* its active-set rounds from warm starts (sum) */
    int32_t sp_ipm_its;       /* its interior-point iterations (sum)          */
    int32_t sp_cold_rounds;   /* its active-set rounds after the IPM (sum)    */
    int32_t sp_refine;        /* its refinement solves (sum)                  */
    double  sp_ms;            /* sparse solver kernel time                    */
    int32_t infeasible;       /* scenarios proven infeasible (Farkas
                                 certificate; status 4): the reference's
                                 scenario_feasible = False, spopt.py:175-194   */
} phx_solve_stats;

/* Scenario-tree reduction layout for Compute_Xbar (phbase.py:27-107): for each
 * tile, the nonant slots [slot_lo, slot_lo+nlen) of one tree node summed over
 * the contiguous local scenarios [s_begin, s_end).  Tiles of one node are
 * consecutive; node_tile_ptr[v]..node_tile_ptr[v+1] lists them, and their
 * partial offsets are consecutive too: tile_out[t] = tile_out[t0] +
 * (t - t0) * 2 * nlen for the tiles t0.. of one node.  Tiles of at most 256
 * scenarios (one per thread of a 256-thread block).                         */
typedef struct phx_tree_desc {
    int32_t ntiles;
    const int32_t* tile_s0;    /* [ntiles] */
    const int32_t* tile_s1;    /* [ntiles] */
    const int32_t* tile_slot;  /* [ntiles] first slot                        */
    const int32_t* tile_nlen;  /* [ntiles] slots of the node                  */
    const int32_t* tile_out;   /* [ntiles] offset into the partial buffer     */
    int32_t nnodes;            /* nodes with at least one local scenario      */
    const int32_t* node_tile_ptr; /* [nnodes+1]                               */
    const int32_t* node_off;   /* [nnodes] offset of the node's slots in the
                                  global node-slot vector (length NNS)        */
    const int32_t* node_nlen;  /* [nnodes]                                    */
    int32_t NNS;               /* global number of (node, slot) entries       */
    int32_t npart;             /* size of the partial buffer (doubles)        */
    int32_t nnodes_cover;      /* sum of node_nlen over the local nodes (== NNS
                                  when every node has a local scenario)       */
    const int32_t* node_key;   /* [N][S] optional (may be NULL): the node-slot
                                  index of each (nonant slot, local scenario),
                                  the x-bar index of phx_update_w.  With it,
                                  small batches (S <= 1024) take phx_xbar /
                                  phx_update_w / phx_iterk's one-block path   */
} phx_tree_desc;

/* ---- lifetime ---------------------------------------------------------- */
int         phx_create(int32_t device, phx_ctx** out);
int         phx_destroy(phx_ctx* ctx);
const char* phx_last_error(const phx_ctx* ctx);
/* Number of compiled gfx targets / a build string, for diagnostics.        */
const char* phx_build_info(void);

/* Replaces the per-scenario model build + SolverFactory/set_instance
 * (SPOpt._create_solvers, spopt.py:839-903).  Copies/derives: CSC view,
 * Ruiz + Pock-Chambolle scaling, per-scenario ||A||_2 (power iteration),
 * polish workspace.  Synchronises the device (setup only).                 */
int phx_set_problem(phx_ctx* ctx, const phx_problem_desc* desc);

/* Per-scenario column bounds ([n][S], unscaled, device) replacing the
 * problem's own for the following solves — how the engine fixes nonants
 * (lb = ub = value: SPOpt._fix_nonants / _restore_nonants, spopt.py:557-662;
 * Xhat_Eval, utils/xhat_eval.py:293-322).  lb = ub = NULL restores the
 * problem's bounds.  While overridden, solves use the generic path (the lane
 * kernels are specialised on the original bound structure).  Enqueued on
 * `stream`; the arrays may be released after the call's work has run.      */
int phx_set_bounds(phx_ctx* ctx, const double* lb, const double* ub, void* stream);

/* PH objective terms for the next solve (attach_PH_to_objective,
 * phbase.py:617-699; W_on/prox_on toggles :409-440):
 *   qN[j][s] = W_on*W[j][s] - prox_on*rho[j][s]*xbar(s,j)
 *   pN[j][s] = prox_on*rho[j][s]
 *   kN[s]    = prox_on*sum_j rho/2*xbar^2
 * with xbar(s,j) = xbar_node[xbar_idx[j*S+s]].  W/rho/xbar may be NULL when
 * W_on = prox_on = 0 (Iter0).                                              */
int phx_set_ph_terms(phx_ctx* ctx, const double* W, const double* rho,
                     const double* xbar_node, const int32_t* xbar_idx,
                     int32_t W_on, int32_t prox_on, void* stream);

/* Batched subproblem solve — replaces PHBase.solve_loop -> SPOpt.solve_loop ->
 * solve_one (phbase.py:494-568, spopt.py:226-307, :85-223).  Restarted
 * reflected-Halpern PDHG on the scaled problem, warm-started, followed by an
 * active-set KKT polish that certifies each scenario's optimum.
 * Outputs (all [.][S]): x_out[n], y_out[m] (row duals), obj_out[S] (objective
 * incl. PH terms, = outer bound), status_out[S] (1 optimal, 2 iteration limit,
 * 3 numerical failure, 4 infeasible: a Farkas certificate from the interior
 * point), iters_out[S].  *total_iters_host = iterations run.
 * Synchronises with the host once per check_every iterations.              */
int phx_solve(phx_ctx* ctx, const phx_solve_opts* opts,
              double* x_out, double* y_out, double* obj_out,
              int32_t* status_out, int32_t* iters_out,
              int32_t* total_iters_host, void* stream);

/* Completes a solve started with opts.defer = 1: waits for the lane kernels
 * (host synchronisation), runs the generic path on the lanes they left, and
 * reports how many there were (*stragglers_host; 0 = every lane's outputs
 * were already final when phx_solve returned).  No-op if nothing is pending.
 * Outputs land in the arrays given to phx_solve.  Replaces the tail of
 * SPOpt.solve_loop (spopt.py:284-307: statuses, feasibility, timing).       */
int phx_solve_finish(phx_ctx* ctx, int32_t* stragglers_host, int32_t* total_iters_host);

/* Objective of the caller's point x ([n][S], unscaled) under the PH terms last
 * set by phx_set_ph_terms: obj[s] = c'x + qN'x_N + 0.5 pN x_N^2 + kN — what
 * the reference evaluates as pyo.value(objective) in Eobjective
 * (spopt.py:327-343).                                                      */
int phx_objective(phx_ctx* ctx, const double* x, double* obj_out, void* stream);

/* Compute_Xbar local part (phbase.py:54-80): node_sums[e] = sum over local
 * scenarios of prob_coeff*x, node_sums[NNS+e] = sum prob_coeff*x^2 for every
 * (node, slot) entry e (zeros for nodes absent locally).  The caller then
 * all-reduces node_sums over ranks (phbase.py:83-87) — one RCCL call.      */
int phx_xbar(phx_ctx* ctx, const phx_tree_desc* tree, const double* x,
             const double* prob_coeff, double* partial, double* node_sums,
             void* stream);

/* Update_W + convergence_diff local part (phbase.py:293-343):
 *   W[j][s] = W_in[j][s] + rho[j][s]*(x_N - xbar)   (if update_w; W_in may
 *             equal W — in place — or be the other buffer of a pair)
 *   dsum[s]  = sum_j |x_N - xbar|            (dsum may be NULL when the
 *                                             segments cover every scenario)
 * then seg_sums[r] = sum of dsum over local scenarios [seg_s0[r], seg_s1[r])
 * (one segment per emulated reference rank, sputils.py:803-810).  When the
 * segments partition the local scenarios, W, dsum and the segment partials
 * come out of one fused pass (k_update_w_seg).                              */
int phx_update_w(phx_ctx* ctx, const double* x, const double* xbar_node,
                 const int32_t* xbar_idx, const double* rho, const double* W_in, double* W,
                 int32_t update_w, double* dsum, int32_t nseg,
                 const int32_t* seg_s0_host, const int32_t* seg_s1_host,
                 double* seg_sums, void* stream);

/* Expectations (Eobjective/Ebound/_update_E1/feas_prob, spopt.py:310-439):
 * out[0] = sum_s p_s*obj_s, out[1] = sum_s p_s, out[2] = sum_s p_s*[status==1]
 * over local scenarios (deterministic tree order).  out is a device [3].    */
int phx_expect(phx_ctx* ctx, const double* prob, const double* obj,
               const int32_t* status, double* out, void* stream);

/* Scenario-major export of a [N][S] slot array (W or nonant x) into
 * out[S*N + 0..] — the flat layout of PHBase._populate_W_cache /
 * PHHub.send_nonants (phbase.py:346-366, hub.py:562-577).                  */
int phx_export_slots(phx_ctx* ctx, const double* src, double* out, void* stream);

int phx_last_solve_stats(const phx_ctx* ctx, phx_solve_stats* out_host);

/* In-place SUM all-reduce of `count` doubles at device `buf` over the ranks,
 * ordered on `stream` (the caller's collective: RCCL through torch.distributed
 * on the GPU).  Returns 0 on success.                                        */
typedef int (*phx_allreduce_fn)(void* user, double* buf, int64_t count, void* stream);

/* The PH main loop after Iter0 (PHBase.iterk_loop, phbase.py:875-979) for
 * runs without per-iteration host hooks (no extensions, converger or hub):
 * per iteration k = 1..max_iters
 *     Compute_Xbar -> [allreduce] -> Update_W -> convergence_diff -> stop if
 *     conv < convthresh (before the solve, phbase.py:914-926) -> solve
 * with the stop test evaluated ON THE DEVICE: the host keeps `depth`
 * iterations enqueued ahead, a device flag turns the kernels of iterations
 * past the stop into no-ops, and the host only polls a mapped progress word
 * (no per-iteration host round trip).  A solve that leaves lanes to the
 * generic path stops the pipeline at the next Update_W (all ranks alike: the
 * count travels in the all-reduced node sums); the host finishes those lanes
 * and resumes, so every iteration sees final x exactly as the Python loop.
 * Requires the lane solver (phx_jit_info "on"), no phx_set_bounds override,
 * a previous solve that is finished or a pending deferred lane-solver solve
 * (adopted, see phx_iterk_result.adopted), and segments that partition the local
 * scenarios.  W is updated in place.  The PH terms are those of the last
 * phx_set_ph_terms (W, rho, xbar_node must be the arrays given here).       */
typedef struct phx_iterk_args {
    double* x; double* y; double* obj; int32_t* status; int32_t* iters;   /* solve outputs */
    const phx_tree_desc* tree; const double* prob_coeff; double* partial;
    double* node_sums;               /* [2*NNS] xbar | xsqbar, published once an iteration proceeds */
    double* node_stage;              /* [2*NNS+1] this iteration's sums (+ straggler count); the
                                        buffer the all-reduce callback receives              */
    const int32_t* xbar_idx; const double* rho; double* W;
    int32_t nseg; const int32_t* seg_s0_host; const int32_t* seg_s1_host; double* seg_sums;
    const double* conv_counts_host;  /* [nseg] element count of each emulated rank (all ranks) */
    int32_t conv_R;                  /* emulated rank count (phbase.py:330-343) */
    double convthresh;
    int32_t max_iters;               /* iterations to run at most                */
    int32_t depth;                   /* iterations kept enqueued ahead (>= 1)    */
    int32_t timing;                  /* T > 0: HIP events around the phx_lane_warm launch of
                                        every T-th iteration (each record costs ~6 us of GPU
                                        time, so the sample is sparse); 0: none; T < 0: one
                                        event pair around ALL the fused launches of a run that
                                        reaches max_iters without a stop (back to back, so
                                        the window is their summed durations; unfused modes:
                                        every |T|-th iteration as T > 0)                   */
    phx_allreduce_fn allreduce;      /* NULL on one rank                         */
    void* allreduce_user;
    int32_t node_stage_len;          /* doubles in node_stage; >= 2*NNS+1+conv_R enables the
                                        fused mode (one launch per PH iteration, two-stage
                                        trees): the all-reduce then carries the conv sums too */
    double* iter0_obj;               /* [S] or NULL: when phx_iterk adopts a pending deferred
                                        solve (Iter0's), its final objectives and statuses are
                                        copied here for the caller's Iter0 expectations (E1,
                                        feas_prob, trivial bound: phbase.py:805-856)         */
    int32_t* iter0_status;           /* [S] or NULL                                          */
    const double* iter0_prob;        /* [S] or NULL: with iter0_expect, phx_iterk also enqueues
                                        phx_expect of the adopted solve (sum p obj, sum p,
                                        sum p [optimal]) into iter0_expect [3] (device) and
                                        copies it to iter0_expect_host [3] (pinned host memory,
                                        final when phx_iterk returns): Iter0's checks without
                                        a kernel launch or a device read after the loop     */
    double* iter0_expect;
    double* iter0_expect_host;
} phx_iterk_args;

typedef struct phx_iterk_result {
    int32_t iters;         /* the reference's _PHIter at loop exit              */
    int32_t converged;     /* 1: conv < convthresh at iteration `iters` (no solve then) */
    double conv;           /* convergence_diff of iteration `iters`             */
    int32_t solves;        /* solves completed                                  */
    int32_t straggler_stops; /* pipeline stops to finish generic-path lanes      */
    int32_t stragglers;    /* lanes finished on the generic path, total         */
    int32_t not_optimal;   /* lanes left uncertified by the last solve          */
    double warm_ms;        /* sum of phx_lane_warm durations (timing = 1)       */
    int32_t warm_launches;
    double wall_ms;
    int32_t fused;         /* 1: the fused one-launch-per-iteration mode ran     */
    int32_t adopted;       /* 1: a pending deferred lane-solver solve (Iter0's) was
                              adopted as the solve before iteration 1 -- enqueued
                              behind without a host round trip; phx_last_solve_stats
                              then reports that solve                           */
    int32_t adopted_stragglers; /* its lanes finished on the generic path      */
} phx_iterk_result;

int phx_iterk(phx_ctx* ctx, const phx_solve_opts* opts, const phx_iterk_args* args,
              phx_iterk_result* result_host, void* stream);

/* The context's own collective for phx_iterk: an RCCL communicator over the
 * ranks of the PH cylinder (one process per GPU), so the per-iteration
 * all-reduce of the fused node buffer is enqueued by phx_iterk itself
 * (ncclAllReduce, SUM, fp64, on the loop's stream) instead of a host callback.
 * Replaces the per-tree-node comms[ndn].Allreduce of _Compute_Xbar
 * (phbase.py:83-87) and the ROOT Allreduce of convergence_diff
 * (phbase.py:341) inside the loop, and the Split communicators they run on
 * (spbase.py:333-375).  phx_comm_unique_id: one rank draws the id (128 bytes,
 * host) and the caller broadcasts it; phx_set_comm: collective over the
 * nranks ranks (ncclCommInitRank).  phx_iterk uses the communicator when
 * args.allreduce is NULL.                                                    */
int phx_comm_unique_id(void* id_host);
int phx_set_comm(phx_ctx* ctx, const void* id_host, int32_t nranks, int32_t rank);

/* Everything phx_iterk allocates or uploads for these arguments (segment
 * tiles, control words, the mapped progress word, the fused mode's second
 * output set, timing events), done ahead of the loop; no work is enqueued.
 * Optional: phx_iterk does it itself on first use.  Replaces nothing in the
 * reference (its loop has no device state); called where the reference
 * builds its solver objects (SPOpt._create_solvers, spopt.py:839-903).      */
int phx_iterk_prepare(phx_ctx* ctx, const phx_iterk_args* args);

/* Human-readable state of the structure-specialised lane solver for this
 * context ("on: ..." or "off: <reason>").                                   */
const char* phx_jit_info(const phx_ctx* ctx);

/* Test hook (no reference counterpart): the workgroup solver's Schur
 * complement inverse (phx_wg.h wg_blk_cholesky -> wg_blk_trtri ->
 * wg_blk_lauum, one 256-thread workgroup, the matrix in LDS) on one
 * symmetric matrix s_host [ma x ma] (lower triangle read), ma <= 64.
 * inv_host [ma x ma] receives the inverse; returns 1 if a pivot was not
 * positive, 0 on success, -1 on a HIP error.                               */
int phx_debug_spd_inverse(const double* s_host, int32_t ma, double* inv_host);

#ifdef __cplusplus
}
#endif
#endif /* PHX_H */
