// phx_wg.h — workgroup-per-scenario warm active-set KKT solve for medium
// subproblems (farmer crops_multiplier=10, sslp relaxations: n in the
// hundreds, m <= ~100), the generic-path counterpart of phx_lane_warm.
//
// Reference semantics being replaced: SPOpt.solve_one (mpisppy/spopt.py:85-223)
// of PH iterations >= 1 (phbase.py:875-979): the external solver warm-starts
// from its previous basis.  Here one 64-lane wavefront owns one scenario: its
// A values, costs, iterate and the dense Schur complement of the active rows
// live in LDS, and every phase is a wavefront-strided loop over columns, rows
// or Schur entries separated by a workgroup barrier (a single wave: the
// barrier only orders LDS).  Starting from the previous solve's point
// (St.xT/yT, scaled) it runs up to `rounds` rounds of
//   classify -> Schur A_RF (P_FF+reg)^-1 A_RF' + reg I -> Cholesky ->
//   iterative refinement on the unregularised KKT -> certificate ->
//   primal-dual active-set update,
// with exactly the classification, refinement and certificate of polish_lane
// (phx_core.h), so a certified lane is as exact as a polished PDHG lane.
// Lanes that do not certify go to the PDHG + polish path unchanged.
//
// Round 3: FOUR wavefronts (256 threads) per scenario.  With one wavefront
// the solve was a chain of LDS latencies on one SIMD (farmer cm=10 x 1,000:
// ~1 wavefront per SIMD, nothing to hide them; ~300 k cycles per round, the
// Cholesky's one-row-per-lane update the largest part).  Now four threads
// share each row of the Cholesky's trailing update, of the explicit inverse's
// column recurrences and of the L^-1 mat-vecs (interleaved columns, combined
// with two lane shuffles inside the quad), and the reductions go through LDS
// across the four wavefronts.
//
// The same code is compiled for the host by tests/emu with WG_NT = 1 (every
// strided loop runs serially, barriers vanish): each phase writes only
// elements it owns, and cross-thread values are exchanged only through LDS
// across a barrier, so the serial run computes the same numbers.
#pragma once
#include "phx_core.h"

namespace phx {

#if defined(__HIP_DEVICE_COMPILE__)
#define WG_TID ((int)threadIdx.x)
#define WG_NT 256
#define WG_SYNC() __syncthreads()
#else
#define WG_TID 0
#define WG_NT 1
#define WG_SYNC() ((void)0)
#endif
// quads: four adjacent threads share one row (or column) of a dense phase
#define WG_QN (WG_NT >= 4 ? WG_NT / 4 : 1)            // quads per workgroup
#define WG_QID (WG_NT >= 4 ? WG_TID >> 2 : 0)         // this thread's quad
#define WG_QL (WG_NT >= 4 ? (WG_TID & 3) : 0)         // its place in the quad
#define WG_QW (WG_NT >= 4 ? 4 : 1)                    // threads per quad
#ifndef WG_SINGLE_AFTER
#define WG_SINGLE_AFTER 99   // rounds of full primal-dual changes before single ones (PHX_WG_SINGLE_AFTER; 2 measured: sslp -2 %, farmer cm=10 +27 %, r04 s19)
#endif

// Schur-complement entries (ia >= ib) whose rows share a column, with the CSR
// positions (ka in row ia, kb in row ib) of every shared column, built once on
// the host from the pattern (phx_set_problem).
struct WgPairs {
    int32_t npair;        // (the first nlong share many columns: a quad each in wg_warm)
    const int32_t* ptr;   // [npair+1] into ka/kb
    const int32_t* ia;    // [npair]
    const int32_t* ib;    // [npair]
    const int32_t* ka;    // [ntrip]
    const int32_t* kb;    // [ntrip]
    // Per-scenario factor cache (null fac: off).  The Schur complement and its
    // inverse factor depend on A (fixed), the active set (column and row codes)
    // and the prox weights pN + the regularisation; they change little from one
    // PH iteration to the next, so the factor of the last set a scenario solved
    // with is kept (its explicit L^-1, lower triangle) under that key and reused
    // when a round's active set and weights match it bit for bit.
    double* fac;          // [S][fac_stride]: L^-1 (ma x ld, rows) then dg (ma)
    int64_t fac_stride;
    int8_t* key;          // [S][key_stride]: column codes (n) then row codes (m)
    int64_t key_stride;
    double* pkey;         // [S][N+1]: pN of the nonant slots, then reg
    int32_t* ok;          // [S]: the cached factor is valid
    int32_t N;
    char* split;          // [S][split_stride] wg_carve's split arrays, or null (all in LDS)
    int64_t split_stride;
    // the split layout's scenario-invariant parts, shared by every workgroup
    // instead of copied into each scenario's area (null: copied): the CSC row
    // indices / CSR positions as 16-bit, and A's values when no entry varies
    const int16_t* pat_ri = nullptr;
    const int16_t* pat_c2 = nullptr;
    const double* a_const = nullptr;
    int32_t single_after = WG_SINGLE_AFTER;   // rounds of full primal-dual changes before single ones
    int32_t nlong = 0;    // pairs [0, nlong) are the long ones (phx_setup.h build_wg_pairs)
    int32_t prof_off = 0; // byte offset of the profiler's 16 LDS slots (after the carve; PHX_WG_PROF)
};

// Carve of the dynamic LDS of one scenario.
struct WgLds {
    double *Sm, *dg, *a, *xp, *r1, *qq, *pp, *z, *t, *u;
    double* red;                       // [8] cross-wavefront reductions (wg_max / wg_sum)
    // 16-bit indices (wg_lds_bytes: nnz, n, m < 32768) keep farmer cm=10's
    // carve under 40 KiB, i.e. four scenarios per CU
    int16_t *cp, *ri, *c2, *rp, *ci;   // pattern: CSC colptr/rowidx/csc2csr, CSR rowptr/colidx
    int16_t *ar, *pos;                 // active rows (compact order) and each row's position (-1: inactive)
    int32_t* flag;
    int8_t *cc, *rc;   // column code 0 free / 1 at l / 2 at u; row code 0 inactive / 1 at bl / 2 at bu
    bool own_a, own_pat;   // a / (ri, c2) are this scenario's copies (else the shared arrays)
};

// Split layout (split = true): the scenario's A values, the column vectors
// (xp, r1, qq, pp) and the CSC row / position indices (ri, c2) live in a
// per-scenario global scratch area (wg_split_bytes) instead of LDS, so that
// more workgroups fit a CU (sslp_15_45: 75 KB of LDS, two per CU, against
// 37 KB, four).  Round 5: the indices (always) and A's values (when none
// varies: sslp) are read from arrays shared by every workgroup (WgPairs
// pat_ri / pat_c2 / a_const, L2-resident) instead -- the per-scenario area
// holds the four column vectors only (sslp: 39 -> 23 KB written and re-read
// per scenario).
PHX_HD size_t wg_split_bytes(int n, int nnz, bool own_a = true, bool own_pat = true) {
    return (8 * ((own_a ? (size_t)nnz : 0) + 4 * (size_t)n) + (own_pat ? 4 * (size_t)nnz : 0) + 15) & ~(size_t)15;
}

PHX_HD size_t wg_lds_bytes(int n, int m, int nnz, bool split = false) {
    if (n >= 32767 || m >= 32767 || nnz >= 32767) return ~(size_t)0;   // 16-bit indices
    const size_t moved_d = split ? 0 : (size_t)nnz + 4 * (size_t)n;
    const size_t idx16 = (size_t)n + 1 + (split ? 1 : 3) * (size_t)nnz + (size_t)m + 1 + 2 * (size_t)m;
    size_t b = 8 * ((size_t)m * (m + 1) + 4 * (size_t)m + moved_d) + 16 + 64 + 2 * idx16 + (size_t)n + (size_t)m;
    return (b + 15) & ~(size_t)15;
}

// gbase: the split arrays' place (null: everything in LDS); with it, the
// shared index arrays (ri_sh, c2_sh) and A values (a_sh) when given
PHX_HD WgLds wg_carve(void* base, int n, int m, int nnz, void* gbase = nullptr, const int16_t* ri_sh = nullptr,
                      const int16_t* c2_sh = nullptr, const double* a_sh = nullptr) {
    WgLds L;
    L.own_a = !(gbase && a_sh);
    L.own_pat = !(gbase && ri_sh && c2_sh);
    double* d = (double*)base;
    L.Sm = d; d += (size_t)m * (m + 1);   // rows padded to an odd stride (wg_warm)
    L.dg = d; d += m;
    L.z = d; d += m;
    L.t = d; d += m;
    L.u = d; d += m;
    double* g = gbase ? (double*)gbase : d;
    if (L.own_a) { L.a = g; g += nnz; }
    else L.a = (double*)a_sh;          // (never written: own_a)
    L.xp = g; g += n;
    L.r1 = g; g += n;
    L.qq = g; g += n;
    L.pp = g; g += n;
    if (!gbase) d = g;
    L.red = d; d += 8;
    L.flag = (int32_t*)d;
    int16_t* w = (int16_t*)(L.flag + 4);
    int16_t* gw = gbase ? (int16_t*)g : nullptr;
    L.cp = w; w += n + 1;
    if (!L.own_pat) { L.ri = (int16_t*)ri_sh; L.c2 = (int16_t*)c2_sh; }   // (never written)
    else if (gw) { L.ri = gw; gw += nnz; L.c2 = gw; gw += nnz; }
    else { L.ri = w; w += nnz; L.c2 = w; w += nnz; }
    L.rp = w; w += m + 1;
    L.ci = w; w += nnz;
    L.ar = w; w += m;
    L.pos = w; w += m;
    int8_t* c = (int8_t*)w;
    L.cc = c; c += n;
    L.rc = c;
    return L;
}

// max over the workgroup: butterfly inside each wavefront, then the four
// wavefront results through LDS (two barriers: red may be reused right after)
PHX_HD double wg_max(double v, double* red) {
#if defined(__HIP_DEVICE_COMPILE__)
    v = wave_reduce<1>(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    v = red[0];
    for (int w = 1; w < WG_NT / 64; ++w) v = fmax(v, red[w]);
#else
    (void)red;
#endif
    return v;
}

// max of two values over the workgroup in one LDS round (two barriers)
PHX_HD void wg_max2(double& a, double& b, double* red) {
#if defined(__HIP_DEVICE_COMPILE__)
    a = wave_reduce<1>(a);
    b = wave_reduce<1>(b);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        red[threadIdx.x >> 6] = a;
        red[4 + (threadIdx.x >> 6)] = b;
    }
    __syncthreads();
    a = red[0];
    b = red[4];
    for (int w = 1; w < WG_NT / 64; ++w) {
        a = fmax(a, red[w]);
        b = fmax(b, red[4 + w]);
    }
#else
    (void)a; (void)b; (void)red;
#endif
}

// (key, element) of the largest key over the workgroup, the smallest element
// on equal keys (keys >= 0; element -1: none); every thread ends with it
PHX_HD void wg_argmax(double& key, int& el, double* red) {
#if defined(__HIP_DEVICE_COMPILE__)
    for (int o = 32; o > 0; o >>= 1) {
        const double k2 = __shfl_xor(key, o, 64);
        const int e2 = __shfl_xor(el, o, 64);
        if (k2 > key || (k2 == key && e2 >= 0 && (el < 0 || e2 < el))) { key = k2; el = e2; }
    }
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        red[threadIdx.x >> 6] = key;
        red[4 + (threadIdx.x >> 6)] = (double)el;
    }
    __syncthreads();
    key = red[0];
    el = (int)red[4];
    for (int w = 1; w < WG_NT / 64; ++w) {
        const double k2 = red[w];
        const int e2 = (int)red[4 + w];
        if (k2 > key || (k2 == key && e2 >= 0 && (el < 0 || e2 < el))) { key = k2; el = e2; }
    }
#else
    (void)key; (void)el; (void)red;
#endif
}

// sum of a value over a quad (its four threads end with the same sum)
PHX_HD double wg_quad_sum(double v) {
#if defined(__HIP_DEVICE_COMPILE__)
    v = quad_reduce<0>(v);
#endif
    return v;
}

// Optional phase timing (PHX_WG_PROF=1 on the host side): per phase, the
// shader-clock cycles of the workgroup's thread 0, accumulated in 16 LDS slots
// (prof: k_wg_warm's, after the carve) and added to the global sums once at the
// kernel's end -- a global atomic per phase stalled the next barrier behind
// 1,000 workgroups' atomics on the same 16 words and moved time between phases.
#if defined(__HIP_DEVICE_COMPILE__)
#define WG_T0() long long _wg_t = prof ? clock64() : 0
#define WG_TP(ph)                                                             \
    do {                                                                      \
        if (prof && threadIdx.x == 0) {                                       \
            const long long _n = clock64();                                   \
            prof[ph] += (unsigned long long)(_n - _wg_t);                     \
            _wg_t = _n;                                                       \
        }                                                                     \
    } while (0)
#define WG_CNT(ph) do { if (prof && threadIdx.x == 0) prof[ph] += 1ull; } while (0)
#else
#define WG_T0() (void)prof
#define WG_TP(ph) ((void)0)
#define WG_CNT(ph) ((void)0)
#endif

// Order-preserving list of the active rows (ar) and each row's position in it
// (pos, -1 when inactive), built by the first wavefront; their count goes to
// L.flag[3] (read by every thread after the caller's barrier).
PHX_HD void wg_compact(const WgLds& L, int m) {
    int cnt = 0;
#if defined(__HIP_DEVICE_COMPILE__)
    const int lane = (int)threadIdx.x;
    if (lane >= 64) return;
    for (int base = 0; base < m; base += 64) {
        const int i = base + lane;
        const bool act = i < m && L.rc[i] != 0;
        const unsigned long long b = __ballot(act);
        if (act) {
            const int p = cnt + __popcll(b & ((1ull << lane) - 1ull));
            L.ar[p] = (int16_t)i;
            L.pos[i] = (int16_t)p;
        } else if (i < m) {
            L.pos[i] = -1;
        }
        cnt += __popcll(b);
    }
    if (lane == 0) L.flag[3] = cnt;
#else
    for (int i = 0; i < m; ++i) {
        if (L.rc[i]) { L.ar[cnt] = (int16_t)i; L.pos[i] = (int16_t)cnt++; }
        else L.pos[i] = -1;
    }
    L.flag[3] = cnt;
#endif
}

// ---- The Schur complement's inverse with f64 MFMA tiles (round 4) ----
// Blocked versions of the three steps, in 16 x 16 blocks (rows and columns
// past ma read as zero, never stored), for a Schur complement of at most
// WG_BLK_MAX rows:
//   wg_blk_cholesky: right-looking Cholesky; per panel the diagonal block is
//     factored by wavefront 0 in registers, the rows below by forward
//     substitution (a thread per row), and the trailing update
//     W_IJ -= L_IP L_JP^T is MFMA.  Output as the scalar factor's: L[i][k]
//     (i > k) at Sm[k*ld + i] (the upper part), 1 / L[k][k] in dg; the lower
//     part is the working matrix.
//   wg_blk_trtri: X = L^-1 into the lower part (diagonal included): diagonal
//     blocks by a thread per column, then block row by block row
//     X_IJ = -X_II sum_K L_IK X_KJ (MFMA).
//   wg_blk_lauum: M^-1 = X^T X, the full symmetric matrix (MFMA), so that a
//     refinement step is ONE dense mat-vec.
// v_mfma_f64_16x16x4_f64 (MI355X_MICROARCH / cdna_hip_programming: lane l holds
// A[l&15][k = 4s + (l>>4)] and B[k][l&15] of k-step s; C/D rows (l>>4) + 4r,
// column l&15 of register r -- so a C tile's register s is the B operand of
// k-step s of a following product).  The numbers are the scalar algorithms'
// in another summation order (stable as they are: an in-place Gauss-Jordan
// inverse was tried first and lost 20 digits on the degenerate faces'
// nearly singular complements).
#define WG_TB 16
#define WG_BLK_MAX 64    // 4 x 4 blocks: wg_blk_lauum keeps a wavefront's tiles in registers
#if defined(__HIP_DEVICE_COMPILE__)
typedef double wg_d4 __attribute__((ext_vector_type(4)));

// Sm[r*ld + c] when r, c < ma (and, with `lower`, r >= c), else 0; a clamped
// address (no read outside the matrix)
__device__ __forceinline__ double wg_el(const double* Sm, int ld, int ma, int r, int c, bool lower = false) {
    const bool in = r < ma && c < ma && (!lower || r >= c);
    const double v = Sm[(in ? r : 0) * ld + (in ? c : 0)];
    return in ? v : 0.0;
}

__device__ __forceinline__ double wg_readlane64(double v, int lane) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u & 0xffffffffull), lane);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), lane);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

#define WG_MFMA(a, b, c) __builtin_amdgcn_mfma_f64_16x16x4f64((a), (b), (c), 0, 0, 0)

// Panel p0's diagonal block (wavefront 0; lane (r, g) = (l&15, l>>4) holds row
// r, columns 4g..4g+3): Cholesky in registers (row / column broadcasts by lane
// permutes), stored as L^T in the upper part and 1/L_jj in dg.  false
// (uniform): a pivot is not positive.
__device__ bool wg_blk_diag(double* Sm, int ld, int ma, int p0, double* dg) {
    const int l = (int)(threadIdx.x & 63), r = l & 15, g = l >> 4;
    const int w = ma - p0 < WG_TB ? ma - p0 : WG_TB;
    double a[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int c = 4 * g + q;
        const bool in = r < w && c < w && c <= r;
        const double v = Sm[(p0 + (in ? r : 0)) * ld + p0 + (in ? c : 0)];
        a[q] = in ? v : (r == c ? 1.0 : 0.0);
    }
    bool ok = true;
#pragma unroll 1
    for (int j = 0; j < WG_TB; ++j) {
        // column j's slot, before this step changes it (a select over the four
        // slots: j is uniform; the loop stays rolled, for the register budget)
        const int js = j & 3;
        const double colj = js == 0 ? a[0] : (js == 1 ? a[1] : (js == 2 ? a[2] : a[3]));
        const double d = wg_readlane64(colj, j + 16 * (j >> 2));    // a_jj
        ok = ok && d > 0.0;
        const double isd = 1.0 / sqrt(d);
        const double lrj = __shfl(colj, r + 16 * (j >> 2), 64) * isd;   // L_rj (r >= j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int c = 4 * g + q;
            const double lcj = __shfl(colj, c + 16 * (j >> 2), 64) * isd;   // L_cj (c >= j)
            if (c == j) a[q] = lrj;
            else if (c > j && c <= r) a[q] = fma(-lrj, lcj, a[q]);
        }
    }
    // L[r][c] (r > c) at Sm[(p0+c)*ld + p0+r]; 1/L_rr in dg
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int c = 4 * g + q;
        if (r < w && c < w) {
            if (c < r) Sm[(p0 + c) * ld + p0 + r] = a[q];
            else if (c == r) dg[p0 + r] = 1.0 / a[q];
        }
    }
    return ok;
}

PHX_HD bool wg_blk_cholesky(double* Sm, int ld, int ma, double* dg, int32_t* flag) {
    const int nb = (ma + WG_TB - 1) / WG_TB;
    const int l = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6), r16 = l & 15, g = l >> 4;
    for (int P = 0; P < nb; ++P) {
        const int p0 = WG_TB * P, w = ma - p0 < WG_TB ? ma - p0 : WG_TB;
        if (threadIdx.x < 64) {
            const bool ok = wg_blk_diag(Sm, ld, ma, p0, dg);
            if (!ok && threadIdx.x == 0) *flag = 1;
        }
        __syncthreads();
        if (*flag) return false;
        if (P + 1 == nb) break;
        // rows below: L[i][p0+j] = (W[i][p0+j] - sum_{k<j} L[i][p0+k] L[p0+j][p0+k]) / L_jj
        // (the solved entries are re-read from LDS, not held in registers: the
        // kernel stays at four workgroups per CU)
        for (int i = p0 + WG_TB + (int)threadIdx.x; i < ma; i += WG_NT) {
            for (int j = 0; j < w; ++j) {
                double v = Sm[i * ld + p0 + j];
                for (int k = 0; k < j; ++k) v = fma(-Sm[(p0 + k) * ld + i], Sm[(p0 + k) * ld + p0 + j], v);
                Sm[(p0 + j) * ld + i] = v * dg[p0 + j];
            }
        }
        __syncthreads();
        // trailing update of the lower tiles (I >= J > P), a tile per wavefront in turn
        const int nt = nb - P - 1, ntile = nt * (nt + 1) / 2;
        for (int t = wv; t < ntile; t += WG_NT / 64) {
            int I = 0;
            while ((I + 1) * (I + 2) / 2 <= t) ++I;
            const int J = t - I * (I + 1) / 2;
            const int I0 = WG_TB * (P + 1 + I), J0 = WG_TB * (P + 1 + J);
            wg_d4 acc;
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[q] = wg_el(Sm, ld, ma, I0 + g + 4 * q, J0 + r16);
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int kc = p0 + 4 * s + g;     // panel column k (its L^T row in the upper part)
                const double av = (kc < p0 + w) ? -wg_el(Sm, ld, ma, kc, I0 + r16) : 0.0;
                const double bv = (kc < p0 + w) ? wg_el(Sm, ld, ma, kc, J0 + r16) : 0.0;
                acc = WG_MFMA(av, bv, acc);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int ri = I0 + g + 4 * q, cj = J0 + r16;
                if (ri < ma && cj < ma && cj <= ri) Sm[ri * ld + cj] = acc[q];
            }
        }
        __syncthreads();
    }
    return true;
}

// X = L^-1 (lower part, diagonal included) from wg_blk_cholesky's output
PHX_HD void wg_blk_trtri(double* Sm, int ld, int ma, const double* dg) {
    const int nb = (ma + WG_TB - 1) / WG_TB;
    const int l = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6), r16 = l & 15, g = l >> 4;
    // diagonal blocks: a thread per (block, column c): X[c][c] = 1/L_cc,
    // X[i][c] = -(sum_{k=c}^{i-1} L[i][k] X[k][c]) / L_ii
    for (int e = (int)threadIdx.x; e < nb * WG_TB; e += WG_NT) {
        const int p0 = (e >> 4) * WG_TB, c = e & 15;
        const int w = ma - p0 < WG_TB ? ma - p0 : WG_TB;
        if (c >= w) continue;
        Sm[(p0 + c) * ld + p0 + c] = dg[p0 + c];
        for (int i = c + 1; i < w; ++i) {
            double v = 0.0;
            for (int k = c; k < i; ++k) v = fma(Sm[(p0 + k) * ld + p0 + i], Sm[(p0 + k) * ld + p0 + c], v);
            Sm[(p0 + i) * ld + p0 + c] = -v * dg[p0 + i];
        }
    }
    __syncthreads();
    for (int I = 1; I < nb; ++I) {
        const int I0 = WG_TB * I;
        for (int J = wv; J < I; J += WG_NT / 64) {
            const int J0 = WG_TB * J;
            wg_d4 tt = {0.0, 0.0, 0.0, 0.0};
            for (int K = J; K < I; ++K) {
                const int K0 = WG_TB * K;
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const int kr = K0 + 4 * s + g;
                    tt = WG_MFMA(wg_el(Sm, ld, ma, kr, I0 + r16),              // L[I0+r][kr] (upper)
                                 wg_el(Sm, ld, ma, kr, J0 + r16, K == J), tt);   // X[kr][J0+j]
                }
            }
            wg_d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int s = 0; s < 4; ++s)
                acc = WG_MFMA(-wg_el(Sm, ld, ma, I0 + r16, I0 + 4 * s + g, true), tt[s], acc);   // -X_II T
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int ri = I0 + g + 4 * q, cj = J0 + r16;
                if (ri < ma && cj < ma) Sm[ri * ld + cj] = acc[q];
            }
        }
        __syncthreads();
    }
}

// M^-1 = X^T X over the whole ma x ma (both triangles), from wg_blk_trtri's X
PHX_HD void wg_blk_lauum(double* Sm, int ld, int ma) {
    const int nb = (ma + WG_TB - 1) / WG_TB;
    const int l = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6), r16 = l & 15, g = l >> 4;
    const int ntile = nb * (nb + 1) / 2;
    constexpr int TPW = (WG_BLK_MAX / WG_TB) * (WG_BLK_MAX / WG_TB + 1) / 2 / (WG_NT / 64) + 1;
    wg_d4 acc[TPW];
    int tI[TPW], tJ[TPW];
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
        const int t = wv + u * (WG_NT / 64);
        tI[u] = -1;
        tJ[u] = 0;
        acc[u] = wg_d4{0.0, 0.0, 0.0, 0.0};
        if (t >= ntile) continue;
        int I = 0;
        while ((I + 1) * (I + 2) / 2 <= t) ++I;
        const int J = t - I * (I + 1) / 2;
        tI[u] = I;
        tJ[u] = J;
        for (int K = I; K < nb; ++K) {
            const int K0 = WG_TB * K;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int kr = K0 + 4 * s + g;
                acc[u] = WG_MFMA(wg_el(Sm, ld, ma, kr, WG_TB * I + r16, true),    // X[kr][I0+r]
                                 wg_el(Sm, ld, ma, kr, WG_TB * J + r16, true), acc[u]);
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
        if (tI[u] < 0) continue;
        const int I0 = WG_TB * tI[u], J0 = WG_TB * tJ[u];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int ri = I0 + g + 4 * q, cj = J0 + r16;
            if (ri < ma && cj < ma) {
                Sm[ri * ld + cj] = acc[u][q];
                Sm[cj * ld + ri] = acc[u][q];
            }
        }
    }
    __syncthreads();
}
#else
// Host (tests/emu, WG_NT = 1): the scalar steps in the same storage
PHX_HD bool wg_blk_cholesky(double* Sm, int ld, int ma, double* dg, int32_t* flag) {
    (void)flag;
    for (int j = 0; j < ma; ++j) {
        const double d = Sm[j * ld + j];
        if (!(d > 0.0)) return false;
        const double sd = sqrt(d);
        dg[j] = 1.0 / sd;
        for (int i = j + 1; i < ma; ++i) Sm[j * ld + i] = Sm[i * ld + j] / sd;
        for (int i = j + 1; i < ma; ++i)
            for (int k = j + 1; k <= i; ++k) Sm[i * ld + k] = fma(-Sm[j * ld + i], Sm[j * ld + k], Sm[i * ld + k]);
    }
    return true;
}
PHX_HD void wg_blk_trtri(double* Sm, int ld, int ma, const double* dg) {
    for (int c = 0; c < ma; ++c) {
        Sm[c * ld + c] = dg[c];
        for (int i = c + 1; i < ma; ++i) {
            double v = 0.0;
            for (int k = c; k < i; ++k) v = fma(Sm[k * ld + i], Sm[k * ld + c], v);
            Sm[i * ld + c] = -v * dg[i];
        }
    }
}
PHX_HD void wg_blk_lauum(double* Sm, int ld, int ma) {
    // row by row from the bottom: M[i][j] (j <= i) needs X rows >= i only,
    // and row i of X is no longer needed once M's row i is written
    for (int i = 0; i < ma; ++i)
        for (int j = 0; j <= i; ++j) {
            double v = 0.0;
            for (int k = i; k < ma; ++k) v = fma(Sm[k * ld + i], Sm[k * ld + j], v);
            Sm[j * ld + i] = v;            // the upper part first (X lives in the lower)
        }
    for (int i = 0; i < ma; ++i)
        for (int j = 0; j < i; ++j) Sm[i * ld + j] = Sm[j * ld + i];
}
#endif

// Returns (uniformly) the number of rounds the lane used when the point in
// L.xp / L.z passes the KKT certificate, else 0; rounds > 1 allow primal-dual
// active-set updates in between.
// BLK (Schur complements of at most WG_BLK_MAX rows): 1, the blocked MFMA
// factor and inverse (wg_blk_cholesky, wg_blk_trtri) in the scalar path's
// storage; 2, also M^-1 = X^T X (wg_blk_lauum) and one dense mat-vec per
// refinement step (measured: as many flops, but 16 % more active-set rounds on
// farmer cm=10 -- the emulation shows the same -- so not the default); 0, the
// scalar paired-pivot Cholesky and explicit inverse.  1 and 0 refine with two
// triangular mat-vecs per step.
template <int BLK>
PHX_HD int wg_warm(const Prob& P, const State& St, const WgPairs& G, const Opts& O, int s, const WgLds& L,
                   int rounds, double tol0, unsigned long long* prof = nullptr) {
    WG_T0();
    const int S = P.S, n = P.n, m = P.m;
    const double reg = O.reg;
    // ---- scenario data and the pattern into LDS ----
    for (int k = WG_TID; k < P.nnz; k += WG_NT) {
        if (L.own_a) L.a[k] = aval(P, k, s);
        if (L.own_pat) {
            L.ri[k] = (int16_t)P.rowidx[k];
            L.c2[k] = (int16_t)P.csc2csr[k];
        }
        L.ci[k] = (int16_t)P.colidx[k];
    }
    for (int j = WG_TID; j <= n; j += WG_NT) L.cp[j] = (int16_t)P.colptr[j];
    for (int i = WG_TID; i <= m; i += WG_NT) L.rp[i] = (int16_t)P.rowptr[i];
    double qm = 0.0;
    for (int j = WG_TID; j < n; j += WG_NT) {
        double q, p;
        col_cost(P, j, s, q, p);
        L.qq[j] = q;
        L.pp[j] = p;
        qm = fmax(qm, fabs(q / P.dc[j]));
    }
    const double dtol = O.kkt_tol * (1.0 + wg_max(qm, L.red));
    const double ptol = O.kkt_tol;
    WG_SYNC();
    const int16_t *cp = L.cp, *ri = L.ri, *c2 = L.c2, *rp = L.rp, *ci = L.ci;
    // ---- round 0: classify the previous solution (polish_lane's rule) ----
    for (int j = WG_TID; j < n; j += WG_NT) {
        const int64_t o = ix(j, s, S);
        const double x = St.xT[o];
        const double l = P.lb.at(j, s), u = P.ub.at(j, s);
        double aty = 0.0;
        for (int k = cp[j]; k < cp[j + 1]; ++k) aty += L.a[c2[k]] * St.yT[ix(ri[k], s, S)];
        const double lam = L.qq[j] + L.pp[j] * x - aty;
        int8_t c = 0;
        if (isfinite(l) && (x - l <= tol0 * (1.0 + fabs(l)) || x - l < lam)) c = 1;
        else if (isfinite(u) && (u - x <= tol0 * (1.0 + fabs(u)) || u - x < -lam)) c = 2;
        L.cc[j] = c;
        L.xp[j] = c == 1 ? l : (c == 2 ? u : x);
    }
    // (rows: a quad each, the row's entries interleaved over its four threads --
    // farmer cm=10's land row has 30, sslp's facility rows 47: one thread per row
    // made them the phase's serial chain)
    for (int i = WG_QID; i < m; i += WG_QN) {
        double ax = 0.0;
        for (int k = rp[i] + WG_QL; k < rp[i + 1]; k += WG_QW) ax += L.a[k] * St.xT[ix(ci[k], s, S)];
        ax = wg_quad_sum(ax);
        if (WG_QL != 0) continue;
        const double bl = P.bl.at(i, s), bu = P.bu.at(i, s);
        const double yv = St.yT[ix(i, s, S)];
        int8_t r = 0;
        if (isfinite(bl) && (ax - bl <= tol0 * (1.0 + fabs(bl)) || ax - bl < yv)) r = 1;
        else if (isfinite(bu) && (bu - ax <= tol0 * (1.0 + fabs(bu)) || bu - ax < -yv)) r = 2;
        L.rc[i] = r;
        L.z[i] = r ? -yv : 0.0;
    }
    WG_SYNC();
    WG_TP(0);
    for (int round = 0; round < rounds; ++round) {
        // active rows in compact order: the Schur complement is ma x ma
        wg_compact(L, m);
        if (WG_TID == 0) { L.flag[0] = 0; L.flag[1] = 0; L.flag[2] = 0; }
        WG_SYNC();
        const int ma = L.flag[3];
        const int ld = ma | 1;
        // ---- the cached factor of this active set and prox weights, if any ----
        const bool cache = G.fac != nullptr;
        bool reused = false;
        if (cache && G.ok[s]) {
            const int8_t* kc = G.key + (int64_t)s * G.key_stride;
            const double* pk = G.pkey + (int64_t)s * (G.N + 1);
            bool diff = false;
            for (int j = WG_TID; j < n; j += WG_NT) diff = diff || kc[j] != L.cc[j];
            for (int i = WG_TID; i < m; i += WG_NT) diff = diff || kc[n + i] != L.rc[i];
            for (int t = WG_TID; t < G.N; t += WG_NT) diff = diff || pk[t] != P.pN[ix(t, s, S)];
            if (WG_TID == 0 && pk[G.N] != reg) diff = true;
            if (diff) L.flag[1] = 1;
            WG_SYNC();
            if (L.flag[1] == 0) {
                // (the refinement reads only L^-1, the lower triangle)
                const double* f = G.fac + (int64_t)s * G.fac_stride;
                for (int e = WG_TID; e < ma * ld; e += WG_NT) {
                    const int i = e / ld, c = e - i * ld;
                    if (BLK == 2 ? c < ma : c <= i) L.Sm[e] = f[e];
                }
                WG_SYNC();
                WG_CNT(10);
                reused = true;
            }
        }
        if (!reused) {
            // ---- Schur complement A_RF (P_FF+reg)^-1 A_RF' + reg I (lower part).
            //      Row stride ld = ma | 1 (odd): a wavefront reading one column of
            //      64 rows hits distinct LDS banks (an even stride of 40 doubles
            //      made that a 16-way conflict) ----
            for (int e = WG_TID; e < ma * ld; e += WG_NT) {
                const int i = e / ld, k = e - i * ld;
                L.Sm[e] = (i == k) ? reg : 0.0;
            }
            // (P_FF + reg)^-1 per column, 0 on the non-free ones: one division per
            // column instead of one per shared-column triple (L.r1 is free here:
            // the refinement's first step rewrites it)
            for (int j = WG_TID; j < n; j += WG_NT) L.r1[j] = L.cc[j] == 0 ? 1.0 / (L.pp[j] + reg) : 0.0;
            WG_SYNC();
            // (the long pairs -- a row with itself -- a quad each, their shared
            // columns interleaved; the others a thread each)
            for (int p = WG_QID; p < G.nlong; p += WG_QN) {
                const int pa = L.pos[G.ia[p]], pb = L.pos[G.ib[p]];
                if (pa < 0 || pb < 0) continue;
                double v = 0.0;
                for (int t = G.ptr[p] + WG_QL; t < G.ptr[p + 1]; t += WG_QW) {
                    const int ka = G.ka[t];
                    v += L.a[ka] * L.a[G.kb[t]] * L.r1[ci[ka]];
                }
                v = wg_quad_sum(v);
                if (WG_QL == 0) L.Sm[pa * ld + pb] += v;
            }
            for (int p = G.nlong + WG_TID; p < G.npair; p += WG_NT) {
                const int pa = L.pos[G.ia[p]], pb = L.pos[G.ib[p]];
                if (pa < 0 || pb < 0) continue;
                double v = 0.0;
                for (int t = G.ptr[p]; t < G.ptr[p + 1]; ++t) {
                    const int ka = G.ka[t];
                    v += L.a[ka] * L.a[G.kb[t]] * L.r1[ci[ka]];
                }
                L.Sm[pa * ld + pb] += v;
            }
            WG_SYNC();
            WG_TP(1);
          if (BLK) {
            if (!wg_blk_cholesky(L.Sm, ld, ma, L.dg, L.flag + 2)) return 0;
            WG_TP(2);
            wg_blk_trtri(L.Sm, ld, ma, L.dg);
            if (BLK == 2) wg_blk_lauum(L.Sm, ld, ma);
            WG_TP(3);
          } else {
            // ---- Cholesky: trailing update on the lower part, L[i][k] (i > k)
            //      stored transposed at Sm[k*ld+i], 1/diagonal in dg ----
            // (a quad per row: its four threads take interleaved columns k, so
            // one pivot's update is spread over 4x as many threads; the pivot
            // row element lij is read by all four, written by none of them)
            bool spd = true;
            // pivots in pairs (a, b = a+1), one barrier per pair: the second
            // pivot's column and diagonal are corrected for the first on the
            // fly with the very expressions the one-pivot step would store
            // (row k col b: Sm[k][b] - (Sm[k][a] / d_a) * Sm[b][a]), so the
            // factor is the same; half the barriers and row round trips
            int j2 = 0;
            for (; j2 + 1 < ma; j2 += 2) {
                const int a = j2, b = j2 + 1;
                const double d0 = L.Sm[a * ld + a];
                if (!(d0 > 0.0)) { spd = false; break; }
                const double e = L.Sm[b * ld + a], id0 = 1.0 / d0;
                const double d1 = L.Sm[b * ld + b] - (e * id0) * e;
                if (!(d1 > 0.0)) { spd = false; break; }
                const double sd0 = sqrt(d0), sd1 = sqrt(d1), id1 = 1.0 / d1;
                // (a group of gw threads per trailing row, as wide as the rows
                // left allow: gw = 16 at 16 rows or fewer, 8 at 32, 4 at 64 --
                // the step's time is its longest row's entries over gw; every
                // entry is still updated by one thread with the same
                // expression, so the factor does not depend on gw)
#if defined(__HIP_DEVICE_COMPILE__)
                const int nrow = ma - b - 1;
                const int gs = nrow <= WG_NT / 16 ? 4 : (nrow <= WG_NT / 8 ? 3 : (nrow <= WG_NT / 4 ? 2 : 1));
                const int gw = 1 << gs, gid = WG_TID >> gs, gl = WG_TID & (gw - 1), gn = WG_NT >> gs;
#else
                const int gw = 1, gid = 0, gl = 0, gn = 1;
#endif
                for (int i = b + 1 + gid; i < ma; i += gn) {
                    double* row = L.Sm + (size_t)i * ld;
                    const double lia = row[a];
                    const double f0 = lia * id0;
                    const double lib = row[b] - f0 * e;
                    const double f1 = lib * id1;
                    int k = b + 1 + gl;
                    for (; k <= i; k += gw) {
                        const double ga = L.Sm[k * ld + a];
                        const double h = L.Sm[k * ld + b] - (ga * id0) * e;
                        const double t = row[k] - f0 * ga;
                        row[k] = t - f1 * h;
                    }
                    if (gl == 0) {
                        L.Sm[a * ld + i] = lia / sd0;
                        L.Sm[b * ld + i] = lib / sd1;
                    }
                }
                if (WG_TID == 0) {
                    L.dg[a] = 1.0 / sd0;
                    L.dg[b] = 1.0 / sd1;
                    L.Sm[a * ld + b] = e / sd0;
                }
                WG_SYNC();
            }
            for (int jj = spd ? j2 : ma; jj < ma; ++jj) {
                const double d = L.Sm[jj * ld + jj];
                if (!(d > 0.0)) { spd = false; break; }
                const double sd = sqrt(d), id = 1.0 / d;
                for (int i = jj + 1 + WG_QID; i < ma; i += WG_QN) {
                    double* row = L.Sm + (size_t)i * ld;
                    const double lij = row[jj];
                    const double f = lij * id;
                    int k = jj + 1 + WG_QL;
                    // batches of 2 per thread: the loads issued before the stores
                    for (; k + WG_QW <= i; k += 2 * WG_QW) {
                        const double g0 = L.Sm[k * ld + jj], g1 = L.Sm[(k + WG_QW) * ld + jj];
                        const double r0 = row[k], r1 = row[k + WG_QW];
                        row[k] = r0 - f * g0;
                        row[k + WG_QW] = r1 - f * g1;
                    }
                    for (; k <= i; k += WG_QW) row[k] -= f * L.Sm[k * ld + jj];
                    if (WG_QL == 0) L.Sm[jj * ld + i] = lij / sd;
                }
                if (WG_TID == 0) L.dg[jj] = 1.0 / sd;
                WG_SYNC();
            }
            if (!spd) {
#if defined(PHX_WG_DEBUG) && !defined(__HIP_DEVICE_COMPILE__)
                fprintf(stderr, "[wg fail] s=%d not spd at round %d ma=%d\n", s, round, ma);
#endif
                return 0;
            }
            WG_TP(2);
            // ---- explicit inverse of L into the lower part (diagonal included).
            //      Round 5: the blocked MFMA inverse (wg_blk_trtri) after the
            //      scalar factor when it fits its tiles -- farmer cm=10: the
            //      scalar inverse's ma-step column chains took 731 against the
            //      blocked one's 311 Mcycles per ten passes (r05 s21), while the
            //      scalar factor beats the blocked one (796 against 1,423) ----
            const bool blk_inv = ma <= WG_BLK_MAX;
            if (blk_inv) wg_blk_trtri(L.Sm, ld, ma, L.dg);
            // (the scalar inverse: a quad per column c, interleaved k, two partial
            // sums per thread, combined inside the quad; every thread of the quad
            // holds the new entry and writes the same value, so the next step's
            // reads of it by the other three need no ordering beyond their own store)
            for (int c = WG_QID; c < (blk_inv ? 0 : ma); c += WG_QN) {
                if (WG_QL == 0) L.Sm[c * ld + c] = L.dg[c];
                for (int i = c + 1; i < ma; ++i) {
                    double v0 = WG_QL == 0 ? L.Sm[c * ld + i] * L.dg[c] : 0.0, v1 = 0.0;
                    int k = c + 1 + WG_QL;
                    for (; k + WG_QW < i; k += 2 * WG_QW) {
                        v0 += L.Sm[k * ld + i] * L.Sm[k * ld + c];
                        v1 += L.Sm[(k + WG_QW) * ld + i] * L.Sm[(k + WG_QW) * ld + c];
                    }
                    for (; k < i; k += WG_QW) v0 += L.Sm[k * ld + i] * L.Sm[k * ld + c];
                    L.Sm[i * ld + c] = -wg_quad_sum(v0 + v1) * L.dg[i];
                }
            }
            WG_SYNC();
            WG_TP(3);
          }
        }
        // ---- iterative refinement on the unregularised KKT (a proximal-point
        //      iteration) ----
        for (int it = 0; it < O.refine_steps; ++it) {
            // r1 = H^-1 (-q - P x - A'z) on the free columns, 0 elsewhere (the
            // division by the column's owner, once; the rows' products below
            // then need none).  Only the first step forms it from the data:
            // after a step the column residual is reg dx exactly (the
            // regularised system's definition, see the update below), so the
            // update writes the next step's r1 and this phase's barrier goes
            for (int j = WG_TID; j < (it == 0 ? n : 0); j += WG_NT) {
                // (operands loaded before the branch: one round trip, the split
                // layout's column vectors being global)
                const int8_t cj = L.cc[j];
                const double qq = L.qq[j], pp = L.pp[j], xj = L.xp[j];
                if (cj) { L.r1[j] = 0.0; continue; }
                double atz = 0.0;
                for (int k = cp[j]; k < cp[j + 1]; ++k) atz += L.a[c2[k]] * L.z[ri[k]];
                L.r1[j] = (-qq - pp * xj - atz) / (pp + reg);
            }
            if (it == 0) WG_SYNC();
            WG_TP(11);
            // t = A_R (x + H^-1 r) - b_R: a quad per active row
            for (int q = WG_QID; q < ma; q += WG_QN) {
                const int i = L.ar[q];
                double adr = 0.0, ax = 0.0;
                for (int k = rp[i] + WG_QL; k < rp[i + 1]; k += WG_QW) {
                    const int j = ci[k];
                    ax += L.a[k] * L.xp[j];
                    adr += L.a[k] * L.r1[j];
                }
                ax = wg_quad_sum(ax);
                adr = wg_quad_sum(adr);
                if (WG_QL == 0) {
                    const double b = L.rc[i] == 1 ? P.bl.at(i, s) : P.bu.at(i, s);
                    L.t[q] = adr - (b - ax);
                }
            }
            WG_SYNC();
            WG_TP(12);
            if (BLK == 2) {
                // dz = M^-1 t (full rows; compact order) into u
                for (int i = WG_QID; i < ma; i += WG_QN) {
                    double v0 = 0.0, v1 = 0.0;
                    const double* row = L.Sm + (size_t)i * ld;
                    int k = WG_QL;
                    for (; k + WG_QW < ma; k += 2 * WG_QW) {
                        v0 += row[k] * L.t[k];
                        v1 += row[k + WG_QW] * L.t[k + WG_QW];
                    }
                    for (; k < ma; k += WG_QW) v0 += row[k] * L.t[k];
                    const double v = wg_quad_sum(v0 + v1);
                    if (WG_QL == 0) L.u[i] = v;
                }
                WG_SYNC();
            } else {
            // u = L^-1 t ; then t = L^-T u (dz, compact order)
            for (int i = WG_QID; i < ma; i += WG_QN) {
                double v0 = 0.0, v1 = 0.0;
                const double* row = L.Sm + (size_t)i * ld;
                int k = WG_QL;
                for (; k + WG_QW <= i; k += 2 * WG_QW) {
                    v0 += row[k] * L.t[k];
                    v1 += row[k + WG_QW] * L.t[k + WG_QW];
                }
                for (; k <= i; k += WG_QW) v0 += row[k] * L.t[k];
                const double v = wg_quad_sum(v0 + v1);
                if (WG_QL == 0) L.u[i] = v;
            }
            WG_SYNC();
            for (int k = WG_QID; k < ma; k += WG_QN) {
                double v0 = 0.0, v1 = 0.0;
                int i = k + WG_QL;
                for (; i + WG_QW < ma; i += 2 * WG_QW) {
                    v0 += L.Sm[i * ld + k] * L.u[i];
                    v1 += L.Sm[(i + WG_QW) * ld + k] * L.u[i + WG_QW];
                }
                for (; i < ma; i += WG_QW) v0 += L.Sm[i * ld + k] * L.u[i];
                const double v = wg_quad_sum(v0 + v1);
                if (WG_QL == 0) L.t[k] = v;
            }
            WG_SYNC();
            }
            WG_TP(13);
            const double* dz = BLK == 2 ? L.u : L.t;
            double dmax = 0.0, xmax = 0.0;
            for (int j = WG_TID; j < n; j += WG_NT) {
                const int8_t cj = L.cc[j];
                const double r1 = L.r1[j], pp = L.pp[j], xj = L.xp[j];
                if (cj) continue;
                double atz = 0.0;
                for (int k = cp[j]; k < cp[j + 1]; ++k) {
                    const int q = L.pos[ri[k]];
                    if (q >= 0) atz += L.a[c2[k]] * dz[q];
                }
                // (P + reg) dx = (P + reg) r1 - A'dz, so the unregularised
                // residual after the step, -q - P x' - A'z', is
                // (P + reg) r1 - P dx - A'dz = reg dx: the next step's r1
                const double ih = 1.0 / (pp + reg);
                const double dx = r1 - atz * ih;
                const double x = xj + dx;
                L.xp[j] = x;
                L.r1[j] = reg * dx * ih;
                dmax = fmax(dmax, fabs(dx));
                xmax = fmax(xmax, fabs(x));
            }
            for (int q = WG_TID; q < ma; q += WG_NT) {
                const int i = L.ar[q];
                const double zn = L.z[i] + dz[q];
                dmax = fmax(dmax, fabs(dz[q]));
                xmax = fmax(xmax, fabs(zn));
                L.z[i] = zn;
            }
            // stop once the correction vanishes (phx_lane.h kkt_refine's rule)
            wg_max2(dmax, xmax, L.red);
            const bool done = dmax <= 1e-10 * (1.0 + xmax);
            WG_TP(14);
            WG_CNT(8);
            if (done) break;
        }
        WG_TP(4);
        WG_CNT(9);
        // ---- certificate (polish_lane's, unscaled quantities); keeps the
        //      multipliers (r1) and row activities (u) for the update ----
        bool bad = false;
        for (int j = WG_TID; j < n; j += WG_NT) {
            const double x = L.xp[j];
            const double l = P.lb.at(j, s), u = P.ub.at(j, s);
            const double dc = P.dc[j], qq = L.qq[j], pp = L.pp[j];
            const int8_t c = L.cc[j];
            if (x < l && (l - x) * dc > ptol * (1.0 + fabs(l * dc))) bad = true;
            if (x > u && (x - u) * dc > ptol * (1.0 + fabs(u * dc))) bad = true;
            double atz = 0.0;
            for (int k = cp[j]; k < cp[j + 1]; ++k) atz += L.a[c2[k]] * L.z[ri[k]];
            const double lam = (qq + pp * x + atz) / dc;
            L.r1[j] = lam;
            if (!(lam - lam == 0.0)) bad = true;   // non-finite x or z: no comparison would fail
            if (c == 0) {
                if (fabs(lam) > dtol) bad = true;
            } else if (!(l == u)) {
                if (c == 1 && lam < -dtol) bad = true;
                if (c == 2 && lam > dtol) bad = true;
            }
        }
        for (int i = WG_QID; i < m; i += WG_QN) {
            double ax = 0.0;
            for (int k = rp[i] + WG_QL; k < rp[i + 1]; k += WG_QW) ax += L.a[k] * L.xp[ci[k]];
            ax = wg_quad_sum(ax);
            if (WG_QL != 0) continue;
            L.u[i] = ax;
            const double dr = P.dr[i];
            const double bl = P.bl.at(i, s), bu = P.bu.at(i, s);
            if (!(ax - ax == 0.0) || !(L.z[i] - L.z[i] == 0.0)) bad = true;
            if (ax < bl && (bl - ax) / dr > ptol * (1.0 + fabs(bl / dr))) bad = true;
            if (ax > bu && (ax - bu) / dr > ptol * (1.0 + fabs(bu / dr))) bad = true;
            // complementarity: an active row sits at its side (the refinement's
            // fixed point; a solve whose refinement stopped short fails here)
#ifndef PHX_WG_NO_COMPL
            if (L.rc[i]) {
                const double b = L.rc[i] == 1 ? bl : bu;
                if (fabs(ax - b) / dr > ptol * (1.0 + fabs(b / dr))) bad = true;
            }
#endif
            if (L.rc[i] && !(bl == bu)) {
                const double y = -L.z[i] * dr;
                if (L.rc[i] == 1 && y < -dtol) bad = true;
                if (L.rc[i] == 2 && y > dtol) bad = true;
            }
        }
        if (bad) L.flag[0] = 1;
        WG_SYNC();
        WG_TP(5);
        if (L.flag[0] == 0) {
            if (cache && !reused) {
                // keep the certified set's factor (L^-1, lower triangle) for the
                // scenario's next solve -- only the final round's: the earlier
                // rounds' sets are left behind (storing every round's wrote 4x
                // the bytes of the whole solve's inputs and outputs, PMC r03 s16)
                double* f = G.fac + (int64_t)s * G.fac_stride;
                for (int e = WG_TID; e < ma * ld; e += WG_NT) {
                    const int i = e / ld, c = e - i * ld;
                    if (BLK == 2 ? c < ma : c <= i) f[e] = L.Sm[e];
                }
                int8_t* kc = G.key + (int64_t)s * G.key_stride;
                double* pk = G.pkey + (int64_t)s * (G.N + 1);
                for (int j = WG_TID; j < n; j += WG_NT) kc[j] = L.cc[j];
                for (int i = WG_TID; i < m; i += WG_NT) kc[n + i] = L.rc[i];
                for (int t = WG_TID; t < G.N; t += WG_NT) pk[t] = P.pN[ix(t, s, S)];
                if (WG_TID == 0) {
                    pk[G.N] = reg;
                    G.ok[s] = 1;
                }
            }
            return round + 1;
        }
        if (round + 1 == rounds) {
#if defined(PHX_WG_DEBUG) && !defined(__HIP_DEVICE_COMPILE__)
            fprintf(stderr, "[wg fail] s=%d no certificate after %d rounds\n", s, rounds);
#endif
            break;
        }
        // ---- primal-dual active-set update: wrong-signed multipliers leave,
        //      violated bounds and rows enter.  Round 4: after WG_SINGLE_AFTER
        //      rounds only the worst violation changes (phx_lane.h's
        //      anti-cycling rule as it was then: the largest relative primal
        //      violation, else the largest wrong-signed multiplier) -- measured on sslp
        //      (emulation, 300 scenarios x 6 iterations): 87 of 1,800 solves
        //      ran out of their 16 full-change rounds, cycling ----
        const bool single = round + 1 >= G.single_after;
        double bk = 0.0;     // the best change's key (0: none): primal 2 + v/(1+v), dual 1 + v/(1+v)
        int bi = -1;         // its element: column j, or n + row i
        for (int j = WG_TID; j < n; j += WG_NT) {
            const double l = P.lb.at(j, s), u = P.ub.at(j, s);
            const double x = L.xp[j], lam = L.r1[j], dc = P.dc[j];
            const int8_t c = L.cc[j];
            if (l == u) continue;
            int8_t cn = c;
            double key = 0.0;
            if (c == 1 && lam < -dtol) { cn = 0; key = 1.0 + (-lam) / (1.0 - lam); }
            else if (c == 2 && lam > dtol) { cn = 0; key = 1.0 + lam / (1.0 + lam); }
            else if (c == 0 && x < l && (l - x) * dc > ptol * (1.0 + fabs(l * dc))) {
                const double v = (l - x) * dc / (1.0 + fabs(l * dc));
                cn = 1; key = 2.0 + v / (1.0 + v);
            } else if (c == 0 && x > u && (x - u) * dc > ptol * (1.0 + fabs(u * dc))) {
                const double v = (x - u) * dc / (1.0 + fabs(u * dc));
                cn = 2; key = 2.0 + v / (1.0 + v);
            }
            if (!single) {
                if (cn != c) { L.cc[j] = cn; if (cn) L.xp[j] = cn == 1 ? l : u; }
            } else if (key > bk) {
                bk = key;
                bi = j;
            }
        }
        for (int i = WG_TID; i < m; i += WG_NT) {
            const double bl = P.bl.at(i, s), bu = P.bu.at(i, s);
            if (bl == bu) continue;
            const double ax = L.u[i], dr = P.dr[i];
            const double y = -L.z[i] * dr;
            const int8_t r = L.rc[i];
            int8_t rn = r;
            double key = 0.0;
            if (r == 1 && y < -dtol) { rn = 0; key = 1.0 + (-y) / (1.0 - y); }
            else if (r == 2 && y > dtol) { rn = 0; key = 1.0 + y / (1.0 + y); }
            else if (r == 0 && ax < bl && (bl - ax) / dr > ptol * (1.0 + fabs(bl / dr))) {
                const double v = (bl - ax) / dr / (1.0 + fabs(bl / dr));
                rn = 1; key = 2.0 + v / (1.0 + v);
            } else if (r == 0 && ax > bu && (ax - bu) / dr > ptol * (1.0 + fabs(bu / dr))) {
                const double v = (ax - bu) / dr / (1.0 + fabs(bu / dr));
                rn = 2; key = 2.0 + v / (1.0 + v);
            }
            if (!single) {
                if (rn != r) { L.rc[i] = rn; if (rn == 0) L.z[i] = 0.0; }
            } else if (key > bk) {
                bk = key;
                bi = n + i;
            }
        }
        if (single) {
            wg_argmax(bk, bi, L.red);      // uniform: the worst violation (smallest element on ties)
            if (WG_TID == 0 && bi >= 0) {
                if (bi < n) {
                    const int j = bi;
                    const int8_t c = L.cc[j];
                    if (c != 0) L.cc[j] = 0;
                    else {
                        const double l = P.lb.at(j, s), u = P.ub.at(j, s);
                        const bool lo = L.xp[j] < l;
                        L.cc[j] = lo ? 1 : 2;
                        L.xp[j] = lo ? l : u;
                    }
                } else {
                    const int i = bi - n;
                    const int8_t r = L.rc[i];
                    if (r != 0) { L.rc[i] = 0; L.z[i] = 0.0; }
                    else L.rc[i] = L.u[i] < P.bl.at(i, s) ? 1 : 2;
                }
            }
        }
        WG_SYNC();
        WG_TP(6);
    }
    return 0;
}

// sum over the workgroup (butterflies, then the wavefronts in order through
// LDS), identity on the host
PHX_HD double wg_sum(double v, double* red) {
#if defined(__HIP_DEVICE_COMPILE__)
    v = wave_reduce<0>(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    v = red[0];
    for (int w = 1; w < WG_NT / 64; ++w) v += red[w];
#else
    (void)red;
#endif
    return v;
}

// A certified lane's outputs, as finalize_lane (phx_core.h) writes them:
// unscaled x and row duals, objective c'x + qN'x_N + pN x_N^2 / 2 + kN.
PHX_HD void wg_write_out(const Prob& P, const WgLds& L, const double* c_unscaled_p, int64_t c_si, int64_t c_ss,
                         int s, double* x_out, double* y_out, double* obj_out) {
    const int S = P.S;
    double f = 0.0;
    for (int j = WG_TID; j < P.n; j += WG_NT) {
        const double x = L.xp[j] * P.dc[j];
        x_out[ix(j, s, S)] = x;
        f += c_unscaled_p[(int64_t)j * c_si + (int64_t)s * c_ss] * x;
        const int sl = P.col_slot[j];
        if (sl >= 0) f += P.qN[ix(sl, s, S)] * x + 0.5 * P.pN[ix(sl, s, S)] * x * x;
    }
    if (y_out)
        for (int i = WG_TID; i < P.m; i += WG_NT) y_out[ix(i, s, S)] = -L.z[i] * P.dr[i];
    f = wg_sum(f, L.red);
    if (WG_TID == 0) obj_out[s] = P.kN[s] + f;
}

// A lane the pass leaves to PDHG: k_begin_solve's warm start (mode 1) for it,
// which the pass replaces when it runs.
PHX_HD void wg_begin_generic(const Prob& P, const State& St, int s) {
    const int S = P.S;
    for (int j = WG_TID; j < P.n; j += WG_NT) St.x0[ix(j, s, S)] = St.x[ix(j, s, S)];
    for (int i = WG_TID; i < P.m; i += WG_NT) St.y0[ix(i, s, S)] = St.y[ix(i, s, S)];
    if (WG_TID == 0) {
        St.hk[s] = 0;
        St.r0[s] = 1e301;
        St.rprev[s] = 1e301;
        St.status[s] = RUNNING;
        St.iters[s] = 0;
        St.err[s] = 1e300;
        St.flags[s] = 0;
    }
}

// A certified lane: its point becomes the solution and the next warm start
// (adopt_polished's effect).
PHX_HD void wg_adopt(const Prob& P, const State& St, const WgLds& L, int s) {
    const int S = P.S;
    for (int j = WG_TID; j < P.n; j += WG_NT) {
        const int64_t o = ix(j, s, S);
        const double v = L.xp[j];
        St.xT[o] = v; St.x[o] = v; St.x0[o] = v;
    }
    for (int i = WG_TID; i < P.m; i += WG_NT) {
        const int64_t o = ix(i, s, S);
        const double v = -L.z[i];
        St.yT[o] = v; St.y[o] = v; St.y0[o] = v;
    }
}

}  // namespace phx
