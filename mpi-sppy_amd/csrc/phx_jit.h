// phx_jit.h — structure of a small subproblem and the source of its
// specialised lane-solver kernel (host side; compiled by hipRTC in
// phx_kernels.hip, instantiated with a runtime pattern by tests/emu).
//
// The kernels are specialised on the STRUCTURE (sparsity pattern, column
// pairs of A D A', nonant column map, which bounds / row sides are finite,
// which columns are fixed, which rows are equalities) and on the numbers that
// are the same for every scenario of the batch (scaled constant A entries,
// costs, bounds, scaling), baked in as exact hex-float literals.  Scenario-
// varying numbers (varying A entries, PH terms, varying costs/bounds/rhs) stay
// run-time inputs.  Compiled once per phx_set_problem (cached by source text).
#pragma once
#include <stdint.h>
#include <math.h>
#include <stdio.h>
#include <algorithm>
#include <sstream>
#include <string>
#include <vector>
#include "phx_setup.h"

namespace phx {

struct LaneStructure {
    int n = 0, m = 0, nnz = 0, npairs = 0, nvar = 0, nslot = 0;
    bool c_vary = false, bnd_vary = false, rhs_vary = false;
    // false (default): the lane solver works on the UNSCALED problem — exact
    // KKT solves need no equilibration, and the +-1 / 0 entries of A, the
    // bounds and the costs then fold into adds and moves instead of literal
    // multiplies; dc/dr (the generic path's scaling) are kept only to hand a
    // lane over to the scaled PDHG path.
    bool scaled = false;
    std::vector<int32_t> row, col, kvar, col_slot;
    std::vector<int32_t> pair_a, pair_b, pair_pos;
    std::vector<uint8_t> lnz;   // packed lower triangle: structurally nonzero in L (pairs + fill)
    // entry k is the first of its row / of its column in CSR order; rows /
    // columns without entries (the mat-vecs start from the first product
    // instead of adding it to 0.0, which IEEE arithmetic keeps as an add)
    std::vector<uint8_t> rfirst, cfirst, rempty, cempty;
    std::vector<uint8_t> lfin, ufin, fixed, blfin, bufin, eq;
    // scenario-invariant numbers (scaled iff `scaled`), baked into the kernel
    // as literals (c / lb,ub / bl,bu only when they do not vary across
    // scenarios); dc, dr: the generic path's column/row scaling
    std::vector<double> Ac, dc, dr, c, lb, ub, bl, bu;
    // the interior point's start scales (lane_scales): primal offsets from the
    // bounds / row sides, bound and row multipliers
    double ipm_xs = 1.0, ipm_zs = 1.0, ipm_ws = 1.0;
    // bounded multi-change active-set updates (phx_lane.h multi_violations):
    // theta (0: off) for the first multi_rounds rounds after single_after
    double multi_theta = 0.0;
    int multi_rounds = 0;
};

// median of the nonzero finite magnitudes (0 if none)
inline double median_mag(std::vector<double> v) {
    std::vector<double> a;
    for (double x : v)
        if (std::isfinite(x) && x != 0.0) a.push_back(std::fabs(x));
    if (a.empty()) return 0.0;
    std::sort(a.begin(), a.end());
    const size_t h = a.size() / 2;
    return a.size() % 2 ? a[h] : 0.5 * (a[h - 1] + a[h]);
}

// Attach the scaled invariant numbers (host copies of the device arrays).
inline void set_lane_values(LaneStructure& L, const std::vector<double>& Ac, const std::vector<double>& dc,
                            const std::vector<double>& dr, const std::vector<double>& c,
                            const std::vector<double>& lb, const std::vector<double>& ub,
                            const std::vector<double>& bl, const std::vector<double>& bu) {
    L.Ac = Ac; L.dc = dc; L.dr = dr;
    // the multipliers' start scale from the costs (half their median
    // magnitude; with scenario-varying costs the first scenario's)
    {
        std::vector<double> cc(c.begin(), c.begin() + std::min(c.size(), (size_t)L.n));
        const double mc = median_mag(cc);
        L.ipm_ws = mc > 0.0 ? std::min(std::max(0.5 * mc, 1e-3), 1e4) : 1.0;
        L.ipm_zs = 0.1 * L.ipm_ws;
    }
    L.c = L.c_vary ? std::vector<double>() : c;
    L.lb = L.bnd_vary ? std::vector<double>() : lb;
    L.ub = L.bnd_vary ? std::vector<double>() : ub;
    L.bl = L.rhs_vary ? std::vector<double>() : bl;
    L.bu = L.rhs_vary ? std::vector<double>() : bu;
}

// The caller's lane-solver tuning (phx_problem_desc lane_multi_*): a theta
// outside (0, 1] or not finite is off; rounds 0 means 4
inline void set_lane_tuning(LaneStructure& L, double multi_theta, int multi_rounds) {
    const bool on = std::isfinite(multi_theta) && multi_theta > 0.0 && multi_theta <= 1.0;
    L.multi_theta = on ? multi_theta : 0.0;
    L.multi_rounds = on ? (multi_rounds > 0 ? std::min(multi_rounds, 64) : 4) : 0;
}

// Limits for the register-resident kernel (beyond them: generic kernels).
constexpr int LANE_MAX_N = 64;
constexpr int LANE_MAX_M = 24;
constexpr int LANE_MAX_NNZ = 384;

// lb/ub/bl/bu: scenario-major host copies of the UNSCALED bounds of every
// scenario (S rows; S = 1 if invariant).  Returns false (with reason) if the
// structure is not uniform across scenarios or too large.
inline bool build_lane_structure(const HostSetup& hs, int n, int m, int nnz, bool c_vary, bool bnd_vary,
                                 bool rhs_vary, const std::vector<double>& lb, const std::vector<double>& ub,
                                 const std::vector<double>& bl, const std::vector<double>& bu, int Sb, int Sr,
                                 LaneStructure& L, std::string& why) {
    if (n > LANE_MAX_N || m > LANE_MAX_M || nnz > LANE_MAX_NNZ || m < 1 || nnz < 1) {
        why = "size";
        return false;
    }
    L.n = n; L.m = m; L.nnz = nnz;
    L.c_vary = c_vary; L.bnd_vary = bnd_vary; L.rhs_vary = rhs_vary;
    L.row.assign(hs.rowof.begin(), hs.rowof.end());
    L.col.assign(hs.colidx.begin(), hs.colidx.end());
    L.kvar.assign(hs.kvar.begin(), hs.kvar.end());
    L.col_slot.assign(hs.col_slot.begin(), hs.col_slot.end());
    L.nvar = 0;
    for (int k = 0; k < nnz; ++k) L.nvar = std::max(L.nvar, hs.kvar[k] + 1);
    L.rfirst.assign(nnz, 0); L.cfirst.assign(nnz, 0); L.rempty.assign(m, 1); L.cempty.assign(n, 1);
    for (int k = 0; k < nnz; ++k) {
        const int i = hs.rowof[k], j = hs.colidx[k];
        if (L.rempty[i]) { L.rfirst[k] = 1; L.rempty[i] = 0; }
        if (L.cempty[j]) { L.cfirst[k] = 1; L.cempty[j] = 0; }
    }
    L.nslot = (int)hs.slot_col.size();
    L.pair_a.clear(); L.pair_b.clear(); L.pair_pos.clear();
    for (int j = 0; j < n; ++j)
        for (int a = hs.colptr[j]; a < hs.colptr[j + 1]; ++a)
            for (int b = hs.colptr[j]; b <= a; ++b) {
                const int ka = hs.csc2csr[a], kb = hs.csc2csr[b];
                const int ia = hs.rowof[ka], ib = hs.rowof[kb];
                const int hi = ia > ib ? ia : ib, lo = ia > ib ? ib : ia;
                L.pair_a.push_back(ka);
                L.pair_b.push_back(kb);
                L.pair_pos.push_back(hi * (hi + 1) / 2 + lo);
            }
    L.npairs = (int)L.pair_a.size();
    // symbolic Cholesky of the normal-matrix pattern (diagonal + pair positions)
    L.lnz.assign((size_t)m * (m + 1) / 2, 0);
    for (int i = 0; i < m; ++i) L.lnz[(size_t)i * (i + 1) / 2 + i] = 1;
    for (int p : L.pair_pos) L.lnz[p] = 1;
    for (int jj = 0; jj < m; ++jj)
        for (int i = jj + 1; i < m; ++i)
            for (int k = 0; k < jj; ++k)
                if (L.lnz[(size_t)i * (i + 1) / 2 + k] && L.lnz[(size_t)jj * (jj + 1) / 2 + k])
                    L.lnz[(size_t)i * (i + 1) / 2 + jj] = 1;
    auto uni = [&](const std::vector<double>& a, int S, int len, int j, auto pred) -> int {
        const int v = pred(a[j]) ? 1 : 0;
        for (int s = 1; s < S; ++s)
            if ((pred(a[(size_t)s * len + j]) ? 1 : 0) != v) return -1;
        return v;
    };
    L.lfin.assign(n, 0); L.ufin.assign(n, 0); L.fixed.assign(n, 0);
    for (int j = 0; j < n; ++j) {
        const int lf = uni(lb, Sb, n, j, [](double v) { return std::isfinite(v); });
        const int uf = uni(ub, Sb, n, j, [](double v) { return std::isfinite(v); });
        if (lf < 0 || uf < 0) { why = "bound finiteness varies across scenarios"; return false; }
        L.lfin[j] = (uint8_t)lf; L.ufin[j] = (uint8_t)uf;
        int fx = lb[j] == ub[j];
        for (int s = 1; s < Sb; ++s)
            if ((lb[(size_t)s * n + j] == ub[(size_t)s * n + j]) != (bool)fx) { why = "fixing varies"; return false; }
        L.fixed[j] = (uint8_t)fx;
    }
    L.blfin.assign(m, 0); L.bufin.assign(m, 0); L.eq.assign(m, 0);
    for (int i = 0; i < m; ++i) {
        const int lf = uni(bl, Sr, m, i, [](double v) { return std::isfinite(v); });
        const int uf = uni(bu, Sr, m, i, [](double v) { return std::isfinite(v); });
        if (lf < 0 || uf < 0) { why = "row finiteness varies across scenarios"; return false; }
        L.blfin[i] = (uint8_t)lf; L.bufin[i] = (uint8_t)uf;
        int e = bl[i] == bu[i];
        for (int s = 1; s < Sr; ++s)
            if ((bl[(size_t)s * m + i] == bu[(size_t)s * m + i]) != (bool)e) { why = "equality varies"; return false; }
        L.eq[i] = (uint8_t)e;
    }
    // the primal start scale: a fifth of the median magnitude of the first
    // scenario's finite bounds and row sides (interior-point iterations on the
    // emulation, Iter0, wave-max mean: farmer 16.3 -> ~11, aircond 11.7 -> ~10;
    // scripts/emu_ipm.py)
    {
        std::vector<double> v;
        for (int j = 0; j < n; ++j) { v.push_back(lb[j]); v.push_back(ub[j]); }
        for (int i = 0; i < m; ++i) { v.push_back(bl[i]); v.push_back(bu[i]); }
        const double mp = median_mag(v);
        L.ipm_xs = mp > 0.0 ? std::min(std::max(0.2 * mp, 1.0), 1e4) : 1.0;
    }
    return true;
}

template <class T>
inline void emit_table(std::ostringstream& o, const char* ret, const char* name, const std::vector<T>& v) {
    o << "  __host__ __device__ static constexpr " << ret << " " << name << "(int k) { constexpr " << ret
      << " a[] = {";
    for (size_t i = 0; i < v.size(); ++i) o << (i ? "," : "") << (long long)v[i];
    if (v.empty()) o << "0";
    o << "}; return a[k]; }\n";
}

// exact hex-float literal table (non-finite entries are never read: emitted as 0)
inline void emit_dtable(std::ostringstream& o, const char* name, const std::vector<double>& v) {
    o << "  __host__ __device__ static constexpr double " << name << "(int k) { constexpr double a[] = {";
    char buf[64];
    for (size_t i = 0; i < v.size(); ++i) {
        snprintf(buf, sizeof(buf), "%a", std::isfinite(v[i]) ? v[i] : 0.0);
        o << (i ? "," : "") << buf;
    }
    if (v.empty()) o << "0.0";
    o << "}; return a[k]; }\n";
}

// HIP source of the specialised kernels `phx_lane_ipm` / `phx_lane_polish`
// (hipRTC input).
// with_map: the warm kernels carry the affine-map paths (PHX_LANE_MAP=1);
// without, that code is compiled out (fewer registers, no spills).
inline std::string lane_kernel_source(const LaneStructure& L, int warm_waves = 1, bool with_map = false,
                                      int cold_waves = 1) {
    const std::string wl = with_map ? "phx_lane::warm_lane<PT, true>" : "phx_lane::warm_lane<PT, false>";
    std::ostringstream o;
    o << "#include \"phx_lane.h\"\n";
    o << "struct PT {\n";
    o << "  static constexpr int NMAX_N = " << L.n << ", NMAX_M = " << L.m << ", NMAX_K = " << L.nnz
      << ", NMAX_V = " << std::max(L.nvar, 1) << ", NMAX_S = " << std::max(L.nslot, 1) << ";\n";
    o << "  __host__ __device__ static constexpr int nvar() { return " << L.nvar << "; }\n";
    o << "  __host__ __device__ static constexpr bool scaled() { return " << (L.scaled ? "true" : "false") << "; }\n";
    o << "  __host__ __device__ static constexpr int nslot() { return " << L.nslot << "; }\n";
    o << "  __host__ __device__ static constexpr int n() { return " << L.n << "; }\n";
    o << "  __host__ __device__ static constexpr int m() { return " << L.m << "; }\n";
    o << "  __host__ __device__ static constexpr int nnz() { return " << L.nnz << "; }\n";
    o << "  __host__ __device__ static constexpr int npairs() { return " << L.npairs << "; }\n";
    o << "  __host__ __device__ static constexpr bool c_vary() { return " << (L.c_vary ? "true" : "false") << "; }\n";
    o << "  __host__ __device__ static constexpr bool bnd_vary() { return " << (L.bnd_vary ? "true" : "false")
      << "; }\n";
    o << "  __host__ __device__ static constexpr bool rhs_vary() { return " << (L.rhs_vary ? "true" : "false")
      << "; }\n";
    {
        char buf[512];
        snprintf(buf, sizeof(buf), "  __host__ __device__ static constexpr double ipm_xs() { return %a; }\n", L.ipm_xs);
        o << buf;
        snprintf(buf, sizeof(buf), "  __host__ __device__ static constexpr double ipm_zs() { return %a; }\n", L.ipm_zs);
        o << buf;
        snprintf(buf, sizeof(buf), "  __host__ __device__ static constexpr double ipm_ws() { return %a; }\n", L.ipm_ws);
        o << buf;
        // the bounded multi-change update (phx_lane.h multi_violations); a
        // PHX_MULTI_THETA / PHX_MULTI_ROUNDS define (PHX_LANE_DEFS) overrides
        snprintf(buf, sizeof(buf),
                 "#ifdef PHX_MULTI_THETA\n  __host__ __device__ static constexpr double multi_theta() { return "
                 "PHX_MULTI_THETA; }\n#else\n  __host__ __device__ static constexpr double multi_theta() { return %a; "
                 "}\n#endif\n",
                 L.multi_theta);
        o << buf;
        snprintf(buf, sizeof(buf),
                 "#ifdef PHX_MULTI_ROUNDS\n  __host__ __device__ static constexpr int multi_rounds() { return "
                 "PHX_MULTI_ROUNDS; }\n#else\n  __host__ __device__ static constexpr int multi_rounds() { return %d; "
                 "}\n#endif\n",
                 L.multi_rounds);
        o << buf;
    }
    emit_table(o, "int", "row", L.row);
    emit_table(o, "int", "col", L.col);
    emit_table(o, "int", "kvar", L.kvar);
    emit_table(o, "int", "col_slot", L.col_slot);
    emit_table(o, "int", "pair_a", L.pair_a);
    emit_table(o, "int", "pair_b", L.pair_b);
    emit_table(o, "int", "pair_pos", L.pair_pos);
    emit_table(o, "bool", "lnz", L.lnz);
    emit_table(o, "bool", "rfirst", L.rfirst);
    emit_table(o, "bool", "cfirst", L.cfirst);
    emit_table(o, "bool", "rempty", L.rempty);
    emit_table(o, "bool", "cempty", L.cempty);
    emit_table(o, "bool", "lfin", L.lfin);
    emit_table(o, "bool", "ufin", L.ufin);
    emit_table(o, "bool", "fixed", L.fixed);
    emit_table(o, "bool", "blfin", L.blfin);
    emit_table(o, "bool", "bufin", L.bufin);
    emit_table(o, "bool", "eq", L.eq);
    emit_dtable(o, "Ac", L.Ac);
    emit_dtable(o, "dcs", L.dc);
    emit_dtable(o, "drs", L.dr);
    {
        std::vector<double> idc(L.dc.size()), idr(L.dr.size());
        for (size_t j = 0; j < idc.size(); ++j) idc[j] = 1.0 / L.dc[j];
        for (size_t i = 0; i < idr.size(); ++i) idr[i] = 1.0 / L.dr[i];
        emit_dtable(o, "idcs", idc);
        emit_dtable(o, "idrs", idr);
    }
    emit_dtable(o, "cs", L.c);
    emit_dtable(o, "lbs", L.lb);
    emit_dtable(o, "ubs", L.ub);
    emit_dtable(o, "bls", L.bl);
    emit_dtable(o, "bus", L.bu);
    o << "};\n";
    // phx_lane_warm: one active-set round over every lane (the per-iteration
    // pass); phx_lane_warm_list: one more round over a compacted lane list
    // (the few lanes whose active set changed), so no wavefront idles while
    // one of its lanes needs a second round.
    o << "extern \"C\" __global__ void __launch_bounds__(64, " << warm_waves
      << ") phx_lane_warm(phx_lane::LaneIO io) {\n"
         "  phx_lane::lane_stamp(io, 0);\n"
         "  if (phx_lane::gated(io.gate)) return;\n"
         "  if (io.fz.on && !phx_lane::fz_prologue(io)) return;\n"
         "  phx_lane::zero_next_counts(io.counts_next);\n"
         "  phx_lane::lane_stamp(io, 1);\n"
         "  const int t = blockIdx.x * 64 + threadIdx.x;\n"
         "  bool still = false;\n"
         "  if (t < io.S) {\n"
         "    if (io.fz.on) (void)phx_lane::fz_update_w<PT>(io, t);\n"
         "    phx_lane::lane_stamp(io, 2);\n"
         "    still = " + wl + "(io, t);\n"
         "  }\n"
         "  phx_lane::lane_stamp(io, 3);\n"
         "  phx_lane::compact_lane(still, t, io.lanes_out, io.count_out);\n"
         "  phx_lane::lane_stamp(io, 4);\n"
         "  if (io.fz.on) phx_lane::fz_epilogue<PT>(io, t, still);\n"
         "  phx_lane::lane_stamp(io, 5);\n"
         "}\n";
    // phx_iterk fused mode: one whole PH iteration per launch, every load of
    // the lane's Update_W and first round issued at entry (phx_lane.h warm_fused)
    o << "extern \"C\" __global__ void __launch_bounds__(64, " << warm_waves
      << ") phx_lane_warm_fz(phx_lane::LaneIO io) {\n"
         "  phx_lane::warm_fused<PT>(io);\n"
         "}\n";
    // ... for batches of at most one wavefront per SIMD: the whole register
    // file (VGPRs + AGPRs) for one wave, no scratch spills
    o << "extern \"C\" __global__ void __launch_bounds__(64, 1) phx_lane_warm_fz1(phx_lane::LaneIO io) {\n"
         "#ifdef PHX_FZ1_RELOAD\n"
         "  phx_lane::warm_fused<PT, false>(io);\n"
         "#else\n"
         "  phx_lane::warm_fused<PT, true>(io);\n"
         "#endif\n"
         "}\n";
    // ... two waves per SIMD with every round on register data (above one
    // wavefront per SIMD; the compiler spills what does not fit 256 registers)
    o << "extern \"C\" __global__ void __launch_bounds__(64, 2) phx_lane_warm_fzr2(phx_lane::LaneIO io) {\n"
         "  phx_lane::warm_fused<PT, true, PHX_FZR2_CARRY_DEF, PHX_FZR2_PARK_DEF>(io);\n"
         "}\n";
    // ... compacting: round 0 per lane, the later rounds of the lanes that need
    // them packed into full wavefronts by each group's last block (phx_lane.h
    // warm_fused_c)
    o << "extern \"C\" __global__ void __launch_bounds__(64, 1) phx_lane_warm_fzc(phx_lane::LaneIO io) {\n"
         "  phx_lane::warm_fused_c<PT>(io);\n"
         "}\n";
    // a whole warm solve (warm rounds, rescue rounds, interior point) in one
    // launch, for batches of at most one wavefront per SIMD (phx_lane.h all_lane)
    o << "extern \"C\" __global__ void __launch_bounds__(64, 1) phx_lane_all(phx_lane::LaneIO io, int rescue) {\n"
         "  if (phx_lane::gated(io.gate)) return;\n"
         "  phx_lane::zero_next_counts(io.counts_next);\n"
         "  const int t = blockIdx.x * 64 + threadIdx.x;\n"
         "  bool still = false;\n"
         "  if (t < io.S) still = phx_lane::all_lane<PT>(io, t, rescue);\n"
         "  phx_lane::compact_lane(still, t, io.lanes_out, io.count_out);\n"
         "}\n";
    // ... its build that re-loads the lane's data per round (the host uses it
    // when phx_lane_all spills to scratch)
    o << "extern \"C\" __global__ void __launch_bounds__(64, 1) phx_lane_all_rl(phx_lane::LaneIO io, int rescue) {\n"
         "  if (phx_lane::gated(io.gate)) return;\n"
         "  phx_lane::zero_next_counts(io.counts_next);\n"
         "  const int t = blockIdx.x * 64 + threadIdx.x;\n"
         "  bool still = false;\n"
         "  if (t < io.S) still = phx_lane::all_lane<PT, false>(io, t, rescue);\n"
         "  phx_lane::compact_lane(still, t, io.lanes_out, io.count_out);\n"
         "}\n";
    // ... and its build with the warm and rescue rounds' data parked in LDS
    // (as_rounds_pk; the host's default over _rl, PHX_ALL_BUILD=reload keeps _rl)
    o << "extern \"C\" __global__ void __launch_bounds__(64, 1) phx_lane_all_pk(phx_lane::LaneIO io, int rescue) {\n"
         "  __shared__ double pk[phx_lane::Data<PT>::PARK * 64];\n"
         "  if (phx_lane::gated(io.gate)) return;\n"
         "  phx_lane::zero_next_counts(io.counts_next);\n"
         "  const int t = blockIdx.x * 64 + threadIdx.x;\n"
         "  bool still = false;\n"
         "  if (t < io.S) still = phx_lane::all_lane<PT, false, true>(io, t, rescue, pk);\n"
         "  phx_lane::compact_lane(still, t, io.lanes_out, io.count_out);\n"
         "}\n";
    // phx_iterk fused mode, after the last enqueued iteration: the decision on
    // its conv (the next warm launch's prologue does it otherwise)
    // (and the copies the host reads after the drain, whether or not the loop
    // stopped earlier: as the copy dispatches they replace)
    o << "extern \"C\" __global__ void __launch_bounds__(64) phx_fz_tail(phx_lane::LaneIO io, phx_lane::TailCopy tc) {\n"
         "  phx_lane::tail_copy(tc);\n"
         "  if (phx_lane::gated(io.gate)) return;\n"
         "  (void)phx_lane::fz_decide(io.fz, io.fz.iter);\n"
         "}\n";
    o << "extern \"C\" __global__ void __launch_bounds__(64, 4) phx_lane_map(phx_lane::LaneIO io) {\n"
         "  if (phx_lane::gated(io.gate)) return;\n"
         "  phx_lane::zero_next_counts(io.counts_next);\n"
         "  const int t = blockIdx.x * 64 + threadIdx.x;\n"
         "  bool still = false;\n"
         "  if (t < io.S) still = phx_lane::map_lane<PT>(io, t);\n"
         "  phx_lane::compact_lane(still, t, io.lanes_out, io.count_out);\n"
         "}\n";
    // (the rescue list: a few per cent of the lanes, at most about one
    // wavefront per SIMD -- the whole register file and every round on the
    // data loaded at entry; PHX_LIST_RELOAD: the warm pass's build)
    const std::string wlr = with_map ? "phx_lane::warm_lane<PT, true, true>" : "phx_lane::warm_lane<PT, false, true>";
    o << "#ifdef PHX_LIST_RELOAD\n#define PHX_LIST_WAVES " << warm_waves << "\n#define PHX_LIST_FN " << wl
      << "\n#else\n#define PHX_LIST_WAVES 1\n#define PHX_LIST_FN " << wlr << "\n#endif\n";
    o << "extern \"C\" __global__ void __launch_bounds__(64, PHX_LIST_WAVES"
      << ") phx_lane_warm_list(phx_lane::LaneIO io, const int* lanes, const int* count) {\n"
         "  if (phx_lane::gated(io.gate)) return;\n"
         "  const int nl = *count;\n"
         "  for (int base = blockIdx.x * 64; base < nl; base += gridDim.x * 64) {\n"
         "    const int t = base + threadIdx.x;\n"
         "    bool still = false;\n"
         "    int sc = -1;\n"
         "    if (t < nl) { sc = lanes[t]; still = PHX_LIST_FN(io, sc); }\n"
         "    phx_lane::compact_lane(still, sc, io.lanes_out, io.count_out);\n"
         "  }\n"
         "}\n";
    // the rescue list and the interior point of what it leaves, in one launch
    // (phx_lane_warm_list, then phx_lane_cold + phx_lane_cold_as over its
    // leftovers: the same per-lane functions and options, in that order)
    o << "extern \"C\" __global__ void __launch_bounds__(64, 1) phx_lane_list_all(phx_lane::LaneIO io, "
         "const int* lanes, const int* count, int as_cold) {\n"
         "  if (phx_lane::gated(io.gate)) return;\n"
         "  const int nl = *count;\n"
         "  for (int base = blockIdx.x * 64; base < nl; base += gridDim.x * 64) {\n"
         "    const int t = base + threadIdx.x;\n"
         "    bool still = false;\n"
         "    int sc = -1;\n"
         "    if (t < nl) { sc = lanes[t]; still = " + wlr + "(io, sc); }\n"
         "    if (still) {\n"
         "      phx_lane::LaneIO io3 = io;\n"
         "      io3.as_rounds = as_cold;\n"
         "      phx_lane::ipm_lane<PT>(io3, sc);\n"
         "      still = phx_lane::cold_rounds_lane<PT>(io3, sc);\n"
         "    }\n"
         "    phx_lane::compact_lane(still, sc, io.lanes_out, io.count_out);\n"
         "  }\n"
         "}\n";
    // Iter0 seeding: every lane takes the active set of its nearest certified
    // template (phx_lane.h seed_block: the template table staged in LDS)
    o << "extern \"C\" __global__ void __launch_bounds__(64) phx_lane_seed(phx_lane::LaneIO io, "
         "const int* tl, int T, const unsigned* tmpl) {\n"
         "  phx_lane::seed_block<PT>(io, tl, T, tmpl);\n"
         "}\n";
    // the cold solve: the interior point (phx_lane_cold), then over the same
    // lanes the classification + active-set rounds (phx_lane_cold_as), which
    // compacts what still needs the generic path (phx_lane.h ipm_lane)
    o << "extern \"C\" __global__ void __launch_bounds__(64, " << cold_waves << ") phx_lane_cold(phx_lane::LaneIO io, "
         "const int* lanes, const int* count) {\n"
         "  if (phx_lane::gated(io.gate)) return;\n"
         "  const int nl = count ? *count : io.S;\n"
         "  for (int base = blockIdx.x * 64; base < nl; base += gridDim.x * 64) {\n"
         "    const int t = base + threadIdx.x;\n"
         "    if (t < nl) phx_lane::ipm_lane<PT>(io, lanes ? lanes[t] : t);\n"
         "  }\n"
         "}\n";
    o << "extern \"C\" __global__ void __launch_bounds__(64) phx_lane_cold_as(phx_lane::LaneIO io, "
         "const int* lanes, const int* count) {\n"
         "  if (phx_lane::gated(io.gate)) return;\n"
         "  phx_lane::zero_next_counts(io.counts_next);\n"
         "  const int nl = count ? *count : io.S;\n"
         "  for (int base = blockIdx.x * 64; base < nl; base += gridDim.x * 64) {\n"
         "    const int t = base + threadIdx.x;\n"
         "    bool still = false;\n"
         "    int sc = -1;\n"
         "    if (t < nl) { sc = lanes ? lanes[t] : t; still = phx_lane::cold_rounds_lane<PT>(io, sc); }\n"
         "    phx_lane::compact_lane(still, sc, io.lanes_out, io.count_out);\n"
         "  }\n"
         "}\n";
    return o.str();
}

}  // namespace phx
