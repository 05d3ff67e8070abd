// phx_setup.h — host-side, once-per-problem setup of the batched solver:
// CSC view of the shared pattern, nonant column map and the Ruiz (x10) +
// Pock-Chambolle (alpha=1) equilibration computed from max_s |A_s| so that a
// single row/column scaling serves every scenario (scenario-invariant A
// entries stay invariant after scaling).  Shared by phx_kernels.hip and the
// test-only CPU emulation (tests/emu).
#pragma once
#include <stdint.h>
#include <math.h>
#include <string>
#include <vector>
#include <algorithm>

namespace phx {

struct HostSetup {
    std::vector<int32_t> rowptr, colidx, kvar, slot_col;
    std::vector<double> Aconst;
    std::vector<int32_t> rowof, colptr, rowidx, csc2csr, col_slot;
    std::vector<double> dr, dc, Acs, vscale;
};

// Fills everything from rowptr/colidx/kvar/Aconst/slot_col (already in hs) and
// the per-entry max |A| over scenarios (vmax for varying entries).  Returns an
// empty string on success, else an error message.
inline std::string build_setup(HostSetup& hs, int n, int m, int nnz, int N, int nvar,
                               const std::vector<double>& vmax) {
    auto& rowptr = hs.rowptr;
    auto& colidx = hs.colidx;
    auto& kvar = hs.kvar;
    if ((int)rowptr.size() != m + 1 || rowptr[0] != 0 || rowptr[m] != nnz) return "bad rowptr";
    hs.rowof.assign(nnz, 0);
    for (int i = 0; i < m; ++i) {
        if (rowptr[i] > rowptr[i + 1]) return "rowptr not monotone";
        for (int k = rowptr[i]; k < rowptr[i + 1]; ++k) hs.rowof[k] = i;
    }
    hs.colptr.assign(n + 1, 0);
    hs.rowidx.assign(nnz, 0);
    hs.csc2csr.assign(nnz, 0);
    for (int k = 0; k < nnz; ++k) {
        if (colidx[k] < 0 || colidx[k] >= n) return "colidx out of range";
        if (kvar[k] >= nvar) return "kvar out of range";
        hs.colptr[colidx[k] + 1]++;
    }
    for (int j = 0; j < n; ++j) hs.colptr[j + 1] += hs.colptr[j];
    {
        std::vector<int32_t> fill(hs.colptr.begin(), hs.colptr.end() - 1);
        for (int k = 0; k < nnz; ++k) {   // row-major walk keeps rows sorted per column
            const int j = colidx[k];
            const int p = fill[j]++;
            hs.rowidx[p] = hs.rowof[k];
            hs.csc2csr[p] = k;
        }
    }
    hs.col_slot.assign(n, -1);
    for (int j = 0; j < N; ++j) {
        const int c = hs.slot_col[j];
        if (c < 0 || c >= n) return "slot_col out of range";
        if (hs.col_slot[c] >= 0) return "duplicate nonant column";
        hs.col_slot[c] = j;
    }
    std::vector<double> amax(nnz, 0.0);
    for (int k = 0; k < nnz; ++k) amax[k] = kvar[k] < 0 ? fabs(hs.Aconst[k]) : vmax[kvar[k]];
    hs.dr.assign(m, 1.0);
    hs.dc.assign(n, 1.0);
    auto& dr = hs.dr;
    auto& dc = hs.dc;
    for (int it = 0; it < 10; ++it) {
        std::vector<double> rn(m, 0.0), cn(n, 0.0);
        for (int i = 0; i < m; ++i)
            for (int k = rowptr[i]; k < rowptr[i + 1]; ++k) {
                const double v = dr[i] * amax[k] * dc[colidx[k]];
                rn[i] = std::max(rn[i], v);
                cn[colidx[k]] = std::max(cn[colidx[k]], v);
            }
        for (int i = 0; i < m; ++i) if (rn[i] > 0) dr[i] /= sqrt(rn[i]);
        for (int j = 0; j < n; ++j) if (cn[j] > 0) dc[j] /= sqrt(cn[j]);
    }
    {
        std::vector<double> rn(m, 0.0), cn(n, 0.0);
        for (int i = 0; i < m; ++i)
            for (int k = rowptr[i]; k < rowptr[i + 1]; ++k) {
                const double v = dr[i] * amax[k] * dc[colidx[k]];
                rn[i] += v;
                cn[colidx[k]] += v;
            }
        for (int i = 0; i < m; ++i) if (rn[i] > 0) dr[i] /= sqrt(rn[i]);
        for (int j = 0; j < n; ++j) if (cn[j] > 0) dc[j] /= sqrt(cn[j]);
    }
    hs.Acs.assign(nnz, 0.0);
    hs.vscale.assign(std::max(nvar, 1), 1.0);
    for (int k = 0; k < nnz; ++k) {
        const double sc = dr[hs.rowof[k]] * dc[colidx[k]];
        hs.Acs[k] = hs.Aconst[k] * sc;
        if (kvar[k] >= 0) hs.vscale[kvar[k]] = sc;
    }
    return std::string();
}

// Deterministic tiling of segments [s0[g], s1[g]) into chunks of <= CH lanes.
inline void build_seg_tiles(const std::vector<int32_t>& s0, const std::vector<int32_t>& s1, int CH,
                            std::vector<int32_t>& ts0, std::vector<int32_t>& ts1,
                            std::vector<int32_t>& ptr) {
    ts0.clear(); ts1.clear(); ptr.assign(1, 0);
    for (size_t g = 0; g < s0.size(); ++g) {
        for (int s = s0[g]; s < s1[g]; s += CH) {
            ts0.push_back(s);
            ts1.push_back(std::min(s1[g], s + CH));
        }
        ptr.push_back((int32_t)ts0.size());
    }
}

// Schur-complement pair list of the workgroup solver (phx_wg.h WgPairs):
// every (ia >= ib) row pair sharing a column, with the CSR positions of the
// shared column in both rows, in (ia, ib) order.  Built from the CSC view.
struct WgPairsHost {
    std::vector<int32_t> ptr, ia, ib, ka, kb;
};

inline void build_wg_pairs(const HostSetup& hs, int n, int m, WgPairsHost& out) {
    std::vector<std::vector<std::pair<int32_t, int32_t>>> trip((size_t)m * m);
    for (int j = 0; j < n; ++j)
        for (int a = hs.colptr[j]; a < hs.colptr[j + 1]; ++a)
            for (int b = hs.colptr[j]; b < hs.colptr[j + 1]; ++b) {
                const int ra = hs.rowidx[a], rb = hs.rowidx[b];
                if (ra < rb) continue;
                trip[(size_t)ra * m + rb].push_back({hs.csc2csr[a], hs.csc2csr[b]});
            }
    out = WgPairsHost{};
    out.ptr.push_back(0);
    for (int ia = 0; ia < m; ++ia)
        for (int ib = 0; ib <= ia; ++ib) {
            const auto& t = trip[(size_t)ia * m + ib];
            if (t.empty()) continue;
            out.ia.push_back(ia);
            out.ib.push_back(ib);
            for (const auto& pr : t) { out.ka.push_back(pr.first); out.kb.push_back(pr.second); }
            out.ptr.push_back((int32_t)out.ka.size());
        }
}

}  // namespace phx
