// phx_setup.h — host-side, once-per-problem setup of the batched solver:
// CSC view of the shared pattern, nonant column map and the Ruiz (x10) +
// Pock-Chambolle (alpha=1) equilibration computed from max_s |A_s| so that a
// single row/column scaling serves every scenario (scenario-invariant A
// entries stay invariant after scaling).  Shared by phx_kernels.hip and the
// test-only CPU emulation (tests/emu).
#pragma once
#include <limits>
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
    int32_t nlong = 0;    // the first nlong pairs share >= WG_LONG_PAIR columns
};
constexpr int WG_LONG_PAIR = 8;

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
    // the long pairs first (a row with itself: every column of the row --
    // farmer cm=10's land row 30, sslp's facility rows 47), the rest after
    // (wg_warm gives the long ones a quad each, the others a thread)
    for (int pass = 0; pass < 2; ++pass) {
        for (int ia = 0; ia < m; ++ia)
            for (int ib = 0; ib <= ia; ++ib) {
                const auto& t = trip[(size_t)ia * m + ib];
                if (t.empty() || ((int)t.size() >= WG_LONG_PAIR) != (pass == 0)) continue;
                out.ia.push_back(ia);
                out.ib.push_back(ib);
                for (const auto& pr : t) { out.ka.push_back(pr.first); out.kb.push_back(pr.second); }
                out.ptr.push_back((int32_t)out.ka.size());
            }
        if (pass == 0) out.nlong = (int32_t)out.ia.size();
    }
}

// Symbolic structure of the sparse workgroup solver (phx_sp.h SpSym): rows
// split into B, a maximal set of rows pairwise without a shared column (greedy,
// fewest neighbouring rows first, then row index), and the separator C (the
// rest, ascending row index); the B-C links with their shared columns; the
// direct and via-B terms of every separator Schur entry.  Deterministic (all
// lists in ascending order).  Returns false with a reason when the separator
// exceeds max_c rows.
struct SpSymHost {
    int nC = 0, nlink = 0;
    std::vector<int32_t> cpos, crow, lptr, lc, lrow, lkp, lkb, lkc, clp, cll, eap, eka, ekb, ebp, el1, el2;
};

// The sparse solver's gather tables (round 5), from the symbolic structure and
// the scaled constant A (hs.Acs): per separator-Schur direct term t the product
// A[eka] A[ekb] (NaN when either entry varies by scenario) and the shared
// column; per link term the same for A[lkb] A[lkc]; A's values and variation
// indices in CSC order.  Each replaces a chain of dependent global loads
// (position -> kvar -> value, position -> column) in the factor's assembly and
// the column loops by loads that only depend on the loop index.
struct SpTablesHost {
    std::vector<double> eab, lab, Acsc;
    std::vector<int32_t> ecol, lcol, kvcsc;
};
inline void build_sp_tables(const HostSetup& hs, const SpSymHost& h, SpTablesHost& t) {
    const double nan = std::numeric_limits<double>::quiet_NaN();
    const auto prod = [&](int ka, int kb) {
        return (hs.kvar[ka] < 0 && hs.kvar[kb] < 0) ? hs.Acs[ka] * hs.Acs[kb] : nan;
    };
    t = SpTablesHost{};
    for (size_t q = 0; q < h.eka.size(); ++q) {
        t.eab.push_back(prod(h.eka[q], h.ekb[q]));
        t.ecol.push_back(hs.colidx[h.eka[q]]);
    }
    for (size_t q = 0; q < h.lkb.size(); ++q) {
        t.lab.push_back(prod(h.lkb[q], h.lkc[q]));
        t.lcol.push_back(hs.colidx[h.lkb[q]]);
    }
    for (size_t k = 0; k < hs.csc2csr.size(); ++k) {
        t.Acsc.push_back(hs.Acs[hs.csc2csr[k]]);
        t.kvcsc.push_back(hs.kvar[hs.csc2csr[k]]);
    }
    // (non-empty, so that their data pointers are valid)
    if (t.eab.empty()) { t.eab.push_back(0.0); t.ecol.push_back(0); }
    if (t.lab.empty()) { t.lab.push_back(0.0); t.lcol.push_back(0); }
    if (t.Acsc.empty()) { t.Acsc.push_back(0.0); t.kvcsc.push_back(-1); }
}

inline bool build_sp_sym(const HostSetup& hs, int n, int m, int max_c, SpSymHost& out, std::string& why) {
    out = SpSymHost{};
    std::vector<std::vector<int32_t>> adj(m);
    for (int j = 0; j < n; ++j)
        for (int a = hs.colptr[j]; a < hs.colptr[j + 1]; ++a)
            for (int b = hs.colptr[j]; b < hs.colptr[j + 1]; ++b)
                if (hs.rowidx[a] != hs.rowidx[b]) adj[hs.rowidx[a]].push_back(hs.rowidx[b]);
    for (auto& v : adj) {
        std::sort(v.begin(), v.end());
        v.erase(std::unique(v.begin(), v.end()), v.end());
    }
    std::vector<int32_t> order(m);
    for (int i = 0; i < m; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return adj[a].size() < adj[b].size(); });
    std::vector<char> inB(m, 0), blocked(m, 0);
    for (int r : order) {
        if (blocked[r]) continue;
        inB[r] = 1;
        for (int q : adj[r]) blocked[q] = 1;
    }
    out.cpos.assign(m, -1);
    for (int i = 0; i < m; ++i)
        if (!inB[i]) {
            out.cpos[i] = (int32_t)out.crow.size();
            out.crow.push_back(i);
        }
    out.nC = (int)out.crow.size();
    if (out.nC > max_c) {
        why = "separator of " + std::to_string(out.nC) + " rows > " + std::to_string(max_c);
        return false;
    }
    const int nC = out.nC;
    // links of each B row, ascending separator position; shared columns ascending
    out.lptr.assign(1, 0);
    out.lkp.assign(1, 0);
    for (int b = 0; b < m; ++b) {
        if (inB[b]) {
            std::vector<std::vector<std::pair<int32_t, int32_t>>> lk(nC);
            for (int kb = hs.rowptr[b]; kb < hs.rowptr[b + 1]; ++kb) {
                const int j = hs.colidx[kb];
                for (int q = hs.colptr[j]; q < hs.colptr[j + 1]; ++q) {
                    const int r = hs.rowidx[q];
                    if (r != b && out.cpos[r] >= 0) lk[out.cpos[r]].push_back({kb, hs.csc2csr[q]});
                }
            }
            for (int c = 0; c < nC; ++c) {
                if (lk[c].empty()) continue;
                out.lc.push_back(c);
                out.lrow.push_back(b);
                for (const auto& pr : lk[c]) { out.lkb.push_back(pr.first); out.lkc.push_back(pr.second); }
                out.lkp.push_back((int32_t)out.lkb.size());
            }
        }
        out.lptr.push_back((int32_t)out.lc.size());
    }
    out.nlink = (int)out.lc.size();
    out.clp.assign(nC + 1, 0);
    for (int l = 0; l < out.nlink; ++l) out.clp[out.lc[l] + 1]++;
    for (int c = 0; c < nC; ++c) out.clp[c + 1] += out.clp[c];
    out.cll.assign(out.nlink, 0);
    {
        std::vector<int32_t> fill(out.clp.begin(), out.clp.end() - 1);
        for (int l = 0; l < out.nlink; ++l) out.cll[fill[out.lc[l]]++] = l;
    }
    // separator Schur entries (c1 >= c2) at c1*nC + c2
    std::vector<std::vector<std::pair<int32_t, int32_t>>> dir((size_t)nC * nC), via((size_t)nC * nC);
    for (int j = 0; j < n; ++j)
        for (int a = hs.colptr[j]; a < hs.colptr[j + 1]; ++a)
            for (int b = hs.colptr[j]; b < hs.colptr[j + 1]; ++b) {
                const int ca = out.cpos[hs.rowidx[a]], cb = out.cpos[hs.rowidx[b]];
                if (ca < 0 || cb < 0 || ca < cb) continue;
                dir[(size_t)ca * nC + cb].push_back({hs.csc2csr[a], hs.csc2csr[b]});
            }
    for (int b = 0; b < m; ++b)
        for (int l1 = out.lptr[b]; l1 < out.lptr[b + 1]; ++l1)
            for (int l2 = out.lptr[b]; l2 < out.lptr[b + 1]; ++l2)
                if (out.lc[l1] >= out.lc[l2]) via[(size_t)out.lc[l1] * nC + out.lc[l2]].push_back({l1, l2});
    out.eap.assign(1, 0);
    out.ebp.assign(1, 0);
    for (size_t p = 0; p < (size_t)nC * nC; ++p) {
        for (const auto& pr : dir[p]) { out.eka.push_back(pr.first); out.ekb.push_back(pr.second); }
        out.eap.push_back((int32_t)out.eka.size());
        for (const auto& pr : via[p]) { out.el1.push_back(pr.first); out.el2.push_back(pr.second); }
        out.ebp.push_back((int32_t)out.el1.size());
    }
    return true;
}

}  // namespace phx
