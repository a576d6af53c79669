// sparse_plan.h -- host-side block-sparse elimination plan of the GN solve (gn_sparse.hip runs
// it): rounds of independent low-degree poses, then a dense core (chol_df.hip / gn_solve.hip).
// Built once per GN call from the pose graph (fixed across the call's iterations), on every rank.
// Host-only code, kept apart from gn_driver.hip so that it builds and is timed without a GPU
// (tools/plan_bench.cpp).  Replaces the reference's per-iteration SparseBlock assembly +
// SimplicialLLT analysis (gn_kernels.cu:57-159) with a plan the device solve replays.
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <utility>
#include <vector>

#include "gn_kernels.h"  // kSpRec, kSpInline, kTailMax, kCholTile, kSolveWStage, kSolveRoundPoses

namespace m3s {

inline size_t sp_align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

struct SpRound {
    int node_begin, nnodes, tbeg, nbt, rbeg, nrt, wbeg, wcount;
};

struct SparsePlan {
    bool enabled = false;
    bool fused = false;       // the whole solve in one gn_solve launch (else multi-launch)
    bool fused_tail = false;  // the dense tail fits the in-register factorisation of gn_solve
    bool hybrid = false;      // multi-launch rounds, then gn_solve's core + back-substitution
    bool core_df = true;      // hybrid: the core by chol_df (else in registers); the planner's choice
    // PCG iterations (gn_pcg.hip; set by the driver): M's rows per workgroup, workgroups, X's
    // leading dimension, the vector stride; device: X (n x ldx f64) and the exchange granules
    bool pcg = false, pcg_onex = false;
    int pcg_from = 0, pcg_lag = 0;  // first PCG iteration; M from iteration pcg_from - pcg_lag
    int pcg_R = 0, pcg_nwg = 0, pcg_ldx = 0, pcg_ldt = 0, pcg_nv = 0, pcg_nitem = 0;
    size_t o_pcgx = 0, o_pcgxt = 0, o_gran = 0;
    // the factor the first inverse reads, copied out of the live one (Lstore .. Linv) when M comes
    // from an earlier iteration than the one before the first PCG (gn_driver.hip pcg_lag)
    size_t o_snap = 0, snap_bytes = 0;
    size_t o_dfcnt = 0;  // the ticketed all-rounds launch's counters (sp_rounds_df_words ints)
    int nblocks = 0, nW = 0, ntail = 0, npad_tail = 0, zero_blk = 0;
    std::vector<SpRound> rounds;
    std::vector<int> nodes, fptr, fronts, tg, tc, rtg, rc, tail, tmap;
    // multi-launch rounds (sp_round_kernel), per contribution past a record's kSpInline inline
    // ones: (v, code_r, code_s) for block targets, (v, code_r, W id, owner node | -1) for RHS
    // targets; code = block * 2 + transposed.  (tg / tc / rtg / rc: the single-workgroup solve's)
    std::vector<int> tc3, rc4;
    // multi-launch rounds: one kSpRec record per target (gn_kernels.h), the first ninl ints of
    // inl.  The buffer is not cleared between plans: a record's inline slots past its
    // contribution count are never read by the kernel, so they are left as they are (most
    // targets have 1-2 of 9; writing the whole 160-B records was most of a cfg4 plan's time)
    std::vector<int> inl;
    size_t ninl = 0;
    // the PCG's matrix-vector product (gn_pcg.hip): per pose its blocks, the diagonal first, as
    // (block, other pose) pairs; built by the driver when the call runs PCG iterations
    std::vector<int> apt, adj;
    // device (one stream-ordered allocation per call)
    char* dbuf = nullptr;
    size_t o_dense = 0, o_linv = 0;  // the dense core (npad_tail + 64) x npad_tail and its tile inverses
    // block-format system: b (npose x 7, padded to bpad doubles), then 49-f64 blocks
    int bpad = 0;
    size_t o_sys = 0, o_y = 0, o_L = 0, o_W = 0, o_xd = 0, o_Lg = 0, o_int = 0;
    // the plan integers, one array: [nodes fptr fronts tail rounds | tmap] (nints_back: what the
    // core + back-substitution launch stages in LDS; without tmap: a back-substitution-only launch)
    // [tg tc rtg rc] (nints: the whole plan of the single-workgroup solve) [tc3 rc4] (multi-launch
    // rounds only)
    size_t i_nodes = 0, i_fptr = 0, i_fronts = 0, i_tg = 0, i_tc = 0, i_rtg = 0, i_rc = 0,
           i_tail = 0, i_tmap = 0, i_rounds = 0, i_tc3 = 0, i_rc4 = 0, i_inl = 0, i_apt = 0, i_adj = 0,
           nints = 0, nints_back = 0;
    template <typename T>
    T* dptr(size_t off) const { return reinterpret_cast<T*>(dbuf + off); }
    const int* iptr(size_t i) const { return reinterpret_cast<const int*>(dbuf + o_int) + i; }
    // a fresh plan that keeps the lists' capacity: plans are rebuilt on every call, and fresh
    // allocations of this size come back as new pages -- a page fault per 4 KiB on every call
    // (tools/plan_bench.cpp)
    void reset() {
        SparsePlan fresh;
        for (auto v : {&SparsePlan::nodes, &SparsePlan::fptr, &SparsePlan::fronts, &SparsePlan::tg,
                       &SparsePlan::tc, &SparsePlan::rtg, &SparsePlan::rc, &SparsePlan::tail,
                       &SparsePlan::tmap, &SparsePlan::tc3, &SparsePlan::rc4, &SparsePlan::apt,
                       &SparsePlan::adj}) {
            (this->*v).clear();
            (fresh.*v).swap(this->*v);
        }
        fresh.inl.swap(inl);  // (kept as it is: see ninl)
        rounds.clear();
        fresh.rounds.swap(rounds);
        *this = std::move(fresh);
    }
};

// Elimination-round policy.  fused (gn_solve, one workgroup): rounds stop once the rest fits
// the in-register tail unless a round still removes >= kmin poses; a round's W blocks / y are
// staged in LDS (capped), RHS contributions name the pose's slot in the round.  multi
// (gn_sparse.hip): low-degree independent sets until fewer than rmin poses qualify, the rest
// goes to the tiled dense Cholesky; RHS contributions name the pose.
// mmd: multiple-minimum-degree candidates -- a round takes only poses of degree
// <= max(2 d_min, d_min + 1) (d_min: the current minimum degree), which keeps the fill close to
// a sequential minimum-degree ordering (cfg3: a 26-pose dense tail after 8 rounds, where taking
// every independent pose of degree <= dcap leaves a 31-35-pose clique).
struct RoundPolicy {
    bool fused;
    int dcap, rmin, rmax, tailcap, kmin;
    bool mmd;
};
// pairs: the unordered pose pairs of the graph's off-diagonal blocks (block id nblk0 + k for
// pairs[k], nblk0 = npose diagonal blocks first); nblk: the graph's block count.
// symbolic: choose the rounds and eliminate only -- no block ids, target / contribution lists
// (rounds, nodes, tail, fused_tail and nints_back as the full plan's, fronts and tmap sized but
// not filled; nblocks, nints and the lists not): what the driver needs to accept or reject a
// policy before building its plan.
// Cost (cfg4, 255 poses, 1007 pairs): counting sorts instead of comparison sorts for the round's
// targets and word-parallel fill keep the host plan well below the first accumulate it overlaps
// once the edges are sharded over several GPUs (tools/plan_bench.cpp).
inline void build_sparse_plan(const std::vector<std::pair<int, int>>& pairs, int nblk, int npose,
                              const RoundPolicy& pol, SparsePlan& sp, bool symbolic = false) {
    sp.reset();
    sp.nodes.reserve(npose);
    sp.fptr.reserve(npose + 1);
    const int dcap = pol.dcap, rmin = pol.rmin, rmax = pol.rmax, tailcap = pol.tailcap, kmin = pol.kmin;
    struct TC { int ki, kj; };  // a block-target contribution: two entries of one pose's front
    // the working lists, kept per thread across calls (capacity reused: see SparsePlan::reset)
    struct Scratch {
        std::vector<uint64_t> adj, fmask;
        std::vector<int> deg, bidm, cand, chosen, cnt;
        std::vector<char> alive, blocked;
        std::vector<std::vector<int>> F;
        std::vector<TC> tcs, tcs2;
        std::vector<int> rcs, rcs2, fq;  // RHS contributions: a front entry, or -1 - q (none)
    };
    static thread_local Scratch S;
    // adjacency as bitsets (one row of nw 64-bit words per pose), degrees, dense block ids
    const int nw = (npose + 63) / 64;
    auto& adj = S.adj;
    auto& fmask = S.fmask;
    auto& deg = S.deg;
    adj.assign((size_t)npose * nw, 0);
    fmask.assign(nw, 0);
    deg.assign(npose, 0);
    auto row = [&](int x) { return &adj[(size_t)x * nw]; };
    auto unlink = [&](int x, int y) {
        uint64_t& w = row(x)[y >> 6];
        const uint64_t m = 1ull << (y & 63);
        if (w & m) {
            w &= ~m;
            deg[x]--;
        }
    };
    auto neighbours = [&](int x, std::vector<int>& out) {  // ascending
        out.clear();
        const uint64_t* a = row(x);
        for (int k = 0; k < nw; k++)
            for (uint64_t w = a[k]; w; w &= w - 1) out.push_back(64 * k + __builtin_ctzll(w));
    };
    auto& bidm = S.bidm;  // upper triangle (x < y) used
    if (!symbolic) bidm.assign((size_t)npose * npose, -1);
    for (size_t k = 0; k < pairs.size(); k++) {
        const int a = pairs[k].first, b = pairs[k].second;
        for (int t = 0; t < 2; t++) {
            const int x = t ? b : a, y = t ? a : b;
            uint64_t& w = row(x)[y >> 6];
            const uint64_t m = 1ull << (y & 63);
            if (!(w & m)) {
                w |= m;
                deg[x]++;
            }
        }
        if (!symbolic) bidm[(size_t)a * npose + b] = npose + (int)k;
    }
    sp.nblocks = nblk;
    auto block_of = [&](int x, int y) -> int {
        if (x == y) return x;
        int& id = bidm[(size_t)std::min(x, y) * npose + std::max(x, y)];
        if (id < 0) id = sp.nblocks++;
        return id;
    };
    auto& alive = S.alive;
    auto& blocked = S.blocked;
    alive.assign(npose, 1);
    blocked.assign(npose, 0);
    int nalive = npose;
    sp.fptr.assign(1, 0);
    auto& cand = S.cand;
    auto& chosen = S.chosen;
    auto& cnt = S.cnt;
    cnt.assign(npose + 2, 0);
    auto& F = S.F;
    auto& tcs = S.tcs;
    auto& tcs2 = S.tcs2;
    auto& rcs = S.rcs;
    auto& rcs2 = S.rcs2;
    auto& fq = S.fq;  // the round's front entries' pose slot q
    // stable counting sort of xs by key(x) in [0, nk): O(n + nk)
    auto csort = [&](auto& xs, auto& tmp, int nk, auto key) {
        std::fill(cnt.begin(), cnt.begin() + nk + 1, 0);
        for (const auto& x : xs) cnt[key(x) + 1]++;
        for (int k = 0; k < nk; k++) cnt[k + 1] += cnt[k];
        tmp.resize(xs.size());
        for (const auto& x : xs) tmp[cnt[key(x)]++] = x;
        xs.swap(tmp);
    };
    int ntg_total = 0, nrtg_total = 0;  // multi-launch records so far (block, RHS targets)
    for (int round = 0; round < rmax && nalive > 0; round++) {
        // a remaining clique is the dense tail (eliminating it pose by pose gains nothing)
        bool clique = true;
        for (int v = 0; v < npose && clique; v++)
            if (alive[v] && deg[v] != nalive - 1) clique = false;
        if (clique && nalive > 1) break;
        cand.clear();
        int dlim = dcap;
        if (pol.mmd) {
            int dmin = npose;
            for (int v = 0; v < npose; v++)
                if (alive[v]) dmin = std::min(dmin, deg[v]);
            dlim = std::min(dcap, std::max(2 * dmin, dmin + 1));
        }
        for (int v = 0; v < npose; v++)
            if (alive[v] && deg[v] <= dlim) cand.push_back(v);
        std::stable_sort(cand.begin(), cand.end(), [&](int a, int b) { return deg[a] < deg[b]; });
        std::fill(blocked.begin(), blocked.end(), 0);
        chosen.clear();
        for (int v : cand) {
            if (blocked[v]) continue;
            chosen.push_back(v);
            blocked[v] = 1;
            const uint64_t* a = row(v);
            for (int k = 0; k < nw; k++)
                for (uint64_t w = a[k]; w; w &= w - 1) blocked[64 * k + __builtin_ctzll(w)] = 1;
        }
        // a round's W blocks and y vectors are staged in LDS: cap its poses (the rest stay
        // for the next round; any subset of an independent set is independent)
        if (pol.fused) {
            size_t k = 0, wsum = 0;
            while (k < chosen.size() && (int)k < kSolveRoundPoses &&
                   (wsum + deg[chosen[k]]) * 49 <= (size_t)kSolveWStage) {
                wsum += deg[chosen[k]];
                k++;
            }
            chosen.resize(k);
        }
        if ((int)chosen.size() < rmin && (int)chosen.size() != nalive) break;
        // multi (no tail cap): a round of fewer than kmin poses that leaves the dense core's tile
        // count unchanged only adds a forward and a back launch -- unless the core it would leave
        // exceeds the dense solve limit (later rounds may still bring it under)
        if (!pol.fused && tailcap == 0 && kmin > 0 && (int)chosen.size() < kmin &&
            (7 * nalive + kCholTile - 1) / kCholTile == (7 * (nalive - (int)chosen.size()) + kCholTile - 1) / kCholTile &&
            (int)sp_align_up((size_t)nalive * 7, kCholTile) <= kMaxNpad)
            break;
        // once the rest fits the in-register dense tail, a round must eliminate enough poses
        // to beat the per-pose cost of the tail steps
        if (nalive <= tailcap && (int)chosen.size() < kmin) break;
        std::sort(chosen.begin(), chosen.end());
        SpRound R;
        R.node_begin = (int)sp.nodes.size();
        R.nnodes = (int)chosen.size();
        R.wbeg = sp.nW;
        if (F.size() < chosen.size()) F.resize(chosen.size());
        tcs.clear();
        rcs.clear();
        fq.clear();
        const int kb = (int)sp.fronts.size() / 4;  // the round's first front entry
        for (size_t q = 0; q < chosen.size(); q++) {
            const int v = chosen[q];
            neighbours(v, F[q]);
            sp.nodes.push_back(v);
            const int k0 = (int)sp.fronts.size() / 4 - kb;
            for (int r : F[q]) {
                const int blk = symbolic ? 0 : block_of(r, v);
                sp.fronts.push_back(r);
                sp.fronts.push_back(blk);
                sp.fronts.push_back(r > v ? 1 : 0);
                sp.fronts.push_back(sp.nW++);
            }
            sp.fptr.push_back((int)sp.fronts.size() / 4);
            if (symbolic) continue;
            // contributions as front-entry indices (k = the round's entry, 8 B per block target
            // contribution): target (r, s) = (fr(ki), fr(kj)) of one pose's front
            const int nf = (int)F[q].size();
            for (int i = 0; i < nf; i++) {
                fq.push_back((int)q);
                for (int j = i; j < nf; j++) tcs.push_back({k0 + i, k0 + j});
                rcs.push_back(k0 + i);
            }
            // multi-launch rounds: a pose without fronts (its neighbours pinned or eliminated)
            // still needs L_v and y_v for the back-substitution -- a contribution to no target
            if (!pol.fused && F[q].empty()) rcs.push_back(-1 - (int)q);
        }
        if (!symbolic) {
            const int* fr = &sp.fronts[4 * (size_t)kb];  // (r, block, transposed, W id) per entry
            auto code = [&](int k) { return 2 * fr[4 * k + 1] + fr[4 * k + 2]; };
            // targets in (r, s) order, contributions in pose order (deterministic sums): they
            // were generated pose by pose, so a stable sort by s and then by r is (r, s, q)
            csort(tcs, tcs2, npose, [&](const TC& x) { return fr[4 * x.kj]; });
            csort(tcs, tcs2, npose, [&](const TC& x) { return fr[4 * x.ki]; });
            csort(rcs, rcs2, npose + 1, [&](int x) { return x < 0 ? 0 : fr[4 * x] + 1; });
            const size_t n = tcs.size();
            if (pol.fused) {
                // single-workgroup solve: targets (block, c0, c1) over (W id, W id) pairs; RHS
                // targets (pose, c0, c1) over (W id, node slot)
                R.tbeg = (int)sp.tg.size() / 3;
                size_t otc = sp.tc.size(), otg = sp.tg.size();
                sp.tc.resize(otc + 2 * n);
                sp.tg.resize(otg + 3 * n);  // (at most one target per contribution; trimmed below)
                int* tc = sp.tc.data() + otc;
                int* tg = sp.tg.data() + otg;
                for (size_t k = 0; k < n;) {
                    const int r = fr[4 * tcs[k].ki], s = fr[4 * tcs[k].kj];
                    const int c0 = (int)(otc / 2);
                    size_t e = k;
                    for (; e < n && fr[4 * tcs[e].ki] == r && fr[4 * tcs[e].kj] == s; e++) {
                        *tc++ = fr[4 * tcs[e].ki + 3];
                        *tc++ = fr[4 * tcs[e].kj + 3];
                        otc += 2;
                    }
                    *tg++ = block_of(r, s);
                    *tg++ = c0;
                    *tg++ = (int)(otc / 2);
                    k = e;
                }
                sp.tg.resize(tg - sp.tg.data());
                R.nbt = (int)sp.tg.size() / 3 - R.tbeg;
                R.rbeg = (int)sp.rtg.size() / 3;
                for (size_t k = 0; k < rcs.size();) {
                    const int r = fr[4 * rcs[k]];
                    const int c0 = (int)sp.rc.size() / 2;
                    size_t e = k;
                    for (; e < rcs.size() && fr[4 * rcs[e]] == r; e++) {
                        sp.rc.push_back(fr[4 * rcs[e] + 3]);
                        sp.rc.push_back(fq[rcs[e]]);
                    }
                    sp.rtg.push_back(r);
                    sp.rtg.push_back(c0);
                    sp.rtg.push_back((int)sp.rc.size() / 2);
                    k = e;
                }
                R.nrt = (int)sp.rtg.size() / 3 - R.rbeg;
            } else {
                // multi-launch rounds (sp_round_kernel): one kSpRec record per target, block
                // targets then RHS targets, the first kSpInline contributions inline; only the
                // rest go to tc3 / rc4, and a record's {c0, c1} is set so that contribution
                // k >= kSpInline is list entry c0 + k
                auto emit = [&](int tgt, int cnt, std::vector<int>& lst, int w, auto put) {
                    if (sp.inl.size() < sp.ninl + kSpRec)
                        sp.inl.resize(std::max(2 * sp.inl.size(), sp.ninl + (size_t)kSpRec * 256));
                    int* d = &sp.inl[sp.ninl];
                    sp.ninl += kSpRec;
                    const int ovf = (int)(lst.size() / w);
                    d[0] = tgt;
                    d[1] = ovf - kSpInline;
                    d[2] = ovf - kSpInline + cnt;
                    d[3] = 0;
                    for (int j = 0; j < std::min(cnt, kSpInline); j++) put(j, d + 4 + 4 * j);
                    for (int j = kSpInline; j < cnt; j++) {
                        int c[4];
                        put(j, c);
                        lst.insert(lst.end(), c, c + w);
                    }
                };
                R.tbeg = ntg_total;
                R.nbt = 0;
                for (size_t k = 0; k < n;) {
                    const int r = fr[4 * tcs[k].ki], s = fr[4 * tcs[k].kj];
                    size_t e = k;
                    while (e < n && fr[4 * tcs[e].ki] == r && fr[4 * tcs[e].kj] == s) e++;
                    emit(block_of(r, s), (int)(e - k), sp.tc3, 3, [&](int j, int* c) {
                        const int ki = tcs[k + j].ki, kj = tcs[k + j].kj;
                        c[0] = chosen[fq[ki]];
                        c[1] = code(ki);
                        c[2] = code(kj);
                        c[3] = 0;
                    });
                    R.nbt++;
                    k = e;
                }
                R.rbeg = nrtg_total;
                R.nrt = 0;
                for (size_t k = 0; k < rcs.size();) {
                    const int r = rcs[k] < 0 ? -1 : fr[4 * rcs[k]];
                    size_t e = k;
                    while (e < rcs.size() && (rcs[e] < 0 ? -1 : fr[4 * rcs[e]]) == r) e++;
                    emit(r, (int)(e - k), sp.rc4, 4, [&](int j, int* c) {
                        const int x = rcs[k + j];
                        const int q = x < 0 ? -1 - x : fq[x], v = chosen[q];
                        // (v, code_r, W id | -1, owner node | -1): the owner is the node's first
                        // front entry (or its no-target entry)
                        const bool first = x < 0 || x == 0 || fq[x - 1] != q;
                        c[0] = v;
                        c[1] = x < 0 ? 2 * v : code(x);
                        c[2] = x < 0 ? -1 : fr[4 * x + 3];
                        c[3] = first ? R.node_begin + q : -1;
                    });
                    R.nrt++;
                    k = e;
                }
                ntg_total += R.nbt;
                nrtg_total += R.nrt;
            }
        }
        R.wcount = sp.nW - R.wbeg;
        sp.rounds.push_back(R);
        // eliminate: drop the poses, connect each front into a clique (fill), word-parallel:
        // every front member's row gains the front's mask (minus itself)
        for (size_t q = 0; q < chosen.size(); q++) {
            const int v = chosen[q];
            for (int r : F[q]) unlink(r, v);
            std::fill(fmask.begin(), fmask.end(), 0);
            for (int r : F[q]) fmask[r >> 6] |= 1ull << (r & 63);
            for (int r : F[q]) {
                uint64_t* a = row(r);
                int added = 0;
                for (int k = 0; k < nw; k++) {
                    const uint64_t m = k == (r >> 6) ? fmask[k] & ~(1ull << (r & 63)) : fmask[k];
                    added += __builtin_popcountll(m & ~a[k]);
                    a[k] |= m;
                }
                deg[r] += added;
            }
            for (int r : F[q]) unlink(v, r);
            alive[v] = 0;
            nalive--;
        }
    }
    for (int v = 0; v < npose; v++)
        if (alive[v]) sp.tail.push_back(v);
    sp.ntail = (int)sp.tail.size();
    sp.zero_blk = sp.nblocks++;  // an all-zero block (zeroed with the fill blocks)
    sp.npad_tail = sp.ntail > 0 ? (int)sp_align_up((size_t)sp.ntail * 7, kCholTile) : 0;
    // the core's block map: code 2 block + (row pose > column pose); the tail is ascending, so
    // the upper triangle reads bidm row by row and the lower one mirrors it
    sp.tmap.assign((size_t)sp.ntail * sp.ntail, -1);
    for (int i = 0; i < (symbolic ? 0 : sp.ntail); i++) {
        const int x = sp.tail[i];
        sp.tmap[(size_t)i * sp.ntail + i] = 2 * x;
        const int* brow = &bidm[(size_t)x * npose];
        for (int j = i + 1; j < sp.ntail; j++) {
            const int id = brow[sp.tail[j]];
            if (id >= 0) {
                sp.tmap[(size_t)i * sp.ntail + j] = 2 * id;
                sp.tmap[(size_t)j * sp.ntail + i] = 2 * id + 1;
            }
        }
    }
    sp.fused_tail = sp.ntail * 7 <= kTailMax;
    sp.fused = pol.fused && sp.fused_tail;
    sp.nints_back = sp.nodes.size() + sp.fptr.size() + sp.fronts.size() + sp.tail.size() +
                    sp.tmap.size() + 8 * sp.rounds.size();
    sp.nints = sp.nints_back + sp.tg.size() + sp.tc.size() + sp.rtg.size() + sp.rc.size();
    sp.enabled = !symbolic;
}

}  // namespace m3s
