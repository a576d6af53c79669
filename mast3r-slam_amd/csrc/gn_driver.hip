// gn_driver.hip -- host driver of the Gauss-Newton ops (C ABI in include/m3s_backend.h).
//
// Replaces gauss_newton_{points,rays,calib}_cuda (reference gn_kernels.cu:725-811,
// 1140-1228, 1546-1637) and SparseBlock (:57-159).  Per call:
//   1. ONE host sync: copy ii/jj (and K) to the host, build the keyframe remap
//      (unique + searchsorted, :161-170), the block-sparse layout of the pose graph and
//      the deterministic CSR contribution lists; upload them into the workspace.
//   2. Enqueue max_iter iterations on the caller's stream with no host round trip:
//      accumulate -> edge reduce -> compact system [-> RCCL all-reduce] -> dense f64
//      blocked Cholesky -> retraction.  The ||dx|| < delta_thresh early exit is a device
//      flag that turns the remaining iterations into no-ops (same result as the
//      reference's host `break`).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <utility>
#include <vector>

#include "../../include/m3s_backend.h"
#include "gn_kernels.h"
#include "m3s_common.h"
#include "m3s_comm.h"

namespace m3s {

namespace {
thread_local std::string g_err;

// Optional phase timing with HIP events on the GN stream (bench.py roofline).
struct Prof {
    bool on = false;
    std::vector<hipEvent_t> pool;
    std::vector<hipEvent_t> marks;  // per iteration: t0 accum t1 system t2 solve t3 retract t4
    hipEvent_t get() {
        if (pool.empty()) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return nullptr;
            return e;
        }
        hipEvent_t e = pool.back();
        pool.pop_back();
        return e;
    }
    void mark(hipStream_t st) {
        if (!on) return;
        hipEvent_t e = get();
        if (e && hipEventRecord(e, st) == hipSuccess) marks.push_back(e);
    }
};
Prof g_prof;
}  // namespace

void set_error(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
}

const char* get_error() { return g_err.c_str(); }

namespace {

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Number of point chunks per directed edge: chunks of ~kChunkTarget points (the per-XCD
// working set of a chunk-major schedule is ~16 keyframes x chunk x 16 B), and at least
// ~4096 workgroups overall when the edge count is small.
int chunk_target() {
    static int t = [] {
        const char* e = getenv("M3S_ACC_CHUNK");
        return e ? std::max(1024, atoi(e)) : 8192;
    }();
    return t;
}

int choose_nchunks(int64_t HW, int64_t E_local) {
    int64_t nc = (HW + chunk_target() - 1) / chunk_target();
    const int64_t want = (4096 + std::max<int64_t>(E_local, 1) - 1) / std::max<int64_t>(E_local, 1);
    nc = std::max(nc, want);
    const int64_t max_nc = std::max<int64_t>(1, (HW + 1023) / 1024);
    nc = std::min(std::max<int64_t>(nc, 1), max_nc);
    int64_t chunk = align_up((size_t)((HW + nc - 1) / nc), 4);
    nc = (HW + chunk - 1) / chunk;
    return (int)std::max<int64_t>(nc, 1);
}

int chunk_points(int64_t HW, int nchunks) {
    return (int)align_up((size_t)((HW + nchunks - 1) / nchunks), 4);
}

struct Layout {
    size_t partials, edgeblk, compact, dense, x, flags, ii_loc, jj_loc, blk_ptr, blk_ent,
        grad_ptr, grad_ent, slotmap, linv, sched, pack, zs, total;
    int nchunks, npad, nblk_max;
};

Layout make_layout(int mode, int64_t N, int64_t HW, int64_t E_total, int64_t E_local) {
    Layout L{};
    const int64_t npose = std::max<int64_t>(N - 1, 0);
    const int64_t n = 7 * npose;
    L.nchunks = choose_nchunks(HW, E_local);
    L.npad = (int)std::max<int64_t>(kCholTile, align_up((size_t)n, kCholTile));
    L.nblk_max = (int)(npose + E_total);
    size_t off = 0;
    auto take = [&](size_t bytes) {
        size_t o = off;
        off = align_up(off + std::max<size_t>(bytes, 1), 256);
        return o;
    };
    L.partials = take(sizeof(float) * (size_t)E_local * L.nchunks * kNaccPad);
    L.edgeblk = take(sizeof(double) * (size_t)E_local * kEdgeBlk);
    L.compact = take(sizeof(double) * ((size_t)L.nblk_max * 28 + (size_t)npose * 7));
    L.dense = take(sizeof(double) * (size_t)(L.npad + kCholTile) * L.npad);
    L.x = take(sizeof(double) * (size_t)L.npad);
    L.flags = take(sizeof(int) * kNumFlags);
    L.ii_loc = take(sizeof(int) * (size_t)E_local);
    L.jj_loc = take(sizeof(int) * (size_t)E_local);
    L.blk_ptr = take(sizeof(int) * ((size_t)L.nblk_max + 1));
    L.blk_ent = take(sizeof(int) * (size_t)E_local * 4);
    L.grad_ptr = take(sizeof(int) * ((size_t)npose + 1));
    L.grad_ent = take(sizeof(int) * (size_t)E_local * 2);
    L.slotmap = take(sizeof(int) * (size_t)npose * npose);
    L.linv = take(sizeof(double) * (size_t)L.npad * kCholTile);
    L.sched = take(sizeof(int) * (size_t)E_local * L.nchunks);
    // iteration-invariant packed stream {code, sqrt q} per directed point-edge (8 B), and the
    // dense depth array of the keyframes (calib)
    L.pack = take(8 * (size_t)E_local * (size_t)HW);
    L.zs = take(mode == M3S_GN_CALIB ? sizeof(float) * (size_t)N * (size_t)HW : 0);
    L.total = off;
    return L;
}

// Host-side plan of the pose graph (identical on every rank: built from ALL edges).
struct Plan {
    int nblk = 0;
    std::vector<int> ii_loc, jj_loc;              // local edges: Twc/Xs rows
    std::vector<int> blk_ptr, blk_ent;            // CSR: slot -> (edge<<1 | neg)
    std::vector<int> grad_ptr, grad_ent;          // CSR: pose -> (edge<<1 | neg)
    std::vector<int> slotmap;                     // (npose x npose) -> slot or -1
    std::vector<int> sched;                       // accumulate task order: e * nchunks + c
    std::vector<std::pair<int, int>> pairs;       // slot nblk0.. -> unordered pose pair (a<b)
    float K[4] = {0, 0, 0, 0};
};

// XCD-aware order of the accumulate tasks (a performance heuristic only: results do not
// depend on it).  Local directed edges sorted by (jx, ix) are split into 8 contiguous
// groups, one per XCD (blocks b, b+8, ... share an XCD under round-robin dispatch); inside a
// group tasks run chunk-major, so the few keyframes of a group stay L2-resident while all
// of their edges stream the same point range.
void build_schedule(const std::vector<int>& ii_loc, const std::vector<int>& jj_loc, int nchunks,
                    std::vector<int>& sched) {
    const int E = (int)ii_loc.size();
    sched.clear();
    sched.reserve((size_t)E * nchunks);
    static const bool off = [] {
        const char* e = getenv("M3S_ACC_SCHED");
        return e && atoi(e) == 0;
    }();
    if (off) {
        for (int e = 0; e < E; e++)
            for (int c = 0; c < nchunks; c++) sched.push_back(e * nchunks + c);
        return;
    }
    std::vector<int> order(E);
    for (int e = 0; e < E; e++) order[e] = e;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
        return jj_loc[a] != jj_loc[b] ? jj_loc[a] < jj_loc[b] : ii_loc[a] < ii_loc[b];
    });
    const int G = 8;
    std::vector<std::vector<int>> lists(G);
    for (int g = 0; g < G; g++) {
        const int lo = (int)((int64_t)E * g / G), hi = (int)((int64_t)E * (g + 1) / G);
        for (int c = 0; c < nchunks; c++)
            for (int q = lo; q < hi; q++) lists[g].push_back(order[q] * nchunks + c);
    }
    std::vector<size_t> pos(G, 0);
    for (bool any = true; any;) {
        any = false;
        for (int g = 0; g < G; g++) {
            if (pos[g] < lists[g].size()) {
                sched.push_back(lists[g][pos[g]++]);
                any = true;
            }
        }
    }
}

int build_plan(const m3s_gn_args& a, hipStream_t st, Plan& plan) {
    const int64_t E = a.E_total;
    std::vector<int64_t> hii(E), hjj(E);
    float Kh[9] = {0};
    if (E > 0) {
        M3S_HIP_CHECK(hipMemcpyAsync(hii.data(), a.ii, sizeof(int64_t) * E, hipMemcpyDeviceToHost, st));
        M3S_HIP_CHECK(hipMemcpyAsync(hjj.data(), a.jj, sizeof(int64_t) * E, hipMemcpyDeviceToHost, st));
    }
    if (a.mode == M3S_GN_CALIB)
        M3S_HIP_CHECK(hipMemcpyAsync(Kh, a.K, sizeof(float) * 9, hipMemcpyDeviceToHost, st));
    M3S_HIP_CHECK(hipStreamSynchronize(st));
    plan.K[0] = Kh[0];  // fx = K[0][0]
    plan.K[1] = Kh[4];  // fy = K[1][1]
    plan.K[2] = Kh[2];  // cx = K[0][2]
    plan.K[3] = Kh[5];  // cy = K[1][2]

    // unique(cat(ii, jj)) sorted; searchsorted (gn_kernels.cu:161-170)
    std::vector<int64_t> u;
    u.reserve(2 * E);
    u.insert(u.end(), hii.begin(), hii.end());
    u.insert(u.end(), hjj.begin(), hjj.end());
    std::sort(u.begin(), u.end());
    u.erase(std::unique(u.begin(), u.end()), u.end());
    auto row_of = [&](int64_t id) {
        return (int64_t)(std::lower_bound(u.begin(), u.end(), id) - u.begin());
    };
    M3S_REQUIRE((int64_t)u.size() <= a.N,
                "gauss_newton: %lld unique keyframe ids in ii/jj but only %lld poses in Twc/Xs",
                (long long)u.size(), (long long)a.N);

    const int npose = (int)(a.N - 1);
    std::vector<int> iopt(E), jopt(E);
    for (int64_t e = 0; e < E; e++) {
        iopt[e] = (int)row_of(hii[e]) - 1;  // pin = num_fix = 1
        jopt[e] = (int)row_of(hjj[e]) - 1;
    }

    // block slots: diagonal blocks first (slot p <-> pose p+1), then unordered pairs in
    // order of first appearance over ALL edges.
    std::map<std::pair<int, int>, int> slot_of;
    plan.nblk = npose;
    for (int64_t e = 0; e < E; e++) {
        const int i = iopt[e], j = jopt[e];
        if (i >= 0 && j >= 0 && i != j) {
            const auto key = std::make_pair(std::min(i, j), std::max(i, j));
            if (!slot_of.count(key)) slot_of[key] = plan.nblk++;
        }
    }
    auto slot = [&](int r, int c) -> int {
        if (r == c) return r;
        return slot_of.at(std::make_pair(std::min(r, c), std::max(r, c)));
    };

    // contributions of the LOCAL edges (update_lhs order: (ii,ii,+) (ii,jj,-) (jj,ii,-) (jj,jj,+))
    std::vector<std::vector<int>> blk_lists(plan.nblk), grad_lists(std::max(npose, 0));
    plan.ii_loc.resize(a.E_local);
    plan.jj_loc.resize(a.E_local);
    for (int64_t el = 0; el < a.E_local; el++) {
        const int64_t e = a.edge_offset + el;
        const int i = iopt[e], j = jopt[e];
        plan.ii_loc[el] = i + 1;
        plan.jj_loc[el] = j + 1;
        const int rr[4] = {i, i, j, j}, cc[4] = {i, j, i, j}, neg[4] = {0, 1, 1, 0};
        for (int b = 0; b < 4; b++) {
            if (rr[b] >= 0 && cc[b] >= 0 && rr[b] <= cc[b])
                blk_lists[slot(rr[b], cc[b])].push_back((int)(el << 1) | neg[b]);
        }
        if (i >= 0) grad_lists[i].push_back((int)(el << 1) | 1);  // vi = -vj
        if (j >= 0) grad_lists[j].push_back((int)(el << 1));
    }
    plan.blk_ptr.assign(1, 0);
    for (auto& l : blk_lists) {
        plan.blk_ent.insert(plan.blk_ent.end(), l.begin(), l.end());
        plan.blk_ptr.push_back((int)plan.blk_ent.size());
    }
    plan.grad_ptr.assign(1, 0);
    for (auto& l : grad_lists) {
        plan.grad_ent.insert(plan.grad_ent.end(), l.begin(), l.end());
        plan.grad_ptr.push_back((int)plan.grad_ent.size());
    }
    plan.slotmap.assign((size_t)std::max(npose, 0) * std::max(npose, 0), -1);
    for (int p = 0; p < npose; p++) plan.slotmap[(size_t)p * npose + p] = p;
    plan.pairs.assign(plan.nblk - npose, std::make_pair(0, 0));
    for (auto& kv : slot_of) {
        const int r = kv.first.first, c = kv.first.second;
        plan.slotmap[(size_t)r * npose + c] = kv.second;
        plan.slotmap[(size_t)c * npose + r] = kv.second;
        plan.pairs[kv.second - npose] = kv.first;
    }
    return M3S_OK;
}


// ---------------------------------------------------------------------------------
// Block-sparse elimination plan (gn_sparse.hip): rounds of independent low-degree poses,
// then a dense core.  Built once per GN call (the pose graph is fixed across iterations).
// ---------------------------------------------------------------------------------
struct SpRound {
    int node_begin, nnodes, tbeg, nbt, rbeg, nrt;
};

struct SparsePlan {
    bool enabled = false;
    int nblocks = 0, nW = 0, ntail = 0, npad_tail = 0;
    std::vector<SpRound> rounds;
    std::vector<int> nodes, fptr, fronts, tg, tc, rtg, rc, tail, tmap;
    // device (one stream-ordered allocation per call)
    char* dbuf = nullptr;
    size_t o_A = 0, o_b = 0, o_y = 0, o_L = 0, o_W = 0, o_xd = 0, o_int = 0;
    size_t i_nodes = 0, i_fptr = 0, i_fronts = 0, i_tg = 0, i_tc = 0, i_rtg = 0, i_rc = 0,
           i_tail = 0, i_tmap = 0;
    template <typename T>
    T* dptr(size_t off) const { return reinterpret_cast<T*>(dbuf + off); }
    const int* iptr(size_t i) const { return reinterpret_cast<const int*>(dbuf + o_int) + i; }
};

int env_int(const char* name, int dflt) {
    const char* e = getenv(name);
    return e ? atoi(e) : dflt;
}

void build_sparse_plan(const Plan& p, int npose, SparsePlan& sp) {
    const int dcap = env_int("M3S_SPARSE_DCAP", 16);
    const int rmin = env_int("M3S_SPARSE_RMIN", 2);
    const int rmax = env_int("M3S_SPARSE_RMAX", 64);
    std::vector<std::set<int>> adj(npose);
    std::map<std::pair<int, int>, int> bid;
    for (size_t k = 0; k < p.pairs.size(); k++) {
        const int a = p.pairs[k].first, b = p.pairs[k].second;
        adj[a].insert(b);
        adj[b].insert(a);
        bid[p.pairs[k]] = npose + (int)k;
    }
    sp.nblocks = p.nblk;
    auto block_of = [&](int x, int y) -> int {
        if (x == y) return x;
        const auto key = std::make_pair(std::min(x, y), std::max(x, y));
        auto it = bid.find(key);
        if (it != bid.end()) return it->second;
        bid[key] = sp.nblocks;
        return sp.nblocks++;
    };
    std::vector<char> alive(npose, 1);
    int nalive = npose;
    sp.fptr.assign(1, 0);
    for (int round = 0; round < rmax && nalive > 0; round++) {
        std::vector<int> cand;
        for (int v = 0; v < npose; v++)
            if (alive[v] && (int)adj[v].size() <= dcap) cand.push_back(v);
        std::stable_sort(cand.begin(), cand.end(), [&](int a, int b) {
            return adj[a].size() != adj[b].size() ? adj[a].size() < adj[b].size() : a < b;
        });
        std::vector<char> blocked(npose, 0);
        std::vector<int> chosen;
        for (int v : cand) {
            if (blocked[v]) continue;
            chosen.push_back(v);
            blocked[v] = 1;
            for (int r : adj[v]) blocked[r] = 1;
        }
        if ((int)chosen.size() < rmin && (int)chosen.size() != nalive) break;
        std::sort(chosen.begin(), chosen.end());
        SpRound R;
        R.node_begin = (int)sp.nodes.size();
        R.nnodes = (int)chosen.size();
        std::map<std::pair<int, int>, std::vector<std::pair<int, int>>> tgt;
        std::map<int, std::vector<std::pair<int, int>>> rtgt;
        std::vector<std::vector<int>> F(chosen.size());
        for (size_t q = 0; q < chosen.size(); q++) {
            const int v = chosen[q];
            F[q].assign(adj[v].begin(), adj[v].end());
            sp.nodes.push_back(v);
            std::map<int, int> wof;
            for (int r : F[q]) {
                const int blk = block_of(r, v);
                const int wid = sp.nW++;
                sp.fronts.insert(sp.fronts.end(), {r, blk, r > v ? 1 : 0, wid});
                wof[r] = wid;
            }
            sp.fptr.push_back((int)sp.fronts.size() / 4);
            for (size_t i = 0; i < F[q].size(); i++)
                for (size_t j = i; j < F[q].size(); j++) {
                    const int r = F[q][i], s2 = F[q][j];  // r <= s2 (sorted)
                    tgt[std::make_pair(r, s2)].push_back(std::make_pair(wof[r], wof[s2]));
                }
            for (int r : F[q]) rtgt[r].push_back(std::make_pair(wof[r], v));
        }
        R.tbeg = (int)sp.tg.size() / 3;
        for (auto& kv : tgt) {
            const int blk = block_of(kv.first.first, kv.first.second);
            const int c0 = (int)sp.tc.size() / 2;
            for (auto& pr : kv.second) sp.tc.insert(sp.tc.end(), {pr.first, pr.second});
            sp.tg.insert(sp.tg.end(), {blk, c0, (int)sp.tc.size() / 2});
        }
        R.nbt = (int)tgt.size();
        R.rbeg = (int)sp.rtg.size() / 3;
        for (auto& kv : rtgt) {
            const int c0 = (int)sp.rc.size() / 2;
            for (auto& pr : kv.second) sp.rc.insert(sp.rc.end(), {pr.first, pr.second});
            sp.rtg.insert(sp.rtg.end(), {kv.first, c0, (int)sp.rc.size() / 2});
        }
        R.nrt = (int)rtgt.size();
        sp.rounds.push_back(R);
        // eliminate: drop the poses, connect each front into a clique (fill)
        for (size_t q = 0; q < chosen.size(); q++) {
            const int v = chosen[q];
            for (int r : F[q]) adj[r].erase(v);
            for (int r : F[q])
                for (int s2 : F[q])
                    if (r != s2) adj[r].insert(s2);
            adj[v].clear();
            alive[v] = 0;
            nalive--;
        }
    }
    for (int v = 0; v < npose; v++)
        if (alive[v]) sp.tail.push_back(v);
    sp.ntail = (int)sp.tail.size();
    sp.npad_tail = sp.ntail > 0 ? (int)align_up((size_t)sp.ntail * 7, kCholTile) : 0;
    sp.tmap.assign((size_t)sp.ntail * sp.ntail, -1);
    for (int i = 0; i < sp.ntail; i++)
        for (int j = 0; j < sp.ntail; j++) {
            const int x = sp.tail[i], y = sp.tail[j];
            int code = -1;
            if (x == y) {
                code = 2 * x;
            } else {
                auto it = bid.find(std::make_pair(std::min(x, y), std::max(x, y)));
                if (it != bid.end()) code = 2 * it->second + (x > y ? 1 : 0);
            }
            sp.tmap[(size_t)i * sp.ntail + j] = code;
        }
    sp.enabled = true;
}

int upload_sparse_plan(SparsePlan& sp, int npose, hipStream_t st) {
    size_t off = 0;
    auto take = [&](size_t bytes) {
        size_t o = off;
        off = align_up(off + std::max<size_t>(bytes, 8), 256);
        return o;
    };
    sp.o_A = take(sizeof(double) * 49 * (size_t)sp.nblocks);
    sp.o_b = take(sizeof(double) * 7 * (size_t)npose);
    sp.o_y = take(sizeof(double) * 7 * (size_t)npose);
    sp.o_L = take(sizeof(double) * 49 * sp.nodes.size());
    sp.o_W = take(sizeof(double) * 49 * (size_t)sp.nW);
    sp.o_xd = take(sizeof(double) * (size_t)std::max(sp.npad_tail, 1));
    std::vector<int> ints;
    auto put = [&](const std::vector<int>& v) {
        size_t i = ints.size();
        ints.insert(ints.end(), v.begin(), v.end());
        return i;
    };
    sp.i_nodes = put(sp.nodes);
    sp.i_fptr = put(sp.fptr);
    sp.i_fronts = put(sp.fronts);
    sp.i_tg = put(sp.tg);
    sp.i_tc = put(sp.tc);
    sp.i_rtg = put(sp.rtg);
    sp.i_rc = put(sp.rc);
    sp.i_tail = put(sp.tail);
    sp.i_tmap = put(sp.tmap);
    sp.o_int = take(sizeof(int) * std::max<size_t>(ints.size(), 1));
    M3S_HIP_CHECK(hipMallocAsync((void**)&sp.dbuf, off, st));
    if (!ints.empty())
        M3S_HIP_CHECK(hipMemcpyAsync(sp.dbuf + sp.o_int, ints.data(), sizeof(int) * ints.size(),
                                     hipMemcpyHostToDevice, st));
    M3S_HIP_CHECK(hipStreamSynchronize(st));  // the host vector dies with this call
    return M3S_OK;
}

int validate(const m3s_gn_args& a) {
    M3S_REQUIRE(a.mode == M3S_GN_POINTS || a.mode == M3S_GN_RAYS || a.mode == M3S_GN_CALIB,
                "gauss_newton: bad mode %d", a.mode);
    M3S_REQUIRE(a.N >= 1 && a.HW >= 1, "gauss_newton: need N >= 1 poses and HW >= 1 points");
    M3S_REQUIRE(a.E_total >= 0 && a.E_local >= 0 && a.edge_offset >= 0 &&
                    a.edge_offset + a.E_local <= a.E_total,
                "gauss_newton: bad edge range");
    M3S_REQUIRE(a.HW < ((int64_t)1 << 31) && a.E_local < (1 << 30),
                "gauss_newton: sizes exceed int32 indexing");
    M3S_REQUIRE(7 * (a.N - 1) <= kMaxNpad,
                "gauss_newton: %lld poses exceed the dense solve limit (%d unknowns)",
                (long long)a.N, kMaxNpad);
    M3S_REQUIRE(a.mode != M3S_GN_CALIB || (a.K != nullptr && a.width > 0 && a.height > 0),
                "gauss_newton_calib: K / image size required");
    M3S_REQUIRE(a.Twc && a.Xs && a.Cs && a.dx, "gauss_newton: null pointer");
    if (a.E_total > 0) M3S_REQUIRE(a.ii && a.jj, "gauss_newton: null ii/jj");
    if (a.E_local > 0) M3S_REQUIRE(a.idx && a.valid && a.Q, "gauss_newton: null edge data");
    const size_t need = make_layout(a.mode, a.N, a.HW, a.E_total, a.E_local).total;
    M3S_REQUIRE(a.ws != nullptr && a.ws_bytes >= need,
                "gauss_newton: workspace too small (%zu < %zu bytes)", a.ws_bytes, need);
    return M3S_OK;
}

struct Ctx {
    bool packed = false;  // per-call packed stream (gn_pack_kernel) feeds the accumulate
    Layout L;
    Plan plan;
    SparsePlan sp;
    AccParams P;
    bool vec;
    char* ws;
    hipStream_t st;
    template <typename T>
    T* at(size_t off) const { return reinterpret_cast<T*>(ws + off); }
};

int setup(const m3s_gn_args& a, Ctx& c) {
    int rc = validate(a);
    if (rc) return rc;
    c.st = (hipStream_t)a.stream;
    c.ws = (char*)a.ws;
    c.L = make_layout(a.mode, a.N, a.HW, a.E_total, a.E_local);
    rc = build_plan(a, c.st, c.plan);
    if (rc) return rc;
    build_schedule(c.plan.ii_loc, c.plan.jj_loc, c.L.nchunks, c.plan.sched);
    const Layout& L = c.L;
    const Plan& p = c.plan;
    auto up = [&](size_t off, const std::vector<int>& v) -> hipError_t {
        if (v.empty()) return hipSuccess;
        return hipMemcpyAsync(c.ws + off, v.data(), sizeof(int) * v.size(), hipMemcpyHostToDevice, c.st);
    };
    M3S_HIP_CHECK(up(L.ii_loc, p.ii_loc));
    M3S_HIP_CHECK(up(L.jj_loc, p.jj_loc));
    M3S_HIP_CHECK(up(L.blk_ptr, p.blk_ptr));
    M3S_HIP_CHECK(up(L.blk_ent, p.blk_ent));
    M3S_HIP_CHECK(up(L.grad_ptr, p.grad_ptr));
    M3S_HIP_CHECK(up(L.grad_ent, p.grad_ent));
    M3S_HIP_CHECK(up(L.slotmap, p.slotmap));
    M3S_HIP_CHECK(up(L.sched, p.sched));
    M3S_HIP_CHECK(hipMemsetAsync(c.ws + L.flags, 0, sizeof(int) * kNumFlags, c.st));
    // the host vectors die with this call: wait for the (pageable) uploads
    M3S_HIP_CHECK(hipStreamSynchronize(c.st));

    AccParams& P = c.P;
    P.s0_inv = 1.0f / a.sigma0;
    P.s1_inv = (a.mode == M3S_GN_POINTS) ? 0.0f : 1.0f / a.sigma1;
    P.C_thresh = a.C_thresh;
    P.Q_thresh = a.Q_thresh;
    P.fx = p.K[0];
    P.fy = p.K[1];
    P.cx = p.K[2];
    P.cy = p.K[3];
    P.pb_lo = (float)a.pixel_border;
    P.pb_hi_u = (float)(a.width - 1 - a.pixel_border);
    P.pb_hi_v = (float)(a.height - 1 - a.pixel_border);
    P.z_eps = a.z_eps;
    P.width = a.width > 0 ? a.width : 1;
    P.height = a.height;
    {   // Granlund-Montgomery: l = ceil(log2 W), m = ceil(2^(31+l) / W) < 2^32
        int l = 0;
        while ((1LL << l) < P.width) l++;
        const unsigned long long num = 1ULL << (31 + l);
        P.div_m = (unsigned)((num + (unsigned long long)P.width - 1) / (unsigned long long)P.width);
        P.div_sh = 31 + l;
    }
    P.HW = (int)a.HW;
    P.chunk = chunk_points(a.HW, L.nchunks);
    P.nchunks = L.nchunks;
    auto al16 = [](const void* ptr) { return ((uintptr_t)ptr & 15) == 0; };
    c.vec = (a.HW % 4 == 0) && al16(a.Xs) && al16(a.Cs) && al16(a.idx) && al16(a.valid) &&
            al16(a.Q);
    // M3S_GN_PACK: 0 never, 1 (default) when the call runs >= 3 iterations, 2 always
    const int pack_mode = env_int("M3S_GN_PACK", 1);
    c.packed = c.vec && a.E_local > 0 && (pack_mode == 2 || (pack_mode == 1 && a.max_iter >= 3));
    return M3S_OK;
}

// Once per call, before the iterations: the packed stream (and calib depth array).
int prepare_iterations(const m3s_gn_args& a, Ctx& c) {
    if (!c.packed) return M3S_OK;
    const Layout& L = c.L;
    M3S_HIP_CHECK(launch_pack(c.st, (int)a.E_local, a.Xs, a.N, a.Cs, c.at<int>(L.ii_loc),
                              c.at<int>(L.jj_loc), a.idx, a.valid, a.Q, c.P, c.at<int4>(L.pack),
                              a.mode == M3S_GN_CALIB ? c.at<float>(L.zs) : nullptr,
                              c.at<int>(L.flags)));
    return M3S_OK;
}

// accumulate + edge reduce + compact (+ all-reduce): the system of one iteration
int enqueue_system(const m3s_gn_args& a, Ctx& c) {
    const Layout& L = c.L;
    int* flags = c.at<int>(L.flags);
    if (a.E_local > 0) {
        g_prof.mark(c.st);
        const dim3 grid((unsigned)(L.nchunks * a.E_local));
        if (c.packed)
            M3S_HIP_CHECK(launch_accum_packed(a.mode, grid, c.st, a.Twc, a.Xs, c.at<float>(L.zs),
                                              c.at<int>(L.ii_loc), c.at<int>(L.jj_loc),
                                              c.at<int4>(L.pack), c.P, c.at<int>(L.sched),
                                              c.at<float>(L.partials), flags));
        else
            M3S_HIP_CHECK(launch_accum(a.mode, c.vec, grid, c.st, a.Twc, a.Xs, a.Cs,
                                       c.at<int>(L.ii_loc), c.at<int>(L.jj_loc), a.idx, a.valid,
                                       a.Q, c.P, c.at<int>(L.sched), c.at<float>(L.partials),
                                       flags));
        g_prof.mark(c.st);
        M3S_HIP_CHECK(launch_edge_reduce((int)a.E_local, c.st, c.at<float>(L.partials), L.nchunks,
                                         a.Twc, c.at<int>(L.ii_loc), c.at<double>(L.edgeblk), flags));
    }
    const int npose = (int)(a.N - 1);
    M3S_HIP_CHECK(launch_compact(c.st, c.at<double>(L.edgeblk), c.at<int>(L.blk_ptr),
                                 c.at<int>(L.blk_ent), c.at<int>(L.grad_ptr),
                                 c.at<int>(L.grad_ent), c.plan.nblk, npose,
                                 c.at<double>(L.compact), flags));
    if (a.comm) {
        const size_t count = (size_t)c.plan.nblk * 28 + (size_t)npose * 7;
        int rc = comm_allreduce_sum_f64(a.comm, c.at<double>(L.compact), count, c.st);
        if (rc) return rc;
    }
    return M3S_OK;
}

int enqueue_solve(const m3s_gn_args& a, Ctx& c) {
    const Layout& L = c.L;
    const int npose = (int)(a.N - 1);
    int* flags = c.at<int>(L.flags);
    if (!c.sp.enabled) {
        M3S_HIP_CHECK(launch_solve(c.st, c.at<double>(L.compact), c.at<int>(L.slotmap), c.plan.nblk,
                                   npose, 7 * npose, L.npad, c.at<double>(L.dense),
                                   c.at<double>(L.linv), c.at<double>(L.x), flags));
        return M3S_OK;
    }
    SparsePlan& sp = c.sp;
    double* A = sp.dptr<double>(sp.o_A);
    double* b = sp.dptr<double>(sp.o_b);
    double* y = sp.dptr<double>(sp.o_y);
    double* Ls = sp.dptr<double>(sp.o_L);
    double* W = sp.dptr<double>(sp.o_W);
    double* x = c.at<double>(L.x);
    M3S_HIP_CHECK(launch_sp_init(c.st, c.at<double>(L.compact), c.plan.nblk, sp.nblocks, npose, A, b,
                                 flags));
    for (const SpRound& R : sp.rounds) {
        M3S_HIP_CHECK(launch_sp_factor(c.st, R.nnodes, sp.iptr(sp.i_nodes), sp.iptr(sp.i_fptr),
                                       sp.iptr(sp.i_fronts), R.node_begin, A, b, Ls, W, y, flags));
        M3S_HIP_CHECK(launch_sp_schur(c.st, sp.iptr(sp.i_tg), sp.iptr(sp.i_tc), R.tbeg, R.nbt,
                                      sp.iptr(sp.i_rtg), sp.iptr(sp.i_rc), R.rbeg, R.nrt, W, y, A, b,
                                      flags));
    }
    M3S_HIP_CHECK(launch_sp_tail(c.st, A, b, sp.iptr(sp.i_tmap), sp.iptr(sp.i_tail), sp.ntail,
                                 sp.npad_tail, c.at<double>(L.dense), c.at<double>(L.linv),
                                 sp.dptr<double>(sp.o_xd), x, flags));
    for (auto it = sp.rounds.rbegin(); it != sp.rounds.rend(); ++it)
        M3S_HIP_CHECK(launch_sp_back(c.st, it->nnodes, sp.iptr(sp.i_nodes), sp.iptr(sp.i_fptr),
                                     sp.iptr(sp.i_fronts), it->node_begin, Ls, W, y, x, flags));
    return M3S_OK;
}

int run(const m3s_gn_args& a) {
    Ctx c;
    int rc = setup(a, c);
    if (rc) return rc;
    const int npose = (int)(a.N - 1);
    if (npose <= 0) return M3S_OK;  // nothing to optimise (all poses pinned)
    const Layout& L = c.L;
    int* flags = c.at<int>(L.flags);
    if (env_int("M3S_SOLVER_DENSE", 0) == 0) {
        build_sparse_plan(c.plan, npose, c.sp);
        rc = upload_sparse_plan(c.sp, npose, c.st);
        if (rc) return rc;
    }
    rc = prepare_iterations(a, c);
    if (rc) return rc;
    for (int itr = 0; itr < a.max_iter; itr++) {
        g_prof.mark(c.st);
        rc = enqueue_system(a, c);
        if (rc) return rc;
        g_prof.mark(c.st);
        rc = enqueue_solve(a, c);
        if (rc) return rc;
        g_prof.mark(c.st);
        M3S_HIP_CHECK(launch_retract(c.st, a.Twc, c.at<double>(L.x), a.dx, (int)a.N,
                                     a.delta_thresh, flags));
        g_prof.mark(c.st);
    }
    if (c.sp.dbuf) M3S_HIP_CHECK(hipFreeAsync(c.sp.dbuf, c.st));
    return M3S_OK;
}

}  // namespace
}  // namespace m3s

using namespace m3s;

extern "C" const char* m3s_last_error(void) { return m3s::get_error(); }

extern "C" const char* m3s_version(void) { return "m3s 0.1.0 gfx950"; }

extern "C" size_t m3s_gn_workspace_bytes(int mode, int64_t N, int64_t HW, int64_t E_total,
                                         int64_t E_local) {
    if (N < 1 || HW < 1 || E_total < 0 || E_local < 0) return 0;
    return make_layout(mode, N, HW, E_total, E_local).total;
}

extern "C" int m3s_gauss_newton(const m3s_gn_args* args) {
    if (!args) {
        set_error("gauss_newton: null args");
        return M3S_ERR_INVALID;
    }
    return run(*args);
}

extern "C" int m3s_gn_build_system(const m3s_gn_args* args, double* H_host, double* b_host) {
    if (!args) {
        set_error("gn_build_system: null args");
        return M3S_ERR_INVALID;
    }
    const m3s_gn_args& a = *args;
    Ctx c;
    int rc = setup(a, c);
    if (rc) return rc;
    const int npose = (int)(a.N - 1);
    const int n = 7 * npose;
    if (npose <= 0) return M3S_OK;
    rc = prepare_iterations(a, c);
    if (rc) return rc;
    rc = enqueue_system(a, c);
    if (rc) return rc;
    const Layout& L = c.L;
    M3S_HIP_CHECK(launch_fill_only(c.st, c.at<double>(L.compact), c.at<int>(L.slotmap), c.plan.nblk,
                                   npose, n, L.npad, c.at<double>(L.dense), c.at<int>(L.flags)));
    M3S_HIP_CHECK(hipMemcpy2DAsync(H_host, sizeof(double) * n, c.at<double>(L.dense),
                                   sizeof(double) * L.npad, sizeof(double) * n, n,
                                   hipMemcpyDeviceToHost, c.st));
    M3S_HIP_CHECK(hipMemcpyAsync(b_host, c.at<double>(L.dense) + (size_t)L.npad * L.npad,
                                 sizeof(double) * n, hipMemcpyDeviceToHost, c.st));
    M3S_HIP_CHECK(hipStreamSynchronize(c.st));
    return M3S_OK;
}

namespace {
m3s_gn_args base_args(int mode, float* Twc, const float* Xs, const float* Cs, const int64_t* ii,
                      const int64_t* jj, const int64_t* idx, const uint8_t* valid, const float* Q,
                      int64_t N, int64_t HW, int64_t E, int max_iter, float delta_thresh,
                      float* dx, void* ws, size_t ws_bytes, void* stream) {
    m3s_gn_args a;
    std::memset(&a, 0, sizeof(a));
    a.mode = mode;
    a.Twc = Twc; a.Xs = Xs; a.Cs = Cs; a.ii = ii; a.jj = jj;
    a.idx = idx; a.valid = valid; a.Q = Q;
    a.N = N; a.HW = HW; a.E_total = E; a.E_local = E; a.edge_offset = 0;
    a.max_iter = max_iter; a.delta_thresh = delta_thresh;
    a.dx = dx; a.ws = ws; a.ws_bytes = ws_bytes; a.stream = stream;
    return a;
}
}  // namespace

extern "C" int m3s_gauss_newton_points(float* Twc, const float* Xs, const float* Cs,
                                       const int64_t* ii, const int64_t* jj, const int64_t* idx,
                                       const uint8_t* valid, const float* Q, int64_t N, int64_t HW,
                                       int64_t E, float sigma_point, float C_thresh,
                                       float Q_thresh, int max_iter, float delta_thresh,
                                       float* dx, void* ws, size_t ws_bytes, void* stream) {
    m3s_gn_args a = base_args(M3S_GN_POINTS, Twc, Xs, Cs, ii, jj, idx, valid, Q, N, HW, E,
                              max_iter, delta_thresh, dx, ws, ws_bytes, stream);
    a.sigma0 = sigma_point;
    a.C_thresh = C_thresh;
    a.Q_thresh = Q_thresh;
    return run(a);
}

extern "C" int m3s_gauss_newton_rays(float* Twc, const float* Xs, const float* Cs,
                                     const int64_t* ii, const int64_t* jj, const int64_t* idx,
                                     const uint8_t* valid, const float* Q, int64_t N, int64_t HW,
                                     int64_t E, float sigma_ray, float sigma_dist, float C_thresh,
                                     float Q_thresh, int max_iter, float delta_thresh, float* dx,
                                     void* ws, size_t ws_bytes, void* stream) {
    m3s_gn_args a = base_args(M3S_GN_RAYS, Twc, Xs, Cs, ii, jj, idx, valid, Q, N, HW, E, max_iter,
                              delta_thresh, dx, ws, ws_bytes, stream);
    a.sigma0 = sigma_ray;
    a.sigma1 = sigma_dist;
    a.C_thresh = C_thresh;
    a.Q_thresh = Q_thresh;
    return run(a);
}

extern "C" int m3s_gauss_newton_calib(float* Twc, const float* Xs, const float* Cs, const float* K,
                                      const int64_t* ii, const int64_t* jj, const int64_t* idx,
                                      const uint8_t* valid, const float* Q, int64_t N, int64_t HW,
                                      int64_t E, int height, int width, int pixel_border,
                                      float z_eps, float sigma_pixel, float sigma_depth,
                                      float C_thresh, float Q_thresh, int max_iter,
                                      float delta_thresh, float* dx, void* ws, size_t ws_bytes,
                                      void* stream) {
    m3s_gn_args a = base_args(M3S_GN_CALIB, Twc, Xs, Cs, ii, jj, idx, valid, Q, N, HW, E,
                              max_iter, delta_thresh, dx, ws, ws_bytes, stream);
    a.K = K;
    a.height = height;
    a.width = width;
    a.pixel_border = pixel_border;
    a.z_eps = z_eps;
    a.sigma0 = sigma_pixel;
    a.sigma1 = sigma_depth;
    a.C_thresh = C_thresh;
    a.Q_thresh = Q_thresh;
    return run(a);
}

// ---- profiling (bench.py): phase times from HIP events on the GN stream ----
extern "C" int m3s_prof_begin(void) {
    for (hipEvent_t e : g_prof.marks) g_prof.pool.push_back(e);
    g_prof.marks.clear();
    g_prof.on = true;
    return M3S_OK;
}

// out[0] accumulate-kernel ms, out[1] edge-reduce/compact/all-reduce ms, out[2] solve ms,
// out[3] retract ms (sums over iterations); *n_iter = iterations recorded.
extern "C" int m3s_prof_end(double* out, int* n_iter) {
    g_prof.on = false;
    const size_t per = 6;  // t0 [a0 a1] t1 t2 t3 (a0/a1 bracket the accumulate kernel)
    double acc[4] = {0, 0, 0, 0};
    int n = 0;
    for (size_t k = 0; k + per <= g_prof.marks.size(); k += per) {
        hipEvent_t* m = &g_prof.marks[k];
        float ms[5];
        for (int q = 0; q < 5; q++) {
            M3S_HIP_CHECK(hipEventSynchronize(m[q + 1]));
            M3S_HIP_CHECK(hipEventElapsedTime(&ms[q], m[q], m[q + 1]));
        }
        acc[0] += ms[1];
        acc[1] += ms[0] + ms[2];
        acc[2] += ms[3];
        acc[3] += ms[4];
        n++;
    }
    for (int q = 0; q < 4; q++) out[q] = acc[q];
    *n_iter = n;
    for (hipEvent_t e : g_prof.marks) g_prof.pool.push_back(e);
    g_prof.marks.clear();
    return M3S_OK;
}
