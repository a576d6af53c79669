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
#include <chrono>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <utility>
#include <vector>

#include "../../include/m3s_backend.h"
#include "gn_kernels.h"
#include "m3s_common.h"
#include "m3s_comm.h"
#include "sparse_plan.h"

namespace m3s {

namespace {
thread_local std::string g_err;

// Optional phase timing with HIP events on the GN stream (bench.py roofline).
int env_int(const char* name, int dflt);

struct Prof {
    bool on = false;
    std::vector<hipEvent_t> pool;
    std::vector<hipEvent_t> marks;  // per iteration: t0 accum t1 system t2 solve t3 retract t4
    hipEvent_t get() {
        if (pool.empty()) {
            // timing-only events: no system-scope release / acquire when recorded (a default
            // event record writes back and invalidates the caches -- idle GPU between the
            // kernels it separates); M3S_PROF_SYSFENCE=1: default events
            static const bool sysfence = env_int("M3S_PROF_SYSFENCE", 0) != 0;
            hipEvent_t e;
            if (sysfence || hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) {
                (void)hipGetLastError();
                if (hipEventCreate(&e) != hipSuccess) return nullptr;
            }
            return e;
        }
        hipEvent_t e = pool.back();
        pool.pop_back();
        return e;
    }
    bool accum_only = false;  // record only the two events bracketing the accumulate kernel
    // (every timed event record is a queue marker; with a release to system scope it left ~5 us
    // of idle GPU each, so the timed bench region carries only the accumulate pair)
    std::vector<char> first;  // accum_only: per event pair, the launch built the packed records
    void mark(hipStream_t st, bool accum = false, bool first_pack = false) {
        if (!on || (accum_only && !accum)) return;
        hipEvent_t e = get();
        if (e && hipEventRecord(e, st) == hipSuccess) {
            marks.push_back(e);
            if (accum_only && marks.size() % 2 == 0) first.push_back(first_pack);
        }
    }
};
Prof g_prof;
std::vector<double> g_prof_launch_ms;  // the last accumulate-only session: the iteration kernel's per-launch ms
std::vector<double> g_prof_solve_ms;   // the last phase session: each iteration's solve ms
}  // namespace

int g_dbg_flags[4] = {0, 0, 0, 0};  // done, fail, packed, ray-constrained accumulate (last call)
int g_dbg_pcg[5] = {0, 0, 0, 0, 0};  // PCG solves, their CG steps, fallbacks, PCG planned, first PCG iteration (last call)

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
struct HostResources {
    std::mutex mu;
    std::vector<std::pair<void*, void (*)(void*)>> items;
    bool shut = false;
};
HostResources& host_resources() {
    static HostResources* r = new HostResources;  // never destroyed (used from atexit)
    return *r;
}
}  // namespace

void register_host_resource(void* obj, void (*release)(void*)) {
    HostResources& r = host_resources();
    std::lock_guard<std::mutex> lk(r.mu);
    r.items.emplace_back(obj, release);
}

namespace {

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Pinned host staging for the per-call plan transfers (D2H of ii/jj/K, H2D of the plan
// integers): one buffer per host thread, reused across calls.  The H2D copies of a call are
// asynchronous; the next call waits for them (an event) before overwriting the buffer.
struct Staging {
    char* buf = nullptr;
    char* dev = nullptr;  // buf's device address (the stage-copy kernel reads it directly)
    size_t cap = 0;
    hipEvent_t done = nullptr;
    bool pending = false;
    // no destructor: released by m3s_shutdown (m3s_common.h)
    static void release(void* p) {
        Staging* s = static_cast<Staging*>(p);
        if (s->pending) (void)hipEventSynchronize(s->done);
        if (s->done) (void)hipEventDestroy(s->done);
        if (s->buf) (void)hipHostFree(s->buf);
        s->buf = s->dev = nullptr;
        s->cap = 0;
        s->done = nullptr;
        s->pending = false;
    }
    // a buffer of >= bytes, free of in-flight copies
    char* get(size_t bytes) {
        if (pending) {
            (void)hipEventSynchronize(done);
            pending = false;
        }
        if (bytes > cap) {
            if (buf) (void)hipHostFree(buf);
            cap = align_up(std::max<size_t>(bytes, 1 << 16) * 2, 4096);
            if (hipHostMalloc((void**)&buf, cap, hipHostMallocDefault) != hipSuccess) {
                buf = nullptr;
                cap = 0;
            } else if (hipHostGetDevicePointer((void**)&dev, buf, 0) != hipSuccess) {
                dev = nullptr;
            }
        }
        return buf;
    }
    // H2D of [h, h + bytes) (inside buf) to dst, stream-ordered: by a kernel reading the pinned
    // buffer (default), or by hipMemcpyAsync (M3S_STAGE_DMA=1, or no device address)
    hipError_t upload(void* dst, const char* h, size_t bytes, hipStream_t st) {
        static const bool dma = [] {
            const char* e = getenv("M3S_STAGE_DMA");
            return e && atoi(e) != 0;
        }();
        if (!dma && dev && (bytes & 3) == 0 && ((uintptr_t)dst & 15) == 0 && ((h - buf) & 15) == 0)
            return launch_stage_copy(st, dst, dev + (h - buf), bytes);
        return hipMemcpyAsync(dst, h, bytes, hipMemcpyHostToDevice, st);
    }
    // D2H of bytes from src (device) into [h, h + bytes) (inside buf), stream-ordered: by the
    // same copy kernel writing the pinned buffer through its device address (default; a DMA
    // transfer's queue handshake costs more than the copy at these sizes), or by
    // hipMemcpyAsync (M3S_STAGE_DMA=1, unaligned, or no device address)
    hipError_t download(char* h, const void* src, size_t bytes, hipStream_t st) {
        static const bool dma = [] {
            const char* e = getenv("M3S_STAGE_DMA");
            return e && atoi(e) != 0;
        }();
        if (!dma && dev && (bytes & 3) == 0 && ((uintptr_t)src & 15) == 0 && ((h - buf) & 15) == 0)
            return launch_stage_copy(st, dev + (h - buf), src, bytes);
        return hipMemcpyAsync(h, src, bytes, hipMemcpyDeviceToHost, st);
    }
    hipError_t mark(hipStream_t st) {
        if (!done) {
            hipError_t e = hipEventCreateWithFlags(&done, hipEventDisableTiming);
            if (e != hipSuccess) return e;
        }
        hipError_t e = hipEventRecord(done, st);
        pending = e == hipSuccess;
        return e;
    }
};
// Per host thread, created on first use and registered for m3s_shutdown (a thread that ends
// leaves its buffers to the shutdown).  The thread_local objects are plain pointers: nothing
// runs at thread or process exit.
struct Stagings {
    Staging in;   // D2H
    Staging out;  // H2D: the sparse solver's plan
    Staging ws;   // H2D: the workspace's plan (CSR lists, schedule)
    Staging tmo;  // D2H: the last call's timeout flag (deferred report, see take_deferred_timeout)
    int tmo_armed = 0;  // 0: nothing to report; 1: tmo holds an int flag; 2: a double (rank sum)
    static void release(void* p) {
        Stagings* s = static_cast<Stagings*>(p);
        Staging::release(&s->in);
        Staging::release(&s->out);
        Staging::release(&s->ws);
        Staging::release(&s->tmo);
        s->tmo_armed = 0;
    }
};
thread_local Stagings* t_stagings = nullptr;
Stagings& stagings() {
    if (!t_stagings) {
        t_stagings = new Stagings;
        register_host_resource(t_stagings, &Stagings::release);
    }
    return *t_stagings;
}

// The PCG's side stream (gn_pcg.hip): M's refresh (sp_inverse_kernel) runs there, beside the
// next iteration's accumulate on the call's stream; per host thread and device (the events must
// not be shared by concurrent calls), released by m3s_shutdown.
struct PcgSide {
    static constexpr int kMaxDev = 64;
    hipStream_t ss[kMaxDev] = {};
    hipEvent_t e1[kMaxDev] = {}, e2[kMaxDev] = {};
    static void release(void* p) {
        PcgSide* s = static_cast<PcgSide*>(p);
        for (int d = 0; d < kMaxDev; d++) {
            if (s->e1[d]) (void)hipEventDestroy(s->e1[d]);
            if (s->e2[d]) (void)hipEventDestroy(s->e2[d]);
            if (s->ss[d]) (void)hipStreamDestroy(s->ss[d]);
            s->e1[d] = s->e2[d] = nullptr;
            s->ss[d] = nullptr;
        }
    }
};
thread_local PcgSide* t_pcg_side = nullptr;
// this thread's side stream and its two events for the current device (created on first use)
int pcg_side(hipStream_t& ss, hipEvent_t& e1, hipEvent_t& e2) {
    if (!t_pcg_side) {
        t_pcg_side = new PcgSide;
        register_host_resource(t_pcg_side, &PcgSide::release);
    }
    int dev = 0;
    M3S_HIP_CHECK(hipGetDevice(&dev));
    M3S_REQUIRE(dev >= 0 && dev < PcgSide::kMaxDev, "gauss_newton: device %d out of range", dev);
    PcgSide& p = *t_pcg_side;
    if (!p.ss[dev]) {
        M3S_HIP_CHECK(hipStreamCreateWithFlags(&p.ss[dev], hipStreamNonBlocking));
        // (device-scope only: a default event's system-scope release / acquire writes back and
        // invalidates the caches on the call's stream at every record -- idle GPU, Prof above)
        M3S_HIP_CHECK(hipEventCreateWithFlags(&p.e1[dev], hipEventDisableTiming | hipEventDisableSystemFence));
        M3S_HIP_CHECK(hipEventCreateWithFlags(&p.e2[dev], hipEventDisableTiming | hipEventDisableSystemFence));
    }
    ss = p.ss[dev];
    e1 = p.e1[dev];
    e2 = p.e2[dev];
    return M3S_OK;
}

// Points per accumulate task (edge x chunk).  16384 (round 3): the chunks amortise the task
// prologue (pose loads, the affine map) and the workgroup reduction over twice the points of the
// former 8192 -- cfg3 accumulate 0.342 -> 0.331 ms, cfg4 1.98 -> 1.94 ms; flat up to ~49k
// (profiles/r03_chunk_ab.txt)
int chunk_target() {
    static int t = [] {
        const char* e = getenv("M3S_ACC_CHUNK");
        return e ? std::max(1024, atoi(e)) : 16384;
    }();
    return t;
}

// Number of point chunks per directed edge: chunks of ~chunk_target() points (the per-XCD
// working set of a chunk-major schedule is ~16 keyframes x chunk x 16 B), and at least
// ~4096 workgroups overall when the edge count is small.
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
    size_t partials, edgeblk, compact, x, flags, ii_loc, jj_loc, blk_ptr, blk_ent, blk_ref, grad_ptr,
        grad_ent, ecnt, cok, sorder, sched, pack, packx, pcnt, zs, twc_save, total;
    int nchunks, npad, nblk_max;
};

int env_int(const char* name, int dflt);

Layout make_layout(int mode, int64_t N, int64_t HW, int64_t E_total, int64_t E_local) {
    Layout L{};
    const int64_t npose = std::max<int64_t>(N - 1, 0);
    const int64_t n = 7 * npose;
    // from the TOTAL edge count: every rank of a sharded call then chunks its edges exactly as one
    // GPU would, so the per-edge f32 partial sums (and the poses, up to the f64 all-reduce order)
    // do not depend on the number of ranks
    L.nchunks = choose_nchunks(HW, E_total);
    L.npad = (int)std::max<int64_t>(kCholTile, align_up((size_t)n, kCholTile));
    L.nblk_max = (int)(npose + E_total);
    size_t off = 0;
    auto take = [&](size_t bytes) {
        size_t o = off;
        off = align_up(off + std::max<size_t>(bytes, 1), 256);
        return o;
    };
    L.partials = take(sizeof(float) * (size_t)E_local * L.nchunks * kNaccPad);
    // per-edge records: the fast path's f64 Hjj/vj (kEdgeBlk doubles), or the reference-order
    // path's f32 D/g (kRefStride floats)
    static_assert(sizeof(float) * kRefStride <= sizeof(double) * kEdgeBlk, "edge record");
    L.edgeblk = take(sizeof(double) * (size_t)E_local * kEdgeBlk);
    L.compact = take(sizeof(double) * ((size_t)L.nblk_max * 28 + (size_t)npose * 7));
    // (the dense f64 matrices -- the dense solver's / debug system's (npad+64) x npad, the sparse
    // solvers' core -- are sized by the solver actually used, in per-call stream-ordered
    // allocations: see Ctx::alloc_dense and upload_sparse_plan)
    L.x = take(sizeof(double) * (size_t)L.npad);
    L.flags = take(sizeof(int) * kNumFlags);
    L.cok = take(sizeof(int) * (size_t)std::max<int64_t>(N, 1));  // per keyframe: every c > C_thresh
    L.twc_save = take(sizeof(float) * 8 * (size_t)std::max<int64_t>(N, 1));  // Twc at the call's start
    L.ii_loc = take(sizeof(int) * (size_t)E_local);
    L.jj_loc = take(sizeof(int) * (size_t)E_local);
    L.blk_ptr = take(sizeof(int) * ((size_t)L.nblk_max + 1));
    // (the CSR lists span ALL edges when the ranks' records are gathered: Plan::gather)
    L.blk_ent = take(sizeof(int) * (size_t)std::max(E_local, E_total) * 4);
    L.blk_ref = take(sizeof(int) * (size_t)E_local * 4);  // reference-order assembly codes
    L.grad_ptr = take(sizeof(int) * ((size_t)npose + 1));
    L.grad_ent = take(sizeof(int) * (size_t)std::max(E_local, E_total) * 2);
    L.ecnt = take(sizeof(int) * (size_t)E_local);  // fused edge reduce: finished chunks per edge
    L.sorder = take(sizeof(int) * (size_t)E_local);  // the accumulate schedule's edge order
    L.sched = take(sizeof(int) * 4 * (size_t)E_local * L.nchunks);  // {edge, chunk, ix, jx} per task
    // iteration-invariant packed stream {code, sqrt q} per directed point-edge (8 B), and the
    // dense depth array of the keyframes (calib)
    if (env_int("M3S_GN_COMPACT", 0) != 0) {
        // compacted stream (opt-in): every (edge, chunk) region holds a whole chunk
        const size_t cap = (size_t)E_local * (size_t)L.nchunks * (size_t)chunk_points(HW, L.nchunks);
        L.pack = take(8 * std::max(cap, (size_t)E_local * (size_t)HW));
        L.packx = take(12 * cap);
        L.pcnt = take(sizeof(int) * (size_t)E_local * L.nchunks);
    } else {
        L.pack = take(8 * (size_t)E_local * (size_t)HW);
        L.packx = L.pcnt = L.pack;  // unused
    }
    // + the ray tables tu[W], tv[H] (gn_depth_kernel); HW floats is an upper bound for W + H
    // + the inverse depths IZs [N, HW] after the tables (gn_accum.hip inv_depths)
    L.zs = take(mode == M3S_GN_CALIB ? sizeof(float) * (2 * (size_t)N + 1) * (size_t)HW + 64 : 0);
    L.total = off;
    return L;
}

// Host-side plan of the pose graph (identical on every rank: built from ALL edges).
struct Plan {
    int nblk = 0;
    std::vector<int> ii_loc, jj_loc;              // local edges: Twc/Xs rows
    std::vector<int> blk_ptr, blk_ent;            // CSR: slot -> (edge<<1 | neg)
    std::vector<int> blk_ref;                     // the same entries as (edge<<3 | type), gn_refacc.hip
    std::vector<int> grad_ptr, grad_ent;          // CSR: pose -> (edge<<1 | neg)
    std::vector<int> slotmap;                     // (npose x npose) -> slot or -1
    std::vector<std::pair<int, int>> pairs;      // slot nblk0.. -> unordered pose pair (a<b)
    float K[4] = {0, 0, 0, 0};
    // Edge-ordered exchange of a sharded call: the ranks' per-edge records are all-gathered into
    // nranks blocks of gchunk records (rank r's edges at r * gchunk), and the CSR lists cover ALL
    // edges in edge order by their gathered position -- every rank assembles exactly the sum one
    // GPU does, so the poses do not depend on the rank count
    bool gather = false;
    int grank = 0, granks = 1, gchunk = 0;
};

// XCD-aware order of the accumulate tasks (a performance heuristic only: results do not
// depend on it).  Local directed edges sorted by (jx, ix) are split into 8 contiguous
// groups, one per XCD (blocks b, b+8, ... share an XCD under round-robin dispatch); inside a
// group tasks run chunk-major, so the few keyframes of a group stay L2-resident while all
// of their edges stream the same point range.  The host orders the edges (two stable
// counting sorts, by ix then by jx: the stable (jx, ix) order, O(E + N)) and sizes the groups;
// the device expands the task records {e, c, ix, jx} (launch_sched_expand): group g's list is
// chunk-major (element k: edge order[lo_g + k % n_g], chunk k / n_g) and the groups are
// interleaved round-robin.  (Written record by record into pinned memory and read back over
// PCIe, the schedule cost ~0.1 ms of host time per cfg4 call.)
void build_schedule_order(const std::vector<int>& ii_loc, const std::vector<int>& jj_loc, int nkey, int* order,
                          SchedGroups& G) {
    const int E = (int)ii_loc.size();
    static const bool off = [] {
        const char* e = getenv("M3S_ACC_SCHED");
        return e && atoi(e) == 0;
    }();
    G = SchedGroups{};
    G.off = off ? 1 : 0;
    if (off || E == 0) return;
    static thread_local std::vector<int> tmp, cnt;
    tmp.resize(E);
    auto pass = [&](const std::vector<int>& key, const int* src, int* dst) {
        cnt.assign((size_t)nkey + 1, 0);
        for (int k = 0; k < E; k++) cnt[key[src ? src[k] : k] + 1]++;
        for (int v = 0; v < nkey; v++) cnt[v + 1] += cnt[v];
        for (int k = 0; k < E; k++) {
            const int e = src ? src[k] : k;
            dst[cnt[key[e]]++] = e;
        }
    };
    pass(ii_loc, nullptr, tmp.data());
    pass(jj_loc, tmp.data(), order);
    constexpr int NG = 8;
    G.q = E;
    for (int g = 0; g < NG; g++) {
        G.lo[g] = (int)((int64_t)E * g / NG);
        G.n[g] = (int)((int64_t)E * (g + 1) / NG) - G.lo[g];
        G.q = std::min(G.q, G.n[g]);
    }
    for (int g = 0; g < NG; g++)
        if (G.n[g] > G.q) G.big[G.nbig++] = g;
}

int gn_order(const m3s_gn_args& a);

// The pose graph's blocks from the edge lists (host copies): keyframe ids -> rows by
// unique(cat(ii, jj)) sorted + searchsorted (gn_kernels.cu:161-170), the first row pinned
// (num_fix = 1); diagonal blocks first (slot p <-> pose p), then the unordered pose pairs in order
// of first appearance over ALL edges; slotmap is the dense (npose x npose) slot table.
int plan_pairs(const int64_t* hii, const int64_t* hjj, int64_t E, int64_t N, Plan& plan, std::vector<int>& iopt,
               std::vector<int>& jopt) {
    const int npose = (int)(N - 1);
    iopt.resize(E);
    jopt.resize(E);
    // keyframe ids are small non-negative integers in practice: rank them through a dense
    // table (O(E + max id)); a comparison sort of the 2E ids took most of this function's
    // ~0.2 ms per cfg4 call.  Other ids: sort + binary search.
    int64_t lo = 0, hi = -1;
    for (int64_t e = 0; e < E; e++) {
        lo = std::min({lo, hii[e], hjj[e]});
        hi = std::max({hi, hii[e], hjj[e]});
    }
    size_t nuniq = 0;
    if (lo >= 0 && hi < std::max<int64_t>(1 << 16, 8 * (E + N))) {
        static thread_local std::vector<int> rank;
        rank.assign((size_t)hi + 1, 0);
        for (int64_t e = 0; e < E; e++) rank[hii[e]] = rank[hjj[e]] = 1;
        for (int64_t id = 0; id <= hi; id++)
            if (rank[id]) rank[id] = (int)nuniq++;
        if ((int64_t)nuniq <= N)
            for (int64_t e = 0; e < E; e++) {
                iopt[e] = rank[hii[e]] - 1;  // pin = num_fix = 1
                jopt[e] = rank[hjj[e]] - 1;
            }
    } else {
        std::vector<int64_t> u(hii, hii + E);
        u.insert(u.end(), hjj, hjj + E);
        std::sort(u.begin(), u.end());
        u.erase(std::unique(u.begin(), u.end()), u.end());
        nuniq = u.size();
        auto row_of = [&](int64_t id) { return (int)(std::lower_bound(u.begin(), u.end(), id) - u.begin()); };
        if ((int64_t)nuniq <= N)
            for (int64_t e = 0; e < E; e++) {
                iopt[e] = row_of(hii[e]) - 1;
                jopt[e] = row_of(hjj[e]) - 1;
            }
    }
    M3S_REQUIRE((int64_t)nuniq <= N,
                "gauss_newton: %lld unique keyframe ids in ii/jj but only %lld poses in Twc/Xs",
                (long long)nuniq, (long long)N);
    plan.slotmap.assign((size_t)std::max(npose, 0) * std::max(npose, 0), -1);
    for (int q = 0; q < npose; q++) plan.slotmap[(size_t)q * npose + q] = q;
    plan.nblk = npose;
    plan.pairs.clear();
    for (int64_t e = 0; e < E; e++) {
        const int i = iopt[e], j = jopt[e];
        if (i >= 0 && j >= 0 && i != j && plan.slotmap[(size_t)i * npose + j] < 0) {
            plan.slotmap[(size_t)i * npose + j] = plan.slotmap[(size_t)j * npose + i] = plan.nblk++;
            plan.pairs.push_back(std::make_pair(std::min(i, j), std::max(i, j)));
        }
    }
    return M3S_OK;
}

double g_plan_sync_us = 0;  // M3S_PROF_HOST: build_plan's edge-list copies + stream sync

// before_wait: enqueued after the edge-list copies, before the host waits for them (work that
// needs no plan runs on the GPU while the host plans)
int build_plan(const m3s_gn_args& a, hipStream_t st, Plan& plan, const std::function<int()>& before_wait = {}) {
    const int64_t E = a.E_total;
    // sharded call: gather the edge records (M3S_GN_GATHER=0: all-reduce the assembled system)
    int grank = 0, granks = 1;
    if (a.comm && gn_order(a) != M3S_GN_ORDER_REFERENCE && env_int("M3S_GN_GATHER", 1) != 0) {
        int rc = comm_rank_size(a.comm, &grank, &granks);
        if (rc) return rc;
    }
    const size_t hb_ranges = align_up(sizeof(int64_t) * 2 * (size_t)E + 64, 64);
    char* hb = stagings().in.get(hb_ranges + sizeof(double) * 2 * (size_t)granks);
    M3S_REQUIRE(hb != nullptr, "gauss_newton: pinned host allocation failed");
    int64_t* hii = reinterpret_cast<int64_t*>(hb);
    int64_t* hjj = hii + E;
    float* Kh = reinterpret_cast<float*>(hjj + E);
    double* hr = reinterpret_cast<double*>(hb + hb_ranges);  // every rank's (edge_offset, E_local)
    double* dr = nullptr;
    if (granks > 1) {
        // the ranks' edge ranges (once per call; exact in f64 below 2^53)
        hr[2 * grank] = (double)a.edge_offset;
        hr[2 * grank + 1] = (double)a.E_local;
        M3S_HIP_CHECK(hipMallocAsync((void**)&dr, sizeof(double) * 2 * (size_t)granks, st));
        Staging& in = stagings().in;
        M3S_HIP_CHECK(in.upload(dr + 2 * grank, reinterpret_cast<const char*>(hr + 2 * grank), sizeof(double) * 2, st));
        int rc = comm_allgather_f64(a.comm, dr, 2, st);
        if (rc) {
            (void)hipFreeAsync(dr, st);
            return rc;
        }
        M3S_HIP_CHECK(in.download(reinterpret_cast<char*>(hr), dr, sizeof(double) * 2 * (size_t)granks, st));
        M3S_HIP_CHECK(hipFreeAsync(dr, st));
    }
    const auto c0 = std::chrono::steady_clock::now();
    Staging& in = stagings().in;
    if (E > 0) {
        M3S_HIP_CHECK(in.download(reinterpret_cast<char*>(hii), a.ii, sizeof(int64_t) * E, st));
        M3S_HIP_CHECK(in.download(reinterpret_cast<char*>(hjj), a.jj, sizeof(int64_t) * E, st));
    }
    if (a.mode == M3S_GN_CALIB)
        M3S_HIP_CHECK(in.download(reinterpret_cast<char*>(Kh), a.K, sizeof(float) * 9, st));
    if (before_wait) {
        static thread_local hipEvent_t copied = nullptr;  // (no destructor: nothing at exit)
        if (!copied) M3S_HIP_CHECK(hipEventCreateWithFlags(&copied, hipEventDisableTiming));
        M3S_HIP_CHECK(hipEventRecord(copied, st));
        int rc = before_wait();
        if (rc) return rc;
        M3S_HIP_CHECK(hipEventSynchronize(copied));
    } else {
        M3S_HIP_CHECK(hipStreamSynchronize(st));
    }
    g_plan_sync_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - c0).count();
    // gathered position of every edge, when the ranks' ranges partition [0, E) (else: the
    // all-reduce of the assembled system, which sums whatever the ranks hold)
    std::vector<int> gpos;
    plan.gather = false;
    plan.grank = grank;
    plan.granks = granks;
    plan.gchunk = 0;
    if (granks > 1) {
        int64_t chunk = 0;
        std::vector<int> cover(E, 0);
        bool ok = true;
        gpos.assign(E, -1);
        for (int r = 0; r < granks && ok; r++) {
            const int64_t off = (int64_t)hr[2 * r], cnt = (int64_t)hr[2 * r + 1];
            ok = off >= 0 && cnt >= 0 && off + cnt <= E;
            chunk = std::max(chunk, cnt);
        }
        for (int r = 0; r < granks && ok; r++) {
            const int64_t off = (int64_t)hr[2 * r], cnt = (int64_t)hr[2 * r + 1];
            for (int64_t k = 0; k < cnt && ok; k++) {
                ok = cover[off + k]++ == 0;
                gpos[off + k] = (int)(r * chunk + k);
            }
        }
        for (int64_t e = 0; e < E && ok; e++) ok = cover[e] == 1;
        ok = ok && (int64_t)granks * chunk < (int64_t)(INT32_MAX >> 3);
        if (ok && chunk > 0) {
            plan.gather = true;
            plan.gchunk = (int)chunk;
        }
    }
    if (a.mode == M3S_GN_CALIB) {
        plan.K[0] = Kh[0];  // fx = K[0][0]
        plan.K[1] = Kh[4];  // fy = K[1][1]
        plan.K[2] = Kh[2];  // cx = K[0][2]
        plan.K[3] = Kh[5];  // cy = K[1][2]
    }

    const int npose = (int)(a.N - 1);
    std::vector<int> iopt, jopt;
    int rc = plan_pairs(hii, hjj, E, a.N, plan, iopt, jopt);
    if (rc) return rc;
    auto slot = [&](int r, int c) { return plan.slotmap[(size_t)r * npose + c]; };

    // contributions of the LOCAL edges as CSR lists (update_lhs order per edge:
    // (ii,ii,+) (ii,jj,-) (jj,ii,-) (jj,jj,+)), built by counting sort
    plan.ii_loc.resize(a.E_local);
    plan.jj_loc.resize(a.E_local);
    plan.blk_ptr.assign(plan.nblk + 1, 0);
    plan.grad_ptr.assign(std::max(npose, 0) + 1, 0);
    for (int pass = 0; pass < 2; pass++) {
        std::vector<int> bfill, gfill;
        if (pass == 1) {
            for (int k = 0; k < plan.nblk; k++) plan.blk_ptr[k + 1] += plan.blk_ptr[k];
            for (int k = 0; k < npose; k++) plan.grad_ptr[k + 1] += plan.grad_ptr[k];
            plan.blk_ent.assign(plan.blk_ptr[plan.nblk], 0);
            plan.blk_ref.assign(plan.gather ? 0 : plan.blk_ptr[plan.nblk], 0);
            plan.grad_ent.assign(plan.grad_ptr[npose], 0);
            bfill.assign(plan.blk_ptr.begin(), plan.blk_ptr.end() - 1);
            gfill.assign(plan.grad_ptr.begin(), plan.grad_ptr.end() - 1);
        }
        // the lists' edges: the local ones, or ALL (by gathered position) when gathering
        const int64_t nlist = plan.gather ? E : a.E_local;
        for (int64_t el = 0; el < nlist; el++) {
            const int64_t e = plan.gather ? el : a.edge_offset + el;
            const int64_t code = plan.gather ? gpos[e] : el;
            const int i = iopt[e], j = jopt[e];
            if (pass == 0 && !plan.gather) {
                plan.ii_loc[el] = i + 1;
                plan.jj_loc[el] = j + 1;
            }
            const int rr[4] = {i, i, j, j}, cc[4] = {i, j, i, j}, neg[4] = {0, 1, 1, 0};
            for (int b = 0; b < 4; b++) {
                if (rr[b] >= 0 && cc[b] >= 0 && rr[b] <= cc[b]) {
                    const int sl = slot(rr[b], cc[b]);
                    if (pass == 0) {
                        plan.blk_ptr[sl + 1]++;
                    } else {
                        // reference-order block types (gn_assemble_ref_kernel): Hs[0]/Hs[3] on
                        // the diagonal, Hs[1] at (ii, jj) when ii < jj, Hs[2] at (jj, ii) when
                        // jj < ii, a self-edge's Hs[1]/Hs[2] on its diagonal block
                        const int type = (b == 0 || b == 3) ? 0 : (i == j ? (b == 1 ? 3 : 4) : (b == 1 ? 2 : 1));
                        if (!plan.gather) plan.blk_ref[bfill[sl]] = (int)(el << 3) | type;
                        plan.blk_ent[bfill[sl]++] = (int)(code << 1) | neg[b];
                    }
                }
            }
            if (i >= 0) {  // vi = -vj
                if (pass == 0) plan.grad_ptr[i + 1]++;
                else plan.grad_ent[gfill[i]++] = (int)(code << 1) | 1;
            }
            if (j >= 0) {
                if (pass == 0) plan.grad_ptr[j + 1]++;
                else plan.grad_ent[gfill[j]++] = (int)(code << 1);
            }
        }
    }
    if (plan.gather) {
        for (int64_t el = 0; el < a.E_local; el++) {
            plan.ii_loc[el] = iopt[a.edge_offset + el] + 1;
            plan.jj_loc[el] = jopt[a.edge_offset + el] + 1;
        }
        plan.blk_ref.clear();  // (the reference order never gathers)
    }
    return M3S_OK;
}


// ---------------------------------------------------------------------------------
// Block-sparse elimination plan (sparse_plan.h builds it, gn_sparse.hip runs it): its round
// policies and the upload.
// ---------------------------------------------------------------------------------
int env_int(const char* name, int dflt) {
    const char* e = getenv(name);
    return e ? atoi(e) : dflt;
}

RoundPolicy fused_policy() {
    return {true, env_int("M3S_SPARSE_DCAP", 64), env_int("M3S_SPARSE_RMIN", 1),
            env_int("M3S_SPARSE_RMAX", 64),
            std::min(kTailPoseMax, env_int("M3S_SPARSE_TAILCAP", kTailPoseMax)),
            env_int("M3S_SPARSE_KMIN", 4), env_int("M3S_SPARSE_MMD", 1) != 0};
}
// multi: dcap 32 (round 5: cfg4 -- 255 free poses, 1007 pose pairs -- 4 rounds and a 125-pose
// core instead of 3 rounds and 141 poses; solve 0.307 -> 0.288 ms per iteration on one box, dcap
// 24 0.292, 64 0.301: profiles/r05_b_dcap*.json)
RoundPolicy multi_policy() {
    return {false, env_int("M3S_MULTI_DCAP", 32), env_int("M3S_MULTI_RMIN", 2),
            env_int("M3S_MULTI_RMAX", 64), 0, env_int("M3S_MULTI_KMIN", 4), env_int("M3S_MULTI_MMD", 0) != 0};
}
// hybrid: multi-launch rounds in minimum-degree order down to a dense core, then gn_solve
// back-substitutes and retracts.  The core is factored by the dataflow launch (M3S_HYB_CORE=1,
// default) -- then it is not bound by gn_solve's in-register factorisation (kTailPoseMax poses)
// and M3S_HYB_TAILCAP may move the rounds' stop point up to kHybDfTailMax poses -- or in
// registers (M3S_HYB_CORE=0, or the cooperative rounds launch: <= kTailPoseMax poses).
// Default stop point with the dataflow core: 36 poses (252 unknowns: still 4 tile columns), where
// a round must remove >= kmin poses to continue -- cfg3: 5 rounds and a 34-pose core instead of 8
// rounds and 26 poses, solve 0.1205 -> 0.1148 ms per iteration (two interleaved same-box rounds;
// caps 30 and 40 with kmin 6 -- 7 rounds / 28 poses, 4 rounds / 39 poses in 5 tiles -- were slower:
// profiles/r05_ap_hyb_tailcap/).
constexpr int kHybDfTailMax = 64;
constexpr int kHybDfTailDefault = 36;
// read by the planner per call and carried with the plan (SparsePlan::core_df), so that
// enqueue_solve factors the core the way the plan was sized for (a per-call read
// beside a per-process one could hand a 28-64-pose core to the in-register factorisation)
bool hyb_core_df() { return env_int("M3S_HYB_CORE", 1) != 0 && env_int("M3S_SOLVE_COOP", 0) == 0; }
RoundPolicy hybrid_policy() {
    const bool df = hyb_core_df();
    return {false, env_int("M3S_HYB_DCAP", 64), env_int("M3S_HYB_RMIN", 1),
            env_int("M3S_HYB_RMAX", 64),
            std::min(df ? kHybDfTailMax : kTailPoseMax, env_int("M3S_HYB_TAILCAP", df ? kHybDfTailDefault : kTailPoseMax)),
            env_int("M3S_HYB_KMIN", 4), env_int("M3S_HYB_MMD", 1) != 0};
}
// the hybrid plan's core fits its factorisation
bool hyb_core_fits(const SparsePlan& p) {
    return hyb_core_df() ? p.ntail <= kHybDfTailMax : p.fused_tail;
}

int upload_sparse_plan(SparsePlan& sp, int npose, hipStream_t st) {
    size_t off = 0;
    auto take = [&](size_t bytes) {
        size_t o = off;
        off = align_up(off + std::max<size_t>(bytes, 8), 256);
        return o;
    };
    sp.bpad = (int)align_up((size_t)npose * 7, 49);
    sp.o_sys = take(sizeof(double) * ((size_t)sp.bpad + 49 * (size_t)sp.nblocks));
    sp.o_y = take(sizeof(double) * 7 * (size_t)npose);
    sp.o_L = take(sizeof(double) * std::max(kLStoreRec, 49) * sp.nodes.size());
    sp.o_W = take(sizeof(double) * 49 * (size_t)sp.nW);
    sp.o_xd = take(sizeof(double) * (size_t)std::max(sp.npad_tail, 1));
    if (sp.npad_tail > 0) {
        sp.o_dense = take(sizeof(double) * (size_t)(sp.npad_tail + kCholTile) * sp.npad_tail);
        sp.o_linv = take(chol_linv_bytes(sp.npad_tail));
    }
    sp.o_Lg = take(sp.fused_tail ? sizeof(double) * 49 * (size_t)sp.ntail * sp.ntail : 0);
    sp.o_dfcnt = take(sizeof(int) * (size_t)sp_rounds_df_words((int)sp.rounds.size()));
    if (sp.pcg) {
        sp.snap_bytes = 0;
        if (sp.pcg_lag >= 2) {
            sp.snap_bytes = (sp.npad_tail > 0 ? sp.o_linv + chol_linv_bytes(sp.npad_tail) : sp.o_xd) - sp.o_L;
            sp.o_snap = take(sp.snap_bytes);
        }
        sp.o_pcgx = take(sizeof(double) * (size_t)npose * 7 * sp.pcg_ldx);
        sp.o_pcgxt = take(sizeof(float) * (size_t)npose * 7 * sp.pcg_ldt);
        sp.o_gran = take(16 * 4 * (size_t)sp.pcg_nv);
    }
    // the plan integers in one array (layout: SparsePlan), the rounds BEFORE tmap: a launch that
    // only back-substitutes stages [nodes fptr fronts tail rounds] and not the core map
    std::vector<const std::vector<int>*> parts = {&sp.nodes, &sp.fptr, &sp.fronts, &sp.tail,
                                                  &sp.tmap, &sp.tg, &sp.tc, &sp.rtg, &sp.rc,
                                                  &sp.tc3, &sp.rc4, &sp.inl, &sp.apt, &sp.adj};
    size_t* offs[] = {&sp.i_nodes, &sp.i_fptr, &sp.i_fronts, &sp.i_tail, &sp.i_tmap, &sp.i_tg,
                      &sp.i_tc, &sp.i_rtg, &sp.i_rc, &sp.i_tc3, &sp.i_rc4, &sp.i_inl, &sp.i_apt, &sp.i_adj};
    // (inl: its first ninl ints; SparsePlan::inl)
    auto len = [&](size_t k) { return parts[k] == &sp.inl ? sp.ninl : parts[k]->size(); };
    size_t n = 0;
    for (size_t k = 0; k < parts.size(); k++) {
        if (k == 4) {
            sp.i_rounds = n;
            n += 8 * sp.rounds.size();
        }
        if (parts[k] == &sp.inl) n = align_up(n, 4);  // 16-B records (int4 loads)
        if (parts[k] == &sp.adj) n = align_up(n, 2);  // int2 entries
        *offs[k] = n;
        n += len(k);
    }
    sp.o_int = take(sizeof(int) * std::max<size_t>(n, 1));
    M3S_HIP_CHECK(hipMallocAsync((void**)&sp.dbuf, off, st));
    M3S_HIP_CHECK(hipMemsetAsync(sp.dbuf + sp.o_dfcnt, 0, sizeof(int) * (size_t)sp_rounds_df_words((int)sp.rounds.size()), st));
    if (sp.npad_tail > 0)  // the dataflow factor's ready words start below every epoch
        M3S_HIP_CHECK(hipMemsetAsync(chol_ready_ptr(sp.dptr<double>(sp.o_linv), sp.npad_tail), 0,
                                     chol_ready_bytes(sp.npad_tail), st));
    if (sp.pcg)  // the exchange's tags start below every launch's
        M3S_HIP_CHECK(hipMemsetAsync(sp.dbuf + sp.o_gran, 0, 16 * 4 * (size_t)sp.pcg_nv, st));
    if (n > 0) {
        int* h = reinterpret_cast<int*>(stagings().out.get(sizeof(int) * n));
        M3S_REQUIRE(h != nullptr, "gauss_newton: pinned host allocation failed");
        for (size_t k = 0; k < parts.size(); k++)
            if (len(k) > 0) std::memcpy(h + *offs[k], parts[k]->data(), sizeof(int) * len(k));
        int* hr = h + sp.i_rounds;
        for (const SpRound& R : sp.rounds) {
            const int v[8] = {R.node_begin, R.nnodes, R.tbeg, R.nbt, R.rbeg, R.nrt, R.wbeg, R.wcount};
            std::memcpy(hr, v, sizeof(v));
            hr += 8;
        }
        M3S_HIP_CHECK(stagings().out.upload(sp.dbuf + sp.o_int, reinterpret_cast<const char*>(h), sizeof(int) * n, st));
        M3S_HIP_CHECK(stagings().out.mark(st));  // no host sync: the staging buffer outlives the copy
    }
    return M3S_OK;
}

// M3S_GN_ORDER_*: the args field, else env M3S_GN_ORDER=reference|fast, else fast
int gn_order(const m3s_gn_args& a) {
    if (a.order == M3S_GN_ORDER_FAST || a.order == M3S_GN_ORDER_REFERENCE) return a.order;
    static const int env = [] {
        const char* e = getenv("M3S_GN_ORDER");
        if (e && (!strcmp(e, "reference") || !strcmp(e, "ref") || !strcmp(e, "2"))) return (int)M3S_GN_ORDER_REFERENCE;
        return (int)M3S_GN_ORDER_FAST;
    }();
    return env;
}

int validate(const m3s_gn_args& a) {
    M3S_REQUIRE(a.order >= M3S_GN_ORDER_DEFAULT && a.order <= M3S_GN_ORDER_REFERENCE,
                "gauss_newton: bad summation order %d", a.order);
    M3S_REQUIRE(a.mode == M3S_GN_POINTS || a.mode == M3S_GN_RAYS || a.mode == M3S_GN_CALIB,
                "gauss_newton: bad mode %d", a.mode);
    M3S_REQUIRE(a.contract == M3S_CONTRACT_NVCC || a.contract == M3S_CONTRACT_OFF ||
                    a.contract == M3S_CONTRACT_NVCC_RIGHT,
                "gauss_newton: unknown contraction convention %d", a.contract);
    M3S_REQUIRE(a.N >= 1 && a.HW >= 1, "gauss_newton: need N >= 1 poses and HW >= 1 points");
    M3S_REQUIRE(a.E_total >= 0 && a.E_local >= 0 && a.edge_offset >= 0 &&
                    a.edge_offset + a.E_local <= a.E_total,
                "gauss_newton: bad edge range");
    M3S_REQUIRE(a.HW < ((int64_t)1 << 31) && a.E_local < (1 << 30),
                "gauss_newton: sizes exceed int32 indexing");
    // the dense solver (M3S_SOLVER_DENSE=1, diagnostics) factors the whole system; the sparse
    // solvers check their dense core against the same limit after planning (run())
    if (env_int("M3S_SOLVER_DENSE", 0) != 0 && a.order != M3S_GN_ORDER_REFERENCE)
        M3S_REQUIRE(7 * (a.N - 1) <= kMaxNpad,
                    "gauss_newton: %lld poses exceed the dense solve limit (%d unknowns)",
                    (long long)a.N, kMaxNpad);
    M3S_REQUIRE(a.mode != M3S_GN_CALIB || (a.K != nullptr && a.width > 0 && a.height > 0),
                "gauss_newton_calib: K / image size required");
    M3S_REQUIRE(a.Twc && a.Xs && a.Cs && a.dx, "gauss_newton: null pointer");
    if (a.E_total > 0) M3S_REQUIRE(a.ii && a.jj, "gauss_newton: null ii/jj");
    if (a.E_local > 0) M3S_REQUIRE(a.idx && a.valid && a.Q, "gauss_newton: null edge data");
    if (a.idx_b || a.valid_b || a.Q_b) {
        M3S_REQUIRE(a.idx_b && a.valid_b && a.Q_b, "gauss_newton: incomplete second edge half");
        M3S_REQUIRE(a.E_a >= 0 && a.E_a <= a.E_local, "gauss_newton: bad edge split E_a = %lld",
                    (long long)a.E_a);
    }
    const size_t need = make_layout(a.mode, a.N, a.HW, a.E_total, a.E_local).total;
    M3S_REQUIRE(a.ws != nullptr && a.ws_bytes >= need,
                "gauss_newton: workspace too small (%zu < %zu bytes)", a.ws_bytes, need);
    return M3S_OK;
}

Plan& tls_plan() {
    static thread_local Plan p;
    return p;
}
SparsePlan& tls_sparse_plan() {
    static thread_local SparsePlan sp;
    return sp;
}

struct Ctx {
    bool need_slotmap = false;  // dense solver / debug system: upload the slot table
    bool packed = false;  // per-call packed stream (gn_pack_kernel) feeds the accumulate
    bool compact = false;  // ... holding only the live points (gn_pack_compact_kernel)
    bool ref_order = false;  // M3S_GN_ORDER_REFERENCE: gn_refacc.hip accumulate + assembly
    bool pack_issued = false;  // prepare_iterations already enqueued (setup's early pack)
    bool acc_enqueued = false;  // iteration 0's accumulate enqueued before the planning
    bool gathered = false;      // ... and, edge-sharded, its records' all-gather too
    // the first accumulate of the call builds the packed records (no separate pack pass)
    bool first_pack = false;
    RefParams R;
    Layout L;
    // the host plans, per thread across calls: their lists keep their capacity (fresh
    // allocations of this size cost a page fault per 4 KiB on every call; sparse_plan.h)
    Plan& plan = tls_plan();
    SparsePlan& sp = tls_sparse_plan();
    AccParams P;
    EdgeSrc es{};
    bool vec;
    char* ws;
    hipStream_t st = nullptr;
    // dense solver / debug system: (npad+64) x npad f64 matrix (RHS as a border row), its 64x64
    // tile inverses and the (npose x npose) slot table, one stream-ordered allocation
    char* dyn = nullptr;
    size_t o_dense = 0, o_linv = 0, o_slot = 0;
    double* eall = nullptr;  // Plan::gather: every rank's edge records (granks x gchunk)
    // where this rank's accumulate writes its f64 edge records, and what the assembly reads
    double* eblk() const {
        return eall ? eall + (size_t)plan.grank * plan.gchunk * kEdgeBlk : at<double>(L.edgeblk);
    }
    const double* eblk_all() const { return eall ? eall : at<double>(L.edgeblk); }
    int chol_epoch = 0;  // dataflow factorisations enqueued in this call (chol_df.hip ready words)
    int pcg_launches = 0;  // PCG launches enqueued in this call (their exchange tags)
    // an M refresh enqueued on the side stream that the call's stream has not waited for yet
    bool inv_pending = false;
    hipEvent_t inv_done = nullptr;
    bool may_timeout = false;  // a solver with bounded device-side waits ran (kFlagTimeout)
    template <typename T>
    T* at(size_t off) const { return reinterpret_cast<T*>(ws + off); }
    template <typename T>
    T* dyn_at(size_t off) const { return reinterpret_cast<T*>(dyn + off); }
    int alloc_dense(int npad, int npose) {
        size_t off = 0;
        auto take = [&](size_t bytes) {
            size_t o = off;
            off = align_up(off + std::max<size_t>(bytes, 8), 256);
            return o;
        };
        o_dense = take(sizeof(double) * (size_t)(npad + kCholTile) * npad);
        o_linv = take(chol_linv_bytes(npad));
        o_slot = take(sizeof(int) * (size_t)npose * npose);
        M3S_HIP_CHECK(hipMallocAsync((void**)&dyn, off, st));
        M3S_HIP_CHECK(hipMemsetAsync(chol_ready_ptr(dyn_at<double>(o_linv), npad), 0, chol_ready_bytes(npad), st));
        return M3S_OK;
    }
    Ctx() { sp.reset(); }  // (no earlier call's plan survives into this one)
    Ctx(const Ctx&) = delete;
    Ctx& operator=(const Ctx&) = delete;
    // every return path of a call releases its per-call buffers (stream-ordered)
    ~Ctx() {
        // (an error path may leave an M refresh in flight on the side stream: it reads the plan
        // buffer, so the call's stream waits for it before the buffer is released)
        if (inv_pending && inv_done) (void)hipStreamWaitEvent(st, inv_done, 0);
        if (sp.dbuf) (void)hipFreeAsync(sp.dbuf, st);
        sp.dbuf = nullptr;
        if (dyn) (void)hipFreeAsync(dyn, st);
        if (eall) (void)hipFreeAsync(eall, st);
    }
};

int prepare_iterations(const m3s_gn_args& a, Ctx& c);

// early_pack: launch the packed stream (prepare_iterations) as soon as the edge lists are on
// the device, before the host builds the accumulate schedule
// The per-call solver buffers come from the device's default stream-ordered pool
// (hipMallocAsync); its default release threshold (0) hands freed memory back to the driver at
// every synchronisation -- and the call synchronises once on its edge lists -- so every call
// mapped its buffers again (~10 MB with the PCG's M and factor copy).  M3S_POOL_KEEP_MB (default
// 1024): keep that much cached in the pool.  Once per device; the pool is the HIP runtime's (not
// torch's caching allocator).
void keep_pool() {
    static std::mutex mu;
    static bool done[64] = {false};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return;
    std::lock_guard<std::mutex> lk(mu);
    if (done[dev]) return;
    done[dev] = true;
    const long mb = env_int("M3S_POOL_KEEP_MB", 1024);
    if (mb <= 0) return;
    hipMemPool_t pool;
    if (hipDeviceGetDefaultMemPool(&pool, dev) != hipSuccess) return;
    uint64_t thr = (uint64_t)mb << 20;
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
}

int setup(const m3s_gn_args& a, Ctx& c, bool early_pack = false) {
    int rc = validate(a);
    if (rc) return rc;
    keep_pool();
    c.st = (hipStream_t)a.stream;
    c.ws = (char*)a.ws;
    c.L = make_layout(a.mode, a.N, a.HW, a.E_total, a.E_local);
    static const bool prof_host = env_int("M3S_PROF_HOST", 0) != 0;
    const auto s0 = std::chrono::steady_clock::now();
    const Layout& L = c.L;
    AccParams& P = c.P;
    P.s0_inv = 1.0f / a.sigma0;
    P.s1_inv = (a.mode == M3S_GN_POINTS) ? 0.0f : 1.0f / a.sigma1;
    P.C_thresh = a.C_thresh;
    P.Q_thresh = a.Q_thresh;
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
    P.nkf = (int)a.N;
    auto al16 = [](const void* ptr) { return ((uintptr_t)ptr & 15) == 0; };
    const bool two = a.idx_b != nullptr;
    c.es.idx[0] = a.idx;
    c.es.valid[0] = a.valid;
    c.es.Q[0] = a.Q;
    c.es.idx[1] = two ? a.idx_b : a.idx;
    c.es.valid[1] = two ? a.valid_b : a.valid;
    c.es.Q[1] = two ? a.Q_b : a.Q;
    c.es.E_a = two ? (int)a.E_a : (int)a.E_local;
    c.vec = (a.HW % 4 == 0) && al16(a.Xs) && al16(a.Cs) && al16(a.idx) && al16(a.valid) &&
            al16(a.Q) && (!two || (al16(a.idx_b) && al16(a.valid_b) && al16(a.Q_b)));
    // M3S_GN_PACK: 0 never, 1 (default) when the call runs >= 3 iterations, 2 always
    const int pack_mode = env_int("M3S_GN_PACK", 1);
    c.packed = c.vec && a.E_local > 0 && (pack_mode == 2 || (pack_mode == 1 && a.max_iter >= 3));
    // M3S_GN_COMPACT=1: the packed stream holds only the live points (gn_accum.hip).  Off by
    // default: on the bench graphs 80-90 % of the points are live, the accumulate gains 3 %
    // (cfg3) / 13 % (cfg4), and the compacting pack (Xj copies, finiteness gathers) costs more
    // per call than the 10 iterations save
    c.compact = c.packed && env_int("M3S_GN_COMPACT", 0) != 0;
    // calib: the packed records carry the match as its pixel (v << 16 | u), decoded with a mask, a
    // bit-field extract and one 24-bit multiply-add instead of a 64-bit division by W per point
    if (a.mode == M3S_GN_CALIB && (a.width >= 65536 || a.height >= 32768)) c.packed = c.compact = false;
    P.pack_uv = c.packed && a.mode == M3S_GN_CALIB;
    // calib: the packed accumulate reads Xj as its 4-B depth when gn_depth_kernel finds every point
    // on its pixel's ray bit for bit (solve_GN_calib's constrain_points_to_ray; bitwise the same
    // result): 16 instead of 24 B per point-edge.  M3S_GN_RAYCHECK=0 keeps the positional path only.
    P.raycheck = c.packed && !c.compact && a.mode == M3S_GN_CALIB && env_int("M3S_GN_RAYCHECK", 1) != 0;

    c.ref_order = gn_order(a) == M3S_GN_ORDER_REFERENCE;
    if (c.ref_order) {
        c.packed = false;  // the reference-order kernel reads the reference's tensors
        RefParams& R = c.R;
        R.s0_inv = (float)(1.0 / (double)a.sigma0);  // `const float sigma_*_inv = 1.0/sigma_*`
        R.s1_inv = (a.mode == M3S_GN_POINTS) ? 0.0f : (float)(1.0 / (double)a.sigma1);
        R.C_thresh = a.C_thresh;
        R.Q_thresh = a.Q_thresh;
        R.z_eps = a.z_eps;
        R.width = a.width > 0 ? a.width : 1;
        R.height = a.height;
        R.pixel_border = a.pixel_border;
        R.HW = a.HW;
        R.variant = env_int("M3S_GN_REF_VARIANT", 0);  // diagnostics
        R.contract = a.contract;
    }
    // the per-call passes that need no edge lists (the keyframes' confidence pass, calib's depth
    // arrays) and the call's device flags are enqueued right after the edge-list copies: they run
    // while the host waits for the copies and plans (the lists upload below no longer carries
    // the flags / cok)
    int* dflags = c.at<int>(L.flags);
    int* dcok = c.at<int>(L.cok);
    auto pre_pass = [&]() -> int {
        M3S_HIP_CHECK(launch_gn_init(c.st, dflags, P.raycheck ? 0 : 1, dcok, a.N));
        if (c.packed)
            M3S_HIP_CHECK(launch_pack_pre(c.st, a.Xs, a.N, a.Cs, P, !c.compact ? dcok : nullptr,
                                          a.mode == M3S_GN_CALIB ? c.at<float>(L.zs) : nullptr, dflags,
                                          a.mode == M3S_GN_CALIB ? a.K : nullptr));
        return M3S_OK;
    };
    // M3S_PREPASS=0 (A/B): the passes after the host's stream wait instead (cfg3 +0.6 % with
    // them before it, two interleaved pairs on one box: profiles/r05_u_prepass/)
    static const bool prepass_early = env_int("M3S_PREPASS", 1) != 0;
    rc = build_plan(a, c.st, c.plan, prepass_early ? pre_pass : std::function<int()>());
    if (!rc && !prepass_early) rc = pre_pass();
    if (rc) return rc;
    if (c.plan.gather)
        M3S_HIP_CHECK(hipMallocAsync((void**)&c.eall,
                                     sizeof(double) * kEdgeBlk * (size_t)c.plan.granks * c.plan.gchunk, c.st));
    const auto s1 = std::chrono::steady_clock::now();
    const Plan& p = c.plan;
    P.fx = p.K[0];
    P.fy = p.K[1];
    P.cx = p.K[2];
    P.cy = p.K[3];
    if (c.ref_order) {
        c.R.fx = p.K[0];
        c.R.fy = p.K[1];
        c.R.cx = p.K[2];
        c.R.cy = p.K[3];
    }
    // the workspace's plan integers (ii_loc .. sched, one contiguous span of the layout) as an
    // image in pinned memory: the edge lists / CSR lists first (what the pack reads), then the
    // accumulate's task records (built while the GPU packs)
    const size_t ntask = (size_t)a.E_local * L.nchunks;
    const size_t lo = L.ii_loc, hi = L.sched;
    const size_t nslot = c.need_slotmap ? p.slotmap.size() : 0;
    if (c.need_slotmap) {
        rc = c.alloc_dense(L.npad, (int)std::max<int64_t>(a.N - 1, 0));
        if (rc) return rc;
    }
    char* h = stagings().ws.get(hi - lo + sizeof(int) * nslot);
    M3S_REQUIRE(h != nullptr, "gauss_newton: pinned host allocation failed");
    auto put = [&](size_t off, const std::vector<int>& v) {
        if (!v.empty()) std::memcpy(h + (off - lo), v.data(), sizeof(int) * v.size());
    };
    put(L.ii_loc, p.ii_loc);
    put(L.jj_loc, p.jj_loc);
    put(L.blk_ptr, p.blk_ptr);
    put(L.blk_ent, p.blk_ent);
    put(L.blk_ref, p.blk_ref);
    put(L.grad_ptr, p.grad_ptr);
    put(L.grad_ent, p.grad_ent);
    std::memset(h + (L.ecnt - lo), 0, sizeof(int) * (size_t)a.E_local);  // (the kernel re-zeroes them)
    SchedGroups G;
    build_schedule_order(p.ii_loc, p.jj_loc, (int)std::max<int64_t>(a.N, 1), reinterpret_cast<int*>(h + (L.sorder - lo)), G);
    M3S_HIP_CHECK(stagings().ws.upload(c.ws + lo, h, L.sched - lo, c.st));
    // the accumulate's task records carry the edge's keyframes: one load, not three levels
    M3S_HIP_CHECK(launch_sched_expand(c.st, c.at<int>(L.sorder), c.at<int>(L.ii_loc), c.at<int>(L.jj_loc), L.nchunks,
                                      G, (int64_t)ntask, c.at<int>(L.sched)));
    // M3S_GN_PACK_FIRST (default 1): a call's first accumulate builds the packed records
    // from the reference's inputs itself (gn_accum_packed_kernel<..., FIRST>): 13 B read + 8 B
    // written per point-edge inside the first iteration instead of a separate 21-B pack pass
    // followed by the first iteration's 8-B record reads (run() only: its early pack)
    c.first_pack = early_pack && c.packed && !c.compact && !c.ref_order && a.max_iter > 0 &&
                   env_int("M3S_GN_PACK_FIRST", 1) != 0;
    if (early_pack) {
        rc = prepare_iterations(a, c);
        if (rc) return rc;
        c.pack_issued = true;
    }
    const auto s2 = std::chrono::steady_clock::now();
    if (nslot) {  // the dense (npose x npose) slot table
        std::memcpy(h + (hi - lo), p.slotmap.data(), sizeof(int) * nslot);
        M3S_HIP_CHECK(hipMemcpyAsync(c.dyn + c.o_slot, h + (hi - lo), sizeof(int) * nslot,
                                     hipMemcpyHostToDevice, c.st));
    }
    M3S_HIP_CHECK(stagings().ws.mark(c.st));
    if (prof_host) {
        auto us = [](std::chrono::steady_clock::time_point x, std::chrono::steady_clock::time_point y) {
            return std::chrono::duration<double, std::micro>(y - x).count();
        };
        fprintf(stderr, "gn host: build_plan %.0f us (of which copies + sync %.0f us), params+lists+schedule+pack "
                "%.0f us, rest %.0f us\n", us(s0, s1), g_plan_sync_us, us(s1, s2), us(s2, std::chrono::steady_clock::now()));
    }
    return M3S_OK;
}

// Once per call, before the iterations: the packed stream (and calib depth array).
int prepare_iterations(const m3s_gn_args& a, Ctx& c) {
    if (!c.packed) return M3S_OK;
    const Layout& L = c.L;
    M3S_HIP_CHECK(launch_pack(a.mode, c.st, (int)a.E_local, a.Xs, a.N, a.Cs, c.at<int>(L.ii_loc),
                              c.at<int>(L.jj_loc), c.es, c.P, c.at<int>(L.cok), c.at<int4>(L.pack),
                              c.compact ? c.at<float>(L.packx) : nullptr, c.at<int>(L.pcnt),
                              c.at<int>(L.flags), c.first_pack));
    return M3S_OK;
}

int enqueue_accumulate(const m3s_gn_args& a, Ctx& c);
int enqueue_assembly(const m3s_gn_args& a, Ctx& c);

// accumulate + edge reduce + compact (+ all-reduce): the system of one iteration
int enqueue_system(const m3s_gn_args& a, Ctx& c) {
    const Layout& L = c.L;
    int* flags = c.at<int>(L.flags);
    const int npose_r = (int)(a.N - 1);
    if (c.ref_order) {
        // the reference kernels' order (gn_refacc.hip), then the block system from the lower
        // triangle of the reference's matrix (the sparse solvers' format)
        M3S_REQUIRE(c.sp.enabled, "gauss_newton: the reference order needs the block-sparse solver");
        g_prof.mark(c.st, true);
        M3S_HIP_CHECK(launch_accum_ref(a.mode, (int)a.E_local, c.st, a.Twc, a.Xs, a.Cs,
                                       c.at<int>(L.ii_loc), c.at<int>(L.jj_loc), c.es,
                                       c.R, c.at<float>(L.edgeblk), flags));
        g_prof.mark(c.st, true);
        SparsePlan& sp = c.sp;
        double* sys = sp.dptr<double>(sp.o_sys);
        M3S_HIP_CHECK(launch_assemble_ref(c.st, c.at<float>(L.edgeblk), c.at<int>(L.blk_ptr),
                                          c.at<int>(L.blk_ref), c.at<int>(L.grad_ptr),
                                          c.at<int>(L.grad_ent), c.plan.nblk, sp.nblocks, npose_r,
                                          sp.bpad, sys, flags));
        if (a.comm) {
            const size_t count = (size_t)sp.bpad + (size_t)c.plan.nblk * 49;
            int rc = comm_allreduce_sum_f64(a.comm, sys, count, c.st);
            if (rc) return rc;
        }
        return M3S_OK;
    }
    if (!c.acc_enqueued) {
        int rc = enqueue_accumulate(a, c);
        if (rc) return rc;
    }
    c.acc_enqueued = false;
    return enqueue_assembly(a, c);
}

// the accumulate (+ edge reduce) of one iteration: needs no elimination plan, so iteration 0's
// is enqueued before the host builds it
int enqueue_accumulate(const m3s_gn_args& a, Ctx& c) {
    const Layout& L = c.L;
    int* flags = c.at<int>(L.flags);
    if (a.E_local > 0) {
        g_prof.mark(c.st, true);
        const dim3 grid((unsigned)(L.nchunks * a.E_local));
        // M3S_GN_FUSE_REDUCE=1 (default): the packed accumulate's last workgroup per edge does
        // the edge reduce (no separate launch); 0: gn_edge_reduce_kernel
        const bool fuse_reduce = env_int("M3S_GN_FUSE_REDUCE", 1) != 0;
        const bool fused = c.packed && fuse_reduce;
        const bool was_first = c.packed && c.first_pack;
        if (c.packed) {
            M3S_HIP_CHECK(launch_accum_packed(a.mode, grid, c.st, a.Twc, a.Xs, c.at<float>(L.zs),
                                              c.at<int>(L.ii_loc), c.at<int>(L.jj_loc),
                                              c.at<int4>(L.pack), c.P, c.at<int4>(L.sched),
                                              c.at<float>(L.partials), flags,
                                              c.compact ? c.at<float>(L.packx) : nullptr,
                                              c.at<int>(L.pcnt), fused ? c.at<int>(L.ecnt) : nullptr,
                                              c.eblk(), c.first_pack ? &c.es : nullptr,
                                              a.Cs, c.at<int>(L.cok)));
            c.first_pack = false;  // the records exist from here on
        } else
            M3S_HIP_CHECK(launch_accum(a.mode, c.vec, grid, c.st, a.Twc, a.Xs, a.Cs,
                                       c.at<int>(L.ii_loc), c.at<int>(L.jj_loc), c.es, c.P,
                                       c.at<int4>(L.sched), c.at<float>(L.partials),
                                       flags));
        g_prof.mark(c.st, true, was_first);
        if (!fused)
            M3S_HIP_CHECK(launch_edge_reduce((int)a.E_local, c.st, c.at<float>(L.partials), L.nchunks,
                                             a.Twc, c.at<int>(L.ii_loc), c.eblk(), flags));
    }
    return M3S_OK;
}

// edge blocks -> the solver's system (+ the all-reduce)
int enqueue_assembly(const m3s_gn_args& a, Ctx& c) {
    const Layout& L = c.L;
    int* flags = c.at<int>(L.flags);
    const int npose = (int)(a.N - 1);
    if (c.plan.gather && !c.gathered) {
        // every rank's edge records, then the assembly of ALL edges in edge order (no all-reduce)
        int rc = comm_allgather_f64(a.comm, c.eall, (size_t)c.plan.gchunk * kEdgeBlk, c.st);
        if (rc) return rc;
    }
    c.gathered = false;
    const bool reduce = a.comm && !c.plan.gather;
    if (c.sp.enabled) {
        // block format for the sparse solves, in the solver's buffer
        SparsePlan& sp = c.sp;
        double* sys = sp.dptr<double>(sp.o_sys);
        M3S_HIP_CHECK(launch_assemble(c.st, c.eblk_all(), c.at<int>(L.blk_ptr),
                                      c.at<int>(L.blk_ent), c.at<int>(L.grad_ptr),
                                      c.at<int>(L.grad_ent), c.plan.nblk, sp.nblocks, npose, sp.bpad,
                                      sys, flags));
        if (reduce) {
            const size_t count = (size_t)sp.bpad + (size_t)c.plan.nblk * 49;
            int rc = comm_allreduce_sum_f64(a.comm, sys, count, c.st);
            if (rc) return rc;
        }
        return M3S_OK;
    }
    M3S_HIP_CHECK(launch_compact(c.st, c.eblk_all(), c.at<int>(L.blk_ptr),
                                 c.at<int>(L.blk_ent), c.at<int>(L.grad_ptr),
                                 c.at<int>(L.grad_ent), c.plan.nblk, npose,
                                 c.at<double>(L.compact), flags));
    if (reduce) {
        const size_t count = (size_t)c.plan.nblk * 28 + (size_t)npose * 7;
        int rc = comm_allreduce_sum_f64(a.comm, c.at<double>(L.compact), count, c.st);
        if (rc) return rc;
    }
    return M3S_OK;
}

// M3S_SOLVE_DEBUG: gn_solve_kernel writes its phase clocks to a device buffer; the driver
// waits for the launch and prints them (debug runs only: the wait serialises the call)
constexpr int kSolveDbgWords = kSolveDbgCycles + 1;
unsigned long long* solve_dbg_buffer() {
    static unsigned long long* p = nullptr;
    if (p == nullptr && hipMalloc(&p, sizeof(unsigned long long) * kSolveDbgWords) != hipSuccess) p = nullptr;
    if (p != nullptr) (void)hipMemset(p, 0, sizeof(unsigned long long) * kSolveDbgWords);
    return p;
}
hipError_t launch_gn_solve_dbg(hipStream_t st, const SolveArgs& S) {
    hipError_t e = launch_gn_solve(st, S);
    if (e != hipSuccess || !S.debug || S.dbg == nullptr) return e;
    unsigned long long h[kSolveDbgWords];
    e = hipMemcpyAsync(h, S.dbg, sizeof(h), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e == hipSuccess) print_solve_debug(h);
    return e;
}

// fallback: the direct solve enqueued behind a PCG launch (it runs only when the PCG did not
// converge; otherwise each of its launches returns at once, ~4-5 us apiece)
int enqueue_solve(const m3s_gn_args& a, Ctx& c, bool fallback = false) {
    const Layout& L = c.L;
    const int npose = (int)(a.N - 1);
    int* flags = c.at<int>(L.flags);
    if (!c.sp.enabled) {
        c.may_timeout = true;  // dense factorisation: chol_df's ready waits
        M3S_HIP_CHECK(launch_solve(c.st, c.at<double>(L.compact), c.dyn_at<int>(c.o_slot), c.plan.nblk,
                                   npose, 7 * npose, L.npad, c.dyn_at<double>(c.o_dense),
                                   c.dyn_at<double>(c.o_linv), c.at<double>(L.x), flags, ++c.chol_epoch));
        return M3S_OK;
    }
    SparsePlan& sp = c.sp;
    SolveArgs S{};
    S.npose = npose;
    S.b = sp.dptr<double>(sp.o_sys);
    S.A = S.b + sp.bpad;
    S.y = sp.dptr<double>(sp.o_y);
    S.Lstore = sp.dptr<double>(sp.o_L);
    S.W = sp.dptr<double>(sp.o_W);
    S.Lg = sp.dptr<double>(sp.o_Lg);
    S.x = c.at<double>(L.x);
    S.meta = sp.iptr(0);
    S.nmeta = (int)sp.nints;
    S.meta_lds = solve_lds_bytes(S.nmeta) <= (size_t)kSolveMaxLds && env_int("M3S_SOLVE_META_LDS", 1);
    S.o_rounds = (int)sp.i_rounds;
    S.o_nodes = (int)sp.i_nodes;
    S.o_fptr = (int)sp.i_fptr;
    S.o_fronts = (int)sp.i_fronts;
    S.o_tg = (int)sp.i_tg;
    S.o_tc = (int)sp.i_tc;
    S.o_rtg = (int)sp.i_rtg;
    S.o_rc = (int)sp.i_rc;
    S.o_tail = (int)sp.i_tail;
    S.o_tmap = (int)sp.i_tmap;
    S.nrounds = (int)sp.rounds.size();
    S.zero_blk = sp.zero_blk;
    S.ntail = sp.ntail;
    S.Twc = a.Twc;
    S.dx = a.dx;
    S.N = (int)a.N;
    S.delta_thresh = a.delta_thresh;
    S.flags = flags;
    S.debug = env_int("M3S_SOLVE_DEBUG", 0);
    S.dbg = S.debug ? solve_dbg_buffer() : nullptr;
    S.contract = a.contract;
    if (S.debug) {
        static int printed = 0;
        if (printed++ == 0) {
            fprintf(stderr, "solve plan: npose %d nblocks %d (real %d) nW %d ntail %d nints %zu meta_lds %d fused %d\n",
                    npose, sp.nblocks, c.plan.nblk, sp.nW, sp.ntail, sp.nints, S.meta_lds, (int)sp.fused_tail);
            for (const SpRound& R : sp.rounds) {
                int ncontrib = 0, maxc = 0;
                for (int t = 0; t < R.nbt; t++) {
                    const int* T = sp.fused ? &sp.tg[3 * (R.tbeg + t)]
                                            : &sp.inl[(size_t)kSpRec * (R.tbeg + R.rbeg + t)];
                    const int k = T[2] - T[1];
                    ncontrib += k;
                    maxc = std::max(maxc, k);
                }
                int nf = 0;
                for (int q = R.node_begin; q < R.node_begin + R.nnodes; q++) nf += sp.fptr[q + 1] - sp.fptr[q];
                fprintf(stderr, "  round: nodes %d fronts %d block targets %d (contrib %d, max %d) rhs targets %d\n",
                        R.nnodes, nf, R.nbt, ncontrib, maxc, R.nrt);
            }
        }
    }
    if (sp.fused) {
        // one launch: rounds, in-register dense tail, back-substitution, retraction
        if (env_int("M3S_SOLVE_SPLIT", 1) && S.nrounds > 0) {
            // the rounds by a wider workgroup (memory latency overlapped across 8 waves), then
            // the in-register tail + back-substitution + retraction
            S.do_fwd = 1;
            S.do_tail = S.do_back = 0;
            M3S_HIP_CHECK(launch_gn_solve_dbg(c.st, S));
            S.do_fwd = 0;
            S.do_tail = S.do_back = 1;
            M3S_HIP_CHECK(launch_gn_solve_dbg(c.st, S));
            return M3S_OK;
        }
        S.do_fwd = S.do_tail = S.do_back = 1;
        M3S_HIP_CHECK(launch_gn_solve_dbg(c.st, S));
        return M3S_OK;
    }
    // multi-launch: one launch per round phase, the tail by the tiled dense Cholesky
    double* A = S.A;
    double* b = S.b;
    double* y = S.y;
    double* Ls = S.Lstore;
    double* W = S.W;
    double* x = S.x;
    // M3S_SOLVE_COOP: 0 (default) = one launch per round; 1 = all rounds (+ the hybrid core's
    // fill) in one launch with an own grid barrier and agent-coherent block accesses
    // (gn_sparse.hip); 2 = the same as a cooperative launch with cooperative-groups grid sync.
    // Measured (cfg3 solve per iteration): 0.24 ms per-round launches, 0.32 ms own barrier,
    // 0.43 ms cooperative groups -- in-kernel a round's chain is ~4 us, but coherent (MALL)
    // block traffic + write-through + the barrier cost as much as the ~5 us launch overhead saved
    static const int coop_mode = env_int("M3S_SOLVE_COOP", 0);
    // M3S_PCG_FALLBACK_COOP (default 1): a PCG iteration's fallback runs its rounds (and the
    // hybrid core's fill) as the one all-rounds launch -- slower when it runs, but a converged
    // PCG skips one launch instead of one per round (cfg3: 5 round launches + the fill)
    static const bool fb_coop = env_int("M3S_PCG_FALLBACK_COOP", 0) != 0;
    // M3S_SOLVE_DF: 1 (default) = a PCG iteration's fallback runs its rounds (and the hybrid core's
    // fill) as ONE plain launch of ticketed targets (sp_rounds_df_kernel: no co-residency); 2 =
    // every direct solve does; 0 = one launch per round everywhere
    static const int df_mode = env_int("M3S_SOLVE_DF", 1);
    const bool df = coop_mode == 0 && !(fallback && fb_coop) && (df_mode == 2 || (df_mode == 1 && fallback));
    const bool coop = coop_mode != 0 || (fallback && fb_coop) || df;
    if (coop) {
        c.may_timeout = true;  // grid barriers
        SpCoopArgs ca{};
        ca.inl = sp.iptr(sp.i_inl);
        ca.tc3 = sp.iptr(sp.i_tc3);
        ca.rc4 = sp.iptr(sp.i_rc4);
        ca.rounds = sp.iptr(sp.i_rounds);
        ca.tmap = sp.iptr(sp.i_tmap);
        ca.tail = sp.iptr(sp.i_tail);
        ca.A = A;
        ca.b = b;
        ca.Lstore = Ls;
        ca.W = W;
        ca.y = y;
        // (the ticketed launch fills the multi plan's core too: one launch less behind a PCG)
        ca.Hd = (sp.hybrid || df) && sp.ntail > 0 ? sp.dptr<double>(sp.o_dense) : nullptr;
        ca.flags = flags;
        ca.nrounds = (int)sp.rounds.size();
        ca.ntail = (sp.hybrid || df) ? sp.ntail : 0;
        ca.npad = sp.npad_tail;
        ca.coop = coop_mode == 2;
        if (df)
            M3S_HIP_CHECK(launch_sp_rounds_df(c.st, ca, sp.dptr<int>(sp.o_dfcnt)));
        else
            M3S_HIP_CHECK(launch_sp_rounds_coop(c.st, ca));
    } else {
        for (const SpRound& R : sp.rounds)
            M3S_HIP_CHECK(launch_sp_round(c.st, sp.iptr(sp.i_inl), R.tbeg + R.rbeg, R.nbt, R.nrt,
                                          sp.iptr(sp.i_tc3), sp.iptr(sp.i_rc4), A, b, Ls, W, y, flags));
    }
    // M3S_HYB_CORE=1 (default): the hybrid's dense core (<= kHybDfTailMax = 64 poses, 36 by
    // default) is factored and solved by the dataflow launch (chol_df.hip: batch-cyclic tile
    // factor, ~100 ns per column on the pivot chain, back-substitution in the same launch)
    // instead of gn_solve's in-register pose steps (~330-430 ns per column); gn_solve then only
    // back-substitutes through the rounds and retracts.  0 (or the cooperative rounds launch):
    // the in-register core, <= 27 poses.  The planner read the switch (hyb_core_df) and sized the
    // core for it: the plan carries the choice.
    const bool core_df = sp.core_df;
    if (sp.hybrid && core_df && sp.ntail > 0) {
        c.may_timeout = true;  // chol_df's bounded waits
        if (!coop)  // (the all-rounds launch filled the core)
            M3S_HIP_CHECK(launch_sp_tail_fill(c.st, A, b, sp.iptr(sp.i_tmap), sp.iptr(sp.i_tail), sp.ntail,
                                              sp.npad_tail, sp.dptr<double>(sp.o_dense), flags));
        M3S_HIP_CHECK(launch_dense_factor_solve(c.st, sp.npad_tail, sp.dptr<double>(sp.o_dense),
                                                sp.dptr<double>(sp.o_linv), sp.dptr<double>(sp.o_xd), flags,
                                                ++c.chol_epoch));
        S.xd = sp.dptr<double>(sp.o_xd);  // gn_solve reads the core's x in its dense order
        S.Hd = nullptr;
        S.nmeta = (int)sp.nints_back;
        S.meta_lds = 1;
        S.do_fwd = 0;
        S.do_tail = 0;
        S.do_back = 1;
        S.x_tail_global = 1;
        M3S_HIP_CHECK(launch_gn_solve_dbg(c.st, S));
        return M3S_OK;
    }
    if (sp.hybrid) {
        M3S_REQUIRE(sp.fused_tail, "gauss_newton: a %d-pose hybrid core exceeds the in-register factorisation",
                    sp.ntail);
        // the <= 27-pose core in registers, the back-substitution through the rounds and the
        // retraction: one single-workgroup launch (gn_solve.hip) reading the plan prefix; the
        // core is first laid out densely by a many-workgroup fill (one CU gathering it block by
        // block took ~28 us) -- inside the cooperative launch, or its own launch
        // M3S_SOLVE_GATHER=1 (A/B): no fill launch, the core gathers its tiles from the blocks
        static const bool gather = env_int("M3S_SOLVE_GATHER", 0) != 0;
        if (!coop && !gather)
            M3S_HIP_CHECK(launch_sp_tail_fill(c.st, A, b, sp.iptr(sp.i_tmap), sp.iptr(sp.i_tail),
                                              sp.ntail, sp.npad_tail, sp.dptr<double>(sp.o_dense), flags));
        S.Hd = sp.ntail > 0 && !gather ? sp.dptr<double>(sp.o_dense) : nullptr;
        S.npad_h = sp.npad_tail;
        S.nmeta = (int)sp.nints_back;
        S.meta_lds = 1;
        S.do_fwd = 0;
        S.do_tail = S.do_back = 1;
        M3S_HIP_CHECK(launch_gn_solve_dbg(c.st, S));
        return M3S_OK;
    }
    if (sp.ntail > 0) c.may_timeout = true;  // the core's dataflow factorisation (chol_df)
    M3S_HIP_CHECK(launch_sp_tail(c.st, A, b, sp.iptr(sp.i_tmap), sp.iptr(sp.i_tail), sp.ntail,
                                 sp.npad_tail, sp.dptr<double>(sp.o_dense), sp.dptr<double>(sp.o_linv),
                                 sp.dptr<double>(sp.o_xd), x, flags, ++c.chol_epoch, !df));
    for (auto it = sp.rounds.rbegin(); it != sp.rounds.rend(); ++it)
        M3S_HIP_CHECK(launch_sp_back(c.st, it->nnodes, sp.iptr(sp.i_nodes), sp.iptr(sp.i_fptr),
                                     sp.iptr(sp.i_fronts), it->node_begin, Ls, W, y, x, flags));
    return M3S_OK;
}

// ---- the lagged-factor PCG (gn_pcg.hip) ----
// From iteration `from` on, the step may be solved by CG preconditioned with the inverse of
// iteration (from - lag)'s system, which that iteration's direct factorisation provides
// (sp_inverse_kernel); the direct solve stays enqueued behind every PCG launch as its fallback and
// returns at once when the PCG converged.  Plans whose factor the inverse reads: elimination
// rounds by sp_round_kernel and a chol_df core (the hybrid with M3S_HYB_CORE=1, the multi plan);
// not the single-workgroup solve, the reference-order mode, the all-rounds launch or the dense
// solver.
//   from (M3S_PCG_FROM, default by the core's size): 3 when the direct solve's dense core has >= 8
//     tile columns -- its factorisation chain (~14 us per column on one CU) is what the iteration
//     waits for, and M = A_1^-1 takes 4 CG steps (cfg4: solve 0.27 -> 0.09 ms); 4 below that --
//     the direct solve is short (cfg3, 4 columns: 0.116 ms) and the 8 direct launches behind a
//     PCG (its fallback, ~4-5 us each even when they return at once) leave room only for M =
//     A_2^-1's 4 steps (0.077 ms), not A_1^-1's 6 (0.094 ms: no net gain).
//   lag (M3S_PCG_LAG, default 2): with lag 1 the inverse (~0.75 ms alone on cfg4, ~2.7 ms beside an
//     accumulate that fills the chip: rocprofv3 trace r06_l) runs over one accumulate and the
//     first PCG waits ~0.7 ms for it; with lag 2 it has an accumulate, a direct solve and
//     another accumulate, and reads a copy of that iteration's factor (the next direct solve
//     overwrites the live one).  Refreshes after a PCG that fell back use lag 1 (the next PCG
//     waits for them).
int pcg_from_for(int tiles) {
    const int v = env_int("M3S_PCG_FROM", 0);
    return v > 0 ? v : (tiles >= 8 ? 3 : 4);
}
int pcg_lag_for(int from) { return std::max(1, std::min(from, env_int("M3S_PCG_LAG", 2))); }
// M3S_GN_PCG: 0 off; 1 (default) on every plan above whose core has >= M3S_PCG_MIN_TILES (1) tile
// columns; 2 always.
void choose_pcg(const m3s_gn_args& a, const Ctx& c, const Plan& plan, int npose, SparsePlan& sp) {
    sp.pcg = false;
    const int n = 7 * npose;
    const int mode = env_int("M3S_GN_PCG", 1);
    const int min_tiles = env_int("M3S_PCG_MIN_TILES", 1);
    const int tiles = sp.npad_tail / kCholTile;
    sp.pcg_from = pcg_from_for(tiles);
    sp.pcg_lag = pcg_lag_for(sp.pcg_from);
    if (mode == 0 || (mode == 1 && tiles < min_tiles) || c.ref_order || !sp.enabled || sp.fused ||
        (sp.hybrid && !sp.core_df) || env_int("M3S_SOLVE_COOP", 0) != 0 || a.max_iter <= sp.pcg_from ||
        n > kPcgMaxN || n < 7)
        return;
    // rows of M per workgroup: 12 or 24, the smaller one giving <= M3S_PCG_WG
    // workgroups (default 64) -- or the largest whose f32 rows fit the LDS beside the vector and
    // the product's lists; never more than 240 workgroups (all resident at once, at most one per CU)
    const int wg_cap = std::max(1, env_int("M3S_PCG_WG", 64));
    // the most (row, block) items of a workgroup's rows: R rows span <= R / 7 + 2 poses
    std::vector<int> deg((size_t)npose, 1);
    for (const auto& pr : plan.pairs) {
        deg[pr.first]++;
        deg[pr.second]++;
    }
    const int maxdeg = npose > 0 ? *std::max_element(deg.begin(), deg.end()) : 1;
    auto items = [&](int R) { return 7 * maxdeg * (R / 7 + 2); };
    // (R = threads / 64 or threads / 32: a row's threads stay within one wave, a power of two)
    // M3S_PCG_ONEX (default 1): one exchange per CG step (B = M A's rows in LDS beside M's) where
    // they fit (cfg3's 896 unknowns: yes; cfg4's 1792: no -- two exchanges per step)
    auto pick = [&](bool ox) {
        int R = kPcgThreads / 64;
        auto fits = [&](int r) { return pcg_lds_bytes(n, r, items(r), ox) <= (size_t)kPcgMaxLds && (!ox || r <= kPcgMaxR); };
        if ((n + R - 1) / R > wg_cap && fits(2 * R)) R *= 2;
        return (n + R - 1) / R > 240 || !fits(R) ? 0 : R;
    };
    bool onex = env_int("M3S_PCG_ONEX", 0) != 0 && pick(true) > 0;
    const int R = pick(onex);
    if (R == 0) return;
    if (inverse_lds_bytes(sp.npad_tail) > (size_t)kPcgMaxLds) return;  // M's core rows in LDS
    sp.pcg_nitem = items(R);
    sp.pcg = true;
    sp.pcg_R = R;
    sp.pcg_onex = onex;
    sp.pcg_nwg = (n + R - 1) / R;
    sp.pcg_ldx = (int)align_up((size_t)n, 16);
    sp.pcg_ldt = (int)align_up((size_t)n, 4);
    sp.pcg_nv = pcg_nv(n);
    // the matrix-vector product's lists: per pose its diagonal block, then its pair blocks
    sp.apt.assign((size_t)npose + 1, 0);
    for (const auto& pr : plan.pairs) {
        sp.apt[pr.first + 1]++;
        sp.apt[pr.second + 1]++;
    }
    for (int v = 0; v < npose; v++) sp.apt[v + 1] += sp.apt[v] + 1;
    sp.adj.assign(2 * (size_t)sp.apt[npose], 0);
    std::vector<int> fill(sp.apt.begin(), sp.apt.end() - 1);
    for (int v = 0; v < npose; v++) {
        sp.adj[2 * (size_t)fill[v]] = v;  // (the diagonal block's slot is the pose)
        sp.adj[2 * (size_t)fill[v] + 1] = v;
        fill[v]++;
    }
    for (size_t k = 0; k < plan.pairs.size(); k++) {
        const int x = plan.pairs[k].first, y = plan.pairs[k].second, slot = npose + (int)k;
        sp.adj[2 * (size_t)fill[x]] = slot;
        sp.adj[2 * (size_t)fill[x]++ + 1] = y;
        sp.adj[2 * (size_t)fill[y]] = slot;
        sp.adj[2 * (size_t)fill[y]++ + 1] = x;
    }
}

// snapshot: read a copy of the factor taken now (sp.o_snap), not the live one
int enqueue_inverse(const m3s_gn_args& a, Ctx& c, bool snapshot) {
    const SparsePlan& sp = c.sp;
    const size_t shift = snapshot ? sp.o_snap - sp.o_L : 0;
    if (snapshot) {
        M3S_REQUIRE(sp.snap_bytes > 0, "PCG: no factor snapshot buffer");
        M3S_HIP_CHECK(hipMemcpyAsync(sp.dbuf + sp.o_snap, sp.dbuf + sp.o_L, sp.snap_bytes, hipMemcpyDeviceToDevice, c.st));
    }
    InvArgs v{};
    v.n = 7 * (int)(a.N - 1);
    v.ldx = sp.pcg_ldx;
    v.nrounds = (int)sp.rounds.size();
    v.ntail = sp.ntail;
    v.npad = sp.npad_tail;
    v.rounds = sp.iptr(sp.i_rounds);
    v.nodes = sp.iptr(sp.i_nodes);
    v.fptr = sp.iptr(sp.i_fptr);
    v.fronts = sp.iptr(sp.i_fronts);
    v.inl = sp.iptr(sp.i_inl);
    v.rc4 = sp.iptr(sp.i_rc4);
    v.tail = sp.iptr(sp.i_tail);
    v.Lstore = sp.dptr<double>(sp.o_L + shift);
    v.W = sp.dptr<double>(sp.o_W + shift);
    v.Hd = sp.dptr<double>(sp.o_dense + shift);
    v.Linv = sp.dptr<double>(sp.o_linv + shift);
    v.X = sp.dptr<double>(sp.o_pcgx);
    v.Xt = sp.dptr<float>(sp.o_pcgxt);
    v.ldt = sp.pcg_ldt;
    v.flags = c.at<int>(c.L.flags);
    // M3S_PCG_SIDE (default 1): on the side stream, beside the next iteration's accumulate (it
    // reads the factor and the flags, writes X only; the next PCG launch waits for it); 0: on
    // the call's stream
    static const bool side = env_int("M3S_PCG_SIDE", 1) != 0;
    if (!side) {
        M3S_HIP_CHECK(launch_sp_inverse(c.st, v));
        return M3S_OK;
    }
    hipStream_t ss;
    hipEvent_t e1, e2;
    int rc = pcg_side(ss, e1, e2);
    if (rc) return rc;
    M3S_HIP_CHECK(hipEventRecord(e1, c.st));
    M3S_HIP_CHECK(hipStreamWaitEvent(ss, e1, 0));
    // M3S_PCG_DEBUG=1: the refresh's duration on the side stream (timing events; serialises)
    static const bool dbg = env_int("M3S_PCG_DEBUG", 0) != 0;
    hipEvent_t t0 = nullptr, t1 = nullptr;
    static long long* ibuf = nullptr;
    if (dbg && !ibuf && hipMalloc(&ibuf, sizeof(long long) * 8) != hipSuccess) ibuf = nullptr;
    v.dbg = dbg ? ibuf : nullptr;
    if (dbg) {
        if (ibuf) M3S_HIP_CHECK(hipMemsetAsync(ibuf, 0, sizeof(long long) * 8, ss));
        M3S_HIP_CHECK(hipEventCreate(&t0));
        M3S_HIP_CHECK(hipEventCreate(&t1));
        M3S_HIP_CHECK(hipEventRecord(t0, ss));
    }
    M3S_HIP_CHECK(launch_sp_inverse(ss, v));
    if (dbg) {
        M3S_HIP_CHECK(hipEventRecord(t1, ss));
        M3S_HIP_CHECK(hipEventSynchronize(t1));
        float ms = 0.f;
        M3S_HIP_CHECK(hipEventElapsedTime(&ms, t0, t1));
        long long h[8] = {0};
        if (ibuf) M3S_HIP_CHECK(hipMemcpy(h, ibuf, sizeof(h), hipMemcpyDeviceToHost));
        fprintf(stderr, "pcg inverse (M refresh): %.1f us, %d workgroups; wg0: init %.1f fwd rounds %.1f core %.1f back rounds %.1f f32 copy %.1f us\n",
                ms * 1e3, (v.n + 15) / 16, (h[1] - h[0]) * 0.01, (h[2] - h[1]) * 0.01, (h[3] - h[2]) * 0.01,
                (h[4] - h[3]) * 0.01, (h[5] - h[4]) * 0.01);
        (void)hipEventDestroy(t0);
        (void)hipEventDestroy(t1);
    }
    M3S_HIP_CHECK(hipEventRecord(e2, ss));
    c.inv_pending = true;
    c.inv_done = e2;
    return M3S_OK;
}

int enqueue_pcg(const m3s_gn_args& a, Ctx& c) {
    const SparsePlan& sp = c.sp;
    PcgArgs g{};
    g.b = sp.dptr<double>(sp.o_sys);
    g.A = g.b + sp.bpad;
    g.adj_ptr = sp.iptr(sp.i_apt);
    g.adj = reinterpret_cast<const int2*>(sp.iptr(sp.i_adj));
    g.nitem = sp.pcg_nitem;
    g.R4 = pcg_r4(sp.pcg_R);
    g.Xt = sp.dptr<float>(sp.o_pcgxt);
    g.ldt = sp.pcg_ldt;
    g.n = 7 * (int)(a.N - 1);
    g.nv = sp.pcg_nv;
    g.onex = sp.pcg_onex ? 1 : 0;
    g.R = sp.pcg_R;
    g.nwg = sp.pcg_nwg;
    g.gran = reinterpret_cast<unsigned long long*>(sp.dbuf + sp.o_gran);
    // tags: unique within the call (the granules are zeroed per call), 2 kmax + 1 exchanges a launch
    static const int kmax = std::max(1, std::min(200, env_int("M3S_PCG_KMAX", 30)));
    static const double tol = [] {
        const char* e = getenv("M3S_PCG_TOL");
        return e ? atof(e) : 1e-6;
    }();
    g.kmax = kmax;
    g.tol2 = tol * tol;
    g.tag0 = 1u + (unsigned)c.pcg_launches * (unsigned)(2 * kmax + 2);
    c.pcg_launches++;
    const char* ft = getenv("M3S_TEST_FORCE_TIMEOUT");
    g.spin_limit = (ft && atoi(ft) != 0) ? 0 : (1 << 22);
    g.Twc = a.Twc;
    g.dx = a.dx;
    g.N = (int)a.N;
    g.delta_thresh = a.delta_thresh;
    g.contract = a.contract;
    g.flags = c.at<int>(c.L.flags);
    // M3S_PCG_DEBUG=1: workgroup 0's phase clocks, printed after the launch (the wait serialises
    // the call: diagnostics only)
    static const bool dbg = env_int("M3S_PCG_DEBUG", 0) != 0;
    static long long* dbuf = nullptr;
    if (dbg && !dbuf && hipMalloc(&dbuf, sizeof(long long) * kPcgDbgSlots) != hipSuccess) dbuf = nullptr;
    if (dbg && dbuf) M3S_HIP_CHECK(hipMemsetAsync(dbuf, 0, sizeof(long long) * kPcgDbgSlots, c.st));
    g.dbg = dbg ? dbuf : nullptr;
    M3S_HIP_CHECK(launch_pcg(c.st, g));
    if (g.dbg) {
        long long h[kPcgDbgSlots];
        M3S_HIP_CHECK(hipMemcpyAsync(h, dbuf, sizeof(h), hipMemcpyDeviceToHost, c.st));
        M3S_HIP_CHECK(hipStreamSynchronize(c.st));
        // s_memrealtime: 100 MHz
        fprintf(stderr, "pcg[%d] R %d nwg %d: stage %.2f us, z0 %.2f us;", c.pcg_launches - 1, g.R, g.nwg,
                (h[1] - h[0]) * 0.01, (h[2] - h[1]) * 0.01);
        long long prev = h[2];
        for (int st = 1; 3 * st + 2 < kPcgDbgSlots && h[3 * st + 2] != 0; st++) {
            fprintf(stderr, " [Ap %.2f pq %.2f z %.2f]", (h[3 * st] - prev) * 0.01, (h[3 * st + 1] - h[3 * st]) * 0.01,
                    (h[3 * st + 2] - h[3 * st + 1]) * 0.01);
            prev = h[3 * st + 2];
        }
        fprintf(stderr, "\n");
    }
    return M3S_OK;
}

// The deferred timeout report of this thread's last gauss_newton call (waits for its flag copy):
// M3S_ERR_TIMEOUT once, then cleared.
int take_deferred_timeout(const char* which) {
    Stagings& sg = stagings();
    if (!sg.tmo_armed) return M3S_OK;
    const int kind = sg.tmo_armed;
    sg.tmo_armed = 0;
    const char* h = sg.tmo.get(64);  // waits for the copy (its event)
    const bool hit = kind == 2 ? *reinterpret_cast<const double*>(h) > 0.0 : *reinterpret_cast<const int*>(h) != 0;
    if (hit) {
        set_error("gauss_newton: %sa device-side wait of the factorisation timed out (the solve was "
                  "discarded; not a singular system)", which);
        return M3S_ERR_TIMEOUT;
    }
    return M3S_OK;
}

// The elimination plan the solve runs for this pose graph (M3S_SOLVER pins
// one).  Default: the hybrid (multi-launch rounds + gn_solve's back-substitution) when its core
// fits, else the multi-launch plan; the single-workgroup solve when the plan needs few rounds.
void choose_sparse_plan(const Plan& plan, int npose, SparsePlan& sp) {
    // M3S_SOLVER: 1 = single-workgroup (gn_solve), 2 = multi-launch, 0 (default) = the
    // single-workgroup solve when its plan needs few rounds, else multi-launch
    const int choice = env_int("M3S_SOLVER", 0);
    const int max_fused_rounds = env_int("M3S_FUSED_MAX_ROUNDS", 3);
    const bool hybrid_on = env_int("M3S_HYBRID", 1) != 0;
    // Default choice: the hybrid plan first.  The fused policy is the hybrid's plus a cap on
    // the poses per round (LDS staging), so it never needs fewer rounds; when the hybrid
    // plan already needs more than max_fused_rounds, the fused solve would be rejected and
    // building its plan (~0.23 ms of host time on cfg3, exposed once the per-call pack is
    // short, e.g. edge-sharded over several GPUs) is skipped.
    bool planned = false;
    if (choice == 0 && hybrid_on) {
        // the hybrid's rounds and core decided symbolically first (no lists): on a graph
        // whose core does not fit the in-register factorisation (cfg4) building the hybrid's
        // lists only to replace them by the multi plan cost ~1.5 ms of host time per call,
        // exposed once the edges are sharded (the first accumulate no longer covers it)
        static thread_local SparsePlan probe;
        build_sparse_plan(plan.pairs, plan.nblk, npose, hybrid_policy(), probe, true);
        if ((int)probe.rounds.size() > max_fused_rounds) {
            const bool hyb = hyb_core_fits(probe) && npose <= solve_max_poses() &&
                             solve_lds_bytes((int)probe.nints_back) <= (size_t)kSolveMaxLds;
            build_sparse_plan(plan.pairs, plan.nblk, npose, hyb ? hybrid_policy() : multi_policy(), sp);
            sp.hybrid = hyb;
            planned = true;
        }
    }
    bool fused_ok = false, meta_fits = false;
    if (!planned) {
        build_sparse_plan(plan.pairs, plan.nblk, npose, fused_policy(), sp);
        meta_fits = solve_lds_bytes((int)sp.nints) <= (size_t)kSolveMaxLds;
        fused_ok = sp.fused && meta_fits && npose <= solve_max_poses() &&
                   (choice == 1 || (choice == 0 && (int)sp.rounds.size() <= max_fused_rounds));
    }
    if (env_int("M3S_SOLVE_DEBUG", 0) && !fused_ok && !planned)
        fprintf(stderr, "fused solve rejected: fused_tail %d (ntail %d) rounds %zu nints %zu meta_fits %d\n",
                (int)sp.fused, sp.ntail, sp.rounds.size(), sp.nints, (int)meta_fits);
    if (!fused_ok && !planned) {
        // M3S_SOLVER=3 / default: multi-launch rounds + the in-register core when it fits
        bool hyb = false;
        if (choice == 3 || (choice == 0 && hybrid_on)) {
            build_sparse_plan(plan.pairs, plan.nblk, npose, hybrid_policy(), sp);
            hyb = hyb_core_fits(sp) && npose <= solve_max_poses() &&
                  solve_lds_bytes((int)sp.nints_back) <= (size_t)kSolveMaxLds;
        }
        if (!hyb) build_sparse_plan(plan.pairs, plan.nblk, npose, multi_policy(), sp);
        sp.hybrid = hyb;
    }
    sp.core_df = hyb_core_df();
}

// m3s_gn_plan_info (include/m3s_backend.h): the plan choose_sparse_plan makes, from host lists
int plan_info(const int64_t* ii, const int64_t* jj, int64_t E, int64_t N, int32_t* info, int32_t* order,
              int32_t* round_ptr, int32_t round_cap) {
    M3S_REQUIRE(info != nullptr && N >= 1 && E >= 0 && (E == 0 || (ii != nullptr && jj != nullptr)),
                "gn_plan_info: bad arguments");
    // the op's per-thread plan objects (no call is in flight on this thread here)
    Plan& plan = tls_plan();
    std::vector<int> iopt, jopt;
    int rc = plan_pairs(ii, jj, E, N, plan, iopt, jopt);
    if (rc) return rc;
    const int npose = (int)(N - 1);
    SparsePlan& sp = tls_sparse_plan();
    sp.reset();
    if (npose > 0) choose_sparse_plan(plan, npose, sp);
    info[0] = npose <= 0 ? -1 : sp.fused ? 0 : sp.hybrid ? 1 : 2;
    info[1] = (int32_t)sp.rounds.size();
    info[2] = (int32_t)sp.nodes.size();
    info[3] = sp.ntail;
    info[4] = sp.npad_tail;
    info[5] = (int32_t)plan.pairs.size();
    info[6] = (int32_t)sp.nints;
    info[7] = sp.npad_tail <= kMaxNpad ? 1 : 0;
    if (order) {
        std::copy(sp.nodes.begin(), sp.nodes.end(), order);
        std::copy(sp.tail.begin(), sp.tail.end(), order + sp.nodes.size());
    }
    if (round_ptr && round_cap >= (int32_t)sp.rounds.size() + 1) {
        for (size_t k = 0; k < sp.rounds.size(); k++) round_ptr[k] = sp.rounds[k].node_begin;
        round_ptr[sp.rounds.size()] = (int32_t)sp.nodes.size();
    }
    return M3S_OK;
}

int run(const m3s_gn_args& a) {
    // M3S_PROF_HOST: host-side phase times of the call (stderr)
    static const bool prof_host = env_int("M3S_PROF_HOST", 0) != 0;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto us = [](std::chrono::steady_clock::time_point x, std::chrono::steady_clock::time_point y) {
        return std::chrono::duration<double, std::micro>(y - x).count();
    };
    const auto t0 = now();
    Ctx c;
    c.need_slotmap = env_int("M3S_SOLVER_DENSE", 0) != 0;
    // the packed stream is launched inside setup as soon as its inputs are on the device: the
    // GPU builds it while the host plans the accumulate schedule and the elimination
    int rc = setup(a, c, a.N > 1);
    if (rc) return rc;
    // an earlier call's timeout (its copy has landed: setup synchronised the stream)
    rc = take_deferred_timeout("an earlier call: ");
    if (rc) return rc;
    const auto t1 = now();
    const int npose = (int)(a.N - 1);
    if (npose <= 0) return M3S_OK;  // nothing to optimise (all poses pinned)
    const Layout& L = c.L;
    int* flags = c.at<int>(L.flags);
    std::chrono::steady_clock::time_point t2 = t1, t3 = t1;
    // M3S_EARLY_ACC (default 1): iteration 0's accumulate is enqueued before the host builds the
    // elimination plan (the GPU works while the host plans; the per-call pack alone no longer
    // covers the planning once the edges are sharded over several GPUs)
    if (!c.ref_order && a.max_iter > 0 && env_int("M3S_EARLY_ACC", 1) != 0) {
        g_prof.mark(c.st);
        rc = enqueue_accumulate(a, c);
        if (rc) return rc;
        c.acc_enqueued = true;
        // edge-sharded: the records' all-gather needs no plan either -- the ranks exchange (and
        // wait for the slowest rank's accumulate) while their hosts plan.  M3S_EARLY_GATHER: -1
        // (default) with RCCL only (a host-callback exchange would block this thread until every
        // rank's accumulate is done), 1 always (tests: the host exchange), 0 never
        static const int early_gather = env_int("M3S_EARLY_GATHER", -1);
        if (c.plan.gather && (early_gather > 0 || (early_gather < 0 && comm_is_async(a.comm)))) {
            rc = comm_allgather_f64(a.comm, c.eall, (size_t)c.plan.gchunk * kEdgeBlk, c.st);
            if (rc) return rc;
            c.gathered = true;
        }
    }
    const auto t1b = now();
    if (env_int("M3S_SOLVER_DENSE", 0) == 0 || c.ref_order) {
        choose_sparse_plan(c.plan, npose, c.sp);
        choose_pcg(a, c, c.plan, npose, c.sp);
        t2 = now();
        M3S_REQUIRE(c.sp.npad_tail <= kMaxNpad,
                    "gauss_newton: the dense core of the elimination (%d unknowns) exceeds the "
                    "dense solve limit (%d)", c.sp.npad_tail, kMaxNpad);
        rc = upload_sparse_plan(c.sp, npose, c.st);
        if (rc) return rc;
        t3 = now();
    }
    if (prof_host)
        fprintf(stderr, "gn host: setup %.0f us, early enqueue %.0f us, plan %.0f us, upload %.0f us\n", us(t0, t1),
                us(t1, t1b), us(t1b, t2), us(t2, t3));
    for (int itr = 0; itr < a.max_iter; itr++) {
        if (!c.acc_enqueued) g_prof.mark(c.st);  // (iteration 0's mark preceded its early accumulate)
        rc = enqueue_system(a, c);
        if (rc) return rc;
        g_prof.mark(c.st);
        // the poses the call started from, so that a timed-out call can restore them (below)
        if (itr == 0) M3S_HIP_CHECK(launch_twc_save(c.st, a.Twc, c.at<float>(L.twc_save), (int)(8 * a.N)));
        const int from = c.sp.pcg_from, lag = c.sp.pcg_lag;
        if (c.sp.pcg && itr >= from) {  // the direct solve below is its fallback
            if (c.inv_pending) {  // M's refresh (side stream) must be complete
                M3S_HIP_CHECK(hipStreamWaitEvent(c.st, c.inv_done, 0));
                c.inv_pending = false;
            }
            rc = enqueue_pcg(a, c);
            if (rc) return rc;
        }
        rc = enqueue_solve(a, c, c.sp.pcg && itr >= from);
        if (rc) return rc;
        g_prof.mark(c.st);
        if (!c.sp.fused && !c.sp.hybrid)  // gn_solve retracts inside its launch
            M3S_HIP_CHECK(launch_retract(c.st, a.Twc, c.at<double>(L.x), a.dx, (int)a.N,
                                         a.delta_thresh, flags, a.contract));
        // M from this iteration's factor: iteration M3S_PCG_FROM - M3S_PCG_LAG's (a copy of it
        // when the lag is 2 or more), then after every PCG that fell back to the direct solve
        // (sp_inverse_kernel returns at once when this iteration's PCG converged: M stays)
        if (c.sp.pcg && (itr == from - lag || itr >= from) && itr + 1 < a.max_iter) {
            rc = enqueue_inverse(a, c, itr < from - 1);
            if (rc) return rc;
        }
        g_prof.mark(c.st);
    }
    // (the per-call solver buffers are released by ~Ctx on this and every error path)
    if (c.may_timeout && a.max_iter > 0) {
        // A bounded device-side wait that gave up discarded that iteration's solve (dx = 0): an
        // error, not a singular system (the reference's host Eigen solve cannot time out).  The
        // call then restores the poses it started from, on the device (twc_guard_kernel), so a
        // timed-out call never commits poses -- whatever its caller does next -- and
        // every rank of a sharded call ends with the same Twc.  The flag leaves the device without
        // a host wait (the same kernel writes it to pinned memory): the error is reported by the
        // next GN call on this thread (once setup() has synchronised the stream) or by
        // m3s_gn_check, like an asynchronous kernel fault.  Waiting here instead left the GPU idle
        // between calls for the host's per-call work (cfg3: 694 vs 318 us call-to-call gap,
        // rocprofv3 trace).  M3S_GN_TIMEOUT_SYNC=1: report it from this call (one stream
        // synchronisation).
        Stagings& sg = stagings();
        char* h = sg.tmo.get(64);
        M3S_REQUIRE(h != nullptr, "gauss_newton: pinned host allocation failed");
        float* save = c.at<float>(L.twc_save);
        const int n8 = (int)(8 * a.N);
        if (a.comm) {
            // edge-sharded: every rank ran the same replicated solve, but the flag is rank-local --
            // OR it over the ranks (a sum of 0 / 1) so that all fail together instead of one rank
            // returning the error while the others go on to their next collective,
            // and all restore their poses
            double* dv = c.at<double>(L.x);  // the solution buffer is free once the call retracted
            M3S_HIP_CHECK(launch_flag_export(c.st, flags + kFlagTimeout, dv, 1));
            rc = comm_allreduce_sum_f64(a.comm, dv, 1, c.st);
            if (rc) return rc;
            M3S_HIP_CHECK(launch_twc_restore_on_flag(c.st, a.Twc, save, n8, dv, 1, sg.tmo.dev));
            if (!sg.tmo.dev) M3S_HIP_CHECK(hipMemcpyAsync(h, dv, sizeof(double), hipMemcpyDeviceToHost, c.st));
            sg.tmo_armed = 2;
        } else {
            M3S_HIP_CHECK(launch_twc_restore_on_flag(c.st, a.Twc, save, n8, flags + kFlagTimeout, 0, sg.tmo.dev));
            if (!sg.tmo.dev)
                M3S_HIP_CHECK(hipMemcpyAsync(h, flags + kFlagTimeout, sizeof(int), hipMemcpyDeviceToHost, c.st));
            sg.tmo_armed = 1;
        }
        M3S_HIP_CHECK(sg.tmo.mark(c.st));
        static const bool sync_report = env_int("M3S_GN_TIMEOUT_SYNC", 0) != 0;
        if (sync_report) {
            rc = take_deferred_timeout("");
            if (rc) return rc;
        }
    }
    if (const int dbg = env_int("M3S_GN_DEBUG_FLAGS", 0)) {  // diagnostics: the device flags after the call
        int hf[kNumFlags];
        M3S_HIP_CHECK(hipMemcpyAsync(hf, flags, sizeof(hf), hipMemcpyDeviceToHost, c.st));
        M3S_HIP_CHECK(hipStreamSynchronize(c.st));
        // m3s_gn_debug_flags: which accumulate path the call took (bench.py prices its bytes)
        g_dbg_flags[0] = hf[kFlagDone];
        g_dbg_flags[1] = hf[kFlagFail];
        g_dbg_flags[2] = c.packed ? 1 : 0;
        g_dbg_flags[3] = (c.packed && c.P.raycheck && hf[kFlagNotRay] == 0) ? 1 : 0;
        g_dbg_pcg[0] = hf[kFlagPcgRuns];
        g_dbg_pcg[1] = hf[kFlagPcgSteps];
        g_dbg_pcg[2] = hf[kFlagPcgFall];
        g_dbg_pcg[3] = c.sp.pcg ? 1 : 0;
        g_dbg_pcg[4] = c.sp.pcg ? c.sp.pcg_from : 0;
        if (dbg != 2)
            fprintf(stderr, "gn flags: done %d fail %d not_ray %d timeout %d packed %d pcg runs %d steps %d fallbacks %d\n",
                    hf[kFlagDone], hf[kFlagFail], hf[kFlagNotRay], hf[kFlagTimeout], (int)c.packed,
                    hf[kFlagPcgRuns], hf[kFlagPcgSteps], hf[kFlagPcgFall]);
    }
    return M3S_OK;
}

}  // namespace
}  // namespace m3s

using namespace m3s;

extern "C" const char* m3s_last_error(void) { return m3s::get_error(); }

extern "C" int m3s_gn_check(void* stream) {
    const hipError_t e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
    if (e != hipSuccess) {
        set_error("gn_check: %s", hipGetErrorString(e));
        return M3S_ERR_HIP;
    }
    return m3s::take_deferred_timeout("");
}

extern "C" void m3s_gn_debug_flags(int* out4) {
    for (int k = 0; k < 4; k++) out4[k] = m3s::g_dbg_flags[k];
}

extern "C" void m3s_gn_pcg_stats(int* out5) {
    for (int k = 0; k < 5; k++) out5[k] = m3s::g_dbg_pcg[k];
}

extern "C" const char* m3s_version(void) { return "m3s 0.1.0 gfx950"; }

extern "C" void m3s_shutdown(void) {
    HostResources& r = host_resources();
    std::lock_guard<std::mutex> lk(r.mu);
    if (r.shut) return;
    r.shut = true;
    for (auto& it : r.items) it.second(it.first);
    r.items.clear();
}

namespace {
// Registered when the library is loaded: after the HIP runtime's own exit-time teardown (and a
// profiler's) was registered, so m3s_shutdown runs before them.
__attribute__((constructor)) void m3s_register_shutdown() { std::atexit(m3s_shutdown); }
}  // namespace

extern "C" size_t m3s_gn_workspace_bytes(int mode, int64_t N, int64_t HW, int64_t E_total,
                                         int64_t E_local) {
    if (N < 1 || HW < 1 || E_total < 0 || E_local < 0) return 0;
    return make_layout(mode, N, HW, E_total, E_local).total;
}

extern "C" int m3s_gn_plan_info(const int64_t* ii, const int64_t* jj, int64_t E, int64_t N, int32_t* info,
                                int32_t* order, int32_t* round_ptr, int32_t round_cap) {
    return m3s::plan_info(ii, jj, E, N, info, order, round_ptr, round_cap);
}

extern "C" int m3s_gauss_newton(const m3s_gn_args* args) {
    if (!args) {
        set_error("gauss_newton: null args");
        return M3S_ERR_INVALID;
    }
    return run(*args);
}

namespace {
// Reference-order per-edge records (kRefStride floats: D[7][7], g[7]) of ONE accumulate pass,
// copied to the host.
int ref_edge_records(const m3s_gn_args& a0, Ctx& c, std::vector<float>& rec) {
    m3s_gn_args a = a0;
    a.order = M3S_GN_ORDER_REFERENCE;
    int rc = setup(a, c);
    if (rc) return rc;
    rec.assign((size_t)a.E_local * kRefStride, 0.0f);
    if (a.E_local == 0) return M3S_OK;
    const Layout& L = c.L;
    M3S_HIP_CHECK(launch_accum_ref(a.mode, (int)a.E_local, c.st, a.Twc, a.Xs, a.Cs, c.at<int>(L.ii_loc),
                                   c.at<int>(L.jj_loc), c.es, c.R, c.at<float>(L.edgeblk),
                                   c.at<int>(L.flags)));
    M3S_HIP_CHECK(hipMemcpyAsync(rec.data(), c.at<float>(L.edgeblk), sizeof(float) * rec.size(),
                                 hipMemcpyDeviceToHost, c.st));
    M3S_HIP_CHECK(hipStreamSynchronize(c.st));
    return M3S_OK;
}

// The reference's four blocks of one edge from its record (see gn_refacc.hip):
// Hs[0] = Hs[3] = lower(D) mirrored, Hs[1] = -D^T, Hs[2] = -D.
double ref_block(const float* D, int blk, int r, int cc) {
    switch (blk) {
        case 0:
        case 3: return (double)D[std::max(r, cc) * 7 + std::min(r, cc)];
        case 1: return -(double)D[cc * 7 + r];
        default: return -(double)D[r * 7 + cc];
    }
}
}  // namespace

extern "C" int m3s_gn_edge_hessians(const m3s_gn_args* args, float* Hs_host, float* gs_host) {
    if (!args || !Hs_host || !gs_host) {
        set_error("gn_edge_hessians: null argument");
        return M3S_ERR_INVALID;
    }
    Ctx c;
    std::vector<float> rec;
    int rc = ref_edge_records(*args, c, rec);
    if (rc) return rc;
    const int64_t E = args->E_local;
    for (int64_t e = 0; e < E; e++) {
        const float* D = rec.data() + e * kRefStride;
        for (int blk = 0; blk < 4; blk++)
            for (int r = 0; r < 7; r++)
                for (int q = 0; q < 7; q++)
                    Hs_host[((blk * E + e) * 7 + r) * 7 + q] = (float)ref_block(D, blk, r, q);
        for (int q = 0; q < 7; q++) {
            gs_host[(0 * E + e) * 7 + q] = -D[49 + q];
            gs_host[(1 * E + e) * 7 + q] = D[49 + q];
        }
    }
    return M3S_OK;
}

extern "C" int m3s_gn_build_system(const m3s_gn_args* args, double* H_host, double* b_host) {
    if (!args) {
        set_error("gn_build_system: null args");
        return M3S_ERR_INVALID;
    }
    const m3s_gn_args& a = *args;
    if (gn_order(a) == M3S_GN_ORDER_REFERENCE) {
        // the full (not exactly symmetric) matrix SparseBlock::update_lhs/update_rhs builds
        // from the reference-order Hs/gs (gn_kernels.cu:71-113)
        Ctx c;
        std::vector<float> rec;
        int rc = ref_edge_records(a, c, rec);
        if (rc) return rc;
        const int64_t n = 7 * (a.N - 1);
        std::fill(H_host, H_host + n * n, 0.0);
        std::fill(b_host, b_host + n, 0.0);
        for (int64_t el = 0; el < a.E_local; el++) {
            const float* D = rec.data() + el * kRefStride;
            const int i = c.plan.ii_loc[el] - 1, j = c.plan.jj_loc[el] - 1;
            const int rr[4] = {i, i, j, j}, cc[4] = {i, j, i, j};
            for (int blk = 0; blk < 4; blk++) {
                if (rr[blk] < 0 || cc[blk] < 0) continue;
                for (int r = 0; r < 7; r++)
                    for (int q = 0; q < 7; q++)
                        H_host[(7 * rr[blk] + r) * n + 7 * cc[blk] + q] += ref_block(D, blk, r, q);
            }
            for (int q = 0; q < 7; q++) {
                if (i >= 0) b_host[7 * i + q] -= (double)D[49 + q];
                if (j >= 0) b_host[7 * j + q] += (double)D[49 + q];
            }
        }
        return M3S_OK;
    }
    Ctx c;
    c.need_slotmap = true;
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
    M3S_HIP_CHECK(launch_fill_only(c.st, c.at<double>(L.compact), c.dyn_at<int>(c.o_slot), c.plan.nblk,
                                   npose, n, L.npad, c.dyn_at<double>(c.o_dense), c.at<int>(L.flags)));
    M3S_HIP_CHECK(hipMemcpy2DAsync(H_host, sizeof(double) * n, c.dyn_at<double>(c.o_dense),
                                   sizeof(double) * L.npad, sizeof(double) * n, n,
                                   hipMemcpyDeviceToHost, c.st));
    M3S_HIP_CHECK(hipMemcpyAsync(b_host, c.dyn_at<double>(c.o_dense) + (size_t)L.npad * L.npad,
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
    g_prof.first.clear();
    g_prof.accum_only = false;
    g_prof.on = true;
    return M3S_OK;
}

extern "C" int m3s_prof_begin_accum(void) {
    int rc = m3s_prof_begin();
    g_prof.accum_only = true;
    return rc;
}

// out[0] accumulate-kernel ms, out[1] edge-reduce/compact/all-reduce ms, out[2] solve ms,
// out[3] retract ms (sums over iterations); *n_iter = iterations recorded.
extern "C" int m3s_prof_end(double* out, int* n_iter) {
    g_prof.on = false;
    double acc[4] = {0, 0, 0, 0};
    int n = 0;
    if (g_prof.accum_only) {  // a0 a1 per iteration
        // out[0] / *n_iter: the iteration kernel (records already packed); out[1] / out[2]: the
        // launches that built the records themselves (a call's first, M3S_GN_PACK_FIRST) and
        // their count
        g_prof.accum_only = false;
        g_prof_launch_ms.clear();
        for (size_t k = 0; k + 2 <= g_prof.marks.size(); k += 2) {
            float ms = 0.f;
            M3S_HIP_CHECK(hipEventSynchronize(g_prof.marks[k + 1]));
            M3S_HIP_CHECK(hipEventElapsedTime(&ms, g_prof.marks[k], g_prof.marks[k + 1]));
            if (k / 2 < g_prof.first.size() && g_prof.first[k / 2]) {
                acc[1] += ms;
                acc[2] += 1;
            } else {
                acc[0] += ms;
                n++;
                g_prof_launch_ms.push_back(ms);
            }
        }
        for (int q = 0; q < 4; q++) out[q] = acc[q];
        *n_iter = n;
        for (hipEvent_t e : g_prof.marks) g_prof.pool.push_back(e);
        g_prof.marks.clear();
        return M3S_OK;
    }
    const size_t per = 6;  // t0 [a0 a1] t1 t2 t3 (a0/a1 bracket the accumulate kernel)
    g_prof_solve_ms.clear();
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
        g_prof_solve_ms.push_back(ms[3]);
        n++;
    }
    for (int q = 0; q < 4; q++) out[q] = acc[q];
    *n_iter = n;
    for (hipEvent_t e : g_prof.marks) g_prof.pool.push_back(e);
    g_prof.marks.clear();
    return M3S_OK;
}

// the per-launch durations (ms) of the iteration kernel from the last m3s_prof_begin_accum ..
// m3s_prof_end session (bench.py: the spread of the accumulate over the timed steps); returns the
// number of launches recorded, copies at most cap of them
extern "C" int m3s_prof_launch_ms(double* out, int cap) {
    const int n = (int)g_prof_launch_ms.size();
    for (int k = 0; k < n && k < cap; k++) out[k] = g_prof_launch_ms[k];
    return n;
}

// each iteration's solve ms from the last m3s_prof_begin .. m3s_prof_end session (bench.py: the
// direct iterations apart from the PCG ones); returns the count, copies at most cap
extern "C" int m3s_prof_solve_ms(double* out, int cap) {
    const int n = (int)g_prof_solve_ms.size();
    for (int k = 0; k < n && k < cap; k++) out[k] = g_prof_solve_ms[k];
    return n;
}
