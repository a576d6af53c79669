// gn_kernels.h -- shared constants / launcher declarations of the GN kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace m3s {

enum { GN_POINTS = 0, GN_RAYS = 1, GN_CALIB = 2 };

#ifndef M3S_ACC_THREADS
#define M3S_ACC_THREADS 256
#endif
constexpr int kAccThreads = M3S_ACC_THREADS;  // accumulate / pack workgroup size
constexpr int kNacc = 35;      // 28 (sym 7x7) + 7 (gradient)
constexpr int kNaccPad = 36;   // partial record stride (floats)
constexpr int kEdgeBlk = 36;   // per-edge record (doubles): Hjj packed 28 + vj 7 + pad
constexpr int kCholTile = 64;  // dense Cholesky tile

constexpr int kFlagDone = 0;   // set once ||dx|| < delta_thresh (skips later iterations)
constexpr int kFlagFail = 1;   // set by the factorisation when a pivot <= 0
constexpr int kFlagNotRay = 2; // calib: some Xs point is not its pixel's ray times its depth
constexpr int kFlagTimeout = 3; // sticky for the call: a bounded device-side wait gave up (chol_df
                                // ready word, grid barrier); the driver returns M3S_ERR_TIMEOUT
constexpr int kFlagBarCount = 4;  // grid barrier of the all-rounds launch: arrivals
constexpr int kFlagBarGen = 5;    // ... and its generation
// The lagged-factor PCG (gn_pcg.hip) of an iteration that converged has retracted the poses
// itself; the direct solve's launches enqueued behind it (its fallback) then return at once
// (solve_skipped).  Set or cleared by every PCG launch; never set in iterations without one.
constexpr int kFlagSkipSolve = 6;
constexpr int kFlagPcgRuns = 7;   // diagnostics (M3S_GN_DEBUG_FLAGS): PCG solves of the call
constexpr int kFlagPcgSteps = 8;  // ... their CG steps in all
constexpr int kFlagPcgFall = 9;   // ... and how many fell back to the direct solve
constexpr int kFlagPcgAbort = 10; // a PCG launch's workgroup gave up on a gather (= that launch's tag)
constexpr int kNumFlags = 16;
// the direct solve's launches of this iteration have nothing to do: the call converged (early
// exit) or the iteration's PCG converged and retracted
__device__ __forceinline__ bool solve_skipped(const int* flags) {
    return (flags[kFlagDone] | flags[kFlagSkipSolve]) != 0;
}

// Where the per-point-edge inputs (idx, valid, Q) of local directed edge e live: edges
// e < E_a in the first arrays (row e), the others in the second arrays (row e - E_a).  One
// contiguous tensor (the reference's layout): both halves the same arrays and E_a = E_local.
// Two halves: the forward and backward edge sets of a two-way edge store, passed without the
// per-call concatenation of global_opt.py:104-110.
struct EdgeSrc {
    const int64_t* idx[2];
    const uint8_t* valid[2];
    const float* Q[2];
    int E_a;
    __device__ __forceinline__ void at(int e, int64_t HW, const int64_t*& i, const uint8_t*& v,
                                       const float*& q) const {
        const int h = e >= E_a;
        const int64_t off = (int64_t)(h ? e - E_a : e) * HW;
        i = idx[h] + off;
        v = valid[h] + off;
        q = Q[h] + off;
    }
};

// Upper-triangle packing of a symmetric 7x7 block: index of (a,b), a <= b.
__host__ __device__ constexpr int sym_idx(int a, int b) {
    return a * 7 - a * (a - 1) / 2 + (b - a);
}

struct AccParams {
    float s0_inv, s1_inv;  // 1/sigma0, 1/sigma1
    float C_thresh, Q_thresh;
    float fx, fy, cx, cy;
    float pb_lo, pb_hi_u, pb_hi_v;  // calib border: (pb, W-1-pb, H-1-pb) as float
    float z_eps;
    unsigned div_m;  // ind / width == (ind * div_m) >> div_sh for 0 <= ind < 2^31
    int div_sh;
    int width, height;
    int HW;
    int chunk;    // points per workgroup (multiple of 4)
    int nchunks;  // chunks per directed edge
    int nkf;      // keyframes (rows of Xs / Zs)
    int pack_uv;  // packed calib stream: code = v << 16 | u of the match (W < 2^16, H < 2^15)
    int raycheck; // M3S_GN_RAYCHECK=1: launch the packed calib kernel that can take the
                  // ray-constrained path (a separate instantiation: its VGPRs do not burden the default)
};

// Reference-order ("parity") accumulate, gn_refacc.hip
constexpr int kRefVals = 56;    // per edge: D[7][7] + g[7]
constexpr int kRefStride = 64;  // floats per edge record
struct RefParams {
    float s0_inv, s1_inv;  // (float)(1.0 / sigma) as the reference computes them
    float C_thresh, Q_thresh;
    float fx, fy, cx, cy;
    float z_eps;
    int width, height, pixel_border;
    int64_t HW;
    int variant;   // diagnostics only (env M3S_GN_REF_VARIANT): kRefVar* formula substitutions
    int contract;  // M3S_CONTRACT_*: FMA contraction of the reference build (contract.h)
};
// Formula substitutions for measuring what each deviation of the fast path's residual model
// from the reference costs in accuracy, under the reference's own summation order.
constexpr int kRefVarLogRatio = 1;  // calib log depth as ln2 * log2(zj * rcp(zi))
constexpr int kRefVarRcp = 2;       // 1/x by v_rcp_f32 instead of the double division
constexpr int kRefVarHuberMin = 4;  // Huber weight as min(1, 1.345 rcp|r|)
hipError_t launch_accum_ref(int mode, int E_local, hipStream_t st, const float* Twc, const float* Xs,
                            const float* Cs, const int* ii_loc, const int* jj_loc, const EdgeSrc& es,
                            const RefParams& P, float* out, const int* flags);
hipError_t launch_assemble_ref(hipStream_t st, const float* ref, const int* blk_ptr, const int* blk_ref,
                               const int* grad_ptr, const int* grad_ent, int nblk, int nblocks,
                               int npose, int bpad, double* out, const int* flags);

hipError_t launch_accum(int mode, bool vec, dim3 grid, hipStream_t st, const float* Twc,
                        const float* Xs, const float* Cs, const int* ii_loc, const int* jj_loc,
                        const EdgeSrc& es, const AccParams& P, const int4* sched, float* partials,
                        const int* flags);
// px == nullptr: the positional packed stream (8 B per point-edge); else the compacted one
// (live points only: records in pack, Xj copies in px, per-(edge, chunk) counts in pcnt)
hipError_t launch_pack(int mode, hipStream_t st, int E_local, const float* Xs, int64_t N, const float* Cs,
                       const int* ii_loc, const int* jj_loc, const EdgeSrc& es, const AccParams& P, int* cok,
                       int4* pack, float* px, int* pcnt, const int* flags, bool skip_pack = false);
// The per-call passes the pack reads that need no edge lists: the keyframes' confidence pass
// (cpass: cok[n] = every C of keyframe n > C_thresh; cok preset to 1) and, calib, the depth /
// inverse-depth arrays and ray tables (Zs != nullptr; K != nullptr: fx, fy, cx, cy read from
// the device K instead of P) -- enqueued while the host still plans.
hipError_t launch_pack_pre(hipStream_t st, const float* Xs, int64_t N, const float* Cs, const AccParams& P, int* cok,
                           float* Zs, int* flags, const float* K);
// The call's device flags (kNumFlags ints: 0, kFlagNotRay = not_ray) and cok[0 .. n) = 1.
hipError_t launch_gn_init(hipStream_t st, int* flags, int not_ray, int* cok, int64_t n);
hipError_t launch_accum_packed(int mode, dim3 grid, hipStream_t st, const float* Twc,
                               const float* Xs, const float* Zs, const int* ii_loc,
                               const int* jj_loc, const int4* pack, const AccParams& P,
                               const int4* sched, float* partials, const int* flags, const float* px,
                               const int* pcnt, int* ecnt = nullptr, double* edgeblk = nullptr,
                               const EdgeSrc* first_es = nullptr, const float* Cs = nullptr,
                               const int* cok = nullptr);
hipError_t launch_edge_reduce(int E_local, hipStream_t st, const float* partials, int nchunks,
                              const float* Twc, const int* ii_loc, double* edgeblk,
                              const int* flags);
hipError_t launch_compact(hipStream_t st, const double* edgeblk, const int* blk_ptr,
                          const int* blk_ent, const int* grad_ptr, const int* grad_ent, int nblk,
                          int npose, double* compact, const int* flags);
hipError_t launch_assemble(hipStream_t st, const double* edgeblk, const int* blk_ptr,
                           const int* blk_ent, const int* grad_ptr, const int* grad_ent, int nblk,
                           int nblocks, int npose, int bpad, double* out, const int* flags);
hipError_t launch_solve(hipStream_t st, const double* compact, const int* slotmap, int nblk,
                        int npose, int n, int npad, double* Hd, double* Linv, double* x,
                        int* flags, int epoch);
constexpr int kMaxNpad = 8192;  // dense solve limit: N <= 1171 keyframes
// Linv region: the npad / 64 tile inverses (64 x 64 f64 each), then the dataflow factor's
// per-tile ready words (chol_df.hip; zeroed once per call, epoch = 1, 2, ... per factorisation)
size_t chol_ready_bytes(int npad);
inline size_t chol_linv_bytes(int npad) {
    return sizeof(double) * (size_t)npad * kCholTile + chol_ready_bytes(npad);
}
inline int* chol_ready_ptr(double* Linv, int npad) {
    return reinterpret_cast<int*>(Linv + (size_t)npad * kCholTile);
}
// The elimination's dense core: the in-launch back-substitution also writes x pose-indexed
// (x_pose[7 tail[i / 7] + i % 7] = x[i], i < 7 ntail) for the back rounds -- no scatter launch
struct DfScatter {
    const int* tail;
    int ntail;
    double* xpose;
};
// x != nullptr: the back-substitution L^T x = y (y: the forward-substituted border row) runs as
// dataflow tasks in the same launch
hipError_t launch_chol_dataflow(hipStream_t st, int npad, double* Hd, double* Linv, int* ready,
                                int epoch, int* flags, double* x = nullptr, const DfScatter* g = nullptr);
hipError_t launch_dense_factor_solve(hipStream_t st, int npad, double* Hd, double* Linv,
                                     double* x, int* flags, int epoch, const DfScatter* g = nullptr);
hipError_t launch_sp_tail_scatter(hipStream_t st, const double* xd, const int* tail, int ntail, double* x,
                                  const int* flags);
// multi-launch block-sparse elimination (gn_sparse.hip): one launch per round
// every elimination round (+ optionally the hybrid core's dense fill) in one cooperative launch
// Per round target, one record of kSpRec ints: {target, c0, c1, 0} then the first kSpInline
// contributions {v, code_r, code_s | W id, 0 | owner} inline (the rest from tc3 / rc4), so a
// workgroup's plan arrives in ONE load round trip with the flag.  Round rd's records start at
// tbeg + rbeg (its block targets, then its RHS targets).
constexpr int kSpInline = 9;
constexpr int kSpRec = 4 + 4 * kSpInline;
struct SpCoopArgs {
    const int *inl, *tc3, *rc4, *rounds, *tmap, *tail;
    double *A, *b, *Lstore, *W, *y, *Hd;
    int* flags;
    int nrounds, ntail, npad;
    int coop;  // 1: cooperative-groups grid sync; 0: own barrier (both as a cooperative launch)
};
hipError_t launch_sp_rounds_coop(hipStream_t st, const SpCoopArgs& args);
// The same rounds (and the hybrid core's fill) in one PLAIN launch without co-residency: the
// workgroups claim (round, target) tickets in order from a counter and a target waits for the
// previous round's completion count -- only ever on tickets running workgroups already hold.
// cnt: 4 + nrounds ints zeroed once (ticket, exits, spare, spare, per-round done counts); the last
// workgroup out re-zeroes them.  (gn_sparse.hip sp_rounds_df_kernel)
hipError_t launch_sp_rounds_df(hipStream_t st, const SpCoopArgs& args, int* cnt);
inline int sp_rounds_df_words(int nrounds) { return (4 + nrounds + 31) / 32 * 32; }
hipError_t launch_sp_round(hipStream_t st, const int* inl, int ibeg, int nbt, int nrt, const int* tc3,
                           const int* rc4, double* A, double* b, double* Lstore, double* W, double* y,
                           int* flags);
hipError_t launch_sp_back(hipStream_t st, int nnodes, const int* nodes, const int* fptr,
                          const int* fronts, int node_begin, const double* Lstore, const double* W,
                          const double* y, double* x, const int* flags);
hipError_t launch_sp_tail_fill(hipStream_t st, const double* A, const double* b, const int* tmap,
                               const int* tail, int ntail, int npad, double* Hd, const int* flags);
hipError_t launch_sp_tail(hipStream_t st, const double* A, const double* b, const int* tmap,
                          const int* tail, int ntail, int npad, double* Hd, double* Linv,
                          double* xd, double* x, int* flags, int epoch, bool fill = true);
hipError_t launch_fill_only(hipStream_t st, const double* compact, const int* slotmap, int nblk,
                            int npose, int n, int npad, double* Hd, const int* flags);
// The lagged-factor PCG (gn_pcg.hip).  X = A^-1 from the last direct solve's factor (the
// elimination rounds and the chol_df core), row-major [n][ldx], ldx = n rounded up to 64.
struct InvArgs {
    int n, ldx, nrounds, ntail, npad;
    const int *rounds, *nodes, *fptr, *fronts, *inl, *rc4, *tail;
    const double *Lstore, *W, *Hd, *Linv;
    double* X;       // [n][ldx] f64 work (the columns as they are solved)
    float* Xt;       // [n][ldt] f32: M row-major (= its columns: M is symmetric), what the PCG reads
    int ldt;         // n rounded up to 4
    const int* flags;
    long long* dbg;  // M3S_PCG_DEBUG: workgroup 0's phase clocks (6), else null
};
size_t inverse_lds_bytes(int npad);  // (the core's rows of 16 columns live in LDS: npad <= ~900)
hipError_t launch_sp_inverse(hipStream_t st, const InvArgs& a);
constexpr int kPcgThreads = 768;             // threads of a PCG workgroup
constexpr int kPcgMaxN = 2304;               // unknowns the PCG takes (3 vector entries per thread)
constexpr int kPcgMaxLds = 160 * 1024 - 1024;  // dynamic LDS of one PCG workgroup
struct PcgArgs {
    const double *b, *A;           // the block-format system (gn_assemble_kernel)
    const int* adj_ptr;            // per pose: its blocks (the diagonal first) ...
    const int2* adj;               // ... as (block, other pose)
    int nitem, R4;                 // max (row, block) items of a workgroup's rows (LDS), pcg_r4(R)
    const float* Xt;               // M (sp_inverse_kernel's f32 copy), row-major, ld ldt
    int ldt;
    int n, nv, R, nwg;             // unknowns, vector stride (pcg_nv), rows of M per workgroup, workgroups
    // onex: one exchange per CG step -- each workgroup also holds its rows of B = M A (f32, formed
    // in the launch's staging) and publishes (A p, B p) together: z is updated as z - alpha B p
    int onex;
    unsigned long long* gran;      // 2 x 2 x nv x 16 B: the exchanges' data-tagged granules (zeroed per call)
    unsigned tag0;                 // this launch's first tag (unique within the call)
    double tol2;                   // converged when r'z <= tol2 * r0'z0
    int kmax, spin_limit;
    float* Twc;
    float* dx;
    int N;
    float delta_thresh;
    int contract;
    int* flags;
    long long* dbg;                // M3S_PCG_DEBUG: phase clocks of workgroup 0 (kPcgDbgSlots), else null
};
constexpr int kPcgDbgSlots = 128;
constexpr int kPcgMaxR = 24;  // rows per workgroup with onex (B's row sums in registers)
int pcg_nv(int n);
int pcg_r4(int R);
size_t pcg_lds_bytes(int n, int R, int nitem, bool onex);
hipError_t launch_pcg(hipStream_t st, const PcgArgs& a);
// Fused single-workgroup solve (gn_solve.hip)
constexpr int kSolveThreads = 256;
#ifndef M3S_SOLVE_ROUND_THREADS
#define M3S_SOLVE_ROUND_THREADS 256
#endif
constexpr int kSolveRoundThreads = M3S_SOLVE_ROUND_THREADS;  // rounds-only launch of the split solve (512: VGPR spills, cfg2 5 us slower)
constexpr int kTailMax = 192;      // in-register dense tail: <= 192 unknowns (12 x 16-wide tiles)
constexpr int kTailPoseMax = 27;   // = kTailMax / 7
constexpr int kLStoreRec = 40;     // per eliminated pose: packed lower L (28) + 1/diag (7) + pad
constexpr int kSolveMaxLds = 160 * 1024 - 2048;  // dynamic LDS cap (static LDS besides)
constexpr int kSolveWStage = 6144;    // doubles: a round's W blocks staged in LDS
constexpr int kSolveRoundPoses = 64;  // poses per round (their y vectors staged in LDS)
struct SolveArgs {
    double *A, *b;          // block-format system (gn_assemble_kernel), updated in place
    double *y, *Lstore, *W, *Lg, *x;
    // the core as a dense row-major matrix (sp_tail_fill_kernel, leading dimension npad_h), or
    // nullptr: the in-register core then gathers its entries from the blocks
    const double* Hd;
    int npad_h;
    // the host plan: one int array; offsets of its parts.  rounds: 8 ints each (node_begin,
    // nnodes, tbeg, nbt, rbeg, nrt, wbeg, wcount); rc: (W id, node slot)
    const int* meta;
    int nmeta, meta_lds;  // meta_lds: stage it in LDS
    int o_rounds, o_nodes, o_fptr, o_fronts, o_tg, o_tc, o_rtg, o_rc, o_tail, o_tmap;
    int nrounds, ntail, npose, zero_blk;
    float* Twc;
    float* dx;
    int N;
    float delta_thresh;
    int* flags;
    int do_fwd, do_tail, do_back;  // rounds | in-kernel dense tail | back rounds + retract
    int debug;                     // M3S_SOLVE_DEBUG: phase times (wall clock, thread 0) ...
    unsigned long long* dbg;       // ... written here ({n, entry, exit, (code, time) x n}); the
                                   // driver prints them (no printf call in the kernel: a call
                                   // gives it a stack frame)
    int contract;                  // the retraction's M3S_CONTRACT_* (m3s_gn_args.contract)
    int x_tail_global;             // the dense core was solved by its own launch (chol_df): its x
                                   // is read from xd (the core's dense order) before the back rounds
    const double* xd;
};
size_t solve_lds_bytes(int nmeta_lds);
int solve_max_poses();  // x stays in LDS: the single-workgroup solve takes at most this many poses
constexpr int kSolveDbgCycles = 3 + 2 * 96;  // SolveArgs::dbg word: shader cycles over the launch
void print_solve_debug(const unsigned long long* host_copy);  // of SolveArgs::dbg
hipError_t launch_gn_solve(hipStream_t st, const SolveArgs& args);
// copy `bytes` (a multiple of 4; both addresses 16-B aligned) from pinned host memory (its
// device address) to device memory, stream-ordered, by a kernel
hipError_t launch_stage_copy(hipStream_t st, void* dst, const void* src_dev, size_t bytes);
// The accumulate's task records {edge, chunk, ix, jx} from the host's edge order (gn_driver.hip
// build_schedule_order): edge-major (off) or 8 XCD groups interleaved round-robin, each group's
// list chunk-major -- expanded on the device instead of written record by record into pinned
// memory and read back over PCIe.
struct SchedGroups {
    int lo[8], n[8];  // group g: edges order[lo[g] .. lo[g] + n[g])
    int big[8];       // the groups with n[g] = q + 1, ascending
    int nbig, q;      // q = min n[g]
    int off;          // 1: plain edge-major order (M3S_ACC_SCHED=0)
};
hipError_t launch_sched_expand(hipStream_t st, const int* order, const int* ii_loc, const int* jj_loc,
                               int nchunks, const SchedGroups& G, int64_t ntask, int* rec);
// flag[0] != 0 as an int (as_f64 = 0) or a double (as_f64 = 1) at dst (device-accessible)
hipError_t launch_flag_export(hipStream_t st, const int* flag, void* dst, int as_f64);
// save[0..n) = Twc[0..n) (before a call's first retraction)
hipError_t launch_twc_save(hipStream_t st, const float* Twc, float* save, int n);
// if the timeout flag (an int, or a double > 0 when flag_f64) is set: Twc[0..n) = save; the flag
// goes to dst (int 0/1, or the double) when dst != null
hipError_t launch_twc_restore_on_flag(hipStream_t st, float* Twc, const float* save, int n, const void* flag,
                                      int flag_f64, void* dst);
hipError_t launch_retract(hipStream_t st, float* Twc, const double* x, float* dx, int N,
                          float delta_thresh, int* flags, int contract);

}  // namespace m3s
