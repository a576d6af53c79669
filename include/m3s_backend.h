/*
 * m3s_backend.h -- C ABI of the MI355X-native MASt3R-SLAM backend
 * (dense iterative-projection matching + Sim3 Gauss-Newton).
 *
 * This is the drop-in boundary that the Python module `mast3r_slam_backends`
 * (mast3r-slam_amd/mast3r_slam_backends) binds with ctypes.  Each entry point
 * replaces one pybind11 op of the reference module
 * (/root/reference/mast3r_slam/backend/src/gn.cpp:116-123; prototypes gn.h:22-117).
 *
 * Conventions
 *   - Every pointer is a DEVICE pointer to contiguous memory (torch.Tensor.data_ptr()).
 *     bool tensors are passed as uint8_t (0/1), fp16 as uint16_t bit patterns.
 *   - `stream` is a hipStream_t (torch.cuda.current_stream().cuda_stream); all work
 *     is enqueued on it.  Matching ops are fully asynchronous.  The GN ops perform
 *     one host synchronisation per call (to plan the sparse system from ii/jj),
 *     then enqueue all iterations without further host round trips.
 *   - Return value: M3S_OK (0) or an error code; m3s_last_error() gives a
 *     thread-local message.  The Python layer raises RuntimeError with it, as the
 *     reference's TORCH_CHECK does.
 */
#ifndef M3S_BACKEND_H
#define M3S_BACKEND_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    M3S_OK = 0,
    M3S_ERR_INVALID = 1, /* bad shape / argument */
    M3S_ERR_HIP = 2,     /* HIP runtime error */
    M3S_ERR_WORKSPACE = 3,
    M3S_ERR_COMM = 4,
    M3S_ERR_TIMEOUT = 5  /* a bounded device-side wait (dataflow factorisation / grid barrier)
                            gave up: the solve's result was discarded -- not a singular system */
};

const char* m3s_last_error(void);
/* Library build identifier ("m3s <version> gfx950"). */
const char* m3s_version(void);
/* Releases the library's cached host resources (pinned staging buffers, events).  Registered
 * with atexit when the library is loaded (and called by the Python module's atexit hook), so no
 * HIP call runs from a static or thread-local destructor during exit().  Idempotent; no other
 * entry point may be called afterwards. */
void m3s_shutdown(void);

/*
 * FMA-contraction convention of the reference build's float arithmetic.  The reference is built
 * by nvcc -O3 (setup.py:29-37: --fmad=true), which fuses a multiply into the add that consumes it;
 * for `a*b + c*d` the left product is fused (LLVM / NVPTX combine order).  The parity paths
 * (iter_proj, refine_matches f32/f64, the reference-order GN accumulate and the retraction)
 * restate that explicitly (mast3r-slam_amd/csrc/contract.h); OFF and NVCC_RIGHT are variants for
 * measuring the convention's effect.
 */
enum {
    M3S_CONTRACT_NVCC = 0,       /* nvcc --fmad=true, left product of a two-product sum fused */
    M3S_CONTRACT_OFF = 1,        /* IEEE multiply, then add (no fusion) */
    M3S_CONTRACT_NVCC_RIGHT = 2, /* the same as NVCC, right product fused */
    M3S_CONTRACT_DEFAULT = M3S_CONTRACT_NVCC  /* 0: a zero-initialised argument is the default */
};

/*
 * iter_proj -- replaces iter_proj (gn.cpp:84-99 -> matching_kernels.cu:279-316).
 *   rays      [B,H,W,9] f32  (ray, d/du, d/dv), H,W >= 3
 *   pts       [B,N,3]   f32  normalised target rays
 *   p_init    [B,N,2]   f32  initial (u,v) in image 1
 *   p_new     [B,N,2]   f32  out
 *   converged [B,N]     u8   out
 */
int m3s_iter_proj(const float* rays, const float* pts, const float* p_init,
                  float* p_new, uint8_t* converged,
                  int64_t B, int64_t H, int64_t W, int64_t N,
                  int max_iter, float lambda_init, float cost_thresh, void* stream);
/* The same with an explicit contraction convention (M3S_CONTRACT_*); m3s_iter_proj uses
 * M3S_CONTRACT_DEFAULT. */
int m3s_iter_proj_ex(const float* rays, const float* pts, const float* p_init,
                     float* p_new, uint8_t* converged,
                     int64_t B, int64_t H, int64_t W, int64_t N,
                     int max_iter, float lambda_init, float cost_thresh, int contract, void* stream);

/*
 * refine_matches -- replaces refine_matches (gn.cpp:101-114 -> matching_kernels.cu:84-116).
 *   D11 [B,H,W,F], D21 [B,N,F]  (fp16 bit patterns, f32 or f64: the reference's
 *   AT_DISPATCH_FLOATING_TYPES_AND_HALF, matching_kernels.cu:103)
 *   p1  [B,N,2] i64 (u,v) -> p1_new [B,N,2] i64
 */
int m3s_refine_matches_f16(const uint16_t* D11, const uint16_t* D21,
                           const int64_t* p1, int64_t* p1_new,
                           int64_t B, int64_t H, int64_t W, int64_t N, int64_t F,
                           int radius, int dilation_max, void* stream);
int m3s_refine_matches_f32(const float* D11, const float* D21,
                           const int64_t* p1, int64_t* p1_new,
                           int64_t B, int64_t H, int64_t W, int64_t N, int64_t F,
                           int radius, int dilation_max, void* stream);
int m3s_refine_matches_f64(const double* D11, const double* D21,
                           const int64_t* p1, int64_t* p1_new,
                           int64_t B, int64_t H, int64_t W, int64_t N, int64_t F,
                           int radius, int dilation_max, void* stream);

/*
 * match_iterative_proj -- the whole matching pipeline of the reference's Python caller
 * (matching.py:52-90: prep_for_iter_proj, iter_proj, p.long(), the occlusion test, refine on
 * .half() descriptors, pixel_to_lin) in five launches.  `contract`: iter_proj's M3S_CONTRACT_*.
 *   X11, X21  [B,H,W,3] f32      D11, D21 [B,H,W,F] f32
 *   idx_init  [B,H*W]   i64 or NULL (identity start)
 *   idx_out   [B,H*W]   i64 out  (u + W v)      valid_out [B,H*W] u8 out (bool)
 *   ws        device workspace of >= m3s_match_workspace_bytes(B, H, W, F) bytes
 */
size_t m3s_match_workspace_bytes(int64_t B, int64_t H, int64_t W, int64_t F);
int m3s_match_iterative_proj(const float* X11, const float* X21, const float* D11, const float* D21,
                             const int64_t* idx_init, int64_t B, int64_t H, int64_t W, int64_t F,
                             int max_iter, float lambda_init, float cost_thresh, float dist_thresh,
                             int radius, int dilation_max, int contract, int64_t* idx_out,
                             uint8_t* valid_out, void* ws, size_t ws_bytes, void* stream);

/* The measured-slower refine_matches variants (LDS tile, MFMA correlation, dot2) are not part of
 * this boundary: include/m3s_variants.h, lib/libm3s_variants.so. */

/* ---------------- Gauss-Newton ---------------- */

/* Diagnostics: with env M3S_GN_DEBUG_FLAGS set (2: silently), a GN call reads back its device
 * flags at the end (one extra synchronisation); out4 = {early exit, pivot failure, packed stream,
 * ray-constrained calib accumulate (Xj read as its depth)} of the last such call. */
void m3s_gn_debug_flags(int* out4);
/* The same call's lagged-factor PCG: out5 = {PCG solves, their CG steps in all,
 * PCG solves that fell back to the direct factorisation, 1 if the call planned PCG iterations,
 * the first PCG iteration (0 if none planned)}. */
void m3s_gn_pcg_stats(int* out5);

/* Deferred error report.  A GN call whose solver has bounded device-side waits (the dataflow
 * factorisation) exports its timeout flag without a host wait.  A call whose wait timed out
 * restores Twc to the poses it started from on the device (its result is discarded; every rank of
 * a sharded call restores), so it never commits poses.  M3S_ERR_TIMEOUT for it is returned by this
 * function, which synchronises `stream` (hipStream_t) first, or else by the next
 * m3s_gauss_newton_* call on the same host thread: that call checks the flag once its per-call
 * setup has synchronised the stream -- after the setup's own work (the edge-range exchange of a
 * sharded call, the plan uploads, the workspace allocation), before its first GN iteration -- and
 * returns without running an iteration.  m3s_gn_build_system and m3s_gn_edge_hessians do not
 * check it.  Env M3S_GN_TIMEOUT_SYNC=1 reports it from the call itself.  Returns M3S_OK,
 * M3S_ERR_TIMEOUT (then cleared) or M3S_ERR_HIP. */
int m3s_gn_check(void* stream);

enum { M3S_GN_POINTS = 0, M3S_GN_RAYS = 1, M3S_GN_CALIB = 2 };

/*
 * Common arguments of gauss_newton_{points,rays,calib} (gn.h:22-117).
 *   Twc   [N,8]  f32  poses [t(3), q(4, xyzw), s], UPDATED IN PLACE (pose 0 pinned)
 *   Xs    [N,HW,3] f32, Cs [N,HW] f32 (rows ordered by sorted unique keyframe id)
 *   ii,jj [E_total] i64 GLOBAL keyframe ids of the directed edges
 *   idx   [E_local,HW] i64, valid [E_local,HW] u8, Q [E_local,HW] f32 for the
 *         directed edges edge_offset .. edge_offset+E_local-1 (single GPU:
 *         edge_offset = 0, E_local = E_total)
 *   dx    [N-1,7] f32 out: the last iteration's update (the op's return value)
 *   ws    device workspace of >= m3s_gn_workspace_bytes(...) bytes
 *   comm  NULL, or an m3s communicator: the per-iteration compact Hessian is
 *         summed over ranks (RCCL all-reduce) before the replicated solve.
 */
typedef struct m3s_gn_args {
    int mode;
    float* Twc;
    const float* Xs;
    const float* Cs;
    const int64_t* ii;
    const int64_t* jj;
    const int64_t* idx;
    const uint8_t* valid;
    const float* Q;
    int64_t N, HW, E_total, E_local, edge_offset;
    /* residual parameters */
    float sigma0;           /* sigma_point | sigma_ray | sigma_pixel */
    float sigma1;           /* -           | sigma_dist | sigma_depth */
    float C_thresh, Q_thresh;
    const float* K;         /* calib: device [3,3] f32; fx,fy,cx,cy = K[0][0],K[1][1],K[0][2],K[1][2] */
    int height, width, pixel_border;
    float z_eps;
    int max_iter;
    float delta_thresh;
    float* dx;
    void* ws;
    size_t ws_bytes;
    void* comm;
    void* stream;
    /* summation order of the per-edge normal equations (M3S_GN_ORDER_*); 0 = the
     * default, overridable by the environment variable M3S_GN_ORDER=reference|fast */
    int order;
    /* Optional second half of the local edges' idx / valid / Q (NULL = one contiguous
     * tensor, the reference's layout): local directed edges 0 .. E_a-1 are rows of idx / valid
     * / Q, edges E_a .. E_local-1 are rows 0 .. E_local-E_a-1 of idx_b / valid_b / Q_b.  A
     * two-way edge store (forward edges, then the same pairs backward) is passed as its two
     * halves instead of the per-call concatenation of prep_two_way_edges
     * (global_opt.py:104-110). */
    const int64_t* idx_b;
    const uint8_t* valid_b;
    const float* Q_b;
    int64_t E_a;
    /* FMA-contraction convention (M3S_CONTRACT_*; 0 = the reference build's) of the
     * reference-order accumulate and of the retraction (the fast path's reformulated sums have
     * none to follow) */
    int contract;
} m3s_gn_args;
enum {
    M3S_GN_ORDER_DEFAULT = 0,
    /* packed stream, pre-adjoint rows, f32 lane chains of <= 32 points + f64 chunk sums
     * (gn_accum.hip): the fast path */
    M3S_GN_ORDER_FAST = 1,
    /* the reference kernels' own order and formulas (gn_refacc.hip): one 256-thread
     * workgroup per edge, 768-long fp32 chains per thread, blockReduce tree, per-point
     * apply_Sim3_adj_inv; the system read from its lower triangle like SimplicialLLT */
    M3S_GN_ORDER_REFERENCE = 2
};

size_t m3s_gn_workspace_bytes(int mode, int64_t N, int64_t HW, int64_t E_total, int64_t E_local);

/* Generic entry: replaces gauss_newton_{points,rays,calib}_cuda
 * (gn_kernels.cu:725-811, 1140-1228, 1546-1637). */
int m3s_gauss_newton(const m3s_gn_args* args);

/* Thin positional wrappers with the reference's argument order (gn.h). */
int m3s_gauss_newton_points(float* Twc, const float* Xs, const float* Cs,
                            const int64_t* ii, const int64_t* jj, const int64_t* idx,
                            const uint8_t* valid, const float* Q,
                            int64_t N, int64_t HW, int64_t E,
                            float sigma_point, float C_thresh, float Q_thresh,
                            int max_iter, float delta_thresh,
                            float* dx, void* ws, size_t ws_bytes, void* stream);
int m3s_gauss_newton_rays(float* Twc, const float* Xs, const float* Cs,
                          const int64_t* ii, const int64_t* jj, const int64_t* idx,
                          const uint8_t* valid, const float* Q,
                          int64_t N, int64_t HW, int64_t E,
                          float sigma_ray, float sigma_dist, float C_thresh, float Q_thresh,
                          int max_iter, float delta_thresh,
                          float* dx, void* ws, size_t ws_bytes, void* stream);
int m3s_gauss_newton_calib(float* Twc, const float* Xs, const float* Cs, const float* K,
                           const int64_t* ii, const int64_t* jj, const int64_t* idx,
                           const uint8_t* valid, const float* Q,
                           int64_t N, int64_t HW, int64_t E,
                           int height, int width, int pixel_border, float z_eps,
                           float sigma_pixel, float sigma_depth, float C_thresh, float Q_thresh,
                           int max_iter, float delta_thresh,
                           float* dx, void* ws, size_t ws_bytes, void* stream);

/*
 * Debug / test entry: run ONE accumulate + assemble pass with the current Twc and
 * write the dense normal equations H [n,n] and b [n] (n = 7(N-1), f64, host
 * pointers), i.e. the system SparseBlock builds (gn_kernels.cu:71-113).
 */
int m3s_gn_build_system(const m3s_gn_args* args, double* H_host, double* b_host);
/*
 * Debug / test entry: ONE reference-order accumulate pass (gn_refacc.hip) with the current
 * Twc, returning exactly the tensors the reference's align kernels write
 * (gn_kernels.cu:1096-1137): Hs [4, E_local, 7, 7] f32 and gs [2, E_local, 7] f32 (host).
 */
int m3s_gn_edge_hessians(const m3s_gn_args* args, float* Hs_host, float* gs_host);

/*
 * Diagnostic (host only, no GPU): the elimination plan m3s_gauss_newton would build for this
 * pose graph -- the step the reference leaves to Eigen's SimplicialLLT symbolic analysis on every
 * solve (gn_kernels.cu:132-153).  ii, jj [E] host i64 global keyframe ids (as the op's), N
 * poses (the first pinned).  info[8]: [0] solver (0 single-workgroup fused, 1 hybrid, 2
 * multi-launch, -1 nothing to solve), [1] elimination rounds, [2] poses eliminated by the
 * rounds, [3] poses in the dense core, [4] the core's padded unknowns, [5] pose pairs (graph
 * blocks off the diagonal), [6] plan integers uploaded per call, [7] 1 if the core fits the
 * dense solve limit.  order (optional, N-1 ints): the poses (0-based rows after the pinned one)
 * round by round, each round ascending, then the core's.  round_ptr (optional, round_cap ints):
 * where each round starts in order, then the core's start -- written when round_cap >=
 * rounds + 1.  Environment knobs as for the op.
 */
int m3s_gn_plan_info(const int64_t* ii, const int64_t* jj, int64_t E, int64_t N, int32_t* info,
                     int32_t* order, int32_t* round_ptr, int32_t round_cap);

/*
 * Phase timing (bench.py): between m3s_prof_begin() and m3s_prof_end() every GN
 * iteration records HIP events on its stream.  out[0] = accumulate kernel ms,
 * out[1] = edge reduce + compact (+ all-reduce) ms, out[2] = solve ms, out[3] = retract
 * ms, summed over the *n_iter recorded iterations.  Not thread-safe; test/bench only.
 */
int m3s_prof_begin(void);
/* The same, recording only the two events around each accumulate launch (every timed event
 * record idles the GPU ~5 us): m3s_prof_end then fills out[0] and *n_iter with the iteration
 * kernel's launches, out[1] / out[2] with the ms and count of the launches that also built the
 * packed records (a calib call's first accumulate, M3S_GN_PACK_FIRST), out[3] = 0. */
int m3s_prof_begin_accum(void);
int m3s_prof_end(double* out /* [4] */, int* n_iter);
/* After an m3s_prof_begin_accum() .. m3s_prof_end() session: the iteration kernel's per-launch
 * ms (out[0 .. min(n, cap) - 1]); returns n, the number of launches recorded (bench.py reports
 * their min / median / max: the accumulate's spread within one run). */
int m3s_prof_launch_ms(double* out, int cap);
/* After an m3s_prof_begin() .. m3s_prof_end() session: each recorded iteration's solve ms
 * (out[0 .. min(n, cap) - 1], call after call); returns n. */
int m3s_prof_solve_ms(double* out, int cap);

/* ---------------- frame tracking (single-pair Sim3 GN) ---------------- */

/*
 * track_sim3 -- replaces the torch loop of FrameTracker.opt_pose_ray_dist_sim3 /
 * opt_pose_calib_sim3 (/root/reference/mast3r_slam/tracker.py:173-266) with its solve
 * (:156-171), huber (nonlinear_optimizer.py:28-33), check_convergence (:5-25) and the
 * residual models point_to_ray_dist / act_Sim3 / project_calib (geometry.py:17-104).
 * The reference has no native op for this (it is torch + lietorch); this entry is an
 * extension of the drop-in module (mast3r_slam_backends.track_sim3).
 *   mode      M3S_GN_RAYS (ray + distance residual, 4 rows) or M3S_GN_CALIB (pixel +
 *             log-depth, 3 rows)
 *   Xf        [HW,3] f32  frame points already gathered by the match (Xf[idx_f2k])
 *   Xk        [HW,3] f32  keyframe points (rays mode; unused by calib)
 *   Qk        [HW]   f32  match confidence sqrt(Qff[idx] * Qkf)
 *   valid     [HW]   u8   valid_opt
 *   meas_k    [HW,3] f32  calib: (u, v, log z) of the keyframe pixel (0 where invalid)
 *   valid_meas[HW]   u8   calib: z_k > depth_eps
 *   K         [3,3]  f32  calib intrinsics (device)
 *   T_WCf, T_WCk [8] f32  lietorch Sim3 data (t, q xyzw, s) (device)
 *   T_WCf_out, T_CkCf_out [8] f32 (device, out)
 *   info      [4] i32 (device, out): iterations run, converged, cholesky failed, 0
 *   cost      [1] f64 (device, out): cost of the last linearisation
 * The python-float parameters (sigmas, huber k, thresholds) are passed as double and
 * rounded where torch rounds them.  One host synchronisation per `check_every`
 * iterations (the reference syncs on every iteration's `.item()`).  A non-positive (or
 * NaN) Cholesky pivot stops the loop and sets info[2] -- the caller raises, as
 * torch.linalg.cholesky does (tracker.py:91).
 */
typedef struct m3s_track_args {
    int mode;
    const float* Xf;
    const float* Xk;
    const float* Qk;
    const uint8_t* valid;
    const float* meas_k;
    const uint8_t* valid_meas;
    const float* K;
    const float* T_WCf;
    const float* T_WCk;
    int64_t HW;
    int height, width, pixel_border;
    double z_eps;
    double sigma0;          /* sigma_ray   | sigma_pixel */
    double sigma1;          /* sigma_dist  | sigma_depth */
    double huber_k;
    int max_iters;
    double rel_error, delta_norm;
    int check_every;        /* iterations between host checks of the convergence flag */
    float* T_WCf_out;
    float* T_CkCf_out;
    int* info;
    double* cost;
    void* ws;
    size_t ws_bytes;
    void* stream;
} m3s_track_args;

size_t m3s_track_workspace_bytes(int64_t HW);
int m3s_track_sim3(const m3s_track_args* args);
/* The last m3s_track_sim3 call's result on this host thread, on the host: info4 = {iterations,
 * converged, cholesky failed, 0}, *cost (the same values as the call's device `info` / `cost`).
 * Free of a device round trip when the call returned on a host check that saw its done flag
 * (converged before max_iters); otherwise it synchronises the call's stream once.  That call's
 * workspace must still be allocated at the first read after the call, which drops the reference
 * to it: later reads (same thread, no new call) return the same host copy without touching device
 * memory.  Per host thread: another thread's calls are not seen.  Extension (the reference's
 * tracker reads them with .item()). */
int m3s_track_last_result(int32_t* info4, double* cost);

/* ---------------- edge construction after matching ---------------- */

/*
 * edge_confidence -- the per-pixel glue of FactorGraph.add_factors (global_opt.py:53-67) in one
 * pass over B keyframe pairs:
 *   Qj = sqrt(Qii[b, idx_i2j] * Qji), Qi = sqrt(Qjj[b, idx_j2i] * Qij)     [B,HW] f32 out
 *   counts[b] = (#(valid_match_j & Qj > Q_conf), #(valid_match_i & Qi > Q_conf))  [B,2] i32 out
 *   idx_* [B,HW] i64, valid_match_* [B,HW] u8, Q* [B,HW] f32.  Bit-exact (same f32 ops).
 */
int m3s_edge_confidence(const int64_t* idx_i2j, const int64_t* idx_j2i,
                        const uint8_t* valid_match_j, const uint8_t* valid_match_i,
                        const float* Qii, const float* Qjj, const float* Qji, const float* Qij,
                        float Q_conf, int64_t B, int64_t HW, float* Qj, float* Qi, int* counts,
                        void* stream);

/* ---------------- keyframe point-map fusion ---------------- */

enum { M3S_FILTER_WEIGHTED_POINTMAP = 0, M3S_FILTER_INDEP_CONF = 1, M3S_FILTER_RECENT = 2 };

/*
 * pointmap_update -- replaces Frame.update_pointmap (frame.py:41-105) for the per-point
 * filtering modes (weighted_pointmap :74-77, indep_conf :69-73, recent :58-61), fused with
 * the transform of the new observation the tracker applies first (tracker.py:98-99).
 *   T      [8] f32 Sim3 data applied to X_new (lietorch act), or NULL for none
 *   X_new  [HW,3], C_new [HW] f32; X [HW,3], C [HW] f32 updated in place
 * Bit-exact against the torch expressions on the same (transformed) inputs.
 */
int m3s_pointmap_update(int mode, const float* T, const float* X_new, const float* C_new,
                        float* X, float* C, int64_t HW, void* stream);

/* ---------------- multi-GPU (RCCL over xGMI) ---------------- */

/*
 * Communicator of the edge-sharded GN op (m3s_gn_args.comm): every iteration the compact
 * block-sparse system (f64) is sum-all-reduced in place before the replicated solve.  The
 * reference is single-GPU (its solve runs in Eigen on the host, gn_kernels.cu:1201-1209);
 * this is the seam SURVEY.md section 8(e) adds.
 */
#define M3S_COMM_ID_BYTES 128
/* RCCL over xGMI (production).  Rank 0 creates the id, the caller broadcasts it (e.g.
 * torch.distributed), every rank calls m3s_comm_init. */
int m3s_comm_get_unique_id(void* id_out /* M3S_COMM_ID_BYTES */);
int m3s_comm_init(const void* id, int nranks, int rank, void** comm_out);
/* Host-callback collective (test hook): the library drains the stream, stages the `count`
 * doubles in pinned host memory and calls fn(user, buf, count), which must replace buf with
 * the element-wise sum over ranks (e.g. a torch.distributed gloo all_reduce) and return 0. */
typedef int (*m3s_host_allreduce_fn)(void* user, double* buf, size_t count);
int m3s_comm_init_host(m3s_host_allreduce_fn fn, void* user, int nranks, int rank, void** comm_out);
int m3s_comm_destroy(void* comm);
/* The number of ranks the communicator spans, as its transport reports it (RCCL:
 * ncclCommCount; host callback: the count it was created with). */
int m3s_comm_size(void* comm, int* nranks_out);

#ifdef __cplusplus
}
#endif
#endif
