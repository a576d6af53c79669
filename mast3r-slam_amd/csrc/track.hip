// track.hip -- single-pair Sim3 Gauss-Newton of the frame tracker (gfx950).
//
// Replaces the torch loop of FrameTracker.opt_pose_ray_dist_sim3 / opt_pose_calib_sim3
// (reference mast3r_slam/tracker.py:173-266).  Per iteration the reference builds the
// whitened Jacobian A [4HW | 3HW, 7] and residual b with ~30 torch kernels, forms
// H = A^T A, g = -A^T b, synchronises on cost.item(), factors H with
// torch.linalg.cholesky and retracts with lietorch.  Here an iteration is two launches:
//   track_accum_kernel  one point per thread: residual and Jacobian (point_to_ray_dist |
//                       project_calib, act_Sim3; geometry.py:17-104), the huber-robustified
//                       sqrt-information (tracker.py:156-163), and the 28 + 7 unique entries
//                       of H, g plus the cost, reduced per workgroup (reduce-scatter, fixed
//                       order) -> one 36-float partial per workgroup
//   track_step_kernel   f64 sums of the partials in a fixed order (1008 threads), 7x7 Cholesky
//                       solve (tracker.py:164-169, in f64), T_CkCf <- Exp(tau) T_CkCf
//                       (lietorch retr), check_convergence (nonlinear_optimizer.py:5-25) ->
//                       a device flag that turns the remaining iterations into no-ops
// The host reads the flag every `check_every` iterations (one sync each) and returns once it is
// set: each live step writes the outputs itself (no final launch behind the host's check).  Deterministic:
// the same inputs give bitwise identical poses.
//
// Arithmetic follows the torch expressions (f32, python-float scalars rounded to f32 where
// torch rounds them); reductions are f32 per lane and f64 across lanes / workgroups, the
// solve is f64 -- the reference's f32 GEMM / Cholesky orders are not reproducible, so parity
// is to a tolerance (tests/test_gpu_track.py).  Invalid points are NOT skipped: their
// whitening factor is 0 and, as in the reference, a non-finite Jacobian still turns the
// system into NaN (which fails the Cholesky here).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>

#include "../../include/m3s_backend.h"
#include "m3s_common.h"
#include "sim3.h"
#include "wave_reduce.h"

namespace m3s {
namespace {

constexpr int kTrkThreads = 256;
constexpr int kTrkPPT = 1;  // points per thread (4 measured 2x slower: 192 workgroups, 4 dependent trips)
constexpr int kTrkNacc = 36;  // H upper triangle 28, g 7, sum of b^2
constexpr int kTrkMaxBlocks = 4096;

struct TrackState {
    float T[8];  // T_CkCf (lietorch data: t, q xyzw, s)
    double old_cost;
    double cost;
    int iters, converged, failed, done;
};

struct TrkParams {
    int HW;
    float s0, s1;  // 1/sigma, as the f32 scalar torch multiplies with
    float k;       // huber threshold (f32)
    float pb_lo, pb_hi_u, pb_hi_v, z_eps;
    double rel_error;
    float delta_norm;
    int max_iters;
};

// the partials are value-major, [kTrkNacc][ldp] with the row stride padded to 4 blocks, so the
// step kernel reads each value's blocks as float4 runs
__host__ __device__ inline int track_ldp(int nblk) { return (nblk + 3) & ~3; }

int track_blocks(int64_t HW) {
    const int64_t per = (int64_t)kTrkThreads * kTrkPPT;
    int64_t nb = (HW + per - 1) / per;
    if (nb < 1) nb = 1;
    if (nb > kTrkMaxBlocks) nb = kTrkMaxBlocks;
    return (int)nb;
}

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ---- lietorch Sim3 group operations (data layout t(3), q(4: x,y,z,w), s) ----

// X.act(p) = s R(q) p + t  (geometry.py:45-52 act_Sim3 -> lietorch act)
__device__ __forceinline__ void sim3_act(const float* T, const float* p, float* o) {
    float r[3];
    act_so3(T + 3, p, r);
    o[0] = T[7] * r[0] + T[0];
    o[1] = T[7] * r[1] + T[1];
    o[2] = T[7] * r[2] + T[2];
}

// X.inv() = (-(1/s) R(q)^-1 t, q^-1, 1/s)
__device__ __forceinline__ void sim3_inv(const float* T, float* o) {
    const float sinv = 1.0f / T[7];
    const float qi[4] = {-T[3], -T[4], -T[5], T[6]};
    float t[3];
    act_so3(qi, T, t);
    o[0] = -sinv * t[0];
    o[1] = -sinv * t[1];
    o[2] = -sinv * t[2];
    o[3] = qi[0]; o[4] = qi[1]; o[5] = qi[2]; o[6] = qi[3];
    o[7] = sinv;
}

// X * Y = (X.t + X.s R_X Y.t, X.q Y.q, X.s Y.s)
__device__ __forceinline__ void sim3_mul(const float* A, const float* B, float* o) {
    float t[3];
    act_so3(A + 3, B, t);
    float q[4];
    quat_comp(A + 3, B + 3, q);
    const float s = A[7] * B[7];
    o[0] = A[0] + A[7] * t[0];
    o[1] = A[1] + A[7] * t[1];
    o[2] = A[2] + A[7] * t[2];
    o[3] = q[0]; o[4] = q[1]; o[5] = q[2]; o[6] = q[3];
    o[7] = s;
}

// One residual row: accumulate A = ris * J (7) into H (upper 28), g -= A b, bb += b^2.
__device__ __forceinline__ void trk_row(float* acc, const float (&J)[7], float ris, float r) {
    float a[7];
#pragma unroll
    for (int c = 0; c < 7; c++) a[c] = ris * J[c];
    const float b = ris * r;
    int k = 0;
#pragma unroll
    for (int i = 0; i < 7; i++)
#pragma unroll
        for (int j = i; j < 7; j++) {
            acc[k] = fmaf(a[i], a[j], acc[k]);
            k++;
        }
#pragma unroll
    for (int i = 0; i < 7; i++) acc[28 + i] = fmaf(-a[i], b, acc[28 + i]);
    acc[35] = fmaf(b, b, acc[35]);
}

// J row = -(m^T dX/dxi) with dX/dxi = [I | -skew(X) | X] (act_Sim3, geometry.py:45-52)
__device__ __forceinline__ void trk_jrow(float m0, float m1, float m2, float x, float y, float z,
                                         float (&J)[7]) {
    J[0] = -m0;
    J[1] = -m1;
    J[2] = -m2;
    J[3] = m1 * z - m2 * y;
    J[4] = m2 * x - m0 * z;
    J[5] = m0 * y - m1 * x;
    J[6] = -((m0 * x + m1 * y) + m2 * z);
}

// huber weight (nonlinear_optimizer.py:28-33) -> robust sqrt information
__device__ __forceinline__ float trk_robust(float si, float r, float k) {
    const float wr = fabsf(si * r);
    const float w = wr < k ? 1.0f : k / wr;
    return si * sqrtf(w);
}

template <int MODE>
__global__ __launch_bounds__(kTrkThreads) void track_accum_kernel(
    const float* __restrict__ Xf, const float* __restrict__ Xk, const float* __restrict__ Qk,
    const uint8_t* __restrict__ valid, const float* __restrict__ meas,
    const uint8_t* __restrict__ vmeas, const float* __restrict__ K, const TrackState* __restrict__ st,
    TrkParams P, float* __restrict__ partials) {
    // the done flag is loaded with the pose and checked only after the point's loads and math, so
    // a live iteration does not wait one memory round trip for the flag before its loads (a
    // finished one computes its one point per thread and drops it)
    const bool done = st->done != 0;
    __shared__ float red[kTrkThreads / 64][kTrkNacc];
    float T[8];
#pragma unroll
    for (int q = 0; q < 8; q++) T[q] = st->T[q];
    float fx = 0.f, fy = 0.f, cx = 0.f, cy = 0.f;
    if constexpr (MODE == M3S_GN_CALIB) {
        fx = K[0];
        fy = K[4];
        cx = K[2];
        cy = K[5];
    }
    float acc[kTrkNacc];
#pragma unroll
    for (int q = 0; q < kTrkNacc; q++) acc[q] = 0.0f;

    const int stride = gridDim.x * kTrkThreads;
    for (int n = blockIdx.x * kTrkThreads + threadIdx.x; n < P.HW; n += stride) {
        const float pf[3] = {Xf[3 * n], Xf[3 * n + 1], Xf[3 * n + 2]};
        float X[3];
        sim3_act(T, pf, X);
        const float x = X[0], y = X[1], z = X[2];
        const float sq = sqrtf(Qk[n]);
        const float v = valid[n] ? 1.0f : 0.0f;
        if constexpr (MODE == M3S_GN_RAYS) {
            // point_to_ray_dist (geometry.py:17-34) of the frame point and of the keyframe point
            const float d = sqrtf((x * x + y * y) + z * z);
            const float dinv = 1.0f / d;
            const float rf0 = dinv * x, rf1 = dinv * y, rf2 = dinv * z;
            const float k0 = Xk[3 * n], k1 = Xk[3 * n + 1], k2 = Xk[3 * n + 2];
            const float dk = sqrtf((k0 * k0 + k1 * k1) + k2 * k2);
            const float dkinv = 1.0f / dk;
            const float r0 = dkinv * k0 - rf0, r1 = dkinv * k1 - rf1, r2 = dkinv * k2 - rf2;
            const float r3 = dk - d;
            // dr/dX = dinv (I - dinv^2 X X^T), dd/dX = r^T
            const float dinv2 = dinv * dinv;
            const float si_r = (P.s0 * v) * sq, si_d = (P.s1 * v) * sq;
            float J[7];
            trk_jrow(dinv * (1.0f - dinv2 * (x * x)), dinv * (0.0f - dinv2 * (x * y)),
                     dinv * (0.0f - dinv2 * (x * z)), x, y, z, J);
            trk_row(acc, J, trk_robust(si_r, r0, P.k), r0);
            trk_jrow(dinv * (0.0f - dinv2 * (y * x)), dinv * (1.0f - dinv2 * (y * y)),
                     dinv * (0.0f - dinv2 * (y * z)), x, y, z, J);
            trk_row(acc, J, trk_robust(si_r, r1, P.k), r1);
            trk_jrow(dinv * (0.0f - dinv2 * (z * x)), dinv * (0.0f - dinv2 * (z * y)),
                     dinv * (1.0f - dinv2 * (z * z)), x, y, z, J);
            trk_row(acc, J, trk_robust(si_r, r2, P.k), r2);
            trk_jrow(rf0, rf1, rf2, x, y, z, J);
            trk_row(acc, J, trk_robust(si_d, r3, P.k), r3);
        } else {
            // project_calib (geometry.py:63-104): p = K P / z, valid border / depth
            const float u = (fx * x + cx * z) / z;
            const float vv = (fy * y + cy * z) / z;
            const bool valid_z = z > P.z_eps;
            const bool ok = (u > P.pb_lo) && (u < P.pb_hi_u) && (vv > P.pb_lo) && (vv < P.pb_hi_v) &&
                            valid_z && vmeas[n];
            const float logz = valid_z ? logf(z) : 0.0f;
            const float m0 = meas[3 * n], m1 = meas[3 * n + 1], m2 = meas[3 * n + 2];
            const float r0 = m0 - u, r1 = m1 - vv, r2 = m2 - logz;
            const float zinv = 1.0f / z;
            const float w2 = ok ? 1.0f : 0.0f;
            const float si_p = w2 * ((P.s0 * v) * sq), si_z = w2 * ((P.s1 * v) * sq);
            float J[7];
            trk_jrow(fx * zinv, 0.0f, ((-fx * x) * zinv) * zinv, x, y, z, J);
            trk_row(acc, J, trk_robust(si_p, r0, P.k), r0);
            trk_jrow(0.0f, fy * zinv, ((-fy * y) * zinv) * zinv, x, y, z, J);
            trk_row(acc, J, trk_robust(si_p, r1, P.k), r1);
            trk_jrow(0.0f, 0.0f, zinv, x, y, z, J);
            trk_row(acc, J, trk_robust(si_z, r2, P.k), r2);
        }
    }
    if (done) return;
    // workgroup reduction in a fixed order: per wave a reduce-scatter (wave_reduce.h), then the
    // 4 waves in order; the partial goes to column blockIdx.x of the value-major [36][ldp] table
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    static_assert(kTrkNacc == 36, "wave_sum36 is laid out for 36 values");
    float x[9];
    wave_sum36(acc, x);
    if ((lane & 15) == 0) {
        const int r = lane >> 4;
#pragma unroll
        for (int j = 0; j < 9; j++) red[wave][j + 9 * r] = x[j];
    }
    __syncthreads();
    if (threadIdx.x < kTrkNacc) {
        float s = red[0][threadIdx.x];
#pragma unroll
        for (int w = 1; w < kTrkThreads / 64; w++) s += red[w][threadIdx.x];
        partials[(int64_t)threadIdx.x * track_ldp(gridDim.x) + blockIdx.x] = s;
    }
}

__global__ __launch_bounds__(64) void track_init_kernel(const float* __restrict__ T_WCf,
                                                        const float* __restrict__ T_WCk,
                                                        TrackState* __restrict__ st,
                                                        int* __restrict__ info) {
    if (threadIdx.x != 0) return;
    // T_CkCf = T_WCk.inv() * T_WCf (tracker.py:180, 225)
    float Ti[8], A[8], B[8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
        A[q] = T_WCk[q];
        B[q] = T_WCf[q];
    }
    sim3_inv(A, Ti);
    sim3_mul(Ti, B, st->T);
    st->old_cost = INFINITY;  // old_cost = float("inf")
    st->cost = 0.0;
    st->iters = st->converged = st->failed = st->done = 0;
    info[0] = info[1] = info[2] = info[3] = 0;
}

// the f64 sum of one value's partials runs as kTrkChains chains of consecutive blocks (one
// thread each, all its loads issued together: one memory round trip for up to 896 blocks), then
// the chains in order: a fixed order, so deterministic
constexpr int kTrkStepThreads = 1024;
constexpr int kTrkChains = 28;   // 36 x 28 = 1008 of the 1024 threads
constexpr int kTrkChainVec = 8;  // float4 loads in flight per chain and batch

__global__ __launch_bounds__(kTrkStepThreads) void track_step_kernel(const float* __restrict__ partials, int nblk,
                                                                 TrackState* __restrict__ st, TrkParams P,
                                                                 int* __restrict__ info,
                                                                 double* __restrict__ cost_out,
                                                                 const float* __restrict__ T_WCk,
                                                                 float* __restrict__ T_WCf_out,
                                                                 float* __restrict__ T_CkCf_out) {
    // the flag, the pose and the old cost are loaded together with the partials (one round trip)
    const bool done = st->done != 0;
    float T[8], Tk[8];
#pragma unroll
    for (int q = 0; q < 8; q++) T[q] = st->T[q];
#pragma unroll
    for (int q = 0; q < 8; q++) Tk[q] = T_WCk[q];
    const double old_cost = st->old_cost;
    const int iters = st->iters, converged0 = st->converged;
    __shared__ double S[kTrkNacc];
    __shared__ double C[kTrkNacc][kTrkChains];
    const int tid = threadIdx.x;
    if (tid < kTrkNacc * kTrkChains) {
        // chain c of value q: blocks [b0, b1), b0 a multiple of 4 (16-B aligned float4 runs; a run
        // may read up to 3 floats past b1 but never past the row's padded end)
        const int q = tid / kTrkChains, c = tid - q * kTrkChains;
        const int per = ((nblk + kTrkChains - 1) / kTrkChains + 3) & ~3;
        const int b0 = min(c * per, nblk), b1 = min(b0 + per, nblk);
        const float* __restrict__ row = partials + (int64_t)q * track_ldp(nblk);
        double s = 0.0;
        for (int b = b0; b < b1; b += 4 * kTrkChainVec) {
            float4 v[kTrkChainVec];
#pragma unroll
            for (int u = 0; u < kTrkChainVec; u++)
                v[u] = b + 4 * u < b1 ? *reinterpret_cast<const float4*>(row + b + 4 * u) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int u = 0; u < kTrkChainVec; u++) {
                const int bb = b + 4 * u;
                if (bb < b1) s += (double)v[u].x;
                if (bb + 1 < b1) s += (double)v[u].y;
                if (bb + 2 < b1) s += (double)v[u].z;
                if (bb + 3 < b1) s += (double)v[u].w;
            }
        }
        C[q][c] = s;
    }
    if (done) return;  // uniform: every thread read the same flag
    __syncthreads();
    if (tid < kTrkNacc) {
        double s = C[tid][0];
#pragma unroll
        for (int c = 1; c < kTrkChains; c++) s += C[tid][c];
        S[tid] = s;
    }
    __syncthreads();
    if (tid != 0) return;
    // H = A^T A, g = -A^T b, cost = 0.5 b^T b (tracker.py:164-166)
    double L[7][7], g[7];
    {
        int k = 0;
        for (int i = 0; i < 7; i++)
            for (int j = i; j < 7; j++) {
                L[j][i] = S[k];  // lower triangle
                k++;
            }
        for (int i = 0; i < 7; i++) g[i] = S[28 + i];
    }
    const double cost = 0.5 * S[35];
    // L L^T = H (tracker.py:168); a pivot that is not > 0 (incl. NaN) fails like torch
    bool bad = false;
    double rinv[7];
    for (int p = 0; p < 7; p++) {
        double d = L[p][p];
        for (int q = 0; q < p; q++) d -= L[p][q] * L[p][q];
        if (!(d > 0.0)) bad = true;
        const double lpp = sqrt(d);
        L[p][p] = lpp;
        rinv[p] = 1.0 / lpp;  // one division per pivot; the column and both solves multiply
        for (int i = p + 1; i < 7; i++) {
            double a = L[i][p];
            for (int q = 0; q < p; q++) a -= L[i][q] * L[p][q];
            L[i][p] = a * rinv[p];
        }
    }
    // every live step also writes the op's outputs, T_WCf = T_WCk * T_CkCf (tracker.py:212,
    // 264): the host returns as soon as it sees the done flag, with no final launch after it
    auto write_out = [&]() {
        float O[8];
        sim3_mul(Tk, T, O);
#pragma unroll
        for (int q = 0; q < 8; q++) {
            T_WCf_out[q] = O[q];
            T_CkCf_out[q] = T[q];
        }
    };
    if (bad) {
        st->failed = 1;
        st->done = 1;
        info[0] = iters;
        info[2] = 1;
        cost_out[0] = cost;
        write_out();
        return;
    }
    // tau = H^-1 g (cholesky_solve, tracker.py:169)
    double y[7], xs[7];
    for (int i = 0; i < 7; i++) {
        double a = g[i];
        for (int q = 0; q < i; q++) a -= L[i][q] * y[q];
        y[i] = a * rinv[i];
    }
    for (int i = 6; i >= 0; i--) {
        double a = y[i];
        for (int q = i + 1; q < 7; q++) a -= L[q][i] * xs[q];
        xs[i] = a * rinv[i];
    }
    float tau[7];
    float nrm2 = 0.0f;
    for (int i = 0; i < 7; i++) {
        tau[i] = (float)xs[i];
        nrm2 = fmaf(tau[i], tau[i], nrm2);
    }
    // T_CkCf = T_CkCf.retr(tau) = Exp(tau) * T_CkCf (tracker.py:195, 247)
    retr_sim3(tau, T);
    for (int q = 0; q < 8; q++) st->T[q] = T[q];
    // check_convergence (nonlinear_optimizer.py:5-25); inf old cost -> NaN -> not converged
    const double rel_dec = fabs((old_cost - cost) / old_cost);
    const float delta = sqrtf(nrm2);
    const bool conv = rel_dec < P.rel_error || delta < P.delta_norm;
    const int it1 = iters + 1;
    const int converged = conv ? 1 : converged0;
    st->old_cost = cost;
    st->cost = cost;
    st->iters = it1;
    st->converged = converged;
    if (conv || it1 >= P.max_iters) st->done = 1;
    info[0] = it1;
    info[1] = converged;
    info[2] = 0;
    cost_out[0] = cost;
    write_out();
}

__global__ __launch_bounds__(64) void track_final_kernel(const float* __restrict__ T_WCk,
                                                         const TrackState* __restrict__ st,
                                                         float* __restrict__ T_WCf_out,
                                                         float* __restrict__ T_CkCf_out) {
    if (threadIdx.x != 0) return;
    // T_WCf = T_WCk * T_CkCf (tracker.py:212, 264)
    float A[8], B[8], O[8];
    for (int q = 0; q < 8; q++) {
        A[q] = T_WCk[q];
        B[q] = st->T[q];
    }
    sim3_mul(A, B, O);
    for (int q = 0; q < 8; q++) {
        T_WCf_out[q] = O[q];
        T_CkCf_out[q] = B[q];
    }
}

// Pinned host copy of the state flags, one per host thread, released by m3s_shutdown (no
// exit-time destructor, m3s_common.h).
struct TrkFlags {
    TrackState* h = nullptr;
    // the last call on this thread: its workspace state, its stream, and whether h already holds
    // its final state (the call returned on a host check that saw the done flag)
    const TrackState* dev = nullptr;
    hipStream_t stream = nullptr;
    bool fresh = false;
    static void release(void* p) {
        TrkFlags* f = static_cast<TrkFlags*>(p);
        if (f->h) (void)hipHostFree(f->h);
        f->h = nullptr;
    }
};
thread_local TrkFlags* t_trk_flags = nullptr;
TrkFlags& trk_flags() {
    if (!t_trk_flags) {
        t_trk_flags = new TrkFlags;
        register_host_resource(t_trk_flags, &TrkFlags::release);
    }
    return *t_trk_flags;
}

}  // namespace
}  // namespace m3s

using namespace m3s;

extern "C" size_t m3s_track_workspace_bytes(int64_t HW) {
    if (HW < 1) return 0;
    return align_up(sizeof(TrackState), 256) + sizeof(float) * kTrkNacc * (size_t)track_ldp(track_blocks(HW));
}

extern "C" int m3s_track_sim3(const m3s_track_args* args) {
    M3S_REQUIRE(args != nullptr, "track_sim3: null args");
    const m3s_track_args& a = *args;
    M3S_REQUIRE(a.mode == M3S_GN_RAYS || a.mode == M3S_GN_CALIB, "track_sim3: bad mode %d", a.mode);
    M3S_REQUIRE(a.HW >= 1 && a.HW < ((int64_t)1 << 31), "track_sim3: bad point count %lld",
                (long long)a.HW);
    M3S_REQUIRE(a.Xf && a.Qk && a.valid && a.T_WCf && a.T_WCk && a.T_WCf_out && a.T_CkCf_out &&
                    a.info && a.cost,
                "track_sim3: null pointer");
    if (a.mode == M3S_GN_RAYS) M3S_REQUIRE(a.Xk != nullptr, "track_sim3: rays mode needs Xk");
    if (a.mode == M3S_GN_CALIB)
        M3S_REQUIRE(a.meas_k && a.valid_meas && a.K && a.width > 0 && a.height > 0,
                    "track_sim3: calib mode needs meas_k, valid_meas, K and the image size");
    M3S_REQUIRE(a.max_iters >= 0, "track_sim3: negative max_iters");
    const size_t need = m3s_track_workspace_bytes(a.HW);
    M3S_REQUIRE(a.ws && a.ws_bytes >= need, "track_sim3: workspace too small (%zu < %zu bytes)",
                a.ws_bytes, need);
    hipStream_t st = (hipStream_t)a.stream;
    TrackState* state = reinterpret_cast<TrackState*>(a.ws);
    float* partials = reinterpret_cast<float*>((char*)a.ws + align_up(sizeof(TrackState), 256));
    const int nblk = track_blocks(a.HW);

    TrkParams P;
    P.HW = (int)a.HW;
    // tracker.py:175-176 / 220-221: (1 / sigma) is a python float multiplied into f32 tensors
    P.s0 = (float)(1.0 / a.sigma0);
    P.s1 = (float)(1.0 / a.sigma1);
    P.k = (float)a.huber_k;
    P.pb_lo = (float)a.pixel_border;
    P.pb_hi_u = (float)(a.width - 1 - a.pixel_border);
    P.pb_hi_v = (float)(a.height - 1 - a.pixel_border);
    P.z_eps = (float)a.z_eps;
    P.rel_error = a.rel_error;
    P.delta_norm = (float)a.delta_norm;
    P.max_iters = a.max_iters;

    if (!trk_flags().h)
        M3S_HIP_CHECK(hipHostMalloc((void**)&trk_flags().h, sizeof(TrackState), hipHostMallocDefault));
    trk_flags().dev = state;
    trk_flags().stream = st;
    trk_flags().fresh = false;
    hipLaunchKernelGGL(track_init_kernel, dim3(1), dim3(64), 0, st, a.T_WCf, a.T_WCk, state, a.info);
    M3S_LAUNCH_CHECK();
    const int every = a.check_every > 0 ? a.check_every : 4;
    for (int it = 0; it < a.max_iters; it++) {
        if (a.mode == M3S_GN_RAYS)
            hipLaunchKernelGGL(track_accum_kernel<M3S_GN_RAYS>, dim3(nblk), dim3(kTrkThreads), 0, st,
                               a.Xf, a.Xk, a.Qk, a.valid, a.meas_k, a.valid_meas, a.K, state, P,
                               partials);
        else
            hipLaunchKernelGGL(track_accum_kernel<M3S_GN_CALIB>, dim3(nblk), dim3(kTrkThreads), 0, st,
                               a.Xf, a.Xk, a.Qk, a.valid, a.meas_k, a.valid_meas, a.K, state, P,
                               partials);
        M3S_LAUNCH_CHECK();
        hipLaunchKernelGGL(track_step_kernel, dim3(1), dim3(kTrkStepThreads), 0, st, partials, nblk, state, P,
                           a.info, a.cost, a.T_WCk, a.T_WCf_out, a.T_CkCf_out);
        M3S_LAUNCH_CHECK();
        if ((it + 1) % every == 0 && it + 1 < a.max_iters) {
            M3S_HIP_CHECK(hipMemcpyAsync(trk_flags().h, state, sizeof(TrackState),
                                         hipMemcpyDeviceToHost, st));
            M3S_HIP_CHECK(hipStreamSynchronize(st));
            if (trk_flags().h->done) {
                trk_flags().fresh = true;  // nothing is enqueued after this state
                break;
            }
        }
    }
    // the outputs were written by the last live step; with no iteration at all, from the start
    if (a.max_iters == 0) {
        hipLaunchKernelGGL(track_final_kernel, dim3(1), dim3(64), 0, st, a.T_WCk, state, a.T_WCf_out,
                           a.T_CkCf_out);
        M3S_LAUNCH_CHECK();
    }
    return M3S_OK;
}

// The last m3s_track_sim3 call's result on this host thread, to the host: {iterations, converged,
// cholesky failed, 0} and the cost.  When that call already synchronised on its done flag (the
// usual tracking case: converged before max_iters, seen at a host check) this reads the pinned copy
// without another device round trip; otherwise it copies the state on the call's stream (one
// synchronisation).  The workspace of that call must still be alive at the FIRST read after the
// call; that read drops the reference to the workspace, so later reads return the
// same host copy and never touch device memory the caller may have freed since.
extern "C" int m3s_track_last_result(int32_t* info4, double* cost) {
    M3S_REQUIRE(info4 != nullptr && cost != nullptr, "track_last_result: null pointer");
    TrkFlags& f = trk_flags();
    M3S_REQUIRE(f.h != nullptr && (f.dev != nullptr || f.fresh), "track_last_result: no track_sim3 call on this thread");
    if (!f.fresh) {
        M3S_HIP_CHECK(hipMemcpyAsync(f.h, f.dev, sizeof(TrackState), hipMemcpyDeviceToHost, f.stream));
        M3S_HIP_CHECK(hipStreamSynchronize(f.stream));
        f.fresh = true;
    }
    f.dev = nullptr;  // read: the host copy is final
    f.stream = nullptr;
    info4[0] = f.h->iters;
    info4[1] = f.h->converged;
    info4[2] = f.h->failed;
    info4[3] = 0;
    cost[0] = f.h->cost;
    return M3S_OK;
}
