// gn_refacc.hip -- the reference-order ("parity") accumulate of the Sim3 Gauss-Newton backend.
//
// M3S_GN_ORDER_REFERENCE (m3s_gn_args.order / env M3S_GN_ORDER=reference): every directed edge
// is accumulated exactly the way the reference's ray_align / calib_proj / point_align kernels
// do it (gn_kernels.cu:813-1138, 1231-1543, 455-723):
//   * one 256-thread workgroup per directed edge, thread t owning points t, t+256, ...
//     (GPU_1D_KERNEL_LOOP, :31-32), one serial fp32 chain per thread and Hessian entry;
//   * the reference's per-point formulas: IEEE 1.0/x in double (as the equal f32 quotient), logf(zj) - logf(zi), the
//     compare-select Huber weight in double, sqrtf, the Jacobian pushed through
//     apply_Sim3_adj_inv(T_i) for EVERY point (:277-297), Ji = -Jj;
//   * the 256 partials reduced by blockReduce's tree (256 -> 128 -> 64 -> 32 -> ... -> 1,
//     :36-55);
//   * FMA contraction as the reference's nvcc build (--fmad=true) fuses this source
//     (m3s_gn_args.contract, default M3S_CONTRACT_NVCC; contract.h): `hij += w Jx[n] Jx[m]` is
//     one fma of the rounded w Jx[n] per term, `u = fx x/z + cx` an fma, the Sim3 library as in
//     sim3.h.  The file is compiled with contraction OFF; the helpers are its only fused ops.
// Output per edge: the 7x7 chain D[n][m] = sum (w Jj[n]) Jj[m] and g[n] = sum (w e) Jj[n] in
// f32 -- the reference's Hs/gs are exactly +-D / +-g (Ji = -Jj makes every one of the 119
// entries a negated copy of one of these 56 chains; negation commutes with every rounding,
// fused or not):
//   Hs[0] = Hs[3] = lower(D) mirrored, Hs[1] = -D^T, Hs[2] = -D, gs[0] = -g, gs[1] = g.
// gn_assemble_ref_kernel then builds the block system from the LOWER triangle of that
// (not exactly symmetric) matrix, as SimplicialLLT reads it (gn_kernels.cu:71-113, 132-153).
//
// This is the parity mode: its Hs/gs match the CPU oracle's (same convention) to a few ulp and its
// poses track the reference's float rounding; the default packed path (gn_accum.hip) is
// ~equally exact in absolute terms but sums in a different order.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "contract.h"
#include "gn_kernels.h"
#include "sim3.h"

#pragma clang fp contract(off)

namespace m3s {
namespace {

// gn_kernels.cu:172-175 (1.345 is a double literal).  Diagnostic variant kVarHuberMin: the fast
// path's min(1, 1.345 rcp|r|) (gn_accum.hip huber before round 2).
__device__ __forceinline__ float huber_ref(float r, int variant = 0) {
    const float r_abs = fabsf(r);
    if (variant & kRefVarHuberMin) return fminf(1.345f * __builtin_amdgcn_rcpf(r_abs), 1.0f);
    // the quotient unconditionally, then a select: the point math stays one basic block, so the
    // scheduler can interleave the unrolled points (gn_accum_ref_kernel)
    const double d = (double)r_abs;
    const float q = (float)(1.345 / d);
    return d < 1.345 ? 1.0f : q;
}

// (float)(1.0 / (double)x) -- or, diagnostic variant kRefVarRcp, the hardware v_rcp_f32.  Computed
// as the IEEE single-precision quotient 1.0f / x: a float quotient rounded to double and then to
// float equals the correctly rounded float quotient (double rounding is innocuous for division
// when the intermediate has >= 2p + 2 bits: 53 >= 2 * 24 + 2), at about half the f64 sequence's
// cost (matching.hip inv_f, the same identity)
__device__ __forceinline__ float inv_ref(float x, int variant) {
    if (variant & kRefVarRcp) return __builtin_amdgcn_rcpf(x);
    return __fdiv_rn(1.0f, x);
}

// gn_kernels.cu:277-297: Y = X Adj(T_i)^{-1} for a row vector X; Y[3..5] += s_inv (...) and
// Y[6] = X[6] + s_inv dot(t, Ra) are fused multiply-adds under nvcc
template <int CM>
__device__ __forceinline__ void adj_inv_ref(const Sim3f& Ti, float s_inv, const float* X, float* Y) {
    float Ra[3];
    act_so3<CM>(Ti.q, &X[0], Ra);
    Y[0] = s_inv * Ra[0];
    Y[1] = s_inv * Ra[1];
    Y[2] = s_inv * Ra[2];
    act_so3<CM>(Ti.q, &X[3], &Y[3]);
    Y[3] = cmad<CM>(s_inv, cmm<CM>(Ti.t[1], Ra[2], -Ti.t[2], Ra[1]), Y[3]);
    Y[4] = cmad<CM>(s_inv, cmm<CM>(Ti.t[2], Ra[0], -Ti.t[0], Ra[2]), Y[4]);
    Y[5] = cmad<CM>(s_inv, cmm<CM>(Ti.t[0], Ra[1], -Ti.t[1], Ra[0]), Y[5]);
    Y[6] = cmad<CM>(s_inv, cdot3<CM>(Ti.t[0], Ra[0], Ti.t[1], Ra[1], Ti.t[2], Ra[2]), X[6]);
}

// points per thread evaluated together before their rows are accumulated (A/B: -DM3S_REF_UNROLL=n).
// 1: 2, 3 and 4 measured 4-6 % slower on cfg3 (profiles/r05_af_refacc/), bitwise the same sums
#ifndef M3S_REF_UNROLL
#define M3S_REF_UNROLL 1
#endif
constexpr int kRefUnroll = M3S_REF_UNROLL;

struct RefAcc {
    float D[7][7];
    float g[7];
};

// The residual rows of one point: Jj = J Adj^{-1} (gn_kernels.cu:999-1000), the weight and the
// error per row -- all of the point's math, none of its accumulation
template <int MODE>
constexpr int ref_nrows() {
    return MODE == GN_RAYS ? 4 : 3;
}
template <int NR>
struct RefRows {
    float Jj[NR][7];
    float w[NR];
    float err[NR];
};

template <int CM, int NR>
__device__ __forceinline__ void set_row(RefRows<NR>& r, int row, const Sim3f& Ti, float s_inv, const float* J,
                                        float w, float err) {
    adj_inv_ref<CM>(Ti, s_inv, J, r.Jj[row]);
    r.w[row] = w;
    r.err[row] = err;
}

// hij += (w Jx[n]) Jx[m], vj += (w e) Jj[n] (gn_kernels.cu:1001-1013 and the two loops after it)
// on the 49 + 7 distinct chains, row after row
template <int CM, int NR>
__device__ __forceinline__ void accum_rows_ref(RefAcc& a, const RefRows<NR>& r) {
#pragma unroll
    for (int row = 0; row < NR; row++) {
        const float w = r.w[row];
#pragma unroll
        for (int n = 0; n < 7; n++) {
            const float wj = w * r.Jj[row][n];
#pragma unroll
            for (int m = 0; m < 7; m++) a.D[n][m] = cmad<CM>(wj, r.Jj[row][m], a.D[n][m]);
        }
        const float we = w * r.err[row];
#pragma unroll
        for (int n = 0; n < 7; n++) a.g[n] = cmad<CM>(we, r.Jj[row][n], a.g[n]);
    }
}

template <int MODE, int CM>
__device__ __forceinline__ void point_ref(const RefParams& P, const Sim3f& Ti, float si_inv,
                                          const Sim3f& Tij, const float* Xi, const float* Xj,
                                          float q, float ci, float cj, bool vm, int64_t ind,
                                          int variant, RefRows<ref_nrows<MODE>()>& a) {
    float Xj_Ci[3];
    act_sim3<CM>(Tij, Xj, Xj_Ci);  // actSim3 (:207-219)
    float J[7];
    if constexpr (MODE == GN_RAYS) {
        // gn_kernels.cu:924-1089
        const float norm2_i = cdot3<CM>(Xi[0], Xi[0], Xi[1], Xi[1], Xi[2], Xi[2]);
        const float norm1_i = sqrtf(norm2_i);
        const float norm1_i_inv = inv_ref(norm1_i, variant);
        const float norm2_j = cdot3<CM>(Xj_Ci[0], Xj_Ci[0], Xj_Ci[1], Xj_Ci[1], Xj_Ci[2], Xj_Ci[2]);
        const float norm1_j = sqrtf(norm2_j);
        const float norm1_j_inv = inv_ref(norm1_j, variant);
        const float rj[3] = {norm1_j_inv * Xj_Ci[0], norm1_j_inv * Xj_Ci[1], norm1_j_inv * Xj_Ci[2]};
        // rj - ri: a two-product difference (ri = norm1_i_inv Xi enters only here)
        const float err[4] = {cmm<CM>(norm1_j_inv, Xj_Ci[0], -norm1_i_inv, Xi[0]),
                              cmm<CM>(norm1_j_inv, Xj_Ci[1], -norm1_i_inv, Xi[1]),
                              cmm<CM>(norm1_j_inv, Xj_Ci[2], -norm1_i_inv, Xi[2]), norm1_j - norm1_i};
        const bool valid = vm & (q > P.Q_thresh) & (ci > P.C_thresh) & (cj > P.C_thresh);
        const float sqrt_w_ray = valid ? P.s0_inv * sqrtf(q) : 0.0f;
        const float sqrt_w_dist = valid ? P.s1_inv * sqrtf(q) : 0.0f;
        float w[4] = {huber_ref(sqrt_w_ray * err[0], variant), huber_ref(sqrt_w_ray * err[1], variant),
                      huber_ref(sqrt_w_ray * err[2], variant), huber_ref(sqrt_w_dist * err[3], variant)};
        const float wc_ray = sqrt_w_ray * sqrt_w_ray;
        const float wc_dist = sqrt_w_dist * sqrt_w_dist;
        w[0] *= wc_ray; w[1] *= wc_ray; w[2] *= wc_ray; w[3] *= wc_dist;
        const float norm3_j_inv = norm1_j_inv / norm2_j;
        const float drx_dPx = cmad<CM>(-(Xj_Ci[0] * Xj_Ci[0]), norm3_j_inv, norm1_j_inv);
        const float dry_dPy = cmad<CM>(-(Xj_Ci[1] * Xj_Ci[1]), norm3_j_inv, norm1_j_inv);
        const float drz_dPz = cmad<CM>(-(Xj_Ci[2] * Xj_Ci[2]), norm3_j_inv, norm1_j_inv);
        const float drx_dPy = ((-Xj_Ci[0]) * Xj_Ci[1]) * norm3_j_inv;
        const float drx_dPz = ((-Xj_Ci[0]) * Xj_Ci[2]) * norm3_j_inv;
        const float dry_dPz = ((-Xj_Ci[1]) * Xj_Ci[2]) * norm3_j_inv;
        J[0] = drx_dPx; J[1] = drx_dPy; J[2] = drx_dPz; J[3] = 0.0f; J[4] = rj[2]; J[5] = -rj[1]; J[6] = 0.0f;
        set_row<CM>(a, 0, Ti, si_inv, J, w[0], err[0]);
        J[0] = drx_dPy; J[1] = dry_dPy; J[2] = dry_dPz; J[3] = -rj[2]; J[4] = 0.0f; J[5] = rj[0]; J[6] = 0.0f;
        set_row<CM>(a, 1, Ti, si_inv, J, w[1], err[1]);
        J[0] = drx_dPz; J[1] = dry_dPz; J[2] = drz_dPz; J[3] = rj[1]; J[4] = -rj[0]; J[5] = 0.0f; J[6] = 0.0f;
        set_row<CM>(a, 2, Ti, si_inv, J, w[2], err[2]);
        J[0] = rj[0]; J[1] = rj[1]; J[2] = rj[2]; J[3] = 0.0f; J[4] = 0.0f; J[5] = 0.0f; J[6] = norm1_j;
        set_row<CM>(a, 3, Ti, si_inv, J, w[3], err[3]);
    } else if constexpr (MODE == GN_CALIB) {
        // gn_kernels.cu:1360-1495
        // ind in [0, HW), HW < 2^31: the 32-bit quotient (the same integers as the 64-bit one)
        const int v_target = (int)ind / P.width;
        const int u_target = (int)ind - v_target * P.width;
        const bool valid_z = (Xj_Ci[2] > P.z_eps) && (Xi[2] > P.z_eps);
        // evaluated unconditionally and selected (no branch in the point math)
        const float zj_inv_all = inv_ref(Xj_Ci[2], variant);
        const float zj_log_all = logf(Xj_Ci[2]), zi_log_all = logf(Xi[2]);
        const float zj_inv = valid_z ? zj_inv_all : 0.0f;
        float zj_log = valid_z ? zj_log_all : 0.0f;
        float zi_log = valid_z ? zi_log_all : 0.0f;
        if (variant & kRefVarLogRatio) {  // the fast path's ln2 * log2(zj / zi) before round 2
            zj_log = valid_z ? 0.69314718055994531f * __builtin_amdgcn_logf(Xj_Ci[2] * __builtin_amdgcn_rcpf(Xi[2]))
                             : 0.0f;
            zi_log = 0.0f;
        }
        const float x_div_z = Xj_Ci[0] * zj_inv;
        const float y_div_z = Xj_Ci[1] * zj_inv;
        const float u = cmad<CM>(P.fx, x_div_z, P.cx);
        const float v = cmad<CM>(P.fy, y_div_z, P.cy);
        const bool valid_u = (u > (float)P.pixel_border) && (u < (float)(P.width - 1 - P.pixel_border));
        const bool valid_v = (v > (float)P.pixel_border) && (v < (float)(P.height - 1 - P.pixel_border));
        const float err[3] = {u - (float)u_target, v - (float)v_target, zj_log - zi_log};
        const bool valid = vm & (q > P.Q_thresh) & (ci > P.C_thresh) & (cj > P.C_thresh) & valid_u &
                           valid_v & valid_z;
        const float sqrt_w_pixel = valid ? P.s0_inv * sqrtf(q) : 0.0f;
        const float sqrt_w_depth = valid ? P.s1_inv * sqrtf(q) : 0.0f;
        float w[3] = {huber_ref(sqrt_w_pixel * err[0], variant), huber_ref(sqrt_w_pixel * err[1], variant),
                      huber_ref(sqrt_w_depth * err[2], variant)};
        const float wc_pixel = sqrt_w_pixel * sqrt_w_pixel;
        const float wc_depth = sqrt_w_depth * sqrt_w_depth;
        w[0] *= wc_pixel; w[1] *= wc_pixel; w[2] *= wc_depth;
        const float fx = P.fx, fy = P.fy;
        J[0] = fx * zj_inv; J[1] = 0.0f; J[2] = ((-fx) * x_div_z) * zj_inv;
        J[3] = ((-fx) * x_div_z) * y_div_z; J[4] = fx * cmad<CM>(x_div_z, x_div_z, 1.0f);
        J[5] = (-fx) * y_div_z; J[6] = 0.0f;
        set_row<CM>(a, 0, Ti, si_inv, J, w[0], err[0]);
        J[0] = 0.0f; J[1] = fy * zj_inv; J[2] = ((-fy) * y_div_z) * zj_inv;
        J[3] = (-fy) * cmad<CM>(y_div_z, y_div_z, 1.0f); J[4] = (fy * x_div_z) * y_div_z;
        J[5] = fy * x_div_z; J[6] = 0.0f;
        set_row<CM>(a, 1, Ti, si_inv, J, w[1], err[1]);
        J[0] = 0.0f; J[1] = 0.0f; J[2] = zj_inv; J[3] = y_div_z; J[4] = -x_div_z; J[5] = 0.0f; J[6] = 1.0f;
        set_row<CM>(a, 2, Ti, si_inv, J, w[2], err[2]);
    } else {
        // point_align_kernel, gn_kernels.cu:564-674
        const float err[3] = {Xj_Ci[0] - Xi[0], Xj_Ci[1] - Xi[1], Xj_Ci[2] - Xi[2]};
        const bool valid = vm & (q > P.Q_thresh) & (ci > P.C_thresh) & (cj > P.C_thresh);
        const float sqrt_w_point = valid ? P.s0_inv * sqrtf(q) : 0.0f;
        float w[3] = {huber_ref(sqrt_w_point * err[0], variant), huber_ref(sqrt_w_point * err[1], variant),
                      huber_ref(sqrt_w_point * err[2], variant)};
        const float wc = sqrt_w_point * sqrt_w_point;
        w[0] *= wc; w[1] *= wc; w[2] *= wc;
        J[0] = 1.0f; J[1] = 0.0f; J[2] = 0.0f; J[3] = 0.0f; J[4] = Xj_Ci[2]; J[5] = -Xj_Ci[1]; J[6] = Xj_Ci[0];
        set_row<CM>(a, 0, Ti, si_inv, J, w[0], err[0]);
        J[0] = 0.0f; J[1] = 1.0f; J[2] = 0.0f; J[3] = -Xj_Ci[2]; J[4] = 0.0f; J[5] = Xj_Ci[0]; J[6] = Xj_Ci[1];
        set_row<CM>(a, 1, Ti, si_inv, J, w[1], err[1]);
        J[0] = 0.0f; J[1] = 0.0f; J[2] = 1.0f; J[3] = Xj_Ci[1]; J[4] = -Xj_Ci[0]; J[5] = 0.0f; J[6] = Xj_Ci[2];
        set_row<CM>(a, 2, Ti, si_inv, J, w[2], err[2]);
    }
}

}  // namespace

// One workgroup per local directed edge; out[e * kRefStride + 0..48] = D (row-major),
// out[.. + 49..55] = g, the blockReduce'd f32 sums.
// VAR: the diagnostic formula variants (RefParams::variant) are read at run time; the parity
// build (VAR = false) has none, so its point math carries no uniform branches between the points
template <int MODE, int CM, bool VAR>
__global__ __launch_bounds__(kAccThreads) void gn_accum_ref_kernel(
    const float* __restrict__ Twc, const float* __restrict__ Xs, const float* __restrict__ Cs,
    const int* __restrict__ ii_loc, const int* __restrict__ jj_loc, EdgeSrc es, RefParams P,
    float* __restrict__ out, const int* __restrict__ flags) {
    if (flags[kFlagDone]) return;
    const int e = blockIdx.x;
    const int tid = threadIdx.x;
    const int ix = ii_loc[e], jx = jj_loc[e];
    const Sim3f Ti = load_sim3(Twc + (int64_t)ix * 8);
    const Sim3f Tj = load_sim3(Twc + (int64_t)jx * 8);
    const Sim3f Tij = rel_sim3<CM>(Ti, Tj);
    const float si_inv = (float)(1.0 / (double)Ti.s);  // apply_Sim3_adj_inv's s_inv
    const int64_t HW = P.HW;
    const int64_t* idx_e;
    const uint8_t* valid_e;
    const float* Q_e;
    es.at(e, HW, idx_e, valid_e, Q_e);
    const int64_t* __restrict__ idx = idx_e;
    const uint8_t* __restrict__ valid = valid_e;
    const float* __restrict__ Q = Q_e;
    const float* __restrict__ Xi_b = Xs + (int64_t)ix * HW * 3;
    const float* __restrict__ Xj_b = Xs + (int64_t)jx * HW * 3;
    const float* __restrict__ Ci_b = Cs + (int64_t)ix * HW;
    const float* __restrict__ Cj_b = Cs + (int64_t)jx * HW;

    RefAcc a;
#pragma unroll
    for (int n = 0; n < 7; n++) {
#pragma unroll
        for (int m = 0; m < 7; m++) a.D[n][m] = 0.0f;
        a.g[n] = 0.0f;
    }
    // The thread's points k, k + 256, ... in order, U at a time: the U points' math first (one
    // basic block, no branch: the diagnostic variants are compiled out, the selects evaluate
    // both sides), then their rows accumulated in point order, so every chain sums the same
    // terms in the same order whatever U.
    constexpr int U = kRefUnroll;
    constexpr int NR = ref_nrows<MODE>();
    for (int64_t k0 = tid; k0 < HW; k0 += U * kAccThreads) {
        RefRows<NR> rows[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            // a point past the end is evaluated on the last point's inputs and not accumulated
            const int64_t k = min(k0 + (int64_t)u * kAccThreads, HW - 1);
            const bool vm = valid[k] != 0;
            const int64_t id = idx[k];  // loaded beside valid[k], not after it
            int64_t ind = vm ? id : 0;
            if ((uint64_t)ind >= (uint64_t)HW) ind = HW - 1;  // the reference reads out of bounds
            const float Xi[3] = {Xi_b[ind * 3], Xi_b[ind * 3 + 1], Xi_b[ind * 3 + 2]};
            const float Xj[3] = {Xj_b[k * 3], Xj_b[k * 3 + 1], Xj_b[k * 3 + 2]};
            point_ref<MODE, CM>(P, Ti, si_inv, Tij, Xi, Xj, Q[k], Ci_b[ind], Cj_b[k], vm, ind, VAR ? P.variant : 0,
                                rows[u]);
        }
        accum_rows_ref<CM>(a, rows[0]);
#pragma unroll
        for (int u = 1; u < U; u++)
            if (k0 + (int64_t)u * kAccThreads < HW) accum_rows_ref<CM>(a, rows[u]);
    }

    // blockReduce (gn_kernels.cu:36-55) of all 56 chains at once: level o adds s[t + o] into
    // s[t] for t < o (the warp-synchronous tail reads before it writes: the same pairing)
    __shared__ float s[kRefVals][kAccThreads];
#pragma unroll
    for (int n = 0; n < 7; n++) {
#pragma unroll
        for (int m = 0; m < 7; m++) s[n * 7 + m][tid] = a.D[n][m];
        s[49 + n][tid] = a.g[n];
    }
    __syncthreads();
    for (int o = kAccThreads / 2; o >= 1; o >>= 1) {
        // a thread reads s[q][t + o] (t + o >= o) and rewrites only its own s[q][t] (t < o):
        // no hazard inside a level
        for (int id = tid; id < kRefVals * o; id += kAccThreads) {
            const int q = id / o, t = id - q * o;
            s[q][t] = s[q][t] + s[q][t + o];
        }
        __syncthreads();
    }
    if (tid < kRefVals) out[(int64_t)e * kRefStride + tid] = s[tid][0];
}

// Block-format system (gn_solve.hip layout: b, then 49-f64 blocks, fill blocks zeroed) from the
// per-edge reference-order sums, reading the lower triangle of the reference's matrix like
// SimplicialLLT: contributions (el << 3 | type) in CSR order per slot, f64 sums.
//   type 0: +lower(D) mirrored (Hs[0] / Hs[3] on a diagonal block)
//   type 1: -D   (stored (min,max) orientation of Hs[2] placed at (jj, ii), ii > jj)
//   type 2: -D^T (Hs[1] placed at (ii, jj), ii < jj)
//   type 3 / 4: a self-edge's Hs[1] / Hs[2] on the diagonal: lower(-D^T) / lower(-D) mirrored
__global__ __launch_bounds__(64) void gn_assemble_ref_kernel(
    const float* __restrict__ ref, const int* __restrict__ blk_ptr, const int* __restrict__ blk_ref,
    const int* __restrict__ grad_ptr, const int* __restrict__ grad_ent, int nblk, int nblocks,
    int npose, int bpad, double* __restrict__ out, const int* __restrict__ flags) {
    if (flags[kFlagDone]) return;
    const int s = blockIdx.x;
    const int tid = threadIdx.x;
    if (s < nblk) {
        if (tid < 49) {
            const int r = tid / 7, c = tid % 7;
            double acc = 0.0;
            for (int k = blk_ptr[s]; k < blk_ptr[s + 1]; k++) {
                const int code = blk_ref[k];
                const float* D = ref + (int64_t)(code >> 3) * kRefStride;
                const int hi = r > c ? r : c, lo = r > c ? c : r;
                double v;
                switch (code & 7) {
                    case 0: v = (double)D[hi * 7 + lo]; break;
                    case 1: v = -(double)D[r * 7 + c]; break;
                    case 2: v = -(double)D[c * 7 + r]; break;
                    case 3: v = -(double)D[lo * 7 + hi]; break;
                    default: v = -(double)D[hi * 7 + lo]; break;
                }
                acc += v;
            }
            out[bpad + (int64_t)s * 49 + tid] = acc;
        }
    } else if (s < nblocks) {
        if (tid < 49) out[bpad + (int64_t)s * 49 + tid] = 0.0;
    } else {
        const int p = s - nblocks;
        if (p < npose && tid < 7) {
            double acc = 0.0;
            for (int k = grad_ptr[p]; k < grad_ptr[p + 1]; k++) {
                const int code = grad_ent[k];
                const double v = (double)ref[(int64_t)(code >> 1) * kRefStride + 49 + tid];
                acc += (code & 1) ? -v : v;  // gs[0] = -g at ii, gs[1] = g at jj
            }
            out[p * 7 + tid] = acc;
        }
    }
}

hipError_t launch_accum_ref(int mode, int E_local, hipStream_t st, const float* Twc, const float* Xs,
                            const float* Cs, const int* ii_loc, const int* jj_loc, const EdgeSrc& es,
                            const RefParams& P, float* out, const int* flags) {
    if (E_local <= 0) return hipSuccess;
#define M3S_REF(MODE, CM)                                                                                   \
    do {                                                                                                    \
        if (P.variant)                                                                                      \
            hipLaunchKernelGGL((gn_accum_ref_kernel<MODE, CM, true>), dim3(E_local), dim3(kAccThreads), 0, st, \
                               Twc, Xs, Cs, ii_loc, jj_loc, es, P, out, flags);                             \
        else                                                                                                \
            hipLaunchKernelGGL((gn_accum_ref_kernel<MODE, CM, false>), dim3(E_local), dim3(kAccThreads), 0, st, \
                               Twc, Xs, Cs, ii_loc, jj_loc, es, P, out, flags);                             \
    } while (0)
#define M3S_REF_MODES(CM)                     \
    if (mode == GN_RAYS) M3S_REF(GN_RAYS, CM); \
    else if (mode == GN_CALIB) M3S_REF(GN_CALIB, CM); \
    else M3S_REF(GN_POINTS, CM)
    if (P.contract == M3S_CONTRACT_OFF) M3S_REF_MODES(M3S_CONTRACT_OFF);
    else if (P.contract == M3S_CONTRACT_NVCC_RIGHT) M3S_REF_MODES(M3S_CONTRACT_NVCC_RIGHT);
    else M3S_REF_MODES(M3S_CONTRACT_NVCC);
#undef M3S_REF_MODES
#undef M3S_REF
    return hipGetLastError();
}

hipError_t launch_assemble_ref(hipStream_t st, const float* ref, const int* blk_ptr, const int* blk_ref,
                               const int* grad_ptr, const int* grad_ent, int nblk, int nblocks,
                               int npose, int bpad, double* out, const int* flags) {
    hipLaunchKernelGGL(gn_assemble_ref_kernel, dim3(nblocks + npose), dim3(64), 0, st, ref, blk_ptr,
                       blk_ref, grad_ptr, grad_ent, nblk, nblocks, npose, bpad, out, flags);
    return hipGetLastError();
}

}  // namespace m3s
