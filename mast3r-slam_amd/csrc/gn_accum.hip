// gn_accum.hip -- the per-iteration accumulate of the Sim3 Gauss-Newton backend (gfx950).
//
//   gn_pack_kernel           once per call: the iteration-invariant packed stream
//                            {match index | invalid bit, sqrt q} per directed point-edge
//   gn_depth_kernel          once per call (calib): the keyframes' depths as a dense array
//   gn_accum_packed_kernel   per iteration: accumulate the unique entries of
//                            M = sum w r r^T and g = sum w e r over RAW (pre-adjoint) Jacobian
//                            rows from the packed stream (>= 3 iterations per call)
//   gn_accum_kernel          per iteration, reading the reference's tensors directly
// Replaces ray_align / calib_proj / point_align (reference gn_kernels.cu:813-1138, 1231-1543,
// 455-723); the adjoint and the 4-block expansion happen per edge in gn_kernels.hip.
// Built with -fno-slp-vectorize (Makefile): the SLP vectorizer re-packs the scalar path into
// v_pk ops with register shuffles (204 instead of 92 VGPRs).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdint>

#include "edge_reduce.h"
#include "gn_kernels.h"
#include "sim3.h"
#include "wave_reduce.h"

// Scheduling of the 4 points of a lane's step (AccStage::compute): 0 (default; what every
// measurement so far ran -- the old default of 1 sat below its first use and never applied) lets
// the compiler interleave the points freely, 1 fences after every point (one point's temporaries
// live at a time), 2 after every second point.
#ifndef M3S_ACC_SCHED_BARRIER
#define M3S_ACC_SCHED_BARRIER 0
#endif
// Diagnostics builds only (tools/build_variants.sh; the results are NOT the normal equations):
// 1 = the packed accumulate's compute alone, 2 = its memory traffic alone.
#ifndef M3S_ACC_DIAG
#define M3S_ACC_DIAG 0
#endif

namespace m3s {

// ---------------------------------------------------------------------------
// Point math, one point-edge per call, generic in the value type V (float here; a packed
// float2 pair variant was measured: on gfx950 a v_pk_*_f32 op costs the SIMD twice the cycles
// of a scalar one, so pairs only save issue slots while doubling the accumulator VGPRs
// (144 vs 92, 3 vs 5 waves/SIMD) and ran 10 % slower -- the kernel is latency-bound).
// ---------------------------------------------------------------------------
template <typename V>
struct VMask {
    typedef bool type;
};

__device__ __forceinline__ float vfma(float a, float b, float c) { return fmaf(a, b, c); }
__device__ __forceinline__ float vsplat(float s, float) { return s; }
__device__ __forceinline__ float vrcp(float a) { return __builtin_amdgcn_rcpf(a); }    // v_rcp_f32
__device__ __forceinline__ float vsqrt(float a) { return __builtin_amdgcn_sqrtf(a); }  // normal or 0 inputs
// sqrt(q) of the point records: correctly rounded, as the reference's sqrtf(conf_weight)
// (gn_kernels.cu:1404-1405; nvcc's sqrtf is IEEE).  Computed once per call (the record builders:
// the pack, the first accumulate, the unpacked path of 1-2 iteration calls), so the ~10 extra
// VALU of the exact expansion are off the iteration kernel.
__device__ __forceinline__ float sqrt_cr(float a) { return __builtin_sqrtf(a); }
__device__ __forceinline__ float vlog2(float a) { return __builtin_amdgcn_logf(a); }   // inputs > z_eps
// rays mode's normalisation (M3S_RAYS_CR): 0 (default) = the hardware v_sqrt_f32 / v_rcp_f32
// (1 ulp); 1 = correctly rounded sqrtf and v_rcp_f32 + one Newton step (the reference's sqrtf /
// 1.0/x are correctly rounded); 2 = v_rsq_f32 + one Newton step.  Measured (tools/
// accuracy_probe.py, profiles/r03_rays_norm_ab.json): the first GN step of cfg4 lands 2.13e-5 /
// 2.11e-5 / 2.16e-5 (of max |dx|) from the exactly summed system with 0 / 1 / 2 -- the per-point
// ulp errors average out in the 4e8-term sums -- while 1 and 2 cost 16 % / 13 % accumulate time.
#ifndef M3S_RAYS_CR
#define M3S_RAYS_CR 0
#endif
__device__ __forceinline__ float vrcp_nr(float a) {
    const float r = __builtin_amdgcn_rcpf(a);
    return fmaf(fmaf(-a, r, 1.0f), r, r);
}
// 1/sqrt(a): v_rsq_f32 plus one Newton step y (1.5 - 0.5 a y^2) (~0.5 ulp)
__device__ __forceinline__ float vrsq_nr(float a) {
    const float y = __builtin_amdgcn_rsqf(a);
    const float h = 0.5f * a * y;
    return fmaf(fmaf(-h, y, 0.5f), y, y);
}
__device__ __forceinline__ float vabs(float a) { return fabsf(a); }
__device__ __forceinline__ float vmin(float a, float b) { return fminf(a, b); }
__device__ __forceinline__ float vsel(bool m, float a, float b) { return m ? a : b; }
__device__ __forceinline__ bool vgt(float a, float b) { return a > b; }
__device__ __forceinline__ bool vlt(float a, float b) { return a < b; }
__device__ __forceinline__ bool vand(bool a, bool b) { return a && b; }

// Huber weight (gn_kernels.cu:172-175): |r| < 1.345 ? 1 : 1.345/|r| as a compare-select, so a
// NaN residual gives a NaN weight like the reference (a min(1, .) form turns it into 1); the
// reciprocal is v_rcp_f32 (1 ulp; DESIGN.md §2 measures what that costs).
template <typename V>
__device__ __forceinline__ V huber(V r) {
    const V a = vabs(r);
    return vsel(vlt(a, 1.345f), vsplat(1.0f, r), vsplat(1.345f, r) * vrcp(a));
}

// Accumulate one raw Jacobian row r (compile-time nonzero mask) with weight w, residual e.
template <int MASK, typename V>
__device__ __forceinline__ void acc_row(V* __restrict__ acc, const V* r, V w, V e) {
    V wr[7];
#pragma unroll
    for (int a = 0; a < 7; a++) wr[a] = (MASK >> a & 1) ? w * r[a] : V(0.0f);
#pragma unroll
    for (int a = 0; a < 7; a++) {
        if (!(MASK >> a & 1)) continue;
#pragma unroll
        for (int b = a; b < 7; b++) {
            if (!(MASK >> b & 1)) continue;
            acc[sym_idx(a, b)] = vfma(wr[a], r[b], acc[sym_idx(a, b)]);
        }
    }
#pragma unroll
    for (int a = 0; a < 7; a++)
        if (MASK >> a & 1) acc[28 + a] = vfma(wr[a], e, acc[28 + a]);
}

template <typename V>
struct PointsIn {
    // calib: xi2 carries the matched point's INVERSE depth, (z > z_eps) ? v_rcp_f32(z) : NaN (the
    // packed path gathers it precomputed per call, gn_depth_kernel; NaN encodes z <= z_eps)
    V xi0, xi1, xi2, xj0, xj1, xj2;
    V sq;                            // sqrt(q)
    typename VMask<V>::type valid;   // match & q > Q_thresh & ci > C_thresh & cj > C_thresh
    V ut, vt;  // calib: pixel of the match, (ind % W, ind / W) as float
};

// T_ij as the 3x4 affine map it applies to a point.  The reference's act_so3
// (gn_kernels.cu:195-205) computes x + w uv + q x uv with uv = 2 q x x, which is linear in x:
// M = I + 2w[q]x + 2[q]x^2 (exactly that map, unit quaternion or not); actSim3 then scales and
// translates (gn_kernels.cu:252-272).  Formed once per workgroup, s M x + t costs 9 FMAs per
// point instead of the 24 operations of the quaternion formula.  The two differ by float
// rounding only; on the bench graphs the normal equations built this way are closer to the
// exactly summed reference system than the quaternion form's, and
// gn_refacc.hip keeps the reference's own formula for the parity mode.
struct RelXf {
    float m[9];  // s * M, row-major
    float t[3];
};

__device__ __forceinline__ RelXf rel_xf(const Sim3f& T) {
    const float x = T.q[0], y = T.q[1], z = T.q[2], w = T.q[3], s = T.s;
    const float xx = x * x, yy = y * y, zz = z * z;
    const float xy = x * y, xz = x * z, yz = y * z, wx = w * x, wy = w * y, wz = w * z;
    RelXf R;
    R.m[0] = s * (1.0f - 2.0f * (yy + zz));
    R.m[1] = s * (2.0f * (xy - wz));
    R.m[2] = s * (2.0f * (xz + wy));
    R.m[3] = s * (2.0f * (xy + wz));
    R.m[4] = s * (1.0f - 2.0f * (xx + zz));
    R.m[5] = s * (2.0f * (yz - wx));
    R.m[6] = s * (2.0f * (xz - wy));
    R.m[7] = s * (2.0f * (yz + wx));
    R.m[8] = s * (1.0f - 2.0f * (xx + yy));
    R.t[0] = T.t[0];
    R.t[1] = T.t[1];
    R.t[2] = T.t[2];
    // workgroup-uniform: keep the 12 coefficients in SGPRs (VALU operands), not VGPRs
#pragma unroll
    for (int k = 0; k < 9; k++) R.m[k] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(R.m[k])));
#pragma unroll
    for (int k = 0; k < 3; k++) R.t[k] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(R.t[k])));
    return R;
}

template <typename V>
__device__ __forceinline__ void apply_rel(const RelXf& T, V x0, V x1, V x2, V& X0, V& X1, V& X2) {
    X0 = vfma(vsplat(T.m[0], x0), x0, vfma(vsplat(T.m[1], x0), x1, vfma(vsplat(T.m[2], x0), x2, vsplat(T.t[0], x0))));
    X1 = vfma(vsplat(T.m[3], x0), x0, vfma(vsplat(T.m[4], x0), x1, vfma(vsplat(T.m[5], x0), x2, vsplat(T.t[1], x0))));
    X2 = vfma(vsplat(T.m[6], x0), x0, vfma(vsplat(T.m[7], x0), x1, vfma(vsplat(T.m[8], x0), x2, vsplat(T.t[2], x0))));
}

// One (pair of) point-edge(s) from its transformed point X = T_ij Xj: residuals, robust
// weights, raw rows -> acc.
template <int MODE, typename V>
__device__ __forceinline__ void point_body_x(const PointsIn<V>& p, V X0, V X1, V X2, const AccParams& P,
                                             V* __restrict__ acc) {
    auto valid = p.valid;
    const V zero = vsplat(0.0f, X0);
    const V sq = p.sq;

    if constexpr (MODE == GN_RAYS) {
        // gn_kernels.cu:924-1089
        const V n2i = vfma(p.xi0, p.xi0, vfma(p.xi1, p.xi1, p.xi2 * p.xi2));
        const V n2j = vfma(X0, X0, vfma(X1, X1, X2 * X2));
#if M3S_RAYS_CR == 1
        const V n1i = __builtin_sqrtf(n2i);
        const V n1i_inv = vrcp_nr(n1i);
        const V n1j = __builtin_sqrtf(n2j);
        const V n1j_inv = vrcp_nr(n1j);
#elif M3S_RAYS_CR == 2
        const V n1i_inv = vrsq_nr(n2i);
        const V n1i = n2i * n1i_inv;
        const V n1j_inv = vrsq_nr(n2j);
        const V n1j = n2j * n1j_inv;
#else
        const V n1i = vsqrt(n2i);
        const V n1i_inv = vrcp(n1i);
        const V n1j = vsqrt(n2j);
        const V n1j_inv = vrcp(n1j);
#endif
        const V rx = n1j_inv * X0, ry = n1j_inv * X1, rz = n1j_inv * X2;
        const V e0 = rx - n1i_inv * p.xi0;
        const V e1 = ry - n1i_inv * p.xi1;
        const V e2 = rz - n1i_inv * p.xi2;
        const V e3 = n1j - n1i;
        const V swr = vsel(valid, vsplat(P.s0_inv, sq) * sq, zero);
        const V swd = vsel(valid, vsplat(P.s1_inv, sq) * sq, zero);
        const V wcr = swr * swr, wcd = swd * swd;
        const V w0 = huber(swr * e0) * wcr;
        const V w1 = huber(swr * e1) * wcr;
        const V w2 = huber(swr * e2) * wcr;
        const V w3 = huber(swd * e3) * wcd;
#if M3S_RAYS_CR == 2
        const V n3 = n1j_inv * n1j_inv * n1j_inv;
#elif M3S_RAYS_CR
        const V n3 = n1j_inv * vrcp_nr(n2j);
#else
        const V n3 = n1j_inv * vrcp(n2j);
#endif
        const V dxx = n1j_inv - X0 * X0 * n3;
        const V dyy = n1j_inv - X1 * X1 * n3;
        const V dzz = n1j_inv - X2 * X2 * n3;
        const V dxy = -X0 * X1 * n3;
        const V dxz = -X0 * X2 * n3;
        const V dyz = -X1 * X2 * n3;
        {
            const V r[7] = {dxx, dxy, dxz, zero, rz, -ry, zero};
            acc_row<0b0110111>(acc, r, w0, e0);
        }
        {
            const V r[7] = {dxy, dyy, dyz, -rz, zero, rx, zero};
            acc_row<0b0101111>(acc, r, w1, e1);
        }
        {
            const V r[7] = {dxz, dyz, dzz, ry, -rx, zero, zero};
            acc_row<0b0011111>(acc, r, w2, e2);
        }
        {
            const V r[7] = {rx, ry, rz, zero, zero, zero, n1j};
            acc_row<0b1000111>(acc, r, w3, e3);
        }
    } else if constexpr (MODE == GN_CALIB) {
        // gn_kernels.cu:1360-1495
        const auto valid_z = vand(vgt(X2, P.z_eps), p.xi2 == p.xi2);  // zi > z_eps <=> 1/zi not NaN
        const V zj_inv = vsel(valid_z, vrcp(X2), zero);
        // log(zj) - log(zi) (gn_kernels.cu:1385-1390) as ln2 * log2(zj / zi): the residual is a
        // small difference of two ~unit logs, so one log of the ratio keeps it to ~1e-7
        // relative where two float logs lose ~1e-4 of it to cancellation (inf/NaN still
        // propagate: 1/inf = 0 -> -inf).
        const V e2 = vsel(valid_z, vsplat(0.69314718055994531f, X2) * vlog2(X2 * p.xi2), zero);
        const V x = X0 * zj_inv, y = X1 * zj_inv;
        const V u = vfma(vsplat(P.fx, x), x, vsplat(P.cx, x));
        const V v = vfma(vsplat(P.fy, y), y, vsplat(P.cy, y));
        valid = vand(vand(valid, valid_z),
                     vand(vand(vgt(u, P.pb_lo), vlt(u, P.pb_hi_u)), vand(vgt(v, P.pb_lo), vlt(v, P.pb_hi_v))));
        const V e0 = u - p.ut;
        const V e1 = v - p.vt;
        const V swp = vsel(valid, vsplat(P.s0_inv, sq) * sq, zero);
        const V swd = vsel(valid, vsplat(P.s1_inv, sq) * sq, zero);
        const V wcp = swp * swp, wcd = swd * swd;
        const V w0 = huber(swp * e0) * wcp;
        const V w1 = huber(swp * e1) * wcp;
        const V w2 = huber(swd * e2) * wcd;
        const V one = vsplat(1.0f, x);
        const V xz = x * zj_inv, yz = y * zj_inv, xy = x * y;
#ifndef M3S_CALIB_FOLD_F
#define M3S_CALIB_FOLD_F 1
#endif
#if M3S_CALIB_FOLD_F
        // the pixel rows are f * r' (r' = the normalised-plane row): w r r^T = (w f^2) r' r'^T and
        // w r e = (w f^2) r' (e / f), so the focal lengths fold into the weight and the residual
        // (2 multiplies per row instead of 5)
        const float fx2 = P.fx * P.fx, fy2 = P.fy * P.fy, fx_inv = 1.0f / P.fx, fy_inv = 1.0f / P.fy;
        {
            const V r[7] = {zj_inv, zero, -xz, -xy, vfma(x, x, one), -y, zero};
            acc_row<0b0111101>(acc, r, w0 * vsplat(fx2, x), e0 * vsplat(fx_inv, x));
        }
        {
            const V r[7] = {zero, zj_inv, -yz, -vfma(y, y, one), xy, x, zero};
            acc_row<0b0111110>(acc, r, w1 * vsplat(fy2, x), e1 * vsplat(fy_inv, x));
        }
#else
        const V fx = vsplat(P.fx, x), fy = vsplat(P.fy, x);
        {
            const V r[7] = {fx * zj_inv, zero, -fx * xz, -fx * xy, fx * vfma(x, x, one), -fx * y, zero};
            acc_row<0b0111101>(acc, r, w0, e0);
        }
        {
            const V r[7] = {zero, fy * zj_inv, -fy * yz, -fy * vfma(y, y, one), fy * xy, fy * x, zero};
            acc_row<0b0111110>(acc, r, w1, e1);
        }
#endif
        {
            const V r[7] = {zero, zero, zj_inv, y, -x, zero, one};
            acc_row<0b1011100>(acc, r, w2, e2);
        }
    } else {
        // point_align_kernel, gn_kernels.cu:564-674
        const V e0 = X0 - p.xi0, e1 = X1 - p.xi1, e2 = X2 - p.xi2;
        const V swp = vsel(valid, vsplat(P.s0_inv, sq) * sq, zero);
        const V wc = swp * swp;
        const V w0 = huber(swp * e0) * wc;
        const V w1 = huber(swp * e1) * wc;
        const V w2 = huber(swp * e2) * wc;
        const V one = vsplat(1.0f, X0);
        {
            const V r[7] = {one, zero, zero, zero, X2, -X1, X0};
            acc_row<0b1110001>(acc, r, w0, e0);
        }
        {
            const V r[7] = {zero, one, zero, -X2, zero, X0, X1};
            acc_row<0b1101010>(acc, r, w1, e1);
        }
        {
            const V r[7] = {zero, zero, one, X1, -X0, zero, X2};
            acc_row<0b1011100>(acc, r, w2, e2);
        }
    }
}

template <int MODE, typename V>
__device__ __forceinline__ void point_body(const PointsIn<V>& p, const RelXf& T, const AccParams& P,
                                           V* __restrict__ acc) {
    V X0, X1, X2;
    apply_rel(T, p.xj0, p.xj1, p.xj2, X0, X1, X2);
    point_body_x<MODE, V>(p, X0, X1, X2, P, acc);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// Match index of a point: invalid -> 0 (the reference's `valid ? idx : 0`); an index outside
// [0, HW) is clamped to HW-1 (the reference would read out of bounds).
__device__ __forceinline__ int match_index(int64_t id, bool vm, int HW) {
    const uint64_t u = (uint64_t)id;
    const int c = u < (uint64_t)HW ? (int)u : HW - 1;
    return vm ? c : 0;
}

// calib: the per-call inverse depths follow the depths Zs [nkf * HW] and the ray tables (<= HW
// floats): IZs = Zs + (nkf + 1) * HW (gn_depth_kernel; the driver sizes the region)
__device__ __forceinline__ float* inv_depths(float* Zs, const AccParams& P) {
    return Zs + ((int64_t)P.nkf + 1) * P.HW;
}
__device__ __forceinline__ const float* inv_depths(const float* Zs, const AccParams& P) {
    return Zs + ((int64_t)P.nkf + 1) * P.HW;
}

// ind / W and ind % W exactly by multiply-shift (Granlund-Montgomery, ind < 2^31).
__device__ __forceinline__ void pixel_of(int ind, const AccParams& P, float& ut, float& vt) {
    const unsigned q = (unsigned)(((uint64_t)(unsigned)ind * P.div_m) >> P.div_sh);
    vt = (float)(int)q;
    ut = (float)(ind - (int)q * P.width);
}

// The packed calib record's match (code & 0x7fffffff = v << 16 | u, AccParams::pack_uv): its
// flat index v W + u (24-bit multiply-add) and its pixel as floats.
__device__ __forceinline__ int uv_index(int code, int width) {
    return (int)__umul24((unsigned)(code >> 16) & 0x7fffu, (unsigned)width) + (code & 0xffff);
}
__device__ __forceinline__ void uv_pixel(int code, float& ut, float& vt) {
    ut = (float)(code & 0xffff);
    vt = (float)((code >> 16) & 0x7fff);
}
// the pack's record code for match index ind (valid or not: bit 31 marks invalid)
__device__ __forceinline__ int pack_code(int ind, bool ok, const AccParams& P) {
    int c = ind;
    if (P.pack_uv) {
        const unsigned q = (unsigned)(((uint64_t)(unsigned)ind * P.div_m) >> P.div_sh);
        c = (int)(q << 16) | (ind - (int)q * P.width);
    }
    return ok ? c : (int)((unsigned)c | 0x80000000u);
}

// Deterministic workgroup reduction of the 35 sums, one 36-float partial per (edge, chunk).
// Per wave a reduce-scatter: 36 values -> 18 (32-lane halves) -> 9 (16-lane rows, row r of
// register j holding value j + 9r), then a 16-lane row sum (126 lane ops instead of the
// 35 x 6 shuffle-adds of a butterfly per value); then the 4 waves in fixed order.
__device__ __forceinline__ void block_partial(const float* accs, float* __restrict__ out, bool coh = false) {
    __shared__ float red[kAccThreads / 64][kNaccPad];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    static_assert(kNaccPad == 36, "reduce-scatter is laid out for 36 values");
    float w[18], x[9];
#pragma unroll
    for (int j = 0; j < 18; j++) w[j] = halfsum32(accs[j], j + 18 < kNacc ? accs[j + 18] : 0.0f);
#pragma unroll
    for (int j = 0; j < 9; j++) x[j] = row_sum16(halfsum16(w[j], w[j + 9]));
    if ((lane & 15) == 0) {
        const int r = lane >> 4;
#pragma unroll
        for (int j = 0; j < 9; j++) red[wave][j + 9 * r] = x[j];
    }
    __syncthreads();
    if (tid < kNacc) {
        float s = red[0][tid];
#pragma unroll
        for (int w = 1; w < kAccThreads / 64; w++) s += red[w][tid];
        if (coh)  // write-through: read by the edge's last workgroup, possibly on another XCD
            __hip_atomic_store(out + tid, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
            out[tid] = s;
    }
}


// The ray-constrained calib stream's transform factored per pixel row (AccStage::compute; A/B
// builds: -DM3S_RC_FACTOR=0 keeps s M x + t on the rebuilt point, bitwise the positional stream)
#ifndef M3S_RC_FACTOR
#define M3S_RC_FACTOR 1
#endif

// One pipeline stage of the packed accumulate: the records, Xj and the gathered matched points
// of 4 consecutive points of one lane.
// PK: the packed path's conventions (calib: the matched inverse depth gathered from Zi_b, the
// record codes are pixels, AccParams::pack_uv); else the unpacked kernel's (raw depth from Xs,
// codes are flat indices).  NP: consecutive points per lane and step (4, or 2 for the packed
// path without RC: fewer loads in flight, fewer VGPRs).
template <int MODE, bool RC = false, bool PK = true, int NP = 4>
struct AccStage {
    static_assert(NP == 4 || NP == 2, "4 or 2 points per step");
    // the records {code, sqrt q} as scalars: kept as two int4 members, the struct was not split
    // into registers (a 16-B stack / LDS round trip per step in the ISA)
    int cd[NP], sb[NP];
    __device__ __forceinline__ void set(int4 a, int4 b) {
        cd[0] = a.x; sb[0] = a.y; cd[1] = a.z; sb[1] = a.w;
        if constexpr (NP == 4) {
            cd[2] = b.x; sb[2] = b.y; cd[3] = b.z; sb[3] = b.w;
        }
    }
    float xv[3 * NP];    // Xj of the points (RC: xv[0..NP) their depths, xv[NP..2NP) tu[u..], xv[2NP] tv[v])
    float g[NP][3];      // gathered matched point (calib: depth only, in g[s][2])
    const float* rc_tu = nullptr;  // RC: the ray tables (after Zs)
    const float* rc_tv = nullptr;
    unsigned rc_m = 0;             // RC: k / W by multiply-shift
    int rc_sh = 0, rc_w = 1;
    int width = 1;                 // PK calib: the image width (record pixel -> flat index)

    template <int M>
    __device__ __forceinline__ void load(const float* __restrict__ Xj_b, const float* __restrict__ Xi_b,
                                         const float* __restrict__ Zi_b, int k) {
        if constexpr (RC) {
            // Xj_b = the depth row of keyframe j; the ray tables follow Zs (gn_depth_kernel)
            // (the NP points share a row: k is a multiple of NP and W of 4)
            const unsigned q = (unsigned)(((uint64_t)(unsigned)k * rc_m) >> rc_sh);
            const int u = k - (int)q * rc_w;
            if constexpr (NP == 4) {
                const float4 za = *reinterpret_cast<const float4*>(Xj_b + k);
                const float4 ta = *reinterpret_cast<const float4*>(rc_tu + u);
                const float t[8] = {za.x, za.y, za.z, za.w, ta.x, ta.y, ta.z, ta.w};
#pragma unroll
                for (int i = 0; i < 8; i++) xv[i] = t[i];
            } else {
                const float2 za = *reinterpret_cast<const float2*>(Xj_b + k);
                const float2 ta = *reinterpret_cast<const float2*>(rc_tu + u);
                xv[0] = za.x; xv[1] = za.y; xv[2] = ta.x; xv[3] = ta.y;
            }
            xv[2 * NP] = rc_tv[q];
        } else if constexpr (NP == 4) {
            const float4 a = *reinterpret_cast<const float4*>(Xj_b + (int64_t)k * 3);
            const float4 b = *reinterpret_cast<const float4*>(Xj_b + (int64_t)k * 3 + 4);
            const float4 c = *reinterpret_cast<const float4*>(Xj_b + (int64_t)k * 3 + 8);
            const float t[12] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
#pragma unroll
            for (int i = 0; i < 12; i++) xv[i] = t[i];
        } else {
            const float2 a = *reinterpret_cast<const float2*>(Xj_b + (int64_t)k * 3);
            const float2 b = *reinterpret_cast<const float2*>(Xj_b + (int64_t)k * 3 + 2);
            const float2 c = *reinterpret_cast<const float2*>(Xj_b + (int64_t)k * 3 + 4);
            const float t[6] = {a.x, a.y, b.x, b.y, c.x, c.y};
#pragma unroll
            for (int i = 0; i < 6; i++) xv[i] = t[i];
        }
        int ind[NP];
#pragma unroll
        for (int s = 0; s < NP; s++) ind[s] = (M == GN_CALIB && PK) ? uv_index(cd[s], width) : (cd[s] & 0x7fffffff);
#pragma unroll
        for (int s = 0; s < NP; s++) {
            if constexpr (M == GN_CALIB) {
                if constexpr (PK)
                    g[s][2] = Zi_b[ind[s]];
                else
                    g[s][2] = Xi_b[(int64_t)ind[s] * 3 + 2];
            } else {
                const float* xp = Xi_b + (int64_t)ind[s] * 3;
                g[s][0] = xp[0];
                g[s][1] = xp[1];
                g[s][2] = xp[2];
            }
        }
    }

    // the points one at a time on scalar accumulators
    template <int M>
    __device__ __forceinline__ void compute(const RelXf& T, const AccParams& P, float* __restrict__ acc) const {
        const int* codes = cd;
        const int* sqb = sb;
        float xj[3 * NP];
        // RC_FACTOR: the ray-constrained point is z (tu, tv, 1), so T_ij Xj = z (tu M_0 + B_v) + t
        // with B_v = tv M_1 + M_2 shared by the lane's NP points (one pixel row): 6 FMAs per point
        // and 3 per step instead of 2 multiplies + 9 FMAs per point (other roundings than the
        // positional stream's s M x + t)
        constexpr bool kFactor = RC && M == GN_CALIB && M3S_RC_FACTOR;
        float Xr[3 * NP];
        if constexpr (kFactor) {
            const float tv = xv[2 * NP];
            const float B0 = fmaf(T.m[1], tv, T.m[2]), B1 = fmaf(T.m[4], tv, T.m[5]), B2 = fmaf(T.m[7], tv, T.m[8]);
#pragma unroll
            for (int s = 0; s < NP; s++) {
                const float z = xv[s], tu = xv[NP + s];
                Xr[3 * s] = fmaf(z, fmaf(T.m[0], tu, B0), T.t[0]);
                Xr[3 * s + 1] = fmaf(z, fmaf(T.m[3], tu, B1), T.t[1]);
                Xr[3 * s + 2] = fmaf(z, fmaf(T.m[6], tu, B2), T.t[2]);
            }
        } else if constexpr (RC) {  // x = z * ((u - cx) / fx), y = z * ((v - cy) / fy): constrain_points_to_ray
#pragma unroll
            for (int s = 0; s < NP; s++) {
                xj[3 * s] = xv[s] * xv[NP + s];
                xj[3 * s + 1] = xv[s] * xv[2 * NP];
                xj[3 * s + 2] = xv[s];
            }
        } else {
#pragma unroll
            for (int q = 0; q < 3 * NP; q++) xj[q] = xv[q];
        }
#pragma unroll
        for (int s = 0; s < NP; s++) {
            PointsIn<float> p;
            if constexpr (M == GN_CALIB) {
                p.xi0 = p.xi1 = 0.0f;
                if constexpr (PK)
                    uv_pixel(codes[s], p.ut, p.vt);
                else
                    pixel_of(codes[s] & 0x7fffffff, P, p.ut, p.vt);
            } else {
                p.xi0 = g[s][0];
                p.xi1 = g[s][1];
            }
            p.xi2 = g[s][2];
            p.valid = codes[s] >= 0;
            p.sq = __int_as_float(sqb[s]);
            if constexpr (kFactor) {
                point_body_x<M, float>(p, Xr[3 * s], Xr[3 * s + 1], Xr[3 * s + 2], P, acc);
            } else {
                p.xj0 = xj[3 * s];
                p.xj1 = xj[3 * s + 1];
                p.xj2 = xj[3 * s + 2];
                point_body<M, float>(p, T, P, acc);
            }
#if M3S_ACC_SCHED_BARRIER == 1
            __builtin_amdgcn_sched_barrier(0);  // one point's temporaries live at a time
#elif M3S_ACC_SCHED_BARRIER == 2
            // two points' temporaries at a time: their dependent residual chains interleave
            if (s & 1) __builtin_amdgcn_sched_barrier(0);
#endif
        }
    }
};

// Points per lane and step of the accumulate (4 or 2), per mode.  Rays / points: 2 -- 74 instead
// of 112 VGPRs (points 61 / 75), 6 instead of 4 waves per SIMD; cfg4 accumulate 2.08 -> 1.96 ms.
// Calib: 4, with the ray-constrained path (Xj read as its depth): 0.337 ms on cfg3 against 0.350
// for the positional path at 2 and 0.358 for the ray-constrained one at 2 (profiles/r03_acc_ab.txt).
// -DM3S_ACC_PPL=n forces n for every mode (A/B builds).
template <int MODE>
__host__ __device__ constexpr int acc_np() {
#ifdef M3S_ACC_PPL
    return M3S_ACC_PPL;
#else
    return MODE == GN_CALIB ? 4 : 2;
#endif
}

// Reads the reference's tensors directly every iteration (used when the call runs < 3
// iterations, or the inputs are not 16-B aligned).  1-D grid over (edge, chunk) tasks in the
// driver's XCD-aware order; 256 threads; VEC: 4 consecutive points per lane per step as two
// packed pairs (16-B loads of idx/Q/Xj/Cj, 4-B valid).
template <int MODE, bool VEC>
__global__ __launch_bounds__(kAccThreads) void gn_accum_kernel(
    const float* __restrict__ Twc, const float* __restrict__ Xs, const float* __restrict__ Cs,
    const int* __restrict__ ii_loc, const int* __restrict__ jj_loc, EdgeSrc es, AccParams P,
    const int4* __restrict__ sched, float* __restrict__ partials, const int* __restrict__ flags) {
    const int4 tk = sched[blockIdx.x];  // {edge, chunk, ix, jx}, loaded together with the flag
    if (flags[kFlagDone]) return;
    const int e = tk.x, c = tk.y, ix = tk.z, jx = tk.w;
    const RelXf T = rel_xf(rel_sim3(load_sim3(Twc + (int64_t)ix * 8), load_sim3(Twc + (int64_t)jx * 8)));

    const int HW = P.HW;
    const int64_t* idx_e;
    const uint8_t* valid_e;
    const float* Q_e;
    es.at(e, HW, idx_e, valid_e, Q_e);
    const int64_t* __restrict__ idx = idx_e;
    const uint8_t* __restrict__ valid = valid_e;
    const float* __restrict__ Q = Q_e;
    const float* __restrict__ Xi_b = Xs + (int64_t)ix * HW * 3;
    const float* __restrict__ Ci_b = Cs + (int64_t)ix * HW;
    const float* __restrict__ Xj_b = Xs + (int64_t)jx * HW * 3;
    const float* __restrict__ Cj_b = Cs + (int64_t)jx * HW;
    const int k0 = c * P.chunk;
    const int k1 = min(k0 + P.chunk, HW);
    const int tid = threadIdx.x;
    float accs[kNacc];

    if constexpr (VEC) {
        // the same stage arithmetic as the packed kernel, from the reference's tensors: the
        // two paths produce bitwise identical partials
#pragma unroll
        for (int q = 0; q < kNacc; q++) accs[q] = 0.0f;
        constexpr int NP = acc_np<MODE>();  // the packed path's points per step: the same sums
        for (int k = k0 + NP * tid; k < k1; k += NP * kAccThreads) {
            bool vm[4];
            int64_t ids[4];
            float qs[4], cjs[4];
            if constexpr (NP == 4) {
                const uchar4 vm4 = *reinterpret_cast<const uchar4*>(valid + k);
                const longlong2 id01 = *reinterpret_cast<const longlong2*>(idx + k);
                const longlong2 id23 = *reinterpret_cast<const longlong2*>(idx + k + 2);
                const float4 q4 = *reinterpret_cast<const float4*>(Q + k);
                const float4 cj4 = *reinterpret_cast<const float4*>(Cj_b + k);
                vm[0] = vm4.x != 0; vm[1] = vm4.y != 0; vm[2] = vm4.z != 0; vm[3] = vm4.w != 0;
                ids[0] = id01.x; ids[1] = id01.y; ids[2] = id23.x; ids[3] = id23.y;
                qs[0] = q4.x; qs[1] = q4.y; qs[2] = q4.z; qs[3] = q4.w;
                cjs[0] = cj4.x; cjs[1] = cj4.y; cjs[2] = cj4.z; cjs[3] = cj4.w;
            } else {
                const uchar2 vm2 = *reinterpret_cast<const uchar2*>(valid + k);
                const longlong2 id01 = *reinterpret_cast<const longlong2*>(idx + k);
                const float2 q2 = *reinterpret_cast<const float2*>(Q + k);
                const float2 cj2 = *reinterpret_cast<const float2*>(Cj_b + k);
                vm[0] = vm2.x != 0; vm[1] = vm2.y != 0;
                ids[0] = id01.x; ids[1] = id01.y;
                qs[0] = q2.x; qs[1] = q2.y;
                cjs[0] = cj2.x; cjs[1] = cj2.y;
            }
            int code[4] = {0, 0, 0, 0}, sqb[4] = {0, 0, 0, 0};
#pragma unroll
            for (int s = 0; s < NP; s++) {
                const int ind = match_index(ids[s], vm[s], HW);
                const bool ok = vm[s] && (qs[s] > P.Q_thresh) && (Ci_b[ind] > P.C_thresh) &&
                                (cjs[s] > P.C_thresh);
                code[s] = ok ? ind : (int)((unsigned)ind | 0x80000000u);
                sqb[s] = __float_as_int(sqrt_cr(qs[s]));
            }
            AccStage<MODE, false, false, NP> st;
            st.set(int4{code[0], sqb[0], code[1], sqb[1]}, int4{code[2], sqb[2], code[3], sqb[3]});
            st.template load<MODE>(Xj_b, Xi_b, nullptr, k);  // calib: the depth from Xs ...
            if constexpr (MODE == GN_CALIB) {
#pragma unroll
                for (int s = 0; s < NP; s++)  // ... as the inverse depth gn_depth_kernel tabulates
                    st.g[s][2] = st.g[s][2] > P.z_eps ? vrcp(st.g[s][2]) : __builtin_nanf("");
            }
            st.template compute<MODE>(T, P, accs);
        }
    } else {
#pragma unroll
        for (int q = 0; q < kNacc; q++) accs[q] = 0.0f;
        for (int k = k0 + tid; k < k1; k += kAccThreads) {
            PointsIn<float> p;
            const bool vm = valid[k] != 0;
            const int ind = match_index(idx[k], vm, HW);
            const float q = Q[k];
            p.xj0 = Xj_b[(int64_t)k * 3 + 0];
            p.xj1 = Xj_b[(int64_t)k * 3 + 1];
            p.xj2 = Xj_b[(int64_t)k * 3 + 2];
            p.xi0 = Xi_b[(int64_t)ind * 3 + 0];
            p.xi1 = Xi_b[(int64_t)ind * 3 + 1];
            p.xi2 = Xi_b[(int64_t)ind * 3 + 2];
            if constexpr (MODE == GN_CALIB) p.xi2 = p.xi2 > P.z_eps ? vrcp(p.xi2) : __builtin_nanf("");
            p.valid = vm && (q > P.Q_thresh) && (Ci_b[ind] > P.C_thresh) && (Cj_b[k] > P.C_thresh);
            p.sq = sqrt_cr(q);
            if constexpr (MODE == GN_CALIB) pixel_of(ind, P, p.ut, p.vt);
            point_body<MODE, float>(p, T, P, accs);
        }
    }
    block_partial(accs, partials + ((int64_t)e * P.nchunks + c) * kNaccPad);
}

// ---------------------------------------------------------------------------
// Iteration-invariant packing (once per GN call, >= 3 iterations): per directed point-edge
// {code, sqrt(q)} with code = match index | (invalid << 31), where "valid" folds the
// reference's pose-independent tests (match, q > Q_thresh, ci > C_thresh, cj > C_thresh;
// gn_kernels.cu:953-957).  Every iteration then streams 8 B per point-edge instead of
// idx 8 + valid 1 + Q 4 + Cj 4 + gathered Ci 4 = 21 B, and the point math is unchanged
// (invalid points are still evaluated with weight 0, so NaN poisoning is kept).
// ---------------------------------------------------------------------------
// Per keyframe n: cok[n] stays 1 (as uploaded) iff every confidence c of it passes c > C_thresh
// (a NaN fails, like the reference's test).  The pack then skips its 8 B per point-edge of Cj
// reads and Ci gathers for edges whose two keyframes pass: the same validity bits, decided from
// one pass over the N x HW confidences instead of one per directed edge (cfg3: 4 per keyframe).
__global__ __launch_bounds__(256) void gn_cpass_kernel(const float* __restrict__ Cs, AccParams P,
                                                       int* __restrict__ cok, const int* __restrict__ flags) {
    if (flags[kFlagDone]) return;
    const int n = blockIdx.y;
    const float* __restrict__ C = Cs + (int64_t)n * P.HW;
    const float t = P.C_thresh;
    bool ok = true;
    if ((P.HW & 3) == 0) {  // 16-B loads (every keyframe row is 16-B aligned)
        const float4* __restrict__ C4 = reinterpret_cast<const float4*>(C);
        for (int k = blockIdx.x * 256 + threadIdx.x; k < (P.HW >> 2); k += gridDim.x * 256) {
            const float4 c = C4[k];
            ok = ok & (c.x > t) & (c.y > t) & (c.z > t) & (c.w > t);
        }
    } else {
        for (int k = blockIdx.x * 256 + threadIdx.x; k < P.HW; k += gridDim.x * 256) ok = ok & (C[k] > t);
    }
    if (!__all(ok) && (threadIdx.x & 63) == 0) cok[n] = 0;  // benign race: every writer stores 0
}

__global__ __launch_bounds__(kAccThreads) void gn_pack_kernel(
    const float* __restrict__ Cs, const int* __restrict__ ii_loc, const int* __restrict__ jj_loc,
    EdgeSrc es, AccParams P, const int* __restrict__ cok, int4* __restrict__ pack, const int* __restrict__ flags) {
    if (flags[kFlagDone]) return;
    const int e = blockIdx.y;
    const int HW = P.HW;
    const int64_t ebase = (int64_t)e * HW;
    const int64_t* idx_e;
    const uint8_t* valid_e;
    const float* Q_e;
    es.at(e, HW, idx_e, valid_e, Q_e);
    const int64_t* __restrict__ idx = idx_e;
    const uint8_t* __restrict__ valid = valid_e;
    const float* __restrict__ Q = Q_e;
    const float* __restrict__ Ci_b = Cs + (int64_t)ii_loc[e] * HW;
    const float* __restrict__ Cj_b = Cs + (int64_t)jj_loc[e] * HW;
    const int k = 4 * (blockIdx.x * kAccThreads + threadIdx.x);
    if (k >= HW) return;
    const uchar4 vm4 = *reinterpret_cast<const uchar4*>(valid + k);
    const longlong2 id01 = *reinterpret_cast<const longlong2*>(idx + k);
    const longlong2 id23 = *reinterpret_cast<const longlong2*>(idx + k + 2);
    const float4 q4 = *reinterpret_cast<const float4*>(Q + k);
    // the edge's keyframes whose every confidence passes (gn_cpass_kernel): no reads of them
    const bool ci_all = cok != nullptr && cok[ii_loc[e]] != 0;
    const bool cj_all = cok != nullptr && cok[jj_loc[e]] != 0;
    const float4 cj4 = cj_all ? make_float4(0.f, 0.f, 0.f, 0.f) : *reinterpret_cast<const float4*>(Cj_b + k);
    const bool vm[4] = {vm4.x != 0, vm4.y != 0, vm4.z != 0, vm4.w != 0};
    const int64_t ids[4] = {id01.x, id01.y, id23.x, id23.y};
    const float qs[4] = {q4.x, q4.y, q4.z, q4.w};
    const float cjs[4] = {cj4.x, cj4.y, cj4.z, cj4.w};
    int code[4], sqb[4];
#pragma unroll
    for (int s = 0; s < 4; s++) {
        const int ind = match_index(ids[s], vm[s], HW);
        const bool ok = vm[s] && (qs[s] > P.Q_thresh) && (ci_all || Ci_b[ind] > P.C_thresh) &&
                        (cj_all || cjs[s] > P.C_thresh);
        code[s] = pack_code(ind, ok, P);
        sqb[s] = __float_as_int(sqrt_cr(qs[s]));
    }
    int4* dst = pack + (ebase + k) / 2;
    dst[0] = int4{code[0], sqb[0], code[1], sqb[1]};
    dst[1] = int4{code[2], sqb[2], code[3], sqb[3]};
}

// ---------------------------------------------------------------------------
// Compacted packed stream (opt-in M3S_GN_COMPACT=1; default: the positional one above).  A point
// whose pose-independent validity fails (match, q, ci, cj) contributes w = 0 every iteration,
// and 0 * (finite Jacobian / residual) = 0 exactly: such a point is "dead" when its own point
// and the matched point it gathers are finite (the reference's NaN poisoning through an invalid
// point needs a non-finite input, and those points are kept).  Per (edge, chunk) the live points
// are written contiguously, in point order (a fixed-order workgroup scan: deterministic), as
// the 8-B record {code, sqrt q} plus a copy of Xj (12 B, iteration-invariant), padded to a
// multiple of 4 with copies of a dead point (exact zeros); the count goes to pcnt.  Every
// iteration then runs the point math only on live points, reading contiguous streams.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool finite3(const float* p) {
    return isfinite(p[0]) && isfinite(p[1]) && isfinite(p[2]);
}

template <int MODE>
__global__ __launch_bounds__(kAccThreads) void gn_pack_compact_kernel(
    const float* __restrict__ Xs, const float* __restrict__ Cs, const int* __restrict__ ii_loc,
    const int* __restrict__ jj_loc, EdgeSrc es, AccParams P, int2* __restrict__ pk, float* __restrict__ px,
    int* __restrict__ pcnt, const int* __restrict__ flags) {
    __shared__ int s_wsum[kAccThreads / 64];
    __shared__ int s_dead;
    if (flags[kFlagDone]) return;
    const int e = blockIdx.y, c = blockIdx.x;
    const int HW = P.HW;
    const int k0 = c * P.chunk, k1 = min(k0 + P.chunk, HW);
    const int64_t obase = ((int64_t)e * P.nchunks + c) * P.chunk;
    const int64_t* idx_e;
    const uint8_t* valid_e;
    const float* Q_e;
    es.at(e, HW, idx_e, valid_e, Q_e);
    const int ix = ii_loc[e], jx = jj_loc[e];
    const float* __restrict__ Ci_b = Cs + (int64_t)ix * HW;
    const float* __restrict__ Cj_b = Cs + (int64_t)jx * HW;
    const float* __restrict__ Xi_b = Xs + (int64_t)ix * HW * 3;
    const float* __restrict__ Xj_b = Xs + (int64_t)jx * HW * 3;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) s_dead = INT_MAX;
    __syncthreads();
    int running = 0;
    for (int base = k0; base < k1; base += 4 * kAccThreads) {
        const int k = base + 4 * tid;
        int code[4], sqb[4];
        bool live[4] = {false, false, false, false};
        float xj[12];
        if (k < k1) {
            const uchar4 vm4 = *reinterpret_cast<const uchar4*>(valid_e + k);
            const longlong2 id01 = *reinterpret_cast<const longlong2*>(idx_e + k);
            const longlong2 id23 = *reinterpret_cast<const longlong2*>(idx_e + k + 2);
            const float4 q4 = *reinterpret_cast<const float4*>(Q_e + k);
            const float4 cj4 = *reinterpret_cast<const float4*>(Cj_b + k);
            const float4 xa = *reinterpret_cast<const float4*>(Xj_b + (int64_t)k * 3);
            const float4 xb = *reinterpret_cast<const float4*>(Xj_b + (int64_t)k * 3 + 4);
            const float4 xc = *reinterpret_cast<const float4*>(Xj_b + (int64_t)k * 3 + 8);
            const float t[12] = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w, xc.x, xc.y, xc.z, xc.w};
#pragma unroll
            for (int q = 0; q < 12; q++) xj[q] = t[q];
            const bool vm[4] = {vm4.x != 0, vm4.y != 0, vm4.z != 0, vm4.w != 0};
            const int64_t ids[4] = {id01.x, id01.y, id23.x, id23.y};
            const float qs[4] = {q4.x, q4.y, q4.z, q4.w};
            const float cjs[4] = {cj4.x, cj4.y, cj4.z, cj4.w};
#pragma unroll
            for (int s = 0; s < 4; s++) {
                const int ind = match_index(ids[s], vm[s], HW);
                const bool ok = vm[s] && (qs[s] > P.Q_thresh) && (Ci_b[ind] > P.C_thresh) && (cjs[s] > P.C_thresh);
                code[s] = pack_code(ind, ok, P);
                sqb[s] = __float_as_int(sqrt_cr(qs[s]));
                const float* xi = Xi_b + (int64_t)ind * 3;
                const bool fin = finite3(&xj[3 * s]) &&
                                 (MODE == GN_CALIB ? (bool)isfinite(xi[2]) : finite3(xi));
                live[s] = ok || !fin;
                if (!live[s]) atomicMin(&s_dead, k + s);
            }
        }
        const int n = (int)live[0] + (int)live[1] + (int)live[2] + (int)live[3];
        // exclusive scan of n over the workgroup in thread order
        int incl = n;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(incl, off, 64);
            if (lane >= off) incl += y;
        }
        if (lane == 63) s_wsum[wave] = incl;
        __syncthreads();
        int wbase = 0, total = 0;
#pragma unroll
        for (int w = 0; w < kAccThreads / 64; w++) {
            wbase += w < wave ? s_wsum[w] : 0;
            total += s_wsum[w];
        }
        int pos = running + wbase + incl - n;
#pragma unroll
        for (int s = 0; s < 4; s++) {
            if (live[s]) {
                pk[obase + pos] = make_int2(code[s], sqb[s]);
                float* o = px + (obase + pos) * 3;
                o[0] = xj[3 * s];
                o[1] = xj[3 * s + 1];
                o[2] = xj[3 * s + 2];
                pos++;
            }
        }
        running += total;
        __syncthreads();  // s_wsum is reused by the next step
    }
    // pad to a multiple of 4 with copies of the first dead point (its contribution is exactly 0)
    const int pad = (4 - (running & 3)) & 3;
    if (tid < pad) {
        const int kd = s_dead;  // pad > 0 implies a dead point exists (chunks are multiples of 4)
        const int64_t id = idx_e[kd];
        const int ind = match_index(id, valid_e[kd] != 0, HW);
        pk[obase + running + tid] = make_int2(pack_code(ind, false, P), __float_as_int(sqrt_cr(Q_e[kd])));
        float* o = px + (obase + running + tid) * 3;
        o[0] = Xj_b[(int64_t)kd * 3];
        o[1] = Xj_b[(int64_t)kd * 3 + 1];
        o[2] = Xj_b[(int64_t)kd * 3 + 2];
    }
    if (tid == 0) pcnt[(int64_t)e * P.nchunks + c] = running + pad;
}

// Zs[n, k] = Xs[n, k, 2], and after the ray tables the inverse depths IZs[n, k] =
// (z > z_eps) ? v_rcp_f32(z) : NaN -- what the calib accumulate gathers for the matched point (4 B
// per point instead of a 12-B stride; the reciprocal and the z_eps test hoisted out of the
// iterations: the same values, one transcendental per point-edge and iteration less).
// Also the ray tables tu[u] = (u - cx) / fx, tv[v] = (v - cy) / fy (after Zs), and a check that
// every point IS its pixel's ray times its depth, bit for bit, i.e. what solve_GN_calib's
// constrain_points_to_ray (global_opt.py:172, geometry.py:37-42/107-123: z * ((u - cx) / fx))
// produces.  If so (flag kFlagNotRay stays 0) the accumulate reads Xj as its 4-B depth and
// applies T_ij to z (tu, tv, 1) factored per pixel row (M3S_RC_FACTOR; with it off, x and y are
// rebuilt with the same two roundings and the result is bitwise the positional stream's).
__global__ __launch_bounds__(256) void gn_depth_kernel(const float* __restrict__ Xs, int64_t total,
                                                       float* __restrict__ Zs, AccParams P,
                                                       int* __restrict__ flags, const float* __restrict__ K) {
    // the intrinsics from the device K when given (the pass runs before the host has read K)
    const float fx = K ? K[0] : P.fx, fy = K ? K[4] : P.fy, cx = K ? K[2] : P.cx, cy = K ? K[5] : P.cy;
    float* __restrict__ tu = Zs + total;
    float* __restrict__ tv = tu + P.width;
    float* __restrict__ IZn = inv_depths(Zs, P) + (int64_t)blockIdx.y * P.HW;
    const int n = blockIdx.y;  // keyframe row
    const int t0 = blockIdx.x * 256 + threadIdx.x;
    if (n == 0 && t0 < P.width) tu[t0] = ((float)t0 - cx) / fx;
    if (n == 0 && t0 < P.height) tv[t0] = ((float)t0 - cy) / fy;
    const float* __restrict__ Xn = Xs + (int64_t)n * P.HW * 3;
    float* __restrict__ Zn = Zs + (int64_t)n * P.HW;
    bool ray = true;
    for (int k = t0; k < P.HW; k += gridDim.x * 256) {
        const float x = Xn[(int64_t)k * 3], y = Xn[(int64_t)k * 3 + 1], z = Xn[(int64_t)k * 3 + 2];
        Zn[k] = z;
        IZn[k] = z > P.z_eps ? vrcp(z) : __builtin_nanf("");
        float u, v;
        pixel_of(k, P, u, v);
        const float xr = z * ((u - cx) / fx);
        const float yr = z * ((v - cy) / fy);
        ray = ray && __float_as_uint(xr) == __float_as_uint(x) && __float_as_uint(yr) == __float_as_uint(y);
    }
    if (!ray) flags[kFlagNotRay] = 1;  // benign race: every writer stores 1
}

// The reference's per-point inputs of one directed edge, for the first iteration's accumulate
// that builds the packed records itself (gn_accum_packed_kernel<..., FIRST>).
struct RawSrc {
    const int64_t* idx;
    const uint8_t* valid;
    const float* Q;
    const float* Ci_b;
    const float* Cj_b;
    int4* pk_w;          // the edge's packed records, written for the later iterations
    bool ci_all, cj_all;  // every confidence of keyframe i / j passes (gn_cpass_kernel)
};

// One lane's steps of the packed accumulate (NP points per step); the records of the next step
// are loaded one step ahead.  RC: Xj_b is keyframe j's depth row and x, y come from the ray
// tables that follow Zs (total = N * HW floats of depth).  FIRST (NP = 4): the records are built
// from the reference's inputs exactly as gn_pack_kernel builds them (and stored for the later
// iterations) instead of being read: the per-call pack pass is folded into the first iteration.
template <int MODE, bool RC, int NP = 4, bool FIRST = false>
__device__ __forceinline__ void accum_steps(const float* __restrict__ Xj_b, const float* __restrict__ Xi_b,
                                            const float* __restrict__ Zi_b, const int4* __restrict__ pk_b,
                                            int k0, int k1, const RelXf& T, const AccParams& P,
                                            const float* __restrict__ Zs, float* __restrict__ acc,
                                            const RawSrc& raw = RawSrc{}) {
    static_assert(NP == 4 || NP == 2, "4 or 2 points per step");
    constexpr int S = NP * kAccThreads;
    AccStage<MODE, RC, true, NP> cur;
    cur.width = P.width;
    if constexpr (RC) {
        cur.rc_tu = Zs + (int64_t)P.nkf * P.HW;
        cur.rc_tv = cur.rc_tu + P.width;
        cur.rc_m = P.div_m;
        cur.rc_sh = P.div_sh;
        cur.rc_w = P.width;
    }
    // the records of NP points: one int4 per two
    auto records = [&](int kk, int4& a, int4& b) {
        if constexpr (FIRST && NP == 2) {
            // (rays / points: 2 points per step) gn_pack_kernel's record, operation for operation
            const uchar2 vm2 = *reinterpret_cast<const uchar2*>(raw.valid + kk);
            const longlong2 id01 = *reinterpret_cast<const longlong2*>(raw.idx + kk);
            const float2 q2 = *reinterpret_cast<const float2*>(raw.Q + kk);
            const float2 cj2 =
                raw.cj_all ? make_float2(0.f, 0.f) : *reinterpret_cast<const float2*>(raw.Cj_b + kk);
            const bool vm[2] = {vm2.x != 0, vm2.y != 0};
            const int64_t ids[2] = {id01.x, id01.y};
            const float qs[2] = {q2.x, q2.y};
            const float cjs[2] = {cj2.x, cj2.y};
            int code[2], sqb[2];
#pragma unroll
            for (int s = 0; s < 2; s++) {
                const int ind = match_index(ids[s], vm[s], P.HW);
                const bool ok = vm[s] && (qs[s] > P.Q_thresh) && (raw.ci_all || raw.Ci_b[ind] > P.C_thresh) &&
                                (raw.cj_all || cjs[s] > P.C_thresh);
                code[s] = pack_code(ind, ok, P);
                sqb[s] = __float_as_int(sqrt_cr(qs[s]));
            }
            a = int4{code[0], sqb[0], code[1], sqb[1]};
            raw.pk_w[kk / 2] = a;
        } else if constexpr (FIRST) {
            const uchar4 vm4 = *reinterpret_cast<const uchar4*>(raw.valid + kk);
            const longlong2 id01 = *reinterpret_cast<const longlong2*>(raw.idx + kk);
            const longlong2 id23 = *reinterpret_cast<const longlong2*>(raw.idx + kk + 2);
            const float4 q4 = *reinterpret_cast<const float4*>(raw.Q + kk);
            const float4 cj4 =
                raw.cj_all ? make_float4(0.f, 0.f, 0.f, 0.f) : *reinterpret_cast<const float4*>(raw.Cj_b + kk);
            const bool vm[4] = {vm4.x != 0, vm4.y != 0, vm4.z != 0, vm4.w != 0};
            const int64_t ids[4] = {id01.x, id01.y, id23.x, id23.y};
            const float qs[4] = {q4.x, q4.y, q4.z, q4.w};
            const float cjs[4] = {cj4.x, cj4.y, cj4.z, cj4.w};
            int code[4], sqb[4];
#pragma unroll
            for (int s = 0; s < 4; s++) {  // gn_pack_kernel's record, operation for operation
                const int ind = match_index(ids[s], vm[s], P.HW);
                const bool ok = vm[s] && (qs[s] > P.Q_thresh) && (raw.ci_all || raw.Ci_b[ind] > P.C_thresh) &&
                                (raw.cj_all || cjs[s] > P.C_thresh);
                code[s] = pack_code(ind, ok, P);
                sqb[s] = __float_as_int(sqrt_cr(qs[s]));
            }
            a = int4{code[0], sqb[0], code[1], sqb[1]};
            b = int4{code[2], sqb[2], code[3], sqb[3]};
            raw.pk_w[kk / 2] = a;
            raw.pk_w[kk / 2 + 1] = b;
        } else {
            a = pk_b[kk / 2];
            if constexpr (NP == 4) b = pk_b[kk / 2 + 1];
        }
    };
    int4 na = int4{0, 0, 0, 0}, nb = int4{0, 0, 0, 0};
    int k = k0 + NP * threadIdx.x;
    if (k < k1) records(k, na, nb);
    for (; k < k1; k += S) {
#if M3S_ACC_DIAG == 1
        // diagnostics: compute only (the first step's data, re-used: no memory after it)
        if (k == k0 + NP * (int)threadIdx.x) {
            cur.set(na, nb);
            cur.template load<MODE>(Xj_b, Xi_b, Zi_b, k);
        }
        cur.template compute<MODE>(T, P, acc);
        __builtin_amdgcn_sched_barrier(0);
        continue;
#elif M3S_ACC_DIAG == 2
        // diagnostics: memory only -- the first step computed (so the system stays solvable and
        // the iterations keep running), then every step's loads with each value merely consumed
        cur.set(na, nb);
        if (k + S < k1) records(k + S, na, nb);
        cur.template load<MODE>(Xj_b, Xi_b, Zi_b, k);
        if (k == k0 + NP * (int)threadIdx.x) {
            cur.template compute<MODE>(T, P, acc);
        } else {
#pragma unroll
            for (int q = 0; q < 3 * NP; q++) asm volatile("" ::"v"(cur.xv[q]));
#pragma unroll
            for (int q = 0; q < NP; q++) asm volatile("" ::"v"(cur.g[q][2]), "v"(cur.g[q][0]), "v"(cur.cd[q]), "v"(cur.sb[q]));
        }
        continue;
#endif
        cur.set(na, nb);
        if (k + S < k1) records(k + S, na, nb);
        cur.template load<MODE>(Xj_b, Xi_b, Zi_b, k);
        cur.template compute<MODE>(T, P, acc);
    }
}

// Per-iteration accumulate over the packed stream: 8 B {code, sqrt q} + Xj 12 B + the gather
// of the matched point (calib: its depth from Zs; rays/points: Xi) per point-edge.

#ifndef M3S_ACC_WAVES
#define M3S_ACC_WAVES 1
#endif
// the rays iteration kernel's occupancy floor (A/B builds; 1 = the compiler's choice)
#ifndef M3S_ACC_WAVES_RAYS
#define M3S_ACC_WAVES_RAYS M3S_ACC_WAVES
#endif
template <int MODE, bool FIRST>
constexpr int acc_waves() {
    return (MODE == GN_RAYS && !FIRST) ? M3S_ACC_WAVES_RAYS : M3S_ACC_WAVES;
}
// FIRST (calib, the positional stream): the first iteration of a call, building the packed
// records from the reference's inputs on the way (RawSrc; no separate gn_pack_kernel pass).
struct FirstSrc {
    EdgeSrc es;
    const float* Cs;
    const int* cok;
    int4* pack_w;
};

template <int MODE, bool COMPACT, bool RCOK = false, bool FIRST = false>
__global__ __launch_bounds__(kAccThreads) __attribute__((amdgpu_waves_per_eu(acc_waves<MODE, FIRST>())))
void gn_accum_packed_kernel(
    const float* __restrict__ Twc, const float* __restrict__ Xs, const float* __restrict__ Zs,
    const int* __restrict__ ii_loc, const int* __restrict__ jj_loc, const int4* __restrict__ pack,
    AccParams P, const int4* __restrict__ sched, float* __restrict__ partials,
    const int* __restrict__ flags, const float* __restrict__ px, const int* __restrict__ pcnt,
    int* __restrict__ ecnt, double* __restrict__ edgeblk, FirstSrc fs) {
    const int4 tk = sched[blockIdx.x];  // {edge, chunk, ix, jx}, loaded together with the flag
    if (flags[kFlagDone]) return;
    const int e = tk.x, c = tk.y, ix = tk.z, jx = tk.w;
    const RelXf T = rel_xf(rel_sim3(load_sim3(Twc + (int64_t)ix * 8), load_sim3(Twc + (int64_t)jx * 8)));

    const int HW = P.HW;
    const int64_t ebase = (int64_t)e * HW;
    const float* __restrict__ Xi_b = Xs + (int64_t)ix * HW * 3;
    const float* __restrict__ Zi_b = MODE == GN_CALIB ? inv_depths(Zs, P) + (int64_t)ix * HW : nullptr;
    const float* __restrict__ Xj_b = Xs + (int64_t)jx * HW * 3;
    const int4* __restrict__ pk_b = pack + ebase / 2;
    const int k0 = c * P.chunk;
    const int k1 = min(k0 + P.chunk, HW);

    float acc[kNacc];
#pragma unroll
    for (int q = 0; q < kNacc; q++) acc[q] = 0.0f;
    // Steps of NP points per lane; the packed records of the next step are loaded one step
    // ahead, so a step waits for one memory round trip (its gathers + Xj) instead of two
    // (records, then the gathers they index).  A deeper pipeline (gathers of the next step
    // in flight too) needs ~180 VGPRs, drops to 2 waves/SIMD and measured 8 % slower (removed).
    if constexpr (COMPACT) {
        // compacted stream: the chunk's live points, Xj copied alongside the records
        const int64_t cb = ((int64_t)e * P.nchunks + c) * P.chunk;
        accum_steps<MODE, false, acc_np<MODE>()>(px + cb * 3, Xi_b, Zi_b, pack + cb / 2, 0, pcnt[(int64_t)e * P.nchunks + c], T, P,
                                 Zs, acc);
    } else if constexpr (FIRST) {
        RawSrc raw;
        fs.es.at(e, HW, raw.idx, raw.valid, raw.Q);
        raw.Ci_b = fs.Cs + (int64_t)ix * HW;
        raw.Cj_b = fs.Cs + (int64_t)jx * HW;
        raw.pk_w = fs.pack_w + ebase / 2;
        raw.ci_all = fs.cok != nullptr && fs.cok[ix] != 0;
        raw.cj_all = fs.cok != nullptr && fs.cok[jx] != 0;
        if (RCOK && flags[kFlagNotRay] == 0 && (P.width & 3) == 0)
            accum_steps<MODE, true, 4, true>(Zs + (int64_t)jx * HW, Xi_b, Zi_b, pk_b, k0, k1, T, P, Zs, acc, raw);
        else
            accum_steps<MODE, false, acc_np<MODE>(), true>(Xj_b, Xi_b, Zi_b, pk_b, k0, k1, T, P, Zs, acc, raw);
    } else if (RCOK && MODE == GN_CALIB && flags[kFlagNotRay] == 0 && (P.width & 3) == 0)
        // calib with ray-constrained keyframe points (gn_depth_kernel's check): Xj from its depth
        accum_steps<MODE, true, acc_np<MODE>()>(Zs + (int64_t)jx * HW, Xi_b, Zi_b, pk_b, k0, k1, T, P, Zs, acc);
    else
        accum_steps<MODE, false, acc_np<MODE>()>(Xj_b, Xi_b, Zi_b, pk_b, k0, k1, T, P, Zs, acc);
    block_partial(acc, partials + ((int64_t)e * P.nchunks + c) * kNaccPad, ecnt != nullptr);
    if (ecnt != nullptr) {
        // fused edge reduce: the edge's last workgroup to finish sums its chunk partials (in
        // chunk order: bitwise the separate gn_edge_reduce_kernel) -- one launch less per
        // iteration, and the reduce overlaps the other edges' accumulation
        __shared__ int s_last;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's partial stores landed
        __syncthreads();
        if (threadIdx.x == 0)
            s_last = __hip_atomic_fetch_add(ecnt + e, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == P.nchunks - 1;
        __syncthreads();
        if (s_last) {
            edge_reduce_body<true>(partials, P.nchunks, Twc, ii_loc, edgeblk, e);
            if (threadIdx.x == 0) __hip_atomic_store(ecnt + e, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

hipError_t launch_accum(int mode, bool vec, dim3 grid, hipStream_t st, const float* Twc,
                        const float* Xs, const float* Cs, const int* ii_loc, const int* jj_loc,
                        const EdgeSrc& es, const AccParams& P, const int4* sched, float* partials,
                        const int* flags) {
#define M3S_ACC(MODE, V)                                                                    \
    hipLaunchKernelGGL((gn_accum_kernel<MODE, V>), grid, dim3(kAccThreads), 0, st, Twc, Xs, \
                       Cs, ii_loc, jj_loc, es, P, sched, partials, flags)
    if (mode == GN_RAYS) {
        if (vec) M3S_ACC(GN_RAYS, true); else M3S_ACC(GN_RAYS, false);
    } else if (mode == GN_CALIB) {
        if (vec) M3S_ACC(GN_CALIB, true); else M3S_ACC(GN_CALIB, false);
    } else {
        if (vec) M3S_ACC(GN_POINTS, true); else M3S_ACC(GN_POINTS, false);
    }
#undef M3S_ACC
    return hipGetLastError();
}

hipError_t launch_pack_pre(hipStream_t st, const float* Xs, int64_t N, const float* Cs, const AccParams& P, int* cok,
                           float* Zs, int* flags, const float* K) {
    if (cok != nullptr && N > 0) {  // per keyframe: do all its confidences pass C_thresh?
        const int bx = (int)std::max<int64_t>(1, std::min<int64_t>((P.HW + 1023) / 1024, 8192 / std::max<int64_t>(N, 1)));
        hipLaunchKernelGGL(gn_cpass_kernel, dim3(bx, (unsigned)N), dim3(256), 0, st, Cs, P, cok, flags);
    }
    if (Zs) {
        const int64_t total = N * (int64_t)P.HW;
        const int bx = (int)std::max<int64_t>(std::min<int64_t>((P.HW + 255) / 256,
                                                                std::max<int64_t>(8192 / std::max<int64_t>(N, 1), 2)),
                                              (std::max(P.width, P.height) + 255) / 256);
        hipLaunchKernelGGL(gn_depth_kernel, dim3(bx, (unsigned)N), dim3(256), 0, st, Xs, total, Zs, P, flags, K);
    }
    return hipGetLastError();
}

hipError_t launch_pack(int mode, hipStream_t st, int E_local, const float* Xs, int64_t N, const float* Cs,
                       const int* ii_loc, const int* jj_loc, const EdgeSrc& es, const AccParams& P, int* cok,
                       int4* pack, float* px, int* pcnt, const int* flags, bool skip_pack) {
    if (E_local > 0 && px) {
        const dim3 grid((unsigned)P.nchunks, (unsigned)E_local);
        int2* pk = reinterpret_cast<int2*>(pack);
        if (mode == GN_RAYS)
            hipLaunchKernelGGL(gn_pack_compact_kernel<GN_RAYS>, grid, dim3(kAccThreads), 0, st, Xs, Cs, ii_loc,
                               jj_loc, es, P, pk, px, pcnt, flags);
        else if (mode == GN_CALIB)
            hipLaunchKernelGGL(gn_pack_compact_kernel<GN_CALIB>, grid, dim3(kAccThreads), 0, st, Xs, Cs, ii_loc,
                               jj_loc, es, P, pk, px, pcnt, flags);
        else
            hipLaunchKernelGGL(gn_pack_compact_kernel<GN_POINTS>, grid, dim3(kAccThreads), 0, st, Xs, Cs, ii_loc,
                               jj_loc, es, P, pk, px, pcnt, flags);
    } else if (E_local > 0) {
        // (cok from the cpass of launch_pack_pre)
        const dim3 grid((unsigned)((P.HW / 4 + kAccThreads - 1) / kAccThreads), (unsigned)E_local);
        if (!skip_pack)  // (else the first iteration's accumulate builds the records)
            hipLaunchKernelGGL(gn_pack_kernel, grid, dim3(kAccThreads), 0, st, Cs, ii_loc, jj_loc, es,
                               P, cok, pack, flags);
    }
    return hipGetLastError();
}

hipError_t launch_accum_packed(int mode, dim3 grid, hipStream_t st, const float* Twc,
                               const float* Xs, const float* Zs, const int* ii_loc,
                               const int* jj_loc, const int4* pack, const AccParams& P,
                               const int4* sched, float* partials, const int* flags, const float* px,
                               const int* pcnt, int* ecnt, double* edgeblk, const EdgeSrc* first_es,
                               const float* Cs, const int* cok) {
    if (first_es != nullptr) {  // the first iteration builds the records (positional stream)
        if (px != nullptr) return hipErrorInvalidValue;
        const FirstSrc fs{*first_es, Cs, cok, const_cast<int4*>(pack)};
        if (mode == GN_RAYS)
            hipLaunchKernelGGL((gn_accum_packed_kernel<GN_RAYS, false, false, true>), grid, dim3(kAccThreads), 0, st,
                               Twc, Xs, Zs, ii_loc, jj_loc, pack, P, sched, partials, flags, px, pcnt, ecnt,
                               edgeblk, fs);
        else if (mode == GN_POINTS)
            hipLaunchKernelGGL((gn_accum_packed_kernel<GN_POINTS, false, false, true>), grid, dim3(kAccThreads), 0, st,
                               Twc, Xs, Zs, ii_loc, jj_loc, pack, P, sched, partials, flags, px, pcnt, ecnt,
                               edgeblk, fs);
        else if (P.raycheck)
            hipLaunchKernelGGL((gn_accum_packed_kernel<GN_CALIB, false, true, true>), grid, dim3(kAccThreads), 0, st,
                               Twc, Xs, Zs, ii_loc, jj_loc, pack, P, sched, partials, flags, px, pcnt, ecnt,
                               edgeblk, fs);
        else
            hipLaunchKernelGGL((gn_accum_packed_kernel<GN_CALIB, false, false, true>), grid, dim3(kAccThreads), 0, st,
                               Twc, Xs, Zs, ii_loc, jj_loc, pack, P, sched, partials, flags, px, pcnt, ecnt,
                               edgeblk, fs);
        return hipGetLastError();
    }
    const FirstSrc fs0{};
#define M3S_ACCP(MODE, CP, RC)                                                                       \
    hipLaunchKernelGGL((gn_accum_packed_kernel<MODE, CP, RC>), grid, dim3(kAccThreads), 0, st, Twc, Xs, Zs, \
                       ii_loc, jj_loc, pack, P, sched, partials, flags, px, pcnt, ecnt, edgeblk, fs0)
#define M3S_ACCP2(MODE, CP) M3S_ACCP(MODE, CP, false)
    const bool cp = px != nullptr;
    if (mode == GN_RAYS) {
        if (cp) M3S_ACCP2(GN_RAYS, true); else M3S_ACCP2(GN_RAYS, false);
    } else if (mode == GN_CALIB) {
        if (cp) M3S_ACCP2(GN_CALIB, true);
        else if (P.raycheck) M3S_ACCP(GN_CALIB, false, true);
        else M3S_ACCP2(GN_CALIB, false);
    } else {
        if (cp) M3S_ACCP2(GN_POINTS, true); else M3S_ACCP2(GN_POINTS, false);
    }
#undef M3S_ACCP2
#undef M3S_ACCP
    return hipGetLastError();
}

}  // namespace m3s
