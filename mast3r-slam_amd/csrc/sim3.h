// sim3.h -- device Sim3 math for the GN kernels (float, reference formulas).
//
// Restates the reference's device library gn_kernels.cu:172-413 (quat_comp, actSO3,
// actSim3, relSim3, expSO3, expSim3, retrSim3), keeping its double-literal promotions
// so the retraction tracks the CPU oracle to a few ulp (sin/cos/exp ulp aside), under an
// FMA-contraction convention CM (contract.h; default the reference build's nvcc --fmad=true:
// a product feeding an add is fused, the left product of `a*b + c*d`).  Every function turns
// contraction off in its body: the helpers are its only fused operations, whatever the
// including file's -ffp-contract.
// Layout: t(3), q(4: x,y,z,w), s; tangent order tau(3), phi(3), sigma(1).
#pragma once

#include <hip/hip_runtime.h>

#include "contract.h"

namespace m3s {

struct Sim3f {
    float t[3];
    float q[4];
    float s;
};

__device__ __forceinline__ Sim3f load_sim3(const float* __restrict__ p) {
    Sim3f T;
    T.t[0] = p[0]; T.t[1] = p[1]; T.t[2] = p[2];
    T.q[0] = p[3]; T.q[1] = p[4]; T.q[2] = p[5]; T.q[3] = p[6];
    T.s = p[7];
    return T;
}

// gn_kernels.cu:178-184: qi * qj, each component a left-to-right sum of four products
template <int CM = M3S_CONTRACT_DEFAULT>
__device__ __forceinline__ void quat_comp(const float* qi, const float* qj, float* out) {
#pragma clang fp contract(off)
    const float o0 = cmad<CM>(-qi[2], qj[1], cmad<CM>(qi[1], qj[2], cmm<CM>(qi[3], qj[0], qi[0], qj[3])));
    const float o1 = cmad<CM>(qi[2], qj[0], cmad<CM>(qi[1], qj[3], cmm<CM>(qi[3], qj[1], -qi[0], qj[2])));
    const float o2 = cmad<CM>(qi[2], qj[3], cmad<CM>(-qi[1], qj[0], cmm<CM>(qi[3], qj[2], qi[0], qj[1])));
    const float o3 = cmad<CM>(-qi[2], qj[2], cmad<CM>(-qi[1], qj[1], cmm<CM>(qi[3], qj[3], -qi[0], qj[0])));
    out[0] = o0; out[1] = o1; out[2] = o2; out[3] = o3;
}

// gn_kernels.cu:195-205 (alias-safe): uv = 2 (u x X) (the 2.0 double multiply is exact),
// Y = (X + w uv) + (u x uv)
template <int CM = M3S_CONTRACT_DEFAULT>
__device__ __forceinline__ void act_so3(const float* q, const float* X, float* Y) {
#pragma clang fp contract(off)
    const float uv0 = 2.0f * cmm<CM>(q[1], X[2], -q[2], X[1]);
    const float uv1 = 2.0f * cmm<CM>(q[2], X[0], -q[0], X[2]);
    const float uv2 = 2.0f * cmm<CM>(q[0], X[1], -q[1], X[0]);
    const float y0 = cmad<CM>(q[3], uv0, X[0]) + cmm<CM>(q[1], uv2, -q[2], uv1);
    const float y1 = cmad<CM>(q[3], uv1, X[1]) + cmm<CM>(q[2], uv0, -q[0], uv2);
    const float y2 = cmad<CM>(q[3], uv2, X[2]) + cmm<CM>(q[0], uv1, -q[1], uv0);
    Y[0] = y0; Y[1] = y1; Y[2] = y2;
}

// gn_kernels.cu:207-219: Y = s R X + t (the scale product feeds the translation add: fused)
template <int CM = M3S_CONTRACT_DEFAULT>
__device__ __forceinline__ void act_sim3(const Sim3f& T, const float* X, float* Y) {
#pragma clang fp contract(off)
    float r[3];
    act_so3<CM>(T.q, X, r);
    Y[0] = cmad<CM>(r[0], T.s, T.t[0]);
    Y[1] = cmad<CM>(r[1], T.s, T.t[1]);
    Y[2] = cmad<CM>(r[2], T.s, T.t[2]);
}

// gn_kernels.cu:252-272: T_ij = T_i^{-1} T_j
template <int CM = M3S_CONTRACT_DEFAULT>
__device__ __forceinline__ Sim3f rel_sim3(const Sim3f& Ti, const Sim3f& Tj) {
#pragma clang fp contract(off)
    Sim3f R;
    const float si_inv = (float)(1.0 / (double)Ti.s);
    R.s = si_inv * Tj.s;
    const float qi_inv[4] = {-Ti.q[0], -Ti.q[1], -Ti.q[2], Ti.q[3]};
    quat_comp<CM>(qi_inv, Tj.q, R.q);
    float t[3] = {Tj.t[0] - Ti.t[0], Tj.t[1] - Ti.t[1], Tj.t[2] - Ti.t[2]};
    act_so3<CM>(qi_inv, t, t);
    R.t[0] = t[0] * si_inv; R.t[1] = t[1] * si_inv; R.t[2] = t[2] * si_inv;
    return R;
}

// gn_kernels.cu:229-240: b <- a x b
template <int CM = M3S_CONTRACT_DEFAULT>
__device__ __forceinline__ void cross_inplace(const float* a, float* b) {
#pragma clang fp contract(off)
    const float x0 = cmm<CM>(a[1], b[2], -a[2], b[1]);
    const float x1 = cmm<CM>(a[2], b[0], -a[0], b[2]);
    const float x2 = cmm<CM>(a[0], b[1], -a[1], b[0]);
    b[0] = x0; b[1] = x1; b[2] = x2;
}

// The Sim(3) exponential's float transcendentals, evaluated in double and rounded once to float
// (oracle/m3s_oracle.c does the same).  That is correctly rounded except in rare double-rounding
// cases: ocml's and glibc's double exp / sin / cos are ~1 ulp in double, not correctly rounded,
// so when the double result lies within ~1 double ulp of a float rounding boundary the GPU and
// the oracle may round to adjacent floats (a 1-ulp difference of the retraction, not observed on
// any test graph).  The reference's CUDA expf / sinf / cosf are <= 2 ulp and platform-specific,
// and its float formulas amplify one ulp of them enormously -- C = (expf(sigma) - 1) / sigma
// moves by ulp(1) / sigma (~1 % at sigma = 1e-5, i.e. ~1e-5 of a pose after a first GN step) --
// so no other platform can reproduce its bits there.
__device__ __forceinline__ float expf_cr(float x) { return (float)exp((double)x); }
__device__ __forceinline__ float sinf_cr(float x) { return (float)sin((double)x); }
__device__ __forceinline__ float cosf_cr(float x) { return (float)cos((double)x); }

// gn_kernels.cu:299-321 (the small-angle series is double arithmetic: fused in double too)
template <int CM = M3S_CONTRACT_DEFAULT>
__device__ __forceinline__ void exp_so3(const float* phi, float* q) {
#pragma clang fp contract(off)
    constexpr bool F = CM != M3S_CONTRACT_OFF;
    const float theta_sq = cdot3<CM>(phi[0], phi[0], phi[1], phi[1], phi[2], phi[2]);
    float imag, real;
    if ((double)theta_sq < 1e-6) {
        const float theta_p4 = theta_sq * theta_sq;
        imag = (float)cmad_d(F, 1.0 / 3840.0, (double)theta_p4, cmad_d(F, -(1.0 / 48.0), (double)theta_sq, 0.5));
        real = (float)cmad_d(F, 1.0 / 384.0, (double)theta_p4, cmad_d(F, -(1.0 / 8.0), (double)theta_sq, 1.0));
    } else {
        const float theta = sqrtf(theta_sq);
        imag = sinf_cr((float)(0.5 * (double)theta)) / theta;
        real = cosf_cr((float)(0.5 * (double)theta));
    }
    q[0] = imag * phi[0];
    q[1] = imag * phi[1];
    q[2] = imag * phi[2];
    q[3] = real;
}

// gn_kernels.cu:323-390 (as written, including B = (C - ...)/theta^2 at :371)
template <int CM = M3S_CONTRACT_DEFAULT>
__device__ __forceinline__ void exp_sim3(const float* xi, float* t, float* q, float* s) {
#pragma clang fp contract(off)
    float tau[3] = {xi[0], xi[1], xi[2]};
    const float phi[3] = {xi[3], xi[4], xi[5]};
    const float sigma = xi[6];
    const float scale = expf_cr(sigma);
    exp_so3<CM>(phi, q);
    s[0] = scale;
    const float theta_sq = cdot3<CM>(phi[0], phi[0], phi[1], phi[1], phi[2], phi[2]);
    const float theta = sqrtf(theta_sq);
    float A, B, C;
    const float one = 1.0f, half = 0.5f;
    if ((double)fabsf(sigma) < 1e-6) {
        C = one;
        if ((double)fabsf(theta) < 1e-6) {
            A = half;
            B = (float)(1.0 / 6.0);
        } else {
            A = (one - cosf_cr(theta)) / theta_sq;
            B = (theta - sinf_cr(theta)) / (theta_sq * theta);
        }
    } else {
        C = (scale - one) / sigma;
        if ((double)fabsf(theta) < 1e-6) {
            const float sigma_sq = sigma * sigma;
            A = cmad<CM>(sigma - one, scale, one) / sigma_sq;
            B = cmad<CM>(-sigma, scale, cmad<CM>(scale * half, sigma_sq, scale) - one) / (sigma_sq * sigma);
        } else {
            const float a = scale * sinf_cr(theta);
            const float b = scale * cosf_cr(theta);
            const float c = cmad<CM>(sigma, sigma, theta_sq);
            A = cmm<CM>(a, sigma, one - b, theta) / (theta * c);
            B = (C - cmm<CM>(b - one, sigma, a, theta) / c) / theta_sq;
        }
    }
    // t = C tau; t += A (phi x tau); t += B (phi x (phi x tau)): the first two are one sum of two
    // products, the third product is fused into the running sum
    const float tau0[3] = {tau[0], tau[1], tau[2]};
    cross_inplace<CM>(phi, tau);
    t[0] = cmm<CM>(C, tau0[0], A, tau[0]);
    t[1] = cmm<CM>(C, tau0[1], A, tau[1]);
    t[2] = cmm<CM>(C, tau0[2], A, tau[2]);
    cross_inplace<CM>(phi, tau);
    t[0] = cmad<CM>(B, tau[0], t[0]);
    t[1] = cmad<CM>(B, tau[1], t[1]);
    t[2] = cmad<CM>(B, tau[2], t[2]);
}

// gn_kernels.cu:392-413 (left composition)
template <int CM = M3S_CONTRACT_DEFAULT>
__device__ __forceinline__ void retr_sim3(const float* xi, float* p /* [8], in/out */) {
#pragma clang fp contract(off)
    float dt[3] = {0, 0, 0}, dq[4] = {0, 0, 0, 1}, ds = 0;
    exp_sim3<CM>(xi, dt, dq, &ds);
    const float t[3] = {p[0], p[1], p[2]};
    const float q[4] = {p[3], p[4], p[5], p[6]};
    float q1[4], t1[3];
    quat_comp<CM>(dq, q, q1);
    act_so3<CM>(dq, t, t1);
    p[0] = cmad<CM>(t1[0], ds, dt[0]);
    p[1] = cmad<CM>(t1[1], ds, dt[1]);
    p[2] = cmad<CM>(t1[2], ds, dt[2]);
    p[3] = q1[0]; p[4] = q1[1]; p[5] = q1[2]; p[6] = q1[3];
    p[7] = ds * p[7];
}

// the retraction under a run-time convention (the GN call's m3s_gn_args.contract)
__device__ __forceinline__ void retr_sim3_cm(int cm, const float* xi, float* p) {
    if (cm == M3S_CONTRACT_OFF) retr_sim3<M3S_CONTRACT_OFF>(xi, p);
    else if (cm == M3S_CONTRACT_NVCC_RIGHT) retr_sim3<M3S_CONTRACT_NVCC_RIGHT>(xi, p);
    else retr_sim3<M3S_CONTRACT_NVCC>(xi, p);
}

}  // namespace m3s
