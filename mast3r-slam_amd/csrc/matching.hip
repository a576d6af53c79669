// matching.hip -- MI355X (gfx950) kernels for the iterative projective matcher.
//
//   iter_proj       : per-pixel Levenberg-Marquardt projection of a target ray onto a
//                     9-channel ray+gradient image (reference matching_kernels.cu:119-275)
//   refine_matches  : dilated-window descriptor argmax with c10::Half per-op rounding
//                     (reference matching_kernels.cu:25-81)
//
// Parity contract: bit-exact with the CPU oracle (oracle/m3s_oracle.c) under each FMA-contraction
// convention (contract.h; M3S_CONTRACT_NVCC, the reference build's, by default).  The file is
// compiled with contraction OFF (-ffp-contract=off and the pragma below): every fused operation
// is an explicit helper call placed where nvcc --fmad=true fuses the reference source, and every
// double literal promotion of the reference source is an explicit double operation.
//
// Launch shape (MI355X-first, not the reference's 16-thread blocks): 256-thread
// workgroups (4 wave64s), one point per lane, consecutive lanes on consecutive pixels
// so the bilinear / window gathers of a wave hit the same L1/L2 lines.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstdlib>

#include "../../include/m3s_backend.h"
#include "contract.h"
#include "m3s_common.h"
#include "refine_common.h"

#pragma clang fp contract(off)

using m3s::cdot3;
using m3s::cmad;
using m3s::cmm;

namespace {

__device__ __forceinline__ float clamp_ref(float x, float lo, float hi) {
    return fminf(fmaxf(x, lo), hi);  // matching_kernels.cu:21-23
}


// (float)(1.0 / (double)x) as the IEEE single-precision division 1.0f / x: a float quotient rounded
// to double and then to float equals the correctly rounded float quotient (double rounding is
// innocuous for division when the intermediate has >= 2p + 2 bits: 53 >= 2 * 24 + 2), and the f32
// division sequence is about half the f64 one's cost.  Bit-exactness against the oracle (which
// keeps the literal double division) is tested.
__device__ __forceinline__ float inv_f(float x) { return __fdiv_rn(1.0f, x); }

// Bilinear weights and texel base pointers (matching_kernels.cu:155-170 and :225-239).
struct Bilin {
    float w11, w12, w21, w22;
    const float *r11, *r12, *r21, *r22;
};

__device__ __forceinline__ Bilin make_bilin(const float* __restrict__ img, int W, float u, float v) {
    Bilin b;
    const int u11 = (int)floorf(u);
    const int v11 = (int)floorf(v);
    const float du = u - (float)u11;
    const float dv = v - (float)v11;
    b.w11 = du * dv;
    b.w12 = (float)((1.0 - (double)du) * (double)dv);
    b.w21 = (float)((double)du * (1.0 - (double)dv));
    b.w22 = (float)((1.0 - (double)du) * (1.0 - (double)dv));
    const int64_t row0 = (int64_t)v11 * W;
    const int64_t row1 = (int64_t)(v11 + 1) * W;
    b.r11 = img + (row1 + u11 + 1) * 9;
    b.r12 = img + (row1 + u11) * 9;
    b.r21 = img + (row0 + u11 + 1) * 9;
    b.r22 = img + (row0 + u11) * 9;
    return b;
}


// w11 r11 + w12 r12 + w21 r21 + w22 r22, left to right (matching_kernels.cu:174-183): under nvcc
// the first two products form one fma and the last two are fused into the running sum
template <int CM>
__device__ __forceinline__ float interp(const Bilin& b, int j) {
    return cmad<CM>(b.w22, b.r22[j], cmad<CM>(b.w21, b.r21[j], cmm<CM>(b.w11, b.r11[j], b.w12, b.r12[j])));
}

// matching_kernels.cu:119-275 under contraction convention CM
template <int CM>
__global__ __launch_bounds__(kBlock) void iter_proj_kernel(
    const float* __restrict__ rays, const float* __restrict__ pts, const float* __restrict__ p_init,
    float* __restrict__ p_new, uint8_t* __restrict__ converged, int H, int W, int64_t N,
    int64_t total, int max_iter, float lambda_init, float cost_thresh) {
    const int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (g >= total) return;
    const int64_t b = g / N;
    const float* __restrict__ img = rays + b * (int64_t)H * W * 9;

    const float2 pi = *reinterpret_cast<const float2*>(p_init + g * 2);
    float u = clamp_ref(pi.x, 1.0f, (float)(W - 2));
    float v = clamp_ref(pi.y, 1.0f, (float)(H - 2));
    const float px = pts[g * 3 + 0], py = pts[g * 3 + 1], pz = pts[g * 3 + 2];
    const float umax = (float)(W - 2), vmax = (float)(H - 2);

    float lambda = lambda_init;
    uint8_t conv = 0;
    for (int it = 0; it < max_iter; it++) {
        const Bilin bl = make_bilin(img, W, u, v);
        const float r0 = interp<CM>(bl, 0), r1 = interp<CM>(bl, 1), r2 = interp<CM>(bl, 2);
        const float gx0 = interp<CM>(bl, 3), gx1 = interp<CM>(bl, 4), gx2 = interp<CM>(bl, 5);
        const float gy0 = interp<CM>(bl, 6), gy1 = interp<CM>(bl, 7), gy2 = interp<CM>(bl, 8);

        // :186-198: r *= 1/|r| then err = r - pts (the scaled ray feeds only the subtraction: fused)
        const float r_norm_inv = inv_f(sqrtf(cdot3<CM>(r0, r0, r1, r1, r2, r2)));
        const float e0 = cmad<CM>(r0, r_norm_inv, -px), e1 = cmad<CM>(r1, r_norm_inv, -py),
                    e2 = cmad<CM>(r2, r_norm_inv, -pz);
        const float cost = cdot3<CM>(e0, e0, e1, e1, e2, e2);

        // :202-210
        float A00 = cdot3<CM>(gx0, gx0, gx1, gx1, gx2, gx2);
        const float A01 = cdot3<CM>(gx0, gy0, gx1, gy1, gx2, gy2);
        float A11 = cdot3<CM>(gy0, gy0, gy1, gy1, gy2, gy2);
        const float b0 = -cdot3<CM>(e0, gx0, e1, gx1, e2, gx2);
        const float b1 = -cdot3<CM>(e0, gy0, e1, gy1, e2, gy2);
        A00 += lambda;
        A11 += lambda;

        // :213-219: u + det_inv * (...) is a fused multiply-add under nvcc
        const float det_inv = inv_f(cmm<CM>(A00, A11, -A01, A01));
        const float u_new = clamp_ref(cmad<CM>(det_inv, cmm<CM>(A11, b0, -A01, b1), u), 1.0f, umax);
        const float v_new = clamp_ref(cmad<CM>(det_inv, cmm<CM>(-A01, b0, A00, b1), v), 1.0f, vmax);

        // :225-256 the cost at the new pixel (ray channels only)
        const Bilin bn = make_bilin(img, W, u_new, v_new);
        const float t0 = interp<CM>(bn, 0), t1 = interp<CM>(bn, 1), t2 = interp<CM>(bn, 2);
        const float n2_inv = inv_f(sqrtf(cdot3<CM>(t0, t0, t1, t1, t2, t2)));
        const float f0 = cmad<CM>(t0, n2_inv, -px), f1 = cmad<CM>(t1, n2_inv, -py),
                    f2 = cmad<CM>(t2, n2_inv, -pz);
        const float new_cost = cdot3<CM>(f0, f0, f1, f1, f2, f2);

        if (new_cost < cost) {
            u = u_new;
            v = v_new;
            lambda = (float)((double)lambda * 0.1);  // `lambda *= 0.1` is a double multiply
            conv = new_cost < cost_thresh;
        } else {
            lambda = (float)((double)lambda * 10.0);
            conv = cost < cost_thresh;
        }
    }
    *reinterpret_cast<float2*>(p_new + g * 2) = make_float2(u, v);
    converged[g] = conv;
}

// ---------------------------------------------------------------------------------
// iter_proj on the fused op's ray image: texels of 3 float4 {ray, 0 | d/du, 0 | d/dv, 0} (48 B,
// 16-B aligned: a bilinear tap is 3 x dwordx4 -- the second evaluation only the first --
// instead of 9 dword loads of the reference's 36-B texels), PPT pixels per thread (independent
// chains interleaved: ILP when the launch is small), and the caller's post-processing fused
// (matching.py:66-76: p.long(), the occlusion test ||X11[p1] - X21|| < dist_thresh on the
// pre-refine pixel, valid = converged & that; p1 as (u, v) for refine, or u + W v without it).
// The arithmetic is iter_proj_kernel's, operation for operation (bitwise the same p_new).
// ---------------------------------------------------------------------------------
struct Bilin4 {
    float w11, w12, w21, w22;
    const float4 *r11, *r12, *r21, *r22;
};

__device__ __forceinline__ Bilin4 make_bilin4(const float4* __restrict__ img, int W, float u, float v) {
    Bilin4 b;
    const int u11 = (int)floorf(u);
    const int v11 = (int)floorf(v);
    const float du = u - (float)u11;
    const float dv = v - (float)v11;
    b.w11 = du * dv;
    b.w12 = (float)((1.0 - (double)du) * (double)dv);
    b.w21 = (float)((double)du * (1.0 - (double)dv));
    b.w22 = (float)((1.0 - (double)du) * (1.0 - (double)dv));
    const int64_t row0 = (int64_t)v11 * W;
    const int64_t row1 = (int64_t)(v11 + 1) * W;
    b.r11 = img + (row1 + u11 + 1) * 3;
    b.r12 = img + (row1 + u11) * 3;
    b.r21 = img + (row0 + u11 + 1) * 3;
    b.r22 = img + (row0 + u11) * 3;
    return b;
}

template <int CM>
__device__ __forceinline__ float3 interp4(const Bilin4& b, int c) {
    const float4 t11 = b.r11[c], t12 = b.r12[c], t21 = b.r21[c], t22 = b.r22[c];
    float3 o;
    o.x = cmad<CM>(b.w22, t22.x, cmad<CM>(b.w21, t21.x, cmm<CM>(b.w11, t11.x, b.w12, t12.x)));
    o.y = cmad<CM>(b.w22, t22.y, cmad<CM>(b.w21, t21.y, cmm<CM>(b.w11, t11.y, b.w12, t12.y)));
    o.z = cmad<CM>(b.w22, t22.z, cmad<CM>(b.w21, t21.z, cmm<CM>(b.w11, t11.z, b.w12, t12.z)));
    return o;
}

struct IpState {
    float u, v, lambda, px, py, pz;
    uint8_t conv;
};

// one LM iteration of one pixel (matching_kernels.cu:153-268; iter_proj_kernel's arithmetic)
template <int CM>
__device__ __forceinline__ void ip_step(IpState& s, const float4* __restrict__ img, int W, float umax, float vmax,
                                        float cost_thresh) {
    const Bilin4 bl = make_bilin4(img, W, s.u, s.v);
    const float3 r = interp4<CM>(bl, 0), gx = interp4<CM>(bl, 1), gy = interp4<CM>(bl, 2);
    const float r_norm_inv = inv_f(sqrtf(cdot3<CM>(r.x, r.x, r.y, r.y, r.z, r.z)));
    const float e0 = cmad<CM>(r.x, r_norm_inv, -s.px), e1 = cmad<CM>(r.y, r_norm_inv, -s.py),
                e2 = cmad<CM>(r.z, r_norm_inv, -s.pz);
    const float cost = cdot3<CM>(e0, e0, e1, e1, e2, e2);
    float A00 = cdot3<CM>(gx.x, gx.x, gx.y, gx.y, gx.z, gx.z);
    const float A01 = cdot3<CM>(gx.x, gy.x, gx.y, gy.y, gx.z, gy.z);
    float A11 = cdot3<CM>(gy.x, gy.x, gy.y, gy.y, gy.z, gy.z);
    const float b0 = -cdot3<CM>(e0, gx.x, e1, gx.y, e2, gx.z);
    const float b1 = -cdot3<CM>(e0, gy.x, e1, gy.y, e2, gy.z);
    A00 += s.lambda;
    A11 += s.lambda;
    const float det_inv = inv_f(cmm<CM>(A00, A11, -A01, A01));
    const float u_new = clamp_ref(cmad<CM>(det_inv, cmm<CM>(A11, b0, -A01, b1), s.u), 1.0f, umax);
    const float v_new = clamp_ref(cmad<CM>(det_inv, cmm<CM>(-A01, b0, A00, b1), s.v), 1.0f, vmax);
    const Bilin4 bn = make_bilin4(img, W, u_new, v_new);
    const float3 t = interp4<CM>(bn, 0);
    const float n2_inv = inv_f(sqrtf(cdot3<CM>(t.x, t.x, t.y, t.y, t.z, t.z)));
    const float f0 = cmad<CM>(t.x, n2_inv, -s.px), f1 = cmad<CM>(t.y, n2_inv, -s.py),
                f2 = cmad<CM>(t.z, n2_inv, -s.pz);
    const float new_cost = cdot3<CM>(f0, f0, f1, f1, f2, f2);
    if (new_cost < cost) {
        s.u = u_new;
        s.v = v_new;
        s.lambda = (float)((double)s.lambda * 0.1);
        s.conv = new_cost < cost_thresh;
    } else {
        s.lambda = (float)((double)s.lambda * 10.0);
        s.conv = cost < cost_thresh;
    }
}

template <int CM, int PPT>
__global__ __launch_bounds__(kBlock) void iter_proj_t4_kernel(
    const float4* __restrict__ rays4, const float* __restrict__ pts, const float* __restrict__ p_init,
    const float* __restrict__ X11, const float* __restrict__ X21, int H, int W, int64_t N, int64_t total,
    int64_t span, int max_iter, float lambda_init, float cost_thresh, float dist_thresh,
    int64_t* __restrict__ p1, int64_t* __restrict__ lin, uint8_t* __restrict__ valid) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const float umax = (float)(W - 2), vmax = (float)(H - 2);
    IpState st[PPT];
    const float4* img[PPT];
    int64_t gs[PPT];
    bool live[PPT];
#pragma unroll
    for (int q = 0; q < PPT; q++) {
        const int64_t g = t + q * span;  // pixel sets one span apart: each wave's lanes stay contiguous
        live[q] = g < total;
        gs[q] = live[q] ? g : 0;
        const int64_t b = gs[q] / N;
        img[q] = rays4 + b * (int64_t)H * W * 3;
        const float2 pi = *reinterpret_cast<const float2*>(p_init + gs[q] * 2);
        st[q].u = clamp_ref(pi.x, 1.0f, umax);
        st[q].v = clamp_ref(pi.y, 1.0f, vmax);
        st[q].px = pts[gs[q] * 3 + 0];
        st[q].py = pts[gs[q] * 3 + 1];
        st[q].pz = pts[gs[q] * 3 + 2];
        st[q].lambda = lambda_init;
        st[q].conv = 0;
    }
    for (int it = 0; it < max_iter; it++) {
#pragma unroll
        for (int q = 0; q < PPT; q++) ip_step<CM>(st[q], img[q], W, umax, vmax, cost_thresh);
    }
    const int64_t HW = (int64_t)H * W;
#pragma unroll
    for (int q = 0; q < PPT; q++) {
        if (!live[q]) continue;
        const int64_t g = gs[q];
        const int64_t b = g / HW;
        // p.long() (truncation); iter_proj keeps p inside [1, W-2] x [1, H-2]
        const int64_t u = (int64_t)st[q].u, v = (int64_t)st[q].v;
        const float* a = X11 + (b * HW + v * W + u) * 3;
        const float* x2 = X21 + g * 3;
        const float d0 = a[0] - x2[0], d1 = a[1] - x2[1], d2 = a[2] - x2[2];
        const float dist = __builtin_sqrtf(__builtin_fmaf(d2, d2, __builtin_fmaf(d1, d1, d0 * d0)));
        valid[g] = (st[q].conv != 0) && (dist < dist_thresh);
        if (lin) {
            lin[g] = u + (int64_t)W * v;
        } else {
            p1[g * 2] = u;
            p1[g * 2 + 1] = v;
        }
    }
}

template <int F, int R>
__global__ __launch_bounds__(kBlock) void refine_f16_kernel(
    const uint16_t* __restrict__ D11, const uint16_t* __restrict__ D21,
    const int64_t* __restrict__ p1, int64_t* __restrict__ p1_new, int64_t* __restrict__ lin, int H,
    int W, int64_t N, int64_t B, TileMap tm, int radius_rt, int dilation_max) {
    static_assert(F % 8 == 0, "vector path needs F % 8 == 0");
    int64_t g;
    if (!tile_pixel(tm, B, W, H, g)) return;
    const int64_t b = g / N;

    half2_t q2[F / 2];
    {
        const uint4* src = reinterpret_cast<const uint4*>(D21 + g * F);
#pragma unroll
        for (int c = 0; c < F / 8; c++) {
            uint4 w = src[c];
            const half2_t* hp = reinterpret_cast<const half2_t*>(&w);
#pragma unroll
            for (int k = 0; k < 4; k++) q2[c * 4 + k] = hp[k];
        }
    }
    const uint16_t* __restrict__ img = D11 + b * (int64_t)H * W * F;

    int64_t u0 = p1[g * 2 + 0];
    int64_t v0 = p1[g * 2 + 1];
    half_t max_score = (half_t)kRefineHalfMaxInit;
    int64_t u_new = u0, v_new = v0;
    const int radius = R >= 0 ? R : radius_rt;
    const int S = 2 * radius + 1;
    for (int d = dilation_max; d > 0; d--) {
        const int rd = radius * d;
        for (int i = 0; i < S; i++) {          // u offset outer (matching_kernels.cu:54)
            const int64_t u = u0 - rd + (int64_t)i * d;
            if constexpr (R >= 0) {
                constexpr int SC = 2 * R + 1;
                uint4 rows[SC][F / 8];
                bool ok[SC];
#pragma unroll
                for (int j = 0; j < SC; j++) {  // v offset inner (:55)
                    const int64_t v = v0 - rd + (int64_t)j * d;
                    ok[j] = inside_image(u, v, W, H);
                    const uint4* src = reinterpret_cast<const uint4*>(img + (ok[j] ? (v * W + u) * F : 0));
#pragma unroll
                    for (int c = 0; c < F / 8; c++) rows[j][c] = src[c];
                }
                half_t score[SC];
                score_f16_multi<F, SC>(q2, rows, score);
#pragma unroll
                for (int j = 0; j < SC; j++) {
                    if (ok[j] && score[j] > max_score) {
                        max_score = score[j];
                        u_new = u;
                        v_new = v0 - rd + (int64_t)j * d;
                    }
                }
            } else {
                for (int j = 0; j < S; j++) {
                    const int64_t v = v0 - rd + (int64_t)j * d;
                    if (inside_image(u, v, W, H)) {
                        uint4 row[F / 8];
                        const uint4* src = reinterpret_cast<const uint4*>(img + (v * W + u) * F);
#pragma unroll
                        for (int c = 0; c < F / 8; c++) row[c] = src[c];
                        const half_t score = score_f16<F>(q2, row);
                        if (score > max_score) {
                            max_score = score;
                            u_new = u;
                            v_new = v;
                        }
                    }
                }
            }
        }
        u0 = u_new;
        v0 = v_new;
    }
    store_match(p1_new, lin, g, W, u_new, v_new);
}

template <typename T>
__device__ __forceinline__ T zero_score();
template <>
__device__ __forceinline__ half_t zero_score<half_t>() { return (half_t)0.0f; }
template <>
__device__ __forceinline__ float zero_score<float>() { return 0.0f; }
template <>
__device__ __forceinline__ double zero_score<double>() { return 0.0; }

// `score += D21[k] * D11[k]` (matching_kernels.cu:62): c10::Half rounds the product to half
// before the add (operator* returns Half), so nothing fuses; float / double are fused by nvcc
// --fmad=true (contract.h, M3S_CONTRACT_NVCC)
__device__ __forceinline__ half_t acc_score(half_t s, half_t a, half_t b) {
    const half_t p = a * b;
    return s + p;
}
__device__ __forceinline__ float acc_score(float s, float a, float b) { return __builtin_fmaf(a, b, s); }
__device__ __forceinline__ double acc_score(double s, double a, double b) { return __builtin_fma(a, b, s); }

template <typename T>
__global__ __launch_bounds__(kBlock) void refine_generic_kernel(
    const T* __restrict__ D11, const T* __restrict__ D21, const int64_t* __restrict__ p1,
    int64_t* __restrict__ p1_new, int64_t* __restrict__ lin, int H, int W, int64_t N, int64_t F,
    int64_t total, int radius, int dilation_max, T max_init) {
    const int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (g >= total) return;
    const int64_t b = g / N;
    const T* __restrict__ q = D21 + g * F;
    const T* __restrict__ img = D11 + b * (int64_t)H * W * F;
    int64_t u0 = p1[g * 2 + 0];
    int64_t v0 = p1[g * 2 + 1];
    T max_score = max_init;
    int64_t u_new = u0, v_new = v0;
    const int S = 2 * radius + 1;
    for (int d = dilation_max; d > 0; d--) {
        const int rd = radius * d;
        for (int i = 0; i < S; i++) {
            const int64_t u = u0 - rd + (int64_t)i * d;
            for (int j = 0; j < S; j++) {
                const int64_t v = v0 - rd + (int64_t)j * d;
                if (inside_image(u, v, W, H)) {
                    const T* row = img + (v * W + u) * F;
                    T score = zero_score<T>();
                    for (int64_t k = 0; k < F; k++) score = acc_score(score, q[k], row[k]);
                    if (score > max_score) {
                        max_score = score;
                        u_new = u;
                        v_new = v;
                    }
                }
            }
        }
        u0 = u_new;
        v0 = v_new;
    }
    store_match(p1_new, lin, g, W, u_new, v_new);
}

inline unsigned grid_for(int64_t total) { return (unsigned)((total + kBlock - 1) / kBlock); }

}  // namespace

extern "C" int m3s_iter_proj(const float* rays, const float* pts, const float* p_init,
                             float* p_new, uint8_t* converged, int64_t B, int64_t H, int64_t W,
                             int64_t N, int max_iter, float lambda_init, float cost_thresh,
                             void* stream) {
    return m3s_iter_proj_ex(rays, pts, p_init, p_new, converged, B, H, W, N, max_iter, lambda_init,
                            cost_thresh, M3S_CONTRACT_DEFAULT, stream);
}

extern "C" int m3s_iter_proj_ex(const float* rays, const float* pts, const float* p_init,
                                float* p_new, uint8_t* converged, int64_t B, int64_t H, int64_t W,
                                int64_t N, int max_iter, float lambda_init, float cost_thresh,
                                int contract, void* stream) {
    M3S_REQUIRE(contract == M3S_CONTRACT_NVCC || contract == M3S_CONTRACT_OFF || contract == M3S_CONTRACT_NVCC_RIGHT,
                "iter_proj: unknown contraction convention %d", contract);
    M3S_REQUIRE(B >= 0 && N >= 0, "iter_proj: negative sizes");
    M3S_REQUIRE(H >= 3 && W >= 3, "iter_proj: ray image must be at least 3x3 (got %lldx%lld)",
                (long long)H, (long long)W);
    M3S_REQUIRE(H * W < (int64_t)1 << 31, "iter_proj: image too large");
    const int64_t total = B * N;
    if (total == 0) return M3S_OK;
    M3S_REQUIRE(rays && pts && p_init && p_new && converged, "iter_proj: null pointer");
#define M3S_IP(CM)                                                                                      \
    hipLaunchKernelGGL(iter_proj_kernel<CM>, dim3(grid_for(total)), dim3(kBlock), 0, (hipStream_t)stream, \
                       rays, pts, p_init, p_new, converged, (int)H, (int)W, N, total, max_iter,            \
                       lambda_init, cost_thresh)
    if (contract == M3S_CONTRACT_OFF) M3S_IP(M3S_CONTRACT_OFF);
    else if (contract == M3S_CONTRACT_NVCC) M3S_IP(M3S_CONTRACT_NVCC);
    else M3S_IP(M3S_CONTRACT_NVCC_RIGHT);
#undef M3S_IP
    M3S_LAUNCH_CHECK();
    return M3S_OK;
}

namespace m3s {
// iter_proj + the caller's post-processing on the fused op's float4-texel ray image (above)
int iter_proj_t4_launch(const float* rays4, const float* pts, const float* p_init, const float* X11,
                        const float* X21, int64_t B, int64_t H, int64_t W, int max_iter, float lambda_init,
                        float cost_thresh, float dist_thresh, int contract, int64_t* p1, int64_t* lin,
                        uint8_t* valid, hipStream_t st) {
    M3S_REQUIRE(contract == M3S_CONTRACT_NVCC || contract == M3S_CONTRACT_OFF || contract == M3S_CONTRACT_NVCC_RIGHT,
                "iter_proj: unknown contraction convention %d", contract);
    const int64_t N = H * W, total = B * N;
    if (total == 0) return M3S_OK;
    // two pixels per thread while that still leaves >= ~2 waves per SIMD (small launches:
    // their chains interleave); one otherwise.  M3S_IP_PPT=1|2 forces it.
    static const int ppt_env = [] {
        const char* e = getenv("M3S_IP_PPT");
        return e ? atoi(e) : 0;
    }();
    const int ppt = ppt_env == 1 || ppt_env == 2 ? ppt_env : (total <= 262144 ? 2 : 1);
    const int64_t span = (total + ppt - 1) / ppt;
    const float4* r4 = reinterpret_cast<const float4*>(rays4);
#define M3S_IPT(CM, P)                                                                                          \
    hipLaunchKernelGGL((iter_proj_t4_kernel<CM, P>), dim3(grid_for(span)), dim3(kBlock), 0, st, r4, pts, p_init, \
                       X11, X21, (int)H, (int)W, N, total, span, max_iter, lambda_init, cost_thresh, dist_thresh,  \
                       p1, lin, valid)
#define M3S_IPT_P(CM)      \
    if (ppt == 2) M3S_IPT(CM, 2); \
    else M3S_IPT(CM, 1)
    if (contract == M3S_CONTRACT_OFF) M3S_IPT_P(M3S_CONTRACT_OFF);
    else if (contract == M3S_CONTRACT_NVCC_RIGHT) M3S_IPT_P(M3S_CONTRACT_NVCC_RIGHT);
    else M3S_IPT_P(M3S_CONTRACT_NVCC);
#undef M3S_IPT_P
#undef M3S_IPT
    M3S_LAUNCH_CHECK();
    return M3S_OK;
}

// refine_matches on fp16 descriptors; lin != nullptr writes u + W v per pixel instead of (u, v)
int refine_f16_launch(const uint16_t* D11, const uint16_t* D21, const int64_t* p1, int64_t* p1_new,
                      int64_t* lin, int64_t B, int64_t H, int64_t W, int64_t N, int64_t F, int radius,
                      int dilation_max, hipStream_t st) {
    int rc = refine_checks(D11, D21, p1, lin ? (void*)lin : (void*)p1_new, B, H, W, N, F, radius, dilation_max);
    if (rc) return rc;
    const int64_t total = B * N;
    if (total == 0) return M3S_OK;
    const bool aligned = ((uintptr_t)D11 % 16 == 0) && ((uintptr_t)D21 % 16 == 0);
    if (F == 24 && aligned && N == H * W) {
        TileMap tm;
        tm.tiles_x = (int)((W + kTile - 1) / kTile);
        tm.tiles_y = (int)((H + kTile - 1) / kTile);
        tm.ntiles = tm.tiles_x * tm.tiles_y;
        const int64_t nblk = (int64_t)tm.ntiles * B;
        const int64_t grid = (nblk + 7) / 8 * 8;  // whole rounds of the 8 XCDs
        if (radius == 3)  // base.yaml:13
            hipLaunchKernelGGL((refine_f16_kernel<24, 3>), dim3((unsigned)grid), dim3(kBlock), 0, st, D11, D21,
                               p1, p1_new, lin, (int)H, (int)W, N, B, tm, radius, dilation_max);
        else
            hipLaunchKernelGGL((refine_f16_kernel<24, -1>), dim3((unsigned)grid), dim3(kBlock), 0, st, D11, D21,
                               p1, p1_new, lin, (int)H, (int)W, N, B, tm, radius, dilation_max);
    } else {
        hipLaunchKernelGGL(refine_generic_kernel<half_t>, dim3(grid_for(total)), dim3(kBlock), 0, st,
                           reinterpret_cast<const half_t*>(D11), reinterpret_cast<const half_t*>(D21), p1,
                           p1_new, lin, (int)H, (int)W, N, F, total, radius, dilation_max,
                           (half_t)kRefineHalfMaxInit);
    }
    M3S_LAUNCH_CHECK();
    return M3S_OK;
}
}  // namespace m3s

extern "C" int m3s_refine_matches_f16(const uint16_t* D11, const uint16_t* D21, const int64_t* p1,
                                      int64_t* p1_new, int64_t B, int64_t H, int64_t W, int64_t N,
                                      int64_t F, int radius, int dilation_max, void* stream) {
    return m3s::refine_f16_launch(D11, D21, p1, p1_new, nullptr, B, H, W, N, F, radius, dilation_max,
                                  (hipStream_t)stream);
}

extern "C" int m3s_refine_matches_f32(const float* D11, const float* D21, const int64_t* p1,
                                      int64_t* p1_new, int64_t B, int64_t H, int64_t W, int64_t N,
                                      int64_t F, int radius, int dilation_max, void* stream) {
    int rc = refine_checks(D11, D21, p1, p1_new, B, H, W, N, F, radius, dilation_max);
    if (rc) return rc;
    const int64_t total = B * N;
    if (total == 0) return M3S_OK;
    hipLaunchKernelGGL(refine_generic_kernel<float>, dim3(grid_for(total)), dim3(kBlock), 0,
                       (hipStream_t)stream, D11, D21, p1, p1_new, nullptr, (int)H, (int)W, N, F, total,
                       radius, dilation_max, kRefineFloatMaxInit);
    M3S_LAUNCH_CHECK();
    return M3S_OK;
}

extern "C" int m3s_refine_matches_f64(const double* D11, const double* D21, const int64_t* p1,
                                      int64_t* p1_new, int64_t B, int64_t H, int64_t W, int64_t N,
                                      int64_t F, int radius, int dilation_max, void* stream) {
    int rc = refine_checks(D11, D21, p1, p1_new, B, H, W, N, F, radius, dilation_max);
    if (rc) return rc;
    const int64_t total = B * N;
    if (total == 0) return M3S_OK;
    hipLaunchKernelGGL(refine_generic_kernel<double>, dim3(grid_for(total)), dim3(kBlock), 0,
                       (hipStream_t)stream, D11, D21, p1, p1_new, nullptr, (int)H, (int)W, N, F, total,
                       radius, dilation_max, kRefineDoubleMaxInit);
    M3S_LAUNCH_CHECK();
    return M3S_OK;
}
