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

#pragma clang fp contract(off)

using m3s::cdot3;
using m3s::cmad;
using m3s::cmm;

namespace {

constexpr int kBlock = 256;

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

// ---------------------------------------------------------------------------------
// refine_matches
// ---------------------------------------------------------------------------------

// cuda::std::numeric_limits<c10::Half>::min() is value-initialised (no libcu++
// specialisation for c10::Half) => 0.0.  Single named constant, see DESIGN.md.
constexpr float kRefineHalfMaxInit = 0.0f;
// For float and double the limits are specialised: FLT_MIN, DBL_MIN.
constexpr float kRefineFloatMaxInit = 1.17549435e-38f;
constexpr double kRefineDoubleMaxInit = 2.2250738585072014e-308;

__device__ __forceinline__ bool inside_image(int64_t u, int64_t v, int W, int H) {
    return v >= 0 && v < H && u >= 0 && u < W;  // matching_kernels.cu:17-19
}

typedef _Float16 half_t;

// The refined match as (u, v), or (fused matching pipeline) as the linear index u + W v the
// caller forms next (matching.py:13-15, 87).
__device__ __forceinline__ void store_match(int64_t* __restrict__ p1_new, int64_t* __restrict__ lin,
                                            int64_t g, int W, int64_t u, int64_t v) {
    if (lin) {
        lin[g] = u + (int64_t)W * v;
    } else {
        p1_new[g * 2 + 0] = u;
        p1_new[g * 2 + 1] = v;
    }
}

// F = 24 fp16 fast path: the query descriptor lives in registers (3 x 16 B loads),
// each candidate row is 48 B = 3 x dwordx4.  Sequential fp16 accumulation exactly as
// c10::Half: round after every * and after every +=.
// Pixel order (locality of the candidate gathers): a workgroup takes a 16x16 pixel tile (a
// wave 4 rows x 16), and tiles are handed out so that the 8 XCDs (workgroups b, b+8, ... share
// an XCD) each sweep a contiguous band of tile rows: an XCD's candidate windows then cover
// ~1/8 of D11 (+ the search radius), which stays in its L2.  Pure performance mapping: every
// pixel is computed exactly once whatever the placement.
constexpr int kTile = 16;
struct TileMap {
    int tiles_x, tiles_y, ntiles;  // per image
};
__device__ __forceinline__ bool tile_pixel(const TileMap& tm, int64_t B, int W, int H, int64_t& g) {
    const int64_t nblk = (int64_t)gridDim.x;
    const int64_t blk = blockIdx.x;
    // XCD-aware: logical block = (blk % 8) * ceil(nblk / 8) + blk / 8
    const int64_t per = (nblk + 7) / 8;
    const int64_t lb = (blk % 8) * per + blk / 8;
    if (lb >= (int64_t)tm.ntiles * B) return false;
    const int64_t b = lb / tm.ntiles;
    const int t = (int)(lb - b * tm.ntiles);
    const int ty = t / tm.tiles_x, tx = t - ty * tm.tiles_x;
    const int lx = threadIdx.x & (kTile - 1), ly = threadIdx.x / kTile;
    const int u = tx * kTile + lx, v = ty * kTile + ly;
    if (u >= W || v >= H) return false;
    g = b * (int64_t)H * W + (int64_t)v * W + u;
    return true;
}

typedef _Float16 half2_t __attribute__((ext_vector_type(2)));

// One candidate's score with c10::Half semantics: p_k = fl16(q_k * h_k), s = fl16(s + p_k) in
// k order.  The products are formed two at a time (v_pk_mul_f16 rounds each half exactly like
// the scalar multiply); the sum stays a sequential chain.
template <int F>
__device__ __forceinline__ half_t score_f16(const half2_t (&q2)[F / 2], const uint4 (&row)[F / 8]) {
    half_t score = (half_t)0.0f;
#pragma unroll
    for (int c = 0; c < F / 8; c++) {
        const half2_t* hp = reinterpret_cast<const half2_t*>(&row[c]);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const half2_t p = q2[c * 4 + k] * hp[k];
            score = score + p.x;
            score = score + p.y;
        }
    }
    return score;
}

// SC candidates' scores at once, each exactly score_f16 (the same per-candidate sequence of
// roundings), but with the k loop outermost so the SC dependent add chains interleave: a
// single chain is one dependent v_add_f16 after another, and the compiler does not interleave
// independent chains on its own.
template <int F, int SC>
__device__ __forceinline__ void score_f16_multi(const half2_t (&q2)[F / 2], const uint4 (&rows)[SC][F / 8],
                                                half_t (&score)[SC]) {
#pragma unroll
    for (int j = 0; j < SC; j++) score[j] = (half_t)0.0f;
#pragma unroll
    for (int c = 0; c < F / 8; c++) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            half2_t p[SC];
#pragma unroll
            for (int j = 0; j < SC; j++) p[j] = q2[c * 4 + k] * reinterpret_cast<const half2_t*>(&rows[j][c])[k];
#pragma unroll
            for (int j = 0; j < SC; j++) score[j] = score[j] + p[j].x;
            __builtin_amdgcn_sched_barrier(0);  // keep the chains interleaved (see above)
#pragma unroll
            for (int j = 0; j < SC; j++) score[j] = score[j] + p[j].y;
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

// F = 24 fp16 fast path: the query descriptor lives in registers (3 x 16 B loads), each
// candidate row is 48 B = 3 x dwordx4.  R = radius when it is a compile-time constant (the
// window column of 2R+1 candidates is unrolled: its loads are issued together and the
// independent score chains interleave), R < 0 for any radius.
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

// ---------------------------------------------------------------------------------
// refine_matches with the correlation on MFMA (opt-in M3S_REFINE_MFMA=1; SURVEY §8(d) prices the
// correlation against the fp16 matrix peak).  Exact by construction:
//
//  1. approximate scores: per dilation level, candidate c (of 49) of 16 pixels at once as one
//     v_mfma_f32_16x16x32_f16: A = the 16 pixels' descriptors (K = 24, zero-padded to 32), B = the
//     16 pixels' candidate-c descriptors, gathered (out-of-image / padding lanes: zeros); the
//     16 wanted dot products are the diagonal of the 16x16 product (fp16 products are exact in
//     fp32, the sum rounds in fp32).  The windows of neighbouring pixels are on different
//     dilation lattices, so no candidate row is shared by two pixels -- the MFMA does 16x the
//     needed MACs and the gathers are the same as the VALU kernel's.
//  2. bound: |s_half - s_mfma| <= E = 0.0126 * ||q|| * Hmax + 4e-6, where s_half is the
//     c10::Half score (24 roundings of products, 24 of the running sum, each <= 2^-11 relative
//     via fp32: 25 * (2^-11 + 2^-23) * 1.015 < 0.0126 of sum |q_k h_k| <= ||q|| ||h||, plus the
//     fp16 subnormal half-spacing 2^-25 per rounding and the MFMA's own fp32 error), Hmax = the
//     largest ||h|| in the image (refine_hmax_kernel).  Non-finite or huge bounds: every
//     candidate is re-scored.
//  3. exact re-scoring: with L = max (s_mfma - E) over the pixel's in-image candidates, only
//     candidates with s_mfma + E >= L (every possible argmax, ties included) and s_mfma + E >
//     max_score (so it could pass the strict '>') get the exact fp16 chain, in the reference's
//     candidate order -> the same winner and the same persisted max_score as scoring all 49.
// ---------------------------------------------------------------------------------
typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef float float4_t __attribute__((ext_vector_type(4)));
constexpr float kRefineBoundRel = 0.0126f;
constexpr float kRefineBoundAbs = 4e-6f;
constexpr float kRefineBoundMax = 3.0e4f;  // sum |q h| beyond: fp16 overflow possible, score all

// per image: max over pixels of sum_k h_k^2 (float bits; +inf if any value is not finite)
__global__ __launch_bounds__(kBlock) void refine_hmax_kernel(const uint16_t* __restrict__ D11, int64_t HW,
                                                             unsigned* __restrict__ hmax2) {
    const int64_t b = blockIdx.y;
    float m = 0.0f;
    for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < HW; p += (int64_t)gridDim.x * kBlock) {
        const uint4* src = reinterpret_cast<const uint4*>(D11 + (b * HW + p) * 24);
        float s = 0.0f;
#pragma unroll
        for (int c = 0; c < 3; c++) {
            uint4 w = src[c];
            const half_t* h = reinterpret_cast<const half_t*>(&w);
#pragma unroll
            for (int k = 0; k < 8; k++) s = fmaf((float)h[k], (float)h[k], s);
        }
        m = (s == s && s <= 3.0e38f) ? fmaxf(m, s) : __int_as_float(0x7f800000);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
    if ((threadIdx.x & 63) == 0) atomicMax(hmax2 + b, __float_as_uint(m));
}

template <int R>
__global__ __launch_bounds__(kBlock) void refine_mfma_kernel(
    const uint16_t* __restrict__ D11, const uint16_t* __restrict__ D21, const int64_t* __restrict__ p1,
    int64_t* __restrict__ p1_new, int64_t* __restrict__ lin, int H, int W, int64_t N, int64_t B, TileMap tm,
    int dilation_max, const unsigned* __restrict__ hmax2, unsigned long long* __restrict__ stats) {
    constexpr int F = 24;
    constexpr int S = 2 * R + 1;
    constexpr int NC = S * S;
    static_assert(NC <= 64, "candidate mask is 64 bits");
    __shared__ float sc[kBlock / 64][NC][64];  // approximate scores, per wave: [candidate][pixel]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int64_t g = 0;
    const bool active = tile_pixel(tm, B, W, H, g);  // every lane stays for the MFMAs
    const int64_t b = active ? g / N : 0;
    const uint16_t* __restrict__ img = D11 + b * (int64_t)H * W * F;

    half2_t q2[F / 2];
    float qn2 = 0.0f;
    {
        const uint4* src = reinterpret_cast<const uint4*>(D21 + (active ? g : 0) * F);
#pragma unroll
        for (int c = 0; c < F / 8; c++) {
            uint4 w = src[c];
            const half2_t* hp = reinterpret_cast<const half2_t*>(&w);
#pragma unroll
            for (int k = 0; k < 4; k++) {
                q2[c * 4 + k] = hp[k];
                qn2 = fmaf((float)hp[k].x, (float)hp[k].x, fmaf((float)hp[k].y, (float)hp[k].y, qn2));
            }
        }
    }
    // A fragments of the wave's 4 row groups: lane l holds pixel (16 r + (l & 15))'s descriptor
    // elements 8 (l >> 4) .. + 7 (zeros for the K padding 24..31)
    const int kc = lane >> 4, col = lane & 15;
    half8_t A[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int64_t gp = __shfl(g, 16 * r + col, 64);
        const bool ap = __shfl((int)active, 16 * r + col, 64) != 0;
        uint4 w = make_uint4(0, 0, 0, 0);
        if (kc < 3 && ap) w = reinterpret_cast<const uint4*>(D21 + gp * F)[kc];
        A[r] = __builtin_bit_cast(half8_t, w);
    }
    // the diagonal of a 16x16 tile: lane l holds C[4 (l >> 4) + q][l & 15]; it is (col, col)
    // for the 16 lanes with (col >> 2) == kc, at q = col & 3
    const bool diag = (col >> 2) == kc;
    const int dq = col & 3;
    const float hmax = sqrtf(__uint_as_float(hmax2[b])) * 1.00001f;
    const float pbound = (sqrtf(qn2) * 1.00001f) * hmax;  // >= sum_k |q_k h_k| for every candidate
    const float E = kRefineBoundRel * pbound + kRefineBoundAbs;
    const bool score_all = !(pbound <= kRefineBoundMax);  // NaN / inf / fp16 overflow possible

    int64_t u0 = active ? p1[g * 2 + 0] : 0;
    int64_t v0 = active ? p1[g * 2 + 1] : 0;
    half_t max_score = (half_t)kRefineHalfMaxInit;
    int64_t u_new = u0, v_new = v0;
    unsigned nresc = 0, ntotal = 0;
    for (int d = dilation_max; d > 0; d--) {
        const int64_t rd = (int64_t)R * d;
        // 1. approximate scores of the 4 row groups' candidates
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int64_t uc = __shfl(u0, 16 * r + col, 64), vc = __shfl(v0, 16 * r + col, 64);
#pragma unroll
            for (int i = 0; i < S; i++) {
                const int64_t u = uc - rd + (int64_t)i * d;
#pragma unroll
                for (int j = 0; j < S; j++) {
                    const int64_t v = vc - rd + (int64_t)j * d;
                    uint4 w = make_uint4(0, 0, 0, 0);
                    if (kc < 3 && inside_image(u, v, W, H))
                        w = reinterpret_cast<const uint4*>(img + (v * W + u) * F)[kc];
                    float4_t acc = {0.0f, 0.0f, 0.0f, 0.0f};
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[r], __builtin_bit_cast(half8_t, w), acc, 0, 0, 0);
                    const float dv = dq == 0 ? acc[0] : dq == 1 ? acc[1] : dq == 2 ? acc[2] : acc[3];
                    if (diag) sc[wave][i * S + j][16 * r + col] = dv;
                }
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's score writes landed
        __builtin_amdgcn_wave_barrier();
        // 2. shortlist: every candidate that can be the level's first argmax and beat max_score
        uint64_t mask = 0;
        float lo = -__int_as_float(0x7f800000);
#pragma unroll
        for (int c = 0; c < NC; c++) {
            const int64_t u = u0 - rd + (int64_t)(c / S) * d, v = v0 - rd + (int64_t)(c % S) * d;
            if (inside_image(u, v, W, H)) lo = fmaxf(lo, sc[wave][c][lane] - E);
        }
        const float beat = (float)max_score;
#pragma unroll
        for (int c = 0; c < NC; c++) {
            const int64_t u = u0 - rd + (int64_t)(c / S) * d, v = v0 - rd + (int64_t)(c % S) * d;
            const float hi = sc[wave][c][lane] + E;
            const bool in = inside_image(u, v, W, H);
            ntotal += in;
            if (in && (score_all || (hi >= lo && hi > beat))) mask |= 1ull << c;
        }
        if (!active) mask = 0;
        nresc += __builtin_popcountll(mask);
        // 3. exact c10::Half scores of the shortlist, in candidate order
        while (mask) {
            const int c = __builtin_ctzll(mask);
            mask &= mask - 1;
            const int64_t u = u0 - rd + (int64_t)(c / S) * d, v = v0 - rd + (int64_t)(c % S) * d;
            uint4 row[F / 8];
            const uint4* src = reinterpret_cast<const uint4*>(img + (v * W + u) * F);
#pragma unroll
            for (int k = 0; k < F / 8; k++) row[k] = src[k];
            const half_t score = score_f16<F>(q2, row);
            if (score > max_score) {
                max_score = score;
                u_new = u;
                v_new = v;
            }
        }
        u0 = u_new;
        v0 = v_new;
        __builtin_amdgcn_wave_barrier();  // the next level overwrites this wave's scores
    }
    if (active) store_match(p1_new, lin, g, W, u_new, v_new);
    if (stats) {  // diagnostics: candidates re-scored exactly / in-image candidates
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            nresc += __shfl_xor(nresc, off, 64);
            ntotal += __shfl_xor(ntotal, off, 64);
        }
        if (lane == 0) {
            atomicAdd(stats, (unsigned long long)nresc);
            atomicAdd(stats + 1, (unsigned long long)ntotal);
        }
    }
}

// ---------------------------------------------------------------------------------
// refine_matches, bound-and-rescore on the VALU (opt-in M3S_REFINE_DOT2=1).  The same
// exactness argument as refine_mfma_kernel, with the approximate scores from v_dot2c_f32_f16
// (12 per candidate: fp16 products exact in fp32, fp32 sums) instead of 48 half-precision ops:
//   1. per window column, the 7 candidates' rows are loaded together (as refine_f16_kernel) and
//      their approximate scores computed as 7 interleaved dot2 chains; the best lower bound
//      L = max (s - E) over the in-image candidates is tracked;
//   2. the exact c10::Half chain runs only for candidates with s + E >= L and s + E > max_score,
//      in the reference's candidate order -> the same winner and persisted max_score.
// E = 0.0126 ||q|| Hmax (the fp16 chain's rounding, see refine_mfma_kernel) + 24 * 2^-14 *
// max(||q||, Hmax) (the terms an fp16-denormal flush inside dot2 could drop: a subnormal
// factor is < 2^-14 and the other <= the norm bound) + 4e-6.
// ---------------------------------------------------------------------------------
constexpr float kRefineFlushRel = 24.0f / 16384.0f;

#ifndef M3S_REFINE_DOT2_WAVES
#define M3S_REFINE_DOT2_WAVES 1
#endif
template <int R>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(M3S_REFINE_DOT2_WAVES))) void refine_dot2_kernel(
    const uint16_t* __restrict__ D11, const uint16_t* __restrict__ D21, const int64_t* __restrict__ p1,
    int64_t* __restrict__ p1_new, int64_t* __restrict__ lin, int H, int W, int64_t N, int64_t B, TileMap tm,
    int dilation_max, const unsigned* __restrict__ hmax2, unsigned long long* __restrict__ stats) {
    constexpr int F = 24;
    constexpr int S = 2 * R + 1;
    constexpr int NC = S * S;
    static_assert(NC <= 64, "candidate mask is 64 bits");
    int64_t g;
    unsigned nresc = 0, ntotal = 0;
    const bool active = tile_pixel(tm, B, W, H, g);
    if (active) {
        const int64_t b = g / N;
        const uint16_t* __restrict__ img = D11 + b * (int64_t)H * W * F;
        half2_t q2[F / 2];
        float qn2 = 0.0f;
        {
            const uint4* src = reinterpret_cast<const uint4*>(D21 + g * F);
#pragma unroll
            for (int c = 0; c < F / 8; c++) {
                uint4 w = src[c];
                const half2_t* hp = reinterpret_cast<const half2_t*>(&w);
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    q2[c * 4 + k] = hp[k];
                    qn2 = fmaf((float)hp[k].x, (float)hp[k].x, fmaf((float)hp[k].y, (float)hp[k].y, qn2));
                }
            }
        }
        const float hmax = sqrtf(__uint_as_float(hmax2[b])) * 1.00001f;
        const float qn = sqrtf(qn2) * 1.00001f;
        const float pbound = qn * hmax;
        const float E = kRefineBoundRel * pbound + kRefineFlushRel * fmaxf(qn, hmax) + kRefineBoundAbs;
        const bool score_all = !(pbound <= kRefineBoundMax) || !(E <= kRefineBoundMax);

        int64_t u0 = p1[g * 2 + 0];
        int64_t v0 = p1[g * 2 + 1];
        half_t max_score = (half_t)kRefineHalfMaxInit;
        int64_t u_new = u0, v_new = v0;
        for (int d = dilation_max; d > 0; d--) {
            const int64_t rd = (int64_t)R * d;
            float sa[NC];
            float lo = -__int_as_float(0x7f800000);
            uint64_t inimg = 0;
#pragma unroll
            for (int i = 0; i < S; i++) {  // u offset outer (matching_kernels.cu:54)
                const int64_t u = u0 - rd + (int64_t)i * d;
                uint4 rows[S][F / 8];
#pragma unroll
                for (int j = 0; j < S; j++) {
                    const int64_t v = v0 - rd + (int64_t)j * d;
                    const bool ok = inside_image(u, v, W, H);
                    inimg |= (uint64_t)ok << (i * S + j);
                    const uint4* src = reinterpret_cast<const uint4*>(img + (ok ? (v * W + u) * F : 0));
#pragma unroll
                    for (int c = 0; c < F / 8; c++) rows[j][c] = src[c];
                }
                float acc[S];
#pragma unroll
                for (int j = 0; j < S; j++) acc[j] = 0.0f;
#pragma unroll
                for (int c = 0; c < F / 8; c++) {
#pragma unroll
                    for (int k = 0; k < 4; k++) {
#pragma unroll
                        for (int j = 0; j < S; j++)
                            acc[j] = __builtin_amdgcn_fdot2(q2[c * 4 + k],
                                                            reinterpret_cast<const half2_t*>(&rows[j][c])[k],
                                                            acc[j], false);
                    }
                }
#pragma unroll
                for (int j = 0; j < S; j++) {
                    sa[i * S + j] = acc[j];
                    if ((inimg >> (i * S + j)) & 1) lo = fmaxf(lo, acc[j] - E);
                }
                // one window column's rows in flight at a time: pin this column's scores here (the
                // compiler would otherwise sink all 49 dot2 chains below the level's 147 row loads,
                // keeping every row live, and spill)
#pragma unroll
                for (int j = 0; j < S; j++) asm volatile("" : "+v"(sa[i * S + j]));
                asm volatile("" : "+v"(lo));
                __builtin_amdgcn_sched_barrier(0);
            }
            const float beat = (float)max_score;
            uint64_t mask = 0;
#pragma unroll
            for (int c = 0; c < NC; c++) {
                const float hi = sa[c] + E;
                if (score_all || (hi >= lo && hi > beat)) mask |= 1ull << c;
            }
            mask &= inimg;
            nresc += __builtin_popcountll(mask);
            ntotal += __builtin_popcountll(inimg);
            while (mask) {  // exact c10::Half scores of the shortlist, in candidate order
                const int c = __builtin_ctzll(mask);
                mask &= mask - 1;
                const int64_t u = u0 - rd + (int64_t)(c / S) * d, v = v0 - rd + (int64_t)(c % S) * d;
                uint4 row[F / 8];
                const uint4* src = reinterpret_cast<const uint4*>(img + (v * W + u) * F);
#pragma unroll
                for (int k = 0; k < F / 8; k++) row[k] = src[k];
                const half_t score = score_f16<F>(q2, row);
                if (score > max_score) {
                    max_score = score;
                    u_new = u;
                    v_new = v;
                }
            }
            u0 = u_new;
            v0 = v_new;
        }
        store_match(p1_new, lin, g, W, u_new, v_new);
    }
    if (stats) {  // diagnostics: candidates re-scored exactly / in-image candidates
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            nresc += __shfl_xor(nresc, off, 64);
            ntotal += __shfl_xor(ntotal, off, 64);
        }
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(stats, (unsigned long long)nresc);
            atomicAdd(stats + 1, (unsigned long long)ntotal);
        }
    }
}

// ---------------------------------------------------------------------------------
// refine_matches, LDS-tiled (F = 24 fp16, radius 3): opt-in (M3S_REFINE_LDS=1), measured slower.
//
// The gather kernel above reads every candidate row (48 B) through the vector L1 / texture path:
// 735 dwordx4 gathers per pixel, ~16 TA cycles each per wave -- the PMC profile shows it
// issue-stalled (SQ_WAIT_INST_ANY 72 % of wave cycles), not arithmetic-bound.  Here a
// 512-thread workgroup takes a 32x16 pixel tile; for each dilation level it
// stages, once, the descriptor rows of the bounding box of all its pixels' (image-clipped)
// candidate windows into LDS (row by row, coalesced 16-B loads), then every pixel scores its
// candidates from LDS (3 x ds_read_b128 per candidate).  Same candidate order, same c10::Half
// arithmetic (score_f16), same strict '>' updates => bitwise the gather kernel's result.  A
// level whose box exceeds the LDS budget (widely scattered matches) reads the candidates from
// global memory for that level only.  Measured (MI355X, bench data = GT matches +- 2 px per
// pixel): 0.93-0.96 vs 0.86 ms for 8 pairs: one 158-KB workgroup per CU leaves 2 waves per SIMD
// waiting on LDS (SQ_WAIT_ANY 64 %), the per-pixel +-2 px jitter makes the ds_read_b128s 2-way
// bank-conflicted on average, and every level's staging is a workgroup-wide stall; prefetching
// the next window column's rows (two register buffers) did not change it.
// ---------------------------------------------------------------------------------
constexpr int kLdsTx = 32, kLdsTy = 16, kLdsThreads = kLdsTx * kLdsTy;
constexpr int kLdsCapPx = 3300;  // 3300 x 48 B = 158,400 B of the CU's 160 KiB
struct LdsTileMap {
    int tiles_x, tiles_y, ntiles;  // per image
};

__device__ __forceinline__ void block_minmax4(int (&v)[4], int* red /* [8 waves][4] */) {
    // v[0], v[2] reduced with min, v[1], v[3] with max, over the workgroup
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        v[0] = min(v[0], __shfl_xor(v[0], off, 64));
        v[1] = max(v[1], __shfl_xor(v[1], off, 64));
        v[2] = min(v[2], __shfl_xor(v[2], off, 64));
        v[3] = max(v[3], __shfl_xor(v[3], off, 64));
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) {
        red[wave * 4 + 0] = v[0];
        red[wave * 4 + 1] = v[1];
        red[wave * 4 + 2] = v[2];
        red[wave * 4 + 3] = v[3];
    }
    __syncthreads();
#pragma unroll
    for (int w = 0; w < kLdsThreads / 64; w++) {
        v[0] = min(v[0], red[w * 4 + 0]);
        v[1] = max(v[1], red[w * 4 + 1]);
        v[2] = min(v[2], red[w * 4 + 2]);
        v[3] = max(v[3], red[w * 4 + 3]);
    }
}

template <int F, int R>
__global__ __launch_bounds__(kLdsThreads) void refine_lds_kernel(
    const uint16_t* __restrict__ D11, const uint16_t* __restrict__ D21,
    const int64_t* __restrict__ p1, int64_t* __restrict__ p1_new, int64_t* __restrict__ lin, int H,
    int W, int64_t B, LdsTileMap tm, int dilation_max, int* __restrict__ stats) {
    static_assert(F == 24, "LDS tile path is for 24-d fp16 descriptors (48-B rows)");
    constexpr int SC = 2 * R + 1;
    constexpr int RU4 = F / 8;  // uint4 per descriptor row
    __shared__ uint4 tile[kLdsCapPx * RU4];
    __shared__ int red[(kLdsThreads / 64) * 4];

    // XCD-banded tile order, as refine_f16_kernel
    const int64_t nblk = (int64_t)gridDim.x;
    const int64_t blk = blockIdx.x;
    const int64_t per = (nblk + 7) / 8;
    const int64_t lb = (blk % 8) * per + blk / 8;
    if (lb >= (int64_t)tm.ntiles * B) return;  // block-uniform
    const int64_t b = lb / tm.ntiles;
    const int t = (int)(lb - b * tm.ntiles);
    const int ty = t / tm.tiles_x, tx = t - ty * tm.tiles_x;
    const int lx = threadIdx.x & (kLdsTx - 1), ly = threadIdx.x / kLdsTx;
    const int pu = tx * kLdsTx + lx, pv = ty * kLdsTy + ly;
    const bool active = pu < W && pv < H;
    const int64_t N = (int64_t)H * W;
    const int64_t g = b * N + (int64_t)pv * W + pu;
    const uint16_t* __restrict__ img = D11 + b * N * F;

    half2_t q2[F / 2];
    int64_t u0 = 0, v0 = 0;
    if (active) {
        const uint4* src = reinterpret_cast<const uint4*>(D21 + g * F);
#pragma unroll
        for (int c = 0; c < RU4; c++) {
            uint4 w = src[c];
            const half2_t* hp = reinterpret_cast<const half2_t*>(&w);
#pragma unroll
            for (int k = 0; k < 4; k++) q2[c * 4 + k] = hp[k];
        }
        u0 = p1[g * 2 + 0];
        v0 = p1[g * 2 + 1];
    }
    half_t max_score = (half_t)kRefineHalfMaxInit;
    int64_t u_new = u0, v_new = v0;
    int n_global_levels = 0;

    for (int d = dilation_max; d > 0; d--) {
        const int64_t rd = (int64_t)R * d;
        // this pixel's candidate window clipped to the image (empty: lo > hi)
        int w4[4] = {INT_MAX, INT_MIN, INT_MAX, INT_MIN};
        if (active) {
            const int64_t ulo = max(u0 - rd, (int64_t)0), uhi = min(u0 + rd, (int64_t)W - 1);
            const int64_t vlo = max(v0 - rd, (int64_t)0), vhi = min(v0 + rd, (int64_t)H - 1);
            if (ulo <= uhi && vlo <= vhi) {
                w4[0] = (int)ulo;
                w4[1] = (int)uhi;
                w4[2] = (int)vlo;
                w4[3] = (int)vhi;
            }
        }
        block_minmax4(w4, red);
        const int umin = w4[0], umax = w4[1], vmin = w4[2], vmax = w4[3];
        const bool any = umin <= umax;
        const int Rw = any ? umax - umin + 1 : 0, Rh = any ? vmax - vmin + 1 : 0;
        const bool use_lds = any && (int64_t)Rw * Rh <= kLdsCapPx;
        if (use_lds) {
            // stage the box: row r of the box is Rw * RU4 contiguous uint4 in global memory
            const int rw4 = Rw * RU4;
            const int n4 = rw4 * Rh;
            const float inv = 1.0f / (float)rw4;
            const uint4* __restrict__ src0 = reinterpret_cast<const uint4*>(img) + ((int64_t)vmin * W + umin) * RU4;
            auto at = [&](int c) {  // box chunk c -> its global source
                int r = (int)((float)c * inv);
                r -= (r * rw4 > c);
                r += ((r + 1) * rw4 <= c);
                return src0 + ((int64_t)r * W * RU4 + (c - r * rw4));
            };
            const int last = n4 - 1;
            for (int c0 = threadIdx.x; c0 < n4; c0 += 4 * kLdsThreads) {
                // four independent loads in flight per lane (clamped indices: the tail re-reads
                // the box's last chunk and does not store it)
                const int c1 = c0 + kLdsThreads, c2 = c0 + 2 * kLdsThreads, c3 = c0 + 3 * kLdsThreads;
                const uint4 a0 = *at(c0);
                const uint4 a1 = *at(min(c1, last));
                const uint4 a2 = *at(min(c2, last));
                const uint4 a3 = *at(min(c3, last));
                tile[c0] = a0;
                if (c1 < n4) tile[c1] = a1;
                if (c2 < n4) tile[c2] = a2;
                if (c3 < n4) tile[c3] = a3;
            }
            __syncthreads();
        } else if (any) {
            n_global_levels++;
        }
        if (active && any && use_lds) {
            // candidates from the staged box (inside the image => inside the box); the rows of the
            // next window column are read from LDS while this column is scored (two register
            // buffers, the column loop fully unrolled so they alternate without copies)
            uint4 ra[SC][RU4], rb[SC][RU4];
            bool oka[SC], okb[SC];
            auto fetch = [&](int i, uint4 (&rw)[SC][RU4], bool (&okk)[SC]) {
                const int64_t u = u0 - rd + (int64_t)i * d;
#pragma unroll
                for (int j = 0; j < SC; j++) {
                    const int64_t v = v0 - rd + (int64_t)j * d;
                    okk[j] = inside_image(u, v, W, H);
                    const int off = okk[j] ? ((int)(v - vmin) * Rw + (int)(u - umin)) * RU4 : 0;
#pragma unroll
                    for (int c = 0; c < RU4; c++) rw[j][c] = tile[off + c];
                }
            };
            auto consume = [&](int i, const uint4 (&rw)[SC][RU4], const bool (&okk)[SC]) {
                half_t score[SC];
                score_f16_multi<F, SC>(q2, rw, score);
                const int64_t u = u0 - rd + (int64_t)i * d;
#pragma unroll
                for (int j = 0; j < SC; j++) {  // v offset inner (:55)
                    if (okk[j] && score[j] > max_score) {
                        max_score = score[j];
                        u_new = u;
                        v_new = v0 - rd + (int64_t)j * d;
                    }
                }
            };
            fetch(0, ra, oka);
#pragma nounroll
            for (int i = 0; i < SC; i += 2) {  // u offset outer (matching_kernels.cu:54)
                if (i + 1 < SC) fetch(i + 1, rb, okb);
                consume(i, ra, oka);
                if (i + 1 < SC) {
                    if (i + 2 < SC) fetch(i + 2, ra, oka);
                    consume(i + 1, rb, okb);
                }
            }
        } else if (active && any) {
            // the box does not fit the LDS budget: this level gathers from global memory
            for (int i = 0; i < SC; i++) {
                const int64_t u = u0 - rd + (int64_t)i * d;
                for (int j = 0; j < SC; j++) {
                    const int64_t v = v0 - rd + (int64_t)j * d;
                    if (inside_image(u, v, W, H)) {
                        uint4 row[RU4];
                        const uint4* src = reinterpret_cast<const uint4*>(img + (v * W + u) * F);
#pragma unroll
                        for (int c = 0; c < RU4; c++) row[c] = src[c];
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
        if (use_lds) __syncthreads();  // the next level's staging overwrites the tile
    }
    if (active) store_match(p1_new, lin, g, W, u_new, v_new);
    if (stats && threadIdx.x == 0 && n_global_levels)
        atomicAdd(stats, n_global_levels);  // diagnostics: levels that did not fit the LDS tile
}

// Generic F (any descriptor width), fp16, f32 or f64 (AT_DISPATCH_FLOATING_TYPES_AND_HALF,
// matching_kernels.cu:103), scalar loads.
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

static int refine_checks(const void* D11, const void* D21, const void* p1, void* out, int64_t B,
                         int64_t H, int64_t W, int64_t N, int64_t F, int radius,
                         int dilation_max) {
    M3S_REQUIRE(B >= 0 && N >= 0 && H >= 0 && W >= 0 && F >= 0, "refine_matches: negative sizes");
    M3S_REQUIRE(H * W < (int64_t)1 << 31, "refine_matches: image too large");
    M3S_REQUIRE(radius >= 0 && dilation_max >= 0, "refine_matches: negative radius/dilation");
    if (B * N > 0) M3S_REQUIRE(D11 && D21 && p1 && out, "refine_matches: null pointer");
    return M3S_OK;
}

// bound-and-rescore diagnostics (m3s_refine_mfma_stats; the MFMA and dot2 paths): exactly
// re-scored / in-image candidates
static bool g_refine_stats_enabled = false;
static unsigned long long g_refine_stats[2] = {0, 0};

extern "C" void m3s_refine_mfma_stats(int enable, unsigned long long* out2) {
    if (out2) {
        out2[0] = g_refine_stats[0];
        out2[1] = g_refine_stats[1];
    }
    g_refine_stats_enabled = enable != 0;
    g_refine_stats[0] = g_refine_stats[1] = 0;
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
    // M3S_REFINE_LDS=1 selects the LDS-tiled kernel (A/B; slower on the bench data, see above)
    const char* lds_env = getenv("M3S_REFINE_LDS");
    const bool lds_ok = lds_env && atoi(lds_env) != 0;
    const char* mf_env = getenv("M3S_REFINE_MFMA");
    const bool mfma_ok = mf_env && atoi(mf_env) != 0;
    // M3S_REFINE_DOT2=1: bound-and-rescore with dot2 approximations (measured slower than
    // scoring every candidate with the fp16 chain, the default: DESIGN.md §4)
    const char* d2_env = getenv("M3S_REFINE_DOT2");
    const bool dot2_ok = d2_env && atoi(d2_env) != 0;
    if (F == 24 && aligned && N == H * W && radius == 3 && (mfma_ok || dot2_ok)) {
        TileMap tm;
        tm.tiles_x = (int)((W + kTile - 1) / kTile);
        tm.tiles_y = (int)((H + kTile - 1) / kTile);
        tm.ntiles = tm.tiles_x * tm.tiles_y;
        const int64_t nblk = (int64_t)tm.ntiles * B;
        const int64_t grid = (nblk + 7) / 8 * 8;
        // per-image max ||h||^2 (+ the optional re-score counters), stream-ordered scratch
        unsigned* scratch = nullptr;
        const size_t sbytes = sizeof(unsigned) * (size_t)B + 2 * sizeof(unsigned long long) + 16;
        M3S_HIP_CHECK(hipMallocAsync((void**)&scratch, sbytes, st));
        M3S_HIP_CHECK(hipMemsetAsync(scratch, 0, sbytes, st));
        unsigned long long* stats = reinterpret_cast<unsigned long long*>(
            reinterpret_cast<char*>(scratch) + ((sizeof(unsigned) * (size_t)B + 15) / 16 * 16));
        unsigned long long* st_arg = g_refine_stats_enabled ? stats : nullptr;
        const int64_t HW = H * W;
        const unsigned hb = (unsigned)std::min<int64_t>((HW + kBlock - 1) / kBlock, 1024);
        hipLaunchKernelGGL(refine_hmax_kernel, dim3(hb, (unsigned)B), dim3(kBlock), 0, st, D11, HW, scratch);
        if (mfma_ok)
            hipLaunchKernelGGL((refine_mfma_kernel<3>), dim3((unsigned)grid), dim3(kBlock), 0, st, D11, D21, p1,
                               p1_new, lin, (int)H, (int)W, N, B, tm, dilation_max, scratch, st_arg);
        else
            hipLaunchKernelGGL((refine_dot2_kernel<3>), dim3((unsigned)grid), dim3(kBlock), 0, st, D11, D21, p1,
                               p1_new, lin, (int)H, (int)W, N, B, tm, dilation_max, scratch, st_arg);
        M3S_LAUNCH_CHECK();
        if (g_refine_stats_enabled) {
            unsigned long long h[2];
            M3S_HIP_CHECK(hipMemcpyAsync(h, stats, sizeof(h), hipMemcpyDeviceToHost, st));
            M3S_HIP_CHECK(hipStreamSynchronize(st));
            g_refine_stats[0] += h[0];
            g_refine_stats[1] += h[1];
        }
        M3S_HIP_CHECK(hipFreeAsync(scratch, st));
    } else if (F == 24 && aligned && N == H * W && radius == 3 && lds_ok) {
        LdsTileMap tm;
        tm.tiles_x = (int)((W + kLdsTx - 1) / kLdsTx);
        tm.tiles_y = (int)((H + kLdsTy - 1) / kLdsTy);
        tm.ntiles = tm.tiles_x * tm.tiles_y;
        const int64_t nblk = (int64_t)tm.ntiles * B;
        const int64_t grid = (nblk + 7) / 8 * 8;
        hipLaunchKernelGGL((refine_lds_kernel<24, 3>), dim3((unsigned)grid), dim3(kLdsThreads), 0, st, D11,
                           D21, p1, p1_new, lin, (int)H, (int)W, B, tm, dilation_max, (int*)nullptr);
    } else if (F == 24 && aligned && N == H * W) {
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
