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
    int64_t total, int max_iter, float lambda_init, float cost_thresh, int xcd_band, int skip_still) {
    // xcd_band: workgroups are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md, dispatch),
    // so block b runs on XCD b % 8; block b takes the logical block (b % 8) * per + b / 8 instead,
    // and each XCD walks ONE contiguous band of pixels -- its bilinear gathers stay in a band of
    // the ray image that its own L2 holds, instead of every XCD touching every row (speed only:
    // the mapping is a bijection whatever the placement)
    int64_t lb = blockIdx.x;
    if (xcd_band) {
        const int64_t per = (int64_t)gridDim.x / 8;  // gridDim.x is a multiple of 8 here
        lb = (int64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
    }
    const int64_t g = lb * kBlock + threadIdx.x;
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
    // The state at (u, v): residual e, cost, and the normal-equation terms without lambda.  A
    // rejected step leaves (u, v) and so all of it unchanged, and an accepted one moves to the
    // trial point whose ray channels, residual and cost were just evaluated (the same operations
    // on the same texels, so the same values) -- each iteration gathers the trial point's 3 ray
    // channels and, after an accepted step, its 6 gradient channels: 12 or 36 dwords per pixel
    // and iteration instead of the reference's 48, bitwise the same arithmetic.
    float e0 = 0.0f, e1 = 0.0f, e2 = 0.0f, cost = 0.0f;
    float A00b = 0.0f, A01 = 0.0f, A11b = 0.0f, b0 = 0.0f, b1 = 0.0f;
    auto normal_terms = [&](const Bilin& bb) {  // :202-210 from the gradients at bb and e
        const float gx0 = interp<CM>(bb, 3), gx1 = interp<CM>(bb, 4), gx2 = interp<CM>(bb, 5);
        const float gy0 = interp<CM>(bb, 6), gy1 = interp<CM>(bb, 7), gy2 = interp<CM>(bb, 8);
        A00b = cdot3<CM>(gx0, gx0, gx1, gx1, gx2, gx2);
        A01 = cdot3<CM>(gx0, gy0, gx1, gy1, gx2, gy2);
        A11b = cdot3<CM>(gy0, gy0, gy1, gy1, gy2, gy2);
        b0 = -cdot3<CM>(e0, gx0, e1, gx1, e2, gx2);
        b1 = -cdot3<CM>(e0, gy0, e1, gy1, e2, gy2);
    };
    if (max_iter > 0) {
        const Bilin bl = make_bilin(img, W, u, v);
        const float r0 = interp<CM>(bl, 0), r1 = interp<CM>(bl, 1), r2 = interp<CM>(bl, 2);
        // :186-198: r *= 1/|r| then err = r - pts (the scaled ray feeds only the subtraction: fused)
        const float r_norm_inv = inv_f(sqrtf(cdot3<CM>(r0, r0, r1, r1, r2, r2)));
        e0 = cmad<CM>(r0, r_norm_inv, -px);
        e1 = cmad<CM>(r1, r_norm_inv, -py);
        e2 = cmad<CM>(r2, r_norm_inv, -pz);
        cost = cdot3<CM>(e0, e0, e1, e1, e2, e2);
        normal_terms(bl);
    }
    for (int it = 0; it < max_iter; it++) {
        const float A00 = A00b + lambda, A11 = A11b + lambda;
        // :213-219: u + det_inv * (...) is a fused multiply-add under nvcc
        const float det_inv = inv_f(cmm<CM>(A00, A11, -A01, A01));
        const float u_new = clamp_ref(cmad<CM>(det_inv, cmm<CM>(A11, b0, -A01, b1), u), 1.0f, umax);
        const float v_new = clamp_ref(cmad<CM>(det_inv, cmm<CM>(-A01, b0, A00, b1), v), 1.0f, vmax);

        // :225-256 the cost at the new pixel (ray channels only).  A step that rounds to zero
        // (u_new == u and v_new == v: most pixels once converged, 43-88 % from the third
        // iteration on the bench pair) evaluates the SAME texels by the same operations, so its
        // cost is exactly the current one and the step is rejected: the gather is skipped and
        // only lambda and the flag move, bitwise as if it had been taken.
        bool accepted = false;
        if (!skip_still || u_new != u || v_new != v) {
            const Bilin bn = make_bilin(img, W, u_new, v_new);
            const float t0 = interp<CM>(bn, 0), t1 = interp<CM>(bn, 1), t2 = interp<CM>(bn, 2);
            const float n2_inv = inv_f(sqrtf(cdot3<CM>(t0, t0, t1, t1, t2, t2)));
            const float f0 = cmad<CM>(t0, n2_inv, -px), f1 = cmad<CM>(t1, n2_inv, -py),
                        f2 = cmad<CM>(t2, n2_inv, -pz);
            const float new_cost = cdot3<CM>(f0, f0, f1, f1, f2, f2);
            if (new_cost < cost) {
                accepted = true;
                u = u_new;
                v = v_new;
                lambda = (float)((double)lambda * 0.1);  // `lambda *= 0.1` is a double multiply
                conv = new_cost < cost_thresh;
                e0 = f0;
                e1 = f1;
                e2 = f2;
                cost = new_cost;
                if (it + 1 < max_iter) normal_terms(bn);
            }
        }
        if (!accepted) {
            lambda = (float)((double)lambda * 10.0);
            conv = cost < cost_thresh;
        }
    }
    *reinterpret_cast<float2*>(p_new + g * 2) = make_float2(u, v);
    converged[g] = conv;
}

#ifndef M3S_REFINE_WAVES
#define M3S_REFINE_WAVES 1
#endif
// Candidates J0 .. J0+NG-1 of one window column (v offsets inner, matching_kernels.cu:55): their
// rows loaded together, the score chains interleaved, then compared in candidate order.  (Scoring
// the column in groups of 1-3 candidates -- 7 instead of 3 waves per SIMD -- and a buffer-load
// form with 32-bit offsets measured no gain at B=8; both were removed.)
template <int F, int J0, int G, int SC>
__device__ __forceinline__ void refine_column(const half2_t (&q2)[F / 2], const uint16_t* __restrict__ img,
                                              int64_t u, int64_t vb, int d, int W, int H,
                                              half_t& max_score, int64_t& u_new, int64_t& v_new) {
    constexpr int NG = G < SC - J0 ? G : SC - J0;
    uint4 rows[NG][F / 8];
    bool ok[NG];
#pragma unroll
    for (int j = 0; j < NG; j++) {
        const int64_t v = vb + (int64_t)(J0 + j) * d;
        ok[j] = inside_image(u, v, W, H);
        const uint4* src = reinterpret_cast<const uint4*>(img + (ok[j] ? (v * W + u) * F : 0));
#pragma unroll
        for (int c = 0; c < F / 8; c++) rows[j][c] = src[c];
    }
    half_t score[NG];
    score_f16_multi<F, NG>(q2, rows, score);
#pragma unroll
    for (int j = 0; j < NG; j++) {
        if (ok[j] && score[j] > max_score) {
            max_score = score[j];
            u_new = u;
            v_new = vb + (int64_t)(J0 + j) * d;
        }
    }
    if constexpr (J0 + NG < SC) refine_column<F, J0 + NG, G, SC>(q2, img, u, vb, d, W, H, max_score, u_new, v_new);
}

template <int F, int R>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(M3S_REFINE_WAVES))) void refine_f16_kernel(
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
                refine_column<F, 0, 2 * R + 1, 2 * R + 1>(q2, img, u, v0 - rd, d, W, H, max_score, u_new,
                                                                 v_new);
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
    // M3S_IP_XCD (default 1): the XCD-banded block order above; 0: blocks in pixel order
    static const int xcd_band = [] {
        const char* e = getenv("M3S_IP_XCD");
        return e ? atoi(e) : 1;
    }();
    // M3S_IP_SKIP: 1 = a zero step skips its trial gather (bitwise the same either way), 0 =
    // always gathers, default: skip on launches of >= 2^19 pixels.  Measured (profiles/r05_s_ip_skip/):
    // 8 pairs of 384x512 0.181 -> 0.171 ms (the gathers are L1/TA-bound there and 43-88 % of the
    // steps from the third iteration on round to zero), one pair 0.046 -> 0.049 ms (3 waves per
    // SIMD: latency-bound, and the divergent branch only costs)
    static const int skip_env = [] {
        const char* e = getenv("M3S_IP_SKIP");
        return e ? atoi(e) : -1;
    }();
    const int skip_still = skip_env >= 0 ? skip_env : (total >= ((int64_t)1 << 19) ? 1 : 0);
    const int64_t nblk = (total + kBlock - 1) / kBlock;
    const unsigned ip_grid = (unsigned)(xcd_band ? (nblk + 7) / 8 * 8 : nblk);
#define M3S_IP(CM)                                                                                      \
    hipLaunchKernelGGL(iter_proj_kernel<CM>, dim3(ip_grid), dim3(kBlock), 0, (hipStream_t)stream,       \
                       rays, pts, p_init, p_new, converged, (int)H, (int)W, N, total, max_iter,            \
                       lambda_init, cost_thresh, xcd_band, skip_still)
    if (contract == M3S_CONTRACT_OFF) M3S_IP(M3S_CONTRACT_OFF);
    else if (contract == M3S_CONTRACT_NVCC) M3S_IP(M3S_CONTRACT_NVCC);
    else M3S_IP(M3S_CONTRACT_NVCC_RIGHT);
#undef M3S_IP
    M3S_LAUNCH_CHECK();
    return M3S_OK;
}

namespace m3s {
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

// the fused matching op's refine (match_glue.hip): D11's fp16 copy is already plane-major
// (refine_planes_kernel, refine_common.h); F = 24, radius 3, N = H * W
int refine_planes_launch(const void* D11_planes, const uint16_t* D21, const int64_t* p1, int64_t* lin, int64_t B,
                         int64_t H, int64_t W, int dilation_max, hipStream_t st) {
    const int64_t N = H * W;
    if (B * N == 0) return M3S_OK;
    TileMap tm;
    tm.tiles_x = (int)((W + kTile - 1) / kTile);
    tm.tiles_y = (int)((H + kTile - 1) / kTile);
    tm.ntiles = tm.tiles_x * tm.tiles_y;
    const int64_t nblk = (int64_t)tm.ntiles * B;
    const int64_t grid = (nblk + 7) / 8 * 8;
    hipLaunchKernelGGL((refine_planes_kernel<3>), dim3((unsigned)grid), dim3(kBlock), 0, st,
                       static_cast<const uint4*>(D11_planes), D21, p1, (int64_t*)nullptr, lin, (int)H, (int)W, N, B,
                       tm, dilation_max);
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
