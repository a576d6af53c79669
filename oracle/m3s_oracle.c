/*
 * m3s_oracle.c -- CPU restatement of the MASt3R-SLAM backend hot path.
 *
 * TEST INFRASTRUCTURE ONLY (parity checker + timed CPU baseline); see
 * m3s_oracle.h for the parity status and the numerics convention.
 * Built by oracle/Makefile with -ffp-contract=off.
 *
 * Every function cites the reference lines it restates
 * (/root/reference/mast3r_slam/backend/src/...).
 */
#include "m3s_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define EPS 1e-6 /* gn_kernels.cu:34 (a double literal) */

int oracle_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

void oracle_set_num_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

/* ------------------------------------------------------------------------ */
/* fp16 (c10::Half) helpers                                                 */
/* ------------------------------------------------------------------------ */

float oracle_f16_to_f32(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t ex = (h >> 10) & 0x1fu;
    uint32_t man = h & 0x3ffu;
    uint32_t bits;
    if (ex == 0x1f) {
        bits = sign | 0x7f800000u | (man << 13);
    } else if (ex == 0) {
        /* zero or subnormal: value = man * 2^-24, exact in float */
        float v = (float)man * 5.9604644775390625e-8f;
        memcpy(&bits, &v, 4);
        bits |= sign;
    } else {
        bits = sign | ((ex + 112u) << 23) | (man << 13);
    }
    float f;
    memcpy(&f, &bits, 4);
    return f;
}

uint16_t oracle_f32_to_f16(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    uint16_t sign = (uint16_t)((x >> 16) & 0x8000u);
    uint32_t ax = x & 0x7fffffffu;
    if (ax >= 0x7f800000u) { /* inf / nan */
        if (ax == 0x7f800000u) return sign | 0x7c00u;
        return sign | 0x7e00u | (uint16_t)((ax >> 13) & 0x3ffu);
    }
    if (ax >= 0x477ff000u) return sign | 0x7c00u; /* >= 65520 rounds to inf */
    if (ax < 0x38800000u) {                       /* below 2^-14: subnormal half */
        float a;
        memcpy(&a, &ax, 4);
        float m = nearbyintf(a * 16777216.0f); /* exact scaling, RNE */
        return sign | (uint16_t)m;
    }
    uint32_t man = ax & 0x7fffffu;
    uint32_t ex = (ax >> 23) - 112u;
    uint32_t h = (ex << 10) | (man >> 13);
    uint32_t rem = man & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
    return sign | (uint16_t)h;
}

/* c10::Half a*b and a+b: compute in float, round to half (exact products). */
static inline uint16_t hmul(uint16_t a, uint16_t b) {
    return oracle_f32_to_f16(oracle_f16_to_f32(a) * oracle_f16_to_f32(b));
}
static inline uint16_t hadd(uint16_t a, uint16_t b) {
    return oracle_f32_to_f16(oracle_f16_to_f32(a) + oracle_f16_to_f32(b));
}

/* ------------------------------------------------------------------------ */
/* FMA contraction convention of the reference build                        */
/* ------------------------------------------------------------------------ */
/* The reference is compiled by nvcc -O3 (setup.py:29-37, so --fmad=true): a multiply feeding an
 * add is fused into one fma; of `a*b + c*d` the LEFT product is fused (ORACLE_CONTRACT_NVCC,
 * LLVM / NVPTX combine order), ORACLE_CONTRACT_NVCC_RIGHT fuses the right one, ORACLE_CONTRACT_OFF
 * is multiply-then-add.  This file is compiled with -ffp-contract=off: these helpers are the only
 * fused operations.  (The same helpers as mast3r-slam_amd/csrc/contract.h, restated in C.) */
static int g_contract = ORACLE_CONTRACT_NVCC; /* the GN restatement's convention */
void oracle_set_contract(int cm) { g_contract = cm; }
int oracle_get_contract(void) { return g_contract; }

static inline float cmad(int cm, float a, float b, float c) { /* a*b + c */
    return cm != ORACLE_CONTRACT_OFF ? fmaf(a, b, c) : a * b + c;
}
static inline float cmm(int cm, float a, float b, float c, float d) { /* a*b + c*d */
    if (cm == ORACLE_CONTRACT_OFF) return a * b + c * d;
    if (cm == ORACLE_CONTRACT_NVCC) return fmaf(a, b, c * d);
    return fmaf(c, d, a * b);
}
static inline float cdot3(int cm, float a0, float b0, float a1, float b1, float a2, float b2) {
    return cmad(cm, a2, b2, cmm(cm, a0, b0, a1, b1)); /* (a0 b0 + a1 b1) + a2 b2 */
}

/* ------------------------------------------------------------------------ */
/* iter_proj  (matching_kernels.cu:119-275)                                 */
/* ------------------------------------------------------------------------ */

/* matching_kernels.cu:21-23 */
static inline float clampf_ref(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }

/* matching_kernels.cu:155-183 (bilinear interpolation of C channels) */
static inline void bilinear(int cm, const float* img, int64_t W, float u, float v, int C, float* out) {
    int u11 = (int)floorf(u);
    int v11 = (int)floorf(v);
    float du = u - (float)u11;
    float dv = v - (float)v11;
    /* double literal 1.0 promotes these three weights (matching_kernels.cu:161-164) */
    float w11 = du * dv;
    float w12 = (float)((1.0 - (double)du) * (double)dv);
    float w21 = (float)((double)du * (1.0 - (double)dv));
    float w22 = (float)((1.0 - (double)du) * (1.0 - (double)dv));
    /* "Pixels are opposite the area calc" (matching_kernels.cu:166-170) */
    const float* r11 = img + ((int64_t)(v11 + 1) * W + (u11 + 1)) * 9;
    const float* r12 = img + ((int64_t)(v11 + 1) * W + u11) * 9;
    const float* r21 = img + ((int64_t)v11 * W + (u11 + 1)) * 9;
    const float* r22 = img + ((int64_t)v11 * W + u11) * 9;
    /* ((w11 r11 + w12 r12) + w21 r21) + w22 r22 */
    for (int j = 0; j < C; j++)
        out[j] = cmad(cm, w22, r22[j], cmad(cm, w21, r21[j], cmm(cm, w11, r11[j], w12, r12[j])));
}

void oracle_iter_proj(const float* rays, const float* pts, const float* p_init,
                      float* p_new, uint8_t* converged,
                      int64_t B, int64_t H, int64_t W, int64_t N,
                      int max_iter, float lambda_init, float cost_thresh, int cm) {
    const int64_t total = B * N;
#pragma omp parallel for schedule(static)
    for (int64_t g = 0; g < total; g++) {
        const int64_t b = g / N;
        const float* img = rays + b * H * W * 9;
        float u = p_init[g * 2 + 0];
        float v = p_init[g * 2 + 1];
        u = clampf_ref(u, 1.0f, (float)(W - 2)); /* :143-144 */
        v = clampf_ref(v, 1.0f, (float)(H - 2));
        const float px = pts[g * 3 + 0], py = pts[g * 3 + 1], pz = pts[g * 3 + 2];
        float lambda = lambda_init;
        uint8_t conv = 0; /* torch::zeros init (:300-301) */
        for (int i = 0; i < max_iter; i++) {
            float s[9];
            bilinear(cm, img, W, u, v, 9, s);
            const float r0 = s[0], r1 = s[1], r2 = s[2];
            const float gx0 = s[3], gx1 = s[4], gx2 = s[5];
            const float gy0 = s[6], gy1 = s[7], gy2 = s[8];
            /* :186-198 normalise, error (r *= inv; err = r - pts: the product feeds the
             * subtraction, fused under nvcc), cost */
            const float r_norm = sqrtf(cdot3(cm, r0, r0, r1, r1, r2, r2));
            const float r_norm_inv = (float)(1.0 / (double)r_norm);
            const float e0 = cmad(cm, r0, r_norm_inv, -px);
            const float e1 = cmad(cm, r1, r_norm_inv, -py);
            const float e2 = cmad(cm, r2, r_norm_inv, -pz);
            const float cost = cdot3(cm, e0, e0, e1, e1, e2, e2);
            /* :202-210 normal equations */
            float A00 = cdot3(cm, gx0, gx0, gx1, gx1, gx2, gx2);
            const float A01 = cdot3(cm, gx0, gy0, gx1, gy1, gx2, gy2);
            float A11 = cdot3(cm, gy0, gy0, gy1, gy1, gy2, gy2);
            const float b0 = -cdot3(cm, e0, gx0, e1, gx1, e2, gx2);
            const float b1 = -cdot3(cm, e0, gy0, e1, gy1, e2, gy2);
            A00 += lambda;
            A11 += lambda;
            /* :213-221  u + det_inv * (...) fused under nvcc */
            const float det_inv = (float)(1.0 / (double)cmm(cm, A00, A11, -A01, A01));
            const float u_new = clampf_ref(cmad(cm, det_inv, cmm(cm, A11, b0, -A01, b1), u), 1.0f, (float)(W - 2));
            const float v_new = clampf_ref(cmad(cm, det_inv, cmm(cm, -A01, b0, A00, b1), v), 1.0f, (float)(H - 2));
            /* :225-256 cost at the new pixel (ray channels only) */
            float t[3];
            bilinear(cm, img, W, u_new, v_new, 3, t);
            const float n2 = sqrtf(cdot3(cm, t[0], t[0], t[1], t[1], t[2], t[2]));
            const float n2_inv = (float)(1.0 / (double)n2);
            const float f0 = cmad(cm, t[0], n2_inv, -px);
            const float f1 = cmad(cm, t[1], n2_inv, -py);
            const float f2 = cmad(cm, t[2], n2_inv, -pz);
            const float new_cost = cdot3(cm, f0, f0, f1, f1, f2, f2);
            /* :259-268  lambda *= 0.1 is a DOUBLE multiply (0.1 != 0.1f) */
            if (new_cost < cost) {
                u = u_new;
                v = v_new;
                lambda = (float)((double)lambda * 0.1);
                conv = new_cost < cost_thresh;
            } else {
                lambda = (float)((double)lambda * 10.0);
                conv = cost < cost_thresh;
            }
        }
        p_new[g * 2 + 0] = u;
        p_new[g * 2 + 1] = v;
        converged[g] = conv;
    }
}

/* ------------------------------------------------------------------------ */
/* refine_matches  (matching_kernels.cu:25-81)                              */
/* ------------------------------------------------------------------------ */

/* The reference initialises max_score with cuda::std::numeric_limits<c10::Half>::min();
 * libcu++ has no specialisation for c10::Half, so that is a value-initialised Half:
 * 0.0 (SURVEY.md §7.3 hard part 1).  Only strictly positive scores can move a match. */
#define REFINE_MAX_SCORE_INIT 0.0f

/* ---------------- matching glue (reference matching.py:25-90, image.py:5-38) ----------------
 * The reference's Python glue with the float arithmetic torch uses on the host (pinned by the
 * reference-generated tests/golden/glue_golden.npz):
 *   F.normalize / linalg.norm: sqrt(fma(x2, x2, fma(x1, x1, x0 * x0))), x / max(n, 1e-12)
 *   img_gradient: reflect pad 1, depthwise 3x3 conv as acc = fma(w, x, acc) over the taps in
 *   row-major order from 0, w = (1/32) * [[-3,0,3],[-10,0,10],[-3,0,3]] and its transpose.   */
static inline void normalize3_ref(const float* x, float* y) {
    const float n = fmaxf(sqrtf(fmaf(x[2], x[2], fmaf(x[1], x[1], x[0] * x[0]))), 1e-12f);
    y[0] = x[0] / n;
    y[1] = x[1] / n;
    y[2] = x[2] / n;
}

static inline int64_t reflect1_ref(int64_t i, int64_t n) { return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i); }

void oracle_match_prep(const float* X11, const float* X21, const int64_t* idx_init, int64_t B, int64_t H,
                       int64_t W, float* rays9, float* pts, float* p_init) {
    static const float wx[9] = {-3.0f / 32, 0.0f, 3.0f / 32, -10.0f / 32, 0.0f, 10.0f / 32, -3.0f / 32, 0.0f, 3.0f / 32};
    static const float wy[9] = {-3.0f / 32, -10.0f / 32, -3.0f / 32, 0.0f, 0.0f, 0.0f, 3.0f / 32, 10.0f / 32, 3.0f / 32};
    const int64_t HW = H * W;
#pragma omp parallel for schedule(static)
    for (int64_t n = 0; n < B * HW; n++) {
        const int64_t b = n / HW, k = n % HW, y = k / W, x = k % W;
        float r[9][3];
        for (int t = 0; t < 9; t++) {
            const int64_t yy = reflect1_ref(y + t / 3 - 1, H), xx = reflect1_ref(x + t % 3 - 1, W);
            normalize3_ref(X11 + ((b * HW) + yy * W + xx) * 3, r[t]);
        }
        float* o = rays9 + n * 9;
        for (int c = 0; c < 3; c++) {
            float gx = 0.0f, gy = 0.0f;
            for (int t = 0; t < 9; t++) {
                gx = fmaf(wx[t], r[t][c], gx);
                gy = fmaf(wy[t], r[t][c], gy);
            }
            o[c] = r[4][c];
            o[3 + c] = gx;
            o[6 + c] = gy;
        }
        normalize3_ref(X21 + n * 3, pts + n * 3);
        int64_t u = x, v = y;
        if (idx_init) { /* lin_to_pixel (matching.py:18-22): Python floor // and % */
            const int64_t id = idx_init[n];
            v = id / W;
            u = id - v * W;
            if (u < 0) {
                u += W;
                v -= 1;
            }
        }
        p_init[n * 2] = (float)u;
        p_init[n * 2 + 1] = (float)v;
    }
}

/* p.long(), occlusion test ||X11[p1] - X21|| < dist_thresh, valid = converged & that
 * (matching.py:66-76) */
void oracle_match_post(const float* X11, const float* X21, const float* p_new, const uint8_t* conv,
                       int64_t B, int64_t H, int64_t W, float dist_thresh, int64_t* p1, uint8_t* valid) {
    const int64_t HW = H * W;
    for (int64_t n = 0; n < B * HW; n++) {
        const int64_t b = n / HW;
        const int64_t u = (int64_t)p_new[n * 2], v = (int64_t)p_new[n * 2 + 1];
        const float* a = X11 + (b * HW + v * W + u) * 3;
        const float* q = X21 + n * 3;
        const float d0 = a[0] - q[0], d1 = a[1] - q[1], d2 = a[2] - q[2];
        const float dist = sqrtf(fmaf(d2, d2, fmaf(d1, d1, d0 * d0)));
        valid[n] = conv[n] && dist < dist_thresh;
        p1[n * 2] = u;
        p1[n * 2 + 1] = v;
    }
}

static inline int inside_image(int64_t u, int64_t v, int64_t W, int64_t H) {
    return v >= 0 && v < H && u >= 0 && u < W; /* matching_kernels.cu:17-19 */
}

void oracle_refine_matches_f16(const uint16_t* D11, const uint16_t* D21,
                               const int64_t* p1, int64_t* p1_new,
                               int64_t B, int64_t H, int64_t W, int64_t N,
                               int64_t F, int radius, int dilation_max) {
    const int64_t total = B * N;
#pragma omp parallel for schedule(dynamic, 256)
    for (int64_t g = 0; g < total; g++) {
        const int64_t b = g / N;
        const uint16_t* d21 = D21 + g * F;
        int64_t u0 = p1[g * 2 + 0];
        int64_t v0 = p1[g * 2 + 1];
        uint16_t max_score = oracle_f32_to_f16(REFINE_MAX_SCORE_INIT);
        int64_t u_new = u0, v_new = v0;
        for (int d = dilation_max; d > 0; d--) {
            const int rd = radius * d;
            const int diam = 2 * rd + 1;
            for (int i = 0; i < diam; i += d) {     /* u offset outer */
                for (int j = 0; j < diam; j += d) { /* v offset inner */
                    const int64_t u = u0 - rd + i;
                    const int64_t v = v0 - rd + j;
                    if (inside_image(u, v, W, H)) {
                        const uint16_t* d11 = D11 + ((b * H + v) * W + u) * F;
                        uint16_t score = 0; /* scalar_t score = 0.0 */
                        for (int64_t k = 0; k < F; k++) score = hadd(score, hmul(d21[k], d11[k]));
                        if (oracle_f16_to_f32(score) > oracle_f16_to_f32(max_score)) {
                            max_score = score;
                            u_new = u;
                            v_new = v;
                        }
                    }
                }
            }
            u0 = u_new; /* :75-76 the window re-centres on the winner */
            v0 = v_new;
        }
        p1_new[g * 2 + 0] = u_new;
        p1_new[g * 2 + 1] = v_new;
    }
}

/* refine_matches_kernel<float> / <double>: the same loop in the accumulator type T, with
 * max_score starting at numeric_limits<T>::min() (specialised for float and double: FLT_MIN,
 * DBL_MIN).  matching_kernels.cu:25-81, dispatched by AT_DISPATCH_FLOATING_TYPES_AND_HALF
 * (:103).  `score += D21 * D11` is one fused multiply-add per term in the nvcc build
 * (ORACLE_CONTRACT_NVCC; c10::Half's operator* rounds first, so the fp16 path has no fusion). */
#define ORACLE_REFINE_REAL(NAME, T, MIN_INIT, FMA)                                          \
    void NAME(const T* D11, const T* D21, const int64_t* p1, int64_t* p1_new, int64_t B,     \
              int64_t H, int64_t W, int64_t N, int64_t F, int radius, int dilation_max) {     \
        const int64_t total = B * N;                                                          \
        _Pragma("omp parallel for schedule(dynamic, 256)")                                   \
        for (int64_t g = 0; g < total; g++) {                                                 \
            const int64_t b = g / N;                                                          \
            const T* d21 = D21 + g * F;                                                       \
            int64_t u0 = p1[g * 2 + 0];                                                       \
            int64_t v0 = p1[g * 2 + 1];                                                       \
            T max_score = MIN_INIT;                                                           \
            int64_t u_new = u0, v_new = v0;                                                   \
            for (int d = dilation_max; d > 0; d--) {                                          \
                const int rd = radius * d;                                                    \
                const int diam = 2 * rd + 1;                                                  \
                for (int i = 0; i < diam; i += d) {                                           \
                    for (int j = 0; j < diam; j += d) {                                       \
                        const int64_t u = u0 - rd + i;                                        \
                        const int64_t v = v0 - rd + j;                                        \
                        if (inside_image(u, v, W, H)) {                                       \
                            const T* d11 = D11 + ((b * H + v) * W + u) * F;                   \
                            T score = 0;                                                      \
                            for (int64_t k = 0; k < F; k++) score = FMA(d21[k], d11[k], score); \
                            if (score > max_score) {                                          \
                                max_score = score;                                            \
                                u_new = u;                                                    \
                                v_new = v;                                                    \
                            }                                                                 \
                        }                                                                     \
                    }                                                                         \
                }                                                                             \
                u0 = u_new;                                                                   \
                v0 = v_new;                                                                   \
            }                                                                                 \
            p1_new[g * 2 + 0] = u_new;                                                        \
            p1_new[g * 2 + 1] = v_new;                                                        \
        }                                                                                     \
    }

ORACLE_REFINE_REAL(oracle_refine_matches_f32, float, 1.17549435e-38f, fmaf)
ORACLE_REFINE_REAL(oracle_refine_matches_f64, double, 2.2250738585072014e-308, fma)

/* ------------------------------------------------------------------------ */
/* Sim3 device library (gn_kernels.cu:172-413), restated in float           */
/* ------------------------------------------------------------------------ */

/* gn_kernels.cu:172-175 (double literal 1.345) */
static inline float huber(float r) {
    const float r_abs = fabsf(r);
    return (double)r_abs < 1.345 ? 1.0f : (float)(1.345 / (double)r_abs);
}

/* Below, every function follows the GN restatement's contraction convention g_contract
 * (oracle_set_contract; default ORACLE_CONTRACT_NVCC, the reference build's): CM is it. */
#define CM g_contract

/* :178-184  qi * qj, quaternion [x,y,z,w]; each component a left-to-right sum of 4 products */
static inline void quat_comp(const float* qi, const float* qj, float* out) {
    float o0 = cmad(CM, -qi[2], qj[1], cmad(CM, qi[1], qj[2], cmm(CM, qi[3], qj[0], qi[0], qj[3])));
    float o1 = cmad(CM, qi[2], qj[0], cmad(CM, qi[1], qj[3], cmm(CM, qi[3], qj[1], -qi[0], qj[2])));
    float o2 = cmad(CM, qi[2], qj[3], cmad(CM, -qi[1], qj[0], cmm(CM, qi[3], qj[2], qi[0], qj[1])));
    float o3 = cmad(CM, -qi[2], qj[2], cmad(CM, -qi[1], qj[1], cmm(CM, qi[3], qj[3], -qi[0], qj[0])));
    out[0] = o0; out[1] = o1; out[2] = o2; out[3] = o3;
}

static inline void quat_inv(const float* q, float* out) { /* :187-193 */
    out[0] = -q[0]; out[1] = -q[1]; out[2] = -q[2]; out[3] = q[3];
}

/* :195-205; safe for X == Y (each Y[k] reads only X[k] and uv).  uv = 2.0 * (...) is a double
 * multiply of a float: exactly 2x. */
static inline void actSO3(const float* q, const float* X, float* Y) {
    float uv0 = (float)(2.0 * (double)cmm(CM, q[1], X[2], -q[2], X[1]));
    float uv1 = (float)(2.0 * (double)cmm(CM, q[2], X[0], -q[0], X[2]));
    float uv2 = (float)(2.0 * (double)cmm(CM, q[0], X[1], -q[1], X[0]));
    float y0 = cmad(CM, q[3], uv0, X[0]) + cmm(CM, q[1], uv2, -q[2], uv1);
    float y1 = cmad(CM, q[3], uv1, X[1]) + cmm(CM, q[2], uv0, -q[0], uv2);
    float y2 = cmad(CM, q[3], uv2, X[2]) + cmm(CM, q[0], uv1, -q[1], uv0);
    Y[0] = y0; Y[1] = y1; Y[2] = y2;
}

/* :207-219: Y = s (R X) + t -- the scale product feeds the translation add (fused) */
static inline void actSim3(const float* t, const float* q, const float* s, const float* X, float* Y) {
    float r[3];
    actSO3(q, X, r);
    Y[0] = cmad(CM, r[0], s[0], t[0]);
    Y[1] = cmad(CM, r[1], s[0], t[1]);
    Y[2] = cmad(CM, r[2], s[0], t[2]);
}

/* :229-240 b <- a x b */
static inline void crossInplace(const float* a, float* b) {
    float x0 = cmm(CM, a[1], b[2], -a[2], b[1]);
    float x1 = cmm(CM, a[2], b[0], -a[0], b[2]);
    float x2 = cmm(CM, a[0], b[1], -a[1], b[0]);
    b[0] = x0; b[1] = x1; b[2] = x2;
}

static inline float dot3(const float* t, const float* s) { return cdot3(CM, t[0], s[0], t[1], s[1], t[2], s[2]); }
static inline float squared_norm3(const float* v) { return cdot3(CM, v[0], v[0], v[1], v[1], v[2], v[2]); }

/* :252-272  T_ij = T_i^{-1} T_j */
static void relSim3(const float* ti, const float* qi, const float* si,
                    const float* tj, const float* qj, const float* sj,
                    float* tij, float* qij, float* sij) {
    float si_inv = (float)(1.0 / (double)si[0]);
    sij[0] = si_inv * sj[0];
    float qi_inv[4];
    quat_inv(qi, qi_inv);
    quat_comp(qi_inv, qj, qij);
    tij[0] = tj[0] - ti[0];
    tij[1] = tj[1] - ti[1];
    tij[2] = tj[2] - ti[2];
    actSO3(qi_inv, tij, tij);
    tij[0] *= si_inv; tij[1] *= si_inv; tij[2] *= si_inv;
}

/* :277-297  Y = X * Adj(T)^{-1} for a row vector X (tangent order tau, phi, sigma);
 * Y[3..5] += s_inv * (...) and Y[6] = X[6] + s_inv * dot are fused multiply-adds */
void oracle_apply_sim3_adj_inv(const float* t, const float* q, const float* s, const float* X, float* Y) {
    const float s_inv = (float)(1.0 / (double)s[0]);
    float Ra[3];
    actSO3(q, &X[0], Ra);
    Y[0] = s_inv * Ra[0];
    Y[1] = s_inv * Ra[1];
    Y[2] = s_inv * Ra[2];
    actSO3(q, &X[3], &Y[3]);
    Y[3] = cmad(CM, s_inv, cmm(CM, t[1], Ra[2], -t[2], Ra[1]), Y[3]);
    Y[4] = cmad(CM, s_inv, cmm(CM, t[2], Ra[0], -t[0], Ra[2]), Y[4]);
    Y[5] = cmad(CM, s_inv, cmm(CM, t[0], Ra[1], -t[1], Ra[0]), Y[5]);
    Y[6] = cmad(CM, s_inv, dot3(t, Ra), X[6]);
}

/* double a*b + c, fused under every contracting convention */
static inline double cmad_d(int cm, double a, double b, double c) { return cm != ORACLE_CONTRACT_OFF ? fma(a, b, c) : a * b + c; }

/* The Sim(3) exponential's float transcendentals correctly rounded (double, rounded once), as
 * the op evaluates them (mast3r-slam_amd/csrc/sim3.h): the reference's CUDA expf / sinf / cosf
 * (<= 2 ulp) are not reproducible off its platform, and its float formulas amplify one ulp
 * ~1/sigma-fold ((expf(sigma) - 1) / sigma), so both sides use the correctly rounded value. */
static inline float expf_cr(float x) { return (float)exp((double)x); }
static inline float sinf_cr(float x) { return (float)sin((double)x); }
static inline float cosf_cr(float x) { return (float)cos((double)x); }

/* :299-321 (the small-angle series is double arithmetic) */
static void expSO3(const float* phi, float* q) {
    float theta_sq = squared_norm3(phi);
    float imag, real;
    if ((double)theta_sq < EPS) {
        float theta_p4 = theta_sq * theta_sq;
        imag = (float)cmad_d(CM, 1.0 / 3840.0, (double)theta_p4, cmad_d(CM, -(1.0 / 48.0), (double)theta_sq, 0.5));
        real = (float)cmad_d(CM, 1.0 / 384.0, (double)theta_p4, cmad_d(CM, -(1.0 / 8.0), (double)theta_sq, 1.0));
    } else {
        float theta = sqrtf(theta_sq);
        imag = sinf_cr((float)(0.5 * (double)theta)) / theta;
        real = cosf_cr((float)(0.5 * (double)theta));
    }
    q[0] = imag * phi[0];
    q[1] = imag * phi[1];
    q[2] = imag * phi[2];
    q[3] = real;
}

/* :323-390 (including the as-written "B = (C - ...)" at :371) */
void oracle_exp_sim3(const float* xi, float* t, float* q, float* s) {
    float tau[3] = {xi[0], xi[1], xi[2]};
    float phi[3] = {xi[3], xi[4], xi[5]};
    float sigma = xi[6];
    float scale = expf_cr(sigma);
    expSO3(phi, q);
    s[0] = scale;
    float theta_sq = squared_norm3(phi);
    float theta = sqrtf(theta_sq);
    float A, B, C;
    const float one = 1.0f;
    const float half = 0.5f;
    if ((double)fabsf(sigma) < EPS) {
        C = one;
        if ((double)fabsf(theta) < EPS) {
            A = half;
            B = (float)(1.0 / 6.0);
        } else {
            A = (one - cosf_cr(theta)) / theta_sq;
            B = (theta - sinf_cr(theta)) / (theta_sq * theta);
        }
    } else {
        C = (scale - one) / sigma;
        if ((double)fabsf(theta) < EPS) {
            float sigma_sq = sigma * sigma;
            A = cmad(CM, sigma - one, scale, one) / sigma_sq;
            B = cmad(CM, -sigma, scale, cmad(CM, scale * half, sigma_sq, scale) - one) / (sigma_sq * sigma);
        } else {
            float a = scale * sinf_cr(theta);
            float b = scale * cosf_cr(theta);
            float c = cmad(CM, sigma, sigma, theta_sq);
            A = cmm(CM, a, sigma, one - b, theta) / (theta * c);
            B = (C - cmm(CM, b - one, sigma, a, theta) / (c)) / (theta_sq);
        }
    }
    /* t = C tau; t += A tau'; t += B tau'' -- the first two products are one two-product sum,
     * the third is fused into the running sum */
    const float tau0[3] = {tau[0], tau[1], tau[2]};
    crossInplace(phi, tau);
    t[0] = cmm(CM, C, tau0[0], A, tau[0]);
    t[1] = cmm(CM, C, tau0[1], A, tau[1]);
    t[2] = cmm(CM, C, tau0[2], A, tau[2]);
    crossInplace(phi, tau);
    t[0] = cmad(CM, B, tau[0], t[0]);
    t[1] = cmad(CM, B, tau[1], t[1]);
    t[2] = cmad(CM, B, tau[2], t[2]);
}

/* :392-413 left-composition retraction */
void oracle_retr_sim3(const float* xi, const float* t, const float* q, const float* s,
                      float* t1, float* q1, float* s1) {
    float dt[3] = {0, 0, 0};
    float dq[4] = {0, 0, 0, 1};
    float ds[1] = {0};
    oracle_exp_sim3(xi, dt, dq, ds);
    quat_comp(dq, q, q1);
    actSO3(dq, t, t1);
    t1[0] = cmad(CM, t1[0], ds[0], dt[0]);
    t1[1] = cmad(CM, t1[1], ds[0], dt[1]);
    t1[2] = cmad(CM, t1[2], ds[0], dt[2]);
    s1[0] = ds[0] * s[0];
}

/* :415-453 */
void oracle_pose_retr(float* Twc, const float* dx, int64_t N, int num_fix) {
    for (int64_t k = num_fix; k < N; k++) {
        float* p = Twc + k * 8;
        float t[3] = {p[0], p[1], p[2]};
        float q[4] = {p[3], p[4], p[5], p[6]};
        float s[1] = {p[7]};
        float xi[7];
        for (int n = 0; n < 7; n++) xi[n] = dx[(k - num_fix) * 7 + n];
        float t1[3], q1[4], s1[1];
        oracle_retr_sim3(xi, t, q, s, t1, q1, s1);
        p[0] = t1[0]; p[1] = t1[1]; p[2] = t1[2];
        p[3] = q1[0]; p[4] = q1[1]; p[5] = q1[2]; p[6] = q1[3];
        p[7] = s1[0];
    }
}

/* ------------------------------------------------------------------------ */
/* Alignment kernels (gn_kernels.cu:455-723, 813-1138, 1231-1543)           */
/* ------------------------------------------------------------------------ */

#define THREADS 256
#define HDIM 105 /* 14*15/2 */
#define NACC (HDIM + 14)

/* Summation mode.  0 (default): every accumulation is the reference's float addition, in
 * its order (values are stored in double but are always float-representable, and a float
 * sum computed in double then rounded to float is the correctly rounded float sum).
 * 1 ("exact sums", a precision reference for the tests / bench accuracy check, not the
 * reference's arithmetic): the same float terms summed in double. */
static int g_exact_sums = 0;
void oracle_set_exact_sums(int on) { g_exact_sums = on != 0; }

/* acc += x * y: the reference's `hij[l] += w * Jx[n] * Jx[m]` / `vi[n] += w * err * Ji[n]` with
 * x the rounded first product -- one fused multiply-add per term under nvcc (g_contract), or
 * (exact sums) the exact product added in double */
static inline double add_prod(double a, float x, float y) {
    if (g_exact_sums) return a + (double)x * (double)y;
    if (g_contract != ORACLE_CONTRACT_OFF) return (double)fmaf(x, y, (float)a);
    return (double)((float)a + x * y);
}
static inline double add_acc(double a, double b) {
    return g_exact_sums ? a + b : (double)((float)a + (float)b);
}

/* blockReduce + warpReduce (gn_kernels.cu:36-55): 256 -> 128 -> 64 -> 32, then a
 * lock-step warp tree (every lane reads before any lane writes). */
static double block_reduce(double* s) {
    for (int t = 0; t < 128; t++) s[t] = add_acc(s[t], s[t + 128]);
    for (int t = 0; t < 64; t++) s[t] = add_acc(s[t], s[t + 64]);
    for (int t = 0; t < 32; t++) s[t] = add_acc(s[t], s[t + 32]);
    for (int o = 16; o >= 1; o >>= 1) {
        double tmp[32];
        for (int t = 0; t < 32; t++) tmp[t] = add_acc(s[t], s[t + o]);
        for (int t = 0; t < 32; t++) s[t] = tmp[t];
    }
    return s[0];
}

/* Accumulate one residual row: Jx = [Ji, Jj], Ji = -Jj after the adjoint
 * (gn_kernels.cu:999-1013). */
static inline void accum_row(double* acc, const float* ti, const float* qi, const float* si,
                             float* Jx, float w, float err) {
    float* Ji = &Jx[0];
    float* Jj = &Jx[7];
    oracle_apply_sim3_adj_inv(ti, qi, si, Ji, Jj);
    for (int n = 0; n < 7; n++) Ji[n] = -Jj[n];
    int l = 0;
    for (int n = 0; n < 14; n++) {
        for (int m = 0; m <= n; m++) {
            acc[l] = add_prod(acc[l], w * Jx[n], Jx[m]);
            l++;
        }
    }
    double* vi = acc + HDIM;
    double* vj = acc + HDIM + 7;
    for (int n = 0; n < 7; n++) {
        vi[n] = add_prod(vi[n], w * err, Ji[n]);
        vj[n] = add_prod(vj[n], w * err, Jj[n]);
    }
}

/* Per-point residual model of the align kernels: the transformed point, residuals, robust
 * weights (Huber x confidence, gn_kernels.cu:963-978 / 1403-1418 / 598-613), the validity
 * flag and the raw (pre-adjoint) Jacobian rows.  Returns the number of residual rows. */
typedef struct {
    float Xj_Ci[3];
    float err[4], w[4];
    float J[4][7];
    int valid;
} point_res;

static int point_residuals(const oracle_gn_params* P, const float* tij, const float* qij,
                           const float* sij, const float* Xi, const float* Xj, float q, float ci,
                           float cj, int valid_match_ind, int64_t ind_Xi, point_res* R) {
    float* Xj_Ci = R->Xj_Ci;
    float* err = R->err;
    float* w = R->w;
    actSim3(tij, qij, sij, Xj, Xj_Ci);
    memset(R->J, 0, sizeof(R->J));
    if (P->mode == ORACLE_GN_RAYS) {
        /* gn_kernels.cu:924-1089 */
        const float sigma_ray_inv = (float)(1.0 / (double)P->sigma0);
        const float sigma_dist_inv = (float)(1.0 / (double)P->sigma1);
        const float norm2_i = squared_norm3(Xi);
        const float norm1_i = sqrtf(norm2_i);
        const float norm1_i_inv = (float)(1.0 / (double)norm1_i);
        /* ri = norm1_i_inv * Xi enters only err below */
        const float norm2_j = squared_norm3(Xj_Ci);
        const float norm1_j = sqrtf(norm2_j);
        const float norm1_j_inv = (float)(1.0 / (double)norm1_j);
        float rj[3];
        for (int i = 0; i < 3; i++) rj[i] = norm1_j_inv * Xj_Ci[i];
        /* rj - ri: a two-product difference (each ray a product with its inverse norm) */
        err[0] = cmm(CM, norm1_j_inv, Xj_Ci[0], -norm1_i_inv, Xi[0]);
        err[1] = cmm(CM, norm1_j_inv, Xj_Ci[1], -norm1_i_inv, Xi[1]);
        err[2] = cmm(CM, norm1_j_inv, Xj_Ci[2], -norm1_i_inv, Xi[2]);
        err[3] = norm1_j - norm1_i;
        const int valid = valid_match_ind & (q > P->Q_thresh) & (ci > P->C_thresh) & (cj > P->C_thresh);
        R->valid = valid;
        const float sqrt_w_ray = valid ? sigma_ray_inv * sqrtf(q) : 0.0f;
        const float sqrt_w_dist = valid ? sigma_dist_inv * sqrtf(q) : 0.0f;
        w[0] = huber(sqrt_w_ray * err[0]);
        w[1] = huber(sqrt_w_ray * err[1]);
        w[2] = huber(sqrt_w_ray * err[2]);
        w[3] = huber(sqrt_w_dist * err[3]);
        const float w_const_ray = sqrt_w_ray * sqrt_w_ray;
        const float w_const_dist = sqrt_w_dist * sqrt_w_dist;
        w[0] *= w_const_ray;
        w[1] *= w_const_ray;
        w[2] *= w_const_ray;
        w[3] *= w_const_dist;
        const float norm3_j_inv = norm1_j_inv / norm2_j;
        const float drx_dPx = cmad(CM, -(Xj_Ci[0] * Xj_Ci[0]), norm3_j_inv, norm1_j_inv);
        const float dry_dPy = cmad(CM, -(Xj_Ci[1] * Xj_Ci[1]), norm3_j_inv, norm1_j_inv);
        const float drz_dPz = cmad(CM, -(Xj_Ci[2] * Xj_Ci[2]), norm3_j_inv, norm1_j_inv);
        const float drx_dPy = ((-Xj_Ci[0]) * Xj_Ci[1]) * norm3_j_inv;
        const float drx_dPz = ((-Xj_Ci[0]) * Xj_Ci[2]) * norm3_j_inv;
        const float dry_dPz = ((-Xj_Ci[1]) * Xj_Ci[2]) * norm3_j_inv;
        float* J0 = R->J[0];
        float* J1 = R->J[1];
        float* J2 = R->J[2];
        float* J3 = R->J[3];
        J0[0] = drx_dPx; J0[1] = drx_dPy; J0[2] = drx_dPz;
        J0[3] = 0.0f; J0[4] = rj[2]; J0[5] = -rj[1]; J0[6] = 0.0f;
        J1[0] = drx_dPy; J1[1] = dry_dPy; J1[2] = dry_dPz;
        J1[3] = -rj[2]; J1[4] = 0.0f; J1[5] = rj[0]; J1[6] = 0.0f;
        J2[0] = drx_dPz; J2[1] = dry_dPz; J2[2] = drz_dPz;
        J2[3] = rj[1]; J2[4] = -rj[0]; J2[5] = 0.0f; J2[6] = 0.0f;
        J3[0] = rj[0]; J3[1] = rj[1]; J3[2] = rj[2];
        J3[3] = 0.0f; J3[4] = 0.0f; J3[5] = 0.0f; J3[6] = norm1_j;
        return 4;
    } else if (P->mode == ORACLE_GN_CALIB) {
        /* gn_kernels.cu:1360-1495 */
        const float fx = P->K[0], fy = P->K[4], cx = P->K[2], cy = P->K[5];
        const float sigma_pixel_inv = (float)(1.0 / (double)P->sigma0);
        const float sigma_depth_inv = (float)(1.0 / (double)P->sigma1);
        const int u_target = (int)(ind_Xi % P->width);
        const int v_target = (int)(ind_Xi / P->width);
        const int valid_z = (Xj_Ci[2] > P->z_eps) && (Xi[2] > P->z_eps);
        const float zj_inv = valid_z ? (float)(1.0 / (double)Xj_Ci[2]) : 0.0f;
        const float zj_log = valid_z ? logf(Xj_Ci[2]) : 0.0f;
        const float zi_log = valid_z ? logf(Xi[2]) : 0.0f;
        const float x_div_z = Xj_Ci[0] * zj_inv;
        const float y_div_z = Xj_Ci[1] * zj_inv;
        const float u = cmad(CM, fx, x_div_z, cx);
        const float v = cmad(CM, fy, y_div_z, cy);
        const int valid_u = (u > (float)P->pixel_border) && (u < (float)(P->width - 1 - P->pixel_border));
        const int valid_v = (v > (float)P->pixel_border) && (v < (float)(P->height - 1 - P->pixel_border));
        err[0] = u - (float)u_target;
        err[1] = v - (float)v_target;
        err[2] = zj_log - zi_log;
        const int valid = valid_match_ind & (q > P->Q_thresh) & (ci > P->C_thresh) & (cj > P->C_thresh) &
                          valid_u & valid_v & valid_z;
        R->valid = valid;
        const float sqrt_w_pixel = valid ? sigma_pixel_inv * sqrtf(q) : 0.0f;
        const float sqrt_w_depth = valid ? sigma_depth_inv * sqrtf(q) : 0.0f;
        w[0] = huber(sqrt_w_pixel * err[0]);
        w[1] = huber(sqrt_w_pixel * err[1]);
        w[2] = huber(sqrt_w_depth * err[2]);
        const float w_const_pixel = sqrt_w_pixel * sqrt_w_pixel;
        const float w_const_depth = sqrt_w_depth * sqrt_w_depth;
        w[0] *= w_const_pixel;
        w[1] *= w_const_pixel;
        w[2] *= w_const_depth;
        float* J0 = R->J[0];
        float* J1 = R->J[1];
        float* J2 = R->J[2];
        J0[0] = fx * zj_inv; J0[1] = 0.0f; J0[2] = ((-fx) * x_div_z) * zj_inv;
        J0[3] = ((-fx) * x_div_z) * y_div_z; J0[4] = fx * cmad(CM, x_div_z, x_div_z, 1.0f);
        J0[5] = (-fx) * y_div_z; J0[6] = 0.0f;
        J1[0] = 0.0f; J1[1] = fy * zj_inv; J1[2] = ((-fy) * y_div_z) * zj_inv;
        J1[3] = (-fy) * cmad(CM, y_div_z, y_div_z, 1.0f); J1[4] = (fy * x_div_z) * y_div_z;
        J1[5] = fy * x_div_z; J1[6] = 0.0f;
        J2[0] = 0.0f; J2[1] = 0.0f; J2[2] = zj_inv;
        J2[3] = y_div_z; J2[4] = -x_div_z; J2[5] = 0.0f; J2[6] = 1.0f;
        err[3] = 0.0f;
        w[3] = 0.0f;
        return 3;
    } else {
        /* point_align_kernel, gn_kernels.cu:564-674 */
        const float sigma_point_inv = (float)(1.0 / (double)P->sigma0);
        err[0] = Xj_Ci[0] - Xi[0];
        err[1] = Xj_Ci[1] - Xi[1];
        err[2] = Xj_Ci[2] - Xi[2];
        const int valid = valid_match_ind & (q > P->Q_thresh) & (ci > P->C_thresh) & (cj > P->C_thresh);
        R->valid = valid;
        const float sqrt_w_point = valid ? sigma_point_inv * sqrtf(q) : 0.0f;
        w[0] = huber(sqrt_w_point * err[0]);
        w[1] = huber(sqrt_w_point * err[1]);
        w[2] = huber(sqrt_w_point * err[2]);
        const float w_const_point = sqrt_w_point * sqrt_w_point;
        w[0] *= w_const_point;
        w[1] *= w_const_point;
        w[2] *= w_const_point;
        float* J0 = R->J[0];
        float* J1 = R->J[1];
        float* J2 = R->J[2];
        J0[0] = 1.0f; J0[1] = 0.0f; J0[2] = 0.0f; J0[3] = 0.0f;
        J0[4] = Xj_Ci[2]; J0[5] = -Xj_Ci[1]; J0[6] = Xj_Ci[0];
        J1[0] = 0.0f; J1[1] = 1.0f; J1[2] = 0.0f; J1[3] = -Xj_Ci[2];
        J1[4] = 0.0f; J1[5] = Xj_Ci[0]; J1[6] = Xj_Ci[1];
        J2[0] = 0.0f; J2[1] = 0.0f; J2[2] = 1.0f; J2[3] = Xj_Ci[1];
        J2[4] = -Xj_Ci[0]; J2[5] = 0.0f; J2[6] = Xj_Ci[2];
        err[3] = 0.0f;
        w[3] = 0.0f;
        return 3;
    }
}

static void align_point(const oracle_gn_params* P, const float* ti, const float* qi, const float* si,
                        const float* tij, const float* qij, const float* sij,
                        const float* Xi, const float* Xj, float q, float ci, float cj,
                        int valid_match_ind, int64_t ind_Xi, double* acc) {
    point_res R;
    const int nrows = point_residuals(P, tij, qij, sij, Xi, Xj, q, ci, cj, valid_match_ind, ind_Xi, &R);
    float Jx[14];
    for (int r = 0; r < nrows; r++) {
        memcpy(Jx, R.J[r], sizeof(float) * 7);
        accum_row(acc, ti, qi, si, Jx, R.w[r], R.err[r]);
    }
}

static void gn_align_impl(const oracle_gn_params* P, const float* Twc, const float* Xs,
                          const float* Cs, const int64_t* ii_edge, const int64_t* jj_edge,
                          const int64_t* idx, const uint8_t* valid, const float* Q,
                          int64_t N, int64_t HW, int64_t E, double* Hs, double* gs) {
    (void)N;
#pragma omp parallel
    {
        double* acc = (double*)malloc(sizeof(double) * THREADS * NACC);
        double* sdata = (double*)malloc(sizeof(double) * THREADS);
#pragma omp for schedule(dynamic, 1)
        for (int64_t e = 0; e < E; e++) {
            const int64_t ix = ii_edge[e], jx = jj_edge[e];
            const float* Ti = Twc + ix * 8;
            const float* Tj = Twc + jx * 8;
            float ti[3] = {Ti[0], Ti[1], Ti[2]}, qi[4] = {Ti[3], Ti[4], Ti[5], Ti[6]}, si[1] = {Ti[7]};
            float tj[3] = {Tj[0], Tj[1], Tj[2]}, qj[4] = {Tj[3], Tj[4], Tj[5], Tj[6]}, sj[1] = {Tj[7]};
            float tij[3], qij[4], sij[1];
            relSim3(ti, qi, si, tj, qj, sj, tij, qij, sij);
            memset(acc, 0, sizeof(double) * THREADS * NACC);
            for (int t = 0; t < THREADS; t++) {
                double* a = acc + (int64_t)t * NACC;
                for (int64_t k = t; k < HW; k += THREADS) { /* GPU_1D_KERNEL_LOOP (:31-32) */
                    const int64_t pe = e * HW + k;
                    const int vm = valid[pe] != 0;
                    const int64_t ind = vm ? idx[pe] : 0;
                    const float* Xi = Xs + (ix * HW + ind) * 3;
                    const float* Xj = Xs + (jx * HW + k) * 3;
                    align_point(P, ti, qi, si, tij, qij, sij, Xi, Xj, Q[pe], Cs[ix * HW + ind],
                                Cs[jx * HW + k], vm, ind, a);
                }
            }
            /* gs (gn_kernels.cu:1097-1112) */
            for (int n = 0; n < 14; n++) {
                for (int t = 0; t < THREADS; t++) sdata[t] = acc[(int64_t)t * NACC + HDIM + n];
                double v = block_reduce(sdata);
                if (n < 7) gs[(0 * E + e) * 7 + n] = v;
                else gs[(1 * E + e) * 7 + (n - 7)] = v;
            }
            /* Hs (gn_kernels.cu:1114-1137) */
            int l = 0;
            for (int n = 0; n < 14; n++) {
                for (int m = 0; m <= n; m++) {
                    for (int t = 0; t < THREADS; t++) sdata[t] = acc[(int64_t)t * NACC + l];
                    double v = block_reduce(sdata);
                    if (n < 7 && m < 7) {
                        Hs[((0 * E + e) * 7 + n) * 7 + m] = v;
                        Hs[((0 * E + e) * 7 + m) * 7 + n] = v;
                    } else if (n >= 7 && m < 7) {
                        Hs[((1 * E + e) * 7 + m) * 7 + (n - 7)] = v;
                        Hs[((2 * E + e) * 7 + (n - 7)) * 7 + m] = v;
                    } else {
                        Hs[((3 * E + e) * 7 + (n - 7)) * 7 + (m - 7)] = v;
                        Hs[((3 * E + e) * 7 + (m - 7)) * 7 + (n - 7)] = v;
                    }
                    l++;
                }
            }
        }
        free(acc);
        free(sdata);
    }
}

void oracle_gn_residuals(const oracle_gn_params* P, const float* Twc, const float* Xs,
                         const float* Cs, const int64_t* ii_edge, const int64_t* jj_edge,
                         const int64_t* idx, const uint8_t* valid, const float* Q,
                         int64_t N, int64_t HW, int64_t E, float* Xj_Ci, float* err, float* w,
                         uint8_t* valid_out) {
    (void)N;
    for (int64_t e = 0; e < E; e++) {
        const int64_t ix = ii_edge[e], jx = jj_edge[e];
        const float* Ti = Twc + ix * 8;
        const float* Tj = Twc + jx * 8;
        float ti[3] = {Ti[0], Ti[1], Ti[2]}, qi[4] = {Ti[3], Ti[4], Ti[5], Ti[6]}, si[1] = {Ti[7]};
        float tj[3] = {Tj[0], Tj[1], Tj[2]}, qj[4] = {Tj[3], Tj[4], Tj[5], Tj[6]}, sj[1] = {Tj[7]};
        float tij[3], qij[4], sij[1];
        relSim3(ti, qi, si, tj, qj, sj, tij, qij, sij);
        for (int64_t k = 0; k < HW; k++) {
            const int64_t pe = e * HW + k;
            const int vm = valid[pe] != 0;
            const int64_t ind = vm ? idx[pe] : 0;
            point_res R;
            point_residuals(P, tij, qij, sij, Xs + (ix * HW + ind) * 3, Xs + (jx * HW + k) * 3, Q[pe],
                            Cs[ix * HW + ind], Cs[jx * HW + k], vm, ind, &R);
            memcpy(Xj_Ci + pe * 3, R.Xj_Ci, sizeof(float) * 3);
            memcpy(err + pe * 4, R.err, sizeof(float) * 4);
            memcpy(w + pe * 4, R.w, sizeof(float) * 4);
            valid_out[pe] = (uint8_t)(R.valid != 0);
        }
    }
}

void oracle_gn_align(const oracle_gn_params* P, const float* Twc, const float* Xs,
                     const float* Cs, const int64_t* ii_edge, const int64_t* jj_edge,
                     const int64_t* idx, const uint8_t* valid, const float* Q,
                     int64_t N, int64_t HW, int64_t E, float* Hs, float* gs) {
    double* Hd = (double*)malloc(sizeof(double) * 4 * E * 49 + 8);
    double* gd = (double*)malloc(sizeof(double) * 2 * E * 7 + 8);
    gn_align_impl(P, Twc, Xs, Cs, ii_edge, jj_edge, idx, valid, Q, N, HW, E, Hd, gd);
    for (int64_t k = 0; k < 4 * E * 49; k++) Hs[k] = (float)Hd[k];
    for (int64_t k = 0; k < 2 * E * 7; k++) gs[k] = (float)gd[k];
    free(Hd);
    free(gd);
}

/* ------------------------------------------------------------------------ */
/* SparseBlock assembly + SimplicialLLT semantics (gn_kernels.cu:57-159)    */
/* ------------------------------------------------------------------------ */

static void gn_assemble_d(const double* Hs, const double* gs, const int64_t* ii_opt,
                          const int64_t* jj_opt, int64_t N, int64_t E, double* H, double* b);

void oracle_gn_assemble(const float* Hs, const float* gs, const int64_t* ii_opt,
                        const int64_t* jj_opt, int64_t N, int64_t E,
                        double* H, double* b) {
    double* Hd = (double*)malloc(sizeof(double) * 4 * E * 49 + 8);
    double* gd = (double*)malloc(sizeof(double) * 2 * E * 7 + 8);
    for (int64_t k = 0; k < 4 * E * 49; k++) Hd[k] = (double)Hs[k];
    for (int64_t k = 0; k < 2 * E * 7; k++) gd[k] = (double)gs[k];
    gn_assemble_d(Hd, gd, ii_opt, jj_opt, N, E, H, b);
    free(Hd);
    free(gd);
}

/* The dense system of one iteration as oracle_gauss_newton forms it (the per-edge blocks kept in
 * double: outside exact-sums mode they are float values already, so this equals gn_align +
 * gn_assemble; in exact-sums mode it is the exactly summed system, unrounded). */
void oracle_gn_system(const oracle_gn_params* P, const float* Twc, const float* Xs, const float* Cs,
                      const int64_t* ii_edge, const int64_t* jj_edge, const int64_t* idx,
                      const uint8_t* valid, const float* Q, int64_t N, int64_t HW, int64_t E,
                      double* H, double* b) {
    double* Hd = (double*)malloc(sizeof(double) * 4 * E * 49 + 8);
    double* gd = (double*)malloc(sizeof(double) * 2 * E * 7 + 8);
    int64_t* ii_opt = (int64_t*)malloc(sizeof(int64_t) * (E + 1));
    int64_t* jj_opt = (int64_t*)malloc(sizeof(int64_t) * (E + 1));
    for (int64_t e = 0; e < E; e++) {
        ii_opt[e] = ii_edge[e] - 1;
        jj_opt[e] = jj_edge[e] - 1;
    }
    gn_align_impl(P, Twc, Xs, Cs, ii_edge, jj_edge, idx, valid, Q, N, HW, E, Hd, gd);
    gn_assemble_d(Hd, gd, ii_opt, jj_opt, N, E, H, b);
    free(Hd);
    free(gd);
    free(ii_opt);
    free(jj_opt);
}

static void gn_assemble_d(const double* Hs, const double* gs, const int64_t* ii_opt,
                          const int64_t* jj_opt, int64_t N, int64_t E, double* H, double* b) {
    const int64_t n = 7 * (N - 1);
    memset(H, 0, sizeof(double) * n * n);
    memset(b, 0, sizeof(double) * n);
    /* update_lhs: rows cat(ii,ii,jj,jj), cols cat(ii,jj,ii,jj), triplet order */
    for (int blk = 0; blk < 4; blk++) {
        const int64_t* rows = (blk < 2) ? ii_opt : jj_opt;
        const int64_t* cols = (blk == 0 || blk == 2) ? ii_opt : jj_opt;
        for (int64_t e = 0; e < E; e++) {
            const int64_t i = rows[e], j = cols[e];
            if (i >= 0 && j >= 0) {
                const double* A = Hs + ((int64_t)blk * E + e) * 49;
                for (int k = 0; k < 7; k++)
                    for (int l = 0; l < 7; l++) H[(7 * i + k) * n + 7 * j + l] += A[k * 7 + l];
            }
        }
    }
    /* update_rhs: cat(ii,jj) */
    for (int blk = 0; blk < 2; blk++) {
        const int64_t* rows = blk == 0 ? ii_opt : jj_opt;
        for (int64_t e = 0; e < E; e++) {
            const int64_t i = rows[e];
            if (i >= 0) {
                const double* g = gs + ((int64_t)blk * E + e) * 7;
                for (int j = 0; j < 7; j++) b[i * 7 + j] += g[j];
            }
        }
    }
}

/* Dense LL^T in double on the lower triangle.  SimplicialLLT fails iff a pivot
 * d <= 0 (a NaN pivot does not fail); then the caller uses dx = 0
 * (gn_kernels.cu:142-150).  Eigen factorises the AMD-permuted matrix; the
 * solution is the same up to double rounding. */
int oracle_cholesky_solve(double* L, const double* b, double* x, int64_t n) {
    for (int64_t k = 0; k < n; k++) {
        double d = L[k * n + k];
        for (int64_t p = 0; p < k; p++) d -= L[k * n + p] * L[k * n + p];
        if (d <= 0.0) {
            for (int64_t i = 0; i < n; i++) x[i] = 0.0;
            return 1;
        }
        const double lkk = sqrt(d);
        L[k * n + k] = lkk;
#pragma omp parallel for schedule(static) if (n - k > 256)
        for (int64_t i = k + 1; i < n; i++) {
            double s = L[i * n + k];
            const double* Li = L + i * n;
            const double* Lk = L + k * n;
            for (int64_t p = 0; p < k; p++) s -= Li[p] * Lk[p];
            L[i * n + k] = s / lkk;
        }
    }
    /* forward L y = b */
    for (int64_t i = 0; i < n; i++) {
        double s = b[i];
        for (int64_t p = 0; p < i; p++) s -= L[i * n + p] * x[p];
        x[i] = s / L[i * n + i];
    }
    /* backward L^T x = y */
    for (int64_t i = n - 1; i >= 0; i--) {
        double s = x[i];
        for (int64_t p = i + 1; p < n; p++) s -= L[p * n + i] * x[p];
        x[i] = s / L[i * n + i];
    }
    return 0;
}

static int cmp_i64(const void* a, const void* b) {
    int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
    return (x > y) - (x < y);
}

static int64_t searchsorted_left(const int64_t* u, int64_t n, int64_t v) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t mid = (lo + hi) / 2;
        if (u[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

/* get_unique_kf_idx + create_inds (gn_kernels.cu:161-170), pin = 0 */
int64_t oracle_remap(const int64_t* ii, const int64_t* jj, int64_t E, int64_t* ii_edge, int64_t* jj_edge) {
    int64_t* u = (int64_t*)malloc(sizeof(int64_t) * (2 * E + 1));
    for (int64_t e = 0; e < E; e++) {
        u[e] = ii[e];
        u[E + e] = jj[e];
    }
    qsort(u, (size_t)(2 * E), sizeof(int64_t), cmp_i64);
    int64_t nu = 0;
    for (int64_t k = 0; k < 2 * E; k++)
        if (nu == 0 || u[k] != u[nu - 1]) u[nu++] = u[k];
    for (int64_t e = 0; e < E; e++) {
        ii_edge[e] = searchsorted_left(u, nu, ii[e]);
        jj_edge[e] = searchsorted_left(u, nu, jj[e]);
    }
    free(u);
    return nu;
}

/* gauss_newton_*_cuda drivers */
int oracle_gauss_newton(const oracle_gn_params* P, float* Twc, const float* Xs,
                        const float* Cs, const int64_t* ii, const int64_t* jj,
                        const int64_t* idx, const uint8_t* valid, const float* Q,
                        int64_t N, int64_t HW, int64_t E, float* dx) {
    const int num_fix = 1;
    const int64_t n = 7 * (N - num_fix);
    int64_t* ii_edge = (int64_t*)malloc(sizeof(int64_t) * (E + 1));
    int64_t* jj_edge = (int64_t*)malloc(sizeof(int64_t) * (E + 1));
    int64_t* ii_opt = (int64_t*)malloc(sizeof(int64_t) * (E + 1));
    int64_t* jj_opt = (int64_t*)malloc(sizeof(int64_t) * (E + 1));
    oracle_remap(ii, jj, E, ii_edge, jj_edge);
    for (int64_t e = 0; e < E; e++) {
        ii_opt[e] = ii_edge[e] - num_fix;
        jj_opt[e] = jj_edge[e] - num_fix;
    }
    double* Hs = (double*)malloc(sizeof(double) * 4 * E * 49 + 8);
    double* gs = (double*)malloc(sizeof(double) * 2 * E * 7 + 8);
    double* H = (double*)malloc(sizeof(double) * (n * n + 1));
    double* b = (double*)malloc(sizeof(double) * (n + 1));
    double* x = (double*)malloc(sizeof(double) * (n + 1));
    int itr;
    for (itr = 0; itr < P->max_iter; itr++) {
        gn_align_impl(P, Twc, Xs, Cs, ii_edge, jj_edge, idx, valid, Q, N, HW, E, Hs, gs);
        gn_assemble_d(Hs, gs, ii_opt, jj_opt, N, E, H, b);
        oracle_cholesky_solve(H, b, x, n);
        double nrm = 0.0;
        for (int64_t k = 0; k < n; k++) {
            dx[k] = -(float)x[k]; /* "dx = -A.solve()" (:1209), solve() returns float */
            nrm += (double)dx[k] * (double)dx[k];
        }
        oracle_pose_retr(Twc, dx, N, num_fix);
        if ((float)sqrt(nrm) < P->delta_thresh) { /* :1219-1222 */
            itr++;
            break;
        }
    }
    free(ii_edge); free(jj_edge); free(ii_opt); free(jj_opt);
    free(Hs); free(gs); free(H); free(b); free(x);
    return itr;
}
