// refine_common.h -- what the refine_matches kernels share (matching.hip: the product kernels;
// refine_variants.hip: the measured-slower A/B variants, built into a separate library).
// Parity contract as matching.hip: contraction OFF, c10::Half per-op rounding.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/m3s_backend.h"
#include "m3s_common.h"

#pragma clang fp contract(off)

namespace {

constexpr int kBlock = 256;

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

// refine_matches (F = 24 fp16, radius R) on a plane-major copy of D11: plane q holds the 16-B
// piece q (halves 8q .. 8q+7) of every cell, [B][3][H*W] x 16 B, so load q of a wave reads ~1/3
// of the cache lines the interleaved 48-B rows cost.  The fused matching op writes D11's .half()
// directly in this layout (match_glue.hip); refine_variants.hip's PLANES variant copies it first.
// Same candidate order and c10::Half chain as refine_f16_kernel => the same matches.
template <int R>
__global__ __launch_bounds__(kBlock) void refine_planes_kernel(const uint4* __restrict__ P, const uint16_t* __restrict__ D21,
                                                              const int64_t* __restrict__ p1, int64_t* __restrict__ p1_new,
                                                              int64_t* __restrict__ lin, int H, int W, int64_t N, int64_t B,
                                                              TileMap tm, int dilation_max) {
    constexpr int F = 24, SC = 2 * R + 1;
    int64_t g;
    if (!tile_pixel(tm, B, W, H, g)) return;
    const int64_t b = g / N;
    const int64_t HW = (int64_t)H * W;
    half2_t q2[F / 2];
    {
        const uint4* src = reinterpret_cast<const uint4*>(D21 + g * F);
#pragma unroll
        for (int c = 0; c < F / 8; c++) {
            const uint4 w = src[c];
            const half2_t* hp = reinterpret_cast<const half2_t*>(&w);
#pragma unroll
            for (int k = 0; k < 4; k++) q2[c * 4 + k] = hp[k];
        }
    }
    const uint4* __restrict__ pl = P + b * 3 * HW;
    int64_t u0 = p1[g * 2 + 0];
    int64_t v0 = p1[g * 2 + 1];
    half_t max_score = (half_t)kRefineHalfMaxInit;
    int64_t u_new = u0, v_new = v0;
    for (int d = dilation_max; d > 0; d--) {
        const int64_t rd = (int64_t)R * d;
        for (int i = 0; i < SC; i++) {  // u offset outer (matching_kernels.cu:54)
            const int64_t u = u0 - rd + (int64_t)i * d;
            uint4 rows[SC][3];
            bool ok[SC];
#pragma unroll
            for (int j = 0; j < SC; j++) {
                const int64_t v = v0 - rd + (int64_t)j * d;
                ok[j] = inside_image(u, v, W, H);
                const int64_t cell = ok[j] ? v * W + u : 0;
#pragma unroll
                for (int q = 0; q < 3; q++) rows[j][q] = pl[q * HW + cell];
            }
            half_t score[SC];
            score_f16_multi<F, SC>(q2, rows, score);
#pragma unroll
            for (int j = 0; j < SC; j++) {  // v offset inner (:55)
                if (ok[j] && score[j] > max_score) {
                    max_score = score[j];
                    u_new = u;
                    v_new = v0 - rd + (int64_t)j * d;
                }
            }
        }
        u0 = u_new;
        v0 = v_new;
    }
    store_match(p1_new, lin, g, W, u_new, v_new);
}

}  // namespace

// argument checks shared by every refine entry point (host)
static inline int refine_checks(const void* D11, const void* D21, const void* p1, void* out, int64_t B,
                                int64_t H, int64_t W, int64_t N, int64_t F, int radius, int dilation_max) {
    M3S_REQUIRE(B >= 0 && N >= 0 && H >= 0 && W >= 0 && F >= 0, "refine_matches: negative sizes");
    M3S_REQUIRE(H * W < (int64_t)1 << 31, "refine_matches: image too large");
    M3S_REQUIRE(radius >= 0 && dilation_max >= 0, "refine_matches: negative radius/dilation");
    if (B * N > 0) M3S_REQUIRE(D11 && D21 && p1 && out, "refine_matches: null pointer");
    return M3S_OK;
}
