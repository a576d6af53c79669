// refine_variants.hip -- the refine_matches kernels that were built, proven exact and measured
// SLOWER than the product kernel (matching.hip refine_f16_kernel) on the bench data: kept for
// the A/Bs in bench.py and DESIGN.md section 4, in their own library (lib/libm3s_variants.so,
// include/m3s_variants.h), not in the drop-in libm3s_backend.so.
//
//   M3S_REFINE_VARIANT_LDS   the candidate box of a 32x16 tile staged in LDS
//   M3S_REFINE_VARIANT_MFMA  approximate scores on v_mfma_f32_16x16x32_f16 + exact re-scoring
//   M3S_REFINE_VARIANT_DOT2  approximate scores with v_dot2 + exact re-scoring
//
// Parity contract as matching.hip (compiled with contraction off; c10::Half per-op rounding).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstdlib>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "../../include/m3s_variants.h"
#include "refine_common.h"

// this library's own error state (m3s_common.h's set_error)
namespace m3s {
namespace {
thread_local std::string g_err;
}
void set_error(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
}
}  // namespace m3s
extern "C" const char* m3s_variants_last_error(void) { return m3s::g_err.c_str(); }

namespace {

// ---------------------------------------------------------------------------------
// refine_matches with the correlation on MFMA (variant M3S_REFINE_VARIANT_MFMA; SURVEY §8(d) prices the
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
// refine_matches with the correlation on MFMA over LATTICE BUCKETS (variant LATTICE).
//
// At dilation d a pixel's 49 candidates are the lattice points c_p + d (i, j), |i|, |j| <= R, of
// ITS centre c_p.  Two pixels share candidates only when their centres are congruent mod d, so
// per level the tile's pixels are bucketed by class (u0 mod d, v0 mod d) -- d^2 classes, members
// kept in pixel order -- and cut into groups of 16.  A group's windows, in lattice coordinates
// (U, V) = floor(c / d), all lie in its box [Umin - R, Umax + R] x [Vmin - R, Vmax + R]; one
// v_mfma_f32_16x16x32_f16 scores the group's 16 descriptors (A, K = 24 zero-padded to 32) against
// 16 box cells (B, one 16-B piece per lane gathered from D11), and each of the 16 x 16 outputs that
// lies in its pixel's window goes to the pixel's score table in LDS.  On smooth matches the boxes
// are small (about (16/d + 6)^2 cells at d >= 4, (16 + 6) x (1 + 6) at d = 1), so every D11 row is
// loaded once per group instead of once per candidate, and 25-45 % of the MFMA outputs are used
// (the diagonal formulation above: 1/16).  Then per pixel the bound-and-rescore of
// refine_mfma_kernel (same bound E, same shortlist rule) re-scores the possible winners exactly
// in candidate order.  A group whose box exceeds kLatCellLimit cells (a discontinuity, far
// starts) and pixels whose bound is not finite score every candidate exactly instead.
// ---------------------------------------------------------------------------------
constexpr int kLatCellLimit = 512;
constexpr int kLatBatch = 8;  // box chunks (16 cells) whose gathers are in flight together
// diagnostics builds only: 1 = no MFMA phase (every pixel scored exactly), 2 = no exact phase
// (the results are then NOT refine_matches'), 3 = neither (bucketing alone)
#ifndef M3S_LAT_DIAG
#define M3S_LAT_DIAG 0
#endif
constexpr int kLatMaxD = 5;  // dilation levels with <= 25 classes; larger dilation_max: the caller falls back
constexpr int kLatMaxCls = kLatMaxD * kLatMaxD;
constexpr int kLatMaxItems = kBlock / 16 + kLatMaxCls;

__device__ __forceinline__ int floordiv(int a, int d) { return a >= 0 ? a / d : -((-a + d - 1) / d); }

template <int R>
__global__ __launch_bounds__(kBlock) void refine_lattice_kernel(
    const uint16_t* __restrict__ D11, const uint16_t* __restrict__ D21, const int64_t* __restrict__ p1,
    int64_t* __restrict__ p1_new, int64_t* __restrict__ lin, int H, int W, int64_t N, int64_t B, TileMap tm,
    int dilation_max, const unsigned* __restrict__ hmax2, unsigned long long* __restrict__ stats) {
    constexpr int F = 24;
    constexpr int S = 2 * R + 1;
    constexpr int NC = S * S;
    static_assert(NC <= 64, "candidate mask is 64 bits");
    // approximate scores [candidate][pixel of the tile], rows padded by one: the 16 lanes that
    // write one pixel's scores (different candidates) hit 16 different banks
    __shared__ float sS[NC][kBlock + 1];
    __shared__ int sU[kBlock], sV[kBlock];   // lattice centre of each pixel at this level
    __shared__ unsigned char sMem[kBlock];   // the tile's pixels sorted by class, pixel order within
    __shared__ unsigned char sFall[kBlock];  // 1: score every candidate exactly at this level
    __shared__ int sCnt[kBlock / 64][kLatMaxCls];
    __shared__ int sBase[kBlock / 64][kLatMaxCls];
    __shared__ int sOff[kLatMaxCls + 1];
    __shared__ int sItem[kLatMaxItems];
    __shared__ int sNItems;

    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    // the tile (the XCD-banded order of tile_pixel), every thread stays for the MFMAs
    const int64_t nblk = (int64_t)gridDim.x, blk = blockIdx.x;
    const int64_t per = (nblk + 7) / 8;
    const int64_t lb = (blk % 8) * per + blk / 8;
    if (lb >= (int64_t)tm.ntiles * B) return;  // uniform over the workgroup
    const int64_t b = lb / tm.ntiles;
    const int tt = (int)(lb - b * tm.ntiles);
    const int ty = tt / tm.tiles_x, tx = tt - ty * tm.tiles_x;
    auto pix_g = [&](int p) { return b * N + (int64_t)(ty * kTile + (p >> 4)) * W + tx * kTile + (p & 15); };
    const bool active = tx * kTile + (t & 15) < W && ty * kTile + (t >> 4) < H;
    const int64_t g = active ? pix_g(t) : 0;
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
    const float pbound = (sqrtf(qn2) * 1.00001f) * hmax;  // >= sum_k |q_k h_k| for every candidate
    const float E = kRefineBoundRel * pbound + kRefineBoundAbs;
    const bool score_all = !(pbound <= kRefineBoundMax);  // NaN / inf / fp16 overflow possible

    int64_t u0 = active ? p1[g * 2 + 0] : 0;
    int64_t v0 = active ? p1[g * 2 + 1] : 0;
    half_t max_score = (half_t)kRefineHalfMaxInit;
    int64_t u_new = u0, v_new = v0;
    unsigned nresc = 0, ntotal = 0, nmfma = 0;
    const int m = lane & 15, kc = lane >> 4;
    for (int d = dilation_max; d > 0; d--) {
        const int64_t rd = (int64_t)R * d;
        const int ncls = d * d;
        // 1. class and lattice centre (int32 lattice math while the centre is within 2^20 px)
        const bool near = u0 >= -(1 << 20) && u0 <= (1 << 20) && v0 >= -(1 << 20) && v0 <= (1 << 20);
        int cls = -1;
        if (active && near) {
            const int uu = (int)u0, vv = (int)v0;
            const int U = floordiv(uu, d), V = floordiv(vv, d);
            sU[t] = U;
            sV[t] = V;
            cls = (uu - U * d) * d + (vv - V * d);
        }
        sFall[t] = (active && (!near || score_all)) ? 1 : 0;
        if (!(active && near && !score_all)) cls = -1;
        // 2. rank within the class (pixel order), per wave
        int rank = 0;
        for (int c = 0; c < ncls; c++) {
            const uint64_t mk = __ballot(cls == c);
            if (cls == c) rank = __popcll(mk & ((1ull << lane) - 1ull));
            if (lane == 0) sCnt[wave][c] = __popcll(mk);
        }
        __syncthreads();
        // 3. class offsets, per-wave bases and the work items (class, group of 16): wave 0
        if (wave == 0) {
            int tot = 0;
            if (lane < ncls) {
#pragma unroll
                for (int w = 0; w < kBlock / 64; w++) tot += sCnt[w][lane];
            }
            int inc = tot, ng = (tot + 15) / 16, ginc = ng;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const int y = __shfl_up(inc, off, 64), z = __shfl_up(ginc, off, 64);
                if (lane >= off) {
                    inc += y;
                    ginc += z;
                }
            }
            if (lane < ncls) {
                int run = inc - tot;
                sOff[lane] = run;
#pragma unroll
                for (int w = 0; w < kBlock / 64; w++) {
                    sBase[w][lane] = run;
                    run += sCnt[w][lane];
                }
                for (int q = 0; q < ng; q++) sItem[ginc - ng + q] = (lane << 8) | q;
            }
            if (lane == ncls - 1) sOff[ncls] = inc;
            if (lane == 63) sNItems = ginc;
        }
        __syncthreads();
        if (cls >= 0) sMem[sBase[wave][cls] + rank] = (unsigned char)t;
        __syncthreads();
        // 4. approximate scores over each group's lattice box
        const int nitems = (M3S_LAT_DIAG & 1) ? 0 : sNItems;
        if ((M3S_LAT_DIAG & 1) && active) sFall[t] = 1;
        for (int it = wave; it < nitems; it += kBlock / 64) {
            const int code = sItem[it];
            const int c = code >> 8, grp = code & 255;
            const int base = sOff[c] + 16 * grp, cnt = min(16, sOff[c + 1] - base);
            const int pm = m < cnt ? (int)sMem[base + m] : -1;
            const int Um = pm >= 0 ? sU[pm] : 0, Vm = pm >= 0 ? sV[pm] : 0;
            int umin = pm >= 0 ? Um : INT_MAX, umax = pm >= 0 ? Um : INT_MIN;
            int vmin = pm >= 0 ? Vm : INT_MAX, vmax = pm >= 0 ? Vm : INT_MIN;
#pragma unroll
            for (int off = 1; off < 16; off <<= 1) {  // over the 16 members (each 16-lane row holds all)
                umin = min(umin, __shfl_xor(umin, off, 64));
                umax = max(umax, __shfl_xor(umax, off, 64));
                vmin = min(vmin, __shfl_xor(vmin, off, 64));
                vmax = max(vmax, __shfl_xor(vmax, off, 64));
            }
            const int bu = umax - umin + 2 * R + 1, bv = vmax - vmin + 2 * R + 1;
            if (bu > kLatCellLimit || bv > kLatCellLimit || bu * bv > kLatCellLimit) {
                if (lane < cnt) sFall[sMem[base + lane]] = 1;  // this group scores exactly
                continue;
            }
            const int cells = bu * bv;
            nmfma += (cells + 15) / 16;  // wave-uniform: counted by every lane, reported by lane 0
            uint4 wa = make_uint4(0, 0, 0, 0);
            if (pm >= 0 && kc < 3) wa = reinterpret_cast<const uint4*>(D21 + pix_g(pm) * F)[kc];
            const half8_t A = __builtin_bit_cast(half8_t, wa);
            // this lane's 4 output rows: members 4 kc + e
            int pe[4], Ue[4], Ve[4];
#pragma unroll
            for (int e = 0; e < 4; e++) {
                pe[e] = __shfl(pm, 4 * kc + e, 64);
                Ue[e] = __shfl(Um, 4 * kc + e, 64);
                Ve[e] = __shfl(Vm, 4 * kc + e, 64);
            }
            const int cu = c / d, cv = c - cu * d;  // the class's residues
            // kLatBatch chunks at a time: their B gathers are issued together, then the MFMAs
            for (int ch0 = 0; ch0 < cells; ch0 += 16 * kLatBatch) {
                uint4 wb[kLatBatch];
                int Ucs[kLatBatch], Vcs[kLatBatch];
#pragma unroll
                for (int q = 0; q < kLatBatch; q++) {
                    const int ci = ch0 + 16 * q + m;
                    const int qv = ci / bu;
                    Ucs[q] = umin - R + (ci - qv * bu);
                    Vcs[q] = vmin - R + qv;
                    const int64_t u = (int64_t)cu + (int64_t)d * Ucs[q], v = (int64_t)cv + (int64_t)d * Vcs[q];
                    wb[q] = make_uint4(0, 0, 0, 0);
                    if (ci < cells && kc < 3 && inside_image(u, v, W, H))
                        wb[q] = reinterpret_cast<const uint4*>(img + (v * W + u) * F)[kc];
                    if (ci >= cells) Ucs[q] = INT_MIN / 2;  // no pixel's window
                }
#pragma unroll
                for (int q = 0; q < kLatBatch; q++) {
                    if (ch0 + 16 * q >= cells) break;  // wave-uniform
                    float4_t acc = {0.0f, 0.0f, 0.0f, 0.0f};
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(A, __builtin_bit_cast(half8_t, wb[q]), acc, 0, 0, 0);
#pragma unroll
                    for (int e = 0; e < 4; e++) {
                        const unsigned di = (unsigned)(Ucs[q] - Ue[e] + R), dj = (unsigned)(Vcs[q] - Ve[e] + R);
                        if (pe[e] >= 0 && di < (unsigned)S && dj < (unsigned)S) sS[di * S + dj][pe[e]] = acc[e];
                    }
                }
            }
        }
        __syncthreads();
        // 5. per pixel: the shortlist of possible winners, re-scored exactly in candidate order
        if (active && !(M3S_LAT_DIAG & 2)) {
            const bool all = sFall[t] != 0;
            uint64_t mask = 0;
            float lo = -__int_as_float(0x7f800000);
            if (!all) {
#pragma unroll
                for (int c = 0; c < NC; c++) {
                    const int64_t u = u0 - rd + (int64_t)(c / S) * d, v = v0 - rd + (int64_t)(c % S) * d;
                    if (inside_image(u, v, W, H)) lo = fmaxf(lo, sS[c][t] - E);
                }
            }
            const float beat = (float)max_score;
#pragma unroll
            for (int c = 0; c < NC; c++) {
                const int64_t u = u0 - rd + (int64_t)(c / S) * d, v = v0 - rd + (int64_t)(c % S) * d;
                const bool in = inside_image(u, v, W, H);
                ntotal += in;
                if (in && (all || (sS[c][t] + E >= lo && sS[c][t] + E > beat))) mask |= 1ull << c;
            }
            nresc += __builtin_popcountll(mask);
            while (mask) {  // up to 4 shortlisted rows in flight, then scored in candidate order
                int cs[4];
                uint4 rows[4][F / 8];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    cs[q] = mask ? __builtin_ctzll(mask) : -1;
                    mask &= mask - 1;
                    if (cs[q] >= 0) {
                        const int64_t u = u0 - rd + (int64_t)(cs[q] / S) * d, v = v0 - rd + (int64_t)(cs[q] % S) * d;
                        const uint4* src = reinterpret_cast<const uint4*>(img + (v * W + u) * F);
#pragma unroll
                        for (int k = 0; k < F / 8; k++) rows[q][k] = src[k];
                    }
                }
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    if (cs[q] < 0) break;
                    const half_t score = score_f16<F>(q2, rows[q]);
                    if (score > max_score) {
                        max_score = score;
                        u_new = u0 - rd + (int64_t)(cs[q] / S) * d;
                        v_new = v0 - rd + (int64_t)(cs[q] % S) * d;
                    }
                }
            }
            u0 = u_new;
            v0 = v_new;
        }
        __syncthreads();  // the next level rewrites the tables
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
            atomicAdd(stats + 2, (unsigned long long)nmfma);
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


// ---------------------------------------------------------------------------------
// refine_matches, plane-major LDS box (M3S_REFINE_VARIANT_BOX, round 5).
//
// A 256-thread workgroup takes a 16x16 pixel tile (lane = pixel, the product kernel's XCD-banded
// tile order).  Per dilation level it stages the bounding box of its pixels' image-clipped
// candidate windows in LDS once -- coalesced 16-B global loads, 48 B per cell -- as 6 planes of
// 8-B pieces (plane p holds halves 4p .. 4p+3 of every cell: a candidate is 6 ds_read_b64, 32
// lanes per LDS cycle, bank pair 2 * cell mod 64), then scores every candidate from LDS with the
// product kernel's exact c10::Half chain (score_f16_multi) in the reference's candidate order, a
// window column of 7 at a time, the next column's reads issued before the current one is scored.
// The 16x16 tile keeps the largest box (d = 5: ~54 x 54 cells) under the 3300-cell cap, where
// the former LDS variant's 32 x 16 tile sent every d = 5 level to its slow global fallback; a
// level whose box still exceeds the cap gathers its candidates from global memory, a window
// column at a time as the product kernel does.  Bitwise the product kernel's matches.
// ---------------------------------------------------------------------------------
constexpr int kBoxCap = 3300;  // cells: 6 planes x 8 B x 3300 = 158,400 B of the CU's 160 KiB

__device__ __forceinline__ void box_minmax4(int (&v)[4], int* red /* [4 waves][4] */) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        v[0] = min(v[0], __shfl_xor(v[0], off, 64));
        v[1] = max(v[1], __shfl_xor(v[1], off, 64));
        v[2] = min(v[2], __shfl_xor(v[2], off, 64));
        v[3] = max(v[3], __shfl_xor(v[3], off, 64));
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 4; k++) red[wave * 4 + k] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (int w = 0; w < 4; w++) {
        v[0] = min(v[0], red[w * 4 + 0]);
        v[1] = max(v[1], red[w * 4 + 1]);
        v[2] = min(v[2], red[w * 4 + 2]);
        v[3] = max(v[3], red[w * 4 + 3]);
    }
    __syncthreads();  // red is rewritten by the next level
}

template <int R, int DIAG = 0>
__global__ __launch_bounds__(kBlock) void refine_box_kernel(const uint16_t* __restrict__ D11,
                                                           const uint16_t* __restrict__ D21,
                                                           const int64_t* __restrict__ p1, int64_t* __restrict__ p1_new,
                                                           int64_t* __restrict__ lin, int H, int W, int64_t N,
                                                           int64_t B, TileMap tm, int dilation_max,
                                                           unsigned long long* __restrict__ stats) {
    constexpr int F = 24, SC = 2 * R + 1;
    __shared__ uint2 box[6 * kBoxCap];
    __shared__ int red[16];
    // tile_pixel's XCD-banded order, keeping the lanes of a partial tile in the workgroup (barriers)
    const int64_t nblk = (int64_t)gridDim.x;
    const int64_t per = (nblk + 7) / 8;
    const int64_t lb = (int64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
    if (lb >= (int64_t)tm.ntiles * B) return;  // workgroup-uniform
    const int64_t b = lb / tm.ntiles;
    const int t = (int)(lb - b * tm.ntiles);
    const int ty = t / tm.tiles_x, tx = t - ty * tm.tiles_x;
    const int pu = tx * kTile + (threadIdx.x & (kTile - 1)), pv = ty * kTile + (threadIdx.x / kTile);
    const bool active = pu < W && pv < H;
    const int64_t g = b * (int64_t)H * W + (int64_t)pv * W + pu;
    const uint16_t* __restrict__ img = D11 + b * (int64_t)H * W * F;

    half2_t q2[F / 2];
    int64_t u0 = 0, v0 = 0;
    if (active) {
        const uint4* src = reinterpret_cast<const uint4*>(D21 + g * F);
#pragma unroll
        for (int c = 0; c < F / 8; c++) {
            const uint4 w = src[c];
            const half2_t* hp = reinterpret_cast<const half2_t*>(&w);
#pragma unroll
            for (int k = 0; k < 4; k++) q2[c * 4 + k] = hp[k];
        }
        u0 = p1[g * 2 + 0];
        v0 = p1[g * 2 + 1];
    }
    half_t max_score = (half_t)kRefineHalfMaxInit;
    int64_t u_new = u0, v_new = v0;
    unsigned n_global = 0;
    for (int d = dilation_max; d > 0; d--) {
        const int64_t rd = (int64_t)R * d;
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
        box_minmax4(w4, red);
        const int umin = w4[0], vmin = w4[2];
        const bool any = w4[0] <= w4[1];
        const int Rw = any ? w4[1] - w4[0] + 1 : 0, Rh = any ? w4[3] - w4[2] + 1 : 0;
        const bool fits = any && Rw * Rh <= kBoxCap;  // workgroup-uniform
        if (fits) {
            // stage: cell c = (r, x) of the box, 4 cells (12 x 16-B loads) in flight per lane
            const int n = Rw * Rh;
            const float inv = 1.0f / (float)Rw;
            for (int c0 = threadIdx.x; c0 < (DIAG == 1 ? 0 : n); c0 += 4 * kBlock) {
                uint4 v[4][3];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int c = min(c0 + k * kBlock, n - 1);
                    const int r = (int)(((float)c + 0.5f) * inv);
                    const uint4* src = reinterpret_cast<const uint4*>(
                        img + ((int64_t)(vmin + r) * W + umin + (c - r * Rw)) * F);
#pragma unroll
                    for (int q = 0; q < 3; q++) v[k][q] = src[q];
                }
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int c = c0 + k * kBlock;
                    if (c < n) {
#pragma unroll
                        for (int q = 0; q < 3; q++) {
                            box[(2 * q) * kBoxCap + c] = make_uint2(v[k][q].x, v[k][q].y);
                            box[(2 * q + 1) * kBoxCap + c] = make_uint2(v[k][q].z, v[k][q].w);
                        }
                    }
                }
            }
            __syncthreads();
            if (active && DIAG != 2) {
                uint4 ra[SC][3], rb[SC][3];
                bool oka[SC], okb[SC];
                auto fetch = [&](int i, uint4 (&rw)[SC][3], bool (&okk)[SC]) {
                    const int64_t u = u0 - rd + (int64_t)i * d;
#pragma unroll
                    for (int j = 0; j < SC; j++) {
                        const int64_t v = v0 - rd + (int64_t)j * d;
                        okk[j] = inside_image(u, v, W, H);
                        const int cell = okk[j] ? (int)(v - vmin) * Rw + (int)(u - umin) : 0;
#pragma unroll
                        for (int q = 0; q < 3; q++) {
                            const uint2 lo = box[(2 * q) * kBoxCap + cell];
                            const uint2 hi = box[(2 * q + 1) * kBoxCap + cell];
                            rw[j][q] = make_uint4(lo.x, lo.y, hi.x, hi.y);
                        }
                    }
                };
                auto consume = [&](int i, const uint4 (&rw)[SC][3], const bool (&okk)[SC]) {
                    half_t score[SC];
                    score_f16_multi<F, SC>(q2, rw, score);
                    const int64_t u = u0 - rd + (int64_t)i * d;
#pragma unroll
                    for (int j = 0; j < SC; j++) {  // v offset inner (matching_kernels.cu:55)
                        if (okk[j] && score[j] > max_score) {
                            max_score = score[j];
                            u_new = u;
                            v_new = v0 - rd + (int64_t)j * d;
                        }
                    }
                };
                fetch(0, ra, oka);
#pragma unroll
                for (int i = 0; i < SC; i += 2) {  // u offset outer (matching_kernels.cu:54)
                    if (i + 1 < SC) fetch(i + 1, rb, okb);
                    consume(i, ra, oka);
                    if (i + 1 < SC) {
                        if (i + 2 < SC) fetch(i + 2, ra, oka);
                        consume(i + 1, rb, okb);
                    }
                }
            }
            __syncthreads();  // the next level's staging overwrites the box
        } else if (active && any) {
            n_global++;
            for (int i = 0; i < SC; i++) {
                const int64_t u = u0 - rd + (int64_t)i * d;
                uint4 rows[SC][3];
                bool ok[SC];
#pragma unroll
                for (int j = 0; j < SC; j++) {
                    const int64_t v = v0 - rd + (int64_t)j * d;
                    ok[j] = inside_image(u, v, W, H);
                    const uint4* src = reinterpret_cast<const uint4*>(img + (ok[j] ? (v * W + u) * F : 0));
#pragma unroll
                    for (int q = 0; q < 3; q++) rows[j][q] = src[q];
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
            }
        }
        u0 = u_new;
        v0 = v_new;
    }
    if (active) store_match(p1_new, lin, g, W, u_new, v_new);
    if (stats && n_global) atomicAdd(stats + 2, (unsigned long long)n_global);  // diagnostics
}


// ---------------------------------------------------------------------------------
// refine_matches on a plane-major copy of D11 (M3S_REFINE_VARIANT_PLANES, round 5).
//
// The product kernel gathers a candidate's 48-B row as 3 dwordx4 loads; the 64 lanes of one load
// read 16 B from each of ~64 cells 48 B apart, so every load instruction touches all ~24-28 cache
// lines of the wave's candidate rows (the L1/TA path, not the VALU, bounds it: DESIGN.md section 4).
// Here D11 is first copied to 3 planes (plane q holds the 16-B piece q of every cell,
// contiguously: [B][3][H*W] x 16 B), so load q of a wave reads 64 consecutive-ish 16-B pieces:
// ~1/3 of the lines per instruction.  The copy is one pass over D11 (read 48 B + write 48 B per
// cell).  Same candidate order, same c10::Half chain (score_f16_multi) => the product's matches.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void d11_planes_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                          int64_t HW, int64_t total) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;  // cell (b, n)
    if (i >= total) return;
    const int64_t b = i / HW, n = i - b * HW;
    const uint4 a0 = src[3 * i], a1 = src[3 * i + 1], a2 = src[3 * i + 2];
    uint4* d = dst + b * 3 * HW + n;
    d[0] = a0;
    d[HW] = a1;
    d[2 * HW] = a2;
}

// (refine_planes_kernel: refine_common.h, shared with the fused matching op)

// Generic F (any descriptor width), fp16, f32 or f64 (AT_DISPATCH_FLOATING_TYPES_AND_HALF,
// matching_kernels.cu:103), scalar loads.
}  // namespace

// exactly re-scored / in-image candidates of the bound-and-rescore variants
static bool g_refine_stats_enabled = false;
static unsigned long long g_refine_stats[3] = {0, 0, 0};

extern "C" void m3s_refine_variant_stats(int enable, unsigned long long* out3) {
    if (out3) {
        for (int k = 0; k < 3; k++) out3[k] = g_refine_stats[k];
    }
    g_refine_stats_enabled = enable != 0;
    g_refine_stats[0] = g_refine_stats[1] = g_refine_stats[2] = 0;
}

extern "C" int m3s_refine_variant_f16(int variant, const uint16_t* D11, const uint16_t* D21, const int64_t* p1,
                                      int64_t* p1_new, int64_t B, int64_t H, int64_t W, int64_t N, int64_t F,
                                      int radius, int dilation_max, void* stream) {
    int rc = refine_checks(D11, D21, p1, p1_new, B, H, W, N, F, radius, dilation_max);
    if (rc) return rc;
    const int64_t total = B * N;
    if (total == 0) return M3S_OK;
    const bool aligned = ((uintptr_t)D11 % 16 == 0) && ((uintptr_t)D21 % 16 == 0);
    M3S_REQUIRE(F == 24 && aligned && N == H * W && radius == 3,
                "refine variant: needs F = 24, 16-B aligned descriptors, N = H*W and radius 3");
    M3S_REQUIRE(variant == M3S_REFINE_VARIANT_LDS || variant == M3S_REFINE_VARIANT_MFMA ||
                    variant == M3S_REFINE_VARIANT_DOT2 || variant == M3S_REFINE_VARIANT_LATTICE ||
                    variant == M3S_REFINE_VARIANT_BOX || variant == M3S_REFINE_VARIANT_PLANES,
                "refine variant: unknown kind %d", variant);
    M3S_REQUIRE(variant != M3S_REFINE_VARIANT_LATTICE || dilation_max <= kLatMaxD,
                "refine variant: the lattice kernel handles dilation_max <= %d", kLatMaxD);
    hipStream_t st = (hipStream_t)stream;
    int64_t* lin = nullptr;
    if (variant == M3S_REFINE_VARIANT_PLANES) {
        TileMap tm;
        tm.tiles_x = (int)((W + kTile - 1) / kTile);
        tm.tiles_y = (int)((H + kTile - 1) / kTile);
        tm.ntiles = tm.tiles_x * tm.tiles_y;
        const int64_t nblk = (int64_t)tm.ntiles * B;
        const int64_t grid = (nblk + 7) / 8 * 8;
        const int64_t cells = B * H * W;
        uint4* planes = nullptr;
        M3S_HIP_CHECK(hipMallocAsync((void**)&planes, sizeof(uint4) * 3 * (size_t)cells, st));
        hipLaunchKernelGGL(d11_planes_kernel, dim3((unsigned)((cells + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                           reinterpret_cast<const uint4*>(D11), planes, H * W, cells);
        hipLaunchKernelGGL((refine_planes_kernel<3>), dim3((unsigned)grid), dim3(kBlock), 0, st, planes, D21, p1,
                           p1_new, lin, (int)H, (int)W, N, B, tm, dilation_max);
        M3S_LAUNCH_CHECK();
        M3S_HIP_CHECK(hipFreeAsync(planes, st));
        return M3S_OK;
    }
    if (variant == M3S_REFINE_VARIANT_BOX) {
        TileMap tm;
        tm.tiles_x = (int)((W + kTile - 1) / kTile);
        tm.tiles_y = (int)((H + kTile - 1) / kTile);
        tm.ntiles = tm.tiles_x * tm.tiles_y;
        const int64_t nblk = (int64_t)tm.ntiles * B;
        const int64_t grid = (nblk + 7) / 8 * 8;
        // M3S_BOX_DIAG (diagnostics, wrong matches): 1 = no staging loads, 2 = no scoring
        static const int diag = [] {
            const char* e = getenv("M3S_BOX_DIAG");
            return e ? atoi(e) : 0;
        }();
        if (diag == 1)
            hipLaunchKernelGGL((refine_box_kernel<3, 1>), dim3((unsigned)grid), dim3(kBlock), 0, st, D11, D21, p1,
                               p1_new, lin, (int)H, (int)W, N, B, tm, dilation_max, (unsigned long long*)nullptr);
        else if (diag == 2)
            hipLaunchKernelGGL((refine_box_kernel<3, 2>), dim3((unsigned)grid), dim3(kBlock), 0, st, D11, D21, p1,
                               p1_new, lin, (int)H, (int)W, N, B, tm, dilation_max, (unsigned long long*)nullptr);
        else
            hipLaunchKernelGGL((refine_box_kernel<3>), dim3((unsigned)grid), dim3(kBlock), 0, st, D11, D21, p1, p1_new,
                               lin, (int)H, (int)W, N, B, tm, dilation_max, (unsigned long long*)nullptr);
        M3S_LAUNCH_CHECK();
        return M3S_OK;
    }
    if (variant != M3S_REFINE_VARIANT_LDS) {
        TileMap tm;
        tm.tiles_x = (int)((W + kTile - 1) / kTile);
        tm.tiles_y = (int)((H + kTile - 1) / kTile);
        tm.ntiles = tm.tiles_x * tm.tiles_y;
        const int64_t nblk = (int64_t)tm.ntiles * B;
        const int64_t grid = (nblk + 7) / 8 * 8;
        // per-image max ||h||^2 (+ the optional re-score counters), stream-ordered scratch
        unsigned* scratch = nullptr;
        const size_t sbytes = sizeof(unsigned) * (size_t)B + 3 * sizeof(unsigned long long) + 16;
        M3S_HIP_CHECK(hipMallocAsync((void**)&scratch, sbytes, st));
        M3S_HIP_CHECK(hipMemsetAsync(scratch, 0, sbytes, st));
        unsigned long long* stats = reinterpret_cast<unsigned long long*>(
            reinterpret_cast<char*>(scratch) + ((sizeof(unsigned) * (size_t)B + 15) / 16 * 16));
        unsigned long long* st_arg = g_refine_stats_enabled ? stats : nullptr;
        const int64_t HW = H * W;
        const unsigned hb = (unsigned)std::min<int64_t>((HW + kBlock - 1) / kBlock, 1024);
        hipLaunchKernelGGL(refine_hmax_kernel, dim3(hb, (unsigned)B), dim3(kBlock), 0, st, D11, HW, scratch);
        if (variant == M3S_REFINE_VARIANT_LATTICE)
            hipLaunchKernelGGL((refine_lattice_kernel<3>), dim3((unsigned)grid), dim3(kBlock), 0, st, D11, D21, p1,
                               p1_new, lin, (int)H, (int)W, N, B, tm, dilation_max, scratch, st_arg);
        else if (variant == M3S_REFINE_VARIANT_MFMA)
            hipLaunchKernelGGL((refine_mfma_kernel<3>), dim3((unsigned)grid), dim3(kBlock), 0, st, D11, D21, p1,
                               p1_new, lin, (int)H, (int)W, N, B, tm, dilation_max, scratch, st_arg);
        else
            hipLaunchKernelGGL((refine_dot2_kernel<3>), dim3((unsigned)grid), dim3(kBlock), 0, st, D11, D21, p1,
                               p1_new, lin, (int)H, (int)W, N, B, tm, dilation_max, scratch, st_arg);
        M3S_LAUNCH_CHECK();
        if (g_refine_stats_enabled) {
            unsigned long long h[3];
            M3S_HIP_CHECK(hipMemcpyAsync(h, stats, sizeof(h), hipMemcpyDeviceToHost, st));
            M3S_HIP_CHECK(hipStreamSynchronize(st));
            for (int k = 0; k < 3; k++) g_refine_stats[k] += h[k];
        }
        M3S_HIP_CHECK(hipFreeAsync(scratch, st));
    } else {
        LdsTileMap tm;
        tm.tiles_x = (int)((W + kLdsTx - 1) / kLdsTx);
        tm.tiles_y = (int)((H + kLdsTy - 1) / kLdsTy);
        tm.ntiles = tm.tiles_x * tm.tiles_y;
        const int64_t nblk = (int64_t)tm.ntiles * B;
        const int64_t grid = (nblk + 7) / 8 * 8;
        hipLaunchKernelGGL((refine_lds_kernel<24, 3>), dim3((unsigned)grid), dim3(kLdsThreads), 0, st, D11,
                           D21, p1, p1_new, lin, (int)H, (int)W, B, tm, dilation_max, (int*)nullptr);
        M3S_LAUNCH_CHECK();
    }
    return M3S_OK;
}
