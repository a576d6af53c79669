// gn_kernels.hip -- MI355X (gfx950) kernels of the Sim3 Gauss-Newton backend.
//
// Per GN iteration (driver in gn_driver.hip), after the accumulate of gn_accum.hip:
//   gn_edge_reduce_kernel   per directed edge: chunk partials summed in f64 (fixed order),
//                           Hjj = A M A^T, vj = A g with A = the Sim3 adjoint map of
//                           apply_Sim3_adj_inv (gn_kernels.cu:277-297).  Because
//                           Ji = -Jj (gn_kernels.cu:1000) the reference's four blocks are
//                           Hii = Hjj, Hij = Hji = -Hjj, vi = -vj.
//   gn_compact_kernel       deterministic CSR sum of edge blocks into the compact
//                           block-sparse system (the RCCL all-reduce payload).
//   gn_fill_dense_kernel    compact -> dense f64 lower system + RHS border row.
//   chol_panel / chol_update / back_step   blocked right-looking LL^T in f64 (T = 64),
//                           SimplicialLLT failure semantics (pivot <= 0 => dx = 0).
//   gn_retract_kernel       dx = -x, left retraction (gn_kernels.cu:415-453), ||dx|| test.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "edge_reduce.h"
#include "gn_kernels.h"
#include "sim3.h"

namespace m3s {

// ---------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------

// Per local edge: f64 chunk sum (fixed order), Hjj = A M A^T, vj = A g (edge_reduce.h).
__global__ __launch_bounds__(64) void gn_edge_reduce_kernel(const float* __restrict__ partials,
                                                            int nchunks,
                                                            const float* __restrict__ Twc,
                                                            const int* __restrict__ ii_loc,
                                                            double* __restrict__ edgeblk,
                                                            const int* __restrict__ flags) {
    if (flags[kFlagDone]) return;
    edge_reduce_body<false>(partials, nchunks, Twc, ii_loc, edgeblk, blockIdx.x);
}

// Compact block-sparse system: slots [0, nblk) hold 28 doubles each, followed by the
// gradient (N-1)*7.  One 64-lane workgroup per block slot / gradient row.
__global__ __launch_bounds__(64) void gn_compact_kernel(
    const double* __restrict__ edgeblk, const int* __restrict__ blk_ptr,
    const int* __restrict__ blk_ent, const int* __restrict__ grad_ptr,
    const int* __restrict__ grad_ent, int nblk, int npose, double* __restrict__ compact,
    const int* __restrict__ flags) {
    if (flags[kFlagDone]) return;
    const int s = blockIdx.x;
    const int tid = threadIdx.x;
    if (s < nblk) {
        if (tid < 28) {
            // entries in batches of 8 (codes, then values in flight together), summed in entry
            // order as before
            double acc = 0.0;
            const int k1 = blk_ptr[s + 1];
            for (int k = blk_ptr[s]; k < k1; k += 8) {
                int code[8];
                double v[8];
#pragma unroll
                for (int u = 0; u < 8; u++) code[u] = k + u < k1 ? blk_ent[k + u] : 0;
#pragma unroll
                for (int u = 0; u < 8; u++) v[u] = k + u < k1 ? edgeblk[(int64_t)(code[u] >> 1) * kEdgeBlk + tid] : 0.0;
#pragma unroll
                for (int u = 0; u < 8; u++)
                    if (k + u < k1) acc += (code[u] & 1) ? -v[u] : v[u];
            }
            compact[(int64_t)s * 28 + tid] = acc;
        }
    } else {
        const int p = s - nblk;
        if (p < npose && tid < 7) {
            double acc = 0.0;
            const int k1 = grad_ptr[p + 1];
            for (int k = grad_ptr[p]; k < k1; k += 8) {
                int code[8];
                double v[8];
#pragma unroll
                for (int u = 0; u < 8; u++) code[u] = k + u < k1 ? grad_ent[k + u] : 0;
#pragma unroll
                for (int u = 0; u < 8; u++) v[u] = k + u < k1 ? edgeblk[(int64_t)(code[u] >> 1) * kEdgeBlk + 28 + tid] : 0.0;
#pragma unroll
                for (int u = 0; u < 8; u++)
                    if (k + u < k1) acc += (code[u] & 1) ? -v[u] : v[u];
            }
            compact[(int64_t)nblk * 28 + p * 7 + tid] = acc;
        }
    }
}

// Block-format system of the sparse solve (gn_solve.hip), written in place of the compact
// one: out = [b (npose x 7, zero-padded to bpad)] [nblk real blocks, 49 f64 row-major (the
// symmetric 7x7 expanded)] [nblocks - nblk fill blocks, zeroed].  The RCCL all-reduce covers
// the first bpad + 49 nblk doubles.  One 64-lane workgroup per block / gradient row.
__global__ __launch_bounds__(64) void gn_assemble_kernel(
    const double* __restrict__ edgeblk, const int* __restrict__ blk_ptr,
    const int* __restrict__ blk_ent, const int* __restrict__ grad_ptr,
    const int* __restrict__ grad_ent, int nblk, int nblocks, int npose, int bpad,
    double* __restrict__ out, const int* __restrict__ flags) {
    if (flags[kFlagDone]) return;
    const int s = blockIdx.x;
    const int tid = threadIdx.x;
    if (s < nblk) {
        if (tid < 28) {
            // entries in batches of 8 (codes, then values in flight together), summed in entry
            // order as before
            double acc = 0.0;
            const int k1 = blk_ptr[s + 1];
            for (int k = blk_ptr[s]; k < k1; k += 8) {
                int code[8];
                double v[8];
#pragma unroll
                for (int u = 0; u < 8; u++) code[u] = k + u < k1 ? blk_ent[k + u] : 0;
#pragma unroll
                for (int u = 0; u < 8; u++) v[u] = k + u < k1 ? edgeblk[(int64_t)(code[u] >> 1) * kEdgeBlk + tid] : 0.0;
#pragma unroll
                for (int u = 0; u < 8; u++)
                    if (k + u < k1) acc += (code[u] & 1) ? -v[u] : v[u];
            }
            int a = 0, r = tid;
            while (r >= 7 - a) {
                r -= 7 - a;
                a++;
            }
            const int b = a + r;
            double* blk = out + bpad + (int64_t)s * 49;
            blk[a * 7 + b] = acc;
            blk[b * 7 + a] = acc;
        }
    } else if (s < nblocks) {
        if (tid < 49) out[bpad + (int64_t)s * 49 + tid] = 0.0;
    } else {
        const int p = s - nblocks;
        if (p < npose && tid < 7) {
            double acc = 0.0;
            const int k1 = grad_ptr[p + 1];
            for (int k = grad_ptr[p]; k < k1; k += 8) {
                int code[8];
                double v[8];
#pragma unroll
                for (int u = 0; u < 8; u++) code[u] = k + u < k1 ? grad_ent[k + u] : 0;
#pragma unroll
                for (int u = 0; u < 8; u++) v[u] = k + u < k1 ? edgeblk[(int64_t)(code[u] >> 1) * kEdgeBlk + 28 + tid] : 0.0;
#pragma unroll
                for (int u = 0; u < 8; u++)
                    if (k + u < k1) acc += (code[u] & 1) ? -v[u] : v[u];
            }
            out[p * 7 + tid] = acc;
        }
    }
}

// Dense f64 matrix [npad + T rows][npad cols]: system in rows < npad (identity on the
// padding), RHS b in row npad (the bordered row: the forward solve rides along with the
// factorisation).
__global__ __launch_bounds__(256) void gn_fill_dense_kernel(const double* __restrict__ compact,
                                                            const int* __restrict__ slotmap,
                                                            int nblk, int npose, int n, int npad,
                                                            double* __restrict__ Hd,
                                                            const int* __restrict__ flags) {
    if (solve_skipped(flags)) return;
    const int64_t total = (int64_t)(npad + kCholTile) * npad;
    for (int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; id < total;
         id += (int64_t)gridDim.x * blockDim.x) {
        const int r = (int)(id / npad), c = (int)(id % npad);
        double val;
        if (r > npad) {
            val = 0.0;  // unused rows of the border tile
        } else if (r == npad) {
            val = c < n ? compact[(int64_t)nblk * 28 + c] : 0.0;
        } else if (r < n && c < n) {
            const int br = r / 7, bc = c / 7;
            const int slot = slotmap[(int64_t)br * npose + bc];
            const int a = r % 7, b = c % 7;
            val = slot >= 0 ? compact[(int64_t)slot * 28 + (a <= b ? sym_idx(a, b) : sym_idx(b, a))]
                            : 0.0;
        } else {
            val = (r == c) ? 1.0 : 0.0;
        }
        Hd[id] = val;
    }
}

// ---- blocked Cholesky, T = 64 --------------------------------------------------
//
// Right-looking tile LL^T of the dense f64 system (rows < npad) with the RHS as a border
// row (row npad), so the forward substitution y = L^{-1} b rides along.  Per panel k:
//   chol_potrf_kernel  (1 WG)      : L_kk and its inverse Li_k (doubling) in LDS
//   chol_trsm_kernel   (nt-k WGs)  : L_ik = A_ik Li_k^T as a 64^3 GEMM (tile nt = border)
//   chol_update_kernel (tiles)     : A_ij -= L_ik L_jk^T
// then chol_backsolve_kernel (1 WG) solves L^T x = y with the stored Li_k.

constexpr int T = kCholTile;

// 1/d to ~1 ulp: v_rcp_f64 + two Newton steps (the solve is not a bit-exact path).
__device__ __forceinline__ double rcp_f64(double d) {
    double r = __builtin_amdgcn_rcp(d);
    r = r * (2.0 - d * r);
    r = r * (2.0 - d * r);
    return r;
}

// potrf of one 64x64 tile + its inverse, one 1024-thread workgroup, LDS-resident.
// Blocked in 8-column sub-panels (16 barriers instead of 64):
//   phase 1 (one wave, lane = row): every lane factors the 8x8 diagonal block in registers
//            (redundantly -- no cross-lane traffic) and solves its own row of the panel;
//   phase 2 (all threads): rank-8 trailing update of the lower triangle.
// Then Li = L^{-1} by doubling, [[A,0],[B,C]]^{-1} = [[Ai,0],[-Ci B Ai, Ci]] (12 barriers).
constexpr int kPotrfThreads = 512;
constexpr int LDP = T + 1;

__device__ __forceinline__ double rsqrt_f64(double d) {
    double r = __builtin_amdgcn_rsq(d);
    r = r * (1.5 - 0.5 * d * r * r);
    r = r * (1.5 - 0.5 * d * r * r);
    return r;
}

template <int S>
__device__ __forceinline__ void inverse_stage(const double (*L)[LDP], double (*Li)[LDP],
                                              double (*Tm)[LDP], int tid) {
    constexpr int P = T / (2 * S);
    constexpr int NOUT = P * S * S;
    // Tm = B Ai   (B = L[p+S.., p..], Ai lower)
    for (int id = tid; id < NOUT; id += kPotrfThreads) {
        const int pi = id / (S * S), rem = id % (S * S);
        const int a = rem / S, bb = rem % S;
        const int p = pi * 2 * S;
        double acc = 0.0;
#pragma unroll
        for (int m = 0; m < S; m++)
            if (m >= bb) acc = fma(L[p + S + a][p + m], Li[p + m][p + bb], acc);
        Tm[p + S + a][p + bb] = acc;
    }
    __syncthreads();
    // Li[p+S.., p..] = -Ci Tm
    for (int id = tid; id < NOUT; id += kPotrfThreads) {
        const int pi = id / (S * S), rem = id % (S * S);
        const int a = rem / S, bb = rem % S;
        const int p = pi * 2 * S;
        double acc = 0.0;
#pragma unroll
        for (int m = 0; m < S; m++)
            if (m <= a) acc = fma(Li[p + S + a][p + S + m], Tm[p + S + m][p + bb], acc);
        Li[p + S + a][p + bb] = -acc;
    }
    __syncthreads();
}

__global__ __launch_bounds__(kPotrfThreads) void chol_potrf_kernel(double* __restrict__ Hd,
                                                                   int npad, int k,
                                                                   double* __restrict__ Linv,
                                                                   int* __restrict__ flags) {
    if (solve_skipped(flags)) return;
    __shared__ double A[T][LDP];
    __shared__ double Li[T][LDP];
    __shared__ double Tm[T][LDP];
    __shared__ int fail;
    const int tid = threadIdx.x;
    double* Akk = Hd + (int64_t)k * T * npad + (int64_t)k * T;
    for (int id = tid; id < T * T; id += kPotrfThreads) {
        const int r = id >> 6, c = id & 63;
        A[r][c] = (c <= r) ? Akk[(int64_t)r * npad + c] : 0.0;
        Li[r][c] = 0.0;
    }
    if (tid == 0) fail = 0;
    __syncthreads();
    const int tx = tid & 31, ty = tid >> 5;  // ty in [0, 16)
    for (int s = 0; s < T / 8; s++) {
        const int c0 = 8 * s;
        if (tid < T && tid >= c0) {
            const int r = tid;
            // all LDS operands first (one latency), then register-only math
            double D[8][8], arow[8];
#pragma unroll
            for (int i = 0; i < 8; i++)
#pragma unroll
                for (int p = 0; p <= i; p++) D[i][p] = A[c0 + i][c0 + p];
#pragma unroll
            for (int p = 0; p < 8; p++) arow[p] = A[r][c0 + p];
            // right-looking in registers: per pivot one rsq + one Newton step, then independent
            // column scalings and trailing updates (dependent depth O(8), not O(8^2)); 1/l_pp is
            // the pivot's rsqrt, so the row solve needs no reciprocal
            double l[8][8], inv[8];
            bool bad = false;
#pragma unroll
            for (int p = 0; p < 8; p++) {
                const double dpp = D[p][p];
                if (dpp <= 0.0) bad = true;  // SimplicialLLT: fails iff a pivot <= 0
                double y = __builtin_amdgcn_rsq(dpp);
                y = y * fma(-0.5 * dpp * y, y, 1.5);
                inv[p] = y;
                l[p][p] = dpp * y;
#pragma unroll
                for (int i = p + 1; i < 8; i++) l[i][p] = D[i][p] * y;
#pragma unroll
                for (int i = p + 1; i < 8; i++)
#pragma unroll
                    for (int j = p + 1; j <= i; j++) D[i][j] = fma(-l[i][p], l[j][p], D[i][j]);
            }
            if (r < c0 + 8) {
                const int i = r - c0;
#pragma unroll
                for (int ii = 0; ii < 8; ii++) {
                    if (ii == i) {
#pragma unroll
                        for (int p = 0; p <= ii; p++) A[r][c0 + p] = l[ii][p];
                    }
                }
                if (bad && r == c0) fail = 1;
            } else {
#pragma unroll
                for (int p = 0; p < 8; p++) {
                    const double xp = arow[p] * inv[p];
                    arow[p] = xp;
#pragma unroll
                    for (int i = p + 1; i < 8; i++) arow[i] = fma(-xp, l[i][p], arow[i]);
                }
#pragma unroll
                for (int p = 0; p < 8; p++) A[r][c0 + p] = arow[p];
            }
        }
        __syncthreads();
        // rank-8 update of the lower trailing block (rows/cols >= c0 + 8)
        const int lo = c0 + 8;
#pragma unroll
        for (int a = 0; a < 4; a++) {
            const int r = ty + 16 * a;
#pragma unroll
            for (int b = 0; b < 2; b++) {
                const int cc = tx + 32 * b;
                if (cc >= lo && cc <= r) {
                    double acc = A[r][cc];
#pragma unroll
                    for (int p = 0; p < 8; p++) acc = fma(-A[r][c0 + p], A[cc][c0 + p], acc);
                    A[r][cc] = acc;
                }
            }
        }
        __syncthreads();
    }
    // inverse by doubling
    if (tid < T) Li[tid][tid] = 1.0 / A[tid][tid];
    __syncthreads();
    inverse_stage<1>(A, Li, Tm, tid);
    inverse_stage<2>(A, Li, Tm, tid);
    inverse_stage<4>(A, Li, Tm, tid);
    inverse_stage<8>(A, Li, Tm, tid);
    inverse_stage<16>(A, Li, Tm, tid);
    inverse_stage<32>(A, Li, Tm, tid);
    double* Lk = Linv + (int64_t)k * T * T;
    for (int id = tid; id < T * T; id += kPotrfThreads) {
        const int r = id >> 6, c = id & 63;
        if (c <= r) Akk[(int64_t)r * npad + c] = A[r][c];
        Lk[id] = (c <= r) ? Li[r][c] : 0.0;
    }
    if (fail && tid == 0) flags[kFlagFail] = 1;
}

// 64x64x64 tile product from LDS (row stride LD2 doubles, 16-B aligned rows): 512 threads,
// each a 4 (rows) x 2 (cols) block, m consumed in pairs (ds_read_b128).
constexpr int LD2 = T + 2;
constexpr int kGemmThreads = 512;
__device__ __forceinline__ void tile_nt(const double (*X)[LD2], const double (*Y)[LD2], int r0,
                                        int c0, double acc[4][2]) {
#pragma unroll 4
    for (int m = 0; m < T; m += 2) {
        double2 xa[4], yb[2];
#pragma unroll
        for (int a = 0; a < 4; a++) xa[a] = *reinterpret_cast<const double2*>(&X[r0 + a][m]);
#pragma unroll
        for (int b = 0; b < 2; b++) yb[b] = *reinterpret_cast<const double2*>(&Y[c0 + b][m]);
#pragma unroll
        for (int a = 0; a < 4; a++)
#pragma unroll
            for (int b = 0; b < 2; b++) {
                acc[a][b] = fma(xa[a].x, yb[b].x, acc[a][b]);
                acc[a][b] = fma(xa[a].y, yb[b].y, acc[a][b]);
            }
    }
}

__device__ __forceinline__ void load_tile(double (*dst)[LD2], const double* __restrict__ src,
                                          int64_t ld, int tid) {
#pragma unroll 4
    for (int id = tid; id < T * T / 2; id += kGemmThreads) {
        const int r = id >> 5, c2 = (id & 31) * 2;
        *reinterpret_cast<double2*>(&dst[r][c2]) =
            *reinterpret_cast<const double2*>(src + (int64_t)r * ld + c2);
    }
}

// L_ik = A_ik Li_k^T for tile rows i = k+1 .. nt (nt = the RHS border tile).
__global__ __launch_bounds__(kGemmThreads) void chol_trsm_kernel(double* __restrict__ Hd, int npad,
                                                                 int k,
                                                                 const double* __restrict__ Linv,
                                                                 const int* __restrict__ flags) {
    if (solve_skipped(flags)) return;
    __shared__ __attribute__((aligned(16))) double Xs_[T][LD2];
    __shared__ __attribute__((aligned(16))) double Li[T][LD2];
    const int tid = threadIdx.x;
    const int i = k + 1 + blockIdx.x;
    double* Aik = Hd + (int64_t)i * T * npad + (int64_t)k * T;
    load_tile(Xs_, Aik, npad, tid);
    load_tile(Li, Linv + (int64_t)k * T * T, T, tid);
    __syncthreads();
    const int r0 = (tid >> 5) * 4, c0 = (tid & 31) * 2;
    double acc[4][2] = {};
    tile_nt(Xs_, Li, r0, c0, acc);
#pragma unroll
    for (int a = 0; a < 4; a++)
        *reinterpret_cast<double2*>(Aik + (int64_t)(r0 + a) * npad + c0) =
            make_double2(acc[a][0], acc[a][1]);
}

// Trailing update after panel k: A_ij -= L_ik L_jk^T for k < j <= i <= nt, j < nt.
__global__ __launch_bounds__(kGemmThreads) void chol_update_kernel(double* __restrict__ Hd,
                                                                   int npad, int nt, int k,
                                                                   const int* __restrict__ flags) {
    if (solve_skipped(flags)) return;
    __shared__ __attribute__((aligned(16))) double Li[T][LD2];
    __shared__ __attribute__((aligned(16))) double Lj[T][LD2];
    int rem = blockIdx.x;  // -> (i, j): j = k+1.., i = j..nt
    int j = k + 1;
    while (rem >= nt - j + 1) { rem -= nt - j + 1; j++; }
    const int i = j + rem;
    const int tid = threadIdx.x;
    load_tile(Li, Hd + (int64_t)i * T * npad + (int64_t)k * T, npad, tid);
    load_tile(Lj, Hd + (int64_t)j * T * npad + (int64_t)k * T, npad, tid);
    __syncthreads();
    const int r0 = (tid >> 5) * 4, c0 = (tid & 31) * 2;
    double acc[4][2] = {};
    tile_nt(Li, Lj, r0, c0, acc);
    double* Aij = Hd + (int64_t)i * T * npad + (int64_t)j * T;
#pragma unroll
    for (int a = 0; a < 4; a++) {
        double2* p = reinterpret_cast<double2*>(Aij + (int64_t)(r0 + a) * npad + c0);
        double2 o = *p;
        o.x -= acc[a][0];
        o.y -= acc[a][1];
        *p = o;
    }
}

// L^T x = y (y = forward-substituted border row), one 1024-thread workgroup:
// for k = nt-1..0: x_k = Li_k^T y_k, then y_j -= L_kj^T x_k for every column left of k.
constexpr int kBackThreads = 1024;
constexpr int kMaxNpadBack = 8192;

__global__ __launch_bounds__(kBackThreads) void chol_backsolve_kernel(
    const double* __restrict__ Hd, int npad, const double* __restrict__ Linv,
    double* __restrict__ x, const int* __restrict__ flags) {
    if (solve_skipped(flags)) return;
    __shared__ double y[kMaxNpadBack];
    __shared__ double Li[T][T + 1];
    __shared__ double part[16][T];
    __shared__ double xk[T];
    const int tid = threadIdx.x;
    const int nt = npad / T;
    const double* yrow = Hd + (int64_t)npad * npad;
    for (int c = tid; c < npad; c += kBackThreads) y[c] = yrow[c];
    {
        const double* Lk = Linv + (int64_t)(nt - 1) * T * T;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int id = tid + q * kBackThreads;
            Li[id >> 6][id & 63] = Lk[id];
        }
    }
    for (int k = nt - 1; k >= 0; k--) {
        __syncthreads();
        {   // x_k[c] = sum_r Li[r][c] y_k[r]: 16 partial sums of 4 rows per column
            const int c = tid & 63, g = tid >> 6;
            double acc = 0.0;
#pragma unroll
            for (int q = 0; q < 4; q++) acc += Li[g * 4 + q][c] * y[k * T + g * 4 + q];
            part[g][c] = acc;
        }
        __syncthreads();
        if (tid < T) {
            double acc = 0.0;
#pragma unroll
            for (int g = 0; g < 16; g++) acc += part[g][tid];
            xk[tid] = acc;
            x[k * T + tid] = acc;
        }
        __syncthreads();
        // the next step's tile inverse in flight (registers) during the row-panel update, then
        // into LDS (its reads of this step's inverse are behind the barrier above)
        double lnext[4];
        if (k > 0) {
            const double* Ln = Linv + (int64_t)(k - 1) * T * T;
#pragma unroll
            for (int q = 0; q < 4; q++) lnext[q] = Ln[tid + q * kBackThreads];
        }
        const double* Lrow = Hd + (int64_t)k * T * npad;  // row panel k: tiles (k, j<k)
        for (int c = tid; c < k * T; c += kBackThreads) {
            double acc[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 16
            for (int b = 0; b < T; b++) acc[b & 3] = fma(Lrow[(int64_t)b * npad + c], xk[b], acc[b & 3]);
            y[c] -= (acc[0] + acc[1]) + (acc[2] + acc[3]);
        }
        if (k > 0) {
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int id = tid + q * kBackThreads;
                Li[id >> 6][id & 63] = lnext[q];
            }
        }
    }
}

// dx = -x (or 0 if the factorisation failed), in-place retraction of poses 1..N-1,
// ||dx|| < delta_thresh => done (gn_kernels.cu:1209-1222).
__global__ __launch_bounds__(256) void gn_retract_kernel(float* __restrict__ Twc,
                                                         const double* __restrict__ x,
                                                         float* __restrict__ dx, int N,
                                                         float delta_thresh,
                                                         int* __restrict__ flags, int contract) {
    if (solve_skipped(flags)) return;
    const int tid = threadIdx.x;
    const bool fail = flags[kFlagFail] != 0;
    double nrm = 0.0;
    for (int p = 1 + tid; p < N; p += blockDim.x) {
        float xi[7];
#pragma unroll
        for (int q = 0; q < 7; q++) {
            const float v = fail ? 0.0f : -(float)x[(int64_t)(p - 1) * 7 + q];
            xi[q] = v;
            dx[(int64_t)(p - 1) * 7 + q] = v;
            nrm += (double)v * (double)v;
        }
        retr_sim3_cm(contract, xi, Twc + (int64_t)p * 8);
    }
    __shared__ double red[256];
    red[tid] = nrm;
    __syncthreads();
    for (int s = 128; s >= 1; s >>= 1) {
        if (tid < s) red[tid] += red[tid + s];
        __syncthreads();
    }
    if (tid == 0) {
        flags[kFlagFail] = 0;
        if ((float)sqrt(red[0]) < delta_thresh) flags[kFlagDone] = 1;
    }
}

// Per-call plan upload: the device reads the pinned host image itself (16 B per lane, 4 B
// for a ragged end).  A hipMemcpyAsync H2D is carried out by a DMA engine, whose handshake with
// the kernel queue left the GPU idle ~100 us around every mid-stream plan upload (rocprofv3
// kernel trace).
__global__ __launch_bounds__(256) void stage_copy_kernel(const uint32_t* __restrict__ src,
                                                         uint32_t* __restrict__ dst, int64_t n4) {
    const int64_t n16 = n4 >> 2;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint4* s16 = reinterpret_cast<const uint4*>(src);
    uint4* d16 = reinterpret_cast<uint4*>(dst);
    for (int64_t i = t0; i < n16; i += stride) d16[i] = s16[i];
    for (int64_t i = 4 * n16 + t0; i < n4; i += stride) dst[i] = src[i];
}

// The call's timeout flag, exported without a host wait: as an int (to pinned host memory, by
// its device address) or as 0.0 / 1.0 (a device word the ranks then sum).
__global__ void flag_export_kernel(const int* __restrict__ flag, void* dst, int as_f64) {
    if (threadIdx.x == 0) {
        const int v = flag[0] != 0 ? 1 : 0;
        if (as_f64) *static_cast<double*>(dst) = (double)v;
        else *static_cast<int*>(dst) = v;
    }
}

// A timed-out call never commits its poses: Twc is saved before the call's first
// retraction (mode 0) and restored at its end when the call's timeout flag -- the rank-local int,
// or the ranks' sum as a double -- is set (mode 1), which then also exports the flag to dst (an
// int, or the double as is) when dst is not null.  All on the device: no host wait.
__global__ __launch_bounds__(256) void twc_guard_kernel(float* __restrict__ Twc, float* __restrict__ save, int n,
                                                        int mode, const void* flag, int flag_f64, void* dst) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (mode == 0) {
        if (i < n) save[i] = Twc[i];
        return;
    }
    const double f = flag_f64 ? *static_cast<const double*>(flag) : (double)*static_cast<const int*>(flag);
    if (f > 0.0 && i < n) Twc[i] = save[i];
    if (dst && i == 0) {
        if (flag_f64) *static_cast<double*>(dst) = f;
        else *static_cast<int*>(dst) = f > 0.0 ? 1 : 0;
    }
}

// ---------------------------------------------------------------------------
// launchers (host)
// ---------------------------------------------------------------------------

hipError_t launch_flag_export(hipStream_t st, const int* flag, void* dst, int as_f64) {
    hipLaunchKernelGGL(flag_export_kernel, dim3(1), dim3(64), 0, st, flag, dst, as_f64);
    return hipGetLastError();
}

hipError_t launch_twc_save(hipStream_t st, const float* Twc, float* save, int n) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(twc_guard_kernel, dim3((n + 255) / 256), dim3(256), 0, st, const_cast<float*>(Twc), save,
                       n, 0, nullptr, 0, nullptr);
    return hipGetLastError();
}

hipError_t launch_twc_restore_on_flag(hipStream_t st, float* Twc, const float* save, int n, const void* flag,
                                      int flag_f64, void* dst) {
    hipLaunchKernelGGL(twc_guard_kernel, dim3(n > 0 ? (n + 255) / 256 : 1), dim3(256), 0, st, Twc,
                       const_cast<float*>(save), n, 1, flag, flag_f64, dst);
    return hipGetLastError();
}

// record t: with full = 8 q nchunks, t < full is (k, g) = (t / 8, t % 8) -- every group still has
// tasks -- and past it only the groups with q + 1 edges remain, in ascending order
__global__ __launch_bounds__(256) void sched_expand_kernel(const int* __restrict__ order, const int* __restrict__ ii_loc,
                                                           const int* __restrict__ jj_loc, int nchunks, SchedGroups G,
                                                           int64_t ntask, int4* __restrict__ rec) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntask) return;
    int e, c;
    if (G.off) {
        e = (int)(t / nchunks);
        c = (int)(t % nchunks);
    } else {
        const int64_t full = 8 * (int64_t)G.q * nchunks;
        int64_t k;
        int g;
        if (t < full) {
            k = t >> 3;
            g = (int)(t & 7);
        } else {
            const int64_t r = t - full;
            k = (int64_t)G.q * nchunks + r / G.nbig;
            g = G.big[r % G.nbig];
        }
        e = order[G.lo[g] + (int)(k % G.n[g])];
        c = (int)(k / G.n[g]);
    }
    rec[t] = make_int4(e, c, ii_loc[e], jj_loc[e]);
}

hipError_t launch_sched_expand(hipStream_t st, const int* order, const int* ii_loc, const int* jj_loc,
                               int nchunks, const SchedGroups& G, int64_t ntask, int* rec) {
    if (ntask <= 0) return hipSuccess;
    if (((uintptr_t)rec & 15) != 0) return hipErrorInvalidValue;
    const int64_t blocks = (ntask + 255) / 256;
    hipLaunchKernelGGL(sched_expand_kernel, dim3((unsigned)blocks), dim3(256), 0, st, order, ii_loc, jj_loc,
                       nchunks, G, ntask, reinterpret_cast<int4*>(rec));
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void gn_init_kernel(int* __restrict__ flags, int not_ray, int* __restrict__ cok,
                                                      int64_t n) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < kNumFlags) flags[t] = t == kFlagNotRay ? not_ray : 0;
    if (t < n) cok[t] = 1;
}

hipError_t launch_gn_init(hipStream_t st, int* flags, int not_ray, int* cok, int64_t n) {
    const int64_t m = std::max<int64_t>(n, kNumFlags);
    hipLaunchKernelGGL(gn_init_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, flags, not_ray, cok, n);
    return hipGetLastError();
}

hipError_t launch_stage_copy(hipStream_t st, void* dst, const void* src_dev, size_t bytes) {
    if (bytes == 0) return hipSuccess;
    if ((bytes & 3) || ((uintptr_t)dst & 15) || ((uintptr_t)src_dev & 15)) return hipErrorInvalidValue;
    const int64_t n4 = (int64_t)(bytes >> 2);
    const int64_t want = ((n4 >> 2) + 255) / 256;
    const int blocks = (int)(want < 1 ? 1 : (want > 256 ? 256 : want));
    hipLaunchKernelGGL(stage_copy_kernel, dim3(blocks), dim3(256), 0, st,
                       reinterpret_cast<const uint32_t*>(src_dev), reinterpret_cast<uint32_t*>(dst), n4);
    return hipGetLastError();
}

hipError_t launch_edge_reduce(int E_local, hipStream_t st, const float* partials, int nchunks,
                              const float* Twc, const int* ii_loc, double* edgeblk,
                              const int* flags) {
    hipLaunchKernelGGL(gn_edge_reduce_kernel, dim3(E_local), dim3(64), 0, st, partials, nchunks,
                       Twc, ii_loc, edgeblk, flags);
    return hipGetLastError();
}

hipError_t launch_compact(hipStream_t st, const double* edgeblk, const int* blk_ptr,
                          const int* blk_ent, const int* grad_ptr, const int* grad_ent, int nblk,
                          int npose, double* compact, const int* flags) {
    hipLaunchKernelGGL(gn_compact_kernel, dim3(nblk + npose), dim3(64), 0, st, edgeblk, blk_ptr,
                       blk_ent, grad_ptr, grad_ent, nblk, npose, compact, flags);
    return hipGetLastError();
}

hipError_t launch_assemble(hipStream_t st, const double* edgeblk, const int* blk_ptr,
                           const int* blk_ent, const int* grad_ptr, const int* grad_ent, int nblk,
                           int nblocks, int npose, int bpad, double* out, const int* flags) {
    hipLaunchKernelGGL(gn_assemble_kernel, dim3(nblocks + npose), dim3(64), 0, st, edgeblk, blk_ptr,
                       blk_ent, grad_ptr, grad_ent, nblk, nblocks, npose, bpad, out, flags);
    return hipGetLastError();
}

hipError_t launch_dense_factor_solve(hipStream_t st, int npad, double* Hd, double* Linv,
                                     double* x, int* flags, int epoch, const DfScatter* g) {
    const int nt = npad / T;
    // M3S_CHOL_DF=1 (default): the whole LL^T as one dataflow launch (chol_df.hip); 0: one
    // potrf / trsm / update launch triple per panel
    const char* df_env = getenv("M3S_CHOL_DF");
    const int df = df_env ? atoi(df_env) : 1;
    bool done = false;
    if (df) {
        // a cooperative launch the device cannot hold (or refuses) falls back to the per-panel
        // launches below instead of failing the call
        // M3S_CHOL_DF_BACK=1 (default): the back-substitution runs in the same launch as dataflow
        // tasks (chol_df.hip back_task); 0: chol_backsolve_kernel after it
        const char* bk_env = getenv("M3S_CHOL_DF_BACK");
        const bool in_launch = bk_env ? atoi(bk_env) != 0 : true;
        // (the pose-indexed copy needs the in-launch back-substitution)
        done = launch_chol_dataflow(st, npad, Hd, Linv, chol_ready_ptr(Linv, npad), epoch, flags,
                                    (in_launch || g) ? x : nullptr, g) == hipSuccess;
        if (!done) (void)hipGetLastError();
        if (done && (in_launch || g)) return hipGetLastError();
    }
    if (!done) {
        for (int k = 0; k < nt; k++) {
            hipLaunchKernelGGL(chol_potrf_kernel, dim3(1), dim3(kPotrfThreads), 0, st, Hd, npad, k, Linv,
                               flags);
            hipLaunchKernelGGL(chol_trsm_kernel, dim3(nt - k), dim3(kGemmThreads), 0, st, Hd, npad, k,
                               Linv, flags);
            int nupd = 0;
            for (int j = k + 1; j < nt; j++) nupd += nt - j + 1;
            if (nupd > 0)
                hipLaunchKernelGGL(chol_update_kernel, dim3(nupd), dim3(kGemmThreads), 0, st, Hd, npad, nt,
                                   k, flags);
        }
    }
    hipLaunchKernelGGL(chol_backsolve_kernel, dim3(1), dim3(kBackThreads), 0, st, Hd, npad, Linv,
                       x, flags);
    if (g && g->xpose) return launch_sp_tail_scatter(st, x, g->tail, g->ntail, g->xpose, flags);
    return hipGetLastError();
}

hipError_t launch_solve(hipStream_t st, const double* compact, const int* slotmap, int nblk,
                        int npose, int n, int npad, double* Hd, double* Linv, double* x,
                        int* flags, int epoch) {
    const int64_t total = (int64_t)(npad + kCholTile) * npad;
    const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    hipLaunchKernelGGL(gn_fill_dense_kernel, dim3(blocks), dim3(256), 0, st, compact, slotmap,
                       nblk, npose, n, npad, Hd, flags);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_dense_factor_solve(st, npad, Hd, Linv, x, flags, epoch);
}

hipError_t launch_fill_only(hipStream_t st, const double* compact, const int* slotmap, int nblk,
                            int npose, int n, int npad, double* Hd, const int* flags) {
    const int64_t total = (int64_t)(npad + kCholTile) * npad;
    const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    hipLaunchKernelGGL(gn_fill_dense_kernel, dim3(blocks), dim3(256), 0, st, compact, slotmap,
                       nblk, npose, n, npad, Hd, flags);
    return hipGetLastError();
}

hipError_t launch_retract(hipStream_t st, float* Twc, const double* x, float* dx, int N,
                          float delta_thresh, int* flags, int contract) {
    hipLaunchKernelGGL(gn_retract_kernel, dim3(1), dim3(256), 0, st, Twc, x, dx, N, delta_thresh,
                       flags, contract);
    return hipGetLastError();
}

}  // namespace m3s
