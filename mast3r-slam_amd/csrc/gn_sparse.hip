// gn_sparse.hip -- the multi-launch block-sparse solve of the pose-graph normal equations.
//
// The GN system is a graph Laplacian with 7x7 blocks: one block row per non-pinned pose,
// a block per co-observing pose pair.  The driver (gn_driver.hip, build_sparse_plan) picks,
// round by round, an independent set of low-degree poses; a round eliminates all of them at
// once (they do not touch each other), one workgroup per pose:
//   sp_factor : L_v = chol(A_vv) (7x7), Li_v = L_v^{-1}, W_rv = A_rv Li_v^T for every front
//               pose r (the L blocks), y_v = Li_v b_v                    (the forward solve)
//   sp_schur  : A_rs -= sum_v W_rv W_sv^T, b_r -= sum_v W_rv y_v over the round, each target
//               summed by one workgroup over a host-ordered contribution list (deterministic)
// The poses left after the rounds (a dense-ish core) are moved into the dense f64 matrix of
// the tiled Cholesky (gn_kernels.hip, sp_tail_*); then sp_back runs the rounds in reverse:
//   x_v = Li_v^T (y_v - sum_r W_rv^T x_r).
// This path serves graphs whose elimination needs many rounds (many workgroups per round hide
// the memory latency); small graphs run the single-workgroup solve of gn_solve.hip instead.
// Failure semantics follow SimplicialLLT (gn_kernels.cu:142-150): a pivot <= 0 sets the
// failure flag and the update becomes zero.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gn_kernels.h"

namespace m3s {

namespace {
__host__ __device__ constexpr int symi(int a, int b) { return a * 7 - a * (a - 1) / 2 + (b - a); }
}  // namespace

// A blocks (49 f64, row-major, block (x,y) stores rows of pose x, x < y) from the compact
// system; fill blocks are zeroed; b from the compact gradient.
__global__ __launch_bounds__(64) void sp_init_kernel(const double* __restrict__ compact, int nblk,
                                                     int nblocks, int npose,
                                                     double* __restrict__ A,
                                                     double* __restrict__ b,
                                                     const int* __restrict__ flags) {
    if (flags[kFlagDone]) return;
    const int s = blockIdx.x, t = threadIdx.x;
    if (s < nblocks) {
        if (t < 49) {
            const int a = t / 7, c = t % 7;
            A[(int64_t)s * 49 + t] =
                s < nblk ? compact[(int64_t)s * 28 + (a <= c ? symi(a, c) : symi(c, a))] : 0.0;
        }
    } else {
        for (int i = t; i < npose * 7; i += 64) b[i] = compact[(int64_t)nblk * 28 + i];
    }
}

// One workgroup per eliminated pose.  fronts: 4 ints per entry (r, block, transposed, W id).
__global__ __launch_bounds__(64) void sp_factor_kernel(
    const int* __restrict__ nodes, const int* __restrict__ fptr, const int* __restrict__ fronts,
    int node_begin, const double* __restrict__ A, const double* __restrict__ b,
    double* __restrict__ Lstore, double* __restrict__ W, double* __restrict__ y,
    int* __restrict__ flags) {
    if (flags[kFlagDone]) return;
    __shared__ double Li[49];
    __shared__ double yv[7];
    const int q = node_begin + blockIdx.x;
    const int v = nodes[q];
    const int t = threadIdx.x;
    if (t == 0) {
        double D[7][7], L[7][7], M[7][7];
#pragma unroll
        for (int i = 0; i < 7; i++)
#pragma unroll
            for (int j = 0; j < 7; j++) D[i][j] = A[(int64_t)v * 49 + i * 7 + j];
        bool bad = false;
#pragma unroll
        for (int p = 0; p < 7; p++) {
            double d = D[p][p];
#pragma unroll
            for (int k = 0; k < p; k++) d -= L[p][k] * L[p][k];
            if (d <= 0.0) bad = true;  // SimplicialLLT: fails iff a pivot <= 0 (NaN passes)
            L[p][p] = sqrt(d);
            const double inv = 1.0 / L[p][p];
#pragma unroll
            for (int i = p + 1; i < 7; i++) {
                double s = D[i][p];
#pragma unroll
                for (int k = 0; k < p; k++) s -= L[i][k] * L[p][k];
                L[i][p] = s * inv;
            }
        }
        // M = L^{-1} (lower), forward substitution on the identity
#pragma unroll
        for (int j = 0; j < 7; j++) {
#pragma unroll
            for (int i = 0; i < 7; i++) {
                if (i < j) {
                    M[i][j] = 0.0;
                } else {
                    double s = (i == j) ? 1.0 : 0.0;
#pragma unroll
                    for (int k = 0; k < 7; k++)
                        if (k >= j && k < i) s -= L[i][k] * M[k][j];
                    M[i][j] = s / L[i][i];
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 7; i++)
#pragma unroll
            for (int j = 0; j < 7; j++) Li[i * 7 + j] = M[i][j];
#pragma unroll
        for (int i = 0; i < 7; i++) {
            double s = 0.0;
#pragma unroll
            for (int k = 0; k <= i; k++) s += M[i][k] * b[(int64_t)v * 7 + k];
            yv[i] = s;
        }
        if (bad) flags[kFlagFail] = 1;
    }
    __syncthreads();
    if (t < 49) Lstore[(int64_t)q * 49 + t] = Li[t];
    if (t < 7) y[(int64_t)v * 7 + t] = yv[t];
    if (t < 49) {
        const int ra = t / 7, cb = t % 7;
        for (int f = fptr[q]; f < fptr[q + 1]; f++) {
            const int blk = fronts[4 * f + 1], tr = fronts[4 * f + 2], wid = fronts[4 * f + 3];
            const double* Ab = A + (int64_t)blk * 49;
            // W[ra][cb] = sum_m A_rv[ra][m] * Li[cb][m]
            double s = 0.0;
#pragma unroll
            for (int m = 0; m < 7; m++) {
                const double arv = tr ? Ab[m * 7 + ra] : Ab[ra * 7 + m];
                s = fma(arv, Li[cb * 7 + m], s);
            }
            W[(int64_t)wid * 49 + t] = s;
        }
    }
}

// Block targets: tg = (block, contribution begin, end); contributions (W_x id, W_y id).
// RHS targets: rtg = (pose r, begin, end); contributions (W id, pose v).
__global__ __launch_bounds__(64) void sp_schur_kernel(
    const int* __restrict__ tg, const int* __restrict__ tc, int tbeg, int nbt,
    const int* __restrict__ rtg, const int* __restrict__ rc, int rbeg, const double* __restrict__ W,
    const double* __restrict__ y, double* __restrict__ A, double* __restrict__ b,
    const int* __restrict__ flags) {
    if (flags[kFlagDone]) return;
    const int g = blockIdx.x, t = threadIdx.x;
    if (g < nbt) {
        const int* T_ = tg + 3 * (tbeg + g);
        if (t < 49) {
            const int ra = t / 7, cb = t % 7;
            double acc = 0.0;
            for (int c = T_[1]; c < T_[2]; c++) {
                const double* Wx = W + (int64_t)tc[2 * c] * 49 + ra * 7;
                const double* Wy = W + (int64_t)tc[2 * c + 1] * 49 + cb * 7;
#pragma unroll
                for (int m = 0; m < 7; m++) acc = fma(Wx[m], Wy[m], acc);
            }
            A[(int64_t)T_[0] * 49 + t] -= acc;
        }
    } else {
        const int* R = rtg + 3 * (rbeg + g - nbt);
        if (t < 7) {
            double acc = 0.0;
            for (int c = R[1]; c < R[2]; c++) {
                const double* Wr = W + (int64_t)rc[2 * c] * 49 + t * 7;
                const double* yv = y + (int64_t)rc[2 * c + 1] * 7;
#pragma unroll
                for (int m = 0; m < 7; m++) acc = fma(Wr[m], yv[m], acc);
            }
            b[(int64_t)R[0] * 7 + t] -= acc;
        }
    }
}

// x_v = Li_v^T (y_v - sum_r W_rv^T x_r)
__global__ __launch_bounds__(64) void sp_back_kernel(
    const int* __restrict__ nodes, const int* __restrict__ fptr, const int* __restrict__ fronts,
    int node_begin, const double* __restrict__ Lstore, const double* __restrict__ W,
    const double* __restrict__ y, double* __restrict__ x, const int* __restrict__ flags) {
    if (flags[kFlagDone]) return;
    __shared__ double z[7];
    const int q = node_begin + blockIdx.x;
    const int v = nodes[q];
    const int t = threadIdx.x;
    if (t < 7) {
        double s = y[(int64_t)v * 7 + t];
        for (int f = fptr[q]; f < fptr[q + 1]; f++) {
            const int r = fronts[4 * f], wid = fronts[4 * f + 3];
            const double* Wr = W + (int64_t)wid * 49;
#pragma unroll
            for (int m = 0; m < 7; m++) s = fma(-Wr[m * 7 + t], x[(int64_t)r * 7 + m], s);
        }
        z[t] = s;
    }
    __syncthreads();
    if (t < 7) {
        const double* Li = Lstore + (int64_t)q * 49;
        double s = 0.0;
#pragma unroll
        for (int m = 0; m < 7; m++) s = fma(Li[m * 7 + t], z[m], s);
        x[(int64_t)v * 7 + t] = s;
    }
}

// Dense core: Hd [npad + 64, npad] from the blocks of the ntail remaining poses (tmap:
// ntail x ntail -> 2*block + transposed, or -1), RHS border row from b.
__global__ __launch_bounds__(256) void sp_tail_fill_kernel(const double* __restrict__ A,
                                                           const double* __restrict__ b,
                                                           const int* __restrict__ tmap,
                                                           const int* __restrict__ tail,
                                                           int ntail, int npad,
                                                           double* __restrict__ Hd,
                                                           const int* __restrict__ flags) {
    if (flags[kFlagDone]) return;
    const int n = ntail * 7;
    const int64_t total = (int64_t)(npad + kCholTile) * npad;
    for (int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; id < total;
         id += (int64_t)gridDim.x * blockDim.x) {
        const int r = (int)(id / npad), c = (int)(id % npad);
        double val;
        if (r > npad) {
            val = 0.0;
        } else if (r == npad) {
            val = c < n ? b[(int64_t)tail[c / 7] * 7 + c % 7] : 0.0;
        } else if (r < n && c < n) {
            const int code = tmap[(r / 7) * ntail + c / 7];
            if (code < 0) {
                val = 0.0;
            } else {
                const double* Ab = A + (int64_t)(code >> 1) * 49;
                val = (code & 1) ? Ab[(c % 7) * 7 + r % 7] : Ab[(r % 7) * 7 + c % 7];
            }
        } else {
            val = (r == c) ? 1.0 : 0.0;
        }
        Hd[id] = val;
    }
}

__global__ __launch_bounds__(256) void sp_tail_scatter_kernel(const double* __restrict__ xd,
                                                              const int* __restrict__ tail,
                                                              int ntail, double* __restrict__ x,
                                                              const int* __restrict__ flags) {
    if (flags[kFlagDone]) return;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < ntail * 7) x[(int64_t)tail[i / 7] * 7 + i % 7] = xd[i];
}

// ------------------------------------------------------------------ launchers

hipError_t launch_sp_init(hipStream_t st, const double* compact, int nblk, int nblocks, int npose,
                          double* A, double* b, const int* flags) {
    hipLaunchKernelGGL(sp_init_kernel, dim3(nblocks + 1), dim3(64), 0, st, compact, nblk, nblocks,
                       npose, A, b, flags);
    return hipGetLastError();
}

hipError_t launch_sp_factor(hipStream_t st, int nnodes, const int* nodes, const int* fptr,
                            const int* fronts, int node_begin, const double* A, const double* b,
                            double* Lstore, double* W, double* y, int* flags) {
    if (nnodes <= 0) return hipSuccess;
    hipLaunchKernelGGL(sp_factor_kernel, dim3(nnodes), dim3(64), 0, st, nodes, fptr, fronts,
                       node_begin, A, b, Lstore, W, y, flags);
    return hipGetLastError();
}

hipError_t launch_sp_schur(hipStream_t st, const int* tg, const int* tc, int tbeg, int nbt,
                           const int* rtg, const int* rc, int rbeg, int nrt, const double* W,
                           const double* y, double* A, double* b, const int* flags) {
    if (nbt + nrt <= 0) return hipSuccess;
    hipLaunchKernelGGL(sp_schur_kernel, dim3(nbt + nrt), dim3(64), 0, st, tg, tc, tbeg, nbt, rtg,
                       rc, rbeg, W, y, A, b, flags);
    return hipGetLastError();
}

hipError_t launch_sp_back(hipStream_t st, int nnodes, const int* nodes, const int* fptr,
                          const int* fronts, int node_begin, const double* Lstore, const double* W,
                          const double* y, double* x, const int* flags) {
    if (nnodes <= 0) return hipSuccess;
    hipLaunchKernelGGL(sp_back_kernel, dim3(nnodes), dim3(64), 0, st, nodes, fptr, fronts,
                       node_begin, Lstore, W, y, x, flags);
    return hipGetLastError();
}

hipError_t launch_sp_tail(hipStream_t st, const double* A, const double* b, const int* tmap,
                          const int* tail, int ntail, int npad, double* Hd, double* Linv,
                          double* xd, double* x, int* flags) {
    if (ntail <= 0) return hipSuccess;
    const int64_t total = (int64_t)(npad + kCholTile) * npad;
    const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    hipLaunchKernelGGL(sp_tail_fill_kernel, dim3(blocks), dim3(256), 0, st, A, b, tmap, tail, ntail,
                       npad, Hd, flags);
    hipError_t e = launch_dense_factor_solve(st, npad, Hd, Linv, xd, flags);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(sp_tail_scatter_kernel, dim3((ntail * 7 + 255) / 256), dim3(256), 0, st, xd,
                       tail, ntail, x, flags);
    return hipGetLastError();
}

}  // namespace m3s
