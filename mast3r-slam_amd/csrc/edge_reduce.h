// edge_reduce.h -- per local edge: f64 chunk sum of the accumulate's partials (fixed chunk
// order), Hjj = A M A^T, vj = A g with A the adjoint map of apply_Sim3_adj_inv
// (gn_kernels.cu:277-297).  Shared by gn_edge_reduce_kernel (its own launch) and the packed
// accumulate's last workgroup per edge (fused: the partials of other workgroups / XCDs are then
// read with agent-coherent loads).  Every thread of the workgroup must call it (barriers);
// threads >= 64 only take part in the barriers.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "gn_kernels.h"

namespace m3s {

template <bool COH>
__device__ __forceinline__ void edge_reduce_body(const float* __restrict__ partials, int nchunks,
                                                 const float* __restrict__ Twc,
                                                 const int* __restrict__ ii_loc,
                                                 double* __restrict__ edgeblk, int e) {
    const int tid = threadIdx.x;
    auto ldp = [](const float* q) -> float {
        if constexpr (COH) return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return *q;
    };
    __shared__ double M[7][7];
    __shared__ double g[7];
    __shared__ double A[7][7];
    __shared__ double AM[7][7];
    // the pose loads (ii -> Twc, two dependent trips) are issued first, so they overlap the
    // chunk-partial loads instead of following them
    float Ti[8];
    if (tid < 3) {
        const float* Tp = Twc + (int64_t)ii_loc[e] * 8;
#pragma unroll
        for (int k = 0; k < 8; k++) Ti[k] = Tp[k];
    }
    if (tid < kNacc) {
        const float* p = partials + (int64_t)e * nchunks * kNaccPad + tid;
        double s = 0.0;
        int c = 0;
        for (; c + 8 <= nchunks; c += 8) {  // 8 loads in flight, summed in chunk order
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = ldp(p + (int64_t)(c + u) * kNaccPad);
#pragma unroll
            for (int u = 0; u < 8; u++) s += (double)v[u];
        }
        for (; c < nchunks; c++) s += (double)ldp(p + (int64_t)c * kNaccPad);
        if (tid < 28) {
            int a = 0, r = tid;
            while (r >= 7 - a) { r -= 7 - a; a++; }
            const int b = a + r;
            M[a][b] = s;
            M[b][a] = s;
        } else {
            g[tid - 28] = s;
        }
    }
    if (tid < 49) A[tid / 7][tid % 7] = 0.0;
    __syncthreads();
    if (tid < 3) {
        // column tid of the adjoint map of apply_Sim3_adj_inv (gn_kernels.cu:277-297)
        const double t0 = Ti[0], t1 = Ti[1], t2 = Ti[2];
        const double qx = Ti[3], qy = Ti[4], qz = Ti[5], qw = Ti[6];
        const double s_inv = 1.0 / (double)Ti[7];
        // R e_c via the actSO3 formula
        double X[3] = {0, 0, 0};
        X[tid] = 1.0;
        const double uv0 = 2.0 * (qy * X[2] - qz * X[1]);
        const double uv1 = 2.0 * (qz * X[0] - qx * X[2]);
        const double uv2 = 2.0 * (qx * X[1] - qy * X[0]);
        const double R0 = X[0] + qw * uv0 + (qy * uv2 - qz * uv1);
        const double R1 = X[1] + qw * uv1 + (qz * uv0 - qx * uv2);
        const double R2 = X[2] + qw * uv2 + (qx * uv1 - qy * uv0);
        A[0][tid] = s_inv * R0;
        A[1][tid] = s_inv * R1;
        A[2][tid] = s_inv * R2;
        A[3][tid] = s_inv * (t1 * R2 - t2 * R1);
        A[4][tid] = s_inv * (t2 * R0 - t0 * R2);
        A[5][tid] = s_inv * (t0 * R1 - t1 * R0);
        A[6][tid] = s_inv * (t0 * R0 + t1 * R1 + t2 * R2);
        A[3][3 + tid] = R0;
        A[4][3 + tid] = R1;
        A[5][3 + tid] = R2;
        if (tid == 0) A[6][6] = 1.0;
    }
    __syncthreads();
    if (tid < 49) {
        const int a = tid / 7, b = tid % 7;
        double s = 0.0;
#pragma unroll
        for (int p = 0; p < 7; p++) s += A[a][p] * M[p][b];
        AM[a][b] = s;
    }
    __syncthreads();
    double* out = edgeblk + (int64_t)e * kEdgeBlk;
    if (tid < 28) {
        int a = 0, r = tid;
        while (r >= 7 - a) { r -= 7 - a; a++; }
        const int b = a + r;
        double s = 0.0;
#pragma unroll
        for (int p = 0; p < 7; p++) s += AM[a][p] * A[b][p];
        out[tid] = s;  // Hjj (upper packed)
    } else if (tid < 35) {
        const int a = tid - 28;
        double s = 0.0;
#pragma unroll
        for (int p = 0; p < 7; p++) s += A[a][p] * g[p];
        out[tid] = s;  // vj
    }
}

}  // namespace m3s
