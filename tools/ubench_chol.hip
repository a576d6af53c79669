// Micro-benchmark of the per-column cost structure of the 64x64 tile factorisation
// (diagnostic only: which part of chol_potrf_kernel costs what on gfx950).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            printf("%s: %s\n", #x, hipGetErrorString(e));                           \
            return 1;                                                                \
        }                                                                            \
    } while (0)

constexpr int T = 64;

// variant 0: 64 barriers only
__global__ __launch_bounds__(256) void k_barriers(double* out) {
    __shared__ double buf[2][T];
    double acc = 0;
    for (int c = 0; c < T; c++) {
        acc += buf[c & 1][threadIdx.x & 63];
        if (threadIdx.x < 64) buf[(c + 1) & 1][threadIdx.x] = acc;
        __syncthreads();
    }
    if (acc == 12345.0) out[0] = acc;
}

// variant 1: barriers + 9 LDS reads + rcp per column
__global__ __launch_bounds__(256) void k_reads(double* out) {
    __shared__ double col[2][T];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    double acc = 0;
    if (threadIdx.x < 64) col[0][threadIdx.x] = 1.0 + threadIdx.x;
    __syncthreads();
    for (int c = 0; c < T; c++) {
        const double d = col[c & 1][c];
        double r = __builtin_amdgcn_rcp(d);
        r = r * (2.0 - d * r);
        r = r * (2.0 - d * r);
#pragma unroll
        for (int a = 0; a < 4; a++) acc += col[c & 1][ty + 16 * a] * r;
#pragma unroll
        for (int b = 0; b < 4; b++) acc += col[c & 1][tx + 16 * b];
        if (threadIdx.x < 64) col[(c + 1) & 1][threadIdx.x] = acc;
        __syncthreads();
    }
    if (acc == 12345.0) out[0] = acc;
}

// variant 2: full branch-free register update (16 fma + 16 fma) per column
__global__ __launch_bounds__(256) void k_full(double* out) {
    __shared__ double col[2][T];
    __shared__ double row[2][T];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    double v[4][4], m[4][4];
    for (int a = 0; a < 4; a++)
        for (int b = 0; b < 4; b++) { v[a][b] = a + b; m[a][b] = a - b; }
    if (threadIdx.x < 64) { col[0][threadIdx.x] = 1.0 + threadIdx.x; row[0][threadIdx.x] = 1.0; }
    __syncthreads();
    for (int c = 0; c < T; c++) {
        const int pb = c & 1;
        const double d = col[pb][c];
        double r = __builtin_amdgcn_rcp(d);
        r = r * (2.0 - d * r);
        r = r * (2.0 - d * r);
        double lr[4], ac[4], mc[4];
#pragma unroll
        for (int a = 0; a < 4; a++) {
            const int rr = ty + 16 * a;
            lr[a] = rr > c ? col[pb][rr] * r : 0.0;
        }
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const int cc = tx + 16 * b;
            ac[b] = cc > c ? col[pb][cc] : 0.0;
            mc[b] = cc <= c ? row[pb][cc] : 0.0;
        }
#pragma unroll
        for (int a = 0; a < 4; a++)
#pragma unroll
            for (int b = 0; b < 4; b++) {
                v[a][b] = fma(-lr[a], ac[b], v[a][b]);
                m[a][b] = fma(-lr[a], mc[b], m[a][b]);
            }
        if (tx == ((c + 1) & 15)) col[pb ^ 1][ty] = v[0][(c + 1) >> 4 & 3];
        if (ty == ((c + 1) & 15)) row[pb ^ 1][tx] = m[0][(c + 1) >> 4 & 3];
        __syncthreads();
    }
    double s = 0;
    for (int a = 0; a < 4; a++)
        for (int b = 0; b < 4; b++) s += v[a][b] + m[a][b];
    out[threadIdx.x] = s;
}

int main() {
    double* out;
    CK(hipMalloc(&out, 4096 * sizeof(double)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, void (*k)(double*)) {
        for (int w = 0; w < 3; w++) hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, out);
        hipEventRecord(e0);
        const int reps = 200;
        for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-12s %8.2f us/launch\n", name, ms * 1e3 / reps);
    };
    timeit("barriers", k_barriers);
    timeit("reads", k_reads);
    timeit("full", k_full);
    return 0;
}
