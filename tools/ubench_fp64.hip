// Diagnostic: measured v_fma_f64 / v_fma_f32 / v_mfma_f64_16x16x4f64 throughput on gfx950
// (chip-wide and for one wave alone), to size the f64 dense solve.
#include <hip/hip_runtime.h>

#include <cstdio>

template <typename F>
__global__ __launch_bounds__(256) void k_fma(F* out, int iters, F a, F b) {
    F x[8];
#pragma unroll
    for (int q = 0; q < 8; q++) x[q] = threadIdx.x * 0.001 + q;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int q = 0; q < 8; q++) x[q] = fma(x[q], a, b);
    }
    F s = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) s += x[q];
    if (s == (F)12345) out[0] = s;
}

typedef double d4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_mfma64(double* out, int iters, double a) {
    d4 acc[4] = {};
    double av = a + threadIdx.x, bv = a - threadIdx.x;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int q = 0; q < 4; q++) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[q], 0, 0, 0);
    }
    double s = 0;
    for (int q = 0; q < 4; q++) s += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
    if (s == 12345.0) out[0] = s;
}

int main() {
    double* out;
    hipMalloc(&out, 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 4096;
    for (int grid : {1, 1024 * 4}) {
        float ms;
        // f64 VALU
        hipLaunchKernelGGL(k_fma<double>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0000001, 1e-9);
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k_fma<double>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0000001, 1e-9);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        double fl = 2.0 * 8 * iters * 256.0 * grid;
        printf("grid %5d  v_fma_f64 : %8.3f ms  %8.2f TFLOP/s  (%.1f cyc/wave-instr @2.4GHz if 1 wave/SIMD)\n", grid, ms,
               fl / ms / 1e9, ms * 1e-3 * 2.4e9 / (8.0 * iters));
        hipLaunchKernelGGL(k_fma<float>, dim3(grid), dim3(256), 0, 0, (float*)out, iters, 1.0000001f, 1e-9f);
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k_fma<float>, dim3(grid), dim3(256), 0, 0, (float*)out, iters, 1.0000001f, 1e-9f);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("grid %5d  v_fma_f32 : %8.3f ms  %8.2f TFLOP/s  (%.1f cyc/wave-instr)\n", grid, ms, fl / ms / 1e9,
               ms * 1e-3 * 2.4e9 / (8.0 * iters));
        hipLaunchKernelGGL(k_mfma64, dim3(grid), dim3(256), 0, 0, out, iters, 1.0);
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k_mfma64, dim3(grid), dim3(256), 0, 0, out, iters, 1.0);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        double flm = 2.0 * 16 * 16 * 4 * 4.0 * iters * 4 * grid;  // 4 waves per WG
        printf("grid %5d  mfma_f64  : %8.3f ms  %8.2f TFLOP/s  (%.1f cyc/instr)\n", grid, ms, flm / ms / 1e9,
               ms * 1e-3 * 2.4e9 / (4.0 * iters));
    }
    return 0;
}
