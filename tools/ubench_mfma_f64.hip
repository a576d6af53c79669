// Throughput of v_mfma_f64_16x16x4_f64 on one SIMD (one wave, 8 independent accumulators) and
// on a whole CU (4 waves), cycles via s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ void k(double* out, unsigned long long* cyc, int iters) {
    d4 acc[8];
    for (int i = 0; i < 8; i++) acc[i] = d4{0, 0, 0, 0};
    double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
    unsigned long long t0 = clock64();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    double s = 0;
    for (int i = 0; i < 8; i++) s += acc[i][0] + acc[i][3];
    unsigned long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
    double* d; unsigned long long* c;
    (void)hipMalloc(&d, 1 << 20); (void)hipMalloc(&c, 1024);
    const int iters = 2000;
    for (int threads : {64, 256}) {
        hipLaunchKernelGGL(k, dim3(1), dim3(threads), 0, 0, d, c, iters);
        (void)hipDeviceSynchronize();
        unsigned long long h; (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
        printf("%d threads: %.1f cycles per MFMA per wave (8 independent accumulators)\n", threads,
               (double)h / (iters * 8.0));
    }
    return 0;
}
