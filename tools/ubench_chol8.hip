// Latency of small in-register Cholesky variants on one wave (cycles per factorisation).
#include <hip/hip_runtime.h>
#include <cstdio>
__host__ __device__ constexpr int pk(int i, int j) { return i * (i + 1) / 2 + j; }
__device__ __forceinline__ double rsq1(double d) {  // rsq + one Newton step
    const double y = __builtin_amdgcn_rsq(d);
    return y * fma(-0.5 * d * y, y, 1.5);
}
__device__ __forceinline__ double rsq0(double d) { return __builtin_amdgcn_rsq(d); }
template <int N, int V>
__device__ __forceinline__ void chol(double (&a)[N * (N + 1) / 2], double (&inv)[N]) {
#pragma unroll
    for (int p = 0; p < N; p++) {
        const double d = a[pk(p, p)];
        double y;
        if (V == 0) y = rsq1(d);
        else if (V == 1) y = rsq0(d);
        else y = 1.0 / sqrt(d);
        inv[p] = y;
        a[pk(p, p)] = d * y;
#pragma unroll
        for (int i = p + 1; i < N; i++) a[pk(i, p)] *= y;
#pragma unroll
        for (int i = p + 1; i < N; i++)
#pragma unroll
            for (int j = p + 1; j <= i; j++) a[pk(i, j)] = fma(-a[pk(i, p)], a[pk(j, p)], a[pk(i, j)]);
    }
}
template <int N, int V>
__global__ void k(double* out, unsigned long long* cyc, int iters) {
    constexpr int M = N * (N + 1) / 2;
    double a[M], inv[N];
    for (int i = 0; i < N; i++)
        for (int j = 0; j <= i; j++) a[pk(i, j)] = (i == j) ? 4.0 + threadIdx.x * 1e-3 : 0.1 * (i + j);
    double acc = 0.0;
    unsigned long long t0 = clock64();
    for (int it = 0; it < iters; it++) {
        double b[M];
#pragma unroll
        for (int q = 0; q < M; q++) b[q] = a[q] + acc * 1e-30;  // dependence on the previous result
        chol<N, V>(b, inv);
        acc += b[M - 1] + inv[N - 1];
    }
    unsigned long long t1 = clock64();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
template <int N, int V>
void run(const char* name) {
    double* d; unsigned long long* c;
    (void)hipMalloc(&d, 4096); (void)hipMalloc(&c, 64);
    const int iters = 2000;
    hipLaunchKernelGGL((k<N, V>), dim3(1), dim3(64), 0, 0, d, c, iters);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL((k<N, V>), dim3(1), dim3(64), 0, 0, d, c, iters);
    (void)hipDeviceSynchronize();
    unsigned long long h; (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("%-28s N=%d: %.0f cycles per factorisation\n", name, N, (double)h / iters);
}
int main() {
    run<7, 0>("rsq + 1 Newton");
    run<7, 1>("rsq only");
    run<7, 2>("1/sqrt (IEEE)");
    run<8, 0>("rsq + 1 Newton");
    run<8, 2>("1/sqrt (IEEE)");
    return 0;
}
