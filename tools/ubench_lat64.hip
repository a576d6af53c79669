// Diagnostic: f64 latency / issue constants on gfx950 for the dense-solve chain (one wave unless
// stated; s_memtime cycles, calibrated against s_memrealtime's 100 MHz in the same launch).
// Each timed region starts with an asm that "modifies" the chain's input, and ends with an asm
// that consumes its output, so the compiler cannot hoist or sink the chain out of the region.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ long long stamp() {
    long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
__device__ __forceinline__ long long rstamp() {
    long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
__device__ __forceinline__ double rdlane(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __hiloint2double(hi, lo);
}
#define PIN(x) asm volatile("" : "+v"(x))
#define USE(x) asm volatile("" ::"v"(x))

__global__ __launch_bounds__(256) void k_probe(double* out, long long* cyc, double a, double b) {
    __shared__ double sh[512];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    double x = lane * 1e-3 + 1.0;
    long long t[20];
    int n = 0;
    const long long r0 = rstamp();
    t[n++] = stamp();
    if (w == 0) {
        // 1. dependent v_fma_f64 x64
        PIN(x);
#pragma unroll
        for (int i = 0; i < 64; i++) x = fma(x, a, b);
        USE(x);
        t[n++] = stamp();
        // 2. 8 independent v_fma_f64 chains x16 (issue rate)
        double y[8];
#pragma unroll
        for (int q = 0; q < 8; q++) y[q] = x + q;
#pragma unroll
        for (int q = 0; q < 8; q++) PIN(y[q]);
        t[n++] = stamp();
#pragma unroll
        for (int i = 0; i < 16; i++)
#pragma unroll
            for (int q = 0; q < 8; q++) y[q] = fma(y[q], a, b);
#pragma unroll
        for (int q = 0; q < 8; q++) USE(y[q]);
        t[n++] = stamp();
        // 3. dependent mfma_f64_16x16x4 x16
        d4 c = {x, y[0], y[1], y[2]};
        PIN(c);
#pragma unroll
        for (int i = 0; i < 16; i++) c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, x, c, 0, 0, 0);
        USE(c);
        t[n++] = stamp();
        // 4. 4 independent mfma chains x8
        d4 cc[4] = {c, c + 1.0, c + 2.0, c + 3.0};
#pragma unroll
        for (int q = 0; q < 4; q++) PIN(cc[q]);
        t[n++] = stamp();
#pragma unroll
        for (int i = 0; i < 8; i++)
#pragma unroll
            for (int q = 0; q < 4; q++) cc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, x, cc[q], 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 4; q++) USE(cc[q]);
        t[n++] = stamp();
        // 5. readlane x2 -> fma chain x32
        x = cc[0][0] + cc[1][1] + cc[2][2] + cc[3][3];
        PIN(x);
        t[n++] = stamp();
#pragma unroll
        for (int i = 0; i < 32; i++) x = fma(rdlane(x, i & 63), a, b);
        USE(x);
        t[n++] = stamp();
        // 6. rsq_f64 -> add chain x16
#pragma unroll
        for (int i = 0; i < 16; i++) x = __builtin_amdgcn_rsq(x) + b;
        USE(x);
        t[n++] = stamp();
        // 7. ds_write_b64 -> ds_read_b64 round trip x16
#pragma unroll
        for (int i = 0; i < 16; i++) {
            sh[lane] = x;
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
            x = sh[(lane + 1) & 63] + b;
        }
        USE(x);
        t[n++] = stamp();
    }
    __syncthreads();
    t[n++] = stamp();
    // 8. s_barrier x16 (4 waves)
#pragma unroll
    for (int i = 0; i < 16; i++) __syncthreads();
    t[n++] = stamp();
    const long long r1 = rstamp();
    out[tid] = x;
    if (tid == 0) {
        for (int k = 0; k < n; k++) cyc[k] = t[k];
        cyc[18] = r1 - r0;
        cyc[19] = n;
    }
}

int main() {
    double* dout;
    long long* dc;
    hipMalloc(&dout, 256 * 8);
    hipMalloc(&dc, 20 * 8);
    long long c[20];
    for (int r = 0; r < 4; r++) hipLaunchKernelGGL(k_probe, dim3(1), dim3(256), 0, 0, dout, dc, 0.999, 1e-3);
    hipDeviceSynchronize();
    hipMemcpy(c, dc, sizeof(c), hipMemcpyDeviceToHost);
    const double ghz = (double)(c[10] - c[0]) / (c[18] * 10.0);  // whole kernel: cycles / ns
    printf("clock %.2f GHz (s_memtime / s_memrealtime over the launch)\n", ghz);
    printf("dependent v_fma_f64        %6.1f cyc/op\n", (c[1] - c[0]) / 64.0);
    printf("independent v_fma_f64 issue %5.1f cyc/op\n", (c[3] - c[2]) / 128.0);
    printf("dependent mfma_f64 16x16x4 %6.1f cyc/op\n", (c[4] - c[3]) / 16.0);
    printf("4 chains mfma_f64 issue    %6.1f cyc/op\n", (c[6] - c[5]) / 32.0);
    printf("readlane x2 + fma chain    %6.1f cyc/step\n", (c[8] - c[7]) / 32.0);
    printf("rsq_f64 + add chain        %6.1f cyc/step\n", (c[9] - c[8]) / 16.0);
    printf("ds_write_b64 -> ds_read_b64 %5.1f cyc/round trip\n", (c[10] - c[9]) / 16.0);
    printf("s_barrier (4 waves)        %6.1f cyc\n", (c[12] - c[11]) / 16.0);
    return 0;
}
