// Diagnostic: single-wave latencies on gfx950 that bound the dense factorisation's column
// chain (dependent f64 FMA, rsq/rcp_f64, readlane broadcast, LDS round trip, barrier).
// Each kernel is one workgroup; cycles from s_memtime around a 256-long dependent chain.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int N = 256;

__device__ __forceinline__ long long now() { return __builtin_amdgcn_s_memtime(); }

__global__ void k_fma64_dep(long long* cyc, double* out, double a, double b) {
    double x = threadIdx.x * 1e-3;
    long long t0 = now();
#pragma unroll
    for (int i = 0; i < N; i++) x = fma(x, a, b);
    __builtin_amdgcn_s_waitcnt(0);
    long long t1 = now();
    if (x == 12345.0) out[0] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_fma64_ind8(long long* cyc, double* out, double a, double b) {
    double x[8];
#pragma unroll
    for (int q = 0; q < 8; q++) x[q] = threadIdx.x * 1e-3 + q;
    long long t0 = now();
#pragma unroll
    for (int i = 0; i < N / 8; i++)
#pragma unroll
        for (int q = 0; q < 8; q++) x[q] = fma(x[q], a, b);
    long long t1 = now();
    double s = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) s += x[q];
    if (s == 12345.0) out[0] = s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_fma32_dep(long long* cyc, double* out, float a, float b) {
    float x = threadIdx.x * 1e-3f;
    long long t0 = now();
#pragma unroll
    for (int i = 0; i < N; i++) x = fmaf(x, a, b);
    long long t1 = now();
    if (x == 12345.0f) out[0] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_rsq64_dep(long long* cyc, double* out, double a, double b) {
    double x = 1.0 + threadIdx.x * 1e-3;
    long long t0 = now();
#pragma unroll
    for (int i = 0; i < N; i++) x = __builtin_amdgcn_rsq(x) + b;
    long long t1 = now();
    if (x == 12345.0) out[0] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// broadcast chain through v_readlane (lane i+1 -> all)
__global__ void k_readlane_dep(long long* cyc, double* out, double a, double b) {
    double x = 1.0 + threadIdx.x * 1e-3;
    long long t0 = now();
#pragma unroll
    for (int i = 0; i < N; i++) {
        const int lo = __builtin_amdgcn_readlane(__double2loint(x), i & 63);
        const int hi = __builtin_amdgcn_readlane(__double2hiint(x), i & 63);
        x = fma(__hiloint2double(hi, lo), a, x);
    }
    long long t1 = now();
    if (x == 12345.0) out[0] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// LDS write -> read round trip chain within one wave
__global__ void k_lds_dep(long long* cyc, double* out, double a, double b) {
    __shared__ double buf[64];
    double x = 1.0 + threadIdx.x * 1e-3;
    long long t0 = now();
    for (int i = 0; i < N; i++) {
        buf[threadIdx.x] = x;
        __builtin_amdgcn_wave_barrier();
        x = fma(buf[(threadIdx.x + 1) & 63], a, b);
        __builtin_amdgcn_wave_barrier();
    }
    long long t1 = now();
    if (x == 12345.0) out[0] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// __syncthreads chain with LDS traffic, blockDim waves
__global__ void k_barrier_dep(long long* cyc, double* out, double a, double b) {
    __shared__ double buf[2][1024];
    double x = 1.0 + threadIdx.x * 1e-3;
    long long t0 = now();
    for (int i = 0; i < N; i++) {
        buf[i & 1][threadIdx.x] = x;
        __syncthreads();
        x = fma(buf[i & 1][(threadIdx.x + 64) % blockDim.x], a, b);
    }
    long long t1 = now();
    if (x == 12345.0) out[0] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    long long* cyc;
    double* out;
    (void)hipMalloc(&cyc, 64);
    (void)hipMalloc(&out, 64);
    struct K {
        const char* name;
        void (*run)(long long*, double*);
    };
    auto report = [&](const char* name) {
        long long h = 0;
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
        printf("%-22s %8.1f cycles/step (s_memtime ticks)\n", name, (double)h / N);
    };
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(k_fma64_dep, 1, 64, 0, 0, cyc, out, 1.0000001, 1e-9);
        report("fma_f64 dependent");
        hipLaunchKernelGGL(k_fma64_ind8, 1, 64, 0, 0, cyc, out, 1.0000001, 1e-9);
        report("fma_f64 8 chains");
        hipLaunchKernelGGL(k_fma32_dep, 1, 64, 0, 0, cyc, out, 1.0000001f, 1e-9f);
        report("fma_f32 dependent");
        hipLaunchKernelGGL(k_rsq64_dep, 1, 64, 0, 0, cyc, out, 1.0, 1e-9);
        report("rsq_f64+add dependent");
        hipLaunchKernelGGL(k_readlane_dep, 1, 64, 0, 0, cyc, out, 1e-9, 0.0);
        report("readlane64+fma dep");
        hipLaunchKernelGGL(k_lds_dep, 1, 64, 0, 0, cyc, out, 1.0000001, 1e-9);
        report("lds wr->rd+fma dep");
        for (int th : {64, 256, 512, 1024}) {
            hipLaunchKernelGGL(k_barrier_dep, 1, th, 0, 0, cyc, out, 1.0000001, 1e-9);
            char nm[64];
            snprintf(nm, sizeof nm, "barrier+lds %4d thr", th);
            report(nm);
        }
    }
    // s_memtime tick vs wall clock
    return 0;
}
