// Probe: largest LDS allocation one workgroup can get on gfx950, and the shader clock
// (s_memtime) against the 100 MHz wall clock.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* out, int n) {
    extern __shared__ int buf[];
    for (int i = threadIdx.x; i < n; i += blockDim.x) buf[i] = i;
    __syncthreads();
    int s = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) s += buf[n - 1 - i];
    atomicAdd(out, s);
}
__global__ void clk(unsigned long long* out) {
    unsigned long long w0 = wall_clock64(), c0 = clock64();
    double x = 1.0;
    for (int i = 0; i < 2000000; i++) x = x * 1.0000001 + 1e-9;
    unsigned long long w1 = wall_clock64(), c1 = clock64();
    out[0] = w1 - w0; out[1] = c1 - c0; out[2] = (unsigned long long)x;
}
int main() {
    int* d; (void)hipMalloc(&d, 4);
    for (int kb : {64, 96, 128, 160}) {
        int n = kb * 1024 / 4;
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, kb * 1024);
        (void)hipMemset(d, 0, 4);
        hipLaunchKernelGGL(k, dim3(1), dim3(256), kb * 1024, 0, d, n);
        hipError_t e = hipDeviceSynchronize();
        hipError_t e2 = hipGetLastError();
        int h = 0; (void)hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
        long long want = (long long)n * (n - 1) / 2;
        printf("LDS %d KB: sync=%s last=%s sum_ok=%d\n", kb, hipGetErrorString(e), hipGetErrorString(e2), (long long)h == (int)want);
    }
    unsigned long long* c; (void)hipMalloc(&c, 24);
    hipLaunchKernelGGL(clk, dim3(1), dim3(64), 0, 0, c);
    unsigned long long hc[3]; (void)hipMemcpy(hc, c, 24, hipMemcpyDeviceToHost);
    printf("clock: wall %llu ticks (%.1f us), s_memtime %llu -> %.0f MHz\n", hc[0], hc[0] * 0.01, hc[1], hc[1] / (hc[0] * 0.01));
    return 0;
}
