// Diagnostic: how many of the GN point records change between the hardware
// v_sqrt_f32 (<= 1 ulp, the round-3 record builders) and the correctly rounded sqrtf the builders
// use since round 4.  count_sqrt_diff(q, n, out[2]): out[0] = values whose two square roots
// differ, out[1] = values counted (finite q > 0).
#include <hip/hip_runtime.h>

#include <cstdint>

__global__ void k_count(const float* __restrict__ q, int64_t n, unsigned long long* out) {
    unsigned long long d = 0, c = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float v = q[i];
        if (v > 0.0f && v < __builtin_huge_valf()) {
            c++;
            d += __float_as_uint(__builtin_amdgcn_sqrtf(v)) != __float_as_uint(__builtin_sqrtf(v));
        }
    }
    atomicAdd(out, d);
    atomicAdd(out + 1, c);
}

extern "C" int count_sqrt_diff(const float* q, int64_t n, unsigned long long* out_host) {
    unsigned long long* d = nullptr;
    if (hipMalloc(&d, 16) != hipSuccess) return 1;
    hipMemset(d, 0, 16);
    hipLaunchKernelGGL(k_count, dim3(1024), dim3(256), 0, 0, q, n, d);
    hipMemcpy(out_host, d, 16, hipMemcpyDeviceToHost);
    hipFree(d);
    return hipGetLastError() != hipSuccess;
}
