// test_hooks.hip -- test-only kernels of the measurement library (include/m3s_variants.h), not part
// of the drop-in boundary.
//
// hold_cus_kernel: workgroups that each hold `lds_bytes` of a CU's LDS for a bounded time, so a
// test can make CUs unavailable to another launch -- the dataflow factorisation (chol_df.hip)
// assumes its grid is resident together; SURVEY.md §8(b): the tracker and the backend process
// launch on the same GPU concurrently.  The wait is bounded by the constant 100 MHz real-time
// counter: every wave finishes.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/m3s_variants.h"

namespace {

__global__ __launch_bounds__(64) void hold_cus_kernel(long long ticks) {
    extern __shared__ int lds_hold[];
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    lds_hold[threadIdx.x] = (int)threadIdx.x;  // touch the allocation
    while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
    if (lds_hold[threadIdx.x] < 0) lds_hold[0] = 1;  // keeps the allocation live
}

}  // namespace

extern "C" int m3s_test_hold_cus(int nblocks, int lds_bytes, int usec, void* stream) {
    if (nblocks <= 0 || nblocks > 4096 || lds_bytes < 256 || lds_bytes > 160 * 1024 || usec < 0 || usec > 2000000)
        return 1;
    const hipStream_t st = static_cast<hipStream_t>(stream);
    if (lds_bytes > 64 * 1024 &&
        hipFuncSetAttribute((const void*)hold_cus_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes) !=
            hipSuccess)
        return 2;
    const long long ticks = (long long)usec * 100;  // s_memrealtime: 100 MHz
    hipLaunchKernelGGL(hold_cus_kernel, dim3(nblocks), dim3(64), lds_bytes, st, ticks);
    return hipGetLastError() == hipSuccess ? 0 : 2;
}
