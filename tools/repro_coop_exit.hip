// repro_coop_exit.hip -- does a process that made ONE cooperative launch exit cleanly under
// rocprofv3 --kernel-trace?  (Diagnostic for the exit-time SIGSEGV of the cfg4 profiler runs,
// the fault is in libhsa-runtime64 called from the HIP runtime's exit
// handler; cfg4 is the only bench path with cooperative launches.)  No torch, no m3s library.
//   usage: repro_coop_exit [coop=1]     (0: the same kernel with a regular launch)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ void touch(int* p) {
    if (threadIdx.x == 0) p[blockIdx.x] = (int)blockIdx.x;
}

int main(int argc, char** argv) {
    const int coop = argc > 1 ? atoi(argv[1]) : 1;
    int* d = nullptr;
    if (hipMalloc(&d, 64 * sizeof(int)) != hipSuccess) return 2;
    hipError_t e;
    if (coop) {
        void* args[] = {&d};
        e = hipLaunchCooperativeKernel((const void*)touch, dim3(64), dim3(64), args, 0, nullptr);
    } else {
        hipLaunchKernelGGL(touch, dim3(64), dim3(64), 0, nullptr, d);
        e = hipGetLastError();
    }
    if (e != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        printf("launch failed: %s\n", hipGetErrorString(e));
        return 3;
    }
    int h[64];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    printf("coop=%d ok (h[63]=%d)\n", coop, h[63]);
    return 0;
}
