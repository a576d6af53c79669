// PMC calibration for gfx950 FETCH_SIZE / WRITE_SIZE (MI355X_MICROARCH.md §HBM):
// kernels with a KNOWN byte count in the access shapes the GN accumulate kernel uses
//   k_stream16 : 16-B/lane coalesced reads of a 1 GiB buffer  (idx / Q / Xj / Cj streams)
//   k_stream4  : 4-B/lane coalesced reads                        (uchar4 valid stream)
//   k_gather12 : 12-B records gathered at local random offsets   (the Xi gather)
// Run under rocprofv3 --pmc FETCH_SIZE (and separately WRITE_SIZE); compare with the
// printed byte counts to get the per-shape correction factor.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_stream16(const float4* __restrict__ a, size_t n, float* out) {
    float s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1234.5f) out[0] = s;
}

__global__ void k_stream4(const uint32_t* __restrict__ a, size_t n, float* out) {
    uint32_t s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        s += a[i];
    if (s == 12345u) out[0] = (float)s;
}

__global__ void k_gather12(const float* __restrict__ a, size_t nrec, float* out) {
    float s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nrec; i += (size_t)gridDim.x * blockDim.x) {
        // local permutation within 64-record windows (like flow-displaced matches)
        size_t j = (i & ~(size_t)63) | ((i * 37 + 11) & 63);
        s += a[j * 3] + a[j * 3 + 1] + a[j * 3 + 2];
    }
    if (s == 1234.5f) out[0] = s;
}

int main() {
    const size_t bytes = (size_t)1 << 30;
    void* buf;
    float* out;
    hipMalloc(&buf, bytes);
    hipMalloc(&out, 64);
    hipMemset(buf, 0, bytes);
    hipDeviceSynchronize();
    k_stream16<<<4096, 256>>>((const float4*)buf, bytes / 16, out);
    k_stream4<<<4096, 256>>>((const uint32_t*)buf, bytes / 4, out);
    k_gather12<<<4096, 256>>>((const float*)buf, bytes / 12, out);
    hipDeviceSynchronize();
    printf("bytes read per kernel: stream16 %zu stream4 %zu gather12 %zu\n", bytes, bytes,
           (bytes / 12) * 12);
    return 0;
}
