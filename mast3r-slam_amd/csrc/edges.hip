// edges.hip -- the per-pixel part of FactorGraph.add_factors after the network (gfx950).
//
// Replaces the torch glue of reference mast3r_slam/global_opt.py:53-67:
//   Qj = sqrt(Qii[b, idx_i2j] * Qji),  Qi = sqrt(Qjj[b, idx_j2i] * Qij)
//   valid_j = valid_match_j & (Qj > Q_conf),  valid_i = valid_match_i & (Qi > Q_conf)
//   n_valid_j[b] = valid_j.sum(),  n_valid_i[b] = valid_i.sum()
// (torch: two gathers, two products, two sqrts, two compares, two ands, two reductions over
// [B,HW,1] tensors) in one pass: per pixel and direction 8 B index + 1 B mask + 4 B own Q +
// 4 B gathered Q read, 4 B written.  Q is computed with the same two f32 operations (product,
// correctly rounded sqrt) -> bit-exact; the counts are integers (exact in any order).
#include <hip/hip_runtime.h>

#include "../../include/m3s_backend.h"
#include "m3s_common.h"

#pragma clang fp contract(off)

namespace m3s {
namespace {

constexpr int kEdgeThreads = 256;

__global__ __launch_bounds__(kEdgeThreads) void edge_confidence_kernel(
    const int64_t* __restrict__ idx_i2j, const int64_t* __restrict__ idx_j2i,
    const uint8_t* __restrict__ vm_j, const uint8_t* __restrict__ vm_i,
    const float* __restrict__ Qii, const float* __restrict__ Qjj, const float* __restrict__ Qji,
    const float* __restrict__ Qij, float Q_conf, int64_t HW, int chunks, float* __restrict__ Qj,
    float* __restrict__ Qi, int* __restrict__ counts) {
    const int b = blockIdx.x / chunks;
    const int c = blockIdx.x - b * chunks;
    const int64_t per = (HW + chunks - 1) / chunks;
    const int64_t n0 = (int64_t)c * per;
    const int64_t n1 = n0 + per < HW ? n0 + per : HW;
    const int64_t base = (int64_t)b * HW;
    int cj = 0, ci = 0;
    for (int64_t n = n0 + threadIdx.x; n < n1; n += kEdgeThreads) {
        const int64_t p = base + n;
        int64_t a = idx_i2j[p], d = idx_j2i[p];
        a = a < 0 ? 0 : (a >= HW ? HW - 1 : a);  // the reference would fault out of range
        d = d < 0 ? 0 : (d >= HW ? HW - 1 : d);
        const float qj = sqrtf(Qii[base + a] * Qji[p]);
        const float qi = sqrtf(Qjj[base + d] * Qij[p]);
        Qj[p] = qj;
        Qi[p] = qi;
        cj += (vm_j[p] != 0) & (qj > Q_conf);
        ci += (vm_i[p] != 0) & (qi > Q_conf);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        cj += __shfl_xor(cj, off, 64);
        ci += __shfl_xor(ci, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(counts + 2 * b, cj);
        atomicAdd(counts + 2 * b + 1, ci);
    }
}

}  // namespace
}  // namespace m3s

extern "C" int m3s_edge_confidence(const int64_t* idx_i2j, const int64_t* idx_j2i,
                                   const uint8_t* valid_match_j, const uint8_t* valid_match_i,
                                   const float* Qii, const float* Qjj, const float* Qji,
                                   const float* Qij, float Q_conf, int64_t B, int64_t HW,
                                   float* Qj, float* Qi, int* counts, void* stream) {
    M3S_REQUIRE(B >= 0 && HW >= 0, "edge_confidence: negative sizes");
    if (B == 0) return M3S_OK;
    M3S_REQUIRE(idx_i2j && idx_j2i && valid_match_j && valid_match_i && Qii && Qjj && Qji && Qij &&
                    Qj && Qi && counts,
                "edge_confidence: null pointer");
    hipStream_t st = (hipStream_t)stream;
    M3S_HIP_CHECK(hipMemsetAsync(counts, 0, sizeof(int) * 2 * (size_t)B, st));
    if (HW == 0) return M3S_OK;
    // ~8 workgroups per CU over the whole batch, at least one chunk per pair
    int64_t chunks = (2048 + B - 1) / B;
    const int64_t max_chunks = (HW + m3s::kEdgeThreads - 1) / m3s::kEdgeThreads;
    if (chunks > max_chunks) chunks = max_chunks;
    if (chunks < 1) chunks = 1;
    M3S_REQUIRE(B * chunks < (int64_t)1 << 31, "edge_confidence: too many pairs");
    hipLaunchKernelGGL(m3s::edge_confidence_kernel, dim3((unsigned)(B * chunks)), dim3(m3s::kEdgeThreads),
                       0, st, idx_i2j, idx_j2i, valid_match_j, valid_match_i, Qii, Qjj, Qji, Qij,
                       Q_conf, HW, (int)chunks, Qj, Qi, counts);
    M3S_LAUNCH_CHECK();
    return M3S_OK;
}
