// wave_reduce.h -- cross-lane sums for wave64 register accumulators (gfx950).
//
// A wave holding 36 per-lane partial sums reduces them as a reduce-scatter: v_permlane32_swap
// halves 36 registers to 18, v_permlane16_swap to 9, then a DPP row sum over each 16-lane row
// (126 lane ops instead of 36 x 6 shuffle-adds of a butterfly per value).  Used by the GN
// accumulate (gn_accum.hip block_partial) and the tracker's accumulate (track.hip).
#pragma once

#include <hip/hip_runtime.h>

namespace m3s {

// Half exchanges of two registers (gfx950 v_permlane32_swap / v_permlane16_swap): afterwards
// a + b holds, in the first half (row pair) of the lanes, a's partial sums and in the second
// b's -- a reduce-scatter step that costs one swap + one add for two values.
__device__ __forceinline__ float halfsum32(float a, float b) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float halfsum16(float a, float b) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// sum over the 16 lanes of each row (every lane of the row gets it): DPP row rotations
template <int N>
__device__ __forceinline__ float row_ror(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x120 + N, 0xf, 0xf, false));
}
__device__ __forceinline__ float row_sum16(float v) {
    v += row_ror<8>(v);
    v += row_ror<4>(v);
    v += row_ror<2>(v);
    v += row_ror<1>(v);
    return v;
}

// The 36 sums of a wave: afterwards lane 16 r of register x[j] holds sum j + 9 r (r = 0..3).
__device__ __forceinline__ void wave_sum36(const float* v, float (&x)[9]) {
    float w[18];
#pragma unroll
    for (int j = 0; j < 18; j++) w[j] = halfsum32(v[j], v[j + 18]);
#pragma unroll
    for (int j = 0; j < 9; j++) x[j] = row_sum16(halfsum16(w[j], w[j + 9]));
}

}  // namespace m3s
