// keyframe.hip -- point-map fusion of a keyframe with a newly registered observation (gfx950).
//
// Replaces Frame.update_pointmap (reference mast3r_slam/frame.py:41-105) for the filtering
// modes that are per-point arithmetic, fused with the Sim3 transform the tracker applies
// first (tracker.py:98-99: Xkk = T_CkCf.act(Xkf); keyframe.update_pointmap(Xkk, Ckf)):
//   weighted_pointmap  X <- ((C X) + (Cn Xn)) / (C + Cn),  C <- C + Cn   (frame.py:74-77)
//   indep_conf         where Cn > C: X <- Xn, C <- Cn                  (frame.py:69-73)
//   recent             X <- Xn, C <- Cn                                 (frame.py:58-61)
// torch runs weighted_pointmap as 5 elementwise kernels over [HW,3] / [HW,1] tensors (plus
// the act); here one pass reads X, C, Xn, Cn and writes X, C: 32 B per point.  Each f32
// operation is the same as torch's and nothing is contracted (-ffp-contract=off in the
// Makefile), so the update is bit-exact against the torch expression on the same inputs.
#include <hip/hip_runtime.h>

#include "../../include/m3s_backend.h"
#include "m3s_common.h"
#include "sim3.h"

#pragma clang fp contract(off)

namespace m3s {
namespace {

constexpr int kKfThreads = 256;

template <int MODE, bool ACT>
__global__ __launch_bounds__(kKfThreads) void pointmap_update_kernel(
    const float* __restrict__ T, const float* __restrict__ Xn, const float* __restrict__ Cn,
    float* __restrict__ X, float* __restrict__ C, int64_t HW) {
    float t[3], q[4], s = 1.0f;
    if constexpr (ACT) {
        t[0] = T[0]; t[1] = T[1]; t[2] = T[2];
        q[0] = T[3]; q[1] = T[4]; q[2] = T[5]; q[3] = T[6];
        s = T[7];
    }
    const int64_t stride = (int64_t)gridDim.x * kKfThreads;
    for (int64_t n = (int64_t)blockIdx.x * kKfThreads + threadIdx.x; n < HW; n += stride) {
        float xn[3] = {Xn[3 * n], Xn[3 * n + 1], Xn[3 * n + 2]};
        if constexpr (ACT) {  // lietorch act: s R(q) p + t
            float r[3];
            act_so3(q, xn, r);
            xn[0] = s * r[0] + t[0];
            xn[1] = s * r[1] + t[1];
            xn[2] = s * r[2] + t[2];
        }
        const float cn = Cn[n];
        if constexpr (MODE == M3S_FILTER_WEIGHTED_POINTMAP) {
            const float c = C[n];
            const float den = c + cn;
#pragma unroll
            for (int k = 0; k < 3; k++) X[3 * n + k] = ((c * X[3 * n + k]) + (cn * xn[k])) / den;
            C[n] = den;
        } else if constexpr (MODE == M3S_FILTER_INDEP_CONF) {
            if (cn > C[n]) {
#pragma unroll
                for (int k = 0; k < 3; k++) X[3 * n + k] = xn[k];
                C[n] = cn;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 3; k++) X[3 * n + k] = xn[k];
            C[n] = cn;
        }
    }
}

template <int MODE>
hipError_t launch(const float* T, const float* Xn, const float* Cn, float* X, float* C, int64_t HW,
                  hipStream_t st) {
    const int64_t want = (HW + kKfThreads - 1) / kKfThreads;
    const int nb = (int)(want < 2048 ? (want < 1 ? 1 : want) : 2048);
    if (T)
        hipLaunchKernelGGL((pointmap_update_kernel<MODE, true>), dim3(nb), dim3(kKfThreads), 0, st, T,
                           Xn, Cn, X, C, HW);
    else
        hipLaunchKernelGGL((pointmap_update_kernel<MODE, false>), dim3(nb), dim3(kKfThreads), 0, st,
                           T, Xn, Cn, X, C, HW);
    return hipGetLastError();
}

}  // namespace
}  // namespace m3s

extern "C" int m3s_pointmap_update(int mode, const float* T, const float* X_new, const float* C_new,
                                   float* X, float* C, int64_t HW, void* stream) {
    M3S_REQUIRE(HW >= 0, "pointmap_update: negative size");
    if (HW == 0) return M3S_OK;
    M3S_REQUIRE(X_new && C_new && X && C, "pointmap_update: null pointer");
    hipStream_t st = (hipStream_t)stream;
    switch (mode) {
        case M3S_FILTER_WEIGHTED_POINTMAP:
            M3S_HIP_CHECK(m3s::launch<M3S_FILTER_WEIGHTED_POINTMAP>(T, X_new, C_new, X, C, HW, st));
            break;
        case M3S_FILTER_INDEP_CONF:
            M3S_HIP_CHECK(m3s::launch<M3S_FILTER_INDEP_CONF>(T, X_new, C_new, X, C, HW, st));
            break;
        case M3S_FILTER_RECENT:
            M3S_HIP_CHECK(m3s::launch<M3S_FILTER_RECENT>(T, X_new, C_new, X, C, HW, st));
            break;
        default:
            m3s::set_error("pointmap_update: unsupported filtering mode %d", mode);
            return M3S_ERR_INVALID;
    }
    return M3S_OK;
}
