// block7.h -- register-resident 7x7 f64 block kernels for the multi-launch block elimination
// (gn_sparse.hip; gn_solve.hip keeps its own copies inside its single-workgroup kernel).
//
// A pose's 7x7 diagonal block is factored serially in the registers of every lane that needs
// it (no cross-lane traffic on the pivot chain); L is kept packed lower (28 doubles) with the
// reciprocal diagonal beside it.  Failure semantics follow SimplicialLLT (reference
// gn_kernels.cu:142-150 via Eigen): a pivot <= 0 fails, NaN passes.
#pragma once

#include <hip/hip_runtime.h>

namespace m3s {
namespace b7 {

__host__ __device__ constexpr int pk(int i, int j) { return i * (i + 1) / 2 + j; }  // packed lower

// 1/sqrt(d) to f64 accuracy: v_rsq_f64 + one Newton step (d <= 0 / NaN propagate)
__device__ __forceinline__ double rsqrt_f64(double d) {
    const double y = __builtin_amdgcn_rsq(d);
    return y * fma(-0.5 * d * y, y, 1.5);
}

// a (packed lower) -> L in place, inv[i] = 1 / L_ii
__device__ __forceinline__ void chol7(double (&a)[28], double (&inv)[7], bool& bad) {
#pragma unroll
    for (int p = 0; p < 7; p++) {
        const double d = a[pk(p, p)];
        bad |= (d <= 0.0);
        const double y = rsqrt_f64(d);
        inv[p] = y;
        a[pk(p, p)] = d * y;
#pragma unroll
        for (int i = p + 1; i < 7; i++) a[pk(i, p)] *= y;
#pragma unroll
        for (int i = p + 1; i < 7; i++)
#pragma unroll
            for (int j = p + 1; j <= i; j++) a[pk(i, j)] = fma(-a[pk(i, p)], a[pk(j, p)], a[pk(i, j)]);
    }
}

// out = L^-1 in (forward substitution), column-oriented: each solved entry is applied to all
// later ones at once, so the dependent chain is 2 ops per entry (14), not up to 7 (28) -- on the
// pivot chain of every pose step (a dependent f64 op costs tens of cycles on one wave)
__device__ __forceinline__ void fwd7(const double (&L)[28], const double (&inv)[7],
                                     const double (&in)[7], double (&out)[7]) {
    double s[7];
#pragma unroll
    for (int c = 0; c < 7; c++) s[c] = in[c];
#pragma unroll
    for (int c = 0; c < 7; c++) {
        out[c] = s[c] * inv[c];
#pragma unroll
        for (int r = c + 1; r < 7; r++) s[r] = fma(-L[pk(r, c)], out[c], s[r]);
    }
}

// z <- L^-T z (backward substitution), column-oriented like fwd7
__device__ __forceinline__ void bwd7(const double (&L)[28], const double (&inv)[7], double (&z)[7]) {
#pragma unroll
    for (int c = 6; c >= 0; c--) {
        z[c] *= inv[c];
#pragma unroll
        for (int m = 0; m < c; m++) z[m] = fma(-L[pk(c, m)], z[c], z[m]);
    }
}

}  // namespace b7
}  // namespace m3s
