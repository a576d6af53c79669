// Microbenchmark of the 64x64 tile potrf of the multi-launch dense solve (gn_kernels.hip,
// chol_potrf_kernel): phase timings with s_memtime inside one launch, and launch durations.
#include "../mast3r-slam_amd/csrc/gn_kernels.hip"

#include <cmath>
#include <cstdio>
#include <vector>

using namespace m3s;
namespace m3s {
#include "potrf_v2.inc"
}
__global__ __launch_bounds__(512) void potrf_v2_kernel(double* Hd, int npad, double* Linv, int* flags,
                                                        unsigned long long* tt) {
    m3s::pv2::potrf64(Hd, npad, Linv, flags, tt);
}

// instrumented copy of the potrf phases: t[0..] = s_memtime after each phase (thread 0)
__global__ __launch_bounds__(kPotrfThreads) void potrf_timed(double* __restrict__ Hd, int npad, int k,
                                                             double* __restrict__ Linv,
                                                             int* __restrict__ flags,
                                                             unsigned long long* __restrict__ t) {
    __shared__ double A[T][LDP];
    __shared__ double Li[T][LDP];
    __shared__ double Tm[T][LDP];
    const int tid = threadIdx.x;
    unsigned long long t0 = clock64();
    double* Akk = Hd + (int64_t)k * T * npad + (int64_t)k * T;
    for (int id = tid; id < T * T; id += kPotrfThreads) {
        const int r = id >> 6, c = id & 63;
        A[r][c] = (c <= r) ? Akk[(int64_t)r * npad + c] : 0.0;
        Li[r][c] = 0.0;
    }
    __syncthreads();
    if (tid == 0) t[0] = clock64() - t0;
    const int tx = tid & 31, ty = tid >> 5;
    unsigned long long tf = 0, tu = 0;
    for (int s = 0; s < T / 8; s++) {
        const int c0 = 8 * s;
        unsigned long long a0 = clock64();
        if (tid < T && tid >= c0) {
            const int r = tid;
            double D[8][8], arow[8];
#pragma unroll
            for (int i = 0; i < 8; i++)
#pragma unroll
                for (int p = 0; p <= i; p++) D[i][p] = A[c0 + i][c0 + p];
#pragma unroll
            for (int p = 0; p < 8; p++) arow[p] = A[r][c0 + p];
            double l[8][8];
#pragma unroll
            for (int p = 0; p < 8; p++) {
                double dpp = D[p][p];
#pragma unroll
                for (int q = 0; q < p; q++) dpp = fma(-l[p][q], l[p][q], dpp);
                const double inv = rsqrt_f64(dpp);
                l[p][p] = dpp * inv;
#pragma unroll
                for (int i = p + 1; i < 8; i++) {
                    double a_ = D[i][p];
#pragma unroll
                    for (int q = 0; q < p; q++) a_ = fma(-l[i][q], l[p][q], a_);
                    l[i][p] = a_ * inv;
                }
            }
            if (r < c0 + 8) {
                const int i = r - c0;
#pragma unroll
                for (int ii = 0; ii < 8; ii++)
                    if (ii == i)
#pragma unroll
                        for (int p = 0; p <= ii; p++) A[r][c0 + p] = l[ii][p];
            } else {
                double x[8];
#pragma unroll
                for (int p = 0; p < 8; p++) {
                    double a_ = arow[p];
#pragma unroll
                    for (int q = 0; q < p; q++) a_ = fma(-x[q], l[p][q], a_);
                    x[p] = a_ * rcp_f64(l[p][p]);
                }
#pragma unroll
                for (int p = 0; p < 8; p++) A[r][c0 + p] = x[p];
            }
        }
        __syncthreads();
        unsigned long long a1 = clock64();
        const int lo = c0 + 8;
#pragma unroll
        for (int a = 0; a < 4; a++) {
            const int r = ty + 16 * a;
#pragma unroll
            for (int b = 0; b < 2; b++) {
                const int cc = tx + 32 * b;
                if (cc >= lo && cc <= r) {
                    double acc = A[r][cc];
#pragma unroll
                    for (int p = 0; p < 8; p++) acc = fma(-A[r][c0 + p], A[cc][c0 + p], acc);
                    A[r][cc] = acc;
                }
            }
        }
        __syncthreads();
        unsigned long long a2 = clock64();
        tf += a1 - a0;
        tu += a2 - a1;
    }
    if (tid == 0) {
        t[1] = tf;
        t[2] = tu;
    }
    unsigned long long b0 = clock64();
    if (tid < T) Li[tid][tid] = 1.0 / A[tid][tid];
    __syncthreads();
    inverse_stage<1>(A, Li, Tm, tid);
    inverse_stage<2>(A, Li, Tm, tid);
    inverse_stage<4>(A, Li, Tm, tid);
    inverse_stage<8>(A, Li, Tm, tid);
    inverse_stage<16>(A, Li, Tm, tid);
    inverse_stage<32>(A, Li, Tm, tid);
    unsigned long long b1 = clock64();
    double* Lk = Linv + (int64_t)k * T * T;
    for (int id = tid; id < T * T; id += kPotrfThreads) {
        const int r = id >> 6, c = id & 63;
        if (c <= r) Akk[(int64_t)r * npad + c] = A[r][c];
        Lk[id] = (c <= r) ? Li[r][c] : 0.0;
    }
    __syncthreads();
    unsigned long long b2 = clock64();
    if (tid == 0) {
        t[3] = b1 - b0;
        t[4] = b2 - b1;
        t[5] = b2 - t0;
    }
}

int main() {
    const int npad = 320;
    std::vector<double> H((size_t)(npad + 64) * npad, 0.0);
    unsigned s = 7;
    std::vector<double> M((size_t)npad * npad);
    for (auto& v : M) { s = s * 1103515245u + 12345u; v = ((s >> 8) % 2000) / 1000.0 - 1.0; }
    for (int i = 0; i < 64; i++)
        for (int j = 0; j <= i; j++) {
            double v = (i == j) ? 64.0 : 0.0;
            for (int k = 0; k < 64; k++) v += M[(size_t)i * npad + k] * M[(size_t)j * npad + k];
            H[(size_t)i * npad + j] = v;
        }
    double *dH, *dL;
    int* dF;
    unsigned long long* dT;
    (void)hipMalloc(&dH, H.size() * 8);
    (void)hipMalloc(&dL, (size_t)npad * 64 * 8);
    (void)hipMalloc(&dF, 64);
    (void)hipMalloc(&dT, 64 * 8);
    (void)hipMemset(dF, 0, 64);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 3; rep++) {
        (void)hipMemcpy(dH, H.data(), H.size() * 8, hipMemcpyHostToDevice);
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(chol_potrf_kernel, dim3(1), dim3(kPotrfThreads), 0, 0, dH, npad, 0, dL, dF);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        (void)hipMemcpy(dH, H.data(), H.size() * 8, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(potrf_timed, dim3(1), dim3(kPotrfThreads), 0, 0, dH, npad, 0, dL, dF, dT);
        (void)hipDeviceSynchronize();
        unsigned long long t[6];
        (void)hipMemcpy(t, dT, sizeof(t), hipMemcpyDeviceToHost);
        printf("potrf launch %.1f us | timed copy (cycles @2.4GHz): load %llu, factor %llu, update %llu, "
               "inverse %llu, store %llu, total %llu (%.1f us)\n",
               ms * 1000, t[0], t[1], t[2], t[3], t[4], t[5], t[5] / 2400.0);
    }
    // v2: timing and agreement with the current kernel
    std::vector<double> H1(H.size()), H2(H.size()), L1((size_t)npad * 64), L2((size_t)npad * 64);
    (void)hipMemcpy(dH, H.data(), H.size() * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(chol_potrf_kernel, dim3(1), dim3(kPotrfThreads), 0, 0, dH, npad, 0, dL, dF);
    (void)hipMemcpy(H1.data(), dH, H.size() * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(L1.data(), dL, 64 * 64 * 8, hipMemcpyDeviceToHost);
    for (int rep = 0; rep < 3; rep++) {
        (void)hipMemcpy(dH, H.data(), H.size() * 8, hipMemcpyHostToDevice);
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(potrf_v2_kernel, dim3(1), dim3(512), 0, 0, dH, npad, dL, dF, dT);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        unsigned long long t[9];
        (void)hipMemcpy(t, dT, sizeof(t), hipMemcpyDeviceToHost);
        printf("potrf v2 launch %.1f us | cycles: load %llu, factor(w0) %llu, barrier %llu, update %llu, inverse %llu, store %llu | sub-panel 0: lds %llu chol %llu inv %llu\n",
               ms * 1000, t[0], t[1], t[2], t[3], t[4], t[5], t[6], t[7], t[8]);
    }
    (void)hipMemcpy(H2.data(), dH, H.size() * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(L2.data(), dL, 64 * 64 * 8, hipMemcpyDeviceToHost);
    double eL = 0, eI = 0, sL = 0, sI = 0;
    for (int r = 0; r < 64; r++)
        for (int c = 0; c <= r; c++) {
            eL = fmax(eL, fabs(H1[(size_t)r * npad + c] - H2[(size_t)r * npad + c]));
            sL = fmax(sL, fabs(H1[(size_t)r * npad + c]));
            eI = fmax(eI, fabs(L1[r * 64 + c] - L2[r * 64 + c]));
            sI = fmax(sI, fabs(L1[r * 64 + c]));
        }
    printf("v2 vs current: max|dL|/max|L| = %.2e, max|dLi|/max|Li| = %.2e\n", eL / sL, eI / sI);
    return 0;
}
