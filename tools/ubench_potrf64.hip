// Diagnostic: the chain workgroup's 64x64 tile LL^T + inverse (chol_df.hip potrf_inverse) alone,
// one workgroup per tile, with cycle stamps inside every panel step (M3S_DF_STAMPS): when wave 0
// finished its look-ahead trailing update, its panel factor, when wave 3 finished its share, and
// when the step's barrier released.  Checks L L^T = A and Li L = I against the input.
#define M3S_DF_STAMPS 1
#include "../mast3r-slam_amd/csrc/chol_df.hip"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#define CK(x)                                                               \
    do {                                                                    \
        hipError_t e_ = (x);                                                \
        if (e_ != hipSuccess) {                                             \
            printf("%s: %s\n", #x, hipGetErrorString(e_));                 \
            return 1;                                                       \
        }                                                                   \
    } while (0)

namespace m3s {
namespace {
__global__ __launch_bounds__(NT) void k_potrf(const double* __restrict__ A0, double* __restrict__ Lout,
                                              double* __restrict__ Liout, long long* __restrict__ pt,
                                              int* __restrict__ flags) {
    __shared__ __attribute__((aligned(16))) double X[T * LD];
    __shared__ __attribute__((aligned(16))) double Y[T * LD];
    __shared__ __attribute__((aligned(16))) double Z[T * LD];
    __shared__ double Dinv[T];
    const int tid = threadIdx.x;
    const double* A = A0 + (size_t)blockIdx.x * T * T;
    for (int id = tid; id < T * T; id += NT) Z[(id >> 6) * LD + (id & 63)] = A[id];
    for (int id = tid; id < T * LD; id += NT) Y[id] = 0.0;
    __syncthreads();
    long long* p = pt + (size_t)blockIdx.x * 64;
    const long long t0 = (long long)__builtin_amdgcn_s_memtime();
    if (tid == 0) p[60] = t0;
    potrf_inverse(Z, Y, X, Dinv, flags, p, nullptr, 0);
    const long long t1 = (long long)__builtin_amdgcn_s_memtime();
    if (tid == 0) p[61] = t1;
    for (int id = tid; id < T * T; id += NT) {
        Lout[(size_t)blockIdx.x * T * T + id] = Z[(id >> 6) * LD + (id & 63)];
        Liout[(size_t)blockIdx.x * T * T + id] = Y[(id >> 6) * LD + (id & 63)];
    }
}
__global__ __launch_bounds__(NT) void k_potrf_cc(const double* __restrict__ A0, double* __restrict__ Lout,
                                                 double* __restrict__ Liout, long long* __restrict__ pt,
                                                 int* __restrict__ flags) {
    __shared__ __attribute__((aligned(16))) double X[T * LD];
    __shared__ __attribute__((aligned(16))) double Y[T * LD];
    __shared__ __attribute__((aligned(16))) double Z[T * LD];
    __shared__ double Dinv[T];
    __shared__ double Scr[kCcScr];
    __shared__ int Sync[kDfSync];
    const int tid = threadIdx.x;
    const double* A = A0 + (size_t)blockIdx.x * T * T;
    for (int id = tid; id < T * T; id += NT) Z[(id >> 6) * LD + (id & 63)] = A[id];
    for (int id = tid; id < T * LD; id += NT) Y[id] = 0.0;
    if (tid < kDfSync) Sync[tid] = 0;
    __syncthreads();
    long long* p = pt + (size_t)blockIdx.x * 64;
    const long long t0 = (long long)__builtin_amdgcn_s_memtime();
    const long long r0 = (long long)__builtin_amdgcn_s_memrealtime();
    potrf_cc(Z, Y, X, Scr, Sync, Dinv, flags, p);
    const long long t1 = (long long)__builtin_amdgcn_s_memtime();
    const long long r1 = (long long)__builtin_amdgcn_s_memrealtime();
    if (tid == 0) {
        p[60] = t0;
        p[61] = t1;
        p[62] = r1 - r0;
    }
    for (int id = tid; id < T * T; id += NT) {
        Lout[(size_t)blockIdx.x * T * T + id] = Z[(id >> 6) * LD + (id & 63)];
        Liout[(size_t)blockIdx.x * T * T + id] = Y[(id >> 6) * LD + (id & 63)];
    }
}
// latency probes, one wave: a dependent chain of N ops, cycles per op
__global__ __launch_bounds__(64) void k_lat(double* out, long long* cyc, double a, double b) {
    const int lane = threadIdx.x;
    double x = lane * 1e-3 + 1.0;
    long long t0 = (long long)__builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < 64; i++) x = fma(x, a, b);
    long long t1 = (long long)__builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < 64; i++) x = fma(x, rdlane(x, i & 7), b);  // readlane -> fma chain
    long long t2 = (long long)__builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < 32; i++) x = __builtin_amdgcn_rsq(x) + b;  // rsq + add chain
    long long t3 = (long long)__builtin_amdgcn_s_memtime();
    double y[8];
#pragma unroll
    for (int q = 0; q < 8; q++) y[q] = x + q;
#pragma unroll
    for (int i = 0; i < 16; i++)
#pragma unroll
        for (int q = 0; q < 8; q++) y[q] = fma(y[q], a, b);  // 8 independent chains: issue rate
    long long t4 = (long long)__builtin_amdgcn_s_memtime();
    for (int q = 0; q < 8; q++) x += y[q];
    out[lane] = x;
    if (lane == 0) {
        cyc[0] = t1 - t0;
        cyc[1] = t2 - t1;
        cyc[2] = t3 - t2;
        cyc[3] = t4 - t3;
    }
}
}  // namespace
}  // namespace m3s

int main(int argc, char** argv) {
    using namespace m3s;
    const int ntile = argc > 1 ? atoi(argv[1]) : 8;
    std::vector<double> A((size_t)ntile * 4096);
    std::mt19937_64 rng(11);
    std::normal_distribution<double> nd;
    for (int t = 0; t < ntile; t++) {
        std::vector<double> B(64 * 64);
        for (auto& v : B) v = nd(rng);
        for (int r = 0; r < 64; r++)
            for (int c = 0; c <= r; c++) {
                double s = 0;
                for (int k = 0; k < 64; k++) s += B[r * 64 + k] * B[c * 64 + k];
                s = s / 64.0 + (r == c ? 0.5 : 0.0);
                A[(size_t)t * 4096 + r * 64 + c] = A[(size_t)t * 4096 + c * 64 + r] = s;
            }
    }
    {
        double* dout;
        long long* dc;
        CK(hipMalloc(&dout, 64 * 8));
        CK(hipMalloc(&dc, 8 * 8));
        for (int r = 0; r < 3; r++) hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, dout, dc, 0.999, 1e-3);
        CK(hipDeviceSynchronize());
        long long c[4];
        CK(hipMemcpy(c, dc, 32, hipMemcpyDeviceToHost));
        printf("one wave: dependent v_fma_f64 %.1f cyc/op; readlane x2 + fma %.1f cyc/step; rsq_f64 + add %.1f "
               "cyc/step; independent fma_f64 issue %.1f cyc/op\n",
               c[0] / 64.0, c[1] / 64.0, c[2] / 32.0, c[3] / 128.0);
    }
    double *dA, *dL, *dLi;
    long long* dpt;
    int* dfl;
    CK(hipMalloc(&dA, A.size() * 8));
    CK(hipMalloc(&dL, A.size() * 8));
    CK(hipMalloc(&dLi, A.size() * 8));
    CK(hipMalloc(&dpt, (size_t)ntile * 64 * 8));
    CK(hipMalloc(&dfl, 64 * 4));
    CK(hipMemset(dfl, 0, 64 * 4));
    CK(hipMemset(dpt, 0, (size_t)ntile * 64 * 8));
    CK(hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice));
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(k_potrf, dim3(ntile), dim3(NT), 0, 0, dA, dL, dLi, dpt, dfl);
        CK(hipDeviceSynchronize());
    }
    std::vector<double> L(A.size()), Li(A.size());
    std::vector<long long> pt((size_t)ntile * 64);
    CK(hipMemcpy(L.data(), dL, A.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(Li.data(), dLi, A.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(pt.data(), dpt, pt.size() * 8, hipMemcpyDeviceToHost));
    double eLL = 0, eLi = 0;
    for (int t = 0; t < ntile; t++) {
        const double* a = &A[(size_t)t * 4096];
        const double* l = &L[(size_t)t * 4096];
        const double* li = &Li[(size_t)t * 4096];
        for (int r = 0; r < 64; r++)
            for (int c = 0; c <= r; c++) {
                double s = 0, u = 0;
                for (int k = 0; k <= c; k++) s += l[r * 64 + k] * l[c * 64 + k];
                for (int k = c; k <= r; k++) u += li[r * 64 + k] * l[k * 64 + c];
                eLL = std::max(eLL, std::fabs(s - a[r * 64 + c]));
                eLi = std::max(eLi, std::fabs(u - (r == c ? 1.0 : 0.0)));
            }
    }
    printf("max |L L^T - A| %.3e, max |Li L - I| %.3e\n", eLL, eLi);
    auto check = [&](const char* name) {
        double e1 = 0, e2 = 0;
        for (int t = 0; t < ntile; t++) {
            const double* a = &A[(size_t)t * 4096];
            const double* l = &L[(size_t)t * 4096];
            const double* li = &Li[(size_t)t * 4096];
            for (int r = 0; r < 64; r++)
                for (int c = 0; c <= r; c++) {
                    double s = 0, u = 0;
                    for (int k = 0; k <= c; k++) s += l[r * 64 + k] * l[c * 64 + k];
                    for (int k = c; k <= r; k++) u += li[r * 64 + k] * l[k * 64 + c];
                    e1 = std::max(e1, std::fabs(s - a[r * 64 + c]));
                    e2 = std::max(e2, std::fabs(u - (r == c ? 1.0 : 0.0)));
                }
            for (int r = 0; r < 64; r++)
                for (int c = r + 1; c < 64; c++) e2 = std::max(e2, std::fabs(li[r * 64 + c]));  // upper Li must be 0
        }
        unsigned long long hsh = 0;  // bit pattern digest of L and Li (variants that claim bitwise equality)
        for (size_t k = 0; k < L.size(); k++) {
            unsigned long long u, v;
            memcpy(&u, &L[k], 8);
            memcpy(&v, &Li[k], 8);
            hsh = (hsh ^ u) * 0x100000001b3ull;
            hsh = (hsh ^ v) * 0x100000001b3ull;
        }
        printf("%s: max |L L^T - A| %.3e, max |Li L - I| (and upper Li) %.3e, digest %016llx\n", name, e1, e2, hsh);
    };
    CK(hipMemset(dpt, 0, (size_t)ntile * 64 * 8));
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(k_potrf_cc, dim3(ntile), dim3(NT), 0, 0, dA, dL, dLi, dpt, dfl);
        CK(hipDeviceSynchronize());
    }
    std::vector<long long> pc((size_t)ntile * 64);
    CK(hipMemcpy(L.data(), dL, A.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(Li.data(), dLi, A.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(pc.data(), dpt, pc.size() * 8, hipMemcpyDeviceToHost));
    check("potrf_cc");
    {
        long long tc = 0, rc = 0;
        for (int t = 0; t < ntile; t++) {
            tc += pc[(size_t)t * 64 + 61] - pc[(size_t)t * 64 + 60];
            rc += pc[(size_t)t * 64 + 62];
        }
        printf("potrf_cc: mean %.0f cycles, %.2f us (s_memrealtime)\n", (double)tc / ntile, rc * 0.01 / ntile);
        printf("potrf_cc tile 0, cycles from start: wave: applied / factored / diag-inv start / X_ww / X_Vw...\n");
        for (int w = 0; w < 4; w++) {
            printf("  wave %d:", w);
#if M3S_DF_BC
            for (int k = 1; k <= 6; k++) printf(" %7lld", pc[8 * w + k] - pc[60]);  // batches lb 0-3 / X_ww / end
#else
            for (int k = 1; k < 4 + 3 - w; k++) printf(" %7lld", pc[8 * w + k] - pc[60]);
#endif
            printf("\n");
        }
        printf("  end: %lld\n", pc[61] - pc[60]);
#if M3S_DF_BC && M3S_DF_BSTAMPS
        printf("per batch (cycles): previous publish -> wait done -> critical apply done -> publish\n");
        for (int nb = 1; nb < 16; nb++) {
            auto pub = [&](int b) { return pc[8 * (b & 3) + 1 + (b >> 2)]; };
            printf("  batch %2d: %5lld %5lld %5lld\n", nb, pc[20 + 2 * nb] - pub(nb - 1),
                   pc[21 + 2 * nb] - pc[20 + 2 * nb], pub(nb) - pc[21 + 2 * nb]);
        }
        printf("inverse (cycles from start): wave: written-wait done / X_ww done / end\n");
        for (int w = 0; w < 4; w++)
            printf("  wave %d: %6lld %6lld %6lld\n", w, pc[52 + w] - pc[60], pc[8 * w + 5] - pc[60], pc[8 * w + 6] - pc[60]);
#endif
    }
    // cycles (s_memtime) for tile 0: per panel step, relative to the previous step's barrier
    const long long* p = &pt[0];
    long long prev = p[60];
    printf("total %lld cycles (%.2f us at 2.4 GHz)\n", p[61] - p[60], (p[61] - p[60]) / 2400.0);
    printf("step : w0 trail  w0 factor  w3 done  barrier (cycles since the previous barrier)\n");
    for (int s = 0; s < 7; s++) {
        printf("  %d  : %7lld %9lld %8lld %8lld\n", s, p[20 + 4 * s] - prev, p[21 + 4 * s] - prev,
               p[22 + 4 * s] - prev, p[23 + 4 * s] - prev);
        prev = p[23 + 4 * s];
    }
    printf("after the steps: inverse stages %lld cycles\n", p[61] - prev);
    long long tot = 0;
    for (int t = 0; t < ntile; t++) tot += pt[(size_t)t * 64 + 61] - pt[(size_t)t * 64 + 60];
    printf("mean over %d tiles: %.0f cycles\n", ntile, (double)tot / ntile);
    return 0;
}
