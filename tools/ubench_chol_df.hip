// Diagnostic: timeline of the dataflow tile LL^T (chol_df.hip) on a random SPD system of
// npad unknowns (+ the RHS border tile): per tile column j, when the diagonal tile started,
// finished its updates, finished potrf + inverse and published, and the same for tile (j+1, j)
// (the critical path is diag(j) -> trsm(j+1, j) -> last update of diag(j+1)).  Also checks
// L L^T = A and the forward substitution against a host f64 Cholesky.
#define M3S_DF_STAMPS 1
#include "../mast3r-slam_amd/csrc/chol_df.hip"

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#define CK(x)                                                                \
    do {                                                                     \
        hipError_t e_ = (x);                                                 \
        if (e_ != hipSuccess) {                                              \
            printf("%s: %s\n", #x, hipGetErrorString(e_));                  \
            return 1;                                                        \
        }                                                                    \
    } while (0)

int main(int argc, char** argv) {
    using namespace m3s;
    const int npad = argc > 1 ? atoi(argv[1]) : 1024;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    const int nt = npad / 64;
    const size_t rows = (size_t)npad + 64;
    std::vector<double> H(rows * npad, 0.0);
    std::mt19937_64 rng(7);
    std::normal_distribution<double> nd;
    // A = B B^T / npad + I (SPD, well conditioned), b random
    std::vector<double> B((size_t)npad * 32);
    for (auto& v : B) v = nd(rng);
    for (int r = 0; r < npad; r++)
        for (int c = 0; c <= r; c++) {
            double s = 0;
            for (int k = 0; k < 32; k++) s += B[(size_t)r * 32 + k] * B[(size_t)c * 32 + k];
            s = s / 32.0 + (r == c ? 1.0 : 0.0);
            H[(size_t)r * npad + c] = H[(size_t)c * npad + r] = s;
        }
    for (int c = 0; c < npad; c++) H[(size_t)npad * npad + c] = nd(rng);
    double *dH, *dH0, *dLinv, *dX;
    int *dflags;
    long long* dtr;
    const int ntiles = num_tasks(nt);
    CK(hipMalloc(&dH, H.size() * 8));
    CK(hipMalloc(&dH0, H.size() * 8));
    CK(hipMalloc(&dLinv, chol_linv_bytes(npad)));
    CK(hipMalloc(&dX, npad * 8));
    CK(hipMalloc(&dflags, 64 * 4));
    CK(hipMalloc(&dtr, (ntiles * 4 + 32 + 12 * nt) * 8));
    CK(hipMemset(dtr, 0, (ntiles * 4 + 32 + 8 * nt) * 8));
    CK(hipMemcpy(dH0, H.data(), H.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemset(dflags, 0, 64 * 4));
    CK(hipMemset(chol_ready_ptr(dLinv, npad), 0, chol_ready_bytes(npad)));
    std::vector<long long> tr(ntiles * 4 + 32 + 12 * nt);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int rep = 1; rep <= reps; rep++) {
        CK(hipMemcpy(dH, dH0, H.size() * 8, hipMemcpyDeviceToDevice));
        DfArgs a{};
        a.Hd = dH;
        a.Linv = dLinv;
        a.ready = chol_ready_ptr(dLinv, npad);
        a.flags = dflags;
        a.npad = npad;
        a.nt = nt;
        a.ntiles = ntiles;
        a.epoch = rep;
        a.spin_limit = 1 << 22;
        a.trace = dtr;
        a.x = dX;
        a.xg = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(a.ready) + chol_words_bytes(npad));
        a.xgran = 1;
        a.tick = a.ready + chol_nwords(npad);
        a.dyn = getenv("M3S_DF_DYN") ? atoi(getenv("M3S_DF_DYN")) : 1;
        int per = 0, ncu = 0;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)chol_df_kernel, NT, 0));
        CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
        const int grid = std::min(ntiles + 1, per * ncu);
        void* kargs[] = {&a};
        CK(hipEventRecord(e0, 0));
        (void)kargs;  // a plain launch, as the product (chol_df.hip launch_dense_factor_solve)
        hipLaunchKernelGGL(chol_df_kernel, dim3(grid), dim3(NT), 0, 0, a);
        CK(hipGetLastError());
        CK(hipEventRecord(e1, 0));
        CK(hipDeviceSynchronize());
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("rep %d: grid %d tiles %d  event %.1f us\n", rep, grid, ntiles, ms * 1e3);
    }
    CK(hipMemcpy(tr.data(), dtr, tr.size() * 8, hipMemcpyDeviceToHost));
    long long t0 = tr[0];
    for (int t = 0; t < ntiles; t++) t0 = std::min(t0, tr[4 * t]);
    const long long* ct = tr.data() + 4 * ntiles + 32;
    t0 = ct[0];
    printf("C chain (us from its start): P(j) loaded / trsm + update done / potrf done\n");
    for (int j = 0; j < nt; j++)
        printf("col %2d  C %7.2f %7.2f %7.2f\n", j, (ct[4 * j] - t0) * 0.01, (ct[4 * j + 1] - t0) * 0.01,
               (ct[4 * j + 2] - t0) * 0.01);
    printf("C end %.2f\n", (ct[4 * (nt - 1) + 3] - t0) * 0.01);
    printf("back-substitution pairs (us from the chain's start): loaded / all x in / x_jh / published\n");
    for (int p = 0; p < (nt + 1) / 2; p++) {
        const long long* b = ct + 8 * nt + 4 * p;
        printf("  pair %2d (%2d,%2d) %8.2f %8.2f %8.2f %8.2f\n", p, nt - 1 - 2 * p, nt - 2 - 2 * p, (b[0] - t0) * 0.01,
               (b[1] - t0) * 0.01, (b[2] - t0) * 0.01, (b[3] - t0) * 0.01);
    }
    printf("per column (us): P loads+staging / L_{j,j-1} GEMM / store+stage / syrk / potrf+inverse / to next\n");
    for (int j = 1; j < nt; j++) {
        const long long* f = ct + 4 * nt + 4 * j;
        const long long nx = j + 1 < nt ? ct[4 * (j + 1)] : ct[4 * (nt - 1) + 3];
        printf("col %2d  %6.2f %6.2f %6.2f %6.2f %6.2f %6.2f\n", j, (f[0] - ct[4 * j]) * 0.01, (f[1] - f[0]) * 0.01,
               (f[2] - f[1]) * 0.01, (f[3] - f[2]) * 0.01, (ct[4 * j + 2] - f[3]) * 0.01, (nx - ct[4 * j + 2]) * 0.01);
    }
    printf("potrf of D_0 (us since its start): ");
    for (int q = 1; q < 18; q++) printf("%.2f ", (tr[4 * ntiles + q] - tr[4 * ntiles]) * 0.01);
    printf("\n");
    // check: forward-substituted border row vs host LL^T
    std::vector<double> L(H.begin(), H.begin() + (size_t)npad * npad), y(npad);
    for (int j = 0; j < npad; j++) {
        double d = L[(size_t)j * npad + j];
        for (int k = 0; k < j; k++) d -= L[(size_t)j * npad + k] * L[(size_t)j * npad + k];
        d = std::sqrt(d);
        L[(size_t)j * npad + j] = d;
        for (int i = j + 1; i < npad; i++) {
            double s = L[(size_t)i * npad + j];
            for (int k = 0; k < j; k++) s -= L[(size_t)i * npad + k] * L[(size_t)j * npad + k];
            L[(size_t)i * npad + j] = s / d;
        }
    }
    for (int i = 0; i < npad; i++) {
        double s = H[(size_t)npad * npad + i];
        for (int k = 0; k < i; k++) s -= L[(size_t)i * npad + k] * y[k];
        y[i] = s / L[(size_t)i * npad + i];
    }
    std::vector<double> Hg(H.size());
    CK(hipMemcpy(Hg.data(), dH, H.size() * 8, hipMemcpyDeviceToHost));
    double err = 0, mx = 0, lerr = 0;
    for (int i = 0; i < npad; i++) {
        err = std::max(err, std::fabs(Hg[(size_t)npad * npad + i] - y[i]));
        mx = std::max(mx, std::fabs(y[i]));
    }
    for (int i = 64; i < npad; i++)
        for (int j = 0; j < (i / 64) * 64; j++)
            lerr = std::max(lerr, std::fabs(Hg[(size_t)i * npad + j] - L[(size_t)i * npad + j]));
    {   // back-substitution L^T x = y
        std::vector<double> x(npad), xg(npad);
        for (int i = npad - 1; i >= 0; i--) {
            double s = y[i];
            for (int k = i + 1; k < npad; k++) s -= L[(size_t)k * npad + i] * x[k];
            x[i] = s / L[(size_t)i * npad + i];
        }
        CK(hipMemcpy(xg.data(), dX, npad * 8, hipMemcpyDeviceToHost));
        double ex = 0, mxx = 0;
        for (int i = 0; i < npad; i++) {
            ex = std::max(ex, std::fabs(xg[i] - x[i]));
            mxx = std::max(mxx, std::fabs(x[i]));
        }
        printf("x max err %.3e (max |x| %.3e)\n", ex, mxx);
    }
    int fl[64];
    CK(hipMemcpy(fl, dflags, sizeof(fl), hipMemcpyDeviceToHost));
    printf("y max err %.3e (max |y| %.3e), off-diagonal L max err %.3e, fail flag %d\n", err, mx, lerr, fl[kFlagFail]);
    return 0;
}
