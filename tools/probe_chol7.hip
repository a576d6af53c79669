// Unit probe of the wave-level 7x7 Cholesky (chol7) and forward substitution (fwd7) of
// gn_solve.hip against a host f64 Cholesky.
#include "../mast3r-slam_amd/csrc/gn_solve.hip"
#include <cmath>
#include <cstdio>
using namespace m3s;
__global__ void kchol(const double* A, double* Lout, int* badout) {
    const int lane = threadIdx.x;
    double r[7], inv = 0.0;
    bool bad = false;
    for (int j = 0; j < 7; j++) r[j] = (lane < 7 && j <= lane) ? A[lane * 7 + j] : 0.0;
    chol7(r, inv, lane, bad);
    if (lane < 7) {
        for (int j = 0; j < 7; j++) Lout[lane * 8 + j] = j <= lane ? r[j] : 0.0;
        Lout[56 + lane] = inv;
    }
    if (lane == 0) badout[0] = bad;
}
int main() {
    double M[49], A[49];
    unsigned s = 1;
    for (int i = 0; i < 49; i++) { s = s * 1103515245u + 12345u; M[i] = ((s >> 8) % 1000) / 500.0 - 1.0; }
    for (int i = 0; i < 7; i++) for (int j = 0; j < 7; j++) {
        double v = (i == j) ? 3.0 : 0.0; for (int k = 0; k < 7; k++) v += M[i * 7 + k] * M[j * 7 + k]; A[i * 7 + j] = v; }
    double L[49] = {0};
    for (int j = 0; j < 7; j++) {
        double d = A[j * 7 + j]; for (int k = 0; k < j; k++) d -= L[j * 7 + k] * L[j * 7 + k];
        L[j * 7 + j] = sqrt(d);
        for (int i = j + 1; i < 7; i++) { double t = A[i * 7 + j]; for (int k = 0; k < j; k++) t -= L[i * 7 + k] * L[j * 7 + k]; L[i * 7 + j] = t / L[j * 7 + j]; }
    }
    double *dA, *dL; int* dB;
    (void)hipMalloc(&dA, 49 * 8); (void)hipMalloc(&dL, 64 * 8); (void)hipMalloc(&dB, 4);
    (void)hipMemcpy(dA, A, 49 * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(kchol, dim3(1), dim3(64), 0, 0, dA, dL, dB);
    double G[64]; int bad;
    (void)hipMemcpy(G, dL, 64 * 8, hipMemcpyDeviceToHost); (void)hipMemcpy(&bad, dB, 4, hipMemcpyDeviceToHost);
    double err = 0;
    for (int i = 0; i < 7; i++) for (int j = 0; j <= i; j++) err = fmax(err, fabs(G[i * 8 + j] - L[i * 7 + j]));
    for (int i = 0; i < 7; i++) err = fmax(err, fabs(G[56 + i] - 1.0 / L[i * 7 + i]));
    printf("chol7: bad=%d max|L_gpu - L_host| = %.3e\n", bad, err);
    for (int i = 0; i < 7; i++) { for (int j = 0; j < 7; j++) printf("%9.5f/%9.5f ", G[i*8+j], L[i*7+j]); printf("\n"); }
    return 0;
}
