// Probe of the v_mfma_f64_16x16x4_f64 operand / result lane maps on gfx950 (exact integer data,
// asymmetric operands).  Prints which C/D row formula matches a host GEMM.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ void k(const double* A, const double* B, double* out) {
    const int l = threadIdx.x;
    d4 acc = {0, 0, 0, 0};
    // A 16x4 row-major, B 4x16 row-major; lane l supplies A[l&15][l>>4], B[l>>4][l&15]
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[(l & 15) * 4 + (l >> 4)], B[(l >> 4) * 16 + (l & 15)], acc, 0, 0, 0);
    for (int r = 0; r < 4; r++) out[l * 4 + r] = acc[r];
}
int main() {
    double A[64], B[64], C[256], out[256];
    for (int i = 0; i < 64; i++) { A[i] = (i * 7 + 3) % 11 - 5; B[i] = (i * 5 + 1) % 13 - 6; }
    for (int i = 0; i < 16; i++) for (int j = 0; j < 16; j++) {
        double s = 0; for (int k = 0; k < 4; k++) s += A[i * 4 + k] * B[k * 16 + j]; C[i * 16 + j] = s; }
    double *dA, *dB, *dO;
    hipMalloc(&dA, 512); hipMalloc(&dB, 512); hipMalloc(&dO, 2048);
    hipMemcpy(dA, A, 512, hipMemcpyHostToDevice); hipMemcpy(dB, B, 512, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dO);
    hipMemcpy(out, dO, 2048, hipMemcpyDeviceToHost);
    int bad1 = 0, bad2 = 0;
    for (int l = 0; l < 64; l++) for (int r = 0; r < 4; r++) {
        const int col = l & 15;
        if (out[l * 4 + r] != C[((l >> 4) + 4 * r) * 16 + col]) bad1++;   // row = (l>>4) + 4r
        if (out[l * 4 + r] != C[(4 * (l >> 4) + r) * 16 + col]) bad2++;   // row = 4(l>>4) + r
    }
    printf("mfma_f64_16x16x4 C/D map: row=(lane>>4)+4r mismatches %d, row=4(lane>>4)+r mismatches %d\n", bad1, bad2);
    return 0;
}
