// gn_pcg.hip -- the GN step off the factorisation's critical path (round 6).
//
// The reference factors every iteration's normal equations on the host (SimplicialLLT,
// gn_kernels.cu:132-153, called per iteration at :1199-1209).  Here iterations 0 and 1 keep the
// direct block-sparse factorisation (gn_sparse.hip rounds + chol_df.hip core); from iteration 2
// on the step is solved by conjugate gradients preconditioned with the inverse of iteration 1's
// system, M = A_1^-1, applied as a dense matrix-vector product:
//   * sp_inverse_kernel: X = A_1^-1 column block by column block through iteration 1's factor
//     (the elimination rounds' L_v / W_rv and the core's L tiles and tile inverses), 64
//     right-hand sides per workgroup, lane = column: forward rounds (nodes, then the RHS targets
//     of the round), the core forward and back substitution as 64x64 f64-MFMA tile products,
//     the back rounds.  Once per call, after iteration 1's solve.
//   * pcg_kernel: one launch per iteration, nwg workgroups, workgroup w holding rows R_w of X in
//     LDS (f32: a preconditioner needs no more).  Every workgroup keeps the full CG vectors
//     (entry e in thread e % 256) and computes q = A p itself from the block-format system in L2;
//     the one exchange per CG step is z = M r -- each workgroup publishes its rows of z as
//     data-tagged granules (MI355X_MICROARCH.md handoff-1to1 / allgather rows; Guideline 16 R2)
//     and gathers the others'.  The scalars are formed redundantly in the same fixed order, so
//     every workgroup takes the same decisions and holds bitwise the same vectors.  Converged:
//     workgroup 0 retracts (gn_retract_kernel's arithmetic) and sets kFlagSkipSolve, so the
//     direct solve's launches enqueued behind it return at once; a CG breakdown (p'Ap <= 0 or not
//     finite), no convergence within kmax steps or a timed-out gather leave kFlagSkipSolve clear:
//     the direct solve runs for that iteration (SimplicialLLT's semantics, failures included).
// Probes of the full-size systems (tools/r06/pcg_probe_full.py, the oracle's systems): with
// M = A_1^-1, iterations 2..9 of cfg3 / cfg4 reach a relative error of 1e-6 in 3-5 CG steps; the
// iteration-0 inverse needs 21-26 (the system changes most between iterations 0 and 1).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "block7.h"
#include "gn_kernels.h"
#include "sim3.h"

namespace m3s {

namespace {

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int T = kCholTile;  // 64
constexpr int LDT = 73;       // LDS tile row stride in doubles (as chol_df.hip: conflict-free MFMA operand reads)
constexpr int NTH = 256;

__device__ __forceinline__ double ld_coh(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void stores_done() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ d4 mfma(double a, double b, d4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// acc[i][c] += sgn * sum_k Xt[i][k] Yt[c][k] for 64 x 64 LDS tiles (stride LDT).  Wave w holds
// rows 16w .. 16w+15: acc[J][e] = element (16w + (lane >> 4) + 4e, 16J + (lane & 15)).
__device__ __forceinline__ void tile_gemm_nt(const double* X, const double* Y, d4 acc[4], double sgn) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = lane & 15, kq = lane >> 4;
    const double* xr = X + (16 * w + r) * LDT + kq;
    const double* yr = Y + r * LDT + kq;
#pragma unroll
    for (int s = 0; s < 16; s++) {
        const double a = sgn * xr[4 * s];
        double b[4];
#pragma unroll
        for (int J = 0; J < 4; J++) b[J] = yr[16 * J * LDT + 4 * s];
#pragma unroll
        for (int J = 0; J < 4; J++) acc[J] = mfma(a, b[J], acc[J]);
    }
}
__device__ __forceinline__ int acc_row(int e) { return 16 * (threadIdx.x >> 6) + ((threadIdx.x & 63) >> 4) + 4 * e; }
__device__ __forceinline__ int acc_col(int J) { return 16 * J + (threadIdx.x & 15); }

}  // namespace

// ---------------------------------------------------------------------------------------------
// X = A^-1 through the factor of the last direct solve
// ---------------------------------------------------------------------------------------------
namespace {

// the core's dense index gi (< 7 ntail) -> its row of the system (pose-major, 7 per pose)
__device__ __forceinline__ int core_row(const int* tail, int gi) { return 7 * tail[gi / 7] + gi % 7; }

__global__ __launch_bounds__(NTH) void sp_inverse_kernel(InvArgs a) {
    // the call has converged (no PCG iteration follows), or this iteration's PCG converged (no
    // new factor: M stays)
    if (a.flags[kFlagDone] || a.flags[kFlagSkipSolve]) return;
    __shared__ __attribute__((aligned(16))) double S0[T * LDT];
    __shared__ __attribute__((aligned(16))) double S1[T * LDT];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int n = a.n;
    const int64_t ldx = a.ldx;
    double* Xc = a.X + (int64_t)blockIdx.x * T;  // this workgroup's 64 columns; lane = column
    const int col = blockIdx.x * T + lane;
    // B = I
    for (int row = w; row < n; row += 4) Xc[row * ldx + lane] = row == col ? 1.0 : 0.0;
    stores_done();
    __syncthreads();
    auto ldrow7 = [&](int pose, double (&v)[7]) {
#pragma unroll
        for (int d = 0; d < 7; d++) v[d] = ld_coh(Xc + (int64_t)(7 * pose + d) * ldx + lane);
    };
    auto strow7 = [&](int pose, const double (&v)[7]) {
#pragma unroll
        for (int d = 0; d < 7; d++) Xc[(int64_t)(7 * pose + d) * ldx + lane] = v[d];
    };
    auto ldL = [&](int q, double (&L)[28], double (&inv)[7]) {
        const double* Ls = a.Lstore + (int64_t)q * kLStoreRec;
#pragma unroll
        for (int k = 0; k < 28; k++) L[k] = Ls[k];
#pragma unroll
        for (int k = 0; k < 7; k++) inv[k] = Ls[28 + k];
    };
    // ---- forward through the elimination rounds: Y_v = L_v^-1 B_v, then B_r -= W_rv Y_v per RHS target
    for (int rd = 0; rd < a.nrounds; rd++) {
        const int* R = a.rounds + 8 * rd;  // node_begin, nnodes, tbeg, nbt, rbeg, nrt, wbeg, wcount
        const int nb = R[0], nn = R[1];
        for (int q = nb + w; q < nb + nn; q += 4) {
            double L[28], inv[7], bv[7], yv[7];
            ldL(q, L, inv);
            ldrow7(a.nodes[q], bv);
            b7::fwd7(L, inv, bv, yv);
            strow7(a.nodes[q], yv);
        }
        stores_done();
        __syncthreads();
        const int* recs = a.inl + (int64_t)(R[2] + R[4] + R[3]) * kSpRec;  // this round's RHS targets
        for (int t = w; t < R[5]; t += 4) {
            const int* rec = recs + (int64_t)t * kSpRec;
            const int tgt = rec[0], c0 = rec[1], cnt = rec[2] - rec[1];
            if (tgt < 0) continue;  // (poses without fronts)
            double br[7];
            ldrow7(tgt, br);
            for (int j = 0; j < cnt; j++) {
                const int* C = j < kSpInline ? rec + 4 + 4 * j : a.rc4 + 4 * (int64_t)(c0 + j);
                const int v = C[0], wid = C[2];
                double yv[7];
                ldrow7(v, yv);
                const double* Wr = a.W + (int64_t)wid * 49;
#pragma unroll
                for (int i = 0; i < 7; i++)
#pragma unroll
                    for (int m = 0; m < 7; m++) br[i] = fma(-Wr[i * 7 + m], yv[m], br[i]);
            }
            strow7(tgt, br);
        }
        stores_done();
        __syncthreads();
    }
    // ---- the core: forward then back substitution with its 64 x 64 tiles (chol_df.hip layout)
    const int nt = a.npad / T, ncore = 7 * a.ntail;
    auto load_rows_T = [&](double* S, int k) {  // S[c][m] = B[core row k*64+m][c] (0 past the core)
        for (int id = tid; id < T * T; id += NTH) {
            const int m = id >> 6, c = id & 63, gi = k * T + m;
            S[c * LDT + m] = gi < ncore ? ld_coh(Xc + (int64_t)core_row(a.tail, gi) * ldx + c) : 0.0;
        }
    };
    auto load_tile = [&](double* S, const double* src, int64_t ld, bool trans) {  // S[i][m] = src[i][m] or src[m][i]
        for (int id = tid; id < T * T; id += NTH) {
            const int i = id >> 6, m = id & 63;
            if (trans) S[m * LDT + i] = src[(int64_t)i * ld + m];
            else S[i * LDT + m] = src[(int64_t)i * ld + m];
        }
    };
    auto acc_load = [&](d4 acc[4], int j) {
#pragma unroll
        for (int J = 0; J < 4; J++)
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const int gi = j * T + acc_row(e);
                acc[J][e] = gi < ncore ? ld_coh(Xc + (int64_t)core_row(a.tail, gi) * ldx + acc_col(J)) : 0.0;
            }
    };
    auto acc_store = [&](const d4 acc[4], int j) {
#pragma unroll
        for (int J = 0; J < 4; J++)
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const int gi = j * T + acc_row(e);
                if (gi < ncore) Xc[(int64_t)core_row(a.tail, gi) * ldx + acc_col(J)] = acc[J][e];
            }
    };
    auto acc_to_lds_T = [&](double* S, const d4 acc[4]) {  // S[c][i] = acc[i][c]
#pragma unroll
        for (int J = 0; J < 4; J++)
#pragma unroll
            for (int e = 0; e < 4; e++) S[acc_col(J) * LDT + acc_row(e)] = acc[J][e];
    };
    // out = Li * acc (Li = Linv_j, or its transpose), via S0 / S1
    auto apply_inv = [&](d4 acc[4], int j, bool trans) {
        __syncthreads();
        acc_to_lds_T(S1, acc);
        load_tile(S0, a.Linv + (int64_t)j * T * T, T, trans);
        __syncthreads();
#pragma unroll
        for (int J = 0; J < 4; J++) acc[J] = d4{0.0, 0.0, 0.0, 0.0};
        tile_gemm_nt(S0, S1, acc, 1.0);
    };
    for (int j = 0; j < nt; j++) {  // Y_j = Linv_j (B_j - sum_{k<j} L_jk Y_k)
        d4 acc[4];
        acc_load(acc, j);
        for (int k = 0; k < j; k++) {
            __syncthreads();
            load_tile(S0, a.Hd + (int64_t)j * T * a.npad + (int64_t)k * T, a.npad, false);
            load_rows_T(S1, k);
            __syncthreads();
            tile_gemm_nt(S0, S1, acc, -1.0);
        }
        apply_inv(acc, j, false);
        acc_store(acc, j);
        stores_done();
        __syncthreads();
    }
    for (int j = nt - 1; j >= 0; j--) {  // X_j = Linv_j^T (Y_j - sum_{k>j} L_kj^T X_k)
        d4 acc[4];
        acc_load(acc, j);
        for (int k = j + 1; k < nt; k++) {
            __syncthreads();
            load_tile(S0, a.Hd + (int64_t)k * T * a.npad + (int64_t)j * T, a.npad, true);
            load_rows_T(S1, k);
            __syncthreads();
            tile_gemm_nt(S0, S1, acc, -1.0);
        }
        apply_inv(acc, j, true);
        acc_store(acc, j);
        stores_done();
        __syncthreads();
    }
    // ---- back through the rounds, last first: X_v = L_v^-T (Y_v - sum_r W_rv^T X_r)
    for (int rd = a.nrounds - 1; rd >= 0; rd--) {
        const int* R = a.rounds + 8 * rd;
        const int nb = R[0], nn = R[1];
        for (int q = nb + w; q < nb + nn; q += 4) {
            double L[28], inv[7], z[7];
            ldL(q, L, inv);
            const int v = a.nodes[q];
            ldrow7(v, z);
            for (int f = a.fptr[q]; f < a.fptr[q + 1]; f++) {
                const int* F = a.fronts + 4 * (int64_t)f;
                double xr[7];
                ldrow7(F[0], xr);
                const double* Wr = a.W + (int64_t)F[3] * 49;
#pragma unroll
                for (int m = 0; m < 7; m++)
#pragma unroll
                    for (int i = 0; i < 7; i++) z[m] = fma(-Wr[i * 7 + m], xr[i], z[m]);
            }
            b7::bwd7(L, inv, z);
            strow7(v, z);
        }
        stores_done();
        __syncthreads();
    }
}

}  // namespace

hipError_t launch_sp_inverse(hipStream_t st, const InvArgs& a) {
    const int grid = (a.n + T - 1) / T;
    hipLaunchKernelGGL(sp_inverse_kernel, dim3(grid), dim3(NTH), 0, st, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// PCG
// ---------------------------------------------------------------------------------------------
namespace {

constexpr int kNE = kPcgMaxN / NTH;  // vector entries per thread (entry e in thread e % 256)

// the workgroup's sum of one value per thread, in a fixed order (every workgroup the same):
// a DPP / permute tree inside each wave, then the 4 wave sums in wave order
__device__ __forceinline__ double wg_sum(double v, double* red) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    const int w = threadIdx.x >> 6;
    __syncthreads();  // (red is reused by the previous sum's readers)
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    return ((red[0] + red[1]) + red[2]) + red[3];
}

struct Gran {
    unsigned long long lo, hi;
};
__device__ __forceinline__ void publish(Gran* g, unsigned tag, double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned long long t = (unsigned long long)tag << 32;
    __hip_atomic_store(&g->lo, t | (b & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&g->hi, t | (b >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(NTH) void pcg_kernel(PcgArgs a) {
    if (a.flags[kFlagDone]) return;  // converged call: every later launch returns
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double* sv = reinterpret_cast<double*>(smem);                // [nv]: the vector the products read
    double* red = sv + a.nv;                                     // [4]
    int2* sadj = reinterpret_cast<int2*>(red + 4);               // [nadj]: the product's (block, pose) lists
    int* sapt = reinterpret_cast<int*>(sadj + a.nadj);           // [npose + 1] (+ pad to 4)
    int* sabort = sapt + a.napt4;                                // this workgroup saw a gather give up
    float* Xs = reinterpret_cast<float*>(sabort + 4);            // [R][n]: this workgroup's rows of M
    const int tid = threadIdx.x;
    const int n = a.n, R = a.R;
    const int row0 = blockIdx.x * R;
    if (tid == 0) *sabort = 0;
    for (int id = tid; id < a.nadj; id += NTH) sadj[id] = a.adj[id];
    for (int id = tid; id <= a.npose; id += NTH) sapt[id] = a.adj_ptr[id];
    for (int id = tid; id < R * n; id += NTH) {
        const int i = id / n, j = id - i * n;
        Xs[id] = row0 + i < n ? (float)a.X[(int64_t)(row0 + i) * a.ldx + j] : 0.0f;
    }
    double x[kNE], r[kNE], p[kNE], z[kNE];
#pragma unroll
    for (int k = 0; k < kNE; k++) {
        const int e = tid + NTH * k;
        x[k] = 0.0;
        r[k] = e < n ? a.b[e] : 0.0;
        p[k] = z[k] = 0.0;
    }
    // z = M r: this workgroup's rows from LDS, published, then every row gathered (exchange s)
    const int tpr = NTH / R;  // threads per row (a power of two <= 32: one wave)
    const int ri = tid / tpr, rs = tid - ri * tpr;
    auto precond = [&](unsigned s) {
#pragma unroll
        for (int k = 0; k < kNE; k++) {
            const int e = tid + NTH * k;
            if (e < n) sv[e] = r[k];
        }
        __syncthreads();
        double acc = 0.0;
        const float* xr = Xs + ri * n;
        for (int j = rs; j < n; j += tpr) acc = fma((double)xr[j], sv[j], acc);
        for (int o = tpr >> 1; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
        Gran* buf = reinterpret_cast<Gran*>(a.gran) + (int64_t)(s & 1) * a.nv;
        const unsigned tag = a.tag0 + s;
        if (rs == 0 && row0 + ri < n) publish(buf + row0 + ri, tag, acc);
        // gather: every entry this thread holds, polled until both granules carry the tag -- all of
        // the thread's granule loads in flight together, re-polling only what has not arrived
        bool ok = true;
        unsigned need = 0;
#pragma unroll
        for (int k = 0; k < kNE; k++)
            if (tid + NTH * k < n) need |= 1u << k;
        for (int spins = 0; need;) {
            unsigned long long lo[kNE], hi[kNE];
#pragma unroll
            for (int k = 0; k < kNE; k++)
                if (need >> k & 1) {
                    lo[k] = __hip_atomic_load(&buf[tid + NTH * k].lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    hi[k] = __hip_atomic_load(&buf[tid + NTH * k].hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
#pragma unroll
            for (int k = 0; k < kNE; k++)
                if ((need >> k & 1) && (unsigned)(lo[k] >> 32) == tag && (unsigned)(hi[k] >> 32) == tag) {
                    z[k] = __hiloint2double((int)(unsigned)hi[k], (int)(unsigned)lo[k]);
                    need &= ~(1u << k);
                }
            if (!need) break;
            if (++spins > a.spin_limit ||
                ((spins & 255) == 0 && __hip_atomic_load(a.flags + kFlagPcgAbort, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT) == (int)a.tag0)) {
                ok = false;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (!ok) {  // a workgroup never published: abandon this PCG, the direct solve runs instead
            *sabort = 1;
            __hip_atomic_store(a.flags + kFlagPcgAbort, (int)a.tag0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        return *sabort == 0;
    };
    auto dot = [&](const double (&u)[kNE], const double (&v)[kNE]) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < kNE; k++) s = fma(u[k], v[k], s);
        return wg_sum(s, red);
    };
    __syncthreads();  // Xs complete
    bool good = precond(0);
    double rho = dot(r, z);
    const double rho0 = rho;
    good = good && rho > 0.0 && isfinite(rho);
    int steps = 0;
    bool conv = false;
#pragma unroll
    for (int k = 0; k < kNE; k++) p[k] = z[k];
    for (int s = 1; good && s <= a.kmax; s++) {
        // q = A p, the whole vector in every workgroup (blocks are symmetric: A_rs = A_sr)
#pragma unroll
        for (int k = 0; k < kNE; k++) {
            const int e = tid + NTH * k;
            if (e < n) sv[e] = p[k];
        }
        __syncthreads();
        double q[kNE];
#pragma unroll
        for (int k = 0; k < kNE; k++) {
            const int e = tid + NTH * k;
            q[k] = 0.0;
            if (e >= n) continue;
            const int pr = e / 7, d = e - 7 * pr;
            const int t0 = sapt[pr], t1 = sapt[pr + 1];
            double acc = 0.0;
            // 4 blocks' rows in flight per batch (the lists come from LDS), summed in list order
            for (int t = t0; t < t1; t += 4) {
                double av[4][7];
                int ps[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int2 bs = sadj[t + u < t1 ? t + u : t0];
                    ps[u] = 7 * bs.y;
                    const double* Ab = a.A + (int64_t)bs.x * 49 + d * 7;
#pragma unroll
                    for (int jj = 0; jj < 7; jj++) av[u][jj] = Ab[jj];
                }
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    if (t + u >= t1) break;
#pragma unroll
                    for (int jj = 0; jj < 7; jj++) acc = fma(av[u][jj], sv[ps[u] + jj], acc);
                }
            }
            q[k] = acc;
        }
        const double pq = dot(p, q);
        if (!(pq > 0.0 && isfinite(pq))) {  // breakdown (not positive definite / not finite)
            good = false;
            break;
        }
        const double alpha = rho / pq;
#pragma unroll
        for (int k = 0; k < kNE; k++) {
            x[k] = fma(alpha, p[k], x[k]);
            r[k] = fma(-alpha, q[k], r[k]);
        }
        __syncthreads();  // (sv is rewritten by precond)
        if (!precond((unsigned)s)) {
            good = false;
            break;
        }
        const double rho1 = dot(r, z);
        steps = s;
        if (!(rho1 >= 0.0 && isfinite(rho1))) {
            good = false;
            break;
        }
        if (rho1 <= a.tol2 * rho0) {
            conv = true;
            break;
        }
        // behind the geometric schedule that reaches tol2 at kmax (from step 4 on): M no longer
        // fits the system (the iterate moved far since M's factorisation); give up early -- the
        // direct solve runs, and its factor refreshes M (sp_inverse_kernel after a fallback)
        if (s >= 4 && rho1 > rho0 * exp(log(a.tol2) * (double)s / (double)a.kmax)) break;
        const double beta = rho1 / rho;
#pragma unroll
        for (int k = 0; k < kNE; k++) p[k] = fma(beta, p[k], z[k]);
        rho = rho1;
    }
    if (blockIdx.x != 0) return;
    // workgroup 0 decides for the iteration (it holds the same vectors as every other one)
    const bool use = good && conv;
    if (use) {
        // the retraction of gn_retract_kernel (same arithmetic, so the same poses as the direct
        // path's retraction of the same x): dx = -x, left retraction, ||dx|| < delta_thresh
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kNE; k++) {
            const int e = tid + NTH * k;
            if (e < n) sv[e] = x[k];
        }
        __syncthreads();
        double nrm = 0.0;
        for (int pp = 1 + tid; pp < a.N; pp += NTH) {
            float xi[7];
#pragma unroll
            for (int qd = 0; qd < 7; qd++) {
                const float v = -(float)sv[(pp - 1) * 7 + qd];
                xi[qd] = v;
                a.dx[(int64_t)(pp - 1) * 7 + qd] = v;
                nrm += (double)v * (double)v;
            }
            retr_sim3_cm(a.contract, xi, a.Twc + (int64_t)pp * 8);
        }
        double* tree = sv;  // (x is no longer needed)
        __syncthreads();
        tree[tid] = nrm;
        __syncthreads();
        for (int s = 128; s >= 1; s >>= 1) {
            if (tid < s) tree[tid] += tree[tid + s];
            __syncthreads();
        }
        if (tid == 0) {
            a.flags[kFlagFail] = 0;
            if ((float)sqrt(tree[0]) < a.delta_thresh) a.flags[kFlagDone] = 1;
        }
    }
    if (tid == 0) {
        a.flags[kFlagSkipSolve] = use ? 1 : 0;
        a.flags[kFlagPcgRuns] += 1;
        a.flags[kFlagPcgSteps] += steps;
        if (!use) a.flags[kFlagPcgFall] += 1;
    }
}

}  // namespace

int pcg_nv(int n) { return n < NTH ? NTH : (n + 3) / 4 * 4; }  // (>= 256: the norm tree of the retraction)
int pcg_napt4(int npose) { return (npose + 1 + 3) / 4 * 4; }
size_t pcg_lds_bytes(int n, int R, int nadj) {
    const int npose = n / 7;
    return sizeof(double) * (size_t)(pcg_nv(n) + 4) + 8 * (size_t)nadj + 4 * (size_t)pcg_napt4(npose) + 16 +
           sizeof(float) * (size_t)R * n;
}

hipError_t launch_pcg(hipStream_t st, const PcgArgs& a) {
    const size_t lds = pcg_lds_bytes(a.n, a.R, a.nadj);
    static bool attr = false;  // (one function, one attribute: the maximum the kernel may ask for)
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)pcg_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           kPcgMaxLds);
        if (e != hipSuccess) return e;
        attr = true;
    }
    if (lds > (size_t)kPcgMaxLds) return hipErrorInvalidValue;
    hipLaunchKernelGGL(pcg_kernel, dim3(a.nwg), dim3(NTH), lds, st, a);
    return hipGetLastError();
}

}  // namespace m3s
