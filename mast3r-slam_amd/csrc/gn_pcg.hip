// gn_pcg.hip -- the GN step off the factorisation's critical path (round 6).
//
// The reference factors every iteration's normal equations on the host (SimplicialLLT,
// gn_kernels.cu:132-153, called per iteration at :1199-1209).  Here iterations 0 and 1 keep the
// direct block-sparse factorisation (gn_sparse.hip rounds + chol_df.hip core); from iteration 2
// on the step is solved by conjugate gradients preconditioned with the inverse of iteration 1's
// system, M = A_1^-1, applied as a dense matrix-vector product:
//   * sp_inverse_kernel: X = A_1^-1 column block by column block through iteration 1's factor
//     (the elimination rounds' L_v / W_rv and the core's L tiles and tile inverses), 16
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
constexpr int NTH = 256;

// X's columns are written and read by the waves of ONE workgroup (one CU, one L1): plain loads
// after a store drain + barrier see them (workgroup scope needs no cache bypass) -- agent-scope
// loads went to the coherence point every time (~1-2 us a round trip): the rounds took 140 us
// each way on cfg4, most of it those round trips
__device__ __forceinline__ void stores_done() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ d4 mfma(double a, double b, d4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// X = A^-1 through the factor of the last direct solve
// ---------------------------------------------------------------------------------------------
namespace {

// the core's dense index gi (< 7 ntail) -> its row of the system (pose-major, 7 per pose)
__device__ __forceinline__ int core_row(const int* tail, int gi) { return 7 * tail[gi / 7] + gi % 7; }

constexpr int ICB = 16;  // right-hand sides (columns of X) per workgroup: thread t = column t % 16, slot t / 16

// One workgroup per 16 columns of X = A^-1 (lane = column, 16 slots): B = I, then
//   forward rounds: Y_v = L_v^-1 B_v for the round's nodes (16 in parallel), then per RHS target
//     B_r -= sum_v W_rv Y_v (targets in parallel, contributions in the plan's order);
//   the core: its rows of B staged in LDS once ([column][row]), forward and back substitution by
//     64 x 64 f64-MFMA tile products -- only the L tiles stream from L2 / HBM, each wave's 16 rows
//     of the next tile loaded straight into registers while the current product runs (no LDS
//     staging, no barrier between two products);
//     the back pass walks k downwards (every product's operand is already final);
//   back rounds: X_v = L_v^-T (Y_v - sum_r W_rv^T X_r) for the round's nodes, last round first;
//   then the 16 columns as an f32 row-major copy Xt[column][row] (M is symmetric: a PCG
//   workgroup's rows of M are these rows), through LDS so the writes are whole rows.
__global__ __launch_bounds__(NTH) void sp_inverse_kernel(InvArgs a) {
    // the call has converged (no PCG iteration follows), or this iteration's PCG converged (no
    // new factor: M stays)
    if (a.flags[kFlagDone] || a.flags[kFlagSkipSolve]) return;
    extern __shared__ __attribute__((aligned(16))) unsigned char ismem[];
    float* St = reinterpret_cast<float*>(ismem);            // [16][65]: the f32 copy's staging
    double* SB = reinterpret_cast<double*>(ismem) + 8 * (T + 1);  // [16][ldb]: the core rows of B / Y / X
    const int ldb = a.npad + 1;
    const int tid = threadIdx.x, c = tid & (ICB - 1), g = tid >> 4;
    const int n = a.n;
    const int64_t ldx = a.ldx;
    double* Xc = a.X + (int64_t)blockIdx.x * ICB;  // this workgroup's columns
    const int col = blockIdx.x * ICB + c;
    // M3S_PCG_DEBUG: workgroup 0's clock at the phase ends (entry, B = I, forward rounds, core, back
    // rounds, f32 copy)
    auto stamp = [&](int slot) {
        if (a.dbg && blockIdx.x == 0 && tid == 0) a.dbg[slot] = (long long)__builtin_amdgcn_s_memrealtime();
    };
    stamp(0);
    for (int row = g; row < n; row += NTH / ICB) Xc[row * ldx + c] = row == col ? 1.0 : 0.0;
    stores_done();
    __syncthreads();
    stamp(1);
    auto ldrow7 = [&](int pose, double (&v)[7]) {
#pragma unroll
        for (int d = 0; d < 7; d++) v[d] = Xc[(int64_t)(7 * pose + d) * ldx + c];
    };
    auto strow7 = [&](int pose, const double (&v)[7]) {
#pragma unroll
        for (int d = 0; d < 7; d++) Xc[(int64_t)(7 * pose + d) * ldx + c] = v[d];
    };
    auto ldL = [&](int q, double (&L)[28], double (&inv)[7]) {
        const double* Ls = a.Lstore + (int64_t)q * kLStoreRec;
#pragma unroll
        for (int k = 0; k < 28; k++) L[k] = Ls[k];
#pragma unroll
        for (int k = 0; k < 7; k++) inv[k] = Ls[28 + k];
    };
    constexpr int NS = NTH / ICB;  // slots
    // ---- forward through the elimination rounds
    for (int rd = 0; rd < a.nrounds; rd++) {
        const int* R = a.rounds + 8 * rd;  // node_begin, nnodes, tbeg, nbt, rbeg, nrt, wbeg, wcount
        const int nb = R[0], nn = R[1];
        for (int q = nb + g; q < nb + nn; q += NS) {
            double L[28], inv[7], bv[7], yv[7];
            ldL(q, L, inv);
            ldrow7(a.nodes[q], bv);
            b7::fwd7(L, inv, bv, yv);
            strow7(a.nodes[q], yv);
        }
        stores_done();
        __syncthreads();
        const int* recs = a.inl + (int64_t)(R[2] + R[4] + R[3]) * kSpRec;  // this round's RHS targets
        for (int t = g; t < R[5]; t += NS) {
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
    stamp(2);
    // ---- the core in LDS: SB[c][gi] = B[core row gi][c] (0 past the core)
    const int nt = a.npad / T, ncore = 7 * a.ntail;
    for (int gi = g; gi < a.npad; gi += NS) SB[c * ldb + gi] = gi < ncore ? Xc[(int64_t)core_row(a.tail, gi) * ldx + c] : 0.0;
    __syncthreads();
    // the product sequence: forward (j up, k = 0 .. j-1, then Linv_j), back (j down, k = nt-1 .. j+1,
    // then Linv_j^T); op = (kind, j, k): kind 0 L_jk, 1 Linv_j, 2 L_kj^T, 3 Linv_j^T
    const int lane = tid & 63, w = tid >> 6;
    const int r16 = lane & 15, kq = lane >> 4;
    auto next = [&](int& kind, int& j, int& k) {  // -> false past the end
        if (kind == 0) {
            if (++k >= j) kind = 1;
        } else if (kind == 1) {
            if (++j >= nt) {
                kind = 2;
                j = nt - 1;
                k = nt - 1;
                if (k <= j) kind = 3;
            } else {
                kind = j > 0 ? 0 : 1;
                k = 0;
            }
        } else if (kind == 2) {
            if (--k <= j) kind = 3;
        } else {
            if (--j < 0) return false;
            k = nt - 1;
            kind = k > j ? 2 : 3;
        }
        return true;
    };
    // the op's 64 x 64 source tile, as the MFMA's row operand [i][kk]
    auto src = [&](int kind, int j, int k, int i, int kk) -> double {
        switch (kind) {
            case 0: return a.Hd[((int64_t)j * T + i) * a.npad + (int64_t)k * T + kk];    // L_jk
            case 1: return a.Linv[(int64_t)j * T * T + i * T + kk];                       // Linv_j
            case 2: return a.Hd[((int64_t)k * T + kk) * a.npad + (int64_t)j * T + i];    // L_kj^T
            default: return a.Linv[(int64_t)j * T * T + kk * T + i];                      // Linv_j^T
        }
    };
    // wave w's row operand of an op, straight from L2 / HBM into registers (no LDS staging, no
    // barrier): a16[s] = X[16w + r16][kq + 4s], X the op's tile as [i][kk]
    auto fetch = [&](int kind, int j, int k, double (&a16)[16]) {
#pragma unroll
        for (int s4 = 0; s4 < 16; s4++) a16[s4] = src(kind, j, k, 16 * w + r16, kq + 4 * s4);
    };
    // acc (wave w: tile rows 16w .. 16w+15, columns 0..15): element (16w + kq + 4e, r16)
    d4 acc = d4{0.0, 0.0, 0.0, 0.0};
    auto acc_load = [&](int j) {
#pragma unroll
        for (int e = 0; e < 4; e++) acc[e] = SB[r16 * ldb + j * T + 16 * w + kq + 4 * e];
    };
    // sgn * X Y^T for the wave's rows (Y: [16][ldb] from a tile's column offset), two independent
    // MFMA chains (even / odd k steps) summed at the end
    auto gemm = [&](const double (&a16)[16], const double* Y, double sgn) {
        const double* yr = Y + r16 * ldb + kq;
        d4 o0 = d4{0.0, 0.0, 0.0, 0.0}, o1 = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s4 = 0; s4 < 16; s4 += 2) {
            o0 = mfma(sgn * a16[s4], yr[4 * s4], o0);
            o1 = mfma(sgn * a16[s4 + 1], yr[4 * s4 + 4], o1);
        }
        return o0 + o1;
    };
    if (nt > 0) {
        int kind = 1, j = 0, k = 0;  // the first op: Linv_0 (row 0 has no products)
        double cur[16], nxt[16];
        fetch(kind, j, k, cur);
        acc_load(0);
        bool more = true;
        while (more) {
            const int ck = kind, cj = j, ckk = k;
            more = next(kind, j, k);
            if (more) fetch(kind, j, k, nxt);  // in flight during this op's products
            if (ck == 0 || ck == 2) {
                acc += gemm(cur, SB + ckk * T, -1.0);  // Y_k / X_k: SB columns of tile k
            } else {
                // apply Linv_j (or its transpose) to the finished row: acc through LDS as the
                // right operand, over tile j's columns of SB (Z_j -> Y_j / X_j in place)
#pragma unroll
                for (int e = 0; e < 4; e++) SB[r16 * ldb + cj * T + 16 * w + kq + 4 * e] = acc[e];
                __syncthreads();
                const d4 y = gemm(cur, SB + cj * T, 1.0);
                __syncthreads();  // (every wave read tile j's Z before any writes its Y)
#pragma unroll
                for (int e = 0; e < 4; e++) SB[r16 * ldb + cj * T + 16 * w + kq + 4 * e] = y[e];
                __syncthreads();
                if (more) acc_load(j);  // the next row starts from its B_j (forward) / Y_j (back)
            }
#pragma unroll
            for (int s4 = 0; s4 < 16; s4++) cur[s4] = nxt[s4];
        }
    }
    __syncthreads();
    for (int gi = g; gi < ncore; gi += NS) Xc[(int64_t)core_row(a.tail, gi) * ldx + c] = SB[c * ldb + gi];
    stores_done();
    __syncthreads();
    stamp(3);
    // ---- back through the rounds, last first
    for (int rd = a.nrounds - 1; rd >= 0; rd--) {
        const int* R = a.rounds + 8 * rd;
        const int nb = R[0], nn = R[1];
        for (int q = nb + g; q < nb + nn; q += NS) {
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
    stamp(4);
    // ---- the f32 copy Xt[column][row], 64 rows at a time through LDS (whole-row writes)
    for (int r0 = 0; r0 < n; r0 += T) {
        for (int id = tid; id < T * ICB; id += NTH) {
            const int rr = id / ICB, cc = id % ICB;
            St[cc * (T + 1) + rr] = r0 + rr < n ? (float)Xc[(int64_t)(r0 + rr) * ldx + cc] : 0.0f;
        }
        __syncthreads();
        for (int id = tid; id < T * ICB; id += NTH) {
            const int cc = id / T, rr = id % T;
            if (r0 + rr < n) a.Xt[(int64_t)(blockIdx.x * ICB + cc) * a.ldt + r0 + rr] = St[cc * (T + 1) + rr];
        }
        __syncthreads();
    }
    stamp(5);
}

}  // namespace

size_t inverse_lds_bytes(int npad) {
    return sizeof(double) * (8 * (size_t)(T + 1) + (size_t)ICB * (npad + 1));
}

hipError_t launch_sp_inverse(hipStream_t st, const InvArgs& a) {
    const int grid = (a.n + ICB - 1) / ICB;
    const size_t lds = inverse_lds_bytes(a.npad);
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)sp_inverse_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           kPcgMaxLds);
        if (e != hipSuccess) return e;
        attr = true;
    }
    if (lds > (size_t)kPcgMaxLds) return hipErrorInvalidValue;
    hipLaunchKernelGGL(sp_inverse_kernel, dim3(grid), dim3(NTH), lds, st, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// PCG
// ---------------------------------------------------------------------------------------------
namespace {

constexpr int PTH = kPcgThreads;          // PCG workgroup: 12 waves (3 per SIMD at <= 170 VGPRs)
constexpr int kNE = (kPcgMaxN + PTH - 1) / PTH;  // vector entries per thread (entry e in thread e % PTH)

// the workgroup's sum of one value per thread, in a fixed order (every workgroup the same):
// a permute tree inside each wave, then the 16 wave sums in wave order
__device__ __forceinline__ double wg_sum(double v, double* red) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    const int w = threadIdx.x >> 6;
    __syncthreads();  // (red is reused by the previous sum's readers)
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    double s = red[0];
#pragma unroll
    for (int k = 1; k < PTH / 64; k++) s += red[k];
    return s;
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

__global__ __launch_bounds__(PTH) void pcg_kernel(PcgArgs a) {
    if (a.flags[kFlagDone]) return;  // converged call: every later launch returns
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x;
    const int n = a.n, R = a.R, ni = a.nitem;
    const int row0 = blockIdx.x * R;
    double* sv = reinterpret_cast<double*>(smem);          // [nv]: the vector the products read
    double* red = sv + a.nv;                               // [16]
    double* sA = red + 16;                                 // [ni][7]: this workgroup's rows of A, block by block
    double* spart = sA + 7 * (size_t)ni;                   // [ni]: their products with p
    int* sps = reinterpret_cast<int*>(spart + ni);         // [ni]: 7 x the pose each block couples to
    int* sib = sps + ni;                                   // [R + 1]: the rows' first item
    int* sabort = sib + a.R4;                              // this workgroup saw a gather give up
    float* Xs = reinterpret_cast<float*>(sabort + 4);      // [R][n]: this workgroup's rows of M
    float* Bs = Xs + (size_t)R * n;                        // [R][n]: its rows of B = M A (onex)
    const bool onex = a.onex != 0;
    if (tid == 0) *sabort = 0;
    // M3S_PCG_DEBUG (diagnostics): workgroup 0's wall clock at the phase ends, one slot per
    // phase (slot 0: entry, 1: staged, 2: z0 gathered, then per step 3s: q gathered, 3s+1: p'q,
    // 3s+2: z gathered)
    auto stamp = [&](int slot) {
        if (a.dbg && blockIdx.x == 0 && tid == 0 && slot < kPcgDbgSlots)
            a.dbg[slot] = (long long)__builtin_amdgcn_s_memrealtime();
    };
    stamp(0);
    // ---- staging: this workgroup's rows of A (items: row e, block t of its pose, in list
    // order) and of M (f32), 16 loads in flight per thread
    // (the rows' item counts loaded in parallel -- one thread walking them was a chain of
    // dependent loads, ~17 us -- then a prefix sum by thread 0 over LDS)
    if (tid < R) {
        const int e = row0 + tid;
        sib[tid + 1] = e < n ? a.adj_ptr[e / 7 + 1] - a.adj_ptr[e / 7] : 0;
    }
    __syncthreads();
    if (tid == 0) {
        sib[0] = 0;
        for (int i = 0; i < R; i++) sib[i + 1] += sib[i];
    }
    __syncthreads();
    for (int it = tid; it < sib[R]; it += PTH) {
        int i = 0;
        while (sib[i + 1] <= it) i++;
        const int e = row0 + i, pr = e / 7, d = e - 7 * pr;
        const int2 bs = a.adj[a.adj_ptr[pr] + (it - sib[i])];
        sps[it] = 7 * bs.y;
        const double* Ab = a.A + (int64_t)bs.x * 49 + d * 7;
#pragma unroll
        for (int jj = 0; jj < 7; jj++) sA[7 * it + jj] = Ab[jj];
    }
    // (this workgroup's rows of M = its columns: sp_inverse_kernel's f32 copy Xt, rows contiguous)
    for (int id0 = tid * 4; id0 < R * a.ldt; id0 += PTH * 4) {
        const int i = id0 / a.ldt, jj = id0 - i * a.ldt;  // (ldt is a multiple of 4)
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (row0 + i < n) v = *reinterpret_cast<const float4*>(a.Xt + (int64_t)(row0 + i) * a.ldt + jj);
        const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int u = 0; u < 4; u++)
            if (jj + u < n) Xs[i * n + jj + u] = vv[u];
    }
    if (onex) {
        // B = M A, this workgroup's rows: column c = 7 pj + d of B is sum over the blocks (pk, pj)
        // of M's columns 7 pk .. 7 pk + 6 times the block's column d (the blocks are symmetric:
        // Ji = -Jj makes every 7x7 block +-D with D symmetric, gn_refacc.hip header).  One thread
        // per column, the R rows in registers, f64 sums rounded once to f32.
        __syncthreads();  // (Xs staged)
        for (int col = tid; col < n; col += PTH) {
            const int pj = col / 7, d = col - 7 * pj;
            double acc[kPcgMaxR];
#pragma unroll
            for (int i = 0; i < kPcgMaxR; i++) acc[i] = 0.0;
            for (int it = a.adj_ptr[pj]; it < a.adj_ptr[pj + 1]; it++) {
                const int2 bs = a.adj[it];
                const double* Ab = a.A + (int64_t)bs.x * 49 + d;
                double ac[7];
#pragma unroll
                for (int c = 0; c < 7; c++) ac[c] = Ab[7 * c];
                const float* xk = Xs + 7 * bs.y;
#pragma unroll
                for (int i = 0; i < kPcgMaxR; i++)
                    if (i < R) {
#pragma unroll
                        for (int c = 0; c < 7; c++) acc[i] = fma((double)xk[i * n + c], ac[c], acc[i]);
                    }
            }
#pragma unroll
            for (int i = 0; i < kPcgMaxR; i++)
                if (i < R) Bs[i * n + col] = (float)acc[i];
        }
    }
    // full vectors in every workgroup (entry e in thread e % PTH); identical in all of them
    double x[kNE], r[kNE], p[kNE], z[kNE], q[kNE], w[kNE];
#pragma unroll
    for (int k = 0; k < kNE; k++) {
        const int e = tid + PTH * k;
        x[k] = 0.0;
        r[k] = e < n ? a.b[e] : 0.0;
        p[k] = z[k] = q[k] = w[k] = 0.0;
    }
    unsigned xchg = 0;  // exchanges so far (tag and buffer parity)
    // publish this workgroup's rows `val` (thread i < R holds row i), then gather every row into
    // out[] -- data-tagged granules, all of a thread's loads in flight together, double-buffered
    // by exchange parity (a workgroup reuses a buffer only after every other one published the
    // next exchange, i.e. finished reading this one)
    auto exchange2 = [&](int nval, double val0, double val1, double (&out0)[kNE], double (&out1)[kNE]) {
        Gran* buf = reinterpret_cast<Gran*>(a.gran) + (int64_t)(xchg & 1) * 2 * a.nv;
        const unsigned tag = a.tag0 + xchg;
        xchg++;
        if (tid < R && row0 + tid < n) {
            publish(buf + row0 + tid, tag, val0);
            if (nval > 1) publish(buf + a.nv + row0 + tid, tag, val1);
        }
        bool ok = true;
        unsigned need = 0;  // bit k: entry k of value 0; bit kNE + k: of value 1
#pragma unroll
        for (int k = 0; k < kNE; k++)
            if (tid + PTH * k < n) need |= (nval > 1 ? 1u | 1u << kNE : 1u) << k;
        for (int spins = 0; need;) {
            unsigned long long lo[2 * kNE], hi[2 * kNE];
#pragma unroll
            for (int k = 0; k < 2 * kNE; k++)
                if (need >> k & 1) {
                    const Gran* g = buf + (k >= kNE ? a.nv : 0) + tid + PTH * (k % kNE);
                    lo[k] = __hip_atomic_load(&g->lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    hi[k] = __hip_atomic_load(&g->hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
#pragma unroll
            for (int k = 0; k < 2 * kNE; k++)
                if ((need >> k & 1) && (unsigned)(lo[k] >> 32) == tag && (unsigned)(hi[k] >> 32) == tag) {
                    const double v = __hiloint2double((int)(unsigned)hi[k], (int)(unsigned)lo[k]);
                    if (k < kNE) out0[k] = v;
                    else out1[k - kNE] = v;
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
    auto exchange = [&](double val, double (&out)[kNE]) { return exchange2(1, val, 0.0, out, out); };
    auto to_sv = [&](const double (&u)[kNE]) {
#pragma unroll
        for (int k = 0; k < kNE; k++) {
            const int e = tid + PTH * k;
            if (e < n) sv[e] = u[k];
        }
        __syncthreads();
    };
    // z = M r: this workgroup's rows from LDS (a row's threads in one wave), then exchanged
    const int tpr = PTH / R;  // threads per row (a power of two <= 64: one wave; R = PTH / 64, PTH / 32)
    const int ri = tid / tpr, rs = tid - ri * tpr;
    auto apply_M = [&]() {  // -> z
        to_sv(r);
        double acc = 0.0;
        const float* xr = Xs + ri * n;
        for (int jj = rs; jj < n; jj += tpr) acc = fma((double)xr[jj], sv[jj], acc);
        for (int o = tpr >> 1; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
        __syncthreads();                // (sv's readers are done)
        if (rs == 0) sv[ri] = acc;      // row ri's sum, for thread ri to publish
        __syncthreads();
        const double mine = tid < R ? sv[tid] : 0.0;
        return exchange(mine, z);
    };
    auto apply_A = [&]() {  // -> q, and w = B p with onex (p in sv)
        to_sv(p);
        for (int it = tid; it < sib[R]; it += PTH) {
            const double* Ar = sA + 7 * it;
            const double* ps = sv + sps[it];
            double acc = 0.0;
#pragma unroll
            for (int jj = 0; jj < 7; jj++) acc = fma(Ar[jj], ps[jj], acc);
            spart[it] = acc;
        }
        double wrow = 0.0;
        if (onex) {  // (the row sums of B p as apply_M's of M r)
            const float* br = Bs + ri * n;
            for (int jj = rs; jj < n; jj += tpr) wrow = fma((double)br[jj], sv[jj], wrow);
            for (int o = tpr >> 1; o >= 1; o >>= 1) wrow += __shfl_xor(wrow, o);
        }
        __syncthreads();
        double mine = 0.0;
        if (tid < R)
            for (int it = sib[tid]; it < sib[tid + 1]; it++) mine += spart[it];
        if (!onex) return exchange(mine, q);
        if (rs == 0) sv[ri] = wrow;  // (p in sv was read before the barrier above)
        __syncthreads();
        const double wmine = tid < R ? sv[tid] : 0.0;
        return exchange2(2, mine, wmine, q, w);
    };
    auto dot = [&](const double (&u)[kNE], const double (&v)[kNE]) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < kNE; k++) s = fma(u[k], v[k], s);
        return wg_sum(s, red);
    };
    __syncthreads();  // staged
    stamp(1);
    bool good = apply_M();
    stamp(2);
    double rho = dot(r, z);
    const double rho0 = rho;
    good = good && rho > 0.0 && isfinite(rho);
    int steps = 0;
    bool conv = false;
#pragma unroll
    for (int k = 0; k < kNE; k++) p[k] = z[k];
    for (int s = 1; good && s <= a.kmax; s++) {
        if (!apply_A()) {
            good = false;
            break;
        }
        stamp(3 * s);
        const double pq = dot(p, q);
        stamp(3 * s + 1);
        if (!(pq > 0.0 && isfinite(pq))) {  // breakdown (not positive definite / not finite)
            good = false;
            break;
        }
        const double alpha = rho / pq;
#pragma unroll
        for (int k = 0; k < kNE; k++) {
            x[k] = fma(alpha, p[k], x[k]);
            r[k] = fma(-alpha, q[k], r[k]);
            if (onex) z[k] = fma(-alpha, w[k], z[k]);  // z = M r = z - alpha M A p
        }
        if (!onex && !apply_M()) {
            good = false;
            break;
        }
        stamp(3 * s + 2);
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
            const int e = tid + PTH * k;
            if (e < n) sv[e] = x[k];
        }
        __syncthreads();
        double nrm = 0.0;
        for (int pp = 1 + tid; tid < 256 && pp < a.N; pp += 256) {  // (gn_retract_kernel's 256 threads)
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
        if (tid < 256) tree[tid] = nrm;
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

int pcg_nv(int n) { return n < 256 ? 256 : (n + 3) / 4 * 4; }  // (>= 256: the norm tree of the retraction)
int pcg_r4(int R) { return (R + 1 + 3) / 4 * 4; }
size_t pcg_lds_bytes(int n, int R, int nitem, bool onex) {
    return sizeof(double) * ((size_t)pcg_nv(n) + 16 + 8 * (size_t)nitem) + sizeof(int) * (2 * (size_t)nitem + pcg_r4(R) + 4) +
           sizeof(float) * (size_t)R * n * (onex ? 2 : 1);
}

hipError_t launch_pcg(hipStream_t st, const PcgArgs& a) {
    const size_t lds = pcg_lds_bytes(a.n, a.R, a.nitem, a.onex != 0);
    if (a.onex && a.R > kPcgMaxR) return hipErrorInvalidValue;
    static bool attr = false;  // (one function, one attribute: the maximum the kernel may ask for)
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)pcg_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           kPcgMaxLds);
        if (e != hipSuccess) return e;
        attr = true;
    }
    if (lds > (size_t)kPcgMaxLds) return hipErrorInvalidValue;
    hipLaunchKernelGGL(pcg_kernel, dim3(a.nwg), dim3(PTH), lds, st, a);
    return hipGetLastError();
}

}  // namespace m3s
