// chol_df.hip -- the dense core's tiled LL^T as ONE dataflow launch (replaces the Eigen
// SimplicialLLT factorisation of gn_kernels.cu:132-153 for cores above the in-register size).
//
// The multi-launch tile Cholesky (gn_kernels.hip) costs three dependent launches per 64-column
// panel (potrf, trsm, update: 48 for cfg4's 141-pose core), ~5 us of dispatch each, and its
// potrf ran the rank-8 trailing updates and the inverse on VALU from LDS (~30 us per tile).
// Here every lower tile (i, j) of the (npad + 64) x npad bordered matrix (the border row tile
// nt carries the RHS, so the forward substitution rides along) is a task of a single launch
// (a plain launch, grid sized by the occupancy query; tasks claimed dynamically), processed left-looking:
//   acc = A_ij;  for k < j: wait L_ik, L_jk final -> acc -= L_ik L_jk^T  (f64 MFMA)
//   i == j: potrf of acc in LDS (8-column panels, per-lane 8x8 factor + row solve, MFMA rank-8
//           trailing updates) and L_jj^-1 by doubling (8x8 blocks from the panel step, MFMA for
//           the 16 and 32 stages) -> publish Linv_j
//   i >  j: wait Linv_j -> L_ij = acc Linv_j^T (MFMA) -> publish L_ij
// Readiness is a per-tile epoch word (ready[i * nt + j] == epoch: final in this launch).  The
// per-XCD L2s are not coherent, so tile data crosses workgroups with agent-scope relaxed
// atomics (sc1 loads, write-through stores), the flag with a release store after the data
// stores completed.  Tiles are numbered column-major and a workgroup walks its tiles in order,
// so every wait targets a tile earlier in some co-resident workgroup's list: no deadlock; the
// spin is bounded (a missing producer fails the solve instead of hanging the GPU).
// Numerics: the same LL^T in a different (left-looking) summation order; the solve is f64 and
// not a bit-exact path (parity through poses, tests/test_gpu_gn.py).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdlib>

#include "gn_kernels.h"

#ifndef M3S_DF_CC
#define M3S_DF_CC 1  // 1: the register tile factor (potrf_cc: batch- or column-cyclic, M3S_DF_BC); 0: the 8-column panel steps (potrf_inverse)
#endif
#ifndef M3S_DF_BC
#define M3S_DF_BC 1  // 1: batch-cyclic tile factor (potrf_bc_w); 0: 16-column blocks per wave (potrf_cc_w)
#endif
#ifndef M3S_DF_BC_SPEC
#define M3S_DF_BC_SPEC 1  // potrf_bc_w: poll the counter and read the batch in one LDS round trip
#endif
#ifndef M3S_DF_BC_RL
#define M3S_DF_BC_RL 1  // potrf_bc_w: the inverse's column-block products right-looking
#endif
#ifndef M3S_DF_BC_W
#define M3S_DF_BC_W 4  // columns per batch of potrf_bc_w (4; 8 measured slower)
#endif
#ifndef M3S_DF_STAMPS
#define M3S_DF_STAMPS 0  // diagnostics (tools/ubench_potrf64.hip): cycle stamps inside the potrf steps
#endif

namespace m3s {

namespace {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int T = kCholTile;  // 64
constexpr int NT = 256;       // 4 waves: wave w owns 16-row block row w of a tile
constexpr int LD = 73;        // LDS row stride (doubles) = 18 dwords mod 64 banks: conflict-free MFMA reads

struct DfArgs {
    double* Hd;
    double* Linv;
    int* ready;
    int* flags;
    int npad, nt, ntiles, epoch;  // ntiles = number of tasks (num_tasks)
    int spin_limit;  // bound of a ready wait (s_sleep(1) steps); < 0: every wait times out (test hook)
    long long* trace;  // diagnostics (tools/ubench_chol_df.hip): 4 timestamps per tile, else null
    double* x;         // != null: the back-substitution L^T x = y runs in this launch too (x: npad)
    DfScatter g;       // g.xpose != null: the back-substitution also writes x pose-indexed
    // the back-substitution's in-launch hand-off of x: per entry two 8-B granules {epoch, 32 bits of
    // the double} (lo, hi), stored and polled as 64-bit agent-scope atomics -- the data is the flag
    // (cdna_hip_programming.md Guideline 16, R2): no store drain, barrier and flag before the
    // consumer sees x, and no flag poll + second load after it
    unsigned long long* xg;
    int xgran;  // x hand-off by granules (M3S_DF_XGRAN, default 1) or by ready words (0)
    int* tick;  // [2]: the task ticket counter and the exit counter (zero between launches)
    int dyn;    // tasks claimed dynamically (M3S_DF_DYN, default 1) or dealt statically (0)
};

// workgroup barrier ordering LDS only (__syncthreads also waits for every outstanding global
// store to be acknowledged: ~1 us after write-through stores)
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ void stamp(const DfArgs& a, int t, int slot) {
    if (a.trace && threadIdx.x == 0) a.trace[4 * t + slot] = (long long)__builtin_amdgcn_s_memrealtime();
}

__device__ __forceinline__ double ld_coh(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_coh(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ d4 mfma(double a, double b, d4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// thread 0 waits until *f reaches the epoch (bounded; on timeout the solve is failed AND the
// sticky timeout flag is raised, which the driver reports as M3S_ERR_TIMEOUT -- a lost publish
// or a starved producer must not pass for a singular system.  Once the solve has failed -- a
// timeout or a pivot <= 0 -- later waits give up early, so a failed factorisation drains
// quickly; its result is discarded: dx = 0)
__device__ __forceinline__ void wait_ready(const int* f, int epoch, int* flags, int spin_limit) {
    int spins = 0;
    while (spin_limit < 0 || __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < epoch) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > spin_limit) {
            __hip_atomic_store(flags + kFlagTimeout, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(flags + kFlagFail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        if ((spins & 1023) == 0 && __hip_atomic_load(flags + kFlagFail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            return;
    }
}

// 64x64 tile (row stride ld) -> LDS [64][LD], agent-coherent loads (one 512-B row per wave step)
__device__ __forceinline__ void load_tile_coh(double* S, const double* src, int64_t ld) {
    const int tid = threadIdx.x;
    double v[16];
#pragma unroll
    for (int q = 0; q < 16; q++) {
        const int id = tid + NT * q;
        v[q] = ld_coh(src + (int64_t)(id >> 6) * ld + (id & 63));
    }
#pragma unroll
    for (int q = 0; q < 16; q++) {
        const int id = tid + NT * q;
        S[(id >> 6) * LD + (id & 63)] = v[q];
    }
}

// acc[J] (16x16 block (w, J) of the tile) += sgn * X Y^T, X / Y: [64][LD] in LDS, K = 64.
// Operand layout of v_mfma_f64_16x16x4f64: lane -> (row | col) = lane & 15, k = lane >> 4;
// result acc[J][e] at row 16 w + (lane >> 4) + 4 e, column 16 J + (lane & 15).
// TRI: Y is lower triangular (a tile inverse), so block column J needs k < 16 J + 16 only:
// 40 instead of 64 MFMAs per wave on the trsm's chain.
template <bool TRI = false>
__device__ __forceinline__ void gemm_nt(const double* X, const double* Y, d4 acc[4], double sgn) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = lane & 15, kq = lane >> 4;
    const double* xr = X + (16 * w + r) * LD + kq;
    const double* yr = Y + r * LD + kq;
#pragma unroll
    for (int s = 0; s < 16; s++) {
        const double a = sgn * xr[4 * s];
        double b[4];
#pragma unroll
        for (int J = 0; J < 4; J++)
            if (!TRI || s <= 4 * J + 3) b[J] = yr[16 * J * LD + 4 * s];
#pragma unroll
        for (int J = 0; J < 4; J++)
            if (!TRI || s <= 4 * J + 3) acc[J] = mfma(a, b[J], acc[J]);
    }
}

// one lane's double, broadcast to the wave (two v_readlane_b32: SGPRs)
__device__ __forceinline__ double rdlane(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __hiloint2double(hi, lo);
}

// Panel step of the tile LL^T, run by wave 0: columns c0 .. c0+7 of every row, lane = row, in
// registers, right-looking over the 8 columns.  A pivot and the panel's diagonal-block entries
// reach the other lanes by v_readlane (no LDS round trip, no barrier on the pivot chain), and
// the rows below the diagonal block get their L entries in the same sweep (the panel's trsm).
// The critical chain per column is readlane -> rsq + Newton -> scale -> the next column's
// update in the next pivot's lane -> readlane.  Dinv[p] = 1 / l_pp (the pivot's rsqrt) for the
// 8x8 inverse block (diag_inv8, off the chain).
__device__ __forceinline__ void panel_factor(double* A, double* Dinv, int c0, int* flags) {
    const int lane = threadIdx.x & 63;
    double a[8], y[8];
#pragma unroll
    for (int p = 0; p < 8; p++) a[p] = A[lane * LD + c0 + p];
    bool bad = false;
    // lanes above a column's pivot hold upper-triangle garbage in it: never broadcast (only the
    // lanes below a pivot are) and never stored, so no masking on the chain
#pragma unroll
    for (int p = 0; p < 8; p++) {
        const double d = rdlane(a[p], c0 + p);
        bad |= d <= 0.0;  // SimplicialLLT: fails iff a pivot <= 0 (NaN passes)
        double r = __builtin_amdgcn_rsq(d);
        r = r * fma(-0.5 * d * r, r, 1.5);
        y[p] = r;
        a[p] *= r;
#pragma unroll
        for (int q = p + 1; q < 8; q++) a[q] = fma(-a[p], rdlane(a[p], c0 + q), a[q]);
    }
    if (lane == 0) {
        if (bad) flags[kFlagFail] = 1;
#pragma unroll
        for (int p = 0; p < 8; p++) Dinv[c0 + p] = y[p];
    }
    // every lane stores its panel row: the rows above the pivots write garbage into the tile's
    // upper triangle, which is never read
#pragma unroll
    for (int p = 0; p < 8; p++) A[lane * LD + c0 + p] = a[p];
}

// the panel's 8x8 inverse block L_pp^-1 -> Li (lanes 0..7 of the calling wave: lane i solves
// L_pp x = e_i, i.e. column i of the inverse), from L_pp in A and 1/l_pp in Dinv
__device__ __forceinline__ void diag_inv8(const double* A, double* Li, const double* Dinv, int c0) {
    const int i = threadIdx.x & 63;
    if (i >= 8) return;
    double L[8][8], inv[8], x[8];
#pragma unroll
    for (int m = 0; m < 8; m++) {
        inv[m] = Dinv[c0 + m];
#pragma unroll
        for (int k = 0; k < m; k++) L[m][k] = A[(c0 + m) * LD + c0 + k];
    }
#pragma unroll
    for (int m = 0; m < 8; m++) {
        double s = m == i ? 1.0 : 0.0;
#pragma unroll
        for (int k = 0; k < m; k++) s = fma(-L[m][k], x[k], s);
        x[m] = m >= i ? s * inv[m] : 0.0;
    }
#pragma unroll
    for (int m = 0; m < 8; m++) Li[(c0 + m) * LD + c0 + i] = x[m];
}

// Block row s (rows 8s .. 8s+7) of Li = L^-1, by one wave, for the column blocks k < s with
// k = part (mod nparts):  X_ss = L_ss^-1 (diag_inv8; every wave that calls this writes the same
// bytes) and X_sk = -X_ss sum_{m=k}^{s-1} L_sm X_mk, lane = (row r, column c) of the 8x8 block.
// Needs the panels <= s factored and X's block rows < s complete: in the potrf step loop block
// row s is built by waves 1-3 during step s, off the pivot chain, so only block row 7 is left
// after the last panel (it replaces the 8 -> 16 -> 32 doubling stages, ~27 % of potrf + inverse).
// scr: 64 doubles of LDS for this wave (the T block between its two products).
__device__ __forceinline__ void inv_row(const double* A, double* Li, const double* Dinv, int s, int part,
                                        int nparts, double* scr) {
    const int lane = threadIdx.x & 63;
    const int r = lane >> 3, c = lane & 7;
    const int c0 = 8 * s;
    diag_inv8(A, Li, Dinv, c0);
    if (s == 0) return;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    double xs[8];  // row r of X_ss
#pragma unroll
    for (int m = 0; m < 8; m++) xs[m] = Li[(c0 + r) * LD + c0 + m];
    for (int k = part; k < s; k += nparts) {
        double t = 0.0;
        for (int m = k; m < s; m++) {
#pragma unroll
            for (int q = 0; q < 8; q++) t = fma(A[(c0 + r) * LD + 8 * m + q], Li[(8 * m + q) * LD + 8 * k + c], t);
        }
        scr[lane] = t;  // T[r][c]
        double x = 0.0;
#pragma unroll
        for (int m = 0; m < 8; m++) x = fma(xs[m], scr[8 * m + c], x);
        Li[(c0 + r) * LD + 8 * k + c] = -x;
    }
}

// A[I-block rows][J-block cols] -= P_I P_J^T with the panel at columns c0 .. c0+7, for the
// trailing columns (>= c0 + 8).  Block columns that still hold the panel itself (its 8 columns
// are the block's first half) get a zero B operand there, so those outputs equal their input and
// every block is stored whole: no per-element masked stores (a diagonal block's upper triangle
// takes garbage, which is never read).
// NB trailing blocks (I[k], J[k]) at once, the blocks with on[k] updated: the two K = 4 MFMAs
// of a block go to separate accumulators and every block's MFMAs are issued before any result
// is read, so a step costs one MFMA latency, not one per block and pass.
template <int NB>
__device__ __forceinline__ void trail_blocks(double* A, int c0, const int (&I)[NB], const int (&J)[NB],
                                             const bool (&on)[NB]) {
    const int lane = threadIdx.x & 63;
    const int r16 = lane & 15, kq = lane >> 4;
    const int lo = c0 + 8;
    d4 c[NB], d[NB];
    double a0[NB], a1[NB], b0[NB], b1[NB];
#pragma unroll
    for (int k = 0; k < NB; k++) {
        if (!on[k]) continue;
#pragma unroll
        for (int e = 0; e < 4; e++) c[k][e] = A[(16 * I[k] + kq + 4 * e) * LD + 16 * J[k] + r16];
        a0[k] = -A[(16 * I[k] + r16) * LD + c0 + kq];
        a1[k] = -A[(16 * I[k] + r16) * LD + c0 + 4 + kq];
        const bool trailing = 16 * J[k] + r16 >= lo;
        b0[k] = trailing ? A[(16 * J[k] + r16) * LD + c0 + kq] : 0.0;
        b1[k] = trailing ? A[(16 * J[k] + r16) * LD + c0 + 4 + kq] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < NB; k++)
        if (on[k]) c[k] = mfma(a0[k], b0[k], c[k]);
#pragma unroll
    for (int k = 0; k < NB; k++)
        if (on[k]) d[k] = mfma(a1[k], b1[k], d4{0.0, 0.0, 0.0, 0.0});
#pragma unroll
    for (int k = 0; k < NB; k++) {
        if (!on[k]) continue;
#pragma unroll
        for (int e = 0; e < 4; e++) A[(16 * I[k] + kq + 4 * e) * LD + 16 * J[k] + r16] = c[k][e] + d[k][e];
    }
}

// LL^T of the lower triangle of A (LDS) in place and Li = L^-1 (Li zeroed by the caller).
// Look-ahead: in step s wave 0 applies panel s to the block column holding panel s+1 and
// factors panel s+1 right away, while waves 1-3 apply panel s to the block columns right of it
// and build block row s of the inverse (inv_row); one barrier per step, and the step loop is
// unrolled, so every step issues only the MFMAs of its live blocks.
// early: a ready word published once every wave's earlier stores landed (after the first panel
// step, when they long have), so the caller's stores need no waiting on its critical path
[[maybe_unused]] __device__ void potrf_inverse(double* A, double* Li, double* Tm, double* Dinv, int* flags, long long* pt,
                              int* early, int epoch) {
    const int tid = threadIdx.x, w = tid >> 6;
    auto pstamp = [&](int slot) {
        if (pt && tid == 0) pt[slot] = (long long)__builtin_amdgcn_s_memrealtime();
    };
    pstamp(0);
    if (w == 0) panel_factor(A, Dinv, 0, flags);
    if (early) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (early && tid == 0) __hip_atomic_store(early, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    pstamp(1);
#pragma unroll
    for (int s = 0; s + 1 < T / 8; s++) {
        const int c0 = 8 * s;
        const int J1 = (c0 + 8) >> 4;  // block column holding panel s+1
        if (w == 0) {
            const int I[4] = {0, 1, 2, 3}, J[4] = {J1, J1, J1, J1};
            const bool on[4] = {0 >= J1, 1 >= J1, 2 >= J1, 3 >= J1};
            trail_blocks<4>(A, c0, I, J, on);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // own LDS writes before the reads
#if M3S_DF_STAMPS
            if (pt && tid == 0) pt[20 + 4 * s] = (long long)__builtin_amdgcn_s_memtime();
#endif
            panel_factor(A, Dinv, c0 + 8, flags);
#if M3S_DF_STAMPS
            if (pt && tid == 0) pt[21 + 4 * s] = (long long)__builtin_amdgcn_s_memtime();
#endif
        } else {
            const int I[3] = {w, w, w};
            const int J[3] = {min(J1 + 1, 3), min(J1 + 2, 3), min(J1 + 3, 3)};
            const bool on[3] = {J1 + 1 <= w, J1 + 2 <= w, J1 + 3 <= w};
            if (on[0]) trail_blocks<3>(A, c0, I, J, on);
            inv_row(A, Li, Dinv, s, w - 1, 3, Tm + 64 * w);
#if M3S_DF_STAMPS
            if (pt && tid == 192) pt[22 + 4 * s] = (long long)__builtin_amdgcn_s_memtime();
#endif
        }
        __syncthreads();
#if M3S_DF_STAMPS
        if (pt && tid == 0) pt[23 + 4 * s] = (long long)__builtin_amdgcn_s_memtime();
#endif
        pstamp(2 + s);
    }
    inv_row(A, Li, Dinv, T / 8 - 1, w, 4, Tm + 64 * w);  // the last block row of the inverse
    __syncthreads();
    pstamp(17);
}

// ---------------------------------------------------------------------------------------------
// Column-cyclic LL^T + inverse of the 64x64 tile (M3S_DF_CC=1, default).  Wave w owns columns
// 16w .. 16w+15, lane = row, in registers.  Column c is factored by its owner (pivot by
// v_readlane, rsq + one Newton step, scale, then rank-1 updates of the owner's remaining
// columns by v_readlane broadcasts: no LDS round trip and no barrier on the pivot chain) and
// published to the LDS column buffer Lc[c][row] with a counter; the later waves apply each
// published column to their own columns as it arrives (they trail the chain by one LDS hop and
// catch up while the owner works, since an apply is cheaper than a factor step).  Measured
// constants (tools/ubench_lat64.hip, gfx950): a dependent f64 VALU op ~5.5 cycles for one wave,
// an LDS write -> read round trip ~131, a dependent f64 MFMA ~74, a balanced s_barrier ~13 --
// the pivot chain of the 8-column panel steps (MFMA trailing update + LDS round trips + a barrier
// per panel) cost ~3x this.
// Each wave then inverts its 16x16 diagonal block, X_ww = [[X_a, 0], [X_ba, X_b]] (two 8x8
// inverses, diag_inv8, and X_ba = -X_b L_ba X_a by VALU), and builds block column w of
// Li = L^-1 (see step 3 below) while the later waves still factor.
// sync (LDS ints): [0] columns published, [1 + w] X_ww written.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int lds_wait_geq(int* p, int v, int* flags) {
    int x, spins = 0;
    while ((x = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < v) {
        __builtin_amdgcn_s_sleep(0);
        if (++spins > (1 << 24)) {  // cannot happen (the producers are this workgroup's waves): fail, never hang
            flags[kFlagFail] = 1;
            return v;
        }
    }
    asm volatile("" ::: "memory");
    return x;
}
__device__ __forceinline__ void lds_publish(int* p, int v) {
    asm volatile("" ::: "memory");  // the data stores first: a wave's LDS operations execute in order
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// X_ww (16x16 diagonal block of Li) by one wave: lanes 0-7 / 8-15 the two 8x8 inverses, then
// X_ba = -X_b (L_ba X_a), lane = (r, c); scr: 64 doubles of this wave's LDS scratch
__device__ __forceinline__ void diag_inv16(const double* A, double* Li, const double* Dinv, int c0, double* scr) {
    const int lane = threadIdx.x & 63;
    {
        const int i = lane & 7, pb = c0 + (lane & 8);
        if (lane < 16) {
            double L[8][8], inv[8], x[8];
#pragma unroll
            for (int m = 0; m < 8; m++) {
                inv[m] = Dinv[pb + m];
#pragma unroll
                for (int k = 0; k < m; k++) L[m][k] = A[(pb + m) * LD + pb + k];
            }
#pragma unroll
            for (int m = 0; m < 8; m++) {
                double s = m == i ? 1.0 : 0.0;
#pragma unroll
                for (int k = 0; k < m; k++) s = fma(-L[m][k], x[k], s);
                x[m] = m >= i ? s * inv[m] : 0.0;
            }
#pragma unroll
            for (int m = 0; m < 8; m++) Li[(pb + m) * LD + pb + i] = x[m];
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int r = lane >> 3, c = lane & 7;
    double t = 0.0;  // (L_ba X_a)[r][c]
#pragma unroll
    for (int m = 0; m < 8; m++) t = fma(A[(c0 + 8 + r) * LD + c0 + m], Li[(c0 + m) * LD + c0 + c], t);
    scr[lane] = t;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    double x = 0.0;
#pragma unroll
    for (int m = 0; m < 8; m++) x = fma(Li[(c0 + 8 + r) * LD + c0 + 8 + m], scr[8 * m + c], x);
    Li[(c0 + 8 + r) * LD + c0 + c] = -x;
}

// LDS ints of the tile factor: [0] columns published, [1 + w] X_ww written, [8 + w] wave w's
// batches written to the tile (potrf_bc_w)
constexpr int kDfSync = 12;
// LDS scratch of potrf_cc (doubles): per wave 64 + a 16x17 block, then per wave a [64][4] batch
constexpr int kCcScrBase = 4 * 64 + 4 * 16 * 17;
constexpr int kCcScr = kCcScrBase + 4 * 256;
template <int W>
__device__ __forceinline__ void potrf_cc_w(double* A, double* Li, double* Lc, double* scratch, int* sync, double* Dinv,
                                           int* flags, long long* pt) {
    const int lane = threadIdx.x & 63;
    constexpr int C0 = 16 * W;
    auto wstamp = [&](int k) {
#if M3S_DF_STAMPS
        if (pt && lane == 0) pt[8 * W + k] = (long long)__builtin_amdgcn_s_memtime();
#endif
    };
    wstamp(0);
    double a[16];
#pragma unroll
    for (int jj = 0; jj < 16; jj++) a[jj] = A[lane * LD + C0 + jj];
    // 1. the earlier waves' columns, as they are published: two columns per half-iteration from
    //    two register buffers, the next pair's LDS loads issued (after polling the counter, when
    //    the backlog does not already cover them) before the current pair's FMAs.  A runtime
    //    loop: unrolled, the scheduler hoists every load and spills.
    if constexpr (W > 0) {
        int avail = lds_wait_geq(sync, 2, flags);
        double pa0, pa1, qa0[16], qa1[16], pb0, pb1, qb0[16], qb1[16];
        auto load = [&](int c, double& p0, double& p1, double (&q0)[16], double (&q1)[16]) {
            p0 = Lc[c * 64 + lane];
            p1 = Lc[(c + 1) * 64 + lane];
#pragma unroll
            for (int jj = 0; jj < 16; jj++) {
                q0[jj] = Lc[c * 64 + C0 + jj];
                q1[jj] = Lc[(c + 1) * 64 + C0 + jj];
            }
        };
        auto apply = [&](double p0, double p1, const double (&q0)[16], const double (&q1)[16]) {
#pragma unroll
            for (int jj = 0; jj < 16; jj++) a[jj] = fma(-p1, q1[jj], fma(-p0, q0[jj], a[jj]));
        };
        load(0, pa0, pa1, qa0, qa1);
#pragma unroll 1
        for (int c = 0; c < C0; c += 4) {
            if (c + 4 > avail) avail = lds_wait_geq(sync, c + 4, flags);
            load(c + 2, pb0, pb1, qb0, qb1);
            apply(pa0, pa1, qa0, qa1);
            if (c + 4 < C0) {
                if (c + 6 > avail) avail = lds_wait_geq(sync, c + 6, flags);
                load(c + 4, pa0, pa1, qa0, qa1);
            }
            apply(pb0, pb1, qb0, qb1);
        }
    }
    wstamp(1);
    // 2. the own columns: the pivot chain, in batches of 4 columns.  Inside a batch each pivot
    //    updates the batch's later columns by v_readlane (on the chain); after a batch, its
    //    rank-4 update of the wave's remaining columns reads the 4 values of each target row from
    //    a row-major copy of the batch (two uniform ds_read_b128 + 4 FMAs per column instead of
    //    4 x (2 v_readlane + FMA): the owner's issue is what bounds its per-column time)
    double y[16];
    bool bad = false;
    double* Lr = scratch + kCcScrBase + 256 * W;  // this wave's batch, row-major [64][4]
#pragma unroll
    for (int ib = 0; ib < 4; ib++) {
#pragma unroll
        for (int p = 0; p < 4; p++) {
            const int jj = 4 * ib + p, c = C0 + jj;
            const double d = rdlane(a[jj], c);
            bad |= d <= 0.0;  // SimplicialLLT: fails iff a pivot <= 0 (NaN passes)
            double r = __builtin_amdgcn_rsq(d);
            r = r * fma(-0.5 * d * r, r, 1.5);
            y[jj] = r;
            a[jj] *= r;
            if (W < 3) {
                Lc[c * 64 + lane] = a[jj];
                lds_publish(sync, c + 1);
            }
#pragma unroll
            for (int q = p + 1; q < 4; q++) a[4 * ib + q] = fma(-a[jj], rdlane(a[jj], C0 + 4 * ib + q), a[4 * ib + q]);
        }
        if (ib < 3) {
            const int NQ = 12 - 4 * ib;  // this batch's target columns: all loaded, then used
#pragma unroll
            for (int p = 0; p < 4; p++) Lr[lane * 4 + p] = a[4 * ib + p];
            double v[12][4];
#pragma unroll
            for (int q = 0; q < 12; q++)
                if (q < NQ) {
#pragma unroll
                    for (int p = 0; p < 4; p++) v[q][p] = Lr[(C0 + 4 * ib + 4 + q) * 4 + p];
                }
#pragma unroll
            for (int q = 0; q < 12; q++)
                if (q < NQ)
#pragma unroll
                for (int p = 0; p < 4; p++) a[4 * ib + 4 + q] = fma(-a[4 * ib + p], v[q][p], a[4 * ib + 4 + q]);
        }
    }
    // L back into the tile (every lane: rows above the pivots write upper-triangle garbage,
    // never read), 1 / l_pp for the inverse
#pragma unroll
    for (int jj = 0; jj < 16; jj++) A[lane * LD + C0 + jj] = a[jj];
    if (lane == 0) {
        if (bad) flags[kFlagFail] = 1;
#pragma unroll
        for (int jj = 0; jj < 16; jj++) Dinv[C0 + jj] = y[jj];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // 3. the inverse: X_WW (diagonal block), flagged; then block column W of X, column-oriented:
    //    X_VW = -X_VV sum_{m=W}^{V-1} L_Vm X_mW for V > W -- the sums need only L (Lc) and this
    //    wave's own earlier blocks, so each is ready before X_VV is flagged and the tail after the
    //    last column is wave 3's X_33 plus one 16x16 product per column block
    double* scr = scratch + 64 * W;               // this wave's scratch
    double* sT = scratch + 4 * 64 + 16 * 17 * W;  // ... and its 16 x 17 block
    wstamp(2);
    diag_inv16(A, Li, Dinv, C0, scr);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    lds_publish(sync + 1 + W, 1);
    wstamp(3);
    const int r16 = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int V = W + 1; V < 4; V++) {
        lds_wait_geq(sync, 16 * V, flags);  // L_Vm, m < V: the columns of blocks < V published
        d4 acc[4];
#pragma unroll
        for (int m = W; m < V; m++) {
            acc[m] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int st = 0; st < 4; st++)
                acc[m] = mfma(Lc[(16 * m + 4 * st + kq) * 64 + 16 * V + r16],
                              Li[(16 * m + 4 * st + kq) * LD + C0 + r16], acc[m]);
        }
        d4 t = acc[W];
#pragma unroll
        for (int m = W + 1; m < V; m++) t += acc[m];
#pragma unroll
        for (int e = 0; e < 4; e++) sT[(kq + 4 * e) * 17 + r16] = t[e];
        lds_wait_geq(sync + 1 + V, 1, flags);  // X_VV
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        d4 x = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int st = 0; st < 4; st++)
            x = mfma(-Li[(16 * V + r16) * LD + 16 * V + 4 * st + kq], sT[(4 * st + kq) * 17 + r16], x);
#pragma unroll
        for (int e = 0; e < 4; e++) Li[(16 * V + kq + 4 * e) * LD + C0 + r16] = x[e];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // X_VW before the next V's sum reads it
        wstamp(4 + V - W - 1);
    }
}

// Batch-cyclic variant (M3S_DF_BC=1): the tile's 16 batches of 4 columns go round-robin to the
// 4 waves (batch b -> wave b % 4; wave w holds columns 16 lb + 4 w + p in registers, lane = row).
// The owner of batch b applies batch b-1 to its 4 columns only, factors them (pivots by
// v_readlane, as potrf_cc) and publishes them as a row-major [64][4] copy (Lb + 256 b; the
// consumers read a target row's 4 values with two uniform ds_read_b128) plus into the tile (the
// inverse reads L there); every wave applies each published batch to its own later columns off
// the critical path.  The pivot chain thus hands over every 4 columns instead of every 16, and
// between two of its columns the owner issues 4 FMAs of rank-4 update instead of the whole
// 16-column block's -- the owner's issue, not the hand-off, bounded potrf_cc (~260 cycles per
// column).  The inverse (X_WW by wave W, then the column-block products) follows the last batch;
// it reads L from the tile, which each wave writes after its publish (off the critical path) and
// announces on its own counter (sync[8 + w]: batches written).  Measured (ubench_potrf64 /
// ubench_chol_df, profiles/r04_ak_*): ~940 cycles per batch hand-off + factor, tile factor +
// inverse 8.0 us vs potrf_cc's 10.2 us in the chain; 8-column batches (M3S_DF_BC_W=8) 9.6 us.
template <int W, int BW>
__device__ __forceinline__ void potrf_bc_w(double* A, double* Li, double* Lb, double* scratch, int* sync, double* Dinv,
                                           int* flags, long long* pt) {
    constexpr int NL = 16 / BW;  // local batches per wave
    const int lane = threadIdx.x & 63;
    auto wstamp = [&](int k) {
#if M3S_DF_STAMPS
        if (pt && lane == 0) pt[8 * W + k] = (long long)__builtin_amdgcn_s_memtime();
#endif
    };
    // per-batch stamps (ubench_potrf64 only: M3S_DF_BSTAMPS): pt[20 + 2 nb] the critical wait
    // done, pt[21 + 2 nb] the critical apply done
    auto bstamp = [&](int k) {
#if M3S_DF_STAMPS && M3S_DF_BSTAMPS
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (pt && lane == 0) pt[20 + k] = (long long)__builtin_amdgcn_s_memtime();
#else
        (void)k;
#endif
    };
    wstamp(0);
    double a[16];  // a[BW lb + p]: column BW (4 lb + W) + p
#pragma unroll
    for (int lb = 0; lb < NL; lb++)
#pragma unroll
        for (int p = 0; p < BW; p++) a[BW * lb + p] = A[lane * LD + BW * (4 * lb + W) + p];
    bool bad = false;
    // batch b (published) applied to my local batches lb0 .. lb1 - 1
    auto apply = [&](int b, int lb0, int lb1) {
        const double* Lr = Lb + 64 * BW * b;
        double2 r[BW / 2];
#pragma unroll
        for (int k = 0; k < BW / 2; k++) r[k] = *reinterpret_cast<const double2*>(Lr + lane * BW + 2 * k);
#pragma unroll
        for (int lb = 0; lb < NL; lb++) {
            if (lb < lb0 || lb >= lb1) continue;
            double2 cv[BW][BW / 2];
#pragma unroll
            for (int p = 0; p < BW; p++)
#pragma unroll
                for (int k = 0; k < BW / 2; k++)
                    cv[p][k] = *reinterpret_cast<const double2*>(Lr + (BW * (4 * lb + W) + p) * BW + 2 * k);
#pragma unroll
            for (int p = 0; p < BW; p++) {
                double v = a[BW * lb + p];
#pragma unroll
                for (int k = 0; k < BW / 2; k++) {
                    v = fma(-r[k].x, cv[p][k].x, v);
                    v = fma(-r[k].y, cv[p][k].y, v);
                }
                a[BW * lb + p] = v;
            }
        }
    };
    constexpr int C0 = 16 * W;
    double* scr = scratch + 64 * W;
    double* sT = scratch + 4 * 64 + 16 * 17 * W;
    // columns < C of L written to the tile: each wave's batches below C / BW (in order per wave)
    auto wait_written = [&](int C) {
        int need[4], spins = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) need[q] = C / BW > q ? (C / BW - q + 3) / 4 : 0;
        for (;;) {  // the four counters read together: one LDS round trip per poll
            int n[4];
#pragma unroll
            for (int q = 0; q < 4; q++) n[q] = __hip_atomic_load(sync + 8 + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (n[0] >= need[0] && n[1] >= need[1] && n[2] >= need[2] && n[3] >= need[3]) break;
            __builtin_amdgcn_s_sleep(0);
            if (++spins > (1 << 24)) {  // cannot happen (the producers are this workgroup's waves)
                flags[kFlagFail] = 1;
                break;
            }
        }
        asm volatile("" ::: "memory");
    };
    // X_WW = (L_WW)^-1 once block column W of L is in the tile.  (Measured slower: doing it for
    // waves 0 and 1 inside the batch loop as soon as their block is complete, 292 vs 283 us on the
    // cfg4-size chain; X_WW as 16 forward substitutions of 16 rows by lanes 0-15 instead of
    // diag_inv16's two 8x8 inverses + products, ~2.8k vs ~1.8k cycles, 284 vs 278 us.)
    auto diag_block = [&]() {
        wait_written(16 * (W + 1));
        bstamp(32 + W);
        diag_inv16(A, Li, Dinv, C0, scr);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        lds_publish(sync + 1 + W, 1);
        wstamp(5);
    };
    int next = 0;  // the next batch to apply to my columns
#pragma unroll
    for (int lb = 0; lb < NL; lb++) {
        const int nb = 4 * lb + W;
        // the other waves' earlier batches, to all my remaining columns (off the critical path)
#pragma unroll 1
        for (; next < nb - 1; next++) {
            lds_wait_geq(sync, BW * (next + 1), flags);
            apply(next, lb, NL);
        }
        if (nb >= 1) {  // the previous batch: to this batch's columns first (the critical path)
#if M3S_DF_BC_SPEC
            // the counter and the batch's values read together, the values kept once the counter
            // shows the batch published (the producer stored them before the counter, and a wave's
            // LDS reads execute in order): one LDS round trip per hand-off instead of two (wait +
            // apply ~490 -> ~400 cycles per batch, bitwise the same L; profiles/r04_ao_*)
            const double* Lr = Lb + 64 * BW * (nb - 1);
            double2 r[BW / 2], cv[BW][BW / 2];
            for (int spins = 0;; spins++) {
                const int n = __hip_atomic_load(sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                asm volatile("" ::: "memory");
#pragma unroll
                for (int k = 0; k < BW / 2; k++) r[k] = *reinterpret_cast<const double2*>(Lr + lane * BW + 2 * k);
#pragma unroll
                for (int p = 0; p < BW; p++)
#pragma unroll
                    for (int k = 0; k < BW / 2; k++)
                        cv[p][k] = *reinterpret_cast<const double2*>(Lr + (BW * nb + p) * BW + 2 * k);
                if (n >= BW * nb) break;
                __builtin_amdgcn_s_sleep(0);
                if (spins > (1 << 24)) {  // cannot happen (the producer is this workgroup's wave)
                    flags[kFlagFail] = 1;
                    break;
                }
            }
            bstamp(2 * nb);
#pragma unroll
            for (int p = 0; p < BW; p++) {
                double v = a[BW * lb + p];
#pragma unroll
                for (int k = 0; k < BW / 2; k++) {
                    v = fma(-r[k].x, cv[p][k].x, v);
                    v = fma(-r[k].y, cv[p][k].y, v);
                }
                a[BW * lb + p] = v;
            }
#else
            lds_wait_geq(sync, BW * nb, flags);
            bstamp(2 * nb);
            apply(nb - 1, lb, lb + 1);
#endif
            bstamp(2 * nb + 1);
        }
        // factor the batch: pivot chain inside it by v_readlane.  (Reading the batch's diagonal
        // block once and factoring it as wave-uniform values -- bitwise the same L -- measured
        // no faster: ~600 cycles per batch either way.)
        const int c0 = BW * nb;
        double y[BW];
#pragma unroll
        for (int p = 0; p < BW; p++) {
            const int jj = BW * lb + p, c = c0 + p;
            const double d = rdlane(a[jj], c);
            bad |= d <= 0.0;  // SimplicialLLT: fails iff a pivot <= 0 (NaN passes)
            double r = __builtin_amdgcn_rsq(d);
            r = r * fma(-0.5 * d * r, r, 1.5);
            y[p] = r;
            a[jj] *= r;
#pragma unroll
            for (int q = p + 1; q < BW; q++) a[BW * lb + q] = fma(-a[jj], rdlane(a[jj], c0 + q), a[BW * lb + q]);
        }
        // publish: the row-major copy, then the counter (a wave's LDS operations execute in order)
        double* Lr = Lb + 64 * BW * nb;
#pragma unroll
        for (int k = 0; k < BW / 2; k++)
            *reinterpret_cast<double2*>(Lr + lane * BW + 2 * k) = double2{a[BW * lb + 2 * k], a[BW * lb + 2 * k + 1]};
        lds_publish(sync, BW * (nb + 1));
        wstamp(1 + lb);
        // the columns into the tile and 1 / l_pp (the inverse reads both): off the critical path,
        // published by this wave's own counter
#pragma unroll
        for (int p = 0; p < BW; p++) A[lane * LD + c0 + p] = a[BW * lb + p];
        {
            double yl = y[0];
#pragma unroll
            for (int p = 1; p < BW; p++) yl = lane == p ? y[p] : yl;
            if (lane < BW) Dinv[c0 + lane] = yl;
        }
        lds_publish(sync + 8 + W, lb + 1);
        // the previous batch and my own, to my later columns
        if (lb < NL - 1) {
            if (nb >= 1) apply(nb - 1, lb + 1, NL);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // my copy of batch nb is in LDS
            apply(nb, lb + 1, NL);
        }
        next = nb + 1;
    }
    if (lane == 0 && bad) flags[kFlagFail] = 1;
    // the inverse, as potrf_cc's step 3, with L read from the tile
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    diag_block();
    const int r16 = lane & 15, kq = lane >> 4;
#if M3S_DF_BC_RL
    // block column W of Li, right-looking: once X_mW is known, its products L_Vm X_mW go into
    // every later block row's accumulator (t_V = sum_m L_Vm X_mW), the next row's first; then
    // X_{m+1,W} = -X_{m+1,m+1} t_{m+1}.  Only the last product waits on X_33, instead of the whole
    // t_3W (up to 12 MFMAs) being issued after X_20 / X_21.  The same products summed in another
    // order than the left-looking form below (the acc[m] chains added in m order): not bitwise.
    // (L's block column m is in the tile: for m = W diag_block waited for it, for m > W the wave
    // that published X_mm did.)
    d4 acc[4];
#pragma unroll
    for (int V = 0; V < 4; V++) acc[V] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int m = W; m < 3; m++) {
#pragma unroll
        for (int V = m + 1; V < 4; V++)
#pragma unroll
            for (int st = 0; st < 4; st++)
                acc[V] = mfma(A[(16 * V + r16) * LD + 16 * m + 4 * st + kq], Li[(16 * m + 4 * st + kq) * LD + C0 + r16],
                              acc[V]);
        const int V = m + 1;
#pragma unroll
        for (int e = 0; e < 4; e++) sT[(kq + 4 * e) * 17 + r16] = acc[V][e];
        lds_wait_geq(sync + 1 + V, 1, flags);  // X_VV
        d4 x = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int st = 0; st < 4; st++)
            x = mfma(-Li[(16 * V + r16) * LD + 16 * V + 4 * st + kq], sT[(4 * st + kq) * 17 + r16], x);
#pragma unroll
        for (int e = 0; e < 4; e++) Li[(16 * V + kq + 4 * e) * LD + C0 + r16] = x[e];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#else
#pragma unroll
    for (int V = W + 1; V < 4; V++) {
        wait_written(16 * V);
        d4 acc[4];
#pragma unroll
        for (int m = W; m < V; m++) {
            acc[m] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int st = 0; st < 4; st++)
                acc[m] = mfma(A[(16 * V + r16) * LD + 16 * m + 4 * st + kq], Li[(16 * m + 4 * st + kq) * LD + C0 + r16],
                              acc[m]);
        }
        d4 t = acc[W];
#pragma unroll
        for (int m = W + 1; m < V; m++) t += acc[m];
#pragma unroll
        for (int e = 0; e < 4; e++) sT[(kq + 4 * e) * 17 + r16] = t[e];
        lds_wait_geq(sync + 1 + V, 1, flags);  // X_VV
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        d4 x = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int st = 0; st < 4; st++)
            x = mfma(-Li[(16 * V + r16) * LD + 16 * V + 4 * st + kq], sT[(4 * st + kq) * 17 + r16], x);
#pragma unroll
        for (int e = 0; e < 4; e++) Li[(16 * V + kq + 4 * e) * LD + C0 + r16] = x[e];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
#endif
    wstamp(6);
}

// the register factor + inverse of the tile: batch-cyclic (potrf_bc_w, M3S_DF_BC=1, default) or
// column-cyclic (potrf_cc_w); sync[0 .. kDfSync) zeroed and visible
__device__ __forceinline__ void potrf_cc(double* A, double* Li, double* Lc, double* scratch, int* sync, double* Dinv,
                                         int* flags, long long* pt = nullptr) {
#if M3S_DF_BC
    switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {
        case 0: potrf_bc_w<0, M3S_DF_BC_W>(A, Li, Lc, scratch, sync, Dinv, flags, pt); break;
        case 1: potrf_bc_w<1, M3S_DF_BC_W>(A, Li, Lc, scratch, sync, Dinv, flags, pt); break;
        case 2: potrf_bc_w<2, M3S_DF_BC_W>(A, Li, Lc, scratch, sync, Dinv, flags, pt); break;
        default: potrf_bc_w<3, M3S_DF_BC_W>(A, Li, Lc, scratch, sync, Dinv, flags, pt); break;
    }
#else
    switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {
        case 0: potrf_cc_w<0>(A, Li, Lc, scratch, sync, Dinv, flags, pt); break;
        case 1: potrf_cc_w<1>(A, Li, Lc, scratch, sync, Dinv, flags, pt); break;
        case 2: potrf_cc_w<2>(A, Li, Lc, scratch, sync, Dinv, flags, pt); break;
        default: potrf_cc_w<3>(A, Li, Lc, scratch, sync, Dinv, flags, pt); break;
    }
#endif
    __syncthreads();
}

// Z (lower 16x16 blocks) -= X X^T, X: [64][LD] in LDS.  The 10 lower blocks are dealt 3/3/2/2 to
// the waves (a wave per block row would give wave 3 four blocks, 64 MFMAs): 48 MFMAs on the
// busiest wave instead of the full product's 64.
template <int W>
__device__ __forceinline__ void syrk_lower_w(double* Z, const double* X) {
    constexpr int BI[4][3] = {{0, 1, 2}, {1, 2, 3}, {2, 3, 0}, {3, 3, 0}};
    constexpr int BJ[4][3] = {{0, 0, 0}, {1, 1, 0}, {2, 1, 0}, {2, 3, 0}};
    constexpr int NB = W < 2 ? 3 : 2;
    const int lane = threadIdx.x & 63;
    const int r = lane & 15, kq = lane >> 4;
    d4 acc[NB];
#pragma unroll
    for (int b = 0; b < NB; b++)
#pragma unroll
        for (int e = 0; e < 4; e++) acc[b][e] = Z[(16 * BI[W][b] + kq + 4 * e) * LD + 16 * BJ[W][b] + r];
#pragma unroll
    for (int st = 0; st < 16; st++) {
        double x[NB], y[NB];
#pragma unroll
        for (int b = 0; b < NB; b++) {
            x[b] = -X[(16 * BI[W][b] + r) * LD + 4 * st + kq];
            y[b] = X[(16 * BJ[W][b] + r) * LD + 4 * st + kq];
        }
#pragma unroll
        for (int b = 0; b < NB; b++) acc[b] = mfma(x[b], y[b], acc[b]);
    }
#pragma unroll
    for (int b = 0; b < NB; b++)
#pragma unroll
        for (int e = 0; e < 4; e++) Z[(16 * BI[W][b] + kq + 4 * e) * LD + 16 * BJ[W][b] + r] = acc[b][e];
}
__device__ __forceinline__ void syrk_lower(double* Z, const double* X) {
    switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {
        case 0: syrk_lower_w<0>(Z, X); break;
        case 1: syrk_lower_w<1>(Z, X); break;
        case 2: syrk_lower_w<2>(Z, X); break;
        default: syrk_lower_w<3>(Z, X); break;
    }
}

// Workgroup 0 runs the whole diagonal chain C: for j = 0 .. nt-1
//   L_{j,j-1} = P_s(j) Linv_{j-1}^T   (Linv_{j-1} still in LDS from the previous step)
//   A'_jj     = P_d(j) - L_{j,j-1} L_{j,j-1}^T
//   potrf(A'_jj) -> L_jj, Linv_j
// where P_s(j) = A_{j,j-1} - sum_{k<=j-2} L_{j,k} L_{j-1,k}^T and P_d(j) = A_jj - sum_{k<=j-2}
// L_{j,k} L_{j,k}^T are left-looking partial sums by helper task H_j (they depend on columns
// <= j-2 only, so they are ready while C factors column j-1).  Between two potrfs only C's own
// registers / LDS are on the critical path.  Helpers (the other workgroups) walk, column-major,
// the regular tiles (i, j), i = j+2 .. nt (and (nt, nt-1)), then H_{j+2}, each left-looking:
//   acc = A_ij - sum_{k<j} L_ik L_jk^T, wait Linv_j, L_ij = acc Linv_j^T.
// C publishes L_{j,j-1} inside potrf(j) (after its first panel step) and Linv_j once its next
// loads drained the store queue, so no store latency sits on the chain either.
__host__ __device__ inline int col_tasks(int j, int nt) {
    return (j < nt - 1 ? nt - j - 1 : 1) + (j + 2 <= nt - 1 ? 1 : 0);
}
__host__ __device__ inline int num_tasks(int nt) {  // helper tasks
    int n = 0;
    for (int j = 0; j < nt; j++) n += col_tasks(j, nt);
    return n;
}
__host__ __device__ inline int hflag(int nt, int j) { return (nt + 1) * nt + j; }  // H_j ready word

__device__ __forceinline__ void acc_to_lds(double* S, const d4 acc[4]) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int J = 0; J < 4; J++)
#pragma unroll
        for (int e = 0; e < 4; e++) S[(16 * w + (lane >> 4) + 4 * e) * LD + 16 * J + (lane & 15)] = acc[J][e];
}
template <bool COH>
__device__ __forceinline__ void load_acc(d4 acc[4], const double* src, int64_t ld) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int J = 0; J < 4; J++)
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const double* p = src + (int64_t)(16 * w + (lane >> 4) + 4 * e) * ld + 16 * J + (lane & 15);
            acc[J][e] = COH ? ld_coh(p) : *p;
        }
}
// the original tile (i, j) of the filled dense matrix
__device__ __forceinline__ void load_src(d4 acc[4], const DfArgs& a, int i, int j) {
    load_acc<false>(acc, a.Hd + (int64_t)i * T * a.npad + (int64_t)j * T, a.npad);
}
__device__ __forceinline__ void store_acc_coh(double* dst, int64_t ld, const d4 acc[4]) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int J = 0; J < 4; J++)
#pragma unroll
        for (int e = 0; e < 4; e++) st_coh(dst + (int64_t)(16 * w + (lane >> 4) + 4 * e) * ld + 16 * J + (lane & 15), acc[J][e]);
}
// after this workgroup's write-through stores landed, set a ready word.  Every handed-off byte
// is stored write-through (sc1) and loaded sc1, and every storing wave waits for its stores
// before the barrier, so the flag is a relaxed sc1 store: no release fence (an L2 write-back,
// ~1.7 us per hand-off; MI355X_MICROARCH.md, "Valid forms", first row of the hand-off table)
__device__ __forceinline__ void publish(const DfArgs& a, int idx) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(a.ready + idx, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__host__ __device__ inline int xflag(int nt, int j) { return (nt + 1) * nt + nt + j; }  // (M3S_DF_XGRAN=0)
// x_j[c] -> its two granules (one lane each call)
__device__ __forceinline__ void publish_x(const DfArgs& a, int j, int c, double xv) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(xv);
    const unsigned long long tag = (unsigned long long)(unsigned)a.epoch << 32;
    unsigned long long* g = a.xg + 2 * ((int64_t)j * T + c);
    __hip_atomic_store(g, tag | (b & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(g + 1, tag | (b >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one wave: x_k, lane c = entry c, once every lane's two granules carry this factorisation's epoch
// (bounded like wait_ready: a timeout fails the solve and raises the sticky timeout flag)
__device__ __forceinline__ double wait_x(const DfArgs& a, int k) {
    const int lane = threadIdx.x & 63;
    const unsigned long long* g = a.xg + 2 * ((int64_t)k * T + lane);
    const unsigned ep = (unsigned)a.epoch;
    unsigned long long lo = 0, hi = 0;
    for (int spins = 0;;) {
        lo = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        hi = __hip_atomic_load(g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__all((unsigned)(lo >> 32) == ep && (unsigned)(hi >> 32) == ep)) break;
        if (a.spin_limit < 0 || ++spins > a.spin_limit) {
            if (lane == 0) {
                __hip_atomic_store(a.flags + kFlagTimeout, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(a.flags + kFlagFail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            break;
        }
        if ((spins & 1023) == 0 && __hip_atomic_load(a.flags + kFlagFail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            break;
        __builtin_amdgcn_s_sleep(1);
    }
    return __hiloint2double((int)(unsigned)hi, (int)(unsigned)lo);
}
// Back-substitution task of the tile columns jh and jl = jh - 1 (jl < 0: jh alone), after the
// factor tasks in the helpers' lists, in descending order: z_j = y_j - sum_{k>j} L_kj^T x_k,
// x_j = Linv_j^T z_j, published as data-tagged granules (publish_x / wait_x).  Each x_k is applied as soon as it is
// published, so when the previous pair's x arrive only their terms, the sums and the Linv
// products are left -- and x_jh feeds x_jl inside the workgroup (L_{jh,jl}^T x_jh): one hand-off
// per two tile columns on the back-substitution chain (a hand-off -- write-through store, flag,
// spin, coherent load -- is ~3 us: 16 of them were 54 us of cfg4's factorisation, r04_r).
// Thread (c, g): column c, rows 16g .. 16g+15 of each tile; the 4 row-group partials are summed
// in fixed order (deterministic).  Every wait targets a task of a smaller ticket (claimed by a
// running workgroup): no deadlock.
__device__ void back_pair(const DfArgs& a, int jh, int jl, double* S) {
    const int tid = threadIdx.x, c = tid & 63, g = tid >> 6;
    const int nt = a.nt;
    const int64_t ld = a.npad;
    const bool two = jl >= 0;
    double* sx = S;                    // x_k (64)
    double* sp = S + 64;               // partials [4][64]
    double* sz = S + 64 + 256;         // z (64)
    double* sxh = S + 64 + 256 + 64;   // x_jh (64)
    auto Lt = [&](int k, int j) { return a.Hd + (int64_t)k * T * ld + (int64_t)j * T; };
    // the tiles this task reads are final long before the x chain reaches it: their words are
    // checked one step ahead and each tile is loaded while the previous x_k is awaited
    double acc_h = 0.0, acc_l = 0.0, lvh[16], lvl[16], lih[16], lil[16], lhl[16];
    // diagnostics (tools/ubench_chol_df.hip, M3S_DF_STAMPS): 4 stamps per pair after the chain's
    auto bstamp = [&](int slot) {
#if M3S_DF_STAMPS
        if (a.trace && tid == 0)
            a.trace[4 * a.ntiles + 32 + 8 * nt + 4 * ((nt - 1 - jh) / 2) + slot] = (long long)__builtin_amdgcn_s_memrealtime();
#endif
    };
    if (tid == 0) {
        wait_ready(a.ready + jh * nt + jh, a.epoch, a.flags, a.spin_limit);  // Linv_jh
        if (jh + 1 < nt) wait_ready(a.ready + (nt - 1) * nt + jh, a.epoch, a.flags, a.spin_limit);
        if (two) {
            wait_ready(a.ready + jl * nt + jl, a.epoch, a.flags, a.spin_limit);  // Linv_jl
            wait_ready(a.ready + jh * nt + jl, a.epoch, a.flags, a.spin_limit);  // L_{jh,jl}
            if (jh + 1 < nt) wait_ready(a.ready + (nt - 1) * nt + jl, a.epoch, a.flags, a.spin_limit);
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 16; q++) lih[q] = ld_coh(a.Linv + (int64_t)jh * T * T + (16 * g + q) * T + c);
    if (two) {
#pragma unroll
        for (int q = 0; q < 16; q++) {
            lil[q] = ld_coh(a.Linv + (int64_t)jl * T * T + (16 * g + q) * T + c);
            lhl[q] = ld_coh(Lt(jh, jl) + (int64_t)(16 * g + q) * ld + c);
        }
    }
    if (jh + 1 < nt) {
#pragma unroll
        for (int q = 0; q < 16; q++) lvh[q] = ld_coh(Lt(nt - 1, jh) + (int64_t)(16 * g + q) * ld + c);
        if (two) {
#pragma unroll
            for (int q = 0; q < 16; q++) lvl[q] = ld_coh(Lt(nt - 1, jl) + (int64_t)(16 * g + q) * ld + c);
        }
    }
    // y_jh, y_jl (the border row: forward-substituted during the factorisation) prefetched, off
    // the x chain
    if (tid == 0) {
        wait_ready(a.ready + nt * nt + jh, a.epoch, a.flags, a.spin_limit);
        if (two) wait_ready(a.ready + nt * nt + jl, a.epoch, a.flags, a.spin_limit);
    }
    __syncthreads();
    const double yh = tid < 64 ? ld_coh(a.Hd + (int64_t)ld * ld + (int64_t)jh * T + c) : 0.0;
    const double yl = (two && tid < 64) ? ld_coh(a.Hd + (int64_t)ld * ld + (int64_t)jl * T + c) : 0.0;
    bstamp(0);
    for (int k = nt - 1; k > jh; k--) {
        if (tid == 0 && k - 1 > jh) {  // the next tiles' words (final long ago: no wait in practice)
            wait_ready(a.ready + (k - 1) * nt + jh, a.epoch, a.flags, a.spin_limit);
            if (two) wait_ready(a.ready + (k - 1) * nt + jl, a.epoch, a.flags, a.spin_limit);
        }
        if (a.xgran) {
            if (tid < 64) sx[tid] = wait_x(a, k);  // wave 0 polls x_k's granules until all are this epoch's
            __syncthreads();
        } else {
            if (tid == 0) wait_ready(a.ready + xflag(nt, k), a.epoch, a.flags, a.spin_limit);
            __syncthreads();
            if (tid < 64) sx[tid] = ld_coh(a.x + (int64_t)k * T + tid);
        }
        double ch[16], cl[16];
#pragma unroll
        for (int q = 0; q < 16; q++) {
            ch[q] = lvh[q];
            cl[q] = lvl[q];
        }
        if (k - 1 > jh) {
#pragma unroll
            for (int q = 0; q < 16; q++) lvh[q] = ld_coh(Lt(k - 1, jh) + (int64_t)(16 * g + q) * ld + c);
            if (two) {
#pragma unroll
                for (int q = 0; q < 16; q++) lvl[q] = ld_coh(Lt(k - 1, jl) + (int64_t)(16 * g + q) * ld + c);
            }
        }
        lds_barrier();
#pragma unroll
        for (int q = 0; q < 16; q++) acc_h = fma(ch[q], sx[16 * g + q], acc_h);
        if (two) {
#pragma unroll
            for (int q = 0; q < 16; q++) acc_l = fma(cl[q], sx[16 * g + q], acc_l);
        }
        lds_barrier();  // sx is rewritten by the next k
    }
    // x_j = Linv_j^T (y_j - acc) for the column (j, y, acc, Linv rows): into xs (LDS), x and
    // xpose (LDS-only barriers: the x stores stay in flight until the publish)
    auto finish = [&](int j, double y, double acc, const double (&li)[16], double* xs) {
        sp[g * 64 + c] = acc;
        lds_barrier();
        if (tid < 64) sz[c] = y - (((sp[c] + sp[64 + c]) + sp[128 + c]) + sp[192 + c]);
        lds_barrier();
        double xp = 0.0;
#pragma unroll
        for (int q = 0; q < 16; q++) xp = fma(li[q], sz[16 * g + q], xp);
        sp[g * 64 + c] = xp;
        lds_barrier();
        if (tid < 64) {
            const double xv = ((sp[c] + sp[64 + c]) + sp[128 + c]) + sp[192 + c];
            xs[c] = xv;
            if (a.xgran) {
                publish_x(a, j, c, xv);  // the granules: the next pair task polls them
                a.x[(int64_t)j * T + c] = xv;  // the copy later launches read
            } else {
                st_coh(a.x + (int64_t)j * T + c, xv);
            }
            const int q = j * T + c;  // the pose-indexed copy the back rounds read (no scatter launch)
            if (a.g.xpose && q < 7 * a.g.ntail) a.g.xpose[(int64_t)a.g.tail[q / 7] * 7 + q % 7] = xv;
        }
        lds_barrier();
    };
    bstamp(1);
    finish(jh, yh, acc_h, lih, sxh);
    bstamp(2);
    if (two) {
#pragma unroll
        for (int q = 0; q < 16; q++) acc_l = fma(lhl[q], sxh[16 * g + q], acc_l);
        finish(jl, yl, acc_l, lil, sx);
    }
    if (!a.xgran) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            __hip_atomic_store(a.ready + xflag(nt, jh), a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (two) __hip_atomic_store(a.ready + xflag(nt, jl), a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    bstamp(3);
}

__global__ __launch_bounds__(NT) void chol_df_kernel(DfArgs a) {
    if (solve_skipped(a.flags)) return;  // written by earlier launches: all workgroups agree
    __shared__ __attribute__((aligned(16))) double X[T * LD];
    __shared__ __attribute__((aligned(16))) double Y[T * LD];
    __shared__ __attribute__((aligned(16))) double Z[T * LD];
    __shared__ double Dinv[T];
    __shared__ double Scr[kCcScr];
    __shared__ int Sync[kDfSync];
    const int tid = threadIdx.x;
    const int nt = a.nt;
    const int64_t ld = a.npad;
    auto tile = [&](int i, int j) { return a.Hd + (int64_t)i * T * ld + (int64_t)j * T; };
    long long* ct = a.trace ? a.trace + 4 * a.ntiles + 32 : nullptr;  // C's per-step stamps
    auto cstamp = [&](int j, int slot) {
        if (ct && tid == 0) ct[4 * j + slot] = (long long)__builtin_amdgcn_s_memrealtime();
    };
    // M3S_DF_STAMPS (diagnostics): finer chain stamps after the P loads, L_{j,j-1}, the syrk
    auto fstamp = [&](int j, int slot) {
#if M3S_DF_STAMPS
        if (ct && tid == 0) ct[4 * nt + 4 * j + slot] = (long long)__builtin_amdgcn_s_memrealtime();
#endif
    };
    // Tasks are dealt dynamically: a workgroup claims ticket after ticket from
    // one counter and leaves once the tickets are spent.  Ticket 0 is the diagonal chain, ticket
    // 1 + t helper task t in the column-major order below, then the back-substitution pairs.
    // Every wait targets the output of a smaller ticket (or a chain step those tickets already
    // passed), and a ticket is only ever held by a RUNNING workgroup -- so the factorisation makes
    // progress with any number of its workgroups resident: a grid that starts partly late (CUs held
    // by another stream's kernels) only runs slower, never deadlocks or times out, and every task
    // computes the same values whichever workgroup runs it (bitwise the unhindered result).
    // The last workgroup to leave re-zeroes the counters for the next launch (stream order).
    __shared__ int s_ticket;
    const int ntasks = a.ntiles + (a.x != nullptr ? (nt + 1) / 2 : 0);
    int nclaim = 0;
    auto claim = [&]() {
        int t;
        if (a.dyn) {
            if (tid == 0) s_ticket = __hip_atomic_fetch_add(a.tick, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __syncthreads();
            t = s_ticket;
            __syncthreads();  // (s_ticket is rewritten by the next claim)
        } else {  // M3S_DF_DYN=0 (A/B): the former static deal -- workgroup 0 the chain, b >= 1 tasks b-1 + k (G-1)
            t = blockIdx.x == 0 ? 0 : (int)blockIdx.x + nclaim * ((int)gridDim.x - 1);
        }
        nclaim++;
        return t;
    };
    // the last workgroup out re-zeroes the ticket and exit counters (the next launch on this
    // stream starts after this one has completed, so it sees them zeroed)
    auto leave = [&]() {
        if (a.dyn && tid == 0 &&
            __hip_atomic_fetch_add(a.tick + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1) {
            __hip_atomic_store(a.tick, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.tick + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    // (the chain and the task loop are separate regions, as with the static deal: wrapped in one
    // claim loop, the chain's registers and the tasks' stayed live together -- 143 VGPRs spilled)
    int ticket = claim();
    if (ticket == 0) {
        // ---- the diagonal chain
        for (int j = 0; j < nt; j++) {
            d4 accd[4];
            if (j >= 2) {
                if (tid == 0) wait_ready(a.ready + hflag(nt, j), a.epoch, a.flags, a.spin_limit);
                lds_barrier();  // (not __syncthreads: Linv_{j-1}'s stores stay in flight until the publish)
            }
            cstamp(j, 0);
            if (j == 0) {
                load_src(accd, a, 0, 0);
                acc_to_lds(Z, accd);
                for (int id = tid; id < T * LD; id += NT) Y[id] = 0.0;
                if (tid < kDfSync) Sync[tid] = 0;
                __syncthreads();
            } else {
                d4 accs[4];
                if (j == 1) {
                    load_src(accs, a, 1, 0);
                    load_src(accd, a, 1, 1);
                } else {
                    load_acc<true>(accs, tile(j, j - 1), ld);
                    load_acc<true>(accd, tile(j, j), ld);
                }
                // the loads drained the queue: Linv_{j-1}'s stores have landed
                publish(a, (j - 1) * nt + (j - 1));
                acc_to_lds(X, accs);
                acc_to_lds(Z, accd);
                lds_barrier();
                fstamp(j, 0);
#pragma unroll
                for (int J = 0; J < 4; J++) accs[J] = d4{0.0, 0.0, 0.0, 0.0};
                gemm_nt<true>(X, Y, accs, 1.0);  // L_{j,j-1}
                fstamp(j, 1);
                store_acc_coh(tile(j, j - 1), ld, accs);
                lds_barrier();  // the GEMM's reads of X and Y are done (the stores stay in flight)
                acc_to_lds(X, accs);
#if !M3S_DF_CC
                for (int id = tid; id < T * LD; id += NT) Y[id] = 0.0;  // Linv_{j-1} read: Y -> the new Li
#endif
                // (potrf_cc writes every block of Li it reads -- the diagonal and lower 16x16 blocks --
                // and the Linv store below writes the upper ones as zeros: no zeroing pass on the chain)
                if (tid < kDfSync) Sync[tid] = 0;
                lds_barrier();
                fstamp(j, 2);
                syrk_lower(Z, X);  // A'_jj = P_d(j) - L_{j,j-1} L_{j,j-1}^T (lower blocks)
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // L_{j,j-1}'s stores landed (long ago)
                __syncthreads();
                fstamp(j, 3);
            }
            cstamp(j, 1);
#if M3S_DF_CC
            if (j >= 1 && tid == 0)  // L_{j,j-1}: every wave waited for its stores before the barrier
                __hip_atomic_store(a.ready + j * nt + (j - 1), a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            potrf_cc(Z, Y, X, Scr, Sync, Dinv, a.flags);  // X (L_{j,j-1}) is free: the column buffer
#else
            potrf_inverse(Z, Y, X, Dinv, a.flags, a.trace && j == 0 ? a.trace + 4 * a.ntiles : nullptr,
                          j >= 1 ? a.ready + j * nt + (j - 1) : nullptr, a.epoch);
#endif
            cstamp(j, 2);
            double* Lk = a.Linv + (int64_t)j * T * T;
#pragma unroll
            for (int q = 0; q < 16; q++) {
                const int id = tid + NT * q;
                const int r = id >> 6, cl = id & 63;
                st_coh(Lk + id, (cl >> 4) > (r >> 4) ? 0.0 : Y[r * LD + cl]);  // upper blocks: zeros
            }
        }
        publish(a, (nt - 1) * nt + (nt - 1));
        cstamp(nt - 1, 3);
        leave();
        return;
    }
    for (;; ticket = claim()) {
        if (ticket > ntasks) break;
        const int t = ticket - 1;
        if (t >= a.ntiles) {
            const int jh = nt - 1 - 2 * (t - a.ntiles);
            back_pair(a, jh, jh - 1, X);
            continue;
        }
        int j = 0, rem = t;
        while (rem >= col_tasks(j, nt)) {
            rem -= col_tasks(j, nt);
            j++;
        }
        stamp(a, t, 0);
        const int nreg = j < nt - 1 ? nt - j - 1 : 1;
        if (rem == nreg) {
            // ---- H_{j+2}: partial sums of tiles (h, h-1), (h, h) over k <= j = h-2
            const int h = j + 2;
            d4 accs[4], accd[4];
            load_src(accs, a, h, h - 1);
            load_src(accd, a, h, h);
            for (int k = 0; k <= j; k++) {
                if (tid == 0) {
                    wait_ready(a.ready + h * nt + k, a.epoch, a.flags, a.spin_limit);
                    wait_ready(a.ready + (h - 1) * nt + k, a.epoch, a.flags, a.spin_limit);
                }
                __syncthreads();
                load_tile_coh(X, tile(h, k), ld);
                load_tile_coh(Y, tile(h - 1, k), ld);
                __syncthreads();
                gemm_nt(X, Y, accs, -1.0);
                gemm_nt(X, X, accd, -1.0);
                __syncthreads();
            }
            stamp(a, t, 1);
            store_acc_coh(tile(h, h - 1), ld, accs);
            store_acc_coh(tile(h, h), ld, accd);
            publish(a, hflag(nt, h));
            stamp(a, t, 3);
        } else {
            // ---- regular tile (i, j), left-looking
            const int i = j < nt - 1 ? j + 2 + rem : nt;
            d4 acc[4];
            load_src(acc, a, i, j);
            for (int k = 0; k < j; k++) {
                if (tid == 0) {
                    wait_ready(a.ready + i * nt + k, a.epoch, a.flags, a.spin_limit);
                    wait_ready(a.ready + j * nt + k, a.epoch, a.flags, a.spin_limit);
                }
                __syncthreads();
                load_tile_coh(X, tile(i, k), ld);
                load_tile_coh(Y, tile(j, k), ld);
                __syncthreads();
                gemm_nt(X, Y, acc, -1.0);
                __syncthreads();
            }
            stamp(a, t, 1);
            acc_to_lds(X, acc);
            if (tid == 0) wait_ready(a.ready + j * nt + j, a.epoch, a.flags, a.spin_limit);
            __syncthreads();
            stamp(a, t, 2);
            load_tile_coh(Y, a.Linv + (int64_t)j * T * T, T);
            __syncthreads();
#pragma unroll
            for (int J = 0; J < 4; J++) acc[J] = d4{0.0, 0.0, 0.0, 0.0};
            gemm_nt<true>(X, Y, acc, 1.0);
            store_acc_coh(tile(i, j), ld, acc);
            publish(a, i * nt + j);
            stamp(a, t, 3);
        }
    }
    leave();
}

}  // namespace

// ready words (tiles, H_j, x_j), the ticket and exit counters, then the x granules (16 B per
// entry, 16-B aligned)
// (the two counters on a 128-B line of their own, away from the polled ready words)
static size_t chol_nwords(int npad) {
    const int nt = npad / T;
    return ((size_t)(nt + 1) * (size_t)nt + 2 * (size_t)nt + 31) / 32 * 32;
}
static size_t chol_words_bytes(int npad) { return sizeof(int) * (chol_nwords(npad) + 32); }
size_t chol_ready_bytes(int npad) { return chol_words_bytes(npad) + 16 * (size_t)npad; }

hipError_t launch_chol_dataflow(hipStream_t st, int npad, double* Hd, double* Linv, int* ready,
                                int epoch, int* flags, double* x, const DfScatter* g) {
    // the grid cap that keeps every workgroup resident, per device: computed once per
    // device id, published with an atomic store (concurrent first calls compute the same value)
    constexpr int kMaxDev = 64;
    static std::atomic<int> maxg_dev[kMaxDev];
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= kMaxDev) return hipErrorInvalidDevice;
    int maxg = maxg_dev[dev].load(std::memory_order_acquire);
    if (maxg == 0) {
        int ncu = 0, per = 0;
        e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)chol_df_kernel, NT, 0);
        if (e != hipSuccess) return e;
        maxg = ncu * per;
        if (maxg <= 0) return hipErrorLaunchFailure;
        maxg_dev[dev].store(maxg, std::memory_order_release);
    }
    DfArgs a{};
    a.Hd = Hd;
    a.Linv = Linv;
    a.ready = ready;
    a.flags = flags;
    a.npad = npad;
    a.nt = npad / T;
    a.ntiles = num_tasks(a.nt);
    a.epoch = epoch;
    a.x = x;
    a.xg = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(ready) + chol_words_bytes(npad));
    a.tick = ready + chol_nwords(npad);
    if (g) a.g = *g;
    // M3S_TEST_FORCE_TIMEOUT=1 (tests only): every ready wait gives up at once, to exercise the
    // timeout -> M3S_ERR_TIMEOUT path without a real hang
    const char* ft = getenv("M3S_TEST_FORCE_TIMEOUT");
    a.spin_limit = (ft && atoi(ft) != 0) ? -1 : (1 << 22);
    // M3S_DF_XGRAN (default 1): the back-substitution's x hand-off by granules; 0: ready words
    // (round-5 A/B on cfg4, one box: solve 0.293 vs 0.296 ms per iteration, profiles/r05_d_*)
    static const int xgran = [] {
        const char* e = getenv("M3S_DF_XGRAN");
        return e ? atoi(e) : 1;
    }();
    a.xgran = xgran;
    static const int dyn = [] {
        const char* e = getenv("M3S_DF_DYN");
        return e ? atoi(e) : 1;
    }();
    a.dyn = dyn;
    const int grid = 1 + a.ntiles < maxg ? 1 + a.ntiles : maxg;  // ticket 0 = the diagonal chain
    // A plain launch of a grid the occupancy query admits (one workgroup per CU here: 131 KB of
    // LDS) without the per-launch host cost of a cooperative one and without the ROCm 7.2
    // exit-time fault of a process that made a cooperative launch (profiles/r03_exit_fault).  The
    // dynamic task claim needs no co-residency: should the device not hold the whole grid
    // (another stream's kernels occupying CUs), the late workgroups only claim later tickets; the
    // bounded waits remain a hang guard (M3S_ERR_TIMEOUT).  M3S_CHOL_COOP=1: cooperative.
    static const bool coop = [] {
        const char* e = getenv("M3S_CHOL_COOP");
        return e && atoi(e) != 0;
    }();
    void* kargs[] = {&a};
    if (coop) return hipLaunchCooperativeKernel((const void*)chol_df_kernel, dim3(grid), dim3(NT), kargs, 0, st);
    hipLaunchKernelGGL(chol_df_kernel, dim3(grid), dim3(NT), 0, st, a);
    return hipGetLastError();
}

}  // namespace m3s
