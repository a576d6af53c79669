// gn_solve.hip -- the whole per-iteration solve + retraction in ONE workgroup (gfx950).
//
// Replaces SparseBlock::solve (Eigen SimplicialLLT, reference gn_kernels.cu:132-153), the
// dx = -solve / pose_retr_kernel / ||dx|| test of the GN drivers (gn_kernels.cu:1209-1222,
// 415-453).  A multi-launch design (one launch per elimination round / 64-tile step) is bound
// by launch latency (~5 us per dependent launch); here ONE 256-thread workgroup (4 waves, one
// per SIMD, 512 registers each) runs the block elimination end to end with __syncthreads()
// between dependent steps (~0.1 us each).  Since one CU issues everything, the design keeps
// dependent chains short: the host plan (integers) is staged into LDS once; every 7x7 factor
// is computed serially in registers by each lane that needs it (no cross-lane traffic on the
// pivot chain); global loads are issued unconditionally (invalid entries read an all-zero
// block) so that independent loads overlap instead of waiting one by one.
//
// The system arrives in block format (gn_assemble_kernel): b, then 49-f64 row-major blocks
// (block (x,y) holds the rows of pose x < y; fill blocks zeroed), and is updated in place.
//
//   rounds    per independent set of poses (host plan, gn_driver.hip): 7 lanes per pose (9
//             poses per wave); every lane factors A_vv = L L^T (packed lower, rsq + one Newton
//             step per pivot) and computes row `ra` of W_rv = A_rv L^-T for each front pose r
//             (forward substitution) into LDS (and global, for the back-substitution); lane 0 of
//             the group y_v = L^-1 b_v.  barrier.  Schur updates, one thread per target BLOCK:
//             A_rs -= sum_v W_rv W_sv^T (49 accumulators, host-ordered contribution list:
//             deterministic), b_r -= sum_v W_rv y_v.  barrier.
//   tail      the remaining dense core (<= 27 poses, 189 unknowns) lives in REGISTERS as 16x16
//             f64 tiles of the lower triangle.  The tile map is a compile-time function of the
//             tail's tile count T: tiles are dealt to the 4 waves by their MFMA work (a tile of
//             column J is updated ~(16 J + 9) / 7 times), each wave's slots sorted by J.
//             Factored right-looking one pose (7 columns) at a time, two barriers per pose:
//               A: every thread factors the 7x7 diagonal block in registers (from LDS
//                  broadcasts) and solves y_K = L^-1 z_K; each thread turns one panel row into a
//                  row of L (forward substitution) and updates its RHS entry; 7 threads produce
//                  the columns of L_KK^-1 for the back-substitution | barrier |
//               B: rank-7 update of the live tiles, two v_mfma_f64_16x16x4_f64 each; the one or
//                  two tile columns holding the next pose are written whole (branch-free) into
//                  an LDS strip | barrier.
//             Back-substitution right-looking (x_K = L_KK^-T z_K as a matvec), one barrier
//             per pose, the L entries prefetched three poses ahead.
//   back      the rounds in reverse: x_v = L^-T (y_v - sum_r W_rv^T x_r), 7 lanes per pose;
//             a round of <= 18 poses (the late, dense ones) splits each pose's fronts over
//             36 / nn groups whose partials meet in LDS (one round trip instead of ~6).
//   retract   dx = -x (0 if a pivot failed), Twc <- exp(dx) * Twc, ||dx|| < delta_thresh.
// Failure semantics follow SimplicialLLT: a pivot <= 0 fails (NaN passes) => dx = 0.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "gn_kernels.h"
#include "sim3.h"

// 1: the tail's pose step factors L_KK in every thread and fuses the panel-row solve into it
// (no L_KK^-1 round trip through LDS, one barrier less per pose); 0: wave 0 factors and inverts,
// a barrier, then a matvec per panel row
#ifndef M3S_TAIL_FUSED_A
#define M3S_TAIL_FUSED_A 1
#endif
// Diagnostic builds only (timing; the results are wrong): bit 1 = no L row stores to global in
// the tail's phase A, bit 2 = no rank-7 MFMA update, bit 4 = no next-panel extraction, bit 8 =
// no 7x7 factor / forward substitutions in phase A
#ifndef M3S_TAIL_DIAG
#define M3S_TAIL_DIAG 0
#endif

namespace m3s {

namespace {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = kSolveThreads;
constexpr int kGroups = 9;   // 7-lane groups (one pose each) per wave
constexpr int kPS = 9;       // LDS row stride (doubles) of the panel buffers: conflict-free MFMA reads
constexpr int kLRec = 28;    // tail per-pose record in LDS: packed lower L_KK^-1
constexpr int kMaxTicks = 96;
constexpr int kSchurBatch = 4;  // Schur targets per 7-lane group with their loads in flight together

// dynamic LDS (doubles): a union of the tail buffers and the round staging, then the plan ints
// The extracted panel is a strip of two whole tile columns (J0, J0 + 1: every pose's 7 columns
// lie in them), written branch-free from the accumulators -- the per-lane row / column tests
// of extracting only the 7 columns cost ~1 us per pose step; row stride 33: one pad double.
constexpr int kSS = 33;
constexpr int kOffPn = 0;
constexpr int kOffPop = kOffPn + kTailMax * kSS;
constexpr int kOffZ = kOffPop + kTailMax * kPS;
constexpr int kOffL = kOffZ + kTailMax;
constexpr int kTailDoubles = kOffL + kTailPoseMax * kLRec;
constexpr int kOffX = kTailDoubles;  // x (7 per pose) after the tail buffers: live from the tail on
constexpr int kOffWst = 0;                                   // round: W blocks of the round
constexpr int kOffYst = kOffWst + kSolveWStage;              // round: y of the round's poses
constexpr int kRoundDoubles = kOffYst + 7 * kSolveRoundPoses;
constexpr int kSolvePosesX = 312;  // poses whose x fits after the tail buffers
constexpr int kRegionDoubles =
    kTailDoubles + 7 * kSolvePosesX > kRoundDoubles ? kTailDoubles + 7 * kSolvePosesX : kRoundDoubles;

__host__ __device__ constexpr int pk(int i, int j) { return i * (i + 1) / 2 + j; }  // packed lower

// Workgroup barrier that orders LDS only: it waits for this wave's LDS operations but not for
// its global stores (a __syncthreads() release fence waits for every outstanding global store
// to be acknowledged, ~1 us).  Global data handed between waves of the solve always crosses a
// full __syncthreads() before it is read.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// 1/sqrt(d) to f64 accuracy: v_rsq_f64 + one Newton step (d <= 0 / NaN propagate)
__device__ __forceinline__ double rsqrt_f64(double d) {
    const double y = __builtin_amdgcn_rsq(d);
    return y * fma(-0.5 * d * y, y, 1.5);
}

// Serial 7x7 LL^T in registers: a (packed lower) -> L, inv[i] = 1 / L_ii.
__device__ __forceinline__ void chol7(double (&a)[28], double (&inv)[7], bool& bad) {
#pragma unroll
    for (int p = 0; p < 7; p++) {
        const double d = a[pk(p, p)];
        bad |= (d <= 0.0);  // SimplicialLLT: fails iff a pivot <= 0 (NaN passes)
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

// Li = L^-1 (packed lower) from L and inv = 1/diag
[[maybe_unused]] __device__ __forceinline__ void inv7(const double (&L)[28], const double (&inv)[7], double (&Li)[28]) {
#pragma unroll
    for (int j = 0; j < 7; j++) {
        Li[pk(j, j)] = inv[j];
#pragma unroll
        for (int i = j + 1; i < 7; i++) {
            double s = 0.0;
#pragma unroll
            for (int k = j; k < i; k++) s = fma(L[pk(i, k)], Li[pk(k, j)], s);
            Li[pk(i, j)] = -s * inv[i];
        }
    }
}

}  // namespace

// ---------------------------------------------------------------------------------
// The in-register dense tail, as seen by wave W (compile time): its slots, their tiles
// (I, J) and the operand registers are all compile-time, so the per-step work is the panel
// operand loads, the MFMAs of the live slots and the extraction of the next panel.
// The accumulators hold -A (so both MFMA operands are the plain panel P: -A += P_I P_J^T).
// ---------------------------------------------------------------------------------
struct SlotMap {
    int n;
    int I[64], J[64];
};
// Tiles are dealt to the 4 waves so that their MFMA issue is balanced: a tile of column J is
// updated at every pose step until its column is factored, ~(16 J + 9) / 7 steps; tiles are
// taken longest-lived first and each goes to the wave with the least work so far (fewest
// slots on a tie).  (The former map -- groups of 4 consecutive rows per column, one row per
// wave -- gave wave 0 twice the slot-steps of wave 3.)  A wave's slots are sorted by J, so the
// live slots at a step are a suffix.
__host__ __device__ constexpr int tile_life(int J) { return (16 * J + 9 + 6) / 7; }
__host__ __device__ constexpr SlotMap make_slot_map(int T, int W) {
    int load[4] = {0, 0, 0, 0}, cnt[4] = {0, 0, 0, 0};
    int owner[16][16] = {};
    for (int J = T - 1; J >= 0; J--) {
        for (int I = T - 1; I >= J; I--) {
            int best = 0;
            for (int w = 1; w < 4; w++)
                if (load[w] < load[best] || (load[w] == load[best] && cnt[w] < cnt[best])) best = w;
            owner[I][J] = best;
            load[best] += tile_life(J);
            cnt[best]++;
        }
    }
    SlotMap m{};
    m.n = 0;
    for (int J = 0; J < T; J++)
        for (int I = J; I < T; I++)
            if (owner[I][J] == W) {
                m.I[m.n] = I;
                m.J[m.n] = J;
                m.n++;
            }
    return m;
}

template <int T, int W, typename Tick>
__device__ __forceinline__ void tail_solve(const SolveArgs& a, const int* __restrict__ M, double* __restrict__ smem,
                                           bool& bad, Tick& tick) {
    constexpr SlotMap SM = make_slot_map(T, W);
    constexpr int NS = SM.n;
    double* __restrict__ sPn = smem + kOffPn;    // extracted strip: tile columns J0, J0 + 1
    double* __restrict__ sPop = smem + kOffPop;  // MFMA operand: L panel rows (0 outside live rows)
    double* __restrict__ sZ = smem + kOffZ;      // tail RHS -> y -> (back) partial sums
    double* __restrict__ sL = smem + kOffL;      // per tail pose: packed L_KK^-1
    double* __restrict__ sX = smem + kOffX;      // the solution x (7 per pose), LDS-resident
    double* __restrict__ A = a.A;
    const int tid = threadIdx.x, lane = tid & 63;
    const int zb = a.zero_blk;
    const int nt = a.ntail, n = 7 * nt;
    const int* __restrict__ Mtail = M + a.o_tail;
    const int* __restrict__ Mtmap = M + a.o_tmap;
    d4 acc[NS > 0 ? NS : 1];
    // -A from the dense fill (coalesced: 16 lanes read 16 consecutive doubles of a row), or
    // from the blocks: every load issued unconditionally (entries outside the tail or of
    // absent blocks read the zero block)
    if (a.Hd != nullptr) {
        const double* __restrict__ Hd = a.Hd;
#pragma unroll
        for (int k = 0; k < NS; k++) {
            const int col = 16 * SM.J[k] + (lane & 15);
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const int row = 16 * SM.I[k] + (lane >> 4) + 4 * e;
                acc[k][e] = -((row < n && col < n) ? Hd[(int64_t)row * a.npad_h + col] : 0.0);
            }
        }
    } else {
#pragma unroll
    for (int k = 0; k < NS; k++) {
        const int col = 16 * SM.J[k] + (lane & 15);
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const int row = 16 * SM.I[k] + (lane >> 4) + 4 * e;
            const bool in = row < n && col < n;
            const int code = in ? Mtmap[(row / 7) * nt + col / 7] : -1;
            const int r7 = row % 7, c7 = col % 7;
            const int64_t off = code < 0 ? (int64_t)zb * 49
                                         : (int64_t)(code >> 1) * 49 + ((code & 1) ? c7 * 7 + r7 : r7 * 7 + c7);
            acc[k][e] = -A[off];
        }
    }
    }
    for (int i = tid; i < kTailMax * kPS; i += kThreads) sPop[i] = 0.0;
    for (int i = tid; i < n; i += kThreads) sZ[i] = a.b[(int64_t)Mtail[i / 7] * 7 + i % 7];
    // the strip of pose 0 (tile column 0)
#pragma unroll
    for (int k = 0; k < NS; k++) {
        if (SM.J[k] == 0) {
#pragma unroll
            for (int e = 0; e < 4; e++) sPn[(16 * SM.I[k] + (lane >> 4) + 4 * e) * kSS + (lane & 15)] = -acc[k][e];
        }
    }
    lds_barrier();
    tick(6);
#if M3S_TAIL_FUSED_A
    double yprev[7];  // y of the previous pose, written to sZ by one thread a phase later
#endif
    for (int K = 0; K < nt; K++) {
        const int c0 = 7 * K;
        const int nrows = n - c0 - 7;  // panel rows below the diagonal block
#if M3S_TAIL_FUSED_A
        // A. every thread factors L_KK in registers (redundantly: no barrier, no L_KK^-1 round
        //    trip through LDS) and runs two forward substitutions: y_K = L_KK^-1 z_K and one
        //    input of its role -- panel row i = c0+7+tid (its row of L, RHS update), or, for the
        //    7 threads after them, e_m (column m of L_KK^-1, for the back-substitution)
        double yK[7];
        if (K > 0 && tid == kThreads - 8) {  // the previous pose's y (nobody reads it in this phase)
#pragma unroll
            for (int c = 0; c < 7; c++) sZ[c0 - 7 + c] = yprev[c];
        }
        {
            double L[28], inv[7], z[7], in[7], out[7];
            const bool prow = tid < nrows;
            const int m = tid - nrows;  // diagonal-column role: 0 <= m < 7
            const int i = c0 + 7 + tid;
            const int so = c0 & 15;  // the pose's first column in the strip
#pragma unroll
            for (int r = 0; r < 7; r++) {
#pragma unroll
                for (int j = 0; j <= r; j++) L[pk(r, j)] = sPn[(c0 + r) * kSS + so + j];
                z[r] = sZ[c0 + r];
            }
#pragma unroll
            for (int c = 0; c < 7; c++) in[c] = prow ? sPn[i * kSS + so + c] : (c == m ? 1.0 : 0.0);
            const double zr0 = prow ? sZ[i] : 0.0;
#if M3S_TAIL_DIAG & 8
#pragma unroll
            for (int c = 0; c < 7; c++) {
                yK[c] = z[c] + L[pk(c, c)];
                out[c] = in[c] + L[pk(6, c)];
                inv[c] = 1.0;
            }
#else
            chol7(L, inv, bad);
            fwd7(L, inv, z, yK);
            fwd7(L, inv, in, out);
#endif
            if (prow) {
                double* Lg = a.Lg + (int64_t)i * n + c0;
                double zr = zr0;
#pragma unroll
                for (int c = 0; c < 7; c++) {
                    sPop[i * kPS + c] = out[c];
                    if (!(M3S_TAIL_DIAG & 1)) Lg[c] = out[c];
                    zr = fma(-out[c], yK[c], zr);
                }
                sZ[i] = zr;
            } else if (m < 7) {
#pragma unroll
                for (int c = 0; c < 7; c++)
                    if (c >= m) sL[K * kLRec + pk(c, 0) + m] = out[c];
            }
            if (tid >= kThreads - 7) {  // the pose's own rows leave the MFMA operand
                const int rr = c0 + (tid - (kThreads - 7));
#pragma unroll
                for (int c = 0; c < 8; c++) sPop[rr * kPS + c] = 0.0;
            }
        }
        if (K >= 3 && K < 5) tick(7);
#else
        // A1. wave 0: L_KK (in-lane serial, every lane), L_KK^-1 and y_K = L_KK^-1 z_K
        if (W == 0) {
            double L[28], inv[7], z[7], y[7], Li[28];
#pragma unroll
            for (int i = 0; i < 7; i++) {
#pragma unroll
                for (int j = 0; j <= i; j++) L[pk(i, j)] = sPn[(c0 + i) * kSS + (c0 & 15) + j];
                z[i] = sZ[c0 + i];
            }
            chol7(L, inv, bad);
            inv7(L, inv, Li);
#pragma unroll
            for (int c = 0; c < 7; c++) {
                double s2 = 0.0;
#pragma unroll
                for (int m = 0; m <= c; m++) s2 = fma(Li[pk(c, m)], z[m], s2);
                y[c] = s2;
            }
            // every lane holds the same values: lane 0 stores them (no per-lane select chains
            // on the critical path)
            if (lane == 0) {
#pragma unroll
                for (int k = 0; k < 28; k++) sL[K * kLRec + k] = Li[k];
#pragma unroll
                for (int c = 0; c < 7; c++) sZ[c0 + c] = y[c];
            }
        }
        if (K >= 3 && K < 5) tick(7);
        lds_barrier();
        // A2. panel rows of L: P_i = L_KK^-1 a_i (matvec), RHS update
        {
            const double* Li = sL + K * kLRec;
            const int i = c0 + 7 + tid;
            if (tid < nrows) {
                double in[7], out[7], y[7];
#pragma unroll
                for (int c = 0; c < 7; c++) {
                    in[c] = sPn[i * kSS + (c0 & 15) + c];
                    y[c] = sZ[c0 + c];
                }
                double zr = sZ[i];
                double* Lg = a.Lg + (int64_t)i * n + c0;
#pragma unroll
                for (int c = 0; c < 7; c++) {
                    double s2 = 0.0;
#pragma unroll
                    for (int m = 0; m <= c; m++) s2 = fma(Li[pk(c, m)], in[m], s2);
                    out[c] = s2;
                    sPop[i * kPS + c] = s2;
                    Lg[c] = s2;
                    zr = fma(-s2, y[c], zr);
                }
                sZ[i] = zr;
            }
            if (tid >= kThreads - 7) {  // the pose's own rows leave the MFMA operand
                const int rr = c0 + (tid - (kThreads - 7));
#pragma unroll
                for (int c = 0; c < 8; c++) sPop[rr * kPS + c] = 0.0;
            }
        }
#endif
        if (K >= 3 && K < 5) tick(8);
        lds_barrier();
#if M3S_TAIL_FUSED_A
#pragma unroll
        for (int c = 0; c < 7; c++) yprev[c] = yK[c];  // stored at the next phase A (or after the loop)
#endif
        // B. -C_IJ += P_I P_J^T for the live tiles (J >= Jmin), operands from registers.  The
        //    slots are sorted by J, so the live ones are a suffix [kf, NS): a fall-through
        //    switch enters the unrolled MFMA sequence at kf with no per-slot tests.  Then the
        //    slots of the next pose's columns (J in [J0, J1], a contiguous range) are extracted.
        {
            const int Jmin = (c0 + 7) >> 4;
            double P0[T], P1[T];
            const int kq = lane >> 4;
#pragma unroll
            for (int t = 0; t < T; t++) {
                const int r = (16 * t + (lane & 15)) * kPS + kq;
                P0[t] = sPop[r];
                P1[t] = sPop[r + 4];
            }
            int kf = 0;
#pragma unroll
            for (int k = 0; k < NS; k++) kf += SM.J[k] < Jmin;
#define M3S_MF(k)                                                                                 \
    case k:                                                                                       \
        if constexpr (k < NS && !(M3S_TAIL_DIAG & 2)) {                                           \
            acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(P0[SM.I[k]], P0[SM.J[k]], acc[k], 0, 0, 0); \
            acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(P1[SM.I[k]], P1[SM.J[k]], acc[k], 0, 0, 0); \
        }                                                                                         \
        [[fallthrough]];
            switch (kf) {
                M3S_MF(0) M3S_MF(1) M3S_MF(2) M3S_MF(3) M3S_MF(4) M3S_MF(5) M3S_MF(6) M3S_MF(7)
                M3S_MF(8) M3S_MF(9) M3S_MF(10) M3S_MF(11) M3S_MF(12) M3S_MF(13) M3S_MF(14)
                M3S_MF(15) M3S_MF(16) M3S_MF(17) M3S_MF(18) M3S_MF(19) M3S_MF(20) M3S_MF(21)
                M3S_MF(22) M3S_MF(23) M3S_MF(24) M3S_MF(25) M3S_MF(26) M3S_MF(27) M3S_MF(28)
                M3S_MF(29) M3S_MF(30) M3S_MF(31)
                default: break;
            }
#undef M3S_MF
            static_assert(NS <= 32, "tail slot map exceeds the unrolled MFMA switch");
            if (K + 1 < nt && !(M3S_TAIL_DIAG & 4)) {
                // the next pose's strip: its tile columns J0 and J1 (= J0 or J0 + 1), whole tiles
                const int c1 = c0 + 7;
                const int J0 = c1 >> 4, J1 = (c1 + 6) >> 4;
#pragma unroll
                for (int k = 0; k < NS; k++) {
                    if (SM.J[k] == J0 || SM.J[k] == J1) {
                        const int cl = 16 * (SM.J[k] - J0) + (lane & 15);
#pragma unroll
                        for (int e = 0; e < 4; e++)
                            sPn[(16 * SM.I[k] + (lane >> 4) + 4 * e) * kSS + cl] = -acc[k][e];
                    }
                }
            }
            if (K >= 3 && K < 5) {
                if (NS > 0) asm volatile("s_nop 0" :: "v"(acc[NS - 1][0]));
                tick(9);
            }
        }
        lds_barrier();
        if (K >= 3 && K < 5) tick(11);
        else tick(15);  // a whole pose step
    }
    tick(2);
#if M3S_TAIL_FUSED_A
    if (nt > 0 && tid == kThreads - 8) {
#pragma unroll
        for (int c = 0; c < 7; c++) sZ[7 * (nt - 1) + c] = yprev[c];
    }
#endif

    __syncthreads();  // the L rows (global, written by every wave) are read below
    // back-substitution L^T x = y over the tail, right-looking: x_K = L_KK^-T z_K, then every
    // z_j (j < 7K) drops its L[7K + c][j] x_K[c] terms.  The L entries a thread needs are
    // prefetched three poses ahead (an L2 round trip is longer than one pose step) into three
    // buffers used in rotation by a loop unrolled by 3, so no register copy waits on a load.
    auto load_lp = [&](int K, double (&dst)[7]) {
        const int c0 = 7 * K;
#pragma unroll
        for (int c = 0; c < 7; c++) dst[c] = (K >= 0 && tid < c0) ? a.Lg[(int64_t)(c0 + c) * n + tid] : 0.0;
    };
    auto back_step = [&](int K, double (&lp)[7]) {
        const int c0 = 7 * K;
        double Li[28], z[7], xk[7];
#pragma unroll
        for (int k = 0; k < 28; k++) Li[k] = sL[K * kLRec + k];
#pragma unroll
        for (int k = 0; k < 7; k++) z[k] = sZ[c0 + k];
#pragma unroll
        for (int c = 0; c < 7; c++) {
            double s2 = 0.0;
#pragma unroll
            for (int i = c; i < 7; i++) s2 = fma(Li[pk(i, c)], z[i], s2);
            xk[c] = s2;
        }
        if (W == 0 && lane == 0) {
            const int xo = Mtail[K] * 7;
#pragma unroll
            for (int c = 0; c < 7; c++) sX[xo + c] = xk[c];
        }
        if (tid < c0) {
            double s2 = sZ[tid];
#pragma unroll
            for (int c = 0; c < 7; c++) s2 = fma(-lp[c], xk[c], s2);
            sZ[tid] = s2;
        }
        if (K >= 3) load_lp(K - 3, lp);  // this buffer's next pose
        lds_barrier();
    };
    double lp0[7], lp1[7], lp2[7];
    load_lp(nt - 1, lp0);
    load_lp(nt - 2, lp1);
    load_lp(nt - 3, lp2);
    for (int K = nt - 1; K >= 0; K -= 3) {
        back_step(K, lp0);
        if (K >= 1) back_step(K - 1, lp1);
        if (K >= 2) back_step(K - 2, lp2);
    }
    lds_barrier();  // x of the tail (LDS) is read by the back rounds
    tick(3);
}

// T = tile rows of the in-register tail (0: no in-kernel tail); NT = threads (the tail needs
// exactly kThreads; a rounds-only launch (T = 0) uses more waves to overlap memory latency)
template <int T, int NT>
__global__ __launch_bounds__(NT) void gn_solve_kernel(SolveArgs a) {
    constexpr int NW = NT / 64;
    __shared__ uint64_t sEntry, sEntryCyc;  // M3S_SOLVE_DEBUG: the clocks before the flag's round trip
    if (a.debug && threadIdx.x == 0) {
        sEntry = wall_clock64();
        sEntryCyc = __builtin_amdgcn_s_memtime();  // shader clock: the effective frequency
    }
    if (solve_skipped(a.flags)) return;
    extern __shared__ double smem[];
    __shared__ double sRed[NW];
    __shared__ int sFail;
    __shared__ uint64_t sT[kMaxTicks];
    __shared__ int sTk[kMaxTicks];

    static_assert(T == 0 || NT == kThreads, "the in-register tail is laid out for kThreads");
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
    bool bad = false;  // per thread; OR-ed into sFail before the retraction
    if (tid == 0) sFail = 0;
    // M3S_SOLVE_DEBUG: thread 0 records the wall clock (100 MHz) after each phase and prints
    // the phase times once at the end (printf inside the timed phases would dominate them)
    int nticks = 0;
    if (a.debug && tid == 0) sT[nticks++] = wall_clock64();
    auto tick = [&](int code) {
        if (a.debug && tid == 0 && nticks < kMaxTicks) {
            sTk[nticks] = code;
            sT[nticks++] = wall_clock64();
        }
    };

    // the plan integers, staged in LDS in one coalesced pass (the host only selects this solver
    // when they fit).  M must be a known-LDS pointer: a generic pointer compiles to FLAT loads,
    // and waiting on a FLAT load also waits for every outstanding global store (~1 us each).
    // Batches of 8 loads per thread in flight before their LDS stores (a plain loop waited for
    // each load in turn: ~14 dependent L2 round trips for cfg3's plan).
    int* __restrict__ M = reinterpret_cast<int*>(smem + kRegionDoubles);
    {
        constexpr int kB = 8;
        for (int i0 = 0; i0 < a.nmeta; i0 += kB * NT) {
            int v[kB];
#pragma unroll
            for (int u = 0; u < kB; u++) {
                const int i = i0 + u * NT + tid;
                v[u] = i < a.nmeta ? a.meta[i] : 0;
            }
#pragma unroll
            for (int u = 0; u < kB; u++) {
                const int i = i0 + u * NT + tid;
                if (i < a.nmeta) M[i] = v[u];
            }
        }
    }
    lds_barrier();
    tick(14);
    const int* __restrict__ Mrounds = M + a.o_rounds;
    const int* __restrict__ Mnodes = M + a.o_nodes;
    const int* __restrict__ Mfptr = M + a.o_fptr;
    const int* __restrict__ Mfronts = M + a.o_fronts;
    double* __restrict__ A = a.A;
    double* __restrict__ b = a.b;
    double* __restrict__ W = a.W;
    const int zb = a.zero_blk;

    double* __restrict__ sX = smem + kOffX;  // x: written by the tail and the back rounds
    // 7-lane groups: lane = 7 g + ra (lane 63 idle)
    const int g = lane / 7, ra = lane - 7 * (lane / 7);

    // ------------------------------------------------------------------ rounds
    if (a.do_fwd) {
        double* __restrict__ sW = smem + kOffWst;
        double* __restrict__ sY = smem + kOffYst;
        for (int rd = 0; rd < a.nrounds; rd++) {
            const int* R = Mrounds + 8 * rd;  // node_begin, nnodes, tbeg, nbt, rbeg, nrt, wbeg, wcount
            const int nb = R[0], nn = R[1], wbeg = R[6];
            for (int base = wave * kGroups; base < nn; base += NW * kGroups) {
                const int qi = base + g;
                if (lane < 7 * kGroups && qi < nn) {
                    const int q = nb + qi, v = Mnodes[q];
                    const int f0 = Mfptr[q], f1 = Mfptr[q + 1];
                    // A_vv, b_v and the rows `ra` of the first 4 front blocks, all in flight
                    double L[28], inv[7], bv[7];
                    const double* Av = A + (int64_t)v * 49;
#pragma unroll
                    for (int i = 0; i < 7; i++)
#pragma unroll
                        for (int j = 0; j <= i; j++) L[pk(i, j)] = Av[i * 7 + j];
#pragma unroll
                    for (int m = 0; m < 7; m++) bv[m] = b[(int64_t)v * 7 + m];
                    double rows[4][7];
                    auto load_rows = [&](int fb) {
#pragma unroll
                        for (int u = 0; u < 4; u++) {
                            const int f = fb + u;
                            const int* F = Mfronts + 4 * (f < f1 ? f : 0);
                            const int blk = f < f1 ? F[1] : zb;
                            const int tr = f < f1 ? F[2] : 0;
                            const double* Ab = A + (int64_t)blk * 49;
#pragma unroll
                            for (int m = 0; m < 7; m++) rows[u][m] = tr ? Ab[m * 7 + ra] : Ab[ra * 7 + m];
                        }
                    };
                    load_rows(f0);
                    chol7(L, inv, bad);
                    {
                        double yv[7];
                        fwd7(L, inv, bv, yv);
                        if (ra == 0) {
#pragma unroll
                            for (int m = 0; m < 7; m++) sY[qi * 7 + m] = yv[m];
                        }
                    }
                    // W rows go to LDS only: a global store here would make every later load
                    // wait for it (vmcnt counts loads and stores in order)
                    for (int fb = f0; fb < f1; fb += 4) {
                        double cur[4][7];
#pragma unroll
                        for (int u = 0; u < 4; u++)
#pragma unroll
                            for (int m = 0; m < 7; m++) cur[u][m] = rows[u][m];
                        if (fb + 4 < f1) load_rows(fb + 4);
#pragma unroll
                        for (int u = 0; u < 4; u++) {
                            if (fb + u < f1) {
                                const int wid = Mfronts[4 * (fb + u) + 3];
                                double out[7];
                                fwd7(L, inv, cur[u], out);
                                double* Ws = sW + (wid - wbeg) * 49 + ra * 7;
#pragma unroll
                                for (int m = 0; m < 7; m++) Ws[m] = out[m];
                            }
                        }
                    }
                    double* Ls = a.Lstore + (int64_t)q * kLStoreRec;
#pragma unroll
                    for (int k = 0; k < 35; k++)
                        if (k % 7 == ra) Ls[k] = k < 28 ? L[k] : inv[k - 28];
                }
            }
            if (rd < 2) tick(12);
            lds_barrier();
            // Schur updates, one 7-lane group per target; lane ra owns COLUMN ra of the block
            // (7 accumulators), so each of the group's 7 loads / stores touches 7 consecutive
            // doubles (a lane per block, or per block row, made every load instruction touch
            // ~64 separate cache lines).  A_rs -= sum W_r W_s^T, b_r -= sum W_r y; W, y from
            // LDS.  kSchurBatch targets per group in flight together.  Per entry the
            // contributions are summed in host order, m inner (deterministic).
            {
                const int tbeg = R[2], nbt = R[3], rbeg = R[4], nrt = R[5];
                const int ntask = nbt + nrt;
                constexpr int NG = NW * kGroups;
                const int gid = wave * kGroups + g;
                if (lane < 7 * kGroups) {
                    for (int t0 = gid; t0 < ntask; t0 += NG * kSchurBatch) {
                        double acc[kSchurBatch][7];
                        int64_t off[kSchurBatch];
#pragma unroll
                        for (int u = 0; u < kSchurBatch; u++) {
                            const int t = t0 + u * NG;
                            if (t < nbt) {
                                off[u] = (int64_t)M[a.o_tg + 3 * (tbeg + t)] * 49 + ra;
#pragma unroll
                                for (int i = 0; i < 7; i++) acc[u][i] = A[off[u] + 7 * i];
                            } else if (t < ntask) {
                                off[u] = (int64_t)M[a.o_rtg + 3 * (rbeg + t - nbt)] * 7 + ra;
                                acc[u][0] = b[off[u]];
                            }
                        }
#pragma unroll
                        for (int u = 0; u < kSchurBatch; u++) {
                            const int t = t0 + u * NG;
                            if (t < nbt) {
                                const int* T_ = M + a.o_tg + 3 * (tbeg + t);
                                for (int c = T_[1]; c < T_[2]; c++) {
                                    const int* C = M + a.o_tc + 2 * c;
                                    const double* Wx = sW + (C[0] - wbeg) * 49;
                                    const double* Wy = sW + (C[1] - wbeg) * 49 + ra * 7;
                                    double wy[7];
#pragma unroll
                                    for (int m = 0; m < 7; m++) wy[m] = Wy[m];
#pragma unroll
                                    for (int m = 0; m < 7; m++)
#pragma unroll
                                        for (int i = 0; i < 7; i++) acc[u][i] = fma(-Wx[i * 7 + m], wy[m], acc[u][i]);
                                }
                            } else if (t < ntask) {
                                const int* Rr = M + a.o_rtg + 3 * (rbeg + t - nbt);
                                double s1 = acc[u][0];
                                for (int c = Rr[1]; c < Rr[2]; c++) {
                                    const int* C = M + a.o_rc + 2 * c;
                                    const double* Wr = sW + (C[0] - wbeg) * 49 + ra * 7;
                                    const double* yv = sY + C[1] * 7;  // C[1]: the pose's slot in the round
#pragma unroll
                                    for (int m = 0; m < 7; m++) s1 = fma(-Wr[m], yv[m], s1);
                                }
                                acc[u][0] = s1;
                            }
                        }
#pragma unroll
                        for (int u = 0; u < kSchurBatch; u++) {
                            const int t = t0 + u * NG;
                            if (t < nbt) {
#pragma unroll
                                for (int i = 0; i < 7; i++) A[off[u] + 7 * i] = acc[u][i];
                            } else if (t < ntask) {
                                b[off[u]] = acc[u][0];
                            }
                        }
                    }
                }
                // the round's W blocks and y vectors (LDS) to global for the back-substitution
                const int wcount = R[7];
                for (int i = tid; i < wcount * 49; i += NT) W[(int64_t)wbeg * 49 + i] = sW[i];
                for (int i = tid; i < nn * 7; i += NT)
                    a.y[(int64_t)Mnodes[nb + i / 7] * 7 + i % 7] = sY[i];
            }
            if (rd < 2) tick(13);
            __syncthreads();
            tick(1);
        }
    }

    // ------------------------------------------------------------------ dense tail
    if constexpr (T > 0) {
        if (a.do_tail && a.ntail > 0) {
            switch (wave) {  // compile-time tile maps per wave
                case 0: tail_solve<T, 0>(a, M, smem, bad, tick); break;
                case 1: tail_solve<T, 1>(a, M, smem, bad, tick); break;
                case 2: tail_solve<T, 2>(a, M, smem, bad, tick); break;
                default: tail_solve<T, 3>(a, M, smem, bad, tick); break;
            }
        }
    }

    // ------------------------------------------------------------------ back rounds
    if (a.do_back) {
        constexpr int NG = NW * kGroups;
        const int gid = wave * kGroups + g;
        if (a.x_tail_global && a.ntail > 0) {
            // the core's x from the dense dataflow launch, in the core's order (no scatter launch)
            const int* __restrict__ Mtail = M + a.o_tail;
            for (int i = tid; i < 7 * a.ntail; i += NT) sX[Mtail[i / 7] * 7 + i % 7] = a.xd[i];
            lds_barrier();
        }
        double* __restrict__ sPart = smem + kOffPn;  // tail scratch, free once the tail is done
        static_assert(NG * 7 <= kOffZ - kOffPn, "back-round partials exceed the tail scratch");
        for (int rd = a.nrounds - 1; rd >= 0; rd--) {
            const int* R = Mrounds + 8 * rd;
            const int nb = R[0], nn = R[1];
            if (2 * nn <= NG) {
                // a small round (the late, dense ones: few poses, many fronts each): S groups
                // per pose, split s takes the front batches s, s + S, ...; one LDS exchange,
                // then split 0 sums the partials in split order (deterministic) and solves
                const int S = NG / nn;
                const bool on = lane < 7 * kGroups && gid < nn * S;
                const int qi = on ? gid / S : 0, s = on ? gid - S * (gid / S) : 0;
                const int q = nb + qi;
                double z = 0.0;
                double L[28], inv[7];
                if (on) {
                    if (s == 0) {
                        const double* Ls = a.Lstore + (int64_t)q * kLStoreRec;
#pragma unroll
                        for (int k = 0; k < 28; k++) L[k] = Ls[k];
#pragma unroll
                        for (int k = 0; k < 7; k++) inv[k] = Ls[28 + k];
                        z = a.y[(int64_t)Mnodes[q] * 7 + ra];
                    }
                    const int f0 = Mfptr[q], f1 = Mfptr[q + 1];
                    for (int fb = f0 + 4 * s; fb < f1; fb += 4 * S) {
                        double wv[4][7], xv[4][7];
#pragma unroll
                        for (int u = 0; u < 4; u++) {
                            const int f = fb + u < f1 ? fb + u : fb;
                            const int* F = Mfronts + 4 * f;
                            const double* Wr = W + (int64_t)F[3] * 49 + ra;
                            const double* xr = sX + F[0] * 7;
#pragma unroll
                            for (int i = 0; i < 7; i++) {
                                wv[u][i] = Wr[i * 7];
                                xv[u][i] = xr[i];
                            }
                        }
#pragma unroll
                        for (int u = 0; u < 4; u++)
                            if (fb + u < f1)
#pragma unroll
                                for (int i = 0; i < 7; i++) z = fma(-wv[u][i], xv[u][i], z);
                    }
                    if (s > 0) sPart[gid * 7 + ra] = z;
                }
                lds_barrier();
                if (on && s == 0)
                    for (int k = 1; k < S; k++) z += sPart[(gid + k) * 7 + ra];
                double zz[7];
#pragma unroll
                for (int m = 0; m < 7; m++) zz[m] = __shfl(z, (lane < 63 ? 7 * g : 0) + m, 64);
                if (on && s == 0) {
                    // zz is the same in the group's 7 lanes: one lane stores it (a per-lane pick
                    // of zz[ra] compiled to a scratch round trip)
                    bwd7(L, inv, zz);
                    if (ra == 0) {
                        const int xo = Mnodes[q] * 7;
#pragma unroll
                        for (int c = 0; c < 7; c++) sX[xo + c] = zz[c];
                    }
                }
                lds_barrier();
                continue;
            }
            for (int base = wave * kGroups; base < nn; base += NW * kGroups) {
                const int qi = base + g;
                const bool on = lane < 7 * kGroups && qi < nn;
                const int q = nb + (on ? qi : 0);
                // lane ra: z_ra = y_v[ra] - sum_r (W_rv^T x_r)[ra]
                double z = 0.0;
                double L[28], inv[7];
                if (on) {
                    const double* Ls = a.Lstore + (int64_t)q * kLStoreRec;
#pragma unroll
                    for (int k = 0; k < 28; k++) L[k] = Ls[k];
#pragma unroll
                    for (int k = 0; k < 7; k++) inv[k] = Ls[28 + k];
                    const int v = Mnodes[q];
                    z = a.y[(int64_t)v * 7 + ra];
                    const int f0 = Mfptr[q], f1 = Mfptr[q + 1];
                    for (int fb = f0; fb < f1; fb += 4) {
                        double wv[4][7], xv[4][7];
#pragma unroll
                        for (int u = 0; u < 4; u++) {
                            const int f = fb + u < f1 ? fb + u : fb;
                            const int* F = Mfronts + 4 * f;
                            const double* Wr = W + (int64_t)F[3] * 49 + ra;
                            const double* xr = sX + F[0] * 7;
#pragma unroll
                            for (int i = 0; i < 7; i++) {
                                wv[u][i] = Wr[i * 7];
                                xv[u][i] = xr[i];
                            }
                        }
#pragma unroll
                        for (int u = 0; u < 4; u++)
                            if (fb + u < f1)
#pragma unroll
                                for (int i = 0; i < 7; i++) z = fma(-wv[u][i], xv[u][i], z);
                    }
                }
                double zz[7];
#pragma unroll
                for (int m = 0; m < 7; m++) zz[m] = __shfl(z, (lane < 63 ? 7 * g : 0) + m, 64);
                if (on) {
                    bwd7(L, inv, zz);
                    if (ra == 0) {
                        const int xo = Mnodes[q] * 7;
#pragma unroll
                        for (int c = 0; c < 7; c++) sX[xo + c] = zz[c];
                    }
                }
            }
            lds_barrier();
        }
        tick(4);

        // -------------------------------------------------------------- retract
        if (bad) sFail = 1;  // benign race: every writer stores 1
        __syncthreads();
        const bool fail = sFail != 0 || a.flags[kFlagFail] != 0;
        double nrm = 0.0;
        for (int p = 1 + tid; p < a.N; p += NT) {
            float xi[7];
#pragma unroll
            for (int q = 0; q < 7; q++) {
                const float v = fail ? 0.0f : -(float)sX[(p - 1) * 7 + q];
                xi[q] = v;
                a.dx[(int64_t)(p - 1) * 7 + q] = v;
                nrm += (double)v * (double)v;
            }
            retr_sim3_cm(a.contract, xi, a.Twc + (int64_t)p * 8);
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) nrm += __shfl_xor(nrm, off, 64);
        if (lane == 0) sRed[wave] = nrm;
        __syncthreads();
        if (tid == 0) {
            double s = 0.0;
            for (int w = 0; w < NW; w++) s += sRed[w];
            a.flags[kFlagFail] = 0;
            if ((float)sqrt(s) < a.delta_thresh) a.flags[kFlagDone] = 1;
        }
        for (int i = tid; i < 7 * a.npose; i += NT) a.x[i] = sX[i];
        tick(5);
    } else if (a.do_fwd) {
        // forward-only launch (the tail is factored by the multi-launch dense path): publish
        // a failed pivot for the retraction launch
        if (bad) sFail = 1;
        __syncthreads();
        if (tid == 0 && sFail) a.flags[kFlagFail] = 1;
    }
    if (a.debug) {
        __syncthreads();
        __builtin_amdgcn_s_waitcnt(0);  // the x / dx / Twc stores acknowledged
        if (tid == 0 && a.dbg != nullptr) {
            const uint64_t t_exit = wall_clock64();
            const uint64_t c_exit = __builtin_amdgcn_s_memtime();
            a.dbg[kSolveDbgCycles] = c_exit - sEntryCyc;
            a.dbg[0] = (unsigned long long)nticks;
            a.dbg[1] = sEntry;
            a.dbg[2] = t_exit;
            for (int k = 0; k < nticks; k++) {
                a.dbg[3 + 2 * k] = (unsigned long long)sTk[k];
                a.dbg[4 + 2 * k] = sT[k];
            }
        }
    }
}

void print_solve_debug(const unsigned long long* h) {
    const int n = (int)h[0];
    if (n <= 0 || n > kMaxTicks) return;
    const unsigned long long* T = h + 3;
    auto us = [](unsigned long long x, unsigned long long y) { return (double)(y - x) * 0.01; };
    fprintf(stderr, "gn_solve entry->first tick %8.2f us\n", us(h[1], T[1]));
    for (int k = 1; k < n; k++) {
        const double d = us(T[2 * k - 1], T[2 * k + 1]);
        const char* what = "retract";
        switch ((int)T[2 * k]) {
            case 1: what = " R: schur+barrier"; break;
            case 2: what = "tail factor"; break;
            case 3: what = "tail back"; break;
            case 4: what = "back rounds"; break;
            case 6: what = "tail load"; break;
            case 7: what = " K: A1 chol (w0)"; break;
            case 8: what = " K: A2 rows"; break;
            case 9: what = " K: B mfma+extract"; break;
            case 11: what = " K: barrier B"; break;
            case 12: what = " R: factor (w0)"; break;
            case 13: what = " R: schur (w0)"; break;
            case 14: what = "plan to LDS"; break;
            case 15: what = " K: pose step"; break;
            default: break;
        }
        fprintf(stderr, "gn_solve %-20s %8.2f us\n", what, d);
    }
    fprintf(stderr, "gn_solve last tick->exit %8.2f us\n", us(T[2 * n - 1], h[2]));
    fprintf(stderr, "gn_solve entry->exit %8.2f us\n", us(h[1], h[2]));
    fprintf(stderr, "gn_solve shader clock %8.0f MHz over the launch\n",
                (double)h[kSolveDbgCycles] / us(h[1], h[2]));
}

int solve_max_poses() { return (kRegionDoubles - kOffX) / 7; }

size_t solve_lds_bytes(int nmeta_lds) {
    return sizeof(double) * kRegionDoubles + sizeof(int) * (size_t)nmeta_lds;
}

hipError_t launch_gn_solve(hipStream_t st, const SolveArgs& args) {
    int T = 0;
    if (args.do_tail && args.ntail > 0) {
        T = (7 * args.ntail + 15) / 16;
        T += T & 1;  // instantiated for even T (a padding tile row is harmless)
    }
    const size_t lds = solve_lds_bytes(args.meta_lds ? args.nmeta : 0);
#define M3S_SOLVE(TT, NTT)                                                                    \
    do {                                                                                      \
        static bool attr = false;                                                             \
        if (!attr) {                                                                          \
            hipError_t e = hipFuncSetAttribute((const void*)gn_solve_kernel<TT, NTT>,         \
                                               hipFuncAttributeMaxDynamicSharedMemorySize,    \
                                               (int)kSolveMaxLds);                            \
            if (e != hipSuccess) return e;                                                    \
            attr = true;                                                                      \
        }                                                                                     \
        hipLaunchKernelGGL((gn_solve_kernel<TT, NTT>), dim3(1), dim3(NTT), lds, st, args);    \
    } while (0)
    if (T == 0 && args.do_fwd && !args.do_back) {
        M3S_SOLVE(0, kSolveRoundThreads);  // rounds only: more waves in flight
        return hipGetLastError();
    }
    switch (T) {
        case 0: M3S_SOLVE(0, kThreads); break;
        case 2: M3S_SOLVE(2, kThreads); break;
        case 4: M3S_SOLVE(4, kThreads); break;
        case 6: M3S_SOLVE(6, kThreads); break;
        case 8: M3S_SOLVE(8, kThreads); break;
        case 10: M3S_SOLVE(10, kThreads); break;
        case 12: M3S_SOLVE(12, kThreads); break;
        default: return hipErrorInvalidValue;
    }
#undef M3S_SOLVE
    return hipGetLastError();
}

}  // namespace m3s
