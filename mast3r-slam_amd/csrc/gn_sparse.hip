// gn_sparse.hip -- the multi-launch block-sparse solve of the pose-graph normal equations.
//
// The GN system is a graph Laplacian with 7x7 blocks, in the block format of
// gn_assemble_kernel: b (npose x 7), then one 49-f64 row-major block per pose and per
// co-observing pose pair (block (x, y), x < y, holds the rows of pose x; fill blocks zeroed).
// The driver (gn_driver.hip, build_sparse_plan) picks, round by round, an independent set V of
// low-degree poses.  A round eliminates all of V in ONE launch, one workgroup per target:
//   block target (r, s):  A_rs -= sum_{v in V} W_rv W_sv^T
//   RHS target r:         b_r  -= sum_{v in V} W_rv y_v
// with L_v L_v^T = A_vv, W_rv = A_rv L_v^-T, y_v = L_v^-1 b_v.  A workgroup recomputes the W
// rows it needs (a 7-lane group per contribution factors A_vv in registers; lane ra
// forward-substitutes row ra of A_rv) rather than reading them from a preceding factor launch:
// a dependent launch costs more than the redundant 7x7 factors.  The RHS target r is the only
// writer of W_rv, and the contribution through v's first front stores L_v and y_v: both are
// kept for the back-substitution.
// The poses left after the rounds are factored either by the in-register core of gn_solve.hip
// (<= 27 poses; that launch also runs the back-substitution through the rounds and the
// retraction) or by the tiled dense Cholesky of gn_kernels.hip (sp_tail_*), after which
// sp_back runs the rounds in reverse: x_v = L_v^-T (y_v - sum_r W_rv^T x_r).
// Each kernel issues its independent loads before it waits (the device flag with the plan
// integers, then the blocks): a dependent global round trip is the unit of cost here.
// Failure semantics follow SimplicialLLT (reference gn_kernels.cu:142-150): a pivot <= 0 sets
// the failure flag and the update becomes zero.
#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "block7.h"
#include "gn_kernels.h"

namespace m3s {

namespace {
constexpr int kGroups = 9;  // 7-lane groups per 64-lane workgroup (lane 63 idle)
constexpr int kLd = 8;      // LDS row stride (doubles) of a staged 7x7 block
static_assert(kSpInline == kGroups, "a target record inlines one contribution per 7-lane group");
}  // namespace

// Round targets: records (kSpRec, gn_kernels.h) {block, begin, end} with contributions
// (v, code_r, code_s) for block targets, {pose r | -1, begin, end} with (v, code_r, W id | -1,
// owner node | -1) for RHS targets; code = block * 2 + transposed (the block holds the rows of
// the other pose).  r = -1 collects the poses without fronts: only their L and y are stored.
// The first kSpInline contributions ride in the record, the rest come from tc3 / rc4.
// COH: the all-rounds launch reads, in round r + 1, blocks other workgroups (other XCDs) wrote
// in round r.  The per-XCD L2s are not coherent, so those A / b accesses are agent-coherent
// (relaxed agent-scope atomics: sc1 loads and write-through stores) and the grid barrier needs
// no L2 write-back or invalidation.
template <bool COH>
__device__ __forceinline__ double ldA(const double* p) {
    if constexpr (COH) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return *p;
}
template <bool COH>
__device__ __forceinline__ void stA(double* p, double v) {
    if constexpr (COH) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}

template <bool COH>
__device__ __forceinline__ void sp_round_target(
    const int* __restrict__ rec, bool blk, const int* __restrict__ tc3, const int* __restrict__ rc4,
    const int* skipf /* the call's flags (solve_skipped), or null */, double* __restrict__ A, double* __restrict__ b,
    double* __restrict__ Lstore, double* __restrict__ W, double* __restrict__ y, int* __restrict__ flags,
    double (*sR)[7 * kLd], double (*sS)[7 * kLd]) {
    const int lane = threadIdx.x;
    const int g = lane / 7, ra = lane - 7 * g;
    // the record header, this group's inline contribution and (per launch) the flag: one round trip
    const int4 hd = *reinterpret_cast<const int4*>(rec);
    const int4 mine = *reinterpret_cast<const int4*>(rec + 4 + 4 * (g < kSpInline ? g : 0));
    if (skipf && solve_skipped(skipf)) return;
    const int tgt = hd.x, c0 = hd.y, c1 = hd.z;
    // this lane's output: entry (er, ec) of the block, or row er of the RHS
    const int nact = tgt < 0 ? 0 : (blk ? 49 : 7);
    const int er = blk ? lane / 7 : lane, ec = lane % 7;
    double* dst = blk ? A + (int64_t)tgt * 49 + lane : b + (int64_t)tgt * 7 + lane;
    const double d0 = lane < nact ? ldA<COH>(dst) : 0.0;
    double acc = 0.0;
    bool bad = false;
    for (int base = c0; base < c1; base += kGroups) {
        const int c = base + g;
        if (g < kGroups && c < c1) {
            int4 C = mine;  // contributions past the inline ones: from the lists
            if (base != c0) {
                if (blk) C = make_int4(tc3[3 * c], tc3[3 * c + 1], tc3[3 * c + 2], 0);
                else C = *reinterpret_cast<const int4*>(rc4 + 4 * c);
            }
            const int v = C.x, cr = C.y, cs = blk ? C.z : 0, wid = blk ? -1 : C.z, owner = blk ? -1 : C.w;
            double L[28], inv[7], rr[7], rs[7];
            const double* Av = A + (int64_t)v * 49;
#pragma unroll
            for (int i = 0; i < 7; i++)
#pragma unroll
                for (int j = 0; j <= i; j++) L[b7::pk(i, j)] = ldA<COH>(Av + i * 7 + j);
            const double* Ar = A + (int64_t)(cr >> 1) * 49;
#pragma unroll
            for (int m = 0; m < 7; m++) rr[m] = ldA<COH>(Ar + ((cr & 1) ? m * 7 + ra : ra * 7 + m));
            if (blk) {
                const double* As = A + (int64_t)(cs >> 1) * 49;
#pragma unroll
                for (int m = 0; m < 7; m++) rs[m] = ldA<COH>(As + ((cs & 1) ? m * 7 + ra : ra * 7 + m));
            } else {
#pragma unroll
                for (int m = 0; m < 7; m++) rs[m] = ldA<COH>(b + (int64_t)v * 7 + m);
            }
            b7::chol7(L, inv, bad);
            double wr[7], ws[7];
            b7::fwd7(L, inv, rr, wr);  // row ra of W_rv
            b7::fwd7(L, inv, rs, ws);  // block: row ra of W_sv; RHS: y_v (the same in every lane)
#pragma unroll
            for (int m = 0; m < 7; m++) sR[g][ra * kLd + m] = wr[m];
            if (blk) {
#pragma unroll
                for (int m = 0; m < 7; m++) sS[g][ra * kLd + m] = ws[m];
            } else {
                if (ra == 0) {
#pragma unroll
                    for (int m = 0; m < 7; m++) sS[g][m] = ws[m];
                }
                if (wid >= 0) {
                    double* Wd = W + (int64_t)wid * 49 + ra * 7;
#pragma unroll
                    for (int m = 0; m < 7; m++) Wd[m] = wr[m];
                }
                if (owner >= 0 && ra == 0) {
                    // L, inv and y_v are the same in the group's 7 lanes: one lane stores them
                    // (a per-lane pick by a runtime index compiled to a scratch round trip)
                    double* Ls = Lstore + (int64_t)owner * kLStoreRec;
#pragma unroll
                    for (int m = 0; m < 7; m++) y[(int64_t)v * 7 + m] = ws[m];
#pragma unroll
                    for (int k = 0; k < 28; k++) Ls[k] = L[k];
#pragma unroll
                    for (int k = 0; k < 7; k++) Ls[28 + k] = inv[k];
                }
            }
        }
        __syncthreads();
        const int n = min(kGroups, c1 - base);
        if (lane < nact) {
            for (int k = 0; k < n; k++) {
                const double* R = &sR[k][er * kLd];
                const double* S = blk ? &sS[k][ec * kLd] : &sS[k][0];
#pragma unroll
                for (int m = 0; m < 7; m++) acc = fma(R[m], S[m], acc);
            }
        }
        __syncthreads();
    }
    if (lane < nact) stA<COH>(dst, d0 - acc);
    if (bad) flags[kFlagFail] = 1;  // benign race: every writer stores 1
}

// One round per launch: workgroup = target (the flag is loaded beside the target record).
__global__ __launch_bounds__(64) void sp_round_kernel(
    const int* __restrict__ inl, int ibeg, int nbt, const int* __restrict__ tc3,
    const int* __restrict__ rc4, double* __restrict__ A, double* __restrict__ b,
    double* __restrict__ Lstore, double* __restrict__ W, double* __restrict__ y,
    int* __restrict__ flags) {
    __shared__ double sR[kGroups][7 * kLd];  // rows of W_rv, per contribution of the batch
    __shared__ double sS[kGroups][7 * kLd];  // block target: rows of W_sv; RHS target: y_v
    sp_round_target<false>(inl + (int64_t)(ibeg + blockIdx.x) * kSpRec, (int)blockIdx.x < nbt, tc3, rc4,
                           flags, A, b, Lstore, W, y, flags, sR, sS);
}

// x_v = L_v^-T (y_v - sum_r W_rv^T x_r), one workgroup per pose of the round; 7-lane group g
// takes the fronts f0 + g, f0 + g + 9, ...; the group partials are summed in fixed order.
__global__ __launch_bounds__(64) void sp_back_kernel(
    const int* __restrict__ nodes, const int* __restrict__ fptr, const int* __restrict__ fronts,
    int node_begin, const double* __restrict__ Lstore, const double* __restrict__ W,
    const double* __restrict__ y, double* __restrict__ x, const int* __restrict__ flags) {
    __shared__ double part[kGroups][kLd];
    const int done = solve_skipped(flags);
    const int q = node_begin + blockIdx.x, lane = threadIdx.x;
    const int v = nodes[q], f0 = fptr[q], f1 = fptr[q + 1];
    if (done) return;
    const int g = lane / 7, ra = lane - 7 * g;
    double L[28], inv[7], z[7];
    const double* Ls = Lstore + (int64_t)q * kLStoreRec;
#pragma unroll
    for (int k = 0; k < 28; k++) L[k] = Ls[k];
#pragma unroll
    for (int k = 0; k < 7; k++) {
        inv[k] = Ls[28 + k];
        z[k] = y[(int64_t)v * 7 + k];
    }
    if (g < kGroups) {
        double s = 0.0;
        for (int f = f0 + g; f < f1; f += kGroups) {
            const int* F = fronts + 4 * f;
            const double* Wr = W + (int64_t)F[3] * 49 + ra;
            const double* xr = x + (int64_t)F[0] * 7;
#pragma unroll
            for (int i = 0; i < 7; i++) s = fma(Wr[i * 7], xr[i], s);
        }
        part[g][ra] = s;
    }
    __syncthreads();
    if (lane == 0) {
#pragma unroll
        for (int m = 0; m < 7; m++) {
            double a = 0.0;
#pragma unroll
            for (int k = 0; k < kGroups; k++) a += part[k][m];
            z[m] -= a;
        }
        b7::bwd7(L, inv, z);
#pragma unroll
        for (int m = 0; m < 7; m++) x[(int64_t)v * 7 + m] = z[m];
    }
}

// Dense core: Hd [npad + 64, npad] from the blocks of the ntail remaining poses (tmap:
// ntail x ntail -> 2*block + transposed, or -1), RHS border row from b.
// (entries first, first + step, ... below end; end < 0: the whole matrix)
template <bool COH>
__device__ __forceinline__ void sp_tail_fill(const double* __restrict__ A, const double* __restrict__ b,
                                             const int* __restrict__ tmap, const int* __restrict__ tail,
                                             int ntail, int npad, double* __restrict__ Hd,
                                             int64_t first = -1, int64_t step = 0, int64_t end = -1) {
    const int n = ntail * 7;
    const int64_t whole = (int64_t)(npad + kCholTile) * npad;
    const int64_t total = end < 0 ? whole : (end < whole ? end : whole);
    if (first < 0) {
        first = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        step = (int64_t)gridDim.x * blockDim.x;
    }
    for (int64_t id = first; id < total; id += step) {
        const int r = (int)(id / npad), c = (int)(id % npad);
        double val;
        if (r > npad) {
            val = 0.0;
        } else if (r == npad) {
            val = c < n ? ldA<COH>(b + (int64_t)tail[c / 7] * 7 + c % 7) : 0.0;
        } else if (r < n && c < n) {
            const int code = tmap[(r / 7) * ntail + c / 7];
            if (code < 0) {
                val = 0.0;
            } else {
                const double* Ab = A + (int64_t)(code >> 1) * 49;
                val = ldA<COH>(Ab + ((code & 1) ? (c % 7) * 7 + r % 7 : (r % 7) * 7 + c % 7));
            }
        } else {
            val = (r == c) ? 1.0 : 0.0;
        }
        Hd[id] = val;
    }
}

__global__ __launch_bounds__(256) void sp_tail_fill_kernel(const double* __restrict__ A,
                                                           const double* __restrict__ b,
                                                           const int* __restrict__ tmap,
                                                           const int* __restrict__ tail,
                                                           int ntail, int npad,
                                                           double* __restrict__ Hd,
                                                           const int* __restrict__ flags) {
    if (solve_skipped(flags)) return;
    sp_tail_fill<false>(A, b, tmap, tail, ntail, npad, Hd);
}

// All elimination rounds (and the hybrid's core fill) in ONE cooperative launch: a round costs
// ~4 us of dependent work per workgroup (target record ~1, block loads ~1.4, 7x7 factor + W rows
// ~1, Schur sums + store ~0.4, measured in-kernel) but ~9 us as its own launch, the rest being
// the dependent launch's dispatch and drain.  Here a grid-wide barrier (cooperative groups,
// co-residency guaranteed by hipLaunchCooperativeKernel) separates the rounds; workgroup w takes
// the round's targets w, w + G, ...  The flag is read once: it was written by the previous
// iteration's kernels, so every workgroup sees the same value and all leave or none.
// Grid-wide barrier over the launch's workgroups (all resident: <= one 64-thread workgroup per
// CU): arrival counter + generation word in the flags area.  Release = the arrival atomic
// (writes back this XCD's L2), acquire = a fence after the generation moved (invalidates L1/L2),
// so blocks written in one round are read fresh in the next on any XCD.  The spin is bounded
// (~0.1 s): a workgroup that never arrives fails the solve and raises the sticky timeout flag
// (reported by the driver as M3S_ERR_TIMEOUT) instead of hanging the GPU; the caller then
// leaves the launch (the arrival counter is no longer consistent).
template <bool FENCED>
__device__ __forceinline__ void grid_barrier(int* __restrict__ flags, unsigned nwg) {
    if constexpr (!FENCED) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // my write-through stores landed
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned* cnt = reinterpret_cast<unsigned*>(flags + kFlagBarCount);
        unsigned* gen = reinterpret_cast<unsigned*>(flags + kFlagBarGen);
        const unsigned g = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned old = FENCED ? __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT)
                                    : __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == nwg - 1) {
            __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            int spins = 0;
            while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1 << 22)) {
                    __hip_atomic_store(flags + kFlagTimeout, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(flags + kFlagFail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
        }
        if constexpr (FENCED) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
}

__global__ __launch_bounds__(64) void sp_rounds_coop_kernel(SpCoopArgs a) {
    __shared__ double sR[kGroups][7 * kLd];
    __shared__ double sS[kGroups][7 * kLd];
    if (solve_skipped(a.flags)) return;
    for (int rd = 0; rd < a.nrounds; rd++) {
        const int* R = a.rounds + 8 * rd;  // node_begin, nnodes, tbeg, nbt, rbeg, nrt, wbeg, wcount
        const int tbeg = R[2], nbt = R[3], rbeg = R[4], nrt = R[5];
        for (int t = blockIdx.x; t < nbt + nrt; t += gridDim.x)
            sp_round_target<true>(a.inl + (int64_t)(tbeg + rbeg + t) * kSpRec, t < nbt, a.tc3, a.rc4, nullptr,
                                  a.A, a.b, a.Lstore, a.W, a.y, a.flags, sR, sS);
        if (a.coop) {
            cooperative_groups::this_grid().sync();
        } else {
            grid_barrier<false>(a.flags, gridDim.x);
            // a timed-out barrier leaves the arrival counter inconsistent: abandon the launch
            // (every workgroup reaches this test after its own barrier wait)
            if (__hip_atomic_load(a.flags + kFlagTimeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
        }
    }
    if (a.ntail > 0 && a.Hd) sp_tail_fill<true>(a.A, a.b, a.tmap, a.tail, a.ntail, a.npad, a.Hd);
}

// The rounds without a grid barrier or co-residency (launch_sp_rounds_df, gn_kernels.h): the
// (round, target) pairs are tickets in round order, then the core fill in chunks of kDfFill
// entries; a workgroup claims the next ticket, waits (one lane, bounded) for the previous round's
// done count (the fill: the last round's), runs it with the coherent block accesses of the
// all-rounds launch and bumps its round's count after its stores landed.  Every wait is on tickets
// that running workgroups hold, so any resident subset progresses; a workgroup's target does not
// change the arithmetic (bitwise the per-round launches).
constexpr int kDfFill = 4096;
__global__ __launch_bounds__(64) void sp_rounds_df_kernel(SpCoopArgs a, int* __restrict__ cnt) {
    __shared__ double sR[kGroups][7 * kLd];
    __shared__ double sS[kGroups][7 * kLd];
    __shared__ int s_tk;
    __shared__ int s_bad;
    if (solve_skipped(a.flags)) return;  // (read once: written by earlier launches; all leave or none)
    const int tid = threadIdx.x;
    int total = 0;
    for (int rd = 0; rd < a.nrounds; rd++) total += a.rounds[8 * rd + 3] + a.rounds[8 * rd + 5];
    const int nround_tk = total;
    const bool fill = a.ntail > 0 && a.Hd;
    const int64_t fill_n = fill ? (int64_t)(a.npad + kCholTile) * a.npad : 0;
    total += (int)((fill_n + kDfFill - 1) / kDfFill);
    int* done = cnt + 4;
    if (tid == 0) s_bad = 0;
    for (;;) {
        __syncthreads();  // (s_tk's previous readers)
        if (tid == 0) s_tk = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        const int tk = s_tk;
        if (tk >= total) break;
        // the ticket's round (rounds are few: a scan)
        int rd = 0, base = 0, need_rd = -1, need = 0;
        if (tk < nround_tk) {
            while (tk >= base + a.rounds[8 * rd + 3] + a.rounds[8 * rd + 5]) {
                base += a.rounds[8 * rd + 3] + a.rounds[8 * rd + 5];
                rd++;
            }
            if (rd > 0) {
                need_rd = rd - 1;
                need = a.rounds[8 * need_rd + 3] + a.rounds[8 * need_rd + 5];
            }
        } else if (a.nrounds > 0) {
            need_rd = a.nrounds - 1;
            need = a.rounds[8 * need_rd + 3] + a.rounds[8 * need_rd + 5];
        }
        if (need_rd >= 0 && tid == 0) {
            int spins = 0;
            while (__hip_atomic_load(done + need_rd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1 << 22)) {
                    __hip_atomic_store(a.flags + kFlagTimeout, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(a.flags + kFlagFail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    s_bad = 1;
                    break;
                }
            }
        }
        __syncthreads();
        if (s_bad) continue;  // (a timed-out wait: drain the remaining tickets without work)
        if (tk < nround_tk) {
            const int* R = a.rounds + 8 * rd;  // node_begin, nnodes, tbeg, nbt, rbeg, nrt, wbeg, wcount
            const int t = tk - base;
            sp_round_target<true>(a.inl + (int64_t)(R[2] + R[4] + t) * kSpRec, t < R[3], a.tc3, a.rc4, nullptr,
                                  a.A, a.b, a.Lstore, a.W, a.y, a.flags, sR, sS);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this target's write-through stores landed
            __syncthreads();
            if (tid == 0) __hip_atomic_fetch_add(done + rd, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            const int64_t f0 = (int64_t)(tk - nround_tk) * kDfFill;
            sp_tail_fill<true>(a.A, a.b, a.tmap, a.tail, a.ntail, a.npad, a.Hd, f0 + tid, 64, f0 + kDfFill);
        }
    }
    // the last workgroup out re-zeroes the counters for the next launch
    if (tid == 0) {
        const int old = __hip_atomic_fetch_add(cnt + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == (int)gridDim.x - 1) {
            for (int k = 0; k < a.nrounds; k++) __hip_atomic_store(done + k, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(cnt + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

__global__ __launch_bounds__(256) void sp_tail_scatter_kernel(const double* __restrict__ xd,
                                                              const int* __restrict__ tail,
                                                              int ntail, double* __restrict__ x,
                                                              const int* __restrict__ flags) {
    if (solve_skipped(flags)) return;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < ntail * 7) x[(int64_t)tail[i / 7] * 7 + i % 7] = xd[i];
}

// ------------------------------------------------------------------ launchers

hipError_t launch_sp_round(hipStream_t st, const int* inl, int ibeg, int nbt, int nrt, const int* tc3,
                           const int* rc4, double* A, double* b, double* Lstore, double* W, double* y,
                           int* flags) {
    if (nbt + nrt <= 0) return hipSuccess;
    hipLaunchKernelGGL(sp_round_kernel, dim3(nbt + nrt), dim3(64), 0, st, inl, ibeg, nbt, tc3, rc4, A, b,
                       Lstore, W, y, flags);
    return hipGetLastError();
}

hipError_t launch_sp_rounds_coop(hipStream_t st, const SpCoopArgs& args) {
    if (args.nrounds <= 0 && (args.ntail <= 0 || !args.Hd)) return hipSuccess;
    static int grid = 0;
    if (grid == 0) {
        int dev = 0, ncu = 0, per = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        if (e == hipSuccess)
            e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)sp_rounds_coop_kernel, 64, 0);
        if (e != hipSuccess) return e;
        grid = std::max(1, std::min(ncu * std::max(per, 1), 256));  // <= one workgroup per CU
    }
    // both barrier flavours need every workgroup resident at once: always a cooperative launch
    // (it refuses a grid the device cannot hold); `coop` only picks the barrier implementation
    SpCoopArgs a = args;
    void* kargs[] = {&a};
    return hipLaunchCooperativeKernel((const void*)sp_rounds_coop_kernel, dim3(grid), dim3(64), kargs, 0, st);
}

hipError_t launch_sp_rounds_df(hipStream_t st, const SpCoopArgs& args, int* cnt) {
    if (args.nrounds <= 0 && (args.ntail <= 0 || !args.Hd)) return hipSuccess;
    // one 64-thread workgroup per CU at most (M3S_SOLVE_DF_WG): the widest round has ~500 targets
    static int grid = 0;
    if (grid == 0) {
        int dev = 0, ncu = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) return e;
        const char* s = getenv("M3S_SOLVE_DF_WG");
        grid = std::max(1, s ? atoi(s) : ncu);
    }
    hipLaunchKernelGGL(sp_rounds_df_kernel, dim3(grid), dim3(64), 0, st, args, cnt);
    return hipGetLastError();
}

hipError_t launch_sp_back(hipStream_t st, int nnodes, const int* nodes, const int* fptr,
                          const int* fronts, int node_begin, const double* Lstore, const double* W,
                          const double* y, double* x, const int* flags) {
    if (nnodes <= 0) return hipSuccess;
    hipLaunchKernelGGL(sp_back_kernel, dim3(nnodes), dim3(64), 0, st, nodes, fptr, fronts,
                       node_begin, Lstore, W, y, x, flags);
    return hipGetLastError();
}

hipError_t launch_sp_tail_fill(hipStream_t st, const double* A, const double* b, const int* tmap,
                               const int* tail, int ntail, int npad, double* Hd, const int* flags) {
    if (ntail <= 0) return hipSuccess;
    const int64_t total = (int64_t)(npad + kCholTile) * npad;
    const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    hipLaunchKernelGGL(sp_tail_fill_kernel, dim3(blocks), dim3(256), 0, st, A, b, tmap, tail, ntail,
                       npad, Hd, flags);
    return hipGetLastError();
}

hipError_t launch_sp_tail_scatter(hipStream_t st, const double* xd, const int* tail, int ntail, double* x,
                                  const int* flags) {
    if (ntail <= 0) return hipSuccess;
    hipLaunchKernelGGL(sp_tail_scatter_kernel, dim3((ntail * 7 + 255) / 256), dim3(256), 0, st, xd,
                       tail, ntail, x, flags);
    return hipGetLastError();
}

// The dense core: filled, then factorised and solved by the dataflow launch, whose
// back-substitution also writes x pose-indexed (no scatter launch: ~5 us for almost no work).
// (Gathering the tiles from the blocks inside the dataflow launch instead of the fill launch was
// measured slower: 0.177 vs 0.156 ms per cfg3 solve, r04_u.)
hipError_t launch_sp_tail(hipStream_t st, const double* A, const double* b, const int* tmap,
                          const int* tail, int ntail, int npad, double* Hd, double* Linv,
                          double* xd, double* x, int* flags, int epoch, bool fill) {
    if (ntail <= 0) return hipSuccess;
    hipError_t e = fill ? launch_sp_tail_fill(st, A, b, tmap, tail, ntail, npad, Hd, flags) : hipSuccess;
    if (e != hipSuccess) return e;
    const DfScatter g{tail, ntail, x};
    return launch_dense_factor_solve(st, npad, Hd, Linv, xd, flags, epoch, &g);
}

}  // namespace m3s
