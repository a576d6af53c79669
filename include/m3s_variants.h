/*
 * m3s_variants.h -- measurement-only refine_matches kernels (lib/libm3s_variants.so).
 *
 * NOT part of the drop-in boundary (m3s_backend.h).  Each variant is bit-exact with the
 * reference's refine_matches (matching_kernels.cu:25-81) -- the same winner for every pixel --
 * and was measured slower than the product kernel on the bench data; they
 * are kept so that bench.py and the tests can A/B them.  Pointers and stream as in m3s_backend.h.
 */
#ifndef M3S_VARIANTS_H
#define M3S_VARIANTS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    M3S_REFINE_VARIANT_LDS = 1,  /* candidate box of a 32x16 pixel tile staged in LDS */
    M3S_REFINE_VARIANT_MFMA = 2, /* approximate scores on v_mfma_f32_16x16x32_f16 + exact re-score */
    M3S_REFINE_VARIANT_DOT2 = 3, /* approximate scores with v_dot2 + exact re-score */
    M3S_REFINE_VARIANT_LATTICE = 4, /* MFMA over per-level lattice buckets of the tile + exact re-score
                                      (dilation_max <= 5) */
    M3S_REFINE_VARIANT_BOX = 5,    /* a 16x16 tile's candidate box staged per level as plane-major
                                      8-B pieces in LDS (round 5) */
    M3S_REFINE_VARIANT_PLANES = 6  /* the product kernel's gathers from a plane-major copy of D11
                                      (3 planes of 16-B pieces, one copy pass per call) */
};

/* refine_matches (fp16, F = 24, radius 3, N = H*W) with one of the variants; returns M3S_OK or an
 * error code (message: m3s_variants_last_error()). */
int m3s_refine_variant_f16(int variant, const uint16_t* D11, const uint16_t* D21, const int64_t* p1,
                           int64_t* p1_new, int64_t B, int64_t H, int64_t W, int64_t N, int64_t F,
                           int radius, int dilation_max, void* stream);
/* Counters of the bound-and-rescore variants (MFMA, DOT2, LATTICE) since the last call: out3[0] =
 * exactly re-scored candidates, out3[1] = in-image candidates, out3[2] = 16x16x32 MFMAs issued by
 * the lattice kernel; enable != 0 turns counting on. */
void m3s_refine_variant_stats(int enable, unsigned long long* out3);
const char* m3s_variants_last_error(void);
/* Test hook (not a refine variant): launch `nblocks` 64-thread workgroups on `stream`, each
 * holding `lds_bytes` of LDS (256 .. 160 KiB) for `usec` microseconds (<= 2 s, bounded by the
 * real-time counter), so that a test can take CUs away from a concurrent launch.  0 = launched. */
int m3s_test_hold_cus(int nblocks, int lds_bytes, int usec, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* M3S_VARIANTS_H */
