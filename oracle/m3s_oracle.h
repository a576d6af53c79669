/*
 * m3s_oracle.h -- CPU restatement of the MASt3R-SLAM backend hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the HIP
 * product path (mast3r-slam_amd/csrc) and the timed CPU baseline of bench.py.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it.  The product path never calls into it.
 *
 * Parity status (see DESIGN.md "Oracle"):
 *   - The reference's native ops (matching_kernels.cu, gn_kernels.cu) cannot be
 *     built here: CUDA-only, Eigen submodule absent.  The reference ships no
 *     golden vectors for them.  => kernel-level parity is "unpinned" by the
 *     reference itself; the restatement is pinned by known-answer tests
 *     (tests/test_oracle_kat.py).
 *   - The Python glue around the ops (img_gradient, prep_for_iter_proj,
 *     match_iterative_proj post-processing, constrain_points_to_ray) IS pinned
 *     against the reference imported in the dev container
 *     (tests/golden/make_golden.py -> tests/golden/ fixtures).
 *
 * Numerics convention (pinned identically in oracle and HIP kernels):
 *   - FMA contraction as the reference's nvcc build does it (--fmad=true, setup.py:29-37):
 *     ORACLE_CONTRACT_NVCC by default, every fused multiply-add explicit (fmaf), the file
 *     itself compiled with -ffp-contract=off; ORACLE_CONTRACT_OFF / _NVCC_RIGHT are variants
 *     for measuring the convention;
 *   - every double-literal promotion in the reference source is reproduced as an
 *     explicit double operation followed by a cast to float;
 *   - fp16 arithmetic of refine_matches rounds after every * and += (c10::Half).
 */
#ifndef M3S_ORACLE_H
#define M3S_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* FMA contraction conventions (mast3r-slam_amd/csrc/contract.h) */
enum { ORACLE_CONTRACT_NVCC = 0, ORACLE_CONTRACT_OFF = 1, ORACLE_CONTRACT_NVCC_RIGHT = 2 };
/* the GN restatement's convention (alignment kernels, Sim3 library, retraction); default NVCC */
void oracle_set_contract(int cm);
int oracle_get_contract(void);

/* matching glue of the reference's Python caller (matching.py:25-90), host arithmetic */
void oracle_match_prep(const float* X11, const float* X21, const int64_t* idx_init, int64_t B, int64_t H,
                       int64_t W, float* rays9, float* pts, float* p_init);
void oracle_match_post(const float* X11, const float* X21, const float* p_new, const uint8_t* conv,
                       int64_t B, int64_t H, int64_t W, float dist_thresh, int64_t* p1, uint8_t* valid);
/* matching_kernels.cu:119-275 (iter_proj_kernel) + :279-316 (launcher), contraction cm */
void oracle_iter_proj(const float* rays, const float* pts, const float* p_init,
                      float* p_new, uint8_t* converged,
                      int64_t B, int64_t H, int64_t W, int64_t N,
                      int max_iter, float lambda_init, float cost_thresh, int cm);

/* matching_kernels.cu:25-81 (refine_matches_kernel<c10::Half>) */
void oracle_refine_matches_f16(const uint16_t* D11, const uint16_t* D21,
                               const int64_t* p1, int64_t* p1_new,
                               int64_t B, int64_t H, int64_t W, int64_t N,
                               int64_t F, int radius, int dilation_max);
/* matching_kernels.cu:25-81 (refine_matches_kernel<float>) */
void oracle_refine_matches_f32(const float* D11, const float* D21,
                               const int64_t* p1, int64_t* p1_new,
                               int64_t B, int64_t H, int64_t W, int64_t N,
                               int64_t F, int radius, int dilation_max);
/* matching_kernels.cu:25-81 (refine_matches_kernel<double>) */
void oracle_refine_matches_f64(const double* D11, const double* D21,
                               const int64_t* p1, int64_t* p1_new,
                               int64_t B, int64_t H, int64_t W, int64_t N,
                               int64_t F, int radius, int dilation_max);

/* fp16 helpers (c10::Half semantics: round-to-nearest-even, subnormals kept) */
uint16_t oracle_f32_to_f16(float f);
float oracle_f16_to_f32(uint16_t h);

/* Residual families of gn_kernels.cu */
enum { ORACLE_GN_POINTS = 0, ORACLE_GN_RAYS = 1, ORACLE_GN_CALIB = 2 };

typedef struct oracle_gn_params {
    int mode;              /* ORACLE_GN_* */
    float sigma0;          /* points: sigma_point; rays: sigma_ray; calib: sigma_pixel */
    float sigma1;          /* rays: sigma_dist; calib: sigma_depth */
    float C_thresh, Q_thresh;
    float K[9];            /* calib only, row-major 3x3 */
    int height, width, pixel_border;
    float z_eps;
    int max_iter;
    float delta_thresh;
} oracle_gn_params;

/*
 * One alignment kernel launch (point_align / ray_align / calib_proj):
 * ii_edge/jj_edge are ROW indices into Twc/Xs/Cs (already remapped).
 * Hs: [4, E, 7, 7], gs: [2, E, 7] in the reference layout.  The per-point sums
 * follow the reference's 256-thread strided loop and shared-memory tree
 * (gn_kernels.cu:31-55, 910-1137) so the float summation order matches.
 */
/*
 * The per-point residual model of the align kernels (no accumulation), for pinning it to the
 * reference's own Python (tests/golden/make_residual_golden.py): per directed point-edge the
 * transformed point T_ij Xj [E,HW,3], residuals [E,HW,4] and robust weights (Huber x
 * confidence) [E,HW,4] (calib/points: 3 rows, the 4th is 0) and the validity flag [E,HW].
 */
void oracle_gn_residuals(const oracle_gn_params* P, const float* Twc, const float* Xs,
                         const float* Cs, const int64_t* ii_edge, const int64_t* jj_edge,
                         const int64_t* idx, const uint8_t* valid, const float* Q,
                         int64_t N, int64_t HW, int64_t E, float* Xj_Ci, float* err, float* w,
                         uint8_t* valid_out);
void oracle_gn_align(const oracle_gn_params* P, const float* Twc, const float* Xs,
                     const float* Cs, const int64_t* ii_edge, const int64_t* jj_edge,
                     const int64_t* idx, const uint8_t* valid, const float* Q,
                     int64_t N, int64_t HW, int64_t E, float* Hs, float* gs);

/*
 * SparseBlock::update_lhs/update_rhs (gn_kernels.cu:71-113) into a dense
 * double system of size n = 7*(N-1) (row-major), b of size n.
 * ii_opt/jj_opt = row index - 1 (pose 0 pinned -> -1 -> dropped).
 */
void oracle_gn_assemble(const float* Hs, const float* gs, const int64_t* ii_opt,
                        const int64_t* jj_opt, int64_t N, int64_t E,
                        double* H, double* b);

/* One iteration's dense system with the per-edge blocks kept in double (equal to align +
 * assemble unless exact sums are on; then the exactly summed system, unrounded). */
void oracle_gn_system(const oracle_gn_params* P, const float* Twc, const float* Xs, const float* Cs,
                      const int64_t* ii_edge, const int64_t* jj_edge, const int64_t* idx,
                      const uint8_t* valid, const float* Q, int64_t N, int64_t HW, int64_t E,
                      double* H, double* b);

/* SimplicialLLT semantics: returns 0 on success, 1 when a pivot <= 0.  */
int oracle_cholesky_solve(double* H, const double* b, double* x, int64_t n);

/* pose_retr_kernel (gn_kernels.cu:415-453), num_fix = 1 */
void oracle_pose_retr(float* Twc, const float* dx, int64_t N, int num_fix);

/*
 * Full driver gauss_newton_{points,rays,calib}_cuda (gn_kernels.cu:725-811,
 * 1140-1228, 1546-1637).  ii/jj are GLOBAL keyframe ids (the op remaps them,
 * gn_kernels.cu:161-170).  Twc [N,8] is updated in place, dx [N-1,7] is the
 * last iteration's update.  Returns the number of iterations run.
 */
int oracle_gauss_newton(const oracle_gn_params* P, float* Twc, const float* Xs,
                        const float* Cs, const int64_t* ii, const int64_t* jj,
                        const int64_t* idx, const uint8_t* valid, const float* Q,
                        int64_t N, int64_t HW, int64_t E, float* dx);

/* unique(cat(ii,jj)) + searchsorted (gn_kernels.cu:161-170).  Writes row
 * indices (pin = 0).  Returns number of unique ids. */
int64_t oracle_remap(const int64_t* ii, const int64_t* jj, int64_t E,
                     int64_t* ii_edge, int64_t* jj_edge);

/* Sim3 helpers, exposed for the known-answer tests. */
void oracle_exp_sim3(const float* xi, float* t, float* q, float* s);
void oracle_retr_sim3(const float* xi, const float* t, const float* q, const float* s,
                      float* t1, float* q1, float* s1);
void oracle_apply_sim3_adj_inv(const float* t, const float* q, const float* s,
                               const float* X, float* Y);

int oracle_num_threads(void);
void oracle_set_num_threads(int n);

/* 1: sum the reference's float terms in double (a precision reference); 0 (default): the
 * reference's float sums in its order */
void oracle_set_exact_sums(int on);

#ifdef __cplusplus
}
#endif
#endif
