/*
 * sfmhip.h — C-ABI of libsfmhip.so, the MI355X (gfx950) backend for the dense
 * compute path of daovietanh190499/3D_Reconstruction (SfM matching, DLT
 * triangulation, reprojection residual / FD Jacobian, voxel-grid work).
 *
 * Conventions (all entry points):
 *   - Every pointer argument that names device data is a HIP device pointer owned
 *     by the caller (normally a torch-ROCm tensor's data_ptr()); the library never
 *     allocates, frees or retains caller memory.
 *   - `stream` is a hipStream_t passed as void* (0 = the null stream).  Calls are
 *     asynchronous on that stream; the Python wrappers synchronise before handing
 *     numpy arrays back, which keeps the cv2 / scipy call semantics.
 *   - Return value: 0 on success, a negative SFMHIP_E_* code on failure; the
 *     message for the calling thread is in sfmhip_last_error().
 *   - Row-major, densely packed arrays unless a stride is given.
 *   - An empty call (zero observations / pairs / rays / points / frames) is a no-op
 *     returning 0, and the arrays of that count may then be null (an empty torch
 *     tensor's data_ptr() is 0); shapes and counts are still validated first.
 *
 * Each entry point cites the reference interface it replaces (file:line in
 * /root/reference).  See INTEGRATION.md for the ctypes binding.
 */
#ifndef SFMHIP_H
#define SFMHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SFMHIP_OK            0
#define SFMHIP_E_ARG        -1   /* bad argument (shape, null pointer, range) */
#define SFMHIP_E_HIP        -2   /* HIP runtime error (launch / memory)        */
#define SFMHIP_E_UNSUPPORTED -3  /* e.g. descriptor dim not in {64,128,256}    */
#define SFMHIP_E_OVERFLOW   -4   /* a bounded loop hit its cap                 */
#define SFMHIP_E_COMM       -5   /* RCCL reported an error                      */

/* element types of sfmhip_allgather */
#define SFMHIP_DT_INT8    0
#define SFMHIP_DT_UINT8   1
#define SFMHIP_DT_INT16   2
#define SFMHIP_DT_INT32   3
#define SFMHIP_DT_INT64   4
#define SFMHIP_DT_FLOAT32 5
#define SFMHIP_DT_FLOAT64 6

/* ---- library ---------------------------------------------------------- */
int         sfmhip_version(void);            /* (major<<16)|(minor<<8)|patch */
const char* sfmhip_last_error(void);         /* thread-local message          */
int         sfmhip_device_arch(char* buf, int len); /* "gfx950" of device 0   */

/* Stream-ordered scratch comes from a library-owned memory pool per device
 * (never the device's default pool); up to 1 GiB of freed scratch stays
 * mapped between calls, and buffers up to 256 MB (1 GiB in all) are cached
 * per (device, stream) so the next call on that stream re-uses them without
 * waiting.  Releases the idle cached buffers of the current device (after a
 * device synchronisation), then trims its pool to `keep` bytes.             */
int         sfmhip_scratch_trim(uint64_t keep);
/* Releases the idle scratch cached for `stream`.  Call it before destroying a
 * stream that was passed to the library (a destroyed stream's buffers are
 * otherwise freed at the next eviction or trim, after a device sync).      */
int         sfmhip_scratch_release_stream(void* stream);
/* Runtime knobs (INTEGRATION.md "Runtime knobs") are read from the environment
 * once, at the first call; this re-reads them (tests switching a knob).      */
int         sfmhip_knobs_reload(void);

/* ---- M1: brute-force L2 matching + ratio test --------------------------
 * Replaces the matcher call site matching.py:20,122-128 (LightGlue forward,
 * output contract lightglue/lightglue.py:442-450).  The BF-L2 + Lowe-ratio
 * semantics are build-defined and pinned by oracle/match.py.
 *
 * Descriptors live in HBM as int8 [n_img][m_pad][d], rows >= n_kpts[img] zero.
 *   mode 0 (SIFT-like, integer values 0..255 stored as f32):  q = x - 128
 *   mode 1 (float, e.g. L2-normalised SuperPoint/DISK):       q = clamp(rint(127*x), -127, 127)
 * Squared L2 on q is exact in int32 (|q|<=128, d<=256).                       */
int sfmhip_desc_quantize(const float* in, int n_img, int m_pad, int d,
                         const int32_t* n_kpts /* device [n_img] */, int mode,
                         int8_t* out /* [n_img][m_pad][d] */, void* stream);

/* norms[img][r] = sum_k q^2 (int32); keys[img][r] = packed column key used by
 * the matcher's fused epilogue (see DESIGN.md "packed key").                  */
int sfmhip_desc_prepare(const int8_t* desc, int n_img, int m_pad, int d,
                        const int32_t* n_kpts, int32_t* norms, int32_t* keys,
                        void* stream);

/* Same as sfmhip_desc_prepare, plus a shifted operand copy for the matcher:
 * desc_shifted = q + shift on valid rows (0 on padding rows), norms and keys
 * adjusted so that sfmhip_match_pairs on (desc_shifted, norms, keys) returns
 * exactly the matches and distances of the unshifted q.  shift in [0, 127];
 * caller guarantees q + shift <= 127 for every valid element (shift 64:
 * q <= 63).
 * Speed only (lower MFMA switching power).                      */
int sfmhip_desc_prepare_shifted(const int8_t* desc, int n_img, int m_pad, int d,
                                const int32_t* n_kpts, int shift, int8_t* desc_shifted,
                                int32_t* norms, int32_t* keys, void* stream);

/* For every pair p=(a,b) and every row i < n_kpts[a] of image a: best column j1
 * (lowest index on ties) and second-best distance d2 over j != j1 in image b.
 * matches0[p][i] = j1 if ratio_den^2 * d1 < ratio_num^2 * d2 (exact, int64)
 * and n_kpts[b] >= 2, else -1; rows i >= n_kpts[a] get -1.
 * dist1/dist2 (nullable) receive d1/d2 (squared, quantised units).
 * m_pad must be a multiple of 128; d in {64,128,256}.                        */
int sfmhip_match_pairs(const int8_t* desc, const int32_t* norms, const int32_t* keys,
                       const int32_t* n_kpts, int n_img, int m_pad, int d,
                       const int32_t* pairs /* device [P][2] */, int P,
                       int ratio_num, int ratio_den,
                       int32_t* matches0 /* [P][m_pad] */,
                       int32_t* dist1, int32_t* dist2, void* stream);

/* The same graph written as int16 (the all-gathered match graph of SURVEY.md §8e,
 * replacing the matching.py:122-128 per-pair LightGlue call over every pair):
 * matches0 entries are identical values; m_pad <= 32767; no distance outputs.  */
int sfmhip_match_pairs_i16(const int8_t* desc, const int32_t* norms, const int32_t* keys,
                           const int32_t* n_kpts, int n_img, int m_pad, int d,
                           const int32_t* pairs, int P, int ratio_num, int ratio_den,
                           int16_t* matches0 /* [P][m_pad] */, void* stream);

/* LightGlue-style mutual filter (lightglue/lightglue.py:235-254 semantics):
 * given forward matches0 (a->b) and backward matches1 (b->a), both [P][m_pad],
 * clear every match that is not mutual, in place.                           */
int sfmhip_mutual_filter(int32_t* matches0, int32_t* matches1, int P, int m_pad,
                         void* stream);

/* Exact float mode (matching.py:111-122 feeds FLOAT DISK / SuperPoint
 * descriptors to the matcher).  Semantics (oracle/match.py bf_match_exact):
 * d(i,j) = sum_k (f64(x_ai,k) - f64(x_bj,k))^2 in k order, one IEEE f64 op
 * per step; j1 = lowest index attaining the minimum, d2 = min over j != j1;
 * accept iff ratio_den^2 * d1 < ratio_num^2 * d2 exactly.
 * sfmhip_desc_residual: per-row bound resid_row [n_img][m_pad] >= |x - v(q)|
 * (v(q) = q/127 for mode 1, q + 128 for mode 0; the int8 q of
 * sfmhip_desc_quantize) and resid_img [n_img] = the image's maximum.          */
int sfmhip_desc_residual(const float* desc_f /* [n_img][m_pad][d] */, const int8_t* desc_q, int n_img, int m_pad,
                         int d, const int32_t* n_kpts, int mode, double* resid_row, double* resid_img,
                         void* stream);

/* The int8 MFMA pass (desc/norms/keys as for sfmhip_match_pairs, shifted or
 * not) certifies every row whose outcome the residual bound decides; the rest
 * are settled against desc_f (f32) by an exact pass over the int8 candidates
 * that can still reach the top two.  matches0 is bit-identical to the exact
 * definition above; dist1/dist2 (nullable) are the int8 pass's quantised
 * distances; n_resolved (nullable, device uint32) = rows the exact pass
 * settled.  desc_q = the unshifted int8 descriptors.                         */
int sfmhip_match_pairs_exact(const int8_t* desc, const int32_t* norms, const int32_t* keys,
                             const int8_t* desc_q, const float* desc_f, const double* resid_row,
                             const double* resid_img, int mode, const int32_t* n_kpts, int n_img, int m_pad, int d,
                             const int32_t* pairs, int P, int ratio_num, int ratio_den,
                             int32_t* matches0, int32_t* dist1, int32_t* dist2, uint32_t* n_resolved,
                             void* stream);

/* sfmhip_match_pairs_exact writing the int16 graph directly (the bench's and
 * dist.match_all_pairs_sharded's graph dtype while m_pad <= 32767; matching.py:122-128
 * over every pair): the same matches0 values, no distance outputs.  Undecided rows
 * carry ceil(8 sqrt(D2)) in their transient mark instead of D2 (a wider candidate
 * radius for the exact pass, never a different result).                      */
int sfmhip_match_pairs_exact_i16(const int8_t* desc, const int32_t* norms, const int32_t* keys,
                                 const int8_t* desc_q, const float* desc_f, const double* resid_row,
                                 const double* resid_img, int mode, const int32_t* n_kpts, int n_img, int m_pad,
                                 int d, const int32_t* pairs, int P, int ratio_num, int ratio_den,
                                 int16_t* matches0, uint32_t* n_resolved, void* stream);

/* ---- M2: scipy.cluster.vq.vq (matching.py:27, bow.py:23) ---------------
 * codes[i] = argmin_c sum_k (obs[i,k]-code[c,k])^2 (lowest index on ties),
 * dist[i] = sqrt(min).  f64 throughout.                                      */
int sfmhip_vq(const double* obs, int64_t n_obs, const double* code_book, int n_codes,
              int d, int32_t* codes, double* dist, void* stream);

/* ---- BoW retrieval ---------------------------------
 * Per-image visual-word histograms (matching.py:30-35): codes of all images
 * concatenated, image i owns codes[offsets[i] : offsets[i+1]];
 * hist [n_img][k] int32.                                                      */
int sfmhip_word_histogram(const int32_t* codes, const int64_t* offsets, int n_img, int k,
                          int32_t* hist, void* stream);

/* scipy.cluster.vq.kmeans centroid update (bow.py:23 -> _vq.update_cluster_means):
 * per cluster, the f64 sum of its observations in index order, / count.
 * book [k][d] rows of empty clusters are left untouched; counts [k].          */
int sfmhip_kmeans_update(const double* obs, int64_t n, int d, const int32_t* codes, int k,
                         double* book, int32_t* counts, void* stream);

/* ---- match-graph consumer, HOST memory ------------
 * Track bookkeeping of matching.py:146-176 for one candidate pair (ref, id):
 * tracks_* are the per-keypoint 3D-point ids of the two images (-1 = none);
 * idx0/idx1 the pair's matches.  interlace = the count of matching.py:146-158;
 * merge = matching.py:161-176 (updates tracks in place, point_ids[n] out,
 * *next_id advanced).  The reference's p1/p2 index quirks are kept.          */
int sfmhip_track_interlace(const int32_t* tracks_ref, int64_t n_ref, const int32_t* tracks_id, int64_t n_id,
                           const int64_t* idx0, const int64_t* idx1, int64_t n, int64_t* interlaced);
int sfmhip_track_merge(int32_t* tracks_ref, int64_t n_ref, int32_t* tracks_id, int64_t n_id,
                       const int64_t* idx0, const int64_t* idx1, int64_t n, int64_t* next_id,
                       int64_t* point_ids);

/* ---- S2: cv2.triangulatePoints (sfm.py:27) ------------------------------
 * OpenCV DLT: per point a 6x4 system (rows x*p3-p1, y*p3-p2, x*p2-y*p1 per
 * view), right singular vector of the smallest singular value (one-sided
 * Jacobi, f64).  x0/x1 are cv2 layout (2,n); X4 is (4,n), unit norm, X4[3]>=0.
 * Batched form: P is [n_pairs][2][3][4] and pair_of_obs[n] selects the pair
 * (pair_of_obs == NULL means one pair).                                      */
int sfmhip_triangulate_dlt(const double* P, const int32_t* pair_of_obs,
                           const double* x0, const double* x1, int64_t n,
                           double* X4, void* stream);

/* ---- S3/S5: reprojection residual + scipy 2-point grouped FD Jacobian ----
 * sfm.py:87-91 (residual via cv2.projectPoints, no distortion) and
 * least_squares(..., jac_sparsity=ba_sparse(...)) sfm.py:37-38.
 * cam: [n_pairs][6] = rvec(3), t(3);  K: [n_pairs][3][3] (fx,fy,cx,cy used);
 * X: [n][3]; pts2d: [n][2]; pair_of_obs: [n] (NULL = one pair).
 * r: [n][2]  residual (pts2d - proj)  (nullable)
 * f0: [n][2] base residual to difference against (NULL = computed here)
 * jvals: [n][2][9] CSR values of J, per row: d/d(rvec0..2,t0..2, X0..2).    */
int sfmhip_reproj_residual(const double* cam, const double* K, const double* X,
                           const double* pts2d, const int32_t* pair_of_obs,
                           int64_t n, double* r, void* stream);
/* HOST arrays (the cv2.projectPoints / calculate_reprojection_error contract
 * sfm.py:87-91, called by scipy's least_squares ~40 times per pair at sfm.py:38):
 * cam[6], K[9], X[n][3], pts2d[n][2] (NULL = zeros, i.e. -projectPoints) and
 * r[n][2] are host memory.  One pinned staging buffer per device (library-owned,
 * grows on demand) that the kernel reads and writes over PCIe (zero-copy), then a synchronisation
 * of `stream`.  Blocking; thread-safe (the staging is locked per device).     */
int sfmhip_reproj_residual_host(const double* cam, const double* K, const double* X,
                                const double* pts2d, int64_t n, double* r, void* stream);
int sfmhip_reproj_fd_jacobian(const double* cam, const double* K, const double* X,
                              const double* pts2d, const int32_t* pair_of_obs,
                              int n_pairs, int64_t n, const double* f0,
                              double* r, double* jvals, void* stream);

/* The BA solve of sfm.py:37-38 (scipy least_squares, method 'trf', tr_solver
 * 'lsmr', jac_sparsity = ba_sparse, x_scale = 'jac', ftol / xtol / gtol) for
 * n_pairs independent problems at once, one workgroup each.  Problem p:
 * x = [cam[p] (rvec 3, t 3), X[off[p]..off[p+1]) (3 each)], residual
 * pts2d - projectPoints(X, rvec, t, K[p]) (calculate_reprojection_error,
 * sfm.py:87-91).  cam (n_pairs, 6) and X (n, 3) are updated in place;
 * pair_off (n_pairs + 1) int64 device offsets (off[0] = 0, observations of a
 * pair contiguous); max_nfev <= 0: scipy's default 100 * len(x).  Outputs per
 * pair: final cost 0.5 |f|^2, nfev, njev, status (scipy's codes 0..4).
 * n_obs = rows of X / pts2d: a pair whose offsets are not
 * 0 <= off[p] <= off[p+1] <= n_obs touches nothing and gets status -1.
 * The Gauss-Newton direction is the exact damped least-squares solution where
 * scipy runs LSMR to 1e-6 (oracle/ba.py). */
int sfmhip_ba_solve(double* cam, const double* K, double* X, const double* pts2d, const int64_t* pair_off,
                    int n_pairs, int64_t n_obs, double ftol, double xtol, double gtol, int max_nfev, double* cost,
                    int32_t* nfev, int32_t* njev, int32_t* status, void* stream);

/* ---- V1: voxel_traversal (voxel_travesal.py:1-73), quirks included -------
 * rays [N][8] f32 = o(3), d(3), near, far.  Pass 1 counts per-ray steps
 * (n_steps[N]; a ray still active after max_steps reports max_steps + 1),
 * pass 2 writes out [N][S][3] f32 (NaN padded) with S = 1 + max(n_steps).   */
int sfmhip_voxel_traversal_count(const float* rays, int64_t N, float bin,
                                 int32_t max_steps, int32_t* n_steps, void* stream);
int sfmhip_voxel_traversal(const float* rays, int64_t N, float bin, int32_t S,
                           float* out, void* stream);
/* One walk instead of two: each ray's visited voxels into rows of width `cap`
 * (buf [N][cap][3]; entries past a row's end are left unwritten) and its step
 * count (n_steps[N]; cap when the ray is still active after cap - 1 steps).
 * When every n_steps < cap, sfmhip_voxel_traversal_rows with S = 1 + max
 * n_steps writes exactly the two-pass form's out [N][S][3] (NaN padded);
 * otherwise the caller falls back to the two-pass form.                    */
int sfmhip_voxel_traversal_capped(const float* rays, int64_t N, float bin, int32_t cap,
                                  float* buf, int32_t* n_steps, void* stream);
int sfmhip_voxel_traversal_rows(const float* buf, int32_t cap, const int32_t* n_steps,
                                int64_t N, int32_t S, float* out, void* stream);

/* ---- V2: trilinear grid sample (sdf.py:284-342, plenoxel.py:31-43) -------
 * grid in the reference layout (1,C,D,H,W) f32.  pts [P][3] world coords.
 * mask_mode 0: sdf.py  (inside iff bmin <= p <= bmax, normalise to [-1,1])
 * mask_mode 1: plenoxel (inside iff |p| < scale=bmax[0], p/scale clipped)
 * out [P][C] (zero outside).  F.grid_sample(align_corners=True, zeros)
 * arithmetic, x->W, y->H, z->D.  bmin/bmax are HOST float[3].               */
int sfmhip_grid_sample(const float* grid, int C, int D, int H, int W,
                       const float* bmin, const float* bmax, int mask_mode,
                       const float* pts, int64_t P, float* out, void* stream);

/* NerfModel.forward (plenoxel.py:31-43) for C = 28 grids in the reference
 * layout: color [P][3] = eval_spherical_function(channels 1..27, dirs),
 * sigma [P] = ReLU(channel 0), both zero outside the mask (mask_mode as in
 * sfmhip_grid_sample); dirs [P][3].  bmin/bmax are HOST float[3].           */
int sfmhip_nerf_forward(const float* grid, int D, int H, int W, const float* bmin, const float* bmax,
                        int mask_mode, const float* pts, const float* dirs, int64_t P, float* color,
                        float* sigma, void* stream);

/* Voxel-major relayout (C,D,H,W) -> (D,H,W,Cp) with Cp = 32 (zero pad) so a
 * corner's channels are one 128-byte line; used by the fused renderer.       */
int sfmhip_grid_to_voxel_major(const float* grid, int C, int D, int H, int W,
                               float* grid_vm, void* stream);

/* ---- V4: fused sample + SH-2 colour + alpha composite --------------------
 * sdf.py:391-406 / plenoxel.py:71-93 for C=28 grids.  rays_o/rays_d [B][3],
 * z [B][S] (sorted sample depths).  rgb [B][3] = sum T*a*c + 1 - sum T*a.
 * grid_vm from sfmhip_grid_to_voxel_major; bmin/bmax are HOST float[3].     */
int sfmhip_render_rays(const float* grid_vm, int D, int H, int W,
                       const float* bmin, const float* bmax, int mask_mode,
                       const float* rays_o, const float* rays_d, const float* z,
                       int64_t B, int S, float* rgb, void* stream);
/* The same render with the SDF (channel 0) also given as the compact reference
 * plane (D,H,W) f32 (grid channel 0 of the (C,D,H,W) layout): each sample's sdf
 * is read from it and the 28-channel voxel lines are fetched only for samples
 * with alpha != 0 (w = T*alpha = 0 otherwise).  The caller guarantees a finite
 * grid; the result is then bit-identical to sfmhip_render_rays.              */
int sfmhip_render_rays_sdf(const float* grid_vm, const float* sdf_plane, int D, int H, int W,
                           const float* bmin, const float* bmax, int mask_mode,
                           const float* rays_o, const float* rays_d, const float* z,
                           int64_t B, int S, float* rgb, void* stream);

/* ---- V5: TSDF integration (build-defined) --------------
 * T, Wt: (D,H,W) f32 grids updated in place for z-slices [z0, z1), laid out
 * like the sdf.py grid (sdf.py:284-304: x -> W, align_corners).
 * depth [F][Hd][Wd] f32 (<= 0 invalid); poses [F][3][4] world->camera;
 * Kf [F][4] = fx, fy, cx, cy; bmin/bmax are HOST float[3] grid bounds;
 * trunc = truncation distance mu (world units).  The frames of one integration
 * step (the call, in steps of at most 512 frames) are fused order-free: per
 * voxel S = sum rint(tsdf * 2^21) and n updates, then W' = W + n,
 * T' = f32((f64 T * W + S 2^-21) / (W + n))  (oracle/voxel.py tsdf_integrate).
 * F = 0 or z0 = z1: a no-op (with F = 0 the frame arrays may be null).        */
int sfmhip_tsdf_integrate(float* T, float* Wt, int D, int H, int W, int z0, int z1,
                          const float* depth, int F, int Hd, int Wd,
                          const float* poses, const float* Kf,
                          const float* bmin, const float* bmax, float trunc,
                          void* stream);

/* The TSDF pre-pass table on its own, for sharing across ranks (multi-GPU
 * z-slabs: each rank computes the table of a frame range and an all-gather
 * assembles it, instead of every rank reading every depth map): {min, max}
 * of every 16x16 depth block, table [F][ceil(Hd/16)][ceil(Wd/16)][2] f32
 * (min poisoned by NaN, max ignoring NaN); rows [f0, f1) are written.      */
int sfmhip_tsdf_block_table(const float* depth, int F, int Hd, int Wd,
                            int f0, int f1, float* table, void* stream);

/* sfmhip_tsdf_integrate with the caller's full block table (all F frames,
 * whole image, as written by sfmhip_tsdf_block_table): bit-identical
 * result, the call's own block pass skipped.                                 */
int sfmhip_tsdf_integrate_tab(float* T, float* Wt, int D, int H, int W, int z0, int z1,
                              const float* depth, int F, int Hd, int Wd,
                              const float* poses, const float* Kf,
                              const float* bmin, const float* bmax, float trunc,
                              const float* table, void* stream);

/* Diagnostics for the TSDF pre-passes (no reference counterpart): runs only
 * the culling / free-space tests of sfmhip_tsdf_integrate over the same
 * arguments and returns HOST int64 stats[3] = (wave sub-tile, frame) pairs
 * tested, culled (no voxel updates), free space (every voxel updates with
 * tsdf = 1, fused without depth gathers).  Synchronises the stream.         */
int sfmhip_tsdf_cull_stats(int D, int H, int W, int z0, int z1,
                           const float* depth, int F, int Hd, int Wd,
                           const float* poses, const float* Kf,
                           const float* bmin, const float* bmax, float trunc,
                           int64_t* stats, void* stream);

/* Per-layer version for z-slab planning (multi-GPU): the same tests over the
 * whole grid, HOST int64 layer_stats[ceil(D/8)][3] (tested, culled, free) per
 * 8-voxel tile layer in z.  Synchronises the stream.                         */
int sfmhip_tsdf_layer_stats(int D, int H, int W, const float* depth, int F, int Hd, int Wd,
                            const float* poses, const float* Kf, const float* bmin, const float* bmax,
                            float trunc, int64_t* layer_stats, void* stream);

/* ---- §8f row 2: geometric verification (batched over image pairs) --------
 * cv2.findEssentialMat(pts0, pts1, K, method=cv2.RANSAC, prob=0.999,
 * threshold=1) at matching.py:134 and sfm.py:108 (OpenCV five-point.cpp +
 * ptsetreg.cpp, maxIters 1000 by default): cv::RNG(-1) 5-point samples,
 * Nister solver, Sampson error (float) <= (thresh/((fx+fy)/2))^2, a model
 * replaces the best iff count > max(best, 4), RANSACUpdateNumIters.
 * Pair p owns rows [offsets[p], offsets[p+1]) of pts0/pts1 ([N][2] f64
 * pixels); cam [n_pairs][4] = fx, fy, cx, cy.  work [N][4] f64 scratch.
 * Out: E [n_pairs][10][9] (row-major; model 0 is the RANSAC result, all
 * models only when a pair has exactly 5 points), n_models (0 = no model,
 * cv2 returns None), mask [N] u8 0/1, n_inliers, iters (hypotheses drawn).
 * All pointers are device memory.                                            */
int sfmhip_find_essential(const double* pts0, const double* pts1, const int64_t* offsets,
                          int n_pairs, const double* cam, double prob, double threshold,
                          int max_iters, double* work, double* E, int32_t* n_models,
                          uint8_t* mask, int32_t* n_inliers, int32_t* iters, void* stream);

/* cv2.recoverPose(E, pts0, pts1, K) at matching.py:139, sfm.py:117,119
 * (distanceThresh = 50): decomposeEssentialMat + DLT cheirality of the 4
 * candidate poses.  E for pair p at E + p*e_stride (e_stride >= 9, 90 for
 * sfmhip_find_essential's output); mask_in [N] u8 or NULL (rows with 0 are
 * excluded, == recoverPose on the compacted points).  Out: R [n_pairs][9],
 * t [n_pairs][3], mask_out [N] u8 0/255, n_good [n_pairs].                   */
int sfmhip_recover_pose(const double* E, int64_t e_stride, const double* pts0, const double* pts1,
                        const int64_t* offsets, int n_pairs, const double* cam,
                        const uint8_t* mask_in, double distance_thresh, double* R, double* t,
                        uint8_t* mask_out, int32_t* n_good, void* stream);

/* cv2.solvePnPRansac(X, pts1, K, zeros(5,1), cv2.SOLVEPNP_ITERATIVE) at
 * sfm.py:116 (iterationsCount 100, reprojectionError 8, confidence 0.99):
 * points converted to float, cv::RNG(-1) 5-point samples solved by EPnP,
 * float squared reprojection error <= reprojectionError^2, the RANSAC pose
 * refined on its inliers by CvLevMarq (20 iterations).  Problem p owns rows
 * [offsets[p], offsets[p+1]) of obj ([N][3] f64) / img ([N][2] f64 pixels);
 * cam [n][4] = fx, fy, cx, cy; work [N][5] f32 scratch.  Out: rvec/tvec
 * [n][3], inlier_mask [N] u8 (RANSAC inliers), n_inliers, iters, ok.
 * n < 5 is reported as ok = 0 (OpenCV would use P3P at n == 4).           */
int sfmhip_pnp_ransac(const double* obj, const double* img, const int64_t* offsets, int n_problems,
                      const double* cam, int iterations, double reprojection_error, double confidence,
                      float* work, double* rvec, double* tvec, uint8_t* inlier_mask, int32_t* n_inliers,
                      int32_t* iters, int32_t* ok, void* stream);

/* ---- §8f row 4: one grid training step (plenoxel.py:100-111, sdf.py:427-438)
 * Fused render forward + mse_loss(gt, rgb) gradient + analytic backward +
 * trilinear scatter-add into grad_vm (voxel-major (D,H,W,32), accumulated;
 * zero it via sfmhip_adam_step's zero_grad).  S <= 256.  Out: rgb [B][3],
 * sqerr [B] = sum_ch (rgb - gt)^2 (loss = sum(sqerr) / (3B)); touched
 * [D*H*W] u8 (nullable): set to 1 for every voxel the scatter adds to.      */
int sfmhip_render_train(const float* grid_vm, int D, int H, int W, const float* bmin, const float* bmax,
                        int mask_mode, const float* rays_o, const float* rays_d, const float* z,
                        const float* gt, int64_t B, int S, float* rgb, float* sqerr, float* grad_vm,
                        uint8_t* touched, void* stream);

/* torch.optim.Adam single-tensor step (weight_decay 0, amsgrad off) over n
 * f32 parameters (n % 4 == 0), step = the step count after increment;
 * zero_grad != 0 also clears grad (optimizer.zero_grad).                     */
int sfmhip_adam_step(float* param, float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                     double lr, double beta1, double beta2, double eps, int64_t step, int zero_grad,
                     void* stream);

/* The same Adam step when the gradient is known to be 0 outside flagged
 * runs: flags [ceil(n / 2^flag_shift)] u8, one per 2^flag_shift parameters
 * (the trainer: one per 32-channel voxel line, set by sfmhip_render_train's
 * `touched`); unflagged gradients are neither read nor re-zeroed, and with
 * zero_grad the flags are cleared too.  Results equal sfmhip_adam_step's.     */
int sfmhip_adam_step_flagged(float* param, float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                             double lr, double beta1, double beta2, double eps, int64_t step, int zero_grad,
                             uint8_t* flags, int flag_shift, void* stream);

/* (D,H,W,32) voxel-major -> (C,D,H,W) reference layout (trainer export).     */
int sfmhip_grid_from_voxel_major(const float* grid_vm, int C, int D, int H, int W, float* grid,
                                 void* stream);

/* ---- V3: GradientBasedSampler's effective samples (sdf.py:154-180, 251-256)
 * Slab ray/AABB test: t_near = max(max_a min(t0, t1), 0), t_far = min_a max(t0,
 * t1), valid = t_far > t_near (NaN rays invalid).  Bounds are HOST float[3]. */
int sfmhip_ray_aabb(const float* rays_o, const float* rays_d, int64_t B, const float* bmin,
                    const float* bmax, float* t_near, float* t_far, uint8_t* valid, void* stream);

/* Stratified uniform samples (sample_uniform, sdf.py:167-180): z = t_near (1-t)
 * + t_far t with t = linspace(0,1,S); perturb: lower + (upper-lower) t_rand.  */
int sfmhip_stratified_samples(const float* t_near, const float* t_far, const float* t_rand, int64_t B,
                              int S, int perturb, float* z, void* stream);

/* ---- multi-GPU: the match-graph collective ---------
 * Thin C-ABI over RCCL (resolved with dlopen at first use: the RCCL already
 * mapped into the process, else $SFMHIP_RCCL, else /opt/rocm/lib/librccl.so.1).
 * The reference has no distributed code; these serve the pair-sharded
 * exhaustive matcher: every rank matches its pairs, then ONE all-gather of the
 * fixed-size matches0 block over xGMI gives every rank the full graph.
 *   one process per GPU: sfmhip_comm_unique_id (one rank) -> broadcast the 128
 *     bytes -> sfmhip_comm_init_rank on every rank (current HIP device);
 *   one process, several GPUs: sfmhip_comm_init_all(ndev, devs, comms[ndev]),
 *     each rank's collective issued between sfmhip_comm_group_start/_end.
 * sfmhip_allgather: `count` elements of SFMHIP_DT_* per rank from `send`,
 * recv = nranks * count elements in rank order; asynchronous on `stream`.    */
int sfmhip_comm_unique_id(void* id /* 128 bytes, host */);
int sfmhip_comm_init_rank(int nranks, const void* id, int rank, void** comm);
int sfmhip_comm_init_all(int ndev, const int* devs /* NULL = 0..ndev-1 */, void** comms /* [ndev] */);
int sfmhip_comm_info(void* comm, int* nranks, int* rank, int* device);
int sfmhip_allgather(void* comm, const void* send, void* recv, size_t count, int dtype, void* stream);
int sfmhip_comm_group_start(void);
int sfmhip_comm_group_end(void);
int sfmhip_comm_destroy(void* comm);

#ifdef __cplusplus
}
#endif
#endif /* SFMHIP_H */
