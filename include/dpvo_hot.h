/*
 * dpvo_hot.h -- C ABI of the MI355X-native DPVO patch-graph hot path.
 *
 * One shared library (libdpvo_hot.so, built from
 * the HIP sources in wild-video-3d-reconstruction_amd/csrc, for gfx950) exports the entry
 * points below.  They replace the three PyTorch extensions the reference
 * builds in setup.py:43-66 (cuda_corr, cuda_ba, lietorch_backends); the
 * Python modules of the same names in wild-video-3d-reconstruction_amd/ bind
 * them with ctypes and keep the reference's call signatures.
 *
 * Conventions
 *  - All data pointers are DEVICE pointers (HIP, gfx950) unless stated.
 *  - Sizes/strides are in ELEMENTS, int64, outermost first (torch order).
 *  - `stream` is a hipStream_t passed as void*; NULL = the null stream.
 *    Nothing here synchronises the host; every call only enqueues work.
 *  - Return value: 0 on success, <0 on error (dpvo_hot_last_error() gives
 *    the message; the Python shims raise RuntimeError with it, matching the
 *    reference's TORCH_CHECK behaviour).
 *  - Outputs are caller-allocated (the shims allocate them with torch so the
 *    caching allocator owns them), as are workspaces (size via *_bytes()).
 */
#ifndef DPVO_HOT_H
#define DPVO_HOT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { DPVO_F16 = 0, DPVO_F32 = 1, DPVO_F64 = 2 };

/* ABI version history:
 *  1 -- rounds 1-2.
 *  2 -- dpvo_rowchain / dpvo_rowchain_gated / dpvo_rowchain3 read every W
 *       k-blocked ([K/32][384][32] instead of [384][K]); dpvo_rowadd_args
 *       gained c16 / c_idx / c_rows.  A caller built against version 1 must
 *       not run against this library. */
#define DPVO_HOT_ABI_VERSION 2

int dpvo_hot_abi_version(void);
const char* dpvo_hot_last_error(void);
/* "sha=<16 hex> flavour=<product|stamps>": the sha256 prefix of the HIP
 * sources the library was compiled from (the .hip and .hpp files of csrc in byte
 * order, then this header, concatenated) and whether it is the diagnostic
 * build with in-kernel stamps (DPVO_STAMPS).  The Python loader refuses a
 * library whose sha differs from the sources shipped beside it, and a stamps
 * build unless DPVO_DIAG=1. */
const char* dpvo_hot_build_info(void);

/* ------------------------------------------------------------------------
 * altcorr -- replaces cuda_corr (reference dpvo/altcorr/correlation.cpp:57-62)
 * --------------------------------------------------------------------- */

/* cuda_corr.forward(fmap1, fmap2, coords, ii, jj, radius)
 * (correlation.cpp:28-35 -> correlation_kernel.cu:193-233).
 * gmap  [B][N1][C][P][P]   (the reference's "fmap1": per-patch features)
 * fmap  [B][N2][C][H2][W2] (one pyramid level; any strides -- channel-last
 *                           storage, stride(C)==1, takes the fast path)
 * coords[B][E][2][P][P] float; ii, jj [E] int64.
 * corr  contiguous [B][E][2r+1 (y)][2r+1 (x)][P][P] of `dtype`: the memory
 *       of the reference's pre-permute tensor (the shim returns the same
 *       .permute(0,1,3,2,4,5) view).
 * fp16 results are bit-identical to the reference's c10::Half arithmetic. */
int dpvo_corr_forward(int dtype, const void* gmap, const int64_t* gmap_size, const int64_t* gmap_stride,
                      const void* fmap, const int64_t* fmap_size, const int64_t* fmap_stride, const float* coords,
                      const int64_t* coords_size, const int64_t* coords_stride, const int64_t* ii, const int64_t* jj,
                      int radius, void* corr, void* stream);

/* Fused DPVO.corr (reference dpvo/dpvo.py:326-333): both pyramid levels of
 * one gmap against `nlev` fmaps with coords scaled by 1/level_scale[l],
 * written directly in the stacked layout the update operator consumes:
 * corr [B][E][2r+1 (x)][2r+1 (y)][P][P][nlev] of `dtype`
 * (= torch.stack([corr1, corr2], -1).view(1, E, -1)). */
int dpvo_corr_forward_pyramid(int dtype, const void* gmap, const int64_t* gmap_size, const int64_t* gmap_stride,
                              int nlev, const void* const* fmaps, const int64_t* fmap_sizes /* nlev*5 */,
                              const int64_t* fmap_strides /* nlev*5 */, const float* level_scale,
                              const float* coords, const int64_t* coords_size, const int64_t* coords_stride,
                              const int64_t* ii, const int64_t* jj, int radius, void* corr, void* stream);

/* Same, with consecutive edges `edge_stride` elements apart (0 = packed), so
 * the update operator's first Linear can read 16-byte aligned rows
 * (882 features padded to 896; pad columns are left untouched), and with the
 * gmap's packed scalar-operand table from dpvo_corr_pack (NULL: packed
 * internally into stream-ordered scratch on every call). */
int dpvo_corr_forward_pyramid_ld(int dtype, const void* gmap, const int64_t* gmap_size, const int64_t* gmap_stride,
                                 int nlev, const void* const* fmaps, const int64_t* fmap_sizes,
                                 const int64_t* fmap_strides, const float* level_scale, const float* coords,
                                 const int64_t* coords_size, const int64_t* coords_stride, const int64_t* ii,
                                 const int64_t* jj, int radius, void* corr, int64_t edge_stride, const void* table,
                                 void* stream);

/* The fp16 fast path reads patch features as scalar operands from a packed
 * table [B*N1][C][5] dwords ((p0,p1)(p2,p3)(p4,p5)(p6,p7)(p8,0) per channel).
 * Pack once per gmap change (a new keyframe) and pass it to
 * dpvo_corr_forward_pyramid_ld; table is 16-byte aligned, size from
 * dpvo_corr_table_bytes. */
size_t dpvo_corr_table_bytes(const int64_t* gmap_size);
int dpvo_corr_pack(const void* gmap, const int64_t* gmap_size, const int64_t* gmap_stride, void* table, void* stream);

/* DPVO.corr (dpvo.py:326-333) on the matrix cores: both pyramid levels, the
 * same 882-wide stacked rows as dpvo_corr_forward_pyramid_ld with radius 3
 * and 3x3 patches, but the 128-channel dot products accumulate in fp32
 * (v_mfma_f32_16x16x32_f16) and the bilinear epilogue runs in fp32, rounded
 * once to fp16 -- more accurate than the reference's fp16 accumulation, not
 * bit-identical to it (dpvo_corr_forward_pyramid_ld is).  table: the gmap
 * ring transposed to [N1][9][128] by dpvo_corr_pack_mfma (gmap [1][N1][128][3][3]);
 * fmaps: 2 levels, [1][N2][128][H][W] channel-last; coords [1][E][2][3][3];
 * corr rows edge_stride halves apart (0: 882).  order (optional, NULL = edge
 * order): a permutation of the edges from dpvo_edge_order(jj) -- edges that
 * read one target frame then run back to back on one XCD, whose L2 holds
 * that frame's map; the output does not depend on it. */
size_t dpvo_corr_pack_mfma_bytes(const int64_t* gmap_size);
int dpvo_corr_pack_mfma(const void* gmap, const int64_t* gmap_size, const int64_t* gmap_stride, void* table,
                        void* stream);
int dpvo_corr_pyramid_mfma(const void* table, int64_t num_patches, const void* const* fmaps,
                           const int64_t* fmap_sizes, const int64_t* fmap_strides, const float* level_scale,
                           const float* coords, const int64_t* coords_size, const int64_t* coords_stride,
                           const int64_t* ii, const int64_t* jj, void* corr, int64_t edge_stride, const int* order,
                           void* stream);

/* A permutation of the E edges grouped by jj (values outside [0,
 * num_buckets) last), by a counting sort; the order inside a group is
 * unspecified.  Workspace: dpvo_edge_order_workspace_bytes(num_buckets). */
size_t dpvo_edge_order_workspace_bytes(int num_buckets);
int dpvo_edge_order(const int64_t* jj, int64_t num_edges, int num_buckets, int* order, void* workspace,
                    size_t workspace_bytes, void* stream);

/* cuda_corr.backward (correlation_kernel.cu:236-286): grad is the returned
 * (permuted) view's gradient given as contiguous [B][E][2r+1 (x)][2r+1 (y)][P][P]
 * float; gmap_grad / fmap_grad (contiguous, dtype, zero-filled by caller)
 * are accumulated with atomics. */
int dpvo_corr_backward(int dtype, const void* gmap, const int64_t* gmap_size, const void* fmap,
                       const int64_t* fmap_size, const float* coords, const int64_t* coords_size, const int64_t* ii,
                       const int64_t* jj, const float* grad, int radius, void* gmap_grad, void* fmap_grad,
                       void* stream);

/* cuda_corr.patchify_forward(net[B][C][H][W], coords[B][M][2] f32, radius)
 * (correlation_kernel.cu:17-47,288-308): patches contiguous [B][M][C][D][D],
 * D = 2r+2; out-of-image taps are written as zero. */
int dpvo_patchify_forward(int dtype, const void* net, const int64_t* net_size, const int64_t* net_stride,
                          const float* coords, int64_t M, int radius, void* patches, void* stream);

/* cuda_corr.patchify_backward (correlation_kernel.cu:50-80,310-333):
 * grad contiguous [B][M][C][D][D]; net_grad contiguous [B][C][H][W], zeroed
 * by the caller, accumulated with atomics (f32/f64 only). */
int dpvo_patchify_backward(int dtype, const int64_t* net_size, const float* coords, int64_t M, int radius,
                           const void* grad, void* net_grad, void* stream);

/* ------------------------------------------------------------------------
 * fastba -- replaces cuda_ba (reference dpvo/fastba/ba.cpp:236-241)
 * --------------------------------------------------------------------- */

/* Workspace bytes for dpvo_ba_forward. */
size_t dpvo_ba_workspace_bytes(int64_t num_edges, int64_t num_patches, int num_opt_poses);

/* cuda_ba.forward(poses, patches, intrinsics, target, weight, lmbda, ii, jj,
 * kk, t0, t1, iterations) (ba.cpp:31-43 -> ba_cuda.cu:422-540).
 * poses [*][7] and patches [num_patches][3][P][P] (contiguous float) are
 * updated IN PLACE; intrinsics row 0 is used; target, weight [E][2];
 * lmbda [1]; ii, jj, kk [E] int64.
 * status (device int, may be NULL) receives 0, or the order of the leading
 * minor at which the Cholesky factorisation failed (the reference raises
 * there); iterations after a failure are skipped. */
int dpvo_ba_forward(float* poses, float* patches, int64_t num_patches, int P, const float* intrinsics,
                    const float* target, const float* weight, const float* lmbda, const int64_t* ii,
                    const int64_t* jj, const int64_t* kk, int64_t num_edges, int t0, int t1, int iterations,
                    void* workspace, size_t workspace_bytes, int* status, void* stream);

/* Same, with a solver choice.  Windows of up to 12 optimised poses (DPVO's
 * sliding window of 10) use the deterministic per-patch path: one wave per
 * unique patch reduces its edges' C, u, E row and pose-block terms without
 * atomics, per-wave partials of S = B - E Q E^T are summed in a fixed order,
 * one workgroup factors S (fp32 Cholesky) -- bitwise repeatable, fully
 * asynchronous.  Windows of 13..64 poses (or DPVO_BA_ATOMIC) use the dense
 * atomic path: dense B / E, one-wave Cholesky.  Larger windows -- the global
 * BA of dpvo.py:436-505, t0 = 1, t1 = n -- or DPVO_BA_SPARSE use the sparse
 * path: per-edge Schur entries instead of the dense E (6N x Mu), S
 * accumulated into 64 x 64 tiles of its band, tiled band Cholesky.  Up to
 * 32767 poses.  The sparse path reads the pose-graph bandwidth back to the
 * host once per call (one stream synchronisation); its status is the failing
 * leading-minor order as above. */
enum { DPVO_BA_AUTO = 0, DPVO_BA_SPARSE = 1, DPVO_BA_ATOMIC = 2, DPVO_BA_KEEP_STATUS = 4 };
/* DPVO_BA_KEEP_STATUS (deterministic sliding-window path): *status is not
 * cleared on entry; when it already holds a failure the call changes nothing
 * (every kernel returns on entry) and the word keeps the earlier failure. */
size_t dpvo_ba_workspace_bytes_ex(int64_t num_edges, int64_t num_patches, int num_opt_poses, int flags);
int dpvo_ba_forward_ex(float* poses, float* patches, int64_t num_patches, int P, const float* intrinsics,
                       const float* target, const float* weight, const float* lmbda, const int64_t* ii,
                       const int64_t* jj, const int64_t* kk, int64_t num_edges, int t0, int t1, int iterations,
                       int flags, void* workspace, size_t workspace_bytes, int* status, void* stream);

/* dpvo_ba_forward_ex with the caller's kk group-by (dpvo_group_by(kk): offs
 * [E+1], perm [E], groups [1], device): the deterministic path's patch CSR.
 * DPVO.update already groups kk for the update operator (SoftAgg over kk,
 * the temporal neighbours), so BA reuses it; NULLs build it here. */
int dpvo_ba_forward_csr(float* poses, float* patches, int64_t num_patches, int P, const float* intrinsics,
                        const float* target, const float* weight, const float* lmbda, const int64_t* ii,
                        const int64_t* jj, const int64_t* kk, int64_t num_edges, int t0, int t1, int iterations,
                        int flags, const int* csr_offs, const int* csr_perm, const int64_t* csr_groups,
                        void* workspace, size_t workspace_bytes, int* status, void* stream);

/* cuda_ba.reproject (ba_cuda.cu:368-418,543-575): coords [E][2][P][P]. */
int dpvo_reproject(const float* poses, const float* patches, int P, const float* intrinsics, const int64_t* ii,
                   const int64_t* jj, const int64_t* kk, int64_t num_edges, float* coords, void* stream);

/* cuda_ba.neighbors(ii, jj) (ba.cpp:113-158), on the device: for every edge
 * the previous / next edge of the same ii in stable jj order, -1 at ends. */
size_t dpvo_neighbors_workspace_bytes(int64_t num_edges);
int dpvo_neighbors(const int64_t* ii, const int64_t* jj, int64_t num_edges, int64_t* ix, int64_t* jx,
                   void* workspace, size_t workspace_bytes, void* stream);

/* cuda_ba.solve_system (ba.cpp:174-234), normal equations on the device:
 * J_i, J_j [r][7][7] float, ii, jj [r] int64, res [r][7] float ->
 * A = J^T J (m x m, fp64, row-major) and b = -J^T res (fp64), with
 * diag(A) <- diag(A) (1 + lm) + ep; rows/columns >= m are dropped (m = 7n,
 * or 7 * freen for the reference's top-left solve).  *status = 1 when an
 * edge has ii == jj (the reference exits the process there).  The factor /
 * solve is a dense fp64 Cholesky (the shim uses rocSOLVER through torch). */
int dpvo_solve_system_assemble(const float* J_i, const float* J_j, const int64_t* ii, const int64_t* jj,
                               const float* res, int64_t r, int64_t m, float ep, float lm, double* A, double* b,
                               int* status, void* stream);

/* ------------------------------------------------------------------------
 * lietorch -- replaces lietorch_backends (reference lietorch.cpp:286-316)
 * group: 1 = SO3, 3 = SE3 (dispatch.h:16-31); dtype F32 or F64.
 * All arrays are flat [n][dim] contiguous (already broadcast).
 * --------------------------------------------------------------------- */
enum {
    DPVO_LIE_EXP = 0, DPVO_LIE_LOG, DPVO_LIE_INV, DPVO_LIE_MUL, DPVO_LIE_ADJ, DPVO_LIE_ADJT,
    DPVO_LIE_ACT, DPVO_LIE_ACT4, DPVO_LIE_MATRIX, DPVO_LIE_PROJECTOR, DPVO_LIE_JINV
};
/* forward: out = op(X[, Y]) -- expm, logm, inv, mul, adj, adjT, act, act4,
 * as_matrix, projector, Jinv (lietorch_gpu.cu:21-296). */
int dpvo_lie_forward(int op, int group, int dtype, const void* X, const void* Y, void* out, int64_t n,
                     void* stream);
/* backward of expm/logm/inv/mul/adj/adjT/act/act4: dX (and dY for binary
 * ops), caller-allocated and zero-filled with the shapes the reference
 * returns (lietorch_gpu.cu:298-601). */
int dpvo_lie_backward(int op, int group, int dtype, const void* grad, const void* X, const void* Y, void* dX,
                      void* dY, int64_t n, void* stream);

/* DPVO.__call__'s DAMPED_LINEAR motion model (dpvo.py:816-825) in one launch:
 * poses[n] = Exp(s * Log(poses[n-1] * poses[n-2]^-1)) * poses[n-1], SE3 rows
 * [t, q] fp32, s = MOTION_DAMPING * dt ratio (n >= 2). */
int dpvo_pose_extrapolate(float* poses, int64_t n, float s, void* stream);
/* out = a * b^-1 for single SE3 rows (keyframe()'s dP, dpvo.py:613). */
int dpvo_pose_relative(const float* a, const float* b, float* out, void* stream);

/* ------------------------------------------------------------------------
 * projective ops -- fused forms of dpvo/projective_ops.py
 * --------------------------------------------------------------------- */
enum { DPVO_TF_DEPTH = 1, DPVO_TF_TONLY = 2, DPVO_TF_CHW = 4 };
/* projective_ops.transform (projective_ops.py:53-68): per edge
 * Gij = poses[jj] * poses[ii]^-1, X1 = Gij * iproj(patches[kk], K[ii]),
 * x = K[jj] proj(X1) with Z clamped to >= 0.1.
 * coords: [E][P][P][2|3] (default) or [E][2|3][P][P] (DPVO_TF_CHW);
 * valid (optional) [E][P][P] float = (Z > 0.2). */
int dpvo_transform(const float* poses, const float* patches, int P, const float* intrinsics, const int64_t* ii,
                   const int64_t* jj, const int64_t* kk, int64_t num_edges, int flags, float* coords, float* valid,
                   void* stream);

/* DPVO.motionmag (dpvo.py:507-514) of both directions keyframe() compares
 * (dpvo.py:609): out[0] = mean flow_mag (projective_ops.py:111-121, weight
 * beta) over the edges with (ii, jj) == (i, j) and their P*P pixels,
 * out[1] = the same for (j, i); NaN for a direction without edges.  out is a
 * 2-float device buffer; no host synchronisation. */
int dpvo_motion_mag(const float* poses, const float* patches, int P, const float* intrinsics, const int64_t* ii,
                    const int64_t* jj, const int64_t* kk, int64_t num_edges, int64_t i, int64_t j, float beta,
                    float* out, void* stream);
/* The same over many workgroups (a caller-provided workspace of
 * dpvo_motion_mag_workspace_bytes for the per-workgroup partials, summed in a
 * fixed order by a second launch). */
size_t dpvo_motion_mag_workspace_bytes(int64_t num_edges);
int dpvo_motion_mag_ws(const float* poses, const float* patches, int P, const float* intrinsics, const int64_t* ii,
                       const int64_t* jj, const int64_t* kk, int64_t num_edges, int64_t i, int64_t j, float beta,
                       float* out, void* workspace, size_t workspace_bytes, void* stream);

/* Keyframe distance matrix of the global BA's distance-based edges
 * (replaces the O(n^2) loop of dpvo.py:383-429 -- two flow_mag calls and one
 * .item() per frame pair): dist [n][n] (device), dist[a][b] = mean over frame
 * a's patches [M a, M (a + 1)) and their P*P pixels of flow_mag(a -> b)
 * (projective_ops.py:111-121, weight beta).  The reference's distance of the
 * pair (i, j) is 0.5 (dist[i][j] + dist[j][i]).  M 6 P^2 floats must fit in
 * LDS (dpvo_keyframe_flow_lds_bytes). */
size_t dpvo_keyframe_flow_lds_bytes(int P, int64_t patches_per_frame);
int dpvo_keyframe_flow(const float* poses, const float* patches, int P, const float* intrinsics, int64_t num_frames,
                       int64_t patches_per_frame, float beta, float* dist, void* stream);

/* projective_ops.point_cloud (projective_ops.py:106-108) of patches[0..m):
 * centre_only=1 -> out [m][3] = xyz/w of the centre pixel (what
 * DPVO.update stores in pg.points_, dpvo.py:747-749); else out [m][P][P][4]. */
int dpvo_point_cloud(const float* poses, const float* patches, int P, const float* intrinsics, const int64_t* ix,
                     int64_t m, int centre_only, float* out, void* stream);

/* ------------------------------------------------------------------------
 * update-operator glue -- replaces torch_scatter 2.1.2 (scatter_softmax +
 * scatter_sum in SoftAgg, reference dpvo/blocks.py:40-48) and the masked
 * neighbour gather of Update.forward (dpvo/net.py:81-86).  Not part of the
 * reference's FFI (torch_scatter is a pip dependency); the dpvo/blocks.py
 * and dpvo/net.py mirrors call them through dpvo_hot.
 * --------------------------------------------------------------------- */

/* SoftAgg core: for every group g in [0,G) and channel d < D
 *   y[g][d] = sum_{e: group[e]==g} f[e][d] * w[e][d],
 *   w[e][d] = exp(s[e][d] - max_g s[.][d]) / (sum_g exp(s[.][d] - max) + eps)
 * (torch_scatter.scatter_softmax then scatter_sum over dim 1), accumulated
 * in fp32 over each group's edges in ascending edge order (deterministic for
 * groups of up to DPVO_SOFTAGG_SORT_CAP edges; larger groups use arrival
 * order).  f rows at f + e*ldf, s rows at s + e*lds (so one fused [E][2D]
 * GEMM output can feed both); y contiguous [G][D] of `dtype`.  Group labels
 * are torch.unique's inverse, in [0,G); edges with labels outside are
 * ignored; an empty group yields 0. */
#define DPVO_SOFTAGG_SORT_CAP 1024
size_t dpvo_softagg_workspace_bytes(int64_t num_edges, int64_t groups);
int dpvo_softagg_forward(int dtype, const void* f, int64_t ldf, const void* s, int64_t lds, const int64_t* group,
                         int64_t num_edges, int D, int64_t groups, float eps, void* y, void* workspace,
                         size_t workspace_bytes, void* stream);

/* Sync-free group-by: torch.unique(key, return_inverse=True) plus the CSR of
 * the groups, without a host round trip.  gid[e] = rank of key[e] among the
 * distinct keys (ascending, = torch.unique's inverse); group g's edges are
 * perm[offs[g] .. offs[g+1]) in ascending edge order; *groups (device int64)
 * = number of distinct keys.  Keys must lie in [0, 2^key_bits) when
 * key_bits <= 32 (a 32-bit radix sort over key_bits bits); key_bits in 33..64
 * sorts the full 64-bit key (any int64; gid order is then unsigned order).
 * offs has n+1 entries, perm n.  With key_bits <= 22 and a workspace of
 * dpvo_group_by_workspace_bytes_for(n, key_bits) bytes the group-by runs as a
 * counting sort over 2^key_bits bins (5 launches, same outputs); a workspace of
 * dpvo_group_by_workspace_bytes(n) bytes always takes the radix-sort path. */
size_t dpvo_group_by_workspace_bytes(int64_t n);
size_t dpvo_group_by_workspace_bytes_for(int64_t n, int key_bits);
int dpvo_group_by(const int64_t* key, int64_t n, int key_bits, int64_t* gid, int* offs, int* perm, int64_t* groups,
                  void* workspace, size_t workspace_bytes, void* stream);

/* cuda_ba.neighbors(kk, jj) (ba.cpp:113-158) over the CSR of dpvo_group_by(kk):
 * within each group, the previous / next edge in (jj, edge) order, -1 at the
 * ends -- the same result as dpvo_neighbors without its 64-bit radix sort.
 * ix, jx [num_edges] int64; *groups read on the device (<= max_groups). */
int dpvo_neighbors_csr(const int64_t* jj, const int* offs, const int* perm, const int64_t* groups,
                       int64_t max_groups, int64_t num_edges, int64_t* ix, int64_t* jx, void* stream);

/* dpvo_softagg_forward over a CSR from dpvo_group_by; the group count is read
 * from device memory (*groups <= max_groups); y rows >= *groups are untouched.
 * Sums run in ascending edge order: deterministic for every group size. */
int dpvo_softagg_csr(int dtype, const void* f, int64_t ldf, const void* s, int64_t lds, const int* offs,
                     const int* perm, const int64_t* groups, int64_t max_groups, int D, float eps, void* y,
                     void* stream);
/* dpvo_softagg_csr for a few long groups (the update operator's frame-pair
 * SoftAgg, ~190 edges per group at C3): groups of >= 64 edges are split over
 * four waves whose online-softmax states are merged in a fixed order
 * (deterministic; not bit-identical to dpvo_softagg_csr for those groups,
 * identical for shorter ones).  fp16 or fp32. */
int dpvo_softagg_csr_long(int dtype, const void* f, int64_t ldf, const void* s, int64_t lds, const int* offs,
                          const int* perm, const int64_t* groups, int64_t max_groups, int D, float eps, void* y,
                          void* stream);

/* torch_scatter 2.1.2 over the CSR of dpvo_group_by(index) -- replaces the
 * third-party scatter_sum / scatter_mean / scatter_max / scatter_softmax the
 * reference calls (blocks.py:42-43, ba.py:40-56, long_term.py:134).
 * src: [outer][E][inner] contiguous (scatter dim in the middle), index [E]
 * int64 (1-D along the scatter dim).  op:
 *   0 sum     out[o][index[e]][c] += sum over e           (out [outer][out_rows][inner])
 *   1 mean    out[o][k][c] = (out + sum) / count           (keys with members)
 *   2 max     out[o][k][c] = max, argmax[o][k][c] = e      (first maximum in edge order)
 *   3 softmax out[o][e][c] = exp(src - gmax) / (gsum + eps) (out shaped like src)
 * Rows of out whose key has no members are not written (the caller fills them:
 * zeros, and argmax = E, as torch_scatter does).  Keys outside [0, out_rows)
 * are skipped.  Sums run in fp32 (fp64 for fp64) in ascending edge order:
 * deterministic.  dtype DPVO_F16 / F32 / F64. */
int dpvo_scatter_csr(int op, int dtype, const void* src, int64_t outer, int64_t E, int64_t inner, const int64_t* index,
                     const int* offs, const int* perm, const int64_t* groups, int64_t max_groups, float eps, void* out,
                     int64_t out_rows, int64_t* argmax, void* stream);

/* Full-row fused GEMM of the update operator (dpvo/net.py:75-93 and
 * blocks.py GatedResidual under autocast), N = 384 output columns per row:
 *   y16  = fp16(A W^T + bias)            A fp16 [M][K] rows at A + r*lda, or
 *                                        gathered rows A + a_idx[m]*lda
 *                                        (a_idx[m] < 0 -> zero_row);
 *                                        W fp16 [384][K]; bias fp16 [384]
 *   RELU / SIGMOID on y16 (fp16 result, as ATen's half kernels)
 *   RES : v = res32[m] (+ res16[res16_idx[m]]) + y   (fp32; res16 rows of 384)
 *   GATE: v = res32[m] + fp16(gate16[m] * y)         (GatedResidual, blocks.py:31)
 *   LN  : v = LayerNorm(v; ln_g, ln_b, ln_eps) in fp32 [LN_RELU: relu(v)]
 *   HEADS: head_out[m] = fp16 {W_d relu(v) + b_d (2), sigmoid(W_w relu(v) + b_w) (2)}
 *          with head_w fp16 [4][384], head_b fp16 [4]   (net.py:63-72)
 *   out32[m] = v (fp32, row stride ldo32) and/or out16[m] = fp16(v) (ldo16).
 * K must be a multiple of 64 (pad W with zero columns; A's pad columns must
 * be finite); A, W, zero_row 16-byte aligned; zero_row holds >= K zeros.
 * Supported flag sets: 0, RELU, SIGMOID, LN|LN_RELU, RES, RES|LN, GATE,
 * GATE|LN, GATE|HEADS; and WKB, WKB|RELU, WKB|SIGMOID (k-blocked W, K a
 * multiple of 64 as well: the kernel's one barrier per two k-steps must fall
 * between one tile's y-tile reads and the next tile's writes). */
enum {
    DPVO_RG_RELU = 1, DPVO_RG_SIGMOID = 2, DPVO_RG_RES = 4, DPVO_RG_GATE = 8, DPVO_RG_LN = 16, DPVO_RG_LN_RELU = 32,
    DPVO_RG_HEADS = 64,
    /* W is k-blocked, [K/32][384][32] (as dpvo_rowchain reads it); with flag
     * sets 0 / RELU / SIGMOID only (and in both args of dpvo_rowgemm_pair) */
    DPVO_RG_WKB = 128
};
typedef struct dpvo_rowgemm_args {
    const void* A; int64_t lda; const int64_t* a_idx; int64_t a_rows;
    const void* W; int K; int N; const void* bias; const void* zero_row;
    int64_t M;
    const void* res32; int64_t ldr; const void* res16; const int64_t* res16_idx;
    const void* gate16;
    const float* ln_g; const float* ln_b; float ln_eps;
    const void* head_w; const void* head_b; void* head_out;
    void* out32; int64_t ldo32; void* out16; int64_t ldo16;
    int flags;
    const int64_t* M_dev;   /* optional: row count read on the device (M is then the upper bound) */
} dpvo_rowgemm_args;
int dpvo_rowgemm(const dpvo_rowgemm_args* args, void* stream);

/* Two plain rowgemms (flags 0) on the same A in one launch: SoftAgg's f and g
 * Linears (blocks.py:33-37 -- agg.f(x), agg.g(x)).  a and b must agree on A,
 * lda, a_idx, a_rows, K, M and M_dev; each has its own W, bias and outputs.
 * Every 128-row tile of A is multiplied by a's W then b's W back to back (the
 * second pass re-reads the tile; at C3 the counters see it come back through
 * the memory side, not from L2). */
int dpvo_rowgemm_pair(const dpvo_rowgemm_args* a, const dpvo_rowgemm_args* b, void* stream);

/* Two chained rowgemms, Y = epi2(act1(A W1^T + b1) W2^T + b2), with the 384-wide
 * intermediate kept on chip (the update operator's Linear -> ReLU -> Linear
 * pairs).  g1: A, lda, a_idx, a_rows, W (K1 % 64 == 0), bias, zero_row, M,
 * M_dev and flags (DPVO_RG_RELU / DPVO_RG_SIGMOID only); its outputs are not
 * written.  g2: W ([384][384]), bias, flags and every epilogue input / output
 * of dpvo_rowgemm (its A, M and M_dev are taken from g1).
 * The chain kernels read every W (W1, W2, and the gate / middle W below)
 * K-BLOCKED: [K/32][384][32] fp16 (k-stage major), so each 32-wide stage of
 * all 384 output rows is one contiguous block and the stage loads read whole
 * 128-B lines (update_ops.kblock re-lays out a [384][K] weight). */
int dpvo_rowchain(const dpvo_rowgemm_args* first, const dpvo_rowgemm_args* second, void* stream);

/* Three chained rowgemms: the update operator's corr MLP and the first
 * LayerNorm (net.py:54-61,78-79) in one launch,
 *   h1 = act1(A W1^T + b1);  h2 = fp16(relu(LN2(fp16(h1 W2^T + b2))));
 *   Y  = epi3(h2 W3^T + b3)
 * with h1 and h2 kept on chip.  first: as dpvo_rowchain's; middle: W, bias,
 * flags == DPVO_RG_LN | DPVO_RG_LN_RELU and ln_g / ln_b / ln_eps; last: W,
 * bias, flags == DPVO_RG_RES | DPVO_RG_LN and every epilogue input / output
 * of dpvo_rowgemm.  Bit-identical to dpvo_rowchain(first, middle) writing
 * fp16 rows followed by dpvo_rowgemm(those rows, last). */
int dpvo_rowchain3(const dpvo_rowgemm_args* first, const dpvo_rowgemm_args* middle, const dpvo_rowgemm_args* last,
                   void* stream);

/* The GRU's GatedResidual (blocks.py:27-30) in one launch:
 *   gate = sigmoid(fp16(A Wg^T + bg)),  Y = epi2(act1(A W1^T + b1) W2^T + b2)
 * with second->flags including DPVO_RG_GATE (GATE|LN or GATE|HEADS) and
 * second->gate16 == NULL: the gate never leaves the chip.  gate: W ([384][K1],
 * like first's W) and bias only.  Same results as dpvo_rowgemm(A, Wg, bg,
 * DPVO_RG_SIGMOID) -> gate16 followed by dpvo_rowchain. */
int dpvo_rowchain_gated(const dpvo_rowgemm_args* gate, const dpvo_rowgemm_args* first,
                        const dpvo_rowgemm_args* second, void* stream);

/* Row add + LayerNorm over 384-wide rows (one pass):
 *   v = (a[m] (+ b16[b_idx[m]])) (+ c16[c_idx[m]])  [-> LayerNorm]  -> out32 [M][384] / out16 [M][384]
 * a is fp16 (a_f16=1) or fp32 with row stride lda (a multiple of 4); b_idx[m] < 0
 * (c_idx[m] < 0) adds nothing; c16 needs b16.  Vector access: a, out32, ln_g /
 * ln_b 16-byte aligned (a 8-byte when fp16), b16, c16 and out16 8-byte aligned.
 * Used for `net + h(y)[:, jx]` after SoftAgg and the GRU's first LayerNorm: the
 * agg_kk add writes out16 only, the agg_ij add passes both SoftAggs' rows
 * (b16 = agg_kk's, c16 = agg_ij's) -- the same fp32 adds in the same order. */
typedef struct dpvo_rowadd_args {
    const void* a; int a_f16; int64_t lda; int64_t M;
    const void* b16; const int64_t* b_idx; int64_t b_rows;
    const float* ln_g; const float* ln_b; float ln_eps;
    void* out32; void* out16;
    const void* c16; const int64_t* c_idx; int64_t c_rows;   /* optional second gathered addend */
} dpvo_rowadd_args;
int dpvo_rowadd_ln(const dpvo_rowadd_args* args, void* stream);

/* dpvo_rowgemm_pair whose A rows are formed as they are staged:
 * A[m] = fp16(pre->a[m] + pre->b16[pre->b_idx[m]]) (fp32 rows a, lda >= 384;
 * the fp16 addend rows gathered, b_idx out of [0, b_rows) = no addend), which
 * is dpvo_rowadd_ln(pre with out16)'s arithmetic: the agg_kk row add
 * (net.py:87) feeding the agg_ij SoftAgg's f and g Linears (:88) without its
 * fp16 rows going through HBM.  a, b: WKB (k-blocked) with K = 384, no a_idx
 * (A is ignored); pre: a, lda, M (= a->M), b16, b_idx, b_rows only. */
int dpvo_rowgemm_pair_pre(const dpvo_rowgemm_args* a, const dpvo_rowgemm_args* b, const dpvo_rowadd_args* pre,
                          void* stream);

/* dpvo_rowchain_gated whose residual rows are not read from second->res32
 * but formed in the row epilogue: base = LayerNorm(pre->a + pre->b16[b_idx]
 * + pre->c16[c_idx]; pre->ln_g, ln_b, ln_eps) with dpvo_rowadd_ln's fp32
 * arithmetic in its order -- the first GRU's `norm(net + agg_kk + agg_ij)`
 * residual (net.py:90-92) without rowadd_ln's fp32 output rows: bit-identical
 * to dpvo_rowadd_ln(pre with out32) followed by dpvo_rowchain_gated with
 * res32 = those rows.  second: flags DPVO_RG_GATE | DPVO_RG_LN, res32 and
 * res16 NULL; first: a ReLU first GEMM; pre: fp32 a (lda >= 384, 16-byte
 * aligned), M = first->M (no M_dev), ln_g / ln_b required, out32 / out16
 * ignored. */
int dpvo_rowchain_gated_pre(const dpvo_rowgemm_args* gate, const dpvo_rowgemm_args* first,
                            const dpvo_rowgemm_args* second, const dpvo_rowadd_args* pre, void* stream);

/* The tracker's per-update edge keys in one launch (DPVO.update / DPVO.corr,
 * dpvo.py:326-327,718 and the SoftAgg group keys of net.py:86-88):
 * key_kk[e] = kk[e] - M base, key_ij[e] = (ii[e] - base) * 64 + (jj[e] - base),
 * ctx[e] = kk[e] mod ring, jslot[e] = jj[e] mod frames.  All int64 [E].
 * flag (optional int32): set to -2 if still 0 when an edge falls outside the
 * window (ii - base, jj - base not in [0, 64) or key_kk not in [0, 64 M)). */
int dpvo_window_keys(const int64_t* ii, const int64_t* jj, const int64_t* kk, int64_t E, int64_t M, int64_t base,
                     int64_t ring, int64_t frames, int64_t* key_kk, int64_t* key_ij, int64_t* ctx, int64_t* jslot,
                     int* flag, void* stream);

/* dpvo_window_keys followed by dpvo_group_by(key_kk, kk_bits) and
 * dpvo_group_by(key_ij, 12) (DPVO.update's per-update grouping: the SoftAgg
 * groups of net.py:86-88 and BA's per-patch CSR), fused into one memset and
 * four launches.  Writes ctx, jslot and flag as dpvo_window_keys does (the
 * key arrays are not written out) and the two CSRs exactly as dpvo_group_by
 * would: gid int64 [E], offs int32 [E + 1], perm int32 [E], groups int64 [1].
 * kk_bits: 1..22, with 64 M <= 2^kk_bits for in-window keys.  jj_order
 * (optional int32 [E]): the edges grouped by target frame (jj - base, in
 * ascending jj; any order within a frame) -- the visiting order of
 * dpvo_corr_pyramid_mfma, as dpvo_edge_order would give it by ring slot.
 * workspace: at least dpvo_window_group_by_workspace_bytes(E, kk_bits) device
 * bytes (0 for a bad kk_bits). */
size_t dpvo_window_group_by_workspace_bytes(int64_t E, int kk_bits);
int dpvo_window_group_by(const int64_t* ii, const int64_t* jj, const int64_t* kk, int64_t E, int64_t M, int64_t base,
                         int64_t ring, int64_t frames, int kk_bits, int64_t* ctx, int64_t* jslot, int* flag,
                         int64_t* kk_gid, int* kk_offs, int* kk_perm, int64_t* kk_groups, int64_t* ij_gid,
                         int* ij_offs, int* ij_perm, int64_t* ij_groups, int* jj_order, void* workspace, size_t workspace_bytes,
                         void* stream);

/* DPVO.__call__'s edge append (dpvo.py:756-769,799-800) in one launch:
 * out = [old edges; forward edges (patches of frames [n-r, n-1) -> frame n-1);
 * backward edges (frame n-1's patches -> frames [n-r, n), patch-major)], with
 * ii = ix[kk]; n = frame count after the new frame, r = PATCH_LIFETIME.
 * Outputs hold E + dpvo_append_edges_count(n, M, r) int64 entries. */
int64_t dpvo_append_edges_count(int64_t n, int64_t M, int64_t r);
int dpvo_append_edges(const int64_t* ii, const int64_t* jj, const int64_t* kk, int64_t E, const int64_t* ix, int64_t n,
                      int64_t M, int64_t r, int64_t* ii_out, int64_t* jj_out, int64_t* kk_out, void* stream);

/* DPVO.update after the update operator (dpvo.py:724-727): target[e] =
 * centre[e] + float(delta[e]), weight[e] = float(w[e]), both fp32 [E][2]
 * contiguous.  delta, w: fp16, row e at delta + e * delta_stride (2 values);
 * centre: fp32, x at centre + e * centre_stride, y at + centre_comp. */
int dpvo_edge_targets(const void* delta, int64_t delta_stride, const void* w, int64_t w_stride, const float* centre,
                      int64_t centre_stride, int64_t centre_comp, int64_t E, float* target, float* weight,
                      void* stream);

/* out[e][:] = idx[e] >= 0 ? x[idx[e]][:] : 0, converting in_dtype -> out_dtype
 * (the mask_ix * net[:, ix] of net.py:82-85; x rows at x + r*ldx, out
 * contiguous [n][D]). */
int dpvo_gather_rows(int in_dtype, const void* x, int64_t ldx, int64_t rows, const int64_t* idx, int64_t n, int D,
                     int out_dtype, void* out, void* stream);


/* ---------------------------------------------------------------------------
 * Frame ingest: the Patchifier's two BasicEncoder4 networks
 * (dpvo/extractor.py:200-264, ResidualBlock :6-53, called from net.py:121-122;
 * the reference runs them as ~100 cuDNN / ATen launches per frame).
 * Activations fp16 NHWC.  Each convolution reads x = xform(a, r), the previous
 * layer's output transformed on load:
 *   xmode 0: x = a;  1: x = relu(IN(a));  2: x = relu(relu(IN(a)) + IN'(r))
 * where IN(a) = (a - mean) * rstd over the Hi x Wi input pixels (instance
 * norm, affine-free), from a_st: the producing launch's per-tile partials
 * [a_st_tiles][a_st_ld] floats, (sum, sumsq) of channel c at 2 (a_co + c);
 * a_st NULL = no norm ('none').  IN'(r) likewise from r_st.  With part != NULL
 * the launch writes its own output's partials, part[tile][2 cout] -- the next
 * layer's a_st.  Every consumer reduces the partials itself, in a fixed order.
 * enc[0..n_enc): up to two encoders (fnet, inet) of the same layer shape in one
 * launch.  Weights fp16 [ks*ks][cin/32][cout][32] and the stem's
 * [5][32][32] (3 x 7 x 7 taps, zero-padded to 160), each 32-wide row's four
 * 8-value chunks XOR-swizzled by (row >> 2) & 3. */
typedef struct dpvo_conv_args {
    const void* a; int64_t a_ps; int a_co;   /* input: pixel stride, channel offset (elements) */
    const float* a_st; int a_st_tiles; int a_st_ld;
    const void* r; int64_t r_ps; int r_co;   /* residual (xmode 2) */
    const float* r_st; int r_st_tiles; int r_st_ld;
    void* xout; int64_t x_ps;                /* x itself, written (stride-1 3x3 only) or NULL */
    const void* w; const void* bias;         /* fp16 */
    void* out; int64_t o_ps; int o_co; float out_scale;   /* out = fp16(fp16(conv + bias) * out_scale) */
    float* part; float eps;
} dpvo_conv_args;
/* number of 8 x 16 output tiles (the part buffer's rows) of a layer */
int64_t dpvo_encoder_tiles(int Hi, int Wi, int ks, int stride);
/* conv1 (7x7 s2 p3, 3 -> 32) on the uint8 frame [3][H][W] with 2 (x / 255) - 0.5
 * (net.py:116) applied on load */
int dpvo_encoder_stem(const uint8_t* image, int H, int W, const dpvo_conv_args* enc, int n_enc, void* stream);
/* one layer: (ks, stride, cin -> cout) in {(3,1,32,32), (3,2,32,128: conv | 1x1
 * downsample as the centre tap), (3,1,64,64), (1,1,64,128)}, xmode per layer */
int dpvo_encoder_conv(int ks, int stride, int cin, int cout, int xmode, int Hi, int Wi, const dpvo_conv_args* enc,
                      int n_enc, void* stream);
/* the final 1x1 convolution (64 -> cout, xmode 2 input) at M pixels (x[m], y[m])
 * only: out[m * o_ps + o_co + c]; w fp16 [cout][64] */
int dpvo_encoder_head_at(const dpvo_conv_args* e, int cout, int Hi, int Wi, const int64_t* x, const int64_t* y,
                         int64_t M, void* stream);

/* The Patchifier's gathers at the M patch centres (x[m], y[m]) on the stride-4
 * map, one launch (net.py:301-315: four altcorr.patchify calls and the
 * coordinate grid, ~80 torch launches in the reference's composition):
 *   gmap    fp32 [M][128][3][3] = patchify(fmap, c, 1)
 *   imap    fp32 [M][dim]       = imap_at (fp16 [M][dim], head_at's rows)
 *   patches fp32 [M][3][3][3]   = patchify((x, y, 1) grid of the h x w map, c, 1)
 *   clr     fp32 [M][3]         = patchify(lut[image], 4 (c + 0.5), 0), or NULL
 * c = (float)(x, y).  patchify: the (2r+2)^2 window at floor(c) - r, zero
 * outside the map (correlation_kernel.cu:288-308), reduced bilinearly with
 * frac(c) in the order of correlation.py:51-69, fp32, no contraction.
 * fmap fp16 with element strides (channel, row, col); image uint8 [3][H][W];
 * lut: 256 floats, lut[v] = the frame normalisation 2 (v / 255) - 0.5 as the
 * caller computes it (net.py:116). */
int dpvo_patch_gather(const void* fmap, const int64_t* fmap_strides, int h, int w, const void* imap_at, int dim,
                      const uint8_t* image, int H, int W, const float* lut, const int64_t* x, const int64_t* y,
                      int64_t M, float* gmap, float* imap, float* patches, float* clr, void* stream);

/* keyframe() (dpvo.py:605-658): both outcomes' edge state before the decision,
 * and the decision's one host read.  For edge e, k the candidate frame:
 *   masks[0][e] = ix[kk] < n - RW (keep: edges retired, :654-658)
 *   masks[1][e] = ix[kk_d] < n - 1 - RW && !drop (drop: retired after the shift)
 *   masks[2][e] = masks[1][e] || drop,  drop = ii == k || jj == k (:616-617)
 *   idx[0..2][e] = ii_d, jj_d, kk_d: ii - (ii > k), jj - (jj > k), kk - M (ii > k)
 * masks uint8 [3][E], idx int64 [3][E]; vals double [7] = mm[0], mm[1] (the
 * motion magnitudes, dpvo_motion_mag_ws), ba_fail[0], any(isnan(pose_k[0..7))),
 * and the three masks' counts.  kk outside [0, ix_len) counts as not old. */
size_t dpvo_keyframe_masks_workspace_bytes(int64_t num_edges);
int dpvo_keyframe_masks(const int64_t* ii, const int64_t* jj, const int64_t* kk, int64_t num_edges,
                        const int64_t* ix, int64_t ix_len, int64_t k, int64_t M, int64_t n, int64_t RW,
                        const float* mm, const int* ba_fail, const float* pose_k, uint8_t* masks, int64_t* idx,
                        double* vals, void* workspace, size_t workspace_bytes, void* stream);

/* A keyframe drop's shift of frames k+1 .. n-1 down by one slot (dpvo.py:626-639)
 * in up to 16 per-frame buffers at once: buffer i holds frame f in slot
 * (rings[i] ? f % rings[i] : f) of slot_bytes[i] bytes at bases[i].  The same
 * result as moving the frames one after another, in ascending order. */
int dpvo_frame_shift(void* const* bases, const int64_t* slot_bytes, const int64_t* rings, int nseg, int64_t k,
                     int64_t n, void* stream);

/* remove_factors (dpvo.py:349-364) as one stable compaction: edges with
 * rm[e] == 0 go, in order, to the kept outputs (*_k); edges to store
 * (store_mode 0: none, 1: every removed edge, 2: store[e] != 0, a subset of
 * the removed ones) are written, in order, to the inactive outputs (*_s: the
 * tails of the inactive lists).  Fields: ii / jj / kk int64, weight / target
 * rows of wt_bytes, edge-state rows of row_bytes (a multiple of 16, 16-byte
 * aligned).  Two launches; the caller sizes the outputs (the counts ride on
 * keyframe()'s host read, dpvo_keyframe_masks). */
size_t dpvo_compact_edges_workspace_bytes(int64_t num_edges);
int dpvo_compact_edges(int64_t num_edges, const uint8_t* rm, const uint8_t* store, int store_mode, const int64_t* ii,
                       const int64_t* jj, const int64_t* kk, const void* weight, const void* target, int wt_bytes,
                       const void* net, int64_t row_bytes, int64_t* ii_k, int64_t* jj_k, int64_t* kk_k,
                       void* weight_k, void* target_k, void* net_k, int64_t* ii_s, int64_t* jj_s, int64_t* kk_s,
                       void* weight_s, void* target_s, void* workspace, size_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DPVO_HOT_H */
