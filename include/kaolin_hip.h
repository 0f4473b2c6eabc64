/* kaolin_hip.h -- C ABI of the MI355X (gfx950) hot-path library libkaolin_hip.so.
 *
 * Plain pointers + sizes, no torch types.  Every pointer argument is DEVICE memory
 * unless the name ends in `_host`.  `stream` is a hipStream_t (NULL = legacy default
 * stream).  All functions return 0 on success or a negative KL_E* code; the message
 * of the last failure on the calling thread is returned by kl_last_error().
 * Nothing in the library exits the process (the reference's CubDebugExit did,
 * mesh_to_spc_cuda.cu:22,50,347).
 *
 * Each entry point replaces one reference `kaolin._C` binding (bindings.cpp:37-99);
 * the reference dispatcher it stands in for is cited above the declaration.  Output
 * buffers are caller-allocated (the reference allocated them in C++ with at::zeros /
 * at::full; here the kernels write every element, so callers may pass
 * uninitialised memory).  Data-dependent outputs (mesh_to_spc, raytrace, voxel
 * subdivision) are allocated through a caller-supplied allocator callback so that
 * device memory comes from the caller's caching allocator.
 */
#ifndef KAOLIN_HIP_H_
#define KAOLIN_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  KL_F32 = 0,
  KL_F64 = 1,
  KL_F16 = 2,
  KL_U8 = 3,
  KL_I8 = 4,
  KL_I16 = 5,
  KL_I32 = 6,
  KL_I64 = 7
} kl_dtype;

enum {
  KL_OK = 0,
  KL_E_INVALID = -1,   /* bad argument / unsupported dtype */
  KL_E_HIP = -2,       /* HIP runtime error */
  KL_E_ALLOC = -3      /* allocator callback returned NULL */
};

typedef void *kl_stream;
/* Device allocator: returns `bytes` of device memory that stays valid until the
 * caller releases `ctx`'s allocations (after the call returns). */
typedef void *(*kl_alloc_fn)(void *ctx, size_t bytes);

/* ABI version of this header: a caller checks kl_abi_version() == KL_ABI_VERSION at load time.
 * 2: the workspace arguments moved before the stream (kl_rasterize_backward,
 *    kl_dibr_soft_mask_backward(_fused), kl_unbatched_triangle_distance_backward) and
 *    kl_soft_mask_compact_bwd_workspace_bytes gained num_faces.
 * 3: kl_dibr_forward / kl_dibr_backward take a state buffer of kl_dibr_state_bytes() bytes
 *    where they took one scratch int32 (the forward lists the backward's work items and zeroes
 *    its accumulator there); added kl_unbatched_triangle_distance_backward_sums; kl_loss_dot2's
 *    workspace holds its arrival ticket and must be ZERO before the first call (each call leaves
 *    it zero; an uninitialised one would never elect a last workgroup, and out[0] would not be
 *    written).
 * 4: kl_dibr_backward takes `soft_acc` (kl_dibr_soft_acc_bytes(): zero on entry, left zero on
 *    return) for the soft mask's per-face sums, which the forward's state no longer holds (the
 *    forward zeroes nothing per call); added kl_sided_distance_backward_sums. */
#define KL_ABI_VERSION 4

const char *kl_last_error(void);
int kl_abi_version(void);
/* 1 while `stream` is being captured into a HIP graph (a caller that keeps scratch across calls
 * gives a captured call its own buffer instead). */
int kl_stream_is_capturing(kl_stream stream);

/* Training-loop helper, not a reference op (bench.py's loss):
 *   out[0] = <a, ga> + <b, gb>   (fp32 inputs, fp64 accumulation, deterministic order).
 * ws: kl_loss_dot2_workspace_bytes() bytes, zeroed before the first call (each call leaves it
 * zeroed); one ws per stream in flight.  One launch (per-block partials, the last block adds them
 * in block order). */
size_t kl_loss_dot2_workspace_bytes(void);
int kl_loss_dot2(const float *a, const float *ga, int64_t na, const float *b, const float *gb, int64_t nb, void *ws,
                 float *out, kl_stream stream);

/* ---------------------------------------------------------------- DIB-R */

/* Workspace of packed_rasterize_forward: the per-pixel visibility buffer (13 B/px) and a
 * queue of large faces.  max_faces_per_mesh: upper bound on (first_idx[b+1] - first_idx[b]). */
size_t kl_rasterize_workspace_bytes(int batch, int height, int width, int64_t max_faces_per_mesh);

/* rasterization.cpp:49-104  packed_rasterize_forward_cuda.
 * face_vertices_z (Nv,3), face_vertices_image (Nv,3,2) (x multiplier), face_bboxes (Nv,4),
 * face_features (Nv,3,D), first_idx (B+1) int64 on device.
 * Outputs: interpolated_features (B,H,W,D), selected_face_idx (B,H,W) int64 (per-mesh
 * packed index, -1 = none), output_weights (B,H,W,3).  dtype: KL_F32 | KL_F64. */
int kl_packed_rasterize_forward(kl_dtype dtype, int height, int width, int batch, int64_t num_faces,
                                int feat_dim, int64_t max_faces_per_mesh,
                                const void *face_vertices_z, const void *face_vertices_image,
                                const void *face_bboxes, const void *face_features,
                                const int64_t *first_idx, float multiplier, float eps,
                                void *interpolated_features, int64_t *selected_face_idx,
                                void *output_weights, void *workspace, size_t workspace_bytes,
                                kl_stream stream);

/* rasterization.cpp:106-168  rasterize_backward_cuda.
 * face_idx: (B,H,W) ORIGINAL face index per mesh; face_vertices_image (B,F,3,2) unscaled.
 * Outputs (fully written): grad_face_vertices_image (B,F,3,2), grad_face_features (B,F,3,D).
 * The reference's per-pixel float terms are summed in double (workspace:
 * kl_rasterize_backward_workspace_bytes) and rounded once, so for f32 the result does not depend
 * on the order of the atomics (the reference's float atomics make it run-to-run
 * nondeterministic).  f64 terms are added with double atomics: rounded per add, order-dependent
 * in the last bits. */
size_t kl_rasterize_backward_workspace_bytes(int batch, int num_faces, int feat_dim);
int kl_rasterize_backward(kl_dtype dtype, int batch, int height, int width, int num_faces, int feat_dim,
                          const void *grad_interpolated_features, const int64_t *face_idx,
                          const void *output_weights, const void *face_vertices_image,
                          const void *face_features, float eps,
                          void *grad_face_vertices_image, void *grad_face_features,
                          void *workspace, size_t workspace_bytes, kl_stream stream);

/* Fused front-end path of rasterize() / RasterizeCuda (rasterization.py:290-388): takes the
 * UNPACKED (B,F) inputs and the optional (B,F) valid mask (uint8/bool) -- or, when it is
 * NULL, the optional (B,F) face_normals_z of dibr_rasterization, valid = face_normals_z >= 0
 * (dibr.py:195), evaluated in-kernel -- directly, applies
 * the multiplier and the bboxes in-kernel with the front-end's own float ops, and writes
 * the ORIGINAL per-mesh face index (what RasterizeCuda.forward returns after its remap).
 * face_vertices_image (B,F,3,2) unscaled; outputs as kl_packed_rasterize_forward. */
size_t kl_dibr_rasterize_workspace_bytes(int batch, int height, int width, int num_faces);
int kl_dibr_rasterize_forward(kl_dtype dtype, int height, int width, int batch, int num_faces, int feat_dim,
                              const void *face_vertices_z, const void *face_vertices_image,
                              const void *face_features, const uint8_t *valid_faces, const void *face_normals_z,
                              float multiplier, float eps,
                              void *interpolated_features, int64_t *face_idx, void *output_weights,
                              void *workspace, size_t workspace_bytes, kl_stream stream);
/* Atomic-free backward of the fused path: 8 lanes per face gather the pixels of the face's
 * exact pixel range (the reference's bbox test, same valid_faces / multiplier as the forward)
 * whose face_idx equals it, summing the reference's terms in double in a fixed lane order
 * (rounded once: deterministic for f32 and f64).  Requires face_idx produced by the fused forward with
 * the same valid_faces and multiplier.  Every face's gradient is written (zeros where it won no
 * pixel).  scratch: NULL, or a zeroed int32 the call uses as its big-face counter instead of
 * zeroing one in the workspace (kl_dibr_forward).  face_ranges: NULL, or kl_dibr_forward's
 * per-face ranges (then the ranges are not recomputed).  feat_dim > 8 takes the scatter path
 * of kl_rasterize_backward.  workspace: kl_dibr_rasterize_bwd_workspace_bytes. */
size_t kl_dibr_rasterize_bwd_workspace_bytes(int batch, int height, int width, int num_faces, int feat_dim);
int kl_dibr_rasterize_backward(kl_dtype dtype, int batch, int height, int width, int num_faces, int feat_dim,
                               const void *grad_interpolated_features, const int64_t *face_idx,
                               const void *output_weights, const void *face_vertices_image,
                               const void *face_features, const uint8_t *valid_faces, const void *face_normals_z,
                               float multiplier, float eps, void *grad_face_vertices_image,
                               void *grad_face_features, int *scratch, const uint32_t *face_ranges,
                               void *workspace, size_t workspace_bytes, kl_stream stream);

size_t kl_soft_mask_workspace_bytes(int batch, int height, int width, int num_faces);

/* dibr_soft_mask.cpp:48-108  dibr_soft_mask_forward_cuda.
 * face_vertices_image (B,F,3,2) and face_large_bboxes (B,F,4) already x multiplier.
 * Outputs (fully written): soft_mask (B,H,W), close_face_prob (B,H,W,K),
 * close_face_idx (B,H,W,K) int64 (-1 pad), close_face_dist_type (B,H,W,K) uint8 (0 pad). */
int kl_dibr_soft_mask_forward(kl_dtype dtype, int batch, int height, int width, int num_faces, int knum,
                              const void *face_vertices_image, const void *face_large_bboxes,
                              const int64_t *selected_face_idx, float sigmainv, float multiplier,
                              void *soft_mask, void *close_face_prob, int64_t *close_face_idx,
                              uint8_t *close_face_dist_type, void *workspace, size_t workspace_bytes,
                              kl_stream stream);

/* Fused front-end path of DibrSoftMaskCuda (dibr.py:27-73): face_vertices_image UNSCALED;
 * `face_vertices_image * multiplier` and the enlarged bboxes (min/max -/+ bbox_pad) are
 * evaluated in-kernel with the front-end's float ops.  bbox_pad = boxlen * multiplier as
 * the caller's double-precision product (the front-end's python-float expression).
 * hits (B,H,W) uint8, optional (NULL = not written; requires knum <= 255): the number of
 * filled slots per pixel, which lets the fused backward skip the slot scan. */
int kl_dibr_soft_mask_forward_fused(kl_dtype dtype, int batch, int height, int width, int num_faces, int knum,
                                    const void *face_vertices_image, const int64_t *selected_face_idx,
                                    float sigmainv, double bbox_pad, float multiplier, void *soft_mask,
                                    void *close_face_prob, int64_t *close_face_idx,
                                    uint8_t *close_face_dist_type, uint8_t *hits, void *workspace,
                                    size_t workspace_bytes, kl_stream stream);
/* hits: the forward's per-pixel slot counts, or NULL to scan the slots up to the first -1
 * as the reference does.  workspace: kl_soft_mask_backward_workspace_bytes (see
 * kl_dibr_soft_mask_backward). */
int kl_dibr_soft_mask_backward_fused(kl_dtype dtype, int batch, int height, int width, int num_faces, int knum,
                                     const void *grad_soft_mask, const void *soft_mask,
                                     const int64_t *selected_face_idx, const void *close_face_prob,
                                     const int64_t *close_face_idx, const uint8_t *close_face_dist_type,
                                     const uint8_t *hits, const void *face_vertices_image, float sigmainv,
                                     float multiplier, void *grad_face_vertices_image, void *workspace,
                                     size_t workspace_bytes, kl_stream stream);

/* Compact fused path of DibrSoftMaskCuda (dibr.py:27-73), the one the front-end runs
 * (knum <= 255).  The reference saves four (B,H,W,knum) slot tensors for its backward
 * (dibr.py:46-49); this path saves instead:
 *   hits     (B,H,W) uint8   the number of filled slots per pixel;
 *   rec_face, rec_prob       one record per filled slot: local face index | dist_type << 28
 *                            (uint32) and the slot's probability (tensor dtype); the records
 *                            of 64-pixel row segment s = (b*H + j) * ceil(W/64) + i/64 occupy
 *                            [s*64*knum, ...) in (pixel, slot) order
 *                            (kl_soft_mask_compact_records() elements to allocate; only the
 *                            filled slots are written);
 *   seg_tot  int32 per row segment (kl_soft_mask_compact_segments()): its number of records;
 *   scratch  one int32 the forward zeroes (see kl_dibr_forward).
 * face_vertices_image UNSCALED as in the _fused entry.  soft_mask equals
 * kl_dibr_soft_mask_forward's bit for bit. */
size_t kl_soft_mask_compact_workspace_bytes(int batch, int height, int width, int num_faces);
size_t kl_soft_mask_compact_records(int batch, int height, int width, int knum);
size_t kl_soft_mask_compact_segments(int batch, int height, int width);
int kl_dibr_soft_mask_forward_compact(kl_dtype dtype, int batch, int height, int width, int num_faces, int knum,
                                      const void *face_vertices_image, const int64_t *selected_face_idx,
                                      float sigmainv, double bbox_pad, float multiplier, void *soft_mask,
                                      uint8_t *hits, uint32_t *rec_face, void *rec_prob, int *seg_tot, int *scratch,
                                      void *workspace, size_t workspace_bytes, kl_stream stream);
/* dibr_soft_mask.cpp:110-183 on the compact state.  The terms are summed in double and
 * rounded once (order-independent for f32 terms, which sum exactly in double; f64 terms are
 * added with double atomics and may differ run to run in the last bits); accumulate = 0: grad_face_vertices_image is overwritten
 * with that sum; 1: the rounded sum is added onto its contents (one float add, as autograd
 * adds the soft-mask gradient to the rasterizer's).  scratch is left zeroed. */
size_t kl_soft_mask_compact_bwd_workspace_bytes(int batch, int height, int width, int num_faces, int knum);
int kl_dibr_soft_mask_backward_compact(kl_dtype dtype, int batch, int height, int width, int num_faces, int knum,
                                       const void *grad_soft_mask, const void *soft_mask, const uint8_t *hits,
                                       const uint32_t *rec_face, const void *rec_prob, const int *seg_tot,
                                       const void *face_vertices_image, float sigmainv, float multiplier,
                                       void *grad_face_vertices_image, int accumulate, int *scratch,
                                       void *workspace, size_t workspace_bytes, kl_stream stream);

/* dibr_rasterization (dibr.py:119-209) in one call per direction: rasterize with
 * valid_faces = face_normals_z >= 0 (evaluated in-kernel), then the compact soft mask on
 * its face index.  Outputs: interpolated_features (B,H,W,D), face_idx (B,H,W) int64,
 * output_weights (B,H,W,3), soft_mask (B,H,W), and the compact soft-mask state (hits,
 * rec_face, rec_prob, seg_tot as above, and `state`: kl_dibr_state_bytes() bytes, no
 * initialisation needed, in which the forward lists the backward's soft-mask work items).  The
 * backward writes grad_face_vertices_image / grad_face_features (every face): the soft-mask terms
 * are summed in double first into `soft_acc` (kl_dibr_soft_acc_bytes() bytes, ZERO on entry: per
 * face 8 doubles and a touched flag), then the gather writes each face's gradient as the rounded
 * sum of its own terms (double) plus the soft mask's rounded sum -- autograd's add of the two
 * gradients in the reference (grad_soft_mask may be NULL; soft_acc may then be NULL too).  The
 * gather reads, re-zeroes and unflags only the faces the soft half touched, so soft_acc is zero
 * again on return: a caller keeps one per stream and zeroes it once.  The state is left as the
 * forward left it, so a retained second backward is the same.
 * face_ranges: NULL, or (B*F) x 2 uint32 the forward fills with each face's exact pixel
 * ranges (x0 | x1 << 16, y0 | y1 << 16; empty for invalid faces) for the backward to reuse.
 * feat_dim <= 8.  Workspaces: kl_dibr_workspace_bytes (forward),
 * kl_dibr_bwd_workspace_bytes (backward). */
size_t kl_dibr_workspace_bytes(int batch, int height, int width, int num_faces);
size_t kl_dibr_bwd_workspace_bytes(int batch, int height, int width, int num_faces, int knum);
size_t kl_dibr_state_bytes(int batch, int height, int width, int num_faces, int knum);
size_t kl_dibr_soft_acc_bytes(int batch, int num_faces);
int kl_dibr_forward(kl_dtype dtype, int batch, int height, int width, int num_faces, int feat_dim, int knum,
                    const void *face_vertices_z, const void *face_vertices_image, const void *face_features,
                    const void *face_normals_z, float sigmainv, double bbox_pad, float multiplier, float eps,
                    void *interpolated_features, int64_t *face_idx, void *output_weights, void *soft_mask,
                    uint8_t *hits, uint32_t *rec_face, void *rec_prob, int *seg_tot, void *state,
                    uint32_t *face_ranges, void *workspace, size_t workspace_bytes, kl_stream stream);
int kl_dibr_backward(kl_dtype dtype, int batch, int height, int width, int num_faces, int feat_dim, int knum,
                     const void *grad_interpolated_features, const void *grad_soft_mask, const int64_t *face_idx,
                     const void *output_weights, const void *face_vertices_image, const void *face_features,
                     const void *face_normals_z, const void *soft_mask, const uint8_t *hits,
                     const uint32_t *rec_face, const void *rec_prob, const int *seg_tot, float sigmainv,
                     float multiplier, float eps, void *grad_face_vertices_image, void *grad_face_features,
                     void *state, const uint32_t *face_ranges, void *soft_acc, void *workspace,
                     size_t workspace_bytes, kl_stream stream);

/* dibr_soft_mask.cpp:110-183  dibr_soft_mask_backward_cuda.
 * Output grad_face_vertices_image (B,F,3,2) (fully written): the reference's per-hit float
 * terms summed in double (workspace: kl_soft_mask_backward_workspace_bytes) and rounded once,
 * independent of the order of the atomics. */
size_t kl_soft_mask_backward_workspace_bytes(int batch, int num_faces);
int kl_dibr_soft_mask_backward(kl_dtype dtype, int batch, int height, int width, int num_faces, int knum,
                               const void *grad_soft_mask, const void *soft_mask,
                               const int64_t *selected_face_idx, const void *close_face_prob,
                               const int64_t *close_face_idx, const uint8_t *close_face_dist_type,
                               const void *face_vertices_image, float sigmainv, float multiplier,
                               void *grad_face_vertices_image, void *workspace, size_t workspace_bytes,
                               kl_stream stream);

/* ------------------------------------------------------ DIB-R input preparation */

/* render/mesh/utils.py:128-175  prepare_vertices (+ camera/legacy.py:22-37 rotate_translate_points,
 * :120-139 perspective_camera, ops/mesh/mesh.py:25-46 index_vertices_by_faces,
 * ops/mesh/trianglemesh.py:313-336 face_normals(unit=True)) -- pure PyTorch in the reference,
 * one launch here.  vertices (Bv,V,3); faces (F,3) int64; camera_rot (Bc,3,3) + camera_trans
 * (Bc,3), or camera_transform (Bc,4,3) (then rot / trans NULL); camera_proj (Bp,3).  Bv, Bc, Bp
 * are 1 or B (broadcast as torch does).  Outputs face_vertices_camera (B,F,3,3),
 * face_vertices_image (B,F,3,2), face_normals (B,F,3).  f32 / f64.  A face index outside
 * [0, V) reads nothing and yields NaN for that face. */
int kl_prepare_vertices_forward(kl_dtype dtype, int B, int Bv, int Bc, int Bp, int64_t V, int64_t F,
                                const void *vertices, const int64_t *faces, const void *camera_rot,
                                const void *camera_trans, const void *camera_transform, const void *camera_proj,
                                void *face_vertices_camera, void *face_vertices_image, void *face_normals,
                                kl_stream stream);

/* Backward of the above (autograd's chain for the reference's ops; per-vertex and per-camera
 * sums in double, rounded once).  Any grad_face_* may be NULL (zero).  Outputs (NULL = not
 * wanted): grad_vertices (Bv,V,3); grad_camera (Bc,12): per camera rot (9, row-major) then
 * trans (3), or transform (4,3) row-major; grad_camera_proj (Bp,3).
 * ws: kl_prepare_vertices_bwd_workspace_bytes(B, V) bytes (zeroed by the call). */
size_t kl_prepare_vertices_bwd_workspace_bytes(int B, int64_t V);
int kl_prepare_vertices_backward(kl_dtype dtype, int B, int Bv, int Bc, int Bp, int64_t V, int64_t F,
                                 const void *vertices, const int64_t *faces, const void *camera_rot,
                                 const void *camera_trans, const void *camera_transform, const void *camera_proj,
                                 const void *grad_face_vertices_camera, const void *grad_face_vertices_image,
                                 const void *grad_face_normals, void *grad_vertices, void *grad_camera,
                                 void *grad_camera_proj, void *ws, size_t ws_bytes, kl_stream stream);

/* ------------------------------------------------------------ DefTet sparse render */

/* deftet.cpp:49-111  deftet_sparse_render_forward_cuda (kernel deftet_cuda.cu:32-190).
 * face_vertices_z (B,F,3), face_vertices_image (B,F,3,2), face_bboxes (B,F,4) [xmin ymin xmax ymax]
 * or NULL (then min / max over the three vertices in-kernel, as deftet.py:290-292 computes them),
 * pixel_coords (B,P,2), pixel_depth_ranges (B,P,2) [lo, hi).  dtype KL_F32 | KL_F64.
 * Outputs (B,P,K), fully written: face_idx int64 (first K hits in mesh order, then -1),
 * pixel_depths (-inf pad), w0, w1 (0 pad).  workspace: kl_deftet_workspace_bytes(B, F) bytes
 * (no initialisation needed).  With `alloc` the faces are binned into a screen grid of
 * mesh-ordered lists (their length is read back: one 8-byte device-to-host copy and a stream
 * synchronisation; the lists come from `alloc`); with NULL each workgroup walks the face tiles
 * that reach its pixels.  Both give the same outputs. */
size_t kl_deftet_workspace_bytes(int64_t batch_size, int64_t num_faces);
int kl_deftet_sparse_render_forward(kl_dtype dtype, int64_t batch_size, int64_t num_faces, int64_t num_pixels,
                                    int64_t knum, const void *face_vertices_z, const void *face_vertices_image,
                                    const void *face_bboxes, const void *pixel_coords,
                                    const void *pixel_depth_ranges, float eps, int64_t *face_idx,
                                    void *pixel_depths, void *w0, void *w1, void *workspace,
                                    size_t workspace_bytes, kl_alloc_fn alloc, void *alloc_ctx,
                                    kl_stream stream);

/* deftet.py:294-306 (the torch glue of DeftetSparseRenderer.forward) in one pass: per pixel the
 * hits of kl_deftet_sparse_render_forward ranked by depth, descending (stable), then
 * sorted_face_idx (B,P,K) int64, weights (B,P,K,3) = (w0, w1, 1 - (w0 + w1)) and
 * interpolated_features (B,P,K,D) = (w0 f0 + w1 f1) + w2 f2 from face_features (B,F,3,D). */
int kl_deftet_sparse_render_resolve(kl_dtype dtype, int64_t batch_size, int64_t num_faces, int64_t num_pixels,
                                    int64_t knum, int64_t feat_dim, const int64_t *face_idx,
                                    const void *pixel_depths, const void *w0, const void *w1,
                                    const void *face_features, int64_t *sorted_face_idx, void *weights,
                                    void *interpolated_features, kl_stream stream);

/* deftet.cpp:113-163  deftet_sparse_render_backward_cuda (kernel deftet_cuda.cu:240-420).
 * grad_interpolated_features (B,P,K,D), face_idx (B,P,K) int64, weights (B,P,K,3),
 * face_vertices_image (B,F,3,2), face_features (B,F,3,D) -> grad_face_vertices_image (B,F,3,2),
 * grad_face_features (B,F,3,D), fully written.  With a workspace of
 * kl_deftet_bwd_workspace_bytes(B, F, P, K) bytes the items are radix-sorted by face and each
 * face sums its items in item order (deterministic, no atomics); with NULL (or sizes past
 * 2^31 items) the reference's float atomics are used. */
size_t kl_deftet_bwd_workspace_bytes(int64_t batch_size, int64_t num_faces, int64_t num_pixels, int64_t knum);
int kl_deftet_sparse_render_backward(kl_dtype dtype, int64_t batch_size, int64_t num_faces, int64_t num_pixels,
                                     int64_t knum, int64_t feat_dim, const void *grad_interpolated_features,
                                     const int64_t *face_idx, const void *weights,
                                     const void *face_vertices_image, const void *face_features, float eps,
                                     void *grad_face_vertices_image, void *grad_face_features, void *workspace,
                                     size_t workspace_bytes, kl_stream stream);

/* ------------------------------------------------------------ distances */

/* unbatched_triangle_distance.cpp:43-72.  points (P,3), face_vertices (F,3,3).
 * Outputs dist (P), face_idx (P) int64, dist_type (P) int32. dtype KL_F32 | KL_F64.
 * workspace (optional, NULL allowed): kl_unbatched_triangle_distance_workspace_bytes(P, F)
 * bytes, used to process points in Hilbert order so that whole waves can skip faces
 * that provably cannot be their nearest, and to hold per-face records computed once per
 * call (results are unchanged). */
size_t kl_unbatched_triangle_distance_workspace_bytes(int64_t num_points, int64_t num_faces);
int kl_unbatched_triangle_distance_forward(kl_dtype dtype, int64_t num_points, int64_t num_faces,
                                           const void *points, const void *face_vertices,
                                           void *dist, int64_t *face_idx, int32_t *dist_type,
                                           void *workspace, size_t workspace_bytes, kl_stream stream);

/* unbatched_triangle_distance.cpp:74-114.  grad_points (P,3) fully written;
 * grad_face_vertices (F,3,3) fully written (zero where no point selected the face).
 * workspace: kl_unbatched_triangle_distance_bwd_workspace_bytes(F) bytes -- the per-point terms
 * are then summed per face coordinate in double and rounded once (deterministic for f32; f64
 * terms are added with double atomics, order-dependent in the last bits); NULL: the
 * reference's float atomics (order-dependent last bits). */
size_t kl_unbatched_triangle_distance_bwd_workspace_bytes(int64_t num_faces);
int kl_unbatched_triangle_distance_backward(kl_dtype dtype, int64_t num_points, int64_t num_faces,
                                            const void *grad_dist, const void *points,
                                            const void *face_vertices, const int64_t *face_idx,
                                            const int32_t *dist_type, void *grad_points,
                                            void *grad_face_vertices, void *workspace, size_t workspace_bytes,
                                            kl_stream stream);

/* The backward above for a sharded caller (not a reference op; kaolin/distributed.py): grad_points
 * (P,3) written; the face gradient's per-coordinate sums of the per-point float terms left in double,
 * gf_sums (F*9 doubles, zeroed here), NOT rounded -- the ranks' sums are all-reduced, then rounded
 * once, which gives the unsharded backward's gradient bit for bit (f32 terms sum exactly in double). */
int kl_unbatched_triangle_distance_backward_sums(kl_dtype dtype, int64_t num_points, int64_t num_faces,
                                                 const void *grad_dist, const void *points,
                                                 const void *face_vertices, const int64_t *face_idx,
                                                 const int32_t *dist_type, void *grad_points, double *gf_sums,
                                                 kl_stream stream);

/* sided_distance.cpp:65-89.  p1 (B,N,3), p2 (B,M,3) -> dist (B,N), idx (B,N) int64.
 * dtype: any kl_dtype (half/float/double and the integer types of DISPATCH_NUM_TYPES). */
int kl_sided_distance_forward(kl_dtype dtype, int batch, int64_t n, int64_t m,
                              const void *p1, const void *p2, void *dist, int64_t *idx,
                              kl_stream stream);

/* sided_distance.cpp:91-122.  grad_p1 (B,N,3), grad_p2 (B,M,3) fully written. */
int kl_sided_distance_backward(kl_dtype dtype, int batch, int64_t n, int64_t m,
                               const void *grad_dist, const void *p1, const void *p2,
                               const int64_t *idx, void *grad_p1, void *grad_p2, kl_stream stream);

/* sided_distance.cpp:91-122 with grad_p2 formed deterministically (float32 / float64 only):
 * grad_p1 (B,N,3) written; grad_p2's per-point float terms (sided_distance_cuda.cu's atomicAdd
 * operands) summed per coordinate in double into g2_sums (B,M,3) (zeroed here first), and, when
 * g2 != NULL, rounded once into g2 (B,M,3).  A caller that shards p1 all-reduces g2_sums and rounds
 * once (kaolin.distributed.sharded_sided_distance): the unsharded gradient bit for bit. */
int kl_sided_distance_backward_sums(kl_dtype dtype, int batch, int64_t n, int64_t m, const void *grad,
                                    const void *p1, const void *p2, const int64_t *idx, void *g1,
                                    double *g2_sums, void *g2, kl_stream stream);

/* ------------------------------------------------------------------ SPC */

/* mesh_to_spc.cpp:28-44 (mesh_to_spc_cuda_impl, mesh_to_spc_cuda.cu:309-463).
 * face_vertices (F,3,3) float32.  Outputs allocated through `alloc`:
 * *octree (num_nodes) u8, *face_idx (num_leaves) int64, *bary (num_leaves,2) f32.
 * Sizes returned in *num_nodes / *num_leaves (0 / 0 for an empty result). */
int kl_mesh_to_spc(int64_t num_faces, const float *face_vertices, uint32_t level,
                   kl_alloc_fn alloc, void *alloc_ctx,
                   uint8_t **octree, int64_t *num_nodes, int64_t **face_idx, float **bary,
                   int64_t *num_leaves, kl_stream stream);

/* Measurement helper, not a reference op: the number of (face, voxel) proposals tested at
 * each level 0..L by the last kl_mesh_to_spc call on the calling thread (N_0 = F).  Copies
 * min(capacity, L+1) counts and returns L+1 (0 before any call). */
int kl_mesh_to_spc_level_counts(int64_t *counts, int capacity);

/* Fixed-capacity mesh_to_spc (no reference counterpart: mesh_to_spc_cuda.cu:351-352,438 read the
 * counts back to size the outputs).  The same levels, every count on the device and nothing read
 * back, so the call can be captured into a HIP graph.  octree (node_capacity) u8, face_idx
 * (leaf_capacity) int64 and bary (leaf_capacity, 2) f32 are caller-allocated; result (3) int64
 * device output = (num_nodes, num_leaves, status): status 0 = written (octree bytes past num_nodes
 * are 0, face_idx rows past num_leaves -1, bary 0), 1 = num_nodes > node_capacity or num_leaves >
 * leaf_capacity (nothing written; the first two entries are the sizes needed), 2 = the workspace's
 * per-level pair buffers (96 per face) overflowed (nothing written: call kl_mesh_to_spc).
 * level in [1, 15); workspace of kl_mesh_to_spc_fixed_workspace_bytes(num_faces) bytes. */
size_t kl_mesh_to_spc_fixed_workspace_bytes(int64_t num_faces);
int kl_mesh_to_spc_fixed(int64_t num_faces, const float *face_vertices, uint32_t level, int64_t node_capacity,
                         int64_t leaf_capacity, uint8_t *octree, int64_t *face_idx, float *bary,
                         int64_t *result, void *workspace, size_t workspace_bytes, kl_stream stream);

/* spc.cpp:55-65 morton_to_octree: sorted unique leaf morton codes -> octree bytes. */
int kl_morton_to_octree(int64_t num_points, const uint64_t *morton, uint32_t level,
                        kl_alloc_fn alloc, void *alloc_ctx, uint8_t **octree, int64_t *num_nodes,
                        kl_stream stream);

/* point_utils.cpp:52-64 points_to_morton_cuda (caller ops/spc/points.py:105):
 * points (N,3) int16 -> morton (N) int64, bit 3i+2 = x_i, 3i+1 = y_i, 3i = z_i (spc_math.h:93-107). */
int kl_points_to_morton(int64_t num_points, const int16_t *points, int64_t *morton, kl_stream stream);

/* point_utils.cpp:36-50 morton_to_points_cuda (caller ops/spc/points.py:131):
 * morton (N) int64 -> points (N,3) int16 (spc_math.h:110-121). */
int kl_morton_to_points(int64_t num_points, const int64_t *morton, int16_t *points, kl_stream stream);

/* spc.cpp:79-107 scan_octrees_cuda.  lengths_host (B) int32 on the host.
 * exsum (sum(lengths) + B) int32 device output; pyramid_host (B,2,17) int32 host output
 * (zero-filled by the callee); returns the level through *level. */
int kl_scan_octrees(int batch, const uint8_t *octrees, const int32_t *lengths_host,
                    int32_t *exsum, int32_t *pyramid_host, int *level, kl_stream stream);

/* spc.cpp:109-134 generate_points_cuda.  pyramids_host (B,2,L+2) int32 host.
 * points: (sum_b pyramids[b,1,L+1], 3) int16 device output. */
int kl_generate_points(int batch, int max_level, const uint8_t *octrees, const int32_t *pyramids_host,
                       const int32_t *exsum, int16_t *points, kl_stream stream);

/* raytrace.cpp:170-214 raytrace_cuda (raytrace_cuda.cu:485-607).
 * Outputs allocated through `alloc`: *nuggets (N,2) int32, *depth (N, with_exit?2:1) f32. */
int kl_raytrace(const uint8_t *octree, int64_t octree_size, const int16_t *points, int64_t num_points,
                const int32_t *exsum, int max_level, const float *ray_o, const float *ray_d,
                int64_t num_rays, uint32_t target_level, int return_depth, int with_exit,
                kl_alloc_fn alloc, void *alloc_ctx, int32_t **nuggets, float **depth,
                int64_t *num_hits, kl_stream stream);

/* Fixed-capacity raytrace (no reference counterpart: raytrace_cuda.cu:557-560 reads each level's
 * count back to size the next).  The same levels with every count kept on the device: nothing is
 * read back, so the call can be captured into a HIP graph.  nuggets (capacity,2) int32 and depth
 * (capacity, with_exit?2:1) f32 are caller-allocated; result (2) int64 device output = (rows
 * written, 1 if some level held more than `capacity` candidates: the last level's nuggets, or an
 * earlier level's untested children, up to 8 per nugget of the level above).  When truncated, the rows are the
 * first rows of kl_raytrace's output (ray-major, front-to-back order is kept).  Rows past
 * result[0]: nugget (-1, -1), depth 0.  num_rays and capacity < 2^28. */
size_t kl_raytrace_fixed_workspace_bytes(int64_t num_rays, int64_t capacity, int with_exit);
int kl_raytrace_fixed(const uint8_t *octree, const int16_t *points, const int32_t *exsum,
                      const float *ray_o, const float *ray_d, int64_t num_rays, uint32_t target_level,
                      int return_depth, int with_exit, int64_t capacity, int32_t *nuggets, float *depth,
                      int64_t *result, void *workspace, size_t workspace_bytes, kl_stream stream);

/* raytrace.cpp:111-166 generate_primary_rays_cuda (deprecated upstream; bindings.cpp:86).
 * eye / at / up (3) and world (4x4 row-major) float on the host; ray_o, ray_d (height*width, 3)
 * f32 device outputs.  The reference's pixel of row t is (t % width, t / height). */
int kl_generate_primary_rays(uint32_t height, uint32_t width, const float *eye, const float *at,
                             const float *up, float fov, const float *world, float *ray_o, float *ray_d,
                             kl_stream stream);

/* raytrace.cpp:234-283 generate_shadow_rays_cuda (deprecated upstream; bindings.cpp:88).
 * ray_o, ray_d (num,3) f32 device; light (3) and plane (4) float on the host; src, dst (num,3)
 * f32 and map (num) int32 device outputs, of which the first *count rows are the answer
 * (*count on the host: one device-to-host read, as the reference's cudaMemcpy). */
size_t kl_generate_shadow_rays_workspace_bytes(int64_t num);
int kl_generate_shadow_rays(int64_t num, const float *ray_o, const float *ray_d, const float *light,
                            const float *plane, float *src, float *dst, int32_t *map, int64_t *count,
                            void *workspace, size_t workspace_bytes, kl_stream stream);

/* raytrace.cpp:216-240 mark_pack_boundaries_cuda: boundaries (N) int32 (1 at pack starts). */
int kl_mark_pack_boundaries(kl_dtype dtype, int64_t num, const void *pack_ids, int32_t *boundaries,
                            kl_stream stream);

/* Packed ray ops (render/spc/raytrace.py:86-296).  feats (num_feats, feat_dim) row-major in
 * f16 / f32 / f64; a pack is the run of rows [pack_indices[p], pack_indices[p+1]), the last
 * one ending at num_feats.  Rows before the first pack keep the reference's initial value
 * (0; 1 for cumprod), which these calls write.  Every output element is written. */

/* raytrace.cpp:285-309 diff_cuda (pack_indices int64): out[i] = feats[i+1] - feats[i]
 * inside a pack, 0 on a pack's last row. */
int kl_pack_diff(kl_dtype dtype, int64_t num_feats, int64_t feat_dim, const void *feats,
                 const int64_t *pack_indices, int64_t num_packs, void *out, kl_stream stream);

/* raytrace.cpp:354-377 cumsum_cuda / :380-402 cumprod_cuda (pack_indices int32), with the
 * reference kernels' exclusive / reverse semantics (raytrace_cuda.cu:391-483). */
int kl_pack_cumsum(kl_dtype dtype, int64_t num_feats, int64_t feat_dim, const void *feats,
                   const int32_t *pack_indices, int64_t num_packs, int exclusive, int reverse, void *out,
                   kl_stream stream);
int kl_pack_cumprod(kl_dtype dtype, int64_t num_feats, int64_t feat_dim, const void *feats,
                    const int32_t *pack_indices, int64_t num_packs, int exclusive, int reverse, void *out,
                    kl_stream stream);

/* raytrace.cpp:311-325 inclusive_sum_cuda: out = inclusive prefix sum of info (int32).
 * ws: kl_inclusive_sum_workspace_bytes(num) bytes of scratch. */
size_t kl_inclusive_sum_workspace_bytes(int64_t num);
int kl_inclusive_sum_i32(int64_t num, const int32_t *info, int32_t *out, void *ws, size_t ws_bytes,
                         kl_stream stream);

/* raytrace.cpp:328-351 sum_reduce_cuda: out (num_out, feat_dim), row r = the sum of the rows i
 * with inclusive_sum[i] == r + 1, added in row order (deterministic; the reference used
 * unordered atomics).  num_out = inclusive_sum[num_feats - 1] in the reference. */
int kl_sum_reduce(kl_dtype dtype, int64_t num_feats, int64_t feat_dim, const void *feats,
                  const int32_t *inclusive_sum, int64_t num_out, void *out, kl_stream stream);

/* ------------------------------------------------------------ check_sign */

/* mesh_intersection.cpp:33-68  unbatched_mesh_intersection_cuda (kernel
 * mesh_intersection_cuda.cu:100-210).  points (P,3), verts_1/2/3 (F,3) face corners, dtype
 * KL_F32 | KL_F64 -> result (P) in the same dtype: the number of faces the ray from each point
 * toward +x crosses (edge / vertex hits counted once).  Fully written.  workspace:
 * kl_check_sign_workspace_bytes(dtype, 1, F, P) bytes; `alloc` as for kl_check_sign below. */
int kl_unbatched_mesh_intersection(kl_dtype dtype, int64_t num_points, int64_t num_faces, const void *points,
                                   const void *verts_1, const void *verts_2, const void *verts_3, void *result,
                                   void *workspace, size_t workspace_bytes, kl_alloc_fn alloc, void *alloc_ctx,
                                   kl_stream stream);

/* check_sign (ops/mesh/check_sign.py:25-154) for a batch: verts (B,V,3), faces (F,3) int64,
 * points (B,P,3), maxlen (B) the per-mesh divisor check_sign.py:140-146 applies to verts and
 * points (NULL: computed here from verts as check_sign.py:140-146 does, exactly; V > 0)
 * -> contains (B,P) bool bytes (odd crossing count).  workspace:
 * kl_check_sign_workspace_bytes(dtype, B, F, P) bytes (no initialisation needed); the (y, z)
 * grid's face lists are allocated through `alloc` once their length is known (one 8-byte
 * device-to-host read and a stream synchronisation).  alloc == NULL: the capturable form --
 * nothing is read back; the lists use the workspace's fixed room, and when they do not fit
 * every point is tested against every face on the device (same answers, O(P F)); a face
 * index outside [0, V) is then clamped, not reported.  Same for kl_unbatched_mesh_intersection. */
size_t kl_check_sign_workspace_bytes(kl_dtype dtype, int64_t batch_size, int64_t num_faces, int64_t num_points);
int kl_check_sign(kl_dtype dtype, int64_t batch_size, int64_t num_vertices, int64_t num_faces, int64_t num_points,
                  const void *verts, const int64_t *faces, const void *points, const void *maxlen,
                  uint8_t *contains, void *workspace, size_t workspace_bytes, kl_alloc_fn alloc, void *alloc_ctx,
                  kl_stream stream);

/* ------------------------------------------------------------ voxelgrid */

/* trianglemeshes_to_voxelgrids (ops/conversions/trianglemesh.py:29-110) for ONE batch
 * element, float32.  points (V,3) are the already normalised vertices
 * ((v - origin) / scale); faces (F,3) int64.  Writes occupancy into grid (R,R,R) of
 * `grid_dtype` (KL_F32 | KL_F64 | KL_F16 | KL_U8); the grid must be zeroed by the caller. */
int kl_voxelgrid_mark(int64_t num_vertices, const float *points, int64_t num_faces, const int64_t *faces,
                      int resolution, kl_dtype grid_dtype, void *grid, kl_alloc_fn alloc, void *alloc_ctx,
                      kl_stream stream);

/* The default origin / scale of trianglemeshes_to_voxelgrids (trianglemesh.py:74-77) for B
 * meshes of V vertices (B,V,3): origin (B,3) = torch.min(vertices, dim=1), scale (B) =
 * torch.max(torch.max(vertices, dim=1) - origin, dim=1), exactly (NaN propagated per
 * coordinate).  f32 / f64.  ws: kl_voxelgrid_bounds_workspace_bytes(B) bytes. */
size_t kl_voxelgrid_bounds_workspace_bytes(int batch);
int kl_voxelgrid_bounds(kl_dtype dtype, int batch, int64_t num_vertices, const void *vertices, void *origin,
                        void *scale, void *workspace, size_t workspace_bytes, kl_stream stream);

/* Same for float64 vertices (the reference subdivides in the vertex dtype). */
int kl_voxelgrid_mark_f64(int64_t num_vertices, const double *points, int64_t num_faces, const int64_t *faces,
                          int resolution, kl_dtype grid_dtype, void *grid, kl_alloc_fn alloc, void *alloc_ctx,
                          kl_stream stream);

/* The same marking with nothing read back to the host, so the call can be captured into a HIP
 * graph (the reference, trianglemesh.py:339-457, sizes every round on the host; kl_voxelgrid_mark
 * reads one count per round).  point_dtype KL_F32 | KL_F64.  Subdivision levels run from two
 * device buffers of `capacity` triangles each; a level with more children to keep, or triangles
 * still needing a split after the levels launched (vertices outside the unit cube), finish their
 * subtree depth-first in the thread, so the grid equals kl_voxelgrid_mark's for any capacity >= 0
 * (capacity sets speed only).  *status (device u32, written by the call): bit 0 = some
 * depth-first walk exceeded 2^20 triangles and stopped (grid incomplete), bit 1 = some level
 * overflowed `capacity`, bit 2 = (r06: levels after the third run in one launch of co-resident
 * workgroups meeting at grid barriers) a barrier wait timed out (grid incomplete).  workspace: kl_voxelgrid_mark_async_workspace_bytes bytes. */
size_t kl_voxelgrid_mark_async_workspace_bytes(kl_dtype point_dtype, int64_t capacity);
int kl_voxelgrid_mark_async(kl_dtype point_dtype, int64_t num_vertices, const void *points, int64_t num_faces,
                            const int64_t *faces, int resolution, kl_dtype grid_dtype, void *grid, int64_t capacity,
                            uint32_t *status, void *workspace, size_t workspace_bytes, kl_stream stream);

/* (r06) One mesh of trianglemeshes_to_voxelgrids' GPU body as the front-end calls it: `vertices` (V,3)
 * as given (f32 / f64), normalised in the kernels as (v - origin[c]) / scale[0] (the front-end's
 * tensor subtraction and division, each rounded in the vertex dtype; origin (3) and scale (1) device
 * tensors of the vertex dtype), and `grid` written whole (zero-filled by the call: it need not be
 * zeroed).  Otherwise kl_voxelgrid_mark_async: the same grid, capacity, status (bit 2 in addition:
 * the persistent kernel of the later levels could not meet at a grid barrier -- grid incomplete) and
 * workspace (kl_voxelgrid_mark_async_workspace_bytes). */
int kl_voxelgrid_async(kl_dtype vertex_dtype, int64_t num_vertices, const void *vertices, const void *origin,
                       const void *scale, int64_t num_faces, const int64_t *faces, int resolution, kl_dtype grid_dtype,
                       void *grid, int64_t capacity, uint32_t *status, void *workspace, size_t workspace_bytes,
                       kl_stream stream);

/* texture_mapping (kaolin/render/mesh/utils.py:23-75): coords (B, N, 2) in [0, 1] (OpenGL, y up;
 * clamped), texture (B, C, TH, TW) -> out (B, N, C), as torch.nn.functional.grid_sample with
 * align_corners=False and padding_mode='border' after the reference's [-1, 1] / y mapping.
 * mode 0 = 'nearest', 1 = 'bilinear'.  Backward: grad_coords (B, N, 2) and/or grad_texture
 * (B, C, TH, TW) (either may be NULL); the texture terms are summed in double (workspace:
 * kl_texture_mapping_bwd_workspace_bytes) and rounded once; terms of a zero incoming gradient
 * are skipped (torch's grid_sample adds them with float atomics). */
int kl_texture_mapping_forward(kl_dtype dtype, int mode, int batch, int64_t num_points, int channels, int tex_height,
                               int tex_width, const void *coords, const void *texture, void *out, kl_stream stream);
size_t kl_texture_mapping_bwd_workspace_bytes(int batch, int channels, int tex_height, int tex_width);
int kl_texture_mapping_backward(kl_dtype dtype, int mode, int batch, int64_t num_points, int channels,
                                int tex_height, int tex_width, const void *grad_out, const void *coords,
                                const void *texture, void *grad_coords, void *grad_texture, void *workspace,
                                size_t workspace_bytes, kl_stream stream);

/* metrics/render.py:18-40 mask_iou (the DIB-R tutorial's silhouette loss), fused: lhs / rhs
 * (B, pixels_per_mask) of one dtype.  Outputs iou_up / iou_down (B) -- the two per-mask sums,
 * formed in the dtype as the reference forms them, summed in double in a fixed order and rounded
 * once -- and loss (1) = 1 - mean(up / (down + 1e-10)).  The backward writes autograd's gradient
 * through the reference's ops (grad_loss: a device scalar; grad_lhs / grad_rhs may be NULL). */
size_t kl_mask_iou_workspace_bytes(int batch, int64_t pixels_per_mask);
int kl_mask_iou_forward(kl_dtype dtype, int batch, int64_t pixels_per_mask, const void *lhs, const void *rhs,
                        void *iou_up, void *iou_down, void *loss, void *workspace, size_t workspace_bytes,
                        kl_stream stream);
int kl_mask_iou_backward(kl_dtype dtype, int batch, int64_t pixels_per_mask, const void *grad_loss, const void *lhs,
                         const void *rhs, const void *iou_up, const void *iou_down, void *grad_lhs, void *grad_rhs,
                         kl_stream stream);

#ifdef __cplusplus
}
#endif

#endif /* KAOLIN_HIP_H_ */
