/*
 * m3d.h -- C-ABI of libm3d.so, the MI355X-native (gfx950) replacement for the
 * native hot path of podtyazhki1337/3d-mask-r-cnn.
 *
 * Conventions
 *   - every pointer is a DEVICE pointer owned by the caller; nothing is
 *     allocated inside an entry point (workspaces are caller-provided);
 *   - every call is enqueued on the caller's stream `s` and never synchronises,
 *     so entry points are hipGraph-capturable;
 *   - tensors are channels-last exactly as the reference: images / feature
 *     maps [B,H,W,D,C] (depth = 3rd spatial dim, C innermost), boxes
 *     (y1,x1,z1,y2,x2,z2) normalised to [0,1], conv kernels Keras-ordered
 *     [kh,kw,kd,Cin,Cout];
 *   - return 0 (M3D_OK) on success, M3D_EINVAL for an argument the reference
 *     op would reject (m3d_last_error() then holds the reference's
 *     InvalidArgument text), M3D_EHIP for a HIP launch error.
 *   - reentrant: no global mutable state apart from the thread-local error
 *     string.  The deterministic-reduction target is an argument of the calls
 *     that use it (m3d_det_t), the fork events of m3d_stream_fork are the
 *     caller's (m3d_fork_event_create).
 */
#ifndef M3D_H
#define M3D_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* m3d_stream_t; /* == hipStream_t */

#define M3D_OK 0
#define M3D_EINVAL (-1)
#define M3D_EHIP (-2)

const char* m3d_last_error(void);
int m3d_abi_version(void);

/* Deterministic reductions (the analogue of TF_DETERMINISTIC_OPS for the
 * reference's training graph, core/models.py:3340-3387), chosen per call: the
 * weight-gradient entry points (m3d_conv3d_bwd_weight*, m3d_gemm_wgrad_f32)
 * and the optimizers (m3d_sgd_keras, m3d_adam_keras, m3d_adadelta_keras) take
 * a `const m3d_det_t* det`.  det == NULL or det->on == 0: m-split partial
 * tiles and clip norms are added with fp32 atomics (fast; the last bits vary
 * with arrival order).  det->on == 1: every weight-gradient GEMM stores its
 * m-split partial tiles into det->scratch and adds them to dW in split order,
 * and the clip norms are summed in chunk order; results are then bitwise
 * identical run to run.  det->scratch (device, 16-B aligned, >= 4096 bytes)
 * is used by that call's kernels only until the call's last kernel on `s`
 * finishes: calls sharing one scratch must be ordered (one stream, or
 * joined); concurrent calls need scratches of their own.  A gradient whose two
 * splits do not fit runs unsplit.  A bad det (on, but NULL / short /
 * misaligned scratch) is M3D_EINVAL.  (ABI 3; replaces the process-wide
 * m3d_set_deterministic of ABI 2.)  The ROIAlign backward keeps its own flag
 * (crop_and_resize3d_bwd_image's `deterministic`, m3d_pyramid_roi_align3d_bwd_det). */
typedef struct m3d_det {
    int32_t on;
    void* scratch;
    size_t bytes;
} m3d_det_t;

/* Stream fork / join of the training step (weight gradients on a side stream):
 * `to` waits for everything enqueued on `from` so far, through the caller's
 * event `ev` (m3d_fork_event_create: hipEventDisableTiming; mode 1: +
 * hipEventReleaseToDevice, mode 2: + hipEventDisableSystemFence, mode 0:
 * neither), recorded on `from`.  Both streams must be on the same device: the
 * event's release need not reach the host.  An event may be re-recorded once
 * the wait that used it is enqueued (a ring of events per device suffices). */
int m3d_fork_event_create(int32_t mode, void** ev);
int m3d_fork_event_destroy(void* ev);
int m3d_stream_fork(m3d_stream_t from, m3d_stream_t to, void* ev);

/* ---------------------------------------------------------------------------
 * CropAndResize3D family.  Replaces the TF custom ops of the vendored wheel
 * tensorflow_nms_car_3d==0.1.0 imported at core/custom_op/custom_op.py:22-24:
 *   crop_and_resize_3d(image, boxes, box_index, crop_size,
 *                      method_name='trilinear', extrapolation_value=0)
 *   crop_and_resize_3d_grad_image(grads, boxes, box_ind, image_size, T, method_name)
 *   crop_and_resize_3d_grad_boxes(grads, image, boxes, box_ind, method_name)
 * called from core/models.py:663 (PyramidROIAlign) and :992 (mask targets),
 * gradient wiring core/custom_op/custom_op.py:28-65.
 * method: 0 = trilinear, 1 = nearest.
 * ------------------------------------------------------------------------- */
int m3d_crop_and_resize3d_fwd(const float* image, int64_t B, int64_t H, int64_t W, int64_t D,
                              int64_t C, const float* boxes, const int32_t* box_ind, int64_t N,
                              int32_t ch, int32_t cw, int32_t cd, int32_t method,
                              float extrapolation, float* crops /*[N,ch,cw,cd,C]*/,
                              m3d_stream_t s);

/* grad_image: every voxel written by the callee.  deterministic=0: zero fill +
 * fp32 atomics (fast; the last bits vary with arrival order);
 * deterministic=1: every output voxel row owned by one thread that adds its
 * terms in the reference's sequential box->y->x->z->corner order (bit-identical
 * to the wheel's CPU scatter, parallel over voxels, no atomics; crops <= 64
 * per axis, larger crops fall back to mode 2); deterministic=2: the
 * per-(image,channel) sequential replay of the same order (slow, the check of
 * mode 1). */
int m3d_crop_and_resize3d_bwd_image(const float* grads, const float* boxes,
                                    const int32_t* box_ind, int64_t N, int32_t ch, int32_t cw,
                                    int32_t cd, int64_t B, int64_t H, int64_t W, int64_t D,
                                    int64_t C, int32_t method, int32_t deterministic,
                                    float* grad_image /*[B,H,W,D,C]*/, m3d_stream_t s);

int m3d_crop_and_resize3d_bwd_boxes(const float* grads, const float* image, int64_t B, int64_t H,
                                    int64_t W, int64_t D, int64_t C, const float* boxes,
                                    const int32_t* box_ind, int64_t N, int32_t ch, int32_t cw,
                                    int32_t cd, float* grad_boxes /*[N,6]*/, m3d_stream_t s);

/* ---------------------------------------------------------------------------
 * PyramidROIAlign fused forward/backward (core/models.py:597-687): clip, min
 * size, level = clamp(4+round_half_even(log2(cbrt(vol)/(224/cbrt(HWD)))),2,5),
 * trilinear crop from P_level, output written in the original (b,n) order,
 * non-finite values scrubbed to 0.  fmaps[l] is P(l+2) [B,H_l,W_l,D_l,C];
 * fshape[l] = {H_l,W_l,D_l}.  image_meta rows of meta_stride floats, image
 * shape at meta[5:8] (core/models.py:7511-7532).
 * boxes_adj [B,N,6] and levels [B,N] receive the clipped boxes / levels and
 * are the inputs of the backward.
 * ------------------------------------------------------------------------- */
int m3d_pyramid_roi_align3d_fwd(const float* const fmaps[4], const int64_t fshape[4][3],
                                int64_t C, const float* boxes, const float* image_meta,
                                int64_t meta_stride, int64_t B, int64_t N, int32_t ph,
                                int32_t pw, int32_t pd, float* out /*[B,N,ph,pw,pd,C]*/,
                                float* boxes_adj, int32_t* levels, m3d_stream_t s);

/* The same forward with a workspace (>= the _workspace_bytes size, device
 * memory, caller-owned): the ROI lines are first counting-sorted by the
 * feature-map column they read, so overlapping ROIs share their rows through
 * L2 (bit-identical output; the order only changes which cache serves them). */
size_t m3d_pyramid_roi_align3d_fwd_workspace_bytes(const int64_t fshape[4][3], int64_t B, int64_t N,
                                                   int32_t ph, int32_t pw);
int m3d_pyramid_roi_align3d_fwd_ws(const float* const fmaps[4], const int64_t fshape[4][3],
                                   int64_t C, const float* boxes, const float* image_meta,
                                   int64_t meta_stride, int64_t B, int64_t N, int32_t ph,
                                   int32_t pw, int32_t pd, float* out, float* boxes_adj,
                                   int32_t* levels, void* workspace, size_t ws_bytes, m3d_stream_t s);

/* gmaps[l] are zero-filled by the callee, then receive the image gradient. */
int m3d_pyramid_roi_align3d_bwd(const float* grad_out, const float* boxes_adj,
                                const int32_t* levels, int64_t B, int64_t N, int32_t ph,
                                int32_t pw, int32_t pd, float* const gmaps[4],
                                const int64_t fshape[4][3], int64_t C, m3d_stream_t s);

/* The same backward, bitwise reproducible: per level, CropAndResize3DGradImage
 * over that level's ROIs in ascending order (the reference's tf.where gather
 * order) with destination-owned sums in its sequential replay order (the
 * deterministic mode 1 kernel of m3d_crop_and_resize3d_bwd_image; crop sizes
 * up to 64; every voxel written).  box_ind_ws: [4][B*N] int32 device scratch.
 * Used when m3d_set_deterministic is on. */
int m3d_pyramid_roi_align3d_bwd_det(const float* grad_out, const float* boxes_adj,
                                    const int32_t* levels, int64_t B, int64_t N, int32_t ph,
                                    int32_t pw, int32_t pd, float* const gmaps[4],
                                    const int64_t fshape[4][3], int64_t C, int32_t* box_ind_ws,
                                    m3d_stream_t s);

/* DetectionTargetLayer mask targets (core/models.py:972-996): out[p] =
 * round_half_even(CropAndResize3D(float(gt_masks[..., assign[p]]), rois[p],
 * (mh,mw,md), trilinear, extrapolation 0)), reading the boolean masks
 * [H,W,D,G] (uint8) in place instead of materialising the [P,H,W,D,1] gather.
 * rois are the (mini-mask-normalised when USE_MINI_MASK) positive boxes;
 * rows with assign[p] < 0 are written as zeros. */
int m3d_mask_targets3d(const uint8_t* gt_masks, int64_t H, int64_t W, int64_t D, int64_t G,
                       const float* rois, const int32_t* assign, int64_t P, int32_t mh,
                       int32_t mw, int32_t md, float* out /*[P,mh,mw,md]*/, m3d_stream_t s);

/* ---------------------------------------------------------------------------
 * NonMaxSuppression3D (core/custom_op/custom_op.py:25; called at
 * core/models.py:453): greedy hard NMS, candidates ordered by (score desc,
 * index asc), score > -FLT_MAX, suppress when IoU > iou_thr.  mode 0: 3-D
 * boxes [N,6]; mode 1: 2-D boxes [N,4] (y1,x1,y2,x2) (TF 2.2 IOU).
 * keep receives min(max_out, #kept) original indices in selection order;
 * *num_keep (device int32) the count.  Bit-exact vs the reference.
 * ------------------------------------------------------------------------- */
size_t m3d_nms3d_workspace_bytes(int64_t N);
int m3d_nms3d(const float* boxes, const float* scores, int64_t N, int32_t max_out, float iou_thr,
              int32_t mode, int32_t* keep, int32_t* num_keep, void* workspace, size_t ws_bytes,
              m3d_stream_t s);

/* ---------------------------------------------------------------------------
 * ProposalLayer pieces (core/models.py:369-503).
 * m3d_score_keys: int64 keys whose descending order is tf.nn.top_k's order
 *   (score desc, lower index first) for scores = probs[:, :, 1].
 * m3d_proposal_decode: gather the top-k anchors/deltas, de-normalise by
 *   rpn_bbox_std_dev, clip +-3, apply_box_deltas_graph, clip to [0,1], enforce
 *   min sizes.  order[k] are int64 anchor indices into anchors [n_anchors,6]
 *   (and probs [n_anchors,2], deltas [n_anchors,6]); k > n_anchors is
 *   M3D_EINVAL.  An index outside [0, n_anchors) is never read: its row gets a
 *   zero box and score -FLT_MAX (never selected by NMS) and the DEVICE int32
 *   *err (may be NULL; the caller zeroes it) is set to 1, checked by the caller
 *   at its next synchronisation (the reference's tf.gather InvalidArgument).
 *   exp is evaluated as (float)exp((double)x).  ABI 2 added n_anchors / err.
 * m3d_proposal_gather: proposals[P,6] = boxes[keep[i]] for i < *num_keep,
 *   zero rows after (core/models.py:476-485).
 * ------------------------------------------------------------------------- */
int m3d_score_keys(const float* probs /*[A,2]*/, int64_t A, int64_t* keys, m3d_stream_t s);
/* tf.nn.top_k(keys, k, sorted=True) (core/models.py:403-404) on distinct int64
 * keys (the m3d_score_keys keys): out_keys [k] the k largest in descending
 * order, out_pos [k] (nullable) their positions in keys.  Radix select of the
 * k-th largest key (six digit passes over the keys, no sort of all n), then a
 * stable sort of the k selected.  Keys equal to the k-th largest are taken in
 * arbitrary order (the count stays exact): distinct keys give a deterministic
 * result.  k > n is M3D_EINVAL (tf.nn.top_k's InvalidArgument).
 * workspace: m3d_topk_workspace_bytes(n, k) bytes of device scratch. */
size_t m3d_topk_workspace_bytes(int64_t n, int64_t k);
int m3d_topk_keys(const int64_t* keys, int64_t n, int64_t k, int64_t* out_keys, int64_t* out_pos, void* workspace,
                  size_t ws_bytes, m3d_stream_t s);
/* Same keys for a depth slab of the volume: gidx[i] is local anchor i's index
 * in the whole volume's (y,x,z,a)-ordered anchor list (NULL = identity), so
 * the merged top-k over all slabs has the single-volume order. */
int m3d_score_keys_mapped(const float* probs, int64_t A, const int64_t* gidx, int64_t* keys,
                          m3d_stream_t s);
int m3d_proposal_decode(const float* probs, const float* deltas, const float* anchors,
                        int64_t n_anchors, const int64_t* order, int64_t k, const float std_dev[6],
                        float image_depth, float* boxes /*[k,6]*/, float* scores /*[k]*/,
                        int32_t* err /*device, nullable*/, m3d_stream_t s);
int m3d_proposal_gather(const float* boxes, const int32_t* keep, const int32_t* num_keep,
                        int32_t P, float* proposals, m3d_stream_t s);

/* ---------------------------------------------------------------------------
 * Conv3D (Keras Conv3D, core/models.py:157-273, 512-557, 3190-3214) as
 * fp32 MFMA implicit GEMMs (v_mfma_f32_32x32x2_f32).
 *
 * m3d_conv3d_fwd: y = act(bn(conv(x, w) + bias) + residual)
 *   x [B,H,W,D,Cin], w [kh,kw,kd,Cin,Cout], output grid [B,OH,OW,OD],
 *   stride (sy,sx,sz), pad-before (py,px,pz) (zero padding, TF 'same'/'valid').
 *   bias/bn_scale/bn_shift: [Cout] or NULL.  z_out (optional) receives
 *   conv+bias before the BN affine.  residual: NULL, or a tensor added before
 *   the activation; res_mode 1 = same shape as y, 2 = (2,2,1)-nearest
 *   upsampled source [B,OH/2,OW/2,OD,Cout] (FPN top-down add).  relu 0/1.
 *   y has row stride ldy >= Cout; if split_n > 0, channels >= split_n go to
 *   y2 (row stride ldy2) at channel n - split_n (RPN class/bbox heads).
 * m3d_conv3d_bwd_data: dx (+)= conv_transpose(dz, w), for stride-1 convs of
 *   any kernel, and 1x1x1 convs of any stride (dx zeroed by the caller for
 *   strided ones).  accumulate: 0 overwrite, 1 add to dx.
 * m3d_conv3d_bwd_weight: dw [kh,kw,kd,Cin,Cout] += sum_m im2col(x)^T dz.
 *   dw must be zeroed by the caller before the first accumulation.
 * ------------------------------------------------------------------------- */
int m3d_conv3d_fwd(const float* x, int64_t B, int64_t H, int64_t W, int64_t D, int64_t Cin,
                   const float* w, int32_t kh, int32_t kw, int32_t kd, int64_t Cout,
                   int64_t OH, int64_t OW, int64_t OD, int32_t sy, int32_t sx, int32_t sz,
                   int32_t py, int32_t px, int32_t pz, const float* bias, const float* bn_scale,
                   const float* bn_shift, const float* residual, int32_t res_mode, int32_t relu,
                   float* z_out, float* y, int64_t ldy, float* y2, int64_t ldy2, int64_t split_n,
                   m3d_stream_t s);
int m3d_conv3d_bwd_data(const float* dz, const float* w, int64_t B, int64_t H, int64_t W,
                        int64_t D, int64_t Cin, int32_t kh, int32_t kw, int32_t kd, int64_t Cout,
                        int64_t OH, int64_t OW, int64_t OD, int32_t sy, int32_t sx, int32_t sz,
                        int32_t py, int32_t px, int32_t pz, float* dx, int32_t accumulate,
                        m3d_stream_t s);
/* Split-K forms of the 1x1x1 convs whose output tiles do not fill the chip
 * (deep stages: few voxels, Cin up to 2048).  m3d_conv3d_splitk_count gives
 * the K-slices for a GEMM of M output rows, reduction K and N columns (1: one
 * pass); the caller passes `splits` (so a depth slab can use the count of the
 * whole volume and stay bit-identical to it) and a workspace of
 * splits * M * N floats (M = B*OH*OW*OD; N = Cout fwd, Cin bwd-data).  The
 * K-slices are summed in slice order (deterministic) and the conv's epilogue
 * applied once: the result equals m3d_conv3d_fwd / _bwd_data up to the order
 * of the K sum.  splits <= 1 runs the one-pass kernels.  Conv3D(1,1,1) of
 * core/models.py (a TF builtin in the reference). */
int32_t m3d_conv3d_splitk_count(int64_t M, int64_t K, int64_t N);
int m3d_conv3d_fwd_splitk(const float* x, int64_t B, int64_t H, int64_t W, int64_t D, int64_t Cin,
                          const float* w, int64_t Cout, int64_t OH, int64_t OW, int64_t OD, int32_t sy,
                          int32_t sx, int32_t sz, const float* bias, const float* bn_scale,
                          const float* bn_shift, const float* residual, int32_t res_mode, int32_t relu,
                          float* z_out, float* y, int32_t splits, void* workspace, size_t ws_bytes,
                          m3d_stream_t s);
int m3d_conv3d_bwd_data_splitk(const float* dz, const float* w, int64_t B, int64_t H, int64_t W, int64_t D,
                               int64_t Cin, int64_t Cout, int64_t OH, int64_t OW, int64_t OD, int32_t sy,
                               int32_t sx, int32_t sz, float* dx, int32_t accumulate, int32_t splits,
                               void* workspace, size_t ws_bytes, m3d_stream_t s);
/* 1x1x1 stride-1 convs as one GEMM on the exact bf16 split (the 1x1x1 convs
 * and data gradients with enough 256x256 output tiles to fill the chip,
 * m3d.nn._conv1_x3).  m3d_conv1_x3_planes splits the Keras kernel w [Cin][Cout] into
 * planes uint16 [3][N][K] (transpose = 1: forward, N = Cout, K = Cin;
 * transpose = 0: data gradient, N = Cin, K = Cout).  Then the forward (epilogue
 * of m3d_conv3d_fwd: bias, z, BN, same-shape or (2,2,1)-upsampled residual,
 * activation; applied by a second in-place pass over y) or the data gradient
 * (dx = dz w^T, no accumulate).  K % 32 == 0, N % 256 == 0.
 * Error vs fp64 at or below the f32 MFMA's (exact split, 6 bf16 MFMAs per
 * product). */
int m3d_conv1_x3_planes(const float* w, int64_t Cin, int64_t Cout, int32_t transpose, uint16_t* planes,
                        m3d_stream_t s);
/* m3d_conv1_x3_planes of many kernels in one launch: items is a DEVICE array of
 * n descriptors; each kernel w [cin][cout] is split once into its forward
 * planes (fwd, transpose = 1 layout) and its data-gradient planes (bwd,
 * transpose = 0 layout), either may be NULL; max_el = max cin*cout.  Same bits
 * as the per-kernel call (the model's forward refreshes every 1x1x1 kernel that
 * runs on the split GEMM at once, m3d.nn.X3Planes). */
typedef struct {
    const float* w;
    uint16_t* fwd;
    uint16_t* bwd;
    int32_t cin;
    int32_t cout;
} m3d_x3_planes_item_t;
int m3d_conv1_x3_planes_batched(const m3d_x3_planes_item_t* items, int32_t n, int64_t max_el, m3d_stream_t s);
int m3d_conv3d_fwd_x3(const float* x, int64_t B, int64_t H, int64_t W, int64_t D, int64_t Cin,
                      const uint16_t* planes, int64_t Cout, const float* bias, const float* bn_scale,
                      const float* bn_shift, const float* residual, int32_t res_mode, int32_t relu,
                      float* z_out, float* y, m3d_stream_t s);
int m3d_conv3d_bwd_data_x3(const float* dz, const uint16_t* planes, int64_t B, int64_t H, int64_t W, int64_t D,
                           int64_t Cin, int64_t Cout, float* dx, m3d_stream_t s);
/* m3d_conv3d_fwd_wino / m3d_conv3d_bwd_data_wino for a kernel shared across
 * calls (rpn_conv_shared1 on P2..P6, core/models.py:512-557): v_ready = 1 means
 * the workspace's transformed-weight region already holds this w's transform
 * from an earlier call on the same stream with the same Cin, Cout and
 * workspace, and the weight transform is skipped (results bit-identical). */
int m3d_conv3d_fwd_wino_v(const float* x, int64_t B, int64_t H, int64_t W, int64_t D, int64_t Cin,
                          const float* w, int64_t Cout, int64_t OD, int32_t pz, const float* bias,
                          const float* bn_scale, const float* bn_shift, const float* residual, int32_t relu,
                          float* z_out, float* y, void* workspace, size_t ws_bytes, int32_t v_ready,
                          m3d_stream_t s);
int m3d_conv3d_bwd_data_wino_v(const float* dz, const float* w, int64_t B, int64_t H, int64_t W, int64_t D,
                               int64_t Cin, int64_t Cout, int64_t OD, int32_t pz, float* dx, int32_t accumulate,
                               void* workspace, size_t ws_bytes, int32_t v_ready, m3d_stream_t s);
int m3d_conv3d_bwd_weight(const float* x, const float* dz, int64_t B, int64_t H, int64_t W,
                          int64_t D, int64_t Cin, int32_t kh, int32_t kw, int32_t kd,
                          int64_t Cout, int64_t OH, int64_t OW, int64_t OD, int32_t sy,
                          int32_t sx, int32_t sz, int32_t py, int32_t px, int32_t pz, float* dw,
                          const m3d_det_t* det, m3d_stream_t s);
/* Depth-slab forms of the direct convs (no halo-extended copy of the slab): x
 * [B,H,W,Dl,Cin] is the local slab, halo [B,H,W,2r,Cin] the neighbours' r
 * boundary planes (planes [0,r) from below, [r,2r) from above; has_lo / has_hi:
 * that neighbour exists); the z window is 'same' kd = 2r+1 at stride 1 with
 * pad pz = r applied only where the volume ends, OD = Dl.  Same taps and sums
 * as the conv on the halo-extended slab.  fwd: the one-channel 7^3 stem only
 * (core/models.py:242, 1 -> 64, strides (2,2,1)); bwd_weight: any direct conv
 * (the stem, the 64-channel 3^3 convs of stage 2). */
int m3d_conv3d_fwd_halo(const float* x, const float* halo, int32_t has_lo, int32_t has_hi, int32_t r,
                        int64_t B, int64_t H, int64_t W, int64_t Dl, int64_t Cin, const float* w,
                        int32_t kh, int32_t kw, int32_t kd, int64_t Cout, int64_t OH, int64_t OW, int64_t OD,
                        int32_t sy, int32_t sx, int32_t sz, int32_t py, int32_t px, int32_t pz,
                        const float* bias, const float* bn_scale, const float* bn_shift, int32_t relu,
                        float* z_out, float* y, m3d_stream_t s);
int m3d_conv3d_bwd_weight_halo(const float* x, const float* halo, int32_t has_lo, int32_t has_hi, int32_t r,
                               const float* dz, int64_t B, int64_t H, int64_t W, int64_t Dl, int64_t Cin,
                               int32_t kh, int32_t kw, int32_t kd, int64_t Cout, int64_t OH, int64_t OW,
                               int64_t OD, int32_t sy, int32_t sx, int32_t sz, int32_t py, int32_t px,
                               int32_t pz, float* dw, const m3d_det_t* det, m3d_stream_t s);

/* Winograd F(2x2x2,3x3x3) versions of the three passes for stride-1 3x3x3
 * convs with 'same' padding in y/x (every 3x3x3 conv of the graph:
 * res*_branch2b, fpn_p*, rpn_conv_shared1): 3.375x fewer multiplies, the 64
 * point-wise products run as batched fp32-MFMA GEMMs.  Cin, Cout multiples of
 * 32.  Same epilogue as m3d_conv3d_fwd (res_mode 1 only).
 * z geometry: x has depth D, y depth OD, z pad-before pz.  'same' is OD == D,
 * pz == 1; a depth slab extended by z-halo planes from its neighbours (multi-
 * GPU depth-slab sharding) has D = OD + #halo planes and pz = 1 - (lower halo
 * present).  Requires pz in {0,1}, 0 <= D - OD <= 2.
 * workspace: m3d_conv3d_wino_workspace_bytes(B,H,W,D,OD,Cin,Cout). */
size_t m3d_conv3d_wino_workspace_bytes(int64_t B, int64_t H, int64_t W, int64_t D, int64_t OD,
                                       int64_t Cin, int64_t Cout);
int m3d_conv3d_fwd_wino(const float* x, int64_t B, int64_t H, int64_t W, int64_t D, int64_t Cin,
                        const float* w, int64_t Cout, int64_t OD, int32_t pz, const float* bias,
                        const float* bn_scale, const float* bn_shift, const float* residual,
                        int32_t relu, float* z_out, float* y, void* workspace, size_t ws_bytes,
                        m3d_stream_t s);
int m3d_conv3d_bwd_data_wino(const float* dz, const float* w, int64_t B, int64_t H, int64_t W,
                             int64_t D, int64_t Cin, int64_t Cout, int64_t OD, int32_t pz,
                             float* dx, int32_t accumulate, void* workspace, size_t ws_bytes,
                             m3d_stream_t s);
int m3d_conv3d_bwd_weight_wino(const float* x, const float* dz, int64_t B, int64_t H, int64_t W,
                               int64_t D, int64_t Cin, int64_t Cout, int64_t OD, int32_t pz,
                               float* dw, void* workspace, size_t ws_bytes, const m3d_det_t* det, m3d_stream_t s);
/* Training variants: the forward keeps its transformed input U = B^T x B
 * ([64][T][Cin], m3d_conv3d_wino_u_bytes) in caller memory (u_keep) and the
 * weight gradient reuses it instead of transforming x again. */
/* z extent of the Winograd output tile (4: F(2x2x4), default; 2: F(2x2x2)
 * when M3D_WINO_NZ=2): 16*(NZ+2) batched point GEMMs per conv. */
int32_t m3d_conv3d_wino_tile_z(void);
/* z extent of the weight gradient's output tile (4: F(2x2x4), the forward's, whose
 * transformed input the forward keeps -- m3d_conv3d_wino_u_bytes > 0; 2: F(2x2x2)). */
int32_t m3d_conv3d_wino_wgrad_tile_z(void);
int32_t m3d_conv3d_wino_tile_y(void);   /* output tile rows along y (2: F(2,3), 4: F(4,3)) */
/* the data gradient's tile (m3d_conv3d_bwd_data_wino*): F(2,3) along y by
 * default (F(2x2x4)) beside the forward's F(4x2x4) -- the accuracy of the
 * gradients every earlier layer receives */
int32_t m3d_conv3d_wino_dgrad_tile_y(void);
int32_t m3d_conv3d_wino_dgrad_tile_z(void);
/* Workspace of one data-gradient call at tile_y (0, 2, 4; 0 = the default):
 * the layout m3d_conv3d_bwd_data_wino(_v, _vy, _bn, _bny) check against
 * (m3d_conv3d_wino_workspace_bytes covers every tile; this is the exact need).
 * 0 for an invalid tile_y. */
size_t m3d_conv3d_wino_dgrad_workspace_bytes(int64_t B, int64_t H, int64_t W, int64_t D, int64_t OD,
                                             int64_t Cin, int64_t Cout, int32_t tile_y);
size_t m3d_conv3d_wino_u_bytes(int64_t B, int64_t H, int64_t W, int64_t OD, int64_t Cin);
int m3d_conv3d_fwd_wino_keep(const float* x, int64_t B, int64_t H, int64_t W, int64_t D, int64_t Cin,
                             const float* w, int64_t Cout, int64_t OD, int32_t pz, const float* bias,
                             const float* bn_scale, const float* bn_shift, const float* residual,
                             int32_t relu, float* z_out, float* y, float* u_keep, void* workspace,
                             size_t ws_bytes, m3d_stream_t s);
int m3d_conv3d_bwd_weight_wino_u(const float* u, const float* dz, int64_t B, int64_t H, int64_t W,
                                 int64_t D, int64_t Cin, int64_t Cout, int64_t OD, int32_t pz,
                                 float* dw, void* workspace, size_t ws_bytes, const m3d_det_t* det, m3d_stream_t s);
/* Depth-slab forms (multi-GPU sharding of one volume, m3d/slab.py): x is this
 * rank's slab [B,H,W,Dl,C] and x_halo [B,H,W,2,C] the neighbours' boundary
 * planes (plane 0 = z -1 from the lower rank, valid if has_lo; plane 1 = z Dl
 * from the upper rank, valid if has_hi) -- the halo-extended slab is never
 * materialised; results are bit-identical to the extended-tensor calls.  The
 * data gradient writes the slab's interior into dx [B,H,W,Dl,Cin] (accumulate
 * as above) and the gradient of the neighbours' planes into dx_halo
 * [B,H,W,2,Cin].  workspace: m3d_conv3d_wino_workspace_bytes(B,H,W,
 * Dl + has_lo + has_hi, Dl, Cin, Cout).  u_keep as m3d_conv3d_fwd_wino_keep
 * (NULL: not kept). */
int m3d_conv3d_fwd_wino_halo(const float* x, const float* x_halo, int32_t has_lo, int32_t has_hi, int64_t B,
                             int64_t H, int64_t W, int64_t Dl, int64_t Cin, const float* w, int64_t Cout,
                             const float* bias, const float* bn_scale, const float* bn_shift,
                             const float* residual, int32_t relu, float* z_out, float* y, float* u_keep,
                             void* workspace, size_t ws_bytes, m3d_stream_t s);
/* The same conv in two launches around the halo exchange (the caller posts the
 * exchange, then): phase 1 -- weight transform and the interior z tiles, x_halo
 * not read (may be NULL); phase 2 -- after the halo planes arrived: the first /
 * last z tiles, the point GEMMs and the output transform.  Same arguments and
 * workspace in both calls; bit-identical to m3d_conv3d_fwd_wino_halo. */
int m3d_conv3d_fwd_wino_halo_phase(const float* x, const float* x_halo, int32_t has_lo, int32_t has_hi,
                                   int64_t B, int64_t H, int64_t W, int64_t Dl, int64_t Cin, const float* w,
                                   int64_t Cout, const float* bias, const float* bn_scale, const float* bn_shift,
                                   const float* residual, int32_t relu, float* z_out, float* y, float* u_keep,
                                   void* workspace, size_t ws_bytes, int32_t phase, m3d_stream_t s);
int m3d_conv3d_bwd_data_wino_halo(const float* dz, const float* w, int32_t has_lo, int32_t has_hi, int64_t B,
                                  int64_t H, int64_t W, int64_t Dl, int64_t Cin, int64_t Cout, float* dx,
                                  float* dx_halo, int32_t accumulate, void* workspace, size_t ws_bytes,
                                  m3d_stream_t s);
int m3d_conv3d_bwd_weight_wino_halo(const float* x, const float* x_halo, int32_t has_lo, int32_t has_hi,
                                    const float* dz, int64_t B, int64_t H, int64_t W, int64_t Dl, int64_t Cin,
                                    int64_t Cout, float* dw, void* workspace, size_t ws_bytes, const m3d_det_t* det, m3d_stream_t s);

/* Data gradients with the producing unit's BN-ReLU backward fused into their
 * epilogue (the bn_act_bwd pass of core/models.py:102-114 / 157-232 folded
 * into the kernel that computes the unit's output gradient): the data
 * gradient t = conv^T(dz) (+ dx when accumulate) of this conv's input x is the
 * output gradient of the unit U that produced x = act(BN(z) [+ res]); instead
 * of t, dx receives U's dz = act'(t) * scale, bn->dres (optional) receives
 * dpre = act'(t) (U's residual gradient), and the channel sums of U's
 * backward are added (+=, fixed order) into sum_dpre (beta), sum_dpre_xhat
 * (gamma; needs z, mean, rstd) and sum_dz (bias) -- m3d_bn_act_bwd's results,
 * without the round trip of t through HBM.  relu: y = U's output (mask y > 0);
 * scale = NULL: no BN.  workspace: m3d_bn_bwd_fused_workspace_bytes(B, H, W,
 * D, Cin) bytes of device scratch for the channel partials.
 * m3d_conv3d_bwd_data_bn: stride-1 convs of m3d_conv3d_bwd_data (the direct
 * implicit GEMM).  m3d_conv3d_bwd_data_wino_bn: m3d_conv3d_bwd_data_wino_v
 * with Cin dividing 256 or a multiple of it.  m3d_conv3d_bwd_data_splitk_bn:
 * m3d_conv3d_bwd_data_splitk of a stride-1 1x1x1 conv (OH,OW,OD = H,W,D), the
 * K-slice reduce doing the BN-ReLU backward (splits <= 1: the one-pass form). */
typedef struct m3d_bn_bwd {
    const float* y;
    const float* z;
    const float* scale;
    const float* mean;
    const float* rstd;
    int32_t relu;
    float* dres;
    float* sum_dpre;
    float* sum_dpre_xhat;
    float* sum_dz;
} m3d_bn_bwd_t;
size_t m3d_bn_bwd_fused_workspace_bytes(int64_t B, int64_t H, int64_t W, int64_t D, int64_t C);
int m3d_conv3d_bwd_data_bn(const float* dz, const float* w, int64_t B, int64_t H, int64_t W, int64_t D,
                           int64_t Cin, int32_t kh, int32_t kw, int32_t kd, int64_t Cout, int64_t OH,
                           int64_t OW, int64_t OD, int32_t sy, int32_t sx, int32_t sz, int32_t py,
                           int32_t px, int32_t pz, float* dx, int32_t accumulate, const m3d_bn_bwd_t* bn,
                           void* workspace, size_t ws_bytes, m3d_stream_t s);
int m3d_conv3d_bwd_data_wino_bn(const float* dz, const float* w, int64_t B, int64_t H, int64_t W, int64_t D,
                                int64_t Cin, int64_t Cout, int64_t OD, int32_t pz, float* dx, int32_t accumulate,
                                void* workspace, size_t ws_bytes, int32_t v_ready, const m3d_bn_bwd_t* bn,
                                void* bn_ws, size_t bn_ws_bytes, m3d_stream_t s);
/* The two data-gradient forms above with the y tile chosen per call: tile_y 2
 * (F(2x2xNZ), the library default: m3d_conv3d_wino_dgrad_tile_y) or 4
 * (F(4x2xNZ): 4.5 instead of 6 points per output, ~4x the point GEMMs'
 * rounding carried into dx), 0 = the default.  A v_ready call must reuse a V
 * transformed with the same tile_y. */
int m3d_conv3d_bwd_data_wino_vy(const float* dz, const float* w, int64_t B, int64_t H, int64_t W, int64_t D,
                                int64_t Cin, int64_t Cout, int64_t OD, int32_t pz, float* dx, int32_t accumulate,
                                void* workspace, size_t ws_bytes, int32_t v_ready, int32_t tile_y, m3d_stream_t s);
int m3d_conv3d_bwd_data_wino_bny(const float* dz, const float* w, int64_t B, int64_t H, int64_t W, int64_t D,
                                 int64_t Cin, int64_t Cout, int64_t OD, int32_t pz, float* dx, int32_t accumulate,
                                 void* workspace, size_t ws_bytes, int32_t v_ready, const m3d_bn_bwd_t* bn, void* bn_ws,
                                 size_t bn_ws_bytes, int32_t tile_y, m3d_stream_t s);
/* Winograd weight transforms into caller memory: the transformed weights
 * depend on w only, so a caller may produce them ahead of the convs (a side
 * stream at the start of the forward) and pass them to the _kv / _xv entries,
 * which then skip their own transform (same kernels, same bits).  dgrad 0: the
 * forward's operand; 1: the data gradient's at tile_y (0 = library default, 2,
 * 4).  Requires the bf16-split GEMMs (0 bytes / M3D_EINVAL otherwise). */
size_t m3d_conv3d_wino_v_bytes(int64_t Cin, int64_t Cout, int32_t dgrad, int32_t tile_y);
int m3d_conv3d_wino_weight_v(const float* w, int64_t Cin, int64_t Cout, int32_t dgrad, int32_t tile_y, void* v,
                             size_t v_bytes, m3d_stream_t s);
/* m3d_conv3d_fwd_wino_keep (u_keep may be NULL) with the transformed weights v */
int m3d_conv3d_fwd_wino_kv(const float* x, int64_t B, int64_t H, int64_t W, int64_t D, int64_t Cin, const float* w,
                           int64_t Cout, int64_t OD, int32_t pz, const float* bias, const float* bn_scale,
                           const float* bn_shift, const float* residual, int32_t relu, float* z_out, float* y,
                           float* u_keep, const void* v, void* workspace, size_t ws_bytes, m3d_stream_t s);
/* m3d_conv3d_bwd_data_wino_vy (bn NULL) / _bny (bn set) with the transformed weights v */
int m3d_conv3d_bwd_data_wino_xv(const float* dz, const float* w, int64_t B, int64_t H, int64_t W, int64_t D,
                                int64_t Cin, int64_t Cout, int64_t OD, int32_t pz, float* dx, int32_t accumulate,
                                void* workspace, size_t ws_bytes, const void* v, int32_t tile_y,
                                const m3d_bn_bwd_t* bn, void* bn_ws, size_t bn_ws_bytes, m3d_stream_t s);
/* m3d_conv3d_bwd_data_x3 (a 1x1x1 stride-1 conv's data gradient on the
 * bf16-split GEMM, accumulate 0) with m3d_conv3d_bwd_data_bn's fused BN-ReLU
 * backward in the GEMM's epilogue; bn_ws: m3d_bn_bwd_fused_workspace_bytes. */
int m3d_conv3d_bwd_data_x3_bn(const float* dz, const uint16_t* planes, int64_t B, int64_t H, int64_t W, int64_t D,
                              int64_t Cin, int64_t Cout, float* dx, const m3d_bn_bwd_t* bn, void* bn_ws,
                              size_t bn_ws_bytes, m3d_stream_t s);
/* The same with accumulate (the identity blocks' 2a data gradient,
 * core/models.py:157-189: dx holds the residual's parked gradient, and the
 * fused epilogue takes t = conv^T(dz) + dx before the BN-ReLU backward, as
 * m3d_conv3d_bwd_data_bn with accumulate 1). */
int m3d_conv3d_bwd_data_x3_bna(const float* dz, const uint16_t* planes, int64_t B, int64_t H, int64_t W, int64_t D,
                               int64_t Cin, int64_t Cout, float* dx, int32_t accumulate, const m3d_bn_bwd_t* bn,
                               void* bn_ws, size_t bn_ws_bytes, m3d_stream_t s);
int m3d_conv3d_bwd_data_splitk_bn(const float* dz, const float* w, int64_t B, int64_t H, int64_t W, int64_t D,
                                  int64_t Cin, int64_t Cout, float* dx, int32_t accumulate, int32_t splits,
                                  void* workspace, size_t ws_bytes, const m3d_bn_bwd_t* bn, void* bn_ws,
                                  size_t bn_ws_bytes, m3d_stream_t s);

/* Plain batched fp32 GEMM on the same MFMA kernel: for b < batch,
 * C[b] = act(A[b] B[b] + bias) (+ C[b] if accumulate); A [M][K], B [K][N],
 * C [M][N] row-major, batches contiguous; N multiple of 4.  The Winograd
 * point-wise products above run this f32-MFMA kernel with M3D_GEMM_X3=0 (by
 * default they run x3_gemm_kernel on the exact bf16 split, conv3d.hip). */
int m3d_gemm_f32(const float* A, const float* B, float* C, int64_t batch, int64_t M, int64_t K,
                 int64_t N, const float* bias, int32_t relu, int32_t accumulate, m3d_stream_t s);

/* Batched weight-gradient GEMM on the conv weight-gradient kernel
 * (conv_wgrad_kernel, fp32 MFMA, M split over workgroups, fp32 atomics):
 * for b < batch, C[b] [K][N] += A[b]^T B[b] with A [M][K], B [M][N], batches
 * contiguous; K, N multiples of 4.  The Winograd weight gradient (Conv3D's
 * kernel gradient, TF Conv3DBackpropFilterV2 in the reference graph) is this
 * call with batch = 64 on the transformed input and output gradient; bench.py
 * prices the RPN head's largest one. */
int m3d_gemm_wgrad_f32(const float* A, const float* B, float* C, int64_t batch, int64_t M, int64_t K,
                       int64_t N, const m3d_det_t* det, m3d_stream_t s);

/* The exact 3-way bf16 split of fp32 data (x = hi + mid + lo, each bf16; exact
 * for normal x): x3 receives the three uint16 planes, plane p at x3 + p*n. */
int m3d_split3_f32(const float* x, int64_t n, uint16_t* x3, m3d_stream_t s);

/* Batched fp32 GEMM on split operands (x3_gemm_kernel: 6 bf16 MFMAs per
 * product, the default for the Winograd point GEMMs above): for b < batch,
 * C[b] [M][N] = A[b] B[b]^T with A3 the m3d_split3_f32 planes of A
 * [batch][M][K] and B3 those of B^T [batch][N][K]; K multiple of 32, N of 4.
 * bench.py prices the RPN head's largest launch with it. */
int m3d_gemm_x3(const uint16_t* A3, const uint16_t* B3, float* C, int64_t batch, int64_t M, int64_t K,
                int64_t N, m3d_stream_t s);
/* m3d_gemm_x3 with A as fp32 [batch][M][K], split in the GEMM on its way into
 * LDS (x3_gemm256_af_kernel for N % 256 == 0, else x3_gemm_kernel<AF32>): the
 * form the Winograd point GEMMs run in the step (M3D_GEMM_X3 bit 4, default),
 * bit-identical to m3d_gemm_x3 on the split planes of the same A. */
int m3d_gemm_x3_af(const float* A, const uint16_t* B3, float* C, int64_t batch, int64_t M, int64_t K,
                   int64_t N, m3d_stream_t s);

/* Strided batched GEMM: for b < batch, C + b*bsc [M][N] (+)= act(A[b] B[b] + bias)
 * with A[b] = A + b*bsa (rows of stride lda >= K), B[b] = B + b*bsb [K][N]; act
 * 0 none / 1 ReLU / 2 sigmoid.  Split-K: batch = #K-slices of width kc (bsa =
 * kc, bsb = kc*N, bsc = M*N) into a workspace, then m3d_splitk_reduce:
 * out[m][n] = act((sum_z ws[z][m][n] + bias[n]) * bn_scale[n] + bn_shift[n])
 * in a fixed z order.  Used for the head convolutions whose kernel covers the
 * whole ROI (mrcnn_class_conv1, core/models.py:1128-1130: K = pool^3 * C). */
int m3d_gemm_f32_ex(const float* A, int64_t lda, int64_t bsa, const float* B, int64_t bsb,
                    float* C, int64_t bsc, int64_t batch, int64_t M, int64_t K, int64_t N,
                    const float* bias, int32_t act, int32_t accumulate, m3d_stream_t s);
int m3d_splitk_reduce(const float* ws, int32_t splits, int64_t M, int64_t N, const float* bias,
                      const float* bn_scale, const float* bn_shift, int32_t act, float* out,
                      m3d_stream_t s);

/* m3d_conv3d_fwd with dilation (dly,dlx,dlz) (mrcnn_mask_conv3b, dilation
 * (2,2,2), core/models.py:1214-1218), activation act = 0 / 1 ReLU / 2 sigmoid
 * (mrcnn_mask), and res_mode 3 = residual added AFTER the activation
 * (KL.Add of two activated branches, mrcnn_mask_res3). */
int m3d_conv3d_fwd_dil(const float* x, int64_t B, int64_t H, int64_t W, int64_t D, int64_t Cin,
                       const float* w, int32_t kh, int32_t kw, int32_t kd, int64_t Cout,
                       int64_t OH, int64_t OW, int64_t OD, int32_t sy, int32_t sx, int32_t sz,
                       int32_t py, int32_t px, int32_t pz, int32_t dly, int32_t dlx, int32_t dlz,
                       const float* bias, const float* bn_scale, const float* bn_shift,
                       const float* residual, int32_t res_mode, int32_t act, float* z_out,
                       float* y, int64_t ldy, float* y2, int64_t ldy2, int64_t split_n,
                       m3d_stream_t s);

/* KL.Conv3DTranspose(Cout, (2,2,2), strides=2) (mrcnn_mask_deconv,
 * core/models.py:1228-1232): x [B,H,W,D,Cin], Keras kernel w [2,2,2,Cout,Cin],
 * y [B,2H,2W,2D,Cout] = act(bias + sum_cin x * w) (no overlap at stride 2).
 * Cin % 32 == 0, Cout % 4 == 0. */
int m3d_deconv3d_k2s2(const float* x, int64_t B, int64_t H, int64_t W, int64_t D, int64_t Cin,
                      const float* w, int64_t Cout, const float* bias, int32_t act, float* y,
                      m3d_stream_t s);

/* ---------------------------------------------------------------------------
 * Mask R-CNN head glue (core/models.py:1121-1190, 1415-1575).
 * m3d_head_outputs: raw [N][ldr] = [class logits (C) | bbox deltas (6C)] of
 *   the two TimeDistributed Dense layers -> logits [N,C] clipped to [-10,10],
 *   probs [N,C] softmax, bbox [N,C,6].
 * m3d_refine_detections: per ROI of refine_detections_graph: fg prob >=
 *   min_conf, class-1 deltas * BBOX_STD_DEV applied to the pixel ROI
 *   (apply_box_deltas_3d_graph, core/utils.py:412-458), clip to the image,
 *   min size (1,1,0.5 px).  boxes_px [N,6], nms_boxes [N,4] (y1,x1,y2,x2),
 *   scores [N] (-FLT_MAX for filtered ROIs).  Then m3d_nms3d(mode 1,
 *   DETECTION_MAX_INSTANCES, DETECTION_NMS_THRESHOLD) on (nms_boxes, scores).
 * m3d_detections_gather: det [max_inst, 8] = (normalised box, class 1, score)
 *   of the kept ROIs in NMS order, zero rows after *num_keep.
 * image_meta: one row (compose_image_meta), image shape at [5:8].
 * ------------------------------------------------------------------------- */
int m3d_head_outputs(const float* raw, int64_t N, int64_t ldr, int32_t num_classes, float* logits,
                     float* probs, float* bbox, m3d_stream_t s);
int m3d_refine_detections(const float* rois, const float* probs, const float* deltas, int64_t N,
                          int32_t num_classes, const float* image_meta,
                          const float bbox_std_dev[6], float min_conf, float* boxes_px,
                          float* nms_boxes, float* scores, m3d_stream_t s);
int m3d_detections_gather(const float* boxes_px, const float* scores, const int32_t* keep,
                          const int32_t* num_keep, int32_t max_inst, const float* image_meta,
                          float* det, m3d_stream_t s);

/* ---------------------------------------------------------------------------
 * DetectionTargetLayer (detection_targets_graph, core/models.py:736-1040) for
 * one image, one workgroup, padded fixed-size outputs (no host round trip).
 * proposals [N,6] (zero rows = padding), gt_class_ids [G], gt_boxes [G,6]
 * normalised (zero rows = padding); N <= 16384, G <= 256.  Positives: IoU max
 * >= positive_iou_threshold, negatives: < negative_iou_threshold; each set in
 * a seeded random order (replaces tf.random.shuffle), positive_count =
 * min(int(f32(T)*ratio), #pos), negatives fill up to T, zero padding after.
 * Outputs [T,...]: rois, roi_gt_boxes, class_ids, deltas
 * (box_refinement_graph / bbox_std_dev), mask_boxes (mini-mask normalised if
 * use_mini_mask) and mask_assign (original GT index, -1 for non-positive
 * rows) for m3d_mask_targets3d; counts[2] = (positives, negatives) (optional).
 * workspace: m3d_detection_targets_workspace_bytes(N). */
size_t m3d_detection_targets_workspace_bytes(int64_t N);
int m3d_detection_targets(const float* proposals, int64_t N, const int32_t* gt_class_ids,
                          const float* gt_boxes, int64_t G, int32_t train_rois_per_image,
                          float roi_positive_ratio, float positive_iou_threshold,
                          float negative_iou_threshold, const float bbox_std_dev[6],
                          int32_t use_mini_mask, uint32_t seed, float* rois, float* roi_gt_boxes,
                          int32_t* class_ids, float* deltas, float* mask_boxes,
                          int32_t* mask_assign, int32_t* counts, void* workspace, size_t ws_bytes,
                          m3d_stream_t s);

/* build_rpn_targets (ATSS, core/data_generators.py:2031-2178) for one volume
 * on the device-resident anchors [A,6] (normalised) and GT boxes [G,6]
 * (normalised, G <= 256): rpn_match [A] int8 (1 / -1 / 0) and rpn_bbox
 * [total,6] (deltas of the positives in anchor order / RPN_BBOX_STD_DEV).
 * Per-GT top-k / ATSS threshold without an [A x G] matrix (per-GT lists of
 * the anchors with IoU > 0, capacity list_cap each); ties where the reference
 * is implementation-defined go to the larger IoU, then the smaller anchor
 * index; np.random.choice of the dropped negatives -> a seeded random subset.
 * m3d_rpn_targets synchronises the stream once at the end (host counts_out[2]
 * = final (positives, negatives) if non-NULL; M3D_EINVAL if a GT overlapped
 * more than list_cap anchors).  m3d_rpn_targets_async is the same computation
 * fully stream-ordered (balancing set up on the device, no host round trip,
 * hipGraph-capturable) for building the targets inside a training step:
 * counts_dev (DEVICE int32[3], may be NULL) = positives, negatives, list
 * overflow flag.
 * workspace: m3d_rpn_targets_workspace_bytes(A, G, list_cap). */
size_t m3d_rpn_targets_workspace_bytes(int64_t A, int64_t G, int64_t list_cap);
int m3d_rpn_targets(const float* anchors, int64_t A, const float* gt_boxes, int64_t G,
                    float pos_iou, float neg_iou, int32_t total, float positive_ratio,
                    int32_t atss_topk, int32_t atss_min_pos, const float rpn_bbox_std_dev[6],
                    uint32_t seed, int8_t* rpn_match, float* rpn_bbox, int64_t list_cap,
                    void* workspace, size_t ws_bytes, int32_t* counts_out, m3d_stream_t s);
int m3d_rpn_targets_async(const float* anchors, int64_t A, const float* gt_boxes, int64_t G,
                          float pos_iou, float neg_iou, int32_t total, float positive_ratio,
                          int32_t atss_topk, int32_t atss_min_pos, const float rpn_bbox_std_dev[6],
                          uint32_t seed, int8_t* rpn_match, float* rpn_bbox, int64_t list_cap,
                          void* workspace, size_t ws_bytes, int32_t* counts_dev, m3d_stream_t s);

/* RPN training losses with their gradients in one pass: rpn_class_loss_graph
 * (core/models.py:1589-1625, focal CE, alpha / gamma) and rpn_bbox_loss_graph
 * (core/models.py:1629-1673, clipped XY/Z Huber), weighted (core/models.py:
 * 3366-3376).  logits [A,2], pred [A,6] (A = all anchors of the batch,
 * flattened), match [A] int8 (1 / -1 / 0), row [A] int32 = the positive's row
 * in gt_bbox [n_gt,6] (n_gt >= 1; read for match == 1 only, clamped).
 * den_cls / den_pos: the K.mean denominators (anchors with match != 0,
 * positives) when > 0, else counted here.  Writes the scalars total (=
 * w_cls * class + w_box * bbox), cls_loss, box_loss, scales[2] = {w_cls /
 * den_cls, w_box / (6 den_pos)} and the unnormalised gradients g_logits [A,2],
 * g_pred [A,6]; m3d_rpn_loss_bwd scales them in place by *g_total * scales[0]
 * (logits) / scales[1] (pred).  Fixed-order sums.
 * workspace: m3d_rpn_loss_workspace_bytes(A). */
size_t m3d_rpn_loss_workspace_bytes(int64_t A);
int m3d_rpn_loss_fwd(const float* logits, const float* pred, const int8_t* match, const int32_t* row,
                     const float* gt_bbox, int64_t n_gt, int64_t A, float alpha, float gamma,
                     int64_t den_cls, int64_t den_pos, float w_cls, float w_box, float* g_logits,
                     float* g_pred, float* total, float* cls_loss, float* box_loss, float* scales,
                     void* workspace, size_t ws_bytes, m3d_stream_t s);
int m3d_rpn_loss_bwd(float* g_logits, float* g_pred, int64_t A, const float* g_total, const float* scales,
                     m3d_stream_t s);

/* ---------------------------------------------------------------------------
 * Elementwise / reduction kernels of the backbone-FPN-RPN graph.
 * ------------------------------------------------------------------------- */
/* KL.MaxPooling3D(k, strides, padding='same'|'valid') (core/models.py:245,3211);
 * argmax [B,OH,OW,OD,C] uint8 window index for the backward (may be NULL). */
int m3d_maxpool3d_fwd(const float* x, int64_t B, int64_t H, int64_t W, int64_t D, int64_t C,
                      int32_t kh, int32_t kw, int32_t kd, int32_t sy, int32_t sx, int32_t sz,
                      int32_t py, int32_t px, int32_t pz, int64_t OH, int64_t OW, int64_t OD,
                      float* y, uint8_t* argmax, m3d_stream_t s);
int m3d_maxpool3d_bwd(const float* dy, const uint8_t* argmax, int64_t B, int64_t H, int64_t W,
                      int64_t D, int64_t C, int32_t kh, int32_t kw, int32_t kd, int32_t sy,
                      int32_t sx, int32_t sz, int32_t py, int32_t px, int32_t pz, int64_t OH,
                      int64_t OW, int64_t OD, float* dx, m3d_stream_t s);
/* Depth-slab form of the pool (core/models.py:245 on one z-slab of the volume):
 * x [B,H,W,Dl,C] is the local slab and halo [B,H,W,2r,C] the neighbours' r
 * boundary planes (planes [0,r) from below, [r,2r) from above; has_lo / has_hi:
 * that neighbour exists), read beside the slab instead of a halo-extended copy;
 * z window kd = 2r+1 at stride 1 with 'same' pad pz = r (applied only where the
 * volume ends), OD = Dl, C % 4 == 0.  The backward writes dx [B,H,W,Dl,C] and
 * dhalo [B,H,W,2r,C] (the gradient of the neighbours' planes, to be returned to
 * them).  Values and summation order are those of the pool on the extended slab. */
int m3d_maxpool3d_fwd_halo(const float* x, const float* halo, int32_t has_lo, int32_t has_hi, int32_t r,
                           int64_t B, int64_t H, int64_t W, int64_t Dl, int64_t C, int32_t kh, int32_t kw,
                           int32_t kd, int32_t sy, int32_t sx, int32_t sz, int32_t py, int32_t px, int32_t pz,
                           int64_t OH, int64_t OW, int64_t OD, float* y, uint8_t* argmax, m3d_stream_t s);
int m3d_maxpool3d_bwd_halo(const float* dy, const uint8_t* argmax, int32_t has_lo, int32_t has_hi, int32_t r,
                           int64_t B, int64_t H, int64_t W, int64_t Dl, int64_t C, int32_t kh, int32_t kw,
                           int32_t kd, int32_t sy, int32_t sx, int32_t sz, int32_t py, int32_t px, int32_t pz,
                           int64_t OH, int64_t OW, int64_t OD, float* dx, float* dhalo, m3d_stream_t s);
/* d_src[b,y,x,z,c] (+)= sum_{i,j in {0,1}} d_up[b,2y+i,2x+j,z,c]  (UpSampling3D((2,2,1)) bwd) */
int m3d_upsample221_bwd(const float* d_up, int64_t B, int64_t H, int64_t W, int64_t D, int64_t C,
                        float* d_src, int32_t accumulate, m3d_stream_t s);
/* y = x[:, ::2, ::2, :, :] (P6, core/models.py:3211) and its adjoint (accumulate into dx). */
int m3d_subsample221_fwd(const float* x, int64_t B, int64_t H, int64_t W, int64_t D, int64_t C,
                         float* y, m3d_stream_t s);
int m3d_subsample221_bwd(const float* dy, int64_t B, int64_t H, int64_t W, int64_t D, int64_t C,
                         float* dx, m3d_stream_t s);
/* Frozen BatchNorm affine of one layer (core/models.py:102-114, inference
 * mode): rstd = 1/sqrt(var+eps), scale = gamma*rstd, shift = beta - mean*scale. */
int m3d_bn_affine(const float* gamma, const float* beta, const float* mean, const float* var,
                  float eps, int64_t C, float* scale, float* shift, float* rstd, m3d_stream_t s);
/* Every frozen-BN affine of a model in one launch (the same expressions as
 * m3d_bn_affine, bit-identical): items is a DEVICE array of n descriptors, one
 * per BatchNorm layer; item i writes out[0..C) = rstd, out[C..2C) = scale,
 * out[2C..3C) = shift.  max_c >= every item's C.  Replaces the per-layer
 * affine of each BatchNorm call in the backbone's forward (core/models.py:
 * 102-114: KL.BatchNormalization(training=False) after every Conv3D). */
typedef struct m3d_bn_affine_item {
    const float* gamma;
    const float* beta;
    const float* mean;
    const float* var;
    float* out;
    float eps;
    int32_t C;
} m3d_bn_affine_item_t;
int m3d_bn_affine_batched(const m3d_bn_affine_item_t* items, int32_t n, int64_t max_c, m3d_stream_t s);

/* Backward of y = act(z*scale + shift [+ residual]) for frozen-statistics BN
 * (TRAIN_BN=False).  dpre = dy * (y > 0 if relu); dz = dpre*scale (or dpre;
 * dz may be NULL when not needed); dres = dpre (may be NULL; accumulate_res
 * adds into it).  Per-channel sums, each added (+=) into its destination when
 * non-NULL, in a fixed order (deterministic, no float atomics):
 *   sum_dpre[c] += sum dpre, sum_dpre_xhat[c] += sum dpre*(z-mean)*rstd,
 *   sum_dz[c] += sum dz.
 * With all three sums NULL it is elementwise only (no workspace needed); with
 * dz and dres NULL it computes the sums only.
 * workspace: m3d_bn_act_bwd_workspace_bytes(M, C) bytes of device scratch. */
size_t m3d_bn_act_bwd_workspace_bytes(int64_t M, int64_t C);
int m3d_bn_act_bwd(const float* dy, const float* y, const float* z, int64_t M, int64_t C,
                   int32_t relu, const float* scale, const float* mean, const float* rstd,
                   float* dz, float* dres, int32_t accumulate_res, float* sum_dpre,
                   float* sum_dpre_xhat, float* sum_dz, void* workspace, size_t ws_bytes,
                   m3d_stream_t s);
/* Column sums of up to M3D_COL_SUMS_MAX row-major [M, C] matrices in two
 * launches: out[c] += sum_m x[m*C + c] per item -- the bias gradients of the
 * bias-only conv units (tf.nn.bias_add's gradient; the FPN's fpn_c*p* /
 * fpn_p* and the RPN class/bbox heads, core/models.py:3190-3214, 540-556),
 * collected during the backward and reduced together.  Each item's sum is
 * bit-identical to m3d_bn_act_bwd(x, ..., relu 0, scale NULL, sum_dz = out)
 * (same block geometry and summation order).  No two items may share `out`.
 * C % 4 == 0; items is a host array (copied into the launch); workspace:
 * m3d_col_sums_batched_workspace_bytes of the same items. */
#define M3D_COL_SUMS_MAX 16
typedef struct {
    const float* x;
    int64_t M;
    int64_t C;
    float* out;
} m3d_col_sums_item_t;
size_t m3d_col_sums_batched_workspace_bytes(const m3d_col_sums_item_t* items, int32_t n);
int m3d_col_sums_batched(const m3d_col_sums_item_t* items, int32_t n, void* workspace, size_t ws_bytes,
                         m3d_stream_t s);
/* Keras 2.3.1 SGD (momentum, per-tensor tf.clip_by_norm, decayed lr computed
 * by the caller) plus the RPN L2 term wd*0.5*||w||^2/size(w) whose gradient
 * l2_coef[seg]*w is added first (core/models.py:3340-3387).  params / grads /
 * moments are one flat buffer of n_chunks*1024 floats; every tensor is a
 * segment padded to whole 1024-float chunks; seg_of_chunk[n_chunks] maps a
 * chunk to its segment; norms is [n_segments] device scratch. */
int m3d_sgd_keras(float* params, const float* grads, float* moments, int64_t n_chunks,
                  const int32_t* seg_of_chunk, const float* l2_coef, int32_t n_segments,
                  float lr, float momentum, float clipnorm, float* norms, const m3d_det_t* det, m3d_stream_t s);
/* Keras 2.3.1 Adam (keras.optimizers.Adam, the `else` branch of RPN.compile,
 * core/models.py:3356-3357) on the same flat buffers: m, v (and vhat when
 * amsgrad; NULL otherwise) are [n_chunks*1024] moment buffers, lr_t =
 * lr_decayed*sqrt(1-beta_2^t)/(1-beta_1^t) (t = iterations+1) is computed by
 * the caller, epsilon defaults to K.epsilon() = 1e-7 in Keras. */
int m3d_adam_keras(float* params, const float* grads, float* m, float* v, float* vhat,
                   int64_t n_chunks, const int32_t* seg_of_chunk, const float* l2_coef,
                   int32_t n_segments, float lr_t, float beta_1, float beta_2, float epsilon,
                   float clipnorm, float* norms, const m3d_det_t* det, m3d_stream_t s);
/* Keras 2.3.1 Adadelta (core/models.py:3354-3355): accum / delta_accum are the
 * accumulators of keras.optimizers.Adadelta, lr the decayed learning rate. */
int m3d_adadelta_keras(float* params, const float* grads, float* accum, float* delta_accum,
                       int64_t n_chunks, const int32_t* seg_of_chunk, const float* l2_coef,
                       int32_t n_segments, float lr, float rho, float epsilon, float clipnorm,
                       float* norms, const m3d_det_t* det, m3d_stream_t s);

#ifdef __cplusplus
}
#endif
#endif /* M3D_H */
