"""ctypes binding of libm3d.so (the C-ABI declared in include/m3d.h).

torch is imported first on purpose: libm3d.so links libamdhip64.so.7 and must
bind to the HIP runtime torch already loaded (same SONAME), never to a second
copy from /opt/rocm.  There is no fallback: if the library is missing or fails
to load, every op raises.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
# M3D_LIB_FILE: another build of the same sources in this directory (A/B runs)
LIB_PATH = os.path.join(_HERE, os.environ.get("M3D_LIB_FILE", "libm3d.so"))

_lib = None

c_i32 = ctypes.c_int32
c_i64 = ctypes.c_int64
c_f = ctypes.c_float
c_p = ctypes.c_void_p
c_sz = ctypes.c_size_t


class Det(ctypes.Structure):
    """m3d_det_t (include/m3d.h): the deterministic-reduction target of one call."""
    _fields_ = [("on", ctypes.c_int32), ("scratch", ctypes.c_void_p), ("bytes", ctypes.c_size_t)]


class BnBwd(ctypes.Structure):
    """m3d_bn_bwd_t (include/m3d.h): the producing unit's BN-ReLU backward fused
    into a data-gradient epilogue."""
    _fields_ = [("y", ctypes.c_void_p), ("z", ctypes.c_void_p), ("scale", ctypes.c_void_p),
                ("mean", ctypes.c_void_p), ("rstd", ctypes.c_void_p), ("relu", ctypes.c_int32),
                ("dres", ctypes.c_void_p), ("sum_dpre", ctypes.c_void_p), ("sum_dpre_xhat", ctypes.c_void_p),
                ("sum_dz", ctypes.c_void_p)]

# name -> argtypes (all return int unless listed in _RESTYPES)
_SIGS = {
    "m3d_last_error": [],
    "m3d_abi_version": [],
    "m3d_crop_and_resize3d_fwd": [c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_i64,
                                  c_i32, c_i32, c_i32, c_i32, c_f, c_p, c_p],
    "m3d_crop_and_resize3d_bwd_image": [c_p, c_p, c_p, c_i64, c_i32, c_i32, c_i32, c_i64, c_i64,
                                        c_i64, c_i64, c_i64, c_i32, c_i32, c_p, c_p],
    "m3d_crop_and_resize3d_bwd_boxes": [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p,
                                        c_i64, c_i32, c_i32, c_i32, c_p, c_p],
    "m3d_pyramid_roi_align3d_fwd": [c_p, c_p, c_i64, c_p, c_p, c_i64, c_i64, c_i64, c_i32, c_i32,
                                    c_i32, c_p, c_p, c_p, c_p],
    "m3d_pyramid_roi_align3d_fwd_ws": [c_p, c_p, c_i64, c_p, c_p, c_i64, c_i64, c_i64, c_i32, c_i32,
                                       c_i32, c_p, c_p, c_p, c_p, c_sz, c_p],
    "m3d_pyramid_roi_align3d_fwd_workspace_bytes": [c_p, c_i64, c_i64, c_i32, c_i32],
    "m3d_pyramid_roi_align3d_bwd": [c_p, c_p, c_p, c_i64, c_i64, c_i32, c_i32, c_i32, c_p, c_p,
                                    c_i64, c_p],
    "m3d_pyramid_roi_align3d_bwd_det": [c_p, c_p, c_p, c_i64, c_i64, c_i32, c_i32, c_i32, c_p, c_p,
                                        c_i64, c_p, c_p],
    "m3d_mask_targets3d": [c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_i64, c_i32, c_i32, c_i32,
                           c_p, c_p],
    "m3d_nms3d_workspace_bytes": [c_i64],
    "m3d_nms3d": [c_p, c_p, c_i64, c_i32, c_f, c_i32, c_p, c_p, c_p, c_sz, c_p],
    "m3d_score_keys": [c_p, c_i64, c_p, c_p],
    "m3d_topk_workspace_bytes": [c_i64, c_i64],
    "m3d_topk_keys": [c_p, c_i64, c_i64, c_p, c_p, c_p, c_sz, c_p],
    "m3d_score_keys_mapped": [c_p, c_i64, c_p, c_p, c_p],
    "m3d_proposal_decode": [c_p, c_p, c_p, c_i64, c_p, c_i64, c_p, c_f, c_p, c_p, c_p, c_p],
    "m3d_proposal_gather": [c_p, c_p, c_p, c_i32, c_p, c_p],
    "m3d_conv3d_fwd": [c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i32, c_i32, c_i32, c_i64,
                       c_i64, c_i64, c_i64, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_p, c_p,
                       c_p, c_p, c_i32, c_i32, c_p, c_p, c_i64, c_p, c_i64, c_i64, c_p],
    "m3d_conv3d_splitk_count": [c_i64, c_i64, c_i64],
    "m3d_conv3d_fwd_splitk": [c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_i64, c_i64, c_i64, c_i32,
                              c_i32, c_i32, c_p, c_p, c_p, c_p, c_i32, c_i32, c_p, c_p, c_i32, c_p, c_sz, c_p],
    "m3d_conv3d_bwd_data_splitk": [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64,
                                   c_i32, c_i32, c_i32, c_p, c_i32, c_i32, c_p, c_sz, c_p],
    "m3d_conv1_x3_planes": [c_p, c_i64, c_i64, c_i32, c_p, c_p],
    "m3d_conv1_x3_planes_batched": [c_p, c_i32, c_i64, c_p],
    "m3d_conv3d_fwd_x3": [c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_p, c_p, c_p, c_i32, c_i32,
                          c_p, c_p, c_p],
    "m3d_conv3d_bwd_data_x3": [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p],
    "m3d_conv3d_bwd_data_x3_bn": [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_sz, c_p],
    "m3d_conv3d_wino_v_bytes": [c_i64, c_i64, c_i32, c_i32],
    "m3d_conv3d_wino_weight_v": [c_p, c_i64, c_i64, c_i32, c_i32, c_p, c_sz, c_p],
    "m3d_conv3d_fwd_wino_kv": [c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_i64, c_i32, c_p, c_p, c_p, c_p,
                               c_i32, c_p, c_p, c_p, c_p, c_p, c_sz, c_p],
    "m3d_conv3d_bwd_data_wino_xv": [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_p, c_i32,
                                    c_p, c_sz, c_p, c_i32, c_p, c_p, c_sz, c_p],
    "m3d_conv3d_bwd_data_x3_bna": [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i32, c_p, c_p, c_sz,
                                   c_p],
    "m3d_conv3d_fwd_wino_v": [c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_i64, c_i32, c_p, c_p, c_p, c_p,
                              c_i32, c_p, c_p, c_p, c_sz, c_i32, c_p],
    "m3d_conv3d_bwd_data_wino_v": [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_p, c_i32, c_p,
                                   c_sz, c_i32, c_p],
    "m3d_conv3d_bwd_data_wino_vy": [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_p, c_i32,
                                    c_p, c_sz, c_i32, c_i32, c_p],
    "m3d_conv3d_bwd_data_wino_bny": [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_p, c_i32,
                                     c_p, c_sz, c_i32, c_p, c_p, c_sz, c_i32, c_p],
    "m3d_bn_bwd_fused_workspace_bytes": [c_i64, c_i64, c_i64, c_i64, c_i64],
    "m3d_conv3d_bwd_data_bn": [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_i32, c_i32,
                               c_i64, c_i64, c_i64, c_i64, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32,
                               c_p, c_i32, c_p, c_p, c_sz, c_p],
    "m3d_conv3d_bwd_data_wino_bn": [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_p, c_i32,
                                    c_p, c_sz, c_i32, c_p, c_p, c_sz, c_p],
    "m3d_conv3d_bwd_data_splitk_bn": [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i32, c_i32,
                                      c_p, c_sz, c_p, c_p, c_sz, c_p],
    "m3d_conv3d_bwd_data": [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_i32, c_i32,
                            c_i64, c_i64, c_i64, c_i64, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32,
                            c_p, c_i32, c_p],
    "m3d_conv3d_bwd_weight": [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_i32, c_i32,
                              c_i64, c_i64, c_i64, c_i64, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32,
                              c_p, c_p, c_p],
    "m3d_conv3d_fwd_wino_halo": [c_p, c_p, c_i32, c_i32, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_p,
                                 c_p, c_p, c_i32, c_p, c_p, c_p, c_p, c_sz, c_p],
    "m3d_conv3d_fwd_wino_halo_phase": [c_p, c_p, c_i32, c_i32, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_p,
                                       c_p, c_p, c_p, c_i32, c_p, c_p, c_p, c_p, c_sz, c_i32, c_p],
    "m3d_conv3d_bwd_data_wino_halo": [c_p, c_p, c_i32, c_i32, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_p,
                                      c_p, c_i32, c_p, c_sz, c_p],
    "m3d_conv3d_bwd_weight_wino_halo": [c_p, c_p, c_i32, c_i32, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64,
                                        c_p, c_p, c_sz, c_p, c_p],
    "m3d_gemm_f32": [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_i32, c_i32, c_p],
    "m3d_gemm_wgrad_f32": [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_p],
    "m3d_split3_f32": [c_p, c_i64, c_p, c_p],
    "m3d_gemm_x3": [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_p],
    "m3d_gemm_x3_af": [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_p],
    "m3d_conv3d_wino_workspace_bytes": [c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64],
    "m3d_conv3d_fwd_wino": [c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_i64, c_i32, c_p,
                            c_p, c_p, c_p, c_i32, c_p, c_p, c_p, c_sz, c_p],
    "m3d_conv3d_bwd_data_wino": [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32,
                                 c_p, c_i32, c_p, c_sz, c_p],
    "m3d_conv3d_bwd_weight_wino": [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64,
                                   c_i32, c_p, c_p, c_sz, c_p, c_p],
    "m3d_conv3d_wino_u_bytes": [c_i64, c_i64, c_i64, c_i64, c_i64],
    "m3d_conv3d_wino_tile_z": [],
    "m3d_conv3d_wino_wgrad_tile_z": [],
    "m3d_conv3d_wino_tile_y": [],
    "m3d_conv3d_wino_dgrad_workspace_bytes": [c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32],
    "m3d_conv3d_wino_dgrad_tile_y": [],
    "m3d_conv3d_wino_dgrad_tile_z": [],
    "m3d_conv3d_fwd_wino_keep": [c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_i64, c_i32, c_p,
                                 c_p, c_p, c_p, c_i32, c_p, c_p, c_p, c_p, c_sz, c_p],
    "m3d_conv3d_bwd_weight_wino_u": [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64,
                                     c_i32, c_p, c_p, c_sz, c_p, c_p],
    "m3d_gemm_f32_ex": [c_p, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p,
                        c_i32, c_i32, c_p],
    "m3d_splitk_reduce": [c_p, c_i32, c_i64, c_i64, c_p, c_p, c_p, c_i32, c_p, c_p],
    "m3d_conv3d_fwd_dil": [c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i32, c_i32, c_i32, c_i64,
                           c_i64, c_i64, c_i64, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32,
                           c_i32, c_i32, c_p, c_p, c_p, c_p, c_i32, c_i32, c_p, c_p, c_i64, c_p,
                           c_i64, c_i64, c_p],
    "m3d_deconv3d_k2s2": [c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i32, c_p, c_p],
    "m3d_head_outputs": [c_p, c_i64, c_i64, c_i32, c_p, c_p, c_p, c_p],
    "m3d_refine_detections": [c_p, c_p, c_p, c_i64, c_i32, c_p, c_p, c_f, c_p, c_p, c_p, c_p],
    "m3d_detections_gather": [c_p, c_p, c_p, c_p, c_i32, c_p, c_p, c_p],
    "m3d_detection_targets_workspace_bytes": [c_i64],
    "m3d_detection_targets": [c_p, c_i64, c_p, c_p, c_i64, c_i32, c_f, c_f, c_f, c_p, c_i32, ctypes.c_uint32,
                              c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_sz, c_p],
    "m3d_rpn_targets_workspace_bytes": [c_i64, c_i64, c_i64],
    "m3d_rpn_targets": [c_p, c_i64, c_p, c_i64, c_f, c_f, c_i32, c_f, c_i32, c_i32, c_p, ctypes.c_uint32, c_p,
                        c_p, c_i64, c_p, c_sz, c_p, c_p],
    "m3d_rpn_targets_async": [c_p, c_i64, c_p, c_i64, c_f, c_f, c_i32, c_f, c_i32, c_i32, c_p, ctypes.c_uint32,
                              c_p, c_p, c_i64, c_p, c_sz, c_p, c_p],
    "m3d_rpn_loss_workspace_bytes": [c_i64],
    "m3d_rpn_loss_fwd": [c_p, c_p, c_p, c_p, c_p, c_i64, c_i64, c_f, c_f, c_i64, c_i64, c_f, c_f, c_p, c_p, c_p,
                         c_p, c_p, c_p, c_p, c_sz, c_p],
    "m3d_rpn_loss_bwd": [c_p, c_p, c_i64, c_p, c_p, c_p],
    "m3d_maxpool3d_fwd": [c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_i32, c_i32, c_i32,
                          c_i32, c_i32, c_i32, c_i32, c_i32, c_i64, c_i64, c_i64, c_p, c_p, c_p],
    "m3d_maxpool3d_bwd": [c_p, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_i32, c_i32, c_i32,
                          c_i32, c_i32, c_i32, c_i32, c_i32, c_i64, c_i64, c_i64, c_p, c_p],
    "m3d_conv3d_fwd_halo": [c_p, c_p, c_i32, c_i32, c_i32, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i32, c_i32,
                            c_i32, c_i64, c_i64, c_i64, c_i64, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_p, c_p,
                            c_p, c_i32, c_p, c_p, c_p],
    "m3d_conv3d_bwd_weight_halo": [c_p, c_p, c_i32, c_i32, c_i32, c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32,
                                   c_i32, c_i32, c_i64, c_i64, c_i64, c_i64, c_i32, c_i32, c_i32, c_i32, c_i32,
                                   c_i32, c_p, c_p, c_p],
    "m3d_maxpool3d_fwd_halo": [c_p, c_p, c_i32, c_i32, c_i32, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_i32,
                               c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i64, c_i64, c_i64, c_p, c_p,
                               c_p],
    "m3d_maxpool3d_bwd_halo": [c_p, c_p, c_i32, c_i32, c_i32, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_i32,
                               c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i64, c_i64, c_i64, c_p, c_p,
                               c_p],
    "m3d_upsample221_bwd": [c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_i32, c_p],
    "m3d_subsample221_fwd": [c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p],
    "m3d_subsample221_bwd": [c_p, c_i64, c_i64, c_i64, c_i64, c_i64, c_p, c_p],
    "m3d_bn_affine": [c_p, c_p, c_p, c_p, c_f, c_i64, c_p, c_p, c_p, c_p],
    "m3d_bn_affine_batched": [c_p, c_i32, c_i64, c_p],
    "m3d_bn_act_bwd_workspace_bytes": [c_i64, c_i64],
    "m3d_bn_act_bwd": [c_p, c_p, c_p, c_i64, c_i64, c_i32, c_p, c_p, c_p, c_p, c_p, c_i32, c_p,
                       c_p, c_p, c_p, c_sz, c_p],
    "m3d_col_sums_batched_workspace_bytes": [c_p, c_i32],
    "m3d_col_sums_batched": [c_p, c_i32, c_p, c_sz, c_p],
    "m3d_sgd_keras": [c_p, c_p, c_p, c_i64, c_p, c_p, c_i32, c_f, c_f, c_f, c_p, c_p, c_p],
    "m3d_adam_keras": [c_p, c_p, c_p, c_p, c_p, c_i64, c_p, c_p, c_i32, c_f, c_f, c_f, c_f, c_f, c_p,
                       c_p, c_p],
    "m3d_adadelta_keras": [c_p, c_p, c_p, c_p, c_i64, c_p, c_p, c_i32, c_f, c_f, c_f, c_f, c_p, c_p, c_p],
    "m3d_fork_event_create": [c_i32, ctypes.POINTER(c_p)],
    "m3d_fork_event_destroy": [c_p],
    "m3d_stream_fork": [c_p, c_p, c_p],
}
_RESTYPES = {"m3d_last_error": ctypes.c_char_p, "m3d_nms3d_workspace_bytes": c_sz,
             "m3d_topk_workspace_bytes": c_sz,
             "m3d_pyramid_roi_align3d_fwd_workspace_bytes": c_sz,
             "m3d_detection_targets_workspace_bytes": c_sz, "m3d_rpn_targets_workspace_bytes": c_sz,
             "m3d_rpn_loss_workspace_bytes": c_sz,
             "m3d_bn_act_bwd_workspace_bytes": c_sz, "m3d_bn_bwd_fused_workspace_bytes": c_sz, "m3d_conv3d_splitk_count": c_i32, "m3d_conv3d_wino_workspace_bytes": c_sz, "m3d_conv3d_wino_dgrad_workspace_bytes": c_sz, "m3d_conv3d_wino_v_bytes": c_sz,
             "m3d_conv3d_wino_u_bytes": c_sz, "m3d_conv3d_wino_tile_z": c_i32, "m3d_conv3d_wino_wgrad_tile_z": c_i32,
             "m3d_conv3d_wino_tile_y": c_i32, "m3d_conv3d_wino_dgrad_tile_y": c_i32,
             "m3d_conv3d_wino_dgrad_tile_z": c_i32, "m3d_col_sums_batched_workspace_bytes": c_sz}

EXPORTED = tuple(_SIGS)


class M3DError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load libm3d.so and attach signatures.  Raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise M3DError(
            f"libm3d.so not found at {path}: build it with `make -C 3d-mask-r-cnn_amd` "
            "(or __graft_entry__.build()); there is no CPU fallback")
    lib = ctypes.CDLL(path)
    for name, args in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = _RESTYPES.get(name, ctypes.c_int)
    _lib = _Lib(lib)
    return _lib


# Entry points taking a per-call m3d_det_t before their stream (ABI 3).  Called
# through load() with the ABI-2 argument list, they receive the deterministic
# target of this process's mode (set_deterministic) -- the mode is the host's
# choice, kept here; libm3d itself holds none.
DET_ENTRY_POINTS = ("m3d_conv3d_bwd_weight", "m3d_conv3d_bwd_weight_halo", "m3d_conv3d_bwd_weight_wino",
                    "m3d_conv3d_bwd_weight_wino_u", "m3d_conv3d_bwd_weight_wino_halo", "m3d_gemm_wgrad_f32",
                    "m3d_sgd_keras", "m3d_adam_keras", "m3d_adadelta_keras")


class BnAffineItem(ctypes.Structure):
    """m3d_bn_affine_item_t (include/m3d.h)."""
    _fields_ = [("gamma", ctypes.c_void_p), ("beta", ctypes.c_void_p), ("mean", ctypes.c_void_p),
                ("var", ctypes.c_void_p), ("out", ctypes.c_void_p), ("eps", ctypes.c_float),
                ("C", ctypes.c_int32)]


class X3PlanesItem(ctypes.Structure):
    """m3d_x3_planes_item_t (include/m3d.h)."""
    _fields_ = [("w", ctypes.c_void_p), ("fwd", ctypes.c_void_p), ("bwd", ctypes.c_void_p),
                ("cin", ctypes.c_int32), ("cout", ctypes.c_int32)]


class ColSumsItem(ctypes.Structure):
    """m3d_col_sums_item_t (include/m3d.h)."""
    _fields_ = [("x", ctypes.c_void_p), ("M", ctypes.c_int64), ("C", ctypes.c_int64), ("out", ctypes.c_void_p)]


COL_SUMS_MAX = 16          # M3D_COL_SUMS_MAX


class _Lib:
    """The loaded CDLL; the DET_ENTRY_POINTS called without their det argument
    get det_arg() inserted before the stream."""

    def __init__(self, cdll):
        self._cdll = cdll
        # every signed entry point bound on the instance: an attribute lookup per
        # launch is then a dict hit, not a __getattr__ round trip (host enqueue)
        for name in _SIGS:
            setattr(self, name, getattr(cdll, name))
        for name in DET_ENTRY_POINTS:
            fn = getattr(cdll, name)
            n = len(fn.argtypes)

            def call(*args, _fn=fn, _n=n):
                if len(args) == _n - 1:
                    args = args[:-1] + (det_arg(),) + args[-1:]
                return _fn(*args)
            setattr(self, name, call)

    def __getattr__(self, name):
        return getattr(self._cdll, name)


def check(rc: int, what: str = "") -> None:
    if rc == 0:
        return
    msg = load().m3d_last_error().decode()
    if rc == -1:
        raise ValueError(msg)
    raise M3DError(f"{what}: {msg}")


def ptr(t) -> int:
    """Device pointer of a tensor (0/None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


try:                   # the raw current stream without a torch.cuda.Stream object per call
    _raw_stream = torch._C._cuda_getCurrentRawStream
    _cur_device = torch._C._cuda_getDevice
except AttributeError:  # pragma: no cover - other torch builds
    _raw_stream = None


def stream() -> int:
    """The current HIP stream of the current device (an int handle)."""
    if _raw_stream is not None:
        return _raw_stream(_cur_device())
    return torch.cuda.current_stream().cuda_stream


_DET = None            # (Det struct, scratch tensor) while deterministic mode is on


def det_arg():
    """The m3d_det_t pointer the DET_ENTRY_POINTS get in this process's mode
    (None = atomic reductions)."""
    return None if _DET is None else ctypes.addressof(_DET[0])


def deterministic() -> bool:
    return _DET is not None


def set_deterministic(on: bool = True, scratch_bytes: int = 256 << 20, device=None) -> None:
    """Bitwise run-to-run reproducible training: the weight-gradient m-splits
    and the clip norms are summed in a fixed order through a device scratch of
    ``scratch_bytes`` instead of fp32 atomics (every weight-gradient / optimizer
    call of this process passes it as its m3d_det_t).  The scratch is shared by
    those reductions, so they must stay ordered on one stream at a time (the
    training step's weight-gradient stream, then the optimizer after the join).
    A weight gradient larger than half the scratch runs unsplit (still
    deterministic, slower).  The PyramidROIAlign backward follows the same mode
    (m3d.ops)."""
    global _DET
    load()
    if not on:
        _DET = None
        return
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    buf = torch.empty(max(int(scratch_bytes), 4096) // 4, dtype=torch.float32, device=dev)
    _DET = (Det(1, buf.data_ptr(), buf.numel() * 4), buf)
