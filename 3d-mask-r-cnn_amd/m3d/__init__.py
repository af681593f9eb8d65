"""m3d -- MI355X-native (gfx950) hot path of podtyazhki1337/3d-mask-r-cnn.

Drop-in surface:
  m3d.ops      crop_and_resize_3d / _grad_image / _grad_boxes, non_max_suppression_3d,
               pyramid_roi_align (core/custom_op/custom_op.py:22-65)
  m3d.layers   ProposalLayer, PyramidROIAlign (core/models.py:369-503, 597-687)
  m3d.backbone ResNet3D (resnet_graph), FPN, RPNHead (build_rpn_model)
  m3d.model    RPN training model, losses, synthetic inputs
  m3d.config   Config / load_config (core/config.py)
  m3d.parallel depth-slab sharding + RCCL gradient all-reduce
All compute runs in libm3d.so (hand-written HIP for gfx950); there is no CPU
fallback.
"""
from . import config  # noqa: F401

__all__ = ["config", "ops", "layers", "backbone", "model", "anchors"]
