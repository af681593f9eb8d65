"""Drop-in replacement for the reference's core/custom_op/custom_op.py (TF 2.2).

The reference imports four op wrappers from the CPU-only wheel
tensorflow_nms_car_3d==0.1.0 (core/custom_op/custom_op.py:22-25) and registers
the CropAndResize3D gradient (custom_op.py:28-65).  This module exports the
same four callables with the same signatures, backed by the GPU kernels of
m3d_tf_ops.cc (which forward TF's device buffers and stream to libm3d.so), and
registers the same gradient.  Copy it over core/custom_op/custom_op.py; nothing
in core/models.py changes: PyramidROIAlign (core/models.py:663), the mask
targets (:992) and ProposalLayer (:453) keep calling
crop_and_resize_3d / non_max_suppression_3d with tf.Tensors inside the graph.

Not executed in this repository (TensorFlow is absent from the image); the
ops it binds are the ones tests/test_gpu_roi_nms.py checks through the C-ABI.
"""
import os

import tensorflow as tf
from tensorflow.python.framework import dtypes, ops
from tensorflow.python.ops import array_ops

_LIB = tf.load_op_library(os.environ.get(
    "M3D_TF_OPS", os.path.join(os.path.dirname(os.path.abspath(__file__)), "_m3d_tf_ops.so")))


def _op(*names):
    # tf.load_op_library's generated wrapper names (snake_case of the op name;
    # the digit boundary is spelled either way across TF versions)
    for n in names:
        if hasattr(_LIB, n):
            return getattr(_LIB, n)
    raise AttributeError(f"{names[0]} not in {_LIB}")


# same argument names and defaults as the wheel's wrappers
crop_and_resize_3d = _op("crop_and_resize3d", "crop_and_resize_3d")
crop_and_resize_3d_grad_image = _op("crop_and_resize3d_grad_image", "crop_and_resize_3d_grad_image")
crop_and_resize_3d_grad_boxes = _op("crop_and_resize3d_grad_boxes", "crop_and_resize_3d_grad_boxes")
non_max_suppression_3d = _op("non_max_suppression3d", "non_max_suppression_3d")


@ops.RegisterGradient("CropAndResize3D")
def _CropAndResize3DGrad(op, grad):
    """[grad_image, grad_boxes, None, None], as custom_op.py:28-65: the image
    gradient only for floating images, the box gradient always (trilinear
    formula also for 'nearest')."""
    image = op.inputs[0]
    if image.get_shape().is_fully_defined():
        image_shape = image.get_shape().as_list()
    else:
        image_shape = array_ops.shape(image)
    if image.dtype in (dtypes.float16, dtypes.float32, dtypes.float64):
        grad0 = crop_and_resize_3d_grad_image(grad, op.inputs[1], op.inputs[2], image_shape,
                                              T=op.get_attr("T"), method_name=op.get_attr("method_name"))
    else:
        grad0 = None
    grad1 = crop_and_resize_3d_grad_boxes(grad, op.inputs[0], op.inputs[1], op.inputs[2])
    return [grad0, grad1, None, None]
