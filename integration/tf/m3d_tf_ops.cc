// TensorFlow (2.2, ROCm build) binding of libm3d.so: registers the four ops of
// the reference's wheel tensorflow_nms_car_3d==0.1.0 -- the op library that
// core/custom_op/custom_op.py:22-25 imports -- under the SAME op names, inputs,
// attrs and outputs, on DEVICE_GPU, each kernel forwarding
// TF's device buffers and TF's GPU stream to the C-ABI in include/m3d.h.
//
// The op definitions restate the wheel's op-def strings:
//   NonMaxSuppression3D       whl:_non_max_suppression_3d_ops.so@0x1cb02-0x1cb4c
//   CropAndResize3D           whl:_crop_and_resize_3d_ops.so@0x33f4
//   CropAndResize3DGradImage  whl:_crop_and_resize_3d_grad_image_ops.so@0x2c54
//   CropAndResize3DGradBoxes  whl:_crop_and_resize_3d_grad_boxes_ops.so@0x2af4
// Only DEVICE_GPU kernels are registered: load this library INSTEAD of the
// wheel's (custom_op_m3d.py), never next to it -- the op names collide.
//
// Build (needs a tensorflow-rocm 2.2 installation, absent from this image, so
// this file is not compiled here):
//   TF_CFLAGS=$(python -c 'import tensorflow as tf; print(" ".join(tf.sysconfig.get_compile_flags()))')
//   TF_LFLAGS=$(python -c 'import tensorflow as tf; print(" ".join(tf.sysconfig.get_link_flags()))')
//   hipcc -std=c++14 -shared -fPIC -O2 -DTENSORFLOW_USE_ROCM=1 m3d_tf_ops.cc \
//         -I../../include $TF_CFLAGS $TF_LFLAGS -L../../3d-mask-r-cnn_amd/m3d -lm3d \
//         -Wl,-rpath,'$ORIGIN/../../3d-mask-r-cnn_amd/m3d' -o _m3d_tf_ops.so

#define EIGEN_USE_GPU
#include "tensorflow/core/framework/op.h"
#include "tensorflow/core/framework/op_kernel.h"
#include "tensorflow/core/framework/shape_inference.h"
#include "tensorflow/core/framework/tensor.h"
#include "unsupported/Eigen/CXX11/Tensor"

#include <hip/hip_runtime.h>
#include <algorithm>

#include "m3d.h"

namespace tensorflow {
namespace {

using GPUDevice = Eigen::GpuDevice;
using shape_inference::InferenceContext;
using shape_inference::ShapeHandle;

// TF's stream for this kernel: the Eigen GPU device wraps the same hipStream_t
// StreamExecutor launches on, so libm3d's work is ordered with the rest of the
// graph without extra synchronisation.
m3d_stream_t stream_of(OpKernelContext* ctx) {
  return reinterpret_cast<m3d_stream_t>(ctx->eigen_device<GPUDevice>().stream());
}

// M3D_EINVAL carries the reference's InvalidArgument text; M3D_EHIP a launch error.
Status m3d_status(int rc) {
  if (rc == M3D_OK) return Status::OK();
  if (rc == M3D_EINVAL) return errors::InvalidArgument(m3d_last_error());
  return errors::Internal("libm3d: ", m3d_last_error());
}

int32 method_code(const string& m) { return m == "nearest" ? 1 : 0; }

// -------------------------------------------------------------- op definitions
REGISTER_OP("CropAndResize3D")
    .Input("image: T")
    .Input("boxes: float")
    .Input("box_index: int32")     // the wheel's name (its grad ops say box_ind)
    .Input("crop_size: int32")
    .Output("crops: float")
    .Attr("T: {uint8, uint16, int8, int16, int32, int64, half, float, double}")
    .Attr("method_name: {'trilinear', 'nearest'} = 'trilinear'")
    .Attr("extrapolation_value: float = 0")
    .SetShapeFn([](InferenceContext* c) {
      ShapeHandle image, boxes, crop;
      TF_RETURN_IF_ERROR(c->WithRank(c->input(0), 5, &image));
      TF_RETURN_IF_ERROR(c->WithRank(c->input(1), 2, &boxes));
      TF_RETURN_IF_ERROR(c->MakeShapeFromShapeTensor(3, &crop));
      TF_RETURN_IF_ERROR(c->WithRank(crop, 3, &crop));
      c->set_output(0, c->MakeShape({c->Dim(boxes, 0), c->Dim(crop, 0), c->Dim(crop, 1),
                                     c->Dim(crop, 2), c->Dim(image, 4)}));
      return Status::OK();
    });

REGISTER_OP("CropAndResize3DGradImage")
    .Input("grads: float")
    .Input("boxes: float")
    .Input("box_ind: int32")
    .Input("image_size: int32")
    .Output("output: T")
    .Attr("T: {float, half, double}")
    .Attr("method_name: {'trilinear', 'nearest'} = 'trilinear'")
    .SetShapeFn([](InferenceContext* c) {
      ShapeHandle out;
      TF_RETURN_IF_ERROR(c->MakeShapeFromShapeTensor(3, &out));
      TF_RETURN_IF_ERROR(c->WithRank(out, 5, &out));
      c->set_output(0, out);
      return Status::OK();
    });

REGISTER_OP("CropAndResize3DGradBoxes")
    .Input("grads: float")
    .Input("image: T")
    .Input("boxes: float")
    .Input("box_ind: int32")
    .Output("output: float")
    .Attr("T: {uint8, uint16, int8, int16, int32, int64, half, float, double}")
    .Attr("method_name: {'trilinear'} = 'trilinear'")
    .SetShapeFn([](InferenceContext* c) {
      c->set_output(0, c->input(2));
      return Status::OK();
    });

REGISTER_OP("NonMaxSuppression3D")
    .Input("boxes: float")
    .Input("scores: float")
    .Input("max_output_size: int32")
    .Output("selected_indices: int32")
    .Attr("iou_threshold: float = 0.5")
    .SetShapeFn([](InferenceContext* c) {
      ShapeHandle boxes, scores, max_out;
      TF_RETURN_IF_ERROR(c->WithRank(c->input(0), 2, &boxes));
      TF_RETURN_IF_ERROR(c->WithRank(c->input(1), 1, &scores));
      TF_RETURN_IF_ERROR(c->WithRank(c->input(2), 0, &max_out));
      c->set_output(0, c->Vector(c->UnknownDim()));
      return Status::OK();
    });

// -------------------------------------------------------------- kernels
// image [B,H,W,D,C] float, boxes [N,6], box_ind [N], crop_size host int32[3]
class CropAndResize3DOp : public OpKernel {
 public:
  explicit CropAndResize3DOp(OpKernelConstruction* ctx) : OpKernel(ctx) {
    string m;
    OP_REQUIRES_OK(ctx, ctx->GetAttr("method_name", &m));
    method_ = method_code(m);
    OP_REQUIRES_OK(ctx, ctx->GetAttr("extrapolation_value", &extrapolation_));
  }
  void Compute(OpKernelContext* ctx) override {
    const Tensor& image = ctx->input(0);
    const Tensor& boxes = ctx->input(1);
    const Tensor& box_ind = ctx->input(2);
    const Tensor& crop_size = ctx->input(3);  // HostMemory
    OP_REQUIRES(ctx, image.dims() == 5, errors::InvalidArgument("input image must be 5-D"));
    OP_REQUIRES(ctx, crop_size.NumElements() == 3,
                errors::InvalidArgument("crop_size must have three elements"));
    const auto cs = crop_size.vec<int32>();
    const int64 N = boxes.dim_size(0), C = image.dim_size(4);
    Tensor* crops = nullptr;
    OP_REQUIRES_OK(ctx, ctx->allocate_output(0, TensorShape({N, cs(0), cs(1), cs(2), C}), &crops));
    if (crops->NumElements() == 0) return;
    OP_REQUIRES_OK(ctx, m3d_status(m3d_crop_and_resize3d_fwd(
        image.flat<float>().data(), image.dim_size(0), image.dim_size(1), image.dim_size(2),
        image.dim_size(3), C, boxes.flat<float>().data(), box_ind.flat<int32>().data(), N,
        cs(0), cs(1), cs(2), method_, extrapolation_, crops->flat<float>().data(),
        stream_of(ctx))));
  }

 private:
  int32 method_;
  float extrapolation_;
};

// grads [N,ch,cw,cd,C], image_size host int32[5] -> [B,H,W,D,C]
class CropAndResize3DGradImageOp : public OpKernel {
 public:
  explicit CropAndResize3DGradImageOp(OpKernelConstruction* ctx) : OpKernel(ctx) {
    string m;
    OP_REQUIRES_OK(ctx, ctx->GetAttr("method_name", &m));
    method_ = method_code(m);
  }
  void Compute(OpKernelContext* ctx) override {
    const Tensor& grads = ctx->input(0);
    const Tensor& boxes = ctx->input(1);
    const Tensor& box_ind = ctx->input(2);
    const Tensor& image_size = ctx->input(3);  // HostMemory
    OP_REQUIRES(ctx, grads.dims() == 5, errors::InvalidArgument("grads image must be 5-D"));
    OP_REQUIRES(ctx, image_size.NumElements() == 5,
                errors::InvalidArgument("image_size must have five elements"));
    const auto is = image_size.vec<int32>();
    Tensor* out = nullptr;
    OP_REQUIRES_OK(ctx, ctx->allocate_output(0, TensorShape({is(0), is(1), is(2), is(3), is(4)}), &out));
    // the wheel's scatter is sequential; deterministic mode 1
    // reproduces its per-voxel summation order with one owner thread per
    // output voxel row (parallel, no atomics), so TF training stays bitwise
    // reproducible as with the reference op at GPU speed
    OP_REQUIRES_OK(ctx, m3d_status(m3d_crop_and_resize3d_bwd_image(
        grads.flat<float>().data(), boxes.flat<float>().data(), box_ind.flat<int32>().data(),
        grads.dim_size(0), grads.dim_size(1), grads.dim_size(2), grads.dim_size(3), is(0), is(1),
        is(2), is(3), is(4), method_, /*deterministic=*/1, out->flat<float>().data(),
        stream_of(ctx))));
  }

 private:
  int32 method_;
};

class CropAndResize3DGradBoxesOp : public OpKernel {
 public:
  explicit CropAndResize3DGradBoxesOp(OpKernelConstruction* ctx) : OpKernel(ctx) {}
  void Compute(OpKernelContext* ctx) override {
    const Tensor& grads = ctx->input(0);
    const Tensor& image = ctx->input(1);
    const Tensor& boxes = ctx->input(2);
    const Tensor& box_ind = ctx->input(3);
    OP_REQUIRES(ctx, grads.dims() == 5 && image.dims() == 5,
                errors::InvalidArgument("grads and image must be 5-D"));
    Tensor* out = nullptr;
    OP_REQUIRES_OK(ctx, ctx->allocate_output(0, boxes.shape(), &out));
    OP_REQUIRES_OK(ctx, m3d_status(m3d_crop_and_resize3d_bwd_boxes(
        grads.flat<float>().data(), image.flat<float>().data(), image.dim_size(0),
        image.dim_size(1), image.dim_size(2), image.dim_size(3), image.dim_size(4),
        boxes.flat<float>().data(), box_ind.flat<int32>().data(), boxes.dim_size(0),
        grads.dim_size(1), grads.dim_size(2), grads.dim_size(3), out->flat<float>().data(),
        stream_of(ctx))));
  }
};

// boxes [N,6], scores [N], max_output_size host scalar -> selected_indices [M].
// The output length is data-dependent, so the keep count comes back to the host
// (one 4-byte copy + stream sync, as TF's own GPU NonMaxSuppressionV2 does).
class NonMaxSuppression3DOp : public OpKernel {
 public:
  explicit NonMaxSuppression3DOp(OpKernelConstruction* ctx) : OpKernel(ctx) {
    OP_REQUIRES_OK(ctx, ctx->GetAttr("iou_threshold", &iou_threshold_));
  }
  void Compute(OpKernelContext* ctx) override {
    const Tensor& boxes = ctx->input(0);
    const Tensor& scores = ctx->input(1);
    const Tensor& max_output_size = ctx->input(2);  // HostMemory
    OP_REQUIRES(ctx, TensorShapeUtils::IsScalar(max_output_size.shape()),
                errors::InvalidArgument("max_output_size must be 0-D, got shape ",
                                        max_output_size.shape().DebugString()));
    const int32 max_out = max_output_size.scalar<int32>()();
    const int64 N = boxes.dims() == 2 ? boxes.dim_size(0) : -1;
    Tensor keep, num, ws;
    OP_REQUIRES_OK(ctx, ctx->allocate_temp(DT_INT32, TensorShape({std::max(max_out, 1)}), &keep));
    OP_REQUIRES_OK(ctx, ctx->allocate_temp(DT_INT32, TensorShape({1}), &num));
    const size_t wsb = m3d_nms3d_workspace_bytes(std::max<int64>(N, 0));
    OP_REQUIRES_OK(ctx, ctx->allocate_temp(DT_UINT8, TensorShape({static_cast<int64>(wsb) + 1}), &ws));
    const m3d_stream_t s = stream_of(ctx);
    OP_REQUIRES_OK(ctx, m3d_status(m3d_nms3d(
        boxes.flat<float>().data(), scores.flat<float>().data(), N, max_out, iou_threshold_,
        /*mode=*/0, keep.flat<int32>().data(), num.flat<int32>().data(), ws.flat<uint8>().data(),
        wsb, s)));
    int32 m = 0;
    OP_REQUIRES(ctx, hipMemcpyAsync(&m, num.flat<int32>().data(), sizeof(m), hipMemcpyDeviceToHost,
                                    reinterpret_cast<hipStream_t>(s)) == hipSuccess &&
                         hipStreamSynchronize(reinterpret_cast<hipStream_t>(s)) == hipSuccess,
                errors::Internal("NonMaxSuppression3D: keep-count copy failed"));
    Tensor* out = nullptr;
    OP_REQUIRES_OK(ctx, ctx->allocate_output(0, TensorShape({m}), &out));
    if (m > 0)
      OP_REQUIRES(ctx, hipMemcpyAsync(out->flat<int32>().data(), keep.flat<int32>().data(),
                                      sizeof(int32) * m, hipMemcpyDeviceToDevice,
                                      reinterpret_cast<hipStream_t>(s)) == hipSuccess,
                  errors::Internal("NonMaxSuppression3D: output copy failed"));
  }

 private:
  float iou_threshold_;
};

REGISTER_KERNEL_BUILDER(Name("CropAndResize3D").Device(DEVICE_GPU).TypeConstraint<float>("T")
                            .HostMemory("crop_size"), CropAndResize3DOp);
REGISTER_KERNEL_BUILDER(Name("CropAndResize3DGradImage").Device(DEVICE_GPU)
                            .TypeConstraint<float>("T").HostMemory("image_size"),
                        CropAndResize3DGradImageOp);
REGISTER_KERNEL_BUILDER(Name("CropAndResize3DGradBoxes").Device(DEVICE_GPU)
                            .TypeConstraint<float>("T"), CropAndResize3DGradBoxesOp);
REGISTER_KERNEL_BUILDER(Name("NonMaxSuppression3D").Device(DEVICE_GPU)
                            .HostMemory("max_output_size"), NonMaxSuppression3DOp);

}  // namespace
}  // namespace tensorflow
