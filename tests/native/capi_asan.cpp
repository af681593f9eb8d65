// ASan/UBSan driver for the host half of libm3d (tests/native/Makefile.sanitize,
// run by tests/test_sanitizers.py; CPU only, no GPU needed or touched).
// Every entry point of include/m3d.h is called with arguments the reference op
// would reject (null buffers, zero/negative sizes, out-of-range attributes,
// undersized workspaces) and must return M3D_EINVAL with a non-empty message;
// the workspace-size functions are evaluated over small..huge shapes (integer
// overflow is what UBSan watches there).  No call reaches a kernel launch.
#include <cstdio>
#include <cstring>
#include <initializer_list>

#include "m3d.h"

static int failures = 0, checks = 0;

#define EXPECT_EINVAL(call)                                                               \
    do {                                                                                  \
        ++checks;                                                                         \
        const int rc_ = (call);                                                           \
        const char* e_ = m3d_last_error();                                                \
        if (rc_ != M3D_EINVAL || !e_ || !*e_) {                                           \
            ++failures;                                                                   \
            std::printf("FAIL line %d: rc %d msg '%s'\n", __LINE__, rc_, e_ ? e_ : "(null)"); \
        }                                                                                 \
    } while (0)

int main() {
    const float* nf = nullptr;
    float* of = nullptr;
    const int32_t* ni = nullptr;
    int32_t* oi = nullptr;
    m3d_stream_t s = nullptr;
    const float sd[6] = {0.1f, 0.1f, 0.1f, 0.2f, 0.2f, 0.2f};
    const float* maps[4] = {nullptr, nullptr, nullptr, nullptr};
    float* gmaps[4] = {nullptr, nullptr, nullptr, nullptr};
    const int64_t fshape[4][3] = {{8, 8, 8}, {4, 4, 8}, {2, 2, 8}, {1, 1, 8}};
    const int64_t bad_fshape[4][3] = {{8, 8, 8}, {0, 4, 8}, {2, 2, 8}, {1, 1, 8}};

    if (m3d_abi_version() != 3) { std::printf("FAIL abi version\n"); return 1; }

    // CropAndResize3D family (wheel ops)
    EXPECT_EINVAL(m3d_crop_and_resize3d_fwd(nf, 1, 4, 4, 4, 1, nf, ni, 1, 0, 2, 2, 0, 0.f, of, s));
    EXPECT_EINVAL(m3d_crop_and_resize3d_fwd(nf, 1, 4, 4, 4, 1, nf, ni, 1, 2, 2, 2, 7, 0.f, of, s));
    EXPECT_EINVAL(m3d_crop_and_resize3d_fwd(nf, -1, 4, 4, 4, 1, nf, ni, 1, 2, 2, 2, 0, 0.f, of, s));
    EXPECT_EINVAL(m3d_crop_and_resize3d_fwd(nf, 1, 4, 4, 4, 0, nf, ni, 1, 2, 2, 2, 0, 0.f, of, s));
    EXPECT_EINVAL(m3d_crop_and_resize3d_bwd_image(nf, nf, ni, 1, 2, -2, 2, 1, 4, 4, 4, 1, 0, 0, of, s));
    EXPECT_EINVAL(m3d_crop_and_resize3d_bwd_image(nf, nf, ni, 1, 2, 2, 2, 1, 4, 4, 4, 1, 9, 0, of, s));
    EXPECT_EINVAL(m3d_crop_and_resize3d_bwd_boxes(nf, nf, 1, 4, 4, 4, 1, nf, ni, 1, 0, 2, 2, of, s));
    EXPECT_EINVAL(m3d_crop_and_resize3d_bwd_boxes(nf, nf, 1, 0, 4, 4, 1, nf, ni, 1, 2, 2, 2, of, s));
    EXPECT_EINVAL(m3d_pyramid_roi_align3d_fwd(maps, fshape, 8, nf, nf, 18, 1, 4, 0, 7, 7, of, of, oi, s));
    EXPECT_EINVAL(m3d_pyramid_roi_align3d_fwd(maps, bad_fshape, 8, nf, nf, 18, 1, 4, 7, 7, 7, of, of, oi, s));
    EXPECT_EINVAL(m3d_pyramid_roi_align3d_bwd(nf, nf, ni, 1, 4, 7, 0, 7, gmaps, fshape, 8, s));
    EXPECT_EINVAL(m3d_mask_targets3d(nullptr, 8, 8, 8, 2, nf, ni, 4, 0, 28, 28, of, s));
    EXPECT_EINVAL(m3d_mask_targets3d(nullptr, 8, -8, 8, 2, nf, ni, 4, 28, 28, 28, of, s));

    // NonMaxSuppression3D (A.3) and the ProposalLayer glue
    EXPECT_EINVAL(m3d_nms3d(nf, nf, 10, 5, 1.5f, 0, oi, oi, nullptr, 0, s));
    EXPECT_EINVAL(m3d_nms3d(nf, nf, 10, 5, -0.1f, 0, oi, oi, nullptr, 0, s));
    EXPECT_EINVAL(m3d_nms3d(nf, nf, 10, 5, 0.5f, 3, oi, oi, nullptr, 0, s));
    EXPECT_EINVAL(m3d_nms3d(nf, nf, 100, 5, 0.5f, 0, oi, oi, nullptr, 8, s));   // workspace too small
    EXPECT_EINVAL(m3d_score_keys(nf, -3, nullptr, s));
    EXPECT_EINVAL(m3d_score_keys_mapped(nf, -3, nullptr, nullptr, s));
    EXPECT_EINVAL(m3d_proposal_decode(nf, nf, nf, 10, nullptr, -1, sd, 8.f, of, of, nullptr, s));
    EXPECT_EINVAL(m3d_proposal_decode(nf, nf, nf, -1, nullptr, 0, sd, 8.f, of, of, nullptr, s));
    EXPECT_EINVAL(m3d_proposal_decode(nf, nf, nf, 4, nullptr, 5, sd, 8.f, of, of, nullptr, s));
    EXPECT_EINVAL(m3d_proposal_gather(nf, ni, ni, -1, of, s));

    // convolutions
    EXPECT_EINVAL(m3d_conv3d_fwd(nf, 1, 8, 8, 8, 4, nf, 3, 3, 3, 0, 8, 8, 8, 1, 1, 1, 1, 1, 1, nf, nf, nf, nf,
                                 0, 0, of, of, 0, of, 0, 0, s));
    EXPECT_EINVAL(m3d_conv3d_fwd(nf, 1, 8, 8, 8, 4, nf, 0, 3, 3, 8, 8, 8, 8, 1, 1, 1, 1, 1, 1, nf, nf, nf, nf,
                                 0, 0, of, of, 0, of, 0, 0, s));
    EXPECT_EINVAL(m3d_conv3d_fwd(nf, 1, 8, 8, 8, 4, nf, 3, 3, 3, 8, 8, 8, 8, 0, 1, 1, 1, 1, 1, nf, nf, nf, nf,
                                 0, 0, of, of, 0, of, 0, 0, s));
    EXPECT_EINVAL(m3d_conv3d_bwd_data(nf, nf, 1, 8, 8, 8, 4, 3, 3, 3, 8, 8, 8, 8, 1, 1, 0, 1, 1, 1, of, 0, s));
    // data gradients with the fused BN-ReLU backward: descriptor checks come first
    {
        float buf[4] = {0, 0, 0, 0};
        m3d_bn_bwd_t bn{};
        EXPECT_EINVAL(m3d_conv3d_bwd_data_bn(nf, nf, 1, 8, 8, 8, 64, 1, 1, 1, 32, 8, 8, 8, 1, 1, 1, 0, 0, 0, of, 0,
                                             nullptr, nullptr, 0, s));                    // no descriptor
        bn.relu = 1;                                                                    // relu without y
        EXPECT_EINVAL(m3d_conv3d_bwd_data_bn(nf, nf, 1, 8, 8, 8, 64, 1, 1, 1, 32, 8, 8, 8, 1, 1, 1, 0, 0, 0, of, 0,
                                             &bn, nullptr, 0, s));
        bn.relu = 0;
        bn.sum_dpre_xhat = buf;                                                         // xhat sums without z
        EXPECT_EINVAL(m3d_conv3d_bwd_data_bn(nf, nf, 1, 8, 8, 8, 64, 1, 1, 1, 32, 8, 8, 8, 1, 1, 1, 0, 0, 0, of, 0,
                                             &bn, nullptr, 0, s));
        bn.sum_dpre_xhat = nullptr;
        bn.sum_dz = buf;                                                                // sums, no workspace
        EXPECT_EINVAL(m3d_conv3d_bwd_data_splitk_bn(nf, nf, 1, 4, 4, 8, 1024, 256, of, 0, 2, nullptr, 0, &bn,
                                                    nullptr, 0, s));
        EXPECT_EINVAL(m3d_conv3d_bwd_data_wino_bn(nf, nf, 1, 8, 8, 8, 96, 64, 8, 1, of, 0, nullptr, 0, 0, &bn,
                                                  nullptr, 0, s));                      // Cin 96: no fused form
    }
    EXPECT_EINVAL(m3d_conv3d_bwd_weight(nf, nf, 1, 8, 8, -8, 4, 3, 3, 3, 8, 8, 8, 8, 1, 1, 1, 1, 1, 1, of, nullptr,
                                         s));
    EXPECT_EINVAL(m3d_conv3d_fwd_dil(nf, 1, 8, 8, 8, 4, nf, 3, 3, 3, 8, 8, 8, 8, 1, 1, 1, 1, 1, 1, 0, 1, 1, nf,
                                     nf, nf, nf, 0, 0, of, of, 0, of, 0, 0, s));
    EXPECT_EINVAL(m3d_deconv3d_k2s2(nf, 1, 4, 4, 4, 0, nf, 8, nf, 0, of, s));
    EXPECT_EINVAL(m3d_conv3d_fwd_wino(nf, 1, 8, 8, 8, 128, nf, 128, 8, 1, nf, nf, nf, nf, 0, of, of, nullptr, 0, s));
    EXPECT_EINVAL(m3d_conv3d_bwd_data_wino(nf, nf, 1, 8, 8, 8, 128, 128, 8, 1, of, 0, nullptr, 0, s));
    EXPECT_EINVAL(m3d_conv3d_bwd_weight_wino(nf, nf, 1, 8, 8, 8, 128, 128, 8, 1, of, nullptr, 0, nullptr, s));
    EXPECT_EINVAL(m3d_conv3d_fwd_wino_keep(nf, 1, 8, 8, 8, 128, nf, 128, 8, 1, nf, nf, nf, nf, 0, of, of, of,
                                           nullptr, 0, s));
    EXPECT_EINVAL(m3d_conv3d_bwd_weight_wino_u(nf, nf, 1, 8, 8, 8, 128, 128, 8, 1, of, nullptr, 0, nullptr, s));

    EXPECT_EINVAL(m3d_conv3d_fwd_wino_halo(nf, nf, 2, 0, 1, 8, 8, 8, 128, nf, 128, nf, nf, nf, nf, 0, of, of,
                                           of, nullptr, 0, s));
    EXPECT_EINVAL(m3d_conv3d_bwd_data_wino_halo(nf, nf, 1, 0, 1, 8, 8, 8, 128, 128, of, nullptr, 0, nullptr, 0,
                                                s));
    EXPECT_EINVAL(m3d_conv3d_bwd_weight_wino_halo(nf, nullptr, 0, 1, nf, 1, 8, 8, 8, 128, 128, of, nullptr, 0,
                                                  nullptr, s));

    // GEMMs
    EXPECT_EINVAL(m3d_gemm_f32(nf, nf, of, 1, 0, 4, 4, nf, 0, 0, s));
    EXPECT_EINVAL(m3d_gemm_wgrad_f32(nf, nf, of, 1, 4, -4, 4, nullptr, s));
    EXPECT_EINVAL(m3d_split3_f32(nf, 0, nullptr, s));
    EXPECT_EINVAL(m3d_gemm_x3(nullptr, nullptr, of, 1, 64, 48, 64, s));        // K % 32
    EXPECT_EINVAL(m3d_gemm_x3(nullptr, nullptr, of, 1, 1LL << 40, 64, 64, s)); // > 4 GiB operand
    EXPECT_EINVAL(m3d_gemm_x3_af(nf, nullptr, of, 1, 64, 48, 64, s));           // K % 32
    EXPECT_EINVAL(m3d_gemm_x3_af(nullptr, nullptr, of, 1, 64, 64, 64, s));      // null A
    EXPECT_EINVAL(m3d_gemm_x3_af(nf, nullptr, of, 1, 1LL << 40, 64, 64, s));    // > 4 GiB operand
    EXPECT_EINVAL(m3d_gemm_f32_ex(nf, 4, 16, nf, 16, of, 16, 1, 4, 0, 4, nf, 0, 0, s));
    EXPECT_EINVAL(m3d_splitk_reduce(nf, 0, 4, 4, nf, nf, nf, 0, of, s));

    // heads / DetectionLayer / target builders
    EXPECT_EINVAL(m3d_head_outputs(nf, 4, 8, 0, of, of, of, s));
    EXPECT_EINVAL(m3d_refine_detections(nf, nf, nf, 4, 0, nf, sd, 0.5f, of, of, of, s));
    EXPECT_EINVAL(m3d_detections_gather(nf, nf, ni, ni, -1, nf, of, s));
    EXPECT_EINVAL(m3d_detection_targets(nf, 16, ni, nf, 2, 0, 0.33f, 0.5f, 0.5f, sd, 1, 7u, of, of, oi, of, of,
                                        oi, oi, nullptr, 0, s));
    EXPECT_EINVAL(m3d_rpn_targets(nf, 64, nf, 2, 0.5f, 0.3f, 0, 0.5f, 9, 1, sd, 7u, nullptr, of, 64, nullptr, 0,
                                  oi, s));
    EXPECT_EINVAL(m3d_rpn_targets_async(nf, 64, nf, 2, 0.5f, 0.3f, 128, 0.5f, 9, 1, sd, 7u, nullptr, of, 0,
                                        nullptr, 0, oi, s));

    // pooling / resampling / BN / optimizers
    EXPECT_EINVAL(m3d_maxpool3d_fwd(nf, 1, 8, 8, 8, 4, 3, 3, 3, 0, 2, 1, 0, 0, 1, 4, 4, 8, of, nullptr, s));
    EXPECT_EINVAL(m3d_maxpool3d_bwd(nf, nullptr, 1, 8, 8, 8, 4, 3, 3, 3, 2, 2, 1, 0, 0, 1, 0, 4, 8, of, s));
    EXPECT_EINVAL(m3d_upsample221_bwd(nf, 1, 4, 4, 4, 0, of, 0, s));
    EXPECT_EINVAL(m3d_subsample221_fwd(nf, 1, -4, 4, 4, 4, of, s));
    EXPECT_EINVAL(m3d_subsample221_bwd(nf, 1, 4, 4, -4, 4, of, s));
    EXPECT_EINVAL(m3d_bn_affine(nf, nf, nf, nf, 1e-3f, 0, of, of, of, s));
    EXPECT_EINVAL(m3d_bn_act_bwd(nf, nf, nf, 0, 8, 1, nf, nf, nf, of, of, 0, of, of, of, nullptr, 0, s));
    EXPECT_EINVAL(m3d_sgd_keras(of, nf, of, -1, ni, nf, 1, 0.01f, 0.9f, 5.f, of, nullptr, s));
    EXPECT_EINVAL(m3d_adam_keras(of, nf, of, of, of, -1, ni, nf, 1, 1e-3f, 0.9f, 0.999f, 1e-7f, 5.f, of, nullptr,
                                 s));
    EXPECT_EINVAL(m3d_adadelta_keras(of, nf, of, of, -1, ni, nf, 1, 1.f, 0.95f, 1e-7f, 5.f, of, nullptr, s));
    {   // per-call deterministic targets (ABI 3): on with no / short / misaligned scratch
        alignas(16) static char scratch[8192];
        const m3d_det_t d0 = {1, nullptr, 1 << 20}, d1 = {1, scratch, 64}, d2 = {1, scratch + 4, 4096};
        EXPECT_EINVAL(m3d_gemm_wgrad_f32(nf, nf, of, 1, 4, 4, 4, &d0, s));
        EXPECT_EINVAL(m3d_sgd_keras(of, nf, of, 1, ni, nf, 1, 0.01f, 0.9f, 5.f, of, &d1, s));
        EXPECT_EINVAL(m3d_conv3d_bwd_weight(nf, nf, 1, 8, 8, 8, 4, 3, 3, 3, 8, 8, 8, 8, 1, 1, 1, 1, 1, 1, of, &d2, s));
        EXPECT_EINVAL(m3d_fork_event_create(3, nullptr));
        EXPECT_EINVAL(m3d_stream_fork(s, s, nullptr));
    }

    // workspace sizing: pure host arithmetic over small .. huge shapes
    size_t acc = 0;
    for (int64_t n : {0LL, 1LL, 63LL, 64LL, 15000LL, 1LL << 20, 1LL << 31})
        acc += m3d_nms3d_workspace_bytes(n) + m3d_detection_targets_workspace_bytes(n) +
               m3d_bn_act_bwd_workspace_bytes(n, 256);
    for (int64_t S : {8LL, 64LL, 128LL, 256LL, 512LL})
        acc += m3d_conv3d_wino_workspace_bytes(1, S / 4, S / 4, S, S, 256, 512) +
               m3d_conv3d_wino_u_bytes(1, S / 4, S / 4, S, 256) +
               m3d_rpn_targets_workspace_bytes(S * S * S / 16, 32, 4096);
    std::printf("%d checks, %d failures (workspace sum %zu)\n", checks, failures, acc);
    return failures ? 1 : 0;
}
