"""Config surface of the reference (core/config.py:10-387).

``Config(**json_dict)`` accepts exactly the reference's keyword set (an
unknown key raises ``TypeError`` like the reference's ``__init__``) and
derives the same fields: IMAGE_SHAPE=[H,W,D,C] (:142), BATCH_SIZE (:298),
IMAGE_META_SIZE=1+4+4+6+1+NUM_CLASSES (:301), ANCHOR_NB (:235-241).
``load_config(path)`` mirrors core/config.py:383-387.
"""
from __future__ import annotations

import copy
import json

import numpy as np

DEFAULTS = dict(
    DATA_DIR="data/", NUM_CLASSES=2, CLASS_NAMES=["neuron"], IMAGE_SIZE=256, IMAGE_DEPTH=12,
    IMAGE_CHANNEL_COUNT=1, MAX_GT_INSTANCES=50, TARGET_RATIO=0.2, USE_MINI_MASK=False,
    MINI_MASK_SHAPE=(56, 56, 56), RPN_BBOX_STD_DEV=[0.1, 0.1, 0.1, 0.2, 0.2, 0.2],
    BBOX_STD_DEV=[0.1, 0.1, 0.1, 0.2, 0.2, 0.2], EVALUATION_STEPS=100,
    OUTPUT_DIR="data/output/", MODE="training", BACKBONE="resnet50",
    BACKBONE_STRIDES=[(4, 4, 1), (8, 8, 1), (16, 16, 1), (32, 32, 1), (64, 64, 2)],
    TOP_DOWN_PYRAMID_SIZE=256, RPN_ANCHOR_SCALES=(24, 39, 56, 84, 96),
    RPN_ANCHOR_RATIOS=[0.05, 0.075, 0.1, 0.15, 0.25], RPN_ANCHOR_STRIDE=1,
    RPN_TRAIN_ANCHORS_PER_IMAGE=1024, RPN_NMS_THRESHOLD=0.9, PRE_NMS_LIMIT=10000,
    POST_NMS_ROIS_TRAINING=3000, POST_NMS_ROIS_INFERENCE=1500, TRAIN_ROIS_PER_IMAGE=512,
    ROI_POSITIVE_RATIO=0.33, POOL_SIZE=7, MASK_POOL_SIZE=14, FPN_CLASSIF_FC_LAYERS_SIZE=1024,
    HEAD_CONV_CHANNEL=256, HEAD_MAX_ROIS=1000, MASK_SHAPE=[28, 28, 28], TELEMETRY=True,
    TELEMETRY_SAMPLE=0.02, EVAL_DET_IOU=0.4, MIN_ROI_SIZE=15, DETECTION_MAX_INSTANCES=50,
    DETECTION_MIN_CONFIDENCE=0.2, DETECTION_NMS_THRESHOLD=0.45, RPN_POSITIVE_IOU=0.60,
    RPN_NEGATIVE_IOU=0.30, IMAGES_PER_GPU=1, GPU_COUNT=1,
    LOSS_WEIGHTS={"rpn_class_loss": 1., "rpn_bbox_loss": 1., "mrcnn_class_loss": 1.,
                  "mrcnn_bbox_loss": 1., "mrcnn_mask_loss": 1., "mrcnn_obj_loss": 0.5,
                  "mrcnn_margin_loss": 0.0},
    TRAIN_BN=False, LEARNING_LAYERS="all", OPTIMIZER={"name": "SGD", "parameters": {}},
    WEIGHT_DIR=None, RPN_WEIGHTS=None, HEAD_WEIGHTS=None, MASK_WEIGHTS=None, EPOCHS=1,
    FROM_EPOCH=0, WEIGHT_DECAY=0.0001, EVAL_TOPK_RPN=512, EVAL_MATCH_IOU=0.50,
    EVAL_MATCH_IOU_GRID=[0.30, 0.40, 0.50], EVAL_TOPK_GRID=[500, 1000, 2000, 4000, 6000, 8000],
    AUTO_TUNE_RPN=False, AUTO_TUNE_SAVE_PATCH=True, AUTO_TUNE_SNAP_SCALE_STEP=8,
    AUTO_TUNE_SNAP_RATIO_STEP=0.02, AUTO_TUNE_RATIO_RANGE=[0.04, 0.30], AUTO_TUNE_SCALES_LIMIT=8,
    AUTO_TUNE_RATIOS_LIMIT=8, MIN_POSITIVE_TARGETS=25, AUGMENT=True, AUG_PROB=0.5,
    AUG_FLIP_Y=True, AUG_FLIP_X=True, AUG_FLIP_Z=False, AUG_BRIGHTNESS_DELTA=0.03,
    AUG_GAUSS_NOISE_STD=0.0, RPN_AUGMENT_GT=True, RPN_GT_JITTER_PER_BOX=3,
    RPN_GT_JITTER_SCALE_SIGMA=0.10, RPN_GT_JITTER_TRANS=[2, 2, 1], ATSS_TOPK=12,
    ATSS_MIN_POS_PER_GT=3, RPN_GT_JITTER_IOU_THR=0.4, VOXEL_Z_OVER_Y=1.0, HEAD_SHUFFLE_ROIS=False,
    HEAD_BALANCE_POS=False, HEAD_POS_FRAC=0.25,
)


class Config:
    """Attribute bag with the reference's keys, defaults and derived fields."""

    def __init__(self, **kwargs):
        unknown = set(kwargs) - set(DEFAULTS)
        if unknown:
            raise TypeError(f"__init__() got an unexpected keyword argument '{sorted(unknown)[0]}'")
        vals = copy.deepcopy(DEFAULTS)
        vals.update(kwargs)
        for k, v in vals.items():
            setattr(self, k, v)
        self.IMAGE_SHAPE = np.array([self.IMAGE_SIZE, self.IMAGE_SIZE, self.IMAGE_DEPTH,
                                     self.IMAGE_CHANNEL_COUNT])
        self.RPN_BBOX_STD_DEV = np.asarray(self.RPN_BBOX_STD_DEV)
        self.BBOX_STD_DEV = np.asarray(self.BBOX_STD_DEV)

        def cells(stride):
            if isinstance(stride, (int, np.integer)):
                sy = sx = sz = int(stride)
            else:
                sy, sx, sz = stride
            return (self.IMAGE_SHAPE[0] / sy) * (self.IMAGE_SHAPE[1] / sx) * (self.IMAGE_SHAPE[2] / sz)

        self.ANCHOR_NB = int(sum(cells(s) for s in self.BACKBONE_STRIDES[:5]))
        self.BATCH_SIZE = self.IMAGES_PER_GPU * self.GPU_COUNT
        self.IMAGE_META_SIZE = 1 + 4 + 4 + 6 + 1 + self.NUM_CLASSES

    def display(self):
        print("\nConfigurations:")
        for a in sorted(vars(self)):
            print("{:30} {}".format(a, getattr(self, a)))
        print("\n")

    def to_dict(self):
        return {k: getattr(self, k) for k in DEFAULTS}


def load_config(config_path):
    with open(config_path) as f:
        return Config(**json.load(f))


def synthetic_rpn_config(size: int, depth: int | None = None, **overrides) -> Config:
    """The rats RPN preset (configs/rpn/scp_rpn_rats.json) at IMAGE_SIZE=IMAGE_DEPTH=size,
    IMAGES_PER_GPU=1, AUGMENT=False -- the synthetic benchmark configs of SURVEY.md 8d."""
    d = dict(
        NUM_CLASSES=2, IMAGE_SIZE=size, IMAGE_DEPTH=depth if depth is not None else size,
        IMAGE_CHANNEL_COUNT=1, RPN_ANCHOR_SCALES=[25, 57, 84, 109, 135],
        RPN_ANCHOR_RATIOS=[0.05, 0.06, 0.15], RPN_ANCHOR_STRIDE=1,
        RPN_BBOX_STD_DEV=[0.1, 0.1, 0.1, 0.213, 0.21, 0.15],
        BBOX_STD_DEV=[0.1, 0.1, 0.1, 0.213, 0.21, 0.15], RPN_NMS_THRESHOLD=0.7,
        MODE="training", BACKBONE_STRIDES=[[4, 4, 1], [8, 8, 1], [16, 16, 1], [32, 32, 1], [64, 64, 1]],
        BACKBONE="resnet50", TOP_DOWN_PYRAMID_SIZE=256, RPN_TRAIN_ANCHORS_PER_IMAGE=1536,
        PRE_NMS_LIMIT=15000, POST_NMS_ROIS_TRAINING=6000, POST_NMS_ROIS_INFERENCE=8000,
        POOL_SIZE=7, MASK_POOL_SIZE=14, TRAIN_ROIS_PER_IMAGE=128, IMAGES_PER_GPU=1, GPU_COUNT=1,
        OPTIMIZER={"name": "SGD", "parameters": {"learning_rate": 0.0002, "momentum": 0.9,
                                                 "clipnorm": 5.0, "decay": 1e-4}},
        WEIGHT_DECAY=0.0005, AUGMENT=False,
    )
    d.update(overrides)
    return Config(**d)


def synthetic_mrcnn_config(size: int, depth: int | None = None, **overrides) -> Config:
    """MaskRCNN inference on the rats preset (configs/mrcnn/scp_mrcnn_rats.json head
    sizes: FPN_CLASSIF_FC_LAYERS_SIZE 512, HEAD_CONV_CHANNEL 256, POOL 7, MASK_POOL 14,
    DETECTION_NMS_THRESHOLD 0.3) with BASELINE configs[3]'s 512 proposals."""
    d = dict(MODE="inference", POST_NMS_ROIS_INFERENCE=512, FPN_CLASSIF_FC_LAYERS_SIZE=512,
             HEAD_CONV_CHANNEL=256, DETECTION_MAX_INSTANCES=40, DETECTION_MIN_CONFIDENCE=0.3,
             DETECTION_NMS_THRESHOLD=0.3, MASK_SHAPE=[28, 28, 28])
    d.update(overrides)
    return synthetic_rpn_config(size, depth, **d)
