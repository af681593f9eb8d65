"""The reference's on-disk dataset format, read without scikit-image / pickle.

Mirrors ``utils.Dataset`` (core/utils.py:694-800) and ``ToyDataset``
(core/data_generators.py:1559-1716):

* ``<data_dir>/datasets/{train,test}.csv`` with (case-insensitive, substring
  matched) columns images / segs (optional) / cabs / masks holding file paths;
* images: Z-first TIFF stacks -> ``(Y, X, Z)``; clipped to the [1, 99]
  percentiles, z-scored, ``tanh(0.5 x)``; returned ``[H, W, D, 1]`` float32
  (core/data_generators.py:1603-1630);
* ``cabs`` (.dat): whitespace rows ``class z1 y1 x1 z2 y2 x2`` (exclusive
  ends), remapped to ``(y1, x1, z1, y2, x2, z2)`` and validated as the loader
  does (core/data_generators.py:1648-1668);
* masks: bz2-compressed pickles of a ``(Z, Y, X, N)`` array, transposed to
  ``(Y, X, Z, N)`` float32 (1679-1708).  The pickle is read with an
  allow-list unpickler that only reconstructs numpy arrays, so a data file
  cannot execute code.

The loaded volumes feed ``m3d.targets.build_rpn_targets`` /
``DetectionTargetLayer`` and the models as ``[1, H, W, D, 1]`` tensors.
"""
from __future__ import annotations

import bz2
import io
import os
import pickle

import numpy as np

from .tiff import imread


class _NumpyOnlyUnpickler(pickle.Unpickler):
    _ALLOWED = {
        ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
        ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "scalar"),
        ("numpy._core.multiarray", "scalar"), ("_codecs", "encode"),
    }

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to load {module}.{name} from a mask file")


def load_mask_pickle(path) -> np.ndarray:
    """The bz2-pickled (Z, Y, X, N) mask array (numpy objects only)."""
    with bz2.BZ2File(path, "rb") as f:
        data = f.read()
    return np.asarray(_NumpyOnlyUnpickler(io.BytesIO(data), encoding="latin1").load())


def normalize_image(image_zyx: np.ndarray) -> np.ndarray:
    """ToyDataset.load_image normalisation: (Z,Y,X) -> [H,W,D,1] float32."""
    image = np.transpose(image_zyx, (1, 2, 0)).astype(np.float32)
    p1, p99 = np.percentile(image, [1, 99])
    image = np.clip(image, p1, p99)
    mean_val, std_val = np.mean(image), np.std(image)
    image = (image - mean_val) / std_val if std_val > 0 else image - mean_val
    image = np.tanh(image * 0.5)
    return image[..., np.newaxis].astype(np.float32, copy=False)


class Dataset:
    """utils.Dataset: class / image registries and id maps."""

    def __init__(self, class_map=None):
        self._image_ids = []
        self.image_info = []
        self.class_info = [{"source": "", "id": 0, "name": "BG"}]
        self.source_class_ids = {}

    def add_class(self, source, class_id, class_name):
        assert "." not in source, "Source name cannot contain a dot"
        for info in self.class_info:
            if info["source"] == source and info["id"] == class_id:
                return
        self.class_info.append({"source": source, "id": class_id, "name": class_name})

    def add_image(self, source, image_id, path, **kwargs):
        info = {"id": image_id, "source": source, "path": path}
        info.update(kwargs)
        self.image_info.append(info)

    def prepare(self, class_map=None):
        def clean_name(name):
            return ",".join(name.split(",")[:1])

        self.num_classes = len(self.class_info)
        self.class_ids = np.arange(self.num_classes)
        self.class_names = [clean_name(c["name"]) for c in self.class_info]
        self.num_images = len(self.image_info)
        self._image_ids = np.arange(self.num_images)
        self.class_from_source_map = {f"{i['source']}.{i['id']}": c for i, c in zip(self.class_info, self.class_ids)}
        self.image_from_source_map = {f"{i['source']}.{i['id']}": c for i, c in zip(self.image_info, self.image_ids)}
        self.sources = list({i["source"] for i in self.class_info})
        self.source_class_ids = {s: [i for i, info in enumerate(self.class_info) if i == 0 or s == info["source"]]
                                 for s in self.sources}

    def map_source_class_id(self, source_class_id):
        return self.class_from_source_map[source_class_id]

    def get_source_class_id(self, class_id, source):
        info = self.class_info[class_id]
        assert info["source"] == source
        return info["id"]

    @property
    def image_ids(self):
        return self._image_ids

    def source_image_link(self, image_id):
        return self.image_info[image_id]["path"]


class ToyDataset(Dataset):
    """core/data_generators.py:1559-1716."""

    def load_dataset(self, data_dir, is_train=True):
        import pandas as pd
        self.add_class("dataset", 1, "neuron")
        split = "train" if is_train else "test"
        td = pd.read_csv(os.path.join(data_dir, "datasets", f"{split}.csv"), sep=None, engine="python")
        cols = {c.lower(): c for c in td.columns}

        def pick(*cands, required=True):
            for c in cands:
                k = c.lower()
                if k in cols:
                    return cols[k]
                for lc, orig in cols.items():
                    if k in lc:
                        return orig
            if required:
                raise KeyError(f"[Dataset.load_dataset] none of columns {cands} found. "
                               f"Available: {list(td.columns)}")
            return None

        col_images = pick("images", "image", "img", "path", "image_path")
        col_segs = pick("segs", "seg", "seg_path", "labels", "label_path", required=False)
        col_cabs = pick("cabs", "cab", "boxes", "cab_path")
        col_masks = pick("masks", "mask", "masks_path", "mask_path")
        for i in range(len(td)):
            img, cab, msk = td.at[i, col_images], td.at[i, col_cabs], td.at[i, col_masks]
            seg = td.at[i, col_segs] if col_segs is not None else None
            for nm, v in (("images", img), ("cabs", cab), ("masks", msk)):
                if not isinstance(v, str):
                    raise ValueError(f"[load_dataset] bad '{nm}' at row {i}")
            self.add_image("dataset", image_id=i, path=img, seg_path=seg, cab_path=cab, m_path=msk)

    def load_image(self, image_id, z_slice=None):
        return normalize_image(imread(self.image_info[image_id]["path"]))

    def load_data(self, image_id, masks_needed=True):
        """-> boxes [N,6] int32 (y1,x1,z1,y2,x2,z2) px, class_ids [N] int32,
        masks [H,W,D,N] float32 (or None)."""
        info = self.image_info[image_id]
        cabs = np.loadtxt(info["cab_path"], ndmin=2, dtype=np.int32)
        if cabs.size:
            boxes = cabs[:, [2, 3, 1, 5, 6, 4]]
            class_ids = cabs[:, 0]
            valid = ((boxes[:, 3] > boxes[:, 0]) & (boxes[:, 4] > boxes[:, 1]) & (boxes[:, 5] > boxes[:, 2]) &
                     (boxes[:, 0] >= 0) & (boxes[:, 1] >= 0) & (boxes[:, 2] >= 0))
            boxes, class_ids = boxes[valid], class_ids[valid]
        else:
            boxes = np.zeros((0, 6), np.int32)
            class_ids = np.zeros((0,), np.int32)
        if not masks_needed:
            return boxes, class_ids, None
        if boxes.shape[0] == 0:
            img = imread(info["path"])
            return boxes, class_ids, np.zeros((img.shape[1], img.shape[2], img.shape[0], 0), np.float32)
        try:
            m = load_mask_pickle(info["m_path"])
            masks = np.transpose(m, (1, 2, 0, 3))
            if masks.dtype == np.bool_:
                masks = masks.astype(np.uint8)
            masks = masks.astype(np.float32, copy=False)
            if masks.shape[-1] != boxes.shape[0]:
                k = min(masks.shape[-1], boxes.shape[0])
                if k > 0:
                    masks, boxes, class_ids = masks[..., :k], boxes[:k], class_ids[:k]
                else:
                    masks = np.zeros((*masks.shape[:3], 0), np.float32)
                    boxes = np.zeros((0, 6), np.int32)
                    class_ids = np.zeros((0,), np.int32)
        except (OSError, EOFError, pickle.UnpicklingError, ValueError):
            img = imread(info["path"])
            masks = np.zeros((img.shape[1], img.shape[2], img.shape[0], 0), np.float32)
        return boxes, class_ids, masks
