"""Keras-H5 weight import / export for the m3d models.

Mirrors ``keras_model.load_weights(path, by_name=True, skip_mismatch=...)`` as
the reference calls it (core/models.py:3428, 3785, 4576-4593, 4843-4856,
5852-5856; keras 2.3.1 ``load_weights_from_hdf5_group_by_name``):

* the weights live at the file root or under ``model_weights`` (full-model
  saves, core/models.py:5154);
* ``layer_names`` (or the chunked ``layer_names0``, ``layer_names1``, ...
  attributes Keras writes above 64 KiB) lists the layer groups; each group's
  ``weight_names`` lists its datasets in the layer's weight order;
* a group is matched to a model layer by name; its values are assigned in the
  layer's Keras weight order (Conv3D/Dense/Conv3DTranspose: kernel, bias;
  BatchNormalization: gamma, beta, moving_mean, moving_variance).  Weights of
  nested models (the reference's ``rpn_model`` wrapper, build_rpn_model
  core/models.py:560-584) are matched by their own ``<layer>/<weight>:0``
  names;
* a count or shape mismatch raises ``ValueError`` with Keras' message, or is
  skipped with a warning when ``skip_mismatch``.

Kernel layouts are Keras' own (Conv3D ``[kh,kw,kd,Cin,Cout]``,
Conv3DTranspose ``[kh,kw,kd,Cout,Cin]``), which is what the m3d kernels read,
so no transposes are needed.  ``save_weights`` writes the same layout with
``m3d.h5write`` (HDF5 superblock 0, the format h5py writes by default).
"""
from __future__ import annotations

import warnings
from collections import OrderedDict

import numpy as np
import torch

from . import h5

_ORDER = {"kernel:0": 0, "bias:0": 1, "gamma:0": 0, "beta:0": 1, "moving_mean:0": 2,
          "moving_variance:0": 3}


def _layers(store):
    """OrderedDict layer name -> [(weight suffix, getter, setter, shape)] in Keras order."""
    out = OrderedDict()

    def add(name, suffix, tensor):
        out.setdefault(name, []).append((suffix, tensor))

    bn_names = {bn.name: bn for bn in store.bns}
    for p in store.params:
        layer, suffix = p.name.rsplit("/", 1)
        add(layer, suffix, p.data)
    for name, bn in bn_names.items():
        add(name, "moving_mean:0", bn.moving_mean)
        add(name, "moving_variance:0", bn.moving_variance)
    for name in out:
        out[name].sort(key=lambda e: _ORDER.get(e[0], 9))
    return out


def _attr_list(group, name):
    a = group.attrs
    if name in a:
        return [v.decode("utf8") if isinstance(v, bytes) else str(v) for v in np.atleast_1d(a[name])]
    vals, i = [], 0
    while f"{name}{i}" in a:
        vals += [v.decode("utf8") for v in np.atleast_1d(a[f"{name}{i}"])]
        i += 1
    return vals


def load_weights(store, filepath, by_name=True, skip_mismatch=False, exclude=()):
    """Load a Keras-H5 weight file into ``store`` (a finalized ParamStore).
    Returns the list of model layers that received weights."""
    if not by_name:
        raise NotImplementedError("topological (by_name=False) loading: the reference always loads by_name")
    f = h5.File(filepath)
    root = f["model_weights"] if "model_weights" in f.keys() else f
    layers = _layers(store)
    flat = {f"{ln}/{sfx}": (ln, i) for ln, ws in layers.items() for i, (sfx, _) in enumerate(ws)}
    loaded = []
    for k, name in enumerate(_attr_list(root, "layer_names")):
        g = root[name]
        wnames = _attr_list(g, "weight_names")
        if not wnames:
            continue
        values = [g[w].read() for w in wnames]
        if name in layers and name not in exclude:
            targets = [t for _, t in layers[name]]
            if len(values) != len(targets):
                msg = (f'Layer #{k} (named "{name}") expects {len(targets)} weight(s), but the saved '
                       f"weights have {len(values)} element(s).")
                if skip_mismatch:
                    warnings.warn("Skipping loading of weights for " + msg)
                    continue
                raise ValueError(msg)
            pairs = list(zip(targets, values, [f"{name}/{s}" for s, _ in layers[name]]))
        else:
            # nested model group (e.g. rpn_model): match every weight by its own name
            pairs = []
            for w, v in zip(wnames, values):
                key = "/".join(w.split("/")[-2:])
                if key in flat and flat[key][0] not in exclude:
                    ln, i = flat[key]
                    pairs.append((layers[ln][i][1], v, key))
            if not pairs:
                continue
        ok = True
        for t, v, wn in pairs:
            if tuple(t.shape) != tuple(v.shape):
                msg = (f'Layer #{k} (named "{name}"), weight {wn} has shape {tuple(t.shape)}, but the saved '
                       f"weight has shape {tuple(v.shape)}.")
                if skip_mismatch:
                    warnings.warn("Skipping loading of weights for " + msg)
                    ok = False
                    continue
                raise ValueError(msg)
        if not ok and skip_mismatch:
            pairs = [(t, v, wn) for t, v, wn in pairs if tuple(t.shape) == tuple(v.shape)]
        with torch.no_grad():
            for t, v, _ in pairs:
                t.copy_(torch.from_numpy(np.ascontiguousarray(v.astype(np.float32, copy=False))))
        loaded.append(name)
    return loaded


def save_weights(store, filepath, keras_version="2.3.1", backend="tensorflow"):
    """Write ``store`` as a Keras ``save_weights`` H5 file (layer groups with
    weight_names, datasets at <layer>/<layer>/<weight>:0)."""
    from . import h5write
    layers = _layers(store)
    tree = h5write.Group()
    tree.attrs["layer_names"] = np.array([n.encode("utf8") for n in layers])
    tree.attrs["backend"] = np.bytes_(backend.encode("utf8"))
    tree.attrs["keras_version"] = np.bytes_(keras_version.encode("utf8"))
    for name, ws in layers.items():
        g = tree.group(name)
        g.attrs["weight_names"] = np.array([f"{name}/{s}".encode("utf8") for s, _ in ws])
        sub = g.group(name)
        for s, t in ws:
            sub.datasets[s] = t.detach().float().cpu().numpy()
    h5write.write(filepath, tree)
