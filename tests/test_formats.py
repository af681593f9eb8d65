"""On-disk formats: Keras-H5 weights (m3d.h5, m3d.h5write,
m3d.weights), TIFF stacks (m3d.tiff) and the CSV/.dat/bz2-mask dataset reader
(m3d.dataset).  The .h5 / .tif fixtures under tests/golden/ were written by the
real HDF5 1.10.6 and libtiff C libraries (tests/golden/h5src/*.c), so the
readers are pinned against the reference libraries' own output; written files
are checked with HDF5's h5dump/h5diff when the image provides them."""
import bz2
import os
import pickle
import shutil
import subprocess
import warnings

import numpy as np
import pytest

from m3d import dataset, h5, h5write, tiff, weights
from m3d.params import BNLayer, ConvLayer, ParamStore

G = os.path.join(os.path.dirname(__file__), "golden")
H5DIFF = "/opt/conda/bin/h5diff"


def _exp(layer, w, shape):
    n = int(np.prod(shape))
    return np.sin(0.37 * np.arange(n) + 1.3 * layer + 0.11 * w).astype(np.float32).reshape(shape)


def _small_store(deconv_shape=(2, 2, 2, 8, 4)):
    st = ParamStore()
    ConvLayer(st, "conv1", (3, 3, 3), 1, 4)
    BNLayer(st, "bn_conv1", 4)
    ConvLayer(st, "rpn_conv_shared1", (3, 3, 3), 4, 8)
    st.add("mrcnn_class_logits/kernel:0", (8, 3), "zeros", True)
    st.add("mrcnn_class_logits/bias:0", (3,), "zeros", True)
    st.add("mrcnn_mask_deconv/kernel:0", deconv_shape, "zeros", True)
    st.add("mrcnn_mask_deconv/bias:0", (8,), "zeros", True)
    return st.finalize("cpu")


LAYERS = [("conv1", [("kernel:0", (3, 3, 3, 1, 4)), ("bias:0", (4,))]),
          ("bn_conv1", [("gamma:0", (4,)), ("beta:0", (4,)), ("moving_mean:0", (4,)), ("moving_variance:0", (4,))]),
          ("rpn_conv_shared1", [("kernel:0", (3, 3, 3, 4, 8)), ("bias:0", (8,))]),
          ("mrcnn_class_logits", [("kernel:0", (8, 3)), ("bias:0", (3,))]),
          ("mrcnn_mask_deconv", [("kernel:0", (2, 2, 2, 8, 4)), ("bias:0", (8,))])]


@pytest.mark.parametrize("fn,root", [("keras_weights_v0.h5", ""), ("keras_model_latest.h5", "model_weights/")])
def test_h5_reader_keras_layout(fn, root):
    f = h5.File(os.path.join(G, fn))
    g = f[root] if root else f
    names = [n.decode() for n in g.attrs["layer_names"]]
    assert names == [n for n, _ in LAYERS]
    if not root:
        assert f.attrs["keras_version"] == b"2.3.1" and f.attrs["backend"] == b"tensorflow"
    for li, (name, ws) in enumerate(LAYERS):
        wn = [w.decode() for w in g[name].attrs["weight_names"]]
        assert wn == [f"{name}/{w}" for w, _ in ws]
        for wi, (w, shape) in enumerate(ws):
            d = g[f"{name}/{name}/{w}"]
            assert d.shape == shape
            np.testing.assert_array_equal(d.read(), _exp(li, wi, shape))


def test_h5_reader_chunked_filters_and_wide_groups():
    f = h5.File(os.path.join(G, "keras_model_latest.h5"))
    a = f["chunked_deflate"].read()                       # chunked + shuffle + deflate, v4 fixed array
    np.testing.assert_array_equal(a.ravel(), (np.arange(210) * 0.5 - 7.0).astype(np.float32))
    w = h5.File(os.path.join(G, "wide_v0.h5"))             # 300 groups: multi-level symbol-table B-tree
    keys = w.keys()
    assert len(keys) == 301 and "layer_299" in keys
    for i in (0, 7, 150, 299):
        np.testing.assert_array_equal(w[f"layer_{i:03d}/ints"].read(), [i, -i, 7 * i])
    np.testing.assert_array_equal(w["chunked_f64"].read().ravel(), 1.0 / (np.arange(90) + 1))
    assert weights._attr_list(w, "layer_names") == [f"layer_{i:03d}" for i in range(300)]


@pytest.mark.parametrize("fn", ["keras_weights_v0.h5", "keras_model_latest.h5"])
def test_load_weights_by_name(fn):
    st = _small_store()
    loaded = weights.load_weights(st, os.path.join(G, fn))
    assert loaded == [n for n, _ in LAYERS]
    sd = st.state_dict()
    for li, (name, ws) in enumerate(LAYERS):
        for wi, (w, shape) in enumerate(ws):
            np.testing.assert_array_equal(sd[f"{name}/{w}"].numpy(), _exp(li, wi, shape))


def test_load_weights_mismatch():
    st = _small_store(deconv_shape=(2, 2, 2, 4, 8))
    with pytest.raises(ValueError, match='named "mrcnn_mask_deconv"'):
        weights.load_weights(st, os.path.join(G, "keras_weights_v0.h5"))
    st = _small_store(deconv_shape=(2, 2, 2, 4, 8))
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        weights.load_weights(st, os.path.join(G, "keras_weights_v0.h5"), skip_mismatch=True)
    assert any("mrcnn_mask_deconv" in str(r.message) for r in rec)
    sd = st.state_dict()
    np.testing.assert_array_equal(sd["conv1/kernel:0"].numpy(), _exp(0, 0, (3, 3, 3, 1, 4)))
    assert not sd["mrcnn_mask_deconv/kernel:0"].numpy().any()      # skipped
    np.testing.assert_array_equal(sd["mrcnn_mask_deconv/bias:0"].numpy(), _exp(4, 1, (8,)))


def test_save_weights_round_trip(tmp_path):
    st = _small_store()
    weights.load_weights(st, os.path.join(G, "keras_weights_v0.h5"))
    out = str(tmp_path / "rt.h5")
    weights.save_weights(st, out)
    st2 = _small_store()
    assert weights.load_weights(st2, out) == [n for n, _ in LAYERS]
    for k, v in st.state_dict().items():
        np.testing.assert_array_equal(st2.state_dict()[k].numpy(), v.numpy())
    if os.path.exists(H5DIFF):          # the real HDF5 library reads our file and finds it identical
        env = dict(os.environ, LD_LIBRARY_PATH="/opt/conda/lib")
        r = subprocess.run([H5DIFF, out, os.path.join(G, "keras_weights_v0.h5")], capture_output=True,
                           text=True, env=env)
        assert r.returncode == 0, r.stdout + r.stderr


def test_h5write_wide_tree(tmp_path):
    g = h5write.Group()
    for i in range(700):
        g.group(f"layer_{i:04d}").datasets["v"] = np.arange(3, dtype=np.int32) + i
    g.datasets["m"] = np.linspace(0, 1, 1000).reshape(10, 100)
    g.attrs["names"] = np.array([b"a", b"bcd"])
    p = str(tmp_path / "w.h5")
    h5write.write(p, g)
    f = h5.File(p)
    assert len(f.keys()) == 701
    np.testing.assert_array_equal(f["layer_0633/v"].read(), [633, 634, 635])
    np.testing.assert_array_equal(f["m"].read(), np.linspace(0, 1, 1000).reshape(10, 100))
    dump = "/opt/conda/bin/h5dump"
    if os.path.exists(dump):
        r = subprocess.run([dump, "-d", "/layer_0633/v", p], capture_output=True, text=True,
                           env=dict(os.environ, LD_LIBRARY_PATH="/opt/conda/lib"))
        assert r.returncode == 0 and "633, 634, 635" in r.stdout


def test_full_model_weights_round_trip(tmp_path):
    """Every weight of the ResNet50 backbone + FPN + RPN head + heads survives save -> load."""
    from m3d.backbone import FPN, ResNet3D, RPNHead
    from m3d.heads import ClassifierHead, MaskHead

    def build(seed):
        st = ParamStore()
        ResNet3D(st, "resnet50")
        FPN(st, 256)
        RPNHead(st, 1, 3, 256)
        ClassifierHead(st, 7, 2, 256, 256)
        MaskHead(st, 2, 64, 256)
        return st.finalize("cpu", seed=seed)

    a, b = build(1), build(2)
    for bn in a.bns:
        bn.moving_mean.uniform_(-1, 1)
        bn.moving_variance.uniform_(0.5, 2)
    p = str(tmp_path / "full.h5")
    weights.save_weights(a, p)
    loaded = weights.load_weights(b, p)
    assert "res5c_branch2c" in loaded and "mrcnn_mask_deconv" in loaded and "bn_conv1" in loaded
    sa, sb = a.state_dict(), b.state_dict()
    assert sa.keys() == sb.keys()
    for k in sa:
        assert np.array_equal(sa[k].numpy(), sb[k].numpy()), k


def _grid(shape, f):
    z, y, x = np.meshgrid(*[np.arange(n) for n in shape], indexing="ij")
    return f(z, y, x)


@pytest.mark.parametrize("fn,shape,f,dt", [
    ("stack_u8.tif", (5, 7, 9), lambda z, y, x: (7 * z + 3 * y + x) % 251, np.uint8),
    ("stack_u16_be_deflate.tif", (4, 6, 11), lambda z, y, x: 1000 * z + 17 * y + 5 * x, np.uint16),
    ("stack_u8_packbits_big.tif", (3, 5, 6), lambda z, y, x: (7 * z + 3 * y + x) % 251, np.uint8)])
def test_tiff_reader(fn, shape, f, dt):
    a = tiff.imread(os.path.join(G, fn))
    assert a.dtype == dt and a.shape == shape
    np.testing.assert_array_equal(a, _grid(shape, f).astype(dt))


class _Evil:
    def __reduce__(self):
        return (os.system, ("echo pwned",))


def _make_dataset(tmp_path, mask_obj=None):
    d = tmp_path / "data"
    (d / "datasets").mkdir(parents=True)
    img = str(d / "img.tif")
    shutil.copy(os.path.join(G, "stack_u8.tif"), img)                 # (Z,Y,X) = (5,7,9)
    cab = str(d / "img.dat")
    # class z1 y1 x1 z2 y2 x2 (prepocess.ipynb order); row 3 is invalid (z2 <= z1)
    np.savetxt(cab, np.array([[1, 0, 1, 2, 3, 5, 6], [1, 1, 0, 0, 4, 3, 9], [1, 3, 1, 1, 3, 2, 2]]), fmt="%d")
    m = np.zeros((5, 7, 9, 2), bool)
    m[0:3, 1:5, 2:6, 0] = True
    m[1:4, 0:3, 0:9, 1] = True
    with bz2.BZ2File(str(d / "m.pickle"), "wb") as f:
        pickle.dump(m if mask_obj is None else mask_obj, f)
    with open(d / "datasets" / "train.csv", "w") as f:
        f.write("Images;Segs;Cabs;Masks\n")
        f.write(f"{img};;{cab};{d / 'm.pickle'}\n")
    return str(d), m


def test_toy_dataset(tmp_path):
    root, m = _make_dataset(tmp_path)
    ds = dataset.ToyDataset()
    ds.load_dataset(root, is_train=True)
    ds.prepare()
    assert ds.num_images == 1 and ds.class_names == ["BG", "neuron"]
    im = ds.load_image(0)
    raw = np.transpose(tiff.imread(os.path.join(G, "stack_u8.tif")), (1, 2, 0)).astype(np.float32)
    p1, p99 = np.percentile(raw, [1, 99])
    c = np.clip(raw, p1, p99)
    np.testing.assert_allclose(im[..., 0], np.tanh((c - c.mean()) / c.std() * 0.5), rtol=1e-6, atol=1e-6)
    assert im.shape == (7, 9, 5, 1) and im.dtype == np.float32
    boxes, cls, masks = ds.load_data(0)
    np.testing.assert_array_equal(boxes, [[1, 2, 0, 5, 6, 3], [0, 0, 1, 3, 9, 4]])
    np.testing.assert_array_equal(cls, [1, 1])
    assert masks.dtype == np.float32 and masks.shape == (7, 9, 5, 2)
    np.testing.assert_array_equal(masks, np.transpose(m, (1, 2, 0, 3)).astype(np.float32))


def test_mask_pickle_refuses_code(tmp_path):
    root, _ = _make_dataset(tmp_path, mask_obj=_Evil())
    with pytest.raises(pickle.UnpicklingError):
        dataset.load_mask_pickle(os.path.join(root, "m.pickle"))
    ds = dataset.ToyDataset()
    ds.load_dataset(root)
    _, _, masks = ds.load_data(0)                    # reference fallback: no masks
    assert masks.shape == (7, 9, 5, 0)
