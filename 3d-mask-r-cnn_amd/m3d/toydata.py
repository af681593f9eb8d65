"""Seeded toy-shapes volumes: the reference's synthetic dataset generator
(generate_data.py:15-231) as an in-memory function, for BASELINE configs[0]
(RPN training on one 64^3 toy-shapes volume) and the tests.

Per volume (generate_data.py create_data, :59-145): 3..20 objects, each an
ellipsoid (class 1), cuboid (2) or pyramid (3) of base size ``base`` times a
factor in [1/2, 2] per axis (getEllipsoid / getCuboid / getPyramid,
:147-190), rotated about the three axes by random angles with 1 voxel of
padding (apply_random_rotation, :34-46; scipy.ndimage.rotate, reshape=True,
mode='nearest', order 3 as scipy's default), cropped to its bounding box,
placed at a random position where it overlaps no earlier object (up to 100
failed trials), intensity += U(0.02, 0.10) on the object; then Poisson(10 I)/10
+ N(0, 0.05) + U(0, 0.01) noise (apply_noise, :19-31) and a min-max rescale
to uint8 (:139-141).  Boxes are (y1, x1, z1, y2+1, x2+1, z2+1) with the class
id (the .dat rows, :123), masks [H, W, D, N] bool (the bz2 pickle, :134).

Differences, stated: the reference draws from Python's ``random`` and
numpy's global state unseeded; here one ``numpy.random.Generator(seed)``
drives everything, so a seed reproduces a volume.  ``base`` defaults to the
reference's 15 scaled by size/128 (the reference's constant assumes 128^3
volumes: at 64^3 its largest objects do not fit and random.randint raises).
The returned arrays are (Y, X, Z) = the network's [H, W, D] order; the
reference writes the same axes (Appendix B.9).
"""
from __future__ import annotations

import numpy as np

NUM_MAX_OBJECTS = 20    # generate_data.py:17
RANGE_RANDOM = 2.0      # :16


def _factor(rng, rr):
    return rng.uniform(1.0 / rr, rr)


def _rotate(obj, rng):
    from scipy.ndimage import rotate
    o = np.pad(obj, 1, mode="constant", constant_values=0)
    ax, ay, az = (rng.uniform(0, 360) for _ in range(3))
    o = rotate(o, ax, axes=(1, 2), reshape=True, mode="nearest")
    o = rotate(o, ay, axes=(0, 2), reshape=True, mode="nearest")
    o = rotate(o, az, axes=(0, 1), reshape=True, mode="nearest")
    return o


def _crop(o):
    nz = np.nonzero(o)
    if not len(nz[0]):
        return None
    return o[nz[0].min():nz[0].max() + 1, nz[1].min():nz[1].max() + 1, nz[2].min():nz[2].max() + 1]


def ellipsoid(base, rr, rng):
    r = [max(1, int(base * _factor(rng, rr))) for _ in range(3)]    # rx, ry, rz
    m = 2 * max(r)
    c = m // 2
    z, y, x = np.meshgrid(np.arange(m), np.arange(m), np.arange(m), indexing="ij")
    e = (((x - c) / r[0]) ** 2 + ((y - c) / r[1]) ** 2 + ((z - c) / r[2]) ** 2 <= 1)
    obj = np.transpose(e, (1, 2, 0)).astype(np.uint8)               # [y, x, z]
    return _crop(_rotate(obj, rng))


def cuboid(base, rr, rng):
    lx, ly, lz = (max(1, 2 * int(base * _factor(rng, rr))) for _ in range(3))
    return _crop(_rotate(np.ones((lx, ly, lz), np.uint8), rng))


def pyramid(base, rr, rng):
    lx, ly, lz = (max(1, 2 * int(base * _factor(rng, rr))) for _ in range(3))
    p = np.zeros((ly, lx, lz), np.uint8)
    for z in range(lz):
        xs, ys = int((1 - z / lz) * lx), int((1 - z / lz) * ly)
        p[:ys, :xs, z] = 1
    return _crop(_rotate(p, rng))


_SHAPES = ((ellipsoid, 1), (cuboid, 2), (pyramid, 3))


def toy_volume(size=64, seed=0, base=None, max_objects=NUM_MAX_OBJECTS):
    """One toy-shapes volume.  Returns dict(image uint8 [S,S,S] (y,x,z),
    boxes int32 [N,6] (y1,x1,z1,y2,x2,z2), class_ids int32 [N],
    masks bool [S,S,S,N])."""
    rng = np.random.default_rng(seed)
    base = 15.0 * size / 128.0 if base is None else float(base)
    shape = (size, size, size)
    img = np.zeros(shape, np.float64)
    seg = np.zeros(shape, np.uint16)
    n_target = int(rng.integers(3, max_objects + 1))
    boxes, classes, masks = [], [], []
    trial = 0
    while len(boxes) < n_target and trial <= 100:
        make, cls = _SHAPES[int(rng.integers(0, 3))]
        obj = make(base, RANGE_RANDOM, rng)
        dy, dx, dz = (int(0.5 * s) for s in obj.shape) if obj is not None else (size, size, size)
        if obj is None or any(2 * d + 1 >= size for d in (dy, dx, dz)):
            trial += 1
            continue
        y = int(rng.integers(dy, size - dy))       # random.randint(d, S - d - 1)
        x = int(rng.integers(dx, size - dx))
        z = int(rng.integers(dz, size - dz))
        cy, cx, cz = np.nonzero(obj)
        cy, cx, cz = cy + y - dy, cx + x - dx, cz + z - dz
        ok = (cy < size) & (cx < size) & (cz < size)
        cy, cx, cz = cy[ok], cx[ok], cz[ok]
        if np.any(seg[cy, cx, cz]):
            trial += 1
            continue
        seg[cy, cx, cz] = len(boxes) + 1
        img[cy, cx, cz] += rng.uniform(0.02, 0.10)
        m = np.zeros(shape, bool)
        m[cy, cx, cz] = True
        masks.append(m)
        boxes.append([cy.min(), cx.min(), cz.min(), cy.max() + 1, cx.max() + 1, cz.max() + 1])
        classes.append(cls)
    img = rng.poisson(img * 10) / 10.0 + rng.normal(0, 0.05, shape) + rng.uniform(0, 0.01, shape)
    img = 255 * (img - img.min()) / (img.max() - img.min())
    return {"image": img.astype(np.uint8),
            "boxes": np.asarray(boxes, np.int32).reshape(-1, 6),
            "class_ids": np.asarray(classes, np.int32),
            "masks": np.stack(masks, -1) if masks else np.zeros(shape + (0,), bool)}


def network_input(image_yxz):
    """The ToyDataset normalisation (m3d.dataset.normalize_image, which takes
    the (Z,Y,X) file order) of a toy volume -> [1, S, S, S, 1] float32."""
    from .dataset import normalize_image
    return normalize_image(np.transpose(image_yxz, (2, 0, 1)))[None]
