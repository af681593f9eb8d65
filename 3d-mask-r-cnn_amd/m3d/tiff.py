"""Minimal multi-page TIFF reader (no scikit-image / tifffile in this image).

The reference reads its volumes with ``skimage.io.imread`` (Z-first stacks,
core/data_generators.py:1609-1610, written by ``io.imsave`` in
generate_data.py:138-143).  This reads baseline TIFF and BigTIFF files, either
byte order, strip-organised, grayscale (or chunky multi-sample) pages of 8/16/
32/64-bit unsigned, signed or IEEE-float samples, uncompressed, PackBits or
Deflate (with horizontal predictor), and stacks the pages into a ``(Z, Y, X)``
(or ``(Z, Y, X, S)``) array.  Tiled or LZW/JPEG files raise
``NotImplementedError``.  Pinned by tests/test_formats.py against files
written by libtiff (tests/golden/h5src/make_tiff_fixtures.c).
"""
from __future__ import annotations

import struct
import zlib

import numpy as np

_TYPES = {1: "B", 2: "B", 3: "H", 4: "I", 5: "II", 6: "b", 8: "h", 9: "i", 10: "ii", 11: "f",
          12: "d", 16: "Q", 17: "q", 18: "Q"}


def _packbits(data: bytes, n: int) -> bytes:
    out = bytearray()
    i = 0
    while i < len(data) and len(out) < n:
        h = data[i]
        i += 1
        if h < 128:
            out += data[i:i + h + 1]
            i += h + 1
        elif h > 128:
            out += bytes([data[i]]) * (257 - h)
            i += 1
    return bytes(out)


def _pages(buf: bytes):
    bo = {b"II": "<", b"MM": ">"}.get(buf[:2])
    if bo is None:
        raise ValueError("not a TIFF file")
    magic = struct.unpack(bo + "H", buf[2:4])[0]
    if magic == 42:
        big, off = False, struct.unpack(bo + "I", buf[4:8])[0]
    elif magic == 43:
        big, off = True, struct.unpack(bo + "Q", buf[8:16])[0]
    else:
        raise ValueError(f"bad TIFF magic {magic}")
    seen = set()
    while off and off not in seen:
        seen.add(off)
        if big:
            n = struct.unpack(bo + "Q", buf[off:off + 8])[0]
            p, esz = off + 8, 20
        else:
            n = struct.unpack(bo + "H", buf[off:off + 2])[0]
            p, esz = off + 2, 12
        tags = {}
        for i in range(n):
            e = p + i * esz
            tag, typ = struct.unpack(bo + "HH", buf[e:e + 4])
            cnt = struct.unpack(bo + ("Q" if big else "I"), buf[e + 4:e + (12 if big else 8)])[0]
            fmt = _TYPES.get(typ)
            if fmt is None:
                continue
            size = struct.calcsize("=" + fmt) * cnt
            inline = 8 if big else 4
            vo = e + (12 if big else 8)
            if size > inline:
                vo = struct.unpack(bo + ("Q" if big else "I"), buf[vo:vo + inline])[0]
            vals = struct.unpack(bo + fmt * cnt, buf[vo:vo + size])
            tags[tag] = vals
        yield bo, tags
        q = p + n * esz
        off = struct.unpack(bo + ("Q" if big else "I"), buf[q:q + (8 if big else 4)])[0]


def _page_array(buf, bo, t):
    w, h = t[256][0], t[257][0]
    spp = t.get(277, (1,))[0]
    bps = t.get(258, (1,))[0]
    fmt = t.get(339, (1,))[0]
    comp = t.get(259, (1,))[0]
    pred = t.get(317, (1,))[0]
    if t.get(284, (1,))[0] != 1 and spp > 1:
        raise NotImplementedError("planar-separate TIFF samples")
    if 322 in t:
        raise NotImplementedError("tiled TIFF")
    kind = {1: "u", 2: "i", 3: "f"}[fmt]
    if bps not in (8, 16, 32, 64):
        raise NotImplementedError(f"{bps}-bit TIFF samples")
    dt = np.dtype(f"{bo}{kind}{bps // 8}")
    offs, counts = t[273], t[279]
    rps = t.get(278, (h,))[0]
    row_bytes = w * spp * dt.itemsize
    out = bytearray()
    for o, c in zip(offs, counts):
        raw = buf[o:o + c]
        need = min(rps, h - len(out) // row_bytes) * row_bytes
        if comp == 1:
            data = raw[:need]
        elif comp in (8, 32946):
            data = zlib.decompress(raw)
        elif comp == 32773:
            data = _packbits(raw, need)
        else:
            raise NotImplementedError(f"TIFF compression {comp}")
        if pred == 2:
            a = np.frombuffer(data[:need], dt).reshape(-1, w, spp).astype(dt.newbyteorder("="))
            a = np.cumsum(a, axis=1, dtype=a.dtype)
            data = a.astype(dt).tobytes()
        elif pred not in (1,):
            raise NotImplementedError(f"TIFF predictor {pred}")
        out += data[:need]
    arr = np.frombuffer(bytes(out[:h * row_bytes]), dt).reshape(h, w, spp) if spp > 1 else \
        np.frombuffer(bytes(out[:h * row_bytes]), dt).reshape(h, w)
    return arr.astype(dt.newbyteorder("="))


def imread(path) -> np.ndarray:
    """All pages of a TIFF file, stacked: (Z, Y, X[, S]); a single page -> (Y, X[, S])."""
    with open(path, "rb") as f:
        buf = f.read()
    pages = [_page_array(buf, bo, t) for bo, t in _pages(buf)]
    if not pages:
        raise ValueError(f"{path}: no image pages")
    return pages[0] if len(pages) == 1 else np.stack(pages)
