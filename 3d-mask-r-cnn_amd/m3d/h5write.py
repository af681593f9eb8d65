"""Minimal HDF5 writer for Keras weight files (superblock 0, v1 object
headers, symbol-table groups, contiguous datasets) -- the layout h5py writes by
default, so files from ``m3d.weights.save_weights`` load in the reference
(``keras_model.load_weights``) and in any HDF5 tool.  Checked in the tests by
reading back with m3d.h5 and, when the image's HDF5 tools are present, with
``h5dump``.

Usage: build a ``Group`` tree (``attrs``: name -> numpy value of a float /
int / fixed-length bytes dtype; ``datasets``: name -> numpy array; ``group(name)``
for sub-groups) and call ``write(path, root)``.
"""
from __future__ import annotations

import struct

import numpy as np

SO = SL = 8
UNDEF = (1 << 64) - 1
LEAF_K = 4            # symbol-table node holds 2*LEAF_K entries
NODE_K = 16           # group B-tree node holds 2*NODE_K children
_FREE_NULL = 1        # local-heap "no free block" marker


class Group:
    def __init__(self):
        self.attrs = {}
        self.datasets = {}
        self.groups = {}

    def group(self, name):
        if "/" in name:
            head, rest = name.split("/", 1)
            return self.group(head).group(rest)
        return self.groups.setdefault(name, Group())


def _pad8(b: bytes) -> bytes:
    return b + b"\0" * (-len(b) % 8)


def _dtype_msg(dt: np.dtype) -> bytes:
    if dt.kind == "f":
        size = dt.itemsize
        be = 1 if dt.byteorder == ">" else 0
        if size == 4:
            props = struct.pack("<HHBBBBI", 0, 32, 23, 8, 0, 23, 127)
            sign = 31
        elif size == 8:
            props = struct.pack("<HHBBBBI", 0, 64, 52, 11, 0, 52, 1023)
            sign = 63
        else:
            raise ValueError(f"float{8 * size}")
        return bytes([0x11, be | 0x20, sign, 0]) + struct.pack("<I", size) + props
    if dt.kind in "iu":
        be = 1 if dt.byteorder == ">" else 0
        signed = 0x08 if dt.kind == "i" else 0
        return bytes([0x10, be | signed, 0, 0]) + struct.pack("<I", dt.itemsize) + \
            struct.pack("<HH", 0, 8 * dt.itemsize)
    if dt.kind == "S":
        return bytes([0x13, 0x01, 0, 0]) + struct.pack("<I", dt.itemsize)   # null-padded ASCII
    raise ValueError(f"unsupported dtype {dt}")


def _space_msg(shape) -> bytes:
    return bytes([1, len(shape), 0, 0]) + b"\0" * 4 + b"".join(struct.pack("<Q", d) for d in shape)


def _msg(mtype: int, data: bytes) -> bytes:
    data = _pad8(data)
    return struct.pack("<HHB3x", mtype, len(data), 0) + data


def _attr_msg(name: str, value) -> bytes:
    a = np.asarray(value)
    if a.dtype.kind == "U":
        a = np.char.encode(a, "utf8")
    if a.dtype.byteorder == "=":
        a = a.astype(a.dtype.newbyteorder("<"))
    nm = name.encode() + b"\0"
    dt, sp = _dtype_msg(a.dtype), _space_msg(a.shape)
    body = struct.pack("<BBHHH", 1, 0, len(nm), len(dt), len(sp)) + _pad8(nm) + _pad8(dt) + _pad8(sp)
    return _msg(0x0C, body + a.tobytes())


def _header(msgs) -> bytes:
    body = b"".join(msgs)
    return struct.pack("<BBHII", 1, 0, len(msgs), 1, len(body)) + b"\0" * 4 + body


class _Out:
    def __init__(self):
        self.buf = bytearray(96)          # superblock, filled last

    def alloc(self, data: bytes) -> int:
        a = len(self.buf)
        self.buf += data
        self.buf += b"\0" * (-len(self.buf) % 8)
        return a


def _write_dataset(out: _Out, arr: np.ndarray) -> int:
    a = np.ascontiguousarray(arr)
    if a.dtype.byteorder == "=":
        a = a.astype(a.dtype.newbyteorder("<"))
    data_addr = out.alloc(a.tobytes()) if a.nbytes else UNDEF
    layout = bytes([3, 1]) + struct.pack("<QQ", data_addr, a.nbytes)
    msgs = [_msg(0x01, _space_msg(a.shape)), _msg(0x03, _dtype_msg(a.dtype)), _msg(0x08, layout)]
    return out.alloc(_header(msgs))


def _write_group(out: _Out, g: Group):
    """Returns (object header address, B-tree address, heap address)."""
    children = {}
    for name, sub in g.groups.items():
        children[name.encode()] = _write_group(out, sub)[0]
    for name, arr in g.datasets.items():
        children[name.encode()] = _write_dataset(out, np.asarray(arr))
    names = sorted(children)
    # local heap: offset 0 = "" (key 0 of the B-tree), then every name
    heap_data = bytearray(8)
    offs = {}
    for n in names:
        offs[n] = len(heap_data)
        heap_data += _pad8(n + b"\0")
    heap_hdr_len = 32
    heap_addr = len(out.buf)
    out.alloc(b"HEAP" + bytes([0, 0, 0, 0]) + struct.pack("<QQQ", len(heap_data), _FREE_NULL,
                                                           heap_addr + heap_hdr_len) + bytes(heap_data))
    # symbol-table nodes, 2*LEAF_K entries each
    snod_cap = 2 * LEAF_K
    leaves = []                           # (address, last name)
    for i in range(0, max(len(names), 1), snod_cap):
        part = names[i:i + snod_cap]
        b = bytearray(b"SNOD" + bytes([1, 0]) + struct.pack("<H", len(part)))
        for n in part:
            b += struct.pack("<QQII16x", offs[n], children[n], 0, 0)
        b += b"\0" * ((snod_cap - len(part)) * (2 * SO + 24))
        leaves.append((out.alloc(bytes(b)), part[-1] if part else b""))
    # B-tree levels, 2*NODE_K children per node, keys = heap offsets of the
    # last name of each child (key 0 = "")
    cap = 2 * NODE_K
    node_size = 8 + 2 * SO + (cap + 1) * SL + cap * SO
    level, nodes = 0, leaves
    while True:
        groups = [nodes[i:i + cap] for i in range(0, len(nodes), cap)]
        addrs = [len(out.buf) + j * node_size for j in range(len(groups))]
        new = []
        for j, grp in enumerate(groups):
            left = addrs[j - 1] if j > 0 else UNDEF
            right = addrs[j + 1] if j + 1 < len(groups) else UNDEF
            b = bytearray(b"TREE" + bytes([0, level]) + struct.pack("<HQQ", len(grp) if names else 0, left, right))
            b += struct.pack("<Q", 0)
            for addr, last in grp:
                b += struct.pack("<QQ", addr, offs.get(last, 0))
            b += b"\0" * (node_size - len(b))
            out.alloc(bytes(b))
            new.append((addrs[j], grp[-1][1]))
        if len(new) == 1:
            btree = new[0][0]
            break
        nodes, level = new, level + 1
    msgs = [_msg(0x11, struct.pack("<QQ", btree, heap_addr))]
    for name, v in g.attrs.items():
        msgs.append(_attr_msg(name, v))
    return out.alloc(_header(msgs)), btree, heap_addr


def write(path, root: Group):
    out = _Out()
    hdr, btree, heap = _write_group(out, root)
    eof = len(out.buf)
    sb = bytearray(b"\x89HDF\r\n\x1a\n")
    sb += bytes([0, 0, 0, 0, 0, SO, SL, 0]) + struct.pack("<HHI", LEAF_K, NODE_K, 0)
    sb += struct.pack("<QQQQ", 0, UNDEF, eof, UNDEF)
    sb += struct.pack("<QQII", 0, hdr, 1, 0) + struct.pack("<QQ", btree, heap)
    assert len(sb) == 96
    out.buf[:96] = sb
    with open(path, "wb") as f:
        f.write(bytes(out.buf))
