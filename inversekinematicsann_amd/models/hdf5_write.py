"""A minimal HDF5 writer -- enough for the Keras `model.save('*.h5')` layout.

ANN.save_model (kinematics/ann.py:87-95 of the reference) writes
`<prefix>_<timestamp>.h5` with Keras and the two scalers with joblib.  Neither
Keras nor h5py is available to the product interpreter, so this module writes
the same file structure from the HDF5 file-format specification directly, in
its "latest" encoding (what h5py writes with libver='latest'):

* superblock version 2 (checksummed);
* version-2 object headers ("OHDR", one chunk, checksummed) holding the
  messages: link info + group info + link messages for groups (compact link
  storage), dataspace + datatype + fill value + contiguous layout for datasets,
  and version-3 attribute messages;
* little-endian IEEE floats / integers and fixed-length ASCII strings (scalar or
  1-D arrays).

The checksums are Bob Jenkins' lookup3 `hashlittle` (initval 0), which the spec
names for every checksummed structure.  models/hdf5_min.py reads these files
back; the CPU tests also read them with h5py where an interpreter has it.
"""
from __future__ import annotations

import struct
from typing import Dict, List, Tuple, Union

import numpy as np

SIGNATURE = b"\x89HDF\r\n\x1a\n"
UNDEF = 0xFFFFFFFFFFFFFFFF

Value = Union[str, bytes, int, float, np.ndarray, List[str], List[bytes]]


def lookup3(data: bytes, initval: int = 0) -> int:
    """Jenkins lookup3 hashlittle (the HDF5 metadata checksum)."""
    M = 0xFFFFFFFF

    def rot(x, k):
        return ((x << k) | (x >> (32 - k))) & M

    n = len(data)
    a = b = c = (0xDEADBEEF + n + initval) & M
    i = 0
    while n > 12:
        a = (a + struct.unpack_from("<I", data, i)[0]) & M
        b = (b + struct.unpack_from("<I", data, i + 4)[0]) & M
        c = (c + struct.unpack_from("<I", data, i + 8)[0]) & M
        a = (a - c) & M; a ^= rot(c, 4); c = (c + b) & M
        b = (b - a) & M; b ^= rot(a, 6); a = (a + c) & M
        c = (c - b) & M; c ^= rot(b, 8); b = (b + a) & M
        a = (a - c) & M; a ^= rot(c, 16); c = (c + b) & M
        b = (b - a) & M; b ^= rot(a, 19); a = (a + c) & M
        c = (c - b) & M; c ^= rot(b, 4); b = (b + a) & M
        i += 12
        n -= 12
    if n == 0:
        return c
    tail = data[i:] + b"\0" * (12 - n)
    a = (a + struct.unpack_from("<I", tail, 0)[0]) & M
    b = (b + struct.unpack_from("<I", tail, 4)[0]) & M
    c = (c + struct.unpack_from("<I", tail, 8)[0]) & M
    c ^= b; c = (c - rot(b, 14)) & M
    a ^= c; a = (a - rot(c, 11)) & M
    b ^= a; b = (b - rot(a, 25)) & M
    c ^= b; c = (c - rot(b, 16)) & M
    a ^= c; a = (a - rot(c, 4)) & M
    b ^= a; b = (b - rot(a, 14)) & M
    c ^= b; c = (c - rot(b, 24)) & M
    return c


# ---- message bodies ----------------------------------------------------------------
def _dtype_msg(dt: np.dtype) -> bytes:
    dt = np.dtype(dt)
    if dt.kind == "f":
        bits = dt.itemsize * 8
        if bits == 32:
            props = struct.pack("<HHBBBBI", 0, 32, 23, 8, 0, 23, 127)
        elif bits == 64:
            props = struct.pack("<HHBBBBI", 0, 64, 52, 11, 0, 52, 1023)
        else:
            raise ValueError(f"float{bits} not supported")
        # class 1, version 1; byte order LE, mantissa normalisation 2 (msb implied),
        # sign at bit (bits - 1)
        return bytes([0x11, 0x20, bits - 1, 0]) + struct.pack("<I", dt.itemsize) + props
    if dt.kind in "iu":
        flags = 0x08 if dt.kind == "i" else 0x00
        return bytes([0x10, flags, 0, 0]) + struct.pack("<I", dt.itemsize) + \
            struct.pack("<HH", 0, dt.itemsize * 8)
    if dt.kind == "S":
        # class 3 (string), version 1; null-padded, ASCII
        return bytes([0x13, 0x01, 0, 0]) + struct.pack("<I", dt.itemsize)
    raise ValueError(f"dtype {dt} not supported")


def _dataspace_msg(shape: Tuple[int, ...]) -> bytes:
    if len(shape) == 0:
        return bytes([2, 0, 0, 0])  # version 2, scalar
    return bytes([2, len(shape), 0, 1]) + b"".join(struct.pack("<Q", d) for d in shape)


def _as_array(v: Value) -> np.ndarray:
    if isinstance(v, np.ndarray):
        return v
    if isinstance(v, (str, bytes)):
        b = v.encode("utf-8") if isinstance(v, str) else v
        return np.array(b, dtype=f"S{max(1, len(b))}")
    if isinstance(v, (list, tuple)):
        bs = [x.encode("utf-8") if isinstance(x, str) else x for x in v]
        return np.array(bs, dtype=f"S{max([1] + [len(x) for x in bs])}")
    if isinstance(v, bool):
        return np.array(int(v), np.int8)
    if isinstance(v, int):
        return np.array(v, np.int64)
    if isinstance(v, float):
        return np.array(v, np.float64)
    raise TypeError(f"attribute value {v!r} not supported")


def _attr_msg(name: str, v: Value) -> bytes:
    a = _as_array(v)
    dt = _dtype_msg(a.dtype)
    ds = _dataspace_msg(a.shape)
    nm = name.encode("utf-8") + b"\0"
    # version 3: no padding of name / datatype / dataspace; encoding 0 (ASCII)
    return struct.pack("<BBHHHB", 3, 0, len(nm), len(dt), len(ds), 0) + nm + dt + ds + \
        np.ascontiguousarray(a).tobytes()


def _link_msg(name: str, addr: int) -> bytes:
    nm = name.encode("utf-8")
    if len(nm) > 255:
        raise ValueError("link names up to 255 bytes")
    # version 1, flags 0: 1-byte name length, hard link, no creation order
    return bytes([1, 0, len(nm)]) + nm + struct.pack("<Q", addr)


# link info (version 0, no creation order, no dense storage) and group info
_LINK_INFO = bytes([0, 0]) + struct.pack("<QQ", UNDEF, UNDEF)
_GROUP_INFO = bytes([0, 0])
# fill value v3: allocation early, write time "if set", no value defined
_FILL = bytes([3, 0x09])


def _ohdr(msgs: List[Tuple[int, bytes]]) -> bytes:
    body = b"".join(struct.pack("<BHB", t, len(d), 0) + d for t, d in msgs)
    n = len(body)
    if n < 256:
        size = struct.pack("<B", n); flags = 0x00
    elif n < 65536:
        size = struct.pack("<H", n); flags = 0x01
    else:
        size = struct.pack("<I", n); flags = 0x02
    h = b"OHDR" + bytes([2, flags]) + size + body
    return h + struct.pack("<I", lookup3(h))


class _Node:
    def __init__(self):
        self.attrs: Dict[str, Value] = {}


class Group(_Node):
    def __init__(self):
        super().__init__()
        self.children: Dict[str, _Node] = {}

    def group(self, path: str) -> "Group":
        g = self
        for part in path.strip("/").split("/"):
            if part not in g.children:
                g.children[part] = Group()
            g = g.children[part]
            if not isinstance(g, Group):
                raise ValueError(f"{path}: {part} is a dataset")
        return g

    def dataset(self, path: str, data: np.ndarray):
        parts = path.strip("/").split("/")
        g = self.group("/".join(parts[:-1])) if len(parts) > 1 else self
        d = Dataset(np.ascontiguousarray(data))
        g.children[parts[-1]] = d
        return d


class Dataset(_Node):
    def __init__(self, data: np.ndarray):
        super().__init__()
        if data.dtype.byteorder == ">":
            data = data.astype(data.dtype.newbyteorder("<"))
        self.data = data


def write(path: str, root: Group):
    """Write the tree under `root` (attributes, groups, datasets) to `path`."""
    blobs: List[bytes] = []
    pos = [48]  # the superblock

    def alloc(b: bytes) -> int:
        a = pos[0]
        blobs.append(b)
        pos[0] += len(b)
        pad = (-pos[0]) % 8
        if pad:
            blobs.append(b"\0" * pad)
            pos[0] += pad
        return a

    def emit(node: _Node) -> int:
        attrs = [(0x000C, _attr_msg(k, v)) for k, v in node.attrs.items()]
        if isinstance(node, Dataset):
            raw = node.data.tobytes()
            daddr = alloc(raw) if raw else UNDEF
            layout = bytes([3, 1]) + struct.pack("<QQ", daddr, len(raw))
            msgs = [(0x0001, _dataspace_msg(node.data.shape)), (0x0003, _dtype_msg(node.data.dtype)),
                    (0x0005, _FILL), (0x0008, layout)] + attrs
        else:
            links = [(0x0006, _link_msg(name, emit(child)))
                     for name, child in node.children.items()]
            msgs = [(0x0002, _LINK_INFO), (0x000A, _GROUP_INFO)] + links + attrs
        return alloc(_ohdr(msgs))

    root_addr = emit(root)
    eof = pos[0]
    sb = SIGNATURE + bytes([2, 8, 8, 0]) + struct.pack("<QQQQ", 0, UNDEF, eof, root_addr)
    sb += struct.pack("<I", lookup3(sb))
    assert len(sb) == 48
    with open(path, "wb") as f:
        f.write(sb)
        for b in blobs:
            f.write(b)
