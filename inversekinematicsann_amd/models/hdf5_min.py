"""A minimal, read-only HDF5 parser -- enough for Keras `model.save('*.h5')` files.

h5py is not available to the product interpreter (nor on the GPU box), so
ANN.load_model (kinematics/ann.py:78-85) reads the reference's model format
with this parser.  It implements the parts of the HDF5 file-format spec that
h5py/libhdf5 write for such files:

* superblock versions 0/1 (libver 'earliest', the h5py default) and 2/3;
* object headers v1 and v2 ("OHDR", with "OCHK" continuation chunks);
* groups as symbol tables (v1 B-tree of "SNOD" nodes + local "HEAP") and as
  compact link messages (libver 'latest');
* attributes (message versions 1-3) with fixed- or variable-length strings
  (global heap "GCOL"), integer and float scalars / arrays;
* datasets with compact or contiguous layout of little/big-endian IEEE floats
  and integers.

Anything else (chunked/filtered datasets, dense attribute or link storage,
external files) raises Hdf5Error.  No code from the file is executed.
"""
from __future__ import annotations

import struct
from typing import Dict, List, Optional

import numpy as np

SIGNATURE = b"\x89HDF\r\n\x1a\n"
UNDEF = 0xFFFFFFFFFFFFFFFF


class Hdf5Error(ValueError):
    pass


class _Msg:
    __slots__ = ("type", "data")

    def __init__(self, t, d):
        self.type = t
        self.data = d


class Datatype:
    def __init__(self, cls, size, order="<", signed=True, vlen_str=False, base=None):
        self.cls = cls
        self.size = size
        self.order = order
        self.signed = signed
        self.vlen_str = vlen_str
        self.base = base

    def numpy(self):
        if self.cls == 0:
            return np.dtype(f"{self.order}{'i' if self.signed else 'u'}{self.size}")
        if self.cls == 1:
            return np.dtype(f"{self.order}f{self.size}")
        raise Hdf5Error(f"no numpy dtype for HDF5 class {self.cls}")


class H5Object:
    """An object header: attributes, links (groups) or data (datasets)."""

    def __init__(self, f: "H5File", addr: int):
        self.f = f
        self.addr = addr
        self.msgs: List[_Msg] = f._read_object_header(addr)

    # -- attributes --------------------------------------------------------
    @property
    def attrs(self) -> Dict[str, object]:
        out = {}
        for m in self.msgs:
            if m.type == 0x000C:
                name, value = self.f._parse_attribute(m.data)
                out[name] = value
            elif m.type == 0x0015:  # attribute info: dense storage if a fractal heap is named
                flags = m.data[1]
                off = 2 + (2 if flags & 1 else 0)
                if struct.unpack_from("<Q", m.data, off)[0] != UNDEF:
                    raise Hdf5Error("dense attribute storage is not supported")
        return out

    # -- groups -------------------------------------------------------------
    def links(self) -> Dict[str, int]:
        out: Dict[str, int] = {}
        for m in self.msgs:
            if m.type == 0x0011:  # symbol table
                btree, heap = struct.unpack_from("<QQ", m.data, 0)
                out.update(self.f._symbol_table_links(btree, heap))
            elif m.type == 0x0006:  # link message
                name, addr = self.f._parse_link(m.data)
                if addr is not None:
                    out[name] = addr
            elif m.type == 0x0002:  # link info: dense storage if a fractal heap is named
                d = m.data
                flags = d[1]
                off = 2 + (8 if flags & 1 else 0)
                heap_addr = struct.unpack_from("<Q", d, off)[0]
                if heap_addr != UNDEF:
                    raise Hdf5Error("dense link storage is not supported")
        return out

    def __getitem__(self, path: str) -> "H5Object":
        obj = self
        for part in [p for p in path.split("/") if p]:
            links = obj.links()
            if part not in links:
                raise KeyError(path)
            obj = H5Object(self.f, links[part])
        return obj

    def __contains__(self, path: str) -> bool:
        try:
            self[path]
            return True
        except KeyError:
            return False

    # -- datasets -----------------------------------------------------------
    def read(self) -> np.ndarray:
        shape = dtype = layout = None
        for m in self.msgs:
            if m.type == 0x0001:
                shape = self.f._parse_dataspace(m.data)
            elif m.type == 0x0003:
                dtype = self.f._parse_datatype(m.data, 0)[0]
            elif m.type == 0x0008:
                layout = m.data
            elif m.type == 0x000B:
                raise Hdf5Error("filtered datasets are not supported")
        if shape is None or dtype is None or layout is None:
            raise Hdf5Error("not a dataset")
        dt = dtype.numpy()
        count = int(np.prod(shape)) if shape else 1
        nbytes = count * dt.itemsize
        ver = layout[0]
        if ver not in (3, 4):  # v4 encodes compact / contiguous exactly as v3
            raise Hdf5Error(f"layout message version {ver} not supported")
        cls = layout[1]
        if cls == 0:  # compact
            size = struct.unpack_from("<H", layout, 2)[0]
            raw = layout[4:4 + size]
        elif cls == 1:  # contiguous
            addr, size = struct.unpack_from("<QQ", layout, 2)
            if addr == UNDEF:
                raw = b"\0" * nbytes
            else:
                raw = self.f._read(addr, nbytes)
        else:
            raise Hdf5Error("chunked datasets are not supported")
        return np.frombuffer(raw[:nbytes], dtype=dt).reshape(shape).astype(dt.newbyteorder("="))


class H5File(H5Object):
    def __init__(self, path: str):
        with open(path, "rb") as fh:
            self.buf = fh.read()
        base = None
        for off in (0, 512, 1024, 2048, 4096, 8192):
            if self.buf[off:off + 8] == SIGNATURE:
                base = off
                break
        if base is None:
            raise Hdf5Error(f"{path}: not an HDF5 file")
        self.base = base
        v = self.buf[base + 8]
        if v in (0, 1):
            so, sl = self.buf[base + 13], self.buf[base + 14]
            if (so, sl) != (8, 8):
                raise Hdf5Error("only 8-byte offsets/lengths are supported")
            p = base + 24 + (4 if v == 1 else 0)
            base_addr = struct.unpack_from("<Q", self.buf, p)[0]
            p += 32  # base, free-space, EOF, driver addresses
            root = struct.unpack_from("<Q", self.buf, p + 8)[0]  # symbol table entry
        elif v in (2, 3):
            so, sl = self.buf[base + 9], self.buf[base + 10]
            if (so, sl) != (8, 8):
                raise Hdf5Error("only 8-byte offsets/lengths are supported")
            base_addr, _ext, _eof, root = struct.unpack_from("<QQQQ", self.buf, base + 12)
        else:
            raise Hdf5Error(f"superblock version {v} not supported")
        self.base_addr = base + base_addr if base_addr == 0 else base_addr
        super().__init__(self, root)

    # -- raw access -----------------------------------------------------------
    def _read(self, addr: int, n: int) -> bytes:
        a = self.base_addr + addr
        if a + n > len(self.buf):
            raise Hdf5Error("read past end of file")
        return self.buf[a:a + n]

    # -- object headers ---------------------------------------------------------
    def _read_object_header(self, addr: int) -> List[_Msg]:
        head = self._read(addr, 16)
        if head[:4] == b"OHDR":
            return self._read_ohdr_v2(addr)
        if head[0] != 1:
            raise Hdf5Error(f"object header version {head[0]} not supported")
        nmsgs, _refc, hsize = struct.unpack_from("<HII", head, 2)
        msgs: List[_Msg] = []
        blocks = [(addr + 16, hsize)]
        while blocks and len(msgs) < nmsgs:
            start, size = blocks.pop(0)
            p, end = start, start + size
            while p + 8 <= end and len(msgs) < nmsgs:
                mt, ms, _flags = struct.unpack_from("<HHB", self._read(p, 5), 0)
                data = self._read(p + 8, ms)
                if mt == 0x0010:
                    caddr, clen = struct.unpack_from("<QQ", data, 0)
                    blocks.append((caddr, clen))
                msgs.append(_Msg(mt, data))
                p += 8 + ms
        return msgs

    def _read_ohdr_v2(self, addr: int) -> List[_Msg]:
        flags = self._read(addr + 5, 1)[0]
        p = addr + 6
        if flags & 0x20:
            p += 16  # times
        if flags & 0x10:
            p += 4  # attribute phase change
        szlen = 1 << (flags & 3)
        size = int.from_bytes(self._read(p, szlen), "little")
        p += szlen
        track_order = bool(flags & 0x04)
        msgs: List[_Msg] = []
        chunks = [(p, size)]
        while chunks:
            start, size = chunks.pop(0)
            q, end = start, start + size
            while q + 4 <= end:
                mt = self._read(q, 1)[0]
                ms = struct.unpack_from("<H", self._read(q + 1, 2), 0)[0]
                q += 4 + (2 if track_order else 0)
                if q + ms > end:
                    break
                data = self._read(q, ms)
                if mt == 0x10:
                    caddr, clen = struct.unpack_from("<QQ", data, 0)
                    if self._read(caddr, 4) != b"OCHK":
                        raise Hdf5Error("bad continuation chunk")
                    chunks.append((caddr + 4, clen - 8))  # minus signature and checksum
                msgs.append(_Msg(mt, data))
                q += ms
        return msgs

    # -- groups -------------------------------------------------------------------
    def _local_heap_data(self, heap: int) -> bytes:
        h = self._read(heap, 32)
        if h[:4] != b"HEAP":
            raise Hdf5Error("bad local heap")
        size, _free, data_addr = struct.unpack_from("<QQQ", h, 8)
        return self._read(data_addr, size)

    def _symbol_table_links(self, btree: int, heap: int) -> Dict[str, int]:
        names = self._local_heap_data(heap)
        out: Dict[str, int] = {}

        def name_at(off):
            end = names.index(b"\0", off)
            return names[off:end].decode("utf-8")

        def walk(node):
            hdr = self._read(node, 24)
            if hdr[:4] != b"TREE" or hdr[4] != 0:
                raise Hdf5Error("bad group B-tree node")
            level = hdr[5]
            used = struct.unpack_from("<H", hdr, 6)[0]
            p = node + 24
            for i in range(used):
                child = struct.unpack_from("<Q", self._read(p + 8, 8), 0)[0]
                p += 16
                if level > 0:
                    walk(child)
                else:
                    snod = self._read(child, 8)
                    if snod[:4] != b"SNOD":
                        raise Hdf5Error("bad symbol table node")
                    nsym = struct.unpack_from("<H", snod, 6)[0]
                    for k in range(nsym):
                        e = self._read(child + 8 + 40 * k, 40)
                        noff, oaddr = struct.unpack_from("<QQ", e, 0)
                        out[name_at(noff)] = oaddr

        walk(btree)
        return out

    def _parse_link(self, d: bytes):
        flags = d[1]
        p = 2
        ltype = 0
        if flags & 0x08:
            ltype = d[p]
            p += 1
        if flags & 0x04:
            p += 8
        if flags & 0x10:
            p += 1
        nlen_size = 1 << (flags & 3)
        nlen = int.from_bytes(d[p:p + nlen_size], "little")
        p += nlen_size
        name = d[p:p + nlen].decode("utf-8")
        p += nlen
        if ltype != 0:
            return name, None  # soft / external links are not followed
        return name, struct.unpack_from("<Q", d, p)[0]

    # -- datatypes / dataspaces ----------------------------------------------------
    def _parse_datatype(self, d: bytes, p: int):
        cls = d[p] & 0x0F
        bits = d[p + 1] | (d[p + 2] << 8) | (d[p + 3] << 16)
        size = struct.unpack_from("<I", d, p + 4)[0]
        q = p + 8
        if cls == 0:  # fixed point
            dt = Datatype(0, size, ">" if bits & 1 else "<", signed=bool(bits & 8))
            q += 4
        elif cls == 1:  # floating point
            dt = Datatype(1, size, ">" if bits & 1 else "<")
            q += 12
        elif cls == 3:  # fixed-length string
            dt = Datatype(3, size)
        elif cls == 9:  # variable length
            base, q = self._parse_datatype(d, q)
            dt = Datatype(9, size, vlen_str=(bits & 0x0F) == 1, base=base)
        else:
            raise Hdf5Error(f"datatype class {cls} not supported")
        return dt, q

    def _parse_dataspace(self, d: bytes):
        ver, rank, flags = d[0], d[1], d[2]
        p = 8 if ver == 1 else 4
        dims = [struct.unpack_from("<Q", d, p + 8 * i)[0] for i in range(rank)]
        if ver == 2 and d[3] == 2:  # null dataspace
            return None
        return tuple(dims)

    def _global_heap_object(self, coll: int, idx: int) -> bytes:
        h = self._read(coll, 16)
        if h[:4] != b"GCOL":
            raise Hdf5Error("bad global heap collection")
        size = struct.unpack_from("<Q", h, 8)[0]
        p, end = coll + 16, coll + size
        while p + 16 <= end:
            oi, _rc = struct.unpack_from("<HH", self._read(p, 4), 0)
            osz = struct.unpack_from("<Q", self._read(p + 8, 8), 0)[0]
            if oi == idx:
                return self._read(p + 16, osz)
            if oi == 0:
                break
            p += 16 + ((osz + 7) & ~7)
        raise Hdf5Error("global heap object not found")

    def _decode_values(self, dt: Datatype, shape, raw: bytes):
        count = int(np.prod(shape)) if shape else 1
        if dt.cls in (0, 1):
            arr = np.frombuffer(raw[:count * dt.size], dtype=dt.numpy())
        elif dt.cls == 3:
            vals = [raw[i * dt.size:(i + 1) * dt.size].split(b"\0")[0] for i in range(count)]
            arr = np.array(vals, dtype=object)
        elif dt.cls == 9 and dt.vlen_str:
            vals = []
            for i in range(count):
                ln, coll, oi = struct.unpack_from("<IQI", raw, 16 * i)
                vals.append(self._global_heap_object(coll, oi)[:ln] if ln else b"")
            arr = np.array(vals, dtype=object)
        else:
            raise Hdf5Error("attribute datatype not supported")
        if not shape:
            return arr[0]
        return arr.reshape(shape)

    def _parse_attribute(self, d: bytes):
        ver = d[0]
        if ver == 1:
            nsz, tsz, ssz = struct.unpack_from("<HHH", d, 2)
            p = 8
            pad = lambda n: (n + 7) & ~7  # noqa: E731
            name = d[p:p + nsz].split(b"\0")[0].decode("utf-8")
            p += pad(nsz)
            dt = self._parse_datatype(d, p)[0]
            p += pad(tsz)
            shape = self._parse_dataspace(d[p:p + ssz])
            p += pad(ssz)
        elif ver in (2, 3):
            nsz, tsz, ssz = struct.unpack_from("<HHH", d, 2)
            p = 8 + (1 if ver == 3 else 0)
            name = d[p:p + nsz].split(b"\0")[0].decode("utf-8")
            p += nsz
            dt = self._parse_datatype(d, p)[0]
            p += tsz
            shape = self._parse_dataspace(d[p:p + ssz])
            p += ssz
        else:
            raise Hdf5Error(f"attribute message version {ver} not supported")
        return name, self._decode_values(dt, shape, d[p:])


def open_file(path: str) -> H5File:
    return H5File(path)


def as_str(v) -> Optional[str]:
    if v is None:
        return None
    if isinstance(v, (bytes, bytearray)):
        return v.decode("utf-8")
    if isinstance(v, np.ndarray) and v.shape == ():
        return as_str(v.item())
    return str(v)
