"""Decode the reference's `*_scaler_{x,y}.bin` StandardScaler files WITHOUT
unpickling.

The reference saves its scalers with joblib.dump(scaler, path, compress=True)
(kinematics/ann.py:94-95) and loads them with joblib.load (ann.py:83-84).  The
file is a zlib stream holding a protocol-4 pickle of sklearn's StandardScaler
whose ndarray attributes are joblib NumpyArrayWrapper records, each followed by
the array's raw bytes outside the pickle opcodes.

This module walks the pickle opcodes with an inert interpreter: GLOBAL /
REDUCE / NEWOBJ / BUILD produce plain tuples describing what the pickle asks
for -- nothing named in the file is imported or called.  Only the attributes
needed for transform / inverse_transform are returned.
"""
from __future__ import annotations

import struct
import zlib
from dataclasses import dataclass

import numpy as np


@dataclass
class ScalerParams:
    mean: np.ndarray        # mean_ (float64)
    scale: np.ndarray       # scale_ (float64)
    var: np.ndarray | None  # var_
    with_mean: bool = True
    with_std: bool = True
    n_samples_seen: int | None = None
    sklearn_version: str | None = None

    def transform(self, X):
        """StandardScaler.transform in float64: (X - mean) / scale."""
        X = np.array(X, dtype=np.float64, copy=True)
        if self.with_mean:
            X -= self.mean
        if self.with_std:
            X /= self.scale
        return X

    def effective(self):
        """(mean, scale) as the fused kernels apply them, (x - mean) / scale and
        y * scale + mean: 0 / 1 where with_mean / with_std are off (sklearn
        then skips the step; a fitted mean_ may still be set), which is exact."""
        mean = np.asarray(self.mean, np.float64) if self.with_mean else np.zeros_like(
            np.asarray(self.mean, np.float64))
        scale = np.asarray(self.scale, np.float64) if self.with_std else np.ones_like(
            np.asarray(self.scale, np.float64))
        return mean, scale

    def inverse_transform(self, X):
        """StandardScaler.inverse_transform keeping a float32 input float32
        (numpy in-place ops with a float64 operand, rounded per op)."""
        X = np.array(X, copy=True)
        if self.with_std:
            X *= self.scale
        if self.with_mean:
            X += self.mean
        return X


class _Obj:
    """An object the pickle would construct: callable + args + state."""

    def __init__(self, func, args):
        self.func = func
        self.args = args
        self.state = None

    def __repr__(self):
        return f"_Obj({self.func!r}, {self.args!r}, state={self.state!r})"


class _Mark:
    pass


_MARK = _Mark()


def _decompress(raw: bytes) -> bytes:
    if raw[:2] in (b"x\x9c", b"x^", b"x\xda", b"x\x01"):
        return zlib.decompress(raw)
    if raw[:1] == b"\x80":  # uncompressed joblib pickle
        return raw
    raise ValueError("unsupported joblib container (only zlib / raw pickles)")


def _dtype_of(obj) -> np.dtype:
    # numpy.dtype('f8', False, True) followed by BUILD state (3, '<', ...)
    if isinstance(obj, _Obj) and obj.func == ("global", "numpy", "dtype"):
        code = obj.args[0]
        order = "<"
        if isinstance(obj.state, tuple) and len(obj.state) > 1 and obj.state[1] in "<>|=":
            order = obj.state[1]
        dt = np.dtype(code)
        return dt.newbyteorder(order) if order in "<>" else dt
    raise ValueError(f"unexpected dtype record {obj!r}")


def _scalar_value(obj):
    # numpy.core.multiarray.scalar(dtype, bytes)
    if isinstance(obj, _Obj) and obj.func[2] == "scalar":
        dt = _dtype_of(obj.args[0])
        return np.frombuffer(obj.args[1], dtype=dt)[0].item()
    return obj


def parse_joblib_pickle(data: bytes):
    """Inert walk of a joblib pickle; returns the top-level object as _Obj/dict tree."""
    stack: list = []
    memo: dict = {}
    pos = 0
    n = len(data)

    def u8():
        nonlocal pos
        v = data[pos]
        pos += 1
        return v

    def take(k):
        nonlocal pos
        v = data[pos:pos + k]
        if len(v) != k:
            raise ValueError("truncated pickle")
        pos += k
        return v

    def pop_mark():
        items = []
        while True:
            v = stack.pop()
            if v is _MARK:
                break
            items.append(v)
        items.reverse()
        return items

    while pos < n:
        op = chr(u8())
        if op == "\x80":  # PROTO
            u8()
        elif op == "\x95":  # FRAME
            take(8)
        elif op == "\x8c":  # SHORT_BINUNICODE
            stack.append(take(u8()).decode("utf-8"))
        elif op == "X":  # BINUNICODE
            stack.append(take(struct.unpack("<I", take(4))[0]).decode("utf-8"))
        elif op == "C":  # SHORT_BINBYTES
            stack.append(bytes(take(u8())))
        elif op == "B":  # BINBYTES
            stack.append(bytes(take(struct.unpack("<I", take(4))[0])))
        elif op == "\x94":  # MEMOIZE
            memo[len(memo)] = stack[-1]
        elif op == "q":  # BINPUT
            memo[u8()] = stack[-1]
        elif op == "r":  # LONG_BINPUT
            memo[struct.unpack("<I", take(4))[0]] = stack[-1]
        elif op == "h":  # BINGET
            stack.append(memo[u8()])
        elif op == "j":  # LONG_BINGET
            stack.append(memo[struct.unpack("<I", take(4))[0]])
        elif op == "\x93":  # STACK_GLOBAL
            name = stack.pop()
            mod = stack.pop()
            stack.append(("global", mod, name))
        elif op == "c":  # GLOBAL
            mod = b""
            while True:
                ch = take(1)
                if ch == b"\n":
                    break
                mod += ch
            name = b""
            while True:
                ch = take(1)
                if ch == b"\n":
                    break
                name += ch
            stack.append(("global", mod.decode(), name.decode()))
        elif op == ")":  # EMPTY_TUPLE
            stack.append(())
        elif op == "}":  # EMPTY_DICT
            stack.append({})
        elif op == "]":  # EMPTY_LIST
            stack.append([])
        elif op == "(":  # MARK
            stack.append(_MARK)
        elif op == "t":  # TUPLE
            stack.append(tuple(pop_mark()))
        elif op == "\x85":  # TUPLE1
            stack.append((stack.pop(),))
        elif op == "\x86":  # TUPLE2
            b = stack.pop(); a = stack.pop()
            stack.append((a, b))
        elif op == "\x87":  # TUPLE3
            c = stack.pop(); b = stack.pop(); a = stack.pop()
            stack.append((a, b, c))
        elif op == "\x88":  # NEWTRUE
            stack.append(True)
        elif op == "\x89":  # NEWFALSE
            stack.append(False)
        elif op == "N":  # NONE
            stack.append(None)
        elif op == "K":  # BININT1
            stack.append(u8())
        elif op == "M":  # BININT2
            stack.append(struct.unpack("<H", take(2))[0])
        elif op == "J":  # BININT
            stack.append(struct.unpack("<i", take(4))[0])
        elif op == "G":  # BINFLOAT
            stack.append(struct.unpack(">d", take(8))[0])
        elif op == "\x8a":  # LONG1
            k = u8()
            stack.append(int.from_bytes(take(k), "little", signed=True))
        elif op in ("\x81", "R"):  # NEWOBJ / REDUCE -> inert record
            args = stack.pop()
            func = stack.pop()
            stack.append(_Obj(func, args))
        elif op == "s":  # SETITEM
            v = stack.pop(); k = stack.pop()
            stack[-1][k] = v
        elif op == "u":  # SETITEMS
            items = pop_mark()
            d = stack[-1]
            for i in range(0, len(items), 2):
                d[items[i]] = items[i + 1]
        elif op == "a":  # APPEND
            v = stack.pop()
            stack[-1].append(v)
        elif op == "e":  # APPENDS
            items = pop_mark()
            stack[-1].extend(items)
        elif op == "b":  # BUILD
            state = stack.pop()
            obj = stack[-1]
            if isinstance(obj, _Obj):
                obj.state = state
                if obj.func == ("global", "joblib.numpy_pickle", "NumpyArrayWrapper"):
                    # the array bytes follow the BUILD opcode in the stream;
                    # joblib >= 1.2 aligns them: one byte of padding length,
                    # then that many pad bytes (numpy_array_alignment_bytes)
                    if state.get("numpy_array_alignment_bytes") is not None:
                        take(u8())
                    dt = _dtype_of(state["dtype"])
                    shape = tuple(state["shape"])
                    count = int(np.prod(shape)) if shape else 1
                    raw = take(count * dt.itemsize)
                    arr = np.frombuffer(raw, dtype=dt).reshape(shape,
                                                              order=state.get("order", "C"))
                    stack[-1] = arr.astype(dt.newbyteorder("="), copy=True)
        elif op == ".":  # STOP
            return stack.pop()
        else:
            raise ValueError(f"unsupported pickle opcode {op!r} at {pos - 1}")
    raise ValueError("pickle without STOP")


def load_scaler(path: str) -> ScalerParams:
    """Read a joblib-dumped sklearn StandardScaler without executing it."""
    with open(path, "rb") as f:
        data = _decompress(f.read())
    top = parse_joblib_pickle(data)
    if not (isinstance(top, _Obj) and isinstance(top.func, tuple)
            and top.func[2] == "StandardScaler" and isinstance(top.state, dict)):
        raise ValueError(f"{path}: not a StandardScaler pickle")
    st = top.state
    mean = st.get("mean_")
    scale = st.get("scale_")
    if mean is None or scale is None:
        raise ValueError(f"{path}: StandardScaler without mean_/scale_")
    nss = _scalar_value(st.get("n_samples_seen_"))
    return ScalerParams(mean=np.asarray(mean, np.float64), scale=np.asarray(scale, np.float64),
                        var=None if st.get("var_") is None else np.asarray(st["var_"]),
                        with_mean=bool(st.get("with_mean", True)),
                        with_std=bool(st.get("with_std", True)),
                        n_samples_seen=None if nss is None else int(nss),
                        sklearn_version=st.get("_sklearn_version"))


def save_scaler_npz(path: str, sc: ScalerParams):
    np.savez(path, mean=sc.mean, scale=sc.scale,
             var=sc.var if sc.var is not None else np.zeros(0),
             with_mean=np.bool_(sc.with_mean), with_std=np.bool_(sc.with_std))


def save_scaler(path: str, sc: ScalerParams):
    """Write a scaler as the reference does (ann.py:94-95: joblib.dump of a
    fitted sklearn StandardScaler, compress=True), so that the reference's
    load_model and load_scaler above both read it.  Needs joblib and
    scikit-learn (writing only: nothing is unpickled here)."""
    try:
        import joblib
        from sklearn.preprocessing import StandardScaler
    except ImportError as e:  # pragma: no cover - both ship in this image
        raise RuntimeError("saving a .bin scaler needs joblib and scikit-learn") from e
    s = StandardScaler(with_mean=bool(sc.with_mean), with_std=bool(sc.with_std))
    s.mean_ = np.asarray(sc.mean, np.float64).copy()
    s.scale_ = np.asarray(sc.scale, np.float64).copy()
    s.var_ = (np.asarray(sc.var, np.float64).copy() if sc.var is not None
              else s.scale_ ** 2)
    s.n_features_in_ = int(s.mean_.shape[0])
    s.n_samples_seen_ = np.int64(sc.n_samples_seen if sc.n_samples_seen is not None else 0)
    joblib.dump(s, path, compress=True)
    return path
