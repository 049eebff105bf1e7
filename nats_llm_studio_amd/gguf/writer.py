"""GGUF v3 writer (streaming). Used to produce random-init checkpoints of the
north-star architectures on the GPU box, where there is no network to fetch
real ones (BASELINE.json: "random-init .gguf weights")."""
from __future__ import annotations

import struct
from typing import Any, Callable, List, Tuple

import numpy as np

from .constants import GGUF_DEFAULT_ALIGNMENT, GGUF_MAGIC, GGUF_VERSION, GGUFValueType, tensor_nbytes


def _pack_string(s: str) -> bytes:
    b = s.encode("utf-8")
    return struct.pack("<Q", len(b)) + b


def _infer_type(v: Any) -> GGUFValueType:
    if isinstance(v, bool):
        return GGUFValueType.BOOL
    if isinstance(v, int):
        return GGUFValueType.UINT32 if 0 <= v < 2 ** 32 else GGUFValueType.INT64
    if isinstance(v, float):
        return GGUFValueType.FLOAT32
    if isinstance(v, str):
        return GGUFValueType.STRING
    if isinstance(v, (list, tuple, np.ndarray)):
        return GGUFValueType.ARRAY
    raise TypeError(f"cannot infer GGUF type of {type(v)}")


_FMT = {
    GGUFValueType.UINT8: "<B", GGUFValueType.INT8: "<b", GGUFValueType.UINT16: "<H",
    GGUFValueType.INT16: "<h", GGUFValueType.UINT32: "<I", GGUFValueType.INT32: "<i",
    GGUFValueType.FLOAT32: "<f", GGUFValueType.BOOL: "<?", GGUFValueType.UINT64: "<Q",
    GGUFValueType.INT64: "<q", GGUFValueType.FLOAT64: "<d",
}
_NP2VT = {
    np.dtype(np.uint8): GGUFValueType.UINT8, np.dtype(np.int8): GGUFValueType.INT8,
    np.dtype(np.uint16): GGUFValueType.UINT16, np.dtype(np.int16): GGUFValueType.INT16,
    np.dtype(np.uint32): GGUFValueType.UINT32, np.dtype(np.int32): GGUFValueType.INT32,
    np.dtype(np.float32): GGUFValueType.FLOAT32, np.dtype(np.bool_): GGUFValueType.BOOL,
    np.dtype(np.uint64): GGUFValueType.UINT64, np.dtype(np.int64): GGUFValueType.INT64,
    np.dtype(np.float64): GGUFValueType.FLOAT64,
}


def _pack_value(v: Any, vt: GGUFValueType) -> bytes:
    if vt == GGUFValueType.STRING:
        return _pack_string(v)
    if vt == GGUFValueType.ARRAY:
        if isinstance(v, np.ndarray):
            et = _NP2VT[v.dtype]
            return struct.pack("<IQ", et, v.size) + np.ascontiguousarray(v).astype(v.dtype.newbyteorder("<")).tobytes()
        v = list(v)
        if not v:
            return struct.pack("<IQ", GGUFValueType.INT32, 0)
        et = _infer_type(v[0])
        if et in (GGUFValueType.UINT32,) and any(isinstance(x, int) and x < 0 for x in v):
            et = GGUFValueType.INT32
        if et == GGUFValueType.FLOAT32:
            return struct.pack("<IQ", et, len(v)) + np.asarray(v, np.float32).tobytes()
        if et in (GGUFValueType.UINT32, GGUFValueType.INT32):
            return struct.pack("<IQ", et, len(v)) + np.asarray(v, np.int64).astype(
                np.uint32 if et == GGUFValueType.UINT32 else np.int32).tobytes()
        return struct.pack("<IQ", et, len(v)) + b"".join(_pack_value(x, et) for x in v)
    return struct.pack(_FMT[vt], v)


class GGUFWriter:
    """Collect metadata + tensor descriptors, then stream the file.

    Tensor data may be given eagerly (uint8 array) or as a zero-arg producer so
    that multi-GB checkpoints are generated one tensor at a time.
    """

    def __init__(self, path: str, arch: str, alignment: int = GGUF_DEFAULT_ALIGNMENT):
        self.path = path
        self.alignment = alignment
        self.kv: List[Tuple[str, GGUFValueType, Any]] = []
        self.tensors: List[Tuple[str, tuple, int, int, Any]] = []
        self.add("general.architecture", arch)
        if alignment != GGUF_DEFAULT_ALIGNMENT:
            self.add("general.alignment", alignment, GGUFValueType.UINT32)

    def add(self, key: str, value: Any, vt: GGUFValueType = None):
        self.kv.append((key, vt if vt is not None else _infer_type(value), value))

    def add_tensor(self, name: str, np_shape: tuple, ggml_type: int, data: Any):
        """np_shape is row-major (outermost first); stored reversed (ggml ne order)."""
        n = 1
        for s in np_shape:
            n *= int(s)
        nbytes = tensor_nbytes(ggml_type, n)
        self.tensors.append((name, tuple(int(s) for s in reversed(np_shape)), int(ggml_type), nbytes, data))

    def write(self, progress: Callable[[str], None] = None):
        a = self.alignment
        with open(self.path, "wb") as f:
            f.write(GGUF_MAGIC + struct.pack("<IQQ", GGUF_VERSION, len(self.tensors), len(self.kv)))
            for key, vt, val in self.kv:
                f.write(_pack_string(key) + struct.pack("<I", vt) + _pack_value(val, vt))
            off = 0
            offsets = []
            for name, ne, gt, nbytes, _ in self.tensors:
                offsets.append(off)
                f.write(_pack_string(name) + struct.pack("<I", len(ne)))
                f.write(b"".join(struct.pack("<Q", d) for d in ne))
                f.write(struct.pack("<IQ", gt, off))
                off = (off + nbytes + a - 1) // a * a
            pos = f.tell()
            pad = (pos + a - 1) // a * a - pos
            f.write(b"\0" * pad)
            for (name, ne, gt, nbytes, data), o in zip(self.tensors, offsets):
                if callable(data):
                    data = data()
                buf = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
                if buf.size != nbytes:
                    raise ValueError(f"{name}: got {buf.size} bytes, expected {nbytes}")
                f.write(memoryview(buf))
                pad = (nbytes + a - 1) // a * a - nbytes
                if pad:
                    f.write(b"\0" * pad)
                if progress:
                    progress(name)
