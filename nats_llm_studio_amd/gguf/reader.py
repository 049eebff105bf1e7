"""GGUF v3 reader: metadata + tensor directory + zero-copy memory-mapped data.

Replaces the model-introspection half of LM Studio's `/api/v0/models` that the
reference calls at `/root/reference/nats_llm_studio.go:61-85` / `:136-156`:
architecture, quantisation and context length come straight from the file.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import numpy as np

from .constants import (GGML_BLOCK, GGMLType, GGUF_DEFAULT_ALIGNMENT, GGUF_MAGIC,
                        GGUFValueType, FILE_TYPE_NAMES, tensor_nbytes)

_SCALAR = {
    GGUFValueType.UINT8: "<B", GGUFValueType.INT8: "<b", GGUFValueType.UINT16: "<H",
    GGUFValueType.INT16: "<h", GGUFValueType.UINT32: "<I", GGUFValueType.INT32: "<i",
    GGUFValueType.FLOAT32: "<f", GGUFValueType.BOOL: "<?", GGUFValueType.UINT64: "<Q",
    GGUFValueType.INT64: "<q", GGUFValueType.FLOAT64: "<d",
}
_NP = {
    GGUFValueType.UINT8: np.uint8, GGUFValueType.INT8: np.int8, GGUFValueType.UINT16: np.uint16,
    GGUFValueType.INT16: np.int16, GGUFValueType.UINT32: np.uint32, GGUFValueType.INT32: np.int32,
    GGUFValueType.FLOAT32: np.float32, GGUFValueType.BOOL: np.bool_, GGUFValueType.UINT64: np.uint64,
    GGUFValueType.INT64: np.int64, GGUFValueType.FLOAT64: np.float64,
}


@dataclass
class TensorInfo:
    name: str
    shape: tuple            # ggml order: ne[0] (innermost) first
    ggml_type: int
    offset: int             # relative to data section
    nbytes: int
    data: Optional[np.ndarray] = field(default=None, repr=False)   # uint8 view

    @property
    def np_shape(self) -> tuple:
        """Row-major numpy shape (outermost first)."""
        return tuple(reversed(self.shape))

    @property
    def n_elements(self) -> int:
        n = 1
        for s in self.shape:
            n *= int(s)
        return n

    @property
    def type_name(self) -> str:
        return GGMLType(self.ggml_type).name


class _Cursor:
    def __init__(self, buf):
        self.buf = buf
        self.pos = 0

    def read(self, fmt: str):
        v = struct.unpack_from(fmt, self.buf, self.pos)[0]
        self.pos += struct.calcsize(fmt)
        return v

    def string(self) -> str:
        n = self.read("<Q")
        s = bytes(self.buf[self.pos:self.pos + n]).decode("utf-8", errors="replace")
        self.pos += n
        return s

    def value(self, vt: int) -> Any:
        vt = GGUFValueType(vt)
        if vt == GGUFValueType.STRING:
            return self.string()
        if vt == GGUFValueType.ARRAY:
            et = GGUFValueType(self.read("<I"))
            n = self.read("<Q")
            if et == GGUFValueType.STRING:
                return [self.string() for _ in range(n)]
            if et == GGUFValueType.ARRAY:
                return [self.value(et) for _ in range(n)]
            dt = np.dtype(_NP[et])
            arr = np.frombuffer(self.buf, dtype=dt, count=n, offset=self.pos).copy()
            self.pos += n * dt.itemsize
            return arr
        return self.read(_SCALAR[vt])


class GGUFReader:
    """Parse a GGUF file. Tensor payloads are numpy views into one read-only mmap,
    so opening a multi-GB checkpoint costs only the header parse."""

    def __init__(self, path: str, mmap: bool = True):
        self.path = path
        if mmap:
            self._mm = np.memmap(path, dtype=np.uint8, mode="r")
        else:
            self._mm = np.fromfile(path, dtype=np.uint8)
        buf = memoryview(self._mm)
        cur = _Cursor(buf)
        if bytes(buf[0:4]) != GGUF_MAGIC:
            raise ValueError(f"{path}: not a GGUF file")
        cur.pos = 4
        self.version = cur.read("<I")
        if self.version not in (2, 3):
            raise ValueError(f"{path}: unsupported GGUF version {self.version}")
        n_tensors = cur.read("<Q")
        n_kv = cur.read("<Q")
        self.metadata: Dict[str, Any] = {}
        for _ in range(n_kv):
            key = cur.string()
            vt = cur.read("<I")
            self.metadata[key] = cur.value(vt)
        self.tensors: Dict[str, TensorInfo] = {}
        order: List[TensorInfo] = []
        for _ in range(n_tensors):
            name = cur.string()
            nd = cur.read("<I")
            shape = tuple(cur.read("<Q") for _ in range(nd))
            gt = cur.read("<I")
            off = cur.read("<Q")
            n = 1
            for s in shape:
                n *= s
            ti = TensorInfo(name, shape, gt, off, tensor_nbytes(gt, n))
            self.tensors[name] = ti
            order.append(ti)
        align = int(self.metadata.get("general.alignment", GGUF_DEFAULT_ALIGNMENT))
        self.alignment = align
        self.data_offset = (cur.pos + align - 1) // align * align
        for ti in order:
            start = self.data_offset + ti.offset
            ti.data = self._mm[start:start + ti.nbytes]
        self.tensor_order = [t.name for t in order]

    # -- convenience -------------------------------------------------------
    def get(self, key: str, default: Any = None) -> Any:
        return self.metadata.get(key, default)

    @property
    def architecture(self) -> str:
        return str(self.metadata.get("general.architecture", "unknown"))

    def arch_get(self, key: str, default: Any = None) -> Any:
        return self.metadata.get(f"{self.architecture}.{key}", default)

    @property
    def file_type_name(self) -> str:
        ft = self.metadata.get("general.file_type")
        if ft is None:
            return "unknown"
        return FILE_TYPE_NAMES.get(int(ft), f"ftype{int(ft)}")

    def tensor(self, name: str) -> TensorInfo:
        return self.tensors[name]

    def dequantized(self, name: str) -> np.ndarray:
        from .quants import dequantize
        ti = self.tensors[name]
        return dequantize(ti.data, ti.ggml_type, ti.np_shape)

    def close(self):
        self._mm = None
        for t in self.tensors.values():
            t.data = None


def read_metadata(path: str) -> Dict[str, Any]:
    """Header-only parse (used by the registry scan; avoids touching tensor pages)."""
    r = GGUFReader(path, mmap=True)
    md = dict(r.metadata)
    md["__n_tensors__"] = len(r.tensors)
    md["__file_type_name__"] = r.file_type_name
    r.close()
    return md
