"""Minimal Arrow 0.12 columnar containers (arrow::array / record_batch).

Buffers are torch uint8 tensors on the host ("cpu") or in HBM ("cuda:N"), laid
out exactly as Arrow 0.12 lays them out (and as include/dfmi.h expects):
  * fixed width: little-endian values, one slot per row (null slots keep bits);
  * Boolean: LSB-first bitmap;
  * Utf8 (arrow BinaryArray): int32 offsets[length+1] + bytes;
  * validity: LSB-first bitmap, None when the array has no nulls.
Every buffer is zero-padded to a multiple of 64 bytes (Arrow alignment), which
also satisfies the ABI's "8-byte padded bitmap" rule.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np
import torch

from .logicalplan import DataType

_NP = {
    DataType.Int8: np.int8, DataType.Int16: np.int16, DataType.Int32: np.int32, DataType.Int64: np.int64,
    DataType.UInt8: np.uint8, DataType.UInt16: np.uint16, DataType.UInt32: np.uint32,
    DataType.UInt64: np.uint64, DataType.Float32: np.float32, DataType.Float64: np.float64,
}


def np_dtype(t: DataType):
    return _NP[t]


def _pad64(n: int) -> int:
    return max(64, (n + 63) // 64 * 64)


def _bytes_tensor(raw: np.ndarray, device="cpu") -> torch.Tensor:
    """uint8 tensor padded to 64 bytes holding raw's bytes."""
    b = np.ascontiguousarray(raw).view(np.uint8).reshape(-1)
    t = torch.zeros(_pad64(b.size), dtype=torch.uint8)
    if b.size:
        t[: b.size] = torch.from_numpy(b.copy())
    return t.to(device) if device != "cpu" else t


def empty_bytes(nbytes: int, device) -> torch.Tensor:
    """Uninitialised device buffer (outputs are fully written by the kernels)."""
    return torch.empty(_pad64(nbytes), dtype=torch.uint8, device=device)


def pack_bits(mask: np.ndarray) -> np.ndarray:
    return np.packbits(np.asarray(mask, dtype=bool), bitorder="little")


def unpack_bits(buf: np.ndarray, n: int) -> np.ndarray:
    return np.unpackbits(np.asarray(buf, dtype=np.uint8), bitorder="little")[:n].astype(bool)


class Field:
    """arrow::datatypes::Field"""

    def __init__(self, name: str, data_type: DataType, nullable: bool = True):
        self.name = name
        # nested types (serde.StructType / ListType) appear only in serialized schemas
        self.data_type = DataType(data_type) if isinstance(data_type, int) else data_type
        self.nullable = nullable

    def __repr__(self):
        return "Field(%r, %r, %s)" % (self.name, self.data_type, self.nullable)

    def __eq__(self, o):
        return isinstance(o, Field) and (self.name, self.data_type, self.nullable) == (o.name, o.data_type, o.nullable)


class Schema:
    """arrow::datatypes::Schema"""

    def __init__(self, fields: Sequence[Field]):
        self.fields = list(fields)

    @staticmethod
    def empty() -> "Schema":
        return Schema([])

    def field(self, i: int) -> Field:
        return self.fields[i]

    def __len__(self):
        return len(self.fields)

    def __repr__(self):
        return ", ".join("%s: %r" % (f.name, f.data_type) for f in self.fields)

    def to_string(self) -> str:
        return repr(self)

    def __eq__(self, o):
        return isinstance(o, Schema) and self.fields == o.fields


class Array:
    """One Arrow array; buffers on the host or on a GPU."""

    def __init__(self, data_type: DataType, length: int, values: torch.Tensor,
                 validity: Optional[torch.Tensor] = None, offsets: Optional[torch.Tensor] = None,
                 null_count: int = 0, offset: int = 0):
        self.data_type = data_type if type(data_type) is DataType else DataType(data_type)
        self.length = int(length)
        self.values = values
        self.validity = validity if null_count else None
        self.offsets = offsets
        self.null_count = int(null_count)
        # arrow ArrayData::offset: logical row i is physical slot offset + i
        # (values, validity / Boolean bits, Utf8 offsets); dfmi_column.offset
        self.offset = int(offset)

    def slice(self, offset: int, length: int) -> "Array":
        """Zero-copy slice (arrow Array::slice): same buffers, a larger offset."""
        assert 0 <= offset and offset + length <= self.length
        m = self.valid_mask()[offset:offset + length]
        nulls = int(length - m.sum()) if self.validity is not None else 0
        return Array(self.data_type, length, self.values, self.validity if nulls else None, self.offsets, nulls,
                     self.offset + offset)

    def __len__(self):
        return self.length

    @property
    def device(self) -> torch.device:
        return self.values.device

    def to(self, device) -> "Array":
        mv = lambda t: None if t is None else t.to(device)
        return Array(self.data_type, self.length, mv(self.values), mv(self.validity), mv(self.offsets),
                     self.null_count, self.offset)

    def cpu(self) -> "Array":
        return self.to("cpu")

    def data_bytes(self) -> int:
        """Utf8: bytes referenced by the offsets."""
        off = self.offsets[self.offset: self.offset + self.length + 1].cpu().numpy()
        return int(off[-1] - off[0]) if self.length else 0

    # ---- host views -------------------------------------------------------
    def valid_mask(self) -> np.ndarray:
        if self.validity is None:
            return np.ones(self.length, dtype=bool)
        return unpack_bits(self.validity.cpu().numpy(), self.offset + self.length)[self.offset:]

    def numpy_values(self) -> np.ndarray:
        """Raw values (fixed width) / bools / list of bytes (Utf8)."""
        v = self.values.cpu().numpy()
        t, o = self.data_type, self.offset
        if t == DataType.Boolean:
            return unpack_bits(v, o + self.length)[o:]
        if t == DataType.Utf8:
            off = self.offsets.cpu().numpy()[o: o + self.length + 1]
            return [bytes(v[off[i]: off[i + 1]]) for i in range(self.length)]
        w = np.dtype(_NP[t]).itemsize
        return v[o * w: (o + self.length) * w].view(_NP[t])

    def to_pylist(self) -> list:
        vals = self.numpy_values()
        valid = self.valid_mask()
        out = []
        for i in range(self.length):
            if not valid[i]:
                out.append(None)
                continue
            x = vals[i]
            if self.data_type == DataType.Utf8:
                out.append(x.decode("utf-8", errors="surrogateescape"))
            elif self.data_type == DataType.Boolean:
                out.append(bool(x))
            elif self.data_type in (DataType.Float32, DataType.Float64):
                out.append(float(x))
            else:
                out.append(int(x))
        return out

    # ---- constructors -----------------------------------------------------
    @staticmethod
    def from_numpy(data_type: DataType, values, valid: Optional[np.ndarray] = None,
                   device="cpu") -> "Array":
        """Fixed-width / Boolean array from a numpy vector (+ optional validity mask)."""
        t = DataType(data_type)
        n = len(values)
        if t == DataType.Boolean:
            vbuf = _bytes_tensor(pack_bits(values), device)
        else:
            vbuf = _bytes_tensor(np.asarray(values, dtype=_NP[t]), device)
        nulls = 0
        vb = None
        if valid is not None:
            valid = np.asarray(valid, dtype=bool)
            nulls = int(n - valid.sum())
            if nulls:
                vb = _bytes_tensor(pack_bits(valid), device)
        return Array(t, n, vbuf, vb, None, nulls)

    @staticmethod
    def from_strings(strings: Sequence[Optional[bytes]], device="cpu") -> "Array":
        """Utf8 array; None entries become nulls with an empty slot."""
        n = len(strings)
        offs = np.zeros(n + 1, dtype=np.int32)
        parts = []
        valid = np.ones(n, dtype=bool)
        pos = 0
        for i, s in enumerate(strings):
            if s is None:
                valid[i] = False
                s = b""
            if isinstance(s, str):
                s = s.encode("utf-8")
            parts.append(s)
            pos += len(s)
            offs[i + 1] = pos
        data = np.frombuffer(b"".join(parts), dtype=np.uint8) if pos else np.zeros(0, np.uint8)
        nulls = int(n - valid.sum())
        vb = _bytes_tensor(pack_bits(valid), device) if nulls else None
        return Array(DataType.Utf8, n, _bytes_tensor(data, device), vb, _offsets_tensor(offs, device), nulls)

    @staticmethod
    def from_pylist(data_type: DataType, values: Sequence, device="cpu") -> "Array":
        t = DataType(data_type)
        valid = np.array([v is not None for v in values], dtype=bool)
        if t == DataType.Utf8:
            return Array.from_strings([None if v is None else (v.encode() if isinstance(v, str) else v)
                                       for v in values], device)
        fill = [(v if v is not None else 0) for v in values]
        if t == DataType.Boolean:
            fill = np.array([bool(v) for v in fill], dtype=bool)
        return Array.from_numpy(t, np.array(fill, dtype=None if t == DataType.Boolean else _NP[t]),
                                valid if not valid.all() else None, device)


class _BlockBuffer:
    """Non-data descriptor for one buffer of a BlockArray: the torch view of
    the block's byte range (dict keys `o` / `n`) is made on first read and
    stored in the instance dict, which from then on shadows this descriptor."""

    __slots__ = ("name", "o", "n", "dtype")

    def __init__(self, name: str, o: str, n: str, dtype=None):
        self.name, self.o, self.n, self.dtype = name, o, n, dtype

    def __get__(self, obj, cls=None):
        if obj is None:
            return self
        d = obj.__dict__
        o = d.get(self.o)
        t = None
        if o is not None:
            t = d["_blk"][o:o + d[self.n]]
            if self.dtype is not None:
                t = t.view(self.dtype)
        d[self.name] = t
        return t


class BlockArray(Array):
    """An Array whose buffers are byte ranges of one host block -- the output
    block of a coalesced host call (dfmi_filter_project_host_batches_into),
    shared by every array of the group, as arrow's Buffer::slice shares one
    Arc'd allocation. Built by the native glue (_dfmi_glue.make_block_batches)
    with the ranges recorded (`_blk`, `_vo`/`_vn`, `_bo`/`_bn`, `_oo`/`_on`);
    each torch view is made when first read, and the glue reads the pointers
    of views not made yet straight from the block."""

    values = _BlockBuffer("values", "_vo", "_vn")
    validity = _BlockBuffer("validity", "_bo", "_bn")
    offsets = _BlockBuffer("offsets", "_oo", "_on", torch.int32)
    offset = 0  # a block array starts at its own slot 0 (the glue sets no instance `offset`)


def _offsets_tensor(offs: np.ndarray, device) -> torch.Tensor:
    n = len(offs)
    t = torch.zeros(max(16, (n + 15) // 16 * 16), dtype=torch.int32)
    t[:n] = torch.from_numpy(offs.astype(np.int32))
    return t.to(device) if device != "cpu" else t


class LazyColumns:
    """Columns of a batch whose buffers already exist (e.g. slices of one
    pinned result block) but whose Array objects are built on first access:
    a pull loop that only forwards batches pays for no Python objects it does
    not read. Subclasses give num_rows, num_columns and materialize()."""

    num_rows = 0
    num_columns = 0

    def materialize(self) -> List[Array]:
        raise NotImplementedError

    # also a read-only sequence of its Arrays
    def __len__(self):
        return self.num_columns

    def __getitem__(self, i):
        return self.materialize()[i]

    def __iter__(self):
        return iter(self.materialize())


class RecordBatch:
    """arrow::record_batch::RecordBatch"""

    _transient = False  # a source's zero-copy view, valid until its next pull (datasource.py)

    def __init__(self, schema: Schema, columns):
        self.schema = schema
        self._columns = columns if isinstance(columns, LazyColumns) else list(columns)

    @classmethod
    def lazy(cls, schema: Schema, columns: LazyColumns) -> "RecordBatch":
        """A batch over LazyColumns, built without __init__'s checks (one
        per output batch of a coalesced call)."""
        b = object.__new__(cls)
        b.schema = schema
        b._columns = columns
        return b

    @property
    def columns(self) -> List[Array]:
        c = self._columns
        if type(c) is not list:
            c = self._columns = c.materialize()
        return c

    @columns.setter
    def columns(self, cols) -> None:
        self._columns = list(cols)

    def num_columns(self) -> int:
        c = self._columns
        return len(c) if type(c) is list else c.num_columns

    def num_rows(self) -> int:
        c = self._columns
        if type(c) is not list:
            return c.num_rows
        return c[0].length if c else 0

    def column(self, i: int) -> Array:
        return self.columns[i]

    def to(self, device) -> "RecordBatch":
        return RecordBatch(self.schema, [c.to(device) for c in self.columns])
