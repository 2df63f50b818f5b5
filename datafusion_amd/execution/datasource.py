"""Data sources (src/execution/datasource.rs:26-50).

CSV parsing stays on the host (north star); ``CsvDataSource`` restates the
arrow 0.12 csv::Reader behaviour the reference relies on (csv_sql.rs:49):
header skipping, fixed batch size, empty numeric field -> null.
``MemoryDataSource`` serves prepared (host or device) batches.
"""
from __future__ import annotations

import csv
from typing import List, Optional, Sequence

import numpy as np

from ..arrow import Array, RecordBatch, Schema
from ..logicalplan import DataType
from .error import ExecutionError


class DataSource:
    def schema(self) -> Schema:
        raise NotImplementedError

    def next(self) -> Optional[RecordBatch]:
        raise NotImplementedError


def _parse_bool(s: str) -> bool:
    if s.lower() == "true":
        return True
    if s.lower() == "false":
        return False
    raise ExecutionError("ArrowError(ParseError)", "Error while parsing value %s" % s)


def _parse_number(dt: DataType, s: str):
    try:
        if dt in (DataType.Float32, DataType.Float64):
            return float(s)
        v = int(s, 10)
    except ValueError:
        raise ExecutionError("ArrowError(ParseError)", "Error while parsing value %s" % s)
    from ..arrow import np_dtype
    info = np.iinfo(np_dtype(dt))
    if not info.min <= v <= info.max:
        raise ExecutionError("ArrowError(ParseError)", "Error while parsing value %s" % s)
    return v


def _parse_column(dt: DataType, cells: List[Optional[str]]) -> Array:
    if dt == DataType.Utf8:
        return Array.from_strings([("" if c is None else c).encode("utf-8") for c in cells])
    vals, valid = [], []
    for c in cells:
        if c is None or c == "":
            vals.append(0)
            valid.append(False)
            continue
        valid.append(True)
        if dt == DataType.Boolean:
            vals.append(_parse_bool(c))
        else:
            vals.append(_parse_number(dt, c))
    valid = np.array(valid, dtype=bool)
    if dt == DataType.Boolean:
        return Array.from_numpy(dt, np.array(vals, dtype=bool), None if valid.all() else valid)
    from ..arrow import np_dtype
    return Array.from_numpy(dt, np.array(vals, dtype=np_dtype(dt)), None if valid.all() else valid)


class CsvDataSource(DataSource):
    """CsvDataSource::new(schema, csv::Reader::new(file, schema, has_header, batch_size, None))."""

    def __init__(self, schema: Schema, path: str, has_header: bool = True, batch_size: int = 1024):
        self._schema = schema
        with open(path, newline="", encoding="utf-8") as f:
            rows = [r for r in csv.reader(f) if r]
        if has_header and rows:
            rows = rows[1:]
        self._rows = rows
        self._pos = 0
        self._batch = batch_size

    def schema(self) -> Schema:
        return self._schema

    def next(self) -> Optional[RecordBatch]:
        if self._pos >= len(self._rows):
            return None
        chunk = self._rows[self._pos: self._pos + self._batch]
        self._pos += len(chunk)
        cols = []
        for i, f in enumerate(self._schema.fields):
            cols.append(_parse_column(f.data_type, [r[i] if i < len(r) else None for r in chunk]))
        return RecordBatch(self._schema, cols)


class NativeCsvDataSource(DataSource):
    """CsvDataSource over the native reader (dfmi_csv_open, include/dfmi_datasource.h):
    host threads parse straight into pinned Arrow buffers and the next batch
    is parsed while the caller works on this one. Same batches as
    CsvDataSource. By default each batch is copied out of the reader's pinned
    buffers, so it can be kept. ``copy=False`` hands out zero-copy views of
    those buffers instead: such a batch is valid only until the next
    ``next()`` (the reference's pull order: csv_sql.rs:60-62 consumes each
    batch before pulling the next); it holds a reference to this source, so
    its memory is never freed under it, but the next batch overwrites it."""

    def __init__(self, schema: Schema, path: str, has_header: bool = True, batch_size: int = 1024,
                 threads: int = 0, copy: bool = True):
        import ctypes as C
        from .. import _abi
        self._schema = schema
        self._copy = copy
        L = _abi.lib()
        fields = (_abi.dfmi_field * max(1, len(schema.fields)))()
        self._names = [f.name.encode() for f in schema.fields]
        for i, f in enumerate(schema.fields):
            fields[i].name = self._names[i]
            fields[i].type = int(f.data_type)
            fields[i].nullable = 1 if f.nullable else 0
        sch = _abi.dfmi_schema(len(schema.fields), 0, fields)
        err = _abi.dfmi_error()
        h = C.c_void_p()
        rc = L.dfmi_csv_open(path.encode(), C.byref(sch), 1 if has_header else 0, batch_size, threads, C.byref(h),
                             C.byref(err))
        if rc != _abi.DFMI_OK:
            raise ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
        self._h = h
        self._close = L.dfmi_csv_close

    def schema(self) -> Schema:
        return self._schema

    def num_records(self) -> int:
        from .. import _abi
        return int(_abi.lib().dfmi_csv_num_records(self._h))

    def next(self) -> Optional[RecordBatch]:
        import ctypes as C
        import torch
        from .. import _abi
        L = _abi.lib()
        b = _abi.dfmi_batch()
        has = C.c_int32()
        err = _abi.dfmi_error()
        rc = L.dfmi_csv_next(self._h, C.byref(b), C.byref(has), C.byref(err))
        if rc != _abi.DFMI_OK:
            raise ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
        if not has.value:
            return None
        n = b.num_rows

        def view(ptr, nbytes, dtype=np.uint8):
            if not nbytes:
                return torch.zeros(8, dtype=torch.uint8 if dtype == np.uint8 else torch.int32)
            a = np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint8)), shape=(nbytes,)).view(dtype)
            return torch.from_numpy(a.copy() if self._copy else a)
        cols = []
        for i, f in enumerate(self._schema.fields):
            c = b.columns[i]
            t = DataType(c.type)
            vb = view(c.validity, (n + 7) // 8) if (c.null_count and c.validity) else None
            if t == DataType.Utf8:
                offs = view(c.offsets, 4 * (n + 1), np.int32)
                nbytes = int(offs[n]) if n else 0
                cols.append(Array(t, n, view(c.values, nbytes), None, offs, 0))
            else:
                nb = (n + 7) // 8 if t == DataType.Boolean else n * t.width
                cols.append(Array(t, n, view(c.values, nb), vb, None, c.null_count))
        rb = RecordBatch(self._schema, cols)
        if not self._copy:
            rb._source = self  # the views' memory lives as long as the batch
            rb._transient = True  # ... but the next pull overwrites it (a Coalescer copies it first)
        return rb

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._close(h)
            self._h = None


class MemoryDataSource(DataSource):
    def __init__(self, schema: Schema, batches: Sequence[RecordBatch]):
        self._schema = schema
        self._batches = list(batches)
        self._pos = 0
        self._ends = None  # rows before each batch's end (next_many), built on first use

    def schema(self) -> Schema:
        return self._schema

    def next(self) -> Optional[RecordBatch]:
        if self._pos >= len(self._batches):
            return None
        b = self._batches[self._pos]
        self._pos += 1
        return b

    def next_many(self, m: int, max_rows: int) -> List[RecordBatch]:
        """What up to m next() calls return, stopping once max_rows rows are
        out (the batch that reaches max_rows is the last one)."""
        import bisect
        if self._ends is None:
            self._ends = np.cumsum([b.num_rows() for b in self._batches], dtype=np.int64).tolist()
        i = self._pos
        end = min(len(self._batches), i + m)
        if i < end:
            before = self._ends[i - 1] if i else 0
            end = min(end, bisect.bisect_left(self._ends, before + max_rows, i, end) + 1)
        self._pos = end
        return self._batches[i:end]
