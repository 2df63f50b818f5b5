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
        elif dt in (DataType.Float32, DataType.Float64):
            vals.append(float(c))
        else:
            vals.append(int(c))
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


class MemoryDataSource(DataSource):
    def __init__(self, schema: Schema, batches: Sequence[RecordBatch]):
        self._schema = schema
        self._batches = list(batches)
        self._pos = 0

    def schema(self) -> Schema:
        return self._schema

    def next(self) -> Optional[RecordBatch]:
        if self._pos >= len(self._batches):
            return None
        b = self._batches[self._pos]
        self._pos += 1
        return b
