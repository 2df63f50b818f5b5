"""Aggregate relation (DFMI_FLAG_EXT_AGGREGATE): LogicalPlan::Aggregate over
an optional Selection (sqlplanner.rs:91-117), without or with one GROUP BY
key. The reference plans it and compiles its AggregateFunctions (compile_expr,
expression.rs:81-116) but its executor stops at context.rs:161
(`unimplemented!()`); here every input batch is one fused predicate +
aggregate pass on the GPU and next() returns the result: one row, or one row
per group in key order (null key last)."""
from __future__ import annotations

from typing import List, Optional

import numpy as np

from ..arrow import Array, RecordBatch, Schema
from ..logicalplan import DataType
from .engine import engine
from .relation import Relation

_NP = {
    DataType.Int8: np.int8, DataType.Int16: np.int16, DataType.Int32: np.int32, DataType.Int64: np.int64,
    DataType.UInt8: np.uint8, DataType.UInt16: np.uint16, DataType.UInt32: np.uint32, DataType.UInt64: np.uint64,
    DataType.Float32: np.float32, DataType.Float64: np.float64,
}


def agg_value_array(v) -> Array:
    """A one-row Array holding an aggregate value (dfmi_agg_value)."""
    t = DataType(v.type)
    dt = np.dtype(_NP[t])
    raw = np.array([v.bits], dtype=np.uint64).view(np.uint8)[: dt.itemsize].copy()
    vals = raw.view(dt)
    return Array.from_numpy(t, vals, np.array([not v.is_null]) if v.is_null else None)


def agg_values_array(vals) -> Array:
    """An Array of several aggregate / group-key values (dfmi_agg_value), one row each."""
    if not vals:
        return Array.from_pylist(DataType.Boolean, [])
    t = DataType(vals[0].type)
    valid = np.array([not v.is_null for v in vals])
    if t == DataType.Boolean:
        return Array.from_numpy(t, np.array([bool(v.bits) for v in vals]), None if valid.all() else valid)
    dt = np.dtype(_NP[t])
    raw = np.array([v.bits for v in vals], dtype=np.uint64).view(np.uint8).reshape(-1, 8)[:, : dt.itemsize].copy()
    return Array.from_numpy(t, raw.reshape(-1).view(dt), None if valid.all() else valid)


def agg_value_py(v):
    """The aggregate value as a Python scalar (None for null)."""
    if v.is_null:
        return None
    return agg_value_array(v).numpy_values()[0].item()


class AggregateRelation(Relation):
    """Aggregate(input, group_expr, aggr_expr) with the input's Selection (if
    any) fused: pulls every batch of `input`, then yields one batch -- the
    group key columns (if any, in group_expr order) followed by the
    aggregates, one row per group in key order."""

    def __init__(self, input: Relation, predicate, aggs: List, schema: Schema, device=None, flags: int = 0,
                 key=None):
        self.input = input
        self.predicate = predicate
        self.aggs = aggs
        # one RuntimeExpr (the single-key form) or a list of them
        self.keys = None if key is None else (list(key) if isinstance(key, (list, tuple)) else [key])
        self._schema = schema
        self.device = device
        self.flags = flags
        self.done = False

    def next(self) -> Optional[RecordBatch]:
        if self.done:
            return None
        self.done = True
        eng = engine(self.device)
        state = eng.agg_state(self.aggs) if self.keys is None else eng.grouped_agg_state(self.keys, self.aggs)
        while True:
            b = self.input.next()
            if b is None:
                break
            state.add(self.predicate, b, self.flags)
        if self.keys is None:
            return RecordBatch(self._schema, [agg_value_array(v) for v in state.finish()])
        keys, vals = state.finish()
        if len(keys) == 0:
            return None
        nk = len(self.keys)
        per_part = [[g[p] for g in keys] for p in range(nk)]  # (the state is created with the key list)
        cols = []
        for p, kv in enumerate(per_part):
            if DataType(kv[0].type) == DataType.Utf8:
                cols.append(Array.from_strings(state.key_strings(p)))
            else:
                cols.append(agg_values_array(kv))
        cols += [agg_values_array([g[j] for g in vals]) for j in range(len(self.aggs))]
        return RecordBatch(self._schema, cols)

    def schema(self) -> Schema:
        return self._schema
