"""Aggregate relation (DFMI_FLAG_EXT_AGGREGATE): LogicalPlan::Aggregate with
no GROUP BY over an optional Selection (sqlplanner.rs:91-117). The reference
plans it and compiles its AggregateFunctions (compile_expr,
expression.rs:81-116) but its executor stops at context.rs:161
(`unimplemented!()`); here every input batch is one fused predicate +
aggregate pass on the GPU and next() returns the single result row."""
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


def agg_value_py(v):
    """The aggregate value as a Python scalar (None for null)."""
    if v.is_null:
        return None
    return agg_value_array(v).numpy_values()[0].item()


class AggregateRelation(Relation):
    """Aggregate(input, group_expr=[], aggr_expr) with the input's Selection
    (if any) fused: pulls every batch of `input`, then yields one batch."""

    def __init__(self, input: Relation, predicate, aggs: List, schema: Schema, device=None, flags: int = 0):
        self.input = input
        self.predicate = predicate
        self.aggs = aggs
        self._schema = schema
        self.device = device
        self.flags = flags
        self.done = False

    def next(self) -> Optional[RecordBatch]:
        if self.done:
            return None
        self.done = True
        state = engine(self.device).agg_state(self.aggs)
        while True:
            b = self.input.next()
            if b is None:
                break
            state.add(self.predicate, b, self.flags)
        return RecordBatch(self._schema, [agg_value_array(v) for v in state.finish()])

    def schema(self) -> Schema:
        return self._schema
