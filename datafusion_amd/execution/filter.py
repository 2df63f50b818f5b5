"""FilterRelation (src/execution/filter.rs:30-111) on the MI355X path."""
from __future__ import annotations

from typing import Optional

from ..arrow import RecordBatch, Schema
from .engine import engine
from .expression import RuntimeExpr
from .relation import Relation


class FilterRelation(Relation):
    """FilterRelation::new(input, expr, schema). next() pulls one batch from
    the input and returns every column filtered by the predicate, in a batch
    whose schema is Schema::empty() (filter.rs:60-61)."""

    def __init__(self, input: Relation, expr: RuntimeExpr, schema: Schema, device=None, flags: int = None):
        self.input = input
        self.expr = expr
        self._schema = schema
        self.device = device
        self.flags = expr.flags if flags is None else flags

    def next(self) -> Optional[RecordBatch]:
        batch = self.input.next()
        if batch is None:
            return None
        eng = engine(self.device)
        if all(c.values.device.type == "cpu" for c in batch.columns):
            cols = eng.filter_project_host(self.expr, None, batch, self.flags)  # host batch: host results
        else:
            cols = eng.filter_project(self.expr, None, batch, self.flags)
        return RecordBatch(Schema.empty(), cols)

    def schema(self) -> Schema:
        return self._schema
