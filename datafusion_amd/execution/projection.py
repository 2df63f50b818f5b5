"""ProjectRelation (src/execution/projection.rs:29-71) on the MI355X path.

When the input is a FilterRelation the Selection and the Projection run as
one fused device pass (no materialised filtered batch); otherwise the
projection runs alone. Per-batch output schema = Field(get_name, get_type,
nullable=true) (projection.rs:52-57).
"""
from __future__ import annotations

from typing import List, Optional

from ..arrow import Field, RecordBatch, Schema
from .engine import engine
from .expression import RuntimeExpr
from .filter import FilterRelation
from .relation import Relation


class ProjectRelation(Relation):
    def __init__(self, input: Relation, expr: List[RuntimeExpr], schema: Schema, device=None,
                 flags: int = None):
        self.input = input
        self.expr = list(expr)
        self._schema = schema
        self.device = device
        if flags is None:
            flags = 0
            for e in self.expr:
                flags |= e.flags
            if isinstance(input, FilterRelation):
                flags |= input.flags
        self.flags = flags

    def next(self) -> Optional[RecordBatch]:
        if isinstance(self.input, FilterRelation):
            batch = self.input.input.next()
            pred = self.input.expr
        else:
            batch = self.input.next()
            pred = None
        if batch is None:
            return None
        eng = engine(self.device)
        if all(c.values.device.type == "cpu" for c in batch.columns):
            # a host batch (e.g. a CSV source's pinned buffers): the pipelined
            # host entry point, host results -- what a Rust caller gets
            cols = eng.filter_project_host(pred, self.expr, batch, self.flags)
        else:
            cols = eng.filter_project(pred, self.expr, batch, self.flags)
        schema = Schema([Field(e.get_name(), e.get_type(), True) for e in self.expr])
        return RecordBatch(schema, cols)

    def schema(self) -> Schema:
        return self._schema
