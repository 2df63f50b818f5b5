"""ProjectRelation (src/execution/projection.rs:29-71) on the MI355X path.

When the input is a FilterRelation the Selection and the Projection run as
one fused device pass (no materialised filtered batch); otherwise the
projection runs alone. Per-batch output schema = Field(get_name, get_type,
nullable=true) (projection.rs:52-57).
"""
from __future__ import annotations

from typing import List, Optional

from ..arrow import Field, LazyColumns, RecordBatch, Schema
from .engine import engine
from .expression import RuntimeExpr
from .filter import Coalescer, FilterRelation, is_host_batch
from .relation import Relation


class ProjectRelation(Relation):
    def __init__(self, input: Relation, expr: List[RuntimeExpr], schema: Schema, device=None,
                 flags: int = None, coalesce: int = 1):
        self.input = input
        self.expr = list(expr)
        self._schema = schema
        self.device = device
        self.coalesce = coalesce
        self._co = None
        self._batch_schema = None
        if flags is None:
            flags = 0
            for e in self.expr:
                flags |= e.flags
            if isinstance(input, FilterRelation):
                flags |= input.flags
        self.flags = flags

    def _source_and_predicate(self):
        if isinstance(self.input, FilterRelation):
            return self.input.input, self.input.expr
        return self.input, None

    def _wrap(self, cols) -> RecordBatch:
        if self._batch_schema is None:  # projection.rs:52-57, the same for every batch
            self._batch_schema = Schema([Field(e.get_name(), e.get_type(), True) for e in self.expr])
        if isinstance(cols, LazyColumns):
            return RecordBatch.lazy(self._batch_schema, cols)
        return RecordBatch(self._batch_schema, cols)

    def _output_schema(self) -> Schema:
        if self._batch_schema is None:  # projection.rs:52-57, the same for every batch
            self._batch_schema = Schema([Field(e.get_name(), e.get_type(), True) for e in self.expr])
        return self._batch_schema

    def _wrap_many(self, results) -> list:
        if results and isinstance(results[0], RecordBatch):  # already batches (HostResultBatch)
            return results
        sch, lazy = self._output_schema(), RecordBatch.lazy
        return [lazy(sch, c) if isinstance(c, LazyColumns) else RecordBatch(sch, c) for c in results]

    def run_batch(self, batch: RecordBatch):
        _, pred = self._source_and_predicate()
        eng = engine(self.device)
        if is_host_batch(batch):
            # a host batch (e.g. a CSV source's pinned buffers): the pipelined
            # host entry point, host results -- what a Rust caller gets
            return eng.filter_project_host(pred, self.expr, batch, self.flags)
        return eng.filter_project(pred, self.expr, batch, self.flags)

    def next(self) -> Optional[RecordBatch]:
        co = self._co
        if co is not None:
            return co.next()
        source, pred = self._source_and_predicate()
        if self.coalesce > 1:  # up to `coalesce` input batches per device launch
            if self._co is None:
                self._co = Coalescer(self.coalesce, source, self.run_batch,
                                     lambda bs: engine(self.device).filter_project_batches(pred, self.expr, bs,
                                                                                           self.flags),
                                     self._wrap,
                                     lambda bs: engine(self.device).filter_project_host_batches(pred, self.expr, bs,
                                                                                                self.flags),
                                     run_many_host_async=lambda bs: engine(self.device).filter_project_host_batches_async(
                                         pred, self.expr, bs, self.flags, schema=self._output_schema(), start=False),
                                     wrap_many=self._wrap_many)
            # later pulls go straight to the Coalescer (one Python frame less
            # per batch at the reference's 1024-row batch size)
            self.next = self._co.next
            return self._co.next()
        batch = source.next()
        if batch is None:
            return None
        return self._wrap(self.run_batch(batch))

    def schema(self) -> Schema:
        return self._schema
