"""FilterRelation (src/execution/filter.rs:30-111) on the MI355X path."""
from __future__ import annotations

from typing import Callable, List, Optional

from ..arrow import RecordBatch, Schema
from .engine import engine
from .expression import RuntimeExpr
from .relation import Relation


class Coalescer:
    """Pulls up to `m` device batches from `source` and runs them as ONE
    launch (dfmi_filter_project_batches), then hands the results out one
    batch per next() -- the same output stream as one pull per batch
    (relation.rs:27-32): one output batch per input batch, in order; on an
    error the batches before the failing one come first, then the error, and
    the batches pulled after it are run one at a time if the caller goes on."""

    def __init__(self, m: int, source: Relation, run_one: Callable, run_many: Callable, wrap: Callable):
        self.m, self.source = m, source
        self.run_one, self.run_many, self.wrap = run_one, run_many, wrap
        self.ready: List = []      # RecordBatches / an exception, in stream order
        self.pending: List = []    # pulled input batches still to run one by one

    def next(self) -> Optional[RecordBatch]:
        while not self.ready:
            if self.pending:
                self.ready.append(self.wrap(self.run_one(self.pending.pop(0))))
                break
            pulled = []
            while len(pulled) < self.m:
                b = self.source.next()
                if b is None:
                    break
                pulled.append(b)
            if not pulled:
                return None
            if any(all(c.values.device.type == "cpu" for c in b.columns) for b in pulled):
                self.pending = pulled  # host batches: the host entry point, one pull each
                continue
            results, err = self.run_many(pulled)
            self.ready = [self.wrap(cols) for cols in results]
            if err is not None:
                self.ready.append(err)
                self.pending = pulled[len(results) + 1:]
        item = self.ready.pop(0)
        if isinstance(item, Exception):
            raise item
        return item


class FilterRelation(Relation):
    """FilterRelation::new(input, expr, schema). next() pulls one batch from
    the input and returns every column filtered by the predicate, in a batch
    whose schema is Schema::empty() (filter.rs:60-61). With coalesce > 1, up
    to that many input batches run as one device launch (Coalescer)."""

    def __init__(self, input: Relation, expr: RuntimeExpr, schema: Schema, device=None, flags: int = None,
                 coalesce: int = 1):
        self.input = input
        self.expr = expr
        self._schema = schema
        self.device = device
        self.flags = expr.flags if flags is None else flags
        self.coalesce = coalesce
        self._co = None

    def run_batch(self, batch: RecordBatch):
        eng = engine(self.device)
        if all(c.values.device.type == "cpu" for c in batch.columns):
            return eng.filter_project_host(self.expr, None, batch, self.flags)
        return eng.filter_project(self.expr, None, batch, self.flags)

    def next(self) -> Optional[RecordBatch]:
        if self.coalesce > 1:
            if self._co is None:
                self._co = Coalescer(self.coalesce, self.input, self.run_batch,
                                     lambda bs: engine(self.device).filter_project_batches(self.expr, None, bs,
                                                                                           self.flags),
                                     lambda cols: RecordBatch(Schema.empty(), cols))
            return self._co.next()
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
