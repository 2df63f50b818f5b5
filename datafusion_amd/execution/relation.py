"""Pull-iterator relations (src/execution/relation.rs:27-54)."""
from __future__ import annotations

from typing import Optional

from ..arrow import RecordBatch, Schema


class Relation:
    """trait Relation { fn next(&mut self) -> Result<Option<RecordBatch>>; fn schema(&self) -> &Arc<Schema>; }"""

    def next(self) -> Optional[RecordBatch]:
        raise NotImplementedError

    def schema(self) -> Schema:
        raise NotImplementedError

    def __iter__(self):
        while True:
            b = self.next()
            if b is None:
                return
            yield b


class DataSourceRelation(Relation):
    """relation.rs:34-54"""

    def __init__(self, ds):
        self.ds = ds
        self._schema = ds.schema()

    def next(self) -> Optional[RecordBatch]:
        return self.ds.next()

    @property
    def next_many(self):
        """The source's next_many(m, max_rows), when it has one: up to m
        batches (fewer once max_rows rows are out) in one call -- what m next()
        calls would return, for a Coalescer's read-ahead."""
        nm = getattr(self.ds, "next_many", None)
        if nm is None:
            raise AttributeError("next_many")
        return nm

    def schema(self) -> Schema:
        return self._schema
