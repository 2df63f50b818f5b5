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

    def schema(self) -> Schema:
        return self._schema
