"""FilterRelation (src/execution/filter.rs:30-111) on the MI355X path."""
from __future__ import annotations

from collections import deque
from typing import Callable, Optional

from ..arrow import LazyColumns, RecordBatch, Schema
from .engine import engine
from .expression import RuntimeExpr
from .relation import Relation


def is_host_batch(b: RecordBatch) -> bool:
    return all(c.values.is_cpu for c in b.columns)


def detach(b: RecordBatch) -> RecordBatch:
    """A batch that owns its buffers: a source's zero-copy views (e.g.
    NativeCsvDataSource(copy=False)) are valid only until its next pull."""
    return RecordBatch(b.schema, [_own(a) for a in b.columns])


def _own(a):
    """A copy of Array `a` that owns its buffers, rebased to offset 0 (a
    sliced array keeps only its rows: values, bitmaps and Utf8 offsets)."""
    from ..arrow import Array
    from ..logicalplan import DataType
    cl = lambda t: None if t is None else t.clone()
    if not a.offset:
        return Array(a.data_type, a.length, cl(a.values), cl(a.validity), cl(a.offsets), a.null_count)
    valid = a.valid_mask() if a.validity is not None else None
    if a.data_type == DataType.Utf8:
        vals = a.numpy_values()
        return Array.from_strings([None if (valid is not None and not valid[i]) else vals[i]
                                   for i in range(a.length)]) if valid is not None else Array.from_strings(vals)
    return Array.from_numpy(a.data_type, a.numpy_values().copy(), valid)


class Coalescer:
    """Pulls up to `m` batches (and at most `max_rows` rows) from `source`
    ahead and runs them as ONE call -- device batches as one launch
    (dfmi_filter_project_batches), host batches as one H2D + launch + D2H
    (dfmi_filter_project_host_batches) -- then hands the results out one
    batch per next(): the same output stream as one pull per batch
    (relation.rs:27-32, csv_sql.rs:60-62). One output batch per input batch,
    in order; on an error the batches before the failing one come first, then
    the error, and the batches pulled after it run one at a time if the
    caller goes on. An error the SOURCE raises while reading ahead comes after
    the batches read before it, as the pull loop would have seen it.

    With `run_many_host_async`, while one group's results are handed out the
    next group of host batches is already read and its call runs on the
    engine's worker thread (staging, PCIe and the launch overlap the pull
    loop); the stream is the same. When that call object can be prepared
    without running (it has submit()), the Coalescer keeps the worker busy:
    group g+2 is read and prepared while g+1 runs, and is submitted the
    moment g+1's call returns -- before g+1's output batches are built and
    handed out -- so the pull loop's own work overlaps the device call
    instead of adding to it."""

    def __init__(self, m: int, source: Relation, run_one: Callable, run_many: Callable, wrap: Callable,
                 run_many_host: Callable = None, max_rows: int = 1 << 20, run_many_host_async: Callable = None,
                 wrap_many: Callable = None):
        self.m, self.source, self.max_rows = m, source, max_rows
        self.run_one, self.run_many, self.run_many_host, self.wrap = run_one, run_many, run_many_host, wrap
        self.wrap_many = wrap_many if wrap_many is not None else (lambda rs: [wrap(c) for c in rs])
        self.run_many_host_async = run_many_host_async
        self.ready = deque()       # RecordBatches / exceptions, in stream order
        self.pending = deque()     # pulled input batches (or a source error) still to run one by one
        self.ahead = None          # the next group read ahead: (call in flight or None, batches, source error)
        self.staged = None         # the group after it: (prepared call, not started, batches, source error)

    def _read_ahead(self):
        many = getattr(self.source, "next_many", None)
        if many is not None:  # a source that hands out many batches at once (MemoryDataSource)
            try:
                return many(self.m, self.max_rows), None
            except Exception as e:
                return [], e
        pulled, rows = [], 0
        nxt = self.source.next
        while len(pulled) < self.m and rows < self.max_rows:
            try:
                b = nxt()
            except Exception as e:  # raised after the batches before it
                return pulled, e
            if b is None:
                break
            if b._transient:
                b = detach(b)
            pulled.append(b)
            rows += b.num_rows()
        return pulled, None

    def _fetch(self, start: bool = True):
        """Read the next group and prepare its call when it can run on the
        worker; start it now unless start=False (a call with submit())."""
        pulled, src_err = self._read_ahead()
        fut = None
        if self.run_many_host_async is not None and len(pulled) > 1 and is_host_batch(pulled[0]):
            try:
                fut = self.run_many_host_async(pulled)
            except ValueError:  # not every batch is in host memory: the synchronous runs
                fut = None
            if fut is not None and start and hasattr(fut, "submit"):
                fut.submit()
        return fut, pulled, src_err

    def _take_ahead(self):
        """The next group: the one in flight, else the prepared one (started
        now), else a freshly read one."""
        if self.ahead is not None:
            a, self.ahead = self.ahead, None
            return a
        if self.staged is not None:
            (fut, pulled, src_err), self.staged = self.staged, None
            if fut is not None:
                fut.submit()
            return fut, pulled, src_err
        return self._fetch()

    def _accept(self, pulled, results, err) -> bool:
        """Results of one coalesced call into ready; after a failing batch the
        rest go to pending. True when the group had no error."""
        if results:
            self.ready.extend(self.wrap_many(results))
        if err is not None:
            self.ready.append(err)
            self.pending.extend(pulled[len(results) + 1:])
            return False
        return True

    def _run(self, pulled) -> None:
        """Results of `pulled` (consecutive runs of host / device batches)
        into self.ready; after a failing batch the rest go to pending."""
        i = 0
        while i < len(pulled):
            host = is_host_batch(pulled[i])
            j = i + 1
            while j < len(pulled) and is_host_batch(pulled[j]) == host:
                j += 1
            run = pulled[i:j]
            many = self.run_many_host if host else self.run_many
            if len(run) == 1:  # (a large batch ends the read-ahead): the single-batch entry point
                many = None
            if many is None:  # one call each, in order
                self.pending.extend(pulled[i:])
                return
            results, err = many(run)
            if not self._accept(pulled[i:], results, err):
                return
            i = j

    def next(self) -> Optional[RecordBatch]:
        ready = self.ready
        if ready:  # the common case: a result of the current group
            item = ready.popleft()
            if isinstance(item, Exception):
                raise item
            return item
        while not self.ready:
            if self.pending:
                item = self.pending.popleft()
                if isinstance(item, Exception):
                    raise item
                return self.wrap(self.run_one(item))
            fut, pulled, src_err = self._take_ahead()
            if not pulled:
                if src_err is not None:
                    raise src_err
                return None
            if fut is not None:
                ok = fut.wait() if hasattr(fut, "wait") else True
                if ok and src_err is None and self.staged is not None:
                    # the worker goes on with the next group while this one's
                    # batches are built and handed out
                    (nf, npulled, nerr), self.staged = self.staged, None
                    if nf is not None:
                        nf.submit()
                    self.ahead = (nf, npulled, nerr)
                results, err = fut.result()
                self._accept(pulled, results, err)
            else:
                self._run(pulled)
            if src_err is not None:
                self.pending.append(src_err)
            elif not self.pending and self.run_many_host_async is not None:
                if self.ahead is None and self.staged is None:
                    self.ahead = self._fetch()  # the next group runs while this one is handed out
                if self.ahead is not None and self.ahead[0] is not None and hasattr(self.ahead[0], "submit") \
                        and self.ahead[2] is None and self.ahead[1] and self.staged is None:
                    self.staged = self._fetch(start=False)  # and the one after it is prepared
        item = self.ready.popleft()
        if isinstance(item, Exception):
            raise item
        return item


def _wrap_many_empty(results) -> list:
    """FilterRelation's output batches (Schema::empty(), filter.rs:60-61):
    ready-made HostResultBatches pass through."""
    if results and isinstance(results[0], RecordBatch):
        return results
    sch = Schema.empty()
    return [RecordBatch.lazy(sch, c) if isinstance(c, LazyColumns) else RecordBatch(sch, c) for c in results]


class FilterRelation(Relation):
    """FilterRelation::new(input, expr, schema). next() pulls one batch from
    the input and returns every column filtered by the predicate, in a batch
    whose schema is Schema::empty() (filter.rs:60-61). With coalesce > 1, up
    to that many input batches run as one device call (Coalescer)."""

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
        if is_host_batch(batch):
            return eng.filter_project_host(self.expr, None, batch, self.flags)
        return eng.filter_project(self.expr, None, batch, self.flags)

    def next(self) -> Optional[RecordBatch]:
        co = self._co
        if co is not None:
            return co.next()
        if self.coalesce > 1:
            if self._co is None:
                self._co = Coalescer(self.coalesce, self.input, self.run_batch,
                                     lambda bs: engine(self.device).filter_project_batches(self.expr, None, bs,
                                                                                           self.flags),
                                     lambda cols: (RecordBatch.lazy(Schema.empty(), cols) if isinstance(cols, LazyColumns)
                                                   else RecordBatch(Schema.empty(), cols)),
                                     lambda bs: engine(self.device).filter_project_host_batches(self.expr, None, bs,
                                                                                                self.flags),
                                     run_many_host_async=lambda bs: engine(self.device).filter_project_host_batches_async(
                                         self.expr, None, bs, self.flags, schema=Schema.empty(), start=False),
                                     wrap_many=_wrap_many_empty)
            return self._co.next()
        batch = self.input.next()
        if batch is None:
            return None
        return RecordBatch(Schema.empty(), self.run_batch(batch))  # host batch: host results

    def schema(self) -> Schema:
        return self._schema
