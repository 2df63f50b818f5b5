"""The relations' read-ahead (execution/filter.py Coalescer) on the CPU, with
stand-in run functions: the stream it hands out must be the one the
reference's pull loop sees (csv_sql.rs:60-62, relation.rs:27-32) -- one
output batch per input batch, in order, errors at the position they arise,
including an error the SOURCE raises while the Coalescer reads ahead, and
zero-copy batches a source overwrites on its next pull."""
import numpy as np
import pytest

from datafusion_amd.arrow import Array, RecordBatch, Schema
from datafusion_amd.execution.error import ExecutionError
from datafusion_amd.execution.filter import Coalescer
from datafusion_amd.logicalplan import DataType


def batch(tag, n=4):
    return RecordBatch(Schema.empty(), [Array.from_numpy(DataType.Float64, np.full(n, float(tag)))])


def tag_of(b):
    return float(b.columns[0].numpy_values()[0])


class Source:
    """Batches 0..n-1; raises at `fail_at` (once); `transient` reuses ONE
    buffer for every batch (a reader's pinned set, overwritten on each pull)."""

    def __init__(self, n, fail_at=None, transient=False):
        self.i, self.n, self.fail_at, self.transient = 0, n, fail_at, transient
        self.buf = batch(-1)

    def next(self):
        if self.i == self.fail_at:
            self.fail_at = None
            raise ExecutionError("ArrowError(ParseError)", "bad row in batch %d" % self.i)
        if self.i >= self.n:
            return None
        t = self.i
        self.i += 1
        if not self.transient:
            return batch(t)
        self.buf.columns[0].values[:32] = batch(t).columns[0].values[:32]  # overwrite in place
        self.buf._transient = True
        return self.buf


FAIL = set()  # batch tags whose evaluation raises DivideByZero


def run_one(b):
    if tag_of(b) in FAIL:
        raise ExecutionError("ArrowError(DivideByZero)", "DivideByZero")
    return [b.columns[0]]


calls = []


def run_many(bs):
    calls.append(len(bs))
    out = []
    for i, b in enumerate(bs):
        if tag_of(b) in FAIL:
            e = ExecutionError("ArrowError(DivideByZero)", "DivideByZero")
            e.failed_batch = i
            return out, e
        out.append([b.columns[0]])
    return out, None


def stream(co):
    """What a pull loop sees: tags and errors, continuing after an error."""
    seen = []
    for _ in range(1000):
        try:
            b = co.next()
        except ExecutionError as e:
            seen.append(e.message)
            continue
        if b is None:
            return seen
        seen.append(tag_of(b))
    raise AssertionError("no end")


class Done:
    """A finished future (the engine's worker thread, stood in for)."""

    def __init__(self, v):
        self.v = v

    def result(self):
        return self.v


def run_many_async(bs):
    return Done(run_many(bs))


log = []


class Staged:
    """A prepared call (the engine's HostBatchesCall with start=False): runs
    on submit(), wait() says whether every batch ran, result() hands over."""

    def __init__(self, bs):
        self.bs, self.v = bs, None
        log.append(("prepare", tag_of(bs[0])))

    def submit(self):
        log.append(("submit", tag_of(self.bs[0])))
        self.v = run_many(self.bs)
        return self

    def wait(self):
        assert self.v is not None, "waited on a call that was never submitted"
        return self.v[1] is None

    def result(self):
        log.append(("result", tag_of(self.bs[0])))
        return self.v


def co(src, m=8, max_rows=1 << 20, asynchronous=False):
    calls.clear()
    log.clear()
    fn = None
    if asynchronous == "staged":
        fn = Staged
    elif asynchronous:
        fn = run_many_async
    return Coalescer(m, src, run_one, None, lambda cols: RecordBatch(Schema.empty(), cols), run_many,
                     max_rows=max_rows, run_many_host_async=fn)


def test_staged_calls_keep_the_worker_busy():
    """With prepared calls, group g+1 is submitted as soon as group g's call
    returns -- before g's results are taken -- and group g+2 is read and
    prepared (not started) while g+1 runs; the stream is unchanged."""
    c = co(Source(40), asynchronous="staged")
    assert tag_of(c.next()) == 0.0
    assert log == [("prepare", 0.0), ("submit", 0.0), ("result", 0.0), ("prepare", 8.0), ("submit", 8.0),
                   ("prepare", 16.0)]
    for _ in range(7):
        c.next()
    log.clear()
    assert tag_of(c.next()) == 8.0
    assert log == [("submit", 16.0), ("result", 8.0), ("prepare", 24.0)]
    assert stream(c) == [float(i) for i in range(9, 40)]


@pytest.mark.parametrize("asynchronous", [False, True, "staged"])
def test_order_and_one_call_per_group(asynchronous):
    assert stream(co(Source(20), asynchronous=asynchronous)) == [float(i) for i in range(20)]
    assert calls == [8, 8, 4]


def test_async_reads_the_next_group_while_handing_out():
    """After the first group, the next group's call is issued before the
    first group's batches are all handed out."""
    c = co(Source(24), asynchronous=True)
    assert tag_of(c.next()) == 0.0
    assert calls == [8, 8]  # group 2 already submitted
    assert stream(c) == [float(i) for i in range(1, 24)]


def test_row_bound_ends_read_ahead():
    assert stream(co(Source(10), m=8, max_rows=12)) == [float(i) for i in range(10)]
    assert calls == [3, 3, 3]  # 4-row batches: three reach 12 rows; the last one runs alone


@pytest.mark.parametrize("asynchronous", [False, True, "staged"])
@pytest.mark.parametrize("m", [8, 16])
def test_error_in_a_middle_batch_then_the_rest(m, asynchronous):
    """Batch 13 fails: 0..12 come first, then the error, then 14.. (the
    pull loop goes on after an error if the caller does)."""
    FAIL.add(13)
    try:
        got = stream(co(Source(20), m=m, asynchronous=asynchronous))
    finally:
        FAIL.clear()
    assert got[:13] == [float(i) for i in range(13)]
    assert got[13] == "DivideByZero"
    assert got[14:] == [float(i) for i in range(14, 20)]


@pytest.mark.parametrize("asynchronous", [False, True, "staged"])
@pytest.mark.parametrize("fail_at", [5, 8, 9, 12])
def test_source_error_while_reading_ahead(fail_at, asynchronous):
    """The source fails on the pull of batch `fail_at`: the batches before it
    come first, then the source's error, then the stream goes on (the pull
    loop's view) -- also when the failing pull belongs to a group read ahead
    while the previous one is handed out."""
    got = stream(co(Source(14, fail_at=fail_at), m=4, asynchronous=asynchronous))
    assert got[:fail_at] == [float(i) for i in range(fail_at)]
    assert got[fail_at] == "bad row in batch %d" % fail_at
    assert got[fail_at + 1:] == [float(i) for i in range(fail_at, 14)]


def test_source_error_while_reading_ahead_m8():
    got = stream(co(Source(10, fail_at=5)))
    assert got[:5] == [float(i) for i in range(5)]
    assert got[5] == "bad row in batch 5"
    assert got[6:] == [float(i) for i in range(5, 10)]


def test_source_error_on_first_pull():
    got = stream(co(Source(3, fail_at=0)))
    assert got == ["bad row in batch 0", 0.0, 1.0, 2.0]


@pytest.mark.parametrize("asynchronous", [False, True, "staged"])
def test_transient_batches_are_copied_before_the_next_pull(asynchronous):
    """A source that overwrites its batch buffers on every pull (e.g.
    NativeCsvDataSource(copy=False)): the read-ahead keeps its own copies."""
    assert stream(co(Source(20, transient=True), asynchronous=asynchronous)) == [float(i) for i in range(20)]


@pytest.mark.parametrize("m", [1, 2, 7])
def test_small_lookahead(m):
    assert stream(co(Source(9), m=m)) == [float(i) for i in range(9)]


@pytest.mark.parametrize("m,max_rows", [(8, 1 << 20), (8, 12), (3, 5), (16, 1), (5, 13)])
def test_memory_source_next_many_is_repeated_next(m, max_rows):
    """MemoryDataSource.next_many (the Coalescer's bulk read-ahead) returns
    exactly what its read-ahead loop of next() calls would: up to m batches,
    the one that reaches max_rows rows the last; ragged and empty batches."""
    from datafusion_amd.execution import MemoryDataSource
    sizes = [4, 0, 7, 1, 0, 0, 9, 3, 4, 4, 12, 1, 0, 2]
    bs = [batch(i, n) for i, n in enumerate(sizes)]
    bulk, loop = MemoryDataSource(Schema.empty(), bs), MemoryDataSource(Schema.empty(), bs)
    while True:
        got = bulk.next_many(m, max_rows)
        want, rows = [], 0
        while len(want) < m and rows < max_rows:
            b = loop.next()
            if b is None:
                break
            want.append(b)
            rows += b.num_rows()
        assert [id(b) for b in got] == [id(b) for b in want]
        if not got:
            break
    assert bulk.next() is None


def test_coalescer_over_memory_source_bulk_read_ahead():
    from datafusion_amd.execution import MemoryDataSource
    from datafusion_amd.execution.relation import DataSourceRelation
    src = DataSourceRelation(MemoryDataSource(Schema.empty(), [batch(i) for i in range(20)]))
    assert stream(co(src, m=8, max_rows=12, asynchronous=True)) == [float(i) for i in range(20)]
    assert calls == [3] * 6 + [2]  # 4-row batches: 12 rows a group
