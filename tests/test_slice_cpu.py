"""Sliced arrays (arrow 0.12 ArrayData::offset, dfmi_column.offset): the
oracle reads logical row i at physical slot offset + i, as value(i) /
get_string(i) / is_null(i) do (filter.rs:88-89,99-100). A sliced batch
must give what a batch holding copies of the same rows gives. (The device
twin of this test is tests/test_gpu_slice.py.)"""
import numpy as np
import pytest

from datafusion_amd._abi import DFMI_FLAG_EXT_GATHER_ALL
from datafusion_amd.arrow import Array, Field, RecordBatch, Schema
from datafusion_amd.execution.error import ExecutionError
from datafusion_amd.logicalplan import BinaryExpr, Column, DataType, Float64, Int64, Literal, Operator
from oracle_ffi import oracle_filter_project

SCHEMA = Schema([Field("x", DataType.Float64, True), Field("i", DataType.Int64, True),
                 Field("b", DataType.Boolean, True), Field("s", DataType.Utf8, True)])


def table(n, seed=1):
    rng = np.random.default_rng(seed)
    words = [b"", b"w17", b"alpha", b"\xe2\x82\xac", b"x" * 30]
    return RecordBatch(SCHEMA, [
        Array.from_numpy(DataType.Float64, rng.random(n), rng.random(n) > 0.2),
        Array.from_numpy(DataType.Int64, rng.integers(-50, 50, n), rng.random(n) > 0.1),
        Array.from_numpy(DataType.Boolean, rng.random(n) < 0.5, rng.random(n) > 0.3),
        Array.from_strings([None if rng.random() < 0.1 else words[rng.integers(0, 5)] for _ in range(n)])])


def materialize(a: Array) -> Array:
    """A fresh offset-0 array holding the slice's logical rows."""
    valid = a.valid_mask() if a.validity is not None else None
    if a.data_type == DataType.Utf8:
        vals = a.numpy_values()
        return Array.from_strings([None if valid is not None and not valid[i] else vals[i] for i in range(a.length)])
    return Array.from_numpy(a.data_type, a.numpy_values(), valid)


def sliced(batch, off, n):
    return RecordBatch(batch.schema, [c.slice(off, n) for c in batch.columns])


QUERIES = [
    (BinaryExpr(Column(0), Operator.Lt, Literal(Float64(0.5))), [Column(0), Column(3), Column(1)]),
    (BinaryExpr(Column(2), Operator.And, BinaryExpr(Column(1), Operator.Gt, Literal(Int64(-10)))),
     [BinaryExpr(Column(1), Operator.Multiply, Literal(Int64(3))), Column(3), Column(2)]),
    (None, [BinaryExpr(Column(0), Operator.Plus, Column(0)), Column(3), Column(2)]),
]


def result(schema, batch, pred, projs):
    try:
        return [(n, a.numpy_values(), a.valid_mask()) for n, a in
                oracle_filter_project(schema, batch, pred, projs, DFMI_FLAG_EXT_GATHER_ALL)]
    except ExecutionError as e:
        return (e.kind, e.message)


def same(x, y):
    if isinstance(x, tuple):
        return x == y
    for (n1, v1, m1), (n2, v2, m2) in zip(x, y):
        assert n1 == n2 and np.array_equal(m1, m2)
        if isinstance(v1, list):
            assert [a for a, k in zip(v1, m1) if k] == [b for b, k in zip(v2, m2) if k]
        else:
            assert np.array_equal(np.asarray(v1)[m1].view(np.uint8), np.asarray(v2)[m2].view(np.uint8))
    return len(x) == len(y)


@pytest.mark.parametrize("off", [0, 1, 5, 8, 63, 64, 100, 777])
def test_oracle_reads_sliced_arrays(off):
    t = table(2000)
    n = 2000 - off - 13
    s = sliced(t, off, n)
    m = RecordBatch(SCHEMA, [materialize(c) for c in s.columns])
    for pred, projs in QUERIES:
        assert same(result(SCHEMA, s, pred, projs), result(SCHEMA, m, pred, projs)), (off, pred)


def test_slice_views_and_null_counts():
    t = table(300)
    a = t.columns[0]
    for off, n in ((0, 300), (7, 100), (64, 1), (299, 1), (10, 0)):
        s = a.slice(off, n)
        assert s.offset == off and s.length == n
        assert np.array_equal(s.valid_mask(), a.valid_mask()[off:off + n])
        assert s.null_count == int((~a.valid_mask()[off:off + n]).sum())
        assert np.array_equal(s.numpy_values(), a.numpy_values()[off:off + n])
    u = t.columns[3].slice(9, 50)
    assert u.numpy_values() == t.columns[3].numpy_values()[9:59]
