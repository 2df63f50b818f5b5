"""Aggregate extension (DFMI_FLAG_EXT_AGGREGATE) on the CPU: the oracle's
semantics against independent restatements (math.fsum for the exactly rounded
Float64 SUM, exact rationals for Float32, numpy for integers / MIN / MAX /
COUNT), compile-time errors of compile_expr's AggregateFunction arm
(expression.rs:81-116), the planner's Aggregate plan (sqlplanner.rs:80-117),
and the aggregate kernels generated and compiled with hipRTC for gfx950.

The reference cannot execute an Aggregate plan (context.rs:161
unimplemented!()), so these semantics are parity unpinned: build-defined,
pinned by the oracle."""
import ctypes as C
import math
from fractions import Fraction

import numpy as np
import pytest

from datafusion_amd import _abi
from datafusion_amd.arrow import Array, Field, RecordBatch, Schema
from datafusion_amd.execution.error import ExecutionError
from datafusion_amd.execution.expression import compile_expr, compile_scalar_expr
from datafusion_amd.logicalplan import (AggregateFunction, BinaryExpr, Column, DataType, Float64, Literal, Operator)
from oracle_ffi import oracle_aggregate
from test_jit_cpu import HostBatch

AGG = _abi.DFMI_FLAG_EXT_AGGREGATE


def agg(name, e, schema):
    t = DataType.UInt64 if name.lower() == "count" else e.get_type(schema)
    return AggregateFunction(name, (e,), t)


def bits_f64(v):
    return int(np.array([v], dtype=np.float64).view(np.uint64)[0])


def bits_f32(v):
    return int(np.array([v], dtype=np.float32).view(np.uint32)[0])


def wild_doubles(rng, n):
    """Random doubles over the whole exponent range, subnormals, exact
    cancellations and signed zeros."""
    mant = rng.random(n) + 1.0
    exp = rng.integers(-1074, 1000, n)
    x = np.ldexp(mant, exp) * np.where(rng.random(n) < 0.5, -1.0, 1.0)
    x[rng.random(n) < 0.05] = 0.0
    x[rng.random(n) < 0.03] = -0.0
    k = n // 10
    x[:k] = np.ldexp(rng.random(k), rng.integers(-20, 20, k))
    x[k:2 * k] = -x[:k]  # cancels exactly
    rng.shuffle(x)
    return x


def f32_round(q: Fraction) -> np.float32:
    """Round an exact rational to float32, half to even."""
    if q == 0:
        return np.float32(0.0)
    c = np.float32(float(q))
    best = None
    for cand in (np.nextafter(c, np.float32(-np.inf)), c, np.nextafter(c, np.float32(np.inf))):
        if not np.isfinite(cand):
            continue
        d = abs(Fraction(float(cand)) - q)
        if best is None or d < best[0] or (d == best[0] and (bits_f32(cand) & 1) == 0):
            best = (d, cand)
    return best[1]


@pytest.mark.parametrize("seed", range(6))
def test_oracle_f64_sum_is_fsum(seed):
    rng = np.random.default_rng(seed)
    x = wild_doubles(rng, 5000)
    s = Schema([Field("x", DataType.Float64, False)])
    b = RecordBatch(s, [Array.from_numpy(DataType.Float64, x)])
    for rows in (0, 8, 1024):
        v = oracle_aggregate(s, b, None, [agg("SUM", Column(0), s)], batch_rows=rows)[0]
        want = math.fsum(x.tolist())
        if want == 0:
            want = 0.0 if any(not (t == 0 and math.copysign(1, t) < 0) for t in x) else -0.0
        assert v.bits == bits_f64(want), (rows, v.bits, bits_f64(want))


def test_oracle_f64_sum_specials():
    s = Schema([Field("x", DataType.Float64, True)])
    cases = [
        ([1.0, float("nan"), 2.0], 0x7FF8000000000000),
        ([float("inf"), 1.0], bits_f64(float("inf"))),
        ([float("-inf"), 1.0], bits_f64(float("-inf"))),
        ([float("inf"), float("-inf")], 0x7FF8000000000000),
        ([-0.0, -0.0], bits_f64(-0.0)),
        ([-0.0, 0.0], bits_f64(0.0)),
        ([1e308, 1e308], bits_f64(float("inf"))),
        ([1e308, 1e308, -1e308], bits_f64(1e308)),
        ([5e-324, 5e-324], bits_f64(1e-323)),
    ]
    for xs, want in cases:
        b = RecordBatch(s, [Array.from_numpy(DataType.Float64, np.array(xs))])
        v = oracle_aggregate(s, b, None, [agg("sum", Column(0), s)])[0]
        assert v.bits == want, (xs, hex(v.bits))
    # nulls are skipped; all-null -> null, COUNT 0
    b = RecordBatch(s, [Array.from_numpy(DataType.Float64, np.array([1.0, 2.0]), np.array([False, False]))])
    v = oracle_aggregate(s, b, None, [agg("SUM", Column(0), s), agg("COUNT", Column(0), s)])
    assert v[0].is_null == 1 and v[1].is_null == 0 and v[1].bits == 0


@pytest.mark.parametrize("seed", range(3))
def test_oracle_f32_sum_exact(seed):
    rng = np.random.default_rng(100 + seed)
    x = (rng.standard_normal(3000) * np.exp2(rng.integers(-140, 120, 3000))).astype(np.float32)
    s = Schema([Field("x", DataType.Float32, False)])
    b = RecordBatch(s, [Array.from_numpy(DataType.Float32, x)])
    v = oracle_aggregate(s, b, None, [agg("SUM", Column(0), s)])[0]
    q = sum(Fraction(float(t)) for t in x)
    assert v.bits == bits_f32(f32_round(q))


@pytest.mark.parametrize("t", [DataType.Int8, DataType.Int16, DataType.Int32, DataType.Int64, DataType.UInt8,
                               DataType.UInt16, DataType.UInt32, DataType.UInt64])
def test_oracle_int_aggregates(t):
    rng = np.random.default_rng(int(t))
    dt = np.dtype({DataType.Int8: np.int8, DataType.Int16: np.int16, DataType.Int32: np.int32,
                   DataType.Int64: np.int64, DataType.UInt8: np.uint8, DataType.UInt16: np.uint16,
                   DataType.UInt32: np.uint32, DataType.UInt64: np.uint64}[t])
    info = np.iinfo(dt)
    x = rng.integers(info.min, info.max, 4000, dtype=dt, endpoint=True)
    valid = rng.random(4000) >= 0.2
    s = Schema([Field("x", t, True)])
    b = RecordBatch(s, [Array.from_numpy(t, x, valid)])
    aggs = [agg(f, Column(0), s) for f in ("SUM", "MIN", "MAX", "COUNT")]
    v = oracle_aggregate(s, b, None, aggs)
    xv = x[valid]
    wsum = np.array([int(xv.astype(object).sum()) % (1 << (8 * dt.itemsize))], dtype=np.uint64).astype(dt)[0]
    def ext(val):  # sign/zero extension to 64 bits
        return int(np.array([val], dtype=dt).astype(np.int64 if info.min < 0 else np.uint64).view(np.uint64)[0])
    assert v[0].bits == ext(wsum)
    assert v[1].bits == ext(xv.min()) and v[2].bits == ext(xv.max())
    assert v[3].bits == int(valid.sum()) and v[3].type == DataType.UInt64


def test_oracle_float_min_max():
    s = Schema([Field("x", DataType.Float64, True)])
    xs = np.array([3.0, -0.0, 0.0, float("nan"), -2.5, float("inf")])
    b = RecordBatch(s, [Array.from_numpy(DataType.Float64, xs)])
    v = oracle_aggregate(s, b, None, [agg("MIN", Column(0), s), agg("MAX", Column(0), s)])
    assert v[0].bits == bits_f64(-2.5) and v[1].bits == bits_f64(float("inf"))
    b = RecordBatch(s, [Array.from_numpy(DataType.Float64, np.array([0.0, -0.0]))])
    v = oracle_aggregate(s, b, None, [agg("MIN", Column(0), s), agg("MAX", Column(0), s)])
    assert v[0].bits == bits_f64(-0.0) and v[1].bits == bits_f64(0.0)
    b = RecordBatch(s, [Array.from_numpy(DataType.Float64, np.array([float("nan")] * 3))])
    v = oracle_aggregate(s, b, None, [agg("MIN", Column(0), s)])
    assert v[0].bits == 0x7FF8000000000000


def test_oracle_predicate_drops_validity():
    """Aggregate(Selection(scan)): the argument sees the FILTERED batch, which
    has no validity (filter() copies raw slots, filter.rs:84-93)."""
    s = Schema([Field("x", DataType.Float64, True), Field("k", DataType.Float64, False)])
    x = np.array([1.0, 2.0, 4.0, 8.0])
    b = RecordBatch(s, [Array.from_numpy(DataType.Float64, x, np.array([True, False, True, True])),
                        Array.from_numpy(DataType.Float64, np.array([0.0, 1.0, 1.0, 0.0]))])
    pred = BinaryExpr(Column(1), Operator.Gt, Literal(Float64(0.5)))
    v = oracle_aggregate(s, b, pred, [agg("SUM", Column(0), s), agg("COUNT", Column(0), s)])
    assert v[0].bits == bits_f64(6.0) and v[1].bits == 2
    v = oracle_aggregate(s, b, None, [agg("SUM", Column(0), s), agg("COUNT", Column(0), s)])
    assert v[0].bits == bits_f64(13.0) and v[1].bits == 3


def compile_agg(name, e, s, flags=AGG):
    return compile_expr(None, agg(name, e, s), s, flags)


def test_compile_aggregate_errors():
    s = Schema([Field("x", DataType.Float64, False), Field("u", DataType.Utf8, False)])
    with pytest.raises(ExecutionError) as ei:
        compile_agg("SUM", Column(0), s, flags=0)
    assert ei.value.kind == "panic" and ei.value.message == "not yet implemented"
    with pytest.raises(ExecutionError) as ei:
        compile_agg("avg", Column(0), s)
    assert ei.value.message == "not yet implemented: Unsupported aggregate function 'avg'"
    with pytest.raises(ExecutionError) as ei:
        compile_agg("SUM", Column(1), s)
    assert ei.value.kind == "NotImplemented"
    a = compile_agg("count", Column(1), s)
    assert a.get_name() == "count" and a.get_type() == DataType.UInt64
    a = compile_agg("Max", Column(0), s)
    assert a.get_type() == DataType.Float64
    # the same errors on the oracle
    b = RecordBatch(s, [Array.from_numpy(DataType.Float64, np.zeros(3)), Array.from_strings([b"a", b"b", b"c"])])
    with pytest.raises(ExecutionError) as ei:
        oracle_aggregate(s, b, None, [agg("avg", Column(0), s)])
    assert ei.value.message == "not yet implemented: Unsupported aggregate function 'avg'"


def _agg_jit(schema, pred, aggs, flags=AGG, compile_=True):
    L = _abi.lib()
    fn = L.dfmi_internal_agg_jit_check
    fn.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.c_int32, C.POINTER(_abi.dfmi_batch), C.c_uint32, C.c_int32,
                   C.c_char_p, C.c_int64, C.POINTER(_abi.dfmi_error)]
    fn.restype = C.c_int64
    hb = HostBatch(schema)
    p = compile_scalar_expr(None, pred, schema, flags) if pred is not None else None
    cs = [compile_expr(None, a, schema, flags) for a in aggs]
    arr = (C.c_void_p * len(cs))(*[c.handle.value for c in cs])
    err = _abi.dfmi_error()
    buf = C.create_string_buffer(1 << 20)
    rc = fn(p.handle if p else None, arr, len(cs), C.byref(hb.batch), flags, int(compile_), buf, len(buf),
            C.byref(err))
    return rc, err.code, err.message.decode(), buf.value.decode()


def test_aggregate_kernels_compile():
    s = Schema([Field("q", DataType.Float64, False), Field("p", DataType.Float64, False),
                Field("d", DataType.Float64, False), Field("i", DataType.Int32, True),
                Field("f", DataType.Float32, True), Field("u", DataType.Utf8, True)])
    pred = BinaryExpr(BinaryExpr(Column(0), Operator.Lt, Literal(Float64(24.0))), Operator.And,
                      BinaryExpr(Column(2), Operator.GtEq, Literal(Float64(0.05))))
    q6 = [agg("SUM", BinaryExpr(Column(1), Operator.Multiply, Column(2)), s)]
    rc, code, msg, src = _agg_jit(s, pred, q6, AGG | _abi.DFMI_FLAG_EXT_GATHER_ALL)
    assert rc > 0, msg
    assert "fsum_add" in src and "agg_block_flush" in src
    allf = [agg(f, Column(c), s) for f in ("SUM", "MIN", "MAX", "COUNT") for c in (3, 4)] + [agg("COUNT", Column(5), s)]
    rc, code, msg, src = _agg_jit(s, None, allf)
    assert rc > 0, msg
    rc, code, msg, src = _agg_jit(s, pred, allf, AGG | _abi.DFMI_FLAG_EXT_GATHER_ALL)
    assert rc > 0, msg


def test_planner_builds_aggregate():
    from datafusion_amd.execution import ExecutionContext, MemoryDataSource
    from datafusion_amd.execution.context import Aggregate, Selection
    from datafusion_amd.sqlplanner import SqlToRel
    s = Schema([Field("a", DataType.Float64, False), Field("b", DataType.Int64, True)])
    ctx = ExecutionContext(flags=AGG)
    ctx.register_datasource("t", MemoryDataSource(s, []))
    p = SqlToRel(ctx).sql_to_rel("SELECT a, SUM(a * 2.0), count(*), MIN(b) FROM t WHERE a > 0.5")
    assert isinstance(p, Aggregate) and isinstance(p.input, Selection) and not p.group_expr
    assert [repr(e) for e in p.aggr_expr] == ["SUM(#0 Multiply Float64(2.0))", "count(#0)", "MIN(#1)"]
    assert [e.return_type for e in p.aggr_expr] == [DataType.Float64, DataType.UInt64, DataType.Int64]
    p = SqlToRel(ctx).sql_to_rel("SELECT MAX(a) FROM t GROUP BY b")
    assert [repr(e) for e in p.group_expr] == ["#1"]


def _grouped_jit(schema, pred, key, aggs, flags=AGG, compile_=True):
    L = _abi.lib()
    fn = L.dfmi_internal_agg_grouped_jit_check
    fn.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p), C.c_int32, C.POINTER(_abi.dfmi_batch), C.c_uint32,
                   C.c_int32, C.c_char_p, C.c_int64, C.POINTER(_abi.dfmi_error)]
    fn.restype = C.c_int64
    hb = HostBatch(schema)
    p = compile_scalar_expr(None, pred, schema, flags) if pred is not None else None
    k = compile_scalar_expr(None, key, schema, flags)
    cs = [compile_expr(None, a, schema, flags) for a in aggs]
    arr = (C.c_void_p * len(cs))(*[c.handle.value for c in cs])
    err = _abi.dfmi_error()
    buf = C.create_string_buffer(1 << 20)
    rc = fn(p.handle if p else None, k.handle, arr, len(cs), C.byref(hb.batch), flags, int(compile_), buf, len(buf),
            C.byref(err))
    return rc, err.code, err.message.decode(), buf.value.decode()


def test_grouped_aggregate_kernels_compile():
    """GROUP BY extension: the grouped kernel (slot per row, per-slot
    reductions, [copies][slots][aggs + 1] accumulators) compiles for a Boolean
    key (3 slots) and an integer key (17 slots), with exact float sums."""
    s = Schema([Field("k", DataType.Boolean, True), Field("i", DataType.Int16, True),
                Field("x", DataType.Float64, True), Field("f", DataType.Float32, False)])
    pred = BinaryExpr(Column(2), Operator.Lt, Literal(Float64(0.7)))
    aggs = [agg("SUM", Column(2), s), agg("MIN", Column(3), s), agg("COUNT", Column(1), s), agg("MAX", Column(1), s)]
    for key, slots in ((Column(0), 3), (Column(1), 17)):
        for p in (None, pred):
            rc, code, msg, src = _grouped_jit(s, p, key, aggs)
            assert rc > 0, msg
            assert "GS = %d" % slots in src and "gsl[k]" in src and "fsum_add(S[g_]" in src


def test_oracle_groups_float_and_utf8_keys():
    """GROUP BY over float and Utf8 keys on the oracle (build-defined, parity
    unpinned: the reference executes no Aggregate): floats one group per bit
    pattern in IEEE 754 totalOrder (-NaN < -inf < ... < -0.0 < +0.0 < ... <
    +inf < +NaN), Utf8 bytewise (a shorter prefix first), the null key last."""
    from oracle_ffi import oracle_aggregate_grouped
    nan = np.frombuffer(np.array([0x7FF8000000000000], np.uint64).tobytes(), np.float64)[0]
    nneg = np.frombuffer(np.array([0xFFF8000000000001], np.uint64).tobytes(), np.float64)[0]
    x = np.array([1.0, -0.0, 0.0, nan, nneg, np.inf, -np.inf, 1.0, 5.0])
    valid = np.array([True] * 8 + [False])
    s = Schema([Field("x", DataType.Float64, True), Field("t", DataType.Utf8, True)])
    t = [b"b", b"", b"a", b"ab", b"\xff", b"a", None, b"ab", b"a"]
    b = RecordBatch(s, [Array.from_numpy(DataType.Float64, x, valid), Array.from_strings(t)])
    keys, vals = oracle_aggregate_grouped(s, b, None, Column(0), [agg("COUNT", Column(1), s)])
    got = [None if k.is_null else int(k.bits) for k in keys]
    bits = lambda v: int(np.array([v], np.float64).view(np.uint64)[0])
    assert got == [bits(nneg), bits(-np.inf), bits(-0.0), bits(0.0), bits(1.0), bits(np.inf), bits(nan), None]
    assert [k.count for k in keys] == [1, 1, 1, 1, 2, 1, 1, 1]
    keys, vals, strs = oracle_aggregate_grouped(s, b, None, Column(1), [agg("COUNT", Column(0), s)], key_strings=True)
    assert strs == [b"", b"a", b"ab", b"b", b"\xff", None]
    assert [k.count for k in keys] == [1, 3, 2, 1, 1, 1]
    assert [v[0].bits for v in vals] == [1, 2, 2, 1, 1, 1]  # COUNT(x): non-null x per group
