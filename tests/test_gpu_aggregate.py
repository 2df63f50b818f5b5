"""GPU parity of the aggregate extension (DFMI_FLAG_EXT_AGGREGATE): the fused
Selection + Aggregate kernels (through the C ABI) against the CPU oracle,
bit for bit -- MIN / MAX / SUM / COUNT over every numeric type, nulls, the
predicate dropping validity (filter.rs:84-93), NaN / infinities / signed
zeros, exact Float64 and Float32 sums over the whole exponent range, many
batches, merged per-shard partials, error order, and the Q6 query
(SUM(l_extendedprice * l_discount)) end to end through ctx.sql().

Parity unpinned: the reference plans Aggregate but cannot execute it
(context.rs:161 unimplemented!()); the oracle restates the build's semantics
and tests/test_aggregate_cpu.py pins the oracle against math.fsum / exact
rationals / numpy."""
import numpy as np
import pytest
import torch

from datafusion_amd import _abi
from datafusion_amd.arrow import Array, Field, RecordBatch, Schema
from datafusion_amd.execution import ExecutionContext, MemoryDataSource
from datafusion_amd.execution.aggregate import agg_value_py
from datafusion_amd.execution.engine import engine, merge_agg_partials
from datafusion_amd.execution.error import ExecutionError
from datafusion_amd.execution.expression import compile_expr, compile_scalar_expr
from datafusion_amd.logicalplan import (AggregateFunction, BinaryExpr, Column, DataType, Float64, Int64, Literal,
                                        Operator)
from oracle_ffi import oracle_aggregate
from test_aggregate_cpu import agg, wild_doubles

pytestmark = pytest.mark.gpu

AGG = _abi.DFMI_FLAG_EXT_AGGREGATE
NP = {DataType.Int8: np.int8, DataType.Int16: np.int16, DataType.Int32: np.int32, DataType.Int64: np.int64,
      DataType.UInt8: np.uint8, DataType.UInt16: np.uint16, DataType.UInt32: np.uint32, DataType.UInt64: np.uint64,
      DataType.Float32: np.float32, DataType.Float64: np.float64}


def slice_batch(b: RecordBatch, r0: int, n: int) -> RecordBatch:
    """Rows [r0, r0+n) as a view of the same buffers: offset-0 views of the
    sliced ranges when r0 is a multiple of 8, else arrow slices (a non-zero
    dfmi_column.offset, unsliced at the boundary)."""
    if r0 % 8:
        return RecordBatch(b.schema, [a.slice(r0, n) for a in b.columns])
    cols = []
    for a in b.columns:
        t = a.data_type
        v = a.validity[r0 // 8:] if a.validity is not None else None
        nulls = 0
        if v is not None:
            bits = np.unpackbits(v[: (n + 7) // 8].cpu().numpy(), bitorder="little")[:n]
            nulls = int(n - bits.sum())
        if t == DataType.Utf8:
            c = Array(t, n, a.values, v, a.offsets[r0:r0 + n + 1], nulls)
        elif t == DataType.Boolean:
            c = Array(t, n, a.values[r0 // 8:], v, None, nulls)
        else:
            w = t.width
            c = Array(t, n, a.values[r0 * w:(r0 + n) * w], v, None, nulls)
        cols.append(c)
    return RecordBatch(b.schema, cols)


def run_agg(schema, batch, pred, aggs, flags=AGG, batch_rows=0):
    """Device values and oracle values (bit-identical), or the same error."""
    ref = ref_err = dev = dev_err = None
    try:
        ref = oracle_aggregate(schema, batch, pred, aggs, flags, batch_rows)
    except ExecutionError as e:
        ref_err = e
    try:
        p = compile_scalar_expr(None, pred, schema, flags) if pred is not None else None
        cs = [compile_expr(None, a, schema, flags) for a in aggs]
        st = engine().agg_state(cs)
        n = batch.num_rows()
        step = batch_rows if batch_rows > 0 else max(n, 1)
        dbatch = batch.to(engine().device)
        for r0 in range(0, max(n, 1), step):
            st.add(p, slice_batch(dbatch, r0, min(step, n - r0)) if n else dbatch, flags)
        dev = st.finish()
    except ExecutionError as e:
        dev_err = e
    if ref_err is not None or dev_err is not None:
        assert ref_err is not None and dev_err is not None, (ref_err, dev_err)
        assert (dev_err.kind, dev_err.message) == (ref_err.kind, ref_err.message)
        return None
    for a, d, r in zip(aggs, dev, ref):
        assert (d.type, d.is_null, d.count) == (r.type, r.is_null, r.count), (repr(a), d.count, r.count)
        if not r.is_null:
            assert d.bits == r.bits, (repr(a), hex(d.bits), hex(r.bits))
    return dev


def test_f64_exact_sum_min_max_count():
    rng = np.random.default_rng(1)
    n = 300_007
    x = wild_doubles(rng, n)
    s = Schema([Field("x", DataType.Float64, True), Field("k", DataType.Float64, False)])
    b = RecordBatch(s, [Array.from_numpy(DataType.Float64, x, rng.random(n) >= 0.1),
                        Array.from_numpy(DataType.Float64, rng.random(n))])
    aggs = [agg(f, Column(0), s) for f in ("SUM", "MIN", "MAX", "COUNT")]
    run_agg(s, b, None, aggs)
    run_agg(s, b, None, aggs, batch_rows=65536)
    pred = BinaryExpr(Column(1), Operator.Lt, Literal(Float64(0.3)))
    run_agg(s, b, pred, aggs)
    # same-digit fast path: values of one binade, heavy cancellation
    y = 1.0 + rng.random(n)
    y[::2] *= -1
    b2 = RecordBatch(s, [Array.from_numpy(DataType.Float64, y), b.columns[1]])
    run_agg(s, b2, None, [agg("SUM", Column(0), s), agg("sum", BinaryExpr(Column(0), Operator.Multiply, Column(1)), s)])


def test_f64_sum_specials():
    s = Schema([Field("x", DataType.Float64, False)])
    for xs in ([1.0, float("nan"), 2.0], [float("inf"), 1.0], [float("-inf"), 3.0], [float("inf"), float("-inf")],
               [-0.0, -0.0], [-0.0, 0.0], [1e308, 1e308], [1e308, 1e308, -1e308], [5e-324, 5e-324],
               [float("nan")] * 3, [0.0, -0.0]):
        x = np.array(xs * 700)
        b = RecordBatch(s, [Array.from_numpy(DataType.Float64, x)])
        run_agg(s, b, None, [agg(f, Column(0), s) for f in ("SUM", "MIN", "MAX", "COUNT")])


@pytest.mark.parametrize("t", list(NP))
def test_every_type_with_nulls_and_predicate(t):
    rng = np.random.default_rng(10 + int(t))
    n = 100_003
    dt = np.dtype(NP[t])
    if dt.kind == "f":
        x = (rng.standard_normal(n) * np.exp2(rng.integers(-60, 60, n))).astype(dt)
        x[rng.random(n) < 0.01] = np.nan
    else:
        info = np.iinfo(dt)
        x = rng.integers(info.min, info.max, n, dtype=dt, endpoint=True)
    s = Schema([Field("x", t, True), Field("k", DataType.Float64, False)])
    b = RecordBatch(s, [Array.from_numpy(t, x, rng.random(n) >= 0.15), Array.from_numpy(DataType.Float64, rng.random(n))])
    aggs = [agg(f, Column(0), s) for f in ("SUM", "MIN", "MAX", "COUNT")]
    run_agg(s, b, None, aggs)
    run_agg(s, b, BinaryExpr(Column(1), Operator.Lt, Literal(Float64(0.4))), aggs, AGG | _abi.DFMI_FLAG_EXT_GATHER_ALL)
    run_agg(s, b, None, aggs, batch_rows=20_000)


def test_empty_and_all_filtered():
    s = Schema([Field("x", DataType.Float64, False)])
    aggs = [agg(f, Column(0), s) for f in ("SUM", "MIN", "MAX", "COUNT")]
    b0 = RecordBatch(s, [Array.from_numpy(DataType.Float64, np.zeros(0))])
    v = run_agg(s, b0, None, aggs)
    assert [x.is_null for x in v] == [1, 1, 1, 0]
    b = RecordBatch(s, [Array.from_numpy(DataType.Float64, np.arange(1000.0))])
    v = run_agg(s, b, BinaryExpr(Column(0), Operator.Gt, Literal(Float64(1e9))), aggs)
    assert [x.is_null for x in v] == [1, 1, 1, 0] and v[3].bits == 0


def test_errors_in_reference_order():
    s = Schema([Field("a", DataType.Float64, False), Field("d", DataType.Float64, False), Field("i", DataType.Int64, False)])
    a = np.arange(1000.0)
    d = np.ones(1000)
    d[500] = 0.0
    b = RecordBatch(s, [Array.from_numpy(DataType.Float64, a), Array.from_numpy(DataType.Float64, d),
                        Array.from_numpy(DataType.Int64, np.arange(1000))])
    q = agg("SUM", BinaryExpr(Column(0), Operator.Divide, Column(1)), s)
    fl = AGG | _abi.DFMI_FLAG_EXT_GATHER_ALL
    assert run_agg(s, b, None, [q], fl) is None  # DivideByZero at row 500
    run_agg(s, b, BinaryExpr(Column(0), Operator.Lt, Literal(Float64(400.0))), [q], fl)  # row 500 not selected
    assert run_agg(s, b, BinaryExpr(Column(0), Operator.Gt, Literal(Float64(400.0))), [q], fl) is None
    # the filtered batch holds an Int64 column: "filter not supported for Int64" (filter.rs:106-110)
    assert run_agg(s, b, BinaryExpr(Column(0), Operator.Lt, Literal(Float64(400.0))), [agg("COUNT", Column(0), s)]) is None
    # SUM(i64::MIN / -1) panics
    i = np.arange(1000)
    i[3] = np.iinfo(np.int64).min
    s2 = Schema([Field("i", DataType.Int64, False), Field("m", DataType.Int64, False)])
    b2 = RecordBatch(s2, [Array.from_numpy(DataType.Int64, i), Array.from_numpy(DataType.Int64, -np.ones(1000, np.int64))])
    assert run_agg(s2, b2, None, [agg("SUM", BinaryExpr(Column(0), Operator.Divide, Column(1)), s2)]) is None


def test_partials_merge_bit_identical():
    """Three shards' exact partials merged on the host == one state over all
    rows == the oracle (the multi-GPU reduction of an aggregate)."""
    rng = np.random.default_rng(5)
    n = 240_000
    x = wild_doubles(rng, n)
    s = Schema([Field("x", DataType.Float64, False), Field("y", DataType.Int32, False)])
    y = rng.integers(-2 ** 31, 2 ** 31 - 1, n, dtype=np.int32)
    b = RecordBatch(s, [Array.from_numpy(DataType.Float64, x), Array.from_numpy(DataType.Int32, y)])
    aggs = [agg("SUM", Column(0), s), agg("MIN", Column(0), s), agg("MAX", Column(1), s), agg("SUM", Column(1), s),
            agg("COUNT", Column(0), s)]
    whole = run_agg(s, b, None, aggs)
    cs = [compile_expr(None, a, s, AGG) for a in aggs]
    db = b.to(engine().device)
    parts = []
    for r0, r1 in ((0, 80_000), (80_000, 160_000), (160_000, n)):
        st = engine().agg_state(cs)
        st.add(None, slice_batch(db, r0, r1 - r0), AGG)
        parts.append(st.partial())
    merged = merge_agg_partials(cs, parts)
    for m, w in zip(merged, whole):
        assert (m.bits, m.count, m.is_null) == (w.bits, w.count, w.is_null)


def test_q6_sum_through_sql():
    """SELECT SUM(l_extendedprice * l_discount) FROM lineitem WHERE <Q6> over
    1M rows of the bench's C4 generator (bench.q6_table) in 4 batches,
    through ctx.sql(), against the oracle."""
    import bench
    n = 1 << 20
    s, dcols = bench.q6_table(engine().device, n, 42)
    cols = [c.cpu().numpy() for c in dcols]
    b = RecordBatch(s, [Array.from_numpy(DataType.Float64, c) for c in cols])
    pred, projs = bench.q6_query()
    q = agg("SUM", projs[0], s)
    ref = oracle_aggregate(s, b, pred, [q], AGG)[0]
    db = b.to(engine().device)
    ctx = ExecutionContext(flags=AGG)
    ctx.register_datasource("lineitem", MemoryDataSource(s, [slice_batch(db, r, n // 4) for r in range(0, n, n // 4)]))
    rel = ctx.sql("SELECT SUM(l_extendedprice * l_discount) FROM lineitem WHERE l_shipdate >= 8766 AND "
                  "l_shipdate < 9131 AND l_discount >= 0.05 AND l_discount <= 0.07 AND l_quantity < 24")
    out = rel.next()
    assert rel.next() is None
    assert out.schema.fields[0].name == "SUM" and out.schema.fields[0].data_type == DataType.Float64
    got = out.columns[0].cpu().numpy_values().view(np.uint64)[0]
    assert int(got) == ref.bits
    m = (cols[3] >= 8766) & (cols[3] < 9131) & (cols[2] >= 0.05) & (cols[2] <= 0.07) & (cols[0] < 24)
    assert abs(agg_value_py(ref) - float((cols[1] * cols[2])[m].sum())) < 1e-3


# ---------------------------------------------------------- round-3 fixtures
def test_sql_min_max_fixture_on_gpu():
    """expected/test_sql_min_max.csv on the device, through ctx.sql()."""
    from golden_cases import CITIES, MIN_MAX_SQL, agg_fixture_value, expected_rows, load_batch
    batch = load_batch(CITIES, "uk_cities.csv", has_header=False)
    ctx = ExecutionContext(flags=AGG)
    ctx.register_datasource("uk_cities", MemoryDataSource(CITIES, [batch.to(engine().device)]))
    out = ctx.sql(MIN_MAX_SQL).next()
    got = [int(c.cpu().numpy_values().view(np.uint64)[0]) for c in out.columns]
    want = expected_rows("test_sql_min_max.csv")[0]
    assert got == [agg_fixture_value(w, DataType.Float64) for w in want]


def test_csv_aggregate_all_types_fixture_on_gpu():
    """expected/csv_aggregate_all_types.csv columns 1-10 and the counts on
    the device, bit-identical to the oracle and to the fixture cells."""
    from golden_cases import agg_fixture_value, all_types_typed, load_batch
    from test_oracle_golden import _agg_plan, all_types_aggregates
    s = all_types_typed()
    batch = load_batch(s, "all_types_flat.csv", has_header=False)
    for sql, cells, types in all_types_aggregates():
        dev = run_agg(s, batch, None, _agg_plan(sql, s, "t"))
        assert [d.bits for d in dev] == [agg_fixture_value(c, t) for c, t in zip(cells, types)], sql
        dev = run_agg(s, batch, None, _agg_plan(sql, s, "t"), batch_rows=64)  # many batches


# ------------------------------------------------------- GROUP BY extension
def run_grouped(schema, batch, pred, key, aggs, flags=AGG, batch_rows=0):
    """Device groups and oracle groups (keys and values bit-identical), or
    the same error."""
    from oracle_ffi import oracle_aggregate_grouped
    ref = ref_err = dev = dev_err = None
    try:
        ref = oracle_aggregate_grouped(schema, batch, pred, key, aggs, flags, batch_rows)
    except ExecutionError as e:
        ref_err = e
    try:
        p = compile_scalar_expr(None, pred, schema, flags) if pred is not None else None
        k = compile_scalar_expr(None, key, schema, flags)
        cs = [compile_expr(None, a, schema, flags) for a in aggs]
        st = engine().grouped_agg_state(k, cs)
        n = batch.num_rows()
        step = batch_rows if batch_rows > 0 else max(n, 1)
        dbatch = batch.to(engine().device)
        for r0 in range(0, max(n, 1), step):
            st.add(p, slice_batch(dbatch, r0, min(step, n - r0)) if n else dbatch, flags)
        dev = st.finish()
    except ExecutionError as e:
        dev_err = e
    if ref_err is not None or dev_err is not None:
        assert ref_err is not None and dev_err is not None, (ref_err, dev_err)
        assert (dev_err.kind, dev_err.message) == (ref_err.kind, ref_err.message)
        return None
    (dk, dv), (rk, rv) = dev, ref
    assert [(k.type, k.is_null, k.bits, k.count) for k in dk] == [(k.type, k.is_null, k.bits, k.count) for k in rk]
    if rk and rk[0].type == int(DataType.Utf8):  # the keys' bytes (dfmi_agg_state_group_keys_utf8)
        rs = oracle_aggregate_grouped(schema, batch, pred, key, aggs, flags, batch_rows, key_strings=True)[2]
        assert st.key_strings() == rs
    for g in range(len(rk)):
        for a, d, r in zip(aggs, dv[g], rv[g]):
            assert (d.type, d.is_null, d.count) == (r.type, r.is_null, r.count), (g, repr(a))
            if not r.is_null:
                assert d.bits == r.bits, (g, repr(a), hex(d.bits), hex(r.bits))
    return dev


def test_group_by_c_bool_fixture_on_gpu():
    """expected/csv_aggregate_by_c_bool.csv (MIN/MAX of every numeric column
    per c_bool group) on the device through ctx.sql(), bit-identical to the
    fixture cells and to the oracle; also pulled as 64-row batches."""
    from golden_cases import agg_fixture_value, all_types_typed, load_batch
    from test_oracle_golden import _agg_plan, by_c_bool_aggregates
    s = all_types_typed()
    batch = load_batch(s, "all_types_flat.csv", has_header=False)
    for sql, cells, types in by_c_bool_aggregates():
        (key,), aggs = _agg_plan(sql, s, "t", grouped=True)
        for br in (0, 64):
            keys, vals = run_grouped(s, batch, None, key, aggs, batch_rows=br)
            assert [(k.is_null, k.bits) for k in keys] == [(0, 0), (0, 1)]
            for g in range(2):
                assert [v.bits for v in vals[g]] == [agg_fixture_value(c, t) for c, t in zip(cells[g], types)]
        ctx = ExecutionContext(flags=AGG)
        ctx.register_datasource("t", MemoryDataSource(s, [batch.to(engine().device)]))
        out = ctx.sql(sql).next()
        assert out.columns[0].cpu().to_pylist() == [False, True]
        assert out.schema.fields[0].name == "c0" and len(out.columns) == 11


def test_group_by_random_keys():
    """Boolean / Int8 / UInt64 / Int64 keys with nulls over many batches whose
    key windows differ (device flushes between windows), with a predicate,
    exact float sums, MIN/MAX, COUNT and wrapping integer sums per group."""
    rng = np.random.default_rng(12)
    n = 200_003
    s = Schema([Field("b", DataType.Boolean, True), Field("i8", DataType.Int8, True),
                Field("u64", DataType.UInt64, False), Field("i64", DataType.Int64, True),
                Field("x", DataType.Float64, True), Field("f", DataType.Float32, True), Field("v", DataType.Int32, True)])
    i8 = (rng.integers(-3, 9, n) + (np.arange(n) // 50_000) * 7).astype(np.int8)  # windows move per 50k rows
    cols = [Array.from_numpy(DataType.Boolean, rng.random(n) < 0.4, rng.random(n) >= 0.05),
            Array.from_numpy(DataType.Int8, i8, rng.random(n) >= 0.02),
            Array.from_numpy(DataType.UInt64, (np.uint64(2 ** 64 - 9) + rng.integers(0, 6, n).astype(np.uint64))),
            Array.from_numpy(DataType.Int64, rng.integers(-8, 7, n).astype(np.int64), rng.random(n) >= 0.1),
            Array.from_numpy(DataType.Float64, wild_doubles(rng, n), rng.random(n) >= 0.1),
            Array.from_numpy(DataType.Float32, rng.standard_normal(n).astype(np.float32), rng.random(n) >= 0.1),
            Array.from_numpy(DataType.Int32, rng.integers(-2 ** 31, 2 ** 31 - 1, n).astype(np.int32))]
    b = RecordBatch(s, cols)
    aggs = [agg("SUM", Column(4), s), agg("MIN", Column(5), s), agg("MAX", Column(5), s), agg("COUNT", Column(4), s),
            agg("SUM", Column(6), s), agg("MAX", Column(3), s)]
    pred = BinaryExpr(Column(4), Operator.Lt, Literal(Float64(0.8)))
    # a Selection over a batch with a Boolean column needs the gather
    # extension (filter.rs:106-110 rejects it otherwise: checked as well)
    assert run_grouped(s, b, pred, Column(0), aggs) is None
    for c in range(4):
        for p in (None, pred):
            for br in ((25_000,) if c == 1 else (0, 25_000)):  # Int8: 16-value windows per 50k rows
                out = run_grouped(s, b, p, Column(c), aggs, AGG | _abi.DFMI_FLAG_EXT_GATHER_ALL, batch_rows=br)
                assert out is not None and len(out[0]) >= 2


def test_group_by_errors():
    """A batch whose selected keys span more than the device's 16-value window
    is merged on the host (aggregate.cpp group_batch_on_host) with the
    kernel's rules: the oracle's groups; an error in the key expression is
    raised by both, before any aggregate's, in the reference's evaluation
    order -- in the window path and in the wide one."""
    n = 4096
    s = Schema([Field("k", DataType.Int64, False), Field("d", DataType.Int64, False), Field("x", DataType.Float64, False)])
    k = np.arange(n, dtype=np.int64) % 40
    d = np.ones(n, dtype=np.int64)
    d[1000] = 0
    b = RecordBatch(s, [Array.from_numpy(DataType.Int64, k), Array.from_numpy(DataType.Int64, d),
                        Array.from_numpy(DataType.Float64, np.arange(n, dtype=np.float64))])
    out = run_grouped(s, b, None, Column(0), [agg("SUM", Column(2), s), agg("MIN", Column(1), s)])
    assert out is not None and len(out[0]) == 40
    # key = k / d: DivideByZero at row 1000, before the aggregate's own error
    key = BinaryExpr(Column(0), Operator.Divide, Column(1))
    bad = [agg("SUM", BinaryExpr(Column(2), Operator.Divide, Literal(Float64(0.0))), s)]
    pred = BinaryExpr(Column(0), Operator.Lt, Literal(Int64(10)))
    run_grouped(s, b, pred, key, bad)
    run_grouped(s, b, pred, Column(0), bad)
    wide = BinaryExpr(Column(0), Operator.Lt, Literal(Int64(30)))  # 30 key values: the host merge
    assert run_grouped(s, b, wide, key, bad) is None
    assert run_grouped(s, b, wide, Column(0), bad) is None


@pytest.mark.parametrize("batch_rows", [0, 7000])
def test_group_by_random_keys_wide(batch_rows):
    """10,000 distinct Int64 keys (and Int32 / UInt16 keys spanning thousands
    of values), nullable keys and arguments, with and without a predicate,
    over one batch or many: every batch is wider than the device window, so
    every row goes through the host merge -- bit-exact against the oracle:
    exact float SUM, MIN/MAX (NaN, -0.0), COUNT, wrapping integer SUM, and
    the per-group row counts."""
    rng = np.random.default_rng(21)
    n = 60_001
    s = Schema([Field("k64", DataType.Int64, True), Field("k32", DataType.Int32, False),
                Field("ku16", DataType.UInt16, False), Field("x", DataType.Float64, True),
                Field("f", DataType.Float32, True), Field("v", DataType.Int64, True)])
    keys = rng.integers(-5000, 5000, n).astype(np.int64)
    cols = [Array.from_numpy(DataType.Int64, keys, rng.random(n) >= 0.01),
            Array.from_numpy(DataType.Int32, rng.integers(-2 ** 31, 2 ** 31 - 1, n).astype(np.int32) // 1_000_000),
            Array.from_numpy(DataType.UInt16, rng.integers(0, 65535, n).astype(np.uint16)),
            Array.from_numpy(DataType.Float64, wild_doubles(rng, n), rng.random(n) >= 0.1),
            Array.from_numpy(DataType.Float32, rng.standard_normal(n).astype(np.float32), rng.random(n) >= 0.1),
            Array.from_numpy(DataType.Int64, rng.integers(-2 ** 62, 2 ** 62, n).astype(np.int64), rng.random(n) >= 0.1)]
    b = RecordBatch(s, cols)
    aggs = [agg("SUM", Column(3), s), agg("MIN", Column(3), s), agg("MAX", Column(4), s), agg("COUNT", Column(3), s),
            agg("SUM", Column(5), s), agg("SUM", Column(4), s)]
    pred = BinaryExpr(Column(3), Operator.Lt, Literal(Float64(0.8)))
    fl = AGG | _abi.DFMI_FLAG_EXT_GATHER_ALL
    for c in range(3):
        for p in (None, pred):
            out = run_grouped(s, b, p, Column(c), aggs, fl, batch_rows=batch_rows)
            assert out is not None and len(out[0]) > 1000


def _nan(bits):
    return np.array([bits], np.uint64).view(np.float64)[0]


@pytest.mark.parametrize("batch_rows", [0, 7_001])
def test_group_by_float64_keys(batch_rows):
    """10,000 distinct Float64 keys plus -0.0 / +0.0, +-inf and NaNs of several
    payloads and signs (one group per bit pattern, IEEE 754 totalOrder, the
    null key last; build-defined, parity unpinned), with and without a
    predicate, over one batch or many -- keys, per-group row counts and every
    aggregate bit-exact against the oracle."""
    rng = np.random.default_rng(51)
    n = 50_003
    pool = np.concatenate([rng.standard_normal(10_000) * 1e3,
                           [0.0, -0.0, np.inf, -np.inf, _nan(0x7FF8000000000000), _nan(0xFFF8000000000000),
                            _nan(0x7FF0000000000001), _nan(0x7FF8DEADBEEF0000)]])
    k = pool[rng.integers(0, len(pool), n)]
    s = Schema([Field("k", DataType.Float64, True), Field("x", DataType.Float64, True), Field("v", DataType.Int64, True)])
    b = RecordBatch(s, [Array.from_numpy(DataType.Float64, k, rng.random(n) >= 0.02),
                        Array.from_numpy(DataType.Float64, wild_doubles(rng, n), rng.random(n) >= 0.1),
                        Array.from_numpy(DataType.Int64, rng.integers(-2 ** 40, 2 ** 40, n), rng.random(n) >= 0.1)])
    aggs = [agg("SUM", Column(1), s), agg("MIN", Column(1), s), agg("MAX", Column(2), s), agg("COUNT", Column(1), s),
            agg("SUM", Column(2), s)]
    fl = AGG | _abi.DFMI_FLAG_EXT_GATHER_ALL
    pred = BinaryExpr(Column(1), Operator.Lt, Literal(Float64(0.5)))
    for p in (None, pred):
        out = run_grouped(s, b, p, Column(0), aggs, fl, batch_rows=batch_rows)
        assert out is not None and len(out[0]) > 5000


def test_group_by_float32_key_and_expression_key():
    """A Float32 key column and a Float64-valued key expression."""
    rng = np.random.default_rng(52)
    n = 20_011
    s = Schema([Field("f", DataType.Float32, True), Field("x", DataType.Float64, False)])
    f = (rng.integers(-300, 300, n) / 8).astype(np.float32)
    f[::97] = -0.0
    b = RecordBatch(s, [Array.from_numpy(DataType.Float32, f, rng.random(n) >= 0.05),
                        Array.from_numpy(DataType.Float64, rng.random(n))])
    aggs = [agg("COUNT", Column(1), s), agg("SUM", Column(1), s)]
    fl = AGG | _abi.DFMI_FLAG_EXT_GATHER_ALL
    assert run_grouped(s, b, None, Column(0), aggs, fl) is not None
    key = BinaryExpr(Column(1), Operator.Multiply, Literal(Float64(16.0)))  # a computed key
    assert run_grouped(s, b, BinaryExpr(Column(1), Operator.Gt, Literal(Float64(0.9))), key, aggs, fl) is not None


@pytest.mark.parametrize("batch_rows", [0, 4_099])
def test_group_by_utf8_keys(batch_rows):
    """1,000 distinct Utf8 keys (empty, multi-byte UTF-8, bytes >= 0x80,
    prefixes of each other), a nullable key column, with and without a
    predicate, one batch or many: keys (bytewise order, null last), their
    bytes, row counts and aggregates bit-exact against the oracle."""
    rng = np.random.default_rng(53)
    n = 40_009
    words = [bytes(rng.integers(97, 123, int(rng.integers(0, 12))).astype(np.uint8)) for _ in range(990)]
    words += [b"", b"a", b"ab", b"abc", "\u20ac".encode(), "\u20acx".encode(), b"\xff", b"\xfe\xff", b"w17", b"w1"]
    keys = [words[i] for i in rng.integers(0, len(words), n)]
    kv = [None if rng.random() < 0.03 else x for x in keys]
    s = Schema([Field("s", DataType.Utf8, True), Field("x", DataType.Float64, True)])
    b = RecordBatch(s, [Array.from_strings(kv), Array.from_numpy(DataType.Float64, wild_doubles(rng, n),
                                                                  rng.random(n) >= 0.1)])
    aggs = [agg("COUNT", Column(1), s), agg("SUM", Column(1), s), agg("MIN", Column(1), s), agg("MAX", Column(1), s)]
    fl = AGG | _abi.DFMI_FLAG_EXT_GATHER_ALL
    for p in (None, BinaryExpr(Column(1), Operator.Lt, Literal(Float64(0.3)))):
        out = run_grouped(s, b, p, Column(0), aggs, fl, batch_rows=batch_rows)
        assert out is not None and len(out[0]) > 500


def test_group_by_utf8_key_through_sql():
    """SELECT s, COUNT(x), SUM(x) FROM t WHERE x > 0.2 GROUP BY s through
    ctx.sql: the AggregateRelation's key column is a Utf8 array in key order."""
    from datafusion_amd.execution import ExecutionContext, MemoryDataSource
    from oracle_ffi import oracle_aggregate_grouped
    rng = np.random.default_rng(54)
    n = 10_000
    words = [b"pear", b"apple", b"fig", b"", b"banana"]
    st = [words[i] for i in rng.integers(0, len(words), n)]
    s = Schema([Field("s", DataType.Utf8, False), Field("x", DataType.Float64, False)])
    x = rng.random(n)
    b = RecordBatch(s, [Array.from_strings(st), Array.from_numpy(DataType.Float64, x)])
    ctx = ExecutionContext(flags=AGG | _abi.DFMI_FLAG_EXT_GATHER_ALL)
    ctx.register_datasource("t", MemoryDataSource(s, [b.to(engine().device)]))
    (rb,) = list(ctx.sql("SELECT s, COUNT(x), SUM(x) FROM t WHERE x > 0.2 GROUP BY s"))
    assert rb.columns[0].to_pylist() == ["", "apple", "banana", "fig", "pear"]
    pred = BinaryExpr(Column(1), Operator.Gt, Literal(Float64(0.2)))
    rk, rv, rs = oracle_aggregate_grouped(s, b, pred, Column(0), [agg("COUNT", Column(1), s), agg("SUM", Column(1), s)],
                                          AGG | _abi.DFMI_FLAG_EXT_GATHER_ALL, key_strings=True)
    assert rs == [w.encode() if isinstance(w, str) else w for w in rb.columns[0].to_pylist()]
    assert rb.columns[1].to_pylist() == [v[0].bits for v in rv]
    assert [int(np.array([y], np.float64).view(np.uint64)[0]) for y in rb.columns[2].to_pylist()] == \
        [v[1].bits for v in rv]
