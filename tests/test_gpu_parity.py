"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on the
same inputs. Bit-exact for masks, integers, Utf8 and comparisons; Float64 and
Float32 bit-exact too (one rounding per operator on both sides,
-ffp-contract=off), NaN payloads included: both sides follow the x86 NaN
rules the reference's scalar loops produce (DESIGN.md "Semantics")."""
import os

import numpy as np
import pytest
import torch

from datafusion_amd._abi import DFMI_FLAG_EXT_GATHER_ALL, DFMI_FLAG_EXT_UTF8_COMPARE
from datafusion_amd.arrow import Array, Field, RecordBatch, Schema
from datafusion_amd.execution import ExecutionContext, MemoryDataSource
from datafusion_amd.execution.engine import engine
from datafusion_amd.execution.error import ExecutionError
from datafusion_amd.execution.expression import compile_scalar_expr
from datafusion_amd.logicalplan import (BinaryExpr, Cast, Column, DataType, Float64, Int64, Literal, Operator,
                                        Utf8, binary_expr_coerced)
from golden_cases import CITIES, GOLDEN, NUMERICS, all_types_schema, expected_rows, load_batch, lit_expr
from oracle_ffi import gen_i64, gen_unit_f64, oracle_filter_project

pytestmark = pytest.mark.gpu

HOST_CHUNK = 512  # rows per pipelined chunk in run_both's second host-path call

CMP = [Operator.Eq, Operator.NotEq, Operator.Lt, Operator.LtEq, Operator.Gt, Operator.GtEq]
MATH = [Operator.Plus, Operator.Minus, Operator.Multiply, Operator.Divide]


def assert_same(dev: Array, ref: Array, what=""):
    assert dev.data_type == ref.data_type, what
    assert dev.length == ref.length, (what, dev.length, ref.length)
    assert dev.null_count == ref.null_count, (what, dev.null_count, ref.null_count)
    n = ref.length
    if ref.null_count:
        assert np.array_equal(dev.valid_mask(), ref.valid_mask()), what
    dv, rv = dev.numpy_values(), ref.numpy_values()
    if ref.data_type == DataType.Utf8:
        assert dv == rv, what
        return
    if ref.data_type == DataType.Boolean:
        assert np.array_equal(dv, rv), what
        return
    if ref.data_type in (DataType.Float64, DataType.Float32):
        # bit for bit, NaN payloads included (x86 NaN rules)
        ib = dv.view(np.uint64 if ref.data_type == DataType.Float64 else np.uint32)
        rb = rv.view(np.uint64 if ref.data_type == DataType.Float64 else np.uint32)
        if ref.null_count:  # null slots hold no value the reference defines
            m = ref.valid_mask()
            ib, rb = ib[m], rb[m]
        assert np.array_equal(ib, rb), (what, np.flatnonzero(ib != rb)[:5])
        return
    assert np.array_equal(dv, rv), what


def run_both(schema, batch, pred, projs, flags=0):
    """Device result (list of Arrays) and oracle result, or the two errors."""
    ref_err = dev_err = None
    try:
        ref = oracle_filter_project(schema, batch, pred, projs, flags)
    except ExecutionError as e:
        ref_err = e
    host_err = host = None
    try:
        p = compile_scalar_expr(None, pred, schema, flags) if pred is not None else None
        cp = [compile_scalar_expr(None, e, schema, flags) for e in projs]
        names = [c.get_name() for c in cp] if cp else [f.name for f in schema.fields]
        try:
            # host-buffer entry point (dfmi_filter_project_host): staged H2D + D2H
            host = engine().filter_project_host(p, cp, batch, flags)
        except ExecutionError as e:
            host_err = e
        if batch.num_rows() > HOST_CHUNK:
            # ... and again cut into pipelined chunks (HOST_CHUNK rows, or ~16
            # chunks for big batches): the same result or the same first error
            # (evaluation order over all rows)
            chunk = max(HOST_CHUNK, (batch.num_rows() // 16) // 512 * 512)
            prev = os.environ.get("DFMI_HOST_CHUNK_ROWS")
            os.environ["DFMI_HOST_CHUNK_ROWS"] = str(chunk)
            try:
                try:
                    chunked = engine().filter_project_host(p, cp, batch, flags)
                    cerr = None
                except ExecutionError as e:
                    chunked, cerr = None, e
            finally:
                if prev is None:
                    del os.environ["DFMI_HOST_CHUNK_ROWS"]
                else:
                    os.environ["DFMI_HOST_CHUNK_ROWS"] = prev
            if host_err is not None:
                assert cerr is not None and (cerr.kind, cerr.message) == (host_err.kind, host_err.message), cerr
            else:
                assert cerr is None, cerr
                for h, c in zip(host, chunked):
                    assert_same(c, h, "chunked host path")
        dev = engine().filter_project(p, cp, batch, flags)
    except ExecutionError as e:
        dev_err = e
    if ref_err is not None or dev_err is not None:
        assert ref_err is not None and dev_err is not None, (ref_err, dev_err)
        assert (dev_err.kind, dev_err.message) == (ref_err.kind, ref_err.message)
        if host_err is not None or host is not None:
            assert host_err is not None and (host_err.kind, host_err.message) == (ref_err.kind, ref_err.message)
        return None
    assert host_err is None, host_err
    assert len(dev) == len(ref) == len(host)
    for i, ((rname, r), d, h) in enumerate(zip(ref, dev, host)):
        assert names[i] == rname
        assert_same(d.cpu(), r, "%s col %d" % (rname, i))
        assert_same(h, r, "host path: %s col %d" % (rname, i))
    return dev, ref


def synth(n, seed=42, nullable=False, int64=False, null_frac=0.1):
    """a, b, c columns: Float64 in [0,1) or Int64 in [-2^20, 2^20)."""
    cols = []
    fields = []
    rng = np.random.default_rng(seed)
    for j, name in enumerate("abc"):
        if int64:
            v = gen_i64(seed, j, 0, n, -(1 << 20), 1 << 20)
            t = DataType.Int64
        else:
            v = gen_unit_f64(seed, j, 0, n)
            t = DataType.Float64
        valid = (rng.random(n) >= null_frac) if nullable else None
        cols.append(Array.from_numpy(t, v, valid))
        fields.append(Field(name, t, nullable))
    s = Schema(fields)
    return s, RecordBatch(s, cols)


# ------------------------------------------------------------ known answers
def test_csv_sql_example_on_gpu():
    """examples/csv_sql.rs:56 through ExecutionContext.sql on the device."""
    ctx = ExecutionContext()
    batch = load_batch(CITIES, "uk_cities.csv", has_header=True)
    ctx.register_datasource("cities", MemoryDataSource(CITIES, [batch]))
    rel = ctx.sql("SELECT city, lat, lng, lat + lng FROM cities WHERE lat > 51.0 AND lat < 53")
    b = rel.next()
    assert b.num_rows() == 18 and b.num_columns() == 4
    assert [f.name for f in b.schema.fields] == ["city", "lat", "lng", "#1 Plus #2"]
    city, lat, lng, comb = [c.cpu().to_pylist() for c in b.columns]
    assert (city[0], lat[0], lng[0], comb[0]) == ("Solihull, Birmingham, UK", 52.412811, -1.778197, 50.634614)
    assert repr(comb[city.index("Oxford, Oxfordshire, UK")]) == "50.494344999999996"
    assert rel.next() is None
    pred = lit_expr(CITIES, 1, Operator.Gt, Float64(51.0))
    run_both(CITIES, batch, BinaryExpr(pred, Operator.And, lit_expr(CITIES, 1, Operator.Lt, Int64(53))),
             [Column(0), Column(1), Column(2), BinaryExpr(Column(1), Operator.Plus, Column(2))])


def test_filter_fixture_on_gpu():
    batch = load_batch(CITIES, "uk_cities.csv", has_header=False)
    exp = [ln.rsplit(",", 2) for ln in open(GOLDEN + "/expected/test_filter.csv", encoding="utf-8").read().splitlines() if ln]
    res = run_both(CITIES, batch, lit_expr(CITIES, 1, Operator.Gt, Float64(52.0)), [])
    city, lat, lng = [c.cpu().to_pylist() for c in res[0]]
    assert [[c, repr(a), repr(b)] for c, a, b in zip(city, lat, lng)] == [[e[0], repr(float(e[1])), repr(float(e[2]))] for e in exp]


@pytest.mark.parametrize("fname,op", [("c_float64_high.csv", Operator.Gt), ("c_float64_low.csv", Operator.Lt)])
def test_all_types_float64_on_gpu(fname, op):
    s = all_types_schema(f64_col=10)
    batch = load_batch(s, "all_types_flat.csv", has_header=False)
    dev, _ = run_both(s, batch, lit_expr(s, 10, op, Float64(0.5)), [Column(10)])
    assert dev[0].cpu().to_pylist() == [float(r[0]) for r in expected_rows(fname)]
    run_both(s, batch, lit_expr(s, 10, op, Float64(0.5)), [])  # FilterRelation output, 11 Utf8 gathers


@pytest.mark.parametrize("fname,op", [("c_int64_positive.csv", Operator.Gt), ("c_int64_negative.csv", Operator.Lt)])
def test_all_types_int64_on_gpu(fname, op):
    s = all_types_schema(i64_col=8)
    batch = load_batch(s, "all_types_flat.csv", has_header=False)
    pred = lit_expr(s, 8, op, Int64(0))
    assert run_both(s, batch, pred, [Column(8)]) is None  # "filter not supported for Int64"
    dev, _ = run_both(s, batch, pred, [Column(8)], DFMI_FLAG_EXT_GATHER_ALL)
    assert dev[0].cpu().to_pylist() == [int(r[0]) for r in expected_rows(fname)]


@pytest.mark.parametrize("op", MATH)
def test_numerics_on_gpu(op):
    batch = load_batch(NUMERICS, "numerics.csv", has_header=True)
    S = NUMERICS
    exprs = [binary_expr_coerced(Column(0), op, Column(1), S), binary_expr_coerced(Column(0), op, Literal(Int64(2)), S),
             binary_expr_coerced(Column(2), op, Column(3), S), binary_expr_coerced(Column(2), op, Literal(Int64(2)), S),
             binary_expr_coerced(Column(2), op, Literal(Float64(2.5)), S)]
    run_both(S, batch, None, exprs)
    run_both(S, batch, lit_expr(S, 2, Operator.GtEq, Float64(2.5)), exprs[2:], 0)


# ------------------------------------------------------------ synthetic
@pytest.mark.parametrize("n", [0, 1, 63, 64, 1000, 1024, 4097, 1 << 20, 1_000_003])
@pytest.mark.parametrize("sel", [0.01, 0.5, 0.99])
def test_c2_float64(n, sel):
    s, batch = synth(n)
    k, m = 1 - sel ** 0.5, sel ** 0.5
    pred = BinaryExpr(BinaryExpr(Column(0), Operator.Gt, Literal(Float64(k))), Operator.And,
                      BinaryExpr(Column(1), Operator.Lt, Literal(Float64(m))))
    proj = [Column(0), Column(1),
            BinaryExpr(BinaryExpr(Column(0), Operator.Multiply, Column(1)), Operator.Plus, Column(2))]
    res = run_both(s, batch, pred, proj)
    if n >= 1 << 20:
        got = res[0][0].length / n
        assert abs(got - sel) < 0.01


@pytest.mark.parametrize("n", [1000, 1_000_003])
def test_c2_int64(n):
    s, batch = synth(n, int64=True)
    pred = BinaryExpr(BinaryExpr(Column(0), Operator.Gt, Literal(Int64(-1000))), Operator.And,
                      BinaryExpr(Column(1), Operator.Lt, Literal(Int64(5000))))
    proj = [Column(0), Column(1),
            BinaryExpr(BinaryExpr(Column(0), Operator.Multiply, Column(1)), Operator.Plus, Column(2))]
    assert run_both(s, batch, pred, proj) is None  # Int64 gather is an extension
    run_both(s, batch, pred, proj, DFMI_FLAG_EXT_GATHER_ALL)


@pytest.mark.parametrize("op", CMP)
@pytest.mark.parametrize("int64", [False, True])
def test_nullable_comparisons(op, int64):
    """arrow 0.12 bool_op null ordering (parity unpinned: restated)."""
    n = 5000
    s, batch = synth(n, seed=7, nullable=True, int64=int64, null_frac=0.3)
    lit = Int64(0) if int64 else Float64(0.5)
    flags = DFMI_FLAG_EXT_GATHER_ALL
    run_both(s, batch, BinaryExpr(Column(0), op, Column(1)), [Column(0), Column(2)], flags)
    run_both(s, batch, BinaryExpr(Column(0), op, Literal(lit)), [Column(1)], flags)
    run_both(s, batch, BinaryExpr(Literal(lit), op, Column(1)), [Column(0)], flags)
    # comparison outputs (Boolean) in the select list, with and without a filter
    run_both(s, batch, None, [BinaryExpr(Column(0), op, Column(1))], flags)
    run_both(s, batch, BinaryExpr(Column(2), Operator.Gt, Literal(lit)), [BinaryExpr(Column(0), op, Column(1))], flags)


@pytest.mark.parametrize("op", MATH)
@pytest.mark.parametrize("int64", [False, True])
def test_nullable_math(op, int64):
    n = 3000
    s, batch = synth(n, seed=11, nullable=True, int64=int64, null_frac=0.2)
    flags = DFMI_FLAG_EXT_GATHER_ALL
    if op == Operator.Divide and int64:
        # make divisors non-zero to test values (zero divisors tested below)
        return
    # projection only: null propagation + validity bitmap + null counts
    run_both(s, batch, None, [BinaryExpr(Column(0), op, Column(1)), BinaryExpr(Column(2), op, Column(0))], flags)
    # in the predicate (nulls propagate, then compare)
    lit = Int64(0) if int64 else Float64(0.5)
    run_both(s, batch, BinaryExpr(BinaryExpr(Column(0), op, Column(1)), Operator.Lt, Literal(lit)),
             [Column(2), BinaryExpr(Column(0), op, Column(1))], flags)


def test_boolean_columns_and_or():
    n = 4000
    rng = np.random.default_rng(3)
    f1 = Array.from_numpy(DataType.Boolean, rng.random(n) < 0.5, rng.random(n) < 0.8)
    f2 = Array.from_numpy(DataType.Boolean, rng.random(n) < 0.5, rng.random(n) < 0.8)
    x = Array.from_numpy(DataType.Float64, gen_unit_f64(5, 0, 0, n))
    s = Schema([Field("f1", DataType.Boolean, True), Field("f2", DataType.Boolean, True), Field("x", DataType.Float64, False)])
    b = RecordBatch(s, [f1, f2, x])
    for op in (Operator.And, Operator.Or):
        # WHERE on a Boolean expression with nulls (null -> value bit 0 -> not selected)
        run_both(s, b, BinaryExpr(Column(0), op, Column(1)), [Column(2)])
        run_both(s, b, None, [BinaryExpr(Column(0), op, Column(1))])
        run_both(s, b, None, [BinaryExpr(Column(0), op, BinaryExpr(Column(2), Operator.Gt, Literal(Float64(0.3))))])
    run_both(s, b, Column(0), [Column(2)])  # WHERE f1: raw value bits
    run_both(s, b, Column(0), [Column(2)], DFMI_FLAG_EXT_GATHER_ALL)
    run_both(s, b, Column(0), [], DFMI_FLAG_EXT_GATHER_ALL)


def test_divide_by_zero_and_overflow():
    n = 2000
    a = np.arange(n, dtype=np.int64) - 1000
    d = np.ones(n, dtype=np.int64)
    d[1500] = 0
    s = Schema([Field("a", DataType.Int64, False), Field("d", DataType.Int64, False),
                Field("x", DataType.Float64, False), Field("y", DataType.Float64, False)])
    x = gen_unit_f64(1, 0, 0, n)
    y = gen_unit_f64(1, 1, 0, n)
    y[700] = -0.0
    b = RecordBatch(s, [Array.from_numpy(DataType.Int64, a), Array.from_numpy(DataType.Int64, d),
                        Array.from_numpy(DataType.Float64, x), Array.from_numpy(DataType.Float64, y)])
    fl = DFMI_FLAG_EXT_GATHER_ALL
    assert run_both(s, b, None, [BinaryExpr(Column(0), Operator.Divide, Column(1))], fl) is None
    assert run_both(s, b, None, [BinaryExpr(Column(2), Operator.Divide, Column(3))], fl) is None
    # the zero divisor row is filtered out -> no error in the projection
    run_both(s, b, BinaryExpr(Column(0), Operator.Lt, Literal(Int64(400))),
             [BinaryExpr(Column(0), Operator.Divide, Column(1)), BinaryExpr(Column(2), Operator.Divide, Column(3))], fl)
    # ... but the predicate sees every row
    assert run_both(s, b, BinaryExpr(BinaryExpr(Column(0), Operator.Divide, Column(1)), Operator.Lt,
                                     Literal(Int64(400))), [Column(2)], fl) is None
    # i64::MIN / -1 panics in the reference
    a2 = a.copy()
    a2[10] = np.iinfo(np.int64).min
    d2 = d.copy()
    d2[10] = -1
    b2 = RecordBatch(s, [Array.from_numpy(DataType.Int64, a2), Array.from_numpy(DataType.Int64, d2), b.columns[2], b.columns[3]])
    assert run_both(s, b2, None, [BinaryExpr(Column(0), Operator.Divide, Column(1))], fl) is None
    # first failing operator wins: static comparison_ops after a dynamic DivideByZero
    e = BinaryExpr(BinaryExpr(BinaryExpr(Column(2), Operator.Divide, Column(3)), Operator.Gt, Literal(Float64(1.0))),
                   Operator.And, BinaryExpr(Column(0), Operator.Gt, Column(2)))
    assert run_both(s, b, e, [Column(2)], fl) is None
    e2 = BinaryExpr(BinaryExpr(Column(0), Operator.Gt, Column(2)), Operator.And,
                    BinaryExpr(BinaryExpr(Column(2), Operator.Divide, Column(3)), Operator.Gt, Literal(Float64(1.0))))
    assert run_both(s, b, e2, [Column(2)], fl) is None


def test_utf8_gather_and_equality():
    n = 5000
    rng = np.random.default_rng(9)
    words = [b"", b"w17", b"alpha", b"w1", b"\xe2\x82\xac uro", b"x" * 40]
    strs = [words[i] for i in rng.integers(0, len(words), n)]
    sv = [None if rng.random() < 0.1 else x for x in strs]
    s = Schema([Field("s", DataType.Utf8, True), Field("v", DataType.Float64, True), Field("t", DataType.Utf8, False)])
    b = RecordBatch(s, [Array.from_strings(sv), Array.from_numpy(DataType.Float64, gen_unit_f64(2, 0, 0, n)),
                        Array.from_strings(strs[::-1])])
    run_both(s, b, BinaryExpr(Column(1), Operator.Lt, Literal(Float64(0.3))), [Column(0), Column(2), Column(1)])
    run_both(s, b, BinaryExpr(Column(1), Operator.Lt, Literal(Float64(0.3))), [])
    # Utf8 equality is an extension (the reference rejects Utf8 literals)
    pred = BinaryExpr(Column(0), Operator.Eq, Literal(Utf8("w17")))
    assert run_both(s, b, pred, [Column(0)]) is None
    for op in (Operator.Eq, Operator.NotEq):
        run_both(s, b, BinaryExpr(Column(0), op, Literal(Utf8("w17"))), [Column(0), Column(1)], DFMI_FLAG_EXT_UTF8_COMPARE)
        run_both(s, b, BinaryExpr(Column(0), op, Column(2)), [Column(2)], DFMI_FLAG_EXT_UTF8_COMPARE)


def test_utf8_many_tiles():
    """Utf8 gather / equality over ~74 tiles: the packed rows+bytes look-back
    word, aligned-word copies at every source/destination alignment, strings
    longer than one 32-byte copy chunk, empty strings and nulls."""
    n = 300_001
    rng = np.random.default_rng(31)
    words = [bytes(rng.integers(97, 123, int(rng.integers(0, 70))).astype(np.uint8)) for _ in range(300)]
    words[7] = b"w7"
    idx = rng.integers(0, len(words), n)
    strs = [words[i] for i in idx]
    sv = [None if rng.random() < 0.05 else x for x in strs]
    s = Schema([Field("s", DataType.Utf8, True), Field("v", DataType.Float64, True)])
    v = gen_unit_f64(5, 0, 0, n)
    b = RecordBatch(s, [Array.from_strings(sv), Array.from_numpy(DataType.Float64, v, rng.random(n) >= 0.1)])
    for k in (0.01, 0.3, 0.97):
        run_both(s, b, BinaryExpr(Column(1), Operator.Lt, Literal(Float64(k))), [Column(0), Column(1)])
    for w in ("w7", words[3].decode()):
        run_both(s, b, BinaryExpr(Column(0), Operator.Eq, Literal(Utf8(w))), [Column(0), Column(1)],
                 DFMI_FLAG_EXT_UTF8_COMPARE)


def test_utf8_multi_channel_many_tiles():
    """Three Utf8 outputs (one look-back channel each, plus rows) over ~100
    tiles: short dictionary words (LDS-staged slices), long strings (slices
    whose source span exceeds the 2 KiB stage: per-lane copy), a string longer
    than the stage itself, empty strings and nulls; equality predicates on a
    nullable column with the offsets shared by predicate and gather."""
    n = 400_003
    rng = np.random.default_rng(77)
    short = [bytes(rng.integers(97, 123, int(rng.integers(0, 25))).astype(np.uint8)) for _ in range(1000)]
    short[17] = b"w17dizjxms"
    longw = [bytes(rng.integers(32, 127, int(rng.integers(20, 300))).astype(np.uint8)) for _ in range(50)]
    longw[3] = b"L" * 5000
    s0 = [short[i] for i in rng.integers(0, len(short), n)]
    s0v = [None if rng.random() < 0.07 else x for x in s0]
    s1 = [longw[i] if rng.random() < 0.3 else short[j] for i, j in zip(rng.integers(0, len(longw), n),
                                                                         rng.integers(0, len(short), n))]
    s2 = [short[i] for i in rng.integers(0, len(short), n)]
    v = gen_unit_f64(8, 0, 0, n)
    s = Schema([Field("a", DataType.Utf8, True), Field("b", DataType.Utf8, False), Field("c", DataType.Utf8, False),
                Field("v", DataType.Float64, True)])
    b = RecordBatch(s, [Array.from_strings(s0v), Array.from_strings(s1), Array.from_strings(s2),
                        Array.from_numpy(DataType.Float64, v, rng.random(n) >= 0.1)])
    for k in (0.002, 0.5, 0.99):
        run_both(s, b, BinaryExpr(Column(3), Operator.Lt, Literal(Float64(k))), [Column(0), Column(1), Column(2), Column(3)])
    run_both(s, b, BinaryExpr(Column(3), Operator.Lt, Literal(Float64(0.6))), [Column(2), Column(0)])
    for w, c in (("w17dizjxms", 0), (short[5].decode(), 2), ("", 0)):
        run_both(s, b, BinaryExpr(Column(c), Operator.Eq, Literal(Utf8(w))), [Column(1), Column(0), Column(3)],
                 DFMI_FLAG_EXT_UTF8_COMPARE)
        run_both(s, b, BinaryExpr(Column(c), Operator.NotEq, Literal(Utf8(w))), [Column(c)], DFMI_FLAG_EXT_UTF8_COMPARE)


def test_utf8_ring_gather(monkeypatch):
    """The ring-staged gather (Launch::ring, forced by DFMI_UTF8_RING=1; by
    default chosen after a large batch of the same query selected >= 15% with
    short strings): one loader wave streams 256-row steps of source bytes into
    an LDS ring, the block stores each step's output image. Short strings
    (every step staged), longer ones (steps over a slot: per-lane copies),
    a string longer than a whole slot, empty strings and nulls, selectivities
    from 1% to 97%, and a source buffer at an odd address -- all against the
    oracle; plus the Utf8 cases above."""
    monkeypatch.setenv("DFMI_DIAG", "1")
    monkeypatch.setenv("DFMI_UTF8_RING", "1")
    n = 300_001
    rng = np.random.default_rng(41)
    short = [bytes(rng.integers(97, 123, int(rng.integers(0, 25))).astype(np.uint8)) for _ in range(500)]
    strs = [short[i] for i in rng.integers(0, len(short), n)]
    for i in range(0, n, 7919):  # a few long strings: their steps exceed a slot
        strs[i] = bytes(rng.integers(32, 127, int(rng.integers(100, 400))).astype(np.uint8))
    strs[150_000] = b"L" * 6000  # longer than a slot by itself
    sv = [None if rng.random() < 0.05 else x for x in strs]
    s = Schema([Field("s", DataType.Utf8, True), Field("v", DataType.Float64, True)])
    v = gen_unit_f64(6, 0, 0, n)
    b = RecordBatch(s, [Array.from_strings(sv), Array.from_numpy(DataType.Float64, v, rng.random(n) >= 0.1)])
    for k in (0.01, 0.3, 0.6, 0.97):
        run_both(s, b, BinaryExpr(Column(1), Operator.Lt, Literal(Float64(k))), [Column(0), Column(1)])
        run_both(s, b, BinaryExpr(Column(1), Operator.Lt, Literal(Float64(k))), [Column(1), Column(0)])
    # the source bytes at an odd address (16-byte chunk staging from a misaligned base)
    import torch
    dev = engine().device
    a = b.columns[0]
    raw = torch.zeros(a.values.numel() + 64, dtype=torch.uint8, device=dev)
    raw[5:5 + a.values.numel()] = a.values.to(dev)
    moved = Array(DataType.Utf8, n, raw[5:], a.validity.to(dev), a.offsets.to(dev), a.null_count)
    db = RecordBatch(s, [moved, b.columns[1].to(dev)])
    pred = BinaryExpr(Column(1), Operator.Lt, Literal(Float64(0.5)))
    p = compile_scalar_expr(None, pred, s)
    cp = [compile_scalar_expr(None, e, s) for e in (Column(0), Column(1))]
    got = engine().filter_project(p, cp, db)
    for d, (_, r) in zip(got, oracle_filter_project(s, b, pred, [Column(0), Column(1)])):
        assert_same(d.cpu(), r, "misaligned source")
    test_utf8_gather_and_equality()
    test_utf8_many_tiles()


@pytest.mark.parametrize("chunks", ["512", "64"])
def test_utf8_equality_dense_variant(monkeypatch, chunks):
    """Utf8 `col = literal` with the wave's whole source spans staged into LDS
    (DFMI_UTF8_EQ_DENSE: arena chunks per wave; 64 = most slices over the arena,
    compared from global memory) against the oracle."""
    monkeypatch.setenv("DFMI_DIAG", "1")
    monkeypatch.setenv("DFMI_UTF8_EQ_DENSE", chunks)
    test_utf8_gather_and_equality()
    test_utf8_many_tiles()


@pytest.mark.parametrize("group", ["4", "8", "1"])
def test_utf8_equality_register_variant(monkeypatch, group):
    """Utf8 `col = literal` with each slice's span in registers (one 16-byte
    load per lane, the candidates' head words by ds_bpermute;
    DFMI_UTF8_EQ_REG: slices per load round; long strings' slices over 64
    chunks take the global head loads) against the oracle."""
    monkeypatch.setenv("DFMI_DIAG", "1")
    monkeypatch.setenv("DFMI_UTF8_EQ_REG", group)
    test_utf8_gather_and_equality()
    test_utf8_many_tiles()


@pytest.mark.parametrize("variant", ["3", "2", "0", "4", "1", "5", "4p", "5p", "4d", "4dp", "4q", "4w", "4wd", "6", "6g1", "6g4"])
def test_utf8_gather_variants(monkeypatch, variant):
    """The Utf8 gather variants (DFMI_UTF8_GATHER under DFMI_DIAG: 3 = two
    passes -- offsets + source starts in the query kernel, bytes by
    k_utf8_copy_rows --, 2 = one staged slice per round trip, 0 = per-lane
    copy, 4 = slices assembled in an LDS image, 1 = output words' strings by
    binary search, 5 = by marker scan, 6 = per-lane unaligned 16-byte loads and
    exact-length stores (g: slices per load group); p: first staging round before the
    look-back; d: double-buffered staging; q: slices' images in pairs; w: the
    image stored in 16-byte chunks) against
    the oracle on the Utf8 parity cases above."""
    plain = variant in ("3", "4") or variant.startswith("6")  # the multi-channel case runs for these
    if "g" in variant:  # direct gather: slices whose loads go out together
        variant, grp = variant.split("g")
        monkeypatch.setenv("DFMI_UTF8_DIRECT_GROUP", grp)
    if variant.endswith("p"):
        monkeypatch.setenv("DFMI_UTF8_PRESTAGE", "1")
        variant = variant[:-1]
    if variant.endswith("d"):  # the arena's halves double-buffer the staging
        monkeypatch.setenv("DFMI_UTF8_DBUF", "1")
        variant = variant[:-1]
    if variant.endswith("w"):  # 16-byte aligned image, 16-byte stores
        monkeypatch.setenv("DFMI_UTF8_ST16", "1")
        variant = variant[:-1]
    if variant.endswith("q"):  # two slices' images assembled together
        monkeypatch.setenv("DFMI_UTF8_PAIRS", "1")
        variant = variant[:-1]
    monkeypatch.setenv("DFMI_DIAG", "1")
    monkeypatch.setenv("DFMI_UTF8_GATHER", variant)
    test_utf8_gather_and_equality()
    test_utf8_many_tiles()
    if plain or os.environ.get("DFMI_UTF8_PAIRS"):  # 0 is the per-lane fallback; the others
        test_utf8_multi_channel_many_tiles()           # differ only in staging / emitting


@pytest.mark.parametrize("m", ["1", "3", "8s0", "8pf"])
def test_utf8_subtile_counts(monkeypatch, m):
    """Utf8-only predicates run M sub-tiles per look-back (8 by default);
    M = 1 (one look-back per 2048-row tile, round 2's form) and an odd M
    (a last tile whose trailing sub-tiles hold no rows) against the oracle."""
    monkeypatch.setenv("DFMI_DIAG", "1")
    if m.endswith("s0"):  # without the sparse (one lane per selected row) output pass
        monkeypatch.setenv("DFMI_SUBTILE_SPARSE", "0")
    if m.endswith("pf"):  # with the sub-tile offsets prefetch
        monkeypatch.setenv("DFMI_SUBTILE_PREFETCH", "1")
    monkeypatch.setenv("DFMI_SUBTILES", m.rstrip("s0pf") or "8")
    test_utf8_gather_and_equality()
    test_utf8_many_tiles()
    if m == "3":
        test_utf8_multi_channel_many_tiles()


def test_host_batch_many_staging_chunks():
    """dfmi_filter_project_host over a batch larger than the two 64 MB pinned
    staging chunks (H2D 20 chunks, D2H 10 per output): identical to the
    HBM-resident path and to a numpy restatement of the selection."""
    n = 30_000_000
    schema = Schema([Field(c, DataType.Float64, False) for c in "abc"])
    vals = [gen_unit_f64(7, j, 0, n) for j in range(3)]
    b = RecordBatch(schema, [Array.from_numpy(DataType.Float64, v) for v in vals])
    pred = BinaryExpr(BinaryExpr(Column(0), Operator.Gt, Literal(Float64(0.2))), Operator.And,
                      BinaryExpr(Column(1), Operator.Lt, Literal(Float64(0.9))))
    projs = [Column(0), BinaryExpr(BinaryExpr(Column(0), Operator.Multiply, Column(1)), Operator.Plus, Column(2))]
    p = compile_scalar_expr(None, pred, schema)
    cp = [compile_scalar_expr(None, e, schema) for e in projs]
    host = engine().filter_project_host(p, cp, b)
    dev = engine().filter_project(p, cp, b)
    sel = (vals[0] > 0.2) & (vals[1] < 0.9)
    assert host[0].length == dev[0].length == int(sel.sum())
    assert np.array_equal(host[0].numpy_values().view(np.uint64), vals[0][sel].view(np.uint64))
    for h, d in zip(host, dev):
        assert np.array_equal(h.numpy_values().view(np.uint64), d.numpy_values().view(np.uint64))


def test_host_batch_pinned_inputs_and_chunk_errors():
    """dfmi_filter_project_host with input buffers in pinned memory (DMA'd
    straight from them, no staging) equals the pageable-input call; and over
    many pipelined chunks the error is the one of the whole batch in the
    reference's evaluation order: a divide-by-zero whose operator comes first
    in the predicate wins over an earlier-row one that comes later, wherever
    the chunk boundaries fall."""
    n = 3_000_000
    s, b = synth(n, seed=5, nullable=True)
    pinned = RecordBatch(s, [Array(a.data_type, a.length, a.values.pin_memory(),
                                   a.validity.pin_memory() if a.validity is not None else None, None, a.null_count)
                             for a in b.columns])
    assert pinned.columns[0].values.is_pinned()
    pred = BinaryExpr(BinaryExpr(Column(0), Operator.Gt, Literal(Float64(0.3))), Operator.And,
                      BinaryExpr(Column(1), Operator.Lt, Literal(Float64(0.8))))
    projs = [Column(0), BinaryExpr(BinaryExpr(Column(0), Operator.Multiply, Column(1)), Operator.Plus, Column(2))]
    p = compile_scalar_expr(None, pred, s)
    cp = [compile_scalar_expr(None, e, s) for e in projs]
    base = engine().filter_project_host(p, cp, b)
    for chunk in (None, "65536"):
        if chunk:
            os.environ["DFMI_HOST_CHUNK_ROWS"] = chunk
        try:
            got = engine().filter_project_host(p, cp, pinned)
        finally:
            os.environ.pop("DFMI_HOST_CHUNK_ROWS", None)
        for g, r in zip(got, base):
            assert_same(g, r, "pinned inputs, chunk %s" % chunk)
    # zero divisors: column b at row 2_900_000 (late chunk), column c at row 10
    n2 = 1_000_000
    sch = Schema([Field(c, DataType.Float64, False) for c in "abc"])
    vals = [gen_unit_f64(9, j, 0, n2) + 0.5 for j in range(3)]
    vals[1][900_000] = 0.0
    vals[2][10] = -0.0
    bb = RecordBatch(sch, [Array.from_numpy(DataType.Float64, v) for v in vals])
    first = BinaryExpr(BinaryExpr(Column(0), Operator.Divide, Column(1)), Operator.Gt, Literal(Float64(0.1)))
    second = BinaryExpr(BinaryExpr(Column(0), Operator.Divide, Column(2)), Operator.Gt, Literal(Float64(0.1)))
    for chunk in ("4096", "65536", None):
        if chunk:
            os.environ["DFMI_HOST_CHUNK_ROWS"] = chunk
        try:
            assert run_both(sch, bb, BinaryExpr(first, Operator.And, second), [Column(0)]) is None
            assert run_both(sch, bb, BinaryExpr(second, Operator.And, first), [Column(0)]) is None
        finally:
            os.environ.pop("DFMI_HOST_CHUNK_ROWS", None)


def test_static_errors_match():
    s, batch = synth(1000)
    cases = [
        (BinaryExpr(Column(0), Operator.Plus, Column(1)), [Column(0)]),  # not boolean
        (BinaryExpr(Column(0), Operator.And, Column(1)), [Column(0)]),   # boolean_ops panic
        (BinaryExpr(Column(0), Operator.Gt, Literal(Int64(1))), [Column(0)]),  # comparison_ops
    ]
    for pred, projs in cases:
        assert run_both(s, batch, pred, projs) is None
    # zero-row batch still raises the type errors
    s0, b0 = synth(0)
    assert run_both(s0, b0, cases[2][0], cases[2][1]) is None


def test_projection_literals_and_passthrough():
    s, batch = synth(10000, nullable=True)
    run_both(s, batch, None, [Column(0), Literal(Int64(5)), Literal(Float64(2.5)), Cast(Literal(Int64(3)), DataType.Float64)])
    run_both(s, batch, BinaryExpr(Column(0), Operator.Gt, Literal(Float64(0.5))),
             [Literal(Int64(5)), Column(1), BinaryExpr(Literal(Float64(2.0)), Operator.Multiply, Column(2))])
    # deep / non-left-deep arithmetic (LDS temporaries)
    e = BinaryExpr(BinaryExpr(Column(0), Operator.Multiply, Column(1)), Operator.Minus,
                   BinaryExpr(Column(2), Operator.Divide, BinaryExpr(Column(0), Operator.Plus, Literal(Float64(1.0)))))
    run_both(s, batch, None, [e])
    run_both(s, batch, BinaryExpr(e, Operator.Gt, Literal(Float64(0.0))), [e, Column(2)])


def test_q6_style_predicate():
    """C4: shipdate range, discount between, quantity < 24; extendedprice*discount."""
    n = 200_000
    rng = np.random.default_rng(6)
    qty = rng.integers(1, 51, n).astype(np.float64)
    disc = rng.integers(0, 11, n) / 100.0
    ship = rng.integers(8036, 10562, n).astype(np.float64)
    price = qty * rng.uniform(900, 2000, n)
    s = Schema([Field(nm, DataType.Float64, False) for nm in ("l_quantity", "l_extendedprice", "l_discount", "l_shipdate")])
    b = RecordBatch(s, [Array.from_numpy(DataType.Float64, v) for v in (qty, price, disc, ship)])
    ctx = ExecutionContext()
    ctx.register_datasource("lineitem", MemoryDataSource(s, [b]))
    rel = ctx.sql("SELECT l_extendedprice * l_discount FROM lineitem WHERE l_shipdate >= 8766 AND l_shipdate < 9131 "
                  "AND l_discount >= 0.05 AND l_discount <= 0.07 AND l_quantity < 24")
    out = rel.next().columns[0].cpu().numpy_values()
    m = (ship >= 8766) & (ship < 9131) & (disc >= 0.05) & (disc <= 0.07) & (qty < 24)
    assert np.array_equal(out, (price * disc)[m])


def test_c4_bench_generator_against_oracle():
    """C4 (Q6-style projection) over 1,048,577 rows of the bench's own
    generator (bench.q6_table), device and host paths against the oracle."""
    import bench
    n = (1 << 20) + 1
    s, dcols = bench.q6_table(engine().device, n, 42)
    b = RecordBatch(s, [Array.from_numpy(DataType.Float64, c.cpu().numpy()) for c in dcols])
    pred, projs = bench.q6_query()
    dev, ref = run_both(s, b, pred, projs)
    assert 0.01 < ref[0][1].length / n < 0.03


def _nan_cols(n, rng, dt):
    """Values with NaNs of many payloads (quiet and signalling, both signs),
    infinities and zeros."""
    if dt == np.float64:
        u = rng.integers(0, 1 << 51, n, dtype=np.uint64)
        nan_bits = (np.uint64(0x7FF0000000000000) | u | np.uint64(1)) | (rng.integers(0, 2, n, dtype=np.uint64) << np.uint64(63))
        nan_bits[rng.random(n) < 0.5] |= np.uint64(1 << 51)
        x = rng.standard_normal(n)
        nanv = nan_bits.view(np.float64)
    else:
        u = rng.integers(0, 1 << 22, n, dtype=np.uint32)
        nan_bits = (np.uint32(0x7F800000) | u | np.uint32(1)) | (rng.integers(0, 2, n, dtype=np.uint32) << np.uint32(31))
        nan_bits[rng.random(n) < 0.5] |= np.uint32(1 << 22)
        x = rng.standard_normal(n).astype(np.float32)
        nanv = nan_bits.view(np.float32)
    pick = rng.random(n)
    x = np.where(pick < 0.25, nanv, x)
    x = np.where((pick >= 0.25) & (pick < 0.35), np.array(np.inf, dt) * np.sign(rng.standard_normal(n)).astype(dt), x)
    x = np.where((pick >= 0.35) & (pick < 0.4), np.array(0, dt), x)
    return x.astype(dt)


@pytest.mark.parametrize("t", [DataType.Float64, DataType.Float32])
def test_nan_payloads_bit_exact(t):
    """NaN operands propagate quieted, the left one first; inf - inf, 0 * inf
    give x86's negative default NaN; CAST between Float32 / Float64 keeps the
    payload the way cvtsd2ss / cvtss2sd do -- bit for bit on both sides."""
    from datafusion_amd._abi import DFMI_FLAG_EXT_CAST
    dt = np.float64 if t == DataType.Float64 else np.float32
    rng = np.random.default_rng(17 + int(t))
    n = 50_000
    a, b = _nan_cols(n, rng, dt), _nan_cols(n, rng, dt)
    b[b == 0] = 1  # a zero divisor is DivideByZero
    s = Schema([Field("a", t, False), Field("b", t, False), Field("k", DataType.Float64, False)])
    bt = RecordBatch(s, [Array.from_numpy(t, a), Array.from_numpy(t, b),
                         Array.from_numpy(DataType.Float64, rng.random(n))])
    other = DataType.Float32 if t == DataType.Float64 else DataType.Float64
    projs = [BinaryExpr(Column(0), op, Column(1)) for op in MATH] + [Cast(Column(0), other)]
    run_both(s, bt, None, projs, DFMI_FLAG_EXT_CAST)
    run_both(s, bt, BinaryExpr(Column(2), Operator.Lt, Literal(Float64(0.5))), projs,
             DFMI_FLAG_EXT_CAST | DFMI_FLAG_EXT_GATHER_ALL)


def test_utf8_gather_aligned_copy_variant(monkeypatch):
    """DFMI_LIGHT_COPY=0: the per-lane fallback copy (slices whose source span
    exceeds the stage) through utf8_copy's aligned 8-word chunks instead of
    the default unaligned 16-/4-byte moves."""
    monkeypatch.setenv("DFMI_DIAG", "1")
    monkeypatch.setenv("DFMI_LIGHT_COPY", "0")
    test_utf8_multi_channel_many_tiles()
    test_utf8_many_tiles()


@pytest.mark.parametrize("mode", ["1", "2"])
def test_utf8_long_copy_variant(monkeypatch, mode):
    """DFMI_LONG_COPY=1: the per-lane fallback for slices over the stage with
    64 bytes in flight per lane (four unaligned 16-byte loads, then exact-length
    stores of the last < 64 bytes); 2: the wave copies such a slice's strings
    8 lanes per string (wave_copy_slice) -- on the Utf8 parity cases."""
    monkeypatch.setenv("DFMI_DIAG", "1")
    monkeypatch.setenv("DFMI_LONG_COPY", mode)
    test_utf8_multi_channel_many_tiles()
    test_utf8_many_tiles()


def test_utf8_long_strings_choose_long_copy():
    """A large batch of long strings (30-300 bytes): its first call records
    the selected bytes per row, the next call of the same query compiles the
    long-copy fallback (exec.cpp kLongLen). Both against the oracle, including
    a data buffer that ends exactly at the last string's last byte (the
    loads past a string's end stop at offs[n_rows])."""
    import torch
    n = (1 << 22) + 77
    rng = np.random.default_rng(97)
    lens = rng.integers(30, 301, n)
    lens[-5:] = [299, 17, 300, 64, 63]
    offs = np.zeros(n + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    assert offs[-1] < 2 ** 31
    data = rng.integers(32, 127, int(offs[-1])).astype(np.uint8)
    dev = engine().device
    s_arr = Array(DataType.Utf8, n, torch.from_numpy(data).to(dev), None,
                  torch.from_numpy(offs.astype(np.int32)).to(dev), 0)
    v = gen_unit_f64(11, 0, 0, n)
    s = Schema([Field("s", DataType.Utf8, False), Field("v", DataType.Float64, False)])
    b = RecordBatch(s, [s_arr, Array.from_numpy(DataType.Float64, v).to(dev)])
    hb = RecordBatch(s, [a.cpu() for a in b.columns])
    pred = BinaryExpr(Column(1), Operator.Lt, Literal(Float64(0.7)))
    p = compile_scalar_expr(None, pred, s)
    cp = [compile_scalar_expr(None, e, s) for e in (Column(0), Column(1))]
    ref = oracle_filter_project(s, hb, pred, [Column(0), Column(1)])
    from datafusion_amd import _abi
    names = []
    for _ in range(2):
        got = engine().filter_project(p, cp, b)
        names.append(_abi.lib().dfmi_last_kernel_name(engine().ctx))
        for d, (_, r) in zip(got, ref):
            assert_same(d.cpu(), r, "long strings")
    assert names[0] != names[1]  # the second call compiled the long-copy shape


def test_utf8_only_predicate_high_selectivity_switches_to_one_tile():
    """`s != 'w'` over a large batch selects almost every row: its first call
    runs the sub-tile kernel (no hint yet), the next the one-tile kernel with
    the LDS-image gather (exec.cpp: high_sel). Both against the oracle, with
    nulls in the Utf8 column and a nullable numeric projection."""
    import torch
    from datafusion_amd import _abi
    n = (1 << 22) + 5
    rng = np.random.default_rng(5)
    words = [bytes(rng.integers(97, 123, int(rng.integers(0, 25))).astype(np.uint8)) for _ in range(300)]
    idx = rng.integers(0, len(words), n)
    lens = np.array([len(w) for w in words])[idx]
    offs = np.zeros(n + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    flat = np.frombuffer(b"".join([words[i] for i in idx]), np.uint8).copy()
    valid = rng.random(n) >= 0.03
    dev = engine().device
    from datafusion_amd.arrow import pack_bits
    vb = torch.from_numpy(pack_bits(valid)).to(dev)
    s_arr = Array(DataType.Utf8, n, torch.from_numpy(flat).to(dev), vb,
                  torch.from_numpy(offs.astype(np.int32)).to(dev), int(n - valid.sum()))
    s = Schema([Field("s", DataType.Utf8, True), Field("v", DataType.Float64, True)])
    v = Array.from_numpy(DataType.Float64, gen_unit_f64(12, 0, 0, n), rng.random(n) >= 0.1)
    b = RecordBatch(s, [s_arr, v.to(dev)])
    hb = RecordBatch(s, [a.cpu() for a in b.columns])
    pred = BinaryExpr(Column(0), Operator.NotEq, Literal(Utf8(words[7].decode())))
    p = compile_scalar_expr(None, pred, s, DFMI_FLAG_EXT_UTF8_COMPARE)
    cp = [compile_scalar_expr(None, e, s, DFMI_FLAG_EXT_UTF8_COMPARE) for e in (Column(0), Column(1))]
    ref = oracle_filter_project(s, hb, pred, [Column(0), Column(1)], DFMI_FLAG_EXT_UTF8_COMPARE)
    names = []
    for _ in range(2):
        got = engine().filter_project(p, cp, b, DFMI_FLAG_EXT_UTF8_COMPARE)
        names.append(_abi.lib().dfmi_last_kernel_name(engine().ctx))
        for d, (_, r) in zip(got, ref):
            assert_same(d.cpu(), r, "s != literal")
    assert names[0] != names[1]
