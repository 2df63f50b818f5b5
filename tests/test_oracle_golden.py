"""CPU suite: pin the oracle (CPU restatement) against every known-answer
fixture the reference tree holds for this path."""
import numpy as np
import pytest

from datafusion_amd._abi import DFMI_FLAG_EXT_GATHER_ALL
from datafusion_amd.arrow import Field, Schema
from datafusion_amd.execution.error import ExecutionError
from datafusion_amd.logicalplan import (BinaryExpr, Cast, Column, DataType, Float64, Int64, Literal, Operator,
                                        binary_expr_coerced)
from datafusion_amd.sqlplanner import SqlToRel
from golden_cases import (ALL_TYPES, ALL_TYPES_CAST, ALL_TYPES_NARROW, GOLDEN, CITIES, NULL_CASES, NULL_TEST,
                          NUMERICS, all_types_schema, cast_fixture_case, expected_rows, fixture_values, load_batch,
                          lit_expr, narrow_fixture_case, smoketest_points, sql_plan)
from datafusion_amd._abi import DFMI_FLAG_EXT_CAST, DFMI_FLAG_EXT_IS_NULL
from oracle_ffi import oracle_compile, oracle_filter_project


class _Ctx:
    def __init__(self, schemas):
        self.schemas = schemas

    def table_schema(self, name):
        return self.schemas.get(name)


def plan(sql, schema, table="t"):
    p = SqlToRel(_Ctx({table: schema})).sql_to_rel(sql)
    pred = p.input.expr if type(p.input).__name__ == "Selection" else None
    return pred, p.expr


def test_csv_sql_example():
    """examples/csv_sql.rs:56 over test/data/uk_cities.csv, has_header=true:
    18 of 36 rows; first row Solihull; Oxford's combined 50.494344999999996."""
    batch = load_batch(CITIES, "uk_cities.csv", has_header=True)
    assert batch.num_rows() == 36
    pred, projs = plan("SELECT city, lat, lng, lat + lng FROM cities WHERE lat > 51.0 AND lat < 53",
                       CITIES, "cities")
    assert repr(pred) == "#1 Gt Float64(51.0) And #1 Lt CAST(Int64(53) AS Float64)"
    out = oracle_filter_project(CITIES, batch, pred, projs)
    names = [n for n, _ in out]
    assert names == ["city", "lat", "lng", "#1 Plus #2"]
    city, lat, lng, comb = [a.to_pylist() for _, a in out]
    assert len(city) == 18
    assert (city[0], lat[0], lng[0], comb[0]) == ("Solihull, Birmingham, UK", 52.412811, -1.778197, 50.634614)
    i = city.index("Oxford, Oxfordshire, UK")
    assert repr(comb[i]) == "50.494344999999996"
    for a, b, c in zip(lat, lng, comb):
        assert c == a + b and 51.0 < a < 53


def test_filter_fixture():
    """expected/test_filter.csv = SELECT * FROM uk_cities WHERE lat > 52.0
    (FilterRelation output, Utf8 + Float64 gather, no header row)."""
    batch = load_batch(CITIES, "uk_cities.csv", has_header=False)
    exp = [ln.rsplit(",", 2) for ln in open(GOLDEN + "/expected/test_filter.csv", encoding="utf-8").read().splitlines() if ln]
    out = oracle_filter_project(CITIES, batch, lit_expr(CITIES, 1, Operator.Gt, Float64(52.0)), [])
    city, lat, lng = [a.to_pylist() for _, a in out]
    assert len(city) == len(exp) == 20
    for (c, la, ln), e in zip(zip(city, lat, lng), exp):
        assert c == e[0] and la == float(e[1]) and ln == float(e[2])


@pytest.mark.parametrize("op,section,count", [(Operator.Lt, 0, 25), (Operator.GtEq, 1, 12)])
def test_smoketest_predicates(op, section, count):
    """smoketest-expected.txt:4-41 and expected/test_simple_predicate.csv:
    lat < 53.0 -> 25 rows, lat >= 53.0 -> 12 rows."""
    batch = load_batch(CITIES, "uk_cities.csv", has_header=False)
    out = oracle_filter_project(CITIES, batch, lit_expr(CITIES, 1, op, Float64(53.0)), [Column(1), Column(2)])
    lat, lng = [a.to_pylist() for _, a in out]
    exp = smoketest_points(section)
    assert len(lat) == len(exp) == count
    assert list(zip(lat, lng)) == exp
    if section == 0:
        pts = [r[0] for r in expected_rows("test_simple_predicate.csv")]
        assert ["POINT (%s %s)" % (repr(a).rstrip("0").rstrip("."), repr(b).rstrip("0").rstrip("."))
                for a, b in zip(lat, lng)][:3] == pts[:3]


@pytest.mark.parametrize("fname,op,count", [("c_float64_high.csv", Operator.Gt, 119),
                                            ("c_float64_low.csv", Operator.Lt, 137)])
def test_all_types_float64(fname, op, count):
    """expected/c_float64_{high,low}.csv: column 10 of all_types_flat.csv vs 0.5."""
    s = all_types_schema(f64_col=10)
    batch = load_batch(s, "all_types_flat.csv", has_header=False)
    out = oracle_filter_project(s, batch, lit_expr(s, 10, op, Float64(0.5)), [Column(10)])
    vals = out[0][1].to_pylist()
    exp = [float(r[0]) for r in expected_rows(fname)]
    assert len(vals) == count == len(exp)
    assert vals == exp


@pytest.mark.parametrize("fname,op,count", [("c_int64_positive.csv", Operator.Gt, 134),
                                            ("c_int64_negative.csv", Operator.Lt, 122)])
def test_all_types_int64(fname, op, count):
    """expected/c_int64_{positive,negative}.csv: column 8 vs 0. The reference
    refuses to filter Int64 (filter.rs:106-110); the extension flag gathers it."""
    s = all_types_schema(i64_col=8)
    batch = load_batch(s, "all_types_flat.csv", has_header=False)
    pred = lit_expr(s, 8, op, Int64(0))
    with pytest.raises(ExecutionError) as e:
        oracle_filter_project(s, batch, pred, [Column(8)])
    assert e.value.kind == "ExecutionError" and e.value.message == "filter not supported for Int64"
    out = oracle_filter_project(s, batch, pred, [Column(8)], DFMI_FLAG_EXT_GATHER_ALL)
    vals = out[0][1].to_pylist()
    exp = [int(r[0]) for r in expected_rows(fname)]
    assert len(vals) == count and vals == exp


@pytest.mark.parametrize("opname,op", [("plus", Operator.Plus), ("minus", Operator.Minus),
                                       ("multiply", Operator.Multiply), ("divide", Operator.Divide)])
def test_numerics(opname, op):
    """expected/numerics_<op>_f64.csv: a OP b, a OP 2 (Int64) and
    a_f OP b_f, a_f OP 2 (cast literal), a_f OP 2.5 (Float64) over numerics.csv."""
    batch = load_batch(NUMERICS, "numerics.csv", has_header=True)
    S = NUMERICS
    exprs = [binary_expr_coerced(Column(0), op, Column(1), S), binary_expr_coerced(Column(0), op, Literal(Int64(2)), S),
             binary_expr_coerced(Column(2), op, Column(3), S), binary_expr_coerced(Column(2), op, Literal(Int64(2)), S),
             binary_expr_coerced(Column(2), op, Literal(Float64(2.5)), S)]
    out = oracle_filter_project(S, batch, None, exprs)
    got = [a.to_pylist() for _, a in out]
    exp = expected_rows("numerics_%s_f64.csv" % opname)
    assert len(exp) == 3
    for r, e in enumerate(exp):
        assert got[0][r] == int(e[0]) and got[1][r] == int(e[1])
        for j, col in ((2, 3), (3, 4), (4, 5)):
            assert got[j][r] == float(e[col]), (opname, r, j)
    assert [n for n, _ in out][3] == "#2 %s CAST(Int64(2) AS Float64)" % op.name
    # column 3 of the fixture (a OP 2.5) needs CAST(#0 AS Float64): not executable
    with pytest.raises(ExecutionError) as e:
        oracle_filter_project(S, batch, None, [binary_expr_coerced(Column(0), op, Literal(Float64(2.5)), S)])
    assert e.value.message == "column reference"


@pytest.mark.parametrize("opname,op", [("plus", Operator.Plus), ("minus", Operator.Minus),
                                       ("multiply", Operator.Multiply), ("divide", Operator.Divide)])
def test_numerics_float32(opname, op):
    """expected/numerics_<op>.csv column 4: a_f OP b_f in Float32."""
    S = Schema([Field("a", DataType.Int64, False), Field("b", DataType.Int64, False),
                Field("a_f", DataType.Float32, False), Field("b_f", DataType.Float32, False)])
    batch = load_batch(S, "numerics.csv", has_header=True)
    out = oracle_filter_project(S, batch, None, [BinaryExpr(Column(2), op, Column(3))])
    got = out[0][1].numpy_values()
    exp = expected_rows("numerics_%s.csv" % opname)
    for r, e in enumerate(exp):
        assert got[r] == np.float32(e[3])


@pytest.mark.parametrize("case", ALL_TYPES_NARROW, ids=[c[0] for c in ALL_TYPES_NARROW])
def test_all_types_narrow(case):
    """expected/c_int{8,16,32}_*.csv, c_float32_{high,low}.csv: comparisons of
    Int8/Int16/Int32/Float32 columns of all_types_flat.csv (same-typed literal,
    comparison_ops! expression.rs:174-203). Gathering them needs the
    extension flag (filter.rs:106-110 rejects every type but Float64/Utf8)."""
    name, col, op, lit = case
    s, pred, projs = narrow_fixture_case(*case)
    batch = load_batch(s, "all_types_flat.csv", has_header=False)
    with pytest.raises(ExecutionError) as e:
        oracle_filter_project(s, batch, pred, projs)
    assert e.value.message == "filter not supported for %r" % ALL_TYPES[col]
    out = oracle_filter_project(s, batch, pred, projs, DFMI_FLAG_EXT_GATHER_ALL)
    assert out[0][1].to_pylist() == fixture_values(name, ALL_TYPES[col])


@pytest.mark.parametrize("case", ALL_TYPES_CAST, ids=[c[0] for c in ALL_TYPES_CAST])
def test_all_types_cast_extension(case):
    """expected/c_*_cast.csv, c_int8_col_*.csv: planner-inserted CAST(column)
    nodes, executable only under DFMI_FLAG_EXT_CAST."""
    name, cols, sql = case
    s, pred, projs = cast_fixture_case(*case)
    batch = load_batch(s, "all_types_flat.csv", has_header=False)
    fl = DFMI_FLAG_EXT_GATHER_ALL | DFMI_FLAG_EXT_CAST
    if "CAST(" in repr(pred) + repr(projs):
        with pytest.raises(ExecutionError) as e:
            oracle_filter_project(s, batch, pred, projs, DFMI_FLAG_EXT_GATHER_ALL)
        assert e.value.message == "column reference"
    out = oracle_filter_project(s, batch, pred, projs, fl)
    assert out[0][1].to_pylist() == fixture_values(name, ALL_TYPES[cols[0]])


@pytest.mark.parametrize("name,sql", NULL_CASES)
def test_is_null_extension(name, sql):
    """expected/is_null_csv.csv, is_not_null_csv.csv over null_test.csv."""
    batch = load_batch(NULL_TEST, "null_test.csv", has_header=True)
    pred, projs = sql_plan(sql, NULL_TEST, "null_test")
    with pytest.raises(ExecutionError) as e:
        oracle_filter_project(NULL_TEST, batch, pred, projs, DFMI_FLAG_EXT_GATHER_ALL)
    assert e.value.message.startswith("expression #1 IS")
    out = oracle_filter_project(NULL_TEST, batch, pred, projs, DFMI_FLAG_EXT_GATHER_ALL | DFMI_FLAG_EXT_IS_NULL)
    assert out[0][1].to_pylist() == [int(r[0]) for r in expected_rows(name)]


def test_cast_rules():
    """num::cast rules of the arrow cast kernel (parity unpinned beyond the
    fixtures): out-of-range and NaN -> null, truncation toward zero."""
    from datafusion_amd.arrow import Array, RecordBatch
    from datafusion_amd.logicalplan import ScalarValue
    f = np.array([1.9, -1.9, 127.5, 128.0, -128.9, -129.0, np.nan, np.inf, 3e38, 4e38, -0.5], dtype=np.float64)
    S = Schema([Field("f", DataType.Float64, False)])
    b = RecordBatch(S, [Array.from_numpy(DataType.Float64, f)])
    fl = DFMI_FLAG_EXT_CAST
    out = oracle_filter_project(S, b, None, [Cast(Column(0), DataType.Int8), Cast(Column(0), DataType.Float32),
                                            Cast(Column(0), DataType.UInt8)], fl)
    assert out[0][0] == "CAST(#0 AS Int8)"
    assert out[0][1].to_pylist() == [1, -1, 127, None, -128, None, None, None, None, None, 0]
    f32 = out[1][1].to_pylist()
    assert f32[8] == float(np.float32(3e38)) and f32[9] is None and f32[7] == float("inf")
    assert out[2][1].to_pylist() == [1, None, 127, 128, None, None, None, None, None, None, 0]
    i = np.array([-1, 255, 256, -(1 << 63), (1 << 63) - 1], dtype=np.int64)
    S2 = Schema([Field("i", DataType.Int64, False)])
    b2 = RecordBatch(S2, [Array.from_numpy(DataType.Int64, i)])
    out = oracle_filter_project(S2, b2, None, [Cast(Column(0), DataType.UInt8), Cast(Column(0), DataType.UInt64),
                                              Cast(Column(0), DataType.Float32)], fl)
    assert out[0][1].to_pylist() == [None, 255, None, None, None]
    assert out[1][1].to_pylist() == [None, 255, 256, None, (1 << 63) - 1]
    assert out[2][1].to_pylist()[3] == -2.0 ** 63
    with pytest.raises(ExecutionError) as e:
        oracle_filter_project(S2, b2, None, [Cast(Literal(ScalarValue(DataType.Int32, 1)), DataType.Int64)], fl)
    assert e.value.kind == "NotImplemented"


def test_projection_unit_test():
    """projection.rs:85-107: people.csv, project Column(0) -> one column "id"."""
    S = Schema([Field("id", DataType.Int32, False), Field("first_name", DataType.Utf8, False)])
    batch = load_batch(S, "people.csv", has_header=True)
    out = oracle_filter_project(S, batch, None, [Column(0)])
    assert len(out) == 1 and out[0][0] == "id"


def test_compile_names_and_errors():
    """compile_scalar_expr names/types and compile-time errors (expression.rs:244-451)."""
    S = NUMERICS
    assert oracle_compile(Literal(Int64(5)), S) == ("5", DataType.Int64)
    assert oracle_compile(Literal(Float64(0.5)), S) == ("0.5", DataType.Float64)
    assert oracle_compile(Literal(Float64(1.0)), S) == ("1", DataType.Float64)
    assert oracle_compile(Cast(Literal(Int64(53)), DataType.Float64), S) == ("lit", DataType.Float64)
    assert oracle_compile(BinaryExpr(Column(0), Operator.Plus, Column(1)), S) == ("#0 Plus #1", DataType.Int64)
    assert oracle_compile(BinaryExpr(Column(2), Operator.Gt, Literal(Float64(2.0))), S) == \
        ("#2 Gt Float64(2.0)", DataType.Boolean)

    def err(e, flags=0):
        with pytest.raises(ExecutionError) as x:
            oracle_compile(e, S, flags)
        return x.value.kind, x.value.message

    from datafusion_amd.logicalplan import IsNull, ScalarValue, Utf8
    assert err(Literal(Utf8("w17"))) == ("ExecutionError", 'No support for literal type Utf8("w17")')
    assert err(Literal(ScalarValue(DataType.Boolean, True))) == ("ExecutionError",
                                                                 "No support for literal type Boolean(true)")
    assert err(Cast(Column(0), DataType.Float64)) == ("ExecutionError", "column reference")
    assert err(Cast(Literal(Int64(1)), DataType.Int32)) == ("NotImplemented", "CAST from Int64 to Int32")
    assert err(Cast(Literal(Float64(1.5)), DataType.Int64)) == ("NotImplemented",
                                                               "CAST from Float64(1.5) to Int64")
    assert err(Cast(BinaryExpr(Column(0), Operator.Plus, Column(1)), DataType.Float64)) == \
        ("General", "CAST not implemented for expression #0 Plus #1")
    assert err(BinaryExpr(Column(0), Operator.Modulus, Column(1))) == ("ExecutionError", "operator: Modulus")
    assert err(IsNull(Column(0))) == ("ExecutionError", "expression #0 IS NULL")
    assert err(Column(9))[0] == "panic"


def test_oracle_x86_nan_rules():
    """The oracle's NaN results follow x86 SSE: a NaN operand
    propagates quieted, the left one first; invalid operations give the
    negative default NaN."""
    import numpy as np
    from datafusion_amd.arrow import Array, Field, RecordBatch, Schema
    from datafusion_amd.logicalplan import BinaryExpr, Column, DataType, Operator
    from oracle_ffi import oracle_filter_project
    q1 = np.array([0x7FF8000000000001], dtype=np.uint64).view(np.float64)[0]
    s1 = np.array([0xFFF0000000000002], dtype=np.uint64).view(np.float64)[0]  # signalling, negative
    a = np.array([q1, 1.0, s1, np.inf, 0.0, q1])
    b = np.array([s1, s1, 2.0, np.inf, np.inf, 3.0])
    s = Schema([Field("a", DataType.Float64, False), Field("b", DataType.Float64, False)])
    bt = RecordBatch(s, [Array.from_numpy(DataType.Float64, a), Array.from_numpy(DataType.Float64, b)])
    (_, add), (_, sub), (_, mul) = oracle_filter_project(
        s, bt, None, [BinaryExpr(Column(0), op, Column(1)) for op in (Operator.Plus, Operator.Minus, Operator.Multiply)])
    bits = lambda arr: [hex(int(x)) for x in arr.numpy_values().view(np.uint64)]
    assert bits(add)[:3] == ["0x7ff8000000000001", "0xfff8000000000002", "0xfff8000000000002"]
    assert bits(sub)[3] == "0xfff8000000000000"   # inf - inf
    assert bits(mul)[4] == "0xfff8000000000000"   # 0 * inf
    assert bits(add)[5] == "0x7ff8000000000001"


# ---------------------------------------------------------- round-3 fixtures
from golden_cases import (MIN_MAX_SQL, RANGE_CASES, WHOLE_F32_FILES, agg_fixture_value,  # noqa: E402
                          all_types_typed, range_fixture_case, whole_f32_case)


@pytest.mark.parametrize("case", RANGE_CASES, ids=[c[0] for c in RANGE_CASES])
def test_int8_range_inclusive(case):
    """expected/c_int8_range_inclusive.csv (98 rows) = c5 >= 2 AND c5 <= 99."""
    name, col = case[0], case[1]
    s, pred, projs = range_fixture_case(*case)
    batch = load_batch(s, "all_types_flat.csv", has_header=False)
    with pytest.raises(ExecutionError) as e:
        oracle_filter_project(s, batch, pred, projs)
    assert e.value.message == "filter not supported for Int8"
    out = oracle_filter_project(s, batch, pred, projs, DFMI_FLAG_EXT_GATHER_ALL)
    assert out[0][1].to_pylist() == fixture_values(name, ALL_TYPES[col])
    assert len(out[0][1].to_pylist()) == 98


@pytest.mark.parametrize("name", WHOLE_F32_FILES)
def test_float32_uint32_files_are_the_whole_column(name):
    """expected/c_float32_*_uint32.csv: the whole c_float32 column, selected by
    CAST(c9 AS UInt32) = 0 (golden_cases.WHOLE_F32_FILES says why)."""
    s, pred, projs = whole_f32_case()
    batch = load_batch(s, "all_types_flat.csv", has_header=False)
    want = fixture_values(name, DataType.Float32)
    assert want == batch.columns[9].to_pylist() and len(want) == 256
    out = oracle_filter_project(s, batch, pred, projs, DFMI_FLAG_EXT_GATHER_ALL | DFMI_FLAG_EXT_CAST)
    assert out[0][1].to_pylist() == want


def _agg_plan(sql, schema, table, grouped=False):
    from datafusion_amd.execution.context import Aggregate
    p = SqlToRel(_Ctx({table: schema})).sql_to_rel(sql)
    assert isinstance(p, Aggregate) and bool(p.group_expr) == grouped
    return (p.group_expr, p.aggr_expr) if grouped else p.aggr_expr


def test_sql_min_max_fixture():
    """expected/test_sql_min_max.csv: MIN/MAX(lat), MIN/MAX(lng) over the 37
    rows of uk_cities.csv, through the planner's Aggregate (sqlplanner.rs:91-117)."""
    from datafusion_amd._abi import DFMI_FLAG_EXT_AGGREGATE as AGG
    from oracle_ffi import oracle_aggregate
    batch = load_batch(CITIES, "uk_cities.csv", has_header=False)
    assert batch.num_rows() == 37
    aggs = _agg_plan(MIN_MAX_SQL, CITIES, "uk_cities")
    got = oracle_aggregate(CITIES, batch, None, aggs, AGG)
    want = expected_rows("test_sql_min_max.csv")[0]
    assert [g.bits for g in got] == [agg_fixture_value(w, DataType.Float64) for w in want]


def all_types_aggregates():
    """csv_aggregate_all_types.csv as (SQL, expected cells) pairs the
    extension executes: COUNT(*) twice, then MIN/MAX of columns 1-10 in two
    plans (a state holds at most 16 aggregates)."""
    want = expected_rows("csv_aggregate_all_types.csv")[0]
    assert len(want) == 26
    plans = [("SELECT COUNT(c0), COUNT(c11) FROM t", want[0:2], [DataType.UInt64] * 2)]
    for lo, hi in ((1, 6), (6, 11)):
        sel = ", ".join("MIN(c%d), MAX(c%d)" % (c, c) for c in range(lo, hi))
        cells = want[2 + 2 * lo: 2 + 2 * hi]
        plans.append(("SELECT %s FROM t" % sel, cells, [ALL_TYPES[c] for c in range(lo, hi) for _ in (0, 1)]))
    return plans


def test_csv_aggregate_all_types_fixture():
    """expected/csv_aggregate_all_types.csv columns 1-10 (every numeric type)
    and the counts; MIN/MAX of Boolean / Utf8 are NotImplemented."""
    from datafusion_amd._abi import DFMI_FLAG_EXT_AGGREGATE as AGG
    from oracle_ffi import oracle_aggregate
    s = all_types_typed()
    batch = load_batch(s, "all_types_flat.csv", has_header=False)
    for sql, cells, types in all_types_aggregates():
        got = oracle_aggregate(s, batch, None, _agg_plan(sql, s, "t"), AGG)
        assert [g.bits for g in got] == [agg_fixture_value(c, t) for c, t in zip(cells, types)], sql
    for c in (0, 11):
        with pytest.raises(ExecutionError) as e:
            oracle_aggregate(s, batch, None, _agg_plan("SELECT MIN(c%d) FROM t" % c, s, "t"), AGG)
        assert e.value.kind == "NotImplemented"


def by_c_bool_aggregates():
    """csv_aggregate_by_c_bool.csv as (SQL, expected cells per group) pairs:
    GROUP BY c0 (Boolean), MIN/MAX of columns 1-10 in two plans; the file's
    Utf8 MIN/MAX (last two cells) are outside the extension."""
    rows = expected_rows("csv_aggregate_by_c_bool.csv")
    assert [r[0] for r in rows] == ["false", "true"] and all(len(r) == 23 for r in rows)
    plans = []
    for lo, hi in ((1, 6), (6, 11)):
        sel = ", ".join("MIN(c%d), MAX(c%d)" % (c, c) for c in range(lo, hi))
        cells = [r[1 + 2 * (lo - 1): 1 + 2 * (hi - 1)] for r in rows]
        plans.append(("SELECT c0, %s FROM t GROUP BY c0" % sel, cells,
                      [ALL_TYPES[c] for c in range(lo, hi) for _ in (0, 1)]))
    return plans


def test_csv_aggregate_by_c_bool_fixture():
    """expected/csv_aggregate_by_c_bool.csv: MIN/MAX of every numeric column
    per c_bool group (false, then true), through the planner's
    Aggregate{group_expr} (sqlplanner.rs:91-117)."""
    from datafusion_amd._abi import DFMI_FLAG_EXT_AGGREGATE as AGG
    from oracle_ffi import oracle_aggregate_grouped
    s = all_types_typed()
    batch = load_batch(s, "all_types_flat.csv", has_header=False)
    for sql, cells, types in by_c_bool_aggregates():
        (key,), aggs = _agg_plan(sql, s, "t", grouped=True)
        keys, vals = oracle_aggregate_grouped(s, batch, None, key, aggs, AGG)
        assert [(k.is_null, k.bits) for k in keys] == [(0, 0), (0, 1)]
        for g in range(2):
            assert [v.bits for v in vals[g]] == [agg_fixture_value(c, t) for c, t in zip(cells[g], types)], (sql, g)
    # batch-size independence and a predicate (count per group)
    sql = "SELECT c0, COUNT(c1), SUM(c8), MIN(c9), MAX(c10) FROM t GROUP BY c0"
    (key,), aggs = _agg_plan(sql, s, "t", grouped=True)
    one = oracle_aggregate_grouped(s, batch, None, key, aggs, AGG)
    for br in (8, 64, 1000):
        again = oracle_aggregate_grouped(s, batch, None, key, aggs, AGG, batch_rows=br)
        assert [(k.is_null, k.bits) for k in again[0]] == [(k.is_null, k.bits) for k in one[0]]
        assert [[(v.is_null, v.bits) for v in g] for g in again[1]] == [[(v.is_null, v.bits) for v in g] for g in one[1]]
    assert sum(v[0].bits for v in one[1]) == batch.num_rows()
