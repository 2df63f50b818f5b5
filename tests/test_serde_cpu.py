"""Wire formats (datafusion_amd/serde.py): the serde_json
plan encoding pinned by the reference's own golden string
(logicalplan.rs:631-648 -> tests/golden/serialize_plan.json), round trips of
planner output and random expressions, DataSourceMeta / PhysicalPlan, and the
Arrow IPC result stream read back with pyarrow. The float layout cases follow
ryu's documented format64/format32 rules (serde_json's float writer); no
reference fixture holds floats, so those are parity unpinned."""
import os
import random

import numpy as np
import pyarrow as pa
import pytest

from datafusion_amd import serde
from datafusion_amd.arrow import Array, Field, RecordBatch, Schema
from datafusion_amd.execution.context import Projection, Selection, TableScan
from datafusion_amd.logicalplan import (AggregateFunction, BinaryExpr, Cast, Column, DataType, IsNotNull, IsNull,
                                        Literal, Operator, ScalarFunction, ScalarValue)
from golden_cases import CITIES, GOLDEN, NUMERICS, sql_plan


def test_reference_golden_serialize_plan():
    """logicalplan.rs:609-649 serialize_plan: TableScan of `people` with a
    Struct column and projection [0, 1, 4]."""
    schema = Schema([Field("first_name", DataType.Utf8, False), Field("last_name", DataType.Utf8, False),
                     Field("address", serde.StructType((Field("street", DataType.Utf8, False),
                                                        Field("zip", DataType.UInt16, False))), False)])
    plan = TableScan("people", schema, "", [0, 1, 4])
    want = open(os.path.join(GOLDEN, "serialize_plan.json")).read()
    assert serde.to_json(plan) == want
    back = serde.from_json(want)
    assert serde.to_json(back) == want
    assert back.projection == [0, 1, 4] and back.schema.fields[2].data_type.fields[1].data_type == DataType.UInt16


@pytest.mark.parametrize("v,want", [
    (1.0, "1.0"), (0.1, "0.1"), (-2.5, "-2.5"), (0.0, "0.0"), (-0.0, "-0.0"), (52.59137, "52.59137"),
    (1e15, "1000000000000000.0"), (1e16, "1e16"), (1.2345678901234568e17, "1.2345678901234568e17"),
    (0.0001, "0.0001"), (1e-5, "0.00001"), (1e-6, "1e-6"), (1.5e-7, "1.5e-7"), (5e-324, "5e-324"),
    (1.7976931348623157e308, "1.7976931348623157e308"), (float("nan"), "null"), (float("inf"), "null"),
    (123.456, "123.456"), (50.494344999999996, "50.494344999999996"),
])
def test_float_layout_f64(v, want):
    assert serde.ryu(v) == want


def test_float_layout_f32():
    assert serde.ryu(0.1, True) == "0.1"  # shortest f32 digits, not the widened f64's
    assert serde.ryu(float(np.float32(0.1)), True) == "0.1"
    assert serde.ryu(1e12, True) == "1000000000000.0"
    assert serde.ryu(1e13, True) == "1e13"
    assert serde.ryu(1e-5, True) == "0.00001" and serde.ryu(1e-6, True) == "0.000001"
    assert serde.ryu(1e-7, True) == "1e-7"


def test_expr_encoding_shapes():
    e = BinaryExpr(Column(1), Operator.Gt, Cast(Literal(ScalarValue(DataType.Int64, 21)), DataType.Float64))
    assert serde.to_json(e) == ('{"BinaryExpr":{"left":{"Column":1},"op":"Gt","right":{"Cast":{"expr":'
                                '{"Literal":{"Int64":21}},"data_type":"Float64"}}}}')
    assert serde.to_json(Literal(ScalarValue(DataType.Null))) == '{"Literal":"Null"}'
    assert serde.to_json(Literal(ScalarValue(DataType.Utf8, 'a"b\\c\n\x01é'))) == \
        '{"Literal":{"Utf8":"a\\"b\\\\c\\n\\u0001é"}}'
    assert serde.to_json(IsNull(Column(0))) == '{"IsNull":{"Column":0}}'
    f = AggregateFunction("SUM", (Column(2),), DataType.Float64)
    assert serde.to_json(f) == '{"AggregateFunction":{"name":"SUM","args":[{"Column":2}],"return_type":"Float64"}}'
    assert serde.to_json(serde.SortExpr(Column(0), False)) == '{"Sort":{"expr":{"Column":0},"asc":false}}'


def _rand_expr(rng, depth):
    if depth == 0 or rng.random() < 0.25:
        r = rng.random()
        if r < 0.4:
            return Column(rng.randrange(6))
        t = rng.choice([DataType.Int8, DataType.Int16, DataType.Int32, DataType.Int64, DataType.UInt8,
                        DataType.UInt64, DataType.Float32, DataType.Float64, DataType.Utf8, DataType.Boolean])
        if t in (DataType.Float32, DataType.Float64):
            v = rng.choice([0.5, -1e-300, 1e300, 3.141592653589793, -0.0, rng.uniform(-1e6, 1e6)])
            if t == DataType.Float32:
                v = float(np.float32(v)) if abs(v) < 3e38 else 1.5
        elif t == DataType.Utf8:
            v = "".join(rng.choice('ab"\\\n\té€x') for _ in range(rng.randrange(6)))
        elif t == DataType.Boolean:
            v = rng.random() < 0.5
        elif t == DataType.UInt64:
            v = rng.randrange(1 << 64)
        else:
            bits = {DataType.Int8: 8, DataType.Int16: 16, DataType.Int32: 32, DataType.Int64: 64, DataType.UInt8: 8}[t]
            v = rng.randrange(1 << bits) - ((1 << (bits - 1)) if t != DataType.UInt8 else 0)
        return Literal(ScalarValue(t, v))
    r = rng.random()
    if r < 0.6:
        return BinaryExpr(_rand_expr(rng, depth - 1), Operator(rng.randrange(13)), _rand_expr(rng, depth - 1))
    if r < 0.75:
        return Cast(_rand_expr(rng, depth - 1), DataType(rng.randrange(1, 13)))
    if r < 0.85:
        return (IsNull if rng.random() < 0.5 else IsNotNull)(_rand_expr(rng, depth - 1))
    cls = AggregateFunction if rng.random() < 0.5 else ScalarFunction
    return cls(rng.choice(["sqrt", "MIN", "count"]), tuple(_rand_expr(rng, depth - 1) for _ in range(rng.randrange(3))),
               DataType(rng.randrange(1, 13)))


def test_random_expr_round_trip():
    rng = random.Random(11)
    for _ in range(500):
        e = _rand_expr(rng, 4)
        s = serde.to_json(e)
        back = serde.from_json(s, "Expr")
        assert back == e, s
        assert serde.to_json(back) == s


def test_planner_plans_round_trip():
    """Plans the SQL planner builds (csv_sql.rs's query, numerics, a Selection
    with casts) survive to_json -> from_json -> to_json, and the projection
    schema is the one ExecutionContext derives (expr_to_field)."""
    from datafusion_amd.sqlplanner import SqlToRel

    class Ctx:
        def __init__(self, tables):
            self.tables = tables

        def table_schema(self, name):
            return self.tables.get(name)
    ctx = Ctx({"cities": CITIES, "numerics": NUMERICS})
    for sql in ["SELECT city, lat, lng, lat + lng FROM cities WHERE lat > 51.0 AND lat < 53",
                "SELECT a * b, a_f / 2.5 FROM numerics WHERE a >= 0 OR b_f < 0.00000015",
                "SELECT city FROM cities WHERE lat IS NOT NULL"]:
        plan = SqlToRel(ctx).sql_to_rel(sql)
        s = serde.to_json(plan)
        back = serde.from_json(s)
        assert serde.to_json(back) == s
        assert isinstance(back, Projection)
        assert [f.name for f in serde.plan_schema(back).fields] == [f.name for f in serde.plan_schema(plan).fields]
        if isinstance(plan.input, Selection):
            assert back.input.expr == plan.input.expr
        assert back.expr == plan.expr
    s = serde.to_json(SqlToRel(ctx).sql_to_rel("SELECT lat + lng FROM cities"))
    assert '"schema":{"fields":[{"name":"binary_expr","data_type":"Float64","nullable":true}]}' in s


def test_datasource_meta_and_physical_plan_round_trip():
    meta = serde.CsvFile("test/data/uk_cities.csv", CITIES, True, None)
    s = serde.to_json(meta)
    assert s.startswith('{"CsvFile":{"filename":"test/data/uk_cities.csv","schema":{"fields":[{"name":"city"')
    assert s.endswith('"has_header":true,"projection":null}}')
    assert serde.to_json(serde.from_json(s, "DataSourceMeta")) == s
    pq = serde.ParquetFile("x.parquet", CITIES, [0, 2])
    assert serde.to_json(serde.from_json(serde.to_json(pq), "DataSourceMeta")) == serde.to_json(pq)
    pred, projs = sql_plan("SELECT city FROM cities WHERE lat > 52.0", CITIES, "cities")
    plan = Projection(projs, Selection(pred, TableScan("cities", CITIES)), Schema([CITIES.fields[0]]))
    for pp in (serde.Interactive(plan), serde.Show(plan, 5), serde.Write(plan, "out.csv", "csv")):
        s = serde.to_json(pp)
        assert serde.to_json(serde.from_json(s, "PhysicalPlan")) == s
    lim = serde.Limit(10, plan, Schema([CITIES.fields[0]]))
    assert serde.to_json(serde.from_json(serde.to_json(lim))) == serde.to_json(lim)
    assert serde.to_json(serde.EmptyRelation(Schema([]))) == '{"EmptyRelation":{"schema":{"fields":[]}}}'
    with pytest.raises(serde.WireError):
        serde.from_json('{"Frobnicate":{}}')


def test_ipc_stream_reads_back():
    """Host batches (nulls, Utf8, Boolean, narrow ints) -> Arrow IPC stream ->
    pyarrow: same values, validity and schema."""
    rng = np.random.default_rng(3)
    n = 1000
    valid = rng.random(n) > 0.2
    strs = [None if i % 7 == 3 else ("s%d" % i).encode() * (i % 4) for i in range(n)]
    schema = Schema([Field("f", DataType.Float64, True), Field("s", DataType.Utf8, True),
                     Field("b", DataType.Boolean, False), Field("i", DataType.Int16, False)])
    b = RecordBatch(schema, [Array.from_numpy(DataType.Float64, rng.standard_normal(n), valid),
                             Array.from_strings(strs),
                             Array.from_numpy(DataType.Boolean, rng.random(n) < 0.5),
                             Array.from_numpy(DataType.Int16, rng.integers(-3000, 3000, n).astype(np.int16))])
    data = serde.ipc_stream(schema, [b, b])
    t = pa.ipc.open_stream(data).read_all()
    assert t.num_rows == 2 * n and t.schema.names == ["f", "s", "b", "i"]
    assert t.schema.field("s").type == pa.utf8()
    col = t.column("f").chunk(0)
    assert np.array_equal(np.asarray(col.is_valid()), valid)
    assert np.array_equal(col.to_numpy(zero_copy_only=False)[valid], b.columns[0].numpy_values()[valid])
    assert t.column("s").chunk(1).to_pylist() == [None if s is None else s.decode() for s in strs]
    assert np.array_equal(t.column("b").chunk(0).to_numpy(zero_copy_only=False), b.columns[2].numpy_values())
    assert np.array_equal(t.column("i").chunk(0).to_numpy(), b.columns[3].numpy_values())
