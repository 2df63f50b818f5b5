"""Wire formats: the reference's serde_json encoding of
its plans, and a worker entry point that runs a serialized plan on the GPU and
returns the result in Arrow IPC stream format.

* ``to_json`` / ``from_json`` restate serde's externally tagged encoding of
  ``LogicalPlan`` / ``Expr`` / ``ScalarValue`` / ``Operator``
  (``#[derive(Serialize, Deserialize)]``, logicalplan.rs:24,66,92,132,307),
  arrow 0.12's ``DataType`` / ``Field`` / ``Schema``, ``DataSourceMeta``
  (datasource.rs:70-85) and ``PhysicalPlan`` (physicalplan.rs:18-33), as
  serde_json 1.0 writes them: compact, struct fields in declaration order,
  unit variants as strings, ``Rc``/``Arc`` transparent (serde's "rc"
  feature), floats in ryu's shortest form, non-finite floats as ``null``.
  Pinned by the reference's own golden string (logicalplan.rs:631-648,
  ``tests/golden/serialize_plan.json``).
* ``run_physical_plan`` is the worker the reference's README lists as
  unbuilt ("receive a query plan, execute the query, and return a result in
  Arrow IPC format", README.md:33): the plan's Selection / Projection run
  through the device path (``ExecutionContext.execute``), the batches are
  encoded as an Arrow IPC stream.
"""
from __future__ import annotations

import json
import math
from dataclasses import dataclass
from typing import List, Optional

from .arrow import Field, Schema
from .logicalplan import (AggregateFunction, BinaryExpr, Cast, Column, DataType, Expr, IsNotNull, IsNull, Literal,
                          Operator, ScalarFunction, ScalarValue, _shortest_digits)


# ------------------------------------------------ serde-only variants
@dataclass(frozen=True)
class StructType:
    """arrow DataType::Struct(Vec<Field>) (schemas only; not executable)."""
    fields: tuple


@dataclass(frozen=True)
class ListType:
    """arrow DataType::List(Box<DataType>) (schemas only; not executable)."""
    value_type: object


@dataclass(frozen=True, eq=True)
class SortExpr(Expr):
    """Expr::Sort { expr, asc } (logicalplan.rs:149)."""
    expr: Expr
    asc: bool


class Limit:
    """LogicalPlan::Limit { limit, input, schema } (logicalplan.rs:310-314)."""

    def __init__(self, limit: int, input, schema: Schema):
        self.limit, self.input, self.schema = limit, input, schema


class Sort:
    """LogicalPlan::Sort { expr, input, schema } (logicalplan.rs:331-335)."""

    def __init__(self, expr, input, schema: Schema):
        self.expr, self.input, self.schema = list(expr), input, schema


class EmptyRelation:
    """LogicalPlan::EmptyRelation { schema } (logicalplan.rs:345)."""

    def __init__(self, schema: Schema):
        self.schema = schema


@dataclass
class CsvFile:
    """DataSourceMeta::CsvFile (datasource.rs:73-78)."""
    filename: str
    schema: Schema
    has_header: bool
    projection: Optional[List[int]] = None


@dataclass
class ParquetFile:
    """DataSourceMeta::ParquetFile (datasource.rs:80-84)."""
    filename: str
    schema: Schema
    projection: Optional[List[int]] = None


@dataclass
class Interactive:
    """PhysicalPlan::Interactive { plan } (physicalplan.rs:20-23)."""
    plan: object


@dataclass
class Write:
    """PhysicalPlan::Write { plan, filename, kind } (physicalplan.rs:24-29)."""
    plan: object
    filename: str
    kind: str


@dataclass
class Show:
    """PhysicalPlan::Show { plan, count } (physicalplan.rs:30-33)."""
    plan: object
    count: int


# ------------------------------------------------ scalars
def ryu(v: float, f32: bool = False) -> str:
    """serde_json's float text: ryu's shortest round-trip digits, laid out as
    ryu's format64 / format32 do (plain decimal when the decimal point falls
    in [-5, 16] digits (f32: [-6, 13]), else scientific); NaN / inf -> null."""
    if math.isnan(v) or math.isinf(v):
        return "null"
    neg = math.copysign(1.0, v) < 0
    if v == 0.0:
        return "-0.0" if neg else "0.0"
    digits, e10 = _shortest_digits(abs(v), f32)
    length = len(digits)
    k = e10 - length + 1  # value = digits * 10^k
    kk = length + k       # 10^(kk-1) <= v < 10^kk
    hi, lo = (13, -6) if f32 else (16, -5)
    if 0 <= k and kk <= hi:
        s = digits + "0" * k + ".0"
    elif 0 < kk <= hi:
        s = digits[:kk] + "." + digits[kk:]
    elif lo < kk <= 0:
        s = "0." + "0" * (-kk) + digits
    elif length == 1:
        s = digits + "e" + str(kk - 1)
    else:
        s = digits[0] + "." + digits[1:] + "e" + str(kk - 1)
    return ("-" if neg else "") + s


def _str(s: str) -> str:
    """serde_json string escaping: ", \\ and control characters; the rest raw."""
    out = ['"']
    for ch in s:
        c = ord(ch)
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif c < 0x20:
            out.append({8: "\\b", 9: "\\t", 10: "\\n", 12: "\\f", 13: "\\r"}.get(c, "\\u%04x" % c))
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def _obj(pairs) -> str:
    return "{" + ",".join(_str(k) + ":" + v for k, v in pairs) + "}"


def _tag(name: str, body: str) -> str:
    return "{" + _str(name) + ":" + body + "}"


# ------------------------------------------------ encode
def _datatype(t) -> str:
    if isinstance(t, StructType):
        return _tag("Struct", "[" + ",".join(_field(f) for f in t.fields) + "]")
    if isinstance(t, ListType):
        return _tag("List", _datatype(t.value_type))
    t = DataType(t)
    if t == DataType.Null:
        raise ValueError("arrow 0.12 DataType has no Null variant")
    return _str(t.name)


def _field(f: Field) -> str:
    return _obj([("name", _str(f.name)), ("data_type", _datatype(f.data_type)),
                 ("nullable", "true" if f.nullable else "false")])


def _schema(s: Schema) -> str:
    return _obj([("fields", "[" + ",".join(_field(f) for f in s.fields) + "]")])


def _scalar(v: ScalarValue) -> str:
    t = v.dtype
    if t == DataType.Null:
        return '"Null"'
    if t == DataType.Boolean:
        body = "true" if v.value else "false"
    elif t in (DataType.Float32, DataType.Float64):
        body = ryu(float(v.value), t == DataType.Float32)
    elif t == DataType.Utf8:
        body = _str(v.value)
    else:
        body = str(int(v.value))
    return _tag(t.name, body)


def _expr(e: Expr) -> str:
    if isinstance(e, Column):
        return _tag("Column", str(int(e.index)))
    if isinstance(e, Literal):
        return _tag("Literal", _scalar(e.value))
    if isinstance(e, BinaryExpr):
        return _tag("BinaryExpr", _obj([("left", _expr(e.left)), ("op", _str(Operator(e.op).name)),
                                        ("right", _expr(e.right))]))
    if isinstance(e, IsNotNull):
        return _tag("IsNotNull", _expr(e.expr))
    if isinstance(e, IsNull):
        return _tag("IsNull", _expr(e.expr))
    if isinstance(e, Cast):
        return _tag("Cast", _obj([("expr", _expr(e.expr)), ("data_type", _datatype(e.data_type))]))
    if isinstance(e, SortExpr):
        return _tag("Sort", _obj([("expr", _expr(e.expr)), ("asc", "true" if e.asc else "false")]))
    if isinstance(e, ScalarFunction):  # AggregateFunction is a subclass
        name = "AggregateFunction" if isinstance(e, AggregateFunction) else "ScalarFunction"
        return _tag(name, _obj([("name", _str(e.name)), ("args", "[" + ",".join(_expr(a) for a in e.args) + "]"),
                                ("return_type", _datatype(e.return_type))]))
    raise TypeError("not an Expr: %r" % (e,))


def _exprs(es) -> str:
    return "[" + ",".join(_expr(e) for e in es) + "]"


def plan_schema(plan) -> Schema:
    """LogicalPlan::schema() (logicalplan.rs:348-360)."""
    from .execution.context import Aggregate, Projection, Selection, TableScan
    if isinstance(plan, Selection):
        return plan_schema(plan.input)
    if isinstance(plan, Projection) and plan.schema is None:
        from .logicalplan import expr_to_field_name_type
        inp = plan_schema(plan.input)
        fields = []
        for e in plan.expr:  # exprlist_to_fields (context.rs:173-209 / sqlplanner.rs)
            if isinstance(e, Column):
                fields.append(inp.fields[e.index])
            else:
                n, t = expr_to_field_name_type(e, inp)
                fields.append(Field(n, t, True))
        return Schema(fields)
    if isinstance(plan, (TableScan, Projection, Aggregate, Limit, Sort, EmptyRelation)):
        return plan.schema
    raise TypeError("not a LogicalPlan: %r" % (plan,))


def _projection(p) -> str:
    return "null" if p is None else "[" + ",".join(str(int(i)) for i in p) + "]"


def _plan(p) -> str:
    from .execution.context import Aggregate, Projection, Selection, TableScan
    if isinstance(p, Limit):
        return _tag("Limit", _obj([("limit", str(int(p.limit))), ("input", _plan(p.input)),
                                   ("schema", _schema(p.schema))]))
    if isinstance(p, Projection):
        return _tag("Projection", _obj([("expr", _exprs(p.expr)), ("input", _plan(p.input)),
                                        ("schema", _schema(plan_schema(p)))]))
    if isinstance(p, Selection):
        return _tag("Selection", _obj([("expr", _expr(p.expr)), ("input", _plan(p.input))]))
    if isinstance(p, Aggregate):
        return _tag("Aggregate", _obj([("input", _plan(p.input)), ("group_expr", _exprs(p.group_expr)),
                                       ("aggr_expr", _exprs(p.aggr_expr)), ("schema", _schema(p.schema))]))
    if isinstance(p, Sort):
        return _tag("Sort", _obj([("expr", _exprs(p.expr)), ("input", _plan(p.input)),
                                  ("schema", _schema(p.schema))]))
    if isinstance(p, TableScan):
        return _tag("TableScan", _obj([("schema_name", _str(getattr(p, "schema_name", ""))),
                                       ("table_name", _str(p.table_name)), ("schema", _schema(p.schema)),
                                       ("projection", _projection(getattr(p, "projection", None)))]))
    if isinstance(p, EmptyRelation):
        return _tag("EmptyRelation", _obj([("schema", _schema(p.schema))]))
    raise TypeError("not a LogicalPlan: %r" % (p,))


def to_json(x) -> str:
    """serde_json::to_string of a LogicalPlan, Expr, ScalarValue, Schema,
    Field, DataSourceMeta or PhysicalPlan."""
    if isinstance(x, Expr):
        return _expr(x)
    if isinstance(x, ScalarValue):
        return _scalar(x)
    if isinstance(x, Schema):
        return _schema(x)
    if isinstance(x, Field):
        return _field(x)
    if isinstance(x, CsvFile):
        return _tag("CsvFile", _obj([("filename", _str(x.filename)), ("schema", _schema(x.schema)),
                                     ("has_header", "true" if x.has_header else "false"),
                                     ("projection", _projection(x.projection))]))
    if isinstance(x, ParquetFile):
        return _tag("ParquetFile", _obj([("filename", _str(x.filename)), ("schema", _schema(x.schema)),
                                         ("projection", _projection(x.projection))]))
    if isinstance(x, Interactive):
        return _tag("Interactive", _obj([("plan", _plan(x.plan))]))
    if isinstance(x, Write):
        return _tag("Write", _obj([("plan", _plan(x.plan)), ("filename", _str(x.filename)), ("kind", _str(x.kind))]))
    if isinstance(x, Show):
        return _tag("Show", _obj([("plan", _plan(x.plan)), ("count", str(int(x.count)))]))
    return _plan(x)


# ------------------------------------------------ decode
class WireError(ValueError):
    pass


def _variant(j, what):
    if isinstance(j, str):
        return j, None
    if isinstance(j, dict) and len(j) == 1:
        return next(iter(j.items()))
    raise WireError("expected an externally tagged %s, got %r" % (what, j))


def _de_datatype(j):
    name, body = _variant(j, "DataType")
    if name == "Struct":
        return StructType(tuple(_de_field(f) for f in body))
    if name == "List":
        return ListType(_de_datatype(body))
    if body is not None or name not in DataType.__members__ or name == "Null":
        raise WireError("unknown DataType %r" % (j,))
    return DataType[name]


def _de_field(j) -> Field:
    f = Field(j["name"], DataType.Null, bool(j["nullable"]))
    f.data_type = _de_datatype(j["data_type"])
    return f


def _de_schema(j) -> Schema:
    return Schema([_de_field(f) for f in j["fields"]])


def _de_scalar(j) -> ScalarValue:
    name, body = _variant(j, "ScalarValue")
    if name == "Null" and body is None:
        return ScalarValue(DataType.Null)
    if name not in DataType.__members__ or body is None:
        raise WireError("unknown ScalarValue %r" % (j,))
    t = DataType[name]
    if t == DataType.Float32:  # f32's shortest digits name one f32
        import numpy as np
        return ScalarValue(t, float(np.float32(float(body))))
    if t == DataType.Float64:
        return ScalarValue(t, float(body))
    if t == DataType.Utf8:
        return ScalarValue(t, str(body))
    if t == DataType.Boolean:
        return ScalarValue(t, bool(body))
    return ScalarValue(t, int(body))


def _de_expr(j) -> Expr:
    name, b = _variant(j, "Expr")
    if name == "Column":
        return Column(int(b))
    if name == "Literal":
        return Literal(_de_scalar(b))
    if name == "BinaryExpr":
        return BinaryExpr(_de_expr(b["left"]), Operator[b["op"]], _de_expr(b["right"]))
    if name == "IsNotNull":
        return IsNotNull(_de_expr(b))
    if name == "IsNull":
        return IsNull(_de_expr(b))
    if name == "Cast":
        return Cast(_de_expr(b["expr"]), _de_datatype(b["data_type"]))
    if name == "Sort":
        return SortExpr(_de_expr(b["expr"]), bool(b["asc"]))
    if name in ("ScalarFunction", "AggregateFunction"):
        cls = AggregateFunction if name == "AggregateFunction" else ScalarFunction
        return cls(b["name"], tuple(_de_expr(a) for a in b["args"]), _de_datatype(b["return_type"]))
    raise WireError("unknown Expr variant %r" % name)


def _de_plan(j):
    from .execution.context import Aggregate, Projection, Selection, TableScan
    name, b = _variant(j, "LogicalPlan")
    if name == "Limit":
        return Limit(int(b["limit"]), _de_plan(b["input"]), _de_schema(b["schema"]))
    if name == "Projection":
        return Projection([_de_expr(e) for e in b["expr"]], _de_plan(b["input"]), _de_schema(b["schema"]))
    if name == "Selection":
        return Selection(_de_expr(b["expr"]), _de_plan(b["input"]))
    if name == "Aggregate":
        return Aggregate(_de_plan(b["input"]), [_de_expr(e) for e in b["group_expr"]],
                         [_de_expr(e) for e in b["aggr_expr"]], _de_schema(b["schema"]))
    if name == "Sort":
        return Sort([_de_expr(e) for e in b["expr"]], _de_plan(b["input"]), _de_schema(b["schema"]))
    if name == "TableScan":
        t = TableScan(b["table_name"], _de_schema(b["schema"]))
        t.schema_name = b["schema_name"]
        t.projection = None if b["projection"] is None else [int(i) for i in b["projection"]]
        return t
    if name == "EmptyRelation":
        return EmptyRelation(_de_schema(b["schema"]))
    raise WireError("unknown LogicalPlan variant %r" % name)


_PHYSICAL = ("Interactive", "Write", "Show")
_META = ("CsvFile", "ParquetFile")


def from_json(s, kind: str = "LogicalPlan"):
    """serde_json::from_str::<kind>: kind is one of LogicalPlan, Expr,
    ScalarValue, Schema, DataSourceMeta, PhysicalPlan."""
    j = json.loads(s)
    if kind == "Expr":
        return _de_expr(j)
    if kind == "ScalarValue":
        return _de_scalar(j)
    if kind == "Schema":
        return _de_schema(j)
    if kind == "DataSourceMeta":
        name, b = _variant(j, "DataSourceMeta")
        proj = None if b.get("projection") is None else [int(i) for i in b["projection"]]
        if name == "CsvFile":
            return CsvFile(b["filename"], _de_schema(b["schema"]), bool(b["has_header"]), proj)
        if name == "ParquetFile":
            return ParquetFile(b["filename"], _de_schema(b["schema"]), proj)
        raise WireError("unknown DataSourceMeta variant %r" % name)
    if kind == "PhysicalPlan":
        name, b = _variant(j, "PhysicalPlan")
        if name == "Interactive":
            return Interactive(_de_plan(b["plan"]))
        if name == "Write":
            return Write(_de_plan(b["plan"]), b["filename"], b["kind"])
        if name == "Show":
            return Show(_de_plan(b["plan"]), int(b["count"]))
        raise WireError("unknown PhysicalPlan variant %r" % name)
    if kind == "LogicalPlan":
        return _de_plan(j)
    raise ValueError("unknown kind %r" % kind)


# ------------------------------------------------ Arrow IPC results
def _pa_type(t):
    import pyarrow as pa
    return {DataType.Boolean: pa.bool_(), DataType.Int8: pa.int8(), DataType.Int16: pa.int16(),
            DataType.Int32: pa.int32(), DataType.Int64: pa.int64(), DataType.UInt8: pa.uint8(),
            DataType.UInt16: pa.uint16(), DataType.UInt32: pa.uint32(), DataType.UInt64: pa.uint64(),
            DataType.Float32: pa.float32(), DataType.Float64: pa.float64(), DataType.Utf8: pa.utf8()}[DataType(t)]


def to_arrow_array(a):
    """One of our Arrays (host or device) as a pyarrow array over the same
    Arrow layout (values / validity / offsets buffers, zero-copy from host)."""
    import numpy as np
    import pyarrow as pa
    a = a.cpu()
    t = _pa_type(a.data_type)
    valid = None
    if a.null_count and a.validity is not None:
        valid = pa.py_buffer(a.validity.numpy().view(np.uint8)[: (a.length + 7) // 8].tobytes())
    if a.data_type == DataType.Utf8:
        offs = a.offsets.numpy().astype(np.int32, copy=False)[: a.length + 1]
        data = a.values.numpy().view(np.uint8)[: int(offs[-1]) if a.length else 0]
        return pa.Array.from_buffers(t, a.length, [valid, pa.py_buffer(offs.tobytes()), pa.py_buffer(data.tobytes())],
                                     a.null_count)
    if a.data_type == DataType.Boolean:
        nb = (a.length + 7) // 8
    else:
        nb = a.length * a.data_type.width
    vals = a.values.numpy().view(np.uint8)[:nb]
    return pa.Array.from_buffers(t, a.length, [valid, pa.py_buffer(vals.tobytes())], a.null_count)


def _pa_schema(schema: Schema):
    import pyarrow as pa
    return pa.schema([pa.field(f.name, _pa_type(f.data_type), f.nullable) for f in schema.fields])


def _pa_batch(pschema, b):
    import pyarrow as pa
    return pa.record_batch([to_arrow_array(c) for c in b.columns], schema=pschema)


def _write_stream(pschema, pbatches) -> bytes:
    import pyarrow as pa
    sink = pa.BufferOutputStream()
    with pa.ipc.new_stream(sink, pschema) as w:
        for b in pbatches:
            w.write_batch(b)
    return sink.getvalue().to_pybytes()


def ipc_stream(schema: Schema, batches) -> bytes:
    """Arrow IPC stream (schema message, one record batch message per batch,
    end-of-stream marker) of RecordBatches."""
    pschema = _pa_schema(schema)
    return _write_stream(pschema, [_pa_batch(pschema, b) for b in batches])


def run_physical_plan(ctx, payload) -> bytes:
    """Worker: a serde_json PhysicalPlan in, the result as an Arrow IPC stream
    out. Interactive runs the plan; Show stops after `count` rows; Write is
    not a worker result (NotImplemented, as the reference has no executor for
    it). The LogicalPlan runs through ``ctx.execute`` -- Selection /
    Projection / Aggregate on the device."""
    from .execution.error import ExecutionError
    pp = from_json(payload, "PhysicalPlan")
    if isinstance(pp, Write):
        raise ExecutionError("NotImplemented", "PhysicalPlan::Write in a worker")
    rel = ctx.execute(pp.plan)
    limit = pp.count if isinstance(pp, Show) else None
    pbatches, rows, pschema = [], 0, None
    while limit is None or rows < limit:
        b = rel.next()
        if b is None:
            break
        if pschema is None:
            pschema = _pa_schema(b.schema)
        pb = _pa_batch(pschema, b)
        if limit is not None and rows + pb.num_rows > limit:
            pb = pb.slice(0, limit - rows)
        rows += pb.num_rows
        pbatches.append(pb)
    if pschema is None:
        pschema = _pa_schema(rel.schema())
    return _write_stream(pschema, pbatches)
