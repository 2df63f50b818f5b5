"""Host-side mirror of the reference's logical-plan vocabulary.

Restates (unchanged, as the north star requires) the types the hot path
consumes:
  * ``Operator``        — src/logicalplan.rs:67-81
  * ``ScalarValue``     — src/logicalplan.rs:93-129
  * ``Expr``            — src/logicalplan.rs:133-261 (get_type :167-195,
                          cast_to :197-212, Debug :263-303)
  * ``get_supertype``   — src/logicalplan.rs:443-551
  * ``can_coerce_from`` — src/logicalplan.rs:553-602

``Expr.to_postfix()`` flattens a tree into the ``dfmi_expr_node`` array that
crosses the C ABI (include/dfmi.h), children first, left before right — the
order compile_scalar_expr (expression.rs:244) evaluates them.
"""
from __future__ import annotations

import enum
import math
import struct
from dataclasses import dataclass
from typing import List, Optional, Sequence


class DataType(enum.IntEnum):
    """arrow::datatypes::DataType subset; values match dfmi_type."""
    Null = 0
    Boolean = 1
    Int8 = 2
    Int16 = 3
    Int32 = 4
    Int64 = 5
    UInt8 = 6
    UInt16 = 7
    UInt32 = 8
    UInt64 = 9
    Float32 = 10
    Float64 = 11
    Utf8 = 12

    def __repr__(self) -> str:  # arrow DataType Debug
        return self.name

    @property
    def width(self) -> int:
        return _WIDTH.get(self, 0)

    @property
    def is_numeric(self) -> bool:
        return DataType.Int8 <= self <= DataType.Float64


_WIDTH = {
    DataType.Int8: 1, DataType.UInt8: 1, DataType.Int16: 2, DataType.UInt16: 2,
    DataType.Int32: 4, DataType.UInt32: 4, DataType.Float32: 4,
    DataType.Int64: 8, DataType.UInt64: 8, DataType.Float64: 8,
}


class Operator(enum.IntEnum):
    """logicalplan::Operator; values match dfmi_operator."""
    Eq = 0
    NotEq = 1
    Lt = 2
    LtEq = 3
    Gt = 4
    GtEq = 5
    Plus = 6
    Minus = 7
    Multiply = 8
    Divide = 9
    Modulus = 10
    And = 11
    Or = 12

    def __repr__(self) -> str:
        return self.name


# --------------------------------------------------------------- formatting
def _shortest_digits(v: float, f32: bool):
    for p in range(1, 18):
        s = "%.*e" % (p - 1, v)
        back = float(s)
        if f32:
            ok = struct.unpack("f", struct.pack("f", back))[0] == struct.unpack("f", struct.pack("f", v))[0]
        else:
            ok = back == v
        if ok:
            break
    mant, exp = s.split("e")
    digits = mant.replace(".", "").rstrip("0") or "0"
    return digits, int(exp)


def rust_float(v: float, f32: bool = False, debug: bool = False) -> str:
    """Rust (2018) `{}` / `{:?}` of f64/f32: shortest round-trip digits, plain
    decimal, `{:?}` appends ".0" to integral values."""
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "inf" if v > 0 else "-inf"
    neg = math.copysign(1.0, v) < 0
    sign = "-" if neg and (v != 0.0 or debug) else ""
    a = abs(v)
    if a == 0.0:
        return sign + ("0.0" if debug else "0")
    d, e10 = _shortest_digits(a, f32)
    point = e10 + 1
    if point <= 0:
        out = "0." + "0" * (-point) + d
    elif point >= len(d):
        out = d + "0" * (point - len(d)) + (".0" if debug else "")
    else:
        out = d[:point] + "." + d[point:]
    return sign + out


def _rust_str_debug(s: str) -> str:
    out = ['"']
    for ch in s:
        c = ord(ch)
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\r":
            out.append("\\r")
        elif ch == "\t":
            out.append("\\t")
        elif ch == "\0":
            out.append("\\0")
        elif c < 0x20 or c == 0x7F:
            out.append("\\u{%x}" % c)
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


# ------------------------------------------------------------- ScalarValue
@dataclass(frozen=True)
class ScalarValue:
    """logicalplan::ScalarValue — ``dtype`` names the variant."""
    dtype: DataType
    value: object = None

    def get_datatype(self) -> DataType:
        if self.dtype == DataType.Null:
            raise NotImplementedError("ScalarValue::Null has no datatype")  # unimplemented!()
        return self.dtype

    def __repr__(self) -> str:  # derive(Debug)
        t = self.dtype
        if t == DataType.Null:
            return "Null"
        if t == DataType.Boolean:
            return "Boolean(%s)" % ("true" if self.value else "false")
        if t == DataType.Float64:
            return "Float64(%s)" % rust_float(float(self.value), False, True)
        if t == DataType.Float32:
            return "Float32(%s)" % rust_float(float(self.value), True, True)
        if t == DataType.Utf8:
            return "Utf8(%s)" % _rust_str_debug(self.value)
        return "%s(%d)" % (t.name, int(self.value))

    def display(self) -> str:  # format!("{}", nn) used by literal_array!
        t = self.dtype
        if t in (DataType.Float64, DataType.Float32):
            return rust_float(float(self.value), t == DataType.Float32, False)
        if t == DataType.Utf8:
            return str(self.value)
        if t == DataType.Boolean:
            return "true" if self.value else "false"
        return str(int(self.value))


def Int64(v: int) -> ScalarValue:
    return ScalarValue(DataType.Int64, int(v))


def Float64(v: float) -> ScalarValue:
    return ScalarValue(DataType.Float64, float(v))


def Utf8(v: str) -> ScalarValue:
    return ScalarValue(DataType.Utf8, v)


# ------------------------------------------------------------------- Expr
class Expr:
    """logicalplan::Expr. Subclasses mirror the enum variants."""

    def get_type(self, schema) -> DataType:
        raise NotImplementedError

    def cast_to(self, cast_to_type: DataType, schema) -> "Expr":
        """logicalplan.rs:197-212."""
        this_type = self.get_type(schema)
        if this_type == cast_to_type:
            return self
        if can_coerce_from(cast_to_type, this_type):
            return Cast(self, cast_to_type)
        raise PlanError("Cannot automatically convert %r to %r" % (this_type, cast_to_type))

    # builder helpers (logicalplan.rs:214-261)
    def eq(self, o): return BinaryExpr(self, Operator.Eq, o)
    def not_eq(self, o): return BinaryExpr(self, Operator.NotEq, o)
    def gt(self, o): return BinaryExpr(self, Operator.Gt, o)
    def gt_eq(self, o): return BinaryExpr(self, Operator.GtEq, o)
    def lt(self, o): return BinaryExpr(self, Operator.Lt, o)
    def lt_eq(self, o): return BinaryExpr(self, Operator.LtEq, o)

    def to_postfix(self) -> list:
        out: list = []
        self._postfix(out)
        return out

    def _postfix(self, out: list) -> None:
        raise NotImplementedError


class PlanError(Exception):
    pass


@dataclass(frozen=True, eq=True)
class Column(Expr):
    index: int

    def get_type(self, schema):
        return schema.field(self.index).data_type

    def __repr__(self):
        return "#%d" % self.index

    def _postfix(self, out):
        out.append(dict(kind=1, column=self.index))


@dataclass(frozen=True, eq=True)
class Literal(Expr):
    value: ScalarValue

    def get_type(self, schema):
        return self.value.get_datatype()

    def __repr__(self):
        return repr(self.value)

    def _postfix(self, out):
        v = self.value
        node = dict(kind=2, data_type=int(v.dtype))
        if v.dtype in (DataType.Float32, DataType.Float64):
            node["f64"] = float(v.value)
        elif v.dtype == DataType.Utf8:
            node["str"] = v.value.encode("utf-8")
        elif v.dtype == DataType.Boolean:
            node["i64"] = 1 if v.value else 0
        elif v.dtype != DataType.Null:
            iv = int(v.value)
            if iv >= 1 << 63:  # UInt64 bit pattern
                iv -= 1 << 64
            node["i64"] = iv
        out.append(node)


@dataclass(frozen=True, eq=True)
class BinaryExpr(Expr):
    left: Expr
    op: Operator
    right: Expr

    def get_type(self, schema):
        if self.op in (Operator.Eq, Operator.NotEq, Operator.Lt, Operator.LtEq,
                       Operator.Gt, Operator.GtEq, Operator.And, Operator.Or):
            return DataType.Boolean
        st = get_supertype(self.left.get_type(schema), self.right.get_type(schema))
        return st if st is not None else DataType.Utf8  # logicalplan.rs:190

    def __repr__(self):
        return "%r %r %r" % (self.left, self.op, self.right)

    def _postfix(self, out):
        self.left._postfix(out)
        self.right._postfix(out)
        out.append(dict(kind=3, op=int(self.op)))


@dataclass(frozen=True, eq=True)
class Cast(Expr):
    expr: Expr
    data_type: DataType

    def get_type(self, schema):
        return self.data_type

    def __repr__(self):
        return "CAST(%r AS %r)" % (self.expr, self.data_type)

    def _postfix(self, out):
        self.expr._postfix(out)
        out.append(dict(kind=4, data_type=int(self.data_type)))


@dataclass(frozen=True, eq=True)
class IsNull(Expr):
    expr: Expr

    def get_type(self, schema):
        return DataType.Boolean

    def __repr__(self):
        return "%r IS NULL" % (self.expr,)

    def _postfix(self, out):
        self.expr._postfix(out)
        out.append(dict(kind=5))


@dataclass(frozen=True, eq=True)
class IsNotNull(Expr):
    expr: Expr

    def get_type(self, schema):
        return DataType.Boolean

    def __repr__(self):
        return "%r IS NOT NULL" % (self.expr,)

    def _postfix(self, out):
        self.expr._postfix(out)
        out.append(dict(kind=6))


@dataclass(frozen=True, eq=True)
class ScalarFunction(Expr):
    name: str
    args: tuple
    return_type: DataType

    def get_type(self, schema):
        return self.return_type

    def __repr__(self):
        return "%s(%s)" % (self.name, ", ".join(repr(a) for a in self.args))

    def _postfix(self, out):
        for a in self.args:
            a._postfix(out)
        out.append(dict(kind=8, column=len(self.args), data_type=int(self.return_type),
                        str=self.name.encode()))


@dataclass(frozen=True, eq=True)
class SortExpr(Expr):
    """Expr::Sort { expr, asc } (logicalplan.rs:160, Debug :272-278): an
    ORDER BY key; compile_scalar_expr rejects it (expression.rs:446-449)."""
    expr: Expr
    asc: bool

    def get_type(self, schema):
        return self.expr.get_type(schema)

    def __repr__(self):
        return "%r %s" % (self.expr, "ASC" if self.asc else "DESC")

    def _postfix(self, out):
        self.expr._postfix(out)
        out.append(dict(kind=7, op=1 if self.asc else 0))


@dataclass(frozen=True, eq=True, repr=False)
class AggregateFunction(ScalarFunction):
    def _postfix(self, out):
        for a in self.args:
            a._postfix(out)
        out.append(dict(kind=9, column=len(self.args), data_type=int(self.return_type),
                        str=self.name.encode()))


# ------------------------------------------------------------ type rules
_I = DataType
_SUPER = {
    (_I.UInt8, _I.Int8): _I.Int8, (_I.UInt8, _I.Int16): _I.Int16, (_I.UInt8, _I.Int32): _I.Int32,
    (_I.UInt8, _I.Int64): _I.Int64, (_I.UInt16, _I.Int16): _I.Int16, (_I.UInt16, _I.Int32): _I.Int32,
    (_I.UInt16, _I.Int64): _I.Int64, (_I.UInt32, _I.Int32): _I.Int32, (_I.UInt32, _I.Int64): _I.Int64,
    (_I.UInt64, _I.Int64): _I.Int64, (_I.Int8, _I.UInt8): _I.Int8, (_I.Int16, _I.UInt8): _I.Int16,
    (_I.Int16, _I.UInt16): _I.Int16, (_I.Int32, _I.UInt8): _I.Int32, (_I.Int32, _I.UInt16): _I.Int32,
    (_I.Int32, _I.UInt32): _I.Int32, (_I.Int64, _I.UInt8): _I.Int64, (_I.Int64, _I.UInt16): _I.Int64,
    (_I.Int64, _I.UInt32): _I.Int64, (_I.Int64, _I.UInt64): _I.Int64,
    (_I.UInt8, _I.UInt8): _I.UInt8, (_I.UInt8, _I.UInt16): _I.UInt16, (_I.UInt8, _I.UInt32): _I.UInt32,
    (_I.UInt8, _I.UInt64): _I.UInt64, (_I.UInt8, _I.Float32): _I.Float32, (_I.UInt8, _I.Float64): _I.Float64,
    (_I.UInt16, _I.UInt8): _I.UInt16, (_I.UInt16, _I.UInt16): _I.UInt16, (_I.UInt16, _I.UInt32): _I.UInt32,
    (_I.UInt16, _I.UInt64): _I.UInt64, (_I.UInt16, _I.Float32): _I.Float32, (_I.UInt16, _I.Float64): _I.Float64,
    (_I.UInt32, _I.UInt8): _I.UInt32, (_I.UInt32, _I.UInt16): _I.UInt32, (_I.UInt32, _I.UInt32): _I.UInt32,
    (_I.UInt32, _I.UInt64): _I.UInt64, (_I.UInt32, _I.Float32): _I.Float32, (_I.UInt32, _I.Float64): _I.Float64,
    (_I.UInt64, _I.UInt8): _I.UInt64, (_I.UInt64, _I.UInt16): _I.UInt64, (_I.UInt64, _I.UInt32): _I.UInt64,
    (_I.UInt64, _I.UInt64): _I.UInt64, (_I.UInt64, _I.Float32): _I.Float32, (_I.UInt64, _I.Float64): _I.Float64,
    (_I.Int8, _I.Int8): _I.Int8, (_I.Int8, _I.Int16): _I.Int16, (_I.Int8, _I.Int32): _I.Int32,
    (_I.Int8, _I.Int64): _I.Int64, (_I.Int8, _I.Float32): _I.Float32, (_I.Int8, _I.Float64): _I.Float64,
    (_I.Int16, _I.Int8): _I.Int16, (_I.Int16, _I.Int16): _I.Int16, (_I.Int16, _I.Int32): _I.Int32,
    (_I.Int16, _I.Int64): _I.Int64, (_I.Int16, _I.Float32): _I.Float32, (_I.Int16, _I.Float64): _I.Float64,
    (_I.Int32, _I.Int8): _I.Int32, (_I.Int32, _I.Int16): _I.Int32, (_I.Int32, _I.Int32): _I.Int32,
    (_I.Int32, _I.Int64): _I.Int64, (_I.Int32, _I.Float32): _I.Float32, (_I.Int32, _I.Float64): _I.Float64,
    (_I.Int64, _I.Int8): _I.Int64, (_I.Int64, _I.Int16): _I.Int64, (_I.Int64, _I.Int32): _I.Int64,
    (_I.Int64, _I.Int64): _I.Int64, (_I.Int64, _I.Float32): _I.Float32, (_I.Int64, _I.Float64): _I.Float64,
    (_I.Float32, _I.Float32): _I.Float32, (_I.Float32, _I.Float64): _I.Float64,
    (_I.Float64, _I.Float32): _I.Float64, (_I.Float64, _I.Float64): _I.Float64,
    (_I.Utf8, _I.Utf8): _I.Utf8, (_I.Boolean, _I.Boolean): _I.Boolean,
}


def get_supertype(l: DataType, r: DataType) -> Optional[DataType]:
    """logicalplan.rs:443-451 (tries (l, r) then (r, l))."""
    return _SUPER.get((l, r), _SUPER.get((r, l)))


_INTS = (_I.Int8, _I.Int16, _I.Int32, _I.Int64)
_UINTS = (_I.UInt8, _I.UInt16, _I.UInt32, _I.UInt64)


def can_coerce_from(left: DataType, other: DataType) -> bool:
    """logicalplan.rs:553-602."""
    table = {
        _I.Int8: (_I.Int8,), _I.Int16: (_I.Int8, _I.Int16), _I.Int32: (_I.Int8, _I.Int16, _I.Int32),
        _I.Int64: _INTS, _I.UInt8: (_I.UInt8,), _I.UInt16: (_I.UInt8, _I.UInt16),
        _I.UInt32: (_I.UInt8, _I.UInt16, _I.UInt32), _I.UInt64: _UINTS,
        _I.Float32: _INTS + _UINTS + (_I.Float32,),
        _I.Float64: _INTS + _UINTS + (_I.Float32, _I.Float64),
    }
    return other in table.get(left, ())


def binary_expr_coerced(left: Expr, op: Operator, right: Expr, schema) -> BinaryExpr:
    """What SqlToRel::sql_to_rex builds for a binary operator
    (sqlplanner.rs:272-287): both sides cast to their supertype."""
    lt, rt = left.get_type(schema), right.get_type(schema)
    st = get_supertype(lt, rt)
    if st is None:
        raise PlanError("No common supertype found for binary operator %r with input types %r and %r"
                        % (op, lt, rt))
    return BinaryExpr(left.cast_to(st, schema), op, right.cast_to(st, schema))


def expr_to_field_name_type(e: Expr, schema):
    """context.rs:173-203 expr_to_field: the relation schema's (name, type)."""
    if isinstance(e, Column):
        f = schema.field(e.index)
        return f.name, f.data_type
    if isinstance(e, Literal):
        return "lit", e.value.get_datatype()
    if isinstance(e, AggregateFunction) or isinstance(e, ScalarFunction):
        return e.name, e.return_type
    if isinstance(e, Cast):
        return "cast", e.data_type
    if isinstance(e, BinaryExpr):
        st = get_supertype(e.left.get_type(schema), e.right.get_type(schema))
        if st is None:
            raise PlanError("called `Option::unwrap()` on a `None` value")
        return "binary_expr", st
    raise PlanError("Cannot determine schema type for expression %r" % (e,))
