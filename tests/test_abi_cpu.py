"""CPU suite for the C ABI: libdfmi.so loads, exports every symbol
include/dfmi.h declares, and its compile_scalar_expr front end agrees with the
oracle on names, types and compile-time errors (no GPU needed)."""
import ctypes as C
import os
import random
import re

import pytest

from datafusion_amd import _abi
from datafusion_amd.arrow import Field, Schema
from datafusion_amd.execution.error import ExecutionError
from datafusion_amd.execution.expression import compile_scalar_expr
from datafusion_amd.logicalplan import (BinaryExpr, Cast, Column, DataType, Float64, Int64, IsNull, Literal,
                                        Operator, ScalarValue, Utf8, rust_float)
from oracle_ffi import oracle_compile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

S = Schema([Field("a", DataType.Int64, True), Field("b", DataType.Float64, True),
            Field("s", DataType.Utf8, True), Field("f", DataType.Boolean, True),
            Field("c", DataType.Float64, False), Field("i32", DataType.Int32, False)])


def test_header_symbols_exported():
    declared = set()
    for h in os.listdir(os.path.join(ROOT, "include")):
        hdr = open(os.path.join(ROOT, "include", h)).read()
        declared |= set(re.findall(r"\b(dfmi_[a-z0-9_]+)\s*\(", hdr))
    assert declared == set(_abi.EXPORTED)
    L = _abi.lib()
    for name in declared:
        assert hasattr(L, name), name


def test_struct_sizes_match_header():
    # layout of the ABI structs (x86-64 / LP64)
    assert C.sizeof(_abi.dfmi_column) == 56
    assert C.sizeof(_abi.dfmi_batch) == 24
    assert C.sizeof(_abi.dfmi_expr_node) == 48
    assert C.sizeof(_abi.dfmi_out_column) == 72
    assert C.sizeof(_abi.dfmi_error) == 504


def lib_compile(e, flags=0):
    try:
        r = compile_scalar_expr(None, e, S, flags)
        return ("ok", r.get_name(), r.get_type())
    except ExecutionError as x:
        return ("err", x.kind, x.message)


def ora_compile(e, flags=0):
    try:
        n, t = oracle_compile(e, S, flags)
        return ("ok", n, t)
    except ExecutionError as x:
        return ("err", x.kind, x.message)


FIXED = [
    Literal(Int64(5)), Literal(Float64(0.5)), Literal(Float64(1.0)), Literal(Float64(-0.0)),
    Literal(Float64(1e21)), Literal(Float64(1.5e-7)), Literal(Int64(-9223372036854775808)),
    Cast(Literal(Int64(53)), DataType.Float64), Cast(Literal(Int64(1)), DataType.Int32),
    Cast(Literal(Float64(1.5)), DataType.Int64), Cast(Column(0), DataType.Float64),
    Cast(BinaryExpr(Column(0), Operator.Plus, Column(0)), DataType.Float64),
    BinaryExpr(Column(0), Operator.Modulus, Column(0)), IsNull(Column(0)), Column(7),
    Literal(Utf8("w17")), Literal(Utf8('q"\n')), Literal(ScalarValue(DataType.Boolean, False)),
    Literal(ScalarValue(DataType.Null)),
    BinaryExpr(Column(1), Operator.Gt, Literal(Float64(51.0))),
    BinaryExpr(BinaryExpr(Column(1), Operator.Gt, Literal(Float64(51.0))), Operator.And,
               BinaryExpr(Column(1), Operator.Lt, Cast(Literal(Int64(53)), DataType.Float64))),
    BinaryExpr(Column(0), Operator.Gt, Column(1)),           # comparison_ops at run time
    BinaryExpr(Column(2), Operator.Eq, Column(2)),           # Utf8 comparison
    BinaryExpr(Column(0), Operator.And, Column(0)),          # boolean_ops panic at run time
    BinaryExpr(Column(3), Operator.Plus, Column(3)),         # math_ops at run time
    BinaryExpr(Column(5), Operator.Plus, Column(5)),         # Int32 math
]


@pytest.mark.parametrize("i", range(len(FIXED)))
def test_compile_matches_oracle(i):
    e = FIXED[i]
    assert lib_compile(e) == ora_compile(e)
    assert lib_compile(e, _abi.DFMI_FLAG_EXT_UTF8_COMPARE) == ora_compile(e, _abi.DFMI_FLAG_EXT_UTF8_COMPARE)


def _rand_expr(rng, depth):
    if depth == 0 or rng.random() < 0.25:
        k = rng.random()
        if k < 0.4:
            return Column(rng.randrange(6))
        if k < 0.6:
            return Literal(Int64(rng.randrange(-1000, 1000)))
        if k < 0.8:
            return Literal(Float64(rng.choice([0.5, -2.25, 1e-3, 3.0, 123456.789, 0.1 + 0.2])))
        if k < 0.9:
            return Cast(Literal(Int64(rng.randrange(100))), rng.choice([DataType.Float64, DataType.Int32]))
        return Literal(Utf8(rng.choice(["x", "w17", ""])))
    op = Operator(rng.randrange(13))
    return BinaryExpr(_rand_expr(rng, depth - 1), op, _rand_expr(rng, depth - 1))


def test_compile_random_matches_oracle():
    rng = random.Random(1234)
    for _ in range(400):
        e = _rand_expr(rng, rng.randrange(1, 5))
        for fl in (0, _abi.DFMI_FLAG_EXT_UTF8_COMPARE):
            assert lib_compile(e, fl) == ora_compile(e, fl), repr(e)


@pytest.mark.parametrize("v", [0.1, 1.0, 100.0, 1e21, 1e-7, 50.494344999999996, 3.0000000000000004, -0.0, 2.5e-308])
def test_rust_float_python_matches_library(v):
    # Python mirror and the C++ library format Rust floats the same way
    r = lib_compile(Literal(Float64(v)))
    assert r[1] == rust_float(v, False, False)
    r = lib_compile(BinaryExpr(Column(1), Operator.Gt, Literal(Float64(v))))
    assert r[1] == "#1 Gt Float64(%s)" % rust_float(v, False, True)
