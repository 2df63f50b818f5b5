"""compile_scalar_expr / RuntimeExpr (src/execution/expression.rs:29-78, :244-451).

The compiled closure of the reference is replaced by a dfmi_program handle:
compile-time checks, names and types come from libdfmi
(dfmi_compile_scalar_expr), evaluation happens in the fused HIP pass.
"""
from __future__ import annotations

import ctypes as C

from .. import _abi
from ..arrow import Schema
from ..logicalplan import AggregateFunction, DataType, Expr
from .error import ExecutionError


class RuntimeExpr:
    """RuntimeExpr::Compiled { name, f, t } — f is a device program."""

    def __init__(self, expr: Expr, handle: int, schema: Schema, flags: int):
        self.expr = expr
        self._handle = C.c_void_p(handle)
        self.flags = flags
        L = _abi.lib()
        self.name = L.dfmi_program_name(self._handle).decode("utf-8", errors="surrogateescape")
        self.t = DataType(L.dfmi_program_type(self._handle))
        self.input_schema = schema

    @property
    def handle(self) -> C.c_void_p:
        return self._handle

    def get_name(self) -> str:
        return self.name

    def get_type(self) -> DataType:
        return self.t

    def __del__(self):
        h = getattr(self, "_handle", None)
        if h is not None and h.value:
            try:
                _abi.lib().dfmi_program_free(h)
            except Exception:
                pass
            self._handle = C.c_void_p(0)


def schema_struct(schema: Schema):
    return _abi.make_schema([(f.name, f.data_type, f.nullable) for f in schema.fields])


def compile_scalar_expr(ctx, expr: Expr, input_schema: Schema, flags: int = None) -> RuntimeExpr:
    """expression.rs:244 — raises ExecutionError exactly where the reference's
    compile_scalar_expr returns Err."""
    if flags is None:
        flags = getattr(ctx, "flags", 0) if ctx is not None else 0
    nodes = _abi.PostfixNodes(expr.to_postfix())
    sch, keep = schema_struct(input_schema)
    out = C.c_void_p()
    err = _abi.dfmi_error()
    rc = _abi.lib().dfmi_compile_scalar_expr(nodes.array, nodes.length, C.byref(sch), flags,
                                            C.byref(out), C.byref(err))
    if rc != _abi.DFMI_OK:
        raise ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
    return RuntimeExpr(expr, out.value, input_schema, flags)


class AggregateExpr:
    """RuntimeExpr::AggregateFunction { name, f, args, t } (expression.rs:51-56):
    a dfmi_aggregate handle over the compiled argument (DFMI_FLAG_EXT_AGGREGATE)."""

    def __init__(self, expr: AggregateFunction, handle: int, arg: RuntimeExpr):
        self.expr = expr
        self.arg = arg
        self._handle = C.c_void_p(handle)
        L = _abi.lib()
        self.name = L.dfmi_aggregate_name(self._handle).decode("utf-8", errors="surrogateescape")
        self.t = DataType(L.dfmi_aggregate_type(self._handle))

    @property
    def handle(self) -> C.c_void_p:
        return self._handle

    def get_name(self) -> str:
        return self.name

    def get_type(self) -> DataType:
        return self.t

    def __del__(self):
        h = getattr(self, "_handle", None)
        if h is not None and h.value:
            try:
                _abi.lib().dfmi_aggregate_free(h)
            except Exception:
                pass
            self._handle = C.c_void_p(0)


def compile_expr(ctx, expr: Expr, input_schema: Schema, flags: int = None):
    """expression.rs:81-116: an AggregateFunction compiles its single argument
    with compile_scalar_expr and maps the name to an AggregateType (anything
    but min/max/count/sum panics); every other expression is
    compile_scalar_expr."""
    if flags is None:
        flags = getattr(ctx, "flags", 0) if ctx is not None else 0
    if not isinstance(expr, AggregateFunction):
        return compile_scalar_expr(ctx, expr, input_schema, flags)
    if len(expr.args) != 1:  # assert_eq!(1, args.len())
        raise ExecutionError("panic", "assertion failed: `(left == right)`\n  left: `1`,\n right: `%d`"
                             % len(expr.args))
    arg = compile_scalar_expr(ctx, expr.args[0], input_schema, flags)
    out = C.c_void_p()
    err = _abi.dfmi_error()
    rc = _abi.lib().dfmi_compile_aggregate(expr.name.encode("utf-8"), arg.handle, int(expr.return_type), flags,
                                          C.byref(out), C.byref(err))
    if rc != _abi.DFMI_OK:
        raise ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
    return AggregateExpr(expr, out.value, arg)
