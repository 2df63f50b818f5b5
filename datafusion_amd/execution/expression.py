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


def compile_expr(ctx, expr: Expr, input_schema: Schema) -> RuntimeExpr:
    """expression.rs:81-119. Aggregates are outside this path."""
    if isinstance(expr, AggregateFunction):
        raise ExecutionError("NotImplemented", "aggregate expressions are not on the device path")
    return compile_scalar_expr(ctx, expr, input_schema)
