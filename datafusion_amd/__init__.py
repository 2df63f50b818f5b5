"""datafusion_amd — MI355X-native Selection + Projection path of
ariesdevil/datafusion (v0.5.1): the reference's ExecutionContext / Relation /
compile_scalar_expr surface over a C ABI (include/dfmi.h) whose work runs as
hand-written CDNA4 HIP kernels (csrc/kernels.hip)."""
from . import logicalplan
from .logicalplan import (BinaryExpr, Cast, Column, DataType, Expr, Literal, Operator, ScalarValue)

__all__ = ["logicalplan", "BinaryExpr", "Cast", "Column", "DataType", "Expr", "Literal", "Operator",
           "ScalarValue"]
