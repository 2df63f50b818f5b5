"""Execution layer mirror (src/execution/)."""
from .context import ExecutionContext, Projection, Selection, TableScan
from .datasource import CsvDataSource, DataSource, MemoryDataSource, NativeCsvDataSource
from .error import ExecutionError
from .expression import RuntimeExpr, compile_expr, compile_scalar_expr
from .filter import FilterRelation
from .projection import ProjectRelation
from .relation import DataSourceRelation, Relation
