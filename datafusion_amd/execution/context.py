"""ExecutionContext (src/execution/context.rs:32-164): register data sources,
turn a LogicalPlan (or SQL, via the host planner) into the relation tree
Projection(Selection?(TableScan)) whose per-batch work runs on the GPU."""
from __future__ import annotations

from typing import Dict

from ..arrow import Field, Schema
from ..logicalplan import Column, Expr, PlanError, expr_to_field_name_type
from .error import ExecutionError
from .expression import compile_scalar_expr
from .filter import FilterRelation
from .projection import ProjectRelation
from .relation import DataSourceRelation, Relation


class TableScan:
    def __init__(self, table_name: str, schema: Schema):
        self.table_name = table_name
        self.schema = schema


class Selection:
    def __init__(self, expr: Expr, input):
        self.expr = expr
        self.input = input


class Projection:
    def __init__(self, expr, input, schema: Schema = None):
        self.expr = list(expr)
        self.input = input
        self.schema = schema


class ExecutionContext:
    def __init__(self, device=None, flags: int = 0):
        self.datasources: Dict[str, object] = {}
        self.device = device
        self.flags = flags

    def register_datasource(self, name: str, ds) -> None:
        self.datasources[name] = ds

    def sql(self, sql: str) -> Relation:
        from ..sqlplanner import SqlToRel
        plan = SqlToRel(self).sql_to_rel(sql)
        return self.execute(plan)

    def table_schema(self, name: str):
        ds = self.datasources.get(name)
        return ds.schema() if ds is not None else None

    def execute(self, plan) -> Relation:
        """context.rs:103-163."""
        if isinstance(plan, TableScan):
            ds = self.datasources.get(plan.table_name)
            if ds is None:
                raise ExecutionError("General", "No table registered as '%s'" % plan.table_name)
            return DataSourceRelation(ds)
        if isinstance(plan, Selection):
            input_rel = self.execute(plan.input)
            input_schema = input_rel.schema()
            rt = compile_scalar_expr(self, plan.expr, input_schema, self.flags)
            return FilterRelation(input_rel, rt, input_schema, self.device, self.flags)
        if isinstance(plan, Projection):
            input_rel = self.execute(plan.input)
            input_schema = input_rel.schema()
            fields = []
            for e in plan.expr:  # exprlist_to_fields (context.rs:173-209)
                if isinstance(e, Column):
                    fields.append(input_schema.fields[e.index])
                else:
                    try:
                        name, t = expr_to_field_name_type(e, input_schema)
                    except PlanError as err:
                        raise ExecutionError("panic", str(err))
                    fields.append(Field(name, t, True))
            project_schema = Schema(fields)
            compiled = [compile_scalar_expr(self, e, input_schema, self.flags) for e in plan.expr]
            return ProjectRelation(input_rel, compiled, project_schema, self.device, self.flags)
        raise ExecutionError("NotImplemented", "unimplemented!() plan %r" % type(plan).__name__)
