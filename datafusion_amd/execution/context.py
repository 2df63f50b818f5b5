"""ExecutionContext (src/execution/context.rs:32-164): register data sources,
turn a LogicalPlan (or SQL, via the host planner) into the relation tree
Projection(Selection?(TableScan)) whose per-batch work runs on the GPU."""
from __future__ import annotations

from typing import Dict

from ..arrow import Field, Schema
from ..logicalplan import Column, DataType, Expr, PlanError, expr_to_field_name_type
from .error import ExecutionError
from .aggregate import AggregateRelation
from .expression import compile_expr, compile_scalar_expr
from .filter import FilterRelation
from .projection import ProjectRelation
from .relation import DataSourceRelation, Relation


class TableScan:
    """LogicalPlan::TableScan { schema_name, table_name, schema, projection } (logicalplan.rs:337-343)."""

    def __init__(self, table_name: str, schema: Schema, schema_name: str = "", projection=None):
        self.table_name = table_name
        self.schema = schema
        self.schema_name = schema_name
        self.projection = projection


class Selection:
    def __init__(self, expr: Expr, input):
        self.expr = expr
        self.input = input


class Projection:
    def __init__(self, expr, input, schema: Schema = None):
        self.expr = list(expr)
        self.input = input
        self.schema = schema


class Aggregate:
    """LogicalPlan::Aggregate { input, group_expr, aggr_expr, schema } (logicalplan.rs:324-329)."""

    def __init__(self, input, group_expr, aggr_expr, schema: Schema = None):
        self.input = input
        self.group_expr = list(group_expr)
        self.aggr_expr = list(aggr_expr)
        self.schema = schema


class ExecutionContext:
    def __init__(self, device=None, flags: int = 0, coalesce: int = 256):
        """coalesce > 1: Selection / Projection relations read up to that many
        input batches (at most 2^20 rows) ahead and run them as one device call
        (dfmi_filter_project_batches / dfmi_filter_project_host_batches), still
        returning one output batch per input batch -- at csv_sql.rs:49's
        1024-row batches one call per batch would cost a GPU round trip each.
        coalesce=1: one call per pull."""
        self.datasources: Dict[str, object] = {}
        self.device = device
        self.flags = flags
        self.coalesce = coalesce

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
            return FilterRelation(input_rel, rt, input_schema, self.device, self.flags, self.coalesce)
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
            return ProjectRelation(input_rel, compiled, project_schema, self.device, self.flags, self.coalesce)
        if isinstance(plan, Aggregate):
            return self._execute_aggregate(plan)
        raise ExecutionError("NotImplemented", "unimplemented!() plan %r" % type(plan).__name__)

    def _execute_aggregate(self, plan: "Aggregate") -> Relation:
        """The Aggregate arm the reference lacks (context.rs:161 unimplemented!()),
        under DFMI_FLAG_EXT_AGGREGATE: the input's Selection fuses into the pass."""
        from .. import _abi
        if not (self.flags & _abi.DFMI_FLAG_EXT_AGGREGATE):
            raise ExecutionError("panic", "not yet implemented")
        if len(plan.group_expr) > 1:
            raise ExecutionError("NotImplemented", "GROUP BY over more than one expression")
        inp, pred = plan.input, None
        if isinstance(inp, Selection):
            source = self.execute(inp.input)
            pred = compile_scalar_expr(self, inp.expr, source.schema(), self.flags)
        else:
            source = self.execute(inp)
        input_schema = source.schema()
        key = None
        fields = []
        if plan.group_expr:  # GROUP BY extension: the key column first (sqlplanner.rs:108-111)
            key = compile_scalar_expr(self, plan.group_expr[0], input_schema, self.flags)
            fields.append(Field(key.get_name(), DataType(key.get_type()), True))
        aggs = [compile_expr(self, e, input_schema, self.flags) for e in plan.aggr_expr]
        fields += [Field(e.name, e.return_type, True) for e in plan.aggr_expr]  # sqlplanner.rs:385-389
        return AggregateRelation(source, pred, aggs, Schema(fields), self.device, self.flags, key)
