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


def _plan_line(plan, indent: int) -> str:
    """LogicalPlan::fmt_with_indent (logicalplan.rs:362-434): each node on its
    own line, two spaces per level -- the plan's Debug string, which the
    reference prints on every execute (context.rs:104) and its planner tests
    compare (sqlplanner.rs:733-740)."""
    head = ("\n" + "  " * indent) if indent > 0 else ""
    return head + plan._node_debug() + (_plan_line(plan.input, indent + 1) if getattr(plan, "input", None) is not None
                                         else "")


class _Plan:
    def __repr__(self) -> str:  # impl fmt::Debug for LogicalPlan (logicalplan.rs:436-440)
        return _plan_line(self, 0)


class EmptyRelation(_Plan):
    """LogicalPlan::EmptyRelation { schema } (logicalplan.rs:344): SELECT without FROM."""

    def __init__(self, schema: Schema = None):
        self.schema = schema if schema is not None else Schema([])
        self.input = None

    def _node_debug(self):
        return "EmptyRelation"


class TableScan(_Plan):
    """LogicalPlan::TableScan { schema_name, table_name, schema, projection } (logicalplan.rs:337-343)."""

    def __init__(self, table_name: str, schema: Schema, schema_name: str = "default", projection=None):
        self.table_name = table_name
        self.schema = schema
        self.schema_name = schema_name
        self.projection = projection
        self.input = None

    def _node_debug(self):
        proj = "None" if self.projection is None else "Some([%s])" % ", ".join(str(i) for i in self.projection)
        return "TableScan: %s projection=%s" % (self.table_name, proj)


class Selection(_Plan):
    def __init__(self, expr: Expr, input):
        self.expr = expr
        self.input = input

    def _node_debug(self):
        return "Selection: %r" % (self.expr,)


class Projection(_Plan):
    def __init__(self, expr, input, schema: Schema = None):
        self.expr = list(expr)
        self.input = input
        self.schema = schema

    def _node_debug(self):
        return "Projection: " + ", ".join(repr(e) for e in self.expr)


class Aggregate(_Plan):
    """LogicalPlan::Aggregate { input, group_expr, aggr_expr, schema } (logicalplan.rs:324-329)."""

    def __init__(self, input, group_expr, aggr_expr, schema: Schema = None):
        self.input = input
        self.group_expr = list(group_expr)
        self.aggr_expr = list(aggr_expr)
        self.schema = schema

    def _node_debug(self):  # "groupBy=[{:?}]" of a Vec<Expr>: [[#4]]
        return "Aggregate: groupBy=[[%s]], aggr=[[%s]]" % (", ".join(repr(e) for e in self.group_expr),
                                                           ", ".join(repr(e) for e in self.aggr_expr))


class Sort(_Plan):
    """LogicalPlan::Sort { expr, input, schema } (logicalplan.rs:331-335): planned, not executable
    (context.rs:161 unimplemented!())."""

    def __init__(self, expr, input, schema: Schema = None):
        self.expr = list(expr)
        self.input = input
        self.schema = schema

    def _node_debug(self):
        return "Sort: " + ", ".join(repr(e) for e in self.expr)


class Limit(_Plan):
    """LogicalPlan::Limit { limit, input, schema } (logicalplan.rs:310-314): planned, not executable."""

    def __init__(self, limit: int, input, schema: Schema = None):
        self.limit = int(limit)
        self.input = input
        self.schema = schema

    def _node_debug(self):
        return "Limit: %d" % self.limit


def exprlist_to_fields(exprs, input_schema: Schema):
    """exprlist_to_fields / expr_to_field (context.rs:173-209)."""
    fields = []
    for e in exprs:
        if isinstance(e, Column):
            fields.append(input_schema.fields[e.index])
        else:
            try:
                name, t = expr_to_field_name_type(e, input_schema)
            except PlanError as err:
                raise ExecutionError("panic", str(err))
            fields.append(Field(name, t, True))
    return fields


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

    def function_meta(self, name: str):
        """ExecutionContextSchemaProvider::get_function_meta (context.rs:222-224): unimplemented!()."""
        raise ExecutionError("panic", "not yet implemented")

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
            project_schema = Schema(exprlist_to_fields(plan.expr, input_schema))
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
        if len(plan.group_expr) > 4:
            raise ExecutionError("NotImplemented", "device program limit: more than 4 GROUP BY expressions")
        inp, pred = plan.input, None
        if isinstance(inp, Selection):
            source = self.execute(inp.input)
            pred = compile_scalar_expr(self, inp.expr, source.schema(), self.flags)
        else:
            source = self.execute(inp)
        input_schema = source.schema()
        keys = []
        fields = []
        for g in plan.group_expr:  # GROUP BY extension: the key columns first (sqlplanner.rs:106-109)
            k = compile_scalar_expr(self, g, input_schema, self.flags)
            keys.append(k)
            fields.append(Field(k.get_name(), DataType(k.get_type()), True))
        aggs = [compile_expr(self, e, input_schema, self.flags) for e in plan.aggr_expr]
        fields += [Field(e.name, e.return_type, True) for e in plan.aggr_expr]  # sqlplanner.rs:385-389
        return AggregateRelation(source, pred, aggs, Schema(fields), self.device, self.flags, keys or None)
