"""The host planner's plans against the reference's own planner tests
(sqlplanner.rs:528-666): the SQL of every quick_test (:733-740) planned over
MockSchemaProvider's `person` schema and `sqrt` function (:742-770) and
formatted with LogicalPlan's Debug (logicalplan.rs:263-303, :362-440) --
byte for byte the expected string, including the planner's implicit casts
that decide which expressions reach the evaluator (`CAST(#3 AS Int64) GtEq
Int64(21)` for the Int32 `age`, which compile_scalar_expr then rejects as
a Cast of a column, expression.rs:281-282). The expected strings are kept
as data in tests/golden/sqlplanner_plans.json."""
import json
import os

import pytest

from datafusion_amd.arrow import Field, Schema
from datafusion_amd.execution.error import ExecutionError
from datafusion_amd.execution.expression import compile_scalar_expr
from datafusion_amd.logicalplan import DataType
from datafusion_amd.sqlplanner import SqlToRel

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "sqlplanner_plans.json")))


class MockSchemaProvider:
    """sqlplanner.rs:742-770."""

    def table_schema(self, name):
        if name == "person":
            return Schema([Field(n, DataType[t], False) for n, t in GOLD["person"]])
        return None

    def function_meta(self, name):
        fm = GOLD["functions"].get(name)
        return None if fm is None else ([DataType[t] for t in fm[0]], DataType[fm[1]])


@pytest.mark.parametrize("case", GOLD["cases"], ids=[c["test"] for c in GOLD["cases"]])
def test_plan_debug_string_matches_reference(case):
    plan = SqlToRel(MockSchemaProvider()).sql_to_rel(case["sql"])
    assert repr(plan) == case["expected"], case["test"]


def test_planner_cast_of_column_is_rejected_by_the_evaluator():
    """`CAST(#3 AS Int64)` (the Int32 age against an Int64 literal,
    select_all_boolean_operators) is not executable: compile_scalar_expr
    refuses a Cast of a column with the reference's message
    (expression.rs:281-282). (The compound selection fails earlier, on its
    Utf8 literal, expression.rs:267-270.)"""
    case = next(c for c in GOLD["cases"] if c["test"] == "select_all_boolean_operators")
    plan = SqlToRel(MockSchemaProvider()).sql_to_rel(case["sql"])
    schema = MockSchemaProvider().table_schema("person")
    with pytest.raises(ExecutionError) as ei:
        compile_scalar_expr(None, plan.input.expr, schema)
    assert "column reference" in ei.value.message
