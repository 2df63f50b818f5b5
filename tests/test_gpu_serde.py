"""Worker path (datafusion_amd/serde.py run_physical_plan): a serde_json
PhysicalPlan runs on the device and returns an Arrow IPC stream equal to the
oracle's result of the same plan."""
import numpy as np
import pyarrow as pa
import pytest

from datafusion_amd import serde
from datafusion_amd.execution import ExecutionContext, MemoryDataSource
from datafusion_amd.sqlplanner import SqlToRel
from golden_cases import CITIES, load_batch
from oracle_ffi import oracle_filter_project

pytestmark = pytest.mark.gpu

SQL = "SELECT city, lat, lng, lat + lng FROM cities WHERE lat > 51.0 AND lat < 53"


def _ctx():
    ctx = ExecutionContext()
    batch = load_batch(CITIES, "uk_cities.csv", has_header=True)
    ctx.register_datasource("cities", MemoryDataSource(CITIES, [batch]))
    return ctx, batch


def test_interactive_plan_to_ipc_matches_oracle():
    ctx, batch = _ctx()
    plan = SqlToRel(ctx).sql_to_rel(SQL)
    payload = serde.to_json(serde.Interactive(plan))
    t = pa.ipc.open_stream(serde.run_physical_plan(ctx, payload)).read_all()
    ref = oracle_filter_project(CITIES, batch, plan.input.expr, plan.expr, 0)
    assert t.num_rows == 18 and t.schema.names == [name for name, _ in ref]
    assert t.column(0).to_pylist() == ref[0][1].to_pylist()
    for i in (1, 2, 3):
        got = t.column(i).to_numpy().view(np.uint64)
        assert np.array_equal(got, ref[i][1].numpy_values().view(np.uint64))


def test_show_plan_truncates():
    ctx, _ = _ctx()
    plan = SqlToRel(ctx).sql_to_rel(SQL)
    t = pa.ipc.open_stream(serde.run_physical_plan(ctx, serde.to_json(serde.Show(plan, 5)))).read_all()
    assert t.num_rows == 5 and t.column(0).to_pylist()[0] == "Solihull, Birmingham, UK"
