"""End to end from a CSV file: the native reader (pinned batches, parsed one
batch ahead) feeding the pipelined host entry point through ctx.sql, against
the oracle over the restatement reader's batches of the same file."""
import numpy as np
import pytest

from datafusion_amd.arrow import Field, Schema
from datafusion_amd.execution import CsvDataSource, ExecutionContext, NativeCsvDataSource
from datafusion_amd.logicalplan import DataType
from oracle_ffi import oracle_filter_project

pytestmark = pytest.mark.gpu


def test_csv_sql_end_to_end(tmp_path):
    rng = np.random.default_rng(21)
    n = 250_000
    a, b, c = rng.random(n), rng.random(n), rng.standard_normal(n)
    words = ["w%d" % i + "x" * (i % 9) for i in range(50)]
    p = tmp_path / "t.csv"
    with open(p, "w") as f:
        f.write("a,b,c,s\n")
        for i in range(n):
            cs = "" if i % 13 == 0 else repr(float(c[i]))
            f.write("%r,%r,%s,%s\n" % (float(a[i]), float(b[i]), cs, words[i % 50]))
    schema = Schema([Field("a", DataType.Float64, False), Field("b", DataType.Float64, False),
                     Field("c", DataType.Float64, True), Field("s", DataType.Utf8, False)])
    sql = "SELECT a, s, a * b + c FROM t WHERE a > 0.3 AND b < 0.8"
    ctx = ExecutionContext()
    ctx.register_datasource("t", NativeCsvDataSource(schema, str(p), True, 65536))
    rel = ctx.sql(sql)
    got = []
    while True:
        bt = rel.next()
        if bt is None:
            break
        got.append([col.cpu() for col in bt.columns])
    assert len(got) == (n + 65535) // 65536
    from datafusion_amd.sqlplanner import SqlToRel
    plan = SqlToRel(ctx).sql_to_rel(sql)
    ref_src = CsvDataSource(schema, str(p), True, 65536)
    for g in got:
        rb = ref_src.next()
        ref = oracle_filter_project(schema, rb, plan.input.expr, plan.expr, 0)
        for (name, r), d in zip(ref, g):
            assert d.length == r.length and d.null_count == r.null_count
            if r.data_type == DataType.Utf8:
                assert d.to_pylist() == r.to_pylist()
            else:
                m = r.valid_mask()
                assert np.array_equal(d.numpy_values().view(np.uint64)[m], r.numpy_values().view(np.uint64)[m])
