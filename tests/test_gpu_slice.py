"""Sliced arrays on the device (dfmi_column.offset; arrow 0.12 ArrayData
offset, filter.rs:88-89,99-100): every entry point -- single batch in HBM
or host memory, coalesced batches in HBM or host memory, the aggregate
extension -- gives for a sliced batch exactly the oracle's result for it,
which equals the result for copies of the same rows (tests/test_slice_cpu.py).
Offsets that are not multiples of 64 rows exercise the bitmap shift."""
import numpy as np
import pytest

from datafusion_amd._abi import DFMI_FLAG_EXT_AGGREGATE, DFMI_FLAG_EXT_GATHER_ALL
from datafusion_amd.arrow import RecordBatch
from datafusion_amd.execution.engine import engine
from datafusion_amd.execution.error import ExecutionError
from datafusion_amd.execution.expression import compile_expr, compile_scalar_expr
from datafusion_amd.logicalplan import AggregateFunction, Column, DataType
from oracle_ffi import oracle_aggregate, oracle_filter_project
from test_gpu_parity import assert_same, run_both
from test_slice_cpu import QUERIES, SCHEMA, sliced, table

pytestmark = pytest.mark.gpu

FL = DFMI_FLAG_EXT_GATHER_ALL


@pytest.mark.parametrize("off", [1, 5, 8, 63, 64, 100, 4099])
def test_single_batch_sliced(off):
    t = table(40_000, seed=off)
    s = sliced(t, off, 40_000 - off - 17)
    for pred, projs in QUERIES:
        run_both(SCHEMA, s, pred, projs, FL)  # device (batch.to keeps the offset), host, chunked host


@pytest.mark.parametrize("host", [False, True])
def test_coalesced_sliced(host):
    t = table(20_000, seed=3)
    bs = [sliced(t, o, n) for o, n in ((0, 1024), (1, 1024), (77, 3000), (64, 64), (5000, 0), (9, 12_000))]
    eng = engine()
    for pred, projs in QUERIES:
        p = compile_scalar_expr(None, pred, SCHEMA, FL) if pred is not None else None
        cp = [compile_scalar_expr(None, e, SCHEMA, FL) for e in projs]
        if host:
            got, err = eng.filter_project_host_batches(p, cp, bs, FL)
        else:
            got, err = eng.filter_project_batches(p, cp, [b.to(eng.device) for b in bs], FL)
        assert err is None, err
        for b, g in zip(bs, got):
            for d, (_, r) in zip(g, oracle_filter_project(SCHEMA, b, pred, projs, FL)):
                assert_same(d.cpu(), r)


def test_aggregate_sliced():
    t = table(50_000, seed=9)
    s = sliced(t, 37, 40_000)
    fl = DFMI_FLAG_EXT_AGGREGATE | FL
    aggs = [AggregateFunction("SUM", (Column(0),), DataType.Float64),
            AggregateFunction("MIN", (Column(1),), DataType.Int64),
            AggregateFunction("COUNT", (Column(3),), DataType.UInt64)]
    pred = QUERIES[1][0]
    st = engine().agg_state([compile_expr(None, a, SCHEMA, fl) for a in aggs])
    st.add(compile_scalar_expr(None, pred, SCHEMA, fl), s.to(engine().device), fl)
    dev = st.finish()
    ref = oracle_aggregate(SCHEMA, s, pred, aggs, fl)
    assert [(d.is_null, d.count, d.bits) for d in dev] == [(r.is_null, r.count, r.bits) for r in ref]
