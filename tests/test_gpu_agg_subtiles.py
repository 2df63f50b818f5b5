"""The aggregate kernel's sub-tile form (jit.cpp generate_agg, Launch::M > 1):
M sub-tiles per block, the predicate passes keep the wave's ballots and a list
of its selected rows, then one lane per selected row loads the arguments and
accumulates -- or, when a wave selected more rows than its list holds, the
arguments are reloaded per sub-tile, lane-masked. Forced here with the
diagnostic knob (DFMI_DIAG=1 DFMI_AGG_SUBTILES=M) on batches of every shape,
and reached through the selectivity hint on a Q6-sized batch; every result
bit-identical to the oracle (tests/test_gpu_aggregate.py run_agg), errors in
the reference's order."""
import numpy as np
import pytest

from datafusion_amd import _abi
from datafusion_amd.arrow import Array, Field, RecordBatch, Schema
from datafusion_amd.execution.engine import engine
from datafusion_amd.execution.expression import compile_expr, compile_scalar_expr
from datafusion_amd.logicalplan import BinaryExpr, Column, DataType, Float64, Literal, Operator
from oracle_ffi import oracle_aggregate
from test_aggregate_cpu import agg, wild_doubles
from test_gpu_aggregate import AGG, NP, run_agg

pytestmark = pytest.mark.gpu

GA = AGG | _abi.DFMI_FLAG_EXT_GATHER_ALL


@pytest.fixture(params=[2, 4, 8])
def subtiles(request, monkeypatch):
    monkeypatch.setenv("DFMI_DIAG", "1")
    monkeypatch.setenv("DFMI_AGG_SUBTILES", str(request.param))
    return request.param


def q6_like(n, seed, sel_hi=0.06):
    rng = np.random.default_rng(seed)
    s = Schema([Field("qty", DataType.Float64, False), Field("price", DataType.Float64, True),
                Field("disc", DataType.Float64, False), Field("ship", DataType.Float64, False)])
    b = RecordBatch(s, [Array.from_numpy(DataType.Float64, rng.integers(1, 51, n).astype(np.float64)),
                        Array.from_numpy(DataType.Float64, wild_doubles(rng, n), rng.random(n) >= 0.05),
                        Array.from_numpy(DataType.Float64, np.round(rng.random(n) * 0.1, 2)),
                        Array.from_numpy(DataType.Float64, rng.random(n))])
    pred = BinaryExpr(BinaryExpr(BinaryExpr(Column(3), Operator.Lt, Literal(Float64(sel_hi))), Operator.And,
                                 BinaryExpr(Column(2), Operator.GtEq, Literal(Float64(0.05)))), Operator.And,
                      BinaryExpr(Column(0), Operator.Lt, Literal(Float64(24.0))))
    prod = BinaryExpr(Column(1), Operator.Multiply, Column(2))
    aggs = [agg("SUM", prod, s), agg("MIN", Column(1), s), agg("MAX", prod, s), agg("COUNT", Column(1), s),
            agg("SUM", Column(0), s)]
    return s, b, pred, aggs


@pytest.mark.parametrize("sel_hi", [0.004, 0.06, 0.9])
def test_q6_shape(subtiles, sel_hi):
    """Low selectivity (sparse pass), and 0.9 of the ship column (most waves'
    lists overflow: the lane-masked per-sub-tile pass); a ragged last block."""
    s, b, pred, aggs = q6_like(300_007, 3, sel_hi)
    run_agg(s, b, pred, aggs, GA)
    run_agg(s, b, pred, aggs, GA, batch_rows=70_000)


@pytest.mark.parametrize("t", list(NP))
def test_every_type(subtiles, t):
    rng = np.random.default_rng(40 + int(t))
    n = 100_003
    dt = np.dtype(NP[t])
    if dt.kind == "f":
        x = (rng.standard_normal(n) * np.exp2(rng.integers(-60, 60, n))).astype(dt)
        x[rng.random(n) < 0.01] = np.nan
    else:
        info = np.iinfo(dt)
        x = rng.integers(info.min, info.max, n, dtype=dt, endpoint=True)
    s = Schema([Field("x", t, True), Field("k", DataType.Float64, False)])
    b = RecordBatch(s, [Array.from_numpy(t, x, rng.random(n) >= 0.15), Array.from_numpy(DataType.Float64, rng.random(n))])
    aggs = [agg(f, Column(0), s) for f in ("SUM", "MIN", "MAX", "COUNT")]
    for k in (0.02, 0.5):
        run_agg(s, b, BinaryExpr(Column(1), Operator.Lt, Literal(Float64(k))), aggs, GA)


def test_errors_in_order(subtiles):
    s = Schema([Field("a", DataType.Float64, False), Field("d", DataType.Float64, False)])
    n = 200_000
    a = np.arange(float(n))
    d = np.ones(n)
    d[150_000] = 0.0
    d[7] = 0.0
    b = RecordBatch(s, [Array.from_numpy(DataType.Float64, a), Array.from_numpy(DataType.Float64, d)])
    q = agg("SUM", BinaryExpr(Column(0), Operator.Divide, Column(1)), s)
    # row 7 not selected, row 150000 selected: DivideByZero
    assert run_agg(s, b, BinaryExpr(Column(0), Operator.Gt, Literal(Float64(100.0))), [q], GA) is None
    # neither selected
    run_agg(s, b, BinaryExpr(Column(0), Operator.Gt, Literal(Float64(160_000.0))), [q], GA)


def test_selectivity_hint_picks_subtiles():
    """No knob: the first batch runs the one-tile kernel and leaves the
    state's selectivity (< 4%); the next batches of the same query run the
    sub-tile kernel (another kernel name) with the same exact results."""
    s, b, pred, aggs = q6_like(1 << 22, 11, 0.05)
    eng = engine()
    p = compile_scalar_expr(None, pred, s, GA)
    st = eng.agg_state([compile_expr(None, a, s, GA) for a in aggs])
    db = b.to(eng.device)
    names = []
    for _ in range(3):
        st.add(p, db, GA)
        names.append(_abi.lib().dfmi_last_kernel_name(eng.ctx).decode())
    assert names[0] != names[1] == names[2], names
    dev = st.finish()
    ref = oracle_aggregate(s, b, pred, aggs, GA)
    for d, r in zip(dev, ref):
        assert (d.is_null, d.count) == (r.is_null, r.count * 3)
    # the same sums, thrice: compare against the oracle over the batch three times
    ref3 = oracle_aggregate(s, RecordBatch(s, [Array.from_numpy(DataType.Float64, np.tile(c.numpy_values(), 3),
                                                                 np.tile(c.valid_mask(), 3) if c.validity is not None
                                                                 else None) for c in b.columns]), pred, aggs, GA)
    for a, d, r in zip(aggs, dev, ref3):
        assert (d.is_null, d.count, d.bits) == (r.is_null, r.count, r.bits), repr(a)
