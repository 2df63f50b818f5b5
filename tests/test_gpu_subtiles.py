"""GPU parity of the low-selectivity form of numeric predicates (exec.cpp
kLowSel, jit.cpp "M sub-tiles"): M sub-tiles share one scan + look-back, the
predicate pass keeps only selection ballots, and the output pass reloads the
columns the outputs read for the selected rows -- one lane per row while a
wave holds at most 256 of them, else a dense pass per slice group. Forced
here at every size with the diagnostic knob (DFMI_NUMERIC_SUBTILES), so the
same cases as test_gpu_parity.py (filter.rs:80-111 semantics, error order)
run through it against the oracle; the last test checks the automatic choice
on a large batch."""
import numpy as np
import pytest

from datafusion_amd import _abi
from datafusion_amd._abi import DFMI_FLAG_EXT_GATHER_ALL
from datafusion_amd.arrow import Array, Field, RecordBatch, Schema
from datafusion_amd.execution.engine import engine
from datafusion_amd.execution.expression import compile_scalar_expr
from datafusion_amd.logicalplan import BinaryExpr, Column, DataType, Float64, Int64, Literal, Operator
from oracle_ffi import gen_unit_f64, oracle_filter_project
from test_gpu_parity import CMP, MATH, assert_same, run_both, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["8", "2"])
def subtiles(request, monkeypatch):
    monkeypatch.setenv("DFMI_DIAG", "1")
    monkeypatch.setenv("DFMI_NUMERIC_SUBTILES", request.param)
    return int(request.param)


def c2(sel):
    k, m = 1 - sel ** 0.5, sel ** 0.5
    pred = BinaryExpr(BinaryExpr(Column(0), Operator.Gt, Literal(Float64(k))), Operator.And,
                      BinaryExpr(Column(1), Operator.Lt, Literal(Float64(m))))
    proj = [Column(0), Column(1),
            BinaryExpr(BinaryExpr(Column(0), Operator.Multiply, Column(1)), Operator.Plus, Column(2))]
    return pred, proj


@pytest.mark.parametrize("n", [1, 63, 1000, 4097, 16_385, 100_003, (1 << 20) + 5])
@pytest.mark.parametrize("sel", [0.001, 0.01, 0.03, 0.5, 0.99])
def test_c2_float64(subtiles, n, sel):
    s, batch = synth(n)
    assert run_both(s, batch, *c2(sel)) is not None


@pytest.mark.parametrize("op", CMP)
def test_nullable_comparisons(subtiles, op):
    s, batch = synth(30_000, seed=7, nullable=True, null_frac=0.3)
    fl = DFMI_FLAG_EXT_GATHER_ALL
    run_both(s, batch, BinaryExpr(Column(0), op, Column(1)), [Column(0), Column(2)], fl)
    run_both(s, batch, BinaryExpr(Column(0), op, Literal(Float64(0.97))), [Column(1), Column(0)], fl)
    # Boolean output of a filtered batch (byte scratch + pack kernel)
    run_both(s, batch, BinaryExpr(Column(2), Operator.Gt, Literal(Float64(0.9))), [BinaryExpr(Column(0), op, Column(1))],
             fl)


@pytest.mark.parametrize("op", MATH)
@pytest.mark.parametrize("int64", [False, True])
def test_nullable_math(subtiles, op, int64):
    if op == Operator.Divide and int64:
        return
    s, batch = synth(20_000, seed=11, nullable=True, int64=int64, null_frac=0.2)
    lit = Int64(-(1 << 19)) if int64 else Float64(0.05)
    run_both(s, batch, BinaryExpr(BinaryExpr(Column(0), op, Column(1)), Operator.Lt, Literal(lit)),
             [Column(2), BinaryExpr(Column(0), op, Column(1))], DFMI_FLAG_EXT_GATHER_ALL)


def test_errors_in_order(subtiles):
    """DivideByZero / overflow raised by the output pass of a selected row,
    and by the predicate, in the reference's evaluation order."""
    n = 40_000
    a = np.arange(n, dtype=np.int64) - 1000
    d = np.ones(n, dtype=np.int64)
    d[1500] = 0
    d[30_000] = 0
    s = Schema([Field("a", DataType.Int64, False), Field("d", DataType.Int64, False),
                Field("x", DataType.Float64, False)])
    x = gen_unit_f64(1, 0, 0, n)
    b = RecordBatch(s, [Array.from_numpy(DataType.Int64, a), Array.from_numpy(DataType.Int64, d),
                        Array.from_numpy(DataType.Float64, x)])
    fl = DFMI_FLAG_EXT_GATHER_ALL
    # selected zero divisor (row 30000: a = 29000 > 28000)
    assert run_both(s, b, BinaryExpr(Column(0), Operator.Gt, Literal(Int64(28_000))),
                    [BinaryExpr(Column(0), Operator.Divide, Column(1))], fl) is None
    # not selected: no error
    run_both(s, b, BinaryExpr(Column(0), Operator.Lt, Literal(Int64(400))),
             [BinaryExpr(Column(0), Operator.Divide, Column(1))], fl)
    # in the predicate: every row evaluated
    assert run_both(s, b, BinaryExpr(BinaryExpr(Column(0), Operator.Divide, Column(1)), Operator.Lt,
                                     Literal(Int64(-990))), [Column(2)], fl) is None


def test_q6_style_and_narrow_types(subtiles):
    import bench
    n = 300_001
    s, dcols = bench.q6_table(engine().device, n, 42)
    b = RecordBatch(s, [Array.from_numpy(DataType.Float64, c.cpu().numpy()) for c in dcols])
    pred, projs = bench.q6_query()
    run_both(s, b, pred, projs)
    rng = np.random.default_rng(4)
    for t, npt in ((DataType.Int32, np.int32), (DataType.UInt16, np.uint16), (DataType.Float32, np.float32)):
        v = (rng.random(n) * 1000).astype(npt)
        w = (rng.random(n) * 1000).astype(npt)
        sch = Schema([Field("v", t, True), Field("w", t, False)])
        bb = RecordBatch(sch, [Array.from_numpy(t, v, rng.random(n) > 0.1), Array.from_numpy(t, w)])
        run_both(sch, bb, BinaryExpr(Column(0), Operator.Lt, Column(1)) if t == DataType.Float32 else
                 BinaryExpr(Column(0), Operator.GtEq, Column(1)), [Column(1), Column(0)], DFMI_FLAG_EXT_GATHER_ALL)


def test_boolean_predicate_column(subtiles):
    n = 50_000
    rng = np.random.default_rng(3)
    f1 = Array.from_numpy(DataType.Boolean, rng.random(n) < 0.02, rng.random(n) < 0.8)
    x = Array.from_numpy(DataType.Float64, gen_unit_f64(5, 0, 0, n))
    s = Schema([Field("f1", DataType.Boolean, True), Field("x", DataType.Float64, False)])
    b = RecordBatch(s, [f1, x])
    run_both(s, b, BinaryExpr(Column(0), Operator.And, BinaryExpr(Column(1), Operator.Gt, Literal(Float64(0.1)))),
             [Column(1)])
    run_both(s, b, Column(0), [Column(1), Column(0)], DFMI_FLAG_EXT_GATHER_ALL)  # Boolean output: dense output pass


def test_automatic_choice_on_a_large_batch():
    """No knob: the first large low-selectivity call runs the one-tile kernel,
    the next call of the same shape the sub-tile kernel (a different code
    object); both equal the oracle over a prefix and each other in full."""
    import torch
    n = (1 << 22) + 4097
    s, batch = synth(n, seed=5)
    db = batch.to(engine().device)
    pred, proj = c2(0.01)
    p = compile_scalar_expr(None, pred, s)
    cp = [compile_scalar_expr(None, e, s) for e in proj]
    eng = engine()
    first = eng.filter_project(p, cp, db)
    k1 = _abi.lib().dfmi_last_kernel_name(eng.ctx).decode()
    second = eng.filter_project(p, cp, db)
    k2 = _abi.lib().dfmi_last_kernel_name(eng.ctx).decode()
    assert k1 != k2, (k1, k2)
    for x, y in zip(first, second):
        assert x.length == y.length
        assert torch.equal(x.values[:x.length * 8], y.values[:y.length * 8])
    m = 1 << 20
    pre = RecordBatch(s, [Array(DataType.Float64, m, c.values[:m * 8]) for c in batch.columns])
    ref = oracle_filter_project(s, pre, pred, proj)
    nsel = ref[0][1].length
    for (_, r), d in zip(ref, second):
        assert_same(Array(DataType.Float64, nsel, d.values[:nsel * 8].cpu()), r)
