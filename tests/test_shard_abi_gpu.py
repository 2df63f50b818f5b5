"""The C-ABI multi-GPU entry points (include/dfmi.h "Multi-GPU") on the GPU
box's one device: a world-size-1 RCCL communicator (dfmi_shard_comm_init),
the shard pass + placement all_gather, the grouped send/recv gather to root,
the aggregate partial all_gather, and error agreement -- each against the
single-GPU entry points and the oracle. Plus the threading contract: two
contexts driven from two host threads at once through the host-buffer path.
(More ranks need more GPUs: the gloo tests in test_shard_cpu.py cover the
same placement logic at world sizes 2 and 3.)"""
import threading

import numpy as np
import pytest

from datafusion_amd import _abi
from datafusion_amd.arrow import Array, Field, RecordBatch, Schema
from datafusion_amd.execution.engine import DeviceEngine, ShardComm, engine
from datafusion_amd.execution.error import ExecutionError
from datafusion_amd.execution.expression import compile_expr, compile_scalar_expr
from datafusion_amd.logicalplan import BinaryExpr, Column, DataType, Float64, Literal, Operator
from oracle_ffi import gen_unit_f64, oracle_aggregate, oracle_filter_project
from test_aggregate_cpu import agg
from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu


def table(n=200_003):
    rng = np.random.default_rng(3)
    words = [bytes(rng.integers(97, 123, int(rng.integers(0, 20))).astype(np.uint8)) for _ in range(100)]
    s = Schema([Field("a", DataType.Float64, False), Field("b", DataType.Float64, True), Field("s", DataType.Utf8, False)])
    b = RecordBatch(s, [Array.from_numpy(DataType.Float64, gen_unit_f64(1, 0, 0, n)),
                        Array.from_numpy(DataType.Float64, gen_unit_f64(1, 1, 0, n), rng.random(n) >= 0.2),
                        Array.from_strings([words[i] for i in rng.integers(0, 100, n)])])
    return s, b


@pytest.fixture(scope="module")
def comm():
    return ShardComm(engine(), 1, 0, ShardComm.unique_id())


def test_shard_pass_placement_and_gather(comm):
    s, b = table()
    pred_e = BinaryExpr(Column(0), Operator.Lt, Literal(Float64(0.4)))
    proj_e = [Column(2), BinaryExpr(Column(0), Operator.Multiply, Column(1)), Column(0)]
    pred = compile_scalar_expr(None, pred_e, s)
    projs = [compile_scalar_expr(None, e, s) for e in proj_e]
    eng = engine()
    cols = eng.filter_project(pred, projs, b, 0, comm=comm)
    ref = oracle_filter_project(s, b, pred_e, proj_e)
    for d, (_, r) in zip(cols, ref):
        assert_same(d.cpu(), r)
    p = comm.placement
    assert (p.world, p.rank, p.row_offset, p.total_rows) == (1, 0, 0, ref[0][1].length)
    assert p.utf8_total[0] == cols[0].data_bytes() and p.utf8_base[0] == 0
    full = comm.gather_to_root(cols, root=0)
    for d, (_, r) in zip(full, ref):
        assert_same(d.cpu(), r)


def test_shard_errors_agree(comm):
    s, b = table(10_000)
    e = BinaryExpr(Column(0), Operator.Divide, BinaryExpr(Column(0), Operator.Minus, Column(0)))
    pred = compile_scalar_expr(None, BinaryExpr(Column(0), Operator.Lt, Literal(Float64(0.5))), s)
    projs = [compile_scalar_expr(None, e, s)]
    with pytest.raises(ExecutionError) as ei:
        engine().filter_project(pred, projs, b, 0, comm=comm)
    assert (ei.value.kind, ei.value.message) == ("ArrowError(DivideByZero)", "DivideByZero")


def test_shard_aggregate_finish(comm):
    s, b = table()
    fl = _abi.DFMI_FLAG_EXT_AGGREGATE
    aggs_e = [agg("SUM", Column(1), s), agg("MIN", Column(0), s), agg("COUNT", Column(2), s)]
    aggs = [compile_expr(None, a, s, fl) for a in aggs_e]
    st = engine().agg_state(aggs)
    st.add(None, b, fl)
    got = comm.agg_finish(st)
    ref = oracle_aggregate(s, b, None, aggs_e, fl)
    for g, r in zip(got, ref):
        assert (g.bits, g.count, g.is_null) == (r.bits, r.count, r.is_null)


def test_two_contexts_two_threads_host_path():
    """dfmi.h threading contract: one host thread per context. Two contexts
    on cuda:0, driven concurrently (ctypes drops the GIL) through
    dfmi_filter_project_host, 20 calls each: every result equals the oracle."""
    s, b = table(300_000)
    pred_e = BinaryExpr(Column(1), Operator.Gt, Literal(Float64(0.3)))
    proj_e = [Column(0), Column(2)]
    ref = oracle_filter_project(s, b, pred_e, proj_e)
    pred = compile_scalar_expr(None, pred_e, s)
    projs = [compile_scalar_expr(None, e, s) for e in proj_e]
    engines = [DeviceEngine(0), DeviceEngine(0)]
    errors = []

    def work(eng):
        try:
            for _ in range(20):
                out = eng.filter_project_host(pred, projs, b)
                for d, (_, r) in zip(out, ref):
                    assert_same(d, r)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=work, args=(e,)) for e in engines]
    for t in th:
        t.start()
    for t in th:
        t.join(100)
    assert not errors, errors[0]
