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


# ---- world sizes > 1 on one device: the loopback transport (csrc/shard.cpp
# LoopTransport: host threads, one context each, device-to-device copies)
# runs the same C++ placement, error agreement, grouped send/recv gather and
# root fix-ups (offset rebase, bit placement) that RCCL drives across GPUs.
def loop_world(world, fn, timeout=120):
    import ctypes as C

    import torch
    L = _abi.lib()
    L.dfmi_internal_loopback_group_create.argtypes = [C.c_int32]
    L.dfmi_internal_loopback_group_create.restype = C.c_void_p
    L.dfmi_internal_loopback_group_destroy.argtypes = [C.c_void_p]
    g = L.dfmi_internal_loopback_group_create(world)
    out, errors = [None] * world, []

    def work(rank):
        try:
            torch.cuda.set_device(0)
            with torch.cuda.stream(torch.cuda.Stream()):
                eng = DeviceEngine(0)
                comm = ShardComm.loopback(eng, g, rank)
                out[rank] = fn(rank, eng, comm)
                torch.cuda.current_stream().synchronize()
        except Exception as e:  # noqa: BLE001
            out[rank] = e
    th = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout)
    assert not any(t.is_alive() for t in th), "a rank is blocked in a collective"
    L.dfmi_internal_loopback_group_destroy(g)
    return out


def shard_of(b, rank, world):
    from datafusion_amd.execution.shard import shard_range
    lo, hi = shard_range(b.num_rows(), rank, world)
    cols = []
    for a in b.columns:
        h = a.cpu()
        if a.data_type == DataType.Utf8:
            vals = h.to_pylist()[lo:hi]
            cols.append(Array.from_strings([v.encode() for v in vals]))
        else:
            v = np.asarray(h.numpy_values())[lo:hi]
            valid = None
            if h.validity is not None:
                from datafusion_amd.arrow import unpack_bits
                valid = unpack_bits(h.validity.numpy(), b.num_rows())[lo:hi].astype(bool)
            cols.append(Array.from_numpy(a.data_type, v, valid))
    return RecordBatch(b.schema, cols)


@pytest.mark.parametrize("world", [2, 3])
def test_loopback_shards_place_and_gather(world):
    s, b = table(100_003)
    pred_e = BinaryExpr(Column(0), Operator.Lt, Literal(Float64(0.4)))
    proj_e = [Column(2), BinaryExpr(Column(0), Operator.Multiply, Column(1)), Column(0)]
    ref = oracle_filter_project(s, b, pred_e, proj_e)
    nsel = ref[0][1].length

    def fn(rank, eng, comm):
        pred = compile_scalar_expr(None, pred_e, s)
        projs = [compile_scalar_expr(None, e, s) for e in proj_e]
        cols = eng.filter_project(pred, projs, shard_of(b, rank, world), 0, comm=comm)
        p = comm.placement
        full = comm.gather_to_root(cols, root=world - 1)  # a root that is not rank 0
        return (p.row_offset, p.total_rows, p.utf8_base[0], p.utf8_total[0],
                [c.cpu() for c in cols], None if full is None else [c.cpu() for c in full])

    out = loop_world(world, fn)
    assert not [o for o in out if isinstance(o, Exception)], out
    off = 0
    for rank, (row_off, tot, ubase, utot, cols, full) in enumerate(out):
        assert (row_off, tot) == (off, nsel)
        assert utot == ref[0][1].data_bytes()
        assert ubase == sum(len(x.encode()) for x in ref[0][1].to_pylist()[:off])
        for d, (_, r) in zip(cols, ref):
            assert d.to_pylist() == r.to_pylist()[off:off + cols[0].length]
        off += cols[0].length
        assert (full is not None) == (rank == world - 1)
    for d, (_, r) in zip(out[-1][5], ref):
        assert_same(d, r)


def test_loopback_dense_bits_and_validity_gather():
    """Projection only (no predicate): a nullable Float64 sum and a Boolean
    comparison -- validity and value bitmaps placed at row offsets that are
    not multiples of 8 on the root."""
    s, b = table(50_001)
    proj_e = [BinaryExpr(Column(0), Operator.Plus, Column(1)), BinaryExpr(Column(1), Operator.Lt, Literal(Float64(0.5)))]
    ref = oracle_filter_project(s, b, None, proj_e)

    def fn(rank, eng, comm):
        projs = [compile_scalar_expr(None, e, s) for e in proj_e]
        cols = eng.filter_project(None, projs, shard_of(b, rank, 3), 0, comm=comm)
        full = comm.gather_to_root(cols, root=0)
        return None if full is None else [c.cpu() for c in full]

    out = loop_world(3, fn)
    assert not [o for o in out if isinstance(o, Exception)], out
    for d, (_, r) in zip(out[0], ref):
        assert_same(d, r)


def test_loopback_first_error_everywhere():
    """Rank 1 alone divides by zero: every rank raises the same error (none blocks)."""
    s, b = table(30_000)
    e = BinaryExpr(Column(0), Operator.Divide, BinaryExpr(Column(0), Operator.Minus, Column(0)))
    pred_e = BinaryExpr(Column(0), Operator.Lt, Literal(Float64(0.5)))

    def fn(rank, eng, comm):
        pred = compile_scalar_expr(None, pred_e, s)
        pe = BinaryExpr(Column(0), Operator.Plus, Column(0)) if rank != 1 else e
        projs = [compile_scalar_expr(None, pe, s)]
        try:
            eng.filter_project(pred, projs, shard_of(b, rank, 3), 0, comm=comm)
        except ExecutionError as x:
            return (x.kind, x.message)
        return None

    out = loop_world(3, fn)
    assert out == [("ArrowError(DivideByZero)", "DivideByZero")] * 3, out


def test_loopback_gather_checks_are_collective():
    """the root's Utf8 data_capacity too small fails EVERY rank
    with the root's error before any transfer (no rank left in a send)."""
    import ctypes as C
    s, b = table(40_000)
    pred_e = BinaryExpr(Column(0), Operator.Lt, Literal(Float64(0.5)))

    def fn(rank, eng, comm):
        pred = compile_scalar_expr(None, pred_e, s)
        projs = [compile_scalar_expr(None, Column(2), s)]
        cols = eng.filter_project(pred, projs, shard_of(b, rank, 2), 0, comm=comm)
        routs = (_abi.dfmi_out_column * 1)()
        keep = None
        if rank == 0:
            oc, keep = eng._alloc_out(DataType.Utf8, comm.placement.total_rows, False, 16)  # far too small
            routs[0] = oc
        err = _abi.dfmi_error()
        rc = _abi.lib().dfmi_shard_gather_to_root(eng.ctx, comm.handle, comm.outputs, routs, 0, C.byref(err))
        del keep, cols
        return rc, err.message.decode()

    out = loop_world(2, fn)
    assert out == [(_abi.DFMI_ERR_CAPACITY, "root Utf8 data_capacity too small")] * 2, out


def test_loopback_aggregate_finish():
    s, b = table(90_000)
    fl = _abi.DFMI_FLAG_EXT_AGGREGATE
    aggs_e = [agg("SUM", Column(1), s), agg("MIN", Column(0), s), agg("COUNT", Column(2), s)]
    ref = oracle_aggregate(s, b, None, aggs_e, fl)

    def fn(rank, eng, comm):
        aggs = [compile_expr(None, a, s, fl) for a in aggs_e]
        st = eng.agg_state(aggs)
        st.add(None, shard_of(b, rank, 3), fl)
        return [(v.bits, v.count, v.is_null) for v in comm.agg_finish(st)]

    out = loop_world(3, fn)
    for got in out:
        assert got == [(r.bits, r.count, r.is_null) for r in ref], got


@pytest.mark.parametrize("world", [2, 3])
def test_loopback_grouped_aggregate_finish(world):
    """GROUP BY across ranks (dfmi_shard_agg_finish_grouped): every rank's
    per-group partials all_gathered and merged -- the oracle's groups over
    the whole table, keys (with row counts) and values bit-identical, on
    every rank; keys both within one device window and far wider."""
    from oracle_ffi import oracle_aggregate_grouped
    rng = np.random.default_rng(17)
    n = 60_000
    s = Schema([Field("k", DataType.Int64, True), Field("x", DataType.Float64, True), Field("v", DataType.Int32, False)])
    b = RecordBatch(s, [Array.from_numpy(DataType.Int64, rng.integers(-900, 900, n), rng.random(n) > 0.02),
                        Array.from_numpy(DataType.Float64, rng.standard_normal(n) * 1e6, rng.random(n) > 0.1),
                        Array.from_numpy(DataType.Int32, rng.integers(-2 ** 31, 2 ** 31 - 1, n).astype(np.int32))])
    fl = _abi.DFMI_FLAG_EXT_AGGREGATE
    aggs_e = [agg("SUM", Column(1), s), agg("MIN", Column(1), s), agg("SUM", Column(2), s), agg("COUNT", Column(1), s)]
    for key_e in (BinaryExpr(Column(1), Operator.Gt, Literal(Float64(0.0))), Column(0)):
        rk, rv = oracle_aggregate_grouped(s, b, None, key_e, aggs_e, fl, 0)

        def fn(rank, eng, comm):
            aggs = [compile_expr(None, a, s, fl) for a in aggs_e]
            st = eng.grouped_agg_state(compile_scalar_expr(None, key_e, s, fl), aggs)
            st.add(None, shard_of(b, rank, world), fl)
            k, v = comm.agg_finish_grouped(st)
            return [(x.is_null, x.bits, x.count) for x in k], [[(y.is_null, y.bits, y.count) for y in g] for g in v]

        out = loop_world(world, fn)
        assert not [o for o in out if isinstance(o, Exception)], out
        want = ([(x.is_null, x.bits, x.count) for x in rk], [[(y.is_null, y.bits, y.count) for y in g] for g in rv])
        for got in out:
            assert got[0] == want[0]
            for g, (dg, rg) in enumerate(zip(got[1], want[1])):
                for d, r in zip(dg, rg):
                    assert d[0] == r[0] and d[2] == r[2] and (r[0] or d[1] == r[1]), (g, d, r)
