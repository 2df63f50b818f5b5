"""Multi-rank placement logic of the sharded path (datafusion_amd/execution/shard.py)
on CPU: world size 2 (and 3) over gloo, one process per rank, exactly as the
GPU ranks run under torchrun -- only the per-shard pass is a numpy stand-in
(there is no GPU here). The concatenation of the shards, and the root gather,
must equal the CPU oracle's output over the whole table."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from datafusion_amd.arrow import Array, Field, RecordBatch, Schema
from datafusion_amd.execution.shard import shard_range
from datafusion_amd.logicalplan import BinaryExpr, Column, DataType, Float64, Literal, Operator

N = 20011  # not a multiple of any world size used
K, M = 0.3, 0.6
WORDS = [b"", b"w17", b"alpha", b"\xe2\x82\xac", b"x" * 33]

SCHEMA = Schema([Field("a", DataType.Float64, True), Field("b", DataType.Float64, True),
                 Field("c", DataType.Float64, False), Field("s", DataType.Utf8, False)])
PRED = BinaryExpr(BinaryExpr(Column(0), Operator.Gt, Literal(Float64(K))), Operator.And,
                  BinaryExpr(Column(1), Operator.Lt, Literal(Float64(M))))
PROJS = [Column(3), Column(0), BinaryExpr(BinaryExpr(Column(0), Operator.Multiply, Column(1)), Operator.Plus, Column(2))]
DENSE = [BinaryExpr(Column(0), Operator.Plus, Column(1))]  # projection only, nulls propagate


def table(lo=0, hi=N, nullable=False):
    rng = np.random.default_rng(123)
    a, b, c = rng.random(N), rng.random(N), rng.random(N)
    va = rng.random(N) >= 0.2
    vb = rng.random(N) >= 0.2
    strs = [WORDS[i] for i in rng.integers(0, len(WORDS), N)]
    cols = [Array.from_numpy(DataType.Float64, a[lo:hi], va[lo:hi] if nullable else None),
            Array.from_numpy(DataType.Float64, b[lo:hi], vb[lo:hi] if nullable else None),
            Array.from_numpy(DataType.Float64, c[lo:hi]),
            Array.from_strings(strs[lo:hi])]
    return RecordBatch(SCHEMA, cols), (a[lo:hi], b[lo:hi], c[lo:hi], strs[lo:hi], va[lo:hi], vb[lo:hi])


def numpy_pass(raw, dense):
    """Stand-in for the device pass on one shard (same result layout)."""
    a, b, c, strs, va, vb = raw
    if dense:
        v = va & vb
        return [Array.from_numpy(DataType.Float64, np.where(v, a + b, 0.0), v)]
    m = (a > K) & (b < M)
    idx = np.flatnonzero(m)
    return [Array.from_strings([strs[i] for i in idx]), Array.from_numpy(DataType.Float64, a[m]),
            Array.from_numpy(DataType.Float64, a[m] * b[m] + c[m])]


def _worker(rank, world, port, dense, q):
    try:
        import torch.distributed as dist

        from datafusion_amd.execution.shard import ShardedFilterProject, gather_to_root
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        lo, hi = shard_range(N, rank, world)
        batch, raw = table(lo, hi, nullable=dense)
        step = ShardedFilterProject(None if dense else PRED, DENSE if dense else PROJS,
                                    run_shard=lambda p, e, bt, f: numpy_pass(raw, dense))
        res = step(batch)
        types = [c.data_type for c in res.columns]
        full = gather_to_root(res, types, root=0)
        shard = [c.to_pylist() for c in res.columns]
        q.put((rank, res.row_offset, res.total_rows, res.utf8_base, shard,
               None if full is None else [c.to_pylist() for c in full],
               None if full is None else [c.null_count for c in full]))
        dist.destroy_process_group()
    except Exception as e:  # surface worker failures in the parent
        import traceback
        q.put(("error", traceback.format_exc(), str(e)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_world(world, dense):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, dense, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(60)
    errs = [o for o in out if o[0] == "error"]
    assert not errs, errs[0][1]
    return sorted(out, key=lambda o: o[0])


def test_shard_range_partition():
    for n in (0, 1, 7, 1000, 10**9):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_filter_project_matches_oracle(world):
    from oracle_ffi import oracle_filter_project
    out = run_world(world, dense=False)
    batch, _ = table()
    ref = [r.to_pylist() for _, r in oracle_filter_project(SCHEMA, batch, PRED, PROJS)]
    # each rank's shard sits at its exchanged global offset
    total = len(ref[0])
    for rank, off, tot, ubase, shard, _, _ in out:
        assert tot == total
        for o in range(3):
            assert shard[o] == ref[o][off: off + len(shard[0])]
        assert ubase[0] == sum(len(s.encode("utf-8")) for s in ref[0][:off])
    # rank-ordered concatenation == the reference's output stream
    cat = [sum((o[4][c] for o in out), []) for c in range(3)]
    assert cat == ref
    # gather to rank 0 (Utf8 offsets rebased)
    assert out[0][5] == ref


def test_sharded_projection_with_nulls_matches_oracle():
    from oracle_ffi import oracle_filter_project
    out = run_world(2, dense=True)
    batch, _ = table(nullable=True)
    ((_, r),) = oracle_filter_project(SCHEMA, batch, None, DENSE)
    assert out[0][5] == [r.to_pylist()]
    assert out[0][6] == [r.null_count]


def _slice_worker(rank, world, port, q):
    """Projection-only shards whose outputs are passthrough columns (the input
    Arrays themselves, expression.rs:272-276) over SLICED inputs (arrow
    ArrayData::offset 3 / 5: bitmaps not byte-aligned): the root gather reads
    each rank's rows from its physical slots."""
    try:
        import torch.distributed as dist

        from datafusion_amd.execution.shard import ShardedFilterProject, gather_to_root
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        lo, hi = shard_range(N, rank, world)
        batch, _ = table(lo, hi, nullable=True)
        off = 3 + 2 * rank
        cols = [c.slice(off, c.length - off - 1) for c in batch.columns]
        bools = Array.from_numpy(DataType.Boolean, np.arange(hi - lo) % 3 == 0).slice(off, hi - lo - off - 1)
        outs = [cols[3], cols[0], bools]
        step = ShardedFilterProject(None, [Column(3), Column(0), Column(4)], run_shard=lambda p, e, bt, f: outs)
        res = step(RecordBatch(SCHEMA, cols))
        full = gather_to_root(res, [c.data_type for c in res.columns], root=0)
        q.put((rank, [c.to_pylist() for c in outs], None if full is None else [c.to_pylist() for c in full]))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put(("error", traceback.format_exc(), str(e)))


def test_gather_of_sliced_passthrough_columns():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_slice_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(60)
    errs = [o for o in out if o[0] == "error"]
    assert not errs, errs[0][1]
    out = sorted(out, key=lambda o: o[0])
    want = [out[0][1][c] + out[1][1][c] for c in range(3)]
    assert out[0][2] == want
    assert any(v is None for v in want[1])  # the nullable column kept its nulls


def _fail_worker(rank, world, port, plan, q):
    """plan[rank] = None (healthy) or (status code, message, evaluation position)."""
    try:
        import torch.distributed as dist

        from datafusion_amd.execution.error import ExecutionError
        from datafusion_amd.execution.shard import ShardedFilterProject
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        lo, hi = shard_range(N, rank, world)
        batch, raw = table(lo, hi)

        def run(p, e, bt, f):
            if plan[rank] is None:
                return numpy_pass(raw, False)
            code, msg, pos = plan[rank]
            err = ExecutionError.from_status(code, msg)
            err.order_key = (pos << 44) | (5 << 4)
            raise err

        try:
            ShardedFilterProject(PRED, PROJS, run_shard=run)(batch)
            q.put((rank, None, None))
        except ExecutionError as e:
            q.put((rank, e.kind, e.message))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put(("error", traceback.format_exc(), str(e)))


@pytest.mark.parametrize("plan,want", [
    # only rank 1 fails: every rank raises its error (none blocks in the exchange)
    ([None, (5, "DivideByZero", 3), None], ("ArrowError(DivideByZero)", "DivideByZero")),
    # rank 0 fails at a later operator than rank 2: the earlier operator wins
    ([(7, "attempt to divide with overflow", 9), None, (5, "DivideByZero", 4)],
     ("ArrowError(DivideByZero)", "DivideByZero")),
    # same operator on two ranks: the earlier rows (lower rank) win
    ([None, (7, "attempt to divide with overflow", 4), (5, "DivideByZero", 4)],
     ("panic", "attempt to divide with overflow")),
])
def test_failing_shard_raises_the_first_error_everywhere(plan, want):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fail_worker, args=(r, 3, port, plan, q)) for r in range(3)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(3)]
    for p in procs:
        p.join(60)
    errs = [o for o in out if o[0] == "error"]
    assert not errs, errs[0][1]
    assert all((o[1], o[2]) == want for o in out), out


def _place_worker(rank, world, port, dense, plan, q):
    """The C++ placement / error agreement (csrc/shard.cpp, through the internal
    hook dfmi_internal_shard_place) over the records this rank's Python
    exchange all_gathers, against ShardedFilterProject.exchange's outcome."""
    try:
        import ctypes as C

        import torch.distributed as dist

        from datafusion_amd import _abi
        from datafusion_amd.execution.error import ExecutionError
        from datafusion_amd.execution.shard import ShardedFilterProject, exchange_counts, shard_record
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        lo, hi = shard_range(N, rank, world)
        batch, raw = table(lo, hi, nullable=dense)
        failure = plan[rank] if plan else None

        def run(p, e, bt, f):
            if failure is None:
                return numpy_pass(raw, dense)
            code, msg, pos = failure
            err = ExecutionError.from_status(code, msg)
            err.order_key = None if pos is None else (pos << 44) | (5 << 4)
            raise err

        step = ShardedFilterProject(None if dense else PRED, DENSE if dense else PROJS, run_shard=run)
        py = None
        try:
            res = step(batch)
            py = ("ok", res.row_offset, res.total_rows, res.utf8_base,
                  [sum(c[1 + o] for c in res.counts) for o in range(len(res.columns))],
                  [sum(c[1 + len(res.columns) + o] for c in res.counts) for o in range(len(res.columns))])
            cols, e = res.columns, None
            nout = len(cols)
        except ExecutionError as ex:
            py = ("error", ex.code, ex.message)
            cols, e = None, ex
            nout = len(DENSE if dense else PROJS)
        if failure is not None:  # this rank's own error, as its pass raised it
            e = ExecutionError.from_status(failure[0], failure[1])
            e.order_key = None if failure[2] is None else (failure[2] << 44) | (5 << 4)
            mine = shard_record(None, e, nout)
        else:
            mine = shard_record(numpy_pass(raw, dense), None, nout)
        recs = exchange_counts(mine)
        L = _abi.lib()
        fn = L.dfmi_internal_shard_place
        fn.argtypes = [C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_int64), C.POINTER(_abi.dfmi_shard_placement),
                       C.POINTER(C.c_int32)]
        fn.restype = C.c_int32
        flat = (C.c_int64 * (world * len(recs[0])))(*[v for r in recs for v in r])
        place = _abi.dfmi_shard_placement()
        first = C.c_int32()
        assert fn(world, rank, nout, flat, C.byref(place), C.byref(first)) == 0
        cpp = ("ok", place.row_offset, place.total_rows, list(place.utf8_base[:nout]), list(place.utf8_total[:nout]),
               list(place.null_total[:nout])) if first.value < 0 else ("error", recs[first.value][0], first.value)
        q.put((rank, py, cpp))
        dist.destroy_process_group()
    except Exception as ex:  # noqa: BLE001
        import traceback
        q.put(("error", traceback.format_exc(), str(ex)))


@pytest.mark.parametrize("world,dense,plan", [
    (2, False, None), (3, False, None), (2, True, None),
    (3, False, [None, (5, "DivideByZero", 3), None]),
    (3, False, [(7, "attempt to divide with overflow", 9), None, (5, "DivideByZero", 4)]),
    (3, False, [None, (7, "attempt to divide with overflow", 4), (5, "DivideByZero", 4)]),
    (2, False, [(10, "device look-back timed out", None), (5, "DivideByZero", 0)]),  # unkeyed sorts last
    (2, False, [(5, "DivideByZero", 0), None]),  # position 0 is the first, not "none"
])
def test_cpp_placement_agrees_with_python_exchange(world, dense, plan):
    """the C-ABI path's placement / error agreement
    (csrc/shard.cpp first_failed_rank + placement_of) and the Python
    ShardedFilterProject.exchange give the same outcome for the same records."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_place_worker, args=(r, world, port, dense, plan, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(60)
    errs = [o for o in out if o[0] == "error"]
    assert not errs, errs[0][1]
    for rank, py, cpp in out:
        if py[0] == "ok":
            assert cpp == py, (rank, py, cpp)
        else:
            # the same failing rank's code (and so its message) on every rank
            assert cpp[0] == "error" and cpp[1] == py[1], (rank, py, cpp)
            assert plan[cpp[2]] is not None and plan[cpp[2]][1] == py[2]
