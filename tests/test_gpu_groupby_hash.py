"""GPU parity of the device GROUP BY hash table (aggregate.cpp "hashed
groups", groupby.hip): several GROUP BY expressions (sqlplanner.rs:97-117
plans group_expr as a Vec<Expr>), the table grown past its first size, keys
forced onto shared hashes (the host merge of colliding rows), the host-merge
A/B, and Utf8 / multi-key grouped partials merged across shards -- keys,
per-group row counts and every aggregate bit-identical to the oracle.

Parity unpinned beyond the one-key csv_aggregate_by_c_bool.csv fixture: the
reference plans Aggregate but cannot execute it (context.rs:161); the oracle
restates the build's key order (lexicographic over the parts, each part's
null last)."""
import os

import numpy as np
import pytest

from datafusion_amd import _abi
from datafusion_amd.arrow import Array, Field, RecordBatch, Schema
from datafusion_amd.execution import ExecutionContext, MemoryDataSource
from datafusion_amd.execution.engine import engine, merge_grouped_partials, merge_grouped_partials_key_strings
from datafusion_amd.execution.error import ExecutionError
from datafusion_amd.execution.expression import compile_expr, compile_scalar_expr
from datafusion_amd.logicalplan import BinaryExpr, Column, DataType, Float64, Int64, Literal, Operator
from oracle_ffi import oracle_aggregate_grouped_multi
from test_aggregate_cpu import agg, wild_doubles
from test_gpu_aggregate import slice_batch

pytestmark = pytest.mark.gpu

AGG = _abi.DFMI_FLAG_EXT_AGGREGATE
FL = AGG | _abi.DFMI_FLAG_EXT_GATHER_ALL


def _vals(vs):
    return [(v.type, v.is_null, v.count, 0 if v.is_null else v.bits) for v in vs]


def run_multi(schema, batch, pred, keys, aggs, flags=FL, batch_rows=0):
    """Device groups of GROUP BY keys against the oracle's: keys (all parts),
    Utf8 key bytes, row counts and values bit for bit; or the same error."""
    ref = ref_err = dev = dev_err = None
    try:
        ref = oracle_aggregate_grouped_multi(schema, batch, pred, keys, aggs, flags, batch_rows)
    except ExecutionError as e:
        ref_err = e
    st = None
    try:
        p = compile_scalar_expr(None, pred, schema, flags) if pred is not None else None
        ks = [compile_scalar_expr(None, k, schema, flags) for k in keys]
        cs = [compile_expr(None, a, schema, flags) for a in aggs]
        st = engine().grouped_agg_state(ks, cs)
        n = batch.num_rows()
        step = batch_rows if batch_rows > 0 else max(n, 1)
        dbatch = batch.to(engine().device)
        for r0 in range(0, max(n, 1), step):
            st.add(p, slice_batch(dbatch, r0, min(step, n - r0)) if n else dbatch, flags)
        dev = st.finish()
    except ExecutionError as e:
        dev_err = e
    if ref_err is not None or dev_err is not None:
        assert ref_err is not None and dev_err is not None, (ref_err, dev_err)
        assert (dev_err.kind, dev_err.message) == (ref_err.kind, ref_err.message)
        return None
    (dk, dv), (rk, rv, rs) = dev, ref
    assert len(dk) == len(rk)
    for g, (a, b) in enumerate(zip(dk, rk)):
        assert [(k.type, k.is_null, k.bits, k.count) for k in a] == [(k.type, k.is_null, k.bits, k.count) for k in b], g
    for p, strs in enumerate(rs):
        if strs is not None:
            assert st.key_strings(p) == strs, p
    for g in range(len(rk)):
        assert _vals(dv[g]) == _vals(rv[g]), g
    return dev


def _table(rng, n):
    words = [bytes(rng.integers(97, 123, int(rng.integers(0, 14))).astype(np.uint8)) for _ in range(300)]
    words += [b"", b"\xff\xfe", "€".encode()]
    s = Schema([Field("k1", DataType.Int64, True), Field("k2", DataType.Utf8, True), Field("f", DataType.Float64, True),
                Field("b", DataType.Boolean, True), Field("x", DataType.Float64, True), Field("v", DataType.Int32, True)])
    cols = [Array.from_numpy(DataType.Int64, rng.integers(-40, 40, n) * 1_000_003, rng.random(n) >= 0.03),
            Array.from_strings([None if rng.random() < 0.03 else words[i] for i in rng.integers(0, len(words), n)]),
            Array.from_numpy(DataType.Float64, rng.integers(-20, 20, n) / 4.0, rng.random(n) >= 0.03),
            Array.from_numpy(DataType.Boolean, rng.random(n) < 0.5, rng.random(n) >= 0.05),
            Array.from_numpy(DataType.Float64, wild_doubles(rng, n), rng.random(n) >= 0.1),
            Array.from_numpy(DataType.Int32, rng.integers(-2 ** 31, 2 ** 31 - 1, n).astype(np.int32),
                             rng.random(n) >= 0.1)]
    return s, RecordBatch(s, cols)


AGGS = lambda s: [agg("SUM", Column(4), s), agg("COUNT", Column(4), s), agg("MIN", Column(4), s),  # noqa: E731
                  agg("MAX", Column(5), s), agg("SUM", Column(5), s)]


@pytest.mark.parametrize("batch_rows", [0, 6_007])
def test_group_by_two_keys_int64_utf8(batch_rows):
    """SELECT k1, k2, SUM(x), COUNT(x), ... GROUP BY k1, k2 (Int64 x Utf8, both
    with nulls), with and without a predicate, one batch or many."""
    rng = np.random.default_rng(61)
    s, b = _table(rng, 40_013)
    pred = BinaryExpr(Column(4), Operator.Lt, Literal(Float64(0.6)))
    for p in (None, pred):
        out = run_multi(s, b, p, [Column(0), Column(1)], AGGS(s), batch_rows=batch_rows)
        assert out is not None and len(out[0]) > 3000


def test_group_by_three_and_four_keys():
    """Boolean, Float64 (-0.0 / +0.0 distinct), Int64 and Utf8 parts in
    several orders, and a computed key part."""
    rng = np.random.default_rng(62)
    s, b = _table(rng, 30_011)
    for keys in ([Column(3), Column(2), Column(0)], [Column(1), Column(3), Column(2), Column(0)],
                 [BinaryExpr(Column(0), Operator.Plus, Literal(Int64(7))), Column(3)]):
        out = run_multi(s, b, BinaryExpr(Column(4), Operator.Gt, Literal(Float64(-0.5))), keys, AGGS(s), batch_rows=9_001)
        assert out is not None and len(out[0]) > 10


def test_group_by_multi_key_errors_in_order():
    """An error in a key part comes before the aggregates' in the reference's
    evaluation order (keys in group_expr order, then the arguments)."""
    n = 4096
    s = Schema([Field("k", DataType.Int64, False), Field("d", DataType.Int64, False), Field("x", DataType.Float64, False)])
    d = np.ones(n, np.int64)
    d[1500] = 0
    b = RecordBatch(s, [Array.from_numpy(DataType.Int64, np.arange(n) % 50), Array.from_numpy(DataType.Int64, d),
                        Array.from_numpy(DataType.Float64, np.arange(n, dtype=np.float64))])
    bad = [agg("SUM", BinaryExpr(Column(2), Operator.Divide, Literal(Float64(0.0))), s)]
    key2 = BinaryExpr(Column(0), Operator.Divide, Column(1))
    assert run_multi(s, b, None, [Column(0), key2], bad) is None
    assert run_multi(s, b, None, [Column(0), Column(1)], bad) is None


def test_group_by_table_growth_many_keys():
    """~150,000 distinct (Int64, Float64) keys in one batch: the claim pass
    overflows the first 65,536-slot table, which is grown and rehashed, and
    the pass is run again; also over batches (keys persisted across them)."""
    rng = np.random.default_rng(63)
    n = 200_003
    s = Schema([Field("a", DataType.Int64, False), Field("f", DataType.Float64, True), Field("x", DataType.Float64, False)])
    b = RecordBatch(s, [Array.from_numpy(DataType.Int64, rng.integers(0, 400, n)),
                        Array.from_numpy(DataType.Float64, rng.integers(0, 500, n) * 0.25, rng.random(n) >= 0.01),
                        Array.from_numpy(DataType.Float64, rng.standard_normal(n))])
    aggs = [agg("SUM", Column(2), s), agg("COUNT", Column(2), s)]
    for br in (0, 50_000):
        out = run_multi(s, b, None, [Column(0), Column(1)], aggs, batch_rows=br)
        assert out is not None and len(out[0]) > 100_000


def test_group_by_forced_hash_collisions(monkeypatch):
    """DFMI_GROUP_HASH_BITS=3 (diagnostics): every key hashes into 8 values,
    so most rows meet a slot holding another key and are listed for the host
    merge -- the merged groups still equal the oracle's; single Float64 key,
    Utf8 key and two keys."""
    monkeypatch.setenv("DFMI_DIAG", "1")
    monkeypatch.setenv("DFMI_GROUP_HASH_BITS", "3")
    rng = np.random.default_rng(64)
    s, b = _table(rng, 12_007)
    for keys in ([Column(2)], [Column(1)], [Column(0), Column(1)]):
        out = run_multi(s, b, None, keys, AGGS(s), batch_rows=5_000)
        assert out is not None and len(out[0]) > 20


def test_group_by_host_merge_ab_matches_device(monkeypatch):
    """The host merge (DFMI_GROUP_HOST=1, the A/B of the device table) and
    the device table give the same groups."""
    rng = np.random.default_rng(65)
    s, b = _table(rng, 20_011)
    dev = run_multi(s, b, None, [Column(1), Column(0)], AGGS(s), batch_rows=7_000)
    monkeypatch.setenv("DFMI_DIAG", "1")
    monkeypatch.setenv("DFMI_GROUP_HOST", "1")
    host = run_multi(s, b, None, [Column(1), Column(0)], AGGS(s), batch_rows=7_000)
    assert [[(k.is_null, k.bits) for k in g] for g in dev[0]] == [[(k.is_null, k.bits) for k in g] for g in host[0]]
    assert [_vals(v) for v in dev[1]] == [_vals(v) for v in host[1]]


def test_group_by_two_keys_through_sql():
    """ctx.sql(... GROUP BY k2, k1): the planner's Aggregate with two
    group_expr, the relation's columns k2 (Utf8), k1, then the aggregates,
    one row per group in key order."""
    rng = np.random.default_rng(66)
    n = 8_000
    words = [b"pear", b"apple", b"fig", b""]
    s = Schema([Field("k1", DataType.Int64, False), Field("k2", DataType.Utf8, False), Field("x", DataType.Float64, False)])
    b = RecordBatch(s, [Array.from_numpy(DataType.Int64, rng.integers(0, 5, n)),
                        Array.from_strings([words[i] for i in rng.integers(0, 4, n)]),
                        Array.from_numpy(DataType.Float64, rng.random(n))])
    ctx = ExecutionContext(flags=FL)
    ctx.register_datasource("t", MemoryDataSource(s, [b.to(engine().device)]))
    (rb,) = list(ctx.sql("SELECT k2, k1, COUNT(x), SUM(x) FROM t WHERE x > 0.1 GROUP BY k2, k1"))
    assert [f.name for f in rb.schema.fields][:2] == ["k2", "k1"]
    pred = BinaryExpr(Column(2), Operator.Gt, Literal(Float64(0.1)))
    rk, rv, rs = oracle_aggregate_grouped_multi(s, b, pred, [Column(1), Column(0)],
                                                [agg("COUNT", Column(2), s), agg("SUM", Column(2), s)], FL)
    assert [w.encode() for w in rb.columns[0].to_pylist()] == rs[0]
    assert rb.columns[1].to_pylist() == [g[1].bits for g in rk]
    assert rb.columns[2].to_pylist() == [v[0].bits for v in rv]
    assert [int(np.array([y], np.float64).view(np.uint64)[0]) for y in rb.columns[3].to_pylist()] == \
        [v[1].bits for v in rv]


def test_grouped_partials_utf8_and_multi_key_merge():
    """Per-shard grouped partials with Utf8 and multi-part keys (the round-5
    NotImplemented): three shards' partials merged equal one state over all
    rows -- keys, Utf8 bytes and values."""
    rng = np.random.default_rng(67)
    s, b = _table(rng, 30_000)
    aggs_e = AGGS(s)
    for keys_e in ([Column(1)], [Column(0), Column(1)]):
        rk, rv, rs = oracle_aggregate_grouped_multi(s, b, None, keys_e, aggs_e, FL)
        parts, cs = [], None
        for r in range(3):
            cs = [compile_expr(None, a, s, FL) for a in aggs_e]
            st = engine().grouped_agg_state([compile_scalar_expr(None, k, s, FL) for k in keys_e], cs)
            st.add(None, slice_batch(b.to(engine().device), r * 10_000, 10_000), FL)
            parts.append(st.partial())
        mk, mv = merge_grouped_partials(cs, parts, len(keys_e), True)
        assert [[(k.is_null, k.bits, k.count) for k in g] for g in mk] == \
            [[(k.is_null, k.bits, k.count) for k in g] for g in rk]
        assert [_vals(v) for v in mv] == [_vals(v) for v in rv]
        for p, strs in enumerate(rs):
            if strs is not None:
                got = merge_grouped_partials_key_strings(cs, parts, p, len(mk))
                assert [None if mk[g][p].is_null else got[g] for g in range(len(mk))] == strs


@pytest.mark.parametrize("buckets", ["0", "1"])
def test_finish_then_more_rows_partial_and_reset(monkeypatch, buckets):
    """The finish's flat groups (aggregate.cpp finish_flat: finished on the
    device, the table kept): a second finish gives the same groups; rows
    added after a finish merge with the finished groups; the grouped partial
    after a finish holds every group; reset empties -- with the atomic
    accumulate pass and with the bucketed passes (DFMI_GROUP_BUCKETS)."""
    monkeypatch.setenv("DFMI_DIAG", "1")
    monkeypatch.setenv("DFMI_GROUP_BUCKETS", buckets)
    rng = np.random.default_rng(68)
    s, b = _table(rng, 24_000)
    aggs_e = AGGS(s)
    db = b.to(engine().device)
    for keys_e in ([Column(2)], [Column(1)], [Column(0), Column(1)]):
        cs = [compile_expr(None, a, s, FL) for a in aggs_e]
        st = engine().grouped_agg_state([compile_scalar_expr(None, k, s, FL) for k in keys_e], cs)
        rk1, rv1, rs1 = oracle_aggregate_grouped_multi(s, slice_batch(b, 0, 10_000), None, keys_e, aggs_e, FL)
        rk, rv, rs = oracle_aggregate_grouped_multi(s, b, None, keys_e, aggs_e, FL)

        def check(out, rk_, rv_, rs_):
            dk, dv = out
            assert [[(k.is_null, k.bits, k.count) for k in g] for g in dk] == \
                [[(k.is_null, k.bits, k.count) for k in g] for g in rk_]
            assert [_vals(v) for v in dv] == [_vals(v) for v in rv_]
            for p, strs in enumerate(rs_):
                if strs is not None:
                    assert st.key_strings(p) == strs

        st.add(None, slice_batch(db, 0, 10_000), FL)
        check(st.finish(), rk1, rv1, rs1)
        check(st.finish(), rk1, rv1, rs1)
        st.add(None, slice_batch(db, 10_000, 14_000), FL)
        check(st.finish(), rk, rv, rs)
        part = st.partial()
        mk, mv = merge_grouped_partials(cs, [part], len(keys_e), True)
        assert [[(k.is_null, k.bits, k.count) for k in g] for g in mk] == \
            [[(k.is_null, k.bits, k.count) for k in g] for g in rk]
        assert [_vals(v) for v in mv] == [_vals(v) for v in rv]
        check(st.finish(), rk, rv, rs)
        st.reset()
        assert len(st.finish()[0]) == 0
        st.add(None, slice_batch(db, 0, 10_000), FL)
        check(st.finish(), rk1, rv1, rs1)


def _rounding_table(rng, n):
    """Per group (a Float64 key, hashed) SUMs that exercise every step of the
    exact rounding: overflow to +-inf, exact cancellation (+0.0) and sums of
    -0.0 (-0.0), subnormal sums, ties to even at 2^-53 and at Float32's
    2^-24, Float32 sums past 2^128, and wild doubles over the whole exponent
    range; a Float32 column of the same values narrowed."""
    g = rng.integers(0, 64, n).astype(np.float64)
    x = wild_doubles(rng, n)
    grp = rng.integers(0, 8, n)
    x[grp == 0] = 1.7e308 * np.where(rng.random(int((grp == 0).sum())) < 0.7, 1.0, -1.0)
    x[grp == 1] = -0.0
    x[grp == 2] = np.ldexp(rng.integers(-9, 10, int((grp == 2).sum())).astype(np.float64), -1074)
    x[grp == 3] = np.where(rng.random(int((grp == 3).sum())) < 0.5, 1.0, np.ldexp(1.0, -53))
    x[grp == 4] = np.where(rng.random(int((grp == 4).sum())) < 0.5, 3.0e38, np.ldexp(1.0, -24))
    g[grp <= 4] = 100 + grp[grp <= 4] * 1000 + rng.integers(0, 3, int((grp <= 4).sum()))
    f32 = np.clip(x, -3.4e38, 3.4e38).astype(np.float32)
    s = Schema([Field("g", DataType.Float64, True), Field("x", DataType.Float64, True),
                Field("y", DataType.Float32, True)])
    return s, RecordBatch(s, [Array.from_numpy(DataType.Float64, g, rng.random(n) >= 0.02),
                              Array.from_numpy(DataType.Float64, x, rng.random(n) >= 0.05),
                              Array.from_numpy(DataType.Float32, f32, rng.random(n) >= 0.05)])


def test_group_by_device_finish_rounding(monkeypatch):
    """The finish rounds every group's exact sum on the device (groupby.hip
    k_group_round): bit-identical to the oracle and to the host's rounding of
    the same table (DFMI_GROUP_HOST_FINISH=1, the A/B), for Float64 and
    Float32 SUMs, one batch and several, and for two keys."""
    rng = np.random.default_rng(69)
    s, b = _rounding_table(rng, 60_000)
    aggs_e = [agg("SUM", Column(1), s), agg("SUM", Column(2), s), agg("COUNT", Column(1), s),
              agg("MIN", Column(2), s), agg("MAX", Column(1), s)]
    for keys in ([Column(0)], [Column(0), Column(2)]):
        for br in (0, 17_000):
            dev = run_multi(s, b, None, keys, aggs_e, batch_rows=br)
            assert dev is not None and len(dev[0]) > 60
            monkeypatch.setenv("DFMI_DIAG", "1")
            monkeypatch.setenv("DFMI_GROUP_HOST_FINISH", "1")
            host = run_multi(s, b, None, keys, aggs_e, batch_rows=br)
            monkeypatch.delenv("DFMI_DIAG")
            monkeypatch.delenv("DFMI_GROUP_HOST_FINISH")
            assert [_vals(v) for v in dev[1]] == [_vals(v) for v in host[1]]
    # the specials really occur among the device's results
    f64 = {int(v[0].bits) for v in run_multi(s, b, None, [Column(0)], aggs_e)[1] if not v[0].is_null}
    assert 0x7FF0000000000000 in f64 or 0xFFF0000000000000 in f64
    assert 0x8000000000000000 in f64


def _bucketed_batches():
    import ctypes as C
    L = _abi.lib()
    L.dfmi_internal_group_bucketed_batches.restype = C.c_long
    return L.dfmi_internal_group_bucketed_batches()


def test_group_by_bucketed_accumulation_forced(monkeypatch):
    """The bucketed passes (groupby.h: rank, scan, scatter, per-bucket LDS
    sums) forced on small batches (DFMI_GROUP_BUCKETS=1): two keys with a
    predicate over many batches, the rounding table's specials, Int32 SUM /
    MIN / MAX with NULLs, keys forced onto shared hashes (the rank pass lists
    the colliding rows) -- every group bit-identical to the oracle."""
    monkeypatch.setenv("DFMI_DIAG", "1")
    monkeypatch.setenv("DFMI_GROUP_BUCKETS", "1")
    before = _bucketed_batches()
    rng = np.random.default_rng(70)
    s, b = _table(rng, 40_013)
    pred = BinaryExpr(Column(4), Operator.Lt, Literal(Float64(0.6)))
    for p in (None, pred):
        out = run_multi(s, b, p, [Column(0), Column(1)], AGGS(s), batch_rows=6_007)
        assert out is not None and len(out[0]) > 3000
    out = run_multi(s, b, None, [Column(3)], AGGS(s), batch_rows=9_001)  # Boolean key: 3 groups, heavy contention
    assert out is not None and len(out[0]) == 3
    s2, b2 = _rounding_table(rng, 50_000)
    aggs2 = [agg("SUM", Column(1), s2), agg("SUM", Column(2), s2), agg("COUNT", Column(1), s2),
             agg("MIN", Column(2), s2), agg("MAX", Column(1), s2)]
    assert run_multi(s2, b2, None, [Column(0)], aggs2, batch_rows=20_000) is not None
    monkeypatch.setenv("DFMI_GROUP_HASH_BITS", "3")
    out = run_multi(s, b, None, [Column(1)], AGGS(s), batch_rows=8_000)
    assert out is not None and len(out[0]) > 20
    assert _bucketed_batches() > before


def test_group_by_bucketed_accumulation_chosen():
    """A batch of 2^21 rows over 1,000 keys (many rows per group): the
    bucketed passes are chosen without any diagnostics switch, and the
    groups equal the oracle's."""
    rng = np.random.default_rng(71)
    n = 1 << 21
    s = Schema([Field("k", DataType.Int64, True), Field("x", DataType.Float64, True), Field("v", DataType.Int32, True)])
    b = RecordBatch(s, [Array.from_numpy(DataType.Int64, rng.integers(0, 1000, n) * 1_000_003, rng.random(n) >= 0.01),
                        Array.from_numpy(DataType.Float64, wild_doubles(rng, n), rng.random(n) >= 0.1),
                        Array.from_numpy(DataType.Int32, rng.integers(-2 ** 31, 2 ** 31 - 1, n).astype(np.int32),
                                         rng.random(n) >= 0.1)])
    aggs_e = [agg("SUM", Column(1), s), agg("COUNT", Column(1), s), agg("MIN", Column(1), s),
              agg("MAX", Column(2), s), agg("SUM", Column(2), s)]
    before = _bucketed_batches()
    out = run_multi(s, b, None, [Column(0)], aggs_e)
    assert out is not None and len(out[0]) == 1001
    assert _bucketed_batches() == before + 1


@pytest.mark.parametrize("buckets", ["0", "1"])
@pytest.mark.parametrize("hash_bits", [None, "3"])
def test_group_by_utf8_keys_inline_and_long(monkeypatch, buckets, hash_bits):
    """Utf8 keys of 0-60 bytes: those of at most 24 bytes are checked
    against the copy kept in their slot (groupby.h kInline), longer ones
    against the representative row / the arena -- over several batches, with
    every key forced onto 8 hash values (DFMI_GROUP_HASH_BITS=3: rows of
    other keys meet inline and long slot keys), atomic and bucketed passes."""
    monkeypatch.setenv("DFMI_DIAG", "1")
    monkeypatch.setenv("DFMI_GROUP_BUCKETS", buckets)
    if hash_bits:
        monkeypatch.setenv("DFMI_GROUP_HASH_BITS", hash_bits)
    rng = np.random.default_rng(72)
    n = 30_000
    words = [bytes(rng.integers(97, 123, int(ln)).astype(np.uint8)) for ln in rng.integers(0, 61, 400)]
    words += [b"x" * 24, b"x" * 25, b"x" * 23, b"y" * 8, b"y" * 16, b"\xff" * 24]
    s = Schema([Field("k", DataType.Utf8, True), Field("x", DataType.Float64, True), Field("j", DataType.Int64, True)])
    b = RecordBatch(s, [Array.from_strings([None if rng.random() < 0.02 else words[i]
                                            for i in rng.integers(0, len(words), n)]),
                        Array.from_numpy(DataType.Float64, wild_doubles(rng, n), rng.random(n) >= 0.05),
                        Array.from_numpy(DataType.Int64, rng.integers(0, 3, n), rng.random(n) >= 0.02)])
    aggs_e = [agg("SUM", Column(1), s), agg("COUNT", Column(1), s), agg("MAX", Column(1), s)]
    # one part (24 inline bytes), two and three parts (the arena / representative row)
    for keys in ([Column(0)], [Column(2), Column(0)], [Column(0), Column(2), Column(2)]):
        out = run_multi(s, b, None, keys, aggs_e, batch_rows=11_000)
        assert out is not None and len(out[0]) > 380


@pytest.mark.parametrize("buckets", ["0", "1"])
def test_group_by_every_argument_type(monkeypatch, buckets):
    """SUM / MIN / MAX / COUNT of every numeric argument type (Int8 ... UInt64,
    Float32) with NULLs, grouped by a Float64 key (the hash table), through the
    atomic accumulate pass and the bucketed passes (LDS records): signed
    values sign-extended, unsigned zero-extended, integer SUM wrapping."""
    monkeypatch.setenv("DFMI_DIAG", "1")
    monkeypatch.setenv("DFMI_GROUP_BUCKETS", buckets)
    rng = np.random.default_rng(73)
    n = 25_000
    types = [DataType.Int8, DataType.Int16, DataType.UInt8, DataType.UInt16, DataType.UInt32, DataType.UInt64,
             DataType.Float32]
    np_t = [np.int8, np.int16, np.uint8, np.uint16, np.uint32, np.uint64, np.float32]
    fields = [Field("g", DataType.Float64, True)] + [Field("c%d" % j, t, True) for j, t in enumerate(types)]
    cols = [Array.from_numpy(DataType.Float64, rng.integers(0, 300, n) / 3.0, rng.random(n) >= 0.02)]
    for t, nt in zip(types, np_t):
        if nt == np.float32:
            vals = (rng.standard_normal(n) * 1e3).astype(np.float32)
        else:
            info = np.iinfo(nt)
            vals = rng.integers(int(info.min), int(info.max), n, dtype=np.int64 if info.min < 0 else np.uint64,
                                endpoint=True).astype(nt)
        cols.append(Array.from_numpy(t, vals, rng.random(n) >= 0.1))
    s = Schema(fields)
    b = RecordBatch(s, cols)
    aggs_e = []
    for j in range(len(types)):
        for fn in ("SUM", "MIN", "MAX", "COUNT"):
            aggs_e.append(agg(fn, Column(1 + j), s))
    for start in range(0, len(aggs_e), 14):  # at most 15 aggregates per grouped state
        out = run_multi(s, b, None, [Column(0)], aggs_e[start:start + 14], batch_rows=9_000)
        assert out is not None and len(out[0]) > 290


@pytest.mark.parametrize("kt", ["int64", "uint64", "float64", "float32", "int8", "boolean"])
def test_group_by_device_emission(monkeypatch, kt):
    """The finish ordered and emitted on the device (aggregate.cpp
    finish_device: sort values, rocPRIM radix sort, the null group moved
    last, dfmi_agg_value records built on the device), forced on small
    tables (DFMI_GROUP_DEVICE_EMIT=1): keys at their type's extremes next to
    the null group (INT64_MAX and UINT64_MAX sort like the null group's
    ~0 before it is moved), Float64 / Float32 keys with NaN, -0.0 and
    infinities; SUM / COUNT / MIN / MAX of every kind -- equal to the oracle."""
    monkeypatch.setenv("DFMI_DIAG", "1")
    monkeypatch.setenv("DFMI_GROUP_DEVICE_EMIT", "1")
    rng = np.random.default_rng(74)
    n = 20_000
    dts = {"int64": (DataType.Int64, np.int64), "uint64": (DataType.UInt64, np.uint64),
           "float64": (DataType.Float64, np.float64), "float32": (DataType.Float32, np.float32),
           "int8": (DataType.Int8, np.int8), "boolean": (DataType.Boolean, np.bool_)}
    dt, nt = dts[kt]
    if kt in ("int64", "uint64", "int8"):
        info = np.iinfo(nt)
        pool = np.array([info.min, info.max, 0, 1, info.max - 1, info.min + 1] +
                        list(rng.integers(int(info.min), int(info.max), 500, endpoint=True,
                                          dtype=np.int64 if info.min < 0 else np.uint64)), dtype=nt)
    elif kt == "boolean":
        pool = np.array([False, True])
    else:
        pool = np.array([np.nan, -np.nan, 0.0, -0.0, np.inf, -np.inf, 1.5, -1.5] +
                        list(rng.standard_normal(500)), dtype=nt)
    keys = pool[rng.integers(0, len(pool), n)]
    s2, b2 = _rounding_table(rng, n)
    s = Schema([Field("k", dt, True)] + list(s2.fields[1:]) + [Field("i", DataType.Int16, True)])
    b = RecordBatch(s, [Array.from_numpy(dt, keys, rng.random(n) >= 0.03)] + list(b2.columns[1:]) +
                    [Array.from_numpy(DataType.Int16, rng.integers(-2 ** 15, 2 ** 15, n).astype(np.int16),
                                      rng.random(n) >= 0.1)])
    aggs_e = [agg("SUM", Column(1), s), agg("SUM", Column(2), s), agg("COUNT", Column(1), s),
              agg("MIN", Column(2), s), agg("MAX", Column(1), s), agg("SUM", Column(3), s),
              agg("MIN", Column(3), s), agg("MAX", Column(3), s)]
    for br in (0, 7_000):
        out = run_multi(s, b, None, [Column(0)], aggs_e, batch_rows=br)
        assert out is not None and len(out[0]) >= 3


def test_group_by_device_emission_chosen():
    """2^17 distinct Int64 keys (more than kDeviceEmitMin groups): the finish
    is ordered and emitted on the device without a diagnostics switch, and
    equals the oracle."""
    rng = np.random.default_rng(75)
    n = 1 << 18
    s = Schema([Field("k", DataType.Int64, True), Field("x", DataType.Float64, True)])
    b = RecordBatch(s, [Array.from_numpy(DataType.Int64, rng.permutation(n) // 2 * 1_000_003, rng.random(n) >= 0.01),
                        Array.from_numpy(DataType.Float64, wild_doubles(rng, n), rng.random(n) >= 0.1)])
    out = run_multi(s, b, None, [Column(0)], [agg("SUM", Column(1), s), agg("COUNT", Column(1), s)])
    assert out is not None and len(out[0]) > 130_000  # (keys whose two rows are both NULL fold into the null group)


def test_group_by_bucketed_large_lds(monkeypatch):
    """~38,000 groups of three exact Float64 SUMs: with 64 KiB of LDS a
    bucket holds 32 records, past the 1,024 buckets, so the bucket pass takes
    one 160 KiB workgroup per CU (64 records per bucket) -- the groups equal
    the oracle's (bucketed passes forced for the 1.2e5-row batch)."""
    monkeypatch.setenv("DFMI_DIAG", "1")
    monkeypatch.setenv("DFMI_GROUP_BUCKETS", "1")
    rng = np.random.default_rng(76)
    n = 120_000
    s = Schema([Field("k", DataType.Int64, True)] + [Field(c, DataType.Float64, True) for c in "xyz"])
    b = RecordBatch(s, [Array.from_numpy(DataType.Int64, rng.integers(0, 40_000, n) * 7, rng.random(n) >= 0.01)] +
                    [Array.from_numpy(DataType.Float64, wild_doubles(rng, n), rng.random(n) >= 0.05) for _ in range(3)])
    before = _bucketed_batches()
    aggs_e = [agg("SUM", Column(1), s), agg("SUM", Column(2), s), agg("SUM", Column(3), s), agg("COUNT", Column(1), s)]
    out = run_multi(s, b, None, [Column(0)], aggs_e, batch_rows=60_000)
    assert out is not None and len(out[0]) > 37_000
    assert _bucketed_batches() == before + 2
