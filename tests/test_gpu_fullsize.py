"""Parity at BASELINE.json's full sizes (C2: 1e9 rows, C4: 600,037,902 rows,
C3: one 1.25e8-row batch), where the CPU oracle would take minutes: the device
outputs are checked bit for bit against the same selection and projection
computed with plain torch ops on the device (separate multiply and add
kernels: one IEEE rounding per operator, as the reference's scalar loops and
the oracle). The oracle itself pins the same query shapes at smaller sizes
(test_gpu_parity.py) and on a 4M-row prefix of these tables (bench.py's
parity gates)."""
import ctypes as C
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from datafusion_amd import _abi  # noqa: E402
from datafusion_amd.arrow import Array, RecordBatch  # noqa: E402
from datafusion_amd.execution.engine import engine  # noqa: E402
from datafusion_amd.execution.expression import compile_scalar_expr  # noqa: E402
from datafusion_amd.logicalplan import BinaryExpr, Column, DataType, Float64, Literal, Operator  # noqa: E402
from datafusion_amd.arrow import Field, Schema  # noqa: E402

pytestmark = pytest.mark.gpu


def _bits(t):
    return t.contiguous().view(torch.int64)


def _run(eng, schema, cols, pred_e, proj_e):
    pred = compile_scalar_expr(None, pred_e, schema)
    projs = [compile_scalar_expr(None, e, schema) for e in proj_e]
    return eng.filter_project(pred, projs, RecordBatch(schema, cols))


@pytest.mark.parametrize("sel", [0.01, 0.5, 0.99])
def test_c2_full_size_against_torch(sel):
    dev = torch.device("cuda", 0)
    eng = engine(dev)
    n = 1_000_000_000
    cols = [torch.empty(n, dtype=torch.float64, device=dev) for _ in range(3)]
    err = _abi.dfmi_error()
    for j, t in enumerate(cols):
        rc = _abi.lib().dfmi_generate_column(eng.ctx, _abi.DFMI_GEN_UNIT_F64, bench.SEED, j, 0, n, 0, 0,
                                              C.c_void_p(t.data_ptr()), C.byref(err))
        assert rc == 0, err.message
    schema = Schema([Field(c, DataType.Float64, False) for c in "abc"])
    pred_e, proj_e = bench.query(sel)
    got = _run(eng, schema, [Array(DataType.Float64, n, c.view(torch.uint8)) for c in cols], pred_e, proj_e)
    k, m = 1.0 - sel ** 0.5, sel ** 0.5
    a, b, c = cols
    mask = (a > k) & (b < m)
    sa, sb = a[mask], b[mask]
    want = [sa, sb, (sa * sb) + c[mask]]
    assert got[0].length == sa.numel()
    assert abs(sa.numel() / n - sel) < 1e-3
    for g, w in zip(got, want):
        assert g.length == w.numel() and g.null_count == 0
        assert torch.equal(_bits(g.values[: 8 * g.length].view(torch.float64)), _bits(w))
    del got, want, mask, sa, sb, cols
    torch.cuda.empty_cache()


def test_c4_full_size_against_torch():
    dev = torch.device("cuda", 0)
    eng = engine(dev)
    n = bench.Q6_ROWS
    schema, cols = bench.q6_table(dev, n, bench.SEED)
    pred_e, proj_e = bench.q6_query()
    got = _run(eng, schema, [Array(DataType.Float64, n, c.view(torch.uint8)) for c in cols], pred_e, proj_e)
    qty, price, disc, ship = cols
    mask = (ship >= 8766.0) & (ship < 9131.0) & (disc >= 0.05) & (disc <= 0.07) & (qty < 24.0)
    want = price[mask] * disc[mask]
    assert got[0].length == want.numel() and 0.015 < want.numel() / n < 0.025
    assert torch.equal(_bits(got[0].values[: 8 * got[0].length].view(torch.float64)), _bits(want))
    del got, want, mask, cols
    torch.cuda.empty_cache()


def test_c3_full_batch_against_torch():
    """One C3 batch (1.25e8 rows, ~1.7 GB of Utf8 bytes): SELECT s, v WHERE
    v < 0.5 over nullable v -- a null v IS selected: arrow 0.12's bool_op
    compares Option<f64>, where None < Some(x)."""
    dev = torch.device("cuda", 0)
    eng = engine(dev)
    words = bench._utf8_dictionary(bench.SEED)
    import numpy as np
    dict_bytes = torch.tensor(np.frombuffer(b"".join(words), dtype=np.uint8), device=dev)
    dict_len = torch.tensor([len(w) for w in words], dtype=torch.int64, device=dev)
    dict_off = torch.cumsum(dict_len, 0) - dict_len
    g = torch.Generator(device=dev)
    g.manual_seed(bench.SEED + 1000)
    n = bench.C3_ROWS // bench.C3_BATCHES
    (s, v), _ = bench._c3_batch(dev, g, n, dict_bytes, dict_off, dict_len)
    schema = Schema([Field("s", DataType.Utf8, False), Field("v", DataType.Float64, True)])
    got = _run(eng, schema, [s, v], BinaryExpr(Column(1), Operator.Lt, Literal(Float64(0.5))), [Column(0), Column(1)])
    vals = v.values.view(torch.float64)
    vb = v.validity
    valid = ((vb.unsqueeze(1) >> torch.arange(8, device=dev, dtype=torch.uint8)) & 1).reshape(-1)[:n].bool()
    mask = ~valid | (vals < 0.5)
    rows = torch.nonzero(mask).squeeze(1)
    _check_gather(got, s, vals, rows)
    del got, s, v
    torch.cuda.empty_cache()


def test_c3_full_batch_equality_against_torch():
    """One C3 batch through bench.py's equality query: SELECT s, v WHERE
    s = <word 17> (DFMI_FLAG_EXT_UTF8_COMPARE; the reference compares the
    strings' bytes, filter.rs:99-100 reading get_string). The torch mask
    compares every row's length and bytes with the literal's."""
    from datafusion_amd.logicalplan import Utf8
    dev = torch.device("cuda", 0)
    eng = engine(dev)
    words = bench._utf8_dictionary(bench.SEED)
    import numpy as np
    dict_bytes = torch.tensor(np.frombuffer(b"".join(words), dtype=np.uint8), device=dev)
    dict_len = torch.tensor([len(w) for w in words], dtype=torch.int64, device=dev)
    dict_off = torch.cumsum(dict_len, 0) - dict_len
    g = torch.Generator(device=dev)
    g.manual_seed(bench.SEED + 1000)
    n = bench.C3_ROWS // bench.C3_BATCHES
    (s, v), _ = bench._c3_batch(dev, g, n, dict_bytes, dict_off, dict_len)
    schema = Schema([Field("s", DataType.Utf8, False), Field("v", DataType.Float64, True)])
    w = words[17]
    fl = _abi.DFMI_FLAG_EXT_UTF8_COMPARE
    pred = compile_scalar_expr(None, BinaryExpr(Column(0), Operator.Eq, Literal(Utf8(w.decode()))), schema, fl)
    projs = [compile_scalar_expr(None, Column(c), schema, fl) for c in (0, 1)]
    got = eng.filter_project(pred, projs, RecordBatch(schema, [s, v]), fl)
    offs = s.offsets.to(torch.int64)
    lens = offs[1:] - offs[:-1]
    rows = torch.nonzero(lens == len(w)).squeeze(1)
    lit = torch.tensor(list(w), dtype=torch.uint8, device=dev)
    keep = torch.ones(rows.numel(), dtype=torch.bool, device=dev)
    for j in range(len(w)):  # byte j of every row of the literal's length
        keep &= s.values[offs[rows] + j] == lit[j]
    rows = rows[keep]
    assert 0 < rows.numel() < n // 100
    _check_gather(got, s, v.values.view(torch.float64), rows)
    del got, s, v
    torch.cuda.empty_cache()


def _check_gather(got, s, vals, rows):
    """SELECT s, v over the selected `rows`: bit-exact v slots (no validity in
    the filtered batch) and s as rebased offsets + concatenated bytes."""
    dev = vals.device
    sel = rows.numel()
    assert got[0].length == got[1].length == sel
    # v: the selected slots' bits, no validity in the filtered batch
    assert got[1].null_count == 0
    assert torch.equal(_bits(got[1].values[: 8 * sel].view(torch.float64)), _bits(vals[rows]))
    # s: rebased i32 offsets and the selected strings' bytes, concatenated
    offs = s.offsets.to(torch.int64)
    lens = offs[rows + 1] - offs[rows]
    want_offs = torch.zeros(sel + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens, 0, out=want_offs[1:])
    assert torch.equal(got[0].offsets[: sel + 1].to(torch.int64), want_offs)
    total = int(want_offs[-1].item())
    gb = got[0].values[:total]
    step = 1 << 24
    for r0 in range(0, sel, step):  # bounded-memory chunks of selected rows
        r1 = min(sel, r0 + step)
        li = lens[r0:r1]
        k = torch.repeat_interleave(torch.arange(r0, r1, device=dev), li)
        within = torch.arange(k.numel(), device=dev) - (want_offs[k] - want_offs[r0])
        want = s.values[offs[rows[k]] + within]
        assert torch.equal(gb[want_offs[r0]:want_offs[r1]], want), (r0, r1)


def test_q6_full_size_exact_sum():
    """Real Q6 (DFMI_FLAG_EXT_AGGREGATE) over 600,037,902 rows: the device SUM
    of extendedprice*discount over the selected rows is the correctly rounded
    exact sum of the rounded products (math.fsum), and its count is the mask's."""
    import math
    import numpy as np
    from datafusion_amd.execution.expression import compile_expr
    from datafusion_amd.logicalplan import AggregateFunction
    dev = torch.device("cuda", 0)
    eng = engine(dev)
    flags = _abi.DFMI_FLAG_EXT_AGGREGATE
    n = bench.Q6_ROWS
    schema, cols = bench.q6_table(dev, n, bench.SEED)
    pred_e, proj_e = bench.q6_query()
    agg = compile_expr(None, AggregateFunction("SUM", (proj_e[0],), DataType.Float64), schema, flags)
    st = eng.agg_state([agg])
    st.add(compile_scalar_expr(None, pred_e, schema, flags),
           RecordBatch(schema, [Array(DataType.Float64, n, c.view(torch.uint8)) for c in cols]), flags)
    v = st.finish()[0]
    qty, price, disc, ship = cols
    mask = (ship >= 8766.0) & (ship < 9131.0) & (disc >= 0.05) & (disc <= 0.07) & (qty < 24.0)
    prods = (price[mask] * disc[mask]).cpu().numpy()
    assert v.count == prods.size
    want = math.fsum(prods.tolist())
    assert v.bits == int(np.array([want], dtype=np.float64).view(np.uint64)[0])
    del cols, mask
    torch.cuda.empty_cache()
