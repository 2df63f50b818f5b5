"""Two processes time-sharing one GPU: each runs the C2 query
over its own HBM-resident 3e7-row table many times, and every launch must
finish without a look-back timeout and with the oracle's selected-row count
(single-pass look-back progress does not depend on having the GPU alone)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r"""
import ctypes as C, json, sys
import numpy as np, torch
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + "/tests")
from datafusion_amd import _abi
from datafusion_amd.arrow import Array, Field, RecordBatch, Schema
from datafusion_amd.execution.engine import engine
from datafusion_amd.execution.expression import compile_scalar_expr
from datafusion_amd.logicalplan import BinaryExpr, Column, DataType, Float64, Literal, Operator
from oracle_ffi import gen_unit_f64
seed, n, reps = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
dev = torch.device("cuda", 0)
eng = engine(dev)
host = [gen_unit_f64(seed, j, 0, n) for j in range(2)]
expect = int(np.count_nonzero((host[0] > 0.3) & (host[1] < 0.6)))
schema = Schema([Field(c, DataType.Float64, False) for c in "ab"])
batch = RecordBatch(schema, [Array(DataType.Float64, n, torch.from_numpy(h.view(np.uint8)).to(dev)) for h in host])
pred = compile_scalar_expr(None, BinaryExpr(BinaryExpr(Column(0), Operator.Gt, Literal(Float64(0.3))), Operator.And,
                                            BinaryExpr(Column(1), Operator.Lt, Literal(Float64(0.6)))), schema)
projs = [compile_scalar_expr(None, BinaryExpr(Column(0), Operator.Multiply, Column(1)), schema)]
counts = set()
for _ in range(reps):
    counts.add(eng.filter_project(pred, projs, batch)[0].length)
print(json.dumps({"expect": expect, "counts": sorted(counts)}), flush=True)
"""


@pytest.mark.gpu
def test_two_processes_share_one_gpu(tmp_path):
    script = tmp_path / "worker.py"
    script.write_text(WORKER)
    env = dict(os.environ)
    procs = [subprocess.Popen([sys.executable, str(script), ROOT, str(7 + i), str(30_000_000), "60"],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env) for i in range(2)]
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        assert p.returncode == 0, e[-2000:]
        outs.append(json.loads(o.strip().splitlines()[-1]))
    for r in outs:
        assert r["counts"] == [r["expect"]], r


@pytest.mark.gpu
def test_relaunch_after_lookback_timeout(monkeypatch):
    """exec.cpp relaunches a launch whose look-back timed out once (over a
    re-zeroed workspace) before reporting DFMI_ERR_DEVICE: a forced timeout
    (diagnostic mode bit 4) still returns the oracle's result."""
    import ctypes as C

    import numpy as np
    from datafusion_amd import _abi
    from datafusion_amd.arrow import Array, Field, RecordBatch, Schema
    from datafusion_amd.execution.engine import engine
    from datafusion_amd.execution.expression import compile_scalar_expr
    from datafusion_amd.logicalplan import BinaryExpr, Column, DataType, Float64, Literal, Operator
    from oracle_ffi import gen_unit_f64, oracle_filter_project
    from test_gpu_parity import assert_same
    n = 300_001
    s = Schema([Field(c, DataType.Float64, False) for c in "ab"])
    b = RecordBatch(s, [Array.from_numpy(DataType.Float64, gen_unit_f64(9, j, 0, n)) for j in range(2)])
    pred_e = BinaryExpr(Column(0), Operator.Lt, Literal(Float64(0.5)))
    proj_e = [Column(1), BinaryExpr(Column(0), Operator.Plus, Column(1))]
    ref = oracle_filter_project(s, b, pred_e, proj_e)
    eng = engine()
    L = _abi.lib()
    L.dfmi_internal_relaunches.argtypes = [C.c_void_p]
    L.dfmi_internal_relaunches.restype = C.c_long
    before = L.dfmi_internal_relaunches(eng.ctx)
    monkeypatch.setenv("DFMI_DIAG", "1")
    monkeypatch.setenv("DFMI_DEBUG_MODE", "16")
    out = eng.filter_project(compile_scalar_expr(None, pred_e, s), [compile_scalar_expr(None, e, s) for e in proj_e], b)
    assert L.dfmi_internal_relaunches(eng.ctx) == before + 1
    for d, (_, r) in zip(out, ref):
        assert_same(d.cpu(), r)


@pytest.mark.gpu
@pytest.mark.parametrize("host", [False, True])
def test_batches_relaunch_after_lookback_timeout(monkeypatch, host):
    """The coalesced entry points (dfmi_filter_project_batches and its host
    form) relaunch a launch whose look-back timed out once, over re-zeroed
    workspace and batch headers, like the single-batch path: a forced
    timeout still returns every batch's oracle result."""
    import ctypes as C

    from datafusion_amd import _abi
    from datafusion_amd.arrow import Array, Field, RecordBatch, Schema
    from datafusion_amd.execution.engine import engine
    from datafusion_amd.execution.expression import compile_scalar_expr
    from datafusion_amd.logicalplan import BinaryExpr, Column, DataType, Float64, Literal, Operator
    from oracle_ffi import gen_unit_f64, oracle_filter_project
    from test_gpu_parity import assert_same
    s = Schema([Field(c, DataType.Float64, False) for c in "ab"])
    bs = [RecordBatch(s, [Array.from_numpy(DataType.Float64, gen_unit_f64(9 + i, j, 0, n)) for j in range(2)])
          for i, n in enumerate([1024, 70_000, 3, 1024])]
    pred_e = BinaryExpr(Column(0), Operator.Lt, Literal(Float64(0.5)))
    proj_e = [Column(1), BinaryExpr(Column(0), Operator.Plus, Column(1))]
    eng = engine()
    L = _abi.lib()
    L.dfmi_internal_relaunches.argtypes = [C.c_void_p]
    L.dfmi_internal_relaunches.restype = C.c_long
    before = L.dfmi_internal_relaunches(eng.ctx)
    monkeypatch.setenv("DFMI_DIAG", "1")
    monkeypatch.setenv("DFMI_DEBUG_MODE", "16")
    p, cp = compile_scalar_expr(None, pred_e, s), [compile_scalar_expr(None, e, s) for e in proj_e]
    if host:
        got, err = eng.filter_project_host_batches(p, cp, bs)
    else:
        got, err = eng.filter_project_batches(p, cp, [b.to(eng.device) for b in bs])
    assert err is None, err
    assert L.dfmi_internal_relaunches(eng.ctx) == before + 1
    for b, g in zip(bs, got):
        for d, (_, r) in zip(g, oracle_filter_project(s, b, pred_e, proj_e)):
            assert_same(d.cpu(), r)
