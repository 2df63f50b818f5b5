"""The on-disk code-object cache (csrc/jit.cpp, DFMI_JIT_CACHE_DIR): a query
shape compiled by one process is loaded, not compiled, by the next -- the
reference's compile_scalar_expr is a cheap closure build per query
(context.rs:131,152-155), so a fresh process must not pay ~190 ms of hipRTC
for a shape it has seen before. Each child process runs the same query on a
fresh engine and checks its result against the oracle."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import ctypes as C, json, sys, time
sys.path.insert(0, %(root)r); sys.path.insert(0, %(root)r + "/tests")
import numpy as np, torch
from datafusion_amd import _abi
from datafusion_amd.arrow import Array, Field, RecordBatch, Schema
from datafusion_amd.execution.engine import engine
from datafusion_amd.execution.expression import compile_scalar_expr
from datafusion_amd.logicalplan import BinaryExpr, Column, DataType, Float64, Literal, Operator
from oracle_ffi import oracle_filter_project
torch.cuda.set_device(0)
(torch.zeros(1, device="cuda") + 1).sum().item()  # runtime initialised before the timed call
eng = engine("cuda:0")
s = Schema([Field("a", DataType.Float64, True), Field("b", DataType.Float64, False), Field("c", DataType.Float64, False)])
rng = np.random.default_rng(3)
n = 50_000
b = RecordBatch(s, [Array.from_numpy(DataType.Float64, rng.random(n), rng.random(n) > 0.1),
                    Array.from_numpy(DataType.Float64, rng.standard_normal(n)),
                    Array.from_numpy(DataType.Float64, rng.random(n))])
db = b.to("cuda:0")
pred = BinaryExpr(BinaryExpr(Column(0), Operator.Lt, Literal(Float64(0.61))), Operator.Or,
                  BinaryExpr(Column(2), Operator.GtEq, Column(0)))
projs = [BinaryExpr(BinaryExpr(Column(2), Operator.Minus, Column(0)), Operator.Divide, Literal(Float64(3.0))),
         Column(0)]
p = compile_scalar_expr(None, pred, s)
cp = [compile_scalar_expr(None, e, s) for e in projs]
torch.cuda.synchronize()
t0 = time.perf_counter()
got = eng.filter_project(p, cp, db)
first_ms = (time.perf_counter() - t0) * 1e3
cm = C.c_double()
_abi.lib().dfmi_last_compile_ms(eng.ctx, C.byref(cm))
ref = oracle_filter_project(s, b, pred, projs)
ok = all(d.length == r.length and
         np.array_equal(d.cpu().numpy_values().view(np.uint64)[r.valid_mask()],
                        r.numpy_values().view(np.uint64)[r.valid_mask()]) for d, (_, r) in zip(got, ref))
print(json.dumps({"compile_ms": cm.value, "first_ms": first_ms, "rows": got[0].length, "ok": bool(ok)}))
"""


def run_child(cache_dir):
    env = dict(os.environ, DFMI_JIT_CACHE_DIR=str(cache_dir))
    out = subprocess.run([sys.executable, "-c", CHILD % {"root": ROOT}], env=env, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_second_process_loads_the_code_object(tmp_path):
    first = run_child(tmp_path)
    assert first["ok"] and first["compile_ms"] > 0, first
    assert any(f.endswith(".co") for f in os.listdir(tmp_path))
    second = run_child(tmp_path)
    assert second["ok"] and second["rows"] == first["rows"], second
    assert second["compile_ms"] == 0, second
    assert second["first_ms"] <= 5.0, (first, second)


def test_damaged_cache_file_is_compiled_again(tmp_path):
    run_child(tmp_path)
    for f in os.listdir(tmp_path):
        if f.endswith(".co"):
            with open(tmp_path / f, "r+b") as fh:
                fh.seek(-16, 2)
                fh.truncate()  # cut short: the file no longer checks out
    again = run_child(tmp_path)
    assert again["ok"] and again["compile_ms"] > 0, again
