"""Ticket-ordered tiles (Launch::ticket): each block takes its tile from an
atomic counter in the order blocks start, so a look-back only ever waits on
tiles whose blocks are running. dfmi_filter_project and the coalesced
batches relaunch with it after a look-back timeout -- the case of two
processes sharing one GPU, where the CUs the next tiles in dispatch order
need can be held by the other process's kernel, itself waiting. Forced here
from the first launch (DFMI_DIAG=1 DFMI_TICKET=1) over the one-tile,
sub-tile, Utf8-gather and coalesced kernels, bit-identical to the oracle;
and two processes running the low-selectivity sub-tile kernel side by side
on one GPU finish every launch with the oracle's counts."""
import json
import os
import subprocess
import sys

import pytest

from test_gpu_parity import run_both, synth, test_utf8_gather_and_equality, test_utf8_multi_channel_many_tiles
from test_gpu_slice import test_coalesced_sliced
from test_gpu_subtiles import c2

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def ticket(monkeypatch):
    monkeypatch.setenv("DFMI_DIAG", "1")
    monkeypatch.setenv("DFMI_TICKET", "1")


@pytest.mark.parametrize("n", [1, 4097, 100_003, (1 << 20) + 5])
@pytest.mark.parametrize("sel", [0.01, 0.5])
@pytest.mark.parametrize("subtiles", [None, "4"])
def test_c2(ticket, monkeypatch, n, sel, subtiles):
    if subtiles:
        monkeypatch.setenv("DFMI_NUMERIC_SUBTILES", subtiles)
    s, batch = synth(n)
    assert run_both(s, batch, *c2(sel)) is not None


def test_utf8(ticket):
    test_utf8_gather_and_equality()
    test_utf8_multi_channel_many_tiles()


@pytest.mark.parametrize("host", [False, True])
def test_coalesced(ticket, host):
    test_coalesced_sliced(host)


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
host = [gen_unit_f64(seed, j, 0, n) for j in range(3)]
expect = int(np.count_nonzero((host[0] > 0.9) & (host[1] < 0.1)))
schema = Schema([Field(c, DataType.Float64, False) for c in "abc"])
batch = RecordBatch(schema, [Array(DataType.Float64, n, torch.from_numpy(h.view(np.uint8)).to(dev)) for h in host])
pred = compile_scalar_expr(None, BinaryExpr(BinaryExpr(Column(0), Operator.Gt, Literal(Float64(0.9))), Operator.And,
                                            BinaryExpr(Column(1), Operator.Lt, Literal(Float64(0.1)))), schema)
projs = [compile_scalar_expr(None, BinaryExpr(Column(0), Operator.Multiply, Column(2)), schema)]
L = _abi.lib()
L.dfmi_internal_relaunches.argtypes = [C.c_void_p]
L.dfmi_internal_relaunches.restype = C.c_long
counts = set()
for _ in range(reps):
    counts.add(eng.filter_project(pred, projs, batch)[0].length)
print(json.dumps({"expect": expect, "counts": sorted(counts),
                  "relaunches": L.dfmi_internal_relaunches(eng.ctx)}), flush=True)
"""


@pytest.mark.parametrize("shared", [False, True])
def test_two_processes_share_one_gpu_subtiles(tmp_path, shared):
    """The low-selectivity sub-tile kernel (1% of rows selected: chosen from
    the second launch on) in two processes at once. With DFMI_SHARED=1 the
    contexts know they share the GPU and start in ticket order: no launch
    waits out the look-back timeout, so nothing is relaunched."""
    script = tmp_path / "worker.py"
    script.write_text(WORKER)
    env = dict(os.environ)
    env.pop("DFMI_SHARED", None)
    if shared:
        env["DFMI_SHARED"] = "1"
    procs = [subprocess.Popen([sys.executable, str(script), ROOT, str(11 + i), str(30_000_000), "80"],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
             for i in range(2)]
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=110)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        assert p.returncode == 0, e[-2000:]
        outs.append(json.loads(o.strip().splitlines()[-1]))
    for r in outs:
        assert r["counts"] == [r["expect"]], r
        if shared:
            assert r["relaunches"] == 0, r
