#!/usr/bin/env python3
"""GROUP BY throughput by key kind (diagnostics): one 1e7-row device batch,
SUM / COUNT of a Float64 column grouped by a key column -- Int64 keys in a
16-value window (the fused grouped kernel), Int64 keys over 10,000 values,
Float64 keys (10,000 values), Utf8 keys (1,000 words and 10,000 words), two
keys Int64 x Utf8 (the device hash table: aggregate.cpp group_batch_hashed)
-- each timed end to end (state creation excluded, finish included) after a
warm-up, and the host-merge A/B (DFMI_DIAG=1 DFMI_GROUP_HOST=1) on the same
batches; --sweep: Float64 keys of 4 ... 1e6 distinct values instead.
--card=C1,C2: the sweep at those cardinalities only; --phases: add and
finish timed apart (add synchronised); --reuse: one state per case, reset
before each run (the hash table keeps the size it grew to, as a state that
takes many batches does).
usage: groupby_probe.py [rows] [--no-host] [--sweep] [--card=...] [--phases] [--reuse]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from datafusion_amd import _abi  # noqa: E402
from datafusion_amd.arrow import Array, DataType, Field, RecordBatch, Schema  # noqa: E402
from datafusion_amd.execution.engine import engine  # noqa: E402
from datafusion_amd.execution.expression import compile_expr, compile_scalar_expr  # noqa: E402
from datafusion_amd.logicalplan import AggregateFunction, Column  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else 10_000_000
host_ab = "--no-host" not in sys.argv
rng = np.random.default_rng(3)
eng = engine()
dev = eng.device
v = Array.from_numpy(DataType.Float64, rng.random(n)).to(dev)
words = [("w%d_" % i + "x" * (i % 17)) for i in range(10_000)]
CARDS = (4, 16, 100, 1000, 10_000, 100_000, 1_000_000)
PHASES = "--phases" in sys.argv
REUSE = "--reuse" in sys.argv  # one state per case, reset before each run (the table keeps its size)
for a in sys.argv:
    if a.startswith("--card="):
        CARDS = tuple(int(float(c)) for c in a[7:].split(","))
if "--sweep" in sys.argv:  # the hash table across key cardinalities (Float64 keys: always the hash path)
    cases = {"float64 %d" % c: [Array.from_numpy(DataType.Float64, rng.integers(0, c, n) / 7.0)]
             for c in CARDS}
else:
    cases = {
        "int64 window": [Array.from_numpy(DataType.Int64, rng.integers(0, 16, n))],
        "int64 10k": [Array.from_numpy(DataType.Int64, rng.integers(0, 10_000, n) * 7919)],
        "float64 10k": [Array.from_numpy(DataType.Float64, rng.integers(0, 10_000, n) / 7.0)],
        "utf8 1k": [Array.from_strings([words[i] for i in rng.integers(0, 1000, n)])],
        "utf8 10k": [Array.from_strings([words[i] for i in rng.integers(0, 10_000, n)])],
        "int64 x utf8 10k": [Array.from_numpy(DataType.Int64, rng.integers(0, 100, n)),
                             Array.from_strings([words[i] for i in rng.integers(0, 100, n)])],
    }
AGG = _abi.DFMI_FLAG_EXT_AGGREGATE


def run(name, kcols, reps=3):
    nk = len(kcols)
    s = Schema([Field("k%d" % i, k.data_type, False) for i, k in enumerate(kcols)] +
               [Field("v", DataType.Float64, False)])
    b = RecordBatch(s, [k.to(dev) for k in kcols] + [v])
    aggs = [AggregateFunction("SUM", (Column(nk),), DataType.Float64),
            AggregateFunction("COUNT", (Column(nk),), DataType.UInt64)]
    cs = [compile_expr(None, a, s, AGG) for a in aggs]
    kp = [compile_scalar_expr(None, Column(i), s, AGG) for i in range(nk)]
    best, groups, split = None, 0, None
    st = eng.grouped_agg_state(kp if nk > 1 else kp[0], cs) if REUSE else None
    for rep in range(reps + 1):  # rep 0 warms up (code objects, allocations, clocks)
        if REUSE:
            st.reset()
        else:
            st = eng.grouped_agg_state(kp if nk > 1 else kp[0], cs)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st.add(None, b, AGG)
        if PHASES:
            torch.cuda.synchronize()
        t1 = time.perf_counter()
        keys_out, vals = st.finish()
        el = time.perf_counter() - t0
        if rep and (best is None or el < best):
            best, split = el, (t1 - t0, el - (t1 - t0))
        groups = len(keys_out)
    if PHASES:
        print("  %s: add %.2f ms, finish %.2f ms" % (name, split[0] * 1e3, split[1] * 1e3), flush=True)
    return best, groups


for name, kcols in cases.items():
    el, g = run(name, kcols)
    line = "%-17s %8.2f ms  %9.3g rows/s  groups %6d" % (name, el * 1e3, n / el, g)
    if host_ab and name != "int64 window":
        os.environ["DFMI_DIAG"] = "1"
        os.environ["DFMI_GROUP_HOST"] = "1"
        he, hg = run(name, kcols, reps=1)
        del os.environ["DFMI_DIAG"], os.environ["DFMI_GROUP_HOST"]
        assert hg == g
        line += "   | host merge %8.1f ms %9.3g rows/s  (device %.0fx)" % (he * 1e3, n / he, he / el)
    print(line, flush=True)
