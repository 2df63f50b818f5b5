#!/usr/bin/env python3
"""GROUP BY throughput by key kind (diagnostics): one 1e7-row device batch,
SUM / COUNT of a Float64 column grouped by a key column -- Int64 keys in a
16-value window (device kernel), Int64 keys over 10,000 values, Float64 keys
(10,000 values), Utf8 keys (1,000 words) (the last three: host merge)."""
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

n = 10_000_000
rng = np.random.default_rng(3)
eng = engine()
dev = eng.device
v = Array.from_numpy(DataType.Float64, rng.random(n)).to(dev)
words = [("w%d_" % i + "x" * (i % 17)) for i in range(1000)]
keys = {
    "int64 window": Array.from_numpy(DataType.Int64, rng.integers(0, 16, n)),
    "int64 wide": Array.from_numpy(DataType.Int64, rng.integers(0, 10_000, n) * 7919),
    "float64": Array.from_numpy(DataType.Float64, rng.integers(0, 10_000, n) / 7.0),
    "utf8": Array.from_strings([words[i] for i in rng.integers(0, 1000, n)]),
}
AGG = _abi.DFMI_FLAG_EXT_AGGREGATE
for name, k in keys.items():
    s = Schema([Field("k", k.data_type, False), Field("v", DataType.Float64, False)])
    b = RecordBatch(s, [k.to(dev), v])
    aggs = [AggregateFunction("SUM", (Column(1),), DataType.Float64),
            AggregateFunction("COUNT", (Column(1),), DataType.UInt64)]
    cs = [compile_expr(None, a, s, AGG) for a in aggs]
    kp = compile_scalar_expr(None, Column(0), s, AGG)
    for rep in range(2):
        st = eng.grouped_agg_state(kp, cs)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st.add(None, b, AGG)
        keys_out, vals = st.finish()
        el = time.perf_counter() - t0
    print("%-13s %8.1f ms  %6.3g rows/s  groups %d" % (name, el * 1e3, n / el, len(keys_out)), flush=True)
