#!/usr/bin/env python3
"""cProfile of the relation pull loop over 1024-row host batches (bench.py
relation_1024_host's pull_and_columns loop, one pass after a warm pass):
where the main thread's Python time goes."""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from datafusion_amd.arrow import Array, DataType, Field, RecordBatch, Schema  # noqa: E402
from datafusion_amd.execution import ExecutionContext, MemoryDataSource  # noqa: E402
from oracle_ffi import gen_unit_f64  # noqa: E402

m, nb = 1024, 4096
n = m * nb
host = [torch.from_numpy(gen_unit_f64(bench.SEED, j, 0, n).view(np.uint8)) for j in range(3)]
schema = Schema([Field(c, DataType.Float64, False) for c in "abc"])
sql = "SELECT a, b, a * b + c FROM t WHERE a > %r AND b < %r" % (1 - 0.5 ** 0.5, 0.5 ** 0.5)


def batches():
    return [RecordBatch(schema, [Array(DataType.Float64, m, t[i * m * 8:(i + 1) * m * 8]) for t in host]) for i in range(nb)]


def loop(bs):
    ctx = ExecutionContext(coalesce=256)
    ctx.register_datasource("t", MemoryDataSource(schema, bs))
    r = ctx.sql(sql)
    rows = 0
    while True:
        b = r.next()
        if b is None:
            break
        rows += b.columns[-1].length
    return rows


loop(batches())
bs = batches()
pr = cProfile.Profile()
pr.enable()
loop(bs)
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
