#!/usr/bin/env python3
"""Where the relations' pull loop over 1024-row HOST batches spends its time
(bench.py relation_1024_host): total per pulled batch, and the main thread's
time waiting for the worker's native call, reading ahead (source + struct
packing + submit) and building the result batches.
usage: tools/relation_probe.py [nbatches] [coalesce]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import datafusion_amd.execution.engine as E  # noqa: E402
import datafusion_amd.execution.filter as F  # noqa: E402
from datafusion_amd.arrow import Array, Field, RecordBatch, Schema  # noqa: E402
from datafusion_amd.execution import ExecutionContext, MemoryDataSource  # noqa: E402
from datafusion_amd.logicalplan import DataType  # noqa: E402

T = {"wait": 0.0, "fetch": 0.0, "finish": 0.0}


def timed(name, fn):
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            T[name] += time.perf_counter() - t0
    return w


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    co = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    torch.cuda.set_device(0)
    m = 1024
    rng = np.random.default_rng(1)
    host = [torch.from_numpy(rng.random(m * nb).view(np.uint8)) for _ in range(3)]
    schema = Schema([Field(c, DataType.Float64, False) for c in "abc"])
    sql = "SELECT a, b, a * b + c FROM t WHERE a > 0.29 AND b < 0.71"
    orig_result = E.HostBatchesFuture.result

    def result(self):
        t0 = time.perf_counter()
        raw = self.fut.result()
        T["wait"] += time.perf_counter() - t0
        if self.eng._inflight is self.fut:
            self.eng._inflight = None
        t1 = time.perf_counter()
        out = E.DeviceEngine._host_batches_finish(self.prep, raw, self.schema)
        T["finish"] += time.perf_counter() - t1
        return out
    E.HostBatchesFuture.result = result
    F.Coalescer._fetch = timed("fetch", F.Coalescer._fetch)
    for rep in range(4):
        for k in T:
            T[k] = 0.0
        bs = [RecordBatch(schema, [Array(DataType.Float64, m, t[i * m * 8:(i + 1) * m * 8]) for t in host])
              for i in range(nb)]
        ctx = ExecutionContext(coalesce=co)
        ctx.register_datasource("t", MemoryDataSource(schema, bs))
        r = ctx.sql(sql)
        t0 = time.perf_counter()
        rows = 0
        while True:
            b = r.next()
            if b is None:
                break
            rows += b.num_rows()
        el = time.perf_counter() - t0
        print("rep %d: %.3f us/batch  wait %.3f  fetch %.3f  finish %.3f  rest %.3f (us per batch)" % (
            rep, el / nb * 1e6, T["wait"] / nb * 1e6, T["fetch"] / nb * 1e6, T["finish"] / nb * 1e6,
            (el - T["wait"] - T["fetch"] - T["finish"]) / nb * 1e6), flush=True)
    E.HostBatchesFuture.result = orig_result


if __name__ == "__main__":
    main()
