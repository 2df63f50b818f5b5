#!/usr/bin/env python3
"""Per-call host cost of dfmi_filter_project at the reference's batch size
(1024 rows, csv_sql.rs:49): wall time per call and, with DFMI_DIAG=1
DFMI_CALL_PROFILE=1 in the environment, the library's phase breakdown.
usage: DFMI_DIAG=1 DFMI_CALL_PROFILE=1 tools/call_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

import bench  # noqa: E402
from datafusion_amd import _abi  # noqa: E402
from datafusion_amd.arrow import DataType, Field, Schema  # noqa: E402
from datafusion_amd.execution.engine import engine  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = engine(dev)
    n = 1 << 20
    cols = [torch.empty(n, dtype=torch.float64, device=dev) for _ in range(3)]
    L = _abi.lib()
    err = _abi.dfmi_error()
    for j, c in enumerate(cols):
        L.dfmi_generate_column(eng.ctx, 1, bench.SEED, j, 0, n, 0, 0, c.data_ptr(), bench.C.byref(err))
    torch.cuda.synchronize(dev)
    schema = Schema([Field(c, DataType.Float64, False) for c in "abc"])
    for m in (1024, 1 << 20):
        outs = [torch.empty(m, dtype=torch.float64, device=dev) for _ in range(3)]
        step = bench.FusedStep(eng, schema, cols, m, *bench.query(0.5), outs)
        for _ in range(100):
            step()
        for timing in (1, 0):
            L.dfmi_context_set_timing(eng.ctx, timing)
            t0 = time.perf_counter()
            for _ in range(3000):
                step()
            el = (time.perf_counter() - t0) / 3000
            print("rows %d, timing events %d: %.2f us per call" % (m, timing, el * 1e6), flush=True)
        L.dfmi_context_set_timing(eng.ctx, 1)


if __name__ == "__main__":
    main()
