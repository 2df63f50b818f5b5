"""CSV ingest probe: opens the 5M-row C2 CSV file (bench.py csv_line's) three times
and reads it batch by batch; DFMI_CSV_PROFILE=1 prints index / per-batch parse times."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, ROOT); sys.path.insert(0, ROOT + "/tests")
import numpy as np, pandas as pd
from datafusion_amd.arrow import Field, Schema
from datafusion_amd.logicalplan import DataType
from datafusion_amd.execution import NativeCsvDataSource
from oracle_ffi import gen_unit_f64
n = 5_000_000
path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "dfmi_c2probe.csv")
if not os.path.exists(path):
    pd.DataFrame({c: gen_unit_f64(42, j, 0, n) for j, c in enumerate("abc")}).to_csv(path, index=False)
schema = Schema([Field(c, DataType.Float64, False) for c in "abc"])
for rep in range(3):
    t0 = time.perf_counter()
    src = NativeCsvDataSource(schema, path, True, 1 << 20, copy=False)
    t1 = time.perf_counter()
    rows = 0
    while True:
        b = src.next()
        if b is None: break
        rows += b.num_rows()
    t2 = time.perf_counter()
    print(rep, rows, "open %.1f ms, batches %.1f ms, %.2f GB/s" % ((t1-t0)*1e3, (t2-t1)*1e3, os.path.getsize(path)/(t2-t0)/1e9))
