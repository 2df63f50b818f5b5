#!/usr/bin/env python3
"""dfmi_filter_project_host on one 1024-row host batch per call (bench.py's
1024_rows_host line) in a loop, for rocprofv3 kernel / memory-copy traces of
the small host call. usage: tools/host_small_probe.py [calls]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

import bench  # noqa: E402
from datafusion_amd.arrow import DataType, Field, Schema  # noqa: E402
from datafusion_amd.execution.engine import engine  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = engine(dev)
    schema = Schema([Field(c, DataType.Float64, False) for c in "abc"])
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    print(json.dumps(bench.host_small_batches(eng, schema, 0.5, 1024, calls=calls)))


if __name__ == "__main__":
    main()
