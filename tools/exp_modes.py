"""Diagnostics: time k_filter_project under environment variants (tile shape,
LDS staging, debug modes), interleaved in one process."""
import os
import sys
import ctypes as C
import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import FusedStep  # noqa
from datafusion_amd import _abi  # noqa
from datafusion_amd.arrow import Field, Schema  # noqa
from datafusion_amd.execution.engine import engine  # noqa
from datafusion_amd.logicalplan import DataType  # noqa

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
sels = [float(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0.01,0.5,0.99").split(",")]
# variants: "cfg:mode:nolds" triples
variants = (sys.argv[3] if len(sys.argv) > 3 else "0:0:0,0:3:0,3:0:0,3:3:0,0:0:1").split(",")
dev = torch.device("cuda", 0)
eng = engine(dev)
cols = [torch.empty(n, dtype=torch.float64, device=dev) for _ in range(3)]
err = _abi.dfmi_error()
for j, t in enumerate(cols):
    assert _abi.lib().dfmi_generate_column(eng.ctx, 1, 42, j, 0, n, 0, 0, C.c_void_p(t.data_ptr()), C.byref(err)) == 0
outs = [torch.empty(n, dtype=torch.float64, device=dev) for _ in range(3)]
schema = Schema([Field(c, DataType.Float64, False) for c in "abc"])
for sel in sels:
    step = FusedStep(eng, schema, cols, n, sel, outs)
    res = {v: [] for v in variants}
    for rnd in range(5):
        for v in variants:
            cfg, mode, nolds = v.split(":")
            os.environ["DFMI_TILE_CFG"], os.environ["DFMI_DEBUG_MODE"], os.environ["DFMI_NO_LDS"] = cfg, mode, nolds
            step()
            if rnd > 0:
                res[v].append(eng.last_timing()[1])
    for v in variants:
        ms = np.median(res[v])
        bpr = 24 + 24 * sel
        print("sel=%.2f cfg:mode:nolds=%s  kernel %.3f ms  %.0f GB/s (min %.3f)" % (sel, v, ms, n * bpr / ms / 1e6, min(res[v])), flush=True)
for k in ("DFMI_TILE_CFG", "DFMI_DEBUG_MODE", "DFMI_NO_LDS"):
    os.environ.pop(k, None)
