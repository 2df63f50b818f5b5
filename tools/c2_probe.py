#!/usr/bin/env python3
"""C2 diagnostics: bench.py's headline batch (1e9 Float64 rows x 3, resident)
and its query at one selectivity, timed under environment variants in one
process -- each variant warmed for 0.5 s after its kernel's compile (an idle
GPU's clocks take that long to come back; profiles/r05/c3_probe_clock.log).

usage: tools/c2_probe.py [--sel S] [--rows N] [VAR=VAL[,VAR=VAL...] ...]   ('-' = defaults)
"""
import argparse
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from datafusion_amd import _abi  # noqa: E402
from datafusion_amd.arrow import DataType, Field, Schema  # noqa: E402
from datafusion_amd.execution.engine import engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sel", type=float, default=0.5)
    ap.add_argument("--rows", type=float, default=1e9)
    ap.add_argument("variants", nargs="*")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = engine(dev)
    n = int(a.rows)
    cols = [torch.empty(n, dtype=torch.float64, device=dev) for _ in range(3)]
    err = _abi.dfmi_error()
    for j, t in enumerate(cols):
        rc = _abi.lib().dfmi_generate_column(eng.ctx, _abi.DFMI_GEN_UNIT_F64, bench.SEED, j, 0, n, 0, 0,
                                              C.c_void_p(t.data_ptr()), C.byref(err))
        assert rc == 0, err.message
    outs = [torch.empty(n, dtype=torch.float64, device=dev) for _ in range(3)]
    schema = Schema([Field(c, DataType.Float64, False) for c in "abc"])
    ref = None
    first = True
    for var in ["-"] + (a.variants or ["-"]):
        env = {}
        if var != "-":
            env["DFMI_DIAG"] = "1"
            for kv in var.split(","):
                k, v = kv.split("=", 1)
                env[k] = v
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        step = bench.FusedStep(eng, schema, cols, n, *bench.query(a.sel), outs)
        ks, it = [], 0
        t_end = None
        while len(ks) < 12:
            sel = step()
            if it == 0:
                t_end = time.perf_counter() + (15.0 if first else 0.5)
            elif time.perf_counter() >= t_end:
                ks.append(eng.last_timing()[1])
            it += 1
        ck = int(outs[2][:sel].view(torch.int64).sum().item())
        ref = ref if ref is not None else ck
        ms = float(np.median(ks))
        bpr = 24.0 + 24.0 * sel / n
        print("%s | %.4f ms  formula %.3f  sel %d %s  [%s]" % ("(warm-up)" if first else var, ms,
                                                             n * bpr / (ms * 1e-3) / 8e12, sel,
                                                             "same" if ck == ref else "DIFF", bench.kernel_name(eng)),
              flush=True)
        first = False
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


if __name__ == "__main__":
    main()
