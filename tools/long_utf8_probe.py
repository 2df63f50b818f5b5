#!/usr/bin/env python3
"""Utf8 gather over LONG strings (diagnostics): 1e7 rows of 40-200-byte
strings (every 64-row slice's source span exceeds the 2 KiB stage, so every
selected string goes through the per-lane fallback copy), `SELECT s, v WHERE
v < 0.5`, timed under environment variants in one process, each variant
warmed for 0.5 s after its compile (tools/c3_probe.py).

usage: tools/long_utf8_probe.py [VAR=VAL[,VAR=VAL...] ...]   ('-' = defaults)
"""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from datafusion_amd import _abi  # noqa: E402
from datafusion_amd.arrow import Array, DataType, Field, Schema  # noqa: E402
from datafusion_amd.execution.engine import column_struct, engine  # noqa: E402
from datafusion_amd.execution.expression import compile_scalar_expr  # noqa: E402
from datafusion_amd.logicalplan import BinaryExpr, Column, Float64, Literal, Operator  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = engine(dev)
    n = 10_000_000
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    lens = torch.randint(40, 201, (n,), generator=g, device=dev, dtype=torch.int32)
    offs = torch.zeros(n + 1, dtype=torch.int32, device=dev)
    offs[1:] = torch.cumsum(lens, 0, dtype=torch.int32)
    nbytes = int(offs[-1].item())
    data = torch.randint(32, 127, (nbytes,), generator=g, device=dev, dtype=torch.uint8)
    v = torch.rand(n, generator=g, device=dev, dtype=torch.float64)
    s_arr = Array(DataType.Utf8, n, data, None, offs, 0)
    v_arr = Array(DataType.Float64, n, v)
    schema = Schema([Field("s", DataType.Utf8, False), Field("v", DataType.Float64, False)])
    out_off = torch.zeros(n + 16, dtype=torch.int32, device=dev)
    out_data = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    out_v = torch.empty(n, dtype=torch.float64, device=dev)
    L = _abi.lib()
    pe = BinaryExpr(Column(1), Operator.Lt, Literal(Float64(0.5)))
    ref = None
    for var in ["-"] + (sys.argv[1:] or ["-"]):
        env = {}
        if var != "-":
            env["DFMI_DIAG"] = "1"
            for kv in var.split(","):
                k, val = kv.split("=", 1)
                env[k] = val
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        pred = compile_scalar_expr(None, pe, schema)
        projs = [compile_scalar_expr(None, Column(j), schema) for j in (0, 1)]
        progs = (C.c_void_p * 2)(*[p.handle.value for p in projs])
        carr = (_abi.dfmi_column * 2)(column_struct(s_arr), column_struct(v_arr))
        cb = _abi.dfmi_batch(2, 0, n, carr)
        outs = (_abi.dfmi_out_column * 2)()
        outs[0].offsets = out_off.data_ptr()
        outs[0].data = out_data.data_ptr()
        outs[0].data_capacity = out_data.numel()
        outs[1].values = out_v.data_ptr()
        err = _abi.dfmi_error()
        ks, it, t_end = [], 0, None
        while len(ks) < 12:
            rc = L.dfmi_filter_project(eng.ctx, pred.handle, progs, 2, C.byref(cb), outs, 0, C.byref(err))
            if rc != 0:
                raise SystemExit("%s: %s" % (var, err.message.decode()))
            if it == 0:
                t_end = time.perf_counter() + 0.5
            elif time.perf_counter() >= t_end:
                ks.append(eng.last_timing()[1])
            it += 1
        sel, sb = outs[0].length, outs[0].data_length
        ck = (int(out_off[: sel + 1].to(torch.int64).sum().item()), int(out_data[:sb].to(torch.int64).sum().item()))
        ref = ref or ck
        ms = float(np.median(ks))
        alg = n * 16.0 + nbytes + sel * 12.0 + sb
        print("%s | %.4f ms  %.0f GB/s  sel %d bytes %d %s" % (var, ms, alg / (ms * 1e-3) / 1e9, sel, sb,
                                                             "same" if ck == ref else "DIFF"), flush=True)
        for k, val in old.items():
            if val is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = val


if __name__ == "__main__":
    main()
