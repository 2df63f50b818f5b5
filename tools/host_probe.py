#!/usr/bin/env python3
"""Host-buffer path diagnostics: raw DMA rates of the box (pinned H2D, D2H,
both at once) and per-phase times of dfmi_filter_project_host
(DFMI_HOST_PROFILE=1) on the C2 query over a HOST batch.

usage: tools/host_probe.py [rows]"""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from datafusion_amd import _abi  # noqa: E402
from datafusion_amd.arrow import DataType, Field, Schema  # noqa: E402
from datafusion_amd.execution.engine import engine  # noqa: E402
from datafusion_amd.execution.expression import compile_scalar_expr  # noqa: E402


def dma_rates(dev):
    nb = 1 << 30
    h = torch.empty(nb, dtype=torch.uint8).pin_memory()
    h2 = torch.empty(nb, dtype=torch.uint8).pin_memory()
    d = torch.empty(nb, dtype=torch.uint8, device=dev)
    d2 = torch.empty(nb, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    out = {}
    for name, fn in (("h2d", lambda: d.copy_(h, non_blocking=True)),
                     ("d2h", lambda: h.copy_(d, non_blocking=True))):
        fn()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(5):
            fn()
        torch.cuda.synchronize(dev)
        out[name] = round(5 * nb / (time.perf_counter() - t0) / 1e9, 1)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(5):
        with torch.cuda.stream(s1):
            d.copy_(h, non_blocking=True)
        with torch.cuda.stream(s2):
            h2.copy_(d2, non_blocking=True)
    torch.cuda.synchronize(dev)
    out["both_each"] = round(5 * nb / (time.perf_counter() - t0) / 1e9, 1)
    # host memory rates: memcpy of 1 GB (one thread) and first touch of fresh pages
    a = np.ones(nb, np.uint8)
    b = np.empty(nb, np.uint8)
    b[:] = 0
    t0 = time.perf_counter()
    b[:] = a
    out["host_memcpy_1thread"] = round(nb / (time.perf_counter() - t0) / 1e9, 1)
    t0 = time.perf_counter()
    c = np.empty(nb, np.uint8)
    c[::4096] = 1
    out["first_touch_1thread"] = round(nb / (time.perf_counter() - t0) / 1e9, 1)
    return out


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 100_000_000
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    print("dma GB/s:", dma_rates(dev), flush=True)
    eng = engine(dev)
    from oracle_ffi import gen_unit_f64
    cols = [gen_unit_f64(bench.SEED, j, 0, n) for j in range(3)]
    schema = Schema([Field(c, DataType.Float64, False) for c in "abc"])
    pred_e, proj_e = bench.query(0.5)
    pred = compile_scalar_expr(None, pred_e, schema)
    projs = [compile_scalar_expr(None, e, schema) for e in proj_e]
    progs = (C.c_void_p * 3)(*[p.handle.value for p in projs])
    L = _abi.lib()
    err = _abi.dfmi_error()

    def batch_of(ptrs):
        carr = (_abi.dfmi_column * 3)()
        for i, p in enumerate(ptrs):
            carr[i].type = int(DataType.Float64)
            carr[i].length = n
            carr[i].values = p
        return _abi.dfmi_batch(3, 0, n, carr), carr

    def run(cb, tag):
        for i in range(4):
            res = C.c_void_p()
            t0 = time.perf_counter()
            rc = L.dfmi_filter_project_host(eng.ctx, pred.handle, progs, 3, C.byref(cb), 0, C.byref(res), C.byref(err))
            t1 = time.perf_counter()
            assert rc == 0, err.message
            L.dfmi_host_result_free(res)
            t2 = time.perf_counter()
            print("%s call %d: %.1f ms (free %.1f ms)" % (tag, i, (t1 - t0) * 1e3, (t2 - t1) * 1e3), flush=True)

    os.environ["DFMI_HOST_PROFILE"] = "1"
    cb, keep = batch_of([c.ctypes.data for c in cols])
    run(cb, "pageable")
    ptrs = []
    for c in cols:
        p = C.c_void_p()
        assert L.dfmi_host_alloc(c.nbytes, C.byref(p), C.byref(err)) == 0
        C.memmove(p.value, c.ctypes.data, c.nbytes)
        ptrs.append(p.value)
    cb2, keep2 = batch_of(ptrs)
    run(cb2, "pinned")
    for chunk in ("1048576", "4194304"):
        os.environ["DFMI_HOST_CHUNK_ROWS"] = chunk
        run(cb2, "pinned chunk " + chunk)
    for p in ptrs:
        L.dfmi_host_free(p)


if __name__ == "__main__":
    main()
