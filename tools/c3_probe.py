#!/usr/bin/env python3
"""C3 diagnostics: one 1.25e8-row C3 batch (bench.py's generator), both C3
queries timed under several environment variants in one process (the query
compiler reads its diagnostic knobs per call and keys its cache on them).

usage: tools/c3_probe.py [VAR=VAL[,VAR=VAL...] ...]   (each arg one variant; '-' = defaults)
"""
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
from datafusion_amd.arrow import Field, Schema  # noqa: E402
from datafusion_amd.execution.engine import column_struct, engine  # noqa: E402
from datafusion_amd.execution.expression import compile_scalar_expr  # noqa: E402
from datafusion_amd.logicalplan import BinaryExpr, Column, DataType, Float64, Literal, Operator, Utf8  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = engine(dev)
    words = bench._utf8_dictionary(bench.SEED)
    w17 = words[17].decode()
    dict_bytes = torch.tensor(np.frombuffer(b"".join(words), dtype=np.uint8), device=dev)
    dict_len = torch.tensor([len(w) for w in words], dtype=torch.int64, device=dev)
    dict_off = torch.cumsum(dict_len, 0) - dict_len
    g = torch.Generator(device=dev)
    g.manual_seed(bench.SEED + 1000)
    nb = bench.C3_ROWS // bench.C3_BATCHES
    b, nbytes = bench._c3_batch(dev, g, nb, dict_bytes, dict_off, dict_len)
    torch.cuda.empty_cache()
    schema = Schema([Field("s", DataType.Utf8, False), Field("v", DataType.Float64, True)])
    out_s_off = torch.zeros(nb + 16, dtype=torch.int32, device=dev)
    out_s_data = torch.empty(b[0].values.numel(), dtype=torch.uint8, device=dev)
    out_v = torch.empty(nb, dtype=torch.float64, device=dev)
    L = _abi.lib()
    F = _abi.DFMI_FLAG_EXT_UTF8_COMPARE
    queries = {
        "eq": BinaryExpr(Column(0), Operator.Eq, Literal(Utf8(w17))),
        "lt": BinaryExpr(Column(1), Operator.Lt, Literal(Float64(0.5))),
    }
    if os.environ.get("C3_PROBE_NE"):  # a Utf8-only predicate selecting ~all rows (sub-tile kernel, dense output)
        queries["ne"] = BinaryExpr(Column(0), Operator.NotEq, Literal(Utf8(w17)))
    variants = sys.argv[1:] or ["-"]
    ref = {}
    # the box runs slower for its first ~minute of GPU work (clocks / memory
    # warming: a first variant measured 1.28 ms, the same kernel 1.13 ms later
    # in the same process): the default kernels first, untimed, ~20 s
    warm = ["-"] * int(os.environ.get("C3_PROBE_WARM", "1"))
    for var in warm + variants:
        env = {}
        if var != "-":
            env["DFMI_DIAG"] = "1"  # the library reads its diagnostic knobs only then
            for kv in var.split(","):
                k, v = kv.split("=", 1)
                env[k] = v
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        line = [var]
        for qn, pe in queries.items():
            pred = compile_scalar_expr(None, pe, schema, F)
            projs = [compile_scalar_expr(None, Column(j), schema, F) for j in (0, 1)]
            progs = (C.c_void_p * 2)(*[p.handle.value for p in projs])
            carr = (_abi.dfmi_column * 2)(column_struct(b[0]), column_struct(b[1]))
            cb = _abi.dfmi_batch(2, 0, nb, carr)
            outs = (_abi.dfmi_out_column * 2)()
            outs[0].offsets = out_s_off.data_ptr()
            outs[0].data = out_s_data.data_ptr()
            outs[0].data_capacity = out_s_data.numel()
            outs[1].values = out_v.data_ptr()
            err = _abi.dfmi_error()
            ks = []
            # untimed calls for >= 0.5 s first: a variant's first call compiles
            # its kernel (seconds of an idle GPU), and the clocks need that long
            # to come back -- timed right after a compile, an unchanged kernel
            # measured 12% slower (profiles/r05/c3_probe_clock.log)
            t_end = None
            it = 0
            while True:
                rc = L.dfmi_filter_project(eng.ctx, pred.handle, progs, 2, C.byref(cb), outs, F, C.byref(err))
                if rc != 0:
                    break
                if it == 0:
                    torch.cuda.synchronize()
                    t_end = time.perf_counter() + (20.0 if not getattr(main, "_warmed", False) and warm else 0.5)
                elif time.perf_counter() >= t_end:
                    ks.append(eng.last_timing()[1])
                    if len(ks) >= 12:
                        break
                it += 1
            if rc != 0:  # a shape this query does not take (e.g. rows per thread past its sub-tile bound)
                line.append("%s error: %s" % (qn, err.message.decode()))
                continue
            sel, sb = outs[0].length, outs[0].data_length
            # checksum of the outputs: equal across variants that keep offsets (mode bit 1 does not)
            ck = (int(out_s_off[: sel + 1].to(torch.int64).sum().item()),
                  int(out_s_data[:sb].to(torch.int64).sum().item()),
                  int(out_v[:sel].view(torch.int64).sum().item()))
            if qn not in ref:
                ref[qn] = ck
            alg = nb * (8.125 + 4.0) + nbytes + sel * 12.0 + sb
            ms = float(np.median(ks))
            line.append("%s %.4f ms frac %.3f sel %d %s" % (qn, ms, alg / (ms * 1e-3) / 8e12, sel,
                                                           "same" if ck == ref[qn] else "DIFF"))
        if warm and var == "-" and not getattr(main, "_warmed", False) and len(line) == 3:
            main._warmed = True
            line[0] = "(warm-up)"
        print(" | ".join(line), flush=True)
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


if __name__ == "__main__":
    main()
