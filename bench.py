#!/usr/bin/env python3
"""Benchmark: filter+project over a synthetic 1e9-row Float64 table per GPU
(BASELINE.json configs[1]): SELECT a, b, a*b+c WHERE a > k AND b < m.

One step = one pull of ProjectRelation(FilterRelation(batch)) over one
HBM-resident batch of --rows rows (inputs generated on the device before the
timed region; outputs preallocated). With --gpus N (torchrun) every rank owns
a row-range shard of a global table (weak scaling) and the per-GPU selected
counts are exchanged with one RCCL all_gather per step -- the only collective
the path needs; results stay sharded.

Prints ONE JSON line (rank 0): metric/value (rows/s, whole job), the HBM
roofline of the fused kernel (HIP events on the launch stream), and the CPU
oracle timed on a bounded sample on this host.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from datafusion_amd import _abi  # noqa: E402
from datafusion_amd.arrow import Field, Schema  # noqa: E402
from datafusion_amd.execution.engine import engine  # noqa: E402
from datafusion_amd.execution.expression import compile_scalar_expr  # noqa: E402
from datafusion_amd.logicalplan import BinaryExpr, Column, DataType, Float64, Literal, Operator  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X spec, MI355X_MICROARCH.md "Chip-level parameters"
SEED = 42


def query(sel):
    k, m = 1.0 - sel ** 0.5, sel ** 0.5  # independent uniforms: s = (1-k)*m
    pred = BinaryExpr(BinaryExpr(Column(0), Operator.Gt, Literal(Float64(k))), Operator.And,
                      BinaryExpr(Column(1), Operator.Lt, Literal(Float64(m))))
    projs = [Column(0), Column(1),
             BinaryExpr(BinaryExpr(Column(0), Operator.Multiply, Column(1)), Operator.Plus, Column(2))]
    return pred, projs


class FusedStep:
    """Pre-built C-ABI call: dfmi_filter_project over a resident batch."""

    def __init__(self, eng, schema, cols, n, sel, outs):
        self.eng = eng
        self.pred_e, self.proj_e = query(sel)
        self.pred = compile_scalar_expr(None, self.pred_e, schema)
        self.projs = [compile_scalar_expr(None, e, schema) for e in self.proj_e]
        self.carr = (_abi.dfmi_column * 3)()
        for j, t in enumerate(cols):
            c = self.carr[j]
            c.type = int(DataType.Float64)
            c.length = n
            c.values = t.data_ptr()
        self.cb = _abi.dfmi_batch(3, 0, n, self.carr)
        self.outs = (_abi.dfmi_out_column * 3)()
        for j, t in enumerate(outs):
            self.outs[j].values = t.data_ptr()
        self.progs = (C.c_void_p * 3)(*[p.handle.value for p in self.projs])
        self.err = _abi.dfmi_error()
        self.L = _abi.lib()

    def __call__(self):
        rc = self.L.dfmi_filter_project(self.eng.ctx, self.pred.handle, self.progs, 3, C.byref(self.cb),
                                        self.outs, 0, C.byref(self.err))
        if rc != 0:
            raise RuntimeError(self.err.message.decode())
        return self.outs[0].length


PROFILE_DIR = os.path.join(ROOT, "profiles", "r01")


def pmc_traffic(n, sel):
    """HBM bytes per launch of the query kernel measured by the rocprofv3
    FETCH_SIZE / WRITE_SIZE passes of tools/profile_round.sh on this
    configuration (corrected by tools/traffic.py); None if not profiled."""
    try:
        t = json.load(open(os.path.join(PROFILE_DIR, "traffic.json")))
    except (OSError, ValueError):
        return None
    if t.get("rows") != n or abs(t.get("selectivity", -1) - sel) > 1e-9:
        return None
    return t["traffic_bytes"]


def cpu_baseline(sel, budget_s=12.0):
    """The oracle (reference-faithful restatement, 1 core) on a host sample,
    batch size 1024 as in csv_sql.rs:49. Sample size is calibrated so the
    measurement takes about budget_s seconds."""
    from datafusion_amd.arrow import Array, RecordBatch
    from oracle_ffi import gen_unit_f64, oracle_run_batched
    schema = Schema([Field(c, DataType.Float64, False) for c in "abc"])
    pred, projs = query(sel)

    def run(n):
        b = RecordBatch(schema, [Array.from_numpy(DataType.Float64, gen_unit_f64(SEED, j, 0, n)) for j in range(3)])
        t0 = time.perf_counter()
        rows = oracle_run_batched(schema, b, pred, projs, 1024)
        return time.perf_counter() - t0, rows

    t, _ = run(1 << 20)
    n = int(min(4e8, max(1 << 20, (1 << 20) * budget_s / max(t, 1e-6))))
    n = (n + 1023) // 1024 * 1024
    t, rows = run(n)
    return {"value": n / t, "unit": "rows/s", "cores": 1, "kind": "port",
            "sample": "%d rows (prefix of the seed-%d table), s=%.2f, batch 1024 rows, %d selected, %.1f s"
                      % (n, SEED, sel, rows, t)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=float, default=1e9, help="rows per GPU")
    ap.add_argument("--sel", type=float, default=0.5, help="headline selectivity")
    ap.add_argument("--sweep", default="0.01,0.5,0.99", help="selectivities also reported (first=headline if set)")
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    n = int(args.rows)
    eng = engine(dev)
    st = torch.cuda.current_stream(dev)
    cols = [torch.empty(n, dtype=torch.float64, device=dev) for _ in range(3)]
    err = _abi.dfmi_error()
    for j, t in enumerate(cols):  # shard rows [rank*n, (rank+1)*n) of the global table
        rc = _abi.lib().dfmi_generate_column(eng.ctx, _abi.DFMI_GEN_UNIT_F64, SEED, j, rank * n, n, 0, 0,
                                              C.c_void_p(t.data_ptr()), C.byref(err))
        assert rc == 0, err.message
    outs = [torch.empty(n, dtype=torch.float64, device=dev) for _ in range(3)]
    torch.cuda.synchronize(dev)
    schema = Schema([Field(c, DataType.Float64, False) for c in "abc"])

    sels = [args.sel] + [float(x) for x in args.sweep.split(",") if x and float(x) != args.sel]
    results = {}
    counts_t = torch.zeros(world, dtype=torch.int64, device=dev)
    for sel in sels:
        step = FusedStep(eng, schema, cols, n, sel, outs)
        for _ in range(args.warmup):
            step()
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
        kern_ms = []
        t0 = time.perf_counter()
        selected = 0
        for _ in range(args.steps):
            selected = step()
            kern_ms.append(eng.last_timing()[1])
            if dist:  # exchange per-GPU selected counts (global output offsets)
                mine = torch.tensor([selected], dtype=torch.int64, device=dev)
                dist.all_gather_into_tensor(counts_t, mine)
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        el = time.perf_counter() - t0
        if dist:
            tt = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = tt.item()
        kms = float(np.mean(kern_ms))
        s_real = selected / n
        bytes_per_row = 24.0 + 24.0 * s_real  # a,b,c read; s*(a,b,a*b+c) written
        achieved = n * bytes_per_row / (kms * 1e-3) / 1e9
        results[sel] = dict(el=el, kms=kms, selected=selected, s=s_real, achieved=achieved, bpr=bytes_per_row)

    h = results[args.sel]
    total_rows = n * world * args.steps
    traffic = pmc_traffic(n, args.sel)
    out = {
        "metric": "filter+project rows/s (1e9-row Float64 table per GPU, SELECT a, b, a*b+c WHERE a > k AND b < m)",
        "value": total_rows / h["el"],
        "unit": "rows/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": h["el"] / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (splitmix64 seed 42, generated in HBM)",
        "config": {"workload": "C2: 1e9-row Float64 a,b,c per GPU; s=%.2f" % args.sel, "rows_per_gpu": n,
                   "selectivity": round(h["s"], 4), "parallelism": "row-range shards, RCCL count all_gather"},
        "roofline": {"bound": "hbm", "achieved": round(h["achieved"], 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(h["achieved"] / HBM_PEAK_GBS, 4),
                     "traffic": traffic,
                     "traffic_source": "rocprofv3 FETCH_SIZE/WRITE_SIZE passes, profiles/r01/traffic.json"
                     if traffic else None,
                     "kernel": "dfmi_query (query-compiled filter+project)", "kernel_ms": round(h["kms"], 4),
                     "algorithmic_bytes_per_row": round(h["bpr"], 3)},
        "sweep": {("%.2f" % s): {"rows_per_s": n * world * args.steps / r["el"], "kernel_ms": round(r["kms"], 4),
                                 "hbm_gbs": round(r["achieved"], 1), "frac": round(r["achieved"] / HBM_PEAK_GBS, 4),
                                 "selected": r["selected"]}
                  for s, r in results.items()},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        cb = cpu_baseline(args.sel)
        cb["cpu_model"] = _cpu_model()
        cb["nproc"] = os.cpu_count()
        out["cpu_baseline"] = cb
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


def _cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    main()
