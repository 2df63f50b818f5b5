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
from datafusion_amd.execution.shard import exchange_counts  # noqa: E402
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

    def __init__(self, eng, schema, cols, n, pred_e, proj_e, outs):
        self.eng = eng
        self.pred = compile_scalar_expr(None, pred_e, schema)
        self.projs = [compile_scalar_expr(None, e, schema) for e in proj_e]
        nc, no = len(cols), len(proj_e)
        self.carr = (_abi.dfmi_column * nc)()
        for j, t in enumerate(cols):
            c = self.carr[j]
            c.type = int(schema.fields[j].data_type)
            c.length = n
            c.values = t.data_ptr()
        self.cb = _abi.dfmi_batch(nc, 0, n, self.carr)
        self.outs = (_abi.dfmi_out_column * no)()
        for j, t in enumerate(outs):
            self.outs[j].values = t.data_ptr()
        self.progs = (C.c_void_p * no)(*[p.handle.value for p in self.projs])
        self.no = no
        self.err = _abi.dfmi_error()
        self.L = _abi.lib()

    def __call__(self):
        rc = self.L.dfmi_filter_project(self.eng.ctx, self.pred.handle, self.progs, self.no, C.byref(self.cb),
                                        self.outs, 0, C.byref(self.err))
        if rc != 0:
            raise RuntimeError(self.err.message.decode())
        return self.outs[0].length


PROFILE_TAG = "profiles/r01"
PROFILE_DIR = os.path.join(ROOT, PROFILE_TAG)


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


def timed_steps(step, steps, warmup, dist, eng, dev):
    """W untimed + K timed steps between barrier + synchronize; per step the
    RCCL count exchange of the sharded path. Returns (max-over-ranks wall s,
    mean kernel ms, selected rows of the last step)."""
    for _ in range(warmup):
        step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    kern_ms = []
    t0 = time.perf_counter()
    selected = 0
    for _ in range(steps):
        selected = step()
        kern_ms.append(eng.last_timing()[1])
        if dist:  # per-GPU selected counts -> global output offsets
            exchange_counts([selected])
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = tt.item()
    return el, float(np.mean(kern_ms)), selected


Q6_ROWS = 600_037_902  # TPC-H SF100 lineitem


def q6_line(eng, dev, rank, world, steps, warmup, dist, rows):
    """C4 (BASELINE.json configs[3]): Q6-style predicate over 4 Float64 columns,
    projecting extendedprice*discount (no aggregate: the reference has none).
    Inputs generated on the device with torch (seeded); parity of the query
    is covered in tests/test_gpu_parity.py::test_q6_style_predicate."""
    n = rows
    g = torch.Generator(device=dev)
    g.manual_seed(SEED + rank)
    qty = torch.randint(1, 51, (n,), device=dev, generator=g).to(torch.float64)
    disc = torch.randint(0, 11, (n,), device=dev, generator=g).to(torch.float64) / 100.0
    ship = torch.randint(8036, 10562, (n,), device=dev, generator=g).to(torch.float64)
    price = qty * (900.0 + 1100.0 * torch.rand(n, device=dev, dtype=torch.float64, generator=g))
    cols = [qty, price, disc, ship]
    names = ("l_quantity", "l_extendedprice", "l_discount", "l_shipdate")
    schema = Schema([Field(nm, DataType.Float64, False) for nm in names])

    def ge(c, v):
        return BinaryExpr(Column(c), Operator.GtEq, Literal(Float64(v)))

    def lt(c, v):
        return BinaryExpr(Column(c), Operator.Lt, Literal(Float64(v)))

    pred = BinaryExpr(BinaryExpr(BinaryExpr(BinaryExpr(ge(3, 8766.0), Operator.And, lt(3, 9131.0)), Operator.And,
                                            ge(2, 0.05)), Operator.And,
                                 BinaryExpr(Column(2), Operator.LtEq, Literal(Float64(0.07)))), Operator.And,
                      lt(0, 24.0))
    projs = [BinaryExpr(Column(1), Operator.Multiply, Column(2))]
    outs = [torch.empty(n, dtype=torch.float64, device=dev)]
    torch.cuda.synchronize(dev)
    step = FusedStep(eng, schema, cols, n, pred, projs, outs)
    el, kms, selected = timed_steps(step, steps, warmup, dist, eng, dev)
    s = selected / n
    bpr = 32.0 + 8.0 * s  # 4 Float64 inputs, s * 8 B output
    ach = n * bpr / (kms * 1e-3) / 1e9
    return {"workload": "C4: TPC-H SF100 lineitem Q6-style predicate, 600037902 rows per GPU, "
                        "SELECT l_extendedprice*l_discount (Float64)",
            "rows_per_s": n * world * steps / el, "ms_per_step": el / steps * 1e3, "kernel_ms": round(kms, 4),
            "selectivity": round(s, 5), "selected": selected,
            "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(ach / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_row": round(bpr, 3)}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=float, default=1e9, help="rows per GPU")
    ap.add_argument("--sel", type=float, default=0.5, help="headline selectivity")
    ap.add_argument("--sweep", default="0.01,0.5,0.99", help="selectivities also reported (first=headline if set)")
    ap.add_argument("--extra", default="c4", help="extra config lines (comma list: c4; empty = none)")
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
    for sel in sels:
        step = FusedStep(eng, schema, cols, n, *query(sel), outs)
        el, kms, selected = timed_steps(step, args.steps, args.warmup, dist, eng, dev)
        s_real = selected / n
        bytes_per_row = 24.0 + 24.0 * s_real  # a,b,c read; s*(a,b,a*b+c) written
        achieved = n * bytes_per_row / (kms * 1e-3) / 1e9
        results[sel] = dict(el=el, kms=kms, selected=selected, s=s_real, achieved=achieved, bpr=bytes_per_row)
    del cols, outs, step
    torch.cuda.empty_cache()

    extra = {}
    for name in [x for x in args.extra.split(",") if x]:
        if name == "c4":
            extra["c4"] = q6_line(eng, dev, rank, world, args.steps, args.warmup, dist, Q6_ROWS)
        else:
            raise SystemExit("unknown extra config %r" % name)
        torch.cuda.empty_cache()

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
                     "traffic_source": "rocprofv3 FETCH_SIZE/WRITE_SIZE passes, %s/traffic.json" % PROFILE_TAG
                     if traffic else None,
                     "kernel": "dfmi_query (query-compiled filter+project)", "kernel_ms": round(h["kms"], 4),
                     "algorithmic_bytes_per_row": round(h["bpr"], 3)},
        "sweep": {("%.2f" % s): {"rows_per_s": n * world * args.steps / r["el"], "kernel_ms": round(r["kms"], 4),
                                 "hbm_gbs": round(r["achieved"], 1), "frac": round(r["achieved"] / HBM_PEAK_GBS, 4),
                                 "selected": r["selected"]}
                  for s, r in results.items()},
    }
    if extra:
        out["extra"] = extra
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
