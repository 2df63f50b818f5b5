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
import socket
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
from datafusion_amd.logicalplan import BinaryExpr, Column, DataType, Float64, Int64, Literal, Operator  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X spec, MI355X_MICROARCH.md "Chip-level parameters"
COPY_CEILING_GBS = 6290.0  # measured read+write copy ceiling, MI355X_MICROARCH.md:36
SEED = 42
# DFMI_BENCH_BACKEND=gloo: rehearsal of the --gpus N path with N ranks sharing
# the visible GPUs (rank -> GPU local_rank % count) and the collectives over
# gloo on host tensors. Timings of such a run are not a scaling measurement.
BACKEND = os.environ.get("DFMI_BENCH_BACKEND", "nccl")


def coll_device(dev):
    """Where collective tensors live: the GPU under RCCL, the host under gloo."""
    return dev if BACKEND == "nccl" else torch.device("cpu")


def query(sel):
    k, m = 1.0 - sel ** 0.5, sel ** 0.5  # independent uniforms: s = (1-k)*m
    pred = BinaryExpr(BinaryExpr(Column(0), Operator.Gt, Literal(Float64(k))), Operator.And,
                      BinaryExpr(Column(1), Operator.Lt, Literal(Float64(m))))
    projs = [Column(0), Column(1),
             BinaryExpr(BinaryExpr(Column(0), Operator.Multiply, Column(1)), Operator.Plus, Column(2))]
    return pred, projs


class FusedStep:
    """Pre-built C-ABI call: dfmi_filter_project over a resident batch -- or,
    with a ShardComm, dfmi_shard_filter_project: this rank's pass plus the
    RCCL all_gather of placement records (the path a Rust caller of
    Relation::next takes on each GPU, relation.rs:27-32)."""

    def __init__(self, eng, schema, cols, n, pred_e, proj_e, outs, comm=None, flags=0):
        self.eng = eng
        self.flags = flags
        self.pred = compile_scalar_expr(None, pred_e, schema, flags)
        self.projs = [compile_scalar_expr(None, e, schema, flags) for e in proj_e]
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
        self.comm = comm
        self.place = _abi.dfmi_shard_placement()

    def __call__(self):
        if self.comm is None:
            rc = self.L.dfmi_filter_project(self.eng.ctx, self.pred.handle, self.progs, self.no, C.byref(self.cb),
                                            self.outs, self.flags, C.byref(self.err))
        else:
            rc = self.L.dfmi_shard_filter_project(self.eng.ctx, self.comm.handle, self.pred.handle, self.progs,
                                                  self.no, C.byref(self.cb), self.outs, self.flags, C.byref(self.place),
                                                  C.byref(self.err))
            self.comm.placement, self.comm.outputs = self.place, self.outs
        if rc != 0:
            raise RuntimeError(self.err.message.decode())
        return self.outs[0].length


PROFILE_TAG = "profiles/r06"
PROFILE_DIR = os.path.join(ROOT, PROFILE_TAG)


def kernel_name(eng):
    """The query kernel the context launched last (dfmi_<kind>_<hash>, as rocprofv3 names it)."""
    return _abi.lib().dfmi_last_kernel_name(eng.ctx).decode()


def profiled(kernel, run="main"):
    """The committed rocprofv3 record of `kernel` (tools/profile_r04.sh: kernel
    trace + separate FETCH_SIZE / WRITE_SIZE passes of the same bench command,
    tools/traffic.py): the entry of its largest grid in PROFILE_DIR/<run>, or None."""
    try:
        t = json.load(open(os.path.join(PROFILE_DIR, run, "traffic.json")))
    except (OSError, ValueError):
        return None
    hits = [e for e in t["kernels"] if e["kernel"] == kernel]
    return max(hits, key=lambda e: e["grid"]) if hits else None


LINE_BYTES = 128  # one memory request per touched 128-B line (profiles/r06/calib_masked/summary.txt)


def lines_touched(mask, rows_per_line=LINE_BYTES // 8):
    """128-B lines of an 8-B column (256-B aligned, row 0 at a line start)
    that hold at least one selected row: what a lane-masked load of that
    column fetches (tools/membw_masked.hip: FETCH_SIZE x 2 = 128 B x these
    lines, exactly)."""
    n = mask.numel()
    full = n // rows_per_line * rows_per_line
    c = int(mask[:full].view(-1, rows_per_line).any(1).sum().item())
    if full < n:
        c += int(mask[full:].any().item())
    return c


def moved_bytes(n, streamed_bpr, masked_cols, mask, written):
    """The HBM bytes a filter kernel over n rows must move, counted from its
    real selection mask: every streamed (predicate) column once, each
    lane-masked 8-B column's 128-B lines that hold a selected row once, and
    the writes. Re-reads (the sub-tile output pass re-loads the predicate's
    columns for the selected rows) are counted as cache hits, i.e. not at
    all: a lower bound, so the credited fraction is one too."""
    return n * streamed_bpr + masked_cols * LINE_BYTES * lines_touched(mask) + written


def roofline(kernel, alg_bytes, kms, rows, launches=1, run="main", moved=None):
    """roofline object of one bench line. `frac` is the fraction the hardware
    backs: the lowest of the FORMULA fraction (SURVEY §8(d)'s algorithmic bytes
    per launch over the kernel's average HIP-event time on the launch stream,
    `formula_frac`), the MOVED fraction (`moved` bytes per launch, counted
    from the selection mask by moved_bytes(): what a kernel that skips the
    unselected lines of its masked columns has to move at the least,
    `moved_frac`) and the PMC fraction (FETCH_SIZE x 2 + WRITE_SIZE of the
    committed profile of the same kernel -- memory-side requests, calibrated
    for streaming and lane-masked 8-B loads, Infinity-Cache hits included --
    over this run's time, `traffic_frac`). Without a PMC record, `frac` never
    exceeds the measured copy ceiling (6.29 of 8 TB/s, MI355X_MICROARCH.md).
    `rocprof` names the committed profile (its box, its average time and
    fraction); the line's own box is the bench JSON's `box`."""
    ach = alg_bytes / (kms * 1e-3) / 1e9
    ffrac = ach / HBM_PEAK_GBS
    r = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": None, "formula_frac": round(ffrac, 4), "kernel": kernel, "kernel_ms": round(kms, 4),
         "launches_per_step": launches, "algorithmic_bytes_per_row": round(alg_bytes * launches / rows, 3),
         "traffic": None}
    p = profiled(kernel, run)
    cands = []  # (fraction, basis): the credited one is the lowest
    if moved is not None:
        mgbs = moved / (kms * 1e-3) / 1e9
        r["moved_bytes_per_row"] = round(moved * launches / rows, 3)
        r["moved_gbs"] = round(mgbs, 1)
        r["moved_frac"] = round(mgbs / HBM_PEAK_GBS, 4)
        cands.append((r["moved_frac"], "moved bytes (selection mask: streamed columns + touched 128-B lines of "
                                       "masked columns + writes)"))
    pmc = False
    if p:
        per_launch_alg = alg_bytes  # alg_bytes and kms are per launch
        avg_ms = p["avg_ns"] * 1e-6
        r["rocprof"] = {"source": "%s/%s/traffic.json" % (PROFILE_TAG, run), "box": p.get("box"),
                        "avg_ms": round(avg_ms, 4), "launches": p["launches"],
                        "formula_frac": round(per_launch_alg / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        "vgpr": p["vgpr"], "sgpr": p["sgpr"], "scratch": p["scratch"], "lds": p["lds"]}
        if "traffic_bytes" in p:
            pmc = True
            r["traffic"] = round(p["traffic_bytes"])
            r["traffic_bytes_per_row"] = round(p["traffic_bytes"] * launches / rows, 3)
            # the profile's bytes per launch over THIS run's kernel time
            tgbs = p["traffic_bytes"] / (kms * 1e-3) / 1e9
            r["traffic_gbs"] = round(tgbs, 1)
            r["traffic_frac"] = round(tgbs / HBM_PEAK_GBS, 4)
            r["rocprof"]["traffic_frac"] = round(p["traffic_bytes"] / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
            cands.append((r["traffic_frac"], "PMC request bytes (FETCH_SIZE x 2 + WRITE_SIZE of the committed profile)"))
    if pmc or moved is not None or ffrac <= COPY_CEILING_GBS / HBM_PEAK_GBS:
        cands.append((ffrac, "formula (SURVEY 8(d) algorithmic bytes)"))
    else:
        cands.append((COPY_CEILING_GBS / HBM_PEAK_GBS, "formula, capped at the copy ceiling (no PMC record)"))
    frac, basis = min(cands)
    r["frac"] = round(frac, 4)
    r["frac_basis"] = basis
    r["formula_exceeds_ceiling"] = ach > COPY_CEILING_GBS
    return r


def cpu_baseline(sel, budget_s=12.0):
    """The oracle (reference-faithful restatement, 1 core) on a host sample,
    batch size 1024 as in csv_sql.rs:49. Sample size is calibrated so the
    measurement takes about budget_s seconds."""
    from datafusion_amd.arrow import Array, RecordBatch
    from oracle_ffi import gen_unit_f64, oracle_run_batched
    schema = Schema([Field(c, DataType.Float64, False) for c in "abc"])
    pred, projs = query(sel)

    def run(n, batch=1024):
        b = RecordBatch(schema, [Array.from_numpy(DataType.Float64, gen_unit_f64(SEED, j, 0, n)) for j in range(3)])
        t0 = time.perf_counter()
        rows = oracle_run_batched(schema, b, pred, projs, batch)
        return time.perf_counter() - t0, rows

    t, _ = run(1 << 20)
    n = int(min(4e8, max(1 << 20, (1 << 20) * budget_s / max(t, 1e-6))))
    n = (n + 1023) // 1024 * 1024
    t, rows = run(n)
    # BASELINE.md's second batch size: 1,048,576-row batches over a 1/4 sample
    nb = max(1 << 20, (n // 4) >> 20 << 20)
    tb, rows_b = run(nb, 1 << 20)
    return {"value": n / t, "unit": "rows/s", "cores": 1, "kind": "port",
            "sample": "%d rows (prefix of the seed-%d table), s=%.2f, batch 1024 rows, %d selected, %.1f s"
                      % (n, SEED, sel, rows, t),
            "batch_1048576": {"value": nb / tb, "unit": "rows/s",
                              "sample": "%d rows, batch 1048576 rows, %d selected, %.1f s" % (nb, rows_b, tb)}}


def timed_steps(step, steps, warmup, dist, eng, dev, py_exchange=True):
    """W untimed + K timed steps between barrier + synchronize; per step the
    count exchange of the sharded path (inside the step on the C-ABI path,
    else torch.distributed's all_gather here). Returns (max-over-ranks wall s,
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
        t = eng.last_timing()  # (None where the step's last call times no kernel)
        kern_ms.append(t[1] if t else 0.0)
        if dist and py_exchange:  # per-GPU selected counts -> global output offsets
            exchange_counts([selected])
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([el], dtype=torch.float64, device=coll_device(dev))
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = tt.item()
    return el, float(np.mean(kern_ms)), selected


def abi_comm(eng, dist, rank, world, dev):
    """The C-ABI RCCL communicator (dfmi_shard_unique_id on rank 0, handed to
    every rank out of band -- here a torch.distributed broadcast -- then
    dfmi_shard_comm_init), as a Rust caller with one thread per GPU sets it up."""
    from datafusion_amd.execution.engine import ShardComm
    # RCCL prints its version banner on stdout at init: keep stdout for the
    # one JSON line (fd-level, the banner comes from C)
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        uid = ShardComm.unique_id() if rank == 0 else bytes(_abi.DFMI_SHARD_ID_BYTES)
        if dist:
            t = torch.tensor(list(uid), dtype=torch.uint8, device=coll_device(dev))
            dist.broadcast(t, 0)
            uid = bytes(t.cpu().tolist())
        return ShardComm(eng, world, rank, uid)
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def _checksum(t):
    """Wrapping int64 sum of a buffer's 8-byte words (order-independent check)."""
    return int(t.view(torch.int64).sum().item()) if t.numel() else 0


def gather_line(eng, comm, schema, cols, n, sel, dist, rank, world, dev, root=0):
    """SURVEY §8(e) / C5's "result gather over xGMI": one dfmi_shard_gather_to_root
    of the C2 outputs (a, b, a*b+c at s=sel) of every rank onto `root`,
    grouped ncclSend/ncclRecv posted at once, timed between barriers (max over
    ranks). Reported apart from `value`: the leg is bound by the root's xGMI
    ingress. Check: every rank's per-column checksum equals the checksum of
    its segment of the gathered columns on the root."""
    outs = [torch.empty(n, dtype=torch.float64, device=dev) for _ in range(3)]
    step = FusedStep(eng, schema, cols, n, *query(sel), outs, comm=comm)
    local_rows = step()
    place = comm.placement
    total = place.total_rows
    need = 3 * total * 8
    free = torch.cuda.mem_get_info(dev)[0] if rank == root else 0
    ok = torch.tensor([1 if (rank != root or need + (4 << 30) < free) else 0], device=coll_device(dev))
    if dist:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if not ok.item():
        return {"skipped": "root lacks %.1f GB of free HBM for the gathered columns" % (need / 1e9)}
    routs = (_abi.dfmi_out_column * 3)()
    keep = []
    if rank == root:
        for j in range(3):
            t = torch.empty(max(total, 1), dtype=torch.float64, device=dev)
            keep.append(t)
            routs[j].values = t.data_ptr()
    err = _abi.dfmi_error()
    L = _abi.lib()
    times = []
    for it in range(3):
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        rc = L.dfmi_shard_gather_to_root(eng.ctx, comm.handle, comm.outputs, routs, root, C.byref(err))
        if rc != 0:
            raise RuntimeError(err.message.decode())
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        el = time.perf_counter() - t0
        if dist:
            tt = torch.tensor([el], dtype=torch.float64, device=coll_device(dev))
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = tt.item()
        times.append(el)
    # checksums: each rank's outputs vs its segment on the root
    mine = torch.tensor([_checksum(o[:local_rows]) for o in outs] + [local_rows], dtype=torch.int64,
                        device=coll_device(dev))
    allc = [torch.empty_like(mine) for _ in range(world)] if dist else [mine]
    if dist:
        dist.all_gather(allc, mine)
    checks = None
    if rank == root:
        checks, r0 = True, 0
        for r in range(world):
            cs = allc[r].cpu().tolist()
            rows = cs[3]
            for j in range(3):
                checks = checks and _checksum(keep[j][r0:r0 + rows]) == cs[j]
            r0 += rows
        checks = checks and r0 == total
    el = min(times)
    moved = (total - (local_rows if rank == root else 0)) * 24 if world > 1 else total * 24
    del keep, outs, step
    return {"workload": "gather C2 outputs (3 x Float64, s=%.2f) of %d rank(s) to rank %d" % (sel, world, root),
            "rows": total, "bytes": total * 24, "ms": round(el * 1e3, 3),
            "transfer": "xGMI (RCCL grouped send/recv)" if world > 1 else "local HBM copy (one rank: no xGMI)",
            "bytes_into_root": moved, "gbs_into_root": round(moved / el / 1e9, 1),
            "checksums_match": checks, "note": "not in value: results stay sharded by default (DESIGN.md §8)"}


def batches_line(eng, schema, cols, sel, dev):
    """Per-call cost at the reference's batch sizes (csv_sql.rs:49 reads 1024-row
    batches): the C2 query over the first 1,024 and 1,048,576 rows of the
    resident table, one synchronous dfmi_filter_project per batch; plus the
    first-call hipRTC compile of a query shape not seen before."""
    out = {}
    for m, calls in ((1024, 4000), (1 << 20, 400)):
        outs = [torch.empty(m, dtype=torch.float64, device=dev) for _ in range(3)]
        step = FusedStep(eng, schema, cols, m, *query(sel), outs)
        for _ in range(50):
            step()
        torch.cuda.synchronize(dev)
        _abi.lib().dfmi_context_set_timing(eng.ctx, 0)  # production setting: no profiling events
        t0 = time.perf_counter()
        for _ in range(calls):
            step()
        el = time.perf_counter() - t0
        _abi.lib().dfmi_context_set_timing(eng.ctx, 1)
        torch.cuda.synchronize(dev)
        kern = 0.0  # device time from HIP events, in a loop of its own (reading them waits)
        for _ in range(200):
            step()
            kern += eng.last_timing()[1]
        us = el / calls * 1e6
        out["%d_rows" % m] = {"kernel": kernel_name(eng), "us_per_batch": round(us, 2),
                              "kernel_us": round(kern / 200 * 1e3, 2),
                              "host_overhead_us": round(us - kern / 200 * 1e3, 2), "calls": calls,
                              "rows_per_s": m / (us * 1e-6)}
        if m == 1024:
            # the workspace-clearing cliff: a warm 1024-row call
            # right after a full-table launch zeroes that launch's look-back
            # status words (tens of MB), spread over all of its own blocks
            n = cols[0].numel()
            big_outs = [torch.empty(n, dtype=torch.float64, device=dev) for _ in range(3)]
            big = FusedStep(eng, schema, cols, n, *query(sel), big_outs)  # the headline's own query
            big()
            _abi.lib().dfmi_context_set_timing(eng.ctx, 0)
            after = []
            for _ in range(3):
                big()
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                step()
                after.append((time.perf_counter() - t0) * 1e6)
            _abi.lib().dfmi_context_set_timing(eng.ctx, 1)
            out["1024_call_after_full_table_us"] = round(min(after), 1)
            del big, big_outs
            torch.cuda.empty_cache()
    out["1024_rows_x256_coalesced"] = coalesced_batches(eng, schema, cols, sel, dev, 1024, 256)
    out["1024_rows_host"] = host_small_batches(eng, schema, sel, 1024)
    out["1024_rows_host_x256_coalesced"] = host_coalesced_batches(eng, schema, sel, 1024, 256)
    out["relation_1024_host"] = relation_host_line(sel)
    # a new query shape: generate + hipRTC compile on the first call, cached after
    pred, projs = query(sel)
    pred = BinaryExpr(pred, Operator.And, BinaryExpr(Column(2), Operator.GtEq, Literal(Float64(0.0))))
    outs = [torch.empty(1024, dtype=torch.float64, device=dev) for _ in range(3)]
    step = FusedStep(eng, schema, cols, 1024, pred, projs, outs)
    t0 = time.perf_counter()
    step()
    first_ms = (time.perf_counter() - t0) * 1e3
    cm = C.c_double()
    _abi.lib().dfmi_last_compile_ms(eng.ctx, C.byref(cm))
    t0 = time.perf_counter()
    step()
    out["first_call"] = {"compile_ms": round(cm.value, 1), "first_call_ms": round(first_ms, 1),
                         "second_call_ms": round((time.perf_counter() - t0) * 1e3, 3)}
    return out


def coalesced_batches(eng, schema, cols, sel, dev, m, nb, calls=300):
    """dfmi_filter_project_batches: `nb` consecutive m-row batches of the
    resident table (each with its own buffers and outputs, one output batch
    per input batch) in one launch per call. Gate: every batch's outputs
    equal dfmi_filter_project's on that batch alone."""
    pred_e, proj_e = query(sel)
    pred = compile_scalar_expr(None, pred_e, schema)
    projs = [compile_scalar_expr(None, e, schema) for e in proj_e]
    progs = (C.c_void_p * 3)(*[p.handle.value for p in projs])
    carrs = []
    cb = (_abi.dfmi_batch * nb)()
    for i in range(nb):
        carr = (_abi.dfmi_column * 3)()
        for j, t in enumerate(cols):
            carr[j].type = int(DataType.Float64)
            carr[j].length = m
            carr[j].values = t.data_ptr() + i * m * 8
        carrs.append(carr)
        cb[i].num_columns, cb[i].num_rows, cb[i].columns = 3, m, carr
    obuf = torch.empty((nb, 3, m), dtype=torch.float64, device=dev)
    outs = (_abi.dfmi_out_column * (nb * 3))()
    for i in range(nb):
        for j in range(3):
            outs[i * 3 + j].values = obuf[i, j].data_ptr()
    L = _abi.lib()
    err = _abi.dfmi_error()
    failed = C.c_int32()

    def call():
        rc = L.dfmi_filter_project_batches(eng.ctx, pred.handle, progs, 3, cb, nb, outs, 0, C.byref(failed),
                                           C.byref(err))
        if rc != 0:
            raise RuntimeError(err.message.decode())
    for _ in range(20):
        call()
    L.dfmi_context_set_timing(eng.ctx, 0)
    t0 = time.perf_counter()
    for _ in range(calls):
        call()
    el = (time.perf_counter() - t0) / calls
    L.dfmi_context_set_timing(eng.ctx, 1)
    kern = 0.0
    for _ in range(50):
        call()
        kern += eng.last_timing()[1]
    kname = kernel_name(eng)
    # gate against the single-batch entry point, batch by batch
    lens = [outs[i * 3].length for i in range(nb)]
    ok = True
    single = [torch.empty(m, dtype=torch.float64, device=dev) for _ in range(3)]
    for i in range(0, nb, max(1, nb // 16)):
        st = FusedStep(eng, schema, [c[i * m:(i + 1) * m] for c in cols], m, pred_e, proj_e, single)
        k = st()
        ok = ok and k == lens[i] and all(torch.equal(single[j][:k].view(torch.int64), obuf[i, j, :k].view(torch.int64))
                                         for j in range(3))
    return {"kernel": kname, "batches_per_call": nb, "rows_per_batch": m, "us_per_call": round(el * 1e6, 2),
            "us_per_batch": round(el * 1e6 / nb, 3), "kernel_us_per_call": round(kern / 50 * 1e3, 2),
            "rows_per_s": nb * m / el, "selected_last_call": int(sum(lens)),
            "matches_single_batch_calls": bool(ok)}


def host_small_batches(eng, schema, sel, m, calls=2000):
    """dfmi_filter_project_host (what the Rust binding calls with arrow 0.12
    host buffers) on one m-row host batch per call."""
    from oracle_ffi import gen_unit_f64
    host = [gen_unit_f64(SEED, j, 0, m) for j in range(3)]
    pred_e, proj_e = query(sel)
    pred = compile_scalar_expr(None, pred_e, schema)
    projs = [compile_scalar_expr(None, e, schema) for e in proj_e]
    progs = (C.c_void_p * 3)(*[p.handle.value for p in projs])
    carr = (_abi.dfmi_column * 3)()
    for j, h in enumerate(host):
        carr[j].type = int(DataType.Float64)
        carr[j].length = m
        carr[j].values = h.ctypes.data
    cb = _abi.dfmi_batch(3, 0, m, carr)
    L = _abi.lib()
    err = _abi.dfmi_error()

    def call():
        res = C.c_void_p()
        rc = L.dfmi_filter_project_host(eng.ctx, pred.handle, progs, 3, C.byref(cb), 0, C.byref(res), C.byref(err))
        if rc != 0:
            raise RuntimeError(err.message.decode())
        L.dfmi_host_result_free(res)
    for _ in range(50):
        call()
    L.dfmi_context_set_timing(eng.ctx, 0)
    t0 = time.perf_counter()
    for _ in range(calls):
        call()
    el = (time.perf_counter() - t0) / calls
    L.dfmi_context_set_timing(eng.ctx, 1)
    return {"us_per_batch": round(el * 1e6, 2), "rows_per_s": m / el, "calls": calls,
            "note": "host buffers in, host results out (PCIe both ways), one synchronous call per batch"}


def host_coalesced_batches(eng, schema, sel, m, nb, calls=200):
    """dfmi_filter_project_host_batches: nb consecutive m-row HOST batches
    (pageable numpy buffers, as csv::Reader hands them out) per call -- packed
    into pinned memory, one H2D, one launch, one D2H; one output batch per
    input batch. Checked against one dfmi_filter_project_host call per batch."""
    from oracle_ffi import gen_unit_f64
    host = [gen_unit_f64(SEED, j, 0, m * nb) for j in range(3)]
    pred_e, proj_e = query(sel)
    pred = compile_scalar_expr(None, pred_e, schema)
    projs = [compile_scalar_expr(None, e, schema) for e in proj_e]
    progs = (C.c_void_p * 3)(*[p.handle.value for p in projs])
    keep = []
    barr = (_abi.dfmi_batch * nb)()
    for b in range(nb):
        carr = (_abi.dfmi_column * 3)()
        for j, h in enumerate(host):
            carr[j].type = int(DataType.Float64)
            carr[j].length = m
            carr[j].values = h.ctypes.data + b * m * 8
        keep.append(carr)
        barr[b] = _abi.dfmi_batch(3, 0, m, carr)
    L = _abi.lib()
    err = _abi.dfmi_error()
    failed = C.c_int32()

    def call(check=False):
        res = C.c_void_p()
        rc = L.dfmi_filter_project_host_batches(eng.ctx, pred.handle, progs, 3, barr, nb, 0, C.byref(res),
                                                C.byref(failed), C.byref(err))
        if rc != 0:
            raise RuntimeError(err.message.decode())
        ok = True
        if check:  # batch by batch against the single-batch host entry point
            for b in (0, nb // 2, nb - 1):
                one = C.c_void_p()
                rc = L.dfmi_filter_project_host(eng.ctx, pred.handle, progs, 3, C.byref(barr[b]), 0, C.byref(one),
                                                C.byref(err))
                if rc != 0:
                    raise RuntimeError(err.message.decode())
                for o in range(3):
                    va, vb = _abi.dfmi_column(), _abi.dfmi_column()
                    L.dfmi_host_result_column(res, b * 3 + o, C.byref(va))
                    L.dfmi_host_result_column(one, o, C.byref(vb))
                    ok = ok and va.length == vb.length and C.string_at(va.values, va.length * 8) == \
                        C.string_at(vb.values, vb.length * 8)
                L.dfmi_host_result_free(one)
        L.dfmi_host_result_free(res)
        return ok
    same = call(check=True)
    for _ in range(20):
        call()
    L.dfmi_context_set_timing(eng.ctx, 0)
    t0 = time.perf_counter()
    for _ in range(calls):
        call()
    el = (time.perf_counter() - t0) / calls
    L.dfmi_context_set_timing(eng.ctx, 1)
    return {"batches_per_call": nb, "rows_per_batch": m, "us_per_call": round(el * 1e6, 2),
            "us_per_batch": round(el * 1e6 / nb, 3), "rows_per_s": m * nb / el, "calls": calls,
            "matches_single_batch_calls": same,
            "note": "pageable host buffers in, pinned host results out (PCIe both ways)"}


def relation_host_line(sel, m=1024, nbatches=4096, passes=5, coalesce=256):
    """The drop-in end to end at the reference's own batch size: ctx.sql of
    the C2 query over `nbatches` m-row HOST batches (csv_sql.rs:49 reads
    1024-row batches from csv::Reader into host memory) pulled through the
    relations one next() at a time (csv_sql.rs:60-62, relation.rs:27-32) --
    ProjectRelation(FilterRelation(DataSourceRelation)) with read-ahead
    `coalesce` (dfmi_filter_project_host_batches per group). Each pass gets
    freshly built batch objects (pageable numpy buffers, built outside the
    timed loop, as the CPU baseline's input is); the loop counts the rows of
    every output batch ("pull"), and a second loop also builds every output
    column's Array ("pull + columns"). Gate: every output batch of one pass
    equals the oracle's for that batch, bit for bit."""
    from datafusion_amd.arrow import Array, RecordBatch
    from datafusion_amd.execution import ExecutionContext, MemoryDataSource
    from oracle_ffi import gen_unit_f64, oracle_filter_project
    n = m * nbatches
    host = [torch.from_numpy(gen_unit_f64(SEED, j, 0, n).view(np.uint8)) for j in range(3)]
    schema = Schema([Field(c, DataType.Float64, False) for c in "abc"])
    k, mm = 1.0 - sel ** 0.5, sel ** 0.5
    sql = "SELECT a, b, a * b + c FROM t WHERE a > %r AND b < %r" % (k, mm)

    def batches():
        return [RecordBatch(schema, [Array(DataType.Float64, m, t[i * m * 8:(i + 1) * m * 8]) for t in host])
                for i in range(nbatches)]

    def rel(bs, co=coalesce):
        ctx = ExecutionContext(coalesce=co)
        ctx.register_datasource("t", MemoryDataSource(schema, bs))
        return ctx.sql(sql)

    def run(touch, co=coalesce):
        best = None
        for p in range(passes + 1):
            r = rel(batches(), co)
            rows = 0
            t0 = time.perf_counter()
            while True:
                b = r.next()
                if b is None:
                    break
                rows += b.columns[-1].length if touch else b.num_rows()
            el = time.perf_counter() - t0
            if p and (best is None or el < best):  # pass 0 warms the query shape up
                best = el
        return {"us_per_batch": round(best / nbatches * 1e6, 3), "rows_per_s": n / best, "selected": rows}

    pc = run(True)
    out = {"workload": "ctx.sql(%r) over %d HOST batches of %d rows (MemoryDataSource), read-ahead %d"
                       % (sql, nbatches, m, coalesce),
           # the relation figure: every pulled batch's output Arrays built
           # (what the reference's next() returns, projection.rs:59-60)
           "rows_per_s": pc["rows_per_s"], "us_per_batch": pc["us_per_batch"],
           "pull_and_columns": pc, "pull": run(False),
           "one_call_per_pull": run(False, co=1) if nbatches <= 4096 else None,
           "rust_binding_path": rust_binding_path(host, schema, sql, sel, m, nbatches, coalesce)}
    # gate: one pass, every batch against the oracle (outside the timed loops)
    pred_e, proj_e = query(sel)
    bs = batches()
    got = list(rel(bs))
    ok = len(got) == nbatches
    for i in range(0, nbatches, 7):
        ref = oracle_filter_project(schema, bs[i], pred_e, proj_e, 0)
        for d, (_, r) in zip(got[i].columns, ref):
            ok = ok and d.length == r.length and np.array_equal(np.asarray(d.numpy_values()).view(np.uint8),
                                                                np.asarray(r.numpy_values()).view(np.uint8))
    out["parity_gate"] = {"batches_checked": len(range(0, nbatches, 7)), "bit_identical_to_oracle": bool(ok)}
    out["rust_binding_path"]["selected_matches_relation"] = out["rust_binding_path"]["selected"] == \
        sum(b.num_rows() for b in got)
    return out


def rust_binding_path(host, schema, sql, sel, m, nbatches, group, passes=5):
    """What INTEGRATION.md's Rust ProjectRelation::run_group does per group of
    `group` 1024-row host batches, on one thread without read-ahead overlap:
    the dfmi_batch structs over the batches' (pageable) buffers, the block
    size (dfmi_host_batches_output_bytes), a FRESH pageable block per group
    (arrow's allocator: malloc, first-touch page faults included), and
    dfmi_filter_project_host_batches_into -- whose selected bytes the library
    copies from its pinned staging into the block. The output arrays are
    slices of that block (Buffer::slice), so nothing is copied after the call.
    Checked: the group outputs equal the relation's for the same batches."""
    from datafusion_amd.arrow import Array, RecordBatch
    from datafusion_amd.execution.engine import _OUT_DTYPE, host_batch_structs
    eng = engine()
    pred_e, proj_e = query(sel)
    pred = compile_scalar_expr(None, pred_e, schema)
    projs = [compile_scalar_expr(None, e, schema) for e in proj_e]
    progs = (C.c_void_p * 3)(*[p.handle.value for p in projs])
    L = _abi.lib()
    err = _abi.dfmi_error()
    failed = C.c_int32()
    size = C.c_size_t()

    def batches():
        return [RecordBatch(schema, [Array(DataType.Float64, m, t[i * m * 8:(i + 1) * m * 8]) for t in host])
                for i in range(nbatches)]
    best, sel_rows = None, 0
    for p in range(passes + 1):
        bs = batches()
        rows = 0
        t0 = time.perf_counter()
        for g in range(0, nbatches, group):
            barr, keep = host_batch_structs(bs[g:g + group], 3)
            nb = len(barr)
            rc = L.dfmi_host_batches_output_bytes(pred.handle, progs, 3, C.cast(barr, C.c_void_p), nb, 0,
                                                  C.byref(size), C.byref(err))
            block = np.empty(size.value + 64, np.uint8)  # pageable, fresh each group
            a = (-block.ctypes.data) % 64
            outs = np.empty(nb * 3, _OUT_DTYPE)
            rc = rc or L.dfmi_filter_project_host_batches_into(eng.ctx, pred.handle, progs, 3, C.cast(barr, C.c_void_p),
                                                               nb, 0, block.ctypes.data + a, size.value,
                                                               outs.ctypes.data, C.byref(failed), C.byref(err))
            if rc != 0:
                raise RuntimeError(err.message.decode())
            rows += int(outs["length"][2::3].sum())
        el = time.perf_counter() - t0
        if p and (best is None or el < best):
            best = el
        sel_rows = rows
    return {"us_per_batch": round(best / nbatches * 1e6, 3), "rows_per_s": nbatches * m / best, "selected": sel_rows,
            "note": "one thread, no read-ahead overlap; pageable caller-owned block per group (one library copy of "
                    "the selected bytes into it)"}


def prefix_gate(eng, schema, dev_cols, m, pred_e, proj_e, flags=0):
    """Correctness gate outside the timed region: the device pass over the
    first m rows of the benchmarked (HBM-resident) columns against the CPU
    oracle over the same rows copied to the host -- row counts and every
    output buffer bit for bit."""
    from datafusion_amd.arrow import Array, RecordBatch
    from oracle_ffi import oracle_filter_project
    pre = []
    for a in dev_cols:
        if a.data_type == DataType.Utf8:
            offs = a.offsets[: m + 1]
            nb = int(offs[-1].item())
            vb = a.values[: max(nb, 1)]
        else:
            offs = None
            vb = a.values[: m * a.data_type.width]
        valid = a.validity[: (m + 7) // 8] if a.validity is not None else None
        nulls = int(m - _popcount(valid, m)) if valid is not None else 0
        pre.append(Array(a.data_type, m, vb, valid, offs, nulls))
    db = RecordBatch(schema, pre)
    hb = db.to("cpu")
    p = compile_scalar_expr(None, pred_e, schema, flags)
    cp = [compile_scalar_expr(None, e, schema, flags) for e in proj_e]
    got = eng.filter_project(p, cp, db, flags)
    ref = oracle_filter_project(schema, hb, pred_e, proj_e, flags)
    ok = len(got) == len(ref)
    for d, (_, r) in zip(got, ref):
        d = d.cpu()
        ok = ok and d.length == r.length and d.null_count == r.null_count
        if not ok:
            break
        if r.data_type == DataType.Utf8:
            ok = d.numpy_values() == r.numpy_values()
        else:
            ok = np.array_equal(np.asarray(d.numpy_values()).view(np.uint8), np.asarray(r.numpy_values()).view(np.uint8))
        if not ok:
            break
    return {"rows": m, "selected": int(got[0].length) if got else 0, "bit_identical_to_oracle": bool(ok)}


def _popcount(bits, m):
    b = bits.cpu().numpy()
    from datafusion_amd.arrow import unpack_bits
    return int(unpack_bits(b, m).sum())


Q6_ROWS = 600_037_902  # TPC-H SF100 lineitem


def q6_line(eng, dev, rank, world, steps, warmup, dist, rows, comm=None):
    """C4 (BASELINE.json configs[3]): Q6-style predicate over 4 Float64 columns,
    projecting extendedprice*discount (no aggregate: the reference has none).
    Inputs generated on the device with torch (seeded); parity of the query
    is covered in tests/test_gpu_parity.py::test_q6_style_predicate."""
    n = rows
    schema, cols = q6_table(dev, n, SEED + rank)
    pred, projs = q6_query()
    outs = [torch.empty(n, dtype=torch.float64, device=dev)]
    torch.cuda.synchronize(dev)
    step = FusedStep(eng, schema, cols, n, pred, projs, outs, comm=comm)
    el, kms, selected = timed_steps(step, steps, warmup, dist, eng, dev, py_exchange=comm is None)
    kname = kernel_name(eng)
    del outs, step
    from datafusion_amd.arrow import Array
    gate = prefix_gate(eng, schema, [Array(DataType.Float64, n, c.view(torch.uint8)) for c in cols], 1 << 22,
                       pred, projs)
    s = selected / n
    bpr = 32.0 + 8.0 * s  # 4 Float64 inputs, s * 8 B output
    # quantity, discount, shipdate streamed by the predicate; extendedprice lane-masked
    moved = moved_bytes(n, 24, 1, q6_mask(cols), 8 * selected)
    return {"workload": "C4: TPC-H SF100 lineitem Q6-style predicate, 600037902 rows per GPU, "
                        "SELECT l_extendedprice*l_discount (Float64)",
            "rows_per_s": n * world * steps / el, "ms_per_step": el / steps * 1e3, "kernel_ms": round(kms, 4),
            "selectivity": round(s, 5), "selected": selected, "parity_gate": gate,
            "roofline": roofline(kname, n * bpr, kms, n, moved=moved)}


I64_RANGE = 1 << 20  # Int64 columns uniform in [0, 2^20): a*b+c never wraps


def c2_i64_line(eng, dev, rank, world, steps, warmup, dist, rows, sel=0.5):
    """The Int64 half of BASELINE.json configs[1]: the C2 query over three
    Int64 columns (uniform in [0, 2^20), generated in HBM), `SELECT a, b, a*b+c
    WHERE a > k AND b < m`. The reference's filter() rejects Int64 columns
    (filter.rs:106-110), so this runs under the build's Int64-gather extension
    (DFMI_FLAG_EXT_GATHER_ALL); parity: the prefix gate against the oracle,
    and tests/test_gpu_parity.py::test_all_types_int64_on_gpu."""
    from datafusion_amd.arrow import Array
    n = rows
    cols = [torch.empty(n, dtype=torch.int64, device=dev) for _ in range(3)]
    err = _abi.dfmi_error()
    for j, t in enumerate(cols):
        rc = _abi.lib().dfmi_generate_column(eng.ctx, _abi.DFMI_GEN_I64, SEED + 7, j, rank * n, n, 0, I64_RANGE,
                                              C.c_void_p(t.data_ptr()), C.byref(err))
        assert rc == 0, err.message
    schema = Schema([Field(c, DataType.Int64, False) for c in "abc"])
    k, m = int(I64_RANGE * (1.0 - sel ** 0.5)), int(I64_RANGE * sel ** 0.5)
    pred = BinaryExpr(BinaryExpr(Column(0), Operator.Gt, Literal(Int64(k))), Operator.And,
                      BinaryExpr(Column(1), Operator.Lt, Literal(Int64(m))))
    projs = [Column(0), Column(1), BinaryExpr(BinaryExpr(Column(0), Operator.Multiply, Column(1)), Operator.Plus,
                                              Column(2))]
    flags = _abi.DFMI_FLAG_EXT_GATHER_ALL
    outs = [torch.empty(n, dtype=torch.int64, device=dev) for _ in range(3)]
    torch.cuda.synchronize(dev)
    step = FusedStep(eng, schema, cols, n, pred, projs, outs, flags=flags)
    el, kms, selected = timed_steps(step, steps, warmup, dist, eng, dev)
    kname = kernel_name(eng)
    del outs, step
    gate = prefix_gate(eng, schema, [Array(DataType.Int64, n, c.view(torch.uint8)) for c in cols], 1 << 22, pred,
                       projs, flags)
    s = selected / n
    bpr = 24.0 + 24.0 * s  # as C2: a, b, c read; s * (a, b, a*b+c) written
    moved = moved_bytes(n, 16, 1, (cols[0] > k) & (cols[1] < m), 24 * selected)
    return {"workload": "C2 over Int64: 1e9-row Int64 a,b,c per GPU (uniform [0, 2^20)), s=%.2f "
                        "(Int64 gather: DFMI_FLAG_EXT_GATHER_ALL)" % sel,
            "rows_per_s": n * world * steps / el, "ms_per_step": el / steps * 1e3, "kernel_ms": round(kms, 4),
            "selectivity": round(s, 5), "selected": selected, "parity_gate": gate,
            "roofline": roofline(kname, n * bpr, kms, n, moved=moved)}


def q6_agg_line(eng, dev, rank, world, steps, warmup, dist, rows, comm=None):
    """Real TPC-H Q6 (DFMI_FLAG_EXT_AGGREGATE): SELECT SUM(l_extendedprice *
    l_discount) FROM lineitem WHERE <Q6 predicate>, one fused predicate +
    exact-sum pass per step over the C4 table; with --gpus N every rank's exact
    partial is all_gathered and merged (bit-identical to one GPU over all rows).
    Gate: the SUM over a 4M-row prefix equals the oracle's bit for bit."""
    from datafusion_amd.arrow import Array, RecordBatch
    from datafusion_amd.execution.engine import merge_agg_partials
    from datafusion_amd.execution.expression import compile_expr
    from datafusion_amd.logicalplan import AggregateFunction
    from oracle_ffi import oracle_aggregate
    flags = _abi.DFMI_FLAG_EXT_AGGREGATE
    n = rows
    schema, cols = q6_table(dev, n, SEED + rank)
    pred_e, projs = q6_query()
    sum_e = AggregateFunction("SUM", (projs[0],), DataType.Float64)
    pred = compile_scalar_expr(None, pred_e, schema, flags)
    agg = compile_expr(None, sum_e, schema, flags)
    st = eng.agg_state([agg])
    batch = RecordBatch(schema, [Array(DataType.Float64, n, c.view(torch.uint8)) for c in cols])
    res = {}

    def step():
        st.reset()
        st.add(pred, batch, flags)
        if comm is not None:  # C-ABI: RCCL all_gather of the exact partials + merge
            v = comm.agg_finish(st)[0]
        elif dist:
            mine = torch.frombuffer(bytearray(st.partial()), dtype=torch.uint8).to(coll_device(dev))
            parts = [torch.empty_like(mine) for _ in range(world)]
            dist.all_gather(parts, mine)
            v = merge_agg_partials([agg], [p.cpu().numpy().tobytes() for p in parts])[0]
        else:
            v = st.finish()[0]
        res["v"] = v
        return v.count

    el, kms, selected = timed_steps(step, steps, warmup, dist, eng, dev, py_exchange=False)
    kname = kernel_name(eng)
    # gate: 4M-row prefix against the oracle
    m = min(n, 1 << 22)
    pre = RecordBatch(schema, [Array(DataType.Float64, m, c[:m].view(torch.uint8)) for c in cols])
    g = eng.agg_state([agg])
    g.add(pred, pre, flags)
    dv = g.finish()[0]
    rv = oracle_aggregate(schema, pre.to("cpu"), pred_e, [sum_e], flags)[0]
    gate = {"rows": m, "sum_bits_equal": bool(dv.bits == rv.bits and dv.count == rv.count), "count": int(rv.count)}
    s = selected / (n * world)  # the merged count covers every rank's rows
    bpr = 32.0  # 4 Float64 inputs; the output is one value
    moved = moved_bytes(n, 24, 1, q6_mask(cols), 0)  # the SUM argument's price column lane-masked
    v = res["v"]
    return {"workload": "C4 real Q6: SELECT SUM(l_extendedprice*l_discount) FROM lineitem WHERE <Q6>, 600037902 "
                        "rows per GPU, exact Float64 sum", "rows_per_s": n * world * steps / el,
            "ms_per_step": el / steps * 1e3, "kernel_ms": round(kms, 4), "selectivity": round(s, 5),
            "sum": float(np.array([v.bits], dtype=np.uint64).view(np.float64)[0]), "parity_gate": gate,
            "roofline": roofline(kname, n * bpr, kms, n, moved=moved)}


def q6_table(dev, n, seed):
    """C4 synthetic lineitem columns in HBM: quantity 1..50,
    extendedprice = quantity * U[900, 2000), discount 0.00..0.10, shipdate day
    8036..10561, all Float64 (reference-executable); torch's seeded RNG."""
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    qty = torch.randint(1, 51, (n,), device=dev, generator=g).to(torch.float64)
    disc = torch.randint(0, 11, (n,), device=dev, generator=g).to(torch.float64) / 100.0
    ship = torch.randint(8036, 10562, (n,), device=dev, generator=g).to(torch.float64)
    price = qty * (900.0 + 1100.0 * torch.rand(n, device=dev, dtype=torch.float64, generator=g))
    names = ("l_quantity", "l_extendedprice", "l_discount", "l_shipdate")
    return Schema([Field(nm, DataType.Float64, False) for nm in names]), [qty, price, disc, ship]


def q6_query():
    """shipdate >= 8766 AND shipdate < 9131 AND discount >= 0.05 AND
    discount <= 0.07 AND quantity < 24; SELECT extendedprice * discount."""
    def ge(c, v):
        return BinaryExpr(Column(c), Operator.GtEq, Literal(Float64(v)))

    def lt(c, v):
        return BinaryExpr(Column(c), Operator.Lt, Literal(Float64(v)))

    pred = BinaryExpr(BinaryExpr(BinaryExpr(BinaryExpr(ge(3, 8766.0), Operator.And, lt(3, 9131.0)), Operator.And,
                                            ge(2, 0.05)), Operator.And,
                                 BinaryExpr(Column(2), Operator.LtEq, Literal(Float64(0.07)))), Operator.And,
                      lt(0, 24.0))
    return pred, [BinaryExpr(Column(1), Operator.Multiply, Column(2))]


def q6_mask(cols):
    """q6_query()'s predicate over q6_table()'s columns, with torch (the
    selection mask moved_bytes() counts lines from)."""
    qty, _, disc, ship = cols
    return (ship >= 8766.0) & (ship < 9131.0) & (disc >= 0.05) & (disc <= 0.07) & (qty < 24.0)


C3_ROWS = 500_000_000
C3_BATCHES = 4  # i32 Utf8 offsets cap one batch's bytes at 2 GiB (arrow BinaryArray)


def _utf8_dictionary(seed, words=1000, max_len=24):
    """'w<i>' padded with lowercase letters to a length drawn from [len, max_len]."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(words):
        w = b"w%d" % i
        ln = int(rng.integers(len(w), max_len + 1))
        out.append(w + bytes(rng.integers(97, 123, ln - len(w)).astype(np.uint8)))
    return out


def _c3_batch(dev, g, n, dict_bytes, dict_off, dict_len):
    """One C3 batch on the device: v Float64 with ~10% nulls, s Utf8 drawn from
    the dictionary (non-null)."""
    from datafusion_amd.arrow import Array
    v = torch.rand(n, device=dev, dtype=torch.float64, generator=g)
    valid = torch.rand(n, device=dev, generator=g) >= 0.10
    pad = (-n) % 64
    vb = torch.cat([valid, torch.zeros(pad, dtype=torch.bool, device=dev)]).view(-1, 8).to(torch.uint8)
    vbits = (vb << torch.arange(8, device=dev, dtype=torch.uint8)).sum(1, dtype=torch.uint8)
    nulls = int(n - valid.sum().item())
    idx = torch.randint(0, len(dict_len), (n,), device=dev, generator=g)
    lens = dict_len[idx]
    offs64 = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens, 0, out=offs64[1:])
    total = int(offs64[-1].item())
    assert total < 2 ** 31
    data = torch.empty(total, dtype=torch.uint8, device=dev)
    step = 1 << 24
    for r0 in range(0, n, step):  # bytes of rows [r0, r1) in bounded-memory chunks
        r1 = min(n, r0 + step)
        li = lens[r0:r1]
        row = torch.repeat_interleave(torch.arange(r0, r1, device=dev), li)
        within = torch.arange(row.numel(), device=dev) - (offs64[row] - offs64[r0])
        data[offs64[r0]:offs64[r1]] = dict_bytes[dict_off[idx[row]] + within]
    s = Array(DataType.Utf8, n, data, None, offs64.to(torch.int32), 0)
    va = Array(DataType.Float64, n, v.view(torch.uint8), vbits, None, nulls)
    return [s, va], total


def c3_line(eng, dev, rank, world, steps, warmup, dist):
    """C3 (BASELINE.json configs[2]): 5e8 rows = 4 batches of 1.25e8 rows, a
    nullable Float64 v and a Utf8 s. Three queries, each one launch per batch:
      eq:  SELECT s, v WHERE s = <word 17> (Utf8 equality, DFMI_FLAG_EXT_UTF8_COMPARE)
      lt:  SELECT s, v WHERE v < 0.5     (nullable predicate, Utf8 offset/byte gather)
      ne:  SELECT s, v WHERE s != <word 17> (Utf8-only predicate selecting ~all rows)
    Parity of both query shapes: tests/test_gpu_parity.py::test_utf8_gather_and_equality."""
    from datafusion_amd._abi import DFMI_FLAG_EXT_UTF8_COMPARE
    from datafusion_amd.execution.engine import column_struct
    from datafusion_amd.logicalplan import Utf8
    words = _utf8_dictionary(SEED)
    w17 = words[17].decode()  # one dictionary word: selectivity ~1/1000
    dict_bytes = torch.tensor(np.frombuffer(b"".join(words), dtype=np.uint8), device=dev)
    dict_len = torch.tensor([len(w) for w in words], dtype=torch.int64, device=dev)
    dict_off = torch.cumsum(dict_len, 0) - dict_len
    g = torch.Generator(device=dev)
    g.manual_seed(SEED + 1000 + rank)
    nb = C3_ROWS // C3_BATCHES
    batches, nbytes = [], 0
    for _ in range(C3_BATCHES):
        b, t = _c3_batch(dev, g, nb, dict_bytes, dict_off, dict_len)
        batches.append(b)
        nbytes += t
    torch.cuda.empty_cache()
    schema = Schema([Field("s", DataType.Utf8, False), Field("v", DataType.Float64, True)])
    out_s_off = torch.zeros(nb + 16, dtype=torch.int32, device=dev)
    out_s_data = torch.empty(max(b[0].values.numel() for b in batches), dtype=torch.uint8, device=dev)
    out_v = torch.empty(nb, dtype=torch.float64, device=dev)
    L = _abi.lib()
    queries = {
        "eq": (BinaryExpr(Column(0), Operator.Eq, Literal(Utf8(w17))), DFMI_FLAG_EXT_UTF8_COMPARE),
        "lt": (BinaryExpr(Column(1), Operator.Lt, Literal(Float64(0.5))), 0),
        # a Utf8-only predicate selecting ~all rows: the one-tile kernel from the
        # second call on (exec.cpp high_sel; the warm-up steps make that switch)
        "ne": (BinaryExpr(Column(0), Operator.NotEq, Literal(Utf8(w17))), DFMI_FLAG_EXT_UTF8_COMPARE),
    }
    res = {}
    for qn, (pe, flags) in queries.items():
        pred = compile_scalar_expr(None, pe, schema, flags)
        projs = [compile_scalar_expr(None, Column(0), schema, flags), compile_scalar_expr(None, Column(1), schema, flags)]
        progs = (C.c_void_p * 2)(*[p.handle.value for p in projs])
        calls = []
        for b in batches:
            carr = (_abi.dfmi_column * 2)(column_struct(b[0]), column_struct(b[1]))
            cb = _abi.dfmi_batch(2, 0, nb, carr)
            outs = (_abi.dfmi_out_column * 2)()
            outs[0].offsets = out_s_off.data_ptr()
            outs[0].data = out_s_data.data_ptr()
            outs[0].data_capacity = out_s_data.numel()
            outs[1].values = out_v.data_ptr()
            calls.append((carr, cb, outs))
        err = _abi.dfmi_error()
        acc = {"sel": 0, "sel_bytes": 0, "kms": 0.0}

        def step():
            acc["sel"] = acc["sel_bytes"] = 0
            acc["kms"] = 0.0
            for carr, cb, outs in calls:
                rc = L.dfmi_filter_project(eng.ctx, pred.handle, progs, 2, C.byref(cb), outs, flags, C.byref(err))
                if rc != 0:
                    raise RuntimeError(err.message.decode())
                acc["sel"] += outs[0].length
                acc["sel_bytes"] += outs[0].data_length
                acc["kms"] += eng.last_timing()[1]
            return acc["sel"]

        kms_all = []

        def timed():
            r = step()
            kms_all.append(acc["kms"])
            return r

        el, _, selected = timed_steps(timed, steps, warmup, dist, eng, dev)
        kname = kernel_name(eng)
        kms = float(np.mean(kms_all[warmup:]))
        gate = prefix_gate(eng, schema, batches[0], 1 << 22, pe, [Column(0), Column(1)], flags)
        n = C3_ROWS
        s = selected / n
        # v 8 B + validity 1/8 B, s offsets 4 B + its bytes; out s*(8 + 4) + selected bytes
        alg = n * (8.0 + 0.125 + 4.0) + nbytes + selected * 12.0 + acc["sel_bytes"]
        # kms sums the step's C3_BATCHES launches: roofline() gets the per-launch mean
        rl = roofline(kname, alg / C3_BATCHES, kms / C3_BATCHES, n, launches=C3_BATCHES)
        rl["kernel_ms_per_step"] = round(kms, 4)
        res[qn] = {"query": "SELECT s, v WHERE " + {"eq": "s = '%s'" % w17, "lt": "v < 0.5", "ne": "s != '%s'" % w17}[qn],
                   "rows_per_s": n * world * steps / el, "ms_per_step": el / steps * 1e3,
                   "kernel_ms": round(kms, 4), "selectivity": round(s, 5), "selected": selected,
                   "parity_gate": gate, "roofline": rl}
    return {"workload": "C3: 5e8 rows per GPU (4 batches of 1.25e8), nullable Float64 v (10%% nulls) + "
                        "Utf8 s (1000-word dictionary, avg %.2f B)" % (nbytes / C3_ROWS), **res}


GROUPBY_ROWS = 100_000_000
GROUPBY_KEYS = 10_000


def groupby_line(eng, dev, rank, world, steps, warmup, dist, rows=GROUPBY_ROWS):
    """GROUP BY on the device (DFMI_FLAG_EXT_AGGREGATE; the reference plans
    Aggregate{group_expr} (sqlplanner.rs:91-117) but cannot execute it,
    context.rs:161): SELECT k, SUM(v), COUNT(v) FROM t GROUP BY k over `rows`
    HBM-resident rows with 10,000 distinct keys -- an Int64 key, a Float64
    key, a Utf8 key, and the two keys (Int64, Utf8) -- each step one
    dfmi_aggregate_batch (fused evaluation pass, hash-table claim and
    accumulate passes) plus the finish (every group back in key order).
    Exact Float64 SUM. Gate: a 2^20-row prefix against the oracle, keys and
    values bit for bit. The batch has 1e4 rows per group, so the bucketed
    passes run (groupby.h: claim, rank, scatter by bucket, per-bucket LDS
    sums): `pass_bytes_per_row` counts what those passes move per row (the
    claim reads the key and writes the slot index, the rank reads both and
    writes the group id, the scatter reads it and v and writes both, the
    bucket pass reads them back), `frac` the algorithmic bytes' rate over
    the HBM peak."""
    from datafusion_amd.arrow import Array, RecordBatch
    from datafusion_amd.execution.expression import compile_expr
    from datafusion_amd.logicalplan import AggregateFunction
    from oracle_ffi import oracle_aggregate_grouped_multi
    AGGF = _abi.DFMI_FLAG_EXT_AGGREGATE
    g = torch.Generator(device=dev)
    g.manual_seed(SEED + 77 + rank)
    n = rows
    ki = torch.randint(0, GROUPBY_KEYS, (n,), device=dev, generator=g)
    v = torch.rand(n, device=dev, dtype=torch.float64, generator=g)
    words = [b"k%d_" % i + b"x" * (i % 13) for i in range(GROUPBY_KEYS)]
    dict_bytes = torch.tensor(np.frombuffer(b"".join(words), dtype=np.uint8), device=dev)
    dict_len = torch.tensor([len(w) for w in words], dtype=torch.int64, device=dev)
    dict_off = torch.cumsum(dict_len, 0) - dict_len
    lens = dict_len[ki]
    offs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens, 0, out=offs[1:])
    data = torch.empty(int(offs[-1].item()), dtype=torch.uint8, device=dev)
    for r0 in range(0, n, 1 << 24):
        r1 = min(n, r0 + (1 << 24))
        row = torch.repeat_interleave(torch.arange(r0, r1, device=dev), lens[r0:r1])
        within = torch.arange(row.numel(), device=dev) - (offs[row] - offs[r0])
        data[offs[r0]:offs[r1]] = dict_bytes[dict_off[ki[row]] + within]
    utf8 = Array(DataType.Utf8, n, data, None, offs.to(torch.int32), 0)
    kint = (ki * 7919 - 5000).contiguous()
    kflt = (ki.to(torch.float64) / 7.0).contiguous()
    vv = Array(DataType.Float64, n, v.view(torch.uint8))
    cases = {
        "int64": [Array(DataType.Int64, n, kint.view(torch.uint8))],
        "float64": [Array(DataType.Float64, n, kflt.view(torch.uint8))],
        "utf8": [utf8],
        "int64_utf8": [Array(DataType.Int64, n, (ki % 100).contiguous().view(torch.uint8)), utf8],
    }
    out = {"workload": "SELECT k, SUM(v), COUNT(v) FROM t GROUP BY k: %d rows per GPU, %d distinct keys, v Float64 "
                       "(exact SUM)" % (n, GROUPBY_KEYS)}
    if world > 1:  # each rank's groups of its own shard; the merge across ranks is a separate entry point
        out["note"] = ("per-rank groups (rows/s counts every rank's rows); merging them across ranks is "
                       "dfmi_shard_agg_finish_grouped (RCCL all_gather of the exact per-group partials), tested "
                       "at world 2 / 3 over the loopback transport (tests/test_shard_abi_gpu.py), not timed here")
    for name, kcols in cases.items():
        nk = len(kcols)
        schema = Schema([Field("k%d" % i, c.data_type, False) for i, c in enumerate(kcols)] +
                        [Field("v", DataType.Float64, False)])
        batch = RecordBatch(schema, kcols + [vv])
        aggs_e = [AggregateFunction("SUM", (Column(nk),), DataType.Float64),
                  AggregateFunction("COUNT", (Column(nk),), DataType.UInt64)]
        aggs = [compile_expr(None, a, schema, AGGF) for a in aggs_e]
        keys = [compile_scalar_expr(None, Column(i), schema, AGGF) for i in range(nk)]
        # the calls the Rust AggregateRelation makes (INTEGRATION.md "Aggregate"), on a state
        # created once per plan: reset, one batch, the groups into caller-owned arrays
        L = _abi.lib()
        st = eng.grouped_agg_state(keys, aggs)
        cb, keep = eng._batch_struct(batch)
        cap = 2 * GROUPBY_KEYS
        kout = (_abi.dfmi_agg_value * (cap * nk))()
        vout = (_abi.dfmi_agg_value * (cap * len(aggs)))()
        ngr = C.c_int64()
        err = _abi.dfmi_error()

        def step():
            rc = L.dfmi_agg_state_reset(eng.ctx, st.handle, C.byref(err))
            rc = rc or L.dfmi_aggregate_batch(eng.ctx, st.handle, None, C.byref(cb), AGGF, C.byref(err))
            rc = rc or L.dfmi_agg_state_finish_grouped(eng.ctx, st.handle, cap, kout, vout, C.byref(ngr),
                                                       C.byref(err))
            if rc != 0:
                raise RuntimeError(err.message.decode())
            return ngr.value

        el, _, groups = timed_steps(step, steps, warmup, dist, eng, dev, py_exchange=False)
        # gate: a 2^20-row prefix against the oracle
        m = 1 << 20
        pre = RecordBatch(schema, [_prefix(c, m) for c in kcols] + [_prefix(vv, m)])
        st = eng.grouped_agg_state(keys, aggs)
        st.add(None, pre, AGGF)
        dk, dv = st.finish()
        rk, rv, rs = oracle_aggregate_grouped_multi(schema, pre.to("cpu"), None, [Column(i) for i in range(nk)],
                                                    aggs_e, AGGF)
        ok = [[(x.is_null, x.bits, x.count) for x in gk] for gk in dk] == \
             [[(x.is_null, x.bits, x.count) for x in gk] for gk in rk]
        ok = ok and [[(x.is_null, x.bits, x.count) for x in gv] for gv in dv] == \
            [[(x.is_null, x.bits, x.count) for x in gv] for gv in rv]
        for p, strs in enumerate(rs):
            if strs is not None:
                ok = ok and st.key_strings(p) == strs
        kb = sum(4 + float(c.values.numel()) / n if c.data_type == DataType.Utf8 else c.data_type.width for c in kcols)
        bpr = kb + 8.0
        ms = el / steps * 1e3
        pbr = 2 * kb + 48.0  # claim kb + 4, rank 4 + kb + 4, scatter 4 + 8 + 4 + 8, bucket 4 + 8
        out[name] = {"rows_per_s": n * world * steps / el, "ms_per_step": round(ms, 3), "groups": groups,
                     "parity_gate": {"rows": m, "groups": len(rk), "bit_identical_to_oracle": bool(ok)},
                     "algorithmic_bytes_per_row": round(bpr, 3),
                     "achieved_gbs": round(n * bpr / (ms * 1e-3) / 1e9, 1),
                     "frac": round(n * bpr / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "pass_bytes_per_row": round(pbr, 3),
                     "pass_gbs": round(n * pbr / (ms * 1e-3) / 1e9, 1),
                     "bound": "the claim and rank passes' dependent random table reads, the scatter and bucket "
                              "passes' streamed-load latency; the whole step incl. the finish (DESIGN.md §6)"}
    del utf8, data, offs, cases
    return out


def _prefix(a, m):
    """The first m rows of an offset-0 device Array (a view)."""
    from datafusion_amd.arrow import Array
    if a.data_type == DataType.Utf8:
        return Array(a.data_type, m, a.values, None, a.offsets[: m + 1], 0)
    return Array(a.data_type, m, a.values[: m * a.data_type.width], None, None, 0)


HOST_ROWS = 100_000_000


def host_line(eng, steps, warmup):
    """PCIe-inclusive rate: the C2 query at s=0.5 over a HOST
    batch through dfmi_filter_project_host (row chunks pipelined: host staging,
    H2D, kernel and D2H of consecutive chunks overlap; the selected rows land
    in library-owned host buffers). Two variants: pageable input buffers
    (staged through pinned memory by host threads) and input buffers in pinned
    memory from dfmi_host_alloc (DMA'd straight from the caller's buffers, as
    a reader parsing into them would hand over). Never `value`."""
    import numpy as np
    from oracle_ffi import gen_unit_f64
    n = HOST_ROWS
    schema = Schema([Field(c, DataType.Float64, False) for c in "abc"])
    host_cols = [gen_unit_f64(SEED, j, 0, n) for j in range(3)]
    pred_e, proj_e = query(0.5)
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

    def run(cb):
        def step():
            res = C.c_void_p()
            rc = L.dfmi_filter_project_host(eng.ctx, pred.handle, progs, 3, C.byref(cb), 0, C.byref(res),
                                            C.byref(err))
            if rc != 0:
                raise RuntimeError(err.message.decode())
            v = _abi.dfmi_column()
            L.dfmi_host_result_column(res, 2, C.byref(v))
            sel = v.length
            chk = float(np.ctypeslib.as_array(C.cast(v.values, C.POINTER(C.c_double)), shape=(sel,))[::4099].sum())
            L.dfmi_host_result_free(res)
            return sel, chk
        for _ in range(warmup):
            step()
        t0 = time.perf_counter()
        for _ in range(steps):
            sel, chk = step()
        el = (time.perf_counter() - t0) / steps
        moved = n * 24 + sel * 24
        return {"rows_per_s": n / el, "ms_per_step": el * 1e3, "selected": sel, "pcie_gbs": round(moved / el / 1e9, 1),
                "bytes_moved_per_step": moved, "checksum": chk}

    cb, keep = batch_of([c.ctypes.data for c in host_cols])
    pageable = run(cb)
    pinned_ptrs = []
    try:
        for c in host_cols:
            p = C.c_void_p()
            if L.dfmi_host_alloc(c.nbytes, C.byref(p), C.byref(err)) != 0:
                raise RuntimeError(err.message.decode())
            pinned_ptrs.append(p.value)
            C.memmove(p.value, c.ctypes.data, c.nbytes)
        cb2, keep2 = batch_of(pinned_ptrs)
        pinned = run(cb2)
    finally:
        for p in pinned_ptrs:
            L.dfmi_host_free(p)
    assert (pinned["selected"], pinned["checksum"]) == (pageable["selected"], pageable["checksum"])
    return {"workload": "C2 query, s=0.5, %d-row HOST batch (dfmi_filter_project_host)" % n,
            **pageable, "pinned_input": pinned,
            "note": "host->HBM + kernel + HBM->host of the selected rows, chunks pipelined; not the headline value"}


CSV_ROWS = 5_000_000


def csv_line(eng, steps, warmup):
    """Ingest from a CSV file (never `value`): the native
    reader (csrc/csv_reader.cpp: host threads parse into pinned Arrow batches,
    one batch ahead) alone, and feeding the C2 query (s = 0.5) through the
    pipelined host entry point batch by batch, as ctx.sql over a CSV table
    runs. File: CSV_ROWS rows of the seed-42 a, b, c columns (repr floats)."""
    import tempfile
    import pandas as pd
    from datafusion_amd.execution import NativeCsvDataSource
    from datafusion_amd.execution.engine import column_struct
    from oracle_ffi import gen_unit_f64
    n = CSV_ROWS
    schema = Schema([Field(c, DataType.Float64, False) for c in "abc"])
    d = tempfile.mkdtemp(prefix="dfmi_csv_")
    path = os.path.join(d, "c2.csv")
    pd.DataFrame({c: gen_unit_f64(SEED, j, 0, n) for j, c in enumerate("abc")}).to_csv(path, index=False)
    size = os.path.getsize(path)
    pred_e, proj_e = query(0.5)
    pred = compile_scalar_expr(None, pred_e, schema)
    projs = [compile_scalar_expr(None, e, schema) for e in proj_e]
    progs = (C.c_void_p * 3)(*[p.handle.value for p in projs])
    L = _abi.lib()
    err = _abi.dfmi_error()
    batch = 1 << 20

    def parse_only():
        src = NativeCsvDataSource(schema, path, True, batch, copy=False)
        rows = 0
        while True:
            b = src.next()
            if b is None:
                return rows
            rows += b.num_rows()

    def end_to_end():
        src = NativeCsvDataSource(schema, path, True, batch, copy=False)
        rows = sel = 0
        while True:
            b = src.next()
            if b is None:
                return rows, sel
            carr = (_abi.dfmi_column * 3)(*[column_struct(a) for a in b.columns])
            cb = _abi.dfmi_batch(3, 0, b.num_rows(), carr)
            res = C.c_void_p()
            rc = L.dfmi_filter_project_host(eng.ctx, pred.handle, progs, 3, C.byref(cb), 0, C.byref(res),
                                            C.byref(err))
            if rc != 0:
                raise RuntimeError(err.message.decode())
            v = _abi.dfmi_column()
            L.dfmi_host_result_column(res, 0, C.byref(v))
            sel += v.length
            L.dfmi_host_result_free(res)
            rows += b.num_rows()

    out = {"workload": "CSV file of %d rows x 3 Float64 (%.0f MB), batches of %d rows" % (n, size / 1e6, batch)}
    for name, fn in (("parse_only", parse_only), ("csv_sql_c2", end_to_end)):
        for _ in range(warmup):
            fn()
        t0 = time.perf_counter()
        for _ in range(steps):
            r = fn()
        el = (time.perf_counter() - t0) / steps
        out[name] = {"ms": round(el * 1e3, 1), "rows_per_s": n / el, "csv_gbs": round(size / el / 1e9, 2)}
        if name == "csv_sql_c2":
            out[name]["selected"] = r[1]
    share = len(os.sched_getaffinity(0))
    if int(os.environ.get("OMP_NUM_THREADS", "0") or 0) > 0:
        share = min(share, int(os.environ["OMP_NUM_THREADS"]))
    out["host_threads"] = int(os.environ.get("DFMI_CSV_THREADS", "0")) or max(1, min(share, 64))
    os.remove(path)
    os.rmdir(d)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=float, default=1e9, help="rows per GPU")
    ap.add_argument("--sel", type=float, default=0.5, help="headline selectivity")
    ap.add_argument("--sweep", default="0.01,0.5,0.99", help="selectivities also reported (first=headline if set)")
    ap.add_argument("--extra", default="c4,q6,c2i64,c3,groupby,batches",
                    help="extra config lines (comma list: c4,q6,c2i64,c3,groupby,batches,host,csv; empty = none)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--exchange", choices=("abi", "torch"), default=None,
                    help="N>1 exchange: the C-ABI RCCL path (dfmi_shard_filter_project, default under nccl) or "
                         "torch.distributed (default for the gloo rehearsal)")
    ap.add_argument("--gather", type=int, default=1, help="time dfmi_shard_gather_to_root of the C2 outputs")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if BACKEND != "nccl":
        local %= torch.cuda.device_count()
        if world > torch.cuda.device_count():
            # ranks sharing a GPU: ticket-ordered tiles from the first launch
            # (DESIGN.md §4 "Look-back": blockIdx order can stall behind the
            # other rank's kernel until the 2 s timeout and its relaunch)
            os.environ["DFMI_SHARED"] = "1"  # dfmi_context_create reads it (dfmi_context_set_shared)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if BACKEND == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(BACKEND)

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

    exchange = args.exchange or ("abi" if BACKEND == "nccl" else "torch")
    comm = None
    if (world > 1 and exchange == "abi") or (args.gather and (BACKEND == "nccl" or world == 1)):
        comm = abi_comm(eng, dist, rank, world, dev)
    step_comm = comm if (world > 1 and exchange == "abi") else None
    sels = [args.sel] + [float(x) for x in args.sweep.split(",") if x and float(x) != args.sel]
    results = {}
    for sel in sels:
        step = FusedStep(eng, schema, cols, n, *query(sel), outs, comm=step_comm)
        el, kms, selected = timed_steps(step, args.steps, args.warmup, dist, eng, dev, py_exchange=step_comm is None)
        s_real = selected / n
        bytes_per_row = 24.0 + 24.0 * s_real  # a,b,c read; s*(a,b,a*b+c) written
        kname = kernel_name(eng)
        k_, m_ = 1.0 - sel ** 0.5, sel ** 0.5  # query(sel)'s literals
        moved = moved_bytes(n, 16, 1, (cols[0] > k_) & (cols[1] < m_), 24 * selected)  # a, b streamed; c masked
        rl = roofline(kname, n * bytes_per_row, kms, n, run="main" if sel == 0.5 else "c2_s%.2f" % sel, moved=moved)
        results[sel] = dict(el=el, kms=kms, selected=selected, s=s_real, rl=rl, bpr=bytes_per_row)
    del outs, step
    torch.cuda.empty_cache()
    gather = None
    if args.gather and comm is not None:
        gather = gather_line(eng, comm, schema, cols, n, args.sel, dist, rank, world, dev)
        torch.cuda.empty_cache()
    from datafusion_amd.arrow import Array
    gate = prefix_gate(eng, schema, [Array(DataType.Float64, n, c.view(torch.uint8)) for c in cols],
                       min(n, 1 << 22), *query(args.sel))
    extras = [x for x in args.extra.split(",") if x]
    extra = {}
    if "batches" in extras:
        extra["batches"] = batches_line(eng, schema, cols, args.sel, dev)
    del cols
    torch.cuda.empty_cache()

    for name in extras:
        if name == "batches":
            continue
        if name == "c4":
            extra["c4"] = q6_line(eng, dev, rank, world, args.steps, args.warmup, dist, Q6_ROWS, comm=step_comm)
        elif name == "q6":
            extra["q6"] = q6_agg_line(eng, dev, rank, world, args.steps, args.warmup, dist, Q6_ROWS, comm=step_comm)
        elif name == "c2i64":
            extra["c2i64"] = c2_i64_line(eng, dev, rank, world, args.steps, args.warmup, dist, n, args.sel)
        elif name == "host":
            if world == 1:
                extra["host"] = host_line(eng, min(args.steps, 3), 1)
        elif name == "csv":
            if world == 1:
                extra["csv"] = csv_line(eng, min(args.steps, 3), 1)
        elif name == "c3":
            extra["c3"] = c3_line(eng, dev, rank, world, args.steps, args.warmup, dist)
        elif name == "groupby":
            extra["groupby"] = groupby_line(eng, dev, rank, world, min(args.steps, 5), 1, dist)
        else:
            raise SystemExit("unknown extra config %r" % name)
        torch.cuda.empty_cache()

    h = results[args.sel]
    total_rows = n * world * args.steps
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
                   "selectivity": round(h["s"], 4),
                   "parallelism": ("row-range shards, C-ABI dfmi_shard_filter_project (RCCL all_gather of "
                                   "placement records)" if step_comm is not None else
                                   "row-range shards, torch.distributed count all_gather" if BACKEND == "nccl" else
                                   "row-range shards, %s rehearsal on shared GPUs" % BACKEND) if world > 1
                   else "one GPU"},
        "roofline": h["rl"],
        "sweep": {("%.2f" % s): {"rows_per_s": n * world * args.steps / r["el"], "kernel_ms": round(r["kms"], 4),
                                 "hbm_gbs": r["rl"]["achieved"], "frac": r["rl"]["frac"], "selected": r["selected"],
                                 "roofline": r["rl"]}
                  for s, r in results.items()},
        "parity_gate": gate,
        "box": {"host": socket.gethostname(), "gpu": _gpu_id(dev)},
    }
    if gather is not None:
        out["gather"] = gather
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


def _gpu_id(dev):
    """The GPU this run measured (name + PCI bus id): which box the line's
    HIP-event times come from, next to the committed profile's box."""
    try:
        p = torch.cuda.get_device_properties(dev)
        return "%s %s uuid %s pci %s" % (p.name, getattr(p, "gcnArchName", ""), getattr(p, "uuid", "?"),
                                          getattr(p, "pci_bus_id", "?"))
    except Exception:  # noqa: BLE001
        return None


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
