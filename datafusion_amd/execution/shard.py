"""Row-range sharding of the Selection + Projection pull across GPUs.

The reference is single-threaded (``Rc<RefCell<..>>``, context.rs:33) and has
no parallelism at all (README.md:30,33-35). Rows are independent through
FilterRelation/ProjectRelation, and ``filter()`` preserves row order
(filter.rs:87-91), so the path shards by row range: one process per GPU
(``torch.distributed``, backend "nccl" = RCCL over xGMI), rank r of N owning
rows ``[r*n//N, (r+1)*n//N)`` of the table as its own HBM-resident batch.

After each rank's fused pass the ONLY exchange is one ``all_gather`` of a few
int64 per rank -- selected rows, Utf8 bytes of every Utf8 output, null count
of every output -- from which every rank knows its global output row offset
and the rebase of its Utf8 offsets. Results stay sharded: per-rank batches in
rank order ARE the reference's output stream. ``gather_to_root`` optionally
concatenates everything on one rank with point-to-point send/recv (RCCL has no
gatherv); that leg is bound by the root's xGMI ingress and is never part of
the headline throughput.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence

import torch
import torch.distributed as dist

from .. import _abi
from ..arrow import Array, RecordBatch
from ..logicalplan import DataType
from .error import ExecutionError


def shard_range(total_rows: int, rank: int, world: int):
    """Rows [start, stop) of the global table owned by `rank`."""
    if world < 1 or not (0 <= rank < world) or total_rows < 0:
        raise ValueError("bad shard geometry")
    return total_rows * rank // world, total_rows * (rank + 1) // world


@dataclass
class ShardResult:
    """One rank's slice of the output stream plus its global placement."""
    columns: List[Array]
    rank: int
    world: int
    row_offset: int           # first global output row of this shard
    total_rows: int           # output rows over all ranks
    counts: List[List[int]]   # per rank: [rows, utf8 bytes per output..., nulls per output...]
    utf8_base: List[int]      # per output: global byte offset of this shard's Utf8 data (0 if not Utf8)


def _exchange_device(group) -> torch.device:
    backend = dist.get_backend(group)
    if backend == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def exchange_counts(mine: Sequence[int], group=None) -> List[List[int]]:
    """The path's one collective: all_gather of this rank's int64 counts
    (RCCL over xGMI under "nccl", 8 B x len(mine) per rank)."""
    world = dist.get_world_size(group)
    dev = _exchange_device(group)
    t = torch.tensor(list(mine), dtype=torch.int64, device=dev)
    allc = torch.empty(world * len(mine), dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(allc, t, group=group)
    return allc.view(world, len(mine)).cpu().tolist()


class ShardedFilterProject:
    """FilterRelation/ProjectRelation pull over a row-range shard.

    ``run_shard(predicate, projections, batch, flags) -> List[Array]`` is the
    per-rank pass; by default the rank's DeviceEngine (the fused HIP kernel),
    which fails loudly without a GPU."""

    def __init__(self, predicate, projections: Optional[Sequence], flags: int = 0, group=None,
                 run_shard: Optional[Callable] = None, device=None):
        self.predicate = predicate
        self.projections = list(projections or [])
        self.flags = flags
        self.group = group
        if run_shard is None:
            from .engine import engine
            eng = engine(device)
            run_shard = eng.filter_project
        self.run_shard = run_shard

    def __call__(self, local_batch: RecordBatch) -> ShardResult:
        try:
            cols = self.run_shard(self.predicate, self.projections, local_batch, self.flags)
        except ExecutionError as e:
            # still take part in the exchange: every rank must learn the query failed
            return self.exchange(None, e)
        except Exception as e:
            # any other failure (device OOM, a bad argument) also joins the
            # exchange -- the other ranks would block in it otherwise -- then
            # re-raises here; the other ranks raise an ExecutionError
            try:
                self.exchange(None, ExecutionError("ExecutionError", "shard %d failed: %s: %s" % (
                    dist.get_rank(self.group), type(e).__name__, e)))
            except ExecutionError:
                pass
            raise
        return self.exchange(cols)

    def exchange(self, cols: Optional[List[Array]], error: Optional[ExecutionError] = None) -> ShardResult:
        """The one all_gather: [status, error position, rows, Utf8 bytes per
        output..., nulls per output...] per rank. When any rank failed, every
        rank raises the error the reference would raise first over the whole
        table: the smallest evaluation position, then the lowest rank (= the
        earliest rows), with that rank's message."""
        world = dist.get_world_size(self.group)
        rank = dist.get_rank(self.group)
        nout = len(cols) if cols is not None else max(1, len(self.projections))
        mine = shard_record(cols, error, nout)
        width = 3 + 2 * _MAX_OUT
        allc = exchange_counts(mine, self.group)
        failed = [r for r in range(world) if allc[r][0]]
        if failed:
            first = min(failed, key=lambda r: (allc[r][1], r))
            msg = error.message if error is not None else ""
            msgs = _exchange_messages(msg, self.group)
            raise ExecutionError.from_status(int(allc[first][0]), msgs[first])
        counts = [[c[2]] + c[3:3 + nout] + c[3 + _MAX_OUT:3 + _MAX_OUT + nout] for c in allc]
        row_offset = sum(counts[r][0] for r in range(rank))
        total = sum(c[0] for c in counts)
        utf8_base = [sum(counts[r][1 + o] for r in range(rank)) for o in range(nout)]
        assert width == len(mine)
        return ShardResult(cols, rank, world, row_offset, total, counts, utf8_base)


_MAX_OUT = 16
_MSG = 512


def shard_record(cols: Optional[List[Array]], error: Optional[ExecutionError], nout: int) -> List[int]:
    """This rank's exchange record, the layout csrc/shard.cpp exchanges too:
    [status, error position (evaluation-order key >> 44; none sorts last),
    rows, Utf8 bytes per output (16), nulls per output (16)]."""
    if error is None:
        rows = cols[0].length if cols else 0
        mine = [0, 0, rows] + [c.data_bytes() if c.data_type == DataType.Utf8 else 0 for c in cols] + \
               [c.null_count for c in cols]
    else:
        key = getattr(error, "order_key", None)
        pos = (((1 << 64) - 1) if key is None else key) >> 44
        mine = [error.code or _abi.DFMI_ERR_EXECUTION, pos, 0] + [0] * (2 * nout)
    # every rank sends the same record length (failed ranks pad)
    return mine[:3] + _pad(mine[3:3 + nout], _MAX_OUT) + _pad(mine[3 + nout:], _MAX_OUT)


def _pad(xs, n):
    xs = list(xs)[:n]
    return xs + [0] * (n - len(xs))


def _exchange_messages(msg: str, group=None) -> List[str]:
    """Every rank's (error) message, fixed-size all_gather."""
    world = dist.get_world_size(group)
    dev = _exchange_device(group)
    b = msg.encode("utf-8")[:_MSG - 1]
    t = torch.zeros(_MSG, dtype=torch.uint8, device=dev)
    if b:
        t[:len(b)] = torch.tensor(list(b), dtype=torch.uint8, device=dev)
    allm = torch.empty(world * _MSG, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(allm, t, group=group)
    out = []
    for r in range(world):
        raw = bytes(allm[r * _MSG:(r + 1) * _MSG].cpu().tolist())
        out.append(raw.split(b"\0", 1)[0].decode("utf-8", errors="replace"))
    return out


def _values_nbytes(t: DataType, rows: int, utf8_bytes: int) -> int:
    if t == DataType.Utf8:
        return utf8_bytes
    if t == DataType.Boolean:
        return (rows + 7) // 8
    return rows * t.width


def _bits_to_bool(buf: torch.Tensor, n: int) -> torch.Tensor:
    shifts = torch.arange(8, device=buf.device, dtype=torch.uint8)
    return ((buf[: (n + 7) // 8].unsqueeze(1) >> shifts) & 1).reshape(-1)[:n].bool()


def _bool_to_bits(b: torch.Tensor) -> torch.Tensor:
    n = b.numel()
    pad = (-n) % 8
    x = torch.cat([b.to(torch.uint8), torch.zeros(pad, dtype=torch.uint8, device=b.device)]).view(-1, 8)
    w = (1 << torch.arange(8, device=b.device, dtype=torch.int32)).to(torch.int32)
    return (x.to(torch.int32) * w).sum(1).to(torch.uint8)


def gather_to_root(res: ShardResult, types: Sequence[DataType], root: int = 0, group=None) -> Optional[List[Array]]:
    """Concatenate every rank's shard on `root` (rank order = reference row
    order). Point-to-point: each non-root rank sends its buffers, the root
    receives them in rank order. Returns the columns on root, None elsewhere."""
    world, rank = res.world, res.rank
    dev = _exchange_device(group)
    nout = len(types)
    rows_of = [c[0] for c in res.counts]
    bytes_of = [[c[1 + o] for c in res.counts] for o in range(nout)]
    nulls_of = [[c[1 + nout + o] for c in res.counts] for o in range(nout)]

    def buffers(cols: List[Array], r: int):
        """(tensor, nbytes) per buffer in the order both sides agree on."""
        out = []
        for o, t in enumerate(types):
            n = rows_of[r]
            nb = _values_nbytes(t, n, bytes_of[o][r])
            out.append(("values", o, nb))
            if t == DataType.Utf8:
                out.append(("offsets", o, (n + 1) * 4))
            if any(nulls_of[o]):
                out.append(("validity", o, (n + 7) // 8))
        return out

    def bits(buf: torch.Tensor, off: int, n: int, nb: int) -> torch.Tensor:
        """Bits [off, off + n) of an LSB-first bitmap as nb bytes from bit 0."""
        if off % 8 == 0:
            return buf[off // 8: off // 8 + nb]
        return _bool_to_bits(_bits_to_bool(buf, off + n)[off:])[:nb]

    def local(kind: str, o: int, nb: int) -> torch.Tensor:
        # a passthrough output is the input Array itself, which may be sliced
        # (arrow ArrayData::offset): read its rows from physical slot `off`
        a = res.columns[o]
        off = a.offset
        if kind == "values":
            if a.data_type == DataType.Utf8:
                start = int(a.offsets[off]) if a.length else 0
                return a.values[start: start + nb]
            if a.data_type == DataType.Boolean:
                return bits(a.values, off, a.length, nb)
            w = a.data_type.width
            return a.values[off * w: off * w + nb]
        if kind == "offsets":  # (the root rebases each part from its first offset)
            return a.offsets[off: off + a.length + 1].contiguous().view(torch.uint8)
        if a.validity is not None:
            return bits(a.validity, off, a.length, nb)
        return _bool_to_bits(torch.ones(a.length, dtype=torch.bool, device=a.values.device))[:nb]

    for o, t in enumerate(types):  # i32 offsets address < 2^31 bytes (arrow BinaryArray)
        if t == DataType.Utf8 and sum(bytes_of[o]) >= (1 << 31):
            raise ExecutionError("Capacity", "gathered Utf8 column exceeds 2^31 bytes")

    # every transfer posted at once (batch_isend_irecv): under RCCL the root
    # receives from all ranks concurrently, over all of its xGMI links
    ops, keep = [], []
    if rank != root:
        for kind, o, nb in buffers(res.columns, rank):
            if nb:
                t = local(kind, o, nb).contiguous().to(dev)
                keep.append(t)
                ops.append(dist.P2POp(dist.isend, t, root, group))
        for req in (dist.batch_isend_irecv(ops) if ops else []):
            req.wait()
        return None

    parts = {}
    for r in range(world):
        for kind, o, nb in buffers(res.columns, r):
            if r == root:
                buf = local(kind, o, nb).contiguous().to(dev)
            else:
                buf = torch.empty(nb, dtype=torch.uint8, device=dev)
                if nb:
                    ops.append(dist.P2POp(dist.irecv, buf, r, group))
            parts[(kind, o, r)] = buf
    for req in (dist.batch_isend_irecv(ops) if ops else []):
        req.wait()

    total = sum(rows_of)
    out = []
    for o, t in enumerate(types):
        if t == DataType.Boolean:
            vals = _bool_to_bits(torch.cat([_bits_to_bool(parts[("values", o, r)], rows_of[r]) for r in range(world)]))
        else:
            vals = torch.cat([parts[("values", o, r)] for r in range(world)])
        offs = None
        if t == DataType.Utf8:
            pieces, base = [], 0
            for r in range(world):
                of = parts[("offsets", o, r)].view(torch.int32)
                of = of - of[0] + base
                pieces.append(of[:-1] if r < world - 1 else of)
                base += bytes_of[o][r]
            offs = torch.cat(pieces) if pieces else torch.zeros(1, dtype=torch.int32, device=dev)
        valid = None
        nulls = sum(nulls_of[o])
        if nulls:
            valid = _bool_to_bits(torch.cat([_bits_to_bool(parts[("validity", o, r)], rows_of[r])
                                             for r in range(world)]))
        pad = (-vals.numel()) % 64 or 0
        vals = torch.cat([vals, torch.zeros(pad + (64 if vals.numel() == 0 else 0), dtype=torch.uint8, device=dev)])
        out.append(Array(t, total, vals, valid, offs, nulls))
    return out


def concat_host(shards: Sequence[ShardResult]) -> List[List]:
    """Python lists of every output column over all shards, rank order
    (test helper for single-process checks of shard placement)."""
    cols = None
    for s in sorted(shards, key=lambda s: s.rank):
        lists = [c.cpu().to_pylist() for c in s.columns]
        cols = lists if cols is None else [a + b for a, b in zip(cols, lists)]
    return cols or []


__all__ = ["shard_range", "exchange_counts", "shard_record", "ShardResult", "ShardedFilterProject", "gather_to_root", "concat_host"]
