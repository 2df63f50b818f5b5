"""The HBM side of the boundary: moves Arrow buffers into HBM, allocates the
output buffers and runs one fused dfmi_filter_project per input batch.

One DeviceEngine per GPU (per process); it owns a dfmi_context whose stream
is torch's current stream on that device, so torch events time our kernels.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence

import numpy as np
import torch

from .. import _abi
from ..arrow import Array, LazyColumns, RecordBatch, empty_bytes
from ..logicalplan import Column, DataType
from .error import ExecutionError

_ENGINES = {}


def engine(device=None) -> "DeviceEngine":
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    device = torch.device(device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx not in _ENGINES:
        _ENGINES[idx] = DeviceEngine(idx)
    return _ENGINES[idx]


def column_struct(a: Array) -> _abi.dfmi_column:
    c = _abi.dfmi_column()
    c.type = int(a.data_type)
    c.length = a.length
    c.null_count = a.null_count
    c.validity = a.validity.data_ptr() if a.validity is not None else None
    c.values = a.values.data_ptr()
    c.offsets = a.offsets.data_ptr() if a.offsets is not None else None
    c.offset = a.offset
    return c


class DeviceEngine:
    def __init__(self, index: int):
        if not torch.cuda.is_available():
            raise RuntimeError("the MI355X path needs a GPU (torch.cuda.is_available() is False)")
        self.index = index
        self.device = torch.device("cuda", index)
        L = _abi.lib()
        ctx = C.c_void_p()
        err = _abi.dfmi_error()
        stream = torch.cuda.current_stream(self.device).cuda_stream
        rc = L.dfmi_context_create(index, C.c_void_p(stream), C.byref(ctx), C.byref(err))
        if rc != _abi.DFMI_OK:
            raise ExecutionError.from_status(rc, err.message.decode())
        self.ctx = ctx
        self._worker = None    # one thread for filter_project_host_batches_async
        self._inflight = None  # its call in flight (every entry point drains it first)

    def __del__(self):
        try:
            self.drain()
            if self.ctx:
                _abi.lib().dfmi_context_destroy(self.ctx)
        except Exception:
            pass

    def last_timing(self):
        self.drain()
        t, m = C.c_double(), C.c_double()
        if _abi.lib().dfmi_last_timing(self.ctx, C.byref(t), C.byref(m)) != _abi.DFMI_OK:
            return None
        return t.value, m.value

    def to_device(self, batch: RecordBatch) -> RecordBatch:
        if all(c.values.device == self.device for c in batch.columns):
            return batch
        return batch.to(self.device)

    def _alloc_out(self, t: DataType, n: int, need_validity: bool, utf8_capacity: int):
        oc = _abi.dfmi_out_column()
        keep = {}
        if t == DataType.Utf8:
            keep["offsets"] = torch.zeros(max(16, n + 1 + 15), dtype=torch.int32, device=self.device)
            keep["data"] = empty_bytes(max(utf8_capacity, 8), self.device)
            oc.offsets = keep["offsets"].data_ptr()
            oc.data = keep["data"].data_ptr()
            oc.data_capacity = keep["data"].numel()
        else:
            nbytes = (n + 63) // 64 * 8 if t == DataType.Boolean else n * max(t.width, 1)
            keep["values"] = empty_bytes(nbytes, self.device)
            oc.values = keep["values"].data_ptr()
        if need_validity:
            keep["validity"] = empty_bytes((n + 63) // 64 * 8, self.device)
            oc.validity = keep["validity"].data_ptr()
        return oc, keep

    def filter_project(self, predicate, projections: Optional[Sequence], batch: RecordBatch,
                       flags: int = 0, comm: "ShardComm" = None) -> List[Array]:
        """One pull of ProjectRelation(FilterRelation(batch)). ``predicate`` /
        ``projections`` are RuntimeExprs (None / [] when absent). With a
        ShardComm the pass is this rank's shard (dfmi_shard_filter_project):
        the placement lands in comm.placement, the outputs in comm.outputs."""
        self.drain()
        L = _abi.lib()
        batch = self.to_device(batch)
        n = batch.num_rows()
        cols = batch.columns
        projections = list(projections or [])
        carr = (_abi.dfmi_column * max(1, len(cols)))()
        for i, a in enumerate(cols):
            carr[i] = column_struct(a)
        cb = _abi.dfmi_batch()
        cb.num_columns = len(cols)
        cb.num_rows = n
        cb.columns = carr

        out_types, outs_list, keeps = self._prepare_outputs(predicate, projections, cols, n)
        outs = (_abi.dfmi_out_column * max(1, len(out_types)))(*outs_list)
        progs = (C.c_void_p * max(1, len(projections)))(*[p.handle.value for p in projections])
        err = _abi.dfmi_error()
        L.dfmi_context_set_stream(self.ctx, C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream))
        if comm is None:
            rc = L.dfmi_filter_project(self.ctx, predicate.handle if predicate is not None else None,
                                       progs, len(projections), C.byref(cb), outs, flags, C.byref(err))
        else:
            place = _abi.dfmi_shard_placement()
            rc = L.dfmi_shard_filter_project(self.ctx, comm.handle, predicate.handle if predicate is not None else None,
                                             progs, len(projections), C.byref(cb), outs, flags, C.byref(place),
                                             C.byref(err))
            comm.placement, comm.outputs, comm.keep = place, outs, (keeps, out_types)
        if rc != _abi.DFMI_OK:
            e = ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
            key = C.c_uint64()
            L.dfmi_last_error_order(self.ctx, C.byref(key))
            e.order_key = key.value  # evaluation-order position (sharded callers pick the first)
            raise e
        return self._results(out_types, [outs[o] for o in range(len(out_types))], keeps, cols)

    def _prepare_outputs(self, predicate, projections, cols, n):
        """Output types, dfmi_out_column structs (worst-case buffers for n
        rows) and the tensors behind them, for one batch."""
        if projections:
            out_types = [p.get_type() for p in projections]
            src_cols = [p.expr.index if isinstance(p.expr, Column) else None for p in projections]
        else:
            out_types = [c.data_type for c in cols]
            src_cols = list(range(len(cols)))
        outs, keeps = [], []
        for o, t in enumerate(out_types):
            passthrough = predicate is None and src_cols[o] is not None
            if passthrough:
                outs.append(_abi.dfmi_out_column())
                keeps.append({})
                continue
            cap = 0
            if t == DataType.Utf8 and src_cols[o] is not None:
                cap = cols[src_cols[o]].values.numel()
            # validity: always without a predicate; after one, a projection
            # with a fallible CAST can still produce nulls
            oc, keep = self._alloc_out(t, n, t != DataType.Utf8, cap)
            outs.append(oc)
            keeps.append(keep)
        return out_types, outs, keeps

    @staticmethod
    def _results(out_types, outs, keeps, cols) -> List[Array]:
        result = []
        for o, t in enumerate(out_types):
            oc = outs[o]
            if oc.passthrough_column >= 0:
                result.append(cols[oc.passthrough_column])
                continue
            k = keeps[o]
            length = oc.length
            nulls = oc.null_count
            if t == DataType.Utf8:
                result.append(Array(t, length, k["data"], None, k["offsets"], 0))
            else:
                result.append(Array(t, length, k["values"], k.get("validity") if nulls else None, None, nulls))
        return result

    def filter_project_batches(self, predicate, projections: Optional[Sequence], batches: Sequence[RecordBatch],
                               flags: int = 0):
        """The pull of filter_project on each batch, in order, as ONE device
        launch (dfmi_filter_project_batches). Returns (results, error):
        results holds one column list per batch before the first failing
        batch (all of them when error is None) -- what a pull loop would have
        received before the error."""
        self.drain()
        L = _abi.lib()
        projections = list(projections or [])
        batches = [self.to_device(b) for b in batches]
        nb = len(batches)
        if nb == 0:
            return [], None
        per, cstructs = [], []
        for b in batches:
            cols = b.columns
            carr = (_abi.dfmi_column * max(1, len(cols)))()
            for i, a in enumerate(cols):
                carr[i] = column_struct(a)
            cstructs.append(carr)
            per.append(self._prepare_outputs(predicate, projections, cols, b.num_rows()))
        nout = len(per[0][0])
        cb = (_abi.dfmi_batch * nb)()
        for i, b in enumerate(batches):
            cb[i].num_columns = len(b.columns)
            cb[i].num_rows = b.num_rows()
            cb[i].columns = cstructs[i]
        outs = (_abi.dfmi_out_column * max(1, nb * nout))()
        for i in range(nb):
            for o in range(nout):
                outs[i * nout + o] = per[i][1][o]
        progs = (C.c_void_p * max(1, len(projections)))(*[p.handle.value for p in projections])
        err = _abi.dfmi_error()
        failed = C.c_int32(-1)
        L.dfmi_context_set_stream(self.ctx, C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream))
        rc = L.dfmi_filter_project_batches(self.ctx, predicate.handle if predicate is not None else None, progs,
                                           len(projections), cb, nb, outs, flags, C.byref(failed), C.byref(err))
        error = None
        done = nb
        if rc != _abi.DFMI_OK:
            error = ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
            key = C.c_uint64()
            L.dfmi_last_error_order(self.ctx, C.byref(key))
            error.order_key = key.value
            done = max(failed.value, 0)
            error.failed_batch = failed.value
        results = []
        for i in range(done):
            results.append(self._results(per[i][0], [outs[i * nout + o] for o in range(nout)], per[i][2],
                                         batches[i].columns))
        return results, error

    def filter_project_host(self, predicate, projections: Optional[Sequence], batch: RecordBatch,
                            flags: int = 0) -> List[Array]:
        """The same pull over a HOST batch through dfmi_filter_project_host:
        the library stages the Arrow buffers into HBM and returns host
        results (the path a Rust caller with arrow 0.12 buffers takes)."""
        self.drain()
        L = _abi.lib()
        cols = batch.columns
        if any(c.values.device.type != "cpu" for c in cols):
            raise ValueError("filter_project_host takes a host batch")
        projections = list(projections or [])
        carr = (_abi.dfmi_column * max(1, len(cols)))()
        for i, a in enumerate(cols):
            carr[i] = column_struct(a)
        cb = _abi.dfmi_batch()
        cb.num_columns = len(cols)
        cb.num_rows = batch.num_rows()
        cb.columns = carr
        progs = (C.c_void_p * max(1, len(projections)))(*[p.handle.value for p in projections])
        err = _abi.dfmi_error()
        res = C.c_void_p()
        L.dfmi_context_set_stream(self.ctx, C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream))
        rc = L.dfmi_filter_project_host(self.ctx, predicate.handle if predicate is not None else None,
                                        progs, len(projections), C.byref(cb), flags, C.byref(res), C.byref(err))
        if rc != _abi.DFMI_OK:
            raise ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
        # views into the result's pinned block where it has one (a small call:
        # no copy), copies of its per-column buffers otherwise; the result is
        # freed with the last view
        n = L.dfmi_host_result_num_columns(res)
        if n == 0:
            L.dfmi_host_result_free(res)
            return []
        return HostBatchColumns(HostResultBlock(res, n, n), 0, n).materialize()

    def filter_project_host_batches(self, predicate, projections: Optional[Sequence], batches: Sequence[RecordBatch],
                                    flags: int = 0):
        """The pull over many small HOST batches in one call
        (dfmi_filter_project_host_batches): (one output column set per batch
        up to the failing one, the error or None) -- the pull loop's view.
        Each column set is a HostBatchColumns: the batch's buffers are slices
        of the result's one pinned block (no copy), its Arrays are built when
        first read, and the block is released when the last slice is."""
        self.drain()
        prep = self._host_batches_prepare(predicate, projections, batches, flags)
        return self._host_batches_finish(prep, self._host_batches_call(prep))

    def filter_project_host_batches_async(self, predicate, projections: Optional[Sequence],
                                          batches: Sequence[RecordBatch], flags: int = 0,
                                          schema: Schema = None, start: bool = True) -> "HostBatchesCall":
        """filter_project_host_batches whose C call runs on the engine's worker
        thread (ctypes releases the GIL for it): the caller hands out the
        previous group's batches while this group's staging, PCIe copies and
        launch proceed. The batches' structs are built here, on the calling
        thread; result() gives what filter_project_host_batches returns -- or,
        with `schema`, the output RecordBatches themselves. With `schema` the
        outputs land in ONE block this binding owns
        (dfmi_filter_project_host_batches_into) -- pinned, so the kernel writes
        it in place -- and the glue builds the group's RecordBatches of
        BlockArrays over it in one native call. start=False prepares the call
        (structs, block) without running it: submit() starts it, so a relation
        can prepare group g+2 while g+1 runs and start it the moment g+1 ends.
        The engine runs one call at a time: submit() and every other entry
        point wait for an in-flight one first (drain)."""
        if start:
            self.drain()
        prep = self._host_batches_prepare(predicate, projections, batches, flags)
        into = self._host_batches_block(prep) if schema is not None and prep[5] else None
        call = HostBatchesCall(self, prep, schema, into)
        return call.submit() if start else call

    def drain(self) -> None:
        """Wait for the in-flight asynchronous call (its result stays with its future)."""
        f = self._inflight
        if f is not None:
            self._inflight = None
            from concurrent.futures import wait
            wait([f])

    def _host_batches_prepare(self, predicate, projections, batches, flags):
        projections = list(projections or [])
        nb = len(batches)
        ncols = batches[0].num_columns() if nb else 0
        nout = len(projections) if projections else ncols
        barr, keep = host_batch_structs(batches, ncols) if nb else (None, None)
        progs = (C.c_void_p * max(1, len(projections)))(*[p.handle.value for p in projections])
        stream = torch.cuda.current_stream(self.device).cuda_stream  # the caller's stream (thread-local in torch)
        # `batches` rides along: the structs hold raw pointers into their
        # buffers, so the call in flight keeps the batches alive itself
        return (predicate.handle if predicate is not None else None, progs, len(projections), barr, keep, nb, nout,
                flags, stream, list(batches))

    def _host_batches_block(self, prep):
        """(block, outs) of a caller-owned call: a pinned host block of the
        worst-case output size (dfmi_host_batches_output_bytes) from the
        pinned block pool, and the dfmi_out_column records to fill."""
        pred, progs, np_, barr, keep, nb, nout, flags = prep[:8]
        L = _abi.lib()
        size = C.c_size_t()
        err = _abi.dfmi_error()
        rc = L.dfmi_host_batches_output_bytes(pred, progs, np_, C.cast(barr, C.c_void_p), nb, flags, C.byref(size),
                                              C.byref(err))
        if rc != _abi.DFMI_OK:
            raise ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
        block = _PINNED.get(max(size.value, 64))
        return block, np.zeros(max(1, nb * nout), dtype=_OUT_DTYPE)

    def _host_batches_into_call(self, prep, into):
        """dfmi_filter_project_host_batches_into (any thread): (rc, failed batch, dfmi_error)."""
        pred, progs, np_, barr, keep, nb, nout, flags, stream = prep[:9]
        block, outs = into
        L = _abi.lib()
        err = _abi.dfmi_error()
        failed = C.c_int32(-1)
        L.dfmi_context_set_stream(self.ctx, C.c_void_p(stream))
        rc = L.dfmi_filter_project_host_batches_into(self.ctx, pred, progs, np_, C.cast(barr, C.c_void_p), nb, flags,
                                                     block.data_ptr(), block.numel(), outs.ctypes.data,
                                                     C.byref(failed), C.byref(err))
        return rc, failed.value, err

    @staticmethod
    def _host_batches_into_finish(prep, raw, schema, into):
        nb, nout, batches = prep[5], prep[6], prep[9]
        rc, failed, err = raw
        error = None
        if rc != _abi.DFMI_OK:
            error = ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
            error.failed_batch = failed
            if failed < 0:  # nothing ran (arguments, capacity)
                raise error
        done = nb if error is None else max(0, failed)
        from .. import _dfmi_glue
        from ..arrow import BlockArray
        block, outs = into
        return _dfmi_glue.make_block_batches(RecordBatch, BlockArray, schema, block, outs, done, nout, batches,
                                             _DTYPES), error

    def _host_batches_call(self, prep):
        """The C call (any thread): (rc, result handle, failed batch, dfmi_error)."""
        pred, progs, np_, barr, keep, nb, nout, flags, stream = prep[:9]
        if nb == 0:
            return _abi.DFMI_OK, None, -1, None
        L = _abi.lib()
        err = _abi.dfmi_error()
        res = C.c_void_p()
        failed = C.c_int32(-1)
        L.dfmi_context_set_stream(self.ctx, C.c_void_p(stream))
        rc = L.dfmi_filter_project_host_batches(self.ctx, pred, progs, np_, barr, nb, flags, C.byref(res),
                                                C.byref(failed), C.byref(err))
        return rc, res, failed.value, err

    @staticmethod
    def _host_batches_finish(prep, raw, schema=None):
        nb, nout = prep[5], prep[6]
        rc, res, failed, err = raw
        if nb == 0:
            return [], None
        error = None
        if rc != _abi.DFMI_OK:
            error = ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
            error.failed_batch = failed
            if not res.value:
                raise error
        done = nb if error is None else max(0, failed)
        block = HostResultBlock(res, done * nout, nout)
        if schema is not None:
            return [HostResultBatch.make(schema, block, b, nout) for b in range(done)], error
        return [HostBatchColumns(block, b, nout) for b in range(done)], error

    # ---- aggregate extension (DFMI_FLAG_EXT_AGGREGATE)
    def _batch_struct(self, batch: RecordBatch):
        cols = batch.columns
        carr = (_abi.dfmi_column * max(1, len(cols)))()
        for i, a in enumerate(cols):
            carr[i] = column_struct(a)
        cb = _abi.dfmi_batch()
        cb.num_columns = len(cols)
        cb.num_rows = batch.num_rows()
        cb.columns = carr
        return cb, carr

    def agg_state(self, aggs: Sequence) -> "AggState":
        """Device accumulators for one Aggregate plan (dfmi_agg_state_create)."""
        return AggState(self, aggs)

    def grouped_agg_state(self, key, aggs: Sequence) -> "GroupedAggState":
        """Device accumulators for one Aggregate plan with a GROUP BY key, or
        a list of 1-4 keys (dfmi_agg_state_create_grouped_multi)."""
        return GroupedAggState(self, key, aggs)


class AggState:
    """dfmi_agg_state: accumulates batches of one Aggregate plan on one GPU."""

    def __init__(self, eng: DeviceEngine, aggs: Sequence, key=None):
        self.eng = eng
        self.aggs = list(aggs)
        self.key = key
        L = _abi.lib()
        arr = (C.c_void_p * len(self.aggs))(*[a.handle.value for a in self.aggs])
        out = C.c_void_p()
        err = _abi.dfmi_error()
        if key is None:
            rc = L.dfmi_agg_state_create(eng.ctx, arr, len(self.aggs), C.byref(out), C.byref(err))
        elif isinstance(key, (list, tuple)):
            karr = (C.c_void_p * len(key))(*[k.handle.value for k in key])
            rc = L.dfmi_agg_state_create_grouped_multi(eng.ctx, karr, len(key), arr, len(self.aggs), C.byref(out),
                                                       C.byref(err))
        else:
            rc = L.dfmi_agg_state_create_grouped(eng.ctx, key.handle, arr, len(self.aggs), C.byref(out), C.byref(err))
        if rc != _abi.DFMI_OK:
            raise ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
        self.handle = out

    def add(self, predicate, batch: RecordBatch, flags: int = 0) -> None:
        """One batch of the aggregate's input (fused Selection when predicate is given)."""
        eng = self.eng
        eng.drain()
        batch = eng.to_device(batch)
        cb, keep = eng._batch_struct(batch)
        err = _abi.dfmi_error()
        L = _abi.lib()
        L.dfmi_context_set_stream(eng.ctx, C.c_void_p(torch.cuda.current_stream(eng.device).cuda_stream))
        rc = L.dfmi_aggregate_batch(eng.ctx, self.handle, predicate.handle if predicate is not None else None,
                                    C.byref(cb), flags, C.byref(err))
        if rc != _abi.DFMI_OK:
            raise ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))

    def reset(self) -> None:
        self.eng.drain()
        err = _abi.dfmi_error()
        rc = _abi.lib().dfmi_agg_state_reset(self.eng.ctx, self.handle, C.byref(err))
        if rc != _abi.DFMI_OK:
            raise ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))

    def finish(self) -> List[_abi.dfmi_agg_value]:
        self.eng.drain()
        out = (_abi.dfmi_agg_value * len(self.aggs))()
        err = _abi.dfmi_error()
        rc = _abi.lib().dfmi_agg_state_finish(self.eng.ctx, self.handle, out, C.byref(err))
        if rc != _abi.DFMI_OK:
            raise ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
        return list(out)

    def partial(self) -> bytes:
        """The exact partial state (for merging shards: dfmi_agg_merge_partials)."""
        self.eng.drain()
        L = _abi.lib()
        nb = L.dfmi_agg_partial_bytes(self.handle)
        buf = C.create_string_buffer(nb)
        err = _abi.dfmi_error()
        rc = L.dfmi_agg_state_partial(self.eng.ctx, self.handle, buf, C.byref(err))
        if rc != _abi.DFMI_OK:
            raise ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
        return buf.raw

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                _abi.lib().dfmi_agg_state_free(h)
            except Exception:
                pass
            self.handle = C.c_void_p(0)


class GroupedAggState(AggState):
    """dfmi_agg_state with GROUP BY keys: finish() returns (keys, values) --
    per group in key order (null last, per key part) its key -- one
    dfmi_agg_value for a single key expression, a list of one per key part
    for several (`key` given as a list) -- and its aggregate values."""

    def __init__(self, eng: DeviceEngine, key, aggs: Sequence):
        super().__init__(eng, aggs, key)
        self.multi = isinstance(key, (list, tuple))
        self.nkeys = len(key) if self.multi else 1

    def finish(self):
        self.eng.drain()
        self._last = _grouped_call(len(self.aggs), lambda cap, keys, vals, ng, err: _abi.lib().dfmi_agg_state_finish_grouped(
            self.eng.ctx, self.handle, cap, keys, vals, ng, err), self.nkeys, self.multi)
        return self._last

    def key_strings(self, part: int = 0) -> List[Optional[bytes]]:
        """The Utf8 key part `part` of the groups of the last finish(), in its
        order (None for a null key): dfmi_agg_state_group_keys_utf8_part."""
        self.eng.drain()
        L = _abi.lib()
        err = _abi.dfmi_error()
        ln = C.c_int64()
        L.dfmi_agg_state_group_keys_utf8_part(self.handle, part, None, 0, None, 0, C.byref(ln), C.byref(err))
        keys, _ = self._last
        offs = np.zeros(len(keys) + 1, np.int32)
        data = np.zeros(max(1, ln.value), np.uint8)
        rc = L.dfmi_agg_state_group_keys_utf8_part(self.handle, part, offs.ctypes.data, offs.size, data.ctypes.data,
                                                   data.size, C.byref(ln), C.byref(err))
        if rc != _abi.DFMI_OK:
            raise ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
        nulls = [(k[part] if self.multi else k).is_null for k in keys]
        return [None if nulls[g] else bytes(data[offs[g]:offs[g + 1]]) for g in range(len(keys))]

    def partial(self) -> bytes:
        """The exact per-group partial state (dfmi_agg_state_grouped_partial)."""
        self.eng.drain()
        L = _abi.lib()
        err = _abi.dfmi_error()
        nb = L.dfmi_agg_state_grouped_partial_bytes(self.eng.ctx, self.handle, C.byref(err))
        if nb < 0:
            raise ExecutionError.from_status(int(-nb), err.message.decode("utf-8", errors="replace"))
        buf = C.create_string_buffer(max(int(nb), 1))
        rc = L.dfmi_agg_state_grouped_partial(self.eng.ctx, self.handle, buf, nb, C.byref(err))
        if rc != _abi.DFMI_OK:
            raise ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
        return buf.raw[:nb]


_AGG_VALUE = np.dtype([("type", "<i4"), ("is_null", "<i4"), ("count", "<i8"), ("bits", "<u8")])


def _grouped_call(n: int, fn, nkeys: int = 1, multi: bool = False):
    """(keys, per-group values) from a grouped finish entry point, growing
    the capacity to the group count it reports. Numpy record arrays over the
    dfmi_agg_value layout (`k.bits`, `k.is_null`, ... per element): keys one
    record per group, or (multi) a row of nkeys records; values a row of n
    records per group."""
    ng = C.c_int64()
    err = _abi.dfmi_error()
    cap = 64
    PV = C.POINTER(_abi.dfmi_agg_value)
    while True:
        keys = np.zeros(max(cap * nkeys, 1), _AGG_VALUE)
        vals = np.zeros(max(cap * n, 1), _AGG_VALUE)
        rc = fn(cap, keys.ctypes.data_as(PV), vals.ctypes.data_as(PV), C.byref(ng), C.byref(err))
        if rc == _abi.DFMI_ERR_INVALID_ARGUMENT and ng.value > cap:
            cap = ng.value
            continue
        if rc != _abi.DFMI_OK:
            raise ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
        g = ng.value
        kr = keys[: g * nkeys].view(np.recarray)
        return (kr.reshape(g, nkeys) if multi else kr), vals[: g * n].view(np.recarray).reshape(g, n)


def merge_grouped_partials(aggs: Sequence, partials: Sequence[bytes], nkeys: int = 1, multi: bool = False):
    """Every shard's per-group partial merged: (keys, per-group values)."""
    arr = (C.c_void_p * len(aggs))(*[a.handle.value for a in aggs])
    bufs = [C.create_string_buffer(p, len(p)) for p in partials]
    parr = (C.c_void_p * len(bufs))(*[C.addressof(b) for b in bufs])
    sizes = (C.c_int64 * len(bufs))(*[len(p) for p in partials])
    return _grouped_call(len(aggs), lambda cap, keys, vals, ng, err: _abi.lib().dfmi_agg_merge_grouped_partials(
        arr, len(aggs), parr, sizes, len(bufs), cap, keys, vals, ng, err), nkeys, multi)


def merge_grouped_partials_key_strings(aggs: Sequence, partials: Sequence[bytes], part: int, num_groups: int):
    """The Utf8 key part `part` of the merged groups (merge_grouped_partials'
    order): dfmi_agg_merge_grouped_partials_keys_utf8 (null keys: b'')."""
    L = _abi.lib()
    arr = (C.c_void_p * len(aggs))(*[a.handle.value for a in aggs])
    bufs = [C.create_string_buffer(p, len(p)) for p in partials]
    parr = (C.c_void_p * len(bufs))(*[C.addressof(b) for b in bufs])
    sizes = (C.c_int64 * len(bufs))(*[len(p) for p in partials])
    err = _abi.dfmi_error()
    ln = C.c_int64()
    L.dfmi_agg_merge_grouped_partials_keys_utf8(arr, len(aggs), parr, sizes, len(bufs), part, None, 0, None, 0,
                                                C.byref(ln), C.byref(err))
    offs = np.zeros(num_groups + 1, np.int32)
    data = np.zeros(max(1, ln.value), np.uint8)
    rc = L.dfmi_agg_merge_grouped_partials_keys_utf8(arr, len(aggs), parr, sizes, len(bufs), part, offs.ctypes.data,
                                                     offs.size, data.ctypes.data, data.size, C.byref(ln), C.byref(err))
    if rc != _abi.DFMI_OK:
        raise ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
    return [bytes(data[offs[g]:offs[g + 1]]) for g in range(num_groups)]


def merge_agg_partials(aggs: Sequence, partials: Sequence[bytes]) -> List[_abi.dfmi_agg_value]:
    """Final values from every shard's exact partial state (host merge)."""
    arr = (C.c_void_p * len(aggs))(*[a.handle.value for a in aggs])
    bufs = [C.create_string_buffer(p, len(p)) for p in partials]
    parr = (C.c_void_p * len(bufs))(*[C.addressof(b) for b in bufs])
    out = (_abi.dfmi_agg_value * len(aggs))()
    err = _abi.dfmi_error()
    rc = _abi.lib().dfmi_agg_merge_partials(arr, len(aggs), parr, len(bufs), out, C.byref(err))
    if rc != _abi.DFMI_OK:
        raise ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
    return list(out)


class ShardComm:
    """dfmi_shard_comm: the RCCL communicator of the C-ABI multi-GPU entry
    points (include/dfmi.h "Multi-GPU"), one per rank."""

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(_abi.DFMI_SHARD_ID_BYTES)
        err = _abi.dfmi_error()
        rc = _abi.lib().dfmi_shard_unique_id(buf, C.byref(err))
        if rc != _abi.DFMI_OK:
            raise ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
        return buf.raw

    def __init__(self, eng: DeviceEngine, world: int, rank: int, uid: bytes):
        eng.drain()
        self.eng = eng
        self.world, self.rank = world, rank
        out = C.c_void_p()
        err = _abi.dfmi_error()
        idb = C.create_string_buffer(uid, _abi.DFMI_SHARD_ID_BYTES)
        rc = _abi.lib().dfmi_shard_comm_init(eng.ctx, world, rank, idb, C.byref(out), C.byref(err))
        if rc != _abi.DFMI_OK:
            raise ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
        self.handle = out
        self.placement = None
        self.outputs = None
        self.keep = None

    @classmethod
    def loopback(cls, eng: DeviceEngine, group, rank: int) -> "ShardComm":
        """Test-only communicator: `rank` of a loopback group of host threads
        sharing one device (csrc/shard.cpp LoopTransport), so the shard entry
        points run at world sizes > 1 on a one-GPU box."""
        L = _abi.lib()
        fn = L.dfmi_internal_shard_comm_loopback
        fn.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(C.c_void_p), C.POINTER(_abi.dfmi_error)]
        fn.restype = C.c_int32
        eng.drain()
        self = cls.__new__(cls)
        self.eng = eng
        self.world, self.rank = None, rank
        out = C.c_void_p()
        err = _abi.dfmi_error()
        rc = fn(eng.ctx, group, rank, C.byref(out), C.byref(err))
        if rc != _abi.DFMI_OK:
            raise ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
        self.handle = out
        self.placement = None
        self.outputs = None
        self.keep = None
        return self

    def gather_to_root(self, cols: List[Array], root: int = 0) -> Optional[List[Array]]:
        """The last shard pass's outputs concatenated on `root` (collective)."""
        self.eng.drain()
        place = self.placement
        n = place.total_rows
        L = _abi.lib()
        routs = (_abi.dfmi_out_column * max(1, len(cols)))()
        keeps = []
        if self.rank == root:
            for o, a in enumerate(cols):
                oc, keep = self.eng._alloc_out(a.data_type, n, bool(place.null_total[o]), int(place.utf8_total[o]))
                routs[o] = oc
                keeps.append(keep)
        err = _abi.dfmi_error()
        rc = L.dfmi_shard_gather_to_root(self.eng.ctx, self.handle, self.outputs, routs, root, C.byref(err))
        if rc != _abi.DFMI_OK:
            raise ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
        if self.rank != root:
            return None
        out = []
        for o, a in enumerate(cols):
            k = keeps[o]
            if a.data_type == DataType.Utf8:
                out.append(Array(a.data_type, n, k["data"], None, k["offsets"], 0))
            else:
                nulls = int(place.null_total[o])
                out.append(Array(a.data_type, n, k["values"], k.get("validity") if nulls else None, None, nulls))
        return out

    def agg_finish(self, state: "AggState") -> List[_abi.dfmi_agg_value]:
        """Every rank's exact aggregate partial merged (collective)."""
        self.eng.drain()
        arr = (C.c_void_p * len(state.aggs))(*[a.handle.value for a in state.aggs])
        out = (_abi.dfmi_agg_value * len(state.aggs))()
        err = _abi.dfmi_error()
        rc = _abi.lib().dfmi_shard_agg_finish(self.eng.ctx, self.handle, state.handle, arr, len(state.aggs), out,
                                              C.byref(err))
        if rc != _abi.DFMI_OK:
            raise ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
        return list(out)

    def agg_finish_grouped(self, state: "GroupedAggState"):
        """Every rank's per-group partials merged (collective): (keys, values);
        state.key_strings() then reads the merged groups' Utf8 keys."""
        self.eng.drain()
        arr = (C.c_void_p * len(state.aggs))(*[a.handle.value for a in state.aggs])
        state._last = _grouped_call(len(state.aggs), lambda cap, keys, vals, ng, err: _abi.lib().dfmi_shard_agg_finish_grouped(
            self.eng.ctx, self.handle, state.handle, arr, len(state.aggs), cap, keys, vals, ng, err), state.nkeys,
            state.multi)
        return state._last

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                _abi.lib().dfmi_shard_comm_destroy(h)
            except Exception:
                pass
            self.handle = C.c_void_p(0)


# ---- host batches: vectorised ABI structs in, zero-copy result slices out

_COL_DTYPE = np.dtype([("type", "<i4"), ("reserved", "<i4"), ("length", "<i8"), ("null_count", "<i8"),
                       ("validity", "<u8"), ("values", "<u8"), ("offsets", "<u8"), ("offset", "<i8")])
_BATCH_DTYPE = np.dtype([("num_columns", "<i4"), ("reserved", "<i4"), ("num_rows", "<i8"), ("columns", "<u8")])
_OUT_DTYPE = np.dtype([("values", "<u8"), ("validity", "<u8"), ("offsets", "<u8"), ("data", "<u8"),
                       ("data_capacity", "<i8"), ("type", "<i4"), ("passthrough_column", "<i4"), ("length", "<i8"),
                       ("null_count", "<i8"), ("data_length", "<i8")])
assert _COL_DTYPE.itemsize == C.sizeof(_abi.dfmi_column) and _BATCH_DTYPE.itemsize == C.sizeof(_abi.dfmi_batch)
assert _OUT_DTYPE.itemsize == C.sizeof(_abi.dfmi_out_column)
_DTYPES = [DataType(i) for i in range(13)]  # dfmi_type -> DataType (the glue's output types)


def host_batch_structs(batches: Sequence[RecordBatch], ncols: int):
    """dfmi_batch[len(batches)] over the batches' host buffers, filled by the
    native glue (csrc/pyglue.c: the fields column_struct() reads, for every
    column of every batch, in one call). Returns (batch array, keep-alive)."""
    from .. import _dfmi_glue
    nb = len(batches)
    cols = np.empty(max(1, nb * ncols), dtype=_COL_DTYPE)
    ba = np.empty(nb, dtype=_BATCH_DTYPE)
    _dfmi_glue.pack_host_batches(batches, ncols, cols, ba)
    return (_abi.dfmi_batch * nb).from_buffer(ba), (cols, ba)


class _PinnedOwner:
    """The numpy view over one pooled pinned block: torch.from_numpy keeps
    this array (and so this owner) alive as long as any tensor over the
    block's memory lives; then the block goes back to the pool."""

    __slots__ = ("pool", "cls", "base", "__array_interface__", "__weakref__")

    def __init__(self, pool, cls, base, size):
        self.pool, self.cls, self.base = pool, cls, base
        self.__array_interface__ = {"shape": (size,), "typestr": "|u1", "data": (base.data_ptr(), False),
                                    "version": 3}

    def __del__(self):
        try:
            self.pool.put(self.cls, self.base)
        except Exception:  # interpreter shutdown
            pass


class _PinnedPool:
    """Pinned host blocks for the caller-owned host-batches calls, reused
    instead of a torch pinned allocation per call (~60 us each on the GPU
    box, a quarter of a 256-batch group's main-thread time): power-of-two
    size classes, a few free blocks kept per class. DFMI_PY_PINNED_POOL=0:
    a fresh torch pinned tensor per call (A/B)."""

    def __init__(self, keep: int = 6):
        import os
        import threading
        self.keep, self.free, self.lock = keep, {}, threading.Lock()
        self.on = os.environ.get("DFMI_PY_PINNED_POOL", "1") != "0"

    def get(self, size: int) -> torch.Tensor:
        if not self.on:
            return torch.empty(size, dtype=torch.uint8, pin_memory=True)
        cls = max(1 << 16, 1 << (size - 1).bit_length())
        with self.lock:
            lst = self.free.get(cls)
            base = lst.pop() if lst else None
        if base is None:
            base = torch.empty(cls, dtype=torch.uint8, pin_memory=True)
        return torch.from_numpy(np.asarray(_PinnedOwner(self, cls, base, size)))

    def put(self, cls: int, base: torch.Tensor) -> None:
        with self.lock:
            lst = self.free.setdefault(cls, [])
            if len(lst) < self.keep:
                lst.append(base)


_PINNED = _PinnedPool()


class HostBatchesCall:
    """One filter_project_host_batches_async call: prepared, then submitted
    to the engine's worker thread, then finished on the caller's thread."""

    __slots__ = ("eng", "prep", "schema", "into", "fut", "raw")

    def __init__(self, eng: DeviceEngine, prep, schema=None, into=None):
        self.eng, self.prep, self.schema, self.into = eng, prep, schema, into
        self.fut = self.raw = None

    def submit(self) -> "HostBatchesCall":
        eng = self.eng
        eng.drain()
        if eng._worker is None:
            from concurrent.futures import ThreadPoolExecutor
            eng._worker = ThreadPoolExecutor(max_workers=1, thread_name_prefix="dfmi-engine")
        if self.into is not None:
            self.fut = eng._worker.submit(eng._host_batches_into_call, self.prep, self.into)
        else:
            self.fut = eng._worker.submit(eng._host_batches_call, self.prep)
        eng._inflight = self.fut
        return self

    def wait(self) -> bool:
        """Wait for the call; True when every batch ran without an error."""
        if self.raw is None:
            if self.fut is None:
                self.submit()
            self.raw = self.fut.result()
            if self.eng._inflight is self.fut:
                self.eng._inflight = None
        return self.raw[0] == _abi.DFMI_OK

    def result(self):
        self.wait()
        if self.into is not None:
            return DeviceEngine._host_batches_into_finish(self.prep, self.raw, self.schema, self.into)
        return DeviceEngine._host_batches_finish(self.prep, self.raw, self.schema)


HostBatchesFuture = HostBatchesCall  # (the name of round 4)


class _ResultOwner:
    """Frees a dfmi_host_result when the last view of its memory is gone."""

    def __init__(self, res):
        self.res = res

    def __del__(self):
        try:
            _abi.lib().dfmi_host_result_free(self.res)
        except Exception:
            pass


class HostResultBlock:
    """One coalesced host result: every column's view (dfmi_host_result_columns,
    one FFI call) and its pinned block as one uint8 tensor. Slices of that
    tensor keep the result alive."""

    def __init__(self, res, ncols: int, nout: int = 0):
        L = _abi.lib()
        owner = _ResultOwner(res)
        views = np.zeros(max(1, ncols), dtype=_COL_DTYPE)
        if ncols:
            L.dfmi_host_result_columns(res, 0, ncols, views.ctypes.data)
        if nout and ncols % nout == 0:  # batch after batch of the same nout output types
            self.type = [DataType(t) for t in views["type"][:nout].tolist()] * (ncols // nout)
        else:
            self.type = [DataType(t) for t in views["type"].tolist()]
        self.length = views["length"].tolist()
        self.nulls = views["null_count"].tolist()
        self.validity = views["validity"].tolist()
        self.values = views["values"].tolist()
        self.offsets = views["offsets"].tolist()
        base, nbytes = C.c_void_p(), C.c_size_t()
        L.dfmi_host_result_block(res, C.byref(base), C.byref(nbytes))
        self.base = base.value or 0
        self.end = self.base + nbytes.value
        if self.base:
            raw = (C.c_uint8 * nbytes.value).from_address(self.base)
            raw._owner = owner  # the memory lives while any tensor over `raw` does
            self.block = torch.from_numpy(np.frombuffer(raw, dtype=np.uint8))
        else:
            self.block = None
        self.owner = owner

    def buffer(self, ptr: int, nbytes: int) -> torch.Tensor:
        """Host tensor of nbytes at ptr: a slice of the block (no copy), or a
        copy for memory outside it (passthrough columns)."""
        from ..arrow import _bytes_tensor
        if self.base <= ptr and ptr + nbytes <= self.end:
            # padded to 64 bytes like every Array buffer (the block's buffers
            # are 256-byte aligned, so the padding stays inside this one)
            o = ptr - self.base
            return self.block[o:min(o + max(64, (nbytes + 63) & ~63), self.end - self.base)]
        if not nbytes:
            return torch.zeros(64, dtype=torch.uint8)
        return _bytes_tensor(np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint8)), shape=(nbytes,)).copy())


class HostBatchColumns(LazyColumns):
    """The output columns of batch b of a HostResultBlock."""

    __slots__ = ("blk", "b", "num_columns", "_cols")

    def __init__(self, blk: HostResultBlock, b: int, nout: int):
        self.blk, self.b, self.num_columns, self._cols = blk, b, nout, None

    @property
    def num_rows(self) -> int:
        return self.blk.length[self.b * self.num_columns] if self.num_columns else 0

    def materialize(self) -> List[Array]:
        if self._cols is None:
            self._cols = self._build()
        return self._cols

    def _build(self) -> List[Array]:
        k = self.blk
        out = []
        for i in range(self.b * self.num_columns, (self.b + 1) * self.num_columns):
            t = k.type[i]
            n = k.length[i]
            nulls = k.nulls[i]
            valid = k.buffer(k.validity[i], (n + 7) // 8) if (nulls and k.validity[i]) else None
            if t == DataType.Utf8:
                offs = k.buffer(k.offsets[i], 4 * (n + 1)).view(torch.int32)
                nbytes = int(offs[n]) if n else 0  # (a passthrough slice's offsets need not start at 0)
                vals = k.buffer(k.values[i], nbytes)
                out.append(Array(t, n, vals, valid, offs, nulls))
                continue
            nb = (n + 7) // 8 if t == DataType.Boolean else n * t.width
            vals = k.buffer(k.values[i], nb)
            out.append(Array(t, n, vals, valid, None, nulls))
        return out


class HostResultBatch(RecordBatch):
    """Output batch b of a HostResultBlock as the RecordBatch itself (the
    relations' pull loop over host batches: one Python object per pulled
    batch). Its Arrays are built when first read (HostBatchColumns)."""

    @classmethod
    def make(cls, schema, blk: "HostResultBlock", b: int, nout: int) -> "HostResultBatch":
        r = object.__new__(cls)
        r.schema, r._blk, r._b, r._n, r._cols = schema, blk, b, nout, None
        return r

    @property
    def _columns(self) -> List[Array]:
        c = self._cols
        if c is None:
            c = self._cols = HostBatchColumns(self._blk, self._b, self._n).materialize()
        return c

    @_columns.setter
    def _columns(self, cols) -> None:
        self._cols = list(cols)

    def num_columns(self) -> int:
        return self._n if self._cols is None else len(self._cols)

    def num_rows(self) -> int:
        if self._cols is not None:
            return self._cols[0].length if self._cols else 0
        return self._blk.length[self._b * self._n] if self._n else 0
