"""Test-only bridge to the CPU oracle (oracle/liboracle.so). The oracle is the
checker: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline use it."""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import List, Optional, Sequence

import numpy as np
import torch

from datafusion_amd import _abi
from datafusion_amd.arrow import Array, Field, RecordBatch, Schema, _bytes_tensor, _offsets_tensor, pack_bits, unpack_bits
from datafusion_amd.logicalplan import DataType, Expr
from datafusion_amd.execution.error import ExecutionError

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")
_L = None


def oracle_lib() -> C.CDLL:
    global _L
    if _L is not None:
        return _L
    if not os.path.exists(ORACLE_SO):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    L = C.CDLL(ORACLE_SO)
    P = C.POINTER
    L.oracle_filter_project.argtypes = [P(_abi.dfmi_expr_node), C.c_int32, P(P(_abi.dfmi_expr_node)),
                                        P(C.c_int32), C.c_int32, P(_abi.dfmi_schema), P(_abi.dfmi_batch),
                                        C.c_uint32, P(C.c_void_p), P(_abi.dfmi_error)]
    L.oracle_filter_project.restype = C.c_int32
    L.oracle_run_batched.argtypes = [P(_abi.dfmi_expr_node), C.c_int32, P(P(_abi.dfmi_expr_node)),
                                     P(C.c_int32), C.c_int32, P(_abi.dfmi_schema), P(_abi.dfmi_batch),
                                     C.c_int64, C.c_uint32, P(C.c_int64), P(_abi.dfmi_error)]
    L.oracle_run_batched.restype = C.c_int32
    L.oracle_result_num_columns.argtypes = [C.c_void_p]
    L.oracle_result_num_columns.restype = C.c_int32
    L.oracle_result_column.argtypes = [C.c_void_p, C.c_int32, P(_abi.dfmi_column), P(C.c_char_p)]
    L.oracle_result_column.restype = C.c_int32
    L.oracle_result_free.argtypes = [C.c_void_p]
    L.oracle_compile_info.argtypes = [P(_abi.dfmi_expr_node), C.c_int32, P(_abi.dfmi_schema), C.c_uint32,
                                      C.c_char_p, C.c_int64, P(C.c_int32), P(_abi.dfmi_error)]
    L.oracle_compile_info.restype = C.c_int32
    L.oracle_aggregate.argtypes = [P(_abi.dfmi_expr_node), C.c_int32, P(C.c_char_p), P(P(_abi.dfmi_expr_node)),
                                   P(C.c_int32), P(C.c_int32), C.c_int32, P(_abi.dfmi_schema), P(_abi.dfmi_batch),
                                   C.c_int64, C.c_uint32, P(_abi.dfmi_agg_value), P(_abi.dfmi_error)]
    L.oracle_aggregate.restype = C.c_int32
    L.oracle_aggregate_grouped.argtypes = [P(_abi.dfmi_expr_node), C.c_int32, P(_abi.dfmi_expr_node), C.c_int32,
                                           P(C.c_char_p), P(P(_abi.dfmi_expr_node)), P(C.c_int32), P(C.c_int32),
                                           C.c_int32, P(_abi.dfmi_schema), P(_abi.dfmi_batch), C.c_int64, C.c_uint32,
                                           C.c_int64, P(_abi.dfmi_agg_value), P(_abi.dfmi_agg_value), P(C.c_int64),
                                           C.c_void_p, C.c_void_p, C.c_int64, P(_abi.dfmi_error)]
    L.oracle_aggregate_grouped.restype = C.c_int32
    L.oracle_aggregate_grouped_multi.argtypes = [P(_abi.dfmi_expr_node), C.c_int32, P(P(_abi.dfmi_expr_node)),
                                                 P(C.c_int32), C.c_int32, P(C.c_char_p), P(P(_abi.dfmi_expr_node)),
                                                 P(C.c_int32), P(C.c_int32), C.c_int32, P(_abi.dfmi_schema),
                                                 P(_abi.dfmi_batch), C.c_int64, C.c_uint32, C.c_int64,
                                                 P(_abi.dfmi_agg_value), P(_abi.dfmi_agg_value), P(C.c_int64),
                                                 C.c_int32, C.c_void_p, C.c_void_p, C.c_int64, P(_abi.dfmi_error)]
    L.oracle_aggregate_grouped_multi.restype = C.c_int32
    L.oracle_gen_unit_f64.argtypes = [C.c_uint64, C.c_uint32, C.c_int64, C.c_int64, C.c_void_p]
    L.oracle_gen_i64.argtypes = [C.c_uint64, C.c_uint32, C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_void_p]
    _L = L
    return L


def _host_column(a: Array) -> _abi.dfmi_column:
    assert a.values.device.type == "cpu"
    c = _abi.dfmi_column()
    c.type = int(a.data_type)
    c.length = a.length
    c.null_count = a.null_count
    c.validity = a.validity.data_ptr() if a.validity is not None else None
    c.values = a.values.data_ptr()
    c.offsets = a.offsets.data_ptr() if a.offsets is not None else None
    c.offset = a.offset
    return c


def _copy_out(col: _abi.dfmi_column) -> Array:
    t = DataType(col.type)
    n = col.length
    if t == DataType.Utf8:
        offs = np.ctypeslib.as_array(C.cast(col.offsets, C.POINTER(C.c_int32)), shape=(n + 1,)).copy()
        nbytes = int(offs[-1])
        data = np.ctypeslib.as_array(C.cast(col.values, C.POINTER(C.c_uint8)), shape=(max(nbytes, 1),))[:nbytes].copy()
        values = _bytes_tensor(data)
        offsets = _offsets_tensor(offs, "cpu")
    else:
        # the oracle's views: buffers start at the slice, bitmaps may start at
        # bit `offset` (< 8) of their first byte (a passed-through sliced input)
        bo = col.offset if t == DataType.Boolean else 0
        nbytes = (bo + n + 7) // 8 if t == DataType.Boolean else n * t.width
        raw = np.ctypeslib.as_array(C.cast(col.values, C.POINTER(C.c_uint8)), shape=(max(nbytes, 1),))[:nbytes].copy()
        if bo:
            raw = pack_bits(unpack_bits(raw, bo + n)[bo:])
        values = _bytes_tensor(raw)
        offsets = None
    validity = None
    if col.null_count:
        vo = col.offset
        vb = np.ctypeslib.as_array(C.cast(col.validity, C.POINTER(C.c_uint8)), shape=((vo + n + 7) // 8,)).copy()
        if vo:
            vb = pack_bits(unpack_bits(vb, vo + n)[vo:])
        validity = _bytes_tensor(vb)
    return Array(t, n, values, validity, offsets, col.null_count)


class Batched:
    """Host batch in ctypes form (keeps the tensors alive)."""

    def __init__(self, batch: RecordBatch):
        self.batch = batch.to("cpu")
        cols = self.batch.columns
        self.carr = (_abi.dfmi_column * max(1, len(cols)))()
        for i, a in enumerate(cols):
            self.carr[i] = _host_column(a)
        self.cb = _abi.dfmi_batch()
        self.cb.num_columns = len(cols)
        self.cb.num_rows = self.batch.num_rows()
        self.cb.columns = self.carr


def _prog_args(predicate: Optional[Expr], projections: Sequence[Expr]):
    pn = _abi.PostfixNodes(predicate.to_postfix()) if predicate is not None else None
    projs = [_abi.PostfixNodes(e.to_postfix()) for e in projections]
    parr = (C.POINTER(_abi.dfmi_expr_node) * max(1, len(projs)))(
        *[C.cast(p.array, C.POINTER(_abi.dfmi_expr_node)) for p in projs])
    lens = (C.c_int32 * max(1, len(projs)))(*[p.length for p in projs])
    return pn, projs, parr, lens


def oracle_filter_project(schema: Schema, batch: RecordBatch, predicate: Optional[Expr],
                          projections: Sequence[Expr], flags: int = 0):
    """Returns (list of (name, Array)) or raises ExecutionError."""
    L = oracle_lib()
    hb = Batched(batch)
    sch, keep = _abi.make_schema([(f.name, f.data_type, f.nullable) for f in schema.fields])
    pn, projs, parr, lens = _prog_args(predicate, projections)
    out = C.c_void_p()
    err = _abi.dfmi_error()
    rc = L.oracle_filter_project(pn.array if pn else None, pn.length if pn else 0, parr, lens, len(projs),
                                 C.byref(sch), C.byref(hb.cb), flags, C.byref(out), C.byref(err))
    if rc != 0:
        raise ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
    try:
        res = []
        for i in range(L.oracle_result_num_columns(out)):
            col = _abi.dfmi_column()
            name = C.c_char_p()
            L.oracle_result_column(out, i, C.byref(col), C.byref(name))
            res.append((name.value.decode("utf-8", errors="surrogateescape"), _copy_out(col)))
        return res
    finally:
        L.oracle_result_free(out)


def oracle_run_batched(schema: Schema, batch: RecordBatch, predicate, projections, batch_rows: int,
                       flags: int = 0) -> int:
    L = oracle_lib()
    hb = Batched(batch)
    sch, keep = _abi.make_schema([(f.name, f.data_type, f.nullable) for f in schema.fields])
    pn, projs, parr, lens = _prog_args(predicate, projections)
    rows = C.c_int64()
    err = _abi.dfmi_error()
    rc = L.oracle_run_batched(pn.array if pn else None, pn.length if pn else 0, parr, lens, len(projs),
                              C.byref(sch), C.byref(hb.cb), batch_rows, flags, C.byref(rows), C.byref(err))
    if rc != 0:
        raise ExecutionError.from_status(rc, err.message.decode())
    return rows.value


def oracle_compile(expr: Expr, schema: Schema, flags: int = 0):
    """(name, type) or raises ExecutionError — compile_scalar_expr restated."""
    L = oracle_lib()
    nodes = _abi.PostfixNodes(expr.to_postfix())
    sch, keep = _abi.make_schema([(f.name, f.data_type, f.nullable) for f in schema.fields])
    name = C.create_string_buffer(4096)
    t = C.c_int32()
    err = _abi.dfmi_error()
    rc = L.oracle_compile_info(nodes.array, nodes.length, C.byref(sch), flags, name, 4096, C.byref(t), C.byref(err))
    if rc != 0:
        raise ExecutionError.from_status(rc, err.message.decode())
    return name.value.decode("utf-8", errors="surrogateescape"), DataType(t.value)


def gen_unit_f64(seed: int, col: int, row0: int, n: int) -> np.ndarray:
    out = np.empty(n, dtype=np.float64)
    oracle_lib().oracle_gen_unit_f64(seed, col, row0, n, out.ctypes.data)
    return out


def gen_i64(seed: int, col: int, row0: int, n: int, lo: int, hi: int) -> np.ndarray:
    out = np.empty(n, dtype=np.int64)
    oracle_lib().oracle_gen_i64(seed, col, row0, n, lo, hi, out.ctypes.data)
    return out


def oracle_aggregate(schema: Schema, batch: RecordBatch, pred: Optional[Expr], aggs: Sequence, flags: int = None,
                     batch_rows: int = 0):
    """Aggregate(Selection?(scan)) on the oracle: aggs are logicalplan
    AggregateFunction expressions; returns dfmi_agg_value per aggregate, or
    raises ExecutionError. batch_rows > 0 pulls the input in batches."""
    if flags is None:
        flags = _abi.DFMI_FLAG_EXT_AGGREGATE
    L = oracle_lib()
    hb = Batched(batch)
    sch, keep = _abi.make_schema([(f.name, f.data_type, f.nullable) for f in schema.fields])
    pn = _abi.PostfixNodes(pred.to_postfix()) if pred is not None else None
    arg_nodes = [_abi.PostfixNodes(a.args[0].to_postfix()) for a in aggs]
    names = (C.c_char_p * len(aggs))(*[a.name.encode() for a in aggs])
    arr = (C.POINTER(_abi.dfmi_expr_node) * len(aggs))(*[C.cast(x.array, C.POINTER(_abi.dfmi_expr_node))
                                                           for x in arg_nodes])
    lens = (C.c_int32 * len(aggs))(*[x.length for x in arg_nodes])
    rts = (C.c_int32 * len(aggs))(*[int(a.return_type) for a in aggs])
    out = (_abi.dfmi_agg_value * len(aggs))()
    err = _abi.dfmi_error()
    rc = L.oracle_aggregate(pn.array if pn else None, pn.length if pn else 0, names, arr, lens, rts, len(aggs),
                            C.byref(sch), C.byref(hb.cb), batch_rows, flags, out, C.byref(err))
    if rc != _abi.DFMI_OK:
        raise ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
    return list(out)


def oracle_aggregate_grouped(schema: Schema, batch: RecordBatch, pred: Optional[Expr], key: Expr, aggs: Sequence,
                             flags: int = None, batch_rows: int = 0, cap: int = 0, key_strings: bool = False):
    """Aggregate{group_expr: [key]}(Selection?(scan)) on the oracle: returns
    (keys, values) -- one dfmi_agg_value key per group (key order, null
    last) and per group the list of aggregate values -- or raises
    ExecutionError. key_strings: also the Utf8 keys' bytes per group
    (keys, values, [bytes | None])."""
    if flags is None:
        flags = _abi.DFMI_FLAG_EXT_AGGREGATE
    L = oracle_lib()
    hb = Batched(batch)
    sch, keep = _abi.make_schema([(f.name, f.data_type, f.nullable) for f in schema.fields])
    pn = _abi.PostfixNodes(pred.to_postfix()) if pred is not None else None
    kn = _abi.PostfixNodes(key.to_postfix())
    n = len(aggs)
    arg_nodes = [_abi.PostfixNodes(a.args[0].to_postfix()) for a in aggs]
    names = (C.c_char_p * max(1, n))(*[a.name.encode() for a in aggs])
    arr = (C.POINTER(_abi.dfmi_expr_node) * max(1, n))(*[C.cast(x.array, C.POINTER(_abi.dfmi_expr_node))
                                                          for x in arg_nodes])
    lens = (C.c_int32 * max(1, n))(*[x.length for x in arg_nodes])
    rts = (C.c_int32 * max(1, n))(*[int(a.return_type) for a in aggs])
    cap = cap or batch.num_rows() + 1  # at most one group per row (+ the null key)
    keys = (_abi.dfmi_agg_value * cap)()
    out = (_abi.dfmi_agg_value * (cap * max(1, n)))()
    ng = C.c_int64()
    err = _abi.dfmi_error()
    koff = np.zeros(cap + 1, np.int32)
    kcap = 1 << 12
    for c in batch.columns:  # the key's bytes are at most every Utf8 column's bytes
        if c.data_type == DataType.Utf8:
            kcap += c.values.numel()
    kdata = np.zeros(kcap, np.uint8)
    rc = L.oracle_aggregate_grouped(pn.array if pn else None, pn.length if pn else 0, kn.array, kn.length, names, arr,
                                    lens, rts, n, C.byref(sch), C.byref(hb.cb), batch_rows, flags, cap, keys, out,
                                    C.byref(ng), koff.ctypes.data, kdata.ctypes.data, kcap, C.byref(err))
    if rc != _abi.DFMI_OK:
        raise ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
    g = ng.value
    res = (list(keys[:g]), [list(out[i * n:(i + 1) * n]) for i in range(g)])
    if not key_strings:
        return res
    strs = [None if keys[i].is_null else bytes(kdata[koff[i]:koff[i + 1]]) for i in range(g)]
    return res + (strs,)


def oracle_aggregate_grouped_multi(schema: Schema, batch: RecordBatch, pred: Optional[Expr], keys: Sequence[Expr],
                                   aggs: Sequence, flags: int = None, batch_rows: int = 0, cap: int = 0):
    """Aggregate{group_expr: keys}(Selection?(scan)) on the oracle: returns
    (keys, values, strings) -- per group (key order: lexicographic over the
    parts, each part's null last) the list of its key parts' dfmi_agg_values,
    its aggregate values, and per Utf8 key part p strings[p] = the groups'
    bytes (None for null; None for a non-Utf8 part) -- or raises ExecutionError."""
    if flags is None:
        flags = _abi.DFMI_FLAG_EXT_AGGREGATE
    L = oracle_lib()
    hb = Batched(batch)
    sch, keep = _abi.make_schema([(f.name, f.data_type, f.nullable) for f in schema.fields])
    pn = _abi.PostfixNodes(pred.to_postfix()) if pred is not None else None
    kns = [_abi.PostfixNodes(k.to_postfix()) for k in keys]
    nk = len(keys)
    karr = (C.POINTER(_abi.dfmi_expr_node) * nk)(*[C.cast(x.array, C.POINTER(_abi.dfmi_expr_node)) for x in kns])
    klens = (C.c_int32 * nk)(*[x.length for x in kns])
    n = len(aggs)
    arg_nodes = [_abi.PostfixNodes(a.args[0].to_postfix()) for a in aggs]
    names = (C.c_char_p * max(1, n))(*[a.name.encode() for a in aggs])
    arr = (C.POINTER(_abi.dfmi_expr_node) * max(1, n))(*[C.cast(x.array, C.POINTER(_abi.dfmi_expr_node))
                                                          for x in arg_nodes])
    lens = (C.c_int32 * max(1, n))(*[x.length for x in arg_nodes])
    rts = (C.c_int32 * max(1, n))(*[int(a.return_type) for a in aggs])
    cap = cap or batch.num_rows() + 1
    kout = (_abi.dfmi_agg_value * (cap * nk))()
    out = (_abi.dfmi_agg_value * (cap * max(1, n)))()
    ng = C.c_int64()
    err = _abi.dfmi_error()
    koff = np.zeros(cap + 1, np.int32)
    kcap = 1 << 12
    for c in batch.columns:
        if c.data_type == DataType.Utf8:
            kcap += c.values.numel()
    kdata = np.zeros(kcap, np.uint8)
    strings = []
    for part in range(nk):
        rc = L.oracle_aggregate_grouped_multi(pn.array if pn else None, pn.length if pn else 0, karr, klens, nk, names,
                                              arr, lens, rts, n, C.byref(sch), C.byref(hb.cb), batch_rows, flags, cap,
                                              kout, out, C.byref(ng), part, koff.ctypes.data, kdata.ctypes.data, kcap,
                                              C.byref(err))
        if rc != _abi.DFMI_OK:
            raise ExecutionError.from_status(rc, err.message.decode("utf-8", errors="replace"))
        g = ng.value
        if kout[part].type == int(DataType.Utf8) if g else False:
            strings.append([None if kout[i * nk + part].is_null else bytes(kdata[koff[i]:koff[i + 1]]) for i in range(g)])
        else:
            strings.append(None)
    g = ng.value
    return ([list(kout[i * nk:(i + 1) * nk]) for i in range(g)], [list(out[i * n:(i + 1) * n]) for i in range(g)],
            strings)
