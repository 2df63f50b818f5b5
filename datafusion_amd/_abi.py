"""ctypes mirror of include/dfmi.h and the loader of libdfmi.so.

The product path has no fallback: if the HIP library is missing or cannot be
loaded, ``lib()`` raises. The same struct definitions are reused by the
tests to talk to the CPU oracle (oracle/oracle.h shares the layouts).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import List, Optional, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libdfmi.so")

# status codes (dfmi_status)
DFMI_OK = 0
DFMI_ERR_EXECUTION = 1
DFMI_ERR_GENERAL = 2
DFMI_ERR_INVALID_COLUMN = 3
DFMI_ERR_NOT_IMPLEMENTED = 4
DFMI_ERR_DIVIDE_BY_ZERO = 5
DFMI_ERR_ARROW_COMPUTE = 6
DFMI_ERR_PANIC = 7
DFMI_ERR_INVALID_ARGUMENT = 8
DFMI_ERR_CAPACITY = 9
DFMI_ERR_DEVICE = 10
DFMI_ERR_ARROW_PARSE = 11

DFMI_FLAG_EXT_GATHER_ALL = 0x1
DFMI_FLAG_EXT_UTF8_COMPARE = 0x2
DFMI_FLAG_EXT_CAST = 0x4
DFMI_FLAG_EXT_IS_NULL = 0x8
DFMI_FLAG_EXT_AGGREGATE = 0x10

# dfmi_agg_fn (AggregateType, expression.rs:33-40)
DFMI_AGG_MIN = 0
DFMI_AGG_MAX = 1
DFMI_AGG_SUM = 2
DFMI_AGG_COUNT = 3

STATUS_NAMES = {
    DFMI_ERR_EXECUTION: "ExecutionError",
    DFMI_ERR_GENERAL: "General",
    DFMI_ERR_INVALID_COLUMN: "InvalidColumn",
    DFMI_ERR_NOT_IMPLEMENTED: "NotImplemented",
    DFMI_ERR_DIVIDE_BY_ZERO: "ArrowError(DivideByZero)",
    DFMI_ERR_ARROW_COMPUTE: "ArrowError(ComputeError)",
    DFMI_ERR_PANIC: "panic",
    DFMI_ERR_INVALID_ARGUMENT: "InvalidArgument",
    DFMI_ERR_CAPACITY: "Capacity",
    DFMI_ERR_DEVICE: "Device",
    DFMI_ERR_ARROW_PARSE: "ArrowError(ParseError)",
}


class dfmi_error(C.Structure):
    _fields_ = [("code", C.c_int32), ("message", C.c_char * 500)]


class dfmi_column(C.Structure):
    _fields_ = [
        ("type", C.c_int32),
        ("reserved", C.c_int32),
        ("length", C.c_int64),
        ("null_count", C.c_int64),
        ("validity", C.c_void_p),
        ("values", C.c_void_p),
        ("offsets", C.c_void_p),
        ("offset", C.c_int64),  # arrow ArrayData::offset (a sliced array)
    ]


class dfmi_batch(C.Structure):
    _fields_ = [
        ("num_columns", C.c_int32),
        ("reserved", C.c_int32),
        ("num_rows", C.c_int64),
        ("columns", C.POINTER(dfmi_column)),
    ]


class dfmi_field(C.Structure):
    _fields_ = [("name", C.c_char_p), ("type", C.c_int32), ("nullable", C.c_int32)]


class dfmi_schema(C.Structure):
    _fields_ = [("num_fields", C.c_int32), ("reserved", C.c_int32), ("fields", C.POINTER(dfmi_field))]


class dfmi_expr_node(C.Structure):
    _fields_ = [
        ("kind", C.c_int32),
        ("op", C.c_int32),
        ("data_type", C.c_int32),
        ("column", C.c_int32),
        ("i64", C.c_int64),
        ("f64", C.c_double),
        ("str", C.c_char_p),
        ("str_len", C.c_int64),
    ]


class dfmi_out_column(C.Structure):
    _fields_ = [
        ("values", C.c_void_p),
        ("validity", C.c_void_p),
        ("offsets", C.c_void_p),
        ("data", C.c_void_p),
        ("data_capacity", C.c_int64),
        ("type", C.c_int32),
        ("passthrough_column", C.c_int32),
        ("length", C.c_int64),
        ("null_count", C.c_int64),
        ("data_length", C.c_int64),
    ]


class dfmi_shard_placement(C.Structure):
    _fields_ = [("world", C.c_int32), ("rank", C.c_int32), ("row_offset", C.c_int64), ("total_rows", C.c_int64),
                ("utf8_base", C.c_int64 * 16), ("utf8_total", C.c_int64 * 16), ("null_total", C.c_int64 * 16)]


DFMI_SHARD_ID_BYTES = 128


class dfmi_agg_value(C.Structure):
    _fields_ = [("type", C.c_int32), ("is_null", C.c_int32), ("count", C.c_int64), ("bits", C.c_uint64)]


# include/dfmi.h's DFMI_ABI_VERSION: lib() refuses a library built from another header
DFMI_ABI_VERSION = 3

# Every symbol include/dfmi.h declares (checked by the CPU test suite).
EXPORTED = [
    "dfmi_abi_version",
    "dfmi_context_set_shared",
    "dfmi_host_batches_output_bytes",
    "dfmi_filter_project_host_batches_into",
    "dfmi_compile_scalar_expr",
    "dfmi_program_name",
    "dfmi_program_type",
    "dfmi_program_free",
    "dfmi_context_create",
    "dfmi_context_destroy",
    "dfmi_context_set_stream",
    "dfmi_filter_project",
    "dfmi_filter_project_batches",
    "dfmi_filter_project_host",
    "dfmi_filter_project_host_batches",
    "dfmi_host_result_num_columns",
    "dfmi_host_result_column",
    "dfmi_host_result_columns",
    "dfmi_host_result_block",
    "dfmi_host_result_free",
    "dfmi_context_set_timing",
    "dfmi_host_alloc",
    "dfmi_host_free",
    "dfmi_host_register",
    "dfmi_host_unregister",
    "dfmi_last_timing",
    "dfmi_last_compile_ms",
    "dfmi_last_error_order",
    "dfmi_last_kernel_name",
    "dfmi_compile_aggregate",
    "dfmi_aggregate_name",
    "dfmi_aggregate_type",
    "dfmi_aggregate_free",
    "dfmi_agg_state_create",
    "dfmi_aggregate_batch",
    "dfmi_agg_state_finish",
    "dfmi_agg_partial_bytes",
    "dfmi_agg_state_partial",
    "dfmi_agg_merge_partials",
    "dfmi_agg_state_reset",
    "dfmi_agg_state_create_grouped",
    "dfmi_agg_state_create_grouped_multi",
    "dfmi_agg_state_num_keys",
    "dfmi_agg_state_finish_grouped",
    "dfmi_agg_state_group_keys_utf8",
    "dfmi_agg_state_group_keys_utf8_part",
    "dfmi_agg_state_grouped_partial_bytes",
    "dfmi_agg_state_grouped_partial",
    "dfmi_agg_merge_grouped_partials",
    "dfmi_agg_merge_grouped_partials_keys_utf8",
    "dfmi_shard_unique_id",
    "dfmi_shard_comm_init",
    "dfmi_shard_comm_destroy",
    "dfmi_shard_filter_project",
    "dfmi_shard_gather_to_root",
    "dfmi_shard_agg_finish",
    "dfmi_shard_agg_finish_grouped",
    "dfmi_agg_state_free",
    "dfmi_generate_column",  # include/dfmi_datasource.h
    "dfmi_csv_open",
    "dfmi_csv_next",
    "dfmi_csv_num_records",
    "dfmi_csv_close",
]

DFMI_GEN_UNIT_F64 = 1
DFMI_GEN_I64 = 2


class PostfixNodes:
    """Keeps a ctypes node array and the bytes its string pointers reference."""

    def __init__(self, nodes: Sequence[dict]):
        self._keep: List[bytes] = []
        self.array = (dfmi_expr_node * len(nodes))()
        for i, d in enumerate(nodes):
            n = self.array[i]
            n.kind = d.get("kind", 0)
            n.op = d.get("op", 0)
            n.data_type = d.get("data_type", 0)
            n.column = d.get("column", 0)
            n.i64 = d.get("i64", 0)
            n.f64 = d.get("f64", 0.0)
            s = d.get("str")
            if s is not None:
                self._keep.append(s)
                n.str = s
                n.str_len = len(s)
        self.length = len(nodes)


def make_schema(fields) -> tuple:
    """fields: sequence of (name, DataType, nullable). Returns (schema, keepalive)."""
    arr = (dfmi_field * max(1, len(fields)))()
    keep = []
    for i, (name, dt, nullable) in enumerate(fields):
        b = name.encode("utf-8")
        keep.append(b)
        arr[i].name = b
        arr[i].type = int(dt)
        arr[i].nullable = 1 if nullable else 0
    s = dfmi_schema()
    s.num_fields = len(fields)
    s.fields = arr
    return s, (arr, keep)


_LIB = None


def lib() -> C.CDLL:
    """Load libdfmi.so (built in-tree by __graft_entry__.build()). Fails loudly."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("libdfmi.so is not built (%s); run __graft_entry__.build()" % LIB_PATH)
    L = C.CDLL(LIB_PATH)
    L.dfmi_abi_version.argtypes = []
    L.dfmi_abi_version.restype = C.c_int32
    v = L.dfmi_abi_version()
    if v != DFMI_ABI_VERSION:
        raise RuntimeError("libdfmi.so has ABI version %d, this binding expects %d (rebuild)" % (v, DFMI_ABI_VERSION))
    L.dfmi_context_set_shared.argtypes = [C.c_void_p, C.c_int32]
    L.dfmi_context_set_shared.restype = C.c_int32
    L.dfmi_host_batches_output_bytes.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.c_int32, C.c_void_p, C.c_int32,
                                                 C.c_uint32, C.POINTER(C.c_size_t), C.POINTER(dfmi_error)]
    L.dfmi_host_batches_output_bytes.restype = C.c_int32
    L.dfmi_filter_project_host_batches_into.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p), C.c_int32,
                                                        C.c_void_p, C.c_int32, C.c_uint32, C.c_void_p, C.c_size_t,
                                                        C.c_void_p, C.POINTER(C.c_int32), C.POINTER(dfmi_error)]
    L.dfmi_filter_project_host_batches_into.restype = C.c_int32
    L.dfmi_compile_scalar_expr.argtypes = [C.POINTER(dfmi_expr_node), C.c_int32, C.POINTER(dfmi_schema),
                                           C.c_uint32, C.POINTER(C.c_void_p), C.POINTER(dfmi_error)]
    L.dfmi_compile_scalar_expr.restype = C.c_int32
    L.dfmi_program_name.argtypes = [C.c_void_p]
    L.dfmi_program_name.restype = C.c_char_p
    L.dfmi_program_type.argtypes = [C.c_void_p]
    L.dfmi_program_type.restype = C.c_int32
    L.dfmi_program_free.argtypes = [C.c_void_p]
    L.dfmi_program_free.restype = None
    L.dfmi_context_create.argtypes = [C.c_int32, C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(dfmi_error)]
    L.dfmi_context_create.restype = C.c_int32
    L.dfmi_context_destroy.argtypes = [C.c_void_p]
    L.dfmi_context_destroy.restype = None
    L.dfmi_context_set_stream.argtypes = [C.c_void_p, C.c_void_p]
    L.dfmi_context_set_stream.restype = C.c_int32
    L.dfmi_filter_project.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p), C.c_int32,
                                      C.POINTER(dfmi_batch), C.POINTER(dfmi_out_column), C.c_uint32,
                                      C.POINTER(dfmi_error)]
    L.dfmi_filter_project.restype = C.c_int32
    L.dfmi_filter_project_batches.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p), C.c_int32,
                                              C.POINTER(dfmi_batch), C.c_int32, C.POINTER(dfmi_out_column), C.c_uint32,
                                              C.POINTER(C.c_int32), C.POINTER(dfmi_error)]
    L.dfmi_filter_project_batches.restype = C.c_int32
    L.dfmi_filter_project_host.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p), C.c_int32,
                                           C.POINTER(dfmi_batch), C.c_uint32, C.POINTER(C.c_void_p),
                                           C.POINTER(dfmi_error)]
    L.dfmi_filter_project_host.restype = C.c_int32
    L.dfmi_filter_project_host_batches.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p), C.c_int32,
                                                   C.POINTER(dfmi_batch), C.c_int32, C.c_uint32,
                                                   C.POINTER(C.c_void_p), C.POINTER(C.c_int32), C.POINTER(dfmi_error)]
    L.dfmi_filter_project_host_batches.restype = C.c_int32
    L.dfmi_host_result_num_columns.argtypes = [C.c_void_p]
    L.dfmi_host_result_num_columns.restype = C.c_int32
    L.dfmi_host_result_column.argtypes = [C.c_void_p, C.c_int32, C.POINTER(dfmi_column)]
    L.dfmi_host_result_column.restype = C.c_int32
    L.dfmi_host_result_columns.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p]
    L.dfmi_host_result_columns.restype = C.c_int32
    L.dfmi_host_result_block.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
    L.dfmi_host_result_block.restype = C.c_int32
    L.dfmi_host_result_free.argtypes = [C.c_void_p]
    L.dfmi_host_result_free.restype = None
    L.dfmi_context_set_timing.argtypes = [C.c_void_p, C.c_int32]
    L.dfmi_context_set_timing.restype = C.c_int32
    L.dfmi_host_alloc.argtypes = [C.c_size_t, C.POINTER(C.c_void_p), C.POINTER(dfmi_error)]
    L.dfmi_host_alloc.restype = C.c_int32
    L.dfmi_host_free.argtypes = [C.c_void_p]
    L.dfmi_host_free.restype = C.c_int32
    L.dfmi_host_register.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(dfmi_error)]
    L.dfmi_host_register.restype = C.c_int32
    L.dfmi_host_unregister.argtypes = [C.c_void_p]
    L.dfmi_host_unregister.restype = C.c_int32
    L.dfmi_last_timing.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.dfmi_last_timing.restype = C.c_int32
    L.dfmi_last_compile_ms.argtypes = [C.c_void_p, C.POINTER(C.c_double)]
    L.dfmi_last_compile_ms.restype = C.c_int32
    L.dfmi_last_error_order.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
    L.dfmi_last_error_order.restype = C.c_int32
    L.dfmi_last_kernel_name.argtypes = [C.c_void_p]
    L.dfmi_last_kernel_name.restype = C.c_char_p
    L.dfmi_generate_column.argtypes = [C.c_void_p, C.c_int32, C.c_uint64, C.c_uint32, C.c_int64, C.c_int64,
                                       C.c_int64, C.c_int64, C.c_void_p, C.POINTER(dfmi_error)]
    L.dfmi_generate_column.restype = C.c_int32
    L.dfmi_csv_open.argtypes = [C.c_char_p, C.POINTER(dfmi_schema), C.c_int32, C.c_int64, C.c_int32,
                                C.POINTER(C.c_void_p), C.POINTER(dfmi_error)]
    L.dfmi_csv_open.restype = C.c_int32
    L.dfmi_csv_next.argtypes = [C.c_void_p, C.POINTER(dfmi_batch), C.POINTER(C.c_int32), C.POINTER(dfmi_error)]
    L.dfmi_csv_next.restype = C.c_int32
    L.dfmi_csv_num_records.argtypes = [C.c_void_p]
    L.dfmi_csv_num_records.restype = C.c_int64
    L.dfmi_csv_close.argtypes = [C.c_void_p]
    L.dfmi_csv_close.restype = None
    P = C.POINTER
    L.dfmi_compile_aggregate.argtypes = [C.c_char_p, C.c_void_p, C.c_int32, C.c_uint32, P(C.c_void_p), P(dfmi_error)]
    L.dfmi_compile_aggregate.restype = C.c_int32
    L.dfmi_aggregate_name.argtypes = [C.c_void_p]
    L.dfmi_aggregate_name.restype = C.c_char_p
    L.dfmi_aggregate_type.argtypes = [C.c_void_p]
    L.dfmi_aggregate_type.restype = C.c_int32
    L.dfmi_aggregate_free.argtypes = [C.c_void_p]
    L.dfmi_aggregate_free.restype = None
    L.dfmi_agg_state_create.argtypes = [C.c_void_p, P(C.c_void_p), C.c_int32, P(C.c_void_p), P(dfmi_error)]
    L.dfmi_agg_state_create.restype = C.c_int32
    L.dfmi_aggregate_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, P(dfmi_batch), C.c_uint32, P(dfmi_error)]
    L.dfmi_aggregate_batch.restype = C.c_int32
    L.dfmi_agg_state_finish.argtypes = [C.c_void_p, C.c_void_p, P(dfmi_agg_value), P(dfmi_error)]
    L.dfmi_agg_state_finish.restype = C.c_int32
    L.dfmi_agg_state_create_grouped.argtypes = [C.c_void_p, C.c_void_p, P(C.c_void_p), C.c_int32, P(C.c_void_p),
                                                P(dfmi_error)]
    L.dfmi_agg_state_create_grouped.restype = C.c_int32
    L.dfmi_agg_state_finish_grouped.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, P(dfmi_agg_value), P(dfmi_agg_value),
                                                P(C.c_int64), P(dfmi_error)]
    L.dfmi_agg_state_finish_grouped.restype = C.c_int32
    L.dfmi_agg_state_group_keys_utf8.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, P(C.c_int64),
                                                 P(dfmi_error)]
    L.dfmi_agg_state_group_keys_utf8.restype = C.c_int32
    L.dfmi_agg_state_create_grouped_multi.argtypes = [C.c_void_p, P(C.c_void_p), C.c_int32, P(C.c_void_p), C.c_int32,
                                                      P(C.c_void_p), P(dfmi_error)]
    L.dfmi_agg_state_create_grouped_multi.restype = C.c_int32
    L.dfmi_agg_state_num_keys.argtypes = [C.c_void_p]
    L.dfmi_agg_state_num_keys.restype = C.c_int32
    L.dfmi_agg_state_group_keys_utf8_part.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_int64, C.c_void_p,
                                                      C.c_int64, P(C.c_int64), P(dfmi_error)]
    L.dfmi_agg_state_group_keys_utf8_part.restype = C.c_int32
    L.dfmi_agg_merge_grouped_partials_keys_utf8.argtypes = [P(C.c_void_p), C.c_int32, P(C.c_void_p), P(C.c_int64),
                                                            C.c_int32, C.c_int32, C.c_void_p, C.c_int64, C.c_void_p,
                                                            C.c_int64, P(C.c_int64), P(dfmi_error)]
    L.dfmi_agg_merge_grouped_partials_keys_utf8.restype = C.c_int32
    L.dfmi_agg_partial_bytes.argtypes = [C.c_void_p]
    L.dfmi_agg_partial_bytes.restype = C.c_int64
    L.dfmi_agg_state_partial.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, P(dfmi_error)]
    L.dfmi_agg_state_partial.restype = C.c_int32
    L.dfmi_agg_merge_partials.argtypes = [P(C.c_void_p), C.c_int32, P(C.c_void_p), C.c_int32, P(dfmi_agg_value),
                                          P(dfmi_error)]
    L.dfmi_agg_merge_partials.restype = C.c_int32
    L.dfmi_agg_state_reset.argtypes = [C.c_void_p, C.c_void_p, P(dfmi_error)]
    L.dfmi_agg_state_reset.restype = C.c_int32
    L.dfmi_shard_unique_id.argtypes = [C.c_void_p, P(dfmi_error)]
    L.dfmi_shard_unique_id.restype = C.c_int32
    L.dfmi_shard_comm_init.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, P(C.c_void_p), P(dfmi_error)]
    L.dfmi_shard_comm_init.restype = C.c_int32
    L.dfmi_shard_comm_destroy.argtypes = [C.c_void_p]
    L.dfmi_shard_comm_destroy.restype = None
    L.dfmi_shard_filter_project.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, P(C.c_void_p), C.c_int32,
                                            P(dfmi_batch), P(dfmi_out_column), C.c_uint32, P(dfmi_shard_placement),
                                            P(dfmi_error)]
    L.dfmi_shard_filter_project.restype = C.c_int32
    L.dfmi_shard_gather_to_root.argtypes = [C.c_void_p, C.c_void_p, P(dfmi_out_column), P(dfmi_out_column), C.c_int32,
                                            P(dfmi_error)]
    L.dfmi_shard_gather_to_root.restype = C.c_int32
    L.dfmi_shard_agg_finish.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, P(C.c_void_p), C.c_int32,
                                        P(dfmi_agg_value), P(dfmi_error)]
    L.dfmi_shard_agg_finish.restype = C.c_int32
    L.dfmi_shard_agg_finish_grouped.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, P(C.c_void_p), C.c_int32, C.c_int64,
                                                P(dfmi_agg_value), P(dfmi_agg_value), P(C.c_int64), P(dfmi_error)]
    L.dfmi_shard_agg_finish_grouped.restype = C.c_int32
    L.dfmi_agg_state_grouped_partial_bytes.argtypes = [C.c_void_p, C.c_void_p, P(dfmi_error)]
    L.dfmi_agg_state_grouped_partial_bytes.restype = C.c_int64
    L.dfmi_agg_state_grouped_partial.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, P(dfmi_error)]
    L.dfmi_agg_state_grouped_partial.restype = C.c_int32
    L.dfmi_agg_merge_grouped_partials.argtypes = [P(C.c_void_p), C.c_int32, P(C.c_void_p), P(C.c_int64), C.c_int32,
                                                  C.c_int64, P(dfmi_agg_value), P(dfmi_agg_value), P(C.c_int64),
                                                  P(dfmi_error)]
    L.dfmi_agg_merge_grouped_partials.restype = C.c_int32
    L.dfmi_agg_state_free.argtypes = [C.c_void_p]
    L.dfmi_agg_state_free.restype = None
    _LIB = L
    return L
