"""Known-answer cases from the reference tree's own fixtures.

Every case names the reference file it comes from. The same cases drive the
oracle (CPU suite, pins the restatement) and the device (GPU suite).
Data files under tests/golden/ are copies of /root/reference/test/data/*
(inputs and expected outputs only).
"""
from __future__ import annotations

import csv
import os
from typing import List

import numpy as np

from datafusion_amd._abi import DFMI_FLAG_EXT_GATHER_ALL
from datafusion_amd.arrow import Field, Schema
from datafusion_amd.execution.datasource import CsvDataSource
from datafusion_amd.logicalplan import (BinaryExpr, Column, DataType, Float64, Int64, Literal, Operator,
                                        ScalarValue, binary_expr_coerced)

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

CITIES = Schema([Field("city", DataType.Utf8, False), Field("lat", DataType.Float64, False),
                 Field("lng", DataType.Float64, False)])
NUMERICS = Schema([Field("a", DataType.Int64, False), Field("b", DataType.Int64, False),
                   Field("a_f", DataType.Float64, False), Field("b_f", DataType.Float64, False)])


def load_batch(schema: Schema, name: str, has_header: bool):
    ds = CsvDataSource(schema, os.path.join(GOLDEN, name), has_header=has_header, batch_size=1 << 20)
    return ds.next()


def expected_rows(name: str) -> List[List[str]]:
    with open(os.path.join(GOLDEN, "expected", name), newline="", encoding="utf-8") as f:
        return [r for r in csv.reader(f) if r]


def smoketest_points(section: int) -> List[tuple]:
    """smoketest-expected.txt: POINT (lat lng) lines of the 1st/2nd query."""
    lines = open(os.path.join(GOLDEN, "smoketest-expected.txt"), encoding="utf-8").read().splitlines()
    out, cur = [], -1
    for ln in lines:
        if ln.startswith("Executing query"):
            cur += 1
            if cur == 0:
                continue
            if cur == 1:
                out.append([])
            else:
                out.append([])
            continue
        if ln.startswith("POINT") and out:
            a, b = ln[len("POINT ("):-1].split()
            out[-1].append((float(a), float(b)))
    return out[section]


def all_types_schema(f64_col: int = None, i64_col: int = None, typed: dict = None) -> Schema:
    """all_types_flat.csv with every column Utf8 except the ones under test
    (so the reference's filter() can gather every column). ``typed`` maps a
    column index to its real type (ALL_TYPES)."""
    typed = dict(typed or {})
    if f64_col is not None:
        typed[f64_col] = DataType.Float64
    if i64_col is not None:
        typed[i64_col] = DataType.Int64
    return Schema([Field("c%d" % i, typed.get(i, DataType.Utf8), False) for i in range(12)])


# all_types_flat.csv column types (the original POC's all_types schema: the
# values of every column fit exactly these types)
ALL_TYPES = [DataType.Boolean, DataType.UInt8, DataType.UInt16, DataType.UInt32, DataType.UInt64, DataType.Int8,
             DataType.Int16, DataType.Int32, DataType.Int64, DataType.Float32, DataType.Float64, DataType.Utf8]

# Known answers from test/data/expected/ over all_types_flat.csv whose queries
# were re-derived here (the POC's tests that produced them are not in the
# reference tree; each query below reproduces its file row for row):
# (file, column, operator, literal value) -> SELECT c<col> WHERE c<col> <op> <lit>,
# the literal typed as the column (no cast).
ALL_TYPES_NARROW = [
    ("c_int8_positive.csv", 5, Operator.GtEq, 0), ("c_int8_negative.csv", 5, Operator.Lt, 0),
    ("c_int8_range_exclusive.csv", 5, Operator.Gt, 100),
    ("c_int16_positive.csv", 6, Operator.Gt, 0), ("c_int16_negative.csv", 6, Operator.Lt, 0),
    ("c_int32_positive.csv", 7, Operator.Gt, 0), ("c_int32_negative.csv", 7, Operator.Lt, 0),
    ("c_float32_high.csv", 9, Operator.Gt, 0.5), ("c_float32_low.csv", 9, Operator.Lt, 0.5),
]


# Known answers that need CAST(column) (DFMI_FLAG_EXT_CAST): the SQL planner
# coerces `c5 < 0` (Int8 vs the Int64 literal) to CAST(#5 AS Int64) Lt Int64(0)
# (sqlplanner.rs:273-278) and `c5 > c6` to CAST(#5 AS Int16) Gt #6, which the
# reference cannot execute ("column reference", expression.rs:281-282).
# The unsigned columns cannot be compared with an Int64 literal at all
# (can_coerce_from(Int64, UInt8) is false, logicalplan.rs:553-602), so their
# files are reproduced by an explicit projection CAST (all 256 rows).
# (file, {column: type}, SQL over table t of all_types_flat.csv)
ALL_TYPES_CAST = [
    ("c_int8_cast.csv", (5,), "SELECT c5 FROM t WHERE c5 < 0"),
    ("c_int16_cast.csv", (6,), "SELECT c6 FROM t WHERE c6 < 0"),
    ("c_int32_cast.csv", (7,), "SELECT c7 FROM t WHERE c7 < 0"),
    ("c_int64_cast.csv", (8,), "SELECT c8 FROM t WHERE c8 < 0"),
    ("c_float32_cast.csv", (9,), "SELECT c9 FROM t WHERE c9 < 0.5"),
    ("c_float64_cast.csv", (10,), "SELECT c10 FROM t WHERE c10 < 0.5"),
    ("c_uint8_cast.csv", (1,), "SELECT CAST(c1 AS BIGINT) FROM t"),
    ("c_uint16_cast.csv", (2,), "SELECT CAST(c2 AS BIGINT) FROM t"),
    ("c_uint32_cast.csv", (3,), "SELECT CAST(c3 AS BIGINT) FROM t"),
    ("c_uint64_cast.csv", (4,), "SELECT CAST(c4 AS BIGINT) FROM t"),
    ("c_int8_col_gt.csv", (5, 6), "SELECT c5 FROM t WHERE c5 > c6"),
    ("c_int8_col_gteq.csv", (5, 6), "SELECT c5 FROM t WHERE c5 >= c6"),
    ("c_int8_col_lt.csv", (5, 6), "SELECT c5 FROM t WHERE c5 < c6"),
    ("c_int8_col_lteq.csv", (5, 6), "SELECT c5 FROM t WHERE c5 <= c6"),
    ("c_int8_col_eq.csv", (5, 6), "SELECT c5 FROM t WHERE c5 = c6"),
    ("c_int8_col_noteq.csv", (5, 6), "SELECT c5 FROM t WHERE c5 != c6"),
]

# expected/is_null_csv.csv / is_not_null_csv.csv over null_test.csv
# (DFMI_FLAG_EXT_IS_NULL; IsNull/IsNotNull are commented out in the reference).
NULL_TEST = Schema([Field("c_int", DataType.Int64, False), Field("c_float", DataType.Float64, True),
                    Field("c_string", DataType.Utf8, True), Field("c_bool", DataType.Boolean, False)])
NULL_CASES = [("is_null_csv.csv", "SELECT c_int FROM null_test WHERE c_float IS NULL"),
              ("is_not_null_csv.csv", "SELECT c_int FROM null_test WHERE c_float IS NOT NULL")]


def sql_plan(sql: str, schema: Schema, table: str):
    """(predicate, projections) the reference's SQL planner produces."""
    from datafusion_amd.sqlplanner import SqlToRel

    class _Ctx:
        def table_schema(self, name):
            return schema if name == table else None
    p = SqlToRel(_Ctx()).sql_to_rel(sql)
    pred = p.input.expr if type(p.input).__name__ == "Selection" else None
    return pred, p.expr


def cast_fixture_case(name, cols, sql):
    """(schema, predicate, projections) of an ALL_TYPES_CAST entry."""
    s = all_types_schema(typed={c: ALL_TYPES[c] for c in cols})
    pred, projs = sql_plan(sql, s, "t")
    return s, pred, projs


def fixture_values(name: str, t: DataType) -> list:
    """One-column expected file as Python values of type t."""
    rows = expected_rows(name)
    if t in (DataType.Float32, DataType.Float64):
        return [float(np.float32(r[0])) if t == DataType.Float32 else float(r[0]) for r in rows]
    return [int(r[0]) for r in rows]


def lit_expr(schema, col, op, value):
    return binary_expr_coerced(Column(col), op, Literal(value), schema)


def narrow_fixture_case(name, col, op, lit):
    """(schema, predicate, projections) of an ALL_TYPES_NARROW entry."""
    t = ALL_TYPES[col]
    s = all_types_schema(typed={col: t})
    return s, BinaryExpr(Column(col), op, Literal(ScalarValue(t, lit))), [Column(col)]


# expected/c_int8_range_inclusive.csv (98 rows): c5 >= 2 AND c5 <= 99 over the
# Int8 column (same-typed Int8 literals; gathering Int8 needs the extension).
RANGE_CASES = [("c_int8_range_inclusive.csv", 5, 2, 99)]


def range_fixture_case(name, col, lo, hi):
    t = ALL_TYPES[col]
    s = all_types_schema(typed={col: t})
    pred = BinaryExpr(BinaryExpr(Column(col), Operator.GtEq, Literal(ScalarValue(t, lo))), Operator.And,
                      BinaryExpr(Column(col), Operator.LtEq, Literal(ScalarValue(t, hi))))
    return s, pred, [Column(col)]


# expected/c_float32_{high,low,cast}_uint32.csv: each file is the WHOLE
# c_float32 column (all 256 rows, file order) -- the output of a predicate
# true on every row. The POC queries behind them are not in the reference
# tree, and the reference cannot name a UInt32 in SQL at all (convert_data_type,
# sqlplanner.rs:363-374, maps no SQL type to UInt32), so the query is not
# recoverable; the files are pinned as "every row selected" through the
# UInt32 comparison their names point at: CAST(c9 AS UInt32) = UInt32(0)
# holds on every row (every value lies in [0, 1) and truncates to 0;
# DFMI_FLAG_EXT_CAST), projecting c9 (Float32 gather: DFMI_FLAG_EXT_GATHER_ALL).
WHOLE_F32_FILES = ["c_float32_high_uint32.csv", "c_float32_low_uint32.csv", "c_float32_cast_uint32.csv"]


def whole_f32_case():
    from datafusion_amd.logicalplan import Cast
    s = all_types_schema(typed={9: DataType.Float32})
    pred = BinaryExpr(Cast(Column(9), DataType.UInt32), Operator.Eq, Literal(ScalarValue(DataType.UInt32, 0)))
    return s, pred, [Column(9)]


# Aggregate fixtures (DFMI_FLAG_EXT_AGGREGATE; the reference plans Aggregate
# but cannot execute it, context.rs:161):
#   expected/test_sql_min_max.csv = MIN(lat), MAX(lat), MIN(lng), MAX(lng)
#     over all 37 rows of uk_cities.csv (read without a header row);
#   expected/csv_aggregate_all_types.csv = COUNT, COUNT, then MIN and MAX of
#     each of the 12 columns of all_types_flat.csv. Columns 1-10 (the numeric
#     ones) are pinned here; MIN/MAX of Boolean (col 0) and Utf8 (col 11) are
#     outside the extension (NotImplemented "aggregate over Boolean/Utf8":
#     arrow 0.12's min/max kernels are numeric only). The file's Utf8 MIN is
#     the bytewise minimum of the column, but its Utf8 MAX repeats the MIN --
#     a defect of the POC that wrote it (the column holds 256 distinct strings).
MIN_MAX_SQL = "SELECT MIN(lat), MAX(lat), MIN(lng), MAX(lng) FROM uk_cities"


def all_types_typed():
    return all_types_schema(typed={i: t for i, t in enumerate(ALL_TYPES)})


def agg_fixture_value(text: str, t: DataType) -> int:
    """A fixture cell as the bits dfmi_agg_value.bits carries (integers
    sign/zero-extended to 64 bits, Float32 bits in the low 32)."""
    if t == DataType.Float64:
        return int(np.array([float(text)], dtype=np.float64).view(np.uint64)[0])
    if t == DataType.Float32:
        return int(np.array([np.float32(text)], dtype=np.float32).view(np.uint32)[0])
    return int(text) & ((1 << 64) - 1)
