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
                                        binary_expr_coerced)

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


def all_types_schema(f64_col: int = None, i64_col: int = None) -> Schema:
    """all_types_flat.csv with every column Utf8 except the one under test
    (so the reference's filter() can gather every column)."""
    fields = []
    for i in range(12):
        t = DataType.Utf8
        if i == f64_col:
            t = DataType.Float64
        if i == i64_col:
            t = DataType.Int64
        fields.append(Field("c%d" % i, t, False))
    return Schema(fields)


def lit_expr(schema, col, op, value):
    return binary_expr_coerced(Column(col), op, Literal(value), schema)
