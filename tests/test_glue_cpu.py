"""The Python binding's native struct packing (csrc/pyglue.cpp, _dfmi_glue):
for every column of every batch it fills exactly the dfmi_column that
engine.column_struct() builds field by field (include/dfmi.h), including
sliced arrays (offset), nullable columns, Utf8 offsets and Boolean bitmaps,
batches whose columns are lazy, and refuses what is not a host batch."""
import ctypes as C

import numpy as np
import pytest

from datafusion_amd import _abi
from datafusion_amd.arrow import Array, LazyColumns, RecordBatch, Schema
from datafusion_amd.execution.engine import column_struct, host_batch_structs
from datafusion_amd.logicalplan import DataType

FIELDS = ("type", "length", "null_count", "validity", "values", "offsets", "offset")


def as_tuple(c):
    return tuple(int(getattr(c, f) or 0) for f in FIELDS)


def batches(n_batches=7, seed=3):
    rng = np.random.default_rng(seed)
    out = []
    for b in range(n_batches):
        n = int(rng.integers(0, 3000))
        cols = [Array.from_numpy(DataType.Float64, rng.random(n), rng.random(n) > 0.2 if b % 2 else None),
                Array.from_numpy(DataType.Int32, rng.integers(-9, 9, n).astype(np.int32)),
                Array.from_numpy(DataType.Boolean, rng.random(n) < 0.5, rng.random(n) > 0.3),
                Array.from_strings([None if rng.random() < 0.1 else b"w%d" % i for i in range(n)])]
        if b % 3 == 2 and n > 10:  # a sliced batch
            off = int(rng.integers(1, n // 2))
            cols = [c.slice(off, n - off - 3) for c in cols]
        out.append(RecordBatch(Schema.empty(), cols))
    return out


def test_pack_matches_column_struct():
    bs = batches()
    barr, keep = host_batch_structs(bs, 4)
    for i, b in enumerate(bs):
        assert barr[i].num_columns == 4 and barr[i].num_rows == b.num_rows()
        cols = C.cast(barr[i].columns, C.POINTER(_abi.dfmi_column))
        for j, a in enumerate(b.columns):
            assert as_tuple(cols[j]) == as_tuple(column_struct(a)), (i, j)


class Lazy(LazyColumns):
    def __init__(self, cols):
        self.cols, self.num_columns, self.num_rows = cols, len(cols), cols[0].length

    def materialize(self):
        return self.cols


def test_lazy_columns_are_read():
    b = batches(1)[0]
    lazy = RecordBatch.lazy(Schema.empty(), Lazy(list(b.columns)))
    barr, keep = host_batch_structs([lazy], 4)
    cols = C.cast(barr[0].columns, C.POINTER(_abi.dfmi_column))
    assert [as_tuple(cols[j]) for j in range(4)] == [as_tuple(column_struct(a)) for a in b.columns]


def test_schema_mismatch_and_non_tensor_buffers_are_refused():
    bs = batches(2)
    with pytest.raises(ValueError):
        host_batch_structs([bs[0], RecordBatch(Schema.empty(), bs[1].columns[:2])], 4)
    bad = Array.from_numpy(DataType.Float64, np.arange(4.0))
    bad.values = np.zeros(32, np.uint8)  # not a torch tensor
    with pytest.raises(TypeError):
        host_batch_structs([RecordBatch(Schema.empty(), [bad])], 1)
