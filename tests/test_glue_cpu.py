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


def fake_block(nb, nout, n):
    """A HostResultBlock over a host tensor: batch b, column o holds the
    float64 values b*100 + o*10 + i (i < n), no nulls."""
    import torch
    from datafusion_amd.execution.engine import HostResultBlock
    blk = HostResultBlock.__new__(HostResultBlock)
    per = ((n * 8 + 255) // 256) * 256
    vals = np.zeros(nb * nout * per // 8, np.float64)
    for b in range(nb):
        for o in range(nout):
            k = (b * nout + o) * per // 8
            vals[k:k + n] = b * 100 + o * 10 + np.arange(n)
    blk.block = torch.from_numpy(vals.view(np.uint8))
    blk.base = blk.block.data_ptr()
    blk.end = blk.base + blk.block.numel()
    m = nb * nout
    blk.type, blk.length, blk.nulls = [DataType.Float64] * m, [n] * m, [0] * m
    blk.validity, blk.offsets = [0] * m, [0] * m
    blk.values = [blk.base + k * per for k in range(m)]
    return blk


def test_host_result_batch():
    """The relations' one-object-per-batch result (engine.HostResultBatch):
    row / column counts without building Arrays, Arrays on first read (views
    of the block), the columns setter, and the glue reading it as input."""
    from datafusion_amd.execution.engine import HostResultBatch
    blk = fake_block(3, 2, 5)
    rb = HostResultBatch.make(Schema.empty(), blk, 1, 2)
    assert rb.num_rows() == 5 and rb.num_columns() == 2 and rb._cols is None
    assert [list(c.numpy_values()) for c in rb.columns] == [[100.0 + i for i in range(5)], [110.0 + i for i in range(5)]]
    barr, keep = host_batch_structs([rb], 2)
    cols = C.cast(barr[0].columns, C.POINTER(_abi.dfmi_column))
    assert [as_tuple(cols[j]) for j in range(2)] == [as_tuple(column_struct(a)) for a in rb.columns]
    rb.columns = rb.columns[:1]
    assert rb.num_columns() == 1 and rb.num_rows() == 5


def test_make_block_batches():
    """_dfmi_glue.make_block_batches (the relations' caller-owned output path):
    BlockArrays over one host block from dfmi_out_column records -- Float64,
    Boolean, nullable, Utf8 and a passthrough column (the input batch's own
    Array) -- each buffer a 64-byte padded range of the block, viewed on first
    read; the struct packing reads a BlockArray's pointers without viewing."""
    import torch
    from datafusion_amd import _dfmi_glue
    from datafusion_amd.arrow import BlockArray
    from datafusion_amd.execution.engine import _DTYPES, _OUT_DTYPE
    blk = torch.zeros(4096, dtype=torch.uint8)
    base = blk.data_ptr()
    f = np.array([1.5, -2.0, 3.25], np.float64)
    blk[0:24] = torch.from_numpy(f.view(np.uint8))
    blk[256] = 0b101  # Boolean values: t f t
    blk[512] = 0b011  # validity: v v n
    offs = np.array([0, 2, 2, 5], np.int32)
    blk[768:784] = torch.from_numpy(offs.view(np.uint8))
    blk[1024:1029] = torch.tensor(list(b"abxyz"), dtype=torch.uint8)
    outs = np.zeros(4, _OUT_DTYPE)
    outs[0] = (base, base + 512, 0, 0, 0, int(DataType.Float64), -1, 3, 1, 0)
    outs[1] = (base + 256, 0, 0, 0, 0, int(DataType.Boolean), -1, 3, 0, 0)
    outs[2] = (0, 0, base + 768, base + 1024, 5, int(DataType.Utf8), -1, 3, 0, 5)
    outs[3] = (0, 0, 0, 0, 0, int(DataType.Int32), 1, 3, 0, 0)
    src = RecordBatch(Schema.empty(), [Array.from_numpy(DataType.Float64, np.zeros(3)),
                                       Array.from_numpy(DataType.Int32, np.array([7, 8, 9], np.int32))])
    (rb,) = _dfmi_glue.make_block_batches(RecordBatch, BlockArray, Schema.empty(), blk, outs, 1, 4, [src], _DTYPES)
    a, b, u, p = rb.columns
    assert type(a) is BlockArray and a.data_type == DataType.Float64 and a.length == 3 and a.null_count == 1
    assert "values" not in a.__dict__
    # the packing reads pointers without making the views
    barr, keep = host_batch_structs([rb], 4)
    cols = C.cast(barr[0].columns, C.POINTER(_abi.dfmi_column))
    assert (cols[0].values, cols[0].validity, cols[2].offsets, cols[2].values) == (base, base + 512, base + 768,
                                                                                    base + 1024)
    assert cols[3].values == src.columns[1].values.data_ptr()
    assert "values" not in a.__dict__
    assert a.to_pylist() == [1.5, -2.0, None]
    assert a.values.numel() == 64 and a.values.data_ptr() == base
    assert b.to_pylist() == [True, False, True] and b.validity is None
    assert u.to_pylist() == ["ab", "", "xyz"] and u.offsets.dtype == torch.int32
    assert p is src.columns[1]
    assert as_tuple(cols[0]) == as_tuple(column_struct(a))
