"""Query compiler on the CPU: the kernel source dfmi_filter_project would
launch is generated for many expression shapes and compiled with hipRTC for
gfx950 (no device needed), through the library's internal test hook
dfmi_internal_jit_check (exec.cpp). The GPU suite then runs the same code
against the oracle; this suite catches generator / skeleton breakage here."""
import ctypes as C
import random

import numpy as np
import pytest

from datafusion_amd import _abi
from datafusion_amd.arrow import Field, Schema
from datafusion_amd.execution.error import ExecutionError
from datafusion_amd.execution.expression import compile_scalar_expr
from datafusion_amd.logicalplan import BinaryExpr, Cast, Column, DataType, Float64, Int64, Literal, Operator, Utf8

S = Schema([Field("a", DataType.Int64, True), Field("b", DataType.Float64, True),
            Field("s", DataType.Utf8, True), Field("f", DataType.Boolean, True),
            Field("c", DataType.Float64, False), Field("i32", DataType.Int32, False)])
N = 1000


def _lib():
    L = _abi.lib()
    fn = L.dfmi_internal_jit_check
    fn.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.c_int32, C.POINTER(_abi.dfmi_batch),
                   C.POINTER(_abi.dfmi_out_column), C.c_uint32, C.c_int32, C.c_char_p, C.c_int64,
                   C.POINTER(_abi.dfmi_error)]
    fn.restype = C.c_int64
    return fn


class HostBatch:
    """Host buffers shaped like S (the hook only reads metadata)."""

    def __init__(self, schema, n=N):
        self.keep = []
        self.carr = (_abi.dfmi_column * len(schema.fields))()
        for i, f in enumerate(schema.fields):
            c = self.carr[i]
            c.type = int(f.data_type)
            c.length = n
            buf = np.zeros(n * 8 + 64, dtype=np.uint8)
            self.keep.append(buf)
            c.values = buf.ctypes.data
            if f.data_type == DataType.Utf8:
                offs = np.zeros(n + 1, dtype=np.int32)
                self.keep.append(offs)
                c.offsets = offs.ctypes.data
            if f.nullable:
                v = np.full((n + 63) // 64 * 8, 0xFF, dtype=np.uint8)
                v[0] = 0xFE
                self.keep.append(v)
                c.validity = v.ctypes.data
                c.null_count = 1
        self.batch = _abi.dfmi_batch(len(schema.fields), 0, n, self.carr)


def jit_check(schema, pred, projs, flags=0, compile_=False):
    hb = HostBatch(schema)
    p = compile_scalar_expr(None, pred, schema, flags) if pred is not None else None
    cp = [compile_scalar_expr(None, e, schema, flags) for e in projs]
    n_out = len(cp) if cp else len(schema.fields)
    outs = (_abi.dfmi_out_column * max(1, n_out))()
    bufs = []
    for o in range(n_out):
        b = np.zeros(N * 8 + 64, dtype=np.uint8)
        bufs.append(b)
        outs[o].values = outs[o].validity = outs[o].offsets = outs[o].data = b.ctypes.data
        outs[o].data_capacity = N * 8
    progs = (C.c_void_p * max(1, len(cp)))(*[x.handle.value for x in cp])
    err = _abi.dfmi_error()
    buf = C.create_string_buffer(1 << 20)
    rc = _lib()(p.handle if p else None, progs, len(cp), C.byref(hb.batch), outs, flags, int(compile_), buf,
                len(buf), C.byref(err))
    return rc, err.code, err.message.decode(), buf.value.decode()


def c2_query(k=0.5, m=0.5):
    pred = BinaryExpr(BinaryExpr(Column(0), Operator.Gt, Literal(Float64(k))), Operator.And,
                      BinaryExpr(Column(1), Operator.Lt, Literal(Float64(m))))
    projs = [Column(0), Column(1),
             BinaryExpr(BinaryExpr(Column(0), Operator.Multiply, Column(1)), Operator.Plus, Column(2))]
    return pred, projs


F3 = Schema([Field(c, DataType.Float64, False) for c in "abc"])


def test_hook_is_exported_but_not_in_header():
    assert hasattr(_abi.lib(), "dfmi_internal_jit_check")
    assert "dfmi_internal_jit_check" not in _abi.EXPORTED


def test_c2_kernel_compiles():
    pred, projs = c2_query()
    rc, code, msg, src = jit_check(F3, pred, projs, compile_=True)
    assert rc > 0, msg
    assert 'extern "C" __global__' in src and "void dfmi_filter_" in src
    # literals are kernel arguments: another k/m generates the same source
    rc2, _, _, src2 = jit_check(F3, *c2_query(0.1, 0.9))
    assert src2 == src


def test_projection_only_kernel_compiles():
    e = BinaryExpr(BinaryExpr(Column(0), Operator.Multiply, Column(1)), Operator.Gt, Column(4))
    rc, code, msg, src = jit_check(S, None, [e, Column(2), BinaryExpr(Column(0), Operator.Divide, Column(0))],
                                   compile_=True)
    assert rc > 0, msg


def test_utf8_gathers_many_channels_compile():
    # FilterRelation over a table with 11 Utf8 columns (all_types_flat.csv shape)
    fields = [Field("c%d" % i, DataType.Utf8, False) for i in range(11)] + [Field("x", DataType.Float64, False)]
    sch = Schema(fields)
    pred = BinaryExpr(Column(11), Operator.Gt, Literal(Float64(0.5)))
    rc, code, msg, src = jit_check(sch, pred, [], compile_=True)
    assert rc > 0, msg
    assert "NCH = 12" in src


def test_utf8_compare_extension_compiles():
    pred = BinaryExpr(BinaryExpr(Column(2), Operator.Eq, Literal(Utf8("w17"))), Operator.Or,
                      BinaryExpr(Column(2), Operator.NotEq, Column(2)))
    rc, code, msg, src = jit_check(S, pred, [Column(2), Column(1)], _abi.DFMI_FLAG_EXT_UTF8_COMPARE, compile_=True)
    assert rc > 0, msg


NARROW = [DataType.Int8, DataType.Int16, DataType.Int32, DataType.UInt8, DataType.UInt16, DataType.UInt32,
          DataType.UInt64, DataType.Float32]


@pytest.mark.parametrize("t", NARROW, ids=[t.name for t in NARROW])
def test_narrow_type_kernels_compile(t):
    """Every fixed-width type lowers to typed loads/compares/math/stores."""
    from datafusion_amd.logicalplan import ScalarValue
    sch = Schema([Field("x", t, True), Field("y", t, False), Field("z", DataType.Float64, False)])
    lit = Literal(ScalarValue(t, 2.5 if t == DataType.Float32 else 3))
    pred = BinaryExpr(BinaryExpr(BinaryExpr(Column(0), Operator.Divide, Column(1)), Operator.Lt, lit), Operator.Or,
                      BinaryExpr(Column(0), Operator.GtEq, Column(1)))
    projs = [Column(0), BinaryExpr(BinaryExpr(Column(0), Operator.Multiply, Column(1)), Operator.Minus, lit), Column(2)]
    rc, code, msg, src = jit_check(sch, pred, projs, _abi.DFMI_FLAG_EXT_GATHER_ALL, compile_=True)
    assert rc > 0, msg
    assert "%s c0[K]" % {DataType.Float32: "float"}.get(t, t.name.lower().replace("uint", "u").replace("int", "i")) in src
    rc, code, msg, src = jit_check(sch, None, projs[1:] + [BinaryExpr(Column(0), Operator.Eq, lit)], compile_=True)
    assert rc > 0, msg


def _rand_expr(rng, depth, boolean=False):
    if boolean:
        if depth == 0 or rng.random() < 0.5:
            op = rng.choice([Operator.Eq, Operator.NotEq, Operator.Lt, Operator.LtEq, Operator.Gt, Operator.GtEq])
            t = rng.choice([0, 1])
            return BinaryExpr(_rand_expr(rng, depth - 1, False) if t else Column(rng.choice([0, 1, 4])), op,
                              _rand_expr(rng, max(0, depth - 1), False))
        return BinaryExpr(_rand_expr(rng, depth - 1, True), rng.choice([Operator.And, Operator.Or]),
                          _rand_expr(rng, depth - 1, True))
    if depth <= 0 or rng.random() < 0.3:
        k = rng.random()
        if k < 0.6:
            return Column(rng.choice([0, 1, 4]))
        if k < 0.8:
            return Literal(Int64(rng.randrange(-1000, 1000)))
        return Literal(Float64(rng.choice([0.5, -2.25, 0.0, 3.0])))
    op = rng.choice([Operator.Plus, Operator.Minus, Operator.Multiply, Operator.Divide])
    return BinaryExpr(_rand_expr(rng, depth - 1), op, _rand_expr(rng, depth - 1))


def _coerced(e):
    """Insert the casts the SQL planner would (Int64 op Float64 -> Float64)."""
    from datafusion_amd.logicalplan import binary_expr_coerced
    if isinstance(e, BinaryExpr):
        return binary_expr_coerced(_coerced(e.left), e.op, _coerced(e.right), S)
    return e


def test_random_shapes_generate_and_sample_compiles():
    rng = random.Random(7)
    generated = compiled = 0
    seen = set()
    for i in range(600):
        try:
            pred = _coerced(_rand_expr(rng, rng.randrange(1, 4), True))
            projs = [_coerced(_rand_expr(rng, rng.randrange(0, 3))) for _ in range(rng.randrange(0, 4))]
            compile_scalar_expr(None, pred, S)
            for p in projs:
                compile_scalar_expr(None, p, S)
        except ExecutionError:
            continue
        do_compile = len(seen) < 12
        rc, code, msg, src = jit_check(S, pred, projs, compile_=False)
        if rc < 0:
            # only reference errors or documented device limits, never a generator failure
            assert code in (_abi.DFMI_ERR_EXECUTION, _abi.DFMI_ERR_NOT_IMPLEMENTED), (msg, repr(pred))
            continue
        generated += 1
        if do_compile and src not in seen:
            seen.add(src)
            rc, code, msg, _ = jit_check(S, pred, projs, compile_=True)
            assert rc > 0, (msg, repr(pred), [repr(p) for p in projs])
            compiled += 1
    assert generated > 150 and compiled >= 10


def test_cast_and_is_null_kernels_compile():
    from datafusion_amd.logicalplan import IsNotNull, IsNull
    types = [DataType.Int8, DataType.UInt16, DataType.Int32, DataType.UInt64, DataType.Float32, DataType.Float64]
    sch = Schema([Field("x%d" % i, t, True) for i, t in enumerate(types)] + [Field("s", DataType.Utf8, True)])
    fl = _abi.DFMI_FLAG_EXT_CAST | _abi.DFMI_FLAG_EXT_IS_NULL | _abi.DFMI_FLAG_EXT_GATHER_ALL
    projs = [Cast(Column(i), u) for i in range(len(types)) for u in types[:2]]
    rc, code, msg, src = jit_check(sch, None, projs[:12], fl, compile_=True)
    assert rc > 0, msg
    assert "num_cast" in src
    pred = BinaryExpr(IsNull(Column(6)), Operator.Or,
                      BinaryExpr(Cast(Column(4), DataType.Int64), Operator.Gt, Cast(Column(0), DataType.Int64)))
    rc, code, msg, src = jit_check(sch, pred, [IsNotNull(Column(1)), Cast(Column(5), DataType.UInt8)], fl, compile_=True)
    assert rc > 0, msg
    # without the flags the reference's compile errors stand
    with pytest.raises(ExecutionError) as e:
        compile_scalar_expr(None, Cast(Column(0), DataType.Int64), sch)
    assert e.value.message == "column reference"


@pytest.mark.parametrize("m", [2, 8])
def test_numeric_subtile_kernel_compiles(m, monkeypatch):
    """The low-selectivity form of a numeric predicate (exec.cpp kLowSel:
    sub-tiles sharing one look-back, output pass reloading the selected rows'
    columns), forced through the diagnostic knob; nullable inputs, a
    fallible projection and a Q6-style 5-term predicate."""
    monkeypatch.setenv("DFMI_DIAG", "1")
    monkeypatch.setenv("DFMI_NUMERIC_SUBTILES", str(m))
    pred, projs = c2_query()
    rc, code, msg, src = jit_check(F3, pred, projs, compile_=True)
    assert rc > 0, msg
    assert "constexpr int M = %d;" % m in src and "SLR" in src
    e = BinaryExpr(BinaryExpr(Column(0), Operator.Lt, Literal(Int64(3))), Operator.And,
                   BinaryExpr(Column(1), Operator.GtEq, Column(4)))
    rc, code, msg, src = jit_check(S, e, [BinaryExpr(Column(4), Operator.Divide, Column(1)), Column(1), Column(2)],
                                   compile_=True)
    assert rc > 0, msg  # (Utf8 output: not a numeric sub-tile kernel, still compiles)
    rc, code, msg, src = jit_check(S, e, [BinaryExpr(Column(4), Operator.Divide, Column(1)), Column(1)],
                                   compile_=True)
    assert rc > 0, msg
    assert "constexpr int M = %d;" % m in src
