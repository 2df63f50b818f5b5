"""The hipRTC module cache is bounded (jit.cpp `compile`, least recently used
evicted): with the bound at 2 modules, four query shapes in turn leave at most
2 loaded, and a shape whose module was evicted is compiled again and still
returns the oracle's result (its shape-cache entry went stale with it)."""
import ctypes as C

import pytest


@pytest.mark.gpu
def test_module_cache_bound_and_recompile():
    from datafusion_amd import _abi
    from datafusion_amd.arrow import Array, Field, RecordBatch, Schema
    from datafusion_amd.execution.engine import engine
    from datafusion_amd.execution.expression import compile_scalar_expr
    from datafusion_amd.logicalplan import BinaryExpr, Column, DataType, Float64, Literal, Operator
    from oracle_ffi import gen_unit_f64, oracle_filter_project
    from test_gpu_parity import assert_same

    L = _abi.lib()
    L.dfmi_internal_jit_cache.argtypes = [C.c_int64]
    L.dfmi_internal_jit_cache.restype = C.c_int64
    n = 100_003
    s = Schema([Field(c, DataType.Float64, False) for c in "ab"])
    b = RecordBatch(s, [Array.from_numpy(DataType.Float64, gen_unit_f64(11, j, 0, n)) for j in range(2)])
    ops = [Operator.Lt, Operator.Gt, Operator.LtEq, Operator.GtEq]
    eng = engine()
    try:
        assert L.dfmi_internal_jit_cache(2) <= 2
        for rnd in range(2):
            for op in ops:
                pred_e = BinaryExpr(Column(0), op, Literal(Float64(0.25 + 0.1 * rnd)))
                proj_e = [Column(1), BinaryExpr(Column(0), Operator.Multiply, Column(1))]
                ref = oracle_filter_project(s, b, pred_e, proj_e)
                out = eng.filter_project(compile_scalar_expr(None, pred_e, s),
                                         [compile_scalar_expr(None, e, s) for e in proj_e], b)
                for d, (_, r) in zip(out, ref):
                    assert_same(d.cpu(), r)
                assert L.dfmi_internal_jit_cache(0) <= 2
    finally:
        L.dfmi_internal_jit_cache(256)
