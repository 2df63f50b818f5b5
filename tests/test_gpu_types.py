"""GPU parity for every fixed-width type the reference's comparison_ops! and
math_ops! accept (expression.rs:133-163, 174-203): Int8/16/32/64,
UInt8/16/32/64, Float32, Float64 -- comparisons with arrow 0.12 null ordering,
wrapping integer + - *, truncating division with DivideByZero and the
iN::MIN / -1 panic, Float32 with one rounding per operator. The device
(through the C ABI) is checked against the CPU oracle on the same inputs, and
on the reference's own fixtures (numerics_<op>.csv col 4, c_int8/16/32_*,
c_float32_*) against the expected files."""
import numpy as np
import pytest

from datafusion_amd._abi import DFMI_FLAG_EXT_GATHER_ALL
from datafusion_amd.arrow import Array, Field, RecordBatch, Schema, np_dtype
from datafusion_amd.logicalplan import BinaryExpr, Column, DataType, Literal, Operator, ScalarValue
from golden_cases import ALL_TYPES, ALL_TYPES_NARROW, expected_rows, fixture_values, load_batch, narrow_fixture_case
from test_gpu_parity import CMP, MATH, run_both

pytestmark = pytest.mark.gpu

INT_TYPES = [DataType.Int8, DataType.Int16, DataType.Int32, DataType.Int64,
             DataType.UInt8, DataType.UInt16, DataType.UInt32, DataType.UInt64]
TYPES = INT_TYPES + [DataType.Float32, DataType.Float64]
GA = DFMI_FLAG_EXT_GATHER_ALL


def typed_values(t, n, rng):
    """Random values of type t over its whole range, with edge values mixed in."""
    dt = np.dtype(np_dtype(t))
    if t in (DataType.Float32, DataType.Float64):
        v = (rng.standard_normal(n) * 10.0 ** rng.integers(-3, 4, n)).astype(dt)
        edge = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.finfo(dt).max, np.finfo(dt).tiny,
                         np.finfo(dt).tiny / 4, 0.5, 3.0], dtype=dt)
    else:
        info = np.iinfo(dt)
        v = rng.integers(info.min, info.max, n, dtype=dt, endpoint=True)
        small = rng.integers(-4 if info.min < 0 else 0, 5, n).astype(dt)
        v = np.where(rng.random(n) < 0.3, small, v)
        edge = np.array([info.min, info.max, 0, 1, info.max - 1] + ([-1] if info.min < 0 else []), dtype=dt)
    pos = rng.integers(0, n, len(edge) * 4)
    v[pos] = np.tile(edge, 4)
    return v


def typed_table(t, n, seed, null_frac=0.2, nonzero=(), no_min_neg1=False):
    rng = np.random.default_rng(seed)
    cols, fields = [], []
    vals = [typed_values(t, n, rng) for _ in range(3)]
    for j in nonzero:  # divisors
        vals[j][vals[j] == 0] = 1
        if no_min_neg1 and t in INT_TYPES[:4]:
            vals[j][vals[j] == -1] = 2
    for j, name in enumerate("abc"):
        valid = rng.random(n) >= null_frac if null_frac else None
        cols.append(Array.from_numpy(t, vals[j], valid))
        fields.append(Field(name, t, bool(null_frac)))
    s = Schema(fields)
    return s, RecordBatch(s, cols), vals


def lit_of(t, x):
    return Literal(ScalarValue(t, x))


@pytest.mark.parametrize("t", TYPES, ids=[t.name for t in TYPES])
def test_comparisons_every_type(t):
    """a op b / a op lit / lit op b for every comparison, with nulls, as a
    predicate (gathering a, c of the same type) and as a projected Boolean."""
    s, b, _ = typed_table(t, 20_000, seed=int(t) * 7)
    lit = lit_of(t, 0.5 if t in (DataType.Float32, DataType.Float64) else 3)
    for op in CMP:
        run_both(s, b, BinaryExpr(Column(0), op, Column(1)), [Column(0), Column(2)], GA)
        run_both(s, b, BinaryExpr(Column(0), op, lit), [Column(1)], GA)
        run_both(s, b, BinaryExpr(lit, op, Column(1)), [Column(0)], GA)
        run_both(s, b, None, [BinaryExpr(Column(0), op, Column(1))], GA)
    # FilterRelation output (every column gathered)
    run_both(s, b, BinaryExpr(Column(0), Operator.Lt, Column(2)), [], GA)
    # without the extension only Float64 can be gathered (filter.rs:106-110)
    assert (run_both(s, b, BinaryExpr(Column(0), Operator.Lt, Column(2)), [Column(1)]) is None) == \
        (t != DataType.Float64)


@pytest.mark.parametrize("t", TYPES, ids=[t.name for t in TYPES])
def test_math_every_type(t):
    """+ - * / with null propagation (projection only: validity bitmaps and
    null counts), in a predicate, and over the filtered rows."""
    s, b, _ = typed_table(t, 20_000, seed=int(t) * 11, nonzero=(1, 2), no_min_neg1=True)
    lit = lit_of(t, 2.5 if t in (DataType.Float32, DataType.Float64) else 7)
    for op in MATH:
        run_both(s, b, None, [BinaryExpr(Column(0), op, Column(1)), BinaryExpr(Column(0), op, lit)], GA)
        run_both(s, b, BinaryExpr(BinaryExpr(Column(0), op, Column(1)), Operator.Lt, BinaryExpr(Column(2), op, lit)),
                 [BinaryExpr(BinaryExpr(Column(0), op, Column(2)), Operator.Plus, Column(1)), Column(0)], GA)
    e = BinaryExpr(BinaryExpr(Column(0), Operator.Multiply, Column(1)), Operator.Minus,
                   BinaryExpr(Column(2), Operator.Divide, BinaryExpr(Column(1), Operator.Plus, Column(1))))
    run_both(s, b, None, [e], GA)


@pytest.mark.parametrize("t", TYPES, ids=[t.name for t in TYPES])
def test_division_errors_every_type(t):
    """A non-null zero divisor is ArrowError(DivideByZero); iN::MIN / -1 is the
    Rust panic; rows a Selection drops never raise."""
    n = 5000
    dt = np.dtype(np_dtype(t))
    a = np.arange(n).astype(dt)
    d = np.ones(n, dtype=dt)
    d[3000] = 0
    s = Schema([Field("a", t, False), Field("d", t, False)])
    b = RecordBatch(s, [Array.from_numpy(t, a), Array.from_numpy(t, d)])
    assert run_both(s, b, None, [BinaryExpr(Column(0), Operator.Divide, Column(1))], GA) is None
    keep = BinaryExpr(Column(0), Operator.Lt, lit_of(t, 100))
    run_both(s, b, keep, [BinaryExpr(Column(0), Operator.Divide, Column(1))], GA)
    if t in INT_TYPES[:4]:
        a2, d2 = a.copy(), np.ones(n, dtype=dt)
        a2[10], d2[10] = np.iinfo(dt).min, -1
        b2 = RecordBatch(s, [Array.from_numpy(t, a2), Array.from_numpy(t, d2)])
        assert run_both(s, b2, None, [BinaryExpr(Column(0), Operator.Divide, Column(1))], GA) is None
        # the panic row filtered out: no error, wrapping values elsewhere
        run_both(s, b2, BinaryExpr(Column(0), Operator.Gt, lit_of(t, 20)),
                 [BinaryExpr(Column(0), Operator.Divide, Column(1))], GA)


@pytest.mark.parametrize("opname,op", [("plus", Operator.Plus), ("minus", Operator.Minus),
                                       ("multiply", Operator.Multiply), ("divide", Operator.Divide)])
def test_numerics_float32_on_gpu(opname, op):
    """expected/numerics_<op>.csv column 4 = a_f OP b_f in Float32, bit-exact."""
    S = Schema([Field("a", DataType.Int64, False), Field("b", DataType.Int64, False),
                Field("a_f", DataType.Float32, False), Field("b_f", DataType.Float32, False)])
    batch = load_batch(S, "numerics.csv", has_header=True)
    dev, _ = run_both(S, batch, None, [BinaryExpr(Column(2), op, Column(3)), BinaryExpr(Column(0), op, Column(1))])
    got = dev[0].cpu().numpy_values()
    exp = np.array([np.float32(e[3]) for e in expected_rows("numerics_%s.csv" % opname)], dtype=np.float32)
    assert got.dtype == np.float32 and np.array_equal(got.view(np.uint32), exp.view(np.uint32))
    assert dev[1].cpu().to_pylist() == [int(e[0]) for e in expected_rows("numerics_%s.csv" % opname)]


@pytest.mark.parametrize("case", ALL_TYPES_NARROW, ids=[c[0] for c in ALL_TYPES_NARROW])
def test_all_types_narrow_on_gpu(case):
    """expected/c_int{8,16,32}_*.csv and c_float32_{high,low}.csv on the device."""
    name, col, op, lit = case
    s, pred, projs = narrow_fixture_case(*case)
    batch = load_batch(s, "all_types_flat.csv", has_header=False)
    assert run_both(s, batch, pred, projs) is None  # "filter not supported for <type>"
    dev, _ = run_both(s, batch, pred, projs, GA)
    assert dev[0].cpu().to_pylist() == fixture_values(name, ALL_TYPES[col])
    run_both(s, batch, pred, [], GA)  # FilterRelation output: 11 Utf8 gathers + the typed column


def test_all_columns_typed_on_gpu():
    """all_types_flat.csv with every column at its real type: comparisons of
    each fixed-width column against the one beside it of the same type are
    not possible, so compare each against itself shifted by a literal and
    gather every column (10 fixed-width + Boolean + Utf8 outputs)."""
    from golden_cases import all_types_schema
    s = all_types_schema(typed={i: t for i, t in enumerate(ALL_TYPES)})
    batch = load_batch(s, "all_types_flat.csv", has_header=False)
    for col in range(1, 11):
        t = ALL_TYPES[col]
        lit = lit_of(t, 0.5 if t in (DataType.Float32, DataType.Float64) else 1)
        run_both(s, batch, BinaryExpr(Column(col), Operator.Gt, lit), [], GA)
        run_both(s, batch, None, [BinaryExpr(Column(col), Operator.Plus, lit), BinaryExpr(Column(col), Operator.LtEq, lit)])


# ------------------------------------------------ CAST / IS NULL extensions
from datafusion_amd._abi import DFMI_FLAG_EXT_CAST, DFMI_FLAG_EXT_IS_NULL  # noqa: E402
from datafusion_amd.logicalplan import Cast, IsNotNull, IsNull  # noqa: E402
from golden_cases import (ALL_TYPES_CAST, NULL_CASES, NULL_TEST, cast_fixture_case,  # noqa: E402
                          sql_plan)

EXT = GA | DFMI_FLAG_EXT_CAST | DFMI_FLAG_EXT_IS_NULL


@pytest.mark.parametrize("case", ALL_TYPES_CAST, ids=[c[0] for c in ALL_TYPES_CAST])
def test_all_types_cast_on_gpu(case):
    """expected/c_*_cast.csv and c_int8_col_*.csv: planner-inserted CAST(column)."""
    name, cols, sql = case
    s, pred, projs = cast_fixture_case(*case)
    batch = load_batch(s, "all_types_flat.csv", has_header=False)
    dev, _ = run_both(s, batch, pred, projs, EXT)
    assert dev[0].cpu().to_pylist() == fixture_values(name, ALL_TYPES[cols[0]])
    if "CAST(" in repr(pred) + repr(projs):
        assert run_both(s, batch, pred, projs, GA) is None  # "column reference" without the flag


@pytest.mark.parametrize("name,sql", NULL_CASES)
def test_is_null_on_gpu(name, sql):
    batch = load_batch(NULL_TEST, "null_test.csv", has_header=True)
    pred, projs = sql_plan(sql, NULL_TEST, "null_test")
    dev, _ = run_both(NULL_TEST, batch, pred, projs, EXT)
    assert dev[0].cpu().to_pylist() == [int(r[0]) for r in expected_rows(name)]
    assert run_both(NULL_TEST, batch, pred, projs, GA) is None  # "expression #1 IS NULL"


@pytest.mark.parametrize("t", TYPES, ids=[t.name for t in TYPES])
def test_cast_every_pair(t):
    """CAST from t to every numeric type over the whole value range (edge
    values, NaN/inf for floats, nulls): values that do not fit become nulls,
    as a projection (dense kernel) and inside a predicate."""
    s, b, _ = typed_table(t, 20_000, seed=int(t) * 13)
    run_both(s, b, None, [Cast(Column(0), u) for u in TYPES], EXT)
    for u in TYPES:
        pred = BinaryExpr(Cast(Column(0), u), Operator.GtEq, Cast(Column(1), u))
        run_both(s, b, pred, [Cast(Column(2), u), Column(0)], EXT)
    # nested: CAST of arithmetic, arithmetic over casts
    e = BinaryExpr(Cast(BinaryExpr(Column(0), Operator.Plus, Column(1)), DataType.Float64), Operator.Multiply,
                   Cast(Column(2), DataType.Float64))
    run_both(s, b, None, [e, Cast(Cast(Column(0), DataType.Int16), DataType.Float32)], EXT)


def test_is_null_every_type():
    """IS NULL / IS NOT NULL of columns of every type (incl. Utf8 and
    Boolean) and of null-propagating expressions, as predicate and projection;
    after a Selection the batch has no nulls (filter() drops validity)."""
    rng = np.random.default_rng(5)
    n = 30_000
    cols, fields = [], []
    for i, t in enumerate(TYPES):
        cols.append(Array.from_numpy(t, typed_values(t, n, rng), rng.random(n) >= 0.25))
        fields.append(Field("x%d" % i, t, True))
    strs = [None if rng.random() < 0.2 else b"s%d" % (i % 97) for i in range(n)]
    cols.append(Array.from_strings(strs))
    fields.append(Field("s", DataType.Utf8, True))
    cols.append(Array.from_numpy(DataType.Boolean, rng.random(n) < 0.5, rng.random(n) >= 0.3))
    fields.append(Field("f", DataType.Boolean, True))
    s = Schema(fields)
    bt = RecordBatch(s, cols)
    nc = len(fields)
    run_both(s, bt, None, [IsNull(Column(i)) for i in range(nc)] + [IsNotNull(Column(0))], EXT)
    for i in range(nc):
        run_both(s, bt, IsNull(Column(i)), [Column(9), IsNull(Column(9))], EXT)
        run_both(s, bt, IsNotNull(Column(i)), [Column(10), Column(3)], EXT)
    e = BinaryExpr(Column(2), Operator.Multiply, Column(2))
    run_both(s, bt, BinaryExpr(IsNull(e), Operator.Or, BinaryExpr(Column(9), Operator.Gt, Column(9))),
             [IsNotNull(e), e], EXT)


# ---------------------------------------------------------- round-3 fixtures
from golden_cases import RANGE_CASES, WHOLE_F32_FILES, range_fixture_case, whole_f32_case  # noqa: E402


@pytest.mark.parametrize("case", RANGE_CASES, ids=[c[0] for c in RANGE_CASES])
def test_int8_range_inclusive_on_gpu(case):
    """expected/c_int8_range_inclusive.csv (98 rows) on the device."""
    s, pred, projs = range_fixture_case(*case)
    batch = load_batch(s, "all_types_flat.csv", has_header=False)
    assert run_both(s, batch, pred, projs) is None  # "filter not supported for Int8"
    dev, _ = run_both(s, batch, pred, projs, GA)
    assert dev[0].cpu().to_pylist() == fixture_values(case[0], ALL_TYPES[case[1]])


@pytest.mark.parametrize("name", WHOLE_F32_FILES)
def test_float32_uint32_files_on_gpu(name):
    """expected/c_float32_*_uint32.csv: the whole c_float32 column (CAST(c9 AS UInt32) = 0)."""
    s, pred, projs = whole_f32_case()
    batch = load_batch(s, "all_types_flat.csv", has_header=False)
    dev, _ = run_both(s, batch, pred, projs, EXT)
    assert dev[0].cpu().to_pylist() == fixture_values(name, DataType.Float32)
