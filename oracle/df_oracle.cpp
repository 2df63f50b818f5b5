// TEST INFRASTRUCTURE ONLY — see oracle.h. CPU restatement of the reference's
// Selection + Projection path, written the reference's way on purpose: every
// operator is its own materialising pass, literals are broadcast to full arrays
// per batch, results are built with builder-style pushes that maintain a
// validity bitmap (arrow 0.12 PrimitiveArrayBuilder), scalar loops only.
// That makes it both the parity checker and the honest single-core CPU
// baseline ("port" of the reference, which cannot be compiled here: no Rust).
//
// Reference lines restated (under /root/reference):
//   compile_scalar_expr            src/execution/expression.rs:244-451
//   literal_array!                 src/execution/expression.rs:224-241
//   comparison_ops!/math_ops!      src/execution/expression.rs:121-208
//   boolean_ops!                   src/execution/expression.rs:210-222
//   FilterRelation::next, filter() src/execution/filter.rs:46-111
//   ProjectRelation::next          src/execution/projection.rs:45-66
//   Expr Debug (output names)      src/logicalplan.rs:263-303
//   arrow 0.12 array_ops bool_op / math_op / and / or (third-party crate
//   datafusion-arrow 0.12.4, Cargo.toml:36, not vendored; semantics in
//   SURVEY.md §8c).
//
// Compile: g++ -O2 -ffp-contract=off (see oracle/Makefile).

#include "oracle.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <functional>
#include <limits>
#include <type_traits>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace {

// ---------------------------------------------------------------- errors ---
struct ExecError {
    int32_t code;
    std::string msg;
};
[[noreturn]] void fail(int32_t code, const std::string& m) { throw ExecError{code, m}; }

// ------------------------------------------------------------ data types ---
bool is_numeric(int t) { return t >= DFMI_TYPE_INT8 && t <= DFMI_TYPE_FLOAT64; }
int type_width(int t) {
    switch (t) {
        case DFMI_TYPE_INT8: case DFMI_TYPE_UINT8: return 1;
        case DFMI_TYPE_INT16: case DFMI_TYPE_UINT16: return 2;
        case DFMI_TYPE_INT32: case DFMI_TYPE_UINT32: case DFMI_TYPE_FLOAT32: return 4;
        case DFMI_TYPE_INT64: case DFMI_TYPE_UINT64: case DFMI_TYPE_FLOAT64: return 8;
        default: return 0;
    }
}
const char* type_name(int t) {  // arrow DataType Debug
    switch (t) {
        case DFMI_TYPE_BOOLEAN: return "Boolean";
        case DFMI_TYPE_INT8: return "Int8";
        case DFMI_TYPE_INT16: return "Int16";
        case DFMI_TYPE_INT32: return "Int32";
        case DFMI_TYPE_INT64: return "Int64";
        case DFMI_TYPE_UINT8: return "UInt8";
        case DFMI_TYPE_UINT16: return "UInt16";
        case DFMI_TYPE_UINT32: return "UInt32";
        case DFMI_TYPE_UINT64: return "UInt64";
        case DFMI_TYPE_FLOAT32: return "Float32";
        case DFMI_TYPE_FLOAT64: return "Float64";
        case DFMI_TYPE_UTF8: return "Utf8";
        default: return "Null";
    }
}

// ---------------------------------------------- Rust float formatting -----
// Shortest round-trip digits, printed in plain decimal (Rust 2018 float
// Display / Debug never use exponents). debug=true appends ".0" to integral
// values, like `{:?}`.
std::string shortest_digits(double v, bool is_f32, int* exp10) {
    char buf[64];
    for (int p = 1; p <= 17; ++p) {
        snprintf(buf, sizeof buf, "%.*e", p - 1, v);
        bool ok = is_f32 ? (float)strtod(buf, nullptr) == (float)v : strtod(buf, nullptr) == v;
        if (ok) break;
    }
    // buf = d.ddddde[+-]XX
    std::string s(buf);
    size_t e = s.find('e');
    *exp10 = atoi(s.c_str() + e + 1);
    std::string digits;
    for (size_t i = 0; i < e; ++i)
        if (s[i] >= '0' && s[i] <= '9') digits.push_back(s[i]);
    while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
    return digits;
}
std::string rust_float(double v, bool is_f32, bool debug) {
    if (std::isnan(v)) return "NaN";
    if (std::isinf(v)) return v > 0 ? "inf" : "-inf";
    std::string sign = (std::signbit(v) && (v != 0.0 || debug)) ? "-" : "";
    double a = std::fabs(v);
    if (a == 0.0) return sign + (debug ? "0.0" : "0");
    int e10;
    std::string d = shortest_digits(a, is_f32, &e10);
    std::string out;
    int point = e10 + 1;  // digits before the decimal point
    if (point <= 0) {
        out = "0." + std::string(-point, '0') + d;
    } else if ((size_t)point >= d.size()) {
        out = d + std::string(point - d.size(), '0');
        if (debug) out += ".0";
    } else {
        out = d.substr(0, point) + "." + d.substr(point);
    }
    return sign + out;
}

std::string rust_str_debug(const char* s, int64_t n) {
    std::string o = "\"";
    for (int64_t i = 0; i < n; ++i) {
        unsigned char c = (unsigned char)s[i];
        switch (c) {
            case '"': o += "\\\""; break;
            case '\\': o += "\\\\"; break;
            case '\n': o += "\\n"; break;
            case '\r': o += "\\r"; break;
            case '\t': o += "\\t"; break;
            case '\0': o += "\\0"; break;
            default:
                if (c < 0x20 || c == 0x7f) {
                    char b[16];
                    snprintf(b, sizeof b, "\\u{%x}", c);
                    o += b;
                } else {
                    o.push_back((char)c);
                }
        }
    }
    return o + "\"";
}

// ---------------------------------------------------------- expressions ---
// The postfix node array rebuilt into a tree (logicalplan::Expr).
struct Expr {
    const dfmi_expr_node* n;
    std::vector<std::shared_ptr<Expr>> kids;
};
using ExprP = std::shared_ptr<Expr>;

ExprP build_tree(const dfmi_expr_node* nodes, int32_t len) {
    if (!nodes || len <= 0) fail(DFMI_ERR_INVALID_ARGUMENT, "empty expression");
    std::vector<ExprP> st;
    for (int32_t i = 0; i < len; ++i) {
        auto e = std::make_shared<Expr>();
        e->n = &nodes[i];
        int arity = 0;
        switch (nodes[i].kind) {
            case DFMI_EXPR_COLUMN: case DFMI_EXPR_LITERAL: arity = 0; break;
            case DFMI_EXPR_BINARY: arity = 2; break;
            case DFMI_EXPR_CAST: case DFMI_EXPR_IS_NULL: case DFMI_EXPR_IS_NOT_NULL:
            case DFMI_EXPR_SORT: arity = 1; break;
            case DFMI_EXPR_SCALAR_FUNCTION: case DFMI_EXPR_AGGREGATE_FUNCTION:
                arity = nodes[i].column; break;
            default: fail(DFMI_ERR_INVALID_ARGUMENT, "bad expression node kind");
        }
        if (arity < 0 || (int)st.size() < arity) fail(DFMI_ERR_INVALID_ARGUMENT, "malformed postfix");
        e->kids.assign(st.end() - arity, st.end());
        st.resize(st.size() - arity);
        st.push_back(e);
    }
    if (st.size() != 1) fail(DFMI_ERR_INVALID_ARGUMENT, "malformed postfix");
    return st[0];
}

const char* op_name(int op) {
    static const char* n[] = {"Eq", "NotEq", "Lt", "LtEq", "Gt", "GtEq", "Plus",
                              "Minus", "Multiply", "Divide", "Modulus", "And", "Or"};
    return (op >= 0 && op <= 12) ? n[op] : "?";
}

std::string scalar_debug(const dfmi_expr_node* n) {  // ScalarValue derive(Debug)
    char b[64];
    switch (n->data_type) {
        case DFMI_TYPE_NULL: return "Null";
        case DFMI_TYPE_BOOLEAN: return std::string("Boolean(") + (n->i64 ? "true" : "false") + ")";
        case DFMI_TYPE_FLOAT32: return "Float32(" + rust_float(n->f64, true, true) + ")";
        case DFMI_TYPE_FLOAT64: return "Float64(" + rust_float(n->f64, false, true) + ")";
        case DFMI_TYPE_UTF8: return "Utf8(" + rust_str_debug(n->str, n->str_len) + ")";
        case DFMI_TYPE_UINT8: case DFMI_TYPE_UINT16: case DFMI_TYPE_UINT32: case DFMI_TYPE_UINT64:
            snprintf(b, sizeof b, "%s(%llu)", type_name(n->data_type), (unsigned long long)n->i64);
            return b;
        default:
            snprintf(b, sizeof b, "%s(%lld)", type_name(n->data_type), (long long)n->i64);
            return b;
    }
}

std::string expr_debug(const Expr& e) {  // impl Debug for Expr, logicalplan.rs:263-303
    const dfmi_expr_node* n = e.n;
    switch (n->kind) {
        case DFMI_EXPR_COLUMN: return "#" + std::to_string(n->column);
        case DFMI_EXPR_LITERAL: return scalar_debug(n);
        case DFMI_EXPR_CAST:
            return "CAST(" + expr_debug(*e.kids[0]) + " AS " + type_name(n->data_type) + ")";
        case DFMI_EXPR_IS_NULL: return expr_debug(*e.kids[0]) + " IS NULL";
        case DFMI_EXPR_IS_NOT_NULL: return expr_debug(*e.kids[0]) + " IS NOT NULL";
        case DFMI_EXPR_BINARY:
            return expr_debug(*e.kids[0]) + " " + op_name(n->op) + " " + expr_debug(*e.kids[1]);
        case DFMI_EXPR_SORT: return expr_debug(*e.kids[0]) + (n->op ? " ASC" : " DESC");
        default: {
            std::string s(n->str ? std::string(n->str, n->str_len) : std::string());
            s += "(";
            for (size_t i = 0; i < e.kids.size(); ++i) {
                if (i) s += ", ";
                s += expr_debug(*e.kids[i]);
            }
            return s + ")";
        }
    }
}

// ---------------------------------------------------------------- arrays ---
// Immutable array (arrow::array::Array). Buffers are either borrowed from the
// caller (input batch) or owned.
struct Array {
    int type = 0;
    int64_t len = 0;
    int64_t null_count = 0;
    const uint8_t* validity = nullptr;  // nullptr => all valid
    const uint8_t* values = nullptr;    // fixed width / bool bits / utf8 bytes
    const int32_t* offsets = nullptr;
    std::vector<uint8_t> own_validity, own_values, own_data;
    std::vector<int32_t> own_offsets;
    // arrow ArrayData offset (< 8 after wrap_input's byte shift) of the
    // bitmaps: validity and Boolean values read bit bit_off + i
    int64_t bit_off = 0;

    bool is_null(int64_t i) const {
        const int64_t j = i + bit_off;
        return validity && !((validity[j >> 3] >> (j & 7)) & 1);
    }
    bool bool_value(int64_t i) const {
        const int64_t j = i + bit_off;
        return (values[j >> 3] >> (j & 7)) & 1;
    }
    template <typename T> T value(int64_t i) const {
        T v;
        memcpy(&v, values + i * (int64_t)sizeof(T), sizeof(T));
        return v;
    }
};
using ArrayRef = std::shared_ptr<const Array>;

struct Batch {
    std::vector<ArrayRef> cols;
    int64_t num_rows = 0;
};

// Bit builder (BooleanBufferBuilder): zero-initialised, one bit per append.
struct BitBuilder {
    std::vector<uint8_t> bytes;
    int64_t len = 0;
    void reserve(int64_t n) { bytes.reserve((n + 7) / 8 + 8); }
    void append(bool b) {
        if ((len & 7) == 0) bytes.push_back(0);
        if (b) bytes.back() |= (uint8_t)(1u << (len & 7));
        ++len;
    }
};

// PrimitiveArrayBuilder<T>: push() appends a value and a validity bit,
// push_null() appends a zero value slot and a cleared validity bit.
template <typename T>
struct PrimBuilder {
    std::vector<T> vals;
    BitBuilder valid;
    int64_t nulls = 0;
    explicit PrimBuilder(int64_t cap) { vals.reserve(cap); valid.reserve(cap); }
    void push(T v) { vals.push_back(v); valid.append(true); }
    void push_null() { vals.push_back(T(0)); valid.append(false); ++nulls; }
    ArrayRef finish(int type) {
        auto a = std::make_shared<Array>();
        a->type = type;
        a->len = (int64_t)vals.size();
        a->own_values.resize(vals.size() * sizeof(T) + 8);
        if (!vals.empty()) memcpy(a->own_values.data(), vals.data(), vals.size() * sizeof(T));
        a->values = a->own_values.data();
        a->null_count = nulls;
        if (nulls) {
            a->own_validity = std::move(valid.bytes);
            a->own_validity.resize(a->own_validity.size() + 8, 0);
            a->validity = a->own_validity.data();
        }
        return a;
    }
};

struct BoolBuilder {
    BitBuilder vals, valid;
    int64_t nulls = 0;
    explicit BoolBuilder(int64_t cap) { vals.reserve(cap); valid.reserve(cap); }
    void push(bool b) { vals.append(b); valid.append(true); }
    void push_null() { vals.append(false); valid.append(false); ++nulls; }
    ArrayRef finish() {
        auto a = std::make_shared<Array>();
        a->type = DFMI_TYPE_BOOLEAN;
        a->len = vals.len;
        a->own_values = std::move(vals.bytes);
        a->own_values.resize(a->own_values.size() + 8, 0);
        a->values = a->own_values.data();
        a->null_count = nulls;
        if (nulls) {
            a->own_validity = std::move(valid.bytes);
            a->own_validity.resize(a->own_validity.size() + 8, 0);
            a->validity = a->own_validity.data();
        }
        return a;
    }
};

// --------------------------------------------- type dispatch helpers ---
template <typename F>
void dispatch_numeric(int t, F&& f) {
    switch (t) {
        case DFMI_TYPE_INT8: f((int8_t)0); break;
        case DFMI_TYPE_INT16: f((int16_t)0); break;
        case DFMI_TYPE_INT32: f((int32_t)0); break;
        case DFMI_TYPE_INT64: f((int64_t)0); break;
        case DFMI_TYPE_UINT8: f((uint8_t)0); break;
        case DFMI_TYPE_UINT16: f((uint16_t)0); break;
        case DFMI_TYPE_UINT32: f((uint32_t)0); break;
        case DFMI_TYPE_UINT64: f((uint64_t)0); break;
        case DFMI_TYPE_FLOAT32: f((float)0); break;
        case DFMI_TYPE_FLOAT64: f((double)0); break;
        default: break;
    }
}

// ------------------------------------------------------ array_ops (L0) ---
// arrow 0.12 bool_op: Option<T> per side, the closure sees (l, r), the result
// is always a non-null bool.
template <typename T, typename Op>
ArrayRef bool_op(const Array& l, const Array& r, Op op) {
    if (l.len != r.len)
        fail(DFMI_ERR_ARROW_COMPUTE, "Cannot perform math operation on arrays of different length");
    BoolBuilder b(l.len);
    for (int64_t i = 0; i < l.len; ++i) {
        bool ln = l.is_null(i), rn = r.is_null(i);
        T lv = ln ? T(0) : l.value<T>(i);
        T rv = rn ? T(0) : r.value<T>(i);
        b.push(op(ln, lv, rn, rv));
    }
    return b.finish();
}

template <typename T>
ArrayRef compare(int op, const Array& l, const Array& r) {
    switch (op) {
        case DFMI_OP_EQ:  // Option<T> == Option<T>
            return bool_op<T>(l, r, [](bool ln, T a, bool rn, T b) {
                return (ln || rn) ? (ln && rn) : (a == b); });
        case DFMI_OP_NOT_EQ:
            return bool_op<T>(l, r, [](bool ln, T a, bool rn, T b) {
                return (ln || rn) ? !(ln && rn) : (a != b); });
        case DFMI_OP_LT:  // (None,_) => true, (_,None) => false
            return bool_op<T>(l, r, [](bool ln, T a, bool rn, T b) {
                return ln ? true : (rn ? false : a < b); });
        case DFMI_OP_LT_EQ:
            return bool_op<T>(l, r, [](bool ln, T a, bool rn, T b) {
                return ln ? true : (rn ? false : a <= b); });
        case DFMI_OP_GT:  // (None,_) => false, (_,None) => true
            return bool_op<T>(l, r, [](bool ln, T a, bool rn, T b) {
                return ln ? false : (rn ? true : a > b); });
        default:  // GtEq
            return bool_op<T>(l, r, [](bool ln, T a, bool rn, T b) {
                return ln ? false : (rn ? true : a >= b); });
    }
}

// Utf8 equality (DFMI_FLAG_EXT_UTF8_COMPARE; not executable in the reference).
ArrayRef compare_utf8(int op, const Array& l, const Array& r) {
    if (l.len != r.len)
        fail(DFMI_ERR_ARROW_COMPUTE, "Cannot perform math operation on arrays of different length");
    BoolBuilder b(l.len);
    for (int64_t i = 0; i < l.len; ++i) {
        bool ln = l.is_null(i), rn = r.is_null(i);
        bool eq;
        if (ln || rn) {
            eq = ln && rn;
        } else {
            int32_t la = l.offsets[i + 1] - l.offsets[i], lb = r.offsets[i + 1] - r.offsets[i];
            eq = la == lb && memcmp(l.values + l.offsets[i], r.values + r.offsets[i], la) == 0;
        }
        b.push(op == DFMI_OP_EQ ? eq : !eq);
    }
    return b.finish();
}

template <typename T> T wrap_add(T a, T b) {
    if constexpr (std::is_integral<T>::value) {
        using U = typename std::make_unsigned<T>::type;
        return (T)(U)((U)a + (U)b);
    } else {
        return a + b;
    }
}
template <typename T> T wrap_sub(T a, T b) {
    if constexpr (std::is_integral<T>::value) {
        using U = typename std::make_unsigned<T>::type;
        return (T)(U)((U)a - (U)b);
    } else {
        return a - b;
    }
}
template <typename T> T wrap_mul(T a, T b) {
    if constexpr (std::is_integral<T>::value) {
        using U = typename std::make_unsigned<T>::type;
        // promote to avoid int-promotion UB on narrow types
        return (T)(U)((uint64_t)(U)a * (uint64_t)(U)b);
    } else {
        return a * b;
    }
}

// arrow 0.12 math_op: null if either side is null (value slot 0), else op.
// divide: a non-null zero divisor (0, -0.0) is ArrowError::DivideByZero; the
// Rust `/` on iN::MIN / -1 panics ("attempt to divide with overflow").
// NaN results as the reference's scalar loops produce them on x86-64 (SSE2
// addsd/subsd/mulsd/divsd with the left operand as the destination): a NaN
// operand propagates quieted, the left one first; an invalid operation on
// non-NaN operands (inf - inf, 0 * inf, ...) gives the default NaN, which on
// x86 is negative (0xFFF8000000000000 / 0xFFC00000). Written out so that
// the result does not depend on which operand order the compiler emits.
template <typename T>
T sse_nan(T r, T a, T b) {
    if (!std::isnan(r)) return r;
    if constexpr (sizeof(T) == 8) {
        uint64_t x;
        if (std::isnan(a)) memcpy(&x, &a, 8), x |= 1ull << 51;
        else if (std::isnan(b)) memcpy(&x, &b, 8), x |= 1ull << 51;
        else x = 0xFFF8000000000000ull;
        memcpy(&r, &x, 8);
    } else {
        uint32_t x;
        if (std::isnan(a)) memcpy(&x, &a, 4), x |= 1u << 22;
        else if (std::isnan(b)) memcpy(&x, &b, 4), x |= 1u << 22;
        else x = 0xFFC00000u;
        memcpy(&r, &x, 4);
    }
    return r;
}

template <typename T>
ArrayRef math(int op, int type, const Array& l, const Array& r) {
    if (l.len != r.len)
        fail(DFMI_ERR_ARROW_COMPUTE, "Cannot perform math operation on arrays of different length");
    PrimBuilder<T> b(l.len);
    for (int64_t i = 0; i < l.len; ++i) {
        if (l.is_null(i) || r.is_null(i)) {
            b.push_null();
            continue;
        }
        T x = l.value<T>(i), y = r.value<T>(i);
        T v;
        switch (op) {
            case DFMI_OP_PLUS: v = wrap_add(x, y); break;
            case DFMI_OP_MINUS: v = wrap_sub(x, y); break;
            case DFMI_OP_MULTIPLY: v = wrap_mul(x, y); break;
            default:
                if (y == T(0)) fail(DFMI_ERR_DIVIDE_BY_ZERO, "DivideByZero");
                if constexpr (std::is_integral<T>::value && std::is_signed<T>::value) {
                    if (x == std::numeric_limits<T>::min() && y == T(-1))
                        fail(DFMI_ERR_PANIC, "attempt to divide with overflow");
                }
                v = x / y;
        }
        if constexpr (std::is_floating_point<T>::value) v = sse_nan(v, x, y);
        b.push(v);
    }
    return b.finish(type);
}

ArrayRef bool_and_or(int op, const Array& l, const Array& r) {  // array_ops::{and, or}
    if (l.len != r.len)
        fail(DFMI_ERR_ARROW_COMPUTE, "Cannot perform boolean operation on arrays of different length");
    BoolBuilder b(l.len);
    for (int64_t i = 0; i < l.len; ++i) {
        if (l.is_null(i) || r.is_null(i)) {
            b.push_null();
        } else {
            bool x = l.bool_value(i), y = r.bool_value(i);
            b.push(op == DFMI_OP_AND ? (x && y) : (x || y));
        }
    }
    return b.finish();
}

// ------------------------------------------ cast kernel (extension) ---
// DFMI_FLAG_EXT_CAST: the arrow 0.12 cast kernel for primitive arrays
// (compute::cast -> numeric_cast: a null stays null; each value goes through
// num::cast::<From, To>, and None -- the value does not fit the target type --
// appends a null). num-traits 0.2 NumCast rules restated:
//   int -> int      Some iff the value is in To's range;
//   int -> float    Some(x as To) (round to nearest even);
//   float -> int    Some(trunc(x)) iff x is not NaN and trunc(x) is in range;
//   f32 -> f64      Some (exact); f64 -> f32: None iff x is finite and outside
//                   [f32::MIN, f32::MAX], else Some(x as f32).
// Parity unpinned beyond the values the c_*_cast fixtures hold.
template <typename From, typename To>
bool num_cast(From x, To* out) {
    if constexpr (std::is_integral<From>::value && std::is_integral<To>::value) {
        using L = std::numeric_limits<To>;
        bool ok;
        if constexpr (std::is_signed<From>::value) {
            ok = x >= 0 ? (uint64_t)x <= (uint64_t)L::max() : (std::is_signed<To>::value && (int64_t)x >= (int64_t)L::min());
        } else {
            ok = (uint64_t)x <= (uint64_t)L::max();
        }
        if (ok) *out = (To)x;
        return ok;
    } else if constexpr (std::is_integral<From>::value) {
        *out = (To)x;
        return true;
    } else if constexpr (std::is_integral<To>::value) {
        const double d = (double)x;
        if (std::isnan(d)) return false;
        const double t = std::trunc(d);
        bool ok;
        if constexpr (sizeof(To) == 8) {
            ok = std::is_signed<To>::value ? (t >= -0x1p63 && t < 0x1p63) : (t >= 0.0 && t < 0x1p64);
        } else {
            ok = t >= (double)std::numeric_limits<To>::min() && t <= (double)std::numeric_limits<To>::max();
        }
        if (ok) *out = (To)t;
        return ok;
    } else {
        if (sizeof(From) > sizeof(To) && std::isfinite((double)x) &&
            ((double)x < -(double)std::numeric_limits<float>::max() || (double)x > (double)std::numeric_limits<float>::max()))
            return false;
        *out = (To)x;
        return true;
    }
}

ArrayRef cast_array(const Array& a, int to) {
    ArrayRef out;
    dispatch_numeric(a.type, [&](auto ftag) {
        using F = decltype(ftag);
        dispatch_numeric(to, [&](auto ttag) {
            using T = decltype(ttag);
            PrimBuilder<T> b(a.len);
            for (int64_t i = 0; i < a.len; ++i) {
                T v;
                if (!a.is_null(i) && num_cast<F, T>(a.value<F>(i), &v))
                    b.push(v);
                else
                    b.push_null();
            }
            out = b.finish(to);
        });
    });
    return out;
}

// DFMI_FLAG_EXT_IS_NULL: Array::is_null / is_not_null -> non-null Boolean.
ArrayRef is_null_array(const Array& a, bool want_null) {
    BoolBuilder b(a.len);
    for (int64_t i = 0; i < a.len; ++i) b.push(a.is_null(i) == want_null);
    return b.finish();
}

// -------------------------------------------------- compiled closures ---
using Fn = std::function<ArrayRef(const Batch&)>;
struct Runtime {  // RuntimeExpr::Compiled {name, f, t}
    std::string name;
    Fn f;
    int t;
};

template <typename T>
ArrayRef literal_fill(const Batch& b, T v, int type) {  // literal_array! per batch
    PrimBuilder<T> builder(b.num_rows);
    for (int64_t i = 0; i < b.num_rows; ++i) builder.push(v);
    return builder.finish(type);
}

ArrayRef utf8_literal_fill(const Batch& b, const std::string& s) {
    auto a = std::make_shared<Array>();
    a->type = DFMI_TYPE_UTF8;
    a->len = b.num_rows;
    a->own_offsets.reserve(b.num_rows + 1);
    a->own_offsets.push_back(0);
    for (int64_t i = 0; i < b.num_rows; ++i) {
        a->own_data.insert(a->own_data.end(), s.begin(), s.end());
        a->own_offsets.push_back((int32_t)a->own_data.size());
    }
    a->own_data.resize(a->own_data.size() + 8);
    a->values = a->own_data.data();
    a->offsets = a->own_offsets.data();
    return a;
}

Runtime compile(const Expr& e, const dfmi_schema& s, uint32_t flags);

Runtime compile_literal(const dfmi_expr_node* n, uint32_t flags) {
    Runtime r;
    r.t = n->data_type;
    switch (n->data_type) {
        case DFMI_TYPE_FLOAT64: case DFMI_TYPE_FLOAT32:
            r.name = rust_float(n->f64, n->data_type == DFMI_TYPE_FLOAT32, false);
            break;
        case DFMI_TYPE_UINT8: case DFMI_TYPE_UINT16: case DFMI_TYPE_UINT32: case DFMI_TYPE_UINT64:
            r.name = std::to_string((unsigned long long)n->i64);
            break;
        case DFMI_TYPE_UTF8:
            if (flags & DFMI_FLAG_EXT_UTF8_COMPARE) {
                std::string v(n->str, n->str_len);
                r.name = v;
                r.f = [v](const Batch& b) { return utf8_literal_fill(b, v); };
                return r;
            }
            // fallthrough
        case DFMI_TYPE_NULL: case DFMI_TYPE_BOOLEAN:
            fail(DFMI_ERR_EXECUTION, "No support for literal type " + scalar_debug(n));
        default:
            r.name = std::to_string((long long)n->i64);
    }
    const int t = n->data_type;
    const int64_t iv = n->i64;
    const double fv = n->f64;
    switch (t) {
        case DFMI_TYPE_INT8: r.f = [=](const Batch& b) { return literal_fill<int8_t>(b, (int8_t)iv, t); }; break;
        case DFMI_TYPE_INT16: r.f = [=](const Batch& b) { return literal_fill<int16_t>(b, (int16_t)iv, t); }; break;
        case DFMI_TYPE_INT32: r.f = [=](const Batch& b) { return literal_fill<int32_t>(b, (int32_t)iv, t); }; break;
        case DFMI_TYPE_INT64: r.f = [=](const Batch& b) { return literal_fill<int64_t>(b, iv, t); }; break;
        case DFMI_TYPE_UINT8: r.f = [=](const Batch& b) { return literal_fill<uint8_t>(b, (uint8_t)iv, t); }; break;
        case DFMI_TYPE_UINT16: r.f = [=](const Batch& b) { return literal_fill<uint16_t>(b, (uint16_t)iv, t); }; break;
        case DFMI_TYPE_UINT32: r.f = [=](const Batch& b) { return literal_fill<uint32_t>(b, (uint32_t)iv, t); }; break;
        case DFMI_TYPE_UINT64: r.f = [=](const Batch& b) { return literal_fill<uint64_t>(b, (uint64_t)iv, t); }; break;
        case DFMI_TYPE_FLOAT32: r.f = [=](const Batch& b) { return literal_fill<float>(b, (float)fv, t); }; break;
        default: r.f = [=](const Batch& b) { return literal_fill<double>(b, fv, t); }; break;
    }
    return r;
}

Runtime compile(const Expr& e, const dfmi_schema& s, uint32_t flags) {
    const dfmi_expr_node* n = e.n;
    switch (n->kind) {
        case DFMI_EXPR_LITERAL:
            return compile_literal(n, flags);
        case DFMI_EXPR_COLUMN: {
            const int idx = n->column;
            if (idx < 0 || idx >= s.num_fields)  // schema.field(i) out of bounds
                fail(DFMI_ERR_PANIC, "index out of bounds: the len is " + std::to_string(s.num_fields) +
                                         " but the index is " + std::to_string(idx));
            Runtime r;
            r.name = s.fields[idx].name;
            r.t = s.fields[idx].type;
            r.f = [idx](const Batch& b) -> ArrayRef {
                if (idx >= (int)b.cols.size()) fail(DFMI_ERR_PANIC, "index out of bounds");
                return b.cols[idx];  // Arc clone
            };
            return r;
        }
        case DFMI_EXPR_CAST: {
            const Expr& inner = *e.kids[0];
            if ((flags & DFMI_FLAG_EXT_CAST) && inner.n->kind != DFMI_EXPR_LITERAL) {
                Runtime c = compile(inner, s, flags);
                const int to = n->data_type;
                if (!is_numeric(c.t) || !is_numeric(to))
                    fail(DFMI_ERR_NOT_IMPLEMENTED,
                         std::string("CAST from ") + type_name(c.t) + " to " + type_name(to));
                Runtime r;
                r.name = expr_debug(e);
                r.t = to;
                Fn cf = c.f;
                if (c.t == to)  // cast(): the same type returns the array itself
                    r.f = cf;
                else
                    r.f = [cf, to](const Batch& b) { return cast_array(*cf(b), to); };
                return r;
            }
            if (inner.n->kind == DFMI_EXPR_COLUMN) fail(DFMI_ERR_EXECUTION, "column reference");
            if (inner.n->kind == DFMI_EXPR_LITERAL) {
                if (inner.n->data_type == DFMI_TYPE_INT64) {
                    if (n->data_type != DFMI_TYPE_FLOAT64)
                        fail(DFMI_ERR_NOT_IMPLEMENTED,
                             std::string("CAST from Int64 to ") + type_name(n->data_type));
                    const double v = (double)inner.n->i64;  // `nn as f64`
                    Runtime r;
                    r.name = "lit";
                    r.t = DFMI_TYPE_FLOAT64;
                    r.f = [v](const Batch& b) { return literal_fill<double>(b, v, DFMI_TYPE_FLOAT64); };
                    return r;
                }
                fail(DFMI_ERR_NOT_IMPLEMENTED, "CAST from " + scalar_debug(inner.n) + " to " +
                                                   type_name(n->data_type));
            }
            fail(DFMI_ERR_GENERAL, "CAST not implemented for expression " + expr_debug(inner));
        }
        case DFMI_EXPR_BINARY: {
            Runtime L = compile(*e.kids[0], s, flags);
            Runtime R = compile(*e.kids[1], s, flags);
            Runtime r;
            r.name = expr_debug(*e.kids[0]) + " " + op_name(n->op) + " " + expr_debug(*e.kids[1]);
            const int op = n->op;
            Fn lf = L.f, rf = R.f;
            if (op >= DFMI_OP_EQ && op <= DFMI_OP_GT_EQ) {
                r.t = DFMI_TYPE_BOOLEAN;
                r.f = [=](const Batch& b) -> ArrayRef {
                    ArrayRef lv = lf(b);
                    ArrayRef rv = rf(b);
                    if (lv->type == rv->type && is_numeric(lv->type)) {
                        ArrayRef out;
                        dispatch_numeric(lv->type, [&](auto tag) {
                            out = compare<decltype(tag)>(op, *lv, *rv);
                        });
                        return out;
                    }
                    if ((flags & DFMI_FLAG_EXT_UTF8_COMPARE) && lv->type == DFMI_TYPE_UTF8 &&
                        rv->type == DFMI_TYPE_UTF8 && (op == DFMI_OP_EQ || op == DFMI_OP_NOT_EQ))
                        return compare_utf8(op, *lv, *rv);
                    fail(DFMI_ERR_EXECUTION, "comparison_ops");
                };
                return r;
            }
            if (op == DFMI_OP_AND || op == DFMI_OP_OR) {
                r.t = DFMI_TYPE_BOOLEAN;
                r.f = [=](const Batch& b) -> ArrayRef {
                    ArrayRef lv = lf(b);
                    ArrayRef rv = rf(b);
                    if (lv->type != DFMI_TYPE_BOOLEAN || rv->type != DFMI_TYPE_BOOLEAN)
                        fail(DFMI_ERR_PANIC, "called `Option::unwrap()` on a `None` value");
                    return bool_and_or(op, *lv, *rv);
                };
                return r;
            }
            if (op >= DFMI_OP_PLUS && op <= DFMI_OP_DIVIDE) {
                r.t = L.t;  // op_type = left_expr.get_type()
                r.f = [=](const Batch& b) -> ArrayRef {
                    ArrayRef lv = lf(b);
                    ArrayRef rv = rf(b);
                    if (lv->type == rv->type && is_numeric(lv->type)) {
                        ArrayRef out;
                        dispatch_numeric(lv->type, [&](auto tag) {
                            out = math<decltype(tag)>(op, lv->type, *lv, *rv);
                        });
                        return out;
                    }
                    fail(DFMI_ERR_EXECUTION, "math_ops");
                };
                return r;
            }
            fail(DFMI_ERR_EXECUTION, std::string("operator: ") + op_name(op));
        }
        case DFMI_EXPR_IS_NULL: case DFMI_EXPR_IS_NOT_NULL:
            if (flags & DFMI_FLAG_EXT_IS_NULL) {
                Runtime c = compile(*e.kids[0], s, flags);
                Runtime r;
                r.name = expr_debug(e);
                r.t = DFMI_TYPE_BOOLEAN;
                Fn cf = c.f;
                const bool want_null = n->kind == DFMI_EXPR_IS_NULL;
                r.f = [cf, want_null](const Batch& b) { return is_null_array(*cf(b), want_null); };
                return r;
            }
            fail(DFMI_ERR_EXECUTION, "expression " + expr_debug(e));
        default:
            fail(DFMI_ERR_EXECUTION, "expression " + expr_debug(e));
    }
}

// ------------------------------------------------- FilterRelation::next ---
ArrayRef filter_column(const Array& a, const Array& mask, uint32_t flags) {
    const int t = a.type;
    if (t == DFMI_TYPE_FLOAT64 || ((flags & DFMI_FLAG_EXT_GATHER_ALL) && is_numeric(t))) {
        ArrayRef out;
        dispatch_numeric(t, [&](auto tag) {
            using T = decltype(tag);
            PrimBuilder<T> b(a.len);
            for (int64_t i = 0; i < a.len; ++i)
                if (mask.bool_value(i)) b.push(a.value<T>(i));  // raw slot bits, no validity
            out = b.finish(t);
        });
        return out;
    }
    if (t == DFMI_TYPE_UTF8) {
        // get_string per selected row, then BinaryArray::from(Vec<&str>)
        std::vector<std::string> vals;
        vals.reserve(a.len);
        for (int64_t i = 0; i < a.len; ++i)
            if (mask.bool_value(i))
                vals.emplace_back((const char*)a.values + a.offsets[i], a.offsets[i + 1] - a.offsets[i]);
        auto o = std::make_shared<Array>();
        o->type = DFMI_TYPE_UTF8;
        o->len = (int64_t)vals.size();
        o->own_offsets.reserve(vals.size() + 1);
        o->own_offsets.push_back(0);
        for (auto& v : vals) {
            o->own_data.insert(o->own_data.end(), v.begin(), v.end());
            o->own_offsets.push_back((int32_t)o->own_data.size());
        }
        o->own_data.resize(o->own_data.size() + 8);
        o->values = o->own_data.data();
        o->offsets = o->own_offsets.data();
        return o;
    }
    if (t == DFMI_TYPE_BOOLEAN && (flags & DFMI_FLAG_EXT_GATHER_ALL)) {
        BoolBuilder b(a.len);
        for (int64_t i = 0; i < a.len; ++i)
            if (mask.bool_value(i)) b.push(a.bool_value(i));
        return b.finish();
    }
    fail(DFMI_ERR_EXECUTION, std::string("filter not supported for ") + type_name(t));
}

struct Plan {
    bool has_pred = false;
    Runtime pred;
    std::vector<Runtime> projs;
    bool has_proj = false;
};

// One pull: ProjectRelation::next(FilterRelation::next(batch)).
Batch run_batch(const Plan& p, const Batch& in, uint32_t flags) {
    Batch cur = in;
    if (p.has_pred) {
        ArrayRef m = p.pred.f(in);
        if (m->type != DFMI_TYPE_BOOLEAN)
            fail(DFMI_ERR_EXECUTION, "Filter expression did not evaluate to boolean");
        Batch fb;
        for (auto& c : in.cols) fb.cols.push_back(filter_column(*c, *m, flags));
        fb.num_rows = fb.cols.empty() ? 0 : fb.cols[0]->len;
        cur = fb;
    }
    if (!p.has_proj) return cur;
    Batch out;
    for (auto& r : p.projs) out.cols.push_back(r.f(cur));
    out.num_rows = out.cols.empty() ? 0 : out.cols[0]->len;
    return out;
}

Batch wrap_input(const dfmi_batch* in, int64_t row0, int64_t rows) {
    Batch b;
    b.num_rows = rows;
    for (int i = 0; i < in->num_columns; ++i) {
        const dfmi_column& c = in->columns[i];
        auto a = std::make_shared<Array>();
        a->type = c.type;
        a->len = rows;
        // logical row i of the column is physical slot offset + i (arrow
        // ArrayData::offset, which value(i) / is_null(i) honour)
        if (c.offset < 0) fail(DFMI_ERR_INVALID_ARGUMENT, "negative array offset");
        const int64_t r0 = row0 + c.offset;
        const int w = type_width(c.type);
        a->values = (const uint8_t*)c.values;
        a->bit_off = r0 & 7;
        if (c.type == DFMI_TYPE_UTF8) {
            a->offsets = c.offsets + r0;
        } else if (c.type == DFMI_TYPE_BOOLEAN) {
            a->values += r0 / 8;
        } else {
            a->values += r0 * w;
        }
        if (c.validity) {
            a->validity = c.validity + r0 / 8;
            int64_t nc = 0;
            for (int64_t r = 0; r < rows; ++r) nc += a->is_null(r);
            a->null_count = nc;
            if (!nc) a->validity = nullptr;
        }
        b.cols.push_back(a);
    }
    return b;
}

Plan make_plan(const dfmi_expr_node* pred_nodes, int32_t pred_len,
               const dfmi_expr_node* const* proj_nodes, const int32_t* proj_lens, int32_t np,
               const dfmi_schema* schema, uint32_t flags) {
    // context.rs:125-160: the Selection is compiled before the projection list.
    Plan p;
    if (pred_nodes) {
        ExprP t = build_tree(pred_nodes, pred_len);
        p.pred = compile(*t, *schema, flags);
        p.has_pred = true;
    }
    if (np > 0) {
        p.has_proj = true;
        for (int i = 0; i < np; ++i) {
            ExprP t = build_tree(proj_nodes[i], proj_lens[i]);
            p.projs.push_back(compile(*t, *schema, flags));
        }
    }
    return p;
}

// ------------------------------------------------ Aggregate extension ---
// LogicalPlan::Aggregate with no GROUP BY (sqlplanner.rs:91-117; compile_expr
// expression.rs:81-116; the reference's executor stops at context.rs:161).
// The input is pulled through FilterRelation::next batch by batch and each
// argument is evaluated over the filtered batch, the reference's way; the
// aggregation semantics are the build's (include/dfmi.h).

// Exact sum of binary64 values: a 2176-bit two's complement integer in units
// of 2^-1074 (every double is m * 2^(b-1074), m < 2^53, 0 <= b <= 2045).
struct ExactSum {
    static constexpr int W = 34;
    uint64_t w[W] = {};
    void add_shifted(uint64_t m, int b, bool neg) {
        const int q = b / 64, r = b % 64;
        uint64_t part[2] = {m << r, r ? (m >> (64 - r)) : 0};
        if (!neg) {
            unsigned __int128 c = 0;
            for (int i = q; i < W; ++i) {
                const uint64_t a = i - q < 2 ? part[i - q] : 0;
                c += (unsigned __int128)w[i] + a;
                w[i] = (uint64_t)c;
                c >>= 64;
                if (i - q >= 1 && c == 0) break;
            }
        } else {
            uint64_t borrow = 0;
            for (int i = q; i < W; ++i) {
                const uint64_t a = i - q < 2 ? part[i - q] : 0;
                const uint64_t x = w[i];
                const uint64_t d = x - a - borrow;
                borrow = (x < a) || (x - a < borrow) ? 1 : 0;
                w[i] = d;
                if (i - q >= 1 && borrow == 0) break;
            }
        }
    }
    void add(double v) {
        uint64_t bits;
        memcpy(&bits, &v, 8);
        const int e = (int)((bits >> 52) & 0x7ff);
        uint64_t m = bits & ((1ull << 52) - 1);
        if (e) m |= 1ull << 52;
        if (!m) return;
        add_shifted(m, (e ? e : 1) - 1, bits >> 63);
    }
    // Round to a binary format with `prec` significand bits whose smallest
    // quantum is 2^(qmin-1074); returns the value as a double (exact for
    // Float32 results, which the caller narrows).
    double round(int prec, int qmin, double overflow_limit, bool* zero) const {
        uint64_t m[W];
        const bool neg = w[W - 1] >> 63;
        if (neg) {  // magnitude = two's complement negation
            uint64_t c = 1;
            for (int i = 0; i < W; ++i) {
                m[i] = ~w[i] + c;
                c = (c && m[i] == 0) ? 1 : 0;
            }
        } else {
            memcpy(m, w, sizeof m);
        }
        int p = -1;
        for (int i = W - 1; i >= 0; --i)
            if (m[i]) {
                p = 64 * i + 63 - __builtin_clzll(m[i]);
                break;
            }
        *zero = p < 0;
        if (p < 0) return 0.0;
        auto bit = [&](int i) -> uint64_t { return i < 0 ? 0 : (m[i / 64] >> (i % 64)) & 1; };
        int q = std::max(p - (prec - 1), qmin);
        uint64_t mant = 0;
        for (int i = p; i >= q; --i) mant = (mant << 1) | bit(i);
        const uint64_t rb = q >= 1 ? bit(q - 1) : 0;
        bool sticky = false;
        for (int i = q - 2; i >= 0 && !sticky; --i) sticky = bit(i);
        if (rb && (sticky || (mant & 1))) {
            ++mant;
            if (mant >> prec) {
                mant >>= 1;
                ++q;
            }
        }
        double d = std::ldexp((double)mant, q - 1074);
        if (d >= overflow_limit) d = std::numeric_limits<double>::infinity();
        return neg ? -d : d;
    }
};

// Total order of non-NaN values: -0.0 below +0.0.
template <typename T>
bool agg_less(T a, T b) {
    if constexpr (std::is_floating_point<T>::value) {
        if (a == b) return std::signbit(a) && !std::signbit(b);
    }
    return a < b;
}

struct AggState {
    int fn = 0, arg_type = 0, ret_type = 0;
    int64_t count = 0;
    uint64_t isum = 0;            // wrapping integer sum
    bool has_key = false;         // MIN/MAX: a non-NaN value seen
    uint64_t key_bits = 0;        // ... its bits
    bool nan = false, pinf = false, ninf = false, non_negzero = false;
    ExactSum exact;
};

template <typename T>
uint64_t to_bits64(T v) {
    if constexpr (std::is_same<T, float>::value) {
        uint32_t b;
        memcpy(&b, &v, 4);
        return b;
    } else if constexpr (std::is_same<T, double>::value) {
        uint64_t b;
        memcpy(&b, &v, 8);
        return b;
    } else if constexpr (std::is_signed<T>::value) {
        return (uint64_t)(int64_t)v;
    } else {
        return (uint64_t)v;
    }
}

template <typename T>
T from_bits64(uint64_t b) {
    T v;
    if constexpr (std::is_same<T, float>::value) {
        uint32_t x = (uint32_t)b;
        memcpy(&v, &x, 4);
    } else if constexpr (std::is_same<T, double>::value) {
        memcpy(&v, &b, 8);
    } else {
        v = (T)b;
    }
    return v;
}

void agg_accumulate_row(AggState& st, const Array& a, int64_t i);

void agg_accumulate(AggState& st, const Array& a) {
    for (int64_t i = 0; i < a.len; ++i) agg_accumulate_row(st, a, i);
}

void agg_accumulate_row(AggState& st, const Array& a, int64_t i) {
    {
        if (a.is_null(i)) return;
        ++st.count;
        if (st.fn == DFMI_AGG_COUNT) return;
        dispatch_numeric(a.type, [&](auto tag) {
            using T = decltype(tag);
            const T v = a.value<T>(i);
            if constexpr (std::is_floating_point<T>::value) {
                if (std::isnan(v)) {
                    st.nan = true;
                    return;
                }
                if (st.fn == DFMI_AGG_SUM) {
                    if (std::isinf(v)) {
                        (v > 0 ? st.pinf : st.ninf) = true;
                        return;
                    }
                    if (!(v == 0 && std::signbit(v))) st.non_negzero = true;
                    st.exact.add((double)v);
                    return;
                }
            } else {
                if (st.fn == DFMI_AGG_SUM) {
                    st.isum += (uint64_t)v;  // wraps in u64, narrowed at the end
                    return;
                }
            }
            const T cur = from_bits64<T>(st.key_bits);
            const bool take = !st.has_key || (st.fn == DFMI_AGG_MIN ? agg_less(v, cur) : agg_less(cur, v));
            if (take) st.key_bits = to_bits64(v);
            st.has_key = true;
        });
    }
}

// GROUP BY key of row i of the key array: (null, order value, bits). Groups
// are ordered by key value -- false < true, integers numerically -- with the
// null group last (the order of expected/csv_aggregate_by_c_bool.csv).
// Floating-point keys (build-defined, parity unpinned: the reference
// executes no Aggregate): one group per bit pattern, ordered by IEEE 754
// totalOrder (Rust's f64::total_cmp: -NaN < -inf < ... < -0.0 < +0.0 < ... <
// +inf < +NaN). Utf8 keys: bytewise order, a shorter prefix first.
struct GroupKey {
    bool null;
    __int128 ord;
    std::string s;
    bool operator<(const GroupKey& o) const {
        if (null != o.null) return !null;
        if (null) return false;
        return ord != o.ord ? ord < o.ord : s < o.s;
    }
};
GroupKey group_key(const Array& a, int64_t i, uint64_t* bits) {
    *bits = 0;
    if (a.is_null(i)) return {true, 0, {}};
    if (a.type == DFMI_TYPE_BOOLEAN) {
        *bits = a.bool_value(i) ? 1 : 0;
        return {false, (__int128)*bits, {}};
    }
    if (a.type == DFMI_TYPE_UTF8)
        return {false, 0, std::string((const char*)a.values + a.offsets[i], (size_t)(a.offsets[i + 1] - a.offsets[i]))};
    __int128 ord = 0;
    dispatch_numeric(a.type, [&](auto tag) {
        using T = decltype(tag);
        const T v = a.value<T>(i);
        *bits = to_bits64(v);
        if constexpr (std::is_integral<T>::value) {
            ord = (__int128)v;
        } else if constexpr (sizeof(T) == 8) {
            const uint64_t b = *bits;
            ord = (__int128)((b >> 63) ? ~b : (b | (1ull << 63)));
        } else {
            const uint32_t b = (uint32_t)*bits;
            ord = (__int128)((b >> 31) ? (uint32_t)~b : (b | 0x80000000u));
        }
    });
    return {false, ord, {}};
}

dfmi_agg_value agg_result(const AggState& st) {
    dfmi_agg_value r;
    r.type = st.ret_type;
    r.count = st.count;
    r.is_null = 0;
    r.bits = 0;
    if (st.fn == DFMI_AGG_COUNT) {
        r.bits = (uint64_t)st.count;
        return r;
    }
    if (st.count == 0) {
        r.is_null = 1;
        return r;
    }
    const bool f32 = st.arg_type == DFMI_TYPE_FLOAT32, f64 = st.arg_type == DFMI_TYPE_FLOAT64;
    const uint64_t qnan = f32 ? 0x7FC00000ull : 0x7FF8000000000000ull;
    if (st.fn == DFMI_AGG_SUM) {
        if (f32 || f64) {
            if (st.nan || (st.pinf && st.ninf)) {
                r.bits = qnan;
            } else if (st.pinf || st.ninf) {
                r.bits = f32 ? to_bits64(st.pinf ? INFINITY : -INFINITY)
                             : to_bits64(st.pinf ? (double)INFINITY : -(double)INFINITY);
            } else {
                bool zero = false;
                double d = f32 ? st.exact.round(24, 925, 0x1p128, &zero) : st.exact.round(53, 0, INFINITY, &zero);
                if (zero) d = st.non_negzero ? 0.0 : -0.0;
                r.bits = f32 ? to_bits64((float)d) : to_bits64(d);
            }
        } else {
            dispatch_numeric(st.arg_type, [&](auto tag) {
                using T = decltype(tag);
                r.bits = to_bits64((T)st.isum);  // wrapping: the low bits of the sum
            });
        }
        return r;
    }
    r.bits = st.has_key ? st.key_bits : qnan;  // only NaNs seen: the canonical NaN
    return r;
}

int agg_fn_of(const std::string& name) {
    std::string l = name;
    for (auto& c : l) c = (char)tolower((unsigned char)c);
    if (l == "min") return DFMI_AGG_MIN;
    if (l == "max") return DFMI_AGG_MAX;
    if (l == "count") return DFMI_AGG_COUNT;
    if (l == "sum") return DFMI_AGG_SUM;
    fail(DFMI_ERR_PANIC, "not yet implemented: Unsupported aggregate function '" + name + "'");
}

void set_err(dfmi_error* err, int32_t code, const std::string& m) {
    if (!err) return;
    err->code = code;
    snprintf(err->message, sizeof err->message, "%s", m.c_str());
}

}  // namespace

struct oracle_result {
    Batch b;
    std::vector<std::string> names;
};

extern "C" {

int32_t oracle_filter_project(const dfmi_expr_node* pred_nodes, int32_t pred_len,
                              const dfmi_expr_node* const* proj_nodes, const int32_t* proj_lens,
                              int32_t np, const dfmi_schema* schema, const dfmi_batch* input,
                              uint32_t flags, oracle_result** out, dfmi_error* err) {
    try {
        set_err(err, DFMI_OK, "");
        Plan p = make_plan(pred_nodes, pred_len, proj_nodes, proj_lens, np, schema, flags);
        Batch in = wrap_input(input, 0, input->num_rows);
        auto* r = new oracle_result();
        r->b = run_batch(p, in, flags);
        if (p.has_proj) {
            for (auto& pr : p.projs) r->names.push_back(pr.name);
        } else {
            for (int i = 0; i < schema->num_fields; ++i) r->names.push_back(schema->fields[i].name);
        }
        *out = r;
        return DFMI_OK;
    } catch (const ExecError& e) {
        set_err(err, e.code, e.msg);
        return e.code;
    } catch (const std::bad_alloc&) {
        set_err(err, DFMI_ERR_INVALID_ARGUMENT, "out of memory");
        return DFMI_ERR_INVALID_ARGUMENT;
    }
}

int32_t oracle_run_batched(const dfmi_expr_node* pred_nodes, int32_t pred_len,
                           const dfmi_expr_node* const* proj_nodes, const int32_t* proj_lens,
                           int32_t np, const dfmi_schema* schema, const dfmi_batch* input,
                           int64_t batch_rows, uint32_t flags, int64_t* out_rows, dfmi_error* err) {
    try {
        set_err(err, DFMI_OK, "");
        Plan p = make_plan(pred_nodes, pred_len, proj_nodes, proj_lens, np, schema, flags);
        int64_t total = 0;
        for (int64_t r0 = 0; r0 < input->num_rows; r0 += batch_rows) {
            int64_t rows = std::min(batch_rows, input->num_rows - r0);
            Batch in = wrap_input(input, r0, rows);
            Batch o = run_batch(p, in, flags);
            total += o.num_rows;
        }
        *out_rows = total;
        return DFMI_OK;
    } catch (const ExecError& e) {
        set_err(err, e.code, e.msg);
        return e.code;
    }
}

int32_t oracle_result_num_columns(const oracle_result* r) { return (int32_t)r->b.cols.size(); }

int32_t oracle_result_column(const oracle_result* r, int32_t i, dfmi_column* v, const char** name) {
    if (i < 0 || i >= (int32_t)r->b.cols.size()) return DFMI_ERR_INVALID_ARGUMENT;
    const Array& a = *r->b.cols[i];
    v->type = a.type;
    v->reserved = 0;
    v->length = a.len;
    v->null_count = a.null_count;
    v->validity = a.null_count ? a.validity : nullptr;
    v->values = a.values;
    v->offsets = a.offsets;
    v->offset = a.bit_off;  // (a passed-through input column keeps its bit offset)
    if (name) *name = r->names[i].c_str();
    return DFMI_OK;
}

void oracle_result_free(oracle_result* r) { delete r; }

int32_t oracle_compile_info(const dfmi_expr_node* nodes, int32_t n, const dfmi_schema* schema,
                            uint32_t flags, char* name, int64_t cap, int32_t* type, dfmi_error* err) {
    try {
        set_err(err, DFMI_OK, "");
        ExprP t = build_tree(nodes, n);
        Runtime r = compile(*t, *schema, flags);
        if (name && cap > 0) snprintf(name, (size_t)cap, "%s", r.name.c_str());
        if (type) *type = r.t;
        return DFMI_OK;
    } catch (const ExecError& e) {
        set_err(err, e.code, e.msg);
        return e.code;
    }
}

int32_t oracle_aggregate(const dfmi_expr_node* pred_nodes, int32_t pred_len, const char* const* names,
                         const dfmi_expr_node* const* arg_nodes, const int32_t* arg_lens,
                         const int32_t* return_types, int32_t n, const dfmi_schema* schema,
                         const dfmi_batch* input, int64_t batch_rows, uint32_t flags, dfmi_agg_value* out,
                         dfmi_error* err) {
    try {
        set_err(err, DFMI_OK, "");
        if (!(flags & DFMI_FLAG_EXT_AGGREGATE)) fail(DFMI_ERR_PANIC, "not yet implemented");  // context.rs:161
        // context.rs order: the input (Selection) first, then compile_expr per aggregate
        Plan p = make_plan(pred_nodes, pred_len, nullptr, nullptr, 0, schema, flags);
        std::vector<Runtime> args;
        std::vector<AggState> st(n);
        for (int j = 0; j < n; ++j) {
            const int fn = agg_fn_of(names[j]);
            ExprP t = build_tree(arg_nodes[j], arg_lens[j]);
            args.push_back(compile(*t, *schema, flags));
            st[j].fn = fn;
            st[j].arg_type = args[j].t;
            st[j].ret_type = return_types[j];
            const int want = fn == DFMI_AGG_COUNT ? DFMI_TYPE_UINT64 : args[j].t;
            if (return_types[j] != want) fail(DFMI_ERR_INVALID_ARGUMENT, "aggregate return type");
            if (fn != DFMI_AGG_COUNT && !is_numeric(args[j].t))
                fail(DFMI_ERR_NOT_IMPLEMENTED, std::string("aggregate over ") + type_name(args[j].t));
        }
        if (batch_rows <= 0) batch_rows = std::max<int64_t>(1, input->num_rows);
        for (int64_t r0 = 0; r0 < input->num_rows; r0 += batch_rows) {
            const int64_t rows = std::min(batch_rows, input->num_rows - r0);
            Batch in = wrap_input(input, r0, rows);
            Batch f = run_batch(p, in, flags);  // FilterRelation::next (or the batch itself)
            for (int j = 0; j < n; ++j) agg_accumulate(st[j], *args[j].f(f));
        }
        for (int j = 0; j < n; ++j) out[j] = agg_result(st[j]);
        return DFMI_OK;
    } catch (const ExecError& e) {
        set_err(err, e.code, e.msg);
        return e.code;
    }
}

// GROUP BY extension: LogicalPlan::Aggregate{group_expr, aggr_expr} (the
// planner's form, sqlplanner.rs:91-117; group_expr a Vec<Expr>, 1 to 4 keys
// here) -- per group the aggregates of the no-GROUP-BY form. Groups are
// ordered lexicographically over the key parts, each part by GroupKey (its
// null last). keys[g * nkeys + p] / out[g * n + j] in group order; the Utf8
// bytes of key part `key_part` (if key_offsets) as a BinaryArray;
// *num_groups is set even when cap is too small. Build-defined (the
// reference executes no Aggregate): parity unpinned beyond the one-key
// fixture expected/csv_aggregate_by_c_bool.csv.
int32_t oracle_aggregate_grouped_multi(const dfmi_expr_node* pred_nodes, int32_t pred_len,
                                       const dfmi_expr_node* const* key_nodes, const int32_t* key_lens, int32_t nkeys,
                                       const char* const* names, const dfmi_expr_node* const* arg_nodes,
                                       const int32_t* arg_lens, const int32_t* return_types, int32_t n,
                                       const dfmi_schema* schema, const dfmi_batch* input, int64_t batch_rows,
                                       uint32_t flags, int64_t cap, dfmi_agg_value* keys, dfmi_agg_value* out,
                                       int64_t* num_groups, int32_t key_part, int32_t* key_offsets, uint8_t* key_data,
                                       int64_t key_data_cap, dfmi_error* err) {
    try {
        set_err(err, DFMI_OK, "");
        if (!(flags & DFMI_FLAG_EXT_AGGREGATE)) fail(DFMI_ERR_PANIC, "not yet implemented");  // context.rs:161
        if (nkeys < 1 || nkeys > 4) fail(DFMI_ERR_NOT_IMPLEMENTED, "device program limit: more than 4 GROUP BY expressions");
        Plan p = make_plan(pred_nodes, pred_len, nullptr, nullptr, 0, schema, flags);
        std::vector<Runtime> key;
        for (int k = 0; k < nkeys; ++k) {
            ExprP kt = build_tree(key_nodes[k], key_lens[k]);
            key.push_back(compile(*kt, *schema, flags));
            const int t = key.back().t;
            if (t != DFMI_TYPE_BOOLEAN && !is_numeric(t) && t != DFMI_TYPE_UTF8)
                fail(DFMI_ERR_NOT_IMPLEMENTED, std::string("GROUP BY over ") + type_name(t));
        }
        std::vector<Runtime> args;
        std::vector<AggState> proto(n);
        for (int j = 0; j < n; ++j) {
            const int fn = agg_fn_of(names[j]);
            ExprP t = build_tree(arg_nodes[j], arg_lens[j]);
            args.push_back(compile(*t, *schema, flags));
            proto[j].fn = fn;
            proto[j].arg_type = args[j].t;
            proto[j].ret_type = return_types[j];
            const int want = fn == DFMI_AGG_COUNT ? DFMI_TYPE_UINT64 : args[j].t;
            if (return_types[j] != want) fail(DFMI_ERR_INVALID_ARGUMENT, "aggregate return type");
            if (fn != DFMI_AGG_COUNT && !is_numeric(args[j].t))
                fail(DFMI_ERR_NOT_IMPLEMENTED, std::string("aggregate over ") + type_name(args[j].t));
        }
        struct KeyN {
            std::vector<GroupKey> k;
            bool operator<(const KeyN& o) const {
                for (size_t i = 0; i < k.size(); ++i) {
                    if (k[i] < o.k[i]) return true;
                    if (o.k[i] < k[i]) return false;
                }
                return false;
            }
        };
        struct Group {
            std::vector<uint64_t> bits;
            std::vector<AggState> st;
            int64_t rows = 0;  // selected rows (keys[g].count)
        };
        std::map<KeyN, Group> groups;
        if (batch_rows <= 0) batch_rows = std::max<int64_t>(1, input->num_rows);
        for (int64_t r0 = 0; r0 < input->num_rows; r0 += batch_rows) {
            const int64_t rows = std::min(batch_rows, input->num_rows - r0);
            Batch in = wrap_input(input, r0, rows);
            Batch f = run_batch(p, in, flags);  // FilterRelation::next (or the batch itself)
            std::vector<ArrayRef> ka;           // the keys first, in order, then the aggregates
            for (int k = 0; k < nkeys; ++k) ka.push_back(key[k].f(f));
            std::vector<ArrayRef> av;
            for (int j = 0; j < n; ++j) av.push_back(args[j].f(f));
            for (int64_t i = 0; i < f.num_rows; ++i) {
                KeyN gk;
                std::vector<uint64_t> bits(nkeys);
                for (int k = 0; k < nkeys; ++k) gk.k.push_back(group_key(*ka[k], i, &bits[k]));
                auto it = groups.find(gk);
                if (it == groups.end()) it = groups.emplace(gk, Group{bits, proto, 0}).first;
                for (int j = 0; j < n; ++j) agg_accumulate_row(it->second.st[j], *av[j], i);
                ++it->second.rows;
            }
        }
        *num_groups = (int64_t)groups.size();
        if ((int64_t)groups.size() > cap) fail(DFMI_ERR_INVALID_ARGUMENT, "group capacity too small");
        int64_t g = 0, pos = 0;
        const bool want_bytes = key_offsets && key_part >= 0 && key_part < nkeys && key[key_part].t == DFMI_TYPE_UTF8;
        if (want_bytes) key_offsets[0] = 0;
        for (const auto& [gk, v] : groups) {
            for (int k = 0; k < nkeys; ++k) {
                dfmi_agg_value& kv = keys[g * nkeys + k];
                kv.type = key[k].t;
                kv.is_null = gk.k[k].null ? 1 : 0;
                kv.bits = v.bits[k];
                kv.count = v.rows;
            }
            for (int j = 0; j < n; ++j) out[g * n + j] = agg_result(v.st[j]);
            if (want_bytes) {  // the key part's column as a BinaryArray
                const std::string& s = gk.k[key_part].s;
                if (pos + (int64_t)s.size() > key_data_cap) fail(DFMI_ERR_INVALID_ARGUMENT, "key bytes capacity");
                memcpy(key_data + pos, s.data(), s.size());
                pos += (int64_t)s.size();
                key_offsets[g + 1] = (int32_t)pos;
            }
            ++g;
        }
        return DFMI_OK;
    } catch (const ExecError& e) {
        set_err(err, e.code, e.msg);
        return e.code;
    }
}

// The one-key form: group_expr = [key].
int32_t oracle_aggregate_grouped(const dfmi_expr_node* pred_nodes, int32_t pred_len, const dfmi_expr_node* key_nodes,
                                 int32_t key_len, const char* const* names, const dfmi_expr_node* const* arg_nodes,
                                 const int32_t* arg_lens, const int32_t* return_types, int32_t n,
                                 const dfmi_schema* schema, const dfmi_batch* input, int64_t batch_rows,
                                 uint32_t flags, int64_t cap, dfmi_agg_value* keys, dfmi_agg_value* out,
                                 int64_t* num_groups, int32_t* key_offsets, uint8_t* key_data, int64_t key_data_cap,
                                 dfmi_error* err) {
    const dfmi_expr_node* kn[1] = {key_nodes};
    const int32_t kl[1] = {key_len};
    return oracle_aggregate_grouped_multi(pred_nodes, pred_len, kn, kl, 1, names, arg_nodes, arg_lens, return_types, n,
                                          schema, input, batch_rows, flags, cap, keys, out, num_groups, 0, key_offsets,
                                          key_data, key_data_cap, err);
}

// Counter-based generator shared with the device (datafusion_amd/csrc/gen.hip).
uint64_t oracle_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static uint64_t col_key(uint64_t seed, uint32_t col) {
    return oracle_splitmix64(seed + (uint64_t)col * 0xD1B54A32D192ED03ull);
}

void oracle_gen_unit_f64(uint64_t seed, uint32_t col, int64_t row0, int64_t n, double* out) {
    const uint64_t k = col_key(seed, col);
    for (int64_t i = 0; i < n; ++i)
        out[i] = (double)(oracle_splitmix64(k ^ (uint64_t)(row0 + i)) >> 11) * 0x1.0p-53;
}

void oracle_gen_i64(uint64_t seed, uint32_t col, int64_t row0, int64_t n, int64_t lo, int64_t hi,
                    int64_t* out) {
    const uint64_t k = col_key(seed, col);
    const uint64_t range = (uint64_t)(hi - lo);
    for (int64_t i = 0; i < n; ++i)
        out[i] = lo + (int64_t)(oracle_splitmix64(k ^ (uint64_t)(row0 + i)) % range);
}

}  // extern "C"
