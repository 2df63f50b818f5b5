// compile_scalar_expr front end of libdfmi (host C++).
//
// Restates src/execution/expression.rs:244-451 as a checker + typed IR: it
// rejects at compile time exactly what the reference rejects at compile time
// (same ExecutionError variant and text), computes RuntimeExpr names/types
// (expression.rs:64-77, Debug of Expr logicalplan.rs:263-303), and records the
// errors the reference would raise only when the closure runs (comparison_ops,
// math_ops, boolean_ops' unwrap panic) so execution reports them in the
// reference's order.
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "dfmi_program.h"

namespace dfmi {

const char* type_debug(int t) {
    static const char* names[] = {"Null", "Boolean", "Int8", "Int16", "Int32", "Int64", "UInt8",
                                  "UInt16", "UInt32", "UInt64", "Float32", "Float64", "Utf8"};
    return (t >= 0 && t <= 12) ? names[t] : "Null";
}

static const char* op_debug(int op) {
    static const char* names[] = {"Eq", "NotEq", "Lt", "LtEq", "Gt", "GtEq", "Plus",
                                  "Minus", "Multiply", "Divide", "Modulus", "And", "Or"};
    return (op >= 0 && op <= 12) ? names[op] : "?";
}

bool is_numeric_type(int t) { return t >= DFMI_TYPE_INT8 && t <= DFMI_TYPE_FLOAT64; }

// Rust (2018) float formatting: shortest round-trip digits, plain decimal;
// Debug appends ".0" to integral values, Display drops the sign of -0.
std::string rust_float(double v, bool f32, bool debug) {
    if (std::isnan(v)) return "NaN";
    if (std::isinf(v)) return v > 0 ? "inf" : "-inf";
    const bool neg = std::signbit(v);
    std::string sign = (neg && (v != 0.0 || debug)) ? "-" : "";
    const double a = std::fabs(v);
    if (a == 0.0) return sign + (debug ? "0.0" : "0");
    char buf[64];
    for (int p = 1; p <= 17; ++p) {
        snprintf(buf, sizeof buf, "%.*e", p - 1, a);
        const double back = strtod(buf, nullptr);
        if (f32 ? ((float)back == (float)a) : (back == a)) break;
    }
    const char* e = strchr(buf, 'e');
    const int e10 = atoi(e + 1);
    std::string d;
    for (const char* c = buf; c < e; ++c)
        if (*c >= '0' && *c <= '9') d.push_back(*c);
    while (d.size() > 1 && d.back() == '0') d.pop_back();
    const int point = e10 + 1;
    std::string out;
    if (point <= 0) {
        out = "0." + std::string(-point, '0') + d;
    } else if ((size_t)point >= d.size()) {
        out = d + std::string(point - d.size(), '0') + (debug ? ".0" : "");
    } else {
        out = d.substr(0, point) + "." + d.substr(point);
    }
    return sign + out;
}

static std::string str_debug(const std::string& s) {
    std::string o = "\"";
    for (unsigned char c : s) {
        if (c == '"') o += "\\\"";
        else if (c == '\\') o += "\\\\";
        else if (c == '\n') o += "\\n";
        else if (c == '\r') o += "\\r";
        else if (c == '\t') o += "\\t";
        else if (c == 0) o += "\\0";
        else if (c < 0x20 || c == 0x7f) {
            char b[16];
            snprintf(b, sizeof b, "\\u{%x}", c);
            o += b;
        } else {
            o.push_back((char)c);
        }
    }
    return o + "\"";
}

static std::string scalar_debug(const dfmi_expr_node& n) {
    char b[80];
    switch (n.data_type) {
        case DFMI_TYPE_NULL: return "Null";
        case DFMI_TYPE_BOOLEAN: return std::string("Boolean(") + (n.i64 ? "true" : "false") + ")";
        case DFMI_TYPE_FLOAT32: return "Float32(" + rust_float(n.f64, true, true) + ")";
        case DFMI_TYPE_FLOAT64: return "Float64(" + rust_float(n.f64, false, true) + ")";
        case DFMI_TYPE_UTF8:
            return "Utf8(" + str_debug(std::string(n.str ? n.str : "", (size_t)n.str_len)) + ")";
        case DFMI_TYPE_UINT8: case DFMI_TYPE_UINT16: case DFMI_TYPE_UINT32: case DFMI_TYPE_UINT64:
            snprintf(b, sizeof b, "%s(%llu)", type_debug(n.data_type), (unsigned long long)n.i64);
            return b;
        default:
            snprintf(b, sizeof b, "%s(%lld)", type_debug(n.data_type), (long long)n.i64);
            return b;
    }
}

namespace {

struct Tree {
    int node;                 // index into the postfix array
    std::vector<int> kids;    // tree indices
};

struct Builder {
    const dfmi_expr_node* nodes;
    int n;
    std::vector<Tree> trees;
    int root = -1;
};

bool build(const dfmi_expr_node* nodes, int n, Builder& b, std::string& why) {
    b.nodes = nodes;
    b.n = n;
    std::vector<int> st;
    for (int i = 0; i < n; ++i) {
        int arity;
        switch (nodes[i].kind) {
            case DFMI_EXPR_COLUMN: case DFMI_EXPR_LITERAL: arity = 0; break;
            case DFMI_EXPR_BINARY: arity = 2; break;
            case DFMI_EXPR_CAST: case DFMI_EXPR_IS_NULL: case DFMI_EXPR_IS_NOT_NULL:
            case DFMI_EXPR_SORT: arity = 1; break;
            case DFMI_EXPR_SCALAR_FUNCTION: case DFMI_EXPR_AGGREGATE_FUNCTION:
                arity = nodes[i].column; break;
            default: why = "unknown expression node kind"; return false;
        }
        if (arity < 0 || (int)st.size() < arity) {
            why = "malformed postfix expression";
            return false;
        }
        Tree t;
        t.node = i;
        t.kids.assign(st.end() - arity, st.end());
        st.resize(st.size() - arity);
        b.trees.push_back(t);
        st.push_back((int)b.trees.size() - 1);
    }
    if (st.size() != 1) {
        why = "malformed postfix expression";
        return false;
    }
    b.root = st[0];
    return true;
}

std::string expr_debug(const Builder& b, int t) {
    const dfmi_expr_node& n = b.nodes[b.trees[t].node];
    const std::vector<int>& k = b.trees[t].kids;
    switch (n.kind) {
        case DFMI_EXPR_COLUMN: return "#" + std::to_string(n.column);
        case DFMI_EXPR_LITERAL: return scalar_debug(n);
        case DFMI_EXPR_CAST:
            return "CAST(" + expr_debug(b, k[0]) + " AS " + type_debug(n.data_type) + ")";
        case DFMI_EXPR_IS_NULL: return expr_debug(b, k[0]) + " IS NULL";
        case DFMI_EXPR_IS_NOT_NULL: return expr_debug(b, k[0]) + " IS NOT NULL";
        case DFMI_EXPR_BINARY:
            return expr_debug(b, k[0]) + " " + op_debug(n.op) + " " + expr_debug(b, k[1]);
        case DFMI_EXPR_SORT: return expr_debug(b, k[0]) + (n.op ? " ASC" : " DESC");
        default: {
            std::string s = n.str ? std::string(n.str, (size_t)n.str_len) : std::string();
            s += "(";
            for (size_t i = 0; i < k.size(); ++i) {
                if (i) s += ", ";
                s += expr_debug(b, k[i]);
            }
            return s + ")";
        }
    }
}

struct CompileError {
    int32_t code;
    std::string msg;
};

// Returns the IR index of the compiled node; throws CompileError for what
// compile_scalar_expr rejects.
int compile_node(const Builder& b, int t, const dfmi_schema& s, uint32_t flags, dfmi_program& p) {
    const dfmi_expr_node& n = b.nodes[b.trees[t].node];
    const std::vector<int>& kids = b.trees[t].kids;
    IrNode ir;
    switch (n.kind) {
        case DFMI_EXPR_LITERAL: {  // expression.rs:253-271
            const int dt = n.data_type;
            if (dt == DFMI_TYPE_UTF8 && (flags & DFMI_FLAG_EXT_UTF8_COMPARE)) {
                ir.kind = IR_LIT;
                ir.type = DFMI_TYPE_UTF8;
                ir.str.assign(n.str ? n.str : "", (size_t)n.str_len);
                ir.name = ir.str;
                break;
            }
            if (!is_numeric_type(dt))
                throw CompileError{DFMI_ERR_EXECUTION, "No support for literal type " + scalar_debug(n)};
            ir.kind = IR_LIT;
            ir.type = dt;
            if (dt == DFMI_TYPE_FLOAT64 || dt == DFMI_TYPE_FLOAT32) {
                ir.name = rust_float(n.f64, dt == DFMI_TYPE_FLOAT32, false);
                if (dt == DFMI_TYPE_FLOAT64) {
                    memcpy(&ir.bits, &n.f64, 8);
                } else {
                    float f = (float)n.f64;
                    uint32_t u;
                    memcpy(&u, &f, 4);
                    ir.bits = u;
                }
            } else if (dt >= DFMI_TYPE_UINT8 && dt <= DFMI_TYPE_UINT64) {
                ir.name = std::to_string((unsigned long long)n.i64);
                ir.bits = (uint64_t)n.i64;
            } else {
                ir.name = std::to_string((long long)n.i64);
                ir.bits = (uint64_t)n.i64;
            }
            break;
        }
        case DFMI_EXPR_COLUMN: {  // expression.rs:272-276
            if (n.column < 0 || n.column >= s.num_fields)
                throw CompileError{DFMI_ERR_PANIC, "index out of bounds: the len is " +
                                                       std::to_string(s.num_fields) + " but the index is " +
                                                       std::to_string(n.column)};
            ir.kind = IR_COL;
            ir.col = n.column;
            ir.type = s.fields[n.column].type;
            ir.name = s.fields[n.column].name ? s.fields[n.column].name : "";
            break;
        }
        case DFMI_EXPR_CAST: {  // expression.rs:277-325
            const int inner = kids[0];
            const dfmi_expr_node& in = b.nodes[b.trees[inner].node];
            if ((flags & DFMI_FLAG_EXT_CAST) && in.kind != DFMI_EXPR_LITERAL) {
                // extension: CAST of a column / expression (expression.rs:281-290)
                const int c = compile_node(b, inner, s, flags, p);
                const int from = p.ir[c].type;
                if (!is_numeric_type(from) || !is_numeric_type(n.data_type))
                    throw CompileError{DFMI_ERR_NOT_IMPLEMENTED, std::string("CAST from ") + type_debug(from) +
                                                                     " to " + type_debug(n.data_type)};
                ir.kind = IR_CAST;
                ir.type = n.data_type;
                ir.l = c;
                ir.name = expr_debug(b, t);
                break;
            }
            if (in.kind == DFMI_EXPR_COLUMN) throw CompileError{DFMI_ERR_EXECUTION, "column reference"};
            if (in.kind == DFMI_EXPR_LITERAL) {
                if (in.data_type == DFMI_TYPE_INT64) {
                    if (n.data_type != DFMI_TYPE_FLOAT64)
                        throw CompileError{DFMI_ERR_NOT_IMPLEMENTED,
                                           std::string("CAST from Int64 to ") + type_debug(n.data_type)};
                    const double v = (double)in.i64;  // `nn as f64`
                    ir.kind = IR_LIT;
                    ir.type = DFMI_TYPE_FLOAT64;
                    memcpy(&ir.bits, &v, 8);
                    ir.name = "lit";
                    break;
                }
                throw CompileError{DFMI_ERR_NOT_IMPLEMENTED, "CAST from " + scalar_debug(in) + " to " +
                                                                 type_debug(n.data_type)};
            }
            throw CompileError{DFMI_ERR_GENERAL, "CAST not implemented for expression " + expr_debug(b, inner)};
        }
        case DFMI_EXPR_BINARY: {  // expression.rs:347-445
            const int l = compile_node(b, kids[0], s, flags, p);
            const int r = compile_node(b, kids[1], s, flags, p);
            ir.kind = IR_BIN;
            ir.op = n.op;
            ir.l = l;
            ir.r = r;
            ir.name = expr_debug(b, kids[0]) + " " + op_debug(n.op) + " " + expr_debug(b, kids[1]);
            const int lt = p.ir[l].type, rt = p.ir[r].type;
            if (n.op >= DFMI_OP_EQ && n.op <= DFMI_OP_GT_EQ) {
                ir.type = DFMI_TYPE_BOOLEAN;
                const bool utf8_ok = (flags & DFMI_FLAG_EXT_UTF8_COMPARE) && lt == DFMI_TYPE_UTF8 &&
                                     rt == DFMI_TYPE_UTF8 && (n.op == DFMI_OP_EQ || n.op == DFMI_OP_NOT_EQ);
                if (!((lt == rt && is_numeric_type(lt)) || utf8_ok)) {
                    ir.rt_code = DFMI_ERR_EXECUTION;
                    ir.rt_msg = "comparison_ops";
                }
            } else if (n.op == DFMI_OP_AND || n.op == DFMI_OP_OR) {
                ir.type = DFMI_TYPE_BOOLEAN;
                if (lt != DFMI_TYPE_BOOLEAN || rt != DFMI_TYPE_BOOLEAN) {
                    ir.rt_code = DFMI_ERR_PANIC;
                    ir.rt_msg = "called `Option::unwrap()` on a `None` value";
                }
            } else if (n.op >= DFMI_OP_PLUS && n.op <= DFMI_OP_DIVIDE) {
                ir.type = lt;  // op_type = left_expr.get_type()
                if (!(lt == rt && is_numeric_type(lt))) {
                    ir.rt_code = DFMI_ERR_EXECUTION;
                    ir.rt_msg = "math_ops";
                }
            } else {
                throw CompileError{DFMI_ERR_EXECUTION, std::string("operator: ") + op_debug(n.op)};
            }
            break;
        }
        case DFMI_EXPR_IS_NULL: case DFMI_EXPR_IS_NOT_NULL:
            if (flags & DFMI_FLAG_EXT_IS_NULL) {  // extension: expression.rs:326-345
                ir.kind = IR_ISNULL;
                ir.op = n.kind == DFMI_EXPR_IS_NULL ? 0 : 1;
                ir.type = DFMI_TYPE_BOOLEAN;
                ir.l = compile_node(b, kids[0], s, flags, p);
                ir.name = expr_debug(b, t);
                break;
            }
            throw CompileError{DFMI_ERR_EXECUTION, "expression " + expr_debug(b, t)};
        default:
            throw CompileError{DFMI_ERR_EXECUTION, "expression " + expr_debug(b, t)};
    }
    ir.ordinal = b.trees[t].node;  // postfix position = evaluation order
    p.ir.push_back(ir);
    return (int)p.ir.size() - 1;
}

void set_err(dfmi_error* err, int32_t code, const std::string& m) {
    if (!err) return;
    err->code = code;
    snprintf(err->message, sizeof err->message, "%s", m.c_str());
}

}  // namespace
}  // namespace dfmi

using namespace dfmi;

extern "C" int32_t dfmi_compile_scalar_expr(const dfmi_expr_node* nodes, int32_t num_nodes,
                                            const dfmi_schema* schema, uint32_t flags,
                                            dfmi_program** out, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    if (!out) {
        set_err(err, DFMI_ERR_INVALID_ARGUMENT, "out is NULL");
        return DFMI_ERR_INVALID_ARGUMENT;
    }
    *out = nullptr;
    if (!nodes || num_nodes <= 0 || !schema || (schema->num_fields > 0 && !schema->fields)) {
        set_err(err, DFMI_ERR_INVALID_ARGUMENT, "empty expression or schema");
        return DFMI_ERR_INVALID_ARGUMENT;
    }
    Builder b;
    std::string why;
    if (!build(nodes, num_nodes, b, why)) {
        set_err(err, DFMI_ERR_INVALID_ARGUMENT, why);
        return DFMI_ERR_INVALID_ARGUMENT;
    }
    dfmi_program* p = new (std::nothrow) dfmi_program();
    if (!p) {
        set_err(err, DFMI_ERR_INVALID_ARGUMENT, "out of memory");
        return DFMI_ERR_INVALID_ARGUMENT;
    }
    try {
        static std::atomic<uint64_t> next_uid{1};
        p->uid = next_uid.fetch_add(1);
        p->flags = flags;
        p->length = num_nodes;
        for (int i = 0; i < schema->num_fields; ++i) p->schema_types.push_back(schema->fields[i].type);
        p->root = compile_node(b, b.root, *schema, flags, *p);
        p->name = p->ir[p->root].name;
        p->type = p->ir[p->root].type;
    } catch (const CompileError& e) {
        delete p;
        set_err(err, e.code, e.msg);
        return e.code;
    }
    *out = p;
    return DFMI_OK;
}

extern "C" const char* dfmi_program_name(const dfmi_program* p) { return p ? p->name.c_str() : ""; }
extern "C" int32_t dfmi_program_type(const dfmi_program* p) { return p ? p->type : 0; }
extern "C" void dfmi_program_free(dfmi_program* p) { delete p; }
