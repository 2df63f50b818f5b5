// dfmi_filter_project: host side of the fused Selection + Projection pass.
//
// Lowers the compiled predicate / projections (dfmi_program IR) into one
// device accumulator program (dfmi_internal.h), decides which input columns
// the pass must load, launches k_filter_project (Selection present) or
// k_project (projection only), and maps device error words back to the
// reference's errors (FilterRelation::next filter.rs:46-72, filter()
// filter.rs:80-111, ProjectRelation::next projection.rs:45-66).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "dfmi_internal.h"
#include "dfmi_program.h"
#include "../../include/dfmi_datasource.h"

namespace dfmi {
hipError_t launch_filter_project(const DLaunch& L, bool nullable, int cfg, hipStream_t st);
hipError_t launch_project(const DLaunch& L, bool nullable, int cfg, hipStream_t st);
hipError_t launch_pack_bools(const uint8_t* bytes, uint8_t* bits, const unsigned long long* count,
                             long long max_rows, hipStream_t st);
int tile_rows_for(int cfg);
}  // namespace dfmi

using namespace dfmi;

// Workspace header layout (device, zeroed before every launch).
static constexpr size_t kHdrTicket = 0;
static constexpr size_t kHdrErr = 8;
static constexpr size_t kHdrTotals = 16;
static constexpr size_t kHdrBytes = 16 + 8 * (kMaxChan + kMaxOut) + 8;  // padded below
static constexpr size_t kHdrAlloc = 512;

struct dfmi_context {
    int device = 0;
    hipStream_t stream = nullptr;
    uint8_t* ws = nullptr;       // header + look-back status
    size_t ws_bytes = 0;
    uint8_t* scratch = nullptr;  // Boolean output bytes (filtered)
    size_t scratch_bytes = 0;
    uint8_t* host_hdr = nullptr; // pinned copy of the header
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
    double last_total_ms = 0, last_main_ms = 0;
    bool timed = false;
};

namespace {

struct Fail {
    int32_t code;
    std::string msg;
};

void set_err(dfmi_error* err, int32_t code, const std::string& m) {
    if (!err) return;
    err->code = code;
    snprintf(err->message, sizeof err->message, "%s", m.c_str());
}

#define HIP_TRY(x)                                                                         \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) throw Fail{DFMI_ERR_DEVICE, std::string(#x ": ") + hipGetErrorString(e_)}; \
    } while (0)

bool is8(int t) { return t == DFMI_TYPE_INT64 || t == DFMI_TYPE_FLOAT64; }
bool gatherable(int t, uint32_t flags) {
    if (t == DFMI_TYPE_FLOAT64 || t == DFMI_TYPE_UTF8) return true;  // filter.rs:84,94
    // extension: every fixed-width type (the device lowers the 8-byte ones and
    // Boolean; others report NotImplemented)
    if (flags & DFMI_FLAG_EXT_GATHER_ALL) return is_numeric_type(t) || t == DFMI_TYPE_BOOLEAN;
    return false;
}

// A candidate error: the reference raises the one with the smallest ordinal.
struct Err {
    bool set = false;
    uint64_t key = ~0ull;  // ordinal << 44 | row << 4
    int32_t code = 0;
    std::string msg;
    void offer(uint64_t k, int32_t c, const std::string& m) {
        if (!set || k < key) {
            set = true;
            key = k;
            code = c;
            msg = m;
        }
    }
};

struct Opnd {
    enum Kind { NUM, BOOL, UTF8COL, UTF8LIT } what = NUM;
    int kind = KD_LIT;  // NUM: KD_*
    int idx = 0;        // NUM index, bool slot, utf8 index, strlit index
};

struct Lower {
    DLaunch L;
    const dfmi_batch* in = nullptr;
    uint32_t flags = 0;
    std::vector<int> num_cols, bool_cols, utf8_cols;  // input column per slot
    unsigned bool_used = 0;                           // bool temp slots in use
    int tmp_depth = 0, tmp_max = 0;
    int n_ins = 0, n_lits = 0, n_strlits = 0, strlit_bytes = 0;
    int ordinal_base = 0;
    bool nullable = false;

    Lower() { memset(&L, 0, sizeof L); }

    [[noreturn]] void limit(const std::string& what) {
        throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "device program limit: " + what};
    }

    int slot_of(std::vector<int>& v, int col, int cap, const char* what) {
        for (size_t i = 0; i < v.size(); ++i)
            if (v[i] == col) return (int)i;
        if ((int)v.size() >= cap) limit(std::string("too many ") + what + " columns");
        v.push_back(col);
        return (int)v.size() - 1;
    }

    void collect(const dfmi_program* p) {  // pre-register referenced columns
        for (const IrNode& n : p->ir) {
            if (n.kind != IR_COL) continue;
            if (n.type == DFMI_TYPE_BOOLEAN) slot_of(bool_cols, n.col, kMaxBoolCols, "Boolean");
            else if (n.type == DFMI_TYPE_UTF8) slot_of(utf8_cols, n.col, kMaxUtf8, "Utf8");
            else if (is8(n.type)) slot_of(num_cols, n.col, kMaxNum, "numeric");
        }
    }

    int alloc_bool() {
        for (int s = (int)bool_cols.size(); s < 32; ++s)
            if (!(bool_used >> s & 1)) {
                bool_used |= 1u << s;
                return s;
            }
        limit("too many boolean temporaries");
    }
    void free_bool(int s) {
        if (s >= (int)bool_cols.size()) bool_used &= ~(1u << s);
    }

    int lit(uint64_t bits) {
        for (int i = 0; i < n_lits; ++i)
            if (L.lits[i] == bits) return i;
        if (n_lits >= kMaxLits) limit("too many literals");
        L.lits[n_lits] = bits;
        return n_lits++;
    }

    int strlit(const std::string& s) {
        if (n_strlits >= kMaxStrLits || strlit_bytes + (int)s.size() > kStrLitBytes) limit("string literals");
        L.strlit_off[n_strlits] = strlit_bytes;
        L.strlit_len[n_strlits] = (int)s.size();
        memcpy(L.strlit + strlit_bytes, s.data(), s.size());
        strlit_bytes += (int)s.size();
        return n_strlits++;
    }

    void emit(uint8_t op, int dst, int a, int b, int ka, int kb, int ordinal) {
        if (n_ins >= kMaxIns) limit("too many instructions");
        DIns& i = L.ins[n_ins++];
        i.op = op;
        i.dst = (uint8_t)dst;
        i.a = (uint8_t)a;
        i.b = (uint8_t)b;
        i.ka = (uint8_t)ka;
        i.kb = (uint8_t)kb;
        i.ordinal = (uint16_t)(ordinal_base + ordinal);
    }

    static bool is_acc_producer(const dfmi_program* p, int i) {
        const IrNode& n = p->ir[i];
        return n.kind == IR_BIN && n.rt_code == 0 && n.op >= DFMI_OP_PLUS && n.op <= DFMI_OP_DIVIDE;
    }

    // Evaluate node i; numeric results come back as an operand (column,
    // literal, or the accumulator), Booleans as a bool slot.
    Opnd gen(const dfmi_program* p, int i) {
        const IrNode& n = p->ir[i];
        Opnd o;
        if (n.kind == IR_COL) {
            if (n.type == DFMI_TYPE_BOOLEAN) {
                o.what = Opnd::BOOL;
                o.idx = slot_of(bool_cols, n.col, kMaxBoolCols, "Boolean");
            } else if (n.type == DFMI_TYPE_UTF8) {
                o.what = Opnd::UTF8COL;
                o.idx = slot_of(utf8_cols, n.col, kMaxUtf8, "Utf8");
            } else if (is8(n.type)) {
                o.kind = KD_COL;
                o.idx = slot_of(num_cols, n.col, kMaxNum, "numeric");
            } else {
                throw Fail{DFMI_ERR_NOT_IMPLEMENTED,
                           std::string("device path: ") + type_debug(n.type) + " column in an expression"};
            }
            return o;
        }
        if (n.kind == IR_LIT) {
            if (n.type == DFMI_TYPE_UTF8) {
                o.what = Opnd::UTF8LIT;
                o.idx = strlit(n.str);
                return o;
            }
            if (!is8(n.type))
                throw Fail{DFMI_ERR_NOT_IMPLEMENTED,
                           std::string("device path: ") + type_debug(n.type) + " literal"};
            o.kind = KD_LIT;
            o.idx = lit(n.bits);
            return o;
        }
        // IR_BIN
        if (n.rt_code) {
            // The reference evaluates both children before failing here: lower
            // them for their dynamic errors, then a placeholder value.
            try {
                Opnd a = gen(p, n.l);
                if (a.what == Opnd::BOOL) free_bool(a.idx);
                Opnd b = gen(p, n.r);
                if (b.what == Opnd::BOOL) free_bool(b.idx);
            } catch (const Fail&) {
            }
            if (n.type == DFMI_TYPE_BOOLEAN) {
                o.what = Opnd::BOOL;
                o.idx = alloc_bool();
                emit(OP_BLIT, o.idx, 0, 0, 0, 0, n.ordinal);
            } else {
                o.kind = KD_LIT;
                o.idx = lit(0);
            }
            return o;
        }
        const int op = n.op;
        if (op == DFMI_OP_AND || op == DFMI_OP_OR) {
            Opnd a = gen(p, n.l);
            Opnd b = gen(p, n.r);
            free_bool(a.idx);
            free_bool(b.idx);
            o.what = Opnd::BOOL;
            o.idx = alloc_bool();
            emit(op == DFMI_OP_AND ? OP_AND : OP_OR, o.idx, a.idx, b.idx, 0, 0, n.ordinal);
            return o;
        }
        const int lt = p->ir[n.l].type;
        if (lt == DFMI_TYPE_UTF8) {  // extension: Utf8 =, !=
            Opnd a = gen(p, n.l);
            Opnd b = gen(p, n.r);
            const bool eq = op == DFMI_OP_EQ;
            o.what = Opnd::BOOL;
            o.idx = alloc_bool();
            if (a.what == Opnd::UTF8LIT && b.what == Opnd::UTF8LIT) {
                const bool same = p->ir[n.l].str == p->ir[n.r].str;
                emit(OP_BLIT, o.idx, 0, (same == eq) ? 1 : 0, 0, 0, n.ordinal);
            } else if (a.what == Opnd::UTF8COL && b.what == Opnd::UTF8COL) {
                emit(eq ? OP_EQ_UTF8_COL : OP_NE_UTF8_COL, o.idx, a.idx, b.idx, 0, 0, n.ordinal);
            } else {
                const Opnd& c = a.what == Opnd::UTF8COL ? a : b;
                const Opnd& s = a.what == Opnd::UTF8COL ? b : a;
                emit(eq ? OP_EQ_UTF8_LIT : OP_NE_UTF8_LIT, o.idx, c.idx, s.idx, 0, 0, n.ordinal);
            }
            return o;
        }
        if (!is8(lt))
            throw Fail{DFMI_ERR_NOT_IMPLEMENTED, std::string("device path: ") + type_debug(lt) + " arithmetic"};
        const bool f64 = lt == DFMI_TYPE_FLOAT64;
        Opnd a, b;
        int t = -1;
        if (is_acc_producer(p, n.l) && is_acc_producer(p, n.r)) {
            a = gen(p, n.l);
            if (tmp_depth >= kMaxTmp) limit("expression too deep");
            t = tmp_depth++;
            tmp_max = std::max(tmp_max, tmp_depth);
            emit(OP_SAVE, t, 0, 0, 0, 0, n.ordinal);
            a.kind = KD_TMP;
            a.idx = t;
            b = gen(p, n.r);
        } else {
            a = gen(p, n.l);
            b = gen(p, n.r);
        }
        static const uint8_t cmp_i[6] = {OP_EQ_I64, OP_NE_I64, OP_LT_I64, OP_LE_I64, OP_GT_I64, OP_GE_I64};
        static const uint8_t cmp_f[6] = {OP_EQ_F64, OP_NE_F64, OP_LT_F64, OP_LE_F64, OP_GT_F64, OP_GE_F64};
        static const uint8_t math_i[4] = {OP_ADD_I64, OP_SUB_I64, OP_MUL_I64, OP_DIV_I64};
        static const uint8_t math_f[4] = {OP_ADD_F64, OP_SUB_F64, OP_MUL_F64, OP_DIV_F64};
        if (op <= DFMI_OP_GT_EQ) {
            o.what = Opnd::BOOL;
            o.idx = alloc_bool();
            emit(f64 ? cmp_f[op] : cmp_i[op], o.idx, a.idx, b.idx, a.kind, b.kind, n.ordinal);
        } else {
            emit(f64 ? math_f[op - DFMI_OP_PLUS] : math_i[op - DFMI_OP_PLUS], 0, a.idx, b.idx, a.kind,
                 b.kind, n.ordinal);
            o.kind = KD_ACC;
            o.idx = 0;
        }
        if (t >= 0) --tmp_depth;
        return o;
    }

    void fill_columns() {
        L.n_num = (int)num_cols.size();
        L.n_bool = (int)bool_cols.size();
        L.n_utf8 = (int)utf8_cols.size();
        const int64_t n = in->num_rows;
        for (size_t i = 0; i < num_cols.size(); ++i) {
            const dfmi_column& c = in->columns[num_cols[i]];
            if (!c.values) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "column values pointer is NULL"};
            if ((uintptr_t)c.values & 7) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "column values must be 8-byte aligned"};
            L.num[i].values = c.values;
            L.num[i].validity = (c.validity && c.null_count > 0) ? c.validity : nullptr;
            L.num[i].bitmap_bytes = (n + 7) / 8;
            nullable |= L.num[i].validity != nullptr;
        }
        for (size_t i = 0; i < bool_cols.size(); ++i) {
            const dfmi_column& c = in->columns[bool_cols[i]];
            if (!c.values) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "column values pointer is NULL"};
            L.boolc[i].values = c.values;
            L.boolc[i].validity = (c.validity && c.null_count > 0) ? c.validity : nullptr;
            L.boolc[i].bitmap_bytes = (n + 7) / 8;
            nullable |= L.boolc[i].validity != nullptr;
        }
        for (size_t i = 0; i < utf8_cols.size(); ++i) {
            const dfmi_column& c = in->columns[utf8_cols[i]];
            if (!c.values || !c.offsets) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "Utf8 column buffers are NULL"};
            L.utf8[i].values = c.values;
            L.utf8[i].offsets = c.offsets;
            L.utf8[i].validity = (c.validity && c.null_count > 0) ? c.validity : nullptr;
            L.utf8[i].bitmap_bytes = (n + 7) / 8;
            nullable |= L.utf8[i].validity != nullptr;
        }
    }
};

void ensure(dfmi_context* ctx, uint8_t** buf, size_t* have, size_t need) {
    if (*have >= need) return;
    if (*buf) HIP_TRY(hipFree(*buf));
    *buf = nullptr;
    *have = 0;
    size_t cap = std::max(need, (size_t)1 << 20);
    HIP_TRY(hipMalloc(buf, cap));
    *have = cap;
}

}  // namespace

extern "C" int32_t dfmi_context_create(int32_t device, void* stream, dfmi_context** out, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    if (!out) {
        set_err(err, DFMI_ERR_INVALID_ARGUMENT, "out is NULL");
        return DFMI_ERR_INVALID_ARGUMENT;
    }
    dfmi_context* c = new (std::nothrow) dfmi_context();
    if (!c) return DFMI_ERR_INVALID_ARGUMENT;
    try {
        HIP_TRY(hipSetDevice(device));
        c->device = device;
        c->stream = (hipStream_t)stream;
        HIP_TRY(hipHostMalloc((void**)&c->host_hdr, kHdrAlloc, hipHostMallocDefault));
        HIP_TRY(hipEventCreate(&c->ev0));
        HIP_TRY(hipEventCreate(&c->ev1));
        HIP_TRY(hipEventCreate(&c->ev2));
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        delete c;
        return f.code;
    }
    *out = c;
    return DFMI_OK;
}

extern "C" void dfmi_context_destroy(dfmi_context* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->ws) (void)hipFree(c->ws);
    if (c->scratch) (void)hipFree(c->scratch);
    if (c->host_hdr) (void)hipHostFree(c->host_hdr);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->ev2) (void)hipEventDestroy(c->ev2);
    delete c;
}

extern "C" int32_t dfmi_context_set_stream(dfmi_context* c, void* stream) {
    if (!c) return DFMI_ERR_INVALID_ARGUMENT;
    c->stream = (hipStream_t)stream;
    return DFMI_OK;
}

extern "C" int32_t dfmi_last_timing(const dfmi_context* c, double* total_ms, double* main_ms) {
    if (!c || !c->timed) return DFMI_ERR_INVALID_ARGUMENT;
    if (total_ms) *total_ms = c->last_total_ms;
    if (main_ms) *main_ms = c->last_main_ms;
    return DFMI_OK;
}

extern "C" int32_t dfmi_filter_project(dfmi_context* ctx, const dfmi_program* pred,
                                       const dfmi_program* const* projs, int32_t np,
                                       const dfmi_batch* in, dfmi_out_column* outs, uint32_t flags,
                                       dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    try {
        if (!ctx || !in || (np > 0 && !projs) || !outs || (in->num_columns > 0 && !in->columns))
            throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        if (!pred && np == 0) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "neither a predicate nor projections"};
        const int64_t n = in->num_rows;
        const int ncols = in->num_columns;
        auto check_schema = [&](const dfmi_program* p) {
            if ((int)p->schema_types.size() != ncols)
                throw Fail{DFMI_ERR_INVALID_ARGUMENT, "batch does not match the compiled schema"};
            for (int i = 0; i < ncols; ++i)
                if (p->schema_types[i] != in->columns[i].type)
                    throw Fail{DFMI_ERR_INVALID_ARGUMENT, "batch column type does not match the schema"};
        };
        if (pred) check_schema(pred);
        for (int j = 0; j < np; ++j) {
            if (!projs[j]) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL projection"};
            check_schema(projs[j]);
        }
        for (int i = 0; i < ncols; ++i)
            if (in->columns[i].length != n) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "ragged batch"};

        // ---- errors every evaluation of this plan raises (reference order)
        Err se;
        const int P = pred ? pred->length : 0;
        if (pred) {
            for (const IrNode& nd : pred->ir)
                if (nd.rt_code) se.offer((uint64_t)nd.ordinal << 44, nd.rt_code, nd.rt_msg);
            if (pred->type != DFMI_TYPE_BOOLEAN)
                se.offer((uint64_t)P << 44, DFMI_ERR_EXECUTION, "Filter expression did not evaluate to boolean");
            for (int i = 0; i < ncols; ++i)
                if (!gatherable(in->columns[i].type, flags)) {
                    se.offer((uint64_t)(P + 1) << 44, DFMI_ERR_EXECUTION,
                             std::string("filter not supported for ") + type_debug(in->columns[i].type));
                    break;
                }
        }
        std::vector<int> proj_base(np);
        int base = P + 2;
        for (int j = 0; j < np; ++j) {
            proj_base[j] = base;
            for (const IrNode& nd : projs[j]->ir)
                if (nd.rt_code) se.offer((uint64_t)(base + nd.ordinal) << 44, nd.rt_code, nd.rt_msg);
            base += projs[j]->length;
        }
        if (base >= 65536) throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "device program limit: expressions too long"};

        // ---- output list
        const int nout = np > 0 ? np : ncols;
        if (nout > kMaxOut) throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "device program limit: too many output columns"};
        for (int o = 0; o < nout; ++o) {
            dfmi_out_column& oc = outs[o];
            oc.type = np > 0 ? projs[o]->type : in->columns[o].type;
            oc.passthrough_column = -1;
            oc.length = 0;
            oc.null_count = 0;
            oc.data_length = 0;
        }

        Lower lw;
        lw.in = in;
        lw.flags = flags;
        DLaunch& L = lw.L;
        if (pred) lw.collect(pred);
        for (int j = 0; j < np; ++j) lw.collect(projs[j]);

        // predicate program
        if (pred) {
            lw.ordinal_base = 0;
            L.pred_begin = lw.n_ins;
            Opnd r;
            try {
                r = lw.gen(pred, pred->root);
            } catch (const Fail& f) {
                if (se.set) throw Fail{se.code, se.msg};
                throw;
            }
            L.pred_end = lw.n_ins;
            if (r.what == Opnd::BOOL) {
                L.pred_slot = r.idx;
            } else {  // not Boolean: error at ordinal P; select nothing
                L.pred_slot = lw.alloc_bool();
                lw.emit(OP_BLIT, L.pred_slot, 0, 0, 0, 0, P);
                L.pred_end = lw.n_ins;
            }
        }

        // projections (or, without projections, FilterRelation's output = every column)
        L.proj_begin = lw.n_ins;
        int n_chan = 1;
        bool any_kernel_out = false;
        std::vector<int> bool_out;  // filtered Boolean outputs (scratch bytes)
        for (int o = 0; o < nout; ++o) {
            const dfmi_program* p = np > 0 ? projs[o] : nullptr;
            const IrNode* root = p ? &p->ir[p->root] : nullptr;
            const bool is_col = !p || root->kind == IR_COL;
            const int col = p ? root->col : o;
            if (is_col && !pred) {  // Arc clone of the input column (expression.rs:274)
                const dfmi_column& c = in->columns[col];
                outs[o].passthrough_column = col;
                outs[o].length = n;
                outs[o].null_count = c.validity ? c.null_count : 0;
                continue;
            }
            if (is_col && pred && !gatherable(in->columns[col].type, flags)) continue;  // error at P+1
            DOut& d = L.out[o];
            d.values = outs[o].values;
            d.validity = outs[o].validity;
            d.offsets = outs[o].offsets;
            d.data = outs[o].data;
            d.data_cap = outs[o].data_capacity;
            lw.ordinal_base = p ? proj_base[o] : 0;
            const int ctype = is_col ? in->columns[col].type : root->type;
            if (is_col && ctype == DFMI_TYPE_UTF8) {
                if (!d.offsets || !d.data) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "Utf8 output buffers are NULL"};
                d.kind = OUT_GATHER_UTF8;
                d.slot = lw.slot_of(lw.utf8_cols, col, kMaxUtf8, "Utf8");
                if (n_chan >= kMaxChan) lw.limit("too many Utf8 outputs");
                d.chan = n_chan;
                L.chan_out[n_chan - 1] = o;
                ++n_chan;
                any_kernel_out = true;
                continue;
            }
            if (!d.values) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "output values pointer is NULL"};
            any_kernel_out = true;
            if (is_col) {
                if (ctype == DFMI_TYPE_BOOLEAN) {
                    d.kind = OUT_GATHER_BOOL;
                    bool_out.push_back(o);
                    lw.emit(OP_STORE_BOOL, o, lw.slot_of(lw.bool_cols, col, kMaxBoolCols, "Boolean"), 0, 0, 0, 0);
                } else if (is8(ctype)) {
                    d.kind = OUT_GATHER_NUM;
                    lw.emit(OP_STORE_COL, o, lw.slot_of(lw.num_cols, col, kMaxNum, "numeric"), 0, 0, 0, 0);
                } else {
                    throw Fail{DFMI_ERR_NOT_IMPLEMENTED,
                               std::string("device path: gather of ") + type_debug(ctype) + " columns"};
                }
                continue;
            }
            Opnd r;
            try {
                r = lw.gen(p, p->root);
            } catch (const Fail& f) {
                if (se.set) throw Fail{se.code, se.msg};
                throw;
            }
            if (r.what == Opnd::BOOL) {
                d.kind = OUT_EXPR_BOOL;
                if (pred) bool_out.push_back(o);
                lw.emit(OP_STORE_BOOL, o, r.idx, 0, 0, 0, 0);
                lw.free_bool(r.idx);
            } else if (r.what == Opnd::NUM) {
                d.kind = OUT_EXPR_NUM;
                if (r.kind == KD_COL) {
                    lw.emit(OP_STORE_COL, o, r.idx, 0, 0, 0, 0);
                } else {
                    if (r.kind != KD_ACC) lw.emit(OP_MOVE, 0, r.idx, 0, r.kind, 0, 0);
                    lw.emit(OP_STORE_ACC, o, 0, 0, 0, 0, 0);
                }
            } else {
                throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "device path: Utf8-valued projection"};
            }
        }
        L.proj_end = lw.n_ins;
        L.n_out = nout;
        L.n_chan = n_chan;
        L.n_tmp = lw.tmp_max;
        L.n_rows = n;
        if (const char* m = getenv("DFMI_DEBUG_MODE")) L.mode = atoi(m);  // diagnostics only
        lw.fill_columns();

        // ---- execute
        HIP_TRY(hipSetDevice(ctx->device));
        hipStream_t st = ctx->stream;
        ctx->timed = false;
        int nc = 3;  // tile shape (kernels.hip host launchers): 1024 threads x 4 rows
        if (const char* c = getenv("DFMI_TILE_CFG")) nc = atoi(c);  // diagnostics only
        const int tile = tile_rows_for(nc);
        // stage as many numeric columns in LDS as fit 64 KiB per block
        // (predicate columns first: Lower::collect registers them first)
        {
            const int cap = (int)(65536 / ((size_t)tile * 8)) - L.n_tmp;
            L.n_lds = std::max(0, std::min(L.n_num, cap));
            if (const char* c = getenv("DFMI_NO_LDS")) { if (atoi(c)) L.n_lds = 0; }  // diagnostics only
        }
        const int64_t n_tiles = (n + tile - 1) / tile;
        if (n_tiles > 0x7fffffff) throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "batch too large"};
        L.n_tiles = (int32_t)n_tiles;

        const bool launch = n > 0 && (pred || any_kernel_out);
        uint64_t dev_key = ~0ull;
        int dev_kind = 0;
        if (launch) {
            const size_t status_bytes = pred ? (size_t)n_chan * n_tiles * 8 : 0;
            ensure(ctx, &ctx->ws, &ctx->ws_bytes, kHdrAlloc + status_bytes);
            if (pred && !bool_out.empty())
                ensure(ctx, &ctx->scratch, &ctx->scratch_bytes, bool_out.size() * (size_t)((n + 63) & ~63ll));
            L.ticket = (unsigned*)(ctx->ws + kHdrTicket);
            L.err = (unsigned long long*)(ctx->ws + kHdrErr);
            L.totals = (unsigned long long*)(ctx->ws + kHdrTotals);
            L.status = (unsigned long long*)(ctx->ws + kHdrAlloc);
            std::vector<uint8_t*> bool_dst;
            if (pred) {
                for (size_t i = 0; i < bool_out.size(); ++i) {
                    DOut& d = L.out[bool_out[i]];
                    bool_dst.push_back((uint8_t*)d.values);
                    d.values = ctx->scratch + i * (size_t)((n + 63) & ~63ll);
                }
            }
            HIP_TRY(hipMemsetAsync(ctx->ws, 0, kHdrAlloc + status_bytes, st));
            HIP_TRY(hipEventRecord(ctx->ev0, st));
            if (pred) HIP_TRY(launch_filter_project(L, lw.nullable, nc, st));
            else HIP_TRY(launch_project(L, lw.nullable, nc, st));
            HIP_TRY(hipEventRecord(ctx->ev1, st));
            for (size_t i = 0; i < bool_dst.size(); ++i)
                HIP_TRY(launch_pack_bools((const uint8_t*)L.out[bool_out[i]].values, bool_dst[i],
                                          L.totals, n, st));
            HIP_TRY(hipMemcpyAsync(ctx->host_hdr, ctx->ws, kHdrAlloc, hipMemcpyDeviceToHost, st));
            HIP_TRY(hipEventRecord(ctx->ev2, st));
            HIP_TRY(hipStreamSynchronize(st));
            float m1 = 0, m2 = 0;
            (void)hipEventElapsedTime(&m1, ctx->ev0, ctx->ev1);
            (void)hipEventElapsedTime(&m2, ctx->ev0, ctx->ev2);
            ctx->last_main_ms = m1;
            ctx->last_total_ms = m2;
            ctx->timed = true;
            uint64_t ew;
            memcpy(&ew, ctx->host_hdr + kHdrErr, 8);
            if (ew) {
                dev_key = ~ew;
                dev_kind = (int)(dev_key & 15);
                dev_key &= ~15ull;
            }
        }
        (void)kHdrBytes;

        // ---- errors: the reference raises the first in evaluation order
        if (dev_kind == ERRK_LOOKBACK_TIMEOUT)
            throw Fail{DFMI_ERR_DEVICE, "device look-back timed out"};
        if (dev_kind == ERRK_CAPACITY)
            throw Fail{DFMI_ERR_CAPACITY, "Utf8 output data_capacity too small"};
        if (dev_kind && (!se.set || dev_key < se.key)) {
            if (dev_kind == ERRK_DIV_ZERO) throw Fail{DFMI_ERR_DIVIDE_BY_ZERO, "DivideByZero"};
            throw Fail{DFMI_ERR_PANIC, "attempt to divide with overflow"};
        }
        if (se.set) throw Fail{se.code, se.msg};

        // ---- results
        uint64_t totals[kMaxChan + kMaxOut];
        memset(totals, 0, sizeof totals);
        if (launch) memcpy(totals, ctx->host_hdr + kHdrTotals, sizeof totals);
        const int64_t out_rows = pred ? (int64_t)totals[0] : n;
        for (int o = 0; o < nout; ++o) {
            dfmi_out_column& oc = outs[o];
            if (oc.passthrough_column >= 0) continue;
            oc.length = out_rows;
            oc.null_count = pred ? 0 : (int64_t)totals[kMaxChan + o];
            if (L.out[o].kind == OUT_GATHER_UTF8) {
                oc.data_length = (int64_t)totals[L.out[o].chan];
                if (!launch || out_rows == 0) {  // offsets = [0]
                    if (oc.offsets) HIP_TRY(hipMemsetAsync(oc.offsets, 0, 4, st));
                    oc.data_length = 0;
                }
            }
        }
        if (!launch) HIP_TRY(hipStreamSynchronize(st));
        return DFMI_OK;
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

// ---------------------------------------------------------------- datasource
namespace dfmi {
hipError_t launch_gen_unit_f64(unsigned long long key, long long row0, long long n, double* out,
                               hipStream_t st);
hipError_t launch_gen_i64(unsigned long long key, long long row0, long long n, long long lo,
                          unsigned long long range, long long* out, hipStream_t st);
}  // namespace dfmi

static uint64_t host_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

extern "C" int32_t dfmi_generate_column(dfmi_context* ctx, int32_t kind, uint64_t seed, uint32_t col,
                                        int64_t row0, int64_t n, int64_t lo, int64_t hi, void* out,
                                        dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    try {
        if (!ctx || !out || n < 0) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "bad argument"};
        HIP_TRY(hipSetDevice(ctx->device));
        const uint64_t key = host_splitmix64(seed + (uint64_t)col * 0xD1B54A32D192ED03ull);
        if (kind == DFMI_GEN_UNIT_F64) {
            HIP_TRY(launch_gen_unit_f64(key, row0, n, (double*)out, ctx->stream));
        } else if (kind == DFMI_GEN_I64) {
            if (hi <= lo) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "empty range"};
            HIP_TRY(launch_gen_i64(key, row0, n, lo, (uint64_t)(hi - lo), (long long*)out, ctx->stream));
        } else {
            throw Fail{DFMI_ERR_INVALID_ARGUMENT, "unknown generator"};
        }
        return DFMI_OK;
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return f.code;
    }
}
