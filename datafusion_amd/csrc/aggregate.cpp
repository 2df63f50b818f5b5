// Aggregate extension (DFMI_FLAG_EXT_AGGREGATE): host side of the fused
// Selection + Aggregate pass with no GROUP BY.
//
// The reference plans `SELECT SUM(e), ... FROM t [WHERE p]` as
// Aggregate(Selection?(TableScan)) (sqlplanner.rs:91-117), compiles each
// AggregateFunction with compile_expr (expression.rs:81-116) and then stops:
// ExecutionContext::execute has no Aggregate arm (context.rs:161
// `unimplemented!()`). Here every input batch is one launch of a
// query-compiled kernel (jit.cpp generate_agg): predicate, argument and
// reduction fused, partials accumulated in device memory across batches; the
// host merges the accumulator copies exactly and rounds once at the end.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <new>
#include <string>
#include <string_view>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "exec_internal.h"
#include "slice.h"
#include "jit_skeleton.hip"

using namespace dfmi;
using namespace dfmi::xi;

// One aggregate's merged state (host): the layout of a device copy with the
// float digits carry-normalised (every digit but the top in [0, 2^32)).
struct Partial_ {
    uint64_t count = 0, flags = 0, key = 0, isum = 0;
    int64_t limbs[dfmi::kAggLimbs] = {};
};

struct dfmi_aggregate {
    std::string name;  // as spelled in the SQL text (the Field name, sqlplanner.rs:385-389)
    int fn = 0;        // dfmi_agg_fn
    int ret_type = 0;
    dfmi_program arg;  // compile_expr's compiled argument (a copy: same uid, same kernels)
};

struct dfmi_agg_state {
    int device = 0;
    std::vector<const dfmi_aggregate*> aggs;
    uint64_t* acc = nullptr;  // [kAggCopies][n][kAggWords]; grouped: [kAggCopies][gslots][n + 1][kAggWords]
    size_t acc_words = 0;
    bool failed = false;      // a batch raised an error: the query has failed
    dfmi_error failure{};
    std::vector<uint64_t> init;  // the zero state (MIN keys all ones)
    // GROUP BY extension (dfmi_agg_state_create_grouped)
    bool grouped = false;
    dfmi_program key;           // the key (a copy: same uid, same kernels)
    int gslots = 0;             // slots per accumulator copy: the key window + the null slot
    uint64_t win_base = 0;      // the window the device accumulators hold ...
    int win_width = -1;         // ... (-1: none yet)
    bool dirty = false;         // the device accumulators hold rows
    struct HKey {
        bool null;
        __int128 ord;
        std::string s;  // Utf8 keys: the bytes (ordered bytewise)
        bool operator<(const HKey& o) const {
            if (null != o.null) return !null;
            if (null) return false;
            return ord != o.ord ? ord < o.ord : s < o.s;
        }
    };
    std::map<HKey, std::pair<uint64_t, std::vector<Partial_>>> groups;  // key -> (bits, partials + row count)
    // the host merge's per-row lookup: a hash index over `groups` (views of
    // the map's own keys; map nodes do not move), cleared with it
    struct HKeyView {
        bool null;
        __int128 ord;
        std::string_view s;
        bool operator==(const HKeyView& o) const { return null == o.null && ord == o.ord && s == o.s; }
    };
    struct HKeyViewHash {
        size_t operator()(const HKeyView& k) const {
            const uint64_t lo = (uint64_t)k.ord, hi = (uint64_t)((unsigned __int128)k.ord >> 64);
            uint64_t h = (lo ^ (hi * 0x9E3779B97F4A7C15ull) ^ (uint64_t)k.null) * 0xBF58476D1CE4E5B9ull;
            if (!k.s.empty()) h ^= std::hash<std::string_view>{}(k.s) + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
            return (size_t)(h ^ (h >> 31));
        }
    };
    std::unordered_map<HKeyView, std::pair<uint64_t, std::vector<Partial_>>*, HKeyViewHash> index;
    // integer keys: the per-batch key window comes from MIN / MAX of the key
    // over the batch's selected rows (a pre-pass through this same extension)
    dfmi_aggregate* mm[2] = {nullptr, nullptr};
    dfmi_agg_state* mm_state = nullptr;
};

namespace {

int agg_fn_of(const std::string& name) {
    std::string l = name;
    for (auto& c : l) c = (char)tolower((unsigned char)c);
    if (l == "min") return DFMI_AGG_MIN;
    if (l == "max") return DFMI_AGG_MAX;
    if (l == "count") return DFMI_AGG_COUNT;
    if (l == "sum") return DFMI_AGG_SUM;
    return -1;
}

bool is_float_type(int t) { return t == DFMI_TYPE_FLOAT32 || t == DFMI_TYPE_FLOAT64; }

// GROUP BY keys merged on the host for every batch (no device key window):
// floating-point keys -- one group per bit pattern, ordered by IEEE 754
// totalOrder (Rust's f64::total_cmp: -NaN < -inf < ... < -0.0 < +0.0 < ... <
// +inf < +NaN) -- and Utf8 keys, ordered bytewise (shorter prefix first).
// Build-defined (the reference executes no Aggregate): parity unpinned.
bool host_keyed(int t) { return is_float_type(t) || t == DFMI_TYPE_UTF8; }

// Order value of a non-null Boolean / integer / float key from its bits
// (integers sign/zero-extended, Float32 bits in the low 32).
bool is_signed_type(int t);
__int128 key_ord(int t, uint64_t bits) {
    if (t == DFMI_TYPE_FLOAT64) return (__int128)((bits >> 63) ? ~bits : (bits | (1ull << 63)));
    if (t == DFMI_TYPE_FLOAT32) {
        const uint32_t b = (uint32_t)bits;
        return (__int128)((b >> 31) ? (uint32_t)~b : (b | 0x80000000u));
    }
    if (t == DFMI_TYPE_BOOLEAN) return (__int128)bits;
    return is_signed_type(t) ? (__int128)(int64_t)bits : (__int128)bits;
}

// ---- exact merge of accumulator copies (host)
using Partial = Partial_;

void merge_into(Partial& p, const uint64_t* w, bool is_min) {
    p.count += w[0];
    if ((w[1] & AGGF_VALUE)) {
        if (!(p.flags & AGGF_VALUE)) p.key = w[2];
        else p.key = is_min ? std::min(p.key, w[2]) : std::max(p.key, w[2]);
    }
    p.flags |= w[1];
    p.isum += w[3];
    for (int i = 0; i < kAggLimbs; ++i) p.limbs[i] += (int64_t)w[4 + i];
}

void normalize(Partial& p) {
    for (int i = 0; i < kAggLimbs - 1; ++i) {
        const int64_t c = p.limbs[i] >> 32;  // floor division by 2^32
        p.limbs[i] -= c * 4294967296ll;
        p.limbs[i + 1] += c;
    }
}

// The exact sum (normalised digits, units of 2^-1074) rounded half-to-even
// to a format of `prec` significand bits whose quantum is at least
// 2^(qmin-1074); `zero` when the exact sum is 0. Result as a double (exact
// for Float32 results).
double round_exact(const Partial& p, int prec, int qmin, double overflow_limit, bool* zero) {
    // magnitude digits (two's complement negation of the digit string)
    int64_t d[kAggLimbs];
    const bool neg = p.limbs[kAggLimbs - 1] < 0;
    if (!neg) {
        memcpy(d, p.limbs, sizeof d);
    } else {
        int64_t borrow = 0;
        for (int i = 0; i < kAggLimbs; ++i) {
            int64_t v = -p.limbs[i] - borrow;
            borrow = 0;
            if (i < kAggLimbs - 1 && v < 0) {
                v += 4294967296ll;
                borrow = 1;
            }
            d[i] = v;
        }
    }
    int top = -1;
    for (int i = kAggLimbs - 1; i >= 0; --i)
        if (d[i]) {
            top = i;
            break;
        }
    *zero = top < 0;
    if (top < 0) return 0.0;
    auto bit = [&](int i) -> uint64_t { return i < 0 ? 0 : ((uint64_t)d[i >> 5] >> (i & 31)) & 1; };
    int msb = 32 * top;  // highest set bit (digits < 2^32 after normalisation)
    for (int b = 31; b >= 0; --b)
        if (((uint64_t)d[top] >> b) & 1) {
            msb = 32 * top + b;
            break;
        }
    int q = std::max(msb - (prec - 1), qmin);
    uint64_t mant = 0;
    for (int i = msb; i >= q; --i) mant = (mant << 1) | bit(i);
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
    double v = std::ldexp((double)mant, q - 1074);
    if (v >= overflow_limit) v = HUGE_VAL;
    return neg ? -v : v;
}

uint64_t key_to_bits(uint64_t key, int t) {
    switch (t) {
        case DFMI_TYPE_FLOAT64: return (key >> 63) ? (key & ~(1ull << 63)) : ~key;
        case DFMI_TYPE_FLOAT32: {
            const uint32_t k = (uint32_t)key;
            return (k >> 31) ? (uint64_t)(k & 0x7fffffffu) : (uint64_t)(uint32_t)~k;
        }
        case DFMI_TYPE_INT8: case DFMI_TYPE_INT16: case DFMI_TYPE_INT32: case DFMI_TYPE_INT64:
            return key ^ (1ull << 63);  // the value sign-extended to 64 bits
        default: return key;
    }
}

uint64_t narrow_int(uint64_t v, int t) {
    switch (t) {
        case DFMI_TYPE_INT8: return (uint64_t)(int64_t)(int8_t)v;
        case DFMI_TYPE_INT16: return (uint64_t)(int64_t)(int16_t)v;
        case DFMI_TYPE_INT32: return (uint64_t)(int64_t)(int32_t)v;
        case DFMI_TYPE_UINT8: return v & 0xffull;
        case DFMI_TYPE_UINT16: return v & 0xffffull;
        case DFMI_TYPE_UINT32: return v & 0xffffffffull;
        default: return v;
    }
}

dfmi_agg_value finish_one(const dfmi_aggregate& a, Partial p) {
    normalize(p);
    dfmi_agg_value r;
    r.type = a.ret_type;
    r.count = (int64_t)p.count;
    r.is_null = 0;
    r.bits = 0;
    const int t = a.arg.type;
    if (a.fn == DFMI_AGG_COUNT) {
        r.bits = p.count;
        return r;
    }
    if (p.count == 0) {
        r.is_null = 1;
        return r;
    }
    const bool f32 = t == DFMI_TYPE_FLOAT32;
    const uint64_t qnan = f32 ? 0x7FC00000ull : 0x7FF8000000000000ull;
    if (a.fn == DFMI_AGG_SUM) {
        if (!is_float_type(t)) {
            r.bits = narrow_int(p.isum, t);
        } else if ((p.flags & AGGF_NAN) || ((p.flags & AGGF_PINF) && (p.flags & AGGF_NINF))) {
            r.bits = qnan;
        } else if (p.flags & (AGGF_PINF | AGGF_NINF)) {
            const bool pos = p.flags & AGGF_PINF;
            r.bits = f32 ? (pos ? 0x7F800000ull : 0xFF800000ull) : (pos ? 0x7FF0000000000000ull : 0xFFF0000000000000ull);
        } else {
            bool zero = false;
            double v = f32 ? round_exact(p, 24, 925, 0x1p128, &zero) : round_exact(p, 53, 0, HUGE_VAL, &zero);
            if (zero) v = (p.flags & AGGF_NONNEGZERO) ? 0.0 : -0.0;
            if (f32) {
                const float fv = (float)v;
                uint32_t b;
                memcpy(&b, &fv, 4);
                r.bits = b;
            } else {
                memcpy(&r.bits, &v, 8);
            }
        }
        return r;
    }
    // MIN / MAX
    r.bits = (p.flags & AGGF_VALUE) ? key_to_bits(p.key, t) : qnan;
    return r;
}

// Static errors, slots and tile shape of one aggregate batch (the filtered
// form of exec.cpp's build_plan: FilterRelation::next, then each argument
// over the filtered batch in aggregate order).
struct AggBuilt {
    Err se;
    jit::Plan plan;
    jit::Launch X;
    int64_t n_tiles = 0;
};

void build_agg_plan(const dfmi_agg_state* st, const dfmi_program* pred, const dfmi_batch* in, uint32_t flags,
                    AggBuilt& B, bool low_sel = false) {
    Err& se = B.se;
    jit::Launch& X = B.X;
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
    if (st->grouped) check_schema(&st->key);
    for (const dfmi_aggregate* a : st->aggs) check_schema(&a->arg);
    for (int i = 0; i < ncols; ++i)
        if (in->columns[i].length != n) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "ragged batch"};
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
    int base = P + 2, nf = 0;
    if (st->grouped) {  // the group key is evaluated before the aggregates
        for (const IrNode& nd : st->key.ir)
            if (nd.rt_code) se.offer((uint64_t)(base + nd.ordinal) << 44, nd.rt_code, nd.rt_msg);
        B.plan.gkey = &st->key;
        B.plan.gkey_ord = base;
        B.plan.gslots = st->gslots;
        base += st->key.length;
    }
    for (const dfmi_aggregate* a : st->aggs) {
        for (const IrNode& nd : a->arg.ir)
            if (nd.rt_code) se.offer((uint64_t)(base + nd.ordinal) << 44, nd.rt_code, nd.rt_msg);
        jit::AggSpec s;
        s.fn = a->fn;
        s.prog = &a->arg;
        s.ord_base = base;
        s.arg_type = a->arg.type;
        if (a->fn == DFMI_AGG_SUM && is_float_type(a->arg.type)) s.fslot = nf++;
        B.plan.aggs.push_back(s);
        base += a->arg.length;
    }
    if (base >= (1 << 19)) throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "device program limit: expressions too long"};
    if (nf > 4) throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "device program limit: more than 4 floating-point SUMs"};
    B.plan.pred = pred;
    X.in = in;
    auto reg_num = [&](int col, std::vector<int>& phase) {
        for (size_t i = 0; i < X.num_cols.size(); ++i)
            if (X.num_cols[i] == col) return;
        X.num_cols.push_back(col);
        phase.push_back((int)X.num_cols.size() - 1);
    };
    auto reg_prog = [&](const dfmi_program* p, std::vector<int>& phase) {
        for (const IrNode& nd : p->ir) {
            if (nd.kind != IR_COL) continue;
            if (nd.type == DFMI_TYPE_UTF8) {
                bool have = false;
                for (int c : X.utf8_cols) have |= c == nd.col;
                if (!have) X.utf8_cols.push_back(nd.col);
            } else if (jit::type_width(nd.type) || nd.type == DFMI_TYPE_BOOLEAN) {
                reg_num(nd.col, phase);
            }
        }
    };
    if (pred) reg_prog(pred, X.pred_slots);
    if (st->grouped) reg_prog(&st->key, X.proj_slots);
    for (const dfmi_aggregate* a : st->aggs) reg_prog(&a->arg, X.proj_slots);
    if ((int)X.num_cols.size() > kArgCols || X.utf8_cols.size() > (size_t)kArgUtf8)
        throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "device program limit: too many input columns"};
    const size_t nload = X.num_cols.size();
    X.BLOCK = 512;
    X.K = nload <= 4 ? 8 : (nload <= 8 ? 4 : 2);
    if (getenv("DFMI_DIAG")) {  // diagnostics only
        if (const char* kk = getenv("DFMI_ROWS_PER_THREAD")) X.K = atoi(kk);
        if (const char* e = getenv("DFMI_PROJ_DENSE")) X.proj_dense = atoi(e) & 1;
    }
    // a predicate that selected < 4% of the rows the last time this state
    // ran the query (dfmi_aggregate_batch keeps the kernel's count): M
    // sub-tiles per block, the arguments loaded by one lane per selected row
    // (jit.cpp generate_agg; numeric, non-Boolean arguments)
    bool can_sub = pred && !st->grouped && X.utf8_cols.empty();
    for (int s : X.proj_slots) can_sub = can_sub && X.col_type(X.num_cols[s]) != DFMI_TYPE_BOOLEAN;
    for (int s : X.pred_slots) can_sub = can_sub && X.col_type(X.num_cols[s]) != DFMI_TYPE_BOOLEAN;
    // (Q6, same-box A/B profiles/r04/q6_ab.log: M = 1 / 2 / 4 -> 2.88 / 2.57 / 2.54 ms)
    if (can_sub && low_sel && in->num_rows >= (1 << 22)) X.M = 4;
    if (getenv("DFMI_DIAG"))  // diagnostics: force M
        if (const char* e = getenv("DFMI_AGG_SUBTILES")) X.M = can_sub ? std::max(1, std::min(16, atoi(e))) : 1;
    if (X.K < 1 || X.K > 32) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "bad tile shape"};
    const int64_t tile_rows = (int64_t)X.BLOCK * X.K * X.M;
    B.n_tiles = (n + tile_rows - 1) / tile_rows;
    if (B.n_tiles > 0x7fffffff) throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "batch too large"};
}

std::vector<Partial> merge_copies(const dfmi_agg_state* st, const std::vector<uint64_t>& h) {
    const size_t n = st->aggs.size();
    std::vector<Partial> parts(n);
    for (size_t j = 0; j < n; ++j) {
        const bool is_min = st->aggs[j]->fn == DFMI_AGG_MIN;
        for (int c = 0; c < kAggCopies; ++c) merge_into(parts[j], &h[((size_t)c * n + j) * kAggWords], is_min);
        normalize(parts[j]);
    }
    return parts;
}

std::vector<uint64_t> read_acc(dfmi_context* ctx, dfmi_agg_state* st) {
    std::vector<uint64_t> h(st->acc_words);
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipMemcpyAsync(h.data(), st->acc, h.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return h;
}

void merge_partial(Partial& into, const Partial& p, bool is_min) {
    uint64_t w[kAggWords];
    w[0] = p.count;
    w[1] = p.flags;
    w[2] = p.key;
    w[3] = p.isum;
    for (int i = 0; i < kAggLimbs; ++i) w[4 + i] = (uint64_t)p.limbs[i];
    merge_into(into, w, is_min);
}

bool is_signed_type(int t) {
    return t == DFMI_TYPE_INT8 || t == DFMI_TYPE_INT16 || t == DFMI_TYPE_INT32 || t == DFMI_TYPE_INT64;
}

// GROUP BY: the device accumulators (window win_base / win_width) merged into
// the host's groups, and the device state reset.
void flush_groups(dfmi_context* ctx, dfmi_agg_state* st) {
    if (!st->dirty) return;
    const std::vector<uint64_t> h = read_acc(ctx, st);
    const size_t n = st->aggs.size(), na = n + 1;
    const int kt = st->key.type;
    for (int g = 0; g <= st->win_width; ++g) {
        std::vector<Partial> parts(na);
        for (size_t j = 0; j < na; ++j) {
            const bool is_min = j < n && st->aggs[j]->fn == DFMI_AGG_MIN;
            for (int c = 0; c < kAggCopies; ++c)
                merge_into(parts[j], &h[(((size_t)c * st->gslots + g) * na + j) * kAggWords], is_min);
            normalize(parts[j]);
        }
        if (parts[n].count == 0) continue;  // no row of this key in the window
        dfmi_agg_state::HKey hk{g == st->win_width, 0, {}};
        uint64_t bits = 0;
        if (!hk.null) {
            bits = st->win_base + (uint64_t)g;
            hk.ord = key_ord(kt, bits);
        }
        auto it = st->groups.find(hk);
        if (it == st->groups.end()) it = st->groups.emplace(hk, std::make_pair(bits, std::vector<Partial>(na))).first;
        for (size_t j = 0; j < n; ++j) merge_partial(it->second.second[j], parts[j], st->aggs[j]->fn == DFMI_AGG_MIN);
        it->second.second[n].count += parts[n].count;  // the hidden count: the group's selected rows
    }
    HIP_TRY(hipMemcpyAsync(st->acc, st->init.data(), st->acc_words * 8, hipMemcpyHostToDevice, ctx->stream));
    st->dirty = false;
}

// ---- GROUP BY over keys wider than the device window: the host merge.
// One value (row i, non-null) of aggregate `a` into p -- the per-row rules
// of the aggregate kernels (jit.cpp generate_agg / generate_agg_grouped,
// jit_skeleton.hip agg_key / agg_sum_flags / fsum_add), restated on the host.
template <typename T>
uint64_t host_agg_key(T v) {
    if constexpr (std::is_same<T, float>::value) {
        uint32_t b;
        memcpy(&b, &v, 4);
        return (b >> 31) ? (uint64_t)(~b) : (uint64_t)(b | 0x80000000u);
    } else if constexpr (std::is_same<T, double>::value) {
        uint64_t b;
        memcpy(&b, &v, 8);
        return (b >> 63) ? ~b : (b | (1ull << 63));
    } else if constexpr (std::is_signed<T>::value) {
        return (uint64_t)(int64_t)v ^ (1ull << 63);
    } else {
        return (uint64_t)v;
    }
}

void host_fsum_add(Partial& p, double v) {  // finite, non-zero v (fsum_add's digit split)
    uint64_t b;
    memcpy(&b, &v, 8);
    const int e = (int)((b >> 52) & 0x7ff);
    const uint64_t m = (b & ((1ull << 52) - 1)) | (e ? (1ull << 52) : 0ull);
    const int pos = (e ? e : 1) - 1;
    const int d = pos >> 5, sh = pos & 31;
    const uint64_t x0 = (m & 0xffffffffull) << sh, x1 = (m >> 32) << sh;
    int64_t c0 = (int64_t)(x0 & 0xffffffffull);
    int64_t c1 = (int64_t)((x0 >> 32) + (x1 & 0xffffffffull));
    int64_t c2 = (int64_t)(x1 >> 32);
    if (b >> 63) {
        c0 = -c0;
        c1 = -c1;
        c2 = -c2;
    }
    p.limbs[d] += c0;
    p.limbs[d + 1] += c1;
    p.limbs[d + 2] += c2;
}

template <typename T>
void host_accumulate_t(Partial& p, int fn, T v) {
    ++p.count;
    if (fn == DFMI_AGG_COUNT) return;
    if (fn == DFMI_AGG_SUM) {
        if constexpr (std::is_floating_point<T>::value) {
            const unsigned f = v != v ? AGGF_NAN
                                      : (std::isinf(v) ? (v > 0 ? AGGF_PINF : AGGF_NINF)
                                                       : ((v == 0 && std::signbit(v)) ? 0u : AGGF_NONNEGZERO));
            p.flags |= f;
            if (f == AGGF_NONNEGZERO && v != 0) host_fsum_add(p, (double)v);
        } else {
            p.isum += std::is_signed<T>::value ? (uint64_t)(int64_t)v : (uint64_t)v;
        }
        return;
    }
    // MIN / MAX
    if constexpr (std::is_floating_point<T>::value)
        if (v != v) {
            p.flags |= AGGF_NAN;
            return;
        }
    const uint64_t k = host_agg_key(v);
    if (!(p.flags & AGGF_VALUE)) p.key = k;
    else p.key = fn == DFMI_AGG_MIN ? std::min(p.key, k) : std::max(p.key, k);
    p.flags |= AGGF_VALUE;
}

void host_accumulate(Partial& p, int fn, int t, const uint8_t* vals, int64_t i) {
    switch (t) {
        case DFMI_TYPE_INT8: return host_accumulate_t(p, fn, ((const int8_t*)vals)[i]);
        case DFMI_TYPE_INT16: return host_accumulate_t(p, fn, ((const int16_t*)vals)[i]);
        case DFMI_TYPE_INT32: return host_accumulate_t(p, fn, ((const int32_t*)vals)[i]);
        case DFMI_TYPE_INT64: return host_accumulate_t(p, fn, ((const int64_t*)vals)[i]);
        case DFMI_TYPE_UINT8: return host_accumulate_t(p, fn, ((const uint8_t*)vals)[i]);
        case DFMI_TYPE_UINT16: return host_accumulate_t(p, fn, ((const uint16_t*)vals)[i]);
        case DFMI_TYPE_UINT32: return host_accumulate_t(p, fn, ((const uint32_t*)vals)[i]);
        case DFMI_TYPE_UINT64: return host_accumulate_t(p, fn, ((const uint64_t*)vals)[i]);
        case DFMI_TYPE_FLOAT32: return host_accumulate_t(p, fn, ((const float*)vals)[i]);
        case DFMI_TYPE_FLOAT64: return host_accumulate_t(p, fn, ((const double*)vals)[i]);
        default: ++p.count;  // COUNT of a Boolean / Utf8 argument: non-null values only
    }
}

// A batch whose selected keys span more than the device window: the key and
// every argument evaluated on the device as one fused Selection + Projection
// pass (dfmi_filter_project: projections [key, args...] -- the same
// evaluation order, ordinals and errors as the grouped kernel), the
// compacted columns copied back, and each row merged into its group on the
// host with the kernels' per-row rules.
void group_batch_on_host(dfmi_context* ctx, dfmi_agg_state* st, const dfmi_program* pred, const dfmi_batch* in,
                         uint32_t flags) {
    const size_t n = st->aggs.size();
    const int no = (int)n + 1;
    const int64_t rows = in->num_rows;
    std::vector<const dfmi_program*> progs(no);
    progs[0] = &st->key;
    for (size_t j = 0; j < n; ++j) progs[j + 1] = &st->aggs[j]->arg;
    std::vector<dfmi_out_column> outs(no);
    std::vector<void*> dev;
    struct Free {
        std::vector<void*>& v;
        ~Free() {
            for (void* p : v) (void)hipFree(p);
        }
    } free_{dev};
    auto dalloc = [&](size_t b) {
        void* p = nullptr;
        HIP_TRY(hipMalloc(&p, std::max<size_t>(b, 64)));
        dev.push_back(p);
        return p;
    };
    for (int o = 0; o < no; ++o) {
        dfmi_out_column& c = outs[o];
        memset(&c, 0, sizeof c);
        const int t = progs[o]->type;
        if (t == DFMI_TYPE_UTF8) {
            const IrNode& root = progs[o]->ir[progs[o]->root];
            size_t cap = 8;
            if (root.kind == IR_COL && root.col >= 0 && root.col < in->num_columns && in->columns[root.col].offsets) {
                int32_t last = 0;
                HIP_TRY(hipMemcpy(&last, in->columns[root.col].offsets + rows, 4, hipMemcpyDeviceToHost));
                cap = std::max<size_t>(cap, (size_t)std::max(0, last));
            }
            c.offsets = (int32_t*)dalloc((size_t)(rows + 1) * 4);
            c.data = (uint8_t*)dalloc(cap);
            c.data_capacity = (int64_t)cap;
        } else {
            const int w = jit::type_width(t);
            c.values = dalloc(t == DFMI_TYPE_BOOLEAN ? (size_t)(rows + 63) / 64 * 8 : (size_t)rows * std::max(w, 1));
        }
        c.validity = (uint8_t*)dalloc((size_t)(rows + 63) / 64 * 8);
    }
    dfmi_error e{};
    if (dfmi_filter_project(ctx, pred, progs.data(), no, in, outs.data(), flags, &e) != DFMI_OK) {
        st->failed = true;
        st->failure = e;
        throw Fail{e.code, e.message};
    }
    // a passthrough-only pass launches nothing, and a sliced batch's shifted
    // bitmaps (slice.cpp) are written on ctx->stream: order the synchronous
    // null-stream copies below after them
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    const int64_t m = outs[0].length;  // selected rows
    // host copies of values (fixed width) and validity
    std::vector<std::vector<uint8_t>> hv(no), hb(no);
    for (int o = 0; o < no; ++o) {
        const dfmi_out_column& c = outs[o];
        const int t = progs[o]->type;
        const dfmi_column* src = c.passthrough_column >= 0 ? &in->columns[c.passthrough_column] : nullptr;
        const int w = jit::type_width(t);
        const size_t vb = t == DFMI_TYPE_BOOLEAN ? (size_t)(m + 7) / 8 : (size_t)m * w;
        if (vb && t != DFMI_TYPE_UTF8) {
            hv[o].resize(vb);
            HIP_TRY(hipMemcpy(hv[o].data(), src ? src->values : c.values, vb, hipMemcpyDeviceToHost));
        }
        const uint8_t* vsrc = src ? (src->null_count > 0 ? src->validity : nullptr) : (c.null_count > 0 ? c.validity : nullptr);
        if (vsrc && m) {
            hb[o].resize((size_t)(m + 7) / 8);
            HIP_TRY(hipMemcpy(hb[o].data(), vsrc, hb[o].size(), hipMemcpyDeviceToHost));
        }
    }
    auto valid = [&](int o, int64_t i) { return hb[o].empty() || ((hb[o][i >> 3] >> (i & 7)) & 1); };
    const int kt = st->key.type;
    // a Utf8 key: its offsets and bytes (the compacted output, or -- no
    // predicate, a Column key -- the input column itself)
    std::vector<int32_t> koff;
    std::vector<uint8_t> kbytes;
    if (kt == DFMI_TYPE_UTF8 && m > 0) {
        const dfmi_out_column& c = outs[0];
        const dfmi_column* src = c.passthrough_column >= 0 ? &in->columns[c.passthrough_column] : nullptr;
        koff.resize((size_t)m + 1);
        HIP_TRY(hipMemcpy(koff.data(), src ? src->offsets : c.offsets, koff.size() * 4, hipMemcpyDeviceToHost));
        const size_t nbytes = (size_t)std::max(0, koff[m] - koff[0]);
        kbytes.resize(std::max<size_t>(nbytes, 1));
        if (nbytes)
            HIP_TRY(hipMemcpy(kbytes.data(), (src ? (const uint8_t*)src->values : c.data) + koff[0], nbytes,
                              hipMemcpyDeviceToHost));
    }
    for (int64_t i = 0; i < m; ++i) {
        dfmi_agg_state::HKeyView kv{!valid(0, i), 0, {}};
        uint64_t bits = 0;
        if (!kv.null) {
            if (kt == DFMI_TYPE_UTF8) {
                kv.s = std::string_view((const char*)kbytes.data() + (koff[i] - koff[0]), (size_t)(koff[i + 1] - koff[i]));
            } else if (kt == DFMI_TYPE_BOOLEAN) {
                bits = (hv[0][i >> 3] >> (i & 7)) & 1;
                kv.ord = (__int128)bits;
            } else {
                const int w = jit::type_width(kt);
                uint64_t raw = 0;
                memcpy(&raw, hv[0].data() + (size_t)i * w, w);
                bits = is_signed_type(kt) ? (uint64_t)(int64_t)narrow_int(raw, kt) : narrow_int(raw, kt);
                kv.ord = key_ord(kt, bits);
            }
        }
        std::pair<uint64_t, std::vector<Partial>>* entry;
        auto ix = st->index.find(kv);
        if (ix != st->index.end()) {
            entry = ix->second;
        } else {  // first row of this key in this state (or since a reset): the ordered map, then the index
            dfmi_agg_state::HKey hk{kv.null, kv.ord, std::string(kv.s)};
            auto it = st->groups.find(hk);
            if (it == st->groups.end())
                it = st->groups.emplace(std::move(hk), std::make_pair(bits, std::vector<Partial>(n + 1))).first;
            entry = &it->second;
            st->index.emplace(dfmi_agg_state::HKeyView{it->first.null, it->first.ord, it->first.s}, entry);
        }
        std::vector<Partial>& g = entry->second;
        ++g[n].count;  // the group's selected rows
        for (size_t j = 0; j < n; ++j)
            if (valid((int)j + 1, i)) host_accumulate(g[j], st->aggs[j]->fn, progs[j + 1]->type, hv[j + 1].data(), i);
    }
    for (auto& kv : st->groups)
        for (Partial& p : kv.second.second) normalize(p);
}

using GroupMap = std::map<dfmi_agg_state::HKey, std::pair<uint64_t, std::vector<Partial>>>;

// Groups in key order as dfmi_agg_state_finish_grouped outputs them.
void emit_groups(const GroupMap& groups, int kt, const dfmi_aggregate* const* aggs, size_t n, int64_t cap,
                 dfmi_agg_value* keys, dfmi_agg_value* values, int64_t* num_groups) {
    *num_groups = (int64_t)groups.size();
    if (*num_groups > cap) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "group capacity too small"};
    if (*num_groups > 0 && (!keys || !values)) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
    int64_t g = 0;
    for (const auto& [hk, v] : groups) {
        keys[g].type = kt;
        keys[g].is_null = hk.null ? 1 : 0;
        keys[g].bits = hk.null ? 0 : (kt == DFMI_TYPE_BOOLEAN ? v.first : narrow_int(v.first, kt));
        keys[g].count = (int64_t)v.second[n].count;  // the group's selected rows
        for (size_t j = 0; j < n; ++j) values[g * n + j] = finish_one(*aggs[j], v.second[j]);
        ++g;
    }
}

// Serialised per-group partials (multi-GPU GROUP BY): a header, then per group
// {null, key bits} and its n + 1 partials (aggregates, then the row count).
struct GroupedHdr {
    uint64_t magic, ngroups, naggs;
    int64_t key_type;
};
constexpr uint64_t kGroupedMagic = 0x31505247494d4644ull;  // "DFMIGRP1"
size_t grouped_bytes(size_t ngroups, size_t n) { return sizeof(GroupedHdr) + ngroups * (16 + (n + 1) * sizeof(Partial)); }

}  // namespace

extern "C" int32_t dfmi_compile_aggregate(const char* name, const dfmi_program* arg, int32_t return_type,
                                          uint32_t flags, dfmi_aggregate** out, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    try {
        if (!name || !arg || !out) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        // ExecutionContext::execute has no Aggregate arm (context.rs:161)
        if (!(flags & DFMI_FLAG_EXT_AGGREGATE)) throw Fail{DFMI_ERR_PANIC, "not yet implemented"};
        const int fn = agg_fn_of(name);  // compile_expr's match (expression.rs:100-106)
        if (fn < 0) throw Fail{DFMI_ERR_PANIC, std::string("not yet implemented: Unsupported aggregate function '") + name + "'"};
        const int want = fn == DFMI_AGG_COUNT ? DFMI_TYPE_UINT64 : arg->type;  // sqlplanner.rs:296-330
        if (return_type != want) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "aggregate return type does not match the planner's"};
        if (fn != DFMI_AGG_COUNT && !is_numeric_type(arg->type))
            throw Fail{DFMI_ERR_NOT_IMPLEMENTED, std::string("aggregate over ") + type_debug(arg->type)};
        dfmi_aggregate* a = new (std::nothrow) dfmi_aggregate();
        if (!a) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "out of memory"};
        a->name = name;
        a->fn = fn;
        a->ret_type = return_type;
        a->arg = *arg;
        *out = a;
        return DFMI_OK;
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

extern "C" const char* dfmi_aggregate_name(const dfmi_aggregate* a) { return a ? a->name.c_str() : ""; }
extern "C" int32_t dfmi_aggregate_type(const dfmi_aggregate* a) { return a ? a->ret_type : 0; }
extern "C" void dfmi_aggregate_free(dfmi_aggregate* a) { delete a; }

extern "C" int32_t dfmi_agg_state_create(dfmi_context* ctx, const dfmi_aggregate* const* aggs, int32_t n,
                                         dfmi_agg_state** out, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    dfmi_agg_state* st = nullptr;
    try {
        if (!ctx || !out || n <= 0 || !aggs) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "bad argument"};
        if (n > 16) throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "device program limit: more than 16 aggregates"};
        st = new dfmi_agg_state();
        st->device = ctx->device;
        for (int j = 0; j < n; ++j) {
            if (!aggs[j]) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL aggregate"};
            st->aggs.push_back(aggs[j]);
        }
        st->acc_words = (size_t)kAggCopies * n * kAggWords;
        std::vector<uint64_t> init(st->acc_words, 0);
        for (int c = 0; c < kAggCopies; ++c)
            for (int j = 0; j < n; ++j)
                if (aggs[j]->fn == DFMI_AGG_MIN) init[((size_t)c * n + j) * kAggWords + 2] = ~0ull;
        HIP_TRY(hipSetDevice(ctx->device));
        HIP_TRY(hipMalloc((void**)&st->acc, st->acc_words * 8));
        HIP_TRY(hipMemcpyAsync(st->acc, init.data(), st->acc_words * 8, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        st->init = std::move(init);
        *out = st;
        return DFMI_OK;
    } catch (const Fail& f) {
        if (st) {
            if (st->acc) (void)hipFree(st->acc);
            delete st;
        }
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

extern "C" int32_t dfmi_agg_state_create_grouped(dfmi_context* ctx, const dfmi_program* key,
                                                 const dfmi_aggregate* const* aggs, int32_t n, dfmi_agg_state** out,
                                                 dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    dfmi_agg_state* st = nullptr;
    try {
        if (!ctx || !out || !key || n <= 0 || !aggs) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "bad argument"};
        const int kt = key->type;
        if (kt != DFMI_TYPE_BOOLEAN && !is_numeric_type(kt) && kt != DFMI_TYPE_UTF8)
            throw Fail{DFMI_ERR_NOT_IMPLEMENTED, std::string("GROUP BY over ") + type_debug(kt)};
        if (n > 15) throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "device program limit: more than 15 grouped aggregates"};
        st = new dfmi_agg_state();
        st->device = ctx->device;
        st->grouped = true;
        st->key = *key;
        st->gslots = kt == DFMI_TYPE_BOOLEAN ? 3 : 17;  // false, true / 16 consecutive values; + null
        for (int j = 0; j < n; ++j) {
            if (!aggs[j]) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL aggregate"};
            st->aggs.push_back(aggs[j]);
        }
        const size_t na = (size_t)n + 1;
        st->acc_words = (size_t)kAggCopies * st->gslots * na * kAggWords;
        std::vector<uint64_t> init(st->acc_words, 0);
        for (size_t cg = 0; cg < (size_t)kAggCopies * st->gslots; ++cg)
            for (int j = 0; j < n; ++j)
                if (aggs[j]->fn == DFMI_AGG_MIN) init[(cg * na + j) * kAggWords + 2] = ~0ull;
        HIP_TRY(hipSetDevice(ctx->device));
        HIP_TRY(hipMalloc((void**)&st->acc, st->acc_words * 8));
        HIP_TRY(hipMemcpyAsync(st->acc, init.data(), st->acc_words * 8, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        st->init = std::move(init);
        if (kt != DFMI_TYPE_BOOLEAN && !host_keyed(kt)) {
            dfmi_error e2{};
            for (int i = 0; i < 2; ++i)
                if (dfmi_compile_aggregate(i ? "MAX" : "MIN", key, kt, DFMI_FLAG_EXT_AGGREGATE, &st->mm[i], &e2) != DFMI_OK)
                    throw Fail{e2.code, e2.message};
            const dfmi_aggregate* mm[2] = {st->mm[0], st->mm[1]};
            if (dfmi_agg_state_create(ctx, mm, 2, &st->mm_state, &e2) != DFMI_OK) throw Fail{e2.code, e2.message};
        }
        *out = st;
        return DFMI_OK;
    } catch (const Fail& f) {
        dfmi_agg_state_free(st);
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

extern "C" int32_t dfmi_agg_state_finish_grouped(dfmi_context* ctx, dfmi_agg_state* st, int64_t cap,
                                                 dfmi_agg_value* keys, dfmi_agg_value* values, int64_t* num_groups,
                                                 dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    try {
        if (!ctx || !st || !num_groups) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        if (!st->grouped) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "not a GROUP BY state"};
        if (st->failed) {
            if (err) *err = st->failure;
            return st->failure.code;
        }
        HIP_TRY(hipSetDevice(ctx->device));
        flush_groups(ctx, st);
        emit_groups(st->groups, st->key.type, st->aggs.data(), st->aggs.size(), cap, keys, values, num_groups);
        return DFMI_OK;
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

extern "C" int32_t dfmi_agg_state_group_keys_utf8(const dfmi_agg_state* st, int32_t* offsets, int64_t num_offsets,
                                                  uint8_t* data, int64_t data_capacity, int64_t* data_length,
                                                  dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    try {
        if (!st || !data_length) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        if (!st->grouped || st->key.type != DFMI_TYPE_UTF8)
            throw Fail{DFMI_ERR_INVALID_ARGUMENT, "not a GROUP BY state over a Utf8 key"};
        int64_t total = 0;
        for (const auto& kv : st->groups) total += (int64_t)kv.first.s.size();
        *data_length = total;
        if (num_offsets < (int64_t)st->groups.size() + 1 || data_capacity < total)
            throw Fail{DFMI_ERR_CAPACITY, "key offsets / bytes capacity too small"};
        if (!offsets || (total && !data)) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        int64_t g = 0, pos = 0;
        offsets[0] = 0;
        for (const auto& kv : st->groups) {
            if (!kv.first.s.empty()) memcpy(data + pos, kv.first.s.data(), kv.first.s.size());
            pos += (int64_t)kv.first.s.size();
            offsets[++g] = (int32_t)pos;
        }
        return DFMI_OK;
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

extern "C" int32_t dfmi_agg_state_reset(dfmi_context* ctx, dfmi_agg_state* st, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    try {
        if (!ctx || !st) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        HIP_TRY(hipSetDevice(ctx->device));
        HIP_TRY(hipMemcpyAsync(st->acc, st->init.data(), st->acc_words * 8, hipMemcpyHostToDevice, ctx->stream));
        st->failed = false;
        st->failure = dfmi_error{};
        st->index.clear();
        st->groups.clear();
        st->win_width = -1;
        st->dirty = false;
        if (st->mm_state) {
            dfmi_error e2{};
            if (dfmi_agg_state_reset(ctx, st->mm_state, &e2) != DFMI_OK) throw Fail{e2.code, e2.message};
        }
        return DFMI_OK;
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

extern "C" void dfmi_agg_state_free(dfmi_agg_state* st) {
    if (!st) return;
    dfmi_agg_state_free(st->mm_state);
    dfmi_aggregate_free(st->mm[0]);
    dfmi_aggregate_free(st->mm[1]);
    if (st->acc) {
        (void)hipSetDevice(st->device);
        (void)hipFree(st->acc);
    }
    delete st;
}

extern "C" int32_t dfmi_aggregate_batch(dfmi_context* ctx, dfmi_agg_state* st, const dfmi_program* pred,
                                        const dfmi_batch* in, uint32_t flags, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    try {
        if (!ctx || !st || !in || (in->num_columns > 0 && !in->columns))
            throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        if (st->failed) {
            if (err) *err = st->failure;
            return st->failure.code;
        }
        Unsliced us_;  // sliced arrays (arrow offsets): offset-0 views / shifted bitmaps (slice.cpp)
        if (any_offset(in, 1)) {
            HIP_TRY(hipSetDevice(ctx->device));
            in = unslice(in, 1, us_, true, ctx->stream);
        }
        if (st->grouped && host_keyed(st->key.type)) {
            // float / Utf8 keys: the key and the arguments through one fused
            // Selection + Projection pass, each row merged on the host
            HIP_TRY(hipSetDevice(ctx->device));
            if (in->num_rows > 0) group_batch_on_host(ctx, st, pred, in, flags);
            return DFMI_OK;
        }
        // the query's selectivity last time (this state, this predicate)
        const uint64_t hint_key = (uint64_t)(uintptr_t)st * 1099511628211ull ^ (uint64_t)(uintptr_t)pred;
        const auto hint = ctx->sel_hint.find(hint_key);
        const bool low_sel = hint != ctx->sel_hint.end() && hint->second < 0.04;
        AggBuilt B;
        try {
            build_agg_plan(st, pred, in, flags, B, low_sel);
        } catch (const Fail& f) {
            if (f.code == DFMI_ERR_NOT_IMPLEMENTED && B.se.set) throw Fail{B.se.code, B.se.msg};
            throw;
        }
        Err& se = B.se;
        const int64_t n = in->num_rows;
        HIP_TRY(hipSetDevice(ctx->device));
        hipStream_t stream = ctx->stream;
        if (st->grouped && n > 0) {
            // the batch's key window: Boolean keys always [false, true];
            // integer keys 16 values from the batch's smallest selected key
            uint64_t wbase = 0;
            int wwidth = 2;
            if (st->key.type != DFMI_TYPE_BOOLEAN) {
                wwidth = st->gslots - 1;
                dfmi_error e2{};
                dfmi_agg_value mm[2];
                if (dfmi_aggregate_batch(ctx, st->mm_state, pred, in, flags, &e2) != DFMI_OK ||
                    dfmi_agg_state_finish(ctx, st->mm_state, mm, &e2) != DFMI_OK ||
                    dfmi_agg_state_reset(ctx, st->mm_state, &e2) != DFMI_OK) {
                    // the predicate or the key failed: evaluated before any aggregate
                    st->failed = true;
                    st->failure = e2;
                    throw Fail{e2.code, e2.message};
                }
                const bool cover = st->win_width == wwidth && (mm[0].count == 0 || ((mm[0].bits - st->win_base) < (uint64_t)wwidth &&
                                                                                   (mm[1].bits - st->win_base) < (uint64_t)wwidth));
                if (cover) {
                    wbase = st->win_base;
                } else {
                    wbase = mm[0].count ? mm[0].bits : 0;
                    if (mm[0].count && mm[1].bits - mm[0].bits >= (uint64_t)wwidth) {
                        // wider than the device window: the host merge (its
                        // fused pass raises the same first error in the same
                        // evaluation order as the grouped kernel would)
                        flush_groups(ctx, st);
                        group_batch_on_host(ctx, st, pred, in, flags);
                        return DFMI_OK;
                    }
                }
            }
            if (st->win_width != wwidth || st->win_base != wbase) {
                flush_groups(ctx, st);
                st->win_base = wbase;
                st->win_width = wwidth;
            }
        }
        ctx->timed = false;
        ctx->last_compile_ms = 0;
        uint64_t dev_key = ~0ull;
        int dev_kind = 0;
        if (n > 0) {
            hipFunction_t fn;
            try {
                fn = jit::get_kernel(ctx->device, B.plan, B.X, &ctx->last_compile_ms);
                ctx->last_kernel = B.X.kname;
            } catch (const Fail& f) {
                if (se.set) throw Fail{se.code, se.msg};
                throw;
            }
            jit::Launch& X = B.X;
            Args A;
            memset(&A, 0, sizeof A);
            A.n_rows = n;
            A.n_tiles = (int)B.n_tiles;
            for (size_t s = 0; s < X.num_cols.size(); ++s) {
                const dfmi_column& c = in->columns[X.num_cols[s]];
                if (!c.values) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "column values pointer is NULL"};
                const int w = jit::type_width(c.type);
                if (w && ((uintptr_t)c.values & (w - 1)))
                    throw Fail{DFMI_ERR_INVALID_ARGUMENT, "column values must be aligned to their width"};
                A.col[s] = c.values;
                A.valid[s] = (c.validity && c.null_count > 0) ? c.validity : nullptr;
            }
            for (size_t u = 0; u < X.utf8_cols.size(); ++u) {
                const dfmi_column& c = in->columns[X.utf8_cols[u]];
                if (!c.values || !c.offsets) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "Utf8 column buffers are NULL"};
                A.offs[u] = c.offsets;
                A.bytes[u] = (const u8*)c.values;
                A.svalid[u] = (c.validity && c.null_count > 0) ? c.validity : nullptr;
            }
            memcpy(A.lits, X.args_lits, sizeof A.lits);
            memcpy(A.str_off, X.str_off, sizeof A.str_off);
            memcpy(A.str_len, X.str_len, sizeof A.str_len);
            memcpy(A.str, X.str, sizeof A.str);
            const WsLease ws = ws_acquire(ctx, 0, stream);
            A.err = (unsigned long long*)(ws.hdr + kHdrErr);
            A.totals = (unsigned long long*)(ws.hdr + kHdrTotals);
            A.ticket = (unsigned*)(ws.hdr + kHdrTicket);
            A.stats = (unsigned long long*)(ws.hdr + kHdrStats);
            A.clear_status = (unsigned long long*)ws.clear_status;
            A.clear_words = ws.clear_words;
            A.clear_hdr = (unsigned long long*)ws.clear_hdr;
            A.agg = (unsigned long long*)st->acc;
            A.gbase = st->win_base;
            A.gwidth = st->win_width;
            HIP_TRY(hipEventRecord(ctx->ev0, stream));
            size_t asz = sizeof A;
            void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &A, HIP_LAUNCH_PARAM_BUFFER_SIZE, &asz, HIP_LAUNCH_PARAM_END};
            HIP_TRY(hipModuleLaunchKernel(fn, (unsigned)B.n_tiles, 1, 1, X.BLOCK, 1, 1, 0, stream, nullptr, cfg));
            ws_commit(ctx, ws);
            HIP_TRY(hipEventRecord(ctx->ev1, stream));
            HIP_TRY(hipMemcpyAsync(ctx->host_hdr, ws.hdr, kHdrAlloc, hipMemcpyDeviceToHost, stream));
            HIP_TRY(hipEventRecord(ctx->ev2, stream));
            HIP_TRY(hipStreamSynchronize(stream));
            uint64_t ew;
            memcpy(&ew, ctx->host_hdr + kHdrErr, 8);
            if (pred && !st->grouped) {  // the kernel's count of selected rows in every 64th block
                uint64_t sel;
                memcpy(&sel, ctx->host_hdr + kHdrTotals, 8);
                const int64_t tile_rows = (int64_t)X.BLOCK * X.K * X.M;
                int64_t sampled = 0;
                for (int64_t b = 0; b < B.n_tiles; b += 64) sampled += std::min(tile_rows, n - b * tile_rows);
                ctx->sel_hint[hint_key] = sampled ? (double)sel / (double)sampled : 1.0;
            }
            if (ew) {
                dev_key = ~ew;
                dev_kind = (int)(dev_key & 15);
                dev_key &= ~15ull;
            }
            float m1 = 0, m2 = 0;
            (void)hipEventElapsedTime(&m1, ctx->ev0, ctx->ev1);
            (void)hipEventElapsedTime(&m2, ctx->ev0, ctx->ev2);
            ctx->last_main_ms = m1;
            ctx->last_total_ms = m2;
            ctx->timed = true;
        }
        if (st->grouped && n > 0) st->dirty = true;
        Fail fail{DFMI_OK, ""};
        if (dev_kind == ERRK_CAPACITY)  // a key outside the window the pre-pass found: cannot happen
            fail = Fail{DFMI_ERR_DEVICE, "GROUP BY key outside the batch's key window"};
        else if (dev_kind && (!se.set || dev_key < se.key))
            fail = dev_kind == ERRK_DIV_ZERO ? Fail{DFMI_ERR_DIVIDE_BY_ZERO, "DivideByZero"}
                                             : Fail{DFMI_ERR_PANIC, "attempt to divide with overflow"};
        else if (se.set)
            fail = Fail{se.code, se.msg};
        if (fail.code != DFMI_OK) {
            // the query has failed (the state holds partial sums of this batch)
            st->failed = true;
            set_err(&st->failure, fail.code, fail.msg);
            throw fail;
        }
        return DFMI_OK;
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

extern "C" int32_t dfmi_agg_state_finish(dfmi_context* ctx, dfmi_agg_state* st, dfmi_agg_value* out,
                                         dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    try {
        if (!ctx || !st || !out) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        if (st->failed) {
            if (err) *err = st->failure;
            return st->failure.code;
        }
        if (st->grouped) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "a GROUP BY state: dfmi_agg_state_finish_grouped"};
        const std::vector<Partial> parts = merge_copies(st, read_acc(ctx, st));
        for (size_t j = 0; j < st->aggs.size(); ++j) out[j] = finish_one(*st->aggs[j], parts[j]);
        return DFMI_OK;
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

extern "C" int64_t dfmi_agg_partial_bytes(const dfmi_agg_state* st) {
    return st ? (int64_t)(st->aggs.size() * sizeof(Partial)) : 0;
}

extern "C" int32_t dfmi_agg_state_partial(dfmi_context* ctx, dfmi_agg_state* st, void* host_out, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    try {
        if (!ctx || !st || !host_out) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        if (st->failed) {
            if (err) *err = st->failure;
            return st->failure.code;
        }
        if (st->grouped) throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "partial state of a GROUP BY aggregate"};
        const std::vector<Partial> parts = merge_copies(st, read_acc(ctx, st));
        memcpy(host_out, parts.data(), parts.size() * sizeof(Partial));
        return DFMI_OK;
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

extern "C" int64_t dfmi_agg_state_grouped_partial_bytes(dfmi_context* ctx, dfmi_agg_state* st, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    try {
        if (!ctx || !st) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        if (!st->grouped) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "not a GROUP BY state"};
        if (st->failed) {
            if (err) *err = st->failure;
            return -(int64_t)st->failure.code;
        }
        if (st->key.type == DFMI_TYPE_UTF8)
            throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "multi-GPU GROUP BY over Utf8"};
        HIP_TRY(hipSetDevice(ctx->device));
        flush_groups(ctx, st);
        return (int64_t)grouped_bytes(st->groups.size(), st->aggs.size());
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return -(int64_t)f.code;
    }
}

extern "C" int32_t dfmi_agg_state_grouped_partial(dfmi_context* ctx, dfmi_agg_state* st, void* host_out, int64_t bytes,
                                                  dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    try {
        if (!ctx || !st || !host_out) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        if (!st->grouped) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "not a GROUP BY state"};
        if (st->failed) {
            if (err) *err = st->failure;
            return st->failure.code;
        }
        if (st->key.type == DFMI_TYPE_UTF8)
            throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "multi-GPU GROUP BY over Utf8"};
        HIP_TRY(hipSetDevice(ctx->device));
        flush_groups(ctx, st);
        const size_t n = st->aggs.size();
        if ((size_t)bytes < grouped_bytes(st->groups.size(), n)) throw Fail{DFMI_ERR_CAPACITY, "partial buffer too small"};
        uint8_t* p = (uint8_t*)host_out;
        const GroupedHdr h{kGroupedMagic, (uint64_t)st->groups.size(), (uint64_t)n, (int64_t)st->key.type};
        memcpy(p, &h, sizeof h);
        p += sizeof h;
        for (const auto& [hk, v] : st->groups) {
            const uint64_t rec[2] = {hk.null ? 1ull : 0ull, v.first};
            memcpy(p, rec, 16);
            p += 16;
            memcpy(p, v.second.data(), (n + 1) * sizeof(Partial));
            p += (n + 1) * sizeof(Partial);
        }
        return DFMI_OK;
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

extern "C" int32_t dfmi_agg_merge_grouped_partials(const dfmi_aggregate* const* aggs, int32_t n,
                                                   const void* const* partials, const int64_t* sizes, int32_t nparts,
                                                   int64_t cap, dfmi_agg_value* keys, dfmi_agg_value* values,
                                                   int64_t* num_groups, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    try {
        if (!aggs || n <= 0 || !partials || !sizes || nparts <= 0 || !num_groups)
            throw Fail{DFMI_ERR_INVALID_ARGUMENT, "bad argument"};
        GroupMap groups;
        int64_t kt = -1;
        for (int r = 0; r < nparts; ++r) {
            const uint8_t* p = (const uint8_t*)partials[r];
            GroupedHdr h;
            if (!p || sizes[r] < (int64_t)sizeof h) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "bad grouped partial"};
            memcpy(&h, p, sizeof h);
            if (h.magic != kGroupedMagic || h.naggs != (uint64_t)n || (kt >= 0 && h.key_type != kt) ||
                (size_t)sizes[r] < grouped_bytes(h.ngroups, (size_t)n))
                throw Fail{DFMI_ERR_INVALID_ARGUMENT, "bad grouped partial"};
            kt = h.key_type;
            p += sizeof h;
            for (uint64_t g = 0; g < h.ngroups; ++g) {
                uint64_t rec[2];
                memcpy(rec, p, 16);
                p += 16;
                dfmi_agg_state::HKey hk{rec[0] != 0, 0, {}};
                if (!hk.null) hk.ord = key_ord((int)kt, rec[1]);
                auto it = groups.find(hk);
                if (it == groups.end()) it = groups.emplace(hk, std::make_pair(rec[1], std::vector<Partial>(n + 1))).first;
                for (int j = 0; j <= n; ++j) {
                    Partial q;
                    memcpy(&q, p + (size_t)j * sizeof(Partial), sizeof q);
                    if (j < n) merge_partial(it->second.second[j], q, aggs[j]->fn == DFMI_AGG_MIN);
                    else it->second.second[n].count += q.count;
                }
                p += (size_t)(n + 1) * sizeof(Partial);
            }
        }
        emit_groups(groups, (int)std::max<int64_t>(kt, 0), aggs, (size_t)n, cap, keys, values, num_groups);
        return DFMI_OK;
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

extern "C" int32_t dfmi_agg_merge_partials(const dfmi_aggregate* const* aggs, int32_t n, const void* const* partials,
                                           int32_t nparts, dfmi_agg_value* out, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    try {
        if (!aggs || n <= 0 || !partials || nparts <= 0 || !out) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "bad argument"};
        for (int j = 0; j < n; ++j) {
            Partial m;
            const bool is_min = aggs[j]->fn == DFMI_AGG_MIN;
            for (int r = 0; r < nparts; ++r) {
                Partial p;
                memcpy(&p, (const uint8_t*)partials[r] + (size_t)j * sizeof(Partial), sizeof p);
                uint64_t w[kAggWords];
                w[0] = p.count;
                w[1] = p.flags;
                w[2] = p.key;
                w[3] = p.isum;
                for (int i = 0; i < kAggLimbs; ++i) w[4 + i] = (uint64_t)p.limbs[i];
                merge_into(m, w, is_min);
            }
            out[j] = finish_one(*aggs[j], m);
        }
        return DFMI_OK;
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

// Internal test hook (not part of the C ABI, not declared in include/): the
// aggregate kernel a dfmi_aggregate_batch call would launch, generated and
// (compile != 0) compiled with hipRTC -- no device needed (tests/test_aggregate_cpu.py).
extern "C" int64_t dfmi_internal_agg_jit_check(const dfmi_program* pred, const dfmi_aggregate* const* aggs, int32_t n,
                                               const dfmi_batch* in, uint32_t flags, int32_t compile, char* buf,
                                               int64_t cap, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    try {
        if (!in || !aggs || n <= 0) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "bad argument"};
        dfmi_agg_state st;
        for (int j = 0; j < n; ++j) st.aggs.push_back(aggs[j]);
        AggBuilt B;
        build_agg_plan(&st, pred, in, flags, B);
        const std::string src = jit::generate(B.plan, B.X);
        if (compile) (void)jit::compile_code(src, nullptr);
        if (buf && cap > 0) snprintf(buf, (size_t)cap, "%s", src.c_str());
        return (int64_t)src.size();
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return -(int64_t)f.code;
    }
}

// Internal test hook: the GROUP BY form of the above (key: a Boolean or
// integer program).
extern "C" int64_t dfmi_internal_agg_grouped_jit_check(const dfmi_program* pred, const dfmi_program* key,
                                                       const dfmi_aggregate* const* aggs, int32_t n,
                                                       const dfmi_batch* in, uint32_t flags, int32_t compile, char* buf,
                                                       int64_t cap, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    try {
        if (!in || !aggs || !key || n <= 0) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "bad argument"};
        dfmi_agg_state st;
        st.grouped = true;
        st.key = *key;
        st.gslots = key->type == DFMI_TYPE_BOOLEAN ? 3 : 17;
        for (int j = 0; j < n; ++j) st.aggs.push_back(aggs[j]);
        AggBuilt B;
        build_agg_plan(&st, pred, in, flags, B);
        const std::string src = jit::generate(B.plan, B.X);
        if (compile) (void)jit::compile_code(src, nullptr);
        if (buf && cap > 0) snprintf(buf, (size_t)cap, "%s", src.c_str());
        return (int64_t)src.size();
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return -(int64_t)f.code;
    }
}
