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
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <new>
#include <string>
#include <string_view>
#include <thread>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "exec_internal.h"
#include "groupby.h"
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

// GROUP BY keys on the host: one part per key expression, ordered
// lexicographically, each part with its null last (aggregate.cpp emit order;
// the oracle's group_key). A non-null part orders by `ord` (key_ord: integers
// numerically, Boolean false < true, floats by IEEE 754 totalOrder), then by
// its bytes (Utf8: bytewise, a shorter prefix first).
struct KeyPart {
    bool null = false;
    __int128 ord = 0;
    uint64_t bits = 0;  // Boolean 0/1, integers sign/zero-extended, float bits
    std::string s;      // Utf8
};
struct HKey {
    std::vector<KeyPart> p;
    bool operator<(const HKey& o) const {
        for (size_t i = 0; i < p.size(); ++i) {
            const KeyPart &a = p[i], &b = o.p[i];
            if (a.null != b.null) return !a.null;
            if (a.null) continue;
            if (a.ord != b.ord) return a.ord < b.ord;
            if (a.s != b.s) return a.s < b.s;
        }
        return false;
    }
};
using GroupMap = std::map<HKey, std::vector<Partial_>>;  // key -> partials + the group's row count

// The device hash table of a grouped state (groupby.h; kernels in groupby.hip).
struct HashDev {
    dfmi::gb::Table t{};
    uint64_t cap = 0;                 // slots
    dfmi::gb::Hdr* hdr = nullptr;     // device counters
    dfmi::gb::Hdr* hh = nullptr;      // pinned host copy
    uint8_t* arena = nullptr;         // Utf8 key bytes
    uint64_t arena_cap = 0;
    unsigned long long* acc = nullptr;      // [acc_cap][words] group records
    uint64_t acc_cap = 0;
    unsigned long long* pattern = nullptr;  // one zero-state record (device)
    std::vector<uint64_t> hpattern;
    int words = 0;
    std::vector<int> off, foff;       // per aggregate: record offset; float SUMs: digit offsets
    int32_t* sidx = nullptr;
    int32_t* coll = nullptr;
    int64_t rows_cap = 0;             // sidx / coll capacity
    uint32_t epoch = 0;
    uint64_t ngroups = 0;             // groups the device holds
    uint64_t rows_since_norm = 0;     // rows added since the digits were last carry-normalised
    struct Buf {
        void* p = nullptr;
        size_t cap = 0;
    };
    std::vector<Buf> bufs;            // the fused pass's output columns (reused across batches)
};

// The device hash table's groups as flat host arrays by group id (read_table;
// for a finish, `rounded`: the records finished on the device and the table
// left as it is):
// keys (null bits, words: the value bits or the Utf8 arena offset, lengths),
// the records, the Utf8 arena, and `order` -- the group ids in key order.
// Pinned host memory that keeps its capacity (a finish's copies land here by
// DMA; no zero-fill, no page faults once warm).
template <typename T>
struct HostBuf {
    T* p = nullptr;
    size_t n = 0, cap = 0;
    HostBuf() = default;
    HostBuf(const HostBuf&) = delete;
    HostBuf& operator=(const HostBuf&) = delete;
    ~HostBuf() {
        if (p) (void)hipHostFree(p);
    }
    void resize(size_t want) {
        if (want > cap) {
            if (p) (void)hipHostFree(p);
            p = nullptr;
            cap = 0;
            const size_t c = std::max<size_t>(want + want / 4, 16);
            HIP_TRY(hipHostMalloc((void**)&p, c * sizeof(T), hipHostMallocDefault));
            cap = c;
        }
        n = want;
    }
    T* data() { return p; }
    const T* data() const { return p; }
    size_t size() const { return n; }
    T& operator[](size_t i) { return p[i]; }
    const T& operator[](size_t i) const { return p[i]; }
};

struct FlatGroups {
    bool rounded = false;  // acc: the device finish's compact records (groupby.h RoundArgs), the table kept
    uint64_t ng = 0;
    size_t nk = 0;
    int words = 0;
    std::vector<int> off;
    std::vector<uint32_t> order;
    HostBuf<unsigned> knull, klen;
    HostBuf<uint64_t> kw, acc;
    HostBuf<uint8_t> arena;
};

struct dfmi_agg_state {
    int device = 0;
    std::vector<const dfmi_aggregate*> aggs;
    uint64_t* acc = nullptr;  // [kAggCopies][n][kAggWords]; grouped: [kAggCopies][gslots][n + 1][kAggWords]
    size_t acc_words = 0;
    bool failed = false;      // a batch raised an error: the query has failed
    dfmi_error failure{};
    std::vector<uint64_t> init;  // the zero state (MIN keys all ones)
    // GROUP BY extension (dfmi_agg_state_create_grouped / _multi)
    bool grouped = false;
    std::vector<dfmi_program> keys;  // the key expressions (copies: same uid, same kernels)
    dfmi_program key;           // keys[0] (the window kernel's key)
    int gslots = 0;             // window slots per accumulator copy: the key window + the null slot
    uint64_t win_base = 0;      // the window the device accumulators hold ...
    int win_width = -1;         // ... (-1: none yet)
    bool dirty = false;         // the device window accumulators hold rows
    GroupMap groups;            // merged groups (window flushes, hash-table drains, host merges)
    // the host merge's per-row lookup: encoded key -> entry of `groups` (map
    // nodes do not move), cleared with it
    std::unordered_map<std::string, std::vector<Partial_>*> index;
    std::shared_ptr<GroupMap> shown;  // groups dfmi_shard_agg_finish_grouped merged (else `groups`)
    HashDev* hd = nullptr;            // device hash table (created on first use)
    std::unique_ptr<FlatGroups> flat; // a finish's groups, not yet in `groups` (finish_flat)
    std::unique_ptr<FlatGroups> spare_flat;  // a used one, its pinned buffers kept for the next drain
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
    uint64_t mant = 0;  // bits [q, msb] (at most prec <= 53 of them), from the top three digits
    if (q <= msb) {
        const int b0 = std::max(top - 2, 0);
        unsigned __int128 w = 0;
        for (int i = top; i >= b0; --i) w = (w << 32) | (uint64_t)d[i];
        mant = (uint64_t)(w >> (q - 32 * b0)) & ((1ull << (msb - q + 1)) - 1);
    }
    const uint64_t rb = q >= 1 ? bit(q - 1) : 0;
    // sticky: any set bit below the round bit, bits [0, q - 2] (whole digits first)
    bool sticky = false;
    if (q >= 2) {
        const int hb = q - 2, hd = hb >> 5;
        for (int i = 0; i < hd && !sticky; ++i) sticky = d[i] != 0;
        const uint64_t m = (hb & 31) == 31 ? 0xffffffffull : ((1ull << ((hb & 31) + 1)) - 1);
        sticky = sticky || ((uint64_t)d[hd] & m) != 0;
    }
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

// A floating-point SUM already rounded (the device finish, k_group_round).
struct Rounded {
    double v;
    bool zero;
};

dfmi_agg_value finish_normalized(const dfmi_aggregate& a, const Partial& p, const Rounded* pre = nullptr);
dfmi_agg_value finish_one(const dfmi_aggregate& a, Partial p) {
    normalize(p);
    return finish_normalized(a, p);
}

// finish_one of a partial whose digits are already carry-normalised (or, with
// `pre`, of a floating-point SUM whose digits the device has rounded).
dfmi_agg_value finish_normalized(const dfmi_aggregate& a, const Partial& p, const Rounded* pre) {
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
            double v;
            if (pre) {
                v = pre->v;
                zero = pre->zero;
            } else {
                v = f32 ? round_exact(p, 24, 925, 0x1p128, &zero) : round_exact(p, 53, 0, HUGE_VAL, &zero);
            }
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

// The group entry of key `hk` (created with n + 1 empty partials).
std::vector<Partial>& group_entry(GroupMap& groups, HKey&& hk, size_t n) {
    auto it = groups.find(hk);
    if (it == groups.end()) it = groups.emplace(std::move(hk), std::vector<Partial>(n + 1)).first;
    return it->second;
}

void merge_group(std::vector<Partial>& into, const std::vector<Partial>& parts, const dfmi_aggregate* const* aggs,
                 size_t n) {
    for (size_t j = 0; j < n; ++j) merge_partial(into[j], parts[j], aggs[j]->fn == DFMI_AGG_MIN);
    into[n].count += parts[n].count;  // the hidden count: the group's selected rows
}

KeyPart fixed_part(int kt, uint64_t bits) {
    KeyPart k;
    k.bits = bits;
    k.ord = key_ord(kt, bits);
    return k;
}

// GROUP BY: the device window accumulators (win_base / win_width) merged into
// the host's groups, and the device window state reset.
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
        HKey hk;
        if (g == st->win_width) {
            hk.p.emplace_back();
            hk.p.back().null = true;
        } else {
            hk.p.push_back(fixed_part(kt, st->win_base + (uint64_t)g));
        }
        merge_group(group_entry(st->groups, std::move(hk), n), parts, st->aggs.data(), n);
    }
    HIP_TRY(hipMemcpyAsync(st->acc, st->init.data(), st->acc_words * 8, hipMemcpyHostToDevice, ctx->stream));
    st->dirty = false;
}

// ---- per-row rules on the host (the host merge: diagnostics A/B, and the
// rows of a batch whose key shares its 63-bit hash with another key's).
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

// ---- the fused evaluation pass of a grouped batch: keys then arguments,
// compacted by the predicate (dfmi_filter_project: the reference's
// evaluation order and first error), into the hash state's reusable device
// buffers. Returns the selected rows; `cols` describes each output (a
// passed-through input column, or the compacted output).
constexpr size_t kDrainBuf = 3 * (dfmi::gb::kMaxKeys + dfmi::gb::kMaxAggs);  // read_table's buffers after the pass's
void* hd_buf(HashDev& H, size_t i, size_t bytes) {
    if (H.bufs.size() <= i) H.bufs.resize(i + 1);
    HashDev::Buf& b = H.bufs[i];
    bytes = std::max<size_t>(bytes, 64);
    if (b.cap < bytes) {
        if (b.p) HIP_TRY(hipFree(b.p));
        b.p = nullptr;
        b.cap = 0;
        const size_t want = bytes + bytes / 4;
        HIP_TRY(hipMalloc(&b.p, want));
        b.cap = want;
    }
    return b.p;
}

HashDev& hashdev(dfmi_context* ctx, dfmi_agg_state* st);

int64_t eval_grouped(dfmi_context* ctx, dfmi_agg_state* st, const dfmi_program* pred, const dfmi_batch* in,
                     uint32_t flags, std::vector<dfmi::gb::Col>& cols) {
    HashDev& H = hashdev(ctx, st);
    const size_t nk = st->keys.size(), n = st->aggs.size();
    const int no = (int)(nk + n);
    const int64_t rows = in->num_rows;
    std::vector<const dfmi_program*> progs(no);
    for (size_t p = 0; p < nk; ++p) progs[p] = &st->keys[p];
    for (size_t j = 0; j < n; ++j) progs[nk + j] = &st->aggs[j]->arg;
    std::vector<dfmi_out_column> outs(no);
    size_t bi = 0;
    for (int o = 0; o < no; ++o) {
        dfmi_out_column& c = outs[o];
        memset(&c, 0, sizeof c);
        const int t = progs[o]->type;
        if (t == DFMI_TYPE_UTF8) {
            const IrNode& root = progs[o]->ir[progs[o]->root];
            size_t cap = 8;
            if (root.kind == IR_COL && root.col >= 0 && root.col < in->num_columns && in->columns[root.col].offsets) {
                int32_t ends[2] = {0, 0};
                HIP_TRY(hipMemcpyAsync(&ends[0], in->columns[root.col].offsets, 4, hipMemcpyDeviceToHost, ctx->stream));
                HIP_TRY(hipMemcpyAsync(&ends[1], in->columns[root.col].offsets + rows, 4, hipMemcpyDeviceToHost,
                                       ctx->stream));
                HIP_TRY(hipStreamSynchronize(ctx->stream));
                cap = std::max<size_t>(cap, (size_t)std::max(0, ends[1] - ends[0]));
            }
            c.offsets = (int32_t*)hd_buf(H, bi++, (size_t)(rows + 1) * 4);
            c.data = (uint8_t*)hd_buf(H, bi++, cap);
            c.data_capacity = (int64_t)cap;
        } else {
            const int w = jit::type_width(t);
            c.values = hd_buf(H, bi++, t == DFMI_TYPE_BOOLEAN ? (size_t)(rows + 63) / 64 * 8 : (size_t)rows * std::max(w, 1));
        }
        c.validity = (uint8_t*)hd_buf(H, bi++, (size_t)(rows + 63) / 64 * 8);
    }
    dfmi_error e{};
    if (dfmi_filter_project(ctx, pred, progs.data(), no, in, outs.data(), flags, &e) != DFMI_OK) {
        st->failed = true;
        st->failure = e;
        throw Fail{e.code, e.message};
    }
    cols.assign(no, dfmi::gb::Col{});
    for (int o = 0; o < no; ++o) {
        const dfmi_out_column& c = outs[o];
        dfmi::gb::Col& d = cols[o];
        d.type = progs[o]->type;
        d.width = d.type == DFMI_TYPE_UTF8 || d.type == DFMI_TYPE_BOOLEAN ? 0 : jit::type_width(d.type);
        if (c.passthrough_column >= 0) {
            const dfmi_column& src = in->columns[c.passthrough_column];
            d.values = src.values;
            d.offsets = src.offsets;
            d.validity = src.null_count > 0 ? src.validity : nullptr;
        } else {
            d.values = d.type == DFMI_TYPE_UTF8 ? (const void*)c.data : c.values;
            d.offsets = c.offsets;
            d.validity = c.null_count > 0 ? c.validity : nullptr;
        }
    }
    return outs[0].length;
}

// Key encoding for the host merge's hash index.
void encode_part(std::string& e, const KeyPart& k) {
    e.push_back(k.null ? 1 : 0);
    if (k.null) return;
    e.append((const char*)&k.ord, sizeof k.ord);
    const uint32_t l = (uint32_t)k.s.size();
    e.append((const char*)&l, 4);
    e.append(k.s);
}

// Rows `rows` (all m rows when null) of the evaluated columns merged into the
// state's groups on the host, with the kernels' per-row rules.
void host_merge_rows(dfmi_context* ctx, dfmi_agg_state* st, const std::vector<dfmi::gb::Col>& cols, int64_t m,
                     const std::vector<int32_t>* rows) {
    const size_t nk = st->keys.size(), n = st->aggs.size(), no = nk + n;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    std::vector<std::vector<uint8_t>> hv(no), hb(no);
    std::vector<std::vector<int32_t>> ho(no);
    for (size_t o = 0; o < no; ++o) {
        const dfmi::gb::Col& c = cols[o];
        if (c.type == DFMI_TYPE_UTF8) {
            ho[o].resize((size_t)m + 1);
            HIP_TRY(hipMemcpy(ho[o].data(), c.offsets, ho[o].size() * 4, hipMemcpyDeviceToHost));
            const int32_t b0 = ho[o][0], b1 = ho[o][m];
            for (int32_t& x : ho[o]) x -= b0;  // (a sliced column's offsets need not start at 0)
            hv[o].resize((size_t)std::max(b1 - b0, 1));
            if (b1 > b0) HIP_TRY(hipMemcpy(hv[o].data(), (const uint8_t*)c.values + b0, (size_t)(b1 - b0),
                                           hipMemcpyDeviceToHost));
        } else {
            const size_t vb = c.type == DFMI_TYPE_BOOLEAN ? (size_t)(m + 7) / 8 : (size_t)m * c.width;
            hv[o].resize(std::max<size_t>(vb, 1));
            if (vb) HIP_TRY(hipMemcpy(hv[o].data(), c.values, vb, hipMemcpyDeviceToHost));
        }
        if (c.validity && m) {
            hb[o].resize((size_t)(m + 7) / 8);
            HIP_TRY(hipMemcpy(hb[o].data(), c.validity, hb[o].size(), hipMemcpyDeviceToHost));
        }
    }
    auto valid = [&](size_t o, int64_t i) { return hb[o].empty() || ((hb[o][i >> 3] >> (i & 7)) & 1); };
    std::vector<std::vector<Partial>*> touched;
    std::string enc;
    const int64_t cnt = rows ? (int64_t)rows->size() : m;
    for (int64_t x = 0; x < cnt; ++x) {
        const int64_t i = rows ? (int64_t)(*rows)[x] : x;
        HKey hk;
        hk.p.resize(nk);
        enc.clear();
        for (size_t p = 0; p < nk; ++p) {
            KeyPart& k = hk.p[p];
            const int kt = cols[p].type;
            if (!valid(p, i)) {
                k.null = true;
            } else if (kt == DFMI_TYPE_UTF8) {
                k.s.assign((const char*)hv[p].data() + ho[p][i], (size_t)(ho[p][i + 1] - ho[p][i]));
            } else if (kt == DFMI_TYPE_BOOLEAN) {
                k = fixed_part(kt, (hv[p][i >> 3] >> (i & 7)) & 1);
            } else {
                uint64_t raw = 0;
                memcpy(&raw, hv[p].data() + (size_t)i * cols[p].width, cols[p].width);
                k = fixed_part(kt, is_signed_type(kt) ? (uint64_t)(int64_t)narrow_int(raw, kt) : narrow_int(raw, kt));
            }
            encode_part(enc, k);
        }
        std::vector<Partial>* entry;
        auto ix = st->index.find(enc);
        if (ix != st->index.end()) {
            entry = ix->second;
        } else {  // first row of this key since the last reset / drain of the index
            entry = &group_entry(st->groups, std::move(hk), n);
            st->index.emplace(enc, entry);
        }
        std::vector<Partial>& g = *entry;
        if (g[n].flags == 0) {  // first touch in this call: normalise it at the end
            g[n].flags = 1;
            touched.push_back(entry);
        }
        ++g[n].count;  // the group's selected rows
        for (size_t j = 0; j < n; ++j)
            if (valid(nk + j, i)) host_accumulate(g[j], st->aggs[j]->fn, cols[nk + j].type, hv[nk + j].data(), i);
    }
    for (std::vector<Partial>* e : touched) {  // only the entries this call touched
        for (Partial& q : *e) normalize(q);
        (*e)[n].flags = 0;
    }
}

// A batch merged on the host, row by row (diagnostics: DFMI_DIAG=1
// DFMI_GROUP_HOST=1, the A/B of the device hash table).
void group_batch_on_host(dfmi_context* ctx, dfmi_agg_state* st, const dfmi_program* pred, const dfmi_batch* in,
                         uint32_t flags) {
    std::vector<dfmi::gb::Col> cols;
    const int64_t m = eval_grouped(ctx, st, pred, in, flags, cols);
    if (m > 0) host_merge_rows(ctx, st, cols, m, nullptr);
}

// ---- the device hash table (groupby.h)
void free_hashdev(HashDev* H) {
    if (!H) return;
    void* ps[] = {H->t.ctl, H->t.slot, H->hdr, H->arena,
                  H->acc, H->pattern, H->sidx, H->coll};
    for (void* p : ps)
        if (p) (void)hipFree(p);
    if (H->hh) (void)hipHostFree(H->hh);
    for (auto& b : H->bufs)
        if (b.p) (void)hipFree(b.p);
    delete H;
}

void alloc_table(dfmi::gb::Table& t, uint64_t cap, hipStream_t stream) {
    t = dfmi::gb::Table{};
    HIP_TRY(hipMalloc((void**)&t.ctl, cap * 8));
    HIP_TRY(hipMalloc((void**)&t.slot, cap * sizeof(dfmi::gb::Slot)));
    HIP_TRY(hipMemsetAsync(t.ctl, 0, cap * 8, stream));
    t.mask = cap - 1;
}

void free_table(dfmi::gb::Table& t) {
    void* ps[] = {t.ctl, t.slot};
    for (void* p : ps)
        if (p) (void)hipFree(p);
    t = dfmi::gb::Table{};
}

constexpr uint64_t kTableSlots0 = 1 << 16;

HashDev& hashdev(dfmi_context* ctx, dfmi_agg_state* st) {
    if (st->hd) return *st->hd;
    HashDev* H = new HashDev();
    try {
        const size_t n = st->aggs.size();
        int w = 1;  // word 0: the group's rows
        for (size_t j = 0; j < n; ++j) {
            H->off.push_back(w);
            const bool fs = st->aggs[j]->fn == DFMI_AGG_SUM && is_float_type(st->aggs[j]->arg.type);
            if (fs) H->foff.push_back(w + 4);
            w += 4 + (fs ? kAggLimbs : 0);
        }
        H->words = w;
        H->hpattern.assign((size_t)w, 0);
        for (size_t j = 0; j < n; ++j)
            if (st->aggs[j]->fn == DFMI_AGG_MIN) H->hpattern[(size_t)H->off[j] + 2] = ~0ull;
        HIP_TRY(hipMalloc((void**)&H->pattern, (size_t)w * 8));
        HIP_TRY(hipMemcpyAsync(H->pattern, H->hpattern.data(), (size_t)w * 8, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(hipMalloc((void**)&H->hdr, sizeof(dfmi::gb::Hdr)));
        HIP_TRY(hipMemsetAsync(H->hdr, 0, sizeof(dfmi::gb::Hdr), ctx->stream));
        HIP_TRY(hipHostMalloc((void**)&H->hh, sizeof(dfmi::gb::Hdr), hipHostMallocDefault));
        H->cap = kTableSlots0;
        alloc_table(H->t, H->cap, ctx->stream);
        H->acc_cap = 1024;
        HIP_TRY(hipMalloc((void**)&H->acc, H->acc_cap * (size_t)w * 8));
        HIP_TRY(dfmi::gb::launch_init(H->acc, H->pattern, w, 0, H->acc_cap, ctx->stream));
        H->arena_cap = 1 << 16;
        HIP_TRY(hipMalloc((void**)&H->arena, H->arena_cap));
    } catch (...) {
        free_hashdev(H);
        throw;
    }
    st->hd = H;
    return *H;
}

void read_hdr(dfmi_context* ctx, HashDev& H) {
    HIP_TRY(hipMemcpyAsync(H.hh, H.hdr, sizeof(dfmi::gb::Hdr), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
}

// A bigger table (cap x 4), every used slot moved (k_group_rehash).
void grow_table(dfmi_context* ctx, HashDev& H) {
    dfmi::gb::Table nt;
    const uint64_t ncap = H.cap * 4;
    alloc_table(nt, ncap, ctx->stream);
    HIP_TRY(dfmi::gb::launch_rehash(H.t, nt, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    free_table(H.t);
    H.t = nt;
    H.cap = ncap;
}

// Device buffer `p` of `have` bytes replaced by one of `want`, the first
// `keep` bytes copied.
template <typename T>
void regrow(dfmi_context* ctx, T*& p, size_t keep, size_t want) {
    T* q = nullptr;
    HIP_TRY(hipMalloc((void**)&q, want));
    if (keep) HIP_TRY(hipMemcpyAsync(q, p, keep, hipMemcpyDeviceToDevice, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    if (p) HIP_TRY(hipFree(p));
    p = q;
}

// Bucketed accumulation (groupby.h): worth it when the batch has many rows per
// group -- the per-bucket sums then replace ~(2 + 3 per float SUM) scattered
// record atomics per row by LDS atomics, and each (bucket, split) block adds
// a group's moved words once. Needs the bucket's records in the LDS left
// beside the bucket starts (groupby.h kBucketRecordLds) and at most
// kBucketMax buckets. DFMI_DIAG=1 DFMI_GROUP_BUCKETS=0 / 1
// forces the choice (tests run small batches through both).
constexpr size_t kBucketBuf = kDrainBuf + 8;

struct BucketShape {
    uint32_t gpb = 0;  // a power of two: 1 << gshift
    int gshift = 0;
    int nbuckets = 0, splits = 0;
};

// Records per bucket: as many as fit the LDS a block keeps beside its bucket
// starts with two blocks per CU (kBucketRecordLds); when that needs more than
// kBucketMax buckets, as many as fit one block per CU (kBucketRecordLdsBig,
// 160 KiB per workgroup on gfx950).
BucketShape bucket_shape(const HashDev& H, uint64_t ng) {
    BucketShape b;
    if (!ng) return b;
    for (int budget : {dfmi::gb::kBucketRecordLds, dfmi::gb::kBucketRecordLdsBig}) {
        const size_t fit = (size_t)budget / ((size_t)H.words * 8);
        if (!fit) continue;
        b.gshift = 0;
        while ((2ull << b.gshift) <= fit) ++b.gshift;
        b.gpb = 1u << b.gshift;
        b.nbuckets = (int)((ng + b.gpb - 1) / b.gpb);
        if (b.nbuckets <= dfmi::gb::kBucketMax) break;
    }
    b.splits = std::max(1, std::min(1024, 2048 / std::max(1, b.nbuckets)));
    return b;
}

bool use_buckets(const dfmi_agg_state* st, const HashDev& H, int64_t m, uint64_t ng) {
    const BucketShape b = bucket_shape(H, ng);
    if (!b.gpb || b.nbuckets > dfmi::gb::kBucketMax || st->aggs.size() > 32) return false;
    if (getenv("DFMI_DIAG"))
        if (const char* e = getenv("DFMI_GROUP_BUCKETS")) return atoi(e) != 0;
    // the partitioned copy of the batch (group id, NULL mask, one 8-byte word
    // per argument) stays within 16 GiB of the 288 GB
    if ((uint64_t)m * (12 + 8 * st->aggs.size()) > (16ull << 30)) return false;
    // ~4 record atomics per row against each block adding a touched group's
    // ~10 moved words once: many rows per group and split
    return (uint64_t)m >= 4ull * ng * (uint64_t)b.splits && m >= (1 << 20);
}

std::atomic<long> g_bucketed_batches{0};  // diagnostics: dfmi_internal_group_bucketed_batches

void accumulate_bucketed(dfmi_context* ctx, dfmi_agg_state* st, HashDev& H, const std::vector<dfmi::gb::Col>& cols,
                         int64_t m, uint64_t ng, uint32_t epoch) {
    g_bucketed_batches.fetch_add(1);
    const size_t nk = st->keys.size(), n = st->aggs.size();
    const BucketShape sh = bucket_shape(H, ng);
    const size_t nbh = (size_t)sh.nbuckets * dfmi::gb::kBucketBlocks;
    dfmi::gb::RankArgs ra{};
    for (size_t p = 0; p < nk; ++p) ra.k[p] = cols[p];
    ra.nkeys = (int)nk;
    ra.epoch = epoch;
    ra.m = m;
    ra.t = H.t;
    ra.arena = H.arena;
    ra.arena_cap = H.arena_cap;
    ra.sidx = H.sidx;
    ra.hdr = H.hdr;
    ra.coll_rows = H.coll;
    ra.rg = (unsigned*)hd_buf(H, kBucketBuf, (size_t)m * 4);
    ra.gshift = sh.gshift;
    ra.nbuckets = sh.nbuckets;
    ra.bh = (unsigned*)hd_buf(H, kBucketBuf + 1, nbh * 4);
    dfmi::gb::ScatterArgs sa{};
    sa.m = m;
    sa.rg = ra.rg;
    sa.gshift = sh.gshift;
    sa.nbuckets = sh.nbuckets;
    sa.base = ra.bh;
    sa.tot = (const unsigned*)hd_buf(H, kBucketBuf + 2, (size_t)sh.nbuckets * 4);
    sa.naggs = (int)n;
    dfmi::gb::BucketArgs ba{};
    bool nullable = false;
    int npay = 0;
    for (size_t j = 0; j < n; ++j) {
        const dfmi::gb::Col& c = cols[nk + j];
        sa.arg[j] = c;
        nullable = nullable || c.validity;
        ba.a[j].c = c;
        ba.a[j].fn = st->aggs[j]->fn;
        ba.a[j].off = H.off[j];
        ba.pcol[j] = -1;
        const bool needs = st->aggs[j]->fn != DFMI_AGG_COUNT && c.type != DFMI_TYPE_UTF8 && c.type != DFMI_TYPE_BOOLEAN;
        if (!needs) continue;
        for (int q = 0; q < npay && ba.pcol[j] < 0; ++q)  // one payload column per distinct argument column
            if (sa.pay[q].values == c.values && sa.pay[q].type == c.type) ba.pcol[j] = q;
        if (ba.pcol[j] < 0) {
            sa.pay[npay] = c;
            ba.pcol[j] = npay++;
        }
    }
    sa.npay = npay;
    sa.pg = (unsigned*)hd_buf(H, kBucketBuf + 3, (size_t)m * 4);
    sa.pn = nullable ? (unsigned*)hd_buf(H, kBucketBuf + 4, (size_t)m * 4) : nullptr;
    sa.pv = (unsigned long long*)hd_buf(H, kBucketBuf + 5, (size_t)std::max(npay, 1) * (size_t)m * 8);
    ba.m = m;
    ba.tot = sa.tot;
    ba.gpb = sh.gpb;
    ba.nbuckets = sh.nbuckets;
    ba.splits = sh.splits;
    ba.ngroups = ng;
    ba.pg = sa.pg;
    ba.pn = sa.pn;
    ba.pv = sa.pv;
    ba.naggs = (int)n;
    ba.words = H.words;
    ba.acc = H.acc;
    ba.pattern = H.pattern;
    HIP_TRY(dfmi::gb::launch_buckets(ra, sa, ba, ctx->stream));
}

// One batch through the device hash table: the fused evaluation pass, the
// claim pass (the table grown and the pass run again while a row finds no
// slot), the accumulate pass; rows whose key shares its hash with another
// key's are merged on the host.
void group_batch_hashed(dfmi_context* ctx, dfmi_agg_state* st, const dfmi_program* pred, const dfmi_batch* in,
                        uint32_t flags) {
    HashDev& H = hashdev(ctx, st);
    std::vector<dfmi::gb::Col> cols;
    const bool prof = getenv("DFMI_DIAG") && getenv("DFMI_FINISH_PROFILE");
    const auto t0 = std::chrono::steady_clock::now();
    const int64_t m = eval_grouped(ctx, st, pred, in, flags, cols);
    if (prof) HIP_TRY(hipStreamSynchronize(ctx->stream));
    const auto t1 = std::chrono::steady_clock::now();
    if (m <= 0) return;
    if (m > 0x7fffffffll) throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "GROUP BY batch of 2^31 selected rows or more"};
    const size_t nk = st->keys.size(), n = st->aggs.size();
    hipStream_t stream = ctx->stream;
    if (H.rows_cap < m) {
        if (H.sidx) HIP_TRY(hipFree(H.sidx));
        if (H.coll) HIP_TRY(hipFree(H.coll));
        H.sidx = H.coll = nullptr;
        H.rows_cap = 0;
        const int64_t want = m + m / 4;
        HIP_TRY(hipMalloc((void**)&H.sidx, (size_t)want * 4));
        HIP_TRY(hipMalloc((void**)&H.coll, (size_t)want * 4));
        H.rows_cap = want;
    }
    uint64_t hash_mask = ~0ull;
    if (getenv("DFMI_DIAG"))  // diagnostics: a hash of so few bits that many keys share one (the host merge path)
        if (const char* e = getenv("DFMI_GROUP_HASH_BITS")) hash_mask = (1ull << std::max(1, std::min(63, atoi(e)))) - 1;
    dfmi::gb::ClaimArgs ca{};
    for (size_t p = 0; p < nk; ++p) ca.k[p] = cols[p];
    ca.nkeys = (int)nk;
    ca.epoch = ++H.epoch;
    ca.m = m;
    ca.hash_mask = hash_mask;
    ca.hdr = H.hdr;
    ca.sidx = H.sidx;
    for (int attempt = 0;; ++attempt) {
        ca.t = H.t;
        ca.limit = H.cap / 2;
        HIP_TRY(hipMemsetAsync(&H.hdr->overflow, 0, 8, stream));
        HIP_TRY(dfmi::gb::launch_claim(ca, stream));
        read_hdr(ctx, H);
        if (!H.hh->overflow) break;
        if (H.cap >= (1ull << 31) || attempt > 16)
            throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "GROUP BY: more than 2^30 groups on one device"};
        grow_table(ctx, H);
    }
    const uint64_t ng = H.hh->ngroups, aend = H.hh->arena_end;
    const auto t2 = std::chrono::steady_clock::now();
    if (ng > H.acc_cap) {
        uint64_t want = H.acc_cap;
        while (want < ng) want *= 2;
        regrow(ctx, H.acc, H.acc_cap * (size_t)H.words * 8, want * (size_t)H.words * 8);
        HIP_TRY(dfmi::gb::launch_init(H.acc, H.pattern, H.words, H.acc_cap, want, stream));
        H.acc_cap = want;
    }
    if (aend > H.arena_cap) {
        uint64_t want = H.arena_cap;
        while (want < aend) want *= 2;
        regrow(ctx, H.arena, H.arena_cap, want);
        H.arena_cap = want;
    }
    // exact-sum digits absorb 2^31 rows between carry normalisations
    if (!H.foff.empty() && H.rows_since_norm + (uint64_t)m > (1ull << 30)) {
        HIP_TRY(dfmi::gb::launch_normalize(H.acc, H.words, H.foff.data(), (int)H.foff.size(), H.ngroups, stream));
        H.rows_since_norm = 0;
    }
    HIP_TRY(hipMemsetAsync(&H.hdr->collided, 0, 8, stream));
    if (use_buckets(st, H, m, ng)) {
        accumulate_bucketed(ctx, st, H, cols, m, ng, ca.epoch);
    } else {
    dfmi::gb::AccArgs aa{};
    for (size_t p = 0; p < nk; ++p) aa.k[p] = cols[p];
    aa.nkeys = (int)nk;
    aa.epoch = ca.epoch;
    aa.m = m;
    aa.t = H.t;
    aa.arena = H.arena;
    aa.arena_cap = H.arena_cap;
    aa.sidx = H.sidx;
    for (size_t j = 0; j < n; ++j) {
        aa.a[j].c = cols[nk + j];
        aa.a[j].fn = st->aggs[j]->fn;
        aa.a[j].off = H.off[j];
    }
    aa.naggs = (int)n;
    aa.words = H.words;
    aa.acc = H.acc;
    aa.hdr = H.hdr;
    aa.coll_rows = H.coll;
    HIP_TRY(dfmi::gb::launch_accumulate(aa, stream));
    }
    read_hdr(ctx, H);
    if (prof) {
        auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
        fprintf(stderr, "[dfmi add] %lld rows, %llu groups: eval %.1f us, claim %.1f us, accumulate %.1f us\n",
                (long long)m, (unsigned long long)ng, us(t0, t1), us(t1, t2), us(t2, std::chrono::steady_clock::now()));
    }
    H.ngroups = ng;
    H.rows_since_norm += (uint64_t)m;
    const uint64_t nc = H.hh->collided;
    if (nc) {  // rows whose key shares its 63-bit hash with another group's key
        std::vector<int32_t> rows((size_t)nc);
        HIP_TRY(hipMemcpy(rows.data(), H.coll, (size_t)nc * 4, hipMemcpyDeviceToHost));
        std::sort(rows.begin(), rows.end());
        host_merge_rows(ctx, st, cols, m, &rows);
    }
}

// fn(i0, i1) over [0, n) in contiguous ranges of at least `grain`, on up to
// DFMI_HOST_THREADS (default min(cores, 8)) threads.
template <typename F>
void parallel_ranges(uint64_t n, uint64_t grain, const F& fn) {
    int hw = (int)std::thread::hardware_concurrency();
    if (const char* e = getenv("DFMI_HOST_THREADS")) hw = atoi(e);
    const uint64_t ways = std::min<uint64_t>((uint64_t)std::max(1, std::min(hw, 8)), std::max<uint64_t>(1, n / grain));
    if (ways <= 1) {
        fn((uint64_t)0, n);
        return;
    }
    std::vector<std::thread> th;
    const uint64_t piece = (n + ways - 1) / ways;
    for (uint64_t w = 1; w < ways; ++w) th.emplace_back([&, w] { fn(std::min(n, w * piece), std::min(n, (w + 1) * piece)); });
    fn(0, std::min(n, piece));
    for (auto& t : th) t.join();
}

// The groups the device hash table holds, copied out as flat arrays by group
// id (keys compacted on the device: k_group_compact), and the table emptied
// (the next batch starts a new one of the same size) -- or, `rounded` (a
// finish), every record finished on the device first (k_group_round: the
// compact records without their exact-sum digits cross PCIe) and the table
// kept as it is, so that more batches can still merge into it.
void read_table(dfmi_context* ctx, dfmi_agg_state* st, FlatGroups& f, bool rounded = false) {
    HashDev& H = *st->hd;
    const size_t nk = st->keys.size(), n = st->aggs.size();
    const uint64_t ng = H.ngroups;
    f.rounded = rounded;
    f.ng = ng;
    f.nk = nk;
    f.words = H.words;
    f.off = H.off;
    const unsigned long long* src = H.acc;
    if (rounded) {
        dfmi::gb::RoundArgs ra{};
        ra.acc = H.acc;
        ra.words = H.words;
        ra.naggs = (int)n;
        for (size_t j = 0; j < n; ++j) {
            ra.off[j] = H.off[j];
            const int t = st->aggs[j]->arg.type;
            ra.kind[j] = st->aggs[j]->fn == DFMI_AGG_SUM && is_float_type(t) ? (t == DFMI_TYPE_FLOAT32 ? 2 : 1) : 0;
            f.off[j] = 1 + 4 * (int)j;
        }
        f.words = 1 + 4 * (int)n;
        ra.ngroups = ng;
        ra.out = (unsigned long long*)hd_buf(H, kDrainBuf + 3, ng * (size_t)f.words * 8);
        HIP_TRY(dfmi::gb::launch_round(ra, ctx->stream));
        src = ra.out;
    }
    unsigned* dnull = (unsigned*)hd_buf(H, kDrainBuf, ng * 4);
    unsigned long long* dkw = (unsigned long long*)hd_buf(H, kDrainBuf + 1, ng * nk * 8);
    unsigned* dklen = (unsigned*)hd_buf(H, kDrainBuf + 2, ng * nk * 4);
    HIP_TRY(dfmi::gb::launch_compact(H.t, (int)nk, dnull, dkw, dklen, ctx->stream));
    f.knull.resize(ng);
    f.klen.resize(ng * nk);
    f.kw.resize(ng * nk);
    f.acc.resize(ng * (size_t)f.words);
    HIP_TRY(hipMemcpyAsync(f.knull.data(), dnull, ng * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipMemcpyAsync(f.kw.data(), dkw, ng * nk * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipMemcpyAsync(f.klen.data(), dklen, ng * nk * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipMemcpyAsync(f.acc.data(), src, f.acc.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
    read_hdr(ctx, H);  // (synchronises the stream)
    f.arena.resize((size_t)H.hh->arena_end);
    if (H.hh->arena_end) HIP_TRY(hipMemcpy(f.arena.data(), H.arena, H.hh->arena_end, hipMemcpyDeviceToHost));
    if (rounded) return;
    // an empty table of the same size for the next batch
    HIP_TRY(hipMemsetAsync(H.t.ctl, 0, H.cap * 8, ctx->stream));
    HIP_TRY(hipMemsetAsync(H.hdr, 0, sizeof(dfmi::gb::Hdr), ctx->stream));
    HIP_TRY(dfmi::gb::launch_init(H.acc, H.pattern, H.words, 0, ng, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    H.ngroups = 0;
    H.rows_since_norm = 0;
}

// f.order: the group ids in key order (HKey's order restated on the flat
// arrays: per part, null last; integers / floats by key_ord; Utf8 bytewise,
// a shorter prefix first).
void sort_flat(const dfmi_agg_state* st, FlatGroups& f) {
    const uint64_t ng = f.ng;
    const size_t nk = f.nk;
    f.order.resize(ng);
    if (nk == 1 && st->keys[0].type != DFMI_TYPE_UTF8) {  // one fixed-width part: sort on (null, ord) values
        // LSD radix sort (16-bit digits) of the order values mapped onto
        // unsigned 64 bits (signed integers offset by 2^63); the null group last
        const int kt = st->keys[0].type;
        const bool sgn = is_signed_type(kt);
        std::vector<uint64_t> kv, kv2;
        std::vector<uint32_t> id, id2;
        kv.reserve(ng);
        id.reserve(ng);
        int64_t null_g = -1;
        for (uint64_t g = 0; g < ng; ++g) {
            if (f.knull[g] & 1) {
                null_g = (int64_t)g;
                continue;
            }
            const __int128 o = key_ord(kt, f.kw[g]);
            kv.push_back(sgn ? (uint64_t)(int64_t)o ^ (1ull << 63) : (uint64_t)o);
            id.push_back((uint32_t)g);
        }
        const size_t m = kv.size();
        if (m < 1024) {
            std::vector<std::pair<uint64_t, uint32_t>> ko(m);
            for (size_t i = 0; i < m; ++i) ko[i] = {kv[i], id[i]};
            std::sort(ko.begin(), ko.end());
            for (size_t i = 0; i < m; ++i) f.order[i] = ko[i].second;
        } else {
            // LSD radix sort, digits of D bits (8 below 2^18 groups: the counts stay in L1; 16 above);
            // a digit every key shares moves nothing and is skipped (one histogram pass finds them all)
            const int D = m < (1u << 18) ? 8 : 16, P = 64 / D;
            const size_t R = (size_t)1 << D;
            kv2.resize(m);
            id2.resize(m);
            std::vector<uint32_t> cnt(R * P, 0);
            for (size_t i = 0; i < m; ++i)
                for (int p = 0; p < P; ++p) ++cnt[(size_t)p * R + ((kv[i] >> (D * p)) & (R - 1))];
            for (int p = 0; p < P; ++p) {
                uint32_t* c = &cnt[(size_t)p * R];
                const int sh = D * p;
                if (c[(kv[0] >> sh) & (R - 1)] == m) continue;  // one digit value: this pass moves nothing
                uint32_t sum = 0;
                for (size_t d = 0; d < R; ++d) {
                    const uint32_t t = c[d];
                    c[d] = sum;
                    sum += t;
                }
                for (size_t i = 0; i < m; ++i) {
                    const uint32_t d = c[(kv[i] >> sh) & (R - 1)]++;
                    kv2[d] = kv[i];
                    id2[d] = id[i];
                }
                kv.swap(kv2);
                id.swap(id2);
            }
            std::copy(id.begin(), id.end(), f.order.begin());
        }
        if (null_g >= 0) f.order[m] = (uint32_t)null_g;
        return;
    }
    for (uint64_t g = 0; g < ng; ++g) f.order[g] = (uint32_t)g;
    std::vector<int> kt(nk);
    for (size_t p = 0; p < nk; ++p) kt[p] = st->keys[p].type;
    auto less = [&](uint32_t a, uint32_t b) {
        for (size_t p = 0; p < nk; ++p) {
            const bool na = (f.knull[a] >> p) & 1, nb = (f.knull[b] >> p) & 1;
            if (na != nb) return !na;
            if (na) continue;
            const uint64_t wa = f.kw[a * nk + p], wb = f.kw[b * nk + p];
            if (kt[p] == DFMI_TYPE_UTF8) {
                const unsigned la = f.klen[a * nk + p], lb = f.klen[b * nk + p];
                const int c = memcmp(f.arena.data() + wa, f.arena.data() + wb, std::min(la, lb));
                if (c) return c < 0;
                if (la != lb) return la < lb;
            } else if (wa != wb) {
                return key_ord(kt[p], wa) < key_ord(kt[p], wb);
            }
        }
        return false;
    };
    if (ng < 256) {
        std::sort(f.order.begin(), f.order.end(), less);
        return;
    }
    // Composite words per group, compared lexicographically: per part a null
    // flag (the null last) and a value -- a fixed-width part its order value,
    // a Utf8 part its first 8 bytes big-endian, zero-padded. LSD radix over the
    // words (8-bit digits, a digit every group shares skipped), then the runs
    // the prefixes cannot order re-sorted with the full comparator.
    const size_t W = 2 * nk;
    std::vector<uint64_t> cw(ng * W);
    bool any_utf8 = false;
    for (uint64_t g = 0; g < ng; ++g)
        for (size_t p = 0; p < nk; ++p) {
            const bool null = (f.knull[g] >> p) & 1;
            uint64_t v = 0;
            if (!null) {
                const uint64_t w = f.kw[g * nk + p];
                if (kt[p] == DFMI_TYPE_UTF8) {
                    any_utf8 = true;
                    const unsigned len = f.klen[g * nk + p];
                    const uint8_t* c = f.arena.data() + w;
                    for (unsigned q = 0; q < 8; ++q) v = (v << 8) | (q < len ? c[q] : 0u);
                } else {
                    const __int128 o = key_ord(kt[p], w);
                    v = is_signed_type(kt[p]) ? (uint64_t)(int64_t)o ^ (1ull << 63) : (uint64_t)o;
                }
            }
            cw[g * W + 2 * p] = null ? 1 : 0;
            cw[g * W + 2 * p + 1] = v;
        }
    std::vector<uint32_t> tmp(ng);
    std::vector<uint32_t> cnt(256);
    for (size_t q = W; q-- > 0;) {
        const int digits = (q & 1) ? 8 : 1;
        for (int d = 0; d < digits; ++d) {
            const int sh = 8 * d;
            std::fill(cnt.begin(), cnt.end(), 0);
            for (uint64_t i = 0; i < ng; ++i) ++cnt[(cw[(size_t)f.order[i] * W + q] >> sh) & 0xff];
            if (cnt[(cw[(size_t)f.order[0] * W + q] >> sh) & 0xff] == ng) continue;
            uint32_t sum = 0;
            for (auto& c : cnt) {
                const uint32_t t = c;
                c = sum;
                sum += t;
            }
            for (uint64_t i = 0; i < ng; ++i) tmp[cnt[(cw[(size_t)f.order[i] * W + q] >> sh) & 0xff]++] = f.order[i];
            std::copy(tmp.begin(), tmp.end(), f.order.begin());
        }
    }
    if (!any_utf8) return;
    // the word order is exact up to the first Utf8 part's prefix: groups that
    // agree on every word up to it may be out of order (the rest of that part
    // decides before any later part), so each such run is re-sorted in full
    size_t p1 = 0;
    while (kt[p1] != DFMI_TYPE_UTF8) ++p1;
    const size_t E = 2 * p1 + 2;
    auto same = [&](uint32_t a, uint32_t b) {
        return std::equal(cw.begin() + (size_t)a * W, cw.begin() + (size_t)a * W + E, cw.begin() + (size_t)b * W);
    };
    for (uint64_t i = 0; i < ng;) {
        uint64_t j = i + 1;
        while (j < ng && same(f.order[i], f.order[j])) ++j;
        if (j - i > 1) std::sort(f.order.begin() + i, f.order.begin() + j, less);
        i = j;
    }
}

// Aggregate j's partial of group record `rec` (the device record layout:
// groupby.h; word 0 the group's rows).
void rec_partial(const dfmi_agg_state* st, const FlatGroups& f, const uint64_t* rec, size_t j, Partial& q) {
    const uint64_t* w = rec + f.off[j];
    const int fn = st->aggs[j]->fn;
    q.count = rec[0] - w[0];  // the group's rows minus its NULL arguments
    if (fn == DFMI_AGG_SUM && is_float_type(st->aggs[j]->arg.type)) {
        q.flags = (w[1] & 0xffffffffull) | (q.count > w[3] ? AGGF_NONNEGZERO : 0);
        if (f.rounded) return;  // (the digits were rounded on the device: w[2])
        for (int i = 0; i < kAggLimbs; ++i) q.limbs[i] = (int64_t)w[4 + i];
        normalize(q);
    } else if (fn == DFMI_AGG_SUM) {
        q.isum = w[3];
    } else if (fn == DFMI_AGG_MIN || fn == DFMI_AGG_MAX) {
        q.key = w[2];
        q.flags = (w[3] ? AGGF_NAN : 0) | (q.count > w[3] ? AGGF_VALUE : 0);
    }
}

// The flat groups merged into st->groups (into an empty map in key order:
// each insertion O(1) at its end).
void materialize_flat(dfmi_agg_state* st, FlatGroups& f) {
    const size_t nk = f.nk, n = st->aggs.size();
    const bool fresh = st->groups.empty();
    if (fresh && f.order.size() != f.ng) sort_flat(st, f);
    for (uint64_t i = 0; i < f.ng; ++i) {
        const uint32_t g = fresh ? f.order[i] : (uint32_t)i;
        HKey hk;
        hk.p.resize(nk);
        for (size_t p = 0; p < nk; ++p) {
            KeyPart& k = hk.p[p];
            const int kt = st->keys[p].type;
            if ((f.knull[g] >> p) & 1) k.null = true;
            else if (kt == DFMI_TYPE_UTF8) k.s.assign((const char*)f.arena.data() + f.kw[g * nk + p], f.klen[g * nk + p]);
            else k = fixed_part(kt, f.kw[g * nk + p]);
        }
        const uint64_t* rec = &f.acc[(size_t)g * f.words];
        std::vector<Partial> parts(n + 1);
        parts[n].count = rec[0];
        for (size_t j = 0; j < n; ++j) rec_partial(st, f, rec, j, parts[j]);
        if (fresh) st->groups.emplace_hint(st->groups.end(), std::move(hk), std::move(parts));
        else merge_group(group_entry(st->groups, std::move(hk), n), parts, st->aggs.data(), n);
    }
}

// A finish's flat groups (st->flat) moved into st->groups before anything
// else merges into or reads the map (a device-finished snapshot is dropped:
// the device table still holds its groups).
void unflatten(dfmi_agg_state* st) {
    if (!st->flat) return;
    std::unique_ptr<FlatGroups> f = std::move(st->flat);
    if (!f->rounded) materialize_flat(st, *f);
    st->spare_flat = std::move(f);
}

std::unique_ptr<FlatGroups> take_flat(dfmi_agg_state* st) {
    std::unique_ptr<FlatGroups> f = st->spare_flat ? std::move(st->spare_flat) : std::make_unique<FlatGroups>();
    f->order.clear();
    return f;
}

// The groups the device hash table holds merged into st->groups, and the
// table emptied.
void drain_hashed(dfmi_context* ctx, dfmi_agg_state* st) {
    unflatten(st);
    if (!st->hd || !st->hd->ngroups) return;
    std::unique_ptr<FlatGroups> f = take_flat(st);
    read_table(ctx, st, *f);
    materialize_flat(st, *f);
    st->spare_flat = std::move(f);
}

// The finish of a state whose groups all sit in the device hash table (no
// window flush, no host merge: the common case): every group finished on the
// device, the results kept flat (st->flat, sorted by key) and emitted from
// there -- no per-group map node, key string, partial copy or exact-sum
// digits on the host; the table keeps the groups for later batches.
bool finish_flat(dfmi_context* ctx, dfmi_agg_state* st) {
    flush_groups(ctx, st);
    if (!st->groups.empty()) return false;
    if (st->flat && !st->flat->rounded && st->hd && st->hd->ngroups) return false;  // (a batch unflattens first)
    if (!st->flat) {
        if (!st->hd || !st->hd->ngroups) return false;
        std::unique_ptr<FlatGroups> f = take_flat(st);
        const auto t0 = std::chrono::steady_clock::now();
        read_table(ctx, st, *f, !(getenv("DFMI_DIAG") && getenv("DFMI_GROUP_HOST_FINISH")));
        const auto t1 = std::chrono::steady_clock::now();
        sort_flat(st, *f);
        if (getenv("DFMI_DIAG") && getenv("DFMI_FINISH_PROFILE"))
            fprintf(stderr, "[dfmi finish] %llu groups: read_table %.1f us, sort %.1f us\n", (unsigned long long)f->ng,
                    std::chrono::duration<double, std::micro>(t1 - t0).count(),
                    std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t1).count());
        st->flat = std::move(f);
    }
    st->shown.reset();
    return true;
}

// The finish of one fixed-width key with many groups, ordered and emitted on
// the device (groupby.h EmitArgs): round, compact, sort values, radix sort,
// emission; only the caller's dfmi_agg_value arrays cross PCIe. Taken from
// kDeviceEmitMin groups (below, the host's sort and emission cost less than
// the launches; at 10^4 groups the device path saves 0.7 ms per finish, at
// 10^6 ~35 ms); DFMI_DIAG=1 DFMI_GROUP_DEVICE_EMIT=0 / 1 forces the choice.
constexpr uint64_t kDeviceEmitMin = 2048;
constexpr size_t kEmitBuf = kBucketBuf + 8;
static_assert(sizeof(dfmi_agg_value) == 24, "dfmi_agg_value as groupby.hip AggValue");

bool finish_device(dfmi_context* ctx, dfmi_agg_state* st, int64_t cap, dfmi_agg_value* keys, dfmi_agg_value* values,
                   int64_t* num_groups) {
    if (st->keys.size() != 1 || st->keys[0].type == DFMI_TYPE_UTF8 || !st->hd ||
        st->aggs.size() > (size_t)dfmi::gb::kMaxAggs)
        return false;
    const bool diag = getenv("DFMI_DIAG") != nullptr;
    if (diag && getenv("DFMI_GROUP_HOST_FINISH")) return false;
    const char* force = diag ? getenv("DFMI_GROUP_DEVICE_EMIT") : nullptr;
    if (force && !atoi(force)) return false;
    flush_groups(ctx, st);
    if (!st->groups.empty() || (st->flat && !st->flat->rounded)) return false;
    HashDev& H = *st->hd;
    const uint64_t ng = H.ngroups;
    if (!ng || (!force && ng < kDeviceEmitMin)) return false;
    *num_groups = (int64_t)ng;
    if (*num_groups > cap) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "group capacity too small"};
    if (!keys || !values) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
    if (st->flat) st->spare_flat = std::move(st->flat);
    const size_t n = st->aggs.size();
    hipStream_t stream = ctx->stream;
    dfmi::gb::RoundArgs ra{};
    ra.acc = H.acc;
    ra.words = H.words;
    ra.naggs = (int)n;
    dfmi::gb::EmitArgs ea{};
    for (size_t j = 0; j < n; ++j) {
        ra.off[j] = H.off[j];
        const int t = st->aggs[j]->arg.type;
        ra.kind[j] = st->aggs[j]->fn == DFMI_AGG_SUM && is_float_type(t) ? (t == DFMI_TYPE_FLOAT32 ? 2 : 1) : 0;
        ea.fn[j] = st->aggs[j]->fn;
        ea.atype[j] = t;
        ea.rtype[j] = st->aggs[j]->ret_type;
    }
    ra.ngroups = ng;
    ra.out = (unsigned long long*)hd_buf(H, kDrainBuf + 3, ng * (1 + 4 * n) * 8);
    HIP_TRY(dfmi::gb::launch_round(ra, stream));
    unsigned* dnull = (unsigned*)hd_buf(H, kDrainBuf, ng * 4);
    unsigned long long* dkw = (unsigned long long*)hd_buf(H, kDrainBuf + 1, ng * 8);
    unsigned* dklen = (unsigned*)hd_buf(H, kDrainBuf + 2, ng * 4);
    HIP_TRY(dfmi::gb::launch_compact(H.t, 1, dnull, dkw, dklen, stream));
    ea.rec = ra.out;
    ea.knull = dnull;
    ea.kw = dkw;
    ea.ngroups = ng;
    ea.ktype = st->keys[0].type;
    ea.naggs = (int)n;
    ea.keys = hd_buf(H, kEmitBuf, ng * sizeof(dfmi_agg_value));
    ea.values = hd_buf(H, kEmitBuf + 1, ng * n * sizeof(dfmi_agg_value));
    auto* sk = (unsigned long long*)hd_buf(H, kEmitBuf + 2, ng * 8);
    auto* sk2 = (unsigned long long*)hd_buf(H, kEmitBuf + 3, ng * 8);
    auto* sv = (unsigned*)hd_buf(H, kEmitBuf + 4, ng * 4);
    auto* sv2 = (unsigned*)hd_buf(H, kEmitBuf + 5, ng * 4);
    auto* null_at = (unsigned*)hd_buf(H, kEmitBuf + 6, 8);
    size_t tb = 0;
    HIP_TRY(dfmi::gb::launch_emit(ea, sk, sk2, sv, sv2, null_at, nullptr, &tb, stream));
    void* tmp = hd_buf(H, kEmitBuf + 7, tb);
    HIP_TRY(dfmi::gb::launch_emit(ea, sk, sk2, sv, sv2, null_at, tmp, &tb, stream));
    HIP_TRY(hipMemcpyAsync(keys, ea.keys, ng * sizeof(dfmi_agg_value), hipMemcpyDeviceToHost, stream));
    if (n) HIP_TRY(hipMemcpyAsync(values, ea.values, ng * n * sizeof(dfmi_agg_value), hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    st->shown.reset();
    return true;
}

void emit_flat(const dfmi_agg_state* st, const FlatGroups& f, int64_t cap, dfmi_agg_value* keys,
               dfmi_agg_value* values, int64_t* num_groups) {
    *num_groups = (int64_t)f.ng;
    if (*num_groups > cap) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "group capacity too small"};
    if (*num_groups > 0 && (!keys || !values)) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
    const size_t nk = f.nk, n = st->aggs.size();
    auto emit_range = [&](uint64_t i0, uint64_t i1) {
        Partial q;
        for (uint64_t i = i0; i < i1; ++i) {
            const uint32_t g = f.order[i];
            const uint64_t* rec = &f.acc[(size_t)g * f.words];
            for (size_t p = 0; p < nk; ++p) {
                dfmi_agg_value& k = keys[i * nk + p];
                const int kt = st->keys[p].type;
                const bool null = (f.knull[g] >> p) & 1;
                k.type = kt;
                k.is_null = null ? 1 : 0;
                k.bits = null || kt == DFMI_TYPE_UTF8 ? 0
                                                      : (kt == DFMI_TYPE_BOOLEAN ? f.kw[g * nk + p] : narrow_int(f.kw[g * nk + p], kt));
                k.count = (int64_t)rec[0];
            }
            for (size_t j = 0; j < n; ++j) {
                q.flags = q.key = q.isum = 0;  // (rec_partial sets count and, for a float SUM, every digit)
                rec_partial(st, f, rec, j, q);
                if (f.rounded && st->aggs[j]->fn == DFMI_AGG_SUM && is_float_type(st->aggs[j]->arg.type)) {
                    const uint64_t* w = rec + f.off[j];
                    Rounded r;
                    memcpy(&r.v, &w[2], 8);
                    r.zero = (w[1] & dfmi::gb::kRoundZero) != 0;
                    values[i * n + j] = finish_normalized(*st->aggs[j], q, &r);
                } else {
                    values[i * n + j] = finish_normalized(*st->aggs[j], q);
                }
            }
        }
    };
    parallel_ranges(f.ng, 32768, emit_range);  // (a thread's start costs more than ~10^4 groups' emission)
}

void emit_key_bytes_flat(const FlatGroups& f, int part, int32_t* offsets, int64_t num_offsets, uint8_t* data,
                         int64_t data_capacity, int64_t* data_length) {
    const size_t nk = f.nk;
    int64_t total = 0;
    for (uint64_t g = 0; g < f.ng; ++g)
        if (!((f.knull[g] >> part) & 1)) total += f.klen[g * nk + part];
    *data_length = total;
    if (total > 0x7fffffffll) throw Fail{DFMI_ERR_CAPACITY, "Utf8 group keys of 2^31 bytes or more"};
    if (num_offsets < (int64_t)f.ng + 1 || data_capacity < total)
        throw Fail{DFMI_ERR_CAPACITY, "key offsets / bytes capacity too small"};
    if (!offsets || (total && !data)) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
    int64_t pos = 0;
    offsets[0] = 0;
    for (uint64_t i = 0; i < f.ng; ++i) {
        const uint32_t g = f.order[i];
        if (!((f.knull[g] >> part) & 1)) {
            const unsigned len = f.klen[g * nk + part];
            if (len) memcpy(data + pos, f.arena.data() + f.kw[g * nk + part], len);
            pos += len;
        }
        offsets[i + 1] = (int32_t)pos;
    }
}

// Every group the state holds (window, hash table, host merges) in st->groups.
void collect_groups(dfmi_context* ctx, dfmi_agg_state* st) {
    flush_groups(ctx, st);
    drain_hashed(ctx, st);
    st->shown.reset();
}

// Groups in key order as dfmi_agg_state_finish_grouped outputs them:
// keys[g * nkeys + p], values[g * n + j].
void emit_groups(const GroupMap& groups, const std::vector<int>& ktypes, const dfmi_aggregate* const* aggs, size_t n,
                 int64_t cap, dfmi_agg_value* keys, dfmi_agg_value* values, int64_t* num_groups) {
    *num_groups = (int64_t)groups.size();
    if (*num_groups > cap) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "group capacity too small"};
    if (*num_groups > 0 && (!keys || !values)) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
    const size_t nk = ktypes.size();
    int64_t g = 0;
    for (const auto& [hk, v] : groups) {
        for (size_t p = 0; p < nk; ++p) {
            dfmi_agg_value& k = keys[g * nk + p];
            const int kt = ktypes[p];
            const KeyPart& kp = hk.p[p];
            k.type = kt;
            k.is_null = kp.null ? 1 : 0;
            k.bits = kp.null || kt == DFMI_TYPE_UTF8 ? 0 : (kt == DFMI_TYPE_BOOLEAN ? kp.bits : narrow_int(kp.bits, kt));
            k.count = (int64_t)v[n].count;  // the group's selected rows
        }
        for (size_t j = 0; j < n; ++j) values[g * n + j] = finish_one(*aggs[j], v[j]);
        ++g;
    }
}

// The Utf8 bytes of key part `part` of `groups`, in order, as a BinaryArray.
void emit_key_bytes(const GroupMap& groups, int part, int32_t* offsets, int64_t num_offsets, uint8_t* data,
                    int64_t data_capacity, int64_t* data_length) {
    int64_t total = 0;
    for (const auto& kv : groups) total += (int64_t)kv.first.p[part].s.size();
    *data_length = total;
    if (total > 0x7fffffffll) throw Fail{DFMI_ERR_CAPACITY, "Utf8 group keys of 2^31 bytes or more"};
    if (num_offsets < (int64_t)groups.size() + 1 || data_capacity < total)
        throw Fail{DFMI_ERR_CAPACITY, "key offsets / bytes capacity too small"};
    if (!offsets || (total && !data)) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
    int64_t g = 0, pos = 0;
    offsets[0] = 0;
    for (const auto& kv : groups) {
        const std::string& s = kv.first.p[part].s;
        if (!s.empty()) memcpy(data + pos, s.data(), s.size());
        pos += (int64_t)s.size();
        offsets[++g] = (int32_t)pos;
    }
}

// Serialised per-group partials (multi-GPU GROUP BY): a header, then per group
// per key part {null, bits, Utf8 length} and the part's bytes (padded to 8),
// then its n + 1 partials (aggregates, then the row count).
struct GroupedHdr {
    uint64_t magic, ngroups, naggs, nkeys;
    int64_t key_types[dfmi::gb::kMaxKeys];
};
constexpr uint64_t kGroupedMagic = 0x32505247494d4644ull;  // "DFMIGRP2"

size_t grouped_bytes(const GroupMap& groups, size_t n) {
    size_t b = sizeof(GroupedHdr);
    for (const auto& kv : groups) {
        b += (n + 1) * sizeof(Partial);
        for (const KeyPart& k : kv.first.p) b += 24 + (k.s.size() + 7) / 8 * 8;
    }
    return b;
}

void serialize_groups(const GroupMap& groups, const std::vector<int>& ktypes, size_t n, uint8_t* p) {
    GroupedHdr h{};
    h.magic = kGroupedMagic;
    h.ngroups = groups.size();
    h.naggs = n;
    h.nkeys = ktypes.size();
    for (size_t i = 0; i < ktypes.size(); ++i) h.key_types[i] = ktypes[i];
    memcpy(p, &h, sizeof h);
    p += sizeof h;
    for (const auto& [hk, v] : groups) {
        for (const KeyPart& k : hk.p) {
            const uint64_t rec[3] = {k.null ? 1ull : 0ull, k.bits, (uint64_t)k.s.size()};
            memcpy(p, rec, 24);
            p += 24;
            if (!k.s.empty()) memcpy(p, k.s.data(), k.s.size());
            const size_t pad = (k.s.size() + 7) / 8 * 8;
            memset(p + k.s.size(), 0, pad - k.s.size());
            p += pad;
        }
        memcpy(p, v.data(), (n + 1) * sizeof(Partial));
        p += (n + 1) * sizeof(Partial);
    }
}

// Every shard's serialised partials merged into `groups` (key types checked).
void merge_serialized(GroupMap& groups, std::vector<int>& ktypes, const dfmi_aggregate* const* aggs, size_t n,
                      const void* const* partials, const int64_t* sizes, int nparts) {
    for (int r = 0; r < nparts; ++r) {
        const uint8_t* p = (const uint8_t*)partials[r];
        GroupedHdr h;
        if (!p || sizes[r] < (int64_t)sizeof h) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "bad grouped partial"};
        memcpy(&h, p, sizeof h);
        if (h.magic != kGroupedMagic || h.naggs != (uint64_t)n || h.nkeys < 1 || h.nkeys > (uint64_t)dfmi::gb::kMaxKeys)
            throw Fail{DFMI_ERR_INVALID_ARGUMENT, "bad grouped partial"};
        std::vector<int> kt(h.key_types, h.key_types + h.nkeys);
        if (!ktypes.empty() && kt != ktypes) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "bad grouped partial"};
        ktypes = kt;
        const uint8_t* end = p + sizes[r];
        p += sizeof h;
        for (uint64_t g = 0; g < h.ngroups; ++g) {
            HKey hk;
            hk.p.resize(h.nkeys);
            for (uint64_t q = 0; q < h.nkeys; ++q) {
                uint64_t rec[3];
                if (end - p < 24) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "bad grouped partial"};
                memcpy(rec, p, 24);
                p += 24;
                const size_t pad = (size_t)(rec[2] + 7) / 8 * 8;
                if ((size_t)(end - p) < pad) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "bad grouped partial"};
                KeyPart& k = hk.p[q];
                if (rec[0]) {
                    k.null = true;
                } else if (kt[q] == DFMI_TYPE_UTF8) {
                    k.s.assign((const char*)p, (size_t)rec[2]);
                } else {
                    k = fixed_part(kt[q], rec[1]);
                }
                p += pad;
            }
            if ((size_t)(end - p) < (n + 1) * sizeof(Partial)) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "bad grouped partial"};
            std::vector<Partial> parts(n + 1);
            memcpy(parts.data(), p, (n + 1) * sizeof(Partial));
            p += (n + 1) * sizeof(Partial);
            merge_group(group_entry(groups, std::move(hk), n), parts, aggs, n);
        }
    }
}

std::vector<int> key_types(const dfmi_agg_state* st) {
    std::vector<int> t;
    for (const dfmi_program& k : st->keys) t.push_back(k.type);
    return t;
}

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

extern "C" int32_t dfmi_agg_state_create_grouped_multi(dfmi_context* ctx, const dfmi_program* const* keys,
                                                       int32_t num_keys, const dfmi_aggregate* const* aggs, int32_t n,
                                                       dfmi_agg_state** out, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    dfmi_agg_state* st = nullptr;
    try {
        if (!ctx || !out || !keys || num_keys <= 0 || n <= 0 || !aggs) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "bad argument"};
        if (num_keys > dfmi::gb::kMaxKeys)
            throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "device program limit: more than 4 GROUP BY expressions"};
        for (int p = 0; p < num_keys; ++p) {
            if (!keys[p]) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL key"};
            const int kt = keys[p]->type;
            if (kt != DFMI_TYPE_BOOLEAN && !is_numeric_type(kt) && kt != DFMI_TYPE_UTF8)
                throw Fail{DFMI_ERR_NOT_IMPLEMENTED, std::string("GROUP BY over ") + type_debug(kt)};
        }
        if (n > dfmi::gb::kMaxAggs) throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "device program limit: more than 15 grouped aggregates"};
        st = new dfmi_agg_state();
        st->device = ctx->device;
        st->grouped = true;
        for (int p = 0; p < num_keys; ++p) st->keys.push_back(*keys[p]);
        st->key = *keys[0];
        const int kt = st->key.type;
        for (int j = 0; j < n; ++j) {
            if (!aggs[j]) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL aggregate"};
            st->aggs.push_back(aggs[j]);
        }
        HIP_TRY(hipSetDevice(ctx->device));
        // one Boolean / integer key: the window kernel (16 consecutive values
        // per batch, more through the hash table); anything else: the hash table
        if (num_keys == 1 && (kt == DFMI_TYPE_BOOLEAN || !host_keyed(kt))) {
            st->gslots = kt == DFMI_TYPE_BOOLEAN ? 3 : 17;  // false, true / 16 consecutive values; + null
            const size_t na = (size_t)n + 1;
            st->acc_words = (size_t)kAggCopies * st->gslots * na * kAggWords;
            std::vector<uint64_t> init(st->acc_words, 0);
            for (size_t cg = 0; cg < (size_t)kAggCopies * st->gslots; ++cg)
                for (int j = 0; j < n; ++j)
                    if (aggs[j]->fn == DFMI_AGG_MIN) init[(cg * na + j) * kAggWords + 2] = ~0ull;
            HIP_TRY(hipMalloc((void**)&st->acc, st->acc_words * 8));
            HIP_TRY(hipMemcpyAsync(st->acc, init.data(), st->acc_words * 8, hipMemcpyHostToDevice, ctx->stream));
            HIP_TRY(hipStreamSynchronize(ctx->stream));
            st->init = std::move(init);
            if (kt != DFMI_TYPE_BOOLEAN) {
                dfmi_error e2{};
                for (int i = 0; i < 2; ++i)
                    if (dfmi_compile_aggregate(i ? "MAX" : "MIN", keys[0], kt, DFMI_FLAG_EXT_AGGREGATE, &st->mm[i], &e2) !=
                        DFMI_OK)
                        throw Fail{e2.code, e2.message};
                const dfmi_aggregate* mm[2] = {st->mm[0], st->mm[1]};
                if (dfmi_agg_state_create(ctx, mm, 2, &st->mm_state, &e2) != DFMI_OK) throw Fail{e2.code, e2.message};
            }
        }
        *out = st;
        return DFMI_OK;
    } catch (const Fail& f) {
        dfmi_agg_state_free(st);
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

extern "C" int32_t dfmi_agg_state_create_grouped(dfmi_context* ctx, const dfmi_program* key,
                                                 const dfmi_aggregate* const* aggs, int32_t n, dfmi_agg_state** out,
                                                 dfmi_error* err) {
    if (!key) {
        set_err(err, DFMI_ERR_INVALID_ARGUMENT, "bad argument");
        return DFMI_ERR_INVALID_ARGUMENT;
    }
    const dfmi_program* keys[1] = {key};
    return dfmi_agg_state_create_grouped_multi(ctx, keys, 1, aggs, n, out, err);
}

extern "C" int32_t dfmi_agg_state_num_keys(const dfmi_agg_state* st) {
    return st && st->grouped ? (int32_t)st->keys.size() : 0;
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
        {
            const auto t0 = std::chrono::steady_clock::now();
            if (finish_device(ctx, st, cap, keys, values, num_groups)) {
                if (getenv("DFMI_DIAG") && getenv("DFMI_FINISH_PROFILE"))
                    fprintf(stderr, "[dfmi finish] %lld groups on the device: %.1f us\n", (long long)*num_groups,
                            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
                return DFMI_OK;
            }
        }
        if (finish_flat(ctx, st)) {
            const auto t0 = std::chrono::steady_clock::now();
            emit_flat(st, *st->flat, cap, keys, values, num_groups);
            if (getenv("DFMI_DIAG") && getenv("DFMI_FINISH_PROFILE"))
                fprintf(stderr, "[dfmi finish] emit %.1f us\n",
                        std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
            return DFMI_OK;
        }
        collect_groups(ctx, st);
        emit_groups(st->groups, key_types(st), st->aggs.data(), st->aggs.size(), cap, keys, values, num_groups);
        return DFMI_OK;
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

extern "C" int32_t dfmi_agg_state_group_keys_utf8_part(const dfmi_agg_state* st, int32_t part, int32_t* offsets,
                                                       int64_t num_offsets, uint8_t* data, int64_t data_capacity,
                                                       int64_t* data_length, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    try {
        if (!st || !data_length) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        if (st->failed) {
            if (err) *err = st->failure;
            return st->failure.code;
        }
        if (!st->grouped || part < 0 || part >= (int32_t)st->keys.size() || st->keys[part].type != DFMI_TYPE_UTF8)
            throw Fail{DFMI_ERR_INVALID_ARGUMENT, "not a GROUP BY state over a Utf8 key"};
        if (!st->shown && st->flat)
            emit_key_bytes_flat(*st->flat, part, offsets, num_offsets, data, data_capacity, data_length);
        else
            emit_key_bytes(st->shown ? *st->shown : st->groups, part, offsets, num_offsets, data, data_capacity,
                           data_length);
        return DFMI_OK;
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

extern "C" int32_t dfmi_agg_state_group_keys_utf8(const dfmi_agg_state* st, int32_t* offsets, int64_t num_offsets,
                                                  uint8_t* data, int64_t data_capacity, int64_t* data_length,
                                                  dfmi_error* err) {
    return dfmi_agg_state_group_keys_utf8_part(st, 0, offsets, num_offsets, data, data_capacity, data_length, err);
}

extern "C" int32_t dfmi_agg_state_reset(dfmi_context* ctx, dfmi_agg_state* st, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    try {
        if (!ctx || !st) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        HIP_TRY(hipSetDevice(ctx->device));
        if (st->acc)
            HIP_TRY(hipMemcpyAsync(st->acc, st->init.data(), st->acc_words * 8, hipMemcpyHostToDevice, ctx->stream));
        if (HashDev* H = st->hd) {  // an empty table of the same size
            HIP_TRY(hipMemsetAsync(H->t.ctl, 0, H->cap * 8, ctx->stream));
            HIP_TRY(hipMemsetAsync(H->hdr, 0, sizeof(dfmi::gb::Hdr), ctx->stream));
            HIP_TRY(dfmi::gb::launch_init(H->acc, H->pattern, H->words, 0, H->ngroups, ctx->stream));
            H->ngroups = 0;
            H->rows_since_norm = 0;
        }
        st->failed = false;
        st->failure = dfmi_error{};
        st->index.clear();
        st->groups.clear();
        if (st->flat) st->spare_flat = std::move(st->flat);
        st->shown.reset();
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
    (void)hipSetDevice(st->device);
    if (st->acc) (void)hipFree(st->acc);
    free_hashdev(st->hd);
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
        if (st->grouped) unflatten(st);  // a finish's flat groups back in the map before more rows merge
        Unsliced us_;  // sliced arrays (arrow offsets): offset-0 views / shifted bitmaps (slice.cpp)
        if (any_offset(in, 1)) {
            HIP_TRY(hipSetDevice(ctx->device));
            in = unslice(in, 1, us_, true, ctx->stream);
        }
        if (st->grouped && (!st->acc || (getenv("DFMI_DIAG") && getenv("DFMI_GROUP_HOST")))) {
            // several keys, a float or Utf8 key: the keys and the arguments
            // through one fused Selection + Projection pass, then the device
            // hash table (or, diagnostics, the host merge)
            HIP_TRY(hipSetDevice(ctx->device));
            if (in->num_rows > 0) {
                if (st->acc) flush_groups(ctx, st);
                if (getenv("DFMI_DIAG") && getenv("DFMI_GROUP_HOST")) group_batch_on_host(ctx, st, pred, in, flags);
                else group_batch_hashed(ctx, st, pred, in, flags);
            }
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
                        // wider than the device window: the hash table (its
                        // fused pass raises the same first error in the same
                        // evaluation order as the grouped kernel would)
                        flush_groups(ctx, st);
                        group_batch_hashed(ctx, st, pred, in, flags);
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
        HIP_TRY(hipSetDevice(ctx->device));
        collect_groups(ctx, st);
        return (int64_t)grouped_bytes(st->groups, st->aggs.size());
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
        HIP_TRY(hipSetDevice(ctx->device));
        collect_groups(ctx, st);
        if ((size_t)bytes < grouped_bytes(st->groups, st->aggs.size()))
            throw Fail{DFMI_ERR_CAPACITY, "partial buffer too small"};
        serialize_groups(st->groups, key_types(st), st->aggs.size(), (uint8_t*)host_out);
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
        std::vector<int> kt;
        merge_serialized(groups, kt, aggs, (size_t)n, partials, sizes, nparts);
        emit_groups(groups, kt, aggs, (size_t)n, cap, keys, values, num_groups);
        return DFMI_OK;
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

extern "C" int32_t dfmi_agg_merge_grouped_partials_keys_utf8(const dfmi_aggregate* const* aggs, int32_t n,
                                                             const void* const* partials, const int64_t* sizes,
                                                             int32_t nparts, int32_t part, int32_t* offsets,
                                                             int64_t num_offsets, uint8_t* data, int64_t data_capacity,
                                                             int64_t* data_length, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    try {
        if (!aggs || n <= 0 || !partials || !sizes || nparts <= 0 || !data_length)
            throw Fail{DFMI_ERR_INVALID_ARGUMENT, "bad argument"};
        GroupMap groups;
        std::vector<int> kt;
        merge_serialized(groups, kt, aggs, (size_t)n, partials, sizes, nparts);
        if (part < 0 || part >= (int32_t)kt.size() || kt[part] != DFMI_TYPE_UTF8)
            throw Fail{DFMI_ERR_INVALID_ARGUMENT, "not a Utf8 key part"};
        emit_key_bytes(groups, part, offsets, num_offsets, data, data_capacity, data_length);
        return DFMI_OK;
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

// dfmi_shard_agg_finish_grouped's merge (shard.cpp): every rank's partials
// merged into the state's shown groups, so the Utf8 key bytes of the merged
// groups come from dfmi_agg_state_group_keys_utf8* afterwards.
int32_t dfmi_agg_state_show_merged(dfmi_agg_state* st, const void* const* partials, const int64_t* sizes, int32_t nparts,
                                   int64_t cap, dfmi_agg_value* keys, dfmi_agg_value* values, int64_t* num_groups,
                                   dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    try {
        if (!st || !st->grouped || !partials || !sizes || nparts <= 0 || !num_groups)
            throw Fail{DFMI_ERR_INVALID_ARGUMENT, "bad argument"};
        auto merged = std::make_shared<GroupMap>();
        std::vector<int> kt = key_types(st);
        merge_serialized(*merged, kt, st->aggs.data(), st->aggs.size(), partials, sizes, nparts);
        emit_groups(*merged, kt, st->aggs.data(), st->aggs.size(), cap, keys, values, num_groups);
        st->shown = merged;
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
// Diagnostics: grouped batches accumulated by the bucketed passes (groupby.h) in this process.
extern "C" long dfmi_internal_group_bucketed_batches() { return g_bucketed_batches.load(); }

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
        st.keys.push_back(*key);
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
