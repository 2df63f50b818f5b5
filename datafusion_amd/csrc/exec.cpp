// dfmi_filter_project: host side of the fused Selection + Projection pass.
//
// Plans the pass from the compiled predicate / projections (dfmi_program IR):
// static errors in the reference's evaluation order, output metadata, which
// input columns the kernel loads (predicate columns for every row,
// projection-only columns only where selected); gets the query kernel from
// the query compiler (jit.cpp), launches it, and maps device error words back
// to the reference's errors (FilterRelation::next filter.rs:46-72, filter()
// filter.rs:80-111, ProjectRelation::next projection.rs:45-66).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <new>
#include <string>
#include <vector>

#include "dfmi_program.h"
#include "jit.h"
#include "jit_skeleton.hip"
#include "../../include/dfmi_datasource.h"

namespace dfmi {
hipError_t launch_pack_bools(const uint8_t* bytes, uint8_t* bits, const unsigned long long* count,
                             long long max_rows, hipStream_t st);
hipError_t launch_utf8_copy_rows(const int32_t* offs, const int32_t* spos, const uint8_t* src, uint8_t* out,
                                 const unsigned long long* totals, int chan, long long cap, long long max_rows,
                                 hipStream_t st);
}  // namespace dfmi

using namespace dfmi;

#include "exec_internal.h"
#include "batch_stage.h"
#include "slice.h"

using namespace dfmi::xi;

namespace {

// Everything about one call that does not need the device: static errors,
// output metadata, the jit plan and the column slot tables.
struct Built {
    Err se;
    jit::Plan plan;
    jit::Launch X;
    bool any_kernel_out = false;
    int64_t n_tiles = 0;
    bool low_sel = false;  // in: this query shape selected few rows last time (dfmi_context::sel_hint)
    bool high_sel = false;  // in: ... or at least kLowSel of them
    bool ring_ok = false;  // in: ... selected many rows with short Utf8 strings (the ring-staged gather)
    bool long_utf8 = false;  // in: ... selected long Utf8 strings (the long per-lane fallback copy)
};

// The ring-staged Utf8 gather stages every byte of a 256-row step (not only
// the selected strings), into slots of kRingSlot 16-byte chunks: chosen when
// the same query shape's previous large batch selected at least kRingSel of
// its rows and its selected strings averaged at most kRingLen bytes (a step
// then fits a slot with ~10% to spare; a longer step copies per lane).
constexpr int kRingSlot = 256;
constexpr double kRingSel = 0.15;
constexpr double kRingLen = 14.5;
constexpr double kLongLen = 24.0;  // selected Utf8 bytes per row from which slices tend to overflow the 2 KiB stage
constexpr bool kRingDefault = false;

// A numeric predicate over a large batch that selects few rows runs the
// sub-tile kernel: M sub-tiles of BLOCK * K rows share one scan + look-back
// (one look-back per 16,384 rows instead of per 4,096), the predicate pass
// keeps only selection ballots, and the output pass reloads just the columns
// the outputs read, for the selected rows (jit.cpp "M sub-tiles"). Chosen
// from the selectivity the same query shape had on its previous large batch
// on this context (below kLowSel); the first call, and any call after a
// batch selected more, runs the one-tile kernel, which keeps every loaded
// value in registers across the look-back.
constexpr int64_t kSubtileMinRows = (int64_t)1 << 22;
constexpr double kLowSel = 0.04;

void build_plan_impl(const dfmi_program* pred, const dfmi_program* const* projs, int32_t np, const dfmi_batch* in,
                     dfmi_out_column* outs, uint32_t flags, Built& B);

// A device limit (NotImplemented) found while planning is reported only when
// the plan raises none of the reference's own errors first: those come
// earlier in its evaluation order (and stand for what it would report).
void build_plan(const dfmi_program* pred, const dfmi_program* const* projs, int32_t np, const dfmi_batch* in,
                dfmi_out_column* outs, uint32_t flags, Built& B) {
    try {
        build_plan_impl(pred, projs, np, in, outs, flags, B);
    } catch (const Fail& f) {
        if (f.code == DFMI_ERR_NOT_IMPLEMENTED && B.se.set) throw Fail{B.se.code, B.se.msg};
        throw;
    }
}

void build_plan_impl(const dfmi_program* pred, const dfmi_program* const* projs, int32_t np, const dfmi_batch* in,
                     dfmi_out_column* outs, uint32_t flags, Built& B) {
    Err& se = B.se;
    jit::Plan& plan = B.plan;
    jit::Launch& X = B.X;
    bool& any_kernel_out = B.any_kernel_out;
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
    if (base >= (1 << 19)) throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "device program limit: expressions too long"};

    // ---- output plan
    const int nout = np > 0 ? np : ncols;
    if (nout > 16) throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "device program limit: too many output columns"};
    plan.pred = pred;
    plan.outs.resize(nout);
    X.in = in;
    for (int o = 0; o < nout; ++o) {
        dfmi_out_column& oc = outs[o];
        const dfmi_program* p = np > 0 ? projs[o] : nullptr;
        const IrNode* root = p ? &p->ir[p->root] : nullptr;
        const bool is_col = !p || root->kind == IR_COL;
        const int col = p ? root->col : o;
        oc.type = p ? p->type : in->columns[o].type;
        oc.passthrough_column = -1;
        oc.length = 0;
        oc.null_count = 0;
        oc.data_length = 0;
        jit::OutSpec& os = plan.outs[o];
        os.out_type = oc.type;
        if (is_col && !pred) {  // Arc clone of the input column (expression.rs:274)
            const dfmi_column& c = in->columns[col];
            oc.passthrough_column = col;
            oc.length = n;
            oc.null_count = c.validity ? c.null_count : 0;
            continue;
        }
        if (is_col) {
            const int ct = in->columns[col].type;
            if (!gatherable(ct, flags)) continue;  // error raised at ordinal P+1
            if (ct == DFMI_TYPE_UTF8) {
                if (!oc.offsets || !oc.data) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "Utf8 output buffers are NULL"};
                os.kind = jit::OutSpec::UTF8;
            } else {
                if (!oc.values) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "output values pointer is NULL"};
                os.kind = jit::OutSpec::GATHER;
            }
            os.col = col;
            any_kernel_out = true;
            continue;
        }
        if (oc.type == DFMI_TYPE_UTF8) throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "device path: Utf8-valued projection"};
        if (!oc.values) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "output values pointer is NULL"};
        os.kind = jit::OutSpec::EXPR;
        os.prog = p;
        os.ord_base = proj_base[o];
        os.nullable = pred && jit::may_introduce_nulls(p);
        if (os.nullable && !oc.validity)
            throw Fail{DFMI_ERR_INVALID_ARGUMENT, "output validity pointer is NULL (the projection can produce nulls)"};
        any_kernel_out = true;
    }

    // ---- column slots: predicate columns first, then projection-only ones
    auto reg_num = [&](int col, std::vector<int>& phase) {
        for (size_t i = 0; i < X.num_cols.size(); ++i)
            if (X.num_cols[i] == col) return;
        X.num_cols.push_back(col);
        phase.push_back((int)X.num_cols.size() - 1);
    };
    auto reg_utf8 = [&](int col) {
        for (size_t i = 0; i < X.utf8_cols.size(); ++i)
            if (X.utf8_cols[i] == col) return (int)i;
        X.utf8_cols.push_back(col);
        return (int)X.utf8_cols.size() - 1;
    };
    auto reg_prog = [&](const dfmi_program* p, std::vector<int>& phase) {
        for (const IrNode& nd : p->ir) {
            if (nd.kind != IR_COL) continue;
            if (nd.type == DFMI_TYPE_UTF8) reg_utf8(nd.col);
            else if (jit::type_width(nd.type) || nd.type == DFMI_TYPE_BOOLEAN) reg_num(nd.col, phase);
        }
    };
    if (pred) reg_prog(pred, X.pred_slots);
    for (int o = 0; o < nout; ++o) {
        const jit::OutSpec& os = plan.outs[o];
        if (os.kind == jit::OutSpec::GATHER) reg_num(os.col, X.proj_slots);
        else if (os.kind == jit::OutSpec::EXPR) reg_prog(os.prog, X.proj_slots);
        else if (os.kind == jit::OutSpec::UTF8) X.utf8_outs.push_back({o, reg_utf8(os.col)});
    }
    if ((int)X.num_cols.size() > kArgCols || X.utf8_cols.size() > (size_t)kArgUtf8)
        throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "device program limit: too many input columns"};
    // rows per thread: keep the tile's column data resident in VGPRs (a
    // Utf8 column holds its offsets per row; a kernel gathering many Utf8
    // columns at K = 8 is also a ~35 s hipRTC compile -- 11 Utf8 outputs:
    // 35 / 15 / 6.6 s at K = 8 / 4 / 2)
    const size_t nload = X.num_cols.size() + X.utf8_cols.size();
    X.BLOCK = 512;
    X.K = nload <= 4 ? 8 : (nload <= 8 ? 4 : 2);
    // a predicate over Utf8 columns only reads ~4 B/row of offsets: its tiles
    // are latency-bound, and 4-wave blocks keep more of them resident
    // (C3 equality 4.94 -> 4.53 ms)
    // (... unless the same query selected >= kLowSel of a large batch last
    // time -- `s != 'w17...'`, 99.9%: the one-tile kernel with the LDS-image
    // gather below, 2.37 -> 1.63 ms per C3 batch; profiles/r05/c3_ne_probe*.log)
    if (pred && X.pred_slots.empty() && !X.utf8_cols.empty() && !B.high_sel) {
        X.BLOCK = 256;
        // ... and are latency-bound on the look-back: a 16-predecessor poll
        // window and 8 waves/SIMD (a few spilled registers) measured faster
        // (C3 equality 0.826 -> 0.675 ms per 1.25e8-row batch)
        X.window = 16;
        X.waves_per_eu = 8;
        // ... and M sub-tiles share one look-back, their output pass two
        // slices per wave at a time: 60 VGPRs, no spills at 8 waves/SIMD
        // (DESIGN.md §4 "Sub-tiles")
        X.M = 8;
        X.KO = 2;
    } else {
        // Utf8 outputs of a numeric predicate: the LDS-image gather (the
        // binary-search emitter's smaller LDS footprint only pays where few
        // rows are selected)
        X.gather = 4;
        if (!X.utf8_outs.empty() && pred) {
            // latency-bound gather: a 2 KiB staging arena per wave, 256-thread
            // blocks and a soft occupancy hint (a shape that would spill at it
            // is compiled again without it)
            X.arena = 128;
            X.waves_soft = true;
            // ... 61 VGPRs since the light fallback copy: 8 waves/SIMD fit
            // without spills (256-thread blocks: 1.045 -> 1.021 ms per C3
            // batch; 7 waves and 72 VGPRs were the budget of utf8_copy's
            // 8-word chunks; profiles/r05/c3_combo.log) ...
            X.waves_per_eu = 8;
            // ... where 512-thread blocks (4096-row tiles: half the look-backs)
            // beat 256 with a 12-predecessor window: 1.076 -> 1.032-1.042 ms
            // same box (1024: 1.087-1.096; windows 4 / 8 / 12 / 32 at 512:
            // 1.077 / 1.036-1.042 / 1.032 / 1.061; profiles/r05/c3_block_ab.log)
            X.BLOCK = 512;
            X.window = 12;
            // ... and where the last large batch selected long strings (slices
            // over the stage), the per-lane fallback with 64 bytes in flight
            // and no occupancy hint (81 VGPRs): 40-200-byte strings 1.29 ->
            // 0.79 ms per 1e7 rows (profiles/r05/long_utf8_copy.log)
            if (B.long_utf8) {
                X.long_copy = 1;
                X.waves_per_eu = 0;
            }
            // ... at high selectivity, the ring-staged gather (one loader wave)
            // when kRingDefault: same-box A/B (profiles/r05/c3_ring_ab.log) put it
            // within the box's spread of the per-wave gather (1.135-1.153 vs
            // 1.138-1.143 ms per C3 batch), so it stays a diagnostic variant
            if (kRingDefault && B.ring_ok && X.utf8_outs.size() == 1 && !X.pred_slots.empty()) {
                X.ring = kRingSlot;
                X.BLOCK = 256;  // a ring step = one 64-row slice per wave of 4
                X.window = 16;
            }
        } else if (pred && B.low_sel && !X.pred_slots.empty() && X.utf8_cols.empty() && n >= kSubtileMinRows) {
            // a numeric predicate that selected < 4% last time: M sub-tiles
            // share one look-back, a sparse output pass re-reads only the
            // selected rows (same-box A/B, profiles/r04/ab_subtiles*.log: C2
            // s = 1% (2 predicate columns) 4.17 / 3.12 / 3.00 / 3.03 ms and C4
            // (4) 3.01 / 2.76 / 2.60 / 2.51 ms at M = 1 / 8 / 4 / 2: more
            // predicate registers per sub-tile, fewer sub-tiles)
            X.BLOCK = 256;
            X.M = X.pred_slots.size() >= 3 ? 2 : 4;
            X.KO = 2;  // the (rare) dense output pass two slices at a time: fewer registers
        }
    }
    // diagnostic knobs (tools/*): read only when DFMI_DIAG is set -- a dozen
    // getenv scans per call would cost the 1024-row batch path microseconds
    const bool diag = getenv("DFMI_DIAG") != nullptr;
    if (diag) {
        if (const char* kk = getenv("DFMI_ROWS_PER_THREAD")) X.K = atoi(kk);
        if (const char* bb = getenv("DFMI_BLOCK")) X.BLOCK = atoi(bb);
        if (const char* ww = getenv("DFMI_WAVES_PER_EU")) X.waves_per_eu = atoi(ww);
        // look-back / tile-order variants
        if (const char* e = getenv("DFMI_LOOKBACK_R")) X.R = std::max(1, std::min(16, atoi(e)));
        if (const char* e = getenv("DFMI_LOOKBACK_SLEEP")) X.sleep = std::max(0, std::min(127, atoi(e)));
        if (const char* e = getenv("DFMI_LOOKBACK_SPREAD")) X.spread = std::max(1, std::min(64, atoi(e)));
        if (const char* e = getenv("DFMI_LOOKBACK_W")) X.window = std::max(1, std::min(64, atoi(e)));
        if (const char* e = getenv("DFMI_NT")) X.nt = atoi(e) & 3;
        if (const char* e = getenv("DFMI_UTF8_PRESTAGE")) X.prestage = atoi(e) & 3;  // 2: not the look-back wave
        if (const char* e = getenv("DFMI_GATHER_PHASES")) X.gather_phases = atoi(e) & 1;
        if (const char* e = getenv("DFMI_UTF8_GATHER")) X.gather = atoi(e) % 7;  // 2 = serial, 3 = two-pass, 4 = LDS image, 5 = marker scan, 6 = direct
        if (const char* e = getenv("DFMI_UTF8_DIRECT_GROUP")) X.direct_grp = atoi(e);
        if (const char* e = getenv("DFMI_LATE_PROJ")) X.late_proj = atoi(e) & 1;
        if (const char* e = getenv("DFMI_PROJ_DENSE")) X.proj_dense = atoi(e) & 1;
        if (const char* e = getenv("DFMI_TICKET")) X.ticket = atoi(e) & 1;  // ticket-ordered tiles from the start
        if (const char* e = getenv("DFMI_UTF8_EARLY")) X.early = atoi(e) & 1;
        if (const char* e = getenv("DFMI_LIGHT_COPY")) X.light_copy = atoi(e) & 1;
        if (const char* e = getenv("DFMI_LONG_COPY")) X.long_copy = atoi(e) & 3;  // 1: per lane, 2: wave-cooperative
        if (const char* e = getenv("DFMI_UTF8_EQ_DENSE")) {  // chunks of the per-wave arena (dense equality A/B)
            X.eq_dense = std::max(0, std::min(1024, atoi(e)));
            if (X.eq_dense) X.waves_per_eu = 0;  // LDS-limited occupancy: no register hint
        }
        if (const char* e = getenv("DFMI_UTF8_EQ_REG")) {  // register-resident dense equality: G slices per round
            const int g = atoi(e);
            if (g == 1 || g == 2 || g == 4 || g == 8) X.eq_dense = X.K % g == 0 ? -g : 0;
        }
        if (const char* e = getenv("DFMI_UTF8_RING"))  // 0: off; > 0: on (slot chunks) where it applies
            if (pred && X.utf8_outs.size() == 1 && !X.pred_slots.empty() && X.M == 1) {
                X.ring = atoi(e) > 1 ? atoi(e) : (atoi(e) == 1 ? kRingSlot : 0);
                if (X.ring) {  // a step = one 64-row slice per wave of 4
                    X.BLOCK = 256;
                    X.window = 16;
                }
            }
        if (const char* e = getenv("DFMI_SUBTILES"))
            if (X.pred_slots.empty() && !X.utf8_cols.empty()) X.M = std::max(1, std::min(32, atoi(e)));
        // the numeric sub-tile kernel at any size (parity tests, A/B runs)
        // (1: the one-tile kernel even where the selectivity hint picks sub-tiles)
        if (const char* e = getenv("DFMI_NUMERIC_SUBTILES"))
            if (pred && !X.pred_slots.empty() && X.utf8_cols.empty()) {
                X.BLOCK = atoi(e) > 1 ? 256 : 512;
                X.M = std::max(1, std::min(8, atoi(e)));
                X.KO = X.M > 1 ? 2 : 0;
            }
        if (const char* e = getenv("DFMI_OUT_SLICES")) X.KO = atoi(e);
        if (const char* e = getenv("DFMI_SUBTILE_PREFETCH")) X.prefetch = atoi(e) & 1;
        if (const char* e = getenv("DFMI_SUBTILE_SPARSE")) X.sparse = atoi(e) & 1;
    }

    if (diag)
        if (const char* e = getenv("DFMI_UTF8_ARENA")) X.arena = std::max(128, std::min(1024, atoi(e)));
    if (diag)
        if (const char* e = getenv("DFMI_UTF8_IMAGE")) X.image = std::max(32, std::min(129, atoi(e)));
    if (diag)
        if (const char* e = getenv("DFMI_UTF8_DBUF")) X.dbuf = atoi(e) & 1;
    if (diag)
        if (const char* e = getenv("DFMI_UTF8_ST16")) X.st16 = atoi(e) & 1;
    if (diag)
        if (const char* e = getenv("DFMI_UTF8_PAIRS")) {
            X.pairs = atoi(e) & 1;
            if (X.pairs) X.image = 130;  // two images of 65 chunks
        }
    if (X.dbuf && X.arena < 128) X.dbuf = 0;  // halves of >= 64 chunks (longer spans copy per lane)
    if (X.M == 1 || X.KO == 0) X.KO = X.K;
    if (X.direct_grp < 1) X.direct_grp = 1;
    while (X.K % X.direct_grp || X.KO % X.direct_grp) X.direct_grp >>= 1;  // divides the slices it groups
    if (X.KO < 1 || X.KO > X.K || X.K % X.KO) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "bad tile shape"};
    if (X.K < 1 || X.K > 32 || X.BLOCK < 64 || X.BLOCK > 1024 || X.BLOCK % 64 || X.K * X.M * X.BLOCK / 64 > 256)
        throw Fail{DFMI_ERR_INVALID_ARGUMENT, "bad tile shape"};
    const int64_t tile_rows = (int64_t)X.BLOCK * X.K * X.M;
    const int64_t n_tiles = (n + tile_rows - 1) / tile_rows;
    if (n_tiles > 0x7fffffff) throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "batch too large"};
    // a filtered batch with one Utf8 output packs rows and bytes into one
    // 62-bit look-back word (31 + 31 bits, jit_skeleton.hip tile_scan_publish)
    if (X.utf8_outs.size() == 1 && n >= (int64_t(1) << 31))
        throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "batch too large"};

    B.n_tiles = n_tiles;
}

// The selectivity hint's key: the programs and the batch's column types /
// nullability (a performance hint only: results never depend on it).
uint64_t sel_hint_key(const dfmi_program* pred, const dfmi_program* const* projs, int32_t np, const dfmi_batch* in,
                      uint32_t flags) {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](uint64_t v) { h = (h ^ v) * 1099511628211ull; };
    mix((uint64_t)(uintptr_t)pred);
    mix((uint64_t)np);
    for (int j = 0; j < np; ++j) mix((uint64_t)(uintptr_t)projs[j]);
    mix(flags);
    for (int i = 0; i < in->num_columns; ++i)
        mix((uint64_t)in->columns[i].type << 1 | (in->columns[i].validity && in->columns[i].null_count > 0));
    return h;
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
        if (const char* e = getenv("DFMI_SHARED")) c->shared = atoi(e) != 0;
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

namespace dfmi {
int ctx_device(const dfmi_context* c) { return c->device; }
hipStream_t ctx_stream(const dfmi_context* c) { return c->stream; }
void*& ctx_host_arena(dfmi_context* c) { return c->host_arena; }
uint64_t& ctx_last_err_key(dfmi_context* c) { return c->last_err_key; }
void host_arena_release(dfmi_context* c);
}  // namespace dfmi

extern "C" void dfmi_context_destroy(dfmi_context* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    dfmi::host_arena_release(c);
    if (c->ws) (void)hipFree(c->ws);
    if (c->scratch) (void)hipFree(c->scratch);
    if (c->utf8_src) (void)hipFree(c->utf8_src);
    if (c->host_hdr) (void)hipHostFree(c->host_hdr);
    if (c->bmeta) (void)hipFree(c->bmeta);
    if (c->bhdr) (void)hipFree(c->bhdr);
    if (c->ones) (void)hipFree(c->ones);
    if (c->host_bmeta) (void)hipHostFree(c->host_bmeta);
    if (c->host_bhdr) (void)hipHostFree(c->host_bhdr);
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

extern "C" int32_t dfmi_abi_version(void) { return DFMI_ABI_VERSION; }

extern "C" int32_t dfmi_context_set_shared(dfmi_context* c, int32_t shared) {
    if (!c) return DFMI_ERR_INVALID_ARGUMENT;
    c->shared = shared != 0;
    return DFMI_OK;
}

extern "C" int32_t dfmi_context_set_timing(dfmi_context* c, int32_t enable) {
    if (!c) return DFMI_ERR_INVALID_ARGUMENT;
    c->timing = enable != 0;
    return DFMI_OK;
}

extern "C" int32_t dfmi_last_timing(const dfmi_context* c, double* total_ms, double* main_ms) {
    if (!c || !c->timed) return DFMI_ERR_INVALID_ARGUMENT;
    if (total_ms) *total_ms = c->last_total_ms;
    if (main_ms) *main_ms = c->last_main_ms;
    return DFMI_OK;
}

extern "C" int32_t dfmi_last_error_order(const dfmi_context* c, uint64_t* key) {
    if (!c || !key) return DFMI_ERR_INVALID_ARGUMENT;
    *key = c->last_err_key;
    return DFMI_OK;
}

// Internal test hook: look-back timeouts relaunched on this context.
extern "C" long dfmi_internal_relaunches(const dfmi_context* c) { return c ? c->relaunches : -1; }
// Internal test hook: the hipRTC module cache's size after bounding it to
// `cap` modules (cap > 0; 0 leaves the bound unchanged).
extern "C" int64_t dfmi_internal_jit_cache(int64_t cap) {
    jit::cache_cap(cap > 0 ? (size_t)cap : 0);
    return (int64_t)jit::cache_size();
}

extern "C" const char* dfmi_last_kernel_name(const dfmi_context* c) {
    return c ? c->last_kernel.c_str() : "";
}

extern "C" int32_t dfmi_last_compile_ms(const dfmi_context* c, double* compile_ms) {
    if (!c || !compile_ms) return DFMI_ERR_INVALID_ARGUMENT;
    *compile_ms = c->last_compile_ms;
    return DFMI_OK;
}

extern "C" int32_t dfmi_filter_project(dfmi_context* ctx, const dfmi_program* pred,
                                       const dfmi_program* const* projs, int32_t np,
                                       const dfmi_batch* in, dfmi_out_column* outs, uint32_t flags,
                                       dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    if (ctx) ctx->last_err_key = ~0ull;
    // DFMI_DIAG + DFMI_CALL_PROFILE: per-phase host time of this entry point,
    // averaged over 1000 calls on stderr (diagnostics only)
    static thread_local double ph[6];
    static thread_local long ncalls;
    static const bool prof = getenv("DFMI_DIAG") && getenv("DFMI_CALL_PROFILE");
    auto tnow = [] { return std::chrono::steady_clock::now(); };
    auto tms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
        return std::chrono::duration<double, std::micro>(b - a).count();
    };
    auto t_a = tnow();
    try {
        if (!ctx || !in || (np > 0 && !projs) || !outs || (in->num_columns > 0 && !in->columns))
            throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        if (!pred && np == 0) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "neither a predicate nor projections"};
        Unsliced us_;  // sliced arrays (arrow offsets): offset-0 views / shifted bitmaps (slice.cpp)
        if (any_offset(in, 1)) {
            HIP_TRY(hipSetDevice(ctx->device));
            in = unslice(in, 1, us_, true, ctx->stream);
        }
        Built B;
        uint64_t hint_key = 0;
        if (pred && in->num_rows >= kSubtileMinRows) {
            hint_key = sel_hint_key(pred, projs, np, in, flags);
            auto it = ctx->sel_hint.find(hint_key);
            B.low_sel = it != ctx->sel_hint.end() && it->second < kLowSel;
            B.high_sel = it != ctx->sel_hint.end() && it->second >= kLowSel;
            const auto lt = ctx->utf8_len_hint.find(hint_key);
            B.ring_ok = it != ctx->sel_hint.end() && it->second >= kRingSel && lt != ctx->utf8_len_hint.end() &&
                        lt->second <= kRingLen;
            B.long_utf8 = lt != ctx->utf8_len_hint.end() && lt->second >= kLongLen;
        }
        build_plan(pred, projs, np, in, outs, flags, B);
        if (ctx->shared) B.X.ticket = 1;  // shared GPU: ticket-ordered tiles from the start
        auto t_b = tnow();
        if (prof) ph[0] += tms(t_a, t_b);
        Err& se = B.se;
        jit::Plan& plan = B.plan;
        jit::Launch& X = B.X;
        const bool any_kernel_out = B.any_kernel_out;
        const int64_t n = in->num_rows;
        const int nout = (int)plan.outs.size();
        const int64_t n_tiles = B.n_tiles;

        // ---- compile (cached per query shape) and launch
        HIP_TRY(hipSetDevice(ctx->device));
        hipStream_t st = ctx->stream;
        ctx->timed = false;
        ctx->last_compile_ms = 0;
        const bool launch = n > 0 && (pred || any_kernel_out);
        uint64_t dev_key = ~0ull;
        int dev_kind = 0;
        Args A;
        memset(&A, 0, sizeof A);
        if (launch) {
            hipFunction_t fn;
            try {
                fn = jit::get_kernel(ctx->device, plan, X, &ctx->last_compile_ms);
                ctx->last_kernel = X.kname;
            } catch (const Fail& f) {
                if (se.set) throw Fail{se.code, se.msg};  // the reference fails first
                throw;
            }
            auto t_c = tnow();
            if (prof) ph[1] += tms(t_b, t_c);
            const int n_chan = pred ? 1 + (int)X.utf8_outs.size() : 0;
            const size_t status_bytes = (size_t)n_chan * n_tiles * 8 * X.spread;
            // filtered outputs written as one byte per row and packed into a
            // bitmap after the kernel: Boolean values, and the validity of
            // projections that can produce nulls (fallible CAST)
            std::vector<int> bool_out, valid_out;
            for (int o = 0; o < nout; ++o) {
                if (!pred || plan.outs[o].kind == jit::OutSpec::SKIP || plan.outs[o].kind == jit::OutSpec::UTF8)
                    continue;
                if (plan.outs[o].out_type == DFMI_TYPE_BOOLEAN) bool_out.push_back(o);
                if (plan.outs[o].nullable) valid_out.push_back(o);
            }
            const size_t row_bytes = (size_t)((n + 63) & ~63ll);
            if (!bool_out.empty() || !valid_out.empty())
                ensure(ctx, &ctx->scratch, &ctx->scratch_bytes, (bool_out.size() + valid_out.size()) * row_bytes);
            const bool two_pass = pred && X.gather == 3 && !X.utf8_outs.empty();
            const size_t src_bytes = ((size_t)n * 4 + 255) & ~(size_t)255;  // one i32 source start per row
            if (two_pass) ensure(ctx, &ctx->utf8_src, &ctx->utf8_src_bytes, X.utf8_outs.size() * src_bytes);
            A.n_rows = n;
            A.n_tiles = (int)n_tiles;
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
            std::vector<uint8_t*> bool_dst(nout, nullptr);
            for (int o = 0; o < nout; ++o) {
                A.out[o] = outs[o].values;
                A.out_valid[o] = pred ? nullptr : outs[o].validity;
                A.out_offs[o] = outs[o].offsets;
                A.out_data[o] = outs[o].data;
                A.out_cap[o] = outs[o].data_capacity;
            }
            if (two_pass)
                for (size_t j = 0; j < X.utf8_outs.size(); ++j)
                    A.out_src[X.utf8_outs[j].first] = (int*)(ctx->utf8_src + j * src_bytes);
            for (size_t i = 0; i < bool_out.size(); ++i) {
                bool_dst[bool_out[i]] = (uint8_t*)outs[bool_out[i]].values;
                A.out[bool_out[i]] = ctx->scratch + i * row_bytes;
            }
            for (size_t i = 0; i < valid_out.size(); ++i)
                A.out_valid[valid_out[i]] = ctx->scratch + (bool_out.size() + i) * row_bytes;
            memcpy(A.lits, X.args_lits, sizeof A.lits);
            memcpy(A.str_off, X.str_off, sizeof A.str_off);
            memcpy(A.str_len, X.str_len, sizeof A.str_len);
            memcpy(A.str, X.str, sizeof A.str);
            // A look-back that made no progress for 2 s (ERRK_LOOKBACK_TIMEOUT:
            // e.g. the GPU time-sliced away from this queue for that long) is
            // relaunched once over a freshly zeroed workspace before it is
            // reported as a device error; the relaunch rewrites every output.
            for (int attempt = 0;; ++attempt) {
                const WsLease ws = ws_acquire(ctx, status_bytes, st);
                uint8_t* hdr = ws.hdr;
                A.ticket = (unsigned*)(hdr + kHdrTicket);
                A.err = (unsigned long long*)(hdr + kHdrErr);
                A.totals = (unsigned long long*)(hdr + kHdrTotals);
                A.status = (unsigned long long*)ws.status;
                A.stats = (unsigned long long*)(hdr + kHdrStats);
                A.clear_status = (unsigned long long*)ws.clear_status;
                A.clear_words = ws.clear_words;
                A.clear_hdr = (unsigned long long*)ws.clear_hdr;
                if (attempt == 0) {
                    A.mode = 0;
                    if (getenv("DFMI_DIAG"))
                        if (const char* m = getenv("DFMI_DEBUG_MODE")) A.mode = atoi(m);  // diagnostics only
                }
                const unsigned grid = (unsigned)n_tiles;  // one block per tile
                if (ctx->timing) HIP_TRY(hipEventRecord(ctx->ev0, st));
                size_t asz = sizeof A;
                void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &A, HIP_LAUNCH_PARAM_BUFFER_SIZE, &asz, HIP_LAUNCH_PARAM_END};
                HIP_TRY(hipModuleLaunchKernel(fn, grid, 1, 1, X.BLOCK, 1, 1, 0, st, nullptr, cfg));
                ws_commit(ctx, ws);
                if (two_pass && !(A.mode & 8))
                    for (size_t j = 0; j < X.utf8_outs.size(); ++j) {
                        const int o = X.utf8_outs[j].first;
                        HIP_TRY(launch_utf8_copy_rows(A.out_offs[o], A.out_src[o], A.bytes[X.utf8_outs[j].second],
                                                      A.out_data[o], A.totals, 1 + (int)j, A.out_cap[o], n, st));
                    }
                if (ctx->timing) HIP_TRY(hipEventRecord(ctx->ev1, st));
                for (int o = 0; o < nout; ++o)
                    if (bool_dst[o]) HIP_TRY(launch_pack_bools((const uint8_t*)A.out[o], bool_dst[o], A.totals, n, st));
                for (int o : valid_out)
                    HIP_TRY(launch_pack_bools(A.out_valid[o], outs[o].validity, A.totals, n, st));
                auto t_d = tnow();
                if (prof) ph[2] += tms(t_c, t_d);
                auto t_e = tnow();
                if (prof) ph[3] += tms(t_d, t_e);
                HIP_TRY(hipMemcpyAsync(ctx->host_hdr, hdr, kHdrAlloc, hipMemcpyDeviceToHost, st));
                if (ctx->timing) HIP_TRY(hipEventRecord(ctx->ev2, st));
                HIP_TRY(hipStreamSynchronize(st));
                auto t_f = tnow();
                if (prof) ph[4] += tms(t_e, t_f);
                uint64_t ew;
                memcpy(&ew, ctx->host_hdr + kHdrErr, 8);
                if (ew) {
                    dev_key = ~ew;
                    dev_kind = (int)(dev_key & 15);
                    dev_key &= ~15ull;
                }
                if (A.mode & 32) {
                    uint64_t g5[5];
                    memcpy(g5, ctx->host_hdr + kHdrStats + 64, sizeof g5);
                    fprintf(stderr, "dfmi utf8 gather cycles (summed over waves): staging %llu setup %llu zero %llu place %llu "
                            "store %llu\n", (unsigned long long)g5[0], (unsigned long long)g5[1], (unsigned long long)g5[2],
                            (unsigned long long)g5[3], (unsigned long long)g5[4]);
                }
                if (A.mode & 4) {
                    uint64_t st3[3];
                    memcpy(st3, ctx->host_hdr + kHdrStats, sizeof st3);
                    fprintf(stderr, "dfmi look-back: tiles %lld polls %llu sleeps %llu wait %.3f ms (summed over tiles)\n",
                            (long long)n_tiles, (unsigned long long)st3[0], (unsigned long long)st3[1], st3[2] * 1e-5);
                }
                if (ctx->timing) {
                    float m1 = 0, m2 = 0;
                    (void)hipEventElapsedTime(&m1, ctx->ev0, ctx->ev1);
                    (void)hipEventElapsedTime(&m2, ctx->ev0, ctx->ev2);
                    ctx->last_main_ms = m1;
                    ctx->last_total_ms = m2;
                    ctx->timed = true;
                }
                if (prof) {
                    ph[5] += tms(t_f, tnow());
                    if (++ncalls % 1000 == 0)
                        fprintf(stderr,
                                "dfmi call (us, mean of 1000): plan %.2f, kernel lookup %.2f, launch %.2f, header "
                                "copy %.2f, sync %.2f, timing %.2f\n",
                                ph[0] / 1000, ph[1] / 1000, ph[2] / 1000, ph[3] / 1000, ph[4] / 1000, ph[5] / 1000);
                    if (ncalls % 1000 == 0)
                        for (double& x : ph) x = 0;
                }
                if (dev_kind == ERRK_LOOKBACK_TIMEOUT && attempt == 0) {
                    ctx->ws_valid = false;  // status words in an unknown state: re-zero all
                    ++ctx->relaunches;
                    A.mode &= ~16;          // (diagnostic forced timeout: once)
                    dev_kind = 0;
                    dev_key = ~0ull;
                    // relaunched with ticket-ordered tiles: every look-back then
                    // waits only on running blocks, whatever else holds the CUs
                    X.ticket = 1;
                    fn = jit::get_kernel(ctx->device, plan, X, &ctx->last_compile_ms);
                    memcpy(A.lits, X.args_lits, sizeof A.lits);  // (that kernel's literal slots)
                    memcpy(A.str_off, X.str_off, sizeof A.str_off);
                    memcpy(A.str_len, X.str_len, sizeof A.str_len);
                    memcpy(A.str, X.str, sizeof A.str);
                    continue;
                }
                break;
            }
        }

        // ---- errors: the reference raises the first in evaluation order
        if (dev_kind == ERRK_LOOKBACK_TIMEOUT) throw Fail{DFMI_ERR_DEVICE, "device look-back timed out"};
        if (dev_kind == ERRK_CAPACITY) throw Fail{DFMI_ERR_CAPACITY, "Utf8 output data_capacity too small"};
        if (dev_kind && (!se.set || dev_key < se.key)) {
            ctx->last_err_key = dev_key;
            if (dev_kind == ERRK_DIV_ZERO) throw Fail{DFMI_ERR_DIVIDE_BY_ZERO, "DivideByZero"};
            throw Fail{DFMI_ERR_PANIC, "attempt to divide with overflow"};
        }
        if (se.set) {
            ctx->last_err_key = se.key;
            throw Fail{se.code, se.msg};
        }

        // ---- results
        uint64_t totals[24];
        memset(totals, 0, sizeof totals);
        if (launch) memcpy(totals, ctx->host_hdr + kHdrTotals, sizeof totals);
        const int64_t out_rows = pred ? (int64_t)totals[0] : n;
        if (hint_key && launch) {  // what this shape selected, for its next large batch
            if (ctx->sel_hint.size() >= 4096) ctx->sel_hint.clear();
            ctx->sel_hint[hint_key] = (double)out_rows / (double)n;
            if (!X.utf8_outs.empty() && out_rows > 0) {
                if (ctx->utf8_len_hint.size() >= 4096) ctx->utf8_len_hint.clear();
                ctx->utf8_len_hint[hint_key] = (double)totals[1] / (double)out_rows;
            }
        }
        for (int o = 0; o < nout; ++o) {
            dfmi_out_column& oc = outs[o];
            if (oc.passthrough_column >= 0) continue;
            oc.length = out_rows;
            oc.null_count = (!pred || plan.outs[o].nullable) ? (int64_t)totals[8 + o] : 0;
            if (plan.outs[o].kind == jit::OutSpec::UTF8) {
                oc.data_length = 0;
                for (size_t j = 0; j < X.utf8_outs.size(); ++j)
                    if (X.utf8_outs[j].first == o) oc.data_length = (int64_t)totals[1 + j];
                if (!launch) {  // offsets = [0] (a launch writes the final offset itself)
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

// ------------------------------------------------------- coalesced batches
// dfmi_filter_project over many batches in ONE launch (include/dfmi.h). Each
// batch keeps its own outputs, row counts and errors: tiles never straddle
// batches, a batch's tiles run the single-pass look-back over their own
// status segment, and every batch has its own header (totals, null counts,
// error word). The plan is built once from a "shape" batch -- the shared
// column types, a column nullable when any batch has nulls in it.
namespace {
constexpr size_t kBHdr = 256;  // per-batch header: [0..8) totals, [8..24) nulls, [24] error word

int32_t batches_one_by_one(dfmi_context* ctx, const dfmi_program* pred, const dfmi_program* const* projs, int32_t np,
                           const dfmi_batch* ins, int32_t nb, dfmi_out_column* outs, int nout, uint32_t flags,
                           int32_t* failed, dfmi_error* err) {
    for (int32_t b = 0; b < nb; ++b) {
        const int32_t rc = dfmi_filter_project(ctx, pred, projs, np, &ins[b], outs + (size_t)b * nout, flags, err);
        if (rc != DFMI_OK) {
            *failed = b;
            return rc;
        }
    }
    return DFMI_OK;
}
}  // namespace

extern "C" int32_t dfmi_filter_project_batches(dfmi_context* ctx, const dfmi_program* pred,
                                               const dfmi_program* const* projs, int32_t np, const dfmi_batch* ins,
                                               int32_t nb, dfmi_out_column* outs, uint32_t flags,
                                               int32_t* failed, dfmi_error* err) {
    return dfmi::filter_project_batches_staged(ctx, pred, projs, np, ins, nb, outs, flags, failed, err, nullptr);
}

int32_t dfmi::filter_project_batches_staged(dfmi_context* ctx, const dfmi_program* pred,
                                            const dfmi_program* const* projs, int32_t np, const dfmi_batch* ins,
                                            int32_t nb, dfmi_out_column* outs, uint32_t flags, int32_t* failed,
                                            dfmi_error* err, const BatchStage* stage) {
    // phases: checks + plan, kernel lookup, batch table, enqueue, synchronisation, results
    static thread_local CallProf prof("batches_staged");
    prof.start();
    set_err(err, DFMI_OK, "");
    int32_t dummy_failed;
    if (!failed) failed = &dummy_failed;
    *failed = -1;
    if (ctx) ctx->last_err_key = ~0ull;
    try {
        if (!ctx || nb < 0 || (nb > 0 && (!ins || !outs)) || (np > 0 && !projs))
            throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        if (!pred && np == 0) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "neither a predicate nor projections"};
        if (nb == 0) return DFMI_OK;
        Unsliced us_;  // sliced arrays (slice.cpp)
        if (any_offset(ins, nb)) {
            HIP_TRY(hipSetDevice(ctx->device));
            ins = unslice(ins, nb, us_, true, ctx->stream);
        }
        const int ncols = ins[0].num_columns;
        const int nout = np > 0 ? np : ncols;
        int64_t maxn = 0;
        for (int32_t b = 0; b < nb; ++b) {
            if (ins[b].num_columns != ncols || (ncols > 0 && !ins[b].columns))
                throw Fail{DFMI_ERR_INVALID_ARGUMENT, "batches do not share a schema"};
            for (int i = 0; i < ncols; ++i)
                if (ins[b].columns[i].type != ins[0].columns[i].type)
                    throw Fail{DFMI_ERR_INVALID_ARGUMENT, "batches do not share a schema"};
            maxn = std::max<int64_t>(maxn, ins[b].num_rows);
        }
        // the shape batch: shared types, nullable where any batch has nulls;
        // the pointers only need to be non-NULL here (the plan reads types
        // and nullability)
        static const uint64_t kDummy[2] = {0, 0};
        std::vector<dfmi_column> shape(ncols);
        std::vector<char> nullable(ncols, 0);
        for (int i = 0; i < ncols; ++i) {
            for (int32_t b = 0; b < nb; ++b)
                if (ins[b].columns[i].validity && ins[b].columns[i].null_count > 0) nullable[i] = 1;
            dfmi_column& c = shape[i];
            c = ins[0].columns[i];
            c.length = maxn;
            c.validity = nullable[i] ? (const uint8_t*)kDummy : nullptr;
            c.null_count = nullable[i] ? 1 : 0;
            c.values = kDummy;
            c.offsets = (const int32_t*)kDummy;
        }
        const dfmi_batch shape_batch{ncols, 0, maxn, shape.data()};
        Built B;
        build_plan(pred, projs, np, &shape_batch, outs, flags, B);
        if (ctx->shared) B.X.ticket = 1;  // shared GPU: ticket-ordered tiles from the start
        jit::Plan& plan = B.plan;
        jit::Launch& X = B.X;
        bool one_by_one = B.se.set || X.gather == 3 || !(pred || B.any_kernel_out);
        if (pred)  // filtered Boolean / nullable outputs are packed per batch after the kernel
            for (const jit::OutSpec& os : plan.outs)
                if (os.kind != jit::OutSpec::SKIP && os.kind != jit::OutSpec::UTF8 &&
                    (os.out_type == DFMI_TYPE_BOOLEAN || os.nullable))
                    one_by_one = true;
        if (one_by_one) {
            if (stage) {
                HIP_TRY(hipSetDevice(ctx->device));
                stage->copy_in(ctx->stream);
            }
            const int32_t rc = batches_one_by_one(ctx, pred, projs, np, ins, nb, outs, nout, flags, failed, err);
            if (stage) {
                stage->copy_out(ctx->stream);
                HIP_TRY(hipStreamSynchronize(ctx->stream));
            }
            return rc;
        }

        X.batched = true;
        HIP_TRY(hipSetDevice(ctx->device));
        hipStream_t st = ctx->stream;
        ctx->timed = false;
        ctx->last_compile_ms = 0;
        // ---- tiles per batch
        const int64_t tile_rows = (int64_t)X.BLOCK * X.K * X.M;
        std::vector<int64_t> first(nb), tiles(nb);
        int64_t T = 0, max_tiles = 0;
        for (int32_t b = 0; b < nb; ++b) {
            tiles[b] = (ins[b].num_rows + tile_rows - 1) / tile_rows;
            first[b] = T;
            T += tiles[b];
            max_tiles = std::max(max_tiles, tiles[b]);
        }
        if (T > 0x7fffffff) throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "batch too large"};
        // ---- batch table (its layout does not depend on hdr_out)
        const int NPW = jit::batch_words(X, nout);
        const size_t table_bytes = (size_t)nb * NPW * 8, meta_bytes = table_bytes + (size_t)T * 4;
        // the table and the per-batch headers: in the caller's staging (one
        // copy each way with its own data), or the context's buffers
        uint8_t *host_meta = nullptr, *dev_meta = nullptr, *dev_hdr = nullptr;
        const uint8_t* host_hdr = nullptr;
        const bool staged = stage && stage->locate &&
                            stage->locate(meta_bytes, (size_t)nb * kBHdr, &host_meta, &dev_meta, &dev_hdr, &host_hdr);
        // one tile per batch and a staged caller that takes the headers in
        // place (decided after locate: an unstaged call reads its headers
        // from ctx->bhdr, which a hdr_out kernel would zero before the D2H)
        X.hdr_out = staged && stage->hdr_out && max_tiles <= 1;
        prof.mark(0);
        hipFunction_t fn = jit::get_kernel(ctx->device, plan, X, &ctx->last_compile_ms);
        ctx->last_kernel = X.kname;
        prof.mark(1);
        if (!staged) {
            ensure_host(&ctx->host_bmeta, &ctx->host_bmeta_bytes, meta_bytes);
            ensure(ctx, &ctx->bmeta, &ctx->bmeta_bytes, meta_bytes);
            ensure_host(&ctx->host_bhdr, &ctx->host_bhdr_bytes, (size_t)nb * kBHdr);
            ensure(ctx, &ctx->bhdr, &ctx->bhdr_bytes, (size_t)nb * kBHdr);
            host_meta = ctx->host_bmeta;
            dev_meta = ctx->bmeta;
            dev_hdr = ctx->bhdr;
            host_hdr = ctx->host_bhdr;
        }
        bool need_ones = false;
        for (int i = 0; i < ncols && !need_ones; ++i)
            if (nullable[i])
                for (int32_t b = 0; b < nb; ++b)
                    if (!(ins[b].columns[i].validity && ins[b].columns[i].null_count > 0)) need_ones = true;
        if (need_ones) {
            const size_t nbm = (size_t)((maxn + 63) / 64 * 8 + 64);
            if (ctx->ones_bytes < nbm) {
                ensure(ctx, &ctx->ones, &ctx->ones_bytes, nbm);
                HIP_TRY(hipMemsetAsync(ctx->ones, 0xff, ctx->ones_bytes, st));
            }
        }
        uint64_t* tab = (uint64_t*)host_meta;
        int32_t* tile_batch = (int32_t*)(host_meta + table_bytes);
        auto valid_of = [&](const dfmi_column& c, int col) -> uint64_t {
            if (!nullable[col]) return 0;
            return (uint64_t)((c.validity && c.null_count > 0) ? c.validity : ctx->ones);
        };
        for (int32_t b = 0; b < nb; ++b) {
            const dfmi_batch& in = ins[b];
            for (int i = 0; i < ncols; ++i)
                if (in.columns[i].length != in.num_rows) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "ragged batch"};
            uint64_t* row = tab + (size_t)b * NPW;
            memset(row, 0, (size_t)NPW * 8);
            row[0] = (uint64_t)in.num_rows;
            row[1] = (uint64_t)tiles[b] | ((uint64_t)first[b] << 32);
            row[2] = (uint64_t)(dev_hdr + (size_t)b * kBHdr);
            row[3] = (uint64_t)(dev_hdr + (size_t)b * kBHdr + 24 * 8);
            for (size_t sl = 0; sl < X.num_cols.size(); ++sl) {
                const dfmi_column& c = in.columns[X.num_cols[sl]];
                const int w = jit::type_width(c.type);
                if (in.num_rows > 0 && !c.values) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "column values pointer is NULL"};
                if (w && ((uintptr_t)c.values & (w - 1)))
                    throw Fail{DFMI_ERR_INVALID_ARGUMENT, "column values must be aligned to their width"};
                row[jit::batch_slot_col((int)sl)] = (uint64_t)c.values;
                row[jit::batch_slot_col((int)sl) + 1] = valid_of(c, X.num_cols[sl]);
            }
            for (size_t u = 0; u < X.utf8_cols.size(); ++u) {
                const dfmi_column& c = in.columns[X.utf8_cols[u]];
                if (in.num_rows > 0 && (!c.values || !c.offsets))
                    throw Fail{DFMI_ERR_INVALID_ARGUMENT, "Utf8 column buffers are NULL"};
                const int sl = jit::batch_slot_utf8(X, (int)u);
                row[sl] = (uint64_t)c.offsets;
                row[sl + 1] = (uint64_t)c.values;
                row[sl + 2] = valid_of(c, X.utf8_cols[u]);
            }
            for (int o = 0; o < nout; ++o) {
                dfmi_out_column& oc = outs[(size_t)b * nout + o];
                const jit::OutSpec& os = plan.outs[o];
                const int sl = jit::batch_slot_out(X, o);
                if (os.kind == jit::OutSpec::UTF8) {
                    if (!oc.offsets || !oc.data) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "Utf8 output buffers are NULL"};
                } else if (os.kind != jit::OutSpec::SKIP) {
                    if (!oc.values) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "output values pointer is NULL"};
                    if (!pred && !oc.validity)
                        throw Fail{DFMI_ERR_INVALID_ARGUMENT, "output validity pointer is NULL"};
                }
                row[sl] = (uint64_t)oc.values;
                row[sl + 1] = pred ? 0 : (uint64_t)oc.validity;
                row[sl + 2] = (uint64_t)oc.offsets;
                row[sl + 3] = (uint64_t)oc.data;
                row[sl + 4] = (uint64_t)oc.data_capacity;
            }
            for (int64_t t = 0; t < tiles[b]; ++t) tile_batch[first[b] + t] = b;
        }
        // ---- launch. A look-back that timed out in any batch (the GPU
        // time-sliced away from this queue for 2 s) is relaunched once over a
        // re-zeroed workspace and headers, as dfmi_filter_project does; the
        // relaunch rewrites every batch's outputs.
        prof.mark(2);
        if (stage) stage->copy_in(st);  // (staged: with the table; headers zeroed by the previous call)
        int mode = 0;
        if (getenv("DFMI_DIAG"))
            if (const char* m = getenv("DFMI_DEBUG_MODE")) mode = atoi(m);  // diagnostics only (bit 4: force a timeout)
        for (int attempt = 0;; ++attempt) {
            if (T > 0) {
                if (!staged && attempt == 0) HIP_TRY(hipMemcpyAsync(dev_meta, host_meta, meta_bytes, hipMemcpyHostToDevice, st));
                if (!staged || attempt > 0) HIP_TRY(hipMemsetAsync(dev_hdr, 0, (size_t)nb * kBHdr, st));
                const int n_chan = pred ? 1 + (int)X.utf8_outs.size() : 0;
                const size_t status_bytes = (size_t)n_chan * T * 8 * X.spread;
                Args A;
                memset(&A, 0, sizeof A);
                A.n_rows = maxn;
                A.n_tiles = (int)T;
                A.mode = mode;
                memcpy(A.lits, X.args_lits, sizeof A.lits);
                memcpy(A.str_off, X.str_off, sizeof A.str_off);
                memcpy(A.str_len, X.str_len, sizeof A.str_len);
                memcpy(A.str, X.str, sizeof A.str);
                const WsLease ws = ws_acquire(ctx, status_bytes, st);
                A.ticket = (unsigned*)(ws.hdr + kHdrTicket);
                A.err = (unsigned long long*)(ws.hdr + kHdrErr);
                A.totals = (unsigned long long*)(ws.hdr + kHdrTotals);
                A.status = (unsigned long long*)ws.status;
                A.stats = (unsigned long long*)(ws.hdr + kHdrStats);
                A.clear_status = (unsigned long long*)ws.clear_status;
                A.clear_words = ws.clear_words;
                A.clear_hdr = (unsigned long long*)ws.clear_hdr;
                A.tile_batch = (const int*)(dev_meta + table_bytes);
                A.batch_ptrs = (void* const*)dev_meta;
                if (stage) {
                    A.clear_bhdr = (unsigned long long*)stage->clear_bhdr;
                    A.clear_bhdr_words = stage->clear_bhdr_words;
                    if (X.hdr_out) A.hdr_out = (unsigned long long*)stage->hdr_out;
                }
                if (ctx->timing) HIP_TRY(hipEventRecord(ctx->ev0, st));
                size_t asz = sizeof A;
                void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &A, HIP_LAUNCH_PARAM_BUFFER_SIZE, &asz, HIP_LAUNCH_PARAM_END};
                HIP_TRY(hipModuleLaunchKernel(fn, (unsigned)T, 1, 1, X.BLOCK, 1, 1, 0, st, nullptr, cfg));
                ws_commit(ctx, ws);
                if (stage && stage->cleared) *stage->cleared = true;
                if (X.hdr_out && stage->hdr_written) *stage->hdr_written = true;
                if (ctx->timing) HIP_TRY(hipEventRecord(ctx->ev1, st));
                if (!staged) HIP_TRY(hipMemcpyAsync(ctx->host_bhdr, ctx->bhdr, (size_t)nb * kBHdr, hipMemcpyDeviceToHost, st));
            }
            for (int32_t b = 0; b < nb; ++b)  // empty batches: Utf8 offsets = [0]
                if (ins[b].num_rows == 0)
                    for (int o = 0; o < nout; ++o)
                        if (plan.outs[o].kind == jit::OutSpec::UTF8 && outs[(size_t)b * nout + o].offsets)
                            HIP_TRY(hipMemsetAsync(outs[(size_t)b * nout + o].offsets, 0, 4, st));
            if (stage) stage->copy_out(st);  // (staged: with the headers)
            prof.mark(3);
            HIP_TRY(hipStreamSynchronize(st));
            prof.mark(4);
            bool timed_out = false;
            for (int32_t b = 0; b < nb && T > 0; ++b) {
                const uint64_t ew = ins[b].num_rows > 0 ? ((const uint64_t*)(host_hdr + (size_t)b * kBHdr))[24] : 0;
                if (ew && (int)(~ew & 15) == ERRK_LOOKBACK_TIMEOUT) timed_out = true;
            }
            if (!timed_out || attempt > 0) break;
            ctx->ws_valid = false;  // status words in an unknown state: re-zero all
            ++ctx->relaunches;
            mode &= ~16;  // (diagnostic forced timeout: once)
            X.ticket = 1;  // ticket-ordered tiles (see dfmi_filter_project)
            fn = jit::get_kernel(ctx->device, plan, X, &ctx->last_compile_ms);
        }
        if (T > 0 && ctx->timing) {
            float m1 = 0;
            (void)hipEventElapsedTime(&m1, ctx->ev0, ctx->ev1);
            ctx->last_main_ms = ctx->last_total_ms = m1;
            ctx->timed = true;
        }
        // ---- per batch, in order: results, or the first batch's error
        for (int32_t b = 0; b < nb; ++b) {
            const uint64_t* h = (const uint64_t*)(host_hdr + (size_t)b * kBHdr);
            const bool ran = ins[b].num_rows > 0;
            const uint64_t ew = ran ? h[24] : 0;
            if (ew) {
                const uint64_t key = ~ew;
                const int kind = (int)(key & 15);
                *failed = b;
                if (kind == ERRK_LOOKBACK_TIMEOUT) throw Fail{DFMI_ERR_DEVICE, "device look-back timed out"};
                if (kind == ERRK_CAPACITY) throw Fail{DFMI_ERR_CAPACITY, "Utf8 output data_capacity too small"};
                ctx->last_err_key = key & ~15ull;
                if (kind == ERRK_DIV_ZERO) throw Fail{DFMI_ERR_DIVIDE_BY_ZERO, "DivideByZero"};
                throw Fail{DFMI_ERR_PANIC, "attempt to divide with overflow"};
            }
            const int64_t n = ins[b].num_rows;
            const int64_t out_rows = pred ? (ran ? (int64_t)h[0] : 0) : n;
            for (int o = 0; o < nout; ++o) {
                dfmi_out_column& oc = outs[(size_t)b * nout + o];
                const dfmi_out_column& tmpl = outs[o];
                oc.type = tmpl.type;
                oc.passthrough_column = tmpl.passthrough_column;
                oc.data_length = 0;
                if (oc.passthrough_column >= 0) {  // Arc clone of this batch's column
                    const dfmi_column& c = ins[b].columns[oc.passthrough_column];
                    oc.length = n;
                    oc.null_count = c.validity ? c.null_count : 0;
                    continue;
                }
                oc.length = out_rows;
                oc.null_count = (!pred && ran) ? (int64_t)h[8 + o] : 0;
                if (plan.outs[o].kind == jit::OutSpec::UTF8 && ran)
                    for (size_t j = 0; j < X.utf8_outs.size(); ++j)
                        if (X.utf8_outs[j].first == o) oc.data_length = (int64_t)h[1 + j];
            }
        }
        prof.mark(5);
        prof.done();
        return DFMI_OK;
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

// Internal test hook (not part of the C ABI, not declared in include/):
// generates the query kernel a dfmi_filter_project call would launch and, if
// compile != 0, compiles it with hipRTC -- no device needed, so the CPU test
// suite checks code generation for every expression shape it covers.
// Returns the source length (the text is truncated to cap), or -status.
extern "C" int64_t dfmi_internal_jit_check(const dfmi_program* pred, const dfmi_program* const* projs, int32_t np,
                                           const dfmi_batch* in, dfmi_out_column* outs, uint32_t flags,
                                           int32_t compile, char* buf, int64_t cap, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    try {
        if (!in || (np > 0 && !projs) || !outs) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        Built B;
        build_plan(pred, projs, np, in, outs, flags & ~0x40000000u, B);
        B.X.batched = (flags & 0x40000000u) != 0;  // the coalesced-batches form of the kernel
        const std::string src = jit::generate(B.plan, B.X);
        if (compile) (void)jit::compile_code(src, nullptr);
        if (buf && cap > 0) snprintf(buf, (size_t)cap, "%s", src.c_str());
        return (int64_t)src.size();
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return -(int64_t)f.code;
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
