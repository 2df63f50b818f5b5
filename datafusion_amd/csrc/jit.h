// Query compiler interface (host side of jit.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "../../include/dfmi.h"
#include "dfmi_program.h"

namespace dfmi {

struct Fail {
    int32_t code;
    std::string msg;
};

namespace jit {

// One output column of the pass.
struct OutSpec {
    enum Kind { SKIP, GATHER, EXPR, UTF8 } kind = SKIP;
    int col = -1;                      // GATHER / UTF8: input column
    const dfmi_program* prog = nullptr;  // EXPR
    int ord_base = 0;                  // evaluation-order base of prog's nodes
    int out_type = 0;
    // EXPR after a Selection whose value can be null although the filtered
    // batch has none (a CAST that rejects a value): validity bytes + count
    bool nullable = false;
};

// One aggregate of the aggregate kernel (DFMI_FLAG_EXT_AGGREGATE).
struct AggSpec {
    int fn = 0;                          // dfmi_agg_fn
    const dfmi_program* prog = nullptr;  // argument
    int ord_base = 0;                    // evaluation-order base of prog's nodes
    int arg_type = 0;
    int fslot = -1;                      // >= 0: exact float sum, its LDS digit block
};

struct Plan {
    const dfmi_program* pred = nullptr;  // nullptr: projection only (dense kernel)
    std::vector<OutSpec> outs;
    std::vector<AggSpec> aggs;           // non-empty: the aggregate kernel (outs unused)
    // GROUP BY extension: the key (Boolean / integer), its evaluation-order
    // base, and the kernel's slot count (key window + the null slot)
    const dfmi_program* gkey = nullptr;
    int gkey_ord = 0;
    int gslots = 0;
};

// Slot tables + literal pools of one launch.
struct Launch {
    int K = 8, BLOCK = 512;
    int waves_per_eu = 0;  // >0: occupancy hint to the register allocator
    bool waves_soft = false;  // ... dropped (recompiled without) when meeting it spills
    // look-back: R windows of 64 status words per round trip, s_sleep(sleep)
    // between polls, one status word per `spread` words (16 = one per 128-byte
    // line: polling blocks then do not contend on shared lines)
    int R = 1, sleep = 32, spread = 16;
    // predecessors read per poll, one lane each: 8 measured best at s=0.5
    // (64 cost ~9% of the C2 kernel in polling traffic)
    int window = 8;
    int late_proj = 0;  // projection-only columns loaded after the look-back (byte-light predicates)
    // coalesced batches of one tile each (host_batch.cpp small calls): every
    // block copies its batch's finished header to Args::hdr_out and zeroes it
    int hdr_out = 0;
    // tiles taken from an atomic ticket in the order blocks start instead of
    // blockIdx: a look-back then only waits on tiles whose blocks are running
    // (the relaunch after a look-back timeout, e.g. when another process's
    // kernel holds the CUs the next tiles in dispatch order would need)
    int ticket = 0;
    int early = 0;  // Utf8 gather: stage the next group before the last slice's stores (DFMI_UTF8_EARLY)
    // Utf8 gather of a numeric predicate at high selectivity: one loader wave
    // streams the tile's source bytes into an LDS ring ahead of use, the block
    // assembles and stores each 256-row step's output together
    // (jit_skeleton.hip "ring-staged Utf8 gather"); ring = chunks per slot
    int ring = 0;
    // Utf8 `col = literal` predicates: stage the wave's whole source spans into
    // an LDS arena of eq_dense 16-byte chunks and compare from there (diagnostic A/B);
    // < 0: the register-resident dense form, -eq_dense slices' spans per load round
    int eq_dense = 0;
    // Utf8 gather: the per-lane fallback copy (a slice whose span is over the
    // stage) as register-light unaligned 16-/4-byte moves instead of
    // utf8_copy's aligned 8-word chunks: C3 -1%, 40-200-byte strings -25%
    // (profiles/r05/c3_light_copy_ab2.log, long_utf8.log)
    int light_copy = 1;
    // Utf8 gather's per-lane fallback for long strings (long_copy): 64 bytes
    // in flight per lane (exec.cpp: the query's last large batch selected
    // strings of >= kLongLen bytes on average)
    int long_copy = 0;
    // gather == 6 (utf8_gather_direct): slices whose loads go out together
    int direct_grp = 2;
    int proj_dense = 0;  // projection-only columns loaded for every row with the predicate's columns (not lane-masked)
    // sub-tiles per tile (> 1: latency-bound predicates): a block runs the
    // predicate over M sub-tiles of BLOCK * K rows, keeping only their
    // selection ballots (LDS), then one scan + look-back for all of them and
    // an output pass that reloads what the selected rows need
    int M = 1;
    int prefetch = 0;  // ... and load sub-tile m+1's Utf8 offsets while sub-tile m's heads are in flight
    int sparse = 1;    // ... with a one-lane-per-row output pass when a wave holds <= 64 selected rows
    int KO = 0;  // ... whose output pass handles KO slices per wave at a time (divides K; 0 = K)
    int gather = 1;  // Utf8 gather: 1 = wave-cooperative, consecutive slices staged together,
                     //     lanes on output words found by binary search (utf8_emit_slice);
                     // 2 = one slice per round trip, 0 = per-lane copy (diagnostics);
                     // 3 = two passes: offsets + source starts, then k_utf8_copy_rows
                     // 4 = as 1, but each slice assembled in an LDS image (round 2's form);
                     // 5 = as 1, output words' strings found by a marker max-scan
                     // 6 = per-lane unaligned loads into registers, exact-length stores (no LDS)
    int arena = 128; // Utf8 gather staging arena per wave, 16-byte chunks
    int pairs = 0;     // gather 4: two slices' LDS images assembled together (image = 2 x 65 chunks)
    int dbuf = 0;      // gather 1 / 4 / 5: the arena's halves double-buffer the staging (ARENA >= 256)
    int image = 129;   // gather 4: LDS image per wave, 16-byte chunks (a longer slice output copies per lane)
    int st16 = 0;      // gather 4: the image 16-byte aligned, stored with 16-byte stores (edge words apart)
    int prestage = 0;
    int gather_phases = 0;  // diagnostics: per-phase cycle counters in utf8_gather (DFMI_DEBUG_MODE bit 5)  // gather 1 / 4: the first staging round is issued before the look-back
    // cache policy of the column streams: bit0 nontemporal loads, bit1 nontemporal stores
    int nt = 0;
    const dfmi_batch* in = nullptr;
    std::vector<int> num_cols;   // arg slot -> input column (numeric and Boolean)
    std::vector<int> pred_slots; // slots the predicate reads (loaded for every row)
    std::vector<int> proj_slots; // slots only projections read (loaded where selected)
    std::vector<int> utf8_cols;  // utf8 slot -> input column
    std::vector<std::pair<int, int>> utf8_outs;  // (output index, utf8 slot)
    uint64_t args_lits[32] = {};
    int n_lits = 0;
    int str_off[8] = {}, str_len[8] = {};
    char str[256] = {};
    int n_str = 0, str_bytes = 0;
    std::string kname;  // generated kernel's name (dfmi_<kind>_<hash>)
    std::shared_ptr<const void> module;  // keeps the kernel's code object loaded (get_kernel)
    // coalesced batches (dfmi_filter_project_batches): blocks map to batches
    // through Args::tile_batch, and each batch's sizes and buffers come from
    // its row of Args::batch_ptrs (layout: batch_slot_* below)
    bool batched = false;

    int col_type(int col) const { return in->columns[col].type; }
    bool col_nullable(int col) const {
        return in->columns[col].validity != nullptr && in->columns[col].null_count > 0;
    }
    int slot_of_col(int col) const {
        for (size_t i = 0; i < num_cols.size(); ++i)
            if (num_cols[i] == col) return (int)i;
        throw Fail{DFMI_ERR_INVALID_ARGUMENT, "query compiler: column not registered"};
    }
    int slot_of_utf8(int col) const {
        for (size_t i = 0; i < utf8_cols.size(); ++i)
            if (utf8_cols[i] == col) return (int)i;
        throw Fail{DFMI_ERR_INVALID_ARGUMENT, "query compiler: Utf8 column not registered"};
    }
};

// Row layout of Args::batch_ptrs for one batch (8-byte words):
//   [0] rows, [1] tiles | first tile << 32, [2] totals, [3] error word,
//   per numeric slot s: values, validity; per Utf8 slot u: offsets, bytes,
//   validity; per output o: values, validity, offsets, data, data capacity.
inline int batch_slot_col(int s) { return 4 + 2 * s; }
inline int batch_slot_utf8(const Launch& X, int u) { return 4 + 2 * (int)X.num_cols.size() + 3 * u; }
inline int batch_slot_out(const Launch& X, int o) {
    return 4 + 2 * (int)X.num_cols.size() + 3 * (int)X.utf8_cols.size() + 5 * o;
}
inline int batch_words(const Launch& X, int nout) { return batch_slot_out(X, nout); }

// Bytes per value of a fixed-width dfmi_type (0 otherwise) and the C++ type
// the generated code holds it in (i8 .. u64, float, double).
int type_width(int t);
const char* ctype(int t);

// True when evaluating p over a batch without nulls can still produce a null
// (a CAST num::cast can reject, DFMI_FLAG_EXT_CAST).
bool may_introduce_nulls(const dfmi_program* p);

// Generated source of the plan's kernel (skeleton + body); fills the literal pools.
std::string generate(const Plan& P, Launch& X);
// Compiled kernel for the plan (cached per source text and device).
hipFunction_t get_kernel(int device, const Plan& P, Launch& X, double* compile_ms);
size_t cache_size();
// Bound of the module cache (least recently used evicted); cap > 0 sets it.
size_t cache_cap(size_t cap);
// hipRTC compile of a generated source to a gfx950 code object (no device needed).
std::vector<char> compile_code(const std::string& src, double* compile_ms);  // on-disk cache, then hipRTC
std::vector<char> compile_code_rtc(const std::string& src, double* compile_ms);  // hipRTC only

}  // namespace jit
}  // namespace dfmi
