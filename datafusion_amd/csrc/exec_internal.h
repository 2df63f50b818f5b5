// Internals shared by the execution entry points (exec.cpp: filter +
// project, aggregate.cpp: the aggregate extension): the context, the
// workspace layout, error plumbing.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <string>

#include "dfmi_program.h"
#include "jit.h"

// Workspace header layout (device, zero when a launch starts).
static constexpr size_t kHdrTicket = 0;
static constexpr size_t kHdrErr = 8;
static constexpr size_t kHdrTotals = 16;
static constexpr size_t kHdrStats = 256;  // look-back statistics (DFMI_DEBUG_MODE bit 4)
static constexpr size_t kHdrAlloc = 512;

struct dfmi_context {
    int device = 0;
    hipStream_t stream = nullptr;
    // Look-back workspace, double-buffered: [hdr 0 | hdr 1 | status 0 | status 1].
    // Launch i uses pair (i & 1), which is zero on entry, and its blocks zero
    // pair (i+1) & 1 -- what launch i-1 dirtied -- for launch i+1 (stream
    // order makes launch i-1 complete first). No memset on the steady path.
    uint8_t* ws = nullptr;
    size_t ws_bytes = 0;
    size_t status_cap = 0;       // bytes per status buffer
    int parity = 0;              // pair the next launch uses
    size_t dirty[2] = {0, 0};    // status bytes [0, dirty[b]) of buffer b may be non-zero
    bool ws_valid = false;       // the invariant above holds (else re-zero everything)
    uint8_t* scratch = nullptr;  // Boolean output bytes (filtered)
    size_t scratch_bytes = 0;
    uint8_t* utf8_src = nullptr;  // two-pass Utf8 gather: source start per selected row
    size_t utf8_src_bytes = 0;
    uint8_t* host_hdr = nullptr; // pinned copy of the header
    bool timing = true;  // record HIP events around launches (dfmi_context_set_timing)
    void* host_arena = nullptr;  // host_batch.cpp's staging arena (per context: no shared state)
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
    double last_total_ms = 0, last_main_ms = 0, last_compile_ms = 0;
    bool timed = false;
    // evaluation-order key (ordinal << 44 | row << 4) of the error the last
    // dfmi_filter_project raised; ~0 for none / an error outside that order
    uint64_t last_err_key = ~0ull;
    std::string last_kernel;  // name of the last launched query kernel (dfmi_last_kernel_name)
};

namespace dfmi {
namespace xi {

inline void set_err(dfmi_error* err, int32_t code, const std::string& m) {
    if (!err) return;
    err->code = code;
    snprintf(err->message, sizeof err->message, "%s", m.c_str());
}

#define HIP_TRY(x)                                                                         \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) throw Fail{DFMI_ERR_DEVICE, std::string(#x ": ") + hipGetErrorString(e_)}; \
    } while (0)

inline bool gatherable(int t, uint32_t flags) {
    if (t == DFMI_TYPE_FLOAT64 || t == DFMI_TYPE_UTF8) return true;  // filter.rs:84,94
    // extension: every fixed-width type and Boolean
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

inline void ensure(dfmi_context* ctx, uint8_t** buf, size_t* have, size_t need) {
    if (*have >= need) return;
    if (*buf) HIP_TRY(hipFree(*buf));
    *buf = nullptr;
    *have = 0;
    size_t cap = std::max(need, (size_t)1 << 20);
    HIP_TRY(hipMalloc(buf, cap));
    *have = cap;
}

// One launch's share of the double-buffered workspace (see dfmi_context):
// its header and status buffer (zero on entry) and what its blocks clear for
// the next launch.
struct WsLease {
    int par = 0;
    size_t status_bytes = 0;
    uint8_t* hdr = nullptr;
    uint8_t* status = nullptr;
    uint8_t* clear_status = nullptr;
    long long clear_words = 0;
    uint8_t* clear_hdr = nullptr;
};

inline WsLease ws_acquire(dfmi_context* ctx, size_t status_bytes, hipStream_t st) {
    if (!ctx->ws || status_bytes > ctx->status_cap) {
        const size_t cap = (std::max(status_bytes, (size_t)1 << 20) + 255) & ~(size_t)255;
        ensure(ctx, &ctx->ws, &ctx->ws_bytes, 2 * kHdrAlloc + 2 * cap);
        ctx->status_cap = cap;
        ctx->ws_valid = false;
    }
    if (!ctx->ws_valid) {  // first use, growth, or an interrupted call
        HIP_TRY(hipMemsetAsync(ctx->ws, 0, 2 * kHdrAlloc + 2 * ctx->status_cap, st));
        ctx->dirty[0] = ctx->dirty[1] = 0;
        ctx->ws_valid = true;
    }
    WsLease l;
    l.par = ctx->parity;
    l.status_bytes = status_bytes;
    l.hdr = ctx->ws + l.par * kHdrAlloc;
    l.status = ctx->ws + 2 * kHdrAlloc + l.par * ctx->status_cap;
    l.clear_status = ctx->ws + 2 * kHdrAlloc + (1 - l.par) * ctx->status_cap;
    l.clear_words = (long long)(ctx->dirty[1 - l.par] / 8);
    l.clear_hdr = ctx->ws + (1 - l.par) * kHdrAlloc;
    ctx->ws_valid = false;  // until the launch is enqueued (ws_commit)
    return l;
}

// The launch using `l` is enqueued: the other pair is clean for the next one.
inline void ws_commit(dfmi_context* ctx, const WsLease& l) {
    ctx->dirty[l.par] = l.status_bytes;
    ctx->dirty[1 - l.par] = 0;
    ctx->parity = 1 - l.par;
    ctx->ws_valid = true;
}

}  // namespace xi
}  // namespace dfmi
