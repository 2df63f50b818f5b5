// Internals shared by the execution entry points (exec.cpp: filter +
// project, aggregate.cpp: the aggregate extension): the context, the
// workspace layout, error plumbing.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <string>
#include <unordered_map>

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
    // Launch i uses pair (i & 1), whose first `need` status bytes must be
    // zero on entry; its blocks zero what launch i-1 dirtied in the other
    // pair, for launch i+1 (stream order makes launch i-1 complete first) --
    // no memset per call. Bytes [dirty_lo[b], dirty_hi[b]) of status buffer b
    // may be non-zero. A launch clears the other pair only up to a few times
    // its own status size (a 1024-row call after a 1e9-row call must not
    // zero 31 MB from one block); a larger leftover is cleared by memset of
    // just the prefix a later launch needs (ws_acquire).
    uint8_t* ws = nullptr;
    size_t ws_bytes = 0;
    size_t status_cap = 0;       // bytes per status buffer
    int parity = 0;              // pair the next launch uses
    size_t dirty_lo[2] = {0, 0}, dirty_hi[2] = {0, 0};
    bool ws_valid = false;       // the invariant above holds (else re-zero everything)
    uint8_t* scratch = nullptr;  // Boolean output bytes (filtered)
    size_t scratch_bytes = 0;
    uint8_t* utf8_src = nullptr;  // two-pass Utf8 gather: source start per selected row
    size_t utf8_src_bytes = 0;
    uint8_t* host_hdr = nullptr; // pinned copy of the header
    bool timing = true;  // record HIP events around launches (dfmi_context_set_timing)
    // the GPU is shared with other processes (dfmi_context_set_shared, or
    // DFMI_SHARED=1 at creation): look-back kernels take their tiles in
    // ticket order from the first launch instead of after a 2 s timeout
    bool shared = false;
    void* host_arena = nullptr;  // host_batch.cpp's staging arena (per context: no shared state)
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
    double last_total_ms = 0, last_main_ms = 0, last_compile_ms = 0;
    bool timed = false;
    // evaluation-order key (ordinal << 44 | row << 4) of the error the last
    // dfmi_filter_project raised; ~0 for none / an error outside that order
    uint64_t last_err_key = ~0ull;
    long relaunches = 0;      // look-back timeouts relaunched (dfmi_internal_relaunches)
    std::string last_kernel;  // name of the last launched query kernel (dfmi_last_kernel_name)
    // coalesced batches (dfmi_filter_project_batches): per-call batch table
    // and per-batch headers, device + pinned host mirrors; an all-valid
    // bitmap for batches without validity in a column others have it for
    uint8_t* bmeta = nullptr;
    size_t bmeta_bytes = 0;
    uint8_t* host_bmeta = nullptr;
    size_t host_bmeta_bytes = 0;
    uint8_t* bhdr = nullptr;
    size_t bhdr_bytes = 0;
    uint8_t* host_bhdr = nullptr;
    size_t host_bhdr_bytes = 0;
    uint8_t* ones = nullptr;
    size_t ones_bytes = 0;
    // selectivity of each query shape's last large batch (exec.cpp
    // kSubtileMinRows): picks the sub-tile kernel for low selectivity
    std::unordered_map<uint64_t, double> sel_hint;
    // ... and the mean bytes of its first Utf8 output's selected strings
    // (picks the ring-staged gather, which stages whole 256-row steps)
    std::unordered_map<uint64_t, double> utf8_len_hint;
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

inline void ensure_host(uint8_t** buf, size_t* have, size_t need) {  // pinned
    if (*have >= need) return;
    if (*buf) HIP_TRY(hipHostFree(*buf));
    *buf = nullptr;
    *have = 0;
    size_t cap = std::max(need, (size_t)1 << 16);
    HIP_TRY(hipHostMalloc((void**)buf, cap, hipHostMallocDefault));
    *have = cap;
}

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
    uint8_t* clear_status = nullptr;  // first status word the kernel zeroes ...
    long long clear_words = 0;        // ... and how many
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
        ctx->dirty_lo[0] = ctx->dirty_lo[1] = ctx->dirty_hi[0] = ctx->dirty_hi[1] = 0;
        ctx->ws_valid = true;
    }
    WsLease l;
    const int p = ctx->parity, q = 1 - p;
    l.par = p;
    l.status_bytes = status_bytes;
    l.hdr = ctx->ws + p * kHdrAlloc;
    l.status = ctx->ws + 2 * kHdrAlloc + p * ctx->status_cap;
    // the prefix this launch needs must be zero: what is left dirty in this
    // pair is cleared whole, by one memset (so a small launch after a large
    // one pays it once, not on every later use of the pair)
    size_t& lo = ctx->dirty_lo[p];
    size_t& hi = ctx->dirty_hi[p];
    if (hi > lo && lo < status_bytes) {
        HIP_TRY(hipMemsetAsync(l.status + lo, 0, hi - lo, st));
        lo = hi = 0;
    }
    // what this launch's blocks zero in the other pair (bounded by its size);
    // a larger leftover (a full-table launch before a 1024-row one) is
    // cleared here once, by one memset, and later launches are back to
    // clearing in the kernel
    uint8_t* other = ctx->ws + 2 * kHdrAlloc + q * ctx->status_cap;
    size_t& qlo = ctx->dirty_lo[q];
    size_t& qhi = ctx->dirty_hi[q];
    if (qhi > qlo && qhi - qlo > std::max<size_t>(4 * status_bytes, (size_t)64 << 10)) {
        HIP_TRY(hipMemsetAsync(other + qlo, 0, qhi - qlo, st));
        qlo = qhi = 0;
    }
    const size_t qd = qhi - qlo;
    if (qd > 0) {
        l.clear_status = other + qlo;
        l.clear_words = (long long)(qd / 8);
    } else {
        l.clear_status = other;
        l.clear_words = 0;
    }
    l.clear_hdr = ctx->ws + q * kHdrAlloc;
    ctx->ws_valid = false;  // until the launch is enqueued (ws_commit)
    return l;
}

// The launch using `l` is enqueued: its status prefix is dirty, and the
// other pair's range it zeroes is clean for the next launch.
inline void ws_commit(dfmi_context* ctx, const WsLease& l) {
    const int p = l.par, q = 1 - p;
    if (l.status_bytes) {
        ctx->dirty_hi[p] = std::max(ctx->dirty_hi[p], l.status_bytes);
        ctx->dirty_lo[p] = 0;
    }
    if (l.clear_words) ctx->dirty_lo[q] = ctx->dirty_hi[q] = 0;
    ctx->parity = q;
    ctx->ws_valid = true;
}

}  // namespace xi
}  // namespace dfmi
