// How a caller of the coalesced-batches launch (exec.cpp) stages its small
// per-call data: the host-batches entry point (host_batch.cpp) moves its
// packed inputs and the batch table with ONE H2D copy (none for small calls,
// whose kernel reads them from pinned memory), and the outputs with the
// per-batch headers with ONE D2H copy; the headers are zeroed by the
// previous call's kernel (clear_bhdr), so a call is at most one copy in, one
// launch, one copy out and one synchronisation.
#pragma once
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>

#include "../../include/dfmi.h"

namespace dfmi {

struct BatchStage {
    // Where the launch's batch table + tile map (meta_bytes) and per-batch
    // headers (hdr_bytes, zero on entry) go: the table is written to
    // *host_meta and must be at *dev_meta when the launch runs, the headers
    // are at *dev_hdr and, after the call's synchronisation, at *host_hdr.
    // false: the batches path uses the context's own buffers and copies.
    std::function<bool(size_t meta_bytes, size_t hdr_bytes, uint8_t** host_meta, uint8_t** dev_meta,
                       uint8_t** dev_hdr, const uint8_t** host_hdr)>
        locate;
    // Issued once on the stream before the first launch (the H2D of the
    // inputs -- with the table and zeroed headers when locate said so).
    std::function<void(hipStream_t)> copy_in;
    // Issued after the launch(es), before the call's synchronisation.
    std::function<void(hipStream_t)> copy_out;
    // Words the coalesced kernel zeroes (the previous call's headers), and
    // set true once a kernel that does so is enqueued.
    uint64_t* clear_bhdr = nullptr;
    int64_t clear_bhdr_words = 0;
    bool* cleared = nullptr;
    // Device-visible address of *host_hdr: when every batch is one tile, the
    // kernel's blocks write the finished headers there themselves
    // (Launch::hdr_out), and *hdr_written is set -- no header copy needed.
    uint64_t* hdr_out = nullptr;
    bool* hdr_written = nullptr;
};

// Diagnostics (DFMI_DIAG + DFMI_CALL_PROFILE): host time per phase of an
// entry point, averaged over 1000 calls and printed on stderr. mark(i) ends
// phase i; done() ends a call.
struct CallProf {
    const char* name;
    double ph[8] = {};
    long n = 0;
    bool on;
    std::chrono::steady_clock::time_point t;
    explicit CallProf(const char* nm) : name(nm), on(getenv("DFMI_DIAG") && getenv("DFMI_CALL_PROFILE")) {}
    void start() {
        if (on) t = std::chrono::steady_clock::now();
    }
    void mark(int i) {
        if (!on) return;
        const auto u = std::chrono::steady_clock::now();
        ph[i] += std::chrono::duration<double, std::micro>(u - t).count();
        t = u;
    }
    // DFMI_CALL_PROFILE=N: the mean phase times of every N calls (N < 1: 1000)
    const long every = [] {
        const char* e = getenv("DFMI_CALL_PROFILE");
        const long v = e ? atol(e) : 0;
        return v > 0 ? v : 1000L;
    }();
    void done() {
        if (!on || ++n % every) return;
        fprintf(stderr, "dfmi call profile %s (us/call):", name);
        for (double& x : ph) {
            fprintf(stderr, " %.2f", x / (double)every);
            x = 0;
        }
        fprintf(stderr, "\n");
    }
};

// dfmi_filter_project_batches with a caller's staging (NULL: none).
int32_t filter_project_batches_staged(dfmi_context* ctx, const dfmi_program* pred, const dfmi_program* const* projs,
                                      int32_t np, const dfmi_batch* ins, int32_t nb, dfmi_out_column* outs,
                                      uint32_t flags, int32_t* failed, dfmi_error* err, const BatchStage* stage);

}  // namespace dfmi
