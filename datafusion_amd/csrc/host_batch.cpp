// dfmi_filter_project_host: the host-buffer form of one FilterRelation /
// ProjectRelation pull, for callers that hold Arrow batches in host memory
// (the Rust reference's arrow 0.12 buffers, csv::Reader output). Moves the
// batch's buffers into HBM through a pinned staging buffer, runs the fused
// pass (exec.cpp), and copies the exact-size results back into buffers the
// library owns until dfmi_host_result_free.
//
// Replaces, for a host batch, FilterRelation::next (filter.rs:46-72) +
// filter() (filter.rs:80-111) + ProjectRelation::next (projection.rs:45-66).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "dfmi_program.h"
#include "jit.h"

using dfmi::Fail;

#define HIP_TRY(x)                                                                         \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) throw Fail{DFMI_ERR_DEVICE, std::string(#x ": ") + hipGetErrorString(e_)}; \
    } while (0)

// context internals the host path needs (exec.cpp)
namespace dfmi {
int ctx_device(const dfmi_context* c);
hipStream_t ctx_stream(const dfmi_context* c);
void*& ctx_host_arena(dfmi_context* c);
}  // namespace dfmi

// Allocator whose resize() leaves bytes uninitialised: result buffers are
// overwritten by the D2H copy, and zero-filling GBs first costs as much as
// the copy itself.
template <class T>
struct uninit_alloc : std::allocator<T> {
    using std::allocator<T>::allocator;
    template <class U>
    struct rebind {
        using other = uninit_alloc<U>;
    };
    template <class U>
    void construct(U* p) noexcept {
        ::new ((void*)p) U;
    }
    template <class U, class... Args>
    void construct(U* p, Args&&... a) {
        ::new ((void*)p) U(std::forward<Args>(a)...);
    }
};

struct dfmi_host_result {
    struct Col {
        int32_t type = 0;
        int64_t length = 0, null_count = 0;
        std::vector<uint8_t, uninit_alloc<uint8_t>> values;
        std::vector<uint8_t> validity;
        std::vector<int32_t> offsets;
    };
    std::vector<Col> cols;
};

namespace {

int width_of(int t) {
    switch (t) {
        case DFMI_TYPE_INT8: case DFMI_TYPE_UINT8: return 1;
        case DFMI_TYPE_INT16: case DFMI_TYPE_UINT16: return 2;
        case DFMI_TYPE_INT32: case DFMI_TYPE_UINT32: case DFMI_TYPE_FLOAT32: return 4;
        case DFMI_TYPE_INT64: case DFMI_TYPE_UINT64: case DFMI_TYPE_FLOAT64: return 8;
        default: return 0;
    }
}

size_t bitmap_bytes(int64_t n) { return (size_t)((n + 63) / 64) * 8; }
size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

size_t values_bytes(const dfmi_column& c) {
    if (c.type == DFMI_TYPE_BOOLEAN) return (size_t)((c.length + 7) / 8);
    if (c.type == DFMI_TYPE_UTF8) return c.offsets ? (size_t)std::max<int32_t>(0, c.offsets[c.length]) : 0;
    return (size_t)c.length * width_of(c.type);
}

// Grow-only device arena + pinned staging, one per context (the path is
// single-threaded per context, like the reference, context.rs:33).
struct Arena {
    uint8_t* dev = nullptr;
    size_t dev_cap = 0, dev_used = 0;
    uint8_t* pin = nullptr;  // two staging chunks
    size_t pin_cap = 0;
    hipEvent_t drained[2] = {nullptr, nullptr};
    bool in_flight[2] = {false, false};
    void reserve(size_t need) {
        if (need <= dev_cap) return;
        if (dev) (void)hipFree(dev);
        dev = nullptr;
        dev_cap = 0;
        HIP_TRY(hipMalloc((void**)&dev, need));
        dev_cap = need;
    }
    uint8_t* take(size_t n) {
        uint8_t* p = dev + dev_used;
        dev_used += align256(std::max<size_t>(n, 8));
        return p;
    }
};

// The arena lives in the context (created on first use, freed with it), so
// contexts driven from different host threads share nothing.
Arena& arena_of(dfmi_context* c) {
    void*& slot = dfmi::ctx_host_arena(c);
    if (!slot) slot = new Arena();
    return *(Arena*)slot;
}

// Host copy split over a few threads: one core's memcpy (~10-20 GB/s) would
// bound the staging below what PCIe Gen5 moves.
void par_memcpy(uint8_t* dst, const uint8_t* src, size_t n) {
    constexpr size_t kMinPiece = (size_t)4 << 20;
    const int nt = (int)std::min<size_t>(8, std::max<size_t>(1, n / kMinPiece));
    if (nt == 1) {
        memcpy(dst, src, n);
        return;
    }
    const size_t piece = (n + nt - 1) / nt;
    std::vector<std::thread> th;
    for (int i = 1; i < nt; ++i) {
        const size_t o = i * piece;
        if (o < n) th.emplace_back([=] { memcpy(dst + o, src + o, std::min(piece, n - o)); });
    }
    memcpy(dst, src, std::min(piece, n));
    for (auto& t : th) t.join();
}

// H2D of one host buffer through two pinned staging chunks: the host fills
// one chunk while the DMA engine drains the other (chunks keep the pinned
// footprint bounded; pageable hipMemcpy would be staged by the runtime
// anyway, serially).
void h2d(Arena& A, hipStream_t st, void* dst, const void* src, size_t n) {
    if (!n) return;
    constexpr size_t chunk = (size_t)64 << 20;
    if (!A.pin) {
        HIP_TRY(hipHostMalloc((void**)&A.pin, 2 * chunk, hipHostMallocDefault));
        A.pin_cap = 2 * chunk;
        for (auto& e : A.drained) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    int b = 0;
    for (size_t off = 0; off < n; off += chunk, b ^= 1) {
        const size_t m = std::min(chunk, n - off);
        uint8_t* buf = A.pin + b * chunk;
        if (A.in_flight[b]) HIP_TRY(hipEventSynchronize(A.drained[b]));  // chunk b free again
        par_memcpy(buf, (const uint8_t*)src + off, m);
        HIP_TRY(hipMemcpyAsync((uint8_t*)dst + off, buf, m, hipMemcpyHostToDevice, st));
        HIP_TRY(hipEventRecord(A.drained[b], st));
        A.in_flight[b] = true;
    }
    HIP_TRY(hipStreamSynchronize(st));
    A.in_flight[0] = A.in_flight[1] = false;
}

// D2H of one device buffer through the same two pinned chunks: the DMA of
// chunk i+1 overlaps the host copy-out of chunk i.
void d2h(Arena& A, hipStream_t st, void* dst, const void* src, size_t n) {
    if (!n) return;
    constexpr size_t chunk = (size_t)64 << 20;
    if (!A.pin) {
        HIP_TRY(hipHostMalloc((void**)&A.pin, 2 * chunk, hipHostMallocDefault));
        A.pin_cap = 2 * chunk;
        for (auto& e : A.drained) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    const size_t nchunks = (n + chunk - 1) / chunk;
    auto issue = [&](size_t i) {
        const size_t off = i * chunk, m = std::min(chunk, n - off);
        HIP_TRY(hipMemcpyAsync(A.pin + (i & 1) * chunk, (const uint8_t*)src + off, m, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipEventRecord(A.drained[i & 1], st));
    };
    issue(0);
    if (nchunks > 1) issue(1);
    for (size_t i = 0; i < nchunks; ++i) {
        const size_t off = i * chunk, m = std::min(chunk, n - off);
        HIP_TRY(hipEventSynchronize(A.drained[i & 1]));
        par_memcpy((uint8_t*)dst + off, A.pin + (i & 1) * chunk, m);
        if (i + 2 < nchunks) issue(i + 2);
    }
}

void set_err(dfmi_error* err, int32_t code, const std::string& m) {
    if (!err) return;
    err->code = code;
    snprintf(err->message, sizeof err->message, "%s", m.c_str());
}

}  // namespace

namespace dfmi {
void host_arena_release(dfmi_context* c) {
    void*& slot = ctx_host_arena(c);
    Arena* a = (Arena*)slot;
    if (!a) return;
    if (a->dev) (void)hipFree(a->dev);
    if (a->pin) (void)hipHostFree(a->pin);
    for (auto e : a->drained)
        if (e) (void)hipEventDestroy(e);
    delete a;
    slot = nullptr;
}
}  // namespace dfmi

extern "C" int32_t dfmi_filter_project_host(dfmi_context* ctx, const dfmi_program* pred,
                                            const dfmi_program* const* projs, int32_t np,
                                            const dfmi_batch* in, uint32_t flags,
                                            dfmi_host_result** out, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    dfmi_host_result* R = nullptr;
    try {
        if (!ctx || !in || !out || (np > 0 && !projs) || (in->num_columns > 0 && !in->columns))
            throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        *out = nullptr;
        const int64_t n = in->num_rows;
        const int ncols = in->num_columns;
        HIP_TRY(hipSetDevice(dfmi::ctx_device(ctx)));
        hipStream_t st = dfmi::ctx_stream(ctx);
        Arena& A = arena_of(ctx);

        // ---- output types (RuntimeExpr::get_type, or the input columns)
        const int nout = np > 0 ? np : ncols;
        std::vector<int> otype(nout), osrc(nout, -1);
        for (int o = 0; o < nout; ++o) {
            if (np > 0) {
                if (!projs[o]) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL projection"};
                otype[o] = projs[o]->type;
                const dfmi::IrNode& root = projs[o]->ir[projs[o]->root];
                if (root.kind == dfmi::IR_COL) osrc[o] = root.col;
            } else {
                otype[o] = in->columns[o].type;
                osrc[o] = o;
            }
        }

        // ---- arena layout: inputs, then worst-case outputs
        size_t need = 0;
        for (int i = 0; i < ncols; ++i) {
            const dfmi_column& c = in->columns[i];
            if (c.length != n) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "ragged batch"};
            if (c.type == DFMI_TYPE_UTF8 && !c.offsets) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "Utf8 offsets are NULL"};
            if (!c.values && values_bytes(c)) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "column values pointer is NULL"};
            need += align256(std::max<size_t>(values_bytes(c), 8));
            if (c.validity) need += align256(bitmap_bytes(n));
            if (c.type == DFMI_TYPE_UTF8) need += align256((size_t)(n + 1) * 4);
        }
        std::vector<size_t> utf8_cap(nout, 0);
        for (int o = 0; o < nout; ++o) {
            const int t = otype[o];
            if (t == DFMI_TYPE_UTF8) {
                utf8_cap[o] = osrc[o] >= 0 ? values_bytes(in->columns[osrc[o]]) : 0;
                need += align256((size_t)(n + 1) * 4) + align256(std::max<size_t>(utf8_cap[o], 8));
            } else {
                need += align256(t == DFMI_TYPE_BOOLEAN ? bitmap_bytes(n) : (size_t)n * std::max(width_of(t), 1));
            }
            if (t != DFMI_TYPE_UTF8) need += align256(bitmap_bytes(n));
        }
        A.dev_used = 0;
        A.reserve(need);

        // ---- H2D
        std::vector<dfmi_column> dcols(std::max(1, ncols));
        for (int i = 0; i < ncols; ++i) {
            const dfmi_column& c = in->columns[i];
            dfmi_column& d = dcols[i];
            d = c;
            uint8_t* v = A.take(values_bytes(c));
            h2d(A, st, v, c.values, values_bytes(c));
            d.values = v;
            if (c.validity) {
                uint8_t* b = A.take(bitmap_bytes(n));
                h2d(A, st, b, c.validity, (size_t)(n + 7) / 8);
                d.validity = b;
            }
            if (c.type == DFMI_TYPE_UTF8) {
                int32_t* of = (int32_t*)A.take((size_t)(n + 1) * 4);
                h2d(A, st, of, c.offsets, (size_t)(n + 1) * 4);
                d.offsets = of;
            }
        }
        dfmi_batch db = *in;
        db.columns = dcols.data();

        std::vector<dfmi_out_column> oc(std::max(1, nout));
        for (int o = 0; o < nout; ++o) {
            memset(&oc[o], 0, sizeof oc[o]);
            const int t = otype[o];
            if (t == DFMI_TYPE_UTF8) {
                oc[o].offsets = (int32_t*)A.take((size_t)(n + 1) * 4);
                oc[o].data = A.take(utf8_cap[o]);
                oc[o].data_capacity = (int64_t)std::max<size_t>(utf8_cap[o], 8);
            } else {
                oc[o].values = A.take(t == DFMI_TYPE_BOOLEAN ? bitmap_bytes(n) : (size_t)n * std::max(width_of(t), 1));
            }
            if (t != DFMI_TYPE_UTF8) oc[o].validity = A.take(bitmap_bytes(n));
        }

        const int32_t rc = dfmi_filter_project(ctx, pred, projs, np, &db, oc.data(), flags, err);
        if (rc != DFMI_OK) return rc;

        // ---- D2H of the exact results
        R = new dfmi_host_result();
        R->cols.resize(nout);
        for (int o = 0; o < nout; ++o) {
            dfmi_host_result::Col& rc_ = R->cols[o];
            const dfmi_out_column& r = oc[o];
            rc_.type = r.type;
            rc_.length = r.length;
            rc_.null_count = r.null_count;
            const int64_t L = r.length;
            if (r.passthrough_column >= 0) {  // Arc clone of the input column (expression.rs:274)
                const dfmi_column& c = in->columns[r.passthrough_column];
                rc_.values.assign((const uint8_t*)c.values, (const uint8_t*)c.values + values_bytes(c));
                if (c.validity && c.null_count > 0)
                    rc_.validity.assign(c.validity, c.validity + (n + 7) / 8);
                else
                    rc_.null_count = 0;
                if (c.type == DFMI_TYPE_UTF8) rc_.offsets.assign(c.offsets, c.offsets + n + 1);
                continue;
            }
            if (r.type == DFMI_TYPE_UTF8) {
                rc_.offsets.resize((size_t)L + 1);
                HIP_TRY(hipMemcpyAsync(rc_.offsets.data(), r.offsets, (size_t)(L + 1) * 4, hipMemcpyDeviceToHost, st));
                rc_.values.resize((size_t)r.data_length);
                HIP_TRY(hipStreamSynchronize(st));
                d2h(A, st, rc_.values.data(), r.data, (size_t)r.data_length);
            } else {
                const size_t vb = r.type == DFMI_TYPE_BOOLEAN ? (size_t)(L + 7) / 8 : (size_t)L * width_of(r.type);
                rc_.values.resize(vb);
                d2h(A, st, rc_.values.data(), r.values, vb);
            }
            if (r.null_count > 0) {
                rc_.validity.resize((size_t)(L + 7) / 8);
                HIP_TRY(hipMemcpyAsync(rc_.validity.data(), r.validity, rc_.validity.size(), hipMemcpyDeviceToHost, st));
            }
        }
        HIP_TRY(hipStreamSynchronize(st));
        *out = R;
        return DFMI_OK;
    } catch (const Fail& f) {
        delete R;
        set_err(err, f.code, f.msg);
        return f.code;
    } catch (const std::bad_alloc&) {
        delete R;
        set_err(err, DFMI_ERR_INVALID_ARGUMENT, "host allocation failed");
        return DFMI_ERR_INVALID_ARGUMENT;
    }
}

extern "C" int32_t dfmi_host_result_num_columns(const dfmi_host_result* r) { return r ? (int32_t)r->cols.size() : 0; }

extern "C" int32_t dfmi_host_result_column(const dfmi_host_result* r, int32_t i, dfmi_column* view) {
    if (!r || !view || i < 0 || i >= (int32_t)r->cols.size()) return DFMI_ERR_INVALID_ARGUMENT;
    const dfmi_host_result::Col& c = r->cols[i];
    memset(view, 0, sizeof *view);
    view->type = c.type;
    view->length = c.length;
    view->null_count = c.null_count;
    view->validity = c.validity.empty() ? nullptr : c.validity.data();
    view->values = c.values.data();
    view->offsets = c.type == DFMI_TYPE_UTF8 ? c.offsets.data() : nullptr;
    return DFMI_OK;
}

extern "C" void dfmi_host_result_free(dfmi_host_result* r) { delete r; }
