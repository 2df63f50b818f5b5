// dfmi_filter_project_host: the host-buffer form of one FilterRelation /
// ProjectRelation pull, for callers that hold Arrow batches in host memory
// (the Rust reference's arrow 0.12 buffers, csv::Reader output).
//
// Replaces, for a host batch, FilterRelation::next (filter.rs:46-72) +
// filter() (filter.rs:80-111) + ProjectRelation::next (projection.rs:45-66).
//
// Rows are independent (filter.rs:87-91 preserves row order), so a host
// batch is cut into row chunks that flow through a three-stage pipeline over
// three slots (device input + output regions, pinned staging for both):
//
//   host threads : stage-in chunk j      | copy-out chunk j-2
//   H2D stream   : chunk j               (DMA engine, host -> HBM)
//   ctx stream   : fused kernel chunk j-1 (exec.cpp, waits on the H2D event)
//   D2H stream   : results chunk j-1     (DMA engine, HBM -> host)
//
// so both PCIe directions, the kernel and the host copies overlap. Columns
// whose buffers are pinned (dfmi_host_alloc / dfmi_host_register) skip the
// staging copy and are DMA'd straight from the caller's memory. Chunk results
// are concatenated on the host in row order: Utf8 offsets rebased, bitmaps
// bit-shifted; the first error in the reference's evaluation order is taken
// over all chunks (smallest ordinal, then earliest global row).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "dfmi_program.h"
#include "jit.h"
#include "batch_stage.h"
#include "slice.h"

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
uint64_t& ctx_last_err_key(dfmi_context* c);
}  // namespace dfmi

// Allocator whose resize() leaves bytes uninitialised: result buffers are
// overwritten by the chunk copies, and zero-filling GBs first costs as much
// as the copy itself (untouched pages of a worst-case reservation are never
// faulted in).
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

namespace dfmi_host {
// Pinned host blocks that hold results, recycled across calls: a result's
// buffers are the DMA target of the D2H copies (no staging copy-out), and a
// freed result's blocks serve the next call -- fresh pageable buffers would
// cost a page fault per 4 KiB on first touch and a TLB shootdown per page on
// free, which measured slower than PCIe itself. Shared by a
// context and the results it made (a result may outlive its context).
class PinnedPool {
   public:
    struct Blk {
        uint8_t* p = nullptr;
        size_t cap = 0;
    };
    PinnedPool() {
        if (const char* e = getenv("DFMI_HOST_POOL_MB")) limit_ = (size_t)std::max(0ll, atoll(e)) << 20;
    }
    ~PinnedPool() {
        for (auto& kv : free_) (void)hipHostFree(kv.second);
    }
    Blk get(size_t bytes) {
        const size_t cap = round(bytes);
        {
            std::lock_guard<std::mutex> g(m_);
            auto it = free_.lower_bound(cap);
            if (it != free_.end() && it->first <= 2 * cap + ((size_t)2 << 20)) {
                Blk b{(uint8_t*)it->second, it->first};
                free_bytes_ -= it->first;
                free_.erase(it);
                return b;
            }
        }
        void* p = nullptr;
        if (hipHostMalloc(&p, cap, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            {
                std::lock_guard<std::mutex> g(m_);
                trim(0);
            }
            const hipError_t e = hipHostMalloc(&p, cap, hipHostMallocDefault);
            if (e != hipSuccess) throw Fail{DFMI_ERR_DEVICE, std::string("hipHostMalloc (result): ") + hipGetErrorString(e)};
        }
        return {(uint8_t*)p, cap};
    }
    void put(Blk& b) {
        if (!b.p) return;
        std::lock_guard<std::mutex> g(m_);
        free_.emplace(b.cap, b.p);
        free_bytes_ += b.cap;
        b = Blk{};
        trim(limit_);
    }

   private:
    void trim(size_t limit) {  // largest blocks first
        while (free_bytes_ > limit && !free_.empty()) {
            auto it = std::prev(free_.end());
            free_bytes_ -= it->first;
            (void)hipHostFree(it->second);
            free_.erase(it);
        }
    }
    static size_t round(size_t b) {
        b = std::max<size_t>(b, 64);
        const size_t q = b < ((size_t)2 << 20) ? 4096 : ((size_t)2 << 20);
        return (b + q - 1) / q * q;
    }
    std::mutex m_;
    std::multimap<size_t, void*> free_;
    size_t free_bytes_ = 0;
    size_t limit_ = (size_t)8 << 30;  // idle pinned bytes kept for reuse
};
}  // namespace dfmi_host

struct dfmi_host_result {
    struct Col {
        int32_t type = 0;
        int64_t length = 0, null_count = 0, data_length = 0;
        dfmi_host::PinnedPool::Blk values, offsets;               // fixed-width / Utf8 bytes; Utf8 offsets
        std::vector<uint8_t, uninit_alloc<uint8_t>> bits;        // Boolean values
        std::vector<uint8_t, uninit_alloc<uint8_t>> validity;
        bool has_validity = false;
        // dfmi_filter_project_host_batches: views into the result's arena
        const uint8_t* v_values = nullptr;
        const int32_t* v_offsets = nullptr;
        const uint8_t* v_validity = nullptr;
    };
    std::shared_ptr<dfmi_host::PinnedPool> pool;
    std::vector<Col> cols;
    dfmi_host::PinnedPool::Blk arena;  // one block holding every column (batches form)
    ~dfmi_host_result() {
        if (pool) {
            for (Col& c : cols) {
                pool->put(c.values);
                pool->put(c.offsets);
            }
            pool->put(arena);
        }
    }
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

// ---------------------------------------------------------------- pinned memory
// Ranges the DMA engines can read directly: dfmi_host_alloc'd or
// dfmi_host_register'd. Process-wide (a buffer may feed any context).
struct PinRegistry {
    std::mutex m;
    std::map<uintptr_t, std::pair<size_t, bool>> r;  // base -> (bytes, registered (vs allocated))
};
PinRegistry& pins() {
    static PinRegistry* p = new PinRegistry();
    return *p;
}
// Pinned by the runtime (hipHostMalloc'd elsewhere, e.g. a torch pinned
// tensor): asked only for large buffers, whose staging copy would matter.
bool runtime_pinned(const void* p) {
    hipPointerAttribute_t a;
    const hipError_t e = hipPointerGetAttributes(&a, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();  // pageable memory: not an error of this call
        return false;
    }
    return a.type == hipMemoryTypeHost;
}
bool is_pinned(const void* p, size_t n) {
    if (!p || !n) return false;
    {
        PinRegistry& R = pins();
        std::lock_guard<std::mutex> g(R.m);
        auto it = R.r.upper_bound((uintptr_t)p);
        if (it != R.r.begin()) {
            --it;
            if ((uintptr_t)p + n <= it->first + it->second.first) return true;
        }
    }
    return n >= ((size_t)1 << 20) && runtime_pinned(p) && runtime_pinned((const uint8_t*)p + n - 1);
}

// ---------------------------------------------------------------- host threads
// Persistent workers for the host copies: one core's memcpy (~10-20 GB/s)
// would bound the pipeline below what PCIe Gen5 moves. Task i runs on worker
// i % (workers + 1) (the caller is worker 0); run() returns when every worker
// has finished its share of this job, so no worker ever sees a stale job.
class Pool {
   public:
    explicit Pool(int workers) {
        for (int w = 0; w < workers; ++w) th_.emplace_back([this, w] { loop(w + 1); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void run(const std::vector<std::function<void()>>& tasks) {
        if (tasks.empty()) return;
        if (th_.empty() || tasks.size() == 1) {
            for (auto& t : tasks) t();
            return;
        }
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = &tasks;
            remaining_ = (int)th_.size();
            ++epoch_;
        }
        cv_.notify_all();
        share(tasks, 0);
        std::unique_lock<std::mutex> l(m_);
        done_.wait(l, [&] { return remaining_ == 0; });
        job_ = nullptr;
    }
    int ways() const { return (int)th_.size() + 1; }

   private:
    void share(const std::vector<std::function<void()>>& t, int me) {
        for (size_t i = me; i < t.size(); i += th_.size() + 1) t[i]();
    }
    void loop(int me) {
        uint64_t seen = 0;
        for (;;) {
            const std::vector<std::function<void()>>* J;
            {
                std::unique_lock<std::mutex> l(m_);
                cv_.wait(l, [&] { return stop_ || epoch_ != seen; });
                if (stop_) return;
                seen = epoch_;
                J = job_;
            }
            share(*J, me);
            std::lock_guard<std::mutex> g(m_);
            if (--remaining_ == 0) done_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::vector<std::function<void()>>* job_ = nullptr;
    uint64_t epoch_ = 0;
    int remaining_ = 0;
    bool stop_ = false;
};

int host_threads() {
    if (const char* e = getenv("DFMI_HOST_THREADS")) return std::max(1, std::min(64, atoi(e)));
    const int hw = (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(hw > 0 ? hw : 1, 8));
}

// Append a copy of n bytes as tasks of >= 4 MiB each (at most `ways` pieces).
void add_copy(std::vector<std::function<void()>>& T, void* dst, const void* src, size_t n, int ways) {
    if (!n) return;
    constexpr size_t kMin = (size_t)4 << 20;
    const size_t k = std::max<size_t>(1, std::min<size_t>((size_t)ways, n / kMin));
    const size_t piece = ((n + k - 1) / k + 63) & ~(size_t)63;
    for (size_t o = 0; o < n; o += piece) {
        const size_t m = std::min(piece, n - o);
        T.emplace_back([=] { memcpy((uint8_t*)dst + o, (const uint8_t*)src + o, m); });
    }
}

// dst[i] = src[i] + add for i < n (Utf8 offset rebase while copying out).
void add_copy_rebase(std::vector<std::function<void()>>& T, int32_t* dst, const int32_t* src, size_t n,
                     int32_t add, int ways) {
    if (!n) return;
    constexpr size_t kMin = (size_t)1 << 20;
    const size_t k = std::max<size_t>(1, std::min<size_t>((size_t)ways, n / kMin));
    const size_t piece = (n + k - 1) / k;
    for (size_t o = 0; o < n; o += piece) {
        const size_t m = std::min(piece, n - o);
        T.emplace_back([=] {
            for (size_t i = 0; i < m; ++i) dst[o + i] = src[o + i] + add;
        });
    }
}

inline uint64_t ld64(const uint8_t* p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v;
}
inline void st64(uint8_t* p, uint64_t v) { memcpy(p, &v, 8); }

// Write bits [0, n) of LSB-first bitmap src at bit position pos of dst.
// Bits of dst below pos are kept; bits past pos + n may be overwritten (the
// next chunk's append, or finish_bitmap, owns them). src holds >= ceil(n/8)
// bytes; dst >= ceil((pos + n)/8) bytes plus 8 of slack.
void append_bits(uint8_t* dst, int64_t pos, const uint8_t* src, int64_t n) {
    if (n <= 0) return;
    uint8_t* d = dst + (pos >> 3);
    const int sh = (int)(pos & 7);
    const int64_t nb = (n + 7) >> 3;
    if (!sh) {
        memcpy(d, src, (size_t)nb);
        return;
    }
    uint8_t carry = d[0] & (uint8_t)((1u << sh) - 1);
    int64_t i = 0;
    for (; i + 8 <= nb; i += 8) {
        const uint64_t v = ld64(src + i);
        st64(d + i, (v << sh) | carry);
        carry = (uint8_t)(v >> (64 - sh));
    }
    for (; i < nb; ++i) {
        const uint8_t b = src[i];
        d[i] = (uint8_t)(b << sh) | carry;
        carry = (uint8_t)(b >> (8 - sh));
    }
    d[nb] = carry;
}

// Set bits [pos, pos + n) (a chunk whose result holds no nulls).
void append_ones(uint8_t* dst, int64_t pos, int64_t n) {
    if (n <= 0) return;
    int64_t p = pos, e = pos + n;
    while (p < e && (p & 7)) {
        dst[p >> 3] |= (uint8_t)(1u << (p & 7));
        ++p;
    }
    if (p < e) {
        const int64_t full = (e - p) >> 3;
        memset(dst + (p >> 3), 0xff, (size_t)full);
        p += full * 8;
        if (p < e) dst[p >> 3] = (uint8_t)((1u << (e - p)) - 1);
    }
}

// Zero the bits of the last byte past n (arrow's bitmaps carry no garbage).
void finish_bitmap(uint8_t* b, int64_t n) {
    if (n & 7) b[n >> 3] &= (uint8_t)((1u << (n & 7)) - 1);
}

// ---------------------------------------------------------------- arena
constexpr int kSlots = 3;
// a host batch up to this size skips the chunk pipeline (one H2D, one
// launch, one D2H, one synchronisation: dfmi_filter_project_host)
constexpr size_t kZeroCopyBytes = 8 << 20;  // inputs + batch table read in place up to this size (DFMI_HOST_ZC;
                                             // 256 x 1024-row batches: 1.28 -> 1.00 us per batch, profiles/r04/zc_ab2.log)
constexpr int64_t kSmallRows = 1 << 16;
constexpr size_t kSmallBytes = (size_t)4 << 20;

// DFMI_HOST_PROFILE=1: per-call phase times on stderr (diagnostics only).
struct PhaseClock {
    bool on = false;
    double t[8] = {};
    std::chrono::steady_clock::time_point t0;
    void start() {
        if (on) t0 = std::chrono::steady_clock::now();
    }
    void stop(int i) {
        if (on) t[i] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
};

// Grow-only device + pinned regions, copy streams and events, one set per
// context (a context is driven by one host thread, context.rs:33).
struct Arena {
    int device = -1;
    uint8_t* dev = nullptr;
    size_t dev_cap = 0;
    uint8_t* pin = nullptr;
    uint8_t* pin_dev = nullptr;  // the device's address of pin (zero-copy reads)
    size_t pin_cap = 0;
    hipStream_t h2d = nullptr, d2h = nullptr;
    hipEvent_t h2d_done[kSlots] = {}, d2h_done[kSlots] = {}, kdone[kSlots] = {};
    bool slot_used[kSlots] = {};
    Pool* pool = nullptr;
    std::shared_ptr<dfmi_host::PinnedPool> results = std::make_shared<dfmi_host::PinnedPool>();
    void init(int dev_id) {
        if (h2d) return;
        device = dev_id;
        HIP_TRY(hipStreamCreateWithFlags(&h2d, hipStreamNonBlocking));
        HIP_TRY(hipStreamCreateWithFlags(&d2h, hipStreamNonBlocking));
        for (int s = 0; s < kSlots; ++s) {
            HIP_TRY(hipEventCreateWithFlags(&h2d_done[s], hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&d2h_done[s], hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&kdone[s], hipEventDisableTiming));
        }
        pool = new Pool(host_threads() - 1);
    }
    void reserve_dev(size_t need) {
        if (need <= dev_cap) return;
        if (dev) (void)hipFree(dev);
        dev = nullptr;
        dev_cap = 0;
        HIP_TRY(hipMalloc((void**)&dev, need));
        dev_cap = need;
    }
    // dfmi_filter_project_host_batches' device region: two halves of
    // [headers (right-aligned in hcap) | outputs (ocap)], used alternately,
    // then the inputs + batch table (icap). A call's kernel zeroes the
    // headers the previous call left in the other half (hb_dirty: bytes at
    // the end of a half's header room that are not known to be zero).
    uint8_t* hb = nullptr;
    size_t hb_hcap = 0, hb_ocap = 0, hb_icap = 0, hb_dirty[2] = {0, 0};
    int hb_half = 0;
    void reserve_hb(size_t H, size_t OB, size_t IM, hipStream_t st) {
        if (hb && H <= hb_hcap && OB <= hb_ocap && IM <= hb_icap) return;
        if (hb) {
            HIP_TRY(hipStreamSynchronize(st));  // (earlier calls synchronised: nothing uses it)
            (void)hipFree(hb);
        }
        hb = nullptr;
        hb_hcap = std::max(H, std::max(hb_hcap, (size_t)64 << 10));
        hb_ocap = std::max(OB, hb_ocap);
        hb_icap = std::max(IM, hb_icap);
        HIP_TRY(hipMalloc((void**)&hb, 2 * (hb_hcap + hb_ocap) + hb_icap));
        for (int h = 0; h < 2; ++h) HIP_TRY(hipMemsetAsync(hb + h * (hb_hcap + hb_ocap), 0, hb_hcap, st));
        hb_dirty[0] = hb_dirty[1] = 0;
    }
    uint8_t* hb_half_base(int h) const { return hb + (size_t)h * (hb_hcap + hb_ocap); }
    void reserve_pin(size_t need) {
        if (need <= pin_cap) return;
        if (pin) (void)hipHostFree(pin);
        pin = nullptr;
        pin_cap = 0;
        HIP_TRY(hipHostMalloc((void**)&pin, need, hipHostMallocDefault));
        pin_cap = need;
        HIP_TRY(hipHostGetDevicePointer((void**)&pin_dev, pin, 0));
    }
    // headers of the caller-owned form (dfmi_filter_project_host_batches_into)
    uint8_t *hdr_pin = nullptr, *hdr_pin_dev = nullptr;
    size_t hdr_pin_cap = 0;
    void reserve_hdr_pin(size_t need) {
        if (need <= hdr_pin_cap) return;
        if (hdr_pin) (void)hipHostFree(hdr_pin);
        hdr_pin = nullptr;
        hdr_pin_cap = 0;
        const size_t cap = std::max<size_t>(need, (size_t)64 << 10);
        HIP_TRY(hipHostMalloc((void**)&hdr_pin, cap, hipHostMallocDefault));
        hdr_pin_cap = cap;
        HIP_TRY(hipHostGetDevicePointer((void**)&hdr_pin_dev, hdr_pin, 0));
    }
    void release() {
        if (h2d) (void)hipStreamSynchronize(h2d);
        if (hdr_pin) (void)hipHostFree(hdr_pin);
        if (d2h) (void)hipStreamSynchronize(d2h);
        if (dev) (void)hipFree(dev);
        if (hb) (void)hipFree(hb);
        if (pin) (void)hipHostFree(pin);
        for (int s = 0; s < kSlots; ++s) {
            if (h2d_done[s]) (void)hipEventDestroy(h2d_done[s]);
            if (d2h_done[s]) (void)hipEventDestroy(d2h_done[s]);
            if (kdone[s]) (void)hipEventDestroy(kdone[s]);
        }
        if (h2d) (void)hipStreamDestroy(h2d);
        if (d2h) (void)hipStreamDestroy(d2h);
        delete pool;
    }
};

Arena& arena_of(dfmi_context* c) {
    void*& slot = dfmi::ctx_host_arena(c);
    if (!slot) slot = new Arena();
    return *(Arena*)slot;
}

void set_err(dfmi_error* err, int32_t code, const std::string& m) {
    if (!err) return;
    err->code = code;
    snprintf(err->message, sizeof err->message, "%s", m.c_str());
}

// One device/staging buffer of a chunk: `off` in the slot's region, copied
// from host `src` (input) or into the result (output).
struct Buf {
    size_t off = 0, bytes = 0;
    const uint8_t* src = nullptr;
    bool direct = false;  // src is pinned: DMA from it, no staging copy
};

struct Chunk {
    int64_t r0 = 0, rows = 0;
};

// Rows per chunk: ~48 MiB of input per chunk (a multiple of 512 rows, so
// chunk validity bitmaps start on a 64-bit word); one chunk for a batch up to
// 1.5 chunks. DFMI_HOST_CHUNK_ROWS overrides (tests / diagnostics).
int64_t chunk_rows_for(int64_t n, double in_bytes_per_row) {
    int64_t r;
    if (const char* e = getenv("DFMI_HOST_CHUNK_ROWS")) {
        r = std::max<int64_t>(512, atoll(e));
    } else {
        constexpr double kTarget = 48.0 * (1 << 20);
        r = (int64_t)(kTarget / std::max(in_bytes_per_row, 1.0));
        r = std::max<int64_t>(r, 1 << 16);
        if (n <= r + r / 2) return std::max<int64_t>(n, 1);
    }
    r &= ~(int64_t)511;
    r = std::max<int64_t>(r, 512);
    return n <= r ? std::max<int64_t>(n, 1) : r;
}

}  // namespace

namespace dfmi {
void host_arena_release(dfmi_context* c) {
    void*& slot = ctx_host_arena(c);
    Arena* a = (Arena*)slot;
    if (!a) return;
    a->release();
    delete a;
    slot = nullptr;
}
}  // namespace dfmi

// ---------------------------------------------------------------- pinned host memory API
extern "C" int32_t dfmi_host_alloc(size_t bytes, void** out, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    if (!out) {
        set_err(err, DFMI_ERR_INVALID_ARGUMENT, "out is NULL");
        return DFMI_ERR_INVALID_ARGUMENT;
    }
    *out = nullptr;
    void* p = nullptr;
    const hipError_t e = hipHostMalloc(&p, std::max<size_t>(bytes, 64), hipHostMallocPortable);
    if (e != hipSuccess) {
        set_err(err, DFMI_ERR_DEVICE, std::string("hipHostMalloc: ") + hipGetErrorString(e));
        return DFMI_ERR_DEVICE;
    }
    {
        PinRegistry& R = pins();
        std::lock_guard<std::mutex> g(R.m);
        R.r[(uintptr_t)p] = {std::max<size_t>(bytes, 64), false};
    }
    *out = p;
    return DFMI_OK;
}

extern "C" int32_t dfmi_host_free(void* p) {
    if (!p) return DFMI_OK;
    {
        PinRegistry& R = pins();
        std::lock_guard<std::mutex> g(R.m);
        auto it = R.r.find((uintptr_t)p);
        if (it == R.r.end() || it->second.second) return DFMI_ERR_INVALID_ARGUMENT;
        R.r.erase(it);
    }
    return hipHostFree(p) == hipSuccess ? DFMI_OK : DFMI_ERR_DEVICE;
}

extern "C" int32_t dfmi_host_register(void* p, size_t bytes, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    if (!p || !bytes) {
        set_err(err, DFMI_ERR_INVALID_ARGUMENT, "NULL or empty range");
        return DFMI_ERR_INVALID_ARGUMENT;
    }
    const hipError_t e = hipHostRegister(p, bytes, hipHostRegisterPortable);
    if (e != hipSuccess) {
        set_err(err, DFMI_ERR_DEVICE, std::string("hipHostRegister: ") + hipGetErrorString(e));
        return DFMI_ERR_DEVICE;
    }
    PinRegistry& R = pins();
    std::lock_guard<std::mutex> g(R.m);
    R.r[(uintptr_t)p] = {bytes, true};
    return DFMI_OK;
}

extern "C" int32_t dfmi_host_unregister(void* p) {
    if (!p) return DFMI_ERR_INVALID_ARGUMENT;
    {
        PinRegistry& R = pins();
        std::lock_guard<std::mutex> g(R.m);
        auto it = R.r.find((uintptr_t)p);
        if (it == R.r.end() || !it->second.second) return DFMI_ERR_INVALID_ARGUMENT;
        R.r.erase(it);
    }
    return hipHostUnregister(p) == hipSuccess ? DFMI_OK : DFMI_ERR_DEVICE;
}

// ---------------------------------------------------------------- the pull
extern "C" int32_t dfmi_filter_project_host(dfmi_context* ctx, const dfmi_program* pred,
                                            const dfmi_program* const* projs, int32_t np,
                                            const dfmi_batch* in, uint32_t flags,
                                            dfmi_host_result** out, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    dfmi_host_result* R = nullptr;
    Arena* Ap = nullptr;
    dfmi_host::PinnedPool::Blk bm_stage;
    try {
        if (!ctx || !in || !out || (np > 0 && !projs) || (in->num_columns > 0 && !in->columns))
            throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        *out = nullptr;
        dfmi::ctx_last_err_key(ctx) = ~0ull;
        dfmi::Unsliced us_;  // sliced arrays (arrow offsets): offset-0 views / shifted bitmaps (slice.cpp)
        if (dfmi::any_offset(in, 1)) in = dfmi::unslice(in, 1, us_, false, nullptr);
        const int64_t n = in->num_rows;
        const int ncols = in->num_columns;
        if (n < 0) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "negative row count"};
        // ---- small batches (csv_sql.rs:49's 1024 rows): no chunk pipeline,
        // copy streams or host threads -- the one-batch form of the
        // host-batches path: pack into pinned memory, one H2D, the launch and
        // one D2H of the output region on the context stream, one sync
        static const bool chunk_env = getenv("DFMI_HOST_CHUNK_ROWS") != nullptr;
        if (n <= kSmallRows && !chunk_env) {
            size_t bytes = 0;
            for (int i = 0; i < ncols; ++i) {
                const dfmi_column& c = in->columns[i];
                bytes += values_bytes(c) + (c.validity ? (size_t)(n + 7) / 8 : 0) +
                         (c.type == DFMI_TYPE_UTF8 ? (size_t)(n + 1) * 4 : 0);
            }
            if (bytes <= kSmallBytes) {
                int32_t failed = -1;
                const int32_t rc = dfmi_filter_project_host_batches(ctx, pred, projs, np, in, 1, flags, out, &failed, err);
                if (rc != DFMI_OK && *out) {
                    dfmi_host_result_free(*out);
                    *out = nullptr;
                }
                return rc;
            }
        }
        HIP_TRY(hipSetDevice(dfmi::ctx_device(ctx)));
        hipStream_t st = dfmi::ctx_stream(ctx);
        Arena& A = arena_of(ctx);
        A.init(dfmi::ctx_device(ctx));
        Ap = &A;
        const int ways = A.pool->ways();
        PhaseClock pc;
        pc.on = getenv("DFMI_HOST_PROFILE") != nullptr;
        const auto call_t0 = std::chrono::steady_clock::now();

        // ---- output types (RuntimeExpr::get_type, or the input columns) and
        // the input columns the device needs
        const int nout = np > 0 ? np : ncols;
        std::vector<int> otype(nout), osrc(nout, -1);
        std::vector<char> passthrough(nout, 0), need(std::max(1, ncols), 0);
        auto mark = [&](const dfmi_program* p) {
            for (const dfmi::IrNode& nd : p->ir)
                if (nd.kind == dfmi::IR_COL && nd.col >= 0 && nd.col < ncols) need[nd.col] = 1;
        };
        if (pred) mark(pred);
        for (int o = 0; o < nout; ++o) {
            if (np > 0) {
                if (!projs[o]) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL projection"};
                otype[o] = projs[o]->type;
                const dfmi::IrNode& root = projs[o]->ir[projs[o]->root];
                if (root.kind == dfmi::IR_COL) osrc[o] = root.col;
                passthrough[o] = !pred && root.kind == dfmi::IR_COL;
                if (!passthrough[o]) mark(projs[o]);
            } else {
                otype[o] = in->columns[o].type;
                osrc[o] = o;
                if (pred) need[o] = 1;  // FilterRelation gathers every column (filter.rs:80-111)
            }
        }
        double in_bpr = 0;
        for (int i = 0; i < ncols; ++i) {
            const dfmi_column& c = in->columns[i];
            if (c.length != n) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "ragged batch"};
            if (c.type == DFMI_TYPE_UTF8 && !c.offsets) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "Utf8 offsets are NULL"};
            if (!c.values && values_bytes(c)) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "column values pointer is NULL"};
            if (!need[i]) continue;
            in_bpr += c.type == DFMI_TYPE_BOOLEAN ? 0.125 : width_of(c.type);
            if (c.validity) in_bpr += 0.125;
            if (c.type == DFMI_TYPE_UTF8) in_bpr += 4.0 + (n ? (double)values_bytes(c) / n : 0);
        }

        // ---- chunks
        const int64_t crows = chunk_rows_for(n, in_bpr);
        std::vector<Chunk> chunks;
        for (int64_t r0 = 0; r0 < n || chunks.empty(); r0 += crows) chunks.push_back({r0, std::min(crows, n - r0)});
        const int nch = (int)chunks.size();
        const int64_t rows_cap = std::max<int64_t>(crows, 1);

        // input buffers of chunk k: staged ones first (one contiguous range,
        // one DMA), then the ones DMA'd from pinned caller memory
        struct InPlan {
            std::vector<Buf> bufs;  // per column: values, validity, offsets (bytes == 0: absent)
            size_t staged_bytes = 0, total = 0;
        };
        auto plan_in = [&](const Chunk& ch) {
            InPlan P;
            P.bufs.assign((size_t)3 * std::max(ncols, 1), Buf{});
            for (int pass = 0; pass < 2; ++pass) {
                for (int i = 0; i < ncols; ++i) {
                    if (!need[i]) continue;
                    const dfmi_column& c = in->columns[i];
                    const int64_t r0 = ch.r0, m = ch.rows;
                    Buf v, b, of;
                    if (c.type == DFMI_TYPE_UTF8) {
                        const int32_t s0 = c.offsets[r0], s1 = c.offsets[r0 + m];
                        v.src = (const uint8_t*)c.values + s0;
                        v.bytes = (size_t)std::max(0, s1 - s0);
                        of.src = (const uint8_t*)(c.offsets + r0);
                        of.bytes = (size_t)(m + 1) * 4;
                    } else {
                        const size_t w = c.type == DFMI_TYPE_BOOLEAN ? 0 : (size_t)width_of(c.type);
                        v.src = (const uint8_t*)c.values + (w ? r0 * (int64_t)w : r0 / 8);
                        v.bytes = w ? (size_t)m * w : (size_t)(m + 7) / 8;
                    }
                    if (c.validity) {
                        b.src = c.validity + r0 / 8;
                        b.bytes = (size_t)(m + 7) / 8;
                    }
                    Buf* dst[3] = {&v, &b, &of};
                    const bool exists[3] = {true, c.validity != nullptr, c.type == DFMI_TYPE_UTF8};
                    for (int k = 0; k < 3; ++k) {
                        if (!exists[k]) continue;
                        Buf& x = *dst[k];
                        x.direct = x.bytes && is_pinned(x.src, x.bytes);
                        if (x.direct != (pass == 1)) continue;
                        // device side: >= 8 bytes (a kernel reads whole words)
                        x.off = P.total;
                        P.total += align256(std::max<size_t>(x.bytes + 8, 16));
                        if (pass == 0) P.staged_bytes = P.total;
                        P.bufs[(size_t)3 * i + k] = x;
                    }
                }
            }
            return P;
        };
        size_t in_cap = 0;
        std::vector<InPlan> inplans(nch);
        for (int k = 0; k < nch; ++k) {
            inplans[k] = plan_in(chunks[k]);
            in_cap = std::max(in_cap, inplans[k].total);
        }
        in_cap = std::max<size_t>(in_cap, 256);

        // output region of a slot (worst case for rows_cap rows); bitmap
        // outputs (Boolean values, validity) get a staging index
        struct OutPlan {
            size_t values = 0, validity = 0, offsets = 0, data = 0;
            size_t values_cap = 0, data_cap = 0;
            int bm_values = -1, bm_valid = -1;
        };
        std::vector<OutPlan> op(nout);
        size_t out_cap = 0;
        int n_bm = 0;
        for (int o = 0; o < nout; ++o) {
            if (passthrough[o]) continue;
            const int t = otype[o];
            OutPlan& p = op[o];
            if (t == DFMI_TYPE_UTF8) {
                size_t dc = 8;
                if (osrc[o] >= 0)
                    for (int k = 0; k < nch; ++k) dc = std::max(dc, inplans[k].bufs[(size_t)3 * osrc[o]].bytes);
                p.offsets = out_cap;
                out_cap += align256((size_t)(rows_cap + 1) * 4);
                p.data = out_cap;
                p.data_cap = dc;
                out_cap += align256(dc + 8);
            } else {
                p.values = out_cap;
                p.values_cap = t == DFMI_TYPE_BOOLEAN ? bitmap_bytes(rows_cap) : (size_t)rows_cap * std::max(width_of(t), 1);
                out_cap += align256(p.values_cap + 8);
                p.validity = out_cap;
                out_cap += align256(bitmap_bytes(rows_cap) + 8);
                if (t == DFMI_TYPE_BOOLEAN) p.bm_values = n_bm++;
                p.bm_valid = n_bm++;
            }
        }
        out_cap = std::max<size_t>(out_cap, 256);
        // a small single chunk returns its whole output region in one DMA
        // (one latency) and is copied into the results on the host
        const bool small = nch == 1 && out_cap <= ((size_t)1 << 20);
        const size_t slot_dev = in_cap + out_cap;
        A.reserve_dev(slot_dev * kSlots);
        A.reserve_pin(in_cap * kSlots + (small ? out_cap : 0));
        auto dev_in = [&](int s) { return A.dev + (size_t)s * slot_dev; };
        auto dev_out = [&](int s) { return A.dev + (size_t)s * slot_dev + in_cap; };
        auto pin_in = [&](int s) { return A.pin + (size_t)s * in_cap; };
        uint8_t* const pin_small = A.pin + (size_t)kSlots * in_cap;
        const size_t bm_chunk = bitmap_bytes(rows_cap);
        if (!small && n_bm) bm_stage = A.results->get((size_t)n_bm * nch * bm_chunk);
        auto bm_at = [&](int idx, int k) { return bm_stage.p + ((size_t)idx * nch + k) * bm_chunk; };

        // ---- results: pinned blocks sized for the worst case (DMA targets)
        R = new dfmi_host_result();
        R->pool = A.results;
        R->cols.resize(nout);
        for (int o = 0; o < nout; ++o) {
            dfmi_host_result::Col& rc = R->cols[o];
            rc.type = otype[o];
            if (passthrough[o]) continue;
            const int t = otype[o];
            if (t == DFMI_TYPE_UTF8) {
                size_t total = 0;
                if (osrc[o] >= 0) total = values_bytes(in->columns[osrc[o]]);
                rc.offsets = A.results->get((size_t)(n + 1) * 4);
                ((int32_t*)rc.offsets.p)[0] = 0;
                rc.values = A.results->get(total + 8);
            } else {
                if (t == DFMI_TYPE_BOOLEAN)
                    rc.bits.resize((size_t)(n + 7) / 8 + 16);
                else
                    rc.values = A.results->get((size_t)n * std::max(width_of(t), 1) + 8);
                rc.validity.resize((size_t)(n + 7) / 8 + 16);
            }
        }

        // ---- pipeline
        struct Done {
            std::vector<dfmi_out_column> oc;
            int64_t row_base = 0;
            std::vector<int64_t> byte_base;
        };
        std::vector<Done> done(nch);
        int64_t rows_so_far = 0;
        std::vector<int64_t> bytes_so_far(nout, 0), nulls(nout, 0);
        bool failed = false;
        // first error in the reference's evaluation order over all chunks
        struct {
            bool set = false;
            uint64_t key = ~0ull;
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
        } first;
        std::vector<std::function<void()>> tasks;

        auto stage_in = [&](int k) {
            const InPlan& P = inplans[k];
            uint8_t* pin = pin_in(k % kSlots);
            for (const Buf& b : P.bufs)
                if (b.bytes && !b.direct) add_copy(tasks, pin + b.off, b.src, b.bytes, ways);
        };
        auto issue_h2d = [&](int k) {
            const int s = k % kSlots;
            const InPlan& P = inplans[k];
            // the slot's inputs were read by the kernel of chunk k - kSlots
            if (A.slot_used[s]) HIP_TRY(hipStreamWaitEvent(A.h2d, A.kdone[s], 0));
            if (P.staged_bytes)
                HIP_TRY(hipMemcpyAsync(dev_in(s), pin_in(s), P.staged_bytes, hipMemcpyHostToDevice, A.h2d));
            for (const Buf& b : P.bufs)
                if (b.bytes && b.direct)
                    HIP_TRY(hipMemcpyAsync(dev_in(s) + b.off, b.src, b.bytes, hipMemcpyHostToDevice, A.h2d));
            HIP_TRY(hipEventRecord(A.h2d_done[s], A.h2d));
        };
        auto run_kernel = [&](int k) {
            const int s = k % kSlots;
            const Chunk& ch = chunks[k];
            const InPlan& P = inplans[k];
            std::vector<dfmi_column> dcols(std::max(1, ncols));
            for (int i = 0; i < ncols; ++i) {
                const dfmi_column& c = in->columns[i];
                dfmi_column& d = dcols[i];
                d = c;
                d.length = ch.rows;
                d.values = nullptr;
                d.validity = nullptr;
                d.offsets = nullptr;
                if (!need[i]) continue;
                const Buf& v = P.bufs[(size_t)3 * i];
                const Buf& b = P.bufs[(size_t)3 * i + 1];
                const Buf& of = P.bufs[(size_t)3 * i + 2];
                uint8_t* base = dev_in(s);
                if (c.type == DFMI_TYPE_UTF8) {
                    d.offsets = (const int32_t*)(base + of.off);
                    // offsets stay absolute: the bytes pointer is shifted by the
                    // chunk's first offset (the kernel only forms bytes + offset)
                    d.values = base + v.off - c.offsets[ch.r0];
                } else {
                    d.values = base + v.off;
                }
                if (c.validity) d.validity = base + b.off;
            }
            dfmi_batch db = *in;
            db.num_rows = ch.rows;
            db.columns = dcols.data();
            Done& D = done[k];
            D.oc.assign(std::max(1, nout), dfmi_out_column{});
            uint8_t* ob = dev_out(s);
            for (int o = 0; o < nout; ++o) {
                dfmi_out_column& c = D.oc[o];
                memset(&c, 0, sizeof c);
                if (passthrough[o]) continue;
                if (otype[o] == DFMI_TYPE_UTF8) {
                    c.offsets = (int32_t*)(ob + op[o].offsets);
                    c.data = ob + op[o].data;
                    c.data_capacity = (int64_t)op[o].data_cap;
                } else {
                    c.values = ob + op[o].values;
                    c.validity = ob + op[o].validity;
                }
            }
            HIP_TRY(hipStreamWaitEvent(st, A.h2d_done[s], 0));
            if (A.slot_used[s]) HIP_TRY(hipStreamWaitEvent(st, A.d2h_done[s], 0));  // its output region is free
            dfmi_error e{};
            const int32_t rc = dfmi_filter_project(ctx, pred, projs, np, &db, D.oc.data(), flags, &e);
            if (rc != DFMI_OK) {
                uint64_t key = dfmi::ctx_last_err_key(ctx);
                if (key == ~0ull) throw Fail{rc, e.message};  // outside the evaluation order: fatal now
                if (rc == DFMI_ERR_DIVIDE_BY_ZERO || rc == DFMI_ERR_PANIC) {
                    // device error: make the row global (key = ordinal << 44 | row << 4)
                    const uint64_t ord = key >> 44, row = ((key >> 4) & ((1ull << 40) - 1)) + (uint64_t)ch.r0;
                    key = ord << 44 | row << 4;
                }
                first.offer(key, rc, e.message);
                failed = true;
                return;
            }
            // the D2H of these results (and the slot's next H2D) run on other
            // streams: they wait for the kernel on the device, not the host
            HIP_TRY(hipEventRecord(A.kdone[s], st));
            HIP_TRY(hipStreamWaitEvent(A.d2h, A.kdone[s], 0));
            D.row_base = rows_so_far;
            D.byte_base.assign(nout, 0);
            int64_t L = 0;
            for (int o = 0; o < nout; ++o) {
                if (passthrough[o]) continue;
                L = D.oc[o].length;
                D.byte_base[o] = bytes_so_far[o];
                bytes_so_far[o] += D.oc[o].data_length;
                nulls[o] += D.oc[o].null_count;
            }
            rows_so_far += L;
        };
        // D2H of chunk k's results straight into the result blocks (bitmaps
        // into per-chunk staging, merged bit-shifted at the end)
        auto issue_d2h = [&](int k) {
            if (failed) return;
            const int s = k % kSlots;
            const Done& D = done[k];
            const uint8_t* dob = dev_out(s);
            auto cp = [&](void* dst, const uint8_t* src, size_t b) {
                if (b) HIP_TRY(hipMemcpyAsync(dst, src, b, hipMemcpyDeviceToHost, A.d2h));
            };
            if (small) {
                cp(pin_small, dob, out_cap);
            } else {
                for (int o = 0; o < nout; ++o) {
                    if (passthrough[o]) continue;
                    dfmi_host_result::Col& rc = R->cols[o];
                    const dfmi_out_column& c = D.oc[o];
                    const int64_t L = c.length;
                    const int t = otype[o];
                    if (t == DFMI_TYPE_UTF8) {
                        cp(rc.offsets.p + (D.row_base + 1) * 4, dob + op[o].offsets + 4, (size_t)L * 4);
                        cp(rc.values.p + D.byte_base[o], dob + op[o].data, (size_t)c.data_length);
                        continue;
                    }
                    if (t == DFMI_TYPE_BOOLEAN)
                        cp(bm_at(op[o].bm_values, k), dob + op[o].values, (size_t)(L + 7) / 8);
                    else
                        cp(rc.values.p + D.row_base * width_of(t), dob + op[o].values, (size_t)L * width_of(t));
                    if (c.null_count > 0) cp(bm_at(op[o].bm_valid, k), dob + op[o].validity, (size_t)(L + 7) / 8);
                }
            }
            HIP_TRY(hipEventRecord(A.d2h_done[s], A.d2h));
            A.slot_used[s] = true;
        };

        pc.t[7] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - call_t0).count();
        for (int j = 0; j <= nch; ++j) {
            // (after an error later chunks still run: one of them may hold an
            // error earlier in the evaluation order)
            if (j < nch) {
                pc.start();
                tasks.clear();
                stage_in(j);
                A.pool->run(tasks);
                pc.stop(0);
                pc.start();
                issue_h2d(j);
                pc.stop(3);
            }
            if (j >= 1) {
                pc.start();
                run_kernel(j - 1);
                pc.stop(4);
                pc.start();
                issue_d2h(j - 1);
                pc.stop(5);
            }
        }
        pc.start();
        HIP_TRY(hipStreamSynchronize(A.h2d));
        HIP_TRY(hipStreamSynchronize(A.d2h));
        for (int s = 0; s < kSlots; ++s) A.slot_used[s] = false;
        pc.stop(6);
        if (failed) {
            dfmi::ctx_last_err_key(ctx) = first.key;
            throw Fail{first.code, first.msg};
        }

        // ---- finish: Utf8 rebase, bitmaps, small-chunk copies, lengths,
        // passthrough copies
        pc.start();
        tasks.clear();
        for (int o = 0; o < nout; ++o) {
            dfmi_host_result::Col& rc = R->cols[o];
            if (passthrough[o]) {  // Arc clone of the input column (expression.rs:274)
                const dfmi_column& c = in->columns[osrc[o]];
                rc.length = n;
                rc.null_count = c.validity ? c.null_count : 0;
                rc.values = A.results->get(values_bytes(c) + 8);
                add_copy(tasks, rc.values.p, c.values, values_bytes(c), ways);
                if (c.validity && c.null_count > 0) {
                    rc.validity.resize((size_t)(n + 7) / 8);
                    add_copy(tasks, rc.validity.data(), c.validity, (size_t)(n + 7) / 8, ways);
                    rc.has_validity = true;
                } else {
                    rc.null_count = 0;
                }
                if (c.type == DFMI_TYPE_UTF8) {
                    rc.offsets = A.results->get((size_t)(n + 1) * 4);
                    add_copy(tasks, rc.offsets.p, c.offsets, (size_t)(n + 1) * 4, ways);
                }
                continue;
            }
            const int t = otype[o];
            rc.length = rows_so_far;
            rc.null_count = nulls[o];
            rc.has_validity = t != DFMI_TYPE_UTF8 && nulls[o] > 0;
            if (t == DFMI_TYPE_UTF8) rc.data_length = bytes_so_far[o];
            if (small) {
                const dfmi_out_column& c = done[0].oc[o];
                const int64_t L = c.length;
                if (t == DFMI_TYPE_UTF8) {
                    add_copy(tasks, rc.offsets.p + 4, pin_small + op[o].offsets + 4, (size_t)L * 4, ways);
                    add_copy(tasks, rc.values.p, pin_small + op[o].data, (size_t)c.data_length, ways);
                    continue;
                }
                if (t == DFMI_TYPE_BOOLEAN)
                    add_copy(tasks, rc.bits.data(), pin_small + op[o].values, (size_t)(L + 7) / 8, ways);
                else
                    add_copy(tasks, rc.values.p, pin_small + op[o].values, (size_t)L * width_of(t), ways);
                if (rc.has_validity) add_copy(tasks, rc.validity.data(), pin_small + op[o].validity, (size_t)(L + 7) / 8, ways);
                continue;
            }
            if (t == DFMI_TYPE_UTF8) {
                for (int k = 1; k < nch; ++k) {  // chunk offsets start at 0: add the bytes before them
                    const Done& D = done[k];
                    const int32_t add = (int32_t)D.byte_base[o];
                    int32_t* p = (int32_t*)rc.offsets.p + D.row_base + 1;
                    add_copy_rebase(tasks, p, p, (size_t)D.oc[o].length, add, ways);
                }
                continue;
            }
            if (t == DFMI_TYPE_BOOLEAN) {
                tasks.emplace_back([&, o] {
                    for (int k = 0; k < nch; ++k)
                        append_bits(R->cols[o].bits.data(), done[k].row_base, bm_at(op[o].bm_values, k), done[k].oc[o].length);
                });
            }
            if (rc.has_validity) {
                tasks.emplace_back([&, o] {
                    for (int k = 0; k < nch; ++k) {
                        const dfmi_out_column& c = done[k].oc[o];
                        if (c.null_count > 0)
                            append_bits(R->cols[o].validity.data(), done[k].row_base, bm_at(op[o].bm_valid, k), c.length);
                        else
                            append_ones(R->cols[o].validity.data(), done[k].row_base, c.length);
                    }
                });
            }
        }
        A.pool->run(tasks);
        for (int o = 0; o < nout; ++o) {
            dfmi_host_result::Col& rc = R->cols[o];
            if (passthrough[o] || otype[o] == DFMI_TYPE_UTF8) continue;
            if (otype[o] == DFMI_TYPE_BOOLEAN) {
                finish_bitmap(rc.bits.data(), rows_so_far);
                rc.bits.resize((size_t)(rows_so_far + 7) / 8);
            }
            if (rc.has_validity) {
                finish_bitmap(rc.validity.data(), rows_so_far);
                rc.validity.resize((size_t)(rows_so_far + 7) / 8);
            } else {
                rc.validity.clear();
            }
        }
        if (bm_stage.p) A.results->put(bm_stage);
        pc.stop(2);
        if (pc.on)
            fprintf(stderr,
                    "dfmi host: %d chunks of %lld rows, setup %.2f ms | stage-in %.2f, issue H2D %.2f, kernel (incl. "
                    "wait H2D) %.2f, issue D2H %.2f, drain %.2f, finish %.2f | total %.2f ms\n",
                    nch, (long long)crows, pc.t[7], pc.t[0], pc.t[3], pc.t[4], pc.t[5], pc.t[6], pc.t[2],
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - call_t0).count());
        *out = R;
        return DFMI_OK;
    } catch (const Fail& f) {
        if (Ap && Ap->h2d) {
            (void)hipStreamSynchronize(Ap->h2d);
            (void)hipStreamSynchronize(Ap->d2h);
            for (int s = 0; s < kSlots; ++s) Ap->slot_used[s] = false;
            if (bm_stage.p) Ap->results->put(bm_stage);
        }
        delete R;
        set_err(err, f.code, f.msg);
        return f.code;
    } catch (const std::bad_alloc&) {
        if (Ap && Ap->h2d) {
            (void)hipStreamSynchronize(Ap->h2d);
            (void)hipStreamSynchronize(Ap->d2h);
            for (int s = 0; s < kSlots; ++s) Ap->slot_used[s] = false;
            if (bm_stage.p) Ap->results->put(bm_stage);
        }
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
    view->validity = c.has_validity ? c.validity.data() : nullptr;
    view->values = c.type == DFMI_TYPE_BOOLEAN && !c.values.p ? (const void*)c.bits.data() : (const void*)c.values.p;
    view->offsets = c.type == DFMI_TYPE_UTF8 ? (const int32_t*)c.offsets.p : nullptr;
    if (c.v_values || c.v_offsets) {  // batches form
        view->values = c.v_values;
        view->offsets = c.type == DFMI_TYPE_UTF8 ? c.v_offsets : nullptr;
        view->validity = c.null_count > 0 ? c.v_validity : nullptr;
    }
    return DFMI_OK;
}

extern "C" int32_t dfmi_host_result_columns(const dfmi_host_result* r, int32_t first, int32_t count,
                                            dfmi_column* views) {
    if (!r || !views || first < 0 || count < 0 || (int64_t)first + count > (int64_t)r->cols.size())
        return DFMI_ERR_INVALID_ARGUMENT;
    for (int32_t k = 0; k < count; ++k) dfmi_host_result_column(r, first + k, &views[k]);
    return DFMI_OK;
}

extern "C" int32_t dfmi_host_result_block(const dfmi_host_result* r, const void** base, size_t* bytes) {
    if (!r || !base || !bytes) return DFMI_ERR_INVALID_ARGUMENT;
    *base = r->arena.p;
    *bytes = r->arena.p ? r->arena.cap : 0;
    return DFMI_OK;
}

extern "C" void dfmi_host_result_free(dfmi_host_result* r) { delete r; }

// ---------------------------------------------------------------------------
// Many small HOST batches in one call (csv_sql.rs:49-62 pulls 1024-row
// batches from csv::Reader, in host memory): every batch's buffers are packed
// into one pinned staging region (host threads), moved with ONE H2D copy,
// run as ONE coalesced launch (dfmi_filter_project_batches), and the outputs
// come back with ONE D2H copy -- into one pinned block the result owns
// (dfmi_filter_project_host_batches: num_batches x n columns, batch-major, as
// views into it), or into the caller's own block
// (dfmi_filter_project_host_batches_into).
namespace {

// Input and worst-case output layout of one host-batches call.
struct HBLayout {
    struct In {
        size_t val = 0, off = 0, vld = 0, nval = 0, noff = 0, nvld = 0;
    };
    struct Out {
        size_t val = 0, vld = 0, off = 0, dat = 0, ndat = 0;
    };
    int ncols = 0, nout = 0;
    std::vector<int> otype;
    std::vector<In> lay;    // [batch][column]
    std::vector<Out> olay;  // [batch][output], offsets in the output region
    size_t in_bytes = 0, out_bytes = 0;
    size_t OB = 0, H = 0, IB = 0, MB = 0;  // outputs, headers, inputs, batch table (aligned)
};

void hb_layout(const dfmi_program* pred, const dfmi_program* const* projs, int32_t np, const dfmi_batch* ins,
               int32_t nb, HBLayout& Lo) {
    if (!pred && np == 0) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "neither a predicate nor projections"};
    const int ncols = ins[0].num_columns;
    const int nout = np > 0 ? np : ncols;
    Lo.ncols = ncols;
    Lo.nout = nout;
    for (int32_t b = 0; b < nb; ++b) {
        if (ins[b].num_columns != ncols || (ncols > 0 && !ins[b].columns))
            throw Fail{DFMI_ERR_INVALID_ARGUMENT, "batches do not share a schema"};
        for (int i = 0; i < ncols; ++i) {
            const dfmi_column& c = ins[b].columns[i];
            if (c.type != ins[0].columns[i].type) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "batches do not share a schema"};
            if (c.length != ins[b].num_rows) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "ragged batch"};
            if (c.type == DFMI_TYPE_UTF8 && !c.offsets) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "Utf8 offsets are NULL"};
            if (!c.values && values_bytes(c)) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "column values pointer is NULL"};
        }
    }
    // ---- input layout: per batch and column, values / offsets / validity
    Lo.lay.assign((size_t)nb * ncols, HBLayout::In{});
    size_t in_bytes = 0;
    for (int32_t b = 0; b < nb; ++b)
        for (int i = 0; i < ncols; ++i) {
            const dfmi_column& c = ins[b].columns[i];
            HBLayout::In& L = Lo.lay[(size_t)b * ncols + i];
            L.nval = values_bytes(c);
            L.val = in_bytes;
            in_bytes += align256(L.nval);
            if (c.type == DFMI_TYPE_UTF8) {
                L.noff = (size_t)(c.length + 1) * 4;
                L.off = in_bytes;
                in_bytes += align256(L.noff);
            }
            if (c.validity && c.null_count > 0) {
                L.nvld = (size_t)((c.length + 7) / 8);
                L.vld = in_bytes;
                in_bytes += align256(L.nvld);
            }
        }
    // ---- output layout (worst case per batch: every row selected)
    Lo.otype.assign(nout, 0);
    for (int o = 0; o < nout; ++o) {
        if (np > 0 && !projs[o]) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL projection"};
        Lo.otype[o] = np > 0 ? projs[o]->type : ins[0].columns[o].type;
    }
    auto osrc = [&](int o) -> int {  // the input column a Utf8 output gathers
        if (np == 0) return o;
        const dfmi::IrNode& root = projs[o]->ir[projs[o]->root];
        return root.kind == dfmi::IR_COL ? root.col : -1;
    };
    Lo.olay.assign((size_t)nb * nout, HBLayout::Out{});
    size_t out_bytes = 0;
    for (int32_t b = 0; b < nb; ++b)
        for (int o = 0; o < nout; ++o) {
            const int64_t n = ins[b].num_rows;
            HBLayout::Out& L = Lo.olay[(size_t)b * nout + o];
            const int t = Lo.otype[o];
            L.val = out_bytes;
            out_bytes += align256(t == DFMI_TYPE_BOOLEAN ? (size_t)bitmap_bytes(n)
                                                         : (t == DFMI_TYPE_UTF8 ? 0 : (size_t)n * width_of(t)));
            L.vld = out_bytes;
            out_bytes += align256(bitmap_bytes(n));
            if (t == DFMI_TYPE_UTF8) {
                L.off = out_bytes;
                out_bytes += align256((size_t)(n + 1) * 4);
                const int c = osrc(o);
                L.ndat = c >= 0 ? values_bytes(ins[b].columns[c]) : 0;
                L.dat = out_bytes;
                out_bytes += align256(std::max<size_t>(L.ndat, 1));
            }
        }
    Lo.in_bytes = in_bytes;
    Lo.out_bytes = out_bytes;
    Lo.OB = align256(std::max<size_t>(out_bytes, 256));
    Lo.H = align256((size_t)nb * 256);
    Lo.IB = align256(std::max<size_t>(in_bytes, 256));
    size_t MB = 256;  // bound on the launch's batch table + tile map (exec.cpp)
    for (int32_t b = 0; b < nb; ++b)
        MB += (size_t)(4 + 3 * ncols + 5 * nout) * 8 + (size_t)((ins[b].num_rows + 63) / 64 + 1) * 4;
    Lo.MB = align256(MB);
}

// Where a host-batches call's headers and outputs land (pinned host memory,
// with the device-visible addresses the kernel writes through when the call
// is zero-copy). `contiguous`: outputs right after the headers (one D2H).
struct HBTarget {
    uint8_t *hdr_host = nullptr, *hdr_dev = nullptr;
    uint8_t *out_host = nullptr, *out_dev = nullptr;
    bool contiguous = false;
};

uint8_t* device_address(uint8_t* host) {
    void* d = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&d, host, 0));
    return (uint8_t*)d;
}

// The common body: layout, packing, the staged coalesced launch. `target`
// is asked once (H, OB, zero-copy) for the output placement. Returns the
// launch's status; *nok = batches completed.
int32_t host_batches_run(dfmi_context* ctx, const dfmi_program* pred, const dfmi_program* const* projs, int32_t np,
                         const dfmi_batch* ins, int32_t nb, uint32_t flags, const HBLayout& Lo,
                         const std::function<HBTarget(size_t H, size_t OB, bool zc)>& target,
                         std::vector<dfmi_out_column>& douts, int32_t* failed, dfmi_error* err, dfmi::CallProf& prof) {
    HIP_TRY(hipSetDevice(dfmi::ctx_device(ctx)));
    hipStream_t st = dfmi::ctx_stream(ctx);
    Arena& A = arena_of(ctx);
    A.init(dfmi::ctx_device(ctx));
    const int ncols = Lo.ncols, nout = Lo.nout;
    const size_t OB = Lo.OB, H = Lo.H, IB = Lo.IB, MB = Lo.MB;
    // ---- regions. Device (Arena::hb): this call's half [headers |
    // outputs], the other half's headers zeroed by this call's kernel, and
    // [inputs | batch table]; pinned staging: [inputs | table] (ONE H2D, or
    // none: small calls read it in place); the target: headers + outputs
    // (ONE D2H, or none: a small call's kernel writes them in place).
    A.reserve_pin(IB + MB);
    A.reserve_hb(H, OB, IB + MB, st);
    uint8_t* const pin_in = A.pin;
    prof.mark(0);
    {
        std::vector<std::function<void()>> tasks;
        const int ways = std::max(1, std::min(A.pool->ways(), (int)(Lo.in_bytes >> 20) + 1));
        for (int w = 0; w < ways; ++w)
            tasks.push_back([&, w] {
                for (int32_t b = w; b < nb; b += ways)
                    for (int i = 0; i < ncols; ++i) {
                        const dfmi_column& c = ins[b].columns[i];
                        const HBLayout::In& L = Lo.lay[(size_t)b * ncols + i];
                        if (L.nval) memcpy(pin_in + L.val, c.values, L.nval);
                        if (L.noff) memcpy(pin_in + L.off, c.offsets, L.noff);
                        if (L.nvld) memcpy(pin_in + L.vld, c.validity, L.nvld);
                    }
            });
        A.pool->run(tasks);
    }
    // zero-copy inputs (small calls): the kernel reads the inputs and the
    // batch table straight from the pinned staging region over PCIe -- no
    // copy in at all on the call's critical path
    static const int zc_env = [] {
        const char* e = getenv("DFMI_HOST_ZC");
        return e ? atoi(e) : -1;
    }();
    const bool zc = zc_env > 0 || (zc_env < 0 && Lo.in_bytes + MB <= kZeroCopyBytes);
    prof.mark(1);
    const int half = A.hb_half, other = 1 - half;
    const HBTarget T = target(H, OB, zc);
    uint8_t* const dhdr = A.hb_half_base(half) + A.hb_hcap - H;  // the kernel's header atomics
    uint8_t* const dout = zc ? T.out_dev : A.hb_half_base(half) + A.hb_hcap;
    uint8_t* const dev = zc ? A.pin_dev : A.hb + 2 * (A.hb_hcap + A.hb_ocap);  // inputs
    std::vector<dfmi_column> dcols((size_t)nb * std::max(1, ncols));
    std::vector<dfmi_batch> dins(nb);
    for (int32_t b = 0; b < nb; ++b) {
        for (int i = 0; i < ncols; ++i) {
            const dfmi_column& c = ins[b].columns[i];
            const HBLayout::In& L = Lo.lay[(size_t)b * ncols + i];
            dfmi_column& d = dcols[(size_t)b * ncols + i];
            d = c;
            d.values = dev + L.val;
            d.offsets = c.type == DFMI_TYPE_UTF8 ? (const int32_t*)(dev + L.off) : nullptr;
            d.validity = L.nvld ? dev + L.vld : nullptr;
            if (!L.nvld) d.null_count = 0;
        }
        dins[b] = dfmi_batch{ncols, 0, ins[b].num_rows, dcols.data() + (size_t)b * ncols};
    }
    douts.assign((size_t)nb * nout, dfmi_out_column{});
    for (size_t k = 0; k < douts.size(); ++k) {
        const HBLayout::Out& L = Lo.olay[k];
        dfmi_out_column& d = douts[k];
        memset(&d, 0, sizeof d);
        d.values = dout + L.val;
        d.validity = dout + L.vld;
        if (Lo.otype[k % nout] == DFMI_TYPE_UTF8) {
            d.offsets = (int32_t*)(dout + L.off);
            d.data = dout + L.dat;
            d.data_capacity = (int64_t)L.ndat;
        }
    }
    // ---- (one H2D), the coalesced launch, (one D2H), one synchronisation
    size_t meta_used = 0;
    hipError_t copy_err = hipSuccess;
    bool cleared = false, hdr_written = false;
    dfmi::BatchStage stage;
    stage.locate = [&](size_t meta_bytes, size_t hdr_bytes, uint8_t** host_meta, uint8_t** dev_meta,
                       uint8_t** dev_hdr, const uint8_t** host_hdr) {
        if (meta_bytes > MB || hdr_bytes > H) return false;
        meta_used = meta_bytes;
        *host_meta = pin_in + IB;
        *dev_meta = dev + IB;
        *dev_hdr = dhdr;
        *host_hdr = T.hdr_host;
        return true;
    };
    stage.copy_in = [&](hipStream_t s) {
        hipError_t e = hipSuccess;
        if (A.hb_dirty[half])  // headers the other half's last kernel did not zero (an earlier failed call)
            e = hipMemsetAsync(A.hb_half_base(half) + A.hb_hcap - A.hb_dirty[half], 0, A.hb_dirty[half], s);
        if (e == hipSuccess && !zc)
            e = hipMemcpyAsync(dev, pin_in, meta_used ? IB + meta_used : Lo.in_bytes, hipMemcpyHostToDevice, s);
        if (e != hipSuccess) copy_err = e;
        else A.hb_dirty[half] = 0;
    };
    stage.copy_out = [&](hipStream_t s) {
        if (zc && hdr_written) return;  // outputs and headers are in place
        hipError_t e;
        if (T.contiguous && !zc) {  // [headers | outputs] in one copy
            e = hipMemcpyAsync(T.hdr_host, dhdr, H + OB, hipMemcpyDeviceToHost, s);
        } else {
            e = hipMemcpyAsync(T.hdr_host, dhdr, H, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess && !zc) e = hipMemcpyAsync(T.out_host, dout, OB, hipMemcpyDeviceToHost, s);
        }
        if (e != hipSuccess) copy_err = e;
    };
    if (zc) {
        stage.hdr_out = (uint64_t*)T.hdr_dev;
        stage.hdr_written = &hdr_written;
    }
    stage.clear_bhdr = (uint64_t*)(A.hb_half_base(other) + A.hb_hcap - A.hb_dirty[other]);
    stage.clear_bhdr_words = (int64_t)(A.hb_dirty[other] / 8);
    stage.cleared = &cleared;
    prof.mark(2);
    const int32_t rc = dfmi::filter_project_batches_staged(ctx, pred, projs, np, dins.data(), nb, douts.data(), flags,
                                                           failed, err, &stage);
    if (rc != DFMI_OK) (void)hipStreamSynchronize(st);  // (a call that failed after copy_in: drain it)
    prof.mark(3);
    if (cleared) {  // this kernel zeroed the other half's headers; this half's are dirty now
        A.hb_dirty[other] = 0;
        A.hb_dirty[half] = std::max(A.hb_dirty[half], H);
        A.hb_half = other;
    }
    HIP_TRY(copy_err);
    return rc;
}

}  // namespace

extern "C" int32_t dfmi_filter_project_host_batches(dfmi_context* ctx, const dfmi_program* pred,
                                                    const dfmi_program* const* projs, int32_t np,
                                                    const dfmi_batch* ins, int32_t nb, uint32_t flags,
                                                    dfmi_host_result** out, int32_t* failed, dfmi_error* err) {
    // phases: checks + layout, packing into pinned memory, structs, the staged call, result views
    static thread_local dfmi::CallProf prof("host_batches");
    prof.start();
    set_err(err, DFMI_OK, "");
    int32_t dummy_failed;
    if (!failed) failed = &dummy_failed;
    *failed = -1;
    dfmi_host_result* R = nullptr;
    try {
        if (!ctx || !out || nb < 0 || (nb > 0 && !ins) || (np > 0 && !projs))
            throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        *out = nullptr;
        dfmi::ctx_last_err_key(ctx) = ~0ull;
        if (!pred && np == 0) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "neither a predicate nor projections"};
        dfmi::Unsliced us_;  // sliced arrays (slice.cpp)
        if (nb > 0 && dfmi::any_offset(ins, nb)) ins = dfmi::unslice(ins, nb, us_, false, nullptr);
        Arena& A = arena_of(ctx);
        A.init(dfmi::ctx_device(ctx));
        R = new dfmi_host_result();
        R->pool = A.results;
        if (nb == 0) {
            *out = R;
            return DFMI_OK;
        }
        HBLayout Lo;
        hb_layout(pred, projs, np, ins, nb, Lo);
        const int ncols = Lo.ncols, nout = Lo.nout;
        std::vector<dfmi_out_column> douts;
        dfmi_error e2{};
        // the result's pinned block [headers | outputs]; a small call's kernel
        // writes its outputs there directly (and, one tile per batch, the
        // finished headers too: Launch::hdr_out) -- no copy back at all
        auto target = [&](size_t H, size_t OB, bool zc) {
            R->arena = R->pool->get(H + OB);
            HBTarget T;
            T.hdr_host = R->arena.p;
            T.out_host = R->arena.p + H;
            T.contiguous = true;
            if (zc) {
                T.hdr_dev = device_address(R->arena.p);
                T.out_dev = T.hdr_dev + H;
            }
            return T;
        };
        const int32_t rc = host_batches_run(ctx, pred, projs, np, ins, nb, flags, Lo, target, douts, failed, &e2, prof);
        const int32_t nok = rc == DFMI_OK ? nb : std::max(0, *failed);
        R->cols.resize((size_t)nb * nout);
        for (int32_t b = 0; b < nb; ++b)
            for (int o = 0; o < nout; ++o) {
                const size_t k = (size_t)b * nout + o;
                dfmi_host_result::Col& c = R->cols[k];
                c.type = Lo.otype[o];
                if (b >= nok) continue;  // a failed call: batches from the failing one are empty
                const dfmi_out_column& d = douts[k];
                const HBLayout::Out& L = Lo.olay[k];
                if (d.passthrough_column >= 0) {  // Arc clone: the caller's own column, copied
                    const dfmi_column& src = ins[b].columns[d.passthrough_column];
                    const HBLayout::In& I = Lo.lay[(size_t)b * ncols + d.passthrough_column];
                    c.length = src.length;
                    c.null_count = I.nvld ? src.null_count : 0;
                    c.values = R->pool->get(std::max<size_t>(I.nval, 1));
                    if (I.nval) memcpy(c.values.p, src.values, I.nval);
                    c.v_values = c.values.p;
                    if (src.type == DFMI_TYPE_UTF8) {
                        c.offsets = R->pool->get(I.noff);
                        memcpy(c.offsets.p, src.offsets, I.noff);
                        c.v_offsets = (const int32_t*)c.offsets.p;
                        c.data_length = (int64_t)I.nval;
                    }
                    if (I.nvld) {
                        c.validity.assign(src.validity, src.validity + I.nvld);
                        c.has_validity = true;
                        c.v_validity = c.validity.data();
                    }
                    continue;
                }
                c.length = d.length;
                c.null_count = d.null_count;
                c.data_length = d.data_length;
                uint8_t* const ob = R->arena.p + Lo.H;  // the outputs, after the headers
                c.v_values = ob + (Lo.otype[o] == DFMI_TYPE_UTF8 ? L.dat : L.val);
                c.v_offsets = Lo.otype[o] == DFMI_TYPE_UTF8 ? (const int32_t*)(ob + L.off) : nullptr;
                c.v_validity = ob + L.vld;
            }
        *out = R;
        R = nullptr;
        if (rc != DFMI_OK) {
            if (err) *err = e2;
            return rc;
        }
        prof.mark(4);
        prof.done();
        return DFMI_OK;
    } catch (const Fail& f) {
        delete R;
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

extern "C" int32_t dfmi_host_batches_output_bytes(const dfmi_program* pred, const dfmi_program* const* projs,
                                                  int32_t np, const dfmi_batch* ins, int32_t nb, uint32_t flags,
                                                  size_t* bytes, dfmi_error* err) {
    (void)flags;
    set_err(err, DFMI_OK, "");
    try {
        if (!bytes || nb < 0 || (nb > 0 && !ins) || (np > 0 && !projs))
            throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        *bytes = 0;
        if (!pred && np == 0) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "neither a predicate nor projections"};
        if (nb == 0) return DFMI_OK;
        dfmi::Unsliced us_;
        if (dfmi::any_offset(ins, nb)) ins = dfmi::unslice(ins, nb, us_, false, nullptr);
        HBLayout Lo;
        hb_layout(pred, projs, np, ins, nb, Lo);
        *bytes = Lo.OB;
        return DFMI_OK;
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

extern "C" int32_t dfmi_filter_project_host_batches_into(dfmi_context* ctx, const dfmi_program* pred,
                                                         const dfmi_program* const* projs, int32_t np,
                                                         const dfmi_batch* ins, int32_t nb, uint32_t flags,
                                                         void* out_block, size_t out_capacity,
                                                         dfmi_out_column* outputs, int32_t* failed, dfmi_error* err) {
    static thread_local dfmi::CallProf prof("host_batches_into");
    prof.start();
    set_err(err, DFMI_OK, "");
    int32_t dummy_failed;
    if (!failed) failed = &dummy_failed;
    *failed = -1;
    Arena* Ap = nullptr;
    dfmi_host::PinnedPool::Blk stage_blk;
    try {
        if (!ctx || nb < 0 || (nb > 0 && (!ins || !outputs || !out_block)) || (np > 0 && !projs))
            throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        dfmi::ctx_last_err_key(ctx) = ~0ull;
        if (!pred && np == 0) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "neither a predicate nor projections"};
        if (nb == 0) return DFMI_OK;
        if ((uintptr_t)out_block & 63) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "out_block must be 64-byte aligned"};
        dfmi::Unsliced us_;
        const dfmi_batch* const caller_ins = ins;
        if (dfmi::any_offset(ins, nb)) ins = dfmi::unslice(ins, nb, us_, false, nullptr);
        HBLayout Lo;
        hb_layout(pred, projs, np, ins, nb, Lo);
        const int nout = Lo.nout;
        if (out_capacity < Lo.OB)
            throw Fail{DFMI_ERR_CAPACITY, "out_block holds " + std::to_string(out_capacity) + " bytes, the outputs need " +
                                              std::to_string(Lo.OB) + " (dfmi_host_batches_output_bytes)"};
        Arena& A = arena_of(ctx);
        A.init(dfmi::ctx_device(ctx));
        Ap = &A;
        uint8_t* const blk = (uint8_t*)out_block;
        // a pinned caller block is the kernel's (or the D2H's) target itself
        uint8_t* blk_dev = nullptr;
        if (is_pinned(blk, 1) && is_pinned(blk, Lo.OB)) {
            blk_dev = device_address(blk);
        } else {
            hipPointerAttribute_t pa;
            if (hipPointerGetAttributes(&pa, blk) == hipSuccess && pa.type == hipMemoryTypeHost &&
                hipPointerGetAttributes(&pa, blk + Lo.OB - 1) == hipSuccess && pa.type == hipMemoryTypeHost)
                blk_dev = device_address(blk);
            else
                (void)hipGetLastError();
        }
        if (prof.on && !blk_dev) {  // diagnostics: a pageable caller block costs a copy of the outputs
            static std::atomic<int> said{0};
            if (said++ < 4) {
                hipPointerAttribute_t pa{};
                const hipError_t pe = hipPointerGetAttributes(&pa, blk);
                (void)hipGetLastError();
                fprintf(stderr, "dfmi host_batches_into: caller block %p not pinned (attr rc %d type %d), %zu bytes\n",
                        (void*)blk, (int)pe, (int)pa.type, Lo.OB);
            }
        }
        std::vector<dfmi_out_column> douts;
        dfmi_error e2{};
        auto target = [&](size_t H, size_t OB, bool zc) {
            HBTarget T;
            A.reserve_hdr_pin(H);
            T.hdr_host = A.hdr_pin;
            T.hdr_dev = A.hdr_pin_dev;
            if (blk_dev) {
                T.out_host = blk;
                T.out_dev = blk_dev;
            } else {  // pageable: the library's pinned staging, copied below
                stage_blk = A.results->get(OB);
                T.out_host = stage_blk.p;
                if (zc) T.out_dev = device_address(stage_blk.p);
            }
            (void)H;
            return T;
        };
        const int32_t rc = host_batches_run(ctx, pred, projs, np, ins, nb, flags, Lo, target, douts, failed, &e2, prof);
        const int32_t nok = rc == DFMI_OK ? nb : std::max(0, *failed);
        // ---- the outputs as views into the caller's block; a pageable block
        // gets the selected bytes (only those) from the staging block
        std::vector<std::function<void()>> tasks;
        const uint8_t* const src = stage_blk.p;
        for (int32_t b = 0; b < nb; ++b)
            for (int o = 0; o < nout; ++o) {
                const size_t k = (size_t)b * nout + o;
                const HBLayout::Out& L = Lo.olay[k];
                dfmi_out_column& u = outputs[k];
                const dfmi_out_column d = douts[k];
                memset(&u, 0, sizeof u);
                u.type = Lo.otype[o];
                u.passthrough_column = -1;
                if (b >= nok) continue;  // a failed call: batches from the failing one are empty
                if (d.passthrough_column >= 0) {  // the caller's own input column (expression.rs:272-276)
                    const dfmi_column& c = caller_ins[b].columns[d.passthrough_column];
                    u.passthrough_column = d.passthrough_column;
                    u.length = c.length;
                    u.null_count = c.validity ? c.null_count : 0;
                    continue;
                }
                u.length = d.length;
                u.null_count = d.null_count;
                u.data_length = d.data_length;
                u.validity = blk + L.vld;
                const int t = Lo.otype[o];
                size_t nv = 0;
                if (t == DFMI_TYPE_UTF8) {
                    u.offsets = (int32_t*)(blk + L.off);
                    u.data = blk + L.dat;
                    u.data_capacity = (int64_t)L.ndat;
                } else {
                    u.values = blk + L.val;
                    nv = t == DFMI_TYPE_BOOLEAN ? (size_t)(d.length + 7) / 8 : (size_t)d.length * width_of(t);
                }
                if (!src) continue;
                const size_t nb_ = (size_t)(d.length + 7) / 8;
                tasks.emplace_back([=] {
                    if (nv) memcpy(blk + L.val, src + L.val, nv);
                    if (d.null_count > 0) memcpy(blk + L.vld, src + L.vld, nb_);
                    if (t == DFMI_TYPE_UTF8) {
                        memcpy(blk + L.off, src + L.off, (size_t)(d.length + 1) * 4);
                        if (d.data_length) memcpy(blk + L.dat, src + L.dat, (size_t)d.data_length);
                    }
                });
            }
        if (!tasks.empty()) {  // batch-sized pieces, spread over the host threads
            const int ways = A.pool->ways();
            std::vector<std::function<void()>> parts((size_t)std::min<size_t>(ways, tasks.size()));
            for (size_t w = 0; w < parts.size(); ++w)
                parts[w] = [&, w] {
                    for (size_t i = w; i < tasks.size(); i += parts.size()) tasks[i]();
                };
            A.pool->run(parts);
        }
        if (stage_blk.p) A.results->put(stage_blk);
        if (rc != DFMI_OK) {
            if (err) *err = e2;
            return rc;
        }
        prof.mark(4);
        prof.done();
        return DFMI_OK;
    } catch (const Fail& f) {
        if (Ap && stage_blk.p) Ap->results->put(stage_blk);
        set_err(err, f.code, f.msg);
        return f.code;
    }
}
