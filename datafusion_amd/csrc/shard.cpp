// Multi-GPU form of the path: row-range shards, one host
// thread / process per GPU, RCCL over xGMI for the only exchange the path
// has. The reference has no parallelism at all (context.rs:33, one
// Rc<RefCell<..>> pull); rows are independent through FilterRelation /
// ProjectRelation and filter() preserves row order (filter.rs:87-91), so the
// per-rank outputs in rank order ARE the reference's output stream.
//
//   dfmi_shard_filter_project: the local fused pass, then ONE all_gather of a
//     fixed record per rank (status, error position, selected rows, Utf8
//     bytes and null count per output, error message) -> every rank's global
//     placement; a failure anywhere becomes the same (globally first) error
//     on every rank.
//   dfmi_shard_gather_to_root: optional concatenation on one rank with grouped
//     send / recv (RCCL has no gatherv), bound by the root's xGMI ingress;
//     Utf8 offsets rebased and bitmaps re-aligned on the root. Every rank's
//     argument checks are agreed on (one small all_gather) BEFORE the
//     transfers, so a caller mistake on one rank fails every rank instead of
//     leaving the others blocked in a send.
//   dfmi_shard_agg_finish: the aggregate extension's exact partials,
//     all_gathered and merged -- bit-identical to one GPU over all rows.
//
// The collectives go through a Transport: RCCL (the product path, one
// process or thread per GPU) or, for tests only, a loopback group of threads
// sharing one device (dfmi_internal_* hooks at the end of this file), so the
// placement, error agreement and gather code runs at world sizes > 1 on a
// one-GPU box.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "exec_internal.h"

using namespace dfmi;
using namespace dfmi::xi;

namespace dfmi {
hipError_t launch_rebase_offsets(const int32_t* src, long long n, long long base, int32_t* dst, hipStream_t st);
hipError_t launch_place_bits(const uint8_t* src, long long n, uint8_t* dst, long long dst_bit, hipStream_t st);
}  // namespace dfmi

// aggregate.cpp: every rank's grouped partials merged into the state's shown groups
int32_t dfmi_agg_state_show_merged(dfmi_agg_state* st, const void* const* partials, const int64_t* sizes, int32_t nparts,
                                   int64_t cap, dfmi_agg_value* keys, dfmi_agg_value* values, int64_t* num_groups,
                                   dfmi_error* err);

namespace {
constexpr int kMaxOut = 16;
// record per rank: status, error position (evaluation-order key >> 44), rows,
// utf8 bytes[16], nulls[16]; then the error message
constexpr int kRec = 3 + 2 * kMaxOut;
constexpr int kMsg = 512;
constexpr size_t kRecBytes = kRec * 8 + kMsg;

#define NCCL_TRY(x)                                                                                         \
    do {                                                                                                    \
        ncclResult_t r_ = (x);                                                                              \
        if (r_ != ncclSuccess) throw Fail{DFMI_ERR_DEVICE, std::string(#x ": ") + ncclGetErrorString(r_)}; \
    } while (0)

// The collectives of the shard path. all_gather works on host buffers (the
// records are a few hundred bytes); send / recv move device buffers and
// complete at group_end (the context stream is synchronised there).
struct Transport {
    virtual ~Transport() = default;
    virtual void all_gather(dfmi_context* ctx, const void* mine, void* all, size_t bytes) = 0;
    virtual void group_start() = 0;
    virtual void send(dfmi_context* ctx, const void* buf, size_t nb, int peer) = 0;
    virtual void recv(dfmi_context* ctx, void* buf, size_t nb, int peer) = 0;
    virtual void group_end(dfmi_context* ctx) = 0;
};

struct RcclTransport : Transport {
    int world, rank;
    ncclComm_t comm = nullptr;
    uint8_t* d = nullptr;  // all_gather staging, world x bytes
    size_t cap = 0;
    RcclTransport(int w, int r) : world(w), rank(r) {}
    ~RcclTransport() override {
        if (comm) ncclCommDestroy(comm);
        if (d) (void)hipFree(d);
    }
    void all_gather(dfmi_context* ctx, const void* mine, void* all, size_t bytes) override {
        hipStream_t st = ctx->stream;
        if (cap < bytes * world) {
            if (d) HIP_TRY(hipFree(d));
            d = nullptr;
            cap = 0;
            HIP_TRY(hipMalloc((void**)&d, bytes * world));
            cap = bytes * world;
        }
        uint8_t* send = d + (size_t)rank * bytes;
        HIP_TRY(hipMemcpyAsync(send, mine, bytes, hipMemcpyHostToDevice, st));
        NCCL_TRY(ncclAllGather(send, d, bytes, ncclUint8, comm, st));  // in place
        HIP_TRY(hipMemcpyAsync(all, d, bytes * world, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    void group_start() override { NCCL_TRY(ncclGroupStart()); }
    void send(dfmi_context* ctx, const void* buf, size_t nb, int peer) override {
        NCCL_TRY(ncclSend(buf, nb, ncclUint8, peer, comm, ctx->stream));
    }
    void recv(dfmi_context* ctx, void* buf, size_t nb, int peer) override {
        NCCL_TRY(ncclRecv(buf, nb, ncclUint8, peer, comm, ctx->stream));
    }
    void group_end(dfmi_context* ctx) override {
        NCCL_TRY(ncclGroupEnd());
        HIP_TRY(hipStreamSynchronize(ctx->stream));
    }
};

// ---- loopback transport (tests): `world` host threads in one process, each
// with its own context on the same device; the collectives are host
// rendezvous + device-to-device copies.
struct LoopGroup {
    int world;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    long generation = 0;
    std::vector<uint8_t> buf;
    struct Post {
        int src, dst;
        const void* p;
        size_t nb;
    };
    std::vector<Post> posts;
    explicit LoopGroup(int w) : world(w) {}
    void barrier(std::unique_lock<std::mutex>& lk) {
        const long g = generation;
        if (++arrived == world) {
            arrived = 0;
            ++generation;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return generation != g; });
        }
    }
};

struct LoopTransport : Transport {
    LoopGroup* g;
    int rank;
    std::vector<LoopGroup::Post> sends, recvs;
    LoopTransport(LoopGroup* grp, int r) : g(grp), rank(r) {}
    void all_gather(dfmi_context*, const void* mine, void* all, size_t bytes) override {
        std::unique_lock<std::mutex> lk(g->mu);
        if (g->buf.size() < bytes * g->world) g->buf.resize(bytes * g->world);
        memcpy(g->buf.data() + (size_t)rank * bytes, mine, bytes);
        g->barrier(lk);
        memcpy(all, g->buf.data(), bytes * g->world);
        g->barrier(lk);
    }
    void group_start() override {
        sends.clear();
        recvs.clear();
    }
    void send(dfmi_context*, const void* buf, size_t nb, int peer) override { sends.push_back({rank, peer, buf, nb}); }
    void recv(dfmi_context*, void* buf, size_t nb, int peer) override { recvs.push_back({peer, rank, buf, nb}); }
    void group_end(dfmi_context* ctx) override {
        hipStream_t st = ctx->stream;
        HIP_TRY(hipStreamSynchronize(st));  // this rank's send buffers are final
        std::unique_lock<std::mutex> lk(g->mu);
        for (const auto& s : sends) g->posts.push_back(s);
        g->barrier(lk);
        std::vector<int> taken(g->posts.size(), 0);
        bool ok = true;
        for (const auto& r : recvs) {  // k-th recv from src <- k-th send from src to us (RCCL's matching)
            bool found = false;
            for (size_t i = 0; i < g->posts.size(); ++i) {
                const auto& s = g->posts[i];
                if (taken[i] || s.src != r.src || s.dst != rank) continue;
                taken[i] = 1;
                found = true;
                if (s.nb != r.nb) ok = false;
                else if (hipMemcpyAsync((void*)r.p, s.p, r.nb, hipMemcpyDeviceToDevice, st) != hipSuccess) ok = false;
                break;
            }
            if (!found) ok = false;
        }
        lk.unlock();
        const hipError_t e = hipStreamSynchronize(st);
        lk.lock();
        g->barrier(lk);  // every receiver done reading the posts
        if (rank == 0) g->posts.clear();
        g->barrier(lk);
        if (!ok) throw Fail{DFMI_ERR_DEVICE, "loopback transport: unmatched send/recv"};
        if (e != hipSuccess) throw Fail{DFMI_ERR_DEVICE, std::string("loopback copy: ") + hipGetErrorString(e)};
    }
};

// ---- placement / error agreement over the exchanged records (pure)
int first_failed_rank(const int64_t* recs, int world, size_t stride_words) {
    int first = -1;
    for (int r = 0; r < world; ++r) {
        const int64_t* rr = recs + (size_t)r * stride_words;
        if (!rr[0]) continue;
        // smallest evaluation position, then the lowest rank (= earliest rows)
        if (first < 0 || (uint64_t)rr[1] < (uint64_t)recs[(size_t)first * stride_words + 1]) first = r;
    }
    return first;
}

void placement_of(const int64_t* recs, int world, int rank, int nout, size_t stride_words, dfmi_shard_placement* p) {
    memset(p, 0, sizeof *p);
    p->world = world;
    p->rank = rank;
    for (int r = 0; r < world; ++r) {
        const int64_t* rr = recs + (size_t)r * stride_words;
        if (r < rank) p->row_offset += rr[2];
        p->total_rows += rr[2];
        for (int o = 0; o < nout; ++o) {
            if (r < rank) p->utf8_base[o] += rr[3 + o];
            p->utf8_total[o] += rr[3 + o];
            p->null_total[o] += rr[3 + kMaxOut + o];
        }
    }
}
}  // namespace

struct dfmi_shard_comm {
    int world = 1, rank = 0, device = 0;
    Transport* tp = nullptr;
    std::vector<int64_t> rec;  // the last exchange: world x kRec
    int nout = 0;              // outputs of the last exchanged pass
    // kept across calls (grow-only): the gather's staging on the root and an
    // all-valid bitmap for a rank without validity; a pinned landing spot for
    // passthrough Utf8 byte spans
    uint8_t* stage = nullptr;
    size_t stage_cap = 0;
    uint8_t* ones = nullptr;
    size_t ones_cap = 0;
    int32_t* pin = nullptr;
    ~dfmi_shard_comm() {
        if (stage) (void)hipFree(stage);
        if (ones) (void)hipFree(ones);
        if (pin) (void)hipHostFree(pin);
    }
};

namespace {
// One all_gather of every rank's record + message; on a failure anywhere,
// every rank throws the globally first error with the failing rank's message.
void exchange(dfmi_context* ctx, dfmi_shard_comm* c, const int64_t* mine, const char* msg) {
    std::vector<uint8_t> me(kRecBytes, 0), all(kRecBytes * c->world);
    memcpy(me.data(), mine, kRec * 8);
    snprintf((char*)me.data() + kRec * 8, kMsg, "%s", msg ? msg : "");
    c->tp->all_gather(ctx, me.data(), all.data(), kRecBytes);
    c->rec.assign((size_t)c->world * kRec, 0);
    for (int r = 0; r < c->world; ++r) memcpy(&c->rec[(size_t)r * kRec], &all[(size_t)r * kRecBytes], kRec * 8);
    const int first = first_failed_rank(c->rec.data(), c->world, kRec);
    if (first < 0) return;
    all[(size_t)first * kRecBytes + kRecBytes - 1] = 0;
    throw Fail{(int32_t)c->rec[(size_t)first * kRec], std::string((const char*)&all[(size_t)first * kRecBytes + kRec * 8])};
}

// Agreement on a local outcome (collective): every rank throws the error of
// the lowest failing rank, or all go on.
void agree(dfmi_context* ctx, dfmi_shard_comm* c, int32_t code, const std::string& msg) {
    std::vector<uint8_t> me(kMsg + 8, 0), all((size_t)(kMsg + 8) * c->world);
    memcpy(me.data(), &code, 4);
    snprintf((char*)me.data() + 8, kMsg, "%s", msg.c_str());
    c->tp->all_gather(ctx, me.data(), all.data(), me.size());
    for (int r = 0; r < c->world; ++r) {
        int32_t rc;
        memcpy(&rc, &all[(size_t)r * (kMsg + 8)], 4);
        if (rc) {
            all[(size_t)(r + 1) * (kMsg + 8) - 1] = 0;
            throw Fail{rc, std::string((const char*)&all[(size_t)r * (kMsg + 8) + 8])};
        }
    }
}
}  // namespace

extern "C" int32_t dfmi_shard_unique_id(uint8_t* id, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    try {
        if (!id) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        ncclUniqueId u;
        NCCL_TRY(ncclGetUniqueId(&u));
        memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
        return DFMI_OK;
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

extern "C" int32_t dfmi_shard_comm_init(dfmi_context* ctx, int32_t world, int32_t rank, const uint8_t* id,
                                        dfmi_shard_comm** out, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    dfmi_shard_comm* c = nullptr;
    try {
        if (!ctx || !id || !out || world < 1 || rank < 0 || rank >= world)
            throw Fail{DFMI_ERR_INVALID_ARGUMENT, "bad argument"};
        c = new dfmi_shard_comm();
        c->world = world;
        c->rank = rank;
        c->device = ctx->device;
        HIP_TRY(hipSetDevice(c->device));
        auto* t = new RcclTransport(world, rank);
        c->tp = t;
        ncclUniqueId u;
        memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
        NCCL_TRY(ncclCommInitRank(&t->comm, world, u, rank));
        c->rec.assign((size_t)world * kRec, 0);
        *out = c;
        return DFMI_OK;
    } catch (const Fail& f) {
        if (c) {
            delete c->tp;
            delete c;
        }
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

extern "C" void dfmi_shard_comm_destroy(dfmi_shard_comm* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    delete c->tp;
    delete c;
}

extern "C" int32_t dfmi_shard_filter_project(dfmi_context* ctx, dfmi_shard_comm* c, const dfmi_program* pred,
                                             const dfmi_program* const* projs, int32_t np, const dfmi_batch* in,
                                             dfmi_out_column* outs, uint32_t flags, dfmi_shard_placement* place,
                                             dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    try {
        if (!ctx || !c || !in || !outs || !place) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        const int nout = np > 0 ? np : in->num_columns;
        if (nout > kMaxOut) throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "device program limit: too many output columns"};
        dfmi_error local;
        int32_t rc = dfmi_filter_project(ctx, pred, projs, np, in, outs, flags, &local);
        int64_t mine[kRec] = {};
        if (rc == DFMI_OK) {
            try {
                mine[2] = nout ? outs[0].length : 0;
                // passthrough (Arc clone) Utf8 outputs: the input column's byte
                // span, both ends of every such column in one async round trip
                bool spans = false;
                for (int o = 0; o < nout; ++o)
                    if (outs[o].type == DFMI_TYPE_UTF8 && outs[o].passthrough_column >= 0 && outs[o].length > 0) {
                        if (!c->pin) HIP_TRY(hipHostMalloc((void**)&c->pin, 2 * kMaxOut * 4, hipHostMallocDefault));
                        const dfmi_column& pc = in->columns[outs[o].passthrough_column];
                        const int32_t* of = pc.offsets + pc.offset;  // (a sliced array's first offset)
                        HIP_TRY(hipMemcpyAsync(&c->pin[2 * o], of, 4, hipMemcpyDeviceToHost, ctx->stream));
                        HIP_TRY(hipMemcpyAsync(&c->pin[2 * o + 1], of + outs[o].length, 4, hipMemcpyDeviceToHost, ctx->stream));
                        spans = true;
                    }
                if (spans) HIP_TRY(hipStreamSynchronize(ctx->stream));
                for (int o = 0; o < nout; ++o) {
                    int64_t nb = outs[o].type == DFMI_TYPE_UTF8 ? outs[o].data_length : 0;
                    if (outs[o].type == DFMI_TYPE_UTF8 && outs[o].passthrough_column >= 0 && outs[o].length > 0)
                        nb = c->pin[2 * o + 1] - c->pin[2 * o];
                    mine[3 + o] = nb;
                    mine[3 + kMaxOut + o] = outs[o].null_count;
                }
            } catch (const Fail& f) {
                rc = f.code;
                set_err(&local, f.code, f.msg);
            }
        }
        if (rc != DFMI_OK) {
            memset(mine, 0, sizeof mine);
            mine[0] = rc;
            mine[1] = (int64_t)(ctx->last_err_key >> 44);  // ~0 (no position) sorts last
        }
        exchange(ctx, c, mine, rc ? local.message : "");  // throws the globally first error on every rank
        c->nout = nout;
        placement_of(c->rec.data(), c->world, c->rank, nout, kRec, place);
        return DFMI_OK;
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

extern "C" int32_t dfmi_shard_gather_to_root(dfmi_context* ctx, dfmi_shard_comm* c, const dfmi_out_column* local,
                                             const dfmi_out_column* root_outs, int32_t root, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    if (!ctx || !c) {
        set_err(err, DFMI_ERR_INVALID_ARGUMENT, "bad argument");
        return DFMI_ERR_INVALID_ARGUMENT;
    }
    try {
        HIP_TRY(hipSetDevice(ctx->device));
        hipStream_t st = ctx->stream;
        const int nout = c->nout, world = c->world;
        auto rec = [&](int r, int i) { return c->rec[(size_t)r * kRec + i]; };
        int64_t total_rows = 0;
        for (int r = 0; r < world; ++r) total_rows += rec(r, 2);
        auto nulls_of = [&](int o) {
            int64_t x = 0;
            for (int r = 0; r < world; ++r) x += rec(r, 3 + kMaxOut + o);
            return x;
        };

        // ---- phase 1: this rank's checks and allocations, then agreement
        struct Piece {
            const void* src;
            void* dst;  // root: final place (nullptr: staged for a fix-up)
            size_t nb;
            int fix;    // -1 none, 0 offsets rebase, 1 value bits, 2 validity bits
            int o, r;
        };
        std::vector<Piece> pieces;  // (o, r) order, the same on every rank
        size_t stage_bytes = 0, ones_bytes = 0;
        int32_t code = DFMI_OK;
        std::string msg;
        try {
            if (!local || root < 0 || root >= world) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "bad argument"};
            if (c->rank == root && !root_outs) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "root outputs are NULL"};
            for (int o = 0; o < nout; ++o) {
                if (local[o].passthrough_column >= 0)
                    throw Fail{DFMI_ERR_INVALID_ARGUMENT, "output is a passthrough input column: gather the input"};
                if (local[o].type == DFMI_TYPE_UTF8) {
                    int64_t tot = 0;
                    for (int r = 0; r < world; ++r) tot += rec(r, 3 + o);
                    // i32 offsets address < 2^31 bytes (arrow BinaryArray)
                    if (tot >= ((int64_t)1 << 31)) throw Fail{DFMI_ERR_CAPACITY, "gathered Utf8 column exceeds 2^31 bytes"};
                    if (c->rank == root && root_outs[o].data_capacity < tot)
                        throw Fail{DFMI_ERR_CAPACITY, "root Utf8 data_capacity too small"};
                }
                if (c->rank == root && nulls_of(o) && !root_outs[o].validity)
                    throw Fail{DFMI_ERR_INVALID_ARGUMENT, "root validity is NULL"};
            }
            for (int o = 0; o < nout; ++o) {
                const int t = local[o].type;
                const int w = jit::type_width(t);
                const bool has_nulls = nulls_of(o) > 0;
                int64_t row0 = 0, b0 = 0;
                for (int r = 0; r < world; ++r) {
                    const int64_t n = rec(r, 2);
                    const bool mine = c->rank == root || r == c->rank;
                    if (n && mine) {
                        std::vector<Piece> pc;
                        if (t == DFMI_TYPE_UTF8) {
                            pc.push_back({local[o].data, c->rank == root ? root_outs[o].data + b0 : nullptr,
                                          (size_t)rec(r, 3 + o), -1, o, r});
                            pc.push_back({local[o].offsets, nullptr, (size_t)(n + 1) * 4, 0, o, r});
                        } else if (t == DFMI_TYPE_BOOLEAN) {
                            pc.push_back({local[o].values, nullptr, (size_t)((n + 7) / 8), 1, o, r});
                        } else {
                            pc.push_back({local[o].values,
                                          c->rank == root ? (uint8_t*)root_outs[o].values + row0 * w : nullptr,
                                          (size_t)(n * w), -1, o, r});
                        }
                        if (has_nulls) pc.push_back({local[o].validity, nullptr, (size_t)((n + 7) / 8), 2, o, r});
                        for (Piece& p : pc) {
                            if (!p.nb) continue;
                            if (r == c->rank && !p.src && p.fix != 2)
                                throw Fail{DFMI_ERR_INVALID_ARGUMENT, "local output buffer is NULL"};
                            if (c->rank == root && p.fix >= 0) {  // staged on the root, fixed up after
                                p.dst = (void*)(uintptr_t)stage_bytes;  // an offset until the staging is sized
                                stage_bytes += (p.nb + 255) & ~(size_t)255;
                            }
                            if (r == c->rank && p.fix == 2 && !p.src) {  // no validity here: all valid
                                ones_bytes = std::max(ones_bytes, p.nb);
                                p.src = nullptr;  // the comm's all-valid bitmap (below)
                            }
                            pieces.push_back(p);
                        }
                    }
                    row0 += n;
                    b0 += rec(r, 3 + o);
                }
            }
            // the staging (root) and the all-valid bitmap, kept in the comm
            if (stage_bytes > c->stage_cap) {
                if (c->stage) HIP_TRY(hipFree(c->stage));
                c->stage = nullptr;
                c->stage_cap = 0;
                HIP_TRY(hipMalloc((void**)&c->stage, stage_bytes));
                c->stage_cap = stage_bytes;
            }
            if (ones_bytes > c->ones_cap) {
                if (c->ones) HIP_TRY(hipFree(c->ones));
                c->ones = nullptr;
                c->ones_cap = 0;
                HIP_TRY(hipMalloc((void**)&c->ones, ones_bytes));
                HIP_TRY(hipMemsetAsync(c->ones, 0xff, ones_bytes, st));
                c->ones_cap = ones_bytes;
            }
            for (Piece& p : pieces) {
                if (c->rank == root && p.fix >= 0) p.dst = c->stage + (uintptr_t)p.dst;
                if (p.r == c->rank && p.fix == 2 && !p.src) p.src = c->ones;
            }
            if (c->rank == root)  // bitmaps are ORed in: start from zero
                for (int o = 0; o < nout; ++o) {
                    if (local[o].type == DFMI_TYPE_BOOLEAN)
                        HIP_TRY(hipMemsetAsync(root_outs[o].values, 0, (size_t)((total_rows + 63) / 64 * 8), st));
                    if (nulls_of(o))
                        HIP_TRY(hipMemsetAsync(root_outs[o].validity, 0, (size_t)((total_rows + 63) / 64 * 8), st));
                }
        } catch (const Fail& f) {
            code = f.code;
            msg = f.msg;
        }
        agree(ctx, c, code, msg);  // every rank fails, or every rank transfers

        // ---- phase 2: the transfers (all posted at once), then the root's fix-ups
        c->tp->group_start();
        for (const Piece& p : pieces) {
            if (c->rank == root) {
                if (p.r == root) HIP_TRY(hipMemcpyAsync(p.dst, p.src, p.nb, hipMemcpyDeviceToDevice, st));
                else c->tp->recv(ctx, p.dst, p.nb, p.r);
            } else {
                c->tp->send(ctx, p.src, p.nb, root);
            }
        }
        c->tp->group_end(ctx);
        if (c->rank == root) {
            for (const Piece& p : pieces) {
                if (p.fix < 0) continue;
                int64_t row0 = 0, b0 = 0;
                for (int q = 0; q < p.r; ++q) {
                    row0 += rec(q, 2);
                    b0 += rec(q, 3 + p.o);
                }
                const int64_t n = rec(p.r, 2);
                if (p.fix == 0)
                    HIP_TRY(launch_rebase_offsets((const int32_t*)p.dst, n, b0, root_outs[p.o].offsets + row0, st));
                else
                    HIP_TRY(launch_place_bits((const uint8_t*)p.dst, n,
                                              p.fix == 1 ? (uint8_t*)root_outs[p.o].values : root_outs[p.o].validity,
                                              row0, st));
            }
            HIP_TRY(hipStreamSynchronize(st));
        }
        return DFMI_OK;
    } catch (const Fail& f) {
        (void)hipStreamSynchronize(ctx->stream);
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

extern "C" int32_t dfmi_shard_agg_finish_grouped(dfmi_context* ctx, dfmi_shard_comm* c, dfmi_agg_state* state,
                                                 const dfmi_aggregate* const* aggs, int32_t n, int64_t cap,
                                                 dfmi_agg_value* keys, dfmi_agg_value* values, int64_t* num_groups,
                                                 dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    try {
        if (!ctx || !c || !state || !aggs || !num_groups) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        // round 1: [status | bytes | message] of every rank (a failed state
        // still takes part; every rank reports the first failing rank's error)
        const size_t rec = 16 + kMsg;
        std::vector<uint8_t> mine(rec, 0), all(rec * c->world);
        dfmi_error local{};
        const int64_t nb = dfmi_agg_state_grouped_partial_bytes(ctx, state, &local);
        std::vector<uint8_t> part(nb > 0 ? (size_t)nb : 0);
        int32_t rc = nb < 0 ? (int32_t)-nb : DFMI_OK;
        if (!rc) rc = dfmi_agg_state_grouped_partial(ctx, state, part.data(), nb, &local);
        memcpy(mine.data(), &rc, 4);
        const int64_t mb = rc ? 0 : nb;
        memcpy(mine.data() + 8, &mb, 8);
        if (rc) snprintf((char*)mine.data() + 16, kMsg, "%s", local.message);
        c->tp->all_gather(ctx, mine.data(), all.data(), rec);
        int64_t maxb = 0;
        std::vector<int64_t> sizes(c->world);
        for (int r = 0; r < c->world; ++r) {
            int32_t rr;
            memcpy(&rr, &all[(size_t)r * rec], 4);
            if (rr) {
                all[(size_t)r * rec + 16 + kMsg - 1] = 0;
                throw Fail{rr, std::string((const char*)&all[(size_t)r * rec + 16])};
            }
            memcpy(&sizes[r], &all[(size_t)r * rec + 8], 8);
            maxb = std::max(maxb, sizes[r]);
        }
        // round 2: every rank's partial, padded to the largest
        part.resize((size_t)maxb, 0);
        std::vector<uint8_t> parts_all((size_t)maxb * c->world);
        c->tp->all_gather(ctx, part.data(), parts_all.data(), (size_t)maxb);
        std::vector<const void*> parts(c->world);
        for (int r = 0; r < c->world; ++r) parts[r] = &parts_all[(size_t)r * maxb];
        (void)aggs;  // the state's own aggregates (the binding passes the same ones)
        return dfmi_agg_state_show_merged(state, parts.data(), sizes.data(), c->world, cap, keys, values, num_groups,
                                          err);
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

extern "C" int32_t dfmi_shard_agg_finish(dfmi_context* ctx, dfmi_shard_comm* c, dfmi_agg_state* state,
                                         const dfmi_aggregate* const* aggs, int32_t n, dfmi_agg_value* out,
                                         dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    try {
        if (!ctx || !c || !state || !aggs || !out) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        const int64_t nb = dfmi_agg_partial_bytes(state);
        // [status | message | partial]: a failed state still takes part (all
        // ranks enter the collective) and every rank reports the first
        // failing rank's error
        const size_t rec = 8 + kMsg + (size_t)nb;
        std::vector<uint8_t> mine(rec, 0), all(rec * c->world);
        dfmi_error local;
        const int32_t rc = dfmi_agg_state_partial(ctx, state, mine.data() + 8 + kMsg, &local);
        memcpy(mine.data(), &rc, 4);
        if (rc) snprintf((char*)mine.data() + 8, kMsg, "%s", local.message);
        c->tp->all_gather(ctx, mine.data(), all.data(), rec);
        for (int r = 0; r < c->world; ++r) {
            int32_t rr;
            memcpy(&rr, &all[(size_t)r * rec], 4);
            if (rr) {
                all[(size_t)r * rec + 8 + kMsg - 1] = 0;
                throw Fail{rr, std::string((const char*)&all[(size_t)r * rec + 8])};
            }
        }
        std::vector<const void*> parts(c->world);
        for (int r = 0; r < c->world; ++r) parts[r] = &all[(size_t)r * rec + 8 + kMsg];
        return dfmi_agg_merge_partials(aggs, n, parts.data(), c->world, out, err);
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

// ------------------------------------------------------------ test hooks
// Internal (not in include/): the C++ placement / error agreement over
// records laid out as ShardedFilterProject.exchange's (execution/shard.py) --
// the CPU suite checks both agree at world sizes 2 and 3 -- and a loopback
// communicator (threads sharing one device) for the GPU suite's
// multi-rank runs of the shard entry points on a one-GPU box.
extern "C" int32_t dfmi_internal_shard_place(int32_t world, int32_t rank, int32_t nout, const int64_t* recs,
                                             dfmi_shard_placement* out, int32_t* first_failed) {
    if (world < 1 || rank < 0 || rank >= world || nout < 0 || nout > kMaxOut || !recs || !out || !first_failed)
        return DFMI_ERR_INVALID_ARGUMENT;
    *first_failed = first_failed_rank(recs, world, kRec);
    placement_of(recs, world, rank, nout, kRec, out);
    return DFMI_OK;
}

extern "C" void* dfmi_internal_loopback_group_create(int32_t world) {
    return world >= 1 ? new LoopGroup(world) : nullptr;
}
extern "C" void dfmi_internal_loopback_group_destroy(void* g) { delete (LoopGroup*)g; }

extern "C" int32_t dfmi_internal_shard_comm_loopback(dfmi_context* ctx, void* group, int32_t rank,
                                                     dfmi_shard_comm** out, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    LoopGroup* g = (LoopGroup*)group;
    if (!ctx || !g || !out || rank < 0 || rank >= g->world) {
        set_err(err, DFMI_ERR_INVALID_ARGUMENT, "bad argument");
        return DFMI_ERR_INVALID_ARGUMENT;
    }
    auto* c = new dfmi_shard_comm();
    c->world = g->world;
    c->rank = rank;
    c->device = ctx->device;
    c->tp = new LoopTransport(g, rank);
    c->rec.assign((size_t)c->world * kRec, 0);
    *out = c;
    return DFMI_OK;
}
