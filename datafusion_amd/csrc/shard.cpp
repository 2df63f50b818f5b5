// Multi-GPU form of the path: row-range shards, one host
// thread / process per GPU, RCCL over xGMI for the only exchange the path
// has. The reference has no parallelism at all (context.rs:33, one
// Rc<RefCell<..>> pull); rows are independent through FilterRelation /
// ProjectRelation and filter() preserves row order (filter.rs:87-91), so the
// per-rank outputs in rank order ARE the reference's output stream.
//
//   dfmi_shard_filter_project: the local fused pass, then ONE ncclAllGather of
//     a fixed int64 record per rank (status, error order key, selected rows,
//     Utf8 bytes and null count per output) -> every rank's global placement;
//     a failure anywhere becomes the same (globally first) error on every rank.
//   dfmi_shard_gather_to_root: optional concatenation on one rank with grouped
//     ncclSend / ncclRecv (RCCL has no gatherv), bound by the root's xGMI
//     ingress; Utf8 offsets rebased and bitmaps re-aligned on the root.
//   dfmi_shard_agg_finish: the aggregate extension's exact partials,
//     ncclAllGather'ed and merged -- bit-identical to one GPU over all rows.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>
#include <vector>

#include "exec_internal.h"

using namespace dfmi;
using namespace dfmi::xi;

namespace dfmi {
hipError_t launch_rebase_offsets(const int32_t* src, long long n, long long base, int32_t* dst, hipStream_t st);
hipError_t launch_place_bits(const uint8_t* src, long long n, uint8_t* dst, long long dst_bit, hipStream_t st);
}  // namespace dfmi

namespace {
constexpr int kMaxOut = 16;
constexpr int kRec = 3 + 2 * kMaxOut;  // status, error key, rows, utf8 bytes[16], nulls[16]
constexpr int kMsg = 512;

#define NCCL_TRY(x)                                                                                         \
    do {                                                                                                    \
        ncclResult_t r_ = (x);                                                                              \
        if (r_ != ncclSuccess) throw Fail{DFMI_ERR_DEVICE, std::string(#x ": ") + ncclGetErrorString(r_)}; \
    } while (0)
}  // namespace

struct dfmi_shard_comm {
    int world = 1, rank = 0, device = 0;
    ncclComm_t comm = nullptr;
    int64_t* d_rec = nullptr;  // [world][kRec] device exchange buffer
    char* d_msg = nullptr;     // [world][kMsg]
    std::vector<int64_t> rec;  // the last exchange, host copy
    int nout = 0;              // outputs of the last exchanged pass
};

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
        HIP_TRY(hipSetDevice(ctx->device));
        ncclUniqueId u;
        memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
        NCCL_TRY(ncclCommInitRank(&c->comm, world, u, rank));
        HIP_TRY(hipMalloc((void**)&c->d_rec, (size_t)world * kRec * 8));
        HIP_TRY(hipMalloc((void**)&c->d_msg, (size_t)world * kMsg));
        c->rec.assign((size_t)world * kRec, 0);
        *out = c;
        return DFMI_OK;
    } catch (const Fail& f) {
        if (c) {
            if (c->comm) ncclCommDestroy(c->comm);
            if (c->d_rec) (void)hipFree(c->d_rec);
            if (c->d_msg) (void)hipFree(c->d_msg);
            delete c;
        }
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

extern "C" void dfmi_shard_comm_destroy(dfmi_shard_comm* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->comm) ncclCommDestroy(c->comm);
    if (c->d_rec) (void)hipFree(c->d_rec);
    if (c->d_msg) (void)hipFree(c->d_msg);
    delete c;
}

namespace {
// One all_gather of every rank's record; on a failure anywhere, every rank
// throws the globally first error -- the smallest evaluation ordinal, then
// the lowest rank (= earliest rows), as the reference over the whole table
// would raise it -- with the failing rank's message.
void exchange(dfmi_context* ctx, dfmi_shard_comm* c, const int64_t* mine, const dfmi_error& local) {
    hipStream_t st = ctx->stream;
    int64_t* send = c->d_rec + (size_t)c->rank * kRec;
    HIP_TRY(hipMemcpyAsync(send, mine, kRec * 8, hipMemcpyHostToDevice, st));
    NCCL_TRY(ncclAllGather(send, c->d_rec, kRec, ncclInt64, c->comm, st));
    HIP_TRY(hipMemcpyAsync(c->rec.data(), c->d_rec, c->rec.size() * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    int first = -1;
    for (int r = 0; r < c->world; ++r) {
        const int64_t* rr = &c->rec[(size_t)r * kRec];
        if (!rr[0]) continue;
        if (first < 0 || ((uint64_t)rr[1] >> 44) < ((uint64_t)c->rec[(size_t)first * kRec + 1] >> 44)) first = r;
    }
    if (first < 0) return;
    char msg[kMsg] = {};
    snprintf(msg, sizeof msg, "%s", local.message);
    char* msend = c->d_msg + (size_t)c->rank * kMsg;
    HIP_TRY(hipMemcpyAsync(msend, msg, kMsg, hipMemcpyHostToDevice, st));
    NCCL_TRY(ncclAllGather(msend, c->d_msg, kMsg, ncclChar, c->comm, st));
    std::vector<char> all((size_t)c->world * kMsg);
    HIP_TRY(hipMemcpyAsync(all.data(), c->d_msg, all.size(), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    all[(size_t)(first + 1) * kMsg - 1] = 0;
    throw Fail{(int32_t)c->rec[(size_t)first * kRec], std::string(&all[(size_t)first * kMsg])};
}
}  // namespace

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
        const int32_t rc = dfmi_filter_project(ctx, pred, projs, np, in, outs, flags, &local);
        int64_t mine[kRec] = {};
        mine[0] = rc;
        mine[1] = rc ? (int64_t)ctx->last_err_key : 0;
        if (rc == DFMI_OK) {
            mine[2] = nout ? outs[0].length : 0;
            for (int o = 0; o < nout; ++o) {
                mine[3 + o] = outs[o].type == DFMI_TYPE_UTF8 ? outs[o].data_length : 0;
                mine[3 + kMaxOut + o] = outs[o].null_count;
            }
        }
        exchange(ctx, c, mine, local);  // throws the globally first error on every rank
        c->nout = nout;
        memset(place, 0, sizeof *place);
        place->world = c->world;
        place->rank = c->rank;
        for (int r = 0; r < c->world; ++r) {
            const int64_t* rr = &c->rec[(size_t)r * kRec];
            if (r < c->rank) place->row_offset += rr[2];
            place->total_rows += rr[2];
            for (int o = 0; o < nout; ++o) {
                if (r < c->rank) place->utf8_base[o] += rr[3 + o];
                place->utf8_total[o] += rr[3 + o];
                place->null_total[o] += rr[3 + kMaxOut + o];
            }
        }
        return DFMI_OK;
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

extern "C" int32_t dfmi_shard_gather_to_root(dfmi_context* ctx, dfmi_shard_comm* c, const dfmi_out_column* local,
                                             const dfmi_out_column* root_outs, int32_t root, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    try {
        if (!ctx || !c || !local || root < 0 || root >= c->world) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "bad argument"};
        if (c->rank == root && !root_outs) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "root outputs are NULL"};
        hipStream_t st = ctx->stream;
        HIP_TRY(hipSetDevice(ctx->device));
        const int nout = c->nout, world = c->world;
        auto rec = [&](int r, int i) { return c->rec[(size_t)r * kRec + i]; };
        for (int o = 0; o < nout; ++o)
            if (local[o].type == DFMI_TYPE_UTF8) {
                int64_t tot = 0;
                for (int r = 0; r < world; ++r) tot += rec(r, 3 + o);
                // i32 offsets address < 2^31 bytes (arrow BinaryArray)
                if (tot >= ((int64_t)1 << 31)) throw Fail{DFMI_ERR_CAPACITY, "gathered Utf8 column exceeds 2^31 bytes"};
                if (c->rank == root && root_outs[o].data_capacity < tot)
                    throw Fail{DFMI_ERR_CAPACITY, "root Utf8 data_capacity too small"};
            }
        // staging on the root for pieces that need re-alignment (offsets, bitmaps)
        std::vector<uint8_t*> stage;
        auto stage_buf = [&](size_t nb) {
            uint8_t* p = nullptr;
            HIP_TRY(hipMalloc((void**)&p, nb ? nb : 8));
            stage.push_back(p);
            return p;
        };
        for (int o = 0; o < nout; ++o)
            if (local[o].passthrough_column >= 0)
                throw Fail{DFMI_ERR_INVALID_ARGUMENT, "output is a passthrough input column: gather the input"};
        int64_t total_rows = 0;
        for (int r = 0; r < world; ++r) total_rows += rec(r, 2);
        if (c->rank == root)  // bitmaps are ORed in: start from zero
            for (int o = 0; o < nout; ++o) {
                int64_t nulls = 0;
                for (int r = 0; r < world; ++r) nulls += rec(r, 3 + kMaxOut + o);
                if (local[o].type == DFMI_TYPE_BOOLEAN)
                    HIP_TRY(hipMemsetAsync(root_outs[o].values, 0, (size_t)((total_rows + 63) / 64 * 8), st));
                if (nulls) {
                    if (!root_outs[o].validity) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "root validity is NULL"};
                    HIP_TRY(hipMemsetAsync(root_outs[o].validity, 0, (size_t)((total_rows + 63) / 64 * 8), st));
                }
            }
        struct Fix {
            int kind;  // 0 offsets rebase, 1 value bits, 2 validity bits
            int o, r;
            uint8_t* buf;
        };
        std::vector<Fix> fixes;
        try {
            NCCL_TRY(ncclGroupStart());
            for (int o = 0; o < nout; ++o) {
                const int t = local[o].type;
                const bool bits = t == DFMI_TYPE_BOOLEAN;
                const int w = jit::type_width(t);
                int64_t nulls = 0;
                for (int r = 0; r < world; ++r) nulls += rec(r, 3 + kMaxOut + o);
                for (int r = 0; r < world; ++r) {
                    const int64_t n = rec(r, 2);
                    if (!n) continue;
                    int64_t row0 = 0, b0 = 0;
                    for (int q = 0; q < r; ++q) {
                        row0 += rec(q, 2);
                        b0 += rec(q, 3 + o);
                    }
                    // (pointer, bytes) of rank r's buffers, in an order both sides agree on
                    struct Piece {
                        const void* src;
                        void* dst;  // root: final place, or nullptr = staged
                        size_t nb;
                        int fix;
                    };
                    std::vector<Piece> pieces;
                    if (t == DFMI_TYPE_UTF8) {
                        pieces.push_back({local[o].data, c->rank == root ? root_outs[o].data + b0 : nullptr,
                                          (size_t)rec(r, 3 + o), -1});
                        pieces.push_back({local[o].offsets, nullptr, (size_t)(n + 1) * 4, 0});
                    } else if (bits) {
                        pieces.push_back({local[o].values, nullptr, (size_t)((n + 7) / 8), 1});
                    } else {
                        pieces.push_back({local[o].values,
                                          c->rank == root ? (uint8_t*)root_outs[o].values + row0 * w : nullptr,
                                          (size_t)(n * w), -1});
                    }
                    if (nulls) pieces.push_back({local[o].validity, nullptr, (size_t)((n + 7) / 8), 2});
                    for (const Piece& p : pieces) {
                        if (!p.nb) continue;
                        if (c->rank == root) {
                            uint8_t* dst = (uint8_t*)p.dst;
                            if (p.fix >= 0) {
                                dst = stage_buf(p.nb);
                                fixes.push_back({p.fix, o, r, dst});
                            }
                            if (r == root) {
                                if (p.fix == 2 && !p.src) {  // this rank has no validity: all valid
                                    HIP_TRY(hipMemsetAsync(dst, 0xff, p.nb, st));
                                } else {
                                    HIP_TRY(hipMemcpyAsync(dst, p.src, p.nb, hipMemcpyDeviceToDevice, st));
                                }
                            } else {
                                NCCL_TRY(ncclRecv(dst, p.nb, ncclUint8, r, c->comm, st));
                            }
                        } else if (r == c->rank) {
                            const void* src = p.src;
                            if (p.fix == 2 && !src) {  // all valid
                                uint8_t* ones = stage_buf(p.nb);
                                HIP_TRY(hipMemsetAsync(ones, 0xff, p.nb, st));
                                src = ones;
                            }
                            NCCL_TRY(ncclSend(src, p.nb, ncclUint8, root, c->comm, st));
                        }
                    }
                }
            }
            NCCL_TRY(ncclGroupEnd());
            // root: rebase offsets / place bitmaps at the global row offset
            if (c->rank == root) {
                for (const Fix& f : fixes) {
                    int64_t row0 = 0, b0 = 0;
                    for (int q = 0; q < f.r; ++q) {
                        row0 += rec(q, 2);
                        b0 += rec(q, 3 + f.o);
                    }
                    const int64_t n = rec(f.r, 2);
                    if (f.kind == 0)
                        HIP_TRY(launch_rebase_offsets((const int32_t*)f.buf, n, b0, root_outs[f.o].offsets + row0, st));
                    else
                        HIP_TRY(launch_place_bits(f.buf, n, f.kind == 1 ? (uint8_t*)root_outs[f.o].values
                                                                        : root_outs[f.o].validity,
                                                  row0, st));
                }
            }
            HIP_TRY(hipStreamSynchronize(st));
        } catch (...) {
            for (uint8_t* p : stage) (void)hipFree(p);
            throw;
        }
        for (uint8_t* p : stage) (void)hipFree(p);
        return DFMI_OK;
    } catch (const Fail& f) {
        set_err(err, f.code, f.msg);
        return f.code;
    }
}

extern "C" int32_t dfmi_shard_agg_finish(dfmi_context* ctx, dfmi_shard_comm* c, dfmi_agg_state* state,
                                         const dfmi_aggregate* const* aggs, int32_t n, dfmi_agg_value* out,
                                         dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    uint8_t* d = nullptr;
    try {
        if (!ctx || !c || !state || !aggs || !out) throw Fail{DFMI_ERR_INVALID_ARGUMENT, "NULL argument"};
        const int64_t nb = dfmi_agg_partial_bytes(state);
        // a failed state still takes part (all ranks must enter the collective)
        std::vector<uint8_t> mine((size_t)nb + 8, 0), all((size_t)(nb + 8) * c->world);
        dfmi_error local;
        int32_t rc = dfmi_agg_state_partial(ctx, state, mine.data() + 8, &local);
        memcpy(mine.data(), &rc, 4);
        hipStream_t st = ctx->stream;
        HIP_TRY(hipMalloc((void**)&d, all.size()));
        HIP_TRY(hipMemcpyAsync(d + (size_t)c->rank * (nb + 8), mine.data(), nb + 8, hipMemcpyHostToDevice, st));
        NCCL_TRY(ncclAllGather(d + (size_t)c->rank * (nb + 8), d, nb + 8, ncclUint8, c->comm, st));
        HIP_TRY(hipMemcpyAsync(all.data(), d, all.size(), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        (void)hipFree(d);
        d = nullptr;
        for (int r = 0; r < c->world; ++r) {
            int32_t rr;
            memcpy(&rr, &all[(size_t)r * (nb + 8)], 4);
            if (rr) {
                if (r == c->rank) throw Fail{rc, local.message};
                throw Fail{rr, "aggregate failed on rank " + std::to_string(r)};
            }
        }
        std::vector<const void*> parts(c->world);
        for (int r = 0; r < c->world; ++r) parts[r] = &all[(size_t)r * (nb + 8) + 8];
        return dfmi_agg_merge_partials(aggs, n, parts.data(), c->world, out, err);
    } catch (const Fail& f) {
        if (d) (void)hipFree(d);
        set_err(err, f.code, f.msg);
        return f.code;
    }
}
