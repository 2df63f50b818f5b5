// Device GROUP BY by hashing (aggregate.cpp "hashed groups", kernels in
// groupby.hip): the shapes shared by the host side and the fixed kernels.
//
// The key and aggregate arguments of a batch are first evaluated by the fused
// Selection + Projection pass (dfmi_filter_project: projections [keys...,
// args...], the reference's evaluation order and first error), so these
// kernels only ever see compacted, offset-0 columns. Per batch:
//   k_group_claim       every row hashes its key and finds its slot in an
//                       open-addressing table (linear probing); a row that
//                       finds an empty slot claims it with a CAS on `ctl`
//                       and becomes the slot's representative row, takes the
//                       next dense group id, and reserves arena bytes for its
//                       Utf8 key parts. Nothing but `ctl` is read from the
//                       table in this kernel, so no cross-XCD hand-off
//                       depends on L2 coherence within the launch.
//   k_group_accumulate  every row checks its key against its slot's key --
//                       the representative row of this batch (a slot
//                       claimed by this launch's claim pass), or the key
//                       persisted by an earlier batch -- and adds its
//                       values into the group's accumulators with atomics;
//                       the representative row persists its key. A row
//                       whose key differs from the slot's (two keys with one
//                       63-bit hash) is listed; the host merges those rows
//                       (exactly, aggregate.cpp).
#ifndef DFMI_GROUPBY_H
#define DFMI_GROUPBY_H

#include <hip/hip_runtime_api.h>

#include <cstdint>

namespace dfmi {
namespace gb {

constexpr int kMaxKeys = 4;   // GROUP BY key expressions
constexpr int kMaxAggs = 15;  // aggregates of one grouped state

// One key part or aggregate argument: a compacted output column (or a
// passed-through input column) of the fused pass.
struct Col {
    int32_t type;              // dfmi_type
    int32_t width;             // value bytes (0: Boolean bitmap / Utf8)
    const void* values;        // fixed-width values / Boolean bitmap / Utf8 bytes
    const int32_t* offsets;    // Utf8
    const uint8_t* validity;   // nullptr: every value valid
};

// A slot's record: one 64-byte line piece, so a row's check of its slot
// (k_group_rank / row_group) is one random access, not one per field.
constexpr unsigned kNullBits = 0xffu;   // Slot::knull: the null bits of the key parts
constexpr unsigned kInline = 1u << 8;   // Slot::knull: a one-part Utf8 key of <= 24 bytes, its bytes in kw[1..3]

struct alignas(64) Slot {
    long long rep;                    // (epoch << 32) | representative row of the claiming batch
    unsigned gid;                     // dense group id
    unsigned knull;                   // bit p: key part p is null; kInline
    unsigned long long kw[kMaxKeys];  // persisted key words (Utf8: arena offset)
    unsigned klen[kMaxKeys];          // Utf8 key bytes
};

// The table (capacity cap = mask + 1 slots): the probe words apart (dense for
// the claim's linear probing), the slots' records beside them.
struct Table {
    unsigned long long* ctl;   // [cap] 0: empty; else the key's hash | 1 (written once, by CAS)
    Slot* slot;                // [cap]
    unsigned long long mask;   // cap - 1
};

// Device header (one per state): counters the host reads after a pass.
struct Hdr {
    unsigned long long ngroups;    // groups (claimed slots)
    unsigned long long arena_end;  // Utf8 arena bytes reserved
    unsigned long long overflow;   // nonzero: a row found no slot (table past its load limit)
    unsigned long long collided;   // rows whose key differs from their slot's (listed)
    unsigned long long pad[4];
};

struct ClaimArgs {
    Col k[kMaxKeys];
    int32_t nkeys;
    uint32_t epoch;                // this batch's number (rep words)
    long long m;                   // rows
    Table t;
    unsigned long long limit;      // claim no slot once ngroups >= limit (the host grows the table)
    unsigned long long hash_mask;  // diagnostics: ~0 (DFMI_GROUP_HASH_BITS narrows it to force collisions)
    Hdr* hdr;
    int32_t* sidx;                 // [m] the row's slot (-1: not placed)
};

struct AggCol {
    Col c;
    int32_t fn;    // dfmi_agg_fn
    int32_t off;   // word offset of this aggregate in a group's record
};

// A group's accumulator record: word 0 = the group's rows, then per
// aggregate [nulls, flags, key, aux] (+ kAggLimbs exact-sum digits for a
// floating-point SUM): nulls = the group's rows whose argument is NULL (the
// non-null count is rows - nulls: no atomic per row for it); aux: integer
// SUM the wrapping sum; MIN / MAX the NaN values seen; float SUM the values
// that are not finite-and-not-(-0.0).
struct AccArgs {
    Col k[kMaxKeys];
    int32_t nkeys;
    uint32_t epoch;
    long long m;
    Table t;
    unsigned char* arena;          // Utf8 key bytes of every group
    unsigned long long arena_cap;  // its allocated bytes
    const int32_t* sidx;
    AggCol a[kMaxAggs];
    int32_t naggs;
    int32_t words;                 // words per group record
    unsigned long long* acc;       // [groups][words]
    Hdr* hdr;
    int32_t* coll_rows;            // [m] rows whose key differs from the slot's
};

// Bucketed accumulation (many rows per group: aggregate.cpp use_buckets). The
// accumulate pass's scattered record atomics -- one request per lane, the
// chip's slowest atomic shape (MI355X_MICROARCH.md "Global float atomics") --
// replaced by a partition of the rows by group and a per-bucket sum in LDS:
//   k_group_rank     the accumulate pass's key check per row (the same
//                    representative / persisted-key rules, colliding rows
//                    listed); the row's group id into rg, and per block the
//                    rows of each bucket (gpb = 2^gshift consecutive group
//                    ids) into bh
//   k_group_scan     per bucket, the exclusive prefix of its per-block
//                    counts (in place) and its total; a bucket starts at the
//                    sum of the totals before it
//   k_group_scatter  the same rows per block as the rank pass: each placed
//                    row's group id, NULL mask and argument bits written at
//                    its bucket's next position (LDS counters)
//   k_group_bucket   per (bucket, split) block: the bucket's records in LDS,
//                    every row of its share added with LDS atomics, then
//                    each record word that moved added once into the
//                    group's global record (atomics over contiguous words)
// Integer digit sums are order-free: the records equal the accumulate pass's.
constexpr int kBucketMax = 1024;  // buckets per pass (4,096 measured slower: 1e8 rows x 10k keys 4.6 -> 5.5 ms,
                                  // the rank / scatter LDS counters cost occupancy; 1e5 keys unchanged)
// LDS bytes of a bucket block's records: 64 KiB less its bucket starts (and the scan's scratch)
constexpr int kBucketRecordLds = 65536 - 4 * (kBucketMax + 1) - 1024;
constexpr int kBucketRecordLdsBig = 163840 - 4 * (kBucketMax + 1) - 1024;  // one block per CU
constexpr int kBucketBlocks = 1024;  // blocks of the rank and scatter passes (= k_group_scan's block size)

struct RankArgs {
    Col k[kMaxKeys];
    int32_t nkeys;
    uint32_t epoch;
    long long m;
    Table t;
    unsigned char* arena;
    unsigned long long arena_cap;
    const int32_t* sidx;
    Hdr* hdr;
    int32_t* coll_rows;
    unsigned* rg;      // [m] the row's group id, ~0u: not added here (listed)
    int32_t gshift;    // groups per bucket: 1 << gshift
    int32_t nbuckets;
    unsigned* bh;      // [nbuckets][kBucketBlocks] rows per (bucket, block) (k_group_scan: their exclusive prefixes)
};

struct ScatterArgs {
    long long m;
    const unsigned* rg;
    int32_t gshift;
    int32_t nbuckets;
    const unsigned* base;        // k_group_scan's output: per (bucket, block) its first position in the bucket
    const unsigned* tot;         // [nbuckets] rows per bucket
    int32_t naggs;
    Col arg[kMaxAggs];           // aggregate j's argument column (its NULLs)
    Col pay[kMaxAggs];           // payload column c's source (the arguments whose values are needed, once each)
    int32_t npay;
    unsigned* pg;                // [placed] group ids in bucket order
    unsigned* pn;                // [placed] NULL mask (bit j: argument j NULL); nullptr: no nullable argument
    unsigned long long* pv;      // [npay][m] argument bits (integers sign/zero-extended, float raw bits)
};

struct BucketArgs {
    long long m;                 // pv's column stride
    const unsigned* tot;
    uint32_t gpb;
    int32_t nbuckets;
    int32_t splits;              // blocks per bucket
    unsigned long long ngroups;
    const unsigned* pg;
    const unsigned* pn;
    const unsigned long long* pv;
    AggCol a[kMaxAggs];          // type, fn, record offset (a[j].c.values unused)
    int32_t pcol[kMaxAggs];
    int32_t naggs;
    int32_t words;
    unsigned long long* acc;
    const unsigned long long* pattern;  // one zero-state record
};

hipError_t launch_buckets(const RankArgs& r, ScatterArgs s, BucketArgs b, hipStream_t stream);

// The finish of every group on the device (k_group_round): per group a
// compact record [rows, then per aggregate nulls, flags, key, aux] -- the
// record without its exact-sum digits; a floating-point SUM's key word holds
// its digits rounded once, half to even (aggregate.cpp round_exact restated:
// kind 1 to a Float64, kind 2 to a Float32's value as a double), and its
// flags word kRoundZero when the exact sum is 0.
struct RoundArgs {
    const unsigned long long* acc;  // [ngroups][words]
    int32_t words;
    int32_t naggs;
    int32_t off[kMaxAggs];          // word offset of aggregate j in a record
    int32_t kind[kMaxAggs];         // 0: copied; 1: Float64 SUM; 2: Float32 SUM
    unsigned long long ngroups;
    unsigned long long* out;        // [ngroups][1 + 4 * naggs]
};
constexpr unsigned long long kRoundZero = 1ull << 32;

// The finish's ordering and emission on the device (one fixed-width key part:
// aggregate.cpp finish_device): every group's sort value (key_ord restated,
// the null group ~0 and moved last afterwards), a radix sort of (value, group
// id), then one dfmi_agg_value per key and per aggregate in key order, from
// the compact records of k_group_round -- aggregate.cpp finish_normalized
// restated.
struct EmitArgs {
    const unsigned long long* rec;   // [ngroups][1 + 4 * naggs] compact records
    const unsigned* knull;           // [ngroups] the key's null bit
    const unsigned long long* kw;    // [ngroups] the key's bits
    const unsigned* order;           // [ngroups] group ids in key order (the null group anywhere)
    const unsigned* null_at;         // [2]: the null group's id (~0u: none), its position in `order`
    unsigned long long ngroups;
    int32_t ktype;
    int32_t naggs;
    int32_t fn[kMaxAggs], atype[kMaxAggs], rtype[kMaxAggs];
    void* keys;                      // [ngroups] dfmi_agg_value
    void* values;                    // [ngroups][naggs] dfmi_agg_value
};
// Sort values and group ids (k_group_sortkey), their radix sort (rocPRIM, the
// temporary storage `tmp` of `tmp_bytes`; tmp == nullptr: *tmp_bytes is set),
// the null group's position, the emission.
hipError_t launch_emit(EmitArgs a, unsigned long long* sk, unsigned long long* sk2, unsigned* sv, unsigned* sv2,
                       unsigned* null_at, void* tmp, size_t* tmp_bytes, hipStream_t stream);

// groupby.hip: launches on `stream` (asynchronous)
hipError_t launch_claim(const ClaimArgs& a, hipStream_t stream);
hipError_t launch_accumulate(const AccArgs& a, hipStream_t stream);
hipError_t launch_rehash(const Table& from, const Table& to, hipStream_t stream);
hipError_t launch_compact(const Table& t, int nkeys, unsigned* knull, unsigned long long* kw, unsigned* klen,
                          hipStream_t stream);
hipError_t launch_init(unsigned long long* acc, const unsigned long long* pattern, int words, unsigned long long g0,
                       unsigned long long g1, hipStream_t stream);
hipError_t launch_round(const RoundArgs& a, hipStream_t stream);
hipError_t launch_normalize(unsigned long long* acc, int words, const int* foff, int nf, unsigned long long ngroups,
                            hipStream_t stream);

}  // namespace gb
}  // namespace dfmi

#endif
