// Device GROUP BY by hashing: the fixed gfx950 kernels (groupby.h has the
// protocol; aggregate.cpp drives them). Every kernel takes compacted,
// offset-0 columns -- the fused Selection + Projection pass has already
// evaluated the keys and the aggregate arguments.
//
// Per-row rules are those of the aggregate kernels (jit_skeleton.hip agg_key
// / agg_sum_flags / fsum_add) and of the host merge (aggregate.cpp
// host_accumulate_t): COUNT counts non-null values, integer SUM wraps, a float
// SUM is the exact sum of 32-bit digits in units of 2^-1074, MIN / MAX use
// the order-preserving key (NaN never keyed, -0.0 below +0.0).
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include "../../include/dfmi.h"
#include "groupby.h"
#include "jit_skeleton.hip"

namespace dfmi {
namespace gb {

typedef unsigned long long u64_ua __attribute__((aligned(1)));

__device__ __forceinline__ u64 gmix(u64 z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ bool valid_at(const Col& c, long long i) {
    return !c.validity || ((c.validity[i >> 3] >> (i & 7)) & 1);
}

// Fixed-width key bits: Boolean 0/1, signed integers sign-extended, unsigned
// zero-extended, floats their raw bits (one group per bit pattern).
__device__ __forceinline__ u64 key_bits(const Col& c, long long i) {
    switch (c.type) {
        case 1: return (((const u8*)c.values)[i >> 3] >> (i & 7)) & 1;  // DFMI_TYPE_BOOLEAN
        case 2: return (u64)(i64)((const i8*)c.values)[i];
        case 3: return (u64)(i64)((const i16*)c.values)[i];
        case 4: return (u64)(i64)((const i32*)c.values)[i];
        case 5: return (u64)((const i64*)c.values)[i];
        case 6: return (u64)((const u8*)c.values)[i];
        case 7: return (u64)((const u16*)c.values)[i];
        case 8: return (u64)((const u32*)c.values)[i];
        case 9: return ((const u64*)c.values)[i];
        case 10: return (u64)((const u32*)c.values)[i];  // Float32 bits
        case 11: return ((const u64*)c.values)[i];       // Float64 bits
        default: return 0;
    }
}

constexpr int kTypeUtf8 = 12;

// Bytes [8j, 8j + 8) of the len bytes at p as a little-endian word, zero
// past len: one unaligned load where it cannot read past `endp` (the
// column's last byte + 1), else byte loads -- the same word either way.
__device__ __forceinline__ u64 load_word(const u8* p, unsigned len, unsigned j, const u8* endp) {
    const unsigned b0 = 8 * j;
    if (len <= b0) return 0;
    const unsigned vb = len - b0 < 8 ? len - b0 : 8;
    if (p + b0 + 8 <= endp) {
        const u64 x = *(const u64_ua*)(p + b0);
        return vb == 8 ? x : x & ((1ull << (8 * vb)) - 1);
    }
    u64 t = 0;
    for (unsigned q = 0; q < vb; ++q) t |= (u64)p[b0 + q] << (8 * q);
    return t;
}

__device__ __forceinline__ u64 hash_bytes(const u8* p, unsigned len, u64 h, const u8* endp) {
    unsigned j = 0;
    for (; j + 8 <= len; j += 8) h = gmix(h ^ *(const u64_ua*)(p + j)) + 0x9E3779B97F4A7C15ull;
    const u64 t = load_word(p, len, j >> 3, endp);
    return gmix(h ^ t ^ ((u64)len << 56));
}

__device__ __forceinline__ bool bytes_eq(const u8* a, const u8* b, unsigned len, const u8* enda, const u8* endb) {
    unsigned j = 0;
    for (; j + 8 <= len; j += 8)
        if (*(const u64_ua*)(a + j) != *(const u64_ua*)(b + j)) return false;
    return j == len || load_word(a, len, j >> 3, enda) == load_word(b, len, j >> 3, endb);
}

// A one-part Utf8 key of at most 24 bytes is kept in the slot itself too
// (Slot::kw[1..3], groupby.h kInline), so that checking a row against its
// slot reads no arena and no representative row.

__device__ __forceinline__ void inline_pack(const u8* p, unsigned len, u64 (&w)[3]) {
    w[0] = w[1] = w[2] = 0;
    for (unsigned j = 0; j < len; ++j) w[j >> 3] |= (u64)p[j] << (8 * (j & 7));
}

__device__ __forceinline__ bool inline_eq(const u8* p, unsigned len, const u64* w, const u8* endp) {
    return load_word(p, len, 0, endp) == w[0] && (len <= 8 || load_word(p, len, 1, endp) == w[1]) &&
           (len <= 16 || load_word(p, len, 2, endp) == w[2]);
}

// The row's key: null mask, fixed-width bits, Utf8 (start, length); its hash.
struct RowKey {
    unsigned nullm;
    u64 w[kMaxKeys];
    const u8* s[kMaxKeys];
    unsigned len[kMaxKeys];
    const u8* end[kMaxKeys];  // Utf8: the column's last byte + 1
};

template <int NK, bool HASH = true>
__device__ __forceinline__ u64 row_key(const Col* k, long long i, long long m, RowKey& r) {
    u64 h = 0x243F6A8885A308D3ull;
    r.nullm = 0;
#pragma unroll
    for (int p = 0; p < NK; ++p) {
        const Col& c = k[p];
        r.w[p] = 0;
        r.s[p] = nullptr;
        r.len[p] = 0;
        if (!valid_at(c, i)) {
            r.nullm |= 1u << p;
            h = gmix(h + 0x5BD1E9955BD1E995ull * (u64)(p + 1));
        } else if (c.type == kTypeUtf8) {
            const int a = c.offsets[i], b = c.offsets[i + 1];
            r.s[p] = (const u8*)c.values + a;
            r.len[p] = (unsigned)(b - a);
            r.end[p] = (const u8*)c.values + c.offsets[m];
            if (HASH) h = hash_bytes(r.s[p], r.len[p], h + (u64)p, r.end[p]);
        } else {
            r.w[p] = key_bits(c, i);
            h = gmix(h ^ (r.w[p] * 0xD6E8FEB86659FD93ull + (u64)p));
        }
    }
    return h;
}

// ------------------------------------------------------------ claim pass
// One row's slot: linear probing from slot s, whose probe word the caller has
// already loaded (`cur`); an empty slot is claimed with a CAS. -1: no slot
// (the table is at its load limit, or past it after 8 probes, or the probe
// ran past kProbeMax slots: the host grows the table and runs the pass again
// -- every row again, so a row given up here is placed then).
constexpr u64 kProbeMax = 4096;

template <int NK>
__device__ __forceinline__ int claim_row(const ClaimArgs& A, const RowKey& r, u64 c, u64 s, u64 cur, long long i) {
    const Table& t = A.t;
    for (u64 probe = 0; probe <= t.mask && probe < kProbeMax; ++probe) {
        if (probe) {
            s = (s + 1) & t.mask;
            cur = __hip_atomic_load(&t.ctl[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        // a long probe into a table past its load limit (claims racing past the
        // limit can fill it): give up, the pass reruns on the grown table
        if (probe == 8 && __hip_atomic_load(&A.hdr->ngroups, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= A.limit)
            return -1;
        if (cur == 0) {
            if (__hip_atomic_load(&A.hdr->ngroups, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= A.limit) return -1;
            cur = atomicCAS(&t.ctl[s], 0ull, c);
            if (cur == 0) {  // claimed: this row represents the slot's key
                Slot& sr = t.slot[s];
                // the next dense group id: one counter add per wave for the lanes claiming together
                // (a single counter takes ~88 adds per us: MI355X_MICROARCH.md "dequeue")
                const u64 cl = __ballot(1);
                const int lead = __builtin_ctzll(cl);
                const unsigned below = __builtin_amdgcn_mbcnt_hi((unsigned)(cl >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)cl, 0u));
                u64 g0 = 0;
                if (below == 0) g0 = atomicAdd(&A.hdr->ngroups, (u64)__builtin_popcountll(cl));
                g0 = readlane_u64(g0, lead);
                sr.gid = (unsigned)(g0 + below);
                sr.rep = ((long long)A.epoch << 32) | (long long)(unsigned)i;
                sr.knull = r.nullm;
#pragma unroll
                for (int p = 0; p < NK; ++p) {
                    u64 w = r.w[p];
                    if (r.s[p]) w = atomicAdd(&A.hdr->arena_end, (u64)r.len[p]);
                    sr.kw[p] = w;
                    sr.klen[p] = r.len[p];
                }
                // a key whose only non-null Utf8 part fits the slot's spare words
                // (kw[NK..3]: 24 bytes with one part, 16 with two, 8 with three): its
                // bytes in the slot too
                if (NK < kMaxKeys) {
                    int nu = 0;
                    const u8* ps = nullptr;
                    unsigned pl = 0;
#pragma unroll
                    for (int p = 0; p < NK; ++p)
                        if (r.s[p]) {
                            ++nu;
                            ps = r.s[p];
                            pl = r.len[p];
                        }
                    if (nu == 1 && pl <= 8u * (kMaxKeys - NK)) {
                        u64 w[3];
                        inline_pack(ps, pl, w);
#pragma unroll
                        for (int q = NK; q < kMaxKeys; ++q) sr.kw[q] = w[q - NK];
                        sr.knull = r.nullm | kInline;
                    }
                }
                return (int)s;
            }
        }
        if (cur == c) return (int)s;
    }
    return -1;
}

// NK: key parts (a template parameter so a row's key stays in registers).
// One row per thread (4 rows per thread with their keys, hashes and first
// probes loaded together measured slower, twice: 0.90 -> 1.13 ms per 1e8 rows
// with agent-scope probes, 0.89 -> 1.04 ms with L1-cached ones).
template <int NK>
__global__ __launch_bounds__(256) void k_group_claim(const ClaimArgs A) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    const Table& t = A.t;
    bool overflow = false;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < A.m; i += stride) {
        RowKey r;
        const u64 c = (row_key<NK>(A.k, i, A.m, r) & A.hash_mask) | 1ull;
        const u64 s = gmix(c) & t.mask;
        // (workgroup scope: a plain, L1-cached load -- a stale 0 only sends the row to the
        // CAS, which returns the slot's real word; with few keys every CU reads the same
        // few lines, which agent-scope loads would take from one L2 channel each time)
        const u64 cur = __hip_atomic_load(&t.ctl[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const int res = cur == c ? (int)s : claim_row<NK>(A, r, c, s, cur, i);
        if (res < 0) overflow = true;
        A.sidx[i] = res;
    }
    if (overflow) atomicOr(&A.hdr->overflow, 1ull);
}

// ------------------------------------------------- exact float sum digits
// (fsum_add's digit split, jit_skeleton.hip): a double is m * 2^(b-1074),
// digits d = b/32 .. d+2 receive the three 32-bit pieces of m << (b % 32).
__device__ __forceinline__ void fsum_pieces(double v, int& d, long long& c0, long long& c1, long long& c2) {
    const u64 b = __builtin_bit_cast(u64, v);
    const int e = (int)((b >> 52) & 0x7ff);
    const u64 m = (b & ((1ull << 52) - 1)) | (e ? (1ull << 52) : 0ull);
    const int pos = (e ? e : 1) - 1;
    d = pos >> 5;
    const int sh = pos & 31;
    const u64 x0 = (m & 0xffffffffull) << sh, x1 = (m >> 32) << sh;
    c0 = (long long)(x0 & 0xffffffffull);
    c1 = (long long)((x0 >> 32) + (x1 & 0xffffffffull));
    c2 = (long long)(x1 >> 32);
    if (b >> 63) {
        c0 = -c0;
        c1 = -c1;
        c2 = -c2;
    }
}

__device__ __forceinline__ void lane_fsum_add(long long* limbs, double v) {
    int d;
    long long c0, c1, c2;
    fsum_pieces(v, d, c0, c1, c2);
    if (c0) atomicAdd((u64*)&limbs[d], (u64)c0);
    if (c1) atomicAdd((u64*)&limbs[d + 1], (u64)c1);
    if (c2) atomicAdd((u64*)&limbs[d + 2], (u64)c2);
}

// The `ok` lanes' values of one group (every lane active): summed across the
// wave when they share a digit (the leader adds three words), else per lane.
__device__ __forceinline__ void gb_fsum_add(long long* limbs, double v, bool ok, int lane, int leader) {
    const u64 vm = __ballot(ok);
    if (!vm) return;
    int d = 0;
    long long c0 = 0, c1 = 0, c2 = 0;
    if (ok) fsum_pieces(v, d, c0, c1, c2);
    const int d0 = __builtin_amdgcn_readlane(d, __builtin_ctzll(vm));
    if (!__ballot(ok && d != d0)) {
        const u64 s0 = wave_sum((u64)c0), s1 = wave_sum((u64)c1), s2 = wave_sum((u64)c2);
        if (lane == leader) {
            if (s0) atomicAdd((u64*)&limbs[d0], s0);
            if (s1) atomicAdd((u64*)&limbs[d0 + 1], s1);
            if (s2) atomicAdd((u64*)&limbs[d0 + 2], s2);
        }
    } else if (ok) {
        if (c0) atomicAdd((u64*)&limbs[d], (u64)c0);
        if (c1) atomicAdd((u64*)&limbs[d + 1], (u64)c1);
        if (c2) atomicAdd((u64*)&limbs[d + 2], (u64)c2);
    }
}

// ------------------------------------------------------- accumulate pass
enum : unsigned { F_NAN = AGGF_NAN, F_PINF = AGGF_PINF, F_NINF = AGGF_NINF, F_NNZ = AGGF_NONNEGZERO };

// One aggregate over the wave's rows of one group (peers P, the leader adds)
// or, with P == 0, each lane with `mine` set adds its own row.
template <typename T>
__device__ __forceinline__ void agg_step(const AggCol& ac, u64* rec, long long i, bool mine, u64 P, int leader,
                                         int lane) {
    const bool act = mine && valid_at(ac.c, i);
    T v = (T)0;
    if constexpr (!__is_same(T, bool)) {
        if (act) v = ((const T*)ac.c.values)[i];
    }
    u64* w = rec + ac.off;
    const int fn = ac.fn;
    if (P) {  // wave-reduced: every lane is active here
        const u64 va = __ballot(act) & P;
        const unsigned cnt = __builtin_popcountll(va);
        // word 0 counts the group's NULL values (non-null count = rows - nulls)
        if (cnt != (unsigned)__builtin_popcountll(P) && lane == leader)
            atomicAdd(&w[0], (u64)(__builtin_popcountll(P) - cnt));
        if constexpr (__is_same(T, bool)) {
            return;
        } else {
            if (fn == DFMI_AGG_COUNT || !cnt) return;
            if (fn == DFMI_AGG_SUM) {
                if constexpr ((T)0.5 != (T)0) {
                    const unsigned f = act ? agg_sum_flags(v) : F_NNZ;
                    const u64 spec = __ballot(act && f != F_NNZ) & P;
                    if (spec) {
                        unsigned fl = 0;
                        if (__ballot(f & F_NAN)) fl |= F_NAN;
                        if (__ballot(f & F_PINF)) fl |= F_PINF;
                        if (__ballot(f & F_NINF)) fl |= F_NINF;
                        if (lane == leader) {
                            atomicAdd(&w[3], (u64)__builtin_popcountll(spec));
                            if (fl) atomicOr(&w[1], (u64)fl);
                        }
                    }
                    const double d = (double)v;
                    const bool ok = act && f == F_NNZ && d != 0.0;
                    gb_fsum_add((long long*)(w + 4), d, ok, lane, leader);
                } else {
                    const u64 x = act ? ((T)-1 < (T)0 ? (u64)(i64)v : (u64)v) : 0ull;
                    const u64 s = wave_sum(x);
                    if (lane == leader && s) atomicAdd(&w[3], s);
                }
                return;
            }
            // MIN / MAX
            const bool is_min = fn == DFMI_AGG_MIN;
            const bool nan = act && agg_isnan(v);
            const u64 nn = __ballot(nan) & P;
            const bool keyed = act && !nan;
            const u64 k = keyed ? agg_key(v) : (is_min ? ~0ull : 0ull);
            const u64 r = is_min ? wave_minmax<true>(k) : wave_minmax<false>(k);
            if (lane == leader) {
                if (nn) atomicAdd(&w[3], (u64)__builtin_popcountll(nn));
                if (__builtin_popcountll(nn) < cnt) {
                    if (is_min) atomicMin(&w[2], r);
                    else atomicMax(&w[2], r);
                }
            }
        }
        return;
    }
    if (!act) {
        if (mine) atomicAdd(&w[0], 1ull);  // a NULL value
        return;
    }
    if constexpr (!__is_same(T, bool)) {
        if (fn == DFMI_AGG_COUNT) return;
        if (fn == DFMI_AGG_SUM) {
            if constexpr ((T)0.5 != (T)0) {
                const unsigned f = agg_sum_flags(v);
                if (f != F_NNZ) {
                    atomicAdd(&w[3], 1ull);
                    if (f) atomicOr(&w[1], (u64)f);
                } else if (v != (T)0) {
                    lane_fsum_add((long long*)(w + 4), (double)v);
                }
            } else {
                const u64 x = (T)-1 < (T)0 ? (u64)(i64)v : (u64)v;
                if (x) atomicAdd(&w[3], x);
            }
            return;
        }
        if (agg_isnan(v)) {
            atomicAdd(&w[3], 1ull);
        } else if (fn == DFMI_AGG_MIN) {
            atomicMin(&w[2], agg_key(v));
        } else {
            atomicMax(&w[2], agg_key(v));
        }
    }
}

// Aggregate j of one row (or the peers' rows) by its argument's type.
__device__ __forceinline__ void agg_dispatch(const AggCol& ac, u64* rec, long long i, bool mine, u64 P, int leader,
                                             int lane) {
    switch (ac.c.type) {
        case 2: return agg_step<i8>(ac, rec, i, mine, P, leader, lane);
        case 3: return agg_step<i16>(ac, rec, i, mine, P, leader, lane);
        case 4: return agg_step<i32>(ac, rec, i, mine, P, leader, lane);
        case 5: return agg_step<i64>(ac, rec, i, mine, P, leader, lane);
        case 6: return agg_step<u8>(ac, rec, i, mine, P, leader, lane);
        case 7: return agg_step<u16>(ac, rec, i, mine, P, leader, lane);
        case 8: return agg_step<u32>(ac, rec, i, mine, P, leader, lane);
        case 9: return agg_step<u64>(ac, rec, i, mine, P, leader, lane);
        case 10: return agg_step<float>(ac, rec, i, mine, P, leader, lane);
        case 11: return agg_step<double>(ac, rec, i, mine, P, leader, lane);
        default: return agg_step<bool>(ac, rec, i, mine, P, leader, lane);  // COUNT of Boolean / Utf8
    }
}

// Row i's group: its slot's group id when the slot holds the row's key -- the
// representative row of this batch (a slot claimed by this launch's claim
// pass; that row persists its Utf8 key bytes here) or the key persisted by an
// earlier batch; a row whose key differs (two keys, one hash) is listed for
// the host merge. False: not added on the device.
template <int NK>
__device__ __forceinline__ bool row_group(const Col* k, long long m, uint32_t epoch, const Table& t, unsigned char* arena,
                                          unsigned long long arena_cap, Hdr* hdr, int32_t* coll_rows, const int32_t* sidx,
                                          long long i, unsigned& g) {
    const int s = sidx[i];
    if (s < 0) return false;
    RowKey r;
    (void)row_key<NK, false>(k, i, m, r);
    const Slot sr = t.slot[s];
    const long long rp = sr.rep;
    const bool cur = (unsigned)((unsigned long long)rp >> 32) == epoch;
    const long long rr = (long long)(unsigned)rp;
    bool same = (sr.knull & kNullBits) == r.nullm;
    if (cur && rr == i) {  // the representative row: persist its Utf8 key bytes
#pragma unroll
        for (int p = 0; p < NK; ++p)
            if (r.s[p]) {
                u8* dst = arena + sr.kw[p];
                for (unsigned j = 0; j < r.len[p]; ++j) dst[j] = r.s[p][j];
            }
    } else {
#pragma unroll
        for (int p = 0; p < NK; ++p) {
            if (!same || ((r.nullm >> p) & 1)) continue;
            const u64 kwv = sr.kw[p];
            if (r.s[p]) {
                const unsigned kl = sr.klen[p];
                if (NK < kMaxKeys && (sr.knull & kInline)) {
                    same = kl == r.len[p] && inline_eq(r.s[p], kl, &sr.kw[NK], r.end[p]);
                    continue;
                }
                const u8* other = cur ? (const u8*)k[p].values + k[p].offsets[rr] : arena + kwv;
                same = kl == r.len[p] && bytes_eq(r.s[p], other, kl, r.end[p], cur ? r.end[p] : arena + arena_cap);
            } else {
                same = kwv == r.w[p];
            }
        }
    }
    if (same) {
        g = sr.gid;
        return true;
    }
    const u64 at = atomicAdd(&hdr->collided, 1ull);  // two keys, one hash: the host merges this row
    coll_rows[at] = (int)i;
    return false;
}

// One wave per 64 consecutive rows. A row whose slot holds its key adds into
// the group's record; rows of one group within the wave are first reduced
// across the wave (the group's leader lane adds once per word) as long as the
// wave finds groups of several rows -- after the second single-row group the
// remaining rows add their own values (many distinct keys: no reduction pays).
template <int NK>
__global__ __launch_bounds__(256) void k_group_accumulate(const AccArgs A) {
    const int lane = threadIdx.x & 63;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long base = (long long)blockIdx.x * blockDim.x + (threadIdx.x & ~63); base < A.m; base += stride) {
        const long long i = base + lane;
        unsigned g = 0;
        const bool ok = i < A.m && row_group<NK>(A.k, A.m, A.epoch, A.t, A.arena, A.arena_cap, A.hdr, A.coll_rows, A.sidx, i, g);
        u64 active = __ballot(ok);
        int singles = 0;
        while (active) {
            const int l = __builtin_ctzll(active);
            const unsigned gl = (unsigned)__builtin_amdgcn_readlane((int)g, l);
            const u64 P = __ballot(ok && ((active >> lane) & 1) && g == gl);
            if (__builtin_popcountll(P) == 1 && ++singles > 2) break;
            u64* rec = A.acc + (u64)gl * (u64)A.words;
            if (lane == l) atomicAdd(&rec[0], (u64)__builtin_popcountll(P));
            const bool mine = (P >> lane) & 1;
            for (int j = 0; j < A.naggs; ++j) agg_dispatch(A.a[j], rec, i, mine, P, l, lane);
            active &= ~P;
        }
        if ((active >> lane) & 1) {
            u64* rec = A.acc + (u64)g * (u64)A.words;
            atomicAdd(&rec[0], 1ull);
            for (int j = 0; j < A.naggs; ++j) agg_dispatch(A.a[j], rec, i, true, 0, 0, lane);
        }
    }
}

// --------------------------------------------------- bucketed accumulation
// (groupby.h "Bucketed accumulation"). The rank and scatter passes run
// kBucketBlocks blocks of 256 threads over the same tiles of kScatterTile rows
// per block, so a block's rows of a bucket fill exactly its positions.
// rows per thread per sub-tile (independent load chains): 4, or 2 with several key
// parts (their keys and slot words in registers: 147 VGPRs, 3 waves / SIMD, at 4)
template <int NK>
constexpr int rank_u() { return NK >= 2 ? 2 : 4; }
constexpr int kScatterTile = 4096;          // rows per block per tile (rank and scatter alike)

template <int NK>
__global__ __launch_bounds__(256) void k_group_rank(const RankArgs A) {
    constexpr int kRankU = rank_u<NK>();
    __shared__ unsigned cnt[kBucketMax];
    for (int b = threadIdx.x; b < A.nbuckets; b += blockDim.x) cnt[b] = 0;
    __syncthreads();
    const Table& t = A.t;
    for (long long T0 = (long long)blockIdx.x * kScatterTile; T0 < A.m; T0 += (long long)gridDim.x * kScatterTile)
    for (long long t0 = T0; t0 < T0 + kScatterTile && t0 < A.m; t0 += 256 * kRankU) {
        // the row_group chain of kRankU rows at once: slots, keys, the slots' words, then the decisions
        int sl[kRankU];
        RowKey r[kRankU];
        Slot sr[kRankU];
#pragma unroll
        for (int u = 0; u < kRankU; ++u) {
            const long long i = t0 + threadIdx.x + 256 * u;
            sl[u] = i < A.m ? A.sidx[i] : -1;
        }
#pragma unroll
        for (int u = 0; u < kRankU; ++u) {
            const long long i = t0 + threadIdx.x + 256 * u;
            const int s = sl[u] < 0 ? 0 : sl[u];
            if (sl[u] >= 0) (void)row_key<NK, false>(A.k, i, A.m, r[u]);
            sr[u] = t.slot[s];
        }
#pragma unroll
        for (int u = 0; u < kRankU; ++u) {
            const long long i = t0 + threadIdx.x + 256 * u;
            if (i >= A.m) break;
            const int s = sl[u];
            bool ok = false;
            if (s >= 0) {
                const bool cur = (unsigned)((unsigned long long)sr[u].rep >> 32) == A.epoch;
                const long long rr = (long long)(unsigned)sr[u].rep;
                bool same = (sr[u].knull & kNullBits) == r[u].nullm;
                if (cur && rr == i) {  // the representative row: persist its Utf8 key bytes
#pragma unroll
                    for (int p = 0; p < NK; ++p)
                        if (r[u].s[p]) {
                            u8* dst = A.arena + sr[u].kw[p];
                            for (unsigned j = 0; j < r[u].len[p]; ++j) dst[j] = r[u].s[p][j];
                        }
                } else {
#pragma unroll
                    for (int p = 0; p < NK; ++p) {
                        if (!same || ((r[u].nullm >> p) & 1)) continue;
                        if (r[u].s[p]) {
                            const unsigned kl = sr[u].klen[p];
                            if (NK < kMaxKeys && (sr[u].knull & kInline)) {
                                same = kl == r[u].len[p] && inline_eq(r[u].s[p], kl, &sr[u].kw[NK], r[u].end[p]);
                                continue;
                            }
                            const u8* other = cur ? (const u8*)A.k[p].values + A.k[p].offsets[rr] : A.arena + sr[u].kw[p];
                            same = kl == r[u].len[p] &&
                                   bytes_eq(r[u].s[p], other, kl, r[u].end[p], cur ? r[u].end[p] : A.arena + A.arena_cap);
                        } else {
                            same = sr[u].kw[p] == r[u].w[p];
                        }
                    }
                }
                if (same) {
                    ok = true;
                } else {  // two keys, one hash: the host merges this row
                    const u64 at = atomicAdd(&A.hdr->collided, 1ull);
                    A.coll_rows[at] = (int)i;
                }
            }
            A.rg[i] = ok ? sr[u].gid : ~0u;
            if (ok) atomicAdd(&cnt[sr[u].gid >> A.gshift], 1u);
        }
    }
    __syncthreads();
    for (int b = threadIdx.x; b < A.nbuckets; b += blockDim.x) A.bh[b * kBucketBlocks + blockIdx.x] = cnt[b];
}

// k_group_rank for keys without Utf8 parts: no representative row to consult
// (the claim persisted every fixed-width key word), so each row reads only its
// slot's group id, null mask and key words, kRankFixedU rows at once.
constexpr int kRankFixedU = 8;

template <int NK>
__global__ __launch_bounds__(256) void k_group_rank_fixed(const RankArgs A) {
    __shared__ unsigned cnt[kBucketMax];
    for (int b = threadIdx.x; b < A.nbuckets; b += blockDim.x) cnt[b] = 0;
    __syncthreads();
    const Slot* slot = A.t.slot;
    constexpr int rows = 256 * kRankFixedU;
    static_assert(kScatterTile % rows == 0, "sub-tiles of the scatter's tile");
    for (long long T0 = (long long)blockIdx.x * kScatterTile; T0 < A.m; T0 += (long long)gridDim.x * kScatterTile)
    for (long long t0 = T0; t0 < T0 + kScatterTile && t0 < A.m; t0 += rows) {
        int sl[kRankFixedU];
        unsigned gid[kRankFixedU], kn[kRankFixedU];
        u64 kw[kRankFixedU][NK];
#pragma unroll
        for (int u = 0; u < kRankFixedU; ++u) {
            const long long i = t0 + threadIdx.x + 256 * u;
            sl[u] = i < A.m ? A.sidx[i] : -1;
        }
#pragma unroll
        for (int u = 0; u < kRankFixedU; ++u) {
            const Slot& q = slot[sl[u] < 0 ? 0 : sl[u]];
            gid[u] = q.gid;
            kn[u] = q.knull & kNullBits;
#pragma unroll
            for (int p = 0; p < NK; ++p) kw[u][p] = q.kw[p];
        }
#pragma unroll
        for (int u = 0; u < kRankFixedU; ++u) {
            const long long i = t0 + threadIdx.x + 256 * u;
            if (i >= A.m) break;
            bool ok = false;
            if (sl[u] >= 0) {
                unsigned nullm = 0;
                bool same = true;
#pragma unroll
                for (int p = 0; p < NK; ++p) {
                    if (!valid_at(A.k[p], i)) nullm |= 1u << p;
                    else same = same && kw[u][p] == key_bits(A.k[p], i);
                }
                same = same && nullm == kn[u];
                if (same) {
                    ok = true;
                } else {  // two keys, one hash: the host merges this row
                    const u64 at = atomicAdd(&A.hdr->collided, 1ull);
                    A.coll_rows[at] = (int)i;
                }
            }
            A.rg[i] = ok ? gid[u] : ~0u;
            if (ok) atomicAdd(&cnt[gid[u] >> A.gshift], 1u);
        }
    }
    __syncthreads();
    for (int b = threadIdx.x; b < A.nbuckets; b += blockDim.x) A.bh[b * kBucketBlocks + blockIdx.x] = cnt[b];
}

// One block of kBucketBlocks threads per bucket: its per-block counts turned
// into exclusive prefixes in place, the bucket's total into tot[b].
__global__ __launch_bounds__(kBucketBlocks) void k_group_scan(unsigned* bh, unsigned* tot) {
    __shared__ unsigned wsum[kBucketBlocks / 64];
    unsigned* c = bh + (u64)blockIdx.x * kBucketBlocks;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const unsigned v = c[t];
    const unsigned incl = (unsigned)wave_incl_scan((u64)v, lane);
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    unsigned before = 0, all = 0;
    for (int q = 0; q < kBucketBlocks / 64; ++q) {
        if (q < w) before += wsum[q];
        all += wsum[q];
    }
    c[t] = before + incl - v;
    if (t == 0) tot[blockIdx.x] = all;
}

// The first position of every bucket (exclusive prefix of the totals) into
// LDS, start[nb] the placed rows (256 threads, kBucketMax / 256 buckets each).
__device__ __forceinline__ void bucket_starts(const unsigned* tot, int nb, unsigned* start) {
    constexpr int P = kBucketMax / 256;
    __shared__ unsigned wtot[4];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    unsigned v[P], sum = 0;
#pragma unroll
    for (int k = 0; k < P; ++k) {
        v[k] = t * P + k < nb ? tot[t * P + k] : 0u;
        sum += v[k];
    }
    const unsigned incl = wave_incl_scan32(sum, lane);
    if (lane == 63) wtot[w] = incl;
    __syncthreads();
    unsigned run = incl - sum, all = 0;
    for (int q = 0; q < 4; ++q) {
        if (q < w) run += wtot[q];
        all += wtot[q];
    }
#pragma unroll
    for (int k = 0; k < P; ++k) {
        if (t * P + k < nb) start[t * P + k] = run;
        run += v[k];
    }
    if (t == 0) start[nb] = all;
    __syncthreads();
}

// a[0 .. nb) -> its exclusive prefix in place, a[nb] the total (LDS; 256
// threads, kBucketMax / 256 entries each).
__device__ __forceinline__ void lds_excl_scan(unsigned* a, int nb) {
    constexpr int P = kBucketMax / 256;
    __shared__ unsigned wtot[4];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    unsigned v[P], sum = 0;
#pragma unroll
    for (int k = 0; k < P; ++k) {
        v[k] = t * P + k < nb ? a[t * P + k] : 0u;
        sum += v[k];
    }
    const unsigned incl = wave_incl_scan32(sum, lane);
    if (lane == 63) wtot[w] = incl;
    __syncthreads();
    unsigned run = incl - sum, all = 0;
    for (int q = 0; q < 4; ++q) {
        if (q < w) run += wtot[q];
        all += wtot[q];
    }
#pragma unroll
    for (int k = 0; k < P; ++k) {
        if (t * P + k < nb) a[t * P + k] = run;
        run += v[k];
    }
    if (t == 0) a[nb] = all;
    __syncthreads();
}

// Per tile, the placed rows are first ordered by bucket in LDS, then written
// out: consecutive lanes write consecutive positions of a bucket's run (whole
// lines), where a per-row store would leave each of the ~buckets x resident
// blocks open lines half written in L2.
__global__ __launch_bounds__(256) void k_group_scatter(const ScatterArgs A) {
    constexpr int PER = kScatterTile / 256;
    __shared__ unsigned cur[kBucketMax + 1];    // the block's next position per bucket
    __shared__ unsigned tcnt[kBucketMax + 1];   // the tile's rows per bucket, then their exclusive prefix
    __shared__ unsigned sg[kScatterTile];       // the tile's placed rows in bucket order: group id ...
    __shared__ unsigned short si[kScatterTile]; // ... and row within the tile
    bucket_starts(A.tot, A.nbuckets, cur);
    for (int b = threadIdx.x; b < A.nbuckets; b += blockDim.x) cur[b] += A.base[b * kBucketBlocks + blockIdx.x];
    for (int b = threadIdx.x; b <= A.nbuckets; b += blockDim.x) tcnt[b] = 0;
    __syncthreads();
    for (long long T0 = (long long)blockIdx.x * kScatterTile; T0 < A.m; T0 += (long long)gridDim.x * kScatterTile) {
        unsigned g[PER], r[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const long long i = T0 + threadIdx.x + 256 * u;
            g[u] = i < A.m ? A.rg[i] : ~0u;
            r[u] = g[u] != ~0u ? atomicAdd(&tcnt[g[u] >> A.gshift], 1u) : 0u;
        }
        __syncthreads();
        lds_excl_scan(tcnt, A.nbuckets);
#pragma unroll
        for (int u = 0; u < PER; ++u)
            if (g[u] != ~0u) {
                const unsigned sp = tcnt[g[u] >> A.gshift] + r[u];
                sg[sp] = g[u];
                si[sp] = (unsigned short)(threadIdx.x + 256 * u);
            }
        __syncthreads();
        const unsigned placed = tcnt[A.nbuckets];
        // four staged rows per thread per round: their argument loads issued before any store
        for (unsigned e0 = threadIdx.x; e0 < placed; e0 += 4 * blockDim.x) {
            unsigned gg[4], pos[4];
            long long i[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const unsigned e = e0 + u * blockDim.x;
                const bool in = e < placed;
                gg[u] = in ? sg[e] : 0u;
                const unsigned b = gg[u] >> A.gshift;
                pos[u] = in ? cur[b] + (e - tcnt[b]) : ~0u;
                i[u] = T0 + (in ? si[e] : 0);
            }
            if (A.pn) {
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    unsigned nm = 0;
                    for (int j = 0; j < A.naggs; ++j)
                        if (!valid_at(A.arg[j], i[u])) nm |= 1u << j;
                    if (pos[u] != ~0u) A.pn[pos[u]] = nm;
                }
            }
            for (int c = 0; c < A.npay; ++c) {
                u64 x[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) x[u] = pos[u] != ~0u ? key_bits(A.pay[c], i[u]) : 0ull;
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (pos[u] != ~0u) A.pv[(u64)c * (u64)A.m + pos[u]] = x[u];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (pos[u] != ~0u) A.pg[pos[u]] = gg[u];
        }
        __syncthreads();
        for (int b = threadIdx.x; b < A.nbuckets; b += blockDim.x) cur[b] += tcnt[b + 1] - tcnt[b];
        __syncthreads();
        for (int b = threadIdx.x; b <= A.nbuckets; b += blockDim.x) tcnt[b] = 0;
        __syncthreads();
    }
}

// agg_step's per-lane rules on an LDS record (ds atomics).
__device__ __forceinline__ void lds_fsum_add(u64* limbs, double v) {
    int d;
    long long c0, c1, c2;
    fsum_pieces(v, d, c0, c1, c2);
    if (c0) atomicAdd(&limbs[d], (u64)c0);
    if (c1) atomicAdd(&limbs[d + 1], (u64)c1);
    if (c2) atomicAdd(&limbs[d + 2], (u64)c2);
}

template <typename T>
__device__ __forceinline__ void lds_agg_step(const AggCol& ac, u64* rec, bool null, u64 bits) {
    u64* w = rec + ac.off;
    if (null) {
        atomicAdd(&w[0], 1ull);  // a NULL value
        return;
    }
    if constexpr (!__is_same(T, bool)) {
        const int fn = ac.fn;
        if (fn == DFMI_AGG_COUNT) return;
        T v;
        if constexpr (__is_same(T, float)) v = __builtin_bit_cast(float, (unsigned)bits);
        else if constexpr (__is_same(T, double)) v = __builtin_bit_cast(double, bits);
        else v = (T)bits;  // (integers sign- or zero-extended by key_bits)
        if (fn == DFMI_AGG_SUM) {
            if constexpr ((T)0.5 != (T)0) {
                const unsigned f = agg_sum_flags(v);
                if (f != F_NNZ) {
                    atomicAdd(&w[3], 1ull);
                    if (f) atomicOr(&w[1], (u64)f);
                } else if (v != (T)0) {
                    lds_fsum_add(w + 4, (double)v);
                }
            } else {
                const u64 x = (T)-1 < (T)0 ? (u64)(i64)v : (u64)v;
                if (x) atomicAdd(&w[3], x);
            }
            return;
        }
        if (agg_isnan(v)) {
            atomicAdd(&w[3], 1ull);
        } else if (fn == DFMI_AGG_MIN) {
            atomicMin(&w[2], agg_key(v));
        } else {
            atomicMax(&w[2], agg_key(v));
        }
    }
}

__device__ __forceinline__ void lds_agg_dispatch(const AggCol& ac, u64* rec, bool null, u64 bits) {
    switch (ac.c.type) {
        case 2: return lds_agg_step<i8>(ac, rec, null, bits);
        case 3: return lds_agg_step<i16>(ac, rec, null, bits);
        case 4: return lds_agg_step<i32>(ac, rec, null, bits);
        case 5: return lds_agg_step<i64>(ac, rec, null, bits);
        case 6: return lds_agg_step<u8>(ac, rec, null, bits);
        case 7: return lds_agg_step<u16>(ac, rec, null, bits);
        case 8: return lds_agg_step<u32>(ac, rec, null, bits);
        case 9: return lds_agg_step<u64>(ac, rec, null, bits);
        case 10: return lds_agg_step<float>(ac, rec, null, bits);
        case 11: return lds_agg_step<double>(ac, rec, null, bits);
        default: return lds_agg_step<bool>(ac, rec, null, bits);
    }
}

// One block per (bucket, split): the bucket's gpb records in LDS (the zero
// state), the split's share of the bucket's rows added, then every record word
// that moved added into the global record (rows / NULLs / sums / digits:
// add; flags: or; MIN / MAX keys: min / max) -- lanes over consecutive words.
__global__ __launch_bounds__(256) void k_group_bucket(const BucketArgs A) {
    extern __shared__ u64 lrec[];
    __shared__ unsigned start[kBucketMax + 1];
    bucket_starts(A.tot, A.nbuckets, start);
    const int b = blockIdx.x / A.splits, sp = blockIdx.x % A.splits;
    const u64 g0 = (u64)b * A.gpb;
    const u64 left = A.ngroups - g0;
    const unsigned nb = (unsigned)(left < (u64)A.gpb ? left : (u64)A.gpb);
    const int W = A.words;
    // (copies of a small bucket's records, the lanes spread over them, measured no
    // faster at 4 and 16 groups: 1.23 ms per 1e8 rows either way -- one copy)
    for (unsigned x = threadIdx.x; x < nb * (unsigned)W; x += blockDim.x) lrec[x] = A.pattern[x % (unsigned)W];
    __syncthreads();
    const unsigned r0 = start[b], len = start[b + 1] - start[b];
    const unsigned q0 = r0 + (unsigned)((u64)len * (u64)sp / (u64)A.splits);
    const unsigned q1 = r0 + (unsigned)((u64)len * (u64)(sp + 1) / (u64)A.splits);
    // kBucketU rows per thread per round: their loads issued together (the
    // streamed group ids and argument words are the pass's only global reads)
    constexpr unsigned kBucketU = 4;
    for (unsigned base = q0 + threadIdx.x; base < q1; base += kBucketU * blockDim.x) {
        unsigned lg[kBucketU], nm[kBucketU];
#pragma unroll
        for (unsigned u = 0; u < kBucketU; ++u) {
            const unsigned pos = base + u * blockDim.x;
            lg[u] = pos < q1 ? A.pg[pos] - (unsigned)g0 : ~0u;
            nm[u] = pos < q1 && A.pn ? A.pn[pos] : 0u;
        }
#pragma unroll
        for (unsigned u = 0; u < kBucketU; ++u)
            if (lg[u] != ~0u) atomicAdd(&lrec[(u64)lg[u] * (u64)W], 1ull);
        for (int j = 0; j < A.naggs; ++j) {
            u64 bits[kBucketU];
#pragma unroll
            for (unsigned u = 0; u < kBucketU; ++u) {
                const unsigned pos = base + u * blockDim.x;
                bits[u] = A.pcol[j] >= 0 && pos < q1 ? A.pv[(u64)A.pcol[j] * (u64)A.m + pos] : 0ull;
            }
#pragma unroll
            for (unsigned u = 0; u < kBucketU; ++u)
                if (lg[u] != ~0u) lds_agg_dispatch(A.a[j], lrec + (u64)lg[u] * (u64)W, (nm[u] >> j) & 1, bits[u]);
        }
    }
    __syncthreads();
    for (unsigned x = threadIdx.x; x < nb * (unsigned)W; x += blockDim.x) {
        const int w = (int)(x % (unsigned)W);
        int j = -1;  // the aggregate owning word w (w = 0: the group's rows)
        for (int q = 0; q < A.naggs; ++q)
            if (A.a[q].off <= w) j = q;
        const int r = j < 0 ? -1 : w - A.a[j].off;
        const int op = r == 1 ? 1 : (r == 2 && A.a[j].fn == DFMI_AGG_MIN) ? 2 : (r == 2 && A.a[j].fn == DFMI_AGG_MAX) ? 3 : 0;
        const u64 v = lrec[x];
        if (v == A.pattern[w]) continue;
        u64* dst = A.acc + (g0 + x / (unsigned)W) * (u64)W + (u64)w;
        if (op == 1) atomicOr(dst, v);
        else if (op == 2) atomicMin(dst, v);
        else if (op == 3) atomicMax(dst, v);
        else atomicAdd(dst, v);
    }
}

// ------------------------------------------------------------ maintenance
// Every used slot of `o` into the (larger, empty) table `n`: same hash word,
// same group id, representative and persisted key.
__global__ __launch_bounds__(256) void k_group_rehash(const Table o, const Table n) {
    const u64 cap = o.mask + 1;
    for (u64 s = (u64)blockIdx.x * blockDim.x + threadIdx.x; s < cap; s += (u64)gridDim.x * blockDim.x) {
        const u64 c = o.ctl[s];
        if (!c) continue;
        u64 q = gmix(c) & n.mask;
        while (atomicCAS(&n.ctl[q], 0ull, c) != 0ull) q = (q + 1) & n.mask;
        n.slot[q] = o.slot[s];
    }
}

// The persisted key of every used slot, by group id (the host's drain reads
// ngroups-sized arrays instead of the whole table).
__global__ __launch_bounds__(256) void k_group_compact(const Table t, int nkeys, unsigned* knull, u64* kw,
                                                       unsigned* klen) {
    const u64 cap = t.mask + 1;
    for (u64 s = (u64)blockIdx.x * blockDim.x + threadIdx.x; s < cap; s += (u64)gridDim.x * blockDim.x) {
        if (!t.ctl[s]) continue;
        const Slot sr = t.slot[s];
        const u64 g = sr.gid;
        knull[g] = sr.knull & kNullBits;
        for (int p = 0; p < nkeys; ++p) {
            kw[g * nkeys + p] = sr.kw[p];
            klen[g * nkeys + p] = sr.klen[p];
        }
    }
}

// Records [g0, g1) set to the zero state (`pattern`: one record).
__global__ __launch_bounds__(256) void k_group_init(u64* acc, const u64* pattern, int words, u64 g0, u64 g1) {
    const u64 w0 = g0 * (u64)words, w1 = g1 * (u64)words;
    for (u64 w = w0 + (u64)blockIdx.x * blockDim.x + threadIdx.x; w < w1; w += (u64)gridDim.x * blockDim.x)
        acc[w] = pattern[(w - w0) % (u64)words];
}

// Carry-normalise every group's exact-sum digits (each digit but the top one
// back in [0, 2^32)), so the digits absorb another 2^31 rows.
struct NormArgs {
    u64* acc;
    int words;
    int nf;
    int foff[kMaxAggs];  // word offsets of the float SUM digits in a record
    u64 ngroups;
};

__global__ __launch_bounds__(256) void k_group_normalize(const NormArgs A) {
    const u64 n = A.ngroups * (u64)A.nf;
    for (u64 x = (u64)blockIdx.x * blockDim.x + threadIdx.x; x < n; x += (u64)gridDim.x * blockDim.x) {
        long long* L = (long long*)(A.acc + (x / A.nf) * (u64)A.words + A.foff[x % A.nf]);
        for (int i = 0; i < kAggLimbs - 1; ++i) {
            const long long c = L[i] >> 32;  // floor division by 2^32
            L[i] -= c * 4294967296ll;
            L[i + 1] += c;
        }
    }
}

// ------------------------------------------------------------ device finish
// One exact sum (kAggLimbs int64 digits in units of 2^-1074, not necessarily
// carry-normalised) rounded half to even to `prec` significand bits with a
// quantum of at least 2^(qmin-1074): aggregate.cpp normalize + round_exact,
// step for step. The thread's digits 0 .. kAggLimbs-2 live in LDS (`d`, with a
// stride of kRoundBlock words: consecutive threads, consecutive banks), the top
// (sign) digit in a register.
constexpr int kRoundBlock = 128;

__device__ double round_digits(const u64* L, unsigned* d, int prec, int qmin, double overflow_limit, bool& zero) {
    constexpr int K = kAggLimbs;
    long long c = 0;
    for (int i = 0; i < K - 1; ++i) {  // carry-normalise: digits in [0, 2^32), floor carries upward
        const long long v = (long long)L[i] + c;
        c = v >> 32;
        d[i * kRoundBlock] = (unsigned)v;
    }
    long long t = (long long)L[K - 1] + c;
    const bool neg = t < 0;
    if (neg) {  // the magnitude: two's complement negation of the digit string
        long long borrow = 0;
        for (int i = 0; i < K - 1; ++i) {
            long long v = -(long long)d[i * kRoundBlock] - borrow;
            borrow = 0;
            if (v < 0) {
                v += 4294967296ll;
                borrow = 1;
            }
            d[i * kRoundBlock] = (unsigned)v;
        }
        t = -t - borrow;
    }
    auto D = [&](int i) -> u64 { return i == K - 1 ? (u64)t : (u64)d[i * kRoundBlock]; };
    int top = -1;
    if (t) top = K - 1;
    else
        for (int i = K - 2; i >= 0; --i)
            if (d[i * kRoundBlock]) {
                top = i;
                break;
            }
    zero = top < 0;
    if (top < 0) return 0.0;
    const unsigned lo = (unsigned)D(top);
    const int msb = 32 * top + (lo ? 31 - __builtin_clz(lo) : 0);
    int q = msb - (prec - 1) > qmin ? msb - (prec - 1) : qmin;
    u64 mant = 0;  // bits [q, msb] from the top three digits
    if (q <= msb) {
        const int b0 = top - 2 > 0 ? top - 2 : 0;
        unsigned __int128 w = 0;
        for (int i = top; i >= b0; --i) w = (w << 32) | (unsigned __int128)D(i);
        mant = (u64)(w >> (q - 32 * b0)) & ((1ull << (msb - q + 1)) - 1);
    }
    auto bit = [&](int i) -> u64 { return i < 0 ? 0 : (D(i >> 5) >> (i & 31)) & 1; };
    const u64 rb = q >= 1 ? bit(q - 1) : 0;
    bool sticky = false;  // any set bit in [0, q - 2]
    if (q >= 2) {
        const int hb = q - 2, hd = hb >> 5;
        for (int i = 0; i < hd && !sticky; ++i) sticky = D(i) != 0;
        const u64 m = (hb & 31) == 31 ? 0xffffffffull : ((1ull << ((hb & 31) + 1)) - 1);
        sticky = sticky || (D(hd) & m) != 0;
    }
    if (rb && (sticky || (mant & 1))) {
        ++mant;
        if (mant >> prec) {
            mant >>= 1;
            ++q;
        }
    }
    double v = ldexp((double)mant, q - 1074);
    if (v >= overflow_limit) v = __builtin_inf();
    return neg ? -v : v;
}

__global__ __launch_bounds__(kRoundBlock) void k_group_round(const RoundArgs A) {
    __shared__ unsigned dg[(kAggLimbs - 1) * kRoundBlock];
    const u64 n = A.ngroups * (u64)A.naggs;
    const int cw = 1 + 4 * A.naggs;
    for (u64 x = (u64)blockIdx.x * kRoundBlock + threadIdx.x; x < n; x += (u64)gridDim.x * kRoundBlock) {
        const u64 g = x / (u64)A.naggs;
        const int j = (int)(x % (u64)A.naggs);
        const u64* rec = A.acc + g * (u64)A.words;
        u64* o = A.out + g * (u64)cw;
        if (j == 0) o[0] = rec[0];
        const u64* w = rec + A.off[j];
        u64* ow = o + 1 + 4 * j;
        u64 flags = w[1], key = w[2];
        if (A.kind[j]) {
            bool zero = false;
            const double v = A.kind[j] == 2 ? round_digits(w + 4, dg + threadIdx.x, 24, 925, 0x1p128, zero)
                                            : round_digits(w + 4, dg + threadIdx.x, 53, 0, __builtin_inf(), zero);
            key = __builtin_bit_cast(u64, v);
            if (zero) flags |= kRoundZero;
        }
        ow[0] = w[0];
        ow[1] = flags;
        ow[2] = key;
        ow[3] = w[3];
    }
}

// ------------------------------------------------------- device emission
__device__ __forceinline__ u64 sort_value(int t, u64 bits) {  // key_ord as an unsigned 64-bit order
    switch (t) {
        case 11: return (bits >> 63) ? ~bits : (bits | (1ull << 63));  // Float64: totalOrder
        case 10: {
            const unsigned b = (unsigned)bits;
            return (u64)((b >> 31) ? ~b : (b | 0x80000000u));
        }
        case 2: case 3: case 4: case 5: return bits ^ (1ull << 63);  // signed: sign-extended bits
        default: return bits;  // unsigned, Boolean
    }
}

__global__ __launch_bounds__(256) void k_group_sortkey(int kt, u64 ng, const unsigned* knull, const u64* kw, u64* sk,
                                                       unsigned* sv, unsigned* null_at) {
    for (u64 g = (u64)blockIdx.x * blockDim.x + threadIdx.x; g < ng; g += (u64)gridDim.x * blockDim.x) {
        const bool null = knull[g] & 1;
        sk[g] = null ? ~0ull : sort_value(kt, kw[g]);
        sv[g] = (unsigned)g;
        if (null) null_at[0] = (unsigned)g;
    }
}

__global__ __launch_bounds__(256) void k_group_nullpos(const unsigned* order, u64 ng, unsigned* null_at) {
    const unsigned ngid = null_at[0];
    if (ngid == ~0u) return;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < ng; i += (u64)gridDim.x * blockDim.x)
        if (order[i] == ngid) null_at[1] = (unsigned)i;
}

struct AggValue {  // dfmi_agg_value
    int type;
    int is_null;
    long long count;
    u64 bits;
};

__device__ __forceinline__ u64 narrow_bits(u64 v, int t) {
    switch (t) {
        case 2: return (u64)(i64)(i8)v;
        case 3: return (u64)(i64)(i16)v;
        case 4: return (u64)(i64)(i32)v;
        case 6: return v & 0xffull;
        case 7: return v & 0xffffull;
        case 8: return v & 0xffffffffull;
        default: return v;
    }
}

__device__ __forceinline__ u64 key_value_bits(u64 key, int t) {  // aggregate.cpp key_to_bits
    switch (t) {
        case 11: return (key >> 63) ? (key & ~(1ull << 63)) : ~key;
        case 10: {
            const unsigned k = (unsigned)key;
            return (k >> 31) ? (u64)(k & 0x7fffffffu) : (u64)(unsigned)~k;
        }
        case 2: case 3: case 4: case 5: return key ^ (1ull << 63);
        default: return key;
    }
}

// aggregate.cpp rec_partial + finish_normalized over a compact record.
__device__ __forceinline__ AggValue finish_value(const u64* rec, int off, int fn, int t, int ret) {
    const u64* w = rec + off;
    AggValue r;
    r.type = ret;
    r.is_null = 0;
    r.bits = 0;
    const u64 count = rec[0] - w[0];
    r.count = (long long)count;
    if (fn == DFMI_AGG_COUNT) {
        r.bits = count;
        return r;
    }
    if (count == 0) {
        r.is_null = 1;
        return r;
    }
    const bool f32 = t == 10, flt = t == 10 || t == 11;
    const u64 qnan = f32 ? 0x7FC00000ull : 0x7FF8000000000000ull;
    if (fn == DFMI_AGG_SUM) {
        if (!flt) {
            r.bits = narrow_bits(w[3], t);
            return r;
        }
        const u64 flags = (w[1] & 0xffffffffull) | (count > w[3] ? (u64)AGGF_NONNEGZERO : 0ull);
        if ((flags & AGGF_NAN) || ((flags & AGGF_PINF) && (flags & AGGF_NINF))) {
            r.bits = qnan;
        } else if (flags & (AGGF_PINF | AGGF_NINF)) {
            const bool pos = flags & AGGF_PINF;
            r.bits = f32 ? (pos ? 0x7F800000ull : 0xFF800000ull) : (pos ? 0x7FF0000000000000ull : 0xFFF0000000000000ull);
        } else {
            double v = __builtin_bit_cast(double, w[2]);
            if (w[1] & kRoundZero) v = (flags & AGGF_NONNEGZERO) ? 0.0 : -0.0;
            r.bits = f32 ? (u64)__builtin_bit_cast(unsigned, (float)v) : __builtin_bit_cast(u64, v);
        }
        return r;
    }
    // MIN / MAX
    const bool value = count > w[3];
    r.bits = value ? key_value_bits(w[2], t) : qnan;
    return r;
}

__global__ __launch_bounds__(256) void k_group_emit(const EmitArgs A) {
    const unsigned ngid = A.null_at[0], npos = A.null_at[1];
    const int cw = 1 + 4 * A.naggs;
    AggValue* keys = (AggValue*)A.keys;
    AggValue* vals = (AggValue*)A.values;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < A.ngroups; i += (u64)gridDim.x * blockDim.x) {
        unsigned g;
        if (ngid == ~0u) g = A.order[i];
        else if (i == A.ngroups - 1) g = ngid;  // the null group last
        else g = A.order[i < npos ? i : i + 1];
        const u64* rec = A.rec + (u64)g * (u64)cw;
        AggValue k;
        k.type = A.ktype;
        k.is_null = (A.knull[g] & 1) ? 1 : 0;
        k.count = (long long)rec[0];
        k.bits = k.is_null ? 0ull : (A.ktype == 1 ? A.kw[g] : narrow_bits(A.kw[g], A.ktype));
        keys[i] = k;
        for (int j = 0; j < A.naggs; ++j) vals[i * (u64)A.naggs + j] = finish_value(rec, 1 + 4 * j, A.fn[j], A.atype[j], A.rtype[j]);
    }
}

static int grid_for(long long items, int per_block = 256, int cap = 8192) {
    long long g = (items + per_block - 1) / per_block;
    return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}

hipError_t launch_claim(const ClaimArgs& a, hipStream_t st) {
    const dim3 g(grid_for(a.m)), b(256);
    switch (a.nkeys) {
        case 1: hipLaunchKernelGGL(k_group_claim<1>, g, b, 0, st, a); break;
        case 2: hipLaunchKernelGGL(k_group_claim<2>, g, b, 0, st, a); break;
        case 3: hipLaunchKernelGGL(k_group_claim<3>, g, b, 0, st, a); break;
        case 4: hipLaunchKernelGGL(k_group_claim<4>, g, b, 0, st, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_accumulate(const AccArgs& a, hipStream_t st) {
    const dim3 g(grid_for(a.m)), b(256);
    switch (a.nkeys) {
        case 1: hipLaunchKernelGGL(k_group_accumulate<1>, g, b, 0, st, a); break;
        case 2: hipLaunchKernelGGL(k_group_accumulate<2>, g, b, 0, st, a); break;
        case 3: hipLaunchKernelGGL(k_group_accumulate<3>, g, b, 0, st, a); break;
        case 4: hipLaunchKernelGGL(k_group_accumulate<4>, g, b, 0, st, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_rehash(const Table& o, const Table& n, hipStream_t st) {
    hipLaunchKernelGGL(k_group_rehash, dim3(grid_for((long long)o.mask + 1)), dim3(256), 0, st, o, n);
    return hipGetLastError();
}

hipError_t launch_compact(const Table& t, int nkeys, unsigned* knull, unsigned long long* kw, unsigned* klen,
                          hipStream_t st) {
    hipLaunchKernelGGL(k_group_compact, dim3(grid_for((long long)t.mask + 1)), dim3(256), 0, st, t, nkeys, knull, kw,
                       klen);
    return hipGetLastError();
}

hipError_t launch_init(u64* acc, const u64* pattern, int words, u64 g0, u64 g1, hipStream_t st) {
    if (g1 <= g0) return hipSuccess;
    hipLaunchKernelGGL(k_group_init, dim3(grid_for((long long)((g1 - g0) * words))), dim3(256), 0, st, acc, pattern,
                       words, g0, g1);
    return hipGetLastError();
}

hipError_t launch_buckets(const RankArgs& r, ScatterArgs s, BucketArgs b, hipStream_t st) {
    const dim3 g(kBucketBlocks), blk(256);
    if (r.nbuckets > kBucketMax || b.gpb != (1u << r.gshift)) return hipErrorInvalidValue;
    bool fixed = true;
    for (int p = 0; p < r.nkeys && p < kMaxKeys; ++p) fixed = fixed && r.k[p].type != kTypeUtf8;
    switch (r.nkeys * 2 + (fixed ? 1 : 0)) {
        case 2: hipLaunchKernelGGL(k_group_rank<1>, g, blk, 0, st, r); break;
        case 3: hipLaunchKernelGGL(k_group_rank_fixed<1>, g, blk, 0, st, r); break;
        case 4: hipLaunchKernelGGL(k_group_rank<2>, g, blk, 0, st, r); break;
        case 5: hipLaunchKernelGGL(k_group_rank_fixed<2>, g, blk, 0, st, r); break;
        case 6: hipLaunchKernelGGL(k_group_rank<3>, g, blk, 0, st, r); break;
        case 7: hipLaunchKernelGGL(k_group_rank_fixed<3>, g, blk, 0, st, r); break;
        case 8: hipLaunchKernelGGL(k_group_rank<4>, g, blk, 0, st, r); break;
        case 9: hipLaunchKernelGGL(k_group_rank_fixed<4>, g, blk, 0, st, r); break;
        default: return hipErrorInvalidValue;
    }
    hipLaunchKernelGGL(k_group_scan, dim3(r.nbuckets), dim3(kBucketBlocks), 0, st, r.bh, (unsigned*)s.tot);
    hipLaunchKernelGGL(k_group_scatter, g, blk, 0, st, s);
    const size_t lds = (size_t)b.gpb * (size_t)b.words * 8;
    if (lds > (size_t)kBucketRecordLdsBig || b.nbuckets > kBucketMax || b.splits < 1) return hipErrorInvalidValue;
    if (lds > (size_t)kBucketRecordLds) {  // more than 64 KiB per workgroup: raise the kernel's limit (once)
        static const hipError_t raised = hipFuncSetAttribute((const void*)k_group_bucket,
                                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                                             kBucketRecordLdsBig);
        if (raised != hipSuccess) return raised;
    }
    hipLaunchKernelGGL(k_group_bucket, dim3(b.nbuckets * b.splits), blk, lds, st, b);
    return hipGetLastError();
}

hipError_t launch_emit(EmitArgs a, u64* sk, u64* sk2, unsigned* sv, unsigned* sv2, unsigned* null_at, void* tmp,
                       size_t* tmp_bytes, hipStream_t st) {
    if (!tmp) return rocprim::radix_sort_pairs(nullptr, *tmp_bytes, sk, sk2, sv, sv2, a.ngroups, 0, 64, st);
    const u64 ng = a.ngroups;
    hipError_t e = hipMemsetAsync(null_at, 0xff, 8, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_group_sortkey, dim3(grid_for((long long)ng)), dim3(256), 0, st, a.ktype, ng, a.knull, a.kw, sk,
                       sv, null_at);
    e = rocprim::radix_sort_pairs(tmp, *tmp_bytes, sk, sk2, sv, sv2, ng, 0, 64, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_group_nullpos, dim3(grid_for((long long)ng)), dim3(256), 0, st, (const unsigned*)sv2, ng,
                       null_at);
    a.order = sv2;
    a.null_at = null_at;
    hipLaunchKernelGGL(k_group_emit, dim3(grid_for((long long)ng)), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_round(const RoundArgs& a, hipStream_t st) {
    if (!a.ngroups || !a.naggs) return hipSuccess;
    hipLaunchKernelGGL(k_group_round, dim3(grid_for((long long)(a.ngroups * a.naggs), kRoundBlock)),
                       dim3(kRoundBlock), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_normalize(u64* acc, int words, const int* foff, int nf, u64 ngroups, hipStream_t st) {
    if (!nf || !ngroups) return hipSuccess;
    NormArgs a{};
    a.acc = acc;
    a.words = words;
    a.nf = nf;
    for (int f = 0; f < nf && f < kMaxAggs; ++f) a.foff[f] = foff[f];
    a.ngroups = ngroups;
    hipLaunchKernelGGL(k_group_normalize, dim3(grid_for((long long)(ngroups * nf))), dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace gb
}  // namespace dfmi
