// Device skeleton of the query-compiled Selection + Projection kernels.
//
// Hand-written CDNA4 code shared by every compiled query: kernel arguments,
// wave64 helpers, the single-pass decoupled look-back, validity / Boolean
// bitmap access, Utf8 helpers and the per-tile compaction step. The query
// compiler (jit.cpp) appends one kernel whose body is the query's predicate
// and projections written out as straight-line code over this skeleton, so
// nothing is interpreted at run time (see DESIGN.md "Kernels").
//
// The text of this file is embedded into libdfmi.so and compiled with hipRTC
// (-O3 -ffp-contract=off, gfx950) together with the generated body; the build
// also compiles it with hipcc against a sample body to catch errors early.
#ifndef DFMI_SKELETON
#define DFMI_SKELETON

typedef unsigned long long u64;
typedef long long i64;
typedef unsigned char u8;
typedef signed char i8;
typedef short i16;
typedef int i32;
typedef unsigned short u16;
typedef unsigned u32;

#ifndef DFMI_LIGHT_COPY
#define DFMI_LIGHT_COPY 0
#endif
#ifndef DFMI_LONG_COPY
#define DFMI_LONG_COPY 0
#endif
namespace dfmi {

constexpr int kArgCols = 16;   // numeric / Boolean input columns
constexpr int kArgUtf8 = 16;   // Utf8 input columns
constexpr int kArgOut = 16;    // output columns
constexpr int kArgLits = 32;   // 64-bit literals
constexpr int kArgStr = 256;   // string literal bytes

struct Args {
    i64 n_rows;
    int n_tiles;
    int mode;                          // bit1: no look-back (diagnostics: wrong offsets, same traffic)
    const void* col[kArgCols];         // numeric values / Boolean bits
    const u8* valid[kArgCols];         // validity bitmaps (nullptr = all valid)
    const int* offs[kArgUtf8];         // Utf8 offsets
    const u8* bytes[kArgUtf8];         // Utf8 bytes
    const u8* svalid[kArgUtf8];        // Utf8 validity
    void* out[kArgOut];                // numeric values / Boolean bytes (filtered) / bits (dense)
    u8* out_valid[kArgOut];            // dense kernels: validity bitmaps
    int* out_offs[kArgOut];            // Utf8 outputs
    u8* out_data[kArgOut];
    i64 out_cap[kArgOut];
    int* out_src[kArgOut];             // two-pass Utf8 gather: source start of each selected row
    u64 lits[kArgLits];
    int str_off[8];
    int str_len[8];
    char str[kArgStr];
    u64* status;                       // [n_chan][n_tiles] look-back words
    unsigned* ticket;                  // spare counter (zeroed per launch)
    u64* err;                          // max(~key) error word
    u64* totals;                       // [0..8) channel totals, [8..24) null counts
    u64* stats;                        // look-back statistics (mode bit 4): polls, sleeps, tiles
    // The context's workspace is double-buffered: this launch uses one
    // header + status array (zero on entry) and zeroes the other pair, which
    // the previous launch used, for the next launch -- no memset per call.
    u64* clear_status;                 // previous launch's status words ...
    i64 clear_words;                   // ... [0, clear_words) to zero
    u64* clear_hdr;                    // previous launch's 512-byte header
    // coalesced host batches (host_batch.cpp): the per-batch headers of the
    // previous call, in the other half of its ping-pong device region
    u64* clear_bhdr;
    i64 clear_bhdr_words;
    u64* hdr_out;  // Launch::hdr_out: [batch][32] finished headers (host memory)
    u64* agg;                          // aggregate extension: [copies][aggs][kAggWords] accumulators
    // coalesced batches (dfmi_filter_project_batches): block -> batch, and
    // per batch a row of pointers / sizes the kernel's prologue loads into a
    // local copy of these Args (see jit.cpp "batched")
    const int* tile_batch;
    void* const* batch_ptrs;  // pointers and sizes (as pointer-sized integers)
    // GROUP BY extension: the batch's key window -- key bits gbase + i for
    // slot i < gwidth, slot gwidth for the null key (aggregate.cpp)
    u64 gbase;
    int gwidth;
};

// This block's share of zeroing the previous launch's workspace.
template <int BLOCK>
__device__ __forceinline__ void clear_previous(const Args& A, unsigned block, int tid) {
    const i64 per = (A.clear_words + A.n_tiles - 1) / A.n_tiles;
    const i64 w0 = (i64)block * per;
    const i64 w1 = w0 + per < A.clear_words ? w0 + per : A.clear_words;
    for (i64 w = w0 + tid; w < w1; w += BLOCK) A.clear_status[w] = 0;
    if (block == 0 && tid < 64) A.clear_hdr[tid] = 0;
    const i64 bper = (A.clear_bhdr_words + A.n_tiles - 1) / A.n_tiles;
    const i64 b0 = (i64)block * bper;
    const i64 b1 = b0 + bper < A.clear_bhdr_words ? b0 + bper : A.clear_bhdr_words;
    for (i64 w = b0 + tid; w < b1; w += BLOCK) A.clear_bhdr[w] = 0;
    // diagnostics (mode bit 4): report a look-back timeout once, to test the
    // host's relaunch (exec.cpp)
    if ((A.mode & 16) && block == 0 && tid == 0) atomicMax(A.err, ~(u64)3);
}

enum ErrKind : unsigned { ERRK_DIV_ZERO = 1, ERRK_DIV_OVERFLOW = 2, ERRK_LOOKBACK_TIMEOUT = 3, ERRK_CAPACITY = 4 };

constexpr u64 FLAG_A = 1ull << 62;
constexpr u64 FLAG_P = 2ull << 62;
constexpr u64 VAL_MASK = (1ull << 62) - 1;

__device__ __forceinline__ double f64(u64 x) { return __builtin_bit_cast(double, x); }

// Pointer at a byte offset from `base`. Addresses are formed by pointer
// arithmetic, never by integer -> pointer casts: the compiler then keeps
// them in the global address space (global_* instructions, not flat_*).
template <typename T, typename B>
__device__ __forceinline__ T* at(B* base, i64 off) {
    return (T*)((u8*)base + off);
}
template <typename T, typename B>
__device__ __forceinline__ const T* at(const B* base, i64 off) {
    return (const T*)((const u8*)base + off);
}
__device__ __forceinline__ u64 bits(double x) { return __builtin_bit_cast(u64, x); }
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
// Lane i's 32 bits, zero-extended (the builtin returns int: a plain cast to
// 64 bits would sign-extend).
__device__ __forceinline__ u64 readlane_u(unsigned v, int i) { return (u64)(unsigned)__builtin_amdgcn_readlane(v, i); }
__device__ __forceinline__ u64 readlane_u64(u64 v, int i) {
    return (readlane_u((unsigned)(v >> 32), i) << 32) | readlane_u((unsigned)v, i);
}

__device__ __forceinline__ unsigned lane_rank(u64 mask) {  // set bits below this lane
    return __builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
}

// Wave-wide scans on DPP lane moves (no LDS round trip): row_shr 1/2/4/8
// within each row of 16 lanes, then row_bcast 15/31 carry the row totals
// into the rows above. Every lane of the wave must be active. A source lane
// outside the row / a disabled row contributes 0.
template <int CTRL, int ROWS>
__device__ __forceinline__ unsigned dpp32(unsigned v) {
    return __builtin_amdgcn_update_dpp(0u, v, CTRL, ROWS, 0xf, false);
}

__device__ __forceinline__ unsigned wave_incl_scan32(unsigned v, int lane) {
    (void)lane;
    v += dpp32<0x111, 0xf>(v);  // row_shr:1
    v += dpp32<0x112, 0xf>(v);  // row_shr:2
    v += dpp32<0x114, 0xf>(v);  // row_shr:4
    v += dpp32<0x118, 0xf>(v);  // row_shr:8
    v += dpp32<0x142, 0xa>(v);  // row_bcast:15 -> rows 1, 3
    v += dpp32<0x143, 0xc>(v);  // row_bcast:31 -> rows 2, 3
    return v;
}

template <int CTRL, int ROWS>
__device__ __forceinline__ u64 dpp64(u64 v) {
    const unsigned lo = dpp32<CTRL, ROWS>((unsigned)v), hi = dpp32<CTRL, ROWS>((unsigned)(v >> 32));
    return ((u64)hi << 32) | lo;
}

__device__ __forceinline__ u64 wave_incl_scan(u64 v, int lane) {
    (void)lane;
    v += dpp64<0x111, 0xf>(v);
    v += dpp64<0x112, 0xf>(v);
    v += dpp64<0x114, 0xf>(v);
    v += dpp64<0x118, 0xf>(v);
    v += dpp64<0x142, 0xa>(v);
    v += dpp64<0x143, 0xc>(v);
    return v;
}

// Sum over the wave (uniform result).
__device__ __forceinline__ u64 wave_sum(u64 v) {
    const u64 t = wave_incl_scan(v, 0);
    return readlane_u64(t, 63);
}

// The value of the next lane (lane 63: 0).
__device__ __forceinline__ int next_lane(int v) { return (int)dpp32<0x130, 0xf>((unsigned)v); }  // wave_shl:1

// 64 bits of an LSB-first bitmap starting at row 64*w (w wave-uniform); the
// tail word is assembled bytewise so nothing past the bitmap is read.
__device__ __forceinline__ u64 bitmap_word(const u8* bm, i64 w, i64 n_rows) {
    const i64 nbytes = (n_rows + 7) >> 3;
    const i64 b0 = w * 8;
    if (b0 + 8 <= nbytes) return *(const u64*)(bm + b0);
    u64 v = 0;
    for (i64 i = b0; i < nbytes; ++i) v |= (u64)bm[i] << (8 * (i - b0));
    return v;
}

__device__ __forceinline__ void report_err(u64* err, unsigned ordinal, i64 row, unsigned kind) {
    const u64 key = ((u64)ordinal << 44) | ((u64)row << 4) | kind;
    atomicMax(err, ~key);
}

// arrow 0.12 bool_op on Option<T>: eq/neq compare the Options; lt/le:
// (None,_) => true, (_,None) => false; gt/ge: (None,_) => false,
// (_,None) => true. The result is never null.
template <int OP>
__device__ __forceinline__ bool cmp_opt(bool lv, bool rv, bool res) {
    if (lv && rv) return res;
    if constexpr (OP == 0) return !lv && !rv;
    else if constexpr (OP == 1) return lv || rv;
    else if constexpr (OP == 2 || OP == 3) return !lv;
    else return lv;
}

// Rust `/` on iN / uN after arrow's zero check: truncating division; MIN / -1
// panics and a zero divisor is DivideByZero (both reported by the caller, the
// value here only has to be defined). Out of line: the 64-bit sequence is long.
template <typename T>
__device__ __noinline__ T idiv(T x, T y) {
    if (y == (T)0) return (T)0;
    if constexpr ((T)-1 < (T)0) {
        if (y == (T)-1) return (T)(0ull - (u64)(i64)x);  // wrapping negation
    }
    return (T)(x / y);
}

// NaN results of a Float32 / Float64 operator as the reference's scalar
// loops produce them on x86-64 (SSE2, left operand first): a NaN operand
// propagates quieted, the left one first; an invalid operation on non-NaN
// operands gives x86's negative default NaN. gfx950 would otherwise return
// its own canonical NaN.
template <typename T>
__device__ __forceinline__ T sse_nan(T r, T a, T b) {
    if (r == r) return r;
    if constexpr (sizeof(T) == 8) {
        const u64 x = a != a ? (bits(a) | (1ull << 51)) : (b != b ? (bits(b) | (1ull << 51)) : 0xFFF8000000000000ull);
        return f64(x);
    } else {
        const unsigned ua = __builtin_bit_cast(unsigned, a), ub = __builtin_bit_cast(unsigned, b);
        const unsigned x = a != a ? (ua | (1u << 22)) : (b != b ? (ub | (1u << 22)) : 0xFFC00000u);
        return __builtin_bit_cast(float, x);
    }
}

// iN::MIN as a value of T (signed T only).
template <typename T>
__device__ __forceinline__ constexpr T int_min() {
    return (T)((u64)1 << (8 * sizeof(T) - 1));
}

// CAST extension (DFMI_FLAG_EXT_CAST): the arrow 0.12 cast kernel's
// num::cast::<From, To>(x) -- false (None -> a null) when x does not fit To:
//   int -> int: x outside To's range; float -> int: NaN or trunc(x) outside
//   the range; f64 -> f32: finite and outside [-FLT_MAX, FLT_MAX].
// int -> float and widening float casts always succeed (`as`, round to nearest).
template <typename To, typename From>
__device__ __forceinline__ bool num_cast(From x, To& out) {
    constexpr bool from_int = (From)0.5 == (From)0, to_int = (To)0.5 == (To)0;
    constexpr bool from_signed = (From)-1 < (From)0, to_signed = (To)-1 < (To)0;
    constexpr u64 tmax = ~0ull >> (64 - 8 * (int)sizeof(To) + (to_signed ? 1 : 0));
    if constexpr (from_int && to_int) {
        bool ok;
        if constexpr (from_signed)
            ok = x >= (From)0 ? (u64)x <= tmax : (to_signed && (i64)x >= -(i64)tmax - 1);
        else
            ok = (u64)x <= tmax;
        out = (To)x;
        return ok;
    } else if constexpr (from_int) {
        out = (To)x;
        return true;
    } else if constexpr (to_int) {
        const double d = (double)x;
        const double t = __builtin_trunc(d);
        bool ok;
        if constexpr (sizeof(To) == 8)
            ok = to_signed ? (t >= -0x1p63 && t < 0x1p63) : (t >= 0.0 && t < 0x1p64);
        else
            ok = t >= (to_signed ? -(double)tmax - 1.0 : 0.0) && t <= (double)tmax;  // false for NaN
        out = ok ? (To)t : (To)0;
        return ok;
    } else {
        if constexpr (sizeof(From) > sizeof(To)) {
            const double d = (double)x;
            if (__builtin_isfinite(d) && (d < -0x1.fffffep127 || d > 0x1.fffffep127)) {
                out = (To)0;
                return false;
            }
            if (d != d) {  // x86 cvtsd2ss: quieted, the fraction's top 22 bits kept
                const u64 b = bits(d);
                out = __builtin_bit_cast(float, (unsigned)((b >> 32) & 0x80000000u) | 0x7FC00000u |
                                                    (unsigned)((b >> 29) & 0x3FFFFFu));
                return true;
            }
        } else if constexpr (sizeof(From) < sizeof(To)) {
            if (x != x) {  // x86 cvtss2sd: quieted, the fraction widened
                const unsigned b = __builtin_bit_cast(unsigned, (float)x);
                out = f64(((u64)(b & 0x80000000u) << 32) | 0x7FF8000000000000ull | ((u64)(b & 0x3FFFFFu) << 29));
                return true;
            }
        }
        out = (To)x;
        return true;
    }
}

// Rows past n_rows (the tail tile) read nothing: the callers mask them out.
// The literal's bytes `q` come from the kernel's own Args (A0.str): in the
// coalesced-batches form `A` is a register copy, which must never be indexed
// with a run-time value.
__device__ __forceinline__ bool utf8_eq_lit(const Args& A, int u, i64 row, int lit, const char* q) {
    if (row >= A.n_rows) return false;
    const int s = A.offs[u][row], e = A.offs[u][row + 1];
    const int len = A.str_len[lit];
    if (e - s != len) return false;
    const u8* p = A.bytes[u] + s;
    // early exit: most equal-length candidates differ within the first bytes
    // (filtered tiles use utf8_eq_lit_tile below)
    for (int i = 0; i < len; ++i)
        if (p[i] != (u8)q[i]) return false;
    return true;
}

// Offsets of Utf8 column u for the K rows of a tile (rows base + k*BLOCK +
// 64*wave + lane): one coalesced load per row (its start, s[k]) plus one
// wave-uniform load per 64-row slice (the next slice's first offset, nx[k]);
// a row's end is its right neighbour's start (utf8_end). Rows past n_rows
// read offs[n_rows] (inside the buffer) and come out empty. Slices whose bit
// in `need` is clear (wave-uniform) load nothing.
template <int BLOCK, int K>
__device__ __forceinline__ void utf8_offs_tile(const Args& A, int u, i64 base, int lane, int wave, unsigned need,
                                               int (&s)[K], int (&nx)[K]) {
    const int* off = A.offs[u];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        s[k] = 0;
        nx[k] = 0;
        if (!((need >> k) & 1)) continue;
        const i64 r0 = base + (i64)k * BLOCK + 64 * wave;  // wave-uniform
        const int* o0 = off + r0;                           // (uniform base + lane offset addressing)
        if (r0 + 64 <= A.n_rows) {
            s[k] = o0[lane];
            nx[k] = o0[64];
        } else {
            s[k] = off[r0 + lane < A.n_rows ? r0 + lane : A.n_rows];
            nx[k] = off[A.n_rows];
        }
    }
}

// End offset of this lane's row (all lanes active).
__device__ __forceinline__ int utf8_end(int s, int nx, int lane) {
    const int d = next_lane(s);
    return lane == 63 ? nx : d;
}

// `utf8 column u = literal` for the K rows of a tile whose offsets are in
// s / e. Every equal-length candidate's first min(len, 4) bytes are fetched
// as the (at most two) aligned words holding them, all in flight together;
// only head matches (rare) compare the rest. Only words holding bytes of the
// candidate are read.
template <int BLOCK, int K>
__device__ __forceinline__ void utf8_eq_lit_tile(const Args& A, int u, int lit, const char* q, const int (&s)[K],
                                                 const int (&nx)[K], int lane, bool (&res)[K]) {
    const int len = A.str_len[lit];
    const u8* by = A.bytes[u];
    const int hn = len < 4 ? len : 4;
    const unsigned hm = hn == 4 ? ~0u : ((1u << (8 * hn)) - 1u);
    const unsigned bmis = (unsigned)((u64)by & 3u);
    unsigned qh = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (i < hn) qh |= (unsigned)(u8)q[i] << (8 * i);
    unsigned h[K];
    int e[K];
#pragma unroll
    for (int k = 0; k < K; ++k) e[k] = utf8_end(s[k], nx[k], lane);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        unsigned w = qh;
        if (e[k] - s[k] == len && hn > 0) {
            // 32-bit unsigned offsets from the uniform base (offsets are >= 0)
            const unsigned sk = (unsigned)s[k];
            const unsigned mis = (sk + bmis) & 3u;
            const unsigned w0 = *at<unsigned>(by, sk - mis);
            const unsigned w1 = *at<unsigned>(by, sk - mis + ((mis + (unsigned)hn - 1u) & ~3u));  // the word of byte hn-1
            w = __builtin_amdgcn_alignbyte(w1, w0, mis);
        }
        h[k] = w;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        bool eq = e[k] - s[k] == len && (h[k] & hm) == qh;
        if (eq) {
            const u8* p = by + s[k];
            for (int i = hn; i < len; ++i)
                if (p[i] != (u8)q[i]) {
                    eq = false;
                    break;
                }
        }
        res[k] = eq;
    }
}

__device__ __forceinline__ bool utf8_eq_col(const Args& A, int u, int v, i64 row) {
    if (row >= A.n_rows) return false;
    const int s0 = A.offs[u][row], e0 = A.offs[u][row + 1];
    const int s1 = A.offs[v][row], e1 = A.offs[v][row + 1];
    if (e0 - s0 != e1 - s1) return false;
    for (int i = 0; i < e0 - s0; ++i)
        if (A.bytes[u][s0 + i] != A.bytes[v][s1 + i]) return false;
    return true;
}

__device__ __forceinline__ bool utf8_valid(const Args& A, int u, i64 row) {
    const u8* v = A.svalid[u];
    return !v || row >= A.n_rows || ((v[row >> 3] >> (row & 7)) & 1);
}

__device__ __forceinline__ void st_status(u64* p, u64 v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 ld_status(u64* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Single-pass decoupled look-back (one wave): publish the tile aggregate,
// then read R windows of 64 predecessor status words (one word per lane per
// window, all R loads in flight together) per round trip, summing aggregates
// until an inclusive prefix is found; publish our own inclusive prefix and
// return the exclusive one. Status words are SPREAD words apart: with one
// word per 128-byte line the hundreds of polling waves do not serialise on a
// few shared lines, and s_sleep(SLEEP) between polls keeps the polling
// traffic off the data path (measured, DESIGN.md "Look-back").
// The spin is bounded in wall time: a tile that could never resolve reports
// a timeout instead of hanging the device.
// Publish the tile aggregate (tile 0: its inclusive prefix) -- lane 0 only.
template <int SPREAD>
__device__ __forceinline__ void lb_publish(u64* st, unsigned tile, u64 agg, int lane) {
    if (lane == 0) st_status(st + (i64)tile * SPREAD, (tile == 0 ? FLAG_P : FLAG_A) | agg);
}

// Resolve the exclusive prefix of a tile whose aggregate is published: read
// R windows of 64 predecessor status words (one per lane per window, all R
// loads in flight together) per round trip, summing aggregates until an
// inclusive prefix is found; publish our own inclusive prefix.
template <int R, int SLEEP, int SPREAD, int W = 64>
__device__ u64 lb_resolve(u64* st, unsigned tile, u64 agg, int lane, u64* err, u64* stats = nullptr) {
    static_assert(W >= 1 && W <= 64, "window of 1..64 predecessors per wave load");
    if (tile == 0) return 0;
    u64 excl = 0;
    i64 j = (i64)tile - 1;  // highest predecessor not yet accounted for
    const u64 t_start = __builtin_amdgcn_s_memrealtime();  // 100 MHz
    u64 t0 = t_start;  // last progress: the timeout is time WITHOUT progress
    unsigned polls = 0, sleeps = 0, idle = 0;  // idle: stalled polls since the last progress
    while (true) {
        ++polls;
        const i64 j_before = j;
        u64 w[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const i64 idx = j - lane - W * r;
            // lanes past the window read nothing and stand for a zero aggregate
            w[r] = lane >= W ? FLAG_A : (idx >= 0 ? ld_status(st + idx * SPREAD) : FLAG_P);
        }
        bool done = false, stall = false;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const unsigned flag = (unsigned)(w[r] >> 62);
            const u64 xm = __ballot(flag == 0);
            const u64 pm = __ballot(flag == 2);
            if (pm) {
                const int first = __builtin_ctzll(pm);
                const u64 need = first == 63 ? ~0ull : ((2ull << first) - 1);
                if (!(xm & need)) {
                    excl += wave_sum(lane <= first ? (w[r] & VAL_MASK) : 0);
                    done = true;
                } else {
                    stall = true;
                }
                break;
            }
            if (xm) {
                stall = true;
                break;
            }
            excl += wave_sum(w[r] & VAL_MASK);
            j -= W;
        }
        if (done) break;
        if (stall) {
            const u64 now = __builtin_amdgcn_s_memrealtime();
            if (j != j_before) {
                t0 = now;  // predecessors resolved this round: progress
                idle = 0;
            } else if (++idle > 200000u && now - t0 > 200000000ull) {
                // 2 s and 200k polls without a single predecessor resolving:
                // report, do not hang. Both bounds: a queue time-sliced off the
                // GPU (processes sharing it) sees the clock jump while its
                // waves are saved, but polls nothing meanwhile.
                if (lane == 0) report_err(err, 0, 0, ERRK_LOOKBACK_TIMEOUT);
                break;
            }
            __builtin_amdgcn_s_sleep(SLEEP);
            ++sleeps;
        }
    }
    if (lane == 0) st_status(st + (i64)tile * SPREAD, FLAG_P | (excl + agg));
    if (stats && lane == 0) {
        atomicAdd(stats, (u64)polls);
        atomicAdd(stats + 1, (u64)sleeps);
        atomicAdd(stats + 2, __builtin_amdgcn_s_memrealtime() - t_start);
    }
    return excl;
}

// Single-pass decoupled look-back (one wave): publish, then resolve. Status
// words are SPREAD words apart: with one word per 128-byte line the hundreds
// of polling waves do not serialise on a few shared lines, and s_sleep(SLEEP)
// between polls keeps the polling traffic off the data path (measured,
// DESIGN.md "Look-back"). The spin is bounded in wall time: a tile that could
// never resolve reports a timeout instead of hanging the device.
template <int R, int SLEEP, int SPREAD>
__device__ u64 lookback(u64* st, unsigned tile, u64 agg, int lane, u64* err) {
    lb_publish<SPREAD>(st, tile, agg, lane);
    return lb_resolve<R, SLEEP, SPREAD>(st, tile, agg, lane, err);
}

// Workgroup barrier ordering LDS only. __syncthreads() also waits for every
// outstanding global load of the wave (vmcnt(0)); the tile barriers only
// publish LDS values, so projection-column loads stay in flight across the
// look-back instead of being drained before it.
__device__ __forceinline__ void lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Per-tile compaction: the selection words of every (k, wave) are counted,
// scanned in row order, and the tile's output offsets found by look-back.
// NCH channels: 0 = rows, 1.. = Utf8 output bytes (lens given per row).
template <int BLOCK, int K, int NCH>
struct Tile {
    static constexpr int WAVES = BLOCK / 64;
    static constexpr int NW = K * WAVES;  // 64-row words per tile
    static_assert(NW <= 256, "one wave scans the tile's words (up to 4 per lane)");
    unsigned cnt[NCH][NW];  // one slice's rows (<= 64) or Utf8 bytes (< 2^31)
    u64 excl[NCH][NW];
    u64 prefix[NCH];
    u64 agg[NCH];
};

// Sub-tile form of the counting step (multi-sub-tile tiles: M sub-tiles of K
// slices per wave share one scan and one look-back): sub-tile words
// [kb, kb + K) of T, and each (k, wave)'s selection ballot into `ws` (the
// output pass reloads them instead of holding them across the look-back).
template <int BLOCK, int K, int NCH, int KT>
__device__ __forceinline__ void subtile_counts(Tile<BLOCK, KT, NCH>& T, u64* ws, int kb, const unsigned (&cnt)[NCH][K],
                                               const u64 (&wm)[K], int lane, int wave) {
    constexpr int WAVES = BLOCK / 64;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch)
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const u64 s = ch == 0 ? (u64)__builtin_popcountll(wm[k]) : readlane_u(wave_incl_scan32(cnt[ch][k], lane), 63);
            if (lane == 0) T.cnt[ch][(kb + k) * WAVES + wave] = (unsigned)s;
        }
#pragma unroll
    for (int k = 0; k < K; ++k)
        if (lane == 0) ws[(kb + k) * WAVES + wave] = wm[k];
}

// Uniform 64-bit LDS word (the same address in every lane) as a scalar.
__device__ __forceinline__ u64 lds_uniform_u64(const u64* p) {
    const u64 v = *p;
    return ((u64)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)(v >> 32)) << 32) |
           (unsigned)__builtin_amdgcn_readfirstlane((unsigned)v);
}

// The one-wave scan of the tile's words (T.cnt, written by every wave before
// the barrier here) and the publication of the tile aggregate.
template <int BLOCK, int K, int NCH, int SPREAD>
__device__ __forceinline__ void tile_scan_lds(const Args& A, Tile<BLOCK, K, NCH>& T, unsigned tile, int lane,
                                              int wave) {
    constexpr int WAVES = BLOCK / 64;
    constexpr int NW = K * WAVES;
    lds_sync();
    if (wave == 0) {
        u64 packed = 0;
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
            constexpr int NPL = (NW + 63) / 64;  // words per lane, contiguous
            u64 c[NPL], tot = 0;
#pragma unroll
            for (int i = 0; i < NPL; ++i) {
                const int w = lane * NPL + i;
                c[i] = w < NW ? (u64)T.cnt[ch][w] : 0ull;
                tot += c[i];
            }
            const u64 incl = wave_incl_scan(tot, lane);
            u64 ex = incl - tot;
#pragma unroll
            for (int i = 0; i < NPL; ++i) {
                const int w = lane * NPL + i;
                if (w < NW) T.excl[ch][w] = ex;
                ex += c[i];
            }
            const u64 agg = readlane_u64(incl, 63);
            if constexpr (NCH == 2) {
                packed |= agg << (31 * ch);
            } else {
                if (!(A.mode & 2)) lb_publish<SPREAD>(A.status + (i64)ch * A.n_tiles * SPREAD, tile, agg, lane);
            }
            if (lane == 0) T.agg[ch] = agg;
        }
        // rows + one Utf8 output: both counts in one status word (31 + 31
        // bits; the host guarantees rows < 2^31, and the bytes of one Utf8
        // array are < 2^31 by its i32 offsets), so one look-back serves both
        if constexpr (NCH == 2)
            if (!(A.mode & 2)) lb_publish<SPREAD>(A.status, tile, packed, lane);
    }
}

// counts[ch][k] : per-lane value for row k (rows: 0/1 selection, Utf8: bytes)
// First half of the tile step: per-(k, wave) counts, the one-wave scan of the
// tile's words and the publication of the tile aggregate (no waiting).
template <int BLOCK, int K, int NCH, int SPREAD = 1>
__device__ __forceinline__ void tile_scan_publish(const Args& A, Tile<BLOCK, K, NCH>& T, unsigned tile,
                                                  const unsigned (&cnt)[NCH][K], int lane, int wave) {
    constexpr int WAVES = BLOCK / 64;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch)
#pragma unroll
        for (int k = 0; k < K; ++k) {
            // Utf8 byte counts of one slice fit 32 bits (an array holds < 2^31 bytes)
            const u64 s = ch == 0 ? (u64)__builtin_popcountll(__ballot(cnt[0][k] != 0))
                                  : readlane_u(wave_incl_scan32(cnt[ch][k], lane), 63);
            if (lane == 0) T.cnt[ch][k * WAVES + wave] = (unsigned)s;
        }
    tile_scan_lds<BLOCK, K, NCH, SPREAD>(A, T, tile, lane, wave);
}

// Second half: wave 0 resolves the tile's global offsets into T.prefix; a
// block barrier (lds_sync) must follow before other waves read them.
template <int BLOCK, int K, int NCH, int R = 1, int SLEEP = 1, int SPREAD = 1, int W = 64>
__device__ __forceinline__ void tile_resolve(const Args& A, Tile<BLOCK, K, NCH>& T, unsigned tile, int lane,
                                             int wave) {
    if (wave == 0) {
        if constexpr (NCH == 2) {
            constexpr u64 M31 = (1ull << 31) - 1;
            const u64 agg = T.agg[0] | (T.agg[1] << 31);
            const u64 pre = (A.mode & 2) ? (u64)tile * BLOCK * K
                                         : lb_resolve<R, SLEEP, SPREAD, W>(A.status, tile, agg, lane, A.err,
                                                                           (A.mode & 4) ? A.stats : nullptr);
            if (lane == 0) {
                T.prefix[0] = pre & M31;
                T.prefix[1] = pre >> 31;
                if (tile == (unsigned)A.n_tiles - 1) {
                    A.totals[0] = (pre & M31) + T.agg[0];
                    A.totals[1] = (pre >> 31) + T.agg[1];
                }
            }
            return;
        }
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
            const u64 agg = T.agg[ch];
            const u64 pre = (A.mode & 2) ? (ch == 0 ? (u64)tile * BLOCK * K : 0ull)
                                         : lb_resolve<R, SLEEP, SPREAD, W>(A.status + (i64)ch * A.n_tiles * SPREAD,
                                                                           tile, agg, lane, A.err,
                                                                           (A.mode & 4) ? A.stats : nullptr);
            if (lane == 0) {
                T.prefix[ch] = pre;
                if (tile == (unsigned)A.n_tiles - 1) A.totals[ch] = pre + agg;
            }
        }
    }
}

// Both halves back to back: the tile's output offsets in T.
template <int BLOCK, int K, int NCH, int R = 1, int SLEEP = 1, int SPREAD = 1, int W = 64>
__device__ __forceinline__ void tile_offsets(const Args& A, Tile<BLOCK, K, NCH>& T, unsigned tile,
                                             const unsigned (&cnt)[NCH][K], int lane, int wave) {
    tile_scan_publish<BLOCK, K, NCH, SPREAD>(A, T, tile, cnt, lane, wave);
    tile_resolve<BLOCK, K, NCH, R, SLEEP, SPREAD, W>(A, T, tile, lane, wave);
    lds_sync();
}

// Copy L > 0 bytes from src to dst (any alignment) with aligned 4-byte
// words: the output is assembled a word at a time from aligned source words
// (v_alignbyte), interior output words are stored whole and only the two edge
// words bytewise. Source words are clamped to the words holding src[0] and
// src[L-1], so nothing outside them is read. 8 output words per chunk: all
// of a chunk's loads are in flight before its stores (a byte-at-a-time
// load->store loop pays one memory latency per byte).
__device__ __forceinline__ void utf8_copy(const u8* src, u8* dst, unsigned L) {
    const int sm = (int)((u64)src & 3u), dm = (int)((u64)dst & 3u);
    // byte offsets relative to src / dst
    const i64 sw0 = -sm, swl = (i64)((sm + (int)L - 1) & ~3) - sm;  // first / last source word holding bytes
    const i64 dwe = (i64)((dm + (int)L + 3) & ~3) - dm;             // end of the last output word
    for (i64 wb = -dm; wb < dwe; wb += 32) {  // output word at dst + wb, source byte src + wb
        const i64 sbw = ((wb + sm) & ~3ll) - sm;
        const unsigned sh = (unsigned)((wb + sm) & 3);
        unsigned sv[9];
#pragma unroll
        for (int j = 0; j < 9; ++j) {
            i64 a = sbw + 4 * j;
            a = a < sw0 ? sw0 : (a > swl ? swl : a);
            sv[j] = *at<unsigned>(src, a);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const i64 p = wb + 4 * j;  // offset of the word's first byte in dst
            if (p >= dwe) break;
            const unsigned val = __builtin_amdgcn_alignbyte(sv[j + 1], sv[j], sh);
            if (p >= 0 && p + 4 <= (i64)L) {
                *at<unsigned>(dst, p) = val;
            } else {
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    if (p + b >= 0 && p + b < (i64)L) dst[p + b] = (u8)(val >> (8 * b));
            }
        }
    }
}

// Per-lane Utf8 gather: each selected lane copies its own string with
// utf8_copy (diagnostic variant, DFMI_UTF8_GATHER=0).
template <int BLOCK, int K, int NCH, int KT = K>
__device__ __forceinline__ void utf8_gather_lane(const Args& A, const Tile<BLOCK, KT, NCH>& T, int ch, int u, int o,
                                                 unsigned selm, const unsigned (&dst)[K], const int (&s)[K],
                                                 const int (&nx)[K], int lane, int wave, int kb = 0) {
    constexpr int WAVES = BLOCK / 64;
    const u64 bpre = T.prefix[ch];
    const i64 obase = (i64)T.prefix[0];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const bool sel = (selm >> k) & 1;
        const int e = utf8_end(s[k], nx[k], lane);  // every lane (DPP)
        const unsigned L = sel ? (unsigned)(e - s[k]) : 0u;
        const unsigned incl = wave_incl_scan32(L, lane);
        if (!sel) continue;
        const u64 ob = bpre + T.excl[ch][(kb + k) * WAVES + wave] + (incl - L);
        A.out_offs[o][obase + dst[k]] = (int)ob;
        if ((i64)(ob + L) > A.out_cap[o]) {
            report_err(A.err, 0, 0, ERRK_CAPACITY);
            continue;
        }
        if (L == 0) continue;
        utf8_copy(A.bytes[u] + s[k], A.out_data[o] + ob, L);
    }
}

// Direct per-lane Utf8 gather (Launch::gather == 6): gfx950 global loads and
// stores take any byte address, so each selected lane moves its string with
// one or two unaligned 16-byte loads straight into registers and stores
// exactly its bytes back (16 / 8 / 4 / 2 / 1-byte pieces: lanes write disjoint
// byte ranges, no LDS image, no staging round, no edge merge). The loads of
// GRP slices go out together before any of their stores. A 16-byte load may
// read past the string, never past the column's last byte (offs[n_rows]);
// a lane whose string is longer than 32 bytes or ends within 32 bytes of
// that copies with the light per-lane loop.
typedef unsigned v4u_ua __attribute__((ext_vector_type(4), aligned(1)));
typedef unsigned v2u_ua __attribute__((ext_vector_type(2), aligned(1)));
typedef unsigned u32_ua __attribute__((aligned(1)));
typedef unsigned short u16_ua __attribute__((aligned(1)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));

// bytes [0, L) (1 <= L <= 32) of the 32-byte register string {x0, x1} to dst
__device__ __forceinline__ void store_exact32(u8* d, v4u x0, v4u x1, unsigned L) {
    v4u a = x0;
    if (L >= 16) {
        *(v4u_ua*)d = x0;
        d += 16;
        a = x1;
    }
    const unsigned r = L >= 16 ? L - 16 : L;  // 0..16
    if (r == 16) {
        *(v4u_ua*)d = a;
        return;
    }
    unsigned w0 = a.x, w1 = a.y;
    if (r & 8) {
        *(v2u_ua*)d = (v2u){a.x, a.y};
        d += 8;
        w0 = a.z;
        w1 = a.w;
    }
    if (r & 4) {
        *(u32_ua*)d = w0;
        d += 4;
        w0 = w1;
    }
    if (r & 2) {
        *(u16_ua*)d = (unsigned short)w0;
        d += 2;
        w0 >>= 16;
    }
    if (r & 1) *d = (u8)w0;
}

__device__ __forceinline__ void light_copy(const u8* sp, u8* dp, unsigned L) {
    unsigned i = 0;
#pragma unroll 1
    for (; i + 16 <= L; i += 16) *(v4u_ua*)(dp + i) = *(const v4u_ua*)(sp + i);
#pragma unroll 1
    for (; i + 4 <= L; i += 4) *(u32_ua*)(dp + i) = *(const u32_ua*)(sp + i);
#pragma unroll 1
    for (; i < L; ++i) dp[i] = sp[i];
}

// The per-lane copy for long strings (Launch::long_copy, chosen when the
// query's last large batch selected strings of >= kLongLen bytes on average,
// whose slices overflow the stage): 64 bytes per round -- four unaligned
// 16-byte loads in flight, then their stores -- and the last < 64 bytes as
// up to four loads and exact-length stores; a load never reads past the
// column's last byte (endb = offs[n_rows]), the light loop covers that edge.
__device__ __forceinline__ void long_copy(const u8* src, int s, u8* dp, unsigned L, int endb) {
    const u8* sp = src + s;
    unsigned i = 0;
#pragma unroll 1
    for (; i + 64 <= L; i += 64) {
        const v4u a = *(const v4u_ua*)(sp + i), b = *(const v4u_ua*)(sp + i + 16);
        const v4u c = *(const v4u_ua*)(sp + i + 32), d = *(const v4u_ua*)(sp + i + 48);
        *(v4u_ua*)(dp + i) = a;
        *(v4u_ua*)(dp + i + 16) = b;
        *(v4u_ua*)(dp + i + 32) = c;
        *(v4u_ua*)(dp + i + 48) = d;
    }
    const unsigned r = L - i;  // < 64
    if (!r) return;
    if ((i64)s + i + ((r + 15) & ~15u) > (i64)endb) {
        light_copy(sp + i, dp + i, r);
        return;
    }
    v4u c[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (16u * j < r) c[j] = *(const v4u_ua*)(sp + i + 16 * j);
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (16u * j < r) {
            const unsigned rem = r - 16u * j;
            if (rem >= 16) *(v4u_ua*)(dp + i + 16 * j) = c[j];
            else store_exact32(dp + i + 16 * j, c[j], c[j], rem);
        }
}

template <int BLOCK, int K, int NCH, int GRP, int KT = K>
__device__ __forceinline__ void utf8_gather_direct(const Args& A, const Tile<BLOCK, KT, NCH>& T, int ch, int u, int o,
                                                   unsigned selm, const unsigned (&dst)[K], const int (&s)[K],
                                                   const int (&nx)[K], int lane, int wave, int kb = 0) {
    static_assert(K % GRP == 0, "slices per group divide the tile's slices");
    constexpr int WAVES = BLOCK / 64;
    const u64 bpre = T.prefix[ch];
    const i64 obase = (i64)T.prefix[0];
    const u8* src = A.bytes[u];
    u8* out = A.out_data[o];
    const int endb = A.offs[u][A.n_rows];  // the column's last byte + 1 (uniform)
#pragma unroll
    for (int g = 0; g < K; g += GRP) {
        v4u q0[GRP], q1[GRP];
        u64 ob[GRP];
        unsigned Lg[GRP];
        bool fast[GRP];
#pragma unroll
        for (int j = 0; j < GRP; ++j) {
            const int k = g + j;
            const bool sel = (selm >> k) & 1;
            const int e = utf8_end(s[k], nx[k], lane);  // every lane (DPP)
            const unsigned L = sel ? (unsigned)(e - s[k]) : 0u;
            const unsigned incl = wave_incl_scan32(L, lane);
            ob[j] = bpre + T.excl[ch][(kb + k) * WAVES + wave] + (incl - L);
            Lg[j] = L;
            if (sel) A.out_offs[o][obase + dst[k]] = (int)ob[j];
            fast[j] = L > 0 && L <= 32 && s[k] + 32 <= endb;
            if (fast[j]) {
                q0[j] = *(const v4u_ua*)(src + s[k]);
                q1[j] = L > 16 ? *(const v4u_ua*)(src + s[k] + 16) : q0[j];
            }
        }
#pragma unroll
        for (int j = 0; j < GRP; ++j) {
            const int k = g + j;
            const unsigned L = Lg[j];
            if (L == 0) continue;
            if ((i64)(ob[j] + L) > A.out_cap[o]) {
                report_err(A.err, 0, 0, ERRK_CAPACITY);
                continue;
            }
            if (fast[j]) store_exact32(out + ob[j], q0[j], q1[j], L);
            else light_copy(src + s[k], out + ob[j], L);
        }
    }
}

// LDS staging of one wave's Utf8 gather.
constexpr int kStageChunks = 128;  // 16-byte source chunks of one slice's span: 2 KiB (longer: per-lane copy)
template <int ARENA = kStageChunks, int DST = kStageChunks + 1>
struct Utf8Stage {
    static_assert(ARENA >= kStageChunks, "the arena holds at least one slice's span");
    static_assert(DST >= 32, "room for utf8_emit_slice's lane table / a 512-byte image");
    uint4 src[ARENA];  // source spans of consecutive slices, whole aligned 16-byte chunks
    // one slice's output bytes at their output address modulo 4 (LDS-image
    // variants; a slice whose output is longer copies per lane), or
    // utf8_emit_slice's lane table (32 chunks)
    uint4 dst[DST];
};

typedef __attribute__((address_space(1))) void dfmi_gvoid;
typedef __attribute__((address_space(3))) void dfmi_lvoid;

// Chunks [0, n) of the 16-byte-chunk span at global `sp` into LDS at `dst`
// (wave-uniform) with direct global->LDS loads (global_load_lds_dwordx4:
// lane l of an instruction writes dst + 16 l; no VGPRs). Completion:
// wait_vm_loads().
__device__ __forceinline__ void stage_span(const uint4* sp, uint4* dst, int n, int lane) {
    for (int c = 0; c < n; c += 64)
        if (c + lane < n) __builtin_amdgcn_global_load_lds((dfmi_gvoid*)(sp + c + lane), (dfmi_lvoid*)(dst + c), 16, 0, 0);
}
__device__ __forceinline__ void wait_vm_loads() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Orders this wave's LDS accesses (a wave's LDS operations execute in
// order; this keeps the compiler from moving them across).
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

// Dense form of utf8_eq_lit_tile (Launch::eq_dense, diagnostic A/B): the
// wave's K slices' whole source spans are staged into its LDS arena with
// direct global->LDS loads (coalesced 16-byte chunks, ~14 B/row at C3's
// strings) instead of fetching only the equal-length candidates' head words
// (scattered, ~6 B/row of 64-byte sectors); candidates then compare from LDS.
// A slice whose span does not fit the arena compares from global memory.
template <int BLOCK, int K, int CAP>
__device__ __forceinline__ void utf8_eq_lit_tile_dense(const Args& A, int u, int lit, const char* q, const int (&s)[K],
                                                       const int (&nx)[K], int lane, bool (&res)[K], uint4* arena) {
    const int len = A.str_len[lit];
    const u8* by = A.bytes[u];
    const int sm = (int)((u64)by & 15u);
    int cs[K], off[K];
    int used = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int s0 = __builtin_amdgcn_readlane(s[k], 0), s1 = __builtin_amdgcn_readfirstlane(nx[k]);
        const int c0 = (int)((((i64)s0 + sm) & ~15ll) - sm);
        const int n = s1 > s0 ? (int)((((i64)s1 - 1 - c0) >> 4)) + 1 : 0;
        cs[k] = c0;
        off[k] = -1;
        if (n > 0 && used + n <= CAP) {
            stage_span(at<uint4>(by, c0), arena + used, n, lane);
            off[k] = 16 * used;
            used += n;
        }
    }
    wait_vm_loads();
    wave_lds_fence();
    const u8* lb = (const u8*)arena;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int e = utf8_end(s[k], nx[k], lane);
        bool eq = e - s[k] == len;
        if (eq) {
            if (off[k] >= 0) {
                const u8* p = lb + off[k] + (s[k] - cs[k]);
#pragma unroll 1
                for (int i = 0; i < len; ++i)
                    if (p[i] != (u8)q[i]) {
                        eq = false;
                        break;
                    }
            } else {
                const u8* p = by + s[k];
#pragma unroll 1
                for (int i = 0; i < len; ++i)
                    if (p[i] != (u8)q[i]) {
                        eq = false;
                        break;
                    }
            }
        }
        res[k] = eq;
    }
    wave_lds_fence();  // the arena is reused by the next sub-tile
}

// Register-resident dense form of utf8_eq_lit_tile (Launch::eq_dense < 0,
// diagnostic A/B): each 64-row slice's whole source span
// is read with ONE coalesced 16-byte load per lane (a span of at most 64
// chunks: ~888 B at C3's strings), G slices' loads in flight together, no
// LDS; an equal-length candidate takes the words holding its first bytes
// from the lanes that loaded them (ds_bpermute of the four dwords of the
// owning lane, plus the next lane's first dword for a head that crosses it).
// A slice whose span needs more than 64 chunks fetches its candidates' head
// words from global memory, as utf8_eq_lit_tile does.
template <int BLOCK, int K, int G>
__device__ __forceinline__ void utf8_eq_lit_tile_reg(const Args& A, int u, int lit, const char* q, const int (&s)[K],
                                                     const int (&nx)[K], int lane, bool (&res)[K]) {
    const int len = A.str_len[lit];
    const u8* by = A.bytes[u];
    const int sm = (int)((u64)by & 15u);
    const int hn = len < 4 ? len : 4;
    const unsigned hm = hn == 4 ? ~0u : ((1u << (8 * hn)) - 1u);
    const unsigned bmis = (unsigned)((u64)by & 3u);
    unsigned qh = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (i < hn) qh |= (unsigned)(u8)q[i] << (8 * i);
#pragma unroll
    for (int g0 = 0; g0 < K; g0 += G) {
        uint4 v[G];
        int c0[G];
        bool fits[G];
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int k = g0 + j;
            v[j] = make_uint4(0u, 0u, 0u, 0u);
            const int s0 = __builtin_amdgcn_readfirstlane(s[k]), s1 = __builtin_amdgcn_readfirstlane(nx[k]);
            c0[j] = (int)((((i64)s0 + sm) & ~15ll) - sm);
            const int nch = s1 > s0 ? (int)(((i64)s1 - 1 - c0[j]) >> 4) + 1 : 0;
            fits[j] = nch <= 64;
            if (fits[j] && lane < nch) v[j] = *at<uint4>(by, (i64)c0[j] + 16 * lane);
        }
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int k = g0 + j;
            const int e = utf8_end(s[k], nx[k], lane);
            const bool cand = e - s[k] == len && hn > 0;
            unsigned w = qh;
            if (fits[j]) {
                const int rel = cand ? s[k] - c0[j] : 0;  // byte of the head in the span
                const int dw = rel >> 2, src = dw >> 2, comp = dw & 3;
                const int a0 = src << 2, a1 = (src + 1 < 64 ? src + 1 : 63) << 2;
                const unsigned x = (unsigned)__builtin_amdgcn_ds_bpermute(a0, (int)v[j].x);
                const unsigned y = (unsigned)__builtin_amdgcn_ds_bpermute(a0, (int)v[j].y);
                const unsigned z = (unsigned)__builtin_amdgcn_ds_bpermute(a0, (int)v[j].z);
                const unsigned ww = (unsigned)__builtin_amdgcn_ds_bpermute(a0, (int)v[j].w);
                const unsigned nxw = (unsigned)__builtin_amdgcn_ds_bpermute(a1, (int)v[j].x);
                const unsigned w0 = comp == 0 ? x : comp == 1 ? y : comp == 2 ? z : ww;
                const unsigned w1 = comp == 0 ? y : comp == 1 ? z : comp == 2 ? ww : nxw;
                if (cand) w = __builtin_amdgcn_alignbyte(w1, w0, (unsigned)(rel & 3));
            } else if (cand) {  // span over 64 chunks: the head words from global memory
                const unsigned sk = (unsigned)s[k];
                const unsigned mis = (sk + bmis) & 3u;
                const unsigned w0 = *at<unsigned>(by, sk - mis);
                const unsigned w1 = *at<unsigned>(by, sk - mis + ((mis + (unsigned)hn - 1u) & ~3u));
                w = __builtin_amdgcn_alignbyte(w1, w0, mis);
            }
            bool eq = cand && (w & hm) == qh;
            if (eq) {
                const u8* p = by + s[k];
                for (int i = hn; i < len; ++i)
                    if (p[i] != (u8)q[i]) {
                        eq = false;
                        break;
                    }
            }
            res[k] = len == 0 ? e - s[k] == 0 : eq;
        }
    }
}

// OR v into the LDS word p (no return value). Through inline asm: the
// compiler's wait-count pass, which does not see the explicit vmcnt wait
// after each staging round, otherwise puts an s_waitcnt vmcnt(0) before
// every LDS atomic after direct global->LDS loads -- which also waits for
// the global stores issued since (the previous slice's image and offsets).
// A wave's LDS operations execute in order: later reads of p see the result.
// The same holds for plain LDS stores issued after global stores (each
// would wait for them): the LDS image's writes all go through these.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(size_t)(__attribute__((address_space(3))) const void*)p;
}
__device__ __forceinline__ void lds_or(unsigned* p, unsigned v) {
    asm volatile("ds_or_b32 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_st32(unsigned* p, unsigned v) {
    asm volatile("ds_write_b32 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_st32x2(unsigned* p, unsigned v0, unsigned v1) {  // p[0], p[1]
    asm volatile("ds_write2_b32 %0, %1, %2 offset1:1" ::"v"(lds_addr(p)), "v"(v0), "v"(v1) : "memory");
}
__device__ __forceinline__ void lds_zero128(uint4* p) {
    const u32x4 z = {0u, 0u, 0u, 0u};
    asm volatile("ds_write_b128 %0, %1" ::"v"(lds_addr(p)), "v"(z) : "memory");
}

// Bytes [lo, hi) of a word as a mask (0 <= lo < hi <= 4).
__device__ __forceinline__ unsigned byte_mask(int lo, int hi) {
    return (0xffffffffu >> (8 * (4 - hi))) & (0xffffffffu << (8 * lo));
}

// Copy the selected rows of Utf8 input u into output o (rebased i32
// offsets + bytes, filter.rs:94-105), one 64-row slice at a time, the wave
// cooperating. The slice's source span (first to last selected string) is
// read with coalesced 16-byte loads into LDS; each selected lane ORs its
// string, assembled into aligned words with v_alignbyte, into a zeroed LDS
// image of the slice's output (strings that share an edge word merge
// there); the wave then stores the image as coalesced aligned words --
// bytewise only the two edge words the slice shares with its neighbours. A
// span over 2 KiB (long strings) falls back to a per-lane copy. Source reads
// are whole aligned 16-byte chunks holding span bytes. One global round trip
// per slice (diagnostic variant DFMI_UTF8_GATHER=2; utf8_gather below stages
// consecutive slices together).
template <int BLOCK, int K, int NCH, int ARENA, int KT = K, int DST = kStageChunks + 1>
__device__ __forceinline__ void utf8_gather_serial(const Args& A, const Tile<BLOCK, KT, NCH>& T, int ch, int u, int o,
                                                   unsigned selm, const u64 (&wm)[K], const unsigned (&dst)[K],
                                                   const int (&s)[K], const int (&nx)[K], Utf8Stage<ARENA, DST>& G,
                                                   int lane, int wave, int kb = 0) {
    constexpr int WAVES = BLOCK / 64;
    const u64 bpre = T.prefix[ch];
    const i64 obase = (i64)T.prefix[0];
    const u8* src = A.bytes[u];
    u8* out = A.out_data[o];
    const unsigned* gs = (const unsigned*)G.src;
    unsigned* gd = (unsigned*)G.dst;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const u64 m = wm[k];
        if (!m) continue;
        const bool sel = (selm >> k) & 1;
        const int e = utf8_end(s[k], nx[k], lane);
        const unsigned L = sel ? (unsigned)(e - s[k]) : 0u;
        const unsigned incl = wave_incl_scan32(L, lane);
        const unsigned rel = incl - L;
        const unsigned Ls = (unsigned)readlane_u(incl, 63);
        const u64 ob0 = bpre + T.excl[ch][(kb + k) * WAVES + wave];
        if (sel) A.out_offs[o][obase + dst[k]] = (int)(ob0 + rel);
        if ((i64)(ob0 + Ls) > A.out_cap[o]) {
            if (lane == 0) report_err(A.err, 0, 0, ERRK_CAPACITY);
            continue;
        }
        if (Ls == 0) continue;
        const int fl = __builtin_ctzll(m), ll = 63 - __builtin_clzll(m);
        const i64 s0 = __builtin_amdgcn_readlane(s[k], fl), s1 = __builtin_amdgcn_readlane(e, ll);  // s1 > s0
        const i64 sm = (i64)((u64)src & 15u);
        const i64 c0 = ((s0 + sm) & ~15ll) - sm;  // offset of the 16-byte chunk holding byte s0, from src
        const int nch = (int)(((s1 - 1 - c0) >> 4)) + 1;
        if (nch > kStageChunks) {
            if (sel && L) utf8_copy(src + s[k], out + ob0 + rel, L);
            continue;
        }
        const int sh = (int)(((u64)out + ob0) & 3u);  // output address mod 4 = the slice's offset in G.dst
        u8* const w0 = out + ((i64)ob0 - sh);        // the aligned word holding the slice's first byte
        const int nw = (sh + (int)Ls + 3) >> 2;
        const uint4* sp = at<uint4>(src, c0);  // wave-uniform
        for (int c = lane; c < nch; c += 64) G.src[c] = sp[c];
        for (int c = lane; 4 * c < nw; c += 64) G.dst[c] = make_uint4(0u, 0u, 0u, 0u);
        wave_lds_fence();
        if (L) {
            // this string: source bytes [a, a + L) of G.src, output bytes [d, d + L) of G.dst
            const int a = (int)(s[k] - c0);
            const int d = sh + (int)rel;
            const int wl = (d + (int)L - 1) >> 2;
            for (int w = d >> 2; w <= wl; ++w) {
                const int p = 4 * w - d;   // position of the word's first byte in the string (>= -3)
                const int sb = a + p;      // ... in G.src (>= -3)
                const int sw = sb >> 2;    // arithmetic shift: -1 at most
                const unsigned lo = gs[sw < 0 ? 0 : sw], hi = gs[sw + 1];
                const unsigned val = __builtin_amdgcn_alignbyte(hi, lo, (unsigned)sb & 3u);
                const unsigned msk = byte_mask(p < 0 ? -p : 0, p + 4 > (int)L ? (int)L - p : 4);
                lds_or(gd + w, val & msk);
            }
        }
        wave_lds_fence();
        for (int j = lane; j < nw; j += 64) {
            const unsigned val = gd[j];
            const int p = 4 * j - sh;  // output position of the word's first byte
            if (p >= 0 && p + 4 <= (int)Ls) {
                *at<unsigned>(w0, 4 * j) = val;
            } else {
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    if (p + b >= 0 && p + b < (int)Ls) w0[4 * j + b] = (u8)(val >> (8 * b));
            }
        }
        wave_lds_fence();
    }
}

// One string into the zeroed LDS output image gd: source bytes [a, a + L)
// of the staged span sg, output bytes [d, d + L) of gd (L > 0). Words
// inside the string are this string's alone and are written whole (one
// v_alignbyte of two aligned source words, two words per iteration); only
// its first and last word, which it may share with the neighbouring
// strings, are OR-merged masked. (Storing the inside words straight to
// global memory instead of through the image measured slower: 1.32 -> 1.34
// ms per C3 batch)
__device__ __forceinline__ void utf8_place(const unsigned* sg, unsigned* gd, int a, int d, int L) {
    const int delta = a - d;  // source byte = output byte + delta
    const int wf = d >> 2, wl = (d + L - 1) >> 2;
    auto edge = [&](int w) {
        const int p = 4 * w - d;  // position of the word's first byte in the string (>= -3)
        const int sb = a + p;     // ... in the span (>= -3)
        const int sw = sb >> 2;   // arithmetic shift: -1 at most
        const unsigned lo = sg[sw < 0 ? 0 : sw], hi = sg[sw + 1];
        const unsigned val = __builtin_amdgcn_alignbyte(hi, lo, (unsigned)sb & 3u);
        const unsigned msk = byte_mask(p < 0 ? -p : 0, p + 4 > L ? L - p : 4);
        lds_or(gd + w, val & msk);
    };
    edge(wf);
    if (wl != wf) edge(wl);
    int w = wf + 1;
    for (; w + 1 < wl; w += 2) {
        const int sb = 4 * w + delta;  // >= 0: an interior word starts inside the string
        const int sw = sb >> 2;
        const unsigned sh = (unsigned)sb & 3u;
        const unsigned x0 = sg[sw], x1 = sg[sw + 1], x2 = sg[sw + 2];
        lds_st32x2(gd + w, __builtin_amdgcn_alignbyte(x1, x0, sh), __builtin_amdgcn_alignbyte(x2, x1, sh));
    }
    if (w < wl) {
        const int sb = 4 * w + delta;
        const int sw = sb >> 2;
        lds_st32(gd + w, __builtin_amdgcn_alignbyte(sg[sw + 1], sg[sw], (unsigned)sb & 3u));
    }
}

// Output words of one slice from its staged source span sg (lanes on
// consecutive output words, no per-string loops, no LDS image): each lane's
// string is described by a two-entry table in LDS -- tend[l], the end of
// lane l's output in image coordinates (image byte 0 = the aligned word
// holding the slice's first output byte, which sits at image byte `sh`), and
// tdel[l], source byte minus image byte for that string (lanes without a
// string: zero length, tend = their left neighbour's). An output word finds
// the string holding its first byte by a 6-step binary search over tend
// (non-decreasing), takes its bytes with one v_alignbyte of two staged source
// words, and repeats for the (rare) next string that starts inside the word:
// at most 4 rounds. Interior words are stored whole; the two edge words the
// slice shares with its neighbours bytewise.
__device__ __forceinline__ int utf8_lb(const int* tend, int q) {  // first lane whose string ends after q
    int i = 0;
#pragma unroll
    for (int st = 32; st >= 1; st >>= 1)
        if (tend[i + st - 1] <= q) i += st;
    return i;
}
__device__ __forceinline__ void utf8_emit_slice(const unsigned* sg, int* tab, u8* w0, int sh, int iend, unsigned incl,
                                                unsigned rel, int a, int lane) {
    int* tend = tab;
    int* tdel = tab + 64;
    tend[lane] = sh + (int)incl;
    tdel[lane] = a - (sh + (int)rel);
    wave_lds_fence();
    const int nw = (iend + 3) >> 2;
    for (int j = lane; j < nw; j += 64) {
        const int P = 4 * j;
        const int hi = P + 4 < iend ? P + 4 : iend;
        int lo = P > sh ? P : sh;
        unsigned val = 0;
#pragma unroll 1
        while (lo < hi) {
            const int i = utf8_lb(tend, lo);  // tend[i] > lo: string i holds image byte lo
            const int e = tend[i] < hi ? tend[i] : hi;
            const int sb = P + tdel[i];  // source byte of image byte P under string i's shift (>= -3)
            const int sw = sb >> 2;      // arithmetic shift: -1 at most
            const unsigned x = __builtin_amdgcn_alignbyte(sg[sw + 1], sg[sw < 0 ? 0 : sw], (unsigned)sb & 3u);
            val |= x & byte_mask(lo - P, e - P);
            lo = e;
        }
        if (P >= sh && P + 4 <= iend) {
            *at<unsigned>(w0, P) = val;
        } else {
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (P + b >= sh && P + b < iend) w0[P + b] = (u8)(val >> (8 * b));
        }
    }
    wave_lds_fence();
}

// Inclusive max-scan over the wave (values >= 0; every lane active).
__device__ __forceinline__ unsigned wave_incl_max32(unsigned v) {
    v = max(v, dpp32<0x111, 0xf>(v));  // row_shr:1
    v = max(v, dpp32<0x112, 0xf>(v));  // row_shr:2
    v = max(v, dpp32<0x114, 0xf>(v));  // row_shr:4
    v = max(v, dpp32<0x118, 0xf>(v));  // row_shr:8
    v = max(v, dpp32<0x142, 0xa>(v));  // row_bcast:15
    v = max(v, dpp32<0x143, 0xc>(v));  // row_bcast:31
    return v;
}

// utf8_emit_slice with the string of each output word found by a marker
// scan instead of a binary search: the last string starting in image word w
// marks mk[w] with its lane + 1 (a string knows it is the last one starting
// in its word when its end lies in a later word or it is the slice's last),
// and a wave max-scan of the markers in word order gives every word the last
// string starting before it -- where its first bytes come from. A word then
// walks forward through the non-empty strings (`ne` ballot) that start inside
// it: one or two rounds, at most four.
__device__ __forceinline__ void utf8_emit_slice_mk(const unsigned* sg, int* tab, u8* mk, u8* w0, int sh, int iend,
                                                   unsigned incl, unsigned rel, unsigned L, int a, int lane) {
    int* tend = tab;
    int* tdel = tab + 64;
    const int st = sh + (int)rel, en = sh + (int)incl;
    tend[lane] = en;
    tdel[lane] = a - st;
    const int nw = (iend + 3) >> 2;
    for (int j = lane; j < nw; j += 64) mk[j] = 0;
    wave_lds_fence();
    const u64 ne = __ballot(L != 0);
    if (L != 0 && ((en >> 2) != (st >> 2) || en >= iend)) mk[st >> 2] = (u8)(lane + 1);
    wave_lds_fence();
    unsigned carry = 0;  // last string starting before this round's first word
    for (int j0 = 0; j0 < nw; j0 += 64) {
        const int j = j0 + lane;
        const unsigned m = j < nw ? (unsigned)mk[j] : 0u;
        const unsigned incm = max(wave_incl_max32(m), carry);
        const unsigned prev = max((unsigned)__builtin_amdgcn_update_dpp(0, (int)incm, 0x138, 0xf, 0xf, false), carry);  // wave_shr:1
        carry = (unsigned)__builtin_amdgcn_readlane((int)incm, 63);
        if (j >= nw) continue;
        const int P = 4 * j;
        const int hi = P + 4 < iend ? P + 4 : iend;
        int lo = P > sh ? P : sh;
        // first candidate: the last string starting before this word, else the first string
        int i = prev ? (int)prev - 1 : __builtin_ctzll(ne);
        unsigned val = 0;
#pragma unroll 1
        while (lo < hi) {
            const int e = tend[i] < hi ? tend[i] : hi;
            if (e > lo) {
                const int sb = P + tdel[i];  // source byte of image byte P under string i's shift (>= -3)
                const int sw = sb >> 2;
                const unsigned x = __builtin_amdgcn_alignbyte(sg[sw + 1], sg[sw < 0 ? 0 : sw], (unsigned)sb & 3u);
                val |= x & byte_mask(lo - P, e - P);
                lo = e;
            }
            const u64 rest = i >= 63 ? 0ull : ne >> (i + 1);
            if (!rest) break;
            i += 1 + __builtin_ctzll(rest);
        }
        if (P >= sh && P + 4 <= iend) {
            *at<unsigned>(w0, P) = val;
        } else {
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (P + b >= sh && P + b < iend) w0[P + b] = (u8)(val >> (8 * b));
        }
    }
    wave_lds_fence();
}

// The 16-byte-chunk source span of slice k (wave-uniform): chunks from the
// one holding the first selected string's first byte to the one holding the
// last one's last byte, as an offset from src and a count (0: no bytes).
// Store a slice's LDS image (output bytes [sh, sh + Ls) of the image, image
// byte 0 at the 16-byte aligned output address w0) with 16-byte stores:
// lanes on the whole chunks (no branches per word), then lanes 0-7 on the
// words of the first and last chunk when they are partial -- shared with
// the neighbouring slices' outputs, written whole words or bytes inside
// [sh, sh + Ls) only.
// The image is zero again afterwards (every word the slice placed is read
// here and zeroed behind the read), so the next slice places without a
// zeroing pass.
__device__ __forceinline__ void utf8_image_store16(uint4* im, u8* w0, int sh, int Ls, int lane) {
    const int e = sh + Ls;
    const int cf = (sh + 15) >> 4;  // first whole chunk
    const int cl = e >> 4;          // one past the last whole chunk
    for (int c = cf + lane; c < cl; c += 64) {
        *at<uint4>(w0, 16 * c) = im[c];
        lds_zero128(im + c);
    }
    // partial chunks: the first (sh > 0, or the slice ends inside it) and the last
    const int pf = (sh & 15) || cl < cf ? 0 : -1;
    const int pl = (e & 15) && (e >> 4) != pf ? (e >> 4) : -1;
    if (lane < 8) {
        const int c = lane < 4 ? pf : pl;
        if (c >= 0) {
            const int w = 4 * c + (lane & 3);  // image word
            const int lo = max(4 * w, sh), hi = min(4 * w + 4, e);
            const unsigned v = ((const unsigned*)im)[w];
            lds_st32((unsigned*)im + w, 0u);
            if (hi - lo == 4) {
                *at<unsigned>(w0, 4 * w) = v;
            } else if (hi > lo) {
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    if (4 * w + b >= lo && 4 * w + b < hi) w0[4 * w + b] = (u8)(v >> (8 * b));
            }
        }
    }
}

// (i32 offsets: the chunk offset, >= -15, fits an int -- 8 SGPRs fewer
// for a tile's spans than i64)
__device__ __forceinline__ void utf8_span(u64 m, int s, int e, int sm, int& c0, int& nch) {
    const int fl = __builtin_ctzll(m), ll = 63 - __builtin_clzll(m);
    const int s0 = __builtin_amdgcn_readlane(s, fl), s1 = __builtin_amdgcn_readlane(e, ll);
    c0 = (int)((((i64)s0 + sm) & ~15ll) - sm);  // offset of the 16-byte chunk holding byte s0, from src
    nch = s1 > s0 ? (int)((((i64)s1 - 1 - c0) >> 4)) + 1 : 0;
}

// Every slice's source span (scalars): chunk offset from src and count.
template <int K>
__device__ __forceinline__ void utf8_spans(const u8* src, const u64 (&wm)[K], const int (&s)[K], const int (&nx)[K],
                                           int lane, int (&cs)[K], int (&cn)[K]) {
    const int sm = (int)((u64)src & 15u);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        cs[k] = 0;
        cn[k] = 0;
        if (wm[k]) utf8_span(wm[k], s[k], utf8_end(s[k], nx[k], lane), sm, cs[k], cn[k]);
    }
}

// Stage the spans of slice k and the following ones while they fit the
// arena (direct global->LDS loads, no wait); returns the last slice covered
// (slices whose span exceeds kStageChunks are copied per lane, not staged).
template <int K, int ARENA>
__device__ __forceinline__ int utf8_stage_group(const u8* src, const u64 (&wm)[K], const int (&cs)[K],
                                                const int (&cn)[K], int k, uint4* arena, int lane,
                                                int scap = kStageChunks) {
    int staged_to = k - 1, used = 0;
    bool full = false;
#pragma unroll
    for (int j = 0; j < K; ++j) {
        if (j < k || full || !wm[j]) continue;
        if (cn[j] > scap) {  // copied per lane when processed
            if (j == k) staged_to = j;
            else full = true;
            continue;
        }
        if (used + cn[j] > ARENA) {
            full = true;
            continue;
        }
        stage_span(at<uint4>(src, cs[j]), arena + used, cn[j], lane);
        used += cn[j];
        staged_to = j;
    }
    return staged_to;
}

// The first staging round of utf8_gather, issued before the tile's look-back
// so that the look-back's wait hides the staging loads; returns the `pre`
// argument of utf8_gather (-1: nothing staged).
template <int K, int CAP, int ARENA, int DST>
__device__ __forceinline__ int utf8_gather_prestage(const Args& A, int u, const u64 (&wm)[K], const int (&s)[K],
                                                    const int (&nx)[K], Utf8Stage<ARENA, DST>& G, int lane) {
    static_assert(CAP <= ARENA, "staging capacity within the arena");
    const u8* src = A.bytes[u];
    int cs[K];
    int cn[K];
    utf8_spans<K>(src, wm, s, nx, lane, cs, cn);
    int k0 = -1;
#pragma unroll
    for (int k = K - 1; k >= 0; --k)
        if (wm[k]) k0 = k;
    return k0 < 0 ? -1 : utf8_stage_group<K, CAP>(src, wm, cs, cn, k0, G.src, lane, CAP < kStageChunks ? CAP : kStageChunks);
}

// Long strings, one slice whose source span overflows the stage
// (Launch::long_copy == 2): the wave copies the slice's selected strings
// itself, 8 lanes per string on consecutive 16-byte chunks -- each load and
// store instruction covers eight 128-byte runs of source and of output
// instead of 64 scattered lanes -- and 4 groups of 8 strings per round, their
// loads in flight together. tab: 64 ints of LDS scratch (the slice's image,
// unused by a slice that takes this path). A chunk that could read past the
// column's last byte (endb) copies with the light loop.
__device__ __forceinline__ void wave_copy_slice(const u8* src, u8* outb, int s_l, unsigned rel_l, unsigned L_l,
                                                int lane, int endb, int* tab) {
    const u64 m = __ballot(L_l > 0);
    if (!m) return;
    if (L_l > 0) tab[lane_rank(m)] = lane;
    wave_lds_fence();
    const int nsel = __builtin_popcountll(m);
    const unsigned maxL = (unsigned)readlane_u(wave_incl_max32(L_l), 63);
    constexpr int G = 4;  // groups of 8 strings per round
    for (int q0 = 0; q0 < nsel; q0 += 8 * G) {
        int sq[G];
        unsigned dq[G], Lq[G];
#pragma unroll
        for (int h = 0; h < G; ++h) {
            const int q = q0 + 8 * h + (lane >> 3);
            const int sl = q < nsel ? tab[q] : lane;
            sq[h] = __builtin_amdgcn_ds_bpermute(sl << 2, s_l);
            dq[h] = (unsigned)__builtin_amdgcn_ds_bpermute(sl << 2, (int)rel_l);
            const unsigned lq = (unsigned)__builtin_amdgcn_ds_bpermute(sl << 2, (int)L_l);
            Lq[h] = q < nsel ? lq : 0u;
        }
        for (unsigned seg = 0; seg < maxL; seg += 128) {
            const unsigned off = seg + 16u * (unsigned)(lane & 7);
            v4u x[G];
#pragma unroll
            for (int h = 0; h < G; ++h)
                if (off < Lq[h] && (i64)sq[h] + off + 16 <= (i64)endb) x[h] = *(const v4u_ua*)(src + sq[h] + off);
#pragma unroll
            for (int h = 0; h < G; ++h) {
                if (off >= Lq[h]) continue;
                const unsigned rem = Lq[h] - off;
                u8* d = outb + dq[h] + off;
                if ((i64)sq[h] + off + 16 <= (i64)endb) {
                    if (rem >= 16) *(v4u_ua*)d = x[h];
                    else store_exact32(d, x[h], x[h], rem);
                } else {
                    light_copy(src + sq[h] + off, d, rem < 16 ? rem : 16u);
                }
            }
        }
    }
    wave_lds_fence();  // tab: the next slice's image
}

// Copy the selected rows of Utf8 input u into output o (rebased i32
// offsets + bytes, filter.rs:94-105), one 64-row slice at a time, the wave
// cooperating: the source spans of consecutive slices are staged into the
// ARENA together with direct global->LDS loads, one wait per arena-full (a
// tile's gather pays about K * (span bytes) / (arena bytes) global round
// trips instead of K; `pre` >= 0: the first round was staged before the
// look-back by utf8_gather_prestage), and each slice's output words are
// written by utf8_emit_slice (or, `image`, assembled in an LDS image first).
// Only scalar state (where the staged round ends, the next arena offset) is
// carried between slices.
template <int BLOCK, int K, int NCH, int ARENA, int KT = K, int DST = kStageChunks + 1>
__device__ __forceinline__ void utf8_gather(const Args& A, const Tile<BLOCK, KT, NCH>& T, int ch, int u, int o,
                                            unsigned selm, const u64 (&wm)[K], const unsigned (&dst)[K],
                                            const int (&s)[K], const int (&nx)[K], Utf8Stage<ARENA, DST>& G, int lane,
                                            int wave, int kb = 0, int emit = 0, int pre = -1, bool prof = false,
                                            bool dbuf = false, bool early = false) {
    constexpr int WAVES = BLOCK / 64;
    const u64 bpre = T.prefix[ch];
    const i64 obase = (i64)T.prefix[0];
    const u8* src = A.bytes[u];
    u8* out = A.out_data[o];
    const unsigned* gs = (const unsigned*)G.src;
    unsigned* gd = (unsigned*)G.dst;
    // early (LDS image, one arena): the next group's spans are staged as soon
    // as the group's last slice is placed -- before that slice's image
    // stores -- so the staging wait counts those stores out instead of
    // waiting for them (vmcnt counts loads and stores in issue order)
    bool e_pend = false;  // a group staged early is in flight: slices (staged_to, e_to]
    int e_to = -1;
    unsigned e_since = 0;  // store instructions issued after it (a lower bound)
    int staged_to = pre;  // slices <= staged_to are in the arena (or need no staging)
    int aoff = 0;         // arena chunk of the next staged slice to process
    int cs[K];
    int cn[K];
    utf8_spans<K>(src, wm, s, nx, lane, cs, cn);
    // diagnostics (`prof`, compiled in by DFMI_GATHER_PHASES, and mode bit 5):
    // shader cycles per phase summed over waves into stats[8..13): staging,
    // slice setup, image zeroing, placing, stores. Reading the counter
    // serialises the wave (~10x slower kernel): relative figures only.
    const bool tp_on = prof && (A.mode & 32) != 0;
    u64 tacc[5] = {0, 0, 0, 0, 0};
    u64 tcur = tp_on ? __builtin_readcyclecounter() : 0;
    auto tick = [&](int ph) {
        if (tp_on) {
            const u64 n = __builtin_readcyclecounter();
            tacc[ph] += n - tcur;
            tcur = n;
        }
    };
    // dbuf: the arena's two halves alternate -- while one group of slices is
    // placed and stored, the next group's spans are already being staged
    // into the other half; its wait counts only the loads, not the stores
    // issued after them (vmcnt counts both, in issue order: at least 2
    // store instructions per slice placed through the image follow them)
    constexpr int HALF = ARENA / 2;
    // longest span staged: a half of the arena under dbuf (a longer slice
    // copies per lane: at 128 chunks, halves of 1 KiB hold a 64-row slice of
    // C3's 13.9-byte strings)
    const int scap = dbuf ? (HALF < kStageChunks ? HALF : kStageChunks) : kStageChunks;
    int cur = 1;          // dbuf: the half holding slices (.., staged_to]
    int next_to = -1;     // dbuf: slices (staged_to, next_to] are being staged into the other half
    unsigned since = 0;   // dbuf: store instructions issued after those loads (a lower bound)
    // emit == 3: two slices' images assembled together (two images of DST/2
    // chunks): zeroing, placing and storing of a pair each pay one LDS round
    // trip instead of two; a slice waits for its partner while it is pending
    constexpr int IM = DST / 2;  // chunks per image in pairs mode
    bool pend = false;           // a slice placed-to-be in image 0 (uniform)
    int p_sh = 0, p_Ls = 0, p_nw = 0, p_off = 0;
    u8* p_w0 = nullptr;
    int p_a = 0, p_d = 0, p_L = 0;  // per lane: its string in the pending slice
    auto img_store = [&](const unsigned* im, u8* w0x, int shx, int Lsx, int nwx) {
        for (int j = lane; j < nwx; j += 64) {
            const unsigned val = im[j];
            const int p = 4 * j - shx;
            if (p >= 0 && p + 4 <= Lsx) {
                *at<unsigned>(w0x, 4 * j) = val;
            } else {
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    if (p + b >= 0 && p + b < Lsx) w0x[4 * j + b] = (u8)(val >> (8 * b));
            }
        }
    };
    auto flush_single = [&]() {  // the pending slice alone
        if (!pend) return;
        unsigned* im = gd;
        for (int c = lane; 4 * c < p_nw; c += 64) ((uint4*)im)[c] = make_uint4(0u, 0u, 0u, 0u);
        wave_lds_fence();
        if (p_L) utf8_place(gs + 4 * p_off, im, p_a, p_d, p_L);
        wave_lds_fence();
        img_store(im, p_w0, p_sh, p_Ls, p_nw);
        wave_lds_fence();
        since += 2;
        pend = false;
    };
    if (emit == 4)
        for (int c = lane; c < DST; c += 64) lds_zero128(G.dst + c);
    if (pre >= 0) {
        if (dbuf) {
            next_to = pre;  // prestaged into half 0 (cur ^ 1)
            staged_to = -1;
        } else {
            wait_vm_loads();
            wave_lds_fence();
        }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const u64 m = wm[k];
        if (!m) continue;
        tick(1);
        if (k > staged_to) {
            if (emit == 3) flush_single();  // the arena is about to be restaged
            if (e_pend) {
                if (e_since >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                else if (e_since >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
                else if (e_since >= 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
                else wait_vm_loads();
                staged_to = e_to;
                e_pend = false;
                aoff = 0;
            } else if (!dbuf) {
                staged_to = utf8_stage_group<K, ARENA>(src, wm, cs, cn, k, G.src, lane);
                wait_vm_loads();
                aoff = 0;
            } else {
                cur ^= 1;
                if (next_to >= k) {
                    staged_to = next_to;
                    if (since >= 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
                    else if (since >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                    else if (since >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                    else if (since >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
                    else wait_vm_loads();
                } else {
                    staged_to = utf8_stage_group<K, HALF>(src, wm, cs, cn, k, G.src + cur * HALF, lane, scap);
                    wait_vm_loads();
                }
                aoff = cur * HALF;
                next_to = -1;
                since = 0;
                if (staged_to + 1 < K) {
                    const int nt = utf8_stage_group<K, HALF>(src, wm, cs, cn, staged_to + 1, G.src + (cur ^ 1) * HALF, lane,
                                                             scap);
                    if (nt > staged_to) next_to = nt;
                }
            }
            wave_lds_fence();
        }
        tick(0);
        const bool sel = (selm >> k) & 1;
        const int e = utf8_end(s[k], nx[k], lane);
        const unsigned L = sel ? (unsigned)(e - s[k]) : 0u;
        const unsigned incl = wave_incl_scan32(L, lane);
        const unsigned rel = incl - L;
        const unsigned Ls = (unsigned)readlane_u(incl, 63);
        const u64 ob0 = bpre + T.excl[ch][(kb + k) * WAVES + wave];
        if (sel) A.out_offs[o][obase + dst[k]] = (int)(ob0 + rel);
        const i64 c0 = cs[k];
        const int nch = cn[k];
        const int my_off = aoff;
        if (nch <= scap) aoff += nch;
        if ((i64)(ob0 + Ls) > A.out_cap[o]) {
            if (lane == 0) report_err(A.err, 0, 0, ERRK_CAPACITY);
            continue;
        }
        if (Ls == 0) continue;
        // the slice's offset in G.dst: output address mod 4 (mod 16 for the
        // 16-byte image stores of emit 4)
        const int sh = (int)(((u64)out + ob0) & (emit == 4 ? 15u : 3u));
        // a span over the stage, or (LDS image) an output over the image: each lane copies its string
        if (nch > scap || ((emit == 1 || emit == 4) && DST >= 32 && ((sh + (int)Ls + 3) >> 2) > 4 * DST) ||
            (emit == 3 && ((sh + (int)Ls + 3) >> 2) > 4 * IM)) {
#if DFMI_LONG_COPY == 2
            if (emit == 1) {  // (the image holds nothing between this path's slices)
                wave_copy_slice(src, out + ob0, s[k], rel, L, lane, A.offs[u][A.n_rows], (int*)gd);
                continue;
            }
#endif
            if (sel && L) {
#if DFMI_LONG_COPY
                // long strings (Launch::long_copy): 64 bytes in flight per lane
                long_copy(src, s[k], out + ob0 + rel, L, A.offs[u][A.n_rows]);
#elif DFMI_LIGHT_COPY
                // the rare per-lane fallback, register-light (Launch::light_copy):
                // unaligned 16- and 4-byte moves, then the tail bytes
                light_copy(src + s[k], out + ob0 + rel, L);
#else
                utf8_copy(src + s[k], out + ob0 + rel, L);
#endif
            }
            continue;
        }
        u8* const w0 = out + ((i64)ob0 - sh);        // the aligned word (chunk) holding the slice's first byte
        if (emit == 2) {
            utf8_emit_slice_mk(gs + 4 * my_off, (int*)gd, (u8*)(gd + 128), w0, sh, sh + (int)Ls, incl, rel, L,
                               (int)(s[k] - c0), lane);
            continue;
        }
        if (emit == 0 || DST < 32) {
            utf8_emit_slice(gs + 4 * my_off, (int*)gd, w0, sh, sh + (int)Ls, incl, rel, (int)(s[k] - c0), lane);
            continue;
        }
        const int nw = (sh + (int)Ls + 3) >> 2;
        if (emit == 3) {
            if (!pend) {  // wait for a partner
                pend = true;
                p_sh = sh, p_Ls = (int)Ls, p_nw = nw, p_off = my_off, p_w0 = w0;
                p_a = (int)(s[k] - c0), p_d = sh + (int)rel, p_L = (int)L;
                continue;
            }
            unsigned* im0 = gd;
            unsigned* im1 = gd + 4 * IM;
            for (int c = lane; 4 * c < p_nw; c += 64) ((uint4*)im0)[c] = make_uint4(0u, 0u, 0u, 0u);
            for (int c = lane; 4 * c < nw; c += 64) ((uint4*)im1)[c] = make_uint4(0u, 0u, 0u, 0u);
            wave_lds_fence();
            if (p_L) utf8_place(gs + 4 * p_off, im0, p_a, p_d, p_L);
            if (L) utf8_place(gs + 4 * my_off, im1, (int)(s[k] - c0), sh + (int)rel, (int)L);
            wave_lds_fence();
            img_store(im0, p_w0, p_sh, p_Ls, p_nw);
            img_store(im1, w0, sh, (int)Ls, nw);
            wave_lds_fence();
            since += 4;
            pend = false;
            continue;
        }
        tick(1);
        if (emit != 4) {  // emit 4: the image is zero (zeroed at the start, and behind each slice's stores)
            for (int c = lane; 4 * c < nw; c += 64) G.dst[c] = make_uint4(0u, 0u, 0u, 0u);
            wave_lds_fence();
        }
        tick(2);
        if (L) utf8_place(gs + 4 * my_off, gd, (int)(s[k] - c0), sh + (int)rel, (int)L);
        wave_lds_fence();
        if (early && !dbuf && emit == 1 && k == staged_to && k + 1 < K) {
            // the arena's last slice is placed: stage the next group now
            const int nt = utf8_stage_group<K, ARENA>(src, wm, cs, cn, k + 1, G.src, lane);
            if (nt > k) {
                e_pend = true;
                e_to = nt;
                e_since = 0;
            }
        }
        tick(3);
        if (emit == 4) {
            utf8_image_store16(G.dst, w0, sh, (int)Ls, lane);
            wave_lds_fence();
            tick(4);
            since += 2;
            continue;
        }
        for (int j = lane; j < nw; j += 64) {
            const unsigned val = gd[j];
            const int p = 4 * j - sh;  // output position of the word's first byte
            if (p >= 0 && p + 4 <= (int)Ls) {
                *at<unsigned>(w0, 4 * j) = val;
            } else {
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    if (p + b >= 0 && p + b < (int)Ls) w0[4 * j + b] = (u8)(val >> (8 * b));
            }
        }
        wave_lds_fence();
        tick(4);
        since += 2;  // this slice's out_offs store and at least one image store
        if (e_pend) e_since += (unsigned)((nw + 63) >> 6);  // one store instruction per round at least
    }
    if (emit == 3) flush_single();
    if (tp_on && lane == 0)
#pragma unroll
        for (int i = 0; i < 5; ++i) atomicAdd(A.stats + 8 + i, tacc[i]);
}

// ------------------------------------------------ ring-staged Utf8 gather
// Launch::ring (numeric predicate, one Utf8 output, high selectivity): the
// tile's source bytes are streamed into LDS by ONE wave of the block ahead of
// use, and the block assembles and stores each step's output together.
// A step is the 256 rows base + k*BLOCK .. (one 64-row slice per wave); its
// source bytes [offs[base + k*BLOCK], offs[base + (k+1)*BLOCK]) are one
// contiguous span, and its selected strings one contiguous output range.
//   - Wave 0 (the loader) knows every step's span from its own offsets (lane
//     0 of its slice k starts step k) plus one load of the tile's end offset,
//     and issues direct global->LDS loads (global_load_lds_dwordx4, no VGPRs)
//     of steps 0..R-1 before the predicate, scan and look-back -- which then
//     hide them -- and of step k+R-1 as soon as step k-1's slot is free.
//   - Per step the block meets once (lds_sync): step k's bytes are in LDS
//     (the loader waited for them with a counted vmcnt, leaving the later
//     steps' loads in flight), every wave placed step k-1, so the block
//     stores step k-1's image -- 16-byte chunks, one or two store
//     instructions per thread -- and zeroes it while every lane places its
//     step-k string into the other image (utf8_place: interior words whole,
//     the two edge words OR-merged).
// No wave waits on its own staging round trips (round 4: 51% of the gather's
// cycles); a step whose span exceeds a slot or whose output exceeds an image
// copies per lane from global memory (utf8_copy).
template <int SLOT>  // 16-byte chunks per ring slot and per image
struct Utf8Ring {
    static constexpr int R = 3;  // ring slots: steps k .. k+2 staged or in flight
    uint4 src[R][SLOT];
    uint4 img[2][SLOT];   // step images, double-buffered; zero between uses
    int c0[16];           // per step: first source chunk (bytes from A.bytes[u], >= -15)
    int nch[16];          // per step: chunks of the span (0: no bytes)
};

// s_waitcnt vmcnt(n) for a wave-uniform n (the largest immediate <= n:
// waiting for more completions than needed is conservative).
__device__ __forceinline__ void wait_vm_at_most(int n) {
    if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (n >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (n >= 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else if (n >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if (n >= 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Load instructions of one staged step (64 chunks each); 0 when not staged.
template <int SLOT>
__device__ __forceinline__ int ring_loads(int nch) { return nch > 0 && nch <= SLOT ? (nch + 63) >> 6 : 0; }

// The loader's prologue (wave 0; call after utf8_offs_tile of the gathered
// column u): every step's span into G.c0 / G.nch, the first R steps issued.
// The values reach the other waves through the tile barrier (tile_offsets).
template <int BLOCK, int K, int SLOT>
__device__ __forceinline__ void ring_prologue(const Args& A, Utf8Ring<SLOT>& G, int u, i64 base, const int (&s)[K],
                                              int lane, int wave) {
    static_assert(K <= 16, "step table");
    for (int c = lane + 64 * wave; c < 2 * SLOT; c += BLOCK) lds_zero128(&G.img[0][0] + c);  // images start zero
    if (wave != 0) return;
    const u8* src = A.bytes[u];
    const int sm = (int)((u64)src & 15u);
    const i64 rend = base + BLOCK * K < A.n_rows ? base + BLOCK * K : A.n_rows;
    int b[K + 1];
#pragma unroll
    for (int k = 0; k < K; ++k) b[k] = __builtin_amdgcn_readlane(s[k], 0);  // offs[min(base + k*BLOCK, n)]
    b[K] = __builtin_amdgcn_readfirstlane(A.offs[u][rend]);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int c0 = (int)((((i64)b[k] + sm) & ~15ll) - sm);
        const int nc = b[k + 1] > b[k] ? (int)((((i64)b[k + 1] - 1 - c0) >> 4)) + 1 : 0;
        if (lane == 0) {
            G.c0[k] = c0;
            G.nch[k] = nc;
        }
        if (k < Utf8Ring<SLOT>::R && nc > 0 && nc <= SLOT) stage_span(at<uint4>(src, c0), G.src[k], nc, lane);
    }
}

// Bytes [lo, hi) of LDS chunk v (0 <= lo < hi <= 16) to the global chunk w
// (an edge chunk shared with another writer's bytes): whole words where the
// range covers them, single bytes at the ends; all stores back to back.
__device__ __forceinline__ void store_chunk_bytes(u8* w, uint4 v, int lo, int hi) {
    const unsigned x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int a = 4 * q > lo ? 4 * q : lo, b = 4 * q + 4 < hi ? 4 * q + 4 : hi;
        if (b - a == 4) {
            *at<unsigned>(w, 4 * q) = x[q];
        } else if (b > a) {
#pragma unroll
            for (int t = 0; t < 4; ++t)
                if (4 * q + t >= a && 4 * q + t < b) w[4 * q + t] = (u8)(x[q] >> (8 * t));
        }
    }
}

// Store a step image with the whole block (image byte 0 at the 16-byte
// aligned output address w0; valid bytes [lo, e): lo > 0 only inside chunk 0,
// the head of a range another writer's bytes precede), zeroing what it reads:
// whole chunks as 16-byte stores, a partial head chunk bytewise. A partial
// tail chunk -- its last bytes belong to the next step's output -- is carried
// into chunk 0 of the next step's image `nx` (OR-merged: the next step's
// strings only OR into the words it shares), or, without a next image (the
// tile's end, or a step that does not stage), stored bytewise.
template <int BLOCK>
__device__ __forceinline__ void ring_store(uint4* im, u8* w0, int lo, int e, uint4* nx, int tid) {
    const int full = e >> 4;  // chunks [0, full) end inside the range
    for (int c = tid; c < full; c += BLOCK) {
        const uint4 v = im[c];
        lds_zero128(im + c);
        if (c == 0 && lo > 0) store_chunk_bytes(w0, v, lo, 16);
        else *at<uint4>(w0, 16 * c) = v;
    }
    if ((e & 15) && tid == BLOCK - 1) {  // the partial tail chunk (another thread than chunk 0's, mostly)
        const uint4 v = im[full];
        lds_zero128(im + full);
        if (nx) {
            unsigned* d = (unsigned*)nx;
            lds_or(d, v.x);
            lds_or(d + 1, v.y);
            lds_or(d + 2, v.z);
            lds_or(d + 3, v.w);
        } else {
            store_chunk_bytes(w0 + 16 * full, v, full == 0 ? lo : 0, e & 15);
        }
    }
}

// The gather (all waves; after tile_offsets and the numeric outputs).
template <int BLOCK, int K, int NCH, int SLOT>
__device__ __forceinline__ void utf8_gather_ring(const Args& A, const Tile<BLOCK, K, NCH>& T, int ch, int u, int o,
                                                 unsigned selm, const unsigned (&dst)[K], const int (&s)[K],
                                                 const int (&nx)[K], Utf8Ring<SLOT>& G, int lane, int wave, int tid) {
    constexpr int WAVES = BLOCK / 64;
    constexpr int RR = Utf8Ring<SLOT>::R;
    constexpr int NW = K * WAVES;
    const u64 bpre = T.prefix[ch];
    const i64 obase = (i64)T.prefix[0];
    const u8* src = A.bytes[u];
    u8* out = A.out_data[o];
    // the image placed last (stored at the start of the next step): its
    // valid bytes [p_lo, p_e), image byte 0 at p_w0
    int p_img = -1, p_lo = 0, p_e = 0;
    u8* p_w0 = nullptr;
    int st_last = 0;  // loader: store instructions issued after the last refill (a lower bound)
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int nc = __builtin_amdgcn_readfirstlane(G.nch[k]);
        const int c0 = __builtin_amdgcn_readfirstlane(G.c0[k]);
        if (wave == 0) {
            // step k's loads are complete once at most the instructions issued
            // after them are outstanding: steps k+1's loads (and, at k = 0,
            // k+2's), then -- k >= 2: k+1 was the refill of iteration k-1 --
            // that iteration's stores (vmcnt counts loads and stores in order;
            // fewer than issued is conservative)
            int after = 0;
            if (k + 1 < K) after += ring_loads<SLOT>(__builtin_amdgcn_readfirstlane(G.nch[k + 1]));
            if (k == 0 && k + 2 < K) after += ring_loads<SLOT>(__builtin_amdgcn_readfirstlane(G.nch[k + 2]));
            if (k >= 2 && k + 1 < K) after += st_last;
            // (diagnostics, A.mode: bit 8 waits for everything, bit 9 not at all -- wrong bytes)
            if (A.mode & 256) after = 0;
            if (!(A.mode & 512)) wait_vm_at_most(after);
        }
        lds_sync();  // step k staged; every wave placed step k-1
        // the loader refills the slot step k-1 used (its placements are done)
        if (wave == 0 && k >= 1 && k + RR - 1 < K) {
            const int j = k + RR - 1;
            const int cj = __builtin_amdgcn_readfirstlane(G.c0[j]), nj = __builtin_amdgcn_readfirstlane(G.nch[j]);
            if (nj > 0 && nj <= SLOT) stage_span(at<uint4>(src, cj), G.src[j % RR], nj, lane);
        }
        // ---- this step's output range (uniform)
        const u64 st0 = T.excl[ch][k * WAVES];  // the step's first output byte (in the tile)
        const u64 st1 = k * WAVES + WAVES < NW ? T.excl[ch][(k + 1) * WAVES] : T.agg[ch];
        const int Ls = (int)(st1 - st0);
        const u64 O = bpre + st0;
        const bool cap_ok = (i64)(O + (u64)Ls) <= A.out_cap[o];
        const int sh = (int)(((u64)out + O) & 15u);
        const bool imaged = cap_ok && nc <= SLOT && sh + Ls <= 16 * SLOT;
        uint4* const im = G.img[k & 1];
        // ---- store the previous step's image; its partial tail chunk goes on
        // in this step's image (the output continues there) when this one has one
        int lo = sh;  // valid start of this image's chunk 0 (sh: nothing before it is ours)
        st_last = 0;
        if (p_img >= 0 && !(A.mode & 128)) {  // (mode bit 7: no image stores, diagnostics)
            ring_store<BLOCK>(G.img[p_img], p_w0, p_lo, p_e, imaged ? im : nullptr, tid);
            st_last += (p_e >> 4) > 0 ? ((p_e >> 4) - 1) / BLOCK + 1 : 0;  // chunk-loop rounds of wave 0
            if (imaged && (p_e & 15)) lo = (p_e >> 4) == 0 ? p_lo : 0;  // carried bytes start the chunk
        }
        p_img = -1;
        // ---- this step: offsets, then the strings into its image
        const bool sel = (selm >> k) & 1;
        const int e = utf8_end(s[k], nx[k], lane);
        const unsigned L = sel ? (unsigned)(e - s[k]) : 0u;
        const unsigned incl = wave_incl_scan32(L, lane);
        const unsigned rel = incl - L;
        const u64 ob = bpre + T.excl[ch][k * WAVES + wave] + rel;
        if (sel) A.out_offs[o][obase + dst[k]] = (int)ob;
        if (__ballot(sel)) ++st_last;
        if (!cap_ok) {
            if (tid == 0 && Ls) report_err(A.err, 0, 0, ERRK_CAPACITY);
            continue;
        }
        if (imaged) {
            if (L && !(A.mode & 64)) utf8_place((const unsigned*)G.src[k % RR], (unsigned*)im, s[k] - c0, sh + (int)(ob - O), (int)L);
            p_img = k & 1;
            p_lo = lo;
            p_e = sh + Ls;
            p_w0 = out + ((i64)O - sh);
        } else if (L) {  // not staged / over the image: each lane copies its string
            // (bytewise, register-light: the ring is chosen for short strings, so this is rare)
            const u8* sp = src + s[k];
            u8* dp = out + ob;
#pragma unroll 1
            for (unsigned i = 0; i < L; ++i) dp[i] = sp[i];
        }
    }
    lds_sync();
    if (p_img >= 0) ring_store<BLOCK>(G.img[p_img], p_w0, p_lo, p_e, nullptr, tid);
}

// Two-pass Utf8 gather, first pass (Launch::gather == 3): the rebased output
// offset and the source start of each selected row of Utf8 input u; the
// library's k_utf8_copy_rows (kernels.hip) then copies the bytes as a dense
// pass over the compacted rows -- lanes on consecutive output words, no
// per-string loops in the query kernel.
template <int BLOCK, int K, int NCH, int KT = K>
__device__ __forceinline__ void utf8_offsets_src(const Args& A, const Tile<BLOCK, KT, NCH>& T, int ch, int o,
                                                 unsigned selm, const u64 (&wm)[K], const unsigned (&dst)[K],
                                                 const int (&s)[K], const int (&nx)[K], int lane, int wave, int kb = 0) {
    constexpr int WAVES = BLOCK / 64;
    const u64 bpre = T.prefix[ch];
    const i64 obase = (i64)T.prefix[0];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        if (!wm[k]) continue;
        const bool sel = (selm >> k) & 1;
        const int e = utf8_end(s[k], nx[k], lane);  // every lane (DPP)
        const unsigned L = sel ? (unsigned)(e - s[k]) : 0u;
        const unsigned incl = wave_incl_scan32(L, lane);
        const u64 ob0 = bpre + T.excl[ch][(kb + k) * WAVES + wave];
        if (sel) {
            A.out_offs[o][obase + dst[k]] = (int)(ob0 + incl - L);
            A.out_src[o][obase + dst[k]] = s[k];
        }
        if (lane == 63 && (i64)(ob0 + incl) > A.out_cap[o]) report_err(A.err, 0, 0, ERRK_CAPACITY);
    }
}

// ------------------------------------------------ aggregate extension
// Fused Selection + Aggregate (no GROUP BY): every block reduces its tile's
// selected rows in registers / LDS and adds the block's partial into one of
// kAggCopies global accumulator copies (blockIdx % copies: atomics spread
// over many addresses); the host merges the copies exactly (aggregate.cpp).
// Accumulator words per aggregate: [0] non-null count, [1] flags, [2] MIN/MAX
// key, [3] wrapping integer sum, [4..] exact float sum digits.
constexpr int kAggCopies = 64;
constexpr int kAggLimbs = 68;                // 32-bit digits of the exact sum in units of 2^-1074, + carries
constexpr int kAggWords = 4 + kAggLimbs;
enum AggFlag : unsigned { AGGF_NAN = 1, AGGF_PINF = 2, AGGF_NINF = 4, AGGF_NONNEGZERO = 8, AGGF_VALUE = 16 };

// Order-preserving key of a MIN/MAX value (-0.0 below +0.0; NaN never keyed).
template <typename T>
__device__ __forceinline__ u64 agg_key(T v) {
    if constexpr (__is_same(T, float)) {
        const unsigned b = __builtin_bit_cast(unsigned, v);
        return (b >> 31) ? (u64)(~b) : (u64)(b | 0x80000000u);
    } else if constexpr (__is_same(T, double)) {
        const u64 b = __builtin_bit_cast(u64, v);
        return (b >> 63) ? ~b : (b | (1ull << 63));
    } else if constexpr ((T)-1 < (T)0) {
        return (u64)(i64)v ^ (1ull << 63);
    } else {
        return (u64)v;
    }
}

template <typename T>
__device__ __forceinline__ bool agg_isnan(T v) {
    if constexpr ((T)0.5 != (T)0) return v != v;
    else return false;
}

// Flag bits of one SUM input value (floats): NaN, +inf, -inf, "not -0.0".
template <typename T>
__device__ __forceinline__ unsigned agg_sum_flags(T v) {
    if constexpr ((T)0.5 != (T)0) {
        if (v != v) return AGGF_NAN;
        if (__builtin_isinf(v)) return v > 0 ? AGGF_PINF : AGGF_NINF;
        return (v == 0 && __builtin_signbit(v)) ? 0u : AGGF_NONNEGZERO;
    } else {
        return 0u;
    }
}

template <int CTRL, int ROWS>
__device__ __forceinline__ unsigned dpp32_id(unsigned v, unsigned id) {
    return __builtin_amdgcn_update_dpp(id, v, CTRL, ROWS, 0xf, false);
}

// Wave-wide min / max of u64 (uniform result; all lanes active).
template <bool MIN>
__device__ __forceinline__ u64 wave_minmax(u64 v) {
    const unsigned id = MIN ? ~0u : 0u;
#define DFMI_MM_STEP(C, R)                                                                  \
    {                                                                                       \
        const u64 o = ((u64)dpp32_id<C, R>((unsigned)(v >> 32), id) << 32) |                \
                      dpp32_id<C, R>((unsigned)v, id);                                      \
        v = MIN ? (o < v ? o : v) : (o > v ? o : v);                                        \
    }
    DFMI_MM_STEP(0x111, 0xf) DFMI_MM_STEP(0x112, 0xf) DFMI_MM_STEP(0x114, 0xf)
    DFMI_MM_STEP(0x118, 0xf) DFMI_MM_STEP(0x142, 0xa) DFMI_MM_STEP(0x143, 0xc)
#undef DFMI_MM_STEP
    return readlane_u64(v, 63);
}

// Block-level (LDS) state of NA aggregates, NF of them exact float sums.
template <int NA, int NF>
struct AggLds {
    u64 count[NA];
    u64 isum[NA];
    u64 key[NA];
    unsigned flags[NA];
    long long limbs[NF > 0 ? NF : 1][kAggLimbs];
    int dlo[NF > 0 ? NF : 1], dhi[NF > 0 ? NF : 1];
};

template <int NA, int NF>
__device__ __forceinline__ void agg_lds_init(AggLds<NA, NF>& S, const unsigned char (&is_min)[NA > 0 ? NA : 1], int tid) {
    for (int i = tid; i < NA; i += 64) {
        S.count[i] = 0;
        S.isum[i] = 0;
        S.key[i] = is_min[i] ? ~0ull : 0ull;
        S.flags[i] = 0;
    }
    for (int i = tid; i < NF * kAggLimbs; i += 64) (&S.limbs[0][0])[i] = 0;
    for (int i = tid; i < NF; i += 64) {
        S.dlo[i] = 0x7fffffff;
        S.dhi[i] = -1;
    }
}

// Exact float sum: this wave's `ok` values (finite, non-zero) added into the
// block's 32-bit-digit accumulator. A double is m * 2^(b-1074) (m < 2^53,
// b = biased exponent - 1, subnormals b = 0): digits d = b/32 .. d+2 receive
// the three 32-bit pieces of m << (b % 32), signed. When every value of the
// wave falls on the same digit (the common case) the wave sums the pieces
// first and one lane adds three words; otherwise each lane adds its own.
__device__ __forceinline__ void fsum_add(long long* limbs, int* dlo, int* dhi, double v, bool ok, int lane) {
    const u64 vm = __ballot(ok);
    if (!vm) return;
    const u64 b = __builtin_bit_cast(u64, v);
    const int e = (int)((b >> 52) & 0x7ff);
    const u64 m = (b & ((1ull << 52) - 1)) | (e ? (1ull << 52) : 0ull);
    const int pos = (e ? e : 1) - 1;
    const int d = pos >> 5, sh = pos & 31;
    const u64 x0 = (m & 0xffffffffull) << sh, x1 = (m >> 32) << sh;
    long long c0 = (long long)(x0 & 0xffffffffull);
    long long c1 = (long long)((x0 >> 32) + (x1 & 0xffffffffull));
    long long c2 = (long long)(x1 >> 32);
    if (b >> 63) {
        c0 = -c0;
        c1 = -c1;
        c2 = -c2;
    }
    if (!ok) c0 = c1 = c2 = 0;
    const int d0 = __builtin_amdgcn_readlane(d, __builtin_ctzll(vm));
    if (!__ballot(ok && d != d0)) {
        const u64 s0 = wave_sum((u64)c0), s1 = wave_sum((u64)c1), s2 = wave_sum((u64)c2);
        if (lane == 0) {
            atomicAdd((unsigned long long*)&limbs[d0], (unsigned long long)s0);
            atomicAdd((unsigned long long*)&limbs[d0 + 1], (unsigned long long)s1);
            atomicAdd((unsigned long long*)&limbs[d0 + 2], (unsigned long long)s2);
            atomicMin(dlo, d0);
            atomicMax(dhi, d0 + 2);
        }
    } else if (ok) {
        atomicAdd((unsigned long long*)&limbs[d], (unsigned long long)c0);
        atomicAdd((unsigned long long*)&limbs[d + 1], (unsigned long long)c1);
        atomicAdd((unsigned long long*)&limbs[d + 2], (unsigned long long)c2);
        atomicMin(dlo, d);
        atomicMax(dhi, d + 2);
    }
}

// One wave's per-lane partials of aggregate j into the block state.
template <int NA, int NF>
__device__ __forceinline__ void agg_wave_flush(AggLds<NA, NF>& S, int j, unsigned cnt, u64 isum, u64 key, bool is_min,
                                               unsigned flags, int lane) {
    const u64 c = wave_sum((u64)cnt), s = wave_sum(isum);
    const u64 k = is_min ? wave_minmax<true>(key) : wave_minmax<false>(key);
    unsigned f = 0;
#pragma unroll
    for (int bit = 0; bit < 5; ++bit) f |= __ballot((flags >> bit) & 1) ? (1u << bit) : 0u;
    if (lane == 0) {
        if (c) atomicAdd((unsigned long long*)&S.count[j], (unsigned long long)c);
        if (s) atomicAdd((unsigned long long*)&S.isum[j], (unsigned long long)s);
        if (is_min) atomicMin((unsigned long long*)&S.key[j], (unsigned long long)k);
        else atomicMax((unsigned long long*)&S.key[j], (unsigned long long)k);
        if (f) atomicOr(&S.flags[j], f);
    }
}

// The block's state into global copy blockIdx % kAggCopies (after a block
// barrier). The float digits are carry-normalised first (every digit but the
// top one in [0, 2^32)), so a global digit absorbs 2^31 block partials.
template <int NA, int NF>
__device__ __forceinline__ void agg_block_flush(const Args& A, AggLds<NA, NF>& S, const int (&fslot)[NF > 0 ? NF : 1],
                                                const unsigned char (&is_min)[NA > 0 ? NA : 1], int tid,
                                                u64* base_ = nullptr) {
    u64* base = base_ ? base_ : A.agg + (u64)(blockIdx.x % kAggCopies) * NA * kAggWords;
    if (tid < NA) {
        u64* w = base + tid * kAggWords;
        if (S.count[tid]) atomicAdd((unsigned long long*)&w[0], (unsigned long long)S.count[tid]);
        if (S.flags[tid]) atomicOr((unsigned long long*)&w[1], (unsigned long long)S.flags[tid]);
        if (S.flags[tid] & AGGF_VALUE) {
            if (is_min[tid]) atomicMin((unsigned long long*)&w[2], (unsigned long long)S.key[tid]);
            else atomicMax((unsigned long long*)&w[2], (unsigned long long)S.key[tid]);
        }
        if (S.isum[tid]) atomicAdd((unsigned long long*)&w[3], (unsigned long long)S.isum[tid]);
    }
    if constexpr (NF > 0) {
        if (tid >= 64 && tid < 64 + NF) {  // one lane per float sum, in another wave
            const int f = tid - 64;
            const int lo = S.dlo[f], hi = S.dhi[f];
            if (hi >= 0) {
                long long* L = S.limbs[f];
                const int top = hi + 2 < kAggLimbs - 1 ? hi + 2 : kAggLimbs - 1;
                for (int i = lo; i < top; ++i) {
                    const long long c = L[i] >> 32;  // arithmetic: floor division by 2^32
                    L[i] -= c * 4294967296ll;
                    L[i + 1] += c;
                }
                u64* w = base + fslot[f] * kAggWords + 4;
                for (int i = lo; i <= top; ++i)
                    if (L[i]) atomicAdd((unsigned long long*)&w[i], (unsigned long long)L[i]);
            }
        }
    }
}

}  // namespace dfmi

#endif  // DFMI_SKELETON
