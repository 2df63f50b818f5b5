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
};

// This block's share of zeroing the previous launch's workspace.
template <int BLOCK>
__device__ __forceinline__ void clear_previous(const Args& A, unsigned block, int tid) {
    const i64 per = (A.clear_words + A.n_tiles - 1) / A.n_tiles;
    const i64 w0 = (i64)block * per;
    const i64 w1 = w0 + per < A.clear_words ? w0 + per : A.clear_words;
    for (i64 w = w0 + tid; w < w1; w += BLOCK) A.clear_status[w] = 0;
    if (block == 0 && tid < 64) A.clear_hdr[tid] = 0;
}

enum ErrKind : unsigned { ERRK_DIV_ZERO = 1, ERRK_DIV_OVERFLOW = 2, ERRK_LOOKBACK_TIMEOUT = 3, ERRK_CAPACITY = 4 };

constexpr u64 FLAG_A = 1ull << 62;
constexpr u64 FLAG_P = 2ull << 62;
constexpr u64 VAL_MASK = (1ull << 62) - 1;

__device__ __forceinline__ double f64(u64 x) { return __builtin_bit_cast(double, x); }
__device__ __forceinline__ u64 bits(double x) { return __builtin_bit_cast(u64, x); }
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ unsigned lane_rank(u64 mask) {  // set bits below this lane
    return __builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
}

__device__ __forceinline__ u64 wave_sum(u64 v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ u64 wave_incl_scan(u64 v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const u64 t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

__device__ __forceinline__ unsigned wave_incl_scan32(unsigned v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

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
        }
        out = (To)x;
        return true;
    }
}

// Rows past n_rows (the tail tile) read nothing: the callers mask them out.
__device__ __forceinline__ bool utf8_eq_lit(const Args& A, int u, i64 row, int lit) {
    if (row >= A.n_rows) return false;
    const int s = A.offs[u][row], e = A.offs[u][row + 1];
    const int len = A.str_len[lit];
    if (e - s != len) return false;
    const u8* p = A.bytes[u] + s;
    const char* q = A.str + A.str_off[lit];
    // early exit: most equal-length candidates differ within the first bytes
    // (filtered tiles use utf8_eq_lit_tile below)
    for (int i = 0; i < len; ++i)
        if (p[i] != (u8)q[i]) return false;
    return true;
}

// `utf8 column u = literal` for the K rows base + k*BLOCK + tid of a tile.
// Per-row early-exit compares serialise one memory latency per k; here every
// row's offsets, then the first min(len, 4) bytes of every equal-length
// candidate, are in flight together, and only head matches (rare) compare
// the rest. Rows past n_rows read nothing and compare false.
template <int BLOCK, int K>
__device__ __forceinline__ void utf8_eq_lit_tile(const Args& A, int u, i64 base, int tid, int lit, bool (&res)[K]) {
    const int len = A.str_len[lit];
    const char* q = A.str + A.str_off[lit];
    const int* off = A.offs[u];
    const u8* by = A.bytes[u];
    int s[K], e[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const i64 row = base + (i64)k * BLOCK + tid;
        const bool in = row < A.n_rows;
        s[k] = in ? off[row] : 0;
        e[k] = in ? off[row + 1] : -1;
    }
    const int hn = len < 4 ? len : 4;
    unsigned qh = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (i < hn) qh |= (unsigned)(u8)q[i] << (8 * i);
    unsigned h[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        unsigned w = ~qh;
        if (e[k] - s[k] == len) {
            const u8* p = by + s[k];
            w = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (i < hn) w |= (unsigned)p[i] << (8 * i);
        }
        h[k] = w;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        bool eq = e[k] - s[k] == len && h[k] == qh;
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
    unsigned polls = 0, sleeps = 0;
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
            } else if (now - t0 > 200000000ull) {
                // 2 s without a single predecessor resolving (a preempted or
                // time-sliced GPU is far below this): report, do not hang
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
    static_assert(NW <= 64, "one wave scans the tile's words");
    u64 cnt[NCH][NW];
    u64 excl[NCH][NW];
    u64 prefix[NCH];
    u64 agg[NCH];
};

// counts[ch][k] : per-lane value for row k (rows: 0/1 selection, Utf8: bytes)
// First half of the tile step: per-(k, wave) counts, the one-wave scan of the
// tile's words and the publication of the tile aggregate (no waiting).
template <int BLOCK, int K, int NCH, int SPREAD = 1>
__device__ __forceinline__ void tile_scan_publish(const Args& A, Tile<BLOCK, K, NCH>& T, unsigned tile,
                                                  const unsigned (&cnt)[NCH][K], int lane, int wave) {
    constexpr int WAVES = BLOCK / 64;
    constexpr int NW = K * WAVES;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch)
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const u64 s = ch == 0 ? (u64)__builtin_popcountll(__ballot(cnt[0][k] != 0)) : wave_sum((u64)cnt[ch][k]);
            if (lane == 0) T.cnt[ch][k * WAVES + wave] = s;
        }
    lds_sync();
    if (wave == 0) {
        u64 packed = 0;
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
            const u64 c = lane < NW ? T.cnt[ch][lane] : 0ull;
            const u64 incl = wave_incl_scan(c, lane);
            if (lane < NW) T.excl[ch][lane] = incl - c;
            const u64 agg = __shfl(incl, NW - 1, 64);
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
    const u64 sa = (u64)src, da = (u64)dst;
    const u64 sw0 = sa & ~3ull, swl = (sa + L - 1) & ~3ull;
    const u64 dw0 = da & ~3ull, dwe = (da + L + 3) & ~3ull;
    for (u64 wb = dw0; wb < dwe; wb += 32) {
        const i64 sb = (i64)sa + ((i64)wb - (i64)da);  // source address of output byte wb
        const u64 sbw = (u64)sb & ~3ull;
        const unsigned sh = (unsigned)sb & 3u;
        unsigned sv[9];
#pragma unroll
        for (int j = 0; j < 9; ++j) {
            u64 a = sbw + 4ull * j;
            a = a < sw0 ? sw0 : (a > swl ? swl : a);
            sv[j] = *(const unsigned*)a;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const u64 w = wb + 4ull * j;
            if (w >= dwe) break;
            const unsigned val = __builtin_amdgcn_alignbyte(sv[j + 1], sv[j], sh);
            const i64 p = (i64)w - (i64)da;  // offset of the word's first byte in dst
            if (p >= 0 && p + 4 <= (i64)L) {
                *(unsigned*)w = val;
            } else {
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    if (p + b >= 0 && p + b < (i64)L) ((u8*)w)[b] = (u8)(val >> (8 * b));
            }
        }
    }
}

// Copy the selected rows of Utf8 input u into output o (rebased i32
// offsets + bytes, filter.rs:94-105).
template <int BLOCK, int K, int NCH>
__device__ __forceinline__ void utf8_gather(const Args& A, const Tile<BLOCK, K, NCH>& T, int ch, int u, int o,
                                            i64 base, unsigned selm, const unsigned (&len)[K],
                                            const unsigned (&dst)[K], int lane, int wave) {
    constexpr int WAVES = BLOCK / 64;
    const u64 bpre = T.prefix[ch];
    const i64 obase = (i64)T.prefix[0];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const unsigned incl = wave_incl_scan32(len[k], lane);
        if (!((selm >> k) & 1)) continue;
        const i64 row = base + (i64)k * BLOCK + threadIdx.x;
        const u64 ob = bpre + T.excl[ch][k * WAVES + wave] + (incl - len[k]);
        A.out_offs[o][obase + dst[k]] = (int)ob;
        if ((i64)(ob + len[k]) > A.out_cap[o]) {
            report_err(A.err, 0, 0, ERRK_CAPACITY);
            continue;
        }
        const unsigned L = len[k];
        if (L == 0) continue;
        utf8_copy(A.bytes[u] + A.offs[u][row], A.out_data[o] + ob, L);
    }
}

}  // namespace dfmi

#endif  // DFMI_SKELETON
