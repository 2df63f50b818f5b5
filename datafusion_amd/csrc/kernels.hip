// CDNA4 (gfx950) kernels of the Selection + Projection path.
//
//   k_filter_project   one pass: load referenced columns (each row read once),
//                      evaluate the predicate program, wave64 __ballot -> row
//                      bitmap words, block scan, single-pass decoupled
//                      look-back for the tile's global output offset (rows and
//                      Utf8 bytes), then evaluate/gather every projection and
//                      store selected rows compacted, in row order.
//                      Replaces FilterRelation::next + filter() +
//                      ProjectRelation::next (filter.rs:46-111,
//                      projection.rs:45-66) and the array_ops passes under them.
//   k_project          no Selection: elementwise programs, ballot-packed
//                      validity / Boolean bitmaps (ProjectRelation::next alone).
//   k_pack_bools       byte-per-row -> LSB-first bitmap for Boolean outputs of
//                      a filtered projection.
//   k_gen_*            counter-based synthetic columns (bench inputs).
//
// Must be compiled with -ffp-contract=off: Float64 math rounds once per
// operator, as the reference's scalar loops do.
#include <hip/hip_runtime.h>

#include "dfmi_internal.h"

namespace dfmi {

typedef unsigned long long u64;
typedef long long i64;

constexpr int BLOCK = 256;
constexpr int WAVES = BLOCK / 64;
constexpr u64 FLAG_A = 1ull << 62;
constexpr u64 FLAG_P = 2ull << 62;
constexpr u64 VAL_MASK = (1ull << 62) - 1;

template <int NS>
struct Slots;
template <>
struct Slots<8> { typedef u64 type __attribute__((ext_vector_type(8))); };
template <>
struct Slots<16> { typedef u64 type __attribute__((ext_vector_type(16))); };

__device__ __forceinline__ double as_f64(u64 x) { return __builtin_bit_cast(double, x); }
__device__ __forceinline__ u64 as_u64(double x) { return __builtin_bit_cast(u64, x); }
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ unsigned lane_rank(u64 mask) {  // set bits below this lane
    return __builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
}

__device__ __forceinline__ u64 wave_sum(u64 v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ u64 wave_incl_scan(u64 v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        u64 t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

__device__ __forceinline__ unsigned wave_incl_scan32(unsigned v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        unsigned t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

// 64 bits of an LSB-first bitmap starting at bit 64*w (w wave-uniform).
// The tail word is assembled bytewise so nothing past bitmap_bytes is read.
__device__ __forceinline__ u64 bitmap_word(const uint8_t* bm, i64 w, i64 nbytes) {
    const i64 b0 = w * 8;
    if (b0 + 8 <= nbytes) return *(const u64*)(bm + b0);
    u64 v = 0;
    for (i64 i = b0; i < nbytes; ++i) v |= (u64)bm[i] << (8 * (i - b0));
    return v;
}

__device__ __forceinline__ void report_err(u64* err, u64 ordinal, u64 row, u64 kind) {
    const u64 key = (ordinal << 44) | (row << 4) | kind;
    atomicMax(err, ~key);
}

__device__ __forceinline__ void st_status(u64* p, u64 v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 ld_status(u64* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Single-pass decoupled look-back (one wave). Publishes the tile aggregate,
// then reads the status words of up to 256 predecessors per round trip (4 per
// lane), summing aggregates until an inclusive prefix is found; publishes its
// own inclusive prefix and returns the exclusive one. Tiles are numbered by a
// dynamic ticket, so every predecessor is already running and the spin ends;
// it is bounded in wall time anyway (error word, never a hang).
constexpr int LB_Q = 4;
__device__ u64 lookback(u64* st, unsigned tile, u64 agg, int lane, u64* err, bool* timeout) {
    if (tile == 0) {
        if (lane == 0) st_status(st, FLAG_P | agg);
        return 0;
    }
    if (lane == 0) st_status(st + tile, FLAG_A | agg);
    u64 excl = 0;
    i64 j = (i64)tile - 1;  // nearest unresolved predecessor
    const u64 t_start = __builtin_amdgcn_s_memrealtime();  // 100 MHz
    while (true) {
        u64 w[LB_Q];
#pragma unroll
        for (int q = 0; q < LB_Q; ++q) {
            const i64 idx = j - q * 64 - lane;
            w[q] = idx >= 0 ? ld_status(st + idx) : FLAG_P;
        }
        bool done = false;
#pragma unroll
        for (int q = 0; q < LB_Q; ++q) {
            const unsigned flag = (unsigned)(w[q] >> 62);
            const u64 xm = __ballot(flag == 0);
            const u64 pm = __ballot(flag == 2);
            if (pm) {
                const int first = __builtin_ctzll(pm);
                const u64 need = first == 63 ? ~0ull : ((2ull << first) - 1);
                if (xm & need) break;  // a predecessor before the prefix is not ready
                excl += wave_sum(lane <= first ? (w[q] & VAL_MASK) : 0);
                done = true;
                break;
            }
            if (xm) break;
            excl += wave_sum(w[q] & VAL_MASK);  // 64 aggregates, keep going back
            j -= 64;
        }
        if (done) break;
        if (__builtin_amdgcn_s_memrealtime() - t_start > 50000000ull) {  // 0.5 s
            if (lane == 0) report_err(err, 0, 0, ERRK_LOOKBACK_TIMEOUT);
            *timeout = true;
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    if (lane == 0) st_status(st + tile, FLAG_P | (excl + agg));
    return excl;
}

// ------------------------------------------------------- interpreter ---
// Per-thread state for the K rows a thread owns in a tile. Column operands are
// NOT kept in registers: every column fetch is a global load of the thread's
// K rows (repeat fetches of a column within a tile hit L1/L2, HBM sees each
// line once), so the register footprint stays small and occupancy high.
template <int BLOCK_, int K_, bool NULLABLE_>
struct Cfg {
    static constexpr int BLOCK = BLOCK_;
    static constexpr int K = K_;
    static constexpr int TILE = BLOCK_ * K_;
    static constexpr int WAVES = BLOCK_ / 64;
    static constexpr bool NULLABLE = NULLABLE_;
};

template <class C>
struct State {
    u64 acc[C::K];
    unsigned accv;       // accumulator validity bits (bit k)
    unsigned tv[C::K];   // temporary validity bits
    unsigned bv[C::K];   // bool slot value bits
    unsigned bvd[C::K];  // bool slot validity bits
    unsigned actm;       // bit k: row k is evaluated (errors only count there)
    unsigned ldst[C::K]; // output row relative to obase (compacted or dense)
    i64 base;            // first row of the tile (wave-uniform)
    i64 obase;           // first output row of the tile (wave-uniform)
    int tid, lane, wave;
    bool cols_valid;     // columns read as all-valid (after a Selection)
    bool dense;          // projection-only kernel: ballot-packed bitmaps
    __device__ bool act(int k) const { return (actm >> k) & 1; }
    __device__ unsigned lrow(int k) const { return (unsigned)(k * C::BLOCK + tid); }
    __device__ i64 row(int k) const { return base + (i64)lrow(k); }
    __device__ i64 word(int k) const { return (base + (i64)k * C::BLOCK + wave * 64) >> 6; }
};

template <int OP, typename T>
__device__ __forceinline__ bool cmp_val(T x, T y) {
    if constexpr (OP == 0) return x == y;
    else if constexpr (OP == 1) return x != y;
    else if constexpr (OP == 2) return x < y;
    else if constexpr (OP == 3) return x <= y;
    else if constexpr (OP == 4) return x > y;
    else return x >= y;
}

// arrow 0.12 bool_op on Option<T>: eq/neq compare Options, lt/le: (None,_)
// => true, (_,None) => false; gt/ge: (None,_) => false, (_,None) => true.
template <int OP>
__device__ __forceinline__ bool cmp_null(bool lv, bool rv, bool res) {
    if (lv && rv) return res;
    if constexpr (OP == 0) return !lv && !rv;
    else if constexpr (OP == 1) return !(!lv && !rv);
    else if constexpr (OP == 2 || OP == 3) return !lv;
    else return lv;
}

// Operand fetch for the thread's K rows; kind and index are wave-uniform.
template <class C>
__device__ __forceinline__ void fetch(const State<C>& S, const DLaunch& L, int kind, int idx,
                                      const u64* stage, const u64* tmp, u64 (&x)[C::K], bool (&v)[C::K]) {
    constexpr int K = C::K;
    if (kind == KD_COL) {
        if (idx < L.n_lds) {  // staged in LDS by DMA (stage_tile)
            const u64* p = stage + idx * C::TILE;
#pragma unroll
            for (int k = 0; k < K; ++k) x[k] = p[S.lrow(k)];
        } else {
            const u64* p = (const u64*)L.num[idx].values + S.base;  // uniform tile base
#pragma unroll
            for (int k = 0; k < K; ++k) x[k] = S.act(k) ? p[S.lrow(k)] : 0ull;
        }
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = true;
        if constexpr (C::NULLABLE) {
            const uint8_t* vb = L.num[idx].validity;
            if (vb && !S.cols_valid) {
#pragma unroll
                for (int k = 0; k < K; ++k)
                    v[k] = (bitmap_word(vb, S.word(k), L.num[idx].bitmap_bytes) >> S.lane) & 1;
            }
        }
    } else if (kind == KD_LIT) {
        const u64 l = L.lits[idx];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            x[k] = l;
            v[k] = true;
        }
    } else if (kind == KD_ACC) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            x[k] = S.acc[k];
            v[k] = C::NULLABLE ? ((S.accv >> k) & 1) : true;
        }
    } else {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            x[k] = tmp[(idx * K + k) * C::BLOCK + S.tid];
            v[k] = C::NULLABLE ? ((S.tv[k] >> idx) & 1) : true;
        }
    }
}

template <class C, bool EQ>
__device__ __forceinline__ void do_utf8_lit(State<C>& S, const DLaunch& L, const DIns in) {
    const DCol& c = L.utf8[in.a];
    const int loff = L.strlit_off[in.b], llen = L.strlit_len[in.b];
    const uint8_t* bytes = (const uint8_t*)c.values;
    const int d = in.dst;
#pragma unroll
    for (int k = 0; k < C::K; ++k) {
        bool eq = false, valid = true;
        if (S.act(k)) {
            const i64 r = S.row(k);
            const int s = c.offsets[r], e = c.offsets[r + 1];
            eq = (e - s) == llen;
            for (int i = 0; eq && i < llen; ++i) eq = bytes[s + i] == (uint8_t)L.strlit[loff + i];
            if constexpr (C::NULLABLE) {
                if (c.validity && !S.cols_valid) valid = (c.validity[r >> 3] >> (r & 7)) & 1;
            }
        }
        // Some(x) == Some(lit); None == Some(lit) -> false
        const bool res = EQ ? (valid && eq) : !(valid && eq);
        S.bv[k] = (S.bv[k] & ~(1u << d)) | ((unsigned)res << d);
        S.bvd[k] |= 1u << d;
    }
}

template <class C, bool EQ>
__device__ __forceinline__ void do_utf8_col(State<C>& S, const DLaunch& L, const DIns in) {
    const DCol& c0 = L.utf8[in.a];
    const DCol& c1 = L.utf8[in.b];
    const uint8_t* b0 = (const uint8_t*)c0.values;
    const uint8_t* b1 = (const uint8_t*)c1.values;
    const int d = in.dst;
#pragma unroll
    for (int k = 0; k < C::K; ++k) {
        bool eq = false, v0 = true, v1 = true;
        if (S.act(k)) {
            const i64 r = S.row(k);
            const int s0 = c0.offsets[r], e0 = c0.offsets[r + 1];
            const int s1 = c1.offsets[r], e1 = c1.offsets[r + 1];
            eq = (e0 - s0) == (e1 - s1);
            for (int i = 0; eq && i < e0 - s0; ++i) eq = b0[s0 + i] == b1[s1 + i];
            if constexpr (C::NULLABLE) {
                if (!S.cols_valid) {
                    if (c0.validity) v0 = (c0.validity[r >> 3] >> (r & 7)) & 1;
                    if (c1.validity) v1 = (c1.validity[r >> 3] >> (r & 7)) & 1;
                }
            }
        }
        const bool oeq = (v0 && v1) ? eq : (!v0 && !v1);
        const bool res = EQ ? oeq : !oeq;
        S.bv[k] = (S.bv[k] & ~(1u << d)) | ((unsigned)res << d);
        S.bvd[k] |= 1u << d;
    }
}

template <int OP, bool F64, int K>
__device__ __forceinline__ void cmp_rows(const u64 (&x)[K], const u64 (&y)[K], bool (&res)[K]) {
#pragma unroll
    for (int k = 0; k < K; ++k)
        res[k] = F64 ? cmp_val<OP>(as_f64(x[k]), as_f64(y[k])) : cmp_val<OP>((i64)x[k], (i64)y[k]);
}

template <int OP, int K>
__device__ __forceinline__ void cmp_nulls(const bool (&vx)[K], const bool (&vy)[K], bool (&res)[K]) {
#pragma unroll
    for (int k = 0; k < K; ++k) res[k] = cmp_null<OP>(vx[k], vy[k], res[k]);
}

// arrow 0.12 math_op: null if either side is null (slot value 0), Int64
// wraps (Rust release), Divide: non-null zero divisor -> DivideByZero,
// i64::MIN / -1 -> panic. Float64: one IEEE rounding (no contraction).
// Out of line: the software 64-bit division is ~60 instructions and ~20
// VGPRs; inlined K times it dominated the kernel's register allocation.
__device__ __noinline__ u64 sdiv64(u64 x, u64 y) {
    const i64 sx = (i64)x, sy = (i64)y;
    if (sy == 0) return 0;
    if (sy == -1) return 0ull - x;  // wraps; MIN / -1 is reported
    return (u64)(sx / sy);
}

template <int OP, bool F64>
__device__ __forceinline__ u64 math_val(u64 x, u64 y) {
    if constexpr (F64) {
        const double fx = as_f64(x), fy = as_f64(y);
        if constexpr (OP == 0) return as_u64(fx + fy);
        else if constexpr (OP == 1) return as_u64(fx - fy);
        else if constexpr (OP == 2) return as_u64(fx * fy);
        else return as_u64(fx / fy);
    } else {
        if constexpr (OP == 0) return x + y;
        else if constexpr (OP == 1) return x - y;
        else if constexpr (OP == 2) return x * y;
        else return sdiv64(x, y);
    }
}

template <class C>
__device__ void run_program(State<C>& S, const DLaunch& L, int begin, int end, const u64* stage,
                            u64* tmp) {
    constexpr int K = C::K;
    for (int i = begin; i < end; ++i) {
        const DIns in = L.ins[i];
        const int op = in.op;
        if (op <= OP_DIV_F64) {  // numeric binary: comparison or math
            u64 x[K], y[K];
            bool vx[K], vy[K];
            fetch<C>(S, L, in.ka, in.a, stage, tmp, x, vx);
            fetch<C>(S, L, in.kb, in.b, stage, tmp, y, vy);
            if (op <= OP_GE_F64) {
                bool res[K];
                switch (op) {
                    case OP_EQ_I64: cmp_rows<0, false>(x, y, res); if (C::NULLABLE) cmp_nulls<0>(vx, vy, res); break;
                    case OP_NE_I64: cmp_rows<1, false>(x, y, res); if (C::NULLABLE) cmp_nulls<1>(vx, vy, res); break;
                    case OP_LT_I64: cmp_rows<2, false>(x, y, res); if (C::NULLABLE) cmp_nulls<2>(vx, vy, res); break;
                    case OP_LE_I64: cmp_rows<3, false>(x, y, res); if (C::NULLABLE) cmp_nulls<3>(vx, vy, res); break;
                    case OP_GT_I64: cmp_rows<4, false>(x, y, res); if (C::NULLABLE) cmp_nulls<4>(vx, vy, res); break;
                    case OP_GE_I64: cmp_rows<5, false>(x, y, res); if (C::NULLABLE) cmp_nulls<5>(vx, vy, res); break;
                    case OP_EQ_F64: cmp_rows<0, true>(x, y, res); if (C::NULLABLE) cmp_nulls<0>(vx, vy, res); break;
                    case OP_NE_F64: cmp_rows<1, true>(x, y, res); if (C::NULLABLE) cmp_nulls<1>(vx, vy, res); break;
                    case OP_LT_F64: cmp_rows<2, true>(x, y, res); if (C::NULLABLE) cmp_nulls<2>(vx, vy, res); break;
                    case OP_LE_F64: cmp_rows<3, true>(x, y, res); if (C::NULLABLE) cmp_nulls<3>(vx, vy, res); break;
                    case OP_GT_F64: cmp_rows<4, true>(x, y, res); if (C::NULLABLE) cmp_nulls<4>(vx, vy, res); break;
                    default:        cmp_rows<5, true>(x, y, res); if (C::NULLABLE) cmp_nulls<5>(vx, vy, res); break;
                }
                const int d = in.dst;
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    S.bv[k] = (S.bv[k] & ~(1u << d)) | ((unsigned)res[k] << d);
                    S.bvd[k] |= 1u << d;
                }
            } else {
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const bool v = C::NULLABLE ? (vx[k] && vy[k]) : true;
                    u64 r;
                    switch (op) {
                        case OP_ADD_I64: r = math_val<0, false>(x[k], y[k]); break;
                        case OP_SUB_I64: r = math_val<1, false>(x[k], y[k]); break;
                        case OP_MUL_I64: r = math_val<2, false>(x[k], y[k]); break;
                        case OP_DIV_I64:
                            if (v && S.act(k)) {
                                if (y[k] == 0) report_err(L.err, in.ordinal, S.row(k), ERRK_DIV_ZERO);
                                else if ((i64)y[k] == -1 && x[k] == 0x8000000000000000ull)
                                    report_err(L.err, in.ordinal, S.row(k), ERRK_DIV_OVERFLOW);
                            }
                            r = math_val<3, false>(x[k], y[k]);
                            break;
                        case OP_ADD_F64: r = math_val<0, true>(x[k], y[k]); break;
                        case OP_SUB_F64: r = math_val<1, true>(x[k], y[k]); break;
                        case OP_MUL_F64: r = math_val<2, true>(x[k], y[k]); break;
                        default:
                            if (v && S.act(k) && as_f64(y[k]) == 0.0)
                                report_err(L.err, in.ordinal, S.row(k), ERRK_DIV_ZERO);
                            r = math_val<3, true>(x[k], y[k]);
                            break;
                    }
                    S.acc[k] = v ? r : 0ull;  // append_null leaves a zero slot
                    if constexpr (C::NULLABLE) S.accv = (S.accv & ~(1u << k)) | ((unsigned)v << k);
                }
            }
            continue;
        }
        switch (op) {
            case OP_AND:
            case OP_OR: {
                const int d = in.dst, a = in.a, b = in.b;
                const bool is_and = op == OP_AND;
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const unsigned x = (S.bv[k] >> a) & 1, y = (S.bv[k] >> b) & 1;
                    unsigned res = is_and ? (x & y) : (x | y);
                    unsigned v = 1;
                    if constexpr (C::NULLABLE) {
                        v = (S.bvd[k] >> a) & (S.bvd[k] >> b) & 1;
                        res &= v;  // append_null leaves a zero value bit
                    }
                    S.bv[k] = (S.bv[k] & ~(1u << d)) | (res << d);
                    S.bvd[k] = (S.bvd[k] & ~(1u << d)) | (v << d);
                }
                break;
            }
            case OP_EQ_UTF8_LIT: do_utf8_lit<C, true>(S, L, in); break;
            case OP_NE_UTF8_LIT: do_utf8_lit<C, false>(S, L, in); break;
            case OP_EQ_UTF8_COL: do_utf8_col<C, true>(S, L, in); break;
            case OP_NE_UTF8_COL: do_utf8_col<C, false>(S, L, in); break;
            case OP_SAVE: {
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    tmp[(in.dst * K + k) * C::BLOCK + S.tid] = S.acc[k];
                    if constexpr (C::NULLABLE)
                        S.tv[k] = (S.tv[k] & ~(1u << in.dst)) | (((S.accv >> k) & 1) << in.dst);
                }
                break;
            }
            case OP_MOVE: {
                u64 x[K];
                bool vx[K];
                fetch<C>(S, L, in.ka, in.a, stage, tmp, x, vx);
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    S.acc[k] = x[k];
                    if constexpr (C::NULLABLE) S.accv = (S.accv & ~(1u << k)) | ((unsigned)vx[k] << k);
                }
                break;
            }
            case OP_BLIT: {
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    S.bv[k] = (S.bv[k] & ~(1u << in.dst)) | ((unsigned)(in.b & 1) << in.dst);
                    S.bvd[k] |= 1u << in.dst;
                }
                break;
            }
            case OP_STORE_ACC:
            case OP_STORE_COL: {
                const DOut& out = L.out[in.dst];
                u64* v = (u64*)out.values;
                u64 x[K];
                bool vx[K];
                if (op == OP_STORE_COL) {
                    fetch<C>(S, L, KD_COL, in.a, stage, tmp, x, vx);
                } else {
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        x[k] = S.acc[k];
                        vx[k] = C::NULLABLE ? ((S.accv >> k) & 1) : true;
                    }
                }
                u64* vt = v + S.obase;  // uniform output base
#pragma unroll
                for (int k = 0; k < K; ++k)
                    if (S.act(k)) vt[S.ldst[k]] = x[k];
                if (S.dense) {  // validity words + null count (projection only)
                    unsigned nulls = 0;
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const i64 w = S.word(k);
                        const u64 vb = __ballot(S.act(k) && vx[k]);
                        nulls += __builtin_popcountll(__ballot(S.act(k) && !vx[k]));
                        if (S.lane == 0 && w * 64 < L.n_rows && out.validity) ((u64*)out.validity)[w] = vb;
                    }
                    if (S.lane == 0 && nulls) atomicAdd(&L.totals[kMaxChan + in.dst], (u64)nulls);
                }
                break;
            }
            case OP_STORE_BOOL: {
                const DOut& out = L.out[in.dst];
                const int s = in.a;
                if (!S.dense) {
                    uint8_t* v = (uint8_t*)out.values + S.obase;
#pragma unroll
                    for (int k = 0; k < K; ++k)
                        if (S.act(k)) v[S.ldst[k]] = (uint8_t)((S.bv[k] >> s) & 1);
                } else {
                    unsigned nulls = 0;
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const i64 w = S.word(k);
                        const bool valid = C::NULLABLE ? ((S.bvd[k] >> s) & 1) : true;
                        const u64 bits = __ballot(S.act(k) && ((S.bv[k] >> s) & 1));
                        const u64 vb = __ballot(S.act(k) && valid);
                        nulls += __builtin_popcountll(__ballot(S.act(k) && !valid));
                        if (S.lane == 0 && w * 64 < L.n_rows) {
                            ((u64*)out.values)[w] = bits;
                            if (out.validity) ((u64*)out.validity)[w] = vb;
                        }
                    }
                    if (S.lane == 0 && nulls) atomicAdd(&L.totals[kMaxChan + in.dst], (u64)nulls);
                }
                break;
            }
            default: break;
        }
    }
}

// Boolean input columns are bit-packed: load them into bool slots 0..n_bool-1.
template <class C>
__device__ __forceinline__ void init_state(State<C>& S, const DLaunch& L) {
    S.accv = ~0u;
    S.actm = 0;
    S.obase = S.base;
#pragma unroll
    for (int k = 0; k < C::K; ++k) {
        S.acc[k] = 0;
        S.tv[k] = ~0u;
        S.bv[k] = 0;
        S.bvd[k] = ~0u;
        S.actm |= (unsigned)(S.row(k) < L.n_rows) << k;
        S.ldst[k] = S.lrow(k);
    }
    for (int j = 0; j < L.n_bool; ++j) {
#pragma unroll
        for (int k = 0; k < C::K; ++k) {
            const u64 bits = bitmap_word((const uint8_t*)L.boolc[j].values, S.word(k), L.boolc[j].bitmap_bytes);
            S.bv[k] |= (unsigned)((bits >> S.lane) & 1) << j;
            if constexpr (C::NULLABLE) {
                if (L.boolc[j].validity) {
                    const u64 vb = bitmap_word(L.boolc[j].validity, S.word(k), L.boolc[j].bitmap_bytes);
                    if (!((vb >> S.lane) & 1)) S.bvd[k] &= ~(1u << j);
                }
            }
        }
    }
}

// Stage the tile's first n_lds numeric columns into LDS: async DMA
// (global_load_lds_dwordx4, 16 B = 2 rows per lane, 1 KiB per wave
// instruction), no VGPR destinations, the whole tile in flight at once.
// Value buffers must be readable to a 16-byte multiple (Arrow pads to 64).
template <class C>
__device__ __forceinline__ void stage_tile(const DLaunch& L, i64 base, u64* stage, int wave, int lane) {
    constexpr int CHUNKS = C::TILE / 128;  // 128-row pieces per column
    for (int c = 0; c < L.n_lds; ++c) {
        const u64* src = (const u64*)L.num[c].values + base;
#pragma unroll
        for (int q = wave; q < CHUNKS; q += C::WAVES) {
            const i64 r = (i64)q * 128 + 2 * lane;
            if (base + r < L.n_rows)
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + r),
                                                 (__attribute__((address_space(3))) void*)(stage + c * C::TILE + q * 128),
                                                 16, 0, 0);
        }
    }
}

// ------------------------------------------------- fused filter+project ---
template <class C>
__global__ __launch_bounds__(C::BLOCK) void k_filter_project(const DLaunch L) {
    constexpr int K = C::K;
    constexpr int WAVES = C::WAVES;
    constexpr int NW = K * WAVES;  // 64-row words per tile
    static_assert(NW <= 64, "one wave scans the tile's words");
    __shared__ u64 s_excl[kMaxChan][NW];
    __shared__ u64 s_cnt[kMaxChan][NW];
    // statics sized to 16-byte multiples: the dynamic region after them stays
    // 16-byte aligned (guide G17)
    __shared__ u64 s_prefix[8];
    __shared__ u64 s_agg[8];
    __shared__ unsigned s_tile_[4];
    unsigned& s_tile = s_tile_[0];
    extern __shared__ __attribute__((aligned(16))) u64 s_tmp[];

    State<C> S;
    S.tid = threadIdx.x;
    S.lane = S.tid & 63;
    S.wave = uni(S.tid >> 6);
    S.dense = false;
    S.cols_valid = false;
    u64* stage = s_tmp;                              // [n_lds][TILE]
    u64* tmp = s_tmp + (size_t)L.n_lds * C::TILE;    // [n_tmp][K][BLOCK]
    // The ticket orders the look-back (every predecessor is running); while
    // it is in flight, speculatively stage tile blockIdx.x -- in-order
    // dispatch makes that the ticket's value nearly always.
    if (S.tid == 0) s_tile = (L.mode & 1) ? blockIdx.x : atomicAdd(L.ticket, 1u);
    stage_tile<C>(L, (i64)blockIdx.x * C::TILE, stage, S.wave, S.lane);
    __syncthreads();
    const unsigned tile = (unsigned)uni((int)s_tile);
    if (tile != blockIdx.x) {  // block-uniform
        stage_tile<C>(L, (i64)tile * C::TILE, stage, S.wave, S.lane);
        __syncthreads();
    }
    S.base = (i64)tile * C::TILE;
    init_state<C>(S, L);
    const unsigned inr = S.actm;

    // phase 0: predicate over every row (FilterRelation::next)
    run_program<C>(S, L, L.pred_begin, L.pred_end, stage, tmp);

    u64 wm[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
    }
    S.actm = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const bool sel = ((inr >> k) & 1) && ((S.bv[k] >> L.pred_slot) & 1);  // mask.value(i)
        S.actm |= (unsigned)sel << k;
        wm[k] = __ballot(sel);
        if (S.lane == 0) s_cnt[0][k * WAVES + S.wave] = __builtin_popcountll(wm[k]);
    }
    // Utf8 byte channels (channel 1+u <-> Utf8 output L.chan_out[u])
    unsigned blen_excl[kMaxUtf8][K];
#pragma unroll
    for (int u = 0; u < kMaxUtf8; ++u) {
        if (u + 1 < L.n_chan) {
            const DCol& c = L.utf8[L.out[L.chan_out[u]].slot];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const i64 r = S.row(k);
                const unsigned len = S.act(k) ? (unsigned)(c.offsets[r + 1] - c.offsets[r]) : 0u;
                const unsigned incl = wave_incl_scan32(len, S.lane);
                blen_excl[u][k] = incl - len;
                if (S.lane == 63) s_cnt[u + 1][k * WAVES + S.wave] = incl;
            }
        }
    }
    __syncthreads();
    if (S.wave == 0) {
        bool timeout = false;
        for (int ch = 0; ch < L.n_chan; ++ch) {
            const u64 c = S.lane < NW ? s_cnt[ch][S.lane] : 0ull;
            const u64 incl = wave_incl_scan(c, S.lane);
            if (S.lane < NW) s_excl[ch][S.lane] = incl - c;
            const u64 agg = __shfl(incl, NW - 1, 64);
            const u64 pre = (L.mode & 2) ? (ch == 0 ? (u64)tile * C::TILE : 0ull)
                                         : lookback(L.status + (i64)ch * L.n_tiles, tile, agg, S.lane, L.err, &timeout);
            if (S.lane == 0) {
                s_prefix[ch] = pre;
                s_agg[ch] = agg;
            }
        }
        if (S.lane == 0 && tile == (unsigned)L.n_tiles - 1) {
            for (int ch = 0; ch < L.n_chan; ++ch) L.totals[ch] = s_prefix[ch] + s_agg[ch];
        }
    }
    __syncthreads();
    S.obase = (i64)s_prefix[0];
#pragma unroll
    for (int k = 0; k < K; ++k) S.ldst[k] = (unsigned)(s_excl[0][k * WAVES + S.wave] + lane_rank(wm[k]));
    // Projection sees the filtered batch: validity dropped (filter.rs:86-92).
    S.cols_valid = true;
#pragma unroll
    for (int k = 0; k < K; ++k) S.bvd[k] = ~0u;

    // phase 1: projections over the selected rows only
    run_program<C>(S, L, L.proj_begin, L.proj_end, stage, tmp);

    // Utf8 gathers: rebased i32 offsets + byte copy (filter.rs:94-105)
#pragma unroll
    for (int u = 0; u < kMaxUtf8; ++u) {
        if (u + 1 < L.n_chan) {
            const DOut& out = L.out[L.chan_out[u]];
            const DCol& c = L.utf8[out.slot];
            const uint8_t* src = (const uint8_t*)c.values;
            const u64 bpre = s_prefix[u + 1];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                if (!S.act(k)) continue;
                const i64 r = S.row(k);
                const int s = c.offsets[r], e = c.offsets[r + 1];
                const u64 ob = bpre + s_excl[u + 1][k * WAVES + S.wave] + blen_excl[u][k];
                out.offsets[S.obase + S.ldst[k]] = (int32_t)ob;
                if ((i64)(ob + (u64)(e - s)) > out.data_cap) {
                    report_err(L.err, 0, 0, ERRK_CAPACITY);
                    continue;
                }
                for (int i = 0; i < e - s; ++i) out.data[ob + i] = src[s + i];
            }
            if (S.tid == 0 && tile == (unsigned)L.n_tiles - 1)
                out.offsets[s_prefix[0] + s_agg[0]] = (int32_t)(bpre + s_agg[u + 1]);
        }
    }
}

// ---------------------------------------------------- projection only ---
template <class C>
__global__ __launch_bounds__(C::BLOCK) void k_project(const DLaunch L) {
    extern __shared__ __attribute__((aligned(16))) u64 s_tmp[];
    State<C> S;
    S.tid = threadIdx.x;
    S.lane = S.tid & 63;
    S.wave = uni(S.tid >> 6);
    S.dense = true;
    S.cols_valid = false;
    S.base = (i64)blockIdx.x * C::TILE;
    u64* stage = s_tmp;
    u64* tmp = s_tmp + (size_t)L.n_lds * C::TILE;
    stage_tile<C>(L, S.base, stage, S.wave, S.lane);
    __syncthreads();
    init_state<C>(S, L);
    run_program<C>(S, L, L.proj_begin, L.proj_end, stage, tmp);
}

// Boolean outputs of a filtered projection: one byte per row -> bitmap.
__global__ void k_pack_bools(const uint8_t* bytes, uint8_t* bits, const u64* count) {
    const i64 n = (i64)*count;
    const i64 nb = (n + 7) >> 3;
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += (i64)gridDim.x * blockDim.x) {
        unsigned v = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const i64 r = i * 8 + j;
            if (r < n) v |= (unsigned)(bytes[r] & 1) << j;
        }
        bits[i] = (uint8_t)v;
    }
}

// ------------------------------------------------- synthetic inputs ---
__device__ __forceinline__ u64 splitmix64(u64 x) {
    u64 z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void k_gen_unit_f64(u64 key, i64 row0, i64 n, double* out) {
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x)
        out[i] = (double)(splitmix64(key ^ (u64)(row0 + i)) >> 11) * 0x1.0p-53;
}

__global__ void k_gen_i64(u64 key, i64 row0, i64 n, i64 lo, u64 range, i64* out) {
    for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x)
        out[i] = lo + (i64)(splitmix64(key ^ (u64)(row0 + i)) % range);
}

// ------------------------------------------------------ host launchers ---
// Tile shapes (threads x rows per thread). The default is chosen by
// measurement (DESIGN.md "Kernels"); DFMI_TILE_CFG selects another for
// experiments.
int tile_rows_for(int cfg) {
    switch (cfg) {
        case 0: return 256 * 4;
        case 1: return 256 * 16;
        case 2: return 512 * 8;
        default: return 1024 * 4;
    }
}

static hipError_t launch_any(bool fp, const DLaunch& L, bool nullable, int cfg, hipStream_t st) {
    const size_t lds = (size_t)(L.n_tmp + L.n_lds) * tile_rows_for(cfg) * sizeof(u64);
#define DFMI_L(B, KK)                                                                             \
    do {                                                                                          \
        if (fp) {                                                                                 \
            if (nullable) hipLaunchKernelGGL((k_filter_project<Cfg<B, KK, true>>), dim3(L.n_tiles), dim3(B), lds, st, L); \
            else hipLaunchKernelGGL((k_filter_project<Cfg<B, KK, false>>), dim3(L.n_tiles), dim3(B), lds, st, L); \
        } else {                                                                                  \
            if (nullable) hipLaunchKernelGGL((k_project<Cfg<B, KK, true>>), dim3(L.n_tiles), dim3(B), lds, st, L); \
            else hipLaunchKernelGGL((k_project<Cfg<B, KK, false>>), dim3(L.n_tiles), dim3(B), lds, st, L); \
        }                                                                                         \
    } while (0)
    switch (cfg) {
        case 0: DFMI_L(256, 4); break;
        case 1: DFMI_L(256, 16); break;
        case 2: DFMI_L(512, 8); break;
        default: DFMI_L(1024, 4); break;
    }
#undef DFMI_L
    return hipGetLastError();
}

hipError_t launch_filter_project(const DLaunch& L, bool nullable, int cfg, hipStream_t st) {
    return launch_any(true, L, nullable, cfg, st);
}

hipError_t launch_project(const DLaunch& L, bool nullable, int cfg, hipStream_t st) {
    return launch_any(false, L, nullable, cfg, st);
}

hipError_t launch_pack_bools(const uint8_t* bytes, uint8_t* bits, const u64* count, i64 max_rows,
                             hipStream_t st) {
    const i64 nb = (max_rows + 7) / 8;
    int grid = (int)std::min<i64>((nb + 255) / 256, 4096);
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(k_pack_bools, dim3(grid), dim3(256), 0, st, bytes, bits, count);
    return hipGetLastError();
}

hipError_t launch_gen_unit_f64(u64 key, i64 row0, i64 n, double* out, hipStream_t st) {
    hipLaunchKernelGGL(k_gen_unit_f64, dim3(8192), dim3(256), 0, st, key, row0, n, out);
    return hipGetLastError();
}

hipError_t launch_gen_i64(u64 key, i64 row0, i64 n, i64 lo, u64 range, i64* out, hipStream_t st) {
    hipLaunchKernelGGL(k_gen_i64, dim3(8192), dim3(256), 0, st, key, row0, n, lo, range, out);
    return hipGetLastError();
}


}  // namespace dfmi
