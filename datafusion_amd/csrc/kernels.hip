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
// sums predecessors' aggregates 64 at a time until an inclusive prefix is
// found, publishes the inclusive prefix, returns the exclusive prefix.
// Tiles are numbered by a dynamic ticket, so every predecessor is already
// running: the spin always ends; it is bounded anyway.
__device__ u64 lookback(u64* st, unsigned tile, u64 agg, int lane, u64* err, bool* timeout) {
    if (tile == 0) {
        if (lane == 0) st_status(st, FLAG_P | agg);
        return 0;
    }
    if (lane == 0) st_status(st + tile, FLAG_A | agg);
    u64 excl = 0;
    i64 j = (i64)tile - 1;
    unsigned spins = 0;
    while (true) {
        const i64 idx = j - lane;
        const u64 w = idx >= 0 ? ld_status(st + idx) : FLAG_P;
        const unsigned flag = (unsigned)(w >> 62);
        const u64 xm = __ballot(flag == 0);
        const u64 pm = __ballot(flag == 2);
        if (pm) {
            const int first = __builtin_ctzll(pm);
            const u64 need = first == 63 ? ~0ull : ((2ull << first) - 1);
            if (!(xm & need)) {
                excl += wave_sum(lane <= first ? (w & VAL_MASK) : 0);
                break;
            }
        } else if (!xm) {
            excl += wave_sum(w & VAL_MASK);
            j -= 64;
            continue;
        }
        if (++spins > (1u << 24)) {
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
// Per-thread state for K rows. c[k] holds the numeric input columns of row
// k (read-only after the load phase), acc[k] the accumulator.
template <bool NULLABLE, int NC>
struct Regs {
    static constexpr int K = 16 / NC;
    typedef u64 colv __attribute__((ext_vector_type(NC)));
    colv c[K];
    u64 acc[K];
    unsigned nv[K];   // numeric column validity bits (bit j = column j)
    bool accv[K];     // accumulator validity
    unsigned tv[K];   // temporary validity bits
    unsigned bv[K];   // bool slot value bits
    unsigned bvd[K];  // bool slot validity bits
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

// Operand fetch for all K rows: kind and index are wave-uniform.
template <bool NULLABLE, int NC>
__device__ __forceinline__ void fetch(const Regs<NULLABLE, NC>& R, int kind, int idx,
                                      const uint64_t* lits, const u64* tmp, int tid,
                                      u64 (&x)[Regs<NULLABLE, NC>::K], bool (&v)[Regs<NULLABLE, NC>::K]) {
    constexpr int K = Regs<NULLABLE, NC>::K;
    if (kind == KD_COL) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            x[k] = R.c[k][idx];
            v[k] = NULLABLE ? ((R.nv[k] >> idx) & 1) : true;
        }
    } else if (kind == KD_LIT) {
        const u64 l = lits[idx];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            x[k] = l;
            v[k] = true;
        }
    } else if (kind == KD_ACC) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            x[k] = R.acc[k];
            v[k] = NULLABLE ? R.accv[k] : true;
        }
    } else {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            x[k] = tmp[(idx * K + k) * BLOCK + tid];
            v[k] = NULLABLE ? ((R.tv[k] >> idx) & 1) : true;
        }
    }
}

template <bool NULLABLE, int NC, bool EQ>
__device__ __forceinline__ void do_utf8_lit(Regs<NULLABLE, NC>& R, const DLaunch& L, const DIns in,
                                            const i64* rows, const bool* inr) {
    constexpr int K = Regs<NULLABLE, NC>::K;
    const DCol& c = L.utf8[in.a];
    const int loff = L.strlit_off[in.b], llen = L.strlit_len[in.b];
    const uint8_t* bytes = (const uint8_t*)c.values;
    const int d = in.dst;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        bool eq = false;
        if (inr[k]) {
            const int s = c.offsets[rows[k]], e = c.offsets[rows[k] + 1];
            eq = (e - s) == llen;
            for (int i = 0; eq && i < llen; ++i) eq = bytes[s + i] == (uint8_t)L.strlit[loff + i];
        }
        bool valid = true;
        if constexpr (NULLABLE) {
            if (c.validity && inr[k]) valid = (c.validity[rows[k] >> 3] >> (rows[k] & 7)) & 1;
        }
        // Some(x) == Some(lit); None == Some(lit) -> false
        const bool res = EQ ? (valid && eq) : !(valid && eq);
        R.bv[k] = (R.bv[k] & ~(1u << d)) | ((unsigned)res << d);
        R.bvd[k] |= 1u << d;
    }
}

template <bool NULLABLE, int NC, bool EQ>
__device__ __forceinline__ void do_utf8_col(Regs<NULLABLE, NC>& R, const DLaunch& L, const DIns in,
                                            const i64* rows, const bool* inr) {
    constexpr int K = Regs<NULLABLE, NC>::K;
    const DCol& c0 = L.utf8[in.a];
    const DCol& c1 = L.utf8[in.b];
    const uint8_t* b0 = (const uint8_t*)c0.values;
    const uint8_t* b1 = (const uint8_t*)c1.values;
    const int d = in.dst;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        bool eq = false, v0 = true, v1 = true;
        if (inr[k]) {
            const int s0 = c0.offsets[rows[k]], e0 = c0.offsets[rows[k] + 1];
            const int s1 = c1.offsets[rows[k]], e1 = c1.offsets[rows[k] + 1];
            eq = (e0 - s0) == (e1 - s1);
            for (int i = 0; eq && i < e0 - s0; ++i) eq = b0[s0 + i] == b1[s1 + i];
            if constexpr (NULLABLE) {
                if (c0.validity) v0 = (c0.validity[rows[k] >> 3] >> (rows[k] & 7)) & 1;
                if (c1.validity) v1 = (c1.validity[rows[k] >> 3] >> (rows[k] & 7)) & 1;
            }
        }
        const bool oeq = (v0 && v1) ? eq : (!v0 && !v1);
        const bool res = EQ ? oeq : !oeq;
        R.bv[k] = (R.bv[k] & ~(1u << d)) | ((unsigned)res << d);
        R.bvd[k] |= 1u << d;
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
        else {
            const i64 sx = (i64)x, sy = (i64)y;
            if (sy == 0) return 0;
            if (sy == -1) return 0ull - x;  // wraps; MIN / -1 is reported
            return (u64)(sx / sy);
        }
    }
}

// Per-row output placement: compacted (filtered) or dense (projection only).
template <int K>
struct Place {
    bool act[K];     // rows this program is evaluated on (errors count only here)
    i64 rows[K];     // input row index
    i64 dst[K];      // output row index (compacted) -- dense: == rows
    bool dense;      // projection-only kernel: write bitmaps by ballot
    int lane, wave;
    i64 base;
};

template <bool NULLABLE, int NC>
__device__ void run_program(Regs<NULLABLE, NC>& R, const DLaunch& L, int begin, int end,
                            const Place<Regs<NULLABLE, NC>::K>& P, const bool* inr, u64* tmp,
                            int tid) {
    constexpr int K = Regs<NULLABLE, NC>::K;
    for (int i = begin; i < end; ++i) {
        const DIns in = L.ins[i];
        const int op = in.op;
        if (op <= OP_DIV_F64) {  // numeric binary: comparison or math
            u64 x[K], y[K];
            bool vx[K], vy[K];
            fetch<NULLABLE, NC>(R, in.ka, in.a, L.lits, tmp, tid, x, vx);
            fetch<NULLABLE, NC>(R, in.kb, in.b, L.lits, tmp, tid, y, vy);
            if (op <= OP_GE_F64) {
                bool res[K];
                switch (op) {
                    case OP_EQ_I64: cmp_rows<0, false>(x, y, res); if (NULLABLE) cmp_nulls<0>(vx, vy, res); break;
                    case OP_NE_I64: cmp_rows<1, false>(x, y, res); if (NULLABLE) cmp_nulls<1>(vx, vy, res); break;
                    case OP_LT_I64: cmp_rows<2, false>(x, y, res); if (NULLABLE) cmp_nulls<2>(vx, vy, res); break;
                    case OP_LE_I64: cmp_rows<3, false>(x, y, res); if (NULLABLE) cmp_nulls<3>(vx, vy, res); break;
                    case OP_GT_I64: cmp_rows<4, false>(x, y, res); if (NULLABLE) cmp_nulls<4>(vx, vy, res); break;
                    case OP_GE_I64: cmp_rows<5, false>(x, y, res); if (NULLABLE) cmp_nulls<5>(vx, vy, res); break;
                    case OP_EQ_F64: cmp_rows<0, true>(x, y, res); if (NULLABLE) cmp_nulls<0>(vx, vy, res); break;
                    case OP_NE_F64: cmp_rows<1, true>(x, y, res); if (NULLABLE) cmp_nulls<1>(vx, vy, res); break;
                    case OP_LT_F64: cmp_rows<2, true>(x, y, res); if (NULLABLE) cmp_nulls<2>(vx, vy, res); break;
                    case OP_LE_F64: cmp_rows<3, true>(x, y, res); if (NULLABLE) cmp_nulls<3>(vx, vy, res); break;
                    case OP_GT_F64: cmp_rows<4, true>(x, y, res); if (NULLABLE) cmp_nulls<4>(vx, vy, res); break;
                    default:        cmp_rows<5, true>(x, y, res); if (NULLABLE) cmp_nulls<5>(vx, vy, res); break;
                }
                const int d = in.dst;
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    R.bv[k] = (R.bv[k] & ~(1u << d)) | ((unsigned)res[k] << d);
                    R.bvd[k] |= 1u << d;
                }
            } else {
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const bool v = NULLABLE ? (vx[k] && vy[k]) : true;
                    u64 r;
                    switch (op) {
                        case OP_ADD_I64: r = math_val<0, false>(x[k], y[k]); break;
                        case OP_SUB_I64: r = math_val<1, false>(x[k], y[k]); break;
                        case OP_MUL_I64: r = math_val<2, false>(x[k], y[k]); break;
                        case OP_DIV_I64:
                            if (v && P.act[k]) {
                                if (y[k] == 0) report_err(L.err, in.ordinal, P.rows[k], ERRK_DIV_ZERO);
                                else if ((i64)y[k] == -1 && x[k] == 0x8000000000000000ull)
                                    report_err(L.err, in.ordinal, P.rows[k], ERRK_DIV_OVERFLOW);
                            }
                            r = math_val<3, false>(x[k], y[k]);
                            break;
                        case OP_ADD_F64: r = math_val<0, true>(x[k], y[k]); break;
                        case OP_SUB_F64: r = math_val<1, true>(x[k], y[k]); break;
                        case OP_MUL_F64: r = math_val<2, true>(x[k], y[k]); break;
                        default:
                            if (v && P.act[k] && as_f64(y[k]) == 0.0)
                                report_err(L.err, in.ordinal, P.rows[k], ERRK_DIV_ZERO);
                            r = math_val<3, true>(x[k], y[k]);
                            break;
                    }
                    R.acc[k] = v ? r : 0ull;  // append_null leaves a zero slot
                    if constexpr (NULLABLE) R.accv[k] = v;
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
                    const unsigned x = (R.bv[k] >> a) & 1, y = (R.bv[k] >> b) & 1;
                    unsigned res = is_and ? (x & y) : (x | y);
                    unsigned v = 1;
                    if constexpr (NULLABLE) {
                        v = (R.bvd[k] >> a) & (R.bvd[k] >> b) & 1;
                        res &= v;  // append_null leaves a zero value bit
                    }
                    R.bv[k] = (R.bv[k] & ~(1u << d)) | (res << d);
                    R.bvd[k] = (R.bvd[k] & ~(1u << d)) | (v << d);
                }
                break;
            }
            case OP_EQ_UTF8_LIT: do_utf8_lit<NULLABLE, NC, true>(R, L, in, P.rows, inr); break;
            case OP_NE_UTF8_LIT: do_utf8_lit<NULLABLE, NC, false>(R, L, in, P.rows, inr); break;
            case OP_EQ_UTF8_COL: do_utf8_col<NULLABLE, NC, true>(R, L, in, P.rows, inr); break;
            case OP_NE_UTF8_COL: do_utf8_col<NULLABLE, NC, false>(R, L, in, P.rows, inr); break;
            case OP_SAVE: {
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    tmp[(in.dst * K + k) * BLOCK + tid] = R.acc[k];
                    if constexpr (NULLABLE)
                        R.tv[k] = (R.tv[k] & ~(1u << in.dst)) | ((unsigned)R.accv[k] << in.dst);
                }
                break;
            }
            case OP_MOVE: {
                u64 x[K];
                bool vx[K];
                fetch<NULLABLE, NC>(R, in.ka, in.a, L.lits, tmp, tid, x, vx);
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    R.acc[k] = x[k];
                    if constexpr (NULLABLE) R.accv[k] = vx[k];
                }
                break;
            }
            case OP_BLIT: {
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    R.bv[k] = (R.bv[k] & ~(1u << in.dst)) | ((unsigned)(in.b & 1) << in.dst);
                    R.bvd[k] |= 1u << in.dst;
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
                    fetch<NULLABLE, NC>(R, KD_COL, in.a, L.lits, tmp, tid, x, vx);
                } else {
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        x[k] = R.acc[k];
                        vx[k] = NULLABLE ? R.accv[k] : true;
                    }
                }
#pragma unroll
                for (int k = 0; k < K; ++k)
                    if (P.act[k]) v[P.dst[k]] = x[k];
                if (P.dense) {  // validity words + null count (projection only)
                    unsigned nulls = 0;
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const i64 w = (P.base + (i64)k * BLOCK + P.wave * 64) >> 6;
                        const u64 vb = __ballot(P.act[k] && vx[k]);
                        nulls += __builtin_popcountll(__ballot(P.act[k] && !vx[k]));
                        if (P.lane == 0 && w * 64 < L.n_rows && out.validity) ((u64*)out.validity)[w] = vb;
                    }
                    if (P.lane == 0 && nulls) atomicAdd(&L.totals[kMaxChan + in.dst], (u64)nulls);
                }
                break;
            }
            case OP_STORE_BOOL: {
                const DOut& out = L.out[in.dst];
                const int s = in.a;
                if (!P.dense) {
                    uint8_t* v = (uint8_t*)out.values;
#pragma unroll
                    for (int k = 0; k < K; ++k)
                        if (P.act[k]) v[P.dst[k]] = (uint8_t)((R.bv[k] >> s) & 1);
                } else {
                    unsigned nulls = 0;
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const i64 w = (P.base + (i64)k * BLOCK + P.wave * 64) >> 6;
                        const bool valid = NULLABLE ? ((R.bvd[k] >> s) & 1) : true;
                        const u64 bits = __ballot(P.act[k] && ((R.bv[k] >> s) & 1));
                        const u64 vb = __ballot(P.act[k] && valid);
                        nulls += __builtin_popcountll(__ballot(P.act[k] && !valid));
                        if (P.lane == 0 && w * 64 < L.n_rows) {
                            ((u64*)out.values)[w] = bits;
                            if (out.validity) ((u64*)out.validity)[w] = vb;
                        }
                    }
                    if (P.lane == 0 && nulls) atomicAdd(&L.totals[kMaxChan + in.dst], (u64)nulls);
                }
                break;
            }
            default: break;
        }
    }
}

// Load the launch's numeric and Boolean input columns for this thread's K rows:
// all loads are issued before any is consumed.
template <bool NULLABLE, int NC>
__device__ __forceinline__ void load_inputs(Regs<NULLABLE, NC>& R, const DLaunch& L, i64 base,
                                            int lane, int wave, const bool* inr, const i64* rows) {
    constexpr int K = Regs<NULLABLE, NC>::K;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        R.c[k] = 0;
        R.acc[k] = 0;
        R.nv[k] = ~0u;
        R.accv[k] = true;
        R.tv[k] = ~0u;
        R.bv[k] = 0;
        R.bvd[k] = ~0u;
    }
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        if (j < L.n_num) {
            const u64* p = (const u64*)L.num[j].values;
#pragma unroll
            for (int k = 0; k < K; ++k) R.c[k][j] = inr[k] ? p[rows[k]] : 0ull;
        }
    }
    if constexpr (NULLABLE) {
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            if (j < L.n_num && L.num[j].validity) {
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const i64 w = (base + (i64)k * BLOCK + wave * 64) >> 6;
                    const u64 bits = bitmap_word(L.num[j].validity, w, L.num[j].bitmap_bytes);
                    if (!((bits >> lane) & 1)) R.nv[k] &= ~(1u << j);
                }
            }
        }
    }
    for (int j = 0; j < L.n_bool; ++j) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const i64 w = (base + (i64)k * BLOCK + wave * 64) >> 6;
            const u64 bits = bitmap_word((const uint8_t*)L.boolc[j].values, w, L.boolc[j].bitmap_bytes);
            R.bv[k] |= (unsigned)((bits >> lane) & 1) << j;
            if constexpr (NULLABLE) {
                if (L.boolc[j].validity) {
                    const u64 vb = bitmap_word(L.boolc[j].validity, w, L.boolc[j].bitmap_bytes);
                    if (!((vb >> lane) & 1)) R.bvd[k] &= ~(1u << j);
                }
            }
        }
    }
}

// ------------------------------------------------- fused filter+project ---
template <bool NULLABLE, int NC>
__global__ __launch_bounds__(BLOCK) void k_filter_project(const DLaunch L) {
    constexpr int K = Regs<NULLABLE, NC>::K;
    constexpr int TILE = BLOCK * K;
    __shared__ u64 s_excl[kMaxChan][K * WAVES];
    __shared__ u64 s_cnt[kMaxChan][K * WAVES];
    __shared__ u64 s_prefix[kMaxChan];
    __shared__ u64 s_agg[kMaxChan];
    __shared__ unsigned s_tile;
    extern __shared__ __attribute__((aligned(16))) u64 s_tmp[];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = uni(tid >> 6);
    if (tid == 0) s_tile = atomicAdd(L.ticket, 1u);
    __syncthreads();
    const unsigned tile = (unsigned)uni((int)s_tile);
    const i64 base = (i64)tile * TILE;

    bool inr[K];
    Place<K> P;
    P.dense = false;
    P.lane = lane;
    P.wave = wave;
    P.base = base;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        P.rows[k] = base + (i64)k * BLOCK + tid;
        inr[k] = P.rows[k] < L.n_rows;
        P.act[k] = inr[k];
        P.dst[k] = 0;
    }

    Regs<NULLABLE, NC> R;
    load_inputs<NULLABLE, NC>(R, L, base, lane, wave, inr, P.rows);

    u64 wm[K];
    unsigned blen_excl[kMaxUtf8][K];
    // phase 0: predicate over every row (FilterRelation::next); then the
    // compaction offsets; phase 1: projections over the selected rows.
#pragma nounroll
    for (int phase = 0; phase < 2; ++phase) {
        run_program<NULLABLE, NC>(R, L, phase ? L.proj_begin : L.pred_begin,
                                  phase ? L.proj_end : L.pred_end, P, inr, s_tmp, tid);
        if (phase) break;

#pragma unroll
        for (int k = 0; k < K; ++k) {
            P.act[k] = inr[k] && ((R.bv[k] >> L.pred_slot) & 1);  // mask.value(i)
            wm[k] = __ballot(P.act[k]);
            if (lane == 0) s_cnt[0][k * WAVES + wave] = __builtin_popcountll(wm[k]);
        }
        // Utf8 byte channels (channel 1+u <-> Utf8 output L.chan_out[u])
#pragma unroll
        for (int u = 0; u < kMaxUtf8; ++u) {
            if (u + 1 < L.n_chan) {
                const DCol& c = L.utf8[L.out[L.chan_out[u]].slot];
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const unsigned len =
                        P.act[k] ? (unsigned)(c.offsets[P.rows[k] + 1] - c.offsets[P.rows[k]]) : 0u;
                    const unsigned incl = wave_incl_scan32(len, lane);
                    blen_excl[u][k] = incl - len;
                    if (lane == 63) s_cnt[u + 1][k * WAVES + wave] = incl;
                }
            }
        }
        __syncthreads();
        if (wave == 0) {
            bool timeout = false;
            for (int ch = 0; ch < L.n_chan; ++ch) {
                const u64 c = lane < K * WAVES ? s_cnt[ch][lane] : 0ull;
                const u64 incl = wave_incl_scan(c, lane);
                if (lane < K * WAVES) s_excl[ch][lane] = incl - c;
                const u64 agg = __shfl(incl, K * WAVES - 1, 64);
                const u64 pre = lookback(L.status + (i64)ch * L.n_tiles, tile, agg, lane, L.err, &timeout);
                if (lane == 0) {
                    s_prefix[ch] = pre;
                    s_agg[ch] = agg;
                }
            }
            if (lane == 0 && tile == (unsigned)L.n_tiles - 1) {
                for (int ch = 0; ch < L.n_chan; ++ch) L.totals[ch] = s_prefix[ch] + s_agg[ch];
            }
        }
        __syncthreads();
        const u64 prefix = s_prefix[0];
#pragma unroll
        for (int k = 0; k < K; ++k)
            P.dst[k] = (i64)(prefix + s_excl[0][k * WAVES + wave] + lane_rank(wm[k]));
        // Projection sees the filtered batch: validity dropped (filter.rs:86-92).
        if constexpr (NULLABLE) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                R.nv[k] = ~0u;
                R.bvd[k] = ~0u;
            }
        }
    }

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
                if (!P.act[k]) continue;
                const int s = c.offsets[P.rows[k]], e = c.offsets[P.rows[k] + 1];
                const u64 ob = bpre + s_excl[u + 1][k * WAVES + wave] + blen_excl[u][k];
                out.offsets[P.dst[k]] = (int32_t)ob;
                if ((i64)(ob + (u64)(e - s)) > out.data_cap) {
                    report_err(L.err, 0, 0, ERRK_CAPACITY);
                    continue;
                }
                for (int i = 0; i < e - s; ++i) out.data[ob + i] = src[s + i];
            }
            if (tid == 0 && tile == (unsigned)L.n_tiles - 1)
                out.offsets[s_prefix[0] + s_agg[0]] = (int32_t)(bpre + s_agg[u + 1]);
        }
    }
}

// ---------------------------------------------------- projection only ---
template <bool NULLABLE, int NC>
__global__ __launch_bounds__(BLOCK) void k_project(const DLaunch L) {
    constexpr int K = Regs<NULLABLE, NC>::K;
    constexpr int TILE = BLOCK * K;
    extern __shared__ __attribute__((aligned(16))) u64 s_tmp[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = uni(tid >> 6);
    const i64 base = (i64)blockIdx.x * TILE;
    bool inr[K];
    Place<K> P;
    P.dense = true;
    P.lane = lane;
    P.wave = wave;
    P.base = base;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        P.rows[k] = base + (i64)k * BLOCK + tid;
        inr[k] = P.rows[k] < L.n_rows;
        P.act[k] = inr[k];
        P.dst[k] = P.rows[k];
    }
    Regs<NULLABLE, NC> R;
    load_inputs<NULLABLE, NC>(R, L, base, lane, wave, inr, P.rows);
    run_program<NULLABLE, NC>(R, L, L.proj_begin, L.proj_end, P, inr, s_tmp, tid);
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
template <bool N, int NC>
static hipError_t launch_fp(const DLaunch& L, size_t lds, hipStream_t st) {
    hipLaunchKernelGGL((k_filter_project<N, NC>), dim3(L.n_tiles), dim3(BLOCK), lds, st, L);
    return hipGetLastError();
}
template <bool N, int NC>
static hipError_t launch_p(const DLaunch& L, size_t lds, hipStream_t st) {
    hipLaunchKernelGGL((k_project<N, NC>), dim3(L.n_tiles), dim3(BLOCK), lds, st, L);
    return hipGetLastError();
}

// Column-file width for n numeric columns; rows per tile follow (K*NC = 16).
int pick_nc(int n_num) { return n_num <= 4 ? 4 : (n_num <= 8 ? 8 : 16); }
int tile_rows_for(int nc) { return BLOCK * (16 / nc); }

hipError_t launch_filter_project(const DLaunch& L, bool nullable, int nc, hipStream_t st) {
    const size_t lds = (size_t)L.n_tmp * tile_rows_for(nc) * sizeof(u64);
    if (nc == 4) return nullable ? launch_fp<true, 4>(L, lds, st) : launch_fp<false, 4>(L, lds, st);
    if (nc == 8) return nullable ? launch_fp<true, 8>(L, lds, st) : launch_fp<false, 8>(L, lds, st);
    return nullable ? launch_fp<true, 16>(L, lds, st) : launch_fp<false, 16>(L, lds, st);
}

hipError_t launch_project(const DLaunch& L, bool nullable, int nc, hipStream_t st) {
    const size_t lds = (size_t)L.n_tmp * tile_rows_for(nc) * sizeof(u64);
    if (nc == 4) return nullable ? launch_p<true, 4>(L, lds, st) : launch_p<false, 4>(L, lds, st);
    if (nc == 8) return nullable ? launch_p<true, 8>(L, lds, st) : launch_p<false, 8>(L, lds, st);
    return nullable ? launch_p<true, 16>(L, lds, st) : launch_p<false, 16>(L, lds, st);
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
