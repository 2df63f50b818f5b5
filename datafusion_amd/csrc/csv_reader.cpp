// Native CSV source: the reference's CsvDataSource (datasource.rs:31-50) over
// arrow 0.12's csv::Reader (csv_sql.rs:49: schema, has_header, batch size),
// producing Arrow batches straight into pinned host memory, so
// dfmi_filter_project_host DMAs them without a staging copy.
//
//   open : mmap the file, index the records (one pass: memchr over '\n' when
//          the file holds no quote character, a quote-aware scan otherwise);
//   next : the batch parsed by host threads (row ranges of whole 64-row
//          words, so validity / Boolean bitmap words are never shared);
//          while the caller works on batch i the reader already parses
//          batch i+1 into the other of two pinned buffer sets.
//
// Field rules (arrow 0.12 reader, as tests/golden_cases' restatement): ','
// separated, a field starting with '"' is quoted ("" = one quote), records
// end at '\n' (a preceding '\r' is dropped), empty records are skipped, a
// missing trailing field or an empty numeric field is null, Utf8 keeps the
// bytes (a null Utf8 field is ""), Boolean is true/false (any case), numbers
// as Rust's str::parse (decimal; inf / infinity / nan words), anything else
// is ArrowError(ParseError) "Error while parsing value <field>".
#include <emmintrin.h>
#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <charconv>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/dfmi.h"
#include "../../include/dfmi_datasource.h"

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

void set_err(dfmi_error* err, int32_t code, const std::string& m) {
    if (!err) return;
    err->code = code;
    snprintf(err->message, sizeof err->message, "%s", m.c_str());
}

// Grow-only host buffer, pinned (hipHostMalloc) when a device is present --
// the DMA engines then read it directly -- else 64-byte aligned pageable
// memory (the host path stages pageable buffers itself).
struct PinBuf {
    uint8_t* p = nullptr;
    size_t cap = 0;
    bool pinned = false;
    void release() {
        if (p) {
            if (pinned) (void)hipHostFree(p);
            else free(p);
        }
        p = nullptr;
        cap = 0;
    }
    bool reserve(size_t n) {
        n = (std::max<size_t>(n, 64) + 63) & ~(size_t)63;
        if (n <= cap) return true;
        release();
        if (hipHostMalloc((void**)&p, n, hipHostMallocPortable) == hipSuccess) {
            pinned = true;
        } else {
            (void)hipGetLastError();
            pinned = false;
            p = (uint8_t*)aligned_alloc(64, n);
            if (!p) return false;
        }
        cap = n;
        return true;
    }
    ~PinBuf() { release(); }
};

// Calls f(nl) for every '\n' of [p, end) in order, until f returns false:
// 64 bytes per step (SSE2 compares, one 64-bit mask), so a short line costs
// a bit scan instead of a memchr call.
template <class F>
void for_each_newline(const char* p, const char* end, F&& f) {
    const __m128i nl = _mm_set1_epi8('\n');
    for (; end - p >= 64; p += 64) {
        uint64_t m = 0;
        for (int k = 0; k < 4; ++k) {
            const __m128i v = _mm_loadu_si128((const __m128i*)(p + 16 * k));
            m |= (uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(v, nl)) << (16 * k);
        }
        while (m) {
            if (!f(p + __builtin_ctzll(m))) return;
            m &= m - 1;
        }
    }
    for (; p < end; ++p)
        if (*p == '\n' && !f(p)) return;
}

bool csv_profile() {
    static const bool on = getenv("DFMI_CSV_PROFILE") != nullptr;
    return on;
}
double ms_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

// One parsed field: [b, e) of the file, quoted (unescape "" when copying).
struct Field {
    const char* b = nullptr;
    const char* e = nullptr;
    bool quoted = false, present = false;
};

// Fields of the record [p, end) (end excludes the line terminator).
void split_record(const char* p, const char* end, int ncols, Field* out) {
    for (int i = 0; i < ncols; ++i) out[i] = Field{};
    int i = 0;
    while (true) {
        Field f;
        f.present = true;
        if (p < end && *p == '"') {
            f.quoted = true;
            const char* q = p + 1;
            const char* s = q;
            while (q < end) {
                if (*q == '"') {
                    if (q + 1 < end && q[1] == '"') {
                        q += 2;
                        continue;
                    }
                    break;
                }
                ++q;
            }
            f.b = s;
            f.e = q;  // closing quote (or end)
            p = q < end ? q + 1 : end;
            while (p < end && *p != ',') ++p;  // bytes after the closing quote are dropped
        } else {
            const char* q = (const char*)memchr(p, ',', (size_t)(end - p));
            if (!q) q = end;
            f.b = p;
            f.e = q;
            p = q;
        }
        if (i < ncols) out[i] = f;
        ++i;
        if (p >= end) break;
        ++p;  // the ','
    }
}

size_t field_len(const Field& f) {
    if (!f.present) return 0;
    if (!f.quoted) return (size_t)(f.e - f.b);
    size_t n = 0;
    for (const char* q = f.b; q < f.e; ++q, ++n)
        if (*q == '"' && q + 1 < f.e && q[1] == '"') ++q;
    return n;
}

void field_copy(const Field& f, uint8_t* dst) {
    if (!f.present) return;
    if (!f.quoted) {
        memcpy(dst, f.b, (size_t)(f.e - f.b));
        return;
    }
    for (const char* q = f.b; q < f.e; ++q) {
        *dst++ = (uint8_t)*q;
        if (*q == '"' && q + 1 < f.e && q[1] == '"') ++q;
    }
}

std::string field_text(const Field& f) {
    std::string s(field_len(f), '\0');
    field_copy(f, (uint8_t*)&s[0]);
    return s;
}

bool lower_eq(const char* b, const char* e, const char* w) {
    const size_t n = strlen(w);
    if ((size_t)(e - b) != n) return false;
    for (size_t i = 0; i < n; ++i)
        if (tolower((unsigned char)b[i]) != w[i]) return false;
    return true;
}

// Rust f32 / f64 ::from_str on [b, e): [+-] then decimal digits with an
// optional '.', an optional exponent, or the words inf / infinity / nan (any
// case); correctly rounded to T (std::from_chars, no locale, no copy).
template <typename T>
bool parse_float(const char* b, const char* e, T* v) {
    const char* p = b;
    bool neg = false;
    if (p < e && (*p == '+' || *p == '-')) neg = *p++ == '-';
    if (lower_eq(p, e, "inf") || lower_eq(p, e, "infinity")) {
        *v = neg ? -INFINITY : INFINITY;
        return true;
    }
    if (lower_eq(p, e, "nan")) {
        *v = NAN;
        return true;
    }
    const char* q = p;
    size_t digits = 0;
    while (q < e && isdigit((unsigned char)*q)) ++q, ++digits;
    if (q < e && *q == '.') {
        ++q;
        while (q < e && isdigit((unsigned char)*q)) ++q, ++digits;
    }
    if (!digits) return false;
    if (q < e && (*q == 'e' || *q == 'E')) {
        ++q;
        if (q < e && (*q == '+' || *q == '-')) ++q;
        size_t ed = 0;
        while (q < e && isdigit((unsigned char)*q)) ++q, ++ed;
        if (!ed) return false;
    }
    if (q != e) return false;
    T x = 0;
    const auto r = std::from_chars(p, e, x);  // p: after any sign ('+' is not from_chars syntax)
    if (r.ec == std::errc::result_out_of_range) {
        // beyond T's range: strtod/strtof give +inf above and 0 / the nearest
        // subnormal below, as Rust's parser does
        const std::string t(p, e);
        x = sizeof(T) == 4 ? (T)strtof(t.c_str(), nullptr) : (T)strtod(t.c_str(), nullptr);
    } else if (r.ec != std::errc() || r.ptr != e) {
        return false;
    }
    *v = neg ? -x : x;
    return true;
}

// Rust iN / uN::from_str on [b, e): optional sign ('-' only for signed),
// decimal digits, in range.
bool parse_int(const char* b, const char* e, bool is_signed, int bits, int64_t* v) {
    const char* p = b;
    bool neg = false;
    if (p < e && (*p == '+' || *p == '-')) {
        neg = *p == '-';
        if (neg && !is_signed) return false;
        ++p;
    }
    if (p == e) return false;
    unsigned __int128 acc = 0;
    for (; p < e; ++p) {
        if (!isdigit((unsigned char)*p)) return false;
        acc = acc * 10 + (unsigned)(*p - '0');
        if (acc > ((unsigned __int128)1 << 64)) return false;
    }
    if (is_signed) {
        const unsigned __int128 lim = (unsigned __int128)1 << (bits - 1);
        if (neg ? acc > lim : acc >= lim) return false;
        *v = neg ? (int64_t)(0 - (uint64_t)acc) : (int64_t)(uint64_t)acc;
    } else {
        if (bits < 64 ? acc >= ((unsigned __int128)1 << bits) : acc > (unsigned __int128)UINT64_MAX) return false;
        *v = (int64_t)(uint64_t)acc;
    }
    return true;
}

struct ColBufs {
    PinBuf values, validity, offsets;
};

struct BatchSet {
    std::vector<ColBufs> cols;
    std::vector<dfmi_column> view;
    int64_t rows = 0;
    int32_t code = DFMI_OK;
    std::string msg;
};

}  // namespace

struct dfmi_csv_reader {
    int fd = -1;
    const char* data = nullptr;
    size_t size = 0;
    std::vector<int> types;
    int64_t batch_size = 1024;
    int threads = 1;
    // record byte ranges (without terminators), records [rec0, n_rec): the
    // header record, when there is one, is skipped by starting at 1
    uint64_t* rec_b = nullptr;
    uint64_t* rec_e = nullptr;
    size_t n_rec = 0, rec0 = 0;
    size_t next_row = 0;  // first record of the batch the next prefetch parses
    BatchSet sets[2];
    int cur = 0;
    std::thread prefetch;
    bool prefetching = false;
    bool ended = false;

    ~dfmi_csv_reader() {
        if (prefetch.joinable()) prefetch.join();
        if (rec_b) munmap(rec_b, rec_bytes);
        if (rec_e) munmap(rec_e, rec_bytes);
        if (data) munmap((void*)data, size);
        if (fd >= 0) close(fd);
    }

    // Index arrays: anonymous mappings advised for transparent huge pages
    // (an 80 MB index of a 5M-record file otherwise takes ~20k page faults
    // on the threads that first write it).
    size_t rec_bytes = 0;
    static uint64_t* map_index(size_t bytes) {
        void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (m == MAP_FAILED) throw std::bad_alloc();
        madvise(m, bytes, MADV_HUGEPAGE);
        return (uint64_t*)m;
    }
    void alloc_index(size_t n) {
        n_rec = n;
        rec_bytes = std::max<size_t>(1, n) * 8;
        rec_b = map_index(rec_bytes);
        rec_e = map_index(rec_bytes);
    }

    void index_records(bool has_header) {
        const char* end = data + size;
        const auto t0 = std::chrono::steady_clock::now();
        // Without quote characters records are lines. Host threads walk the
        // lines starting in their share of the file twice: counting records
        // (and looking for quotes), then -- at their prefix offsets -- writing
        // them straight into the index. Any quote falls back to the
        // sequential state machine.
        const int nt = (int)std::max<size_t>(1, std::min<size_t>((size_t)threads, size / ((size_t)4 << 20) + 1));
        std::vector<size_t> cnt(nt + 1, 0);
        std::vector<char> quoted(nt, 0);
        auto walk_share = [&](int t, auto&& rec) {  // rec(b, e) per nonempty record
            const char* c0 = data + size / nt * t;
            const char* c1 = t + 1 == nt ? end : data + size / nt * (t + 1);
            const char* q = c0;
            if (t > 0 && c0[-1] != '\n') {  // the line in progress belongs to the share before
                const char* nl = (const char*)memchr(c0, '\n', (size_t)(end - c0));
                q = nl ? nl + 1 : end;
            }
            auto line = [&](const char* e) {  // the record [q, e)
                const char* e2 = (e > q && e[-1] == '\r') ? e - 1 : e;
                if (e2 > q) rec(q, e2);  // empty records are skipped
            };
            if (q < c1) {
                for_each_newline(q, end, [&](const char* nl) {
                    line(nl);
                    q = nl + 1;
                    return q < c1;
                });
                if (q < c1) line(end);  // the last record has no terminator
            }
        };
        auto count_share = [&](int t) {
            const char* c0 = data + size / nt * t;
            const char* c1 = t + 1 == nt ? end : data + size / nt * (t + 1);
            quoted[t] = memchr(c0, '"', (size_t)(c1 - c0)) != nullptr;
            if (quoted[t]) return;
            size_t n = 0;
            walk_share(t, [&](const char*, const char*) { ++n; });
            cnt[t + 1] = n;
        };
        run(nt, count_share);
        bool quotes = false;
        for (char x : quoted) quotes = quotes || x;
        if (!quotes) {
            for (int t = 0; t < nt; ++t) cnt[t + 1] += cnt[t];
            alloc_index(cnt[nt]);
            auto write_share = [&](int t) {
                uint64_t* b = rec_b + cnt[t];
                uint64_t* e = rec_e + cnt[t];
                walk_share(t, [&](const char* rb, const char* re) {
                    *b++ = (uint64_t)(rb - data);
                    *e++ = (uint64_t)(re - data);
                });
            };
            run(nt, write_share);
        } else {
            std::vector<uint64_t> lb, le;
            auto add = [&](const char* b, const char* e) {
                if (e > b && e[-1] == '\r') --e;
                if (e > b) {  // empty records are skipped
                    lb.push_back((uint64_t)(b - data));
                    le.push_back((uint64_t)(e - data));
                }
            };
            // a quote opens a quoted field only at the field's start; inside
            // one, "" is a literal quote and a lone " closes it
            enum { START, PLAIN, QUOTED, QUOTE } st = START;
            const char* p = data;
            const char* b = p;
            for (; p < end; ++p) {
                const char ch = *p;
                switch (st) {
                    case START:
                        st = ch == '"' ? QUOTED : PLAIN;
                        if (ch == ',') st = START;
                        break;
                    case PLAIN:
                        if (ch == ',') st = START;
                        break;
                    case QUOTED:
                        if (ch == '"') st = QUOTE;
                        break;
                    case QUOTE:  // "" (literal quote) or the field's end
                        st = ch == '"' ? QUOTED : (ch == ',' ? START : PLAIN);
                        break;
                }
                if (ch == '\n' && st != QUOTED) {
                    add(b, p);
                    b = p + 1;
                    st = START;
                }
            }
            if (b < end) add(b, end);
            alloc_index(lb.size());
            if (!lb.empty()) {
                memcpy(rec_b, lb.data(), lb.size() * 8);
                memcpy(rec_e, le.data(), le.size() * 8);
            }
        }
        if (csv_profile())
            fprintf(stderr, "dfmi csv: indexed %zu records of %zu bytes in %.2f ms (%d threads%s)\n", n_rec, size,
                    ms_since(t0), nt, quotes ? ", quoted: sequential" : "");
        rec0 = has_header && n_rec > 0 ? 1 : 0;
        next_row = rec0;
    }

    // Parse records [r0, r0 + n) into set S.
    void parse(BatchSet& S, size_t r0, int64_t n) {
        const auto t0 = std::chrono::steady_clock::now();
        const int nc = (int)types.size();
        S.rows = n;
        S.code = DFMI_OK;
        S.msg.clear();
        S.cols.resize(nc);
        S.view.assign(std::max(1, nc), dfmi_column{});
        const size_t bm = (size_t)((n + 63) / 64) * 8;
        for (int c = 0; c < nc; ++c) {
            const int t = types[c];
            ColBufs& B = S.cols[c];
            bool ok = B.validity.reserve(bm);
            if (t == DFMI_TYPE_UTF8) ok = ok && B.offsets.reserve((size_t)(n + 1) * 4);
            else ok = ok && B.values.reserve(t == DFMI_TYPE_BOOLEAN ? bm : (size_t)n * width_of(t));
            if (!ok) {
                S.code = DFMI_ERR_DEVICE;
                S.msg = "hipHostMalloc failed for a CSV batch";
                return;
            }
        }
        // row ranges of whole 64-row words per thread (bitmap words are never shared)
        const int64_t words = (n + 63) / 64;
        // a thread per >= 16 Ki rows: csv_sql.rs:49's 1024-row batches parse on one
        // thread (starting threads would cost more than the parse)
        const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(threads, std::min<int64_t>(words, n / 16384 + 1)));
        std::vector<int64_t> nulls((size_t)nt * std::max(1, nc), 0);
        // a parse error: arrow's reader builds the batch column by column, so
        // the one it reports is the first failing row of the first failing column
        std::vector<std::string> errs(nt);
        std::vector<int64_t> err_row(nt, -1);
        std::vector<int> err_col(nt, 1 << 30);
        auto range = [&](int t, int64_t& a, int64_t& b) {
            a = std::min<int64_t>(n, words * t / nt * 64);
            b = std::min<int64_t>(n, words * (t + 1) / nt * 64);
        };
        // pass 1: numeric / Boolean values, validity, Utf8 lengths (into offsets[row + 1])
        auto pass1 = [&](int t) {
            int64_t a, b;
            range(t, a, b);
            std::vector<Field> f(std::max(1, nc));
            for (int64_t r = a; r < b; ++r) {
                split_record(data + rec_b[r0 + r], data + rec_e[r0 + r], nc, f.data());
                for (int c = 0; c < nc; ++c) {
                    const int ty = types[c];
                    ColBufs& B = S.cols[c];
                    uint64_t* vw = (uint64_t*)B.validity.p;
                    const int64_t w = r >> 6;
                    const uint64_t bit = 1ull << (r & 63);
                    if ((r & 63) == 0) vw[w] = 0;
                    if (ty == DFMI_TYPE_UTF8) {
                        ((int32_t*)B.offsets.p)[r + 1] = (int32_t)field_len(f[c]);
                        if (f[c].present) vw[w] |= bit;
                        else ++nulls[(size_t)t * nc + c];
                        continue;
                    }
                    if (ty == DFMI_TYPE_BOOLEAN && (r & 63) == 0) ((uint64_t*)B.values.p)[w] = 0;
                    const bool empty = !f[c].present || f[c].e == f[c].b;
                    if (empty) {  // null
                        if (ty != DFMI_TYPE_BOOLEAN) memset(B.values.p + (size_t)r * width_of(ty), 0, width_of(ty));
                        ++nulls[(size_t)t * nc + c];
                        continue;
                    }
                    vw[w] |= bit;
                    // the field's text: in place, unless quoted ("" unescaped)
                    std::string unq;
                    const char* fb = f[c].b;
                    const char* fe = f[c].e;
                    if (f[c].quoted) {
                        unq = field_text(f[c]);
                        fb = unq.data();
                        fe = fb + unq.size();
                    }
                    bool ok = true;
                    if (ty == DFMI_TYPE_BOOLEAN) {
                        if (lower_eq(fb, fe, "true")) ((uint64_t*)B.values.p)[w] |= bit;
                        else ok = lower_eq(fb, fe, "false");
                    } else if (ty == DFMI_TYPE_FLOAT64) {
                        double d = 0;
                        ok = parse_float(fb, fe, &d);
                        memcpy(B.values.p + (size_t)r * 8, &d, 8);
                    } else if (ty == DFMI_TYPE_FLOAT32) {
                        float x = 0;  // parsed to f32 directly: one rounding, as Rust's f32 parse
                        ok = parse_float(fb, fe, &x);
                        memcpy(B.values.p + (size_t)r * 4, &x, 4);
                    } else {
                        const bool sg = ty >= DFMI_TYPE_INT8 && ty <= DFMI_TYPE_INT64;
                        const int wdt = width_of(ty);
                        int64_t v = 0;
                        ok = parse_int(fb, fe, sg, 8 * wdt, &v);
                        memcpy(B.values.p + (size_t)r * wdt, &v, wdt);  // little-endian low bytes
                    }
                    if (!ok && c < err_col[t]) {
                        err_col[t] = c;
                        err_row[t] = r;
                        errs[t] = "Error while parsing value " + std::string(fb, fe);
                    }
                }
            }
        };
        const double t_res = ms_since(t0);
        run(nt, pass1);
        if (csv_profile())
            fprintf(stderr, "dfmi csv: batch of %lld rows: buffers %.2f ms, parse %.2f ms (%d threads)\n",
                    (long long)n, t_res, ms_since(t0) - t_res, nt);
        int bt = -1;
        for (int t = 0; t < nt; ++t)  // threads hold ascending row ranges
            if (err_row[t] >= 0 && (bt < 0 || err_col[t] < err_col[bt])) bt = t;
        if (bt >= 0) {
            S.code = DFMI_ERR_ARROW_PARSE;
            S.msg = errs[bt];
            return;
        }
        // Utf8 offsets: prefix sums; bytes: pass 2
        for (int c = 0; c < nc; ++c) {
            if (types[c] != DFMI_TYPE_UTF8) continue;
            int32_t* of = (int32_t*)S.cols[c].offsets.p;
            of[0] = 0;
            int64_t acc = 0;
            for (int64_t r = 0; r < n; ++r) {
                acc += of[r + 1];
                if (acc >= ((int64_t)1 << 31)) {
                    S.code = DFMI_ERR_CAPACITY;
                    S.msg = "a CSV batch's Utf8 column exceeds 2^31 bytes (i32 offsets)";
                    return;
                }
                of[r + 1] = (int32_t)acc;
            }
            if (!S.cols[c].values.reserve((size_t)acc + 8)) {
                S.code = DFMI_ERR_DEVICE;
                S.msg = "hipHostMalloc failed for a CSV batch";
                return;
            }
        }
        bool any_utf8 = false;
        for (int c = 0; c < nc; ++c) any_utf8 |= types[c] == DFMI_TYPE_UTF8;
        if (any_utf8) {
            auto pass2 = [&](int t) {
                int64_t a, b;
                range(t, a, b);
                std::vector<Field> f(std::max(1, nc));
                for (int64_t r = a; r < b; ++r) {
                    split_record(data + rec_b[r0 + r], data + rec_e[r0 + r], nc, f.data());
                    for (int c = 0; c < nc; ++c)
                        if (types[c] == DFMI_TYPE_UTF8)
                            field_copy(f[c], S.cols[c].values.p + ((int32_t*)S.cols[c].offsets.p)[r]);
                }
            };
            run(nt, pass2);
        }
        for (int c = 0; c < nc; ++c) {
            int64_t nn = 0;
            for (int t = 0; t < nt; ++t) nn += nulls[(size_t)t * nc + c];
            dfmi_column& v = S.view[c];
            v.type = types[c];
            v.length = n;
            v.null_count = types[c] == DFMI_TYPE_UTF8 ? 0 : nn;  // a null Utf8 field reads as "" (no validity)
            v.validity = (types[c] != DFMI_TYPE_UTF8 && nn) ? S.cols[c].validity.p : nullptr;
            v.values = S.cols[c].values.p;
            v.offsets = types[c] == DFMI_TYPE_UTF8 ? (const int32_t*)S.cols[c].offsets.p : nullptr;
        }
    }

    template <class F>
    void run(int nt, F& f) {
        std::vector<std::thread> th;
        for (int t = 1; t < nt; ++t) th.emplace_back([&, t] { f(t); });
        f(0);
        for (auto& x : th) x.join();
    }

    void start_prefetch(int set) {
        const size_t r0 = next_row;
        const int64_t n = (int64_t)std::min<size_t>((size_t)batch_size, n_rec - r0);
        next_row = r0 + (size_t)n;
        prefetching = true;
        prefetch = std::thread([this, set, r0, n] { parse(sets[set], r0, n); });
    }
};

// Parse threads when the caller names none: the CPUs this process may run
// on (its affinity mask, not the machine's count), capped by
// OMP_NUM_THREADS when the host sets one (a shared box's CPU share) and at 64.
static int default_parse_threads() {
    int n = (int)std::thread::hardware_concurrency();
    cpu_set_t cs;
    if (sched_getaffinity(0, sizeof cs, &cs) == 0) n = CPU_COUNT(&cs);
    if (const char* e = getenv("OMP_NUM_THREADS"))
        if (atoi(e) > 0) n = std::min(n, atoi(e));
    return std::max(1, std::min(n, 64));
}

extern "C" int32_t dfmi_csv_open(const char* path, const dfmi_schema* schema, int32_t has_header, int64_t batch_size,
                                 int32_t threads, dfmi_csv_reader** out, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    if (!path || !schema || !out || batch_size <= 0 || (schema->num_fields > 0 && !schema->fields)) {
        set_err(err, DFMI_ERR_INVALID_ARGUMENT, "bad argument");
        return DFMI_ERR_INVALID_ARGUMENT;
    }
    *out = nullptr;
    dfmi_csv_reader* R = new dfmi_csv_reader();
    for (int i = 0; i < schema->num_fields; ++i) {
        const int t = schema->fields[i].type;
        if (t != DFMI_TYPE_UTF8 && t != DFMI_TYPE_BOOLEAN && !width_of(t)) {
            delete R;
            set_err(err, DFMI_ERR_NOT_IMPLEMENTED, "CSV column type");
            return DFMI_ERR_NOT_IMPLEMENTED;
        }
        R->types.push_back(t);
    }
    R->batch_size = batch_size;
    if (threads <= 0)
        if (const char* e = getenv("DFMI_CSV_THREADS")) threads = atoi(e);
    R->threads = threads > 0 ? std::min(threads, 64) : default_parse_threads();
    R->fd = open(path, O_RDONLY);
    if (R->fd < 0) {
        const std::string m = std::string(path) + ": " + strerror(errno);
        delete R;
        set_err(err, DFMI_ERR_GENERAL, "IoError: " + m);  // ExecutionError::IoError (error.rs:27)
        return DFMI_ERR_GENERAL;
    }
    struct stat st;
    fstat(R->fd, &st);
    R->size = (size_t)st.st_size;
    if (R->size) {
        void* m = mmap(nullptr, R->size, PROT_READ, MAP_PRIVATE, R->fd, 0);
        if (m == MAP_FAILED) {
            delete R;
            set_err(err, DFMI_ERR_GENERAL, "IoError: mmap failed");
            return DFMI_ERR_GENERAL;
        }
        R->data = (const char*)m;
        madvise(m, R->size, MADV_SEQUENTIAL);
        try {
            R->index_records(has_header != 0);
        } catch (const std::bad_alloc&) {
            delete R;
            set_err(err, DFMI_ERR_GENERAL, "out of host memory indexing the CSV file");
            return DFMI_ERR_GENERAL;
        }
    }
    if (R->next_row < R->n_rec) R->start_prefetch(0);
    *out = R;
    return DFMI_OK;
}

extern "C" int32_t dfmi_csv_next(dfmi_csv_reader* R, dfmi_batch* out, int32_t* has_batch, dfmi_error* err) {
    set_err(err, DFMI_OK, "");
    if (!R || !out || !has_batch) {
        set_err(err, DFMI_ERR_INVALID_ARGUMENT, "NULL argument");
        return DFMI_ERR_INVALID_ARGUMENT;
    }
    *has_batch = 0;
    if (!R->prefetching) return DFMI_OK;  // end of the file
    R->prefetch.join();
    R->prefetching = false;
    const int set = R->cur;
    BatchSet& S = R->sets[set];
    if (S.code != DFMI_OK) {
        set_err(err, S.code, S.msg);
        return S.code;
    }
    R->cur ^= 1;
    if (R->next_row < R->n_rec) R->start_prefetch(R->cur);  // batch i+1 while the caller runs batch i
    out->num_columns = (int32_t)R->types.size();
    out->reserved = 0;
    out->num_rows = S.rows;
    out->columns = S.view.data();
    *has_batch = 1;
    return DFMI_OK;
}

extern "C" int64_t dfmi_csv_num_records(const dfmi_csv_reader* R) { return R ? (int64_t)(R->n_rec - R->rec0) : -1; }

extern "C" void dfmi_csv_close(dfmi_csv_reader* R) { delete R; }
