// Host-code sanitizer driver (TEST INFRASTRUCTURE): the library's host-only
// front ends -- the expression compiler (csrc/compile.cpp) and the CSV
// reader (csrc/csv_reader.cpp) -- plus the CPU oracle, built with
// AddressSanitizer + UndefinedBehaviorSanitizer and driven over random
// expressions, random batches and generated CSV files (quotes, CRLF, empty
// and missing fields, bad numbers). Exit 0 = no finding; the sanitizers
// abort on the first one. Built and run by tests/test_sanitize_cpu.py.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../include/dfmi.h"
#include "../../include/dfmi_datasource.h"
#include "../../oracle/oracle.h"

namespace {

std::mt19937_64 rng(7);
int rnd(int n) { return (int)(rng() % (uint64_t)n); }

const int kTypes[] = {DFMI_TYPE_INT64, DFMI_TYPE_FLOAT64, DFMI_TYPE_INT32, DFMI_TYPE_FLOAT32, DFMI_TYPE_UTF8,
                      DFMI_TYPE_BOOLEAN, DFMI_TYPE_UINT8};
constexpr int kCols = 7;

// A random postfix expression over the schema (any shape: the compilers
// must reject what the reference rejects without misbehaving).
void gen(std::vector<dfmi_expr_node>& out, int depth, std::vector<std::string>& strs) {
    dfmi_expr_node nd;
    memset(&nd, 0, sizeof nd);
    const int r = rnd(10);
    if (depth == 0 || r < 3) {
        if (rnd(2)) {
            nd.kind = DFMI_EXPR_COLUMN;
            nd.column = rnd(kCols + 1) - (rnd(20) == 0 ? 3 : 0);  // sometimes out of range
        } else {
            nd.kind = DFMI_EXPR_LITERAL;
            nd.data_type = 1 + rnd(12);
            nd.i64 = (int64_t)rng();
            nd.f64 = (double)(int64_t)rng() / 1e9;
            if (nd.data_type == DFMI_TYPE_UTF8) {
                strs.push_back(std::string(rnd(6), 'a' + rnd(3)));
                nd.str = strs.back().c_str();
                nd.str_len = (int64_t)strs.back().size();
            }
        }
        out.push_back(nd);
        return;
    }
    if (r < 8) {
        gen(out, depth - 1, strs);
        gen(out, depth - 1, strs);
        nd.kind = DFMI_EXPR_BINARY;
        nd.op = rnd(13);
    } else if (r < 9) {
        gen(out, depth - 1, strs);
        nd.kind = DFMI_EXPR_CAST;
        nd.data_type = 1 + rnd(12);
    } else {
        gen(out, depth - 1, strs);
        nd.kind = rnd(2) ? DFMI_EXPR_IS_NULL : DFMI_EXPR_IS_NOT_NULL;
    }
    out.push_back(nd);
}

int check_expressions() {
    dfmi_field fields[kCols];
    const char* names[kCols] = {"i", "f", "i32", "f32", "s", "b", "u8"};
    for (int c = 0; c < kCols; ++c) fields[c] = {names[c], kTypes[c], 1};
    dfmi_schema schema = {kCols, 0, fields};
    // a random 300-row batch with nulls
    const int n = 300;
    std::vector<int64_t> vi(n);
    std::vector<double> vf(n);
    std::vector<int32_t> vi32(n), offs(n + 1);
    std::vector<float> vf32(n);
    std::vector<uint8_t> vu8(n), bits((n + 63) / 64 * 8), valid((n + 63) / 64 * 8);
    std::string bytes;
    for (int r = 0; r < n; ++r) {
        vi[r] = (int64_t)rng() >> rnd(60);
        vf[r] = (double)(int64_t)rng() / 1e12;
        vi32[r] = (int32_t)rng();
        vf32[r] = (float)vf[r];
        vu8[r] = (uint8_t)rng();
        offs[r] = (int32_t)bytes.size();
        bytes += std::string(rnd(5), 'a' + rnd(3));
        if (rnd(2)) bits[r / 8] |= (uint8_t)(1 << (r % 8));
        if (rnd(10)) valid[r / 8] |= (uint8_t)(1 << (r % 8));
    }
    offs[n] = (int32_t)bytes.size();
    dfmi_column cols[kCols];
    memset(cols, 0, sizeof cols);
    const void* vals[kCols] = {vi.data(), vf.data(), vi32.data(), vf32.data(), bytes.data(), bits.data(), vu8.data()};
    for (int c = 0; c < kCols; ++c) {
        cols[c].type = kTypes[c];
        cols[c].length = n;
        cols[c].values = vals[c];
        cols[c].validity = c % 2 ? valid.data() : nullptr;
        cols[c].null_count = c % 2 ? 30 : 0;
        cols[c].offsets = kTypes[c] == DFMI_TYPE_UTF8 ? offs.data() : nullptr;
    }
    dfmi_batch batch = {kCols, 0, n, cols};
    int compiled = 0;
    for (int it = 0; it < 3000; ++it) {
        std::vector<dfmi_expr_node> nodes;
        std::vector<std::string> strs;
        strs.reserve(64);
        gen(nodes, 1 + rnd(4), strs);
        const uint32_t flags = (uint32_t)rnd(32);
        dfmi_program* prog = nullptr;
        dfmi_error err;
        if (dfmi_compile_scalar_expr(nodes.data(), (int32_t)nodes.size(), &schema, flags, &prog, &err) == DFMI_OK) {
            ++compiled;
            (void)dfmi_program_name(prog);
            dfmi_program_free(prog);
        }
        char name[256];
        int32_t type = 0;
        (void)oracle_compile_info(nodes.data(), (int32_t)nodes.size(), &schema, flags, name, sizeof name, &type, &err);
        // the oracle evaluates it as a predicate and as a projection
        const dfmi_expr_node* pn[1] = {nodes.data()};
        const int32_t pl[1] = {(int32_t)nodes.size()};
        oracle_result* res = nullptr;
        if (oracle_filter_project(nodes.data(), (int32_t)nodes.size(), pn, pl, 1, &schema, &batch, flags, &res, &err) ==
            DFMI_OK)
            oracle_result_free(res);
        res = nullptr;
        if (oracle_filter_project(nullptr, 0, pn, pl, 1, &schema, &batch, flags, &res, &err) == DFMI_OK) {
            dfmi_column v;
            const char* nm = nullptr;
            for (int i = 0; i < oracle_result_num_columns(res); ++i) oracle_result_column(res, i, &v, &nm);
            oracle_result_free(res);
        }
    }
    printf("expressions: 3000 generated, %d compiled\n", compiled);
    return 0;
}

std::string cell(int t) {
    if (rnd(12) == 0) return "";
    if (rnd(200) == 0) return "x?";  // a parse error now and then
    switch (t) {
        case DFMI_TYPE_UTF8: {
            std::string s;
            for (int i = rnd(8); i > 0; --i) s += "ab,\"x\n"[rnd(6)];
            if (s.find_first_of(",\"\n") != std::string::npos || rnd(4) == 0) {
                std::string q = "\"";
                for (char ch : s) q += ch == '"' ? std::string("\"\"") : std::string(1, ch);
                return q + "\"";
            }
            return s;
        }
        case DFMI_TYPE_BOOLEAN: return rnd(2) ? "true" : "FALSE";
        case DFMI_TYPE_FLOAT64: case DFMI_TYPE_FLOAT32: return std::to_string((double)(int64_t)rng() / 1e9);
        case DFMI_TYPE_UINT8: return std::to_string(rnd(256));
        default: return std::to_string((int32_t)rng());
    }
}

int check_csv() {
    dfmi_field fields[kCols];
    const char* names[kCols] = {"i", "f", "i32", "f32", "s", "b", "u8"};
    for (int c = 0; c < kCols; ++c) fields[c] = {names[c], kTypes[c], 1};
    dfmi_schema schema = {kCols, 0, fields};
    long batches = 0, errors = 0;
    for (int file = 0; file < 12; ++file) {
        char path[64];
        snprintf(path, sizeof path, "/tmp/dfmi_sanitize_%d.csv", file);
        FILE* f = fopen(path, "wb");
        if (!f) return 1;
        const int rows = 1 + rnd(3000);
        const char* nl = file % 2 ? "\r\n" : "\n";
        for (int r = 0; r < rows; ++r) {
            int nc = rnd(30) ? kCols : 1 + rnd(kCols);  // missing trailing fields
            for (int c = 0; c < nc; ++c) fprintf(f, "%s%s", c ? "," : "", cell(kTypes[c]).c_str());
            fputs(rnd(40) ? nl : "", f);  // sometimes no terminator (last line / joined line)
            if (rnd(50) == 0) fputs(nl, f);  // empty record
        }
        fclose(f);
        for (int bs : {1, 3, 64, 1000}) {
            for (int th : {1, 3}) {
                dfmi_csv_reader* R = nullptr;
                dfmi_error err;
                if (dfmi_csv_open(path, &schema, file % 3 == 0, bs, th, &R, &err) != DFMI_OK) return 2;
                while (true) {
                    dfmi_batch b;
                    int32_t has = 0;
                    if (dfmi_csv_next(R, &b, &has, &err) != DFMI_OK) {
                        ++errors;
                        break;
                    }
                    if (!has) break;
                    ++batches;
                    volatile uint64_t acc = 0;  // touch every buffer the batch exposes
                    for (int c = 0; c < b.num_columns; ++c) {
                        const dfmi_column& col = b.columns[c];
                        if (col.type == DFMI_TYPE_UTF8) {
                            for (int64_t r = 0; r <= col.length; ++r) acc += (uint64_t)col.offsets[r];
                            for (int32_t i = 0; i < col.offsets[col.length]; ++i) acc += ((const uint8_t*)col.values)[i];
                        } else if (col.type == DFMI_TYPE_BOOLEAN) {
                            for (int64_t i = 0; i < (col.length + 7) / 8; ++i) acc += ((const uint8_t*)col.values)[i];
                        } else {
                            const int w = col.type == DFMI_TYPE_UINT8 ? 1 : (col.type == DFMI_TYPE_INT32 || col.type == DFMI_TYPE_FLOAT32 ? 4 : 8);
                            for (int64_t i = 0; i < col.length * w; ++i) acc += ((const uint8_t*)col.values)[i];
                        }
                        if (col.validity)
                            for (int64_t i = 0; i < (col.length + 7) / 8; ++i) acc += col.validity[i];
                    }
                }
                dfmi_csv_close(R);
            }
        }
        remove(path);
    }
    printf("csv: %ld batches read, %ld parse errors raised\n", batches, errors);
    return 0;
}

}  // namespace

int main() {
    if (int rc = check_expressions()) return rc;
    if (int rc = check_csv()) return rc;
    printf("sanitize driver: clean\n");
    return 0;
}
