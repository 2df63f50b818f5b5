// Query compiler: writes the query's Selection + Projection as one
// straight-line gfx950 kernel over the hand-written skeleton
// (jit_skeleton.hip), compiles it with hipRTC once per query shape and
// launches it. Replaces the per-row interpretation of the reference's
// compiled closures (expression.rs:29-451, filter.rs:80-111) -- and of an
// earlier device interpreter here, whose per-operator decode made the pass
// scalar-issue bound (DESIGN.md "Kernels").
//
// Shape of every generated kernel (filtered form):
//   1. load the predicate's columns for the thread's K rows (all loads first);
//   2. evaluate the predicate per row -> selection bits;
//   3. lane-masked loads of projection-only columns (only where selected);
//   4. ballot / per-(k,wave) counts, tile scan, decoupled look-back;
//   5. evaluate projections, store compacted rows; Utf8 gathers.
// Literal values and buffer addresses are kernel arguments, so one binary
// serves every instance of a query shape.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "dfmi_program.h"
#include "jit.h"

extern const char dfmi_skeleton_src[];  // jit_skeleton.hip, embedded by the Makefile
namespace {
const std::string& skeleton_text() {
    static const std::string s(dfmi_skeleton_src);
    return s;
}
}  // namespace

namespace dfmi {
namespace jit {

namespace {

const char* cmp_sym(int op) {
    static const char* s[] = {"==", "!=", "<", "<=", ">", ">="};
    return s[op];
}
const char* math_sym(int op) {
    static const char* s[] = {"+", "-", "*", "/"};
    return s[op - DFMI_OP_PLUS];
}

bool is_float(int t) { return t == DFMI_TYPE_FLOAT32 || t == DFMI_TYPE_FLOAT64; }
bool is_signed_int(int t) { return t >= DFMI_TYPE_INT8 && t <= DFMI_TYPE_INT64; }

// Casts num::cast can never reject: int -> float, Float32 -> Float64, and an
// integer into a type holding all of its values.
bool cast_total(int from, int to) {
    if (is_float(to)) return !is_float(from) || type_width(from) <= type_width(to);
    if (is_float(from)) return false;
    const int wf = type_width(from), wt = type_width(to);
    if (is_signed_int(from) == is_signed_int(to)) return wt >= wf;
    return !is_signed_int(from) && wt > wf;  // unsigned into a wider signed type
}

// Unsigned type integer math is done in (Rust's wrapping +, -, * on every
// width; C++ signed overflow is undefined and u16 * u16 would promote to int).
const char* math_type(int t) { return type_width(t) == 8 ? "u64" : "u32"; }

struct Val {
    std::string v;  // C++ expression / local of the node's C++ type (ctype), or bool
    std::string n;  // validity expression ("true" when statically valid)
};

}  // namespace

int type_width(int t) {
    switch (t) {
        case DFMI_TYPE_INT8: case DFMI_TYPE_UINT8: return 1;
        case DFMI_TYPE_INT16: case DFMI_TYPE_UINT16: return 2;
        case DFMI_TYPE_INT32: case DFMI_TYPE_UINT32: case DFMI_TYPE_FLOAT32: return 4;
        case DFMI_TYPE_INT64: case DFMI_TYPE_UINT64: case DFMI_TYPE_FLOAT64: return 8;
        default: return 0;
    }
}

bool may_introduce_nulls(const dfmi_program* p) {
    for (const IrNode& n : p->ir)
        if (n.kind == IR_CAST && !cast_total(p->ir[n.l].type, n.type)) return true;
    return false;
}

const char* ctype(int t) {
    switch (t) {
        case DFMI_TYPE_INT8: return "i8";
        case DFMI_TYPE_INT16: return "i16";
        case DFMI_TYPE_INT32: return "i32";
        case DFMI_TYPE_INT64: return "i64";
        case DFMI_TYPE_UINT8: return "u8";
        case DFMI_TYPE_UINT16: return "u16";
        case DFMI_TYPE_UINT32: return "u32";
        case DFMI_TYPE_FLOAT32: return "float";
        case DFMI_TYPE_FLOAT64: return "double";
        default: return "u64";
    }
}

// ------------------------------------------------------------- generator
struct Gen {
    const Plan& P;
    Launch& X;  // slot tables + Args being filled
    std::ostringstream o;
    int tmp = 0;
    bool filtered_cols = false;  // projection after a Selection: columns all-valid
    std::string sfx;             // name suffix of the register set being evaluated
    // predicate loop of a filtered tile: Utf8 `col = literal` comparisons are
    // evaluated tile-wide before the loop (utf8_eq_lit_tile); each entry is
    // (array name, utf8 slot, string literal index)
    bool tile_pre = false;
    std::vector<std::tuple<std::string, int, int>> pre_eq;

    Gen(const Plan& p, Launch& x) : P(p), X(x) {}

    std::string t() { return "t" + std::to_string(tmp++); }

    // one slot per literal node (no sharing of equal values: the source text,
    // and so the compiled kernel, must not depend on literal values)
    int lit(uint64_t b) {
        if (X.n_lits >= 32) throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "query compiler: too many literals"};
        X.args_lits[X.n_lits] = b;
        return X.n_lits++;
    }
    int strlit(const std::string& s) {
        if (X.n_str >= 8 || X.str_bytes + (int)s.size() > 256)
            throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "query compiler: string literals too long"};
        X.str_off[X.n_str] = X.str_bytes;
        X.str_len[X.n_str] = (int)s.size();
        memcpy(X.str + X.str_bytes, s.data(), s.size());
        X.str_bytes += (int)s.size();
        return X.n_str++;
    }

    // column value for the current row k (inside a per-k loop)
    Val col(const IrNode& n) {
        const int s = X.slot_of_col(n.col);
        const std::string id = std::to_string(s) + sfx;
        Val r;
        if (n.type == DFMI_TYPE_BOOLEAN) {
            r.v = "(((bw" + id + "[k] >> lane) & 1) != 0)";
        } else {
            r.v = "c" + id + "[k]";
        }
        r.n = (!filtered_cols && X.col_nullable(n.col)) ? "(((vw" + id + "[k] >> lane) & 1) != 0)" : "true";
        return r;
    }

    // Literal slot read as a value of type t (the slot holds the raw bits:
    // Float32 in the low 32 bits, integers sign/zero-extended).
    static std::string lit_value(int t, int slot) {
        const std::string a = "A.lits[" + std::to_string(slot) + "]";
        if (t == DFMI_TYPE_FLOAT64) return "__builtin_bit_cast(double, " + a + ")";
        if (t == DFMI_TYPE_FLOAT32) return "__builtin_bit_cast(float, (u32)" + a + ")";
        return "((" + std::string(ctype(t)) + ")" + a + ")";
    }

    // Emit node i of program p; act = C++ bool expression "row is evaluated".
    Val emit(const dfmi_program* p, int i, int ord_base, const char* act) {
        const IrNode& n = p->ir[i];
        if (n.kind == IR_COL) {
            if (n.type == DFMI_TYPE_UTF8) {  // value only inside Utf8 compares; validity for IS NULL
                if (filtered_cols || !X.col_nullable(n.col)) return Val{"", "true"};
                return Val{"", "dfmi::utf8_valid(A, " + std::to_string(X.slot_of_utf8(n.col)) + ", row)"};
            }
            if (!type_width(n.type) && n.type != DFMI_TYPE_BOOLEAN)
                throw Fail{DFMI_ERR_NOT_IMPLEMENTED,
                           std::string("device path: ") + type_debug(n.type) + " column in an expression"};
            return col(n);
        }
        if (n.kind == IR_LIT) {
            if (n.type == DFMI_TYPE_UTF8) return Val{"", "true"};
            if (!type_width(n.type))
                throw Fail{DFMI_ERR_NOT_IMPLEMENTED, std::string("device path: ") + type_debug(n.type) + " literal"};
            return Val{lit_value(n.type, lit(n.bits)), "true"};
        }
        if (n.kind == IR_ISNULL) {  // extension: the operand's validity, never null
            const Val a = emit(p, n.l, ord_base, act);
            if (a.n == "true") return Val{n.op == 0 ? "false" : "true", "true"};
            const std::string v = t();
            o << "    const bool " << v << " = " << (n.op == 0 ? "!" : "") << "(" << a.n << ");\n";
            return Val{v, "true"};
        }
        if (n.kind == IR_CAST) {  // extension: arrow cast kernel, unfit values -> null
            const Val a = emit(p, n.l, ord_base, act);
            const int from = p->ir[n.l].type, to = n.type;
            if (from == to) return a;
            const std::string v = t();
            o << "    " << ctype(to) << " " << v << ";\n";
            if (cast_total(from, to)) {
                o << "    (void)dfmi::num_cast<" << ctype(to) << ">(" << a.v << ", " << v << ");\n";
                if (a.n != "true") o << "    if (!(" << a.n << ")) " << v << " = (" << ctype(to) << ")0;\n";
                return Val{v, a.n};
            }
            o << "    const bool " << v << "_n = dfmi::num_cast<" << ctype(to) << ">(" << a.v << ", " << v << ")"
              << (a.n != "true" ? " && (" + a.n + ")" : "") << ";\n";
            o << "    if (!" << v << "_n) " << v << " = (" << ctype(to) << ")0;\n";
            return Val{v, v + "_n"};
        }
        const int ord = ord_base + n.ordinal;
        if (n.rt_code) {
            // the reference evaluates both children before failing here
            try {
                emit(p, n.l, ord_base, act);
                emit(p, n.r, ord_base, act);
            } catch (const Fail&) {
            }
            if (n.type == DFMI_TYPE_BOOLEAN) return Val{"false", "true"};
            return Val{"((" + std::string(ctype(n.type)) + ")0)", "true"};
        }
        const int op = n.op;
        const IrNode& L = p->ir[n.l];
        if (L.type == DFMI_TYPE_UTF8 && op <= DFMI_OP_GT_EQ) {  // extension: Utf8 =, !=
            const IrNode& R = p->ir[n.r];
            const bool eq = op == DFMI_OP_EQ;
            const std::string v = t();
            if (L.kind == IR_LIT && R.kind == IR_LIT) {
                o << "    const bool " << v << " = " << (((L.str == R.str) == eq) ? "true" : "false") << ";\n";
            } else if (L.kind == IR_COL && R.kind == IR_COL) {
                const int u = X.slot_of_utf8(L.col), w = X.slot_of_utf8(R.col);
                const std::string vu = filtered_cols ? "true" : "dfmi::utf8_valid(A, " + std::to_string(u) + ", row)";
                const std::string vw = filtered_cols ? "true" : "dfmi::utf8_valid(A, " + std::to_string(w) + ", row)";
                o << "    bool " << v << ";\n    { const bool a_ = " << vu << ", b_ = " << vw << ";\n"
                  << "      const bool e_ = (a_ && b_) ? dfmi::utf8_eq_col(A, " << u << ", " << w << ", row) : (!a_ && !b_);\n"
                  << "      " << v << " = " << (eq ? "e_" : "!e_") << "; }\n";
            } else {
                const IrNode& C = L.kind == IR_COL ? L : R;
                const IrNode& S = L.kind == IR_COL ? R : L;
                const int u = X.slot_of_utf8(C.col);
                const int sl = strlit(S.str);
                const std::string vu = filtered_cols ? "true" : "dfmi::utf8_valid(A, " + std::to_string(u) + ", row)";
                if (tile_pre) {
                    const std::string arr = "uq" + std::to_string(pre_eq.size()) + sfx;
                    pre_eq.emplace_back(arr, u, sl);
                    o << "    const bool " << v << "_e = " << vu << " && " << arr << "[k];\n";
                } else {
                    o << "    const bool " << v << "_e = " << vu << " && dfmi::utf8_eq_lit(A, " << u << ", row, " << sl
                      << ", A0.str + A0.str_off[" << sl << "]);\n";
                }
                o << "    const bool " << v << " = " << (eq ? "" : "!") << v << "_e;\n";
            }
            return Val{v, "true"};
        }
        const Val a = emit(p, n.l, ord_base, act);
        const Val b = emit(p, n.r, ord_base, act);
        const bool nul = a.n != "true" || b.n != "true";
        if (op == DFMI_OP_AND || op == DFMI_OP_OR) {
            const std::string v = t();
            const std::string nn = nul ? "(" + a.n + " && " + b.n + ")" : "true";
            o << "    const bool " << v << "_n = " << nn << ";\n";
            o << "    const bool " << v << " = " << v << "_n && (" << a.v << (op == DFMI_OP_AND ? " && " : " || ")
              << b.v << ");\n";  // null -> zero value bit (append_null)
            return Val{v, nul ? v + "_n" : "true"};
        }
        // same-typed operands (anything else carries rt_code): compare / compute
        // in the operand type -- iN/uN wrap, Float32 and Float64 round once per
        // operator (-ffp-contract=off)
        const int ty = L.type;
        const bool f = is_float(ty);
        const std::string ct = ctype(ty);
        const std::string v = t();
        if (op <= DFMI_OP_GT_EQ) {
            const std::string cmp = "(" + a.v + ") " + cmp_sym(op) + " (" + b.v + ")";
            if (nul) {
                o << "    const bool " << v << " = dfmi::cmp_opt<" << op << ">(" << a.n << ", " << b.n << ", " << cmp
                  << ");\n";
            } else {
                o << "    const bool " << v << " = " << cmp << ";\n";
            }
            return Val{v, "true"};
        }
        // math: null if either side is null (zero slot), one rounding per op
        const std::string nn = nul ? "(" + a.n + " && " + b.n + ")" : "true";
        if (nul) o << "    const bool " << v << "_n = " << nn << ";\n";
        const std::string valid = nul ? v + "_n" : "true";
        if (op == DFMI_OP_DIVIDE) {
            o << "    if ((" << act << ") && " << valid << ") {\n"
              << "      if ((" << b.v << ") == (" << ct << ")0) dfmi::report_err(A.err, " << ord
              << ", row, dfmi::ERRK_DIV_ZERO);\n";
            if (is_signed_int(ty))
                o << "      else if ((" << b.v << ") == (" << ct << ")-1 && (" << a.v << ") == dfmi::int_min<" << ct
                  << ">()) dfmi::report_err(A.err, " << ord << ", row, dfmi::ERRK_DIV_OVERFLOW);\n";
            o << "    }\n";
            if (f)
                o << "    " << ct << " " << v << " = dfmi::sse_nan<" << ct << ">((" << a.v << ") / (" << b.v << "), "
                  << a.v << ", " << b.v << ");\n";
            else
                o << "    " << ct << " " << v << " = dfmi::idiv<" << ct << ">(" << a.v << ", " << b.v << ");\n";
        } else if (f) {
            o << "    " << ct << " " << v << " = dfmi::sse_nan<" << ct << ">((" << a.v << ") " << math_sym(op) << " ("
              << b.v << "), " << a.v << ", " << b.v << ");\n";
        } else {
            const char* mt = math_type(ty);
            o << "    " << ct << " " << v << " = (" << ct << ")((" << mt << ")(" << a.v << ") " << math_sym(op) << " ("
              << mt << ")(" << b.v << "));\n";
        }
        if (nul) o << "    if (!" << v << "_n) " << v << " = (" << ct << ")0;\n";
        return Val{v, valid};
    }
};

// ------------------------------------------------------------ compile cache
// Loaded code objects, keyed by device + source text, bounded (least recently
// used evicted past the cap). A module is unloaded when the last holder lets
// go: the cache, and every Launch that got its kernel from get_kernel
// (Launch::module) -- so a launch in flight keeps its code object loaded.
// The map itself is never destroyed: modules still cached at process exit
// are left to the runtime's teardown, as before the bound.
namespace {
struct Compiled {
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;
    ~Compiled() {
        if (mod) (void)hipModuleUnload(mod);
    }
};
struct CacheEntry {
    std::shared_ptr<Compiled> c;
    uint64_t used = 0;
};
std::mutex g_mu;
auto& g_cache = *new std::map<std::string, CacheEntry>();  // guarded by g_mu
uint64_t g_tick = 0;
size_t g_cap = [] {
    const char* e = getenv("DFMI_JIT_CACHE_MODULES");
    return e && atoi(e) > 0 ? (size_t)atoi(e) : (size_t)256;
}();
// caller holds g_mu
void evict_to(size_t cap) {
    while (g_cache.size() > cap) {
        auto lru = g_cache.begin();
        for (auto it = g_cache.begin(); it != g_cache.end(); ++it)
            if (it->second.used < lru->second.used) lru = it;
        g_cache.erase(lru);
    }
}
}  // namespace

// ------------------------------------------------------- on-disk code objects
// A process's first call of a query shape would pay the hipRTC compile
// (~190 ms); the reference's compile_scalar_expr is a closure build
// (context.rs:131,152-155). Code objects are therefore also kept on disk,
// keyed by a hash of the generated source, the compile options, the hipRTC
// version and the target: DFMI_JIT_CACHE_DIR (empty: off), else
// $XDG_CACHE_HOME/dfmi-jit, else $HOME/.cache/dfmi-jit. A file holds the full
// source it was compiled from and is used only when that source matches
// byte for byte (a hash collision cannot load the wrong code); files are
// written to a temporary name and renamed, so a reader never sees a partial
// one, and a damaged or foreign file is ignored (compiled again).
namespace {
const char* const kOpts[] = {"--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17",
                             "-Wno-unused-variable", "-Wno-unused-but-set-variable"};

const std::string& disk_dir() {
    static const std::string dir = [] {
        std::string d;
        if (const char* e = getenv("DFMI_JIT_CACHE_DIR")) {
            d = e;  // "" disables
        } else if (const char* x = getenv("XDG_CACHE_HOME"); x && *x) {
            d = std::string(x) + "/dfmi-jit";
        } else if (const char* h = getenv("HOME"); h && *h) {
            d = std::string(h) + "/.cache/dfmi-jit";
        }
        if (!d.empty()) {  // mkdir -p
            for (size_t i = 1; i <= d.size(); ++i)
                if (i == d.size() || d[i] == '/') (void)::mkdir(d.substr(0, i).c_str(), 0755);
            struct stat st;
            if (::stat(d.c_str(), &st) != 0 || !S_ISDIR(st.st_mode)) d.clear();
        }
        return d;
    }();
    return dir;
}

uint64_t fnv1a(const void* p, size_t n, uint64_t h) {
    const unsigned char* b = (const unsigned char*)p;
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 0x100000001b3ull;
    return h;
}

std::string disk_path(const std::string& src) {
    int maj = 0, min = 0;
    hiprtcVersion(&maj, &min);
    std::string salt = "dfmi-co-1 hiprtc " + std::to_string(maj) + "." + std::to_string(min);
    for (const char* o : kOpts) salt += std::string(" ") + o;
    uint64_t h1 = fnv1a(salt.data(), salt.size(), 0xcbf29ce484222325ull);
    h1 = fnv1a(src.data(), src.size(), h1);
    uint64_t h2 = fnv1a(src.data(), src.size(), 0x84222325cbf29ce4ull ^ src.size());
    h2 = fnv1a(salt.data(), salt.size(), h2);
    char name[64];
    snprintf(name, sizeof name, "/%016llx%016llx.co", (unsigned long long)h1, (unsigned long long)h2);
    return disk_dir() + name;
}

constexpr char kMagic[8] = {'D', 'F', 'M', 'I', 'C', 'O', '1', '\n'};

bool disk_load(const std::string& path, const std::string& src, std::vector<char>& code) {
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return false;
    bool ok = false;
    char magic[8];
    uint64_t ns = 0, nc = 0;
    if (fread(magic, 1, 8, f) == 8 && !memcmp(magic, kMagic, 8) && fread(&ns, 8, 1, f) == 1 && ns == src.size()) {
        std::string s(ns, '\0');
        if (fread(&s[0], 1, ns, f) == ns && s == src && fread(&nc, 8, 1, f) == 1 && nc > 0 && nc < ((uint64_t)1 << 30)) {
            code.resize(nc);
            ok = fread(code.data(), 1, nc, f) == nc && fgetc(f) == EOF;
        }
    }
    fclose(f);
    return ok;
}

void disk_store(const std::string& path, const std::string& src, const std::vector<char>& code) {
    char tmp[64];
    snprintf(tmp, sizeof tmp, ".tmp.%d.%llx", (int)getpid(),
             (unsigned long long)std::chrono::steady_clock::now().time_since_epoch().count());
    const std::string t = path + tmp;
    FILE* f = fopen(t.c_str(), "wb");
    if (!f) return;
    const uint64_t ns = src.size(), nc = code.size();
    bool ok = fwrite(kMagic, 1, 8, f) == 8 && fwrite(&ns, 8, 1, f) == 1 && fwrite(src.data(), 1, ns, f) == ns &&
              fwrite(&nc, 8, 1, f) == 1 && fwrite(code.data(), 1, nc, f) == nc;
    ok = fclose(f) == 0 && ok;
    if (!ok || ::rename(t.c_str(), path.c_str()) != 0) ::unlink(t.c_str());
}
}  // namespace

std::vector<char> compile_code(const std::string& src, double* compile_ms) {
    if (compile_ms) *compile_ms = 0;
    std::string path;
    if (!disk_dir().empty()) {
        path = disk_path(src);
        std::vector<char> code;
        if (disk_load(path, src, code)) return code;  // no compile: *compile_ms stays 0
    }
    std::vector<char> code = compile_code_rtc(src, compile_ms);
    if (!path.empty()) disk_store(path, src, code);
    return code;
}

std::vector<char> compile_code_rtc(const std::string& src, double* compile_ms) {
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "dfmi_query.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
        throw Fail{DFMI_ERR_DEVICE, "hiprtcCreateProgram failed"};
    const auto t0 = std::chrono::steady_clock::now();
    const hiprtcResult rc = hiprtcCompileProgram(prog, (int)(sizeof kOpts / sizeof *kOpts), kOpts);
    if (compile_ms)
        *compile_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (rc != HIPRTC_SUCCESS) {
        size_t n = 0;
        hiprtcGetProgramLogSize(prog, &n);
        std::string log(n, '\0');
        if (n) hiprtcGetProgramLog(prog, &log[0]);
        hiprtcDestroyProgram(&prog);
        if (getenv("DFMI_JIT_DUMP")) fprintf(stderr, "%s\n----\n%s\n", src.c_str(), log.c_str());
        throw Fail{DFMI_ERR_DEVICE, "query compile failed: " + log.substr(0, 400)};
    }
    size_t size = 0;
    hiprtcGetCodeSize(prog, &size);
    std::vector<char> code(size);
    hiprtcGetCode(prog, code.data());
    hiprtcDestroyProgram(&prog);
    return code;
}

static std::shared_ptr<Compiled> compile(int device, const std::string& src, const std::string& name,
                                         double* compile_ms) {
    const std::string key = std::to_string(device) + "\n" + src;
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_cache.find(key);
    if (it != g_cache.end()) {
        it->second.used = ++g_tick;
        return it->second.c;
    }
    const std::vector<char> code = compile_code(src, compile_ms);
    auto c = std::make_shared<Compiled>();
    if (hipModuleLoadData(&c->mod, code.data()) != hipSuccess) {
        c->mod = nullptr;
        throw Fail{DFMI_ERR_DEVICE, "hipModuleLoadData failed"};
    }
    if (hipModuleGetFunction(&c->fn, c->mod, name.c_str()) != hipSuccess)
        throw Fail{DFMI_ERR_DEVICE, "hipModuleGetFunction failed"};
    evict_to(g_cap - 1);
    g_cache[key] = CacheEntry{c, ++g_tick};
    return c;
}

size_t cache_size() {
    std::lock_guard<std::mutex> lk(g_mu);
    return g_cache.size();
}

size_t cache_cap(size_t cap) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (cap > 0) {
        g_cap = cap;
        evict_to(cap);
    }
    return g_cap;
}

// --------------------------------------------------------------- kernels
// Register arrays of the given slots (suffix names a ping-pong set).
static void emit_decls(std::ostream& o, const std::vector<int>& slots, const Launch& X, const std::string& sfx,
                       bool valid_words) {
    for (int s : slots) {
        const int col = X.num_cols[s];
        const int ty = X.col_type(col);
        if (ty == DFMI_TYPE_BOOLEAN)
            o << "  u64 bw" << s << sfx << "[K];\n";
        else
            o << "  " << ctype(ty) << " c" << s << sfx << "[K];\n";
        if (valid_words && X.col_nullable(col)) o << "  u64 vw" << s << sfx << "[K];\n";
    }
}

// Loads of the K rows per thread of the tile at `base` (wave-uniform): a
// branch-free form for full tiles and a guarded one for the last tile. Value
// loads of projection-only slots are lane-masked by `guard` (selected rows).
static void emit_loads(std::ostream& o, const std::vector<int>& slots, const Launch& X, const std::string& sfx,
                       const std::string& base, const char* guard, bool valid_words) {
    if (slots.empty()) return;
    for (int full = 1; full >= 0; --full) {
        o << (full ? "  if (A.n_rows - " + base + " >= BLOCK * K) {\n" : "  } else {\n");
        for (int s : slots) {
            const int col = X.num_cols[s];
            const std::string id = std::to_string(s) + sfx;
            if (X.col_type(col) == DFMI_TYPE_BOOLEAN) {
                o << "#pragma unroll\n    for (int k = 0; k < K; ++k) bw" << id
                  << "[k] = dfmi::bitmap_word((const u8*)A.col[" << s << "], (" << base
                  << " >> 6) + k * WAVES + wave, A.n_rows);\n";
            } else {
                // 64 lanes x width bytes per wave load, contiguous in row order
                std::string g = guard ? std::string(guard) : "";
                if (!full) g = g.empty() ? "(" + base + " + k * BLOCK + tid < A.n_rows)"
                                         : "(" + base + " + k * BLOCK + tid < A.n_rows) && " + g;
                const std::string ct = ctype(X.col_type(col));
                const std::string ld = (X.nt & 1) ? "__builtin_nontemporal_load(p_ + k * BLOCK)" : "p_[k * BLOCK]";
                o << "    { const " << ct << "* p_ = (const " << ct << "*)A.col[" << s << "] + " << base << " + tid;\n"
                  << "#pragma unroll\n      for (int k = 0; k < K; ++k) c" << id << "[k] = "
                  << (g.empty() ? ld + ";" : "(" + g + ") ? " + ld + " : (" + ct + ")0;") << " }\n";
            }
            if (valid_words && X.col_nullable(col)) {
                o << "#pragma unroll\n    for (int k = 0; k < K; ++k) vw" << id << "[k] = dfmi::bitmap_word(A.valid[" << s
                  << "], (" << base << " >> 6) + k * WAVES + wave, A.n_rows);\n";
            }
        }
    }
    o << "  }\n";
}

// Numeric / Boolean slots the outputs read (a sub-tile kernel's output pass
// reloads exactly these for the selected rows).
static std::vector<int> output_slots(const Plan& P, const Launch& X) {
    std::vector<int> out;
    auto add_col = [&](int col) {
        for (size_t s = 0; s < X.num_cols.size(); ++s)
            if (X.num_cols[s] == col && std::find(out.begin(), out.end(), (int)s) == out.end()) out.push_back((int)s);
    };
    for (const OutSpec& os : P.outs) {
        if (os.kind == OutSpec::GATHER) add_col(os.col);
        if (os.kind == OutSpec::EXPR)
            for (const IrNode& nd : os.prog->ir)
                if (nd.kind == IR_COL) add_col(nd.col);
    }
    std::sort(out.begin(), out.end());
    return out;
}

// The predicate of a filtered tile: `unsigned selm` (bit k = row base + k*BLOCK
// + tid selected, mask.value(i)); Utf8 columns' offsets (us<u> / ux<u>) are
// loaded tile-wide in front of the predicate loop -- the predicate's `col =
// literal` compares and the columns in `extra_offs` (Utf8 outputs: their byte
// counts are needed before the look-back, so they share the first memory
// round trip). Returns the Utf8 slots whose offsets are in registers.
static std::vector<int> emit_predicate(Gen& g, std::ostringstream& o, const Plan& P, Launch& X, const std::string& cur,
                                       const std::vector<int>& extra_offs, bool preloaded = false) {
    const std::string head = o.str();
    g.tile_pre = true;
    g.pre_eq.clear();
    o << "  unsigned selm = 0;\n#pragma unroll\n  for (int k = 0; k < K; ++k) {\n";
    o << "    const i64 row = base + k * BLOCK + tid;\n    const bool in = row < A.n_rows;\n";
    const Val r = g.emit(P.pred, P.pred->root, 0, "in");
    if (P.pred->type == DFMI_TYPE_BOOLEAN && !r.v.empty())
        o << "    selm |= (unsigned)(in && (" << r.v << ")) << k;\n";  // mask.value(i)
    o << "  }\n";
    g.tile_pre = false;
    std::vector<int> offs_loaded;
    auto offs_name = [&](int u) { return std::to_string(u) + cur; };
    std::ostringstream pre;
    auto load_offs = [&](int u) {
        if (std::find(offs_loaded.begin(), offs_loaded.end(), u) != offs_loaded.end()) return;
        offs_loaded.push_back(u);
        if (preloaded) return;  // us<u> / ux<u> already in scope (sub-tile prefetch)
        pre << "  int us" << offs_name(u) << "[K], ux" << offs_name(u)
            << "[K];\n  dfmi::utf8_offs_tile<BLOCK, K>(A, " << u << ", base, lane, wave, ~0u, us" << offs_name(u)
            << ", ux" << offs_name(u) << ");\n";
    };
    for (const auto& pe : g.pre_eq) load_offs(std::get<1>(pe));
    for (int u : extra_offs) load_offs(u);
    for (const auto& [arr, u, sl] : g.pre_eq)
        if (X.eq_dense < 0)
            pre << "  bool " << arr << "[K];\n  dfmi::utf8_eq_lit_tile_reg<BLOCK, K, " << -X.eq_dense << ">(A, " << u << ", "
                << sl << ", A0.str + A0.str_off[" << sl << "], us" << offs_name(u) << ", ux" << offs_name(u) << ", lane, "
                << arr << ");\n";
        else if (X.eq_dense)
            pre << "  bool " << arr << "[K];\n  dfmi::utf8_eq_lit_tile_dense<BLOCK, K, " << X.eq_dense << ">(A, " << u << ", "
                << sl << ", A0.str + A0.str_off[" << sl << "], us" << offs_name(u) << ", ux" << offs_name(u) << ", lane, "
                << arr << ", EQA[wave]);\n";
        else
        pre << "  bool " << arr << "[K];\n  dfmi::utf8_eq_lit_tile<BLOCK, K>(A, " << u << ", " << sl << ", A0.str + A0.str_off["
            << sl << "], us" << offs_name(u) << ", ux" << offs_name(u) << ", lane, " << arr << ");\n";
    if (!pre.str().empty()) {  // splice in front of the predicate loop
        const std::string loop = o.str().substr(head.size());
        o.str(head + pre.str() + loop);
        o.seekp(0, std::ios_base::end);
    }
    return offs_loaded;
}

// Numeric slots the aggregates' arguments read (the sub-tile form's
// accumulation passes reload exactly these for the selected rows).
static std::vector<int> agg_arg_slots(const Plan& P, const Launch& X) {
    std::vector<int> out;
    for (const AggSpec& a : P.aggs)
        for (const IrNode& nd : a.prog->ir)
            if (nd.kind == IR_COL)
                for (size_t s = 0; s < X.num_cols.size(); ++s)
                    if (X.num_cols[s] == nd.col && std::find(out.begin(), out.end(), (int)s) == out.end())
                        out.push_back((int)s);
    std::sort(out.begin(), out.end());
    return out;
}

// Fused Selection + Aggregate kernel (DFMI_FLAG_EXT_AGGREGATE): no compaction
// and no look-back -- the selected rows' argument values are reduced in
// registers, the block's partial goes to a global accumulator copy
// (jit_skeleton.hip "aggregate extension"). One tile per block; or, for a
// predicate that selected few rows last time (aggregate.cpp, Launch::M > 1),
// M sub-tiles per block: the predicate passes keep only each wave's ballots
// (LDS) and a list of its selected rows, then one lane per selected row loads
// the arguments and accumulates -- one dependent round of loads for the M
// sub-tiles instead of one per tile (a wave whose list overflows reloads its
// arguments per sub-tile, lane-masked). The kernel also counts the selected
// rows (totals[0]), which the host keeps as the query shape's selectivity.
static void generate_agg(Gen& g, std::ostringstream& o, const Plan& P, Launch& X) {
    const int NA = (int)P.aggs.size();
    int NF = 0;
    for (const AggSpec& a : P.aggs) NF += a.fslot >= 0;
    o << "  constexpr int NA = " << NA << ", NF = " << NF << ";\n";
    o << "  __shared__ dfmi::AggLds<NA, NF> S;\n  const unsigned char is_min[NA] = {";
    for (int j = 0; j < NA; ++j) o << (j ? ", " : "") << (P.aggs[j].fn == DFMI_AGG_MIN ? 1 : 0);
    o << "};\n  const int fslot[NF > 0 ? NF : 1] = {";
    {
        bool any = false;
        for (int j = 0; j < NA; ++j)
            if (P.aggs[j].fslot >= 0) {
                o << (any ? ", " : "") << j;
                any = true;
            }
        if (!any) o << "0";
    }
    o << "};\n";
    o << "  if (wave == 0) dfmi::agg_lds_init<NA, NF>(S, is_min, lane);\n";
    if (P.pred) o << "  __shared__ unsigned NSEL_;\n  if (tid == 0) NSEL_ = 0;\n";
    o << "  const unsigned t = tile_;\n";
    // the reduction of row `row` (selected: `sel`) at register index k
    auto emit_accumulate = [&]() {
        for (int j = 0; j < NA; ++j) {
            const AggSpec& a = P.aggs[j];
            const Val v = g.emit(a.prog, a.prog->root, a.ord_base, "sel");
            const std::string ok = "ok" + std::to_string(j) + "_";
            o << "    { const bool " << ok << " = sel && (" << v.n << ");\n";
            o << "      acnt" << j << " += " << ok << " ? 1u : 0u;\n";
            if (a.fn == DFMI_AGG_SUM && a.fslot < 0) {
                o << "      asum" << j << " += " << ok << " ? (u64)(" << (is_signed_int(a.arg_type) ? "i64" : "u64") << ")("
                  << v.v << ") : 0ull;\n";
            } else if (a.fn == DFMI_AGG_SUM) {
                o << "      afl" << j << " |= " << ok << " ? dfmi::agg_sum_flags(" << v.v << ") : 0u;\n"
                  << "      const bool fin_ = " << ok << " && (dfmi::agg_sum_flags(" << v.v
                  << ") == dfmi::AGGF_NONNEGZERO) && (" << v.v << ") != 0;\n"
                  << "      dfmi::fsum_add(S.limbs[" << a.fslot << "], &S.dlo[" << a.fslot << "], &S.dhi[" << a.fslot
                  << "], (double)(" << v.v << "), fin_, lane);\n";
            } else if (a.fn == DFMI_AGG_MIN || a.fn == DFMI_AGG_MAX) {
                const char* cmp = a.fn == DFMI_AGG_MIN ? "<" : ">";
                o << "      const bool nan_ = dfmi::agg_isnan(" << v.v << ");\n"
                  << "      afl" << j << " |= " << ok
                  << " ? (nan_ ? (unsigned)dfmi::AGGF_NAN : (unsigned)dfmi::AGGF_VALUE) : 0u;\n"
                  << "      if (" << ok << " && !nan_) { const u64 k_ = dfmi::agg_key(" << v.v << "); if (k_ " << cmp
                  << " akey" << j << ") akey" << j << " = k_; }\n";
            }
            o << "    }\n";
        }
    };
    auto emit_acc_decls = [&]() {
        for (int j = 0; j < NA; ++j)
            o << "  unsigned acnt" << j << " = 0, afl" << j << " = 0;\n  u64 asum" << j << " = 0, akey" << j << " = "
              << (P.aggs[j].fn == DFMI_AGG_MIN ? "~0ull" : "0ull") << ";\n";
    };
    // selected rows of this wave's K slices, summed for the host's hint
    auto emit_count = [&]() {
        o << "#pragma unroll\n  for (int k = 0; k < K; ++k) nsel_ += (unsigned)__builtin_popcountll(__ballot((selm >> k) & 1));\n";
    };
    if (X.M > 1 && P.pred) {
        const std::vector<int> arg_slots = agg_arg_slots(P, X);
        o << "  constexpr int M = " << X.M << ";\n  constexpr unsigned CAP_ = 256;\n"
          << "  __shared__ unsigned short SLA[WAVES][CAP_];\n  __shared__ u64 WSA[M * K * WAVES];\n"
          << "  unsigned tot_ = 0, nsel_ = 0;\n";
        emit_acc_decls();
        o << "  dfmi::lds_sync();\n";
        // predicate passes: ballots and the list of selected rows
        o << "  for (int m_ = 0; m_ < M; ++m_) {\n  const i64 base = ((i64)t * M + m_) * (BLOCK * K);\n  {\n";
        g.filtered_cols = false;
        emit_decls(o, X.pred_slots, X, "", true);
        emit_loads(o, X.pred_slots, X, "", "base", nullptr, true);
        emit_predicate(g, o, P, X, "", {});
        o << "#pragma unroll\n  for (int k = 0; k < K; ++k) {\n"
          << "    const u64 w_ = __ballot((selm >> k) & 1);\n"
          << "    if (lane == 0) WSA[(m_ * K + k) * WAVES + wave] = w_;\n"
          << "    if (tot_ + (unsigned)__builtin_popcountll(w_) <= CAP_ && ((w_ >> lane) & 1))\n"
          << "      SLA[wave][tot_ + dfmi::lane_rank(w_)] = (unsigned short)((m_ * K + k) * 64 + lane);\n"
          << "    tot_ += (unsigned)__builtin_popcountll(w_);\n  }\n  }\n  }\n"
          << "  nsel_ = tot_;\n  dfmi::wave_lds_fence();\n";
        // sparse: one lane per selected row
        g.filtered_cols = true;
        o << "  if (tot_ <= CAP_) {\n  for (unsigned r_ = 0; r_ < tot_; r_ += 64) {\n"
          << "    const bool sel = r_ + (unsigned)lane < tot_;\n"
          << "    const unsigned e_ = sel ? (unsigned)SLA[wave][r_ + lane] : 0u;\n"
          << "    const int q_ = (int)(e_ >> 6), ls_ = (int)(e_ & 63u);\n"
          << "    const i64 row = ((i64)t * M + q_ / K) * (BLOCK * K) + (i64)(q_ % K) * BLOCK + 64 * wave + ls_;\n"
          << "    const int k = 0;\n";
        for (int sl : arg_slots) {
            const std::string ct = ctype(X.col_type(X.num_cols[sl]));
            o << "    " << ct << " c" << sl << "[1];\n    c" << sl << "[0] = sel ? ((const " << ct << "*)A.col[" << sl
              << "])[row] : (" << ct << ")0;\n";
        }
        emit_accumulate();
        o << "  }\n  } else {\n";
        // dense: each sub-tile's arguments reloaded where selected
        o << "  for (int m_ = 0; m_ < M; ++m_) {\n  const i64 base = ((i64)t * M + m_) * (BLOCK * K);\n"
          << "  unsigned selm = 0;\n#pragma unroll\n  for (int k = 0; k < K; ++k)\n"
          << "    selm |= (unsigned)((dfmi::lds_uniform_u64(&WSA[(m_ * K + k) * WAVES + wave]) >> lane) & 1) << k;\n"
          << "  if (!__ballot(selm != 0)) continue;\n";
        emit_decls(o, arg_slots, X, "", false);
        emit_loads(o, arg_slots, X, "", "base", "(selm >> k) & 1", false);
        o << "#pragma unroll\n  for (int k = 0; k < K; ++k) {\n"
          << "    const i64 row = base + k * BLOCK + tid;\n    const bool sel = (selm >> k) & 1;\n";
        emit_accumulate();
        o << "  }\n  }\n  }\n";
    } else {
        emit_decls(o, X.pred_slots, X, "", true);
        emit_decls(o, X.proj_slots, X, "", !P.pred);
        emit_loads(o, X.pred_slots, X, "", "(i64)t * (BLOCK * K)", nullptr, true);
        o << "  unsigned nsel_ = 0;\n  {\n  const i64 base = (i64)t * (BLOCK * K);\n";
        if (P.pred) {
            g.filtered_cols = false;
            // proj_dense: argument-only columns loaded for every row, in the
            // predicate's memory round trip
            if (X.proj_dense) emit_loads(o, X.proj_slots, X, "", "base", nullptr, false);
            emit_predicate(g, o, P, X, "", {});
            // argument-only columns, loaded only where selected
            if (!X.proj_dense) emit_loads(o, X.proj_slots, X, "", "base", "(selm >> k) & 1", false);
            emit_count();
        } else {
            o << "  unsigned selm = 0;\n#pragma unroll\n  for (int k = 0; k < K; ++k) selm |= (unsigned)(base + k * BLOCK "
                 "+ tid < A.n_rows) << k;\n";
            emit_loads(o, X.proj_slots, X, "", "base", nullptr, true);
        }
        // arguments over the filtered batch (no validity) or the batch itself
        g.filtered_cols = P.pred != nullptr;
        emit_acc_decls();
        o << "  dfmi::lds_sync();\n";
        o << "#pragma unroll\n  for (int k = 0; k < K; ++k) {\n"
          << "    const i64 row = base + k * BLOCK + tid;\n    const bool sel = (selm >> k) & 1;\n";
        emit_accumulate();
        o << "  }\n";
    }
    for (int j = 0; j < NA; ++j)
        o << "  dfmi::agg_wave_flush<NA, NF>(S, " << j << ", acnt" << j << ", asum" << j << ", akey" << j << ", "
          << (P.aggs[j].fn == DFMI_AGG_MIN ? "true" : "false") << ", afl" << j << ", lane);\n";
    // the selected-row count, sampled: every 64th block adds its count (one
    // global atomic per 64 blocks -- a counter every wave hit would serialise)
    if (P.pred) o << "  if (lane == 0 && nsel_) atomicAdd(&NSEL_, nsel_);\n";
    o << "  dfmi::lds_sync();\n  dfmi::agg_block_flush<NA, NF>(A, S, fslot, is_min, tid);\n";
    if (P.pred) o << "  if (tid == 0 && NSEL_ && (blockIdx.x & 63u) == 0) atomicAdd(A.totals, (u64)NSEL_);\n";
    if (!(X.M > 1 && P.pred)) o << "  }\n";
}

// GROUP BY form of the aggregate kernel (one Boolean / integer key): every
// selected row's slot in the batch's key window (Args::gbase / gwidth, null
// key: slot gwidth) is computed once; then, per slot present in the wave
// (uniform loop), the arguments are reduced over that slot's rows exactly as
// in generate_agg and flushed into the slot's LDS state. A hidden last
// aggregate counts the slot's rows (so a group whose arguments are all null
// still exists). Accumulators: [copies][GS][NA + 1][kAggWords].
static void generate_agg_grouped(Gen& g, std::ostringstream& o, const Plan& P, Launch& X) {
    const int NA = (int)P.aggs.size() + 1;  // + the group's row count
    int NF = 0;
    for (const AggSpec& a : P.aggs) NF += a.fslot >= 0;
    o << "  constexpr int NA = " << NA << ", NF = " << NF << ", GS = " << P.gslots << ";\n";
    o << "  __shared__ dfmi::AggLds<NA, NF> S[GS];\n  const unsigned char is_min[NA] = {";
    for (int j = 0; j + 1 < NA; ++j) o << (P.aggs[j].fn == DFMI_AGG_MIN ? 1 : 0) << ", ";
    o << "0};\n  const int fslot[NF > 0 ? NF : 1] = {";
    {
        bool any = false;
        for (int j = 0; j + 1 < NA; ++j)
            if (P.aggs[j].fslot >= 0) {
                o << (any ? ", " : "") << j;
                any = true;
            }
        if (!any) o << "0";
    }
    o << "};\n";
    o << "  const int nslot = A.gwidth + 1;  // <= GS (host-checked)\n";
    o << "  for (int g_ = wave; g_ < nslot; g_ += WAVES) dfmi::agg_lds_init<NA, NF>(S[g_], is_min, lane);\n";
    o << "  const unsigned t = tile_;\n";
    emit_decls(o, X.pred_slots, X, "", true);
    emit_decls(o, X.proj_slots, X, "", !P.pred);
    emit_loads(o, X.pred_slots, X, "", "(i64)t * (BLOCK * K)", nullptr, true);
    o << "  {\n  const i64 base = (i64)t * (BLOCK * K);\n";
    if (P.pred) {
        g.filtered_cols = false;
        if (X.proj_dense) emit_loads(o, X.proj_slots, X, "", "base", nullptr, false);
        emit_predicate(g, o, P, X, "", {});
        if (!X.proj_dense) emit_loads(o, X.proj_slots, X, "", "base", "(selm >> k) & 1", false);
    } else {
        o << "  unsigned selm = 0;\n#pragma unroll\n  for (int k = 0; k < K; ++k) selm |= (unsigned)(base + k * BLOCK "
             "+ tid < A.n_rows) << k;\n";
        emit_loads(o, X.proj_slots, X, "", "base", nullptr, true);
    }
    g.filtered_cols = P.pred != nullptr;
    // the key of every selected row (evaluated before the aggregates: its
    // errors come first in evaluation order) -> its slot
    o << "  unsigned gsl[K];\n#pragma unroll\n  for (int k = 0; k < K; ++k) {\n"
      << "    const i64 row = base + k * BLOCK + tid;\n    const bool sel = (selm >> k) & 1;\n";
    {
        const Val kv = g.emit(P.gkey, P.gkey->root, P.gkey_ord, "sel");
        if (P.gkey->type == DFMI_TYPE_BOOLEAN) {
            o << "    gsl[k] = !(" << kv.n << ") ? (unsigned)A.gwidth : ((" << kv.v << ") ? 1u : 0u);\n";
        } else {
            o << "    { const u64 d_ = (u64)(" << (is_signed_int(P.gkey->type) ? "i64" : "u64") << ")(" << kv.v
              << ") - A.gbase;\n"
              << "      gsl[k] = !(" << kv.n << ") ? (unsigned)A.gwidth : (d_ < (u64)A.gwidth ? (unsigned)d_ : ~0u);\n"
              << "      if (sel && gsl[k] == ~0u) dfmi::report_err(A.err, 0, 0, dfmi::ERRK_CAPACITY); }\n";
        }
    }
    o << "  }\n  dfmi::lds_sync();\n";
    o << "  for (int g_ = 0; g_ < nslot; ++g_) {\n"
      << "    bool any_ = false;\n#pragma unroll\n    for (int k = 0; k < K; ++k) any_ |= ((selm >> k) & 1) && gsl[k] == (unsigned)g_;\n"
      << "    if (!__ballot(any_)) continue;\n";
    for (int j = 0; j < NA; ++j)
        o << "  unsigned acnt" << j << " = 0, afl" << j << " = 0;\n  u64 asum" << j << " = 0, akey" << j << " = "
          << (j + 1 < NA && P.aggs[j].fn == DFMI_AGG_MIN ? "~0ull" : "0ull") << ";\n";
    o << "#pragma unroll\n  for (int k = 0; k < K; ++k) {\n"
      << "    const i64 row = base + k * BLOCK + tid;\n    const bool sel = ((selm >> k) & 1) && gsl[k] == (unsigned)g_;\n"
      << "    acnt" << NA - 1 << " += sel ? 1u : 0u;\n";
    for (int j = 0; j + 1 < NA; ++j) {
        const AggSpec& a = P.aggs[j];
        const Val v = g.emit(a.prog, a.prog->root, a.ord_base, "sel");
        const std::string ok = "ok" + std::to_string(j) + "_";
        o << "    { const bool " << ok << " = sel && (" << v.n << ");\n";
        o << "      acnt" << j << " += " << ok << " ? 1u : 0u;\n";
        if (a.fn == DFMI_AGG_SUM && a.fslot < 0) {
            o << "      asum" << j << " += " << ok << " ? (u64)(" << (is_signed_int(a.arg_type) ? "i64" : "u64") << ")("
              << v.v << ") : 0ull;\n";
        } else if (a.fn == DFMI_AGG_SUM) {
            o << "      afl" << j << " |= " << ok << " ? dfmi::agg_sum_flags(" << v.v << ") : 0u;\n"
              << "      const bool fin_ = " << ok << " && (dfmi::agg_sum_flags(" << v.v << ") == dfmi::AGGF_NONNEGZERO) && ("
              << v.v << ") != 0;\n"
              << "      dfmi::fsum_add(S[g_].limbs[" << a.fslot << "], &S[g_].dlo[" << a.fslot << "], &S[g_].dhi["
              << a.fslot << "], (double)(" << v.v << "), fin_, lane);\n";
        } else if (a.fn == DFMI_AGG_MIN || a.fn == DFMI_AGG_MAX) {
            const char* cmp = a.fn == DFMI_AGG_MIN ? "<" : ">";
            o << "      const bool nan_ = dfmi::agg_isnan(" << v.v << ");\n"
              << "      afl" << j << " |= " << ok << " ? (nan_ ? (unsigned)dfmi::AGGF_NAN : (unsigned)dfmi::AGGF_VALUE) : 0u;\n"
              << "      if (" << ok << " && !nan_) { const u64 k_ = dfmi::agg_key(" << v.v << "); if (k_ " << cmp << " akey" << j
              << ") akey" << j << " = k_; }\n";
        }
        o << "    }\n";
    }
    o << "  }\n";
    for (int j = 0; j < NA; ++j)
        o << "  dfmi::agg_wave_flush<NA, NF>(S[g_], " << j << ", acnt" << j << ", asum" << j << ", akey" << j << ", "
          << (j + 1 < NA && P.aggs[j].fn == DFMI_AGG_MIN ? "true" : "false") << ", afl" << j << ", lane);\n";
    o << "  }\n  dfmi::lds_sync();\n"
      << "  for (int g_ = 0; g_ < nslot; ++g_)\n"
      << "    dfmi::agg_block_flush<NA, NF>(A, S[g_], fslot, is_min, tid, A.agg + ((u64)(blockIdx.x % dfmi::kAggCopies) * GS + "
         "g_) * NA * dfmi::kAggWords);\n  }\n";
}

// Coalesced batches: this block's batch, its local tile index `tile_`, and a
// local copy of the Args with the batch's rows, tiles, look-back status
// segment, totals / error words and buffers (the copy is only ever indexed
// with constants, so it lives in registers: no scratch).
static void emit_batched_prologue(std::ostream& o, const Plan& P, const Launch& X) {
    const int np = batch_words(X, (int)P.outs.size());
    o << "  const int b_ = A0.tile_batch[bid_];\n"
      << "  void* const* bp_ = A0.batch_ptrs + (i64)b_ * " << np << ";\n"
      << "  dfmi::Args A = A0;\n"
      << "  A.n_rows = (i64)(u64)bp_[0];\n"
      << "  const u64 tt_ = (u64)bp_[1];\n"
      << "  A.n_tiles = (int)(unsigned)tt_;\n"
      << "  const unsigned tile_ = bid_ - (unsigned)(tt_ >> 32);\n"
      << "  A.totals = (u64*)bp_[2];\n  A.err = (u64*)bp_[3];\n"
      // diagnostics (mode bit 4): the forced look-back timeout in the first
      // batch's own error word, which the coalesced launch's host reads
      << "  if ((A.mode & 16) && blockIdx.x == 0 && tid == 0) atomicMax(A.err, ~(u64)3);\n";
    if (P.pred)  // [ch][tile] status words of this batch's tiles
        o << "  A.status = A0.status + (i64)(tt_ >> 32) * " << (1 + X.utf8_outs.size()) * (size_t)X.spread << ";\n";
    for (size_t s = 0; s < X.num_cols.size(); ++s)
        o << "  A.col[" << s << "] = bp_[" << batch_slot_col((int)s) << "];\n  A.valid[" << s << "] = (const u8*)bp_["
          << batch_slot_col((int)s) + 1 << "];\n";
    for (size_t u = 0; u < X.utf8_cols.size(); ++u) {
        const int b = batch_slot_utf8(X, (int)u);
        o << "  A.offs[" << u << "] = (const int*)bp_[" << b << "];\n  A.bytes[" << u << "] = (const u8*)bp_[" << b + 1
          << "];\n  A.svalid[" << u << "] = (const u8*)bp_[" << b + 2 << "];\n";
    }
    for (size_t oi = 0; oi < P.outs.size(); ++oi) {
        const int b = batch_slot_out(X, (int)oi);
        o << "  A.out[" << oi << "] = bp_[" << b << "];\n  A.out_valid[" << oi << "] = (u8*)bp_[" << b + 1
          << "];\n  A.out_offs[" << oi << "] = (int*)bp_[" << b + 2 << "];\n  A.out_data[" << oi << "] = (u8*)bp_["
          << b + 3 << "];\n  A.out_cap[" << oi << "] = (i64)(u64)bp_[" << b + 4 << "];\n";
    }
}

std::string generate(const Plan& P, Launch& X) {
    X.n_lits = X.n_str = X.str_bytes = 0;  // (slots are assigned anew by every generation)
    Gen g(P, X);
    std::ostringstream& o = g.o;
    const int K = X.K, BLOCK = X.BLOCK;
    o << "\n// ---- generated query kernel ----\n";
    o << "extern \"C\" __global__ __launch_bounds__(" << BLOCK << ")";
    if (X.waves_per_eu > 0) o << " __attribute__((amdgpu_waves_per_eu(" << X.waves_per_eu << ")))";
    o << " void DFMI_KNAME(const dfmi::Args A0) {\n";
    o << "  constexpr int BLOCK = " << BLOCK << ", K = " << K << ", WAVES = BLOCK / 64;\n";
    o << "  const int tid = threadIdx.x, lane = tid & 63, wave = dfmi::uni(tid >> 6);\n";
    o << "  dfmi::clear_previous<BLOCK>(A0, blockIdx.x, tid);\n";
    if (X.ticket && P.pred && P.aggs.empty())
        o << "  __shared__ unsigned tk_;\n  if (tid == 0) tk_ = atomicAdd(A0.ticket, 1u);\n  __syncthreads();\n"
          << "  const unsigned bid_ = tk_;\n";
    else
        o << "  const unsigned bid_ = blockIdx.x;\n";
    if (X.batched) {
        if (!P.aggs.empty()) throw Fail{DFMI_ERR_NOT_IMPLEMENTED, "batched launch of an aggregate"};
        emit_batched_prologue(o, P, X);
    } else {
        o << "  const dfmi::Args& A = A0;\n  const unsigned tile_ = bid_;\n";
    }
    if (!P.aggs.empty() && P.gkey) {
        generate_agg_grouped(g, o, P, X);
    } else if (!P.aggs.empty()) {
        generate_agg(g, o, P, X);
    } else if (P.pred) {
        const int nch = 1 + (int)X.utf8_outs.size();
        o << "  constexpr int NCH = " << nch << ";\n";
        const std::string tparams = std::to_string(X.R) + ", " + std::to_string(X.sleep) + ", " +
                                    std::to_string(X.spread) + ", " + std::to_string(X.window);
        std::vector<int> utf8_out_cols;
        for (const auto& uo : X.utf8_outs) utf8_out_cols.push_back(uo.second);
        const std::vector<int> out_slots = output_slots(P, X);
        auto offs_name = [&](int u) { return std::to_string(u); };
        // The predicate over the rows at `base`: selm, the projection-only
        // loads (unless late), the selection ballots wm and counts cnt.
        auto emit_select = [&]() {
            g.filtered_cols = false;
            const bool dense = X.proj_dense && !X.late_proj && X.M == 1;
            if (dense) emit_loads(o, X.proj_slots, X, "", "base", nullptr, false);
            emit_predicate(g, o, P, X, "", utf8_out_cols);
            // projection-only columns, loaded only where selected
            if (!dense && !X.late_proj && X.M == 1) emit_loads(o, X.proj_slots, X, "", "base", "(selm >> k) & 1", false);
            // compaction offsets (rows + Utf8 bytes)
            o << "  unsigned cnt[NCH][K];\n  u64 wm[K];\n#pragma unroll\n  for (int k = 0; k < K; ++k) {\n"
              << "    wm[k] = __ballot((selm >> k) & 1);\n    cnt[0][k] = (selm >> k) & 1;\n  }\n";
            for (size_t j = 0; j < X.utf8_outs.size(); ++j) {
                const int u = X.utf8_outs[j].second;
                o << "#pragma unroll\n  for (int k = 0; k < K; ++k) { const int e_ = dfmi::utf8_end(us" << offs_name(u)
                  << "[k], ux" << offs_name(u) << "[k], lane); cnt[" << (j + 1) << "][k] = ((selm >> k) & 1) ? "
                  << "(unsigned)(e_ - us" << offs_name(u) << "[k]) : 0u; }\n";
            }
        };
        // Compacted stores of the selected rows at `base` (selm, wm, the
        // Utf8 offsets and the column registers in scope; the tile's offsets
        // resolved in T); `kb`: the rows' first word of the tile.
        // The numeric / Boolean outputs of one selected row (`k`, `row` and its
        // output index `d` in scope; the column registers c<slot>[k]).
        auto emit_out_values = [&]() {
            for (size_t oi = 0; oi < P.outs.size(); ++oi) {
                const OutSpec& os = P.outs[oi];
                if (os.kind == OutSpec::SKIP || os.kind == OutSpec::UTF8) continue;
                Val v;
                if (os.kind == OutSpec::GATHER) {
                    IrNode c;
                    c.kind = IR_COL;
                    c.col = os.col;
                    c.type = X.col_type(os.col);
                    v = g.col(c);
                } else {
                    v = g.emit(os.prog, os.prog->root, os.ord_base, "true");
                }
                const std::string ct = ctype(os.out_type);
                if (os.nullable)  // compacted validity as bytes (packed after the kernel)
                    o << "    { const bool v_ = " << v.n << "; ((u8*)A.out_valid[" << oi << "] + obase)[d] = v_ ? 1 : 0;"
                      << " nn" << oi << " += v_ ? 0u : 1u; }\n";
                if (os.out_type == DFMI_TYPE_BOOLEAN)
                    o << "    ((u8*)A.out[" << oi << "] + obase)[d] = (" << v.v << ") ? 1 : 0;\n";
                else if (X.nt & 2)
                    o << "    __builtin_nontemporal_store((" << ct << ")(" << v.v << "), (" << ct << "*)A.out[" << oi
                      << "] + obase + d);\n";
                else
                    o << "    ((" << ct << "*)A.out[" << oi << "] + obase)[d] = " << v.v << ";\n";
            }
        };
        auto emit_outputs = [&](const std::string& kb, bool prestaged) {
            // byte-light predicates: projection-only columns after the look-back
            // (fewer registers held across it; few rows are selected)
            if (X.M > 1) emit_loads(o, out_slots, X, "", "base", "(selm >> k) & 1", false);
            else if (X.late_proj) emit_loads(o, X.proj_slots, X, "", "base", "(selm >> k) & 1", false);
            o << "  const i64 obase = (i64)T.prefix[0];\n  unsigned dst[K];\n#pragma unroll\n"
              << "  for (int k = 0; k < K; ++k) dst[k] = (unsigned)T.excl[0][(" << kb
              << " + k) * WAVES + wave] + dfmi::lane_rank(wm[k]);\n";
            // projections over the selected rows (filtered batch: no validity)
            g.filtered_cols = true;
            for (size_t oi = 0; oi < P.outs.size(); ++oi)
                if (P.outs[oi].nullable) o << "  unsigned nn" << oi << " = 0;\n";
            o << "#pragma unroll\n  for (int k = 0; k < K; ++k) {\n    if (!((selm >> k) & 1)) continue;\n"
              << "    const i64 row = base + k * BLOCK + tid;\n    const unsigned d = dst[k];\n";
            emit_out_values();
            o << "  }\n";
            for (size_t oi = 0; oi < P.outs.size(); ++oi)
                if (P.outs[oi].nullable)
                    o << "  { const u64 s_ = dfmi::wave_sum((u64)nn" << oi << "); if (lane == 0 && s_) atomicAdd(&A.totals[8 + "
                      << oi << "], s_); }\n";
            if (!X.utf8_outs.empty()) o << "  if (!(A.mode & 8)) {  // mode bit 3: skip the byte copies (diagnostics)\n";
            for (size_t j = 0; j < X.utf8_outs.size(); ++j) {
                const int u = X.utf8_outs[j].second;
                const std::string tail = ", us" + offs_name(u) + ", ux" + offs_name(u) + ", ";
                if (X.gather == 3)
                    o << "  dfmi::utf8_offsets_src<BLOCK, K, NCH>(A, T, " << (j + 1) << ", " << X.utf8_outs[j].first
                      << ", selm, wm, dst" << tail << "lane, wave, " << kb << ");\n";
                else if (X.ring && j == 0)
                    o << "  dfmi::utf8_gather_ring<BLOCK, K, NCH, " << X.ring << ">(A, T, 1, " << u << ", "
                      << X.utf8_outs[j].first << ", selm, dst" << tail << "RG, lane, wave, tid);\n";
                else if (X.gather == 0)
                    o << "  dfmi::utf8_gather_lane<BLOCK, K, NCH>(A, T, " << (j + 1) << ", " << u << ", "
                      << X.utf8_outs[j].first << ", selm, dst" << tail << "lane, wave, " << kb << ");\n";
                else if (X.gather == 6)
                    o << "  dfmi::utf8_gather_direct<BLOCK, K, NCH, " << X.direct_grp << ">(A, T, " << (j + 1) << ", "
                      << u << ", " << X.utf8_outs[j].first << ", selm, dst" << tail << "lane, wave, " << kb << ");\n";
                else
                    o << "  dfmi::utf8_gather" << (X.gather == 2 ? "_serial" : "") << "<BLOCK, K, NCH, ARENA>(A, T, "
                      << (j + 1) << ", " << u << ", " << X.utf8_outs[j].first << ", selm, wm, dst" << tail
                      << "G[wave], lane, wave, " << kb
                      << (X.gather == 2 ? "" : X.gather == 4 ? (X.pairs ? ", 3" : X.st16 ? ", 4" : ", 1") : X.gather == 5 ? ", 2" : ", 0")
                      << (X.gather == 2 ? "" : (prestaged && j == 0 ? ", pre_" : ", -1"))
                      << (X.gather == 2 ? "" : X.gather_phases ? ", true" : ", false")
                      << (X.gather == 2 ? "" : X.dbuf ? ", true" : ", false")
                      << (X.gather == 2 || !X.early ? "" : ", true") << ");\n";
            }
            if (!X.utf8_outs.empty()) o << "  }\n";
        };
        // The last tile writes every Utf8 output's final offset.
        auto emit_last_offsets = [&]() {
            if (X.utf8_outs.empty()) return;
            o << "  if (tid == 0 && t == (unsigned)A.n_tiles - 1) {\n";
            for (size_t j = 0; j < X.utf8_outs.size(); ++j)
                o << "    A.out_offs[" << X.utf8_outs[j].first << "][T.prefix[0] + T.agg[0]] = (int)(T.prefix[" << (j + 1)
                  << "] + T.agg[" << (j + 1) << "]);\n";
            o << "  }\n";
        };
        // one tile per block in dispatch order (in order per XCD, so every
        // tile a block waits on in the look-back is running or done)
        if (X.ring)
            o << "  __shared__ dfmi::Utf8Ring<" << X.ring << "> RG;\n";
        if (X.eq_dense > 0) o << "  __shared__ uint4 EQA[WAVES][" << X.eq_dense << "];\n";
        if (!X.utf8_outs.empty() && X.gather && X.gather != 3 && X.gather != 6 && !(X.ring && X.utf8_outs.size() == 1))
            o << "  constexpr int ARENA = " << X.arena << ";\n  __shared__ dfmi::Utf8Stage<ARENA, "
              << (X.gather == 1 ? 32 : X.gather == 5 ? 72 : X.gather == 2 ? 129 : X.image) << "> G[WAVES];\n";
        o << "  const unsigned t = tile_;\n";
        if (X.M == 1) {
            // One tile: predicate, projection-only loads, scan + look-back,
            // compacted stores.
            o << "  __shared__ dfmi::Tile<BLOCK, K, NCH> T;\n";
            emit_decls(o, X.pred_slots, X, "", true);
            emit_decls(o, X.proj_slots, X, "", false);
            emit_loads(o, X.pred_slots, X, "", "(i64)t * (BLOCK * K)", nullptr, true);
            o << "  {\n  const i64 base = (i64)t * (BLOCK * K);\n";
            emit_select();
            if (X.ring)  // the loader wave issues the first steps' source bytes now
                o << "  dfmi::ring_prologue<BLOCK, K, " << X.ring << ">(A, RG, " << X.utf8_outs[0].second
                  << ", base, us" << offs_name(X.utf8_outs[0].second) << ", lane, wave);\n";
            // the first Utf8 output's first staging round goes out before the
            // look-back, whose wait then hides it
            const bool pre = !X.utf8_outs.empty() && (X.gather == 1 || X.gather >= 4) && X.prestage;
            // (prestage 2: every wave but wave 0, whose look-back polls would
            // otherwise wait behind its staging loads -- vmcnt counts in order)
            if (pre)
                o << "  const int pre_ = " << (X.prestage == 2 ? "wave == 0 ? -1 : " : "")
                  << "dfmi::utf8_gather_prestage<K, " << (X.dbuf ? "ARENA / 2" : "ARENA") << ">(A, "
                  << X.utf8_outs[0].second
                  << ", wm, us" << offs_name(X.utf8_outs[0].second) << ", ux" << offs_name(X.utf8_outs[0].second)
                  << ", G[wave], lane);\n";
            o << "  dfmi::tile_offsets<BLOCK, K, NCH, " << tparams << ">(A, T, t, cnt, lane, wave);\n";
            emit_outputs("0", pre);
            emit_last_offsets();
            o << "  }\n";
        } else {
            // M sub-tiles: the predicate pass keeps only each sub-tile's
            // ballots and counts (LDS), one scan + look-back covers all of
            // them, and the output pass revisits the sub-tiles with selected
            // rows, reloading the Utf8 offsets and column values they need.
            // (a numeric predicate loads its columns per sub-tile; its output
            // pass reloads the columns the outputs read for the selected rows
            // only -- chosen for low selectivity, exec.cpp)
            o << "  constexpr int M = " << X.M << ";\n"
              << "  __shared__ dfmi::Tile<BLOCK, K * M, NCH> T;\n  __shared__ u64 WS[K * M * WAVES];\n";
            // software pipeline: sub-tile m+1's Utf8 offsets are loaded while
            // sub-tile m's dependent loads (equality heads) are in flight
            const size_t nu = X.utf8_cols.size();
            for (size_t u = 0; u < nu && X.prefetch; ++u)
                o << "  int usN" << u << "[K], uxN" << u << "[K];\n  dfmi::utf8_offs_tile<BLOCK, K>(A, " << u
                  << ", (i64)t * M * (BLOCK * K), lane, wave, ~0u, usN" << u << ", uxN" << u << ");\n";

            o << "  for (int m_ = 0; m_ < M; ++m_) {\n  const i64 base = ((i64)t * M + m_) * (BLOCK * K);\n"
              << "  if (base >= A.n_rows) { if (tid < K * WAVES) { WS[m_ * K * WAVES + tid] = 0; }\n"
              << "    for (int c_ = tid; c_ < NCH * K * WAVES; c_ += BLOCK) T.cnt[c_ / (K * WAVES)][m_ * K * WAVES + c_ % (K * WAVES)] = 0;\n"
              << "    continue; }\n";
            for (size_t u = 0; u < nu; ++u)
                if (X.prefetch)
                    o << "  int us" << u << "[K], ux" << u << "[K];\n#pragma unroll\n  for (int k = 0; k < K; ++k) { us" << u
                      << "[k] = usN" << u << "[k]; ux" << u << "[k] = uxN" << u << "[k]; }\n"
                      << "  if (m_ + 1 < M) dfmi::utf8_offs_tile<BLOCK, K>(A, " << u
                      << ", base + BLOCK * K, lane, wave, ~0u, usN" << u << ", uxN" << u << ");\n";
                else  // (diagnostics: each sub-tile loads its own offsets when it starts)
                    o << "  int us" << u << "[K], ux" << u << "[K];\n  dfmi::utf8_offs_tile<BLOCK, K>(A, " << u
                      << ", base, lane, wave, ~0u, us" << u << ", ux" << u << ");\n";
            g.filtered_cols = false;
            if (!X.pred_slots.empty()) {
                o << "  {\n";
                emit_decls(o, X.pred_slots, X, "", true);
                emit_loads(o, X.pred_slots, X, "", "base", nullptr, true);
            }
            emit_predicate(g, o, P, X, "", utf8_out_cols, true);
            o << "  unsigned cnt[NCH][K];\n  u64 wm[K];\n#pragma unroll\n  for (int k = 0; k < K; ++k) {\n"
              << "    wm[k] = __ballot((selm >> k) & 1);\n    cnt[0][k] = (selm >> k) & 1;\n  }\n";
            for (size_t j = 0; j < X.utf8_outs.size(); ++j) {
                const int u = X.utf8_outs[j].second;
                o << "#pragma unroll\n  for (int k = 0; k < K; ++k) { const int e_ = dfmi::utf8_end(us" << offs_name(u)
                  << "[k], ux" << offs_name(u) << "[k], lane); cnt[" << (j + 1) << "][k] = ((selm >> k) & 1) ? "
                  << "(unsigned)(e_ - us" << offs_name(u) << "[k]) : 0u; }\n";
            }
            o << "  dfmi::subtile_counts<BLOCK, K, NCH>(T, WS, m_ * K, cnt, wm, lane, wave);\n";
            if (!X.pred_slots.empty()) o << "  }\n";
            o << "  }\n";
            const std::string sp = std::to_string(X.spread);
            o << "  dfmi::tile_scan_lds<BLOCK, K * M, NCH, " << sp << ">(A, T, t, lane, wave);\n"
              << "  dfmi::tile_resolve<BLOCK, K * M, NCH, " << tparams << ">(A, T, t, lane, wave);\n"
              << "  dfmi::lds_sync();\n";
            // sparse output pass: when the wave's sub-tiles hold at most 64
            // selected rows (an equality on a Utf8 column), one lane per
            // selected row loads what it needs and stores its outputs -- one
            // round of loads for the whole wave instead of one per slice
            // (not with the two-pass gather: its second kernel reads the source
            // starts only the dense pass's utf8_offsets_src writes)
            bool sparse = X.sparse && X.gather != 3;
            for (int sl : out_slots) sparse = sparse && X.col_type(X.num_cols[sl]) != DFMI_TYPE_BOOLEAN;
            if (sparse) {
                // Utf8 outputs: one round of 64 rows (their byte offsets come
                // from one wave scan); numeric outputs: up to 4 rounds
                const int cap = X.utf8_outs.empty() ? 256 : 64;
                o << "  constexpr unsigned CAP_ = " << cap << ";\n"
                  << "  __shared__ unsigned short SLR[WAVES][CAP_];\n  unsigned tot_ = 0;\n"
                  << "  for (int q_ = 0; q_ < M * K; ++q_) {\n"
                  << "    const u64 w_ = dfmi::lds_uniform_u64(&WS[q_ * WAVES + wave]);\n    if (!w_) continue;\n"
                  << "    if (tot_ + (unsigned)__builtin_popcountll(w_) <= CAP_ && ((w_ >> lane) & 1))\n"
                  << "      SLR[wave][tot_ + dfmi::lane_rank(w_)] = (unsigned short)(q_ * 64 + lane);\n"
                  << "    tot_ += (unsigned)__builtin_popcountll(w_);\n  }\n"
                  << "  if (tot_ <= CAP_) {\n  dfmi::wave_lds_fence();\n";
                if (cap > 64) o << "  for (unsigned r_ = 0; r_ < tot_; r_ += 64) {\n";
                else o << "  { const unsigned r_ = 0;\n";
                o << "  const bool have_ = r_ + (unsigned)lane < tot_;\n"
                  << "  const unsigned e_ = have_ ? (unsigned)SLR[wave][r_ + lane] : 0u;\n"
                  << "  const int qs_ = (int)(e_ >> 6), ls_ = (int)(e_ & 63u);\n"
                  << "  const i64 row = ((i64)t * M + qs_ / K) * (BLOCK * K) + (i64)(qs_ % K) * BLOCK + 64 * wave + ls_;\n"
                  << "  const u64 wq_ = have_ ? WS[qs_ * WAVES + wave] : 0ull;\n"
                  << "  const unsigned d = have_ ? (unsigned)T.excl[0][qs_ * WAVES + wave] + "
                     "(unsigned)__builtin_popcountll(wq_ & ((1ull << ls_) - 1ull)) : 0u;\n"
                  << "  const i64 obase = (i64)T.prefix[0];\n  const int k = 0;\n";
                for (int sl : out_slots) {
                    const std::string ct = ctype(X.col_type(X.num_cols[sl]));
                    o << "  " << ct << " c" << sl << "[1];\n  c" << sl << "[0] = have_ ? ((const " << ct << "*)A.col[" << sl
                      << "])[row] : (" << ct << ")0;\n";
                }
                for (size_t j = 0; j < X.utf8_outs.size(); ++j)
                    o << "  const int su" << j << "_ = have_ ? A.offs[" << X.utf8_outs[j].second << "][row] : 0, eu" << j
                      << "_ = have_ ? A.offs[" << X.utf8_outs[j].second << "][row + 1] : 0;\n";
                g.filtered_cols = true;
                for (size_t oi = 0; oi < P.outs.size(); ++oi)
                    if (P.outs[oi].nullable) o << "  unsigned nn" << oi << " = 0;\n";
                o << "  if (have_) {\n";
                emit_out_values();
                o << "  }\n";
                for (size_t oi = 0; oi < P.outs.size(); ++oi)
                    if (P.outs[oi].nullable)
                        o << "  { const u64 s_ = dfmi::wave_sum((u64)nn" << oi
                          << "); if (lane == 0 && s_) atomicAdd(&A.totals[8 + " << oi << "], s_); }\n";
                if (!X.utf8_outs.empty()) {
                    // each selected row's bytes: its slice's byte offset plus the
                    // lengths of the selected rows before it in the slice
                    o << "  const int qp_ = __builtin_amdgcn_ds_bpermute(((lane + 63) & 63) << 2, qs_);\n"
                      << "  const u64 first_ = __ballot(have_ && (lane == 0 || qp_ != qs_));\n"
                      << "  const int fl_ = 63 - __builtin_clzll(first_ & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull)));\n";
                    for (size_t j = 0; j < X.utf8_outs.size(); ++j) {
                        const int oo = X.utf8_outs[j].first, u = X.utf8_outs[j].second;
                        o << "  { const unsigned L_ = have_ ? (unsigned)(eu" << j << "_ - su" << j << "_) : 0u;\n"
                          << "    const unsigned x_ = dfmi::wave_incl_scan32(L_, lane) - L_;\n"
                          << "    const unsigned xf_ = (unsigned)__builtin_amdgcn_ds_bpermute(fl_ << 2, (int)x_);\n"
                          << "    const u64 ob_ = T.prefix[" << (j + 1) << "] + (have_ ? T.excl[" << (j + 1)
                          << "][qs_ * WAVES + wave] : 0ull) + (x_ - xf_);\n"
                          << "    if (have_) {\n      A.out_offs[" << oo << "][obase + d] = (int)ob_;\n"
                          << "      if ((i64)(ob_ + L_) > A.out_cap[" << oo
                          << "]) dfmi::report_err(A.err, 0, 0, dfmi::ERRK_CAPACITY);\n"
                          << "      else if (L_ && !(A.mode & 8)) dfmi::utf8_copy(A.bytes[" << u << "] + su" << j << "_, A.out_data["
                          << oo << "] + ob_, L_);\n    }\n  }\n";
                    }
                }
                o << "  }\n  } else {\n";  // (the rounds; then the dense output pass)
            }
            // output pass in steps of KO slices (fewer registers than K)
            o << "  {\n  constexpr int KS = K, K = " << X.KO << ";  // slices per sub-tile / per output step\n"
              << "  for (int q_ = 0; q_ < M * KS; q_ += K) {\n"
              << "  const i64 base = ((i64)t * M + q_ / KS) * (BLOCK * KS) + (i64)(q_ % KS) * BLOCK;\n"
              << "  u64 wm[K];\n  unsigned selm = 0, need_ = 0;\n#pragma unroll\n  for (int k = 0; k < K; ++k) {\n"
              << "    wm[k] = dfmi::lds_uniform_u64(&WS[(q_ + k) * WAVES + wave]);\n"
              << "    selm |= (unsigned)((wm[k] >> lane) & 1) << k;\n    need_ |= (unsigned)(wm[k] != 0) << k;\n  }\n"
              << "  if (!need_) continue;\n";
            for (int u : utf8_out_cols)
                o << "  int us" << offs_name(u) << "[K], ux" << offs_name(u) << "[K];\n  dfmi::utf8_offs_tile<BLOCK, K>(A, "
                  << u << ", base, lane, wave, need_, us" << offs_name(u) << ", ux" << offs_name(u) << ");\n";
            emit_decls(o, out_slots, X, "", false);
            emit_outputs("q_", false);
            o << "  }\n  }\n";
            if (sparse) o << "  }\n";
            emit_last_offsets();
        }
    } else {
        // projection only: dense rows, ballot-packed validity / Boolean bitmaps
        o << "  const i64 base = (i64)tile_ * (BLOCK * K);\n";
        std::vector<int> all = X.pred_slots;
        all.insert(all.end(), X.proj_slots.begin(), X.proj_slots.end());
        emit_decls(o, all, X, "", true);
        emit_loads(o, all, X, "", "base", nullptr, true);
        o << "  unsigned nulls[" << std::max<size_t>(1, P.outs.size()) << "] = {0};\n";
        o << "#pragma unroll\n  for (int k = 0; k < K; ++k) {\n"
          << "    const i64 row = base + k * BLOCK + tid;\n    const bool in = row < A.n_rows;\n"
          << "    const i64 w = (base >> 6) + k * WAVES + wave;\n";
        for (size_t oi = 0; oi < P.outs.size(); ++oi) {
            const OutSpec& os = P.outs[oi];
            if (os.kind != OutSpec::EXPR) continue;
            const Val v = g.emit(os.prog, os.prog->root, os.ord_base, "in");
            if (os.out_type == DFMI_TYPE_BOOLEAN) {
                o << "    { const u64 vb_ = __ballot(in && (" << v.v << ")); const u64 nb_ = __ballot(in && ("
                  << v.n << "));\n"
                  << "      nulls[" << oi << "] += __builtin_popcountll(__ballot(in && !(" << v.n << ")));\n"
                  << "      if (lane == 0 && w * 64 < A.n_rows) { ((u64*)A.out[" << oi << "])[w] = vb_;"
                  << " if (A.out_valid[" << oi << "]) ((u64*)A.out_valid[" << oi << "])[w] = nb_; } }\n";
            } else {
                o << "    if (in) ((" << ctype(os.out_type) << "*)A.out[" << oi << "])[row] = " << v.v << ";\n";
                o << "    { const u64 nb_ = __ballot(in && (" << v.n << "));\n"
                  << "      nulls[" << oi << "] += __builtin_popcountll(__ballot(in && !(" << v.n << ")));\n"
                  << "      if (lane == 0 && w * 64 < A.n_rows && A.out_valid[" << oi << "]) ((u64*)A.out_valid[" << oi
                  << "])[w] = nb_; }\n";
            }
        }
        o << "  }\n";
        for (size_t oi = 0; oi < P.outs.size(); ++oi)
            if (P.outs[oi].kind == OutSpec::EXPR)
                o << "  if (lane == 0 && nulls[" << oi << "]) atomicAdd(&A.totals[8 + " << oi << "], (u64)nulls[" << oi
                  << "]);\n";
    }
    if (X.batched && X.hdr_out)
        // one tile per batch: this block made its batch's whole header (row /
        // byte totals, null counts, error word) -- once every wave's atomics
        // are done, copy it out (the host's pinned result block: no copy
        // back after the kernel) and leave it zero for the next call
        o << "  __threadfence();\n  __syncthreads();\n"
          << "  if (tid < 32) {\n    u64* h_ = (u64*)bp_[2];\n"
          << "    const u64 v_ = __hip_atomic_load(h_ + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n"
          << "    A0.hdr_out[(i64)b_ * 32 + tid] = v_;\n    h_[tid] = 0;\n  }\n";
    o << "}\n";
    // kernel name: the plan kind and a hash of the whole generated source
    // (prefix, skeleton, body), so that rocprofv3 reports every query shape
    // as its own kernel and a skeleton change renames every kernel (a
    // committed profile never matches code it did not measure)
    std::string body = o.str();
    const std::string prefix = std::string(X.light_copy ? "#define DFMI_LIGHT_COPY 1\n" : "") +
                               (X.long_copy ? "#define DFMI_LONG_COPY " + std::to_string(X.long_copy) + "\n" : "");
    static const uint64_t skel_h = [] {  // FNV-1a over the skeleton, once
        uint64_t v = 1469598103934665603ull;
        for (unsigned char ch : skeleton_text()) v = (v ^ ch) * 1099511628211ull;
        return v;
    }();
    uint64_t h = skel_h;
    for (const std::string* part : {&prefix, (const std::string*)&body})
        for (unsigned char ch : *part) h = (h ^ ch) * 1099511628211ull;
    char nm[64];
    snprintf(nm, sizeof nm, "dfmi_%s_%08llx", !P.aggs.empty() ? "agg" : (P.pred ? "filter" : "project"),
             (unsigned long long)(h & 0xffffffffull));
    X.kname = nm;
    body.replace(body.find("DFMI_KNAME"), 10, X.kname);
    return prefix + skeleton_text() + body;
}

// ------------------------------------------------------- shape fast path
// A call whose programs, batch column types / nullability and tile shape
// match an earlier call launches the same kernel with the same literal
// tables: programs are immutable and carry a never-reused uid, so the key
// below identifies the generated source without generating it (~20 KB of
// text per call otherwise).
namespace {
struct ShapeHit {
    std::weak_ptr<Compiled> mod;  // an evicted module makes the entry stale
    std::string kname;
    uint64_t lits[32];
    int n_lits;
    int str_off[8], str_len[8];
    char str[256];
    int n_str, str_bytes;
};
std::unordered_map<std::string, ShapeHit> g_shapes;  // guarded by g_mu

template <typename T>
void put(std::string& k, T v) {
    k.append((const char*)&v, sizeof v);
}

std::string shape_key(int device, const Plan& P, const Launch& X) {
    std::string k;
    k.reserve(256);
    put(k, device);
    put(k, P.pred ? P.pred->uid : 0ull);
    put(k, P.gkey ? P.gkey->uid : 0ull);
    put(k, P.gkey_ord);
    put(k, P.gslots);
    for (const AggSpec& a : P.aggs) {
        put(k, a.fn);
        put(k, a.prog ? a.prog->uid : 0ull);
        put(k, a.ord_base);
        put(k, a.fslot);
    }
    for (const OutSpec& os : P.outs) {
        put(k, (int)os.kind);
        put(k, os.col);
        put(k, os.prog ? os.prog->uid : 0ull);
        put(k, os.ord_base);
        put(k, os.out_type);
        put(k, (char)os.nullable);
    }
    const int tile[] = {X.K,  X.BLOCK,  X.waves_per_eu, X.R,     X.sleep,          X.spread,
                        X.window, X.nt, X.gather,       X.late_proj, X.arena, (int)X.batched, X.M, X.KO, X.prestage, X.prefetch, X.gather_phases, X.image, X.dbuf, X.sparse, X.pairs, X.st16, X.proj_dense, X.hdr_out, X.ticket, X.early, X.ring, X.eq_dense, X.light_copy, X.direct_grp, X.long_copy};
    k.append((const char*)tile, sizeof tile);
    for (int c : X.num_cols) {
        put(k, c);
        put(k, (char)X.col_type(c));
        put(k, (char)X.col_nullable(c));
    }
    put(k, (int)X.pred_slots.size());
    for (int c : X.utf8_cols) {
        put(k, c);
        put(k, (char)X.col_nullable(c));
    }
    for (const auto& uo : X.utf8_outs) {
        put(k, uo.first);
        put(k, uo.second);
    }
    return k;
}
}  // namespace

hipFunction_t get_kernel(int device, const Plan& P, Launch& X, double* compile_ms) {
    if (compile_ms) *compile_ms = 0;
    const std::string key = shape_key(device, P, X);
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = g_shapes.find(key);
        std::shared_ptr<Compiled> c;
        if (it != g_shapes.end() && !(c = it->second.mod.lock())) g_shapes.erase(it), it = g_shapes.end();
        if (it != g_shapes.end()) {
            const ShapeHit& h = it->second;
            X.module = c;
            memcpy(X.args_lits, h.lits, sizeof h.lits);
            X.n_lits = h.n_lits;
            memcpy(X.str_off, h.str_off, sizeof h.str_off);
            memcpy(X.str_len, h.str_len, sizeof h.str_len);
            memcpy(X.str, h.str, sizeof h.str);
            X.n_str = h.n_str;
            X.str_bytes = h.str_bytes;
            X.kname = h.kname;
            return c->fn;
        }
    }
    std::string src = generate(P, X);
    if (getenv("DFMI_JIT_PRINT"))  // the generated body (after the skeleton)
        fprintf(stderr, "%s\n", src.c_str() + std::min(src.size(), src.find(skeleton_text()) + skeleton_text().size()));
    ShapeHit h;
    std::shared_ptr<Compiled> c = compile(device, src, X.kname, compile_ms);
    if (X.waves_soft && X.waves_per_eu > 0) {
        // a soft occupancy hint: if the register allocator had to spill more
        // than a little to meet it, the query shape is compiled again without
        // it (the C3 gather kernel spills 72 B/lane under hipRTC at 8
        // waves/SIMD and is still 6% faster than at 6 waves)
        constexpr int kSoftSpill = 128;
        int scratch = 0, regs = 0;
        const bool got = hipFuncGetAttribute(&scratch, HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES, c->fn) == hipSuccess;
        (void)hipFuncGetAttribute(&regs, HIP_FUNC_ATTRIBUTE_NUM_REGS, c->fn);
        if (getenv("DFMI_JIT_VERBOSE"))
            fprintf(stderr, "dfmi jit: %s waves_per_eu %d: scratch %d B/lane, %d VGPRs%s\n", X.kname.c_str(),
                    X.waves_per_eu, scratch, regs, got && scratch > kSoftSpill ? " -> recompiled without the hint" : "");
        if (got && scratch > kSoftSpill) {
            double ms2 = 0;
            X.waves_per_eu = 0;
            src = generate(P, X);
            c = compile(device, src, X.kname, &ms2);
            if (compile_ms) *compile_ms += ms2;
        }
    }
    h.mod = c;
    X.module = c;
    h.kname = X.kname;
    memcpy(h.lits, X.args_lits, sizeof h.lits);
    h.n_lits = X.n_lits;
    memcpy(h.str_off, X.str_off, sizeof h.str_off);
    memcpy(h.str_len, X.str_len, sizeof h.str_len);
    memcpy(h.str, X.str, sizeof h.str);
    h.n_str = X.n_str;
    h.str_bytes = X.str_bytes;
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_shapes.size() >= 4096) g_shapes.clear();  // bounded: programs come and go
    g_shapes[key] = h;
    return c->fn;
}

}  // namespace jit
}  // namespace dfmi
