// history.edn reader / writer (native Jepsen history
// ingestion; the store/ layout the demo writes, .gitignore:13, and that
// `lein run analyze` re-checks).
//
// Input: the op maps Jepsen writes, one per line or inside one vector, e.g.
//   {:type :invoke, :f :cas, :value [3 [1 4]], :process 7, :time 1234, :index 12}
//   {:type :info, :f :start, :value nil, :process :nemesis, :time 99, :index 13}
// Fields read: :type :f :process :value :index.  Every other field (and any
// EDN value: maps, sets, lists, strings, chars, tagged literals, metadata) is
// skipped by a generic reader.
//
// Independent tuples: EDN prints a jepsen.independent tuple (a MapEntry) as a
// plain [k v] vector, so the reader decides per history: if every client op
// (:f :read/:write/:cas) has a 2-element vector value, values are [k v]
// tuples (the register workload, etcdemo.clj:90, :120); otherwise values are
// used as they are.

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cctype>
#include <cstring>
#include <string>
#include <string_view>
#include <system_error>
#include <thread>
#include <unordered_map>

#include "common.hpp"

// Parsing is allocation-free per op (string_view tokens, fixed-depth value
// records) and, for the one-op-per-line form, split at line starts over up to
// 16 threads whose row blocks are concatenated in order.  Anything the split
// could misread (an op map spanning a line break inside a string) fails its
// chunk, and the whole text is then re-read serially, which gives the exact
// result or error.  LC_EDN_THREADS caps the thread count (1 = serial).

namespace {

enum : uint8_t { K_NIL, K_INT, K_VEC, K_OTHER };

// A :value, only as deep as the register workloads need: [k [a b]].
struct Leaf { uint8_t kind = K_OTHER; int64_t i = 0; };
struct Node { uint8_t kind = K_OTHER; int64_t i = 0; uint32_t n = 0; Leaf e[2]; };
struct Top { uint8_t kind = K_OTHER; int64_t i = 0; uint32_t n = 0; Node e[2]; };

struct Delims {
    bool d[256] = {};
    Delims() {
        for (unsigned char c : std::string_view(" \t\n\r,)]}([{\";")) d[c] = true;
    }
};
const Delims DELIM;

// A token of up to 8 bytes as one little-endian word (longer: ~0), so that
// keyword and symbol comparisons are integer compares, not library calls.
inline uint64_t pack8(std::string_view t) {
    if (t.size() > 8) return ~0ull;
    uint64_t x = 0;
    for (size_t i = 0; i < t.size(); ++i) x |= (uint64_t)(unsigned char)t[i] << (8 * i);
    return x;
}
template <size_t N>
constexpr uint64_t P8(const char (&s)[N]) {
    static_assert(N - 1 <= 8, "P8: at most 8 bytes");
    uint64_t x = 0;
    for (size_t i = 0; i + 1 < N; ++i) x |= (uint64_t)(unsigned char)s[i] << (8 * i);
    return x;
}

struct Parser {
    const char *p, *end, *base;
    std::string err;
    size_t err_off = 0;

    bool fail(const std::string &m) {
        if (err.empty()) { err = m; err_off = (size_t)(p - base); }
        return false;
    }
    void ws() {
        while (p < end) {
            const char c = *p;
            if (c == ' ' || c == ',' || c == '\n' || c == '\t' || c == '\r') ++p;
            else if (c == ';') { while (p < end && *p != '\n') ++p; }
            else break;
        }
    }
    std::string_view token() {
        const char *s = p;
        while (p < end && !DELIM.d[(unsigned char)*p]) ++p;
        return std::string_view(s, (size_t)(p - s));
    }
    bool string_lit() {
        ++p;
        while (p < end && *p != '"') p += (*p == '\\') ? 2 : 1;
        if (p >= end) return fail("unterminated string");
        ++p;
        return true;
    }
    // Metadata (^m) and discards (#_ x) in front of a value.
    bool prefixes() {
        ws();
        if (p < end && *p != '^' && *p != '#') return true;  // the common case
        for (;;) {
            ws();
            if (p >= end) return fail("unexpected end of input");
            if (*p == '^') { ++p; if (!skip()) return false; continue; }
            if (*p == '#' && p + 1 < end && p[1] == '_') { p += 2; if (!skip()) return false; continue; }
            return true;
        }
    }
    bool skip_seq(char close) {
        ++p;
        for (;;) {
            ws();
            if (p >= end) return fail("unterminated collection");
            if (*p == close) { ++p; return true; }
            if (!skip()) return false;
        }
    }
    // Read one scalar token (number / nil / true / false / symbol).
    bool scalar(uint8_t &kind, int64_t &v) {
        // the common case first: a decimal integer of at most 18 digits
        // followed by a delimiter (no overflow possible)
        {
            const char *q = p;
            const bool neg = q < end && *q == '-';
            if (q < end && (*q == '-' || *q == '+')) ++q;
            const char *d0 = q;
            uint64_t acc = 0;
            while (q < end && q - d0 < 18 && (unsigned)(*q - '0') < 10u) acc = acc * 10 + (uint64_t)(*q++ - '0');
            if (q > d0 && (q == end || DELIM.d[(unsigned char)*q])) {
                const int64_t val = neg ? -(int64_t)acc : (int64_t)acc;
                if (val != LC_NIL) {
                    p = q;
                    kind = K_INT;
                    v = val;
                    return true;
                }
            }
        }
        const char c = *p;
        std::string_view t = token();
        kind = K_OTHER;
        if (t.empty()) return fail(std::string("unexpected character '") + c + "'");
        if (pack8(t) == P8("nil")) { kind = K_NIL; return true; }
        const char f0 = t[0];
        const bool num = (f0 >= '0' && f0 <= '9') || ((f0 == '-' || f0 == '+') && t.size() > 1 && t[1] >= '0' && t[1] <= '9');
        if (!num) return true;  // true / false / symbol
        std::string_view d = t;
        if (d.back() == 'N' || d.back() == 'M') d.remove_suffix(1);
        if (d.find_first_of(".eE/") != std::string_view::npos) return true;  // not integral
        bool neg = false;
        size_t j = 0;
        if (d[0] == '-' || d[0] == '+') { neg = d[0] == '-'; j = 1; }
        unsigned __int128 acc = 0;
        for (; j < d.size(); ++j) {
            const char x = d[j];
            if (x < '0' || x > '9') return fail("integer out of range: " + std::string(t));
            acc = acc * 10 + (unsigned)(x - '0');
            if (acc > (unsigned __int128)INT64_MAX + 1) return fail("integer out of range: " + std::string(t));
        }
        if (!neg && acc > (unsigned __int128)INT64_MAX) return fail("integer out of range: " + std::string(t));
        const int64_t val = neg ? (int64_t)(0 - (uint64_t)acc) : (int64_t)acc;
        if (val == LC_NIL) return fail("integer reserved for nil: " + std::string(t));
        kind = K_INT;
        v = val;
        return true;
    }
    // Skip one value of any EDN kind.
    bool skip() {
        if (!prefixes()) return false;
        switch (*p) {
            case '[': return skip_seq(']');
            case '(': return skip_seq(')');
            case '{': return skip_seq('}');
            case '"': return string_lit();
            case '\\': ++p; if (p < end) ++p; token(); return true;  // char literal
            case ':': ++p; token(); return true;
            case '#': {
                ++p;
                if (p < end && *p == '{') return skip_seq('}');  // set
                if (p < end && *p == '"') return string_lit();   // regex
                token();                                         // tagged literal
                return skip();
            }
            default: {
                uint8_t k;
                int64_t v;
                return scalar(k, v);
            }
        }
    }
    // A value whose shape we keep: scalars, and vectors down to `depth`.
    template <class V>
    bool shaped(V &out);
    bool keyword(std::string_view &kw, bool &is_kw) {
        if (!prefixes()) return false;
        is_kw = *p == ':';
        if (!is_kw) return skip();
        ++p;
        kw = token();
        return true;
    }
};

template <class V>
bool Parser::shaped(V &out) {
    if (!prefixes()) return false;
    out.kind = K_OTHER;
    const char c = *p;
    if (c == '[') {
        out.kind = K_VEC;
        out.n = 0;
        ++p;
        for (;;) {
            ws();
            if (p >= end) return fail("unterminated collection");
            if (*p == ']') { ++p; return true; }
            bool ok;
            if constexpr (sizeof(V) == sizeof(Leaf)) {
                ok = skip();
            } else {
                if (out.n < 2) ok = shaped(out.e[out.n]);
                else ok = skip();
            }
            if (!ok) return false;
            ++out.n;
        }
    }
    if (c == '(' || c == '{' || c == '"' || c == '\\' || c == ':' || c == '#') return skip();
    return scalar(out.kind, out.i);
}
template <>
bool Parser::shaped<Leaf>(Leaf &out) {
    if (!prefixes()) return false;
    out.kind = K_OTHER;
    const char c = *p;
    if (c == '[' || c == '(' || c == '{' || c == '"' || c == '\\' || c == ':' || c == '#') return skip();
    return scalar(out.kind, out.i);
}

struct RawOp {
    uint8_t type = 255, f = LC_F_OTHER;
    int8_t nem = -1;  // nemesis :f :start (1) / :stop (0)
    int64_t process = LC_NO_PROCESS, index = -1;
    Top value;
    const char *vb = nullptr;  // where the :value's text starts (a :txn value is read again from there)
};

// Register names of :txn micro-ops, interned in order of first appearance.
struct Names {
    std::unordered_map<std::string, int64_t> id;
    std::vector<std::string> names;
    int64_t of(std::string_view t) {
        auto it = id.find(std::string(t));
        if (it != id.end()) return it->second;
        const int64_t v = LC_NAMED_REG_BASE + (int64_t)names.size();
        names.emplace_back(t);
        id.emplace(names.back(), v);
        return v;
    }
};

// A :txn op's value is [k txn] (an independent tuple) when its first element
// is an integer; a txn of two micro-ops starts with a vector instead.
bool txn_tuple(const Top &v) { return v.kind == K_VEC && v.n == 2 && v.e[0].kind == K_INT; }

// The op-map keys read, by length and spelling (one compare per key).
enum Field { FLD_OTHER, FLD_TYPE, FLD_F, FLD_PROCESS, FLD_INDEX, FLD_VALUE };
inline Field field_of(std::string_view k) {
    switch (pack8(k)) {
        case P8("f"): return FLD_F;
        case P8("type"): return FLD_TYPE;
        case P8("value"): return FLD_VALUE;
        case P8("index"): return FLD_INDEX;
        case P8("process"): return FLD_PROCESS;
        default: return FLD_OTHER;
    }
}

bool read_op(Parser &ps, RawOp &op) {
    ++ps.p;  // at '{'
    for (;;) {
        ps.ws();
        if (ps.p >= ps.end) return ps.fail("unterminated op map");
        if (*ps.p == '}') { ++ps.p; break; }
        std::string_view k;
        bool is_kw = false;
        if (!ps.keyword(k, is_kw)) return false;
        if (!is_kw) {  // non-keyword key: skip its value
            if (!ps.skip()) return false;
            continue;
        }
        const Field fld = field_of(k);
        if (fld == FLD_TYPE || fld == FLD_F) {
            std::string_view v;
            bool vk = false;
            if (!ps.keyword(v, vk)) return false;
            if (fld == FLD_TYPE) {
                if (!vk) return ps.fail(":type is not a keyword");
                switch (pack8(v)) {
                    case P8("invoke"): op.type = LC_INVOKE; break;
                    case P8("ok"): op.type = LC_OK_T; break;
                    case P8("fail"): op.type = LC_FAIL; break;
                    case P8("info"): op.type = LC_INFO; break;
                    default: return ps.fail("unknown :type :" + std::string(v));
                }
            } else {
                op.f = LC_F_OTHER;
                op.nem = -1;
                if (vk) {
                    switch (pack8(v)) {
                        case P8("read"): op.f = LC_F_READ; break;
                        case P8("write"): op.f = LC_F_WRITE; break;
                        case P8("cas"): op.f = LC_F_CAS; break;
                        case P8("acquire"): op.f = LC_F_ACQUIRE; break;  // (model/mutex)
                        case P8("release"): op.f = LC_F_RELEASE; break;
                        case P8("txn"): op.f = LC_F_TXN; break;          // (model/multi-register)
                        case P8("start"): op.nem = 1; break;             // nemesis
                        case P8("stop"): op.nem = 0; break;
                        default: break;
                    }
                }
            }
        } else if (fld == FLD_PROCESS || fld == FLD_INDEX) {
            Leaf v;
            if (!ps.shaped(v)) return false;
            if (fld == FLD_PROCESS) op.process = v.kind == K_INT ? v.i : LC_NO_PROCESS;
            else op.index = v.kind == K_INT ? v.i : -1;
        } else if (fld == FLD_VALUE) {
            if (!ps.prefixes()) return false;
            op.vb = ps.p;
            if (!ps.shaped(op.value)) return false;
        } else {
            if (!ps.skip()) return false;
        }
    }
    if (op.type == 255) return ps.fail("op map without :type");
    return true;
}

enum { CONV_OK = 0, CONV_KEY = 1, CONV_VALUE = 2, CONV_TXN = 3 };

// One micro-op [f k v]: f :read/:write (or :r/:w), k an integer or a name,
// v an integer or nil.
bool micro_op(Parser &ps, Names &names, std::vector<int64_t> &out) {
    if (!ps.prefixes() || *ps.p != '[') return false;
    ++ps.p;
    std::string_view f;
    bool fk = false;
    if (!ps.keyword(f, fk) || !fk) return false;
    int64_t code;
    if (f == "read" || f == "r") code = LC_MOP_READ;
    else if (f == "write" || f == "w") code = LC_MOP_WRITE;
    else return false;
    if (!ps.prefixes()) return false;
    int64_t reg;
    const char c = *ps.p;
    if (c == ':' || c == '"' || (c != '-' && c != '+' && (c < '0' || c > '9'))) {
        const char *b = ps.p;
        if (!ps.skip()) return false;
        const std::string_view t(b, (size_t)(ps.p - b));
        if (t == "nil" || t.empty()) return false;
        reg = names.of(t);
    } else {
        uint8_t kind;
        if (!ps.scalar(kind, reg) || kind != K_INT || reg >= LC_NAMED_REG_BASE) return false;
    }
    Leaf v;
    if (!ps.shaped(v) || (v.kind != K_INT && v.kind != K_NIL)) return false;
    const int64_t val = v.kind == K_NIL ? LC_NIL : v.i;
    if (val == LC_NIL + 1) return false;  // the multi-register model's "absent"
    ps.ws();
    if (ps.p >= ps.end || *ps.p != ']') return false;
    ++ps.p;
    out.push_back(code);
    out.push_back(reg);
    out.push_back(val);
    return true;
}

// A :txn value (nil, or a vector of micro-ops), read from its text.
bool txn_value(Parser &ps, Names &names, std::vector<int64_t> &out) {
    if (!ps.prefixes()) return false;
    if (*ps.p != '[') {
        uint8_t kind;
        int64_t v;
        return ps.scalar(kind, v) && kind == K_NIL;
    }
    ++ps.p;
    for (;;) {
        ps.ws();
        if (ps.p >= ps.end) return false;
        if (*ps.p == ']') { ++ps.p; return true; }
        if (!micro_op(ps, names, out)) return false;
    }
}

template <class V>
int64_t scal(const V &v, bool &ok) {
    if (v.kind == K_NIL) return LC_NIL;
    if (v.kind == K_INT) return v.i;
    ok = false;
    return LC_NIL;
}

template <class V>
bool register_value(uint8_t f, const V &val, int64_t &v0, int64_t &v1) {
    bool ok = true;
    if (f == LC_F_ACQUIRE || f == LC_F_RELEASE) return true;  // mutex ops carry no register value
    if (f == LC_F_CAS) {
        if (val.kind == K_VEC && val.n == 2) { v0 = scal(val.e[0], ok); v1 = scal(val.e[1], ok); }
        else if (val.kind != K_NIL) ok = false;
        return ok;
    }
    v0 = scal(val, ok);
    return ok;
}

// One row from a parsed op.  indep: values are [k v] tuples.  A :txn row's
// micro-ops are read from the value's text (names: the register interner).
int convert(const RawOp &o, bool indep, lc_hist &h, Names *names, const char *end, const char *base) {
    int64_t key = LC_NO_KEY, v0 = LC_NIL, v1 = LC_NIL;
    if (o.f == LC_F_TXN) {
        std::vector<int64_t> mops;
        if (o.vb) {
            Parser tp{o.vb, end, base};
            if (indep) {
                tp.ws();
                ++tp.p;  // '[' of the [k txn] tuple (txn_tuple checked it)
                uint8_t kind;
                tp.ws();
                if (!tp.scalar(kind, key) || kind != K_INT) return CONV_KEY;
            }
            if (!txn_value(tp, *names, mops)) return CONV_TXN;
        }
        h.push(o.type, o.f, o.process, key, v0, v1, o.index);
        h.set_mops(mops.data(), mops.size() / 3);
        return CONV_OK;
    }
    if (o.f == LC_F_OTHER) {
        if (o.nem >= 0) v0 = o.nem;
    } else if (indep) {
        bool ok = true;
        key = scal(o.value.e[0], ok);
        if (!ok || key == LC_NIL) return CONV_KEY;
        if (!register_value(o.f, o.value.e[1], v0, v1)) return CONV_VALUE;
    } else {
        if (!register_value(o.f, o.value, v0, v1)) return CONV_VALUE;
    }
    h.push(o.type, o.f, o.process, key, v0, v1, o.index);
    return CONV_OK;
}

// Parse [b, e) of one-op-per-line text (or, whole=true, the full text in
// either form) into rows.  Tuple mode is assumed; a client op whose value is
// not a 2-vector ends the chunk with not_indep set.
struct alignas(256) Chunk {
    lc_hist rows;
    std::string err;
    size_t err_off = 0;
    int conv_err = CONV_OK;
    int64_t conv_row = -1;  // chunk-local op number of a conversion error
    bool not_indep = false, any_client = false;
    bool need_serial = false;  // a :txn op in a parallel chunk (one interner for the whole file)
    Names names;
};

void parse_range(const char *base, const char *b, const char *e, bool indep, bool whole, Chunk &out) {
    Parser ps{b, e, base};
    out.rows.reserve((size_t)(e - b) / 64 + 16);  // ~70-100 bytes per Jepsen op line
    auto one = [&](void) -> bool {
        RawOp op;
        if (!read_op(ps, op)) return false;
        if (op.f == LC_F_TXN && !whole) { out.need_serial = true; return false; }
        if (op.f != LC_F_OTHER) {
            out.any_client = true;
            const bool tup = op.f == LC_F_TXN ? txn_tuple(op.value) : (op.value.kind == K_VEC && op.value.n == 2);
            if (indep && !tup) { out.not_indep = true; return false; }
        }
        const int rc = convert(op, indep, out.rows, &out.names, e, base);
        if (rc != CONV_OK) { out.conv_err = rc; out.conv_row = out.rows.size(); return false; }
        return true;
    };
    for (;;) {
        ps.ws();
        if (ps.p >= ps.end) break;
        if (*ps.p == '{') {
            if (!one()) break;
        } else if (whole && *ps.p == '[') {  // a vector of op maps
            ++ps.p;
            bool closed = false;
            for (;;) {
                ps.ws();
                if (ps.p >= ps.end) { ps.fail("unterminated history vector"); break; }
                if (*ps.p == ']') { ++ps.p; closed = true; break; }
                if (*ps.p != '{') { ps.fail("expected an op map"); break; }
                if (!one()) break;
            }
            if (!closed) break;
        } else {
            ps.fail("expected an op map");
            break;
        }
    }
    out.err = ps.err;
    out.err_off = ps.err_off;
}

int64_t line_of(const char *text, size_t off) {
    return 1 + (int64_t)std::count(text, text + off, '\n');
}

int finish_serial(const char *text, int64_t len, lc_hist **out) {
    // pass 1 assumes [k v] tuples; a client op that is not one means the
    // history is not independent and it is read again with plain values
    for (int pass = 0; pass < 2; ++pass) {
        const bool indep = pass == 0;
        auto *c = new (std::nothrow) Chunk();
        if (!c) return lc::fail(LC_E_NOMEM, "lc_edn: out of memory");
        parse_range(text, text, text + len, indep, true, *c);
        if (!c->err.empty()) {
            const int rc = lc::fail(LC_E_PARSE, "lc_edn: line %lld: %s", (long long)line_of(text, c->err_off),
                                    c->err.c_str());
            delete c;
            return rc;
        }
        if (indep && (c->not_indep || !c->any_client)) { delete c; continue; }
        if (c->conv_err != CONV_OK) {
            const int rc = c->conv_err == CONV_KEY
                               ? lc::fail(LC_E_UNSUPPORTED, "lc_edn: op %lld: tuple key is not an integer",
                                          (long long)c->conv_row)
                           : c->conv_err == CONV_TXN
                               ? lc::fail(LC_E_UNSUPPORTED,
                                          "lc_edn: op %lld: :txn value is not nil or [[:read|:write k v] ...]",
                                          (long long)c->conv_row)
                               : lc::fail(LC_E_UNSUPPORTED,
                                          "lc_edn: op %lld: value is not an integer, nil or [old new]",
                                          (long long)c->conv_row);
            delete c;
            return rc;
        }
        lc_hist *h = new (std::nothrow) lc_hist(std::move(c->rows));
        if (h) {
            h->reg_names = std::move(c->names.names);
            h->finish_mops();
        }
        delete c;
        if (!h) return lc::fail(LC_E_NOMEM, "lc_edn: out of memory");
        *out = h;
        return LC_OK;
    }
    return lc::fail(LC_E_PARSE, "lc_edn: internal error");  // not reached
}

}  // namespace

extern "C" int lc_edn_parse(const char *text, int64_t len, lc_hist **out) {
    lc::Range range("lc_edn_parse");
    if (!text || !out || len < 0) return lc::fail(LC_E_INVALID, "lc_edn_parse: null argument");
    try {
        const char *b = text, *e = text + len;
        while (b < e && (*b == ' ' || *b == '\n' || *b == '\t' || *b == '\r' || *b == ',')) ++b;
        const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
        int T = (int)std::min<int64_t>({16, (int64_t)hw, len >> 20});
        if (const char *ev = std::getenv("LC_EDN_THREADS")) T = std::min(T, std::atoi(ev));
        if (T < 2 || b >= e || *b != '{') return finish_serial(text, len, out);
        // split at line starts that open an op map
        std::vector<const char *> cut{b};
        for (int i = 1; i < T; ++i) {
            const char *q = std::max(cut.back(), text + len * i / T);
            while (q < e && !(q[-1] == '\n' && *q == '{')) ++q;
            if (q < e && q > cut.back()) cut.push_back(q);
        }
        cut.push_back(e);
        const size_t n = cut.size() - 1;
        std::vector<Chunk> ch(n);
        std::vector<std::thread> th;
        th.reserve(n);
        bool spawned = true;
        try {
            for (size_t i = 0; i < n; ++i)
                th.emplace_back([&, i] { parse_range(text, cut[i], cut[i + 1], true, false, ch[i]); });
        } catch (const std::system_error &) {
            spawned = false;  // joined below, then the serial read
        }
        for (auto &t : th) t.join();
        if (!spawned) return finish_serial(text, len, out);
        bool any_client = false;
        for (auto &c : ch) {
            if (!c.err.empty() || c.not_indep || c.need_serial || c.conv_err != CONV_OK) return finish_serial(text, len, out);
            any_client |= c.any_client;
        }
        if (!any_client) return finish_serial(text, len, out);
        lc_hist *h = new (std::nothrow) lc_hist();
        if (!h) return lc::fail(LC_E_NOMEM, "lc_edn: out of memory");
        size_t total = 0;
        for (auto &c : ch) total += c.rows.type.size();
        h->reserve(total);
        for (auto &c : ch) {
            auto app = [](auto &dst, auto &src) { dst.insert(dst.end(), src.begin(), src.end()); };
            app(h->type, c.rows.type); app(h->f, c.rows.f); app(h->process, c.rows.process);
            app(h->key, c.rows.key); app(h->v0, c.rows.v0); app(h->v1, c.rows.v1); app(h->index, c.rows.index);
            c.rows = lc_hist();
        }
        *out = h;
        return LC_OK;
    } catch (const std::bad_alloc &) {
        return lc::fail(LC_E_NOMEM, "lc_edn: out of memory");
    } catch (const std::system_error &) {
        return finish_serial(text, len, out);  // no threads: serial read
    }
}

extern "C" int lc_edn_read(const char *path, lc_hist **out) {
    if (!path || !out) return lc::fail(LC_E_INVALID, "lc_edn_read: null argument");
    FILE *f = std::fopen(path, "rb");
    if (!f) return lc::fail(LC_E_IO, "lc_edn_read: cannot open %s", path);
    std::string s;
    try {
        if (std::fseek(f, 0, SEEK_END) == 0) {
            const long sz = std::ftell(f);
            if (sz > 0) s.resize((size_t)sz);
            std::rewind(f);
        }
        size_t got = s.empty() ? 0 : std::fread(&s[0], 1, s.size(), f);
        s.resize(got);
        char buf[1 << 16];
        size_t r;
        while ((r = std::fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, r);  // growing / unseekable files
    } catch (const std::bad_alloc &) {
        std::fclose(f);
        return lc::fail(LC_E_NOMEM, "lc_edn_read: out of memory");
    }
    std::fclose(f);
    return lc_edn_parse(s.data(), (int64_t)s.size(), out);
}

static void put_scalar(std::string &o, int64_t v) {
    if (v == LC_NIL) o += "nil"; else o += std::to_string(v);
}

// A register name as lc_edn_read keeps it (":x", "\"z\"", ...) is written back
// verbatim when it reads as one EDN token; anything else becomes :r<i>.
static bool edn_token(const char *s) {
    if (!s || !*s) return false;
    if (*s == '"') {
        const size_t n = std::strlen(s);
        if (n < 2 || s[n - 1] != '"') return false;
        for (size_t i = 1; i + 1 < n; ++i)
            if (s[i] == '"' || s[i] == '\\' || s[i] == '\n') return false;
        return true;
    }
    for (const char *c = s; *c; ++c)
        if (std::isspace((unsigned char)*c) || std::strchr("[](){}\",;\\", *c)) return false;
    return true;
}

extern "C" int lc_edn_write(const char *path, const lc_history *h) { return lc_edn_write_named(path, h, nullptr, 0); }

extern "C" int lc_edn_write_named(const char *path, const lc_history *h, const char *const *reg_names,
                                  int64_t n_reg_names) {
    if (!path || !h || h->n < 0) return lc::fail(LC_E_INVALID, "lc_edn_write: null argument");
    if (n_reg_names < 0 || (n_reg_names > 0 && !reg_names))
        return lc::fail(LC_E_INVALID, "lc_edn_write_named: bad register names");
    FILE *f = std::fopen(path, "wb");
    if (!f) return lc::fail(LC_E_IO, "lc_edn_write: cannot open %s", path);
    static const char *types[] = {"invoke", "ok", "fail", "info"};
    static const char *fs[] = {"read", "write", "cas", "", "acquire", "release", "txn"};
    std::string line;
    for (int64_t r = 0; r < h->n; ++r) {
        line.clear();
        if (h->type[r] > LC_INFO || h->f[r] > LC_F_TXN) { std::fclose(f); return lc::fail(LC_E_INVALID, "lc_edn_write: bad row %lld", (long long)r); }
        line += "{:type :"; line += types[h->type[r]];
        if (h->f[r] == LC_F_TXN) {
            // [[:read k v] ...]; named registers (ids from LC_NAMED_REG_BASE) by
            // their names when given, else as :r<i>
            std::string v = "nil";
            const int64_t mb = h->mop_off ? h->mop_off[r] : 0, me = h->mop_off ? h->mop_off[r + 1] : 0;
            if (me > mb) {
                v = "[";
                for (int64_t m = mb; m < me; ++m) {
                    const int64_t *t = h->mop + 3 * m;
                    v += m > mb ? " [:" : "[:";
                    v += t[0] == LC_MOP_WRITE ? "write " : "read ";
                    const int64_t ni = t[1] - LC_NAMED_REG_BASE;
                    if (t[1] >= LC_NAMED_REG_BASE && ni < n_reg_names && edn_token(reg_names[ni])) v += reg_names[ni];
                    else if (t[1] >= LC_NAMED_REG_BASE) { v += ":r"; v += std::to_string(ni); }
                    else v += std::to_string(t[1]);
                    v += " ";
                    put_scalar(v, t[2]);
                    v += "]";
                }
                v += "]";
            }
            line += ", :f :txn, :value ";
            if (h->key[r] != LC_NO_KEY) { line += "["; line += std::to_string(h->key[r]); line += " "; line += v; line += "]"; }
            else line += v;
        } else if (h->f[r] == LC_F_OTHER) {
            line += ", :f :"; line += h->v0[r] == 1 ? "start" : h->v0[r] == 0 ? "stop" : "nemesis";
            line += ", :value nil";
        } else {
            line += ", :f :"; line += fs[h->f[r]];
            line += ", :value ";
            std::string v;
            if (h->f[r] == LC_F_ACQUIRE || h->f[r] == LC_F_RELEASE) {
                v = "nil";
            } else if (h->f[r] == LC_F_CAS) {
                if (h->v0[r] == LC_NIL && h->v1[r] == LC_NIL && h->type[r] == LC_INVOKE) v = "nil";
                else { v = "["; put_scalar(v, h->v0[r]); v += " "; put_scalar(v, h->v1[r]); v += "]"; }
            } else {
                put_scalar(v, h->v0[r]);
            }
            if (h->key[r] != LC_NO_KEY) { line += "["; line += std::to_string(h->key[r]); line += " "; line += v; line += "]"; }
            else line += v;
        }
        line += ", :process ";
        if (h->process[r] == LC_NO_PROCESS) line += ":nemesis"; else line += std::to_string(h->process[r]);
        line += ", :index ";
        line += std::to_string(h->index && h->index[r] >= 0 ? h->index[r] : r);
        line += "}\n";
        if (std::fwrite(line.data(), 1, line.size(), f) != line.size()) { std::fclose(f); return lc::fail(LC_E_IO, "lc_edn_write: write failed"); }
    }
    if (std::fclose(f) != 0) return lc::fail(LC_E_IO, "lc_edn_write: close failed");
    return LC_OK;
}
