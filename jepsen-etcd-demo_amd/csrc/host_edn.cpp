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

#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>

#include "common.hpp"

namespace {

// A parsed value, only as deep as this workload needs.
struct Val {
    enum Kind { NIL, INT, KW, VEC, OTHER } kind = OTHER;
    int64_t i = 0;
    std::string kw;
    std::vector<Val> v;
};

struct Parser {
    const char *p, *end;
    int64_t line = 1;
    std::string err;

    bool fail(const std::string &m) {
        if (err.empty()) err = "line " + std::to_string(line) + ": " + m;
        return false;
    }
    void ws() {
        while (p < end) {
            char c = *p;
            if (c == '\n') { ++line; ++p; }
            else if (c == ' ' || c == '\t' || c == '\r' || c == ',') ++p;
            else if (c == ';') { while (p < end && *p != '\n') ++p; }
            else break;
        }
    }
    static bool delim(char c) {
        return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == ',' || c == ')' || c == ']' ||
               c == '}' || c == '(' || c == '[' || c == '{' || c == '"' || c == ';';
    }
    std::string token() {
        const char *s = p;
        while (p < end && !delim(*p)) ++p;
        return std::string(s, p);
    }
    bool parse_seq(char close, Val *out) {
        ++p;  // opening bracket
        for (;;) {
            ws();
            if (p >= end) return fail("unterminated collection");
            if (*p == close) { ++p; return true; }
            Val x;
            if (!value(out ? &x : nullptr)) return false;
            if (out) out->v.push_back(std::move(x));
        }
    }
    bool string_lit() {
        ++p;
        while (p < end && *p != '"') {
            if (*p == '\\') ++p;
            else if (*p == '\n') ++line;
            ++p;
        }
        if (p >= end) return fail("unterminated string");
        ++p;
        return true;
    }
    // Parse one value; out may be null (skip).
    bool value(Val *out) {
        ws();
        if (p >= end) return fail("unexpected end of input");
        char c = *p;
        if (out) out->kind = Val::OTHER;
        switch (c) {
            case '[':
                if (out) out->kind = Val::VEC;
                return parse_seq(']', out);
            case '(': return parse_seq(')', nullptr);
            case '{': return parse_seq('}', nullptr);
            case '"': return string_lit();
            case '\\': ++p; if (p < end) ++p; token(); return true;  // char literal
            case '^': ++p; if (!value(nullptr)) return false; return value(out);  // metadata
            case '#': {
                ++p;
                if (p < end && *p == '{') return parse_seq('}', nullptr);  // set
                if (p < end && *p == '_') { ++p; if (!value(nullptr)) return false; return value(out); }
                if (p < end && *p == '"') return string_lit();            // regex
                token();                                                  // tag
                return value(nullptr);
            }
            case ':': {
                ++p;
                std::string t = token();
                if (out) { out->kind = Val::KW; out->kw = t; }
                return true;
            }
            default: break;
        }
        std::string t = token();
        if (t.empty()) return fail(std::string("unexpected character '") + c + "'");
        if (t == "nil") { if (out) out->kind = Val::NIL; return true; }
        if (t == "true" || t == "false") return true;
        char first = t[0];
        if ((first >= '0' && first <= '9') || ((first == '-' || first == '+') && t.size() > 1 && t[1] >= '0' && t[1] <= '9')) {
            std::string num = t;
            if (!num.empty() && (num.back() == 'N' || num.back() == 'M')) num.pop_back();
            bool integral = num.find_first_of(".eE/") == std::string::npos;
            if (integral && out) {
                errno = 0;
                char *e = nullptr;
                long long v = std::strtoll(num.c_str(), &e, 10);
                if (errno || *e) return fail("integer out of range: " + t);
                if (v == LC_NIL) return fail("integer reserved for nil: " + t);
                out->kind = Val::INT;
                out->i = v;
            }
            return true;
        }
        return true;  // symbol
    }
};

struct RawOp {
    uint8_t type = 255, f = LC_F_OTHER;
    int64_t process = LC_NO_PROCESS, index = -1;
    Val value;
    bool has_value = false;
};

bool read_op(Parser &ps, RawOp &op) {
    // at '{'
    ++ps.p;
    for (;;) {
        ps.ws();
        if (ps.p >= ps.end) return ps.fail("unterminated op map");
        if (*ps.p == '}') { ++ps.p; break; }
        Val k;
        if (!ps.value(&k)) return false;
        if (k.kind != Val::KW) {  // non-keyword key: skip its value
            if (!ps.value(nullptr)) return false;
            continue;
        }
        if (k.kw == "type" || k.kw == "f") {
            Val v;
            if (!ps.value(&v)) return false;
            if (k.kw == "type") {
                if (v.kind != Val::KW) return ps.fail(":type is not a keyword");
                if (v.kw == "invoke") op.type = LC_INVOKE;
                else if (v.kw == "ok") op.type = LC_OK_T;
                else if (v.kw == "fail") op.type = LC_FAIL;
                else if (v.kw == "info") op.type = LC_INFO;
                else return ps.fail("unknown :type :" + v.kw);
            } else {
                if (v.kind == Val::KW && v.kw == "read") op.f = LC_F_READ;
                else if (v.kind == Val::KW && v.kw == "write") op.f = LC_F_WRITE;
                else if (v.kind == Val::KW && v.kw == "cas") op.f = LC_F_CAS;
                else if (v.kind == Val::KW && v.kw == "acquire") op.f = LC_F_ACQUIRE;  // (model/mutex)
                else if (v.kind == Val::KW && v.kw == "release") op.f = LC_F_RELEASE;
                else {
                    op.f = LC_F_OTHER;
                    if (v.kind == Val::KW) op.value.kw = v.kw;  // remembered for nemesis :start/:stop
                }
            }
        } else if (k.kw == "process") {
            Val v;
            if (!ps.value(&v)) return false;
            op.process = v.kind == Val::INT ? v.i : LC_NO_PROCESS;
        } else if (k.kw == "index") {
            Val v;
            if (!ps.value(&v)) return false;
            op.index = v.kind == Val::INT ? v.i : -1;
        } else if (k.kw == "value") {
            std::string keep = op.value.kw;
            if (!ps.value(&op.value)) return false;
            if (op.value.kw.empty()) op.value.kw = keep;
            op.has_value = true;
        } else {
            if (!ps.value(nullptr)) return false;
        }
    }
    if (op.type == 255) return ps.fail("op map without :type");
    return true;
}

int64_t scalar(const Val &v, bool &ok) {
    if (v.kind == Val::NIL) return LC_NIL;
    if (v.kind == Val::INT) return v.i;
    ok = false;
    return LC_NIL;
}

int build(std::vector<RawOp> &ops, lc_hist **out) {
    // independent iff every client op's value is a 2-vector
    bool indep = false, any_client = false;
    for (const RawOp &o : ops) {
        if (o.f == LC_F_OTHER) continue;
        any_client = true;
        indep = true;
    }
    for (const RawOp &o : ops) {
        if (o.f == LC_F_OTHER) continue;
        if (!(o.value.kind == Val::VEC && o.value.v.size() == 2)) { indep = false; break; }
    }
    if (!any_client) indep = false;
    lc_hist *h = new (std::nothrow) lc_hist();
    if (!h) return lc::fail(LC_E_NOMEM, "lc_edn: out of memory");
    h->reserve(ops.size());
    for (size_t i = 0; i < ops.size(); ++i) {
        const RawOp &o = ops[i];
        int64_t key = LC_NO_KEY, v0 = LC_NIL, v1 = LC_NIL;
        bool ok = true;
        const Val *val = &o.value;
        if (o.f == LC_F_OTHER) {
            if (o.value.kw == "start") v0 = 1;
            else if (o.value.kw == "stop") v0 = 0;
        } else {
            if (indep) {
                key = scalar(o.value.v[0], ok);
                if (!ok || key == LC_NIL) { delete h; return lc::fail(LC_E_UNSUPPORTED, "lc_edn: op %zu: tuple key is not an integer", i); }
                val = &o.value.v[1];
            }
            if (o.f == LC_F_ACQUIRE || o.f == LC_F_RELEASE) {
                // mutex ops carry no register value (knossos.model/mutex ignores it)
            } else if (o.f == LC_F_CAS) {
                if (val->kind == Val::VEC && val->v.size() == 2) {
                    v0 = scalar(val->v[0], ok);
                    v1 = scalar(val->v[1], ok);
                } else if (val->kind != Val::NIL) {
                    ok = false;
                }
            } else {
                v0 = scalar(*val, ok);
            }
            if (!ok) { delete h; return lc::fail(LC_E_UNSUPPORTED, "lc_edn: op %zu: value is not an integer, nil or [old new]", i); }
        }
        h->push(o.type, o.f, o.process, key, v0, v1, o.index);
    }
    *out = h;
    return LC_OK;
}

}  // namespace

extern "C" int lc_edn_parse(const char *text, int64_t len, lc_hist **out) {
    if (!text || !out || len < 0) return lc::fail(LC_E_INVALID, "lc_edn_parse: null argument");
    Parser ps{text, text + len};
    std::vector<RawOp> ops;
    try {
        for (;;) {
            ps.ws();
            if (ps.p >= ps.end) break;
            if (*ps.p == '{') {
                RawOp op;
                if (!read_op(ps, op)) return lc::fail(LC_E_PARSE, "lc_edn: %s", ps.err.c_str());
                ops.push_back(std::move(op));
            } else if (*ps.p == '[') {  // a vector of op maps
                ++ps.p;
                for (;;) {
                    ps.ws();
                    if (ps.p >= ps.end) return lc::fail(LC_E_PARSE, "lc_edn: unterminated history vector");
                    if (*ps.p == ']') { ++ps.p; break; }
                    if (*ps.p != '{') return lc::fail(LC_E_PARSE, "lc_edn: line %lld: expected an op map", (long long)ps.line);
                    RawOp op;
                    if (!read_op(ps, op)) return lc::fail(LC_E_PARSE, "lc_edn: %s", ps.err.c_str());
                    ops.push_back(std::move(op));
                }
            } else {
                return lc::fail(LC_E_PARSE, "lc_edn: line %lld: expected an op map", (long long)ps.line);
            }
        }
        return build(ops, out);
    } catch (const std::bad_alloc &) {
        return lc::fail(LC_E_NOMEM, "lc_edn: out of memory");
    }
}

extern "C" int lc_edn_read(const char *path, lc_hist **out) {
    if (!path || !out) return lc::fail(LC_E_INVALID, "lc_edn_read: null argument");
    std::ifstream in(path, std::ios::binary);
    if (!in) return lc::fail(LC_E_IO, "lc_edn_read: cannot open %s", path);
    std::ostringstream ss;
    ss << in.rdbuf();
    std::string s = ss.str();
    return lc_edn_parse(s.data(), (int64_t)s.size(), out);
}

static void put_scalar(std::string &o, int64_t v) {
    if (v == LC_NIL) o += "nil"; else o += std::to_string(v);
}

extern "C" int lc_edn_write(const char *path, const lc_history *h) {
    if (!path || !h || h->n < 0) return lc::fail(LC_E_INVALID, "lc_edn_write: null argument");
    FILE *f = std::fopen(path, "wb");
    if (!f) return lc::fail(LC_E_IO, "lc_edn_write: cannot open %s", path);
    static const char *types[] = {"invoke", "ok", "fail", "info"};
    static const char *fs[] = {"read", "write", "cas", "", "acquire", "release"};
    std::string line;
    for (int64_t r = 0; r < h->n; ++r) {
        line.clear();
        if (h->type[r] > LC_INFO || h->f[r] > LC_F_RELEASE) { std::fclose(f); return lc::fail(LC_E_INVALID, "lc_edn_write: bad row %lld", (long long)r); }
        line += "{:type :"; line += types[h->type[r]];
        if (h->f[r] == LC_F_OTHER) {
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
