// test.fressian reader / writer ("and later test.fressian":
// the binary store file Jepsen writes beside history.edn for each run, under
// the store/ layout the demo keeps, .gitignore:13).
//
// Parity unpinned: the reference holds no stored run (store/ is
// dangling symlinks) and the image has neither a JVM nor a Fressian library.
// The decoder follows the published Fressian encoding (org.fressian 0.6.x,
// the version jepsen 0.2.x pulls in through clojure.data.fressian 0.2.1):
// byte codes, packed ints, the priority cache, struct types and the struct
// cache, chunked strings/bytes, closed and open lists, and the footer.  Values
// are decoded into a small tree; every tagged struct whose handler this
// reader does not know becomes a "tagged" node holding its fields, so a
// history survives whichever handlers wrote the surrounding test map.
//
// What is read: the top-level object is either the test map (the history is
// its :history entry) or a list of op maps.  From each op map the fields
// :type :f :process :value :index, with the same rules as history.edn
// (host_edn.cpp): [k v] independent tuples when every client op's value is a
// 2-element sequence, [old new] for :cas, :nemesis processes as
// LC_NO_PROCESS.  A tuple may arrive as a list or as a tagged struct of two
// fields (a MapEntry under a "map-entry"/"tuple" handler) or of one list field
// (a "vec" handler); all three read the same.

#include <cstdio>
#include <cstring>
#include <string>
#include <string_view>

#include "common.hpp"

namespace {

// Fressian byte codes (org.fressian.impl.Codes).
enum : uint8_t {
    PRIORITY_CACHE_PACKED_START = 0x80, PRIORITY_CACHE_PACKED_END = 0xA0,
    STRUCT_CACHE_PACKED_START = 0xA0, STRUCT_CACHE_PACKED_END = 0xB0,
    LONG_ARRAY = 0xB0, DOUBLE_ARRAY = 0xB1, BOOLEAN_ARRAY = 0xB2, INT_ARRAY = 0xB3,
    FLOAT_ARRAY = 0xB4, OBJECT_ARRAY = 0xB5,
    MAP = 0xC0, SET = 0xC1, UUID = 0xC3, REGEX = 0xC4, URI = 0xC5, BIGINT = 0xC6,
    BIGDEC = 0xC7, INST = 0xC8, SYM = 0xC9, KEY = 0xCA,
    GET_PRIORITY_CACHE = 0xCC, PUT_PRIORITY_CACHE = 0xCD, PRECACHE = 0xCE, FOOTER = 0xCF,
    BYTES_PACKED_LENGTH_START = 0xD0, BYTES_CHUNK = 0xD8, BYTES = 0xD9,
    STRING_PACKED_LENGTH_START = 0xDA, STRING_CHUNK = 0xE2, STRING = 0xE3,
    LIST_PACKED_LENGTH_START = 0xE4, LIST = 0xEC, BEGIN_CLOSED_LIST = 0xED,
    BEGIN_OPEN_LIST = 0xEE, STRUCTTYPE = 0xEF, STRUCT = 0xF0, META = 0xF1,
    TRUE = 0xF5, FALSE = 0xF6, NULL_ = 0xF7, INT = 0xF8, FLOAT = 0xF9, DOUBLE = 0xFA,
    DOUBLE_0 = 0xFB, DOUBLE_1 = 0xFC, END_COLLECTION = 0xFD, RESET_CACHES = 0xFE,
};

enum : uint8_t { V_NIL, V_BOOL, V_INT, V_DBL, V_STR, V_KW, V_SYM, V_LIST, V_MAP, V_SET, V_TAGGED, V_BLOB };

// One decoded value.  Strings live in the string pool (a, n); collections
// hold their children's node ids in the kids array (a, n; a map's are k, v
// pairs); a keyword / symbol holds its name (a, n) and namespace string node
// (ns, or -1); a tagged struct its tag string node (ns) and fields (a, n).
struct Val {
    uint8_t kind = V_NIL;
    int64_t i = 0;
    uint64_t a = 0;
    uint32_t n = 0;
    int64_t ns = -1;
};

constexpr int MAX_DEPTH = 256;

struct Reader {
    const uint8_t *p, *end, *base;
    std::vector<Val> nodes;
    std::vector<uint32_t> kids;
    std::string pool;
    std::vector<uint32_t> stk;    // elements of the collections being read (one stack for all)
    std::vector<uint32_t> cache;  // priority cache: node ids
    struct SType { int64_t tag; int64_t n; };
    std::vector<SType> stypes;  // struct cache
    std::string err;
    size_t err_off = 0;
    int depth = 0;

    bool fail(const std::string &m) {
        if (err.empty()) { err = m; err_off = (size_t)(p - base); }
        return false;
    }
    bool byte(uint8_t &b) {
        if (p >= end) return fail("unexpected end of input");
        b = *p++;
        return true;
    }
    bool raw(uint64_t &v, int n) {  // big-endian
        if (end - p < n) return fail("unexpected end of input");
        v = 0;
        for (int k = 0; k < n; ++k) v = (v << 8) | *p++;
        return true;
    }
    uint32_t node(const Val &v) {
        nodes.push_back(v);
        return (uint32_t)(nodes.size() - 1);
    }
    // An integer whose code byte is already read.
    bool int_of(uint8_t c, int64_t &v) {
        uint64_t r;
        if (c <= 0x3F) { v = c; return true; }
        if (c == 0xFF) { v = -1; return true; }
        if (c >= 0x40 && c < 0x60) { if (!raw(r, 1)) return false; v = (int64_t)(((int64_t)c - 0x50) * 256) | (int64_t)r; return true; }
        if (c >= 0x60 && c < 0x70) { if (!raw(r, 2)) return false; v = (int64_t)(((int64_t)c - 0x68) * 65536) | (int64_t)r; return true; }
        if (c >= 0x70 && c < 0x74) { if (!raw(r, 3)) return false; v = (int64_t)(((int64_t)c - 0x72) * (1ll << 24)) | (int64_t)r; return true; }
        if (c >= 0x74 && c < 0x78) { if (!raw(r, 4)) return false; v = (int64_t)(((int64_t)c - 0x76) * (1ll << 32)) | (int64_t)r; return true; }
        if (c >= 0x78 && c < 0x7C) { if (!raw(r, 5)) return false; v = (int64_t)(((int64_t)c - 0x7A) * (1ll << 40)) | (int64_t)r; return true; }
        if (c >= 0x7C && c < 0x80) { if (!raw(r, 6)) return false; v = (int64_t)(((int64_t)c - 0x7E) * (1ll << 48)) | (int64_t)r; return true; }
        if (c == INT) { if (!raw(r, 8)) return false; v = (int64_t)r; return true; }
        return fail("expected an integer");
    }
    bool read_int(int64_t &v) {
        uint8_t c;
        return byte(c) && int_of(c, v);
    }
    bool count(int64_t &n) {
        if (!read_int(n)) return false;
        if (n < 0 || n > end - p) return fail("bad length");  // every element takes a byte at least
        return true;
    }
    bool bytes_into(bool keep, int64_t n) {
        if (n < 0 || end - p < n) return fail("unexpected end of input");
        if (keep) pool.append((const char *)p, (size_t)n);
        p += n;
        return true;
    }
    // Chunked strings / bytes: CHUNK len bytes ... then a final packed or full form.
    // String bytes go to the pool; bytes values are skipped.
    bool chunks(uint8_t c, bool str) {
        const uint8_t packed0 = str ? STRING_PACKED_LENGTH_START : BYTES_PACKED_LENGTH_START;
        const uint8_t chunk = str ? STRING_CHUNK : BYTES_CHUNK, full = str ? STRING : BYTES;
        for (;;) {
            int64_t n;
            if (c >= packed0 && c < packed0 + 8) return bytes_into(str, c - packed0);
            if (c != chunk && c != full) return fail(str ? "bad string chunk" : "bad bytes chunk");
            if (!read_int(n) || !bytes_into(str, n)) return false;
            if (c == full) return true;
            if (!byte(c)) return false;
        }
    }
    bool string_node(uint8_t c, uint8_t kind, uint32_t &out) {
        Val v;
        v.kind = kind;
        v.a = pool.size();
        if (!chunks(c, true)) return false;
        v.n = (uint32_t)(pool.size() - v.a);
        out = node(v);
        return true;
    }
    bool list_items(int64_t n, bool until_end, bool open) {
        for (int64_t k = 0; until_end || k < n; ++k) {
            if (until_end) {
                if (p >= end) {
                    if (open) return true;
                    return fail("unterminated list");
                }
                if (*p == END_COLLECTION) { ++p; return true; }
                // an open list may run into the file's footer (it ends there;
                // the footer is left for the top level, which stops reading)
                if (open && *p == FOOTER) return true;
            }
            uint32_t x;
            if (!value(x)) return false;
            stk.push_back(x);
        }
        return true;
    }
    // A collection of the elements stacked since `mark`.
    uint32_t coll(uint8_t kind, size_t mark, int64_t tag = -1) {
        Val v;
        v.kind = kind;
        v.a = kids.size();
        v.n = (uint32_t)(stk.size() - mark);
        v.ns = tag;
        kids.insert(kids.end(), stk.begin() + (std::ptrdiff_t)mark, stk.end());
        stk.resize(mark);
        return node(v);
    }
    // A list object (what MAP / SET / OBJECT_ARRAY wrap).
    bool list() {
        uint8_t c;
        if (!byte(c)) return false;
        int64_t n;
        if (c >= LIST_PACKED_LENGTH_START && c < LIST_PACKED_LENGTH_START + 8) return list_items(c - LIST_PACKED_LENGTH_START, false, false);
        if (c == LIST) return count(n) && list_items(n, false, false);
        if (c == BEGIN_CLOSED_LIST) return list_items(0, true, false);
        if (c == BEGIN_OPEN_LIST) return list_items(0, true, true);
        --p;
        uint32_t x;  // any other value in that place (a cached list): use its elements
        if (!value(x)) return false;
        const Val &v = nodes[x];
        if (v.kind != V_LIST) return fail("expected a list");
        stk.insert(stk.end(), kids.begin() + (std::ptrdiff_t)v.a, kids.begin() + (std::ptrdiff_t)(v.a + v.n));
        return true;
    }
    bool value(uint32_t &out) {
        if (++depth > MAX_DEPTH) return fail("nesting too deep");
        const bool ok = value1(out);
        --depth;
        return ok;
    }
    bool value1(uint32_t &out) {
        uint8_t c;
        if (!byte(c)) return false;
        Val v;
        uint64_t r;
        int64_t n;
        const size_t mark = stk.size();
        if (c <= 0x7F || c == 0xFF || c == INT) {
            v.kind = V_INT;
            if (!int_of(c, v.i)) return false;
            out = node(v);
            return true;
        }
        if (c >= PRIORITY_CACHE_PACKED_START && c < PRIORITY_CACHE_PACKED_END) return cached(c - PRIORITY_CACHE_PACKED_START, out);
        if (c >= STRUCT_CACHE_PACKED_START && c < STRUCT_CACHE_PACKED_END) return fields(c - STRUCT_CACHE_PACKED_START, out);
        if ((c >= STRING_PACKED_LENGTH_START && c < STRING_PACKED_LENGTH_START + 8) || c == STRING_CHUNK || c == STRING)
            return string_node(c, V_STR, out);
        if ((c >= BYTES_PACKED_LENGTH_START && c < BYTES_PACKED_LENGTH_START + 8) || c == BYTES_CHUNK || c == BYTES) {
            if (!chunks(c, false)) return false;
            v.kind = V_BLOB;
            out = node(v);
            return true;
        }
        if (c >= LIST_PACKED_LENGTH_START && c < LIST_PACKED_LENGTH_START + 8) {
            if (!list_items(c - LIST_PACKED_LENGTH_START, false, false)) return false;
            out = coll(V_LIST, mark);
            return true;
        }
        switch (c) {
            case LIST: if (!count(n) || !list_items(n, false, false)) return false; out = coll(V_LIST, mark); return true;
            case BEGIN_CLOSED_LIST: if (!list_items(0, true, false)) return false; out = coll(V_LIST, mark); return true;
            case BEGIN_OPEN_LIST: if (!list_items(0, true, true)) return false; out = coll(V_LIST, mark); return true;
            case MAP:
                if (!list()) return false;
                if ((stk.size() - mark) & 1) return fail("map with an odd number of forms");
                out = coll(V_MAP, mark);
                return true;
            case SET: case OBJECT_ARRAY:
                if (c == OBJECT_ARRAY) { if (!count(n) || !list_items(n, false, false)) return false; }
                else if (!list()) return false;
                out = coll(c == SET ? V_SET : V_LIST, mark);
                return true;
            case KEY: case SYM: {
                uint32_t ns, nm;
                if (!value(ns) || !value(nm)) return false;
                if (nodes[nm].kind != V_STR) return fail("keyword / symbol name is not a string");
                v = nodes[nm];
                v.kind = c == KEY ? V_KW : V_SYM;
                v.ns = nodes[ns].kind == V_STR ? (int64_t)ns : -1;
                out = node(v);
                return true;
            }
            case TRUE: case FALSE: v.kind = V_BOOL; v.i = c == TRUE; out = node(v); return true;
            case NULL_: out = 0; return true;  // the shared nil node
            case FLOAT: if (!raw(r, 4)) return false; v.kind = V_DBL; out = node(v); return true;
            case DOUBLE: if (!raw(r, 8)) return false; v.kind = V_DBL; out = node(v); return true;
            case DOUBLE_0: case DOUBLE_1: v.kind = V_DBL; out = node(v); return true;
            case INST: if (!read_int(n)) return false; v.kind = V_BLOB; v.i = n; out = node(v); return true;
            case UUID: case REGEX: case URI: case BIGINT: {
                uint32_t x;
                if (!value(x)) return false;  // bytes / string payload
                v.kind = V_BLOB;
                out = node(v);
                return true;
            }
            case BIGDEC: {
                uint32_t x, y;
                if (!value(x) || !value(y)) return false;  // unscaled bytes, scale
                v.kind = V_BLOB;
                out = node(v);
                return true;
            }
            case LONG_ARRAY: case INT_ARRAY: case BOOLEAN_ARRAY: {
                if (!count(n) || !list_items(n, false, false)) return false;
                out = coll(V_LIST, mark);
                return true;
            }
            case DOUBLE_ARRAY: case FLOAT_ARRAY: {
                if (!count(n)) return false;
                const int64_t w = c == DOUBLE_ARRAY ? 8 : 4;
                if ((end - p) / w < n) return fail("unexpected end of input");
                p += n * w;
                v.kind = V_BLOB;
                out = node(v);
                return true;
            }
            // The slot is taken BEFORE the value is read, as org.fressian's
            // readAndCacheObject does (and its writer numbers the outer value
            // first): a cached value holding cached strings gets the lower index.
            case PUT_PRIORITY_CACHE: {
                const size_t slot = cache.size();
                cache.push_back(0);
                if (!value(out)) return false;
                cache[slot] = out;
                return true;
            }
            case PRECACHE: {
                const size_t slot = cache.size();
                cache.push_back(0);
                uint32_t x;
                if (!value(x)) return false;
                cache[slot] = x;
                return value(out);
            }
            case GET_PRIORITY_CACHE: if (!read_int(n)) return false; return cached(n, out);
            case STRUCTTYPE: {
                uint32_t tag;
                if (!value(tag) || !read_int(n)) return false;
                if (nodes[tag].kind != V_STR || n < 0) return fail("bad struct type");
                stypes.push_back({(int64_t)tag, n});
                return fields((int64_t)stypes.size() - 1, out);
            }
            case STRUCT: if (!read_int(n)) return false; return fields(n, out);
            case META: {
                uint32_t m;
                return value(m) && value(out);  // metadata, then the value it annotates
            }
            case RESET_CACHES: cache.clear(); stypes.clear(); return value(out);
            // the footer follows the top-level value (which decode() stops
            // after) or ends an open list (list_items); anywhere else -- in a
            // closed or counted list, a struct's fields, as the first byte --
            // the file is malformed
            case FOOTER: return fail("unexpected footer");
            case END_COLLECTION: return fail("unexpected end of collection");
            default: return fail("unknown code 0x" + hex(c));
        }
    }
    static std::string hex(uint8_t c) {
        char b[4];
        std::snprintf(b, sizeof b, "%02X", c);
        return b;
    }
    bool cached(int64_t i, uint32_t &out) {
        if (i < 0 || (uint64_t)i >= cache.size()) return fail("priority cache index out of range");
        out = cache[(size_t)i];
        return true;
    }
    // A struct of cached type t: its fields.  Core tags come through codes, so
    // every tag here is a handler's ("map" under some writers included).
    bool fields(int64_t t, uint32_t &out) {
        if (t < 0 || (uint64_t)t >= stypes.size()) return fail("struct cache index out of range");
        const SType st = stypes[(size_t)t];
        const size_t mark = stk.size();
        if (!list_items(st.n, false, false)) return false;
        const std::string_view tag = str(st.tag);
        if ((tag == "map" || tag == "set" || tag == "vec" || tag == "list") && stk.size() - mark == 1 &&
            nodes[stk[mark]].kind == V_LIST) {
            const Val l = nodes[stk[mark]];  // a collection handler writing its elements as one list field
            if (tag == "map" && (l.n & 1)) return fail("map with an odd number of forms");
            stk.resize(mark);
            Val v = l;
            v.kind = tag == "map" ? V_MAP : tag == "set" ? V_SET : V_LIST;
            out = node(v);  // the same elements, read as that collection
            return true;
        }
        out = coll(V_TAGGED, mark, st.tag);
        return true;
    }
    std::string_view str(int64_t id) const {
        const Val &v = nodes[(size_t)id];
        return std::string_view(pool.data() + v.a, v.n);
    }
    bool is_kw(uint32_t id, const char *name) const {
        const Val &v = nodes[id];
        return v.kind == V_KW && v.ns < 0 && str(id) == name;
    }
    // A sequence view: lists, sets, one-list-field structs, or a struct's fields.
    bool seq(uint32_t id, const uint32_t *&b, uint32_t &n) const {
        const Val &v = nodes[id];
        if (v.kind == V_TAGGED && v.n == 1 && nodes[kids[v.a]].kind == V_LIST) return seq(kids[v.a], b, n);
        if (v.kind != V_LIST && v.kind != V_TAGGED) return false;
        b = kids.data() + v.a;
        n = v.n;
        return true;
    }
};

struct Op {
    uint8_t type = 255, f = LC_F_OTHER;
    int8_t nem = -1;
    int64_t process = LC_NO_PROCESS, index = -1;
    int64_t value = -1;  // node id
};

bool scal(const Reader &r, uint32_t id, int64_t &out) {
    const Val &v = r.nodes[id];
    if (v.kind == V_NIL) { out = LC_NIL; return true; }
    if (v.kind == V_INT && v.i != LC_NIL) { out = v.i; return true; }
    return false;
}

bool register_value(const Reader &r, uint8_t f, uint32_t id, int64_t &v0, int64_t &v1) {
    if (f == LC_F_ACQUIRE || f == LC_F_RELEASE) return true;
    if (f == LC_F_CAS) {
        const uint32_t *e;
        uint32_t n;
        if (r.nodes[id].kind == V_NIL) return true;
        return r.seq(id, e, n) && n == 2 && scal(r, e[0], v0) && scal(r, e[1], v1);
    }
    return scal(r, id, v0);
}

bool read_op(Reader &r, uint32_t id, Op &op, std::string &why) {
    const Val &m = r.nodes[id];
    if (m.kind != V_MAP) { why = "expected an op map"; return false; }
    for (uint32_t k = 0; k < m.n; k += 2) {
        const uint32_t key = r.kids[m.a + k], val = r.kids[m.a + k + 1];
        const Val &vv = r.nodes[val];
        if (r.is_kw(key, "type")) {
            const std::string_view t = vv.kind == V_KW ? r.str(val) : std::string_view();
            if (t == "invoke") op.type = LC_INVOKE;
            else if (t == "ok") op.type = LC_OK_T;
            else if (t == "fail") op.type = LC_FAIL;
            else if (t == "info") op.type = LC_INFO;
            else { why = vv.kind == V_KW ? "unknown :type :" + std::string(t) : ":type is not a keyword"; return false; }
        } else if (r.is_kw(key, "f")) {
            op.f = LC_F_OTHER;
            op.nem = -1;
            if (vv.kind == V_KW) {
                const std::string_view t = r.str(val);
                if (t == "read") op.f = LC_F_READ;
                else if (t == "write") op.f = LC_F_WRITE;
                else if (t == "cas") op.f = LC_F_CAS;
                else if (t == "acquire") op.f = LC_F_ACQUIRE;
                else if (t == "release") op.f = LC_F_RELEASE;
                else if (t == "start") op.nem = 1;
                else if (t == "stop") op.nem = 0;
            }
        } else if (r.is_kw(key, "process")) {
            op.process = vv.kind == V_INT ? vv.i : LC_NO_PROCESS;
        } else if (r.is_kw(key, "index")) {
            op.index = vv.kind == V_INT ? vv.i : -1;
        } else if (r.is_kw(key, "value")) {
            op.value = val;
        }
    }
    if (op.type == 255) { why = "op map without :type"; return false; }
    return true;
}

int decode(const uint8_t *buf, int64_t len, lc_hist **out) {
    Reader r{buf, buf + len, buf};
    r.nodes.reserve((size_t)len / 4 + 16);
    r.kids.reserve((size_t)len / 4 + 16);
    r.nodes.push_back(Val{});  // node 0: nil
    uint32_t top;
    if (len == 0) return lc::fail(LC_E_PARSE, "lc_fressian: empty input");
    if (!r.value(top)) return lc::fail(LC_E_PARSE, "lc_fressian: byte %zu: %s", r.err_off, r.err.c_str());
    // the history: the test map's :history, or a top-level list of op maps
    int64_t hist = -1;
    if (r.nodes[top].kind == V_MAP) {
        const Val &m = r.nodes[top];
        for (uint32_t k = 0; k < m.n; k += 2)
            if (r.is_kw(r.kids[m.a + k], "history")) hist = r.kids[m.a + k + 1];
        if (hist < 0) return lc::fail(LC_E_PARSE, "lc_fressian: the test map has no :history");
    } else {
        hist = top;
    }
    const uint32_t *ops;
    uint32_t n;
    if (!r.seq((uint32_t)hist, ops, n))
        return lc::fail(LC_E_PARSE, "lc_fressian: the history is not a list of op maps");
    std::vector<Op> rows(n);
    bool indep = false, all_tuples = true;
    for (uint32_t i = 0; i < n; ++i) {
        std::string why;
        if (!read_op(r, ops[i], rows[i], why)) return lc::fail(LC_E_PARSE, "lc_fressian: op %u: %s", i, why.c_str());
        if (rows[i].f != LC_F_OTHER) {
            const uint32_t *e;
            uint32_t m = 0;
            const bool tup = rows[i].value >= 0 && r.seq((uint32_t)rows[i].value, e, m) && m == 2;
            indep = true;
            all_tuples &= tup;
        }
    }
    indep &= all_tuples;
    lc_hist *h = new (std::nothrow) lc_hist();
    if (!h) return lc::fail(LC_E_NOMEM, "lc_fressian: out of memory");
    h->reserve(n);
    for (uint32_t i = 0; i < n; ++i) {
        const Op &o = rows[i];
        int64_t key = LC_NO_KEY, v0 = LC_NIL, v1 = LC_NIL;
        if (o.f == LC_F_OTHER) {
            if (o.nem >= 0) v0 = o.nem;
        } else {
            uint32_t val = o.value >= 0 ? (uint32_t)o.value : 0;  // a missing :value reads as nil
            if (indep) {
                const uint32_t *e = nullptr;
                uint32_t m = 0;
                if (!r.seq(val, e, m) || m != 2) { delete h; return lc::fail(LC_E_UNSUPPORTED, "lc_fressian: op %u: not a [k v] tuple", i); }
                const uint32_t e0 = e[0], e1 = e[1];
                if (!scal(r, e0, key) || key == LC_NIL) { delete h; return lc::fail(LC_E_UNSUPPORTED, "lc_fressian: op %u: tuple key is not an integer", i); }
                val = e1;
            }
            if (!register_value(r, o.f, val, v0, v1)) {
                delete h;
                return lc::fail(LC_E_UNSUPPORTED, "lc_fressian: op %u: value is not an integer, nil or [old new]", i);
            }
        }
        h->push(o.type, o.f, o.process, key, v0, v1, o.index);
    }
    *out = h;
    return LC_OK;
}

// ---- writer ----------------------------------------------------------------

struct Writer {
    std::string o;
    std::vector<std::string> cache;  // strings put in the priority cache, by index

    void code(uint8_t c) { o.push_back((char)c); }
    void be(uint64_t v, int n) {
        for (int k = n - 1; k >= 0; --k) o.push_back((char)(uint8_t)(v >> (8 * k)));
    }
    // The shortest of Fressian's packed int forms.
    void int_(int64_t v) {
        auto fits = [&](int bits) { return v >= -(1ll << (bits - 1)) && v < (1ll << (bits - 1)); };
        if (v >= -1 && v <= 63) code(v < 0 ? 0xFF : (uint8_t)v);
        else if (fits(13)) { code((uint8_t)(0x50 + (v >> 8))); be((uint64_t)v, 1); }
        else if (fits(20)) { code((uint8_t)(0x68 + (v >> 16))); be((uint64_t)v, 2); }
        else if (fits(26)) { code((uint8_t)(0x72 + (v >> 24))); be((uint64_t)v, 3); }
        else if (fits(34)) { code((uint8_t)(0x76 + (v >> 32))); be((uint64_t)v, 4); }
        else if (fits(42)) { code((uint8_t)(0x7A + (v >> 40))); be((uint64_t)v, 5); }
        else if (fits(50)) { code((uint8_t)(0x7E + (v >> 48))); be((uint64_t)v, 6); }
        else { code(INT); be((uint64_t)v, 8); }
    }
    void string(std::string_view s) {
        if (s.size() < 8) code((uint8_t)(STRING_PACKED_LENGTH_START + s.size()));
        else { code(STRING); int_((int64_t)s.size()); }
        o.append(s.data(), s.size());
    }
    void cached_string(std::string_view s) {
        for (size_t i = 0; i < cache.size(); ++i) {
            if (cache[i] == s) {
                if (i < 32) code((uint8_t)(PRIORITY_CACHE_PACKED_START + i));
                else { code(GET_PRIORITY_CACHE); int_((int64_t)i); }
                return;
            }
        }
        code(PUT_PRIORITY_CACHE);
        string(s);
        cache.emplace_back(s);
    }
    void keyword(std::string_view name) {
        code(KEY);
        code(NULL_);
        cached_string(name);
    }
    void scalar(int64_t v) {
        if (v == LC_NIL) code(NULL_);
        else int_(v);
    }
    void list_header(size_t n) {
        if (n < 8) code((uint8_t)(LIST_PACKED_LENGTH_START + n));
        else { code(LIST); int_((int64_t)n); }
    }
};

}  // namespace

extern "C" int lc_fressian_parse(const uint8_t *buf, int64_t len, lc_hist **out) {
    if (!buf || !out || len < 0) return lc::fail(LC_E_INVALID, "lc_fressian_parse: null argument");
    try {
        return decode(buf, len, out);
    } catch (const std::bad_alloc &) {
        return lc::fail(LC_E_NOMEM, "lc_fressian: out of memory");
    }
}

extern "C" int lc_fressian_read(const char *path, lc_hist **out) {
    if (!path || !out) return lc::fail(LC_E_INVALID, "lc_fressian_read: null argument");
    FILE *f = std::fopen(path, "rb");
    if (!f) return lc::fail(LC_E_IO, "lc_fressian_read: cannot open %s", path);
    std::string s;
    try {
        char buf[1 << 16];
        size_t r;
        while ((r = std::fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, r);
    } catch (const std::bad_alloc &) {
        std::fclose(f);
        return lc::fail(LC_E_NOMEM, "lc_fressian_read: out of memory");
    }
    std::fclose(f);
    return lc_fressian_parse((const uint8_t *)s.data(), (int64_t)s.size(), out);
}

// A test map {:name "lincheck", :history [op ...]} in the encoding Jepsen's
// writer produces for op maps: keywords with cached names, packed ints,
// [k v] tuples and [old new] cas values as lists.
extern "C" int lc_fressian_write(const char *path, const lc_history *h) {
    if (!path || !h || h->n < 0) return lc::fail(LC_E_INVALID, "lc_fressian_write: null argument");
    static const char *types[] = {"invoke", "ok", "fail", "info"};
    static const char *fs[] = {"read", "write", "cas", "", "acquire", "release"};
    Writer w;
    try {
        w.code(MAP);
        w.list_header(4);
        w.keyword("name");
        w.string("lincheck");
        w.keyword("history");
        w.list_header((size_t)h->n);
        for (int64_t r = 0; r < h->n; ++r) {
            if (h->type[r] > LC_INFO || h->f[r] > LC_F_RELEASE)
                return lc::fail(LC_E_INVALID, "lc_fressian_write: bad row %lld", (long long)r);
            w.code(MAP);
            w.list_header(10);
            w.keyword("type");
            w.keyword(types[h->type[r]]);
            w.keyword("f");
            const bool nem = h->f[r] == LC_F_OTHER;
            w.keyword(nem ? (h->v0[r] == 1 ? "start" : h->v0[r] == 0 ? "stop" : "nemesis") : fs[h->f[r]]);
            w.keyword("value");
            const bool tuple = !nem && h->key[r] != LC_NO_KEY;
            if (tuple) { w.list_header(2); w.int_(h->key[r]); }
            if (nem || h->f[r] == LC_F_ACQUIRE || h->f[r] == LC_F_RELEASE) {
                w.code(NULL_);
            } else if (h->f[r] == LC_F_CAS) {
                if (h->v0[r] == LC_NIL && h->v1[r] == LC_NIL && h->type[r] == LC_INVOKE) w.code(NULL_);
                else { w.list_header(2); w.scalar(h->v0[r]); w.scalar(h->v1[r]); }
            } else {
                w.scalar(h->v0[r]);
            }
            w.keyword("process");
            if (h->process[r] == LC_NO_PROCESS) w.keyword("nemesis");
            else w.int_(h->process[r]);
            w.keyword("index");
            w.int_(h->index && h->index[r] >= 0 ? h->index[r] : r);
        }
    } catch (const std::bad_alloc &) {
        return lc::fail(LC_E_NOMEM, "lc_fressian_write: out of memory");
    }
    FILE *f = std::fopen(path, "wb");
    if (!f) return lc::fail(LC_E_IO, "lc_fressian_write: cannot open %s", path);
    const bool ok = std::fwrite(w.o.data(), 1, w.o.size(), f) == w.o.size();
    if (std::fclose(f) != 0 || !ok) return lc::fail(LC_E_IO, "lc_fressian_write: write failed");
    return LC_OK;
}
