// lc_pack: Jepsen history -> packed per-key event streams for the device search.
//
// Host-side restatement of the steps between the raw history and
// knossos.linear's search loop:
//
//   A2 jepsen.independent/checker (etcdemo.clj:115): history-keys + subhistory.
//      Ops whose :value is a tuple [k v] go to key k, unwrapped to v; ops with a
//      non-tuple value (the nemesis :info :start/:stop of etcdemo.clj:138-143)
//      belong to every key's sub-history.
//   A3 knossos.history/complete + without-failures: an :invoke is paired with
//      the next completion of the same :process.  :ok -> the invocation takes
//      (or invocation-value completion-value) (a read learns what it read);
//      :fail -> invocation and completion are dropped; :info, or no completion
//      at all -> the op stays pending (callable) forever.  A second :invoke by a
//      process with an op outstanding leaves the first pending forever (the
//      pending index is overwritten, as complete's assoc! does).  A completion
//      with no outstanding invocation is an error (complete asserts).
//   A9 errors are per key: independent/checker wraps each key's check in
//      check-safe (etcdemo.clj:115), so a key whose sub-history fails
//      complete's assertion or holds an op the model cannot step is reported
//      :unknown with the error while every other key is checked.  Such a key
//      keeps its place in the batch with no events and key_error set.
//   A4/A5 knossos.model/cas-register + knossos.model.memo: every surviving op
//      becomes a transition descriptor over interned register states (state 0
//      = nil, the initial value of (model/cas-register), etcdemo.clj:117).
//      (model/multi-register): memo proper -- the maps
//      reachable from the initial one under the key's distinct :txn ops are
//      numbered breadth-first, and each op becomes a row of next-state ids
//      (lc_batch.table).
//
// The pending-window slot of each op (lowest free slot at invoke, released at
// :ok) is assigned here too: it is config-independent, so every device config
// can name linearized ops by slot bit.

#include <algorithm>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <unordered_map>

#include "common.hpp"
#include "packed.hpp"

namespace {

// Ops a model can step (knossos.model: cas-register, register, mutex,
// multi-register).
inline bool is_client_f(uint8_t f, int model) {
    if (model == LC_MODEL_MULTI_REGISTER) return f == LC_F_TXN;
    if (model == LC_MODEL_MUTEX) return f == LC_F_ACQUIRE || f == LC_F_RELEASE;
    if (model == LC_MODEL_REGISTER) return f == LC_F_READ || f == LC_F_WRITE;
    return f == LC_F_READ || f == LC_F_WRITE || f == LC_F_CAS;
}

// Small process -> outstanding-op map; linear scan while small, hash beyond.
struct ProcMap {
    std::vector<std::pair<int64_t, int32_t>> small;
    std::unordered_map<int64_t, int32_t> big;
    bool use_big = false;
    int32_t *find(int64_t p) {
        if (use_big) { auto it = big.find(p); return it == big.end() ? nullptr : &it->second; }
        for (auto &e : small) if (e.first == p) return &e.second;
        return nullptr;
    }
    void set(int64_t p, int32_t op) {
        if (int32_t *x = find(p)) { *x = op; return; }
        if (!use_big && small.size() >= 64) {
            use_big = true;
            for (auto &e : small) big.emplace(e.first, e.second);
            small.clear();
        }
        if (use_big) big.emplace(p, op); else small.emplace_back(p, op);
    }
    void erase(int64_t p) {
        if (use_big) { big.erase(p); return; }
        for (size_t i = 0; i < small.size(); ++i)
            if (small[i].first == p) { small[i] = small.back(); small.pop_back(); return; }
    }
};

// One surviving client op of a key, before interning.
struct KOp {
    int64_t row_inv, row_ret;  // row_ret = -1: never returns
    uint8_t f, fate;           // fate: 0 pending-forever, 1 ok, 2 failed
    int64_t v0, v1;
    int64_t mrow;              // :txn: the row whose micro-ops the op carries
};

// Micro-op range of row r of a history ([m0, m1) triples; empty if none).
inline void mop_range(const lc_history &h, int64_t r, int64_t &m0, int64_t &m1) {
    m0 = m1 = 0;
    if (h.mop_off && h.mop) { m0 = h.mop_off[r]; m1 = h.mop_off[r + 1]; }
}

struct KeyOut {
    std::vector<uint32_t> ev;     // event words, trans field = local op index for now
    std::vector<int64_t> ev_row;
    std::vector<int32_t> ev_op;   // op index per invoke event (-1 for ok)
    std::vector<KOp> ops;
    int width = 0;
    int err = 0;
    std::string msg;
};

// A3 pairing of one key (rows in history order): `ops` in invoke order and
// `row_op[i]` = the op invoked or completed :ok/:fail at row i (-1: none).
// false (err/msg set, ops cleared) on a sub-history complete rejects.
bool pair_rows(const lc_history &h, const int64_t *rows, int64_t nrows, int model, std::vector<KOp> &ops,
               std::vector<int32_t> &row_op, int &err, std::string &msg) {
    // process -> outstanding op: a direct table over the key's process range
    // when it is narrow (Jepsen numbers processes densely), else ProcMap
    ProcMap pm;
    int64_t pmin = INT64_MAX, pmax = INT64_MIN;
    for (int64_t i = 0; i < nrows; ++i) {
        const int64_t p = h.process[rows[i]];
        pmin = std::min(pmin, p);
        pmax = std::max(pmax, p);
    }
    // (differences in unsigned arithmetic: process ids span all of int64)
    auto off = [&](int64_t p) { return (size_t)((uint64_t)p - (uint64_t)pmin); };
    const bool direct = nrows > 0 && (uint64_t)pmax - (uint64_t)pmin < 4096;
    static thread_local std::vector<int32_t> dmap;
    if (direct) dmap.assign(off(pmax) + 1, -1);
    auto pfind = [&](int64_t p) -> int32_t * {
        if (!direct) return pm.find(p);
        int32_t &x = dmap[off(p)];
        return x >= 0 ? &x : nullptr;
    };
    ops.clear();
    ops.reserve((size_t)nrows / 2 + 1);
    row_op.assign((size_t)nrows, -1);
    for (int64_t i = 0; i < nrows; ++i) {
        int64_t r = rows[i];
        uint8_t t = h.type[r];
        int64_t p = h.process[r];
        if (t == LC_INVOKE) {
            if (!is_client_f(h.f[r], model)) {
                static const char *names[] = {"cas-register", "register", "mutex", "multi-register"};
                err = LC_E_UNSUPPORTED;
                msg = "row " + std::to_string(r) + ": " + names[model] + " cannot step this :f";
                ops.clear();
                return false;
            }
            int32_t id = (int32_t)ops.size();
            ops.push_back({r, -1, h.f[r], 0, h.v0[r], h.v1[r], r});
            if (direct) dmap[off(p)] = id;
            else pm.set(p, id);
            row_op[(size_t)i] = id;
        } else if (t == LC_OK_T || t == LC_FAIL) {
            int32_t *pid = pfind(p);
            if (!pid) {
                err = LC_E_INVALID;
                msg = "row " + std::to_string(r) + ": process completed an operation without a prior invocation";
                ops.clear();
                return false;
            }
            KOp &op = ops[(size_t)*pid];
            if (t == LC_OK_T) {
                op.fate = 1;
                op.row_ret = r;
                // (or (:value invocation) (:value completion))
                if (op.f == LC_F_TXN) {
                    // a :txn takes its completion's micro-ops when it has
                    // some: the reads learn what they read
                    int64_t m0, m1;
                    mop_range(h, r, m0, m1);
                    if (m1 > m0) op.mrow = r;
                } else if (op.f == LC_F_CAS) {
                    if (op.v0 == LC_NIL && op.v1 == LC_NIL) { op.v0 = h.v0[r]; op.v1 = h.v1[r]; }
                } else if (op.v0 == LC_NIL) {
                    op.v0 = h.v0[r];
                }
                row_op[(size_t)i] = *pid;
            } else {
                op.fate = 2;
            }
            if (direct) dmap[off(p)] = -1;
            else pm.erase(p);
        } else if (t == LC_INFO) {  // crashed: pending forever
            if (direct) dmap[off(p)] = -1;
            else if (pm.find(p)) pm.erase(p);
        }
    }
    return true;
}

// Events of a paired key in row order, failed pairs dropped, each invoke
// given the lowest free window slot (released at its :ok): ev[j] = slot << 24
// | op id (invoke) or LC_EV_OK_BIT | slot << 24, ev_row[j] its row, ev_op[j]
// (may be null) the op id (-1 for :ok).  Returns the event count (<= nrows).
int64_t emit_events(const int64_t *rows, int64_t nrows, const std::vector<KOp> &ops,
                    const std::vector<int32_t> &row_op, uint32_t *ev, int64_t *ev_row, int32_t *ev_op, int &width) {
    uint64_t freemask[2] = {~0ull, ~0ull};
    static thread_local std::vector<int8_t> slot_of;
    slot_of.assign(ops.size(), -1);
    int64_t ne = 0;
    int maxslot = -1;
    for (int64_t i = 0; i < nrows; ++i) {
        int32_t id = row_op[(size_t)i];
        if (id < 0) continue;
        const KOp &op = ops[(size_t)id];
        if (op.fate == 2) continue;  // without-failures
        int64_t r = rows[i];
        if (op.row_inv == r) {  // the op's invoke
            int s;
            if (freemask[0]) s = __builtin_ctzll(freemask[0]);
            else if (freemask[1]) s = 64 + __builtin_ctzll(freemask[1]);
            else s = 128;
            if (s < 127) freemask[s >> 6] &= ~(1ull << (s & 63));
            int enc = s < 127 ? s : 127;  // >= 127 cannot be encoded; the search stops earlier
            slot_of[(size_t)id] = (int8_t)enc;
            maxslot = std::max(maxslot, s);
            ev[ne] = ((uint32_t)enc << 24) | (uint32_t)id;
            if (ev_op) ev_op[ne] = id;
        } else {
            int s = slot_of[(size_t)id];
            if (s < 127) freemask[s >> 6] |= 1ull << (s & 63);
            ev[ne] = LC_EV_OK_BIT | ((uint32_t)s << 24);
            if (ev_op) ev_op[ne] = -1;
        }
        ev_row[ne++] = r;
    }
    width = std::min(maxslot + 1, 255);
    return ne;
}

// Pairing + event emission for one key into a KeyOut (multi-register).
void pack_key(const lc_history &h, const int64_t *rows, int64_t nrows, int model, KeyOut &out) {
    static thread_local std::vector<int32_t> row_op;
    if (!pair_rows(h, rows, nrows, model, out.ops, row_op, out.err, out.msg)) return;
    out.ev.resize((size_t)nrows);
    out.ev_row.resize((size_t)nrows);
    out.ev_op.resize((size_t)nrows);
    const int64_t ne = emit_events(rows, nrows, out.ops, row_op, out.ev.data(), out.ev_row.data(), out.ev_op.data(),
                                   out.width);
    out.ev.resize((size_t)ne);
    out.ev_row.resize((size_t)ne);
    out.ev_op.resize((size_t)ne);
}

// lc_pack's per-event staging (register models), reused across calls.
struct Staging {
    lc::uninit_vector<uint32_t> ev;
    lc::uninit_vector<int64_t> row;
};
Staging g_staging;
std::mutex g_staging_mu;

// (model/multi-register) memo of one key: registers, reachable maps, table.
constexpr int64_t ABSENT = LC_NIL + 1;  // a register the map lacks (reserved value)

struct MrKey {
    std::vector<int64_t> regs;      // register ids, ascending
    std::vector<int64_t> states;    // S x R values (ABSENT / LC_NIL / integer)
    std::vector<uint32_t> tid;      // per op of the key: its :txn id
    std::vector<uint16_t> table;    // T x S next-state ids
    uint32_t S = 0, T = 0;
    bool too_many = false;          // > LC_WIDE_MAX_STATES maps
    int err = 0;
    std::string msg;
};

struct VecHash {
    size_t operator()(const std::vector<int64_t> &v) const {
        uint64_t x = 0x9E3779B97F4A7C15ull ^ v.size();
        for (int64_t e : v) { x ^= (uint64_t)e + 0x9E3779B97F4A7C15ull + (x << 6) + (x >> 2); }
        return (size_t)x;
    }
};

void memo_multi_register(const lc_history &h, const KeyOut &o, const int64_t *init, int32_t n_init, MrKey &mk) {
    // distinct :txn values (flattened triples, register ids as given)
    std::unordered_map<std::vector<int64_t>, uint32_t, VecHash> tix;
    std::vector<std::vector<int64_t>> txns;
    std::vector<int64_t> regs;
    for (int32_t i = 0; i < n_init; ++i) regs.push_back(init[2 * i]);
    mk.tid.assign(o.ops.size(), 0);
    for (size_t q = 0; q < o.ops.size(); ++q) {
        const KOp &op = o.ops[q];
        if (op.fate == 2) continue;
        int64_t m0, m1;
        mop_range(h, op.mrow, m0, m1);
        std::vector<int64_t> t;
        for (int64_t m = m0; m < m1; ++m) {
            const int64_t f = h.mop[3 * m], k = h.mop[3 * m + 1], v = h.mop[3 * m + 2];
            if ((f != LC_MOP_READ && f != LC_MOP_WRITE) || v == ABSENT) {
                mk.err = LC_E_INVALID;
                mk.msg = "row " + std::to_string(op.mrow) + ": bad :txn micro-op";
                return;
            }
            t.push_back(f); t.push_back(k); t.push_back(v);
            regs.push_back(k);
        }
        auto it = tix.find(t);
        if (it == tix.end()) {
            it = tix.emplace(t, (uint32_t)txns.size()).first;
            txns.push_back(t);
        }
        mk.tid[q] = it->second;
    }
    std::sort(regs.begin(), regs.end());
    regs.erase(std::unique(regs.begin(), regs.end()), regs.end());
    mk.regs = regs;
    const size_t R = regs.size();
    auto ridx = [&](int64_t k) { return (size_t)(std::lower_bound(regs.begin(), regs.end(), k) - regs.begin()); };
    // the txns with register indices
    std::vector<std::vector<int64_t>> tx(txns.size());
    for (size_t t = 0; t < txns.size(); ++t)
        for (size_t j = 0; j < txns[t].size(); j += 3) {
            tx[t].push_back(txns[t][j]);
            tx[t].push_back((int64_t)ridx(txns[t][j + 1]));
            tx[t].push_back(txns[t][j + 2]);
        }
    std::vector<int64_t> s0(R, ABSENT);
    for (int32_t i = 0; i < n_init; ++i) s0[ridx(init[2 * i])] = init[2 * i + 1];
    std::unordered_map<std::vector<int64_t>, uint32_t, VecHash> six;
    std::vector<std::vector<int64_t>> st{s0};
    six.emplace(s0, 0);
    // breadth-first over (state, txn); next[t][s] as the states appear
    std::vector<std::vector<uint32_t>> next(tx.size());
    std::vector<int64_t> cur;
    for (size_t s = 0; s < st.size(); ++s) {
        for (size_t t = 0; t < tx.size(); ++t) {
            cur = st[s];
            bool ok = true;
            for (size_t j = 0; j < tx[t].size() && ok; j += 3) {
                const size_t r = (size_t)tx[t][j + 1];
                const int64_t v = tx[t][j + 2];
                if (tx[t][j] == LC_MOP_READ) ok = v == LC_NIL || (cur[r] != ABSENT && cur[r] == v);
                else cur[r] = v;
            }
            uint32_t id = LC_TABLE_NONE;
            if (ok) {
                auto it = six.find(cur);
                if (it == six.end()) {
                    if (st.size() >= (size_t)LC_WIDE_MAX_STATES) { mk.too_many = true; break; }
                    it = six.emplace(cur, (uint32_t)st.size()).first;
                    st.push_back(cur);
                }
                id = it->second;
            }
            next[t].push_back(id);
        }
        if (mk.too_many) break;
    }
    mk.T = (uint32_t)tx.size();
    if (mk.too_many) {
        mk.S = LC_WIDE_MAX_STATES + 1;
        return;
    }
    mk.S = (uint32_t)st.size();
    mk.states.reserve(st.size() * R);
    for (auto &v : st) mk.states.insert(mk.states.end(), v.begin(), v.end());
    mk.table.reserve((size_t)mk.T * mk.S);
    for (size_t t = 0; t < tx.size(); ++t) mk.table.insert(mk.table.end(), next[t].begin(), next[t].end());
}

// A4/A5 for (model/multi-register): memo per key (in parallel), then the
// packed arrays.  Keys whose micro-ops are malformed become per-key errors.
void pack_multi_register(const lc_history &h, const int64_t *init, int32_t n_init, std::vector<KeyOut> &ko,
                         unsigned nt, lc_packed *P) {
    const int64_t K = (int64_t)ko.size();
    std::vector<MrKey> mr((size_t)K);
    {
        auto work = [&](unsigned t) {
            for (int64_t k = t; k < K; k += nt)
                if (!ko[(size_t)k].err) memo_multi_register(h, ko[(size_t)k], init, n_init, mr[(size_t)k]);
        };
        lc::run_threads(nt, work);
    }
    for (int64_t k = 0; k < K; ++k) {
        MrKey &m = mr[(size_t)k];
        KeyOut &o = ko[(size_t)k];
        if (!m.err) continue;
        if (P->key_error.empty()) {
            P->key_error.assign((size_t)K, 0);
            P->key_msg.assign((size_t)K, std::string());
        }
        P->key_error[(size_t)k] = 1;
        P->key_msg[(size_t)k] = m.msg;
        std::vector<uint32_t>().swap(o.ev);
        std::vector<int64_t>().swap(o.ev_row);
        std::vector<int32_t>().swap(o.ev_op);
        std::vector<KOp>().swap(o.ops);
        o.width = 0;
        m = MrKey{};
    }
    P->model = LC_MODEL_MULTI_REGISTER;
    P->key_states.assign((size_t)K, 0);
    P->key_width.assign((size_t)K, 0);
    P->trans_off.assign((size_t)K, 0);
    P->ev_off.assign((size_t)K + 1, 0);
    P->mr_reg_off.assign((size_t)K + 1, 0);
    P->mr_state_off.assign((size_t)K + 1, 0);
    for (int64_t k = 0; k < K; ++k) P->ev_off[(size_t)k + 1] = P->ev_off[(size_t)k] + ko[(size_t)k].ev.size();
    P->events.alloc((size_t)P->ev_off[(size_t)K], true);
    P->ev_row.resize((size_t)P->ev_off[(size_t)K]);
    for (int64_t k = 0; k < K; ++k) {
        MrKey &m = mr[(size_t)k];
        KeyOut &o = ko[(size_t)k];
        if (m.S == 0) m.S = 1;  // an error key: the initial map alone
        P->key_states[(size_t)k] = (uint16_t)std::min<uint32_t>(m.S, 65535u);
        P->key_width[(size_t)k] = (uint8_t)o.width;
        P->trans_off[(size_t)k] = (uint32_t)P->trans.size();
        const uint64_t tbase = P->table.size();
        if (tbase + m.table.size() > 0xFFFFFFFFull) throw std::length_error("table");
        for (uint32_t t = 0; t < m.T; ++t) P->trans.push_back(m.too_many ? 0u : (uint32_t)(tbase + (uint64_t)t * m.S));
        P->table.insert(P->table.end(), m.table.begin(), m.table.end());
        P->mr_regs.insert(P->mr_regs.end(), m.regs.begin(), m.regs.end());
        P->mr_reg_off[(size_t)k + 1] = P->mr_regs.size();
        P->mr_states.insert(P->mr_states.end(), m.states.begin(), m.states.end());
        P->mr_state_off[(size_t)k + 1] = P->mr_states.size();
        const uint64_t base = P->ev_off[(size_t)k];
        for (size_t j = 0; j < o.ev.size(); ++j) {
            uint32_t w = o.ev[j];
            if (!(w & LC_EV_OK_BIT)) w = (w & 0xFF000000u) | m.tid[(size_t)o.ev_op[j]];
            P->events[base + j] = w;
            P->ev_row[base + j] = o.ev_row[j];
        }
        std::vector<uint32_t>().swap(o.ev);
        std::vector<int64_t>().swap(o.ev_row);
        std::vector<int32_t>().swap(o.ev_op);
        std::vector<KOp>().swap(o.ops);
        m = MrKey{};
    }
    if (P->trans.empty()) P->trans.push_back(0);
    if (P->table.empty()) P->table.push_back(LC_TABLE_NONE);
}


// ---- register models: interning shared by both pack paths ----------------

// Keys' surviving ops, interned, in arenas (no allocation per key): per key
// the state values a write / cas can install and the distinct (f, a, b)
// triples of its invokes, both in order of first appearance (invoke
// order); number_and_describe then gives each triple its transition id.
struct Arena {
    std::vector<int64_t> vals;  // state values, key after key
    std::vector<int64_t> trip;  // triples (3 words each), key after key
    std::vector<uint32_t> tid;  // per triple: its transition id (number_and_describe)
};
struct KeySpan {                // one key's part of an arena
    uint32_t arena = 0, nv = 0, nt = 0;  // values, triples
    uint64_t v0 = 0, t0 = 0;    // first value, first triple (in triples)
};

// Per-thread interning tables, reset per key.  Small values (0 .. 14, and
// nil) -- what Jepsen register tests write -- go through direct tables
// stamped per key; others through a set / an open-addressing table of index
// + 1 kept under half full.
class Interner {
  public:
    void begin(Arena *A, int model) {
        A_ = A;
        model_ = model;
        v0_ = A->vals.size();
        t0_ = A->trip.size();
        if (dstamp_.empty()) { dstamp_.assign(8 * 16 * 16, 0); dtrip_.assign(8 * 16 * 16, 0); }
        if (++kstamp_ == 0) { std::fill(dstamp_.begin(), dstamp_.end(), 0u); kstamp_ = 1; }
        vseen_ = 0;
        seen_.clear();
        tmask_ = 255;
        tt_.assign(tmask_ + 1, 0);
        if (model == LC_MODEL_MUTEX) A->vals.push_back(1);  // state 1 = locked (state 0, "nil", = unlocked)
    }
    // this key's span (call after its last op)
    KeySpan end(uint32_t arena) const {
        KeySpan sp;
        sp.arena = arena;
        sp.v0 = v0_;
        sp.nv = (uint32_t)(A_->vals.size() - v0_);
        sp.t0 = t0_ / 3;
        sp.nt = (uint32_t)((A_->trip.size() - t0_) / 3);
        return sp;
    }
    // A surviving op (its values after complete's fill): its state value,
    // and the index of its (f, a, b) triple among the key's.
    uint32_t op(int64_t f, int64_t v0, int64_t v1) {
        if (model_ != LC_MODEL_MUTEX) {
            if (f == LC_F_WRITE) add(v0);
            if (f == LC_F_CAS) add(v1);
        }
        const int64_t a = (f == LC_F_ACQUIRE || f == LC_F_RELEASE) ? 0 : v0;
        const int64_t b = f == LC_F_CAS ? v1 : 0;
        const int64_t sa = small(a), sb = small(b);
        if (sa >= 0 && sb >= 0 && f < 8) {
            const size_t di = (size_t)f * 256 + (size_t)sa * 16 + (size_t)sb;
            if (dstamp_[di] != kstamp_) {
                dstamp_[di] = kstamp_;
                dtrip_[di] = new_trip(f, a, b);
            }
            return dtrip_[di];
        }
        const int64_t *tr = A_->trip.data() + t0_;
        size_t x = thash(f, a, b) & tmask_;
        for (;; x = (x + 1) & tmask_) {
            const uint64_t e = tt_[x];
            if (!e) {
                const uint32_t ti = new_trip(f, a, b);
                tt_[x] = ti + 1;
                if ((size_t)(ti + 1) * 2 > tmask_) {  // grow
                    tmask_ = tmask_ * 2 + 1;
                    tt_.assign(tmask_ + 1, 0);
                    const int64_t *t2 = A_->trip.data() + t0_;
                    for (uint32_t u = 0; u <= ti; ++u) {
                        size_t y = thash(t2[3 * u], t2[3 * u + 1], t2[3 * u + 2]) & tmask_;
                        while (tt_[y]) y = (y + 1) & tmask_;
                        tt_[y] = u + 1;
                    }
                }
                return ti;
            }
            const uint32_t u = (uint32_t)e - 1;
            if (tr[3 * u] == f && tr[3 * u + 1] == a && tr[3 * u + 2] == b) return u;
        }
    }

  private:
    static constexpr int64_t SMALL = 15;  // values 0 .. 14, plus nil as 15
    static int64_t small(int64_t v) { return v == LC_NIL ? SMALL : (v >= 0 && v < SMALL ? v : -1); }
    static size_t thash(int64_t f, int64_t a, int64_t b) {
        uint64_t x = (uint64_t)f * 0x9E3779B97F4A7C15ull ^ (uint64_t)a * 0xC2B2AE3D27D4EB4Full ^
                     (uint64_t)b * 0x165667B19E3779F9ull;
        return (size_t)(x ^ (x >> 29));
    }
    void add(int64_t v) {
        if (v == LC_NIL) return;
        std::vector<int64_t> &vals = A_->vals;
        const int64_t sv = small(v);
        if (sv >= 0) {
            if (vseen_ >> sv & 1u) return;
            vseen_ |= 1u << sv;
            vals.push_back(v);
            if (!seen_.empty()) seen_.emplace(v, 0);
            return;
        }
        if (vals.size() - v0_ < 16) {
            if (std::find(vals.begin() + (std::ptrdiff_t)v0_, vals.end(), v) == vals.end()) vals.push_back(v);
            return;
        }
        if (seen_.empty())
            for (size_t i = v0_; i < vals.size(); ++i) seen_.emplace(vals[i], 0);
        if (seen_.emplace(v, 0).second) vals.push_back(v);
    }
    uint32_t new_trip(int64_t f, int64_t a, int64_t b) {
        const uint32_t ti = (uint32_t)((A_->trip.size() - t0_) / 3);
        A_->trip.push_back(f);
        A_->trip.push_back(a);
        A_->trip.push_back(b);
        return ti;
    }
    Arena *A_ = nullptr;
    size_t v0_ = 0, t0_ = 0;
    int model_ = 0;
    std::vector<uint32_t> dstamp_, dtrip_;  // (f, a, b) small -> stamp, index
    uint32_t kstamp_ = 0;
    uint32_t vseen_ = 0;  // small state values seen
    std::unordered_map<int64_t, char> seen_;
    std::vector<uint64_t> tt_;
    size_t tmask_ = 255;
};

// Tasks over the pack pool (or threads of its own when another pack holds
// the pool): fn(i) for every i in [0, n_tasks), claimed dynamically.
struct Par {
    lc::HostPool *pool = nullptr;
    unsigned nt = 1;
    template <class F>
    void run(uint64_t n_tasks, const F &fn) const {
        if (n_tasks == 0) return;
        std::atomic<uint64_t> next{0};
        // A task that throws (std::bad_alloc in a task's allocations) stops
        // the claiming of tasks; every thread is joined and the first
        // exception is rethrown here, on the caller.
        std::mutex em;
        std::exception_ptr ex;
        auto body = [&](unsigned) {
            try {
                for (uint64_t i; (i = next.fetch_add(1, std::memory_order_relaxed)) < n_tasks;) fn(i);
            } catch (...) {
                next.store(n_tasks, std::memory_order_relaxed);
                std::lock_guard<std::mutex> g(em);
                if (!ex) ex = std::current_exception();
            }
        };
        const unsigned w = (unsigned)std::min<uint64_t>(nt, n_tasks);
        if (w <= 1) {
            body(0);
        } else if (pool) {
            const std::function<void(unsigned)> f = body;
            pool->run(w, f);
        } else {
            std::vector<std::thread> th;
            for (unsigned t = 1; t < w; ++t) th.emplace_back(body, t);
            body(0);
            for (auto &x : th) x.join();
        }
        if (ex) std::rethrow_exception(ex);
    }
};

// Open-addressing map of 64-bit keys to u32, kept under half full.  Slot
// occupancy is its own byte array, so every 64-bit key -- -1 and INT64_MAX
// included -- is a key like any other (no key value doubles as "empty").
// For the interning tables lc_pack builds per batch.
class FlatMap {
  public:
    explicit FlatMap(size_t expect = 16) {
        size_t c = 32;
        while (c < 2 * expect) c <<= 1;
        k_.resize(c);
        v_.resize(c);
        used_.assign(c, 0);
    }
    // the value of key, or `none`
    uint32_t get(uint64_t key, uint32_t none) const {
        for (size_t x = hash(key) & (k_.size() - 1);; x = (x + 1) & (k_.size() - 1)) {
            if (!used_[x]) return none;
            if (k_[x] == key) return v_[x];
        }
    }
    // insert key -> val unless present; returns the value it maps to
    uint32_t put(uint64_t key, uint32_t val) {
        for (size_t x = hash(key) & (k_.size() - 1);; x = (x + 1) & (k_.size() - 1)) {
            if (!used_[x]) {
                used_[x] = 1;
                k_[x] = key;
                v_[x] = val;
                if (++n_ * 2 > k_.size()) grow();
                return val;
            }
            if (k_[x] == key) return v_[x];
        }
    }
    size_t size() const { return n_; }

  private:
    static size_t hash(uint64_t x) {
        x *= 0x9E3779B97F4A7C15ull;
        return (size_t)(x ^ (x >> 31));
    }
    void grow() {
        std::vector<uint64_t> ok;
        std::vector<uint32_t> ov;
        std::vector<uint8_t> ou;
        ok.swap(k_);
        ov.swap(v_);
        ou.swap(used_);
        k_.resize(ok.size() * 2);
        v_.resize(ok.size() * 2);
        used_.assign(ok.size() * 2, 0);
        for (size_t i = 0; i < ok.size(); ++i)
            if (ou[i])
                for (size_t x = hash(ok[i]) & (k_.size() - 1);; x = (x + 1) & (k_.size() - 1))
                    if (!used_[x]) { used_[x] = 1; k_[x] = ok[i]; v_[x] = ov[i]; break; }
    }
    std::vector<uint64_t> k_;
    std::vector<uint32_t> v_;
    std::vector<uint8_t> used_;
    size_t n_ = 0;
};

// (2) the state numbering (one shared by every key while the batch has <
// 255 values, else per key), (3) every triple's descriptor, and (4) the
// descriptors' transition ids -- in order of first appearance over the keys
// in order and each key's triples in order, the ids one serial pass over
// keys and events would give -- into each arena's `tid`.  *max_tid = the
// largest transition id a word carries.  false: more than 2^24 distinct
// operations.
bool number_and_describe(lc_packed *P, const std::vector<KeySpan> &ks, std::vector<Arena> &ar, const Par &par,
                         uint32_t *max_tid) {
    const int64_t K = (int64_t)ks.size();
    for (Arena &A : ar) A.tid.resize(A.trip.size() / 3);
    // (2) the shared numbering: values in order of first appearance over the
    // keys (a few per key)
    FlatMap gstate;
    std::vector<int64_t> gvals;
    bool shared = true;
    for (int64_t k = 0; k < K && shared; ++k) {
        const KeySpan &sp = ks[(size_t)k];
        const int64_t *v = ar[sp.arena].vals.data() + sp.v0;
        for (uint32_t i = 0; i < sp.nv; ++i) {
            const uint32_t id = (uint32_t)gvals.size() + 1;
            if (gstate.put((uint64_t)v[i], id) == id) {
                if (gvals.size() >= LC_NARROW_MAX_STATES - 1) { shared = false; break; }
                gvals.push_back(v[i]);
            }
        }
    }
    if (shared) {
        P->state_vals.assign(gvals.size() + 1, LC_NIL);
        for (size_t i = 0; i < gvals.size(); ++i) P->state_vals[i + 1] = gvals[i];
    } else {
        P->state_off.assign((size_t)K + 1, 0);
    }
    P->key_states.assign((size_t)K, 0);
    // (3) per key (contiguous blocks in parallel): each triple's descriptor.
    // Shared numbering: `tid` holds the descriptor for now, and each block
    // lists the descriptors in order of their first appearance in it, so
    // that (4) is a serial merge of short lists.  Per-key numbering: each
    // key's distinct descriptors (its transition table) and local ids.
    const uint64_t blocks = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)K, 64u * par.nt));
    std::vector<std::vector<uint32_t>> bdesc(blocks);
    std::vector<std::vector<uint32_t>> kud(shared ? 0 : (size_t)K);
    std::vector<std::vector<int64_t>> ktab(shared ? 0 : (size_t)K);
    par.run(blocks, [&](uint64_t bi) {
        FlatMap bseen;
        for (int64_t k = (int64_t)(bi * (uint64_t)K / blocks); k < (int64_t)((bi + 1) * (uint64_t)K / blocks); ++k) {
            const KeySpan &sp = ks[(size_t)k];
            Arena &A = ar[sp.arena];
            const int64_t *vals = A.vals.data() + sp.v0;
            std::unordered_map<int64_t, uint32_t> lstate;
            if (!shared) {
                for (uint32_t i = 0; i < sp.nv; ++i)
                    lstate.emplace(vals[i], lstate.size() < LC_STATE_NONE - 1 ? (uint32_t)lstate.size() + 1 : LC_STATE_NONE);
            }
            auto sid = [&](int64_t v) -> uint32_t {
                if (v == LC_NIL) return 0;
                if (shared) return gstate.get((uint64_t)v, LC_STATE_NONE);
                auto it = lstate.find(v);
                return it == lstate.end() ? LC_STATE_NONE : it->second;
            };
            P->key_states[(size_t)k] = (uint16_t)std::min<size_t>((size_t)sp.nv + 1, 65535);
            const int64_t *tr = A.trip.data() + 3 * sp.t0;
            uint32_t *tid = A.tid.data() + sp.t0;
            FlatMap local(shared ? 1 : sp.nt);
            for (uint32_t u = 0; u < sp.nt; ++u) {
                const int64_t f = tr[3 * u], a = tr[3 * u + 1], b = tr[3 * u + 2];
                uint32_t d;
                if (f == LC_F_ACQUIRE) d = LC_DESC(LC_T_CAS, 0, sid(1));  // unlocked -> locked
                else if (f == LC_F_RELEASE) d = LC_DESC(LC_T_CAS, sid(1), 0);  // locked -> unlocked
                else if (f == LC_F_READ) d = a == LC_NIL ? LC_DESC(LC_T_READ_ANY, 0, 0) : LC_DESC(LC_T_READ, sid(a), 0);
                else if (f == LC_F_WRITE) d = LC_DESC(LC_T_WRITE, 0, sid(a));
                else d = LC_DESC(LC_T_CAS, sid(a), sid(b));
                if (shared) {
                    tid[u] = d;
                    const size_t before = bseen.size();
                    bseen.put(d, 0);
                    if (bseen.size() > before) bdesc[bi].push_back(d);
                } else {
                    std::vector<uint32_t> &ud = kud[(size_t)k];
                    const uint32_t q = (uint32_t)ud.size();
                    const uint32_t at = local.put(d, q);
                    if (at == q) ud.push_back(d);
                    tid[u] = at;  // the key's own id (< 2^24: its distinct descriptors are fewer)
                }
            }
            if (!shared) {  // the key's state table, kept in lstate order as state ids
                std::vector<int64_t> &tab = ktab[(size_t)k];
                tab.assign(lstate.size() + 1, LC_NIL);
                for (auto &kv : lstate)
                    if (kv.second != LC_STATE_NONE) tab[kv.second] = kv.first;
            }
        }
    });
    // (4) transition ids, in key order
    bool too_many = false;
    uint32_t mt = 0;
    if (!shared) {
        P->trans_off.assign((size_t)K, 0);
        for (int64_t k = 0; k < K && !too_many; ++k) {
            const std::vector<uint32_t> &ud = kud[(size_t)k];
            P->state_off[(size_t)k] = P->state_vals.size();
            P->state_vals.insert(P->state_vals.end(), ktab[(size_t)k].begin(), ktab[(size_t)k].end());
            P->trans_off[(size_t)k] = (uint32_t)P->trans.size();
            P->trans.insert(P->trans.end(), ud.begin(), ud.end());
            too_many = ud.size() > 0x1000000u;
            if (!ud.empty()) mt = std::max<uint32_t>(mt, (uint32_t)ud.size() - 1);
        }
        P->state_off[(size_t)K] = P->state_vals.size();
    } else {
        // first appearance over the keys = over the blocks' own lists in block order
        FlatMap gtrans;
        for (const std::vector<uint32_t> &bd : bdesc)
            for (uint32_t d : bd) {
                const uint32_t id = (uint32_t)P->trans.size();
                if (gtrans.put(d, id) == id) P->trans.push_back(d);
            }
        too_many = P->trans.size() > 0x1000000u;
        if (!too_many)
            par.run(blocks, [&](uint64_t bi) {
                for (int64_t k = (int64_t)(bi * (uint64_t)K / blocks); k < (int64_t)((bi + 1) * (uint64_t)K / blocks); ++k) {
                    const KeySpan &sp = ks[(size_t)k];
                    uint32_t *tid = ar[sp.arena].tid.data() + sp.t0;
                    for (uint32_t u = 0; u < sp.nt; ++u) tid[u] = gtrans.get(tid[u], 0);  // now: the global id
                }
            });
        if (!P->trans.empty()) mt = (uint32_t)P->trans.size() - 1;
    }
    *max_tid = mt;
    return !too_many;
}

inline uint16_t word16(uint32_t w) {
    return (uint16_t)(((w >> 16) & 0x8000u) | (LC_EV_SLOT(w) << 11) | LC_EV_TRANS(w));
}

// ---- register models, key-major histories --------------------------------
//
// Every key's rows one run of the history and no row shared by every key:
// what the demo writes (independent/concurrent-generator hands its 10
// threads one key at a time, etcdemo.clj:120-125) and what the synthetic
// C2-C5 generator writes.  No row list is built then.  One pass over the
// history, in row ranges (one per thread; a run belongs to the range it
// starts in), takes each key while its rows are in cache: (0) the run's end,
// row-type counts and process span (validating :type / :f); (1) complete's
// pairing, which records only each op's fate and completion row; (2) the
// events in row order -- failed pairs dropped, lowest free slot at each
// invoke, the op's values after complete's fill interned -- as words with
// the key's own triple indices (16 bits while they fit, the common case,
// else the pass restarts with 32-bit words), into the range's staging, and
// a bit per row that emits no event (how each event's row is found again).
// Then (2)-(4) as on the other path, and one pass writing each word with its
// transition id into the arrays the device reads (page-locked): the 16-bit
// words when every word fits, else the 32-bit ones.  The batch is
// byte-identical to the bucketing path's (tests/test_pack_fast.py).
//
// *took = false (nothing kept) when the history is not key-major, or a key
// needs complete's error or a sparse process map: the bucketing path then
// packs it.
struct KmRec {      // a key's run, as its range packed it
    int64_t key, r0, n;
    uint64_t w0, nw;  // its words in the range's staging
    uint64_t b0;      // its skip bitmap in the range's (ceil(n / 64) words)
    int width;
    KeySpan sp;       // its values and triples in the range's arena
};
struct KmRange {
    std::vector<KmRec> recs;
    Arena A;
    lc::uninit_vector<uint16_t> w16;
    lc::uninit_vector<uint32_t> w32;
    lc::uninit_vector<uint64_t> bits;
};

template <bool W16>
bool km_ranges(const lc_history *h, int model, const Par &par, std::vector<KmRange> &rg, std::atomic<int> &stop) {
    const int64_t n = h->n;
    const unsigned nr = (unsigned)rg.size();
    uint8_t client[256] = {0};  // :f codes the model steps
    for (int f = 0; f <= LC_F_TXN; ++f) client[f] = is_client_f((uint8_t)f, model);
    par.run(nr, [&](uint64_t t) {
        static thread_local std::vector<uint8_t> fate, slot_of;
        static thread_local std::vector<uint32_t> ret, inv_ev, inv_row, inv_id;
        static thread_local std::vector<int32_t> dmap;
        static thread_local Interner in;
        KmRange &R = rg[t];
        R.recs.clear();
        R.A.vals.clear();
        R.A.trip.clear();
        const int64_t R0 = n * (int64_t)t / nr, R1 = n * (int64_t)(t + 1) / nr;
        int64_t r = R0;
        if (t > 0)
            while (r < R1 && h->key[r] == h->key[R0 - 1]) ++r;  // the run of the range before
        uint64_t nw = 0, nb = 0;
        {
            // the staging sized once for the range's rows (its last run may
            // pass R1: the resizes below still grow it), not grown by
            // doubling -- each doubling copied the words written so far
            const uint64_t guess = (uint64_t)(R1 - r) + 8192;
            if (W16) { if (R.w16.size() < guess) R.w16.resize(guess); }
            else if (R.w32.size() < guess) R.w32.resize(guess);
            if (R.bits.size() < guess / 64 + 256) R.bits.resize(guess / 64 + 256);
        }
        while (r < R1) {
            if (stop.load(std::memory_order_relaxed)) return;
            // (0) the run: its end, counts, process span
            const int64_t k = h->key[r];
            if (k == LC_NO_KEY) { stop = 1; return; }  // rows shared by every key: the other path
            int64_t e = r;
            int64_t pmin = h->process[r], pmax = pmin;
            uint64_t ninv = 0;
            for (; e < n && h->key[e] == k; ++e) {
                const uint8_t ty = h->type[e];
                if (ty > LC_INFO || h->f[e] > LC_F_TXN) { stop = 1; return; }
                const int64_t p = h->process[e];
                pmin = std::min(pmin, p);
                pmax = std::max(pmax, p);
                ninv += ty == LC_INVOKE;
            }
            const int64_t nrow = e - r;
            if ((uint64_t)pmax - (uint64_t)pmin >= 4096 || nrow >= (1ll << 32)) { stop = 1; return; }
            const uint64_t pm0 = (uint64_t)pmin;
            dmap.assign((size_t)((uint64_t)pmax - pm0) + 1, -1);
            if (fate.size() < ninv + 1) { fate.resize(ninv + 1); ret.resize(ninv + 1); slot_of.resize(ninv + 1); }
            const uint8_t *ty = h->type + r, *fn = h->f + r;
            const int64_t *pr = h->process + r, *v0 = h->v0 + r, *v1 = h->v1 + r;
            // (1) pairing: each op's fate (0 pending forever, 1 ok, 2 failed)
            // and completion row.  Branch-free (the row types come in no
            // predictable order): a row that records nothing writes the
            // scratch entry past the ops.
            uint32_t q = 0;
            {
                const uint32_t scratch = (uint32_t)ninv;
                uint32_t err = 0;
                for (int64_t i = 0; i < nrow; ++i) {
                    const size_t pi = (size_t)((uint64_t)pr[i] - pm0);
                    const int32_t m = dmap[pi];
                    const uint32_t t8 = ty[i];
                    const uint32_t inv = t8 == LC_INVOKE, info = t8 == LC_INFO, comp = inv == 0 && info == 0;
                    err |= (comp & (uint32_t)(m < 0)) | (inv & (uint32_t)!client[fn[i]]);
                    const uint32_t idx = inv ? q : ((comp && m >= 0) ? (uint32_t)m : scratch);
                    fate[idx] = (uint8_t)(inv ? 0 : (t8 == LC_OK_T ? 1 : 2));
                    ret[idx] = (uint32_t)i;
                    dmap[pi] = inv ? (int32_t)q : -1;
                    q += inv;
                }
                // a completion without an invocation, or an op the model cannot
                // step: complete's error (the other path reports it)
                if (err) { stop = 1; return; }
            }
            // (2) the events, into the range's staging
            const uint64_t cap = nw + (uint64_t)nrow;
            if (W16) { if (R.w16.size() < cap) R.w16.resize(std::max<uint64_t>(cap, R.w16.size() * 2)); }
            else if (R.w32.size() < cap) R.w32.resize(std::max<uint64_t>(cap, R.w32.size() * 2));
            const uint64_t nbw = ((uint64_t)nrow + 63) / 64;
            if (R.bits.size() < nb + nbw) R.bits.resize(std::max<uint64_t>(nb + nbw, R.bits.size() * 2));
            uint16_t *o16 = W16 ? R.w16.data() + nw : nullptr;
            uint32_t *o32 = W16 ? nullptr : R.w32.data() + nw;
            uint64_t *ob = R.bits.data() + nb;
            R.recs.emplace_back();
            KmRec &rec = R.recs.back();
            rec.key = k; rec.r0 = r; rec.n = nrow; rec.w0 = nw; rec.b0 = nb;
            std::fill(dmap.begin(), dmap.end(), -1);
            in.begin(&R.A, model);
            int maxslot = -1;
            uint64_t ne = 0, skipw = 0;
            uint64_t freemask[2] = {~0ull, ~0ull};  // (32-bit words)
            q = 0;
            if (W16) {
                // (2a) branch-free: slots, :ok words, skip bits, and the list
                // of surviving invokes (event, row, op) ...
                const uint32_t scratch = (uint32_t)ninv;
                if (inv_ev.size() < ninv + 1) { inv_ev.resize(ninv + 1); inv_row.resize(ninv + 1); inv_id.resize(ninv + 1); }
                uint64_t free64 = ~0ull;
                uint32_t ni = 0, wide = 0;
                for (int64_t i = 0; i < nrow; ++i) {
                    if ((i & 63) == 0 && i) { ob[(i >> 6) - 1] = skipw; skipw = 0; }
                    const size_t pi = (size_t)((uint64_t)pr[i] - pm0);
                    const int32_t m = dmap[pi];
                    const uint32_t t8 = ty[i];
                    const uint32_t inv = t8 == LC_INVOKE, ok = t8 == LC_OK_T;
                    const uint32_t id = inv ? q : (ok ? (uint32_t)m : scratch);
                    const uint32_t ei = inv & (uint32_t)(fate[inv ? q : scratch] != 2);
                    const uint32_t s_new = (uint32_t)__builtin_ctzll(free64);
                    const uint32_t s_ok = slot_of[ok ? id : scratch];
                    slot_of[ei ? id : scratch] = (uint8_t)s_new;
                    free64 = (free64 & ~((uint64_t)ei << s_new)) | ((uint64_t)ok << (s_ok & 63));
                    wide |= ei & (uint32_t)(s_new > LC_EV16_MAX_SLOT);
                    maxslot = std::max(maxslot, ei ? (int)s_new : -1);
                    o16[ne] = (uint16_t)(ok ? (0x8000u | s_ok << 11) : (s_new << 11));
                    inv_ev[ni] = (uint32_t)ne;
                    inv_row[ni] = (uint32_t)i;
                    inv_id[ni] = id;
                    ni += ei;
                    ne += ei | ok;
                    skipw |= (uint64_t)((ei | ok) ^ 1u) << (i & 63);
                    dmap[pi] = inv ? (int32_t)q : -1;
                    q += inv;
                }
                if (wide) { stop = 2; return; }  // a slot past 15: 32-bit words
                // ... (2b) their values after complete's fill, interned in
                // invoke order
                for (uint32_t j = 0; j < ni; ++j) {
                    const uint32_t i = inv_row[j], id = inv_id[j];
                    const int64_t f = fn[i];
                    int64_t a = v0[i], b = v1[i];
                    if (fate[id] == 1) {  // (or (:value invocation) (:value completion))
                        const uint32_t rr = ret[id];
                        if (f == LC_F_CAS) {
                            if (a == LC_NIL && b == LC_NIL) { a = v0[rr]; b = v1[rr]; }
                        } else if (a == LC_NIL) {
                            a = v0[rr];
                        }
                    }
                    const uint32_t ti = in.op(f, a, b);
                    if (ti > LC_EV16_MAX_TRANS) { stop = 2; return; }  // 32-bit words
                    o16[inv_ev[j]] |= (uint16_t)ti;
                }
            } else
            for (int64_t i = 0; i < nrow; ++i) {
                if ((i & 63) == 0 && i) { ob[(i >> 6) - 1] = skipw; skipw = 0; }
                int32_t &m = dmap[(size_t)((uint64_t)pr[i] - pm0)];
                const uint8_t t8 = ty[i];
                if (t8 == LC_INVOKE) {
                    const uint32_t id = q++;
                    m = (int32_t)id;
                    const uint8_t fa = fate[id];
                    if (fa == 2) { skipw |= 1ull << (i & 63); continue; }  // without-failures
                    int s;
                    if (freemask[0]) s = __builtin_ctzll(freemask[0]);
                    else if (freemask[1]) s = 64 + __builtin_ctzll(freemask[1]);
                    else s = 128;
                    if (s < 127) freemask[s >> 6] &= ~(1ull << (s & 63));
                    const int enc = s < 127 ? s : 127;  // >= 127 cannot be encoded; the search stops earlier
                    slot_of[id] = (uint8_t)enc;
                    maxslot = std::max(maxslot, s);
                    // (or (:value invocation) (:value completion))
                    const int64_t f = fn[i];
                    int64_t a = v0[i], b = v1[i];
                    if (fa == 1) {
                        const uint32_t rr = ret[id];
                        if (f == LC_F_CAS) {
                            if (a == LC_NIL && b == LC_NIL) { a = v0[rr]; b = v1[rr]; }
                        } else if (a == LC_NIL) {
                            a = v0[rr];
                        }
                    }
                    const uint32_t ti = in.op(f, a, b);
                    if (W16) {
                        if (s > (int)LC_EV16_MAX_SLOT || ti > LC_EV16_MAX_TRANS) { stop = 2; return; }  // 32-bit words
                        o16[ne++] = (uint16_t)((uint32_t)s << 11 | ti);
                    } else {
                        o32[ne++] = ((uint32_t)enc << 24) | ti;
                    }
                } else if (t8 == LC_OK_T) {
                    const uint32_t s = slot_of[(size_t)m];
                    if (s < 127) freemask[s >> 6] |= 1ull << (s & 63);
                    m = -1;
                    if (W16) o16[ne++] = (uint16_t)(0x8000u | s << 11);
                    else o32[ne++] = LC_EV_OK_BIT | (s << 24);
                } else {
                    m = -1;
                    skipw |= 1ull << (i & 63);
                }
            }
            ob[nbw - 1] = skipw;
            rec.sp = in.end((uint32_t)t);
            rec.nw = ne;
            rec.width = std::min(maxslot + 1, 255);
            nw += ne;
            nb += nbw;
            r = e;
        }
    });
    return stop.load() == 0;
}

int pack_key_major(const lc_history *h, int model, lc_packed *P, const Par &par, bool *took) {
    *took = false;
    const int64_t n = h->n;
    if (n == 0 || (h->mop_off && h->mop)) return LC_OK;  // (:txn rows: the other path)
    static const bool timing = std::getenv("LC_TIMING") != nullptr;
    auto tprev = std::chrono::steady_clock::now();
    auto lap = [&](const char *what) {
        if (!timing) return;
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "lc_pack (key-major): %-22s %8.1f ms\n", what,
                     std::chrono::duration<double, std::milli>(t - tprev).count());
        tprev = t;
    };
    const unsigned nr = n >= (1 << 16) ? 4 * par.nt : 1u;
    std::vector<KmRange> rg(nr);
    std::atomic<int> stop{0};
    bool w16 = true;
    if (!km_ranges<true>(h, model, par, rg, stop)) {
        if (stop.load() != 2) return LC_OK;  // not key-major (or complete's error): the other path
        stop = 0;
        w16 = false;
        if (!km_ranges<false>(h, model, par, rg, stop)) return LC_OK;
    }
    lap(w16 ? "runs, pairing, events" : "runs, pairing, events (32-bit)");
    // the keys in row order; each must be one run
    int64_t K = 0;
    for (const KmRange &R : rg) K += (int64_t)R.recs.size();
    {
        std::unordered_map<int64_t, char> seen;
        seen.reserve((size_t)K * 2);
        for (const KmRange &R : rg)
            for (const KmRec &x : R.recs)
                if (!seen.emplace(x.key, 0).second) return LC_OK;  // a key in two runs
    }
    P->keys.resize((size_t)K);
    P->key_row0.resize((size_t)K);
    P->krow_off.assign((size_t)K + 1, 0);
    P->ev_off.resize((size_t)K + 1);
    P->ev_off[0] = 0;
    P->skip_off.assign((size_t)K + 1, 0);
    P->key_width.assign((size_t)K, 0);
    std::vector<KeySpan> ks((size_t)K);
    std::vector<Arena> ar(nr);
    std::vector<int64_t> rk(nr + 1, 0);  // first key of each range
    {
        int64_t k = 0;
        for (unsigned t = 0; t < nr; ++t) {
            rk[t] = k;
            ar[t].vals.swap(rg[t].A.vals);
            ar[t].trip.swap(rg[t].A.trip);
            for (const KmRec &x : rg[t].recs) {
                P->keys[(size_t)k] = x.key;
                P->key_row0[(size_t)k] = x.r0;
                P->krow_off[(size_t)k + 1] = P->krow_off[(size_t)k] + (uint64_t)x.n;
                P->ev_off[(size_t)k + 1] = P->ev_off[(size_t)k] + x.nw;
                P->skip_off[(size_t)k + 1] = P->skip_off[(size_t)k] + ((uint64_t)x.n + 63) / 64;
                P->key_width[(size_t)k] = (uint8_t)x.width;
                ks[(size_t)k] = x.sp;
                ++k;
            }
        }
        rk[nr] = k;
    }
    const uint64_t n_ev = P->ev_off[(size_t)K];
    lap("keys, offsets");
    uint32_t max_tid = 0;
    if (!number_and_describe(P, ks, ar, par, &max_tid))
        return lc::fail(LC_E_UNSUPPORTED, "lc_pack: more than 2^24 distinct operations");
    lap("numbering, descriptors");
    // (5) the words with their transition ids: 16-bit when every word fits
    int maxw = 0;
    for (int64_t k = 0; k < K; ++k) maxw = std::max(maxw, (int)P->key_width[(size_t)k]);
    const bool fit16 = n_ev > 0 && maxw <= (int)LC_EV16_MAX_SLOT + 1 && max_tid <= LC_EV16_MAX_TRANS;
    if (fit16) P->events16.alloc(n_ev, true);
    else P->events.alloc(n_ev, true);
    P->skip.alloc(std::max<uint64_t>(P->skip_off[(size_t)K], 1), false);
    P->skip_pre.resize(std::max<uint64_t>(P->skip_off[(size_t)K], 1));
    uint16_t *const E16 = P->events16.data();
    uint32_t *const E32 = P->events.data();
    par.run(nr, [&](uint64_t t) {
        const KmRange &R = rg[t];
        for (int64_t k = rk[t]; k < rk[t + 1]; ++k) {
            const KmRec &x = R.recs[(size_t)(k - rk[t])];
            const uint32_t *tid = ar[t].tid.data() + x.sp.t0;
            const uint64_t e0 = P->ev_off[(size_t)k];
            if (w16) {
                // (an :ok word's id field is 0, and tid[0] exists: the key
                // has an invoke; the select keeps the loop free of branches)
                const uint16_t *src = R.w16.data() + x.w0;
                if (E16) {
                    // (four words per 8-byte non-temporal store: the array is
                    // read next by the DMA engine, not by this core, so its
                    // lines need not be fetched first)
                    uint16_t *dst = E16 + e0;
                    auto word = [&](uint64_t j) -> uint16_t {
                        const uint32_t w = src[j];
                        const uint32_t id = tid[w & 0x7FFu];
                        return (uint16_t)((w & 0xF800u) | ((w & 0x8000u) ? 0u : id));
                    };
                    uint64_t j = 0;
                    for (; j < x.nw && ((uintptr_t)(dst + j) & 7u); ++j) dst[j] = word(j);
                    for (; j + 4 <= x.nw; j += 4) {
                        const uint64_t q = (uint64_t)word(j) | (uint64_t)word(j + 1) << 16 |
                                           (uint64_t)word(j + 2) << 32 | (uint64_t)word(j + 3) << 48;
                        __builtin_nontemporal_store(q, (uint64_t *)(dst + j));
                    }
                    for (; j < x.nw; ++j) dst[j] = word(j);
                } else {
                    uint32_t *dst = E32 + e0;
                    for (uint64_t j = 0; j < x.nw; ++j) {
                        const uint32_t w = src[j];
                        const uint32_t id = tid[w & 0x7FFu];
                        dst[j] = ((w & 0x8000u) << 16) | ((w >> 11 & 0xFu) << 24) | ((w & 0x8000u) ? 0u : id);
                    }
                }
            } else {
                const uint32_t *src = R.w32.data() + x.w0;
                for (uint64_t j = 0; j < x.nw; ++j) {
                    const uint32_t w = src[j];
                    const uint32_t v = (w & LC_EV_OK_BIT) ? w : (w & 0xFF000000u) | tid[w & 0xFFFFFFu];
                    if (E16) E16[e0 + j] = word16(v);
                    else E32[e0 + j] = v;
                }
            }
            const uint64_t s0 = P->skip_off[(size_t)k], s1 = P->skip_off[(size_t)k + 1];
            std::memcpy(P->skip.data() + s0, R.bits.data() + x.b0, (s1 - s0) * 8);
            uint32_t kept = 0;
            for (uint64_t w = s0; w < s1; ++w) {
                P->skip_pre[w] = kept;
                kept += (uint32_t)__builtin_popcountll(~P->skip[w]);
            }
        }
    });
    if (P->trans.empty()) P->trans.push_back(LC_DESC(LC_T_READ_ANY, 0, 0));
    std::atomic_thread_fence(std::memory_order_seq_cst);  // (the non-temporal stores drained: sfence)
    lap("transition ids");
    P->key_major = true;
    *took = true;
    return LC_OK;
}
}  // namespace


extern "C" int lc_pack(const lc_history *h, const lc_pack_opts *opts, lc_packed **out) {
    if (!h || !out) return lc::fail(LC_E_INVALID, "lc_pack: null argument");
    const int model = opts ? opts->model : LC_MODEL_CAS_REGISTER;
    if (model < LC_MODEL_CAS_REGISTER || model > LC_MODEL_MULTI_REGISTER)
        return lc::fail(LC_E_INVALID, "lc_pack: unknown model %d", model);
    if (opts && (opts->flags & ~LC_PACK_GENERAL)) return lc::fail(LC_E_INVALID, "lc_pack: unknown flags 0x%x", opts->flags);
    const int32_t n_init = (opts && model == LC_MODEL_MULTI_REGISTER) ? opts->n_init : 0;
    if (n_init < 0 || (n_init > 0 && !opts->init)) return lc::fail(LC_E_INVALID, "lc_pack: bad initial registers");
    if (h->n < 0 || (h->n > 0 && (!h->type || !h->f || !h->process || !h->key || !h->v0 || !h->v1)))
        return lc::fail(LC_E_INVALID, "lc_pack: history arrays missing");
    const int64_t n = h->n;
    lc::Range range("lc_pack");
    lc_packed *P = new (std::nothrow) lc_packed();
    if (!P) return lc::fail(LC_E_NOMEM, "lc_pack: out of memory");
    static const bool timing = std::getenv("LC_TIMING") != nullptr;
    auto tprev = std::chrono::steady_clock::now();
    auto lap = [&](const char *what) {
        if (!timing) return;
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "lc_pack: %-28s %8.1f ms\n", what, std::chrono::duration<double, std::milli>(t - tprev).count());
        tprev = t;
    };
    try {
        if (model != LC_MODEL_MULTI_REGISTER && !(opts && (opts->flags & LC_PACK_GENERAL))) {
            bool took = false;
            int rc;
            {
                const lc::PackPoolGuard hold;  // released on every exit
                Par par;
                par.pool = hold.pool;
                par.nt = par.pool ? par.pool->size() : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
                rc = pack_key_major(h, model, P, par, &took);
            }
            if (rc) { delete P; return rc; }
            if (took) {
                lap("key-major pack");
                *out = P;
                return LC_OK;
            }
        }
        // ---- A2: key discovery + bucketing (stable) ----
        // Rows in contiguous ranges, one per thread: each range numbers its
        // keys in order of first appearance; the ranges' key lists are then
        // merged in range order (= the order of first appearance in the
        // history), and the rows are bucketed by key through per-range counts.
        const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        const unsigned nr = n >= (1 << 20) ? hw : 1u;
        auto range_rows = [&](const auto &fn) {
            auto work = [&](unsigned t) { fn(t, n * (int64_t)t / nr, n * (int64_t)(t + 1) / nr); };
            lc::run_threads(nr, work);
        };
        lc::uninit_vector<int32_t> row_key((size_t)n);  // every row written below
        std::vector<std::vector<int64_t>> rkeys(nr), rshared(nr);
        std::vector<int64_t> bad_row(nr, -1), bad_mop(nr, -1);
        range_rows([&](unsigned t, int64_t r0, int64_t r1) {
            std::unordered_map<int64_t, int32_t> kidx;
            int64_t last_key = LC_NO_KEY;
            int32_t last_idx = -1;
            for (int64_t r = r0; r < r1; ++r) {
                if (h->type[r] > LC_INFO || h->f[r] > LC_F_TXN) { bad_row[t] = r; return; }
                if (h->mop_off && h->mop && (h->mop_off[r] < 0 || h->mop_off[r + 1] < h->mop_off[r])) {
                    bad_mop[t] = r;
                    return;
                }
                const int64_t k = h->key[r];
                if (k == LC_NO_KEY) {
                    row_key[(size_t)r] = -1;
                    // Non-tuple ops are shared by every sub-history (subhistory keeps
                    // them): the nemesis's :info ops are no-ops there, and any other
                    // op is paired and stepped in every key as it stands.
                    rshared[t].push_back(r);
                    continue;
                }
                if (k != last_key || last_idx < 0) {
                    auto it = kidx.find(k);
                    if (it == kidx.end()) {
                        it = kidx.emplace(k, (int32_t)rkeys[t].size()).first;
                        rkeys[t].push_back(k);
                    }
                    last_key = k;
                    last_idx = it->second;
                }
                row_key[(size_t)r] = last_idx;  // the range's own number, for now
            }
        });
        for (unsigned t = 0; t < nr; ++t) {
            if (bad_row[t] >= 0) {
                delete P;
                return lc::fail(LC_E_INVALID, "lc_pack: row %lld has a bad :type/:f code", (long long)bad_row[t]);
            }
            if (bad_mop[t] >= 0) {
                delete P;
                return lc::fail(LC_E_INVALID, "lc_pack: mop_off not monotone at row %lld", (long long)bad_mop[t]);
            }
        }
        std::vector<std::vector<int32_t>> rglobal(nr);  // range key number -> packed key
        {
            std::unordered_map<int64_t, int32_t> kidx;
            for (unsigned t = 0; t < nr; ++t) {
                for (int64_t k : rkeys[t]) {
                    auto it = kidx.emplace(k, (int32_t)P->keys.size());
                    if (it.second) P->keys.push_back(k);
                    rglobal[t].push_back(it.first->second);
                }
                P->shared_rows.insert(P->shared_rows.end(), rshared[t].begin(), rshared[t].end());
            }
        }
        const int64_t K = (int64_t)P->keys.size();
        // per-range counts of each key's rows: the range's write positions
        std::vector<std::vector<uint64_t>> rcount(nr, std::vector<uint64_t>());
        range_rows([&](unsigned t, int64_t r0, int64_t r1) {
            std::vector<uint64_t> &c = rcount[t];
            c.assign((size_t)K, 0);
            const std::vector<int32_t> &g = rglobal[t];
            for (int64_t r = r0; r < r1; ++r) {
                int32_t &rk = row_key[(size_t)r];
                if (rk < 0) continue;
                rk = g[(size_t)rk];
                ++c[(size_t)rk];
            }
        });
        lap("A2 key discovery");
        P->krow_off.assign((size_t)K + 1, 0);
        for (int64_t k = 0; k < K; ++k) {
            uint64_t at = P->krow_off[(size_t)k];
            for (unsigned t = 0; t < nr; ++t) {
                const uint64_t c = rcount[t][(size_t)k];
                rcount[t][(size_t)k] = at;  // where range t writes key k's rows
                at += c;
            }
            P->krow_off[(size_t)k + 1] = at;
        }
        P->krows.resize((size_t)P->krow_off[(size_t)K]);
        range_rows([&](unsigned t, int64_t r0, int64_t r1) {
            std::vector<uint64_t> &cur = rcount[t];
            for (int64_t r = r0; r < r1; ++r)
                if (row_key[(size_t)r] >= 0) P->krows[cur[(size_t)row_key[(size_t)r]]++] = r;
        });
        lc::uninit_vector<int32_t>().swap(row_key);
        lap("A2 bucketing");

        // ---- A3: per-key pairing, fail-drop, slots (parallel over keys) ----
        unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        if (K < 64) nt = 1;
        auto par_keys = [&](const auto &fn) {  // fn(key, thread)
            auto work = [&](unsigned t) {
                for (int64_t k = t; k < K; k += nt) fn(k, t);
            };
            lc::run_threads(nt, work);
        };
        // key k's rows plus the shared rows, in history order
        auto key_rows = [&](int64_t k, std::vector<int64_t> &merged, const int64_t *&rows, int64_t &nrows) {
            const int64_t *kr = P->krows.data() + P->krow_off[(size_t)k];
            const int64_t nk = (int64_t)(P->krow_off[(size_t)k + 1] - P->krow_off[(size_t)k]);
            if (P->shared_rows.empty()) {
                rows = kr;
                nrows = nk;
                return;
            }
            merged.resize((size_t)nk + P->shared_rows.size());
            std::merge(kr, kr + nk, P->shared_rows.begin(), P->shared_rows.end(), merged.begin());
            rows = merged.data();
            nrows = (int64_t)merged.size();
        };
        auto key_error = [&](int64_t k, const std::string &msg) {  // serial
            if (P->key_error.empty()) {
                P->key_error.assign((size_t)K, 0);
                P->key_msg.assign((size_t)K, std::string());
            }
            P->key_error[(size_t)k] = 1;  // no events: the search never looks at this key
            P->key_msg[(size_t)k] = msg;
        };
        if (model == LC_MODEL_MULTI_REGISTER) {
            std::vector<KeyOut> ko((size_t)K);
            par_keys([&](int64_t k, unsigned) {
                static thread_local std::vector<int64_t> merged;
                const int64_t *rows;
                int64_t nrows;
                key_rows(k, merged, rows, nrows);
                pack_key(*h, rows, nrows, model, ko[(size_t)k]);
            });
            lap("A3 pairing (parallel)");
            for (int64_t k = 0; k < K; ++k) {
                KeyOut &o = ko[(size_t)k];
                if (!o.err) continue;
                key_error(k, o.msg);
                std::vector<uint32_t>().swap(o.ev);
                std::vector<int64_t>().swap(o.ev_row);
                std::vector<int32_t>().swap(o.ev_op);
                std::vector<KOp>().swap(o.ops);
                o.width = 0;
            }
            pack_multi_register(*h, n_init ? opts->init : nullptr, n_init, ko, nt, P);
            *out = P;
            return LC_OK;
        }

        // ---- A3-A5 for the register models ----
        // A state is a value some surviving write / cas could install.  Keys
        // are independent up to the shared numbering, so: (1) per key, in
        // parallel: pairing, its events into a flat staging array (its rows'
        // span plus the shared rows) with each invoke's index among the key's
        // distinct (f, value) triples in the trans field, its state values in
        // order of first appearance; (2) serially, the shared state numbering
        // (or per-key tables past 254 values); (3) per key, in parallel, the
        // descriptor of each triple and the key's distinct descriptors in
        // order of first appearance; (4) serially over keys (a few dozen
        // descriptors each), their global transition ids; (5) per key, in
        // parallel, the event words.  The ids are those of one serial pass
        // over keys and events.  Per key only short lists outlive step (1).
        struct GenKey {
            int64_t n_ev = 0;
            int width = 0, err = 0;
            std::string msg;
        };
        std::vector<GenKey> gk((size_t)K);
        std::vector<KeySpan> ks((size_t)K);
        std::vector<Arena> ar(nt);  // one per thread
        const uint64_t n_shared = P->shared_rows.size();
        auto stage_off = [&](int64_t k) { return P->krow_off[(size_t)k] + (uint64_t)k * n_shared; };
        // staging kept between calls (its pages stay mapped: no fresh page
        // faults per call); a call that finds it taken allocates its own
        Staging own;
        std::unique_lock<std::mutex> lk(g_staging_mu, std::try_to_lock);
        Staging &stg = lk.owns_lock() ? g_staging : own;
        stg.ev.resize(std::max<uint64_t>(stage_off(K), 1));
        stg.row.resize(std::max<uint64_t>(stage_off(K), 1));
        uint32_t *const st_ev = stg.ev.data();
        int64_t *const st_row = stg.row.data();
        par_keys([&](int64_t k, unsigned t) {
            static thread_local std::vector<int64_t> merged;
            static thread_local std::vector<KOp> ops;
            static thread_local std::vector<int32_t> row_op;
            static thread_local std::vector<uint32_t> tix;
            GenKey &o = gk[(size_t)k];
            const int64_t *rows;
            int64_t nrows;
            key_rows(k, merged, rows, nrows);
            if (!pair_rows(*h, rows, nrows, model, ops, row_op, o.err, o.msg)) {
                ks[(size_t)k] = KeySpan{t, 0, 0, ar[t].vals.size(), ar[t].trip.size() / 3};
                if (model == LC_MODEL_MUTEX) {  // (the mutex's state value, as Interner.begin adds it)
                    ks[(size_t)k].nv = 1;
                    ar[t].vals.push_back(1);
                }
                return;
            }
            uint32_t *ev = st_ev + stage_off(k);
            o.n_ev = emit_events(rows, nrows, ops, row_op, ev, st_row + stage_off(k), nullptr, o.width);
            // (1) distinct state values, and each surviving op's triple
            // index (the fields its descriptor reads), distinct triples in
            // invoke order (Interner)
            static thread_local Interner in;
            in.begin(&ar[t], model);
            tix.resize(ops.size());
            for (size_t q = 0; q < ops.size(); ++q) {
                const KOp &op = ops[q];
                if (op.fate == 2) continue;
                tix[q] = in.op(op.f, op.v0, op.v1);
            }
            ks[(size_t)k] = in.end(t);
            for (int64_t j = 0; j < o.n_ev; ++j)
                if (!(ev[j] & LC_EV_OK_BIT)) ev[j] = (ev[j] & 0xFF000000u) | tix[ev[j] & 0xFFFFFFu];
        });
        lap("A3/A4 (1) pairing, values, triples");
        for (int64_t k = 0; k < K; ++k)
            if (gk[(size_t)k].err) key_error(k, gk[(size_t)k].msg);
        P->key_width.assign((size_t)K, 0);
        P->ev_off.assign((size_t)K + 1, 0);
        for (int64_t k = 0; k < K; ++k) P->ev_off[(size_t)k + 1] = P->ev_off[(size_t)k] + (uint64_t)gk[(size_t)k].n_ev;
        P->events.alloc((size_t)P->ev_off[(size_t)K], true);
        P->ev_row.resize((size_t)P->ev_off[(size_t)K]);
        lap("A4 (2) arrays");
        {
            Par par;
            par.nt = nt;
            uint32_t max_tid = 0;
            if (!number_and_describe(P, ks, ar, par, &max_tid)) {
                delete P;
                return lc::fail(LC_E_UNSUPPORTED, "lc_pack: more than 2^24 distinct operations");
            }
        }
        lap("A5 (2)-(4) numbering, descriptors, transition ids");
        // (5) event words with transition ids, rows, widths
        par_keys([&](int64_t k, unsigned) {
            const GenKey &o = gk[(size_t)k];
            const uint32_t *tid = ar[ks[(size_t)k].arena].tid.data() + ks[(size_t)k].t0;
            const uint32_t *src = st_ev + stage_off(k);
            const int64_t *srow = st_row + stage_off(k);
            const uint64_t base = P->ev_off[(size_t)k];
            for (int64_t j = 0; j < o.n_ev; ++j) {
                const uint32_t w = src[j];
                P->events[base + (uint64_t)j] = (w & LC_EV_OK_BIT) ? w : (w & 0xFF000000u) | tid[w & 0xFFFFFFu];
                P->ev_row[base + (uint64_t)j] = srow[j];
            }
            P->key_width[(size_t)k] = (uint8_t)o.width;
        });
        if (P->trans.empty()) P->trans.push_back(LC_DESC(LC_T_READ_ANY, 0, 0));
        lap("A5 (5) event words");
        // 16-bit event words (lc_batch.events16) when every word fits: half
        // the bytes over the host link for the register tier (both passes
        // split over the threads in contiguous ranges)
        const size_t n_ev = P->events.size();
        std::vector<char> fits(nt, 1);
        auto range_pass = [&](const auto &fn) {
            auto work = [&](unsigned t) { fn(t, n_ev * t / nt, n_ev * (t + 1) / nt); };
            lc::run_threads(nt, work);
        };
        range_pass([&](unsigned t, size_t j0, size_t j1) {
            for (size_t j = j0; j < j1 && fits[t]; ++j) {
                const uint32_t w = P->events[j];
                fits[t] = LC_EV_SLOT(w) <= LC_EV16_MAX_SLOT && LC_EV_TRANS(w) <= LC_EV16_MAX_TRANS;
            }
        });
        const bool fit16 = n_ev > 0 && std::all_of(fits.begin(), fits.end(), [](char c) { return c != 0; });
        if (fit16) {
            P->events16.alloc(n_ev, true);
            range_pass([&](unsigned, size_t j0, size_t j1) {
                for (size_t j = j0; j < j1; ++j) P->events16[j] = word16(P->events[j]);
            });
            P->events.release();  // the 16-bit words are the batch's (the device widens them)
        }
        lap("16-bit words");
    } catch (const std::bad_alloc &) {
        delete P;
        return lc::fail(LC_E_NOMEM, "lc_pack: out of memory");
    } catch (const std::length_error &) {
        delete P;
        return lc::fail(LC_E_UNSUPPORTED, "lc_pack: transition table beyond 2^32 entries");
    }
    *out = P;
    return LC_OK;
}

extern "C" void lc_packed_free(lc_packed *p) { delete p; }

extern "C" int lc_packed_view(const lc_packed *p, lc_batch *b) {
    if (!p || !b) return lc::fail(LC_E_INVALID, "lc_packed_view: null argument");
    b->n_keys = (int64_t)p->keys.size();
    b->ev_off = p->ev_off.data();
    b->events = p->events.data();
    b->trans = p->trans.data();
    b->n_trans = (int64_t)p->trans.size();
    b->trans_off = p->trans_off.empty() ? nullptr : p->trans_off.data();
    b->key_width = p->key_width.data();
    b->key_states = p->key_states.data();
    b->init_state = 0;
    b->key_error = p->key_error.empty() ? nullptr : p->key_error.data();
    b->table = p->table.empty() ? nullptr : p->table.data();
    b->n_table = (int64_t)p->table.size();
    b->events16 = p->events16.empty() ? nullptr : p->events16.data();
    return LC_OK;
}

extern "C" int64_t lc_packed_state_map(const lc_packed *p, int64_t i, uint32_t s, int64_t *regs, int64_t *vals,
                                       int64_t cap) {
    if (!p || i < 0 || i >= (int64_t)p->keys.size() || cap < 0 || (cap && (!regs || !vals)))
        return lc::fail(LC_E_INVALID, "lc_packed_state_map: bad argument");
    if (p->model != LC_MODEL_MULTI_REGISTER) return lc::fail(LC_E_INVALID, "lc_packed_state_map: not a multi-register batch");
    const uint64_t r0 = p->mr_reg_off[(size_t)i], R = p->mr_reg_off[(size_t)i + 1] - r0;
    const uint64_t s0 = p->mr_state_off[(size_t)i], n = p->mr_state_off[(size_t)i + 1] - s0;
    if ((uint64_t)s * R >= n && !(R == 0 && s == 0))
        return lc::fail(LC_E_INVALID, "lc_packed_state_map: state %u out of range", s);
    int64_t m = 0;
    for (uint64_t r = 0; r < R; ++r) {
        const int64_t v = p->mr_states[s0 + (uint64_t)s * R + r];
        if (v == ABSENT) continue;
        if (m < cap) { regs[m] = p->mr_regs[r0 + r]; vals[m] = v; }
        ++m;
    }
    return m;
}

extern "C" const char *lc_packed_key_error(const lc_packed *p, int64_t i) {
    if (!p || i < 0 || i >= (int64_t)p->keys.size() || p->key_error.empty() || !p->key_error[(size_t)i])
        return nullptr;
    return p->key_msg[(size_t)i].c_str();
}

extern "C" int64_t lc_packed_key(const lc_packed *p, int64_t i) {
    if (!p || i < 0 || i >= (int64_t)p->keys.size()) return lc::fail(LC_E_INVALID, "lc_packed_key: bad index"), LC_NO_KEY;
    return p->keys[(size_t)i];
}

extern "C" int64_t lc_packed_event_row(const lc_packed *p, int64_t i, int64_t j) {
    if (!p || i < 0 || i >= (int64_t)p->keys.size()) return lc::fail(LC_E_INVALID, "lc_packed_event_row: bad key");
    uint64_t b = p->ev_off[(size_t)i], e = p->ev_off[(size_t)i + 1];
    if (j < 0 || (uint64_t)j >= e - b) return lc::fail(LC_E_INVALID, "lc_packed_event_row: bad event");
    return p->event_row((size_t)i, b + (uint64_t)j);
}

extern "C" int lc_packed_path(const lc_packed *p) { return p && p->key_major ? 1 : 0; }

extern "C" int64_t lc_packed_event_rows(const lc_packed *p, int64_t *out) {
    if (!p) return lc::fail(LC_E_INVALID, "lc_packed_event_rows: null packed batch");
    const size_t K = p->keys.size();
    const int64_t n = K ? (int64_t)p->ev_off[K] : 0;
    if (out) p->event_rows(out);
    return n;
}

void lc_packed::event_rows(int64_t *out) const {
    const size_t K = keys.size();
    for (size_t k = 0; k < K; ++k) {
        if (!key_major) {
            for (uint64_t e = ev_off[k]; e < ev_off[k + 1]; ++e) out[e] = ev_row[e];
            continue;
        }
        uint64_t e = ev_off[k];
        for (uint64_t w = skip_off[k]; w < skip_off[k + 1] && e < ev_off[k + 1]; ++w)
            for (uint64_t x = ~skip[w]; x && e < ev_off[k + 1]; x &= x - 1)
                out[e++] = key_row0[k] + (int64_t)(64 * (w - skip_off[k])) + __builtin_ctzll(x);
    }
}

extern "C" int64_t lc_packed_subhistory(const lc_packed *p, int64_t i, int64_t *out_rows) {
    if (!p || i < 0 || i >= (int64_t)p->keys.size()) return lc::fail(LC_E_INVALID, "lc_packed_subhistory: bad key");
    int64_t na = (int64_t)(p->krow_off[(size_t)i + 1] - p->krow_off[(size_t)i]);
    if (p->key_major) {  // the key's rows are one run (no shared rows)
        if (out_rows)
            for (int64_t j = 0; j < na; ++j) out_rows[j] = p->key_row0[(size_t)i] + j;
        return na;
    }
    const int64_t *a = p->krows.data() + p->krow_off[(size_t)i];
    const int64_t *s = p->shared_rows.data();
    int64_t ns = (int64_t)p->shared_rows.size();
    if (out_rows) std::merge(a, a + na, s, s + ns, out_rows);
    return na + ns;
}

extern "C" int lc_packed_state_value(const lc_packed *p, int64_t i, uint32_t s, int64_t *value, int *is_nil) {
    if (!p || !value || !is_nil || i < 0 || i >= (int64_t)p->keys.size())
        return lc::fail(LC_E_INVALID, "lc_packed_state_value: bad argument");
    if (s == 0) { *is_nil = 1; *value = LC_NIL; return LC_OK; }
    uint64_t base = p->state_off.empty() ? 0 : p->state_off[(size_t)i];
    uint64_t lim = p->state_off.empty() ? p->state_vals.size() : p->state_off[(size_t)i + 1];
    if (base + s >= lim) return lc::fail(LC_E_INVALID, "lc_packed_state_value: state %u out of range", s);
    *is_nil = 0;
    *value = p->state_vals[base + s];
    return LC_OK;
}
