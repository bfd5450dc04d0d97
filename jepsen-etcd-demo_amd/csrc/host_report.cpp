// lc_report: the Knossos-shaped counterexample of one key, rendered from its
// verdict record and the final configs the device returned (SURVEY.md 8(a)
// A8, 8(f) F-2).  jepsen.checker/linearizable (etcdemo.clj:117-118) reports,
// for an invalid key, the :ok that could not be linearized (:op), the last
// :ok before it (:previous-ok / :last-op), the config set standing before it
// (:configs) and :final-paths -- from each of those configs, every sequence of
// further pending ops the model allows, ending with the failing op, which is
// inconsistent in every state so reached (that is why the set emptied).
// Knossos iterates a hash set here, so only the SET of paths is comparable;
// paths are generated depth-first, shortest first, from the configs in device
// order, up to max_paths distinct ones (jepsen truncates to 10).  Both
// bindings (Python lincheck.checker, the JVM's gpu_checker.clj) decode this
// one rendering.
//
// lc_report_wgl shapes the same key for :algorithm :wgl (knossos.wgl, SURVEY
// 8(f) F-3; parity unpinned -- restated in oracle/wgl_ref.py).  The Wing-Gong
// search with Lowe's cache gets stuck, at its deepest, on the same :ok (the
// first whose prefix cannot be linearized: a property of the history), and
// its frontier there is every (model, linearized pending ops) it reached at
// that return entry: the closure of the config set standing before the :ok
// under the pending ops other than the failing one.  :configs are those
// frontier configs, breadth first from the device's configs (so a subset of
// the frontier when the device truncated them); :op, :previous-ok,
// :last-op and :final-paths are shaped as for :linear.

#include <algorithm>
#include <set>
#include <vector>

#include "common.hpp"
#include "packed.hpp"

namespace {

// One interned transition from state st (include/lincheck.h LC_DESC): the
// next state, or LC_STATE_NONE when the model step is inconsistent.
uint32_t desc_step(uint32_t d, uint32_t st) {
    const uint32_t t = d & 3u, a = (d >> 2) & 0x7FFFu, b = d >> 17;
    if (t == LC_T_READ_ANY) return st;
    if (t == LC_T_READ) return st == a ? st : LC_STATE_NONE;
    if (t == LC_T_WRITE) return b;
    return st == a ? b : LC_STATE_NONE;
}

struct KeyView {
    const lc_packed *p;
    int64_t key;
    uint64_t eb, n;             // the key's events: [eb, eb + n)
    // (slot, invoke event (ordinal)) holding it at `upto`, in slot order.
    // Built from a per-slot array in one pass: a std::map updated at every
    // event was most of a C5 counterexample's rendering (~70 us per key).
    std::vector<std::pair<uint32_t, uint64_t>> held;
    int64_t last_ok = -1;       // last :ok event before `upto`

    KeyView(const lc_packed *pk, int64_t k, uint64_t upto) : p(pk), key(k) {
        eb = p->ev_off[(size_t)k];
        n = p->ev_off[(size_t)k + 1] - eb;
        upto = std::min<uint64_t>(upto, n);
        constexpr uint32_t NS = 128;  // LC_EV_SLOT's range
        uint64_t at[NS];
        bool on[NS] = {};
        for (uint64_t j = 0; j < upto; ++j) {
            const uint32_t w = p->word(eb + j);
            const uint32_t s = LC_EV_SLOT(w);
            if (w & LC_EV_OK_BIT) {
                on[s] = false;
                last_ok = (int64_t)j;
            } else {
                on[s] = true;
                at[s] = j;
            }
        }
        for (uint32_t s = 0; s < NS; ++s)
            if (on[s]) held.push_back({s, at[s]});
    }
    const std::pair<uint32_t, uint64_t> *find(uint32_t s) const {
        for (const auto &h : held)
            if (h.first == s) return &h;
        return nullptr;
    }
    int64_t row(uint64_t j) const { return p->event_row((size_t)key, eb + j); }
    // the row completing invoke event j (its slot's next event, when an :ok)
    int64_t done_row(uint64_t j) const {
        const uint32_t s = LC_EV_SLOT(p->word(eb + j));
        for (uint64_t i = j + 1; i < n; ++i) {
            const uint32_t w = p->word(eb + i);
            if (LC_EV_SLOT(w) == s) return (w & LC_EV_OK_BIT) ? row(i) : -1;
        }
        return -1;
    }
    uint32_t desc(uint64_t j) const {
        const uint64_t tb = p->trans_off.empty() ? 0 : p->trans_off[(size_t)key];
        return p->trans[tb + LC_EV_TRANS(p->word(eb + j))];
    }
    // the op of invoke event j from state st: next state or LC_STATE_NONE
    uint32_t step(uint64_t j, uint32_t st) const {
        const uint32_t d = desc(j);
        if (p->table.empty()) return desc_step(d, st);
        const uint16_t s2 = p->table[(size_t)d + st];  // a table-model row (lc_batch.table)
        return s2 == LC_TABLE_NONE ? LC_STATE_NONE : s2;
    }
    int64_t value(uint32_t st) const {
        if (p->model == LC_MODEL_MULTI_REGISTER) return st;  // a map: lc_packed_state_map
        if (st == 0) return LC_NIL;
        const uint64_t base = p->state_off.empty() ? 0 : p->state_off[(size_t)key];
        const uint64_t lim = p->state_off.empty() ? p->state_vals.size() : p->state_off[(size_t)key + 1];
        return base + st < lim ? p->state_vals[base + st] : LC_NIL;
    }
};

}  // namespace

static int64_t report(const lc_packed *p, int64_t key, int32_t valid, int32_t fail_event,
                      const uint64_t *final_configs, uint32_t n_final, int32_t max_paths, bool wgl, int64_t *out,
                      int64_t cap) {
    if (!p || key < 0 || key >= (int64_t)p->keys.size() || (n_final && !final_configs) || cap < 0 ||
        (cap && !out))
        return lc::fail(LC_E_INVALID, "lc_report: bad argument");
    if (!p->key_error.empty() && p->key_error[(size_t)key])
        return lc::fail(LC_E_INVALID, "lc_report: key %lld could not be prepared: %s", (long long)key,
                        p->key_msg[(size_t)key].c_str());
    const uint64_t n_ev = p->ev_off[(size_t)key + 1] - p->ev_off[(size_t)key];
    if (fail_event >= 0 && (uint64_t)fail_event >= n_ev) return lc::fail(LC_E_INVALID, "lc_report: bad fail_event");
    const uint64_t upto = fail_event >= 0 ? (uint64_t)fail_event : n_ev;
    try {
        KeyView kv(p, key, upto);
        std::vector<int64_t> o;
        o.push_back(fail_event >= 0 ? kv.row((uint64_t)fail_event) : -1);
        o.push_back(kv.last_ok >= 0 ? kv.row((uint64_t)kv.last_ok) : -1);
        o.push_back(0);  // n_configs
        o.push_back(0);  // n_paths
        // final configs: {state, slot mask} as the device writes them
        std::vector<std::pair<uint32_t, std::pair<uint64_t, uint64_t>>> finals;
        for (uint32_t c = 0; c < n_final; ++c) {
            const uint64_t lo = final_configs[2 * c], hi = final_configs[2 * c + 1];
            finals.push_back({(uint32_t)((hi >> 48) & 0x7FFFu), {lo, hi & ((1ull << 48) - 1)}});
        }
        auto in_mask = [](const std::pair<uint64_t, uint64_t> &m, uint32_t s) {
            return s < 64 ? ((m.first >> s) & 1) != 0 : ((m.second >> (s - 64)) & 1) != 0;
        };
        const uint32_t p_slot = fail_event >= 0 ? LC_EV_SLOT(p->word(kv.eb + (uint64_t)fail_event)) : 0xFFFFFFFFu;
        const size_t want = (size_t)std::max(max_paths, 0);
        std::vector<std::pair<uint32_t, std::pair<uint64_t, uint64_t>>> shown(
            finals.begin(), finals.begin() + (ptrdiff_t)std::min(finals.size(), want));
        if (wgl && valid == LC_INVALID && fail_event >= 0) {
            // WGL's frontier at the stuck return entry: breadth first from the
            // device's configs, every legal linearization of a further pending
            // op other than the failing one, each distinct config once
            std::set<std::pair<uint32_t, std::pair<uint64_t, uint64_t>>> seen(finals.begin(), finals.end());
            std::vector<std::pair<uint32_t, std::pair<uint64_t, uint64_t>>> q(finals.begin(), finals.end());
            for (size_t at = 0; at < q.size() && shown.size() < want && seen.size() < (1u << 16); ++at) {
                const auto c = q[at];
                for (auto &h : kv.held) {
                    if (h.first == p_slot || in_mask(c.second, h.first)) continue;
                    const uint32_t s2 = kv.step(h.second, c.first);
                    if (s2 == LC_STATE_NONE) continue;
                    auto m2 = c.second;
                    if (h.first < 64) m2.first |= 1ull << h.first;
                    else m2.second |= 1ull << (h.first - 64);
                    const std::pair<uint32_t, std::pair<uint64_t, uint64_t>> c2{s2, m2};
                    if (!seen.insert(c2).second) continue;
                    q.push_back(c2);
                    if (shown.size() < want) shown.push_back(c2);
                }
            }
        }
        const size_t n_cfg = shown.size();
        for (size_t c = 0; c < n_cfg; ++c) {
            o.push_back(kv.value(shown[c].first));
            for (int lin = 0; lin < 2; ++lin) {
                const size_t at = o.size();
                o.push_back(0);
                for (auto &h : kv.held)
                    if (in_mask(shown[c].second, h.first) == (lin == 1)) {
                        o.push_back(kv.row(h.second));
                        o.push_back(kv.done_row(h.second));
                        ++o[at];
                    }
            }
        }
        o[2] = (int64_t)n_cfg;
        if (valid == LC_INVALID && fail_event >= 0 && max_paths > 0) {
            const auto *ph = kv.find(p_slot);
            if (ph) {
                const uint64_t p_inv = ph->second;
                std::vector<std::pair<uint32_t, uint64_t>> others;  // (slot, invoke event)
                for (auto &h : kv.held)
                    if (h.first != p_slot) others.push_back(h);
                std::set<std::vector<uint64_t>> seen;
                std::vector<std::pair<uint64_t, uint32_t>> steps;  // (invoke event, state after)
                int64_t visits = 0, n_paths = 0;
                const int64_t max_visits = 1 << 16;
                uint32_t st0 = 0;
                auto emit = [&](uint32_t st) {
                    std::vector<uint64_t> id{st0};
                    for (auto &s : steps) id.push_back(s.first);
                    if (!seen.insert(id).second) return;
                    o.push_back(kv.value(st0));
                    o.push_back((int64_t)steps.size());
                    for (auto &s : steps) {
                        o.push_back(kv.row(s.first));
                        o.push_back(kv.done_row(s.first));
                        o.push_back(kv.value(s.second));
                    }
                    o.push_back(kv.value(st));  // the state the failing op cannot be stepped in
                    ++n_paths;
                };
                std::vector<char> used(others.size(), 0);
                auto dfs = [&](auto &&self, uint32_t st) -> void {
                    ++visits;
                    if (n_paths >= max_paths || visits > max_visits) return;
                    if (kv.step(p_inv, st) == LC_STATE_NONE) emit(st);
                    for (size_t q = 0; q < others.size(); ++q) {
                        if (used[q]) continue;
                        const uint32_t s2 = kv.step(others[q].second, st);
                        if (s2 == LC_STATE_NONE) continue;
                        used[q] = 1;
                        steps.push_back({others[q].second, s2});
                        self(self, s2);
                        steps.pop_back();
                        used[q] = 0;
                        if (n_paths >= max_paths || visits > max_visits) return;
                    }
                };
                for (auto &f : finals) {
                    if (n_paths >= max_paths) break;
                    st0 = f.first;
                    for (size_t q = 0; q < others.size(); ++q) used[q] = in_mask(f.second, others[q].first);
                    dfs(dfs, st0);
                }
                o[3] = n_paths;
            }
        }
        if ((int64_t)o.size() <= cap) std::copy(o.begin(), o.end(), out);
        return (int64_t)o.size();
    } catch (const std::bad_alloc &) {
        return lc::fail(LC_E_NOMEM, "lc_report: out of memory");
    }
}

extern "C" int64_t lc_report(const lc_packed *p, int64_t key, int32_t valid, int32_t fail_event,
                             const uint64_t *final_configs, uint32_t n_final, int32_t max_paths, int64_t *out,
                             int64_t cap) {
    return report(p, key, valid, fail_event, final_configs, n_final, max_paths, false, out, cap);
}

extern "C" int64_t lc_report_wgl(const lc_packed *p, int64_t key, int32_t valid, int32_t fail_event,
                                 const uint64_t *final_configs, uint32_t n_final, int32_t max_paths, int64_t *out,
                                 int64_t cap) {
    return report(p, key, valid, fail_event, final_configs, n_final, max_paths, true, out, cap);
}

extern "C" int lc_packed_keys(const lc_packed *p, int64_t *out) {
    if (!p || (!out && !p->keys.empty())) return lc::fail(LC_E_INVALID, "lc_packed_keys: null argument");
    std::copy(p->keys.begin(), p->keys.end(), out);
    return LC_OK;
}
