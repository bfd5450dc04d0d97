// Synthetic cas-register histories with the etcd demo's shape.
//
// What the reference fixes and this generator reproduces:
//   - ops: read nil / write (rand-int 5) / cas [(rand-int 5) (rand-int 5)]
//     picked uniformly (gen/mix [r w cas])            etcdemo.clj:67-69, :124
//   - ops per key bounded by gen/limit                 etcdemo.clj:125
//   - `concurrency` client threads per key             etcdemo.clj:120-121
//   - outcomes: read :ok with the value read (nil when never written),
//     write :ok, cas :ok / :fail on mismatch; a timed-out write/cas is :info,
//     and a crashed process is replaced by process + concurrency
//                                                      etcdemo.clj:83-105
//   - independent tuples [k v] on every client op      etcdemo.clj:90, :120
//   - nemesis :info :start / :stop on a fixed period   etcdemo.clj:138-143
//
// Every op gets a linearization point uniform in [invoke, complete] and is
// applied to a ground-truth register in that order, so a history without
// injected anomalies is linearizable by construction.  Anomalies (C5): one
// stale read (returns the value a completed newer write overwrote) or one
// lost cas (reported :ok, effect not applied) per corrupted key.
//
// Deterministic: xoshiro256** seeded per key from (seed, key id), so any key
// range can be generated independently (sharding, tests).

#include <algorithm>
#include <cmath>
#include <cstring>
#include <thread>

#include "common.hpp"

namespace {

struct Rng {
    uint64_t s[4];
    static uint64_t splitmix(uint64_t &x) {
        uint64_t z = (x += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    Rng(uint64_t seed, uint64_t stream) {
        uint64_t x = seed * 0xD1B54A32D192ED03ull ^ (stream + 0x632BE59BD9B4E019ull);
        for (auto &w : s) w = splitmix(x);
    }
    static uint64_t rotl(uint64_t v, int k) { return (v << k) | (v >> (64 - k)); }
    uint64_t next() {
        uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
        s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
        return r;
    }
    double u01() { return (double)((next() >> 11) + 1) * (1.0 / 9007199254740992.0); }  // (0, 1]
    double expo(double mean) { return -std::log(u01()) * mean; }
    int64_t below(int64_t n) { return (int64_t)(next() % (uint64_t)n); }
};

struct SOp {
    double t_inv, t_done, t_lin;
    uint8_t f;        // LC_F_*
    int64_t v0, v1;   // write value / cas old,new
    int64_t process;
    bool crash, applied;
    uint8_t outcome;  // LC_OK_T / LC_FAIL / LC_INFO
    int64_t read_val;
};

struct Row { double t; int seq; uint8_t type, f; int64_t p, v0, v1; };

// Simulate one key.  proc[] holds each thread's current process id and is
// advanced past crashes (Jepsen: a crashed process p is replaced by p + c).
void simulate_key(const lc_synth_opts &o, int64_t key, std::vector<int64_t> &proc,
                  std::vector<Row> &rows, bool &anomalous) {
    Rng rng(o.seed, (uint64_t)key);
    const int c = o.concurrency;
    const int64_t nv = o.n_values > 0 ? o.n_values : 5;
    std::vector<double> next_t(c);
    for (int t = 0; t < c; ++t) next_t[t] = rng.expo(o.mean_think);

    std::vector<SOp> ops((size_t)o.ops_per_key);
    for (int64_t i = 0; i < o.ops_per_key; ++i) {
        int th = 0;
        for (int t = 1; t < c; ++t) if (next_t[t] < next_t[th]) th = t;
        SOp &op = ops[(size_t)i];
        op.t_inv = next_t[th];
        double d = rng.expo(o.mean_latency);
        op.t_done = op.t_inv + d;
        op.t_lin = op.t_inv + rng.u01() * d;
        int fsel = (int)rng.below(3);
        op.f = fsel == 0 ? LC_F_READ : fsel == 1 ? LC_F_WRITE : LC_F_CAS;
        op.v0 = op.v1 = LC_NIL;
        if (op.f == LC_F_WRITE) op.v0 = rng.below(nv);
        if (op.f == LC_F_CAS) { op.v0 = rng.below(nv); op.v1 = rng.below(nv); }
        op.process = proc[th];
        op.crash = op.f != LC_F_READ && o.info_rate > 0 && rng.u01() <= o.info_rate;
        op.applied = !op.crash || rng.u01() <= o.info_effect_p;
        op.read_val = LC_NIL;
        next_t[th] = op.t_done + rng.expo(o.mean_think);
        if (op.crash) proc[th] += c;
    }

    // Anomaly selection (C5): decided before the ground truth runs.
    anomalous = o.anomaly_rate > 0 && rng.u01() <= o.anomaly_rate;
    bool want_stale = anomalous && (rng.next() & 1);
    int64_t lost_cas = -1;
    if (anomalous && !want_stale) {
        std::vector<int64_t> cands;
        for (int64_t i = 0; i < o.ops_per_key; ++i)
            if (ops[(size_t)i].f == LC_F_CAS && !ops[(size_t)i].crash) cands.push_back(i);
        if (cands.empty()) want_stale = true; else lost_cas = cands[(size_t)rng.below((int64_t)cands.size())];
    }

    // Ground truth in linearization-point order.
    std::vector<int64_t> order((size_t)o.ops_per_key);
    for (int64_t i = 0; i < o.ops_per_key; ++i) order[(size_t)i] = i;
    std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
        return ops[(size_t)a].t_lin < ops[(size_t)b].t_lin || (ops[(size_t)a].t_lin == ops[(size_t)b].t_lin && a < b);
    });
    struct Change { int64_t op; int64_t before; };
    std::vector<Change> changes;  // register changes in lin order
    int64_t reg = LC_NIL;
    for (int64_t i : order) {
        SOp &op = ops[(size_t)i];
        if (op.f == LC_F_READ) { op.read_val = reg; op.outcome = LC_OK_T; continue; }
        if (op.f == LC_F_WRITE) {
            op.outcome = op.crash ? LC_INFO : LC_OK_T;
            if (op.applied) { changes.push_back({i, reg}); reg = op.v0; }
            continue;
        }
        bool match = reg == op.v0;
        if (i == lost_cas) { op.outcome = LC_OK_T; continue; }  // claims success, no effect
        op.outcome = op.crash ? LC_INFO : (match ? LC_OK_T : LC_FAIL);
        if (match && op.applied) { changes.push_back({i, reg}); reg = op.v1; }
    }
    if (want_stale) {
        // A read that starts after some change completed returns the value that
        // change overwrote (when it differs from what the read saw).
        std::vector<int64_t> reads;
        for (int64_t i = 0; i < o.ops_per_key; ++i) if (ops[(size_t)i].f == LC_F_READ) reads.push_back(i);
        for (int tries = 0; tries < 16 && !reads.empty(); ++tries) {
            SOp &r = ops[(size_t)reads[(size_t)rng.below((int64_t)reads.size())]];
            const Change *best = nullptr;
            for (const Change &ch : changes)
                if (ops[(size_t)ch.op].t_done < r.t_inv &&
                    (!best || ops[(size_t)ch.op].t_lin > ops[(size_t)best->op].t_lin)) best = &ch;
            if (best && best->before != r.read_val) { r.read_val = best->before; break; }
        }
    }

    rows.clear();
    rows.reserve((size_t)o.ops_per_key * 2);
    int seq = 0;
    for (const SOp &op : ops) {
        int64_t iv0 = op.f == LC_F_READ ? LC_NIL : op.v0;
        rows.push_back({op.t_inv, seq++, LC_INVOKE, op.f, op.process, iv0, op.v1});
        int64_t cv0 = op.f == LC_F_READ ? op.read_val : op.v0;
        rows.push_back({op.t_done, seq++, op.outcome, op.f, op.process, cv0, op.v1});
    }
    std::stable_sort(rows.begin(), rows.end(), [](const Row &a, const Row &b) {
        return a.t < b.t || (a.t == b.t && a.seq < b.seq);
    });
}

}  // namespace

extern "C" int lc_synth_generate(const lc_synth_opts *o, lc_hist **out) {
    if (!o || !out) return lc::fail(LC_E_INVALID, "lc_synth_generate: null argument");
    if (o->n_keys < 0 || o->ops_per_key < 0 || o->concurrency <= 0 || o->concurrency > 4096)
        return lc::fail(LC_E_INVALID, "lc_synth_generate: bad sizes");
    if (o->mean_think <= 0 || o->mean_latency <= 0)
        return lc::fail(LC_E_INVALID, "lc_synth_generate: mean_think/mean_latency must be > 0");
    lc_hist *h = new (std::nothrow) lc_hist();
    if (!h) return lc::fail(LC_E_NOMEM, "lc_synth_generate: out of memory");
    const int64_t K = o->n_keys;
    try {
        if (!o->interleave) {
            // Key-major: keys are independent; generate in parallel, concatenate in order.
            unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
            std::vector<std::vector<Row>> per((size_t)K);
            std::vector<uint8_t> anom((size_t)K, 0);
            auto work = [&](unsigned t) {
                std::vector<int64_t> proc((size_t)o->concurrency);
                for (int64_t k = t; k < K; k += nt) {
                    for (int i = 0; i < o->concurrency; ++i) proc[(size_t)i] = i;
                    bool a = false;
                    simulate_key(*o, o->key_base + k, proc, per[(size_t)k], a);
                    anom[(size_t)k] = a;
                }
            };
            lc::run_threads(nt, work);
            // concatenation: every key's rows at its offset, in parallel
            std::vector<int64_t> off((size_t)K + 1, 0);
            for (int64_t k = 0; k < K; ++k) off[(size_t)k + 1] = off[(size_t)k] + (int64_t)per[(size_t)k].size();
            const size_t n = (size_t)off[(size_t)K];
            h->type.resize(n); h->f.resize(n); h->process.resize(n); h->key.resize(n);
            h->v0.resize(n); h->v1.resize(n); h->index.resize(n);
            auto fill = [&](unsigned t) {
                for (int64_t k = t; k < K; k += nt) {
                    size_t i = (size_t)off[(size_t)k];
                    for (const Row &r : per[(size_t)k]) {
                        h->type[i] = r.type; h->f[i] = r.f; h->process[i] = r.p; h->key[i] = o->key_base + k;
                        h->v0[i] = r.v0; h->v1[i] = r.v1; h->index[i] = (int64_t)i;
                        ++i;
                    }
                    std::vector<Row>().swap(per[(size_t)k]);
                }
            };
            lc::run_threads(nt, fill);
            for (int64_t k = 0; k < K; ++k)
                if (anom[(size_t)k]) h->anomalous_keys.push_back(o->key_base + k);
        } else {
            // One Jepsen-style history: a single thread group works through the
            // keys in sequence (independent/concurrent-generator), process ids
            // carry across keys, nemesis :info ops interleave on a fixed period.
            h->reserve((size_t)(K * o->ops_per_key * 2 + 16));
            std::vector<int64_t> proc((size_t)o->concurrency);
            for (int i = 0; i < o->concurrency; ++i) proc[(size_t)i] = i;
            struct GRow { double t; int64_t seq; uint8_t type, f; int64_t p, k, v0, v1; };
            std::vector<GRow> all;
            std::vector<Row> rows;
            double t0 = 0;
            int64_t seq = 0;
            for (int64_t k = 0; k < K; ++k) {
                bool a = false;
                simulate_key(*o, o->key_base + k, proc, rows, a);
                if (a) h->anomalous_keys.push_back(o->key_base + k);
                double tmax = t0;
                for (const Row &r : rows) {
                    all.push_back({t0 + r.t, seq++, r.type, r.f, r.p, o->key_base + k, r.v0, r.v1});
                    tmax = std::max(tmax, t0 + r.t);
                }
                t0 = tmax;
            }
            if (o->nemesis_period > 0) {
                bool start = true;
                for (double t = o->nemesis_period; t < t0; t += o->nemesis_period, start = !start) {
                    // invoke + completion, both :info from the :nemesis process
                    all.push_back({t, seq++, LC_INFO, LC_F_OTHER, LC_NO_PROCESS, LC_NO_KEY, start ? 1 : 0, LC_NIL});
                    all.push_back({t + 1e-3, seq++, LC_INFO, LC_F_OTHER, LC_NO_PROCESS, LC_NO_KEY, start ? 1 : 0, LC_NIL});
                }
            }
            std::stable_sort(all.begin(), all.end(), [](const GRow &a, const GRow &b) {
                return a.t < b.t || (a.t == b.t && a.seq < b.seq);
            });
            int64_t idx = 0;
            for (const GRow &r : all) h->push(r.type, r.f, r.p, r.k, r.v0, r.v1, idx++);
        }
    } catch (const std::bad_alloc &) {
        delete h;
        return lc::fail(LC_E_NOMEM, "lc_synth_generate: out of memory");
    }
    *out = h;
    return LC_OK;
}

extern "C" int lc_hist_view(const lc_hist *h, lc_history *out) {
    if (!h || !out) return lc::fail(LC_E_INVALID, "lc_hist_view: null argument");
    *out = h->view();
    return LC_OK;
}

extern "C" int64_t lc_hist_anomalous_keys(const lc_hist *h, int64_t *out_keys) {
    if (!h) return lc::fail(LC_E_INVALID, "lc_hist_anomalous_keys: null argument");
    if (out_keys) std::memcpy(out_keys, h->anomalous_keys.data(), h->anomalous_keys.size() * sizeof(int64_t));
    return (int64_t)h->anomalous_keys.size();
}

extern "C" void lc_hist_free(lc_hist *h) { delete h; }

extern "C" int64_t lc_hist_n_reg_names(const lc_hist *h) {
    if (!h) return lc::fail(LC_E_INVALID, "lc_hist_n_reg_names: null argument");
    return (int64_t)h->reg_names.size();
}

extern "C" const char *lc_hist_reg_name(const lc_hist *h, int64_t i) {
    if (!h || i < 0 || (uint64_t)i >= h->reg_names.size()) return nullptr;
    return h->reg_names[(size_t)i].c_str();
}
