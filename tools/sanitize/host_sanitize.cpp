// Host-code sanitizer driver ("Race detection /
// sanitizers"): the host half of liblincheck (history.edn and test.fressian
// readers/writers, lc_pack, lc_report, the synthetic generator) and the C
// oracle, built with -fsanitize=address,undefined (make asan) or
// -fsanitize=thread (make tsan) and driven over generated histories, round
// trips through history.edn and test.fressian, the parallel EDN split (files
// above 1 MB), mangled EDN text and Fressian bytes, and malformed op
// sequences.  Exit status 0 = every check passed and no sanitizer fired.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../include/lincheck.h"

extern "C" {
typedef struct oracle_key_result {
    int8_t valid;
    uint8_t cause;
    int32_t fail_event;
    uint32_t peak;
    uint64_t probes;
    uint64_t n_events;
} oracle_key_result;  // oracle/linear_ref.c
int64_t oracle_check_history_model(const lc_history *h, int model, uint64_t budget, int n_threads,
                                   int64_t *out_keys, oracle_key_result *out, int64_t max_keys);
}

static int failures = 0;
#define CHECK(c)                                                                   \
    do {                                                                           \
        if (!(c)) {                                                                \
            std::fprintf(stderr, "%s:%d: check failed: %s (%s)\n", __FILE__, __LINE__, #c, lc_last_error()); \
            ++failures;                                                            \
        }                                                                          \
    } while (0)

// pack, render every key's report, run the oracle; returns keys
static int64_t exercise(const lc_history &h, int model, const int64_t *init = nullptr, int32_t n_init = 0) {
    lc_pack_opts po{model, n_init, init};
    lc_packed *p = nullptr;
    if (lc_pack(&h, &po, &p) != LC_OK) return -1;
    lc_batch b;
    CHECK(lc_packed_view(p, &b) == LC_OK);
    std::vector<int64_t> keys((size_t)b.n_keys + 1);
    CHECK(lc_packed_keys(p, keys.data()) == LC_OK);
    std::vector<int64_t> rows;
    std::mt19937_64 rng(7);
    for (int64_t i = 0; i < b.n_keys; ++i) {
        const int64_t n = lc_packed_subhistory(p, i, nullptr);
        rows.resize((size_t)n + 1);
        CHECK(lc_packed_subhistory(p, i, rows.data()) == n);
        const uint64_t ne = b.ev_off[i + 1] - b.ev_off[i];
        for (uint64_t j = 0; j < ne; ++j) CHECK(lc_packed_event_row(p, i, (int64_t)j) >= 0);
        // reports with made-up final configs: any state id of the key, any slots
        uint64_t fin[2 * 10];
        uint32_t nf = (uint32_t)(rng() % 11);
        const uint32_t ns = b.key_states ? std::max<uint32_t>(b.key_states[i], 1) : 1;
        for (uint32_t c = 0; c < nf; ++c) {
            fin[2 * c] = rng();
            fin[2 * c + 1] = ((uint64_t)(rng() % ns) << 48) | (rng() & 0xFFFFFFull);
        }
        const int32_t fe = ne ? (int32_t)(rng() % ne) : -1;
        std::vector<int64_t> w(4096);
        for (int valid : {LC_VALID, LC_INVALID, LC_UNKNOWN}) {
            int64_t need = lc_report(p, i, valid, valid == LC_VALID ? -1 : fe, fin, nf, 10, w.data(), (int64_t)w.size());
            if (lc_packed_key_error(p, i)) { CHECK(need < 0); continue; }
            CHECK(need >= 4);
            if (model == LC_MODEL_MULTI_REGISTER && b.key_states[i] <= LC_WIDE_MAX_STATES) {
                // every map a state id stands for
                int64_t regs[64], vals[64];
                for (uint32_t st = 0; st < b.key_states[i]; ++st)
                    CHECK(lc_packed_state_map(p, i, st, regs, vals, 64) >= 0);
            }
            if (need > (int64_t)w.size()) {
                w.resize((size_t)need);
                CHECK(lc_report(p, i, valid, valid == LC_VALID ? -1 : fe, fin, nf, 10, w.data(), need) == need);
            }
        }
    }
    const int64_t nk = b.n_keys;
    lc_packed_free(p);
    if (model == LC_MODEL_MULTI_REGISTER) return nk;  // the C oracle has no table models
    int64_t ok = oracle_check_history_model(&h, model, 1 << 14, 4, nullptr, nullptr, 0);
    if (ok > 0) {
        std::vector<int64_t> ok_keys((size_t)ok);
        std::vector<oracle_key_result> res((size_t)ok);
        CHECK(oracle_check_history_model(&h, model, 1 << 14, 4, ok_keys.data(), res.data(), ok) == ok);
    }
    return nk;
}

static std::string slurp(const char *path) {
    std::string s;
    if (FILE *f = std::fopen(path, "rb")) {
        char buf[65536];
        size_t n;
        while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, n);
        std::fclose(f);
    }
    return s;
}

int main(int argc, char **argv) {
    const char *tmp = argc > 1 ? argv[1] : "/tmp/lc_sanitize_history.edn";
    struct Shape { int64_t keys, ops; int conc; double info, anomaly; int interleave; double nemesis; int values; };
    const Shape shapes[] = {
        {20, 200, 10, 0.0, 0.2, 1, 5.0, 5},     // C1-like: interleaved tuples + nemesis
        {40, 300, 14, 0.02, 0.1, 0, 0.0, 5},    // crashed ops (C4-like)
        {8, 400, 8, 0.01, 0.3, 1, 3.0, 3000},   // many register values: per-key tables
        {3000, 120, 10, 0.0, 0.05, 1, 5.0, 5},  // > 1 MB of EDN: the parallel split
    };
    for (const Shape &s : shapes) {
        lc_synth_opts o{};
        o.n_keys = s.keys; o.ops_per_key = s.ops; o.concurrency = s.conc; o.n_values = s.values;
        o.info_rate = s.info; o.info_effect_p = 0.5; o.anomaly_rate = s.anomaly; o.mean_think = 1.0;
        o.mean_latency = 1.0; o.interleave = s.interleave; o.nemesis_period = s.nemesis; o.seed = 11;
        lc_hist *h = nullptr;
        CHECK(lc_synth_generate(&o, &h) == LC_OK);
        if (!h) continue;
        lc_history v;
        CHECK(lc_hist_view(h, &v) == LC_OK);
        CHECK(exercise(v, LC_MODEL_CAS_REGISTER) == s.keys);
        CHECK(lc_edn_write(tmp, &v) == LC_OK);
        lc_hist *r = nullptr;
        CHECK(lc_edn_read(tmp, &r) == LC_OK);
        if (r) {
            lc_history rv;
            CHECK(lc_hist_view(r, &rv) == LC_OK);
            CHECK(rv.n == v.n);
            for (int64_t i = 0; i < v.n && i < rv.n; ++i)
                CHECK(rv.type[i] == v.type[i] && rv.key[i] == v.key[i] && rv.v0[i] == v.v0[i] &&
                      rv.v1[i] == v.v1[i] && rv.process[i] == v.process[i]);
            lc_hist_free(r);
        }
        // the same text, mangled: truncated at many points and with bytes flipped
        const std::string text = slurp(tmp);
        std::mt19937_64 rng(s.keys);
        for (int t = 0; t < 40 && !text.empty(); ++t) {
            std::string m = text.substr(0, (size_t)(rng() % text.size()));
            for (int k = 0; k < 8 && !m.empty(); ++k) m[(size_t)(rng() % m.size())] = (char)(rng() & 0xFF);
            lc_hist *x = nullptr;
            if (lc_edn_parse(m.data(), (int64_t)m.size(), &x) == LC_OK && x) {
                lc_history xv;
                lc_hist_view(x, &xv);
                exercise(xv, LC_MODEL_CAS_REGISTER);  // may hold malformed op sequences: errors, not faults
                lc_hist_free(x);
            }
        }
        // the same history through test.fressian, then its bytes mangled
        const std::string ftmp = std::string(tmp) + ".fressian";
        CHECK(lc_fressian_write(ftmp.c_str(), &v) == LC_OK);
        r = nullptr;
        CHECK(lc_fressian_read(ftmp.c_str(), &r) == LC_OK);
        if (r) {
            lc_history rv;
            CHECK(lc_hist_view(r, &rv) == LC_OK);
            CHECK(rv.n == v.n);
            for (int64_t i = 0; i < v.n && i < rv.n; ++i)
                CHECK(rv.type[i] == v.type[i] && rv.key[i] == v.key[i] && rv.v0[i] == v.v0[i] &&
                      rv.v1[i] == v.v1[i] && rv.process[i] == v.process[i] && rv.index[i] == v.index[i]);
            lc_hist_free(r);
        }
        const std::string bin = slurp(ftmp.c_str());
        for (int t = 0; t < 40 && !bin.empty(); ++t) {
            std::string m = bin.substr(0, (size_t)(rng() % bin.size()));
            for (int k = 0; k < 8 && !m.empty(); ++k) m[(size_t)(rng() % m.size())] = (char)(rng() & 0xFF);
            lc_hist *x = nullptr;
            if (lc_fressian_parse((const uint8_t *)m.data(), (int64_t)m.size(), &x) == LC_OK && x) {
                lc_history xv;
                lc_hist_view(x, &xv);
                exercise(xv, LC_MODEL_CAS_REGISTER);
                lc_hist_free(x);
            }
        }
        // footers where they do not belong: inside a closed list (refused, no
        // loop), after an open list of op maps (the list ends there)
        {
            const uint8_t closed_footer[] = {0xED, 0xCF};
            lc_hist *x = nullptr;
            CHECK(lc_fressian_parse(closed_footer, 2, &x) != LC_OK && !x);
            const uint8_t counted_footer[] = {0xE6, 0x01, 0xCF, 0xCF, 0xCF, 0xCF};
            CHECK(lc_fressian_parse(counted_footer, 6, &x) != LC_OK && !x);
            const uint8_t open_footer[] = {0xEE, 0xCF, 0xCF, 0xCF, 0xCF, 0, 0, 0, 1, 0, 0, 0, 0};
            CHECK(lc_fressian_parse(open_footer, (int64_t)sizeof open_footer, &x) == LC_OK && x);
            if (x) lc_hist_free(x);
        }
        lc_hist_free(h);
    }
    // :txn histories in EDN (multi-register): parsed, packed, and mangled
    {
        std::string txt;
        std::mt19937_64 rng(9);
        const char *regs[] = {":x", ":y", "3", "\"z\""};
        for (int i = 0; i < 400; ++i) {
            const int k = (int)(rng() % 4), p = (int)(rng() % 5);
            std::string v = "[";
            for (int m = 0, nm = 1 + (int)(rng() % 3); m < nm; ++m) {
                v += (rng() & 1) ? "[:read " : "[:w ";
                v += regs[rng() % 4];
                v += (rng() % 3) ? " " + std::to_string(rng() % 4) + "]" : " nil]";
            }
            v += "]";
            for (const char *t : {"invoke", "ok"})
                txt += std::string("{:type :") + t + ", :f :txn, :value [" + std::to_string(k) + " " + v +
                       "], :process " + std::to_string(p) + ", :index " + std::to_string(i) + "}\n";
        }
        lc_hist *x = nullptr;
        CHECK(lc_edn_parse(txt.data(), (int64_t)txt.size(), &x) == LC_OK);
        if (x) {
            lc_history xv;
            lc_hist_view(x, &xv);
            CHECK(xv.mop_off != nullptr && lc_hist_n_reg_names(x) == 3);
            exercise(xv, LC_MODEL_MULTI_REGISTER);
            lc_hist_free(x);
        }
        for (int t = 0; t < 60; ++t) {
            std::string m = txt.substr(0, (size_t)(rng() % txt.size()));
            for (int k = 0; k < 8 && !m.empty(); ++k) m[(size_t)(rng() % m.size())] = (char)(rng() & 0xFF);
            x = nullptr;
            if (lc_edn_parse(m.data(), (int64_t)m.size(), &x) == LC_OK && x) {
                lc_history mv;
                lc_hist_view(x, &mv);
                exercise(mv, LC_MODEL_MULTI_REGISTER);
                lc_hist_free(x);
            }
        }
    }
    // random op sequences over three processes and two keys: completions
    // without invocations, double invokes, unknown :f codes, :txn rows with
    // random (and malformed) micro-ops for (model/multi-register)
    std::mt19937_64 rng(3);
    for (int t = 0; t < 2000; ++t) {
        const int n = 1 + (int)(rng() % 24);
        std::vector<uint8_t> ty(n), f(n);
        std::vector<int64_t> pr(n), key(n), v0(n), v1(n), idx(n), mop_off(n + 1, 0), mop;
        for (int i = 0; i < n; ++i) {
            ty[i] = (uint8_t)(rng() % 4); f[i] = (uint8_t)(rng() % 7);
            pr[i] = (int64_t)(rng() % 3); key[i] = (rng() % 5) ? (int64_t)(rng() % 2) : LC_NO_KEY;
            v0[i] = (rng() % 4) ? (int64_t)(rng() % 3) : LC_NIL; v1[i] = (int64_t)(rng() % 3); idx[i] = i;
            const int nm = f[i] == LC_F_TXN ? (int)(rng() % 4) : 0;
            for (int m = 0; m < nm; ++m) {
                mop.push_back((rng() % 50) ? (int64_t)(rng() % 2) : 7);  // an unknown micro-op now and then
                mop.push_back((int64_t)(rng() % 3));
                mop.push_back((rng() % 4) ? (int64_t)(rng() % 3) : LC_NIL);
            }
            mop_off[i + 1] = (int64_t)mop.size() / 3;
        }
        mop.push_back(0);
        lc_history h{n, ty.data(), f.data(), pr.data(), key.data(), v0.data(), v1.data(), idx.data(),
                     mop_off.data(), mop.data()};
        for (int model : {LC_MODEL_CAS_REGISTER, LC_MODEL_REGISTER, LC_MODEL_MUTEX, LC_MODEL_MULTI_REGISTER})
            exercise(h, model);
        const int64_t init[4] = {0, 1, 2, LC_NIL};
        exercise(h, LC_MODEL_MULTI_REGISTER, init, 2);
    }
    std::remove(tmp);
    std::printf("host sanitizer driver: %d failed checks\n", failures);
    return failures ? 1 : 0;
}
