// Shared host-side plumbing for liblincheck: error reporting and owned
// history storage.  Host code only (no device code in this header).
#pragma once

#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/lincheck.h"

namespace lc {

// Thread-local last error (lc_last_error).  Every failing entry point sets it.
void set_error(const std::string &msg);
int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

}  // namespace lc

// Owned history: the storage behind lc_synth_generate / lc_edn_read.
struct lc_hist {
    std::vector<uint8_t> type, f;
    std::vector<int64_t> process, key, v0, v1, index;
    std::vector<int64_t> anomalous_keys;

    void reserve(size_t n) {
        type.reserve(n); f.reserve(n); process.reserve(n); key.reserve(n);
        v0.reserve(n); v1.reserve(n); index.reserve(n);
    }
    void push(uint8_t t, uint8_t fn, int64_t p, int64_t k, int64_t a, int64_t b, int64_t idx) {
        type.push_back(t); f.push_back(fn); process.push_back(p); key.push_back(k);
        v0.push_back(a); v1.push_back(b); index.push_back(idx);
    }
    int64_t size() const { return (int64_t)type.size(); }
    lc_history view() const {
        lc_history h;
        h.n = size();
        h.type = type.data(); h.f = f.data(); h.process = process.data(); h.key = key.data();
        h.v0 = v0.data(); h.v1 = v1.data(); h.index = index.data();
        return h;
    }
};
