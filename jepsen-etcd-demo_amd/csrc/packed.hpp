// The packed batch lc_pack builds (library-owned; include/lincheck.h
// lc_packed): per-key event streams plus the maps back to history rows that
// result shaping (host_report.cpp) needs.  Host code only.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "common.hpp"

struct lc_packed {
    std::vector<int64_t> keys;
    lc::pinned_vector<uint64_t> ev_off;  // page-locked on a GPU host: lc_check_* DMA it directly
    // the event words, page-locked for the device; left out (empty) when
    // the 16-bit form below is given (the device widens it; word() here)
    lc::host_array<uint32_t> events;
    // the same words in 16 bits when all fit (empty otherwise), page-locked
    lc::host_array<uint16_t> events16;
    uint32_t word(uint64_t e) const { return events.empty() ? LC_EV16_WIDE(events16[e]) : events[e]; }
    // history row of each event: ev_row (the bucketing path), or, when every
    // key's rows are one run of the history (key_major), a bitmap of the
    // key's rows that emit no event (skip, from word skip_off[key]): event j
    // of key k is the j-th row of its run without a skip bit
    lc::uninit_vector<int64_t> ev_row;
    lc::host_array<uint64_t> skip;
    std::vector<uint64_t> skip_off;
    std::vector<int64_t> key_row0;
    bool key_major = false;
    int64_t event_row(size_t key, uint64_t e) const {  // e: index into the event words
        if (!key_major) return ev_row[e];
        uint64_t j = e - ev_off[key];
        const uint64_t *w = skip.data() + skip_off[key];
        for (int64_t base = 0;; base += 64, ++w) {
            const uint64_t keep = ~*w;
            const uint64_t c = (uint64_t)__builtin_popcountll(keep);
            if (j < c) {
                uint64_t x = keep;
                for (uint64_t i = 0; i < j; ++i) x &= x - 1;  // drop the j lowest kept rows
                return key_row0[key] + base + __builtin_ctzll(x);
            }
            j -= c;
        }
    }
    std::vector<uint32_t> trans;
    std::vector<uint32_t> trans_off;  // empty = shared table
    std::vector<uint8_t> key_width;
    std::vector<uint16_t> key_states;
    // sub-history rows: per-key rows + rows shared by every key (key_major:
    // krows empty, key k's rows are key_row0[k] + [0, krow_off[k+1] - krow_off[k]))
    std::vector<uint64_t> krow_off;
    lc::uninit_vector<int64_t> krows;
    std::vector<int64_t> shared_rows;
    // state id -> register value: shared table, or per key (state_off[k] ..)
    std::vector<int64_t> state_vals;  // index 0 unused (nil)
    std::vector<uint64_t> state_off;  // empty = shared
    // keys that could not be prepared (A9): empty = none
    std::vector<uint8_t> key_error;
    std::vector<std::string> key_msg;
    int32_t model = LC_MODEL_CAS_REGISTER;
    // (model/multi-register): the transition table (lc_batch.table) and, per
    // key, its registers and the map each state id stands for
    std::vector<uint16_t> table;
    std::vector<uint64_t> mr_reg_off, mr_state_off;  // [K + 1]
    std::vector<int64_t> mr_regs, mr_states;
};
