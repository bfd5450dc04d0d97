// The packed batch lc_pack builds (library-owned; include/lincheck.h
// lc_packed): per-key event streams plus the maps back to history rows that
// result shaping (host_report.cpp) needs.  Host code only.
#pragma once

#include <algorithm>
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
    // skip_pre[w]: rows kept before skip word w within its key, so a lookup
    // is a binary search over the key's words (not a walk from its start)
    lc::uninit_vector<uint32_t> skip_pre;
    int64_t event_row(size_t key, uint64_t e) const {  // e: index into the event words
        if (!key_major) return ev_row[e];
        const uint64_t j = e - ev_off[key];
        const uint32_t *p0 = skip_pre.data() + skip_off[key], *p1 = skip_pre.data() + skip_off[key + 1];
        const uint32_t *at = std::upper_bound(p0, p1, (uint32_t)j) - 1;  // the last word starting at or before j
        const uint64_t w = (uint64_t)(at - p0);
        uint64_t x = ~skip[skip_off[key] + w];
        for (uint64_t i = *at; i < j; ++i) x &= x - 1;  // drop the kept rows before event j
        return key_row0[key] + (int64_t)(64 * w) + __builtin_ctzll(x);
    }
    // every event's row, key by key (one forward scan of each key's words)
    void event_rows(int64_t *out) const;
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
