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
    lc::pinned_vector<uint32_t> events;
    lc::pinned_vector<uint16_t> events16;  // the same words in 16 bits when all fit (empty otherwise)
    lc::uninit_vector<int64_t> ev_row;
    std::vector<uint32_t> trans;
    std::vector<uint32_t> trans_off;  // empty = shared table
    std::vector<uint8_t> key_width;
    std::vector<uint16_t> key_states;
    // sub-history rows: per-key rows + rows shared by every key
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
