// Kernel argument block and launchers shared by device_search.hip and the
// host orchestration in device_api.hip.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace lcd {

struct Args {
    // packed batch (device pointers; include/lincheck.h lc_batch)
    const uint64_t *ev_off;
    const uint32_t *events;
    const uint32_t *trans;
    const uint32_t *trans_off;   // may be null
    const uint8_t *key_width;    // may be null
    const uint16_t *key_states;  // may be null
    const uint8_t *key_error;    // may be null: nonzero = :unknown (LC_CAUSE_ERROR), not searched
    const uint16_t *table;       // may be null: a table model's rows (lc_batch.table); trans[] are row offsets
    uint32_t init_state;
    uint32_t shared_states;      // state ids used by the shared table (trans_off == null)
    uint64_t budget;
    int32_t max_final;
    int32_t debug_mode;          // 0; ablation builds only (lc_opts.debug_mode)
    int32_t count_probes;        // lc_opts.flags & LC_OPT_COUNT_PROBES
    // work list of this launch: keys order[0 .. n) with n = n_in ? *n_in : n_order
    const int32_t *order;
    int32_t n_order;
    const int32_t *n_in;
    int32_t *ticket;         // zeroed before the launch
    int32_t *err;            // T0: [0] LC_BATCH_E_* bits, [1] 1 + largest malformed key
    uint32_t n_trans;        // entries of trans[]
    int32_t strict;          // T0: the host did not validate the events (T0_STRICT)
    int32_t err_base;        // added to a malformed key's index in err[1]: the launch's
                             // first key in the caller's batch (a chunk or shard of it)
    // per-key results (device pointers)
    int8_t *valid;
    int32_t *fail_event;
    uint8_t *cause;
    uint32_t *peak;          // may be null
    uint64_t *final_cfg;     // may be null: [key][max_final][2]
    uint32_t *n_final;       // may be null
    uint64_t *rec;           // may be null: the key's verdict record (LC_REC_*) is written here too
    uint32_t *lat_ws;            // T0 workspace: lat_ws_words() per resident block
    // counters
    unsigned long long *probes;
    unsigned long long *ev_count;
    unsigned long long *keys_done;
    unsigned long long *stream_bytes;  // layered HBM tier: set-array bytes streamed
    // output work lists
    int32_t *spill;
    int32_t *n_spill;
    int32_t *wide;
    int32_t *n_wide;
    // T0 only: keys wider than LC_DIRECT_T3_WIDTH skip the LDS tiers (their
    // sets outgrow them; every tier computes the same sets, so this is
    // routing, not semantics) and go straight to the HBM tier's list
    int32_t *deep;
    int32_t *n_deep;
    int32_t list_cap;        // entries of each work list above
};

// Malformed-batch reasons T0 reports when it validates a batch itself.
constexpr int32_t LC_BATCH_E_SLOTS = 1;  // :ok of a slot with no pending op / :invoke into an occupied slot
constexpr int32_t LC_BATCH_E_TRANS = 2;  // transition id out of range / installs a state the key lacks
constexpr int32_t LC_BATCH_E_FIT = 4;    // a key declared to fit T0 (width, states) does not

// Ops pending at once above which a key leaving T0 goes straight to T3.
constexpr uint32_t LC_DIRECT_T3_WIDTH = 28;

// The speculative segments' 8-wave build (k_spec<8, 8>, device_lattice.hip)
// held to 8 waves per SIMD -- 64 VGPRs, the rest spilled -- so a batch of up
// to 1,024 keys (C2, C5) has all 8 walks of every key resident at once: the
// launch chooses 8 segments per key there instead of 4 (round 5, C2
// 0.2488 -> 0.2415 ms per resident step).  1 = no bound (then 8 segments
// only for batches of <= 512 keys, where 8 x keys waves fit at 4 per SIMD).
#ifndef LC_SPEC8_WAVES
#define LC_SPEC8_WAVES 8
#endif

// Per-block HBM workspace of the T3 tier (one slot per resident block).
struct HbmWs {
    char *base;
    size_t slot_bytes;
    uint32_t cap;    // array capacity per set (budget + block + margin)
    uint32_t hmask;  // hash slots - 1
    size_t off_S0, off_S1, off_I, off_hS, off_hI, off_pS0, off_pS1, off_pI;
};

size_t lds_bytes_t1();
size_t lds_bytes_t2();
hipError_t launch_t0(const Args &a, const Args *a_dev, int grid, bool wide, hipStream_t s, uint32_t ticket_base);
size_t lat_ws_words();
// The batch's event-by-event validation (err words), a kernel of its own for
// a second stream: T0_STRICT steps (general = false: a register-tier batch),
// or any batch the host did not walk (general = true: every width; the later
// tiers read the err words first and do nothing over a malformed batch)
hipError_t launch_validate(const Args &a, hipStream_t s, bool general);

// Key segments (device_lattice.hip, "Key segments"): a register-tier step
// whose keys are cut at quiescent points and searched as independent
// segments, then composed per key.  Device arrays of seg_cap entries each
// (seg_cap = n_keys * max_seg), sized by the host.
struct SegArgs {
    const uint64_t *ev_off;
    const uint32_t *events;
    const uint32_t *trans;       // the shared table (segments need it)
    const uint8_t *key_error;    // may be null
    uint32_t n_trans;
    int32_t n_keys;
    uint32_t seg_len;            // cut at the first quiescent point this far past the last cut
    uint32_t max_seg;            // segments per key at most
    uint32_t *seg_cnt;           // [n_keys]
    uint32_t *seg_end;           // [n_keys * max_seg] end event (exclusive) of each segment
    uint32_t *seg_out;           // [n_keys * max_seg] final word (0: every start dead)
    int32_t *seg0_fev;           // [n_keys] failing event of segment 0 (searched exactly)
    uint32_t *work;              // [n_keys * max_seg] key << 8 | segment
    uint32_t *rerun;             // [n_keys] key << 8 | segment, then its start states
    uint32_t *rerun_init;        // [n_keys]
    int32_t *ctl;                // [0] work items, [1] search ticket, [2] reruns, [3] rerun ticket
    int32_t *err;                // T0_STRICT error words (a key that does not fit)
    int8_t *valid;
    int32_t *fail_event;
    uint8_t *cause;
    uint64_t *rec;               // may be null: LC_REC_* records (Args::rec)
    int32_t strict;
    int32_t err_base;            // as Args::err_base
};
constexpr uint32_t SEG_MAX = 256;  // work items are key << 8 | segment
hipError_t launch_segments(const SegArgs &a, int grid, hipStream_t s);
// Speculative key segments (device_lattice.hip): keys order[0 .. n_order) of
// a verdicts-only register-tier step, each a workgroup of `segs` waves (2, 3,
// 4, 6, 8) searching segments from the full set and checking them against
// each other, then a launch for the keys left to the unsegmented search;
// results through a_dev like launch_t0.  rr: n_order + 2 ints of scratch
// (both counts zero before the first launch; `parity` alternates).
// validate_blocks > 0: the T0_STRICT validation runs in that many extra blocks.
size_t spec_ws_words(int64_t n_keys, int segs);
// events16: the batch's 16-bit event words (read in place), or null (the
// 32-bit words); cost_cuts: cuts at equal estimated cost instead of equal
// event counts;
// prio: TOP walks' issue priority by progress (s_setprio).
size_t spec_fin_words(int64_t n_keys, int segs);
hipError_t launch_spec(const Args &a, const Args *a_dev, int segs, int waves, uint32_t *ws, int32_t *rr, int parity,
                       uint32_t ck1, uint32_t ck2, int rerun_grid, int validate_blocks, const uint16_t *events16,
                       bool cost_cuts, bool prio, bool vfirst, uint32_t *fin, bool stage, hipStream_t s);
uint32_t t0_max_width();   // most ops pending at once that T0 holds
uint32_t t0_max_states();  // most register states T0 holds
hipError_t launch_t1(const Args &a, int grid, hipStream_t s);
hipError_t launch_t2(const Args &a, int grid, hipStream_t s);
// Layered HBM tier (device_layers.hip): per-block arrays S[2], I[2] of cap
// entries (u64 each), one 1,024-thread block per key.  Keys with more than 8
// states go to a.spill (the config-keyed narrow tier), wide ones to a.wide.
struct LayWs {
    char *base;
    size_t slot_bytes;
    uint32_t cap;    // entries per array (budget + t3l_slack() + margin)
    size_t off_S0, off_S1, off_I0, off_I1;
};
hipError_t launch_t3_layers(const Args &a, const LayWs &w, int grid, hipStream_t s);
int t3l_slack();
hipError_t launch_t3_narrow(const Args &a, const HbmWs &w, int grid, hipStream_t s);
hipError_t launch_t3_wide(const Args &a, const HbmWs &w, int grid, hipStream_t s);
int t3_block();
size_t cfg_bytes_narrow();
size_t cfg_bytes_wide();

// knossos.wgl on the device (device_wgl.hip): one wave per key walks the
// Wing & Gong search with Lowe's cache in HBM.  Per resident wave a slot of
// slot_bytes: the cache table (tab_mask + 1 entries of 32 B), the frame
// stack, the per-event slot history.
struct WglWs {
    char *base;
    size_t slot_bytes;
    uint32_t tab_mask;
    size_t off_frames, off_prev;
    bool same_layout(const WglWs &o) const {
        return slot_bytes == o.slot_bytes && tab_mask == o.tab_mask && off_frames == o.off_frames && off_prev == o.off_prev;
    }
};
struct WglArgs {
    const uint64_t *ev_off;
    const uint32_t *events;
    const uint32_t *trans;
    const uint32_t *trans_off;   // may be null
    const uint16_t *key_states;  // may be null
    const uint8_t *key_error;    // may be null
    const uint16_t *table;       // may be null: a table model's rows
    uint32_t init_state;
    uint32_t n_trans;
    uint64_t budget;             // Lowe's cache holds at most this many pairs
    int32_t max_final;
    uint32_t lds_events;         // events (and their slot history) per key kept in LDS
    uint32_t lds_tab;            // entries of the LDS tier of Lowe's cache (power of 2; 0: none)
    const uint8_t *key_width;    // may be null (then no key takes the LDS tier)
    const int32_t *order;        // keys order[0 .. n) with n = n_in ? *n_in : n_order
    int32_t n_order;
    const int32_t *n_in;
    int32_t *ticket;             // zeroed before the launch
    const int32_t *err;          // validation error words: a refused batch is not searched
    uint64_t gen_base;           // launch << 32: a table entry is the key's when its stamp is gen_base | ticket + 1
    uint32_t spill_at;           // > 0: a key whose cache would pass this many pairs goes to spill (a larger table)
    int32_t *spill;
    int32_t *n_spill;
    WglWs ws;
    int8_t *valid;
    int32_t *fail_event;
    uint8_t *cause;
    uint32_t *peak;              // may be null: the cache size at the end
    uint64_t *final_cfg;         // may be null: the frontier at the stuck :ok (first max_final, walk order)
    uint32_t *n_final;           // may be null
    uint8_t *analyzer;           // may be null: LC_ALGO_WGL written for every key searched here
    uint64_t *rec;               // may be null: LC_REC_* records
    unsigned long long *ev_count;   // search steps
    unsigned long long *keys_done;
    unsigned long long *probes;     // may be null: cache lookups (one per legal candidate of a probe round)
};
WglWs wgl_layout(uint64_t budget, uint32_t max_events, uint32_t table_entries);
size_t wgl_table_entries(uint64_t budget);
hipError_t launch_wgl(const WglArgs &a, int grid, hipStream_t s);
size_t wgl_lds_bytes(uint32_t lds_events, uint32_t lds_tab);  // dynamic LDS of a k_wgl block
bool wgl_allow_lds(size_t bytes);  // lets k_wgl blocks take `bytes` of dynamic LDS (false: not granted)
hipError_t launch_collect_budget(const uint8_t *cause, int32_t n, int32_t *list, int32_t *count, hipStream_t s);

}  // namespace lcd
