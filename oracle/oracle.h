/*
 * oracle.h -- shared declarations of the C restatements (linear_ref.c,
 * wgl_ref.c) -- TEST ORACLE.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg load oracle/_build/liboracle.so.
 */
#ifndef ORACLE_H
#define ORACLE_H

#include <stdint.h>

#include "../include/lincheck.h"

typedef struct {
    int8_t valid;       /* 1 / 0 / -1 */
    uint8_t cause;      /* LC_CAUSE_* */
    int32_t fail_event; /* ordinal in the key's reduced event list, or -1 */
    uint32_t peak;      /* :linear: largest config set; :wgl: Lowe's cache size at the end */
    uint64_t probes;    /* :linear: successor probes; :wgl: cache lookups */
    uint64_t n_events;  /* :linear: events processed; :wgl: search steps (linearizations + backtracks) */
} oracle_key_result;

typedef int (*oracle_key_fn)(void *ctx, int64_t k);

int64_t oracle_split_keys(const lc_history *h, int64_t **keys_out, uint64_t **off_out, int64_t **rows_out);
int oracle_run_pool(int n_threads, int64_t nkeys, oracle_key_fn fn, void *ctx);

#endif /* ORACLE_H */
