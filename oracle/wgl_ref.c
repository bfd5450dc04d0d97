/*
 * wgl_ref.c -- C restatement of knossos.wgl (Wing & Gong with Lowe's cache)
 * -- TEST ORACLE and the timed CPU :wgl baseline (bench.py cpu_baseline.wgl,
 * kind "port").
 *
 * Test infrastructure: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this (oracle/_build/liboracle.so).  The product
 * (liblincheck.so) never links or calls it.
 *
 * Same search as oracle/wgl_ref.py (whose header states it; the
 * :algorithm :wgl value of the slot at etcdemo.clj:118; parity against
 * Knossos itself is UNPINNED), step for step:
 *   the key's reduced events (keyprep.h: complete + without-failures) are a
 *   doubly linked list of call / return entries; the walk starts at the head;
 *   at a call entry whose op the model can step and whose (linearized set,
 *   state) is not in the cache, the pair is cached, the call and its return
 *   are lifted out of the list and the walk restarts at the head; otherwise it
 *   moves on.  At a return entry it is stuck: the deepest such entries'
 *   (state, linearized pending ops) form the frontier, and the walk backtracks
 *   to the last linearization (unlifting it) and moves past it.  Running off
 *   the end is :valid? true; stuck with nothing to backtrack is false at the
 *   deepest return entry; a cache of more than `budget` pairs is :unknown
 *   (cause budget).
 * The cache key is (R, X, state): R the first return entry still in the list
 * and X the window slots (lowest free at invoke, as lc_pack assigns them) of
 * the linearized ops pending at R.  Every op returning before R is
 * linearized, so (R, X) names the linearized set exactly (a bijection), and
 * the cache behaves as a cache of (linearized set, state) pairs.  The same
 * representation limits as linear_ref.c, applied before the search: a key
 * needing window slot >= 112 is :unknown "window" (fail_event = that
 * :invoke), more than 32767 register values :unknown "states".
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/lincheck.h"
#include "keyprep.h"
#include "oracle.h"

typedef struct { uint64_t lo, hi, rs; } wkey;  /* X lo, X hi, R | state << 32 */
#define WKEY_EMPTY (~0ull)

typedef struct { wkey *tab; uint64_t cap, n; } wset;

static uint64_t wkey_hash(wkey k) { return kp_mix64(k.lo ^ kp_mix64(k.hi ^ kp_mix64(k.rs + 0x9E3779B97F4A7C15ull))); }

static int wset_init(wset *s, uint64_t cap) {
    s->cap = cap; s->n = 0;
    s->tab = (wkey *)malloc(cap * sizeof(wkey));
    if (!s->tab) return -1;
    for (uint64_t i = 0; i < cap; ++i) s->tab[i].rs = WKEY_EMPTY;
    return 0;
}
static int wset_insert(wset *s, wkey k);
static int wset_grow(wset *s) {
    wset t;
    if (wset_init(&t, s->cap * 2)) return -1;
    for (uint64_t i = 0; i < s->cap; ++i)
        if (s->tab[i].rs != WKEY_EMPTY) wset_insert(&t, s->tab[i]);
    free(s->tab);
    *s = t;
    return 0;
}
/* 1 = inserted, 0 = present, -1 = no memory */
static int wset_insert(wset *s, wkey k) {
    if ((s->n + 1) * 2 > s->cap && wset_grow(s)) return -1;
    uint64_t m = s->cap - 1, h = wkey_hash(k) & m;
    for (;;) {
        wkey *e = &s->tab[h];
        if (e->rs == WKEY_EMPTY) { *e = k; s->n++; return 1; }
        if (e->rs == k.rs && e->lo == k.lo && e->hi == k.hi) return 0;
        h = (h + 1) & m;
    }
}

static inline void m_set(uint64_t *lo, uint64_t *hi, int s) { if (s < 64) *lo |= 1ull << s; else *hi |= 1ull << (s - 64); }
static inline void m_clr(uint64_t *lo, uint64_t *hi, int s) { if (s < 64) *lo &= ~(1ull << s); else *hi &= ~(1ull << (s - 64)); }

typedef struct { int64_t e0; uint32_t s; int64_t R; uint64_t lo, hi; } wframe;

/*
 * One key.  finals (may be NULL): up to max_final frontier entries in the
 * order the search reached them, 3 words each: X lo, X hi, register value of
 * the state (LC_NIL = nil / unlocked); *n_final = how many were written.
 */
static int wgl_key(const lc_history *h, const int64_t *rows, int64_t nr, uint64_t budget, int model, uint32_t init,
                   int max_final, oracle_key_result *res, int64_t *finals, uint32_t *n_final) {
    memset(res, 0, sizeof *res);
    res->valid = 1; res->fail_event = -1;
    if (n_final) *n_final = 0;
    kp_key kk;
    int prc = kp_reduce(h, rows, nr, model, &kk);
    if (prc) return prc;
    if (kk.nstates > LC_WIDE_MAX_STATES) {
        res->valid = -1; res->cause = LC_CAUSE_STATES;
        kp_free(&kk);
        return 0;
    }
    const int64_t n = kk.nev, END = n, HEAD = n + 1;
    int64_t *nxt = (int64_t *)malloc((size_t)(n + 2) * sizeof(int64_t));
    int64_t *prv = (int64_t *)malloc((size_t)(n + 2) * sizeof(int64_t));
    int64_t *ret_of = (int64_t *)malloc((size_t)(kk.nops + 1) * sizeof(int64_t));
    int16_t *slot_of = (int16_t *)malloc((size_t)(kk.nops + 1) * sizeof(int16_t));
    uint8_t *lin = (uint8_t *)calloc((size_t)kk.nops + 1, 1);
    wframe *stack = (wframe *)malloc((size_t)(kk.nops + 1) * sizeof(wframe));
    wset cache = {0, 0, 0};
    int rc = 0;
    if (!nxt || !prv || !ret_of || !slot_of || !lin || !stack || wset_init(&cache, 1024)) { rc = LC_E_NOMEM; goto out; }
    /* window slots: lowest free at :invoke, freed at :ok (crashed ops keep theirs) */
    {
        uint64_t freem[2] = {~0ull, ~0ull};
        for (int64_t i = 0; i < n; ++i) {
            const int32_t o = kk.ev_op[i];
            if (kk.ev_ok[i]) {
                const int s = slot_of[o];
                freem[s >> 6] |= 1ull << (s & 63);
                ret_of[o] = i;
                continue;
            }
            const int s = freem[0] ? __builtin_ctzll(freem[0]) : (freem[1] ? 64 + __builtin_ctzll(freem[1]) : 128);
            if (s >= LC_WIDE_MAX_SLOTS) {
                res->valid = -1; res->cause = LC_CAUSE_WINDOW; res->fail_event = (int32_t)i;
                goto out;
            }
            freem[s >> 6] &= ~(1ull << (s & 63));
            slot_of[o] = (int16_t)s;
            ret_of[o] = -1;
        }
    }
    for (int64_t i = 0; i < n; ++i) { nxt[i] = i + 1; prv[i] = i ? i - 1 : HEAD; }
    nxt[HEAD] = n ? 0 : END;
    prv[END] = n ? n - 1 : HEAD;
    nxt[END] = END;
    prv[HEAD] = HEAD;
#define UNLINK(i) do { nxt[prv[i]] = nxt[i]; prv[nxt[i]] = prv[i]; } while (0)
#define RELINK(i) do { nxt[prv[i]] = (i); prv[nxt[i]] = (i); } while (0)
    uint32_t s = init;
    uint64_t xlo = 0, xhi = 0;
    int64_t R = END;
    for (int64_t i = 0; i < n; ++i) if (kk.ev_ok[i]) { R = i; break; }
    int64_t depth = 0, deepest = -1;
    uint32_t nfront = 0;
    int64_t entry = nxt[HEAD];
    for (;;) {
        if (entry == END) break;  /* every return passed: linearizable */
        if (!kk.ev_ok[entry]) {
            const int32_t o = kk.ev_op[entry];
            uint32_t s2;
            if (kp_step(s, kk.desc[o], &s2)) {
                res->probes++;
                uint64_t lo2 = xlo, hi2 = xhi;
                m_set(&lo2, &hi2, slot_of[o]);
                int64_t R2 = R;
                if (ret_of[o] == R) {
                    /* o's return leaves the list: the first return still in it
                     * is the next one whose op is not linearized; the ops
                     * returning before it leave X */
                    R2 = END;
                    for (int64_t j = R; j < n; ++j) {
                        if (!kk.ev_ok[j]) continue;
                        const int32_t q = kk.ev_op[j];
                        if (q == o || lin[q]) m_clr(&lo2, &hi2, slot_of[q]);
                        else { R2 = j; break; }
                    }
                }
                const wkey k = {lo2, hi2, (uint64_t)(uint32_t)R2 | (uint64_t)s2 << 32};
                const int ins = wset_insert(&cache, k);
                if (ins < 0) { rc = LC_E_NOMEM; goto out; }
                if (ins == 1) {
                    if (cache.n > budget) { res->valid = -1; res->cause = LC_CAUSE_BUDGET; break; }
                    stack[depth++] = (wframe){entry, s, R, xlo, xhi};
                    s = s2; xlo = lo2; xhi = hi2; R = R2;
                    lin[o] = 1;
                    UNLINK(entry);
                    if (ret_of[o] >= 0) UNLINK(ret_of[o]);
                    res->n_events++;
                    entry = nxt[HEAD];
                    continue;
                }
            }
            entry = nxt[entry];
            continue;
        }
        /* a return entry whose op is not linearized (the first one, R): stuck */
        if (entry >= deepest) {
            if (entry > deepest) { deepest = entry; nfront = 0; }
            if (finals && (int)nfront < max_final) {
                finals[3 * nfront + 0] = (int64_t)xlo;
                finals[3 * nfront + 1] = (int64_t)xhi;
                finals[3 * nfront + 2] = kk.state_val[s];
            }
            nfront++;
        }
        if (depth == 0) {
            res->valid = 0; res->cause = LC_CAUSE_NONLIN; res->fail_event = (int32_t)deepest;
            if (n_final) *n_final = nfront < (uint32_t)max_final ? nfront : (uint32_t)max_final;
            break;
        }
        const wframe f = stack[--depth];
        const int32_t o = kk.ev_op[f.e0];
        lin[o] = 0;
        if (ret_of[o] >= 0) RELINK(ret_of[o]);
        RELINK(f.e0);
        s = f.s; xlo = f.lo; xhi = f.hi; R = f.R;
        res->n_events++;
        entry = nxt[f.e0];
    }
#undef UNLINK
#undef RELINK
    res->peak = (uint32_t)(cache.n > 0xFFFFFFFFull ? 0xFFFFFFFFull : cache.n);
out:
    free(nxt); free(prv); free(ret_of); free(slot_of); free(lin); free(stack); free(cache.tab);
    kp_free(&kk);
    return rc;
}

typedef struct {
    const lc_history *h;
    const int64_t *rows;
    const uint64_t *off;
    uint64_t budget;
    int model, max_final;
    oracle_key_result *out;
    int64_t *finals;
    uint32_t *n_final;
} wgl_job;

static int wgl_job_key(void *ctx, int64_t k) {
    wgl_job *j = (wgl_job *)ctx;
    int rc = wgl_key(j->h, j->rows + j->off[k], (int64_t)(j->off[k + 1] - j->off[k]), j->budget, j->model, 0,
                     j->max_final, &j->out[k], j->finals ? j->finals + (size_t)k * j->max_final * 3 : NULL,
                     j->n_final ? j->n_final + k : NULL);
    if (rc == LC_E_INVALID || rc == LC_E_UNSUPPORTED) {  /* check-safe: this key alone */
        memset(&j->out[k], 0, sizeof j->out[k]);
        j->out[k].valid = -1; j->out[k].cause = LC_CAUSE_ERROR; j->out[k].fail_event = -1;
        if (j->n_final) j->n_final[k] = 0;
        return 0;
    }
    return rc;
}

/*
 * independent/checker over linearizable {:algorithm :wgl}: every key of a
 * history (keys in order of first appearance, as lc_pack).  Returns the key
 * count or a negative LC_E_*; call with max_keys = 0 to count.  finals:
 * [max_keys * max_final * 3] or NULL; n_final: [max_keys] or NULL.
 */
int64_t oracle_wgl_check_history_model(const lc_history *h, int model, uint64_t budget, int n_threads, int max_final,
                                       int64_t *out_keys, oracle_key_result *out, int64_t *finals, uint32_t *n_final,
                                       int64_t max_keys) {
    int64_t *keys, *rows;
    uint64_t *off;
    int64_t nk = oracle_split_keys(h, &keys, &off, &rows);
    if (nk < 0) return nk;
    if (max_keys == 0 || max_keys < nk) { free(keys); free(off); free(rows); return max_keys == 0 ? nk : LC_E_INVALID; }
    wgl_job j = {h, rows, off, budget ? budget : (1ull << 20), model, max_final < 0 ? 0 : max_final, out, finals, n_final};
    int rc = oracle_run_pool(n_threads, nk, wgl_job_key, &j);
    if (out_keys) memcpy(out_keys, keys, (size_t)nk * sizeof(int64_t));
    free(keys); free(off); free(rows);
    return rc ? rc : nk;
}
