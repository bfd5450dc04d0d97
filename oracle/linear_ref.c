/*
 * linear_ref.c -- C restatement of knossos.linear (cas-register) -- TEST ORACLE
 * and the timed CPU baseline (bench.py cpu_baseline, kind "port").
 *
 * Test infrastructure: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this (oracle/_build/liboracle.so).  The product
 * (liblincheck.so) never links or calls it.
 *
 * Same semantics as oracle/linear_ref.py (whose header states them and their
 * upstream sources; parity against Knossos itself is UNPINNED -- knossos 0.3.7
 * is absent):
 *   jepsen.independent/checker split (etcdemo.clj:115), knossos.history
 *   complete + without-failures, cas-register step (etcdemo.clj:117), the JIT
 *   config-set search of knossos.linear (:algorithm :linear, etcdemo.clj:118)
 *   with a deterministic config budget in place of knossos.search's abort.
 *   A key whose sub-history complete rejects (a completion with no
 *   outstanding invocation) or that holds an op the model cannot step is
 *   :unknown with cause LC_CAUSE_ERROR, and the other keys are checked:
 *   independent/checker's check-safe per key (etcdemo.clj:115).
 * Written independently of the device code: plain sequential search, one
 * growable open-addressed hash set per set, a pthread pool over keys standing
 * in for independent/checker's bounded-pmap.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/lincheck.h"
#include "keyprep.h"

typedef struct { uint64_t lo, hi; } cfg_t;  /* lo: slots 0..63; hi: slots 64..111 | state << 48 */
#define CFG_EMPTY_HI (~0ull)

#include "oracle.h"

/* ------------------------------------------------------------------ hash set */
typedef struct { cfg_t *tab; uint64_t cap, n; } cset;

static uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}
static uint64_t cfg_hash(cfg_t c) { return mix64(c.lo ^ mix64(c.hi + 0x9E3779B97F4A7C15ull)); }

static int cset_init(cset *s, uint64_t cap) {
    s->cap = cap; s->n = 0;
    s->tab = (cfg_t *)malloc(cap * sizeof(cfg_t));
    if (!s->tab) return -1;
    for (uint64_t i = 0; i < cap; ++i) s->tab[i].hi = CFG_EMPTY_HI;
    return 0;
}
static void cset_clear(cset *s) {
    if (s->cap > 4096 && s->n * 16 < s->cap) {  /* sparse after a big event: shrink */
        cfg_t *t = (cfg_t *)malloc(4096 * sizeof(cfg_t));
        if (t) { free(s->tab); s->tab = t; s->cap = 4096; s->n = 1; }
    }
    if (s->n) for (uint64_t i = 0; i < s->cap; ++i) s->tab[i].hi = CFG_EMPTY_HI;
    s->n = 0;
}
static int cset_insert(cset *s, cfg_t c);
static int cset_grow(cset *s) {
    cset t;
    if (cset_init(&t, s->cap * 2)) return -1;
    for (uint64_t i = 0; i < s->cap; ++i)
        if (s->tab[i].hi != CFG_EMPTY_HI) cset_insert(&t, s->tab[i]);
    free(s->tab);
    *s = t;
    return 0;
}
/* 1 = inserted, 0 = present, -1 = no memory */
static int cset_insert(cset *s, cfg_t c) {
    if ((s->n + 1) * 2 > s->cap && cset_grow(s)) return -1;
    uint64_t m = s->cap - 1, h = cfg_hash(c) & m;
    for (;;) {
        cfg_t *e = &s->tab[h];
        if (e->hi == CFG_EMPTY_HI) { *e = c; s->n++; return 1; }
        if (e->hi == c.hi && e->lo == c.lo) return 0;
        h = (h + 1) & m;
    }
}

typedef struct { cfg_t *v; uint64_t n, cap; } cvec;
static int cvec_push(cvec *a, cfg_t c) {
    if (a->n == a->cap) {
        uint64_t nc = a->cap ? a->cap * 2 : 256;
        cfg_t *nv = (cfg_t *)realloc(a->v, nc * sizeof(cfg_t));
        if (!nv) return -1;
        a->v = nv; a->cap = nc;
    }
    a->v[a->n++] = c;
    return 0;
}

static inline int cfg_has(cfg_t c, int s) { return s < 64 ? (int)((c.lo >> s) & 1) : (int)((c.hi >> (s - 64)) & 1); }
static inline cfg_t cfg_set(cfg_t c, int s) { if (s < 64) c.lo |= 1ull << s; else c.hi |= 1ull << (s - 64); return c; }
static inline cfg_t cfg_clr(cfg_t c, int s) { if (s < 64) c.lo &= ~(1ull << s); else c.hi &= ~(1ull << (s - 64)); return c; }
static inline uint32_t cfg_state(cfg_t c) { return (uint32_t)(c.hi >> 48); }
static inline cfg_t cfg_with_state(cfg_t c, uint32_t st) { c.hi = (c.hi & 0xFFFFFFFFFFFFull) | ((uint64_t)st << 48); return c; }

/* ------------------------------------------------------------- the search */
static inline int step(uint32_t s, desc_t d, uint32_t *out) { return kp_step(s, d, out); }

/* Check one key: rows[] are its sub-history rows (history order). */
static int check_key(const lc_history *h, const int64_t *rows, int64_t nr, uint64_t budget, int model,
                     oracle_key_result *res) {
    memset(res, 0, sizeof *res);
    res->valid = 1; res->fail_event = -1; res->peak = 1;
    kp_key kk;
    int prc = kp_reduce(h, rows, nr, model, &kk);
    if (prc) return prc;
    const desc_t *desc = kk.desc;
    if (kk.nstates > LC_WIDE_MAX_STATES) {
        res->valid = -1; res->cause = LC_CAUSE_STATES;
        kp_free(&kk);
        return 0;
    }
    /* knossos.linear JIT search */
    cset S, Sn, I;
    cvec list = {0, 0, 0};
    if (cset_init(&S, 64) || cset_init(&Sn, 64) || cset_init(&I, 64)) { kp_free(&kk); return LC_E_NOMEM; }
    int rc = 0;
    cfg_t init = {0, 0};
    cset_insert(&S, init);
    int32_t *slot_of = (int32_t *)malloc((size_t)(kk.nops + 1) * sizeof(int32_t));
    if (!slot_of) { free(S.tab); free(Sn.tab); free(I.tab); kp_free(&kk); return LC_E_NOMEM; }
    desc_t slot_desc[128];
    uint64_t freem[2] = {~0ull, ~0ull};
    int pend_slots[128];
    int npend = 0;
    int64_t ev = 0;
    for (int64_t e = 0; e < kk.nev && rc == 0; ++e) {
        int32_t id = kk.ev_op[e];
        if (!kk.ev_ok[e]) {
            int s = freem[0] ? __builtin_ctzll(freem[0]) : (freem[1] ? 64 + __builtin_ctzll(freem[1]) : 128);
            if (s >= LC_WIDE_MAX_SLOTS) { res->valid = -1; res->cause = LC_CAUSE_WINDOW; res->fail_event = (int32_t)ev; break; }
            freem[s >> 6] &= ~(1ull << (s & 63));
            slot_of[id] = s;
            slot_desc[s] = desc[id];
            pend_slots[npend++] = s;
            ev++;
            continue;
        }
        /* :ok of op id in slot p */
        int p = slot_of[id];
        desc_t dp = slot_desc[p];
        cset_clear(&Sn); cset_clear(&I);
        list.n = 0;
        res->probes += S.n;
        for (uint64_t k = 0; k < S.cap; ++k) {
            cfg_t c = S.tab[k];
            if (c.hi == CFG_EMPTY_HI) continue;
            if (cfg_has(c, p)) { if (cset_insert(&Sn, cfg_clr(c, p)) < 0) rc = LC_E_NOMEM; }
            else { if (cset_insert(&I, c) < 0 || cvec_push(&list, c)) rc = LC_E_NOMEM; }
        }
        /* closure: list doubles as the FIFO work queue */
        uint64_t head = 0;
        while (rc == 0 && head < list.n) {
            cfg_t c = list.v[head++];
            uint32_t st = cfg_state(c);
            for (int q = 0; q < npend; ++q) {
                int sq = pend_slots[q];
                if (sq == p || cfg_has(c, sq)) continue;
                uint32_t s2;
                if (!step(st, slot_desc[sq], &s2)) continue;
                res->probes++;
                cfg_t c2 = cfg_with_state(cfg_set(c, sq), s2);
                int ins = cset_insert(&I, c2);
                if (ins < 0) { rc = LC_E_NOMEM; break; }
                if (ins == 1) {
                    if (I.n > budget) { res->valid = -1; res->cause = LC_CAUSE_BUDGET; res->fail_event = (int32_t)ev; goto done; }
                    if (cvec_push(&list, c2)) { rc = LC_E_NOMEM; break; }
                }
            }
        }
        for (uint64_t k = 0; rc == 0 && k < list.n; ++k) {
            cfg_t c = list.v[k];
            uint32_t s2;
            if (!step(cfg_state(c), dp, &s2)) continue;
            res->probes++;
            if (cset_insert(&Sn, cfg_with_state(c, s2)) < 0) rc = LC_E_NOMEM;
        }
        if (rc) break;
        if (Sn.n == 0) { res->valid = 0; res->cause = LC_CAUSE_NONLIN; res->fail_event = (int32_t)ev; break; }
        if (Sn.n > budget) { res->valid = -1; res->cause = LC_CAUSE_BUDGET; res->fail_event = (int32_t)ev; break; }
        { cset t = S; S = Sn; Sn = t; }
        if (S.n > res->peak) res->peak = (uint32_t)S.n;
        freem[p >> 6] |= 1ull << (p & 63);
        for (int q = 0; q < npend; ++q) if (pend_slots[q] == p) { pend_slots[q] = pend_slots[--npend]; break; }
        ev++;
    }
done:
    res->n_events = (uint64_t)ev;
    free(S.tab); free(Sn.tab); free(I.tab); free(list.v);
    free(slot_of); kp_free(&kk);
    return rc;
}

/* ---------------------------------------------------------- independent split */
typedef struct { int64_t k; int64_t idx; int used; } kent;

/*
 * jepsen.independent/checker's split (etcdemo.clj:115): the keys in order of
 * first appearance (as lc_pack) and, per key, its sub-history rows -- the
 * key's own rows and every non-tuple row, in history order.  Returns the key
 * count (or a negative LC_E_*); *keys, *off ([nk + 1]) and *rows are malloc'ed.
 */
int64_t oracle_split_keys(const lc_history *h, int64_t **keys_out, uint64_t **off_out, int64_t **rows_out) {
    if (!h || h->n < 0) return LC_E_INVALID;
    int64_t n = h->n;
    uint64_t cap = 64;
    while (cap < (uint64_t)n * 2 + 2) cap <<= 1;
    kent *kt = (kent *)calloc(cap, sizeof(kent));
    int64_t *rk = (int64_t *)malloc((size_t)(n + 1) * sizeof(int64_t));
    int64_t *keys = (int64_t *)malloc((size_t)(n + 1) * sizeof(int64_t));
    if (!kt || !rk || !keys) { free(kt); free(rk); free(keys); return LC_E_NOMEM; }
    int64_t nk = 0, nshared = 0;
    for (int64_t r = 0; r < n; ++r) {
        int64_t k = h->key[r];
        if (k == LC_NO_KEY) {  /* not a tuple: in every key's sub-history */
            rk[r] = -1;
            nshared++;
            continue;
        }
        uint64_t s = (uint64_t)((uint64_t)k * 0x9E3779B97F4A7C15ull) & (cap - 1);
        while (kt[s].used && kt[s].k != k) s = (s + 1) & (cap - 1);
        if (!kt[s].used) { kt[s].used = 1; kt[s].k = k; kt[s].idx = nk; keys[nk++] = k; }
        rk[r] = kt[s].idx;
    }
    free(kt);
    uint64_t *off = (uint64_t *)calloc((size_t)nk + 1, sizeof(uint64_t));
    int64_t *rows = (int64_t *)malloc((size_t)(n - nshared + nk * nshared + 1) * sizeof(int64_t));
    uint64_t *cur = (uint64_t *)malloc((size_t)(nk + 1) * sizeof(uint64_t));
    if (!off || !rows || !cur) { free(rk); free(keys); free(off); free(rows); free(cur); return LC_E_NOMEM; }
    for (int64_t r = 0; r < n; ++r) if (rk[r] >= 0) off[rk[r] + 1]++;
    for (int64_t k = 0; k < nk; ++k) off[k + 1] += off[k] + (uint64_t)nshared;
    memcpy(cur, off, (size_t)nk * sizeof(uint64_t));
    for (int64_t r = 0; r < n; ++r) {
        if (rk[r] >= 0) rows[cur[rk[r]]++] = r;
        else for (int64_t k = 0; k < nk; ++k) rows[cur[k]++] = r;
    }
    free(cur); free(rk);
    *keys_out = keys; *off_out = off; *rows_out = rows;
    return nk;
}

typedef struct {
    oracle_key_fn fn;
    void *ctx;
    int64_t nkeys;
    int64_t next;
    int rc;
    pthread_mutex_t mu;
} job_t;

static void *worker(void *arg) {
    job_t *j = (job_t *)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        int64_t k = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (k >= j->nkeys) break;
        int rc = j->fn(j->ctx, k);
        if (rc) { pthread_mutex_lock(&j->mu); j->rc = rc; pthread_mutex_unlock(&j->mu); }
    }
    return NULL;
}

/* fn(ctx, k) for k in [0, nkeys) on a pool of n_threads (independent/checker's
 * bounded-pmap).  Returns the first nonzero fn result, else 0. */
int oracle_run_pool(int n_threads, int64_t nkeys, oracle_key_fn fn, void *ctx) {
    job_t j = {fn, ctx, nkeys, 0, 0, PTHREAD_MUTEX_INITIALIZER};
    if (n_threads < 1) n_threads = 1;
    if (n_threads > 256) n_threads = 256;
    pthread_t th[256];
    for (int t = 1; t < n_threads; ++t) pthread_create(&th[t], NULL, worker, &j);
    worker(&j);
    for (int t = 1; t < n_threads; ++t) pthread_join(th[t], NULL);
    return j.rc;
}

typedef struct {
    const lc_history *h;
    const int64_t *rows;
    const uint64_t *off;
    uint64_t budget;
    int model;
    oracle_key_result *out;
} lin_job;

static int lin_key(void *ctx, int64_t k) {
    lin_job *j = (lin_job *)ctx;
    int rc = check_key(j->h, j->rows + j->off[k], (int64_t)(j->off[k + 1] - j->off[k]), j->budget, j->model, &j->out[k]);
    if (rc == LC_E_INVALID || rc == LC_E_UNSUPPORTED) {  /* check-safe: this key alone */
        memset(&j->out[k], 0, sizeof j->out[k]);
        j->out[k].valid = -1; j->out[k].cause = LC_CAUSE_ERROR; j->out[k].fail_event = -1;
        return 0;
    }
    return rc;
}

/*
 * Check every independent key of a history.  Keys in order of first
 * appearance (as lc_pack).  Returns the key count (or a negative LC_E_*);
 * out_keys / out must hold max_keys entries (call with max_keys = 0 to count).
 */
int64_t oracle_check_history_model(const lc_history *h, int model, uint64_t budget, int n_threads,
                                   int64_t *out_keys, oracle_key_result *out, int64_t max_keys) {
    int64_t *keys, *rows;
    uint64_t *off;
    int64_t nk = oracle_split_keys(h, &keys, &off, &rows);
    if (nk < 0) return nk;
    if (max_keys == 0 || max_keys < nk) { free(keys); free(off); free(rows); return max_keys == 0 ? nk : LC_E_INVALID; }
    lin_job j = {h, rows, off, budget ? budget : (1ull << 20), model, out};
    int rc = oracle_run_pool(n_threads, nk, lin_key, &j);
    if (out_keys) memcpy(out_keys, keys, (size_t)nk * sizeof(int64_t));
    free(keys); free(off); free(rows);
    return rc ? rc : nk;
}

/* The demo's model, (model/cas-register) (etcdemo.clj:117). */
int64_t oracle_check_history(const lc_history *h, uint64_t budget, int n_threads,
                             int64_t *out_keys, oracle_key_result *out, int64_t max_keys) {
    return oracle_check_history_model(h, LC_MODEL_CAS_REGISTER, budget, n_threads, out_keys, out, max_keys);
}
