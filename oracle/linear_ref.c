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

typedef struct { uint64_t lo, hi; } cfg_t;  /* lo: slots 0..63; hi: slots 64..111 | state << 48 */
#define CFG_EMPTY_HI (~0ull)

typedef struct {
    int8_t valid;       /* 1 / 0 / -1 */
    uint8_t cause;      /* LC_CAUSE_* */
    int32_t fail_event; /* ordinal in the key's reduced event list, or -1 */
    uint32_t peak;
    uint64_t probes;
    uint64_t n_events;
} oracle_key_result;

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

/* --------------------------------------------------------- per-key reduction */
typedef struct {
    uint8_t f;
    int64_t v0, v1;
    int8_t fate;    /* 0 pending forever, 1 ok, 2 failed */
} kop_t;

typedef struct { int64_t p; int32_t op; } pent;

/* cas-register step over state ids (0 = nil, NONE = unproducible value) */
typedef struct { uint8_t kind; uint32_t a, b; } desc_t;  /* kind: LC_T_* */
static inline int step(uint32_t s, desc_t d, uint32_t *out) {
    switch (d.kind) {
        case LC_T_READ_ANY: *out = s; return 1;
        case LC_T_READ: if (s != d.a) return 0; *out = s; return 1;
        case LC_T_WRITE: *out = d.b; return 1;
        default: if (s != d.a) return 0; *out = d.b; return 1;
    }
}

typedef struct { int64_t v; uint32_t id; int used; } vent;

static uint32_t vmap_get(vent *tab, uint64_t cap, int64_t v) {
    if (v == LC_NIL) return 0;
    uint64_t h = mix64((uint64_t)v) & (cap - 1);
    while (tab[h].used) { if (tab[h].v == v) return tab[h].id; h = (h + 1) & (cap - 1); }
    return LC_STATE_NONE;
}
static void vmap_put(vent *tab, uint64_t cap, int64_t v, uint32_t *next) {
    uint64_t h = mix64((uint64_t)v) & (cap - 1);
    while (tab[h].used) { if (tab[h].v == v) return; h = (h + 1) & (cap - 1); }
    tab[h].used = 1; tab[h].v = v; tab[h].id = (*next)++;
}

/* Ops each model can step (knossos.model cas-register / register / mutex). */
static int model_steps(int model, uint8_t f) {
    if (model == LC_MODEL_MUTEX) return f == LC_F_ACQUIRE || f == LC_F_RELEASE;
    if (model == LC_MODEL_REGISTER) return f == LC_F_READ || f == LC_F_WRITE;
    return f == LC_F_READ || f == LC_F_WRITE || f == LC_F_CAS;
}

/* Check one key: rows[] are its sub-history rows (history order). */
static int check_key(const lc_history *h, const int64_t *rows, int64_t nr, uint64_t budget, int model,
                     oracle_key_result *res) {
    memset(res, 0, sizeof *res);
    res->valid = 1; res->fail_event = -1; res->peak = 1;
    kop_t *ops = (kop_t *)malloc((size_t)(nr + 1) * sizeof(kop_t));
    int32_t *row_op = (int32_t *)malloc((size_t)(nr + 1) * sizeof(int32_t));
    pent *pm = (pent *)malloc((size_t)(nr + 1) * sizeof(pent));
    if (!ops || !row_op || !pm) { free(ops); free(row_op); free(pm); return LC_E_NOMEM; }
    int64_t nops = 0, npm = 0;
    /* knossos.history/complete */
    for (int64_t i = 0; i < nr; ++i) {
        int64_t r = rows[i];
        uint8_t t = h->type[r];
        int64_t p = h->process[r];
        row_op[i] = -1;
        int64_t j;
        for (j = 0; j < npm; ++j) if (pm[j].p == p) break;
        if (t == LC_INVOKE) {
            if (!model_steps(model, h->f[r])) { free(ops); free(row_op); free(pm); return LC_E_UNSUPPORTED; }
            ops[nops].f = h->f[r]; ops[nops].v0 = h->v0[r]; ops[nops].v1 = h->v1[r]; ops[nops].fate = 0;
            if (j < npm) pm[j].op = (int32_t)nops; else { pm[npm].p = p; pm[npm].op = (int32_t)nops; npm++; }
            row_op[i] = (int32_t)nops++;
        } else if (t == LC_OK_T || t == LC_FAIL) {
            if (j == npm) { free(ops); free(row_op); free(pm); return LC_E_INVALID; }
            kop_t *o = &ops[pm[j].op];
            if (t == LC_OK_T) {
                o->fate = 1;
                if (o->f == LC_F_CAS) { if (o->v0 == LC_NIL && o->v1 == LC_NIL) { o->v0 = h->v0[r]; o->v1 = h->v1[r]; } }
                else if (o->v0 == LC_NIL) o->v0 = h->v0[r];
                row_op[i] = pm[j].op;
            } else {
                o->fate = 2;
            }
            pm[j] = pm[--npm];
        } else if (t == LC_INFO) {
            if (j < npm) pm[j] = pm[--npm];
        }
    }
    free(pm);
    /* register values -> state ids */
    uint64_t vcap = 16;
    while (vcap < (uint64_t)nops * 2 + 2) vcap <<= 1;
    vent *vt = (vent *)calloc(vcap, sizeof(vent));
    if (!vt) { free(ops); free(row_op); return LC_E_NOMEM; }
    uint32_t nstates = 1;
    for (int64_t k = 0; k < nops; ++k) {
        if (ops[k].fate == 2) continue;
        if (ops[k].f == LC_F_WRITE && ops[k].v0 != LC_NIL) vmap_put(vt, vcap, ops[k].v0, &nstates);
        if (ops[k].f == LC_F_CAS && ops[k].v1 != LC_NIL) vmap_put(vt, vcap, ops[k].v1, &nstates);
    }
    desc_t *desc = (desc_t *)malloc((size_t)(nops + 1) * sizeof(desc_t));
    if (!desc) { free(vt); free(ops); free(row_op); return LC_E_NOMEM; }
    if (model == LC_MODEL_MUTEX) nstates = 2;  /* 0 unlocked (initial), 1 locked */
    for (int64_t k = 0; k < nops; ++k) {
        desc_t d;
        if (ops[k].f == LC_F_ACQUIRE) {        /* legal iff unlocked */
            d.kind = LC_T_CAS; d.a = 0; d.b = 1;
        } else if (ops[k].f == LC_F_RELEASE) { /* legal iff locked */
            d.kind = LC_T_CAS; d.a = 1; d.b = 0;
        } else if (ops[k].f == LC_F_READ) {
            d.kind = ops[k].v0 == LC_NIL ? LC_T_READ_ANY : LC_T_READ;
            d.a = vmap_get(vt, vcap, ops[k].v0); d.b = 0;
        } else if (ops[k].f == LC_F_WRITE) {
            d.kind = LC_T_WRITE; d.a = 0; d.b = vmap_get(vt, vcap, ops[k].v0);
        } else {
            d.kind = LC_T_CAS; d.a = vmap_get(vt, vcap, ops[k].v0); d.b = vmap_get(vt, vcap, ops[k].v1);
        }
        desc[k] = d;
    }
    free(vt);
    if (nstates > LC_WIDE_MAX_STATES) {
        res->valid = -1; res->cause = LC_CAUSE_STATES;
        free(desc); free(ops); free(row_op);
        return 0;
    }
    /* knossos.linear JIT search */
    cset S, Sn, I;
    cvec list = {0, 0, 0};
    if (cset_init(&S, 64) || cset_init(&Sn, 64) || cset_init(&I, 64)) {
        free(desc); free(ops); free(row_op); return LC_E_NOMEM;
    }
    int rc = 0;
    cfg_t init = {0, 0};
    cset_insert(&S, init);
    int32_t *slot_of = (int32_t *)malloc((size_t)(nops + 1) * sizeof(int32_t));
    if (!slot_of) { free(S.tab); free(Sn.tab); free(I.tab); free(desc); free(ops); free(row_op); return LC_E_NOMEM; }
    desc_t slot_desc[128];
    uint64_t freem[2] = {~0ull, ~0ull};
    int pend_slots[128];
    int npend = 0;
    int64_t ev = 0;
    for (int64_t i = 0; i < nr && rc == 0; ++i) {
        int32_t id = row_op[i];
        if (id < 0 || ops[id].fate == 2) continue;
        int64_t r = rows[i];
        if (h->type[r] == LC_INVOKE) {
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
    free(slot_of); free(desc); free(ops); free(row_op);
    return rc;
}

/* ---------------------------------------------------------- independent split */
typedef struct { int64_t k; int64_t idx; int used; } kent;

typedef struct {
    const lc_history *h;
    const int64_t *rows;
    const uint64_t *off;
    int64_t nkeys;
    uint64_t budget;
    int model;
    oracle_key_result *out;
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
        int rc = check_key(j->h, j->rows + j->off[k], (int64_t)(j->off[k + 1] - j->off[k]), j->budget, j->model,
                           &j->out[k]);
        if (rc == LC_E_INVALID || rc == LC_E_UNSUPPORTED) {  /* check-safe: this key alone */
            memset(&j->out[k], 0, sizeof j->out[k]);
            j->out[k].valid = -1; j->out[k].cause = LC_CAUSE_ERROR; j->out[k].fail_event = -1;
        } else if (rc) {
            pthread_mutex_lock(&j->mu); j->rc = rc; pthread_mutex_unlock(&j->mu);
        }
    }
    return NULL;
}

/*
 * Check every independent key of a history.  Keys in order of first
 * appearance (as lc_pack).  Returns the key count (or a negative LC_E_*);
 * out_keys / out must hold max_keys entries (call with max_keys = 0 to count).
 */
int64_t oracle_check_history_model(const lc_history *h, int model, uint64_t budget, int n_threads,
                                   int64_t *out_keys, oracle_key_result *out, int64_t max_keys) {
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
    if (max_keys == 0) { free(rk); free(keys); return nk; }
    if (max_keys < nk) { free(rk); free(keys); return LC_E_INVALID; }
    uint64_t *off = (uint64_t *)calloc((size_t)nk + 1, sizeof(uint64_t));
    int64_t *rows = (int64_t *)malloc((size_t)(n - nshared + nk * nshared + 1) * sizeof(int64_t));
    if (!off || !rows) { free(rk); free(keys); free(off); free(rows); return LC_E_NOMEM; }
    for (int64_t r = 0; r < n; ++r) if (rk[r] >= 0) off[rk[r] + 1]++;
    for (int64_t k = 0; k < nk; ++k) off[k + 1] += off[k] + (uint64_t)nshared;
    {
        uint64_t *cur = (uint64_t *)malloc((size_t)(nk + 1) * sizeof(uint64_t));
        if (!cur) { free(rk); free(keys); free(off); free(rows); return LC_E_NOMEM; }
        memcpy(cur, off, (size_t)nk * sizeof(uint64_t));
        /* jepsen.independent/subhistory: the key's own rows and every
         * non-tuple row, in history order */
        for (int64_t r = 0; r < n; ++r) {
            if (rk[r] >= 0) rows[cur[rk[r]]++] = r;
            else for (int64_t k = 0; k < nk; ++k) rows[cur[k]++] = r;
        }
        free(cur);
    }
    free(rk);
    job_t j = {h, rows, off, nk, budget ? budget : (1ull << 20), model, out, 0, 0, PTHREAD_MUTEX_INITIALIZER};
    if (n_threads < 1) n_threads = 1;
    if (n_threads > 256) n_threads = 256;
    pthread_t th[256];
    for (int t = 1; t < n_threads; ++t) pthread_create(&th[t], NULL, worker, &j);
    worker(&j);
    for (int t = 1; t < n_threads; ++t) pthread_join(th[t], NULL);
    if (out_keys) memcpy(out_keys, keys, (size_t)nk * sizeof(int64_t));
    free(keys); free(off); free(rows);
    return j.rc ? j.rc : nk;
}

/* The demo's model, (model/cas-register) (etcdemo.clj:117). */
int64_t oracle_check_history(const lc_history *h, uint64_t budget, int n_threads,
                             int64_t *out_keys, oracle_key_result *out, int64_t max_keys) {
    return oracle_check_history_model(h, LC_MODEL_CAS_REGISTER, budget, n_threads, out_keys, out, max_keys);
}
