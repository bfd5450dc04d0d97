/*
 * keyprep.h -- one key's sub-history reduced to the search's input -- TEST
 * ORACLE (shared by linear_ref.c and wgl_ref.c; see linear_ref.c's header for
 * what may load it).
 *
 * knossos.history/complete + without-failures (reached via etcdemo.clj:117)
 * and the cas-register / register / mutex memo (knossos.model.memo), restated
 * as in oracle/linear_ref.py's header:
 *   - pair invoke -> next completion of the same process; :ok copies
 *     (or invocation-value completion-value); :fail drops the pair; :info, or
 *     no completion at all, leaves the op pending forever; a second :invoke by
 *     the same process leaves the first op pending forever;
 *   - a completion with no outstanding invocation is complete's assertion
 *     (LC_E_INVALID: check-safe makes the key :unknown, cause error); an op
 *     the model cannot step likewise (LC_E_UNSUPPORTED);
 *   - register values become state ids in op order (0 = nil).
 * The reduced event list holds an :invoke per surviving op and an :ok per
 * completed one, in history order; :info completions emit nothing.
 */
#ifndef ORACLE_KEYPREP_H
#define ORACLE_KEYPREP_H

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/lincheck.h"

typedef struct { uint8_t kind; uint32_t a, b; } desc_t;  /* kind: LC_T_* */

/* cas-register step over state ids (0 = nil, NONE = unproducible value) */
static inline int kp_step(uint32_t s, desc_t d, uint32_t *out) {
    switch (d.kind) {
        case LC_T_READ_ANY: *out = s; return 1;
        case LC_T_READ: if (s != d.a) return 0; *out = s; return 1;
        case LC_T_WRITE: *out = d.b; return 1;
        default: if (s != d.a) return 0; *out = d.b; return 1;
    }
}

static inline uint64_t kp_mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}

typedef struct {
    int64_t nops;
    desc_t *desc;        /* [nops] */
    int64_t *state_val;  /* [nstates] register value of each state id (LC_NIL for nil / unlocked) */
    uint32_t nstates;
    int64_t nev;
    int32_t *ev_op;      /* [nev] op of each reduced event */
    uint8_t *ev_ok;      /* [nev] 1 = :ok completion, 0 = :invoke */
} kp_key;

static inline void kp_free(kp_key *k) {
    free(k->desc); free(k->state_val); free(k->ev_op); free(k->ev_ok);
    memset(k, 0, sizeof *k);
}

/* Ops each model can step (knossos.model cas-register / register / mutex). */
static inline int kp_model_steps(int model, uint8_t f) {
    if (model == LC_MODEL_MUTEX) return f == LC_F_ACQUIRE || f == LC_F_RELEASE;
    if (model == LC_MODEL_REGISTER) return f == LC_F_READ || f == LC_F_WRITE;
    return f == LC_F_READ || f == LC_F_WRITE || f == LC_F_CAS;
}

typedef struct { int64_t v; uint32_t id; int used; } kp_vent;

static inline uint32_t kp_vmap_get(kp_vent *tab, uint64_t cap, int64_t v) {
    if (v == LC_NIL) return 0;
    uint64_t h = kp_mix64((uint64_t)v) & (cap - 1);
    while (tab[h].used) { if (tab[h].v == v) return tab[h].id; h = (h + 1) & (cap - 1); }
    return LC_STATE_NONE;
}
static inline void kp_vmap_put(kp_vent *tab, uint64_t cap, int64_t v, uint32_t *next, int64_t *vals) {
    uint64_t h = kp_mix64((uint64_t)v) & (cap - 1);
    while (tab[h].used) { if (tab[h].v == v) return; h = (h + 1) & (cap - 1); }
    tab[h].used = 1; tab[h].v = v; tab[h].id = *next;
    vals[*next] = v;
    (*next)++;
}

typedef struct { int8_t fate; uint8_t f; int64_t v0, v1; } kp_op;  /* fate: 0 pending forever, 1 ok, 2 failed */
typedef struct { int64_t p; int32_t op; } kp_pent;

/* Reduce the key whose sub-history rows are rows[0..nr).  Returns 0,
 * LC_E_INVALID (complete's assertion), LC_E_UNSUPPORTED or LC_E_NOMEM. */
static inline int kp_reduce(const lc_history *h, const int64_t *rows, int64_t nr, int model, kp_key *out) {
    memset(out, 0, sizeof *out);
    kp_op *ops = (kp_op *)malloc((size_t)(nr + 1) * sizeof(kp_op));
    int32_t *row_op = (int32_t *)malloc((size_t)(nr + 1) * sizeof(int32_t));
    kp_pent *pm = (kp_pent *)malloc((size_t)(nr + 1) * sizeof(kp_pent));
    if (!ops || !row_op || !pm) { free(ops); free(row_op); free(pm); return LC_E_NOMEM; }
    int64_t nops = 0, npm = 0;
    for (int64_t i = 0; i < nr; ++i) {
        int64_t r = rows[i];
        uint8_t t = h->type[r];
        int64_t p = h->process[r];
        row_op[i] = -1;
        int64_t j;
        for (j = 0; j < npm; ++j) if (pm[j].p == p) break;
        if (t == LC_INVOKE) {
            if (!kp_model_steps(model, h->f[r])) { free(ops); free(row_op); free(pm); return LC_E_UNSUPPORTED; }
            ops[nops].f = h->f[r]; ops[nops].v0 = h->v0[r]; ops[nops].v1 = h->v1[r]; ops[nops].fate = 0;
            if (j < npm) pm[j].op = (int32_t)nops; else { pm[npm].p = p; pm[npm].op = (int32_t)nops; npm++; }
            row_op[i] = (int32_t)nops++;
        } else if (t == LC_OK_T || t == LC_FAIL) {
            if (j == npm) { free(ops); free(row_op); free(pm); return LC_E_INVALID; }
            kp_op *o = &ops[pm[j].op];
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
    kp_vent *vt = (kp_vent *)calloc(vcap, sizeof(kp_vent));
    int64_t *vals = (int64_t *)malloc((size_t)(nops * 2 + 2) * sizeof(int64_t));
    desc_t *desc = (desc_t *)malloc((size_t)(nops + 1) * sizeof(desc_t));
    if (!vt || !vals || !desc) { free(vt); free(vals); free(desc); free(ops); free(row_op); return LC_E_NOMEM; }
    uint32_t nstates = 1;
    vals[0] = LC_NIL;
    for (int64_t k = 0; k < nops; ++k) {
        if (ops[k].fate == 2) continue;
        if (ops[k].f == LC_F_WRITE && ops[k].v0 != LC_NIL) kp_vmap_put(vt, vcap, ops[k].v0, &nstates, vals);
        if (ops[k].f == LC_F_CAS && ops[k].v1 != LC_NIL) kp_vmap_put(vt, vcap, ops[k].v1, &nstates, vals);
    }
    if (model == LC_MODEL_MUTEX) { nstates = 2; vals[1] = 1; }  /* 0 unlocked (initial), 1 locked */
    for (int64_t k = 0; k < nops; ++k) {
        desc_t d;
        if (ops[k].f == LC_F_ACQUIRE) {        /* legal iff unlocked */
            d.kind = LC_T_CAS; d.a = 0; d.b = 1;
        } else if (ops[k].f == LC_F_RELEASE) { /* legal iff locked */
            d.kind = LC_T_CAS; d.a = 1; d.b = 0;
        } else if (ops[k].f == LC_F_READ) {
            d.kind = ops[k].v0 == LC_NIL ? LC_T_READ_ANY : LC_T_READ;
            d.a = kp_vmap_get(vt, vcap, ops[k].v0); d.b = 0;
        } else if (ops[k].f == LC_F_WRITE) {
            d.kind = LC_T_WRITE; d.a = 0; d.b = kp_vmap_get(vt, vcap, ops[k].v0);
        } else {
            d.kind = LC_T_CAS; d.a = kp_vmap_get(vt, vcap, ops[k].v0); d.b = kp_vmap_get(vt, vcap, ops[k].v1);
        }
        desc[k] = d;
    }
    free(vt);
    /* the reduced event list (without-failures; :info completions emit nothing) */
    int32_t *ev_op = (int32_t *)malloc((size_t)(nr + 1) * sizeof(int32_t));
    uint8_t *ev_ok = (uint8_t *)malloc((size_t)(nr + 1));
    if (!ev_op || !ev_ok) { free(ev_op); free(ev_ok); free(vals); free(desc); free(ops); free(row_op); return LC_E_NOMEM; }
    int64_t nev = 0;
    for (int64_t i = 0; i < nr; ++i) {
        int32_t id = row_op[i];
        if (id < 0 || ops[id].fate == 2) continue;
        ev_op[nev] = id;
        ev_ok[nev] = h->type[rows[i]] == LC_INVOKE ? 0 : 1;
        nev++;
    }
    free(ops); free(row_op);
    out->nops = nops; out->desc = desc; out->state_val = vals; out->nstates = nstates;
    out->nev = nev; out->ev_op = ev_op; out->ev_ok = ev_ok;
    return 0;
}

#endif /* ORACLE_KEYPREP_H */
