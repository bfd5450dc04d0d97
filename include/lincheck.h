/*
 * lincheck.h -- C ABI of the MI355X linearizability checker (liblincheck.so).
 *
 * Drop-in for the check phase of the Jepsen etcd demo:
 *
 *   (independent/checker
 *     (checker/compose
 *       {:linear (checker/linearizable {:model (model/cas-register)
 *                                       :algorithm :linear}) ...}))
 *
 * at /root/reference/src/jepsen/etcdemo.clj:115-119.  The reference path is
 * jepsen.independent/checker -> jepsen.checker/linearizable ->
 * knossos.linear/analysis (knossos 0.3.7, jepsen.etcdemo.iml:58), all Clojure.
 * Nothing in the reference is native, so every entry point below replaces a
 * Clojure function; each cites the reference call site it stands behind.
 *
 * Layers:
 *   lc_synth_*   synthetic cas-register histories with the demo's shape
 *                (etcdemo.clj:67-69, :83-105, :120-125).          [test input]
 *   lc_edn_*     Jepsen history.edn reader/writer (store/ layout,
 *                .gitignore:13; SURVEY F-1).                        [ingest]
 *   lc_pack      jepsen.independent/subhistory + knossos.history complete /
 *                without-failures + knossos.model.memo, producing packed
 *                per-key event streams (rows A1-A5).                 [host]
 *   lc_check_*   knossos.linear/analysis on the GPU (rows A6, A7) and the
 *                per-key verdict records jepsen.checker/linearizable and
 *                independent/checker turn into result maps (A8, A9). [device]
 *
 * Conventions: the caller owns every array it passes in or out.  The library
 * copies inputs to the device and never keeps caller pointers after a call
 * returns.  Every function returns 0 on success and a negative LC_E_* code on
 * failure; lc_last_error() (thread-local) describes the last failure.  The
 * library never calls exit() or abort().  One lc_ctx serialises its own calls
 * with an internal mutex; distinct contexts may run concurrently.
 */
#ifndef LINCHECK_H
#define LINCHECK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LC_ABI_VERSION 11

/* ---- error codes --------------------------------------------------------- */
#define LC_OK            0
#define LC_E_INVALID    -1  /* bad argument / malformed history               */
#define LC_E_NOMEM      -2  /* host or device allocation failed               */
#define LC_E_DEVICE     -3  /* HIP runtime error / no usable gfx950 device    */
#define LC_E_PARSE      -4  /* EDN syntax error                               */
#define LC_E_UNSUPPORTED -5 /* op the cas-register model cannot step          */
#define LC_E_IO         -6  /* file could not be read / written               */

/* ---- history vocabulary (etcdemo.clj:67-69, :83-105) --------------------- */
/* :type of an op map */
#define LC_INVOKE 0
#define LC_OK_T   1
#define LC_FAIL   2
#define LC_INFO   3
/* :f of an op map */
#define LC_F_READ  0
#define LC_F_WRITE 1
#define LC_F_CAS   2
#define LC_F_OTHER 3   /* nemesis :start/:stop and anything else */
#define LC_F_ACQUIRE 4 /* (model/mutex) :acquire                  */
#define LC_F_RELEASE 5 /* (model/mutex) :release                  */
#define LC_F_TXN     6 /* (model/multi-register) :txn            */

/* A :txn value is a sequence of micro-ops [f k v] (knossos.model/multi-register):
 * f LC_MOP_READ (v nil reads anything) or LC_MOP_WRITE, k a register id, v
 * an integer or LC_NIL.  lc_history.mop holds them as int64 triples. */
#define LC_MOP_READ  0
#define LC_MOP_WRITE 1
/* Register ids from LC_NAMED_REG_BASE up name non-integer registers (:x ...):
 * lc_edn_read gives the i-th distinct name LC_NAMED_REG_BASE + i
 * (lc_hist_reg_name). */
#define LC_NAMED_REG_BASE ((int64_t)1 << 62)

#define LC_NIL        INT64_MIN  /* a nil value                                */
#define LC_NO_KEY     INT64_MIN  /* :value is not an independent tuple [k v]   */
#define LC_NO_PROCESS INT64_MIN  /* :process is not an integer (:nemesis)      */

/*
 * A raw Jepsen history as struct-of-arrays, one row per op map, in history
 * order.  This is what the Clojure side marshals a `history` vector into
 * (INTEGRATION.md), what lc_edn_read produces and what lc_synth emits.
 *   key   the k of an independent tuple [k v] (jepsen.independent/tuple,
 *         etcdemo.clj:90,120) or LC_NO_KEY;
 *   v0/v1 the unwrapped v: read/write -> v0 (v1 = LC_NIL); cas [old new] ->
 *         v0 = old, v1 = new; LC_NIL for nil;
 *   index the op's :index, or -1 when the map has none.
 */
typedef struct lc_history {
    int64_t        n;
    const uint8_t *type;     /* LC_INVOKE / LC_OK_T / LC_FAIL / LC_INFO */
    const uint8_t *f;        /* LC_F_*                                   */
    const int64_t *process;  /* or LC_NO_PROCESS                         */
    const int64_t *key;      /* or LC_NO_KEY                             */
    const int64_t *v0;
    const int64_t *v1;
    const int64_t *index;    /* may be NULL: rows are then their own index */
    /* :txn values (LC_F_TXN rows; ABI 8).  Row r's micro-ops are the triples
     * mop[3*i .. 3*i+2] for i in [mop_off[r], mop_off[r + 1]); a row with an
     * empty range has a nil :value.  Both may be NULL when no row is a :txn. */
    const int64_t *mop_off;  /* [n + 1] or NULL */
    const int64_t *mop;      /* [3 * mop_off[n]] (f, register, value)       */
} lc_history;

/* ---- packed per-key event streams (rows A3-A5) ---------------------------- */
/*
 * Event word (u32), one per surviving client event of a key sub-history:
 *   bit 31      0 = :invoke, 1 = :ok completion
 *   bits 30..24 slot: the op's position in the key's pending window
 *               (lowest free slot at invoke, freed at :ok; crashed ops keep
 *               theirs forever)
 *   bits 23..0  invoke: transition id (index into trans[] after adding
 *               trans_off[key]); ok: 0
 * Failed ops (:fail) are gone (knossos.history/without-failures); :info
 * completions produce no event (the op stays callable forever).
 */
#define LC_EV_OK_BIT     0x80000000u
#define LC_EV_SLOT(e)    (((e) >> 24) & 0x7Fu)
#define LC_EV_TRANS(e)   ((e) & 0x00FFFFFFu)

/*
 * Transition descriptor (u32) = one interned cas-register op
 * (knossos.model/cas-register step, knossos.model.memo):
 *   bits 1..0   LC_T_READ_ANY (read of nil: legal in every state, no change)
 *               LC_T_READ  (legal iff state == a, no change)
 *               LC_T_WRITE (state := b)
 *               LC_T_CAS   (legal iff state == a, then state := b)
 *   bits 16..2  a (state id; LC_STATE_NONE = a value no op can produce)
 *   bits 31..17 b (state id)
 * State 0 is nil, the register's initial value ((model/cas-register) at
 * etcdemo.clj:117).
 */
#define LC_T_READ_ANY 0u
#define LC_T_READ     1u
#define LC_T_WRITE    2u
#define LC_T_CAS      3u
#define LC_STATE_NONE 0x7FFFu
#define LC_DESC(f, a, b) ((uint32_t)(f) | ((uint32_t)(a) << 2) | ((uint32_t)(b) << 17))

/* Table models ((model/multi-register), whose state is a map of registers):
 * lc_batch.table holds, per key, one row of key_states[key] u16 entries per
 * distinct op -- the next state id from each state, LC_TABLE_NONE when the
 * step is inconsistent -- and the op's descriptor trans[] entry is the offset
 * of its row in table[] (knossos.model.memo's state x transition table).
 * Such a batch needs trans_off and key_states. */
#define LC_TABLE_NONE 0xFFFFu

/* Limits of the packed form.  A key beyond them is reported :unknown with
 * cause LC_CAUSE_WINDOW / LC_CAUSE_STATES (identically in oracle/). */
#define LC_NARROW_MAX_SLOTS  56   /* u64 config: 8-bit state | 56 slot bits   */
#define LC_NARROW_MAX_STATES 255
#define LC_WIDE_MAX_SLOTS    112  /* 2 x u64 config                          */
#define LC_WIDE_MAX_STATES   32767

/* A packed batch: caller-visible view of lc_pack output or caller-built. */
typedef struct lc_batch {
    int64_t         n_keys;
    const uint64_t *ev_off;     /* [n_keys + 1] offsets into events          */
    const uint32_t *events;     /* [ev_off[n_keys]]                           */
    const uint32_t *trans;      /* transition descriptors                     */
    int64_t         n_trans;
    const uint32_t *trans_off;  /* [n_keys] per-key base into trans, or NULL  */
    const uint8_t  *key_width;  /* [n_keys] max slots used (1 + max slot), or NULL */
    const uint16_t *key_states; /* [n_keys] state ids used, or NULL           */
    uint32_t        init_state; /* state id of the initial value (0 = nil)    */
    const uint8_t  *key_error;  /* [n_keys] nonzero: the key's sub-history could
                                   not be prepared (lc_pack: knossos.history/
                                   complete's assertion, an op the model cannot
                                   step); the key is :unknown with cause
                                   LC_CAUSE_ERROR and its events are ignored --
                                   jepsen.checker/check-safe around that one key
                                   (etcdemo.clj:115).  NULL = no such key.       */
    const uint16_t *table;      /* [n_table] transition table of a table model
                                   (LC_TABLE_NONE above), or NULL: trans[] are
                                   LC_DESC descriptors (ABI 8)                 */
    int64_t         n_table;
    const uint16_t *events16;   /* [ev_off[n_keys]] or NULL: the same event
                                   words in 16 bits (LC_EV16_* below), given
                                   when every word fits; a register-tier batch
                                   then crosses the host link at 2 bytes per
                                   event and is widened on the device (ABI 8) */
} lc_batch;

/* 16-bit event word: bit 15 :ok, bits 14..11 slot (< 16), bits 10..0
 * transition id (< 2048).  Widened: LC_EV16_WIDE(e). */
#define LC_EV16_MAX_SLOT  15u
#define LC_EV16_MAX_TRANS 2047u
#define LC_EV16_WIDE(e) ((((uint32_t)(e) & 0x8000u) << 16) | ((((uint32_t)(e) >> 11) & 0xFu) << 24) | \
                         ((uint32_t)(e) & 0x7FFu))

/* The Knossos model a batch is checked against (knossos.model, SURVEY.md
 * 8(f) F-4).  The demo uses (model/cas-register) at etcdemo.clj:117; the
 * other two map onto the same transition descriptors:
 *   register     read / write of integer values (no cas)
 *   mutex        two states, unlocked (state 0, the initial one) and locked:
 *                :acquire = cas unlocked -> locked, :release = cas locked ->
 *                unlocked; :value is ignored                            */
#define LC_MODEL_CAS_REGISTER 0
#define LC_MODEL_REGISTER     1
#define LC_MODEL_MUTEX        2
/*   multi-register  knossos.model/multi-register: a map of registers, one
 *                :f :txn whose :value is a sequence of [:read k v] /
 *                [:write k v] micro-ops applied in order (a read of v legal
 *                iff v is nil or register k holds v).  States are the maps
 *                reachable from the initial one (memo), numbered per key; ops
 *                become rows of lc_batch.table.  A key with more than
 *                LC_WIDE_MAX_STATES reachable maps is :unknown (cause
 *                states).  An :ok completion's micro-ops replace the
 *                invocation's (a read learns what it read).             */
#define LC_MODEL_MULTI_REGISTER 3

typedef struct lc_pack_opts {
    int32_t model;     /* LC_MODEL_* (0 = cas-register) */
    int32_t n_init;    /* multi-register: initial registers, pairs        */
    const int64_t *init;  /* [2 * n_init] (register, value); others absent */
    uint32_t flags;    /* LC_PACK_* (ABI 11); 0 = the library's choice     */
} lc_pack_opts;

/* lc_pack_opts.flags: path pins for A/B runs and tests; the packed batch is
 * byte-identical whichever path builds it. */
#define LC_PACK_GENERAL 0x1u  /* always the bucketing path (rows of a key
                                 gathered through a row list), never the
                                 key-major one (each key's rows one run)   */

typedef struct lc_packed lc_packed;  /* library-owned */

/* jepsen.independent/checker's split (history-keys + subhistory, per
 * etcdemo.clj:115) followed by knossos.history/complete + without-failures
 * and model memoisation, for the cas-register model.  Keys appear in order
 * of first appearance.  Non-tuple ops belong to every key's sub-history
 * (jepsen.independent/subhistory keeps them): the nemesis's :info ops are
 * no-ops there, and any other op is paired and stepped in every key.
 *
 * Errors are per key, as independent/checker runs check-safe per key: a key
 * whose sub-history fails complete's assertion (a completion with no
 * outstanding invocation of its process) or holds an op the model cannot
 * step keeps its place with no events and key_error set (lc_batch), and the
 * other keys are packed as usual; lc_packed_key_error names the cause.
 * Only malformed arrays (bad :type / :f codes, missing pointers) fail the
 * whole call. */
int  lc_pack(const lc_history *h, const lc_pack_opts *opts, lc_packed **out);
void lc_packed_free(lc_packed *p);
/* Borrowed view of the packed arrays (valid until lc_packed_free). */
int  lc_packed_view(const lc_packed *p, lc_batch *out);
/* Independent key of packed key i. */
int64_t lc_packed_key(const lc_packed *p, int64_t i);
/* History row (0-based position in the lc_history) of event j of key i. */
int64_t lc_packed_event_row(const lc_packed *p, int64_t i, int64_t j);
/* Which lc_pack path built p (diagnostics, ABI 11): 1 = key-major (every
 * key's rows one run of the history), 0 = bucketing. */
int lc_packed_path(const lc_packed *p);
/* The history row of every event, in event order (ev_off's numbering);
 * out may be NULL to query the count (ABI 11). */
int64_t lc_packed_event_rows(const lc_packed *p, int64_t *out);
/* Number of history rows in key i's sub-history (incl. nemesis rows) and the
 * rows themselves (out may be NULL to query the count). */
int64_t lc_packed_subhistory(const lc_packed *p, int64_t i, int64_t *out_rows);
/* Why key i could not be prepared (NULL when it was; borrowed, valid until
 * lc_packed_free). */
const char *lc_packed_key_error(const lc_packed *p, int64_t i);
/* Register value of state id s of key i (state 0 = nil -> *is_nil = 1). */
int lc_packed_state_value(const lc_packed *p, int64_t i, uint32_t s, int64_t *value, int *is_nil);
/* Every key at once (n_keys entries), in packed order. */
int lc_packed_keys(const lc_packed *p, int64_t *out);
/* multi-register: the map state id s of key i stands for, as (register,
 * value) pairs in register order (a register the map lacks is absent; a
 * present nil is LC_NIL).  Writes at most cap pairs; returns how many the
 * state has. */
int64_t lc_packed_state_map(const lc_packed *p, int64_t i, uint32_t s, int64_t *regs, int64_t *vals, int64_t cap);

/* ---- Knossos-shaped result of one key -------- */
/* jepsen.checker/linearizable's result map (etcdemo.clj:117-118) for packed
 * key i, from its verdict record (valid, fail_event) and the final configs
 * the device returned for it (lc_result.final_configs + i * max_final * 2,
 * n_final[i]).  Ops are named by history rows (positions in the lc_history
 * given to lc_pack); an op is (invoke row, completion row or -1), from which
 * a binding builds the op map knossos.history/complete would (the
 * invocation, taking the completion's :value when it has none).  Model
 * states are register values (LC_NIL for nil; multi-register: state ids, see
 * lc_packed_state_map).  Writes int64 words:
 *   [0] :op row (the :ok that could not be linearized) or -1
 *   [1] :previous-ok row (= :last-op: the last :ok before it) or -1
 *   [2] n_configs (<= max_paths)   [3] n_paths (<= max_paths)
 *   per config: state, n_pending, n_pending x op, n_linearized, n_linearized x op
 *   per path:   start state (the :previous-ok step's model), n_steps,
 *               n_steps x (op, state after it), and the state in which the
 *               failing op is inconsistent (its "can't ..." message)
 * Paths (invalid keys only): from each final config, every sequence of
 * further pending ops the model allows, then the failing op; depth-first,
 * shortest first, in device config order, at most max_paths distinct ones
 * (Knossos iterates a hash set there: only the SET is comparable).  Returns
 * the number of words; nothing is written when that exceeds cap (call again
 * with a larger buffer). */
int64_t lc_report(const lc_packed *p, int64_t i, int32_t valid, int32_t fail_event, const uint64_t *final_configs,
                  uint32_t n_final, int32_t max_paths, int64_t *out, int64_t cap);
/* The same key shaped as knossos.wgl's analysis (:algorithm :wgl,
 * etcdemo.clj:118 slot; ABI 9; parity unpinned, restated in oracle/wgl_ref.py):
 * the same words, with :configs = the Wing-Gong search's frontier at the
 * return entry it is stuck on (the failing :ok) -- every (state, linearized
 * pending ops) reachable from the given final configs by linearizing further
 * pending ops other than the failing one, breadth first, at most max_paths. */
int64_t lc_report_wgl(const lc_packed *p, int64_t i, int32_t valid, int32_t fail_event,
                      const uint64_t *final_configs, uint32_t n_final, int32_t max_paths, int64_t *out, int64_t cap);

/* ---- device checking (rows A6-A9) ------------------------------------------ */
#define LC_ALGO_LINEAR      0  /* :algorithm :linear (etcdemo.clj:118)              */
#define LC_ALGO_WGL         1  /* :algorithm :wgl              */
#define LC_ALGO_COMPETITION 2  /* jepsen.checker/linearizable's default             */
/* LC_ALGO_LINEAR: knossos.linear's config-set search (the tiers T0-T3).
 * LC_ALGO_WGL (ABI 10): knossos.wgl's own search on the device -- the Wing &
 * Gong depth-first walk with Lowe's cache of (linearized set, state) pairs,
 * one wavefront per key; max_configs bounds the cache (more pairs: :unknown,
 * cause budget), so a key the :linear budget gives up on may still be decided
 * (and the other way round).  final_configs of an invalid key are the WGL
 * frontier at the return entry the walk is stuck on (the first max_final the
 * walk reaches), shaped by lc_report_wgl.  Restated in oracle/wgl_ref.py and
 * oracle/wgl_ref.c; parity with Knossos unpinned.
 * LC_ALGO_COMPETITION (knossos.competition races the two and takes the first
 * answer): the :linear search, then WGL for the keys :linear left :unknown at
 * its budget; lc_result.analyzer names the analysis each key's answer came
 * from. */

#define LC_MAX_DEVICES   8    /* devices one context drives (one node)        */
#define LC_COMM_ID_BYTES 128  /* an RCCL unique id (ncclUniqueId)             */

typedef struct lc_opts {
    int32_t  device;        /* HIP device ordinal (n_devices <= 1)              */
    int32_t  algorithm;     /* LC_ALGO_*                                        */
    uint64_t max_configs;   /* search budget B (0 = default 1<<20): a key whose
                               config set or JIT closure exceeds B configs is
                               :unknown (LC_CAUSE_BUDGET); replaces
                               knossos.search's heap-dependent abort (row A7)   */
    int32_t  max_final;     /* configs kept per invalid key (<= 16, default 10,
                               the truncation of jepsen.checker/linearizable)   */
    int32_t  lds_configs;   /* per-wave LDS frontier capacity (0 = default)     */
    int32_t  deep_slots;    /* concurrently searched HBM-tier keys (0 = auto)    */
    int32_t  flags;         /* LC_OPT_*                                          */
    int32_t  debug_mode;    /* 0 (ablation builds only)                          */
    /* One process, several GPUs (independent/checker's pmap over the node's
     * devices): n_devices in 2..LC_MAX_DEVICES checks every
     * batch as contiguous key shards of about equal event counts, one per
     * devices[g] (a device may repeat: shards then share it), all at once.
     * 0 or 1: `device` alone. */
    int32_t  n_devices;
    int32_t  devices[LC_MAX_DEVICES];
    /* One process per GPU (the launcher's ranks): comm_size > 1 makes this
     * context rank comm_rank of an RCCL communicator over comm_size ranks,
     * created here (ncclCommInitRank; it waits for every rank) from comm_id,
     * which rank 0 takes from lc_comm_id and hands to every rank (comm_size
     * 1 with a nonzero comm_id: a one-rank communicator).  lc_check_node
     * all-gathers the verdict records over it. */
    int32_t  comm_rank;
    int32_t  comm_size;
    uint8_t  comm_id[LC_COMM_ID_BYTES];
    /* Search-path choices (ABI 9, in the bytes ABI 8 reserved; all 0 =
     * automatic, the library's own choice per batch).  They pin one choice for
     * A/B measurements and tests, never change a result, and are read at
     * lc_create only: the caller's environment does not steer the kernels. */
    int32_t  path_flags;    /* LC_PATH_*                                         */
    int32_t  spec_segs;     /* speculative segments per key: 2, 3, 4, 6 or 8      */
    int32_t  spec_ck;       /* speculative checkpoints, events past a cut:
                               (ck1 + 1) | (ck2 + 1) << 16 (0: 32 and 120)      */
    int32_t  seg_len;       /* quiescent-point segments: events per segment      */
} lc_opts;

/* lc_opts.path_flags */
#define LC_PATH_SPLIT_ON     0x01  /* quiescent-point key segments where they apply  */
#define LC_PATH_SPLIT_OFF    0x02  /* never (else: when sampled keys say they pay)    */
#define LC_PATH_SPEC_OFF     0x04  /* no speculative key segments                     */
#define LC_PATH_LAYERS_OFF   0x08  /* HBM tier: config-keyed sets only (no T3L)       */
#define LC_PATH_NODE_SYNC    0x10  /* lc_check_node_async runs as lc_check_node        */
#define LC_PATH_NODE_STAGED  0x20  /* one rank: records through HBM, not device-mapped */
#define LC_PATH_CHUNKS_ON    0x40  /* lc_check_node: chunked upload whatever the size  */
#define LC_PATH_CHUNKS_OFF   0x80  /* lc_check_node: one upload whatever the size      */
#define LC_PATH_SPEC_COST    0x100 /* speculative cuts at equal estimated cost
                                      instead of equal event counts                 */
#define LC_PATH_EV32         0x200 /* upload 32-bit event words even when 16-bit ones
                                      are given (lc_batch.events16)                 */
#define LC_PATH_SPEC_NOPRIO  0x400 /* speculative walks: issue priority by wave age
                                      alone, not by progress                        */
#define LC_PATH_WGL_SMALL    0x800 /* WGL: Lowe's caches start in 2^14-entry tables
                                      (keys outgrowing them are searched again with a
                                      table the budget fits)                        */
#define LC_PATH_SPEC_NOSTAGE 0x1000 /* speculative segments: event words read from HBM
                                      by every run, not staged in LDS once per key  */
#define LC_PATH_WGL_EV_HBM   0x2000 /* WGL: every key's events read from HBM, none
                                       staged in LDS (tests of that walk; ABI 11)   */
#define LC_PATH_ALL          0x3FFF

/* lc_opts.flags */
#define LC_OPT_COUNT_PROBES 0x1  /* count successor-config probes (lc_stats.probes,
                                    SURVEY.md 8(d) D-4); off, the register-lattice
                                    tier skips the per-event popcounts          */

/* :valid? per key */
#define LC_VALID    1
#define LC_INVALID  0
#define LC_UNKNOWN -1

/* why a key ended */
#define LC_CAUSE_NONE    0  /* valid                                         */
#define LC_CAUSE_NONLIN  1  /* invalid: config set empty at fail_event       */
#define LC_CAUSE_BUDGET  2  /* unknown: > max_configs configs                 */
#define LC_CAUSE_WINDOW  3  /* unknown: > LC_WIDE_MAX_SLOTS ops pending       */
#define LC_CAUSE_STATES  4  /* unknown: > LC_WIDE_MAX_STATES register values  */
#define LC_CAUSE_ERROR   5  /* unknown: the key's sub-history could not be
                                   prepared (lc_batch.key_error; check-safe)   */

typedef struct lc_result {
    int8_t   *valid;         /* [n_keys] LC_VALID / LC_INVALID / LC_UNKNOWN         */
    int32_t  *fail_event;    /* [n_keys] event ordinal (within the key's stream) of
                                the :ok that could not be linearized, else -1       */
    uint8_t  *cause;         /* [n_keys] LC_CAUSE_*                                  */
    uint32_t *peak_configs;  /* [n_keys] max config-set size seen (may be NULL); a
                                key WGL answered: its cache size at the end       */
    uint64_t *final_configs; /* [n_keys * max_final * 2] (may be NULL): for invalid
                                keys, up to max_final configs of the last non-empty
                                set, as {state, slot mask lo} / {slot mask hi}      */
    uint32_t *n_final;       /* [n_keys] configs written to final_configs (may be NULL) */
    uint8_t  *analyzer;      /* [n_keys] LC_ALGO_LINEAR / LC_ALGO_WGL: the analysis
                                whose answer the key carries (may be NULL; ABI 10) */
} lc_result;

typedef struct lc_stats {
    double   kernel_ms;       /* device time of the search kernels (HIP events) */
    double   total_ms;        /* wall time of the call                          */
    uint64_t probes;          /* successor-config insert attempts (all tiers);
                                 0 unless lc_opts.flags has LC_OPT_COUNT_PROBES */
    uint64_t lds_keys;        /* keys finished in the LDS tier                  */
    uint64_t deep_keys;       /* keys (re)searched in the HBM tier              */
    uint64_t events;          /* events processed (0, like lds_keys, when the
                                 step was T0 alone: no counter readback)     */
    double   tier0_ms;        /* device time of the register-lattice tier alone */
    double   tier3_ms;        /* device time of the HBM tier launches (0 if none) */
    uint64_t probes_t3;       /* the part of `probes` made by the HBM tier      */
    uint64_t t3_bytes;        /* algorithmic HBM bytes of the layered HBM tier:
                                 8 per config-set entry it streams in or out
                                 (ABI 7)                                       */
    uint32_t t0_path;         /* the register tier's kernel this step (ABI 9):
                                 LC_T0_PATH_*                                   */
    uint32_t ev_word_bytes;   /* bytes per event word it read: 2 (lc_batch.events16
                                 read in place) or 4                            */
    double   wgl_ms;          /* device time of the WGL launches (ABI 10)       */
    uint64_t wgl_keys;        /* keys the WGL search answered                   */
    uint64_t wgl_spilled;     /* of those, keys searched again with a table the
                                 budget fits (they outgrew the shared tables)   */
    uint64_t wgl_steps;       /* WGL walk steps (linearizations + backtracks)   */
} lc_stats;

/* lc_stats.t0_path */
#define LC_T0_PATH_NONE      0  /* no register-tier launch (table model, no keys) */
#define LC_T0_PATH_LATTICE   1  /* k_search_lattice: one wave per key            */
#define LC_T0_PATH_SPEC      2  /* k_spec: speculative key segments              */
#define LC_T0_PATH_SEGMENTS  3  /* k_search_segments: quiescent-point segments    */

typedef struct lc_ctx lc_ctx;
typedef struct lc_dev_batch lc_dev_batch;

int         lc_abi_version(void);
const char *lc_last_error(void);
int         lc_device_count(void);
/* Give back the host blocks the library keeps for reuse (page-locked and
 * heap; up to 1 GB each, held after their arrays are freed).  Also done when
 * the last context is destroyed.  Arrays still in use are not touched. */
void        lc_trim(void);

int  lc_create(const lc_opts *opts, lc_ctx **out);
void lc_destroy(lc_ctx *ctx);

/* One call per batch: H2D, search, D2H into caller-owned result arrays.
 * Validation: every array index is checked before a kernel follows it.  The
 * per-event checks (an :ok names a pending slot, transition ids in range,
 * key_width / key_states honest) run on the device, one wave per key beside
 * the register tier (which stays in bounds on any input, and for a batch
 * declared to fit it refuses a key that does not); the set tiers that follow
 * trust the events, so over a refused batch they do nothing, and a malformed
 * key ends the call with LC_E_INVALID naming it.  A table model's batch
 * (lc_batch.table) is checked on the host, rows included.
 * The result arrays of a refused call are unspecified.  Event words in
 * page-locked memory (lc_pack's output on a GPU host) are uploaded directly;
 * others through a pinned staging copy. */
int  lc_check_batch(lc_ctx *ctx, const lc_batch *b, lc_result *r, lc_stats *s);

/* Device-resident batches: upload once, check many times (the bench's step). */
int  lc_upload(lc_ctx *ctx, const lc_batch *b, lc_dev_batch **out);
void lc_dev_batch_free(lc_dev_batch *db);
/* Search an uploaded batch.  flags:
 *   LC_DEV_RESULT  the result arrays in r are DEVICE pointers (e.g. torch
 *                  tensors for an RCCL all-gather) and nothing is copied back;
 *                  without it they are host arrays.
 *   LC_DEV_ASYNC   (with LC_DEV_RESULT) when the step is the register tier
 *                  alone (every key fits it, no probe counting), return once it
 *                  is enqueued on the context's stream: s is zeroed, and results
 *                  are ready after lc_wait.  Other steps run synchronously. */
#define LC_DEV_RESULT 1
#define LC_DEV_ASYNC  2
int  lc_check_device(lc_ctx *ctx, const lc_dev_batch *db, lc_result *r,
                     int flags, lc_stats *s);
/* Wait for every step enqueued on the context.  Returns the number of
 * LC_DEV_ASYNC steps since the previous lc_wait (or a negative LC_E_* code);
 * s->kernel_ms = their span (HIP events, first start .. last end) and
 * s->tier0_ms = span / count. */
int  lc_wait(lc_ctx *ctx, lc_stats *s);
/* Wait until the LC_DEV_ASYNC step `back` steps before the latest (0 = the
 * latest, at most 3) has finished, leaving later ones running; with no such
 * step on record, wait for everything on the context's stream.  Returns
 * LC_E_INVALID, naming the key, when a finished step's batch was malformed
 * (an error a later, still running step has raised already may be reported
 * here too); the error is cleared then. */
int  lc_wait_step(lc_ctx *ctx, int back);

/* ---- one process per GPU: node-wide verdict records ------- */
/* A key's verdict record: (valid + 1) | cause << 8 | (fail_event + 1) << 16
 * (8 bytes; 0 = padding).  Each rank checks its shard of the keys and the
 * records of every rank are all-gathered over RCCL (xGMI) -- the one
 * exchange step of the path; the shards share no state. */
#define LC_REC_VALID(r)      ((int)((r) & 0xFFu) - 1)
#define LC_REC_CAUSE(r)      ((int)(((r) >> 8) & 0xFFu))
#define LC_REC_FAIL_EVENT(r) ((int32_t)((int64_t)((r) >> 16) - 1))

/* A fresh RCCL unique id (LC_COMM_ID_BYTES) for lc_opts.comm_id; rank 0
 * calls it and the launcher distributes the bytes. */
int  lc_comm_id(uint8_t *out);
/* This rank's shard, from host SoA: upload, search, pack the shard's
 * records into a block of `block` (>= shard keys; padded with 0), all-gather
 * the blocks of every rank (comm_size of them, rank order), and copy the
 * node's block * comm_size records to `node` (host).  One rank: node = the
 * shard's block. */
int  lc_check_node(lc_ctx *ctx, const lc_batch *shard, int64_t block, uint64_t *node, lc_stats *s);
/* Pipelined lc_check_node.  A step that is the register tier alone
 * (every key fits it, no probe counting, node page-locked: lc_host_alloc)
 * is only enqueued and returns 1:
 * its upload overlaps the search of the step before it (two steps in flight)
 * and its records are in `node` once lc_wait (or lc_wait_step over it)
 * returns; errors surface there.  The shard's arrays and `node` must stay
 * untouched until then.  One rank (no communicator): the search writes the
 * records straight into `node` (device-mapped), and lc_node_records has none
 * of them.  Any other step runs as lc_check_node (returns 0). */
int  lc_check_node_async(lc_ctx *ctx, const lc_batch *shard, int64_t block, uint64_t *node, lc_stats *s);
/* Page-locked host memory (for lc_check_node_async's records). */
void *lc_host_alloc(size_t bytes);
void  lc_host_free(void *p);
/* The same from a resident shard (lc_upload), records left in HBM until
 * lc_node_records; flags LC_DEV_ASYNC: a step that is the register tier
 * alone is only enqueued (lc_wait ends the run). */
int  lc_check_node_device(lc_ctx *ctx, const lc_dev_batch *shard, int64_t block, int flags, lc_stats *s);
/* The first n records of the last gather (waits for it). */
int  lc_node_records(lc_ctx *ctx, uint64_t *node, int64_t n);

/* ---- synthetic histories ------------------------------ */
typedef struct lc_synth_opts {
    int64_t  n_keys;
    int64_t  ops_per_key;    /* client invocations per key (gen/limit, :125)     */
    int32_t  concurrency;    /* client threads per key (concurrent-generator 10) */
    int32_t  n_values;       /* values 0..n_values-1 (rand-int 5, :68-69)         */
    double   info_rate;      /* fraction of write/cas that complete :info         */
    double   info_effect_p;  /* probability a crashed op took effect              */
    double   anomaly_rate;   /* fraction of keys given one stale read / lost cas  */
    double   mean_think;     /* mean think time between a thread's ops            */
    double   mean_latency;   /* mean op latency                                   */
    int32_t  interleave;     /* 1: one time-ordered Jepsen history (keys in
                                sequence per thread group, tuples, :index);
                                0: key-major blocks                               */
    double   nemesis_period; /* > 0 and interleave: nemesis :info :start/:stop
                                every period (etcdemo.clj:138-143)                */
    uint64_t seed;
    int64_t  key_base;       /* first key id (shards of a larger key space)       */
} lc_synth_opts;

typedef struct lc_hist lc_hist;      /* library-owned history storage */
int  lc_synth_generate(const lc_synth_opts *o, lc_hist **out);
int  lc_hist_view(const lc_hist *h, lc_history *out);  /* borrowed view */
/* Keys the generator corrupted (anomaly_rate), ascending; out may be NULL to
 * query the count. */
int64_t lc_hist_anomalous_keys(const lc_hist *h, int64_t *out_keys);
void lc_hist_free(lc_hist *h);
/* Named registers of a history read by lc_edn_read: their count, and the
 * i-th name as written in the file (e.g. ":x"), or NULL past the end. */
int64_t     lc_hist_n_reg_names(const lc_hist *h);
const char *lc_hist_reg_name(const lc_hist *h, int64_t i);

/* ---- history.edn (Jepsen store format) ------------------------------------- */
/* Parse a Jepsen history.edn (one op map per line, or one vector of maps)
 * into an owned history.  Supports the op maps this workload produces:
 * :type :f :process :value (nil, ints, [k v] tuples, [old new]) :index :time
 * :error; other keys are skipped.  (model/multi-register) :f :txn values
 * [[:read k v] [:write k v] ...] (also :r / :w), optionally as [key txn]
 * tuples, fill lc_history.mop_off / mop: integer registers keep their ids,
 * other register names get LC_NAMED_REG_BASE + i.  lc_edn_write writes
 * :txn rows back, named registers as :r<i> keywords (lc_edn_write_named: by
 * their names). */
int  lc_edn_read(const char *path, lc_hist **out);
int  lc_edn_parse(const char *text, int64_t len, lc_hist **out);
int  lc_edn_write(const char *path, const lc_history *h);
/* lc_edn_write with named registers written back under their names:
 * reg_names[i] names register LC_NAMED_REG_BASE + i as lc_hist_reg_name gives
 * it (":x"); a name that is not one EDN token is written as :r<i>.  (ABI 9) */
int  lc_edn_write_named(const char *path, const lc_history *h, const char *const *reg_names, int64_t n_reg_names);

/* ---- test.fressian (Jepsen store format, binary) ---------------------------- */
/* Read the history out of a Fressian-encoded Jepsen test map (its :history
 * entry) or a Fressian list of op maps, with the op rules of lc_edn_read.
 * The decoder covers the whole Fressian encoding (caches, struct types,
 * chunked strings, open lists); tagged values of unknown handlers are kept
 * as their fields.  lc_fressian_write emits {:name "lincheck" :history [...]}.
 * Replaces the :history of jepsen.store's test.fressian load (SURVEY.md 8(f)
 * F-1); parity unpinned, no stored run or Fressian library to check against. */
int  lc_fressian_read(const char *path, lc_hist **out);
int  lc_fressian_parse(const uint8_t *buf, int64_t len, lc_hist **out);
int  lc_fressian_write(const char *path, const lc_history *h);

#ifdef __cplusplus
}
#endif
#endif /* LINCHECK_H */
