// device_wgl.hip -- knossos.wgl on the device: the Wing & Gong depth-first
// linearization search with Lowe's cache of (linearized set, model state)
// pairs, one wavefront per key (:algorithm :wgl, the slot at etcdemo.clj:118;
// SURVEY.md 8(f) F-3; the search north_star names).  Restated in
// oracle/wgl_ref.py (the list walk as knossos.wgl writes it) and
// oracle/wgl_ref.c; parity against Knossos itself is unpinned.
//
// The search is sequential by definition -- its :unknown (a cache of more
// than `budget` pairs) depends on the order it explores -- so a key's walk is
// the walk the restatement makes, step for step, and the parallelism is over
// keys (one wave each) and, within a key, over the ops pending at once (one
// lane per window slot: the candidates of a step are evaluated together).
//
// Representation (the same as oracle/wgl_ref.c):
//   a search node is (R, X, s): R the first return entry still in the list
//   (the :ok of the earliest op not linearized yet; every op returning before
//   R is linearized), X the window slots of the linearized ops pending at R,
//   s the model state.  (R, X) names the linearized set exactly, so Lowe's
//   cache is a set of (R, X, s).
//   The list walk from the head visits the call entries of the ops pending at
//   R and not linearized, in invoke order, then stops at R.  A node's
//   candidates are therefore those slots (pending mask minus X), tried in
//   order of their :invoke; a candidate is taken when the model can step it
//   and its child (R', X', s') is not cached.  Taking the op of R itself
//   moves R to the next :ok whose op is not linearized (the ops returning in
//   between leave X).
//
// One probe round per node.  The cache status of a node's candidates is read
// once, when the node is first reached (every candidate probed at once, one
// lane each), and kept in its frame: while the subtree of a candidate c is
// searched, every pair cached there has c in its linearized set, and no
// other candidate's child has, so the remaining candidates' status cannot
// change before the walk comes back.  A backtrack therefore costs a frame
// load and no probe; a step down costs one probe round (plus, when resuming
// a node, one coalesced read of 64 consecutive table entries to find the
// insertion slot, which the subtree may have taken).
//
// Memory per resident wave (lcd::WglWs): Lowe's cache, an open-addressed
// table of 32-byte entries {X lo, X hi, R, s, stamp} in HBM, at most half
// full (sized from the budget); an entry belongs to the current key when its
// stamp is the key's (launch << 32 | ticket + 1), so tables are never
// cleared between keys or launches.  The frame stack (64 B per level; depth
// <= ops of the key) in HBM.  The key's event words and, per :invoke event,
// the :invoke that held its window slot before it (to undo a move of R) in
// LDS for the first `lds_events` events, in HBM beyond.

#include "device_common.hpp"

namespace lcd {
namespace {

constexpr uint32_t WGL_END = 0xFFFFFFFFu;  // R past the last return: every :ok passed
constexpr uint32_t WGL_NONE = 0xFFFFFFFFu; // no :invoke (prev of a slot's first op)
constexpr uint32_t WGL_RING = 32;          // frames of the walk's top levels kept in LDS
constexpr uint32_t WGL_PEND_LANES = 8;     // HBM tier: entries read for the pending pair's slot with the probes

extern "C" __device__ int lc_wgl_writelane(int x, int l, int v) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ uint32_t wsetl(uint32_t v, uint32_t l, uint32_t x) {
    return (uint32_t)lc_wgl_writelane((int)x, (int)l, (int)v);
}
__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t uni64(uint64_t x) {
    return (uint64_t)uni((uint32_t)x) | (uint64_t)uni((uint32_t)(x >> 32)) << 32;
}
__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

__device__ __forceinline__ bool mbit(uint64_t lo, uint64_t hi, uint32_t s) {
    return ((s < 64 ? lo : hi) >> (s & 63)) & 1ull;
}
// (written as selects of both words: a branch between the two references
// made the compiler keep the pair in scratch memory, indexed by s >> 6)
__device__ __forceinline__ void mset(uint64_t &lo, uint64_t &hi, uint32_t s) {
    const uint64_t b = 1ull << (s & 63u);
    lo |= s < 64 ? b : 0ull;
    hi |= s < 64 ? 0ull : b;
}
__device__ __forceinline__ void mclr(uint64_t &lo, uint64_t &hi, uint32_t s) {
    const uint64_t b = 1ull << (s & 63u);
    lo &= s < 64 ? ~b : ~0ull;
    hi &= s < 64 ? ~0ull : ~b;
}

// Table hash of a pair (R, X, s).  X enters through its Zobrist code zx =
// XOR of zob(slot) over the slots in X, which the walk keeps as X changes
// (one XOR per slot added or dropped; a frame holds its node's code) -- a
// candidate's child is then zx ^ zob(its slot), and a pair costs one 32-bit
// finalizer instead of four 64-bit products per lane.
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h;
}
__device__ __forceinline__ uint32_t zob(uint32_t slot) { return fmix32(slot * 0x9E3779B9u + 0x7F4A7C15u); }
__device__ __forceinline__ uint32_t wgl_hash(uint32_t R, uint32_t s, uint32_t zx) {
    return fmix32(zx ^ (R * 0x27D4EB2Fu) ^ (s * 0x165667B1u + 0x61C88647u));
}

// The walk's slot sets live one bit per lane: lane l holds, for window slots
// l and l + 64, whether each is linearized (X: bits 0, 1), pending at R (P:
// bits 2, 3) and still a candidate of the node (C: bits 4, 5) -- one VGPR
// instead of six 64-bit scalar pairs, which left the kernel's scalar file
// spilling into VGPR lanes on every step.
constexpr uint32_t LM_X = 0, LM_P = 2, LM_C = 4;
__device__ __forceinline__ uint32_t lm_bit(uint32_t lm, uint32_t sl, uint32_t base) {  // sl uniform
    return (rdl(lm, sl & 63u) >> (base + (sl >> 6))) & 1u;
}
__device__ __forceinline__ uint32_t lm_one(uint32_t sl, uint32_t base) {  // this lane's bit of slot sl
    return __lane_id() == (sl & 63u) ? 1u << (base + (sl >> 6)) : 0u;
}

struct Frame {  // one level of the walk: the node a step down left (80 B)
    uint32_t R, s, zx, pad;  // zx: X's Zobrist code
    uint8_t m[64];           // per lane: its X / P / C bits (C: candidates still to try)
};
constexpr uint32_t FRAME_WORDS = sizeof(Frame) / 4;

extern "C" __device__ uint32_t __ockl_wfred_min_u32(uint32_t);

// Diagnostic build only (make variant NAME=wglprof VFLAGS=-DLC_WGL_PROF):
// cycles of the walk's phases summed over keys (tools/wgl_prof.py reads them
// back through lc_debug_wgl_prof): [0] staging, [1] probe rounds, [2] child
// scans inside them, [3] backtracks, [4] steps down before advance, [5]
// advances, [6] probe-loop iterations, [7] steps.
#ifndef LC_WGL_ADOPT
#define LC_WGL_ADOPT 1
#endif
#ifdef LC_WGL_PROF
__device__ unsigned long long lc_wgl_prof[8];
#define WP_DECL uint64_t wp[8] = {0, 0, 0, 0, 0, 0, 0, 0}; uint64_t wp_t = __builtin_amdgcn_s_memtime();
#define WP_MARK(i) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); wp[i] += t_ - wp_t; wp_t = t_; } while (0)
#define WP_ADD(i, x) do { wp[i] += (x); } while (0)
#define WP_DUMP() do { if (__lane_id() == 0) for (int q_ = 0; q_ < 8; ++q_) atomicAdd(&lc_wgl_prof[q_], (unsigned long long)wp[q_]); } while (0)
#else
#define WP_DECL
#define WP_MARK(i) do {} while (0)
#define WP_ADD(i, x) do {} while (0)
#define WP_DUMP() do {} while (0)
#endif

// The block's dynamic LDS (one wave per block): from word 0, the key's first
// E = lds_events event words, then per event the :invoke that held its slot
// before it (prev), then per event its transition descriptor (0 for an :ok);
// the LDS tier of the cache (lds_tab u64); the frame ring (WGL_RING x 16
// words).  Declared here, not passed as a pointer, so its accesses are LDS
// instructions rather than flat ones.
extern __shared__ uint32_t wgl_lds[];

// The key's events, their slot history and descriptors: all in LDS (LDS:
// the key fits lds_events), else all in HBM.  (One source per key: written
// as a per-event choice, the compiler merged the two loads into one flat
// load through a selected pointer.)
template <bool LDS>
struct KeyIo {
    const uint32_t *gev;   // the key's event words (HBM)
    uint32_t *gprev;       // prev (HBM form)
    const uint32_t *trans; // the key's transition descriptors (HBM form)
    uint32_t ntr;          // entries of trans
    uint32_t E;            // LDS layout stride (lds_events)
    __device__ __forceinline__ uint32_t ev(uint32_t j) const { return uni(LDS ? wgl_lds[j] : gev[j]); }
    __device__ __forceinline__ uint32_t prev(uint32_t j) const { return uni(LDS ? wgl_lds[E + j] : gprev[j]); }
    __device__ __forceinline__ void set_prev(uint32_t j, uint32_t v) const {
        if (__lane_id() == 0) {
            if (LDS) wgl_lds[E + j] = v;
            else gprev[j] = v;
        }
    }
    // the descriptor of :invoke event j
    __device__ __forceinline__ uint32_t dsc(uint32_t j) const {
        if (LDS) return uni(wgl_lds[2 * E + j]);
        const uint32_t t = LC_EV_TRANS(uni(gev[j]));
        return t < ntr ? uni(trans[t]) : 0u;
    }
    // per lane: event j (this lane's; j < n), its slot's previous :invoke and,
    // for an :invoke, its descriptor
    __device__ __forceinline__ uint32_t ev_at(uint32_t j) const { return LDS ? wgl_lds[j] : gev[j]; }
    __device__ __forceinline__ uint32_t prev_at(uint32_t j) const { return LDS ? wgl_lds[E + j] : gprev[j]; }
    __device__ __forceinline__ uint32_t dsc_at(uint32_t j, uint32_t w) const {
        if (LDS) return wgl_lds[2 * E + j];
        const uint32_t t = LC_EV_TRANS(w);
        return (!(w & LC_EV_OK_BIT) && t < ntr) ? trans[t] : 0u;
    }
};

// A forward scan's window of 64 events (and their descriptors) held one per
// lane: a scan reads each event with a v_readlane instead of waiting on one
// memory round trip per event.
template <bool LDS, bool DSC>
struct EvWindow {
    const KeyIo<LDS> &io;
    uint32_t n, base = 0x80000000u, w = 0, d = 0;  // (base: no window yet -- j - base >= 64 for every j < 2^31)
    __device__ __forceinline__ EvWindow(const KeyIo<LDS> &io_, uint32_t n_) : io(io_), n(n_) {}
    __device__ __forceinline__ void at(uint32_t j) {  // j uniform, < n
        if (j - base >= 64u) {
            base = j;
            const uint32_t k = j + __lane_id();
            w = k < n ? io.ev_at(k) : 0u;
            if (DSC) d = k < n ? io.dsc_at(k, w) : 0u;
        }
    }
    __device__ __forceinline__ uint32_t ev(uint32_t j) { at(j); return rdl(w, j - base); }
    __device__ __forceinline__ uint32_t dsc(uint32_t j) { at(j); return rdl(d, j - base); }
};

// A backward scan's window (a backtrack's restore): per lane an event, its
// slot's previous :invoke and that :invoke's descriptor -- the gather of the
// descriptors done by all lanes at once.
template <bool LDS>
struct EvWindowRev {
    const KeyIo<LDS> &io;
    uint32_t base = 0x80000000u, w = 0, pv = 0, pd = 0;  // (no window yet, as EvWindow)
    __device__ __forceinline__ explicit EvWindowRev(const KeyIo<LDS> &io_) : io(io_) {}
    __device__ __forceinline__ void at(uint32_t j) {  // j uniform, < n
        if (j - base >= 64u) {
            base = j >= 63u ? j - 63u : 0u;
            const uint32_t k = base + __lane_id();  // <= j < n for the lanes read
            w = k <= j ? io.ev_at(k) : LC_EV_OK_BIT;
            pv = (!(w & LC_EV_OK_BIT)) ? io.prev_at(k) : WGL_NONE;
            pd = pv != WGL_NONE ? io.dsc_at(pv, io.ev_at(pv)) : 0u;
        }
    }
};

// The launch's arguments as the kernarg segment holds them, through an
// opaque pointer: the result arrays and lists the walk touches once per key
// are loaded where they are used.  (Read through the kernel's by-value
// parameter, every field used anywhere is loaded at the kernel's entry and
// stays in a scalar register for the whole walk: the scalar file spilled into
// VGPR lanes, and every step paid the reloads.)
using KargWgl = const __attribute__((address_space(4))) WglArgs;
__device__ __forceinline__ KargWgl &cold_args() {
    KargWgl *p = (KargWgl *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *p;
}

__device__ __forceinline__ void wgl_finish(const WglArgs &, int32_t key, int verdict, int cause, int32_t fev,
                                           uint32_t cache_n, uint32_t n_front, uint64_t steps, uint64_t lookups = 0) {
    KargWgl &a = cold_args();
    if (__lane_id() == 0) {
        if (a.probes) atomicAdd(a.probes, (unsigned long long)lookups);
        a.valid[key] = (int8_t)verdict;
        a.cause[key] = (uint8_t)cause;
        a.fail_event[key] = fev;
        if (a.peak) a.peak[key] = cache_n;
        if (a.n_final) a.n_final[key] = verdict == LC_INVALID ? n_front : 0u;
        if (a.analyzer) a.analyzer[key] = (uint8_t)LC_ALGO_WGL;
        if (a.rec)
            a.rec[key] = (uint64_t)(uint8_t)(verdict + 1) | (uint64_t)(uint8_t)cause << 8 |
                         (uint64_t)(uint32_t)(fev + 1) << 16;
        atomicAdd(a.ev_count, (unsigned long long)steps);
        atomicAdd(a.keys_done, 1ull);
    }
}

// Search one key (the whole wave).  Every lane runs the same control flow:
// every branch below is on a wave-uniform value.  LDS: the key's events fit
// the block's LDS (lds_events).
// WIDE: the key's window reaches slot 64 (the second slot of each lane is in
// use); without, every slot-64-127 term is the constant zero and drops out of
// the walk (a lone wave per SIMD issues an instruction per 4 cycles, so the
// walk's time is its instruction count).  Returns false when a narrow walk
// finds a slot >= 64 its key_width did not declare (the caller walks it wide).
template <bool LDS, bool WIDE>
__device__ bool wgl_key(const WglArgs &a, int32_t key, uint32_t ticket, char *slot_ws) {
    const uint32_t lane = __lane_id();
    WP_DECL
    const uint64_t eb = a.ev_off[key];
    const uint32_t n = (uint32_t)(a.ev_off[key + 1] - eb);
    if (a.key_error && a.key_error[key]) {
        wgl_finish(a, key, LC_UNKNOWN, LC_CAUSE_ERROR, -1, 0, 0, 0);
        return true;
    }
    if (a.key_states && a.key_states[key] > LC_WIDE_MAX_STATES) {
        wgl_finish(a, key, LC_UNKNOWN, LC_CAUSE_STATES, -1, 0, 0, 0);
        return true;
    }
    const uint32_t tb = a.trans_off ? a.trans_off[key] : 0u;
    const uint64_t gen = a.gen_base | (uint64_t)(ticket + 1u);
    uint4 *tab = (uint4 *)slot_ws;  // 2 x uint4 per entry
    Frame *frames = (Frame *)(slot_ws + a.ws.off_frames);
    KeyIo<LDS> io;
    io.gev = a.events + eb;
    io.gprev = (uint32_t *)(slot_ws + a.ws.off_prev);
    io.ntr = a.n_trans > tb ? a.n_trans - tb : 0u;
    io.trans = a.trans + (io.ntr ? tb : 0u);
    io.E = a.lds_events;
    // Stage the events and their descriptors (LDS part), and look for an
    // :invoke the window cannot hold (slot >= LC_WIDE_MAX_SLOTS): the key is
    // then :unknown "window" at the first such :invoke, before any search
    // (as the restatement).
    uint32_t win_ev = WGL_END;
    bool past64 = false;  // an :invoke into slot >= 64
    for (uint32_t base = 0; base < n; base += 64) {
        const uint32_t j = base + lane;
        uint32_t w = 0;
        if (j < n) w = io.gev[j];
        if (LDS && j < n) {
            const uint32_t t = LC_EV_TRANS(w);
            wgl_lds[j] = w;
            wgl_lds[2 * io.E + j] = (!(w & LC_EV_OK_BIT) && t < io.ntr) ? io.trans[t] : 0u;
        }
        const bool wide = j < n && !(w & LC_EV_OK_BIT) && LC_EV_SLOT(w) >= LC_WIDE_MAX_SLOTS;
        if (!WIDE) past64 = past64 || ballot(j < n && !(w & LC_EV_OK_BIT) && LC_EV_SLOT(w) >= 64u) != 0;
        const uint64_t m = ballot(wide);
        if (m && win_ev == WGL_END) win_ev = base + (uint32_t)__builtin_ctzll(m);
    }
    __syncthreads();
    if (!WIDE && past64 && win_ev == WGL_END) return false;
    if (win_ev != WGL_END) {
        wgl_finish(a, key, LC_UNKNOWN, LC_CAUSE_WINDOW, (int32_t)win_ev, 0, 0, 0);
        return true;
    }
    // per lane: the op holding window slot `lane` (occ0, dsc0) and `lane + 64`
    // (occ1, dsc1) at R -- its :invoke event and its transition descriptor
    uint32_t occ0 = WGL_NONE, occ1 = WGL_NONE, dsc0 = 0, dsc1 = 0;
    uint32_t lm = 0;  // this lane's X / P / C bits
    uint32_t zx = 0;  // Zobrist code of X
    const uint32_t zl0 = zob(lane), zl1 = zob(lane + 64u);  // this lane's slots' codes
    uint32_t s = a.init_state;
    uint32_t R = WGL_END;
    // Move R forward from `from` (the op of R already in X): the :oks of ops
    // in X leave X and the pending set; the :invokes passed become pending.
    auto advance = [&](uint32_t from) {
        R = WGL_END;
        EvWindow<LDS, true> win(io, n);
        for (uint32_t j = from; j < n; ++j) {
            const uint32_t w = win.ev(j);
            const uint32_t sl = LC_EV_SLOT(w);
            if (w & LC_EV_OK_BIT) {
                if (lm_bit(lm, sl, LM_X)) {
                    lm &= ~(lm_one(sl, LM_X) | lm_one(sl, LM_P));
                    zx ^= zob(sl);
                    continue;
                }
                R = j;
                break;
            }
            const uint32_t d = win.dsc(j);
            const uint32_t l = sl & 63u;
            if (!WIDE || sl < 64) { io.set_prev(j, rdl(occ0, l)); occ0 = wsetl(occ0, l, j); dsc0 = wsetl(dsc0, l, d); }
            else { io.set_prev(j, rdl(occ1, l)); occ1 = wsetl(occ1, l, j); dsc1 = wsetl(dsc1, l, d); }
            lm |= lm_one(sl, LM_P);
        }
    };
    advance(0);
    // ---- Lowe's cache ----
    // Narrow keys (<= 24 window slots, < 2^24 - 1 events) start in an LDS
    // table of 8-byte entries, X | s << 24 | R << 39 (R = n for the end of
    // the list; all ones = empty), and move to the HBM table when it is half
    // full; other keys use the HBM table from the start.
    const uint32_t mask = a.ws.tab_mask;
    const bool narrow = a.lds_tab != 0 && a.key_width && a.key_width[key] <= 24u && n < (1u << 24) - 1u;
    bool in_lds = narrow;
    uint64_t *const ltab = (uint64_t *)(wgl_lds + 3 * a.lds_events);
    uint32_t *const lfr = wgl_lds + 3 * a.lds_events + 2 * a.lds_tab;  // frame ring: WGL_RING frames
    const uint32_t lmask = a.lds_tab - 1u;
    if (in_lds) {
        for (uint32_t i = lane; i < a.lds_tab; i += 64) ltab[i] = ~0ull;
        __syncthreads();
    }
    auto lkey = [&](uint32_t R_, uint32_t s_, uint64_t x_) -> uint64_t {
        return (x_ & 0xFFFFFFull) | (uint64_t)s_ << 24 | (uint64_t)(R_ == WGL_END ? n : R_) << 39;
    };
    // Move every LDS entry to the HBM table (the LDS tier is half full):
    // lanes insert at once, a slot claimed by raising its stamp to this key's
    // (stamps only grow, so a larger old stamp is impossible and an equal one
    // is another entry of this key).
    auto migrate = [&]() {
        for (uint32_t i = lane; i < a.lds_tab; i += 64) {
            const uint64_t e = ltab[i];
            if (e == ~0ull) continue;
            const uint32_t eR0 = (uint32_t)(e >> 39), es = (uint32_t)(e >> 24) & 0x7FFFu;
            const uint32_t eR = eR0 == n ? WGL_END : eR0;
            const uint64_t ex = e & 0xFFFFFFull;
            uint32_t ez = 0;
            for (uint64_t m = ex; m; m &= m - 1) ez ^= zob((uint32_t)__builtin_ctzll(m));
            uint32_t h = wgl_hash(eR, es, ez) & mask;
            for (uint32_t probe = 0; probe <= mask; ++probe) {
                unsigned long long *g = (unsigned long long *)(tab + 2 * (size_t)h + 1) + 1;
                const unsigned long long old = atomicMax(g, (unsigned long long)gen);
                if (old != gen) {
                    tab[2 * (size_t)h] = make_uint4((uint32_t)ex, 0u, 0u, 0u);
                    uint32_t *w1 = (uint32_t *)(tab + 2 * (size_t)h + 1);
                    w1[0] = eR;
                    w1[1] = es;
                    break;
                }
                h = (h + 1) & mask;
            }
        }
        // the lines this CU's L1 may hold were written at the memory side
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        in_lds = false;
    };
    uint32_t depth = 0, cache_n = 0, n_front = 0;
    uint32_t ring_lo = 0;  // frames [ring_lo, depth) are in the LDS ring too
    uint32_t deepest = WGL_NONE;  // the deepest return entry the walk got stuck on
    uint64_t steps = 0;
    uint64_t lookups = 0;    // cache lookups: one per legal candidate of a probe round
    bool fresh = true;       // the current node has not been probed yet
    // the child the op of R leads to, as its probe round moved R there (valid
    // for a step down in the same iteration as the probe)
    bool have_child = false;
    uint32_t ch_lm = 0, ch_occ0 = 0, ch_occ1 = 0, ch_dsc0 = 0, ch_dsc1 = 0, ch_R = 0, ch_z = 0;
    bool have_pos = false;   // ipos0/1 are insertion slots (nothing inserted since the probe)
    uint32_t ipos0 = 0, ipos1 = 0;
    // the last step down's pair, inserted during the next probe round (its
    // slot search shares that round's wait); pend_pos known when the probe
    // that chose it found its slot.  The pending pair is always the node of
    // the probe round that inserts it (the node the step down reached).
    bool pend = false, pend_known = false;
    uint32_t pend_pos = 0;
    // hard bound on the loop: every step down inserts a new pair, so a walk
    // takes at most 2 (budget + 1) steps; the bound only guards the kernel
    const uint64_t max_it = 2 * (a.budget + 2) + 4;
    WP_MARK(0);
    for (uint64_t it = 0; it < max_it; ++it) {
        // ---- candidates of the current node ----
        const bool has_R = R != WGL_END;
        const uint32_t rs = has_R ? LC_EV_SLOT(io.ev(R)) : 0xFFu;
        if (fresh) {
            fresh = false;
            // X as two scalar words (keys, the pending pair)
            const uint64_t xlo = ballot(lm & 1u), xhi = WIDE ? ballot(lm & 2u) : 0ull;
            const uint32_t sl0 = lane, sl1 = lane + 64u;
            uint32_t s20 = 0, s21 = 0;
            const bool ok0 = (lm & 4u) && !(lm & 1u) && step(a.table, s, dsc0, s20);
            const bool ok1 = WIDE && (lm & 8u) && !(lm & 2u) && step(a.table, s, dsc1, s21);
            const bool r_ok = has_R && ((ballot(rs < 64 ? ok0 : ok1) >> (rs & 63)) & 1ull);
            lookups += (uint64_t)__builtin_popcountll(ballot(ok0)) + (WIDE ? (uint64_t)__builtin_popcountll(ballot(ok1)) : 0ull);
            // the child reached by taking the op of R: R moves on (tentatively;
            // the ops returning in between leave X)
            uint32_t R2 = WGL_END, z2 = 0;
            uint64_t x2lo = 0, x2hi = 0;
            have_child = false;
            if (r_ok) {
                // narrow walks: the whole move of R (the advance a step down
                // taking R's op makes), into the child's own lane state: the
                // step down adopts it instead of scanning again (the
                // :invokes' prev words written on the way are functions of the
                // event alone).  Wide walks: only the child's key (the :oks)
                // -- with many candidates R's op is seldom the one taken, and
                // the whole scan is wasted (C2: 8.33 -> 8.07 ms with it, C4,
                // mostly wide: 201 -> 220 ms; gating it on R's op having the
                // earliest legal :invoke, two wave minima per round: 8.37 /
                // 225 ms).  LC_WGL_ADOPT (A/B): 0 never, 2 every walk.
                WP_MARK(1);
                constexpr uint32_t whole = LC_WGL_ADOPT == 2 ? 1u : LC_WGL_ADOPT == 1 ? (WIDE ? 0u : 1u) : 0u;
                uint32_t x2 = (lm & 0xFu) | lm_one(rs, LM_X);
                uint32_t o0 = occ0, o1 = occ1, d0 = dsc0, d1 = dsc1;
                z2 = zx ^ zob(rs);
                EvWindow<LDS, true> win(io, n);
                for (uint32_t j = R; j < n; ++j) {
                    const uint32_t w = win.ev(j);
                    const uint32_t sl = LC_EV_SLOT(w);
                    if (w & LC_EV_OK_BIT) {
                        if (lm_bit(x2, sl, LM_X)) {
                            x2 &= ~(lm_one(sl, LM_X) | lm_one(sl, LM_P));
                            z2 ^= zob(sl);
                            continue;
                        }
                        R2 = j;
                        break;
                    }
                    if (!whole) continue;
                    const uint32_t d = win.dsc(j);
                    const uint32_t l = sl & 63u;
                    if (!WIDE || sl < 64) { io.set_prev(j, rdl(o0, l)); o0 = wsetl(o0, l, j); d0 = wsetl(d0, l, d); }
                    else { io.set_prev(j, rdl(o1, l)); o1 = wsetl(o1, l, j); d1 = wsetl(d1, l, d); }
                    x2 |= lm_one(sl, LM_P);
                }
                x2lo = ballot(x2 & 1u);
                x2hi = WIDE ? ballot(x2 & 2u) : 0ull;
                ch_lm = x2; ch_occ0 = o0; ch_occ1 = o1; ch_dsc0 = d0; ch_dsc1 = d1; ch_R = R2; ch_z = z2;
                have_child = whole != 0;
                WP_MARK(2);
            }
            // each candidate's child key
            uint64_t k0lo = xlo, k0hi = xhi, k1lo = xlo, k1hi = xhi;
            mset(k0lo, k0hi, sl0);
            mset(k1lo, k1hi, sl1);
            uint32_t kR0 = R, kR1 = R, kz0 = zx ^ zl0, kz1 = zx ^ zl1;
            if (sl0 == rs) { kR0 = R2; k0lo = x2lo; k0hi = x2hi; kz0 = z2; }
            if (sl1 == rs) { kR1 = R2; k1lo = x2lo; k1hi = x2hi; kz1 = z2; }
            const uint32_t h0 = wgl_hash(kR0, s20, kz0), h1 = wgl_hash(kR1, s21, kz1);
            // (0/1 words, not bools: a bool carried around a loop becomes a
            // lane mask in scalar pairs, merged with EXEC at every step)
            uint32_t act0 = ok0 ? 1u : 0u, act1 = ok1 ? 1u : 0u, hit0 = 0, hit1 = 0;
            uint32_t p0, p1;
            // the pending pair's slot search: 64 entries from its home, read
            // beside the first probes
            const uint32_t ph = wgl_hash(R, s, zx);
            bool pfree = false;
            if (in_lds) {
                const uint64_t q0 = lkey(kR0, s20, k0lo), q1 = lkey(kR1, s21, k1lo);
                p0 = h0 & lmask;
                p1 = h1 & lmask;
                if (pend && !pend_known) pfree = ltab[(ph + lane) & lmask] == ~0ull;
                // (branch-free per lane: every lane reads its two slots, a
                // finished probe just stops moving -- no EXEC-mask juggling)
                for (uint32_t probe = 0; probe <= lmask; ++probe) {
                    if (!ballot((act0 | act1) != 0u)) break;
                    WP_ADD(6, 1);
                    const uint64_t e0 = ltab[p0], e1 = ltab[p1];
                    const uint32_t eq0 = e0 == q0 ? 1u : 0u, eq1 = e1 == q1 ? 1u : 0u;
                    const uint32_t em0 = e0 == ~0ull ? 1u : 0u, em1 = e1 == ~0ull ? 1u : 0u;
                    hit0 |= act0 & eq0;
                    hit1 |= act1 & eq1;
                    act0 &= ~(eq0 | em0) & 1u;
                    act1 &= ~(eq1 | em1) & 1u;
                    p0 = (p0 + act0) & lmask;
                    p1 = (p1 + act1) & lmask;
                }
            } else {
                p0 = h0 & mask;
                p1 = h1 & mask;
                // (the stamp words of the first WGL_PEND_LANES entries from
                // its home: all 64 read 2 KB of lines per probe round, 5x the
                // walk's algorithmic bytes, for a slot that is nearly always
                // among the first few).  Loaded here and compared after the
                // probe loop, so the load shares the probes' wait: compared
                // at once, the compiler waited for it before the first probe
                // -- a serial round trip of its own at every probe round
                // after a backtrack (round 6).
                // (every lane loads, with no branch around it: a slot when the
                // pair's slot is wanted, else entry 0's stamp, a line that
                // stays cached -- a load under a lane condition drew the
                // compiler's copies, and their wait, into the branch)
                const bool want_ps = pend && !pend_known && lane < WGL_PEND_LANES;
                const size_t ps_at = pend && !pend_known ? (size_t)((ph + (lane & (WGL_PEND_LANES - 1u))) & mask) : 0u;
                const uint2 ps = *((const uint2 *)(tab + 2 * ps_at + 1) + 1);
                // (one entry per round trip: reading two, p and p + 1, was
                // measured in round 5 -- C2 8.21 -> 8.54 ms, C4 at 2^16 204 ->
                // 208 ms, at 2^20 3,255 -> 3,187 ms; not kept)
                for (uint32_t probe = 0; probe <= mask; ++probe) {
                    if (!ballot((act0 | act1) != 0u)) break;
                    WP_ADD(6, 1);
                    // Both candidates' entries loaded without a branch and
                    // every field of both compared with bitwise ANDs, so the
                    // loads go out together and share one wait.  Loaded under
                    // `if (act0)` / `if (act1)`, or compared with a
                    // short-circuit &&, the compiler waited for the first
                    // entry (or for its stamp word alone) before issuing the
                    // rest -- dependent HBM round trips within one probe
                    // iteration on the wide walks (round 6).  A lane whose
                    // probe is done reads entry 0 (one line for all such
                    // lanes of a load, instead of one line each).
                    const size_t q0 = act0 ? (size_t)p0 : 0u, q1 = act1 ? (size_t)p1 : 0u;
                    const uint4 e00 = tab[2 * q0], e01 = tab[2 * q0 + 1];
                    uint4 e10 = {}, e11 = {};
                    if constexpr (WIDE) { e10 = tab[2 * q1]; e11 = tab[2 * q1 + 1]; }
                    const uint32_t own0 = (uint32_t)(e01.z == (uint32_t)gen) & (uint32_t)(e01.w == (uint32_t)(gen >> 32));
                    const uint32_t own1 = (uint32_t)(e11.z == (uint32_t)gen) & (uint32_t)(e11.w == (uint32_t)(gen >> 32));
                    const uint32_t eq0 = own0 & (uint32_t)(e01.x == kR0) & (uint32_t)(e01.y == s20) &
                                         (uint32_t)(e00.x == (uint32_t)k0lo) & (uint32_t)(e00.y == (uint32_t)(k0lo >> 32)) &
                                         (uint32_t)(e00.z == (uint32_t)k0hi) & (uint32_t)(e00.w == (uint32_t)(k0hi >> 32));
                    const uint32_t eq1 = own1 & (uint32_t)(e11.x == kR1) & (uint32_t)(e11.y == s21) &
                                         (uint32_t)(e10.x == (uint32_t)k1lo) & (uint32_t)(e10.y == (uint32_t)(k1lo >> 32)) &
                                         (uint32_t)(e10.z == (uint32_t)k1hi) & (uint32_t)(e10.w == (uint32_t)(k1hi >> 32));
                    hit0 |= act0 & eq0;
                    hit1 |= act1 & eq1;
                    act0 &= own0 & (eq0 ^ 1u);
                    act1 &= own1 & (eq1 ^ 1u);
                    p0 = (p0 + act0) & mask;
                    p1 = (p1 + act1) & mask;
                }
                pfree = want_ps && ((uint64_t)ps.x | (uint64_t)ps.y << 32) != gen;
            }
            lm = (lm & 0xFu) | (ok0 && !hit0 ? 1u << LM_C : 0u) | (ok1 && !hit1 ? 2u << LM_C : 0u);
            (void)act0;
            (void)act1;
            ipos0 = p0;
            ipos1 = p1;
            have_pos = true;
            if (pend) {
                // the pending pair goes in now (nothing looked for it: every
                // pair probed here has the pending step's op linearized too)
                const uint32_t tm = in_lds ? lmask : mask;
                if (!pend_known) {
                    const uint64_t fm = ballot(pfree);
                    if (fm) {
                        pend_pos = (ph + (uint32_t)__builtin_ctzll(fm)) & tm;
                    } else {  // the first ones all taken (a table at most half full: rare)
                        pend_pos = ph & tm;
                        for (uint32_t probe = in_lds ? 64u : WGL_PEND_LANES; probe <= tm; probe += 64) {
                            const uint32_t q = (ph + probe + lane) & tm;
                            bool fr;
                            if (in_lds) fr = ltab[q] == ~0ull;
                            else {
                                const uint4 e1 = tab[2 * (size_t)q + 1];
                                fr = ((uint64_t)e1.z | (uint64_t)e1.w << 32) != gen;
                            }
                            const uint64_t f2 = ballot(fr);
                            if (f2) { pend_pos = (ph + probe + (uint32_t)__builtin_ctzll(f2)) & tm; break; }
                        }
                    }
                }
                if (lane == 0) {
                    if (in_lds) {
                        ltab[pend_pos] = lkey(R, s, xlo);
                    } else {
                        tab[2 * (size_t)pend_pos] = make_uint4((uint32_t)xlo, (uint32_t)(xlo >> 32),
                                                               (uint32_t)xhi, (uint32_t)(xhi >> 32));
                        tab[2 * (size_t)pend_pos + 1] = make_uint4(R, s, (uint32_t)gen, (uint32_t)(gen >> 32));
                    }
                }
                pend = false;
                // a candidate whose probe ended at that slot (then empty) has
                // no insertion slot now: it searches again if chosen
                if (ipos0 == pend_pos) ipos0 = WGL_NONE;
                if (ipos1 == pend_pos) ipos1 = WGL_NONE;
            }
            WP_MARK(1);
        }
        if (!ballot((lm >> LM_C) & 3u)) {
            // ---- no candidate left ----
            if (!has_R) {  // the walk runs off the end of the list: linearizable
                WP_DUMP();
                wgl_finish(a, key, LC_VALID, LC_CAUSE_NONE, -1, cache_n, 0, steps, lookups);
                return true;
            }
            // stuck on the return entry R: the deepest such entries' nodes
            // are the frontier (the first max_final of them, in walk order)
            if (deepest == WGL_NONE || R >= deepest) {
                if (deepest == WGL_NONE || R > deepest) { deepest = R; n_front = 0; }
                KargWgl &ca = cold_args();
                if (ca.final_cfg && n_front < (uint32_t)ca.max_final) {
                    const uint64_t xlo = ballot(lm & 1u), xhi = ballot(lm & 2u);
                    if (lane == 0) {
                        uint64_t *f = ca.final_cfg + ((size_t)key * ca.max_final + n_front) * 2;
                        f[0] = xlo;
                        f[1] = (xhi & ((1ull << 48) - 1)) | (uint64_t)s << 48;
                    }
                }
                if (n_front < (uint32_t)ca.max_final) ++n_front;
            }
            if (depth == 0) {
                WP_DUMP();
                wgl_finish(a, key, LC_INVALID, LC_CAUSE_NONLIN, (int32_t)deepest, cache_n, n_front, steps, lookups);
                return true;
            }
            // backtrack: the frame of the node above (the LDS ring holds the
            // last WGL_RING levels), and the slots of the :invokes the step
            // down passed restored (newest first)
            --depth;
            ++steps;
            uint32_t word, mbyte;
            if (depth >= ring_lo) {
                const uint32_t *f = lfr + (depth % WGL_RING) * FRAME_WORDS;
                word = lane < 4 ? f[lane] : 0u;
                mbyte = ((const uint8_t *)(f + 4))[lane];
            } else {  // (the bytes as words here: loads the compiler cannot merge with the LDS ones above)
                const uint32_t *f = (const uint32_t *)(frames + depth);
                word = lane < 4 ? f[lane] : 0u;
                mbyte = (f[4 + (lane >> 2)] >> (8u * (lane & 3u))) & 0xFFu;
                ring_lo = depth;
            }
            const uint32_t fR = rdl(word, 0), fs = rdl(word, 1), fz = rdl(word, 2);
            if (fR != R) {
                EvWindowRev<LDS> win(io);
                for (uint32_t j = (R == WGL_END ? n : R); j-- > fR;) {
                    win.at(j);
                    const uint32_t w = rdl(win.w, j - win.base);
                    if (w & LC_EV_OK_BIT) continue;
                    const uint32_t sl = LC_EV_SLOT(w), l = sl & 63u;
                    const uint32_t pj = rdl(win.pv, j - win.base), d = rdl(win.pd, j - win.base);
                    if (!WIDE || sl < 64) { occ0 = wsetl(occ0, l, pj); dsc0 = wsetl(dsc0, l, d); }
                    else { occ1 = wsetl(occ1, l, pj); dsc1 = wsetl(dsc1, l, d); }
                }
            }
            R = fR; s = fs; zx = fz; lm = mbyte;
            have_pos = false;
            have_child = false;
            WP_MARK(3);
            continue;
        }
        // ---- step down: the candidate with the earliest :invoke ----
        const uint32_t v0 = (lm & (1u << LM_C)) ? occ0 : WGL_NONE;
        const uint32_t v1 = (WIDE && (lm & (2u << LM_C))) ? occ1 : WGL_NONE;
        const uint32_t inv = uni(__ockl_wfred_min_u32(v0 < v1 ? v0 : v1));
        const uint64_t m0 = ballot(v0 == inv), m1 = WIDE ? ballot(v1 == inv) : 0ull;
        const uint32_t c = (!WIDE || m0) ? (uint32_t)__builtin_ctzll(m0) : 64u + (uint32_t)__builtin_ctzll(m1);
        const uint32_t cl = c & 63u;
        const uint32_t cd = (!WIDE || c < 64) ? rdl(dsc0, cl) : rdl(dsc1, cl);
        uint32_t sc = 0;
        (void)step(a.table, s, cd, sc);
        sc = uni(sc);
        if (a.spill_at && cache_n + 1 > a.spill_at) {
            // the table would pass half full: the key is searched again with
            // a table the budget fits (no result written here).  Growing the
            // table in place instead (a rehash into a 4x table from a pool)
            // was built and measured in round 5: the rehash code alone, never
            // run, made every walk ~15 % slower (C2 8.6 -> 9.9 ms, C4 at 2^16
            // 216 -> 250 ms).
            if (lane == 0) {
                KargWgl &ca = cold_args();
                const int32_t i = atomicAdd(ca.n_spill, 1);
                ca.spill[i] = key;
            }
            WP_DUMP();
            return true;
        }
        ++cache_n;
        ++steps;
        if ((uint64_t)cache_n > a.budget) {
            WP_DUMP();
            wgl_finish(a, key, LC_UNKNOWN, LC_CAUSE_BUDGET, -1, cache_n, 0, steps, lookups);
            return true;
        }
        // the pair joins the cache in the next probe round; at the slot this
        // round's probe found for it, unless the round was an earlier one
        // (the subtree may have taken it) or the table changes tier now
        pend = true;
        pend_pos = have_pos ? ((!WIDE || c < 64) ? rdl(ipos0, cl) : rdl(ipos1, cl)) : WGL_NONE;
        pend_known = pend_pos != WGL_NONE;
        if (in_lds && cache_n > a.lds_tab / 2) {
            migrate();
            pend_known = false;
        }
        have_pos = false;
        // the node's frame, with c no longer to try (HBM, and the LDS ring)
        {
            const uint32_t wv = lane == 0 ? R : lane == 1 ? s : zx;
            const uint8_t mb = (uint8_t)(lm & ~lm_one(c, LM_C));
            uint32_t *f = (uint32_t *)(frames + depth);
            uint32_t *fl = lfr + (depth % WGL_RING) * FRAME_WORDS;
            if (lane < 3) { f[lane] = wv; fl[lane] = wv; }
            ((uint8_t *)(f + 4))[lane] = mb;
            ((uint8_t *)(fl + 4))[lane] = mb;
        }
        ++depth;
        if (depth - ring_lo > WGL_RING) ring_lo = depth - WGL_RING;
        // apply the step (taking R's op moves R: the child's R and X are then
        // what the probe round's tentative scan found)
        s = sc;
        WP_ADD(7, 1);
        WP_MARK(4);
        if (c == rs && have_child) {
            // (C bits: set by the child's own probe round)
            lm = ch_lm;
            occ0 = ch_occ0; dsc0 = ch_dsc0;
            if (WIDE) { occ1 = ch_occ1; dsc1 = ch_dsc1; }
            R = ch_R;
            zx = ch_z;
        } else {
            lm |= lm_one(c, LM_X);
            zx ^= zob(c);
            if (c == rs) advance(R);
        }
        have_child = false;
        WP_MARK(5);
        fresh = true;
    }
    // not reached: the walk ends within max_it steps
    wgl_finish(a, key, LC_UNKNOWN, LC_CAUSE_ERROR, -1, cache_n, 0, steps);
    return true;
}

__global__ __launch_bounds__(64) void k_wgl(WglArgs a) {
    if (a.err && __builtin_amdgcn_readfirstlane(*(volatile const int32_t *)a.err) != 0) return;  // refused batch
    char *slot_ws = a.ws.base + (size_t)blockIdx.x * a.ws.slot_bytes;
    const int32_t n_work = a.n_in ? *a.n_in : a.n_order;
    // a fixed trip count over a uni()-uniform ticket (the loop shape
    // device_lattice.hip's k_spec had to adopt: an open `for (;;) ... break`
    // once compiled into an exec-masked loop that never exited)
    for (int32_t guard = 0; guard <= n_work; ++guard) {
        int32_t w = 0;
        if (__lane_id() == 0) w = atomicAdd(a.ticket, 1);
        w = (int32_t)uni((uint32_t)w);
        if (w >= n_work) break;
        const int32_t key = a.order[w];
        const uint64_t nev = a.ev_off[key + 1] - a.ev_off[key];
        const bool lds = nev <= a.lds_events;
        // narrow walk unless key_width says the window reaches slot 64 (or
        // the walk finds it does)
        const bool wide = !a.key_width || a.key_width[key] > 64u;
        bool done = false;
        if (!wide) done = lds ? wgl_key<true, false>(a, key, (uint32_t)w, slot_ws)
                              : wgl_key<false, false>(a, key, (uint32_t)w, slot_ws);
        if (!done) {
            if (lds) wgl_key<true, true>(a, key, (uint32_t)w, slot_ws);
            else wgl_key<false, true>(a, key, (uint32_t)w, slot_ws);
        }
        __syncthreads();  // the next key's staging overwrites the LDS copies
    }
}

// Keys a :linear step left :unknown at the budget (knossos.competition: the
// other analysis answers them).
__global__ void k_collect_budget(const uint8_t *cause, int32_t n, int32_t *list, int32_t *count) {
    for (int32_t i = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x); i < n; i += (int32_t)(gridDim.x * blockDim.x))
        if (cause[i] == LC_CAUSE_BUDGET) list[atomicAdd(count, 1)] = i;
}

}  // namespace

#ifdef LC_WGL_PROF
extern "C" int lc_debug_wgl_prof(unsigned long long *host, int reset) {
    hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(lc_wgl_prof), sizeof(lc_wgl_prof), 0, hipMemcpyDeviceToHost);
    if (e == hipSuccess && reset) {
        static const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(lc_wgl_prof), z, sizeof(z), 0, hipMemcpyHostToDevice);
    }
    return (int)e;
}
#endif

WglWs wgl_layout(uint64_t budget, uint32_t max_events, uint32_t table_entries) {
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    WglWs w{};
    uint64_t T = table_entries ? table_entries : wgl_table_entries(budget);
    w.tab_mask = (uint32_t)(T - 1);
    size_t off = al(T * 32);
    w.off_frames = off;
    off += al(((size_t)max_events + 2) * sizeof(Frame));
    w.off_prev = off;
    off += al(((size_t)max_events + 1) * 4);
    w.slot_bytes = off;
    return w;
}

// Lowe's cache holds at most budget + 1 pairs (the one past the budget ends
// the walk :unknown): a table of twice the budget keeps linear probing at
// most half full.
size_t wgl_table_entries(uint64_t budget) {
    uint64_t T = 64;
    while (T < 2 * budget || T < budget + 64) T <<= 1;
    return (size_t)T;
}

size_t wgl_lds_bytes(uint32_t lds_events, uint32_t lds_tab) {
    return (size_t)lds_events * 3 * sizeof(uint32_t) + (size_t)lds_tab * 8 + (size_t)WGL_RING * sizeof(Frame);
}

bool wgl_allow_lds(size_t bytes) {
    if (bytes <= (64u << 10)) return true;
    return hipFuncSetAttribute((const void *)k_wgl, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) ==
           hipSuccess;
}

hipError_t launch_wgl(const WglArgs &a, int grid, hipStream_t s) {
    const size_t lds = wgl_lds_bytes(a.lds_events, a.lds_tab);
    hipLaunchKernelGGL(k_wgl, dim3(grid), dim3(64), lds, s, a);
    return hipGetLastError();
}

hipError_t launch_collect_budget(const uint8_t *cause, int32_t n, int32_t *list, int32_t *count, hipStream_t s) {
    const int blocks = (int)std::min<int64_t>(((int64_t)n + 255) / 256, 1024);
    hipLaunchKernelGGL(k_collect_budget, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, s, cause, n, list, count);
    return hipGetLastError();
}

}  // namespace lcd
