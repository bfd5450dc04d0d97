// device_hbm.hip -- HBM tier (T3) of the JIT linearization search.
//
// Same set computation as the LDS tiers (device_search.hip; semantics in
// oracle/linear_ref.py), for keys whose config sets outgrow LDS or whose
// window needs more than 56 slots / 255 register states.  One workgroup of
// WG (1,024) threads searches one key; its S / S' / I arrays and the two
// open-addressed hash sets live in a per-block HBM workspace slot sized from
// the search budget (a key can never hold more than budget + t3_block()
// configs: insertion stops as soon as a count passes the budget, which is
// exactly the LC_CAUSE_BUDGET verdict).  Per :ok, sets of up to 2,048 / 4,096
// configs (narrow) use hash tables in LDS instead; a pass that outgrows them
// is discarded and redone on the HBM tables (ok_pass, PASS_REDO).
//
// Hash sets, open addressing with linear probing:
//   narrow (u64 configs): one 64-bit atomicCAS on EMPTY per probe, U per
//     lane in flight, with an L1-bypassing read first in full batches so
//     that duplicates cost no memory-side atomic.
//   wide (2 x u64: lo = slots 0..63, hi = slots 64..111 | state << 48):
//     CAS hi from EMPTY to hi|BUSY, store lo, release-store hi; a prober
//     that meets its own hi still BUSY waits (bounded) for the publisher,
//     which is always another wave: publishers of this wave store before
//     any lane of the wave compares (publish step precedes compare step).
// Tables stay clean between keys: every inserted slot index is recorded and
// the entries are erased through those records, never by sweeping.

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/lincheck.h"
#include "device_common.hpp"
#include "device_search.hpp"

namespace lcd {

// Diagnostic build only (make variant VFLAGS=-DLC_T3_PROF): thread 0 of the
// first blocks accumulates shader cycles per :ok phase and prints them when a
// key finishes.  Never in the product library.
#ifdef LC_T3_PROF
#define T3P_DECL uint64_t t3p[6] = {0, 0, 0, 0, 0, 0}, t3last = 0, t3lev = 0, t3gen = 0, t3nok = 0;
#define T3P_MARK(i) do { if (tid == 0) { const uint64_t t_ = __builtin_readcyclecounter(); if ((i) >= 0) t3p[(i) < 0 ? 0 : (i)] += t_ - t3last; t3last = t_; } } while (0)
#define T3P_ADD(v, x) do { if (tid == 0) v += (x); } while (0)
#define T3P_PRINT() do { if (tid == 0) printf("T3KEY blk %d key %d ok %llu between %llu setup %llu hbm %llu lds %llu n_lds %llu n_redo %llu nS %u\n", (int)blockIdx.x, key, (unsigned long long)t3nok, (unsigned long long)t3p[1], (unsigned long long)t3p[0], (unsigned long long)t3p[2], (unsigned long long)t3p[3], (unsigned long long)t3p[4], (unsigned long long)t3p[5], nS); } while (0)
#else
#define T3P_DECL
#define T3P_MARK(i) do {} while (0)
#define T3P_ADD(v, x) do {} while (0)
#define T3P_PRINT() do {} while (0)
#endif

#ifndef LC_T3_U
#define LC_T3_U 2  // measured on C4: 2 beats 4 and 8 (the memory side is the bound, not latency)
#endif

constexpr uint32_t NOPOS = 0xFFFFFFFFu;
constexpr uint64_t BUSY = 1ull << 63;

struct Narrow {
    using T = uint64_t;
    static constexpr uint32_t MAX_SLOTS = LC_NARROW_MAX_SLOTS;
    __device__ static T init(uint32_t s) { return (uint64_t)s << 56; }
    __device__ static uint32_t state(T c) { return (uint32_t)(c >> 56); }
    __device__ static bool has(T c, uint32_t s) { return (c >> s) & 1ull; }
    __device__ static T lin(T c, uint32_t q, uint32_t s2) { return ((uint64_t)s2 << 56) | (c & LMASK) | (1ull << q); }
    __device__ static T restate(T c, uint32_t s2) { return ((uint64_t)s2 << 56) | (c & LMASK); }
    __device__ static T drop(T c, uint32_t p) { return c & ~(1ull << p); }
    __device__ static void rec(T c, uint64_t &w0, uint64_t &w1) { w0 = c & LMASK; w1 = (c >> 56) << 48; }
    __device__ static void erase(T *tab, uint32_t pos) { tab[pos] = EMPTY; }
    static constexpr int U = LC_T3_U;  // closure inserts in flight per lane
    static constexpr int UA = 2;       // partition / apply (4 measured no better on C4)
    // Small :oks keep both hash sets in LDS (S': LDS_ES slots, I: LDS_EI,
    // each at most half full); larger ones use the HBM tables.
    static constexpr bool LDS_MODE = true;
    static constexpr bool NARROW = true;
    static constexpr uint32_t LDS_ES = 4096, LDS_EI = 8192, LIM_S = LDS_ES / 2, LIM_I = LDS_EI / 2;
    __device__ static bool insert(T *tab, uint32_t mask, T key, uint32_t &pos, uint32_t *err) {
        return insert_at(tab, mask, key, hash64(key) & mask, pos);
    }
    __device__ static bool insert_at(T *tab, uint32_t mask, T key, uint32_t h, uint32_t &pos) {
        for (;;) {
            unsigned long long old = atomicCAS((unsigned long long *)&tab[h], (unsigned long long)EMPTY,
                                               (unsigned long long)key);
            if (old == EMPTY) { pos = h; return true; }
            if (old == key) { pos = h; return false; }
            h = (h + 1) & mask;
        }
    }
    // U inserts per lane with their first probes in flight together: the
    // CASes are independent, so one wait covers all of them; a lane whose
    // first slot holds another config continues serially from there.
    // Two thirds of the closure's probes meet a config already in the set
    // (C4), and every atomic executes at the memory side, so the home slots
    // are read first (L2-served, L1 bypassed): a slot that already holds the
    // key is a duplicate and costs no atomic.  A stale EMPTY only means one
    // CAS more; a key cannot read stale, since its slot was erased by this
    // workgroup's own earlier stores.
    // probe_first: only for full batches.  The read costs a round trip, which
    // a small (latency-bound) closure level cannot hide; a large level is
    // bound by memory-side traffic, where the saved atomics pay.
    template <int U>
    __device__ static void insert_n(T *tab, uint32_t mask, const T (&key)[U], const bool (&act)[U],
                                    uint32_t (&pos)[U], bool (&isnew)[U], uint32_t *err, bool probe_first) {
        uint32_t h[U];
        unsigned long long old[U];
        bool need[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            h[u] = hash64(key[u]) & mask;
            old[u] = act[u] && probe_first ? __hip_atomic_load((unsigned long long *)&tab[h[u]], __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT)
                                           : (act[u] ? EMPTY : (unsigned long long)key[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            need[u] = old[u] != (unsigned long long)key[u];
            old[u] = need[u] ? atomicCAS((unsigned long long *)&tab[h[u]], (unsigned long long)EMPTY,
                                         (unsigned long long)key[u])
                             : old[u];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            pos[u] = h[u];
            isnew[u] = act[u] && old[u] == EMPTY;
            if (act[u] && old[u] != EMPTY && old[u] != key[u])
                isnew[u] = insert_at(tab, mask, key[u], (h[u] + 1) & mask, pos[u]);
        }
    }
};

struct WideCfg { uint64_t lo, hi; };

struct Wide {
    using T = WideCfg;
    static constexpr uint32_t MAX_SLOTS = LC_WIDE_MAX_SLOTS;
    static constexpr uint64_t HMASK = (1ull << 48) - 1;
    __device__ static T init(uint32_t s) { return T{0, (uint64_t)s << 48}; }
    __device__ static uint32_t state(T c) { return (uint32_t)(c.hi >> 48) & 0x7FFFu; }
    __device__ static bool has(T c, uint32_t s) { return s < 64 ? ((c.lo >> s) & 1ull) : ((c.hi >> (s - 64)) & 1ull); }
    __device__ static T lin(T c, uint32_t q, uint32_t s2) {
        T r{c.lo, (c.hi & HMASK) | ((uint64_t)s2 << 48)};
        if (q < 64) r.lo |= 1ull << q; else r.hi |= 1ull << (q - 64);
        return r;
    }
    __device__ static T restate(T c, uint32_t s2) { return T{c.lo, (c.hi & HMASK) | ((uint64_t)s2 << 48)}; }
    __device__ static T drop(T c, uint32_t p) {
        if (p < 64) c.lo &= ~(1ull << p); else c.hi &= ~(1ull << (p - 64));
        return c;
    }
    __device__ static void rec(T c, uint64_t &w0, uint64_t &w1) { w0 = c.lo; w1 = c.hi; }
    __device__ static void erase(T *tab, uint32_t pos) { tab[pos].hi = EMPTY; }
    __device__ static uint32_t hash(T c) { return hash64(c.lo ^ (c.hi * 0x9E3779B97F4A7C15ull)); }
    static constexpr int U = 2;
    static constexpr int UA = 2;
    static constexpr bool LDS_MODE = false;  // the publish protocol is HBM-only
    static constexpr bool NARROW = false;
    static constexpr uint32_t LDS_ES = 1, LDS_EI = 1, LIM_S = 0, LIM_I = 0;
    // Wide inserts keep their publish protocol: one at a time.
    template <int U>
    __device__ static void insert_n(T *tab, uint32_t mask, const T (&key)[U], const bool (&act)[U],
                                    uint32_t (&pos)[U], bool (&isnew)[U], uint32_t *err, bool) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            pos[u] = NOPOS;
            isnew[u] = act[u] && insert(tab, mask, key[u], pos[u], err);
        }
    }
    __device__ static bool insert(T *tab, uint32_t mask, T key, uint32_t &pos, uint32_t *err) {
        uint32_t h = hash(key) & mask;
        for (;;) {
            uint64_t *whi = &tab[h].hi, *wlo = &tab[h].lo;
            const unsigned long long old = atomicCAS((unsigned long long *)whi, (unsigned long long)EMPTY,
                                                     (unsigned long long)(key.hi | BUSY));
            const bool won = old == EMPTY;
            if (won) {  // publish
                __hip_atomic_store(wlo, key.lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(whi, key.hi, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            }
            __builtin_amdgcn_wave_barrier();
            if (won) { pos = h; return true; }
            uint64_t cur = old;
            if ((cur & ~BUSY) == key.hi) {  // same hi: compare lo once published
                uint32_t spins = 0;
                while (cur & BUSY) {
                    __builtin_amdgcn_s_sleep(1);
                    cur = __hip_atomic_load(whi, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                    if (++spins > (1u << 24)) { *err = 1; pos = h; return false; }
                }
                if (cur == key.hi) {
                    const uint64_t lo = __hip_atomic_load(wlo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (lo == key.lo) { pos = h; return false; }
                }
            }
            h = (h + 1) & mask;
        }
    }
};

template <class C, int WG>
struct HbmShared {
    uint32_t ev[WG];
    uint32_t dsc[WG];
    uint32_t slot_desc[128];
    uint32_t cand_slot[128];
    uint32_t cand_desc[128];
    uint64_t legal[C::NARROW ? 256 : 1];  // narrow: candidate slots legal from each state
    uint32_t nSn, nI, stop, err, redo;
    int32_t work;
    unsigned long long probes;
    // closure successors staged per wave until 64 x U are ready to insert
    typename C::T stage[WG / 64][64 * C::U + 64];
    uint64_t ltS[C::LDS_ES];  // LDS-mode hash sets: S'
    uint64_t ltI[C::LDS_EI];  //                     I
};

// Sum of one value over the workgroup (every thread gets it).
template <int WG>
__device__ __forceinline__ uint64_t block_sum(uint64_t v, unsigned long long *acc) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t lo2 = __shfl_xor(lo, o), hi2 = __shfl_xor(hi, o);
        const uint64_t s = ((uint64_t)hi << 32 | lo) + ((uint64_t)hi2 << 32 | lo2);
        lo = (uint32_t)s; hi = (uint32_t)(s >> 32);
    }
    if (lane_id() == 0) atomicAdd(acc, ((unsigned long long)hi << 32) | lo);
    __syncthreads();
    return *acc;
}

// Block-wide append: returns this thread's position for a set flag.
template <int WG>
__device__ __forceinline__ uint32_t block_append(uint32_t *counter, bool flag) {
    const uint64_t m = __ballot(flag);
    uint32_t base = 0;
    if (m) {
        if (lane_id() == 0) base = atomicAdd(counter, (uint32_t)__popcll(m));
        base = __shfl(base, 0);
    }
    return base + rank_of(m);
}

template <class C>
struct Slot {
    typename C::T *S[2];
    typename C::T *I;
    typename C::T *hS;
    typename C::T *hI;
    uint32_t *posS[2];
    uint32_t *posI;
};

template <class C>
__device__ Slot<C> slot_ptrs(const HbmWs &w, uint32_t slot) {
    char *base = w.base + (size_t)slot * w.slot_bytes;
    Slot<C> s;
    s.S[0] = (typename C::T *)(base + w.off_S0);
    s.S[1] = (typename C::T *)(base + w.off_S1);
    s.I = (typename C::T *)(base + w.off_I);
    s.hS = (typename C::T *)(base + w.off_hS);
    s.hI = (typename C::T *)(base + w.off_hI);
    s.posS[0] = (uint32_t *)(base + w.off_pS0);
    s.posS[1] = (uint32_t *)(base + w.off_pS1);
    s.posI = (uint32_t *)(base + w.off_pI);
    return s;
}

template <class C, int WG>
__device__ void write_final_hbm(KArgs &a, int32_t key, const typename C::T *S, uint32_t nS) {
    if (!a.final_cfg) return;
    const uint32_t nf = nS < (uint32_t)a.max_final ? nS : (uint32_t)a.max_final;
    for (uint32_t i = threadIdx.x; i < nf; i += WG) {
        uint64_t w0, w1;
        C::rec(S[i], w0, w1);
        a.final_cfg[((size_t)key * a.max_final + i) * 2 + 0] = w0;
        a.final_cfg[((size_t)key * a.max_final + i) * 2 + 1] = w1;
    }
    if (threadIdx.x == 0 && a.n_final) a.n_final[key] = nf;
}

template <class C, int WG>
__device__ void erase_all(const HbmWs &w, Slot<C> &sl, const uint32_t *posI, uint32_t nI, const uint32_t *posS,
                          uint32_t nS) {
    for (uint32_t j = threadIdx.x; j < nI; j += WG) C::erase(sl.hI, posI[j]);
    for (uint32_t j = threadIdx.x; j < nS; j += WG) if (posS[j] != NOPOS) C::erase(sl.hS, posS[j]);
    __syncthreads();
}

// Insert into an LDS-mode hash set (narrow configs).  The probe sequence is
// bounded: a table that fills up (a set past its limit, plus other waves'
// in-flight batches) raises `redo` and the :ok is run again on HBM tables.
template <uint32_t E>
__device__ __forceinline__ bool lds_set_insert(uint64_t *tab, uint64_t key, bool active, uint32_t &pos,
                                               uint32_t *redo) {
    bool isnew = false;
    uint32_t h = hash64(key) & (E - 1);
    bool done = !active;
    for (uint32_t n = 0; !done; ++n) {
        if (n == E) { *redo = 1; break; }
        const unsigned long long old = atomicCAS((unsigned long long *)&tab[h], (unsigned long long)EMPTY,
                                                 (unsigned long long)key);
        if (old == EMPTY) { isnew = true; done = true; }
        else if (old == key) { done = true; }
        else { h = (h + 1) & (E - 1); }
    }
    pos = h;
    return isnew;
}

template <class C, int WG, bool LDS, int N>
__device__ __forceinline__ void set_insert_n(HbmShared<C, WG> &sh, typename C::T *htab, int which, uint32_t hmask, bool big,
                                             const typename C::T (&key)[N], const bool (&act)[N],
                                             uint32_t (&pos)[N], bool (&nw)[N]) {
    if constexpr (LDS) {
#pragma unroll
        for (int u = 0; u < N; ++u)
            nw[u] = which == 0 ? lds_set_insert<C::LDS_ES>(sh.ltS, key[u], act[u], pos[u], &sh.redo)
                               : lds_set_insert<C::LDS_EI>(sh.ltI, key[u], act[u], pos[u], &sh.redo);
    } else {
        C::template insert_n<N>(htab, hmask, key, act, pos, nw, &sh.err, big);
    }
}

// Position r of a new config in set `which` (0 S', 1 I): past the cap it is
// an error in HBM mode (cap covers every overshoot), past the LDS set's
// limit a redo in LDS mode.
template <class C, int WG, bool LDS>
__device__ __forceinline__ bool take_pos(HbmShared<C, WG> &sh, uint32_t r, uint32_t cap, int which) {
    if (LDS && r >= (which == 0 ? C::LIM_S : C::LIM_I)) { sh.redo = 1; sh.stop = 1; }
    if (r < cap) return true;
    sh.err = 1;
    return false;
}

// Insert the first n (<= 64 x U) staged successors of this wave into the I
// set and append the new ones (wave-uniform call).  A stop raised by any wave
// caps the overshoot past the budget at WG x U configs (cap covers it).
template <class C, int WG, bool LDS>
__device__ void flush_stage(typename C::T *stg, uint32_t n, Slot<C> &sl, HbmShared<C, WG> &sh, uint32_t hmask,
                            uint32_t cap, uint64_t budget) {
    constexpr int U = C::U;
    typename C::T key[U];
    bool act[U], nw[U];
    uint32_t pos[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t i = (uint32_t)u * 64u + lane_id();
        act[u] = i < n;
        key[u] = act[u] ? stg[i] : C::init(0);
    }
    set_insert_n<C, WG, LDS, U>(sh, sl.hI, 1, hmask, n == 64u * U, key, act, pos, nw);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t r = block_append<WG>(&sh.nI, nw[u]);
        if (nw[u]) {
            if (take_pos<C, WG, LDS>(sh, r, cap, 1)) { sl.I[r] = key[u]; sl.posI[r] = pos[u]; }
            if (r + 1 > budget) sh.stop = 1;
        }
    }
}

enum { PASS_OK = 0, PASS_CLOSURE_STOP = 1, PASS_REDO = 2 };

// One :ok(p) over the config set S (nS configs): S' into Sn, I in sl.I, with
// the hash sets in LDS (LDS) or in the block's HBM tables.  Counters sh.nSn /
// sh.nI / stop / err / redo are zero on entry.
template <class C, int WG, bool LDS>
__device__ int ok_pass(const Args &a, Slot<C> &sl, HbmShared<C, WG> &sh, typename C::T *S, uint32_t nS,
                       typename C::T *Sn, uint32_t *posSn, uint32_t p, uint32_t dp, uint32_t nc, uint32_t cap,
                       uint32_t hmask, uint32_t nstates, uint64_t &probes) {
    using T = typename C::T;
    constexpr int U = C::U, UA = C::UA;
    const uint32_t tid = threadIdx.x;
    if constexpr (LDS) {
        for (uint32_t j = tid; j < C::LDS_ES; j += WG) sh.ltS[j] = EMPTY;
        for (uint32_t j = tid; j < C::LDS_EI; j += WG) sh.ltI[j] = EMPTY;
    }
    if constexpr (C::NARROW) {  // per state, the candidates whose step is legal there
        for (uint32_t st = tid; st < nstates; st += WG) {
            uint64_t m = 0;
            for (uint32_t k = 0; k < nc; ++k) {
                uint32_t s2;
                if (step(a.table, st, sh.cand_desc[k], s2)) m |= 1ull << sh.cand_slot[k];
            }
            sh.legal[st] = m;
        }
    }
    if constexpr (LDS || C::NARROW) __syncthreads();
    // -- partition S (UA configs per thread, their inserts in flight together)
    for (uint32_t j0 = 0; j0 < nS; j0 += WG * UA) {
        T kS[UA], kI[UA];
        bool hasp[UA], toI[UA], ns[UA], ni[UA];
        uint32_t pS[UA], pI[UA];
#pragma unroll
        for (int u = 0; u < UA; ++u) {
            const uint32_t j = j0 + u * WG + tid;
            const bool act = j < nS;
            const T c = act ? S[j] : C::init(0);
            hasp[u] = act && C::has(c, p);
            toI[u] = act && !hasp[u];
            kS[u] = C::drop(c, p);
            kI[u] = c;
        }
        set_insert_n<C, WG, LDS, UA>(sh, sl.hS, 0, hmask, nS >= WG * UA, kS, hasp, pS, ns);
        set_insert_n<C, WG, LDS, UA>(sh, sl.hI, 1, hmask, nS >= WG * UA, kI, toI, pI, ni);
#pragma unroll
        for (int u = 0; u < UA; ++u) {
            const uint32_t rs = block_append<WG>(&sh.nSn, ns[u]);
            const uint32_t ri = block_append<WG>(&sh.nI, ni[u]);
            if (ns[u] && take_pos<C, WG, LDS>(sh, rs, cap, 0)) { Sn[rs] = kS[u]; posSn[rs] = pS[u]; }
            if (ni[u] && take_pos<C, WG, LDS>(sh, ri, cap, 1)) { sl.I[ri] = kI[u]; sl.posI[ri] = pI[u]; }
        }
    }
    if (tid == 0) probes += nS;
    __syncthreads();
    // -- JIT closure, level by level.  Each wave stages the legal successors
    // of its configs in LDS and inserts them 64 x U at a time, so every
    // insert batch is full whatever fraction of the (config, candidate)
    // pairs is legal.
    uint32_t head = 0;
    T *stg = sh.stage[tid >> 6];
    while (true) {
        const uint32_t end = sh.nI < cap ? sh.nI : cap;
        if (head >= end || sh.stop || nc == 0) break;
        uint32_t nst = 0;  // wave-uniform
        bool halt = false;
        for (uint32_t j0 = head; j0 < end && !halt; j0 += WG) {
            const uint32_t j = j0 + tid;
            const bool in = j < end;
            const T c = in ? sl.I[j] : C::init(0);
            const uint32_t st = C::state(c);
            if constexpr (C::NARROW) {
                // each lane walks only its config's legal, unlinearized
                // candidates: the wave loops max-over-lanes times, not nc
                uint64_t m = in ? (sh.legal[st] & ~(c & LMASK)) : 0ull;
                for (;;) {
                    const bool act = m != 0;
                    const uint64_t bm = __ballot(act);
                    if (bm == 0) break;
                    const uint32_t q = act ? (uint32_t)__builtin_ctzll(m) : 0u;
                    m &= m - 1;
                    uint32_t s2 = st;
                    (void)step(a.table, st, sh.slot_desc[q], s2);
                    probes += act;
                    if (act) stg[nst + rank_of(bm)] = C::lin(c, q, s2);
                    nst += (uint32_t)__popcll(bm);
                    if (nst >= 64u * U) {
                        flush_stage<C, WG, LDS>(stg, 64u * U, sl, sh, hmask, cap, a.budget);
                        nst -= 64u * U;
                        if (lane_id() < nst) stg[lane_id()] = stg[64u * U + lane_id()];
                        if (*(volatile uint32_t *)&sh.stop) { halt = true; break; }
                    }
                }
                continue;
            }
            for (uint32_t k = 0; k < nc; ++k) {
                const uint32_t q = sh.cand_slot[k];
                uint32_t s2 = 0;
                const bool act = in && !C::has(c, q) && step(a.table, st, sh.cand_desc[k], s2);
                probes += act;
                const uint64_t m = __ballot(act);
                if (m == 0) continue;
                if (act) stg[nst + rank_of(m)] = C::lin(c, q, s2);
                nst += (uint32_t)__popcll(m);
                if (nst >= 64u * U) {
                    flush_stage<C, WG, LDS>(stg, 64u * U, sl, sh, hmask, cap, a.budget);
                    nst -= 64u * U;
                    if (lane_id() < nst) stg[lane_id()] = stg[64u * U + lane_id()];
                    if (*(volatile uint32_t *)&sh.stop) { halt = true; break; }
                }
            }
        }
        if (nst && !halt) flush_stage<C, WG, LDS>(stg, nst, sl, sh, hmask, cap, a.budget);
        __syncthreads();
        head = end;
    }
    __syncthreads();
    if (LDS && sh.redo) return PASS_REDO;
    if (sh.nI > a.budget || sh.err) return PASS_CLOSURE_STOP;
    // -- apply p
    const uint32_t nI = sh.nI;
    for (uint32_t j0 = 0; j0 < nI; j0 += WG * UA) {
        if (*(volatile uint32_t *)&sh.stop) break;
        T k2[UA];
        bool act[UA], nw[UA];
        uint32_t pos[UA];
#pragma unroll
        for (int u = 0; u < UA; ++u) {
            const uint32_t j = j0 + u * WG + tid;
            const T c = j < nI ? sl.I[j] : C::init(0);
            uint32_t s2 = 0;
            act[u] = j < nI && step(a.table, C::state(c), dp, s2);
            probes += act[u];
            k2[u] = C::restate(c, s2);
        }
        set_insert_n<C, WG, LDS, UA>(sh, sl.hS, 0, hmask, nI >= WG * UA, k2, act, pos, nw);
#pragma unroll
        for (int u = 0; u < UA; ++u) {
            const uint32_t r = block_append<WG>(&sh.nSn, nw[u]);
            if (nw[u]) {
                if (take_pos<C, WG, LDS>(sh, r, cap, 0)) { Sn[r] = k2[u]; posSn[r] = pos[u]; }
                if (r + 1 > a.budget) sh.stop = 1;
            }
        }
    }
    __syncthreads();
    if (LDS && sh.redo) return PASS_REDO;
    return PASS_OK;
}

// Search one key with the whole workgroup.  Returns K_DONE or K_WIDE.
template <class C, int WG>
__device__ int search_key_hbm(const Args &a, const HbmWs &w, int32_t key, Slot<C> &sl, HbmShared<C, WG> &sh) {
    const uint32_t tid = threadIdx.x;
    const uint64_t b = a.ev_off[key], e = a.ev_off[key + 1];
    const uint32_t tb = a.trans_off ? a.trans_off[key] : 0u;
    const uint32_t cap = w.cap, hmask = w.hmask;
    uint32_t nstates = a.trans_off ? (a.key_states ? (uint32_t)a.key_states[key] : 256u) : a.shared_states;
    nstates = nstates < 256u ? nstates : 256u;  // narrow configs hold 8-bit states
    if (a.key_states && a.key_states[key] > LC_WIDE_MAX_STATES) {
        if (tid == 0) finish_key(kargs(), key, LC_UNKNOWN, LC_CAUSE_STATES, -1, 1, 0, 0);
        return K_DONE;
    }
    if (tid == 0) { sl.S[0][0] = C::init(a.init_state); sl.posS[0][0] = NOPOS; sh.err = 0; sh.probes = 0; }
    __syncthreads();
    int cur = 0;
    uint32_t nS = 1, nSprev = 0, nIlast = 0, peak = 1, nIbig = 0;
    uint64_t pend0 = 0, pend1 = 0;
    uint64_t probes = 0;  // this thread's share
    T3P_DECL
    for (uint64_t base = b; base < e; base += WG) {
        const uint32_t cnt = (uint32_t)((e - base) < WG ? (e - base) : WG);
        __syncthreads();
        if (tid < cnt) {
            const uint32_t ev = a.events[base + tid];
            sh.ev[tid] = ev;
            sh.dsc[tid] = (ev & LC_EV_OK_BIT) ? 0u : a.trans[tb + LC_EV_TRANS(ev)];
        }
        __syncthreads();
        for (uint32_t i = 0; i < cnt; ++i) {
            const uint32_t evi = sh.ev[i];
            const uint32_t slot = LC_EV_SLOT(evi);
            const int32_t evno = (int32_t)(base + i - b);
            if (!(evi & LC_EV_OK_BIT)) {
                if (slot >= C::MAX_SLOTS) {
                    erase_all<C, WG>(w, sl, sl.posI, nIlast, sl.posS[cur], nSprev);
                    if (C::MAX_SLOTS == LC_NARROW_MAX_SLOTS) return K_WIDE;
                    write_final_hbm<C, WG>(kargs(), key, sl.S[cur], nS);
                    if (tid == 0) finish_key(kargs(), key, LC_UNKNOWN, LC_CAUSE_WINDOW, evno, peak, 0, (uint64_t)evno);
                    return K_DONE;
                }
                if (slot < 64) pend0 |= 1ull << slot; else pend1 |= 1ull << (slot - 64);
                if (tid == 0) sh.slot_desc[slot] = sh.dsc[i];
                continue;
            }
            // ---- :ok of the op in `slot` ----
            const uint32_t p = slot;
            typename C::T *S = sl.S[cur];
            typename C::T *Sn = sl.S[cur ^ 1];
            uint32_t *posSn = sl.posS[cur ^ 1];
            __syncthreads();  // slot_desc of earlier invokes visible
            T3P_MARK(1);
            T3P_ADD(t3nok, 1);
            const uint32_t dp = sh.slot_desc[p];
            for (uint32_t j = tid; j < nIlast; j += WG) C::erase(sl.hI, sl.posI[j]);
            for (uint32_t j = tid; j < nSprev; j += WG) {
                const uint32_t ps = sl.posS[cur][j];
                if (ps != NOPOS) C::erase(sl.hS, ps);
            }
            const uint64_t c0 = pend0 & ~(p < 64 ? 1ull << p : 0ull);
            const uint64_t c1 = pend1 & ~(p >= 64 ? 1ull << (p - 64) : 0ull);
            const uint32_t nc = (uint32_t)(__popcll(c0) + __popcll(c1));
            if (tid < 128) {
                const bool on = tid < 64 ? ((c0 >> tid) & 1ull) : ((c1 >> (tid - 64)) & 1ull);
                if (on) {
                    const uint32_t r = tid < 64 ? (uint32_t)__popcll(c0 & ((1ull << tid) - 1ull))
                                                : (uint32_t)(__popcll(c0) + __popcll(c1 & ((1ull << (tid - 64)) - 1ull)));
                    sh.cand_slot[r] = tid;
                    sh.cand_desc[r] = sh.slot_desc[tid];
                }
            }
            // Small sets run with both hash sets in LDS; a pass that outgrows
            // them is discarded (S is untouched) and run again on the HBM
            // tables, which the erasure above has left clean.
            bool lds = C::LDS_MODE && nS <= C::LIM_S && nIbig <= C::LIM_I;
            const uint64_t probes0 = probes;
            int pr;
            uint32_t pr_redos = 0;
            for (;;) {
                if (tid == 0) { sh.nSn = 0; sh.nI = 0; sh.stop = 0; sh.redo = 0; }
                __threadfence_block();
                __syncthreads();
                T3P_MARK(0);
                if constexpr (C::LDS_MODE) {
                    if (lds)
                        pr = ok_pass<C, WG, true>(a, sl, sh, S, nS, Sn, posSn, p, dp, nc, cap, hmask, nstates, probes);
                    else
                        pr = ok_pass<C, WG, false>(a, sl, sh, S, nS, Sn, posSn, p, dp, nc, cap, hmask, nstates, probes);
                } else {
                    pr = ok_pass<C, WG, false>(a, sl, sh, S, nS, Sn, posSn, p, dp, nc, cap, hmask, nstates, probes);
                }
                if (pr != PASS_REDO) break;
                lds = false;
                ++pr_redos;
                probes = probes0;
            }
            (void)pr_redos;
            T3P_MARK(lds ? 3 : 2);
            T3P_ADD(t3p[4], lds ? 1 : 0);
            T3P_ADD(t3p[5], pr_redos);
            const uint32_t nI = sh.nI < cap ? sh.nI : cap;
            nIbig = sh.nI;
            if (pr == PASS_CLOSURE_STOP) {
                T3P_PRINT();
                const int cause = sh.err ? LC_CAUSE_ERROR : LC_CAUSE_BUDGET;
                const uint32_t nSn_now = sh.nSn;
                if (!lds) erase_all<C, WG>(w, sl, sl.posI, nI, posSn, nSn_now);
                write_final_hbm<C, WG>(kargs(), key, S, nS);
                probes = block_sum<WG>(probes, &sh.probes);
                if (tid == 0) finish_key(kargs(), key, LC_UNKNOWN, cause, evno, peak, probes, (uint64_t)evno);
                return K_DONE;
            }
#ifdef LC_T3_PROF
            if (tid == 0 && blockIdx.x == 0)
                printf("T3OK key %d ev %d nS %u nI %u nSn %u nc %u lds %d setup %llu pass %llu\n", key, evno, nS, nI, sh.nSn, nc,
                       (int)lds, (unsigned long long)t3p[0], (unsigned long long)(t3p[2] + t3p[3]));
#endif
            const uint32_t nSn_all = sh.nSn;
            const uint32_t nSn = nSn_all < cap ? nSn_all : cap;
            nIlast = lds ? 0u : nI;  // HBM entries the next :ok erases
            if (nSn_all == 0 || nSn_all > a.budget || sh.err) {
                const int verdict = nSn_all == 0 ? LC_INVALID : LC_UNKNOWN;
                const int cause = sh.err ? LC_CAUSE_ERROR : (nSn_all == 0 ? LC_CAUSE_NONLIN : LC_CAUSE_BUDGET);
                if (!lds) erase_all<C, WG>(w, sl, sl.posI, nI, posSn, nSn);
                write_final_hbm<C, WG>(kargs(), key, S, nS);
                probes = block_sum<WG>(probes, &sh.probes);
                if (tid == 0)
                    finish_key(kargs(), key, verdict, cause, evno, peak, probes, (uint64_t)evno + (verdict == LC_INVALID));
                return K_DONE;
            }
            nSprev = lds ? 0u : nSn;
            cur ^= 1;
            nS = nSn;
            peak = nS > peak ? nS : peak;
            if (p < 64) pend0 &= ~(1ull << p); else pend1 &= ~(1ull << (p - 64));
        }
    }
    __syncthreads();
    T3P_PRINT();
    erase_all<C, WG>(w, sl, sl.posI, nIlast, sl.posS[cur], nSprev);
    write_final_hbm<C, WG>(kargs(), key, sl.S[cur], nS);
    probes = block_sum<WG>(probes, &sh.probes);
    if (tid == 0) finish_key(kargs(), key, LC_VALID, LC_CAUSE_NONE, -1, peak, probes, e - b);
    return K_DONE;
}

template <class C, int WG>
__global__ __launch_bounds__(WG) void k_search_hbm(Args a, HbmWs w) {
    __shared__ HbmShared<C, WG> sh;
    Slot<C> sl = slot_ptrs<C>(w, blockIdx.x);
    // (the work list and results through kargs(): device_common.hpp)
    int32_t n;
    {
        KArgs &ka = kargs();
        n = ka.n_in ? min(*ka.n_in, ka.list_cap) : ka.n_order;
        if (n == 0 || batch_refused(ka)) return;  // empty work list / malformed batch
    }
    for (;;) {
        if (threadIdx.x == 0) sh.work = atomicAdd(kargs().ticket, 1);
        __syncthreads();
        const int32_t wi = sh.work;
        __syncthreads();
        if (wi >= n) break;
        const int32_t key = kargs().order[wi];
        const int r = search_key_hbm<C, WG>(a, w, key, sl, sh);
        if (r == K_WIDE && threadIdx.x == 0) {
            KArgs &ka = kargs();
            const int32_t i = atomicAdd(ka.n_wide, 1);
            ka.wide[i] = key;
        }
        __syncthreads();
    }
}

constexpr int T3_WG = 1024;

hipError_t launch_t3_narrow(const Args &a, const HbmWs &w, int grid, hipStream_t s) {
    hipLaunchKernelGGL((k_search_hbm<Narrow, T3_WG>), dim3(grid), dim3(T3_WG), 0, s, a, w);
    return hipGetLastError();
}
hipError_t launch_t3_wide(const Args &a, const HbmWs &w, int grid, hipStream_t s) {
    hipLaunchKernelGGL((k_search_hbm<Wide, T3_WG>), dim3(grid), dim3(T3_WG), 0, s, a, w);
    return hipGetLastError();
}
// Configs a set can pass the budget by before every wave sees the stop flag:
// each wave has at most one batch of U inserts per lane in flight.
int t3_block() {
    constexpr int u = Narrow::U > Narrow::UA ? Narrow::U : Narrow::UA, w = Wide::U > Wide::UA ? Wide::U : Wide::UA;
    return T3_WG * (u > w ? u : w);
}
size_t cfg_bytes_narrow() { return sizeof(Narrow::T); }
size_t cfg_bytes_wide() { return sizeof(Wide::T); }

}  // namespace lcd
