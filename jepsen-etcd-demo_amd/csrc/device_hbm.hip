// device_hbm.hip -- HBM tier (T3) of the JIT linearization search.
//
// Same set computation as the LDS tiers (device_search.hip; semantics in
// oracle/linear_ref.py), for keys whose config sets outgrow LDS or whose
// window needs more than 56 slots / 255 register states.  One workgroup of
// WG threads searches one key; its S / S' / I arrays and the two
// open-addressed hash sets live in a per-block HBM workspace slot sized from
// the search budget (a key can never hold more than budget + WG configs:
// insertion stops as soon as a count passes the budget, which is exactly
// the LC_CAUSE_BUDGET verdict).
//
// Hash sets, open addressing with linear probing:
//   narrow (u64 configs): one 64-bit atomicCAS on EMPTY per probe.
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
    __device__ static bool insert(T *tab, uint32_t mask, T key, uint32_t &pos, uint32_t *err) {
        uint32_t h = hash64(key) & mask;
        for (;;) {
            unsigned long long old = atomicCAS((unsigned long long *)&tab[h], (unsigned long long)EMPTY,
                                               (unsigned long long)key);
            if (old == EMPTY) { pos = h; return true; }
            if (old == key) { pos = h; return false; }
            h = (h + 1) & mask;
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
    uint32_t nSn, nI, stop, err;
    int32_t work;
    unsigned long long probes;
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
__device__ void write_final_hbm(const Args &a, int32_t key, const typename C::T *S, uint32_t nS) {
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

// Search one key with the whole workgroup.  Returns K_DONE or K_WIDE.
template <class C, int WG>
__device__ int search_key_hbm(const Args &a, const HbmWs &w, int32_t key, Slot<C> &sl, HbmShared<C, WG> &sh) {
    const uint32_t tid = threadIdx.x;
    const uint64_t b = a.ev_off[key], e = a.ev_off[key + 1];
    const uint32_t tb = a.trans_off ? a.trans_off[key] : 0u;
    const uint32_t cap = w.cap, hmask = w.hmask;
    if (a.key_states && a.key_states[key] > LC_WIDE_MAX_STATES) {
        if (tid == 0) finish_key(a, key, LC_UNKNOWN, LC_CAUSE_STATES, -1, 1, 0, 0);
        return K_DONE;
    }
    if (tid == 0) { sl.S[0][0] = C::init(a.init_state); sl.posS[0][0] = NOPOS; sh.err = 0; sh.probes = 0; }
    __syncthreads();
    int cur = 0;
    uint32_t nS = 1, nSprev = 0, nIlast = 0, peak = 1;
    uint64_t pend0 = 0, pend1 = 0;
    uint64_t probes = 0;  // this thread's share
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
                    write_final_hbm<C, WG>(a, key, sl.S[cur], nS);
                    if (tid == 0) finish_key(a, key, LC_UNKNOWN, LC_CAUSE_WINDOW, evno, peak, 0, (uint64_t)evno);
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
            if (tid == 0) { sh.nSn = 0; sh.nI = 0; sh.stop = 0; }
            __threadfence_block();
            __syncthreads();
            // -- partition S
            for (uint32_t j0 = 0; j0 < nS; j0 += WG) {
                const uint32_t j = j0 + tid;
                const bool act = j < nS;
                typename C::T c = act ? S[j] : C::init(0);
                const bool hasp = act && C::has(c, p);
                const bool toI = act && !hasp;
                uint32_t pos = NOPOS;
                bool ns = false, ni = false;
                if (hasp) ns = C::insert(sl.hS, hmask, C::drop(c, p), pos, &sh.err);
                if (toI) ni = C::insert(sl.hI, hmask, c, pos, &sh.err);
                const uint32_t rs = block_append<WG>(&sh.nSn, ns);
                const uint32_t ri = block_append<WG>(&sh.nI, ni);
                if (ns) { Sn[rs] = C::drop(c, p); posSn[rs] = pos; }
                if (ni) { sl.I[ri] = c; sl.posI[ri] = pos; }
            }
            if (tid == 0) probes += nS;
            __syncthreads();
            // -- JIT closure, level by level
            uint32_t head = 0;
            while (true) {
                const uint32_t end = sh.nI;
                if (head >= end || sh.stop || nc == 0) break;
                const uint32_t total = (end - head) * nc;
                for (uint32_t it0 = 0; it0 < total; it0 += WG) {
                    const uint32_t item = it0 + tid;
                    bool act = item < total && !*(volatile uint32_t *)&sh.stop;
                    const uint32_t ci = act ? head + item / nc : head;
                    const uint32_t k = act ? item % nc : 0;
                    const typename C::T c = sl.I[ci];
                    const uint32_t q = sh.cand_slot[k];
                    uint32_t s2 = 0;
                    act = act && !C::has(c, q) && step(C::state(c), sh.cand_desc[k], s2);
                    probes += act;
                    uint32_t pos = NOPOS;
                    const typename C::T c2 = C::lin(c, q, s2);
                    const bool nw = act && C::insert(sl.hI, hmask, c2, pos, &sh.err);
                    const uint32_t r = block_append<WG>(&sh.nI, nw);
                    if (nw) {
                        if (r < cap) { sl.I[r] = c2; sl.posI[r] = pos; } else sh.err = 1;
                        if (r + 1 > a.budget) sh.stop = 1;
                    }
                }
                __syncthreads();
                head = end;
            }
            __syncthreads();
            const uint32_t nI = sh.nI < cap ? sh.nI : cap;
            if (sh.nI > a.budget || sh.err) {
                const int cause = sh.err ? LC_CAUSE_ERROR : LC_CAUSE_BUDGET;
                const uint32_t nSn_now = sh.nSn;
                erase_all<C, WG>(w, sl, sl.posI, nI, posSn, nSn_now);
                write_final_hbm<C, WG>(a, key, S, nS);
                probes = block_sum<WG>(probes, &sh.probes);
                if (tid == 0) finish_key(a, key, LC_UNKNOWN, cause, evno, peak, probes, (uint64_t)evno);
                return K_DONE;
            }
            // -- apply p
            for (uint32_t j0 = 0; j0 < nI; j0 += WG) {
                const uint32_t j = j0 + tid;
                bool act = j < nI && !*(volatile uint32_t *)&sh.stop;
                const typename C::T c = act ? sl.I[j] : C::init(0);
                uint32_t s2 = 0;
                act = act && step(C::state(c), dp, s2);
                probes += act;
                uint32_t pos = NOPOS;
                const typename C::T c2 = C::restate(c, s2);
                const bool nw = act && C::insert(sl.hS, hmask, c2, pos, &sh.err);
                const uint32_t r = block_append<WG>(&sh.nSn, nw);
                if (nw) {
                    if (r < cap) { Sn[r] = c2; posSn[r] = pos; } else sh.err = 1;
                    if (r + 1 > a.budget) sh.stop = 1;
                }
            }
            __syncthreads();
            const uint32_t nSn_all = sh.nSn;
            const uint32_t nSn = nSn_all < cap ? nSn_all : cap;
            nIlast = nI;
            if (nSn_all == 0 || nSn_all > a.budget || sh.err) {
                const int verdict = nSn_all == 0 ? LC_INVALID : LC_UNKNOWN;
                const int cause = sh.err ? LC_CAUSE_ERROR : (nSn_all == 0 ? LC_CAUSE_NONLIN : LC_CAUSE_BUDGET);
                erase_all<C, WG>(w, sl, sl.posI, nI, posSn, nSn);
                write_final_hbm<C, WG>(a, key, S, nS);
                probes = block_sum<WG>(probes, &sh.probes);
                if (tid == 0)
                    finish_key(a, key, verdict, cause, evno, peak, probes, (uint64_t)evno + (verdict == LC_INVALID));
                return K_DONE;
            }
            nSprev = nSn;
            cur ^= 1;
            nS = nSn;
            peak = nS > peak ? nS : peak;
            if (p < 64) pend0 &= ~(1ull << p); else pend1 &= ~(1ull << (p - 64));
        }
    }
    __syncthreads();
    erase_all<C, WG>(w, sl, sl.posI, nIlast, sl.posS[cur], nSprev);
    write_final_hbm<C, WG>(a, key, sl.S[cur], nS);
    probes = block_sum<WG>(probes, &sh.probes);
    if (tid == 0) finish_key(a, key, LC_VALID, LC_CAUSE_NONE, -1, peak, probes, e - b);
    return K_DONE;
}

template <class C, int WG>
__global__ __launch_bounds__(WG) void k_search_hbm(Args a, HbmWs w) {
    __shared__ HbmShared<C, WG> sh;
    Slot<C> sl = slot_ptrs<C>(w, blockIdx.x);
    const int32_t n = a.n_in ? *a.n_in : a.n_order;
    if (n == 0) return;  // empty work list
    for (;;) {
        if (threadIdx.x == 0) sh.work = atomicAdd(a.ticket, 1);
        __syncthreads();
        const int32_t wi = sh.work;
        __syncthreads();
        if (wi >= n) break;
        const int32_t key = a.order[wi];
        const int r = search_key_hbm<C, WG>(a, w, key, sl, sh);
        if (r == K_WIDE && threadIdx.x == 0) {
            const int32_t i = atomicAdd(a.n_wide, 1);
            a.wide[i] = key;
        }
        __syncthreads();
    }
}

constexpr int T3_WG = 512;

hipError_t launch_t3_narrow(const Args &a, const HbmWs &w, int grid, hipStream_t s) {
    hipLaunchKernelGGL((k_search_hbm<Narrow, T3_WG>), dim3(grid), dim3(T3_WG), 0, s, a, w);
    return hipGetLastError();
}
hipError_t launch_t3_wide(const Args &a, const HbmWs &w, int grid, hipStream_t s) {
    hipLaunchKernelGGL((k_search_hbm<Wide, T3_WG>), dim3(grid), dim3(T3_WG), 0, s, a, w);
    return hipGetLastError();
}
int t3_block() { return T3_WG; }
size_t cfg_bytes_narrow() { return sizeof(Narrow::T); }
size_t cfg_bytes_wide() { return sizeof(Wide::T); }

}  // namespace lcd
