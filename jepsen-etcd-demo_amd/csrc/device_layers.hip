// device_layers.hip -- the HBM tier in layered form (T3L).
//
// Same sets as every other tier (semantics in oracle/linear_ref.py; the
// knossos.linear JIT search behind etcdemo.clj:117-118), for narrow keys
// (<= 56 window slots) with at most 8 register states -- the demo's
// cas-register over values 0..4 has 6 (etcdemo.clj:67-69) -- whose config
// sets outgrew the LDS tiers (the frontier blow-up).
//
// Two changes of representation against the config-keyed HBM hash sets of
// device_hbm.hip:
//
//  * An entry is a set of linearized ops L with the MASK of register states
//    the configs (s, L) of the set hold: L | M << 56, one u64.  Configs
//    sharing L share an entry (2.7-2.9 configs per entry in C4's closures,
//    tools/t3_mask_stats.py), and an op's step is a mask transfer,
//    T(M) = min(M & k, cap) << b (read-any: k = cap = all; read a: k = {a};
//    write b: cap = 1; cas a -> b: k = {a}, cap = 1), as in the register tier.
//
//  * Sets are kept ordered by |L| ("layers").  Linearizing an op adds one
//    element to L, so the JIT closure I of :ok(p) is built layer by layer,
//    I_{k+1} = (S_{k+1} without p) U successors of I_k, and every entry of
//    I_{k+1} is final once layer k is done; likewise
//    S'_k = {(L - p, M) : (L, M) in S_{k+1}, p in L} U {(L, T_p(M)) : I_k}.
//    Duplicates can only meet inside one layer, so one step per layer
//    merges I_{k+1} and S'_k in two LDS hash tables at once (one barrier to
//    merge, one to stream them out): I_{k+1} into a compact LDS array (HBM
//    when larger), S'_k appended to the next config set's array in HBM.  The
//    (entry, candidate op) pairs of I_k's successors are spread over all
//    1,024 threads.  A layer too large for its half of the LDS (or a merge
//    that overflows its table) is redone on the whole 16,384-slot table, in
//    P passes if needed (pass j: the entries whose hash has top bits j).
//    No hash table lives in HBM: HBM traffic is the coalesced streaming of
//    the set arrays.
//
// Budget, verdicts, failing events, peaks and probe counts are config counts
// (popcounts of the masks), identical to the oracle's: a key is :unknown as
// soon as |I| or |S'| exceeds the budget at an :ok (both only grow while the
// :ok is processed, so the event is the oracle's).  Keys this form does not
// hold go on: more than 8 states -> the config-keyed narrow tier (a.spill),
// a window slot >= 56 -> the wide tier (a.wide), as from device_hbm.hip.

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../../include/lincheck.h"
#include "device_common.hpp"
#include "device_search.hpp"

namespace lcd {
namespace {

extern "C" __device__ int32_t __ockl_wfred_add_i32(int32_t);

#ifndef LC_T3L_LWG
#define LC_T3L_LWG 1024
#endif
constexpr int LWG = LC_T3L_LWG;         // threads per key (A/B: make variant VFLAGS=-DLC_T3L_LWG=n)
constexpr uint32_t TS = 16384;          // LDS table slots (128 KB): two halves, or one table
constexpr uint32_t TSH = TS / 2;        // a half (the fused step's I and S' tables)
constexpr uint32_t CLAIM_MAX = 12288;   // entries per full-table pass (75 % load)
constexpr uint32_t LAY_STATES = 8;      // register states a mask holds
constexpr uint32_t NLAY = LC_NARROW_MAX_SLOTS + 1;  // |L| = 0 .. 56
constexpr uint32_t ECH = 256;           // events staged per chunk
constexpr uint32_t LCAP = 2560;         // entries of a layer kept compact in LDS

// Per-step counters, two sets used in turn: a step's set is zeroed during
// the step before it, so a step needs no barrier of its own to reset them.
struct StepCtr {
    uint32_t claims, emit, ovf, pad;
    unsigned long long cfg, cfg2, probes;
};

struct LayShared {
    uint64_t tab[TS];          // merge tables: 0 = empty, else L | M << 56
    uint64_t icmp[LCAP];       // the current closure layer, when it fits
    uint32_t ev[ECH];
    uint32_t evx[ECH];         // invokes: their mask transfer (k | cap << 8 | b << 16)
    uint32_t sxf[64];          // per window slot: the pending op's transfer
    uint32_t cq[64], cx[64];   // this :ok's candidate slots and their transfers
    uint32_t soff[2][NLAY + 1];  // layer offsets of the two S arrays
    StepCtr ct[2];
    uint32_t n_sn, err;
    int32_t work;
    int32_t coop_part;  // a cooperative pass claimed (-1: none left), broadcast by thread 0
    int32_t coop_slot;  // a helper's job slot
    uint32_t coop_res;  // a cooperative step: 1 a pass overflowed, 2 the wait timed out
#ifdef LC_T3L_CNT
    unsigned long long sc[6];  // whole-table steps (thread 0): insert / scan cycles (I, S'), passes (I, S'), entries in
#endif
};

// Mask transfer of a descriptor (include/lincheck.h LC_T_*) over <= 8 states.
__device__ __forceinline__ uint32_t xfer_of8(uint32_t d) {
    const uint32_t f = d & 3u, a = (d >> 2) & 0x7FFFu, b = d >> 17;
    uint32_t k = (f == LC_T_READ_ANY || f == LC_T_WRITE) ? 0xFFu : (a < LAY_STATES ? 1u << a : 0u);
    const uint32_t cap = f >= LC_T_WRITE ? 1u : 0xFFu;
    const uint32_t sh = f >= LC_T_WRITE ? b : 0u;
    if (sh >= LAY_STATES) k = 0;  // a state the key lacks: never legal (validated batches have none)
    return k | cap << 8 | (sh & 7u) << 16;
}
__device__ __forceinline__ uint32_t xfer8(uint32_t M, uint32_t x) {
    return min(M & x & 0xFFu, (x >> 8) & 0xFFu) << (x >> 16);
}

__device__ __forceinline__ uint32_t pow2_at_least(uint32_t x) {
    return x <= 1u ? 1u : 1u << (32 - __builtin_clz(x - 1u));
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t s = ((uint64_t)hi << 32 | lo) + ((uint64_t)__shfl_xor(hi, o) << 32 | __shfl_xor(lo, o));
        lo = (uint32_t)s;
        hi = (uint32_t)(s >> 32);
    }
    return (uint64_t)hi << 32 | lo;
}

// Merge (L, M) into a table (slot hash h, tsm = slots - 1).  Returns 1 if it
// claimed an empty slot.  A probe sequence longer than PMAX (a table filling
// up) gives up and raises *ovf: the caller redoes the merge with more room.
constexpr uint32_t PMAX = 64;
__device__ __forceinline__ uint32_t tab_merge(uint64_t *tab, uint32_t h, uint32_t tsm, uint64_t L, uint32_t M,
                                              uint32_t *ovf) {
    const uint64_t want = L | (uint64_t)M << 56;
    for (uint32_t n = 0;; ++n) {
        if (n == PMAX) { *ovf = 1u; return 0u; }
        h &= tsm;
        // CAS first: in LDS an atomic costs what a load does, and it answers
        // both "empty" (claimed) and "who is here" in one round trip
        const uint64_t cur = atomicCAS((unsigned long long *)&tab[h], 0ull, (unsigned long long)want);
        if (cur == 0) return 1u;
        if ((cur & LMASK) == L) {
            if (((uint32_t)(cur >> 56) & M) != M)
                (void)__hip_atomic_fetch_or(&tab[h], (uint64_t)M << 56, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            return 0u;
        }
        ++h;
    }
}

// U merges with their first probes (CASes) in flight together; a merge whose
// home slot holds another entry continues serially.  Returns the claims.
template <int U>
__device__ __forceinline__ uint32_t tab_merge_n(uint64_t *tab, uint32_t tsm, const uint64_t (&L)[U],
                                                const uint32_t (&M)[U], const uint32_t (&h)[U], const bool (&act)[U],
                                                uint32_t *ovf) {
    uint64_t cur[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        cur[u] = act[u] ? atomicCAS((unsigned long long *)&tab[h[u] & tsm], 0ull,
                                    (unsigned long long)(L[u] | (uint64_t)M[u] << 56))
                        : 1ull;
    uint32_t claims = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (!act[u]) continue;
        if (cur[u] == 0) { ++claims; continue; }
        if ((cur[u] & LMASK) == L[u]) {
            if (((uint32_t)(cur[u] >> 56) & M[u]) != M[u])
                (void)__hip_atomic_fetch_or(&tab[h[u] & tsm], (uint64_t)M[u] << 56, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_WORKGROUP);
            continue;
        }
        claims += tab_merge(tab, h[u] + 1u, tsm, L[u], M[u], ovf);
    }
    return claims;
}

// This wave's claims into c->claims (no return: checked after the barrier).
__device__ __forceinline__ void count_claims(StepCtr *c, uint32_t claimed) {
    const uint64_t bm = __ballot(claimed != 0u);
    if (bm && lane_id() == 0) __hip_atomic_fetch_add(&c->claims, (uint32_t)__popcll(bm), __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Scan slots [0, tsm] of a table: append every entry to out (positions from
// *count, at most cap), clear the slot, and hand the entry to the visitor
// (this thread's accumulators).
template <class F>
__device__ __forceinline__ void scan_emit(LayShared &sh, uint64_t *tab, uint32_t tsm, uint64_t *out, uint32_t cap,
                                          uint32_t *count, F &&visit) {
    const uint32_t tid = threadIdx.x;
    for (uint32_t s0 = 0; s0 <= tsm; s0 += LWG) {
        const uint32_t s = s0 + tid;
        uint64_t e = 0;
        if (s <= tsm) {
            e = tab[s];
            if (e) tab[s] = 0;
        }
        const uint64_t bm = __ballot(e != 0);
        if (bm == 0) continue;
        uint32_t base = 0;
        if (lane_id() == 0) base = atomicAdd(count, (uint32_t)__popcll(bm));
        base = __builtin_amdgcn_readfirstlane(base);
        if (e) {
            const uint32_t pos = base + rank_of(bm);
            if (pos < cap) out[pos] = e;
            else sh.err = 1u;
            visit(e);
        }
    }
}

// The fused step's two scans in one loop (their LDS round trips overlap):
// table A (tsa slots, if ta) into ia (cap_a), table B (tsb slots, if tb) into
// sb_out from *nb.
template <class FA, class FB>
__device__ __forceinline__ void scan_emit2(LayShared &sh, uint64_t *ta, uint32_t tsa, uint64_t *ia, uint32_t cap_a,
                                           uint32_t *na, FA &&va, uint64_t *tb, uint32_t tsb, uint64_t *sb_out,
                                           uint32_t cap_b, uint32_t *nb, FB &&vb) {
    const uint32_t tid = threadIdx.x;
    const uint32_t n = max(ta ? tsa : 0u, tb ? tsb : 0u);
    for (uint32_t s0 = 0; s0 < n; s0 += LWG) {
        const uint32_t s = s0 + tid;
        uint64_t ea = 0, eb = 0;
        if (ta && s < tsa) {
            ea = ta[s];
            if (ea) ta[s] = 0;
        }
        if (tb && s < tsb) {
            eb = tb[s];
            if (eb) tb[s] = 0;
        }
        const uint64_t ba = __ballot(ea != 0), bb = __ballot(eb != 0);
        uint32_t base_a = 0, base_b = 0;
        if (lane_id() == 0) {
            if (ba) base_a = atomicAdd(na, (uint32_t)__popcll(ba));
            if (bb) base_b = atomicAdd(nb, (uint32_t)__popcll(bb));
        }
        base_a = __builtin_amdgcn_readfirstlane(base_a);
        base_b = __builtin_amdgcn_readfirstlane(base_b);
        if (ea) {
            const uint32_t pos = base_a + rank_of(ba);
            if (pos < cap_a) ia[pos] = ea;
            else sh.err = 1u;
            va(ea);
        }
        if (eb) {
            const uint32_t pos = base_b + rank_of(bb);
            if (pos < cap_b) sb_out[pos] = eb;
            else sh.err = 1u;
            vb(eb);
        }
    }
}

__device__ __forceinline__ void clear_slots(uint64_t *tab, uint32_t n) {
    for (uint32_t s = threadIdx.x; s < n; s += LWG) tab[s] = 0;
}

// Block-wide sums of this thread's accumulators into c (read after a
// barrier).  Per thread and step they fit 32 bits (<= 16 entries of <= 57
// candidates x 8 states each).
__device__ __forceinline__ void add_sums(StepCtr *c, uint32_t c1, uint32_t c2, uint32_t pr) {
    const uint32_t s1 = (uint32_t)__ockl_wfred_add_i32((int32_t)c1);
    const uint32_t s2 = (uint32_t)__ockl_wfred_add_i32((int32_t)c2);
    const uint32_t s3 = (uint32_t)__ockl_wfred_add_i32((int32_t)pr);
    if (lane_id() == 0) {
        if (s1) atomicAdd(&c->cfg, (unsigned long long)s1);
        if (s2) atomicAdd(&c->cfg2, (unsigned long long)s2);
        if (s3) atomicAdd(&c->probes, (unsigned long long)s3);
    }
}

__device__ void write_final_layers(int32_t key, const uint64_t *S, uint32_t nS) {
    KArgs &a = kargs();
    if (!a.final_cfg || threadIdx.x != 0) return;
    uint32_t nf = 0;
    for (uint32_t j = 0; j < nS && nf < (uint32_t)a.max_final; ++j) {
        const uint64_t e = S[j];
        for (uint32_t m = (uint32_t)(e >> 56); m && nf < (uint32_t)a.max_final; m &= m - 1u) {
            const uint32_t s = (uint32_t)__builtin_ctz(m);
            a.final_cfg[((size_t)key * a.max_final + nf) * 2 + 0] = e & LMASK;
            a.final_cfg[((size_t)key * a.max_final + nf) * 2 + 1] = (uint64_t)s << 48;
            ++nf;
        }
    }
    if (a.n_final) a.n_final[key] = nf;
}

enum { K_OLD = 3 };  // more states than a mask holds: the config-keyed narrow tier

// Diagnostic build only (make variant NAME=t3lcnt VFLAGS=-DLC_T3L_CNT):
// thread 0 accumulates per-key phase cycles and step counts and writes them
// over the key's final-config words (tools/t3l_cnt.py reads them back).
#ifdef LC_T3L_CNT
#define LC_DECL uint64_t lq[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}; uint64_t lq_t = __builtin_amdgcn_s_memtime(), lq_0 = lq_t;
#define LC_MARK(i) do { if (tid == 0) { const uint64_t t_ = __builtin_amdgcn_s_memtime(); lq[i] += t_ - lq_t; lq_t = t_; } } while (0)
#define LC_ADD(i, x) do { if (tid == 0) lq[i] += (x); } while (0)
#define LC_DUMP() do { KArgs &a = kargs(); if (tid == 0 && a.final_cfg) { lq[9] = __builtin_amdgcn_s_memtime() - lq_0; \
    for (int q_ = 0; q_ < 10; ++q_) a.final_cfg[(size_t)key * a.max_final * 2 + q_] = lq[q_]; \
    for (int q_ = 0; q_ < 6; ++q_) a.final_cfg[(size_t)key * a.max_final * 2 + 10 + q_] = sh.sc[q_]; } } while (0)
#else
#define LC_DECL
#define LC_MARK(i) do {} while (0)
#define LC_ADD(i, x) do {} while (0)
#define LC_DUMP() do {} while (0)
#endif


// One :ok's view of the sets (every thread holds the same values).
struct OkCtx {
    const uint64_t *S;   // the config set, layer-ordered
    const uint32_t *so;  // its layer offsets
    uint64_t *Sn;        // the next config set (appended)
    uint64_t cand;       // pending slots other than p
    uint32_t p, xp, nc;
    uint32_t cap;
    bool probes;         // count probes
};

// Per emitted closure entry: its configs, and (counting probes) the legal
// successor steps and applications of p the oracle counts for it.
struct IVisit {
    const LayShared &sh;
    const OkCtx &o;
    uint32_t &cfg, &pr;
    __device__ void operator()(uint64_t en) const {
        const uint32_t M = (uint32_t)(en >> 56);
        cfg += (uint32_t)__builtin_popcount(M);
        if (o.probes) {
            for (uint64_t mm = o.cand & ~en & LMASK; mm; mm &= mm - 1)
                pr += (uint32_t)__builtin_popcount(M & sh.sxf[__builtin_ctzll(mm)] & 0xFFu);
            pr += (uint32_t)__builtin_popcount(M & o.xp & 0xFFu);
        }
    }
};
struct SVisit {
    uint32_t &cfg;
    __device__ void operator()(uint64_t en) const { cfg += (uint32_t)__builtin_popcount((uint32_t)(en >> 56)); }
};

// Inserts of one step, filtered to a partition: S_{k+1} entries (sources of
// I_{k+1} without p -> table A, with p -> Ret into table B), I_k's entries
// (T_p -> B) and their successor pairs (-> A).  A null table skips its
// inserts.  Claims into A are counted into c; a merge that gives up raises
// c->ovf.
struct Part {
    uint32_t shift, part;
    bool multi;
    __device__ bool mine(uint32_t h) const { return !multi || (h >> shift) == part; }
};
// The fused step's sizing (A/B: make variant VFLAGS="-DLC_T3L_EST=n -DLC_T3L_FILL=m"):
// I_{k+1} is estimated as |S_{k+1}| + EST x |I_k| + 64 entries, and a layer
// takes the fused step while both estimates fit FILL/8 of a half table.
#ifndef LC_T3L_EST
#define LC_T3L_EST 2u  // C4 at 2^16: 15.62 ms against 15.78 (3) and 16.23 (1)
#endif
#ifndef LC_T3L_FILL
#define LC_T3L_FILL 6u
#endif
#ifndef LC_T3L_UP
#define LC_T3L_UP 2
#endif
// the fused step's table sizes: I_{k+1}'s at least TSA/2 x its estimate, S'_k's
// at least (1 + 1/TSB) x its bound (A/B: make variant VFLAGS=-DLC_T3L_TSA=n)
#ifndef LC_T3L_TSA
#define LC_T3L_TSA 4u
#endif
#ifndef LC_T3L_TSB
#define LC_T3L_TSB 2u  // C4 at 2^16: 14.09-14.12 ms against 14.28-14.32 (3) and 14.37 (5), tools/gpu_r4zb.sh, gpu_r4zc.sh
#endif
constexpr int UP = LC_T3L_UP;  // successor pairs per thread in flight (A/B: make variant VFLAGS=-DLC_T3L_UP=n)
// The first two entries per thread of an S layer [sb, se), loaded ahead.
struct SPre {
    uint64_t s0, s1;
};
__device__ __forceinline__ SPre s_prefetch(const OkCtx &o, uint32_t sb, uint32_t se) {
    const uint32_t tid = threadIdx.x;
    SPre r{0, 0};
    if (sb + tid < se) r.s0 = o.S[sb + tid];
    if (sb + LWG + tid < se) r.s1 = o.S[sb + LWG + tid];
    return r;
}

template <class SRC>
__device__ __forceinline__ void step_inserts(LayShared &sh, const OkCtx &o, uint32_t sb, uint32_t se,
                                             const SRC *Ik, uint32_t nk, uint64_t *ta, uint32_t tsma,
                                             uint64_t *tb, uint32_t tsmb, const Part &pt, StepCtr *c,
                                             const SPre &pre) {
    const uint32_t tid = threadIdx.x;
    // S_{k+1}: the first two entries per thread were loaded ahead (pre) and
    // are merged after the successor pairs
    const uint64_t s0 = pre.s0, s1 = pre.s1;
    const bool h0 = sb + tid < se, h1 = sb + LWG + tid < se;
    uint32_t claims = 0;
// LC_T3L_PAIR2 (default): each thread keeps one candidate and walks entries;
// 0: pairs by index, the entry from a corrected float quotient (C4 at 2^16:
// 15.1 ms against 14.2 with the candidate per thread)
#ifndef LC_T3L_PAIR2
#define LC_T3L_PAIR2 1
#endif
    if (LC_T3L_PAIR2 && ta && o.nc) {
        // thread t takes candidate t mod nc of entries t / nc, t / nc + LWG /
        // nc, ...: the candidate's slot and transfer are loaded once, and no
        // pair index is divided
        const uint32_t nc = o.nc, cidx = tid % nc, stride = LWG / nc;
        const uint32_t j0 = tid / nc;
        const bool lane_on = j0 < stride;  // the last tid % nc lanes of the block idle
        const uint32_t q = lane_on ? sh.cq[cidx] : 0u, xq = lane_on ? sh.cx[cidx] : 0u;
        for (uint32_t jb = 0; jb < nk; jb += stride * UP) {
            uint64_t L2[UP];
            uint32_t M2[UP], h[UP];
            bool act[UP];
#pragma unroll
            for (int u = 0; u < UP; ++u) {
                const uint32_t j = jb + (uint32_t)u * stride + j0;
                act[u] = false;
                L2[u] = 0;
                M2[u] = 0;
                h[u] = 0;
                if (lane_on && j < nk) {
                    const uint64_t en = Ik[j];
                    M2[u] = ((en >> q) & 1ull) ? 0u : xfer8((uint32_t)(en >> 56), xq);
                    L2[u] = (en & LMASK) | 1ull << q;
                    h[u] = hash64(L2[u]);
                    act[u] = M2[u] != 0 && pt.mine(h[u]);
                }
            }
            claims += tab_merge_n<UP>(ta, tsma, L2, M2, h, act, &c->ovf);
        }
    } else if (ta && o.nc) {
        // pair i = (entry i / nc, candidate i % nc); the quotient from a float
        // reciprocal, corrected
        const uint32_t npairs = nk * o.nc;
        const float inv = 1.0f / (float)o.nc;
        for (uint32_t i0 = 0; i0 < npairs; i0 += LWG * UP) {
            uint64_t L2[UP];
            uint32_t M2[UP], h[UP];
            bool act[UP];
#pragma unroll
            for (int u = 0; u < UP; ++u) {
                const uint32_t i = i0 + (uint32_t)u * LWG + tid;
                act[u] = false;
                L2[u] = 0;
                M2[u] = 0;
                h[u] = 0;
                if (i < npairs) {
                    uint32_t j = (uint32_t)((float)i * inv);
                    while (j * o.nc > i) --j;
                    while ((j + 1) * o.nc <= i) ++j;
                    const uint32_t cidx = i - j * o.nc;
                    const uint64_t en = Ik[j];
                    const uint32_t q = sh.cq[cidx];
                    M2[u] = ((en >> q) & 1ull) ? 0u : xfer8((uint32_t)(en >> 56), sh.cx[cidx]);
                    L2[u] = (en & LMASK) | 1ull << q;
                    h[u] = hash64(L2[u]);
                    act[u] = M2[u] != 0 && pt.mine(h[u]);
                }
            }
            claims += tab_merge_n<UP>(ta, tsma, L2, M2, h, act, &c->ovf);
        }
    }
    if (tb) {
        for (uint32_t j0 = 0; j0 < nk; j0 += LWG) {
            const uint32_t j = j0 + tid;
            if (j < nk) {
                const uint64_t en = Ik[j];
                const uint32_t M2 = xfer8((uint32_t)(en >> 56), o.xp);
                if (M2) {
                    const uint64_t L = en & LMASK;
                    const uint32_t h = hash64(L);
                    if (pt.mine(h)) (void)tab_merge(tb, h, tsmb, L, M2, &c->ovf);
                }
            }
        }
    }
    auto s_entry = [&](uint64_t en) {
        const uint64_t L = en & LMASK;
        const uint32_t M = (uint32_t)(en >> 56);
        if ((L >> o.p) & 1ull) {
            if (tb) {
                const uint64_t L2 = L & ~(1ull << o.p);
                const uint32_t h = hash64(L2);
                if (pt.mine(h)) (void)tab_merge(tb, h, tsmb, L2, M, &c->ovf);
            }
        } else if (ta) {
            const uint32_t h = hash64(L);
            if (pt.mine(h)) claims += tab_merge(ta, h, tsma, L, M, &c->ovf);
        }
    };
    if (h0) s_entry(s0);
    if (h1) s_entry(s1);
    for (uint32_t j = sb + 2 * LWG + tid; j < se; j += LWG) s_entry(o.S[j]);
    if (ta) {
        // this thread's claims, summed over the wave, into c->claims
        const uint32_t w = (uint32_t)__ockl_wfred_add_i32((int32_t)claims);
        if (lane_id() == 0 && w)
            __hip_atomic_fetch_add(&c->claims, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

__device__ __forceinline__ void zero_ctr(StepCtr *c) {
    c->claims = 0; c->emit = 0; c->ovf = 0;
    c->cfg = 0; c->cfg2 = 0; c->probes = 0;
}

// ---- cooperating blocks (the slowest key's whole-table steps)
//
// A block whose key queue is empty does not exit: it helps the blocks still
// searching with their whole-table steps.  Such a step is P independent
// passes, one per hash partition of its entries (pass j merges the entries
// whose hash has top bits j into an LDS table of its own and appends them to
// the step's output array); a block that reaches one with helpers idle posts
// it on the launch's board (one job slot per block), split into at least as
// many partitions as there are idle helpers (2 .. LC_T3L_COOP_MAX), and waits
// while they run them.  Output positions come from one counter in HBM, the
// sums (configs, overflow, errors) from atomics on the job.  Helpers leave
// only when no block searches a key, so a posted job always has one.  The output is the same set of entries as the block's own passes
// produce (its order within a layer is a scan order either way), so records
// are unchanged.  Not used while counting probes (a pass's early exit at the
// budget is the sequential step's).
#ifndef LC_T3L_COOP
#define LC_T3L_COOP 1
#endif
#ifndef LC_T3L_COOP_MAX
#define LC_T3L_COOP_MAX 8u
#endif
struct CoopHead {
    uint32_t active;   // blocks searching a key
    uint32_t broken;   // a wait timed out: no more posting in this launch
    uint32_t passes;   // passes run by helpers (lc_stats.t3_coop_passes; offset 8)
    uint32_t pad0;
    uint32_t idle[8];  // per XCD: blocks helping (their queue is empty)
    uint32_t busy[8];  // per XCD: blocks searching a key
    uint32_t open[8];  // per XCD: jobs open -- what the helpers poll (scanning every slot at each
                       // poll took the fabric's request rate from the searches)
    uint32_t pad1[36];
};
// One block's job: word = seq << 32 | passes claimed (seq odd: open).  The
// fields are stored before the word; a claim is a CAS on the word, so it
// belongs to the job the fields describe.
struct CoopJob {
    unsigned long long word;
    uint32_t P, kind, done, emit, ovf, err, xcc, pad1;
    unsigned long long cfg;
    const uint64_t *S, *Ik;
    uint64_t *out;
    uint64_t cand;
    uint32_t sb, se, nk, cap, p, xp, nc, pad0;
    uint32_t cq[64], cx[64];
};
constexpr size_t COOP_HEAD = 256, COOP_STRIDE = 1024;
static_assert(sizeof(CoopHead) <= COOP_HEAD && sizeof(CoopJob) <= COOP_STRIDE, "board layout");
__device__ __forceinline__ CoopHead *coop_head(const LayWs &w) { return (CoopHead *)w.coop; }
__device__ __forceinline__ CoopJob *coop_job(const LayWs &w, uint32_t slot) {
    return (CoopJob *)(w.coop + COOP_HEAD + (size_t)slot * COOP_STRIDE);
}
// A job is helped only by blocks of the poster's XCD: they share its L2, so
// the passes' output, the job's fields and the poster's arrays meet there
// and the handoff needs no more than the CU's L1 invalidated (agent-scope
// fences write back and invalidate whole L2s: posting through them made
// every search of the launch 2-6x slower, its set arrays evicted).
#ifndef LC_T3L_COOP_FENCE  // 2: the poster's XCD, agent-scope fences; 1: any XCD; 0: the same XCD, L1 only
#define LC_T3L_COOP_FENCE 2
#endif
#if LC_T3L_COOP_FENCE == 3  // the poster's XCD; device-scope invalidate, no L2 write-back
__device__ __forceinline__ uint32_t xcc_id() { return __builtin_amdgcn_s_getreg((31 << 11) | 20) & 7u; }
__device__ __forceinline__ void l1_inv() { asm volatile("buffer_inv sc1" ::: "memory"); }
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
#elif LC_T3L_COOP_FENCE
#if LC_T3L_COOP_FENCE == 2  // ... helpers of the poster's XCD only
__device__ __forceinline__ uint32_t xcc_id() { return __builtin_amdgcn_s_getreg((31 << 11) | 20) & 7u; }
#else
__device__ __forceinline__ uint32_t xcc_id() { return 0u; }
#endif
__device__ __forceinline__ void l1_inv() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent"); }
__device__ __forceinline__ void vm_drain() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent"); }
#else
__device__ __forceinline__ uint32_t xcc_id() { return __builtin_amdgcn_s_getreg((31 << 11) | 20) & 7u; }
__device__ __forceinline__ void l1_inv() { asm volatile("buffer_inv sc0" ::: "memory"); }
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
#endif
__device__ __forceinline__ uint32_t ld_rlx(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_rlx64(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_rlx(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_rlx64(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Thread 0: claim a pass of the job open in j (its index), or -1.  After a
// claim the CU's L1 is invalidated: the job's fields and arrays are read
// fresh from the XCD's L2.
__device__ int coop_claim(CoopJob *j) {
    unsigned long long w = __hip_atomic_load(&j->word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int t = 0; t < 64; ++t) {
        if (!((w >> 32) & 1ull)) return -1;
        // (P is the open job's once the CAS below succeeds on this word)
        const uint32_t P = ld_rlx(&j->P);
        if ((uint32_t)w >= P) return -1;
        if (__hip_atomic_compare_exchange_strong(&j->word, &w, w + 1ull, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)) {
            l1_inv();
            return (int)(uint32_t)w;
        }
    }
    return -1;
}

// One pass (partition `part` of P) of job j, by the whole block: kind 0
// merges I_{k+1}, kind 1 S'_k, into sh.tab, and appends the partition to
// j->out from j->emit.  Counts itself done in j.  Leaves the table clear and
// ct[0] dirty.
__device__ void coop_pass(LayShared &sh, const OkCtx &o, uint32_t sb, uint32_t se, const uint64_t *Ik, uint32_t nk,
                          uint32_t kind, uint32_t P, uint32_t part, uint64_t *out, uint32_t cap, CoopJob *j) {
    const uint32_t tid = threadIdx.x;
    StepCtr *c = &sh.ct[0];
    const Part pt{32u - (uint32_t)__builtin_ctz(P), part, P > 1};
    __syncthreads();
    if (tid == 0) { zero_ctr(c); sh.err = 0; }
    __syncthreads();
    if (kind == 0)
        step_inserts(sh, o, sb, se, Ik, nk, sh.tab, TS - 1, nullptr, 0, pt, c, s_prefetch(o, sb, se));
    else
        step_inserts(sh, o, sb, se, Ik, nk, nullptr, 0, sh.tab, TS - 1, pt, c, s_prefetch(o, sb, se));
    __syncthreads();
    const bool bad = c->ovf || (kind == 0 && c->claims > CLAIM_MAX);
    if (bad) {
        clear_slots(sh.tab, TS);
    } else {
        uint32_t ca = 0, pa = 0, cs = 0;
        if (kind == 0) scan_emit(sh, sh.tab, TS - 1, out, cap, &j->emit, IVisit{sh, o, ca, pa});
        else scan_emit(sh, sh.tab, TS - 1, out, cap, &j->emit, SVisit{cs});
        add_sums(c, ca, cs, 0);
    }
    vm_drain();  // this thread's output stores in the XCD's L2
    __syncthreads();
    if (tid == 0) {
        if (bad) atomicOr(&j->ovf, 1u);
        else atomicAdd(&j->cfg, kind == 0 ? c->cfg : c->cfg2);
        if (sh.err) atomicOr(&j->err, 1u);
        sh.err = 0;
        vm_drain();
        __hip_atomic_fetch_add(&j->done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Partitions for a cooperative step now: the idle helpers as a power of two,
// at least 2 (1: no cooperation).
__device__ __forceinline__ uint32_t coop_parts(const LayWs &w) {
    if (!LC_T3L_COOP || !w.coop) return 1u;
    CoopHead *hd = coop_head(w);
    if (ld_rlx(&hd->broken)) return 1u;
    // helpers per searching block of the XCD: posting with fewer swamps the
    // helpers (every pass generates all the step's pairs) while the posters
    // wait -- C4 at 2^16 measured 2x slower posting whenever 2 helpers were idle
    const uint32_t x = xcc_id();
    const uint32_t n = min(ld_rlx(&hd->idle[x]) / max(ld_rlx(&hd->busy[x]), 1u), (uint32_t)LC_T3L_COOP_MAX);
    return n < 2u ? 1u : 1u << (31 - __builtin_clz(n));
}

// A whole-table step's passes (kind, P) through this block's job slot: the
// helpers run them, the block waits (its own registers stay the search's:
// the passes' code lives in coop_help only).  Output from `base` in out.  Returns in sh.coop_res
// (after a barrier) 0, 1 (a pass overflowed: redo with more passes) or 2
// (the wait timed out); the job's output count and configs in ct[0].emit /
// ct[0].cfg.
__device__ void coop_step(LayShared &sh, const LayWs &w, const OkCtx &o, uint32_t sb, uint32_t se,
                          const uint64_t *Ik, uint32_t nk, uint32_t kind, uint32_t P, uint64_t *out, uint32_t base) {
    const uint32_t tid = threadIdx.x;
    CoopJob *j = coop_job(w, blockIdx.x);
    // (the board is read and written with agent-scope atomics only: a plain
    // store waits dirty in the poster's L2 where the helpers' atomic loads
    // do not look -- they read an earlier job's fields)
    if (tid < 64) { st_rlx(&j->cq[tid], sh.cq[tid]); st_rlx(&j->cx[tid], sh.cx[tid]); }
    const uint32_t xcc = xcc_id();
    if (tid == 0) {
        st_rlx(&j->P, P); st_rlx(&j->kind, kind); st_rlx(&j->done, 0); st_rlx(&j->emit, base); st_rlx(&j->ovf, 0);
        st_rlx(&j->err, 0); st_rlx64((uint64_t *)&j->cfg, 0); st_rlx(&j->xcc, xcc);
        st_rlx64((uint64_t *)&j->S, (uint64_t)o.S); st_rlx64((uint64_t *)&j->Ik, (uint64_t)Ik);
        st_rlx64((uint64_t *)&j->out, (uint64_t)out); st_rlx64(&j->cand, o.cand);
        st_rlx(&j->sb, sb); st_rlx(&j->se, se); st_rlx(&j->nk, nk); st_rlx(&j->cap, o.cap); st_rlx(&j->p, o.p);
        st_rlx(&j->xp, o.xp); st_rlx(&j->nc, o.nc);
    }
    vm_drain();  // the fields, and the I_k copy in `spare`, in the XCD's L2
    __syncthreads();
    if (tid == 0) {
        const unsigned long long seq = (__hip_atomic_load(&j->word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 32) + 1ull;
        __hip_atomic_store(&j->word, seq << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // open
        atomicAdd(&coop_head(w)->open[xcc], 1u);
    }
    if (tid == 0) {
        uint32_t res = 0;
        for (uint32_t spins = 0; ld_rlx(&j->done) < P; ++spins) {
            if (spins > (1u << 24)) {  // ~seconds: a helper cannot take that long; never hang the launch
                res = 2;
                __hip_atomic_store(&coop_head(w)->broken, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(8);
        }
        l1_inv();  // the passes' output, fresh from the XCD's L2 for every thread of the CU
        if (res == 0 && ld_rlx(&j->ovf)) res = 1;
        if (ld_rlx(&j->err)) sh.err = 1u;
        sh.ct[0].emit = ld_rlx(&j->emit);
        sh.ct[0].cfg = __hip_atomic_load(&j->cfg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long wd = __hip_atomic_load(&j->word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&j->word, ((wd >> 32) + 1ull) << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // close
        atomicSub(&coop_head(w)->open[xcc], 1u);
        sh.coop_res = res;
    }
    __syncthreads();  // (thread 0's acquire invalidated the CU's and the XCD's caches for every thread)
}

// A helper: runs other blocks' passes until no block searches a key.
__device__ void coop_help(LayShared &sh, const LayWs &w) {
    const uint32_t tid = threadIdx.x, lane = lane_id();
    CoopHead *hd = coop_head(w);
    const uint32_t ns = w.coop_slots, xcc = xcc_id();
    if (tid == 0) atomicAdd(&hd->idle[xcc], 1u);
    for (;;) {
        if (tid < 64) {  // wave 0 looks for an open job with passes left, from a slot of its own
            int got = -1, slot = -1;
            const bool any = ld_rlx(&hd->open[xcc]) != 0;
            for (uint32_t b0 = 0; any && b0 < ns && got < 0; b0 += 64) {
                const uint32_t s = (b0 + lane + blockIdx.x) % ns;
                bool open = false;
                if (b0 + lane < ns) {
                    CoopJob *j = coop_job(w, s);
                    const unsigned long long wd = __hip_atomic_load(&j->word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    open = ((wd >> 32) & 1ull) && (uint32_t)wd < ld_rlx(&j->P) && ld_rlx(&j->xcc) == xcc;
                }
                uint64_t bm = __ballot(open);
                while (bm && got < 0) {
                    const uint32_t l = (uint32_t)__builtin_ctzll(bm);
                    bm &= bm - 1ull;
                    const uint32_t s2 = (b0 + l + blockIdx.x) % ns;
                    int g = -1;
                    if (lane == 0) g = coop_claim(coop_job(w, s2));
                    g = __builtin_amdgcn_readfirstlane(g);
                    if (g >= 0) { got = g; slot = (int)s2; }
                }
            }
            if (lane == 0) {
                sh.coop_part = got;
                sh.coop_slot = slot;
                // done: nothing open and no block searching (it could post)
                if (got < 0) sh.coop_res = ld_rlx(&hd->active) == 0 ? 1u : 0u;
            }
        }
        __syncthreads();
        const int part = sh.coop_part;
        if (part < 0) {
            const bool done = sh.coop_res != 0;
            __syncthreads();
            if (done) break;
            __builtin_amdgcn_s_sleep(64);  // ~4k cycles between polls
            continue;
        }
        // the job's fields (stable: our pass is claimed and not done), read
        // with vector loads: a uniform field read through the scalar cache,
        // which no L1 invalidation reaches, returned an earlier job's
        CoopJob *j = coop_job(w, (uint32_t)sh.coop_slot);
        if (tid < 64) { sh.cq[tid] = ld_rlx(&j->cq[tid]); sh.cx[tid] = ld_rlx(&j->cx[tid]); }
        OkCtx o;
        o.S = (const uint64_t *)ld_rlx64((const uint64_t *)&j->S);
        o.so = nullptr;
        uint64_t *out = (uint64_t *)ld_rlx64((const uint64_t *)&j->out);
        o.Sn = out;
        o.cand = ld_rlx64(&j->cand);
        o.p = ld_rlx(&j->p); o.xp = ld_rlx(&j->xp); o.nc = ld_rlx(&j->nc); o.cap = ld_rlx(&j->cap); o.probes = false;
        const uint32_t sb = ld_rlx(&j->sb), se = ld_rlx(&j->se), nk = ld_rlx(&j->nk), kind = ld_rlx(&j->kind),
                       P = ld_rlx(&j->P);
        const uint64_t *Ik = (const uint64_t *)ld_rlx64((const uint64_t *)&j->Ik);
        __syncthreads();  // cq / cx
        coop_pass(sh, o, sb, se, Ik, nk, kind, P, (uint32_t)part, out, o.cap, j);
        if (tid == 0) atomicAdd(&hd->passes, 1u);
        __syncthreads();
    }
}

// The whole-table form of one step (a layer too large for the fused step, or
// one whose fused merge overflowed): I_{k+1} (if want_i) in P passes into
// `iout` (HBM), doubling P while a pass overflows; then S'_k (if want_s),
// likewise.  Adds the configs to cfg_i / cfg_s and thread 0's probes.
// Returns false when the budget was exceeded (or err).  Uses ct[0]; leaves
// both counter sets zeroed.
// Cooperative (coop: helpers idle, no probe counting): each pass list goes
// through coop_step instead, at least as many passes as helpers plus one;
// an I_k held in LDS is first copied to `spare` (an HBM array no step output
// uses), where the helpers can read it.
__device__ bool step_slow(LayShared &sh, const OkCtx &o, uint32_t sb, uint32_t se, const uint64_t *Ik, uint32_t nk,
                          bool want_i, bool want_s, uint64_t *iout, uint32_t &n_out, uint32_t &pc, uint64_t &cfg_i,
                          uint64_t &cfg_s, uint64_t &probes, uint64_t budget, const LayWs &w, uint64_t *spare,
                          bool coop) {
    const uint32_t tid = threadIdx.x;
    StepCtr *c = &sh.ct[0];
    bool ok = true;
    // (one thread reads the board: the block must agree on the branch)
    if (coop) {
        __syncthreads();
        if (tid == 0) sh.coop_part = (int32_t)coop_parts(w);
        __syncthreads();
    }
    const uint32_t cp = coop ? (uint32_t)sh.coop_part : 1u;
    if (cp > 1u) {
        const uint64_t *src = Ik;
        if (Ik == sh.icmp && nk) {
            for (uint32_t q = tid; q < nk; q += LWG) spare[q] = sh.icmp[q];
            src = spare;  // (made visible to the helpers by coop_step's fence before it posts)
        }
        if (want_i) {
            uint32_t P = max(pc, cp);
            for (;;) {
                coop_step(sh, w, o, sb, se, src, nk, 0u, P, iout, 0u);
                const uint32_t res = sh.coop_res;
                if (res == 2u) { if (tid == 0) sh.err = 1u; break; }
                if (res == 0u) break;
                P *= 2u;
                if (P > 65536u) { if (tid == 0) sh.err = 1u; break; }
            }
            n_out = c->emit;
            cfg_i += c->cfg;
            const uint32_t want = (uint32_t)((2ull * n_out + CLAIM_MAX - 1) / CLAIM_MAX);
            pc = pow2_at_least(want > 0 ? want : 1u);
            __syncthreads();  // ct[0] read
            if (cfg_i > budget || sh.err) ok = false;
        }
        if (ok && want_s) {
            const uint64_t bound = (uint64_t)nk + (se - sb);
            uint32_t P2 = max(cp, pow2_at_least((uint32_t)((2 * bound + CLAIM_MAX - 1) / CLAIM_MAX)));
            __syncthreads();
            const uint32_t n0 = sh.n_sn;
            for (;;) {
                coop_step(sh, w, o, sb, se, src, nk, 1u, P2, o.Sn, n0);
                const uint32_t res = sh.coop_res;
                if (res == 2u) { if (tid == 0) sh.err = 1u; break; }
                if (res == 0u) break;
                P2 *= 2u;
                if (P2 > 65536u) { if (tid == 0) sh.err = 1u; break; }
            }
            cfg_s += c->cfg;
            const uint32_t n1 = c->emit;
            __syncthreads();  // ct[0] read
            if (tid == 0) sh.n_sn = n1;
            if (cfg_s > budget || sh.err) ok = false;
        }
        __syncthreads();
        if (tid == 0) { zero_ctr(&sh.ct[0]); zero_ctr(&sh.ct[1]); }
        __syncthreads();
        return ok;
    }
    if (want_i) {
        uint32_t P = pc;
        uint64_t cfg = 0, pr = 0;
        uint32_t emit = 0;
        for (;;) {  // until no pass overflows
            cfg = 0; pr = 0; emit = 0;
            bool redo = false;
            for (uint32_t part = 0; part < P; ++part) {
                const Part pt{32u - (uint32_t)__builtin_ctz(P), part, P > 1};
                __syncthreads();
                if (tid == 0) { zero_ctr(c); c->emit = emit; }
                __syncthreads();
#ifdef LC_T3L_CNT
                const uint64_t tq0 = __builtin_amdgcn_s_memtime();
#endif
                step_inserts(sh, o, sb, se, Ik, nk, sh.tab, TS - 1, nullptr, 0, pt, c, s_prefetch(o, sb, se));
                __syncthreads();
#ifdef LC_T3L_CNT
                const uint64_t tq1 = __builtin_amdgcn_s_memtime();
                if (tid == 0) { sh.sc[0] += tq1 - tq0; sh.sc[2] += 1; sh.sc[5] += (uint64_t)nk * o.nc + (se - sb); }
#endif
                if (c->ovf || c->claims > CLAIM_MAX) {
                    clear_slots(sh.tab, TS);
                    redo = true;
                    break;
                }
                uint32_t ca = 0, pa = 0;
                scan_emit(sh, sh.tab, TS - 1, iout, o.cap, &c->emit, IVisit{sh, o, ca, pa});
                add_sums(c, ca, 0, pa);
                __syncthreads();
#ifdef LC_T3L_CNT
                if (tid == 0) sh.sc[1] += __builtin_amdgcn_s_memtime() - tq1;
#endif
                cfg += c->cfg;
                pr += c->probes;
                emit = c->emit;
                if (cfg_i + cfg > budget || sh.err) break;
            }
            if (!redo) break;
            P *= 2u;
            if (P > 65536u) {  // cannot happen below a 2^29 budget; never spin
                if (tid == 0) sh.err = 1u;
                break;
            }
        }
        n_out = emit;
        cfg_i += cfg;
        if (tid == 0) probes += pr;
        const uint32_t want = (uint32_t)((2ull * n_out + CLAIM_MAX - 1) / CLAIM_MAX);
        pc = pow2_at_least(want > 0 ? want : 1u);
        if (cfg_i > budget || sh.err) ok = false;
    }
    if (ok && want_s) {
        const uint64_t bound = (uint64_t)nk + (se - sb);
        // half-full passes: a partition's share of the bound varies
        uint32_t P2 = pow2_at_least((uint32_t)((2 * bound + CLAIM_MAX - 1) / CLAIM_MAX));
        __syncthreads();
        const uint32_t n0 = sh.n_sn;  // this layer's start in Sn
        for (;;) {
            uint64_t cfg = 0;
            bool redo = false;
            for (uint32_t part = 0; part < P2; ++part) {
                const Part pt{32u - (uint32_t)__builtin_ctz(P2), part, P2 > 1};
                __syncthreads();
                if (tid == 0) zero_ctr(c);
                __syncthreads();
#ifdef LC_T3L_CNT
                const uint64_t tq0 = __builtin_amdgcn_s_memtime();
#endif
                step_inserts(sh, o, sb, se, Ik, nk, nullptr, 0, sh.tab, TS - 1, pt, c, s_prefetch(o, sb, se));
                __syncthreads();
#ifdef LC_T3L_CNT
                const uint64_t tq1 = __builtin_amdgcn_s_memtime();
                if (tid == 0) { sh.sc[0] += tq1 - tq0; sh.sc[3] += 1; }
#endif
                if (c->ovf) {
                    clear_slots(sh.tab, TS);
                    redo = true;
                    break;
                }
                uint32_t cs = 0;
                scan_emit(sh, sh.tab, TS - 1, o.Sn, o.cap, &sh.n_sn, SVisit{cs});
                add_sums(c, 0, cs, 0);
                __syncthreads();
#ifdef LC_T3L_CNT
                if (tid == 0) sh.sc[4] += __builtin_amdgcn_s_memtime() - tq1;
#endif
                cfg += c->cfg2;
                if (cfg_s + cfg > budget || sh.err) break;
            }
            if (!redo) {
                cfg_s += cfg;
                break;
            }
            __syncthreads();
            if (tid == 0) sh.n_sn = n0;  // drop this layer's partial output
            P2 *= 2u;
            if (P2 > 65536u) {
                if (tid == 0) sh.err = 1u;
                cfg_s += cfg;
                break;
            }
        }
        if (cfg_s > budget || sh.err) ok = false;
    }
    __syncthreads();
    if (tid == 0) { zero_ctr(&sh.ct[0]); zero_ctr(&sh.ct[1]); }
    __syncthreads();
    return ok;
}

// Search one key with the whole workgroup.
__device__ int search_key_layers(const Args &a, const LayWs &w, int32_t key, LayShared &sh) {
    const uint32_t tid = threadIdx.x;
    // (the key's setup and results through kargs(): see device_common.hpp)
    KArgs &ka = kargs();
    const uint64_t b = ka.ev_off[key], e = ka.ev_off[key + 1];
    const uint32_t tb = ka.trans_off ? ka.trans_off[key] : 0u;
    const uint32_t nstates = ka.trans_off ? (ka.key_states ? (uint32_t)ka.key_states[key] : 256u) : ka.shared_states;
    const uint32_t init_state = ka.init_state;
    if (ka.key_states && ka.key_states[key] > LC_WIDE_MAX_STATES) {
        if (tid == 0) finish_key(kargs(), key, LC_UNKNOWN, LC_CAUSE_STATES, -1, 1, 0, 0);
        return K_DONE;
    }
    if (nstates > LAY_STATES || init_state >= LAY_STATES) return K_OLD;
    char *base = w.base + (size_t)blockIdx.x * w.slot_bytes;
    uint64_t *const S0 = (uint64_t *)(base + w.off_S0), *const S1 = (uint64_t *)(base + w.off_S1);
    uint64_t *const I0 = (uint64_t *)(base + w.off_I0), *const I1 = (uint64_t *)(base + w.off_I1);
    const uint64_t budget = a.budget;
    int cur = 0;
    if (tid == 0) {
        S0[0] = (uint64_t)(1u << init_state) << 56;  // {(init, {})}
        sh.err = 0;
    }
    if (tid <= NLAY) sh.soff[0][tid] = tid == 0 ? 0u : 1u;
    uint64_t nScfg = 1, pend = 0, probes = 0;  // probes: thread 0's running total
    uint64_t sbytes = 0;  // thread 0: set-array bytes streamed (S read, S' written, spilled I layers)
#ifdef LC_T3L_CNT
    if (tid < 6) sh.sc[tid] = 0;
#endif
    uint32_t peak = 1;
    LC_DECL
    for (uint64_t cb = b; cb < e; cb += ECH) {
        const uint32_t cnt = (uint32_t)((e - cb) < ECH ? (e - cb) : ECH);
        __syncthreads();
        if (tid < cnt) {
            const uint32_t ev = a.events[cb + tid];
            sh.ev[tid] = ev;
            sh.evx[tid] = (ev & LC_EV_OK_BIT) ? 0u : xfer_of8(a.trans[tb + LC_EV_TRANS(ev)]);
        }
        __syncthreads();
        for (uint32_t i = 0; i < cnt; ++i) {
            const uint32_t evi = sh.ev[i];
            const uint32_t slot = LC_EV_SLOT(evi);
            const int32_t evno = (int32_t)(cb + i - b);
            if (!(evi & LC_EV_OK_BIT)) {
                if (slot >= LC_NARROW_MAX_SLOTS) return K_WIDE;
                pend |= 1ull << slot;
                if (tid == 0) sh.sxf[slot] = sh.evx[i];
                continue;
            }
            // ---- :ok of the op in `slot` ----
            const uint32_t p = slot;
            OkCtx o;
            o.S = cur ? S1 : S0;
            o.so = sh.soff[cur];
            o.Sn = cur ? S0 : S1;
            o.cand = pend & ~(1ull << p);
            o.p = p;
            o.nc = (uint32_t)__popcll(o.cand);
            o.cap = w.cap;
            o.probes = a.count_probes != 0;
            uint32_t *sn = sh.soff[cur ^ 1];
            if (tid == 0) { zero_ctr(&sh.ct[0]); zero_ctr(&sh.ct[1]); sh.n_sn = 0; }
            __syncthreads();  // sxf of earlier invokes visible
            LC_MARK(0);
            LC_ADD(6, 1);
            if (tid < 64) {
                const bool on = (o.cand >> tid) & 1ull;
                if (on) {
                    const uint32_t r = (uint32_t)__popcll(o.cand & ((1ull << tid) - 1ull));
                    sh.cq[r] = tid;
                    sh.cx[r] = sh.sxf[tid];
                }
            }
            o.xp = sh.sxf[p];
            // the config set's lowest and highest non-empty layers: one
            // ballot over the layer offsets (every wave; NLAY <= 64)
            uint32_t smin = NLAY, smax = 0;
            {
                const uint32_t l = lane_id();
                const uint64_t ne = __ballot(l < NLAY && o.so[l + 1] > o.so[l]);
                if (ne) {
                    smin = (uint32_t)__builtin_ctzll(ne);
                    smax = 63u - (uint32_t)__builtin_clzll(ne);
                }
            }
            if (tid == 0 && a.count_probes) probes += nScfg;  // |S| (oracle: probes += S.n)
            uint64_t nIcfg = 0, nSncfg = 0;
            bool over = false;
            // I_k: compact in LDS (sh.icmp) or in an HBM array; k = smin - 1
            // starts with I_k empty (k = -1: no S'_k to build)
            const uint64_t *Ik = sh.icmp;
            uint32_t nk = 0, pc = 1, par = 0;
            int ib = 0;  // the HBM I array the next spilled layer goes to
            int k = (int)smin - 1;
            if (tid <= NLAY && (int)tid <= k) sn[tid] = 0;
            __syncthreads();  // cq / cx
            LC_MARK(1);
            // S_{k+1}'s first entries per thread, loaded one step ahead
            SPre pre = s_prefetch(o, smin <= smax ? o.so[smin] : 0u, smin <= smax ? o.so[smin + 1] : 0u);
            for (;; ++k) {
                const uint32_t k1 = (uint32_t)(k + 1);
                if (nk == 0 && k1 > smax) break;
                const uint32_t sb = k1 <= smax ? o.so[k1] : 0u, se = k1 <= smax ? o.so[k1 + 1] : 0u;
                const SPre cur_pre = pre;
                {
                    const uint32_t k2 = k1 + 1;
                    pre = s_prefetch(o, k2 <= smax ? o.so[k2] : 0u, k2 <= smax ? o.so[k2 + 1] : 0u);
                }
                const bool want_s = k >= 0;
                const bool want_i = k1 < NLAY;
                if (tid == 0 && want_s) sn[k] = sh.n_sn;
                // fused step: both tables in their LDS halves when the sizes allow
                const uint32_t bound_s = nk + (se - sb);
                const uint32_t est_i = (se - sb) + LC_T3L_EST * nk + 64u;
                const bool fast = bound_s <= (TSH * LC_T3L_FILL) / 8u && est_i <= (TSH * LC_T3L_FILL) / 8u;
                bool done = false;
                uint32_t n_next = 0;
                uint64_t *inext = nullptr;
                if (fast) {
                    StepCtr *c = &sh.ct[par];
                    const uint32_t tsa = min(TSH, max(128u, pow2_at_least(LC_T3L_TSA * est_i / 2u)));
                    const uint32_t tsb = min(TSH, max(64u, pow2_at_least(bound_s + bound_s / LC_T3L_TSB + 1u)));
                    uint64_t *ta = sh.tab, *tbl = sh.tab + TSH;
                    if (Ik == sh.icmp)  // typed LDS reads of the layer (no flat loads)
                        step_inserts(sh, o, sb, se, sh.icmp, nk, want_i ? ta : nullptr, tsa - 1,
                                     want_s ? tbl : nullptr, tsb - 1, Part{0, 0, false}, c, cur_pre);
                    else
                        step_inserts(sh, o, sb, se, Ik, nk, want_i ? ta : nullptr, tsa - 1, want_s ? tbl : nullptr,
                                     tsb - 1, Part{0, 0, false}, c, cur_pre);
                    __syncthreads();
                    LC_MARK(2);
                    if (tid == 0) zero_ctr(&sh.ct[par ^ 1]);  // the next step's set
                    const uint32_t na = c->claims;
                    if (!c->ovf) {  // every merge found its slot
                        inext = na <= LCAP ? sh.icmp : (ib ? I1 : I0);
                        uint32_t ci = 0, cs = 0, pr = 0;
                        scan_emit2(sh, want_i ? ta : nullptr, tsa, inext, na <= LCAP ? LCAP : o.cap, &c->emit,
                                   IVisit{sh, o, ci, pr}, want_s ? tbl : nullptr, tsb, o.Sn, o.cap, &sh.n_sn, SVisit{cs});
                        add_sums(c, ci, cs, pr);
                        __syncthreads();
                        n_next = c->emit;
                        nIcfg += c->cfg;
                        nSncfg += c->cfg2;
                        if (tid == 0) probes += c->probes;
                        if (n_next > LCAP) {
                            ib ^= 1;
                            sbytes += 16ull * n_next;  // written, read back next step
                        }
                        par ^= 1u;
                        done = true;
                        LC_MARK(3);
                        LC_ADD(7, n_next);
                        LC_ADD(4, 1);
                        if (nIcfg > budget || nSncfg > budget || sh.err) { over = true; break; }
                    } else {  // a table overflowed: clear both halves, redo on the whole table
                        clear_slots(sh.tab, TS);
                        LC_ADD(8, 1);
                    }
                }
                if (!done) {
                    // Ik may live in sh.icmp, which the whole-table passes do
                    // not touch; I_{k+1} goes to HBM
                    inext = ib ? I1 : I0;
                    if (!step_slow(sh, o, sb, se, Ik, nk, want_i, want_s, inext, n_next, pc, nIcfg, nSncfg, probes,
                                   budget, w, ib ? I0 : I1, !a.count_probes)) { over = true; break; }
                    ib ^= 1;
                    par = 0;
                    sbytes += want_i ? 16ull * n_next : 0ull;
                    LC_MARK(5);
                    LC_ADD(7, n_next);
                    LC_ADD(8, 1 << 20);
                }
                Ik = inext;
                nk = want_i ? n_next : 0u;
            }
            __syncthreads();
            sbytes += 8ull * (o.so[NLAY] + sh.n_sn);
            if (over) {
                const int cause = sh.err ? LC_CAUSE_ERROR : LC_CAUSE_BUDGET;
                clear_slots(sh.tab, TS);
                write_final_layers(key, o.S, o.so[NLAY]);
                LC_DUMP();
                if (tid == 0) {
                    finish_key(kargs(), key, LC_UNKNOWN, cause, evno, peak, probes, (uint64_t)evno);
                    atomicAdd(kargs().stream_bytes, (unsigned long long)sbytes);
                }
                __syncthreads();
                return K_DONE;
            }
            if ((int)tid >= (k < 0 ? 0 : k) && tid <= NLAY) sn[tid] = sh.n_sn;
            __syncthreads();
            if (nSncfg == 0) {
                write_final_layers(key, o.S, o.so[NLAY]);
                if (tid == 0) {
                    finish_key(kargs(), key, LC_INVALID, LC_CAUSE_NONLIN, evno, peak, probes, (uint64_t)evno + 1);
                    atomicAdd(kargs().stream_bytes, (unsigned long long)sbytes);
                }
                __syncthreads();
                return K_DONE;
            }
            cur ^= 1;
            nScfg = nSncfg;
            peak = nScfg > peak ? (uint32_t)(nScfg < 0xFFFFFFFFull ? nScfg : 0xFFFFFFFFull) : peak;
            pend &= ~(1ull << p);
        }
    }
    __syncthreads();
    write_final_layers(key, cur ? S1 : S0, sh.soff[cur][NLAY]);
    if (tid == 0) {
        finish_key(kargs(), key, LC_VALID, LC_CAUSE_NONE, -1, peak, probes, e - b);
        atomicAdd(kargs().stream_bytes, (unsigned long long)sbytes);
    }
    __syncthreads();
    return K_DONE;
}

__global__ __launch_bounds__(LWG) void k_search_layers(Args a, LayWs w) {
    __shared__ LayShared sh;
    // (the work list and results through kargs(); the walk keeps only the
    // fields it reads per event from the by-value parameter)
    int32_t n;
    {
        KArgs &ka = kargs();
        n = ka.n_in ? min(*ka.n_in, ka.list_cap) : ka.n_order;
        if (n == 0 || batch_refused(ka)) return;  // empty work list / malformed batch
    }
    clear_slots(sh.tab, TS);
    // cooperating blocks: the board is this launch's (one job slot per block)
    const bool coop = LC_T3L_COOP && w.coop && w.coop_slots >= gridDim.x;
    LayWs wl = w;
    if (!coop) wl.coop = nullptr;
    for (;;) {
        if (threadIdx.x == 0) {
            // counted as searching before the ticket: a helper stops only
            // when no block searches, or is about to
            if (coop) atomicAdd(&coop_head(wl)->active, 1u);
            sh.work = atomicAdd(kargs().ticket, 1);
            if (coop && sh.work >= n) atomicSub(&coop_head(wl)->active, 1u);
            if (coop && sh.work < n) atomicAdd(&coop_head(wl)->busy[xcc_id()], 1u);
        }
        __syncthreads();
        const int32_t wi = sh.work;
        __syncthreads();
        if (wi >= n) break;
        const int32_t key = kargs().order[wi];
        const int r = search_key_layers(a, wl, key, sh);
        if (threadIdx.x == 0 && coop) {
            atomicSub(&coop_head(wl)->busy[xcc_id()], 1u);
            atomicSub(&coop_head(wl)->active, 1u);
        }
        if (threadIdx.x == 0 && (r == K_WIDE || r == K_OLD)) {
            KArgs &ka = kargs();
            int32_t *list = r == K_WIDE ? ka.wide : ka.spill, *count = r == K_WIDE ? ka.n_wide : ka.n_spill;
            const int32_t i = atomicAdd(count, 1);
            if (i < ka.list_cap) list[i] = key;
        }
        __syncthreads();
    }
    if (coop) coop_help(sh, wl);
}

}  // namespace

hipError_t launch_t3_layers(const Args &a, const LayWs &w, int grid, hipStream_t s) {
    hipLaunchKernelGGL(k_search_layers, dim3(grid), dim3(LWG), 0, s, a, w);
    return hipGetLastError();
}
// Entries a set array can hold past the budget before the block sees it.
int t3l_slack() { return (int)TS; }
size_t t3l_coop_bytes(int slots) { return COOP_HEAD + (size_t)(slots > 0 ? slots : 1) * COOP_STRIDE; }
size_t t3l_coop_passes_offset() { return offsetof(CoopHead, passes); }

}  // namespace lcd
