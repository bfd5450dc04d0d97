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
#ifdef LC_T3L_CNT
    unsigned long long sc[6];  // whole-table steps (thread 0): insert / scan cycles (I, S'), passes (I, S'), -, inputs
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

// The whole-table form of one step (a layer too large for the fused step, or
// one whose fused merge overflowed): I_{k+1} (if want_i) in P passes into
// `iout` (HBM), doubling P while a pass overflows; then S'_k (if want_s),
// likewise.  Adds the configs to cfg_i / cfg_s and thread 0's probes.
// Returns false when the budget was exceeded (or err).  Uses ct[0]; leaves
// both counter sets zeroed.
__device__ bool step_slow(LayShared &sh, const OkCtx &o, uint32_t sb, uint32_t se, const uint64_t *Ik, uint32_t nk,
                          bool want_i, bool want_s, uint64_t *iout, uint32_t &n_out, uint32_t &pc, uint64_t &cfg_i,
                          uint64_t &cfg_s, uint64_t &probes, uint64_t budget) {
    const uint32_t tid = threadIdx.x;
    StepCtr *c = &sh.ct[0];
    bool ok = true;
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
                                   budget)) { over = true; break; }
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
    for (;;) {
        if (threadIdx.x == 0) sh.work = atomicAdd(kargs().ticket, 1);
        __syncthreads();
        const int32_t wi = sh.work;
        __syncthreads();
        if (wi >= n) break;
        const int32_t key = kargs().order[wi];
        const int r = search_key_layers(a, w, key, sh);
        if (threadIdx.x == 0 && (r == K_WIDE || r == K_OLD)) {
            KArgs &ka = kargs();
            int32_t *list = r == K_WIDE ? ka.wide : ka.spill, *count = r == K_WIDE ? ka.n_wide : ka.n_spill;
            const int32_t i = atomicAdd(count, 1);
            if (i < ka.list_cap) list[i] = key;
        }
        __syncthreads();
    }
}

}  // namespace

hipError_t launch_t3_layers(const Args &a, const LayWs &w, int grid, hipStream_t s) {
    hipLaunchKernelGGL(k_search_layers, dim3(grid), dim3(LWG), 0, s, a, w);
    return hipGetLastError();
}
// Entries a set array can hold past the budget before the block sees it.
int t3l_slack() { return (int)TS; }

}  // namespace lcd
