// device_search.hip -- the JIT linearization search of knossos.linear on gfx950.
//
// Replaces knossos.linear/analysis (:algorithm :linear, etcdemo.clj:118) for
// the cas-register model (etcdemo.clj:117), batched over every independent
// key of a history (independent/checker, etcdemo.clj:115).  Semantics are
// those written out in oracle/linear_ref.py; this file only organises the
// same set computation for the hardware.
//
// Per :ok(p) event a key's config set S becomes
//     S' = { (s, L \ p) : (s, L) in S, p in L }  U  apply_p(I)
// where I is the JIT closure of { (s, L) in S : p not in L } under
// linearizing pending ops other than p.  Configs are packed integers:
//     narrow (u64): state << 56 | L   (L = pending-window slot bits 0..55)
//
// Tiers (each a persistent kernel over a device work list; a key that
// outgrows a tier is re-searched from its first event by the next one, so
// every tier computes exactly the same sets):
//   T1  one wavefront per key, S / S' / I and two open-addressed hash sets in
//       LDS (~20 KB per wave, 8 waves per CU): the common case.
//   T2  the same code with ~6x the LDS (1 wave per CU).
//   T3  (HBM tier, device_hbm.hip) keys beyond T2 or needing > 56 window
//       slots / > 255 register states.
//
// Hash sets: open addressing, linear probing, 64-bit ds_cmpst (LDS) CAS on
// EMPTY; the slot each new config landed in is remembered so the table is
// cleared by the entries it holds, not by sweeping it.  Appends are
// wave-synchronous: ballot + mbcnt give each new config its array position.

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/lincheck.h"
#include "device_search.hpp"
#include "device_common.hpp"

namespace lcd {

// ---------------------------------------------------------------- LDS tiers
template <int CAP_S, int CAP_I>
struct LdsTier {
    static constexpr int HS = 2 * CAP_S;  // hash slots for S'
    static constexpr int HI = 2 * CAP_I;  // hash slots for I
    uint64_t S[2][CAP_S];
    uint64_t I[CAP_I];
    uint64_t hS[HS];
    uint64_t hI[HI];
    uint16_t posS[2][CAP_S];  // hash slot of each S' entry (for clearing)
    uint16_t posI[CAP_I];
    uint32_t desclist[64];
    uint8_t slotlist[64];
};


template <int CAP_S, int CAP_I>
__device__ int search_key_lds(const Args &a, int32_t key, LdsTier<CAP_S, CAP_I> &t) {
    using T = LdsTier<CAP_S, CAP_I>;
    const uint32_t lane = lane_id();
    const uint64_t b = a.ev_off[key], e = a.ev_off[key + 1];
    const uint32_t tb = a.trans_off ? a.trans_off[key] : 0u;
    if (a.key_error && a.key_error[key]) {  // a table-model batch starts here, not in T0
        finish_key(kargs(), key, LC_UNKNOWN, LC_CAUSE_ERROR, -1, 0, 0, 0);
        return K_DONE;
    }
    if (a.key_states && a.key_states[key] > LC_WIDE_MAX_STATES) {
        finish_key(kargs(), key, LC_UNKNOWN, LC_CAUSE_STATES, -1, 1, 0, 0);
        return K_DONE;
    }
    // Too many register states for an 8-bit state field: wide configs.  A
    // wide window is decided per invoke (slot >= 56), not from key_width: a
    // key often ends (budget, failure) long before its widest moment.
    if (a.trans_off && a.key_states && a.key_states[key] > LC_NARROW_MAX_STATES) return K_WIDE;

    // fresh tables for this key
    for (int i = (int)lane; i < T::HS; i += 64) t.hS[i] = EMPTY;
    for (int i = (int)lane; i < T::HI; i += 64) t.hI[i] = EMPTY;
    if (lane == 0) { t.S[0][0] = (uint64_t)a.init_state << 56; t.posS[0][0] = 0xFFFF; }
    __syncthreads();

    int cur = 0;
    uint32_t nS = 1, nSprev_hash = 0;  // entries of S still present in hS (from its build)
    uint64_t pending = 0;
    uint32_t my_desc = 0;
    uint32_t peak = 1;
    uint64_t probes = 0;
    int verdict = LC_VALID, cause = LC_CAUSE_NONE;
    int32_t fev = -1;
    uint32_t nI_last = 0;

    for (uint64_t base = b; base < e; base += 64) {
        const uint32_t cnt = (uint32_t)((e - base) < 64 ? (e - base) : 64);
        const uint32_t ev = lane < cnt ? a.events[base + lane] : 0u;
        const uint32_t dsc = (lane < cnt && !(ev & LC_EV_OK_BIT)) ? a.trans[tb + LC_EV_TRANS(ev)] : 0u;
        for (uint32_t i = 0; i < cnt; ++i) {
            const uint32_t evi = __builtin_amdgcn_readlane(ev, i);
            const uint32_t slot = LC_EV_SLOT(evi);
            if (!(evi & LC_EV_OK_BIT)) {  // :invoke
                if (slot >= LC_NARROW_MAX_SLOTS) return K_WIDE;
                const uint32_t d = __builtin_amdgcn_readlane(dsc, i);
                if (lane == slot) my_desc = d;
                pending |= 1ull << slot;
                continue;
            }
            // ---- :ok of the op in `slot` ----
            const uint32_t p = slot;
            const uint64_t pbit = 1ull << p;
            const uint32_t dp = __builtin_amdgcn_readlane(my_desc, p);
            uint64_t *S = t.S[cur];
            uint64_t *Sn = t.S[cur ^ 1];
            uint16_t *posSn = t.posS[cur ^ 1];
            // clear what the previous event left in the hash sets
            for (uint32_t j = lane; j < nI_last; j += 64) t.hI[t.posI[j]] = EMPTY;
            for (uint32_t j = lane; j < nSprev_hash; j += 64) {
                uint16_t ps = t.posS[cur][j];
                if (ps != 0xFFFF) t.hS[ps] = EMPTY;
            }
            __syncthreads();
            uint32_t nI = 0, nSn = 0;
            // -- partition S: p already linearized -> S' (p returns); else seed I
            for (uint32_t j = 0; j < nS; j += 64) {
                const uint32_t idx = j + lane;
                const bool act = idx < nS;
                const uint64_t c = act ? S[idx] : 0;
                const bool hasp = act && (c & pbit);
                const bool toI = act && !hasp;
                uint32_t posa = 0, posb = 0;
                const bool ns = lds_insert(t.hS, T::HS - 1, c & ~pbit, hasp, posa);
                const bool ni = lds_insert(t.hI, T::HI - 1, c, toI, posb);
                const uint64_t ms = __ballot(ns), mi = __ballot(ni);
                if (ns) { uint32_t r = nSn + rank_of(ms); Sn[r] = c & ~pbit; posSn[r] = (uint16_t)posa; }
                if (ni) { uint32_t r = nI + rank_of(mi); t.I[r] = c; t.posI[r] = (uint16_t)posb; }
                nSn += (uint32_t)__popcll(ms);
                nI += (uint32_t)__popcll(mi);
            }
            probes += nS;
            __syncthreads();
            // -- JIT closure over the other pending ops
            const uint64_t cand = pending & ~pbit;
            const uint32_t nc = (uint32_t)__popcll(cand);
            bool overflow = false;
            if (nc) {
                if (lane < 64 && (cand >> lane) & 1ull) {
                    uint32_t r = (uint32_t)__popcll(cand & ((1ull << lane) - 1ull));
                    t.slotlist[r] = (uint8_t)lane;
                    t.desclist[r] = my_desc;
                }
                __syncthreads();
                uint32_t head = 0;
                while (head < nI && !overflow) {
                    const uint32_t end = nI;
                    const uint32_t total = (end - head) * nc;
                    for (uint32_t it = 0; it < total; it += 64) {
                        const uint32_t item = it + lane;
                        bool act = item < total;
                        const uint32_t ci = head + (act ? item / nc : 0);
                        const uint32_t k = act ? item % nc : 0;
                        const uint64_t c = t.I[ci];
                        const uint32_t q = t.slotlist[k];
                        const uint32_t dq = t.desclist[k];
                        uint32_t s2 = 0;
                        act = act && !((c >> q) & 1ull) && step(a.table, (uint32_t)(c >> 56), dq, s2);
                        const uint64_t c2 = ((uint64_t)s2 << 56) | (c & LMASK) | (1ull << q);
                        probes += (uint64_t)__popcll(__ballot(act));
                        uint32_t pos = 0;
                        const bool nw = lds_insert(t.hI, T::HI - 1, c2, act, pos);
                        const uint64_t mn = __ballot(nw);
                        if (nw) {
                            uint32_t r = nI + rank_of(mn);
                            if (r < CAP_I) { t.I[r] = c2; t.posI[r] = (uint16_t)pos; }
                        }
                        nI += (uint32_t)__popcll(mn);
                        if (nI > a.budget) { verdict = LC_UNKNOWN; cause = LC_CAUSE_BUDGET; overflow = true; break; }
                        if (nI > CAP_I) { overflow = true; break; }
                    }
                    __syncthreads();
                    head = end;
                }
            }
            if (overflow) {
                if (verdict == LC_UNKNOWN) {
                    fev = (int32_t)(base + i - b);
                    write_final_narrow(kargs(), key, S, nS);
                    finish_key(kargs(), key, verdict, cause, fev, peak, probes, base + i - b);
                    return K_DONE;
                }
                return K_SPILL;
            }
            // -- apply p to every config of the closure
            for (uint32_t j = 0; j < nI; j += 64) {
                const uint32_t idx = j + lane;
                const uint64_t c = idx < nI ? t.I[idx] : 0;
                uint32_t s2 = 0;
                const bool act = idx < nI && step(a.table, (uint32_t)(c >> 56), dp, s2);
                const uint64_t c2 = ((uint64_t)s2 << 56) | (c & LMASK);
                probes += (uint64_t)__popcll(__ballot(act));
                uint32_t pos = 0;
                const bool nw = lds_insert(t.hS, T::HS - 1, c2, act, pos);
                const uint64_t mn = __ballot(nw);
                if (nw) {
                    uint32_t r = nSn + rank_of(mn);
                    if (r < CAP_S) { Sn[r] = c2; posSn[r] = (uint16_t)pos; }
                }
                nSn += (uint32_t)__popcll(mn);
                if (nSn > a.budget || nSn > CAP_S) break;
            }
            __syncthreads();
            nI_last = nI < CAP_I ? nI : CAP_I;
            if (nSn == 0) {
                verdict = LC_INVALID; cause = LC_CAUSE_NONLIN; fev = (int32_t)(base + i - b);
                write_final_narrow(kargs(), key, S, nS);
                finish_key(kargs(), key, verdict, cause, fev, peak, probes, base + i + 1 - b);
                return K_DONE;
            }
            if (nSn > a.budget) {
                verdict = LC_UNKNOWN; cause = LC_CAUSE_BUDGET; fev = (int32_t)(base + i - b);
                write_final_narrow(kargs(), key, S, nS);
                finish_key(kargs(), key, verdict, cause, fev, peak, probes, base + i - b);
                return K_DONE;
            }
            if (nSn > CAP_S) return K_SPILL;
            // S' was deduplicated in hS: its entries stay there until the next
            // event clears them through posS.
            nSprev_hash = nSn;
            cur ^= 1;
            nS = nSn;
            peak = nS > peak ? nS : peak;
            pending &= ~pbit;
        }
    }
    write_final_narrow(kargs(), key, t.S[cur], nS);
    finish_key(kargs(), key, LC_VALID, LC_CAUSE_NONE, -1, peak, probes, e - b);
    return K_DONE;
}

template <int CAP_S, int CAP_I>
__global__ __launch_bounds__(64) void k_search_lds(Args a) {
    __shared__ LdsTier<CAP_S, CAP_I> t;
    // (the work list and results through kargs(): device_common.hpp)
    int32_t n;
    {
        KArgs &ka = kargs();
        n = ka.n_in ? min(*ka.n_in, ka.list_cap) : ka.n_order;
        if (n == 0 || batch_refused(ka)) return;  // empty work list / malformed batch: no ticket traffic
    }
    for (int32_t w = next_work(kargs()); w < n; w = next_work(kargs())) {
        const int32_t key = kargs().order[w];
        const int r = search_key_lds<CAP_S, CAP_I>(a, key, t);
        if (r == K_SPILL || r == K_WIDE) {
            KArgs &ka = kargs();
            if (r == K_SPILL) push_list(ka.spill, ka.n_spill, key, ka.list_cap);
            else push_list(ka.wide, ka.n_wide, key, ka.list_cap);
        }
        __syncthreads();
    }
}

// Tier geometry (LDS per wave): T1 ~22 KB -> 7 waves/CU; T2 ~140 KB -> 1 wave/CU.
constexpr int T1_S = 256, T1_I = 512;
constexpr int T2_S = 1024, T2_I = 4096;

size_t lds_bytes_t1() { return sizeof(LdsTier<T1_S, T1_I>); }
size_t lds_bytes_t2() { return sizeof(LdsTier<T2_S, T2_I>); }

hipError_t launch_t1(const Args &a, int grid, hipStream_t s) {
    hipLaunchKernelGGL((k_search_lds<T1_S, T1_I>), dim3(grid), dim3(64), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_t2(const Args &a, int grid, hipStream_t s) {
    hipLaunchKernelGGL((k_search_lds<T2_S, T2_I>), dim3(grid), dim3(64), 0, s, a);
    return hipGetLastError();
}

}  // namespace lcd
