// device_lattice.hip -- T0: the JIT linearization search with the config set
// held as a subset lattice in registers (one wavefront per key).
//
// Same sets as every other tier (semantics: oracle/linear_ref.py).  The
// representation exploits two facts of the packed form:
//   * a config is (register state, set L of linearized pending ops), and ops
//     are named by their pending-window slot (lowest free slot at invoke,
//     lc_pack), so L is a subset of {0 .. width-1} with width = the key's
//     largest concurrency (<= 10 for the demo's 10 client threads);
//   * the register has few states (6 for the demo's values 0..4 + nil).
// So S is stored as W[L] = bitmask of states s with (s, L) in S, one 32-bit
// mask per subset L, subset index = lane + 64 * register.  A wave's 64 lanes
// x R registers cover 2^(6 + log2 R) subsets (R = 16: width 10).
//
// Per :ok(p) event:
//   Ret[L]  = W[L u {p}]              (configs that already linearized p)
//   I[L]    = W[L]          for p not in L; then the JIT closure
//   I[L u {q}] |= T_q(I[L]) for every pending q != p, to a fixpoint,
//   S'[L]   = Ret[L] | T_p(I[L])
// where T_q maps a state mask through op q's cas-register step (read a: keep
// bit a; write b: any -> {b}; cas a->b: bit a -> {b}).  "L u {q}" is the
// lane/register whose index differs in bit q: a DPP / ds_swizzle / bpermute
// exchange for q < 6, a register pair for q >= 6.  Set sizes (for the budget,
// the peak and the probe count) are popcounts reduced over the wave, so every
// number reported equals the oracle's.
//
// Keys outside T0's reach (width > 10, > 32 register states, or a caller
// batch whose slots exceed its key_width) go to the hash-set tiers.

#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "../../include/lincheck.h"
#include "device_common.hpp"
#include "device_search.hpp"

extern "C" __device__ uint32_t __ockl_wfred_add_u32(uint32_t);

namespace lcd {

constexpr int T0_RMAX = 4;        // lattice registers per lane: n <= 8 pending ops
constexpr int T0_RMEM = 16;       // workspace lattice (global memory): n <= 10
constexpr uint32_t T0_MAX_WIDTH = 10;  // = 6 + log2(T0_RMEM)
constexpr uint32_t T0_MAX_STATES = 32;

// Mask of states reachable from mask M through op d (0 if illegal for all).
__device__ __forceinline__ uint32_t tmask(uint32_t M, uint32_t d) {
    const uint32_t f = d & 3u, a = (d >> 2) & 0x7FFFu, b = d >> 17;
    const uint32_t abit = a < 32u ? (M >> a) & 1u : 0u;
    if (f == LC_T_READ_ANY) return M;
    if (f == LC_T_READ) return abit << (a & 31u);
    if (f == LC_T_WRITE) return M ? (1u << b) : 0u;
    return abit ? (1u << b) : 0u;  // CAS
}

// Number of configs of mask M for which op d is legal (probe count).
__device__ __forceinline__ uint32_t legal_cnt(uint32_t M, uint32_t d) {
    const uint32_t f = d & 3u, a = (d >> 2) & 0x7FFFu;
    if (f == LC_T_READ_ANY || f == LC_T_WRITE) return (uint32_t)__popc(M);
    return a < 32u ? (M >> a) & 1u : 0u;
}

// Branch-free form of an op's state transfer: T(M) = (M & pass) | (M & keep ? set : 0)
//   read-any: pass = all         read a: pass = {a}
//   write b:  keep = all, set = {b}      cas a->b: keep = {a}, set = {b}
// and the number of configs of M where the op is legal is popc(M & (pass | keep)).
struct Xfer { uint32_t pass, keep, set; };

__device__ __forceinline__ Xfer xfer_of(uint32_t d) {  // branch-free (uniform d: scalar selects)
    const uint32_t f = d & 3u, a = (d >> 2) & 0x7FFFu, b = d >> 17;
    const uint32_t abit = a < 32u ? 1u << (a & 31u) : 0u, bbit = b < 32u ? 1u << (b & 31u) : 0u;
    Xfer x;
    x.pass = f == LC_T_READ_ANY ? 0xFFFFFFFFu : (f == LC_T_READ ? abit : 0u);
    x.keep = f == LC_T_WRITE ? 0xFFFFFFFFu : (f == LC_T_CAS ? abit : 0u);
    x.set = f >= LC_T_WRITE ? bbit : 0u;
    return x;
}

__device__ __forceinline__ uint32_t xapply(uint32_t M, uint32_t pass, uint32_t keep, uint32_t set) {
    return (M & pass) | ((M & keep) ? set : 0u);
}

// x from lane (lane ^ 2^Q), Q < 6, in VALU only (DPP row shifts, gfx950
// permlane swaps): no LDS round trip.
template <int Q>
__device__ __forceinline__ uint32_t xv(uint32_t x, uint32_t lane) {
    if constexpr (Q == 0) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);
    else if constexpr (Q == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);
    else if constexpr (Q == 2) {
        const uint32_t up = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x104, 0xF, 0xF, true);  // row_shl:4
        const uint32_t dn = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x114, 0xF, 0xF, true);  // row_shr:4
        return (lane & 4u) ? dn : up;
    } else if constexpr (Q == 3) {
        const uint32_t up = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x108, 0xF, 0xF, true);  // row_shl:8
        const uint32_t dn = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x118, 0xF, 0xF, true);  // row_shr:8
        return (lane & 8u) ? dn : up;
    } else if constexpr (Q == 4) {
        const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        return (lane & 16u) ? r[0] : r[1];
    } else {
        const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return (lane & 32u) ? r[0] : r[1];
    }
}

// x from lane (lane ^ 2^Q), Q < 6.
template <int Q>
__device__ __forceinline__ uint32_t xchg(uint32_t x) {
    if constexpr (Q == 0) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);  // quad_perm 1,0,3,2
    else if constexpr (Q == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);  // quad_perm 2,3,0,1
    else if constexpr (Q == 2) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x101F);  // xor 4
    else if constexpr (Q == 3) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x201F);  // xor 8
    else if constexpr (Q == 4) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x401F);  // xor 16
    else return (uint32_t)__shfl_xor((int)x, 32);
}

using Lat = uint32_t[T0_RMAX];

// P[k] = X[k's partner along subset bit `bit`] (run-time bit; lanes active).
template <int RL>
__device__ __forceinline__ void xchg_rt(const Lat &X, Lat &P, uint32_t bit) {
    if (bit < 6) {
        const int m = 1 << bit;
#pragma unroll
        for (int k = 0; k < RL; ++k) P[k] = (uint32_t)__shfl_xor((int)X[k], m);
        return;
    }
    const uint32_t r = bit - 6;
#pragma unroll
    for (int k = 0; k < RL; ++k) {
        uint32_t v = X[k];
        if constexpr (RL > 1) v = r == 0 ? X[k ^ 1] : v;
        if constexpr (RL > 2) v = r == 1 ? X[k ^ 2] : v;
        if constexpr (RL > 4) v = r == 2 ? X[k ^ 4] : v;
        if constexpr (RL > 8) v = r == 3 ? X[k ^ 8] : v;
        P[k] = v;
    }
}

__device__ __forceinline__ bool idx_has(uint32_t lane, int k, uint32_t q) {
    return q < 6 ? ((lane >> q) & 1u) : (((uint32_t)k >> (q - 6)) & 1u);
}

template <int RL>
constexpr int lat_bits() { return RL == 1 ? 6 : RL == 2 ? 7 : RL == 4 ? 8 : RL == 8 ? 9 : 10; }

// One :ok(p) event on a lattice of RL registers (n <= 6 + log2 RL pending
// ops).  Every subset bit position is applied in every sweep, branch-free:
// positions that are not candidates carry zero transfer masks.  Lane bits
// move through VALU exchanges (xv), register bits through register pairs.
// W = S on entry, S' (relocated so index n-1 is free) on a normal return.
// Returns 0 normal, 1 invalid, 2 budget exceeded.
template <int RL>
__device__ __forceinline__ int ok_event_r(Lat &W, uint32_t p, uint32_t n, uint32_t pass_v, uint32_t keep_v,
                                          uint32_t set_v, uint32_t lane, uint64_t budget, uint32_t &probes,
                                          uint32_t &nSn_out, bool want_size) {
    constexpr int NB = lat_bits<RL>();
    const uint32_t cand = ((1u << n) - 1u) & ~(1u << p);
    uint32_t ps[NB], kp[NB], st[NB];
#pragma unroll
    for (int q = 0; q < NB; ++q) {
        const bool on = (cand >> q) & 1u;
        ps[q] = on ? __builtin_amdgcn_readlane(pass_v, q) : 0u;
        kp[q] = on ? __builtin_amdgcn_readlane(keep_v, q) : 0u;
        st[q] = on ? __builtin_amdgcn_readlane(set_v, q) : 0u;
    }
    const uint32_t pp = __builtin_amdgcn_readlane(pass_v, p), pk = __builtin_amdgcn_readlane(keep_v, p),
                   pt = __builtin_amdgcn_readlane(set_v, p);
    Lat Ret, I;  // with W: the only three lattice arrays (register budget)
#pragma unroll
    for (int k = 0; k < RL; ++k) probes += (uint32_t)__popc(W[k]);
    xchg_rt<RL>(W, Ret, p);
#pragma unroll
    for (int k = 0; k < RL; ++k) {
        const bool hp = idx_has(lane, k, p);
        Ret[k] = hp ? 0u : Ret[k];
        I[k] = hp ? 0u : W[k];
    }
    for (;;) {  // Jacobi sweeps to the fixpoint; W is scratch from here on
        bool ch = false;
#pragma unroll
        for (int k = 0; k < RL; ++k) {
            uint32_t acc = I[k];
#define LC_LANEBIT(Q)                                                                  \
            {                                                                          \
                const uint32_t x = xv<Q>(I[k], lane);                                  \
                acc |= ((lane >> Q) & 1u) ? xapply(x, ps[Q], kp[Q], st[Q]) : 0u;      \
            }
            LC_LANEBIT(0) LC_LANEBIT(1) LC_LANEBIT(2) LC_LANEBIT(3) LC_LANEBIT(4) LC_LANEBIT(5)
#undef LC_LANEBIT
#pragma unroll
            for (int q = 6; q < NB; ++q)
                if ((k >> (q - 6)) & 1) acc |= xapply(I[k ^ (1 << (q - 6))], ps[q], kp[q], st[q]);
            W[k] = acc;
        }
#pragma unroll
        for (int k = 0; k < RL; ++k) { ch |= W[k] != I[k]; I[k] = W[k]; }
        if (!__any(ch)) break;
    }
    uint32_t cI = 0, cS = 0;
#pragma unroll
    for (int k = 0; k < RL; ++k) {
#pragma unroll
        for (int q = 0; q < NB; ++q)
            if (!idx_has(lane, k, (uint32_t)q)) probes += (uint32_t)__popc(I[k] & (ps[q] | kp[q]));
        Ret[k] |= xapply(I[k], pp, pk, pt);
        probes += (uint32_t)__popc(I[k] & (pp | pk));
        cI += (uint32_t)__popc(I[k]);
        cS += (uint32_t)__popc(Ret[k]);
    }
    // The lattice holds at most RL*64*32 configs: below that budget sizes
    // decide :unknown; above it only emptiness matters (one ballot), and the
    // exact |S'| is reduced only when a peak was asked for.
    if (budget < (uint64_t)RL * 64u * 32u) {
        const uint32_t nI = __ockl_wfred_add_u32(cI);
        if (nI > budget) return 2;
    }
    if (!__any(cS != 0u)) { nSn_out = 0; return 1; }
    if (budget < (uint64_t)RL * 64u * 32u || want_size) {
        const uint32_t nSn = __ockl_wfred_add_u32(cS);
        nSn_out = nSn;
        if (nSn > budget) return 2;
    }
    const uint32_t last = n - 1;
    if (p == last) {
#pragma unroll
        for (int k = 0; k < RL; ++k) W[k] = Ret[k];
        return 0;
    }
    // the op at index `last` moves to index p: S'[L] for L with p comes from
    // L ^ {p, last}; no config keeps bit `last`
    xchg_rt<RL>(Ret, W, p);
    xchg_rt<RL>(W, I, last);
#pragma unroll
    for (int k = 0; k < RL; ++k) {
        const bool hp = idx_has(lane, k, p), hl = idx_has(lane, k, last);
        W[k] = hl ? 0u : (hp ? I[k] : Ret[k]);
    }
    return 0;
}

// One :ok(p) event when at most 6 ops are pending: the whole lattice is one
// register, every subset bit is a lane bit, and each closure sweep applies
// all six bit positions branch-free (non-candidates carry zero masks).
__device__ __forceinline__ int ok_event_1(uint32_t &W, uint32_t p, uint32_t n, uint32_t pass_v, uint32_t keep_v,
                                          uint32_t set_v, uint32_t lane, uint64_t budget, uint32_t &probes,
                                          uint32_t &nSn_out, bool want_size) {
    const uint32_t cand = ((1u << n) - 1u) & ~(1u << p);
    uint32_t ps[6], kp[6], st[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) {
        const bool on = (cand >> q) & 1u;
        ps[q] = on ? __builtin_amdgcn_readlane(pass_v, q) : 0u;
        kp[q] = on ? __builtin_amdgcn_readlane(keep_v, q) : 0u;
        st[q] = on ? __builtin_amdgcn_readlane(set_v, q) : 0u;
    }
    const uint32_t pp = __builtin_amdgcn_readlane(pass_v, p), pk = __builtin_amdgcn_readlane(keep_v, p),
                   pt = __builtin_amdgcn_readlane(set_v, p);
    probes += (uint32_t)__popc(W);
    const bool hp = (lane >> p) & 1u;
    const uint32_t wp = (uint32_t)__shfl_xor((int)W, 1 << p);
    uint32_t Ret = hp ? 0u : wp;
    uint32_t I = hp ? 0u : W;
    // Jacobi sweeps: the six bit positions read the same I, so their lane
    // exchanges are independent (ILP); the exchange runs with every lane
    // active, only its result is masked.  Repeat until nothing new.
    for (;;) {
#define LC_EXPAND(Q) \
        const uint32_t x##Q = xv<Q>(I, lane); \
        const uint32_t t##Q = ((lane >> Q) & 1u) ? xapply(x##Q, ps[Q], kp[Q], st[Q]) : 0u;
        LC_EXPAND(0) LC_EXPAND(1) LC_EXPAND(2) LC_EXPAND(3) LC_EXPAND(4) LC_EXPAND(5)
#undef LC_EXPAND
        const uint32_t nv = I | t0 | t1 | t2 | t3 | t4 | t5;
        const bool ch = nv != I;
        I = nv;
        if (!__any(ch)) break;
    }
#pragma unroll
    for (int q = 0; q < 6; ++q)
        if (!((lane >> q) & 1u)) probes += (uint32_t)__popc(I & (ps[q] | kp[q]));
    Ret |= xapply(I, pp, pk, pt);
    probes += (uint32_t)__popc(I & (pp | pk));
    // One register holds at most 64 x 32 configs: with a larger budget only
    // emptiness matters (a ballot); exact sizes only when asked for (peak).
    if (budget < 64u * 32u) {
        const uint32_t nI = __ockl_wfred_add_u32((uint32_t)__popc(I));
        if (nI > budget) return 2;
    }
    if (!__any(Ret != 0u)) { nSn_out = 0; return 1; }
    if (budget < 64u * 32u || want_size) {
        const uint32_t nSn = __ockl_wfred_add_u32((uint32_t)__popc(Ret));
        nSn_out = nSn;
        if (nSn > budget) return 2;
    }
    const uint32_t last = n - 1;
    if (p == last) { W = Ret; return 0; }
    // op at index `last` moves to index p
    const uint32_t r2 = (uint32_t)__shfl_xor((int)Ret, (1 << p) | (1 << last));
    const bool hl = (lane >> last) & 1u;
    W = hl ? 0u : (hp ? r2 : Ret);
    return 0;
}

// Lattice of a key with 9 or 10 ops pending: 16 x 64 words per array in a
// per-block global workspace, index k * 64 + lane.  Every lane reads and
// writes only its own column (register-bit partners are in the same lane;
// lane-bit partners are exchanged in registers), so no cross-lane memory
// ordering is involved.  Such events are rare (< 0.2 % of C2's); keeping
// them out of registers keeps T0 at 4 waves per SIMD.
struct LatMem {
    uint32_t *W, *R, *I;
};

template <int RL>
__device__ __forceinline__ int ok_event_mem(const LatMem &m, uint32_t p, uint32_t n, uint32_t pass_v,
                                            uint32_t keep_v, uint32_t set_v, uint32_t lane, uint64_t budget,
                                            uint32_t &probes, uint32_t &nSn_out, bool want_size) {
    constexpr int NB = lat_bits<RL>();
    const uint32_t cand = ((1u << n) - 1u) & ~(1u << p);
    // transfer of candidate q: lane q of pass_v/keep_v/set_v, read at use
    // (not hoisted: 3 x NB scalars would spill SGPRs into the VGPR budget)
    const uint32_t cpass = pass_v & (((cand >> lane) & 1u) ? ~0u : 0u);
    const uint32_t ckeep = keep_v & (((cand >> lane) & 1u) ? ~0u : 0u);
#define PS(Q) __builtin_amdgcn_readlane(cpass, Q)
#define KP(Q) __builtin_amdgcn_readlane(ckeep, Q)
#define ST(Q) __builtin_amdgcn_readlane(set_v, Q)
    const uint32_t pp = __builtin_amdgcn_readlane(pass_v, p), pk = __builtin_amdgcn_readlane(keep_v, p),
                   pt = __builtin_amdgcn_readlane(set_v, p);
    const uint32_t plm = p < 6 ? 1u << p : 0u, prm = p >= 6 ? 1u << (p - 6) : 0u;
#pragma unroll 1
    for (int k = 0; k < RL; ++k) {
        const uint32_t w = m.W[k * 64 + lane];
        probes += (uint32_t)__popc(w);
        const uint32_t src = (uint32_t)__shfl_xor((int)m.W[(k ^ prm) * 64 + lane], (int)plm);
        const bool hp = (lane & plm) || ((uint32_t)k & prm);
        m.R[k * 64 + lane] = hp ? 0u : src;
        m.I[k * 64 + lane] = hp ? 0u : w;
    }
    for (;;) {  // sweeps in place (monotone: any order reaches the fixpoint)
        bool ch = false;
    #pragma unroll 1
    for (int k = 0; k < RL; ++k) {
            const uint32_t x = m.I[k * 64 + lane];
            uint32_t acc = x;
#define LC_LANEBIT(Q)                                                                  \
            {                                                                          \
                const uint32_t y = xv<Q>(x, lane);                                     \
                acc |= ((lane >> Q) & 1u) ? xapply(y, PS(Q), KP(Q), ST(Q)) : 0u;      \
            }
            LC_LANEBIT(0) LC_LANEBIT(1) LC_LANEBIT(2) LC_LANEBIT(3) LC_LANEBIT(4) LC_LANEBIT(5)
#undef LC_LANEBIT
#pragma unroll
            for (int q = 6; q < NB; ++q)
                if ((k >> (q - 6)) & 1) acc |= xapply(m.I[(k ^ (1 << (q - 6))) * 64 + lane], PS(q), KP(q), ST(q));
            if (acc != x) { m.I[k * 64 + lane] = acc; ch = true; }
        }
        if (!__any(ch)) break;
    }
    uint32_t cI = 0, cS = 0;
#pragma unroll 1
    for (int k = 0; k < RL; ++k) {
        const uint32_t x = m.I[k * 64 + lane];
#pragma unroll
        for (int q = 0; q < NB; ++q)
            if (!idx_has(lane, k, (uint32_t)q)) probes += (uint32_t)__popc(x & (PS(q) | KP(q)));
        const uint32_t r = m.R[k * 64 + lane] | xapply(x, pp, pk, pt);
        probes += (uint32_t)__popc(x & (pp | pk));
        m.R[k * 64 + lane] = r;
        cI += (uint32_t)__popc(x);
        cS += (uint32_t)__popc(r);
    }
    if (budget < (uint64_t)RL * 64u * 32u) {
        const uint32_t nI = __ockl_wfred_add_u32(cI);
        if (nI > budget) return 2;
    }
    if (!__any(cS != 0u)) { nSn_out = 0; return 1; }
    if (budget < (uint64_t)RL * 64u * 32u || want_size) {
        const uint32_t nSn = __ockl_wfred_add_u32(cS);
        nSn_out = nSn;
        if (nSn > budget) return 2;
    }
#undef PS
#undef KP
#undef ST
    // relocation: the op at index `last` moves to index p
    const uint32_t last = n - 1;
    const uint32_t llm = last < 6 ? 1u << last : 0u, lrm = last >= 6 ? 1u << (last - 6) : 0u;
#pragma unroll 1
    for (int k = 0; k < RL; ++k) {
        const uint32_t r = m.R[k * 64 + lane];
        const uint32_t src = (uint32_t)__shfl_xor((int)m.R[(k ^ (prm | lrm)) * 64 + lane], (int)(plm | llm));
        const bool hp = (lane & plm) || ((uint32_t)k & prm);
        const bool hl = (lane & llm) || ((uint32_t)k & lrm);
        m.W[k * 64 + lane] = p == last ? r : (hl ? 0u : (hp ? src : r));
    }
    return 0;
}

// First max_final configs of the lattice held in m.W (register lattices are
// stored there first), in (register, lane, state) order, with dense op
// indices translated back to window slots (slot_v: lane j holds the slot of
// dense index j).
__device__ __forceinline__ void write_final_mem(const Args &a, int32_t key, const LatMem &m, uint32_t lane,
                                                uint32_t slot_v, uint32_t n) {
    if (!a.final_cfg) return;
    const uint32_t mf = (uint32_t)a.max_final;
    const int live = n <= 6 ? 1 : (1 << (n - 6));
    uint32_t base = 0;
#pragma unroll 1
    for (int k = 0; k < live; ++k) {
        const uint32_t w = m.W[k * 64 + lane];
        const uint32_t c = (uint32_t)__popc(w);
        uint32_t x = c;  // inclusive prefix over lanes
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o);
            if (lane >= (uint32_t)o) x += y;
        }
        const uint32_t tot = __shfl(x, 63);
        uint32_t r = base + x - c;
        uint64_t smask = 0;
        const uint32_t L = lane + 64u * (uint32_t)k;
        for (uint32_t j = 0; j < n; ++j) {
            const uint32_t sj = __builtin_amdgcn_readlane(slot_v, j);
            if ((L >> j) & 1u) smask |= 1ull << sj;
        }
        uint32_t mm = w;
        while (mm && r < mf) {
            const uint32_t st = (uint32_t)__ffs(mm) - 1;
            mm &= mm - 1;
            a.final_cfg[((size_t)key * a.max_final + r) * 2 + 0] = smask;
            a.final_cfg[((size_t)key * a.max_final + r) * 2 + 1] = (uint64_t)st << 48;
            ++r;
        }
        base += tot;
    }
    if (lane == 0 && a.n_final) a.n_final[key] = base < mf ? base : mf;
}

// The lattice is indexed by DENSE op indices 0..n-1 (n = ops pending), not by
// window slots: an invoke appends index n; when the op at index j returns, the
// op at index n-1 takes index j (its configs move from bit n-1 to bit j, a
// two-bit exchange).  So the lattice spans 2^n subsets, n = pending count.
template <int RMAX>
__device__ __forceinline__ int lattice_key(const Args &a, int32_t key) {
    const uint32_t lane = lane_id();
    const LatMem m{a.lat_ws + (size_t)blockIdx.x * (3 * T0_RMEM * 64),
                   a.lat_ws + (size_t)blockIdx.x * (3 * T0_RMEM * 64) + T0_RMEM * 64,
                   a.lat_ws + (size_t)blockIdx.x * (3 * T0_RMEM * 64) + 2 * T0_RMEM * 64};
    bool in_mem = false;  // lattice lives in m.W (9 or 10 ops pending)
    const uint64_t b = a.ev_off[key], e = a.ev_off[key + 1];
    const uint32_t tb = a.trans_off ? a.trans_off[key] : 0u;
    if (a.key_states && a.key_states[key] > LC_WIDE_MAX_STATES) {
        finish_key(a, key, LC_UNKNOWN, LC_CAUSE_STATES, -1, 1, 0, 0);
        return K_DONE;
    }
    const uint32_t nstates = a.trans_off ? (a.key_states ? a.key_states[key] : 0xFFFFu) : a.shared_states;
    const uint32_t width = a.key_width ? a.key_width[key] : 0xFFu;  // = max ops pending at once
    if (nstates > T0_MAX_STATES || width > T0_MAX_WIDTH || a.init_state >= T0_MAX_STATES) return K_SPILL;
    const uint64_t budget = a.budget;
    const int dbg = a.debug_mode;  // 0 in every real run (ablation builds only)
    const bool want_peak = a.peak != nullptr;

    Lat W;
#pragma unroll
    for (int k = 0; k < T0_RMAX; ++k) W[k] = 0;
    if (lane == 0) W[0] = 1u << a.init_state;
    uint32_t desc_v = 0;   // lane j: descriptor of the op at dense index j
    uint32_t pass_v = 0, keep_v = 0, set_v = 0;  // lane j: its Xfer masks
    uint32_t slot_v = 0;   // lane j: window slot of the op at dense index j
    uint32_t dense_v = 0;  // lane s: dense index of the op in window slot s
    uint32_t n = 0;        // ops pending
    uint32_t peak = 1, probes = 0;

    // events arrive 64 at a time, one per lane; the next chunk's words and
    // descriptors are loaded while this chunk is searched
    uint32_t ev_next = b + lane < e ? a.events[b + lane] : 0u;
    for (uint64_t base = b; base < e; base += 64) {
        const uint32_t cnt = (uint32_t)((e - base) < 64 ? (e - base) : 64);
        const uint32_t ev = ev_next;
        const uint32_t dsc = (lane < cnt && !(ev & LC_EV_OK_BIT)) ? a.trans[tb + LC_EV_TRANS(ev)] : 0u;
        ev_next = base + 64 + lane < e ? a.events[base + 64 + lane] : 0u;
        for (uint32_t i = 0; i < cnt; ++i) {
            const uint32_t evi = __builtin_amdgcn_readlane(ev, i);
            const uint32_t slot = LC_EV_SLOT(evi);
            if (!(evi & LC_EV_OK_BIT)) {
                if (n >= T0_MAX_WIDTH || slot >= 64) return K_SPILL;
                if (n == 8) {  // 9 pending: move the lattice to the workspace
#pragma unroll
                    for (int k = 0; k < T0_RMEM; ++k) m.W[k * 64 + lane] = k < T0_RMAX ? W[k < T0_RMAX ? k : 0] : 0u;
                    in_mem = true;
                }
                const uint32_t d = __builtin_amdgcn_readlane(dsc, i);
                const Xfer x = xfer_of(d);
                if (lane == n) { desc_v = d; slot_v = slot; pass_v = x.pass; keep_v = x.keep; set_v = x.set; }
                if (lane == slot) dense_v = n;
                ++n;
                continue;
            }
            const uint32_t p = __builtin_amdgcn_readlane(dense_v, slot);
            uint32_t nSn = 0;
            int r = 0;
            if (dbg == 1) {  // ablation: bookkeeping only
                const uint32_t last = n - 1;
                const uint32_t d_last = __builtin_amdgcn_readlane(desc_v, last);
                const uint32_t s_last = __builtin_amdgcn_readlane(slot_v, last);
                if (lane == p) { desc_v = d_last; slot_v = s_last; }
                if (lane == s_last) dense_v = p;
                --n;
                continue;
            }
            if (n <= 6) r = ok_event_1(W[0], p, n, pass_v, keep_v, set_v, lane, budget, probes, nSn, want_peak);
            else if (n == 7) r = ok_event_r<2>(W, p, n, pass_v, keep_v, set_v, lane, budget, probes, nSn, want_peak);
            else if (n == 8) r = ok_event_r<4>(W, p, n, pass_v, keep_v, set_v, lane, budget, probes, nSn, want_peak);
            else if (n == 9) r = ok_event_mem<8>(m, p, n, pass_v, keep_v, set_v, lane, budget, probes, nSn, want_peak);
            else r = ok_event_mem<16>(m, p, n, pass_v, keep_v, set_v, lane, budget, probes, nSn, want_peak);
            if (r) {
                const int32_t evno = (int32_t)(base + i - b);
                if (!in_mem) {
#pragma unroll
                    for (int k = 0; k < T0_RMAX; ++k) m.W[k * 64 + lane] = W[k];
                }
                write_final_mem(a, key, m, lane, slot_v, n);
                const uint32_t pr = __ockl_wfred_add_u32(probes);
                finish_key(a, key, r == 1 ? LC_INVALID : LC_UNKNOWN, r == 1 ? LC_CAUSE_NONLIN : LC_CAUSE_BUDGET,
                           evno, peak, pr, (uint64_t)evno + (r == 1 ? 1u : 0u));
                return K_DONE;
            }
            peak = nSn > peak ? nSn : peak;
            const uint32_t last = n - 1;
            if (p != last) {
                const uint32_t d_last = __builtin_amdgcn_readlane(desc_v, last);
                const uint32_t s_last = __builtin_amdgcn_readlane(slot_v, last);
                const uint32_t x0 = __builtin_amdgcn_readlane(pass_v, last), x1 = __builtin_amdgcn_readlane(keep_v, last),
                               x2 = __builtin_amdgcn_readlane(set_v, last);
                if (lane == p) { desc_v = d_last; slot_v = s_last; pass_v = x0; keep_v = x1; set_v = x2; }
                if (lane == s_last) dense_v = p;
            }
            --n;
            if (in_mem && n == 8) {  // back to registers: no config holds index 8 or 9
#pragma unroll
                for (int k = 0; k < T0_RMAX; ++k) W[k] = m.W[k * 64 + lane];
                in_mem = false;
            }
        }
    }
    if (!in_mem) {
#pragma unroll
        for (int k = 0; k < T0_RMAX; ++k) m.W[k * 64 + lane] = W[k];
    }
    write_final_mem(a, key, m, lane, slot_v, n);
    const uint32_t pr = __ockl_wfred_add_u32(probes);
    finish_key(a, key, LC_VALID, LC_CAUSE_NONE, -1, peak, pr, e - b);
    return K_DONE;
}

// T0 over a work list: one wavefront per key (lattice in 4 registers, or the
// workspace for 9-10 pending ops).
__global__ __launch_bounds__(64) void k_search_lattice(Args a) {
    const int32_t n = a.n_in ? *a.n_in : a.n_order;
    for (int32_t w = next_work(a); w < n; w = next_work(a)) {
        const int32_t key = a.order[w];
        const int r = lattice_key<T0_RMAX>(a, key);
        if (r == K_SPILL) push_list(a.spill, a.n_spill, key);
    }
}

size_t lat_ws_words() { return 3 * T0_RMEM * 64; }

hipError_t launch_t0(const Args &a, int grid, hipStream_t s) {
    hipLaunchKernelGGL(k_search_lattice, dim3(grid), dim3(64), 0, s, a);
    return hipGetLastError();
}

}  // namespace lcd
