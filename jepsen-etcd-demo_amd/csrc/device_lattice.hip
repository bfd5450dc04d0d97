// device_lattice.hip -- T0: the JIT linearization search with the config set
// held as a subset lattice in registers (one wavefront per key).
//
// Same sets as every other tier (semantics: oracle/linear_ref.py).  The
// representation exploits two facts of the packed form:
//   * a config is (register state, set L of linearized pending ops), and the
//     pending ops are numbered densely 0..n-1 (n = ops pending; when op j
//     returns, op n-1 takes number j), so L is a subset of {0 .. n-1} and
//     n <= the key's concurrency (10 for the demo's 10 client threads);
//   * the register has few states (6 for the demo's values 0..4 + nil).
// So S is stored as W[L] = bitmask of states s with (s, L) in S, one 32-bit
// mask per subset L, subset index = lane + 64 * register.
//
// Per :ok(p) event:
//   Ret[L]  = W[L u {p}]              (configs that already linearized p)
//   I[L]    = W[L]          for p not in L; then the JIT closure
//   I[L u {q}] |= T_q(I[L]) for every pending q != p, to a fixpoint,
//   S'[L]   = Ret[L] | T_p(I[L])
// where T_q maps a state mask through op q's cas-register step, branch-free:
//   T(M) = min(M & k, cap) << b
//   (k = the states the op accepts, cap = ~0 for reads (T(M) = M & k, b = 0)
//    and 1 for writes / cas (T(M) = {b} if M & k is not empty):
//    read nil: k = all; read a: k = {a}; write b: k = all, cap = 1;
//    cas a->b: k = {a}, cap = 1).
// The closure runs as Gauss-Seidel sweeps over the subset-bit positions:
// lanes (subsets) WITH bit q gather I from the subset without it -- one
// DPP / permlane instruction for a lane bit, a register for a register bit --
// and positions are applied in place, so one sweep follows every path that
// adds ops in increasing index order.  A sweep that changes nothing ends the
// closure, and n - 1 sweeps always suffice (a path has at most n - 1 steps).
// Accept masks are lane-masked once per event (zero on lanes without bit q
// and for q = p), so a sweep position is 3 VALU instructions (v_and_b32_dpp
// with the gather folded in, v_min_u32, v_lshl_or_b32).
//
// Set sizes (budget, peak) are wave popcount reductions and the probe count
// (LC_OPT_COUNT_PROBES) is accumulated per lane, so every number reported
// equals the oracle's.  Keys outside T0's reach (more than 10 ops pending,
// more than 32 register states) go to the hash-set tiers.

#include <hip/hip_runtime.h>

#include <type_traits>

#include <algorithm>
#include <cstdint>

#include "../../include/lincheck.h"
#include "device_common.hpp"
#include "device_search.hpp"

extern "C" __device__ uint32_t __ockl_wfred_add_u32(uint32_t);

namespace lcd {

// Lattice registers per lane: the compact build holds n <= 8 pending ops in
// 4 registers (9-10 in the LDS workspace) and fits 4 waves per SIMD; the
// wide build holds n <= 10 in 16 registers (2 waves per SIMD) and is used
// when every key can be resident at once (launch_t0).
constexpr int T0_RSMALL = 4, T0_RBIG = 16;
constexpr int T0_RMEM = 16;            // workspace lattice (global memory): n <= 10
#ifndef LC_T0_MAX_WIDTH
#define LC_T0_MAX_WIDTH 10
#endif
constexpr uint32_t T0_MAX_WIDTH = LC_T0_MAX_WIDTH;  // <= 6 + log2(T0_RMEM)
constexpr uint32_t T0_MAX_STATES = 32;
uint32_t t0_max_width() { return T0_MAX_WIDTH; }
uint32_t t0_max_states() { return T0_MAX_STATES; }

struct Xfer { uint32_t k, cap, b, m; };

// A key's event words as the register tier reads them: the 32-bit form, or
// the 16-bit form lc_pack emits when every word fits (lc_batch.events16,
// LC_EV16_WIDE), read in place -- half the bytes per event and no widening
// pass over the batch before the search.
template <bool E16> struct EvSrc;
template <> struct EvSrc<false> {
    const uint32_t *p;
    __device__ __forceinline__ uint32_t operator[](uint64_t j) const { return p[j]; }
    __device__ __forceinline__ EvSrc operator+(uint64_t o) const { return {p + o}; }
};
template <> struct EvSrc<true> {
    const uint16_t *p;
    __device__ __forceinline__ uint32_t operator[](uint64_t j) const { return LC_EV16_WIDE(p[j]); }
    __device__ __forceinline__ EvSrc operator+(uint64_t o) const { return {p + o}; }
};
// A key's 16-bit event words staged in its workgroup's LDS (k_spec): the
// first n_lds words from there, the rest from HBM.  The cut search, every
// segment's TOP walk and its verifying run then read HBM once between them.
// (The LDS copy is held as an LDS-typed pointer: a generic one made every
// read a select between the two pointers and a flat load, waited on for both
// counters at once -- C2 / C5 / C3-shard times equal either way, tools/
// gpu_r4s.sh, but the window refill is a ds_read again.)
using LdsU16 = __attribute__((address_space(3))) const uint16_t;
struct EvStaged {
    LdsU16 *l;          // the LDS copy
    const uint16_t *g;  // the words in HBM
    uint32_t n_lds;
    __device__ __forceinline__ uint32_t operator[](uint64_t j) const {
        uint32_t w;
        if (j < n_lds) w = l[j];
        else w = g[j];
        return LC_EV16_WIDE(w);
    }
    __device__ __forceinline__ EvStaged operator+(uint64_t o) const {
        return {l + o, g + o, n_lds > o ? n_lds - (uint32_t)o : 0u};
    }
};

__device__ __forceinline__ Xfer xfer_of(uint32_t d) {
    const uint32_t f = d & 3u, a = (d >> 2) & 0x7FFFu, b = d >> 17;
    const uint32_t abit = a < 32u ? 1u << (a & 31u) : 0u;
    Xfer x;
    x.k = (f == LC_T_READ || f == LC_T_CAS) ? abit : 0xFFFFFFFFu;
    x.cap = f >= LC_T_WRITE ? 1u : 0xFFFFFFFFu;
    x.b = f >= LC_T_WRITE ? (b & 31u) : 0u;
    x.m = ~0u;
    return x;
}

// Tagged transfers (key segments, see k_search_segments): the lattice word
// holds 5 groups of 6 bits, group t = the states reachable from initial
// state t + 1 (register states 1..5, bit s - 1 of a group; bit 5 spare, 0).
// An op's transfer on a word is
//   T(M) = (((M & K) + C) >> s) & Mb
// with K = the accepted states in every group, and for a write / cas of
// state b: C = 31 in every group (a nonempty group carries into its bit 5),
// s = 6 - b (that bit lands on bit b - 1), Mb = bit b - 1 in every group;
// for a read C = 0, s = 0, Mb = ~0 (T(M) = M & K).  K = 0 gives 0 in every
// case (31 >> s never reaches bit b - 1), as the untagged form's does.
constexpr uint32_t TAG_REP = 0x1041041u;  // 1 in each 6-bit group
constexpr uint32_t TAG_ID = 0x10204081u;  // group t holds state t + 1: the identity start

__device__ __forceinline__ Xfer xfer_tag(uint32_t d) {
    const uint32_t f = d & 3u, a = (d >> 2) & 0x7FFFu, b = d >> 17;
    const uint32_t abit = (a >= 1u && a <= 5u) ? 1u << (a - 1u) : 0u;
    Xfer x;
    x.k = (f == LC_T_READ || f == LC_T_CAS) ? abit * TAG_REP : 0x1Fu * TAG_REP;
    const bool inst = f >= LC_T_WRITE && b >= 1u && b <= 5u;
    x.cap = inst ? 31u * TAG_REP : 0u;            // C
    x.b = inst ? 6u - b : 0u;                     // s
    x.m = inst ? (1u << (b - 1u)) * TAG_REP : ~0u;  // Mb
    if (f >= LC_T_WRITE && !inst) x.k = 0u;       // installs a state outside the tags: never taken
    return x;
}

// v with lane l (uniform, < 64) set to x: one v_writelane_b32.  Written as
// `lane == l ? x : v` the compiler masks EXEC around a move per value.
extern "C" __device__ int lc_writelane(int x, int l, int v) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ uint32_t setl(uint32_t v, uint32_t l, uint32_t x) {
    return (uint32_t)lc_writelane((int)x, (int)l, (int)v);
}

// x from lane (lane ^ 2^q), q < 6 uniform: one ds_bpermute on an address
// (lane * 4) ^ (4 << q).  __shfl_xor adds a width check (a compare and a
// select) and the shift of the lane index on every call.
__device__ __forceinline__ uint32_t xor_lane(uint32_t x, uint32_t q, uint32_t lane) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lane << 2) ^ (4u << q)), (int)x);
}

// s & v as one v_and_b32 (kept opaque: the compiler would turn an AND with a
// 0/~0 lane mask into a select through an SGPR pair)
__device__ __forceinline__ uint32_t vand(uint32_t s, uint32_t v) {
    uint32_t r;
    asm("v_and_b32 %0, %1, %2" : "=v"(r) : "s"(s), "v"(v));
    return r;
}

// acc | T(x) = acc | (min(x & k, cap) << b): v_and_b32, v_min_u32, v_lshl_or_b32
// (tagged: acc | ((((x & K) + C) >> s) & Mb): v_and, v_add, v_lshrrev, v_and_or)
template <bool TAG = false>
__device__ __forceinline__ uint32_t xacc(uint32_t acc, uint32_t x, uint32_t k, uint32_t cap, uint32_t b,
                                         uint32_t mb = ~0u) {
    if constexpr (TAG) return ((((x & k) + cap) >> b) & mb) | acc;
    else return (__builtin_elementwise_min(x & k, cap) << b) | acc;
}

// One-directional gathers along subset bit q < 6 (a lane-index bit):
//   gdown<q>(x)[L] = x[L - 2^q]   (meaningful on lanes WITH bit q)
//   gup<q>(x)[L]   = x[L + 2^q]   (meaningful on lanes WITHOUT bit q)
// One VALU instruction each: DPP quad_perm (q = 0, 1), DPP row_shr / row_shl
// (q = 2, 3; lanes whose source leaves the row read 0), gfx950
// v_permlane16_swap / v_permlane32_swap (q = 4, 5; the other half of the
// lanes reads garbage, which every caller masks).
// A DPP move whose lanes without a source read 0 (bound_ctrl) is written as
// update_dpp(0, x), so the compiler folds it into the single VALU op that
// consumes it (v_and_b32_dpp in a sweep).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp0(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, true);
}
template <int Q>
__device__ __forceinline__ uint32_t gdown(uint32_t x) {
    if constexpr (Q == 0) return dpp0<0xA0>(x);        // quad_perm [0,0,2,2]
    else if constexpr (Q == 1) return dpp0<0x44>(x);   // quad_perm [0,1,0,1]
    else if constexpr (Q == 2) return dpp0<0x114>(x);  // row_shr:4
    else if constexpr (Q == 3) return dpp0<0x118>(x);  // row_shr:8
    else if constexpr (Q == 4) return __builtin_amdgcn_permlane16_swap(x, x, false, false)[0];
    else return __builtin_amdgcn_permlane32_swap(x, x, false, false)[0];
}
// gdown with a dead register as the permlane's other operand: the swap
// clobbers both, so this saves one copy of x
template <int Q>
__device__ __forceinline__ uint32_t gdown_j(uint32_t x, uint32_t junk) {
    if constexpr (Q == 4) return __builtin_amdgcn_permlane16_swap(junk, x, false, false)[0];
    else if constexpr (Q == 5) return __builtin_amdgcn_permlane32_swap(junk, x, false, false)[0];
    else return gdown<Q>(x);
}
template <int Q>
__device__ __forceinline__ uint32_t gup(uint32_t x) {
    if constexpr (Q == 0) return dpp0<0xF5>(x);        // quad_perm [1,1,3,3]
    else if constexpr (Q == 1) return dpp0<0xEE>(x);   // quad_perm [2,3,2,3]
    else if constexpr (Q == 2) return dpp0<0x104>(x);  // row_shl:4
    else if constexpr (Q == 3) return dpp0<0x108>(x);  // row_shl:8
    else if constexpr (Q == 4) return __builtin_amdgcn_permlane16_swap(x, x, false, false)[1];
    else return __builtin_amdgcn_permlane32_swap(x, x, false, false)[1];
}
// Run-time bit (uniform q < 6): a scalar branch to one of the above.
__device__ __forceinline__ uint32_t gdown_rt(uint32_t x, uint32_t q) {
    switch (q) {
        case 0: return gdown<0>(x);
        case 1: return gdown<1>(x);
        case 2: return gdown<2>(x);
        case 3: return gdown<3>(x);
        case 4: return gdown<4>(x);
        default: return gdown<5>(x);
    }
}
__device__ __forceinline__ uint32_t gup_rt(uint32_t x, uint32_t q) {
    switch (q) {
        case 0: return gup<0>(x);
        case 1: return gup<1>(x);
        case 2: return gup<2>(x);
        case 3: return gup<3>(x);
        case 4: return gup<4>(x);
        default: return gup<5>(x);
    }
}

// x from lane (lane ^ 2^Q), both directions (workspace path).  Both gathers
// are evaluated unconditionally: a cross-lane op written inside `c ? a : b`
// would run under a divergent EXEC mask and read inactive source lanes.
template <int Q>
__device__ __forceinline__ uint32_t xv(uint32_t x, uint32_t lane) {
    const uint32_t d = gdown<Q>(x), u = gup<Q>(x);
    return ((lane >> Q) & 1u) ? d : u;
}

template <bool TAG = false>
__device__ __forceinline__ uint32_t xapply(uint32_t M, uint32_t k, uint32_t cap, uint32_t b, uint32_t mb = ~0u) {
    if constexpr (TAG) return (((M & k) + cap) >> b) & mb;
    else return __builtin_elementwise_min(M & k, cap) << b;
}

__device__ __forceinline__ bool idx_has(uint32_t lane, int k, uint32_t q) {
    return q < 6 ? ((lane >> q) & 1u) : (((uint32_t)k >> (q - 6)) & 1u);
}

template <int RL>
constexpr int lat_bits() { return RL == 1 ? 6 : RL == 2 ? 7 : RL == 4 ? 8 : RL == 8 ? 9 : 10; }

using Lat = uint32_t[T0_RBIG];

// T0's kernel arguments: only what the event loop reads, so the loop keeps
// its scalar registers (the full Args would spill SGPRs into VGPR lanes).
constexpr uint32_t T0_COUNT = 1, T0_WANT_PEAK = 2, T0_DBG_NOEVENTS = 4, T0_DBG_NOFINAL = 8, T0_WANT_FINAL = 16;
// T0_STRICT: the host skipped its per-event validation (a T0-only step: every
// key declared to fit the lattice).  T0 then checks the event stream itself
// as it walks it, and a key that would leave T0 is an error, not a spill (no
// later tier is launched to take it).
constexpr uint32_t T0_STRICT = 32;
// k_spec: cuts at equal estimated cost (spec_targets_cost) instead of equal
// event counts
constexpr uint32_t T0_SPEC_COST = 64;
// k_spec: TOP walks leave issue priority to age alone (no progress priority)
constexpr uint32_t T0_SPEC_NOPRIO = 128;
// k_spec: the T0_STRICT validation blocks come first in the grid (batches of
// more keys than the chip holds at once: dispatched last, they would run
// after the last round of keys, alone)
constexpr uint32_t T0_SPEC_VFIRST = 256;
// k_spec: events read from HBM, not staged in LDS (A/B)
constexpr uint32_t T0_SPEC_NOSTAGE = 512;
struct T0Args {
    const uint64_t *ev_off;
    const uint32_t *events;
    const uint16_t *events16;    // the same words in 16 bits, or null (E16 kernels read these)
    const uint32_t *trans;
    const uint32_t *trans_off;   // may be null
    const uint8_t *key_width;    // may be null
    const uint16_t *key_states;  // may be null
    const uint8_t *key_error;    // may be null
    const int32_t *order;
    int32_t *ticket;
    int32_t *err;                // [0] LC_BATCH_E_* bits, [1] 1 + largest malformed key
    int32_t err_base;            // that key's index in the caller's batch = err_base + key
    uint32_t *lat_ws;            // unused (the 9-10-pending workspace is in LDS)
    const Args *full;            // device copy: results, counters, spill list
    uint64_t budget;
    int32_t n_order;
    uint32_t init_state, shared_states, flags;
    uint32_t n_trans;            // entries of trans[]
    uint32_t ticket_base;        // ticket value this launch starts from (see launch_t0)
    uint32_t spec_ck1, spec_ck2; // speculative segments: checkpoint distances past a cut
    int32_t *spec_rr;            // speculative segments: keys left to the unsegmented search,
    int32_t *spec_nrr;           //   their count (zero at the launch)
    int32_t *spec_nrr_next;      //   and the next launch's count (zeroed by k_spec_rerun)
    uint32_t *spec_fin;          // exact segments: each run's saved set (2 per segment, SPEC_SAVE_WORDS each)
};

// T0Args read through the kernarg segment where a field is used (k_spec,
// LC_SPEC_KARG): a kernel that takes its arguments by value loads every field
// it uses anywhere at its entry and holds it in a scalar register for its
// whole life; with the walk's own scalars the file overflows into VGPR lanes
// and uniform loop words are kept in VGPRs (copied at every event).  The empty
// asm makes each use's pointer opaque, so no load is hoisted or shared.
using KT0 = const __attribute__((address_space(4))) T0Args;
__device__ __forceinline__ KT0 &t0k() {
    KT0 *p = (KT0 *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *p;
}

template <bool E16, class A = T0Args>
__device__ __forceinline__ EvSrc<E16> ev_src(const A &a) {
    if constexpr (E16) return {a.events16};
    else return {a.events};
}

template <class A = T0Args>
__device__ __forceinline__ void t0_malformed(const A &a, int32_t key, uint32_t why) {
    if (lane_id() == 0) {
        atomicOr(&a.err[0], (int32_t)why);
        atomicMax(&a.err[1], a.err_base + key + 1);
    }
}

// The lane index made opaque where it is used (workspace rows, lane masks).
// For the workspace: a row array's lane column, its address formed where
// used: with a plain m.W[k * 64 + lane] the compiler hoisted the 16 rows'
// 64-bit addresses out of the walk's event loop and kept them for its whole
// life -- 16 VGPR pairs, spilled to scratch in the 64-VGPR k_spec builds and
// rewritten there at every walk's start (round 5's 29.8x traffic).  The empty
// asm makes the lane index opaque, so each use site rebuilds one address and
// the rows are immediate offsets from it.
__device__ __forceinline__ uint32_t opq_lane(uint32_t lane) {
    asm volatile("" : "+v"(lane));
    return lane;
}

// Transfer masks of one event: vk[q] = op q's accept mask on lanes with bit
// q (0 elsewhere and for q = p); sc[q] / sb[q] = op q's cap / shift.
struct LaneMasks {
    uint32_t vk[6], sc[10], sb[10], sm[10];
};

template <int N, bool TAG = false>
__device__ __forceinline__ void lane_masks(LaneMasks &m, uint32_t p, uint32_t k_v, uint32_t cap_v, uint32_t b_v,
                                           uint32_t lane, uint32_t m_v = 0) {
#pragma unroll
    for (int q = 0; q < 6; ++q) m.vk[q] = 0u;
#pragma unroll
    for (int q = 0; q < 10; ++q) { m.sc[q] = 0u; m.sb[q] = 0u; }
    // (lane bit q as a 0 / ~0 word from an opaque lane index, p's mask
    // cleared in the scalar: written as `lane bit q && q != p ? sk : 0`, the
    // six lane conditions became loop-invariant 64-bit scalar masks, hoisted
    // out of the walk and spilled into VGPR lanes -- 12 v_readlane and 12
    // scalar selects at every 7-10-pending :ok of the 64-VGPR k_spec builds)
    const uint32_t ol = opq_lane(lane);
#pragma unroll
    for (int q = 0; q < (N < 6 ? N : 6); ++q) {
        const uint32_t sk = (uint32_t)q != p ? (uint32_t)__builtin_amdgcn_readlane(k_v, q) : 0u;
        m.vk[q] = sk & (uint32_t)__builtin_amdgcn_sbfe((int)ol, q, 1);
    }
#pragma unroll
    for (int q = 0; q < (N < 10 ? N : 10); ++q) {
        m.sc[q] = __builtin_amdgcn_readlane(cap_v, q);
        m.sb[q] = __builtin_amdgcn_readlane(b_v, q);
        if constexpr (TAG) m.sm[q] = __builtin_amdgcn_readlane(m_v, q);
    }
}

// One Gauss-Seidel pass over lane-bit positions Q .. min(N, 6) - 1.  A
// position is T_Q applied to the gathered word: min(x & k, cap) << b, OR-ed
// into cur.  The DPP gathers (Q < 4) have a single use and fold into the
// v_and_b32 (v_and_b32_dpp); the permlane swaps (Q = 4, 5) clobber both
// operands, so their other operand is `prev`, the previous position's min()
// result, dead once it has been shifted into cur -- one copy of cur per swap.
template <int Q, int N, bool TAG = false>
__device__ __forceinline__ uint32_t sweep_lanes(uint32_t cur, const LaneMasks &m, uint32_t prev = 0) {
    if constexpr (Q >= N || Q >= 6) {
        return cur;
    } else if constexpr (TAG) {
        const uint32_t x = gdown_j<Q>(cur, prev);
        const uint32_t t = (x & m.vk[Q]) + m.sc[Q];
        return sweep_lanes<Q + 1, N, TAG>(((t >> m.sb[Q]) & m.sm[Q]) | cur, m, t);
    } else {
        const uint32_t x = gdown_j<Q>(cur, prev);
        const uint32_t t = __builtin_elementwise_min(x & m.vk[Q], m.sc[Q]);
        return sweep_lanes<Q + 1, N>((t << m.sb[Q]) | cur, m, t);
    }
}

// Probe count of the oracle for one event (LC_OPT_COUNT_PROBES only): legal
// successors over I plus legal applications of p.
template <int RL, int NB>
__device__ __forceinline__ uint32_t event_probes(const uint32_t *I, uint32_t p, uint32_t cand, uint32_t k_v,
                                                 uint32_t lane, uint32_t pm) {
    uint32_t pr = 0;  // pm: p's accept mask
#pragma unroll
    for (int q = 0; q < NB; ++q) {
        const uint32_t m = ((cand >> q) & 1u) ? __builtin_amdgcn_readlane(k_v, q) : 0u;
#pragma unroll
        for (int k = 0; k < RL; ++k)
            if (!idx_has(lane, k, (uint32_t)q)) pr += (uint32_t)__popc(I[k] & m);
    }
#pragma unroll
    for (int k = 0; k < RL; ++k) pr += (uint32_t)__popc(I[k] & pm);
    return pr;
}

#ifdef LC_T0_COUNT_SWEEPS
// Diagnostic build only: histogram of (closure width nc, sweeps run).
__device__ unsigned long long lc_sweep_hist[8 * 8];
extern "C" int lc_debug_sweep_hist(unsigned long long *host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(lc_sweep_hist), sizeof(lc_sweep_hist), 0, hipMemcpyDeviceToHost);
}
#endif

// One :ok(p) event while every live op index is < 6: the whole lattice is
// one register and every subset bit is a lane bit.  Op indices are assigned
// lowest-free at invoke (not compacted), so an :ok only frees index p -- no
// relocation: S' lands on the lanes without bit p and lanes with bit p stay
// empty, which is exactly the state a later invoke into index p needs.  One
// code path for every live set (free positions and p carry zero masks), so an
// event costs no dispatch branches; the gather along the run-time bit p is one
// ds_bpermute, issued first so its latency hides under the mask setup.
// lm[q] (0 / ~0) is lane bit q as a VGPR mask.  W = S on entry, S' on a
// normal return.  Returns 0 normal, 1 invalid, 2 budget exceeded.
// The closure sweeps run until one changes nothing, without a trip counter
// (the sweeps only grow the set inside its closure, a finite lattice): the
// loop is the sweep, one v_cmp and a vcc branch -- six scalar instructions
// and a counter fewer per sweep than `for (s < nc) ... if (!__any) break`.
// C2 k_spec 0.2786 -> 0.2754 ms, C5 0.2834 -> 0.2808 (A/B on one box,
// tools/gpu_r4o.sh); LC_T0_SWEEP_DO=0 keeps the counted loop.
#ifndef LC_T0_SWEEP_DO
#define LC_T0_SWEEP_DO 1
#endif
template <int T>  // T = 1 + the highest live index (positions T.. are empty)
__device__ __forceinline__ int ok_lane(uint32_t &W, uint32_t p, uint32_t live, uint32_t k_v, uint32_t cap_v,
                                       uint32_t b_v, uint32_t pk, uint32_t pc, uint32_t pb, uint32_t lane,
                                       const uint32_t (&lm)[6], uint64_t budget, bool count, uint32_t &probes,
                                       uint32_t &nSn_out, bool want_size) {
    const uint32_t cand = live & ~(1u << p);
    const uint32_t wup = xor_lane(W, p, lane);
    // free indices and p hold zero accept masks in k_v (the caller cleared
    // lane p), so a position's masks need no gating by `cand`
    LaneMasks m;
#pragma unroll
    for (int q = 0; q < T; ++q) {
        m.vk[q] = vand(__builtin_amdgcn_readlane(k_v, q), lm[q]);
        m.sc[q] = __builtin_amdgcn_readlane(cap_v, q);
        m.sb[q] = __builtin_amdgcn_readlane(b_v, q);
    }
    const bool hp = (lane >> p) & 1u;
    if (count) probes += (uint32_t)__popc(W);
    uint32_t Ret = hp ? 0u : wup;
    uint32_t I = hp ? 0u : W;
    const uint32_t nc = (uint32_t)__popc(cand);  // a closure path has at most nc steps
#ifdef LC_T0_COUNT_SWEEPS
    uint32_t done_s = nc;
#endif
#if LC_T0_SWEEP_DO && !defined(LC_T0_COUNT_SWEEPS)
    // until a sweep changes nothing (see ok_lane_closed)
    (void)nc;
    bool ch;
    do {
        const uint32_t nv = sweep_lanes<0, T>(I, m);
        ch = nv != I;
        I = nv;
    } while (__any(ch));
#else
#pragma unroll 1
    for (uint32_t s = 0; s < nc; ++s) {
        const uint32_t nv = sweep_lanes<0, T>(I, m);
        const bool ch = nv != I;
        I = nv;
        if (!__any(ch)) {
#ifdef LC_T0_COUNT_SWEEPS
            done_s = s + 1;
#endif
            break;
        }
    }
#endif
#ifdef LC_T0_COUNT_SWEEPS
    if (lane == 0) atomicAdd(&lc_sweep_hist[nc * 8 + (done_s < 7 ? done_s : 7)], 1ull);
#endif
    if (count) probes += event_probes<1, 6>(&I, p, cand, k_v, lane, pk);
    Ret = xacc(Ret, I, pk, pc, pb);
    // One register holds at most 64 x 32 configs: with a larger budget only
    // emptiness matters (a ballot); exact sizes only when asked for (peak).
    if (__builtin_expect(budget < 64u * 32u, 0)) {
        const uint32_t nI = __ockl_wfred_add_u32((uint32_t)__popc(I));
        if (nI > budget) return 2;
    }
    if (!__any(Ret != 0u)) { nSn_out = 0; return 1; }
    if (__builtin_expect(budget < 64u * 32u || want_size, 0)) {
        const uint32_t nSn = __ockl_wfred_add_u32((uint32_t)__popc(Ret));
        nSn_out = nSn;
        if (nSn > budget) return 2;
    }
    W = Ret;
    return 0;
}

// Fast path (verdicts only): the lane lattice is kept CLOSED under every
// pending op instead of holding exactly Knossos's set S.  With C(S) the
// closure of S under the pending ops, the projection
//     { (s, L \ p) : (s, L) in C(S_k), p in L }  =  C(S_{k+1}),
// so an :ok(p) is "close W, then keep the lanes with bit p, shifted down":
// S_{k+1} is empty iff that projection is.  Any W with S <= W <= C(S) closes
// to C(S), and W is already closed when no op was invoked since the last
// :ok (`dirty` false): then the :ok is the projection alone.  Sets are
// supersets of Knossos's, so this path is used only when no set size, probe
// count or config list is asked for (FAST in lattice_key).
// Returns 0 normal, 1 invalid (W unchanged).
template <int T, bool TAG = false>
__device__ __forceinline__ int ok_lane_closed(uint32_t &W, uint32_t p, uint32_t live, uint32_t k_v, uint32_t cap_v,
                                              uint32_t b_v, uint32_t lane, const uint32_t (&lm)[6], bool dirty,
                                              uint32_t m_v = 0) {
    uint32_t C = W;
    if (dirty) {
        LaneMasks m;
#pragma unroll
        for (int q = 0; q < T; ++q) {
            m.vk[q] = vand(__builtin_amdgcn_readlane(k_v, q), lm[q]);
            m.sc[q] = __builtin_amdgcn_readlane(cap_v, q);
            m.sb[q] = __builtin_amdgcn_readlane(b_v, q);
            if constexpr (TAG) m.sm[q] = __builtin_amdgcn_readlane(m_v, q);
        }
#if LC_T0_SWEEP_DO
        // until a sweep changes nothing: the sweeps only grow C inside the
        // closure, a finite lattice, so the loop ends (no trip counter)
        bool ch;
        do {
            const uint32_t nv = sweep_lanes<0, T, TAG>(C, m);
            ch = nv != C;
            C = nv;
        } while (__any(ch));
#else
        const uint32_t nc = (uint32_t)__popc(live);  // a path has at most nc steps
#pragma unroll 1
        for (uint32_t s = 0; s < nc; ++s) {
            const uint32_t nv = sweep_lanes<0, T, TAG>(C, m);
            const bool ch = nv != C;
            C = nv;
            if (!__any(ch)) break;
        }
#endif
    }
    // (a DPP switch on p measured slower, in the compact T0 and in the
    // speculative segments' walk: 1,224 against 1,142 cycles per event)
    const uint32_t up = xor_lane(C, p, lane);
    // (lane bit p as a 0 / ~0 word: one v_bfe, and the select a v_bfi)
    const uint32_t Wn = up & ~(uint32_t)__builtin_amdgcn_sbfe((int)lane, (int)p, 1);
    if (!__any(Wn != 0u)) return 1;
    W = Wn;
    return 0;
}

// One :ok(p) event on a lattice of RL registers (N = 7 or 8 ops pending):
// lane bits 0..5 as in ok_lane, register bits 6.. through register pairs.
template <int RL, int RM, bool TAG = false>
__device__ __forceinline__ int ok_reg(uint32_t (&W)[RM], uint32_t p, uint32_t k_v, uint32_t cap_v, uint32_t b_v,
                                      uint32_t lane, uint64_t budget, bool count, uint32_t &probes,
                                      uint32_t &nSn_out, bool want_size, uint32_t m_v = 0) {
    constexpr int NB = lat_bits<RL>();  // = ops pending
    constexpr int NR = NB - 6;          // register bits
    LaneMasks m;
    lane_masks<NB, TAG>(m, p, k_v, cap_v, b_v, lane, m_v);
    uint32_t rk[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const bool on = (uint32_t)(6 + r) != p;
        const uint32_t sk = __builtin_amdgcn_readlane(k_v, 6 + r);
        rk[r] = on ? sk : 0u;
    }
    const uint32_t pk = __builtin_amdgcn_readlane(k_v, p), pc = __builtin_amdgcn_readlane(cap_v, p),
                   pb = __builtin_amdgcn_readlane(b_v, p);
    const uint32_t pm = TAG ? __builtin_amdgcn_readlane(m_v, p) : ~0u;
    uint32_t Ret[RL], I[RL];
    if (count) {
#pragma unroll
        for (int k = 0; k < RL; ++k) probes += (uint32_t)__popc(W[k]);
    }
    if (p < 6) {
        const bool hp = (lane >> p) & 1u;
#pragma unroll
        for (int k = 0; k < RL; ++k) {
            const uint32_t u = gup_rt(W[k], p);
            Ret[k] = hp ? 0u : u;
            I[k] = hp ? 0u : W[k];
        }
    } else {
        const uint32_t r = p - 6;
#pragma unroll
        for (int k = 0; k < RL; ++k) {
            uint32_t src = W[k];
#pragma unroll
            for (int rr = 0; rr < NR; ++rr)
                if (r == (uint32_t)rr) src = W[k | (1 << rr)];
            const bool hk = ((uint32_t)k >> r) & 1u;
            Ret[k] = hk ? 0u : src;
            I[k] = hk ? 0u : W[k];
        }
    }
#pragma unroll 1
    for (int s = 1; s < NB; ++s) {
        uint32_t nv[RL];
#pragma unroll
        for (int k = 0; k < RL; ++k) nv[k] = sweep_lanes<0, 6, TAG>(I[k], m);
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
            for (int k = 0; k < RL; ++k)
                if ((k >> r) & 1)
                    nv[k] = xacc<TAG>(nv[k], nv[k ^ (1 << r)], rk[r], m.sc[6 + r], m.sb[6 + r], TAG ? m.sm[6 + r] : ~0u);
        bool ch = false;
#pragma unroll
        for (int k = 0; k < RL; ++k) { ch |= nv[k] != I[k]; I[k] = nv[k]; }
        if (!__any(ch)) break;
    }
    if (count)
        probes += event_probes<RL, NB>(I, p, ((1u << NB) - 1u) & ~(1u << p), k_v, lane, pk);
    uint32_t cI = 0, cS = 0;
#pragma unroll
    for (int k = 0; k < RL; ++k) {
        Ret[k] = xacc<TAG>(Ret[k], I[k], pk, pc, pb, pm);
        cI += (uint32_t)__popc(I[k]);
        cS += (uint32_t)__popc(Ret[k]);
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
    constexpr int rl = NR - 1;  // `last` = NB - 1 is register bit rl
    if (p == (uint32_t)(NB - 1)) {
#pragma unroll
        for (int k = 0; k < RL; ++k) W[k] = Ret[k];
        return 0;
    }
    if (p < 6) {
        const bool hp = (lane >> p) & 1u;
#pragma unroll
        for (int k = 0; k < RL; ++k) {
            if ((k >> rl) & 1) { W[k] = 0u; continue; }
            const uint32_t z = gdown_rt(Ret[k | (1 << rl)], p);
            W[k] = hp ? z : Ret[k];
        }
    } else {
        const uint32_t r = p - 6;
#pragma unroll
        for (int k = 0; k < RL; ++k) {
            if ((k >> rl) & 1) { W[k] = 0u; continue; }
            uint32_t src = Ret[k];
#pragma unroll
            for (int rr = 0; rr < NR; ++rr)
                if (r == (uint32_t)rr) src = Ret[(k ^ (1 << rr)) | (1 << rl)];
            W[k] = (((uint32_t)k >> r) & 1u) ? src : Ret[k];
        }
    }
    return 0;
}

// Lattice of a key with 9 or 10 ops pending: 16 x 64 words per array in the
// block's LDS workspace, index k * 64 + lane.  Every lane reads and writes
// only its own column (register-bit partners are in the same lane; lane-bit
// partners are exchanged in registers), so no cross-lane memory ordering is
// involved.  Such events are rare (< 0.2 % of C2's); keeping them out of
// registers keeps T0's register budget small.
struct LatMem {
    uint32_t *W, *R, *I;
};


template <int RL, bool TAG = false>
__device__ __forceinline__ int ok_event_mem(const LatMem &m, uint32_t p, uint32_t n, uint32_t k_v,
                                            uint32_t cap_v, uint32_t b_v, uint32_t lane, uint64_t budget,
                                            bool count, uint32_t &probes, uint32_t &nSn_out, bool want_size,
                                            uint32_t m_v = 0) {
    constexpr int NB = lat_bits<RL>();
    const uint32_t cand = ((1u << n) - 1u) & ~(1u << p);
    // transfer of candidate q: lane q of k_v/cap_v/b_v, read at use
    // (not hoisted: 3 x NB scalars would spill SGPRs into the VGPR budget)
    const uint32_t ck = k_v & (((cand >> lane) & 1u) ? ~0u : 0u);
#define KK(Q) __builtin_amdgcn_readlane(ck, Q)
#define CP(Q) __builtin_amdgcn_readlane(cap_v, Q)
#define SB(Q) __builtin_amdgcn_readlane(b_v, Q)
#define SM(Q) (TAG ? __builtin_amdgcn_readlane(m_v, Q) : ~0u)
    const uint32_t pk = __builtin_amdgcn_readlane(k_v, p), pc = __builtin_amdgcn_readlane(cap_v, p),
                   pb = __builtin_amdgcn_readlane(b_v, p), pm = SM(p);
    const uint32_t plm = p < 6 ? 1u << p : 0u, prm = p >= 6 ? 1u << (p - 6) : 0u;
#pragma unroll 1
    for (int k = 0; k < RL; ++k) {
        const uint32_t w = m.W[k * 64 + lane];
        if (count) probes += (uint32_t)__popc(w);
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
                acc |= ((lane >> Q) & 1u) ? xapply<TAG>(y, KK(Q), CP(Q), SB(Q), SM(Q)) : 0u; \
            }
            LC_LANEBIT(0) LC_LANEBIT(1) LC_LANEBIT(2) LC_LANEBIT(3) LC_LANEBIT(4) LC_LANEBIT(5)
#undef LC_LANEBIT
#pragma unroll
            for (int q = 6; q < NB; ++q)
                if ((k >> (q - 6)) & 1)
                    acc |= xapply<TAG>(m.I[(k ^ (1 << (q - 6))) * 64 + lane], KK(q), CP(q), SB(q), SM(q));
            if (acc != x) { m.I[k * 64 + lane] = acc; ch = true; }
        }
        if (!__any(ch)) break;
    }
    uint32_t cI = 0, cS = 0;
#pragma unroll 1
    for (int k = 0; k < RL; ++k) {
        const uint32_t x = m.I[k * 64 + lane];
        if (count) {
#pragma unroll
            for (int q = 0; q < NB; ++q)
                if (!idx_has(lane, k, (uint32_t)q)) probes += (uint32_t)__popc(x & KK(q));
            probes += (uint32_t)__popc(x & pk);
        }
        const uint32_t r = m.R[k * 64 + lane] | xapply<TAG>(x, pk, pc, pb, pm);
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
#undef KK
#undef CP
#undef SB
#undef SM
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

// ok_event_mem's closure as Gauss-Seidel sweeps (verdicts only: no sizes or
// probes): each row a one-directional lane sweep (sweep_lanes, 3 VALU per
// position), then the register bits from the rows below it, already updated
// in this sweep.  The bidirectional per-row form above needs about twice the
// instructions per sweep and more sweeps.
template <int RL>
__device__ __forceinline__ int ok_event_mem_gs(const LatMem &m, uint32_t p, uint32_t n, uint32_t k_v, uint32_t cap_v,
                                               uint32_t b_v, uint32_t lane) {
    constexpr int NB = lat_bits<RL>();
    constexpr int NR = NB - 6;
    LaneMasks lmk;
    lane_masks<NB>(lmk, p, k_v, cap_v, b_v, lane);
    uint32_t rk[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) rk[r] = (uint32_t)(6 + r) != p ? __builtin_amdgcn_readlane(k_v, 6 + r) : 0u;
    const uint32_t pk = __builtin_amdgcn_readlane(k_v, p), pc = __builtin_amdgcn_readlane(cap_v, p),
                   pb = __builtin_amdgcn_readlane(b_v, p);
    const uint32_t plm = p < 6 ? 1u << p : 0u, prm = p >= 6 ? 1u << (p - 6) : 0u;
    const uint32_t ol = opq_lane(lane);
    uint32_t *const mW = m.W + ol, *const mR = m.R + ol, *const mI = m.I + ol;
#pragma unroll 1
    for (int k = 0; k < RL; ++k) {
        const uint32_t w = mW[k * 64];
        const uint32_t src = (uint32_t)__shfl_xor((int)mW[(k ^ prm) * 64], (int)plm);
        const bool hp = (lane & plm) || ((uint32_t)k & prm);
        mR[k * 64] = hp ? 0u : src;
        mI[k * 64] = hp ? 0u : w;
    }
#pragma unroll 1
    for (int s = 0; s < NB; ++s) {
        bool ch = false;
#pragma unroll 1
        for (int k = 0; k < RL; ++k) {
            const uint32_t x = mI[k * 64];
            uint32_t nv = sweep_lanes<0, 6>(x, lmk);
#pragma unroll
            for (int r = 0; r < NR; ++r)
                if ((k >> r) & 1) nv = xacc(nv, mI[(k ^ (1 << r)) * 64], rk[r], lmk.sc[6 + r], lmk.sb[6 + r]);
            if (nv != x) {
                mI[k * 64] = nv;
                ch = true;
            }
        }
        if (!__any(ch)) break;
    }
    uint32_t cS = 0;
#pragma unroll 1
    for (int k = 0; k < RL; ++k) {
        const uint32_t r = mR[k * 64] | xapply(mI[k * 64], pk, pc, pb);
        mR[k * 64] = r;
        cS |= r;
    }
    if (!__any(cS != 0u)) return 1;
    const uint32_t last = n - 1;
    const uint32_t llm = last < 6 ? 1u << last : 0u, lrm = last >= 6 ? 1u << (last - 6) : 0u;
#pragma unroll 1
    for (int k = 0; k < RL; ++k) {
        const uint32_t r = mR[k * 64];
        const uint32_t src = (uint32_t)__shfl_xor((int)mR[(k ^ (prm | lrm)) * 64], (int)(plm | llm));
        const bool hp = (lane & plm) || ((uint32_t)k & prm);
        const bool hl = (lane & llm) || ((uint32_t)k & lrm);
        mW[k * 64] = p == last ? r : (hl ? 0u : (hp ? src : r));
    }
    return 0;
}

// The max_final smallest configs of the lattice held in m.W (register
// lattices are stored there first) in (slot mask, state) order, op indices
// translated back to window slots (slot_v: lane j holds the slot of the op
// at index j; `live` = the occupied indices).  The order is the window's, not
// the op indices', so every run that holds the same set -- the unsegmented
// search, a speculative segment's that assigned its own indices -- writes
// the same records (Knossos's truncation to 10 is of an unordered set; any
// fixed choice matches it).  Selection: max_final rounds of a wave minimum.
__device__ __forceinline__ void write_final_mem(const Args &a, int32_t key, const LatMem &m, uint32_t lane,
                                                uint32_t slot_v, uint32_t live_ops) {
    if (!a.final_cfg) return;
    const uint32_t mf = (uint32_t)a.max_final;
    const uint32_t top = live_ops ? 32u - (uint32_t)__clz(live_ops) : 0u;  // index bits in use
    const int live = top <= 6 ? 1 : (1 << (top - 6));
    // slot mask of subset L = lane + 64 k: the lane's bits (indices 0..5)
    // and the row's (6..), the latter uniform
    uint64_t lo = 0;
    uint32_t cnt = 0;
    for (uint32_t j = 0; j < top && j < 6u; ++j) {
        const uint32_t sj = __builtin_amdgcn_readlane(slot_v, j);
        if (((lane & live_ops) >> j) & 1u) lo |= 1ull << sj;
    }
#pragma unroll 1
    for (int k = 0; k < live; ++k) cnt += (uint32_t)__popc(m.W[k * 64 + lane]);
    const uint32_t tot = __ockl_wfred_add_u32(cnt);
    const uint32_t nw = tot < mf ? tot : mf;
    uint64_t last_m = 0;
    int last_s = -1;
#pragma unroll 1
    for (uint32_t r = 0; r < nw; ++r) {
        const uint32_t above = last_s < 0 ? ~0u : last_s >= 31 ? 0u : ~((2u << last_s) - 1u);
        uint64_t bm = ~0ull;
        uint32_t bs = 32;
#pragma unroll 1
        for (int k = 0; k < live; ++k) {
            uint32_t w = m.W[k * 64 + lane];
            uint64_t hi = 0;
            for (uint32_t j = 6; j < top; ++j)
                if ((((uint32_t)k << 6) & live_ops) >> j & 1u) hi |= 1ull << __builtin_amdgcn_readlane(slot_v, j);
            const uint64_t sm = lo | hi;
            if (sm == last_m) w &= above;
            if (w && sm >= last_m && sm < bm) {
                bm = sm;
                bs = (uint32_t)__ffs(w) - 1;
            }
        }
        uint64_t mn = bm;
        for (int o = 32; o >= 1; o >>= 1) {
            const uint32_t l2 = (uint32_t)__shfl_xor((int)(uint32_t)mn, o), h2 = (uint32_t)__shfl_xor((int)(uint32_t)(mn >> 32), o);
            const uint64_t v = ((uint64_t)h2 << 32) | l2;
            mn = v < mn ? v : mn;
        }
        uint32_t st = bm == mn ? bs : 32u;
        for (int o = 32; o >= 1; o >>= 1) {
            const uint32_t v = (uint32_t)__shfl_xor((int)st, o);
            st = v < st ? v : st;
        }
        if (lane == 0) {
            a.final_cfg[((size_t)key * a.max_final + r) * 2 + 0] = mn;
            a.final_cfg[((size_t)key * a.max_final + r) * 2 + 1] = (uint64_t)st << 48;
        }
        last_m = mn;
        last_s = (int)st;
    }
    if (lane == 0 && a.n_final) a.n_final[key] = nw;
}

// Op indices: an invoke takes the lowest free index.  While at most 6 ops are
// pending every live index is < 6 and an :ok just frees its index (ok_lane);
// from 7 pending on the indices are dense (0..n-1) and an :ok refills the
// freed index p with the op at index n-1 (a two-bit exchange of the lattice),
// so the lattice spans 2^n subsets.
//
// The event loop has one exit test per event and no early returns: the
// compiler then keeps one flat loop (no state-machine phi copies), and with
// the 9-10-pending workspace in LDS there are no global stores in the loop,
// so the prefetch of the next chunk is never waited for early.
//
// Register budget: the loop only touches the T0Args fields it needs; result
// pointers, counters and work lists are read through `full` (a copy of the
// tier's Args in device memory) once per key.
#ifdef LC_T0_PROFILE
// Diagnostic build only: cycles and counts per event class (invoke, :ok with
// <= 6, 7, 8, 9, 10 pending), summed over every key.
__device__ unsigned long long lc_t0_prof[12];
__shared__ unsigned long long lc_t0_prof_lds[12];
extern "C" int lc_debug_t0_prof(unsigned long long *host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(lc_t0_prof), sizeof(lc_t0_prof), 0, hipMemcpyDeviceToHost);
}
#endif

// FAST: no probe counting, no peak sizes and a budget no lattice can exceed
// (>= 16 x 64 x 32 configs), so every size reduction and budget test folds
// away -- the common case, and the bench's.
template <int RM, bool FAST, bool E16 = false>
__device__ __forceinline__ int lattice_key(const T0Args &a, int32_t key, uint32_t *ws) {
    const uint32_t lane = lane_id();
    const LatMem m{ws, ws + T0_RMEM * 64, ws + 2 * T0_RMEM * 64};
    const uint64_t eb = a.ev_off[key], ee = a.ev_off[key + 1];
    const uint32_t tb = a.trans_off ? a.trans_off[key] : 0u;
    if (a.key_error && a.key_error[key]) {  // lc_pack could not prepare it (check-safe)
        finish_key(*a.full, key, LC_UNKNOWN, LC_CAUSE_ERROR, -1, 0, 0, 0);
        return K_DONE;
    }
    if (a.key_states && a.key_states[key] > LC_WIDE_MAX_STATES) {
        finish_key(*a.full, key, LC_UNKNOWN, LC_CAUSE_STATES, -1, 1, 0, 0);
        return K_DONE;
    }
    const uint32_t nstates = a.trans_off ? (a.key_states ? a.key_states[key] : 0xFFFFu) : a.shared_states;
    const uint32_t width = a.key_width ? a.key_width[key] : 0xFFu;  // = max ops pending at once
    if (nstates > T0_MAX_STATES || width > T0_MAX_WIDTH || a.init_state >= T0_MAX_STATES) return K_SPILL;
    const uint64_t budget = FAST ? ~0ull : a.budget;
    const bool want_peak = !FAST && (a.flags & T0_WANT_PEAK) != 0;
    const bool count = !FAST && (a.flags & T0_COUNT) != 0;
    const EvSrc<E16> evp = ev_src<E16>(a) + eb;
    // The key may name transitions trans[tb + t], t < ntr.  A batch the host
    // did not validate may hold larger ids: they load nothing (the event is
    // then a read of nil), and the batch's validation waves report them.
    // Every other malformation (an :ok of a slot that is not pending, an
    // :invoke into an occupied one) leaves T0 in bounds -- indices stay below
    // T0_MAX_WIDTH and lanes below 64 -- with a verdict the failed call
    // does not return.
    const uint32_t ntr = a.n_trans > tb ? a.n_trans - tb : 0u;
    const uint32_t *const trp = a.trans + (ntr ? tb : 0u);
    const uint32_t nev = (a.flags & T0_DBG_NOEVENTS) ? 0u : (uint32_t)(ee - eb);
    auto ldesc = [&](uint32_t w, bool have) -> uint32_t {
        const uint32_t t = LC_EV_TRANS(w);
        return (have && !(w & LC_EV_OK_BIT) && t < ntr) ? trp[t] : 0u;
    };

    uint32_t W[RM];
#pragma unroll
    for (int k = 0; k < RM; ++k) W[k] = 0;
    if (lane == 0) W[0] = 1u << a.init_state;
    bool in_mem = false;   // lattice lives in m.W (9 or 10 ops pending)
    uint32_t k_v = 0, cap_v = 0, b_v = 0;  // lane j: transfer (k, cap, b) of the op at index j
    uint32_t slot_v = 0;   // lane j: window slot of the op at index j
    uint32_t dense_v = 0;  // lane s: index of the op in window slot s
    uint32_t n = 0;        // ops pending
    uint32_t live = 0;     // occupied op indices (all < 6 while n <= 6; 0..n-1 beyond)
    uint32_t lm[6];        // lane bit q as a 0 / ~0 mask
#pragma unroll
    for (int q = 0; q < 6; ++q) lm[q] = (uint32_t)__builtin_amdgcn_sbfe((int)lane, q, 1);
    uint32_t peak = 1, probes = 0;
    int status = 0;        // 1 invalid, 2 budget, 3 spill
    uint32_t fev = 0;

    // Event cursor: events arrive 64 at a time, one per lane; the next
    // chunk's words and descriptors are in flight while this one is searched.
    uint32_t ev = lane < nev ? evp[lane] : 0u;
    uint32_t dsc = ldesc(ev, lane < nev);
    uint32_t ev_n = 64 + lane < nev ? evp[64 + lane] : 0u;
    uint32_t dsc_n = ldesc(ev_n, 64 + lane < nev);
    uint32_t ev_nn = 128 + lane < nev ? evp[128 + lane] : 0u;
    // each lane decodes its event's transition once per chunk (VALU, all 64
    // at a time), so an invoke only reads three lanes
    Xfer xc = xfer_of(dsc);
    uint32_t e = 0, i = 0, base = 0;
    uint32_t lim = nev;  // 0 once the key has a verdict: each loop's only exit is its head
    auto advance = [&]() {
        ++e;
        if (++i == 64u) {
            i = 0; base += 64;
            ev = ev_n; dsc = dsc_n; ev_n = ev_nn;
            xc = xfer_of(dsc);
            dsc_n = ldesc(ev_n, base + 64 + lane < nev);
            ev_nn = base + 128 + lane < nev ? evp[base + 128 + lane] : 0u;
        }
    };
#ifdef LC_T0_PROFILE
#define T0_PROF_BEGIN const unsigned long long pt0 = __builtin_amdgcn_s_memtime(); const uint32_t pn0 = n;
#define T0_PROF_END(evi)                                                                   \
    {                                                                                      \
        const unsigned long long pt1 = __builtin_amdgcn_s_memtime();                       \
        const uint32_t cat = !((evi) & LC_EV_OK_BIT) ? 0u : (pn0 <= 6 ? 1u : pn0 - 5u);    \
        if (lane == 0 && cat < 6) { lc_t0_prof_lds[cat] += pt1 - pt0; lc_t0_prof_lds[6 + cat] += 1; } \
    }
#else
#define T0_PROF_BEGIN
#define T0_PROF_END(evi)
#endif

    // Two phases, each a loop of its own, so that neither carries the
    // other's values through its back edge (one loop for both made the
    // register allocator copy every loop-carried value twice per event):
    //   lane phase  -- at most 6 ops pending, every live index < 6, the
    //                  lattice in one register (W0);
    //   dense phase -- 7 to 10 pending, dense indices, W[0..3] or the LDS
    //                  workspace; left after the :ok that brings n back to 6.
    uint32_t W0 = W[0];
    bool dirty = true;  // FAST: an op was invoked since the lattice was last closed
    for (uint32_t phase = 0; phase <= nev && e < lim; ++phase) {
        while (e < lim) {
            T0_PROF_BEGIN
            const uint32_t evi = __builtin_amdgcn_readlane(ev, i);
            const uint32_t slot = LC_EV_SLOT(evi);
            if (!(evi & LC_EV_OK_BIT)) {
                if (n == 6) break;  // a 7th pending op: the dense phase takes this invoke
                if (n >= T0_MAX_WIDTH || slot >= 64) {
                    status = 3;
                } else {
                    const Xfer x{(uint32_t)__builtin_amdgcn_readlane(xc.k, i),
                                 (uint32_t)__builtin_amdgcn_readlane(xc.cap, i),
                                 (uint32_t)__builtin_amdgcn_readlane(xc.b, i)};
                    const uint32_t idx = (uint32_t)__builtin_ctz(~live);  // lowest free index
                    slot_v = setl(slot_v, idx, slot);
                    k_v = setl(k_v, idx, x.k);
                    cap_v = setl(cap_v, idx, x.cap);
                    b_v = setl(b_v, idx, x.b);
                    dense_v = setl(dense_v, slot, idx);
                    live |= 1u << idx;
                    ++n;
                    dirty = true;
                }
            } else {
                const uint32_t p = __builtin_amdgcn_readlane(dense_v, slot & 63u);
                uint32_t nSn = 0;
                int r;
                if constexpr (FAST && RM == T0_RSMALL) {
                    // closed sets (compact build only: on C2's lone waves the
                    // projection's exposed bpermute ate the saved sweeps)
                    const uint32_t top = 32u - (uint32_t)__builtin_clz(live);
                    if (top >= 6) r = ok_lane_closed<6>(W0, p, live, k_v, cap_v, b_v, lane, lm, dirty);
                    else if (top == 5) r = ok_lane_closed<5>(W0, p, live, k_v, cap_v, b_v, lane, lm, dirty);
                    else r = ok_lane_closed<4>(W0, p, live, k_v, cap_v, b_v, lane, lm, dirty);
                    dirty = false;
                    k_v = setl(k_v, p, 0u);
                } else {
                // p's transfer, then p's lane cleared for good: its index is
                // free after this :ok (and an invalid key stops here)
                const uint32_t pk = __builtin_amdgcn_readlane(k_v, p), pc = __builtin_amdgcn_readlane(cap_v, p),
                               pb = __builtin_amdgcn_readlane(b_v, p);
                k_v = setl(k_v, p, 0u);
                // Compact build (many keys per SIMD, throughput): sweeps cover
                // the positions below the highest live index only.  Wide build
                // (one key per SIMD, latency): one sweep body for every event --
                // the specialised copies cost more in instruction-cache misses
                // across a CU's four lone waves than they save.
                const uint32_t top = 32u - (uint32_t)__builtin_clz(live);
#ifndef LC_T0_WIDE_SPEC  // 1: specialise the wide build too (measured slower on C2)
#define LC_T0_WIDE_SPEC 0
                if ((RM == T0_RBIG && !LC_T0_WIDE_SPEC) || top >= 6)
                    r = ok_lane<6>(W0, p, live, k_v, cap_v, b_v, pk, pc, pb, lane, lm, budget, count, probes, nSn,
                                   want_peak);
                else if (top == 5)
                    r = ok_lane<5>(W0, p, live, k_v, cap_v, b_v, pk, pc, pb, lane, lm, budget, count, probes, nSn,
                                   want_peak);
                else
                    r = ok_lane<4>(W0, p, live, k_v, cap_v, b_v, pk, pc, pb, lane, lm, budget, count, probes, nSn,
                                   want_peak);
                }
#endif
                live = r ? live : live & ~(1u << p);
                n = r ? n : n - 1;
                peak = nSn > peak ? nSn : peak;
                status = r;
                fev = e;
            }
            T0_PROF_END(evi)
            lim = status ? 0u : lim;
            advance();
        }
        if (e >= lim) break;
        W[0] = W0;
#pragma unroll
        for (int k = 1; k < RM; ++k) W[k] = 0u;
        while (e < lim) {
            T0_PROF_BEGIN
            const uint32_t evi = __builtin_amdgcn_readlane(ev, i);
            const uint32_t slot = LC_EV_SLOT(evi);
            if (!(evi & LC_EV_OK_BIT)) {
                if (n >= T0_MAX_WIDTH || slot >= 64) {
                    status = 3;
                } else {
                    if (RM < 16 && n == 8) {  // 9 pending: move the lattice to the workspace
#pragma unroll
                        for (int k = 0; k < T0_RMEM; ++k) m.W[k * 64 + lane] = k < RM ? W[k < RM ? k : 0] : 0u;
                        in_mem = true;
                    }
                    const Xfer x{(uint32_t)__builtin_amdgcn_readlane(xc.k, i),
                                 (uint32_t)__builtin_amdgcn_readlane(xc.cap, i),
                                 (uint32_t)__builtin_amdgcn_readlane(xc.b, i)};
                    const uint32_t idx = n;  // dense: every index below n is taken
                    slot_v = setl(slot_v, idx, slot);
                    k_v = setl(k_v, idx, x.k);
                    cap_v = setl(cap_v, idx, x.cap);
                    b_v = setl(b_v, idx, x.b);
                    dense_v = setl(dense_v, slot, idx);
                    live |= 1u << idx;
                    ++n;
                }
            } else {
                const uint32_t p = __builtin_amdgcn_readlane(dense_v, slot & 63u);
                uint32_t nSn = 0;
                int r;
                if (n == 7) r = ok_reg<2>(W, p, k_v, cap_v, b_v, lane, budget, count, probes, nSn, want_peak);
                else if (n == 8) r = ok_reg<4>(W, p, k_v, cap_v, b_v, lane, budget, count, probes, nSn, want_peak);
                else if constexpr (RM < 16) {
                    if (n == 9)
                        r = ok_event_mem<8>(m, p, n, k_v, cap_v, b_v, lane, budget, count, probes, nSn, want_peak);
                    else
                        r = ok_event_mem<16>(m, p, n, k_v, cap_v, b_v, lane, budget, count, probes, nSn, want_peak);
                } else {
                    if (n == 9) r = ok_reg<8>(W, p, k_v, cap_v, b_v, lane, budget, count, probes, nSn, want_peak);
                    else r = ok_reg<16>(W, p, k_v, cap_v, b_v, lane, budget, count, probes, nSn, want_peak);
                }
                // the op at index `last` takes index p (a no-op when p == last)
                const uint32_t last = n - 1;
                const uint32_t s_last = __builtin_amdgcn_readlane(slot_v, last);
                const uint32_t x0 = __builtin_amdgcn_readlane(k_v, last),
                               x1 = __builtin_amdgcn_readlane(cap_v, last), x2 = __builtin_amdgcn_readlane(b_v, last);
                if (!r) {
                    slot_v = setl(slot_v, p, s_last);
                    k_v = setl(k_v, p, x0);
                    cap_v = setl(cap_v, p, x1);
                    b_v = setl(b_v, p, x2);
                    dense_v = setl(dense_v, s_last & 63u, p);
                    // index `last` is free now: zero transfer (the lane phase relies on it)
                    k_v = setl(k_v, last, 0u);
                }
                live = r ? live : (1u << last) - 1u;
                if (RM < 16 && in_mem && n == 9 && !r) {  // back to registers: no config holds index 8 or 9
#pragma unroll
                    for (int k = 0; k < RM; ++k) W[k] = m.W[k * 64 + lane];
                    in_mem = false;
                }
                n = r ? n : n - 1;
                peak = nSn > peak ? nSn : peak;
                status = r;
                fev = e;
            }
            T0_PROF_END(evi)
            lim = status ? 0u : lim;
            advance();
            if (n <= 6) break;  // dense indices 0..5: the lane phase's invariant holds
        }
        W0 = W[0];
        dirty = true;  // the dense phase keeps exact sets, not closed ones
    }
#undef T0_PROF_BEGIN
#undef T0_PROF_END
    W[0] = W0;
    if (status == 3) return K_SPILL;
    // per-key epilogue (results through `full`); on a failure W / live still
    // hold the set before the failing event, which is what is reported
    const Args &f = *a.full;

    if (!in_mem) {
#pragma unroll
        for (int k = 0; k < RM; ++k) m.W[k * 64 + lane] = W[k];
    }
    if (!(a.flags & T0_DBG_NOFINAL)) write_final_mem(f, key, m, lane, slot_v, live);
    const uint32_t pr = __ockl_wfred_add_u32(probes);
    if (status)
        finish_key(f, key, status == 1 ? LC_INVALID : LC_UNKNOWN, status == 1 ? LC_CAUSE_NONLIN : LC_CAUSE_BUDGET,
                   (int32_t)fev, peak, pr, (uint64_t)fev + (status == 1 ? 1u : 0u));
    else
        finish_key(f, key, LC_VALID, LC_CAUSE_NONE, -1, peak, pr, nev);
    return K_DONE;
}

// T0 over a work list: one wavefront per key (lattice in 4 registers, or the
// workspace for 9-10 pending ops); a persistent grid so the workspace stays
// one slot per resident block.
#ifdef LC_T0_STAMPS
// Diagnostic build only: per-block clock stamps and hardware placement.
__device__ unsigned long long lc_t0_stamps[8192 * 6];
#endif

// Inclusive XOR prefix over the wave's lanes (DPP row shifts, then the
// row broadcasts across the wave's four rows).
__device__ __forceinline__ uint32_t wave_xor_scan(uint32_t x) {
    x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);  // row_shr:1
    x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);  // row_shr:2
    x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);  // row_shr:4
    x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);  // row_shr:8
    x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return x;
}

// The slot protocol of one 64-event chunk, all slots at once: the events of a
// slot alternate :invoke, :ok, :invoke ... from its state at the chunk's
// start.  Each lane's slot as a one-hot bit over NW 32-bit words, XOR-scanned
// over the lanes: bit s of the exclusive prefix is the parity of slot s's
// earlier events in the chunk, so an event is an :ok exactly when its slot was
// pending at the chunk's start XOR that parity.  pend: the slots pending at
// the chunk's start (NW words, wave-uniform), updated to its end.  Returns
// whether any tracked lane breaks the protocol.
template <int NW>
__device__ __forceinline__ bool slot_protocol(bool tracked, bool ok, uint32_t s, uint32_t (&pend)[NW]) {
    const uint32_t q = s >> 5, bit = 1u << (s & 31u);
    uint32_t par = 0, b = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        const uint32_t oh = (tracked && q == (uint32_t)w) ? bit : 0u;
        const uint32_t x = wave_xor_scan(oh);
        par = q == (uint32_t)w ? (x ^ oh) : par;  // the exclusive prefix of the lane's word
        b = q == (uint32_t)w ? pend[w] : b;
        pend[w] ^= (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
    }
    const bool pending = (((par ^ b) & bit) != 0);
    return __any(tracked && ok != pending);
}

// Validation of a batch the host did not check event by event (T0_STRICT
// steps): a kernel of its own on a second stream, running beside the search
// (which stays in bounds on any input).  One wave per key, 64 events per
// pass: every transition id in range and installing only states the key
// has, every slot below 64, and the slot protocol (slot_protocol: one XOR
// scan per 32 slots and chunk, all slots at once).  Violations set the
// batch's error words (the call then returns LC_E_INVALID).
// GEN (a batch of any width whose events the host did not walk either):
// window slots up to 126, the slot-127 marker of ops beyond the encodable
// window exempt from the slot protocol (the search stops before it follows
// one), and every :invoke's slot below the key's key_width.
// One 64-event chunk of a key's validation (w: lane i holds event i of the
// chunk, in: it is one): transition ids, window slots, the slot protocol.
// Returns the LC_BATCH_E_* reasons found (0: none; pend is then advanced).
template <bool GEN, int NW>
__device__ __forceinline__ int32_t validate_chunk(uint32_t w, bool in, const uint32_t *trp, uint32_t ntr, uint32_t ns,
                                                  uint32_t width, uint32_t (&pend)[NW]) {
    int32_t why = 0;
    const bool ok = (w & LC_EV_OK_BIT) != 0;
    const uint32_t s = LC_EV_SLOT(w), t = LC_EV_TRANS(w);
    const uint32_t d = (in && !ok && t < ntr) ? trp[t] : 0u;
    if (__any(in && !ok && (t >= ntr || ((d & 3u) >= LC_T_WRITE && (d >> 17) >= ns)))) why |= LC_BATCH_E_TRANS;
    const bool beyond = GEN && s == 127u;  // past the encodable window: no slot to track
    if (__any(in && !beyond && (GEN ? (!ok && s >= width) : s >= 64u))) why |= LC_BATCH_E_FIT;
    if (why) return why;
    if (slot_protocol<NW>(in && !beyond, ok, s, pend)) why |= LC_BATCH_E_SLOTS;
    return why;
}

template <bool GEN, bool E16 = false>
__device__ __forceinline__ void validate_key(const T0Args &a, int64_t k) {
    const uint32_t lane = lane_id();
    if (a.key_error && a.key_error[k]) return;
    const uint64_t eb = a.ev_off[k], ee = a.ev_off[k + 1];
    const uint32_t tb = a.trans_off ? a.trans_off[k] : 0u;
    const uint32_t ntr = a.n_trans > tb ? a.n_trans - tb : 0u;
    const uint32_t ns = a.trans_off ? (a.key_states ? a.key_states[k] : 0u) : a.shared_states;
    const uint32_t width = GEN ? (a.key_width ? a.key_width[k] : 127u) : 64u;
    constexpr int NW = GEN ? 4 : 2;
    uint32_t pend[NW];
#pragma unroll
    for (int w = 0; w < NW; ++w) pend[w] = 0;
    int32_t why = 0;
    uint32_t w_next = lane < ee - eb ? (E16 ? LC_EV16_WIDE(a.events16[eb + lane]) : a.events[eb + lane]) : 0u;
    for (uint64_t base = eb; base < ee && !why; base += 64) {
        const uint64_t j = base + lane;
        const bool in = j < ee;
        const uint32_t w = w_next;
        const uint64_t jn = j + 64;
        w_next = jn < ee ? (E16 ? LC_EV16_WIDE(a.events16[jn]) : a.events[jn]) : 0u;  // the next chunk, in flight
        why = validate_chunk<GEN, NW>(w, in, a.trans + (ntr ? tb : 0u), ntr, ns, width, pend);
    }
    if (why && lane == 0) {
        atomicOr(&a.err[0], why);
        atomicMax(&a.err[1], a.err_base + (int32_t)k + 1);
    }
}

template <bool GEN>
__global__ __launch_bounds__(64) void k_validate(T0Args a) {
    for (int64_t k = blockIdx.x; k < a.n_order; k += gridDim.x) validate_key<GEN>(a, k);
}

template <int RM>
__global__ __launch_bounds__(64) void k_search_lattice(T0Args a) {
    __shared__ uint32_t ws[3 * T0_RMEM * 64];  // lattices of 9-10 pending ops (12 KB)

#ifdef LC_T0_STAMPS
    const unsigned long long st0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
    uint32_t nkeys = 0, lastkey = 0;
#endif
#ifdef LC_T0_PROFILE
    if (lane_id() < 12) lc_t0_prof_lds[lane_id()] = 0;
#endif
    const bool fast = !(a.flags & (T0_COUNT | T0_WANT_PEAK | T0_WANT_FINAL)) && a.budget >= 16ull * 64u * 32u;
    for (int32_t guard = 0; guard <= a.n_order; ++guard) {  // every wave takes at most n_order keys
        int32_t w = 0;
        if (lane_id() == 0) w = (int32_t)((uint32_t)atomicAdd(a.ticket, 1) - a.ticket_base);
        w = __builtin_amdgcn_readfirstlane(w);
        if ((uint32_t)w >= (uint32_t)a.n_order) break;
        const int32_t key = a.order[w];
        const int kr = fast ? lattice_key<RM, true>(a, key, ws) : lattice_key<RM, false>(a, key, ws);
        if (kr == K_SPILL) {
            const Args &f = *a.full;
            if (a.flags & T0_STRICT) {  // declared to fit T0, and it does not: no later tier runs
                t0_malformed(a, key, LC_BATCH_E_FIT);
                finish_key(f, key, LC_UNKNOWN, LC_CAUSE_ERROR, -1, 0, 0, 0);
            } else {
                const bool deep = f.deep && a.key_width && a.key_width[key] > LC_DIRECT_T3_WIDTH;
                push_list(deep ? f.deep : f.spill, deep ? f.n_deep : f.n_spill, key, f.list_cap);
            }
        }
#ifdef LC_T0_STAMPS
        ++nkeys;
        lastkey = (uint32_t)key;
#endif
    }
#ifdef LC_T0_PROFILE
    if (lane_id() < 12) atomicAdd(&lc_t0_prof[lane_id()], lc_t0_prof_lds[lane_id()]);
#endif
#ifdef LC_T0_STAMPS
    if (lane_id() == 0 && blockIdx.x < 8192) {
        unsigned long long *o = lc_t0_stamps + blockIdx.x * 6;
        o[0] = st0; o[1] = __builtin_amdgcn_s_memtime(); o[2] = rt0; o[3] = __builtin_amdgcn_s_memrealtime();
        o[4] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4)    // HW_REG_HW_ID
               | ((unsigned long long)lastkey << 32);
        o[5] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) | ((unsigned long long)nkeys << 32);  // XCC_ID
    }
#endif
}

#ifdef LC_T0_STAMPS
extern "C" int lc_debug_t0_stamps(unsigned long long *host, int n_blocks) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(lc_t0_stamps), (size_t)n_blocks * 6 * 8, 0, hipMemcpyDeviceToHost);
}
#endif

size_t lat_ws_words() { return 3 * T0_RMEM * 64; }

// Every block ends with exactly one ticket past the work list, so a launch
// leaves the ticket at ticket_base + n_order + grid: back-to-back launches
// can start from there instead of re-zeroing it.
static T0Args make_t0(const Args &a, const Args *a_dev) {
    T0Args t{};
    t.ev_off = a.ev_off; t.events = a.events; t.trans = a.trans; t.trans_off = a.trans_off;
    t.key_width = a.key_width; t.key_states = a.key_states; t.key_error = a.key_error; t.order = a.order;
    t.ticket = a.ticket;
    t.err = a.err;
    t.err_base = a.err_base;
    t.n_trans = a.n_trans;
    t.lat_ws = a.lat_ws; t.full = a_dev; t.budget = a.budget; t.n_order = a.n_order;
    t.init_state = a.init_state; t.shared_states = a.shared_states;
    t.flags = (a.count_probes ? T0_COUNT : 0u) | (a.peak ? T0_WANT_PEAK : 0u) | (a.final_cfg ? T0_WANT_FINAL : 0u) |
              (a.debug_mode == 2 ? T0_DBG_NOEVENTS : 0u) | (a.debug_mode == 3 ? T0_DBG_NOFINAL : 0u) |
              (a.strict ? T0_STRICT : 0u);
    return t;
}

hipError_t launch_t0(const Args &a, const Args *a_dev, int grid, bool wide, hipStream_t s, uint32_t ticket_base) {
    T0Args t = make_t0(a, a_dev);
    t.ticket_base = ticket_base;
    if (wide) hipLaunchKernelGGL(k_search_lattice<T0_RBIG>, dim3(grid), dim3(64), 0, s, t);
    else hipLaunchKernelGGL(k_search_lattice<T0_RSMALL>, dim3(grid), dim3(64), 0, s, t);
    return hipGetLastError();
}

hipError_t launch_validate(const Args &a, hipStream_t s, bool general) {
    T0Args t{};
    t.ev_off = a.ev_off; t.events = a.events; t.trans = a.trans; t.trans_off = a.trans_off;
    t.key_states = a.key_states; t.key_error = a.key_error; t.err = a.err; t.key_width = a.key_width;
    t.err_base = a.err_base;
    t.n_order = a.n_order; t.shared_states = a.shared_states; t.n_trans = a.n_trans;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(a.n_order, 2048));
    if (general) hipLaunchKernelGGL(k_validate<true>, dim3(grid), dim3(64), 0, s, t);
    else hipLaunchKernelGGL(k_validate<false>, dim3(grid), dim3(64), 0, s, t);
    return hipGetLastError();
}

// ---- Key segments ------------------------------------------------------------
//
// With every key's events strictly serial, a batch of about one key per SIMD
// (C2: 1,000 keys on 1,024 SIMDs) leaves each SIMD one wave whose dependency
// chains are all exposed.  The search distributes over initial states: the
// set after any event, from an initial set S, is the union of the sets
// reached from each s in S.  So a key is cut at quiescent points (no op
// pending: the config set is a plain set of register states) and each
// segment is searched on a wave of its own from every start state at once:
// the lattice word holds one 6-bit group per start state (xfer_tag), valid
// where the key's values are interned as states 1..5 and no op installs nil
// (state 0): a cut is placed only after a write or cas has been invoked
// (and, the point being quiescent, completed), so nil cannot be a start
// state.  Segment 0 starts from the initial state alone and is searched
// untagged.  A per-key composition then walks the segments: the states
// after segment s are the union, over the states standing before it, of
// their groups in its final word; the key dies in the first segment whose
// union is empty, and only that segment is searched again, untagged, from
// the states before it, for the failing event.  Verdicts only (the FAST
// path): no set sizes, probes or final configs.

// Inclusive prefix sum over the wave's lanes, by DPP: Hillis-Steele within
// each row of 16 (row_shr 1, 2, 4, 8), then row_bcast 15 and 31 carry each
// row's total into the rows above it.
__device__ __forceinline__ int32_t wave_scan(int32_t x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, true);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, true);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, true);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, true);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return x;
}

// Cut points of one key per wave: a chunk of 64 events per pass (the next
// chunk's words in flight), the pending count as a wave prefix sum, a cut
// after an event that leaves nothing pending once a write / cas has been
// invoked, at least seg_len events past the previous cut (longer for a key
// that would otherwise need more than max_seg segments).
__global__ __launch_bounds__(64) void k_seg_prep(SegArgs a) {
    const uint32_t lane = lane_id();
    for (int32_t key = blockIdx.x; key < a.n_keys; key += gridDim.x) {
        uint32_t *ends = a.seg_end + (size_t)key * a.max_seg;
        if (a.key_error && a.key_error[key]) {
            if (lane == 0) a.seg_cnt[key] = 0;
            continue;
        }
        const uint64_t eb = a.ev_off[key];
        const uint32_t nev = (uint32_t)(a.ev_off[key + 1] - eb);
        const uint32_t seg_len = max(a.seg_len, (nev + a.max_seg - 2) / (a.max_seg - 1));
        int32_t count = 0;   // ops pending before this chunk
        bool wseen = false;  // a write / cas invoked before this chunk
        uint32_t last = 0, nseg = 0;
        uint32_t w_next = lane < nev ? a.events[eb + lane] : LC_EV_OK_BIT;
        for (uint32_t base = 0; base < nev; base += 64) {
            const uint32_t j = base + lane;
            const bool in = j < nev;
            const uint32_t w = w_next;
            w_next = j + 64 < nev ? a.events[eb + j + 64] : LC_EV_OK_BIT;
            const bool ok = (w & LC_EV_OK_BIT) != 0;
            const uint32_t t = LC_EV_TRANS(w);
            const uint32_t d = (in && !ok && t < a.n_trans) ? a.trans[t] : 0u;
            const int32_t x = wave_scan(in ? (ok ? -1 : 1) : 0);
            const int32_t cnt = count + x;  // ops pending after event j
            const uint64_t wb = __ballot(in && !ok && (d & 3u) >= LC_T_WRITE);
            const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
            const bool wsj = wseen || (wb & upto) != 0;
            uint64_t cand = __ballot(in && cnt == 0 && wsj && j + 1 < nev);
            while (cand && nseg + 1 < a.max_seg) {
                const uint32_t l = (uint32_t)__builtin_ctzll(cand);
                cand &= cand - 1;
                const uint32_t pos = base + l + 1;
                if (pos - last >= seg_len) {
                    if (lane == 0) ends[nseg] = pos;
                    ++nseg;
                    last = pos;
                }
            }
            count = __shfl(cnt, 63);
            wseen = wseen || wb != 0;
        }
        if (lane == 0) {
            ends[nseg] = nev;
            ++nseg;
            a.seg_cnt[key] = nseg;
            const int32_t at = atomicAdd(&a.ctl[0], (int32_t)nseg);
            for (uint32_t s = 0; s < nseg; ++s) a.work[at + (int32_t)s] = ((uint32_t)key << 8) | s;
        }
    }
}

// One segment [sb, se) of a key from the start word `init` (untagged: a
// state mask; tagged: TAG_ID), on the compact lattice with closed sets (the
// register tier's FAST path).  status 0: fin = the OR of every config word
// left (for a quiescent end, lane 0's word); 1: every start died at event
// fev (key-relative); 3: the key does not fit the register tier.
template <bool TAG>
__device__ __forceinline__ void segment_search(const SegArgs &a, int32_t key, uint32_t sb, uint32_t se,
                                               uint32_t init, uint32_t *ws, int &status_out, uint32_t &fev_out,
                                               uint32_t &fin_out) {
    constexpr int RM = T0_RSMALL;
    const uint32_t lane = lane_id();
    const LatMem m{ws, ws + T0_RMEM * 64, ws + 2 * T0_RMEM * 64};
    const uint32_t *const evp = a.events + a.ev_off[key] + sb;
    const uint32_t nev = se - sb;
    const uint32_t ntr = a.n_trans;
    auto ldesc = [&](uint32_t w, bool have) -> uint32_t {
        const uint32_t t = LC_EV_TRANS(w);
        return (have && !(w & LC_EV_OK_BIT) && t < ntr) ? a.trans[t] : 0u;
    };
    auto decode = [](uint32_t d) -> Xfer { return TAG ? xfer_tag(d) : xfer_of(d); };
    uint32_t W[RM];
#pragma unroll
    for (int k = 0; k < RM; ++k) W[k] = 0;
    if (lane == 0) W[0] = init;
    bool in_mem = false;
    uint32_t k_v = 0, cap_v = 0, b_v = 0, m_v = 0;
    uint32_t slot_v = 0, dense_v = 0, n = 0, live = 0;
    uint32_t lm[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) lm[q] = (uint32_t)__builtin_amdgcn_sbfe((int)lane, q, 1);
    int status = 0;
    uint32_t fev = 0;
    uint32_t ev = lane < nev ? evp[lane] : 0u;
    uint32_t dsc = ldesc(ev, lane < nev);
    uint32_t ev_n = 64 + lane < nev ? evp[64 + lane] : 0u;
    uint32_t dsc_n = ldesc(ev_n, 64 + lane < nev);
    uint32_t ev_nn = 128 + lane < nev ? evp[128 + lane] : 0u;
    Xfer xc = decode(dsc);
    uint32_t e = 0, i = 0, base = 0, lim = nev;
    auto advance = [&]() {
        ++e;
        if (++i == 64u) {
            i = 0; base += 64;
            ev = ev_n; dsc = dsc_n; ev_n = ev_nn;
            xc = decode(dsc);
            dsc_n = ldesc(ev_n, base + 64 + lane < nev);
            ev_nn = base + 128 + lane < nev ? evp[base + 128 + lane] : 0u;
        }
    };
    uint32_t W0 = W[0];
    bool dirty = true;
    for (uint32_t phase = 0; phase <= nev && e < lim; ++phase) {
        while (e < lim) {  // lane phase: <= 6 pending
            const uint32_t evi = __builtin_amdgcn_readlane(ev, i);
            const uint32_t slot = LC_EV_SLOT(evi);
            if (!(evi & LC_EV_OK_BIT)) {
                if (n == 6) break;
                if (n >= T0_MAX_WIDTH || slot >= 64) {
                    status = 3;
                } else {
                    const uint32_t idx = (uint32_t)__builtin_ctz(~live);
                    const bool me = lane == idx;
                    slot_v = me ? slot : slot_v;
                    k_v = me ? (uint32_t)__builtin_amdgcn_readlane(xc.k, i) : k_v;
                    cap_v = me ? (uint32_t)__builtin_amdgcn_readlane(xc.cap, i) : cap_v;
                    b_v = me ? (uint32_t)__builtin_amdgcn_readlane(xc.b, i) : b_v;
                    if constexpr (TAG) m_v = me ? (uint32_t)__builtin_amdgcn_readlane(xc.m, i) : m_v;
                    dense_v = lane == slot ? idx : dense_v;
                    live |= 1u << idx;
                    ++n;
                    dirty = true;
                }
            } else {
                const uint32_t p = __builtin_amdgcn_readlane(dense_v, slot & 63u);
                const uint32_t top = 32u - (uint32_t)__builtin_clz(live);
                int r;
                if (top >= 6) r = ok_lane_closed<6, TAG>(W0, p, live, k_v, cap_v, b_v, lane, lm, dirty, m_v);
                else if (top == 5) r = ok_lane_closed<5, TAG>(W0, p, live, k_v, cap_v, b_v, lane, lm, dirty, m_v);
                else r = ok_lane_closed<4, TAG>(W0, p, live, k_v, cap_v, b_v, lane, lm, dirty, m_v);
                dirty = false;
                k_v = setl(k_v, p, 0u);
                live = r ? live : live & ~(1u << p);
                n = r ? n : n - 1;
                status = r;
                fev = e;
            }
            lim = status ? 0u : lim;
            advance();
        }
        if (e >= lim) break;
        W[0] = W0;
#pragma unroll
        for (int k = 1; k < RM; ++k) W[k] = 0u;
        while (e < lim) {  // dense phase: 7-10 pending
            const uint32_t evi = __builtin_amdgcn_readlane(ev, i);
            const uint32_t slot = LC_EV_SLOT(evi);
            if (!(evi & LC_EV_OK_BIT)) {
                if (n >= T0_MAX_WIDTH || slot >= 64) {
                    status = 3;
                } else {
                    if (n == 8) {  // 9 pending: the lattice moves to the workspace
#pragma unroll
                        for (int k = 0; k < T0_RMEM; ++k) m.W[k * 64 + lane] = k < RM ? W[k < RM ? k : 0] : 0u;
                        in_mem = true;
                    }
                    const uint32_t idx = n;
                    const bool me = lane == idx;
                    slot_v = me ? slot : slot_v;
                    k_v = me ? (uint32_t)__builtin_amdgcn_readlane(xc.k, i) : k_v;
                    cap_v = me ? (uint32_t)__builtin_amdgcn_readlane(xc.cap, i) : cap_v;
                    b_v = me ? (uint32_t)__builtin_amdgcn_readlane(xc.b, i) : b_v;
                    if constexpr (TAG) m_v = me ? (uint32_t)__builtin_amdgcn_readlane(xc.m, i) : m_v;
                    dense_v = lane == slot ? idx : dense_v;
                    live |= 1u << idx;
                    ++n;
                }
            } else {
                const uint32_t p = __builtin_amdgcn_readlane(dense_v, slot & 63u);
                uint32_t nSn = 0, probes = 0;
                int r;
                if (n == 7) r = ok_reg<2, RM, TAG>(W, p, k_v, cap_v, b_v, lane, ~0ull, false, probes, nSn, false, m_v);
                else if (n == 8) r = ok_reg<4, RM, TAG>(W, p, k_v, cap_v, b_v, lane, ~0ull, false, probes, nSn, false, m_v);
                else if (n == 9)
                    r = ok_event_mem<8, TAG>(m, p, n, k_v, cap_v, b_v, lane, ~0ull, false, probes, nSn, false, m_v);
                else
                    r = ok_event_mem<16, TAG>(m, p, n, k_v, cap_v, b_v, lane, ~0ull, false, probes, nSn, false, m_v);
                const uint32_t last = n - 1;
                const uint32_t s_last = __builtin_amdgcn_readlane(slot_v, last);
                const uint32_t x0 = __builtin_amdgcn_readlane(k_v, last), x1 = __builtin_amdgcn_readlane(cap_v, last),
                               x2 = __builtin_amdgcn_readlane(b_v, last);
                const uint32_t x3 = TAG ? __builtin_amdgcn_readlane(m_v, last) : 0u;
                const bool mp = lane == p && !r;
                slot_v = mp ? s_last : slot_v;
                k_v = mp ? x0 : k_v;
                cap_v = mp ? x1 : cap_v;
                b_v = mp ? x2 : b_v;
                if constexpr (TAG) m_v = mp ? x3 : m_v;
                dense_v = (lane == s_last && !r) ? p : dense_v;
                k_v = (lane == last && !r) ? 0u : k_v;
                live = r ? live : (1u << last) - 1u;
                if (in_mem && n == 9 && !r) {
#pragma unroll
                    for (int k = 0; k < RM; ++k) W[k] = m.W[k * 64 + lane];
                    in_mem = false;
                }
                n = r ? n : n - 1;
                status = r;
                fev = e;
            }
            lim = status ? 0u : lim;
            advance();
            if (n <= 6) break;
        }
        W0 = W[0];
        dirty = true;
    }
    W[0] = W0;
    uint32_t f = 0;
    if (in_mem) {
#pragma unroll 1
        for (int k = 0; k < T0_RMEM; ++k) f |= m.W[k * 64 + lane];
    } else {
#pragma unroll
        for (int k = 0; k < RM; ++k) f |= W[k];
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) f |= (uint32_t)__shfl_xor((int)f, o);
    status_out = status;
    fev_out = sb + fev;
    fin_out = status ? 0u : f;
}

// Every segment of the work list, one wave each (persistent grid, tickets).
__global__ __launch_bounds__(64) void k_search_segments(SegArgs a) {
    __shared__ uint32_t ws[3 * T0_RMEM * 64];
    const int32_t nwork = a.ctl[0];
    for (int32_t guard = 0; guard <= nwork; ++guard) {
        int32_t w = 0;
        if (lane_id() == 0) w = atomicAdd(&a.ctl[1], 1);
        w = __builtin_amdgcn_readfirstlane(w);
        if (w >= nwork) break;
        const uint32_t item = a.work[w];
        const int32_t key = (int32_t)(item >> 8);
        const uint32_t s = item & 0xFFu;
        const uint32_t *ends = a.seg_end + (size_t)key * a.max_seg;
        const uint32_t sb = s ? ends[s - 1] : 0u, se = ends[s];
        int status;
        uint32_t fev, fin;
        if (s == 0) segment_search<false>(a, key, sb, se, 1u, ws, status, fev, fin);  // from nil (state 0)
        else segment_search<true>(a, key, sb, se, TAG_ID, ws, status, fev, fin);
        if (lane_id() == 0) {
            a.seg_out[(size_t)key * a.max_seg + s] = fin;
            if (s == 0) a.seg0_fev[key] = status == 1 ? (int32_t)fev : -1;
            if (status == 3) {  // declared to fit the register tier, and it does not
                atomicOr(&a.err[0], LC_BATCH_E_FIT);
                atomicMax(&a.err[1], a.err_base + key + 1);
            }
        }
    }
}

// A segmented key's verdict (and its LC_REC_* record when asked for).
__device__ __forceinline__ void seg_verdict(const SegArgs &a, int32_t key, int v, int cause, int32_t fev) {
    a.valid[key] = (int8_t)v; a.cause[key] = (uint8_t)cause; a.fail_event[key] = fev;
    if (a.rec)
        a.rec[key] = (uint64_t)(uint8_t)(v + 1) | (uint64_t)(uint8_t)cause << 8 | (uint64_t)(uint32_t)(fev + 1) << 16;
}

// Per key (one thread each): compose the segments' final words.
__global__ __launch_bounds__(256) void k_seg_compose(SegArgs a) {
    for (int32_t key = blockIdx.x * blockDim.x + threadIdx.x; key < a.n_keys; key += gridDim.x * blockDim.x) {
        if (a.key_error && a.key_error[key]) {
            seg_verdict(a, key, LC_UNKNOWN, LC_CAUSE_ERROR, -1);
            continue;
        }
        const uint32_t n = a.seg_cnt[key];
        const uint32_t *out = a.seg_out + (size_t)key * a.max_seg;
        if (out[0] == 0u) {  // segment 0 is searched from the initial state itself
            seg_verdict(a, key, LC_INVALID, LC_CAUSE_NONLIN, a.seg0_fev[key]);
            continue;
        }
        uint32_t S = (out[0] >> 1) & 0x1Fu;  // state ids 1..5 -> start groups 0..4
        bool dead = false;
        for (uint32_t s = 1; s < n && !dead; ++s) {
            const uint32_t F = out[s];
            uint32_t S2 = 0;
#pragma unroll
            for (uint32_t t = 0; t < 5; ++t)
                if ((S >> t) & 1u) S2 |= (F >> (6u * t)) & 0x1Fu;
            if (!S2) {
                const int32_t at = atomicAdd(&a.ctl[2], 1);
                a.rerun[at] = ((uint32_t)key << 8) | s;
                a.rerun_init[at] = S << 1;  // back to state ids
                dead = true;
            }
            S = S2;
        }
        if (!dead) {
            seg_verdict(a, key, LC_VALID, LC_CAUSE_NONE, -1);
        }
    }
}

// The segment each dead key died in, searched again untagged from the states
// standing before it: the failing event.
__global__ __launch_bounds__(64) void k_seg_rerun(SegArgs a) {
    __shared__ uint32_t ws[3 * T0_RMEM * 64];
    const int32_t nr = a.ctl[2];
    for (int32_t guard = 0; guard <= nr; ++guard) {
        int32_t w = 0;
        if (lane_id() == 0) w = atomicAdd(&a.ctl[3], 1);
        w = __builtin_amdgcn_readfirstlane(w);
        if (w >= nr) break;
        const uint32_t item = a.rerun[w];
        const int32_t key = (int32_t)(item >> 8);
        const uint32_t s = item & 0xFFu;
        const uint32_t *ends = a.seg_end + (size_t)key * a.max_seg;
        int status;
        uint32_t fev, fin;
        segment_search<false>(a, key, ends[s - 1], ends[s], a.rerun_init[w], ws, status, fev, fin);
        if (lane_id() == 0) {
            if (status == 1) {
                seg_verdict(a, key, LC_INVALID, LC_CAUSE_NONLIN, (int32_t)fev);
            } else {  // cannot happen for a consistent batch: report it as malformed
                seg_verdict(a, key, LC_UNKNOWN, LC_CAUSE_ERROR, -1);
                atomicOr(&a.err[0], LC_BATCH_E_FIT);
                atomicMax(&a.err[1], a.err_base + key + 1);
            }
        }
    }
}

hipError_t launch_segments(const SegArgs &a, int grid, hipStream_t s) {
    hipLaunchKernelGGL(k_seg_prep, dim3((unsigned)std::max(1, a.n_keys)), dim3(64), 0, s, a);
    hipLaunchKernelGGL(k_search_segments, dim3((unsigned)grid), dim3(64), 0, s, a);
    hipLaunchKernelGGL(k_seg_compose, dim3((unsigned)std::max(1, (a.n_keys + 255) / 256)), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_seg_rerun, dim3(256), dim3(64), 0, s, a);
    return hipGetLastError();
}

// ---- Speculative key segments -----------------------------------------------
//
// The other way to cut a serial key (no quiescent point needed).  The search
// is monotone: from a larger config set every later set is at least as large.
// So segment s of a key (s >= 1, cut where at most 6 ops are pending) is
// searched from TOP = every register state with every subset of the ops
// pending at the cut linearized -- a superset of the real set there, whatever
// came before.  Runs from different start sets through the same events meet
// quickly (a completed write collapses the register; measured on C2-shaped
// keys with tools/spec_conv.py: within 8 events at the median, 25 at most),
// and once two runs hold equal sets they stay equal.  One workgroup per key,
// one wave per segment:
//   1. every wave searches its segment from TOP (segment 0 from the initial
//      state, exactly), recording the set after the first :ok past cut + ck1
//      and past cut + ck2 (checkpoints), its failing event if it dies, and its
//      set at the segment's end;
//   2. every wave s >= 1 then searches its segment again from the set segment
//      s - 1 ended with, until the two runs meet at a checkpoint.  Inductively
//      every set is then exact: where they meet, the TOP run IS the real run
//      from there on, so its death (or survival) is the segment's;
//   3. wave 0 walks the segments in order: the key fails in the first
//      segment whose real run dies.  A pair of runs that never met (not seen
//      on any measured history) sends the key to the unsegmented search.
// Compared sets are the closed sets the FAST path keeps, taken right after an
// :ok, where they are canonical (ok_lane_closed); both runs of a segment start
// from the same op-index assignment (slot order at the cut), so the
// assignments stay equal event by event.  Verdicts only.
extern "C" __device__ int32_t __ockl_wfred_add_i32(int32_t);
extern "C" __device__ uint32_t __ockl_wfred_min_u32(uint32_t);
extern "C" __device__ uint32_t __ockl_wfred_xor_u32(uint32_t);

constexpr uint32_t SPEC_NONE = 0xFFFFFFFFu;
constexpr uint32_t SPEC_MIN_LEN = 128;  // events per segment at least
constexpr uint32_t SPEC_MAX_PEND = 6;   // ops pending at a cut at most (the lane phase)

// A wave-uniform value the compiler cannot prove uniform (a reduction's
// result, an LDS read): into a scalar register, so control flow on it stays
// scalar (no EXEC masking).
__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ int32_t uni(int32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t uni(uint64_t x) {
    return (uint64_t)uni((uint32_t)x) | ((uint64_t)uni((uint32_t)(x >> 32)) << 32);
}

// Ops invoked minus ops completed over events [b, e) of a key (the change in
// the pending count across them): one ballot pair per 64 events, 8 chunks'
// loads in flight.
template <class EvT>
__device__ __forceinline__ int32_t spec_net(EvT evp, uint32_t b, uint32_t e) {
    constexpr uint32_t G = 8;
    const uint32_t lane = lane_id();
    int32_t cnt = 0;
    for (uint32_t gb = b; gb < e; gb += 64 * G) {
        uint32_t wg[G];
#pragma unroll
        for (uint32_t g = 0; g < G; ++g) {
            const uint32_t j = gb + 64 * g + lane;
            wg[g] = j < e ? evp[j] : 0u;
        }
#pragma unroll
        for (uint32_t g = 0; g < G; ++g) {
            const uint32_t base = gb + 64 * g;
            if (base >= e) continue;
            const bool in = base + lane < e;
            cnt += __popcll(__ballot(in && !(wg[g] >> 31))) - __popcll(__ballot(in && (wg[g] >> 31)));
        }
    }
    return cnt;
}

// Estimated cost of an event, in 1/8 of a lane-phase event: the per-event fit
// of DESIGN.md section 3 (707 cycles per event, +171 per :ok with 7-8 ops
// pending, ~21k per :ok with 9-10 pending -- the last in the LDS workspace).
constexpr uint32_t SPEC_W_EV = 8, SPEC_W_MID = 2, SPEC_W_HEAVY = 240;

// One 64-event chunk's classes (w: lane i holds event base + i; cnt: ops
// pending before the chunk): the lanes that are events, :oks with 7-8 and
// with 9-10 ops pending, each lane's pending count before its event, and the
// chunk's cost.  Pending counts come from two ballots and mbcnt (no scan).
struct ChunkCost {
    uint64_t in, inv, oks, mid, heavy;
    int32_t pend;   // per lane: ops pending before the lane's event
    uint32_t cost;  // the chunk's, uniform
};
__device__ __forceinline__ ChunkCost chunk_cost(uint32_t w, uint32_t base, uint32_t nev, int32_t cnt) {
    const uint32_t lane = lane_id();
    ChunkCost c;
    const bool in = base + lane < nev;
    const bool ok = in && (w >> 31);
    c.in = __ballot(in);
    c.inv = __ballot(in && !ok);
    c.oks = __ballot(ok);
    c.pend = cnt + (int32_t)rank_of(c.inv) - (int32_t)rank_of(c.oks);
    c.mid = __ballot(ok && c.pend >= 7 && c.pend <= 8);
    c.heavy = __ballot(ok && c.pend >= 9);
    c.cost = SPEC_W_EV * (uint32_t)__popcll(c.in) + SPEC_W_MID * (uint32_t)__popcll(c.mid) +
             SPEC_W_HEAVY * (uint32_t)__popcll(c.heavy);
    return c;
}

// Segment boundaries at equal estimated cost: target s (1 .. eff-1) at
// s/eff of the key's total cost (chunk_cost), lane s of pos_v, with the ops
// pending there in lane s of pend_v.  Two passes of ballots over the key's
// events (the total, then the targets), 8 chunks' loads in flight.  A
// segment's walk time is its events plus its 9-10-pending :oks (~30 events'
// time each, 2-5 of them in the slowest walks): equal event counts left the
// slowest of C2's 4,000 walks at 1.65x the median.
template <class EvT>
__device__ __forceinline__ void spec_targets_cost(EvT evp, uint32_t nev, uint32_t eff, uint32_t &pos_v,
                                                  int32_t &pend_v) {
    constexpr uint32_t G = 8;
    const uint32_t lane = lane_id();
    uint32_t total = 0;
    int32_t cnt = 0;
    for (uint32_t gb = 0; gb < nev; gb += 64 * G) {
        uint32_t wg[G];
#pragma unroll
        for (uint32_t g = 0; g < G; ++g) {
            const uint32_t j = gb + 64 * g + lane;
            wg[g] = j < nev ? evp[j] : 0u;
        }
#pragma unroll
        for (uint32_t g = 0; g < G; ++g) {
            const uint32_t base = gb + 64 * g;
            if (base >= nev) continue;
            const ChunkCost c = chunk_cost(wg[g], base, nev, cnt);
            total += c.cost;
            cnt += __popcll(c.inv) - __popcll(c.oks);
        }
    }
    pos_v = 0;
    pend_v = 0;
    uint32_t next = 1, acc = 0;
    uint32_t t_next = (uint32_t)((uint64_t)total / eff);
    cnt = 0;
    for (uint32_t gb = 0; gb < nev && next < eff; gb += 64 * G) {
        uint32_t wg[G];
#pragma unroll
        for (uint32_t g = 0; g < G; ++g) {
            const uint32_t j = gb + 64 * g + lane;
            wg[g] = j < nev ? evp[j] : 0u;
        }
#pragma unroll
        for (uint32_t g = 0; g < G; ++g) {
            const uint32_t base = gb + 64 * g;
            if (base >= nev || next >= eff) continue;
            const ChunkCost c = chunk_cost(wg[g], base, nev, cnt);
            if (acc + c.cost >= t_next) {
                // each lane's cost up to and including its event
                const uint64_t me = 1ull << lane;
                const uint32_t incl = SPEC_W_EV * (rank_of(c.in) + 1u) +
                                      SPEC_W_MID * (rank_of(c.mid) + ((c.mid & me) ? 1u : 0u)) +
                                      SPEC_W_HEAVY * (rank_of(c.heavy) + ((c.heavy & me) ? 1u : 0u));
                const bool in = (c.in & me) != 0;
                while (next < eff && acc + c.cost >= t_next) {
                    const uint64_t hit = __ballot(in && acc + incl >= t_next);
                    const uint32_t l = (uint32_t)__builtin_ctzll(hit);
                    const int32_t at = __builtin_amdgcn_readlane(c.pend, l);
                    pos_v = lane == next ? base + l : pos_v;
                    pend_v = lane == next ? at : pend_v;
                    ++next;
                    t_next = (uint32_t)((uint64_t)total * next / eff);
                }
            }
            acc += c.cost;
            cnt += __popcll(c.inv) - __popcll(c.oks);
        }
    }
}

// The cut for target position t (c_t ops pending there): of the boundaries t
// .. t + 64 (t + i = before event t + i), the one with the fewest ops pending,
// the earliest of those, if that is at most SPEC_MAX_PEND and it lies inside
// the key; else SPEC_NONE.  n_at: ops pending at the cut.
// w: lane i holds event t + i (0 past the key).
__device__ __forceinline__ uint32_t spec_cut_at(uint32_t w, uint32_t nev, uint32_t t, int32_t c_t, uint32_t &n_at) {
    const uint32_t lane = lane_id();
    const uint32_t j = t + lane;  // event j; boundary j + 1 after it
    const int32_t d = j < nev ? 1 - 2 * (int32_t)(w >> 31) : 0;
    const int32_t cnt = c_t + wave_scan(d);
    uint32_t key = (j + 1u < nev && cnt >= 0 && cnt <= (int32_t)SPEC_MAX_PEND) ? ((uint32_t)cnt << 7) | (lane + 1u)
                                                                               : ~0u;
    if (lane == 0 && t < nev && c_t >= 0 && c_t <= (int32_t)SPEC_MAX_PEND) key = min(key, (uint32_t)c_t << 7);
    const uint32_t best = uni(__ockl_wfred_min_u32(key));
    if (best == ~0u) return SPEC_NONE;
    n_at = best >> 7;
    return t + (best & 127u);
}

// The ops pending at boundary c (n expected, n <= 6): each slot is decided by
// its last event before c, walking back.  Returns their :invoke words in slot
// order, word j in lane j; found = how many.
template <class EvT>
__device__ __forceinline__ uint32_t spec_pending(EvT evp, uint32_t c, uint32_t n, uint32_t &found) {
    const uint32_t lane = lane_id();
    uint64_t seen = 0, pm = 0;
    uint32_t byslot = 0;
    found = 0;
    n = min(n, SPEC_MAX_PEND);
    for (uint32_t j = c; found < n && j > 0;) {
        const uint32_t base = j > 64u ? j - 64u : 0u, cnt = j - base;
        const uint32_t w = lane < cnt ? evp[base + lane] : 0u;
        for (int32_t i = (int32_t)cnt - 1; i >= 0 && found < n; --i) {
            const uint32_t wi = __builtin_amdgcn_readlane(w, i);
            const uint32_t sl = LC_EV_SLOT(wi) & 63u;
            if (!((seen >> sl) & 1ull)) {
                seen |= 1ull << sl;
                if (!(wi & LC_EV_OK_BIT)) {
                    pm |= 1ull << sl;
                    byslot = lane == sl ? wi : byslot;
                    ++found;
                }
            }
        }
        j = base;
    }
    uint32_t words = 0;
    for (uint32_t k = 0; k < found; ++k) {
        const uint32_t sl = (uint32_t)__builtin_ctzll(pm);
        pm &= pm - 1;
        const uint32_t wi = __builtin_amdgcn_readlane(byslot, sl);
        words = lane == k ? wi : words;
    }
    return words;
}

// Register-tier state of a walk (the lane phase's registers).
struct SpecState {
    uint32_t W0, k_v, cap_v, b_v, slot_v, dense_v, n, live;
};

// The ops pending at a cut (words in lanes 0 .. n-1, slot order) take op
// indices 0 .. n-1.
__device__ __forceinline__ void spec_setup(SpecState &st, uint32_t words, uint32_t n, const uint32_t *trp,
                                           uint32_t ntr) {
    const uint32_t lane = lane_id();
    const bool me = lane < n;
    const uint32_t t = LC_EV_TRANS(words);
    const Xfer x = xfer_of((me && t < ntr) ? trp[t] : 0u);
    st.k_v = me ? x.k : 0u;
    st.cap_v = me ? x.cap : 0u;
    st.b_v = me ? x.b : 0u;
    st.slot_v = me ? (LC_EV_SLOT(words) & 63u) : 0u;
    st.dense_v = 0;
    for (uint32_t j = 0; j < n; ++j) {
        const uint32_t sl = __builtin_amdgcn_readlane(st.slot_v, j);
        st.dense_v = lane == sl ? j : st.dense_v;
    }
    st.n = n;
    st.live = (1u << n) - 1u;
}

// Events [b, e_end) of a key from st, on the compact lattice with closed sets
// (the register tier's FAST path).  MODE 0 (TOP run): records the set after
// the first lane-phase :ok at or past b + ck1 and past b + ck2 into ck_w /
// ck_e.  MODE 1 (verifying run): compares with them at those events.
// Returns 0 alive at e_end (st: the walk's state there; st.W0 the lattice if
// st.n <= 6), 1 dead at fev, 3 the key does not fit the register tier,
// 4 (MODE 1) met the TOP run, 5 (MODE 1) passed both checkpoints unmet.
// The 9-10-pending workspace: one of the workgroup's NWS LDS slots while one
// is free (busy flags in LDS), else the wave's global slot (an :ok there costs
// ~40k cycles against ~2k in LDS).  NWS = 1, 2, 3 slots for 2, 4, 8 waves
// keep 4 waves per SIMD within the CU's LDS; the 8-wave build held to 8
// waves per SIMD (LC_SPEC8_WAVES) has 2, so that 4 of its workgroups fit.
#ifndef LC_SPEC8_NWS
#define LC_SPEC8_NWS (LC_SPEC8_WAVES >= 8 ? 2 : 3)
#endif
// The 2-wave build keeps no LDS workspace (its 9-10-pending :oks use the
// waves' global ones): 12 KB of LDS per workgroup held it to 5.5 waves per
// SIMD, and the occupancy is worth more to the many-key batches it runs
// than the rare 9-10-pending :ok (LC_SPEC2_WAVES below).
#ifndef LC_SPEC2_NWS
#define LC_SPEC2_NWS 0
#endif
template <int S>
constexpr int spec_lds_ws() { return S <= 2 ? LC_SPEC2_NWS : S <= 3 ? 1 : S <= 6 ? 2 : LC_SPEC8_NWS; }
// Issue priority of a TOP walk by progress (MODE 0, prio): the SIMD's
// arbiter favours the higher s_setprio, then the older wave, so with age
// alone the last-dispatched blocks' walks trail by up to a quarter of a walk
// and end running alone on their SIMDs.  A walk in its first quarter runs at
// priority 3, its last quarter at 0: the four walks a SIMD holds advance
// together and keep it busy to the end.
#ifndef LC_SPEC_PRIO_TOP
#define LC_SPEC_PRIO_TOP 3
#endif
__device__ __forceinline__ void spec_prio(uint32_t quarter) {
    const int lv = LC_SPEC_PRIO_TOP - (int)quarter;
    if (lv >= 3) __builtin_amdgcn_s_setprio(3);
    else if (lv == 2) __builtin_amdgcn_s_setprio(2);
    else if (lv == 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}

// Words of a run's saved set (EX): T0_RMEM lattice rows, the slot of each op
// index (one row), the live op indices.
constexpr uint32_t SPEC_SAVE_WORDS = (T0_RMEM + 2) * 64;

// EX: Knossos's exact sets (ok_lane) instead of closed ones in the lane
// phase, for steps that report final configs; `save` (EX, may be null)
// receives the run's set at its end or before its failing :ok, in the
// LatMem row layout write_final_mem reads, with its slots and live indices.
#ifndef LC_SPEC_CK_SPLIT
#define LC_SPEC_CK_SPLIT 1
#endif
// Checkpoints of a TOP run: at ck1, ck2 and evenly between (a verifying run
// compares its set at each and stops at the first match; one that passes
// them all unmet sends the key to the unsegmented search).  A third one
// between measured no faster in round 5 (C2 0.2472 ms with two, 0.2492
// with three; A/B: make variant VFLAGS=-DLC_SPEC_NCK=n).
#ifndef LC_SPEC_NCK
#define LC_SPEC_NCK 2
#endif
constexpr uint32_t SPEC_NCK = LC_SPEC_NCK;
// With three (a diagnostic build): an early one at ck1 / 4 before them
// (LC_SPEC_CK_EARLY), where most pairs of runs have already met; one that
// has not goes on to ck1 and ck2 as with two.  Measured in round 6
// (profiles/r06_segments_seeds.txt): (8, 32, 120) no faster than (32, 120) on
// C2 or C5.
#ifndef LC_SPEC_CK_EARLY
#define LC_SPEC_CK_EARLY 1
#endif
__device__ __forceinline__ uint32_t spec_ck_target(uint32_t i, uint32_t ck1, uint32_t ck2) {
    if (LC_SPEC_CK_EARLY && SPEC_NCK == 3) return i == 0 ? max(ck1 / 4u, 4u) : i == 1 ? ck1 : ck2;
    return i == 0 ? ck1 : i + 1 >= SPEC_NCK ? ck2 : ck1 + (ck2 - ck1) * i / (SPEC_NCK - 1);
}
// Flags between the waves of one k_spec workgroup (LDS, workgroup scope).  A
// wave publishes after its stores (a release fence for the whole wave, then
// lane 0's store); a waiter polls with an acquire load and sleeps between
// polls, a fixed trip count over a uniform value (the queue loops' rule
// below).  The wait is bounded: a waiter that gives up takes the exact path
// (the key is searched unsegmented), so a timeout costs time, never a result.
constexpr uint32_t SPEC_WAIT_MAX = 1u << 22;
__device__ __forceinline__ void spec_publish(int32_t *f, int32_t v = 1) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane_id() == 0) __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ int32_t spec_load(const int32_t *f) {
    return uni(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ bool spec_wait(const int32_t *f) {
#pragma unroll 1
    for (uint32_t it = 0; it < SPEC_WAIT_MAX; ++it) {
        if (spec_load(f) != 0) return true;
        __builtin_amdgcn_s_sleep(2);
    }
    return false;
}
// A verifying run's checkpoint event i (relative to nothing: the event
// index), read while the TOP run it compares with may still be walking
// (LC_SPEC_OVERLAP): waits until that run has recorded it or has ended
// without it (-1: no such checkpoint); -1 on a timeout too.
__device__ __forceinline__ int32_t spec_ck_event(const int32_t *ck_e, uint32_t i, const int32_t *top_done) {
    if (!top_done) return uni(ck_e[i]);
#pragma unroll 1
    for (uint32_t it = 0; it < SPEC_WAIT_MAX; ++it) {
        const int32_t e = spec_load(ck_e + i);
        if (e >= 0) return e;
        if (spec_load(top_done) != 0) return spec_load(ck_e + i);
        __builtin_amdgcn_s_sleep(2);
    }
    return -1;
}

template <int MODE, int NWS, class EvT, bool EX = false>
__device__ __forceinline__ int spec_walk(EvT evp, const uint32_t *trp, uint32_t ntr, uint32_t b,
                                         uint32_t e_end, SpecState &st, uint32_t *ws, uint32_t *lds_ws,
                                         int32_t *lds_busy, uint32_t (*ck_w)[64], int32_t *ck_e, uint32_t ck1,
                                         uint32_t ck2, uint32_t &fev_out, bool prio = false,
                                         uint32_t *save = nullptr, const int32_t *top_done = nullptr) {
    constexpr int RM = T0_RSMALL;
    const uint32_t lane = lane_id();
    LatMem m{ws, ws + T0_RMEM * 64, ws + 2 * T0_RMEM * 64};
    int32_t held = -1;  // LDS slot held
    const EvT ep = evp + b;
    const uint32_t nev = e_end - b;
    auto ldesc = [&](uint32_t w, bool have) -> uint32_t {
        const uint32_t t = LC_EV_TRANS(w);
        return (have && !(w & LC_EV_OK_BIT) && t < ntr) ? trp[t] : 0u;
    };
    uint32_t W[RM];
#pragma unroll
    for (int k = 0; k < RM; ++k) W[k] = 0;
    bool in_mem = false;
    uint32_t k_v = st.k_v, cap_v = st.cap_v, b_v = st.b_v, slot_v = st.slot_v, dense_v = st.dense_v;
    uint32_t n = st.n, live = st.live;
    uint32_t lm[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) lm[q] = (uint32_t)__builtin_amdgcn_sbfe((int)lane, q, 1);
    int status = 0;
    uint32_t fev = 0;
    uint32_t ev = lane < nev ? ep[lane] : 0u;
    uint32_t dsc = ldesc(ev, lane < nev);
    uint32_t ev_n = 64 + lane < nev ? ep[64 + lane] : 0u;
    uint32_t dsc_n = ldesc(ev_n, 64 + lane < nev);
    uint32_t ev_nn = 128 + lane < nev ? ep[128 + lane] : 0u;
    Xfer xc = xfer_of(dsc);
    uint32_t e = 0, i = 0, base = 0, lim = nev;
    // progress steps of the walk (its priority steps down at each)
#ifndef LC_SPEC_PRIO_STEPS  // diagnostic builds: 1 = at 1/2, 3/4 and 7/8 of the walk
#define LC_SPEC_PRIO_STEPS 0
#endif
#if LC_SPEC_PRIO_STEPS == 1
    const uint32_t q1 = nev / 2u, q2 = nev - nev / 4u, q3 = nev - nev / 8u;
#else
    const uint32_t q1 = nev / 4u, q2 = nev / 2u, q3 = nev - nev / 4u;
#endif
    if (MODE == 0 && prio) spec_prio(0);
    auto advance = [&]() {
        ++e;
        if (++i == 64u) {
            i = 0; base += 64;
            ev = ev_n; dsc = dsc_n; ev_n = ev_nn;
            xc = xfer_of(dsc);
            dsc_n = ldesc(ev_n, base + 64 + lane < nev);
            ev_nn = base + 128 + lane < nev ? ep[base + 128 + lane] : 0u;
            if (MODE == 0 && prio) spec_prio(base >= q3 ? 3u : base >= q2 ? 2u : base >= q1 ? 1u : 0u);
        }
    };
    // next checkpoint (relative event; ~0u: none)
    uint32_t ck_i = 0;
    uint32_t ck_at = ck1;
    if constexpr (MODE != 0) {
        const int32_t e0 = spec_ck_event(ck_e, 0, top_done);
        ck_at = e0 >= 0 ? (uint32_t)e0 - b : ~0u;
    }
    uint32_t W0 = st.W0;
    bool dirty = true;
    // One lane-phase event (<= 6 pending); true: an :invoke with 6 pending,
    // for the dense phase.  CK: the event may be a checkpoint's :ok.  The
    // events before the next checkpoint run the body without that test
    // (LC_SPEC_CK_SPLIT), so the checkpoint words stay out of the hot loop.
    auto lane_event = [&](auto ck_t) -> bool {
        constexpr bool CK = decltype(ck_t)::value;
        const uint32_t evi = __builtin_amdgcn_readlane(ev, i);
        const uint32_t slot = LC_EV_SLOT(evi);
        if (!(evi & LC_EV_OK_BIT)) {
            if (n == 6) return true;
            // (n >= T0_MAX_WIDTH || slot >= 64 as one compare)
            if ((n | (slot & ~63u)) >= T0_MAX_WIDTH) {
                status = 3;
            } else {
                const uint32_t idx = (uint32_t)__builtin_ctz(~live);
                // the op's transfer read out first, then written: no wait
                // states between a v_readlane and the v_writelane of its value
                const uint32_t xk = (uint32_t)__builtin_amdgcn_readlane(xc.k, i),
                               xcap = (uint32_t)__builtin_amdgcn_readlane(xc.cap, i),
                               xb = (uint32_t)__builtin_amdgcn_readlane(xc.b, i);
                slot_v = setl(slot_v, idx, slot);
                k_v = setl(k_v, idx, xk);
                cap_v = setl(cap_v, idx, xcap);
                b_v = setl(b_v, idx, xb);
                dense_v = setl(dense_v, slot, idx);
                live |= 1u << idx;
                ++n;
                dirty = true;
            }
        } else {
            const uint32_t p = __builtin_amdgcn_readlane(dense_v, slot & 63u);
            int r;
            // closed sets: exact ones (ok_lane, as the wide T0 keeps
            // them) measured 10 % slower per event here
            // sweeps specialised to the highest live index (one body for
            // every live set measured 4 % slower per event here)
            const uint32_t top = 32u - (uint32_t)__builtin_clz(live);
            if constexpr (EX) {
                // exact sets: p's transfer, then its lane cleared (as in lattice_key)
                const uint32_t pk = __builtin_amdgcn_readlane(k_v, p), pc = __builtin_amdgcn_readlane(cap_v, p),
                               pb = __builtin_amdgcn_readlane(b_v, p);
                k_v = setl(k_v, p, 0u);
                uint32_t probes = 0, nSn = 0;
                if (top >= 6)
                    r = ok_lane<6>(W0, p, live, k_v, cap_v, b_v, pk, pc, pb, lane, lm, ~0ull, false, probes, nSn,
                                   false);
                else if (top == 5)
                    r = ok_lane<5>(W0, p, live, k_v, cap_v, b_v, pk, pc, pb, lane, lm, ~0ull, false, probes, nSn,
                                   false);
                else
                    r = ok_lane<4>(W0, p, live, k_v, cap_v, b_v, pk, pc, pb, lane, lm, ~0ull, false, probes, nSn,
                                   false);
            } else {
                if (top >= 6) r = ok_lane_closed<6>(W0, p, live, k_v, cap_v, b_v, lane, lm, dirty);
                else if (top == 5) r = ok_lane_closed<5>(W0, p, live, k_v, cap_v, b_v, lane, lm, dirty);
                else r = ok_lane_closed<4>(W0, p, live, k_v, cap_v, b_v, lane, lm, dirty);
                dirty = false;
                k_v = setl(k_v, p, 0u);
            }
            live = r ? live : live & ~(1u << p);
            n = r ? n : n - 1;
            status = r;
            fev = e;
            if (CK && !r && e >= ck_at) {  // a checkpoint (a lane-phase :ok: the set is canonical)
                if constexpr (MODE == 0) {
                    ck_w[ck_i][lane] = W0;
                    spec_publish(&ck_e[ck_i], (int32_t)(b + e));  // (after the set: a verifier may be waiting)
                    ++ck_i;
                    ck_at = ck_i < SPEC_NCK ? max(spec_ck_target(ck_i, ck1, ck2), e + 1u) : ~0u;
                } else {
                    if (!__any(W0 != ck_w[ck_i][lane])) {
                        status = 4;
                    } else {
                        ++ck_i;
                        const int32_t nx = ck_i < SPEC_NCK ? spec_ck_event(ck_e, ck_i, top_done) : -1;
                        ck_at = nx >= 0 ? (uint32_t)nx - b : ~0u;
                        if (ck_i == SPEC_NCK) status = 5;
                    }
                }
            }
        }
        lim = status ? 0u : lim;
        advance();
        return false;
    };
    for (uint32_t phase = 0; phase <= nev && e < lim; ++phase) {
        bool dense = false;
        while (e < lim) {  // lane phase: <= 6 pending
#if LC_SPEC_CK_SPLIT
            uint32_t stop = min(lim, ck_at);
            while (e < stop) {
                if (lane_event(std::false_type{})) { dense = true; break; }
                stop = min(stop, lim);
            }
            if (dense || e >= lim) break;
#endif
            if (lane_event(std::true_type{})) { dense = true; break; }
        }
        (void)dense;
        if (e >= lim) break;
        W[0] = W0;
#pragma unroll
        for (int k = 1; k < RM; ++k) W[k] = 0u;
        while (e < lim) {  // dense phase: 7-10 pending
            const uint32_t evi = __builtin_amdgcn_readlane(ev, i);
            const uint32_t slot = LC_EV_SLOT(evi);
            if (!(evi & LC_EV_OK_BIT)) {
                if (n >= T0_MAX_WIDTH || slot >= 64) {
                    status = 3;
                } else {
                    if (n == 8) {  // 9 pending: the lattice moves to the workspace
                        int32_t got = -1;
                        if (lane == 0) {
                            for (int q = 0; q < NWS && got < 0; ++q)
                                if (atomicCAS(&lds_busy[q], 0, 1) == 0) got = q;
                        }
                        held = uni(got);
                        uint32_t *const mb = held >= 0 ? lds_ws + (size_t)held * (3 * T0_RMEM * 64) : ws;
                        m = LatMem{mb, mb + T0_RMEM * 64, mb + 2 * T0_RMEM * 64};
                        uint32_t *const mW = m.W + opq_lane(lane);
#pragma unroll
                        for (int k = 0; k < T0_RMEM; ++k) mW[k * 64] = k < RM ? W[k < RM ? k : 0] : 0u;
                        in_mem = true;
                    }
                    const uint32_t idx = n;
                    slot_v = setl(slot_v, idx, slot);
                    k_v = setl(k_v, idx, (uint32_t)__builtin_amdgcn_readlane(xc.k, i));
                    cap_v = setl(cap_v, idx, (uint32_t)__builtin_amdgcn_readlane(xc.cap, i));
                    b_v = setl(b_v, idx, (uint32_t)__builtin_amdgcn_readlane(xc.b, i));
                    dense_v = setl(dense_v, slot, idx);
                    live |= 1u << idx;
                    ++n;
                }
            } else {
                const uint32_t p = __builtin_amdgcn_readlane(dense_v, slot & 63u);
                uint32_t nSn = 0, probes = 0;
                int r;
                if (n == 7) r = ok_reg<2, RM>(W, p, k_v, cap_v, b_v, lane, ~0ull, false, probes, nSn, false);
                else if (n == 8) r = ok_reg<4, RM>(W, p, k_v, cap_v, b_v, lane, ~0ull, false, probes, nSn, false);
                else if (n == 9) r = ok_event_mem_gs<8>(m, p, n, k_v, cap_v, b_v, lane);
                else r = ok_event_mem_gs<16>(m, p, n, k_v, cap_v, b_v, lane);
                const uint32_t last = n - 1;
                const uint32_t s_last = __builtin_amdgcn_readlane(slot_v, last);
                const uint32_t x0 = __builtin_amdgcn_readlane(k_v, last), x1 = __builtin_amdgcn_readlane(cap_v, last),
                               x2 = __builtin_amdgcn_readlane(b_v, last);
                if (!r) {
                    slot_v = setl(slot_v, p, s_last);
                    k_v = setl(k_v, p, x0);
                    cap_v = setl(cap_v, p, x1);
                    b_v = setl(b_v, p, x2);
                    dense_v = setl(dense_v, s_last & 63u, p);
                    k_v = setl(k_v, last, 0u);
                }
                live = r ? live : (1u << last) - 1u;
                if (in_mem && n == 9 && !r) {
                    const uint32_t *const mW = m.W + opq_lane(lane);
#pragma unroll
                    for (int k = 0; k < RM; ++k) W[k] = mW[k * 64];
                    in_mem = false;
                    if (held >= 0 && lane == 0) atomicExch(&lds_busy[held], 0);
                    held = -1;
                }
                n = r ? n : n - 1;
                status = r;
                fev = e;
            }
            lim = status ? 0u : lim;
            advance();
            if (n <= 6) break;
        }
        W0 = W[0];
        dirty = true;
    }
    if constexpr (EX) {
        if (save) {
            // the set standing at the end (or before the failing :ok): the
            // dense lattice (registers or the workspace) from 7 ops pending on
            if (n > 6) {
#pragma unroll 1
                for (int k = 0; k < T0_RMEM; ++k) {
                    uint32_t x = 0;
                    if (in_mem) x = m.W[k * 64 + opq_lane(lane)];
                    else {
#pragma unroll
                        for (int q = 0; q < RM; ++q)
                            if (q == k) x = W[q];
                    }
                    save[k * 64 + lane] = x;
                }
            } else {
                save[lane] = W0;
            }
            save[T0_RMEM * 64 + lane] = slot_v;
            if (lane == 0) save[(T0_RMEM + 1) * 64] = live;
        }
    }
    if (held >= 0 && lane == 0) atomicExch(&lds_busy[held], 0);
    if (MODE == 0 && prio) __builtin_amdgcn_s_setprio(0);
    st.W0 = W0;
    st.k_v = k_v; st.cap_v = cap_v; st.b_v = b_v; st.slot_v = slot_v; st.dense_v = dense_v;
    st.n = n; st.live = live;
    fev_out = b + fev;
    return status;
}

#ifdef LC_SPEC_STAMPS
// Diagnostic build only: per (block, wave) clock stamps of the phases.
__device__ unsigned long long lc_spec_stamps[4096 * 8 * 12];
extern "C" int lc_debug_spec_stamps(unsigned long long *host, int n) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(lc_spec_stamps), (size_t)n * 8 * 12 * 8, 0, hipMemcpyDeviceToHost);
}
#define SPEC_STAMP(s, k, v) \
    if (lane == 0 && blk < 4096 && (s) < 8) lc_spec_stamps[((size_t)blk * 8 + (s)) * 12 + (k)] = (v);
#else
#define SPEC_STAMP(s, k, v)
#endif

// Checked builds only (LC_SPEC_CHECK_UNIFORM): a queue index that is not
// wave-uniform refuses the batch instead of walking on a divergent index.
#ifdef LC_SPEC_CHECK_UNIFORM
#define SPEC_CHECK_UNIFORM(x)                                                        \
    if (__any((x) != (uint32_t)__builtin_amdgcn_readfirstlane(x)) && lane == 0) {  \
        atomicOr(&a.err[0], (int32_t)LC_BATCH_E_FIT);                              \
        atomicMax(&a.err[1], a.err_base + key + 1);                                \
    }
#else
#define SPEC_CHECK_UNIFORM(x)
#endif

// One workgroup of W waves per key (blockIdx = LPT position), the key cut into
// up to S segments; the waves take the segments' TOP walks, then their
// verifying runs, from two block-local queues (launched with S = W: more
// segments than waves, a wave taking another walk instead of waiting at the
// barrier for the slowest, measured slower -- every extra cut costs a
// verifying run and a walk's start-up).  Results go through a.full like
// T0's; a.lat_ws holds each wave's 9-10-pending fallback workspace (global
// memory: the workgroup's LDS workspaces are shared, NWS of them).
// 16-bit event words of a key k_spec stages in LDS: none for 2-segment
// workgroups (the many-key batches, where 6 KB more per block would cost
// occupancy), 4,096 (8 KB) otherwise -- C2's keys have ~1,470.  (The 8-wave
// build's 4 workgroups per CU, 8 waves per SIMD, fit the CU's 160 KB with
// these and 2 checkpoint sets per segment; a third set needs 3,072 here.)
template <int S, bool E16>
constexpr uint32_t spec_ev_lds() { return (E16 && S > 2) ? (S >= 8 && SPEC_NCK > 2 ? 3072u : 4096u) : 0u; }

#ifndef LC_SPEC_KARG
#define LC_SPEC_KARG 1
#endif
// The 2-wave build (the many-key batches: C3's shards, throughput-bound) is
// held to 8 waves per SIMD: 64 VGPRs, 140 B per lane spilled to scratch, and
// no LDS workspace (LC_SPEC2_NWS) so that 8 fit.  A/B on one box, the C3
// shard (12,500 x 2,000), two rounds each (round 5): 6 waves per SIMD with
// the LDS workspace (5.5 resident) 3.881 ms per step, kernel 3.694; 6
// without it 3.814 / 3.650; 7 3.607 / 3.421; 8 3.601 / 3.427.  Records
// identical.  (Before: 84 VGPRs, 4 waves, 4.04 ms per step.)
#ifndef LC_SPEC2_WAVES
#define LC_SPEC2_WAVES 8
#endif
template <int S, int W, bool E16, bool EX = false>
__global__ __launch_bounds__(64 * W, (W == 2 ? LC_SPEC2_WAVES : W == 8 ? LC_SPEC8_WAVES : 1)) void k_spec(T0Args a) {
#if LC_SPEC_KARG
#define KA t0k()
#else
#define KA a
#endif
    constexpr uint32_t EVC = spec_ev_lds<S, E16>();
    __shared__ uint16_t s_ev[EVC ? EVC : 1];  // the key's event words (EvStaged)
    __shared__ uint32_t s_end[S][64];     // TOP run's set at the segment's end
    __shared__ uint32_t s_ck[S][SPEC_NCK][64];  // TOP run's checkpoint sets
    __shared__ uint32_t s_pend[S][8];     // ops pending at the cut ([0..5] words, [6] count)
    __shared__ uint64_t s_map[S];         // end: byte i = 0x80 | slot of live op index i
    __shared__ int32_t s_ck_e[S][SPEC_NCK];  // checkpoint events (-1: none)
    __shared__ int32_t s_cut[S], s_segend[S];  // segment [cut, end); cut -1: no segment
    __shared__ int32_t s_top[S];          // TOP run: -1 alive, -2 does not fit, -3 lost, else its failing event
    __shared__ int32_t s_ver[S], s_vfev[S];
    __shared__ int32_t s_net[S];          // cut search: pending-count change over each part
    __shared__ int32_t s_cand[S], s_ncand[S];  // each target's cut (-1: none) and ops pending there
    __shared__ int32_t s_next[2];         // the block's queues: TOP walks, verifying runs
    __shared__ int32_t s_prdy[S], s_done[S];  // LC_SPEC_OVERLAP: s_pend / s_top -3 of s out; TOP run of s ended
    __shared__ uint32_t s_vx[W][2];       // self-validation: each wave's part, XOR of its slots' one-hots
    constexpr int NWS = spec_lds_ws<W>();
    __shared__ uint32_t s_ws[NWS ? NWS * 3 * T0_RMEM * 64 : 1];  // 9-10-pending workspaces (12 KB each)
    __shared__ int32_t s_ws_busy[NWS ? NWS : 1];
    const uint32_t lane = lane_id(), wv = uni((uint32_t)threadIdx.x >> 6);  // uniform per wave
    // T0_STRICT steps: the event-by-event validation, in nb blocks after the
    // keys' (no second stream, no cross-stream waits around the step), or
    // before them (T0_SPEC_VFIRST)
    const uint32_t nb = gridDim.x - (uint32_t)KA.n_order;
    const bool vfirst = (KA.flags & T0_SPEC_VFIRST) != 0;
    const uint32_t blk = vfirst ? blockIdx.x - nb : blockIdx.x;  // the key block's LPT position
    if (vfirst ? blockIdx.x < nb : blockIdx.x >= (uint32_t)KA.n_order) {
        const uint32_t vb = vfirst ? blockIdx.x : blockIdx.x - (uint32_t)KA.n_order;
        for (int64_t k = (int64_t)vb * W + wv; k < KA.n_order; k += (int64_t)nb * W) {
            // (a key whose words its own block stages whole is validated
            // there, from LDS: see below)
            if (EVC > 0 && !(KA.flags & T0_SPEC_NOSTAGE) && KA.ev_off[k + 1] - KA.ev_off[k] <= EVC) continue;
            validate_key<false, E16>(a, k);
        }
        return;  // the whole block: no barrier below is reached by half of it
    }
    // The block's set-up -- staging, validation, the cuts -- at a TOP walk's
    // first-quarter issue priority (LC_SPEC_CUT_PRIO=1, A/B): measured in
    // round 6 at -0.3 % on C2 / C5 and other seeds (tools/gpu_r6n.sh,
    // profiles/r06_segments_seeds.txt), within noise; not the default.
#ifndef LC_SPEC_CUT_PRIO
#define LC_SPEC_CUT_PRIO 0
#endif
    if (LC_SPEC_CUT_PRIO && !(KA.flags & T0_SPEC_NOPRIO)) __builtin_amdgcn_s_setprio(3);
    // (scalar: as a VGPR it was the 64-VGPR builds' last spill to scratch)
    const int32_t key = (int32_t)uni((uint32_t)KA.order[blk]);
    uint32_t *ws = KA.lat_ws + ((size_t)blk * W + wv) * (3 * T0_RMEM * 64);
    const uint64_t eb = KA.ev_off[key];
    const uint32_t nev = (uint32_t)(KA.ev_off[key + 1] - eb);
    // the key's words: staged in LDS (8 loads in flight per thread, then the
    // stores; made visible by the barrier below), else read from HBM
    uint32_t n_lds = 0;
    if constexpr (EVC > 0) {
        if (!(KA.flags & T0_SPEC_NOSTAGE)) {
            n_lds = nev < EVC ? nev : EVC;
            const uint16_t *g = KA.events16 + eb;
            for (uint32_t base = 0; base < n_lds; base += 64u * W * 8u) {
                uint16_t v[8];
#pragma unroll
                for (uint32_t q = 0; q < 8; ++q) {
                    const uint32_t j = base + q * 64u * W + threadIdx.x;
                    v[q] = j < n_lds ? g[j] : (uint16_t)0;
                }
#pragma unroll
                for (uint32_t q = 0; q < 8; ++q) {
                    const uint32_t j = base + q * 64u * W + threadIdx.x;
                    if (j < n_lds) s_ev[j] = v[q];
                }
            }
        }
    }
    using EvK = typename std::conditional<(EVC > 0), EvStaged, EvSrc<E16>>::type;
    EvK evp;
    if constexpr (EVC > 0) evp = EvStaged{(LdsU16 *)s_ev, KA.events16 + eb, n_lds};
    else evp = ev_src<E16>(KA) + eb;
    const uint32_t tb = KA.trans_off ? KA.trans_off[key] : 0u;
    const uint32_t ntr = KA.n_trans > tb ? KA.n_trans - tb : 0u;
    const uint32_t *const trp = KA.trans + (ntr ? tb : 0u);
    const uint32_t nstates = KA.trans_off ? (KA.key_states ? KA.key_states[key] : 0xFFFFu) : KA.shared_states;
    const uint32_t width = KA.key_width ? KA.key_width[key] : 0xFFu;
    // keys for the unsegmented search: errors, keys outside the tier (it
    // reports them), and keys too short to cut
    const bool plain = (KA.key_error && KA.key_error[key]) || nstates > T0_MAX_STATES || nstates == 0 ||
                       width > T0_MAX_WIDTH || KA.init_state >= T0_MAX_STATES || nev < 2 * SPEC_MIN_LEN;
    const uint32_t eff = plain ? 1u : min((uint32_t)S, nev / SPEC_MIN_LEN);
    const uint32_t topmask = nstates >= 32 ? ~0u : (1u << nstates) - 1u;

    if (threadIdx.x < NWS) s_ws_busy[threadIdx.x] = 0;
    if (threadIdx.x < 2) s_next[threadIdx.x] = 0;
    __syncthreads();
    // T0_STRICT batches whose key the block staged whole: the key's
    // validation here, from LDS, its 64-event chunks split over the W waves
    // (the slot protocol's state at a wave's first chunk is the XOR of the
    // earlier waves' slot parities, exchanged at the cut search's barrier),
    // instead of a second HBM read of the words in the validation blocks.
    bool self_val = false;
    uint32_t vc0 = 0, vc1 = 0;
    if constexpr (EVC > 0) {
        self_val = (KA.flags & T0_STRICT) && !(KA.flags & T0_SPEC_NOSTAGE) && n_lds == nev &&
                   !(KA.key_error && KA.key_error[key]);
        const uint32_t nch = (nev + 63u) / 64u;
        vc0 = nch * wv / W;
        vc1 = nch * (wv + 1u) / W;
        if (self_val) {
            uint32_t x0 = 0, x1 = 0;
            for (uint32_t ch = vc0; ch < vc1; ++ch) {
                const uint32_t j = ch * 64u + lane;
                if (j < nev) {
                    const uint32_t sl = LC_EV_SLOT(LC_EV16_WIDE(s_ev[j]));
                    x0 ^= sl < 32u ? 1u << sl : 0u;
                    x1 ^= (sl >= 32u && sl < 64u) ? 1u << (sl - 32u) : 0u;
                }
            }
            x0 = uni(__ockl_wfred_xor_u32(x0));
            x1 = uni(__ockl_wfred_xor_u32(x1));
            if (lane == 0) { s_vx[wv][0] = x0; s_vx[wv][1] = x1; }
        }
    }
    if (wv == 0) {
        for (uint32_t s = 0; s < (uint32_t)S; ++s) { SPEC_STAMP(s, 0, __builtin_amdgcn_s_memtime()) }
    }
    // 0. the cuts.  Targets at s/eff of the key's events (T0_SPEC_COST: of its
    // estimated cost, each wave computing every target); each moved to the
    // boundary with the fewest ops pending within 64 events.  Equal event
    // counts: the waves count the pending-count change over the parts
    // [t_p, t_p+1) (part p on wave p mod W), the parts' prefix gives the count
    // at each target, and the waves place the cuts likewise -- two barriers.
    const bool cost = (KA.flags & T0_SPEC_COST) != 0;
    if (!plain && !cost) {
        for (uint32_t p = wv; p + 1 < eff; p += W) {
            const uint32_t t0 = (uint32_t)((uint64_t)nev * p / eff), t1 = (uint32_t)((uint64_t)nev * (p + 1) / eff);
            const int32_t d = spec_net(evp, t0, t1);
            if (lane == 0) s_net[p] = d;
        }
    }
    __syncthreads();
    if constexpr (EVC > 0) {
        if (self_val) {
            // (the states a transition may install: as validate_key reads them)
            const uint32_t vns = KA.trans_off ? (KA.key_states ? KA.key_states[key] : 0u) : KA.shared_states;
            uint32_t pend[2] = {0u, 0u};
            for (uint32_t q = 0; q < wv; ++q) { pend[0] ^= uni(s_vx[q][0]); pend[1] ^= uni(s_vx[q][1]); }
            int32_t why = 0;
            for (uint32_t ch = vc0; ch < vc1 && !why; ++ch) {
                const uint32_t j = ch * 64u + lane;
                const bool in = j < nev;
                const uint32_t w = in ? LC_EV16_WIDE(s_ev[j]) : 0u;
                why = validate_chunk<false, 2>(w, in, trp, ntr, vns, 64u, pend);
            }
            if (why && lane == 0) {
                atomicOr(&KA.err[0], why);
                atomicMax(&KA.err[1], KA.err_base + key + 1);
            }
        }
    }
    if (!plain && !cost) {
        for (uint32_t s = wv; s < eff; s += W) {
            if (s == 0) continue;
            int32_t pend = 0;
            for (uint32_t q = 0; q < s; ++q) pend += uni(s_net[q]);
            const uint32_t t = (uint32_t)((uint64_t)nev * s / eff);
            const uint32_t w = t + lane < nev ? evp[t + lane] : 0u;
            uint32_t n2 = 0;
            const uint32_t c2 = spec_cut_at(w, nev, t, pend, n2);
            if (lane == 0) {
                s_cand[s] = c2 == SPEC_NONE ? -1 : (int32_t)c2;
                s_ncand[s] = (int32_t)n2;
            }
        }
    }
    if (!plain && cost && wv < eff) {
        uint32_t pos_v;
        int32_t pend_v;
        spec_targets_cost(evp, nev, eff, pos_v, pend_v);
        for (uint32_t s = wv; s < eff; s += W) {  // every wave has every target: each places its own cuts
            if (s == 0) continue;
            const uint32_t t = uni(__builtin_amdgcn_readlane(pos_v, s));
            const uint32_t w = t + lane < nev ? evp[t + lane] : 0u;
            uint32_t n2 = 0;
            const uint32_t c2 = spec_cut_at(w, nev, t, uni(__builtin_amdgcn_readlane(pend_v, s)), n2);
            if (lane == 0) {
                s_cand[s] = c2 == SPEC_NONE ? -1 : (int32_t)c2;
                s_ncand[s] = (int32_t)n2;
            }
        }
    }
    __syncthreads();
    // the kept cuts (each past the last kept one; a segment ends at the next
    // kept cut), by one thread
    if (threadIdx.x == 0 && !plain) {
        int32_t last = 0;
        s_cut[0] = 0;
        for (uint32_t s = 1; s < eff; ++s) {
            int32_t c2 = s_cand[s];
            if (c2 >= 0 && c2 <= last) c2 = -1;
            if (c2 >= 0) last = c2;
            s_cut[s] = c2;
        }
        int32_t end = (int32_t)nev;
        for (uint32_t s = eff; s-- > 0;) {
            s_segend[s] = end;
            if (s_cut[s] >= 0) end = s_cut[s];
            for (uint32_t q = 0; q < SPEC_NCK; ++q) s_ck_e[s][q] = -1;
            s_top[s] = -1;
        }
        for (uint32_t s = 0; s < (uint32_t)S; ++s) {
            s_prdy[s] = 0;
            s_done[s] = 0;
            s_ver[s] = 0;
            s_vfev[s] = -1;
        }
    }
    __syncthreads();
#ifndef LC_SPEC_OVERLAP
#define LC_SPEC_OVERLAP 1
#endif
    if constexpr (LC_SPEC_OVERLAP && S == W) {
        // 1 + 2, overlapped (LC_SPEC_OVERLAP): wave w walks segment w from
        // TOP, then at once verifies the next kept segment from the set its
        // own walk ended with -- without waiting at a barrier for every TOP
        // walk of the block.  The verifying run compares with that segment's
        // TOP run at its checkpoints, which that run publishes as it passes
        // them (spec_ck_event waits for one not reached yet), and with its end
        // set once it has ended.  A block then takes about its slowest TOP
        // walk, not its slowest TOP walk plus its slowest verifying run.
        if (!plain) {
            const uint32_t s = wv;
            const bool kept = s < eff && uni(s_cut[s]) >= 0;
            int32_t top_s = -1;
            if (kept) {
                const int32_t cut_i = uni(s_cut[s]);
                const uint32_t cut = (uint32_t)cut_i, end = (uint32_t)uni(s_segend[s]);
                const uint32_t n0 = s == 0 ? 0u : (uint32_t)uni(s_ncand[s]);
                SPEC_STAMP(s, 1, __builtin_amdgcn_s_memtime())
                SPEC_STAMP(s, 6, ((unsigned long long)end << 32) | cut)
                SPEC_STAMP(s, 8, (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
                                     ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32))
                SPEC_STAMP(s, 9, (unsigned long long)key)
                SpecState st{};
                uint32_t words = 0, np = 0;
                if (s == 0) {
                    st.W0 = lane == 0 ? 1u << KA.init_state : 0u;
                } else {
                    words = spec_pending(evp, cut, n0, np);
                    spec_setup(st, words, np, trp, ntr);
                    st.W0 = lane < (1u << np) ? topmask : 0u;
                }
                if (lane < 6) s_pend[s][lane] = words;
                if (lane == 6) s_pend[s][6] = np;
                const bool lost = s != 0 && np != n0;
                if (lost && lane == 0) s_top[s] = -3;
                spec_publish(&s_prdy[s]);
                uint32_t fev = 0;
                uint32_t *const sv = EX ? KA.spec_fin + ((size_t)blk * S + s) * 2 * SPEC_SAVE_WORDS : nullptr;
                const int r = lost ? 6
                                   : spec_walk<0, NWS, EvK, EX>(evp, trp, ntr, cut, end, st, ws, s_ws, s_ws_busy,
                                                                       s_ck[s], s_ck_e[s], KA.spec_ck1, KA.spec_ck2,
                                                                       fev, !(KA.flags & T0_SPEC_NOPRIO), sv);
                s_end[s][lane] = st.W0;
                uint64_t map = 0;
                for (uint32_t q = 0; q < 6; ++q) {
                    const uint32_t sl = __builtin_amdgcn_readlane(st.slot_v, q);
                    if ((st.live >> q) & 1u) map |= (uint64_t)(0x80u | sl) << (8 * q);
                }
                SPEC_STAMP(s, 2, __builtin_amdgcn_s_memtime())
                top_s = r == 1 ? (int32_t)fev : r == 3 ? -2 : r == 6 ? -3 : -1;
                if (lane == 0) {
                    s_map[s] = map;
                    s_top[s] = top_s;
                }
                spec_publish(&s_done[s]);
            }
            // the next kept segment (its predecessor is this one)
            uint32_t v = s + 1;
            while (v < eff && uni(s_cut[v]) < 0) ++v;
            if (kept && top_s == -1 && v < eff) {
                SPEC_STAMP(v, 3, __builtin_amdgcn_s_memtime())
                int32_t ver = 3, vfev = -1;  // (a wait that gives up: the key goes unsegmented)
                uint32_t fev = 0;
                if (spec_wait(&s_prdy[v]) && spec_load(&s_top[v]) != -3) {
                    const uint32_t cut = (uint32_t)uni(s_cut[v]), end = (uint32_t)uni(s_segend[v]);
                    const uint32_t np = uni(s_pend[v][6]);
                    SpecState st{};
                    spec_setup(st, lane < 6 ? s_pend[v][lane] : 0u, np, trp, ntr);
                    // this walk's end set, relabelled from its op indices to v's
                    const uint64_t map = uni(s_map[s]);
                    uint32_t src = 0;
                    for (uint32_t j = 0; j < np; ++j) {
                        const uint32_t sl = __builtin_amdgcn_readlane(st.slot_v, j);
                        uint32_t at = 31;
                        for (uint32_t q = 0; q < 6; ++q)
                            if (((map >> (8 * q)) & 0xFFu) == (0x80u | sl)) at = q;
                        src |= ((lane >> j) & 1u) << at;
                    }
                    const uint32_t E = (uint32_t)__shfl((int)s_end[s][lane], (int)(src & 63u));
                    st.W0 = lane < (1u << np) ? E : 0u;
                    uint32_t *const sv =
                        EX ? KA.spec_fin + ((size_t)blk * S + v) * 2 * SPEC_SAVE_WORDS + SPEC_SAVE_WORDS : nullptr;
// (issue priority of the verifying runs: 0; 2 and 3 measured slower on
// C2 and most seeds in round 6, profiles/r06_segments_seeds.txt)
#ifndef LC_SPEC_VER_PRIO
#define LC_SPEC_VER_PRIO 0
#endif
                    if (LC_SPEC_VER_PRIO) __builtin_amdgcn_s_setprio(LC_SPEC_VER_PRIO);
                    const int r = spec_walk<1, NWS, EvK, EX>(evp, trp, ntr, cut, end, st, ws, s_ws, s_ws_busy,
                                                                    s_ck[v], s_ck_e[v], 0, 0, fev, false, sv,
                                                                    &s_done[v]);
                    if (LC_SPEC_VER_PRIO) __builtin_amdgcn_s_setprio(0);
                    bool last = true;
                    for (uint32_t q = v + 1; q < eff; ++q) last = last && uni(s_cut[q]) < 0;
                    if (r == 4) ver = 1;                        // met the TOP run
                    else if (r == 1) { ver = 2; vfev = (int32_t)fev; }  // died before meeting it
                    else if (r == 3) ver = 6;                   // does not fit
                    else if (r == 5) ver = 3;                   // never met
                    else if (last) ver = 5;                     // the last segment, searched exactly to its end
                    else if (spec_wait(&s_done[v])) ver = (st.n <= 6 && !__any(st.W0 != s_end[v][lane])) ? 1 : 3;
                }
                SPEC_STAMP(v, 7, ((unsigned long long)ver << 32) | (fev - (uint32_t)uni(s_cut[v])))
                SPEC_STAMP(v, 4, __builtin_amdgcn_s_memtime())
                if (lane == 0) {
                    s_ver[v] = ver;
                    s_vfev[v] = vfev;
                }
            }
        }
    } else {
    // 1. every segment from TOP (segment 0 exactly), from the block's queue.
    // INVARIANT (both queue loops below): a fixed trip count (S, S - 1) and a
    // queue index made wave-uniform by uni() before any branch on it.  With
    // `for (;;) ... break` the compiler built an exec-masked loop whose exit
    // hung the wave after its first walk (round 3).  tests/test_pack.py::
    // test_spec_queue_loops_keep_fixed_trip_counts checks the shape of these
    // loops in this file; the LC_SPEC_CHECK_UNIFORM build (make variant
    // NAME=specchk VFLAGS=-DLC_SPEC_CHECK_UNIFORM) also checks at run time that
    // the index is uniform, refusing the batch (LC_BATCH_E_FIT) if it is not.
    if (!plain) {
#pragma unroll 1
        for (uint32_t k = 0; k < (uint32_t)S; ++k) {
            uint32_t s = 0;
            if (lane == 0) s = (uint32_t)atomicAdd(&s_next[0], 1);
            s = uni(s);
            SPEC_CHECK_UNIFORM(s);
            if (s >= eff || uni(s_cut[s]) < 0) continue;
            const int32_t cut_i = uni(s_cut[s]);
            const uint32_t cut = (uint32_t)cut_i, end = (uint32_t)uni(s_segend[s]);
            const uint32_t n0 = s == 0 ? 0u : (uint32_t)uni(s_ncand[s]);
            SPEC_STAMP(s, 1, __builtin_amdgcn_s_memtime())
            SPEC_STAMP(s, 6, ((unsigned long long)end << 32) | cut)
            SPEC_STAMP(s, 8, (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
                                 ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32))
            SPEC_STAMP(s, 9, (unsigned long long)key)
            SpecState st{};
            uint32_t words = 0, np = 0;
            if (s == 0) {
                st.W0 = lane == 0 ? 1u << KA.init_state : 0u;
            } else {
                words = spec_pending(evp, cut, n0, np);
                spec_setup(st, words, np, trp, ntr);
                st.W0 = lane < (1u << np) ? topmask : 0u;
            }
            if (lane < 6) s_pend[s][lane] = words;
            if (lane == 6) s_pend[s][6] = np;
            uint32_t fev = 0;
            // the ops found pending must be as many as the count says (else
            // the event stream is malformed): the key is searched unsegmented
            const bool lost = s != 0 && np != n0;
            uint32_t *const sv = EX ? KA.spec_fin + ((size_t)blk * S + s) * 2 * SPEC_SAVE_WORDS : nullptr;
            const int r = lost ? 6
                               : spec_walk<0, NWS, EvK, EX>(evp, trp, ntr, cut, end, st, ws, s_ws, s_ws_busy,
                                                                   s_ck[s], s_ck_e[s], KA.spec_ck1, KA.spec_ck2, fev,
                                                                   !(KA.flags & T0_SPEC_NOPRIO), sv);
            s_end[s][lane] = st.W0;
            uint64_t map = 0;
            for (uint32_t q = 0; q < 6; ++q) {
                const uint32_t sl = __builtin_amdgcn_readlane(st.slot_v, q);
                if ((st.live >> q) & 1u) map |= (uint64_t)(0x80u | sl) << (8 * q);
            }
            SPEC_STAMP(s, 2, __builtin_amdgcn_s_memtime())
            if (lane == 0) {
                s_map[s] = map;
                s_top[s] = r == 1 ? (int32_t)fev : r == 3 ? -2 : r == 6 ? -3 : -1;
            }
        }
    }
    __syncthreads();
    // 2. every segment s >= 1 again, from the set segment s - 1 ended with,
    // until the runs meet (from the block's second queue)
    if (!plain) {
#pragma unroll 1
        for (uint32_t k = 1; k < (uint32_t)S; ++k) {
            uint32_t s = 0;
            if (lane == 0) s = (uint32_t)atomicAdd(&s_next[1], 1) + 1u;
            s = uni(s);
            SPEC_CHECK_UNIFORM(s);
            if (s >= eff || uni(s_cut[s]) < 0 || uni(s_top[s]) == -3) continue;
            SPEC_STAMP(s, 3, __builtin_amdgcn_s_memtime())
            uint32_t pw = s - 1;
            while (uni(s_cut[pw]) < 0) --pw;  // s_cut[0] = 0
            int32_t ver = 0, vfev = -1;
            if (uni(s_top[pw]) == -1) {
                const uint32_t cut = (uint32_t)uni(s_cut[s]), end = (uint32_t)uni(s_segend[s]);
                const uint32_t np = uni(s_pend[s][6]);
                SpecState st{};
                spec_setup(st, lane < 6 ? s_pend[s][lane] : 0u, np, trp, ntr);
                // the predecessor's end set, relabelled from its op indices to these
                const uint64_t map = uni(s_map[pw]);
                uint32_t src = 0;
                for (uint32_t j = 0; j < np; ++j) {
                    const uint32_t sl = __builtin_amdgcn_readlane(st.slot_v, j);
                    uint32_t at = 31;
                    for (uint32_t q = 0; q < 6; ++q)
                        if (((map >> (8 * q)) & 0xFFu) == (0x80u | sl)) at = q;
                    src |= ((lane >> j) & 1u) << at;
                }
                const uint32_t E = (uint32_t)__shfl((int)s_end[pw][lane], (int)(src & 63u));
                st.W0 = lane < (1u << np) ? E : 0u;
                uint32_t fev = 0;
                uint32_t *const sv =
                    EX ? KA.spec_fin + ((size_t)blk * S + s) * 2 * SPEC_SAVE_WORDS + SPEC_SAVE_WORDS : nullptr;
                // (the verifying runs at a TOP walk's highest issue priority,
                // against the other blocks' TOP walks on the SIMD, measured
                // slower in round 5: C2 0.2484 -> 0.2501, C5 0.2997 -> 0.3068)
                const int r = spec_walk<1, NWS, EvK, EX>(evp, trp, ntr, cut, end, st, ws, s_ws, s_ws_busy,
                                                                s_ck[s], s_ck_e[s], 0, 0, fev, false, sv);
                bool last = true;
                for (uint32_t q = s + 1; q < eff; ++q) last = last && uni(s_cut[q]) < 0;
                if (r == 4) ver = 1;                        // met the TOP run
                else if (r == 1) { ver = 2; vfev = (int32_t)fev; }  // died before meeting it
                else if (r == 3) ver = 6;                   // does not fit
                else if (r == 5) ver = 3;                   // never met
                else if (last) ver = 5;                     // the last segment, searched exactly to its end
                else ver = (st.n <= 6 && !__any(st.W0 != s_end[s][lane])) ? 1 : 3;
                SPEC_STAMP(s, 7, ((unsigned long long)ver << 32) | (fev - cut))
            }
            SPEC_STAMP(s, 4, __builtin_amdgcn_s_memtime())
            if (lane == 0) { s_ver[s] = ver; s_vfev[s] = vfev; }
        }
    }
    }  // LC_SPEC_OVERLAP
    if (LC_SPEC_CUT_PRIO) __builtin_amdgcn_s_setprio(0);
    __syncthreads();
    if (wv == 0) {
        for (uint32_t s = 0; s < (uint32_t)S; ++s) { SPEC_STAMP(s, 5, __builtin_amdgcn_s_memtime()) }
    }
    // 3. the key's verdict: the first segment whose real run dies
    if (wv == 0) {
        const Args &f = *KA.full;
        bool rerun = plain, bad = false;
        int32_t fv = -1;
        // EX: the run whose set is the key's final one -- 2 x segment, + 1 for
        // the verifying run: the run that truly died, or the last segment's
        // true run
        uint32_t fin_run = 0;
        if (!plain) {
            for (uint32_t s = 0; s < eff && fv < 0 && !rerun && !bad; ++s) {
                if (uni(s_cut[s]) < 0) continue;
                const int32_t top = uni(s_top[s]);
                if (top == -2) { bad = true; break; }
                if (top == -3) { rerun = true; break; }
                fin_run = 2 * s;
                if (s == 0) { fv = top; continue; }
                const int32_t ver = uni(s_ver[s]);
                if (ver == 1) fv = top;
                else if (ver == 2) { fv = uni(s_vfev[s]); fin_run = 2 * s + 1; }
                else if (ver == 5) fin_run = 2 * s + 1;
                else if (ver == 6) bad = true;
                else rerun = true;  // never met (or nothing to start from): unsegmented
            }
        }
        int kr = K_DONE;
        // the unsegmented search runs in a launch of its own (k_spec_rerun):
        // inlined here it cost this kernel 27 VGPRs, 6 -> 4 waves per SIMD
        if (rerun) {
            if (lane == 0) KA.spec_rr[atomicAdd(KA.spec_nrr, 1)] = key;
        } else if (bad) kr = K_SPILL;
        else if (fv >= 0) finish_key(f, key, LC_INVALID, LC_CAUSE_NONLIN, fv, 0, 0, (uint64_t)fv + 1u);
        else finish_key(f, key, LC_VALID, LC_CAUSE_NONE, -1, 0, 0, nev);
        if constexpr (EX) {
            if (!rerun && !bad) {
                uint32_t *const sv = KA.spec_fin + ((size_t)blk * S * 2 + fin_run) * SPEC_SAVE_WORDS;
                const LatMem fm{sv, sv, sv};
                write_final_mem(f, key, fm, lane, sv[T0_RMEM * 64 + lane], uni(sv[(T0_RMEM + 1) * 64]));
            }
        }
        if (kr == K_SPILL) {
            if (KA.flags & T0_STRICT) {
                t0_malformed(KA, key, LC_BATCH_E_FIT);
                finish_key(f, key, LC_UNKNOWN, LC_CAUSE_ERROR, -1, 0, 0, 0);
            } else {
                const bool deep = f.deep && KA.key_width && KA.key_width[key] > LC_DIRECT_T3_WIDTH;
                push_list(deep ? f.deep : f.spill, deep ? f.n_deep : f.n_spill, key, f.list_cap);
            }
        }
    }
}
#undef KA

// The keys k_spec left to the unsegmented search (compact T0, FAST).
constexpr int SPEC_RERUN_WAVES = 4;
template <bool E16, bool EX = false>
__global__ __launch_bounds__(64 * SPEC_RERUN_WAVES) void k_spec_rerun(T0Args a) {
    // a few workgroups of several waves: the launch is in every step and
    // usually finds no key, so its dispatch is what it costs
    __shared__ uint32_t ws_all[SPEC_RERUN_WAVES][3 * T0_RMEM * 64];
    uint32_t *const ws = ws_all[threadIdx.x >> 6];
    const int32_t n = *a.spec_nrr;
    if (blockIdx.x == 0 && threadIdx.x == 0) *a.spec_nrr_next = 0;  // two counters in turn: no memset per step
    for (int32_t w = blockIdx.x * SPEC_RERUN_WAVES + (int32_t)(threadIdx.x >> 6); w < n;
         w += gridDim.x * SPEC_RERUN_WAVES) {
        const int32_t key = a.spec_rr[w];
        const int kr = lattice_key<T0_RSMALL, !EX, E16>(a, key, ws);
        if (kr == K_SPILL) {
            const Args &f = *a.full;
            if (a.flags & T0_STRICT) {
                t0_malformed(a, key, LC_BATCH_E_FIT);
                finish_key(f, key, LC_UNKNOWN, LC_CAUSE_ERROR, -1, 0, 0, 0);
            } else {
                const bool deep = f.deep && a.key_width && a.key_width[key] > LC_DIRECT_T3_WIDTH;
                push_list(deep ? f.deep : f.spill, deep ? f.n_deep : f.n_spill, key, f.list_cap);
            }
        }
    }
}

size_t spec_ws_words(int64_t n_keys, int segs) { return (size_t)std::max<int64_t>(n_keys, 1) * segs * lat_ws_words(); }

// Keys order[0 .. n_order) in workgroups of `segs` segments (2, 3, 4, 6 or
// 8); rerun_grid: workgroups of the rerun launch at most; ws: spec_ws_words(n_order, segs) words; rr: n_order + 2 ints (two
// rerun counts used in turn -- `parity` picks this launch's, which must be
// zero, and k_spec_rerun zeroes the other -- then the rerun list).
// validate: add the T0_STRICT validation blocks.
// fin: exact segments (final configs wanted, no peaks): spec_fin_words(n_order,
// segs) words for the runs' saved sets, segs 2, 4 or 8; null: closed sets.
size_t spec_fin_words(int64_t n_keys, int segs) {
    return (size_t)std::max<int64_t>(n_keys, 1) * segs * 2 * SPEC_SAVE_WORDS;
}
hipError_t launch_spec(const Args &a, const Args *a_dev, int segs, int waves, uint32_t *ws, int32_t *rr, int parity,
                       uint32_t ck1, uint32_t ck2, int rerun_grid, int validate_blocks, const uint16_t *events16,
                       bool cost_cuts, bool prio, bool vfirst, uint32_t *fin, bool stage, hipStream_t s) {
    T0Args t = make_t0(a, a_dev);
    t.events16 = events16;
    if (cost_cuts) t.flags |= T0_SPEC_COST;
    if (!stage) t.flags |= T0_SPEC_NOSTAGE;
    if (vfirst && validate_blocks > 0) t.flags |= T0_SPEC_VFIRST;
    if (!prio) t.flags |= T0_SPEC_NOPRIO;
    t.lat_ws = ws;
    t.spec_ck1 = ck1;
    t.spec_ck2 = ck2;
    t.spec_nrr = rr + (parity & 1);
    t.spec_nrr_next = rr + ((parity & 1) ^ 1);
    t.spec_rr = rr + 2;
    t.spec_fin = fin;
    const dim3 grid((unsigned)std::max(1, a.n_order + std::max(0, validate_blocks)));
    const dim3 rgrid((unsigned)std::max(1, std::min((a.n_order + SPEC_RERUN_WAVES - 1) / SPEC_RERUN_WAVES, rerun_grid)));
    // one wave per segment: more segments than waves (8, 12 or 16 on 4
    // waves, 4 or 8 on 2) measured slower (device_api.hip)
    (void)waves;
#define LC_SPEC_L(SS, WW, E, X) hipLaunchKernelGGL((k_spec<SS, WW, E, X>), grid, dim3(64 * WW), 0, s, t)
#define LC_SPEC_ALL(E)                                                   \
    if (fin) {                                                           \
        if (segs >= 8) LC_SPEC_L(8, 8, E, true);                         \
        else if (segs >= 4) LC_SPEC_L(4, 4, E, true);                    \
        else LC_SPEC_L(2, 2, E, true);                                   \
    } else if (segs >= 8) LC_SPEC_L(8, 8, E, false);                    \
    else if (segs >= 6) LC_SPEC_L(6, 6, E, false);                       \
    else if (segs >= 4) LC_SPEC_L(4, 4, E, false);                       \
    else if (segs >= 3) LC_SPEC_L(3, 3, E, false);                       \
    else LC_SPEC_L(2, 2, E, false);
    if (events16) { LC_SPEC_ALL(true) } else { LC_SPEC_ALL(false) }
#undef LC_SPEC_ALL
#undef LC_SPEC_L
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (events16) {
        if (fin) hipLaunchKernelGGL((k_spec_rerun<true, true>), rgrid, dim3(64 * SPEC_RERUN_WAVES), 0, s, t);
        else hipLaunchKernelGGL((k_spec_rerun<true, false>), rgrid, dim3(64 * SPEC_RERUN_WAVES), 0, s, t);
    } else {
        if (fin) hipLaunchKernelGGL((k_spec_rerun<false, true>), rgrid, dim3(64 * SPEC_RERUN_WAVES), 0, s, t);
        else hipLaunchKernelGGL((k_spec_rerun<false, false>), rgrid, dim3(64 * SPEC_RERUN_WAVES), 0, s, t);
    }
    return hipGetLastError();
}

}  // namespace lcd
