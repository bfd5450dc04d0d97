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

#include "../../include/lincheck.h"
#include "device_common.hpp"
#include "device_search.hpp"

extern "C" __device__ uint32_t __ockl_wfred_add_u32(uint32_t);

namespace lcd {

constexpr int T0_RMAX = 16;       // registers per lane -> 1024 subsets
constexpr uint32_t T0_MAX_WIDTH = 10;
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

// Partner of register k of X along subset bit Q (lane exchange or register pair).
template <int Q, int R>
__device__ __forceinline__ uint32_t partner(const uint32_t (&X)[R], int k) {
    if constexpr (Q < 6) return xchg<Q>(X[k]);
    else return X[k ^ (1 << (Q - 6))];
}

template <int Q>
__device__ __forceinline__ bool has_bit(uint32_t lane, int k) {
    if constexpr (Q < 6) return (lane >> Q) & 1u;
    else return (k >> (Q - 6)) & 1;
}

// One closure step along candidate op Q: X[L u {Q}] |= T_Q(X[L]).  Returns
// whether this lane changed.  live = registers that can be non-zero.
template <int Q, int R>
__device__ __forceinline__ bool expand(uint32_t (&X)[R], uint32_t dq, uint32_t lane, int live) {
    bool ch = false;
#pragma unroll
    for (int k = 0; k < R; ++k) {
        bool on = k < live;
        if constexpr (Q >= 6) on = on && ((k >> (Q - 6)) & 1);
        if (on) {
            const uint32_t src = partner<Q, R>(X, k);
            uint32_t up = tmask(src, dq);
            if constexpr (Q < 6) up = has_bit<Q>(lane, k) ? up : 0u;
            const uint32_t nv = X[k] | up;
            ch |= nv != X[k];
            X[k] = nv;
        }
    }
    return ch;
}

template <int R>
__device__ __forceinline__ bool expand_any(uint32_t q, uint32_t (&X)[R], uint32_t dq, uint32_t lane, int live) {
    switch (q) {
        case 0: return expand<0, R>(X, dq, lane, live);
        case 1: return expand<1, R>(X, dq, lane, live);
        case 2: return expand<2, R>(X, dq, lane, live);
        case 3: return expand<3, R>(X, dq, lane, live);
        case 4: return expand<4, R>(X, dq, lane, live);
        case 5: return expand<5, R>(X, dq, lane, live);
        case 6: if constexpr (R > 1) return expand<6, R>(X, dq, lane, live); else return false;
        case 7: if constexpr (R > 2) return expand<7, R>(X, dq, lane, live); else return false;
        case 8: if constexpr (R > 4) return expand<8, R>(X, dq, lane, live); else return false;
        default: if constexpr (R > 8) return expand<9, R>(X, dq, lane, live); else return false;
    }
}

// Probe count of candidate q: configs of subsets without q where q is legal.
template <int Q, int R>
__device__ __forceinline__ uint32_t probes_q(const uint32_t (&X)[R], uint32_t dq, uint32_t lane, int live) {
    uint32_t n = 0;
#pragma unroll
    for (int k = 0; k < R; ++k)
        if (k < live && !has_bit<Q>(lane, k)) n += legal_cnt(X[k], dq);
    return n;
}

template <int R>
__device__ __forceinline__ uint32_t probes_any(uint32_t q, const uint32_t (&X)[R], uint32_t dq, uint32_t lane, int live) {
    switch (q) {
        case 0: return probes_q<0, R>(X, dq, lane, live);
        case 1: return probes_q<1, R>(X, dq, lane, live);
        case 2: return probes_q<2, R>(X, dq, lane, live);
        case 3: return probes_q<3, R>(X, dq, lane, live);
        case 4: return probes_q<4, R>(X, dq, lane, live);
        case 5: return probes_q<5, R>(X, dq, lane, live);
        case 6: if constexpr (R > 1) return probes_q<6, R>(X, dq, lane, live); else return 0;
        case 7: if constexpr (R > 2) return probes_q<7, R>(X, dq, lane, live); else return 0;
        case 8: if constexpr (R > 4) return probes_q<8, R>(X, dq, lane, live); else return 0;
        default: if constexpr (R > 8) return probes_q<9, R>(X, dq, lane, live); else return 0;
    }
}

// Ret (configs holding p, moved to L without p) and I seed (configs without p).
template <int Q, int R>
__device__ __forceinline__ void split_p(const uint32_t (&W)[R], uint32_t (&Ret)[R], uint32_t (&I)[R], uint32_t lane,
                                        int live) {
#pragma unroll
    for (int k = 0; k < R; ++k) {
        if (k >= live) { Ret[k] = 0; I[k] = 0; continue; }
        const uint32_t src = partner<Q, R>(W, k);
        const bool hp = has_bit<Q>(lane, k);
        Ret[k] = hp ? 0u : src;
        I[k] = hp ? 0u : W[k];
    }
}

template <int R>
__device__ __forceinline__ void split_any(uint32_t p, const uint32_t (&W)[R], uint32_t (&Ret)[R], uint32_t (&I)[R],
                                          uint32_t lane, int live) {
    switch (p) {
        case 0: split_p<0, R>(W, Ret, I, lane, live); break;
        case 1: split_p<1, R>(W, Ret, I, lane, live); break;
        case 2: split_p<2, R>(W, Ret, I, lane, live); break;
        case 3: split_p<3, R>(W, Ret, I, lane, live); break;
        case 4: split_p<4, R>(W, Ret, I, lane, live); break;
        case 5: split_p<5, R>(W, Ret, I, lane, live); break;
        case 6: if constexpr (R > 1) split_p<6, R>(W, Ret, I, lane, live); break;
        case 7: if constexpr (R > 2) split_p<7, R>(W, Ret, I, lane, live); break;
        case 8: if constexpr (R > 4) split_p<8, R>(W, Ret, I, lane, live); break;
        default: if constexpr (R > 8) split_p<9, R>(W, Ret, I, lane, live); break;
    }
}

template <int R>
__device__ __forceinline__ uint32_t wave_count(const uint32_t (&X)[R], int live) {
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < R; ++k)
        if (k < live) c += (uint32_t)__popc(X[k]);
    return __ockl_wfred_add_u32(c);
}

// First max_final configs of the lattice, in (register, lane, state) order.
template <int R>
__device__ __forceinline__ void write_final_lattice(const Args &a, int32_t key, const uint32_t (&W)[R], uint32_t lane) {
    if (!a.final_cfg) return;
    const uint32_t mf = (uint32_t)a.max_final;
    uint32_t base = 0;
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const uint32_t c = (uint32_t)__popc(W[k]);
        // exclusive prefix over lanes of c
        uint32_t x = c;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o);
            if (lane >= (uint32_t)o) x += y;
        }
        const uint32_t tot = __shfl(x, 63);
        uint32_t r = base + x - c;
        uint32_t m = W[k];
        while (m && r < mf) {
            const uint32_t s = (uint32_t)__ffs(m) - 1;
            m &= m - 1;
            a.final_cfg[((size_t)key * a.max_final + r) * 2 + 0] = (uint64_t)(lane + 64u * (uint32_t)k);
            a.final_cfg[((size_t)key * a.max_final + r) * 2 + 1] = (uint64_t)s << 48;
            ++r;
        }
        base += tot;
    }
    if (lane == 0 && a.n_final) a.n_final[key] = base < mf ? base : mf;
}

template <int R>
__device__ __forceinline__ int lattice_key(const Args &a, int32_t key) {
    const uint32_t lane = lane_id();
    const uint64_t b = a.ev_off[key], e = a.ev_off[key + 1];
    const uint32_t tb = a.trans_off ? a.trans_off[key] : 0u;
    if (a.key_states && a.key_states[key] > LC_WIDE_MAX_STATES) {
        finish_key(a, key, LC_UNKNOWN, LC_CAUSE_STATES, -1, 1, 0, 0);
        return K_DONE;
    }
    const uint32_t nstates = a.trans_off ? (a.key_states ? a.key_states[key] : 0xFFFFu) : a.shared_states;
    const uint32_t width = a.key_width ? a.key_width[key] : 0xFFu;
    if (nstates > T0_MAX_STATES || width > T0_MAX_WIDTH || a.init_state >= T0_MAX_STATES) return K_SPILL;

    uint32_t W[R];
#pragma unroll
    for (int k = 0; k < R; ++k) W[k] = 0;
    if (lane == 0) W[0] = 1u << a.init_state;
    uint32_t desc_v = 0;  // lane q: descriptor of the op in slot q
    uint64_t pending = 0;
    uint32_t peak = 1, probes = 0;

    for (uint64_t base = b; base < e; base += 64) {
        const uint32_t cnt = (uint32_t)((e - base) < 64 ? (e - base) : 64);
        const uint32_t ev = lane < cnt ? a.events[base + lane] : 0u;
        const uint32_t dsc = (lane < cnt && !(ev & LC_EV_OK_BIT)) ? a.trans[tb + LC_EV_TRANS(ev)] : 0u;
        for (uint32_t i = 0; i < cnt; ++i) {
            const uint32_t evi = __builtin_amdgcn_readlane(ev, i);
            const uint32_t slot = LC_EV_SLOT(evi);
            if (!(evi & LC_EV_OK_BIT)) {
                if (slot >= T0_MAX_WIDTH) return K_SPILL;
                const uint32_t d = __builtin_amdgcn_readlane(dsc, i);
                if (lane == slot) desc_v = d;
                pending |= 1ull << slot;
                continue;
            }
            const uint32_t p = slot;
            const int32_t evno = (int32_t)(base + i - b);
            const uint64_t pbit = 1ull << p;
            const uint32_t dp = __builtin_amdgcn_readlane(desc_v, p);
            // registers that can hold configs: subsets of slots < hi
            const uint32_t hi = 64u - (uint32_t)__builtin_clzll(pending);  // pending != 0 (p is pending)
            const int live = hi <= 6 ? 1 : (1 << (hi - 6));
            uint32_t Ret[R], I[R];
#pragma unroll
            for (int k = 0; k < R; ++k)
                if (k < live) probes += (uint32_t)__popc(W[k]);  // |S| (oracle: one probe per config of S)
            split_any<R>(p, W, Ret, I, lane, live);
            const uint64_t cand = pending & ~pbit;
            for (;;) {
                bool ch = false;
                for (uint64_t m = cand; m; m &= m - 1) {
                    const uint32_t q = (uint32_t)__builtin_ctzll(m);
                    ch |= expand_any<R>(q, I, __builtin_amdgcn_readlane(desc_v, q), lane, live);
                }
                if (!__any(ch)) break;
            }
            const uint32_t nI = wave_count<R>(I, live);
            for (uint64_t m = cand; m; m &= m - 1) {
                const uint32_t q = (uint32_t)__builtin_ctzll(m);
                probes += probes_any<R>(q, I, __builtin_amdgcn_readlane(desc_v, q), lane, live);
            }
            uint32_t Sn[R];
#pragma unroll
            for (int k = 0; k < R; ++k) {
                if (k >= live) { Sn[k] = 0; continue; }
                Sn[k] = Ret[k] | tmask(I[k], dp);
                probes += legal_cnt(I[k], dp);
            }
            const uint32_t nSn = wave_count<R>(Sn, live);
            if (nI > a.budget || nSn == 0 || nSn > a.budget) {
                const bool invalid = nI <= a.budget && nSn == 0;
                write_final_lattice<R>(a, key, W, lane);
                const uint32_t pr = __ockl_wfred_add_u32(probes);
                finish_key(a, key, invalid ? LC_INVALID : LC_UNKNOWN, invalid ? LC_CAUSE_NONLIN : LC_CAUSE_BUDGET,
                           evno, peak, pr, (uint64_t)evno + (invalid ? 1u : 0u));
                return K_DONE;
            }
#pragma unroll
            for (int k = 0; k < R; ++k) W[k] = Sn[k];
            peak = nSn > peak ? nSn : peak;
            pending &= ~pbit;
        }
    }
    write_final_lattice<R>(a, key, W, lane);
    const uint32_t pr = __ockl_wfred_add_u32(probes);
    finish_key(a, key, LC_VALID, LC_CAUSE_NONE, -1, peak, pr, e - b);
    return K_DONE;
}

__global__ __launch_bounds__(64) void k_search_lattice(Args a) {
    const int32_t n = a.n_in ? *a.n_in : a.n_order;
    for (int32_t w = next_work(a); w < n; w = next_work(a)) {
        const int32_t key = a.order[w];
        const int r = lattice_key<T0_RMAX>(a, key);
        if (r == K_SPILL) push_list(a.spill, a.n_spill, key);
    }
}

hipError_t launch_t0(const Args &a, int grid, hipStream_t s) {
    hipLaunchKernelGGL(k_search_lattice, dim3(grid), dim3(64), 0, s, a);
    return hipGetLastError();
}

}  // namespace lcd
