// Device helpers shared by the LDS tiers (device_search.hip) and the HBM
// tier (device_hbm.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/lincheck.h"
#include "device_search.hpp"

namespace lcd {

// Outcome of searching one key in a tier.
enum { K_DONE = 0, K_SPILL = 1, K_WIDE = 2 };

constexpr uint64_t EMPTY = ~0ull;
constexpr uint64_t LMASK = (1ull << 56) - 1;

__device__ __forceinline__ uint32_t hash64(uint64_t c) {
    c ^= c >> 29;
    c *= 0xBF58476D1CE4E5B9ull;
    return (uint32_t)(c >> 32) ^ (uint32_t)c;
}

// cas-register step on a descriptor (include/lincheck.h LC_T_*), branch-free:
//   READ_ANY: legal, same state   READ: legal iff s == a, same state
//   WRITE:    legal, state := b   CAS:  legal iff s == a, state := b
// A table model (tab != null, uniform per launch): d is the offset of the
// op's row, whose entry s is the next state (LC_TABLE_NONE: inconsistent).
__device__ __forceinline__ bool step(const uint16_t *tab, uint32_t s, uint32_t d, uint32_t &s2) {
    if (tab) {
        const uint32_t t = tab[d + s];
        s2 = t;
        return t != LC_TABLE_NONE;
    }
    uint32_t f = d & 3u, a = (d >> 2) & 0x7FFFu, b = d >> 17;
    s2 = f >= LC_T_WRITE ? b : s;
    return f == LC_T_READ_ANY || f == LC_T_WRITE || s == a;
}

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// Rank of this lane among the lanes whose flag is set (wave-synchronous).
__device__ __forceinline__ uint32_t rank_of(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// Insert key into an LDS hash set; returns true if it was not there.
// pos receives the table slot holding key.
__device__ __forceinline__ bool lds_insert(uint64_t *tab, uint32_t mask, uint64_t key, bool active,
                                           uint32_t &pos) {
    bool isnew = false;
    uint32_t h = hash64(key) & mask;
    bool done = !active;
    while (!done) {
        unsigned long long old = atomicCAS((unsigned long long *)&tab[h], (unsigned long long)EMPTY,
                                           (unsigned long long)key);
        if (old == EMPTY) { isnew = true; done = true; }
        else if (old == key) { done = true; }
        else { h = (h + 1) & mask; }
    }
    pos = h;
    return isnew;
}

// A launch's Args as the kernarg segment holds them (the kernel's first
// parameter), through an opaque pointer: fields read through it are scalar
// loads where they are used.  Read through the kernel's by-value parameter,
// every field used anywhere is loaded at the kernel's entry and held in a
// scalar register for the whole kernel; past the scalar file the compiler
// spills them into VGPR lanes and reloads them inside the hot loops.  The
// set tiers read their cold fields (results, work lists, per-key setup)
// through this.
using KArgs = const __attribute__((address_space(4))) Args;
__device__ __forceinline__ KArgs &kargs() {
    KArgs *p = (KArgs *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *p;
}

template <class A>
__device__ __forceinline__ void write_final_narrow(A &a, int32_t key, const uint64_t *S, uint32_t nS) {
    if (!a.final_cfg) return;
    uint32_t nf = nS < (uint32_t)a.max_final ? nS : (uint32_t)a.max_final;
    for (uint32_t i = lane_id(); i < nf; i += 64) {
        uint64_t c = S[i];
        a.final_cfg[((size_t)key * a.max_final + i) * 2 + 0] = c & LMASK;
        a.final_cfg[((size_t)key * a.max_final + i) * 2 + 1] = (c >> 56) << 48;
    }
    if (lane_id() == 0 && a.n_final) a.n_final[key] = nf;
}

// Append key to a work list of `cap` entries (a list holds each key of a
// step at most once, and cap >= the step's keys; the bound is a guard).
__device__ __forceinline__ void push_list(int32_t *list, int32_t *count, int32_t key, int32_t cap) {
    if (lane_id() == 0) {
        int32_t i = atomicAdd(count, 1);
        if (i < cap) list[i] = key;
    }
}


template <class A>
__device__ __forceinline__ void finish_key(A &a, int32_t key, int verdict, int cause,
                                           int32_t fev, uint32_t peak, uint64_t probes, uint64_t nev) {
    if (lane_id() == 0) {
        a.valid[key] = (int8_t)verdict;
        a.cause[key] = (uint8_t)cause;
        a.fail_event[key] = fev;
        if (a.peak) a.peak[key] = peak;
        // the node exchange's record (include/lincheck.h LC_REC_*), written as
        // the key finishes: no packing pass over the keys afterwards
        if (a.rec)
            a.rec[key] = (uint64_t)(uint8_t)(verdict + 1) | (uint64_t)(uint8_t)cause << 8 |
                         (uint64_t)(uint32_t)(fev + 1) << 16;
        if (a.count_probes) atomicAdd(a.probes, (unsigned long long)probes);
        atomicAdd(a.ev_count, (unsigned long long)nev);
        atomicAdd(a.keys_done, 1ull);
    }
}

// The batch was found malformed by the validation that ran before this
// launch (err words, stream order): the set tiers trust validated events, so
// over a refused batch they do nothing (the call returns LC_E_INVALID).
template <class A>
__device__ __forceinline__ bool batch_refused(A &a) {
    return a.err && __builtin_amdgcn_readfirstlane(*(volatile const int32_t *)a.err) != 0;
}

// Next entry of this launch's work list (dynamic: one atomic ticket per key,
// so long keys -- listed first by the host's LPT order -- do not serialise).
template <class A>
__device__ __forceinline__ int32_t next_work(A &a) {
    int32_t w = 0;
    if (lane_id() == 0) w = atomicAdd(a.ticket, 1);
    return __builtin_amdgcn_readfirstlane(w);
}


}  // namespace lcd
