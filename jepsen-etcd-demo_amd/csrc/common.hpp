// Shared host-side plumbing for liblincheck: error reporting and owned
// history storage.  Host code only (no device code in this header).
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <memory>
#include <exception>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lincheck.h"

namespace lc {

// Thread-local last error (lc_last_error).  Every failing entry point sets it.
void set_error(const std::string &msg);
int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

// roctx ranges (tracing) around the host steps of a check --
// pack, upload, search enqueue, gather, wait -- visible in rocprofv3
// --marker-trace timelines beside the kernels.  The roctx library is opened
// at first use (no link-time dependency); without it the ranges cost nothing.
void range_push(const char *name);
void range_pop();
struct Range {
    explicit Range(const char *name) { range_push(name); }
    ~Range() { range_pop(); }
    Range(const Range &) = delete;
    Range &operator=(const Range &) = delete;
};

// Page-locked when a GPU is visible (a direct DMA source), else malloc.
void *pinned_alloc(size_t bytes);
void pinned_free(void *p);

template <class T>
struct PinnedAlloc {
    using value_type = T;
    PinnedAlloc() = default;
    template <class U>
    PinnedAlloc(const PinnedAlloc<U> &) {}
    T *allocate(size_t n) {
        void *p = pinned_alloc(n * sizeof(T));
        if (!p) throw std::bad_alloc();
        return (T *)p;
    }
    void deallocate(T *p, size_t) { pinned_free(p); }
    // resize() default-initialises (no zero fill: the arrays are written
    // whole, in parallel, right after)
    template <class U>
    void construct(U *p) noexcept { ::new ((void *)p) U; }
    template <class U, class... A>
    void construct(U *p, A &&...a) { ::new ((void *)p) U(static_cast<A &&>(a)...); }
    template <class U>
    bool operator==(const PinnedAlloc<U> &) const { return true; }
    template <class U>
    bool operator!=(const PinnedAlloc<U> &) const { return false; }
};
template <class T>
using pinned_vector = std::vector<T, PinnedAlloc<T>>;

// Blocks of 1 MB and more, kept when freed (up to 1 GB) and handed to the
// next request they fit within 2x: a packed batch's arrays are the same
// sizes from one check to the next, and fresh ones cost a page fault per
// 4 KB on first touch.
void *big_alloc(size_t bytes);
void big_free(void *p, size_t bytes);
constexpr size_t BIG_BLOCK = 1u << 20;

// std::allocator whose resize() default-initialises (no zero fill), large
// blocks through big_alloc
template <class T>
struct UninitAlloc : std::allocator<T> {
    using value_type = T;
    UninitAlloc() = default;
    template <class U>
    UninitAlloc(const UninitAlloc<U> &) {}
    template <class U>
    struct rebind { using other = UninitAlloc<U>; };
    T *allocate(size_t n) {
        if (n * sizeof(T) >= BIG_BLOCK) {
            void *p = big_alloc(n * sizeof(T));
            if (!p) throw std::bad_alloc();
            return (T *)p;
        }
        return std::allocator<T>::allocate(n);
    }
    void deallocate(T *p, size_t n) {
        if (n * sizeof(T) >= BIG_BLOCK) big_free(p, n * sizeof(T));
        else std::allocator<T>::deallocate(p, n);
    }
    template <class U>
    void construct(U *p) noexcept { ::new ((void *)p) U; }
    template <class U, class... A>
    void construct(U *p, A &&...a) { ::new ((void *)p) U(static_cast<A &&>(a)...); }
};
template <class T>
using uninit_vector = std::vector<T, UninitAlloc<T>>;


// Host memory of a size fixed at allocation, page-locked or not by a choice
// made at run time (lc_pack decides after the pairing pass which event
// array the device will read: the 16-bit words when every word fits, else
// the 32-bit ones).  Not zero-filled.
template <class T>
class host_array {
  public:
    host_array() = default;
    host_array(const host_array &) = delete;
    host_array &operator=(const host_array &) = delete;
    ~host_array() { release(); }
    void alloc(size_t n, bool pinned) {
        release();
        if (n == 0) return;
        const size_t bytes = n * sizeof(T);
        void *p = pinned ? pinned_alloc(bytes) : (bytes >= BIG_BLOCK ? big_alloc(bytes) : std::malloc(bytes));
        if (!p) throw std::bad_alloc();
        p_ = (T *)p;
        n_ = n;
        pinned_ = pinned;
    }
    // Take another array's storage (and its pinning).
    void adopt(host_array &o) {
        release();
        p_ = o.p_; n_ = o.n_; pinned_ = o.pinned_;
        o.p_ = nullptr; o.n_ = 0;
    }
    void release() {
        if (p_) {
            const size_t bytes = n_ * sizeof(T);
            if (pinned_) pinned_free(p_);
            else if (bytes >= BIG_BLOCK) big_free(p_, bytes);
            else std::free(p_);
        }
        p_ = nullptr;
        n_ = 0;
    }
    T *data() { return p_; }
    const T *data() const { return p_; }
    size_t size() const { return n_; }
    bool empty() const { return n_ == 0; }
    bool pinned() const { return pinned_; }
    T &operator[](size_t i) { return p_[i]; }
    const T &operator[](size_t i) const { return p_[i]; }

  private:
    T *p_ = nullptr;
    size_t n_ = 0;
    bool pinned_ = false;
};

// Drop every cached host block (pinned and heap): lc_trim, and the last
// lc_destroy.
void trim_host_caches();

// Host worker threads kept for the life of a context (per-event validation
// and staging copies; one driver per extra device).  run(n, fn) calls
// fn(0..n-1) on the workers and the caller, and returns when all have
// finished.  Not reentrant: one run at a time.
class HostPool {
  public:
    explicit HostPool(unsigned n) {
        for (unsigned i = 0; i < n; ++i) th_.emplace_back([this, i] { loop(i + 1); });
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    unsigned size() const { return (unsigned)th_.size() + 1; }
    void run(unsigned n, const std::function<void(unsigned)> &fn) {
        n = std::min(n, size());
        {
            std::lock_guard<std::mutex> g(m_);
            fn_ = &fn;
            n_ = n;
            pending_ = n > 1 ? n - 1 : 0;
            ++gen_;
        }
        cv_.notify_all();
        // The workers hold references to fn: wait for them whatever fn(0)
        // does, then hand the first exception (caller's or a worker's) on.
        std::exception_ptr ex;
        try {
            fn(0);
        } catch (...) {
            ex = std::current_exception();
        }
        std::unique_lock<std::mutex> g(m_);
        done_.wait(g, [this] { return pending_ == 0; });
        fn_ = nullptr;
        if (!ex) ex = ex_;
        ex_ = nullptr;
        g.unlock();
        if (ex) std::rethrow_exception(ex);
    }

  private:
    void loop(unsigned id) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(unsigned)> *fn;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                if (id >= n_) continue;
                fn = fn_;
            }
            std::exception_ptr ex;
            try {
                (*fn)(id);
            } catch (...) {  // never out of a worker thread (std::terminate)
                ex = std::current_exception();
            }
            std::lock_guard<std::mutex> g(m_);
            if (ex && !ex_) ex_ = ex;
            if (--pending_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(unsigned)> *fn_ = nullptr;
    std::exception_ptr ex_;  // a worker's first exception in this run
    unsigned n_ = 0, pending_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// The process's host worker pool for lc_pack (created on first use, up to 16
// threads with the caller).  run() is not reentrant: a caller that finds it
// busy (another thread packing) gets nullptr and works without it.
HostPool *pack_pool_acquire();
void pack_pool_release();

// work(0..n-1) on n-1 fresh threads and the caller; joins them all, then
// rethrows the first exception any of them raised (none escapes a thread).
template <class F>
void run_threads(unsigned n, const F &work) {
    std::mutex em;
    std::exception_ptr ex;
    auto guarded = [&](unsigned t) {
        try {
            work(t);
        } catch (...) {
            std::lock_guard<std::mutex> g(em);
            if (!ex) ex = std::current_exception();
        }
    };
    std::vector<std::thread> th;
    for (unsigned t = 1; t < n; ++t) th.emplace_back(guarded, t);
    guarded(0);
    for (auto &x : th) x.join();
    if (ex) std::rethrow_exception(ex);
}

// Holds the pack pool for a scope (released on every exit, exceptions too).
struct PackPoolGuard {
    HostPool *pool = pack_pool_acquire();
    PackPoolGuard() = default;
    PackPoolGuard(const PackPoolGuard &) = delete;
    PackPoolGuard &operator=(const PackPoolGuard &) = delete;
    ~PackPoolGuard() {
        if (pool) pack_pool_release();
    }
};

}  // namespace lc

// Owned history: the storage behind lc_synth_generate / lc_edn_read.
struct lc_hist {
    lc::uninit_vector<uint8_t> type, f;
    lc::uninit_vector<int64_t> process, key, v0, v1, index;
    std::vector<int64_t> anomalous_keys;
    // :txn micro-ops (lc_history.mop_off / mop); empty when no row is a :txn
    std::vector<int64_t> mop_off, mop;
    // names of named registers (lc_edn_read): id LC_NAMED_REG_BASE + i is reg_names[i]
    std::vector<std::string> reg_names;

    void reserve(size_t n) {
        type.reserve(n); f.reserve(n); process.reserve(n); key.reserve(n);
        v0.reserve(n); v1.reserve(n); index.reserve(n);
    }
    void push(uint8_t t, uint8_t fn, int64_t p, int64_t k, int64_t a, int64_t b, int64_t idx) {
        type.push_back(t); f.push_back(fn); process.push_back(p); key.push_back(k);
        v0.push_back(a); v1.push_back(b); index.push_back(idx);
    }
    // Row `size() - 1`'s micro-ops (call right after its push); the offsets
    // of earlier rows are filled in on the first :txn row.
    void set_mops(const int64_t *triples, size_t n) {
        const size_t rows = type.size();
        if (mop_off.empty()) mop_off.assign(rows, 0);
        while (mop_off.size() < rows) mop_off.push_back((int64_t)(mop.size() / 3));
        mop.insert(mop.end(), triples, triples + 3 * n);
        mop_off.push_back((int64_t)(mop.size() / 3));
    }
    // Close the offsets (n + 1 entries) once every row is pushed.
    void finish_mops() {
        if (mop_off.empty()) return;
        while (mop_off.size() < type.size() + 1) mop_off.push_back((int64_t)(mop.size() / 3));
    }
    int64_t size() const { return (int64_t)type.size(); }
    lc_history view() const {
        lc_history h;
        h.n = size();
        h.type = type.data(); h.f = f.data(); h.process = process.data(); h.key = key.data();
        h.v0 = v0.data(); h.v1 = v1.data(); h.index = index.data();
        const bool txn = !mop_off.empty();
        h.mop_off = txn ? mop_off.data() : nullptr;
        h.mop = txn ? mop.data() : nullptr;
        return h;
    }
};
