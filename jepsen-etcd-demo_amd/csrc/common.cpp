// Error reporting shared by every entry point of liblincheck.
#include <hip/hip_runtime_api.h>

#include <dlfcn.h>

#include <sys/mman.h>

#include <algorithm>
#include <cstdarg>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>
#include <map>
#include <unordered_map>
#include <mutex>
#include <unordered_set>

#include "common.hpp"

namespace lc {

static thread_local std::string g_last_error;

void set_error(const std::string &msg) { g_last_error = msg; }

int fail(int code, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

namespace {
struct Roctx {
    int (*push)(const char *) = nullptr;
    int (*pop)() = nullptr;
};
const Roctx &roctx() {
    static Roctx r;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = nullptr;
        for (const char *name : {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4"})
            if (!h) h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        r.push = (int (*)(const char *))dlsym(h, "roctxRangePushA");
        r.pop = (int (*)())dlsym(h, "roctxRangePop");
        if (!r.push || !r.pop) r.push = nullptr, r.pop = nullptr;
    });
    return r;
}
}  // namespace

void range_push(const char *name) {
    const Roctx &r = roctx();
    if (r.push) r.push(name);
}

void range_pop() {
    const Roctx &r = roctx();
    if (r.pop) r.pop();
}

// Page-locked host memory for arrays the device reads whole (lc_pack's event
// words): the DMA engine reads them directly instead of through a bounce
// buffer.  Without a visible GPU (or for small arrays) plain malloc.  Freed
// blocks are kept (up to 1 GB) and handed to the next request they fit
// within 2x: pinning and unpinning cost milliseconds per call (hipHostFree
// synchronises), and a Jepsen-shaped caller packs a history per check.
static std::mutex g_pin_mu;
static std::unordered_map<void *, size_t> g_pinned;  // live and cached blocks -> size
static std::multimap<size_t, void *> g_pin_free;     // cached blocks by size
static size_t g_pin_cached = 0;
static std::unordered_set<void *> g_registered;      // blocks from hipHostRegister (else hipHostMalloc)

static void pin_release(void *p) {  // (g_pin_mu not held)
    bool reg;
    {
        std::lock_guard<std::mutex> g(g_pin_mu);
        reg = g_registered.erase(p) > 0;
    }
    if (reg) {
        (void)hipHostUnregister(p);
        std::free(p);
    } else {
        (void)hipHostFree(p);
    }
}
constexpr size_t PIN_CACHE_MAX = 1ull << 30;

void *pinned_alloc(size_t bytes) {
    static const bool gpu = [] {
        int n = 0;
        const bool ok = hipGetDeviceCount(&n) == hipSuccess && n > 0;
        (void)hipGetLastError();
        return ok;
    }();
    if (gpu && bytes >= (64u << 10) && bytes <= (2ull << 30)) {
        {
            std::lock_guard<std::mutex> g(g_pin_mu);
            auto it = g_pin_free.lower_bound(bytes);
            if (it != g_pin_free.end() && it->first <= 2 * bytes) {
                void *p = it->second;
                g_pin_cached -= it->first;
                g_pin_free.erase(it);
                return p;
            }
        }
        void *p = nullptr;
        if (bytes >= (16u << 20)) {
            // large blocks: transparent-huge-page memory faulted in by 16
            // threads, then registered.  hipHostMalloc faults and zeroes the
            // block single-threaded: 124 ms for 660 MB on the box against
            // 3.3 + 1.3 ms this way (tools/probe/pin_probe.cpp).
            void *q = nullptr;
            const size_t len = (bytes + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
            if (posix_memalign(&q, 2u << 20, len) == 0) {
                (void)madvise(q, len, MADV_HUGEPAGE);
                const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
                std::vector<std::thread> th;
                for (unsigned t = 0; t < nt; ++t)
                    th.emplace_back([=] {
                        char *c = (char *)q;
                        std::memset(c + len * t / nt, 0, len * (t + 1) / nt - len * t / nt);
                    });
                for (auto &x : th) x.join();
                if (hipHostRegister(q, len, hipHostRegisterDefault) == hipSuccess) {
                    std::lock_guard<std::mutex> g(g_pin_mu);
                    g_pinned[q] = bytes;
                    g_registered.insert(q);
                    return q;
                }
                (void)hipGetLastError();
                std::free(q);
            }
        }
        if (hipHostMalloc(&p, bytes, hipHostMallocDefault) == hipSuccess && p) {
            std::lock_guard<std::mutex> g(g_pin_mu);
            g_pinned[p] = bytes;
            return p;
        }
        (void)hipGetLastError();
    }
    return std::malloc(bytes ? bytes : 1);
}

void pinned_free(void *p) {
    if (!p) return;
    {
        std::lock_guard<std::mutex> g(g_pin_mu);
        auto it = g_pinned.find(p);
        if (it == g_pinned.end()) {
            std::free(p);  // (malloc'd: no GPU, or a small block)
            return;
        }
        const size_t sz = it->second;
        if (g_pin_cached + sz <= PIN_CACHE_MAX) {
            g_pin_free.emplace(sz, p);
            g_pin_cached += sz;
            return;
        }
        g_pinned.erase(it);
    }
    pin_release(p);
}

// (never destroyed: arrays in static objects of other files may be freed
// after any destructor of this one would run; the cache holds each block by
// the start of its allocation, so a leak checker finds them reachable)
struct BigCache {
    std::mutex mu;
    std::multimap<size_t, char *> free;  // cached blocks by size -> their allocation
    size_t cached = 0;
};
static BigCache &big_cache() {  // (made on first use: no static-initialisation order)
    static BigCache *c = new BigCache;
    return *c;
}
constexpr size_t BIG_CACHE_MAX = 1ull << 30;

void *big_alloc(size_t bytes) {
    BigCache &g_big = big_cache();
    {
        std::lock_guard<std::mutex> g(g_big.mu);
        auto it = g_big.free.lower_bound(bytes);
        if (it != g_big.free.end() && it->first <= 2 * bytes) {
            char *raw = it->second;
            g_big.cached -= it->first;
            g_big.free.erase(it);
            return raw + 64;
        }
    }
    // the size in a 64-byte header, so a reused block goes back under its own size
    char *raw = nullptr;
    if (bytes >= (8u << 20)) {
        // 2 MB-aligned and marked for transparent huge pages: first touch
        // then faults a 2 MB page at a time (a C3-sized pack writes GBs of
        // fresh arrays; 4 KB faults cost more than the writes)
        // (the whole rounded length is allocated, so the advice covers only
        // this block's own pages)
        void *q = nullptr;
        const size_t len = (bytes + 64 + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
        if (posix_memalign(&q, 2u << 20, len) == 0) {
            raw = (char *)q;
            (void)madvise(raw, len, MADV_HUGEPAGE);
        }
    } else {
        raw = (char *)std::malloc(bytes + 64);
    }
    if (!raw) return nullptr;
    *(size_t *)raw = bytes;
    return raw + 64;
}

void big_free(void *p, size_t) {
    if (!p) return;
    char *raw = (char *)p - 64;
    const size_t sz = *(size_t *)raw;
    BigCache &g_big = big_cache();
    std::lock_guard<std::mutex> g(g_big.mu);
    if (g_big.cached + sz <= BIG_CACHE_MAX) {
        g_big.free.emplace(sz, raw);
        g_big.cached += sz;
    } else {
        std::free(raw);
    }
}

void trim_host_caches() {
    std::vector<void *> pins;
    {
        std::lock_guard<std::mutex> g(g_pin_mu);
        for (auto &e : g_pin_free) {
            pins.push_back(e.second);
            g_pinned.erase(e.second);
        }
        g_pin_free.clear();
        g_pin_cached = 0;
    }
    for (void *p : pins) pin_release(p);
    BigCache &g_big = big_cache();
    std::vector<char *> raws;
    {
        std::lock_guard<std::mutex> g(g_big.mu);
        for (auto &e : g_big.free) raws.push_back(e.second);
        g_big.free.clear();
        g_big.cached = 0;
    }
    for (char *r : raws) std::free(r);
}

// lc_pack's workers: up to 16 threads with the caller (the box's cgroup
// quota; hardware_concurrency counts the whole machine), made on first use
// and kept; one pack at a time uses them.
static std::mutex g_pack_pool_mu;
HostPool *pack_pool_acquire() {
    if (!g_pack_pool_mu.try_lock()) return nullptr;
    static HostPool *pool = new HostPool(std::max(1u, std::min(16u, std::thread::hardware_concurrency())) - 1);
    return pool;
}
void pack_pool_release() { g_pack_pool_mu.unlock(); }

}  // namespace lc

extern "C" void lc_trim(void) { lc::trim_host_caches(); }

extern "C" const char *lc_last_error(void) { return lc::g_last_error.c_str(); }
extern "C" int lc_abi_version(void) { return LC_ABI_VERSION; }
