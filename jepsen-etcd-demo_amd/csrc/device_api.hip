// device_api.hip -- host orchestration of the device search (C ABI: lc_create,
// lc_upload, lc_check_device, lc_check_batch; include/lincheck.h).
//
// This is the native side of the drop-in at etcdemo.clj:115-119: one call
// checks every key of a batch (independent/checker's per-key pmap becomes a
// work list walked by persistent kernels).  Inputs are validated on the host
// before any launch, so a malformed batch can never drive a kernel out of
// bounds.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <cstring>
#include <mutex>
#include <numeric>
#include <thread>
#include <vector>

#include "common.hpp"
#include "device_search.hpp"

#define HIPCHK(expr)                                                                       \
    do {                                                                                   \
        hipError_t _e = (expr);                                                            \
        if (_e != hipSuccess)                                                              \
            return lc::fail(LC_E_DEVICE, "%s failed: %s", #expr, hipGetErrorString(_e));  \
    } while (0)

namespace {

template <class T>
hipError_t dalloc(T **p, size_t n) {
    *p = nullptr;
    if (n == 0) n = 1;
    return hipMalloc((void **)p, n * sizeof(T));
}

template <class T>
void dfree(T *&p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}

}  // namespace

// Host worker threads kept for the life of a context, so the per-event
// validation pass of every lc_check_batch does not pay thread creation.
// run(n, fn) calls fn(0..n-1) on the workers and the caller, and returns when
// all have finished.
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
        {
            std::lock_guard<std::mutex> g(m_);
            fn_ = &fn;
            n_ = n;
            pending_ = n > 1 ? n - 1 : 0;
            ++gen_;
        }
        cv_.notify_all();
        fn(0);
        std::unique_lock<std::mutex> g(m_);
        done_.wait(g, [this] { return pending_ == 0; });
        fn_ = nullptr;
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
            (*fn)(id);
            std::lock_guard<std::mutex> g(m_);
            if (--pending_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(unsigned)> *fn_ = nullptr;
    unsigned n_ = 0, pending_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

struct lc_dev_batch {
    int device = 0;
    int64_t n_keys = 0;
    uint64_t n_events = 0;
    int64_t n_trans = 0;
    uint32_t init_state = 0;
    uint32_t shared_states = 0;  // 1 + largest state id in a shared table
    bool has_trans_off = false;
    uint64_t *ev_off = nullptr;
    uint32_t *events = nullptr;
    uint32_t *trans = nullptr;
    uint32_t *trans_off = nullptr;
    uint8_t *key_width = nullptr;
    uint16_t *key_states = nullptr;
    uint8_t *key_error = nullptr;
    int32_t *order = nullptr;  // LPT: keys by event count, descending
    bool t0_only = false;      // every key fits the register lattice: T0 never spills
    size_t input_bytes = 0;    // bytes the search reads per pass (events + offsets + tables)
    // Device storage behind the arrays above, grown on demand: a batch that is
    // re-uploaded (the ctx's staging batch for lc_check_batch) keeps it, so a
    // host-to-host check allocates nothing once its sizes have been seen.
    struct Mem {
        void *p = nullptr;
        size_t cap = 0;
    } mem[8];
    ~lc_dev_batch() {
        for (Mem &m : mem)
            if (m.p) (void)hipFree(m.p);
    }
};

// Point p at m's storage, growing it to hold n elements of T.
template <class T>
static hipError_t grow(lc_dev_batch::Mem &m, T *&p, size_t n) {
    const size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
    if (bytes > m.cap) {
        if (m.p) (void)hipFree(m.p);
        m.p = nullptr;
        m.cap = 0;
        p = nullptr;
        hipError_t e = hipMalloc(&m.p, bytes);
        if (e != hipSuccess) return e;
        m.cap = bytes;
    }
    p = (T *)m.p;
    return hipSuccess;
}

constexpr size_t CTL_BYTES = 4 * sizeof(unsigned long long) + 16 * sizeof(int32_t);

struct lc_ctx {
    lc_opts o{};
    int device = 0;
    int cu_count = 256;
    hipStream_t stream = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr, et0 = nullptr, et3a = nullptr, et3b = nullptr;
    hipEvent_t ea0 = nullptr, ea1 = nullptr;  // span of the LC_DEV_ASYNC steps since lc_wait
    uint32_t n_async = 0;
    hipEvent_t ring[4] = {};  // end of each of the last 4 LC_DEV_ASYNC steps (lc_wait_step)
    uint64_t async_seq = 0;
    std::mutex mu;
    // scratch, grown on demand
    int64_t cap_keys = 0;
    int32_t *lists = nullptr;      // 4 x cap_keys: spill0, spill1, spill2, wide
    // one 96-byte control block, zeroed and read back in one operation each:
    // acc (4 x u64: probes, events, keys_done) then counters (16 x i32:
    // n_spill0, n_spill1, n_spill2, n_wide, -, tickets[8..15])
    unsigned long long *ctl = nullptr;
    unsigned long long *acc = nullptr;
    int32_t *counters = nullptr;
    unsigned long long *hctl = nullptr;  // pinned host copy of ctl
    int8_t *valid = nullptr;
    int32_t *fail_event = nullptr;
    uint8_t *cause = nullptr;
    uint32_t *peak = nullptr;
    uint64_t *final_cfg = nullptr;
    uint32_t *n_final = nullptr;
    uint32_t *lat_ws = nullptr;    // T0 workspace (lattices of 9-10 pending ops)
    lcd::Args *dargs = nullptr;    // device copy of T0's Args (read once per key)
    lcd::Args *hargs = nullptr;    // its pinned host staging copy (copied only when it changes)
    bool hargs_valid = false;
    // lc_check_batch's staging batch (device arrays reused across calls) and
    // the lock that keeps one lc_check_batch at a time on it
    lc_dev_batch *staged = nullptr;
    uint32_t *hstage = nullptr;  // pinned copy of its event words
    HostPool *pool = nullptr;    // validation workers, created on first use
    size_t hstage_cap = 0;
    std::mutex batch_mu;
    // T0-only steps (lc_check_device) skip re-zeroing the control block: the
    // ticket continues from where the previous such step left it.
    bool ticket_live = false;
    uint32_t ticket_next = 0;
    int lat_ws_blocks = 0;
    // T3 (HBM tier) workspaces: narrow / wide configs
    struct Ws {
        char *base = nullptr;
        size_t bytes = 0;
        int slots = 0;
        lcd::HbmWs w{};
    } ws[2];
    ~lc_ctx() {
        dfree(lists); dfree(ctl); dfree(valid); dfree(fail_event);
        if (hctl) (void)hipHostFree(hctl);
        dfree(cause); dfree(peak); dfree(final_cfg); dfree(n_final);
        dfree(ws[0].base); dfree(ws[1].base); dfree(lat_ws); dfree(dargs);
        if (hargs) (void)hipHostFree(hargs);
        delete staged;
        delete pool;
        if (hstage) (void)hipHostFree(hstage);
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
        if (et0) (void)hipEventDestroy(et0);
        if (et3a) (void)hipEventDestroy(et3a);
        if (et3b) (void)hipEventDestroy(et3b);
        if (ea0) (void)hipEventDestroy(ea0);
        if (ea1) (void)hipEventDestroy(ea1);
        for (hipEvent_t &e : ring)
            if (e) (void)hipEventDestroy(e);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

static int ensure_capacity(lc_ctx *c, int64_t n_keys) {
    if (n_keys <= c->cap_keys) return LC_OK;
    int64_t cap = std::max<int64_t>(n_keys, 1024);
    dfree(c->lists); dfree(c->valid); dfree(c->fail_event); dfree(c->cause);
    dfree(c->peak); dfree(c->final_cfg); dfree(c->n_final);
    HIPCHK(dalloc(&c->lists, (size_t)cap * 4));
    HIPCHK(dalloc(&c->valid, (size_t)cap));
    HIPCHK(dalloc(&c->fail_event, (size_t)cap));
    HIPCHK(dalloc(&c->cause, (size_t)cap));
    HIPCHK(dalloc(&c->peak, (size_t)cap));
    HIPCHK(dalloc(&c->final_cfg, (size_t)cap * (size_t)c->o.max_final * 2));
    HIPCHK(dalloc(&c->n_final, (size_t)cap));
    c->cap_keys = cap;
    return LC_OK;
}

// Lay out (and if needed allocate) a T3 workspace for `want` blocks.
static int ensure_ws(lc_ctx *c, int wide, int want, int *slots_out) {
    lc_ctx::Ws &W = c->ws[wide];
    const size_t cfg = wide ? lcd::cfg_bytes_wide() : lcd::cfg_bytes_narrow();
    const uint64_t cap = c->o.max_configs + (uint64_t)lcd::t3_block() + 64;
    uint64_t H = 1;
    while (H < 2 * cap) H <<= 1;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    lcd::HbmWs w{};
    size_t off = 0;
    w.off_S0 = off; off += al(cap * cfg);
    w.off_S1 = off; off += al(cap * cfg);
    w.off_I = off; off += al(cap * cfg);
    w.off_hS = off; off += al(H * cfg);
    w.off_hI = off; off += al(H * cfg);
    w.off_pS0 = off; off += al(cap * 4);
    w.off_pS1 = off; off += al(cap * 4);
    w.off_pI = off; off += al(cap * 4);
    w.slot_bytes = off;
    w.cap = (uint32_t)cap;
    w.hmask = (uint32_t)(H - 1);
    size_t free_b = 0, total_b = 0;
    HIPCHK(hipMemGetInfo(&free_b, &total_b));
    const int max_slots = c->o.deep_slots > 0 ? c->o.deep_slots : 2 * c->cu_count;
    int slots = std::min(want, max_slots);
    const size_t limit = (W.bytes ? W.bytes : 0) + free_b / 2;
    while (slots > 1 && (size_t)slots * w.slot_bytes > limit) slots /= 2;
    if ((size_t)slots * w.slot_bytes > limit)
        return lc::fail(LC_E_NOMEM, "T3 workspace: one slot needs %zu bytes (budget %llu)", w.slot_bytes,
                        (unsigned long long)c->o.max_configs);
    if (!W.base || W.w.slot_bytes != w.slot_bytes || W.slots < slots) {
        dfree(W.base);
        W.bytes = 0; W.slots = 0;
        HIPCHK(hipMalloc((void **)&W.base, (size_t)slots * w.slot_bytes));
        HIPCHK(hipMemsetAsync(W.base, 0xFF, (size_t)slots * w.slot_bytes, c->stream));  // EMPTY tables
        W.bytes = (size_t)slots * w.slot_bytes;
        W.slots = slots;
    }
    w.base = W.base;
    W.w = w;
    *slots_out = std::min(slots, W.slots);
    return LC_OK;
}

extern "C" int lc_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

extern "C" int lc_create(const lc_opts *opts, lc_ctx **out) {
    if (!out) return lc::fail(LC_E_INVALID, "lc_create: null out");
    lc_opts o{};
    if (opts) o = *opts;
    if (o.algorithm < LC_ALGO_LINEAR || o.algorithm > LC_ALGO_COMPETITION)
        return lc::fail(LC_E_INVALID, "lc_create: algorithm must be LC_ALGO_LINEAR, _WGL or _COMPETITION");
    if (o.max_configs == 0) o.max_configs = 1ull << 20;
    if (o.max_configs > (1ull << 31)) return lc::fail(LC_E_INVALID, "lc_create: max_configs above 2^31");
    if (o.max_final <= 0) o.max_final = 10;
    if (o.max_final > 16) return lc::fail(LC_E_INVALID, "lc_create: max_final above 16");
    if (o.flags & ~LC_OPT_COUNT_PROBES) return lc::fail(LC_E_INVALID, "lc_create: unknown flags 0x%x", o.flags);
    for (int32_t r : o.reserved)
        if (r) return lc::fail(LC_E_INVALID, "lc_create: reserved fields must be 0");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return lc::fail(LC_E_DEVICE, "lc_create: no HIP device visible");
    if (o.device < 0 || o.device >= ndev) return lc::fail(LC_E_DEVICE, "lc_create: device %d of %d", o.device, ndev);
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, o.device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return lc::fail(LC_E_DEVICE, "lc_create: device %d is %s, this build targets gfx950", o.device, prop.gcnArchName);
    lc_ctx *c = new (std::nothrow) lc_ctx();
    if (!c) return lc::fail(LC_E_NOMEM, "lc_create: out of memory");
    c->o = o;
    c->device = o.device;
    c->cu_count = prop.multiProcessorCount;
    int rc = LC_OK;
    auto init = [&]() -> int {
        HIPCHK(hipSetDevice(o.device));
        HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        HIPCHK(hipEventCreate(&c->e0));
        HIPCHK(hipEventCreate(&c->e1));
        HIPCHK(hipEventCreate(&c->et0));
        HIPCHK(hipEventCreate(&c->et3a));
        HIPCHK(hipEventCreate(&c->et3b));
        HIPCHK(hipEventCreate(&c->ea0));
        HIPCHK(hipEventCreate(&c->ea1));
        for (hipEvent_t &e : c->ring) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        HIPCHK(dalloc(&c->ctl, 16));
        c->acc = c->ctl;
        c->counters = (int32_t *)(c->ctl + 4);
        HIPCHK(hipHostMalloc((void **)&c->hctl, 16 * sizeof(unsigned long long), hipHostMallocDefault));
        HIPCHK(dalloc(&c->dargs, 1));
        HIPCHK(hipHostMalloc((void **)&c->hargs, sizeof(lcd::Args), hipHostMallocDefault));
        return LC_OK;
    };
    rc = init();
    if (rc) { delete c; return rc; }
    *out = c;
    return LC_OK;
}

extern "C" void lc_destroy(lc_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    delete c;
}

// Per-event validation of a packed batch (every :ok names a pending slot,
// every invoke's transition id is in range), over nt threads of its own.
// Returns 0 or a reason code (1..3) with the first bad key in *badkey; sets
// no error text, so it may run beside the caller's uploads.
// stage (optional): pinned host buffer that receives a copy of the event
// words; each thread copies the contiguous run of keys it validates, so the
// events are read once, in cache, on their way to the DMA engine.
static int validate_events(const lc_batch *b, int64_t *badkey_out, uint32_t *stage = nullptr,
                           HostPool *hp = nullptr) {
    const int64_t K = b->n_keys;
    unsigned nt = hp ? hp->size() : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (K < 256) nt = 1;
    std::vector<int> bad((size_t)nt, 0);
    std::vector<int64_t> badkey((size_t)nt, -1);
    // contiguous key runs of about equal event counts
    const uint64_t n_ev = b->ev_off[K];
    std::vector<int64_t> cut((size_t)nt + 1, K);
    cut[0] = 0;
    for (unsigned t = 1; t < nt; ++t)
        cut[t] = std::upper_bound(b->ev_off, b->ev_off + K, n_ev * t / nt) - b->ev_off - 1;
    auto work = [&](unsigned t) {
        const int64_t k0 = std::max<int64_t>(cut[t], 0), k1 = std::max<int64_t>(cut[t + 1], k0);
        if (stage && k1 > k0)
            std::memcpy(stage + b->ev_off[k0], b->events + b->ev_off[k0], (b->ev_off[k1] - b->ev_off[k0]) * 4);
        for (int64_t k = k0; k < k1 && !bad[t]; ++k) {
            if (b->key_error && b->key_error[k]) continue;  // not searched
            uint64_t tb = b->trans_off ? b->trans_off[k] : 0;
            uint64_t pend[2] = {0, 0};
            for (uint64_t j = b->ev_off[k]; j < b->ev_off[k + 1]; ++j) {
                uint32_t ev = b->events[j];
                uint32_t s = LC_EV_SLOT(ev);
                // slot 127 marks ops beyond the encodable window: the search
                // stops (LC_CAUSE_WINDOW) before it could follow one.
                if (ev & LC_EV_OK_BIT) {
                    if (s == 127) continue;
                    if (!((pend[s >> 6] >> (s & 63)) & 1)) { bad[t] = 1; badkey[t] = k; break; }
                    pend[s >> 6] &= ~(1ull << (s & 63));
                } else {
                    if (tb + LC_EV_TRANS(ev) >= (uint64_t)b->n_trans) { bad[t] = 2; badkey[t] = k; break; }
                    if (s == 127) continue;
                    if ((pend[s >> 6] >> (s & 63)) & 1) { bad[t] = 3; badkey[t] = k; break; }
                    pend[s >> 6] |= 1ull << (s & 63);
                }
            }
        }
    };
    if (hp) {
        hp->run(nt, work);
    } else if (nt == 1) {
        work(0);
    } else {
        std::vector<std::thread> pool;
        for (unsigned t = 0; t < nt; ++t) pool.emplace_back(work, t);
        for (auto &th : pool) th.join();
    }
    for (size_t t = 0; t < bad.size(); ++t)
        if (bad[t]) { *badkey_out = badkey[t]; return bad[t]; }
    return 0;
}

static int events_error(int why, int64_t key) {
    static const char *text[] = {"", ":ok of a slot with no pending op", "transition id out of range",
                                 ":invoke into an occupied slot"};
    return lc::fail(LC_E_INVALID, "batch: key %lld: %s", (long long)key, text[why]);
}

// Host validation of a packed batch: every index a kernel will follow is in
// range, every :ok names a slot that is pending.  events = false leaves the
// per-event pass to the caller (validate_events).
static int validate_batch(const lc_batch *b, bool events = true) {
    if (!b || b->n_keys < 0) return lc::fail(LC_E_INVALID, "batch: bad n_keys");
    if (b->n_keys == 0) return LC_OK;
    if (!b->ev_off || !b->trans || b->n_trans <= 0) return lc::fail(LC_E_INVALID, "batch: missing arrays");
    if (b->ev_off[0] != 0) return lc::fail(LC_E_INVALID, "batch: ev_off[0] != 0");
    for (int64_t k = 0; k < b->n_keys; ++k) {
        if (b->ev_off[k + 1] < b->ev_off[k]) return lc::fail(LC_E_INVALID, "batch: ev_off not monotone at key %lld", (long long)k);
        if (b->ev_off[k + 1] - b->ev_off[k] > 0x7FFFFFFFull) return lc::fail(LC_E_INVALID, "batch: key %lld has > 2^31 events", (long long)k);
    }
    if (b->ev_off[b->n_keys] && !b->events) return lc::fail(LC_E_INVALID, "batch: events missing");
    if (b->init_state >= LC_STATE_NONE) return lc::fail(LC_E_INVALID, "batch: bad init_state");
    if (events) {
        int64_t bk = -1;
        if (int why = validate_events(b, &bk)) return events_error(why, bk);
    }
    for (int64_t i = 0; i < b->n_trans; ++i) {
        uint32_t d = b->trans[i];
        uint32_t f = d & 3u, a = (d >> 2) & 0x7FFFu, bb = d >> 17;
        if ((f == LC_T_WRITE || f == LC_T_CAS) && bb >= LC_STATE_NONE)
            return lc::fail(LC_E_INVALID, "batch: transition %lld installs an invalid state", (long long)i);
        (void)a;
    }
    return LC_OK;
}

// Copy a validated batch into d's device arrays (grown as needed); c->mu held.
// events_src: where the event words are copied from (b->events by default;
// lc_check_batch passes its pinned staging copy).
static int upload_into(lc_ctx *c, const lc_batch *b, lc_dev_batch *d, const uint32_t *events_src = nullptr) {
    const int64_t K = b->n_keys;
    d->device = c->device;
    d->n_keys = K;
    d->n_events = K ? b->ev_off[K] : 0;
    d->n_trans = b->n_trans > 0 ? b->n_trans : 1;
    d->init_state = b->init_state;
    d->has_trans_off = b->trans_off != nullptr;
    {
        uint32_t mx = b->init_state;
        for (int64_t i = 0; i < b->n_trans; ++i) {
            const uint32_t t = b->trans[i], f = t & 3u, a = (t >> 2) & 0x7FFFu, bb = t >> 17;
            if ((f == LC_T_READ || f == LC_T_CAS) && a != LC_STATE_NONE) mx = std::max(mx, a);
            if (f == LC_T_WRITE || f == LC_T_CAS) mx = std::max(mx, bb);
        }
        d->shared_states = mx + 1;
    }
    // LPT order: longest keys first
    std::vector<int32_t> order((size_t)K);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int32_t x, int32_t y) {
        return b->ev_off[x + 1] - b->ev_off[x] > b->ev_off[y + 1] - b->ev_off[y];
    });
    d->trans_off = nullptr;
    d->key_width = nullptr;
    d->key_states = nullptr;
    d->key_error = nullptr;
    auto up = [&]() -> int {
        HIPCHK(grow(d->mem[0], d->ev_off, (size_t)K + 1));
        HIPCHK(grow(d->mem[1], d->events, (size_t)d->n_events));
        HIPCHK(grow(d->mem[2], d->trans, (size_t)d->n_trans));
        HIPCHK(grow(d->mem[3], d->order, (size_t)K));
        if (K) {
            HIPCHK(hipMemcpyAsync(d->ev_off, b->ev_off, ((size_t)K + 1) * 8, hipMemcpyHostToDevice, c->stream));
            HIPCHK(hipMemcpyAsync(d->order, order.data(), (size_t)K * 4, hipMemcpyHostToDevice, c->stream));
        }
        if (d->n_events)
            HIPCHK(hipMemcpyAsync(d->events, events_src ? events_src : b->events, (size_t)d->n_events * 4,
                                  hipMemcpyHostToDevice, c->stream));
        if (b->n_trans > 0)
            HIPCHK(hipMemcpyAsync(d->trans, b->trans, (size_t)b->n_trans * 4, hipMemcpyHostToDevice, c->stream));
        if (b->trans_off && K) {
            HIPCHK(grow(d->mem[4], d->trans_off, (size_t)K));
            HIPCHK(hipMemcpyAsync(d->trans_off, b->trans_off, (size_t)K * 4, hipMemcpyHostToDevice, c->stream));
        }
        if (b->key_width && K) {
            HIPCHK(grow(d->mem[5], d->key_width, (size_t)K));
            HIPCHK(hipMemcpyAsync(d->key_width, b->key_width, (size_t)K, hipMemcpyHostToDevice, c->stream));
        }
        if (b->key_states && K) {
            HIPCHK(grow(d->mem[6], d->key_states, (size_t)K));
            HIPCHK(hipMemcpyAsync(d->key_states, b->key_states, (size_t)K * 2, hipMemcpyHostToDevice, c->stream));
        }
        if (b->key_error && K) {
            HIPCHK(grow(d->mem[7], d->key_error, (size_t)K));
            HIPCHK(hipMemcpyAsync(d->key_error, b->key_error, (size_t)K, hipMemcpyHostToDevice, c->stream));
        }
        HIPCHK(hipStreamSynchronize(c->stream));
        return LC_OK;
    };
    int rc = up();
    if (rc) return rc;
    // T0 spills a key only for its width (ops pending at once), its state
    // count or the initial state; all three are known here.
    {
        bool ok = K > 0 && b->key_width && b->init_state < lcd::t0_max_states();
        for (int64_t k = 0; ok && k < K; ++k) ok = b->key_width[k] <= lcd::t0_max_width();
        if (ok && b->trans_off) {
            ok = b->key_states != nullptr;
            for (int64_t k = 0; ok && k < K; ++k) ok = b->key_states[k] <= lcd::t0_max_states();
        } else if (ok) {
            ok = d->shared_states <= lcd::t0_max_states();
        }
        d->t0_only = ok;
    }
    d->input_bytes = (size_t)d->n_events * 4 + ((size_t)K + 1) * 8;
    return LC_OK;
}

extern "C" int lc_upload(lc_ctx *c, const lc_batch *b, lc_dev_batch **out) {
    if (!c || !b || !out) return lc::fail(LC_E_INVALID, "lc_upload: null argument");
    std::lock_guard<std::mutex> g(c->mu);
    int rc = validate_batch(b);
    if (rc) return rc;
    HIPCHK(hipSetDevice(c->device));
    lc_dev_batch *d = new (std::nothrow) lc_dev_batch();
    if (!d) return lc::fail(LC_E_NOMEM, "lc_upload: out of memory");
    rc = upload_into(c, b, d);
    if (rc) { delete d; return rc; }
    *out = d;
    return LC_OK;
}

extern "C" void lc_dev_batch_free(lc_dev_batch *d) {
    if (!d) return;
    (void)hipSetDevice(d->device);
    delete d;
}

extern "C" int lc_check_device(lc_ctx *c, const lc_dev_batch *d, lc_result *r, int flags, lc_stats *st) {
    if (flags & ~(LC_DEV_RESULT | LC_DEV_ASYNC)) return lc::fail(LC_E_INVALID, "lc_check_device: unknown flags 0x%x", flags);
    const bool dev_result = (flags & LC_DEV_RESULT) != 0;
    if (!c || !d || !r || !r->valid || !r->fail_event || !r->cause)
        return lc::fail(LC_E_INVALID, "lc_check_device: null argument");
    if (d->device != c->device) return lc::fail(LC_E_INVALID, "lc_check_device: batch lives on another device");
    std::lock_guard<std::mutex> g(c->mu);
    auto t0 = std::chrono::steady_clock::now();
    HIPCHK(hipSetDevice(c->device));
    const int64_t K = d->n_keys;
    if (K > 0x7FFFFFFF) return lc::fail(LC_E_INVALID, "lc_check_device: too many keys");
    int rc = ensure_capacity(c, K);
    if (rc) return rc;

    lcd::Args a{};
    a.ev_off = d->ev_off; a.events = d->events; a.trans = d->trans; a.trans_off = d->trans_off;
    a.key_width = d->key_width; a.key_states = d->key_states; a.key_error = d->key_error;
    a.init_state = d->init_state; a.shared_states = d->shared_states;
    a.budget = c->o.max_configs; a.max_final = c->o.max_final; a.debug_mode = c->o.debug_mode;
    a.count_probes = (c->o.flags & LC_OPT_COUNT_PROBES) ? 1 : 0;
    if (dev_result) {
        a.valid = r->valid; a.fail_event = r->fail_event; a.cause = r->cause;
        a.peak = r->peak_configs; a.final_cfg = r->final_configs; a.n_final = r->n_final;
    } else {
        a.valid = c->valid; a.fail_event = c->fail_event; a.cause = c->cause;
        a.peak = c->peak; a.final_cfg = c->final_cfg; a.n_final = c->n_final;
    }
    a.probes = c->acc + 0; a.ev_count = c->acc + 1; a.keys_done = c->acc + 2;
    int32_t *spill0 = c->lists, *spill1 = c->lists + c->cap_keys, *spill2 = c->lists + 2 * c->cap_keys;
    int32_t *wide = c->lists + 3 * c->cap_keys;
    int32_t *n_spill0 = c->counters + 0, *n_spill1 = c->counters + 1, *n_spill2 = c->counters + 2;
    int32_t *n_wide = c->counters + 3;

    // Nothing counted and no key can leave T0: no T1/T2 launches, no counter
    // readback and no control-block memset -- the step is T0 alone (plus the
    // result download when the results go to host memory).
    const bool t0_step = K > 0 && d->t0_only && !(c->o.flags & LC_OPT_COUNT_PROBES);
    // LC_DEV_ASYNC: such a step is only enqueued; lc_wait ends the run
    const bool async = t0_step && dev_result && (flags & LC_DEV_ASYNC);
    uint32_t ticket_base = 0;
    if (t0_step && c->ticket_live) ticket_base = c->ticket_next;
    else HIPCHK(hipMemsetAsync(c->ctl, 0, CTL_BYTES, c->stream));
    c->ticket_live = false;
    if (a.n_final && K > 0) HIPCHK(hipMemsetAsync(a.n_final, 0, (size_t)K * 4, c->stream));
    // T0: every key, LPT order; keys outside the register lattice spill to T1
    lcd::Args a0 = a;
    a0.order = d->order; a0.n_order = (int32_t)K; a0.n_in = nullptr; a0.ticket = c->counters + 8;
    a0.spill = spill0; a0.n_spill = n_spill0; a0.wide = wide; a0.n_wide = n_wide;
    a0.deep = spill2; a0.n_deep = n_spill2;  // very wide keys: straight to T3
    // T0 has two builds: 16 lattice registers (n <= 10 pending in VGPRs, 2
    // waves per SIMD) when every key can be resident at once -- each key's
    // events are serial, so there per-key latency is the whole story -- and
    // 4 registers (9-10 pending in LDS, 4 waves per SIMD) for larger batches,
    // where occupancy hides latency across keys.
    const bool t0_wide = K <= (int64_t)c->cu_count * 8;
    const int g0 = (int)std::max<int64_t>(1, std::min<int64_t>(K, (int64_t)c->cu_count * (t0_wide ? 8 : 16)));
    a0.lat_ws = nullptr;
    // T0 reads the result/counter/list pointers from a device copy of its
    // Args, refreshed (outside the timed region) only when they change
    if (!c->hargs_valid || std::memcmp(c->hargs, &a0, sizeof a0) != 0) {
        // the pinned staging copy may still feed an enqueued copy
        if (c->n_async) HIPCHK(hipStreamSynchronize(c->stream));
        std::memcpy(c->hargs, &a0, sizeof a0);
        HIPCHK(hipMemcpyAsync(c->dargs, c->hargs, sizeof(lcd::Args), hipMemcpyHostToDevice, c->stream));
        c->hargs_valid = true;
    }
    HIPCHK(hipEventRecord(c->e0, c->stream));
    if (async && c->n_async == 0) HIPCHK(hipEventRecord(c->ea0, c->stream));
    if (K > 0) {
        HIPCHK(lcd::launch_t0(a0, c->dargs, g0, t0_wide, c->stream, ticket_base));
        HIPCHK(hipEventRecord(c->et0, c->stream));
    }
    if (async) {
        HIPCHK(hipEventRecord(c->ea1, c->stream));
        HIPCHK(hipEventRecord(c->ring[c->async_seq % 4], c->stream));
        ++c->async_seq;
        ++c->n_async;
        c->ticket_next = ticket_base + (uint32_t)K + (uint32_t)g0;
        c->ticket_live = true;
        if (st) *st = lc_stats{};  // times come from lc_wait
        return LC_OK;
    }
    if (K > 0 && !t0_step) {
        // T1: LDS hash sets
        lcd::Args a1 = a;
        a1.order = spill0; a1.n_order = 0; a1.n_in = n_spill0; a1.ticket = c->counters + 9;
        a1.spill = spill1; a1.n_spill = n_spill1; a1.wide = wide; a1.n_wide = n_wide;
        int g1 = (int)std::min<int64_t>(K, (int64_t)c->cu_count * 7);
        HIPCHK(lcd::launch_t1(a1, g1, c->stream));
        // T2: keys that outgrew T1
        lcd::Args a2 = a;
        a2.order = spill1; a2.n_order = 0; a2.n_in = n_spill1; a2.ticket = c->counters + 10;
        a2.spill = spill2; a2.n_spill = n_spill2; a2.wide = wide; a2.n_wide = n_wide;
        HIPCHK(lcd::launch_t2(a2, c->cu_count, c->stream));
    }
    // One readback for the common case.  The T3 (HBM) tier is launched only
    // when T2 left keys for it (its workspace is sized from those counts),
    // after which the readback is repeated.
    const unsigned long long *acc = c->hctl;
    const int32_t *cnt = (const int32_t *)(c->hctl + 4);
    auto readback = [&]() -> int {
        HIPCHK(hipEventRecord(c->e1, c->stream));
        HIPCHK(hipMemcpyAsync(c->hctl, c->ctl, CTL_BYTES, hipMemcpyDeviceToHost, c->stream));
        if (!dev_result && K > 0) {
            HIPCHK(hipMemcpyAsync(r->valid, c->valid, (size_t)K, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipMemcpyAsync(r->fail_event, c->fail_event, (size_t)K * 4, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipMemcpyAsync(r->cause, c->cause, (size_t)K, hipMemcpyDeviceToHost, c->stream));
            if (r->peak_configs)
                HIPCHK(hipMemcpyAsync(r->peak_configs, c->peak, (size_t)K * 4, hipMemcpyDeviceToHost, c->stream));
            if (r->final_configs)
                HIPCHK(hipMemcpyAsync(r->final_configs, c->final_cfg, (size_t)K * c->o.max_final * 16,
                                      hipMemcpyDeviceToHost, c->stream));
            if (r->n_final)
                HIPCHK(hipMemcpyAsync(r->n_final, c->n_final, (size_t)K * 4, hipMemcpyDeviceToHost, c->stream));
        }
        HIPCHK(hipStreamSynchronize(c->stream));
        return LC_OK;
    };
    if (t0_step) {
        if (dev_result) {
            HIPCHK(hipEventRecord(c->e1, c->stream));
            HIPCHK(hipEventSynchronize(c->e1));
        } else {
            rc = readback();
            if (rc) return rc;
        }
        std::memset(c->hctl, 0, CTL_BYTES);  // counters not kept on this path
        c->ticket_next = ticket_base + (uint32_t)K + (uint32_t)g0;
        c->ticket_live = true;
    } else {
        rc = readback();
        if (rc) return rc;
    }
    bool t3 = false;
    const unsigned long long probes_pre_t3 = acc[0];
    if (K > 0 && (cnt[2] > 0 || cnt[3] > 0)) {
        // T3 (HBM tier): keys beyond T2, then keys needing wide configs
        t3 = true;
        HIPCHK(hipEventRecord(c->et3a, c->stream));
        lcd::Args a3 = a;
        a3.wide = wide; a3.n_wide = n_wide;
        if (cnt[2] > 0) {
            int slots = 0;
            rc = ensure_ws(c, 0, cnt[2], &slots);
            if (rc) return rc;
            a3.order = spill2; a3.n_order = 0; a3.n_in = n_spill2; a3.ticket = c->counters + 11;
            HIPCHK(lcd::launch_t3_narrow(a3, c->ws[0].w, slots, c->stream));
            HIPCHK(hipMemcpyAsync(c->hctl, c->ctl, CTL_BYTES, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
        }
        if (cnt[3] > 0) {
            int slots = 0;
            rc = ensure_ws(c, 1, cnt[3], &slots);
            if (rc) return rc;
            a3.order = wide; a3.n_order = 0; a3.n_in = n_wide; a3.ticket = c->counters + 12;
            HIPCHK(lcd::launch_t3_wide(a3, c->ws[1].w, slots, c->stream));
        }
        HIPCHK(hipEventRecord(c->et3b, c->stream));
        rc = readback();
        if (rc) return rc;
    }
    float ms = 0, ms0 = 0, ms3 = 0;
    HIPCHK(hipEventElapsedTime(&ms, c->e0, c->e1));
    if (K > 0) HIPCHK(hipEventElapsedTime(&ms0, c->e0, c->et0));
    if (t3) HIPCHK(hipEventElapsedTime(&ms3, c->et3a, c->et3b));
    if (st) {
        st->kernel_ms = ms;
        st->tier0_ms = ms0;
        st->tier3_ms = ms3;
        st->probes_t3 = t3 ? acc[0] - probes_pre_t3 : 0;
        st->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        st->probes = acc[0];
        st->events = acc[1];
        st->lds_keys = acc[2];
        st->deep_keys = (uint64_t)(cnt[2] + cnt[3]);  // keys the HBM tier (re)searched
    }
    return LC_OK;
}

extern "C" int lc_wait(lc_ctx *c, lc_stats *st) {
    if (!c) return lc::fail(LC_E_INVALID, "lc_wait: null context");
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    const int n = (int)c->n_async;
    float ms = 0;
    if (n) HIPCHK(hipEventElapsedTime(&ms, c->ea0, c->ea1));
    c->n_async = 0;
    if (st) {
        *st = lc_stats{};
        st->kernel_ms = ms;                    // first enqueued step's start .. last one's end
        st->tier0_ms = n ? ms / (float)n : 0;  // per step, gaps between launches included
    }
    return n;
}

extern "C" int lc_wait_step(lc_ctx *c, int back) {
    if (!c) return lc::fail(LC_E_INVALID, "lc_wait_step: null context");
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    if (back < 0 || back >= 4 || (uint64_t)back >= c->async_seq) {
        HIPCHK(hipStreamSynchronize(c->stream));  // no such step on record: everything
    } else {
        HIPCHK(hipEventSynchronize(c->ring[(c->async_seq - 1 - (uint64_t)back) % 4]));
    }
    return LC_OK;
}

extern "C" int lc_check_batch(lc_ctx *c, const lc_batch *b, lc_result *r, lc_stats *st) {
    auto t0 = std::chrono::steady_clock::now();
    if (!c || !b) return lc::fail(LC_E_INVALID, "lc_check_batch: null argument");
    std::lock_guard<std::mutex> gb(c->batch_mu);
    auto t_val = t0;
    int rc;
    {
        std::lock_guard<std::mutex> g(c->mu);
        rc = validate_batch(b, false);
        if (rc) return rc;
        HIPCHK(hipSetDevice(c->device));
        if (!c->staged) {
            c->staged = new (std::nothrow) lc_dev_batch();
            if (!c->staged) return lc::fail(LC_E_NOMEM, "lc_check_batch: out of memory");
            c->staged->device = c->device;
        }
        // The per-event pass copies the event words into pinned staging as it
        // validates them (one parallel read of the caller's array); the DMA
        // then runs from pinned memory instead of the driver's pageable path.
        // Batches above 256 MB of events keep the pageable path (no pinned
        // allocation that large).
        const size_t n_ev = b->n_keys ? (size_t)b->ev_off[b->n_keys] : 0;
        const bool stage = n_ev > 0 && n_ev <= (256u << 20) / 4;
        if (stage && n_ev > c->hstage_cap) {
            if (c->hstage) (void)hipHostFree(c->hstage);
            c->hstage = nullptr;
            c->hstage_cap = 0;
            HIPCHK(hipHostMalloc((void **)&c->hstage, n_ev * 4, hipHostMallocDefault));
            c->hstage_cap = n_ev;
        }
        int64_t bk = -1;
        if (b->n_keys >= 256 && !c->pool)
            c->pool = new HostPool(std::max(1u, std::min(16u, std::thread::hardware_concurrency())) - 1);
        if (b->n_keys)
            if (int why = validate_events(b, &bk, stage ? c->hstage : nullptr, b->n_keys >= 256 ? c->pool : nullptr))
                return events_error(why, bk);
        t_val = std::chrono::steady_clock::now();
        rc = upload_into(c, b, c->staged, stage ? c->hstage : nullptr);
        if (rc) return rc;
    }
    const auto t_up = std::chrono::steady_clock::now();
    rc = lc_check_device(c, c->staged, r, 0, st);
    if (std::getenv("LC_TIMING")) {
        using ms = std::chrono::duration<double, std::milli>;
        const auto t_end = std::chrono::steady_clock::now();
        std::fprintf(stderr, "lc_check_batch: validate %.3f ms, upload %.3f ms, check %.3f ms\n",
                     ms(t_val - t0).count(), ms(t_up - t_val).count(), ms(t_end - t_up).count());
    }
    if (st && rc == LC_OK)
        st->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}
