// device_api.hip -- host orchestration of the device search (C ABI: lc_create,
// lc_upload, lc_check_device, lc_check_batch, lc_check_node; include/lincheck.h).
//
// This is the native side of the drop-in at etcdemo.clj:115-119: one call
// checks every key of a batch.  independent/checker's per-key pmap becomes
//   * across GPUs: contiguous key shards balanced by event count, one per
//     device of the context (one host driver thread per device), or one
//     shard per process with the verdict records all-gathered over RCCL
//     (lc_check_node);
//   * within a GPU: a work list walked by persistent kernels.
// Nothing a kernel follows is trusted unchecked: the host validates every
// index of a batch, except the per-event ones of a batch whose keys all fit
// the register tier, which T0 checks itself as it walks the events (a
// malformed event stops its key and the call returns LC_E_INVALID).

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <numeric>
#include <string>
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

#define RCCLCHK(expr)                                                                      \
    do {                                                                                   \
        ncclResult_t _r = (expr);                                                          \
        if (_r != ncclSuccess)                                                             \
            return lc::fail(LC_E_DEVICE, "%s failed: %s", #expr, R->error(_r));            \
    } while (0)

namespace {

constexpr int MAX_DEV = LC_MAX_DEVICES;

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

// RCCL, loaded on first use from the directory of the HIP runtime this
// library is bound to (a process may hold two: torch bundles its own), so
// the communicator and our streams belong to one runtime.
struct Rccl {
    void *h = nullptr;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    const char *error(ncclResult_t r) const { return error_string ? error_string(r) : "rccl error"; }
};

const Rccl *rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = nullptr;
        Dl_info info;
        if (dladdr((void *)&hipStreamCreateWithFlags, &info) && info.dli_fname) {
            std::string dir = info.dli_fname;
            dir = dir.substr(0, dir.find_last_of('/') + 1);
            for (const char *name : {"librccl.so.1", "librccl.so"})
                if (!h) h = dlopen((dir + name).c_str(), RTLD_NOW | RTLD_LOCAL);
        }
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
        r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(h, "ncclCommInitRank");
        r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
        r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
        r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
        if (r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.all_gather) r.h = h;
    });
    return r.h ? &r : nullptr;
}

// 16-bit event words (lc_batch.events16) widened to the 32-bit form every
// kernel reads (LC_EV16_WIDE): 4 words per thread, 8-byte loads, 16-byte stores.
__global__ void k_widen16(const uint16_t *in, uint32_t *out, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t n4 = n / 4;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        const uint2 v = reinterpret_cast<const uint2 *>(in)[i];
        uint4 w;
        w.x = LC_EV16_WIDE(v.x & 0xFFFFu); w.y = LC_EV16_WIDE(v.x >> 16);
        w.z = LC_EV16_WIDE(v.y & 0xFFFFu); w.w = LC_EV16_WIDE(v.y >> 16);
        reinterpret_cast<uint4 *>(out)[i] = w;
    }
    for (uint64_t i = n4 * 4 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        out[i] = LC_EV16_WIDE(in[i]);
}

// Read and clear the error words of the ring slots in `mask` (one atomic
// exchange per word, so an error a still-running step raises meanwhile is
// never lost, only reported by the next read).
__global__ void k_take_err(int32_t *words, uint32_t mask, int32_t *out) {
    if (threadIdx.x != 0) return;
    for (int q = 0; q < 4; ++q) {
        const bool on = (mask >> q) & 1u;
        out[2 * q] = on ? atomicExch(&words[2 * q], 0) : 0;
        out[2 * q + 1] = on ? atomicExch(&words[2 * q + 1], 0) : 0;
    }
}

// Verdict record of one key (include/lincheck.h LC_REC_*), 0 for padding.
__global__ void k_pack_records(const int8_t *valid, const uint8_t *cause, const int32_t *fail_event, int64_t n,
                               int64_t block, uint64_t *out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < block; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t r = 0;
        if (i < n)
            r = (uint64_t)(uint8_t)(valid[i] + 1) | (uint64_t)cause[i] << 8 | (uint64_t)(uint32_t)(fail_event[i] + 1) << 16;
        out[i] = r;
    }
}

}  // namespace

using lc::HostPool;

// One device's part of a batch in HBM.
struct DevBatch {
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
    uint16_t *table = nullptr; // a table model's rows (lc_batch.table), or null
    int64_t n_table = 0;
    int32_t *order = nullptr;  // LPT: keys by event count, descending
    bool t0_only = false;      // every key declared to fit the register lattice
    bool taggable = false;     // keys may be cut into segments (shared table, states 0..5, no op installs nil)
    bool seg_pays = false;     // sampled keys have quiescent points close enough for segments to pay
    bool validated = false;    // the host checked every event (else the device does: T0_STRICT or k_validate<true>)
    int64_t narrow_keys = 0;   // keys with at most 24 window slots (key_width): the WGL walk's LDS cache tier
    // Device storage behind the arrays above, grown on demand: a batch that is
    // re-uploaded (a context's staging batch for lc_check_batch) keeps it, so
    // a host-to-host check allocates nothing once its sizes have been seen.
    struct Mem {
        void *p = nullptr;
        size_t cap = 0;
    } mem[8];
    // pinned host staging of the per-key arrays and the transition table
    // (one copy per upload); `hmeta_done` marks the end of the last copy out
    // of it, so it is not rewritten while that copy may still read it
    char *hmeta = nullptr;
    size_t hmeta_cap = 0;
    hipEvent_t hmeta_done = nullptr;
    uint16_t *events16 = nullptr;    // 16-bit event words (mem[3]), or null: a register-tier batch
                                     // uploaded at 2 bytes per event (lc_batch.events16)
    mutable bool ev32_ready = true;  // `events` holds the 32-bit words (else widened, once, by the
                                     // first step whose kernels read them: all but k_spec)
    // the LPT order of the last upload and the offsets it was computed from
    // (a batch re-uploaded with the same offsets reuses it)
    std::vector<uint64_t> order_off;
    std::vector<int32_t> order_of;
    ~DevBatch() {
        if (hmeta_done) (void)hipEventSynchronize(hmeta_done);
        for (Mem &m : mem)
            if (m.p) (void)hipFree(m.p);
        if (hmeta) (void)hipHostFree(hmeta);
        if (hmeta_done) (void)hipEventDestroy(hmeta_done);
    }
};

struct lc_dev_batch {
    int n_parts = 0;
    int64_t n_keys = 0;
    int64_t key0[MAX_DEV + 1] = {};  // part g holds keys [key0[g], key0[g + 1])
    DevBatch *part[MAX_DEV] = {};
    ~lc_dev_batch() {
        for (DevBatch *p : part)
            if (p) {
                (void)hipSetDevice(p->device);
                delete p;
            }
    }
};

// Point p at m's storage, growing it to hold n elements of T.
template <class T>
static hipError_t grow(DevBatch::Mem &m, T *&p, size_t n) {
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
// Beyond CTL_BYTES in the 256-byte control block: counters[16..19] the WGL
// step's, [20] the keys a competition step hands to WGL, [24..31] the error words of the last 4 LC_DEV_ASYNC steps (slot =
// the step's sequence number mod 4: a refusal is reported by the wait for
// that step), [32..39] where k_take_err leaves what it read.
constexpr int ERR_RING = 24, ERR_TAKEN = 32;
// Most device memory the speculative segments' per-key workspaces may take.
constexpr uint64_t SPEC_WS_MAX_BYTES = 8ull << 30;

// One device of a context: its stream, scratch and result arrays.
struct Dev {
    const lc_opts *o = nullptr;  // the context's options
    int device = 0;
    int cu_count = 256;
    hipStream_t stream = nullptr;
    hipStream_t vstream = nullptr;  // validation of host-unchecked batches, beside T0
    hipStream_t cstream = nullptr;  // lc_check_node's chunked uploads, ahead of the searches
    hipStream_t estream = nullptr;  // lc_wait_step's error reads (behind no upload or step)
    static constexpr int NODE_CHUNKS = 4;
    DevBatch *chunk[NODE_CHUNKS] = {};
    hipEvent_t chunk_ready[NODE_CHUNKS] = {};
    hipEvent_t vin = nullptr, vdone = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr, et0 = nullptr, et3a = nullptr, et3b = nullptr;
    hipEvent_t ea0 = nullptr, ea1 = nullptr;  // span of the LC_DEV_ASYNC steps since lc_wait
    uint32_t n_async = 0;
    bool ea1_pending = false;  // asynchronous steps enqueued since ea1 was last recorded
    hipEvent_t ring[4] = {};  // end of each of the last 4 LC_DEV_ASYNC steps (lc_wait_step)
    uint64_t async_seq = 0;
    // scratch, grown on demand
    int64_t cap_keys = 0;
    int32_t *lists = nullptr;      // 5 x cap_keys: spill0, spill1, spill2, wide, old (T3L -> narrow T3)
    // one 96-byte control block, zeroed and read back in one operation each:
    // acc (4 x u64: probes, events, keys_done, T3L stream bytes) then counters (16 x i32:
    // n_spill0, n_spill1, n_spill2, n_wide, err bits, 1 + bad key, n_old, -,
    // tickets[8..15])
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
    // Device copies of T0's Args (read once per key): a ring of 4, so steps
    // alternating between result sets (the N > 1 bench) each find theirs
    // without a copy; a slot's pinned staging copy is rewritten only after
    // the copy out of it (args_ev) has run.
    static constexpr int ARGS_RING = 4;
    lcd::Args *dargs = nullptr;    // [ARGS_RING]
    lcd::Args *hargs = nullptr;    // [ARGS_RING] pinned
    hipEvent_t args_ev[ARGS_RING] = {};
    bool args_ok[ARGS_RING] = {};
    uint32_t args_next = 0;
    DevBatch *staged = nullptr;    // lc_check_batch's staging batch (device arrays reused)
    // T0-only steps skip re-zeroing the control block: the ticket continues
    // from where the previous such step left it.
    bool ticket_live = false;
    uint32_t ticket_next = 0;
    // key segments (register-tier steps of a batch of about one key per
    // SIMD): per-key cut points, segment results, work lists
    int64_t seg_keys = 0;
    uint32_t *seg_cnt = nullptr, *seg_end = nullptr, *seg_out = nullptr, *seg_work = nullptr;
    uint32_t *seg_rerun = nullptr, *seg_rerun_init = nullptr;
    int32_t *seg0_fev = nullptr, *seg_ctl = nullptr;
    // speculative segments: each wave's 9-10-pending workspace, the rerun list
    uint32_t *spec_ws = nullptr;
    size_t spec_ws_words = 0;
    uint32_t *spec_fin = nullptr;  // exact speculative segments: each run's saved set
    size_t spec_fin_words = 0;
    int32_t *spec_rr = nullptr;    // two rerun counts (used in turn), then the rerun list
    int64_t spec_rr_cap = 0;
    int spec_parity = 0;
    // node records (lc_check_node): this rank's block and the gathered node
    uint64_t *send = nullptr, *node = nullptr;
    int64_t node_cap = 0, node_n = 0;
    uint64_t *rec_out = nullptr;  // set around a node step's search: finish_key writes the records there
    uint64_t *hnode = nullptr;  // pinned landing area of the node's records (lc_check_node)
    int64_t hnode_cap = 0;
    // lc_check_node_async: two staging batches used in turn, so a step's
    // upload (on cstream) runs while the step before it searches; pipe_ready
    // = a slot's upload is done; the step that read a slot is done when its
    // ring event (async_seq pipe_seq[s]) is
    static constexpr int PIPE = 2;
    DevBatch *pipe[PIPE] = {};
    hipEvent_t pipe_ready[PIPE] = {};
    uint64_t pipe_seq[PIPE] = {};
    bool pipe_busy[PIPE] = {};
    uint64_t pipe_next = 0;
    // T3 (HBM tier) workspaces: narrow / wide configs
    struct Ws {
        char *base = nullptr;
        size_t bytes = 0;
        int slots = 0;
        lcd::HbmWs w{};
    } ws[2];
    // layered T3 workspace (device_layers.hip)
    struct LWs {
        char *base = nullptr;
        size_t bytes = 0;
        int slots = 0;
        lcd::LayWs w{};
    } lws;
    // knossos.wgl workspaces (device_wgl.hip): [0] tables sized to share at
    // most a share of the free HBM (WGL_SHARE_MAX), [1] tables the budget
    // fits, for the keys that outgrow [0]; zeroed once (entries are stamped)
    struct WWs {
        char *base = nullptr;
        size_t bytes = 0;
        lcd::WglWs layout{};  // the layout its contents were written under
        int slots = 0;
    } wws[2];
    uint32_t wgl_seq = 0;     // launches so far (the high half of every cache stamp)
    uint8_t *analyzer = nullptr;  // [cap_keys] LC_ALGO_* that answered each key
    ~Dev() {
        (void)hipSetDevice(device);
        if (stream) (void)hipStreamSynchronize(stream);
        dfree(lists); dfree(ctl); dfree(valid); dfree(fail_event);
        if (hctl) (void)hipHostFree(hctl);
        dfree(cause); dfree(peak); dfree(final_cfg); dfree(n_final);
        dfree(ws[0].base); dfree(ws[1].base); dfree(lws.base); dfree(dargs); dfree(send); dfree(node);
        dfree(wws[0].base); dfree(wws[1].base); dfree(analyzer);
        dfree(seg_cnt); dfree(seg_end); dfree(seg_out); dfree(seg_work); dfree(seg_rerun); dfree(seg_rerun_init);
        dfree(seg0_fev); dfree(seg_ctl); dfree(spec_ws); dfree(spec_rr); dfree(spec_fin);
        if (hargs) (void)hipHostFree(hargs);
        if (hnode) (void)hipHostFree(hnode);
        for (hipEvent_t &e : args_ev)
            if (e) (void)hipEventDestroy(e);
        delete staged;
        for (int i = 0; i < PIPE; ++i) {
            delete pipe[i];
            for (hipEvent_t e : {pipe_ready[i]})
                if (e) (void)hipEventDestroy(e);
        }
        for (int i = 0; i < NODE_CHUNKS; ++i) {
            delete chunk[i];
            if (chunk_ready[i]) (void)hipEventDestroy(chunk_ready[i]);
        }
        if (cstream) (void)hipStreamSynchronize(cstream);
        if (cstream) (void)hipStreamDestroy(cstream);
        if (estream) (void)hipStreamSynchronize(estream);
        if (estream) (void)hipStreamDestroy(estream);
        if (vstream) (void)hipStreamSynchronize(vstream);
        for (hipEvent_t e : {e0, e1, et0, et3a, et3b, ea0, ea1, vin, vdone})
            if (e) (void)hipEventDestroy(e);
        if (vstream) (void)hipStreamDestroy(vstream);
        for (hipEvent_t &e : ring)
            if (e) (void)hipEventDestroy(e);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

struct lc_ctx {
    lc_opts o{};
    int n_dev = 0;
    Dev *dev[MAX_DEV] = {};
    std::mutex mu;                 // one call at a time (include/lincheck.h)
    HostPool *pool = nullptr;      // validation / staging workers, created on first use
    HostPool *drivers = nullptr;   // one thread per device beyond the first
    uint32_t *hstage = nullptr;    // pinned copy of a batch's event words
    size_t hstage_cap = 0;
    // one process per GPU: RCCL communicator over the node's ranks
    ncclComm_t comm = nullptr;
    int rank = 0, size = 1;
    ~lc_ctx() {
        if (comm) {
            (void)hipSetDevice(dev[0]->device);
            (void)hipStreamSynchronize(dev[0]->stream);
            if (const Rccl *R = rccl()) (void)R->comm_destroy(comm);
        }
        for (Dev *d : dev) delete d;
        delete pool;
        delete drivers;
        if (hstage) (void)hipHostFree(hstage);
    }
};

static int ensure_capacity(Dev *c, int64_t n_keys) {
    if (n_keys <= c->cap_keys) return LC_OK;
    int64_t cap = std::max<int64_t>(n_keys, 1024);
    dfree(c->lists); dfree(c->valid); dfree(c->fail_event); dfree(c->cause);
    dfree(c->peak); dfree(c->final_cfg); dfree(c->n_final); dfree(c->analyzer);
    HIPCHK(dalloc(&c->lists, (size_t)cap * 5));
    HIPCHK(dalloc(&c->analyzer, (size_t)cap));
    HIPCHK(dalloc(&c->valid, (size_t)cap));
    HIPCHK(dalloc(&c->fail_event, (size_t)cap));
    HIPCHK(dalloc(&c->cause, (size_t)cap));
    HIPCHK(dalloc(&c->peak, (size_t)cap));
    HIPCHK(dalloc(&c->final_cfg, (size_t)cap * (size_t)c->o->max_final * 2));
    HIPCHK(dalloc(&c->n_final, (size_t)cap));
    c->cap_keys = cap;
    for (bool &v : c->args_ok) v = false;
    return LC_OK;
}

// Lay out (and if needed allocate) the layered T3 workspace for `want`
// blocks: four arrays of budget + slack entries (8 B) per block.
static int ensure_lay_ws(Dev *c, int want, int *slots_out) {
    Dev::LWs &W = c->lws;
    const uint64_t cap = c->o->max_configs + (uint64_t)lcd::t3l_slack() + 64;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    lcd::LayWs w{};
    size_t off = 0;
    w.off_S0 = off; off += al(cap * 8);
    w.off_S1 = off; off += al(cap * 8);
    w.off_I0 = off; off += al(cap * 8);
    w.off_I1 = off; off += al(cap * 8);
    w.slot_bytes = off;
    w.cap = (uint32_t)std::min<uint64_t>(cap, 0xFFFFFFFFull);
    size_t free_b = 0, total_b = 0;
    HIPCHK(hipMemGetInfo(&free_b, &total_b));
    int slots = std::min(want, c->cu_count);
    const size_t limit = W.bytes + free_b / 2;
    while (slots > 1 && (size_t)slots * w.slot_bytes > limit) slots /= 2;
    if ((size_t)slots * w.slot_bytes > limit)
        return lc::fail(LC_E_NOMEM, "T3 workspace: one slot needs %zu bytes (budget %llu)", w.slot_bytes,
                        (unsigned long long)c->o->max_configs);
    if (!W.base || W.w.slot_bytes != w.slot_bytes || W.slots < slots) {
        dfree(W.base);
        W.bytes = 0; W.slots = 0;
        HIPCHK(hipMalloc((void **)&W.base, (size_t)slots * w.slot_bytes));
        W.bytes = (size_t)slots * w.slot_bytes;
        W.slots = slots;
    }
    w.base = W.base;
    W.w = w;
    *slots_out = std::min(slots, W.slots);
    return LC_OK;
}

// Lay out (and if needed allocate) a T3 workspace for `want` blocks.
static int ensure_ws(Dev *c, int wide, int want, int *slots_out) {
    Dev::Ws &W = c->ws[wide];
    const size_t cfg = wide ? lcd::cfg_bytes_wide() : lcd::cfg_bytes_narrow();
    const uint64_t cap = c->o->max_configs + (uint64_t)lcd::t3_block() + 64;
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
    const int max_slots = c->o->deep_slots > 0 ? c->o->deep_slots : 2 * c->cu_count;
    int slots = std::min(want, max_slots);
    const size_t limit = (W.bytes ? W.bytes : 0) + free_b / 2;
    while (slots > 1 && (size_t)slots * w.slot_bytes > limit) slots /= 2;
    if ((size_t)slots * w.slot_bytes > limit)
        return lc::fail(LC_E_NOMEM, "T3 workspace: one slot needs %zu bytes (budget %llu)", w.slot_bytes,
                        (unsigned long long)c->o->max_configs);
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

static int dev_init(Dev *c, int device) {
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return lc::fail(LC_E_DEVICE, "lc_create: device %d is %s, this build targets gfx950", device, prop.gcnArchName);
    c->device = device;
    c->cu_count = prop.multiProcessorCount;
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&c->vstream, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&c->estream, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&c->vin, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&c->vdone, hipEventDisableTiming));
    for (hipEvent_t *e : {&c->e0, &c->e1, &c->et0, &c->et3a, &c->et3b, &c->ea0, &c->ea1}) HIPCHK(hipEventCreate(e));
    for (hipEvent_t &e : c->ring) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHK(dalloc(&c->ctl, 32));
    c->acc = c->ctl;
    c->counters = (int32_t *)(c->ctl + 4);
    HIPCHK(hipMemset(c->ctl, 0, 32 * sizeof(unsigned long long)));
    HIPCHK(hipHostMalloc((void **)&c->hctl, 32 * sizeof(unsigned long long), hipHostMallocDefault));
    std::memset(c->hctl, 0, 32 * sizeof(unsigned long long));
    HIPCHK(dalloc(&c->dargs, Dev::ARGS_RING));
    HIPCHK(hipHostMalloc((void **)&c->hargs, sizeof(lcd::Args) * Dev::ARGS_RING, hipHostMallocDefault));
    for (hipEvent_t &e : c->args_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return LC_OK;
}

extern "C" int lc_comm_id(uint8_t *out) {
    if (!out) return lc::fail(LC_E_INVALID, "lc_comm_id: null out");
    const Rccl *R = rccl();
    if (!R) return lc::fail(LC_E_DEVICE, "lc_comm_id: librccl.so.1 could not be loaded");
    ncclUniqueId id;
    RCCLCHK(R->get_unique_id(&id));
    std::memcpy(out, id.internal, LC_COMM_ID_BYTES);
    return LC_OK;
}

static std::atomic<int> g_live_ctx{0};

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
    if (o.path_flags & ~LC_PATH_ALL) return lc::fail(LC_E_INVALID, "lc_create: unknown path_flags 0x%x", o.path_flags);
    if ((o.path_flags & LC_PATH_SPLIT_ON) && (o.path_flags & LC_PATH_SPLIT_OFF))
        return lc::fail(LC_E_INVALID, "lc_create: LC_PATH_SPLIT_ON and _OFF together");
    if ((o.path_flags & LC_PATH_CHUNKS_ON) && (o.path_flags & LC_PATH_CHUNKS_OFF))
        return lc::fail(LC_E_INVALID, "lc_create: LC_PATH_CHUNKS_ON and _OFF together");
    if (o.spec_segs != 0 && o.spec_segs != 2 && o.spec_segs != 3 && o.spec_segs != 4 && o.spec_segs != 6 &&
        o.spec_segs != 8)
        return lc::fail(LC_E_INVALID, "lc_create: spec_segs must be 0, 2, 3, 4, 6 or 8");
    if (o.seg_len < 0) return lc::fail(LC_E_INVALID, "lc_create: seg_len < 0");
    // (a negative word is a ck2 past 32766 that wrapped: refused, not read as another value)
    if (o.spec_ck < 0 || (o.spec_ck && (((uint32_t)o.spec_ck & 0xFFFFu) == 0 || ((uint32_t)o.spec_ck >> 16) == 0)))
        return lc::fail(LC_E_INVALID, "lc_create: spec_ck must be 0 or (ck1 + 1) | (ck2 + 1) << 16, "
                                      "0 <= ck1 <= 65534, 0 <= ck2 <= 32766");
    if (o.n_devices < 0 || o.n_devices > MAX_DEV)
        return lc::fail(LC_E_INVALID, "lc_create: n_devices must be 0..%d", MAX_DEV);
    if (o.comm_size < 0 || o.comm_size > 4096 || (o.comm_size > 1 && (o.comm_rank < 0 || o.comm_rank >= o.comm_size)))
        return lc::fail(LC_E_INVALID, "lc_create: comm_rank %d of comm_size %d", o.comm_rank, o.comm_size);
    if (o.comm_size > 1 && o.n_devices > 1)
        return lc::fail(LC_E_INVALID, "lc_create: a rank of a multi-process node drives one device");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return lc::fail(LC_E_DEVICE, "lc_create: no HIP device visible");
    const int n = o.n_devices > 1 ? o.n_devices : 1;
    int list[MAX_DEV];
    for (int g = 0; g < n; ++g) {
        list[g] = o.n_devices > 1 ? o.devices[g] : o.device;
        if (list[g] < 0 || list[g] >= ndev) return lc::fail(LC_E_DEVICE, "lc_create: device %d of %d", list[g], ndev);
    }
    lc_ctx *c = new (std::nothrow) lc_ctx();
    if (!c) return lc::fail(LC_E_NOMEM, "lc_create: out of memory");
    c->o = o;
    for (int g = 0; g < n; ++g) {
        c->dev[g] = new (std::nothrow) Dev();
        if (!c->dev[g]) { delete c; return lc::fail(LC_E_NOMEM, "lc_create: out of memory"); }
        c->dev[g]->o = &c->o;
        c->n_dev = g + 1;
        int rc = dev_init(c->dev[g], list[g]);
        if (rc) { delete c; return rc; }
    }
    if (n > 1) c->drivers = new HostPool((unsigned)n - 1);
    // comm_size 1 with an id: a one-rank communicator (the exchange runs
    // through RCCL all the same)
    bool want_comm = o.comm_size > 1;
    for (uint8_t byte : o.comm_id) want_comm |= o.comm_size == 1 && byte != 0;
    if (want_comm) {
        const Rccl *R = rccl();
        if (!R) { delete c; return lc::fail(LC_E_DEVICE, "lc_create: librccl.so.1 could not be loaded"); }
        ncclUniqueId id;
        std::memcpy(id.internal, o.comm_id, LC_COMM_ID_BYTES);
        (void)hipSetDevice(list[0]);
        ncclResult_t r = R->comm_init_rank(&c->comm, o.comm_size, id, o.comm_rank);
        if (r != ncclSuccess) {
            c->comm = nullptr;
            delete c;
            return lc::fail(LC_E_DEVICE, "lc_create: ncclCommInitRank (rank %d of %d) failed: %s", o.comm_rank,
                            o.comm_size, R->error(r));
        }
        c->rank = o.comm_rank;
        c->size = o.comm_size;
    }
    *out = c;
    g_live_ctx.fetch_add(1);
    return LC_OK;
}

// The last context's destruction also gives back the host blocks the
// library keeps for reuse (page-locked memory is a limited resource; a JVM
// that checked once should not hold it for its life).  lc_trim does it
// at any time.
extern "C" void lc_destroy(lc_ctx *c) {
    if (!c) return;
    delete c;
    if (g_live_ctx.fetch_sub(1) == 1) lc::trim_host_caches();
}

// ---- validation -------------------------------------------------------------

// Per-event validation of a packed batch over the worker pool: every :ok
// names a pending slot, no :invoke lands in an occupied slot, every
// transition id is in range, no key uses more slots than its key_width says
// or (per-key tables) installs a state beyond its key_states.  Returns 0 or
// a reason code with the first bad key in *badkey; sets no error text.
// stage (optional): pinned host buffer that receives a copy of the event
// words; each thread copies the contiguous run of keys it validates, so the
// events are read once, in cache, on their way to the DMA engine.
// check = false: the copy alone (a batch T0 validates itself).
// Event word j of b: the 32-bit words, or the 16-bit ones widened (lc_pack
// gives only those when every word fits).
static inline uint32_t ev_at(const lc_batch *b, uint64_t j) {
    return b->events ? b->events[j] : LC_EV16_WIDE(b->events16[j]);
}

static int validate_events(const lc_batch *b, int64_t *badkey_out, uint32_t *stage, HostPool *hp, bool check = true) {
    const int64_t K = b->n_keys;
    unsigned nt = hp ? hp->size() : 1;
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
        if (stage && k1 > k0) {
            if (b->events)
                std::memcpy(stage + b->ev_off[k0], b->events + b->ev_off[k0], (b->ev_off[k1] - b->ev_off[k0]) * 4);
            else
                for (uint64_t j = b->ev_off[k0]; j < b->ev_off[k1]; ++j) stage[j] = LC_EV16_WIDE(b->events16[j]);
        }
        if (!check) return;
        for (int64_t k = k0; k < k1 && !bad[t]; ++k) {
            if (b->key_error && b->key_error[k]) continue;  // not searched
            const uint64_t tb = b->trans_off ? b->trans_off[k] : 0;
            const uint32_t ns = (b->trans_off && b->key_states) ? b->key_states[k] : 0xFFFFFFFFu;
            // a table model: each op's row must lie in table[] and name only
            // states of the key (a key beyond LC_WIDE_MAX_STATES is never stepped)
            const bool rows = b->table && ns <= LC_WIDE_MAX_STATES;
            uint64_t tmax = 0;
            uint64_t pend[2] = {0, 0};
            uint32_t width = 0;
            for (uint64_t j = b->ev_off[k]; j < b->ev_off[k + 1]; ++j) {
                const uint32_t ev = ev_at(b, j);
                const uint32_t s = LC_EV_SLOT(ev);
                // slot 127 marks ops beyond the encodable window: the search
                // stops (LC_CAUSE_WINDOW) before it could follow one.
                if (ev & LC_EV_OK_BIT) {
                    if (s == 127) continue;
                    if (!((pend[s >> 6] >> (s & 63)) & 1)) { bad[t] = 1; break; }
                    pend[s >> 6] &= ~(1ull << (s & 63));
                } else {
                    const uint64_t ti = tb + LC_EV_TRANS(ev);
                    if (ti >= (uint64_t)b->n_trans) { bad[t] = 2; break; }
                    const uint32_t d = b->trans[ti], f = d & 3u;
                    if (b->table) tmax = std::max(tmax, ti + 1);
                    else if ((f == LC_T_WRITE || f == LC_T_CAS) && (d >> 17) >= ns) { bad[t] = 5; break; }
                    if (s == 127) continue;
                    if ((pend[s >> 6] >> (s & 63)) & 1) { bad[t] = 3; break; }
                    pend[s >> 6] |= 1ull << (s & 63);
                    width = std::max(width, s + 1);
                }
            }
            if (!bad[t] && b->key_width && width > b->key_width[k]) bad[t] = 4;
            for (uint64_t ti = tb; rows && !bad[t] && ti < tmax; ++ti) {
                const uint64_t r0 = b->trans[ti];
                if (r0 + ns > (uint64_t)b->n_table) { bad[t] = 5; break; }
                for (uint64_t j = 0; j < ns; ++j)
                    if (b->table[r0 + j] != LC_TABLE_NONE && b->table[r0 + j] >= ns) { bad[t] = 5; break; }
            }
            if (bad[t]) badkey[t] = k;
        }
    };
    if (hp && nt > 1) hp->run(nt, work);
    else work(0);
    for (size_t t = 0; t < bad.size(); ++t)
        if (bad[t]) { *badkey_out = badkey[t]; return bad[t]; }
    return 0;
}

static int events_error(int why, int64_t key) {
    static const char *text[] = {"", ":ok of a slot with no pending op", "transition id out of range",
                                 ":invoke into an occupied slot", "uses more window slots than key_width says",
                                 "installs a state beyond key_states"};
    return lc::fail(LC_E_INVALID, "batch: key %lld: %s", (long long)key, text[why]);
}

// Host validation of everything but the events: offsets, the transition
// table, init_state.  O(keys + transitions).
static int validate_batch(const lc_batch *b) {
    if (!b || b->n_keys < 0) return lc::fail(LC_E_INVALID, "batch: bad n_keys");
    if (b->n_keys == 0) return LC_OK;
    if (!b->ev_off || !b->trans || b->n_trans <= 0) return lc::fail(LC_E_INVALID, "batch: missing arrays");
    if (b->n_trans > 0xFFFFFFFFll) return lc::fail(LC_E_INVALID, "batch: more than 2^32 transitions");
    if (b->ev_off[0] != 0) return lc::fail(LC_E_INVALID, "batch: ev_off[0] != 0");
    for (int64_t k = 0; k < b->n_keys; ++k) {
        if (b->ev_off[k + 1] < b->ev_off[k]) return lc::fail(LC_E_INVALID, "batch: ev_off not monotone at key %lld", (long long)k);
        if (b->ev_off[k + 1] - b->ev_off[k] > 0x7FFFFFFFull) return lc::fail(LC_E_INVALID, "batch: key %lld has > 2^31 events", (long long)k);
    }
    if (b->ev_off[b->n_keys] && !b->events && !b->events16) return lc::fail(LC_E_INVALID, "batch: events missing");
    if (b->init_state >= LC_STATE_NONE) return lc::fail(LC_E_INVALID, "batch: bad init_state");
    if (b->table) {
        // rows of a table model: trans[] are offsets into table[], checked per
        // key against its state count with the events (validate_events)
        if (b->n_table <= 0 || b->n_table > 0xFFFFFFFFll || !b->trans_off || !b->key_states)
            return lc::fail(LC_E_INVALID, "batch: a table model needs n_table, trans_off and key_states");
        return LC_OK;
    }
    for (int64_t i = 0; i < b->n_trans; ++i) {
        uint32_t d = b->trans[i];
        uint32_t f = d & 3u, bb = d >> 17;
        if ((f == LC_T_WRITE || f == LC_T_CAS) && bb >= LC_STATE_NONE)
            return lc::fail(LC_E_INVALID, "batch: transition %lld installs an invalid state", (long long)i);
    }
    return LC_OK;
}

// What the register tier needs to know of a batch before any upload: the
// state count of a shared table and whether every key is declared to fit T0
// (width, states, initial state).  A batch that does is validated by T0
// itself (T0_STRICT), so the host skips its per-event pass.
struct Shape {
    uint32_t shared_states = 0;
    bool t0_only = false;
    bool taggable = false;  // segments (lcd::SegArgs): shared table, states 0..5 from nil, nothing installs nil
    bool seg_pays = false;  // sampled keys: the longest stretch without a quiescent point is short
    bool host_checked = false;  // prepare_batch walked every event (table models: their rows too)
};

// Would key segments pay?  A segment ends only at a quiescent point, so the
// longest stretch without one bounds the segmented search, as the whole key
// bounds the unsegmented one.  Up to 4 keys spread over the batch are
// scanned on the host (a few thousand events); segments pay when their
// longest stretch is at most a quarter of their length.
static bool segments_pay(const lc_batch *b) {
    const int64_t K = b->n_keys;
    if (K <= 0 || (!b->events && !b->events16)) return false;
    uint64_t len = 0, gap = 0;
    for (int s = 0; s < 4; ++s) {
        const int64_t k = K * s / 4;
        const uint64_t e0 = b->ev_off[k], e1 = b->ev_off[k + 1];
        int64_t pend = 0;
        uint64_t last = e0;
        for (uint64_t j = e0; j < e1; ++j) {
            pend += (ev_at(b, j) & LC_EV_OK_BIT) ? -1 : 1;
            if (pend == 0) {
                gap = std::max(gap, j + 1 - last);
                last = j + 1;
            }
        }
        gap = std::max(gap, e1 - last);
        len += e1 - e0;
    }
    return len >= 4 * 512 && gap * 4 * 4 <= len;
}

static Shape batch_shape(const lc_batch *b) {
    Shape s;
    if (b->table) return s;  // a table model: the set tiers only (no register lattice)
    uint32_t mx = b->init_state;
    for (int64_t i = 0; i < b->n_trans; ++i) {
        const uint32_t t = b->trans[i], f = t & 3u, a = (t >> 2) & 0x7FFFu, bb = t >> 17;
        if ((f == LC_T_READ || f == LC_T_CAS) && a != LC_STATE_NONE) mx = std::max(mx, a);
        if (f == LC_T_WRITE || f == LC_T_CAS) mx = std::max(mx, bb);
    }
    s.shared_states = mx + 1;
    bool installs_nil = false;
    for (int64_t i = 0; i < b->n_trans; ++i) {
        const uint32_t t = b->trans[i], f = t & 3u;
        installs_nil |= (f == LC_T_WRITE || f == LC_T_CAS) && (t >> 17) == 0;
    }
    s.taggable = !b->trans_off && s.shared_states <= 6 && b->init_state == 0 && !installs_nil;
    s.seg_pays = s.taggable && segments_pay(b);
    const int64_t K = b->n_keys;
    bool ok = K > 0 && b->key_width && b->init_state < lcd::t0_max_states();
    for (int64_t k = 0; ok && k < K; ++k) ok = b->key_width[k] <= lcd::t0_max_width();
    if (ok && b->trans_off) {
        ok = b->key_states != nullptr;
        for (int64_t k = 0; ok && k < K; ++k) ok = b->key_states[k] <= lcd::t0_max_states() && b->key_states[k] > 0;
    } else if (ok) {
        ok = s.shared_states <= lcd::t0_max_states();
    }
    s.t0_only = ok;
    return s;
}

// Is p page-locked host memory (a DMA source without a bounce)?
static bool pinned(const void *p) {
    if (!p) return false;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at.type == hipMemoryTypeHost;
}

// Keys [k0, k1) of b as a batch of their own (ev_off rebased into `off`).
static lc_batch sub_batch(const lc_batch *b, int64_t k0, int64_t k1, std::vector<uint64_t> &off) {
    lc_batch s = *b;
    s.n_keys = k1 - k0;
    off.resize((size_t)(k1 - k0) + 1);
    const uint64_t base = b->ev_off[k0];
    for (int64_t k = k0; k <= k1; ++k) off[(size_t)(k - k0)] = b->ev_off[k] - base;
    s.ev_off = off.data();
    s.events = b->events ? b->events + base : nullptr;
    if (b->trans_off) s.trans_off = b->trans_off + k0;
    if (b->key_width) s.key_width = b->key_width + k0;
    if (b->key_states) s.key_states = b->key_states + k0;
    if (b->key_error) s.key_error = b->key_error + k0;
    if (b->events16) s.events16 = b->events16 + base;
    return s;
}

// Contiguous key shards of about equal event counts, one per device.
static void shard_keys(const lc_batch *b, int n, int64_t *key0) {
    const int64_t K = b->n_keys;
    const uint64_t tot = K ? b->ev_off[K] : 0;
    key0[0] = 0;
    for (int g = 1; g < n; ++g) {
        int64_t k = tot ? std::upper_bound(b->ev_off, b->ev_off + K + 1, tot * (uint64_t)g / (uint64_t)n) - b->ev_off - 1
                        : K * g / n;
        key0[g] = std::min(std::max(k, key0[g - 1]), K);
    }
    key0[n] = K;
}

// Copy a validated batch into d's device arrays (grown as needed).
// events_src: where the event words are copied from (b->events by default;
// lc_check_batch passes its pinned staging copy).  The per-key arrays and the
// transition table go through one pinned staging block and one copy; the
// event words are copied straight from the caller's (page-locked) memory.
// sync: wait for the copies (the caller may free its arrays on return);
// otherwise the caller keeps them alive until its stream has passed them.
static int upload_into(Dev *c, const lc_batch *b, DevBatch *d, const Shape &sh, bool validated,
                       const uint32_t *events_src = nullptr, bool sync = true, hipStream_t stream = nullptr) {
    lc::Range range("lincheck: upload");
    hipStream_t cs = stream ? stream : c->stream;
    const int64_t K = b->n_keys;
    d->device = c->device;
    d->n_keys = K;
    d->n_events = K ? b->ev_off[K] : 0;
    d->n_trans = b->n_trans > 0 ? b->n_trans : 1;
    d->init_state = b->init_state;
    d->has_trans_off = b->trans_off != nullptr;
    d->shared_states = sh.shared_states;
    d->t0_only = sh.t0_only;
    d->taggable = sh.taggable;
    d->seg_pays = sh.seg_pays;
    d->validated = validated;
    d->narrow_keys = 0;
    if (b->key_width && c->o->algorithm != LC_ALGO_LINEAR)
        for (int64_t k = 0; k < K; ++k) d->narrow_keys += b->key_width[k] <= 24;
    HIPCHK(hipSetDevice(c->device));
    // The event words first: their copy (the bulk of the bytes) runs while
    // the host stages the per-key arrays below.  A register-tier batch with
    // page-locked 16-bit words crosses the host link at 2 bytes per event and
    // is widened on the device (the register tier validates what it reads).
    HIPCHK(grow(d->mem[1], d->events, (size_t)d->n_events));
    // (a batch with no 32-bit words at all crosses as 16-bit words whatever
    // its tiers: prepare_batch widened them into events_src where the host
    // must, and the device widens them otherwise)
    const bool use16 = d->n_events && b->events16 &&
                       ((sh.t0_only && !(c->o->path_flags & LC_PATH_EV32) && (!events_src || events_src == b->events) &&
                         pinned(b->events16)) ||
                        (!b->events && !events_src));
    d->ev32_ready = !use16;
    if (use16) {
        // widened on the device only if a step's kernels need the 32-bit
        // words (dev_search); the speculative segments read these in place
        HIPCHK(grow(d->mem[3], d->events16, (size_t)d->n_events + 4));
        HIPCHK(hipMemcpyAsync(d->events16, b->events16, (size_t)d->n_events * 2, hipMemcpyHostToDevice, cs));
    } else if (d->n_events) {
        d->events16 = nullptr;
        HIPCHK(hipMemcpyAsync(d->events, events_src ? events_src : b->events, (size_t)d->n_events * 4,
                              hipMemcpyHostToDevice, cs));
    }
    // layout of the staging block (16-byte aligned pieces)
    auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
    const size_t Kz = (size_t)K;
    const size_t o_off = 0, o_order = al(o_off + (Kz + 1) * 8), o_trans = al(o_order + Kz * 4);
    const size_t o_toff = al(o_trans + (size_t)d->n_trans * 4);
    const size_t o_width = al(o_toff + (b->trans_off ? Kz * 4 : 0));
    const size_t o_states = al(o_width + (b->key_width ? Kz : 0));
    const size_t o_err = al(o_states + (b->key_states ? Kz * 2 : 0));
    const size_t bytes = al(o_err + (b->key_error ? Kz : 0));
    if (!d->hmeta_done) HIPCHK(hipEventCreateWithFlags(&d->hmeta_done, hipEventDisableTiming));
    HIPCHK(hipEventSynchronize(d->hmeta_done));  // the previous copy out of the block is done
    if (bytes > d->hmeta_cap) {
        if (d->hmeta) (void)hipHostFree(d->hmeta);
        d->hmeta = nullptr;
        d->hmeta_cap = 0;
        HIPCHK(hipHostMalloc((void **)&d->hmeta, bytes, hipHostMallocDefault));
        d->hmeta_cap = bytes;
    }
    char *h = d->hmeta;
    std::memcpy(h + o_off, b->ev_off, (Kz + 1) * 8);
    // LPT order: longest keys first (kept from the last upload when the
    // offsets are the same)
    int32_t *order = (int32_t *)(h + o_order);
    if (d->order_off.size() == Kz + 1 && std::memcmp(d->order_off.data(), b->ev_off, (Kz + 1) * 8) == 0) {
        std::memcpy(order, d->order_of.data(), Kz * 4);
    } else {
        std::vector<uint64_t> lk(Kz);  // (length << 32 | key), descending = LPT, ties by key
        for (size_t k = 0; k < Kz; ++k)
            lk[k] = (std::min<uint64_t>(b->ev_off[k + 1] - b->ev_off[k], 0xFFFFFFFFull) << 32) | (0xFFFFFFFFu - (uint32_t)k);
        std::sort(lk.begin(), lk.end(), std::greater<uint64_t>());
        for (size_t k = 0; k < Kz; ++k) order[k] = (int32_t)(0xFFFFFFFFu - (uint32_t)lk[k]);
        d->order_off.assign(b->ev_off, b->ev_off + Kz + 1);
        d->order_of.assign(order, order + Kz);
    }
    if (b->n_trans > 0) std::memcpy(h + o_trans, b->trans, (size_t)b->n_trans * 4);
    else std::memset(h + o_trans, 0, 4);
    if (b->trans_off) std::memcpy(h + o_toff, b->trans_off, Kz * 4);
    if (b->key_width) std::memcpy(h + o_width, b->key_width, Kz);
    if (b->key_states) std::memcpy(h + o_states, b->key_states, Kz * 2);
    if (b->key_error) std::memcpy(h + o_err, b->key_error, Kz);
    char *dm = nullptr;
    HIPCHK(grow(d->mem[0], dm, bytes));
    d->table = nullptr;
    d->n_table = b->table ? b->n_table : 0;
    if (b->table) {
        // a table model's rows (small next to the events; pageable source)
        HIPCHK(grow(d->mem[2], d->table, (size_t)b->n_table));
        HIPCHK(hipMemcpyAsync(d->table, b->table, (size_t)b->n_table * 2, hipMemcpyHostToDevice, cs));
    }
    d->ev_off = (uint64_t *)(dm + o_off);
    d->order = (int32_t *)(dm + o_order);
    d->trans = (uint32_t *)(dm + o_trans);
    d->trans_off = b->trans_off ? (uint32_t *)(dm + o_toff) : nullptr;
    d->key_width = b->key_width ? (uint8_t *)(dm + o_width) : nullptr;
    d->key_states = b->key_states ? (uint16_t *)(dm + o_states) : nullptr;
    d->key_error = b->key_error ? (uint8_t *)(dm + o_err) : nullptr;
    HIPCHK(hipMemcpyAsync(dm, h, bytes, hipMemcpyHostToDevice, cs));
    HIPCHK(hipEventRecord(d->hmeta_done, cs));
    if (sync) HIPCHK(hipStreamSynchronize(cs));
    return LC_OK;
}

// ---- one device's search ----------------------------------------------------

static int batch_error(int why, int64_t key) {
    return lc::fail(LC_E_INVALID, "batch: key %lld: %s", (long long)key,
                    (why & lcd::LC_BATCH_E_SLOTS)   ? "an :ok of a slot with no pending op, or an :invoke into an occupied slot"
                    : (why & lcd::LC_BATCH_E_TRANS) ? "transition id out of range, or a state beyond key_states"
                                                    : "key_width / key_states understate the key");
}

// After a readback of the control block: a malformed batch a synchronous
// step found.  The kernels name the key by its index in the caller's batch
// (Args::err_base).
static int take_error(Dev *c) {
    int32_t *cnt = (int32_t *)(c->hctl + 4);
    if (!cnt[4]) return LC_OK;
    const int why = cnt[4];
    const int64_t key = (int64_t)cnt[5] - 1;
    cnt[4] = cnt[5] = 0;
    HIPCHK(hipMemsetAsync(c->counters + 4, 0, 2 * sizeof(int32_t), c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return batch_error(why, key);
}

// The error words of the LC_DEV_ASYNC steps in ring slots `mask` (first
// `first`, when it is one of them), read and cleared on stream s.
// (enqueue, then ring_taken after the stream has passed it: dev_wait does
// both around its one synchronisation)
static int take_ring_enqueue(Dev *c, uint32_t mask, hipStream_t s) {
    hipLaunchKernelGGL(k_take_err, dim3(1), dim3(64), 0, s, c->counters + ERR_RING, mask, c->counters + ERR_TAKEN);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync((int32_t *)(c->hctl + 16), c->counters + ERR_TAKEN, 8 * sizeof(int32_t),
                          hipMemcpyDeviceToHost, s));
    return LC_OK;
}
static int ring_taken(Dev *c, int first) {
    const int32_t *h = (const int32_t *)(c->hctl + 16);
    int q = first >= 0 && h[2 * first] ? first : -1;
    for (int i = 0; i < 4 && q < 0; ++i)
        if (h[2 * i]) q = i;
    if (q < 0) return LC_OK;
    return batch_error(h[2 * q], (int64_t)h[2 * q + 1] - 1);
}
static int take_ring(Dev *c, uint32_t mask, int first, hipStream_t s) {
    const int rc = take_ring_enqueue(c, mask, s);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(s));
    return ring_taken(c, first);
}

// Segment arrays for n_keys keys (grown on demand).
static int ensure_segments(Dev *c, int64_t n_keys) {
    if (n_keys <= c->seg_keys && c->seg_ctl) return LC_OK;
    const int64_t cap = std::max<int64_t>(n_keys, 1024);
    const size_t per = (size_t)cap * lcd::SEG_MAX;
    dfree(c->seg_cnt); dfree(c->seg_end); dfree(c->seg_out); dfree(c->seg_work); dfree(c->seg_rerun);
    dfree(c->seg_rerun_init); dfree(c->seg0_fev); dfree(c->seg_ctl);
    HIPCHK(dalloc(&c->seg_cnt, (size_t)cap));
    HIPCHK(dalloc(&c->seg_end, per));
    HIPCHK(dalloc(&c->seg_out, per));
    HIPCHK(dalloc(&c->seg_work, per));
    HIPCHK(dalloc(&c->seg_rerun, (size_t)cap));
    HIPCHK(dalloc(&c->seg_rerun_init, (size_t)cap));
    HIPCHK(dalloc(&c->seg0_fev, (size_t)cap));
    HIPCHK(dalloc(&c->seg_ctl, 4));
    c->seg_keys = cap;
    return LC_OK;
}

// ---- knossos.wgl (device_wgl.hip) ---------------------------------------------

// Lowe's caches of the resident waves share at most this much of the free
// HBM (a third, and at most 96 GB); a key whose cache outgrows its share is
// searched again with a table the budget fits (fewer waves at once).  C4 at
// a budget of 2^22 (256 keys x a 2^23-entry table, 64 GB) then searches
// every key once; with a 4 GB share, 253 of its 256 keys outgrew their
// 2^19-entry tables and were searched twice (profiles/r05_c4_budget_sweep.json).
constexpr size_t WGL_SHARE_MAX = 96ull << 30;
constexpr uint64_t WGL_SPILL_ENTRIES = 1ull << 19;  // first tables when the budget's do not fit the share
constexpr uint32_t WGL_LDS_EVENTS = 8192;  // events (+ slot history) per key held in LDS

// Allocate (or reuse) WGL workspace `which` for `slots` waves of layout w.
// Contents written under another layout are cleared (a table entry is the
// key's by its stamp only where every earlier write was a table entry too).
static int ensure_wgl_ws(Dev *c, int which, const lcd::WglWs &w, int want, int *slots_out) {
    Dev::WWs &W = c->wws[which];
    size_t free_b = 0, total_b = 0;
    HIPCHK(hipMemGetInfo(&free_b, &total_b));
    int slots = std::max(want, 1);
    const size_t limit = W.bytes + free_b / 2;
    while (slots > 1 && (size_t)slots * w.slot_bytes > limit) slots /= 2;
    if ((size_t)slots * w.slot_bytes > limit)
        return lc::fail(LC_E_NOMEM, "WGL workspace: one wave needs %zu bytes (budget %llu)", w.slot_bytes,
                        (unsigned long long)c->o->max_configs);
    const size_t need = (size_t)slots * w.slot_bytes;
    if (!W.base || W.bytes < need) {
        if (W.base) HIPCHK(hipStreamSynchronize(c->stream));
        dfree(W.base);
        W.bytes = 0; W.slots = 0; W.layout = lcd::WglWs{};
        HIPCHK(hipMalloc((void **)&W.base, need));
        HIPCHK(hipMemsetAsync(W.base, 0, need, c->stream));  // stamp 0: never a key's
        W.bytes = need;
    } else if (!W.layout.same_layout(w)) {
        HIPCHK(hipMemsetAsync(W.base, 0, W.bytes, c->stream));
    }
    W.layout = w;
    W.slots = (int)std::min<size_t>(W.bytes / w.slot_bytes, (size_t)INT32_MAX);
    *slots_out = std::min(slots, W.slots);
    return LC_OK;
}

// knossos.wgl over keys order[0 .. n): n = n_order, or *n_in (a device
// count) when n_in is given (n_hint bounds it).  Results through a's arrays;
// analyzer (device, may be null) gets LC_ALGO_WGL per key searched.
static int run_wgl(Dev *c, const DevBatch *d, const lcd::Args &a, const int32_t *order, int32_t n_order,
                   const int32_t *n_in, int64_t n_hint, uint8_t *analyzer, lc_stats *st) {
    if (n_hint <= 0 || d->n_keys == 0) return LC_OK;
    const lc_opts &o = *c->o;
    // the longest key (LPT order: the first), for the frame stack and slot history
    uint64_t max_ev = 1;
    if (!d->order_of.empty()) {
        const int32_t k0 = d->order_of[0];
        max_ev = std::max<uint64_t>(1, d->order_off[(size_t)k0 + 1] - d->order_off[(size_t)k0]);
    }
    if (max_ev > 0x7FFFFFFFull) return lc::fail(LC_E_INVALID, "WGL: a key with more than 2^31 events");
    const uint64_t need = lcd::wgl_table_entries(o.max_configs);
    const int slots_a = (int)std::min<int64_t>(n_hint, (int64_t)c->cu_count * 4);
    // Lowe's tables of the first launch: the budget's table for every resident
    // wave -- twice that (a quarter full at the budget) when the share holds
    // it -- if a third of the free HBM holds them (C4 at 2^22: 64 GB); else
    // 2^19 entries, and the keys that pass half of that are searched again
    // with the budget's table (early, so the walk repeated is short).  Both
    // measured in round 5 against tables that grow into a pool.
    size_t free_b = 0, total_b = 0;
    HIPCHK(hipMemGetInfo(&free_b, &total_b));
    const uint64_t share = std::min<uint64_t>((c->wws[0].bytes + free_b) / 3, WGL_SHARE_MAX);
    const uint64_t per = 32ull * (uint64_t)slots_a;
    uint64_t t_a = need * per <= share ? need : std::min<uint64_t>(need, WGL_SPILL_ENTRIES);
    if (t_a == need && 2 * need * per <= share) t_a = 2 * need;
    if (o.path_flags & LC_PATH_WGL_SMALL) t_a = 1ull << 14;
    t_a = std::min(t_a, 2 * need);
    const lcd::WglWs wa = lcd::wgl_layout(o.max_configs, (uint32_t)max_ev, (uint32_t)t_a);
    int slots = 0;
    int rc = ensure_wgl_ws(c, 0, wa, slots_a, &slots);
    if (rc) return rc;
    int32_t *const ctl = c->counters + 16;  // [0] -, [1] ticket, [2] spill count, [3] spill ticket
    int32_t *const spill = c->lists + 4 * c->cap_keys;
    HIPCHK(hipMemsetAsync(ctl, 0, 4 * sizeof(int32_t), c->stream));
    lcd::WglArgs w{};
    w.ev_off = a.ev_off; w.events = a.events; w.trans = a.trans; w.trans_off = a.trans_off;
    w.key_states = a.key_states; w.key_error = a.key_error; w.table = a.table;
    w.init_state = a.init_state; w.n_trans = a.n_trans; w.budget = o.max_configs; w.max_final = o.max_final;
    // LDS per block: the first events of the key, their slot history and
    // descriptors (12 B per event), the LDS tier of the cache (8 B per entry; narrow keys), the
    // frame ring -- within a fourth of the CU's 160 KB when the launch has
    // four keys per CU (one wave each), up to 64 KB otherwise
    // (a key whose events do not all fit is searched from HBM; more than 64
    // KB per block when the launch has about one key per CU: C4's 10,000
    // events take 120 KB)
    const int64_t per_cu = std::min<int64_t>(4, std::max<int64_t>(1, (n_hint + c->cu_count - 1) / c->cu_count));
    size_t lds_cap = (160u << 10) / (size_t)per_cu - 1024;
    if (!lcd::wgl_allow_lds(lds_cap)) lds_cap = std::min<size_t>(lds_cap, 64u << 10);
    w.lds_events = (uint32_t)std::min<uint64_t>(max_ev, WGL_LDS_EVENTS);
    if (d->narrow_keys == 0) w.lds_events = (uint32_t)std::min<uint64_t>(max_ev, 3 * WGL_LDS_EVENTS / 2);
    if (o.path_flags & LC_PATH_WGL_EV_HBM) w.lds_events = 0;  // every key's events from HBM (tests)
    w.lds_tab = d->narrow_keys > 0 ? 4096u : 0u;
    w.lds_events = (w.lds_events + 1u) & ~1u;  // even: the cache tier after it is 8-byte aligned
    while (lcd::wgl_lds_bytes(w.lds_events, w.lds_tab) > lds_cap) {
        if (w.lds_tab > 1024) w.lds_tab /= 2;
        else w.lds_events = w.lds_events > 1024 ? w.lds_events - 256 : (w.lds_events / 2 + 1u) & ~1u;
    }
    w.key_width = a.key_width;
    w.order = order; w.n_order = n_order; w.n_in = n_in;
    w.ticket = ctl + 1;
    w.err = a.err;
    w.gen_base = (uint64_t)(++c->wgl_seq) << 32;
    w.spill_at = t_a < need ? (uint32_t)(t_a / 2 - 1) : 0u;
    w.spill = spill; w.n_spill = ctl + 2;
    w.ws = wa;
    w.ws.base = c->wws[0].base;
    w.valid = a.valid; w.fail_event = a.fail_event; w.cause = a.cause; w.peak = a.peak;
    w.final_cfg = a.final_cfg; w.n_final = a.n_final; w.analyzer = analyzer; w.rec = a.rec;
    w.ev_count = a.ev_count; w.keys_done = a.keys_done;
    w.probes = o.algorithm == LC_ALGO_WGL ? a.probes : nullptr;  // (competition: :linear's probe count)
    HIPCHK(hipEventRecord(c->et3a, c->stream));
    HIPCHK(lcd::launch_wgl(w, slots, c->stream));
    int32_t n_spill = 0;
    if (w.spill_at) {
        int32_t *h = (int32_t *)(c->hctl + 4) + 18;
        HIPCHK(hipMemcpyAsync(h, ctl + 2, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        n_spill = *h;
        if (n_spill > 0) {
            const lcd::WglWs wb = lcd::wgl_layout(o.max_configs, (uint32_t)max_ev, 0);
            rc = ensure_wgl_ws(c, 1, wb, (int)std::min<int64_t>(n_spill, (int64_t)c->cu_count * 4), &slots);
            if (rc) return rc;
            w.order = spill; w.n_order = 0; w.n_in = ctl + 2;
            w.ticket = ctl + 3;
            w.gen_base = (uint64_t)(++c->wgl_seq) << 32;
            w.spill_at = 0;
            w.ws = wb;
            w.ws.base = c->wws[1].base;
            HIPCHK(lcd::launch_wgl(w, slots, c->stream));
        }
    }
    HIPCHK(hipEventRecord(c->et3b, c->stream));
    if (st) st->wgl_spilled += (uint64_t)n_spill;
    return LC_OK;
}

enum ResMode { RES_HOST = 0, RES_DEV = 1, RES_CTX = 2 };

// Search d on c.  RES_HOST: r's arrays are host memory and receive the
// results; RES_DEV: r's arrays are device memory on c; RES_CTX: results stay
// in c's own device arrays (r unused).  allow_async: a step that is T0 alone
// is only enqueued (*enqueued = true; errors surface at the next wait).
// k_spec_rerun's workgroups at most (0: one per CU; A/B: make variant
// VFLAGS=-DLC_SPEC_RERUN_BLOCKS=n -- 16 and 64 measured the same as 256 on
// C2 in round 5, 0.2552-0.2556 ms per step)
#ifndef LC_SPEC_RERUN_BLOCKS
#define LC_SPEC_RERUN_BLOCKS 0
#endif
static int dev_search(Dev *c, const DevBatch *d, const lc_result *r, ResMode mode, bool allow_async, int64_t key0,
                      lc_stats *st, bool *enqueued = nullptr, int64_t res_off = 0) {
    lc::Range range("lincheck: search");
    if (enqueued) *enqueued = false;
    auto t0 = std::chrono::steady_clock::now();
    HIPCHK(hipSetDevice(c->device));
    const int64_t K = d->n_keys;
    if (K > 0x7FFFFFFF) return lc::fail(LC_E_INVALID, "lc_check_device: too many keys");
    int rc = ensure_capacity(c, K);
    if (rc) return rc;
    const lc_opts &o = *c->o;

    lcd::Args a{};
    a.ev_off = d->ev_off; a.events = d->events; a.trans = d->trans; a.trans_off = d->trans_off;
    a.key_width = d->key_width; a.key_states = d->key_states; a.key_error = d->key_error;
    a.table = d->table;
    a.init_state = d->init_state; a.shared_states = d->shared_states;
    a.n_trans = (uint32_t)d->n_trans;
    // T0_STRICT: a register-tier batch the host did not walk (T0 refuses a key
    // that does not fit instead of spilling it); other unwalked batches get
    // the general validation kernel ahead of the set tiers
    a.strict = (!d->validated && d->t0_only) ? 1 : 0;
    const bool gen_validate = !d->validated && !d->t0_only;
    a.budget = o.max_configs; a.max_final = o.max_final; a.debug_mode = o.debug_mode;
    a.count_probes = (o.flags & LC_OPT_COUNT_PROBES) ? 1 : 0;
    if (mode == RES_DEV) {
        a.valid = r->valid; a.fail_event = r->fail_event; a.cause = r->cause;
        a.peak = r->peak_configs; a.final_cfg = r->final_configs; a.n_final = r->n_final;
    } else {
        a.valid = c->valid + res_off; a.fail_event = c->fail_event + res_off; a.cause = c->cause + res_off;
        a.peak = (mode == RES_HOST && r->peak_configs) ? c->peak : nullptr;
        a.final_cfg = (mode == RES_HOST && r->final_configs) ? c->final_cfg : nullptr;
        a.n_final = (mode == RES_HOST && r->n_final) ? c->n_final : nullptr;
    }
    a.rec = c->rec_out ? c->rec_out + res_off : nullptr;
    a.probes = c->acc + 0; a.ev_count = c->acc + 1; a.keys_done = c->acc + 2; a.stream_bytes = c->acc + 3;
    a.err = c->counters + 4;
    a.err_base = (int32_t)key0;  // malformed keys are reported by their index in the caller's batch
    a.list_cap = (int32_t)c->cap_keys;
    // which analysis answered each key (lc_result.analyzer)
    uint8_t *const analyzer = mode == RES_DEV ? r->analyzer : (mode == RES_HOST && r->analyzer) ? c->analyzer : nullptr;
    if (analyzer && K > 0 && o.algorithm != LC_ALGO_WGL)
        HIPCHK(hipMemsetAsync(analyzer, LC_ALGO_LINEAR, (size_t)K, c->stream));
    if (o.algorithm == LC_ALGO_WGL) {
        // knossos.wgl's own search (device_wgl.hip) for every key
        if (enqueued) *enqueued = false;
        HIPCHK(hipMemsetAsync(c->ctl, 0, 4 * sizeof(unsigned long long) + 4 * sizeof(int32_t), c->stream));
        HIPCHK(hipMemsetAsync(c->counters + 6, 0, 10 * sizeof(int32_t), c->stream));
        c->ticket_live = false;
        if (!d->ev32_ready && d->n_events) {
            const uint64_t n4 = (d->n_events + 3) / 4;
            const int blocks = (int)std::min<uint64_t>((n4 + 255) / 256, (uint64_t)c->cu_count * 8);
            hipLaunchKernelGGL(k_widen16, dim3(std::max(blocks, 1)), dim3(256), 0, c->stream, d->events16, d->events,
                               d->n_events);
            HIPCHK(hipGetLastError());
            d->ev32_ready = true;
        }
        if (a.n_final && K > 0) HIPCHK(hipMemsetAsync(a.n_final, 0, (size_t)K * 4, c->stream));
        HIPCHK(hipEventRecord(c->e0, c->stream));
        if (!d->validated && K > 0) {  // the per-event checks the host skipped, ahead of the walk
            lcd::Args av = a;
            av.n_order = (int32_t)K;
            HIPCHK(lcd::launch_validate(av, c->stream, true));
        }
        lc_stats ws{};
        rc = run_wgl(c, d, a, d->order, (int32_t)K, nullptr, K, analyzer, &ws);
        if (rc) return rc;
        HIPCHK(hipEventRecord(c->e1, c->stream));
        HIPCHK(hipMemcpyAsync(c->hctl, c->ctl, CTL_BYTES, hipMemcpyDeviceToHost, c->stream));
        if (mode == RES_HOST && K > 0) {
            HIPCHK(hipMemcpyAsync(r->valid, c->valid, (size_t)K, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipMemcpyAsync(r->fail_event, c->fail_event, (size_t)K * 4, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipMemcpyAsync(r->cause, c->cause, (size_t)K, hipMemcpyDeviceToHost, c->stream));
            if (r->peak_configs)
                HIPCHK(hipMemcpyAsync(r->peak_configs, c->peak, (size_t)K * 4, hipMemcpyDeviceToHost, c->stream));
            if (r->final_configs)
                HIPCHK(hipMemcpyAsync(r->final_configs, c->final_cfg, (size_t)K * o.max_final * 16,
                                      hipMemcpyDeviceToHost, c->stream));
            if (r->n_final)
                HIPCHK(hipMemcpyAsync(r->n_final, c->n_final, (size_t)K * 4, hipMemcpyDeviceToHost, c->stream));
            if (r->analyzer)
                HIPCHK(hipMemcpyAsync(r->analyzer, c->analyzer, (size_t)K, hipMemcpyDeviceToHost, c->stream));
        }
        HIPCHK(hipStreamSynchronize(c->stream));
        rc = take_error(c);
        if (rc) return rc;
        float ms = 0, msw = 0;
        HIPCHK(hipEventElapsedTime(&ms, c->e0, c->e1));
        if (K > 0) HIPCHK(hipEventElapsedTime(&msw, c->et3a, c->et3b));
        if (st) {
            *st = lc_stats{};
            st->kernel_ms = ms;
            st->wgl_ms = msw;
            st->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            st->lds_keys = c->hctl[2];
            st->wgl_keys = c->hctl[2];
            st->wgl_steps = c->hctl[1];
            st->events = c->hctl[1];
            st->probes = c->hctl[0];  // Lowe's cache lookups
            st->wgl_spilled = ws.wgl_spilled;
        }
        return LC_OK;
    }
    const bool competition = o.algorithm == LC_ALGO_COMPETITION;
    if (competition) allow_async = false;  // the WGL step needs the :linear step's causes
    int32_t *spill0 = c->lists, *spill1 = c->lists + c->cap_keys, *spill2 = c->lists + 2 * c->cap_keys;
    int32_t *wide = c->lists + 3 * c->cap_keys, *old_narrow = c->lists + 4 * c->cap_keys;
    int32_t *n_spill0 = c->counters + 0, *n_spill1 = c->counters + 1, *n_spill2 = c->counters + 2;
    int32_t *n_wide = c->counters + 3;

    // Nothing counted and no key can leave T0: no T1/T2 launches, no counter
    // readback and no control-block memset -- the step is T0 alone (plus the
    // result download when the results go to host memory).
    const bool t0_step = K > 0 && d->t0_only && !(o.flags & LC_OPT_COUNT_PROBES);
    const bool async = t0_step && allow_async && mode != RES_HOST;
    if (!async && c->ea1_pending) {  // the asynchronous steps' span ends before this one
        HIPCHK(hipEventRecord(c->ea1, c->stream));
        c->ea1_pending = false;
    }
    // an enqueued step reports a malformed batch through its own error words
    if (async) a.err = c->counters + ERR_RING + 2 * (int)(c->async_seq % 4);
    // Key segments (device_lattice.hip): verdicts only, a batch of about one
    // key per SIMD or fewer (where each key's serial chain is exposed), and
    // quiescent points close enough for the cuts to pay (segments_pay: on
    // C2, whose clients think about as long as an op takes, the longest
    // stretch without one is most of a key, so its keys stay whole).
    // lc_opts.path_flags LC_PATH_SPLIT_ON / _OFF pin the choice (A/B and tests).
    const bool fast = !a.peak && !a.final_cfg && o.max_configs >= 16ull * 64 * 32;
    const bool want = (o.path_flags & LC_PATH_SPLIT_ON) ? true : (o.path_flags & LC_PATH_SPLIT_OFF) ? false : d->seg_pays;
    const bool split = t0_step && fast && d->taggable && want && K <= (int64_t)c->cu_count * 8;
    if (split) {
        rc = ensure_segments(c, K);
        if (rc) return rc;
    }
    // Speculative segments (device_lattice.hip): the same regime without
    // quiescent points -- every key a workgroup of `segs` waves, about four
    // segment waves per SIMD in all (C2: 1,000 keys x 4).  The kernel's 80
    // VGPRs would allow six, but 6-wave workgroups land unevenly on a CU's
    // four SIMDs (5-7 waves each): C2 0.357 ms at 4 segments per key, 0.406
    // at 6, 0.386 at 8.  lc_opts: LC_PATH_SPEC_OFF turns them off, spec_segs
    // pins the segments per key.
    //
    // Large batches too (C3 shards: 2 segments per key; 12,500 x 2,000 4.44
    // ms against 5.51 unsegmented, the whole C3 key space 33.2 against 38.0).
    // More segments than waves (a key's waves taking its segments from a
    // block-local queue, see k_spec) measured slower: C2 8 segments on 4 waves
    // 0.302 ms, 12 on 4 0.332, against 0.273 for 4 on 4; a C3 shard 4 on 2
    // 4.75 ms, 8 on 2 5.30, against 4.40 for 2 on 2.
    int segs = K > 0 ? (int)std::min<int64_t>(8, (int64_t)c->cu_count * 4 * 4 / std::max<int64_t>(K, 1)) : 0;
    segs = segs >= 8 ? 8 : segs >= 4 ? 4 : K > 0 ? 2 : 0;
    // Final configs wanted and no set sizes (the Jepsen-shaped checkers):
    // the segments with exact sets (Knossos's S, not its closure), each run
    // saving its set at its end or death, the true run's written as the
    // key's final configs (k_spec<.., EX>).
    const bool exact_spec = !a.peak && a.final_cfg && a.n_final && o.max_configs >= 16ull * 64 * 32;
    // 8 per key while 8 x keys waves are resident at the 8-wave build's 8
    // per SIMD (device_search.hpp LC_SPEC8_WAVES).  The exact segments too
    // since round 6 (spill-free builds, overlapped verifying runs;
    // tools/ex_segs_ab.py, records equal): C2 0.2843 -> 0.2530 ms, a C5-shaped
    // batch of another seed 0.2822 -> 0.2627, BASELINE's C5 0.2717 -> 0.2755.
    // (Round 5, before both: C5 0.289 -> 0.352 ms with 8.)
    if (LC_SPEC8_WAVES >= 8 && (fast || exact_spec) && K > 0 && K * 8 <= (int64_t)c->cu_count * 4 * 8) segs = 8;
    if (o.spec_segs) segs = o.spec_segs;
    if (exact_spec && !fast) segs = segs >= 8 ? 8 : segs >= 4 ? 4 : 2;  // the exact builds
    const int waves = segs;
    bool spec = !split && t0_step && (fast || exact_spec) && segs >= 2 && !(o.path_flags & LC_PATH_SPEC_OFF);
    // The segments' workspaces are per key: a batch whose keys
    // would need more than SPEC_WS_MAX_BYTES of them takes the unsegmented
    // register tier, whose workspace is per resident wave.
    if (spec && (uint64_t)(lcd::spec_ws_words(K, waves) + (exact_spec && !fast ? lcd::spec_fin_words(K, segs) : 0)) * 4 >
                    SPEC_WS_MAX_BYTES)
        spec = false;
    if (spec) {
        const size_t need = lcd::spec_ws_words(K, waves);
        if (need > c->spec_ws_words) {
            if (c->n_async) HIPCHK(hipStreamSynchronize(c->stream));
            dfree(c->spec_ws);
            c->spec_ws = nullptr;
            c->spec_ws_words = 0;
            HIPCHK(dalloc(&c->spec_ws, need));
            c->spec_ws_words = need;
        }
        const size_t fneed = exact_spec && !fast ? lcd::spec_fin_words(K, segs) : 0;
        if (fneed > c->spec_fin_words) {
            if (c->n_async) HIPCHK(hipStreamSynchronize(c->stream));
            dfree(c->spec_fin);
            c->spec_fin = nullptr;
            c->spec_fin_words = 0;
            HIPCHK(dalloc(&c->spec_fin, fneed));
            c->spec_fin_words = fneed;
        }
        if (K + 2 > c->spec_rr_cap) {
            if (c->n_async) HIPCHK(hipStreamSynchronize(c->stream));
            dfree(c->spec_rr);
            c->spec_rr = nullptr;
            c->spec_rr_cap = 0;
            HIPCHK(dalloc(&c->spec_rr, (size_t)K + 2));
            HIPCHK(hipMemsetAsync(c->spec_rr, 0, 2 * sizeof(int32_t), c->stream));
            c->spec_rr_cap = K + 2;
        }
    }
    // The speculative segments read 16-bit event words in place; every other
    // kernel reads the 32-bit form, widened here once per upload.
    const uint16_t *ev16 = (spec && d->events16) ? d->events16 : nullptr;
    const uint32_t t0_path = K == 0 || d->table ? LC_T0_PATH_NONE
                             : split            ? LC_T0_PATH_SEGMENTS
                             : spec             ? LC_T0_PATH_SPEC
                                                : LC_T0_PATH_LATTICE;
    if (!ev16 && !d->ev32_ready && d->n_events) {
        const uint64_t n4 = (d->n_events + 3) / 4;
        const int blocks = (int)std::min<uint64_t>((n4 + 255) / 256, (uint64_t)c->cu_count * 8);
        hipLaunchKernelGGL(k_widen16, dim3(std::max(blocks, 1)), dim3(256), 0, c->stream, d->events16, d->events,
                           d->n_events);
        HIPCHK(hipGetLastError());
        d->ev32_ready = true;
    }
    uint32_t ticket_base = 0;
    if (t0_step && c->ticket_live && !competition) {
        ticket_base = c->ticket_next;
    } else {
        // zero everything but the error words (a malformed batch reported at
        // the next wait keeps them until then)
        HIPCHK(hipMemsetAsync(c->ctl, 0, 4 * sizeof(unsigned long long) + 4 * sizeof(int32_t), c->stream));
        HIPCHK(hipMemsetAsync(c->counters + 6, 0, 10 * sizeof(int32_t), c->stream));
    }
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
    // Args: a ring slot holding these Args, else the next slot, refreshed
    // (device copies are rewritten in stream order, after the launches that
    // read them)
    int aslot = -1;
    for (int q = 0; q < Dev::ARGS_RING && aslot < 0; ++q)
        if (c->args_ok[q] && std::memcmp(c->hargs + q, &a0, sizeof a0) == 0) aslot = q;
    if (aslot < 0) {
        aslot = (int)(c->args_next++ % Dev::ARGS_RING);
        HIPCHK(hipEventSynchronize(c->args_ev[aslot]));  // its staging copy has been read
        std::memcpy(c->hargs + aslot, &a0, sizeof a0);
        HIPCHK(hipMemcpyAsync(c->dargs + aslot, c->hargs + aslot, sizeof(lcd::Args), hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipEventRecord(c->args_ev[aslot], c->stream));
        c->args_ok[aslot] = true;
    }
    lcd::Args *const dargs = c->dargs + aslot;
    // timing events only where their times are read (each recorded event
    // costs the stream a few microseconds between kernels): an enqueued step
    // is timed by the span ea0 .. ea1 alone
    if (!async) HIPCHK(hipEventRecord(c->e0, c->stream));
    if (async && c->n_async == 0) HIPCHK(hipEventRecord(c->ea0, c->stream));
    const bool side_validate = K > 0 && ((a.strict && !spec) || gen_validate);
    if (side_validate) {
        // the event-by-event validation the host skipped: on the second
        // stream, beside T0, joined before the set tiers and the readback
        HIPCHK(hipEventRecord(c->vin, c->stream));
        HIPCHK(hipStreamWaitEvent(c->vstream, c->vin, 0));
        lcd::Args av = a;
        av.n_order = (int32_t)K;
        HIPCHK(lcd::launch_validate(av, c->vstream, gen_validate));
        HIPCHK(hipEventRecord(c->vdone, c->vstream));
    }
    if (split) {
        lcd::SegArgs sa{};
        sa.ev_off = d->ev_off; sa.events = d->events; sa.trans = d->trans; sa.key_error = d->key_error;
        sa.n_trans = (uint32_t)d->n_trans; sa.n_keys = (int32_t)K; sa.max_seg = lcd::SEG_MAX;
        // segments of about fill x (resident waves / keys) per key
        const int grid = c->cu_count * 12;
        const double per_key = std::max(1.0, 2.0 * grid / (double)K);
        sa.seg_len = (uint32_t)std::max<double>(64.0, (double)d->n_events / (double)K / per_key);
        if (o.seg_len > 0) sa.seg_len = (uint32_t)o.seg_len;
        sa.seg_cnt = c->seg_cnt; sa.seg_end = c->seg_end; sa.seg_out = c->seg_out; sa.seg0_fev = c->seg0_fev;
        sa.work = c->seg_work; sa.rerun = c->seg_rerun; sa.rerun_init = c->seg_rerun_init; sa.ctl = c->seg_ctl;
        sa.err = a.err; sa.valid = a.valid; sa.fail_event = a.fail_event; sa.cause = a.cause;
        sa.rec = a.rec;
        sa.strict = a.strict;
        sa.err_base = a.err_base;
        HIPCHK(hipMemsetAsync(c->seg_ctl, 0, 4 * sizeof(int32_t), c->stream));
        HIPCHK(lcd::launch_segments(sa, grid, c->stream));
        if (!async) HIPCHK(hipEventRecord(c->et0, c->stream));
    } else if (spec) {
        // (spec_ck == 0: the defaults; else (ck1 + 1) | (ck2 + 1) << 16)
        const uint32_t ck1 = o.spec_ck ? ((uint32_t)o.spec_ck & 0xFFFFu) - 1u : 32u;
        const uint32_t ck2 = o.spec_ck ? ((uint32_t)o.spec_ck >> 16) - 1u : 120u;
        // the validation of a host-unchecked batch runs in extra blocks of
        // the same launch (a second stream cost ~40 us of cross-stream waits)
        const int vblocks = a.strict ? (int)std::min<int64_t>(K, c->cu_count) : 0;
        HIPCHK(lcd::launch_spec(a0, dargs, segs, waves, c->spec_ws, c->spec_rr, c->spec_parity, ck1, ck2,
                                // (rerun blocks: the launch usually finds no
                                // key, so one block per CU keeps its dispatch
                                // short; a longer rerun list walks the grid)
                                LC_SPEC_RERUN_BLOCKS > 0 ? LC_SPEC_RERUN_BLOCKS : c->cu_count, vblocks, ev16,
                                (o.path_flags & LC_PATH_SPEC_COST) != 0,
                                !(o.path_flags & LC_PATH_SPEC_NOPRIO),
                                K * waves > (int64_t)c->cu_count * 16,  // more keys than one resident round
                                exact_spec && !fast ? c->spec_fin : nullptr,
                                !(o.path_flags & LC_PATH_SPEC_NOSTAGE), c->stream));
        c->spec_parity ^= 1;
        if (!async) HIPCHK(hipEventRecord(c->et0, c->stream));
    } else if (K > 0 && !d->table) {
        HIPCHK(lcd::launch_t0(a0, dargs, g0, t0_wide, c->stream, ticket_base));
        if (!async) HIPCHK(hipEventRecord(c->et0, c->stream));
    } else if (K > 0) {
        HIPCHK(hipEventRecord(c->et0, c->stream));  // a table model: no register lattice
    }
    if (side_validate) HIPCHK(hipStreamWaitEvent(c->stream, c->vdone, 0));
    if (async) {
        // (the span's end, ea1, is recorded by dev_wait after the last
        // enqueued step: one timing event per step cost the stream a few
        // microseconds between searches)
        HIPCHK(hipEventRecord(c->ring[c->async_seq % 4], c->stream));
        c->ea1_pending = true;
        ++c->async_seq;
        ++c->n_async;
        c->ticket_next = (split || spec) ? ticket_base : ticket_base + (uint32_t)K + (uint32_t)g0;
        c->ticket_live = true;
        if (st) {  // times come from lc_wait
            *st = lc_stats{};
            st->t0_path = t0_path;
            st->ev_word_bytes = t0_path ? (ev16 ? 2u : 4u) : 0u;
        }
        if (enqueued) *enqueued = true;
        return LC_OK;
    }
    if (K > 0 && !t0_step) {
        // T1: LDS hash sets
        lcd::Args a1 = a;
        a1.order = spill0; a1.n_order = 0; a1.n_in = n_spill0; a1.ticket = c->counters + 9;
        if (d->table) { a1.order = d->order; a1.n_order = (int32_t)K; a1.n_in = nullptr; }  // every key
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
        if (mode == RES_HOST && K > 0) {
            HIPCHK(hipMemcpyAsync(r->valid, c->valid, (size_t)K, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipMemcpyAsync(r->fail_event, c->fail_event, (size_t)K * 4, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipMemcpyAsync(r->cause, c->cause, (size_t)K, hipMemcpyDeviceToHost, c->stream));
            if (r->peak_configs)
                HIPCHK(hipMemcpyAsync(r->peak_configs, c->peak, (size_t)K * 4, hipMemcpyDeviceToHost, c->stream));
            if (r->final_configs)
                HIPCHK(hipMemcpyAsync(r->final_configs, c->final_cfg, (size_t)K * o.max_final * 16,
                                      hipMemcpyDeviceToHost, c->stream));
            if (r->n_final)
                HIPCHK(hipMemcpyAsync(r->n_final, c->n_final, (size_t)K * 4, hipMemcpyDeviceToHost, c->stream));
            if (r->analyzer)
                HIPCHK(hipMemcpyAsync(r->analyzer, c->analyzer, (size_t)K, hipMemcpyDeviceToHost, c->stream));
        }
        HIPCHK(hipStreamSynchronize(c->stream));
        return take_error(c);
    };
    if (t0_step) {
        if (mode != RES_HOST) {
            // only the error words come back
            HIPCHK(hipEventRecord(c->e1, c->stream));
            HIPCHK(hipMemcpyAsync(c->hctl + 6, c->counters + 4, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
            rc = take_error(c);
        } else {
            rc = readback();
        }
        std::memset(c->hctl, 0, CTL_BYTES);  // counters not kept on this path
        c->ticket_next = (split || spec) ? ticket_base : ticket_base + (uint32_t)K + (uint32_t)g0;
        c->ticket_live = true;
        if (rc) return rc;
    } else {
        rc = readback();
        if (rc) return rc;
    }
    bool t3 = false;
    const unsigned long long probes_pre_t3 = acc[0];
    const int32_t n_deep = cnt[2], n_widek = cnt[3];
    if (K > 0 && (n_deep > 0 || n_widek > 0)) {
        // T3 (HBM tier): keys beyond T2, then keys needing wide configs
        t3 = true;
        HIPCHK(hipEventRecord(c->et3a, c->stream));
        lcd::Args a3 = a;
        a3.wide = wide; a3.n_wide = n_wide;
        // Narrow keys: the layered form first (<= 8 states; LC_PATH_LAYERS_OFF
        // turns it off for A/B runs), the config-keyed narrow tier for the
        // keys it hands on (cnt[6]).
        // (the layered form steps ops as register-state masks: not a table model)
        const bool layers = !d->table && !(o.path_flags & LC_PATH_LAYERS_OFF);
        int32_t *narrow_list = spill2, *narrow_n = n_spill2;
        int32_t n_narrow = n_deep;
        if (n_deep > 0 && layers) {
            int slots = 0;
            rc = ensure_lay_ws(c, n_deep, &slots);
            if (rc) return rc;
            a3.order = spill2; a3.n_order = 0; a3.n_in = n_spill2; a3.ticket = c->counters + 11;
            a3.spill = old_narrow; a3.n_spill = c->counters + 6;
            HIPCHK(lcd::launch_t3_layers(a3, c->lws.w, slots, c->stream));
            HIPCHK(hipMemcpyAsync(c->hctl, c->ctl, CTL_BYTES, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
            narrow_list = old_narrow; narrow_n = c->counters + 6;
            n_narrow = cnt[6];
        }
        if (n_narrow > 0) {
            int slots = 0;
            rc = ensure_ws(c, 0, n_narrow, &slots);
            if (rc) return rc;
            a3.order = narrow_list; a3.n_order = 0; a3.n_in = narrow_n; a3.ticket = c->counters + 13;
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
    // knossos.competition: the keys :linear left :unknown at its budget are
    // answered by WGL's search (the analysis that could still finish)
    uint64_t wgl_keys = 0, wgl_steps = 0, wgl_spilled = 0;
    float msw = 0;
    if (competition && K > 0) {
        int32_t *const list = c->lists, *const count = c->counters + 20;  // (run_wgl zeroes [16..19])
        HIPCHK(hipMemsetAsync(count, 0, sizeof(int32_t), c->stream));
        HIPCHK(lcd::launch_collect_budget(a.cause, (int32_t)K, list, count, c->stream));
        int32_t *h = (int32_t *)(c->hctl + 4) + 20;
        HIPCHK(hipMemcpyAsync(c->hctl, c->ctl, CTL_BYTES, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipMemcpyAsync(h, count, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        const int32_t n_b = *h;
        const uint64_t ev0 = acc[1];
        if (n_b > 0) {
            lc_stats ws{};
            rc = run_wgl(c, d, a, list, 0, count, n_b, analyzer, &ws);
            if (rc) return rc;
            rc = readback();
            if (rc) return rc;
            HIPCHK(hipEventElapsedTime(&msw, c->et3a, c->et3b));
            HIPCHK(hipEventElapsedTime(&ms, c->e0, c->e1));
            wgl_keys = (uint64_t)n_b;
            wgl_steps = acc[1] - ev0;
            wgl_spilled = ws.wgl_spilled;
        }
    }
    if (st) {
        st->kernel_ms = ms;
        st->tier0_ms = ms0;
        st->tier3_ms = ms3;
        st->probes_t3 = t3 ? acc[0] - probes_pre_t3 : 0;
        st->t3_bytes = t3 ? acc[3] : 0;
        st->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        st->probes = acc[0];
        st->events = acc[1];
        st->lds_keys = acc[2];
        st->deep_keys = (uint64_t)(n_deep + n_widek);  // keys the HBM tier (re)searched
        st->t0_path = t0_path;
        st->ev_word_bytes = t0_path ? (ev16 ? 2u : 4u) : 0u;
        st->wgl_ms = msw;
        st->wgl_keys = wgl_keys;
        st->wgl_steps = wgl_steps;
        st->wgl_spilled = wgl_spilled;
    }
    return LC_OK;
}

// Wait for everything enqueued on c; *n_async / *span_ms: the asynchronous
// steps since the last wait and their HIP-event span.
static int dev_wait(Dev *c, int *n_async, float *span_ms) {
    lc::Range range("lincheck: wait");
    HIPCHK(hipSetDevice(c->device));
    if (c->ea1_pending) HIPCHK(hipEventRecord(c->ea1, c->stream));
    c->ea1_pending = false;
    HIPCHK(hipMemcpyAsync(c->hctl + 6, c->counters + 4, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    // every step's ring slot read and cleared behind them: one
    // synchronisation for the wait and both error reads
    const int re = take_ring_enqueue(c, 0xFu, c->stream);
    if (re) return re;
    HIPCHK(hipStreamSynchronize(c->stream));
    *n_async = (int)c->n_async;
    *span_ms = 0;
    if (c->n_async) HIPCHK(hipEventElapsedTime(span_ms, c->ea0, c->ea1));
    c->n_async = 0;
    const int rr = ring_taken(c, -1);
    const int rs = take_error(c);
    return rs ? rs : rr;
}

static void merge_stats(lc_stats &t, const lc_stats &s) {
    t.kernel_ms = std::max(t.kernel_ms, s.kernel_ms);
    t.tier0_ms = std::max(t.tier0_ms, s.tier0_ms);
    t.tier3_ms = std::max(t.tier3_ms, s.tier3_ms);
    t.probes += s.probes;
    t.probes_t3 += s.probes_t3;
    t.t3_bytes += s.t3_bytes;
    t.lds_keys += s.lds_keys;
    t.deep_keys += s.deep_keys;
    t.events += s.events;
    t.t0_path = std::max(t.t0_path, s.t0_path);
    t.ev_word_bytes = std::max(t.ev_word_bytes, s.ev_word_bytes);
    t.wgl_ms = std::max(t.wgl_ms, s.wgl_ms);
    t.wgl_keys += s.wgl_keys;
    t.wgl_spilled += s.wgl_spilled;
    t.wgl_steps += s.wgl_steps;
}

// Run fn(g) for every device g of c at once (one driver thread per device
// beyond the first); returns the first nonzero code.
static int each_device(lc_ctx *c, const std::function<int(int)> &fn) {
    if (c->n_dev == 1) return fn(0);
    std::vector<int> rc((size_t)c->n_dev, 0);
    std::vector<std::string> err((size_t)c->n_dev);
    c->drivers->run((unsigned)c->n_dev, [&](unsigned g) {
        rc[g] = fn((int)g);
        if (rc[g]) err[g] = lc_last_error();
    });
    for (int g = 0; g < c->n_dev; ++g)
        if (rc[g]) return lc::fail(rc[g], "%s", err[g].c_str());
    return LC_OK;
}

// Validate b (events too unless T0 will) and, when its event words are not
// page-locked, copy them into the context's pinned staging buffer.  *src:
// where the uploads read the events from (b->events or the staging copy).
static int prepare_batch(lc_ctx *c, const lc_batch *b, Shape *sh, const uint32_t **src) {
    lc::Range range("lincheck: prepare");
    int rc = validate_batch(b);
    if (rc) return rc;
    *sh = batch_shape(b);
    *src = b->events;
    const int64_t K = b->n_keys;
    if (!K) return LC_OK;
    const size_t n_ev = (size_t)b->ev_off[K];
    // Batches above 256 MB of events keep the pageable path (no pinned
    // allocation that large); page-locked caller memory is used as it is.
    // A batch given only as 16-bit words is widened here when its upload
    // needs the 32-bit ones (keys beyond the register tier, or the A/B flag
    // LC_PATH_EV32); a register-tier batch uploads the 16-bit words.
    const bool up16 = b->events16 && sh->t0_only && !(c->o.path_flags & LC_PATH_EV32);
    const bool widen = n_ev > 0 && !b->events && !up16;
    const bool stage = widen || (n_ev > 0 && b->events && n_ev <= (256u << 20) / 4 && !pinned(b->events) &&
                                 !(up16 && pinned(b->events16)));
    if (stage && n_ev > c->hstage_cap) {
        if (c->hstage) (void)hipHostFree(c->hstage);
        c->hstage = nullptr;
        c->hstage_cap = 0;
        HIPCHK(hipHostMalloc((void **)&c->hstage, n_ev * 4, hipHostMallocDefault));
        c->hstage_cap = n_ev;
    }
    // The device validates every event of a batch (k_validate beside the
    // first tier; the later tiers do nothing over a refused batch), so the
    // host walks the events only to stage pageable ones -- and to check a
    // table model, whose rows are checked against the key's states here.
    sh->host_checked = b->table != nullptr;
    if (!stage && !sh->host_checked) return LC_OK;  // nothing to copy, the device validates
    if (K >= 256 && !c->pool)
        c->pool = new HostPool(std::max(1u, std::min(16u, std::thread::hardware_concurrency())) - 1);
    int64_t bk = -1;
    if (int why = validate_events(b, &bk, stage ? c->hstage : nullptr, K >= 256 ? c->pool : nullptr, sh->host_checked))
        return events_error(why, bk);
    if (stage) *src = c->hstage;
    return LC_OK;
}

// ---- C ABI ------------------------------------------------------------------

extern "C" int lc_upload(lc_ctx *c, const lc_batch *b, lc_dev_batch **out) {
    if (!c || !b || !out) return lc::fail(LC_E_INVALID, "lc_upload: null argument");
    std::lock_guard<std::mutex> g(c->mu);
    Shape sh;
    const uint32_t *src = nullptr;
    int rc = prepare_batch(c, b, &sh, &src);
    if (rc) return rc;
    lc_dev_batch *d = new (std::nothrow) lc_dev_batch();
    if (!d) return lc::fail(LC_E_NOMEM, "lc_upload: out of memory");
    d->n_parts = c->n_dev;
    d->n_keys = b->n_keys;
    shard_keys(b, c->n_dev, d->key0);
    for (int p = 0; p < c->n_dev; ++p) {
        d->part[p] = new (std::nothrow) DevBatch();
        if (!d->part[p]) { delete d; return lc::fail(LC_E_NOMEM, "lc_upload: out of memory"); }
        d->part[p]->device = c->dev[p]->device;
    }
    rc = each_device(c, [&](int p) {
        std::vector<uint64_t> off;
        const lc_batch s = c->n_dev > 1 ? sub_batch(b, d->key0[p], d->key0[p + 1], off) : *b;
        const uint32_t *es = src ? src + (b->n_keys ? b->ev_off[d->key0[p]] : 0) : nullptr;
        return upload_into(c->dev[p], &s, d->part[p], sh, sh.host_checked, es);
    });
    if (rc) { delete d; return rc; }
    *out = d;
    return LC_OK;
}

extern "C" void lc_dev_batch_free(lc_dev_batch *d) { delete d; }

extern "C" int lc_check_device(lc_ctx *c, const lc_dev_batch *d, lc_result *r, int flags, lc_stats *st) {
    if (flags & ~(LC_DEV_RESULT | LC_DEV_ASYNC)) return lc::fail(LC_E_INVALID, "lc_check_device: unknown flags 0x%x", flags);
    const bool dev_result = (flags & LC_DEV_RESULT) != 0;
    if (!c || !d || !r || !r->valid || !r->fail_event || !r->cause)
        return lc::fail(LC_E_INVALID, "lc_check_device: null argument");
    if (d->n_parts != c->n_dev) return lc::fail(LC_E_INVALID, "lc_check_device: batch uploaded by another context shape");
    for (int p = 0; p < d->n_parts; ++p)
        if (d->part[p]->device != c->dev[p]->device)
            return lc::fail(LC_E_INVALID, "lc_check_device: batch lives on another device");
    if (dev_result && c->n_dev > 1)
        return lc::fail(LC_E_INVALID, "lc_check_device: LC_DEV_RESULT needs a one-device context");
    std::lock_guard<std::mutex> g(c->mu);
    if (c->n_dev == 1)
        return dev_search(c->dev[0], d->part[0], r, dev_result ? RES_DEV : RES_HOST, (flags & LC_DEV_ASYNC) != 0, 0, st);
    auto t0 = std::chrono::steady_clock::now();
    std::vector<lc_stats> ps((size_t)c->n_dev);
    const int mf = c->o.max_final;
    int rc = each_device(c, [&](int p) {
        const int64_t k0 = d->key0[p];
        lc_result rp = *r;
        rp.valid = r->valid + k0;
        rp.fail_event = r->fail_event + k0;
        rp.cause = r->cause + k0;
        if (r->peak_configs) rp.peak_configs = r->peak_configs + k0;
        if (r->final_configs) rp.final_configs = r->final_configs + (size_t)k0 * mf * 2;
        if (r->n_final) rp.n_final = r->n_final + k0;
        return dev_search(c->dev[p], d->part[p], &rp, RES_HOST, false, k0, &ps[(size_t)p]);
    });
    if (rc) return rc;
    if (st) {
        *st = lc_stats{};
        for (const lc_stats &s : ps) merge_stats(*st, s);
        st->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return LC_OK;
}

extern "C" int lc_wait(lc_ctx *c, lc_stats *st) {
    if (!c) return lc::fail(LC_E_INVALID, "lc_wait: null context");
    lc::Range range("lc_wait");
    std::lock_guard<std::mutex> g(c->mu);
    int n = 0;
    float ms = 0;
    int rc = LC_OK;
    for (int p = 0; p < c->n_dev; ++p) {
        int np = 0;
        float mp = 0;
        int r = dev_wait(c->dev[p], &np, &mp);
        if (r && !rc) rc = r;
        n = std::max(n, np);
        ms = std::max(ms, mp);
    }
    if (rc) return rc;
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
    int rc = LC_OK;
    for (int p = 0; p < c->n_dev; ++p) {
        Dev *d = c->dev[p];
        HIPCHK(hipSetDevice(d->device));
        int r;
        if (back < 0 || back >= 4 || (uint64_t)back >= d->async_seq) {
            HIPCHK(hipStreamSynchronize(d->stream));  // no such step on record: everything
            r = take_ring(d, 0xFu, -1, d->stream);
        } else {
            // Errors of the finished step surface here (include/lincheck.h):
            // its own error words, read and cleared atomically on a stream of
            // their own, so the later steps still running keep theirs (one 4
            // steps later shares the slot: an error it has raised already is
            // reported now too)
            const int q = (int)((d->async_seq - 1 - (uint64_t)back) % 4);
            HIPCHK(hipEventSynchronize(d->ring[q]));
            r = take_ring(d, 1u << q, q, d->estream);
        }
        if (r && !rc) rc = r;
    }
    return rc;
}

extern "C" int lc_check_batch(lc_ctx *c, const lc_batch *b, lc_result *r, lc_stats *st) {
    lc::Range range("lc_check_batch");
    auto t0 = std::chrono::steady_clock::now();
    if (!c || !b || !r || !r->valid || !r->fail_event || !r->cause)
        return lc::fail(LC_E_INVALID, "lc_check_batch: null argument");
    std::lock_guard<std::mutex> g(c->mu);
    Shape sh;
    const uint32_t *src = nullptr;
    int rc = prepare_batch(c, b, &sh, &src);
    if (rc) return rc;
    const auto t_val = std::chrono::steady_clock::now();
    int64_t key0[MAX_DEV + 1];
    shard_keys(b, c->n_dev, key0);
    std::vector<lc_stats> ps((size_t)c->n_dev);
    const int mf = c->o.max_final;
    rc = each_device(c, [&](int p) {
        Dev *d = c->dev[p];
        if (!d->staged) {
            d->staged = new (std::nothrow) DevBatch();
            if (!d->staged) return lc::fail(LC_E_NOMEM, "lc_check_batch: out of memory");
        }
        std::vector<uint64_t> off;
        const lc_batch s = c->n_dev > 1 ? sub_batch(b, key0[p], key0[p + 1], off) : *b;
        const uint32_t *es = src ? src + (b->n_keys ? b->ev_off[key0[p]] : 0) : nullptr;
        int e = upload_into(d, &s, d->staged, sh, sh.host_checked, es);
        if (e) return e;
        const int64_t k0 = key0[p];
        lc_result rp = *r;
        rp.valid = r->valid + k0;
        rp.fail_event = r->fail_event + k0;
        rp.cause = r->cause + k0;
        if (r->peak_configs) rp.peak_configs = r->peak_configs + k0;
        if (r->final_configs) rp.final_configs = r->final_configs + (size_t)k0 * mf * 2;
        if (r->n_final) rp.n_final = r->n_final + k0;
        if (r->analyzer) rp.analyzer = r->analyzer + k0;
        return dev_search(d, d->staged, &rp, RES_HOST, false, k0, &ps[(size_t)p]);
    });
    if (std::getenv("LC_TIMING")) {
        using ms = std::chrono::duration<double, std::milli>;
        std::fprintf(stderr, "lc_check_batch: validate/stage %.3f ms, upload + check %.3f ms\n",
                     ms(t_val - t0).count(), ms(std::chrono::steady_clock::now() - t_val).count());
    }
    if (rc) return rc;
    if (st) {
        *st = lc_stats{};
        for (const lc_stats &s : ps) merge_stats(*st, s);
        st->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return LC_OK;
}

// ---- one process per GPU: node-wide verdict records ---------------------------

// Pack this rank's verdicts (c's device arrays) into its block and all-gather
// the blocks of every rank over RCCL (one rank: the block is the node), on
// c's stream.
// The rank's record block (and the node's), grown on demand; the search that
// follows writes its records straight into the block (Dev::rec_out), and the
// padding past the shard's n keys is zeroed.
static int node_buffers(lc_ctx *x, Dev *c, int64_t n, int64_t block) {
    if (block > c->node_cap || !c->send) {
        if (c->n_async) HIPCHK(hipStreamSynchronize(c->stream));  // an enqueued step may still write them
        dfree(c->send);
        dfree(c->node);
        HIPCHK(dalloc(&c->send, (size_t)std::max<int64_t>(block, 1)));
        HIPCHK(dalloc(&c->node, (size_t)std::max<int64_t>(block, 1) * x->size));
        c->node_cap = block;
    }
    uint64_t *blk = x->comm ? c->send : c->node;
    if (block > n) HIPCHK(hipMemsetAsync(blk + n, 0, (size_t)(block - n) * 8, c->stream));
    c->rec_out = blk;
    return LC_OK;
}

static int gather_node(lc_ctx *x, Dev *c, int64_t n, int64_t block, bool packed = false) {
    lc::Range range("lincheck: gather");
    const int64_t total = block * x->size;
    c->rec_out = nullptr;
    if (block > 0 && !packed) {
        const int threads = 256;
        const int blocks = (int)std::min<int64_t>((block + threads - 1) / threads, 4096);
        hipLaunchKernelGGL(k_pack_records, dim3(blocks), dim3(threads), 0, c->stream, c->valid, c->cause, c->fail_event,
                           n, block, x->comm ? c->send : c->node);
        HIPCHK(hipGetLastError());
    }
    if (x->comm) {
        const Rccl *R = rccl();
        RCCLCHK(R->all_gather(c->send, c->node, (size_t)block, ncclUint64, x->comm, c->stream));
    }
    c->node_n = total;
    return LC_OK;
}

static int node_check_args(lc_ctx *c, int64_t n_keys, int64_t block) {
    if (c->n_dev != 1) return lc::fail(LC_E_INVALID, "lc_check_node: needs a one-device context");
    if (block < n_keys) return lc::fail(LC_E_INVALID, "lc_check_node: block %lld < the shard's %lld keys",
                                        (long long)block, (long long)n_keys);
    return LC_OK;
}

extern "C" int lc_check_node(lc_ctx *c, const lc_batch *b, int64_t block, uint64_t *node, lc_stats *st) {
    lc::Range range("lc_check_node");
    auto t0 = std::chrono::steady_clock::now();
    if (!c || !b || !node) return lc::fail(LC_E_INVALID, "lc_check_node: null argument");
    std::lock_guard<std::mutex> g(c->mu);
    int rc = node_check_args(c, b->n_keys, block);
    if (rc) return rc;
    Shape sh;
    const uint32_t *src = nullptr;
    rc = prepare_batch(c, b, &sh, &src);
    if (rc) return rc;
    Dev *d = c->dev[0];
    if (!d->staged) {
        d->staged = new (std::nothrow) DevBatch();
        if (!d->staged) return lc::fail(LC_E_NOMEM, "lc_check_node: out of memory");
    }
    rc = node_buffers(c, d, b->n_keys, block);
    if (rc) return rc;
    struct RecOff {  // every return below stops later searches writing records
        Dev *d;
        ~RecOff() { d->rec_out = nullptr; }
    } rec_off{d};
    const auto t_prep = std::chrono::steady_clock::now();
    // A large register-tier shard (throughput-bound: many keys per SIMD) is
    // uploaded and searched in NODE_CHUNKS key chunks: the copies run on a
    // stream of their own, and each chunk's search waits only for its own
    // copy, so the host-to-device transfer overlaps the search
    // (lc_opts.path_flags LC_PATH_CHUNKS_ON / _OFF pin the choice).
    const int64_t K = b->n_keys;
    const uint64_t n_ev = K ? b->ev_off[K] : 0;
    const bool can_chunk = sh.t0_only && !(c->o.flags & LC_OPT_COUNT_PROBES) && K >= Dev::NODE_CHUNKS;
    bool big = K >= 16 * (int64_t)d->cu_count && n_ev >= (8u << 20);
    if (c->o.path_flags & LC_PATH_CHUNKS_ON) big = true;
    if (c->o.path_flags & LC_PATH_CHUNKS_OFF) big = false;
    // (Searching page-locked event words in place, over the host link, was
    // measured slower: 0.468 against 0.332 ms for C2's search, the link
    // sustaining ~31 GB/s of kernel reads; the 16-bit upload won instead.)
    const int chunks = can_chunk && big ? Dev::NODE_CHUNKS : 1;
    lc_result none{};
    bool enq = false;
    // on an error below, the copies out of the caller's arrays are waited for
    auto drained = [&](int e) {
        (void)hipStreamSynchronize(d->cstream);
        (void)hipStreamSynchronize(d->stream);
        return e;
    };
    std::chrono::steady_clock::time_point t_up;
    if (chunks > 1) {
        rc = ensure_capacity(d, K);
        if (rc) return rc;
        int64_t key0[Dev::NODE_CHUNKS + 1];
        shard_keys(b, chunks, key0);
        for (int i = 0; i < chunks; ++i) {
            if (!d->chunk[i]) {
                d->chunk[i] = new (std::nothrow) DevBatch();
                if (!d->chunk[i]) return drained(lc::fail(LC_E_NOMEM, "lc_check_node: out of memory"));
            }
            if (!d->chunk_ready[i]) HIPCHK(hipEventCreateWithFlags(&d->chunk_ready[i], hipEventDisableTiming));
            std::vector<uint64_t> off;
            const lc_batch s = sub_batch(b, key0[i], key0[i + 1], off);
            const uint32_t *es = src ? src + b->ev_off[key0[i]] : nullptr;
            rc = upload_into(d, &s, d->chunk[i], sh, sh.host_checked, es, false, d->cstream);
            if (rc) return drained(rc);
            HIPCHK(hipEventRecord(d->chunk_ready[i], d->cstream));
        }
        t_up = std::chrono::steady_clock::now();
        for (int i = 0; i < chunks && rc == 0; ++i) {
            HIPCHK(hipStreamWaitEvent(d->stream, d->chunk_ready[i], 0));
            bool e = false;
            rc = dev_search(d, d->chunk[i], &none, RES_CTX, true, key0[i], st, &e, key0[i]);
            enq = i == 0 ? e : (enq && e);
        }
        if (rc) return drained(rc);
        if (!enq) return drained(lc::fail(LC_E_DEVICE, "lc_check_node: a chunk left the register tier"));
    } else {
        rc = upload_into(d, b, d->staged, sh, sh.host_checked, src, false);
        if (rc) return rc;
        t_up = std::chrono::steady_clock::now();
        rc = dev_search(d, d->staged, &none, RES_CTX, true, 0, st, &enq);
        if (rc) return drained(rc);
    }
    const auto t_search = std::chrono::steady_clock::now();
    rc = gather_node(c, d, b->n_keys, block, true);  // the search wrote the records
    if (rc) return drained(rc);
    // the records land in pinned memory (a copy into the caller's pageable
    // array would be a synchronous staged copy) and are copied out after the wait
    if (d->node_n > d->hnode_cap) {
        if (d->hnode) (void)hipHostFree(d->hnode);
        d->hnode = nullptr;
        d->hnode_cap = 0;
        if (hipHostMalloc((void **)&d->hnode, (size_t)d->node_n * 8, hipHostMallocDefault) != hipSuccess)
            return drained(lc::fail(LC_E_NOMEM, "lc_check_node: pinned record buffer"));
        d->hnode_cap = d->node_n;
    }
    if (d->node_n && hipMemcpyAsync(d->hnode, d->node, (size_t)d->node_n * 8, hipMemcpyDeviceToHost, d->stream) !=
                         hipSuccess)
        return drained(lc::fail(LC_E_DEVICE, "lc_check_node: record download failed"));
    const auto t_gather = std::chrono::steady_clock::now();
    if (enq) {  // a T0-only step (or chunks): one wait for the search, the exchange and the download
        int n_async = 0;
        float span = 0;
        rc = dev_wait(d, &n_async, &span);
        if (rc) return drained(rc);
        if (st) st->kernel_ms = st->tier0_ms = span;
    } else {
        HIPCHK(hipStreamSynchronize(d->stream));
    }
    if (d->node_n) std::memcpy(node, d->hnode, (size_t)d->node_n * 8);
    if (std::getenv("LC_TIMING")) {
        using ms = std::chrono::duration<double, std::milli>;
        std::fprintf(stderr, "lc_check_node: prepare %.3f, upload %.3f, search enqueue %.3f, gather enqueue %.3f, "
                     "wait %.3f ms (search span %.3f)\n", ms(t_prep - t0).count(), ms(t_up - t_prep).count(),
                     ms(t_search - t_up).count(), ms(t_gather - t_search).count(),
                     ms(std::chrono::steady_clock::now() - t_gather).count(), st ? st->kernel_ms : 0.f);
    }
    if (st) st->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return LC_OK;
}

// The pipelined form of lc_check_node.  A register-tier step (every key fits
// the register lattice, no probe counting, one upload, records to page-locked
// memory) is only enqueued: its upload goes into the staging slot the step
// two back used (once that step is done) on the copy stream, its search waits
// for that upload on the search stream, and the records are downloaded into
// `node` behind the search.  So step i + 1's host-to-device copy overlaps step
// i's search, and the host enqueues ahead instead of waiting between steps.
// Anything else runs as lc_check_node.
extern "C" int lc_check_node_async(lc_ctx *c, const lc_batch *b, int64_t block, uint64_t *node, lc_stats *st) {
    lc::Range range("lc_check_node_async");
    if (!c || !b || !node) return lc::fail(LC_E_INVALID, "lc_check_node_async: null argument");
    Dev *d = nullptr;
    Shape sh;
    const uint32_t *src = nullptr;
    {
        std::lock_guard<std::mutex> g(c->mu);
        int rc = node_check_args(c, b->n_keys, block);
        if (rc) return rc;
        d = c->dev[0];
        HIPCHK(hipSetDevice(d->device));
        const int64_t K = b->n_keys;
        const uint64_t n_ev = K ? b->ev_off[K] : 0;
        // (a large shard is not cut into chunks here: its whole upload
        // overlaps the previous step's search instead)
        if (K > 0 && n_ev > 0 && !b->table && !(c->o.flags & LC_OPT_COUNT_PROBES) && pinned(node) &&
            !(c->o.path_flags & LC_PATH_NODE_SYNC)) {
            rc = prepare_batch(c, b, &sh, &src);
            if (rc) return rc;
            if (sh.t0_only) {
                const int s = (int)(d->pipe_next % Dev::PIPE);
                if (!d->pipe[s]) {
                    d->pipe[s] = new (std::nothrow) DevBatch();
                    if (!d->pipe[s]) return lc::fail(LC_E_NOMEM, "lc_check_node_async: out of memory");
                    // (a device-scope release: the host only learns from it
                    // that the upload's device writes are done)
                    if (hipEventCreateWithFlags(&d->pipe_ready[s], hipEventDisableTiming | hipEventReleaseToDevice) !=
                        hipSuccess) {
                        (void)hipGetLastError();
                        HIPCHK(hipEventCreateWithFlags(&d->pipe_ready[s], hipEventDisableTiming));
                    }
                }
                // the step that last read this slot has finished (at most one
                // other step stays in flight), so its buffers may be rewritten
                // or regrown.  Its end is the ring event its search recorded:
                // a marker of its own after every step cost the stream ~5 us
                // between consecutive searches (a system-scope fence each).
                // (A ring slot re-recorded since by a later step only makes
                // this wait for that later step.)
                if (d->pipe_busy[s]) HIPCHK(hipEventSynchronize(d->ring[d->pipe_seq[s] % 4]));
                // One rank: the search writes the records straight into the
                // caller's page-locked buffer (device-mapped), so no download
                // follows it; with a communicator they go through HBM for the
                // all-gather.
                uint64_t *dnode = nullptr;
                const bool direct = !c->comm && !(c->o.path_flags & LC_PATH_NODE_STAGED) &&
                                    hipHostGetDevicePointer((void **)&dnode, node, 0) == hipSuccess && dnode;
                if (direct) {
                    if (block > K) std::memset(node + K, 0, (size_t)(block - K) * 8);
                    d->rec_out = dnode;
                } else {
                    rc = node_buffers(c, d, K, block);
                    if (rc) return rc;
                }
                struct RecOff {
                    Dev *d;
                    ~RecOff() { d->rec_out = nullptr; }
                } rec_off{d};
                auto drained = [&](int e) {
                    (void)hipStreamSynchronize(d->cstream);
                    (void)hipStreamSynchronize(d->stream);
                    return e;
                };
                rc = upload_into(d, b, d->pipe[s], sh, sh.host_checked, src, false, d->cstream);
                if (rc) return drained(rc);
                HIPCHK(hipEventRecord(d->pipe_ready[s], d->cstream));
                // The host waits for the upload (the previous step's search
                // is running meanwhile) and then enqueues the search: no
                // cross-stream wait on the device, whose latency sat between
                // consecutive searches (C2 0.3415 -> 0.3365 ms per step).  It
                // also frees the context's staging copy of pageable events.
                HIPCHK(hipEventSynchronize(d->pipe_ready[s]));
                lc_result none{};
                bool enq = false;
                rc = dev_search(d, d->pipe[s], &none, RES_CTX, true, 0, st, &enq);
                if (rc) return drained(rc);
                if (direct) {
                    d->node_n = 0;  // the records are in `node` only (lc_node_records has none)
                } else {
                    rc = gather_node(c, d, K, block, true);
                    if (rc) return drained(rc);
                    if (d->node_n && hipMemcpyAsync(node, d->node, (size_t)d->node_n * 8, hipMemcpyDeviceToHost,
                                                    d->stream) != hipSuccess)
                        return drained(lc::fail(LC_E_DEVICE, "lc_check_node_async: record download failed"));
                }
                d->pipe_busy[s] = enq;
                d->pipe_seq[s] = d->async_seq - 1;
                ++d->pipe_next;
                if (enq) return 1;
                HIPCHK(hipStreamSynchronize(d->stream));  // not reached for a register-tier batch
                return LC_OK;
            }
        }
    }
    return lc_check_node(c, b, block, node, st);
}

extern "C" void *lc_host_alloc(size_t bytes) {
    void *p = nullptr;
    if (hipHostMalloc(&p, std::max<size_t>(bytes, 1), hipHostMallocDefault) != hipSuccess) {
        lc::set_error("lc_host_alloc: page-locked allocation failed");
        return nullptr;
    }
    return p;
}

extern "C" void lc_host_free(void *p) {
    if (p) (void)hipHostFree(p);
}

extern "C" int lc_check_node_device(lc_ctx *c, const lc_dev_batch *db, int64_t block, int flags, lc_stats *st) {
    if (!c || !db) return lc::fail(LC_E_INVALID, "lc_check_node_device: null argument");
    if (flags & ~LC_DEV_ASYNC) return lc::fail(LC_E_INVALID, "lc_check_node_device: unknown flags 0x%x", flags);
    std::lock_guard<std::mutex> g(c->mu);
    int rc = node_check_args(c, db->n_keys, block);
    if (rc) return rc;
    if (db->n_parts != 1 || db->part[0]->device != c->dev[0]->device)
        return lc::fail(LC_E_INVALID, "lc_check_node_device: batch lives on another device");
    Dev *d = c->dev[0];
    lc_result none{};
    bool enq = false;
    rc = node_buffers(c, d, db->n_keys, block);
    if (rc) return rc;
    rc = dev_search(d, db->part[0], &none, RES_CTX, (flags & LC_DEV_ASYNC) != 0, 0, st, &enq);
    if (rc) { d->rec_out = nullptr; return rc; }
    rc = gather_node(c, d, db->n_keys, block, true);
    if (rc) return rc;
    if (!enq) HIPCHK(hipStreamSynchronize(d->stream));
    return LC_OK;
}

extern "C" int lc_node_records(lc_ctx *c, uint64_t *node, int64_t n) {
    if (!c || (!node && n)) return lc::fail(LC_E_INVALID, "lc_node_records: null argument");
    std::lock_guard<std::mutex> g(c->mu);
    Dev *d = c->dev[0];
    if (n > d->node_n) return lc::fail(LC_E_INVALID, "lc_node_records: %lld records asked, %lld gathered",
                                       (long long)n, (long long)d->node_n);
    HIPCHK(hipSetDevice(d->device));
    if (n) HIPCHK(hipMemcpyAsync(node, d->node, (size_t)n * 8, hipMemcpyDeviceToHost, d->stream));
    HIPCHK(hipStreamSynchronize(d->stream));
    return LC_OK;
}
