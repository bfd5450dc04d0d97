"""Mirror of jepsen.checker for this path (etcdemo.clj:7, :116-119, :165-167).

    linearizable({"model": model.cas_register(), "algorithm": "linear"})
        jepsen.checker/linearizable -> knossos.linear/analysis, here the
        device search in liblincheck.so.  Result maps follow Knossos's shape:
        {"valid?": True/False/"unknown", "op": ..., "previous-ok": ...,
         "last-op": ..., "configs": [...], "final-paths": [...],
         "analyzer": "linear"} with :configs / :final-paths truncated to 10.
    compose({name: checker}) / merge_valid / check_safe
        jepsen.checker/compose, merge-valid, check-safe.

Under independent.checker the linearizable check is batched: every key goes
to the device in one call (Batch below).  Device failures raise; check_safe
turns an exception into {"valid?": "unknown", "error": ...} exactly where
Jepsen's check-safe would.
"""

from __future__ import annotations

import ctypes as C
import gc
import os
import threading
import time
import traceback
import warnings
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from . import _native as N
from .history import NAMED_REG_BASE, History
from .model import MODELS, CASRegister, MultiRegister, fmt

DEFAULT_BUDGET = 1 << 20
TRUNCATE = 10  # jepsen.checker/linearizable truncates :final-paths and :configs


# ---------------------------------------------------------------- packing
class Packed:
    """lc_pack output: per-key event streams plus the row maps back to ops."""

    def __init__(self, hist: History, model=None):
        self.hist = hist
        self.model = model if model is not None else CASRegister()
        self._c = hist.as_c()
        handle = C.c_void_p()
        opts = N.LcPackOpts(self.model.code)
        self.reg_names = dict(hist.reg_names)  # register id -> name (multi-register)
        if isinstance(self.model, MultiRegister):
            ids = {name: rid for rid, name in self.reg_names.items()}

            def reg_id(r):
                if isinstance(r, (int, np.integer)) and not isinstance(r, bool):
                    return int(r)
                if r not in ids:
                    ids[r] = NAMED_REG_BASE + len(ids)
                return ids[r]
            pairs = self.model.init_pairs(reg_id)
            self.reg_names = {rid: name for name, rid in ids.items()}
            self._init = np.array([x for k, v in pairs for x in (k, N.LC_NIL if v is None else v)] or [0], np.int64)
            opts.n_init, opts.init = len(pairs), N.ptr(self._init, C.c_int64)
        N.check(N.lib().lc_pack(C.byref(self._c), C.byref(opts), C.byref(handle)))
        self.handle = handle
        v = N.LcBatch()
        N.check(N.lib().lc_packed_view(self.handle, C.byref(v)))
        self.view = v
        self.n_keys = int(v.n_keys)
        self.ev_off = N.carray(v.ev_off, self.n_keys + 1, np.uint64)
        keys = np.zeros(max(self.n_keys, 1), np.int64)
        N.check(N.lib().lc_packed_keys(self.handle, N.ptr(keys, C.c_int64)))
        self.keys = [int(k) for k in keys[:self.n_keys]]

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            N.lib().lc_packed_free(h)
            self.handle = None

    def n_events(self, i: int) -> int:
        return int(self.ev_off[i + 1] - self.ev_off[i])

    def all_events(self) -> np.ndarray:
        """Every event word (u32), widened from the 16-bit form when lc_pack
        gave only that (lc_batch.events NULL, ABI 11)."""
        n = int(self.ev_off[-1]) if self.n_keys else 0
        if n == 0:
            return np.zeros(0, np.uint32)
        if self.view.events:
            return np.ctypeslib.as_array(self.view.events, shape=(n,)).copy()
        e = np.ctypeslib.as_array(self.view.events16, shape=(n,)).astype(np.uint32)
        return ((e & 0x8000) << 16) | (((e >> 11) & 0xF) << 24) | (e & 0x7FF)

    def events(self, i: int) -> np.ndarray:
        b, e = int(self.ev_off[i]), int(self.ev_off[i + 1])
        if e == b:
            return np.zeros(0, np.uint32)
        if self.view.events:
            return np.ctypeslib.as_array(self.view.events, shape=(int(self.ev_off[-1]) or 1,))[b:e].copy()
        e16 = np.ctypeslib.as_array(self.view.events16, shape=(int(self.ev_off[-1]) or 1,))[b:e].astype(np.uint32)
        return ((e16 & 0x8000) << 16) | (((e16 >> 11) & 0xF) << 24) | (e16 & 0x7FF)

    def event_row(self, i: int, j: int) -> int:
        return int(N.check(N.lib().lc_packed_event_row(self.handle, i, j)))

    def desc(self, i: int, t: int) -> int:
        """Transition descriptor t of key i (LC_EV_TRANS + trans_off[i])."""
        if not hasattr(self, "_trans"):
            self._trans = N.carray(self.view.trans, max(int(self.view.n_trans), 1), np.uint32)
            self._trans_off = N.carray(self.view.trans_off, self.n_keys, np.uint32)
        base = int(self._trans_off[i]) if len(self._trans_off) else 0
        return int(self._trans[base + t])

    def key_error(self, i: int) -> Optional[str]:
        """Why key i could not be prepared (lc_packed_key_error), or None."""
        msg = N.lib().lc_packed_key_error(self.handle, i)
        return None if msg is None else msg.decode(errors="replace")

    def state_value(self, i: int, s: int):
        v = C.c_int64(); nil = C.c_int()
        N.check(N.lib().lc_packed_state_value(self.handle, i, s, C.byref(v), C.byref(nil)))
        return None if nil.value else int(v.value)

    def state_map(self, i: int, s: int) -> list:
        """multi-register: the (register, value) pairs state id s of key i
        stands for (lc_packed_state_map), registers by name where named."""
        n = N.check(N.lib().lc_packed_state_map(self.handle, i, s, None, None, 0))
        regs, vals = np.zeros(max(n, 1), np.int64), np.zeros(max(n, 1), np.int64)
        N.check(N.lib().lc_packed_state_map(self.handle, i, s, N.ptr(regs, C.c_int64), N.ptr(vals, C.c_int64), n))
        return [(self.reg_names.get(int(r), int(r)), None if v == N.LC_NIL else int(v)) for r, v in zip(regs[:n], vals[:n])]


# ---------------------------------------------------------------- device
@dataclass
class KeyResults:
    valid: np.ndarray        # int8: 1 / 0 / -1
    fail_event: np.ndarray   # int32
    cause: np.ndarray        # uint8
    peak: np.ndarray         # uint32
    final: np.ndarray        # uint64 [K, max_final, 2]
    n_final: np.ndarray      # uint32
    stats: Dict[str, float]
    analyzer: Optional[np.ndarray] = None  # uint8 LC_ALGO_LINEAR / LC_ALGO_WGL per key


def comm_id() -> bytes:
    """lc_comm_id: a fresh RCCL unique id (rank 0 hands it to every rank)."""
    buf = (C.c_uint8 * N.LC_COMM_ID_BYTES)()
    N.check(N.lib().lc_comm_id(buf))
    return bytes(buf)


class PinnedRecords(np.ndarray):
    """A uint64 array in page-locked memory (lc_host_alloc), freed with it."""

    def __new__(cls, n: int):
        n = max(int(n), 1)
        p = N.lib().lc_host_alloc(n * 8)
        if not p:
            raise N.LincheckError(-2, N.lib().lc_last_error().decode(errors="replace"))
        buf = (C.c_uint64 * n).from_address(p)
        obj = np.frombuffer(buf, np.uint64).view(cls)
        obj[:] = 0
        obj._owner = _HostBlock(p)
        return obj

    def __array_finalize__(self, obj):
        if obj is not None:
            self._owner = getattr(obj, "_owner", None)


class _HostBlock:
    def __init__(self, p):
        self.p = p

    def __del__(self):
        if self.p:
            N.lib().lc_host_free(self.p)
            self.p = None


class Device:
    """An lc_ctx (lc_create) on one GPU, on several (devices=[...]: one
    contiguous key shard per entry, checked at once), or as one rank of a
    multi-process node (comm=(rank, size, comm_id bytes): lc_check_node
    all-gathers the verdict records over RCCL)."""

    def __init__(self, device: int = 0, budget: int = DEFAULT_BUDGET, max_final: int = TRUNCATE,
                 debug_mode: int = 0, count_probes: bool = False, algorithm: int = N.LC_ALGO_LINEAR,
                 devices: Optional[Sequence[int]] = None, comm: Optional[tuple] = None,
                 path_flags: int = 0, spec_segs: int = 0, spec_ck: Optional[tuple] = None, seg_len: int = 0):
        """path_flags / spec_segs / spec_ck (ck1, ck2) / seg_len pin search-path
        choices (lc_opts, ABI 9; A/B runs and tests): results never depend on them."""
        o = N.LcOpts()
        o.device, o.algorithm, o.max_configs, o.max_final = device, algorithm, budget, max_final
        o.flags = N.LC_OPT_COUNT_PROBES if count_probes else 0
        o.debug_mode = debug_mode  # ablation builds only; 0 = the real search
        o.path_flags, o.spec_segs, o.seg_len = path_flags, spec_segs, seg_len
        if spec_ck is not None:
            ck1, ck2 = int(spec_ck[0]), int(spec_ck[1])
            if not (0 <= ck1 <= 65534 and 0 <= ck2 <= 32766):  # the int32 word holds ck + 1 in 16 / 15 bits
                raise ValueError(f"spec_ck ({ck1}, {ck2}) out of range: 0 <= ck1 <= 65534, 0 <= ck2 <= 32766")
            o.spec_ck = (ck1 + 1) | ((ck2 + 1) << 16)
        if devices is not None and len(devices) > 1:
            o.n_devices = len(devices)
            for g, d in enumerate(devices):
                o.devices[g] = d
        if comm is not None:
            o.comm_rank, o.comm_size = comm[0], comm[1]
            C.memmove(o.comm_id, comm[2], N.LC_COMM_ID_BYTES)
        h = C.c_void_p()
        N.check(N.lib().lc_create(C.byref(o), C.byref(h)))
        self.handle, self.device, self.budget, self.max_final = h, device, budget, max_final
        self.count_probes = count_probes
        self.world = comm[1] if comm is not None and comm[1] > 1 else 1

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            N.lib().lc_destroy(h)
            self.handle = None

    def _alloc(self, K: int):
        K1 = max(K, 1)
        arrs = dict(valid=np.zeros(K1, np.int8), fail_event=np.zeros(K1, np.int32),
                    cause=np.zeros(K1, np.uint8), peak=np.zeros(K1, np.uint32),
                    final=np.zeros((K1, self.max_final, 2), np.uint64), n_final=np.zeros(K1, np.uint32),
                    analyzer=np.zeros(K1, np.uint8))
        r = N.LcResult(N.ptr(arrs["valid"], C.c_int8), N.ptr(arrs["fail_event"], C.c_int32),
                       N.ptr(arrs["cause"], C.c_uint8), N.ptr(arrs["peak"], C.c_uint32),
                       N.ptr(arrs["final"], C.c_uint64), N.ptr(arrs["n_final"], C.c_uint32),
                       N.ptr(arrs["analyzer"], C.c_uint8))
        return arrs, r

    def _results(self, arrs, K, st) -> KeyResults:
        return KeyResults(arrs["valid"][:K], arrs["fail_event"][:K], arrs["cause"][:K],
                          arrs["peak"][:K], arrs["final"][:K], arrs["n_final"][:K],
                          dict(kernel_ms=st.kernel_ms, tier0_ms=st.tier0_ms, tier3_ms=st.tier3_ms, total_ms=st.total_ms,
                               probes=st.probes, probes_t3=st.probes_t3, t3_bytes=st.t3_bytes,
                               keys_done=st.lds_keys, deep_keys=st.deep_keys, events=st.events,
                               t0_path=N.T0_PATH_NAMES.get(st.t0_path, st.t0_path), ev_word_bytes=st.ev_word_bytes,
                               wgl_ms=st.wgl_ms, wgl_keys=st.wgl_keys, wgl_spilled=st.wgl_spilled,
                               wgl_steps=st.wgl_steps),
                          arrs["analyzer"][:K])

    def check(self, packed: Packed, verdicts_only: bool = False, peaks: bool = True) -> KeyResults:
        """lc_check_batch: H2D, search, D2H.  verdicts_only: no peak sizes and
        no final configs are requested (the library's fast path; `peak`,
        `final` and `n_final` come back zero).  peaks=False: final configs
        but no peak sizes (what a Knossos-shaped result needs: the library
        then runs the segmented search with exact sets; `peak` comes back
        zero)."""
        K = packed.n_keys
        arrs, r = self._alloc(K)
        if verdicts_only:
            r = N.LcResult(r.valid, r.fail_event, r.cause, None, None, None, r.analyzer)
        elif not peaks:
            r = N.LcResult(r.valid, r.fail_event, r.cause, None, r.final_configs, r.n_final, r.analyzer)
        st = N.LcStats()
        N.check(N.lib().lc_check_batch(self.handle, C.byref(packed.view), C.byref(r), C.byref(st)))
        return self._results(arrs, K, st)

    def check_node(self, packed: Packed, block: int, out: Optional[np.ndarray] = None):
        """lc_check_node: this rank's shard from host SoA to the node's verdict
        records (block per rank, all-gathered).  Returns (records, stats)."""
        n = block * self.world
        if out is None or out.size < n:
            out = np.zeros(max(n, 1), np.uint64)
        st = N.LcStats()
        N.check(N.lib().lc_check_node(self.handle, C.byref(packed.view), block, N.ptr(out, C.c_uint64), C.byref(st)))
        return out[:n], st

    def check_node_async(self, packed: Packed, block: int, out: np.ndarray):
        """lc_check_node_async: the pipelined step.  `out` must be page-locked
        (pinned_records) and, like `packed`, left untouched until wait();
        returns (enqueued, stats): enqueued True when the step was only
        enqueued (records valid after wait; stats zero), False when it ran as
        check_node."""
        n = block * self.world
        if out.size < n or out.dtype != np.uint64:
            raise ValueError(f"records buffer of {out.size} < {n}")
        st = N.LcStats()
        rc = N.check(N.lib().lc_check_node_async(self.handle, C.byref(packed.view), block,
                                                 N.ptr(out, C.c_uint64), C.byref(st)))
        return rc == 1, st

    def node_records(self, n: int) -> np.ndarray:
        """lc_node_records: the first n records of the last gather."""
        out = np.zeros(max(n, 1), np.uint64)
        N.check(N.lib().lc_node_records(self.handle, N.ptr(out, C.c_uint64), n))
        return out[:n]

    def wait(self):
        """lc_wait: (number of asynchronous steps since the last wait, their
        span in ms from the first start to the last end)."""
        st = N.LcStats()
        n = N.check(N.lib().lc_wait(self.handle, C.byref(st)))
        return n, float(st.kernel_ms)

    def wait_step(self, back: int = 0):
        """lc_wait_step: wait for the asynchronous step `back` steps before the
        latest (later ones keep running)."""
        N.check(N.lib().lc_wait_step(self.handle, back))

    def upload(self, packed: Packed) -> "DevBatch":
        return DevBatch(self, packed)


class DevBatch:
    """A batch resident in HBM (lc_upload); check() re-runs the search on it."""

    def __init__(self, dev: Device, packed: Packed):
        self.dev, self.n_keys = dev, packed.n_keys
        h = C.c_void_p()
        N.check(N.lib().lc_upload(dev.handle, C.byref(packed.view), C.byref(h)))
        self.handle = h
        self.arrs, self.r = dev._alloc(self.n_keys)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            N.lib().lc_dev_batch_free(h)
            self.handle = None

    def check(self, peak: bool = True) -> KeyResults:
        st = N.LcStats()
        r = self.r
        if not peak:  # peak config-set sizes cost a wave reduction per event
            r = N.LcResult(r.valid, r.fail_event, r.cause, None, r.final_configs, r.n_final, r.analyzer)
        N.check(N.lib().lc_check_device(self.dev.handle, self.handle, C.byref(r), 0, C.byref(st)))
        return self.dev._results({k: v.copy() for k, v in self.arrs.items()}, self.n_keys, st)

    def check_node(self, block: int, asynchronous: bool = False) -> N.LcStats:
        """lc_check_node_device: search the resident shard and all-gather the
        node's verdict records (left in HBM; Device.node_records reads them)."""
        st = N.LcStats()
        N.check(N.lib().lc_check_node_device(self.dev.handle, self.handle, block,
                                             N.LC_DEV_ASYNC if asynchronous else 0, C.byref(st)))
        return st

    def check_into(self, r: N.LcResult, asynchronous: bool = False) -> N.LcStats:
        """Search with results written to caller-provided DEVICE arrays (no D2H).
        asynchronous: a register-tier-only step is only enqueued (LC_DEV_ASYNC);
        its stats are zero and the results are ready after Device.wait()."""
        st = N.LcStats()
        flags = N.LC_DEV_RESULT | (N.LC_DEV_ASYNC if asynchronous else 0)
        N.check(N.lib().lc_check_device(self.dev.handle, self.handle, C.byref(r), flags, C.byref(st)))
        return st


_devices: Dict[tuple, Device] = {}
_devices_lock = threading.Lock()


def device_for(device: int = 0, budget: int = DEFAULT_BUDGET, algorithm: int = N.LC_ALGO_LINEAR) -> Device:
    with _devices_lock:
        key = (device, budget, algorithm)
        if key not in _devices:
            _devices[key] = Device(device, budget, algorithm=algorithm)
        return _devices[key]


# ---------------------------------------------------------------- result maps
def merge_valid(vals: Sequence[Any]) -> Any:
    """jepsen.checker/merge-valid: false > :unknown > true."""
    out = True
    for v in vals:
        if v is False:
            return False
        if v is not True and v == "unknown":
            out = "unknown"
    return out


def _sub_op(packed: Packed, row: int) -> Dict:
    """Row as it appears in the key's sub-history (independent/subhistory
    unwraps the tuple value)."""
    return packed.hist.sub_op(row)


def _report(packed: Packed, i: int, res: "KeyResults", analyzer: str = "linear") -> np.ndarray:
    """lc_report (lc_report_wgl for :wgl): the key's Knossos-shaped
    counterexample as int64 words (include/lincheck.h), rendered natively --
    the same rendering the JVM binding decodes."""
    fin = np.ascontiguousarray(res.final[i], dtype=np.uint64) if len(res.final) else np.zeros((1, 2), np.uint64)
    nf = int(res.n_final[i]) if len(res.n_final) else 0
    fn = N.lib().lc_report_wgl if analyzer == "wgl" else N.lib().lc_report
    cap = 4096  # (C5's counterexamples: a few hundred words; a second call only past this)
    while True:
        buf = np.empty(cap, np.int64)
        n = N.check(fn(packed.handle, i, int(res.valid[i]), int(res.fail_event[i]),
                       N.ptr(fin, C.c_uint64), nf, TRUNCATE, N.ptr(buf, C.c_int64), cap))
        if n <= cap:
            return buf[:n]
        cap = n


def _render_key(packed: Packed, i: int, res: KeyResults, sub_rows: Optional[np.ndarray],
                analyzer: str = "linear") -> Dict:
    """Knossos-shaped result for key i,
    decoded from lc_report."""
    v = int(res.valid[i])
    cause = N.CAUSES.get(int(res.cause[i]), "error")
    if v == N.LC_UNKNOWN and int(res.cause[i]) == N.LC_CAUSE_ERROR:
        # the key's sub-history could not be prepared: what check-safe makes
        # of the exception knossos would throw (etcdemo.clj:115)
        return {"valid?": "unknown", "error": packed.key_error(i) or "error"}
    if v == N.LC_VALID:
        # nothing to render: the device keeps final configs of invalid keys
        # only (as gpu_checker.clj, which skips lc_report here too)
        return {"analyzer": analyzer, "configs": [], "final-paths": [], "valid?": True}
    w = _report(packed, i, res, analyzer).tolist()  # Python ints: no numpy scalar per word
    ops: Dict[tuple, Dict] = {}

    def op(inv: int, done: int) -> Dict:
        """The invocation as knossos.history/complete leaves it: it takes its
        completion's :value when it has none."""
        if (inv, done) not in ops:
            o = _sub_op(packed, inv)
            if done >= 0 and (o.get("value") is None or o.get("f") == "txn"):
                # a :txn takes its completion's micro-ops when it has some
                dv = _sub_op(packed, done).get("value")
                if dv is not None or o.get("f") != "txn":
                    o["value"] = dv
            ops[(inv, done)] = o
        return ops[(inv, done)]

    states: Dict[int, Any] = {}  # state id -> (model state, its rendered map): a key has a few

    def state_of(x: int):
        got = states.get(x)
        if got is None:
            if isinstance(packed.model, MultiRegister):
                st = packed.model.of_map(packed.state_map(i, x))
            else:
                st = packed.model.of_state(None if x == N.LC_NIL else x)
            got = states[x] = (st, st.render())
        return got

    def state(x: int):
        return state_of(x)[0]

    def rendered(x: int) -> Dict:
        return state_of(x)[1]

    op_row, prev_row, n_cfg, n_paths = w[:4]
    prev = _sub_op(packed, prev_row) if prev_row >= 0 else None
    at = 4
    configs = []
    for _ in range(n_cfg):
        st = rendered(w[at]); at += 1
        lists = []
        for _ in range(2):
            n = w[at]; at += 1
            lists.append([op(w[at + 2 * j], w[at + 2 * j + 1]) for j in range(n)])
            at += 2 * n
        configs.append({"model": st, "last-op": prev, "pending": lists[0], "linearized": lists[1]})
    paths = []
    fail_op = _sub_op(packed, op_row) if op_row >= 0 else None
    for _ in range(n_paths):
        path = [{"op": prev, "model": rendered(w[at])}]
        n = w[at + 1]; at += 2
        for j in range(n):
            path.append({"op": op(w[at], w[at + 1]), "model": rendered(w[at + 2])})
            at += 3
        f, val = fail_op["f"], fail_op.get("value")
        bad = state(w[at]).step(f, val); at += 1
        path.append({"op": fail_op, "model": {"msg": getattr(bad, "msg", None) or f"can't {f} {fmt(val)}"}})
        paths.append(path)
    out: Dict[str, Any] = {"analyzer": analyzer, "configs": configs, "final-paths": []}
    if v == N.LC_VALID:
        out["valid?"] = True
    elif v == N.LC_INVALID:
        out["valid?"] = False
        out["op"] = fail_op
        out["previous-ok"] = prev
        out["last-op"] = prev
        out["final-paths"] = paths
    else:
        out["valid?"] = "unknown"
        out["cause"] = cause
        if op_row >= 0:
            out["op"] = fail_op
    return out


# ---------------------------------------------------------------- checkers
def _analyzer_of(res: KeyResults, i: int) -> str:
    """:analyzer of key i: the analysis whose answer it carries."""
    return N.ANALYZERS.get(int(res.analyzer[i]), "linear") if res.analyzer is not None else "linear"


def _draw(test: Optional[Dict], sub: Sequence[dict], lin: Dict, subdirectory: Sequence) -> None:
    """jepsen.checker/linearizable's drawing of an analysis that is not valid
    (`when-not (:valid? a)`: :unknown is not drawn): linear.svg under the
    key's directory of the test's store, here `test["store-path"]` (the
    Python mirror has no store layout of its own; without it nothing is
    drawn).  An error while drawing is a warning, never raised, as there."""
    if lin.get("valid?") is not False or not (test or {}).get("store-path"):
        return
    try:
        from .report import render_analysis
        render_analysis(sub, lin, os.path.join(test["store-path"], *[str(d) for d in subdirectory], "linear.svg"))
    except Exception as e:  # noqa: BLE001 -- linearizable logs and goes on
        warnings.warn(f"Error rendering linearizability analysis: {e!r}")


class Linearizable:
    """jepsen.checker/linearizable (etcdemo.clj:117-118) on the device."""

    def __init__(self, opts: Dict):
        model = opts.get("model")
        if model is None:
            raise ValueError("The linearizable checker requires a model.")
        if not isinstance(model, MODELS):
            raise NotImplementedError("supported models: (model/cas-register), (model/register), (model/mutex), "
                                      "(model/multi-register)")
        # jepsen.checker/linearizable: :linear, :wgl, anything else -> competition
        algo = str(opts.get("algorithm", "competition")).lstrip(":")
        self.algorithm = {"linear": N.LC_ALGO_LINEAR, "wgl": N.LC_ALGO_WGL}.get(algo, N.LC_ALGO_COMPETITION)
        # knossos.competition returns whichever analysis finishes first: here
        # the :linear search, and WGL's for the keys :linear leaves :unknown at
        # the budget (lc_result.analyzer says which answered each key)
        self.analyzer = "wgl" if self.algorithm == N.LC_ALGO_WGL else "linear"
        self.model = model
        self.budget = int(opts.get("max-configs", DEFAULT_BUDGET))
        self.device = int(opts.get("device", 0))

    def _dev(self) -> Device:
        return device_for(self.device, self.budget, self.algorithm)

    def check(self, test: Dict, history, opts: Dict | None = None) -> Dict:
        """One key's (unwrapped) sub-history, as at etcdemo.clj:117."""
        hist = history if isinstance(history, History) else History.from_ops(history, default_key=0)
        packed = Packed(hist, self.model)
        if packed.n_keys == 0:
            return {"valid?": True, "configs": [], "final-paths": [], "analyzer": self.analyzer}
        res = self._dev().check(packed, peaks=False)
        out = _render_key(packed, 0, res, None, _analyzer_of(res, 0))
        _draw(test, history if not isinstance(history, History) else history.to_ops(), out,
              (opts or {}).get("subdirectory") or [])
        return out

    # batched form, used by independent.checker
    def check_independent(self, test, history, opts, inner) -> Dict:
        from .independent import merge_results, subhistory
        t0 = time.perf_counter()
        hist = history if isinstance(history, History) else History.from_ops(history)
        packed = Packed(hist, self.model)
        t1 = time.perf_counter()
        res = self._dev().check(packed, peaks=False) if packed.n_keys else None
        t2 = time.perf_counter()
        # the result maps are thousands of small dicts, none cyclic: the
        # collector's passes over the process's objects while they are made
        # cost more than making them (3x on the box, bench --jepsen)
        gc_was = gc.isenabled()
        gc.disable()
        try:
            return self._shape(test, history, opts, inner, hist, packed, res, t0, t1, t2)
        finally:
            if gc_was:
                gc.enable()

    def _shape(self, test, history, opts, inner, hist, packed, res, t0, t1, t2) -> Dict:
        from .independent import merge_results, subhistory
        results = {}
        ops_cache = None
        # the other checkers of a compose, and whether any reads a sub-history
        parts = [] if inner is self else list(inner.checkers.items())
        # compose members whose answer is a constant (:timeline's stand-in):
        # their map per key without the check-safe call and the per-key opts
        const = {name for name, ch in parts if type(ch) is UnbridledOptimism}
        only_const = all(ch is self or name in const for name, ch in parts)
        draw = bool((test or {}).get("store-path"))
        if not draw and (inner is self or only_const) and res is not None and SHARED_VALID_MAPS:
            return self._shape_fast(parts, inner, packed, res, t0, t1, t2)
        valid = res.valid.tolist() if res is not None else []
        names = {code: name for code, name in N.ANALYZERS.items()}
        anl = res.analyzer.tolist() if res is not None and res.analyzer is not None else None
        for i, k in enumerate(packed.keys):
            analyzer = names.get(anl[i], "linear") if anl is not None else "linear"
            if valid[i] == N.LC_VALID:
                # nothing to render (as _render_key): the common case, inline
                lin = {"analyzer": analyzer, "configs": [], "final-paths": [], "valid?": True}
            else:
                lin = _render_key(packed, i, res, None, analyzer)
            if draw and lin.get("valid?") is False:
                if ops_cache is None:
                    ops_cache = history if not isinstance(history, History) else history.to_ops()
                _draw(test, subhistory(ops_cache, k), lin, ["independent", str(k)])
            if inner is self:
                results[k] = lin
                continue
            if only_const:
                # {:linear lin, :timeline {:valid? true}}: merge-valid is lin's
                r = {name: (lin if ch is self else {"valid?": True}) for name, ch in parts}
                r["valid?"] = merge_valid((lin.get("valid?"),))
                results[k] = r
                continue
            # compose: run the other checkers per key on the host (the
            # sub-history is built only for checkers that read one)
            sub = None
            r = {}
            for name, ch in parts:
                if ch is self:
                    r[name] = lin
                    continue
                if name in const:
                    r[name] = {"valid?": True}
                    continue
                if sub is None and getattr(ch, "needs_history", True):
                    if ops_cache is None:
                        ops_cache = history if not isinstance(history, History) else history.to_ops()
                    sub = subhistory(ops_cache, k)
                r[name] = check_safe(ch, test, sub, dict(opts or {}, **{"history-key": k}))
            r["valid?"] = merge_valid([x.get("valid?") for x in r.values()])
            results[k] = r
        out = merge_results(results)
        if res is not None:
            out["stats"] = res.stats
        # where the call went (bench.py --jepsen): history -> packed SoA,
        # lc_check_batch (H2D, search, D2H), result maps + counterexamples
        self.last_timing = {"pack_ms": (t1 - t0) * 1e3, "search_ms": (t2 - t1) * 1e3,
                            "shape_ms": (time.perf_counter() - t2) * 1e3}
        return out


    def _shape_fast(self, parts, inner, packed, res, t0, t1, t2) -> Dict:
        """_shape for the drop-in's own expression (etcdemo.clj:115-119:
        linearizable alone, or composed with constant checkers such as
        :timeline's stand-in) when nothing is drawn.  The valid keys -- nearly
        all of them -- carry one shared result map per analyzer, placed by
        dict.fromkeys, the key-order failure list and merge-valid come from
        the verdict array, and only the other keys are rendered one by one.
        The maps are values, as Clojure's persistent maps are (do not mutate
        them: a valid key's map is shared with the other valid keys of the
        same check).  VERDICT r5 next #7: C5's 1,000-key result shaping."""
        keys = packed.keys
        valid = np.asarray(res.valid)
        names = N.ANALYZERS
        anl = np.asarray(res.analyzer) if res.analyzer is not None else None
        base_code = N.LC_ALGO_WGL if self.analyzer == "wgl" else N.LC_ALGO_LINEAR

        def wrap(lin):
            if inner is self:
                return lin
            r = {name: (lin if ch is self else {"valid?": True}) for name, ch in parts}
            r["valid?"] = merge_valid((lin.get("valid?"),))
            return r

        shared = {}

        def valid_map(code):
            m = shared.get(code)
            if m is None:
                m = shared[code] = wrap({"analyzer": names.get(code, "linear"), "configs": [], "final-paths": [],
                                         "valid?": True})
            return m
        results = dict.fromkeys(keys, valid_map(base_code))
        odd = valid != N.LC_VALID
        if anl is not None:
            odd |= anl != base_code
        for i in np.flatnonzero(odd).tolist():
            code = int(anl[i]) if anl is not None else base_code
            analyzer = names.get(code, "linear")
            results[keys[i]] = valid_map(code) if valid[i] == N.LC_VALID else wrap(_render_key(packed, i, res, None,
                                                                                               analyzer))
        bad = np.flatnonzero(valid == N.LC_INVALID)
        # merge-valid over the keys: false > :unknown > true
        out = {"valid?": False if bad.size else ("unknown" if (valid != N.LC_VALID).any() else True),
               "results": results, "failures": [keys[i] for i in bad.tolist()]}
        out["stats"] = res.stats
        self.last_timing = {"pack_ms": (t1 - t0) * 1e3, "search_ms": (t2 - t1) * 1e3,
                            "shape_ms": (time.perf_counter() - t2) * 1e3}
        return out


# The fast result shaping (Linearizable._shape_fast); False takes the general
# per-key path (tests compare the two).
SHARED_VALID_MAPS = True


class Compose:
    """jepsen.checker/compose."""

    def __init__(self, checkers: Dict[str, Any]):
        self.checkers = dict(checkers)

    def check(self, test, history, opts=None) -> Dict:
        r = {name: check_safe(ch, test, history, opts) for name, ch in self.checkers.items()}
        r["valid?"] = merge_valid([x.get("valid?") for x in r.values()])
        return r


class UnbridledOptimism:
    """jepsen.checker/unbridled-optimism: always valid (stands in for :timeline)."""

    needs_history = False

    def check(self, test, history, opts=None) -> Dict:
        return {"valid?": True}


def linearizable(opts: Dict) -> Linearizable:
    return Linearizable(opts)


def compose(checkers: Dict[str, Any]) -> Compose:
    return Compose(checkers)


def unbridled_optimism() -> UnbridledOptimism:
    return UnbridledOptimism()


def check_safe(checker, test, history, opts=None) -> Dict:
    """jepsen.checker/check-safe: exceptions become {:valid? :unknown :error ...}."""
    try:
        return checker.check(test, history, opts or {})
    except Exception as e:  # noqa: BLE001 -- mirrors check-safe catching Throwable
        return {"valid?": "unknown", "error": "".join(traceback.format_exception_only(type(e), e)).strip()}


def batched_linearizable(inner) -> Optional[Linearizable]:
    """The Linearizable inside `inner` if independent.checker can batch it."""
    if isinstance(inner, Linearizable):
        return inner
    if isinstance(inner, Compose):
        lins = [c for c in inner.checkers.values() if isinstance(c, Linearizable)]
        if len(lins) == 1:
            return lins[0]
    return None
