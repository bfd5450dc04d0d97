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
import threading
import traceback
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from . import _native as N
from .history import History
from .model import MODELS, CASRegister, fmt

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
        N.check(N.lib().lc_pack(C.byref(self._c), C.byref(opts), C.byref(handle)))
        self.handle = handle
        v = N.LcBatch()
        N.check(N.lib().lc_packed_view(self.handle, C.byref(v)))
        self.view = v
        self.n_keys = int(v.n_keys)
        self.ev_off = N.carray(v.ev_off, self.n_keys + 1, np.uint64)
        self.keys = [int(N.lib().lc_packed_key(self.handle, i)) for i in range(self.n_keys)]

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            N.lib().lc_packed_free(h)
            self.handle = None

    def n_events(self, i: int) -> int:
        return int(self.ev_off[i + 1] - self.ev_off[i])

    def events(self, i: int) -> np.ndarray:
        b, e = int(self.ev_off[i]), int(self.ev_off[i + 1])
        if e == b:
            return np.zeros(0, np.uint32)
        return np.ctypeslib.as_array(self.view.events, shape=(int(self.ev_off[-1]) or 1,))[b:e].copy()

    def event_row(self, i: int, j: int) -> int:
        return int(N.check(N.lib().lc_packed_event_row(self.handle, i, j)))

    def state_value(self, i: int, s: int):
        v = C.c_int64(); nil = C.c_int()
        N.check(N.lib().lc_packed_state_value(self.handle, i, s, C.byref(v), C.byref(nil)))
        return None if nil.value else int(v.value)


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


class Device:
    """An lc_ctx on one GPU (lc_create)."""

    def __init__(self, device: int = 0, budget: int = DEFAULT_BUDGET, max_final: int = TRUNCATE,
                 debug_mode: int = 0, count_probes: bool = False):
        o = N.LcOpts()
        o.device, o.algorithm, o.max_configs, o.max_final = device, 0, budget, max_final
        o.flags = N.LC_OPT_COUNT_PROBES if count_probes else 0
        o.debug_mode = debug_mode  # ablation builds only; 0 = the real search
        h = C.c_void_p()
        N.check(N.lib().lc_create(C.byref(o), C.byref(h)))
        self.handle, self.device, self.budget, self.max_final = h, device, budget, max_final
        self.count_probes = count_probes

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            N.lib().lc_destroy(h)
            self.handle = None

    def _alloc(self, K: int):
        K1 = max(K, 1)
        arrs = dict(valid=np.zeros(K1, np.int8), fail_event=np.zeros(K1, np.int32),
                    cause=np.zeros(K1, np.uint8), peak=np.zeros(K1, np.uint32),
                    final=np.zeros((K1, self.max_final, 2), np.uint64), n_final=np.zeros(K1, np.uint32))
        r = N.LcResult(N.ptr(arrs["valid"], C.c_int8), N.ptr(arrs["fail_event"], C.c_int32),
                       N.ptr(arrs["cause"], C.c_uint8), N.ptr(arrs["peak"], C.c_uint32),
                       N.ptr(arrs["final"], C.c_uint64), N.ptr(arrs["n_final"], C.c_uint32))
        return arrs, r

    def _results(self, arrs, K, st) -> KeyResults:
        return KeyResults(arrs["valid"][:K], arrs["fail_event"][:K], arrs["cause"][:K],
                          arrs["peak"][:K], arrs["final"][:K], arrs["n_final"][:K],
                          dict(kernel_ms=st.kernel_ms, tier0_ms=st.tier0_ms, total_ms=st.total_ms, probes=st.probes,
                               keys_done=st.lds_keys, deep_keys=st.deep_keys, events=st.events))

    def check(self, packed: Packed) -> KeyResults:
        """lc_check_batch: H2D, search, D2H."""
        K = packed.n_keys
        arrs, r = self._alloc(K)
        st = N.LcStats()
        N.check(N.lib().lc_check_batch(self.handle, C.byref(packed.view), C.byref(r), C.byref(st)))
        return self._results(arrs, K, st)

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
            r = N.LcResult(r.valid, r.fail_event, r.cause, None, r.final_configs, r.n_final)
        N.check(N.lib().lc_check_device(self.dev.handle, self.handle, C.byref(r), 0, C.byref(st)))
        return self.dev._results({k: v.copy() for k, v in self.arrs.items()}, self.n_keys, st)

    def check_into(self, r: N.LcResult) -> N.LcStats:
        """Search with results written to caller-provided DEVICE arrays (no D2H)."""
        st = N.LcStats()
        N.check(N.lib().lc_check_device(self.dev.handle, self.handle, C.byref(r), 1, C.byref(st)))
        return st


_devices: Dict[tuple, Device] = {}
_devices_lock = threading.Lock()


def device_for(device: int = 0, budget: int = DEFAULT_BUDGET) -> Device:
    with _devices_lock:
        key = (device, budget)
        if key not in _devices:
            _devices[key] = Device(device, budget)
        return _devices[key]


# ---------------------------------------------------------------- result maps
def merge_valid(vals: Sequence[Any]) -> Any:
    """jepsen.checker/merge-valid: false > :unknown > true."""
    vals = list(vals)
    if any(v is False for v in vals):
        return False
    if any(v == "unknown" for v in vals):
        return "unknown"
    return True


def _render_key(packed: Packed, i: int, res: KeyResults, sub_rows: Optional[np.ndarray]) -> Dict:
    """Knossos-shaped result for key i."""
    hist = packed.hist
    v = int(res.valid[i])
    cause = N.CAUSES.get(int(res.cause[i]), "error")
    ev = packed.events(i)
    fe = int(res.fail_event[i])
    upto = fe if fe >= 0 else len(ev)
    # which op holds each window slot just before event `upto`
    slot_op: Dict[int, int] = {}
    last_ok = None
    for j in range(upto):
        w = int(ev[j]); s = (w >> 24) & 0x7F
        if w & N.LC_EV_OK_BIT:
            slot_op.pop(s, None)
            last_ok = j
        else:
            slot_op[s] = j
    configs = []
    for c in range(int(res.n_final[i])):
        lo, hi = int(res.final[i, c, 0]), int(res.final[i, c, 1])
        st = (hi >> 48) & 0x7FFF
        mask = lo | ((hi & ((1 << 48) - 1)) << 64)
        pend = [hist.op(packed.event_row(i, slot_op[s])) for s in sorted(slot_op) if not (mask >> s) & 1]
        lin = [hist.op(packed.event_row(i, slot_op[s])) for s in sorted(slot_op) if (mask >> s) & 1]
        configs.append({"model": packed.model.of_state(packed.state_value(i, st)).render(),
                        "pending": pend, "linearized": lin})
    out: Dict[str, Any] = {"analyzer": "linear", "configs": configs[:TRUNCATE], "final-paths": []}
    if v == N.LC_VALID:
        out["valid?"] = True
    elif v == N.LC_INVALID:
        out["valid?"] = False
        op = hist.op(packed.event_row(i, fe))
        out["op"] = op
        prev = hist.op(packed.event_row(i, last_ok)) if last_ok is not None else None
        out["previous-ok"] = prev
        out["last-op"] = prev
    else:
        out["valid?"] = "unknown"
        out["cause"] = cause
        if fe >= 0:
            out["op"] = hist.op(packed.event_row(i, fe))
    return out


# ---------------------------------------------------------------- checkers
class Linearizable:
    """jepsen.checker/linearizable (etcdemo.clj:117-118) on the device."""

    def __init__(self, opts: Dict):
        model = opts.get("model")
        if model is None:
            raise ValueError("The linearizable checker requires a model.")
        if not isinstance(model, MODELS):
            raise NotImplementedError("supported models: (model/cas-register), (model/register), (model/mutex)")
        algo = opts.get("algorithm", "linear")
        if algo not in ("linear", ":linear"):
            raise NotImplementedError(f"algorithm {algo!r}: only :linear is implemented")
        self.model = model
        self.budget = int(opts.get("max-configs", DEFAULT_BUDGET))
        self.device = int(opts.get("device", 0))

    def _dev(self) -> Device:
        return device_for(self.device, self.budget)

    def check(self, test: Dict, history, opts: Dict | None = None) -> Dict:
        """One key's (unwrapped) sub-history, as at etcdemo.clj:117."""
        hist = history if isinstance(history, History) else History.from_ops(history, default_key=0)
        packed = Packed(hist, self.model)
        if packed.n_keys == 0:
            return {"valid?": True, "configs": [], "final-paths": [], "analyzer": "linear"}
        res = self._dev().check(packed)
        return _render_key(packed, 0, res, None)

    # batched form, used by independent.checker
    def check_independent(self, test, history, opts, inner) -> Dict:
        from .independent import merge_results, subhistory
        hist = history if isinstance(history, History) else History.from_ops(history)
        packed = Packed(hist, self.model)
        res = self._dev().check(packed) if packed.n_keys else None
        results = {}
        ops_cache = None
        for i, k in enumerate(packed.keys):
            lin = _render_key(packed, i, res, None)
            if inner is self:
                results[k] = lin
                continue
            # compose: run the other checkers per key on the host
            if ops_cache is None:
                ops_cache = history if not isinstance(history, History) else history.to_ops()
            sub = subhistory(ops_cache, k)
            r = {}
            for name, ch in inner.checkers.items():
                r[name] = lin if ch is self else check_safe(ch, test, sub, dict(opts or {}, **{"history-key": k}))
            r["valid?"] = merge_valid([x.get("valid?") for x in r.values()])
            results[k] = r
        out = merge_results(results)
        if res is not None:
            out["stats"] = res.stats
        return out


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
