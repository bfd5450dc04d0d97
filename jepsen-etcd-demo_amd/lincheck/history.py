"""Jepsen histories <-> the struct-of-arrays lc_history of include/lincheck.h.

An op is a dict with Jepsen's keys as strings: "type" (invoke/ok/fail/info),
"f" (read/write/cas/...), "value", "process", optional "index", "time",
"error".  Independent ops carry `independent.tuple(k, v)` values
(etcdemo.clj:90, :120); cas values are [old new] lists (etcdemo.clj:69);
(model/multi-register) :txn values are lists of ["read"|"write", register, v]
micro-ops (registers: integers or names, interned to integer ids here).

`History` keeps the integer columns the C ABI consumes; this is the
marshalling the Clojure side does before its JNA call.
"""

from __future__ import annotations

import ctypes as C
from typing import Iterable, List, Optional, Sequence

import numpy as np

from . import _native as N
from .independent import Tuple, is_tuple

TYPES = {"invoke": N.LC_INVOKE, "ok": N.LC_OK_T, "fail": N.LC_FAIL, "info": N.LC_INFO}
TYPE_NAMES = {v: k for k, v in TYPES.items()}
FS = {"read": N.LC_F_READ, "write": N.LC_F_WRITE, "cas": N.LC_F_CAS,
      "acquire": N.LC_F_ACQUIRE, "release": N.LC_F_RELEASE, "txn": N.LC_F_TXN}
MOPS = {"read": N.LC_MOP_READ, "write": N.LC_MOP_WRITE}
MOP_NAMES = {v: k for k, v in MOPS.items()}
NAMED_REG_BASE = 1 << 62  # register names (non-integer registers) get ids from here
F_NAMES = {v: k for k, v in FS.items()}
NIL = N.LC_NIL


def _int_or_nil(v, what: str) -> int:
    if v is None:
        return NIL
    if isinstance(v, bool) or not isinstance(v, (int, np.integer)):
        raise ValueError(f"{what}: only integer (or nil) register values are supported, got {v!r}")
    v = int(v)
    if v == NIL:
        raise ValueError(f"{what}: {v} is reserved for nil")
    return v


class _HistOwner:
    """An lc_hist handle, freed when the last numpy view of it goes."""

    def __init__(self, handle):
        self.handle = handle

    def __del__(self):
        if self.handle and N is not None:  # (at interpreter exit the module may be gone)
            N.lib().lc_hist_free(self.handle)
            self.handle = None


def _borrow(owner: _HistOwner, p, n: int, ctype) -> np.ndarray:
    """n elements at p as a numpy view; the buffer under it holds `owner`."""
    n = int(n)
    if not p or n == 0:
        return np.zeros(0, np.dtype(ctype))
    buf = (ctype * n).from_address(C.addressof(p.contents))
    buf._owner = owner
    return np.frombuffer(buf, np.dtype(ctype))


class History:
    """Columns of one history (numpy arrays, history order)."""

    def __init__(self, type_, f, process, key, v0, v1, index, other_f=None, mop_off=None, mop=None,
                 reg_names=None):
        self.type = np.ascontiguousarray(type_, dtype=np.uint8)
        self.f = np.ascontiguousarray(f, dtype=np.uint8)
        self.process = np.ascontiguousarray(process, dtype=np.int64)
        self.key = np.ascontiguousarray(key, dtype=np.int64)
        self.v0 = np.ascontiguousarray(v0, dtype=np.int64)
        self.v1 = np.ascontiguousarray(v1, dtype=np.int64)
        self.index = np.ascontiguousarray(index, dtype=np.int64)
        self.other_f = other_f or {}   # row -> original :f name for LC_F_OTHER rows
        self.anomalous_keys: List[int] = []
        # :txn micro-ops (lc_history.mop_off / mop), None when no row is a :txn
        self.mop_off = None if mop_off is None else np.ascontiguousarray(mop_off, dtype=np.int64)
        self.mop = None if mop is None else np.ascontiguousarray(mop, dtype=np.int64)
        self.reg_names = dict(reg_names or {})  # register id -> name, for named registers

    def __len__(self):
        return int(self.type.shape[0])

    # -- construction -------------------------------------------------------
    @classmethod
    def from_ops(cls, ops: Sequence[dict], default_key: Optional[int] = None) -> "History":
        """Columns of a list of op maps.  default_key files non-tuple client ops
        under that key (a single key's unwrapped sub-history, etcdemo.clj:117)."""
        n = len(ops)
        t = np.empty(n, np.uint8); f = np.empty(n, np.uint8)
        p = np.empty(n, np.int64); k = np.empty(n, np.int64)
        a = np.empty(n, np.int64); b = np.empty(n, np.int64); ix = np.empty(n, np.int64)
        other = {}
        txn_rows = {}                  # row -> [(f, register id, value)]
        reg_ids = {}                   # register name -> id
        for i, op in enumerate(ops):
            try:
                t[i] = TYPES[op["type"]]
            except KeyError:
                raise ValueError(f"op {i}: bad :type {op.get('type')!r}")
            fn = op.get("f")
            f[i] = FS.get(fn, N.LC_F_OTHER)
            if f[i] == N.LC_F_OTHER:
                other[i] = fn
            proc = op.get("process")
            p[i] = proc if isinstance(proc, (int, np.integer)) and not isinstance(proc, bool) else N.LC_NO_PROCESS
            v = op.get("value")
            if is_tuple(v):
                k[i] = _int_or_nil(v[0], f"op {i} key")
                v = v[1]
            elif default_key is not None and f[i] != N.LC_F_OTHER:
                k[i] = default_key
            else:
                k[i] = N.LC_NO_KEY
            if f[i] in (N.LC_F_ACQUIRE, N.LC_F_RELEASE):
                a[i] = b[i] = NIL          # (model/mutex) ignores the value
            elif f[i] == N.LC_F_CAS:
                if v is None:
                    a[i] = b[i] = NIL
                else:
                    if len(v) != 2:
                        raise ValueError(f"op {i}: cas value must be [old new], got {v!r}")
                    a[i] = _int_or_nil(v[0], f"op {i}"); b[i] = _int_or_nil(v[1], f"op {i}")
            elif f[i] == N.LC_F_OTHER:
                a[i] = b[i] = NIL
            elif f[i] == N.LC_F_TXN:
                a[i] = b[i] = NIL
                if v is not None:
                    txn_rows[i] = [cls._mop(i, m, reg_ids) for m in v]
            else:
                a[i] = _int_or_nil(v, f"op {i}"); b[i] = NIL
            idx = op.get("index")
            ix[i] = idx if isinstance(idx, (int, np.integer)) else -1
        mop_off = mop = None
        if txn_rows:
            mop_off = np.zeros(n + 1, np.int64)
            for i, ms in txn_rows.items():
                mop_off[i + 1] = len(ms)
            mop_off = np.cumsum(mop_off)
            mop = np.array([x for i in sorted(txn_rows) for m in txn_rows[i] for x in m], np.int64)
        return cls(t, f, p, k, a, b, ix, other, mop_off, mop, {v: k2 for k2, v in reg_ids.items()})

    @staticmethod
    def _mop(i: int, m, reg_ids: dict) -> tuple:
        """One [f k v] micro-op of row i's :txn as (LC_MOP_*, register id, value)."""
        if len(m) != 3 or str(m[0]).lstrip(":") not in MOPS:
            raise ValueError(f"op {i}: a :txn micro-op is [read|write k v], got {m!r}")
        reg = m[1]
        if isinstance(reg, (int, np.integer)) and not isinstance(reg, bool):
            rid = int(reg)
            if rid >= NAMED_REG_BASE or rid == NIL:
                raise ValueError(f"op {i}: register id {rid} is reserved")
        else:
            rid = reg_ids.setdefault(reg, NAMED_REG_BASE + len(reg_ids))
        val = _int_or_nil(m[2], f"op {i}")
        if val == NIL + 1:
            raise ValueError(f"op {i}: {val} is reserved")
        return (MOPS[str(m[0]).lstrip(":")], rid, val)

    @classmethod
    def _from_owned(cls, handle) -> "History":
        """The columns of a library-owned history (lc_synth / lc_edn_read /
        lc_fressian_read) as numpy views of its memory, not copies (a C3
        history is 17 GB): every view keeps the lc_hist alive, and the last
        one to go frees it."""
        L = N.lib()
        v = N.LcHistory()
        N.check(L.lc_hist_view(handle, C.byref(v)))
        n = v.n
        owner = _HistOwner(handle)
        h = cls(_borrow(owner, v.type, n, C.c_uint8), _borrow(owner, v.f, n, C.c_uint8),
                _borrow(owner, v.process, n, C.c_int64), _borrow(owner, v.key, n, C.c_int64),
                _borrow(owner, v.v0, n, C.c_int64), _borrow(owner, v.v1, n, C.c_int64),
                _borrow(owner, v.index, n, C.c_int64))
        if v.mop_off:
            h.mop_off = _borrow(owner, v.mop_off, n + 1, C.c_int64)
            nm = 3 * int(h.mop_off[-1])
            h.mop = _borrow(owner, v.mop, nm, C.c_int64) if nm else np.zeros(0, np.int64)
        for i in range(L.lc_hist_n_reg_names(handle)):
            h.reg_names[NAMED_REG_BASE + i] = L.lc_hist_reg_name(handle, i).decode()
        na = L.lc_hist_anomalous_keys(handle, None)
        if na > 0:
            buf = np.zeros(na, np.int64)
            L.lc_hist_anomalous_keys(handle, N.ptr(buf, C.c_int64))
            h.anomalous_keys = buf.tolist()
        return h

    # -- key subsets (a rank's shard) ---------------------
    def select_keys(self, keys) -> "History":
        """The rows of the given keys plus every row without a key (those
        belong to every key's sub-history, independent/subhistory), in
        history order; :index kept, so results name the original ops."""
        if self.mop is not None:
            raise NotImplementedError("select_keys: :txn histories")
        keep = np.isin(self.key, np.asarray(keys, np.int64)) | (self.key == N.LC_NO_KEY)
        rows = np.flatnonzero(keep)
        h = History(self.type[rows], self.f[rows], self.process[rows], self.key[rows], self.v0[rows],
                    self.v1[rows], self.index[rows], reg_names=self.reg_names)
        h.other_f = {int(j): self.other_f[int(r)] for j, r in enumerate(rows) if int(r) in self.other_f}
        return h

    @classmethod
    def concat(cls, parts: Sequence["History"]) -> "History":
        """One history of the parts' rows in order (keys must not overlap);
        :index renumbered to the row position, as a single run's history."""
        if any(p.mop is not None for p in parts):
            raise NotImplementedError("concat: :txn histories")
        cat = lambda a: np.concatenate([getattr(p, a) for p in parts])
        n = sum(len(p) for p in parts)
        h = cls(cat("type"), cat("f"), cat("process"), cat("key"), cat("v0"), cat("v1"), np.arange(n, dtype=np.int64))
        base = 0
        for p in parts:
            h.other_f.update({base + r: f for r, f in p.other_f.items()})
            h.anomalous_keys += p.anomalous_keys
            base += len(p)
        return h

    # -- views --------------------------------------------------------------
    def as_c(self) -> N.LcHistory:
        h = N.LcHistory()
        h.n = len(self)
        h.type = N.ptr(self.type, C.c_uint8); h.f = N.ptr(self.f, C.c_uint8)
        h.process = N.ptr(self.process, C.c_int64); h.key = N.ptr(self.key, C.c_int64)
        h.v0 = N.ptr(self.v0, C.c_int64); h.v1 = N.ptr(self.v1, C.c_int64)
        h.index = N.ptr(self.index, C.c_int64)
        if self.mop_off is not None:
            h.mop_off = N.ptr(self.mop_off, C.c_int64)
            h.mop = N.ptr(self.mop if self.mop.size else np.zeros(1, np.int64), C.c_int64)
        h._keep = self  # arrays stay alive with the struct
        return h

    def op(self, i: int) -> dict:
        """Row i as a Jepsen op map (tuples re-wrapped)."""
        i = int(i)
        f = int(self.f[i])
        fn = F_NAMES.get(f, self.other_f.get(i, "nemesis" if f == N.LC_F_OTHER else f))
        nil = lambda x: None if x == NIL else int(x)
        if f == N.LC_F_CAS:
            val = [nil(self.v0[i]), nil(self.v1[i])]
        elif f in (N.LC_F_OTHER, N.LC_F_ACQUIRE, N.LC_F_RELEASE):
            val = None
        elif f == N.LC_F_TXN:
            val = self.txn(i)
        else:
            val = nil(self.v0[i])
        if self.key[i] != N.LC_NO_KEY:
            val = Tuple(int(self.key[i]), val)
        proc = int(self.process[i])
        op = {"type": TYPE_NAMES[int(self.type[i])], "f": fn, "value": val,
              "process": "nemesis" if proc == N.LC_NO_PROCESS else proc}
        op["index"] = int(self.index[i]) if self.index[i] >= 0 else i
        return op

    def sub_op(self, i: int) -> dict:
        """Row i as it appears in its key's sub-history (independent/subhistory
        unwraps the tuple value): op() without building the tuple."""
        i = int(i)
        f = int(self.f[i])
        fn = F_NAMES.get(f, self.other_f.get(i, "nemesis" if f == N.LC_F_OTHER else f))
        if f == N.LC_F_CAS:
            a, b = int(self.v0[i]), int(self.v1[i])
            val = [None if a == NIL else a, None if b == NIL else b]
        elif f in (N.LC_F_OTHER, N.LC_F_ACQUIRE, N.LC_F_RELEASE):
            val = None
        elif f == N.LC_F_TXN:
            val = self.txn(i)
        else:
            a = int(self.v0[i])
            val = None if a == NIL else a
        proc = int(self.process[i])
        ix = int(self.index[i])
        return {"type": TYPE_NAMES[int(self.type[i])], "f": fn, "value": val,
                "process": "nemesis" if proc == N.LC_NO_PROCESS else proc, "index": ix if ix >= 0 else i}

    def txn(self, i: int):
        """Row i's :txn micro-ops as [f, register, value] lists (None: nil)."""
        if self.mop_off is None or self.mop_off[i + 1] == self.mop_off[i]:
            return None
        out = []
        for m in range(int(self.mop_off[i]), int(self.mop_off[i + 1])):
            f, r, v = (int(x) for x in self.mop[3 * m: 3 * m + 3])
            out.append([MOP_NAMES[f], self.reg_names.get(r, r), None if v == NIL else v])
        return out

    def to_ops(self) -> List[dict]:
        return [self.op(i) for i in range(len(self))]


# ---- generator / EDN --------------------------------------------------------
def synth(n_keys: int, ops_per_key: int, concurrency: int = 10, *, n_values: int = 5,
          info_rate: float = 0.0, info_effect_p: float = 0.5, anomaly_rate: float = 0.0,
          mean_think: float = 1.0, mean_latency: float = 1.0, interleave: bool = False,
          nemesis_period: float = 0.0, seed: int = 1, key_base: int = 0) -> History:
    """Synthetic cas-register history (lc_synth_generate)."""
    o = N.LcSynthOpts(n_keys, ops_per_key, concurrency, n_values, info_rate, info_effect_p,
                      anomaly_rate, mean_think, mean_latency, int(interleave), nemesis_period,
                      seed, key_base)
    handle = C.c_void_p()
    N.check(N.lib().lc_synth_generate(C.byref(o), C.byref(handle)))
    return History._from_owned(handle)


CONFIGS = {
    # SURVEY.md 8(d) D-2 / BASELINE.md
    "C1": dict(n_keys=6, ops_per_key=100, concurrency=10, interleave=True, nemesis_period=5.0, seed=1),
    "C2": dict(n_keys=1000, ops_per_key=1000, concurrency=10, seed=2),
    "C3": dict(n_keys=100_000, ops_per_key=2000, concurrency=10, seed=3),
    "C4": dict(n_keys=256, ops_per_key=5000, concurrency=30, info_rate=0.02, seed=4),
    "C5": dict(n_keys=1000, ops_per_key=1000, concurrency=10, anomaly_rate=0.05, seed=5),
}


def read_edn(path: str) -> History:
    handle = C.c_void_p()
    N.check(N.lib().lc_edn_read(path.encode(), C.byref(handle)))
    return History._from_owned(handle)


def parse_edn(text: str) -> History:
    raw = text.encode()
    handle = C.c_void_p()
    N.check(N.lib().lc_edn_parse(raw, len(raw), C.byref(handle)))
    return History._from_owned(handle)


def write_edn(path: str, h: History) -> None:
    """lc_edn_write_named: named :txn registers keep their names (":x")."""
    names = [h.reg_names.get(NAMED_REG_BASE + i) for i in range(len(h.reg_names))]
    if names and all(isinstance(n, str) for n in names):
        arr = (C.c_char_p * len(names))(*[n.encode() for n in names])
        N.check(N.lib().lc_edn_write_named(path.encode(), C.byref(h.as_c()), arr, len(names)))
    else:
        N.check(N.lib().lc_edn_write(path.encode(), C.byref(h.as_c())))


def read_fressian(path: str) -> History:
    """The :history of a Jepsen test.fressian (or a Fressian list of op maps)."""
    handle = C.c_void_p()
    N.check(N.lib().lc_fressian_read(path.encode(), C.byref(handle)))
    return History._from_owned(handle)


def parse_fressian(data: bytes) -> History:
    handle = C.c_void_p()
    N.check(N.lib().lc_fressian_parse(data, len(data), C.byref(handle)))
    return History._from_owned(handle)


def write_fressian(path: str, h: History) -> None:
    N.check(N.lib().lc_fressian_write(path.encode(), C.byref(h.as_c())))
