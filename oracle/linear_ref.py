"""CPU restatement of knossos.linear for the cas-register model -- TEST ORACLE.

This file is test infrastructure.  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import it, and only as the checker, never as
the thing measured or shipped.  The product path (liblincheck.so) never
routes through here.

Parity status: the reference's algorithm lives in knossos 0.3.7
(jepsen.etcdemo.iml:58), a Clojure dependency that is NOT in /root/reference
and has no JVM to run on here.  The reference ships no
golden vectors or fixtures for this path (test/jepsen/etcdemo_test.clj:5-7 is
`(is (= 0 1))`; store/latest is a dangling symlink).  This restatement is
therefore pinned only against the definitional brute-force checker in
oracle/brute.py and the hand-written known-answer histories in tests/golden/:
**parity against Knossos itself is unpinned.**

What is restated, from the published knossos 0.3.7 / jepsen 0.2.x sources
(upstream, cited by namespace; call sites in the reference are cited by line):

  jepsen.independent/checker, subhistory  (etcdemo.clj:115)
      split by tuple key; non-tuple ops (nemesis) go to every sub-history.
  knossos.history/complete, without-failures  (reached via etcdemo.clj:117)
      pair invoke -> next completion of the same process; :ok copies
      (or invocation-value completion-value) into the invocation; :fail drops
      the pair; :info / no completion leaves the op pending forever.
  knossos.model/cas-register  (etcdemo.clj:15,117)
      nil initial value; write v -> v; cas [a b] legal iff cur = a; read v
      legal iff v is nil or v = cur.
  knossos.model/register, knossos.model/mutex  
      register: the cas-register without cas.  mutex: unlocked initially;
      :acquire legal iff unlocked (-> locked), :release legal iff locked
      (-> unlocked).
  knossos.model/multi-register  
      a map of registers (initially the given one); :txn applies its
      [:read k v] / [:write k v] micro-ops in order, a read legal iff v is nil
      or k holds v (a register the map lacks holds nothing, not even nil).
      An :ok :txn takes its completion's micro-ops when it has some (the reads
      learn what they read).  A key with more than 32767 maps reachable from
      the initial one under its distinct :txn ops is :unknown "states".
  knossos.linear/analysis with :algorithm :linear  (etcdemo.clj:118)
      the just-in-time config-set search.  A config is (model state, set of
      pending ops already linearized).  :invoke adds the op to the pending
      set; :info changes nothing; :ok(p) replaces the config set S by
          S' = { (s, L - {p}) : (s, L) in S, p in L }
             U { (step(s', p), L')   : (s', L') in I, step legal }
      where I, the JIT closure, is every config reachable from
      { (s, L) in S : p not in L } by linearizing pending, not-yet-linearized
      ops other than p.  The history is invalid at the first :ok whose S' is
      empty (that event is the reported :op).
  jepsen.checker/check-safe around each key (independent/checker,
      etcdemo.clj:115): a key whose sub-history complete rejects, or that
      holds an op the model cannot step, is :unknown with cause "error"
      (check_independent / analysis_safe); the other keys are still checked.
  knossos.search (abort -> :unknown) is replaced by a deterministic budget:
      a key whose closure I or config set S' exceeds `budget` configs is
      :unknown with cause "budget".  Two representation limits are applied in
      the same event order as the device: an :invoke that needs pending-window
      slot >= 112 (lowest free slot at invoke, freed at :ok) -> :unknown
      "window"; a key with more than 32767 register values -> :unknown
      "states" before its first event.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, FrozenSet, Iterable, List, Optional, Sequence, Tuple

WIDE_MAX_SLOTS = 112      # include/lincheck.h LC_WIDE_MAX_SLOTS
WIDE_MAX_STATES = 32767   # include/lincheck.h LC_WIDE_MAX_STATES
DEFAULT_BUDGET = 1 << 20  # include/lincheck.h lc_opts.max_configs default

INCONSISTENT = object()


def is_tuple(v) -> bool:
    """jepsen.independent/tuple? -- the product's Tuple marks itself."""
    return bool(getattr(v, "_lc_tuple", False))


# --------------------------------------------------------------------------- A2
def history_keys(history: Sequence[dict]) -> List[Any]:
    """jepsen.independent/history-keys: tuple keys in order of first use."""
    seen, out = set(), []
    for op in history:
        v = op.get("value")
        if is_tuple(v) and v[0] not in seen:
            seen.add(v[0])
            out.append(v[0])
    return out


def subhistory(history: Sequence[dict], k) -> List[dict]:
    """jepsen.independent/subhistory: ops on key k (unwrapped) + non-tuple ops."""
    out = []
    for op in history:
        v = op.get("value")
        if is_tuple(v):
            if v[0] == k:
                o = dict(op)
                o["value"] = v[1]
                out.append(o)
        else:
            out.append(op)
    return out


# --------------------------------------------------------------------------- A3
@dataclass
class Op:
    """One client operation after knossos.history/complete."""
    id: int
    f: str
    value: Any
    invoke_pos: int              # position of the :invoke in the sub-history
    complete_pos: Optional[int]  # position of the :ok, None if pending forever
    failed: bool = False


class HistoryError(Exception):
    """knossos.history/complete's assertion (or an op the model cannot step)."""


MODEL_FS = {"cas-register": ("read", "write", "cas"), "register": ("read", "write"),
            "mutex": ("acquire", "release"), "multi-register": ("txn",)}


def complete(history: Sequence[dict], model: str = "cas-register") -> Tuple[List[Op], List[Tuple[str, int, int]]]:
    """knossos.history/complete + without-failures.

    Returns (ops, events) where events is the sub-history reduced to the
    search's input: ("invoke", op_id, pos) and ("ok", op_id, pos), in order;
    failed ops are gone and :info completions produce no event.
    """
    ops: List[Op] = []
    outstanding: Dict[Any, int] = {}
    ok_at: Dict[int, int] = {}
    for pos, op in enumerate(history):
        t, p = op.get("type"), op.get("process")
        if t == "invoke":
            if op.get("f") not in MODEL_FS[model]:
                raise HistoryError(f"{model} cannot step {op.get('f')!r}")
            ops.append(Op(len(ops), op["f"], op.get("value"), pos, None))
            outstanding[p] = len(ops) - 1   # assoc! overwrites an older one
        elif t in ("ok", "fail"):
            if p not in outstanding:
                raise HistoryError(f"process {p!r} completed an operation without a prior invocation")
            o = ops[outstanding.pop(p)]
            if t == "ok":
                if o.f == "txn":             # a :txn learns its completion's micro-ops
                    if op.get("value") is not None:
                        o.value = op.get("value")
                elif o.value is None:        # (or (:value invocation) (:value op))
                    o.value = op.get("value")
                o.complete_pos = pos
                ok_at[pos] = o.id
            else:
                o.failed = True
        elif t == "info":
            outstanding.pop(p, None)         # crashed: pending forever
    events = []
    for pos, op in enumerate(history):
        t = op.get("type")
        if t == "invoke":
            o = next_op_at(ops, pos)
            if o is not None and not o.failed:
                events.append(("invoke", o.id, pos))
        elif t == "ok" and pos in ok_at:
            events.append(("ok", ok_at[pos], pos))
    return ops, events


def next_op_at(ops: List[Op], pos: int) -> Optional[Op]:
    # ops are created in invoke order; binary search by invoke_pos
    lo, hi = 0, len(ops)
    while lo < hi:
        mid = (lo + hi) // 2
        if ops[mid].invoke_pos < pos:
            lo = mid + 1
        else:
            hi = mid
    return ops[lo] if lo < len(ops) and ops[lo].invoke_pos == pos else None


# --------------------------------------------------------------------------- A4
def cas_register_step(state, f: str, value):
    """knossos.model/cas-register's CASRegister step."""
    if f == "write":
        return value
    if f == "cas":
        cur, new = (value if value is not None else (None, None))
        return new if cur == state else INCONSISTENT
    if f == "read":
        return state if (value is None or value == state) else INCONSISTENT
    raise HistoryError(f"cas-register cannot step {f!r}")


def mutex_step(locked: bool, f: str, value=None):
    """knossos.model/mutex's Mutex step (locked? = True / False)."""
    if f == "acquire":
        return INCONSISTENT if locked else True
    if f == "release":
        return False if locked else INCONSISTENT
    raise HistoryError(f"mutex cannot step {f!r}")


def _reg_order(kv):
    return (str(type(kv[0])), kv[0])


def multi_register_step(state, f: str, value):
    """knossos.model/multi-register's MultiRegister step; state = the map as a
    sorted tuple of (register, value)."""
    if f != "txn":
        raise HistoryError(f"multi-register cannot step {f!r}")
    regs = dict(state)
    for m in (value or ()):
        mf, k, v = m
        mf = str(mf).lstrip(":")
        if mf == "read":
            if v is not None and (k not in regs or regs[k] != v):
                return INCONSISTENT
        elif mf == "write":
            regs[k] = v
        else:
            raise HistoryError(f"multi-register cannot step micro-op {mf!r}")
    return tuple(sorted(regs.items(), key=_reg_order))


def multi_register_init(values=None):
    return tuple(sorted((values or {}).items(), key=_reg_order))


def reachable_maps(ops: Iterable[Op], initial, cap: int) -> int:
    """knossos.model.memo for multi-register: how many maps are reachable
    from `initial` under the distinct :txn values of the surviving ops
    (counting stops past cap)."""
    txns = []
    seen_t = set()
    for o in ops:
        if o.failed:
            continue
        key = repr(o.value)
        if key not in seen_t:
            seen_t.add(key)
            txns.append(o.value)
    seen = {initial}
    frontier = [initial]
    while frontier and len(seen) <= cap:
        nxt = []
        for st in frontier:
            for t in txns:
                s2 = multi_register_step(st, "txn", t)
                if s2 is not INCONSISTENT and s2 not in seen:
                    seen.add(s2)
                    nxt.append(s2)
        frontier = nxt
    return len(seen)


def model_step(model: str):
    """(step fn, initial state) of a model."""
    if model == "mutex":
        return mutex_step, False
    if model == "multi-register":
        return multi_register_step, multi_register_init()
    return cas_register_step, None


def register_values(ops: Iterable[Op]) -> set:
    """Values a surviving write / cas can install (the key's state count - 1)."""
    vals = set()
    for o in ops:
        if o.failed:
            continue
        if o.f == "write" and o.value is not None:
            vals.add(o.value)
        if o.f == "cas" and o.value is not None and o.value[1] is not None:
            vals.add(o.value[1])
    return vals


# --------------------------------------------------------------------------- A6
Config = Tuple[Any, FrozenSet[int]]


@dataclass
class Analysis:
    valid: Any                      # True / False / "unknown"
    cause: str = "none"             # none / nonlin / budget / window / states
    op_id: Optional[int] = None     # op that could not be linearized
    fail_event: Optional[int] = None  # ordinal in the reduced event list
    fail_pos: Optional[int] = None  # position in the sub-history
    previous_ok_pos: Optional[int] = None
    final_configs: List[Config] = field(default_factory=list)
    final_slots: Dict[int, int] = field(default_factory=dict)  # op id -> window slot at failure
    peak_configs: int = 1
    probes: int = 0
    ops: List[Op] = field(default_factory=list)
    events: list = field(default_factory=list)


def analysis(history: Sequence[dict], budget: int = DEFAULT_BUDGET,
             initial=None, model: str = "cas-register") -> Analysis:
    """knossos.linear/analysis over one key's sub-history (default: cas-register)."""
    ops, events = complete(history, model)
    step, init = model_step(model)
    if initial is None:
        initial = init
    res = Analysis(valid=True, ops=ops, events=events)
    if model == "multi-register":
        if reachable_maps(ops, initial, WIDE_MAX_STATES) > WIDE_MAX_STATES:
            res.valid, res.cause = "unknown", "states"
            return res
    elif len(register_values(ops)) + 1 > WIDE_MAX_STATES:
        res.valid, res.cause = "unknown", "states"
        return res
    S = {(initial, frozenset())}
    pending: List[int] = []           # op ids, in invoke order
    free_slots = list(range(128))
    slot_of: Dict[int, int] = {}
    last_ok_pos = None
    for ei, (kind, oid, pos) in enumerate(events):
        if kind == "invoke":
            s = min(free_slots)
            if s >= WIDE_MAX_SLOTS:
                res.valid, res.cause = "unknown", "window"
                return res
            free_slots.remove(s)
            slot_of[oid] = s
            pending.append(oid)
            continue
        p = oid
        res.probes += len(S)
        S_next = set()
        frontier = []
        I = set()
        for (st, L) in S:
            if p in L:
                S_next.add((st, L - {p}))
            else:
                I.add((st, L))
                frontier.append((st, L))
        # JIT closure over pending ops other than p
        while frontier:
            nxt = []
            for (st, L) in frontier:
                for q in pending:
                    if q == p or q in L:
                        continue
                    s2 = step(st, ops[q].f, ops[q].value)
                    if s2 is INCONSISTENT:
                        continue
                    res.probes += 1
                    c = (s2, L | {q})
                    if c not in I:
                        I.add(c)
                        if len(I) > budget:
                            res.valid, res.cause = "unknown", "budget"
                            res.fail_event, res.fail_pos = ei, pos
                            return res
                        nxt.append(c)
            frontier = nxt
        for (st, L) in I:
            s2 = step(st, ops[p].f, ops[p].value)
            if s2 is INCONSISTENT:
                continue
            res.probes += 1
            S_next.add((s2, L))
        if not S_next:
            res.valid, res.cause = False, "nonlin"
            res.op_id, res.fail_event, res.fail_pos = p, ei, pos
            res.previous_ok_pos = last_ok_pos
            res.final_configs = sorted(S, key=config_sort_key)
            res.final_slots = dict(slot_of)
            return res
        if len(S_next) > budget:
            res.valid, res.cause = "unknown", "budget"
            res.fail_event, res.fail_pos = ei, pos
            return res
        S = S_next
        res.peak_configs = max(res.peak_configs, len(S))
        pending.remove(p)
        free_slots.append(slot_of.pop(p))
        last_ok_pos = pos
    return res


def final_paths(res: Analysis, sub: Sequence[dict], model: str = "cas-register",
                cap: int = 1 << 16) -> set:
    """Every final path of an invalid analysis, as a set
    of tuples ((index, state), ..., (index, "inconsistent")): from each final
    config, each sequence of further pending ops (other than the failing op p)
    that the model allows, then p, which is inconsistent in every state so
    reached.  The first element is (previous-ok's :index or None, config
    state); ops are named by their invocation's :index, p by its :ok's.
    None when there are more than `cap` paths (the set is then not known)."""
    assert res.valid is False
    step, _ = model_step(model)
    ops = res.ops
    p = res.op_id
    idx = lambda pos: sub[pos].get("index", pos)
    prev = idx(res.previous_ok_pos) if res.previous_ok_pos is not None else None
    pend = sorted((q for q in res.final_slots if q != p), key=lambda q: res.final_slots[q])
    out = set()

    def dfs(st0, st, L, steps):
        if len(out) >= cap:
            return
        if step(st, ops[p].f, ops[p].value) is INCONSISTENT:
            out.add(((prev, st0),) + tuple(steps) + ((idx(res.fail_pos), "inconsistent"),))
        for q in pend:
            if q in L:
                continue
            s2 = step(st, ops[q].f, ops[q].value)
            if s2 is not INCONSISTENT:
                steps.append((idx(ops[q].invoke_pos), s2))
                dfs(st0, s2, L | {q}, steps)
                steps.pop()

    for st, L in res.final_configs:
        dfs(st, st, L, [])
    return None if len(out) >= cap else out


def config_sort_key(c: Config):
    st, L = c
    if isinstance(st, tuple):  # a multi-register map
        return (repr(st), sorted(L))
    return (-1 if st is None else int(st), sorted(L))


def analysis_safe(history: Sequence[dict], budget: int = DEFAULT_BUDGET, model: str = "cas-register",
                  initial=None) -> Analysis:
    """check-safe around analysis: a HistoryError makes the key :unknown
    (cause "error") instead of aborting the whole check."""
    try:
        return analysis(history, budget, initial=initial, model=model)
    except HistoryError as e:
        a = Analysis(valid="unknown", cause="error", peak_configs=0)
        a.error = str(e)
        return a


def check_independent(history: Sequence[dict], budget: int = DEFAULT_BUDGET,
                      model: str = "cas-register", initial=None) -> Dict[Any, Analysis]:
    """independent/checker over linearizable(model): per-key analyses."""
    return {k: analysis_safe(subhistory(history, k), budget, model=model, initial=initial)
            for k in history_keys(history)}
