"""CPU restatement of knossos.wgl for one key -- TEST ORACLE.

This file is test infrastructure.  Only tests/ may import it, and only as the
checker, never as the thing measured or shipped.  The product path
(liblincheck.so) never routes through here.

Parity status: knossos 0.3.7 (jepsen.etcdemo.iml:58) is absent from
/root/reference and has no JVM to run on here; the
reference holds no fixtures for this path.  **Parity against Knossos itself
is unpinned.**  What is restated, from the published algorithm knossos.wgl
implements (Wing & Gong 1993, with Lowe's cache of (linearized set, model
state) pairs; SURVEY.md 8(f) F-3, the `:algorithm :wgl` value of the slot at
etcdemo.clj:118):

  The key's sub-history (after knossos.history/complete + without-failures,
  restated in linear_ref.complete) becomes a list of call and return entries
  in history order; an op that never returns (:info, or no completion) has
  a call entry only.  A depth-first search walks the list from its head: at
  a call entry it tries to linearize the op (the model step is legal and the
  resulting (linearized set, state) is not in the cache), and if so records
  it, lifts the call and its return out of the list and restarts from the
  head; otherwise it moves to the next entry.  At a return entry -- an op
  that is not linearized yet -- it is stuck and backtracks to the last
  linearized call (unlifting it) and moves past it.  The history is valid
  when the walk runs off the end of the list (every return passed), invalid
  when it is stuck with nothing to backtrack.

What the analysis reports (the restated result shape; unpinned):

  :op           the return entry of the deepest stuck point (the :ok that
                could not be linearized);
  :previous-ok  the last :ok before it in the sub-history;
  :configs      the frontier there: every (model state, pending ops already
                linearized) the search was stuck at on that return entry.

Independent of the device and of linear_ref's config-set search: it is a
different algorithm (a backtracking walk over a linked entry list), so
agreeing with it on verdicts, failing ops and frontiers is evidence, not a
restatement of the same code.  A key whose search caches more than `budget`
pairs is "unknown" (cause "budget").  The representation limits of the packed
form apply as in linear_ref, before the search: a key whose :invoke needs
window slot >= 112 (lowest free at invoke, freed at :ok) is "unknown"
("window"), one with more than 32767 register values "unknown" ("states").
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, List, Optional, Sequence, Set, Tuple

import linear_ref as L

DEFAULT_BUDGET = 1 << 20


@dataclass
class WglAnalysis:
    valid: Any                               # True / False / "unknown"
    cause: str = "none"
    op_id: Optional[int] = None
    fail_pos: Optional[int] = None           # position of the stuck return in the sub-history
    previous_ok_pos: Optional[int] = None
    frontier: Set[Tuple[Any, frozenset]] = field(default_factory=set)  # (state, linearized pending op ids)
    ops: List[L.Op] = field(default_factory=list)
    cache_size: int = 0


def analysis(history: Sequence[dict], budget: int = DEFAULT_BUDGET, model: str = "cas-register",
             initial=None) -> WglAnalysis:
    """knossos.wgl over one key's sub-history."""
    ops, events = L.complete(history, model)
    step, init = L.model_step(model)
    state = init if initial is None else initial
    res = WglAnalysis(valid=True, ops=ops)
    if model == "multi-register":
        if L.reachable_maps(ops, state, L.WIDE_MAX_STATES) > L.WIDE_MAX_STATES:
            res.valid, res.cause = "unknown", "states"
            return res
    elif len(L.register_values(ops)) + 1 > L.WIDE_MAX_STATES:
        res.valid, res.cause = "unknown", "states"
        return res
    free = list(range(128))
    slot_of = {}
    for kind, oid, pos in events:
        if kind == "invoke":
            s = min(free)
            if s >= L.WIDE_MAX_SLOTS:
                res.valid, res.cause = "unknown", "window"
                return res
            free.remove(s)
            slot_of[oid] = s
        else:
            free.append(slot_of[oid])
    # the entry list: ("call" | "ret", op id, position), history order
    E = [("call" if kind == "invoke" else "ret", oid, pos) for kind, oid, pos in events]
    n = len(E)
    END, HEAD = n, n + 1
    nxt = list(range(1, n + 1)) + [END, 0 if n else END]
    prv = [HEAD] + list(range(0, n - 1)) + [n - 1 if n else HEAD, HEAD]
    ret_of = {oid: i for i, (k, oid, _) in enumerate(E) if k == "ret"}

    def unlink(i):
        nxt[prv[i]] = nxt[i]
        prv[nxt[i]] = prv[i]

    def relink(i):
        nxt[prv[i]] = i
        prv[nxt[i]] = i

    def lift(i):
        unlink(i)
        r = ret_of.get(E[i][1])
        if r is not None:
            unlink(r)

    def unlift(i):  # in reverse order of lift
        r = ret_of.get(E[i][1])
        if r is not None:
            relink(r)
        relink(i)

    linearized: frozenset = frozenset()
    cache = set()
    stack: List[Tuple[int, Any, frozenset]] = []
    entry = nxt[HEAD]
    deepest = -1
    while True:
        if entry == END:
            res.cache_size = len(cache)
            return res  # every return passed: linearizable
        kind, oid, pos = E[entry]
        if kind == "call":
            s2 = step(state, ops[oid].f, ops[oid].value)
            if s2 is not L.INCONSISTENT:
                lin2 = linearized | {oid}
                if (lin2, s2) not in cache:
                    cache.add((lin2, s2))
                    if len(cache) > budget:
                        res.valid, res.cause, res.cache_size = "unknown", "budget", len(cache)
                        return res
                    stack.append((entry, state, linearized))
                    state, linearized = s2, lin2
                    lift(entry)
                    entry = nxt[HEAD]
                    continue
            entry = nxt[entry]
            continue
        # a return entry whose op is not linearized: stuck here
        if pos >= deepest:
            if pos > deepest:
                deepest, res.frontier = pos, set()
            pend = frozenset(q for q in linearized
                             if ops[q].invoke_pos < pos and (ops[q].complete_pos is None or ops[q].complete_pos > pos))
            res.frontier.add((state, pend))
        if not stack:
            res.valid, res.cause = False, "nonlin"
            res.fail_pos = deepest
            res.op_id = next(o.id for o in ops if o.complete_pos == deepest)
            oks = [p for k, _, p in E if k == "ret" and p < deepest]
            res.previous_ok_pos = oks[-1] if oks else None
            res.cache_size = len(cache)
            return res
        e0, state, linearized = stack.pop()
        unlift(e0)
        entry = nxt[e0]


def closure(res_linear: L.Analysis, model: str = "cas-register") -> Set[Tuple[Any, frozenset]]:
    """linear_ref's side of the comparison: the closure of the config set
    standing before the failing :ok under the pending ops other than it --
    what the WGL frontier must equal."""
    step, _ = L.model_step(model)
    ops, p = res_linear.ops, res_linear.op_id
    pend = [q for q in res_linear.final_slots if q != p]
    seen = set(res_linear.final_configs)
    todo = list(seen)
    while todo:
        st, lin = todo.pop()
        for q in pend:
            if q in lin:
                continue
            s2 = step(st, ops[q].f, ops[q].value)
            if s2 is L.INCONSISTENT:
                continue
            c = (s2, lin | {q})
            if c not in seen:
                seen.add(c)
                todo.append(c)
    return seen


def check_independent(history: Sequence[dict], budget: int = DEFAULT_BUDGET, model: str = "cas-register"):
    """independent/checker over linearizable {:algorithm :wgl}: per-key analyses
    (a key complete rejects is "unknown", cause "error", as check-safe has it)."""
    out = {}
    for k in L.history_keys(history):
        try:
            out[k] = analysis(L.subhistory(history, k), budget, model=model)
        except L.HistoryError as e:
            a = WglAnalysis(valid="unknown", cause="error")
            a.error = str(e)
            out[k] = a
    return out
