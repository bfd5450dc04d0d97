"""Definitional brute-force linearizability checker -- TEST ORACLE.

Test infrastructure only (see oracle/linear_ref.py's header for who may
import it).  It does not follow any Knossos algorithm: it applies the
definition of linearizability (Herlihy & Wing) directly, so it pins the JIT
restatement in linear_ref.py independently of how that search is organised.

For a key sub-history reduced by knossos.history/complete +
without-failures (linear_ref.complete), the prefix ending at event e is
linearizable iff there is a sequence of ops that
  * contains every op whose :ok is at or before e,
  * may contain any other op invoked before e (it is still pending at e),
  * respects real time: if a's :ok precedes b's :invoke, a comes first,
  * is legal for the model (cas-register, register or mutex) from its
    initial value.
The history is valid iff every prefix ending at an :ok is linearizable; the
reported failure is the first :ok whose prefix is not.  That event is what
knossos.linear reports as :op (its config set empties exactly there).

Exponential: meant for <= ~10 ops per key.
"""

from __future__ import annotations

from functools import lru_cache
from typing import Optional, Sequence

from linear_ref import INCONSISTENT, complete, model_step


def prefix_linearizable(ops, events, e: int, initial=None, step=None) -> bool:
    inv_at = {}
    ok_at = {}
    for i, (kind, oid, _pos) in enumerate(events[: e + 1]):
        if kind == "invoke":
            inv_at[oid] = i
        else:
            ok_at[oid] = i
    cand = sorted(inv_at)                      # ops invoked by e
    required = frozenset(o for o in cand if o in ok_at)
    # must_precede[b] = ops whose :ok is before b's :invoke
    must = {b: frozenset(a for a in cand if a in ok_at and ok_at[a] < inv_at[b]) for b in cand}

    @lru_cache(maxsize=None)
    def search(state_key, done: frozenset) -> bool:
        state = state_key[1]
        if required <= done:
            return True
        for q in cand:
            if q in done or not must[q] <= done:
                continue
            s2 = step(state, ops[q].f, ops[q].value)
            if s2 is INCONSISTENT:
                continue
            if search((s2 is None, s2), done | {q}):
                return True
        return False

    return search((initial is None, initial), frozenset())


def brute_check(history: Sequence[dict], initial=None, model: str = "cas-register"):
    """Returns (valid, fail_event_ordinal or None) over the reduced events."""
    ops, events = complete(history, model)
    step, init = model_step(model)
    if initial is None:
        initial = init
    for e, (kind, _oid, _pos) in enumerate(events):
        if kind == "ok" and not prefix_linearizable(ops, events, e, initial, step):
            return False, e
    return True, None
