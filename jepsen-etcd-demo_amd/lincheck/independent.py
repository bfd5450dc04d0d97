"""Mirror of jepsen.independent for this path (etcdemo.clj:12, :115, :120).

`tuple(k, v)` marks an op value as belonging to independent key k (a
clojure.lang.MapEntry upstream, so it is never confused with a cas [old new]
vector).  `checker(inner)` is independent/checker: it splits the history by
key, runs `inner` on every key's sub-history and merges the results as
{"valid?": merge_valid(...), "results": {k: r}, "failures": [k ...]}.

When `inner` is (a compose of) lincheck.checker.linearizable, the whole
history goes to the device in ONE batched call (lc_pack + lc_check_batch)
instead of one search per key: that is the drop-in this repository exists for.
"""

from __future__ import annotations

from typing import Any, Dict, List, Sequence


class Tuple(tuple):
    """jepsen.independent/tuple -- a [k v] pair that marks a keyed op value."""
    _lc_tuple = True

    def __new__(cls, k, v):
        return super().__new__(cls, (k, v))

    @property
    def key(self):
        return self[0]

    @property
    def value(self):
        return self[1]

    def __repr__(self):
        return f"tuple({self[0]!r}, {self[1]!r})"


def tuple_(k, v) -> Tuple:  # `tuple` shadows the builtin; both names exported
    return Tuple(k, v)


globals()["tuple"] = tuple_


def is_tuple(v) -> bool:
    return bool(getattr(v, "_lc_tuple", False))


def history_keys(history: Sequence[dict]) -> List[Any]:
    """independent/history-keys: tuple keys in order of first appearance."""
    seen, out = set(), []
    for op in history:
        v = op.get("value")
        if is_tuple(v) and v[0] not in seen:
            seen.add(v[0])
            out.append(v[0])
    return out


def subhistory(history: Sequence[dict], k) -> List[dict]:
    """independent/subhistory: key k's ops (values unwrapped) + non-tuple ops."""
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


class IndependentChecker:
    def __init__(self, inner):
        self.inner = inner

    def check(self, test: Dict, history, opts: Dict | None = None) -> Dict:
        from . import checker as ck
        opts = dict(opts or {})
        batched = ck.batched_linearizable(self.inner)
        if batched is not None:
            return batched.check_independent(test, history, opts, self.inner)
        results = {}
        for k in history_keys(history):
            o = dict(opts)
            o["subdirectory"] = ["independent", str(k)]
            o["history-key"] = k
            results[k] = ck.check_safe(self.inner, test, subhistory(history, k), o)
        return merge_results(results)


def merge_results(results: Dict[Any, Dict]) -> Dict:
    from .checker import merge_valid
    failures = [k for k, r in results.items() if r.get("valid?") is False]
    return {"valid?": merge_valid([r.get("valid?") for r in results.values()]),
            "results": results,
            "failures": failures}


def checker(inner) -> IndependentChecker:
    """independent/checker (etcdemo.clj:115)."""
    return IndependentChecker(inner)
