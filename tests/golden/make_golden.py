"""Writes tests/golden/kat.json: hand-derived known-answer histories for the
cas-register linearizability check.

The reference ships no fixtures for this path (test/jepsen/etcdemo_test.clj
is `(is (= 0 1))`, store/latest dangles), so every expectation below was
derived by hand from the cas-register model (knossos.model/cas-register,
etcdemo.clj:117) and the definition of linearizability, and is re-checked
against oracle/brute.py when this script runs.

Histories use the demo's op shapes (etcdemo.clj:67-69, :83-105): reads
invoke with nil and complete with the value read, writes carry a value,
cas carries [old new]; client timeouts are :info for write/cas; the nemesis
emits :info :start/:stop from :process :nemesis (etcdemo.clj:138-143).
Values are wrapped as independent tuples [k v] (etcdemo.clj:90, :120).

Expectation per key: valid? and, for invalid keys, the :index of the :ok op
knossos reports as :op and of the :ok before it (:previous-ok).

Run: python tests/golden/make_golden.py
"""

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))


def T(k, v):
    return {"tuple": [k, v]}


class H:
    """Tiny history builder: ops get sequential :index values."""

    def __init__(self):
        self.ops = []

    def add(self, type_, f, value, process):
        self.ops.append({"type": type_, "f": f, "value": value, "process": process, "index": len(self.ops)})
        return len(self.ops) - 1

    def inv(self, p, f, v=None, k=0):
        return self.add("invoke", f, T(k, v), p)

    def ok(self, p, f, v=None, k=0):
        return self.add("ok", f, T(k, v), p)

    def fail(self, p, f, v=None, k=0):
        return self.add("fail", f, T(k, v), p)

    def info(self, p, f, v=None, k=0):
        return self.add("info", f, T(k, v), p)

    def nemesis(self, f):
        self.add("info", f, None, "nemesis")
        return self.add("info", f, None, "nemesis")

    def seq(self, p, f, v_inv, v_ok, k=0):
        self.inv(p, f, v_inv, k)
        return self.ok(p, f, v_ok, k)


def kats():
    out = []

    def case(name, h, expect, note, model="cas-register"):
        out.append({"name": name, "note": note, "history": h.ops, "expect": expect, "model": model})

    # 1: the tutorial's stale read -- "can't read 1 from register 3"
    h = H(); h.seq(0, "write", 1, 1); prev = h.seq(1, "write", 3, 3); bad = h.seq(2, "read", None, 1)
    case("stale-read", h, {"0": {"valid?": False, "op": bad, "previous-ok": prev}},
         "read of 1 starts after write 3 completed")
    # 2: read concurrent with a write may see it
    h = H(); h.inv(0, "write", 1); h.inv(1, "read"); h.ok(1, "read", 1); h.ok(0, "write", 1)
    case("concurrent-read-sees-write", h, {"0": {"valid?": True}}, "")
    # 3: read concurrent with a write may also miss it (sees nil)
    h = H(); h.inv(0, "write", 1); h.inv(1, "read"); h.ok(1, "read", None); h.ok(0, "write", 1)
    case("concurrent-read-misses-write", h, {"0": {"valid?": True}}, "")
    # 4: knossos quirk: an :ok read of nil is legal in every state
    h = H(); h.seq(0, "write", 2, 2); h.seq(1, "read", None, None)
    case("nil-read-any-state", h, {"0": {"valid?": True}}, "cas-register read nil is always legal")
    # 5: lost cas: cas 0->4 succeeded, later read sees 0
    h = H(); h.seq(0, "write", 0, 0); prev = h.seq(1, "cas", [0, 4], [0, 4]); bad = h.seq(2, "read", None, 0)
    case("lost-cas", h, {"0": {"valid?": False, "op": bad, "previous-ok": prev}}, "")
    # 6: a :fail cas is dropped (without-failures), even one that 'could' succeed
    h = H(); h.seq(0, "write", 0, 0); h.inv(1, "cas", [0, 2]); h.fail(1, "cas", [0, 2]); h.seq(2, "read", None, 0)
    case("failed-cas-dropped", h, {"0": {"valid?": True}}, "")
    # 7: a cas that reports :ok although the register held something else
    h = H(); h.seq(0, "write", 1, 1); bad = h.seq(1, "cas", [3, 4], [3, 4])
    case("impossible-cas", h, {"0": {"valid?": False, "op": bad, "previous-ok": 1}}, "can't CAS 1 from 3 to 4")
    # 8: crashed write takes effect late
    h = H(); h.seq(0, "write", 1, 1); h.inv(1, "write", 2); h.info(1, "write", 2)
    h.seq(2, "read", None, 1); h.seq(3, "read", None, 2)
    case("crashed-write-late", h, {"0": {"valid?": True}}, ":info op stays callable forever")
    # 9: crashed write never takes effect
    h = H(); h.seq(0, "write", 1, 1); h.inv(1, "write", 2); h.info(1, "write", 2)
    h.seq(2, "read", None, 1); h.seq(3, "read", None, 1)
    case("crashed-write-never", h, {"0": {"valid?": True}}, "")
    # 10: once the crashed write is visible the register cannot go back
    h = H(); h.seq(0, "write", 1, 1); h.inv(1, "write", 2); h.info(1, "write", 2)
    prev = h.seq(2, "read", None, 2); bad = h.seq(3, "read", None, 1)
    case("crashed-write-no-going-back", h, {"0": {"valid?": False, "op": bad, "previous-ok": prev}}, "")
    # 11: nemesis ops are in every sub-history and change nothing
    h = H(); h.nemesis("start"); h.seq(0, "write", 4, 4); h.nemesis("stop"); h.seq(1, "read", None, 4)
    case("nemesis-ignored", h, {"0": {"valid?": True}}, "")
    # 12: two independent keys, one bad
    h = H(); h.seq(0, "write", 1, 1, k=0); h.seq(1, "write", 1, 1, k=1); h.seq(2, "write", 3, 3, k=1)
    h.seq(3, "read", None, 1, k=0); bad = h.seq(4, "read", None, 1, k=1)
    case("two-keys-one-bad", h, {"0": {"valid?": True}, "1": {"valid?": False, "op": bad, "previous-ok": 5}},
         "failures = [1]")
    # 13: invocation with no completion at all is pending forever
    h = H(); h.inv(0, "write", 3); h.seq(1, "read", None, 3); h.seq(2, "read", None, 3)
    case("unmatched-invoke", h, {"0": {"valid?": True}}, "")
    # 14: cas from nil (= nil nil) on the initial register
    h = H(); h.seq(0, "cas", [None, 3], [None, 3]); h.seq(1, "read", None, 3)
    case("cas-from-nil", h, {"0": {"valid?": True}}, "")
    # 15: two concurrent writes, reads pin the order; the third read contradicts
    h = H(); h.inv(0, "write", 1); h.inv(1, "write", 2); h.ok(0, "write", 1); h.ok(1, "write", 2)
    h.seq(2, "read", None, 1); prev = h.seq(3, "read", None, 1); bad = h.seq(4, "read", None, 2)
    case("concurrent-writes-order", h, {"0": {"valid?": False, "op": bad, "previous-ok": prev}},
         "reads fix write 2 before write 1, so 2 cannot reappear")
    # 16: cas chain under concurrency, valid
    h = H(); h.seq(0, "write", 0, 0); h.inv(1, "cas", [0, 1]); h.inv(2, "cas", [1, 2]); h.ok(2, "cas", [1, 2])
    h.ok(1, "cas", [0, 1]); h.seq(3, "read", None, 2)
    case("concurrent-cas-chain", h, {"0": {"valid?": True}}, "cas 0->1 linearized before cas 1->2")
    # 17: crashed read (timeouts make reads :fail in the demo, but :info is legal input)
    h = H(); h.seq(0, "write", 4, 4); h.inv(1, "read"); h.info(1, "read"); h.seq(2, "read", None, 4)
    case("crashed-read", h, {"0": {"valid?": True}}, "")
    # 18: a read of a value nobody wrote
    h = H(); h.seq(0, "write", 1, 1); bad = h.seq(1, "read", None, 7)
    case("read-unwritten-value", h, {"0": {"valid?": False, "op": bad, "previous-ok": 1}}, "")
    # 19: empty key sub-history other than failed ops
    h = H(); h.inv(0, "write", 1); h.fail(0, "write", 1)
    case("only-failed-ops", h, {"0": {"valid?": True}}, "")
    # 20: a process crashes and its successor (p + concurrency) carries on
    h = H(); h.inv(0, "cas", [None, 1]); h.info(0, "cas", [None, 1]); prev = h.seq(10, "write", 3, 3)
    bad = h.seq(1, "read", None, 1)
    case("crashed-cas-cannot-land", h, {"0": {"valid?": False, "op": bad, "previous-ok": prev}},
         "crashed cas nil->1 needs nil, so it cannot land after write 3 and is overwritten before it")
    # --- other Knossos models: (model/mutex), (model/register)
    # 21: acquire / release in turn
    h = H(); h.seq(0, "acquire", None, None); h.seq(0, "release", None, None)
    h.seq(1, "acquire", None, None); h.seq(1, "release", None, None)
    case("mutex-in-turn", h, {"0": {"valid?": True}}, "", model="mutex")
    # 22: a second acquire completes while the lock is held
    h = H(); prev = h.seq(0, "acquire", None, None); bad = h.seq(1, "acquire", None, None)
    case("mutex-double-acquire", h, {"0": {"valid?": False, "op": bad, "previous-ok": prev}}, "already held",
         model="mutex")
    # 23: two overlapping acquires both complete, nobody releases
    h = H(); h.inv(0, "acquire"); h.inv(1, "acquire"); prev = h.ok(0, "acquire"); bad = h.ok(1, "acquire")
    case("mutex-concurrent-acquires", h, {"0": {"valid?": False, "op": bad, "previous-ok": prev}},
         "whichever goes first, the other finds the lock held", model="mutex")
    # 24: release of a lock nobody holds
    h = H(); h.seq(0, "acquire", None, None); prev = h.seq(0, "release", None, None)
    bad = h.seq(1, "release", None, None)
    case("mutex-release-unheld", h, {"0": {"valid?": False, "op": bad, "previous-ok": prev}}, "not held",
         model="mutex")
    # 25: a crashed release may have taken effect
    h = H(); h.seq(0, "acquire", None, None); h.inv(0, "release"); h.info(0, "release")
    h.seq(1, "acquire", None, None)
    case("mutex-crashed-release", h, {"0": {"valid?": True}}, ":info release stays callable", model="mutex")
    # 26: a failed acquire is dropped
    h = H(); h.seq(0, "acquire", None, None); h.inv(1, "acquire"); h.fail(1, "acquire")
    h.seq(0, "release", None, None)
    case("mutex-failed-acquire-dropped", h, {"0": {"valid?": True}}, "", model="mutex")
    # 27: the register model: the tutorial's stale read
    h = H(); h.seq(0, "write", 1, 1); prev = h.seq(1, "write", 3, 3); bad = h.seq(2, "read", None, 1)
    case("register-stale-read", h, {"0": {"valid?": False, "op": bad, "previous-ok": prev}}, "3 vs 1",
         model="register")
    # 28: the register model, concurrent write and read
    h = H(); h.inv(0, "write", 1); h.inv(1, "read"); h.ok(1, "read", 1); h.ok(0, "write", 1)
    h.seq(2, "read", None, None)
    case("register-concurrent", h, {"0": {"valid?": True}}, "", model="register")
    # --- per-key error isolation (independent/checker's check-safe per key,
    # etcdemo.clj:115): a key knossos cannot analyse is :unknown with :error,
    # the others are checked as usual
    # 29: a completion with no invocation (complete's assertion) in key 2
    h = H(); h.seq(0, "write", 1, 1, k=0); h.seq(1, "read", None, 1, k=0)
    h.seq(2, "write", 1, 1, k=1); prev = h.seq(3, "write", 3, 3, k=1); bad = h.seq(4, "read", None, 1, k=1)
    h.ok(5, "write", 2, k=2); h.seq(6, "read", None, None, k=2)
    case("malformed-key-isolated", h,
         {"0": {"valid?": True}, "1": {"valid?": False, "op": bad, "previous-ok": prev},
          "2": {"valid?": "unknown", "error": True}},
         "key 2 completes an op it never invoked: :unknown there, key 1 still fails")
    # 30: an op the model cannot step in key 1
    h = H(); h.seq(0, "write", 2, 2, k=0); h.seq(1, "read", None, 2, k=0)
    h.seq(2, "add", 5, 5, k=1)
    case("unsteppable-op-isolated", h, {"0": {"valid?": True}, "1": {"valid?": "unknown", "error": True}},
         "cas-register cannot step :add")
    # 31: a non-tuple client op is in every key's sub-history and stepped there
    h = H(); h.seq(0, "write", 1, 1, k=0); h.seq(1, "write", 1, 1, k=1)
    prev = h.add("invoke", "write", 3, 9); prev = h.add("ok", "write", 3, 9)
    bad = h.seq(2, "read", None, 1, k=0); h.seq(3, "read", None, 3, k=1)
    case("non-tuple-op-in-every-key", h,
         {"0": {"valid?": False, "op": bad, "previous-ok": prev}, "1": {"valid?": True}},
         "the un-keyed write 3 lands in both keys: key 0's later read of 1 is stale")
    return out


def to_oracle_ops(ops):
    from linear_ref import subhistory  # noqa: F401 (import check)

    class Tup(tuple):
        _lc_tuple = True

    res = []
    for op in ops:
        o = dict(op)
        v = op["value"]
        if isinstance(v, dict) and "tuple" in v:
            k, x = v["tuple"]
            o["value"] = Tup((k, x))
        res.append(o)
    return res


def main():
    import brute
    import linear_ref as LR
    cases = kats()
    for c in cases:
        ops = to_oracle_ops(c["history"])
        keys = LR.history_keys(ops)
        for k in keys:
            sub = LR.subhistory(ops, k)
            exp = c["expect"][str(k)]
            if exp["valid?"] == "unknown":  # check-safe: the analysis throws
                a = LR.analysis_safe(sub, model=c["model"])
                assert a.valid == "unknown" and a.cause == "error", (c["name"], k)
                continue
            ok, fe = brute.brute_check(sub, model=c["model"])
            a = LR.analysis(sub, model=c["model"])
            assert ok == exp["valid?"], (c["name"], k, ok)
            assert a.valid == exp["valid?"], (c["name"], k, a.valid)
            if not ok:
                _ops, events = LR.complete(sub, c["model"])
                assert fe == a.fail_event, (c["name"], fe, a.fail_event)
                assert sub[events[fe][2]]["index"] == exp["op"], (c["name"], sub[events[fe][2]]["index"], exp["op"])
                assert sub[a.previous_ok_pos]["index"] == exp["previous-ok"], c["name"]
    path = os.path.join(HERE, "kat.json")
    with open(path, "w") as f:
        json.dump(cases, f, indent=1)
    print(f"wrote {len(cases)} cases to {path}")


if __name__ == "__main__":
    main()
