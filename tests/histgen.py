"""Random small Jepsen histories for property tests (any interleaving,
crashes, failures, unmatched invocations, nil reads, several keys, nemesis)."""
import random

from lincheck.independent import Tuple


def random_history(seed: int, n_keys=1, max_ops=7, procs=3, values=(0, 1, 2), p_info=0.15,
                   p_fail=0.1, p_open=0.05, p_nemesis=0.05, p_garbage_read=0.3, model="cas-register"):
    """model: which ops to draw -- cas-register (read/write/cas), register
    (read/write) or mutex (acquire/release)."""
    fs = {"cas-register": ["read", "write", "cas"], "register": ["read", "write"],
          "mutex": ["acquire", "release"]}[model]
    rng = random.Random(seed)
    ops = []
    pending = {}   # process -> (key, f, value)
    next_proc = procs
    idle = list(range(procs))
    budget = {k: rng.randint(1, max_ops) for k in range(n_keys)}
    while idle or pending:
        choices = []
        if idle and any(budget.values()):
            choices.append("invoke")
        if pending:
            choices.append("complete")
        if not choices:
            break
        if rng.random() < p_nemesis:
            f = rng.choice(["start", "stop"])
            ops.append({"type": "info", "f": f, "value": None, "process": "nemesis"})
            ops.append({"type": "info", "f": f, "value": None, "process": "nemesis"})
        c = rng.choice(choices)
        if c == "invoke":
            p = idle.pop(rng.randrange(len(idle)))
            k = rng.choice([k for k, b in budget.items() if b > 0])
            budget[k] -= 1
            f = rng.choice(fs)
            v = None if f in ("read", "acquire", "release") else (
                rng.choice(values) if f == "write" else [rng.choice(values), rng.choice(values)])
            ops.append({"type": "invoke", "f": f, "value": Tuple(k, v), "process": p})
            pending[p] = (k, f, v)
        else:
            p = rng.choice(list(pending))
            k, f, v = pending.pop(p)
            r = rng.random()
            if r < p_open:          # never completes
                continue
            if r < p_open + p_info:
                ops.append({"type": "info", "f": f, "value": Tuple(k, v), "process": p})
                np_ = next_proc; next_proc += 1
                idle.append(np_)
                continue
            if r < p_open + p_info + p_fail:
                ops.append({"type": "fail", "f": f, "value": Tuple(k, v), "process": p})
                idle.append(p)
                continue
            if f == "read":
                v = rng.choice(list(values) + [None]) if rng.random() < p_garbage_read else rng.choice(list(values))
            ops.append({"type": "ok", "f": f, "value": Tuple(k, v), "process": p})
            idle.append(p)
    for i, op in enumerate(ops):
        op["index"] = i
    return ops


def mutex_history(seed: int, n_keys=100, rounds=40, procs=6, width=2.0, corrupt=0.2):
    """(model/mutex) histories that are linearizable by construction: each
    round one process acquires at lock-free time t and releases at t + hold;
    every op's interval contains its linearization point (width sets how far
    intervals spread, hence how many ops are pending at once).  A corrupted
    key loses one release, so a later acquire finds the lock held."""
    rng = random.Random(seed)
    rows = []
    for k in range(n_keys):
        t = 0.0
        busy_until = {p: -1e9 for p in range(procs)}
        drop = rng.randrange(1, rounds) if rng.random() < corrupt else -1
        for r in range(rounds):
            free = [p for p in range(procs) if busy_until[p] < t - width]
            p = rng.choice(free) if free else min(busy_until, key=busy_until.get)
            hold = rng.uniform(0.5, 2.0)
            a_lin, r_lin = t, t + hold
            a_inv = max(a_lin - rng.uniform(0, width), busy_until[p] + 1e-3)
            a_ok = a_lin + rng.uniform(0, min(width, hold) * 0.9)
            r_inv = max(r_lin - rng.uniform(0, width), a_ok + 1e-3)
            r_ok = r_lin + rng.uniform(0, width)
            rows.append((a_inv, "invoke", "acquire", k, p))
            rows.append((a_ok, "ok", "acquire", k, p))
            if r != drop:
                rows.append((r_inv, "invoke", "release", k, p))
                rows.append((r_ok, "ok", "release", k, p))
                busy_until[p] = r_ok
            else:
                busy_until[p] = a_ok
            t = r_lin + rng.uniform(0.01, 0.5)
    rows.sort(key=lambda x: x[0])
    ops = [{"type": ty, "f": f, "value": Tuple(k, None), "process": 100 * k + p} for _t, ty, f, k, p in rows]
    for i, op in enumerate(ops):
        op["index"] = i
    return ops
