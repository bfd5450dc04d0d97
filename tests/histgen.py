"""Random small Jepsen histories for property tests (any interleaving,
crashes, failures, unmatched invocations, nil reads, several keys, nemesis)."""
import random

from lincheck.independent import Tuple


def random_history(seed: int, n_keys=1, max_ops=7, procs=3, values=(0, 1, 2), p_info=0.15,
                   p_fail=0.1, p_open=0.05, p_nemesis=0.05, p_garbage_read=0.3, model="cas-register"):
    """model: which ops to draw -- cas-register (read/write/cas), register
    (read/write), mutex (acquire/release) or multi-register (:txn of 1-3
    micro-ops over registers "x" / "y"; reads complete with random values)."""
    fs = {"cas-register": ["read", "write", "cas"], "register": ["read", "write"],
          "mutex": ["acquire", "release"], "multi-register": ["txn"]}[model]
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
            if f == "txn":
                v = [[rng.choice(["read", "write"]), rng.choice(["x", "y"]), None] for _ in range(rng.randint(1, 3))]
                for m in v:
                    if m[0] == "write":
                        m[2] = rng.choice(values)
            else:
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
            elif f == "txn":
                v = [[m[0], m[1], (rng.choice(list(values) + [None]) if m[0] == "read" else m[2])] for m in v]
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


def multi_register_history(seed: int, n_keys=50, n_ops=60, procs=5, regs=("x", "y", "z"), values=(0, 1, 2, 3),
                           width=2.0, corrupt=0.2, p_info=0.0, init=None):
    """(model/multi-register) histories linearizable by construction: each op
    is a :txn of 1-3 micro-ops with a linearization point inside its
    interval, applied there to a ground-truth map; reads complete with what
    they saw (the invocation carries nil reads).  A corrupted key has one
    read return a value the register did not hold.  p_info: a crashed op
    (:info, its effect applied with probability 1/2, the process retired)."""
    rng = random.Random(seed)
    rows = []
    for k in range(n_keys):
        points = sorted(rng.uniform(0, n_ops * 1.0) for _ in range(n_ops))
        truth = dict(init or {})
        bad = rng.randrange(n_ops) if rng.random() < corrupt else -1
        free_at = {p: -1e9 for p in range(procs)}
        next_p = procs
        for i, t in enumerate(points):
            txn = [[rng.choice(["read", "write"]), rng.choice(regs), None] for _ in range(rng.randint(1, 3))]
            cands = [p for p in free_at if free_at[p] < t]
            p = rng.choice(cands) if cands else None
            if p is None:
                p = next_p; next_p += 1
            inv = max(t - rng.uniform(0, width), free_at.get(p, -1e9) + 1e-3)
            done = t + rng.uniform(0, width)
            crashed = rng.random() < p_info
            apply = not crashed or rng.random() < 0.5
            seen = dict(truth)
            out = []
            for m in txn:
                if m[0] == "write":
                    m[2] = rng.choice(values)
                    seen[m[1]] = m[2]
                    out.append(list(m))
                else:
                    out.append([m[0], m[1], seen.get(m[1])])
            if i == bad and any(m[0] == "read" for m in out):
                j = next(j for j, m in enumerate(out) if m[0] == "read")
                out[j][2] = rng.choice([v for v in values if v != out[j][2]])
            if apply:
                truth = seen
            rows.append((inv, "invoke", k, p, [list(m) for m in txn]))
            rows.append((done, "info" if crashed else "ok", k, p, [list(m) for m in txn] if crashed else out))
            if crashed:
                free_at[p] = float("inf")  # a crashed process is retired
            else:
                free_at[p] = done
    rows.sort(key=lambda x: x[0])
    ops = [{"type": ty, "f": "txn", "value": Tuple(k, v), "process": 1000 * k + p} for _t, ty, k, p, v in rows]
    for i, op in enumerate(ops):
        op["index"] = i
    return ops
