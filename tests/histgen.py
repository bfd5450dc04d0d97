"""Random small Jepsen histories for property tests (any interleaving,
crashes, failures, unmatched invocations, nil reads, several keys, nemesis)."""
import random

from lincheck.independent import Tuple


def random_history(seed: int, n_keys=1, max_ops=7, procs=3, values=(0, 1, 2), p_info=0.15,
                   p_fail=0.1, p_open=0.05, p_nemesis=0.05, p_garbage_read=0.3):
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
            f = rng.choice(["read", "write", "cas"])
            v = None if f == "read" else (rng.choice(values) if f == "write" else [rng.choice(values), rng.choice(values)])
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
