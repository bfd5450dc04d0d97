"""Static checks on kernel source shapes that once hung a wave on the GPU.

Round 3: a `for (;;) ... break` walk loop in k_spec (device_lattice.hip) was
compiled into an exec-masked loop whose exit hung the wave after its first
walk; it was replaced by fixed trip counts over uni()-uniform queue indices.
No run-time test can see a future edit that undoes that (the hang only
shows on the GPU), so the loop shapes are checked here, in the source."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "jepsen-etcd-demo_amd", "csrc")


def _body(src: str, head: str) -> str:
    """The brace-balanced body of the first definition starting with head."""
    i = src.index(head)
    j = src.index("{", i)
    depth = 0
    for k in range(j, len(src)):
        depth += {"{": 1, "}": -1}.get(src[k], 0)
        if depth == 0:
            return src[j:k + 1]
    raise AssertionError(f"unbalanced {head}")


def _code(text: str) -> str:
    """text without // comments"""
    return "\n".join(line.split("//")[0] for line in text.splitlines())


def test_spec_queue_loops_keep_fixed_trip_counts():
    src = open(os.path.join(CSRC, "device_lattice.hip")).read()
    head = re.search(r"__global__ __launch_bounds__\(64 \* W[^)]*\)\) void k_spec\(", src)
    assert head, "k_spec's definition not found"
    body = _code(_body(src, head.group(0)))
    assert not re.search(r"for\s*\(\s*;\s*;\s*\)|while\s*\(\s*(true|1)\s*\)", body), "an open loop in k_spec"
    for start, queue in (("0", "s_next[0]"), ("1", "s_next[1]")):
        m = re.search(r"for \(uint32_t k = %s; k < \(uint32_t\)S; \+\+k\) \{(.{0,400})" % start, body, re.S)
        assert m, f"k_spec's queue loop from {start} lost its fixed trip count"
        head = m.group(1)
        assert queue in head and "s = uni(s);" in head, f"queue index of loop {start} not made uniform by uni()"
        assert "SPEC_CHECK_UNIFORM(s);" in head


def test_wgl_work_loop_is_bounded():
    src = _code(open(os.path.join(CSRC, "device_wgl.hip")).read())
    body = _body(src, "__global__ __launch_bounds__(64) void k_wgl(")
    assert not re.search(r"for\s*\(\s*;\s*;\s*\)|while\s*\(\s*(true|1)\s*\)", body)
    assert re.search(r"for \(int32_t guard = 0; guard <= n_work; \+\+guard\)", body)
    assert "w = (int32_t)uni((uint32_t)w);" in body
    key = _body(src, "__device__ bool wgl_key(")
    assert re.search(r"for \(uint64_t it = 0; it < max_it; \+\+it\)", key), "the walk lost its step bound"
