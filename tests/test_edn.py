"""history.edn ingestion: round trips and Jepsen's
line format with fields and values this workload never reads."""
import ctypes as C

import numpy as np
import pytest

from lincheck import _native as N
from lincheck import history as H
from lincheck.checker import Packed

JEPSEN_LINES = """\
{:type :invoke, :f :write, :value [0 3], :process 0, :time 21304010, :index 0}
{:type :info, :f :start, :value nil, :process :nemesis, :time 22000000, :index 1}
{:type :info, :f :start, :value [:isolated {"n1" #{"n2" "n3"}, "n2" #{"n1"}}], :process :nemesis, :time 22000100, :index 2}
{:type :ok, :f :write, :value [0 3], :process 0, :time 23000000, :index 3}
{:type :invoke, :f :cas, :value [0 [3 1]], :process 1, :time 24000000, :index 4}
{:type :info, :f :cas, :value [0 [3 1]], :process 1, :time 29000000, :error :timeout, :index 5}
; a comment line
{:type :invoke, :f :read, :value [0 nil], :process 0, :time 30000000, :index 6}
{:type :ok, :f :read, :value [0 1], :process 0, :time 31000000, :index 7}
{:type :invoke, :f :read, :value [1 nil], :process 11, :time 32000000, :index 8}
{:type :fail, :f :read, :value [1 nil], :process 11, :time 33000000, :error [:not-found "Key not found"], :index 9}
"""


def test_parse_jepsen_lines():
    h = H.parse_edn(JEPSEN_LINES)
    assert len(h) == 10
    assert list(h.type) == [0, 3, 3, 1, 0, 3, 0, 1, 0, 2]
    assert list(h.key[[0, 3, 4, 6, 8]]) == [0, 0, 0, 0, 1]
    assert h.key[1] == N.LC_NO_KEY and h.process[1] == N.LC_NO_PROCESS
    assert (h.v0[4], h.v1[4]) == (3, 1)
    assert h.v0[6] == N.LC_NIL and h.v0[7] == 1
    assert list(h.index) == list(range(10))
    pk = Packed(h)
    assert pk.keys == [0, 1]


def test_vector_form():
    h = H.parse_edn("[" + JEPSEN_LINES.replace("\n; a comment line", "") + "]")
    assert len(h) == 10


@pytest.mark.parametrize("interleave", [True, False])
def test_round_trip(tmp_path, interleave):
    h = H.synth(n_keys=5, ops_per_key=60, concurrency=6, info_rate=0.05, interleave=interleave,
                nemesis_period=2.0 if interleave else 0.0, seed=3)
    path = str(tmp_path / "history.edn")
    H.write_edn(path, h)
    g = H.read_edn(path)
    for col in ("type", "f", "process", "key", "v0", "v1", "index"):
        np.testing.assert_array_equal(getattr(g, col), getattr(h, col), err_msg=col)


@pytest.mark.parametrize("text", ["{:type :invoke", "{:type :wat}", "[{:type :ok} 3]", "{:f :read}"])
def test_parse_errors(text):
    with pytest.raises(N.LincheckError):
        H.parse_edn(text)


def test_missing_file():
    with pytest.raises(N.LincheckError, match="io"):
        H.read_edn("/nonexistent/history.edn")


def _parse_with_threads(text: str, threads: int):
    import os
    old = os.environ.get("LC_EDN_THREADS")
    os.environ["LC_EDN_THREADS"] = str(threads)
    try:
        return H.parse_edn(text)
    finally:
        if old is None:
            del os.environ["LC_EDN_THREADS"]
        else:
            os.environ["LC_EDN_THREADS"] = old


COLS = ("type", "f", "process", "key", "v0", "v1", "index")


def test_parallel_parse_matches_serial(tmp_path):
    """Texts over 2 MB are split at line starts and parsed on several threads;
    the rows must be the serial reader's, in order."""
    h = H.synth(n_keys=60, ops_per_key=400, concurrency=10, info_rate=0.01, interleave=True,
                nemesis_period=3.0, seed=9)
    path = str(tmp_path / "history.edn")
    H.write_edn(path, h)
    text = open(path).read()
    assert len(text) > 2 << 20
    a, b = _parse_with_threads(text, 1), _parse_with_threads(text, 8)
    for col in COLS:
        np.testing.assert_array_equal(getattr(a, col), getattr(b, col), err_msg=col)
        np.testing.assert_array_equal(getattr(b, col), getattr(h, col), err_msg=col)


def test_parallel_parse_multiline_strings_fall_back(tmp_path):
    """Op maps whose :error strings span lines that start with '{': a split
    inside one fails its chunk and the text is re-read serially."""
    h = H.synth(n_keys=40, ops_per_key=400, concurrency=10, seed=10)
    path = str(tmp_path / "history.edn")
    H.write_edn(path, h)
    lines = open(path).read().splitlines()
    lines = [ln[:-1] + ', :error "boom\n{:type :ok, :f :read}\n"}' if i % 3 == 0 else ln
             for i, ln in enumerate(lines)]
    text = "\n".join(lines) + "\n"
    assert len(text) > 2 << 20
    a, b = _parse_with_threads(text, 1), _parse_with_threads(text, 8)
    for col in COLS:
        np.testing.assert_array_equal(getattr(a, col), getattr(b, col), err_msg=col)
        np.testing.assert_array_equal(getattr(b, col), getattr(h, col), err_msg=col)


def test_non_independent_values():
    """Plain (non-tuple) values: the reader takes them as they are."""
    text = ("{:type :invoke, :f :write, :value 3, :process 0, :index 0}\n"
            "{:type :ok, :f :write, :value 3, :process 0, :index 1}\n"
            "{:type :invoke, :f :cas, :value [3 4], :process 1, :index 2}\n")
    h = H.parse_edn(text)
    assert list(h.key) == [N.LC_NO_KEY] * 3
    assert (h.v0[2], h.v1[2]) == (3, 4) and h.v0[0] == 3


def _edn(x):
    """EDN text of a Python value from histgen's op maps (strings as keywords)."""
    if x is None:
        return "nil"
    if isinstance(x, str):
        return ":" + x
    if isinstance(x, (list, tuple)):
        return "[" + " ".join(_edn(y) for y in x) + "]"
    return str(int(x))


def _txn_lines(ops):
    out = []
    for o in ops:
        proc = ":nemesis" if o.get("process") is None or isinstance(o.get("process"), str) else str(o["process"])
        out.append("{:type :%s, :f :%s, :value %s, :process %s, :time 1, :index %d}" % (
            o["type"], o["f"], _edn(o.get("value")), proc, o["index"]))
    return "\n".join(out) + "\n"


@pytest.mark.parametrize("seed", [1, 2])
def test_txn_histories(seed):
    """(model/multi-register) :txn ops in history.edn: [k txn] tuples of
    [:read|:write register value] micro-ops, registers as keywords, read back
    with the same rows, micro-ops and register ids as History.from_ops gives
    the op maps (names in order of first appearance)."""
    from histgen import multi_register_history
    ops = multi_register_history(seed, n_keys=6, n_ops=40, corrupt=0.3, p_info=0.05)
    for i, o in enumerate(ops):
        o["index"] = i
    ref = H.History.from_ops(ops)
    g = H.parse_edn(_txn_lines(ops))
    for col in ("type", "f", "process", "key", "v0", "v1", "index", "mop_off", "mop"):
        np.testing.assert_array_equal(getattr(g, col), getattr(ref, col), err_msg=col)
    assert {k: v.lstrip(":") for k, v in g.reg_names.items()} == ref.reg_names
    from lincheck import model
    assert Packed(g, model.multi_register()).keys == Packed(ref, model.multi_register()).keys


def test_txn_forms_and_round_trip(tmp_path):
    text = ("{:type :invoke, :f :txn, :value [[:r :x nil] [:w 7 2]], :process 0, :index 0}\n"
            "{:type :ok, :f :txn, :value [[:read :x 1] [:write 7 2]], :process 0, :index 1}\n"
            "{:type :invoke, :f :txn, :value nil, :process 1, :index 2}\n"
            "{:type :fail, :f :txn, :value [[:write \"y\" 3]], :process 1, :index 3}\n")
    h = H.parse_edn(text)
    base = H.NAMED_REG_BASE
    assert list(h.f) == [N.LC_F_TXN] * 4 and (h.key == N.LC_NO_KEY).all()
    assert list(h.mop_off) == [0, 2, 4, 4, 5]
    assert h.mop.reshape(-1, 3).tolist() == [[0, base, N.LC_NIL], [1, 7, 2], [0, base, 1], [1, 7, 2],
                                             [1, base + 1, 3]]
    assert h.reg_names == {base: ":x", base + 1: '"y"'}
    path = str(tmp_path / "history.edn")
    H.write_edn(path, h)
    g = H.read_edn(path)
    for col in ("type", "f", "process", "key", "v0", "v1", "index", "mop_off", "mop"):
        np.testing.assert_array_equal(getattr(g, col), getattr(h, col), err_msg=col)
    assert g.reg_names == {base: ":x", base + 1: '"y"'}  # names written back verbatim
    assert ":x" in open(path).read() and '"y"' in open(path).read()
    # without names (lc_edn_write on a bare view) they become :r<i>
    N.check(N.lib().lc_edn_write(path.encode(), C.byref(h.as_c())))
    assert H.read_edn(path).reg_names == {base: ":r0", base + 1: ":r1"}
    # a name that is not one EDN token falls back to :r<i> too
    arr = (C.c_char_p * 2)(b":x", b"bad name")
    N.check(N.lib().lc_edn_write_named(path.encode(), C.byref(h.as_c()), arr, 2))
    assert H.read_edn(path).reg_names == {base: ":x", base + 1: ":r1"}


@pytest.mark.parametrize("value", ["[[:cas :x 1]]", "[[:read :x]]", "[[:read :x 1 2]]", "[:read :x 1]",
                                   "[[:read nil 1]]", "[[:read :x :y]]", "7"])
def test_txn_errors(value):
    with pytest.raises(N.LincheckError, match="txn"):
        H.parse_edn("{:type :invoke, :f :txn, :value %s, :process 0, :index 0}\n" % value)
