"""test.fressian ingestion ("and later test.fressian").

Parity unpinned: the reference holds no stored run and the image has no JVM
or Fressian library, so the files here come from `FressianOut`, an encoder
written in this test from the published Fressian encoding, independently of
csrc/host_fressian.cpp.  It exercises what a real Jepsen test.fressian
carries around the history -- cached keywords past the 32 packed cache slots,
struct types and struct-cache references for handler-tagged values, chunked
strings, closed and open lists, metadata, sets, doubles, instants, a cache
reset and a footer -- and each file is read back against the same history
through history.edn."""
import struct

import numpy as np
import pytest

from lincheck import _native as N
from lincheck import history as H
from lincheck.checker import Packed

COLS = ("type", "f", "process", "key", "v0", "v1", "index")


class Kw(str):
    pass


class Tagged:
    def __init__(self, tag, *fields):
        self.tag, self.fields = tag, fields


class Open(list):
    """A list written as BEGIN_OPEN_LIST ... (only valid last in a file)."""


class Closed(list):
    """A list written as BEGIN_CLOSED_LIST ... END_COLLECTION."""


class Chunked(str):
    """A string written in STRING_CHUNK pieces."""


class FressianOut:
    def __init__(self):
        self.b = bytearray()
        self.cache = {}
        self.stypes = {}

    def int_(self, v):
        b = self.b
        if -1 <= v <= 63:
            b.append(v & 0xFF)
            return
        for bits, base, nbytes in ((13, 0x50, 1), (20, 0x68, 2), (26, 0x72, 3), (34, 0x76, 4), (42, 0x7A, 5),
                                   (50, 0x7E, 6)):
            if -(1 << (bits - 1)) <= v < (1 << (bits - 1)):
                b.append(base + (v >> (8 * nbytes)))
                b += (v & ((1 << (8 * nbytes)) - 1)).to_bytes(nbytes, "big")
                return
        b.append(0xF8)
        b += struct.pack(">q", v)

    def string(self, s):
        raw = s.encode()
        if isinstance(s, Chunked):
            pieces = [raw[i:i + 3] for i in range(0, len(raw), 3)] or [b""]
            for piece in pieces[:-1]:
                self.b.append(0xE2)
                self.int_(len(piece))
                self.b += piece
            self.b.append(0xE3)
            self.int_(len(pieces[-1]))
            self.b += pieces[-1]
            return
        if len(raw) < 8:
            self.b.append(0xDA + len(raw))
        else:
            self.b.append(0xE3)
            self.int_(len(raw))
        self.b += raw

    def cached(self, s):
        if s in self.cache:
            i = self.cache[s]
            if i < 32:
                self.b.append(0x80 + i)
            else:
                self.b.append(0xCC)
                self.int_(i)
            return
        self.b.append(0xCD)
        self.string(s)
        self.cache[s] = len(self.cache)

    def list_(self, xs):
        if isinstance(xs, Open):
            self.b.append(0xEE)
        elif isinstance(xs, Closed):
            self.b.append(0xED)
        elif len(xs) < 8:
            self.b.append(0xE4 + len(xs))
        else:
            self.b.append(0xEC)
            self.int_(len(xs))
        for x in xs:
            self.obj(x)
        if isinstance(xs, Closed):
            self.b.append(0xFD)

    def obj(self, x):
        b = self.b
        if x is None:
            b.append(0xF7)
        elif x is True or x is False:
            b.append(0xF5 if x else 0xF6)
        elif isinstance(x, Kw):
            b.append(0xCA)
            if "/" in x:
                ns, nm = x.split("/")
                self.cached(ns)
            else:
                nm = x
                b.append(0xF7)
            self.cached(nm)
        elif isinstance(x, str):
            self.string(x)
        elif isinstance(x, int):
            self.int_(x)
        elif isinstance(x, float):
            if x in (0.0, 1.0):
                b.append(0xFB if x == 0.0 else 0xFC)
            else:
                b.append(0xFA)
                b += struct.pack(">d", x)
        elif isinstance(x, dict):
            b.append(0xC0)
            self.list_([y for kv in x.items() for y in kv])
        elif isinstance(x, (set, frozenset)):
            b.append(0xC1)
            self.list_(sorted(x, key=repr))
        elif isinstance(x, Tagged):
            if x.tag in self.stypes:
                i = self.stypes[x.tag]
                if i < 16:
                    b.append(0xA0 + i)
                else:
                    b.append(0xF0)
                    self.int_(i)
            else:
                b.append(0xEF)
                self.string(x.tag)
                self.int_(len(x.fields))
                self.stypes[x.tag] = len(self.stypes)
            for f in x.fields:
                self.obj(f)
        elif isinstance(x, list):
            self.list_(x)
        else:
            raise TypeError(type(x))

    def meta(self, m, x):
        self.b.append(0xF1)
        self.obj(m)
        self.obj(x)

    def inst(self, ms):
        self.b.append(0xC8)
        self.int_(ms)

    def footer(self):
        n = len(self.b)
        self.b += bytes([0xCF, 0xCF, 0xCF, 0xCF]) + struct.pack(">ii", n, 0)


TYPES = ["invoke", "ok", "fail", "info"]
FS = ["read", "write", "cas", None, "acquire", "release"]


def op_maps(h, tuple_style="list", extra=True):
    """Jepsen op maps for history h (the fields lc_edn_write emits, plus :time
    and :error values the reader has to skip)."""
    out = []
    for r in range(len(h)):
        t, f = TYPES[h.type[r]], FS[h.f[r]]
        nil = lambda v: None if v == N.LC_NIL else int(v)
        if f is None:
            fk = "start" if h.v0[r] == 1 else "stop" if h.v0[r] == 0 else "nemesis"
            val = None
        elif f in ("acquire", "release"):
            fk, val = f, None
        elif f == "cas":
            fk = f
            val = None if (h.v0[r] == N.LC_NIL and h.v1[r] == N.LC_NIL and h.type[r] == 0) else [nil(h.v0[r]), nil(h.v1[r])]
        else:
            fk, val = f, nil(h.v0[r])
        if f is not None and h.key[r] != N.LC_NO_KEY:
            k = int(h.key[r])
            val = {"list": [k, val], "entry": Tagged("map-entry", k, val), "vec": Tagged("vec", [k, val])}[tuple_style]
        m = {Kw("type"): Kw(t), Kw("f"): Kw(fk), Kw("value"): val,
             Kw("process"): Kw("nemesis") if h.process[r] == N.LC_NO_PROCESS else int(h.process[r])}
        if extra:
            m[Kw("time")] = 1_000_000_007 * (r + 1)
            if t == "info" and f is not None:
                m[Kw("error")] = [Kw("timeout"), Chunked("request to n3 timed out after 5000 ms")]
        m[Kw("index")] = int(h.index[r])
        out.append(m)
    return out


def jepsen_test_map(h, **kw):
    ops = op_maps(h, **kw)
    return {Kw("name"): "etcd q=false", Kw("nodes"): ["n1", "n2", "n3", "n4", "n5"],
            Kw("concurrency"): 10, Kw("start-time"): Tagged("date-time", "20211027T165458.000Z"),
            Kw("nemesis-opts"): {Kw("interval"): 5.0, Kw("targets"): {"n1", "n2"}, Kw("ratio"): 0.0},
            Kw("jepsen.etcdemo/quorum"): False,
            Kw("history"): ops}


def encode(obj, footer=False):
    w = FressianOut()
    w.obj(obj)
    if footer:
        w.footer()
    return bytes(w.b)


def same(g, h):
    for col in COLS:
        np.testing.assert_array_equal(getattr(g, col), getattr(h, col), err_msg=col)


@pytest.fixture(scope="module")
def c1():
    return H.synth(n_keys=6, ops_per_key=100, concurrency=10, interleave=True, nemesis_period=5.0,
                   info_rate=0.05, seed=1)


@pytest.mark.parametrize("tuple_style", ["list", "entry", "vec"])
def test_jepsen_test_map(c1, tuple_style):
    data = encode(jepsen_test_map(c1, tuple_style=tuple_style), footer=True)
    same(H.parse_fressian(data), c1)


def test_matches_edn(tmp_path, c1):
    H.write_edn(str(tmp_path / "history.edn"), c1)
    (tmp_path / "test.fressian").write_bytes(encode(jepsen_test_map(c1)))
    same(H.read_fressian(str(tmp_path / "test.fressian")), H.read_edn(str(tmp_path / "history.edn")))


def test_history_only_forms(c1):
    ops = op_maps(c1, extra=False)
    same(H.parse_fressian(encode(ops)), c1)              # LIST n
    same(H.parse_fressian(encode(Closed(ops))), c1)      # closed list
    same(H.parse_fressian(encode(Open(ops))), c1)        # open list to the end of the file
    same(H.parse_fressian(encode(Tagged("vec", ops))), c1)  # a vector handler


def test_cache_past_packed_slots_and_reset():
    """Keyword names cached past the 32 packed slots (GET_PRIORITY_CACHE
    references), then a cache reset in front of the history, after which the
    names are put again from index 0; metadata on the test map."""
    h = H.parse_edn("{:type :invoke, :f :write, :value [0 3], :process 0, :index 0}\n"
                    "{:type :ok, :f :write, :value [0 3], :process 0, :index 1}\n"
                    "{:type :invoke, :f :read, :value [0 nil], :process 1, :index 2}\n"
                    "{:type :ok, :f :read, :value [0 3], :process 1, :index 3}\n")
    w = FressianOut()
    w.obj({**{Kw(f"x{i}"): i for i in range(40)}, Kw("history"): op_maps(h)})
    assert 0xCC in w.b  # names at cache index >= 32
    same(H.parse_fressian(bytes(w.b)), h)

    w = FressianOut()
    w.b.append(0xF1)  # META: the annotation, then the test map
    w.obj({Kw("line"): 12})
    w.b.append(0xC0)
    w.b.append(0xED)
    for i in range(3):
        w.obj(Kw(f"y{i}"))
        w.obj(i)
    w.obj(Kw("history"))
    w.b.append(0xFE)  # RESET_CACHES, then the history value
    w.cache = {}
    w.obj(op_maps(h))
    w.b.append(0xFD)
    same(H.parse_fressian(bytes(w.b)), h)


def test_skipped_values():
    """Values the history reader skips: doubles, floats, instants, UUIDs,
    bytes, sets, symbols, primitive arrays, nested structs and structs
    referenced through the struct cache."""
    h = H.parse_edn("{:type :invoke, :f :cas, :value [7 [1 2]], :process 3, :index 0}\n"
                    "{:type :ok, :f :cas, :value [7 [1 2]], :process 3, :index 1}\n")
    w = FressianOut()
    w.b.append(0xC0)
    w.b.append(0xED)  # closed list of k v forms
    w.obj(Kw("a")); w.obj(2.5)
    w.obj(Kw("b")); w.obj(1.0)
    w.obj(Kw("c")); w.obj({1, 2, 3})
    w.obj(Kw("d")); w.obj(Tagged("atom", 5))
    w.obj(Kw("e")); w.obj(Tagged("atom", 6))  # struct cache reference
    assert 0xA0 in w.b
    w.obj(Kw("inst")); w.inst(1635353698000)
    w.obj(Kw("uuid")); w.b.append(0xC3); w.b.append(0xD0 + 4); w.b += b"\x00\x01\x02\x03"
    w.obj(Kw("sym")); w.b.append(0xC9); w.b.append(0xF7); w.cached("jepsen.etcdemo/r")
    w.obj(Kw("longs")); w.b.append(0xB0); w.int_(3); w.int_(1); w.int_(-2); w.int_(1 << 40)
    w.obj(Kw("doubles")); w.b.append(0xB1); w.int_(2); w.b += struct.pack(">dd", 0.5, 2.0)
    w.obj(Kw("bytes")); w.b.append(0xD9); w.int_(9); w.b += bytes(range(9))
    w.obj(Kw("float")); w.b.append(0xF9); w.b += struct.pack(">f", 1.5)
    w.obj(Kw("nested")); w.obj(Tagged("box", Tagged("box", [Kw("a"), None, True])))
    w.obj(Kw("history")); w.obj(op_maps(h))
    w.b.append(0xFD)
    same(H.parse_fressian(bytes(w.b)), h)


@pytest.mark.parametrize("interleave", [True, False])
def test_write_read_round_trip(tmp_path, interleave):
    h = H.synth(n_keys=5, ops_per_key=60, concurrency=6, info_rate=0.05, interleave=interleave,
                nemesis_period=2.0 if interleave else 0.0, seed=3)
    path = str(tmp_path / "test.fressian")
    H.write_fressian(path, h)
    same(H.read_fressian(path), h)
    # the library's writer and this test's encoder agree byte for byte on op maps
    w = FressianOut()
    w.obj({Kw("name"): "lincheck", Kw("history"): op_maps(h, extra=False)})
    assert open(path, "rb").read() == bytes(w.b)


def test_mutex_and_plain_values():
    h = H.parse_edn("{:type :invoke, :f :acquire, :value nil, :process 0, :index 0}\n"
                    "{:type :ok, :f :acquire, :value nil, :process 0, :index 1}\n"
                    "{:type :invoke, :f :release, :value nil, :process 0, :index 2}\n"
                    "{:type :ok, :f :release, :value nil, :process 0, :index 3}\n")
    same(H.parse_fressian(encode(op_maps(h))), h)
    g = H.parse_edn("{:type :invoke, :f :write, :value 4, :process 0, :index 0}\n"
                    "{:type :ok, :f :write, :value 4, :process 0, :index 1}\n"
                    "{:type :invoke, :f :read, :value nil, :process 1, :index 2}\n"
                    "{:type :ok, :f :read, :value 4, :process 1, :index 3}\n")
    same(H.parse_fressian(encode(op_maps(g))), g)
    assert Packed(H.parse_fressian(encode(op_maps(g)))).keys == Packed(g).keys


def test_large_ints():
    rows = "".join(f"{{:type :invoke, :f :write, :value [{k} {v}], :process 0, :index {2*i}}}\n"
                   f"{{:type :ok, :f :write, :value [{k} {v}], :process 0, :index {2*i+1}}}\n"
                   for i, (k, v) in enumerate([(0, 64), (1, -4097), (2, 1 << 19), (3, -(1 << 25)), (4, 1 << 33),
                                               (5, -(1 << 41)), (6, 1 << 49), (7, (1 << 62) + 5), (8, -65)]))
    h = H.parse_edn(rows)
    same(H.parse_fressian(encode(op_maps(h))), h)


@pytest.mark.parametrize("data", [b"", b"\xc0", b"\xc0\xe4", b"\xc0\xe2\xca\xf7\xcd\xdf", b"\x9f",
                                  b"\xa3", b"\xec\x7f", b"\xe5\xc0\xe2\xca\xf7\xcd\xdftype\xca\xf7\xcd\xdbok\xca"])
def test_malformed(data):
    with pytest.raises(N.LincheckError):
        H.parse_fressian(data)


def test_errors_name_the_op():
    h = H.parse_edn("{:type :invoke, :f :write, :value [0 3], :process 0, :index 0}\n")
    ops = op_maps(h)
    ops[0][Kw("type")] = Kw("wat")
    with pytest.raises(N.LincheckError, match="op 0"):
        H.parse_fressian(encode(ops))
    with pytest.raises(N.LincheckError, match="no :history"):
        H.parse_fressian(encode({Kw("name"): "x"}))
    ops = op_maps(h)
    ops[0][Kw("value")] = [0, "three"]
    with pytest.raises(N.LincheckError, match="value is not an integer"):
        H.parse_fressian(encode(ops))


def test_missing_file(tmp_path):
    with pytest.raises(N.LincheckError):
        H.read_fressian(str(tmp_path / "nope.fressian"))


def test_deep_nesting_is_refused():
    data = b"\xe5" * 10000 + b"\x01"
    with pytest.raises(N.LincheckError, match="too deep"):
        H.parse_fressian(data)


@pytest.mark.parametrize("data", [b"\xed\xcf", b"\xe6\x01\xcf\xcf\xcf\xcf", b"\xcf\xcf\xcf\xcf",
                                  b"\xc0\xed\xca\xf7\xcd\xdetype\xcf"])
def test_footer_inside_a_collection_is_refused(data):
    """A FOOTER code inside a closed or counted list (or as the first byte) is
    a malformed file: refused at once, never read again and again."""
    with pytest.raises(N.LincheckError, match="footer"):
        H.parse_fressian(data)


def test_open_list_ends_at_the_footer(c1):
    """An open list of op maps followed by the file's footer: the list ends
    there (org.fressian's writer closes a top-level open list with it)."""
    w = FressianOut()
    w.obj(Open(op_maps(c1, extra=False)))
    w.footer()
    same(H.parse_fressian(bytes(w.b)), c1)


def test_nested_priority_cache_indices():
    """PUT_PRIORITY_CACHE around a value that itself puts strings in the cache
    (a whole keyword cached, its name cached inside it): org.fressian's reader
    takes the outer slot before reading the value (readAndCacheObject) and its
    writer numbers the outer value first, so the keyword gets index i and its
    name i + 1.  Later packed references (0x80 + i) must find the keyword."""
    h = H.parse_edn("{:type :invoke, :f :write, :value [0 3], :process 0, :index 0}\n"
                    "{:type :ok, :f :write, :value [0 3], :process 0, :index 1}\n"
                    "{:type :invoke, :f :read, :value [0 nil], :process 1, :index 2}\n"
                    "{:type :ok, :f :read, :value [0 3], :process 1, :index 3}\n")
    w = FressianOut()
    slot = {}

    def kw(name):
        if name in slot:
            w.b.append(0x80 + slot[name])
            return
        w.b.append(0xCD)                     # PUT_PRIORITY_CACHE: the keyword itself ...
        slot[name] = len(w.cache)
        w.cache[("kw", name)] = slot[name]   # (the outer slot, taken first)
        w.b += b"\xca\xf7"                   # ... KEY, nil namespace,
        w.cached(name)                       # ... and its name, cached at the next slot
        assert w.cache[name] == slot[name] + 1

    ops = op_maps(h, extra=False)
    w.b.append(0xE4 + len(ops))
    for m in ops:
        w.b.append(0xC0)
        w.b.append(0xEC)
        w.int_(2 * len(m))
        for k, v in m.items():
            kw(str(k))
            if isinstance(v, Kw):
                kw(str(v))
            else:
                w.obj(v)
    assert sum(1 for x in w.b if 0x80 <= x < 0xA0) > 10  # keywords referenced by slot
    same(H.parse_fressian(bytes(w.b)), h)
