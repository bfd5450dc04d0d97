"""Static guard for the Clojure binding (clj/**/*.clj; no JVM in this image).

A local that shadows a clojure.core var turns every later call of that var in
its scope into a call of the local: round 2's gpu_checker.clj bound
`key (Memory. ...)` in `marshal` and then called `(key value)` on every
independent tuple, so the drop-in at etcdemo.clj:115-119 threw on its first
keyed op.  This test reads the .clj sources with a small reader of its own and
fails if any binding form -- let / loop / when-let / if-let / binding / doseq /
for / dotimes / with-open / letfn, fn / defn parameters, destructuring
included -- binds one of the names below.
"""

import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLJ = sorted(glob.glob(os.path.join(ROOT, "jepsen-etcd-demo_amd", "clj", "**", "*.clj"), recursive=True))

# clojure.core vars a local must not shadow (the round-2 verdict's list, and the
# other core functions this binding or a later edit would plausibly call)
BANNED = set("""
key val type fn keys vals name count first next map keep list set vec str int long byte char
range filter remove reduce some second last rest seq into get assoc update merge comp partial apply
identity min max bytes short double float boolean num class meta hash time print println format
find sort sort-by group-by frequencies partition take drop concat cons conj disj dissoc empty
every? not-any? nth peek pop subs symbol keyword ns var ref atom agent future promise deliver
force delay test methods replace shuffle distinct flatten interleave interpose repeat cycle iterate
""".split())

BINDING_VECTOR_FORMS = {"let", "loop", "when-let", "if-let", "when-some", "if-some", "binding", "doseq",
                        "for", "dotimes", "with-open", "with-local-vars", "when-first"}
FN_FORMS = {"fn", "defn", "defn-", "defmacro", "bound-fn"}


class Sym(str):
    pass


class Kw(str):
    pass


class Vec(list):
    pass


class Map(list):
    pass


class Lst(list):
    pass


TOKEN = re.compile(r"""
    (?P<ws>[\s,]+)
  | (?P<comment>;[^\n]*)
  | (?P<string>"(?:\\.|[^"\\])*")
  | (?P<char>\\(?:newline|space|tab|formfeed|backspace|return|u[0-9a-fA-F]{4}|o[0-7]{1,3}|.))
  | (?P<open>\#\{|\#\(|\#\?\(|\#\?@\(|[(\[{])
  | (?P<close>[)\]}])
  | (?P<regex>\#"(?:\\.|[^"\\])*")
  | (?P<discard>\#_)
  | (?P<meta>\^)
  | (?P<quote>'|`|~@|~|@|\#')
  | (?P<atom>[^\s,;()\[\]{}"\\^]+)
""", re.X)


def read_all(text):
    """The top-level forms of a Clojure source (enough of the reader for the
    binding forms: strings, chars, comments, metadata and reader macros)."""
    stack = [Lst()]
    pending_meta = []   # ^meta applies to the next form: dropped
    discard = []
    for m in TOKEN.finditer(text):
        kind = m.lastgroup
        tok = m.group(kind)
        if kind in ("ws", "comment"):
            continue
        if kind == "open":
            node = Vec() if tok == "[" else Map() if tok == "{" else Lst()
            stack.append(node)
            continue
        if kind == "close":
            node = stack.pop()
            _emit(stack, node, pending_meta, discard)
            continue
        if kind in ("meta", "discard", "quote"):
            if kind == "meta":
                pending_meta.append(len(stack))
            elif kind == "discard":
                discard.append(len(stack))
            continue
        if kind == "atom":
            node = Kw(tok) if tok.startswith(":") else Sym(tok)
        else:
            node = tok  # strings, chars, regexes
        _emit(stack, node, pending_meta, discard)
    assert len(stack) == 1, "unbalanced forms"
    return stack[0]


def _emit(stack, node, pending_meta, discard):
    depth = len(stack)
    if pending_meta and pending_meta[-1] == depth:
        # this form is the metadata itself; the next form at this depth is the target
        pending_meta.pop()
        return
    if discard and discard[-1] == depth:
        discard.pop()
        return
    stack[-1].append(node)


def binding_names(form):
    """Symbols a destructuring form binds."""
    out = []
    if isinstance(form, Sym):
        if form not in ("&", "_"):
            out.append(str(form))
    elif isinstance(form, Vec):
        it = iter(form)
        for x in it:
            if isinstance(x, Kw) and x == ":as":
                out += binding_names(next(it, None))
            else:
                out += binding_names(x)
    elif isinstance(form, Map):
        items = list(form)
        for k, v in zip(items[0::2], items[1::2]):
            if isinstance(k, Kw) and k in (":keys", ":strs", ":syms") and isinstance(v, Vec):
                out += [str(s).split("/")[-1] for s in v if isinstance(s, (Sym, Kw))]
            elif isinstance(k, Kw) and k == ":as":
                out += binding_names(v)
            elif isinstance(k, Kw) and k == ":or":
                continue
            else:
                out += binding_names(k)
    return out


def _vector_bindings(vec, seq_form):
    out = []
    items = list(vec)
    i = 0
    while i + 1 < len(items):
        target, value = items[i], items[i + 1]
        if seq_form and isinstance(target, Kw):
            if target == ":let" and isinstance(value, Vec):
                out += _vector_bindings(value, False)
        else:
            out += binding_names(target)
        i += 2
    return out


def bound_names(form):
    """(line-less) names bound anywhere inside form, with the binding form's head."""
    found = []

    def walk(x):
        if isinstance(x, Lst) and x and isinstance(x[0], Sym):
            head = str(x[0])
            if head in BINDING_VECTOR_FORMS and len(x) > 1 and isinstance(x[1], Vec):
                found.extend((head, n) for n in _vector_bindings(x[1], head in ("doseq", "for")))
            elif head == "letfn" and len(x) > 1 and isinstance(x[1], Vec):
                for f in x[1]:
                    if isinstance(f, Lst) and f:
                        found.extend(("letfn", n) for n in binding_names(f[0]))
                        for part in f[1:]:
                            if isinstance(part, Vec):
                                found.extend(("letfn", n) for n in binding_names(part))
                            elif isinstance(part, Lst) and part and isinstance(part[0], Vec):
                                found.extend(("letfn", n) for n in binding_names(part[0]))
            elif head in FN_FORMS:
                rest = x[1:]
                if rest and isinstance(rest[0], Sym) and head == "fn":
                    found.append(("fn", str(rest[0])))  # a named fn binds its name locally
                for part in rest:
                    if isinstance(part, Vec):
                        found.extend((head, n) for n in binding_names(part))
                        break
                    if isinstance(part, Lst) and part and isinstance(part[0], Vec):  # multi-arity
                        found.extend((head, n) for n in binding_names(part[0]))
        if isinstance(x, list):
            for y in x:
                walk(y)

    walk(form)
    return found


def test_reader_sees_the_round2_bug():
    # the shape that broke round 2: a Memory bound to `key`, then (key value)
    src = '(defn- marshal [h] (let [n (count h) key (Memory. 8) [k v] [(key value) 1]] key))'
    names = [n for _, n in bound_names(read_all(src))]
    assert "key" in names and "k" in names and "v" in names
    src2 = '(defn f [{:keys [keep hist] :as opts} & more] (for [x xs :let [vals 1] :when x] x))'
    names2 = [n for _, n in bound_names(read_all(src2))]
    assert {"keep", "hist", "opts", "more", "x", "vals"} <= set(names2)


def test_reader_skips_strings_comments_and_metadata():
    src = '(ns a "doc (let [key 1])") ; (let [type 2])\n(defn ^:private g ^long [^long x] (str "[fn]" \\( x))'
    names = [n for _, n in bound_names(read_all(src))]
    assert names == ["x"]


@pytest.mark.parametrize("path", CLJ, ids=[os.path.relpath(p, ROOT) for p in CLJ])
def test_no_local_shadows_clojure_core(path):
    forms = read_all(open(path, encoding="utf-8").read())
    bad = sorted({(head, n) for head, n in bound_names(forms) if n in BANNED})
    assert not bad, f"{os.path.relpath(path, ROOT)}: locals shadowing clojure.core: {bad}"


def test_clj_sources_exist():
    assert CLJ, "no Clojure sources found under jepsen-etcd-demo_amd/clj"


# ---- struct layouts the binding writes by byte offset -----------------------
# gpu_checker.clj fills lc_opts / lc_history / lc_pack_opts / lc_result through
# JNA Memory at hand-written offsets (no JVM here to run it).  Those offsets and
# sizes are checked against the ctypes mirror of include/lincheck.h, whose own
# sizes tests/test_abi.py pins against the compiled library.

def _clj_text():
    return open(os.path.join(ROOT, "jepsen-etcd-demo_amd", "clj", "jepsen", "etcdemo", "gpu_checker.clj"),
                encoding="utf-8").read()


def _native():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "jepsen-etcd-demo_amd"))
    from lincheck import _native as N
    return N


def test_lc_opts_offsets_match_header():
    N = _native()
    src = _clj_text()
    size = int(re.search(r"\(Memory\. (\d+)\)[^;\n]*; sizeof\(lc_opts\)", src).group(1))
    assert size == C_sizeof(N.LcOpts)
    # (.setX opts OFF ...) ; field
    pairs = re.findall(r"\(\.set(?:Int|Long) opts (\d+|\(\+ (\d+) \(\* 4 g\)\)) .*?; (\w+)", src)
    seen = {}
    for off, base, field in pairs:
        seen[field] = int(base or off)
    assert seen, "no lc_opts writes found"
    for field, off in seen.items():
        assert getattr(N.LcOpts, field).offset == off, (field, off)


def test_lc_history_and_result_offsets_match_header():
    N = _native()
    src = _clj_text()
    assert int(re.search(r"hist\s+\(Memory\. (\d+)\)", src).group(1)) == C_sizeof(N.LcHistory)
    order = ["type", "f", "process", "key", "v0", "v1", "index", "mop_off", "mop"]
    offs = [int(x) for x in re.findall(r"\[(\d+) [\w-]+\]", src[src.index("(doseq [[off m]"):])[:len(order)]]
    assert offs == [getattr(N.LcHistory, f).offset for f in order]
    assert int(re.search(r"\(Memory\. (\d+)\)[^;\n]*; sizeof\(lc_pack_opts\)", src).group(1)) == C_sizeof(N.LcPackOpts)
    assert int(re.search(r"\(Memory\. (\d+)\)[^;\n]*; sizeof\(lc_batch\)", src).group(1)) == C_sizeof(N.LcBatch)
    assert int(re.search(r"\(Memory\. (\d+)\)[^;\n]*; sizeof\(lc_result\)", src).group(1)) == C_sizeof(N.LcResult)
    res = dict((f, int(o)) for o, f in re.findall(r"\(\.setPointer result (\d+) ([\w-]+)\)", src))
    want = {"valid": "valid", "fail-ev": "fail_event", "cause": "cause", "finals": "final_configs",
            "n-final": "n_final", "analyzer": "analyzer"}
    assert set(res) == set(want)
    for local, field in want.items():
        assert getattr(N.LcResult, field).offset == res[local], (local, field)


def C_sizeof(t):
    import ctypes
    return ctypes.sizeof(t)
