"""lincheck/report.py: the Python mirror's linear.svg (knossos.linear.report/
render-analysis!, which jepsen.checker/linearizable calls for an invalid
key).  Display only -- no Knossos rendering exists here to compare against,
so the layout is unpinned; these tests check the drawing's content."""
import xml.etree.ElementTree as ET

from lincheck import checker as ck
from lincheck.report import render_analysis, render_svg

NS = "{http://www.w3.org/2000/svg}"

# process 0 writes 3 and completes; process 1 then reads 1: the tutorial's
# "can't read 1 from register 3" shape
HIST = [
    {"index": 0, "process": 0, "type": "invoke", "f": "write", "value": 3},
    {"index": 1, "process": 0, "type": "ok", "f": "write", "value": 3},
    {"index": 2, "process": 1, "type": "invoke", "f": "read", "value": None},
    {"index": 3, "process": 2, "type": "invoke", "f": "cas", "value": [3, 4]},
    {"index": 4, "process": 1, "type": "ok", "f": "read", "value": 1},
]
ANALYSIS = {
    "valid?": False, "analyzer": "linear",
    "op": HIST[4], "previous-ok": HIST[1], "last-op": HIST[1],
    "configs": [],
    "final-paths": [
        [{"op": HIST[1], "model": {"value": 3}},
         {"op": HIST[4], "model": {"msg": "can't read 1 from register 3"}}],
        [{"op": HIST[1], "model": {"value": 3}},
         {"op": {"index": 3, "process": 2, "type": "invoke", "f": "cas", "value": [3, 4]}, "model": {"value": 4}},
         {"op": HIST[4], "model": {"msg": "can't read 1 from register 4"}}],
    ],
}


def test_svg_content():
    root = ET.fromstring(render_svg(HIST, ANALYSIS))
    texts = [t.text or "" for t in root.iter(NS + "text")]
    assert any("valid? false" in t for t in texts)
    # one box per operation of the window, the failing one outlined red, the previous :ok green
    rects = list(root.iter(NS + "rect"))
    assert len(rects) == 3
    assert sum(r.get("stroke") == "#c00" for r in rects) == 1
    assert sum(r.get("stroke") == "#070" for r in rects) == 1
    # the crashed (never completed) cas is dashed
    assert sum(r.get("stroke-dasharray") is not None for r in rects) == 1
    # both final paths: a line each with at least two points, their reasons named
    assert len(list(root.iter(NS + "polyline"))) == 2
    assert any("can't read 1 from register 3" in t for t in texts)
    assert any("can't read 1 from register 4" in t for t in texts)
    assert any(t.startswith("path 2: cas [3 4] => 4") for t in texts)


def test_render_writes_file(tmp_path):
    p = render_analysis(HIST, ANALYSIS, str(tmp_path / "a" / "b" / "linear.svg"))
    ET.parse(p)


def test_draw_only_invalid_and_never_raises(tmp_path):
    ck._draw({"store-path": str(tmp_path)}, HIST, dict(ANALYSIS, **{"valid?": "unknown"}), ["k"])
    ck._draw({}, HIST, ANALYSIS, ["k"])
    assert not list(tmp_path.iterdir())
    ck._draw({"store-path": str(tmp_path)}, HIST, ANALYSIS, ["independent", 7])
    assert (tmp_path / "independent" / "7" / "linear.svg").exists()
    # a broken analysis is a warning, as linearizable's catch-and-warn
    import pytest
    with pytest.warns(UserWarning):
        ck._draw({"store-path": str(tmp_path)}, HIST, {"valid?": False, "final-paths": 5}, ["x"])
