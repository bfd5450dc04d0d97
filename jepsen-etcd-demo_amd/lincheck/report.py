"""Counterexample drawing: the Python side of knossos.linear.report/render-analysis!,
which jepsen.checker/linearizable calls for a key whose analysis is not valid,
writing linear.svg under the key's store directory.

The JVM drop-in (clj/jepsen/etcdemo/gpu_checker.clj) calls Knossos's own
renderer on the decoded analysis.  This module draws the same content for the
Python mirror, laid out its own way (display only; no rendering of Knossos's
is available here to compare against, so the layout is unpinned): one row per
process, one box per operation from its invocation to its completion in
history order, the :previous-ok and failing :op outlined, and each final path
as a line through the operations it linearizes, labelled with the model state
after each step; the last step names why the failing operation cannot
linearize.
"""
from __future__ import annotations

import os
from html import escape
from typing import Any, Dict, List, Optional, Sequence

ROW, COL, PAD, BOX = 40, 46, 16, 26  # px: process row, history column, margins, box height
PATH_COLOURS = ["#1f77b4", "#2ca02c", "#9467bd", "#8c564b", "#e377c2", "#17becf", "#bcbd22", "#7f7f7f",
                "#ff7f0e", "#393b79"]


def _fmt(v: Any) -> str:
    if v is None:
        return "nil"
    if isinstance(v, (list, tuple)):
        return "[" + " ".join(_fmt(x) for x in v) + "]"
    if isinstance(v, dict):
        return "{" + ", ".join(f"{_fmt(k)} {_fmt(x)}" for k, x in v.items()) + "}"
    return str(v)


def _model_label(m: Any) -> str:
    if isinstance(m, dict) and "msg" in m:
        return str(m["msg"])
    if isinstance(m, dict) and "value" in m:
        return _fmt(m["value"])
    return _fmt(m)


def _pairs(history: Sequence[Dict]) -> List[Dict]:
    """Invocation / completion pairs in history order (a process has one
    operation open at a time); an invocation never completed runs to the end."""
    open_: Dict[Any, Dict] = {}
    out: List[Dict] = []
    for pos, o in enumerate(history):
        p = o.get("process")
        t = o.get("type")
        if t == "invoke":
            e = {"process": p, "f": o.get("f"), "value": o.get("value"), "start": pos, "end": None,
                 "index": o.get("index", pos), "type": None}
            open_[p] = e
            out.append(e)
        elif p in open_:
            e = open_.pop(p)
            e["end"], e["type"] = pos, t
            if e["value"] is None:
                e["value"] = o.get("value")
            e["done_index"] = o.get("index", pos)
    for e in out:
        if e["end"] is None:
            e["end"] = len(history)
    return out


def _find(pairs: List[Dict], op: Optional[Dict]) -> Optional[Dict]:
    """The pair an analysis op (an invocation or a completion) belongs to."""
    if not op:
        return None
    idx = op.get("index")
    for e in pairs:
        if idx is not None and (e["index"] == idx or e.get("done_index") == idx):
            return e
    for e in pairs:  # histories without :index
        if e["process"] == op.get("process") and e["f"] == op.get("f") and e["value"] == op.get("value"):
            return e
    return None


def render_svg(history: Sequence[Dict], analysis: Dict) -> str:
    """SVG text for one key's analysis (valid or not)."""
    pairs = _pairs(history)
    prev, bad = _find(pairs, analysis.get("previous-ok")), _find(pairs, analysis.get("op"))
    paths = [[(_find(pairs, s.get("op")), s.get("model")) for s in p] for p in analysis.get("final-paths") or []]
    # the window drawn: from the previous :ok's invocation to the failing op's completion
    lo = prev["start"] if prev else 0
    hi = bad["end"] if bad else len(history)
    for p in paths:
        for e, _ in p:
            if e:
                lo, hi = min(lo, e["start"]), max(hi, e["end"])
    shown = [e for e in pairs if e["end"] >= lo and e["start"] <= hi]
    cols = sorted({e["start"] for e in shown} | {e["end"] for e in shown})
    x = {c: PAD + 140 + i * COL for i, c in enumerate(cols)}
    procs = sorted({e["process"] for e in shown}, key=lambda v: (isinstance(v, str), str(v)))
    y = {p: PAD + 30 + i * ROW for i, p in enumerate(procs)}
    width = PAD * 2 + 140 + max(1, len(cols)) * COL + 160
    height = PAD * 2 + 30 + max(1, len(procs)) * ROW + 20 * len(paths) + 20
    out = [f'<svg xmlns="http://www.w3.org/2000/svg" width="{width}" height="{height}" '
           f'font-family="sans-serif" font-size="11">',
           f'<text x="{PAD}" y="{PAD + 8}" font-size="13">linearizability analysis: valid? '
           f'{escape(_fmt(analysis.get("valid?")).lower())}</text>']
    for p in procs:
        out.append(f'<text x="{PAD}" y="{y[p] + BOX / 2 + 4}">process {escape(_fmt(p))}</text>')
    for e in shown:
        x0, x1 = x[e["start"]], x[e["end"]] + COL * 0.8
        colour = "#fdd" if e is bad else "#dfd" if e is prev else "#eee" if e["type"] == "ok" else "#fff"
        stroke = "#c00" if e is bad else "#070" if e is prev else "#999"
        dash = "" if e["type"] == "ok" else ' stroke-dasharray="4 2"'
        out.append(f'<rect x="{x0:.0f}" y="{y[e["process"]]}" width="{x1 - x0:.0f}" height="{BOX}" rx="3" '
                   f'fill="{colour}" stroke="{stroke}"{dash}/>')
        out.append(f'<text x="{x0 + 4:.0f}" y="{y[e["process"]] + BOX / 2 + 4}">'
                   f'{escape(str(e["f"]))} {escape(_fmt(e["value"]))}</text>')
    for j, p in enumerate(paths):
        colour = PATH_COLOURS[j % len(PATH_COLOURS)]
        pts = []
        for k, (e, m) in enumerate(p):
            if not e:
                continue
            cx = (x[e["start"]] + x[e["end"]] + COL * 0.8) / 2 + 3 * j
            cy = y[e["process"]] + BOX + 4 + 2 * j
            pts.append((cx, cy))
            last = k == len(p) - 1
            out.append(f'<circle cx="{cx:.0f}" cy="{cy}" r="3" fill="{"#c00" if last else colour}"/>')
            out.append(f'<text x="{cx + 4:.0f}" y="{cy + 10}" fill="{"#c00" if last else colour}">'
                       f'{escape(_model_label(m))}</text>')
        if len(pts) > 1:
            out.append(f'<polyline fill="none" stroke="{colour}" stroke-width="1.5" points="'
                       + " ".join(f"{a:.0f},{b}" for a, b in pts) + '"/>')
        ly = PAD + 30 + len(procs) * ROW + 20 * j + 10
        steps = " -> ".join(f'{e["f"] if e else "?"} {_fmt(e["value"]) if e else ""} => {_model_label(m)}'
                            for e, m in p[1:])
        out.append(f'<text x="{PAD}" y="{ly}" fill="{colour}">path {j + 1}: {escape(steps)}</text>')
    out.append("</svg>")
    return "\n".join(out)


def render_analysis(history: Sequence[Dict], analysis: Dict, path: str) -> str:
    """Writes render_svg's drawing to `path` (directories created); returns it."""
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w") as f:
        f.write(render_svg(history, analysis))
    return path
