#!/usr/bin/env python3
"""Plot the simulator's visualizer log (``-visualizer_enabled 1``).

The reference writes a gz log each sample period (visualizer.cc:56-84) that
its AerialVision GUI turns into time-series and per-core heat maps.  This is
the non-interactive equivalent: one HTML page with IPC, cache and DRAM
activity over time and a per-SM instruction heat map.

    visualizer.py gpgpusim_visualizer.log -o visualizer.html
"""
from __future__ import annotations

import argparse
import html
import os
import sys
from typing import Dict, List

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from accel_sim_framework_distributed_amd.plotting import svg  # noqa: E402
else:
    from . import svg


def parse(path: str) -> List[Dict]:
    rows = []
    for line in open(path):
        d: Dict = {}
        for tok in line.split():
            if "=" not in tok:
                continue
            k, v = tok.split("=", 1)
            if k == "sm_insn":
                d[k] = [int(x) for x in v.split(",") if x]
            elif k == "kernel":
                d[k] = v
            else:
                try:
                    d[k] = float(v)
                except ValueError:
                    d[k] = v
        if d:
            rows.append(d)
    return rows


def line_chart(xs: List[float], series: Dict[str, List[float]], title: str, width=900, height=260) -> str:
    if not xs:
        return ""
    m = 50
    W, H = width - 2 * m, height - 2 * m
    x0, x1 = min(xs), max(xs) or 1
    hi = max((max(v) for v in series.values() if v), default=1.0) or 1.0
    out = [f'<svg xmlns="http://www.w3.org/2000/svg" width="{width}" height="{height}" font-family="sans-serif" '
           f'font-size="11"><rect width="100%" height="100%" fill="white"/>',
           f'<text x="{width / 2}" y="18" text-anchor="middle" font-size="13">{html.escape(title)}</text>',
           f'<rect x="{m}" y="{m}" width="{W}" height="{H}" fill="none" stroke="#444"/>',
           f'<text x="{m}" y="{m + H + 16}">{x0:.0f}</text><text x="{m + W}" y="{m + H + 16}" text-anchor="end">'
           f'{x1:.0f} cycles</text><text x="{m - 4}" y="{m + 4}" text-anchor="end">{hi:.3g}</text>']
    for i, (name, ys) in enumerate(series.items()):
        pts = " ".join(f"{m + (x - x0) / max(1e-9, x1 - x0) * W:.1f},{m + H - y / hi * H:.1f}" for x, y in zip(xs, ys))
        c = svg.PALETTE[i % len(svg.PALETTE)]
        out.append(f'<polyline fill="none" stroke="{c}" stroke-width="1.5" points="{pts}"/>')
        out.append(f'<text x="{m + 8}" y="{m + 14 + 13 * i}" fill="{c}">{html.escape(name)}</text>')
    out.append("</svg>")
    return "".join(out)


def heatmap(rows: List[Dict], width=900) -> str:
    mats = [r.get("sm_insn", []) for r in rows]
    if not mats or not mats[0]:
        return ""
    n_sm = max(len(m) for m in mats)
    hi = max((max(m) for m in mats if m), default=1) or 1
    cw = max(1.0, (width - 100) / len(mats))
    ch = max(2.0, min(6.0, 600 / n_sm))
    h = int(ch * n_sm + 60)
    out = [f'<svg xmlns="http://www.w3.org/2000/svg" width="{width}" height="{h}" font-family="sans-serif" '
           f'font-size="11"><text x="10" y="16">warp instructions per SM per sample (max {hi})</text>']
    for t, m in enumerate(mats):
        for s, v in enumerate(m):
            if v:
                a = v / hi
                out.append(f'<rect x="{60 + t * cw:.1f}" y="{30 + s * ch:.1f}" width="{cw:.1f}" height="{ch:.1f}" '
                           f'fill="rgb({int(255 * a)},{int(80 * (1 - a))},{int(255 * (1 - a))})"/>')
    out.append(f'<text x="10" y="{30 + n_sm * ch / 2:.0f}">SM</text></svg>')
    return "".join(out)


def render(rows: List[Dict]) -> str:
    xs = [r["cycle"] for r in rows]
    body = [f"<h2>visualizer: {len(rows)} samples</h2>",
            line_chart(xs, {"IPC": [r.get("ipc", 0) for r in rows]}, "IPC (thread instructions / cycle)"),
            line_chart(xs, {"DRAM utilisation": [r.get("dram_util", 0) for r in rows]}, "DRAM bandwidth utilisation"),
            line_chart(xs, {"L1 misses": [r.get("l1_miss", 0) for r in rows],
                            "L2 accesses": [r.get("l2_access", 0) for r in rows],
                            "L2 misses": [r.get("l2_miss", 0) for r in rows]}, "cache activity per sample"),
            heatmap(rows)]
    return svg.page("visualizer", body)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("log")
    ap.add_argument("-o", "--out", default="visualizer.html")
    o = ap.parse_args(argv)
    rows = parse(o.log)
    with open(o.out, "w") as f:
        f.write(render(rows))
    print(f"wrote {o.out} ({len(rows)} samples)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
