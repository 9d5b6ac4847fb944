"""Dependency-free SVG/HTML charts (plotly/matplotlib are not part of this
image): log/linear scatter with a y=x line for correlation plots, grouped
bars for get_stats CSVs."""
from __future__ import annotations

import html
import math
from typing import Dict, List, Optional, Sequence, Tuple

PALETTE = ["#1f77b4", "#d62728", "#2ca02c", "#ff7f0e", "#9467bd", "#8c564b", "#e377c2", "#7f7f7f", "#bcbd22",
           "#17becf"]


def _ticks(lo: float, hi: float, log: bool) -> List[float]:
    if log:
        a, b = math.floor(math.log10(lo)), math.ceil(math.log10(hi))
        return [10.0 ** e for e in range(a, b + 1)]
    step = 10 ** math.floor(math.log10(max(hi - lo, 1e-12)))
    while (hi - lo) / step > 8:
        step *= 2
    t, out = math.floor(lo / step) * step, []
    while t <= hi + 1e-12:
        out.append(t)
        t += step
    return out


def scatter(series: Dict[str, Sequence[Tuple[float, float, str]]], title: str, xlabel: str, ylabel: str,
            log: bool = True, width: int = 720, height: int = 560) -> str:
    """series: name -> [(hw, sim, label)].  Returns an <svg> string."""
    pts = [(x, y) for s in series.values() for x, y, _ in s if (x > 0 and y > 0) or not log]
    if not pts:
        return f"<p>{html.escape(title)}: no data</p>"
    lo = min(min(p) for p in pts)
    hi = max(max(p) for p in pts)
    if log:
        lo, hi = lo / 1.5, hi * 1.5
    else:
        pad = (hi - lo) * 0.05 or 1.0
        lo, hi = lo - pad, hi + pad
    m = 70
    W, H = width - 2 * m, height - 2 * m

    def tx(v):
        f = (math.log10(v) - math.log10(lo)) / (math.log10(hi) - math.log10(lo)) if log else (v - lo) / (hi - lo)
        return m + f * W

    def ty(v):
        f = (math.log10(v) - math.log10(lo)) / (math.log10(hi) - math.log10(lo)) if log else (v - lo) / (hi - lo)
        return m + H - f * H

    out = [f'<svg xmlns="http://www.w3.org/2000/svg" width="{width}" height="{height}" font-family="sans-serif" '
           f'font-size="12"><rect width="100%" height="100%" fill="white"/>',
           f'<text x="{width / 2}" y="24" text-anchor="middle" font-size="15">{html.escape(title)}</text>',
           f'<rect x="{m}" y="{m}" width="{W}" height="{H}" fill="none" stroke="#444"/>']
    for t in _ticks(lo, hi, log):
        if lo <= t <= hi:
            out.append(f'<line x1="{tx(t):.1f}" y1="{m + H}" x2="{tx(t):.1f}" y2="{m + H + 5}" stroke="#444"/>'
                       f'<text x="{tx(t):.1f}" y="{m + H + 18}" text-anchor="middle">{t:.3g}</text>'
                       f'<line x1="{m - 5}" y1="{ty(t):.1f}" x2="{m}" y2="{ty(t):.1f}" stroke="#444"/>'
                       f'<text x="{m - 8}" y="{ty(t) + 4:.1f}" text-anchor="end">{t:.3g}</text>')
    out.append(f'<line x1="{tx(lo):.1f}" y1="{ty(lo):.1f}" x2="{tx(hi):.1f}" y2="{ty(hi):.1f}" stroke="#999" '
               f'stroke-dasharray="4,3"/>')
    for i, (name, s) in enumerate(series.items()):
        c = PALETTE[i % len(PALETTE)]
        for x, y, lab in s:
            if log and (x <= 0 or y <= 0):
                continue
            out.append(f'<circle cx="{tx(x):.1f}" cy="{ty(y):.1f}" r="4" fill="{c}" fill-opacity="0.75">'
                       f'<title>{html.escape(lab)}: hw={x:.4g} sim={y:.4g}</title></circle>')
        out.append(f'<rect x="{m + 10}" y="{m + 10 + 18 * i}" width="10" height="10" fill="{c}"/>'
                   f'<text x="{m + 26}" y="{m + 19 + 18 * i}">{html.escape(name)}</text>')
    out.append(f'<text x="{width / 2}" y="{height - 12}" text-anchor="middle">{html.escape(xlabel)}</text>')
    out.append(f'<text x="16" y="{height / 2}" text-anchor="middle" transform="rotate(-90 16 {height / 2})">'
               f'{html.escape(ylabel)}</text></svg>')
    return "".join(out)


def bars(groups: List[str], series: Dict[str, List[Optional[float]]], title: str, ylabel: str,
         width: int = 900, height: int = 420) -> str:
    vals = [v for s in series.values() for v in s if v is not None]
    if not vals:
        return f"<p>{html.escape(title)}: no data</p>"
    hi = max(vals) * 1.1 or 1.0
    m, mb = 60, 110
    W, H = width - 2 * m, height - m - mb
    n = max(1, len(series))
    gw = W / max(1, len(groups))
    bw = gw * 0.8 / n
    out = [f'<svg xmlns="http://www.w3.org/2000/svg" width="{width}" height="{height}" font-family="sans-serif" '
           f'font-size="11"><rect width="100%" height="100%" fill="white"/>',
           f'<text x="{width / 2}" y="22" text-anchor="middle" font-size="14">{html.escape(title)}</text>',
           f'<line x1="{m}" y1="{m + H}" x2="{m + W}" y2="{m + H}" stroke="#444"/>']
    for t in _ticks(0, hi, False):
        y = m + H - t / hi * H
        out.append(f'<text x="{m - 6}" y="{y + 4:.1f}" text-anchor="end">{t:.3g}</text>'
                   f'<line x1="{m}" y1="{y:.1f}" x2="{m + W}" y2="{y:.1f}" stroke="#eee"/>')
    for gi, g in enumerate(groups):
        x0 = m + gi * gw + gw * 0.1
        for si, (name, s) in enumerate(series.items()):
            v = s[gi] if gi < len(s) else None
            if v is None:
                continue
            h = v / hi * H
            out.append(f'<rect x="{x0 + si * bw:.1f}" y="{m + H - h:.1f}" width="{bw:.1f}" height="{h:.1f}" '
                       f'fill="{PALETTE[si % len(PALETTE)]}"><title>{html.escape(g)} / {html.escape(name)}: '
                       f'{v:.4g}</title></rect>')
        out.append(f'<text x="{m + gi * gw + gw / 2:.1f}" y="{m + H + 12}" text-anchor="end" '
                   f'transform="rotate(-45 {m + gi * gw + gw / 2:.1f} {m + H + 12})">{html.escape(g[:40])}</text>')
    for si, name in enumerate(series):
        out.append(f'<rect x="{m + W - 200}" y="{m + 14 * si}" width="10" height="10" '
                   f'fill="{PALETTE[si % len(PALETTE)]}"/><text x="{m + W - 185}" y="{m + 9 + 14 * si}">'
                   f'{html.escape(name)}</text>')
    out.append(f'<text x="14" y="{m + H / 2}" text-anchor="middle" transform="rotate(-90 14 {m + H / 2})">'
               f'{html.escape(ylabel)}</text></svg>')
    return "".join(out)


def page(title: str, body: List[str]) -> str:
    return ("<!DOCTYPE html><html><head><meta charset='utf-8'><title>" + html.escape(title) +
            "</title></head><body style='font-family:sans-serif'>" + "\n".join(body) + "</body></html>\n")
