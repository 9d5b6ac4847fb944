#!/usr/bin/env python3
"""Visualizer for the simulator's sample log (``-visualizer_enabled 1``): the
AerialVision equivalent.

The reference writes a gz log each sample period (``visualizer_printstat``,
``gpgpu-sim/src/gpgpu-sim/visualizer.cc:56-84``; per DRAM channel
``dram.cc:815-853``; per L2 sub-partition ``l2cache.cc:866``) and its
Python/Tk GUI AerialVision (``gpu-simulator/gpgpu-sim/aerialvision/``) turns
it into time-lapse views: global counters over time, per-shader / per-channel
heat maps, the warp-divergence breakdown, memory-latency distributions, and
several runs side by side.

This tool builds one self-contained HTML page (no network, no plotting
library): static SVG charts for a quick look, plus an interactive viewer in
plain JavaScript with the same views as AerialVision's main window:

* time series of any global variable, one line per log (run comparison);
* a per-unit heat map (SM or memory channel x sample) of any vector variable,
  with a value read-out under the mouse;
* the stacked issue breakdown per sample (idle / scoreboard / stall / issued
  with 1-8, 9-16, ... 57-64 active lanes: the warp-divergence view);
* the L1-miss round-trip latency histogram over a chosen cycle range;
* a cycle-range zoom shared by every view, kernel boundaries marked.

The log is one ``key=value`` line per sample period (``simulator.cc``
``write_visualizer_sample``); ``.gz`` logs are read as well.

    visualizer.py run.log [other.log ...] -o visualizer.html
    visualizer.py run.log --csv sm_insn        # one variable as CSV (sample x unit)
"""
from __future__ import annotations

import argparse
import gzip
import html
import json
import os
import sys
from typing import Dict, List, Sequence

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from accel_sim_framework_distributed_amd.plotting import svg  # noqa: E402
else:
    from . import svg

# vector variables: per SM, per memory channel, or distributions
SM_VECTORS = ("sm_insn", "sm_l1_miss_rate", "sm_occupancy", "sm_active", "sm_pkts_out")
CH_VECTORS = ("ch_dram_util", "ch_dram_queue", "ch_dram_req", "ch_dram_act", "ch_l2_hit", "ch_l2_miss")
DISTRIBUTIONS = ("issue_distro", "mf_lat_hist")
VECTORS = SM_VECTORS + CH_VECTORS + DISTRIBUTIONS


def _open(path: str):
    return gzip.open(path, "rt") if path.endswith(".gz") else open(path)


def parse(path: str) -> List[Dict]:
    """One dict per sample: floats for scalars, lists for vector variables."""
    rows = []
    with _open(path) as fh:
        for line in fh:
            d: Dict = {}
            for tok in line.split():
                if "=" not in tok:
                    continue
                k, v = tok.split("=", 1)
                if k == "kernel":
                    d[k] = v
                elif k in VECTORS or "," in v:
                    try:
                        d[k] = [float(x) for x in v.split(",") if x]
                    except ValueError:
                        d[k] = v
                else:
                    try:
                        d[k] = float(v)
                    except ValueError:
                        d[k] = v
            if d:
                rows.append(d)
    return rows


def scalar_keys(rows: Sequence[Dict]) -> List[str]:
    keys: List[str] = []
    for r in rows:
        for k, v in r.items():
            if isinstance(v, float) and k not in keys and k not in ("cycle",):
                keys.append(k)
    return keys


def vector_keys(rows: Sequence[Dict]) -> List[str]:
    keys: List[str] = []
    for r in rows:
        for k, v in r.items():
            if isinstance(v, list) and k not in keys:
                keys.append(k)
    return keys


def issue_groups(distro: Sequence[float]) -> Dict[str, float]:
    """Collapse the issue distribution (idle, scoreboard, stall, then issued
    with k = 1..64 active lanes) into AerialVision-style bins."""
    out = {"idle": 0.0, "scoreboard": 0.0, "stall": 0.0}
    if not distro:
        return out
    out["idle"], out["scoreboard"], out["stall"] = distro[0], distro[1], distro[2]
    for lo in range(1, 65, 8):
        out[f"W{lo}-{lo + 7}"] = float(sum(distro[2 + k] for k in range(lo, lo + 8) if 2 + k < len(distro)))
    return out


def to_csv(rows: Sequence[Dict], key: str) -> str:
    """One variable as CSV: cycle, then the value (scalar) or one column per unit."""
    lines = []
    for r in rows:
        v = r.get(key)
        if v is None:
            continue
        vals = v if isinstance(v, list) else [v]
        lines.append(",".join([f"{r.get('cycle', 0):.0f}"] + [f"{x:g}" for x in vals]))
    return "\n".join(lines) + "\n"


# ---------------------------------------------------------------------------
# static SVG (quick look without JavaScript)
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


def heatmap(rows: List[Dict], key: str = "sm_insn", width=900) -> str:
    mats = [r.get(key, []) for r in rows]
    if not mats or not mats[0]:
        return ""
    n_u = max(len(m) for m in mats)
    hi = max((max(m) for m in mats if m), default=1) or 1
    cw = max(1.0, (width - 100) / len(mats))
    ch = max(2.0, min(6.0, 600 / n_u))
    h = int(ch * n_u + 60)
    out = [f'<svg xmlns="http://www.w3.org/2000/svg" width="{width}" height="{h}" font-family="sans-serif" '
           f'font-size="11"><text x="10" y="16">{html.escape(key)} per unit per sample (max {hi:g})</text>']
    for t, m in enumerate(mats):
        for s, v in enumerate(m):
            if v:
                a = v / hi
                out.append(f'<rect x="{60 + t * cw:.1f}" y="{30 + s * ch:.1f}" width="{cw:.1f}" height="{ch:.1f}" '
                           f'fill="rgb({int(255 * a)},{int(80 * (1 - a))},{int(255 * (1 - a))})"/>')
    out.append(f'<text x="10" y="{30 + n_u * ch / 2:.0f}">unit</text></svg>')
    return "".join(out)


# ---------------------------------------------------------------------------
# interactive viewer
_JS = r"""
const RUNS = JSON.parse(document.getElementById('asim-data').textContent);
const PAL = %PALETTE%;
const $ = id => document.getElementById(id);
function keysOf(kind) {
  const s = new Set();
  for (const r of RUNS) for (const row of r.rows) for (const k in row)
    if ((kind === 'v') === Array.isArray(row[k]) && k !== 'kernel' && k !== 'cycle') s.add(k);
  return [...s];
}
function fill(sel, keys, def) {
  sel.innerHTML = keys.map(k => `<option${k === def ? ' selected' : ''}>${k}</option>`).join('');
}
function range() {
  let lo = parseFloat($('c0').value), hi = parseFloat($('c1').value);
  if (!isFinite(lo)) lo = -Infinity; if (!isFinite(hi)) hi = Infinity;
  return [lo, hi];
}
function rowsIn(run) { const [lo, hi] = range(); return run.rows.filter(r => r.cycle >= lo && r.cycle <= hi); }
function svgEl(w, h) { return `<svg xmlns="http://www.w3.org/2000/svg" width="${w}" height="${h}" font-size="11" font-family="sans-serif">`; }
function kernelMarks(rows, x, top, bot) {
  let out = '', prev = null;
  for (const r of rows) {
    if (r.kernel !== prev && prev !== null)
      out += `<line x1="${x(r.cycle)}" x2="${x(r.cycle)}" y1="${top}" y2="${bot}" stroke="#999" stroke-dasharray="3,3"/>` +
             `<text x="${x(r.cycle) + 2}" y="${top + 10}" fill="#666">${r.kernel}</text>`;
    prev = r.kernel;
  }
  return out;
}
function drawSeries() {
  const k = $('svar').value, W = 900, H = 280, m = 50;
  let xs = [], ys = [];
  const sets = RUNS.map(run => rowsIn(run).filter(r => typeof r[k] === 'number'));
  for (const s of sets) for (const r of s) { xs.push(r.cycle); ys.push(r[k]); }
  if (!xs.length) { $('series').innerHTML = '<p>no samples in range</p>'; return; }
  const x0 = Math.min(...xs), x1 = Math.max(...xs), hi = Math.max(...ys, 1e-12), lo = Math.min(0, ...ys);
  const x = c => m + (c - x0) / Math.max(1e-9, x1 - x0) * (W - 2 * m);
  const y = v => H - m - (v - lo) / (hi - lo) * (H - 2 * m);
  let o = svgEl(W, H) + `<rect x="${m}" y="${m}" width="${W - 2 * m}" height="${H - 2 * m}" fill="none" stroke="#444"/>`;
  o += `<text x="${m - 4}" y="${m + 4}" text-anchor="end">${hi.toPrecision(3)}</text>`;
  o += `<text x="${m}" y="${H - m + 16}">${x0}</text><text x="${W - m}" y="${H - m + 16}" text-anchor="end">${x1} cycles</text>`;
  o += kernelMarks(sets[0] || [], x, m, H - m);
  sets.forEach((s, i) => {
    const pts = s.map(r => `${x(r.cycle).toFixed(1)},${y(r[k]).toFixed(1)}`).join(' ');
    o += `<polyline fill="none" stroke="${PAL[i % PAL.length]}" stroke-width="1.5" points="${pts}"/>`;
    o += `<text x="${m + 8}" y="${m + 14 + 13 * i}" fill="${PAL[i % PAL.length]}">${RUNS[i].name}: ${k}</text>`;
  });
  $('series').innerHTML = o + '</svg>';
}
function drawHeat() {
  const k = $('vvar').value, run = RUNS[parseInt($('hrun').value) || 0], rows = rowsIn(run).filter(r => Array.isArray(r[k]));
  if (!rows.length) { $('heat').innerHTML = '<p>no samples in range</p>'; return; }
  const nu = Math.max(...rows.map(r => r[k].length)), hi = Math.max(...rows.map(r => Math.max(...r[k])), 1e-12);
  const W = 900, cw = Math.max(1, (W - 80) / rows.length), ch = Math.max(2, Math.min(8, 640 / nu));
  let o = svgEl(W, ch * nu + 50) + `<text x="10" y="14">${run.name}: ${k} (max ${hi.toPrecision(4)})</text>`;
  rows.forEach((r, t) => r[k].forEach((v, u) => {
    if (!v) return;
    const a = v / hi;
    o += `<rect x="${(60 + t * cw).toFixed(1)}" y="${(24 + u * ch).toFixed(1)}" width="${cw.toFixed(1)}" height="${ch.toFixed(1)}" ` +
         `fill="rgb(${Math.round(255 * a)},${Math.round(80 * (1 - a))},${Math.round(255 * (1 - a))})" ` +
         `data-v="unit ${u} cycle ${r.cycle}: ${v}"/>`;
  }));
  $('heat').innerHTML = o + `<text x="10" y="${24 + nu * ch / 2}">unit</text></svg>`;
  $('heat').querySelectorAll('rect').forEach(e => e.onmousemove = () => { $('hval').textContent = e.dataset.v; });
}
function issueBins(d) {
  const b = {idle: d[0] || 0, scoreboard: d[1] || 0, stall: d[2] || 0};
  for (let lo = 1; lo <= 64; lo += 8) { let s = 0; for (let j = lo; j < lo + 8; ++j) s += d[2 + j] || 0; b[`W${lo}-${lo + 7}`] = s; }
  return b;
}
function drawIssue() {
  const run = RUNS[parseInt($('hrun').value) || 0], rows = rowsIn(run).filter(r => Array.isArray(r.issue_distro));
  if (!rows.length) { $('issue').innerHTML = '<p>no issue distribution in this log</p>'; return; }
  const W = 900, H = 300, m = 50, cw = (W - 2 * m) / rows.length;
  const names = Object.keys(issueBins(rows[0].issue_distro));
  let o = svgEl(W, H + 20) + `<text x="10" y="14">${run.name}: scheduler cycles by outcome (fraction per sample)</text>`;
  rows.forEach((r, t) => {
    const b = issueBins(r.issue_distro), tot = Object.values(b).reduce((a, c) => a + c, 0) || 1;
    let yb = H - m;
    names.forEach((n, i) => {
      const h = b[n] / tot * (H - 2 * m);
      o += `<rect x="${(m + t * cw).toFixed(1)}" y="${(yb - h).toFixed(1)}" width="${Math.max(cw, 1).toFixed(1)}" height="${h.toFixed(1)}" fill="${PAL[i % PAL.length]}"/>`;
      yb -= h;
    });
  });
  names.forEach((n, i) => { o += `<rect x="${m + i * 85}" y="${H - 10}" width="10" height="10" fill="${PAL[i % PAL.length]}"/><text x="${m + 14 + i * 85}" y="${H}">${n}</text>`; });
  $('issue').innerHTML = o + '</svg>';
}
function drawLat() {
  const W = 900, H = 240, m = 50;
  const hs = RUNS.map(run => { const h = new Array(16).fill(0); for (const r of rowsIn(run)) (r.mf_lat_hist || []).forEach((v, i) => h[i] += v); return h; });
  const hi = Math.max(1, ...hs.flat()), bw = (W - 2 * m) / 16 / RUNS.length;
  let o = svgEl(W, H) + `<text x="10" y="14">L1-miss round trip (core cycles, log2 buckets) over the cycle range</text>`;
  hs.forEach((h, j) => h.forEach((v, i) => {
    const hh = v / hi * (H - 2 * m);
    o += `<rect x="${m + (i * RUNS.length + j) * bw}" y="${H - m - hh}" width="${bw - 1}" height="${hh}" fill="${PAL[j % PAL.length]}"/>`;
  }));
  for (let i = 0; i < 16; i += 2) o += `<text x="${m + i * RUNS.length * bw}" y="${H - m + 14}">${1 << i}</text>`;
  $('lat').innerHTML = o + '</svg>';
}
function drawAll() { drawSeries(); drawHeat(); drawIssue(); drawLat(); }
fill($('svar'), keysOf('s'), 'ipc');
fill($('vvar'), keysOf('v').filter(k => k !== 'issue_distro' && k !== 'mf_lat_hist'), 'sm_insn');
$('hrun').innerHTML = RUNS.map((r, i) => `<option value="${i}">${r.name}</option>`).join('');
for (const id of ['svar', 'vvar', 'hrun', 'c0', 'c1']) $(id).onchange = drawAll;
drawAll();
"""


def interactive(runs: Sequence[tuple]) -> str:
    data = [{"name": name, "rows": rows} for name, rows in runs]
    js = _JS.replace("%PALETTE%", json.dumps(svg.PALETTE))
    payload = json.dumps(data).replace("</", "<\\/")
    return ("<h2>interactive viewer</h2>"
            "<div>global variable <select id='svar'></select> &nbsp; per-unit variable <select id='vvar'></select>"
            " &nbsp; run <select id='hrun'></select> &nbsp; cycles <input id='c0' size='9' placeholder='from'>"
            " - <input id='c1' size='9' placeholder='to'></div>"
            "<div id='series'></div><div id='heat'></div><div id='hval' style='height:1.2em;color:#444'></div>"
            "<div id='issue'></div><div id='lat'></div>"
            f"<script type='application/json' id='asim-data'>{payload}</script><script>{js}</script>")


def render(rows: List[Dict], others: Sequence[tuple] = (), name: str = "run") -> str:
    xs = [r["cycle"] for r in rows]
    body = [f"<h2>visualizer: {len(rows)} samples</h2>",
            line_chart(xs, {"IPC": [r.get("ipc", 0) for r in rows]}, "IPC (thread instructions / cycle)"),
            line_chart(xs, {"DRAM utilisation": [r.get("dram_util", 0) for r in rows]}, "DRAM bandwidth utilisation"),
            line_chart(xs, {"L1 misses": [r.get("l1_miss", 0) for r in rows],
                            "L2 accesses": [r.get("l2_access", 0) for r in rows],
                            "L2 misses": [r.get("l2_miss", 0) for r in rows]}, "cache activity per sample"),
            heatmap(rows),
            interactive([(name, rows)] + list(others))]
    return svg.page("visualizer", body)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("logs", nargs="+", help="visualizer logs (text or .gz); the first is the primary run")
    ap.add_argument("-o", "--out", default="visualizer.html")
    ap.add_argument("--csv", help="write this variable of the first log as CSV to stdout instead")
    o = ap.parse_args(argv)
    runs = [(os.path.basename(p), parse(p)) for p in o.logs]
    if o.csv:
        sys.stdout.write(to_csv(runs[0][1], o.csv))
        return 0
    with open(o.out, "w") as f:
        f.write(render(runs[0][1], runs[1:], runs[0][0]))
    print(f"wrote {o.out} ({', '.join(f'{n}: {len(r)} samples' for n, r in runs)})")
    return 0


if __name__ == "__main__":
    sys.exit(main())
