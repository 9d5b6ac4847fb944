"""Run the CDNA4 micro-benchmark suite (bin/ubench/*, built from csrc/ubench)
and collect what the tuner reads: `-<gpgpusim option> <value>` lines and
`# <measurement> <value>` lines (reference util/tuner/GPU_Microbenchmark,
whose programs print the same kinds of lines)."""
from __future__ import annotations

import os
import re
import subprocess
from typing import Dict, List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
BIN = os.path.join(ROOT, "bin", "ubench")
_OPT = re.compile(r"^(-[A-Za-z0-9_:]+)\s+(.+?)\s*$")
_MEAS = re.compile(r"^#\s*([A-Za-z0-9_]+)\s+([-+0-9.eE]+)\s*$")


def programs() -> List[str]:
    return sorted(f for f in os.listdir(BIN) if f.startswith("ub_")) if os.path.isdir(BIN) else []


def parse(text: str) -> Dict[str, Dict[str, str]]:
    """{'options': {flag: value}, 'measurements': {key: value}} from a program's output."""
    opts, meas = {}, {}
    for line in text.splitlines():
        m = _OPT.match(line)
        if m:
            opts[m.group(1)] = m.group(2)
            continue
        m = _MEAS.match(line)
        if m:
            meas[m.group(1)] = m.group(2)
    return dict(options=opts, measurements=meas)


def run(names: Optional[List[str]] = None, out_dir: Optional[str] = None, timeout: int = 240) -> Dict[str, Dict]:
    """Run the named programs (default: all built ones) one at a time, each
    under its own time limit; stop at the first failure."""
    res = {}
    for name in names or programs():
        p = subprocess.run([os.path.join(BIN, name)], capture_output=True, text=True, timeout=timeout)
        if out_dir:
            os.makedirs(out_dir, exist_ok=True)
            with open(os.path.join(out_dir, name + ".log"), "w") as f:
                f.write(p.stdout + p.stderr)
        if p.returncode != 0:
            raise RuntimeError(f"{name} failed (rc={p.returncode}): {p.stderr[-500:]}")
        res[name] = parse(p.stdout)
    return res
