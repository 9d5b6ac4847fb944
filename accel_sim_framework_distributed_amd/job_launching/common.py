"""Shared helpers of the job-launching tools.

Same data model as the reference (util/job_launching/common.py:44-125):
suites / executables / argument lists from ``apps/define-*.yml``, base
configs + composable extras (``BASE-EXTRA1-EXTRA2``) from
``configs/define-*.yml``, run directories ``<run>/<app>/<argfolder>/<cfg>/``.
Base configs may name a preset of this framework (``preset: QV100``), which is
rendered to gpgpusim.config/trace.config on demand, or an explicit
``base_file``.
"""
from __future__ import annotations

import glob
import hashlib
import os
import re
from typing import Dict, List, Optional, Tuple

import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)
REPO_ROOT = os.path.dirname(PKG_ROOT)


def argfoldername(args) -> str:
    """Run-subdirectory name of an argument string (reference get_argfoldername)."""
    if args is None or str(args).strip() == "":
        return "NO_ARGS"
    s = str(args).strip()
    if len(s) > 256:
        return "hashed_args_" + hashlib.md5(s.encode()).hexdigest()
    return re.sub(r"[^a-zA-Z0-9]", "_", s)


def config_root() -> str:
    return os.environ.get("ASIM_CONFIG_ROOT", os.path.join(REPO_ROOT, "configs", "generated"))


def log_dir() -> str:
    d = os.environ.get("ASIM_JOB_LOGDIR", os.path.join(HERE, "logfiles"))
    os.makedirs(d, exist_ok=True)
    return d


class Registry:
    """Apps and configs defined by the YAML files."""

    def __init__(self, extra_dirs: Optional[List[str]] = None):
        self.apps: Dict[str, List[Tuple[str, str, str, List[Dict]]]] = {}
        self.base: Dict[str, Dict] = {}
        self.extra: Dict[str, str] = {}
        dirs = [HERE] + (extra_dirs or []) + [d for d in os.environ.get("ASIM_YAML_PATH", "").split(":") if d]
        for d in dirs:
            for f in sorted(glob.glob(os.path.join(d, "apps", "define-*.yml"))):
                self._load_apps(f)
            for f in sorted(glob.glob(os.path.join(d, "configs", "define-*.yml"))):
                self._load_configs(f)

    def _load_apps(self, path: str) -> None:
        data = yaml.safe_load(open(path)) or {}
        for suite, desc in data.items():
            self.apps.setdefault(suite, [])
            for exe in desc.get("execs", []):
                name = list(exe.keys())[0]
                args_list = list(exe.values())[0] or [{"args": None}]
                for a in args_list:
                    a.setdefault("accel-sim-mem", "4G")
                entry = (desc.get("exec_dir", ""), desc.get("data_dirs", ""), name, args_list)
                self.apps[suite].append(entry)
                self.apps[f"{suite}:{name}"] = [entry]
                for i, a in enumerate(args_list):
                    self.apps[f"{suite}:{name}:{i}"] = [(entry[0], entry[1], name, [a])]

    def _load_configs(self, path: str) -> None:
        data = yaml.safe_load(open(path)) or {}
        for name, desc in data.items():
            if "base_file" in desc or "preset" in desc:
                self.base[name] = desc
            elif "extra_params" in desc:
                self.extra[name] = desc["extra_params"]

    def benchmarks(self, suites: List[str]):
        out = []
        for s in suites:
            if s not in self.apps:
                raise KeyError(f"unknown benchmark suite {s!r}; defined: {sorted(k for k in self.apps if ':' not in k)}")
            out += self.apps[s]
        return out

    def config(self, name: str) -> Tuple[str, str, str]:
        """(name, extra_params_text, base_gpgpusim_config_path)."""
        toks = name.split("-")
        if toks[0] not in self.base:
            raise KeyError(f"unknown base config {toks[0]!r}; defined: {sorted(self.base)}")
        extra = ""
        for t in toks[1:]:
            if t not in self.extra:
                raise KeyError(f"unknown extra config {t!r}; defined: {sorted(self.extra)}")
            extra += f"\n#{t}\n{self.extra[t]}\n"
        return name, extra, self.base_file(toks[0])

    def base_file(self, base: str) -> str:
        desc = self.base[base]
        if "base_file" in desc:
            p = os.path.expandvars(desc["base_file"])
            return p if os.path.isabs(p) else os.path.join(REPO_ROOT, p)
        from ..models import presets
        d = os.path.join(config_root(), desc["preset"])
        p = os.path.join(d, "gpgpusim.config")
        if not os.path.exists(p):
            presets.write_config(desc["preset"], d)
        return p


def file_or_rel(name: str) -> str:
    name = os.path.expandvars(name)
    if os.path.exists(name):
        return os.path.abspath(name)
    alt = os.path.join(os.getcwd(), name)
    if os.path.exists(alt):
        return alt
    raise FileNotFoundError(name)


def simulator_binary() -> str:
    b = os.environ.get("ASIM_BINARY", os.path.join(REPO_ROOT, "bin", "accel-sim.out"))
    if not os.path.exists(b):
        raise FileNotFoundError(f"simulator binary {b} missing: run build_native.py")
    return b


def build_version() -> str:
    """Version string recorded per launch (reference extract_version)."""
    try:
        import subprocess
        h = subprocess.run(["git", "-C", REPO_ROOT, "rev-parse", "--short", "HEAD"], capture_output=True,
                           text=True, timeout=10).stdout.strip()
    except Exception:
        h = ""
    from .. import __version__
    return f"asim-{__version__}-{h or 'nogit'}"
