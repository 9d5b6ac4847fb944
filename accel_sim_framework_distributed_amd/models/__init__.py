"""Simulated GPU models (config presets rendered to gpgpusim.config/trace.config)."""
from .presets import PRESETS, args_for, get_preset, write_config  # noqa: F401
